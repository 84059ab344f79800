// Micro-benchmark (GPU box): where a split-K dW step's time goes.  One workgroup per CU runs
// `steps` 64-row steps of one 128x128 (or 64x64) dW tile, dW = G^T U over G, U [rows][512] fp32,
// the staging and MFMA loop of td3_amd/csrc/kernels.hip dwsk_matrix128 / dwsk_matrix, in modes
//   0 full (LDS-DMA double buffer + MFMA from LDS)   1 MFMA from LDS only (no DMA)
//   2 DMA + barriers only (no MFMA)                   3 MFMA from registers only
// Prints us per step per CU and the MFMA fraction of the f32 peak.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/dwsk_micro.hip -o tools/exp/dwsk_micro
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void* lptr;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void glds16(const float* src, float* lds) {
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lptr)lds);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
}

constexpr int LD = 512;

template <int MODE>
__global__ __launch_bounds__(512, 1) void k128(const float* G, const float* U, float* out, int steps) {
  __shared__ float sm[2 * 2 * 64 * 128];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, i = lane & 31, h = lane >> 5;
  const int t = blockIdx.x & 15, n0 = (t >> 2) * 128, k0 = (t & 3) * 128;
  const int qn = wave >> 1, qk0 = wave & 1, qk1 = qk0 + 2;
  const int lr = lane >> 5, lc = (lane & 31) * 4;
  int gcol[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 8 * wave + 2 * j + lr;
    gcol[j] = lc ^ (((row >> 4) & 1) << 5);
  }
  const size_t base = (size_t)(blockIdx.x >> 4) * steps * 64;   // row block of this workgroup
  auto issue = [&](int st, int buf) {
    float* g = sm + buf * 2 * 8192;
    float* u = g + 8192;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int rl = 8 * wave + 2 * j;
      const size_t row = base + (size_t)(st * 64 + rl + lr);
      glds16(G + row * LD + n0 + gcol[j], g + rl * 128);
      glds16(U + row * LD + k0 + gcol[j], u + rl * 128);
    }
  };
  f32x16 acc0, acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) { acc0[r] = 0.f; acc1[r] = 0.f; }
  const int ca = (qn ^ h) * 32 + i, cb0 = (qk0 ^ h) * 32 + i, cb1 = (qk1 ^ h) * 32 + i;
  if (MODE == 0 || MODE == 2) issue(0, 0);
  float ra = (float)lane, rb = (float)tid;
  for (int st = 0; st < steps; ++st) {
    const int buf = st & 1;
    if (MODE == 0 || MODE == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if ((MODE == 0 || MODE == 2) && st + 1 < steps) issue(st + 1, buf ^ 1);
    if (MODE == 2) continue;
    if (MODE == 3) {
#pragma unroll
      for (int s2 = 0; s2 < 32; ++s2) {
        acc0 = mfma(ra, rb, acc0);
        acc1 = mfma(rb, ra, acc1);
      }
      continue;
    }
    const float* g = sm + buf * 2 * 8192 + 16 * h * 128;
    const float* u = g + 8192;
#pragma unroll
    for (int s2 = 0; s2 < 32; ++s2) {
      const int r = 32 * (s2 >> 4) + (s2 & 15);
      const float ga = g[r * 128 + ca];
      acc0 = mfma(ga, u[r * 128 + cb0], acc0);
      acc1 = mfma(ga, u[r * 128 + cb1], acc1);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) s += acc0[r] + acc1[r];
  out[blockIdx.x * 512 + tid] = s;
}

template <int MODE>
__global__ __launch_bounds__(512, 2) void k64(const float* G, const float* U, float* out, int steps) {
  __shared__ float sm[2 * 2 * 64 * 64];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, i = lane & 31, h = lane >> 5;
  const int t = blockIdx.x & 63, n0 = (t >> 3) * 64, k0 = (t & 7) * 64;
  const int qn = (wave >> 1) & 1, qk = wave & 1, rh = wave >> 2;
  const int lr = lane >> 4, lc = (lane & 15) * 4;
  int gcol[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = 8 * wave + 4 * j + lr;
    gcol[j] = lc ^ (((row >> 4) & 1) << 5);
  }
  const size_t base = (size_t)(blockIdx.x >> 6) * steps * 64;
  auto issue = [&](int st, int buf) {
    float* g = sm + buf * 2 * 4096;
    float* u = g + 4096;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int rl = 8 * wave + 4 * j;
      const size_t row = base + (size_t)(st * 64 + rl + lr);
      glds16(G + row * LD + n0 + gcol[j], g + rl * 64);
      glds16(U + row * LD + k0 + gcol[j], u + rl * 64);
    }
  };
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const int ca = (qn ^ h) * 32 + i, cb = (qk ^ h) * 32 + i;
  if (MODE == 0 || MODE == 2) issue(0, 0);
  float ra = (float)lane, rb = (float)tid;
  for (int st = 0; st < steps; ++st) {
    const int buf = st & 1;
    if (MODE == 0 || MODE == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if ((MODE == 0 || MODE == 2) && st + 1 < steps) issue(st + 1, buf ^ 1);
    if (MODE == 2) continue;
    if (MODE == 3) {
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) acc = mfma(ra, rb, acc);
      continue;
    }
    const float* g = sm + buf * 2 * 4096 + (rh * 32 + 16 * h) * 64;
    const float* u = g + 4096;
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2) acc = mfma(g[s2 * 64 + ca], u[s2 * 64 + cb], acc);
  }
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) s += acc[r];
  out[blockIdx.x * 512 + tid] = s;
}

template <typename K>
static float run(K kern, int grid, const float* G, const float* U, float* out, int steps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, 0, G, U, out, steps);
  CK(hipEventRecord(a));
  const int reps = 20;
  for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, 0, G, U, out, steps);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / reps;
}

int main(int argc, char** argv) {
  const int steps = argc > 1 ? atoi(argv[1]) : 16;
  const int grid = 256;
  const size_t rows = (size_t)(grid / 16 + 1) * steps * 64 + 64;   // k128: 16 row blocks; k64: 4
  float *G, *U, *out;
  CK(hipMalloc(&G, rows * LD * 4));
  CK(hipMalloc(&U, rows * LD * 4));
  CK(hipMalloc(&out, grid * 2 * 512 * 4));
  CK(hipMemset(G, 0, rows * LD * 4));
  CK(hipMemset(U, 0, rows * LD * 4));
  const double peak_cu = 157.3e12 / 256;
  const char* names[4] = {"full", "mfma_lds", "dma_only", "mfma_reg"};
  for (int m = 0; m < 4; ++m) {
    float us = 0;
    switch (m) {
      case 0: us = run(k128<0>, grid, G, U, out, steps); break;
      case 1: us = run(k128<1>, grid, G, U, out, steps); break;
      case 2: us = run(k128<2>, grid, G, U, out, steps); break;
      case 3: us = run(k128<3>, grid, G, U, out, steps); break;
    }
    const double fl = 2.0 * 128 * 128 * 64 * steps;
    printf("k128 %-9s steps %3d  %8.2f us  %6.3f us/step  mfma frac %.3f\n", names[m], steps, us, us / steps,
           fl / (us * 1e-6) / peak_cu);
  }
  for (int g2 : {256, 512}) {
    for (int m = 0; m < 4; ++m) {
      float us = 0;
      switch (m) {
        case 0: us = run(k64<0>, g2, G, U, out, steps); break;
        case 1: us = run(k64<1>, g2, G, U, out, steps); break;
        case 2: us = run(k64<2>, g2, G, U, out, steps); break;
        case 3: us = run(k64<3>, g2, G, U, out, steps); break;
      }
      const double fl = 2.0 * 64 * 64 * 64 * steps * (g2 / 256);
      printf("k64 grid %d %-9s steps %3d  %8.2f us  %6.3f us/step/CU  mfma frac %.3f\n", g2, names[m], steps, us,
             us / steps / (g2 / 256), fl / (us * 1e-6) / peak_cu);
    }
  }
  return 0;
}
