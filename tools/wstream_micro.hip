// Micro-benchmark (GPU box): how fast a GEMM stage's weight fragments reach the registers, by the
// per-lane pattern of the loads.  The F_fwd01 shape of l0r16_kernel<5, 2> (td3_amd/csrc/kernels.hip):
// 240 workgroups of 10 waves, 3 networks x 5 column tiles of 80 x 16 row tiles; wave (c, kq) loads
// rows n0 + 16c + (lane & 15) of W [400][512] over its half of K in 32-deep chunks (160 KB per
// workgroup, 2.4 MB distinct), as the MFMA fragments of v_mfma_f32_16x16x4_f32 need them.
//   0  lane (j16, g): k = 8g .. 8g+3 and 8g+4 .. 8g+7 of the chunk (the kernels' pattern today)
//   1  lane (j16, g): k = 4g .. 4g+3 and 16+4g .. 16+4g+3 (each instruction: 64 contiguous B per row)
//   2  coalesced: instruction r covers rows 8r .. 8r+7 of the wave's 16, 128 B per row (not an MFMA
//      layout: the bandwidth ceiling of the same bytes)
//   3  pattern 0 in two rounds of 8 loads (half the bytes in flight)
//   4  LDS-DMA (global_load_lds_dwordx4), coalesced as 2, rounds of 4 instructions per wave
//   5  LDS-DMA, rounds of 8 instructions per wave (80 KB in flight per workgroup)
//   9  no loads (launch + epilogue floor)
// Each launch follows a kernel that rewrites W (the previous step's Adam update), so the weights
// arrive from wherever C_dw leaves them.  Prints the average launch time per pattern (HIP events).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/wstream_micro.hip -o tools/exp/wstream_micro
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int REP = 4;                                              // networks streamed per workgroup
constexpr int NNET = 3 * REP, NOUT = 400, LDW = 512, MT = 16, NCT = 5, WK = 2, NW = NCT * WK;
constexpr int NTILE = (NOUT + 16 * NCT - 1) / (16 * NCT);          // 5 column tiles of 80
constexpr int NWG = 3 * NTILE * MT;                                 // 240
constexpr int NCH = LDW / 32, CPW = NCH / WK;                       // 16 chunks, 8 per wave

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
typedef __attribute__((address_space(3))) void* lptr;
__device__ __forceinline__ void glds16(const float* src, float* lds) {
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lptr)lds);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
}

template <int PAT>
__global__ __launch_bounds__(64 * NW) void wstream(const float* W, float* out) {
  const int b = blockIdx.x;
  // consecutive tiles on one XCD (as xcd_tile): workgroup id b runs on XCD b % 8
  const int per = (NWG + 7) / 8, t = (b & 7) * per + (b >> 3);
  if (t >= NWG) return;
  const int net0 = t / (NTILE * MT), r = t % (NTILE * MT), nt = r / MT;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, j16 = lane & 15, g = lane >> 4;
  const int c = wave % NCT, kq = wave / NCT;
  const int n0 = nt * 16 * NCT + 16 * c;
  float4 v[2 * CPW];
  float tot = 0.f;
  for (int rep = 0; rep < REP; ++rep) {
  const float* Wn = W + (size_t)(net0 + 3 * rep) * NOUT * LDW;
  if constexpr (PAT == 4 || PAT == 5) {
    // per wave: an LDS slot of R KB, refilled CPW*2/R times (rounds of R 1-KB instructions)
    extern __shared__ float4 sm4[];
    constexpr int R = PAT == 4 ? 4 : 8;
    float* slot = reinterpret_cast<float*>(sm4) + wave * R * 256;
    const int row = lane >> 3, col = (lane & 7) * 4;
    float s = 0.f;
#pragma unroll
    for (int q0 = 0; q0 < 2 * CPW; q0 += R) {
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const int q = (q0 + j) >> 1, hf = (q0 + j) & 1;
        const int kb = (kq * CPW + q) * 32;
        glds16(Wn + (size_t)min(n0 + 8 * hf + row, NOUT - 1) * LDW + kb + col, slot + j * 256);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      s += slot[lane * 4];
    }
    tot += s;
    continue;
  }
  if constexpr (PAT == 9) break;
#pragma unroll
  for (int q = 0; q < CPW; ++q) {
    if (PAT == 3 && q == CPW / 2) {
      float s = 0.f;
#pragma unroll
      for (int u = 0; u < CPW; ++u) s += v[u].x + v[u].y + v[u].z + v[u].w;
      v[0].x = s;
      __builtin_amdgcn_sched_barrier(0);
    }
    const int kb = (kq * CPW + q) * 32;
    if (PAT == 0 || PAT == 3) {
      const float* p = Wn + (size_t)min(n0 + j16, NOUT - 1) * LDW + kb + 8 * g;
      v[2 * q] = ld4(p);
      v[2 * q + 1] = ld4(p + 4);
    } else if (PAT == 1) {
      const float* p = Wn + (size_t)min(n0 + j16, NOUT - 1) * LDW + kb + 4 * g;
      v[2 * q] = ld4(p);
      v[2 * q + 1] = ld4(p + 16);
    } else if (PAT == 6) {            // k-quad image of W: piece (n, j) at (j * NOUT + n) * 4
      const float* p = Wn + ((size_t)((kb >> 2) + 2 * g) * NOUT + min(n0 + j16, NOUT - 1)) * 4;
      v[2 * q] = ld4(p);
      v[2 * q + 1] = ld4(p + 4 * NOUT);
    } else {
      const int row = lane >> 3, col = (lane & 7) * 4;
      v[2 * q] = ld4(Wn + (size_t)min(n0 + row, NOUT - 1) * LDW + kb + col);
      v[2 * q + 1] = ld4(Wn + (size_t)min(n0 + 8 + row, NOUT - 1) * LDW + kb + col);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 2 * CPW; ++q) s += v[q].x + v[q].y + v[q].z + v[q].w;
  tot += s;
  }
  out[(size_t)b * 64 * NW + threadIdx.x] = tot;
}

__global__ void touch(float* W, int n, float a) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) W[i] = W[i] * a;
}

template <int PAT>
static float run(float* W, float* out, int n, int reps, bool dirty) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float tot = 0.f;
  for (int i = 0; i < reps + 5; ++i) {
    if (dirty) hipLaunchKernelGGL(touch, dim3(512), dim3(256), 0, 0, W, n, 1.0f);
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(wstream<PAT>, dim3(NWG), dim3(64 * NW), (PAT == 4 || PAT == 5) ? NW * 8 * 1024 : 0, 0, W, out);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (i >= 5) tot += ms;
  }
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return tot / reps * 1000.f;
}

int main() {
  const int n = NNET * NOUT * LDW;
  float *W, *out;
  CK(hipMalloc(&W, (size_t)n * 4));
  CK(hipMalloc(&out, (size_t)NWG * 64 * NW * 4));
  CK(hipMemset(W, 0, (size_t)n * 4));
  const int reps = 200;
  CK(hipFuncSetAttribute((const void*)wstream<4>, hipFuncAttributeMaxDynamicSharedMemorySize, NW * 8 * 1024));
  CK(hipFuncSetAttribute((const void*)wstream<5>, hipFuncAttributeMaxDynamicSharedMemorySize, NW * 8 * 1024));
  printf("[%d wg x %d waves, %d KB per wg]\n", NWG, NW, REP * CPW * 2 * 1024 * NW / 1024);
  for (int rnd = 0; rnd < 2; ++rnd) {
    for (int d = 0; d < 2; ++d) {
      const float t0 = run<0>(W, out, n, reps, d), t1 = run<1>(W, out, n, reps, d), t2 = run<2>(W, out, n, reps, d);
      const float t3 = run<3>(W, out, n, reps, d), t4 = run<4>(W, out, n, reps, d), t5 = run<5>(W, out, n, reps, d);
      const float t6 = run<6>(W, out, n, reps, d), t9 = run<9>(W, out, n, reps, d);
      printf("round %d %-18s: 8g-split %.2f  4g-contig %.2f  coalesced %.2f  8g-2rounds %.2f  ldsdma-r4 %.2f  "
             "ldsdma-r8 %.2f  kquad-image %.2f  empty %.2f us\n", rnd, d ? "after a W rewrite" : "back to back", t0, t1, t2, t3,
             t4, t5, t6, t9);
    }
  }
  CK(hipFree(W));
  CK(hipFree(out));
  return 0;
}
