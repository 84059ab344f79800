// Launch-floor probe (GPU box helper, not product code): wall time per kernel of a
// hipGraph-replayed chain of N dependent kernels, by grid size / LDS / kernarg size,
// plus the same chain launched eagerly.  Built as an exe (ROCm runtime) and as a .so
// (exported probe_main) so it can also run inside a torch process (torch's runtime).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

struct Big { float* p; int pad[70]; };

__global__ void k_small(float* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1.f;
}
__global__ void k_grid(float* p) {
  p[blockIdx.x * blockDim.x + threadIdx.x] += 1.f;
}
__global__ void k_lds(float* p) {
  extern __shared__ float s[];
  s[threadIdx.x] = p[blockIdx.x * blockDim.x + threadIdx.x];
  __syncthreads();
  p[blockIdx.x * blockDim.x + threadIdx.x] = s[(threadIdx.x + 1) % blockDim.x] + 1.f;
}
__global__ void k_big(Big b) {
  b.p[blockIdx.x * blockDim.x + threadIdx.x] += (float)b.pad[threadIdx.x % 70];
}
// dependent chain of 3 global loads through a table (like our problem descriptors)
struct Tab { const float* a; float* c; int n; };
__global__ void k_chain(const Tab* t) {
  const Tab T = t[0];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float v = T.a[i];
  int j = ((int)v) & (T.n - 1);
  T.c[i] = T.a[j] + 1.f;
}

template <class F>
static int time_chain(const char* name, int nk, F launch, hipStream_t s) {
  // eager
  for (int w = 0; w < 3; ++w) for (int k = 0; k < nk; ++k) launch(s);
  CK(hipStreamSynchronize(s));
  const int reps = 200;
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; ++r) for (int k = 0; k < nk; ++k) launch(s);
  CK(hipStreamSynchronize(s));
  double eager = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / (reps * nk);
  // graph
  hipStream_t cs;
  CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  CK(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
  for (int k = 0; k < nk; ++k) launch(cs);
  hipGraph_t g;
  CK(hipStreamEndCapture(cs, &g));
  hipGraphExec_t ge;
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int w = 0; w < 5; ++w) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
  auto t1 = std::chrono::steady_clock::now();
  CK(hipStreamSynchronize(s));
  auto t2 = std::chrono::steady_clock::now();
  double host = std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
  double graph = std::chrono::duration<double, std::micro>(t2 - t0).count() / (reps * nk);
  // device time via events around one replay
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < 20; ++r) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::printf("%-28s nk=%2d  eager %6.2f us/kernel  graph %6.2f us/kernel (events %6.2f)  host graphLaunch %7.2f us\n",
              name, nk, eager, graph, ms * 1e3 / (20 * nk), host);
  hipGraphExecDestroy(ge); hipGraphDestroy(g); hipStreamDestroy(cs);
  hipEventDestroy(e0); hipEventDestroy(e1);
  return 0;
}

extern "C" int probe_main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float* p;
  CK(hipMalloc(&p, 64 << 20));
  CK(hipMemset(p, 0, 64 << 20));
  Tab* t;
  CK(hipMalloc(&t, sizeof(Tab)));
  Tab th{p, p + (8 << 20), 1 << 20};
  CK(hipMemcpy(t, &th, sizeof(Tab), hipMemcpyHostToDevice));
  CK(hipFuncSetAttribute((const void*)k_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  for (int nk : {1, 20}) {
    time_chain("1 WG", nk, [&](hipStream_t st) { k_small<<<1, 64, 0, st>>>(p); }, s);
    time_chain("256 WG x 256", nk, [&](hipStream_t st) { k_grid<<<256, 256, 0, st>>>(p); }, s);
    time_chain("1024 WG x 256", nk, [&](hipStream_t st) { k_grid<<<1024, 256, 0, st>>>(p); }, s);
    time_chain("256 WG x 256, 66KB LDS", nk, [&](hipStream_t st) { k_lds<<<256, 256, 66 * 1024, st>>>(p); }, s);
    time_chain("512 WG x 256, 66KB LDS", nk, [&](hipStream_t st) { k_lds<<<512, 256, 66 * 1024, st>>>(p); }, s);
    time_chain("256 WG, 300B kernarg", nk, [&](hipStream_t st) { Big b{}; b.p = p; k_big<<<256, 256, 0, st>>>(b); }, s);
    time_chain("256 WG, table+2 dep loads", nk, [&](hipStream_t st) { k_chain<<<256, 256, 0, st>>>(t); }, s);
  }
  hipFree(p); hipFree(t); hipStreamDestroy(s);
  return 0;
}

#ifndef PROBE_LIB
int main() { return probe_main(); }
#endif
