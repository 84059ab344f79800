// Probe (GPU box helper, not product code): do independent branches of a captured hipGraph
// run concurrently?  Two chains of K kernels each (one workgroup spinning ~T us per kernel),
// captured from two streams forked / joined with events, vs the same kernels on one stream.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void spin(long long cycles, float* p) {
  long long t0 = clock64();
  while (clock64() - t0 < cycles) {}
  if (threadIdx.x == 0) p[blockIdx.x] += 1.f;
}

static double run_graph(hipGraphExec_t ge, hipStream_t s, int reps) {
  for (int i = 0; i < 3; ++i) (void)hipGraphLaunch(ge, s);
  (void)hipStreamSynchronize(s);
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < reps; ++i) (void)hipGraphLaunch(ge, s);
  (void)hipStreamSynchronize(s);
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
}

extern "C" int probe_main() {
  const int K = 10;
  const long long cyc = 20000;     // ~10 us at ~2 GHz
  float* p;
  CK(hipMalloc(&p, 1 << 20));
  hipStream_t s0, s1, cs0, cs1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&cs0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&cs1, hipStreamNonBlocking));
  hipEvent_t fork, join;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  for (int wgs : {1, 128}) {
    // serial: 2K kernels on one stream
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(cs0, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < 2 * K; ++k) spin<<<wgs, 64, 0, cs0>>>(cyc, p);
    CK(hipStreamEndCapture(cs0, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    double ser = run_graph(ge, s0, 20);
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
    // branched: fork cs1 from cs0, K kernels on each, join
    CK(hipStreamBeginCapture(cs0, hipStreamCaptureModeThreadLocal));
    CK(hipEventRecord(fork, cs0));
    CK(hipStreamWaitEvent(cs1, fork, 0));
    for (int k = 0; k < K; ++k) {
      spin<<<wgs, 64, 0, cs0>>>(cyc, p);
      spin<<<wgs, 64, 0, cs1>>>(cyc, p + 512);
    }
    CK(hipEventRecord(join, cs1));
    CK(hipStreamWaitEvent(cs0, join, 0));
    CK(hipStreamEndCapture(cs0, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    double br = run_graph(ge, s0, 20);
    size_t nn = 0;
    CK(hipGraphGetNodes(g, nullptr, &nn));
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
    // eager two streams
    for (int i = 0; i < 2; ++i) {
      for (int k = 0; k < K; ++k) {
        spin<<<wgs, 64, 0, s0>>>(cyc, p);
        spin<<<wgs, 64, 0, s1>>>(cyc, p + 512);
      }
    }
    CK(hipDeviceSynchronize());
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < 20; ++r)
      for (int k = 0; k < K; ++k) {
        spin<<<wgs, 64, 0, s0>>>(cyc, p);
        spin<<<wgs, 64, 0, s1>>>(cyc, p + 512);
      }
    CK(hipDeviceSynchronize());
    double eg = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 20;
    std::printf("wgs=%3d  serial graph %7.1f us | branched graph %7.1f us (%zu nodes) | eager 2 streams %7.1f us\n",
                wgs, ser, br, nn, eg);
  }
  return 0;
}

#ifndef PROBE_LIB
int main() { return probe_main(); }
#endif
