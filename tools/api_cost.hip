// Host-side cost of the HIP runtime calls the acting loop makes (GPU box helper, not product
// code): enqueue cost and idle round trips of launches, copies, events and graph replays.
//   hipcc --offload-arch=gfx950 -O2 tools/api_cost.hip -o tools/api_cost && tools/api_cost
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

__global__ void empty_kernel() {}

__global__ void copy_kernel(const float* __restrict__ src, float* __restrict__ dst, int n) {
  int i = threadIdx.x;
  if (i < n) dst[i] = src[i] + 1.f;
}

static double time_us(const std::function<void()>& f, int n = 2000) {
  for (int i = 0; i < 100; ++i) f();
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) f();
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t ev, ev2;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&ev2, hipEventDisableTiming));
  float *d_a, *d_b, *h_pin, *h_map, *h_map_out, *d_map, *d_map_out;
  CK(hipMalloc(&d_a, 1 << 20));
  CK(hipMalloc(&d_b, 1 << 20));
  CK(hipHostMalloc(&h_pin, 1 << 16, hipHostMallocDefault));
  CK(hipHostMalloc(&h_map, 1 << 16, hipHostMallocMapped));
  CK(hipHostMalloc(&h_map_out, 1 << 16, hipHostMallocMapped));
  CK(hipHostGetDevicePointer((void**)&d_map, h_map, 0));
  CK(hipHostGetDevicePointer((void**)&d_map_out, h_map_out, 0));
  float* h_page = (float*)malloc(1 << 16);
  for (int i = 0; i < 64; ++i) h_page[i] = h_pin[i] = h_map[i] = (float)i;

  struct R { const char* name; double us; };
  R res[32];
  int nr = 0;
  auto add = [&](const char* name, const std::function<void()>& f, int n = 2000) {
    CK(hipStreamSynchronize(s));
    res[nr++] = {name, time_us(f, n)};
  };

  add("launch (enqueue only, 64 in flight max)", [&] {
    for (int i = 0; i < 64; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
    CK(hipStreamSynchronize(s));
  }, 100);
  res[nr - 1].us /= 64;
  add("launch + stream sync", [&] {
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
    CK(hipStreamSynchronize(s));
  });
  add("4 launches + stream sync", [&] {
    for (int i = 0; i < 4; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
    CK(hipStreamSynchronize(s));
  });
  add("stream sync (idle)", [&] { CK(hipStreamSynchronize(s)); });
  add("event record (idle stream)", [&] { CK(hipEventRecord(ev, s)); });
  add("event sync (completed)", [&] { CK(hipEventSynchronize(ev)); });
  add("event query (completed)", [&] { (void)hipEventQuery(ev); });
  add("stream wait event (completed, other stream)", [&] { CK(hipStreamWaitEvent(s2, ev, 0)); });
  add("memcpyAsync H2D 256B pinned + sync", [&] {
    CK(hipMemcpyAsync(d_a, h_pin, 256, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
  });
  add("memcpyAsync H2D 256B pageable + sync", [&] {
    CK(hipMemcpyAsync(d_a, h_page, 256, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
  });
  add("memcpyAsync D2H 32B pageable + sync", [&] {
    CK(hipMemcpyAsync(h_page, d_a, 32, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
  });
  add("memcpyAsync D2H 32B pinned + sync", [&] {
    CK(hipMemcpyAsync(h_pin, d_a, 32, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
  });
  add("memcpy2DAsync H2D 17x1 pageable + sync", [&] {
    CK(hipMemcpy2DAsync(d_a, 128, h_page, 68, 68, 1, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
  });
  add("H2D pinned + kernel + D2H pinned + sync", [&] {
    CK(hipMemcpyAsync(d_a, h_pin, 256, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(copy_kernel, dim3(1), dim3(64), 0, s, d_a, d_b, 64);
    CK(hipMemcpyAsync(h_pin + 128, d_b, 32, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
  });
  add("kernel mapped-in -> mapped-out + sync", [&] {
    hipLaunchKernelGGL(copy_kernel, dim3(1), dim3(64), 0, s, d_map, d_map_out, 64);
    CK(hipStreamSynchronize(s));
  });
  add("kernel mapped-in -> device + event record", [&] {
    hipLaunchKernelGGL(copy_kernel, dim3(1), dim3(64), 0, s, d_map, d_b, 64);
    CK(hipEventRecord(ev, s));
  });
  CK(hipStreamSynchronize(s));
  // graph of 4 kernels (mapped in -> 2 empty -> mapped out)
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  hipLaunchKernelGGL(copy_kernel, dim3(1), dim3(64), 0, s, d_map, d_a, 64);
  hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
  hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
  hipLaunchKernelGGL(copy_kernel, dim3(1), dim3(64), 0, s, d_a, d_map_out, 64);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  add("graph(4 kernels, mapped io) launch + sync", [&] {
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
  });
  add("graph(4 kernels) launch only (drained per 16)", [&] {
    for (int i = 0; i < 16; ++i) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
  }, 200);
  res[nr - 1].us /= 16;
  // correctness of the mapped round trip
  CK(hipStreamSynchronize(s));
  for (int i = 0; i < 64; ++i) h_map[i] = (float)(3 * i);
  hipLaunchKernelGGL(copy_kernel, dim3(1), dim3(64), 0, s, d_map, d_map_out, 64);
  CK(hipStreamSynchronize(s));
  int bad = 0;
  for (int i = 0; i < 64; ++i) bad += h_map_out[i] != (float)(3 * i) + 1.f;
  for (int i = 0; i < nr; ++i) printf("%-48s %8.2f us\n", res[i].name, res[i].us);
  printf("mapped round trip mismatches: %d\n", bad);
  return bad != 0;
}
