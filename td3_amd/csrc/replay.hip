// Replay ring kernels + the rb_* C-ABI (include/td3.h).
//
// Reference: /root/reference/my_replay_buffer.py
//   ReplayBuffer_featured.__init__  :73-89   -> rb_create
//   ReplayBuffer_featured.add       :109-117 -> rb_add (batched, pinned staging, async H2D)
//   ReplayBuffer_featured.sample    :119-128 -> rb_sample / gather_kernel (Philox + HBM gather)
//   ReplayBuffer_featured.save/load :91-107  -> rb_read_records / rb_write_records
//   ReplayBuffer_particles          :6-69    -> rb_create_particles / rb_add_particles /
//                                               rb_sample_particles (same ring, wider record)
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <atomic>
#include <mutex>
#include <set>

#include "replay.h"
#include "../../include/td3.h"

namespace td3 {

// ------------------------------------------------------------------ gather
// One wave per sampled row: the row index is drawn once per wave, the record
// (rec floats, 16-B aligned) is read as float4 (all of it in flight at once) into the
// wave's LDS slot and written to every destination segment.  A segment whose row start is
// 16-B aligned (every network-input segment: row strides are multiples of 32 floats) is
// stored as float4 -- four LDS dwords per lane, whatever the record offset, into one 16-B
// global store -- and its tail / unaligned segments as dwords.  Rows B..Bp-1 are
// zero-filled so padded batch rows stay finite and contribute nothing downstream.
// Bytes moved per live row: rec*4 read + sum(len)*4 written (td3.hip input_from_ring).
__device__ __forceinline__ int64_t gather_row_index(const GatherArgs& a, int row) {
  if (a.inject_idx) return a.inject_idx[row];
  const uint64_t size = (uint64_t)*a.d_size;  // issued alongside the counter load
  const uint64_t step = a.ctr ? (uint64_t)(a.ctr->total_it + 1) : a.step;
  return (int64_t)philox_index(a.seed, step, (uint32_t)row, size);
}

template <bool STAGED>
__global__ __launch_bounds__(256) void gather_kernel(GatherArgs a) {
  __shared__ float rec_lds[STAGED ? 4 : 1][STAGED ? kMaxRecord : 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = blockIdx.x * 4 + wave;
  if (row >= a.Bp) return;
  const bool live = row < a.B;
  if constexpr (STAGED) {
    float* lr = rec_lds[wave];
    if (live) {
      const int64_t idx = gather_row_index(a, row);
      const float4* src = reinterpret_cast<const float4*>(a.data + (size_t)idx * a.rec);
      // All of the row's loads are issued before the first LDS write: a runtime-trip loop
      // waits out one HBM round trip per 64 float4 (4 serial trips for a 3 KB record).
      constexpr int kPer = kMaxRecord / 4 / 64;
      const int n4 = a.rec >> 2;
      float4 v[kPer];
#pragma unroll
      for (int i = 0; i < kPer; ++i) v[i] = src[min(lane + 64 * i, n4 - 1)];  // unguarded: clamped
#pragma unroll  // unguarded too (the slot holds kMaxRecord floats), or the loads sink into the guards
      for (int i = 0; i < kPer; ++i) reinterpret_cast<float4*>(lr)[lane + 64 * i] = v[i];
      if (a.idx_out && lane == 0) a.idx_out[row] = idx;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    for (int s = 0; s < a.nseg; ++s) {
      const GatherSeg g = a.seg[s];
      float* d = g.dst + (size_t)row * g.ld + g.col;
      const float* l = lr + g.src;
      const int n4 = (reinterpret_cast<uintptr_t>(d) & 15) == 0 ? (g.len >> 2) : 0;
      for (int q = lane; q < n4; q += 64) {
        const float4 v = live ? make_float4(l[4 * q], l[4 * q + 1], l[4 * q + 2], l[4 * q + 3])
                              : make_float4(0.f, 0.f, 0.f, 0.f);
        reinterpret_cast<float4*>(d)[q] = v;
      }
      for (int c = 4 * n4 + lane; c < g.len; c += 64) d[c] = live ? l[c] : 0.f;
    }
  } else {
    const float* src = nullptr;
    if (live) {
      const int64_t idx = gather_row_index(a, row);
      if (a.idx_out && lane == 0) a.idx_out[row] = idx;
      src = a.data + (size_t)idx * a.rec;
    }
    for (int s = 0; s < a.nseg; ++s) {
      const GatherSeg g = a.seg[s];
      float* d = g.dst + (size_t)row * g.ld + g.col;
      for (int c = lane; c < g.len; c += 64) d[c] = src ? src[g.src + c] : 0.f;
    }
  }
}

int launch_gather(const GatherArgs& a, hipStream_t s) {
  if (a.Bp <= 0) return 0;
  dim3 grid((a.Bp + 3) / 4);
  if (a.rec <= kMaxRecord) hipLaunchKernelGGL(gather_kernel<true>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(gather_kernel<false>, grid, dim3(256), 0, s, a);
  TD3_HIP(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------ synthetic fill
// state, next_state ~ N(0,1); action ~ U(-max_action, max_action);
// reward ~ N(0,1); not_done = 1 with probability 0.99.  Philox keyed by (seed, row).
__global__ __launch_bounds__(256) void fill_kernel(float* data, int rec, int o_a, int ad, int o_r,
                                                   int o_nd, int64_t start, int64_t n, int64_t cap,
                                                   float max_action, uint64_t seed) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const int64_t slot = (start + i) % cap;
  float* r = data + (size_t)slot * rec;
  for (int c0 = lane * 4; c0 < rec; c0 += 256) {
    float z[4];
    philox_normal4(seed, (uint64_t)i, kStreamFill, (uint32_t)c0, z);
    u32x4 u = philox4x32_10(u32x4{(uint32_t)c0, kStreamFill + 7u, (uint32_t)i, (uint32_t)(i >> 32)},
                            (uint32_t)seed, (uint32_t)(seed >> 32));
    uint32_t uu[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = c0 + j;
      if (c >= rec) break;
      float v;
      if (c > o_nd) v = 0.f;                                            // record pad
      else if (c == o_nd) v = ((float)(uu[j] >> 8) * (1.f / 16777216.f)) < 0.01f ? 0.f : 1.f;
      else if (c >= o_a && c < o_a + ad)
        v = max_action * (2.f * ((float)(uu[j] >> 8) * (1.f / 16777216.f)) - 1.f);
      else v = z[j];                                                    // states, particles, reward
      r[c] = v;
    }
  }
  (void)o_r;
}

__global__ void set_i64_kernel(int64_t* p, int64_t v) { *p = v; }

// Small adds: n staged records, read in place from mapped pinned host memory, into the ring rows
// ptr, ptr+1, ... (wrapping), and the new size -- one launch instead of a DMA copy per ring
// segment plus the size update.  rec is a multiple of 4 (replay.h), so records move as float4.
__global__ __launch_bounds__(256) void ring_put_kernel(float4* __restrict__ data, int64_t cap, int rec4,
                                                       const float4* __restrict__ src, int64_t n, int64_t ptr,
                                                       int64_t* d_size, int64_t new_size) {
  const int64_t total = n * rec4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / rec4, c = i - row * rec4;
    int64_t dst = ptr + row;
    if (dst >= cap) dst -= cap;
    data[dst * rec4 + c] = src[i];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *d_size = new_size;
}

// Adds of a few records travel in the kernel arguments (no host staging buffer whose reuse would
// need an event): rows [0, n) of `rows` (rec floats each) into ring rows ptr, ptr+1, .. (wrapping).
constexpr int kPutArgFloats = 960;
struct RingPutArgs {
  float4* data;
  int64_t* d_size;
  int64_t cap, ptr, n, new_size;
  int rec4;
  float rows[kPutArgFloats];
};
__global__ __launch_bounds__(256) void ring_put_args_kernel(RingPutArgs a) {
  const int64_t total = a.n * a.rec4;
  for (int64_t i = threadIdx.x; i < total; i += 256) {
    const int64_t row = i / a.rec4, c = i - row * a.rec4;
    int64_t dst = a.ptr + row;
    if (dst >= a.cap) dst -= a.cap;
    a.data[dst * a.rec4 + c] = reinterpret_cast<const float4*>(a.rows)[i];
  }
  if (threadIdx.x == 0) *a.d_size = a.new_size;
}

// The lazy ordering of Ring::read_stream / write_stream: when `s` differs from the noted stream,
// an event recorded there now (it covers everything queued so far) is waited on by `s`.
static int order_after(hipStream_t s, hipStream_t noted, bool pending, hipEvent_t ev, hipStream_t& seen_by) {
  if (!pending || !noted || noted == s || seen_by == s) return 0;
  TD3_HIP(hipEventRecord(ev, noted));
  TD3_HIP(hipStreamWaitEvent(s, ev, 0));
  seen_by = s;
  return 0;
}

static std::mutex g_rings_mu;
static std::set<Ring*> g_rings;

void ring_forget_stream(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_rings_mu);
  for (Ring* r : g_rings) {
    if (r->read_stream == s) {
      r->read_stream = nullptr;
      r->reads_pending = false;
    }
    if (r->write_stream == s) {
      r->write_stream = nullptr;
      r->writes_pending = false;
    }
    if (r->reads_seen_by == s) r->reads_seen_by = nullptr;
    if (r->writes_seen_by == s) r->writes_seen_by = nullptr;
  }
}

int ring_begin_read(Ring* r, hipStream_t s) {
  TD3_RC(order_after(s, r->write_stream, r->writes_pending, r->write_ev, r->writes_seen_by));  // adds so far
  TD3_RC(order_after(s, r->read_stream, r->reads_pending, r->read_ev, r->reads_seen_by));     // chained readers
  return 0;
}

int ring_end_read(Ring* r, hipStream_t s) {
  r->read_stream = s;
  r->reads_pending = true;
  r->reads_seen_by = nullptr;
  return 0;
}

bool ring_alive(const Ring* r, uint64_t gen) {
  std::lock_guard<std::mutex> lk(g_rings_mu);
  return r && g_rings.count(const_cast<Ring*>(r)) && r->gen == gen;
}

}  // namespace td3

using namespace td3;

// ================================================================== C-ABI
extern "C" {

static std::atomic<uint64_t> g_ring_gen{0};

static int ring_alloc(Ring* r, int64_t max_size, int device, uint64_t seed, rb_handle** out) {
  r->gen = ++g_ring_gen;
  r->cap = max_size;
  r->seed = seed;
  r->device = device;
  hipError_t e = hipMalloc(&r->data, (size_t)max_size * r->rec * sizeof(float));
  if (e != hipSuccess) {
    set_error("rb_create: hipMalloc(%zu bytes) failed: %s",
              (size_t)max_size * r->rec * sizeof(float), hipGetErrorString(e));
    delete r;
    return -2;
  }
  TD3_HIP(hipMemset(r->data, 0, (size_t)max_size * r->rec * sizeof(float)));
  TD3_HIP(hipMalloc(&r->d_size, sizeof(int64_t)));
  TD3_HIP(hipMemset(r->d_size, 0, sizeof(int64_t)));
  // the memsets ran on the null stream, which does not order the ring's non-blocking stream:
  // finish them before any add / sample can be queued
  TD3_HIP(hipDeviceSynchronize());
  TD3_HIP(hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking));
  TD3_HIP(hipEventCreateWithFlags(&r->write_ev, TD3_EV_FLAGS));
  TD3_HIP(hipEventCreateWithFlags(&r->read_ev, TD3_EV_FLAGS));
  for (auto& ev : r->stage_buf_ev) TD3_HIP(hipEventCreateWithFlags(&ev, TD3_EV_FLAGS));
  {
    std::lock_guard<std::mutex> lk(g_rings_mu);
    g_rings.insert(r);
  }
  *out = reinterpret_cast<rb_handle*>(r);
  return 0;
}

int rb_create(int state_dim, int action_dim, int64_t max_size, int device, uint64_t seed,
              rb_handle** out) {
  TD3_ARG(out != nullptr, "out is null");
  TD3_ARG(state_dim > 0 && action_dim > 0, "dims must be positive");
  TD3_ARG(pad4(2 * state_dim + action_dim + 2) <= kMaxRecord, "record too wide");
  TD3_ARG(max_size > 0, "max_size must be positive");
  TD3_HIP(hipSetDevice(device));
  Ring* r = new Ring();
  r->sd = state_dim;
  r->ad = action_dim;
  r->o_s = 0;
  r->o_a = state_dim;
  r->o_s2 = state_dim + action_dim;
  r->o_r = 2 * state_dim + action_dim;
  r->o_nd = r->o_r + 1;
  r->rec = pad4(2 * state_dim + action_dim + 2);
  return ring_alloc(r, max_size, device, seed, out);
}

int rb_create_particles(int feat_dim, int n_particles, int particle_dim, int action_dim, int64_t max_size,
                        int device, uint64_t seed, rb_handle** out) {
  TD3_ARG(out != nullptr, "out is null");
  TD3_ARG(feat_dim > 0 && n_particles > 0 && particle_dim > 0 && action_dim > 0, "dims must be positive");
  TD3_ARG(max_size > 0, "max_size must be positive");
  TD3_HIP(hipSetDevice(device));
  Ring* r = new Ring();
  const int np = n_particles * particle_dim;
  r->particles = 1;
  r->N = n_particles;
  r->D = particle_dim;
  r->sd = feat_dim;
  r->ad = action_dim;
  r->o_s = 0;
  r->o_p = feat_dim;
  r->o_a = feat_dim + np;
  r->o_s2 = r->o_a + action_dim;
  r->o_p2 = r->o_s2 + feat_dim;
  r->o_r = r->o_p2 + np;
  r->o_nd = r->o_r + 1;
  r->rec = pad4(r->o_nd + 1);
  return ring_alloc(r, max_size, device, seed, out);
}

int rb_destroy(rb_handle* h) {
  if (!h) return 0;
  Ring* r = reinterpret_cast<Ring*>(h);
  (void)hipSetDevice(r->device);
  {
    std::lock_guard<std::mutex> lk(g_rings_mu);
    g_rings.erase(r);
  }
  // no reader or writer of the ring still in flight, whatever stream it was queued on
  (void)hipDeviceSynchronize();
  (void)hipFree(r->data);
  (void)hipFree(r->d_size);
  (void)hipFree(r->d_idx);
  for (int i = 0; i < 2; ++i) {
    if (r->stage_buf_ev[i]) (void)hipEventSynchronize(r->stage_buf_ev[i]);
    if (r->stage[i]) (void)hipHostFree(r->stage[i]);
    (void)hipEventDestroy(r->stage_buf_ev[i]);
  }
  (void)hipEventDestroy(r->write_ev);
  (void)hipEventDestroy(r->read_ev);
  (void)hipStreamDestroy(r->stream);
  delete r;
  return 0;
}

void* rb_stream(rb_handle* h) { return h ? (void*)reinterpret_cast<Ring*>(h)->stream : nullptr; }

int rb_info(const rb_handle* h, rb_info_t* info) {
  TD3_ARG(h && info, "null handle");
  const Ring* r = reinterpret_cast<const Ring*>(h);
  info->state_dim = r->sd;
  info->action_dim = r->ad;
  info->record_floats = r->rec;
  info->max_size = r->cap;
  info->ptr = r->ptr;
  info->size = r->size;
  info->data = r->data;
  info->device = r->device;
  info->n_particles = r->N;
  info->particle_dim = r->D;
  return 0;
}

// Pinned staging for the next add: alternate between two buffers so the host packs the next
// rows while the previous upload (which may be waiting behind a step that reads the ring) is
// still queued; only the upload before that one must have consumed its buffer.
static float* ensure_stage(Ring* r, size_t floats) {
  const int i = r->stage_cur;
  r->stage_cur ^= 1;
  if (hipEventSynchronize(r->stage_buf_ev[i]) != hipSuccess) return nullptr;
  if (floats > r->stage_cap[i]) {
    if (r->stage[i]) (void)hipHostFree(r->stage[i]);
    r->stage[i] = nullptr;
    r->stage_cap[i] = 0;
    const size_t cap = std::max(floats, (size_t)r->rec * 4096);
    hipError_t e = hipHostMalloc(&r->stage[i], cap * sizeof(float), hipHostMallocMapped);
    void* d = nullptr;
    if (e == hipSuccess) e = hipHostGetDevicePointer(&d, r->stage[i], 0);
    if (e != hipSuccess) {
      set_error("rb_add: hipHostMalloc(%zu bytes) failed: %s", cap * sizeof(float), hipGetErrorString(e));
      return nullptr;
    }
    r->stage_dev[i] = static_cast<float*>(d);
    r->stage_cap[i] = cap;
  }
  return r->stage[i];
}

static int stage_index(const Ring* r, const float* host) {
  for (int i = 0; i < 2; ++i)
    if (host == r->stage[i]) return i;
  return -1;
}

// Writes (records, d_size) on `stream` start after every read and every other-stream write queued
// so far (Ring::read_stream / write_stream).
static int ring_begin_write(Ring* r, hipStream_t stream) {
  TD3_RC(order_after(stream, r->read_stream, r->reads_pending, r->read_ev, r->reads_seen_by));
  TD3_RC(order_after(stream, r->write_stream, r->writes_pending, r->write_ev, r->writes_seen_by));
  return 0;
}

static int ring_end_write(Ring* r, hipStream_t stream) {
  r->write_stream = stream;
  r->writes_pending = true;
  r->writes_seen_by = nullptr;
  return 0;
}

constexpr size_t kPutKernelBytes = 256 << 10;   // adds up to this size take ring_put_kernel

// Copy n packed records (host staging) into the ring at ptr, wrapping (the ring
// semantics of my_replay_buffer.py:115-116 applied n times).
static int push_staged(Ring* r, const float* host, int64_t n, hipStream_t stream) {
  TD3_RC(ring_begin_write(r, stream));
  const int si = stage_index(r, host);
  int64_t done = 0;
  // Only the last `cap` records survive when n > cap.
  int64_t skip = 0;
  if (n > r->cap) {
    skip = n - r->cap;
    r->ptr = (r->ptr + skip) % r->cap;
    n = r->cap;
    r->size = r->cap;
  }
  const int64_t new_size = std::min<int64_t>(r->size + n, r->cap);
  if ((int64_t)n * r->rec <= kPutArgFloats) {       // the records in the kernel arguments
    RingPutArgs pa;
    pa.data = reinterpret_cast<float4*>(r->data);
    pa.d_size = r->d_size;
    pa.cap = r->cap;
    pa.ptr = r->ptr;
    pa.n = n;
    pa.new_size = new_size;
    pa.rec4 = r->rec / 4;
    memcpy(pa.rows, host + (size_t)skip * r->rec, (size_t)n * r->rec * sizeof(float));
    hipLaunchKernelGGL(ring_put_args_kernel, dim3(1), dim3(256), 0, stream, pa);
    TD3_HIP(hipGetLastError());
    r->ptr = (r->ptr + n) % r->cap;
    r->size = new_size;
    return ring_end_write(r, stream);
  }
  if (si >= 0 && (size_t)n * r->rec * sizeof(float) <= kPutKernelBytes) {
    const int64_t total4 = n * (r->rec / 4);
    const int grid = (int)std::min<int64_t>((total4 + 255) / 256, 256);
    hipLaunchKernelGGL(ring_put_kernel, dim3(grid), dim3(256), 0, stream, reinterpret_cast<float4*>(r->data),
                       r->cap, r->rec / 4, reinterpret_cast<const float4*>(r->stage_dev[si] + (size_t)skip * r->rec),
                       n, r->ptr, r->d_size, new_size);
    TD3_HIP(hipGetLastError());
    r->ptr = (r->ptr + n) % r->cap;
  } else {
    const float* src = host + (size_t)skip * r->rec;
    while (done < n) {
      int64_t chunk = std::min<int64_t>(n - done, r->cap - r->ptr);
      TD3_HIP(hipMemcpyAsync(r->data + (size_t)r->ptr * r->rec, src + (size_t)done * r->rec,
                             (size_t)chunk * r->rec * sizeof(float), hipMemcpyHostToDevice, stream));
      r->ptr = (r->ptr + chunk) % r->cap;
      done += chunk;
    }
    hipLaunchKernelGGL(set_i64_kernel, dim3(1), dim3(1), 0, stream, r->d_size, new_size);
    TD3_HIP(hipGetLastError());
  }
  r->size = new_size;
  if (si >= 0) TD3_HIP(hipEventRecord(r->stage_buf_ev[si], stream));   // the staging buffer is free
  return ring_end_write(r, stream);
}

int rb_add(rb_handle* h, const double* state, const double* action, const double* next_state,
           const double* reward, const double* done, int64_t n, void* stream) {
  TD3_ARG(h != nullptr, "null handle");
  TD3_ARG(n >= 0, "n must be >= 0");
  if (n == 0) return 0;
  TD3_ARG(state && action && next_state && reward && done, "null input");
  Ring* r = reinterpret_cast<Ring*>(h);
  TD3_ARG(!r->particles, "rb_add on a particle ring (use rb_add_particles)");
  TD3_HIP(hipSetDevice(r->device));
  float small[kPutArgFloats];                      // few records: packed here, shipped as launch arguments
  const bool few = n * r->rec <= kPutArgFloats;
  float* stage = few ? small : ensure_stage(r, (size_t)n * r->rec);
  if (!stage) return -2;
  for (int64_t i = 0; i < n; ++i) {
    float* d = stage + (size_t)i * r->rec;
    for (int c = 0; c < r->sd; ++c) d[r->o_s + c] = (float)state[i * r->sd + c];
    for (int c = 0; c < r->ad; ++c) d[r->o_a + c] = (float)action[i * r->ad + c];
    for (int c = 0; c < r->sd; ++c) d[r->o_s2 + c] = (float)next_state[i * r->sd + c];
    d[r->o_r] = (float)reward[i];
    d[r->o_nd] = (float)(1.0 - done[i]);                  // my_replay_buffer.py:114
    for (int c = r->o_nd + 1; c < r->rec; ++c) d[c] = 0.f;
  }
  hipStream_t s = stream ? (hipStream_t)stream : r->stream;
  return push_staged(r, stage, n, s);
}

int rb_add_particles(rb_handle* h, const double* feat, const double* part, const double* action,
                     const double* next_feat, const double* next_part, const double* reward,
                     const double* done, int64_t n, void* stream) {
  TD3_ARG(h != nullptr, "null handle");
  TD3_ARG(n >= 0, "n must be >= 0");
  if (n == 0) return 0;
  TD3_ARG(feat && part && action && next_feat && next_part && reward && done, "null input");
  Ring* r = reinterpret_cast<Ring*>(h);
  TD3_ARG(r->particles, "rb_add_particles on a featured ring");
  TD3_HIP(hipSetDevice(r->device));
  float* stage = ensure_stage(r, (size_t)n * r->rec);
  if (!stage) return -2;
  const int np = r->N * r->D;
  for (int64_t i = 0; i < n; ++i) {                        // my_replay_buffer.py:46-56
    float* d = stage + (size_t)i * r->rec;
    for (int c = 0; c < r->sd; ++c) d[r->o_s + c] = (float)feat[i * r->sd + c];
    for (int c = 0; c < np; ++c) d[r->o_p + c] = (float)part[i * np + c];
    for (int c = 0; c < r->ad; ++c) d[r->o_a + c] = (float)action[i * r->ad + c];
    for (int c = 0; c < r->sd; ++c) d[r->o_s2 + c] = (float)next_feat[i * r->sd + c];
    for (int c = 0; c < np; ++c) d[r->o_p2 + c] = (float)next_part[i * np + c];
    d[r->o_r] = (float)reward[i];
    d[r->o_nd] = (float)(1.0 - done[i]);
    for (int c = r->o_nd + 1; c < r->rec; ++c) d[c] = 0.f;
  }
  hipStream_t s = stream ? (hipStream_t)stream : r->stream;
  return push_staged(r, stage, n, s);
}

int rb_add_records(rb_handle* h, const float* records, int64_t n, void* stream) {
  TD3_ARG(h != nullptr, "null handle");
  TD3_ARG(n >= 0, "n must be >= 0");
  if (n == 0) return 0;
  TD3_ARG(records != nullptr, "null records");
  Ring* r = reinterpret_cast<Ring*>(h);
  TD3_HIP(hipSetDevice(r->device));
  hipStream_t s = stream ? (hipStream_t)stream : r->stream;
  if (n * r->rec <= kPutArgFloats) return push_staged(r, records, n, s);   // launch arguments
  float* stage = ensure_stage(r, (size_t)n * r->rec);
  if (!stage) return -2;
  memcpy(stage, records, (size_t)n * r->rec * sizeof(float));
  return push_staged(r, stage, n, s);
}

int rb_fill_synthetic(rb_handle* h, int64_t n, float max_action, uint64_t seed, void* stream) {
  TD3_ARG(h != nullptr, "null handle");
  TD3_ARG(n >= 0, "n must be >= 0");
  Ring* r = reinterpret_cast<Ring*>(h);
  TD3_HIP(hipSetDevice(r->device));
  hipStream_t s = stream ? (hipStream_t)stream : r->stream;
  if (n > r->cap) n = r->cap;
  TD3_RC(ring_begin_write(r, s));
  if (n > 0) {
    dim3 grid((unsigned)((n + 3) / 4));
    hipLaunchKernelGGL(fill_kernel, grid, dim3(256), 0, s, r->data, r->rec, r->o_a, r->ad, r->o_r, r->o_nd,
                       r->ptr, n, r->cap, max_action, seed);
    TD3_HIP(hipGetLastError());
  }
  r->ptr = (r->ptr + n) % r->cap;
  r->size = std::min<int64_t>(r->size + n, r->cap);
  hipLaunchKernelGGL(set_i64_kernel, dim3(1), dim3(1), 0, s, r->d_size, r->size);
  TD3_HIP(hipGetLastError());
  return ring_end_write(r, s);
}

int rb_sample(rb_handle* h, int batch, float* state, float* action, float* next_state,
              float* reward, float* not_done, const int64_t* inject_idx, int64_t* idx_out,
              void* stream) {
  TD3_ARG(h != nullptr, "null handle");
  Ring* r = reinterpret_cast<Ring*>(h);
  TD3_ARG(!r->particles, "rb_sample on a particle ring (use rb_sample_particles)");
  TD3_ARG(batch >= 0, "batch must be >= 0");
  TD3_ARG(r->size > 0 || batch == 0 || inject_idx, "sample from an empty buffer");
  TD3_ARG(state && action && next_state && reward && not_done, "null output");
  TD3_HIP(hipSetDevice(r->device));
  GatherArgs a{};
  a.seg[0] = GatherSeg{state, r->sd, 0, r->o_s, r->sd};
  a.seg[1] = GatherSeg{action, r->ad, 0, r->o_a, r->ad};
  a.seg[2] = GatherSeg{next_state, r->sd, 0, r->o_s2, r->sd};
  a.seg[3] = GatherSeg{reward, 1, 0, r->o_r, 1};
  a.seg[4] = GatherSeg{not_done, 1, 0, r->o_nd, 1};
  a.nseg = 5;
  a.B = a.Bp = batch;
  a.data = r->data;
  a.rec = r->rec;
  a.d_size = r->d_size;
  a.inject_idx = inject_idx;
  a.idx_out = idx_out;
  a.seed = r->seed;
  a.ctr = nullptr;
  a.step = ++r->sample_calls;
  hipStream_t s = stream ? (hipStream_t)stream : r->stream;
  TD3_RC(ring_begin_read(r, s));                     // add() before sample() (main.py:261, :269)
  TD3_RC(launch_gather(a, s));
  return ring_end_read(r, s);
}

int rb_sample_particles(rb_handle* h, int batch, float* feat, float* part, float* action, float* next_feat,
                        float* next_part, float* reward, float* not_done, const int64_t* inject_idx,
                        int64_t* idx_out, void* stream) {
  TD3_ARG(h != nullptr, "null handle");
  Ring* r = reinterpret_cast<Ring*>(h);
  TD3_ARG(r->particles, "rb_sample_particles on a featured ring");
  TD3_ARG(batch >= 0, "batch must be >= 0");
  TD3_ARG(r->size > 0 || batch == 0 || inject_idx, "sample from an empty buffer");
  TD3_ARG(feat && part && action && next_feat && next_part && reward && not_done, "null output");
  TD3_HIP(hipSetDevice(r->device));
  const int np = r->N * r->D;
  GatherArgs a{};
  a.seg[0] = GatherSeg{feat, r->sd, 0, r->o_s, r->sd};
  a.seg[1] = GatherSeg{part, np, 0, r->o_p, np};
  a.seg[2] = GatherSeg{action, r->ad, 0, r->o_a, r->ad};
  a.seg[3] = GatherSeg{next_feat, r->sd, 0, r->o_s2, r->sd};
  a.seg[4] = GatherSeg{next_part, np, 0, r->o_p2, np};
  a.seg[5] = GatherSeg{reward, 1, 0, r->o_r, 1};
  a.seg[6] = GatherSeg{not_done, 1, 0, r->o_nd, 1};
  a.nseg = 7;
  a.B = a.Bp = batch;
  a.data = r->data;
  a.rec = r->rec;
  a.d_size = r->d_size;
  a.inject_idx = inject_idx;
  a.idx_out = idx_out;
  a.seed = r->seed;
  a.ctr = nullptr;
  a.step = ++r->sample_calls;
  hipStream_t s = stream ? (hipStream_t)stream : r->stream;
  TD3_RC(ring_begin_read(r, s));                     // add() before sample() (main.py:261, :269)
  TD3_RC(launch_gather(a, s));
  return ring_end_read(r, s);
}

int rb_read_records(const rb_handle* h, int64_t start, int64_t n, float* out) {
  TD3_ARG(h && out, "null argument");
  const Ring* r = reinterpret_cast<const Ring*>(h);
  TD3_ARG(start >= 0 && n >= 0 && start + n <= r->cap, "range out of bounds");
  TD3_HIP(hipSetDevice(r->device));
  TD3_HIP(hipStreamSynchronize(r->stream));
  TD3_HIP(hipDeviceSynchronize());
  TD3_HIP(hipMemcpy(out, r->data + (size_t)start * r->rec, (size_t)n * r->rec * sizeof(float),
                    hipMemcpyDeviceToHost));
  return 0;
}

int rb_write_records(rb_handle* h, int64_t start, int64_t n, const float* in, int64_t ptr,
                     int64_t size) {
  TD3_ARG(h && in, "null argument");
  Ring* r = reinterpret_cast<Ring*>(h);
  TD3_ARG(start >= 0 && n >= 0 && start + n <= r->cap, "range out of bounds");
  TD3_ARG(ptr >= 0 && ptr < r->cap && size >= 0 && size <= r->cap, "ptr/size out of bounds");
  TD3_HIP(hipSetDevice(r->device));
  TD3_HIP(hipDeviceSynchronize());
  TD3_HIP(hipMemcpy(r->data + (size_t)start * r->rec, in, (size_t)n * r->rec * sizeof(float),
                    hipMemcpyHostToDevice));
  r->ptr = ptr;
  r->size = size;
  TD3_HIP(hipMemcpy(r->d_size, &r->size, sizeof(int64_t), hipMemcpyHostToDevice));
  return 0;
}

int rb_sync(rb_handle* h) {
  TD3_ARG(h != nullptr, "null handle");
  Ring* r = reinterpret_cast<Ring*>(h);
  TD3_HIP(hipSetDevice(r->device));
  TD3_HIP(hipStreamSynchronize(r->stream));
  if (r->write_stream) TD3_HIP(hipStreamSynchronize(r->write_stream));   // adds flushed by a learner
  if (r->read_stream) TD3_HIP(hipStreamSynchronize(r->read_stream));
  return 0;
}

}  // extern "C"
