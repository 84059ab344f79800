// HBM-resident replay ring (device side of my_replay_buffer.ReplayBuffer_*).
#pragma once
#include "common.h"

namespace td3 {

// One transition = one AoS record of `rec` floats in HBM:
//   [ state(sd) | action(ad) | next_state(sd) | reward | not_done | pad to 16 B ]
// (the reference keeps 5 float64 SoA arrays, my_replay_buffer.py:81-85; one
// record per row makes the sample gather one contiguous read per index).
// TD3_particles rings (ReplayBuffer_particles, my_replay_buffer.py:6-69) use the record
//   [ features(F) | particles(N*D) | action(A) | next_features(F) | next_particles(N*D) |
//     reward | not_done | pad ]
// with sd = F, ad = A; the learner's encoder reads the particle blocks in place (no gather).
struct Ring {
  uint64_t gen = 0;                // unique per allocation: captured graphs bake this ring in
  int sd = 0, ad = 0;
  int rec = 0;
  int o_s = 0, o_a = 0, o_s2 = 0, o_r = 0, o_nd = 0;
  int particles = 0, N = 0, D = 0;  // particle rings only
  int o_p = 0, o_p2 = 0;
  int64_t cap = 0;
  int64_t ptr = 0, size = 0;       // host mirror of my_replay_buffer.py:76-77
  float* data = nullptr;           // [cap][rec]
  int64_t* d_size = nullptr;       // device copy of `size` (read by graph-replayed sample)
  uint64_t seed = 0;
  uint64_t sample_calls = 0;       // Philox counter of the stand-alone sample()
  int device = 0;
  hipStream_t stream = nullptr;
  float* stage[2] = {nullptr, nullptr};     // pinned host staging for add(), double-buffered
  float* stage_dev[2] = {nullptr, nullptr}; // their device addresses (small adds read them in place)
  size_t stage_cap[2] = {0, 0};
  hipEvent_t stage_buf_ev[2] = {nullptr, nullptr};  // the write out of stage[i] finished
  int stage_cur = 0;
  hipEvent_t stage_ev = nullptr;   // recorded after writes that use no staging buffer
  hipEvent_t last_write = nullptr; // the last write (records + d_size), stage_ev or a stage_buf_ev:
                                   // readers wait on it
  // Ordering of writes after reads.  Every reader (a learner step, a stand-alone sample) records
  // read_ev on its stream after the work that reads the records or d_size; a later write waits on
  // it, so a step in flight never sees d_size or a record change under it.  Readers on different
  // streams are chained (the new reader waits on read_ev first), so read_ev covers them all.
  hipEvent_t read_ev = nullptr;
  const void* read_stream = nullptr;        // stream of the last read_ev record (compared only)
  int64_t* d_idx = nullptr;        // last drawn indices (rows) of sample()
  int idx_cap = 0;
};

// Reader protocol (see Ring::read_ev): ring_begin_read before enqueuing reads on s (waits on
// the last write and, on a new stream, on the previous readers), ring_end_read after them.
int ring_begin_read(Ring* r, hipStream_t s);
int ring_end_read(Ring* r, hipStream_t s);

// One gather destination: rows [0, Bp) of dst[r*ld + col + c] = record[src + c], c < len.
struct GatherSeg {
  float* dst;
  int ld, col, src, len;
};

constexpr int kMaxSegs = 12;
constexpr int kMaxRecord = 2048;   // records up to this width are staged whole in LDS; wider
                                   // records (particle rings) are gathered segment by segment
struct GatherArgs {
  GatherSeg seg[kMaxSegs];
  int nseg;
  int B, Bp;
  const float* data;
  int rec;
  const int64_t* d_size;        // sample range [0, *d_size)
  const int64_t* inject_idx;    // nullable: use these rows instead of Philox
  int64_t* idx_out;             // nullable: record drawn rows
  uint64_t seed;
  const Counters* ctr;          // nullable: Philox step = ctr->total_it + 1
  uint64_t step;                // used when ctr == nullptr
};

int launch_gather(const GatherArgs& a, hipStream_t s);

}  // namespace td3
