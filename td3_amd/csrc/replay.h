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
  float* stage[2] = {nullptr, nullptr};     // pinned host staging for large adds, double-buffered
  float* stage_dev[2] = {nullptr, nullptr}; // their device addresses
  size_t stage_cap[2] = {0, 0};
  hipEvent_t stage_buf_ev[2] = {nullptr, nullptr};  // the write out of stage[i] finished
  int stage_cur = 0;
  // Ordering between the streams that read (a learner step, a stand-alone sample) and write
  // (adds, fills) the ring, recorded lazily: an access only notes its stream; an access on ANOTHER
  // stream records an event on the noted stream at that moment (covering everything queued there
  // so far) and waits on it.  Accesses on one stream need nothing (stream order), so a learner
  // that also flushes the adds on its own stream records no event per step -- a record is a
  // marker packet that drains the queue: ~4 us of GPU time per step (C2 9.60k vs 9.97k steps/s).
  // Readers are chained (a reader on a new stream waits on the previous one's), so the last
  // read stream covers them all; writes likewise.
  hipStream_t read_stream = nullptr, write_stream = nullptr;
  bool reads_pending = false, writes_pending = false;
  // the stream already ordered after the current reads / writes (nothing to wait for again)
  hipStream_t reads_seen_by = nullptr, writes_seen_by = nullptr;
  hipEvent_t read_ev = nullptr, write_ev = nullptr;
  int64_t* d_idx = nullptr;        // last drawn indices (rows) of sample()
  int idx_cap = 0;
};

// Reader protocol (Ring::read_stream): ring_begin_read before enqueuing reads on s (orders them
// after the writes and the earlier readers of other streams), ring_end_read after them.
int ring_begin_read(Ring* r, hipStream_t s);
int ring_end_read(Ring* r, hipStream_t s);
// A stream that is about to be destroyed (synchronised by the caller) stops being a ring's
// noted reader / writer.
void ring_forget_stream(hipStream_t s);
// True while `r` is a live ring of allocation generation `gen` (not destroyed, not reused).
bool ring_alive(const Ring* r, uint64_t gen);

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
