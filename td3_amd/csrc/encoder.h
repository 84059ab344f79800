// Particle set encoder of TD3_particles (device side): the per-particle two-layer MLP
// (conv1 1xD -> ReLU -> conv2 1x1 -> ReLU), the mean over particles and its backward.
//
// Reference (/root/reference/TD3_particles.py): Actor.__init__ :29-32 / forward :52-58,
// Q_network.__init__ :80-83 / forward :103-109.  AvgPool2d((1, N)) on the 3-D conv2 output
// pools over the particle axis; a ReLU follows the pool (:57 / :107).
#pragma once
#include "common.h"
#include "kernels.h"

namespace td3 {

constexpr int kEncC1 = 256;      // conv1 channels   (num_features * 2, TD3_particles.py:29)
constexpr int kEncC2 = 128;      // conv2 channels   (num_features)
constexpr int kEncMaxD = 16;     // particle feature width the kernels stage (D <= 16)
constexpr int kMaxEnc = 6;       // encoder evaluations per launch

// Encoder parameters inside a group arena, reference state_dict order:
//   conv1.weight [256][1][1][D] | conv1.bias [256] | conv2.weight [128][256][1] | conv2.bias [128]
struct EncOff {
  static __host__ __device__ inline int64_t w1(int) { return 0; }
  static __host__ __device__ inline int64_t b1(int D) { return (int64_t)kEncC1 * D; }
  static __host__ __device__ inline int64_t w2(int D) { return (int64_t)kEncC1 * D + kEncC1; }
  static __host__ __device__ inline int64_t b2(int D) { return w2(D) + (int64_t)kEncC2 * kEncC1; }
  static __host__ __device__ inline int64_t size(int D) { return b2(D) + kEncC2; }
};

// ---------------------------------------------------------------- forward
struct EncFwdProb {
  const float* enc;        // encoder parameter block (EncOff layout)
  int part_off;            // float offset of the [N][D] particle block inside a record
  float* out; int ldo;     // pooled features -> out[b * ldo + c], c < 128
  uint64_t* mask;          // nullable: ReLU bits for the backward: conv2 [Bp][ntile][64] words
                           // (word j*16+r: channel tile j, MFMA reg r), then conv1
                           // [Bp][ntile][2][64] words (half g, lane L = 16(c&3) + r of chunk
                           // c = 4g + L/16: channel 32c + crow(r) low / + 4 high, crow(r) =
                           // (r&3) + 8(r>>2), bit R = tile row R), then float counts of the
                           // positive conv2 rows [Bp][128]
};

struct EncFwdArgs {
  EncFwdProb p[kMaxEnc];
  int nprob;
  const float* data; int rec;   // ring records (or a packed [n][N*D] batch with rec = N*D)
  const int64_t* idx;           // record of each batch row
  int B, Bp, N, D, ntile;       // ntile = ceil(N / 32)
};

// ---------------------------------------------------------------- backward
// Role A workgroups: dh1 = dz2 * W2 (MFMA), dz1 = relu'(z1) dh1 (the forward's conv1 bits),
// dW1 = dz1^T x (MFMA), db1.
// Role B workgroups: dW2 = dz2^T h1 (MFMA, h1 recomputed into LDS), db2 (mask popcounts).
// dz2[n][c] = mask[n][c] * gpool[b][c] / N, gpool = relu'(pooled) * (LN_in backward of the MLP
// input grad)[0..127].  Each workgroup owns a contiguous range of batch rows and writes its
// partial sums to its own slab; enc_adam_kernel reduces the slabs in a fixed order.
struct EncBwdProb {
  const float* enc;
  int part_off;
  const uint64_t* mask;
  const float* X; int ldx;          // MLP input rows [pooled | features | action]
  const float* GU; int ldgu;        // grad of the lnorm1 output (or of X when norm is None)
  const float* stats;               // lnorm1 (mean, rstd) [2][Bp]; nullable: norm None
  const float* gamma;               // lnorm1 weight
  int Kin;                          // real width of the MLP input row
  float* partial;                   // [nwg][EncOff::size(D)]
  float* gpool;                     // [Bp][128] dz2 row scale: relu'(pooled) * dpooled / N
};

struct EncBwdArgs {
  EncBwdProb p[3];
  int nprob;
  const float* data; int rec;
  const int64_t* idx;
  int B, Bp, N, D, ntile;
  int nwg;                          // workgroups per role per encoder
};

struct EncAdamProb {
  const float* partial;             // [nwg][size]
  int64_t off;                      // encoder block offset inside the group arenas
};

#ifndef TD3_ENC_FUSED
#define TD3_ENC_FUSED 1      // enc_bwd_kernel<DK, 2>: roles A and B on each staged tile (0: two launches)
#endif
int launch_enc_fwd(const EncFwdArgs& a, hipStream_t s);
int launch_enc_bwd(const EncBwdArgs& a, hipStream_t s);
// sum of the partial slabs -> grad -> Adam (+ Polyak) or the grad arena (mode = DwMode)
struct EncAdamArgs {
  EncAdamProb p[3];
  int nprob, nwg;
  int64_t size;                     // EncOff::size(D)
  AdamArgs adam;
  int mode;                         // DwMode
};
int launch_enc_adam(const EncAdamArgs& a, hipStream_t s);
int encoder_init();

}  // namespace td3
