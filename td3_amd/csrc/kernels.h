// Problem descriptors of the TD3 step kernels (device-memory tables, read with
// scalar loads by every workgroup; pointers are fixed for the handle's life so
// the launches can be captured once into a hipGraph and replayed).
#pragma once
#include "common.h"

namespace td3 {

// ------------------------------------------------------------------ batch-row GEMM stage
// C[Bp x Nout] = epi( pro(A)[Bp x Kp] * B[Kp x Nout] )
//   MODE 0 (forward layer):  B[k][j] = W[n0+j][k]   (W row-major [Nout][Kp], torch Linear layout)
//   MODE 1 (input grad):     B[k][j] = W[k][n0+j]   (W row-major [Kp][Nout]; dX = dZ * W)
enum Pro : int { kProNone = 0, kProLN = 1, kProLNBwd = 2, kProReluBwd = 3 };

struct GemmProb {
  const float* A; int lda;        // batch rows of the A side
  int Kreal, Kp;                  // reduction length (real / padded to 32), Kp <= 512
  int pro;                        // prologue on each full A row (Pro)
  const float* lng; const float* lnb;   // LayerNorm affine of the A-side features
  const float* H; int ldh;        // kProLNBwd / kProReluBwd: post-ReLU activations of the A side
  float* stats;                   // [2][Bp] (mean, rstd): written by kProLN (n-tile 0), read by kProLNBwd
  float* Aout; int ldao;          // nullable: n-tile 0 stores pro(A) rows (U_{l-1} or dZ_l)
  const float* W; int ldw;
  const float* bias;              // MODE 0, nullable
  int Nout;                       // padded output width (multiple of 32)
  float* C; int ldc;
  int relu;
  int ntiles;                     // output column tiles of 32*WN
  int tile_begin;                 // first flat workgroup id of this problem
};

// ------------------------------------------------------------------ row-wise head kernels
enum HeadMode : int { kHeadTargetAction = 0, kHeadPolicy = 1, kHeadQ = 2 };

struct HeadProb {
  const float* H3; int ldh; int K3;          // last hidden (post-ReLU), real width K3
  const float* lng; const float* lnb;        // LN3 (nullable: norm=None)
  float* U3; int ldu;                        // nullable: store LN3 output (input of the head Linear)
  float* stats;                              // nullable: store LN3 (mean, rstd) [2][Bp]
  const float* W4; int ldw; const float* b4; int nout;
  int mode;
  float* out; int ldo; int out_col;          // TargetAction: X_S2A[:, sd:]; Policy: X_SP[:, sd:]; Q: Qv[Bp]
  float* tanh_out;                           // Policy: tanh(z) [Bp][32]
  float* noise; int ldn;                     // TargetAction: N(0,1) draw [Bp][ldn] (written when generated)
};

struct HeadArgs {
  const HeadProb* probs;
  int B, Bp;
  float max_action, policy_noise, noise_clip;
  const Counters* ctr;      // Philox step of the target-policy noise (total_it after the bump)
  uint64_t seed;
  int gen_noise;            // 1: draw N(0,1) with Philox (and store it); 0: read injected noise
};

// Critic loss + start of the twin-critic backward (TD3_featured.py:139-148).
struct CriticLossArgs {
  // target twin heads
  const float* TH3[2]; const float* Tlng[2]; const float* Tlnb[2];
  const float* TW4[2]; const float* Tb4[2];
  // online twin: Q values, last hidden, stats, LN3 gamma, head weight
  const float* Qv[2];
  const float* H3[2]; const float* stats3[2]; const float* lng3[2]; const float* W4[2];
  float* GZ4[2]; int ldgz4;
  float* GU3[2]; float* GZ3[2];
  int ldh, K3;             // shared width of H3 / GU3 / GZ3 rows
  const float* R; const float* ND;
  float* Y; float* sqerr;  // [Bp], [2][Bp]
  int B, Bp; float discount;
  int norm;
};

// Actor loss: Q1(s, pi(s)) head, dL/dQ = -1/B, LN3 backward (TD3_featured.py:159).
struct ActorLossArgs {
  const float* H3; int ldh, K3;
  const float* lng; const float* lnb; const float* W4; const float* b4;
  float* Qv;
  float* GZ3;
  int B, Bp; int norm;
};

// LN1 backward of Q1 -> dL/da -> tanh/max_action backward -> actor head -> actor LN3 backward.
struct ActorHeadBwdArgs {
  const float* GU1; const float* H1; const float* stats1; const float* lng1; int ld1, K1;
  const float* W1; int ldw1; int sd, ad;          // critic q1 first Linear [Np1][Kp0]
  const float* T; int ldt; float max_action;      // tanh output of the policy head
  float* GZ4; int ldgz4;
  const float* W4; int ldw4;                      // actor head [32][Kp3]
  const float* H3; const float* stats3; const float* lng3; int ld3, K3;
  float* GU3; float* GZ3;
  int B, Bp; int norm;
};

// dZ = relu'(LN_bwd(dU)) on full rows (used where no GEMM follows).
struct LnBwdProb {
  const float* GU; const float* H; const float* stats; const float* lng; int ld, K;
  float* GZ;
};

// ------------------------------------------------------------------ parameter-grad + Adam
struct DwProb {
  const float* G; int ldg;        // dZ_l   [Bp][ldg]  (columns n)
  const float* U; int ldu;        // U_{l-1}[Bp][ldu]  (columns k)
  int Np, Kp;
  int64_t offW, offb;             // offsets inside the group arenas
  int64_t offg, offbeta;          // LayerNorm_l affine, -1 when absent
  const float* GU; int ldgu;      // dU_l  (LN grads)
  const float* H; int ldh; const float* stats;
  int ntk;                        // k tiles
  int tile_begin;
};

enum DwMode : int { kDwGrad = 0, kDwAdam = 1, kDwAdamPolyak = 2 };

struct AdamArgs {
  float* P; float* G; float* M; float* V; float* T;   // group arenas
  const Counters* ctr; int which;                     // 0: critic_step, 1: actor_step
  double lr, beta1, beta2, eps;
  float tau;
  float grad_scale;                                   // 1/world for the all-reduced path
};

struct DwArgs {
  const DwProb* probs; int nprob; int Bp;
  AdamArgs adam;
  int mode;
};

// ------------------------------------------------------------------ launchers (kernels.hip)
int launch_gemm(int mode, int wn, const GemmProb* d_probs, int nprob, int nblocks, int Bp,
                int lds_bytes, Counters* bump, int bump_actor, hipStream_t s);
int launch_heads(const HeadArgs& a, int nprob, hipStream_t s);
int launch_critic_loss(const CriticLossArgs& a, hipStream_t s);
int launch_actor_loss(const ActorLossArgs& a, hipStream_t s);
int launch_actor_head_bwd(const ActorHeadBwdArgs& a, hipStream_t s);
int launch_lnbwd_rows(const LnBwdProb* d_probs, int nprob, int Bp, int norm, hipStream_t s);
int launch_dw(const DwArgs& a, int nblocks, hipStream_t s);
int launch_adam_flat(const AdamArgs& a, int64_t n, int polyak, hipStream_t s);
int launch_polyak_flat(float* T, const float* P, int64_t n, float tau, hipStream_t s);
int kernels_init();

}  // namespace td3
