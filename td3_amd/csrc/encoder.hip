// Particle set encoder (TD3_particles) on gfx950: fused forward and backward.
//
//   enc_fwd_kernel   conv1 (1xD) + ReLU on MFMA (transposed: its output registers are the conv2
//                    A operand), conv2 (256->128) on v_mfma_f32_32x32x2_f32 with W2 staged once per
//                    workgroup in LDS, ReLU, the mean over particles and the pool ReLU in the
//                    epilogue (TD3_particles.py:52-58 / :103-109).  Neither h1 [B*N][256] nor
//                    h2 [B*N][128] touches HBM: only their ReLU bits (1 bit per element, from
//                    wave ballots) are kept for the backward.
//   enc_bwd_kernel   the backward of the same, one pass over each staged particle tile: role A
//                    forms dh1 = dz2*W2 and dW1, db1 (relu'(z1) from the conv1 bits); role B dW2
//                    and db2 with h1 recomputed from the particles.
//   enc_adam_kernel  fixed-order sum of the per-workgroup partial slabs, then torch Adam
//                    (+ Polyak), or the grad arena on the all-reduced path.
//
// Shapes: particles [N][D] per batch row (D <= 16), conv1 256 channels, conv2 128.  Particle
// rows are processed in tiles of 32 (the MFMA M); rows >= N of the last tile are masked.
#include <math.h>

#include "dev.h"
#include "encoder.h"

namespace td3 {

// x tile rows of a batch row: rows r >= N read as zero.
__device__ __forceinline__ float part_ld(const float* base, int n, int N, int D, int d) {
  return (n < N && d < D) ? gld(base + (size_t)n * D + d) : 0.f;
}

// v_writelane_b32: lane `lane` of `old` <- the uniform `val` (no builtin in this toolchain).  The
// lane select goes through M0 as a register-constrained operand, so the compiler owns M0.
__device__ __forceinline__ uint32_t writelane(uint32_t old, uint32_t val, int lane) {
  asm volatile("v_writelane_b32 %0, %1, m0" : "+v"(old) : "s"(val), "{m0}"(lane));
  return old;
}

// lane L gets v when bit L of the uniform word m is set, else 0 (one v_cndmask on an SGPR pair)
__device__ __forceinline__ float lane_select(uint64_t m, float v) {
  return __builtin_amdgcn_inverse_ballot_w64(m) ? v : 0.f;
}

// mfma_row(r, lane) = crow(r) + 4 * (lane >> 5): the r-dependent part is a compile-time constant
// after unrolling, so LDS addresses are one lane base + an immediate offset per r.
__device__ __forceinline__ constexpr int crow(int r) { return (r & 3) + 8 * (r >> 2); }

// ================================================================== forward
constexpr int kEncS2 = 260;    // LDS row stride of W2 [128][256] (== 4 mod 64: b128 conflict-free)
constexpr int kEncFwdLds = (kEncC2 * kEncS2 + kEncMaxD * kEncC1 + kEncC1 + kEncC2) * 4;

// One wave per batch row (8 rows of one encoder per workgroup, 512 threads, 1 workgroup/CU).
// DK = D rounded up to 4 (the conv1 FMA loops run to DK; W1 / x columns >= D are zero).
template <int DK>
__global__ __launch_bounds__(512) void enc_fwd_kernel(EncFwdArgs a) {
  extern __shared__ float4 sm4[];
  float* w2s = reinterpret_cast<float*>(sm4);          // [128][kEncS2]
  float* w1t = w2s + kEncC2 * kEncS2;                  // [16][256]  (W1 transposed, d >= D zero)
  float* b1s = w1t + kEncMaxD * kEncC1;                // [256]
  float* b2s = b1s + kEncC1;                           // [128]
  const EncFwdProb& P = a.p[blockIdx.y];
  const int tid = threadIdx.x, D = a.D;
  const float* W1 = P.enc + EncOff::w1(D);
  const float* B1 = P.enc + EncOff::b1(D);
  const float* W2 = P.enc + EncOff::w2(D);
  const float* B2 = P.enc + EncOff::b2(D);
  for (int e = tid; e < kEncC2 * (kEncC1 / 4); e += 512) {
    const int r = e >> 6, c4 = (e & 63) << 2;
    *reinterpret_cast<float4*>(w2s + r * kEncS2 + c4) = gld4(W2 + r * kEncC1 + c4);
  }
  for (int e = tid; e < kEncMaxD * kEncC1; e += 512) {
    const int d = e >> 8, k = e & 255;
    w1t[e] = d < D ? gld(W1 + k * D + d) : 0.f;
  }
  for (int e = tid; e < kEncC1; e += 512) b1s[e] = gld(B1 + e);
  for (int e = tid; e < kEncC2; e += 512) b2s[e] = gld(B2 + e);
  __syncthreads();

  const int wave = tid >> 6, lane = tid & 63, i = lane & 31, h = lane >> 5;
  const int b = blockIdx.x * 8 + wave;
  if (b >= a.Bp) return;
  if (b >= a.B) {                                       // padded batch rows: pooled = 0
    for (int c = lane; c < kEncC2; c += 64) gst(P.out + ((size_t)b * P.ldo + c), 0.f);
    return;
  }
  const float* base = a.data + (size_t)a.idx[b] * a.rec + P.part_off;
  uint64_t* mask1 = P.mask ? P.mask + (size_t)a.Bp * a.ntile * 64 : nullptr;
  double cs[4] = {0.0, 0.0, 0.0, 0.0};
  float npos[4] = {0.f, 0.f, 0.f, 0.f};                // rows with conv2 output > 0 (backward db2)
  // conv1 on MFMA, transposed: per 32-channel chunk c, z1^T[channel][particle] = W1 x^T + b1 on
  // v_mfma_f32_32x32x2_f32 (A = W1[32c + i][2s + h], B = x[particle i][2s + h]; K = D rounded up
  // to even, k in order: the fmaf chain b1 + sum_d W1[k][d] x[d] of role B's recompute, bitwise).
  // Lane (i, h) then holds h1[particle i][channel 32c + crow(r) + 4h] in register r, which IS the
  // conv2 A operand when conv2's reduction runs over the chunk's channels in the order
  // k(s, h) = crow(s) + 4h: its B operand W2[j*32 + i][32c + 4h + 8q + e] (s = 4q + e) is four
  // float4 LDS reads.  No VALU conv1, no register shuffle.
  constexpr int KS = (DK + 1) / 2;                        // conv1 MFMA steps (features 2s, 2s + 1)
  for (int t = 0; t < a.ntile; ++t) {
    const int n = t * 32 + i;
    float xk[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) xk[s] = part_ld(base, n, a.N, D, 2 * s + h);
    f32x16 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    uint32_t m1lo = 0, m1hi = 0;
    auto conv1 = [&](int c, f32x16& z) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(b1s + c * 32 + 4 * h + 8 * q);
        z[4 * q + 0] = v.x; z[4 * q + 1] = v.y; z[4 * q + 2] = v.z; z[4 * q + 3] = v.w;
      }
#pragma unroll
      for (int s = 0; s < KS; ++s)
        if (2 * s < D) z = mfma32x32x2(w1t[(2 * s + h) * kEncC1 + c * 32 + i], xk[s], z);   // ceil(D/2) steps
    };
    f32x16 zn;
    conv1(0, zn);
#pragma unroll 1
    for (int c = 0; c < kEncC1 / 32; ++c) {
      float av[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) av[r] = fmaxf(zn[r], 0.f);
      if (c + 1 < kEncC1 / 32) conv1(c + 1, zn);          // next chunk's conv1 in the shadow of this one's conv2
      if (mask1) {
        // conv1 ReLU bits: ballot r of chunk c = the 32 particles of channel 32c + crow(r) (low) /
        // 32c + crow(r) + 4 (high); lane (c&3)*16+r keeps it, every 4 chunks the wave stores 64 words
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const uint64_t w = __ballot(av[r] > 0.f);
          m1lo = writelane(m1lo, (uint32_t)w, (c & 3) * 16 + r);
          m1hi = writelane(m1hi, (uint32_t)(w >> 32), (c & 3) * 16 + r);
        }
        if ((c & 3) == 3)
          *(GAS uint64_t*)(mask1 + (((size_t)b * a.ntile + t) * 2 + (c >> 2)) * 64 + lane) =
              ((uint64_t)m1hi << 32) | m1lo;
      }
      // B operand: W2[j*32 + i][32c + 4h + crow(s)]; conv2 output tile j (32 channels)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float* wr = w2s + (j * 32 + i) * kEncS2 + c * 32 + 4 * h;
        float bv[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 v = *reinterpret_cast<const float4*>(wr + 8 * q);
          bv[4 * q + 0] = v.x; bv[4 * q + 1] = v.y; bv[4 * q + 2] = v.z; bv[4 * q + 3] = v.w;
        }
#pragma unroll
        for (int s = 0; s < 16; ++s) acc[j] = mfma32x32x2(av[s], bv[s], acc[j]);
      }
    }
    // epilogue: bias, ReLU, row mask, column sums; one ReLU bit word per (channel tile, reg)
    // and the count of positive rows per channel
    uint32_t wlo = 0, whi = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float bias = b2s[j * 32 + i];
      float part = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = t * 32 + mfma_row(r, lane);
        const float v = row < a.N ? fmaxf(acc[j][r] + bias, 0.f) : 0.f;
        part += v;
        if (P.mask) {
          const uint64_t w = __ballot(v > 0.f);           // uniform; lane j*16+r keeps it
          wlo = writelane(wlo, (uint32_t)w, j * 16 + r);
          whi = writelane(whi, (uint32_t)(w >> 32), j * 16 + r);
          npos[j] += v > 0.f ? 1.f : 0.f;
        }
      }
      cs[j] += (double)part;
    }
    if (P.mask) *(GAS uint64_t*)(P.mask + ((size_t)b * a.ntile + t) * 64 + lane) = ((uint64_t)whi << 32) | wlo;
  }
  // lanes i and i + 32 hold the same channel (different rows): combine, mean, pool ReLU
  float* cnt = P.mask ? reinterpret_cast<float*>(P.mask + (size_t)a.Bp * a.ntile * 192) : nullptr;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const double v = cs[j] + __shfl_xor(cs[j], 32, 64);
    if (h == 0) gst(P.out + ((size_t)b * P.ldo + j * 32 + i), fmaxf((float)(v / (double)a.N), 0.f));
    if (cnt) {
      const float c = npos[j] + __shfl_xor(npos[j], 32, 64);
      if (h == 0) gst(cnt + ((size_t)b * kEncC2 + j * 32 + i), c);
    }
  }
}

// ================================================================== backward
constexpr int kEncS1 = 17;       // W1 [256][17] in LDS (odd stride: lane-indexed rows conflict-free)
constexpr int kEncST = 132;      // W2^T [256][132] rows (== 4 mod 64)
constexpr int kEncBufs = 2;      // staging double buffer: tile it+1 lands while tile it is used
// role A stages W2^T [256][132]; role B keeps h1 in registers

template <int ROLE>
constexpr int enc_big() { return ROLE != 1 ? kEncC1 * kEncST : 0; }
template <int ROLE>
constexpr int enc_bwd_lds() {
  return (enc_big<ROLE>() + kEncC1 * kEncS1 + kEncBufs * (32 * kEncMaxD + 64 * 2 + kEncC2) + kEncC1) * 4;
}
static_assert(enc_bwd_lds<2>() <= 160 * 1024, "encoder backward LDS");

// rows of the forward's ballot words: word (j, r) holds channel j*32 + lane&31 of row
// mfma_row(r, lane); row R lives in word r = (R&3) + 4(R>>3), half (R>>2)&1.
__device__ __forceinline__ int word_of_row(int R) { return (R & 3) + 4 * (R >> 3); }
__device__ __forceinline__ int half_of_row(int R) { return (R >> 2) & 1; }

// Pooled-feature grad of every batch row (one wave per row): LN_in backward of the MLP input
// grad (no ReLU before lnorm1), then the pool ReLU (pooled > 0) and the 1/N of the mean.
__global__ __launch_bounds__(256) void enc_gpool_kernel(EncBwdArgs a) {
  const EncBwdProb& P = a.p[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= a.B) return;
  float gu[1][8], xr[1][8], gm[8], mean[1], rstd[1];
  rv_load(gu[0], P.GU + (size_t)b * P.ldgu, P.Kin, lane);
  rv_load(xr[0], P.X + (size_t)b * P.ldx, P.Kin, lane);
  if (P.stats) {
    rv_load(gm, P.gamma, P.Kin, lane);
    mean[0] = gld(P.stats + b);
    rstd[0] = gld(P.stats + (a.Bp + b));
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) gm[j] = 1.f;
    mean[0] = 0.f;
    rstd[0] = 1.f;
  }
  ln_bwd_rows<1, false>(gu, xr, gm, mean, rstd, P.Kin, lane, P.stats ? 1 : 0);
  const float invn = 1.0f / (float)a.N;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = rcol(lane, j);
    if (c < kEncC2) gst(P.gpool + ((size_t)b * kEncC2 + c), xr[0][j] > 0.f ? gu[0][j] * invn : 0.f);
  }
}

// ROLE 0: role A only, 1: role B only, 2: both on every staged tile (one pass over the particles,
// masks and pooled grads; the role B h1 recompute and dW2 MFMAs interleave with role A's chains)
#ifndef TD3_ENC_SKEW
#define TD3_ENC_SKEW 1
#endif
template <int DK, int ROLE>
__global__ __launch_bounds__(512) void enc_bwd_kernel(EncBwdArgs a) {
  constexpr bool kA = ROLE != 1, kB = ROLE != 0;
  extern __shared__ float4 sm4[];
  float* big = reinterpret_cast<float*>(sm4);           // role A: W2^T [256][132]
  float* w1s = big + enc_big<ROLE>();                   // [256][17]
  float* xs = w1s + kEncC1 * kEncS1;                    // [kEncBufs][32][16]
  uint64_t* ms = reinterpret_cast<uint64_t*>(xs + kEncBufs * 32 * kEncMaxD);   // [kEncBufs][64]
  float* gs = reinterpret_cast<float*>(ms + kEncBufs * 64);    // [kEncBufs][128]
  float* b1s = gs + kEncBufs * kEncC2;                  // [256]
  const EncBwdProb& P = a.p[blockIdx.y];
  const int tid = threadIdx.x, D = a.D;
  const int wave = tid >> 6, lane = tid & 63, i = lane & 31, h = lane >> 5;
  const float* W1 = P.enc + EncOff::w1(D);
  const float* W2 = P.enc + EncOff::w2(D);
  if constexpr (kA) {
    for (int e = tid; e < kEncC2 * kEncC1; e += 512) {     // W2^T: row k, column c
      const int c = e >> 8, k = e & 255;
      big[k * kEncST + c] = gld(W2 + e);
    }
  }
  if constexpr (kB) {
    for (int e = tid; e < kEncC1 * kEncMaxD; e += 512) {
      const int k = e >> 4, d = e & 15;
      if (d < D) w1s[k * kEncS1 + d] = gld(W1 + k * D + d);
      else if (d < kEncS1) w1s[k * kEncS1 + d] = 0.f;
    }
    for (int e = tid; e < kEncC1; e += 512) b1s[e] = gld(P.enc + EncOff::b1(D) + e);
  }
  __syncthreads();

  const int k_own = wave * 32 + i;                      // this lane's conv1 channel (h1 tiles)
  float w1r[kB ? DK : 1];
  float b1k = 0.f;
  if constexpr (kB) {
#pragma unroll
    for (int d = 0; d < DK; ++d) w1r[d] = w1s[k_own * kEncS1 + d];
    b1k = b1s[k_own];
  }

  // role A: dW1[k_own][d] of this lane's rows (crow(s) + 4h), on the VALU: as a 32x32x2 MFMA
  // tile its N would be the D (<= 16) particle features, 72 % of the MFMA issue wasted at D = 9;
  // the lane's 16 x DK FMAs run beside the other wave's MFMA chain instead
  float w1acc[kA ? DK : 1];
  f32x16 accB[kB ? 4 : 1];                              // role B: dW2 tiles
#pragma unroll
  for (int d = 0; d < (kA ? DK : 1); ++d) w1acc[d] = 0.f;
#pragma unroll
  for (int q = 0; q < (kB ? 4 : 1); ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) accB[q][r] = 0.f;
  float gb1 = 0.f;

  const int g = blockIdx.x;
  const int b_begin = (int)((int64_t)g * a.B / a.nwg), b_end = (int)((int64_t)(g + 1) * a.B / a.nwg);
  const int ntot = (b_end - b_begin) * a.ntile;
  // staging of one tile: thread (row = tid>>4, d = tid&15) one particle coordinate, threads < 64
  // one ReLU-bit word, threads < 128 one pooled-grad channel; tile it+1 is requested while
  // tile it is multiplied
  const int srow = tid >> 4, sd = tid & 15;
  float st_x = 0.f, st_g = 0.f;
  uint64_t st_m = 0;
  // role A: the forward's conv1 ReLU word of channel k_own (bit R = row R of the tile)
  // (channel 32c + m sits in the forward's ballot r = (m & 3) + 4 (m >> 3) of chunk c, half (m >> 2) & 1)
  const uint64_t* mask1 = P.mask + (size_t)a.Bp * a.ntile * 64 + (wave >> 2) * 64 + (wave & 3) * 16 +
                          ((i & 3) + 4 * (i >> 3));
  const int m1_sh = 32 * ((i >> 2) & 1);
  uint32_t st_r = 0;
  auto fetch = [&](int it) {
    const int b = b_begin + it / a.ntile, t = it % a.ntile;
    const float* base = a.data + (size_t)a.idx[b] * a.rec + P.part_off;
    st_x = part_ld(base, t * 32 + srow, a.N, D, sd);
    if (kA && tid < 64) st_m = *(const GAS uint64_t*)(P.mask + ((size_t)b * a.ntile + t) * 64 + tid);
    if (tid < kEncC2) st_g = gld(P.gpool + ((size_t)b * kEncC2 + tid));
    if constexpr (kA) st_r = (uint32_t)(*(const GAS uint64_t*)(mask1 + ((size_t)b * a.ntile + t) * 128) >> m1_sh);
  };
  // ---- dh1 tile (rows i, channels k_own): A = dz2[row i][c], B = W2^T[k][c]
  auto role_a_dh1 = [&](f32x16& ac, const uint64_t* mb, const float* gsb) {
#pragma unroll
    for (int r = 0; r < 16; ++r) ac[r] = 0.f;
    const int wr = word_of_row(i), hr = half_of_row(i);
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {
      const uint32_t bits = (uint32_t)(mb[cc * 16 + wr] >> (32 * hr)) >> (16 * h);
      const float* gp = gsb + cc * 32 + 16 * h;
      const float* wp = big + k_own * kEncST + cc * 32 + 16 * h;
      float av[16], bv[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 gv = *reinterpret_cast<const float4*>(gp + 4 * q);
        const float4 wv = *reinterpret_cast<const float4*>(wp + 4 * q);
        av[4 * q + 0] = gv.x; av[4 * q + 1] = gv.y; av[4 * q + 2] = gv.z; av[4 * q + 3] = gv.w;
        bv[4 * q + 0] = wv.x; bv[4 * q + 1] = wv.y; bv[4 * q + 2] = wv.z; bv[4 * q + 3] = wv.w;
      }
#pragma unroll
      for (int s = 0; s < 16; ++s) av[s] = ((bits >> s) & 1u) ? av[s] : 0.f;
#pragma unroll
      for (int s = 0; s < 16; ++s) ac = mfma32x32x2(av[s], bv[s], ac);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // ---- dz1 = relu'(z1) dh1 at (row mfma_row(r), channel k_own), relu'(z1) from the forward's
  // conv1 bits (rb: bit R = tile row R); db1; dW1 += dz1^T x
  auto role_a_dw1 = [&](const f32x16& ac, const float* xb, uint32_t rb) {
    rb >>= 4 * h;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const float gz = ((rb >> crow(s)) & 1u) ? ac[s] : 0.f;
      gb1 += gz;
      const float* xr = xb + (crow(s) + 4 * h) * kEncMaxD;   // one row per lane half: broadcast reads
#pragma unroll
      for (int q = 0; q < DK / 4; ++q) {
        const float4 xv = *reinterpret_cast<const float4*>(xr + 4 * q);
        w1acc[4 * q + 0] = __fmaf_rn(gz, xv.x, w1acc[4 * q + 0]);
        w1acc[4 * q + 1] = __fmaf_rn(gz, xv.y, w1acc[4 * q + 1]);
        w1acc[4 * q + 2] = __fmaf_rn(gz, xv.z, w1acc[4 * q + 2]);
        w1acc[4 * q + 3] = __fmaf_rn(gz, xv.w, w1acc[4 * q + 3]);
      }
    }
  };

  if (ntot > 0) fetch(0);
  for (int it = 0; it < ntot; ++it) {
    const int buf = it % kEncBufs;
    float* xb = xs + buf * 32 * kEncMaxD;
    uint64_t* mb = ms + buf * 64;
    float* gsb = gs + buf * kEncC2;
    xb[srow * kEncMaxD + sd] = st_x;
    if (kA && tid < 64) mb[tid] = st_m;
    if (tid < kEncC2) gsb[tid] = st_g;
    const uint32_t rb_now = st_r;
    __syncthreads();
    if (it + 1 < ntot) fetch(it + 1);
    auto do_a = [&]() {
      if constexpr (kA) {
        f32x16 acc;
        role_a_dh1(acc, mb, gsb);
        role_a_dw1(acc, xb, rb_now);
      }
    };
    auto do_b = [&]() {
      if constexpr (kB) {
        // ---- h1 of this wave's channels k_own at rows crow(r) + 4h, kept in registers as the
        // B operand: lane (i, h) of step s supplies h1[row crow(s)+4h][k_own].
        // A = dz2[row crow(s)+4h][mt*32 + i]: the forward's ballot word (mt, s) has bit
        // i + 32h = lane for exactly that element, so one v_cndmask on the word (scalar
        // loaded, one channel tile ahead) builds each operand (read from the staged tile in LDS
        // and made uniform by v_readfirstlane instead: CB_enc 3.99 -> 4.15 ms)
        const uint64_t* mw = P.mask + ((size_t)(b_begin + it / a.ntile) * a.ntile + it % a.ntile) * 64;
        uint64_t wq[16];
#pragma unroll
        for (int s = 0; s < 16; ++s) wq[s] = mw[s];
        __builtin_amdgcn_sched_barrier(0);
        const float* xbase = xb + 4 * h * kEncMaxD;
        float hv[16];
#pragma unroll
        for (int r0 = 0; r0 < 16; r0 += 4) {      // 4 rows at a time: independent FMA chains
          float z[4], xv[4][DK];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            z[q] = b1k;
#pragma unroll
            for (int d = 0; d < DK; ++d) xv[q][d] = xbase[crow(r0 + q) * kEncMaxD + d];
          }
#pragma unroll
          for (int d = 0; d < DK; ++d)
#pragma unroll
            for (int q = 0; q < 4; ++q) z[q] = __fmaf_rn(w1r[d], xv[q][d], z[q]);
#pragma unroll
          for (int q = 0; q < 4; ++q) hv[r0 + q] = fmaxf(z[q], 0.f);
          __builtin_amdgcn_sched_barrier(0);
        }
        // ---- dW2 tiles (conv2 channels mt*32 + m) x (conv1 channels k_own), K = the 32 rows
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          uint64_t wn[16];
          if (mt < 3)
#pragma unroll
            for (int s = 0; s < 16; ++s) wn[s] = mw[(mt + 1) * 16 + s];
          const float gsc = gsb[mt * 32 + i];
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int s = 0; s < 16; ++s) accB[mt] = mfma32x32x2(lane_select(wq[s], gsc), hv[s], accB[mt]);
          __builtin_amdgcn_sched_barrier(0);
          if (mt < 3)
#pragma unroll
            for (int s = 0; s < 16; ++s) wq[s] = wn[s];
        }
      }
    };
    // the two waves of a SIMD (w, w + 4) run the roles in opposite order: each role is an MFMA
    // phase and a VALU phase (A: dh1 chain, then dz1 / dW1 FMAs; B: h1 recompute, then dW2
    // chain), so one wave's VALU phase meets the other's MFMA chain instead of both waves
    // reaching their VALU phases together after the tile barrier
    if (ROLE == 2 && TD3_ENC_SKEW && wave >= 4) {
      do_b();
      do_a();
    } else {
      do_a();
      do_b();
    }
  }
  // ---- partial slab of this workgroup
  float* out = P.partial + (size_t)g * EncOff::size(D);
  if constexpr (kA) {
#pragma unroll
    for (int d = 0; d < DK; ++d) {                         // lane halves: rows +0 / +4 of each group
      const float v = w1acc[d] + __shfl_xor(w1acc[d], 32, 64);
      if (h == 0 && d < D) gst(out + (EncOff::w1(D) + (int64_t)k_own * D + d), v);
    }
    const float v = gb1 + __shfl_xor(gb1, 32, 64);
    if (h == 0) gst(out + (EncOff::b1(D) + k_own), v);
  }
  if constexpr (kB) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c = q * 32 + mfma_row(r, lane);
        gst(out + (EncOff::w2(D) + (int64_t)c * kEncC1 + k_own), accB[q][r]);
      }
    // db2[c] = sum over rows of dz2 = sum_b gpool[b][c] * (positive rows of channel c in b)
    if (tid < kEncC2) {
      const float* cnt = reinterpret_cast<const float*>(P.mask + (size_t)a.Bp * a.ntile * 192);
      float gb2 = 0.f;
      for (int b = b_begin; b < b_end; ++b)
        gb2 = __fmaf_rn(gld(P.gpool + ((size_t)b * kEncC2 + tid)), gld(cnt + ((size_t)b * kEncC2 + tid)), gb2);
      gst(out + (EncOff::b2(D) + tid), gb2);
    }
  }
}

// ================================================================== reduce + Adam
__global__ __launch_bounds__(256) void enc_adam_kernel(EncAdamArgs a) {
  const EncAdamProb& P = a.p[blockIdx.y];
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= a.size) return;
  // 8 independent partial sums (fixed order) keep 8 slab loads in flight per thread
  float ps[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const float* src = P.partial + e;
  int w = 0;
  for (; w + 8 <= a.nwg; w += 8)
#pragma unroll
    for (int u = 0; u < 8; ++u) ps[u] += gld(src + (size_t)(w + u) * a.size);
  for (; w < a.nwg; ++w) ps[0] += gld(src + (size_t)w * a.size);
  const float g = ((ps[0] + ps[1]) + (ps[2] + ps[3])) + ((ps[4] + ps[5]) + (ps[6] + ps[7]));
  const int64_t idx = P.off + e;
  if (a.mode == kDwGrad) {
    gst(a.adam.G + idx, g);
    return;
  }
  const AdamK k = make_adam(a.adam);
  adam_elem(a.adam.P + idx, a.adam.M + idx, a.adam.V + idx, g, k,
            a.mode == kDwAdamPolyak ? a.adam.T + idx : nullptr);
}

// ================================================================== launchers
int launch_enc_fwd(const EncFwdArgs& a, hipStream_t s) {
  if (a.Bp <= 0 || a.nprob <= 0) return 0;
  if (a.D > kEncMaxD || a.nprob > kMaxEnc) {
    set_error("launch_enc_fwd: D %d / nprob %d out of range", a.D, a.nprob);
    return -1;
  }
  const dim3 grid((a.Bp + 7) / 8, a.nprob);
  switch ((a.D + 3) / 4) {
    case 1: hipLaunchKernelGGL(enc_fwd_kernel<4>, grid, dim3(512), kEncFwdLds, s, a); break;
    case 2: hipLaunchKernelGGL(enc_fwd_kernel<8>, grid, dim3(512), kEncFwdLds, s, a); break;
    case 3: hipLaunchKernelGGL(enc_fwd_kernel<12>, grid, dim3(512), kEncFwdLds, s, a); break;
    default: hipLaunchKernelGGL(enc_fwd_kernel<16>, grid, dim3(512), kEncFwdLds, s, a); break;
  }
  TD3_HIP(hipGetLastError());
  return 0;
}

int launch_enc_bwd(const EncBwdArgs& a, hipStream_t s) {
  if (a.B <= 0 || a.nprob <= 0) return 0;
  if (a.D > kEncMaxD || a.nprob > 3) {
    set_error("launch_enc_bwd: D %d / nprob %d out of range", a.D, a.nprob);
    return -1;
  }
  hipLaunchKernelGGL(enc_gpool_kernel, dim3((a.B + 3) / 4, a.nprob), dim3(256), 0, s, a);
  const dim3 grid(a.nwg, a.nprob);
#if TD3_ENC_FUSED
#define TD3_ENC_BWD(DK) hipLaunchKernelGGL((enc_bwd_kernel<DK, 2>), grid, dim3(512), enc_bwd_lds<2>(), s, a)
#else
#define TD3_ENC_BWD(DK)                                                                        \
  hipLaunchKernelGGL((enc_bwd_kernel<DK, 0>), grid, dim3(512), enc_bwd_lds<0>(), s, a);       \
  hipLaunchKernelGGL((enc_bwd_kernel<DK, 1>), grid, dim3(512), enc_bwd_lds<1>(), s, a)
#endif
  switch ((a.D + 3) / 4) {
    case 1: TD3_ENC_BWD(4); break;
    case 2: TD3_ENC_BWD(8); break;
    case 3: TD3_ENC_BWD(12); break;
    default: TD3_ENC_BWD(16); break;
  }
#undef TD3_ENC_BWD
  TD3_HIP(hipGetLastError());
  return 0;
}

int launch_enc_adam(const EncAdamArgs& a, hipStream_t s) {
  if (a.nprob <= 0) return 0;
  hipLaunchKernelGGL(enc_adam_kernel, dim3((unsigned)((a.size + 255) / 256), a.nprob), dim3(256), 0, s, a);
  TD3_HIP(hipGetLastError());
  return 0;
}

template <int DK>
static int enc_attr() {
  TD3_HIP(hipFuncSetAttribute((const void*)enc_fwd_kernel<DK>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              kEncFwdLds));
  TD3_HIP(hipFuncSetAttribute((const void*)enc_bwd_kernel<DK, 0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              enc_bwd_lds<0>()));
  TD3_HIP(hipFuncSetAttribute((const void*)enc_bwd_kernel<DK, 1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              enc_bwd_lds<1>()));
  TD3_HIP(hipFuncSetAttribute((const void*)enc_bwd_kernel<DK, 2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              enc_bwd_lds<2>()));
  return 0;
}

int encoder_init() {
  int rc = enc_attr<4>();
  if (!rc) rc = enc_attr<8>();
  if (!rc) rc = enc_attr<12>();
  if (!rc) rc = enc_attr<16>();
  return rc;
}

}  // namespace td3
