// Particle set encoder (TD3_particles) on gfx950: fused forward and backward.
//
//   enc_fwd_kernel   conv1 (1xD) + ReLU computed in registers as the MFMA A operand,
//                    conv2 (256->128) on v_mfma_f32_32x32x2_f32 with W2 staged once per
//                    workgroup in LDS, ReLU, the mean over particles and the pool ReLU in the
//                    epilogue (TD3_particles.py:52-58 / :103-109).  Neither h1 [B*N][256] nor
//                    h2 [B*N][128] touches HBM: only the conv2 ReLU bits (1 bit per h2 element)
//                    are kept for the backward.
//   enc_bwd_kernel   the backward of the same, h1 recomputed from the particles: role A
//                    workgroups form dh1 = dz2*W2 and dW1, db1; role B workgroups dW2 and db2.
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
  double cs[4] = {0.0, 0.0, 0.0, 0.0};
  for (int t = 0; t < a.ntile; ++t) {
    const int n = t * 32 + i;
    float x[DK];
#pragma unroll
    for (int d = 0; d < DK; ++d) x[d] = part_ld(base, n, a.N, D, d);
    f32x16 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
#pragma unroll 1
    for (int c = 0; c < kEncC1 / 32; ++c) {
      // A operand: h1[n][k] = relu(b1[k] + sum_d W1[k][d] x[n][d]), k = 32c + 16h + s
      const int k0 = c * 32 + 16 * h;
      float av[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(b1s + k0 + 4 * q);
        av[4 * q + 0] = v.x; av[4 * q + 1] = v.y; av[4 * q + 2] = v.z; av[4 * q + 3] = v.w;
      }
#pragma unroll
      for (int d = 0; d < DK; ++d) {
        float xd = x[d];
        asm volatile("" : "+v"(xd));         // no loop-invariant splats of x hoisted out of c
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 w = *reinterpret_cast<const float4*>(w1t + d * kEncC1 + k0 + 4 * q);
          av[4 * q + 0] = __fmaf_rn(w.x, xd, av[4 * q + 0]);
          av[4 * q + 1] = __fmaf_rn(w.y, xd, av[4 * q + 1]);
          av[4 * q + 2] = __fmaf_rn(w.z, xd, av[4 * q + 2]);
          av[4 * q + 3] = __fmaf_rn(w.w, xd, av[4 * q + 3]);
        }
      }
#pragma unroll
      for (int s = 0; s < 16; ++s) av[s] = fmaxf(av[s], 0.f);
      // B operand: W2[j*32 + i][k]; conv2 output tile j (32 channels)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float* wr = w2s + (j * 32 + i) * kEncS2 + k0;
        float bv[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 v = *reinterpret_cast<const float4*>(wr + 4 * q);
          bv[4 * q + 0] = v.x; bv[4 * q + 1] = v.y; bv[4 * q + 2] = v.z; bv[4 * q + 3] = v.w;
        }
#pragma unroll
        for (int s = 0; s < 16; ++s) acc[j] = mfma32x32x2(av[s], bv[s], acc[j]);
      }
    }
    // epilogue: bias, ReLU, row mask, column sums; one ReLU bit word per (channel tile, reg)
    int wlo = 0, whi = 0;
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
          const bool mine = lane == j * 16 + r;
          wlo = mine ? (int)(uint32_t)w : wlo;
          whi = mine ? (int)(uint32_t)(w >> 32) : whi;
        }
      }
      cs[j] += (double)part;
    }
    if (P.mask) {
      const uint64_t word = ((uint64_t)(uint32_t)whi << 32) | (uint32_t)wlo;
      *(GAS uint64_t*)(P.mask + ((size_t)b * a.ntile + t) * 64 + lane) = word;
    }
  }
  // lanes i and i + 32 hold the same channel (different rows): combine, mean, pool ReLU
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const double v = cs[j] + __shfl_xor(cs[j], 32, 64);
    if (h == 0) gst(P.out + ((size_t)b * P.ldo + j * 32 + i), fmaxf((float)(v / (double)a.N), 0.f));
  }
}

// ================================================================== backward
constexpr int kEncS1 = 17;       // W1 [256][17] in LDS (odd stride: lane-indexed rows conflict-free)
constexpr int kEncST = 132;      // W2^T [256][132] rows (== 4 mod 64)
// role A stages W2^T [256][132]; role B the h1 tile [32][256]
template <int ROLE>
constexpr int enc_big() { return ROLE == 0 ? kEncC1 * kEncST : 32 * kEncC1; }
template <int ROLE>
constexpr int enc_bwd_lds() {
  return (enc_big<ROLE>() + kEncC1 * kEncS1 + 2 * 32 * kEncMaxD + 2 * 64 * 2 + 2 * kEncC2 + kEncC1) * 4;
}
static_assert(enc_bwd_lds<0>() <= 160 * 1024, "encoder backward LDS");

// rows of the forward's ballot words: word (j, r) holds channel j*32 + lane&31 of row
// mfma_row(r, lane); row R lives in word r = (R&3) + 4(R>>3), half (R>>2)&1.
__device__ __forceinline__ int word_of_row(int R) { return (R & 3) + 4 * (R >> 3); }
__device__ __forceinline__ int half_of_row(int R) { return (R >> 2) & 1; }
// role B's h1 tile [32][256] in LDS, XOR-swizzled so the two lane halves (rows 4 apart) use
// disjoint bank halves
__device__ __forceinline__ int h1_at(int R, int k) { return R * kEncC1 + (k ^ (((R >> 2) & 1) << 5)); }
// mfma_row(r, lane) = crow(r) + 4 * (lane >> 5): the r-dependent part is a compile-time constant
// after unrolling, so LDS addresses are one lane base + an immediate offset per r.
__device__ __forceinline__ constexpr int crow(int r) { return (r & 3) + 8 * (r >> 2); }

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

template <int DK, int ROLE>
__global__ __launch_bounds__(512) void enc_bwd_kernel(EncBwdArgs a) {
  extern __shared__ float4 sm4[];
  float* big = reinterpret_cast<float*>(sm4);           // role A: W2^T [256][132]; role B: h1 [32][256]
  float* w1s = big + enc_big<ROLE>();                   // [256][17]
  float* xs = w1s + kEncC1 * kEncS1;                    // [2][32][16]
  uint64_t* ms = reinterpret_cast<uint64_t*>(xs + 2 * 32 * kEncMaxD);   // [2][64]
  float* gs = reinterpret_cast<float*>(ms + 2 * 64);    // [2][128]
  float* b1s = gs + 2 * kEncC2;                         // [256]
  const EncBwdProb& P = a.p[blockIdx.y];
  const int tid = threadIdx.x, D = a.D;
  const int wave = tid >> 6, lane = tid & 63, i = lane & 31, h = lane >> 5;
  const float* W1 = P.enc + EncOff::w1(D);
  const float* W2 = P.enc + EncOff::w2(D);
  if constexpr (ROLE == 0) {
    for (int e = tid; e < kEncC2 * kEncC1; e += 512) {     // W2^T: row k, column c
      const int c = e >> 8, k = e & 255;
      big[k * kEncST + c] = gld(W2 + e);
    }
  }
  for (int e = tid; e < kEncC1 * kEncMaxD; e += 512) {
    const int k = e >> 4, d = e & 15;
    if (d < D) w1s[k * kEncS1 + d] = gld(W1 + k * D + d);
    else if (d < kEncS1) w1s[k * kEncS1 + d] = 0.f;
  }
  for (int e = tid; e < kEncC1; e += 512) b1s[e] = gld(P.enc + EncOff::b1(D) + e);
  __syncthreads();

  const int k_own = wave * 32 + i;                      // this lane's conv1 channel (h1 tiles)
  float w1r[DK];
#pragma unroll
  for (int d = 0; d < DK; ++d) w1r[d] = w1s[k_own * kEncS1 + d];
  const float b1k = b1s[k_own];
  const int mt = wave & 3, kt0 = 4 * (wave >> 2);       // role B: dW2 tiles of this wave

  f32x16 accW1;                                         // role A: dW1 tile
  f32x16 accB[ROLE == 1 ? 4 : 1];                       // role B: dW2 tiles
#pragma unroll
  for (int r = 0; r < 16; ++r) accW1[r] = 0.f;
#pragma unroll
  for (int q = 0; q < (ROLE == 1 ? 4 : 1); ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) accB[q][r] = 0.f;
  float gb1 = 0.f, gb2 = 0.f;

  const int g = blockIdx.x;
  const int b_begin = (int)((int64_t)g * a.B / a.nwg), b_end = (int)((int64_t)(g + 1) * a.B / a.nwg);
  const int ntot = (b_end - b_begin) * a.ntile;
  // staging of one tile: thread (row = tid>>4, d = tid&15) one particle coordinate, threads < 64
  // one ReLU-bit word, threads < 128 one pooled-grad channel; tile it+1 is requested while
  // tile it is multiplied
  const int srow = tid >> 4, sd = tid & 15;
  float st_x = 0.f, st_g = 0.f;
  uint64_t st_m = 0;
  auto fetch = [&](int it) {
    const int b = b_begin + it / a.ntile, t = it % a.ntile;
    const float* base = a.data + (size_t)a.idx[b] * a.rec + P.part_off;
    st_x = part_ld(base, t * 32 + srow, a.N, D, sd);
    if (tid < 64) st_m = *(const GAS uint64_t*)(P.mask + ((size_t)b * a.ntile + t) * 64 + tid);
    if (tid < kEncC2) st_g = gld(P.gpool + ((size_t)b * kEncC2 + tid));
  };
  if (ntot > 0) fetch(0);
  for (int it = 0; it < ntot; ++it) {
    const int buf = it & 1;
    float* xb = xs + buf * 32 * kEncMaxD;
    uint64_t* mb = ms + buf * 64;
    float* gsb = gs + buf * kEncC2;
    xb[srow * kEncMaxD + sd] = st_x;
    if (tid < 64) mb[tid] = st_m;
    if (tid < kEncC2) gsb[tid] = st_g;
    __syncthreads();
    if (it + 1 < ntot) fetch(it + 1);
    {
      if constexpr (ROLE == 0) {
        // ---- dh1 tile (rows i, channels k_own): A = dz2[row i][c], B = W2^T[k][c]
        f32x16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
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
          for (int s = 0; s < 16; ++s) acc = mfma32x32x2(av[s], bv[s], acc);
          __builtin_amdgcn_sched_barrier(0);
        }
        // ---- dz1 = relu'(z1) dh1 at (row mfma_row(r), channel k_own); db1; dW1 += dz1^T x
        float gz1[16];
        const float* xbase = xb + 4 * h * kEncMaxD;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float* xr = xbase + crow(r) * kEncMaxD;
          float z = b1k;
#pragma unroll
          for (int d = 0; d < DK; ++d) z = __fmaf_rn(w1r[d], xr[d], z);
          gz1[r] = z > 0.f ? acc[r] : 0.f;
          gb1 += gz1[r];
          __builtin_amdgcn_sched_barrier(0);   // one row of x at a time (VGPR budget)
        }
        const float* xcol = xbase + (i & 15);
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const float xv = i < kEncMaxD ? xcol[crow(s) * kEncMaxD] : 0.f;
          accW1 = mfma32x32x2(gz1[s], xv, accW1);
        }
      } else {
        // ---- h1 tile into LDS (this wave: channels k_own of all 32 rows)
        const float* xbase = xb + 4 * h * kEncMaxD;
        float* hw = big + h1_at(4 * h, k_own);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float* xr = xbase + crow(r) * kEncMaxD;
          float z = b1k;
#pragma unroll
          for (int d = 0; d < DK; ++d) z = __fmaf_rn(w1r[d], xr[d], z);
          hw[crow(r) * kEncC1] = fmaxf(z, 0.f);
          __builtin_amdgcn_sched_barrier(0);
        }
        __syncthreads();
        // ---- dW2 tiles (channels c = mt*32 + i) x (conv1 channels kt*32 + i), K = the 32 rows
        const float gsc = gsb[mt * 32 + i];
        float av[16];
        int cnt = 0;
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const uint32_t bit = (uint32_t)(mb[mt * 16 + s] >> (i + 32 * h)) & 1u;
          av[s] = bit ? gsc : 0.f;
          cnt += (int)bit;
        }
        if (wave < 4) gb2 += gsc * (float)cnt;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float* hr = big + h1_at(4 * h, (kt0 + q) * 32 + i);
#pragma unroll
          for (int s = 0; s < 16; ++s) accB[q] = mfma32x32x2(av[s], hr[crow(s) * kEncC1], accB[q]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  }
  // ---- partial slab of this workgroup
  float* out = P.partial + (size_t)g * EncOff::size(D);
  if constexpr (ROLE == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k = wave * 32 + mfma_row(r, lane);
      if (i < D) gst(out + (EncOff::w1(D) + (int64_t)k * D + i), accW1[r]);
    }
    const float v = gb1 + __shfl_xor(gb1, 32, 64);
    if (h == 0) gst(out + (EncOff::b1(D) + k_own), v);
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c = mt * 32 + mfma_row(r, lane), k = (kt0 + q) * 32 + i;
        gst(out + (EncOff::w2(D) + (int64_t)c * kEncC1 + k), accB[q][r]);
      }
    const float v = gb2 + __shfl_xor(gb2, 32, 64);
    if (wave < 4 && h == 0) gst(out + (EncOff::b2(D) + wave * 32 + i), v);
  }
}

// ================================================================== reduce + Adam
__global__ __launch_bounds__(256) void enc_adam_kernel(EncAdamArgs a) {
  const EncAdamProb& P = a.p[blockIdx.y];
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= a.size) return;
  float g = 0.f;
  for (int w = 0; w < a.nwg; ++w) g += gld(P.partial + ((size_t)w * a.size + e));
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
#define TD3_ENC_BWD(DK)                                                                        \
  hipLaunchKernelGGL((enc_bwd_kernel<DK, 0>), grid, dim3(512), enc_bwd_lds<0>(), s, a);       \
  hipLaunchKernelGGL((enc_bwd_kernel<DK, 1>), grid, dim3(512), enc_bwd_lds<1>(), s, a)
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
