// TD3 gradient-step kernels for gfx950 (MI355X).
//
// What each kernel restates (reference = /root/reference):
//   gemm_kernel<0,*>      nn.Linear forward + ReLU, with the previous layer's
//                         LayerNorm (ReLU -> LN order, TD3_featured.py:41-46 / :75-80)
//                         applied to the input rows in the prologue
//   gemm_kernel<1,*>      dX = dZ * W of a Linear, with LN-backward + ReLU-backward
//                         of the following layer applied to the dZ rows in the prologue
//   head_kernel           last LN + output Linear + {target smoothing :131-137,
//                         max_action*tanh :47-48, Q value :81}
//   critic_loss_kernel    min(Q1',Q2'), y = r + nd*gamma*min (:140-142), mse grads (:148)
//   actor_loss_kernel     -mean(Q1(s, pi(s))) backward into LN3 (:159)
//   actor_head_bwd_kernel dQ1/da -> tanh / max_action backward -> actor head backward
//   dw_kernel             weight / bias / LN-affine grads (batch reductions) fused
//                         with torch Adam (adam.py:457-547) and Polyak (:167-171)
//
// Compute dtype: fp32 everywhere.  Matrix products use v_mfma_f32_32x32x2_f32
// (exact fp32 FMA chain, MI355X_MICROARCH.md § Matrix cores).
#include <math.h>

#include "kernels.h"

namespace td3 {

// ================================================================== helpers
template <int Q>
__device__ __forceinline__ void ln_stats(const float (&x)[Q], int K, int lane, float& mean,
                                         float& rstd) {
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < Q; ++q)
    if (lane + 64 * q < K) s += x[q];
  s = wave_sum(s);
  mean = s / (float)K;
  float v = 0.f;
#pragma unroll
  for (int q = 0; q < Q; ++q)
    if (lane + 64 * q < K) {
      float d = x[q] - mean;
      v += d * d;
    }
  v = wave_sum(v) / (float)K;
  rstd = 1.0f / sqrtf(v + 1e-5f);
}

// dH of LayerNorm followed by the ReLU mask, for one row held as x[q] (col lane+64q).
// gx = gu*gamma; dh = rstd*((gx - mean(gx)) - xhat*mean(gx*xhat)); dz = h>0 ? dh : 0.
template <int Q>
__device__ __forceinline__ void ln_relu_bwd(const float (&gu)[Q], const float (&h)[Q],
                                            const float* __restrict__ gam, int K, int lane,
                                            float mean, float rstd, int norm, float (&gz)[Q]) {
  if (!norm) {
#pragma unroll
    for (int q = 0; q < Q; ++q) gz[q] = h[q] > 0.f ? gu[q] : 0.f;
    return;
  }
  float gx[Q], xh[Q];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int c = lane + 64 * q;
    if (c < K) {
      xh[q] = (h[q] - mean) * rstd;
      gx[q] = gu[q] * gam[c];
      s1 += gx[q];
      s2 += gx[q] * xh[q];
    } else {
      xh[q] = 0.f;
      gx[q] = 0.f;
    }
  }
  const float m1 = wave_sum(s1) / (float)K;
  const float m2 = wave_sum(s2) / (float)K;
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const float dh = rstd * ((gx[q] - m1) - xh[q] * m2);
    gz[q] = (h[q] > 0.f && lane + 64 * q < K) ? dh : 0.f;
  }
}

// Head value: LN(h) . w + b over one row (Q cols per lane); returns the full sum on every lane.
template <int Q>
__device__ __forceinline__ float head_dot(const float (&x)[Q], int K, int lane,
                                          const float* __restrict__ g, const float* __restrict__ bb,
                                          const float* __restrict__ w, float bias) {
  float u[Q];
  if (g) {
    float mean, rstd;
    ln_stats<Q>(x, K, lane, mean, rstd);
    const float nb = -mean * rstd;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int c = lane + 64 * q;
      u[q] = c < K ? (x[q] * rstd + nb) * g[c] + bb[c] : 0.f;
    }
  } else {
#pragma unroll
    for (int q = 0; q < Q; ++q) u[q] = x[q];
  }
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int c = lane + 64 * q;
    if (c < K) s += u[q] * w[c];
  }
  return wave_sum(s) + bias;
}

constexpr int QR = 8;   // row-kernel columns per lane: rows up to 512 wide

template <int Q>
__device__ __forceinline__ void load_row(const float* __restrict__ p, int K, int lane, float (&x)[Q]) {
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int c = lane + 64 * q;
    x[q] = c < K ? p[c] : 0.f;
  }
}

template <int Q>
__device__ __forceinline__ void store_row(float* __restrict__ p, int ld, int lane, const float (&x)[Q]) {
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int c = lane + 64 * q;
    if (c < ld) p[c] = x[q];
  }
}

// ================================================================== batch-row GEMM stage
// Workgroup = 4 waves = one 32-row batch tile x (32*WN) output columns.
//  * prologue: the workgroup's 32 A rows (full Kp) are read from HBM/L2 with float4
//    loads, transformed row-wise (LayerNorm fwd, or LN bwd + ReLU bwd) by one wave
//    per row and written to an LDS tile [32][S] (S == 4 mod 64: conflict-free b128
//    fragment reads); n-tile 0 also stores the transformed rows for the dW kernel.
//  * main loop: each wave owns a 32x32 output tile and a 1/WK slice of K; per 32-deep
//    chunk a lane reads 16 A values (4x ds_read_b128) and 16 B values, and issues 16
//    v_mfma_f32_32x32x2_f32 (lane half h supplies k = 16h + s of MFMA s).
//  * WK > 1: the WK partial tiles are summed through LDS; epilogue bias/ReLU.
template <int MODE, int WN>
__global__ __launch_bounds__(256) void gemm_kernel(const GemmProb* __restrict__ probs, int nprob,
                                                   int Bp, Counters* bump, int bump_actor) {
  extern __shared__ float4 smem4[];
  float* smem = reinterpret_cast<float*>(smem4);
  constexpr int WK = 4 / WN;
  const int b = blockIdx.x;
  if (bump && b == 0 && threadIdx.x == 0) {
    bump->total_it += 1;                       // TD3_featured.py:124
    bump->critic_step += 1;
    if (bump_actor) bump->actor_step += 1;
  }
  int pi = 0;
  for (int i = 1; i < nprob; ++i)
    if (b >= probs[i].tile_begin) pi = i;
  const GemmProb& P = probs[pi];
  const int mtiles = Bp >> 5;
  const int t = b - P.tile_begin;
  const int mt = t % mtiles, nt = t / mtiles;
  const int m0 = mt << 5;
  const int n0 = nt * 32 * WN;
  const int Kp = P.Kp;
  const int S = lds_stride(Kp);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool store_a = (nt == 0) && (P.Aout != nullptr);
  const bool store_stats = (nt == 0) && (P.stats != nullptr);

  // ---------------- prologue: 8 rows per wave, lane owns cols lane*4 + 256q
  for (int rr = 0; rr < 8; ++rr) {
    const int row = wave * 8 + rr, grow = m0 + row;
    float4 x[2];
    bool valid[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c = lane * 4 + 256 * q;
      valid[q] = c < Kp;
      x[q] = valid[q] ? *reinterpret_cast<const float4*>(P.A + (size_t)grow * P.lda + c)
                      : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (P.pro == kProLN) {
      const int K = P.Kreal;
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int c = lane * 4 + 256 * q;
        if (c + 0 < K) s += x[q].x;
        if (c + 1 < K) s += x[q].y;
        if (c + 2 < K) s += x[q].z;
        if (c + 3 < K) s += x[q].w;
      }
      const float mean = wave_sum(s) / (float)K;
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int c = lane * 4 + 256 * q;
        float d;
        if (c + 0 < K) { d = x[q].x - mean; v += d * d; }
        if (c + 1 < K) { d = x[q].y - mean; v += d * d; }
        if (c + 2 < K) { d = x[q].z - mean; v += d * d; }
        if (c + 3 < K) { d = x[q].w - mean; v += d * d; }
      }
      const float rstd = 1.0f / sqrtf(wave_sum(v) / (float)K + 1e-5f);
      const float nb = -mean * rstd;
      if (store_stats && lane == 0) {
        P.stats[grow] = mean;
        P.stats[Bp + grow] = rstd;
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if (!valid[q]) continue;
        const int c = lane * 4 + 256 * q;
        const float4 g = *reinterpret_cast<const float4*>(P.lng + c);
        const float4 bb = *reinterpret_cast<const float4*>(P.lnb + c);
        x[q].x = (x[q].x * rstd + nb) * g.x + bb.x;
        x[q].y = (x[q].y * rstd + nb) * g.y + bb.y;
        x[q].z = (x[q].z * rstd + nb) * g.z + bb.z;
        x[q].w = (x[q].w * rstd + nb) * g.w + bb.w;
      }
    } else if (P.pro == kProLNBwd || P.pro == kProReluBwd) {
      float4 hh[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int c = lane * 4 + 256 * q;
        hh[q] = valid[q] ? *reinterpret_cast<const float4*>(P.H + (size_t)grow * P.ldh + c)
                         : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      if (P.pro == kProLNBwd) {
        const int K = P.Kreal;
        const float mean = P.stats[grow], rstd = P.stats[Bp + grow];
        float4 xh[2], gx[2];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int c = lane * 4 + 256 * q;
          float4 g = valid[q] ? *reinterpret_cast<const float4*>(P.lng + c)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
          xh[q].x = (hh[q].x - mean) * rstd;
          xh[q].y = (hh[q].y - mean) * rstd;
          xh[q].z = (hh[q].z - mean) * rstd;
          xh[q].w = (hh[q].w - mean) * rstd;
          gx[q].x = x[q].x * g.x;
          gx[q].y = x[q].y * g.y;
          gx[q].z = x[q].z * g.z;
          gx[q].w = x[q].w * g.w;
          if (c + 0 < K) { s1 += gx[q].x; s2 += gx[q].x * xh[q].x; }
          if (c + 1 < K) { s1 += gx[q].y; s2 += gx[q].y * xh[q].y; }
          if (c + 2 < K) { s1 += gx[q].z; s2 += gx[q].z * xh[q].z; }
          if (c + 3 < K) { s1 += gx[q].w; s2 += gx[q].w * xh[q].w; }
        }
        const float m1 = wave_sum(s1) / (float)K;
        const float m2 = wave_sum(s2) / (float)K;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          x[q].x = hh[q].x > 0.f ? rstd * ((gx[q].x - m1) - xh[q].x * m2) : 0.f;
          x[q].y = hh[q].y > 0.f ? rstd * ((gx[q].y - m1) - xh[q].y * m2) : 0.f;
          x[q].z = hh[q].z > 0.f ? rstd * ((gx[q].z - m1) - xh[q].z * m2) : 0.f;
          x[q].w = hh[q].w > 0.f ? rstd * ((gx[q].w - m1) - xh[q].w * m2) : 0.f;
        }
      } else {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          x[q].x = hh[q].x > 0.f ? x[q].x : 0.f;
          x[q].y = hh[q].y > 0.f ? x[q].y : 0.f;
          x[q].z = hh[q].z > 0.f ? x[q].z : 0.f;
          x[q].w = hh[q].w > 0.f ? x[q].w : 0.f;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (!valid[q]) continue;
      const int c = lane * 4 + 256 * q;
      *reinterpret_cast<float4*>(smem + row * S + c) = x[q];
      if (store_a) *reinterpret_cast<float4*>(P.Aout + (size_t)grow * P.ldao + c) = x[q];
    }
  }
  __syncthreads();

  // ---------------- MFMA main loop
  const int wn = wave % WN, wk = wave / WN;
  const int nch = Kp >> 5;
  const int cb = wk * nch / WK, ce = (wk + 1) * nch / WK;
  const int i = lane & 31, h = lane >> 5;
  const int ncol0 = n0 + wn * 32;
  const bool active = ncol0 < P.Nout;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  if (active) {
    const float* arow = smem + i * S + 16 * h;
    const float* wbase = (MODE == 0) ? P.W + (size_t)(ncol0 + i) * P.ldw + 16 * h
                                     : P.W + (size_t)(16 * h) * P.ldw + ncol0 + i;
    for (int c = cb; c < ce; ++c) {
      const int kb = c * 32;
      float av[16], bv[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(arow + kb + 4 * q);
        av[4 * q + 0] = v.x; av[4 * q + 1] = v.y; av[4 * q + 2] = v.z; av[4 * q + 3] = v.w;
      }
      if (MODE == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 v = *reinterpret_cast<const float4*>(wbase + kb + 4 * q);
          bv[4 * q + 0] = v.x; bv[4 * q + 1] = v.y; bv[4 * q + 2] = v.z; bv[4 * q + 3] = v.w;
        }
      } else {
        const float* wc = wbase + (size_t)kb * P.ldw;
#pragma unroll
        for (int s = 0; s < 16; ++s) bv[s] = wc[(size_t)s * P.ldw];
      }
#pragma unroll
      for (int s = 0; s < 16; ++s) acc = mfma32x32x2(av[s], bv[s], acc);
    }
  }

  // ---------------- epilogue
  if constexpr (WK == 1) {
    if (active) {
      const int col = ncol0 + i;
      const float bias = (MODE == 0 && P.bias) ? P.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = mfma_row(r, lane);
        float v = acc[r];
        if (MODE == 0 && P.bias) v = v + bias;
        if (P.relu) v = fmaxf(v, 0.f);
        P.C[(size_t)(m0 + row) * P.ldc + col] = v;
      }
    }
  } else {
    __syncthreads();
    float* red = smem;  // [4][32][33]
#pragma unroll
    for (int r = 0; r < 16; ++r) red[(wave * 32 + mfma_row(r, lane)) * 33 + i] = acc[r];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = threadIdx.x + 256 * q;
      const int row = e >> 5, col = e & 31;
      float v = red[row * 33 + col];
#pragma unroll
      for (int w = 1; w < 4; ++w) v = v + red[(w * 32 + row) * 33 + col];
      if (MODE == 0 && P.bias) v = v + P.bias[n0 + col];
      if (P.relu) v = fmaxf(v, 0.f);
      P.C[(size_t)(m0 + row) * P.ldc + n0 + col] = v;
    }
  }
}

// ================================================================== heads (row-wise)
__global__ __launch_bounds__(256) void head_kernel(HeadArgs a) {
  const HeadProb& P = a.probs[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.Bp) return;
  float x[QR];
  load_row<QR>(P.H3 + (size_t)row * P.ldh, P.K3, lane, x);
  float u[QR];
  if (P.lng) {
    float mean, rstd;
    ln_stats<QR>(x, P.K3, lane, mean, rstd);
    const float nb = -mean * rstd;
#pragma unroll
    for (int q = 0; q < QR; ++q) {
      const int c = lane + 64 * q;
      u[q] = c < P.K3 ? (x[q] * rstd + nb) * P.lng[c] + P.lnb[c] : 0.f;
    }
    if (P.stats && lane == 0) {
      P.stats[row] = mean;
      P.stats[a.Bp + row] = rstd;
    }
  } else {
#pragma unroll
    for (int q = 0; q < QR; ++q) u[q] = x[q];
  }
  if (P.U3) store_row<QR>(P.U3 + (size_t)row * P.ldu, P.ldu, lane, u);
  float zl = 0.f;
  for (int o = 0; o < P.nout; ++o) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < QR; ++q) {
      const int c = lane + 64 * q;
      if (c < P.K3) s += u[q] * P.W4[(size_t)o * P.ldw + c];
    }
    const float z = wave_sum(s) + P.b4[o];
    if (lane == o) zl = z;
  }
  if (lane >= P.nout) return;
  const int o = lane;
  const bool live = row < a.B;
  if (P.mode == kHeadTargetAction) {
    // TD3_featured.py:131-137 (noise = randn_like(action) * policy_noise, clamped)
    float z;
    if (a.gen_noise) {
      float g4[4];
      philox_normal4(a.seed, (uint64_t)a.ctr->total_it, kStreamNoise, (uint32_t)(row * 8 + (o >> 2)), g4);
      z = g4[o & 3];
      P.noise[(size_t)row * P.ldn + o] = z;
    } else {
      z = P.noise[(size_t)row * P.ldn + o];
    }
    float n = z * a.policy_noise;
    n = fminf(fmaxf(n, -a.noise_clip), a.noise_clip);
    float v = a.max_action * tanhf(zl) + n;
    v = fminf(fmaxf(v, -a.max_action), a.max_action);
    P.out[(size_t)row * P.ldo + P.out_col + o] = live ? v : 0.f;
  } else if (P.mode == kHeadPolicy) {
    const float th = tanhf(zl);                                  // TD3_featured.py:47-48
    P.out[(size_t)row * P.ldo + P.out_col + o] = live ? a.max_action * th : 0.f;
    P.tanh_out[(size_t)row * 32 + o] = th;
  } else {
    if (o == 0) P.out[row] = zl;
  }
}

__global__ __launch_bounds__(256) void critic_loss_kernel(CriticLossArgs a, float two_over_b) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.Bp) return;
  const bool live = row < a.B;
  float tq[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    float x[QR];
    load_row<QR>(a.TH3[j] + (size_t)row * a.ldh, a.K3, lane, x);
    tq[j] = head_dot<QR>(x, a.K3, lane, a.norm ? a.Tlng[j] : nullptr, a.Tlnb[j], a.TW4[j], a.Tb4[j][0]);
  }
  const float tmin = fminf(tq[0], tq[1]);                             // :141
  const float y = a.R[row] + (a.ND[row] * a.discount) * tmin;        // :142
  if (lane == 0) a.Y[row] = y;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float d = a.Qv[j][row] - y;
    const float dq = live ? two_over_b * d : 0.f;                    // mse_loss backward
    if (lane == 0) {
      a.sqerr[j * a.Bp + row] = live ? d * d : 0.f;
      a.GZ4[j][(size_t)row * a.ldgz4] = dq;
    }
    float gu[QR], h[QR], gz[QR];
#pragma unroll
    for (int q = 0; q < QR; ++q) {
      const int c = lane + 64 * q;
      gu[q] = c < a.K3 ? dq * a.W4[j][c] : 0.f;
    }
    load_row<QR>(a.H3[j] + (size_t)row * a.ldh, a.K3, lane, h);
    float mean = 0.f, rstd = 1.f;
    if (a.norm) {
      mean = a.stats3[j][row];
      rstd = a.stats3[j][a.Bp + row];
    }
    ln_relu_bwd<QR>(gu, h, a.lng3[j], a.K3, lane, mean, rstd, a.norm, gz);
    store_row<QR>(a.GU3[j] + (size_t)row * a.ldh, a.ldh, lane, gu);
    store_row<QR>(a.GZ3[j] + (size_t)row * a.ldh, a.ldh, lane, gz);
  }
}

__global__ __launch_bounds__(256) void actor_loss_kernel(ActorLossArgs a, float neg_inv_b) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.Bp) return;
  float h[QR];
  load_row<QR>(a.H3 + (size_t)row * a.ldh, a.K3, lane, h);
  float mean = 0.f, rstd = 1.f;
  if (a.norm) ln_stats<QR>(h, a.K3, lane, mean, rstd);
  const float q = head_dot<QR>(h, a.K3, lane, a.norm ? a.lng : nullptr, a.lnb, a.W4, a.b4[0]);
  if (lane == 0) a.Qv[row] = q;
  const float dq = row < a.B ? neg_inv_b : 0.f;                    // d(-mean)/dQ
  float gu[QR], gz[QR];
#pragma unroll
  for (int qq = 0; qq < QR; ++qq) {
    const int c = lane + 64 * qq;
    gu[qq] = c < a.K3 ? dq * a.W4[c] : 0.f;
  }
  ln_relu_bwd<QR>(gu, h, a.lng, a.K3, lane, mean, rstd, a.norm, gz);
  store_row<QR>(a.GZ3 + (size_t)row * a.ldh, a.ldh, lane, gz);
}

__global__ __launch_bounds__(256) void actor_head_bwd_kernel(ActorHeadBwdArgs a) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.Bp) return;
  // Q1 layer-1: dZ1 = relu'(LN1_bwd(dU1))
  float gu1[QR], h1[QR], gz1[QR];
  load_row<QR>(a.GU1 + (size_t)row * a.ld1, a.K1, lane, gu1);
  load_row<QR>(a.H1 + (size_t)row * a.ld1, a.K1, lane, h1);
  float mean = 0.f, rstd = 1.f;
  if (a.norm) {
    mean = a.stats1[row];
    rstd = a.stats1[a.Bp + row];
  }
  ln_relu_bwd<QR>(gu1, h1, a.lng1, a.K1, lane, mean, rstd, a.norm, gz1);
  // dL/da = dZ1 * W1[:, sd:sd+ad]  (cat([state, action]) backward, TD3_featured.py:74)
  float gz4 = 0.f;
  for (int o = 0; o < a.ad; ++o) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < QR; ++q) {
      const int c = lane + 64 * q;
      if (c < a.K1) s += gz1[q] * a.W1[(size_t)c * a.ldw1 + a.sd + o];
    }
    const float ga = wave_sum(s);
    if (lane == o) {
      const float t = a.T[(size_t)row * a.ldt + o];
      gz4 = row < a.B ? (ga * a.max_action) * (1.f - t * t) : 0.f;   // max_action*tanh backward
    }
  }
  if (lane < a.ad) a.GZ4[(size_t)row * a.ldgz4 + lane] = gz4;
  // actor head backward: dU3 = dZ4 * W4
  float gu3[QR];
#pragma unroll
  for (int q = 0; q < QR; ++q) gu3[q] = 0.f;
  for (int o = 0; o < a.ad; ++o) {
    const float g = __shfl(gz4, o, 64);
#pragma unroll
    for (int q = 0; q < QR; ++q) {
      const int c = lane + 64 * q;
      if (c < a.K3) gu3[q] += g * a.W4[(size_t)o * a.ldw4 + c];
    }
  }
  float h3[QR], gz3[QR];
  load_row<QR>(a.H3 + (size_t)row * a.ld3, a.K3, lane, h3);
  if (a.norm) {
    mean = a.stats3[row];
    rstd = a.stats3[a.Bp + row];
  }
  ln_relu_bwd<QR>(gu3, h3, a.lng3, a.K3, lane, mean, rstd, a.norm, gz3);
  store_row<QR>(a.GU3 + (size_t)row * a.ld3, a.ld3, lane, gu3);
  store_row<QR>(a.GZ3 + (size_t)row * a.ld3, a.ld3, lane, gz3);
}

__global__ __launch_bounds__(256) void lnbwd_rows_kernel(const LnBwdProb* __restrict__ probs, int Bp,
                                                         int norm) {
  const LnBwdProb& P = probs[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= Bp) return;
  float gu[QR], h[QR], gz[QR];
  load_row<QR>(P.GU + (size_t)row * P.ld, P.K, lane, gu);
  load_row<QR>(P.H + (size_t)row * P.ld, P.K, lane, h);
  float mean = 0.f, rstd = 1.f;
  if (norm) {
    mean = P.stats[row];
    rstd = P.stats[Bp + row];
  }
  ln_relu_bwd<QR>(gu, h, P.lng, P.K, lane, mean, rstd, norm, gz);
  store_row<QR>(P.GZ + (size_t)row * P.ld, P.ld, lane, gz);
}

// ================================================================== Adam / Polyak
struct AdamK {
  float w1, b2, c2, bc2s, negss, eps, tau, omt, gscale;
};

__device__ __forceinline__ AdamK make_adam(const AdamArgs& a) {
  AdamK k;
  const int64_t step = a.which ? a.ctr->actor_step : a.ctr->critic_step;
  const double bc1 = 1.0 - pow(a.beta1, (double)step);
  const double bc2 = 1.0 - pow(a.beta2, (double)step);
  k.negss = (float)(-(a.lr / bc1));
  k.bc2s = (float)sqrt(bc2);
  k.w1 = (float)(1.0 - a.beta1);
  k.b2 = (float)a.beta2;
  k.c2 = (float)(1.0 - a.beta2);
  k.eps = (float)a.eps;
  k.tau = a.tau;
  k.omt = (float)(1.0 - (double)a.tau);
  k.gscale = a.grad_scale;
  return k;
}

// torch _single_tensor_adam (adam.py:520-547): lerp, mul/addcmul, sqrt/div/add, addcdiv.
__device__ __forceinline__ void adam_elem(float* __restrict__ p, float* __restrict__ m,
                                          float* __restrict__ v, float g, const AdamK& k,
                                          float* __restrict__ t) {
  float mm = *m, vv = *v, pp = *p;
  mm = __fmaf_rn(k.w1, g - mm, mm);
  vv = vv * k.b2;
  vv = vv + (k.c2 * g) * g;
  const float denom = sqrtf(vv) / k.bc2s + k.eps;
  pp = pp + (k.negss * mm) / denom;
  *m = mm;
  *v = vv;
  *p = pp;
  if (t) *t = k.tau * pp + k.omt * (*t);     // TD3_featured.py:167-171
}

__device__ __forceinline__ void apply_grad(const DwArgs& a, const AdamK& k, int64_t idx, float g) {
  if (a.mode == kDwGrad) {
    a.adam.G[idx] = g;
  } else {
    adam_elem(a.adam.P + idx, a.adam.M + idx, a.adam.V + idx, g, k,
              a.mode == kDwAdamPolyak ? a.adam.T + idx : nullptr);
  }
}

// dW[n][k] = sum_r dZ[r][n] * U[r][k]  (32x32 tile per workgroup, rows split over 4 waves),
// then bias / LN-affine reductions (k-tile 0 only) and the fused optimizer update.
__global__ __launch_bounds__(256) void dw_kernel(DwArgs a) {
  __shared__ float red[4 * 32 * 33];
  __shared__ float vred[3][8][32];
  const int b = blockIdx.x;
  int pi = 0;
  for (int i = 1; i < a.nprob; ++i)
    if (b >= a.probs[i].tile_begin) pi = i;
  const DwProb& P = a.probs[pi];
  const int t = b - P.tile_begin;
  const int kt = t % P.ntk, nt = t / P.ntk;
  const int n0 = nt * 32, k0 = kt * 32;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i = lane & 31, h = lane >> 5;
  const int nrc = a.Bp >> 5;
  const int cb = wave * nrc / 4, ce = (wave + 1) * nrc / 4;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const float* gp = P.G + n0 + i;
  const float* up = P.U + k0 + i;
  for (int rc = cb; rc < ce; ++rc) {
    const int rb = rc * 32 + 16 * h;
    float av[16], bv[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      av[s] = gp[(size_t)(rb + s) * P.ldg];
      bv[s] = up[(size_t)(rb + s) * P.ldu];
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = mfma32x32x2(av[s], bv[s], acc);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) red[(wave * 32 + mfma_row(r, lane)) * 33 + i] = acc[r];

  const bool vec = (kt == 0);
  if (vec) {
    // column sums over the batch: db = sum dZ, dgamma = sum dU*xhat, dbeta = sum dU
    const int c = threadIdx.x & 31, rg = threadIdx.x >> 5;
    float sb = 0.f, sg = 0.f, sbeta = 0.f;
    const bool ln = P.offg >= 0;
    for (int r = rg; r < a.Bp; r += 8) {
      sb += P.G[(size_t)r * P.ldg + n0 + c];
      if (ln) {
        const float gu = P.GU[(size_t)r * P.ldgu + n0 + c];
        const float xh = (P.H[(size_t)r * P.ldh + n0 + c] - P.stats[r]) * P.stats[a.Bp + r];
        sg += gu * xh;
        sbeta += gu;
      }
    }
    vred[0][rg][c] = sb;
    vred[1][rg][c] = sg;
    vred[2][rg][c] = sbeta;
  }
  __syncthreads();
  const AdamK k = make_adam(a.adam);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e = threadIdx.x + 256 * q;
    const int n = e >> 5, kk = e & 31;
    float g = red[n * 33 + kk];
#pragma unroll
    for (int w = 1; w < 4; ++w) g = g + red[(w * 32 + n) * 33 + kk];
    apply_grad(a, k, P.offW + (int64_t)(n0 + n) * P.Kp + k0 + kk, g);
  }
  if (vec && threadIdx.x < 32) {
    const int c = threadIdx.x;
    float sb = 0.f, sg = 0.f, sbeta = 0.f;
#pragma unroll
    for (int rg = 0; rg < 8; ++rg) {
      sb += vred[0][rg][c];
      sg += vred[1][rg][c];
      sbeta += vred[2][rg][c];
    }
    apply_grad(a, k, P.offb + n0 + c, sb);
    if (P.offg >= 0) {
      apply_grad(a, k, P.offg + n0 + c, sg);
      apply_grad(a, k, P.offbeta + n0 + c, sbeta);
    }
  }
}

__global__ __launch_bounds__(256) void adam_flat_kernel(AdamArgs a, int64_t n, int polyak) {
  const AdamK k = make_adam(a);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float g = a.G[i] * k.gscale;
    adam_elem(a.P + i, a.M + i, a.V + i, g, k, polyak ? a.T + i : nullptr);
  }
}

__global__ __launch_bounds__(256) void polyak_flat_kernel(float* T, const float* P, int64_t n, float tau,
                                                          float omt) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    T[i] = tau * P[i] + omt * T[i];
}

// ================================================================== launchers
template <int MODE, int WN>
static void gemm_launch_t(const GemmProb* d, int nprob, int nblocks, int Bp, int lds, Counters* bump,
                          int bump_actor, hipStream_t s) {
  hipLaunchKernelGGL((gemm_kernel<MODE, WN>), dim3(nblocks), dim3(256), lds, s, d, nprob, Bp, bump,
                     bump_actor);
}

int launch_gemm(int mode, int wn, const GemmProb* d, int nprob, int nblocks, int Bp, int lds,
                Counters* bump, int bump_actor, hipStream_t s) {
  if (nblocks <= 0) return 0;
  if (mode == 0 && wn == 1) gemm_launch_t<0, 1>(d, nprob, nblocks, Bp, lds, bump, bump_actor, s);
  else if (mode == 0 && wn == 4) gemm_launch_t<0, 4>(d, nprob, nblocks, Bp, lds, bump, bump_actor, s);
  else if (mode == 1 && wn == 1) gemm_launch_t<1, 1>(d, nprob, nblocks, Bp, lds, bump, bump_actor, s);
  else if (mode == 1 && wn == 4) gemm_launch_t<1, 4>(d, nprob, nblocks, Bp, lds, bump, bump_actor, s);
  else {
    set_error("launch_gemm: unsupported mode %d wn %d", mode, wn);
    return -1;
  }
  TD3_HIP(hipGetLastError());
  return 0;
}

int launch_heads(const HeadArgs& a, int nprob, hipStream_t s) {
  hipLaunchKernelGGL(head_kernel, dim3(a.Bp / 4, nprob), dim3(256), 0, s, a);
  TD3_HIP(hipGetLastError());
  return 0;
}

int launch_critic_loss(const CriticLossArgs& a, hipStream_t s) {
  const float two_over_b = (float)(2.0 / (double)a.B);
  hipLaunchKernelGGL(critic_loss_kernel, dim3(a.Bp / 4), dim3(256), 0, s, a, two_over_b);
  TD3_HIP(hipGetLastError());
  return 0;
}

int launch_actor_loss(const ActorLossArgs& a, hipStream_t s) {
  const float neg_inv_b = (float)(-1.0) / (float)a.B;
  hipLaunchKernelGGL(actor_loss_kernel, dim3(a.Bp / 4), dim3(256), 0, s, a, neg_inv_b);
  TD3_HIP(hipGetLastError());
  return 0;
}

int launch_actor_head_bwd(const ActorHeadBwdArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(actor_head_bwd_kernel, dim3(a.Bp / 4), dim3(256), 0, s, a);
  TD3_HIP(hipGetLastError());
  return 0;
}

int launch_lnbwd_rows(const LnBwdProb* d, int nprob, int Bp, int norm, hipStream_t s) {
  hipLaunchKernelGGL(lnbwd_rows_kernel, dim3(Bp / 4, nprob), dim3(256), 0, s, d, Bp, norm);
  TD3_HIP(hipGetLastError());
  return 0;
}

int launch_dw(const DwArgs& a, int nblocks, hipStream_t s) {
  if (nblocks <= 0) return 0;
  hipLaunchKernelGGL(dw_kernel, dim3(nblocks), dim3(256), 0, s, a);
  TD3_HIP(hipGetLastError());
  return 0;
}

int launch_adam_flat(const AdamArgs& a, int64_t n, int polyak, hipStream_t s) {
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(adam_flat_kernel, dim3(blocks), dim3(256), 0, s, a, n, polyak);
  TD3_HIP(hipGetLastError());
  return 0;
}

int launch_polyak_flat(float* T, const float* P, int64_t n, float tau, hipStream_t s) {
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 2048);
  const float omt = (float)(1.0 - (double)tau);
  hipLaunchKernelGGL(polyak_flat_kernel, dim3(blocks), dim3(256), 0, s, T, P, n, tau, omt);
  TD3_HIP(hipGetLastError());
  return 0;
}

int kernels_init() {
  const int max_lds = 160 * 1024;
  TD3_HIP(hipFuncSetAttribute((const void*)gemm_kernel<0, 1>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, max_lds));
  TD3_HIP(hipFuncSetAttribute((const void*)gemm_kernel<0, 4>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, max_lds));
  TD3_HIP(hipFuncSetAttribute((const void*)gemm_kernel<1, 1>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, max_lds));
  TD3_HIP(hipFuncSetAttribute((const void*)gemm_kernel<1, 4>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, max_lds));
  return 0;
}

}  // namespace td3
