// Shared device/host helpers for libtd3hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

// Ordering events (stream -> stream waits, host completion checks): device-scope release.  The
// default system-scope release writes back the L2s at every record: ~4 us of GPU time per
// step for the ring's read event (C2 9.60k -> 9.97k steps/s without it).  The data these events
// order is written by kernels, whose end-of-kernel release already makes it device-visible.
#define TD3_EV_FLAGS (hipEventDisableTiming | hipEventReleaseToDevice)

// ---------------------------------------------------------------- error plumbing
namespace td3 {
void set_error(const char* fmt, ...);
}  // namespace td3

#define TD3_HIP(expr)                                                              \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) {                                                        \
      td3::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr,                  \
                     hipGetErrorString(_e));                                       \
      return -2;                                                                   \
    }                                                                              \
  } while (0)

#define TD3_ARG(cond, msg)                                                         \
  do {                                                                             \
    if (!(cond)) {                                                                 \
      td3::set_error("argument error: %s (%s)", msg, #cond);                        \
      return -1;                                                                   \
    }                                                                              \
  } while (0)

#define TD3_RC(expr)          \
  do {                        \
    int _rc = (expr);         \
    if (_rc) return _rc;      \
  } while (0)

namespace td3 {

constexpr int kWave = 64;
constexpr int kTile = 32;   // MFMA 32x32 output tile; every feature dim is padded to it

__host__ __device__ inline int pad32(int x) { return (x + 31) & ~31; }
__host__ __device__ inline int pad4(int x) { return (x + 3) & ~3; }

// LDS row stride (floats) for a [32][Kp] tile read with ds_read_b128 by the
// 32x32x2 fragment pattern: stride == 4 (mod 64) dwords is conflict-free for
// the gfx950 b128 lane groups (MI355X_MICROARCH.md §LDS).
__host__ __device__ inline int lds_stride(int kp) { return kp + ((4 - kp) % 64 + 64) % 64; }

// ---------------------------------------------------------------- Philox4x32-10
struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 ctr, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t hi0 = __umulhi(M0, ctr.x), lo0 = M0 * ctr.x;
    uint32_t hi1 = __umulhi(M1, ctr.z), lo1 = M1 * ctr.z;
    ctr = u32x4{hi1 ^ ctr.y ^ k0, lo1, hi0 ^ ctr.w ^ k1, lo0};
    k0 += W0;
    k1 += W1;
  }
  return ctr;
}

// Stream ids of the per-step Philox draws.
enum : uint32_t { kStreamIndex = 1u, kStreamNoise = 2u, kStreamFill = 3u };

// Uniform integer in [0, n) from 64 random bits (multiply-high; bias < n / 2^64).
__device__ __forceinline__ uint64_t philox_index(uint64_t seed, uint64_t step, uint32_t row,
                                                 uint64_t n) {
  u32x4 c{row, kStreamIndex, (uint32_t)step, (uint32_t)(step >> 32)};
  u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  uint64_t bits = ((uint64_t)r.x << 32) | r.y;
  return __umul64hi(bits, n);
}

__device__ __forceinline__ float u01_open(uint32_t x) {   // (0, 1]
  return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

// Four standard normals per counter (Box-Muller on two Philox outputs pairs).
__device__ __forceinline__ void philox_normal4(uint64_t seed, uint64_t step, uint32_t stream,
                                               uint32_t idx, float out[4]) {
  u32x4 c{idx, stream, (uint32_t)step, (uint32_t)(step >> 32)};
  u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  float u1 = u01_open(r.x), u2 = u01_open(r.y), u3 = u01_open(r.z), u4 = u01_open(r.w);
  // hardware transcendentals (v_log_f32 = log2, v_sqrt_f32, v_sin / v_cos_f32 of revolutions):
  // u is in [2^-24, 1], so the libm range / denormal fix-ups (a long chain on the policy head's
  // tail) are not needed
  constexpr float kM2Ln2 = -2.0f * 0.693147180559945f;
  const float rad1 = __builtin_amdgcn_sqrtf(kM2Ln2 * __builtin_amdgcn_logf(u1));
  const float rad2 = __builtin_amdgcn_sqrtf(kM2Ln2 * __builtin_amdgcn_logf(u3));
  const float s1 = __builtin_amdgcn_sinf(u2), c1 = __builtin_amdgcn_cosf(u2);
  const float s2 = __builtin_amdgcn_sinf(u4), c2 = __builtin_amdgcn_cosf(u4);
  out[0] = rad1 * c1;
  out[1] = rad1 * s1;
  out[2] = rad2 * c2;
  out[3] = rad2 * s2;
}

// ---------------------------------------------------------------- wave reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------- MFMA
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma32x32x2(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// C/D map of v_mfma_f32_32x32x2_f32: register r of lane l holds
// row (r&3) + 8*(r>>2) + 4*(l>>5), column l&31 (cdna_hip_programming.md §3).
__device__ __forceinline__ int mfma_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// Device-side step counters (read inside graph-replayed kernels).
struct Counters {
  int64_t total_it;     // TD3_base.total_it (TD3_base.py:19)
  int64_t critic_step;  // critic Adam step (torch state['step'])
  int64_t actor_step;   // actor Adam step
  int64_t pad;
  // beta^step of the Adam bias corrections (torch adam.py:531-533: 1 - beta**step), kept as running
  // products by the step bump so no workgroup evaluates pow(): [0] beta1^critic_step,
  // [1] beta2^critic_step, [2] beta1^actor_step, [3] beta2^actor_step
  double pw[4];
  double beta[4];       // the factor of each pw[] (critic beta1, beta2, actor beta1, beta2)
};

}  // namespace td3
