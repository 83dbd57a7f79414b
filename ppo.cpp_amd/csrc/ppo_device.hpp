// ppo_device.hpp — device-side building blocks for gfx950 (CDNA4, wave64).
//
//  * Philox4x32-10 counter RNG + Box-Muller + Marsaglia-Tsang gamma (replaces at::normal /
//    at::_sample_dirichlet, include/rl_utils.h:34-37, :59-62) — counter-based, so samples do not
//    depend on stream, batching or thread order (fixes the README.md:80-85 determinism caveat).
//  * digamma / trigamma with ATen's calc_digamma / calc_trigamma structure (fp32).
//  * 16x16x4 f32 MFMA helpers for the "batch-on-lanes" layout used by every agent kernel:
//      a wave owns 16 batch rows; lane l = (j = l & 15, g = l >> 4); feature f of row j lives in
//      lane (j, g = (f >> 2) & 3), register (tile t = f >> 4, component r = f & 3).
//    The MFMA computes Z^T = W . H^T: A = W rows (out features), B = activations, D = Z^T tile.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f4 __attribute__((ext_vector_type(4)));

#define PPO_DEV __device__ __forceinline__
#define PPO_DEV_HOST __host__ __device__

// ------------------------------------------------------------------------------------------
// RNG contract (mirrored by oracle/ppo_oracle.c)
// ------------------------------------------------------------------------------------------
PPO_DEV void philox4x32(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                        uint32_t out[4]) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
    const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

PPO_DEV uint32_t mix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85EBCA6Bu;
  h ^= h >> 13; h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

PPO_DEV float u01(uint32_t x) { return ((float)(x >> 8) + 0.5f) * 5.9604644775390625e-8f; }

struct SampleKey {
  uint32_t k0, k1;
};
PPO_DEV SampleKey sample_key(uint64_t seed, int rank) {
  return SampleKey{(uint32_t)seed, (uint32_t)(seed >> 32) ^ (0x85EBCA6Bu * (uint32_t)(rank + 1))};
}
PPO_DEV void philox_draw(SampleKey k, long env, long step, uint32_t draw, uint32_t out[4]) {
  philox4x32((uint32_t)env, (uint32_t)step, (uint32_t)((uint64_t)step >> 32), draw, k.k0, k.k1, out);
}
PPO_DEV void box_muller(uint32_t a, uint32_t b, float& z0, float& z1) {
  const float u0 = u01(a), u1 = u01(b);
  const float r = sqrtf(-2.0f * logf(u0));
  const float th = 6.2831853071795865f * u1;
  float s, c;
  sincosf(th, &s, &c);
  z0 = r * c;
  z1 = r * s;
}

// Marsaglia-Tsang Gamma(alpha >= 1) — same acceptance test as ATen's sample_gamma.
PPO_DEV float gamma_mt(float alpha, SampleKey k, long env, long step, uint32_t draw_base) {
  const float d = alpha - 0.33333334f;
  const float cc = 1.0f / sqrtf(9.0f * d);
  for (uint32_t t = 0; t < 64; ++t) {
    uint32_t r[4];
    philox_draw(k, env, step, draw_base + t, r);
    float z, z1;
    box_muller(r[0], r[1], z, z1);
    const float y = 1.0f + cc * z;
    if (y <= 0.0f) continue;
    const float v = y * y * y;
    const float u = u01(r[2]);
    const float xx = z * z;
    if (u < 1.0f - 0.0331f * xx * xx) return d * v;
    if (logf(u) < 0.5f * xx + d * (1.0f - v + logf(v))) return d * v;
  }
  return d;
}

// The first Marsaglia-Tsang attempt's normal / uniform do not depend on alpha: act kernels draw
// them at kernel start (under the weight fetch) and finish with gamma_mt_d0, which is gamma_mt
// with attempt 0's draw supplied (same arithmetic, same result).
struct GammaDraw {
  float z, u;
};
PPO_DEV GammaDraw gamma_draw(SampleKey k, long env, long step, uint32_t draw) {
  uint32_t r[4];
  philox_draw(k, env, step, draw, r);
  float z, z1;
  box_muller(r[0], r[1], z, z1);
  return GammaDraw{z, u01(r[2])};
}
PPO_DEV float gamma_mt_d0(float alpha, GammaDraw d0, SampleKey k, long env, long step, uint32_t draw_base) {
  const float d = alpha - 0.33333334f;
  const float cc = 1.0f / sqrtf(9.0f * d);
  for (uint32_t t = 0; t < 64; ++t) {
    float z = d0.z, u = d0.u;
    if (t > 0) {
      const GammaDraw g = gamma_draw(k, env, step, draw_base + t);
      z = g.z;
      u = g.u;
    }
    const float y = 1.0f + cc * z;
    if (y <= 0.0f) continue;
    const float v = y * y * y;
    const float xx = z * z;
    if (u < 1.0f - 0.0331f * xx * xx) return d * v;
    if (logf(u) < 0.5f * xx + d * (1.0f - v + logf(v))) return d * v;
  }
  return d;
}

// Feistel permutation of [0,B) keyed by (seed, rank, epoch counter); replaces torch::randperm
// (ppo:490, ac:804). Mirrors orc_perm_index.
struct PermKey {
  uint32_t k[4];
  int half;
  uint32_t mask;
};
inline PermKey make_perm_key(uint64_t seed, int rank, long epoch_counter, long B) {
  auto hmix = [](uint32_t h) {
    h ^= h >> 16; h *= 0x85EBCA6Bu;
    h ^= h >> 13; h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
  };
  PermKey pk;
  int bits = 2;
  while ((1L << bits) < B) bits += 2;
  pk.half = bits / 2;
  pk.mask = (1u << pk.half) - 1u;
  const uint32_t base = hmix((uint32_t)seed ^ 0x1B873593u) ^ hmix((uint32_t)(seed >> 32) + 0x68E31DA4u) ^
                        hmix((uint32_t)rank * 0x632BE5ABu + 0x2545F491u) ^ hmix((uint32_t)epoch_counter * 2u + 1u);
  for (int r = 0; r < 4; ++r) pk.k[r] = hmix(base + (uint32_t)r * 0x9E3779B9u);
  return pk;
}
PPO_DEV uint32_t perm_index(uint32_t i, uint32_t B, const PermKey& pk) {
  uint32_t x = i;
  do {
    uint32_t L = x >> pk.half, R = x & pk.mask;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t F = mix32(R * 0x9E3779B1u + pk.k[r]) & pk.mask;
      const uint32_t nR = L ^ F;
      L = R;
      R = nR;
    }
    x = (L << pk.half) | R;
  } while (x >= B);
  return x;
}

// ------------------------------------------------------------------------------------------
// Special functions (fp32; ATen Math.h calc_digamma / calc_trigamma structure)
// ------------------------------------------------------------------------------------------
PPO_DEV float digammaf_(float x) {
  // valid for x > 0 (Beta concentrations are >= 1)
  float result = 0.0f;
  while (x < 10.0f) {
    result -= 1.0f / x;
    x += 1.0f;
  }
  if (x == 10.0f) return result + 2.25175258906672110764f;
  const float z = 1.0f / (x * x);
  float p = 8.33333333333333333333E-2f;
  p = p * z + -2.10927960927960927961E-2f;
  p = p * z + 7.57575757575757575758E-3f;
  p = p * z + -4.16666666666666666667E-3f;
  p = p * z + 3.96825396825396825397E-3f;
  p = p * z + -8.33333333333333333333E-3f;
  p = p * z + 8.33333333333333333333E-2f;
  return result + logf(x) - (0.5f / x) - z * p;
}
PPO_DEV float trigammaf_(float x) {
  float result = 0.0f;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    result += 1.0f / (x * x);
    x += 1.0f;
  }
  const float ixx = 1.0f / (x * x);
  result += (1.0f + 1.0f / (2.0f * x) + ixx * (1.0f / 6.0f - ixx * (1.0f / 30.0f - ixx * (1.0f / 42.0f)))) / x;
  return result;
}
// digamma and trigamma of one argument x >= 1 in one pass (the Beta loss gradient needs both at
// alpha, beta and alpha + beta): shift x to >= 6 with one v_rcp_f32 per step (at most 5, as
// predicated selects), then the asymptotic series. ~2 ulp; ATen's calc_digamma / calc_trigamma
// (IEEE divisions, shifts to 10 / by 6) agree to that accuracy.
PPO_DEV void digamma_trigamma(float x, float& dg, float& tg) {
  float d = 0.0f, t = 0.0f;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const bool m = x < 6.0f;
    const float r = __builtin_amdgcn_rcpf(x);
    d = m ? d - r : d;
    t = m ? fmaf(r, r, t) : t;
    x = m ? x + 1.0f : x;
  }
  const float r = __builtin_amdgcn_rcpf(x), r2 = r * r;
  dg = d + logf(x) - 0.5f * r -
       r2 * (1.0f / 12 - r2 * (1.0f / 120 - r2 * (1.0f / 252 - r2 * (1.0f / 240 - r2 * (1.0f / 132)))));
  tg = t + r * (1.0f + 0.5f * r + r2 * (1.0f / 6 - r2 * (1.0f / 30 - r2 * (1.0f / 42 - r2 * (1.0f / 30)))));
}
// lgamma, digamma and trigamma of one argument x >= 1 from one shared shift: lgamma(x) =
// Stirling(x + n) - log(x (x + 1) ... (x + n - 1)). Absolute lgamma error ~1e-6 near its zeros at
// 1 and 2 (the shift's log cancels there), relative ~1e-7 elsewhere.
PPO_DEV void lgamma_digamma_trigamma(float x, float& lg, float& dg, float& tg) {
  float d = 0.0f, t = 0.0f, prod = 1.0f;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const bool m = x < 6.0f;
    const float r = __builtin_amdgcn_rcpf(x);
    d = m ? d - r : d;
    t = m ? fmaf(r, r, t) : t;
    prod = m ? prod * x : prod;
    x = m ? x + 1.0f : x;
  }
  const float r = __builtin_amdgcn_rcpf(x), r2 = r * r, lx = logf(x);
  lg = ((x - 0.5f) * lx - x + 0.918938533204672742f) +
       r * (1.0f / 12 - r2 * (1.0f / 360 - r2 * (1.0f / 1260 - r2 * (1.0f / 1680)))) - logf(prod);
  dg = d + lx - 0.5f * r -
       r2 * (1.0f / 12 - r2 * (1.0f / 120 - r2 * (1.0f / 252 - r2 * (1.0f / 240 - r2 * (1.0f / 132)))));
  tg = t + r * (1.0f + 0.5f * r + r2 * (1.0f / 6 - r2 * (1.0f / 30 - r2 * (1.0f / 42 - r2 * (1.0f / 30)))));
}
PPO_DEV float softplusf_(float x) { return x > 20.0f ? x : log1pf(expf(x)); }
PPO_DEV float softplus_d(float x) {
  if (x > 20.0f) return 1.0f;
  const float z = expf(x);
  return z / (z + 1.0f);
}
PPO_DEV float xlogyf_(float a, float b) {
  if (b != b) return b;
  if (a == 0.0f) return 0.0f;
  return a * logf(b);
}

// ------------------------------------------------------------------------------------------
// MFMA + cross-lane helpers
// ------------------------------------------------------------------------------------------
PPO_DEV f4 mfma16(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
// split-bf16 operands (ppo_kernels.hpp split3_bits): 8 bf16 per lane as 4 dwords
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
PPO_DEV f4 mfma16bx(u32x4 a, u32x4 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
// two fp32 values -> their (hi, mid, lo) split-bf16 pieces, packed (x0 in the low half): hi = x with
// the low 16 bits cleared, mid = (x - hi) the same way, lo = the exact rest (at most 8 significant bits)
PPO_DEV void split3_pair(float x0, float x1, unsigned& hi, unsigned& mid, unsigned& lo) {
  const unsigned u0 = __float_as_uint(x0), u1 = __float_as_uint(x1);
  const float r0 = x0 - __uint_as_float(u0 & 0xffff0000u), r1 = x1 - __uint_as_float(u1 & 0xffff0000u);
  const unsigned v0 = __float_as_uint(r0), v1 = __float_as_uint(r1);
  const float l0 = r0 - __uint_as_float(v0 & 0xffff0000u), l1 = r1 - __uint_as_float(v1 & 0xffff0000u);
  hi = __builtin_amdgcn_perm(u1, u0, 0x07060302u);
  mid = __builtin_amdgcn_perm(v1, v0, 0x07060302u);
  lo = __builtin_amdgcn_perm(__float_as_uint(l1), __float_as_uint(l0), 0x07060302u);
}
typedef float f32x16 __attribute__((ext_vector_type(16)));
// eight fp32 values (one lane's k slots of a bf16 MFMA operand) -> their three pieces
struct Split3 {
  u32x4 hi, mid, lo;
};
PPO_DEV Split3 split3(const float (&x)[8]) {
  Split3 s;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    unsigned h, m, l;
    split3_pair(x[2 * p], x[2 * p + 1], h, m, l);
    s.hi[p] = h;
    s.mid[p] = m;
    s.lo[p] = l;
  }
  return s;
}
PPO_DEV f32x16 mfma_bx(u32x4 a, u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
// acc += A.B over one 16-k block as NP piece products, smallest first
// (NP = 6: k_upd's six, without mid.lo + lo.mid + lo.lo < 2^-21 |a.b|)
template <int NP>
PPO_DEV f32x16 mfma_split(const Split3& A, const Split3& B, f32x16 acc) {
  if constexpr (NP >= 9) acc = mfma_bx(A.lo, B.lo, acc);
  if constexpr (NP >= 8) {
    acc = mfma_bx(A.lo, B.mid, acc);
    acc = mfma_bx(A.mid, B.lo, acc);
  }
  acc = mfma_bx(A.lo, B.hi, acc);
  acc = mfma_bx(A.mid, B.mid, acc);
  acc = mfma_bx(A.hi, B.lo, acc);
  acc = mfma_bx(A.mid, B.hi, acc);
  acc = mfma_bx(A.hi, B.mid, acc);
  acc = mfma_bx(A.hi, B.hi, acc);
  return acc;
}

// two fp32 values exact in bf16 (e.g. byte values 0..255) packed as bf16 (x0 in the low half)
PPO_DEV unsigned pack_bf16_exact(float x0, float x1) {
  return __builtin_amdgcn_perm(__float_as_uint(x1), __float_as_uint(x0), 0x07060302u);
}

PPO_DEV float shfl_xor(float v, int m) { return __shfl_xor(v, m, 64); }

// Cross-lane moves that stay off the LDS pipe: DPP inside 16-lane rows, v_permlane{16,32}_swap
// across rows. xor16_sum(v) = v + v[lane ^ 16] and xor32_sum(v) = v + v[lane ^ 32], bitwise equal
// to the shuffle forms (the swaps hand both operands to every lane; float + is commutative).
template <int CTRL>
PPO_DEV float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
enum : int { kDppQuadXor1 = 0xB1, kDppQuadXor2 = 0x4E, kDppQuadMirror = 0x1B, kDppHalfMirror = 0x141, kDppRowRor8 = 0x128 };
// sum over each aligned group of 8 lanes, the same bits in all 8 (pairwise sums are commutative)
PPO_DEV float group8_sum(float v) {
  v += dpp_f<kDppQuadXor1>(v);
  v += dpp_f<kDppQuadXor2>(v);
  return v + dpp_f<kDppHalfMirror>(v);
}
PPO_DEV float xor16_sum(float v) {
  const auto p = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                                  false, false);
  return __builtin_bit_cast(float, (unsigned)p[0]) + __builtin_bit_cast(float, (unsigned)p[1]);
}
PPO_DEV float xor32_sum(float v) {
  const auto p = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                                  false, false);
  return __builtin_bit_cast(float, (unsigned)p[0]) + __builtin_bit_cast(float, (unsigned)p[1]);
}

// sum over the 4 lane-groups g (lanes j, j+16, j+32, j+48) — completes a per-row feature sum
PPO_DEV float row_allreduce(float v) { return xor32_sum(xor16_sum(v)); }

PPO_DEV f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }
PPO_DEV void st4(float* p, f4 v) { *reinterpret_cast<f4*>(p) = v; }
