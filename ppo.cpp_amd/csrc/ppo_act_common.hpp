// ppo_act_common.hpp — building blocks shared by the per-step act kernel (k_act3, ppo_act.hip) and
// the persistent rollout / critic kernels (k_rollout, k_values, ppo_rollout.hip) of the 256-wide
// agents. Kernels that use the same pieces in the same order produce bitwise identical results.
#pragma once

#include "ppo_agent.hpp"
#include "ppo_kernels.hpp"

namespace act {

constexpr int kActThreads = 512, kActWaves = 8;

template <int NTO, int NHT, int RT>
struct ActGeo {
  static constexpr int kActRows = 16 * RT;
  static constexpr int H = 256, OP = NTO * 16, NHP = 16 * NHT;
  static constexpr int LDX = ((OP + 63) / 64) * 64 + 4;
  static constexpr int LDH = H + 4;
  static constexpr int LDP = NHP + 4;
  static constexpr int NSP = 6 * H + NHP * H;  // staged params: b1 g1 be1 b2 g2 be2, head rows
  static constexpr int oXS = 0;
  static constexpr int oHB = oXS + kActRows * LDX;
  static constexpr int oSP = oHB + kActRows * LDH;
  static constexpr int oHBIAS = oSP + NSP;                    // NHP head biases
  static constexpr int oRED = oHBIAS + NHP;                   // 2 x 8 x 16
  static constexpr int oHP = oRED + 2 * kActWaves * kActRows;  // 8 x NHP x 16 head partials
  static constexpr int oPRE = oHP + kActWaves * NHP * kActRows;  // 16 x LDP
  static constexpr int total = oPRE + kActRows * LDP;
  // distribution scratch reuses the input / hidden-activation region (dead after layer 2)
  static constexpr int oITM = 0;                               // R x A x 2 x 4 (A <= 24)
  static constexpr int oLP = oITM + kActRows * 24 * 2 * 4;    // R x A x 2
  static_assert(oLP + kActRows * 24 * 2 <= oSP, "distribution scratch must fit in the XS/HB region");
  // staged param vectors inside SP
  static constexpr int sB1 = 0, sG1 = H, sBE1 = 2 * H, sB2 = 3 * H, sG2 = 4 * H, sBE2 = 5 * H, sW3 = 6 * H;
};

// one Linear layer for this wave's 2 output tiles x RT row tiles:
// acc[u][rt] (+)= W[32 w + 16 u + i][:] . IN[16 rt + j][:], A-operands streamed through a PD-deep
// register ring from the swizzled copy (sw_index: tile u, k-block t at wlane + 256 (NKB u + t));
// bfrag(t, rt) = this lane's B f4 for k-block t of row tile rt
template <int NKB, int PD, int RT, typename BF>
PPO_DEV void act_layer(f4 (&acc)[2][RT], PBuf wb, int wlane, BF bfrag) {
  constexpr int D = PD < NKB ? PD : NKB;
  f4 w[D][2];
#pragma unroll
  for (int p = 0; p < D; ++p)
#pragma unroll
    for (int u = 0; u < 2; ++u) w[p][u] = pld4(wb, wlane, 256 * (NKB * u + p));
  // keep the scheduler from sinking the ring loads towards their uses (it otherwise re-issues
  // them two k-blocks ahead and waits vmcnt(0) every block)
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int t = 0; t < NKB; ++t) {
    f4 b[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) b[rt] = bfrag(t, rt);
    // k-step c outermost: 2 RT independent accumulator chains interleaved (16x16x4 f32: 40-cycle
    // dependent latency against a 32-cycle issue); each chain's order is unchanged
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int u = 0; u < 2; ++u) acc[u][rt] = mfma16(w[t % D][u][c], b[rt][c], acc[u][rt]);
    if (t + D < NKB) {
#pragma unroll
      for (int u = 0; u < 2; ++u) w[t % D][u] = pld4(wb, wlane, 256 * (NKB * u + t + D));
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// LayerNorm + ReLU (LN net) or tanh over the 256 features of each row; 8 waves exchange row sums
template <int KIND, int RT>
PPO_DEV void act_activate(f4 (&acc)[2][RT], const float* sp_g, const float* sp_b, float* red, int wave, int j, int g) {
  constexpr int R = 16 * RT;
  if constexpr (KIND == PPO_NET_LN_BETA) {
    float mu[RT], rs[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      float s = (acc[0][rt].x + acc[0][rt].y) + (acc[0][rt].z + acc[0][rt].w) +
                ((acc[1][rt].x + acc[1][rt].y) + (acc[1][rt].z + acc[1][rt].w));
      s = row_allreduce(s);
      if (g == 0) red[wave * R + 16 * rt + j] = s;
    }
    lds_barrier();
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < kActWaves; ++w) t += red[w * R + 16 * rt + j];
      mu[rt] = t * (1.0f / 256);
      // explicit FMAs: `q += d * d` leaves the contraction to the compiler, which fused some
      // terms and not others (a different choice per kernel breaks the bitwise contract with
      // k_rollout_v's statistics lanes)
      float q = 0.f;
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = acc[u][rt][r] - mu[rt];
          q = __fmaf_rn(d, d, q);
        }
      q = row_allreduce(q);
      if (g == 0) red[(kActWaves + wave) * R + 16 * rt + j] = q;
    }
    lds_barrier();
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < kActWaves; ++w) v += red[(kActWaves + w) * R + 16 * rt + j];
      rs[rt] = 1.0f / sqrtf(__fmaf_rn(v, 1.0f / 256, 1e-5f));
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int f = 32 * wave + 16 * u + 4 * g;
      const f4 gm = *reinterpret_cast<const f4*>(sp_g + f), bt = *reinterpret_cast<const f4*>(sp_b + f);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float y = __fmaf_rn(gm[r], (acc[u][rt][r] - mu[rt]) * rs[rt], bt[r]);
          acc[u][rt][r] = y > 0.0f ? y : 0.0f;
        }
    }
  } else {
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[u][rt][r] = tanhf(acc[u][rt][r]);
  }
}

PPO_DEV float bld1f(PBuf b, int off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(b.r, off * 4, 0, 0));
}

PPO_DEV int act_head_row(const PackedLayout& K, int trunk, int h) {
  if (trunk == 0) return h == 0 ? K.cW3 : -1;
  if (K.kind == PPO_NET_LN_BETA) {
    if (h < K.A) return K.aW3 + h * K.H;
    if (h < 2 * K.A) return K.bW3 + (h - K.A) * K.H;
    return -1;
  }
  return h < K.A ? K.aW3 + h * K.H : -1;
}
PPO_DEV int act_head_bias(const PackedLayout& K, int trunk, int h) {
  if (trunk == 0) return h == 0 ? K.cb3 : -1;
  if (K.kind == PPO_NET_LN_BETA) {
    if (h < K.A) return K.ab3 + h;
    if (h < 2 * K.A) return K.bb3 + (h - K.A);
    return -1;
  }
  return h < K.A ? K.ab3 + h : -1;
}


// act_layer with the A operands already in registers (weight-resident kernels): the same MFMA
// chain in the same order as act_layer, so the results are bitwise equal.
template <int NKB, int RT, typename BF>
PPO_DEV void act_layer_regs(f4 (&acc)[2][RT], const f4 (&w)[NKB][2], BF bfrag) {
#pragma unroll
  for (int t = 0; t < NKB; ++t) {
    f4 b[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) b[rt] = bfrag(t, rt);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int u = 0; u < 2; ++u) acc[u][rt] = mfma16(w[t][u][c], b[rt][c], acc[u][rt]);
  }
}

}  // namespace act
