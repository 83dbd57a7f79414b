// ppo_agent.hpp — the agent (actor + critic trunks) in the batch-on-lanes MFMA layout.
//
// Layout recap (ppo_device.hpp): a wave owns 16 batch rows; lane = (j = row, g = lane >> 4);
// a width-H activation is NT = H/16 f4 registers per lane: register t holds features
// 16t + 4g + {0,1,2,3}. A Linear layer Z^T = W . H^T runs as NT_OUT x NT_IN x 4 MFMAs
// v_mfma_f32_16x16x4_f32: A = four consecutive input columns of a weight row (one 16-byte load
// per lane), B = the activation register itself — no LDS, no transposes between layers.
// LayerNorm over features = in-lane sum + two cross-lane adds (row_allreduce).
#pragma once

#include "ppo_device.hpp"
#include "ppo_packed.hpp"

// Buffer-resource loads (T8): a wave-uniform 128-bit descriptor + one 32-bit per-lane offset; the
// per-(tile, out-tile) displacement goes in the scalar soffset, so an unrolled layer needs no
// 64-bit VGPR address pairs (hipcc otherwise hoists and spills hundreds of them).
struct PBuf {
  __amdgpu_buffer_rsrc_t r;
};
PPO_DEV PBuf make_pbuf(const float* base, int nfloats) {
  return PBuf{__builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, nfloats * 4, 0x00020000)};
}
// f4 at float offset (lane_floats + uni_floats); lane part per lane, uniform part in soffset
PPO_DEV f4 pld4(PBuf b, int lane_floats, int uni_floats) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(b.r, lane_floats * 4, uni_floats * 4, 0));
}

// Z^T tile chain: out = W . in (+ bias), W row-major [NT_OUT*16][LDW].
template <int NT_OUT, int NT_IN, int LDW, bool BIAS>
PPO_DEV void mm_layer(f4 (&out)[NT_OUT], const f4 (&in)[NT_IN], const float* __restrict__ W,
                      const float* __restrict__ bias, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const PBuf wb = make_pbuf(W, NT_OUT * 16 * LDW);
  const int lo = i * LDW + 4 * g;
  if constexpr (BIAS) {
    const PBuf bb = make_pbuf(bias, NT_OUT * 16);
#pragma unroll
    for (int ot = 0; ot < NT_OUT; ++ot) out[ot] = pld4(bb, 4 * g, 16 * ot);
  } else {
#pragma unroll
    for (int ot = 0; ot < NT_OUT; ++ot) out[ot] = f4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int t = 0; t < NT_IN; ++t) {
    f4 w[NT_OUT];
#pragma unroll
    for (int ot = 0; ot < NT_OUT; ++ot) w[ot] = pld4(wb, lo, 16 * ot * LDW + 16 * t);
#pragma unroll
    for (int c = 0; c < 4; ++c)  // independent chains interleaved, each in its own order
#pragma unroll
      for (int ot = 0; ot < NT_OUT; ++ot) out[ot] = mfma16(w[ot][c], in[t][c], out[ot]);
  }
}

// Workgroup barrier that orders LDS traffic only: waits for this wave's LDS ops (lgkmcnt) and
// leaves global loads/stores in flight (a plain __syncthreads() may also drain vmcnt).
PPO_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Block-cooperative layer for 256-thread (4-wave) workgroups whose waves all need the same W:
// W is streamed k-tile by k-tile (16 input columns x NT_OUT*16 rows) through a double-buffered
// LDS slab, register-staged one tile ahead (load t+2 after the barrier, write it after computing t),
// so every weight byte leaves L2 once per workgroup instead of once per wave.
// wlds: 2 * NT_OUT * 256 floats. Every thread of the block must call it (uniform control flow).
template <int NT_OUT, int NT_IN, int LDW, bool BIAS>
PPO_DEV void mm_layer_lds(f4 (&out)[NT_OUT], const f4 (&in)[NT_IN], const float* __restrict__ W,
                          const float* __restrict__ bias, float* wlds, int lane, int tid) {
  constexpr int ROWS = NT_OUT * 16;
  constexpr int SLAB = ROWS * 16;
  constexpr int F4PT = (SLAB / 4 + 255) / 256;
  const PBuf wb = make_pbuf(W, ROWS * LDW);
  const int i = lane & 15, g = lane >> 4;
  f4 st[F4PT];
  auto load = [&](int t) {
#pragma unroll
    for (int u = 0; u < F4PT; ++u) {
      const int c = tid + 256 * u;
      st[u] = (c < SLAB / 4) ? pld4(wb, (c >> 2) * LDW + 4 * (c & 3), 16 * t) : f4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int u = 0; u < F4PT; ++u) {
      const int c = tid + 256 * u;
      if (c < SLAB / 4) *reinterpret_cast<f4*>(wlds + buf * SLAB + 4 * c) = st[u];
    }
  };
  if constexpr (BIAS) {
    const PBuf bb = make_pbuf(bias, ROWS);
#pragma unroll
    for (int ot = 0; ot < NT_OUT; ++ot) out[ot] = pld4(bb, 4 * g, 16 * ot);
  } else {
#pragma unroll
    for (int ot = 0; ot < NT_OUT; ++ot) out[ot] = f4{0.f, 0.f, 0.f, 0.f};
  }
  load(0);
  store(0);
  lds_barrier();
  if constexpr (NT_IN > 1) load(1);
#pragma unroll
  for (int t = 0; t < NT_IN; ++t) {
    const float* sb = wlds + (t & 1) * SLAB + i * 16 + 4 * g;
    f4 w[NT_OUT];
#pragma unroll
    for (int ot = 0; ot < NT_OUT; ++ot) w[ot] = *reinterpret_cast<const f4*>(sb + ot * 256);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int ot = 0; ot < NT_OUT; ++ot) out[ot] = mfma16(w[ot][c], in[t][c], out[ot]);
    if (t + 1 < NT_IN) store((t + 1) & 1);
    lds_barrier();
    if (t + 2 < NT_IN) load(t + 2);
  }
}

// normalized agent input (AC: (x - mean_) / std_, ac:189 / :215), zero padded to NTO*16 features
template <int NTO, int KIND>
PPO_DEV void load_input(f4 (&xin)[NTO], const float* __restrict__ xrow, int O, const float* __restrict__ omean,
                        const float* __restrict__ ostd, int g) {
#pragma unroll
  for (int t = 0; t < NTO; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 16 * t + 4 * g + r;
      float v = 0.0f;
      if (xrow && f < O) {
        v = xrow[f];
        if constexpr (KIND == PPO_NET_LN_BETA) v = (v - omean[f]) / ostd[f];
      }
      xin[t][r] = v;
    }
  }
}

template <int NT>
PPO_DEV void ln_stats(const f4 (&z)[NT], float& mu, float& rs) {
  constexpr float invH = 1.0f / (16 * NT);
  float s = 0.0f;
#pragma unroll
  for (int t = 0; t < NT; ++t) s += (z[t].x + z[t].y) + (z[t].z + z[t].w);
  s = row_allreduce(s);
  mu = s * invH;
  float q = 0.0f;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float d = z[t][r] - mu;
      q += d * d;
    }
  }
  q = row_allreduce(q);
  rs = 1.0f / sqrtf(q * invH + 1e-5f);
}

// in place: z -> x_hat = (z - mu) * rs
template <int NT>
PPO_DEV void ln_normalize(f4 (&z)[NT], float mu, float rs) {
#pragma unroll
  for (int t = 0; t < NT; ++t) z[t] = (z[t] - mu) * rs;
}

// h = relu(gamma * x_hat + beta)
template <int NT>
PPO_DEV void affine_relu(f4 (&h)[NT], const f4 (&xh)[NT], PBuf pb, int gam, int bet, int g) {
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const f4 gm = pld4(pb, 4 * g, gam + 16 * t), bt = pld4(pb, 4 * g, bet + 16 * t);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float y = __fmaf_rn(gm[r], xh[t][r], bt[r]);
      h[t][r] = y > 0.0f ? y : 0.0f;
    }
  }
}

template <int NT>
PPO_DEV void tanh_inplace(f4 (&z)[NT]) {
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) z[t][r] = tanhf(z[t][r]);
}

// one output of a Linear(H, k) head for this lane's row: sum_f w[f] h[f] + b (all 4 g-lanes get it)
template <int NT>
PPO_DEV float head_dot(const f4 (&h)[NT], PBuf pb, int w, float b, int g) {
  float p = 0.0f;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const f4 wv = pld4(pb, 4 * g, w + 16 * t);
    p += (wv.x * h[t].x + wv.y * h[t].y) + (wv.z * h[t].z + wv.w * h[t].w);
  }
  return row_allreduce(p) + b;
}

// Full trunk forward: returns the last hidden activation in h (width H). For the LN net, also
// returns the layer-1/2 statistics (needed by the fused backward).
template <int H, int KIND, int NTO>
PPO_DEV void trunk_forward(const TrunkDev& T, const float* __restrict__ P, PBuf pb, const f4 (&xin)[NTO],
                           f4 (&h)[H / 16], int lane) {
  constexpr int NT = H / 16;
  const int g = lane >> 4;
  f4 a[NT];
  mm_layer<NT, NTO, NTO * 16, true>(a, xin, P + T.W1, P + T.b1, lane);
  if constexpr (KIND == PPO_NET_LN_BETA) {
    float mu, rs;
    ln_stats<NT>(a, mu, rs);
    ln_normalize<NT>(a, mu, rs);
    affine_relu<NT>(a, a, pb, T.g1, T.be1, g);
  } else {
    tanh_inplace<NT>(a);
  }
  mm_layer<NT, NT, H, true>(h, a, P + T.W2, P + T.b2, lane);
  if constexpr (KIND == PPO_NET_LN_BETA) {
    float mu, rs;
    ln_stats<NT>(h, mu, rs);
    ln_normalize<NT>(h, mu, rs);
    affine_relu<NT>(h, h, pb, T.g2, T.be2, g);
  } else {
    tanh_inplace<NT>(h);
  }
}

// ---------------------------------------------------------------------------------------------
// Per-row distribution math. Every g-lane of a row computes the same per-row values; action
// dimensions are distributed over the 4 g-lanes (a = g, g+4, ...) and summed with row_allreduce.
// ---------------------------------------------------------------------------------------------
static constexpr float kLz = 0.91893853320467274178f;   // log(sqrt(2 pi))  (rl_utils.h:20)
static constexpr float kEntC = 1.4189385332046727418f;  // 0.5 + 0.5 log(2 pi) (rl_utils.h:44)
