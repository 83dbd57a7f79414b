// ppo_kernels.hip — hand-written gfx950 kernels of the rollout -> GAE -> PPO-update hot path.
//
//   k_act        Agent::get_action_and_value / get_value + rollout stores (ppo:145-157, :387-400;
//                ac:212-249, :649-660). One wave = 16 env rows x one trunk, MFMA 16x16x4 f32.
//   k_fwdbwd     fused minibatch gather + forward + PPO loss + backward of one trunk
//                (ppo:495-538, ac:815-875); emits H1/DZ1/DZ2/Xn for the dW GEMMs and the
//                per-block "small gradient" slab (biases, LayerNorm affine, heads, logstd).
//   k_dw         dW = DZ^T . IN split-K partial GEMM (MFMA 32x32x2 f32) for the two Linear
//                weight matrices of each trunk.
//   k_colsum     deterministic slab reductions -> packed gradient
//   k_gradnorm   clip_grad_norm_ (norm of per-tensor norms, torch/nn/utils/clip_grad.h)
//   k_adam       clip scale + optim::Adam step (torch/optim/adam.cpp) + W2^T refresh
//   k_gae        GAE(lambda) (ppo:447-467) — op-for-op fp32, bit-exact with the reference formula
//   k_perm / k_adv_*  minibatch permutation and (distributed) advantage statistics (ac:830-849)
//   k_synth_*    synthetic HalfCheetah-shaped device env (bench/test env; not the hot path)
#include "ppo_agent.hpp"
#include "ppo_kernels.hpp"
#include "ppo_wrap.hpp"

#include <algorithm>
#include <cstdlib>
#include <type_traits>
// cache policy of k_dw_dma's read-once streams (the two-phase dW of wide inputs, e.g. Ant): 0 default,
// 2 non-temporal (A/B)
#ifndef PPO_DWD_AUX
#define PPO_DWD_AUX 0
#endif

// =============================================================================================
// k_act
// =============================================================================================
template <int H, int KIND, int NTO>
__global__ __launch_bounds__(64) void k_act(ActArgs a) {
  constexpr int NT = H / 16;
  const int lane = threadIdx.x, j = lane & 15, g = lane >> 4;
  const int trunk = blockIdx.y;
  const int row = blockIdx.x * 16 + j;
  const bool valid = row < a.n;
  const PackedLayout& K = a.K;
  const float* __restrict__ P = a.P;
  const float* xrow = valid ? a.x + (size_t)row * a.ldx : nullptr;
  const long env = a.env_base + row;
  const long srow = (long)a.store_step * a.E + env;  // storage row when storing

  f4 xin[NTO];
  load_input<NTO, KIND>(xin, xrow, K.O, P + (K.omean >= 0 ? K.omean : 0), P + (K.ostd >= 0 ? K.ostd : 0), g);
  const PBuf pbuf = make_pbuf(P, K.size);
  f4 h[NT];
  trunk_forward<H, KIND, NTO>(K.tr[trunk], P, pbuf, xin, h, lane);

  if (trunk == 0) {
    const float v = head_dot<NT>(h, pbuf, K.cW3, P[K.cb3], g);
    if (valid && g == 0) {
      if (a.value_out) a.value_out[row] = v;
      if (a.store_step >= 0) {
        a.s_values[srow] = v;
        a.s_dones[srow] = a.next_done ? a.next_done[row] : 0.0f;
      }
    }
    if (valid && a.store_step >= 0)
      for (int f = g; f < K.O; f += 4) a.s_obs[srow * K.O + f] = xrow[f];
    return;
  }
  if (!a.need_actor) return;

  const int A = K.A;
  const SampleKey key = sample_key(a.seed, a.rank);
  float lp = 0.0f, ent = 0.0f;
  if constexpr (KIND == PPO_NET_TANH_NORMAL) {
    for (int ai = 0; ai < A; ++ai) {
      const float mu = head_dot<NT>(h, pbuf, K.aW3 + ai * H, P[K.ab3 + ai], g);
      if ((ai & 3) == g) {
        const float sd = expf(P[K.logstd + ai]);
        const float var = sd * sd, lsd = logf(sd);
        float act;
        if (a.mode == PPO_GIVEN) {
          act = valid ? a.action_in[(size_t)row * A + ai] : 0.0f;
        } else if (a.mode == PPO_MEAN) {
          act = mu;
        } else {
          uint32_t rr[4];
          philox_draw(key, env, a.step_id, (uint32_t)(ai >> 1), rr);
          float z0, z1;
          box_muller(rr[0], rr[1], z0, z1);
          act = mu + ((ai & 1) ? z1 : z0) * sd;
        }
        const float d = act - mu;
        lp += -(d * d) / (2.0f * var) - lsd - kLz;
        ent += kEntC + lsd;
        if (valid) {
          if (a.action_out) a.action_out[(size_t)row * A + ai] = act;
          if (a.store_step >= 0) a.s_actions[srow * A + ai] = act;
        }
      }
    }
  } else {
    const float hi = P[K.hi], lo = P[K.lo];
    for (int ai = 0; ai < A; ++ai) {
      const float pa = head_dot<NT>(h, pbuf, K.aW3 + ai * H, P[K.ab3 + ai], g);
      const float pb = head_dot<NT>(h, pbuf, K.bW3 + ai * H, P[K.bb3 + ai], g);
      if ((ai & 3) == g) {
        const float al = softplusf_(pa) + 1.0f, be = softplusf_(pb) + 1.0f;
        float s;
        if (a.mode == PPO_GIVEN) {
          const float av = valid ? a.action_in[(size_t)row * A + ai] : 0.5f * (hi + lo);
          s = (av - lo) / (hi - lo) * (1.0f - 0.0f) + 0.0f;
          s = fminf(fmaxf(s, 1e-7f), 1.0f + 1e-7f);
        } else if (a.mode == PPO_MEAN) {
          s = al / (al + be);
        } else {
          const float ga = gamma_mt(al, key, env, a.step_id, 0x10000u + (uint32_t)(ai * 2 + 0) * 64u);
          const float gb = gamma_mt(be, key, env, a.step_id, 0x10000u + (uint32_t)(ai * 2 + 1) * 64u);
          s = ga / (ga + gb);
        }
        const float ab = al + be;
        const float lga = lgammaf(al), lgb = lgammaf(be), lgab = lgammaf(ab);
        lp += xlogyf_(al - 1.0f, s) + xlogyf_(be - 1.0f, 1.0f - s) + (lgab - (lga + lgb));
        ent += (lga + lgb) - lgab - (2.0f - ab) * digammaf_(ab) -
               ((al - 1.0f) * digammaf_(al) + (be - 1.0f) * digammaf_(be));
        const float act = (s - 0.0f) / (1.0f - 0.0f) * (hi - lo) + lo;
        if (valid) {
          if (a.action_out) a.action_out[(size_t)row * A + ai] = act;
          if (a.store_step >= 0) a.s_actions[srow * A + ai] = act;
        }
      }
    }
  }
  lp = row_allreduce(lp);
  ent = row_allreduce(ent);
  if (valid && g == 0) {
    if (a.logprob_out) a.logprob_out[row] = lp;
    if (a.entropy_out) a.entropy_out[row] = ent;
    if (a.store_step >= 0) a.s_logp[srow] = lp;
  }
}

// =============================================================================================
// k_act2 — the same agent forward as k_act, block-cooperative: a 256-thread workgroup owns
// ROWS = 16*RG env rows of one trunk and its 4 waves SPLIT THE OUTPUT FEATURES (wave w computes
// feature tiles [w*NT/4, (w+1)*NT/4) of every layer), so a rollout step of 4096 envs runs on
// 2 x 4096/ROWS workgroups with 4x less serial MFMA work per wave than k_act. Activations are
// exchanged through LDS (one [ROWS][H] buffer); LayerNorm row moments are reduced over the four
// waves through LDS; head outputs are reduced per row; the per-(row, action-dim) distribution math
// runs one item per thread. Every weight byte is read once per workgroup.
// =============================================================================================
template <int H, int KIND, int NTO, int RG>
__global__ __launch_bounds__(256) void k_act2(ActArgs a) {
  constexpr int NT = H / 16, NTW = NT / 4;
  constexpr int ROWS = 16 * RG;
  constexpr int MAXNH = 40;
  constexpr int LDH = H + 4;  // row stride = 4 mod 64 banks: conflict-free ds_read_b128 B operands
  __shared__ __attribute__((aligned(16))) float hbuf[ROWS * LDH];
  __shared__ float red[4][ROWS];
  __shared__ float headp[4][ROWS][MAXNH + 1];
  __shared__ float itm[ROWS][MAXNH / 2 + 1][2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  const int trunk = blockIdx.y;
  const PackedLayout& K = a.K;
  const TrunkDev& T = K.tr[trunk];
  const float* __restrict__ P = a.P;
  const PBuf pbuf = make_pbuf(P, K.size);
  const int row0 = blockIdx.x * ROWS;
  const int O = K.O, A = K.A;
  const int nh = trunk == 0 ? 1 : (KIND == PPO_NET_LN_BETA ? 2 * A : A);
  if (trunk == 1 && !a.need_actor) return;

  // ---- inputs (every wave loads its rows' inputs; batch-on-lanes layout) ----
  f4 xin[RG][NTO];
#pragma unroll
  for (int rg = 0; rg < RG; ++rg) {
    const int row = row0 + 16 * rg + j;
    load_input<NTO, KIND>(xin[rg], row < a.n ? a.x + (size_t)row * a.ldx : nullptr, O,
                          P + (K.omean >= 0 ? K.omean : 0), P + (K.ostd >= 0 ? K.ostd : 0), g);
  }
  // own output tiles: [wave*NTW, (wave+1)*NTW)
  auto layer = [&](f4 (&acc)[RG][NTW], auto&& bfrag, int NTIN, const float* W, int ldw, int boff) {
    const PBuf wb = make_pbuf(W, H * ldw);
#pragma unroll
    for (int rg = 0; rg < RG; ++rg)
#pragma unroll
      for (int u = 0; u < NTW; ++u) acc[rg][u] = pld4(pbuf, 4 * g, boff + 16 * (wave * NTW + u));
    // weight k-blocks prefetched two ahead (the L2 latency is otherwise exposed every k-block)
    f4 w[3][NTW];
    auto wload = [&](f4 (&dst)[NTW], int t) {
#pragma unroll
      for (int u = 0; u < NTW; ++u) dst[u] = pld4(wb, (16 * (wave * NTW + u) + j) * ldw + 4 * g, 16 * t);
    };
    auto step = [&](const f4 (&wt)[NTW], int t) {
      f4 b[RG];
#pragma unroll
      for (int rg = 0; rg < RG; ++rg) b[rg] = bfrag(rg, t);
#pragma unroll
      for (int c = 0; c < 4; ++c)  // independent chains interleaved, each in its own order
#pragma unroll
        for (int rg = 0; rg < RG; ++rg)
#pragma unroll
          for (int u = 0; u < NTW; ++u) acc[rg][u] = mfma16(wt[u][c], b[rg][c], acc[rg][u]);
    };
    wload(w[0], 0);
    if (NTIN > 1) wload(w[1], 1);
    int t = 0;
    for (; t + 3 <= NTIN; t += 3) {
      if (t + 2 < NTIN) wload(w[2], t + 2);
      step(w[0], t);
      if (t + 3 < NTIN) wload(w[0], t + 3);
      step(w[1], t + 1);
      if (t + 4 < NTIN) wload(w[1], t + 4);
      step(w[2], t + 2);
    }
    if (t < NTIN) step(w[0], t);
    if (t + 1 < NTIN) step(w[1], t + 1);
  };
  // LayerNorm (+ReLU) or tanh over the full H features of each row, own tiles in registers
  auto activate = [&](f4 (&acc)[RG][NTW], int gam, int bet) {
    if constexpr (KIND == PPO_NET_LN_BETA) {
      float mu[RG], rs[RG];
#pragma unroll
      for (int rg = 0; rg < RG; ++rg) {
        float sm = 0.f;
#pragma unroll
        for (int u = 0; u < NTW; ++u) sm += (acc[rg][u].x + acc[rg][u].y) + (acc[rg][u].z + acc[rg][u].w);
        sm = row_allreduce(sm);
        if (g == 0) red[wave][16 * rg + j] = sm;
      }
      lds_barrier();
#pragma unroll
      for (int rg = 0; rg < RG; ++rg) {
        const int r = 16 * rg + j;
        mu[rg] = (((red[0][r] + red[1][r]) + red[2][r]) + red[3][r]) * (1.0f / H);
      }
      lds_barrier();
#pragma unroll
      for (int rg = 0; rg < RG; ++rg) {
        float q = 0.f;
#pragma unroll
        for (int u = 0; u < NTW; ++u)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float d = acc[rg][u][r] - mu[rg];
            q += d * d;
          }
        q = row_allreduce(q);
        if (g == 0) red[wave][16 * rg + j] = q;
      }
      lds_barrier();
#pragma unroll
      for (int rg = 0; rg < RG; ++rg) {
        const int r = 16 * rg + j;
        const float q = (((red[0][r] + red[1][r]) + red[2][r]) + red[3][r]) * (1.0f / H);
        rs[rg] = 1.0f / sqrtf(q + 1e-5f);
      }
#pragma unroll
      for (int rg = 0; rg < RG; ++rg)
#pragma unroll
        for (int u = 0; u < NTW; ++u) {
          const int ft = wave * NTW + u;
          const f4 gm = pld4(pbuf, 4 * g, gam + 16 * ft), bt = pld4(pbuf, 4 * g, bet + 16 * ft);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float y = __fmaf_rn(gm[r], (acc[rg][u][r] - mu[rg]) * rs[rg], bt[r]);
            acc[rg][u][r] = y > 0.0f ? y : 0.0f;
          }
        }
    } else {
#pragma unroll
      for (int rg = 0; rg < RG; ++rg)
#pragma unroll
        for (int u = 0; u < NTW; ++u)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[rg][u][r] = tanhf(acc[rg][u][r]);
    }
  };

  f4 acc[RG][NTW];
  layer(acc, [&](int rg, int t) { return xin[rg][t]; }, NTO, P + T.W1, NTO * 16, T.b1);
  activate(acc, T.g1, T.be1);
  // h1 -> LDS (row-major [ROWS][H]) for the layer-2 B operands
#pragma unroll
  for (int rg = 0; rg < RG; ++rg)
#pragma unroll
    for (int u = 0; u < NTW; ++u)
      *reinterpret_cast<f4*>(hbuf + (16 * rg + j) * LDH + 16 * (wave * NTW + u) + 4 * g) = acc[rg][u];
  lds_barrier();
  layer(acc, [&](int rg, int t) { return *reinterpret_cast<const f4*>(hbuf + (16 * rg + j) * LDH + 16 * t + 4 * g); },
        NT, P + T.W2, H, T.b2);
  activate(acc, T.g2, T.be2);
  // ---- heads: partial dots over this wave's features, reduced over waves through LDS ----
  const int hW = trunk == 0 ? K.cW3 : K.aW3;
  for (int k = 0; k < nh; ++k) {
    const int wrow = (KIND == PPO_NET_LN_BETA && trunk == 1 && k >= A) ? K.bW3 + (k - A) * H : hW + k * H;
#pragma unroll
    for (int rg = 0; rg < RG; ++rg) {
      float p = 0.f;
#pragma unroll
      for (int u = 0; u < NTW; ++u) {
        const f4 w = pld4(pbuf, 4 * g, wrow + 16 * (wave * NTW + u));
        p += (w.x * acc[rg][u].x + w.y * acc[rg][u].y) + (w.z * acc[rg][u].z + w.w * acc[rg][u].w);
      }
      p = row_allreduce(p);
      if (g == 0) headp[wave][16 * rg + j][k] = p;
    }
  }
  lds_barrier();
  auto head_out = [&](int r, int k) {
    const int bo = (trunk == 0) ? K.cb3 : ((KIND == PPO_NET_LN_BETA && k >= A) ? K.bb3 + (k - A) : K.ab3 + k);
    return (((headp[0][r][k] + headp[1][r][k]) + headp[2][r][k]) + headp[3][r][k]) + P[bo];
  };
  if (trunk == 0) {
    if (tid < ROWS) {
      const int row = row0 + tid;
      if (row < a.n) {
        const float v = head_out(tid, 0);
        const long env = a.env_base + row;
        if (a.value_out) a.value_out[row] = v;
        if (a.store_step >= 0) {
          const long srow = (long)a.store_step * a.E + env;
          a.s_values[srow] = v;
          a.s_dones[srow] = a.next_done ? a.next_done[row] : 0.0f;
        }
      }
    }
    if (a.store_step >= 0) {
      for (int idx = tid; idx < ROWS * O; idx += 256) {
        const int r = idx / O, f = idx % O, row = row0 + r;
        if (row < a.n) a.s_obs[((long)a.store_step * a.E + a.env_base + row) * O + f] = a.x[(size_t)row * a.ldx + f];
      }
    }
    return;
  }
  // ---- actor: one (row, action-dim) item per thread ----
  const SampleKey key = sample_key(a.seed, a.rank);
  for (int idx = tid; idx < ROWS * A; idx += 256) {
    const int r = idx / A, ai = idx % A, row = row0 + r;
    const long env = a.env_base + row;
    const bool valid = row < a.n;
    float lp = 0.f, ent = 0.f, act = 0.f;
    if constexpr (KIND == PPO_NET_TANH_NORMAL) {
      const float mu = head_out(r, ai);
      const float sd = expf(P[K.logstd + ai]);
      const float var = sd * sd, lsd = logf(sd);
      if (a.mode == PPO_GIVEN) {
        act = valid ? a.action_in[(size_t)row * A + ai] : 0.0f;
      } else if (a.mode == PPO_MEAN) {
        act = mu;
      } else {
        uint32_t rr[4];
        philox_draw(key, env, a.step_id, (uint32_t)(ai >> 1), rr);
        float z0, z1;
        box_muller(rr[0], rr[1], z0, z1);
        act = mu + ((ai & 1) ? z1 : z0) * sd;
      }
      const float d = act - mu;
      lp = -(d * d) / (2.0f * var) - lsd - kLz;
      ent = kEntC + lsd;
    } else {
      const float hi = P[K.hi], lo = P[K.lo];
      const float al = softplusf_(head_out(r, ai)) + 1.0f, be = softplusf_(head_out(r, A + ai)) + 1.0f;
      float sv;
      if (a.mode == PPO_GIVEN) {
        const float av = valid ? a.action_in[(size_t)row * A + ai] : 0.5f * (hi + lo);
        sv = (av - lo) / (hi - lo) * (1.0f - 0.0f) + 0.0f;
        sv = fminf(fmaxf(sv, 1e-7f), 1.0f + 1e-7f);
      } else if (a.mode == PPO_MEAN) {
        sv = al / (al + be);
      } else {
        const float ga = gamma_mt(al, key, env, a.step_id, 0x10000u + (uint32_t)(ai * 2 + 0) * 64u);
        const float gb = gamma_mt(be, key, env, a.step_id, 0x10000u + (uint32_t)(ai * 2 + 1) * 64u);
        sv = ga / (ga + gb);
      }
      const float ab = al + be;
      const float lga = lgammaf(al), lgb = lgammaf(be), lgab = lgammaf(ab);
      lp = xlogyf_(al - 1.0f, sv) + xlogyf_(be - 1.0f, 1.0f - sv) + (lgab - (lga + lgb));
      ent = (lga + lgb) - lgab - (2.0f - ab) * digammaf_(ab) -
            ((al - 1.0f) * digammaf_(al) + (be - 1.0f) * digammaf_(be));
      act = (sv - 0.0f) / (1.0f - 0.0f) * (hi - lo) + lo;
    }
    itm[r][ai][0] = lp;
    itm[r][ai][1] = ent;
    if (valid) {
      if (a.action_out) a.action_out[(size_t)row * A + ai] = act;
      if (a.store_step >= 0) a.s_actions[((long)a.store_step * a.E + env) * A + ai] = act;
    }
  }
  lds_barrier();
  if (tid < ROWS) {
    const int row = row0 + tid;
    if (row < a.n) {
      float lp = 0.f, ent = 0.f;
      for (int ai = 0; ai < A; ++ai) { lp += itm[tid][ai][0]; ent += itm[tid][ai][1]; }
      if (a.logprob_out) a.logprob_out[row] = lp;
      if (a.entropy_out) a.entropy_out[row] = ent;
      if (a.store_step >= 0) a.s_logp[(long)a.store_step * a.E + a.env_base + row] = lp;
    }
  }
}

// =============================================================================================
// k_fwdbwd — fused gather + forward + loss + backward of one trunk for 16 rows per wave
// =============================================================================================

// Butterfly reduce-scatter of a per-lane feature vector over the 16 rows of a wave (lanes with the
// same g). On return lane j holds V/16 sums: slots [(V/16) j, (V/16)(j+1)), slot s <-> feature
// 16 (s >> 2) + 4 g + (s & 3). Adds them into the wave's LDS accumulator at `acc` (feature index).
template <int NT, typename Fn>
PPO_DEV void rows_reduce_fn(Fn f, float* acc, int lane) {
  constexpr int V = 4 * NT;
  const int j = lane & 15, g = lane >> 4;
  float v[V / 2];
  {
    const bool bit = (j & 8) != 0;
#pragma unroll
    for (int i = 0; i < V / 2; ++i) {
      const float lo = f(i), hi = f(i + V / 2);
      const float keep = bit ? hi : lo, send = bit ? lo : hi;
      v[i] = keep + shfl_xor(send, 8);
    }
  }
#pragma unroll
  for (int m = 4, len = V / 2; m >= 1; m >>= 1, len >>= 1) {
    const bool bit = (j & m) != 0;
#pragma unroll
    for (int i = 0; i < len / 2; ++i) {
      const float lo = v[i], hi = v[i + len / 2];
      const float keep = bit ? hi : lo, send = bit ? lo : hi;
      v[i] = keep + shfl_xor(send, m);
    }
  }
  constexpr int PER = V / 16;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int s = PER * j + q;
    const int f2 = 16 * (s >> 2) + 4 * g + (s & 3);
    acc[f2] += v[q];
  }
}
#define SLOT(arr, s) (arr)[(s) >> 2][(s) & 3]

// per-row scalar -> sum over the 16 rows of lane group g; lane j == 0 of the group gets the sum
PPO_DEV float rows_sum16(float v) {
  v += shfl_xor(v, 1);
  v += shfl_xor(v, 2);
  v += shfl_xor(v, 4);
  v += shfl_xor(v, 8);
  return v;
}

template <int NT>
PPO_DEV void store_rows(float* __restrict__ dst, int ld, const f4 (&v)[NT], bool valid, int g) {
  if (!valid) return;
#pragma unroll
  for (int t = 0; t < NT; ++t) st4(dst + 16 * t + 4 * g, v[t]);
}

template <int H, int KIND, int NTO>
__global__ __launch_bounds__(256) void k_fwdbwd(UpdArgs a) {
  constexpr int NT = H / 16;
  constexpr int V = 4 * NT;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, j = lane & 15, g = lane >> 4;
  const int trunk = blockIdx.y;
  const PackedLayout& K = a.K;
  const TrunkDev& T = K.tr[trunk];
  const float* __restrict__ P = a.P;
  const PBuf pbuf = make_pbuf(P, K.size);
  const SmallGradLayout sg = a.sg[trunk];
  float* acc = lds + wave * sg.size;
  float* wlds = lds + a.wlds_off;  // 2 x H*16 floats: weight k-tile double buffer
  for (int i = lane; i < sg.size; i += 64) acc[i] = 0.0f;

  const int O = K.O, A = K.A, OP = K.OP;
  const float c = a.clip_coef;
  const float adv_mean = a.adv_stats[0], adv_std = a.adv_stats[1];

  for (int tile = 0; tile < a.tiles_per_block; ++tile) {
    const int m = (blockIdx.x * a.tiles_per_block + tile) * 64 + wave * 16 + j;
    const bool valid = m < a.M;
    const long b = valid ? (long)a.perm[m] : 0;
    const float* xrow = valid ? a.obs + b * O : nullptr;
    f4 xin[NTO];
    load_input<NTO, KIND>(xin, xrow, O, P + (K.omean >= 0 ? K.omean : 0), P + (K.ostd >= 0 ? K.ostd : 0), g);
    if (trunk == 0) store_rows<NTO>(a.Xn + (size_t)m * OP, OP, xin, valid, g);

    // ---------------- forward ----------------
    f4 hA[NT];   // layer-1 output; later dh1 accumulator
    f4 hC[NT];   // layer-2: x_hat2 (LN) or h2 (tanh); later dz2
    float mu1 = 0.f, rs1 = 0.f, mu2 = 0.f, rs2 = 0.f;
    mm_layer_lds<NT, NTO, NTO * 16, true>(hA, xin, P + T.W1, P + T.b1, wlds, lane, threadIdx.x);
    if constexpr (KIND == PPO_NET_LN_BETA) {
      ln_stats<NT>(hA, mu1, rs1);
      ln_normalize<NT>(hA, mu1, rs1);
      affine_relu<NT>(hA, hA, pbuf, T.g1, T.be1, g);
    } else {
      tanh_inplace<NT>(hA);
    }
    store_rows<NT>(a.H1[trunk] + (size_t)m * H, H, hA, valid, g);
    mm_layer_lds<NT, NT, H, true>(hC, hA, P + T.W2, P + T.b2, wlds, lane, threadIdx.x);
    if constexpr (KIND == PPO_NET_LN_BETA) {
      ln_stats<NT>(hC, mu2, rs2);
      ln_normalize<NT>(hC, mu2, rs2);  // hC = x_hat2
    } else {
      tanh_inplace<NT>(hC);  // hC = h2
    }
    // h2 view (recomputed from x_hat2 for the LN net)
    auto h2_tile = [&](int t) -> f4 {
      if constexpr (KIND == PPO_NET_LN_BETA) {
        const f4 gm = pld4(pbuf, 4 * g, T.g2 + 16 * t), bt = pld4(pbuf, 4 * g, T.be2 + 16 * t);
        f4 r;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float y = __fmaf_rn(gm[q], hC[t][q], bt[q]);
          r[q] = y > 0.0f ? y : 0.0f;
        }
        return r;
      } else {
        return hC[t];
      }
    };
    // f4 h2[NT] materialised once (needed by several head loops)
    f4 h2[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) h2[t] = h2_tile(t);

    // ---------------- heads + loss (per row) + head backward ----------------
    f4 dh[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) dh[t] = f4{0.f, 0.f, 0.f, 0.f};
    float st_pg = 0.f, st_v = 0.f, st_ent = 0.f, st_okl = 0.f, st_kl = 0.f, st_cf = 0.f;

    if (trunk == 0) {
      const float v = head_dot<NT>(h2, pbuf, K.cW3, P[K.cb3], g);
      const float rt = valid ? a.ret[b] : 0.f, ov = valid ? a.val[b] : 0.f;
      float gv;
      if (a.clip_vloss) {
        const float vu = (v - rt) * (v - rt);
        const float dv = v - ov;
        const float vcl = ov + fminf(fmaxf(dv, -c), c);
        const float vc = (vcl - rt) * (vcl - rt);
        st_v = fmaxf(vu, vc);
        const float w1 = vu > vc ? 1.0f : (vu == vc ? 0.5f : 0.0f);
        const float inr = (dv >= -c && dv <= c) ? 1.0f : 0.0f;
        gv = 0.5f * a.vf_coef * a.inv_m * (w1 * 2.0f * (v - rt) + (1.0f - w1) * 2.0f * (vcl - rt) * inr);
      } else {
        st_v = (v - rt) * (v - rt);
        gv = 0.5f * a.vf_coef * a.inv_m * 2.0f * (v - rt);
      }
      if (!valid) { gv = 0.f; st_v = 0.f; }
      // head weight / bias grads and dh2
#pragma unroll
      for (int t = 0; t < NT; ++t) dh[t] = pld4(pbuf, 4 * g, K.cW3 + 16 * t) * gv;
      rows_reduce_fn<NT>([&](int sI) { return gv * SLOT(h2, sI); }, acc + sg.hW, lane);
      const float gsum = rows_sum16(gv);
      if (lane == 0) acc[sg.hb] += gsum;
    } else {
      // ---- actor: pass 1 (log-prob, entropy of the stored action) ----
      float lp = 0.f, ent = 0.f;
      float own_x[5], own_p[5], own_q[5];  // per owned action dim (a = g + 4k): action / head pre-acts
#pragma unroll
      for (int k = 0; k < 5; ++k) { own_x[k] = 0.f; own_p[k] = 0.f; own_q[k] = 0.f; }
      if constexpr (KIND == PPO_NET_TANH_NORMAL) {
        for (int ai = 0; ai < A; ++ai) {
          const float mu = head_dot<NT>(h2, pbuf, K.aW3 + ai * H, P[K.ab3 + ai], g);
          if ((ai & 3) == g) {
            const float sd = expf(P[K.logstd + ai]);
            const float var = sd * sd, lsd = logf(sd);
            const float act = valid ? a.actions[b * A + ai] : mu;
            const float d = act - mu;
            lp += -(d * d) / (2.0f * var) - lsd - kLz;
            ent += kEntC + lsd;
#pragma unroll
            for (int k = 0; k < 5; ++k)
              if ((ai >> 2) == k) { own_x[k] = act; own_p[k] = mu; }
          }
        }
      } else {
        const float hi = P[K.hi], lo = P[K.lo];
        for (int ai = 0; ai < A; ++ai) {
          const float pa = head_dot<NT>(h2, pbuf, K.aW3 + ai * H, P[K.ab3 + ai], g);
          const float pb = head_dot<NT>(h2, pbuf, K.bW3 + ai * H, P[K.bb3 + ai], g);
          if ((ai & 3) == g) {
            const float al = softplusf_(pa) + 1.0f, be = softplusf_(pb) + 1.0f;
            const float av = valid ? a.actions[b * A + ai] : 0.5f * (hi + lo);
            float s = (av - lo) / (hi - lo) * (1.0f - 0.0f) + 0.0f;
            s = fminf(fmaxf(s, 1e-7f), 1.0f + 1e-7f);
            const float ab = al + be;
            const float lga = lgammaf(al), lgb = lgammaf(be), lgab = lgammaf(ab);
            lp += xlogyf_(al - 1.0f, s) + xlogyf_(be - 1.0f, 1.0f - s) + (lgab - (lga + lgb));
            ent += (lga + lgb) - lgab - (2.0f - ab) * digammaf_(ab) -
                   ((al - 1.0f) * digammaf_(al) + (be - 1.0f) * digammaf_(be));
#pragma unroll
            for (int k = 0; k < 5; ++k)
              if ((ai >> 2) == k) { own_x[k] = s; own_p[k] = pa; own_q[k] = pb; }
          }
        }
      }
      lp = row_allreduce(lp);
      ent = row_allreduce(ent);
      // ---- PPO clipped surrogate (per row) ----
      const float oldlp = valid ? a.logp[b] : lp;
      const float logratio = lp - oldlp;
      const float ratio = expf(logratio);
      st_okl = -logratio;
      st_kl = (ratio - 1.0f) - logratio;
      st_cf = fabsf(ratio - 1.0f) > c ? 1.0f : 0.0f;
      st_ent = ent;
      float an = valid ? a.adv[b] : 0.f;
      if (a.norm_adv) an = (an - adv_mean) / (adv_std + 1e-8f);
      const float rc = fminf(fmaxf(ratio, 1.0f - c), 1.0f + c);
      const float pg1 = -an * ratio, pg2 = -an * rc;
      st_pg = fmaxf(pg1, pg2);
      const float w1 = pg1 > pg2 ? 1.0f : (pg1 == pg2 ? 0.5f : 0.0f);
      const float inr = (ratio >= 1.0f - c && ratio <= 1.0f + c) ? 1.0f : 0.0f;
      float g_logp = a.inv_m * (w1 * (-an) + (1.0f - w1) * (-an) * inr) * ratio;
      float g_ent = -a.ent_coef * a.inv_m;
      if (!valid) { g_logp = 0.f; g_ent = 0.f; st_pg = st_okl = st_kl = st_cf = st_ent = 0.f; }

      // ---- pass 2: per owned action dim gradients wrt head pre-activations ----
      float own_ga[5], own_gb[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        own_ga[k] = 0.f; own_gb[k] = 0.f;
        const int ai = g + 4 * k;
        if (ai < A) {
          if constexpr (KIND == PPO_NET_TANH_NORMAL) {
            const float sd = expf(P[K.logstd + ai]);
            const float var = sd * sd;
            const float d = own_x[k] - own_p[k];
            own_ga[k] = g_logp * d / var;                                 // d loss / d mu
            own_gb[k] = g_logp * (d * d / var - 1.0f) + g_ent;            // d loss / d logstd
          } else {
            const float al = softplusf_(own_p[k]) + 1.0f, be = softplusf_(own_q[k]) + 1.0f;
            const float ab = al + be, s = own_x[k];
            const float psab = digammaf_(ab), tab = trigammaf_(ab);
            const float dla = ((al - 1.0f) != 0.0f ? logf(s) : 0.0f) + psab - digammaf_(al);
            const float dlb = ((be - 1.0f) != 0.0f ? logf(1.0f - s) : 0.0f) + psab - digammaf_(be);
            const float dea = (ab - 2.0f) * tab - (al - 1.0f) * trigammaf_(al);
            const float deb = (ab - 2.0f) * tab - (be - 1.0f) * trigammaf_(be);
            own_ga[k] = (g_logp * dla + g_ent * dea) * softplus_d(own_p[k]);
            own_gb[k] = (g_logp * dlb + g_ent * deb) * softplus_d(own_q[k]);
          }
        }
      }
      // scalar grads: head biases (and logstd) summed over the wave's rows
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const float sa = rows_sum16(own_ga[k]);
        const float sb = rows_sum16(own_gb[k]);
        const int ai = g + 4 * k;
        if (j == 0 && ai < A) {
          acc[sg.hb + ai] += sa;
          if constexpr (KIND == PPO_NET_TANH_NORMAL) acc[sg.ls + ai] += sb;
          else acc[sg.hb + A + ai] += sb;
        }
      }
      // head weight grads + dh2: every lane needs every head's per-row gradient
      const int nh = (KIND == PPO_NET_TANH_NORMAL) ? A : 2 * A;
      for (int hk = 0; hk < nh; ++hk) {
        const int ai = hk % A;
        const bool second = hk >= A;
        float mine = 0.f;
#pragma unroll
        for (int k = 0; k < 5; ++k)
          if ((ai >> 2) == k) mine = second ? own_gb[k] : own_ga[k];
        const float gk = __shfl(mine, j + 16 * (ai & 3), 64);
        const int wrow = (KIND == PPO_NET_TANH_NORMAL) ? K.aW3 + ai * H : (second ? K.bW3 + ai * H : K.aW3 + ai * H);
#pragma unroll
        for (int t = 0; t < NT; ++t) dh[t] += pld4(pbuf, 4 * g, wrow + 16 * t) * gk;
        rows_reduce_fn<NT>([&](int sI) { return gk * SLOT(h2, sI); }, acc + sg.hW + hk * H, lane);
      }
    }
    // loss statistics (one lane group per row)
    {
      const float s0 = rows_sum16(g == 0 ? st_pg : 0.f), s1 = rows_sum16(g == 0 ? st_v : 0.f);
      const float s2 = rows_sum16(g == 0 ? st_ent : 0.f), s3 = rows_sum16(g == 0 ? st_okl : 0.f);
      const float s4 = rows_sum16(g == 0 ? st_kl : 0.f), s5 = rows_sum16(g == 0 ? st_cf : 0.f);
      if (lane == 0) {
        acc[sg.stats + ST_PG] += s0; acc[sg.stats + ST_V] += s1; acc[sg.stats + ST_ENT] += s2;
        acc[sg.stats + ST_OKL] += s3; acc[sg.stats + ST_KL] += s4; acc[sg.stats + ST_CF] += s5;
      }
    }

    // ---------------- layer-2 backward: dh2 -> dz2 (in hC) ----------------
    {
      if constexpr (KIND == PPO_NET_LN_BETA) {
        // dy2 = dh2 * relu'(y2); dgamma2, dbeta2; LN backward
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const f4 gm = pld4(pbuf, 4 * g, T.g2 + 16 * t);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float dy = h2[t][q] > 0.0f ? dh[t][q] : 0.0f;  // y2 > 0 <=> relu output > 0
            dh[t][q] = dy;
            const float dx = dy * gm[q];
            s1 += dx;
            s2 += dx * hC[t][q];
          }
        }
        s1 = row_allreduce(s1) * (1.0f / H);
        s2 = row_allreduce(s2) * (1.0f / H);
        rows_reduce_fn<NT>([&](int sI) { return SLOT(dh, sI); }, acc + sg.be2, lane);
        rows_reduce_fn<NT>([&](int sI) { return SLOT(dh, sI) * SLOT(hC, sI); }, acc + sg.g2, lane);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const f4 gm = pld4(pbuf, 4 * g, T.g2 + 16 * t);
          hC[t] = rs2 * (dh[t] * gm - s1 - hC[t] * s2);
        }
      } else {
#pragma unroll
        for (int t = 0; t < NT; ++t) hC[t] = dh[t] * (1.0f - hC[t] * hC[t]);
      }
      rows_reduce_fn<NT>([&](int sI) { return SLOT(hC, sI); }, acc + sg.b2, lane);
      store_rows<NT>(a.DZ2[trunk] + (size_t)m * H, H, hC, valid, g);
    }
    // ---------------- dh1 = W2^T dz2 ----------------
    mm_layer_lds<NT, NT, H, false>(dh, hC, a.W2T[trunk], nullptr, wlds, lane, threadIdx.x);
    // ---------------- recompute layer 1, layer-1 backward ----------------
    mm_layer_lds<NT, NTO, NTO * 16, true>(hA, xin, P + T.W1, P + T.b1, wlds, lane, threadIdx.x);
    {
      if constexpr (KIND == PPO_NET_LN_BETA) {
        ln_normalize<NT>(hA, mu1, rs1);  // x_hat1 (bit-identical recompute)
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const f4 gm = pld4(pbuf, 4 * g, T.g1 + 16 * t), bt = pld4(pbuf, 4 * g, T.be1 + 16 * t);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float y = __fmaf_rn(gm[q], hA[t][q], bt[q]);
            const float dy = y > 0.0f ? dh[t][q] : 0.0f;
            dh[t][q] = dy;
            const float dx = dy * gm[q];
            s1 += dx;
            s2 += dx * hA[t][q];
          }
        }
        s1 = row_allreduce(s1) * (1.0f / H);
        s2 = row_allreduce(s2) * (1.0f / H);
        rows_reduce_fn<NT>([&](int sI) { return SLOT(dh, sI); }, acc + sg.be1, lane);
        rows_reduce_fn<NT>([&](int sI) { return SLOT(dh, sI) * SLOT(hA, sI); }, acc + sg.g1, lane);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const f4 gm = pld4(pbuf, 4 * g, T.g1 + 16 * t);
          hA[t] = rs1 * (dh[t] * gm - s1 - hA[t] * s2);
        }
      } else {
        tanh_inplace<NT>(hA);
#pragma unroll
        for (int t = 0; t < NT; ++t) hA[t] = dh[t] * (1.0f - hA[t] * hA[t]);
      }
      rows_reduce_fn<NT>([&](int sI) { return SLOT(hA, sI); }, acc + sg.b1, lane);
      store_rows<NT>(a.DZ1[trunk] + (size_t)m * H, H, hA, valid, g);
    }
  }
  // ---------------- block reduction of the 4 wave accumulators (fixed order) ----------------
  __syncthreads();
  float* out = a.slab[trunk] + (size_t)blockIdx.x * sg.size;
  for (int i = threadIdx.x; i < sg.size; i += blockDim.x)
    out[i] = ((lds[i] + lds[sg.size + i]) + lds[2 * sg.size + i]) + lds[3 * sg.size + i];
}

// =============================================================================================
// k_dw — split-K weight gradients of one trunk for one chunk of minibatch rows:
//   phase 2: dW2[o][i] = sum_m DZ2[m][o] * H1[m][i]     (H x H)
//   phase 1: dW1[o][i] = sum_m DZ1[m][o] * Xn[m][i]     (H x OP)
// 4 waves; MFMA 32x32x2 f32; rows staged 16 at a time through a double-buffered LDS tile
// (register-staged, one sub-chunk ahead); wave (wo, wi) owns o-tiles [wo*TOW, ..) x i-tiles
// [wi*TIW, ..). Partial sums go to a per-chunk slab (deterministic reduction in k_colsum).
// =============================================================================================
typedef float f16v __attribute__((ext_vector_type(16)));

template <int NO, int NI, int LDI, int WO, int WI, int NTH>
PPO_DEV void dw_phase(const float* __restrict__ DZ, const float* __restrict__ IN, long m0, long m1,
                      float* __restrict__ out, float* lds, int tid, const int32_t* __restrict__ perm = nullptr,
                      int O = 0) {
  constexpr int TO = NO / 32, TI = (NI + 31) / 32;
  constexpr int TOW = TO / WO, TIW = (TI + WI - 1) / WI;
  constexpr int KS = 16;                       // rows per stage
  constexpr int LDZ = NO + 4, LDN = LDI + 4;   // padded LDS rows (the two half-waves read rows k, k+1)
  constexpr int ADZ = KS * LDZ, AIN = KS * LDN; // floats per stage
  constexpr int STG = ADZ + AIN;
  constexpr int NF4Z = KS * NO / 4, NF4 = NF4Z + KS * LDI / 4;
  constexpr int F4PT = (NF4 + NTH - 1) / NTH;
  const int lane = tid & 63, wave = tid >> 6;
  const int wo = wave % WO, wi = wave / WO;
  const int l32 = lane & 31, hs = lane >> 5;
  f16v acc[TOW][TIW];
#pragma unroll
  for (int u = 0; u < TOW; ++u)
#pragma unroll
    for (int v = 0; v < TIW; ++v)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[u][v][r] = 0.0f;
  f4 st[F4PT];
  auto load = [&](long mb) {
#pragma unroll
    for (int u = 0; u < F4PT; ++u) {
      const int c = tid + NTH * u;
      f4 v = f4{0.f, 0.f, 0.f, 0.f};
      if (c < NF4Z) {
        const long row = mb + (4 * c) / NO;
        if (row < m1) v = ld4(DZ + row * NO + (4 * c) % NO);
      } else if (c < NF4) {
        const int f2 = 4 * (c - NF4Z);
        const long row = mb + f2 / LDI;
        if (row < m1) {
          if (perm) {  // IN = obs rows [.][O] through the permutation, zero padded to LDI
            const int col = f2 % LDI;
            const float* src = IN + (long)perm[row] * O + col;
            if ((O & 3) == 0) {
              if (col < O) v = ld4(src);
            } else {
#pragma unroll
              for (int q = 0; q < 4; ++q) v[q] = col + q < O ? src[q] : 0.f;
            }
          } else {
            v = ld4(IN + row * LDI + f2 % LDI);
          }
        }
      }
      st[u] = v;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int u = 0; u < F4PT; ++u) {
      const int c = tid + NTH * u;
      if (c < NF4Z) {
        const int fl = 4 * c;
        *reinterpret_cast<f4*>(lds + buf * STG + (fl / NO) * LDZ + fl % NO) = st[u];
      } else if (c < NF4) {
        const int f2 = 4 * (c - NF4Z);
        *reinterpret_cast<f4*>(lds + buf * STG + ADZ + (f2 / LDI) * LDN + f2 % LDI) = st[u];
      }
    }
  };
  const int nst = (int)((m1 - m0 + KS - 1) / KS);
  load(m0);
  store(0);
  lds_barrier();
  if (nst > 1) load(m0 + KS);
  for (int sI = 0; sI < nst; ++sI) {
    const float* sdz = lds + (sI & 1) * STG;
    const float* sin = sdz + ADZ;
#pragma unroll
    for (int k = 0; k < KS; k += 2) {
      float av[TOW], bv[TIW];
#pragma unroll
      for (int u = 0; u < TOW; ++u) av[u] = sdz[(k + hs) * LDZ + (wo * TOW + u) * 32 + l32];
#pragma unroll
      for (int v = 0; v < TIW; ++v) {
        const int col = (wi * TIW + v) * 32 + l32;
        bv[v] = (col < LDI) ? sin[(k + hs) * LDN + col] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < TOW; ++u)
#pragma unroll
        for (int v = 0; v < TIW; ++v) acc[u][v] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[v], acc[u][v], 0, 0, 0);
    }
    if (sI + 1 < nst) store((sI + 1) & 1);
    lds_barrier();
    if (sI + 2 < nst) load(m0 + (long)(sI + 2) * KS);
    __builtin_amdgcn_sched_barrier(0);  // keep the next-next stage's loads issued here
  }
#pragma unroll
  for (int u = 0; u < TOW; ++u)
#pragma unroll
    for (int v = 0; v < TIW; ++v)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = (wo * TOW + u) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hs;
        const int i = (wi * TIW + v) * 32 + l32;
        if (i < LDI) out[(size_t)o * LDI + i] = acc[u][v][r];
      }
}

// s_waitcnt vmcnt(n) for a wave-uniform n in [0, 7]
PPO_DEV void wait_vmcnt_upto7(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
  }
}

// dw_phase with the stage rows moved by LDS DMA (16 bytes a lane, one 1 KB wave instruction per
// 256 floats; rows contiguous in HBM, IN rows of LDI floats, no permutation) into three unpadded
// stage buffers two stages ahead — k_dwf_dma's pipeline for the two-phase k_dw (wide inputs: Ant's
// OP = 112). Same operands and MFMA order as dw_phase: bitwise. NP > 0 (dw_mfma=bf16x6 / x8 / x9):
// a 16-row stage is one v_mfma_f32_32x32x16_bf16 k block of NP split-bf16 piece products (k_dwf_bx's
// scheme; each lane splits its column of rows 8 hs .. 8 hs + 7 as read).
template <int NO, int NI, int LDI, int WO, int WI, int NP = 0>
PPO_DEV void dw_phase_dma(const float* __restrict__ DZ, const float* __restrict__ IN, long M, long m0, long m1,
                          float* __restrict__ out, float* lds, int tid) {
  constexpr int TO = NO / 32, TI = (NI + 31) / 32;
  constexpr int TOW = TO / WO, TIW = (TI + WI - 1) / WI;
  constexpr bool FULL = TI * 32 == LDI && WI * TIW == TI;  // every input column tile is real: no masking
  constexpr int KS = 16, NBUF = 3;
  constexpr int ADZ = KS * NO, STG = ADZ + KS * LDI;
  constexpr int ND = KS * NO / 256, NIN = KS * LDI / 256, NT = ND + NIN;  // DMA instructions per stage
  static_assert(KS * NO % 256 == 0 && KS * LDI % 256 == 0, "dw_phase_dma: whole 1 KB instructions");
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wo = wave % WO, wi = wave / WO;
  const int l32 = lane & 31, hs = lane >> 5;
  const PBuf bdz = make_pbuf(DZ, (int)(M * NO)), bin = make_pbuf(IN, (int)(M * LDI));
  f16v acc[TOW][TIW];
#pragma unroll
  for (int u = 0; u < TOW; ++u)
#pragma unroll
    for (int v = 0; v < TIW; ++v)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[u][v][r] = 0.0f;
  // wave w moves instructions w, w + 8, ... of a stage: [0, ND) DZ rows, [ND, NT) IN floats
  const int nmine = (NT - wave + 7) / 8;
  auto issue = [&](long mb, int buf) {
    float* b = lds + buf * STG;
#pragma unroll
    for (int q = 0; q < (NT + 7) / 8; ++q) {
      const int i = wave + 8 * q;
      if (i < ND) {
        const long row = mb + i / (NO / 256);
        const uint32_t voff = row < m1 ? (uint32_t)(((long)i * 256 + mb * NO) * 4 + lane * 16) : 0xFFFFFFF0u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(bdz.r, (__attribute__((address_space(3))) void*)(b + i * 256), 16,
                                                 voff, 0, 0, PPO_DWD_AUX);
      } else if (i < NT) {
        const int e = (i - ND) * 256 + lane * 4;  // float of the stage's IN block
        const long row = mb + e / LDI;
        const uint32_t voff = row < m1 ? (uint32_t)((mb * LDI + e) * 4) : 0xFFFFFFF0u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(bin.r, (__attribute__((address_space(3))) void*)(b + ADZ + (i - ND) * 256),
                                                 16, voff, 0, 0, PPO_DWD_AUX);
      }
    }
  };
  const int nst = (int)((m1 - m0 + KS - 1) / KS);
  issue(m0, 0);
  if (nst > 1) issue(m0 + KS, 1);
  for (int sI = 0; sI < nst; ++sI) {
    wait_vmcnt_upto7(sI + 1 < nst ? nmine : 0);  // stage sI landed; sI + 1 may stay in flight
    lds_barrier();
    if (sI + 2 < nst) issue(m0 + (long)(sI + 2) * KS, (sI + 2) % NBUF);
    __builtin_amdgcn_sched_barrier(0);
    const float* sdz = lds + (sI % NBUF) * STG;
    const float* sin = sdz + ADZ;
    if constexpr (NP > 0) {
      Split3 as[TOW];
#pragma unroll
      for (int u = 0; u < TOW; ++u) {
        float v8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v8[e] = sdz[(8 * hs + e) * NO + (wo * TOW + u) * 32 + l32];
        as[u] = split3(v8);
      }
#pragma unroll
      for (int v = 0; v < TIW; ++v) {
        const int col = (wi * TIW + v) * 32 + l32;
        float w8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e)
          w8[e] = (FULL || col < LDI) ? sin[(8 * hs + e) * LDI + (FULL ? col : min(col, LDI - 1))] : 0.0f;
        const Split3 bs = split3(w8);
#pragma unroll
        for (int u = 0; u < TOW; ++u) acc[u][v] = mfma_split<NP>(as[u], bs, acc[u][v]);
      }
      continue;
    }
#pragma unroll
    for (int k = 0; k < KS; k += 2) {
      float av[TOW], bv[TIW];
#pragma unroll
      for (int u = 0; u < TOW; ++u) av[u] = sdz[(k + hs) * NO + (wo * TOW + u) * 32 + l32];
#pragma unroll
      for (int v = 0; v < TIW; ++v) {
        const int col = (wi * TIW + v) * 32 + l32;
        bv[v] = (FULL || col < LDI) ? sin[(k + hs) * LDI + col] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < TOW; ++u)
#pragma unroll
        for (int v = 0; v < TIW; ++v) acc[u][v] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[v], acc[u][v], 0, 0, 0);
    }
  }
  lds_barrier();  // the buffers are free for the next phase
#pragma unroll
  for (int u = 0; u < TOW; ++u)
#pragma unroll
    for (int v = 0; v < TIW; ++v)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = (wo * TOW + u) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hs;
        const int i = (wi * TIW + v) * 32 + l32;
        if (FULL || i < LDI) out[(size_t)o * LDI + i] = acc[u][v][r];
      }
}

template <int H, int OP, int NP = 0>
__global__ __launch_bounds__(512) void k_dw_dma(DwArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int TO = H / 32;
  constexpr int WO2 = TO >= 4 ? 4 : TO, WI2 = 8 / WO2;
  constexpr int WO1 = TO >= 8 ? 8 : TO, WI1 = 8 / WO1;
  const int trunk = blockIdx.y;
  const long m0 = (long)blockIdx.x * a.rows_per_chunk;
  const long m1 = min((long)a.M, m0 + a.rows_per_chunk);
  float* out = a.slab[trunk] + (size_t)blockIdx.x * a.slab_stride;
  if (m0 < m1) {
    dw_phase_dma<H, H, H, WO2, WI2, NP>(a.dz2[trunk], a.h1[trunk], a.M, m0, m1, out, lds, threadIdx.x);
    dw_phase_dma<H, OP, OP, WO1, WI1, NP>(a.dz1[trunk], a.xn, a.M, m0, m1, out + H * H, lds, threadIdx.x);
  }
}

// 8 waves (two per SIMD): dW2 as a 4 x 2 grid of 64 x 128 wave tiles (128 accumulator registers
// per wave), then dW1 (H x OP) with the waves split over the output rows.
template <int H, int OP>
__global__ __launch_bounds__(512) void k_dw(DwArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int TO = H / 32;
  constexpr int WO2 = TO >= 4 ? 4 : TO, WI2 = 8 / WO2;
  constexpr int WO1 = TO >= 8 ? 8 : TO, WI1 = 8 / WO1;
  const int trunk = blockIdx.y;
  const long m0 = (long)blockIdx.x * a.rows_per_chunk;
  const long m1 = min((long)a.M, m0 + a.rows_per_chunk);
  float* out = a.slab[trunk] + (size_t)blockIdx.x * a.slab_stride;
  if (m0 < m1) {
    dw_phase<H, H, H, WO2, WI2, 512>(a.dz2[trunk], a.h1[trunk], m0, m1, out, lds, threadIdx.x);
    lds_barrier();
    if (a.perm)
      dw_phase<H, OP, OP, WO1, WI1, 512>(a.dz1[trunk], a.obs, m0, m1, out + H * H, lds, threadIdx.x, a.perm, a.O);
    else
      dw_phase<H, OP, OP, WO1, WI1, 512>(a.dz1[trunk], a.xn, m0, m1, out + H * H, lds, threadIdx.x);
  }
}

// k_dwf — the same two products of one trunk in ONE pass over the chunk's rows (H = 256, OP <= 32).
// Every 16-row stage carries DZ2, H1, DZ1 and Xn rows, so the memory-bound dW1 product (K = OP,
// one 32x32 MFMA per wave and row pair) rides under the MFMA-bound dW2 product (eight per wave)
// instead of running as a second, load-bound phase. 8 waves: dW2 as a 4 x 2 grid of 64 x 128
// wave tiles, dW1 as one 32-row o-tile per wave. Slab layout as k_dw.
template <int H, int OP, int NSL>
__global__ __launch_bounds__(512) void k_dwf(DwArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int KS = 16, NTH = 512;
  constexpr int LDH = H + 4, LDX = OP + 4;
  constexpr int oH1 = KS * LDH, oDZ1 = 2 * KS * LDH, oXN = 3 * KS * LDH;
  constexpr int STG = 3 * KS * LDH + KS * LDX;
  constexpr int N2 = KS * H / 4, NX = KS * OP / 4;  // f4 per stage of a width-H / width-OP source
  static_assert(H == 256 && OP <= 32 && N2 % NTH == 0, "k_dwf geometry");
  constexpr int PW = N2 / NTH;                      // f4 per thread per width-H source
  constexpr int NXT = (NX + NTH - 1) / NTH;
  // dW2 wave tile: TOW x 4 32x32 tiles; with NSL output slices a workgroup owns dW2^T rows
  // [s H / NSL, (s + 1) H / NSL) and dW1^T's rows in that range (its waves 0 .. 8 / NSL - 1)
  constexpr int TOW = 2 / NSL, TIW = 4;
  static_assert(NSL == 1 || NSL == 2, "k_dwf slices");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, hs = lane >> 5;
  const int wo = wave & 3, wi = wave >> 2;
  const int trunk = blockIdx.y, slice = NSL > 1 ? (int)blockIdx.z : 0;
  const int obase = slice * (H / NSL);                       // first dW2^T / dW1^T row of the slice
  const bool w1_wave = NSL == 1 || wave < 8 / NSL;          // this wave owns a dW1^T row tile
  const int w1row = obase + wave * 32;                       // its first row
  const long m0 = (long)blockIdx.x * a.rows_per_chunk;
  const long m1 = min((long)a.M, m0 + a.rows_per_chunk);
  if (m0 >= m1) return;
  const float* __restrict__ src3[3] = {a.dz2[trunk], a.h1[trunk], a.dz1[trunk]};
  const float* __restrict__ XN = a.xn;
  f16v acc[TOW][TIW], acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    acc1[r] = 0.0f;
#pragma unroll
    for (int u = 0; u < TOW; ++u)
#pragma unroll
      for (int v = 0; v < TIW; ++v) acc[u][v][r] = 0.0f;
  }
  f4 st[3 * PW], sx[NXT];
  auto load = [&](long mb) {
#pragma unroll
    for (int s3 = 0; s3 < 3; ++s3)
#pragma unroll
      for (int p = 0; p < PW; ++p) {
        const int fl = 4 * (tid + NTH * p);
        const long row = mb + fl / H;
        st[s3 * PW + p] = row < m1 ? ld4(src3[s3] + row * H + fl % H) : f4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
    for (int p = 0; p < NXT; ++p) {
      const int fl = 4 * (tid + NTH * p);
      const long row = mb + fl / OP;
      sx[p] = (fl < KS * OP && row < m1) ? ld4(XN + row * OP + fl % OP) : f4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto store = [&](int buf) {
    float* b = lds + buf * STG;
#pragma unroll
    for (int s3 = 0; s3 < 3; ++s3)
#pragma unroll
      for (int p = 0; p < PW; ++p) {
        const int fl = 4 * (tid + NTH * p);
        *reinterpret_cast<f4*>(b + s3 * KS * LDH + (fl / H) * LDH + fl % H) = st[s3 * PW + p];
      }
#pragma unroll
    for (int p = 0; p < NXT; ++p) {
      const int fl = 4 * (tid + NTH * p);
      if (fl < KS * OP) *reinterpret_cast<f4*>(b + oXN + (fl / OP) * LDX + fl % OP) = sx[p];
    }
  };
  const int nst = (int)((m1 - m0 + KS - 1) / KS);
  load(m0);
  store(0);
  lds_barrier();
  if (nst > 1) load(m0 + KS);
  for (int sI = 0; sI < nst; ++sI) {
    const float* sb = lds + (sI & 1) * STG;
#pragma unroll
    for (int k = 0; k < KS; k += 2) {
      const float* rowp = sb + (k + hs) * LDH;
      float av[TOW], bv[TIW];
#pragma unroll
      for (int u = 0; u < TOW; ++u) av[u] = rowp[obase + (wo * TOW + u) * 32 + l32];
#pragma unroll
      for (int v = 0; v < TIW; ++v) bv[v] = rowp[oH1 + (wi * TIW + v) * 32 + l32];
      const float a1 = rowp[oDZ1 + (w1_wave ? w1row : 0) + l32];
      const float b1 = l32 < OP ? sb[oXN + (k + hs) * LDX + l32] : 0.0f;
#pragma unroll
      for (int u = 0; u < TOW; ++u)
#pragma unroll
        for (int v = 0; v < TIW; ++v) acc[u][v] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[v], acc[u][v], 0, 0, 0);
      if (w1_wave) acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc1, 0, 0, 0);
    }
    if (sI + 1 < nst) store((sI + 1) & 1);
    lds_barrier();
    if (sI + 2 < nst) load(m0 + (long)(sI + 2) * KS);
    __builtin_amdgcn_sched_barrier(0);  // keep the next-next stage's loads issued here
  }
  float* out = a.slab[trunk] + (size_t)blockIdx.x * a.slab_stride;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int orow = (r & 3) + 8 * (r >> 2) + 4 * hs;
#pragma unroll
    for (int u = 0; u < TOW; ++u)
#pragma unroll
      for (int v = 0; v < TIW; ++v)
        out[(size_t)(obase + (wo * TOW + u) * 32 + orow) * H + (wi * TIW + v) * 32 + l32] = acc[u][v][r];
    if (w1_wave && l32 < OP) out[(size_t)H * H + (size_t)(w1row + orow) * OP + l32] = acc1[r];
  }
}

// k_dwf_dma — k_dwf with the stage rows moved by LDS DMA (buffer_load ... lds, 16 bytes a lane: one
// wave instruction per 1 KB row) into three stage buffers, two stages ahead: no register staging,
// no ds_write phase between the MFMA blocks, and a stage's loads have two MFMA blocks to land.
// Rows are unpadded (a 32-lane operand read of two rows meets a 2-way bank conflict, which costs
// far less than the MFMAs it feeds); the MFMA loop and its operands are k_dwf's, so the result is
// bitwise k_dwf's. Rows past the chunk read as 0 through an out-of-range offset.
template <int H, int OP, int NSL>
__global__ __launch_bounds__(512) void k_dwf_dma(DwArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int KS = 16, NBUF = 3;
  constexpr int LDH = H, LDX = OP;
  constexpr int oH1 = KS * LDH, oDZ1 = 2 * KS * LDH, oXN = 3 * KS * LDH;
  constexpr int STG = 3 * KS * LDH + KS * LDX;
  static_assert(H == 256 && (OP == 16 || OP == 32), "k_dwf_dma geometry");
  // DMA instructions per stage: 3 x KS rows of H floats (one each) + the XN rows (KS * OP / 256)
  constexpr int NXI = KS * OP / 256;
  static_assert(KS == 16 && NXI <= 8, "k_dwf_dma: 2 rows of each source per wave + XN on waves 0 .. NXI-1");
  constexpr int TOW = 2 / NSL, TIW = 4;
  static_assert(NSL == 1 || NSL == 2, "k_dwf slices");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, hs = lane >> 5;
  const int wo = wave & 3, wi = wave >> 2;
  const int trunk = blockIdx.y, slice = NSL > 1 ? (int)blockIdx.z : 0;
  const int obase = slice * (H / NSL);
  const bool w1_wave = NSL == 1 || wave < 8 / NSL;
  const int w1row = obase + wave * 32;
  const long m0 = (long)blockIdx.x * a.rows_per_chunk;
  const long m1 = min((long)a.M, m0 + a.rows_per_chunk);
  if (m0 >= m1) return;
  const uint32_t rows_bytes = (uint32_t)((long)a.M * H * 4), xn_bytes = (uint32_t)((long)a.M * OP * 4);
  const PBuf bdz2 = make_pbuf(a.dz2[trunk], (int)(rows_bytes / 4)), bh1 = make_pbuf(a.h1[trunk], (int)(rows_bytes / 4));
  const PBuf bdz1 = make_pbuf(a.dz1[trunk], (int)(rows_bytes / 4));
  const PBuf bxn = make_pbuf(a.xn, (int)(xn_bytes / 4));
  f16v acc[TOW][TIW], acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    acc1[r] = 0.0f;
#pragma unroll
    for (int u = 0; u < TOW; ++u)
#pragma unroll
      for (int v = 0; v < TIW; ++v) acc[u][v][r] = 0.0f;
  }
  // stage at rows mb into buffer buf: wave w moves rows 2 w and 2 w + 1 of each of the three
  // row sources, waves 0 .. NXI-1 one XN instruction each (256 floats = 256 / OP rows)
  auto issue = [&](long mb, int buf) {
    float* b = lds + buf * STG;
#ifdef PPO_DIAG
    if (a.hot) mb = m0;  // diagnostic: L2-hot rows (bandwidth bound or not)
#endif
#pragma unroll
    for (int s3 = 0; s3 < 3; ++s3) {
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
        const int r = 2 * wave + rr;
        const long row = mb + r;
        const uint32_t voff = row < m1 ? (uint32_t)((row * H) * 4 + lane * 16) : 0xFFFFFFF0u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds((s3 == 0 ? bdz2 : s3 == 1 ? bh1 : bdz1).r,
                                                 (__attribute__((address_space(3))) void*)(b + s3 * KS * LDH + r * LDH), 16,
                                                 voff, 0, 0, 0);
      }
    }
    if (wave < NXI) {
      const int e = wave * 256 + lane * 4, r = e / OP;  // 4 floats of row r
      const long row = mb + r;
      const uint32_t voff = row < m1 ? (uint32_t)((row * OP + (e - r * OP)) * 4) : 0xFFFFFFF0u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(bxn.r, (__attribute__((address_space(3))) void*)(b + oXN + wave * 256), 16,
                                               voff, 0, 0, 0);
    }
  };
  // instructions this wave issues per stage: the vmcnt that leaves only the newest stage in flight
  const bool xw = wave < NXI;
  const int nst = (int)((m1 - m0 + KS - 1) / KS);
  issue(m0, 0);
  if (nst > 1) issue(m0 + KS, 1);
  for (int sI = 0; sI < nst; ++sI) {
    if (sI + 1 < nst) {  // stage sI + 1 may stay in flight
      if (xw) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    lds_barrier();  // every wave's stage-sI rows have landed; stage sI - 1's buffer is free
    if (sI + 2 < nst) issue(m0 + (long)(sI + 2) * KS, (sI + 2) % NBUF);
    __builtin_amdgcn_sched_barrier(0);
    const float* sb = lds + (sI % NBUF) * STG;
#pragma unroll
    for (int k = 0; k < KS; k += 2) {
      const float* rowp = sb + (k + hs) * LDH;
      float av[TOW], bv[TIW];
#pragma unroll
      for (int u = 0; u < TOW; ++u) av[u] = rowp[obase + (wo * TOW + u) * 32 + l32];
#pragma unroll
      for (int v = 0; v < TIW; ++v) bv[v] = rowp[oH1 + (wi * TIW + v) * 32 + l32];
      const float a1 = rowp[oDZ1 + (w1_wave ? w1row : 0) + l32];
      const float b1 = l32 < OP ? sb[oXN + (k + hs) * LDX + l32] : 0.0f;
#pragma unroll
      for (int u = 0; u < TOW; ++u)
#pragma unroll
        for (int v = 0; v < TIW; ++v) acc[u][v] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[v], acc[u][v], 0, 0, 0);
      if (w1_wave) acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc1, 0, 0, 0);
    }
  }
  float* out = a.slab[trunk] + (size_t)blockIdx.x * a.slab_stride;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int orow = (r & 3) + 8 * (r >> 2) + 4 * hs;
#pragma unroll
    for (int u = 0; u < TOW; ++u)
#pragma unroll
      for (int v = 0; v < TIW; ++v)
        out[(size_t)(obase + (wo * TOW + u) * 32 + orow) * H + (wi * TIW + v) * 32 + l32] = acc[u][v][r];
    if (w1_wave && l32 < OP) out[(size_t)H * H + (size_t)(w1row + orow) * OP + l32] = acc1[r];
  }
}

// =============================================================================================
// k_dwf_bx — k_dwf_dma's products on BF16 MFMAs with every fp32 operand split exactly in three
// (create option dw_mfma=bf16x9 / bf16x8; the default: see ppo_capi.hip).
//
// On gfx950 the fp32 MFMA runs at 1/16 of the BF16 rate (MI355X_MICROARCH.md: 157 vs ~2 500
// TF/s), and k_dwf_dma is MFMA-bound (matrix pipe 0.77 busy, 1.9 VALU per MFMA). Every fp32 x is
// the exact sum of three bf16 numbers: hi = x with the low 16 bits cleared (truncation), r = x - hi
// (exact: a prefix of x's significand is removed), mid = r truncated the same way, lo = r - mid
// (exact, at most 8 significant bits: a bf16). So a.b = sum over the nine piece products, each
// product of two 8-bit significands exact in fp32, and the MFMA accumulates them in fp32 like the
// fp32 MFMA accumulates a.b: NP = 9 keeps every piece product (an exact-product fp32 GEMM in a
// different summation order), NP = 8 drops lo.lo (< 2^-30 |a.b|: 64x below an fp32 rounding). The
// passes of one k-block run smallest first. v_mfma_f32_32x32x16_bf16 takes 32 cycles for 16 k
// against 8 x 64 cycles of v_mfma_f32_32x32x2_f32: 9 passes are 0.56 of the fp32 MFMA time, 8 0.50.
// Operand layout (cdna_hip_programming.md): lane (r = l & 31, h = l >> 5) holds A[r][8 h + e] and
// B[8 h + e][r] in element e = 0..7; the accumulator layout is the 32x32x2 one, so the slab stores
// are k_dwf_dma's. Per 16-row stage a lane reads its column of rows 8 h .. 8 h + 7 (ds_read_b32,
// the same count as k_dwf_dma's 8 k-steps) and splits each value once (v_and / v_sub / v_perm).
// Staging (LDS DMA, three buffers, two stages ahead) is k_dwf_dma's.
// =============================================================================================
// RC (DwArgs::h1_recompute): the stages carry DZ2 | DZ1 | Xn | the rows' layer-1 LayerNorm statistics
// (64 floats); H1 of a stage is recomputed into one buffer H1B behind the three stages, from the staged Xn
// rows, W1 (swizzled copy, staged once per workgroup in W1S) and the bias / LayerNorm affine (PRM) —
// k_upd's chain, so bitwise the H1 rows k_upd would have stored; k_upd then writes 8 bytes per row
// instead of 1 KB (the hand-off's H1 third).
// cache policy of k_dwf_bx's hand-off stream (read once): 2 non-temporal (dW 3.41 -> 3.31 ms per metric
// iteration, bitwise the same; profiles/r06/dw_nt/), 0 the default policy
#ifndef PPO_DW_AUX
#define PPO_DW_AUX 2
#endif
// k_dwf_bx's split-K partials (read once by k_colsum): PPO_DW_NTST = 1 stores them non-temporal (A/B)
#ifndef PPO_DW_NTST
#define PPO_DW_NTST 0
#endif
PPO_DEV void dw_st(float* p, float v) {
#if PPO_DW_NTST
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
template <int H, int OP, bool RC>
struct DwbxGeo {
  static constexpr int KS = 16, LDH = H, LDX = OP;
  static constexpr int oH1 = RC ? 0 : KS * LDH;  // (RC: H1 lives in H1B)
  static constexpr int oDZ1 = RC ? KS * LDH : 2 * KS * LDH;
  static constexpr int oXN = RC ? 2 * KS * LDH : 3 * KS * LDH;
  static constexpr int oLNS = oXN + KS * LDX;     // RC: [16][2] (mean, 1 / std) + 32 floats the DMA zero-fills
  static constexpr int STG = oXN + KS * LDX + (RC ? 64 : 0);
  static constexpr int oH1B = 3 * STG, oW1S = oH1B + KS * LDH, oPRM = oW1S + H * OP;
  static constexpr int total = RC ? oPRM + 3 * H : 3 * STG;  // floats
};
template <int H, int OP, int NSL, int NP, bool RC = false>
__global__ __launch_bounds__(512) void k_dwf_bx(DwArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  using GE = DwbxGeo<H, OP, RC>;
  constexpr int KS = 16, NBUF = 3;
  constexpr int LDH = H, LDX = OP;
  constexpr int oH1 = GE::oH1, oDZ1 = GE::oDZ1, oXN = GE::oXN;
  constexpr int STG = GE::STG;
  static_assert(H == 256 && (OP == 16 || OP == 32), "k_dwf_bx geometry");
  constexpr int NXI = KS * OP / 256;
  constexpr int TOW = 2 / NSL, TIW = 4;
  static_assert(NSL == 1 || NSL == 2, "k_dwf slices");
  static_assert(NP == 6 || NP == 8 || NP == 9, "k_dwf_bx passes");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, hs = lane >> 5;
  const int wo = wave & 3, wi = wave >> 2;
  const int trunk = blockIdx.y, slice = NSL > 1 ? (int)blockIdx.z : 0;
  const int obase = slice * (H / NSL);
  const bool w1_wave = NSL == 1 || wave < 8 / NSL;
  const int w1row = obase + wave * 32;
  const long m0 = (long)blockIdx.x * a.rows_per_chunk;
  const long m1 = min((long)a.M, m0 + a.rows_per_chunk);
  if (m0 >= m1) return;
  const uint32_t rows_bytes = (uint32_t)((long)a.M * H * 4), xn_bytes = (uint32_t)((long)a.M * OP * 4);
  const PBuf bdz2 = make_pbuf(a.dz2[trunk], (int)(rows_bytes / 4)), bh1 = make_pbuf(a.h1[trunk], (int)(rows_bytes / 4));
  const PBuf bdz1 = make_pbuf(a.dz1[trunk], (int)(rows_bytes / 4));
  const PBuf bxn = make_pbuf(a.xn, (int)(xn_bytes / 4));
  const PBuf blns = make_pbuf(RC ? a.lns[trunk] : a.xn, RC ? 2 * a.M : 0);
  if constexpr (RC) {
    // W1 (swizzled, H x OP) and the bias / gamma / beta of layer 1, staged once per workgroup; waited for
    // here, before the stage pipeline's DMAs (whose wait counts assume nothing else in flight)
    constexpr int NW = H * OP / 4 / 512;
    f4 wv[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) wv[q] = *reinterpret_cast<const f4*>(a.w1sw[trunk] + 4 * (tid + 512 * q));
    const float pv1 = tid < H ? a.b1[trunk][tid] : 0.f;
    const float pv2 = tid < H ? a.g1[trunk][tid] : 0.f;
    const float pv3 = tid < H ? a.be1[trunk][tid] : 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) *reinterpret_cast<f4*>(lds + GE::oW1S + 4 * (tid + 512 * q)) = wv[q];
    if (tid < H) {
      lds[GE::oPRM + tid] = pv1;
      lds[GE::oPRM + H + tid] = pv2;
      lds[GE::oPRM + 2 * H + tid] = pv3;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  f16v acc[TOW][TIW], acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    acc1[r] = 0.0f;
#pragma unroll
    for (int u = 0; u < TOW; ++u)
#pragma unroll
      for (int v = 0; v < TIW; ++v) acc[u][v][r] = 0.0f;
  }
  auto issue = [&](long mb, int buf) {
    float* b = lds + buf * STG;
#ifdef PPO_DIAG
    if (a.hot) mb = m0;  // diagnostic: L2-hot rows (bandwidth bound or not)
#endif
#pragma unroll
    for (int s3 = 0; s3 < 3; ++s3) {
      if (RC && s3 == 1) continue;  // H1 is recomputed
      const int dst = s3 == 0 ? 0 : s3 == 1 ? oH1 : oDZ1;
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
        const int r = 2 * wave + rr;
        const long row = mb + r;
        const uint32_t voff = row < m1 ? (uint32_t)((row * H) * 4 + lane * 16) : 0xFFFFFFF0u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds((s3 == 0 ? bdz2 : s3 == 1 ? bh1 : bdz1).r,
                                                 (__attribute__((address_space(3))) void*)(b + dst + r * LDH), 16,
                                                 voff, 0, 0, PPO_DW_AUX);
      }
    }
    if (RC && wave == 7) {  // the stage's 16 rows x (mean, 1 / std): 32 dwords (lanes 32..63 zero-fill the pad)
      const long row = mb + (lane >> 1);
      const uint32_t voff = lane < 32 && row < m1 ? (uint32_t)(row * 8 + (lane & 1) * 4) : 0xFFFFFFF0u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(blns.r, (__attribute__((address_space(3))) void*)(b + GE::oLNS), 4, voff,
                                               0, 0, 0);
    }
    if (wave < NXI) {
      const int e = wave * 256 + lane * 4, r = e / OP;
      const long row = mb + r;
      const uint32_t voff = row < m1 ? (uint32_t)((row * OP + (e - r * OP)) * 4) : 0xFFFFFFF0u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(bxn.r, (__attribute__((address_space(3))) void*)(b + oXN + wave * 256), 16,
                                               voff, 0, 0, PPO_DW_AUX);
    }
  };
  const bool xw = wave < NXI;
  const int nst = (int)((m1 - m0 + KS - 1) / KS);
  issue(m0, 0);
  if (nst > 1) issue(m0 + KS, 1);
  for (int sI = 0; sI < nst; ++sI) {
    if (sI + 1 < nst) {  // this wave's DMAs of stage sI + 1 stay in flight
      if constexpr (RC) {
        if (xw || wave == 7) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      } else {
        if (xw) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      }
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    lds_barrier();
    if (sI + 2 < nst) issue(m0 + (long)(sI + 2) * KS, (sI + 2) % NBUF);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (RC) {
      // H1 of this stage (16 rows x H): wave w computes features 32 w .. 32 w + 31 as two 16x16 tiles with
      // k_upd's layer-1 chain, then its LayerNorm + affine + ReLU from the row's stored statistics
      constexpr int NTO = OP / 16;
      const int j16 = lane & 15, g16 = lane >> 4, f0 = 32 * wave;
      const float* stg = lds + (sI % NBUF) * STG;
      f4 z[2];
#pragma unroll
      for (int ft = 0; ft < 2; ++ft) z[ft] = *reinterpret_cast<const f4*>(lds + GE::oPRM + f0 + 16 * ft + 4 * g16);
#pragma unroll
      for (int kb = 0; kb < NTO; ++kb) {
        const f4 bv = *reinterpret_cast<const f4*>(stg + oXN + j16 * LDX + 16 * kb + 4 * g16);
        f4 w[2];
#pragma unroll
        for (int ft = 0; ft < 2; ++ft)
          w[ft] = *reinterpret_cast<const f4*>(lds + GE::oW1S + (((f0 >> 4) + ft) * NTO + kb) * 256 + 4 * lane);
        const bool full = kb + 1 < NTO || a.kl1 >= 4;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (c > 0 && !full) break;
#pragma unroll
          for (int ft = 0; ft < 2; ++ft) z[ft] = mfma16(w[ft][c], bv[c], z[ft]);
        }
      }
      const float mu = stg[GE::oLNS + 2 * j16], rs = stg[GE::oLNS + 2 * j16 + 1];
#pragma unroll
      for (int ft = 0; ft < 2; ++ft) {
        const int f = f0 + 16 * ft + 4 * g16;
        const f4 gm = *reinterpret_cast<const f4*>(lds + GE::oPRM + H + f);
        const f4 bt = *reinterpret_cast<const f4*>(lds + GE::oPRM + 2 * H + f);
        f4 h;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float xh = (z[ft][r] - mu) * rs;
          const float y = __fmaf_rn(gm[r], xh, bt[r]);
          h[r] = y > 0.0f ? y : 0.0f;
        }
        *reinterpret_cast<f4*>(lds + GE::oH1B + j16 * LDH + f) = h;
      }
      lds_barrier();
    }
    const float* sb = lds + (sI % NBUF) * STG + (8 * hs) * LDH;  // this lane's rows 8 hs .. 8 hs + 7
    const float* hb = (RC ? lds + GE::oH1B : lds + (sI % NBUF) * STG + oH1) + (8 * hs) * LDH;
    Split3 as[TOW], a1s, b1s;
    {
      float x[8];
#pragma unroll
      for (int u = 0; u < TOW; ++u) {
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = sb[e * LDH + obase + (wo * TOW + u) * 32 + l32];
        as[u] = split3(x);
      }
      if (w1_wave) {
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = sb[oDZ1 + e * LDH + w1row + l32];
        a1s = split3(x);
        const float* xb = lds + (sI % NBUF) * STG + oXN + (8 * hs) * LDX;
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = l32 < OP ? xb[e * LDX + l32] : 0.0f;
        b1s = split3(x);
      }
    }
#pragma unroll
    for (int v = 0; v < TIW; ++v) {
      float x[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = hb[e * LDH + (wi * TIW + v) * 32 + l32];
      const Split3 bs = split3(x);
#pragma unroll
      for (int u = 0; u < TOW; ++u) acc[u][v] = mfma_split<NP>(as[u], bs, acc[u][v]);
    }
    if (w1_wave) acc1 = mfma_split<NP>(a1s, b1s, acc1);
  }
  float* out = a.slab[trunk] + (size_t)blockIdx.x * a.slab_stride;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int orow = (r & 3) + 8 * (r >> 2) + 4 * hs;
#pragma unroll
    for (int u = 0; u < TOW; ++u)
#pragma unroll
      for (int v = 0; v < TIW; ++v)
        dw_st(out + (size_t)(obase + (wo * TOW + u) * 32 + orow) * H + (wi * TIW + v) * 32 + l32, acc[u][v][r]);
    if (w1_wave && l32 < OP) dw_st(out + (size_t)H * H + (size_t)(w1row + orow) * OP + l32, acc1[r]);
  }
}

// =============================================================================================
// k_colsum — dst[seg] = sum_{c < C} src[c * stride + seg]   (fixed order => deterministic)
// =============================================================================================
// The segments are cut into 64-float column tiles, numbered consecutively over all segments
// (ColsumArgs::tile0 = first tile of each segment). A workgroup owns one tile: thread (c, q) sums
// float4 column c over rows q, q + 16, q + 32, ... (four loads in flight), and the 16 row phases
// are added in a fixed order through LDS — deterministic, and every workgroup has work.
// gradnorm=fold, wave 0 of a tile's workgroup (lanes 0..15 hold the squares of the values they wrote):
// the tile's sum (fixed lane tree) stored write-through (agent-scope atomic store = sc1) and drained
// before the segment's counter add; the last arriver reads every tile's sum with sc1 loads (no L1 /
// other-XCD L2 copy can be stale: cdna_hip_programming.md Guideline 16, counter form) and adds them in
// tile order. Determinism: every sum has a fixed order whatever the arrival order.
typedef __attribute__((address_space(1))) float gfl;
typedef __attribute__((address_space(1))) unsigned gu32;
PPO_DEV void colsum_fold(const ColsumArgs& a, int sgi, int b, float ss) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) ss += __shfl_xor(ss, m, 64);  // lanes 0..15: one closed group
  unsigned ticket = 0;
  if (lane == 0) {
    __hip_atomic_store((gfl*)(a.sq + b), ss, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ticket = __hip_atomic_fetch_add((gu32*)(a.cnt + sgi), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  ticket = __shfl(ticket, 0, 64);
  const int t0 = a.tile0[sgi], n = a.tile0[sgi + 1] - t0;
  if ((int)ticket != n - 1) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the loads below the ticket
  // up to 16 loads in flight per lane (one memory round trip per 1 024 tiles), added in tile order
  float acc = 0.f;
  for (int k0 = 0; k0 < n; k0 += 1024) {
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int k = k0 + lane + 64 * j;
      v[j] = __hip_atomic_load((gfl*)(a.sq + t0 + min(k, n - 1)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) acc += (k0 + lane + 64 * j < n) ? v[j] : 0.f;
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 64);
  if (lane < PPO_GN_SPLIT) a.part[a.seg_t[sgi] * PPO_GN_SPLIT + lane] = lane == 0 ? acc : 0.f;
  if (lane == 0) __hip_atomic_store((gu32*)(a.cnt + sgi), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// split-K partials are read once: PPO_CS_NT = 1 loads them non-temporal (A/B)
#ifndef PPO_CS_NT
#define PPO_CS_NT 0
#endif
PPO_DEV f4 cs_ld4(const float* p) {
#if PPO_CS_NT
  return __builtin_nontemporal_load(reinterpret_cast<const f4*>(p));
#else
  return ld4(p);
#endif
}
__global__ __launch_bounds__(256) void k_colsum(ColsumArgs a) {
  __shared__ f4 part[16][16];
  const int b = blockIdx.x;
  int sgi = 0;
  while (sgi + 1 < a.nseg && b >= a.tile0[sgi + 1]) ++sgi;
  const ColsumSeg& S = a.seg[sgi];
  const int tid = threadIdx.x, c = tid & 15, q = tid >> 4;
  const long col0 = (long)(b - a.tile0[sgi]) * 64;
  const bool vec = ((((uintptr_t)S.src) | ((uintptr_t)S.dst)) & 15) == 0 && (S.stride & 3) == 0 && (S.len & 3) == 0;
  if (vec) {
    const long i = col0 + 4 * c;
    f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
    if (i < S.len) {
      const float* src = S.src + i;
      int r = q;
      // eight loads in flight (one round trip for the usual 128 chunks); each accumulator still
      // takes its rows in the order of the four-wide loop below, so the sums are unchanged
      for (; r + 112 < S.count; r += 128) {
        const f4 x0 = cs_ld4(src + (size_t)r * S.stride), x1 = cs_ld4(src + (size_t)(r + 16) * S.stride);
        const f4 x2 = cs_ld4(src + (size_t)(r + 32) * S.stride), x3 = cs_ld4(src + (size_t)(r + 48) * S.stride);
        const f4 x4 = cs_ld4(src + (size_t)(r + 64) * S.stride), x5 = cs_ld4(src + (size_t)(r + 80) * S.stride);
        const f4 x6 = cs_ld4(src + (size_t)(r + 96) * S.stride), x7 = cs_ld4(src + (size_t)(r + 112) * S.stride);
        acc0 += x0;
        acc1 += x1;
        acc2 += x2;
        acc3 += x3;
        acc0 += x4;
        acc1 += x5;
        acc2 += x6;
        acc3 += x7;
      }
      for (; r + 48 < S.count; r += 64) {
        acc0 += cs_ld4(src + (size_t)r * S.stride);
        acc1 += cs_ld4(src + (size_t)(r + 16) * S.stride);
        acc2 += cs_ld4(src + (size_t)(r + 32) * S.stride);
        acc3 += cs_ld4(src + (size_t)(r + 48) * S.stride);
      }
      for (; r < S.count; r += 16) acc0 += cs_ld4(src + (size_t)r * S.stride);
    }
    part[q][c] = (acc0 + acc1) + (acc2 + acc3);
    __syncthreads();
    float ss = 0.f;
    if (q == 0 && i < S.len) {
      f4 t = part[0][c];
#pragma unroll
      for (int p = 1; p < 16; ++p) t += part[p][c];
      const f4 w = t * S.scale;
      st4(S.dst + i, w);
      ss = (w.x * w.x + w.y * w.y) + (w.z * w.z + w.w * w.w);
    }
    if (a.fold && a.seg_t[sgi] >= 0 && tid < 64) colsum_fold(a, sgi, b, ss);
    return;
  }
  // unaligned / ragged segments (biases of width 1..A, loss stats): same 16 row phases, scalar,
  // 16 columns at a time
  float* sp = reinterpret_cast<float*>(part);
  float ss = 0.f;
  for (int cb = 0; cb < 64 && col0 + cb < S.len; cb += 16) {
    const long i = col0 + cb + c;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    if (i < S.len) {
      const float* src = S.src + i;
      int r = q;
      for (; r + 48 < S.count; r += 64) {
        a0 += src[(size_t)r * S.stride];
        a1 += src[(size_t)(r + 16) * S.stride];
        a2 += src[(size_t)(r + 32) * S.stride];
        a3 += src[(size_t)(r + 48) * S.stride];
      }
      for (; r < S.count; r += 16) a0 += src[(size_t)r * S.stride];
    }
    sp[q * 16 + c] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (q == 0 && i < S.len) {
      float t = sp[c];
#pragma unroll
      for (int p = 1; p < 16; ++p) t += sp[p * 16 + c];
      const float w = t * S.scale;
      S.dst[i] = w;
      ss += w * w;
    }
    __syncthreads();
  }
  if (a.fold && a.seg_t[sgi] >= 0 && tid < 64) colsum_fold(a, sgi, b, ss);
}

// =============================================================================================
// k_gradnorm — clip_grad_norm_: per-tensor L2 norms (fp32 tensors), norm of norms, clip coef
// =============================================================================================
// pass 1 (k_gradnorm): grid (tensor, PPO_GN_SPLIT slices) -> partial sums of squares;
// pass 2 (head of k_adam, every block): per-tensor norms from the slices in order, total, coef.
PPO_DEV void gradnorm_slice(const NormArgs& a, int t, int sp, float* red) {
  const int tid = threadIdx.x;
  const int len = a.len[t], sl = (((len + PPO_GN_SPLIT - 1) / PPO_GN_SPLIT) + 3) & ~3;
  const int i0 = sp * sl, i1 = min(len, i0 + sl);
  const float* g = a.grad + a.off[t];
  float s = 0.0f;
  if (((a.off[t] | sl) & 3) == 0) {
    for (int i = i0 + 4 * tid; i < i1; i += 1024) {
      if (i + 3 < i1) {
        const f4 v = ld4(g + i);
        s += (v.x * v.x + v.y * v.y) + (v.z * v.z + v.w * v.w);
      } else {
        for (int k = i; k < i1; ++k) s += g[k] * g[k];
      }
    }
  } else {
    for (int i = i0 + tid; i < i1; i += 256) s += g[i] * g[i];
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) a.part[t * PPO_GN_SPLIT + sp] = (red[0] + red[1]) + (red[2] + red[3]);
}
__global__ __launch_bounds__(256) void k_gradnorm(NormArgs a) {
  __shared__ float red[4];
  gradnorm_slice(a, blockIdx.x, blockIdx.y, red);
}

// =============================================================================================
// k_adam — grad *= clip coef; Adam (bias-corrected, torch::optim::Adam); refresh W2^T copies
// =============================================================================================
PPO_DEV void adam_block(const AdamArgs& a, int bid, float* s_norm, float& s_coef) {
  const int blockIdx_x = bid;
  if (threadIdx.x < a.nt) {
    float q = 0.0f;
#pragma unroll
    for (int sp = 0; sp < PPO_GN_SPLIT; ++sp) q += a.part[threadIdx.x * PPO_GN_SPLIT + sp];
    s_norm[threadIdx.x] = sqrtf(q);  // per-tensor L2 norm (an fp32 tensor, clip_grad.h: grad.norm())
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    // clip_grad_norm_: total = ||(||g_t||)_t||, coef = clamp(max_norm / (total + 1e-6), max = 1)
    float tot = 0.0f;
    for (int t = 0; t < a.nt; ++t) tot += s_norm[t] * s_norm[t];
    const float total = sqrtf(tot);
    float coef = a.max_norm / (total + 1e-6f);
    coef = coef > 1.0f ? 1.0f : coef;
    s_coef = coef;
    if (blockIdx_x == 0) {
      a.norm_out[0] = total;
      a.norm_out[1] = coef;
      if (a.stat_out) a.stat_out[0] = total;
    }
  }
  if (blockIdx_x == 0 && threadIdx.x < a.nt) a.norm_out[2 + threadIdx.x] = s_norm[threadIdx.x];
  __syncthreads();
  const long i = (long)blockIdx_x * 256 + threadIdx.x;
  if (i >= a.n) return;  // (no barrier follows)
  const long p = a.begin + i;
  const float coef = s_coef;
  const float gv = a.grad[p] * coef;
  const float m = a.m[p] * 0.9f + gv * 0.1f;
  const float v = a.v[p] * 0.999f + gv * gv * 0.001f;
  a.m[p] = m;
  a.v[p] = v;
  const float sbc2 = a.sched ? a.sched[2 * a.gi + 1] : a.sbc2;
  const float step_size = a.sched ? a.sched[2 * a.gi] : a.step_size;
  const float denom = sqrtf(v) / sbc2 + a.eps;
  const float np = a.param[p] - step_size * (m / denom);
  a.param[p] = np;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const long o = p - a.w2_off[k];
    if (o >= 0 && o < (long)a.H * a.H) {
      const int r = (int)(o / a.H), cI = (int)(o % a.H);
      a.w2t[k][(size_t)cI * a.H + r] = np;
      if (a.wsw[k]) {
        float* w = a.wsw[k] + (long)a.H * a.OP;
        w[sw_index(r, cI, a.H)] = np;
        w[(long)a.H * a.H + sw_index(cI, r, a.H)] = np;
        if (a.bx == 1) {  // split-bf16 pieces of W2 | W2^T (bx_index), after the fp32 copies
          uint16_t* pw = reinterpret_cast<uint16_t*>(a.wsw[k] + sw_size(a.H, a.OP));
          uint16_t pc[3];
          split3_bits(np, pc);
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            pw[bx_index(r, cI, a.H, q)] = pc[q];
            pw[3L * a.H * a.H + bx_index(cI, r, a.H, q)] = pc[q];
          }
        }
      }
    }
    const long o1 = p - a.w1_off[k];
    if (a.wsw[k] && o1 >= 0 && o1 < (long)a.H * a.OP) {
      const int r = (int)(o1 / a.OP), cI = (int)(o1 % a.OP);
      a.wsw[k][sw_index(r, cI, a.OP)] = np;
      if (a.bx == 2) {  // split-bf16 pieces of W1 (bx_index), after the fp32 copies
        uint16_t* pw = reinterpret_cast<uint16_t*>(a.wsw[k] + sw_size(a.H, a.OP));
        uint16_t pc[3];
        split3_bits(np, pc);
#pragma unroll
        for (int q = 0; q < 3; ++q) pw[bx_index(r, cI, a.OP, q)] = pc[q];
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_adam(AdamArgs a) {
  __shared__ float s_norm[PPO_LAYOUT_MAX_TENSORS];
  __shared__ float s_coef;
  adam_block(a, blockIdx.x, s_norm, s_coef);
}

// k_gradnorm and k_adam as ONE cooperative launch: workgroups 0 .. nt * PPO_GN_SPLIT - 1 first run
// the norm slices of k_gradnorm, a grid barrier makes the partials visible, then every workgroup
// runs its k_adam block. Same functions, same partial order: bitwise the two-launch result, one
// launch floor fewer per minibatch (320 minibatches per iteration at cfg1 / cfg2).
__global__ __launch_bounds__(256) void k_gradstep(NormArgs na, AdamArgs a, unsigned* bar, unsigned target) {
  __shared__ float red[4];
  __shared__ float s_norm[PPO_LAYOUT_MAX_TENSORS];
  __shared__ float s_coef;
  if ((int)blockIdx.x < na.nt * PPO_GN_SPLIT) gradnorm_slice(na, blockIdx.x / PPO_GN_SPLIT, blockIdx.x % PPO_GN_SPLIT, red);
  grid_barrier(bar, target);
  adam_block(a, blockIdx.x, s_norm, s_coef);
}

// swizzled copies of one trunk (sw_index): [W1 (H x OP) | W2 (H x H) | W2^T (H x H)]
// bx: also the split-bf16 pieces (bx_index) after them: 1 of W2 | W2^T, 2 of W1
__global__ void k_swizzle(const float* __restrict__ w1, const float* __restrict__ w2, float* __restrict__ dst, int H,
                          int OP, int bx) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n1 = (long)H * OP, n2 = (long)H * H;
  if (i < n1) {
    const int r = (int)(i / OP), c = (int)(i % OP);
    dst[sw_index(r, c, OP)] = w1[i];
    if (bx == 2) {
      uint16_t* pw = reinterpret_cast<uint16_t*>(dst + sw_size(H, OP));
      uint16_t pc[3];
      split3_bits(w1[i], pc);
      for (int q = 0; q < 3; ++q) pw[bx_index(r, c, OP, q)] = pc[q];
    }
  } else if (i < n1 + n2) {
    const long o = i - n1;
    const int r = (int)(o / H), c = (int)(o % H);
    dst[n1 + sw_index(r, c, H)] = w2[o];
    dst[n1 + n2 + sw_index(c, r, H)] = w2[o];
    if (bx == 1) {
      uint16_t* pw = reinterpret_cast<uint16_t*>(dst + sw_size(H, OP));
      uint16_t pc[3];
      split3_bits(w2[o], pc);
      for (int q = 0; q < 3; ++q) {
        pw[bx_index(r, c, H, q)] = pc[q];
        pw[3 * n2 + bx_index(c, r, H, q)] = pc[q];
      }
    }
  }
}

__global__ void k_transpose(const float* __restrict__ src, float* __restrict__ dst, int H) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= H * H) return;
  const int r = i / H, c = i % H;
  dst[(size_t)c * H + r] = src[i];
}

// =============================================================================================
// k_gae — one thread per env, t = T-1 .. 0; op-for-op fp32 (no contraction), ppo:447-467.
// The recurrence stays serial per env (bit-exact with the reference's order); its inputs are not:
// rewards / values / dones of kGaeChunk steps are loaded together (coalesced over envs, loads
// unconditional with a clamped step), and the next chunk's loads are issued before the current
// chunk's recurrence runs (two register buffers), so the memory round trips overlap the serial
// chain instead of alternating with it. 64-thread workgroups spread few envs over many CUs (cfg2:
// E = 1 024 envs on 16 CUs instead of 4).
// =============================================================================================
constexpr int kGaeChunk = 32;
struct GaeChunk {
  float r[kGaeChunk], v[kGaeChunk], d[kGaeChunk];
};
PPO_DEV void gae_load(const GaeArgs& a, int e, int t1, GaeChunk& c) {
  const long E = a.E;
#pragma unroll
  for (int k = 0; k < kGaeChunk; ++k) {
    const int t = t1 - k >= 0 ? t1 - k : 0;
    const long idx = (long)t * E + e;
    c.r[k] = a.rewards[idx];
    c.v[k] = a.values[idx];
    c.d[k] = a.dones[idx];
  }
}
PPO_DEV void gae_run(const GaeArgs& a, int e, int t1, const GaeChunk& c, float& last, float& nnt, float& nv) {
#pragma clang fp contract(off)
  const long E = a.E;
  const float gl = (a.gamma * a.lam);
#pragma unroll
  for (int k = 0; k < kGaeChunk; ++k) {
    if (t1 - k < 0) break;
    const long idx = (long)(t1 - k) * E + e;
    const float r = c.r[k], v = c.v[k];
    const float gnv = (a.gamma * nv);
    const float delta = ((r + (gnv * nnt)) - v);
    const float adv = (delta + ((gl * nnt) * last));
    a.adv[idx] = adv;
    a.ret[idx] = (adv + v);
    last = adv;
    nnt = (1.0f - c.d[k]);
    nv = v;
  }
}
__global__ __launch_bounds__(64) void k_gae(GaeArgs a) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.E) return;
  float last = 0.0f;
  float nnt = (1.0f - a.next_done[e]);
  float nv = a.next_value[e];
  GaeChunk c0, c1;
  int t1 = a.T - 1;
  gae_load(a, e, t1, c0);
  while (t1 >= 0) {
    const int t2 = t1 - kGaeChunk;
    if (t2 >= 0) gae_load(a, e, t2, c1);
    gae_run(a, e, t1, c0, last, nnt, nv);
    if (t2 < 0) break;
    const int t3 = t2 - kGaeChunk;
    if (t3 >= 0) gae_load(a, e, t3, c0);
    gae_run(a, e, t2, c1, last, nnt, nv);
    t1 = t3;
  }
}

// k_gae_scan — the same recurrence as a segmented scan over T (create option gae=scan; north_star's
// wavefront scan): A_t = delta_t + c_t A_{t+1}, c_t = gamma lambda (1 - d_{t+1}), is an affine map of
// A_{t+1}; a workgroup holds 64 envs (lane = env: every step's loads are 256 contiguous bytes) and
// 16 waves, wave w the w-th of 16 segments of the steps. Pass 1: each lane composes its segment's maps
// from the end, A_{t_lo} = b + a A_{t_hi}. The segments' (a, b) meet in LDS, each wave composes those
// of the later segments into its incoming A_{t_hi} (A_T = 0), and pass 2 runs the reference's serial
// recurrence over the segment from that value. Within fp32 rounding of the serial form (the incoming
// values are composed in another order), not bit-exact: the serial k_gae stays the default.
constexpr int kScanSeg = 16, kScanChunk = 8;
__global__ __launch_bounds__(1024) void k_gae_scan(GaeArgs a) {
#pragma clang fp contract(off)
  __shared__ float sa[kScanSeg][64], sb[kScanSeg][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + lane;
  const bool ok = e < a.E;
  const int ec = ok ? e : 0;  // clamped for the loads
  const long E = a.E;
  const int S = (a.T + kScanSeg - 1) / kScanSeg;
  const int t_lo = min(a.T, w * S), t_hi = min(a.T, t_lo + S);
  const float gam = a.gamma, gl = (a.gamma * a.lam);
  const float nv_hi = t_hi == a.T ? a.next_value[ec] : a.values[(long)t_hi * E + ec];
  const float nd_hi = t_hi == a.T ? a.next_done[ec] : a.dones[(long)t_hi * E + ec];
  // the steps t_hi - 1 - k, k < kScanChunk, of chunk c (clamped loads; masked by the step test)
  auto load = [&](int t1, float (&r)[kScanChunk], float (&v)[kScanChunk], float (&d)[kScanChunk]) {
#pragma unroll
    for (int k = 0; k < kScanChunk; ++k) {
      const int t = t1 - k >= t_lo ? t1 - k : t_lo;
      const long idx = (long)t * E + ec;
      r[k] = a.rewards[idx];
      v[k] = a.values[idx];
      d[k] = a.dones[idx];
    }
  };
  float ca = 1.0f, cb = 0.0f;
  {
    float nv = nv_hi, nnt = (1.0f - nd_hi);
    for (int t1 = t_hi - 1; t1 >= t_lo; t1 -= kScanChunk) {
      float r[kScanChunk], v[kScanChunk], d[kScanChunk];
      load(t1, r, v, d);
#pragma unroll
      for (int k = 0; k < kScanChunk; ++k) {
        if (t1 - k < t_lo) break;
        const float gnv = (gam * nv);
        const float delta = ((r[k] + (gnv * nnt)) - v[k]);
        const float c = (gl * nnt);
        cb = (delta + (c * cb));
        ca = (c * ca);
        nnt = (1.0f - d[k]);
        nv = v[k];
      }
    }
  }
  sa[w][lane] = ca;
  sb[w][lane] = cb;
  __syncthreads();
  float last = 0.0f;
  for (int u = kScanSeg - 1; u > w; --u) last = (sb[u][lane] + (sa[u][lane] * last));
  {
    float nv = nv_hi, nnt = (1.0f - nd_hi);
    for (int t1 = t_hi - 1; t1 >= t_lo; t1 -= kScanChunk) {
      float r[kScanChunk], v[kScanChunk], d[kScanChunk];
      load(t1, r, v, d);
#pragma unroll
      for (int k = 0; k < kScanChunk; ++k) {
        if (t1 - k < t_lo) break;
        const long idx = (long)(t1 - k) * E + ec;
        const float gnv = (gam * nv);
        const float delta = ((r[k] + (gnv * nnt)) - v[k]);
        const float adv = (delta + ((gl * nnt) * last));
        if (ok) {
          a.adv[idx] = adv;
          a.ret[idx] = (adv + v[k]);
        }
        last = adv;
        nnt = (1.0f - d[k]);
        nv = v[k];
      }
    }
  }
}

// =============================================================================================
// minibatch permutations and advantage statistics
// =============================================================================================
__global__ __launch_bounds__(256) void k_perm(int32_t* __restrict__ out, uint32_t B, PermKey pk) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < B) out[i] = (int32_t)perm_index(i, B, pk);
}

// Advantage statistics of every minibatch, PPO_ADV_SPLIT workgroups per minibatch: each sums a
// contiguous slice of the minibatch's permutation entries (double), the partials are then added
// in slice order by one thread per minibatch — deterministic.
PPO_DEV double block_sum_d(double s, double* red) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0)
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
  return t;
}
// pass 1: slice sums of the gathered advantages
__global__ __launch_bounds__(256) void k_adv_sum(AdvArgs a) {
  __shared__ double red[4];
  const int mb = blockIdx.x, sl = blockIdx.y;
  const int len = (a.M + PPO_ADV_SPLIT - 1) / PPO_ADV_SPLIT;
  const int i0 = sl * len, i1 = min(a.M, i0 + len);
  const int32_t* perm = a.perm + (long)mb * a.M;
  double s = 0.0;
  for (int i = i0 + threadIdx.x; i < i1; i += 256) s += (double)a.adv[perm[i]];
  const double t = block_sum_d(s, red);
  if (threadIdx.x == 0) a.part[mb * PPO_ADV_SPLIT + sl] = t;
}
// -> stats[2mb] = local mean (all-reduced with ncclAvg when G > 1)
__global__ void k_adv_mean(AdvArgs a) {
  const int mb = blockIdx.x * blockDim.x + threadIdx.x;
  if (mb >= a.nmb) return;
  double t = 0.0;
  for (int sl = 0; sl < PPO_ADV_SPLIT; ++sl) t += a.part[mb * PPO_ADV_SPLIT + sl];
  a.stats[2 * mb + 0] = (float)(t / a.M);
}
// pass 2: slice sums of (adv - mean)^2 with the (global) mean
__global__ __launch_bounds__(256) void k_adv_sq(AdvArgs a) {
  __shared__ double red[4];
  const int mb = blockIdx.x, sl = blockIdx.y;
  const int len = (a.M + PPO_ADV_SPLIT - 1) / PPO_ADV_SPLIT;
  const int i0 = sl * len, i1 = min(a.M, i0 + len);
  const int32_t* perm = a.perm + (long)mb * a.M;
  const float mu = a.stats[2 * mb + 0];
  double s = 0.0;
  for (int i = i0 + threadIdx.x; i < i1; i += 256) {
    const double d = (double)(a.adv[perm[i]] - mu);
    s += d * d;
  }
  const double t = block_sum_d(s, red);
  if (threadIdx.x == 0) a.part[mb * PPO_ADV_SPLIT + sl] = t;
}
// -> sq[mb] = local sum of squares (all-reduced with ncclSum when G > 1); with_std: also the std
__global__ void k_adv_sqsum(AdvArgs a, int with_std) {
  const int mb = blockIdx.x * blockDim.x + threadIdx.x;
  if (mb >= a.nmb) return;
  double t = 0.0;
  for (int sl = 0; sl < PPO_ADV_SPLIT; ++sl) t += a.part[mb * PPO_ADV_SPLIT + sl];
  a.sq[mb] = (float)t;
  if (with_std) a.stats[2 * mb + 1] = sqrtf((float)((double)a.sq[mb] / (double)(a.world * (long)a.M - 1)));
}
// std = sqrt(sum_sq_global / (G * M - 1))  (ac:845-846; ppo's Tensor::std() for G = 1)
__global__ void k_adv_finalize(AdvArgs a) {
  const int mb = blockIdx.x * blockDim.x + threadIdx.x;
  if (mb < a.nmb) a.stats[2 * mb + 1] = sqrtf((float)((double)a.sq[mb] / (double)(a.world * (long)a.M - 1)));
}

// =============================================================================================
// synthetic device env (SeqVectorEnv + RecordEpisodeStatistics semantics; bit-identical to the
// host SyntheticCheetah and the oracle)
// =============================================================================================
// ---------------------------------------------------------------------------------------------
// PPO env wrapper chain (ppo:41-49) on the device, one state per env. Same fp32 operations, in the
// same order, as gymcpp/wrappers.h and the oracle (orc_vwrap_*): no contraction, IEEE division and
// square root, so the chain is bit-exact against both.
// ---------------------------------------------------------------------------------------------
// The chain as its own pass over envs [e0, e1) of a vector env's output (pwrap_step / pwrap_reset):
// one wave per env, lanes over the observation. is_reset[e] != 0 marks the next-step autoreset
// (gym.h:141-149: the reward, 0, bypasses NormalizeReward); reward == nullptr: observations only.
__global__ __launch_bounds__(256) void k_wrap_step(WrapArgs w, int O, int e0, int e1, float* __restrict__ obs,
                                                   float* __restrict__ reward, const float* __restrict__ term,
                                                   const float* __restrict__ is_reset) {
  const int lane = threadIdx.x & 63;
  const int e = e0 + blockIdx.x * 4 + (threadIdx.x >> 6);
  if (e >= e1) return;  // uniform per wave
  const float oc = w.ocount[e];
  for (int i = lane; i < O; i += 64) obs[(long)e * O + i] = wrap_obs_dim(w, e, O, i, oc, obs[(long)e * O + i]);
  if (lane != 0) return;
  w.ocount[e] = oc + 1.0f;
  if (reward && !(is_reset && is_reset[e] != 0.0f)) reward[e] = wrap_reward(w, e, reward[e], term ? term[e] : 0.0f);
}

PPO_DEV void synth_reset_one(SynthArgs& a, int e, int seed, float* obs) {
#pragma clang fp contract(off)
  if (seed > 0) { a.rseed[e] = (uint32_t)seed; a.rcount[e] = 0; }
  const uint32_t rs = a.rseed[e], rc = a.rcount[e];
  const float oc = a.w.on ? a.w.ocount[e] : 0.0f;
  for (int i = 0; i < a.O; ++i) {
    uint32_t r[4];
    philox4x32(rc, (uint32_t)i, 0u, 0u, rs, 0x5EED5EEDu, r);
    const float q = (0.1f * ((2.0f * u01(r[0])) - 1.0f));
    a.q[(long)e * a.O + i] = q;
    obs[(long)e * a.O + i] = a.w.on ? wrap_obs_dim(a.w, e, a.O, i, oc, q) : q;
  }
  if (a.w.on) a.w.ocount[e] = oc + 1.0f;
  a.rcount[e] = rc + 1;
  a.t[e] = 0;
  a.ep_ret[e] = 0.0f;
  a.ep_len[e] = 0;
}

__global__ __launch_bounds__(256) void k_synth_reset(SynthArgs a, int seed, float* obs, float* done) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.E) return;
  synth_reset_one(a, e, seed + e, obs);
  a.autoreset[e] = 0;
  if (done) done[e] = 0.0f;
}

// One thread per (env, observation dim): 32 lanes per env (2 envs per wave), q_(i+1) comes from the
// neighbouring lane, so all reads of the old state happen before any write; lane 0 of each env does
// the per-env reward / time limit / episode statistics. Same fp32 ops as synth_reset_one and the
// oracle (no contraction): bit-exact.
__global__ __launch_bounds__(256) void k_synth_step(SynthArgs a, int e0, int e1, const float* __restrict__ act,
                                                    float lo, float hi, float* __restrict__ obs,
                                                    float* __restrict__ reward, float* __restrict__ done) {
#pragma clang fp contract(off)
  const int i = threadIdx.x & 31;
  const int e = e0 + blockIdx.x * 8 + (threadIdx.x >> 5);
  const bool live = e < e1;
  const int O = a.O, A = a.A;
  const int ec = live ? e : e0;
  const bool reset = a.autoreset[ec] != 0;
  float* __restrict__ q = a.q + (long)ec * O;
  const float* __restrict__ ar = act + (long)(ec - e0) * A;
  const float qi = (live && i < O) ? q[i] : 0.0f;
  // old q_(i+1 mod O) from the neighbouring lane (lane - i is this env's i = 0)
  const int lane = threadIdx.x & 63;
  const float qn = __shfl(qi, (i + 1 < O) ? lane + 1 : lane - i, 64);
  if (!live || i >= O) return;
  const float oc = a.w.on ? a.w.ocount[e] : 0.0f;  // read by every lane before lane 0 stores oc + 1
  if (reset) {
    const uint32_t rs = a.rseed[e], rc = a.rcount[e];
    uint32_t r[4];
    philox4x32(rc, (uint32_t)i, 0u, 0u, rs, 0x5EED5EEDu, r);
    const float v = (0.1f * ((2.0f * u01(r[0])) - 1.0f));
    q[i] = v;
    obs[(long)e * O + i] = a.w.on ? wrap_obs_dim(a.w, e, O, i, oc, v) : v;
    if (i == 0) {
      if (a.w.on) a.w.ocount[e] = oc + 1.0f;
      a.rcount[e] = rc + 1;
      a.t[e] = 0;
      a.ep_ret[e] = 0.0f;
      a.ep_len[e] = 0;
      reward[e] = 0.0f;
      done[e] = 0.0f;
      a.autoreset[e] = 0;
    }
    return;
  }
  // q'_i = 0.9 q_i + (0.1 a_(i mod A) + 0.05 q_(i+1 mod O))  (fmaf, no contraction)
  const float ai = fminf(fmaxf(ar[i % A], lo), hi);
  const float nq = __fmaf_rn(0.9f, qi, __fmaf_rn(0.1f, ai, (0.05f * qn)));
  q[i] = nq;
  obs[(long)e * O + i] = a.w.on ? wrap_obs_dim(a.w, e, O, i, oc, nq) : nq;
  if (i != 0) return;
  if (a.w.on) a.w.ocount[e] = oc + 1.0f;
  const float vel = ((nq - qi) / 0.05f);
  float ctrl = 0.0f;
  for (int k = 0; k < A; ++k) {
    const float ak = fminf(fmaxf(ar[k], lo), hi);
    ctrl = (ctrl + ((0.1f * ak) * ak));
  }
  const float r = (vel - ctrl);
  const int t = a.t[e] + 1;
  a.t[e] = t;
  const bool tr = t >= 1000;
  reward[e] = a.w.on ? wrap_reward(a.w, e, r, 0.0f) : r;  // the synthetic env never terminates
  done[e] = tr ? 1.0f : 0.0f;
  a.ep_ret[e] = (a.ep_ret[e] + r);
  a.ep_len[e] += 1;
  if (tr) {
    a.fin_ret[e] += a.ep_ret[e];
    a.fin_len[e] += (float)a.ep_len[e];
    a.fin_cnt[e] += 1.0f;
  }
  a.autoreset[e] = tr ? 1 : 0;
}

// Wide observations (32 < O <= 64 * kSynthWideChunks, e.g. Ant 105, Humanoid 376): one wave per
// env, lane l holds dims l, l + 64, ...; every old q is in registers before any write, so the
// in-place update keeps the same semantics (and the same fp32 ops) as k_synth_step.
constexpr int kSynthWideChunks = 6;
__global__ __launch_bounds__(256) void k_synth_step_wide(SynthArgs a, int e0, int e1, const float* __restrict__ act,
                                                         float lo, float hi, float* __restrict__ obs,
                                                         float* __restrict__ reward, float* __restrict__ done) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const int e = e0 + blockIdx.x * 4 + (threadIdx.x >> 6);
  if (e >= e1) return;  // uniform per wave
  const int O = a.O, A = a.A;
  float* __restrict__ q = a.q + (long)e * O;
  const float* __restrict__ ar = act + (long)(e - e0) * A;
  float qv[kSynthWideChunks];
#pragma unroll
  for (int c = 0; c < kSynthWideChunks; ++c) {
    const int i = 64 * c + lane;
    qv[c] = q[i < O ? i : O - 1];
  }
  const bool reset = a.autoreset[e] != 0;
  const float oc = a.w.on ? a.w.ocount[e] : 0.0f;  // read by every lane before lane 0 stores oc + 1
  if (reset) {
    const uint32_t rs = a.rseed[e], rc = a.rcount[e];
#pragma unroll
    for (int c = 0; c < kSynthWideChunks; ++c) {
      const int i = 64 * c + lane;
      if (i < O) {
        uint32_t r[4];
        philox4x32(rc, (uint32_t)i, 0u, 0u, rs, 0x5EED5EEDu, r);
        const float v = (0.1f * ((2.0f * u01(r[0])) - 1.0f));
        q[i] = v;
        obs[(long)e * O + i] = a.w.on ? wrap_obs_dim(a.w, e, O, i, oc, v) : v;
      }
    }
    if (lane == 0) {
      if (a.w.on) a.w.ocount[e] = oc + 1.0f;
      a.rcount[e] = rc + 1;
      a.t[e] = 0;
      a.ep_ret[e] = 0.0f;
      a.ep_len[e] = 0;
      reward[e] = 0.0f;
      done[e] = 0.0f;
      a.autoreset[e] = 0;
    }
    return;
  }
  const float q0 = __shfl(qv[0], 0, 64);
  float q0_new = 0.0f, q0_old = 0.0f;
#pragma unroll
  for (int c = 0; c < kSynthWideChunks; ++c) {
    // old q_(i+1 mod O): the next lane, lane 0 of the next chunk, or q_0 for i = O - 1
    const float up = __shfl(qv[c], (lane + 1) & 63, 64);
    const float nxt = c + 1 < kSynthWideChunks ? __shfl(qv[c + 1 < kSynthWideChunks ? c + 1 : c], 0, 64) : 0.0f;
    const int i = 64 * c + lane;
    const float qn = (i + 1 == O) ? q0 : (lane < 63 ? up : nxt);
    if (i < O) {
      const float ai = fminf(fmaxf(ar[i % A], lo), hi);
      const float nq = __fmaf_rn(0.9f, qv[c], __fmaf_rn(0.1f, ai, (0.05f * qn)));
      q[i] = nq;
      obs[(long)e * O + i] = a.w.on ? wrap_obs_dim(a.w, e, O, i, oc, nq) : nq;
      if (i == 0) { q0_new = nq; q0_old = qv[c]; }
    }
  }
  if (lane != 0) return;
  if (a.w.on) a.w.ocount[e] = oc + 1.0f;
  const float vel = ((q0_new - q0_old) / 0.05f);
  float ctrl = 0.0f;
  for (int k = 0; k < A; ++k) {
    const float ak = fminf(fmaxf(ar[k], lo), hi);
    ctrl = (ctrl + ((0.1f * ak) * ak));
  }
  const float r = (vel - ctrl);
  const int t = a.t[e] + 1;
  a.t[e] = t;
  const bool tr = t >= 1000;
  reward[e] = a.w.on ? wrap_reward(a.w, e, r, 0.0f) : r;  // the synthetic env never terminates
  done[e] = tr ? 1.0f : 0.0f;
  a.ep_ret[e] = (a.ep_ret[e] + r);
  a.ep_len[e] += 1;
  if (tr) {
    a.fin_ret[e] += a.ep_ret[e];
    a.fin_len[e] += (float)a.ep_len[e];
    a.fin_cnt[e] += 1.0f;
  }
  a.autoreset[e] = tr ? 1 : 0;
}

// =============================================================================================
// explicit instantiations / launch wrappers
// =============================================================================================
// supported (H, kind, OP/16) instantiations: AC agent H=256, PPO agent H=64; inputs up to 384
template <typename F>
static int dispatch_net(const PackedLayout& K, F&& f) {
  const int nto = K.OP / 16;
#define PPO_NET_CASE(H_, KIND_, NTO_) \
  if (K.H == H_ && K.kind == KIND_ && nto == NTO_) return f(std::integral_constant<int, H_>{}, std::integral_constant<int, KIND_>{}, std::integral_constant<int, NTO_>{});
  PPO_NET_CASE(256, PPO_NET_LN_BETA, 1) PPO_NET_CASE(256, PPO_NET_LN_BETA, 2) PPO_NET_CASE(256, PPO_NET_LN_BETA, 7)
  PPO_NET_CASE(256, PPO_NET_LN_BETA, 24) PPO_NET_CASE(64, PPO_NET_TANH_NORMAL, 1) PPO_NET_CASE(64, PPO_NET_TANH_NORMAL, 2)
  PPO_NET_CASE(64, PPO_NET_TANH_NORMAL, 7) PPO_NET_CASE(64, PPO_NET_TANH_NORMAL, 24) PPO_NET_CASE(64, PPO_NET_LN_BETA, 2)
  PPO_NET_CASE(256, PPO_NET_TANH_NORMAL, 2)
#undef PPO_NET_CASE
  return -1;
}

int launch_act(const ActArgs& a, hipStream_t s) {
  if (launch_act3(a, s) == 0) return 0;  // 256-wide agents (ppo_act.hip)
  if ((a.kernel & 0xFF) != 2 && launch_act4(a, s) == 0) return 0;  // 64-wide tanh agent (ppo_act_narrow.hip)
  return dispatch_net(a.K, [&](auto H_, auto KIND_, auto NTO_) {
    constexpr int H = decltype(H_)::value, KIND = decltype(KIND_)::value, NTO = decltype(NTO_)::value;
    if (a.K.A > 20) return -1;
    // 16 rows per workgroup unless that still leaves > 2 workgroups per CU (then 32)
#ifdef PPO_DIAG
    static const int force_rg = [] { const char* e = getenv("PPO_ACT_RG"); return e ? atoi(e) : 0; }();
#else
    constexpr int force_rg = 0;
#endif
    if (force_rg == 1 || (force_rg == 0 && (a.n + 15) / 16 <= 512)) {
      dim3 grid((a.n + 15) / 16, a.need_actor ? 2 : 1);
      hipLaunchKernelGGL((k_act2<H, KIND, NTO, 1>), grid, dim3(256), 0, s, a);
    } else {
      dim3 grid((a.n + 31) / 32, a.need_actor ? 2 : 1);
      hipLaunchKernelGGL((k_act2<H, KIND, NTO, 2>), grid, dim3(256), 0, s, a);
    }
    return 0;
  });
}

int launch_act_wave(const ActArgs& a, hipStream_t s) {
  dim3 grid((a.n + 15) / 16, a.need_actor ? 2 : 1);
  return dispatch_net(a.K, [&](auto H_, auto KIND_, auto NTO_) {
    hipLaunchKernelGGL((k_act<decltype(H_)::value, decltype(KIND_)::value, decltype(NTO_)::value>), grid, dim3(64), 0,
                       s, a);
    return 0;
  });
}

int launch_fwdbwd(const UpdArgs& a, int nblocks, size_t lds_bytes, hipStream_t s) {
  dim3 grid(nblocks, 2);
  return dispatch_net(a.K, [&](auto H_, auto KIND_, auto NTO_) {
    hipLaunchKernelGGL((k_fwdbwd<decltype(H_)::value, decltype(KIND_)::value, decltype(NTO_)::value>), grid,
                       dim3(256), lds_bytes, s, a);
    return 0;
  });
}

int fwdbwd_set_lds(const PackedLayout& K, size_t lds_bytes) {
  return dispatch_net(K, [&](auto H_, auto KIND_, auto NTO_) {
    return hipFuncSetAttribute(
               (const void*)k_fwdbwd<decltype(H_)::value, decltype(KIND_)::value, decltype(NTO_)::value>,
               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes) == hipSuccess
               ? 0
               : -2;
  });
}

// dW of both Linear weight matrices of both trunks, grid = (chunks, 2 trunks)
template <int H, int OP>
static int launch_dw_t(const DwArgs& a, int nchunks, size_t lds, hipStream_t s) {
  auto k = k_dw<H, OP>;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return -2;
    attr = true;
  }
  hipLaunchKernelGGL(k, dim3(nchunks, 2), dim3(512), lds, s, a);
  return 0;
}

size_t dw_lds_bytes(int H, int OP) {
  const int KS = 16;
  const int m = std::max(H, OP) + 4;
  return (size_t)2 * (KS * (H + 4) + KS * m) * sizeof(float);
}

template <int H, int OP, int NSL>
static int launch_dwf_t(const DwArgs& a0, int nchunks, hipStream_t s) {
  DwArgs a = a0;
#ifdef PPO_DIAG
  static const int hot = [] { const char* e = getenv("PPO_DW_HOT"); return e ? atoi(e) : 0; }();
  a.hot = hot;
#endif
  // the DMA kernels address their sources through 32-bit buffer descriptors (make_pbuf: int floats)
  if (a.bx && (long)a.M * H < (1L << 29)) {
    const bool rc = a.h1_recompute != 0;
    auto k = rc ? (a.bx == 9 ? k_dwf_bx<H, OP, NSL, 9, true> : a.bx == 8 ? k_dwf_bx<H, OP, NSL, 8, true>
                                                              : k_dwf_bx<H, OP, NSL, 6, true>)
                : (a.bx == 9 ? k_dwf_bx<H, OP, NSL, 9> : a.bx == 8 ? k_dwf_bx<H, OP, NSL, 8> : k_dwf_bx<H, OP, NSL, 6>);
    const size_t lds = (size_t)(rc ? DwbxGeo<H, OP, true>::total : DwbxGeo<H, OP, false>::total) * sizeof(float);
    static_assert(DwbxGeo<H, OP, true>::total * sizeof(float) <= 160 * 1024, "k_dwf_bx (H1 recompute) LDS");
    static bool attr[6] = {false, false, false, false, false, false};
    const int ai = (a.bx == 9 ? 2 : a.bx == 8 ? 1 : 0) + (rc ? 3 : 0);
    if (!attr[ai]) {
      if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return -2;
      attr[ai] = true;
    }
    hipLaunchKernelGGL(k, dim3(nchunks, 2, NSL), dim3(512), lds, s, a);
    return 0;
  }
  if (a.dma && (long)a.M * H < (1L << 29)) {
    auto k = k_dwf_dma<H, OP, NSL>;
    constexpr size_t lds = (size_t)3 * (3 * 16 * H + 16 * OP) * sizeof(float);
    static bool attr = false;
    if (!attr) {
      if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return -2;
      attr = true;
    }
    hipLaunchKernelGGL(k, dim3(nchunks, 2, NSL), dim3(512), lds, s, a);
    return 0;
  }
  auto k = k_dwf<H, OP, NSL>;
  constexpr size_t lds = (size_t)2 * (3 * 16 * (H + 4) + 16 * (OP + 4)) * sizeof(float);
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return -2;
    attr = true;
  }
  hipLaunchKernelGGL(k, dim3(nchunks, 2, NSL), dim3(512), lds, s, a);
  return 0;
}

// k_dw_dma: the stage buffers of the larger phase, three of them
template <int H, int OP>
static int launch_dw_dma_t(const DwArgs& a, int nchunks, hipStream_t s) {
  auto k = a.bx == 6 ? k_dw_dma<H, OP, 6> : a.bx == 8 ? k_dw_dma<H, OP, 8> : a.bx == 9 ? k_dw_dma<H, OP, 9> : k_dw_dma<H, OP, 0>;
  constexpr int big = H > OP ? H : OP;
  constexpr size_t lds = (size_t)3 * 16 * (H + big) * sizeof(float);
  static bool attr[10] = {};
  const int ai = a.bx >= 0 && a.bx < 10 ? a.bx : 0;
  if (!attr[ai]) {
    if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return -2;
    attr[ai] = true;
  }
  hipLaunchKernelGGL(k, dim3(nchunks, 2), dim3(512), lds, s, a);
  return 0;
}

int launch_dw(const DwArgs& a, int H, int OP, int nchunks, hipStream_t s) {
  if (H == 256 && a.fused) {  // a.fused = 0: the two-phase k_dw (PPO_DW_FUSED=0 at ppo_create)
    if (OP == 16) return a.slices == 2 ? launch_dwf_t<256, 16, 2>(a, nchunks, s) : launch_dwf_t<256, 16, 1>(a, nchunks, s);
    if (OP == 32) return a.slices == 2 ? launch_dwf_t<256, 32, 2>(a, nchunks, s) : launch_dwf_t<256, 32, 1>(a, nchunks, s);
  }
  if (a.dma && !a.perm && H == 256 && OP == 112 && (long)a.M * H < (1L << 29))  // Ant (cfg4); 32-bit descriptors
    return launch_dw_dma_t<256, 112>(a, nchunks, s);
  const size_t lds = dw_lds_bytes(H, OP);
  if (H == 256 && OP == 16) return launch_dw_t<256, 16>(a, nchunks, lds, s);
  if (H == 256 && OP == 32) return launch_dw_t<256, 32>(a, nchunks, lds, s);
  if (H == 256 && OP == 112) return launch_dw_t<256, 112>(a, nchunks, lds, s);
  if (H == 256 && OP == 384) return launch_dw_t<256, 384>(a, nchunks, lds, s);
  if (H == 64 && OP == 16) return launch_dw_t<64, 16>(a, nchunks, lds, s);
  if (H == 64 && OP == 32) return launch_dw_t<64, 32>(a, nchunks, lds, s);
  if (H == 64 && OP == 112) return launch_dw_t<64, 112>(a, nchunks, lds, s);
  if (H == 64 && OP == 384) return launch_dw_t<64, 384>(a, nchunks, lds, s);
  return -1;
}

void launch_colsum(const ColsumArgs& a_in, int nseg, long maxlen, hipStream_t s) {
  (void)maxlen;
  ColsumArgs a = a_in;
  a.nseg = nseg;
  int t = 0;
  for (int i = 0; i < nseg; ++i) {
    a.tile0[i] = t;
    t += (a.seg[i].len + 63) / 64;
  }
  a.tile0[nseg] = t;
  hipLaunchKernelGGL(k_colsum, dim3((unsigned)t), dim3(256), 0, s, a);
}
void launch_gradnorm(const NormArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_gradnorm, dim3(a.nt, PPO_GN_SPLIT), dim3(256), 0, s, a);
}
int launch_gradstep(const NormArgs& na, const AdamArgs& a, unsigned* bar, unsigned* count, hipStream_t s) {
  const unsigned g = (unsigned)std::max<long>((a.n + 255) / 256, (long)na.nt * PPO_GN_SPLIT);
  unsigned target = *count + g;
  NormArgs n2 = na;
  AdamArgs a2 = a;
  void* args[] = {&n2, &a2, &bar, &target};
  if (hipLaunchCooperativeKernel((const void*)k_gradstep, dim3(g), dim3(256), args, 0, s) != hipSuccess) return -2;
  *count = target;
  return 0;
}
void launch_adam(const AdamArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_adam, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, s, a);
}
void launch_transpose(const float* src, float* dst, int H, hipStream_t s) {
  hipLaunchKernelGGL(k_transpose, dim3((H * H + 255) / 256), dim3(256), 0, s, src, dst, H);
}
void launch_swizzle(const float* w1, const float* w2, float* dst, int H, int OP, int bx, hipStream_t s) {
  const long n = (long)H * OP + (long)H * H;
  hipLaunchKernelGGL(k_swizzle, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, w1, w2, dst, H, OP, bx);
}
void launch_gae(const GaeArgs& a, hipStream_t s, bool scan) {
  if (scan) hipLaunchKernelGGL(k_gae_scan, dim3((a.E + 63) / 64), dim3(1024), 0, s, a);
  else hipLaunchKernelGGL(k_gae, dim3((a.E + 63) / 64), dim3(64), 0, s, a);
}
void launch_perm(int32_t* out, uint32_t B, const PermKey& pk, hipStream_t s) {
  hipLaunchKernelGGL(k_perm, dim3((B + 255) / 256), dim3(256), 0, s, out, B, pk);
}
static unsigned nmb_blocks(int nmb) { return (unsigned)((nmb + 255) / 256); }
void launch_adv_sum(const AdvArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_adv_sum, dim3(a.nmb, PPO_ADV_SPLIT), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_adv_mean, dim3(nmb_blocks(a.nmb)), dim3(256), 0, s, a);
}
void launch_adv_sq(const AdvArgs& a, int with_std, hipStream_t s) {
  hipLaunchKernelGGL(k_adv_sq, dim3(a.nmb, PPO_ADV_SPLIT), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_adv_sqsum, dim3(nmb_blocks(a.nmb)), dim3(256), 0, s, a, with_std);
}
void launch_adv_finalize(const AdvArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_adv_finalize, dim3(nmb_blocks(a.nmb)), dim3(256), 0, s, a);
}
void launch_wrap_step(const WrapArgs& w, int O, int e0, int e1, float* obs, float* reward, const float* term,
                      const float* is_reset, hipStream_t s) {
  hipLaunchKernelGGL(k_wrap_step, dim3((e1 - e0 + 3) / 4), dim3(256), 0, s, w, O, e0, e1, obs, reward, term, is_reset);
}
void launch_synth_reset(const SynthArgs& a, int seed, float* obs, float* done, hipStream_t s) {
  hipLaunchKernelGGL(k_synth_reset, dim3((a.E + 255) / 256), dim3(256), 0, s, a, seed, obs, done);
}
void launch_synth_step(const SynthArgs& a, int e0, int e1, const float* act, float lo, float hi, float* obs,
                       float* reward, float* done, hipStream_t s) {
  if (a.O > 32) {
    hipLaunchKernelGGL(k_synth_step_wide, dim3((e1 - e0 + 3) / 4), dim3(256), 0, s, a, e0, e1, act, lo, hi, obs,
                       reward, done);
    return;
  }
  hipLaunchKernelGGL(k_synth_step, dim3((e1 - e0 + 7) / 8), dim3(256), 0, s, a, e0, e1, act, lo, hi, obs, reward,
                     done);
}
