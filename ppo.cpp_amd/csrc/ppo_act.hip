// ppo_act.hip — k_act3: Agent::get_action_and_value / get_value + rollout stores for the 256-wide
// agents (ac:212-249, :649-660; ppo:145-157, :387-400), latency-first.
//
// A rollout step is a single pass over E rows, so every launch starts with cold weights (the
// per-XCD L2 is not kept across kernel boundaries): the time of one launch is one workgroup's
// critical path of ~1 us memory round trips, not its MFMA work. The layout below removes the
// serial round trips instead of adding parallel work:
//  * 16 rows x 8 waves per workgroup; wave w owns output features [32 w, 32 w + 32) (2 MFMA tiles);
//  * every small parameter the workgroup needs later (biases, LayerNorm affine, head weights and
//    biases) is fetched at kernel start, in the same latency window as the inputs and W1, and
//    parked in LDS;
//  * the 256 x 256 layer streams its weight A-operands through an 8-deep register ring (8 of the
//    16 k-blocks in flight), so the layer costs ~2 round trips instead of 16;
//  * heads are MFMAs (split-K over the waves' features, partials reduced through LDS);
//  * Beta sampling runs one (row, action, alpha|beta) item per thread, so the two Marsaglia-Tsang
//    gamma draws and their lgamma/digamma chains run side by side.
// The per-(row, action) arithmetic and the Philox counters are the ones of k_act / k_act2, so
// samples are identical for any batching.
#include "ppo_act_common.hpp"

#include <cstdlib>

using namespace act;

template <int KIND, int NTO, int NHT, int RT>
__global__ __launch_bounds__(512) void k_act3(ActArgs a) {
  using GE = ActGeo<NTO, NHT, RT>;
  constexpr int H = 256, OP = GE::OP, NHP = GE::NHP, LDX = GE::LDX, LDH = GE::LDH, LDP = GE::LDP, R = GE::kActRows;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* XS = lds + GE::oXS;
  float* HB = lds + GE::oHB;
  float* SP = lds + GE::oSP;
  float* HBIAS = lds + GE::oHBIAS;
  float* RED = lds + GE::oRED;
  float* HP = lds + GE::oHP;
  float* PRE = lds + GE::oPRE;
  float* ITM = lds + GE::oITM;
  float* LPE = lds + GE::oLP;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  const int trunk = blockIdx.y;
  if (trunk == 1 && !a.need_actor) return;
  const PackedLayout& K = a.K;
  const TrunkDev& T = K.tr[trunk];
  const float* __restrict__ P = a.P;
  const PBuf pb = make_pbuf(P, K.size);
  const int row0 = blockIdx.x * R;
  const int O = K.O, A = K.A;
  const int nh = trunk == 0 ? 1 : (KIND == PPO_NET_LN_BETA ? 2 * A : A);

  // ---- kernel start: issue every independent load (inputs, W1 ring, staged params) ----
  // Branch-free: clamped addresses with the value masked afterwards, or buffer loads whose
  // offset is past the descriptor's end (they return 0). A load under a per-lane branch gets its
  // own s_waitcnt vmcnt(0), which serialises the prologue into several memory round trips.
  constexpr int NX = (R * OP + kActThreads - 1) / kActThreads;
  float xv[NX];
#pragma unroll
  for (int k = 0; k < NX; ++k) {
    const int idx = tid + kActThreads * k, r = idx / OP, f = idx - r * OP, row = row0 + r;
    const float v = a.x[(size_t)min(row, a.n - 1) * a.ldx + min(f, O - 1)];
    xv[k] = (idx < R * OP && row < a.n && f < O) ? v : 0.0f;
  }
  constexpr int NSP4 = GE::NSP / 4;
  constexpr int NSPT = (NSP4 + kActThreads - 1) / kActThreads;
  f4 spv[NSPT];
#pragma unroll
  for (int k = 0; k < NSPT; ++k) {
    const int q = tid + kActThreads * k;  // f4 index into SP
    f4 v = f4{0.f, 0.f, 0.f, 0.f};
    if (q < NSP4) {
      // q / 64 is the wave index plus 8 k: wave-uniform, so the source selection is scalar
      const int fl = 4 * q, vec = __builtin_amdgcn_readfirstlane(fl / H), off = fl - vec * H;
      int src = -1;
      if (vec < 6) {
        const int base = vec == 0 ? T.b1 : vec == 1 ? T.g1 : vec == 2 ? T.be1 : vec == 3 ? T.b2 : vec == 4 ? T.g2 : T.be2;
        src = base >= 0 ? base + off : -1;
      } else {
        const int hr = act_head_row(K, trunk, vec - 6);
        src = hr >= 0 ? hr + off : -1;
      }
      v = pld4(pb, src >= 0 ? src : K.size, 0);  // past the end: 0
    }
    spv[k] = v;
  }
  const int hbo = tid < NHP ? act_head_bias(K, trunk, tid) : -1;
  const float hbias = bld1f(pb, hbo >= 0 ? hbo : K.size);
  float ndone = 0.f;  // the critic stores next_done with the value (rollout)
  if (trunk == 0 && a.store_step >= 0 && a.next_done) ndone = a.next_done[min(row0 + (tid & (R - 1)), a.n - 1)];
  // the sampling draws of this thread's first distribution item do not depend on the network:
  // computed here, under the weight fetch (Beta: Marsaglia-Tsang attempt 0; Normal: the z pair)
  const SampleKey key = sample_key(a.seed, a.rank);
  GammaDraw gd0 = GammaDraw{0.f, 0.f};
  float nz0 = 0.f;
  if (trunk == 1 && a.mode == PPO_SAMPLE) {
    if constexpr (KIND == PPO_NET_LN_BETA) {
      if (tid < R * A * 2) {
        const int which = tid & 1, ra = tid >> 1, r = ra / A, ai = ra - r * A;
        gd0 = gamma_draw(key, a.env_base + row0 + r, a.step_id, 0x10000u + (uint32_t)(ai * 2 + which) * 64u);
      }
    } else {
      if (tid < R * A) {
        const int r = tid / A, ai = tid - r * A;
        uint32_t rr[4];
        philox_draw(key, a.env_base + row0 + r, a.step_id, (uint32_t)(ai >> 1), rr);
        float z0, z1;
        box_muller(rr[0], rr[1], z0, z1);
        nz0 = (ai & 1) ? z1 : z0;
      }
    }
  }
  // ---- inputs -> LDS (normalized for the LN agent); the raw rows into the rollout storage ----
#pragma unroll
  for (int k = 0; k < NX; ++k) {
    const int idx = tid + kActThreads * k, r = idx / OP, f = idx - r * OP;
    if (trunk == 0 && a.store_step >= 0 && idx < R * OP && row0 + r < a.n && f < O)
      a.s_obs[((long)a.store_step * a.E + a.env_base + row0 + r) * O + f] = xv[k];
    if (idx < R * OP) {
      float v = xv[k];
      if constexpr (KIND == PPO_NET_LN_BETA)
        if (row0 + r < a.n && f < O) v = (v - P[K.omean + f]) / P[K.ostd + f];
      XS[r * LDX + f] = v;
    }
  }
  if (trunk == 0 && a.skip_critic) {
    // the rollout's critic pass is deferred (ppo_compute_gae / ppo_rollout_values: one batched critic
    // launch over the stored rows, the persistent rollout's k_vbx): store next_done with the rows only
    if (tid < R && a.store_step >= 0 && row0 + tid < a.n)
      a.s_dones[(long)a.store_step * a.E + a.env_base + row0 + tid] = ndone;
    return;
  }
  lds_barrier();
  // ---- layer 1 ----
  f4 acc[2][RT];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const f4 bv = pld4(pb, T.b1 + 32 * wave + 16 * u + 4 * g, 0);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[u][rt] = bv;
  }
  const float* xin = XS + j * LDX + 4 * g;
  const PBuf wsw = make_pbuf(a.WSW[trunk], (int)sw_size(H, OP));
  act_layer<NTO, 8, RT>(acc, wsw, ((2 * wave) * NTO * 64 + lane) * 4,
                            [&](int t, int rt) { return *reinterpret_cast<const f4*>(xin + 16 * rt * LDX + 16 * t); });
  // staged params land in LDS (visible after the next barrier)
#pragma unroll
  for (int k = 0; k < NSPT; ++k) {
    const int q = tid + kActThreads * k;
    if (q < NSP4) *reinterpret_cast<f4*>(SP + 4 * q) = spv[k];
  }
  if (tid < NHP) HBIAS[tid] = hbias;
  act_activate<KIND, RT>(acc, SP + GE::sG1, SP + GE::sBE1, RED, wave, j, g);
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
      *reinterpret_cast<f4*>(HB + (16 * rt + j) * LDH + 32 * wave + 16 * u + 4 * g) = acc[u][rt];
  lds_barrier();
  // ---- layer 2 ----
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const f4 bv = *reinterpret_cast<const f4*>(SP + GE::sB2 + 32 * wave + 16 * u + 4 * g);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[u][rt] = bv;
  }
  const float* hin = HB + j * LDH + 4 * g;
#ifdef PPO_STAMPS
  // diagnostic build only: a.kernel bit 8 skips layer 2 (h2 := h1), bit 9 the layer-2 LayerNorm
  const int diag = a.kernel >> 8;
  if (!(diag & 1))
#endif
  act_layer<16, 8, RT>(acc, wsw, H * OP + ((2 * wave) * 16 * 64 + lane) * 4,
                          [&](int t, int rt) { return *reinterpret_cast<const f4*>(hin + 16 * rt * LDH + 16 * t); });
#ifdef PPO_STAMPS
  if (!(diag & 2))
#endif
  act_activate<KIND, RT>(acc, SP + GE::sG2, SP + GE::sBE2, RED, wave, j, g);
  // ---- heads: split-K partials over this wave's 32 features ----
#pragma unroll
  for (int ht = 0; ht < NHT; ++ht) {
    f4 hp[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) hp[rt] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const f4 wv = *reinterpret_cast<const f4*>(SP + GE::sW3 + (16 * ht + j) * H + 32 * wave + 16 * u + 4 * g);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        hp[rt] = mfma16(wv.x, acc[u][rt].x, hp[rt]);
        hp[rt] = mfma16(wv.y, acc[u][rt].y, hp[rt]);
        hp[rt] = mfma16(wv.z, acc[u][rt].z, hp[rt]);
        hp[rt] = mfma16(wv.w, acc[u][rt].w, hp[rt]);
      }
    }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) HP[(wave * NHP + 16 * ht + 4 * g + r) * R + 16 * rt + j] = hp[rt][r];
  }
  lds_barrier();
  for (int idx = tid; idx < R * nh; idx += kActThreads) {
    const int r = idx / nh, h = idx - r * nh;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < kActWaves; ++w) s += HP[(w * NHP + h) * R + r];
    PRE[r * LDP + h] = s + HBIAS[h];
  }
  lds_barrier();

  if (trunk == 0) {
    if (tid < R) {
      const int row = row0 + tid;
      if (row < a.n) {
        const float v = PRE[tid * LDP];
        if (a.value_out) a.value_out[row] = v;
        if (a.store_step >= 0) {
          const long srow = (long)a.store_step * a.E + a.env_base + row;
          a.s_values[srow] = v;
          a.s_dones[srow] = ndone;
        }
      }
    }
    return;
  }

  // ---- actor distribution ----
#ifdef PPO_STAMPS
  if (diag & 4) {  // diagnostic: skip the distribution, write the head pre-activations
    if (tid < R * A) {
      const int r = tid / A, ai = tid - r * A;
      if (row0 + r < a.n && a.action_out) a.action_out[(size_t)(row0 + r) * A + ai] = PRE[r * LDP + ai];
    }
    return;
  }
#endif
  if constexpr (KIND == PPO_NET_LN_BETA) {
    // stage 1: one (row, action, alpha|beta) item per thread
    for (int idx = tid; idx < R * A * 2; idx += kActThreads) {
      const int which = idx & 1, ra = idx >> 1, r = ra / A, ai = ra - r * A;
      const long env = a.env_base + row0 + r;
      const float c = softplusf_(PRE[r * LDP + ai + which * A]) + 1.0f;
      float gs = 0.f;
      if (a.mode == PPO_SAMPLE) {
        const uint32_t db = 0x10000u + (uint32_t)(ai * 2 + which) * 64u;
        gs = idx == tid ? gamma_mt_d0(c, gd0, key, env, a.step_id, db) : gamma_mt(c, key, env, a.step_id, db);
      }
      float* it = ITM + ((r * A + ai) * 2 + which) * 4;
      it[0] = c;
      it[1] = gs;
      float tg_unused;
      lgamma_digamma_trigamma(c, it[2], it[3], tg_unused);
    }
    lds_barrier();
    // stage 2: combine per (row, action)
    for (int idx = tid; idx < R * A; idx += kActThreads) {
      const int r = idx / A, ai = idx - r * A, row = row0 + r;
      const long env = a.env_base + row;
      const bool valid = row < a.n;
      const float* ia = ITM + (idx * 2 + 0) * 4;
      const float* ib = ITM + (idx * 2 + 1) * 4;
      const float al = ia[0], be = ib[0];
      const float hi = P[K.hi], lo = P[K.lo];
      float sv;
      if (a.mode == PPO_GIVEN) {
        const float av = valid ? a.action_in[(size_t)row * A + ai] : 0.5f * (hi + lo);
        sv = (av - lo) / (hi - lo) * (1.0f - 0.0f) + 0.0f;
        sv = fminf(fmaxf(sv, 1e-7f), 1.0f + 1e-7f);
      } else if (a.mode == PPO_MEAN) {
        sv = al / (al + be);
      } else {
        sv = ia[1] / (ia[1] + ib[1]);
      }
      const float ab = al + be;
      float lgab, psab, tab_unused;
      lgamma_digamma_trigamma(ab, lgab, psab, tab_unused);
      const float lga = ia[2], lgb = ib[2];
      const float lp = xlogyf_(al - 1.0f, sv) + xlogyf_(be - 1.0f, 1.0f - sv) + (lgab - (lga + lgb));
      const float ent = (lga + lgb) - lgab - (2.0f - ab) * psab - ((al - 1.0f) * ia[3] + (be - 1.0f) * ib[3]);
      const float act = (sv - 0.0f) / (1.0f - 0.0f) * (hi - lo) + lo;
      LPE[idx * 2 + 0] = lp;
      LPE[idx * 2 + 1] = ent;
      if (valid) {
        if (a.action_out) a.action_out[(size_t)row * A + ai] = act;
        if (a.store_step >= 0) a.s_actions[((long)a.store_step * a.E + env) * A + ai] = act;
      }
    }
  } else {
    for (int idx = tid; idx < R * A; idx += kActThreads) {
      const int r = idx / A, ai = idx - r * A, row = row0 + r;
      const long env = a.env_base + row;
      const bool valid = row < a.n;
      const float mu = PRE[r * LDP + ai];
      const float sd = expf(P[K.logstd + ai]);
      const float var = sd * sd, lsd = logf(sd);
      float act;
      if (a.mode == PPO_GIVEN) {
        act = valid ? a.action_in[(size_t)row * A + ai] : 0.0f;
      } else if (a.mode == PPO_MEAN) {
        act = mu;
      } else {
        float z = nz0;
        if (idx != tid) {
          uint32_t rr[4];
          philox_draw(key, env, a.step_id, (uint32_t)(ai >> 1), rr);
          float z0, z1;
          box_muller(rr[0], rr[1], z0, z1);
          z = (ai & 1) ? z1 : z0;
        }
        act = mu + z * sd;
      }
      const float d = act - mu;
      LPE[idx * 2 + 0] = -(d * d) / (2.0f * var) - lsd - kLz;
      LPE[idx * 2 + 1] = kEntC + lsd;
      if (valid) {
        if (a.action_out) a.action_out[(size_t)row * A + ai] = act;
        if (a.store_step >= 0) a.s_actions[((long)a.store_step * a.E + env) * A + ai] = act;
      }
    }
  }
  lds_barrier();
  if (tid < R) {
    const int row = row0 + tid;
    if (row < a.n) {
      float lp = 0.f, ent = 0.f;
      for (int ai = 0; ai < A; ++ai) { lp += LPE[(tid * A + ai) * 2]; ent += LPE[(tid * A + ai) * 2 + 1]; }
      if (a.logprob_out) a.logprob_out[row] = lp;
      if (a.entropy_out) a.entropy_out[row] = ent;
      if (a.store_step >= 0) a.s_logp[(long)a.store_step * a.E + a.env_base + row] = lp;
    }
  }
}

template <int KIND, int NTO, int NHT, int RT>
static int launch_act3_rt(const ActArgs& a, hipStream_t s) {
  using GE = ActGeo<NTO, NHT, RT>;
  const size_t lds = (size_t)GE::total * sizeof(float);
  static const bool ok = hipFuncSetAttribute((const void*)k_act3<KIND, NTO, NHT, RT>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess;
  if (!ok) return -2;
  dim3 grid((a.n + GE::kActRows - 1) / GE::kActRows, a.need_actor ? 2 : 1);
  hipLaunchKernelGGL((k_act3<KIND, NTO, NHT, RT>), grid, dim3(kActThreads), lds, s, a);
  return 0;
}
// rows per workgroup: 16 at every E since the layer-2 weights stream in MFMA order (swizzled
// copies); before, wide batches used 32 rows to halve the per-row weight bytes. Measured at E = 4 096
// (rollout act): 19.4 us with 16 rows, 20.3 with 32, 32.7 with 64 (profiles/r02/act/act_rt_ab.txt)
template <int KIND, int NTO, int NHT>
static int launch_act3_t(const ActArgs& a, hipStream_t s) {
#ifdef PPO_DIAG
  static const int force = [] { const char* e = getenv("PPO_ACT_RT"); return e ? atoi(e) : 0; }();
  const int rt = force ? force : 1;
#else
  const int rt = 1;
#endif
  if (rt == 4) return launch_act3_rt<KIND, NTO, NHT, 4>(a, s);
  if (rt == 2) return launch_act3_rt<KIND, NTO, NHT, 2>(a, s);
  return launch_act3_rt<KIND, NTO, NHT, 1>(a, s);
}

// 256-wide agents; returns -1 when the shape is not covered (the caller falls back to k_act2)
int launch_act3(const ActArgs& a, hipStream_t s) {
#ifdef PPO_DIAG
  static const bool off = [] { const char* e = getenv("PPO_ACT3"); return e && e[0] == '0'; }();
  if (off) return -1;
#endif
  if (a.K.H != 256 || a.K.A > 24) return -1;
  const int nto = a.K.OP / 16;
  const int nh = a.K.kind == PPO_NET_LN_BETA ? 2 * a.K.A : a.K.A;
  const int nht = (nh + 15) / 16;
  if (a.K.kind == PPO_NET_LN_BETA) {
    if (nto == 1 && nht == 1) return launch_act3_t<PPO_NET_LN_BETA, 1, 1>(a, s);
    if (nto == 2 && nht == 1) return launch_act3_t<PPO_NET_LN_BETA, 2, 1>(a, s);
    if (nto == 7 && nht == 1) return launch_act3_t<PPO_NET_LN_BETA, 7, 1>(a, s);
    if (nto == 24 && nht == 3) return launch_act3_t<PPO_NET_LN_BETA, 24, 3>(a, s);
    if (nto == 2 && nht == 3) return launch_act3_t<PPO_NET_LN_BETA, 2, 3>(a, s);
  } else {
    if (nto == 2 && nht == 1) return launch_act3_t<PPO_NET_TANH_NORMAL, 2, 1>(a, s);
  }
  return -1;
}
