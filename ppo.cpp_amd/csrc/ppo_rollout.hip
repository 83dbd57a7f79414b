// ppo_rollout.hip — the device-env rollout as one persistent launch, and the critic as one pass
// over the stored observations (ppo:387-434, ac:641-698).
//
// A per-step rollout costs two launches per step (agent act, env step), each ~5 us of launch floor
// plus a cold 256 KB stream of W2 from L2 into every CU ("Why the act launches cost what
// they cost"). Here:
//  * k_rollout: one workgroup owns 16 envs for all T steps. The actor's W2 slice of each wave
//    (32 output features x 256 inputs, 128 VGPRs) and W1 slice stay in registers; obs -> actor ->
//    Beta sample -> action -> env step -> obs loops inside the kernel with LDS barriers only. The
//    critic is not on this chain: the value of step t depends only on obs[t], so it is computed
//    afterwards for all T x E stored rows at once (k_values).
//  * k_values: the critic forward of n stored rows; the critic's weights resident in registers
//    the same way, workgroups walk 32- / 64-row blocks.
//  * k_rollout_v (AC agent, E <= 512): 2 envs per workgroup on the VALU, each layer output one
//    fmaf chain in the MFMA's k order, so bitwise k_rollout's results.
//  * k_rollout4 / k_values4: the same for the 64-wide PPO agent (k_act4's arithmetic).
// They use the building blocks of k_act3 (ppo_act_common.hpp) in the same order: every action,
// log-prob, value, reward and observation is bitwise the one the per-step path produces
// (tests/test_gpu_rollout.py).
#include "ppo_act_common.hpp"
#include "ppo_wrap.hpp"

#include <type_traits>

using namespace act;

#ifdef PPO_STAMPS
// diagnostic build only: shader-clock stamps at the phase ends of the first 16 steps, wave 0 of
// workgroup 0 (k_rollout: 8 phases, k_rollout4: 8 phases); read with ppo_diag_read_roll_stamps
__device__ unsigned long long g_roll_stamps[16 * 8];
#define ROLL_STAMP(t, k)                                                                      \
  do {                                                                                        \
    if (blockIdx.x == 0 && threadIdx.x == 0 && (t) < 16)                                      \
      g_roll_stamps[(t) * 8 + (k)] = __builtin_amdgcn_s_memtime();                           \
  } while (0)
extern "C" int ppo_diag_read_roll_stamps(unsigned long long* host, long n) {
  if (n > 16 * 8) n = 16 * 8;
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_roll_stamps), n * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? (int)n : -2;
}
// intermediate values of one env (g_rdbg_env) at step 0: [0] k_rollout, [1] k_rollout_v; slots
// layer-1 out 0.., h1 260.., layer-2 out 516.., h2 776.., head partials [8][16] 1032.., pre 1160..
__device__ float g_rdbg[2][1280];
#define RDBG(k, i, v) (g_rdbg[k][i] = (v))
extern "C" int ppo_diag_read_rdbg(float* host) {
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_rdbg), sizeof(g_rdbg), 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}
constexpr int kRdbgEnv = 26;
#else
#define ROLL_STAMP(t, k) do {} while (0)
#endif

namespace {

constexpr int kRows = 16;  // envs (rows) per workgroup

template <int NTO, int NHT, int ROWS = kRows>
struct RollGeo {
  static constexpr int kRows = ROWS;  // rows per pass (16: the rollout's env block; 32: k_values)
  static constexpr int H = 256, OP = NTO * 16, NHP = 16 * NHT;
  static constexpr int LDX = ((OP + 63) / 64) * 64 + 4;
  static constexpr int LDH = H + 4;
  static constexpr int LDP = NHP + 4;
  static constexpr int LDQ = OP + 1;                           // env state / obs rows (O <= OP)
  static constexpr int NSP = 6 * H + NHP * H;
  static constexpr int oXS = 0;
  static constexpr int oHB = oXS + kRows * LDX;
  static constexpr int oSP = oHB + kRows * LDH;
  static constexpr int oHBIAS = oSP + NSP;
  static constexpr int oRED = oHBIAS + NHP;
  static constexpr int oHP = oRED + 2 * kActWaves * kRows;
  static constexpr int oPRE = oHP + kActWaves * NHP * kRows;
  static constexpr int oXO = oPRE + kRows * LDP;               // agent input obs of the current step
  static constexpr int oQ = oXO + kRows * LDQ;                 // env state q
  static constexpr int oNRM = oQ + kRows * LDQ;                // obs mean | std (OP each)
  static constexpr int oACT = oNRM + 2 * OP;                   // actions [16][24]
  static constexpr int oENV = oACT + kRows * 24;               // per-env scalars, 16 x 16
  static constexpr int total = oENV + 16 * kRows;
  // distribution scratch in the XS / HB region (dead after layer 2), as in k_act3
  static constexpr int oITM = 0;
  static constexpr int oLP = oITM + kRows * 24 * 2 * 4;
  static_assert(oLP + kRows * 24 * 2 <= oSP, "distribution scratch must fit in the XS/HB region");
  // staged param vectors inside SP (as ActGeo)
  static constexpr int sB1 = 0, sG1 = H, sBE1 = 2 * H, sB2 = 3 * H, sG2 = 4 * H, sBE2 = 5 * H, sW3 = 6 * H;
};

// per-env scalar slots in the oENV region
// (the wrapper chain's per-env scalars: obs count, return accumulator, reward mean / var / count)
enum { EV_DONE = 0, EV_AR, EV_T, EV_RSEED, EV_RCOUNT, EV_EPR, EV_EPL, EV_FR, EV_FL, EV_FC,
       EV_WOC, EV_WRA, EV_WRM, EV_WRV, EV_WRC, EV_NSLOT };

// staged small parameters of one trunk into LDS (biases, LayerNorm affine, head rows, head biases)
template <int NHP>
PPO_DEV void stage_params(const PackedLayout& K, const TrunkDev& T, PBuf pb, int trunk, float* SP, float* HBIAS,
                          int tid) {
  constexpr int H = 256, NSP4 = (6 * H + NHP * H) / 4;
  for (int q = tid; q < NSP4; q += kActThreads) {
    const int fl = 4 * q, vec = fl / H, off = fl - vec * H;
    int src = -1;
    if (vec < 6) {
      const int base = vec == 0 ? T.b1 : vec == 1 ? T.g1 : vec == 2 ? T.be1 : vec == 3 ? T.b2 : vec == 4 ? T.g2 : T.be2;
      src = base >= 0 ? base + off : -1;
    } else {
      const int hr = act_head_row(K, trunk, vec - 6);
      src = hr >= 0 ? hr + off : -1;
    }
    *reinterpret_cast<f4*>(SP + fl) = pld4(pb, src >= 0 ? src : K.size, 0);
  }
  if (tid < NHP) {
    const int hbo = act_head_bias(K, trunk, tid);
    HBIAS[tid] = bld1f(pb, hbo >= 0 ? hbo : K.size);
  }
}

// One trunk forward for the 16 rows whose (normalised, zero-padded) inputs are in XS: layer 1,
// LayerNorm + ReLU, layer 2, LayerNorm + ReLU, heads; leaves the head pre-activations (+ bias) in
// PRE [16][LDP]. Weights: w1 / w2 register slices of this wave. Same operations, same order as
// k_act3 (LN_BETA, RT = 1).
// PRE_PASS false: stop once the per-wave head partials are in HP (after the barrier); the caller
// adds them itself (the same adds in the same order: bitwise the PRE values).
template <int NTO, int NHT, int RT = 1, bool PRE_PASS = true, typename PRE_L2 = int>
PPO_DEV void trunk_rows(const f4 (&w1)[NTO][2], const f4 (&w2)[16][2], float* lds, int nh, int tid,
                        PRE_L2 pre_l2 = 0, int stamp_t = -1) {
  (void)stamp_t;  // ROLL_STAMP step index (stamps build; -1: none)
  using GE = RollGeo<NTO, NHT, 16 * RT>;
  constexpr int H = 256, LDX = GE::LDX, LDH = GE::LDH, LDP = GE::LDP, NHP = GE::NHP, R = 16 * RT;
  float* XS = lds + GE::oXS;
  float* HB = lds + GE::oHB;
  float* SP = lds + GE::oSP;
  float* HBIAS = lds + GE::oHBIAS;
  float* RED = lds + GE::oRED;
  float* HP = lds + GE::oHP;
  float* PRE = lds + GE::oPRE;
  const int lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  f4 acc[2][RT];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const f4 b1 = *reinterpret_cast<const f4*>(SP + GE::sB1 + 32 * wave + 16 * u + 4 * g);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[u][rt] = b1;
  }
  const float* xin = XS + j * LDX + 4 * g;
  act_layer_regs<NTO, RT>(acc, w1, [&](int t, int rt) { return *reinterpret_cast<const f4*>(xin + 16 * rt * LDX + 16 * t); });
#ifdef PPO_STAMPS
  const bool dbg = stamp_t == 0 && RT == 1 && (int)blockIdx.x * 16 + j == kRdbgEnv;
  auto dump = [&](int base) {
    if (dbg)
      for (int u = 0; u < 2; ++u)
        for (int r = 0; r < 4; ++r) RDBG(0, base + 32 * wave + 16 * u + 4 * g + r, acc[u][0][r]);
  };
#else
  auto dump = [](int) {};
#endif
  dump(0);
  act_activate<PPO_NET_LN_BETA, RT>(acc, SP + GE::sG1, SP + GE::sBE1, RED, wave, j, g);
  dump(260);
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
      *reinterpret_cast<f4*>(HB + (16 * rt + j) * LDH + 32 * wave + 16 * u + 4 * g) = acc[u][rt];
  lds_barrier();
  if (stamp_t >= 0) ROLL_STAMP(stamp_t, 5);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const f4 b2 = *reinterpret_cast<const f4*>(SP + GE::sB2 + 32 * wave + 16 * u + 4 * g);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[u][rt] = b2;
  }
  const float* hin = HB + j * LDH + 4 * g;
  // independent VALU work placed in the layer-2 block: the scheduler interleaves it with the MFMAs,
  // whose issue leaves the SIMD's vector pipe mostly free
  if constexpr (!std::is_same_v<PRE_L2, int>) pre_l2();
  act_layer_regs<16, RT>(acc, w2, [&](int t, int rt) { return *reinterpret_cast<const f4*>(hin + 16 * rt * LDH + 16 * t); });
  if (stamp_t >= 0) {
#ifdef PPO_STAMPS
    asm volatile("s_nop 0" ::"v"(acc[0][0].x), "v"(acc[1][0].x));  // the layer-2 results exist here
#endif
    ROLL_STAMP(stamp_t, 6);
  }
  dump(516);
  act_activate<PPO_NET_LN_BETA, RT>(acc, SP + GE::sG2, SP + GE::sBE2, RED, wave, j, g);
  dump(776);
  if (stamp_t >= 0) ROLL_STAMP(stamp_t, 7);
#pragma unroll
  for (int ht = 0; ht < NHT; ++ht) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      f4 hp = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const f4 wv = *reinterpret_cast<const f4*>(SP + GE::sW3 + (16 * ht + j) * H + 32 * wave + 16 * u + 4 * g);
        hp = mfma16(wv.x, acc[u][rt].x, hp);
        hp = mfma16(wv.y, acc[u][rt].y, hp);
        hp = mfma16(wv.z, acc[u][rt].z, hp);
        hp = mfma16(wv.w, acc[u][rt].w, hp);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) HP[(wave * NHP + 16 * ht + 4 * g + r) * R + 16 * rt + j] = hp[r];
#ifdef PPO_STAMPS
      if (dbg && ht == 0)
        for (int r = 0; r < 4; ++r) RDBG(0, 1032 + wave * 16 + 4 * g + r, hp[r]);
#endif
    }
  }
  lds_barrier();
  if constexpr (!PRE_PASS) return;
  for (int idx = tid; idx < R * nh; idx += kActThreads) {
    const int r = idx / nh, h = idx - r * nh;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < kActWaves; ++w) s += HP[(w * NHP + h) * R + r];
    PRE[r * LDP + h] = s + HBIAS[h];
  }
  lds_barrier();
}

// this wave's register slices of a trunk's W1 (NTO k-blocks) and W2 (16 k-blocks), 2 feature tiles
template <int NTO>
PPO_DEV void load_weight_slices(PBuf wsw, int wave, int lane, f4 (&w1)[NTO][2], f4 (&w2)[16][2]) {
  constexpr int H = 256, OP = NTO * 16;
  const int l1 = ((2 * wave) * NTO * 64 + lane) * 4;
  const int l2 = H * OP + ((2 * wave) * 16 * 64 + lane) * 4;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
#pragma unroll
    for (int t = 0; t < NTO; ++t) w1[t][u] = pld4(wsw, l1, 256 * (NTO * u + t));
#pragma unroll
    for (int t = 0; t < 16; ++t) w2[t][u] = pld4(wsw, l2, 256 * (16 * u + t));
  }
}

}  // namespace

// =============================================================================================
// k_rollout: T steps of {actor act + sample, synthetic env step} for 16 envs per workgroup
// =============================================================================================
template <int NTO, int NHT>
__global__ __launch_bounds__(512) void k_rollout(RolloutArgs a) {
  using GE = RollGeo<NTO, NHT>;
  constexpr int OP = GE::OP, LDX = GE::LDX, LDP = GE::LDP, LDQ = GE::LDQ, R = kRows;
  constexpr int NCH = (OP + 31) / 32;  // 32-dim chunks of the env state per env lane group
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* XS = lds + GE::oXS;
  float* PRE = lds + GE::oPRE;
  float* ITM = lds + GE::oITM;
  float* LPE = lds + GE::oLP;
  float* XO = lds + GE::oXO;
  float* Q = lds + GE::oQ;
  float* NRM = lds + GE::oNRM;
  float* ACT = lds + GE::oACT;
  float* EV = lds + GE::oENV;
  int* EVI = reinterpret_cast<int*>(EV);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const PackedLayout& K = a.K;
  const float* __restrict__ P = a.P;
  const PBuf pb = make_pbuf(P, K.size);
  const int O = K.O, A = K.A, E = a.E;
  const int row0 = blockIdx.x * R;
  const SynthArgs& sv = a.env;

  // ---- prologue: resident weights, staged parameters, env state of this block ----
  f4 w1[NTO][2], w2[16][2];
  load_weight_slices<NTO>(make_pbuf(a.WSW, (int)sw_size(256, OP)), wave, lane, w1, w2);
  stage_params<GE::NHP>(K, K.tr[1], pb, 1, lds + GE::oSP, lds + GE::oHBIAS, tid);
  for (int f = tid; f < OP; f += kActThreads) {
    NRM[f] = f < O ? P[K.omean + f] : 0.0f;
    NRM[OP + f] = f < O ? P[K.ostd + f] : 1.0f;
  }
  for (int idx = tid; idx < R * O; idx += kActThreads) {
    const int r = idx / O, f = idx - r * O, e = row0 + r;
    XO[r * LDQ + f] = e < E ? a.next_obs[(long)e * O + f] : 0.0f;
    Q[r * LDQ + f] = e < E ? sv.q[(long)e * O + f] : 0.0f;
  }
  if (tid < R) {
    const int e = min(row0 + tid, E - 1);
    EV[EV_DONE * R + tid] = a.next_done[e];
    EVI[EV_AR * R + tid] = sv.autoreset[e];
    EVI[EV_T * R + tid] = sv.t[e];
    EVI[EV_RSEED * R + tid] = (int)sv.rseed[e];
    EVI[EV_RCOUNT * R + tid] = (int)sv.rcount[e];
    EV[EV_EPR * R + tid] = sv.ep_ret[e];
    EVI[EV_EPL * R + tid] = sv.ep_len[e];
    EV[EV_FR * R + tid] = sv.fin_ret[e];
    EV[EV_FL * R + tid] = sv.fin_len[e];
    EV[EV_FC * R + tid] = sv.fin_cnt[e];
  }
  lds_barrier();
  const SampleKey key = sample_key(a.seed, a.rank);
  const float hi = P[K.hi], lo = P[K.lo];
  // this thread's Beta item (row, action, alpha | beta): the R * 2A items spread evenly over the
  // waves (2A <= 16: at most 32 per wave), so fewer lanes per wave wait on a rejected gamma attempt
  const int bper = (R * A * 2 + kActWaves - 1) / kActWaves;
  const int bitem = lane < bper ? wave * bper + lane : R * A * 2;
  const bool defer = a.s_beta != nullptr;

  for (int t = 0; t < a.T; ++t) {
    const long step_id = a.step0 + t;
    ROLL_STAMP(t, 0);
    // ---- inputs: rollout stores of obs[t] / dones[t]; normalised rows into XS (k_act3 order) ----
    for (int idx = tid; idx < R * OP; idx += kActThreads) {
      const int r = idx / OP, f = idx - r * OP, e = row0 + r;
      const bool valid = e < E && f < O;
      const float x = valid ? XO[r * LDQ + f] : 0.0f;
      if (valid) a.s_obs[((long)t * E + e) * O + f] = x;
      XS[r * LDX + f] = valid ? (x - NRM[f]) / NRM[OP + f] : x;
    }
    if (tid < R && row0 + tid < E) a.s_dones[(long)t * E + row0 + tid] = EV[EV_DONE * R + tid];
    lds_barrier();
    // the first Marsaglia-Tsang attempt's draws of this thread's item (bitem) do not depend on the
    // network: computed inside layer 2, under its MFMAs (k_act3 computes them under its weight
    // fetch; gamma_mt_d0 with them is gamma_mt, bitwise)
    GammaDraw gd0 = GammaDraw{0.f, 0.f};
    ROLL_STAMP(t, 1);
    // deferred log-probs (a.s_beta, the AC rollout): no PRE pass — each Beta item adds its head's
    // per-wave partials itself (the same adds in the same order as the pass: bitwise its PRE), one
    // LDS pass and one barrier fewer per step
    const auto draw0 = [&] {
      if (bitem < R * A * 2) {
        const int which = bitem & 1, ra = bitem >> 1, r = ra / A, ai = ra - r * A;
        const uint32_t db = 0x10000u + (uint32_t)(ai * 2 + which) * 64u;
        gd0 = gamma_draw(key, (long)(row0 + r), step_id, db);
      }
    };
    if (defer) trunk_rows<NTO, NHT, 1, false>(w1, w2, lds, 2 * A, tid, draw0, (int)t);
    else trunk_rows<NTO, NHT>(w1, w2, lds, 2 * A, tid, draw0, (int)t);
    // ---- Beta sample (k_act3 stage 1 / 2, PPO_SAMPLE); the log-prob terms either here (as k_act3)
    // or, with a.s_beta, stored for k_beta_logp after the rollout (they are not on the env's path) ----
    ROLL_STAMP(t, 2);
    if (bitem < R * A * 2) {
      const int idx = bitem, which = idx & 1, ra = idx >> 1, r = ra / A, ai = ra - r * A;
      const long env = row0 + r;
      float pre;
      if (defer) {
        const int h = ai + which * A;
        const float* HP = lds + GE::oHP;
        float sm = 0.f;
#pragma unroll
        for (int w = 0; w < kActWaves; ++w) sm += HP[(w * GE::NHP + h) * R + r];
        pre = sm + lds[GE::oHBIAS + h];
      } else {
        pre = PRE[r * LDP + ai + which * A];
      }
#ifdef PPO_STAMPS
      if (t == 0 && env == kRdbgEnv) RDBG(0, 1160 + ai + which * A, pre);
#endif
      const float c = softplusf_(pre) + 1.0f;
      const uint32_t db = 0x10000u + (uint32_t)(ai * 2 + which) * 64u;
      const float gs = gamma_mt_d0(c, gd0, key, env, step_id, db);
      float* it = ITM + ((r * A + ai) * 2 + which) * 4;
      it[0] = c;
      it[1] = gs;
      if (!defer) {
        float tg_unused;
        lgamma_digamma_trigamma(c, it[2], it[3], tg_unused);
      }
    }
    lds_barrier();
    for (int idx = tid; idx < R * A; idx += kActThreads) {
      const int r = idx / A, ai = idx - r * A, e = row0 + r;
      const float* ia = ITM + (idx * 2 + 0) * 4;
      const float* ib = ITM + (idx * 2 + 1) * 4;
      const float al = ia[0], be = ib[0];
      const float s01 = ia[1] / (ia[1] + ib[1]);
      const float act = (s01 - 0.0f) / (1.0f - 0.0f) * (hi - lo) + lo;
      ACT[r * 24 + ai] = act;
      if (e < E) a.s_actions[((long)t * E + e) * A + ai] = act;
      if (defer) {
        if (e < E) {
          float* d = a.s_beta + (((long)t * E + e) * A + ai) * 3;
          d[0] = al;
          d[1] = be;
          d[2] = s01;
        }
      } else {
        const float ab = al + be;
        float lgab, psab, tab_unused;
        lgamma_digamma_trigamma(ab, lgab, psab, tab_unused);
        const float lga = ia[2], lgb = ib[2];
        LPE[idx * 2 + 0] = xlogyf_(al - 1.0f, s01) + xlogyf_(be - 1.0f, 1.0f - s01) + (lgab - (lga + lgb));
      }
    }
    lds_barrier();
    if (!defer && tid < R && row0 + tid < E) {
      float lp = 0.f;
      for (int ai = 0; ai < A; ++ai) lp += LPE[(tid * A + ai) * 2];
      a.s_logp[(long)t * E + row0 + tid] = lp;
    }
    ROLL_STAMP(t, 3);
    // ---- env step (k_synth_step / k_synth_step_wide arithmetic): 32 lanes per env ----
    {
#pragma clang fp contract(off)
      const int r = tid >> 5, i0 = tid & 31, e = row0 + r;
      const bool live = e < E;
      const bool reset = EVI[EV_AR * R + r] != 0;
      float* q = Q + r * LDQ;
      float* xo = XO + r * LDQ;
      const float* ar = ACT + r * 24;
      if (live && reset) {
        const uint32_t rs = (uint32_t)EVI[EV_RSEED * R + r], rc = (uint32_t)EVI[EV_RCOUNT * R + r];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          const int i = 32 * c + i0;
          if (i < O) {
            uint32_t rr[4];
            philox4x32(rc, (uint32_t)i, 0u, 0u, rs, 0x5EED5EEDu, rr);
            const float v = (0.1f * ((2.0f * u01(rr[0])) - 1.0f));
            q[i] = v;
            xo[i] = v;
          }
        }
        if (i0 == 0) {
          EVI[EV_RCOUNT * R + r] = (int)(rc + 1);
          EVI[EV_T * R + r] = 0;
          EV[EV_EPR * R + r] = 0.0f;
          EVI[EV_EPL * R + r] = 0;
          EV[EV_DONE * R + r] = 0.0f;
          EVI[EV_AR * R + r] = 0;
          a.s_rewards[(long)t * E + e] = 0.0f;
        }
      } else if (live) {
        float qo[NCH], qn[NCH];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          const int i = 32 * c + i0;
          qo[c] = i < O ? q[i] : 0.0f;
          qn[c] = i < O ? q[i + 1 < O ? i + 1 : 0] : 0.0f;
        }
        float q0_new = 0.0f;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          const int i = 32 * c + i0;
          if (i < O) {
            const float ai = fminf(fmaxf(ar[i % A], a.lo), a.hi);
            const float nq = __fmaf_rn(0.9f, qo[c], __fmaf_rn(0.1f, ai, (0.05f * qn[c])));
            q[i] = nq;
            xo[i] = nq;
            if (c == 0) q0_new = nq;
          }
        }
        if (i0 == 0) {
          const float vel = ((q0_new - qo[0]) / 0.05f);
          float ctrl = 0.0f;
          for (int k = 0; k < A; ++k) {
            const float ak = fminf(fmaxf(ar[k], a.lo), a.hi);
            ctrl = (ctrl + ((0.1f * ak) * ak));
          }
          const float rw = (vel - ctrl);
          const int tt = EVI[EV_T * R + r] + 1;
          EVI[EV_T * R + r] = tt;
          const bool tr = tt >= 1000;
          a.s_rewards[(long)t * E + e] = rw;
          EV[EV_DONE * R + r] = tr ? 1.0f : 0.0f;
          const float epr = (EV[EV_EPR * R + r] + rw);
          EV[EV_EPR * R + r] = epr;
          const int epl = EVI[EV_EPL * R + r] + 1;
          EVI[EV_EPL * R + r] = epl;
          if (tr) {
            EV[EV_FR * R + r] += epr;
            EV[EV_FL * R + r] += (float)epl;
            EV[EV_FC * R + r] += 1.0f;
          }
          EVI[EV_AR * R + r] = tr ? 1 : 0;
        }
      }
    }
    lds_barrier();
    ROLL_STAMP(t, 4);
  }
  // ---- epilogue: next_obs / next_done and the env state back to HBM ----
  for (int idx = tid; idx < R * O; idx += kActThreads) {
    const int r = idx / O, f = idx - r * O, e = row0 + r;
    if (e < E) {
      a.next_obs[(long)e * O + f] = XO[r * LDQ + f];
      sv.q[(long)e * O + f] = Q[r * LDQ + f];
    }
  }
  if (tid < R && row0 + tid < E) {
    const int e = row0 + tid;
    a.next_done[e] = EV[EV_DONE * R + tid];
    sv.autoreset[e] = EVI[EV_AR * R + tid];
    sv.t[e] = EVI[EV_T * R + tid];
    sv.rseed[e] = (uint32_t)EVI[EV_RSEED * R + tid];
    sv.rcount[e] = (uint32_t)EVI[EV_RCOUNT * R + tid];
    sv.ep_ret[e] = EV[EV_EPR * R + tid];
    sv.ep_len[e] = EVI[EV_EPL * R + tid];
    sv.fin_ret[e] = EV[EV_FR * R + tid];
    sv.fin_len[e] = EV[EV_FL * R + tid];
    sv.fin_cnt[e] = EV[EV_FC * R + tid];
  }
}

// =============================================================================================
// k_beta_logp: the rollout's Beta log-probs from the stored (alpha, beta, sample) of every
// (row, action), after the rollout (k_act3's stage-1 / stage-2 terms and row sum, same order)
// =============================================================================================
__global__ __launch_bounds__(256) void k_beta_logp(const float* __restrict__ sb, float* __restrict__ logp, long n,
                                                   int A) {
  const long row = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= n) return;
  float lp = 0.f;
  for (int ai = 0; ai < A; ++ai) {
    const float* d = sb + (row * A + ai) * 3;
    const float al = d[0], be = d[1], s01 = d[2];
    float lga, lgb, lgab, u0, u1;
    lgamma_digamma_trigamma(al, lga, u0, u1);
    lgamma_digamma_trigamma(be, lgb, u0, u1);
    const float ab = al + be;
    lgamma_digamma_trigamma(ab, lgab, u0, u1);
    lp += xlogyf_(al - 1.0f, s01) + xlogyf_(be - 1.0f, 1.0f - s01) + (lgab - (lga + lgb));
  }
  logp[row] = lp;
}

int launch_beta_logp(const float* s_beta, float* logp, long n, int A, hipStream_t s) {
  hipLaunchKernelGGL(k_beta_logp, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, s_beta, logp, n, A);
  return 0;
}

// =============================================================================================
// k_values: critic(obs[i]) for n stored rows; workgroups walk R-row blocks
// =============================================================================================
// 32 or 64 rows per pass (two or four 16-row MFMA tiles per wave): the LayerNorm exchanges and
// barriers of a pass are shared by more rows; every row's arithmetic is the 16-row pass's (bitwise).
// 64 only for the narrow observation widths: at NTO = 7 the fourth tile's accumulators spill.
template <int NTO>
constexpr int val_rows() { return NTO <= 2 ? 64 : 32; }
template <int NTO, int NHT>
__global__ __launch_bounds__(512) void k_values(ValuesArgs a) {
  constexpr int R = val_rows<NTO>();
  using GE = RollGeo<NTO, NHT, R>;
  constexpr int OP = GE::OP, LDX = GE::LDX, LDP = GE::LDP;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* XS = lds + GE::oXS;
  float* PRE = lds + GE::oPRE;
  float* NRM = lds + GE::oXO;  // the env regions from oXO on are unused here: the statistics go there
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const PackedLayout& K = a.K;
  const float* __restrict__ P = a.P;
  const PBuf pb = make_pbuf(P, K.size);
  const int O = K.O;
  f4 w1[NTO][2], w2[16][2];
  load_weight_slices<NTO>(make_pbuf(a.WSW, (int)sw_size(256, OP)), wave, lane, w1, w2);
  stage_params<GE::NHP>(K, K.tr[0], pb, 0, lds + GE::oSP, lds + GE::oHBIAS, tid);
  for (int f = tid; f < OP; f += kActThreads) {
    NRM[f] = f < O ? P[K.omean + f] : 0.0f;
    NRM[OP + f] = f < O ? P[K.ostd + f] : 1.0f;
  }
  const long nblk = (a.n + R - 1) / R;
  // the block's observations (R x OP <= 64 x 32 or 32 x 112: at most 7 per thread) are loaded one block ahead,
  // under the previous block's layers
  constexpr int NXI = (R * OP + kActThreads - 1) / kActThreads;
  float xnext[NXI];
  auto load_obs = [&](long b) {
#pragma unroll
    for (int u = 0; u < NXI; ++u) {
      const int idx = tid + kActThreads * u, r = idx / OP, f = idx - r * OP;
      const long row = b * R + r;
      const bool valid = b < nblk && idx < R * OP && row < a.n && f < O;
      const float x = a.obs[(valid ? row : 0) * O + (valid ? f : 0)];
      xnext[u] = valid ? x : 0.0f;
    }
  };
  load_obs(blockIdx.x);
  for (long b = blockIdx.x; b < nblk; b += gridDim.x) {
    const long row0 = b * R;
    lds_barrier();  // previous block's PRE reads done; NRM / SP staged (first pass)
#pragma unroll
    for (int u = 0; u < NXI; ++u) {
      const int idx = tid + kActThreads * u, r = idx / OP, f = idx - r * OP;
      const long row = row0 + r;
      const bool valid = row < a.n && f < O;
      const float x = xnext[u];
      if (idx < R * OP) XS[r * LDX + f] = valid ? (x - NRM[f]) / NRM[OP + f] : x;
    }
    load_obs(b + gridDim.x);
    lds_barrier();
    trunk_rows<NTO, NHT, R / 16>(w1, w2, lds, 1, tid);
    if (tid < R && row0 + tid < a.n) a.values[row0 + tid] = PRE[tid * LDP];
  }
}

// =============================================================================================
// The PPO agent (two 64-wide tanh trunks, Normal head; ppo:120-157): k_rollout4 / k_values4 run
// k_act4's arithmetic (ppo_act_narrow.hip: layer 1 split over K across the 4 waves, partial sums met
// in LDS in a fixed order) with the weights in registers, and the device env with the PPO wrapper
// chain (ppo:41-49) fused, for all T steps.
// =============================================================================================
namespace {
constexpr int kR4Threads = 256, kR4Rows = 16, kR4H = 64, kR4LDP = kR4Rows + 1, kR4LDH = kR4H + 4;

template <int NTO, int NHT>
struct Roll4Geo {
  static constexpr int OP = NTO * 16, NHP = NHT * 16, LDQ = OP + 1;
};

// this wave's register operands of one trunk, exactly those k_act4 loads at kernel start
template <int NTO, int NKW>
PPO_DEV void load4_weights(PBuf wsw, int lane, int ks, f4 (&wa)[NKW][4], f4 (&w2v)[4]) {
  constexpr int H = kR4H, OP = NTO * 16;
  const int kb0 = ks * NKW;
#pragma unroll
  for (int q = 0; q < NKW; ++q)
#pragma unroll
    for (int ft = 0; ft < 4; ++ft) wa[q][ft] = pld4(wsw, 4 * lane, 256 * (ft * NTO + min(kb0 + q, NTO - 1)));
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) w2v[kb] = pld4(wsw, H * OP + 4 * lane, 256 * (4 * ks + kb));
}

// k_act4's trunk body for the 16 rows whose inputs this lane holds in xv: layer 1 partials (P1),
// tanh(b1 + sum of the 4 slices) (H1), layer 2 tile ks, tanh; returns h2 (this wave's tile ks)
template <int NTO, int NKW, typename PRE_L1>
PPO_DEV f4 trunk4(const f4 (&xv)[NKW], const f4 (&wa)[NKW][4], const f4 (&w2v)[4], f4 b1, f4 b2,
                  float (*P1)[kR4H][kR4LDP], float (*H1)[kR4LDH], int ks, int j, int g, PRE_L1 pre_l1) {
  const int kb0 = ks * NKW;
  {
    f4 acc[4];
#pragma unroll
    for (int ft = 0; ft < 4; ++ft) acc[ft] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < NKW; ++q) {
      if (kb0 + q < NTO) {
#pragma unroll
        for (int c = 0; c < 4; ++c)  // 4 independent chains interleaved, each in its own order
#pragma unroll
          for (int ft = 0; ft < 4; ++ft) acc[ft] = mfma16(wa[q][ft][c], xv[q][c], acc[ft]);
      }
    }
    // independent VALU work (the step's Normal draws) issued under the layer-1 MFMAs
    pre_l1();
#pragma unroll
    for (int ft = 0; ft < 4; ++ft)
#pragma unroll
      for (int r = 0; r < 4; ++r) P1[ks][16 * ft + 4 * g + r][j] = acc[ft][r];
  }
  __syncthreads();
  {
    f4 h;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 16 * ks + 4 * g + r;
      const float z = (((P1[0][f][j] + P1[1][f][j]) + P1[2][f][j]) + P1[3][f][j]) + b1[r];
      h[r] = tanhf(z);
    }
    *reinterpret_cast<f4*>(&H1[j][16 * ks + 4 * g]) = h;
  }
  __syncthreads();
  f4 z2 = b2;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    const f4 hb = *reinterpret_cast<const f4*>(&H1[j][16 * kb + 4 * g]);
    z2 = mfma16(w2v[kb].x, hb.x, z2);
    z2 = mfma16(w2v[kb].y, hb.y, z2);
    z2 = mfma16(w2v[kb].z, hb.z, z2);
    z2 = mfma16(w2v[kb].w, hb.w, z2);
  }
  f4 h2;
#pragma unroll
  for (int r = 0; r < 4; ++r) h2[r] = tanhf(z2[r]);
  return h2;
}
}  // namespace

// RR envs per workgroup (4 or 16): the MFMA tiles keep 16 rows (rows RR..15 are zero padding, which
// no real row's arithmetic sees), the env / wrapper phase gets 256 / RR lanes per env. With RR = 4
// a 1 024-env rollout spreads over 256 CUs instead of 64: the per-step layer MFMAs cost the same,
// the VALU-bound wrapper chain a quarter.
template <int NTO, int NHT, int RR>
__global__ __launch_bounds__(256) void k_rollout4(RolloutArgs a) {
  constexpr int H = kR4H, R = RR, OP = NTO * 16, NKW = (NTO + 3) / 4, NHP = NHT * 16;
  constexpr int LPE = kR4Threads / RR;  // env lanes per env (one env within one wave)
  constexpr int LDQ = Roll4Geo<NTO, NHT>::LDQ, NCE = (OP + LPE - 1) / LPE, kEnvGroup = 12;
  static_assert(RR == 4 || RR == 16, "k_rollout4: 4 or 16 envs per workgroup");
  __shared__ float P1[4][H][kR4LDP];
  __shared__ __attribute__((aligned(16))) float H1[kR4Rows][kR4LDH];
  __shared__ float HP[4][NHP][kR4LDP];
  __shared__ float ITM[R * NHP][2];
  __shared__ float XO[R * LDQ];   // the agent's input of the current step (the wrapped obs)
  __shared__ float Q[R * LDQ];    // env state q
  __shared__ float ACT[R * 32];
  __shared__ float EV[EV_NSLOT * R];
  __shared__ float WOM[R * LDQ];  // the wrapper chain's running obs mean / var of the block's envs
  __shared__ float WOV[R * LDQ];
  int* EVI = reinterpret_cast<int*>(EV);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4, ks = wave;
  const PackedLayout& K = a.K;
  const TrunkDev& T = K.tr[1];
  const float* __restrict__ P = a.P;
  const PBuf pb = make_pbuf(P, K.size);
  const int row0 = blockIdx.x * R, O = K.O, A = K.A, E = a.E;
  const int kb0 = ks * NKW;
  const SynthArgs& sv = a.env;
  const WrapArgs& w = a.env.w;

  f4 wa[NKW][4], w2v[4], hw[NHT];
  load4_weights<NTO, NKW>(make_pbuf(a.WSW, (int)sw_size(H, OP)), lane, ks, wa, w2v);
  const f4 b1 = pld4(pb, T.b1 + 16 * ks + 4 * g, 0);
  const f4 b2 = pld4(pb, T.b2 + 16 * ks + 4 * g, 0);
#pragma unroll
  for (int ht = 0; ht < NHT; ++ht) {
    const int h = 16 * ht + j;
    const f4 wv = pld4(pb, K.aW3 + min(h, A - 1) * H + 16 * ks + 4 * g, 0);
    hw[ht] = h < A ? wv : f4{0.f, 0.f, 0.f, 0.f};
  }
  constexpr int NI = (R * NHP + kR4Threads - 1) / kR4Threads;
  // per-item parameters of the Normal head: constant over the rollout, so std, var and log std
  // (k_act4's per-launch arithmetic) are computed once
  float i_b3[NI], i_sd[NI], i_var[NI], i_lsd[NI];
#pragma unroll
  for (int u = 0; u < NI; ++u) {
    const int idx = min(tid + kR4Threads * u, R * A - 1), ir = idx / A, ia = idx - ir * A;
    (void)ir;
    i_b3[u] = P[K.ab3 + ia];
    const float sd = expf(P[K.logstd + ia]);
    i_sd[u] = sd;
    i_var[u] = sd * sd;
    i_lsd[u] = logf(sd);
  }
  for (int idx = tid; idx < R * O; idx += kR4Threads) {
    const int r = idx / O, f = idx - r * O, e = row0 + r;
    XO[r * LDQ + f] = e < E ? a.next_obs[(long)e * O + f] : 0.0f;
    Q[r * LDQ + f] = e < E ? sv.q[(long)e * O + f] : 0.0f;
    if (w.on) {
      WOM[r * LDQ + f] = e < E ? w.om[(long)e * O + f] : 0.0f;
      WOV[r * LDQ + f] = e < E ? w.ov[(long)e * O + f] : 1.0f;
    }
  }
  if (tid < R) {
    const int e = min(row0 + tid, E - 1);
    if (w.on) {
      EV[EV_WOC * R + tid] = w.ocount[e];
      EV[EV_WRA * R + tid] = w.racc[e];
      EV[EV_WRM * R + tid] = w.rmean[e];
      EV[EV_WRV * R + tid] = w.rvar[e];
      EV[EV_WRC * R + tid] = w.rcount[e];
    }
    EV[EV_DONE * R + tid] = a.next_done[e];
    EVI[EV_AR * R + tid] = sv.autoreset[e];
    EVI[EV_T * R + tid] = sv.t[e];
    EVI[EV_RSEED * R + tid] = (int)sv.rseed[e];
    EVI[EV_RCOUNT * R + tid] = (int)sv.rcount[e];
    EV[EV_EPR * R + tid] = sv.ep_ret[e];
    EVI[EV_EPL * R + tid] = sv.ep_len[e];
    EV[EV_FR * R + tid] = sv.fin_ret[e];
    EV[EV_FL * R + tid] = sv.fin_len[e];
    EV[EV_FC * R + tid] = sv.fin_cnt[e];
  }
  __syncthreads();
  const SampleKey key = sample_key(a.seed, a.rank);
  const int row = row0 + j;
  const bool rvalid = j < R && row < E;  // MFMA tile row j is one of this block's envs

  for (int t = 0; t < a.T; ++t) {
    const long step_id = a.step0 + t;
    ROLL_STAMP(t, 0);
    // ---- inputs (k_act4's xv: this wave's k-slice), rollout stores of obs[t] / dones[t] ----
    f4 xv[NKW];
#pragma unroll
    for (int q = 0; q < NKW; ++q) {
      const int kb = kb0 + q;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int col = 16 * kb + 4 * g + c;
        const float v = XO[min(j, R - 1) * LDQ + min(col, O - 1)];
        xv[q][c] = (kb < NTO && col < O && rvalid) ? v : 0.f;
      }
    }
    // rollout store of obs[t] from the registers it arrived in (k_act4's store): lane (j, g) holds
    // columns 16 kb + 4 g .. + 3 of row j
    if (rvalid) {
      float* so = a.s_obs + ((long)t * E + row) * O;
#pragma unroll
      for (int q = 0; q < NKW; ++q) {
        const int col = 16 * (kb0 + q) + 4 * g;
        if (kb0 + q < NTO && col < O) {
          if ((O & 3) == 0) {
            *reinterpret_cast<f4*>(so + col) = xv[q];
          } else {
#pragma unroll
            for (int c = 0; c < 4; ++c)
              if (col + c < O) so[col + c] = xv[q][c];
          }
        }
      }
    }
    if (tid < R && row0 + tid < E) a.s_dones[(long)t * E + row0 + tid] = EV[EV_DONE * R + tid];
    ROLL_STAMP(t, 1);
    // the Normal draws of this step (k_act4: computed under the weight fetch; here under layer 1)
    float nz[NI];
    const f4 h2 = trunk4<NTO, NKW>(xv, wa, w2v, b1, b2, P1, H1, ks, j, g, [&] {
#pragma unroll
      for (int u = 0; u < NI; ++u) {
        const int idx = min(tid + kR4Threads * u, R * A - 1), ir = idx / A, ia = idx - ir * A;
        uint32_t rr[4];
        philox_draw(key, (long)(row0 + ir), step_id, (uint32_t)(ia >> 1), rr);
        float z0, z1;
        box_muller(rr[0], rr[1], z0, z1);
        nz[u] = (ia & 1) ? z1 : z0;
      }
    });
    ROLL_STAMP(t, 2);
#pragma unroll
    for (int ht = 0; ht < NHT; ++ht) {
      f4 hp = f4{0.f, 0.f, 0.f, 0.f};
      hp = mfma16(hw[ht].x, h2.x, hp);
      hp = mfma16(hw[ht].y, h2.y, hp);
      hp = mfma16(hw[ht].z, h2.z, hp);
      hp = mfma16(hw[ht].w, h2.w, hp);
#pragma unroll
      for (int r = 0; r < 4; ++r) HP[ks][16 * ht + 4 * g + r][j] = hp[r];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const int idx = tid + kR4Threads * u;
      if (idx < R * A) {
        const int ir = idx / A, ia = idx - ir * A, irow = row0 + ir;
        const float mu = (((HP[0][ia][ir] + HP[1][ia][ir]) + HP[2][ia][ir]) + HP[3][ia][ir]) + i_b3[u];
        const float sd = i_sd[u], var = i_var[u], lsd = i_lsd[u];
        const float act = mu + nz[u] * sd;
        const float d = act - mu;
        ITM[idx][0] = -(d * d) / (2.0f * var) - lsd - kLz;
        ACT[ir * 32 + ia] = act;
        if (irow < E) a.s_actions[((long)t * E + irow) * A + ia] = act;
      }
    }
    __syncthreads();
    if (tid < R && row0 + tid < E) {
      float lp = 0.f;
      for (int ai = 0; ai < A; ++ai) lp += ITM[tid * A + ai][0];
      a.s_logp[(long)t * E + row0 + tid] = lp;
    }
    ROLL_STAMP(t, 3);
    // ---- env step (k_synth_step / _wide arithmetic, wrapper chain fused): LPE lanes per env, all
    // RR envs at once (the per-env reward / episode bookkeeping of lane 0 runs once per step) ----
    {
#pragma clang fp contract(off)
      const int r = tid / LPE, i0 = tid % LPE, e = row0 + r;
      if (e < E) {
        const bool reset = EVI[EV_AR * R + r] != 0;
        float* q = Q + r * LDQ;
        float* xo = XO + r * LDQ;
        float* om = WOM + r * LDQ;
        float* ov = WOV + r * LDQ;
        const float* ar = ACT + r * 32;
        const float oc = EV[EV_WOC * R + r];  // read by every lane before lane 0 stores oc + 1
        if (reset) {
          const uint32_t rs = (uint32_t)EVI[EV_RSEED * R + r], rc = (uint32_t)EVI[EV_RCOUNT * R + r];
#pragma unroll
          for (int c = 0; c < NCE; ++c) {
            const int i = LPE * c + i0;
            if (i < O) {
              uint32_t rr[4];
              philox4x32(rc, (uint32_t)i, 0u, 0u, rs, 0x5EED5EEDu, rr);
              const float v = (0.1f * ((2.0f * u01(rr[0])) - 1.0f));
              q[i] = v;
              xo[i] = w.on ? wrap_obs_at(om + i, ov + i, oc, v) : v;
            }
          }
          if (i0 == 0) {
            if (w.on) EV[EV_WOC * R + r] = oc + 1.0f;
            EVI[EV_RCOUNT * R + r] = (int)(rc + 1);
            EVI[EV_T * R + r] = 0;
            EV[EV_EPR * R + r] = 0.0f;
            EVI[EV_EPL * R + r] = 0;
            EV[EV_DONE * R + r] = 0.0f;
            EVI[EV_AR * R + r] = 0;
            a.s_rewards[(long)t * E + e] = 0.0f;
          }
        } else {
          // Groups of up to 12 elements per lane: every LDS operand of a group is read before any
          // of its results is written (independent element chains; interleaved loads and stores
          // through possibly aliasing LDS pointers would serialise them). One env's LPE lanes are in
          // one wave, so a q[i + 1] read precedes the neighbour's store in program order; the wrap
          // to q[0] reads the value from before the step.
          const float q0_old = q[0];
          const Recip rtot = recip_of(oc + 1.0f);
          float q0_new = 0.0f;
          int ai = i0 % A;
          const int astep = LPE % A;
#pragma unroll
          for (int c0 = 0; c0 < NCE; c0 += kEnvGroup) {
            float qo[kEnvGroup], qn[kEnvGroup], wm[kEnvGroup], wv[kEnvGroup], ac[kEnvGroup];
#pragma unroll
            for (int u = 0; u < kEnvGroup; ++u) {
              if (c0 + u < NCE) {
                const int i = min(LPE * (c0 + u) + i0, O - 1);
                qo[u] = q[i];
                qn[u] = i + 1 < O ? q[i + 1] : q0_old;
                ac[u] = ar[ai];
                ai += astep;
                ai = ai >= A ? ai - A : ai;
                if (w.on) {
                  wm[u] = om[i];
                  wv[u] = ov[i];
                }
              }
            }
            float nq[kEnvGroup], xn[kEnvGroup];
#pragma unroll
            for (int u = 0; u < kEnvGroup; ++u) {
              if (c0 + u < NCE) {
                const float aic = fminf(fmaxf(ac[u], a.lo), a.hi);
                nq[u] = __fmaf_rn(0.9f, qo[u], __fmaf_rn(0.1f, aic, (0.05f * qn[u])));
                xn[u] = w.on ? wrap_obs_at_r(&wm[u], &wv[u], oc, rtot, nq[u]) : nq[u];
              }
            }
            if (c0 == 0) q0_new = nq[0];
#pragma unroll
            for (int u = 0; u < kEnvGroup; ++u) {
              const int i = LPE * (c0 + u) + i0;
              if (c0 + u < NCE && i < O) {
                q[i] = nq[u];
                xo[i] = xn[u];
                if (w.on) {
                  om[i] = wm[u];
                  ov[i] = wv[u];
                }
              }
            }
          }
          if (i0 == 0) {
            if (w.on) EV[EV_WOC * R + r] = oc + 1.0f;
            const float vel = ((q0_new - q0_old) / 0.05f);
            float ctrl = 0.0f;
            for (int k = 0; k < A; ++k) {
              const float ak = fminf(fmaxf(ar[k], a.lo), a.hi);
              ctrl = (ctrl + ((0.1f * ak) * ak));
            }
            const float rw = (vel - ctrl);
            const int tt = EVI[EV_T * R + r] + 1;
            EVI[EV_T * R + r] = tt;
            const bool tr = tt >= 1000;
            a.s_rewards[(long)t * E + e] =
                w.on ? wrap_reward_at(EV + EV_WRA * R + r, EV + EV_WRM * R + r, EV + EV_WRV * R + r,
                                      EV + EV_WRC * R + r, w.gamma, rw, 0.0f)
                     : rw;
            EV[EV_DONE * R + r] = tr ? 1.0f : 0.0f;
            const float epr = (EV[EV_EPR * R + r] + rw);
            EV[EV_EPR * R + r] = epr;
            const int epl = EVI[EV_EPL * R + r] + 1;
            EVI[EV_EPL * R + r] = epl;
            if (tr) {
              EV[EV_FR * R + r] += epr;
              EV[EV_FL * R + r] += (float)epl;
              EV[EV_FC * R + r] += 1.0f;
            }
            EVI[EV_AR * R + r] = tr ? 1 : 0;
          }
        }
      }
    }
    __syncthreads();
    ROLL_STAMP(t, 4);
  }
  for (int idx = tid; idx < R * O; idx += kR4Threads) {
    const int r = idx / O, f = idx - r * O, e = row0 + r;
    if (e < E) {
      a.next_obs[(long)e * O + f] = XO[r * LDQ + f];
      sv.q[(long)e * O + f] = Q[r * LDQ + f];
      if (w.on) {
        w.om[(long)e * O + f] = WOM[r * LDQ + f];
        w.ov[(long)e * O + f] = WOV[r * LDQ + f];
      }
    }
  }
  if (tid < R && row0 + tid < E) {
    const int e = row0 + tid;
    if (w.on) {
      w.ocount[e] = EV[EV_WOC * R + tid];
      w.racc[e] = EV[EV_WRA * R + tid];
      w.rmean[e] = EV[EV_WRM * R + tid];
      w.rvar[e] = EV[EV_WRV * R + tid];
      w.rcount[e] = EV[EV_WRC * R + tid];
    }
    a.next_done[e] = EV[EV_DONE * R + tid];
    sv.autoreset[e] = EVI[EV_AR * R + tid];
    sv.t[e] = EVI[EV_T * R + tid];
    sv.rseed[e] = (uint32_t)EVI[EV_RSEED * R + tid];
    sv.rcount[e] = (uint32_t)EVI[EV_RCOUNT * R + tid];
    sv.ep_ret[e] = EV[EV_EPR * R + tid];
    sv.ep_len[e] = EVI[EV_EPL * R + tid];
    sv.fin_ret[e] = EV[EV_FR * R + tid];
    sv.fin_len[e] = EV[EV_FL * R + tid];
    sv.fin_cnt[e] = EV[EV_FC * R + tid];
  }
}

// the PPO critic over n stored rows (k_act4's critic workgroups: the same chain and partial order)
template <int NTO>
__global__ __launch_bounds__(256) void k_values4(ValuesArgs a) {
  constexpr int H = kR4H, R = kR4Rows, OP = NTO * 16, NKW = (NTO + 3) / 4;
  __shared__ float P1[4][H][kR4LDP];
  __shared__ __attribute__((aligned(16))) float H1[R][kR4LDH];
  __shared__ float VP[4][R];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4, ks = wave;
  const PackedLayout& K = a.K;
  const TrunkDev& T = K.tr[0];
  const float* __restrict__ P = a.P;
  const PBuf pb = make_pbuf(P, K.size);
  const int O = K.O, kb0 = ks * NKW;
  f4 wa[NKW][4], w2v[4];
  load4_weights<NTO, NKW>(make_pbuf(a.WSW, (int)sw_size(H, OP)), lane, ks, wa, w2v);
  const f4 b1 = pld4(pb, T.b1 + 16 * ks + 4 * g, 0);
  const f4 b2 = pld4(pb, T.b2 + 16 * ks + 4 * g, 0);
  const f4 hv = pld4(pb, K.cW3 + 16 * ks + 4 * g, 0);
  const float c_b3 = P[K.cb3];
  const long nblk = (a.n + R - 1) / R;
  for (long b = blockIdx.x; b < nblk; b += gridDim.x) {
    const long row0 = b * R, row = row0 + j, rowc = row < a.n ? row : a.n - 1;
    f4 xv[NKW];
#pragma unroll
    for (int q = 0; q < NKW; ++q) {
      const int kb = kb0 + q;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int col = 16 * kb + 4 * g + c;
        const float v = a.obs[rowc * O + min(col, O - 1)];
        xv[q][c] = (kb < NTO && col < O && row < a.n) ? v : 0.f;
      }
    }
    __syncthreads();  // the previous block's VP / P1 / H1 readers are done
    const f4 h2 = trunk4<NTO, NKW>(xv, wa, w2v, b1, b2, P1, H1, ks, j, g, [] {});
    float p = (hv.x * h2.x + hv.y * h2.y) + (hv.z * h2.z + hv.w * h2.w);
    p = row_allreduce(p);
    if (g == 0) VP[ks][j] = p;
    __syncthreads();
    if (tid < R && row0 + tid < a.n) a.values[row0 + tid] = (((VP[0][tid] + VP[1][tid]) + VP[2][tid]) + VP[3][tid]) + c_b3;
  }
}

// =============================================================================================
// k_rollout_v: the AC rollout for few envs per GPU (E <= 512: the E = 4096 / 8 shard), on the VALU
// instead of MFMA, 2 envs per workgroup.
//
// k_rollout's step is bounded by layer 2 on one CU: 1 024 16x16x4 MFMAs for its 16-env block
// (8.2 K cycles per SIMD), whatever number of those 16 rows is real — at E = 512 its 32 workgroups
// leave 224 CUs idle and every step still pays the 16-row layer. Here a workgroup owns 2 envs (all
// CUs busy at E = 512) and the layers run as v_fma_f32 chains, one lane per (row, output feature),
// the f32 VALU's rate equal to the MFMA's. Results are bitwise k_act3's: an f32 MFMA is a k-ordered
// fmaf chain (MI355X guide; scripts/probe/fma_chain_probe, fma_chain_big_probe: 0 mismatches), so
// each layer runs the k_act3 chain order k = 16 t + 4 g + c (t, c outer, g inner) from the bias; the
// LayerNorm statistics, head partials and their sums repeat k_act3's partial-sum trees exactly (lane
// partials over the same 8 features, the g-butterfly, the wave-order sums).
//  * 8 waves: row w >> 2, feature quarter w & 3 (lane = feature 64 (w & 3) + lane); each lane keeps
//    its W1 row and W2 chain positions 0..127 in registers (160 VGPRs) for the whole rollout, and
//    positions 128..255 come from one 128 KB LDS copy shared by the two rows (float4 per 4
//    positions, lane-consecutive: conflict-free);
//  * B operands (the layer inputs) sit in LDS in chain order per row, read as broadcast ds_read_b128;
//  * LayerNorm statistics: the layer's outputs go to LDS and 8 x 2 x 4 "stats lanes" (old wave, row,
//    lane group g) recompute k_act3's lane partials from there;
//  * heads: one lane per (head, old wave, row) runs that wave's 32-feature MFMA chain order from
//    float4 reads;
//  * Beta sampling, the env step and the episode bookkeeping are k_rollout's, for 2 envs;
//  * log-probs deferred to k_beta_logp (a.s_beta) only.
// =============================================================================================
namespace {
template <int NTO>
struct RollVGeo {
  static constexpr int R = 2, H = 256, OP = NTO * 16, NHP = 16, LDZ = H + 4, LDQ = OP + 1;
  static constexpr int oW2L = 0;                    // W2 chain positions 128..255: [32][H] float4s
  // layer inputs by chain position p = 16 i + k, k-major so that lane k of every 16-lane row loads
  // positions k, 16 + k, ... as one contiguous run (row_newbcast then broadcasts position p from
  // lane k): layer 1 [R][16][4] (i < OP / 16 <= 2), layer 2 [R][16][LDK] (i < 16, stride 20:
  // conflict-free ds_read_b128)
  static constexpr int LDK = 20;
  static constexpr int oXV = oW2L + 128 * H;
  static constexpr int oHV = oXV + R * 16 * 4;
  static constexpr int oZL = oHV + R * 16 * LDK;    // layer outputs, natural order: [R][LDZ]
  static constexpr int oH2 = oZL + R * LDZ;         // head inputs h2: [R][LDZ]
  static constexpr int oRS = oH2 + R * LDZ;         // stats partials: sums [8][R], squares [8][R]
  static constexpr int oW3 = oRS + 16 * R;          // head rows [NHP][H]
  static constexpr int oHB = oW3 + NHP * H;         // head biases [NHP]
  static constexpr int oHP = oHB + NHP;             // head partials [8][NHP][R]
  static constexpr int oXO = oHP + 8 * NHP * R;     // agent input obs of the step [R][LDQ]
  static constexpr int oQ = oXO + R * LDQ;          // env state q [R][LDQ]
  static constexpr int oNRM = oQ + R * LDQ;         // obs mean | std [2][OP]
  static constexpr int oACT = oNRM + 2 * OP;        // actions [R][24]
  static constexpr int oENV = oACT + R * 24;        // per-env scalars [16][R]
  static constexpr int total = oENV + 16 * R;
};
// chain position of input k in a 16x16x4 layer chain: k-block t, k-step c, lane group g
PPO_DEV int chain_pos(int k) { return (k & ~15) | ((k & 3) << 2) | ((k >> 2) & 3); }
// acc = fma(w, x, acc) as one v_fma_f32 (single rounding: the MFMA chain's step). Written as asm so
// the SLP vectorizer cannot pack FMAs of one weight into v_pk_fma_f32 with the weight duplicated
// into a register pair (2 VGPRs per resident weight: the layer's 160 no longer fit)
PPO_DEV void fma_v(float& acc, float w, float x) { asm("v_fma_f32 %0, %1, %2, %0" : "+v"(acc) : "v"(w), "v"(x)); }
// acc = fma(x from lane K of this lane's 16-lane row, w, acc): v_fmac_f32 with a row_newbcast DPP
// source — one rounding, so bitwise fma(w, x, acc); the layer input reaches every lane without an
// LDS broadcast read per position (4 LDS cycles per ds_read_b128 however many lanes share the
// address). x is never written by a VALU instruction right before (loaded from LDS; an s_nop 1
// precedes each chain), so the DPP read-after-VALU-write hazard cannot occur.
template <int K>
PPO_DEV void fmac_bc(float& acc, float x, float w) {
  asm volatile("v_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(x), "v"(w), "n"(K));
}
template <int... Is, typename F>
PPO_DEV void static_for_impl(std::integer_sequence<int, Is...>, F&& f) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
PPO_DEV void static_for(F&& f) {
  static_for_impl(std::make_integer_sequence<int, N>{}, f);
}
}  // namespace

constexpr int kRVThreads = 512;
template <int NTO>
__global__ __launch_bounds__(kRVThreads) void k_rollout_v(RolloutArgs a) {
  using GE = RollVGeo<NTO>;
  constexpr int R = GE::R, H = 256, OP = GE::OP, NHP = GE::NHP, LDZ = GE::LDZ, LDQ = GE::LDQ;
  constexpr int NCH = (OP + 31) / 32;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* W2L = lds + GE::oW2L;
  float* XV = lds + GE::oXV;
  float* HV = lds + GE::oHV;
  float* ZL = lds + GE::oZL;
  float* H2 = lds + GE::oH2;
  float* RS = lds + GE::oRS;
  float* W3 = lds + GE::oW3;
  float* HBIAS = lds + GE::oHB;
  float* HP = lds + GE::oHP;
  float* XO = lds + GE::oXO;
  float* Q = lds + GE::oQ;
  float* NRM = lds + GE::oNRM;
  float* ACT = lds + GE::oACT;
  float* EV = lds + GE::oENV;
  int* EVI = reinterpret_cast<int*>(EV);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rg = wave >> 2, f = 64 * (wave & 3) + lane;  // this lane's row and output feature
  const PackedLayout& K = a.K;
  const TrunkDev& T = K.tr[1];
  const float* __restrict__ P = a.P;
  const int O = K.O, A = K.A, E = a.E, nh = 2 * A;
  const int row0 = blockIdx.x * R;
  const SynthArgs& sv = a.env;

  // ---- prologue: this lane's weights in chain order (W1 row, W2 row positions 0..127 in
  // registers, 128..255 in LDS shared by the two rows), staged head rows, env state ----
  float w1r[OP], w2r[128];
#pragma unroll
  for (int t = 0; t < NTO; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f4 v = ld4(P + T.W1 + (long)f * OP + 16 * t + 4 * g);
#pragma unroll
      for (int c = 0; c < 4; ++c) w1r[16 * t + 4 * c + g] = v[c];
    }
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f4 v = ld4(P + T.W2 + (long)f * H + 16 * t + 4 * g);
#pragma unroll
      for (int c = 0; c < 4; ++c) w2r[16 * t + 4 * c + g] = v[c];
    }
  for (int i = tid; i < 128 * H; i += kRVThreads) {
    const int pp = i / H, ff = i - pp * H;  // chain position 128 + pp of feature ff's row
    W2L[((pp >> 2) * H + ff) * 4 + (pp & 3)] = P[T.W2 + (long)ff * H + 128 + chain_pos(pp)];
  }
  const float b1 = P[T.b1 + f], b2 = P[T.b2 + f];
  const float g1 = P[T.g1 + f], be1 = P[T.be1 + f], g2 = P[T.g2 + f], be2 = P[T.be2 + f];
  for (int i = tid; i < NHP * H; i += kRVThreads) {
    const int h = i / H, k = i - h * H;
    const int hr = act_head_row(K, 1, h);
    W3[i] = hr >= 0 ? P[hr + k] : 0.0f;
  }
  if (tid < NHP) {
    const int hbo = act_head_bias(K, 1, tid);
    HBIAS[tid] = hbo >= 0 ? P[hbo] : 0.0f;
  }
  for (int i = tid; i < OP; i += kRVThreads) {
    NRM[i] = i < O ? P[K.omean + i] : 0.0f;
    NRM[OP + i] = i < O ? P[K.ostd + i] : 1.0f;
  }
  for (int idx = tid; idx < R * O; idx += kRVThreads) {
    const int r = idx / O, ff = idx - r * O, e = row0 + r;
    XO[r * LDQ + ff] = e < E ? a.next_obs[(long)e * O + ff] : 0.0f;
    Q[r * LDQ + ff] = e < E ? sv.q[(long)e * O + ff] : 0.0f;
  }
  if (tid < R) {
    const int e = min(row0 + tid, E - 1);
    EV[EV_DONE * R + tid] = a.next_done[e];
    EVI[EV_AR * R + tid] = sv.autoreset[e];
    EVI[EV_T * R + tid] = sv.t[e];
    EVI[EV_RSEED * R + tid] = (int)sv.rseed[e];
    EVI[EV_RCOUNT * R + tid] = (int)sv.rcount[e];
    EV[EV_EPR * R + tid] = sv.ep_ret[e];
    EVI[EV_EPL * R + tid] = sv.ep_len[e];
    EV[EV_FR * R + tid] = sv.fin_ret[e];
    EV[EV_FL * R + tid] = sv.fin_len[e];
    EV[EV_FC * R + tid] = sv.fin_cnt[e];
  }
  lds_barrier();
  const SampleKey key = sample_key(a.seed, a.rank);
  const float hi = P[K.hi], lo = P[K.lo];
  // Beta items (row, action, alpha | beta) spread evenly over waves 1-7, which are idle during the
  // env step (wave 0): the next step's first Marsaglia-Tsang draws are computed there. An even
  // count per wave keeps an action's alpha and beta items in adjacent lanes (2 m, 2 m + 1)
  const int bper = 2 * ((R * A + 6) / 7);
  const int bitem = (wave > 0 && lane < bper) ? (wave - 1) * bper + lane : R * A * 2;
  auto draw0 = [&](long step) {
    GammaDraw d = GammaDraw{0.f, 0.f};
    if (bitem < R * A * 2) {
      const int which = bitem & 1, ra = bitem >> 1, r = ra / A, ai = ra - r * A;
      d = gamma_draw(key, (long)(row0 + r), step, 0x10000u + (uint32_t)(ai * 2 + which) * 64u);
    }
    return d;
  };
  GammaDraw gd0 = draw0(a.step0);
  // LayerNorm statistics lanes: (old wave ow, row r, lane group g), 8 R x 4 of them (wave 0)
  constexpr int NSL = 8 * R * 4;
  const int sg = tid & 3, sr = (tid >> 2) & (R - 1), sow = tid / (4 * R);
  // LayerNorm of the layer outputs in ZL (k_act3 act_activate's statistics, bitwise): mean and
  // 1 / std of row r, every thread; 2 barriers
  auto ln_stats = [&](float (&mu)[R], float (&rs)[R]) {
    f4 va = f4{0.f, 0.f, 0.f, 0.f}, vb = va;
    if (tid < NSL) {
      va = *reinterpret_cast<const f4*>(ZL + sr * LDZ + 32 * sow + 4 * sg);
      vb = *reinterpret_cast<const f4*>(ZL + sr * LDZ + 32 * sow + 16 + 4 * sg);
      float s = (va.x + va.y) + (va.z + va.w) + ((vb.x + vb.y) + (vb.z + vb.w));
      s = s + dpp_f<kDppQuadXor1>(s);
      s = s + dpp_f<kDppQuadXor2>(s);
      if (sg == 0) RS[sow * R + sr] = s;
    }
    lds_barrier();
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < kActWaves; ++w) t += RS[w * R + r];
      mu[r] = t * (1.0f / 256);
    }
    if (tid < NSL) {
      float q = 0.f;
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float d = (u ? vb : va)[c] - mu[sr];
          q = __fmaf_rn(d, d, q);
        }
      q = q + dpp_f<kDppQuadXor1>(q);
      q = q + dpp_f<kDppQuadXor2>(q);
      if (sg == 0) RS[(8 + sow) * R + sr] = q;
    }
    lds_barrier();
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < kActWaves; ++w) v += RS[(8 + w) * R + r];
      rs[r] = 1.0f / sqrtf(__fmaf_rn(v, 1.0f / 256, 1e-5f));
    }
    // no barrier for RS's reuse: the next call writes the sums only after other barriers, and the
    // squares only after its own first barrier, which every reader of these squares passes first
  };
  const int kl = lane & 15;  // this lane's position in its 16-lane row
  const float* xv = XV + rg * 64 + kl * 4;
  const float* hv = HV + rg * 16 * GE::LDK + kl * GE::LDK;
  for (int t = 0; t < a.T; ++t) {
    const long step_id = a.step0 + t;
    ROLL_STAMP(t, 0);
#ifdef PPO_STAMPS
    const int dbg_r = (t == 0 && kRdbgEnv == row0 + rg) ? rg : -1;
#endif
    // ---- inputs: rollout stores of obs[t] / dones[t]; normalised rows into XV (chain order) ----
    for (int idx = tid; idx < R * OP; idx += kRVThreads) {
      const int r = idx / OP, ff = idx - r * OP, e = row0 + r;
      const bool valid = e < E && ff < O;
      const float x = valid ? XO[r * LDQ + ff] : 0.0f;
      if (valid) a.s_obs[((long)t * E + e) * O + ff] = x;
      const int p = chain_pos(ff);
      XV[r * 64 + (p & 15) * 4 + (p >> 4)] = valid ? (x - NRM[ff]) / NRM[OP + ff] : x;
    }
    if (tid < R && row0 + tid < E) a.s_dones[(long)t * E + row0 + tid] = EV[EV_DONE * R + tid];
    lds_barrier();
    ROLL_STAMP(t, 1);
    // ---- layer 1 (k_act3's chain from the bias), one row per 4 waves ----
    float acc = b1;
    {
      const f4 x = *reinterpret_cast<const f4*>(xv);  // positions kl, 16 + kl
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_nop 1" ::: "memory");
      static_for<OP>([&](auto P) {
        constexpr int p = decltype(P)::value;
        fmac_bc<p & 15>(acc, x[p >> 4], w1r[p]);
      });
    }
    ZL[rg * LDZ + f] = acc;
#ifdef PPO_STAMPS
    if (dbg_r >= 0) RDBG(1, f, acc);
#endif
    lds_barrier();
    float mu[R], rs[R];
    ln_stats(mu, rs);
    {
      const float y = __fmaf_rn(g1, (acc - mu[rg]) * rs[rg], be1);
      const int p = chain_pos(f);
      HV[rg * 16 * GE::LDK + (p & 15) * GE::LDK + (p >> 4)] = y > 0.0f ? y : 0.0f;
#ifdef PPO_STAMPS
      if (dbg_r >= 0) RDBG(1, 260 + f, y > 0.0f ? y : 0.0f);
#endif
    }
    lds_barrier();
    ROLL_STAMP(t, 5);
    // ---- layer 2: weights of chain positions 0..127 from registers, 128..255 from LDS; the
    // inputs (this row's 256 h1 values, 16 per lane, the same in every 16-lane row) by row_newbcast ----
    acc = b2;
    {
      float x[16];
#pragma unroll
      for (int i = 0; i < 16; i += 4) *reinterpret_cast<f4*>(x + i) = *reinterpret_cast<const f4*>(hv + i);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_nop 1" ::: "memory");
      static_for<128>([&](auto P) {
        constexpr int p = decltype(P)::value;
        fmac_bc<p & 15>(acc, x[p >> 4], w2r[p]);
      });
      static_for<32>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        if constexpr (q % 8 == 0) __builtin_amdgcn_sched_barrier(0);  // bound the weight reads in flight
        const f4 w = *reinterpret_cast<const f4*>(W2L + (q * H + f) * 4);
        static_for<4>([&](auto C) {
          constexpr int c = decltype(C)::value, p = 128 + 4 * q + c;
          fmac_bc<p & 15>(acc, x[p >> 4], w[c]);
        });
      });
    }
    ZL[rg * LDZ + f] = acc;
#ifdef PPO_STAMPS
    if (dbg_r >= 0) RDBG(1, 516 + f, acc);
#endif
    lds_barrier();
    ROLL_STAMP(t, 6);
    ln_stats(mu, rs);
    {
      const float y = __fmaf_rn(g2, (acc - mu[rg]) * rs[rg], be2);
      H2[rg * LDZ + f] = y > 0.0f ? y : 0.0f;
#ifdef PPO_STAMPS
      if (dbg_r >= 0) RDBG(1, 776 + f, y > 0.0f ? y : 0.0f);
#endif
    }
    lds_barrier();
    ROLL_STAMP(t, 7);
    // ---- heads: (head, old wave, row) partials in the MFMA chain order of that wave's features ----
    for (int idx = tid; idx < nh * 8 * R; idx += kRVThreads) {
      const int r = idx % R, ow = (idx / R) & 7, h = idx / (8 * R);
      float hp = 0.f;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        f4 wq[4], xq[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          wq[g] = *reinterpret_cast<const f4*>(W3 + h * H + 32 * ow + 16 * u + 4 * g);
          xq[g] = *reinterpret_cast<const f4*>(H2 + r * LDZ + 32 * ow + 16 * u + 4 * g);
        }
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int g = 0; g < 4; ++g) hp = __builtin_fmaf(wq[g][c], xq[g][c], hp);
      }
      HP[(ow * NHP + h) * R + r] = hp;
#ifdef PPO_STAMPS
      if (t == 0 && kRdbgEnv == row0 + r) RDBG(1, 1032 + ow * 16 + h, hp);
#endif
    }
    lds_barrier();
    ROLL_STAMP(t, 2);
    // ---- Beta sample (k_rollout / k_act3 stages 1 and 2): the alpha and beta items of an action
    // sit in adjacent lanes, so stage 2 takes the partner's concentration and gamma sample by DPP
    // (quad xor 1) instead of a round trip through LDS and a barrier ----
    float bc = 1.0f, bg = 1.0f;
    if (bitem < R * A * 2) {
      const int which = bitem & 1, ra = bitem >> 1, r = ra / A, ai = ra - r * A, h = ai + which * A;
      float sm = 0.f;
#pragma unroll
      for (int w = 0; w < kActWaves; ++w) sm += HP[(w * NHP + h) * R + r];
      bc = softplusf_(sm + HBIAS[h]) + 1.0f;
#ifdef PPO_STAMPS
      if (t == 0 && kRdbgEnv == row0 + r) RDBG(1, 1160 + h, sm + HBIAS[h]);
#endif
      const uint32_t db = 0x10000u + (uint32_t)(ai * 2 + which) * 64u;
      bg = gamma_mt_d0(bc, gd0, key, (long)(row0 + r), step_id, db);
    }
    {
      const float pc = dpp_f<kDppQuadXor1>(bc), pg = dpp_f<kDppQuadXor1>(bg);  // every lane of the wave
      if (bitem < R * A * 2 && (bitem & 1) == 0) {
        const int ra = bitem >> 1, r = ra / A, ai = ra - r * A, e = row0 + r;
        const float al = bc, be = pc;
        const float s01 = bg / (bg + pg);
        const float act = (s01 - 0.0f) / (1.0f - 0.0f) * (hi - lo) + lo;
        ACT[r * 24 + ai] = act;
        if (e < E) {
          a.s_actions[((long)t * E + e) * A + ai] = act;
          float* d = a.s_beta + (((long)t * E + e) * A + ai) * 3;
          d[0] = al;
          d[1] = be;
          d[2] = s01;
        }
      }
    }
    lds_barrier();
    ROLL_STAMP(t, 3);
    // ---- env step (k_rollout's: 32 lanes per env) ----
    if (tid < 32 * R) {
#pragma clang fp contract(off)
      const int r = tid >> 5, i0 = tid & 31, e = row0 + r;
      const bool live = e < E;
      const bool reset = EVI[EV_AR * R + r] != 0;
      float* q = Q + r * LDQ;
      float* xo = XO + r * LDQ;
      const float* ar = ACT + r * 24;
      if (live && reset) {
        const uint32_t rsd = (uint32_t)EVI[EV_RSEED * R + r], rc = (uint32_t)EVI[EV_RCOUNT * R + r];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          const int i = 32 * c + i0;
          if (i < O) {
            uint32_t rr[4];
            philox4x32(rc, (uint32_t)i, 0u, 0u, rsd, 0x5EED5EEDu, rr);
            const float v = (0.1f * ((2.0f * u01(rr[0])) - 1.0f));
            q[i] = v;
            xo[i] = v;
          }
        }
        if (i0 == 0) {
          EVI[EV_RCOUNT * R + r] = (int)(rc + 1);
          EVI[EV_T * R + r] = 0;
          EV[EV_EPR * R + r] = 0.0f;
          EVI[EV_EPL * R + r] = 0;
          EV[EV_DONE * R + r] = 0.0f;
          EVI[EV_AR * R + r] = 0;
          a.s_rewards[(long)t * E + e] = 0.0f;
        }
      } else if (live) {
        float qo[NCH], qn[NCH];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          const int i = 32 * c + i0;
          qo[c] = i < O ? q[i] : 0.0f;
          qn[c] = i < O ? q[i + 1 < O ? i + 1 : 0] : 0.0f;
        }
        float q0_new = 0.0f;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          const int i = 32 * c + i0;
          if (i < O) {
            const float ai = fminf(fmaxf(ar[i % A], a.lo), a.hi);
            const float nq = __fmaf_rn(0.9f, qo[c], __fmaf_rn(0.1f, ai, (0.05f * qn[c])));
            q[i] = nq;
            xo[i] = nq;
            if (c == 0) q0_new = nq;
          }
        }
        if (i0 == 0) {
          const float vel = ((q0_new - qo[0]) / 0.05f);
          float ctrl = 0.0f;
          for (int k = 0; k < A; ++k) {
            const float ak = fminf(fmaxf(ar[k], a.lo), a.hi);
            ctrl = (ctrl + ((0.1f * ak) * ak));
          }
          const float rw = (vel - ctrl);
          const int tt = EVI[EV_T * R + r] + 1;
          EVI[EV_T * R + r] = tt;
          const bool tr = tt >= 1000;
          a.s_rewards[(long)t * E + e] = rw;
          EV[EV_DONE * R + r] = tr ? 1.0f : 0.0f;
          const float epr = (EV[EV_EPR * R + r] + rw);
          EV[EV_EPR * R + r] = epr;
          const int epl = EVI[EV_EPL * R + r] + 1;
          EVI[EV_EPL * R + r] = epl;
          if (tr) {
            EV[EV_FR * R + r] += epr;
            EV[EV_FL * R + r] += (float)epl;
            EV[EV_FC * R + r] += 1.0f;
          }
          EVI[EV_AR * R + r] = tr ? 1 : 0;
        }
      }
    }
    // the first Marsaglia-Tsang attempt's draws of the next step (independent of the network)
    if (wave > 0 && t + 1 < a.T) gd0 = draw0(step_id + 1);
    lds_barrier();
    ROLL_STAMP(t, 4);
  }
  // ---- epilogue: next_obs / next_done and the env state back to HBM ----
  for (int idx = tid; idx < R * O; idx += kRVThreads) {
    const int r = idx / O, ff = idx - r * O, e = row0 + r;
    if (e < E) {
      a.next_obs[(long)e * O + ff] = XO[r * LDQ + ff];
      sv.q[(long)e * O + ff] = Q[r * LDQ + ff];
    }
  }
  if (tid < R && row0 + tid < E) {
    const int e = row0 + tid;
    a.next_done[e] = EV[EV_DONE * R + tid];
    sv.autoreset[e] = EVI[EV_AR * R + tid];
    sv.t[e] = EVI[EV_T * R + tid];
    sv.rseed[e] = (uint32_t)EVI[EV_RSEED * R + tid];
    sv.rcount[e] = (uint32_t)EVI[EV_RCOUNT * R + tid];
    sv.ep_ret[e] = EV[EV_EPR * R + tid];
    sv.ep_len[e] = EVI[EV_EPL * R + tid];
    sv.fin_ret[e] = EV[EV_FR * R + tid];
    sv.fin_len[e] = EV[EV_FL * R + tid];
    sv.fin_cnt[e] = EV[EV_FC * R + tid];
  }
}

// =============================================================================================
// launchers
// =============================================================================================
int rollout_supported(const PackedLayout& K) {
  const int nto = K.OP / 16;
  if (K.kind == PPO_NET_LN_BETA && K.H == 256 && 2 * K.A <= 16) return (nto == 1 || nto == 2 || nto == 7) ? 0 : -1;
  if (K.kind == PPO_NET_TANH_NORMAL && K.H == 64 && K.A <= 32)
    return (nto == 1 || nto == 2 || nto == 7 || nto == 24) ? 0 : -1;
  return -1;
}

// 4 envs per workgroup while that still fits one workgroup per CU (the kernel's registers allow
// one), 16 beyond
template <int NTO, int NHT>
static int launch_rollout4_t(const RolloutArgs& a, hipStream_t s) {
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  if ((a.E + 3) / 4 <= ncu)
    hipLaunchKernelGGL((k_rollout4<NTO, NHT, 4>), dim3((a.E + 3) / 4), dim3(kR4Threads), 0, s, a);
  else
    hipLaunchKernelGGL((k_rollout4<NTO, NHT, 16>), dim3((a.E + 15) / 16), dim3(kR4Threads), 0, s, a);
  return 0;
}
template <int NTO>
static int launch_values4_t(const ValuesArgs& a, hipStream_t s) {
  const long nblk = (a.n + kR4Rows - 1) / kR4Rows;
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const long grid = nblk < 2L * ncu ? nblk : 2L * ncu;
  hipLaunchKernelGGL((k_values4<NTO>), dim3((unsigned)grid), dim3(kR4Threads), 0, s, a);
  return 0;
}

template <int NTO, int NHT>
static int launch_rollout_t(const RolloutArgs& a, hipStream_t s) {
  using GE = RollGeo<NTO, NHT>;
  const size_t lds = (size_t)GE::total * sizeof(float);
  static const bool ok = hipFuncSetAttribute((const void*)k_rollout<NTO, NHT>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess;
  if (!ok) return -2;
  hipLaunchKernelGGL((k_rollout<NTO, NHT>), dim3((a.E + kRows - 1) / kRows), dim3(kActThreads), lds, s, a);
  return 0;
}

template <int NTO>
static int launch_rollout_v_t(const RolloutArgs& a, hipStream_t s) {
  const size_t lds = (size_t)RollVGeo<NTO>::total * sizeof(float);
  static const bool ok = hipFuncSetAttribute((const void*)k_rollout_v<NTO>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)lds) == hipSuccess;
  if (!ok) return -2;
  hipLaunchKernelGGL((k_rollout_v<NTO>), dim3((a.E + 1) / 2), dim3(kRVThreads), lds, s, a);
  return 0;
}

// the VALU rollout where it applies: AC agent, O <= 32, and few envs (auto: E <= 512, the N = 8
// shard of the metric config); a.variant 1 forces k_rollout, 2 k_rollout_v
static bool use_rollout_v(const RolloutArgs& a) {
  if (a.K.kind != PPO_NET_LN_BETA || a.K.OP > 32 || a.env.w.on || !a.s_beta || a.variant == 1) return false;
  return a.variant == 2 || a.E <= 512;
}

int launch_rollout(const RolloutArgs& a, hipStream_t s) {
  if (rollout_supported(a.K) != 0) return -1;
  // an explicit rollout_kernel=valu that cannot apply is an error, not a silent k_rollout
  if (a.variant == 2 && !use_rollout_v(a)) return -3;
  if (use_rollout_v(a)) return a.K.OP == 16 ? launch_rollout_v_t<1>(a, s) : launch_rollout_v_t<2>(a, s);
  if (a.K.kind == PPO_NET_TANH_NORMAL) {
    const int nht = (a.K.A + 15) / 16;
    switch (a.K.OP / 16) {
      case 1: return nht == 1 ? launch_rollout4_t<1, 1>(a, s) : launch_rollout4_t<1, 2>(a, s);
      case 2: return nht == 1 ? launch_rollout4_t<2, 1>(a, s) : launch_rollout4_t<2, 2>(a, s);
      case 7: return nht == 1 ? launch_rollout4_t<7, 1>(a, s) : launch_rollout4_t<7, 2>(a, s);
      case 24: return nht == 1 ? launch_rollout4_t<24, 1>(a, s) : launch_rollout4_t<24, 2>(a, s);
    }
    return -1;
  }
  if (a.env.w.on) return -1;
  switch (a.K.OP / 16) {
    case 1: return launch_rollout_t<1, 1>(a, s);
    case 2: return launch_rollout_t<2, 1>(a, s);
    case 7: return launch_rollout_t<7, 1>(a, s);
  }
  return -1;
}

template <int NTO, int NHT>
static int launch_values_t(const ValuesArgs& a, hipStream_t s) {
  constexpr int R = val_rows<NTO>();
  using GE = RollGeo<NTO, NHT, R>;
  constexpr int total = GE::oXO + 2 * GE::OP;  // trunk regions + the observation statistics
  static_assert(total * sizeof(float) <= 160 * 1024, "k_values LDS above 160 KB");
  const size_t lds = (size_t)total * sizeof(float);
  static const bool ok = hipFuncSetAttribute((const void*)k_values<NTO, NHT>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess;
  if (!ok) return -2;
  const long nblk = (a.n + R - 1) / R;
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const long grid = nblk < ncu ? nblk : ncu;  // one resident workgroup per CU (registers hold the weights)
  hipLaunchKernelGGL((k_values<NTO, NHT>), dim3((unsigned)grid), dim3(kActThreads), lds, s, a);
  return 0;
}

int launch_values(const ValuesArgs& a, hipStream_t s) {
  if (rollout_supported(a.K) != 0) return -1;
  if (a.K.kind == PPO_NET_TANH_NORMAL) {
    switch (a.K.OP / 16) {
      case 1: return launch_values4_t<1>(a, s);
      case 2: return launch_values4_t<2>(a, s);
      case 7: return launch_values4_t<7>(a, s);
      case 24: return launch_values4_t<24>(a, s);
    }
    return -1;
  }
  switch (a.K.OP / 16) {
    case 1: return launch_values_t<1, 1>(a, s);
    case 2: return launch_values_t<2, 1>(a, s);
    case 7: return launch_values_t<7, 1>(a, s);
  }
  return -1;
}
