// ppo_act_narrow.hip — k_act4: Agent::get_action_and_value / get_value + rollout stores for the
// PPO agent (two 64-wide tanh trunks + Normal head, ppo:120-157, rollout step ppo:387-400),
// latency-first for wide observations (cfg2 Humanoid O = 376).
//
// A rollout launch is one pass over E rows with cold weights, so its time is the critical path of
// dependent memory round trips, not MFMA work. k_act2 (one trunk per workgroup, waves split the
// output features) streams the 376-wide W1 k-block by k-block: 24 dependent L2/MALL fetches.
// Here a 256-thread workgroup owns 16 rows of ONE trunk (the launch time is set by the weight bytes
// each CU must pull in, so the trunks go to different CUs), layer 1 is split over K (wave ks owns
// k-blocks [ks NKW, ks NKW + NKW) for all 64 outputs), and EVERY operand the wave needs — its input
// columns, its W1 slice, its W2 rows, head rows, biases and the per-item parameters and Normal
// draws — is requested at kernel start, so the launch costs about one round trip plus ~100 MFMAs
// per wave. Partial sums meet in LDS in a fixed order. Sampling uses the Philox contract of k_act2
// (same counters), so samples match it for any batching.
#include "ppo_agent.hpp"
#include "ppo_kernels.hpp"

namespace {
constexpr int kA4Threads = 256, kA4Rows = 16, kA4H = 64, kA4LDP = kA4Rows + 1, kA4LDH = kA4H + 4;
}

template <int NTO, int NHT>
__global__ __launch_bounds__(256) void k_act4(ActArgs a) {
  constexpr int H = kA4H, R = kA4Rows, OP = NTO * 16, NKW = (NTO + 3) / 4, NHP = NHT * 16;
  constexpr int LDP = kA4LDP, LDH = kA4LDH;
  __shared__ float P1[4][H][LDP];          // layer-1 partials per k-slice
  __shared__ __attribute__((aligned(16))) float H1[R][LDH];
  __shared__ float HP[4][NHP][LDP];        // actor head partials per k-slice (feature quarter)
  __shared__ float VP[4][R];               // critic head partials
  __shared__ float ITM[R * NHP][2];        // per (row, action): log-prob / entropy terms
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  const int trunk = blockIdx.y, ks = wave;
  const PackedLayout& K = a.K;
  const TrunkDev& T = K.tr[trunk];
  const float* __restrict__ P = a.P;
  const PBuf pb = make_pbuf(P, K.size);
  const PBuf wsw = make_pbuf(a.WSW[trunk], (int)sw_size(H, OP));  // swizzled W1 | W2 (sw_index)
  const int row0 = blockIdx.x * R, O = K.O, A = K.A;
  const int row = row0 + j, rowc = min(row, a.n - 1);
  const int kb0 = ks * NKW;

  // ---------------- kernel start: every independent load ----------------
  f4 xv[NKW], wa[NKW][4], w2v[4];
  f4 b1 = f4{0.f, 0.f, 0.f, 0.f}, b2 = b1, hv = b1, hw[NHT];
  {
#pragma unroll
    for (int q = 0; q < NKW; ++q) {
      const int kb = kb0 + q;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int col = 16 * kb + 4 * g + c;
        const float v = a.x[(size_t)rowc * a.ldx + min(col, O - 1)];  // unconditional, masked below
        xv[q][c] = (kb < NTO && col < O && row < a.n) ? v : 0.f;
      }
#pragma unroll
      for (int ft = 0; ft < 4; ++ft)
        wa[q][ft] = pld4(wsw, 4 * lane, 256 * (ft * NTO + min(kb, NTO - 1)));
    }
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) w2v[kb] = pld4(wsw, H * OP + 4 * lane, 256 * (4 * ks + kb));
    b1 = pld4(pb, T.b1 + 16 * ks + 4 * g, 0);
    b2 = pld4(pb, T.b2 + 16 * ks + 4 * g, 0);
    if (trunk == 0) hv = pld4(pb, K.cW3 + 16 * ks + 4 * g, 0);
#pragma unroll
    for (int ht = 0; ht < NHT; ++ht) {
      const int h = 16 * ht + j;
      const f4 w = pld4(pb, K.aW3 + min(h, A - 1) * H + 16 * ks + 4 * g, 0);
      hw[ht] = (trunk == 1 && h < A) ? w : f4{0.f, 0.f, 0.f, 0.f};
    }
  }
  // the rollout keeps the observation the action was taken on: the critic's waves hold every
  // (row, column) of the tile once between them, stored as soon as it arrives
  if (trunk == 0 && a.store_step >= 0 && row < a.n) {
    float* so = a.s_obs + ((long)a.store_step * a.E + a.env_base + row) * O;
#pragma unroll
    for (int q = 0; q < NKW; ++q)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int col = 16 * (kb0 + q) + 4 * g + c;
        if (kb0 + q < NTO && col < O) so[col] = xv[q][c];
      }
  }
  // per-item parameters (item tid + 256 u: row / A, action % A) and the Normal draws, which do not
  // depend on the network: all fetched / computed here, under the weight fetch
  constexpr int NI = (R * NHP + kA4Threads - 1) / kA4Threads;
  float i_b3[NI], i_lstd[NI], i_act[NI], nz[NI];
  float c_b3 = 0.f, c_done = 0.f;
  const SampleKey key = sample_key(a.seed, a.rank);
#pragma unroll
  for (int u = 0; u < NI; ++u) {
    const int idx = min(tid + kA4Threads * u, R * A - 1), ir = idx / A, ia = idx - ir * A, irow = row0 + ir;
    i_b3[u] = 0.f; i_lstd[u] = 0.f; i_act[u] = 0.f; nz[u] = 0.f;
    if (trunk == 1) {
      i_b3[u] = P[K.ab3 + ia];
      i_lstd[u] = P[K.logstd + ia];
      if (a.mode == PPO_GIVEN) i_act[u] = a.action_in[(size_t)min(irow, a.n - 1) * A + ia];
      if (a.mode == PPO_SAMPLE) {
        uint32_t rr[4];
        philox_draw(key, a.env_base + irow, a.step_id, (uint32_t)(ia >> 1), rr);
        float z0, z1;
        box_muller(rr[0], rr[1], z0, z1);
        nz[u] = (ia & 1) ? z1 : z0;
      }
    }
  }
  if (trunk == 0 && tid < R) {
    c_b3 = P[K.cb3];
    if (a.next_done) c_done = a.next_done[min(row0 + tid, a.n - 1)];
  }

  // ---------------- layer 1: partial products over this wave's k-blocks ----------------
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
#pragma unroll
    for (int ft = 0; ft < 4; ++ft)
#pragma unroll
      for (int r = 0; r < 4; ++r) P1[ks][16 * ft + 4 * g + r][j] = acc[ft][r];
  }
  __syncthreads();
  // ---------------- h1 tile ks = tanh(b1 + sum of the 4 k-slices) ----------------
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
  // ---------------- layer 2 (output tile ks), heads ----------------
  {
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
    if (trunk == 0) {
      float p = (hv.x * h2.x + hv.y * h2.y) + (hv.z * h2.z + hv.w * h2.w);
      p = row_allreduce(p);
      if (g == 0) VP[ks][j] = p;
    } else {
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
    }
  }
  __syncthreads();

  // ---------------- outputs ----------------
  if (trunk == 0 && tid < R) {
    const int rw = row0 + tid;
    if (rw < a.n) {
      const float v = (((VP[0][tid] + VP[1][tid]) + VP[2][tid]) + VP[3][tid]) + c_b3;
      if (a.value_out) a.value_out[rw] = v;
      if (a.store_step >= 0) {
        const long srow = (long)a.store_step * a.E + a.env_base + rw;
        a.s_values[srow] = v;
        a.s_dones[srow] = a.next_done ? c_done : 0.0f;
      }
    }
  }
#pragma unroll
  for (int u = 0; u < NI; ++u) {
    const int idx = tid + kA4Threads * u;
    if (trunk == 1 && idx < R * A) {
      const int ir = idx / A, ia = idx - ir * A, irow = row0 + ir;
      const long env = a.env_base + irow;
      const bool valid = irow < a.n;
      const float mu = (((HP[0][ia][ir] + HP[1][ia][ir]) + HP[2][ia][ir]) + HP[3][ia][ir]) + i_b3[u];
      const float sd = expf(i_lstd[u]);
      const float var = sd * sd, lsd = logf(sd);
      float act;
      if (a.mode == PPO_GIVEN) act = valid ? i_act[u] : 0.0f;
      else if (a.mode == PPO_MEAN) act = mu;
      else act = mu + nz[u] * sd;
      const float d = act - mu;
      ITM[idx][0] = -(d * d) / (2.0f * var) - lsd - kLz;
      ITM[idx][1] = kEntC + lsd;
      if (valid) {
        if (a.action_out) a.action_out[(size_t)irow * A + ia] = act;
        if (a.store_step >= 0) a.s_actions[((long)a.store_step * a.E + env) * A + ia] = act;
      }
    }
  }
  if (trunk == 0) return;
  __syncthreads();
  if (tid < R) {
    const int rw = row0 + tid;
    if (rw < a.n) {
      float lp = 0.f, ent = 0.f;
      for (int ai = 0; ai < A; ++ai) {
        lp += ITM[tid * A + ai][0];
        ent += ITM[tid * A + ai][1];
      }
      if (a.logprob_out) a.logprob_out[rw] = lp;
      if (a.entropy_out) a.entropy_out[rw] = ent;
      if (a.store_step >= 0) a.s_logp[(long)a.store_step * a.E + a.env_base + rw] = lp;
    }
  }
}

// H = 64 tanh-Normal agent (measured on MI355X, scripts/act_micro.py, O = 376: 21.7 vs 21.8 us at
// E = 1024 and 22.7 vs 35.6 us at E = 4096 against k_act2; at O = 17 k_act2's feature split is
// faster per launch, 6.3 vs 8.0 us, but k_act4 is the arithmetic of the persistent device-env
// rollout (k_rollout4) and of the critic pass, so every shape uses it: one summation order for the
// rollout, the values and the GAE bootstrap whichever env backend runs). Option act_kernel=2
// selects k_act2. Returns -1 when not covered (caller: k_act2).
int launch_act4(const ActArgs& a, hipStream_t s) {
  if (a.K.H != 64 || a.K.kind != PPO_NET_TANH_NORMAL || a.K.A > 32 || a.n <= 0) return -1;
  const int nto = a.K.OP / 16, nht = (a.K.A + 15) / 16;
  const dim3 grid((a.n + kA4Rows - 1) / kA4Rows, a.need_actor ? 2 : 1);
#define PPO_ACT4_CASE(NTO_, NHT_)                                                    \
  if (nto == NTO_ && nht == NHT_) {                                                  \
    hipLaunchKernelGGL((k_act4<NTO_, NHT_>), grid, dim3(kA4Threads), 0, s, a);       \
    return 0;                                                                        \
  }
  PPO_ACT4_CASE(1, 1) PPO_ACT4_CASE(2, 1) PPO_ACT4_CASE(7, 1) PPO_ACT4_CASE(24, 2) PPO_ACT4_CASE(2, 2)
  PPO_ACT4_CASE(24, 1)
#undef PPO_ACT4_CASE
  return -1;
}
