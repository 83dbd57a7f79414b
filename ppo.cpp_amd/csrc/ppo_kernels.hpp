// ppo_kernels.hpp — kernel argument blocks and launch wrappers (host <-> device contract).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "ppo_device.hpp"
#include "ppo_packed.hpp"

#include "../../include/ppo_hip.h"

struct ActArgs {
  const float* P;
  PackedLayout K;
  int n;
  const float* x;
  int ldx;
  int mode;
  int need_actor;
  const float* action_in;
  uint64_t seed;
  int rank;
  long env_base;
  long step_id;
  float* action_out;
  float* logprob_out;
  float* entropy_out;
  float* value_out;
  int store_step;  // < 0: no rollout stores
  int E;
  const float* next_done;
  float *s_obs, *s_actions, *s_logp, *s_dones, *s_values;
  int kernel;  // 0: fastest for the shape; 2 / 4: force k_act2 / k_act4 (A/B comparisons)
  const float* WSW[2];  // swizzled W1 | W2 | W2^T per trunk (k_act3)
  int skip_critic;      // k_act3, rollout stores: the critic workgroups store obs / dones only (deferred pass)
};

// A-operand ("swizzled") copies of a trunk's weight matrices: the 16 x 16 block (feature block fb,
// k-block kb) of a row-major [NR][NC] matrix is stored as 64 lane-major float4s, lane (j, g) =
// j + 16 g holding row 16 fb + j, columns 16 kb + 4 g .. + 3, i.e. exactly the float4 that lane
// reads as its MFMA A operand, so one wave-load reads 1 KB contiguous (the row-major layout reads
// 16 rows x 64 B: ~2.6x less L2 throughput, scripts/probe/l2bw_probe.hip). Per trunk:
// [W1 (H x OP) | W2 (H x H) | W2^T (H x H)], refreshed by k_adam with the parameters.
PPO_DEV_HOST inline long sw_index(int r, int c, int ncols) {
  return ((long)((r >> 4) * (ncols >> 4) + (c >> 4)) * 64 + ((c & 15) >> 2) * 16 + (r & 15)) * 4 + (c & 3);
}
PPO_DEV_HOST inline long sw_size(int H, int OP) { return (long)H * OP + 2L * H * H; }

// Split-bf16 pieces. Every fp32 x is the exact sum of three bf16 numbers: hi = x with the low 16
// bits cleared (truncation), r = x - hi (exact: a prefix of x's significand is removed), mid = r
// truncated the same way, lo = r - mid (exact, at most 8 significant bits: a bf16). A product a.b is
// then a sum of piece products, each exact in fp32.
PPO_DEV_HOST inline void split3_bits(float x, uint16_t (&pc)[3]) {
  const uint32_t u = __builtin_bit_cast(uint32_t, x);
  const float r = x - __builtin_bit_cast(float, u & 0xffff0000u);
  const uint32_t v = __builtin_bit_cast(uint32_t, r);
  const float l = r - __builtin_bit_cast(float, v & 0xffff0000u);
  pc[0] = (uint16_t)(u >> 16);
  pc[1] = (uint16_t)(v >> 16);
  pc[2] = (uint16_t)(__builtin_bit_cast(uint32_t, l) >> 16);
}
// Piece copies of W2 | W2^T for k_upd's split-bf16 GEMMs (create option upd_mfma=bx6), stored after a
// trunk's fp32 swizzled copies (H = 256 contexts). Element (r, c) of an [NR][NC] matrix, piece p, sits
// (in bf16 units) where lane (j, g) = j + 16 g reads it as the v_mfma_f32_16x16x32_bf16 A operand of
// feature block r >> 4 and 32-wide k block c >> 5: element e = 4 ((c >> 4) & 1) + (c & 3) of the
// lane's 16-byte piece p, i.e. lane k slot 8 g + e holds column 32 kk + 16 (e >> 2) + 4 g + (e & 3) —
// the columns k_upd's 16x16x4 form gives lane group g in its two k-blocks 2 kk, 2 kk + 1. One
// wave-load of a piece is 1 KB contiguous.
PPO_DEV_HOST inline long bx_index(int r, int c, int ncols, int p) {
  const int lane = (r & 15) + 16 * ((c & 15) >> 2), e = 4 * ((c >> 4) & 1) + (c & 3);
  return ((((long)(r >> 4) * (ncols >> 5) + (c >> 5)) * 3 + p) * 64 + lane) * 8 + e;
}
PPO_DEV_HOST inline long bx_size(int H) { return 3L * H * H; }  // floats: W2 | W2^T pieces
// the 64-wide agent (k_upd2's split-bf16 layer 1): the pieces of W1 (H x OP) instead, same layout
PPO_DEV_HOST inline long bx_w1_size(int H, int OP) { return 3L * H * OP / 2; }
// floats of a trunk's piece region (after its fp32 swizzled copies)
PPO_DEV_HOST inline long bx_region(int H, int OP) { return H == 256 ? bx_size(H) : H == 64 ? bx_w1_size(H, OP) : 0; }

struct UpdArgs {
  const float* P;
  const float* W2T[2];
  const float* WSW[2];  // swizzled W1 | W2 | W2^T per trunk (sw_index)
  PackedLayout K;
  SmallGradLayout sg[2];
  int M;
  int tiles_per_block;
  int wlds_off;  // float offset of the weight staging buffers in dynamic LDS
  const int32_t* perm;
  const float *obs, *actions, *logp, *adv, *ret, *val;
  long rows_n, obs_n;      // rollout storage rows (T E) and obs floats (T E O): k_upd2's buffer descriptors
  const float* adv_stats;  // [2] mean, std of this minibatch
  float clip_coef, ent_coef, vf_coef, inv_m;
  int clip_vloss, norm_adv;
  float* Xn;
  float* H1[2];
  float* DZ1[2];
  float* DZ2[2];
  float* slab[2];
  int actn_off, acc_off, spar_off;  // k_upd: runtime LDS offsets (floats)
  int hw_global;                    // k_upd: the actor's dW3 accumulators live in its slab row (UpdGeoOut)
  float* Z1;              // k_l1g -> k_upd2 (split form): layer-1 pre-activations [M][128], critic | actor
  int trunk_mask;         // k_upd: trunks to run (bit t = trunk t; 3 = both; other values: PPO_DIAG builds only)
  int sched;              // k_upd: bit 0 actor workgroups dispatched first, bit 1 actor wave priority
  int hot;                // diagnostic build only (PPO_UPD2_HOT): k_upd2 gathers the rows of its first 8 tiles only
  int bx;                 // k_upd: 1 runs the 256-wide GEMMs as split-bf16 piece products (upd_mfma=bx6);
                          // k_upd2: 2 runs layer 1 that way
  int h1_skip;            // k_upd: no H1 hand-off rows; LNS gets each row's layer-1 LayerNorm (mean, 1 / std)
  float* LNS[2];          //   [M][2] per trunk, from which k_dwf_bx recomputes H1 (h1_handoff=recompute)
};

// k_upd geometry (ppo_update.hip)
#define PPO_UPD_MAXA 24
struct UpdGeoOut {
  size_t lds_bytes;
  int actn_off, acc_off, spar_off, rows;
  int hw_global;  // 1: the actor's head-weight gradient accumulates in its slab row, not in LDS
};

struct DwArgs {
  const float* dz2[2];
  const float* h1[2];
  const float* dz1[2];
  const float* xn;
  const int32_t* perm;  // non-null: dW1's input rows are gathered as obs[perm[m]] (O wide, zero padded to OP)
  const float* obs;     //   instead of read from xn (k_upd2: no input normalisation, no Xn round trip)
  long obs_n;           // floats in obs (k_dw2_dma's buffer descriptor)
  int O;
  float* slab[2];     // [nchunks][H*H + H*OP] per trunk
  long slab_stride;
  int M;
  int rows_per_chunk;
  int fused;          // 1: k_dwf (dW2 and dW1 in one pass) where it applies; 0: two-phase k_dw
  int slices;         // k_dwf: output-row slices per chunk (grid z); 2 halves the chunks, so the
                      // split-K partials, for small minibatches (dw_slices)
  int dma;            // k_dwf: 1 stages the rows by LDS DMA, three buffers (k_dwf_dma), bitwise k_dwf
  int bx;             // k_dwf: 8 / 9 runs the products as exact bf16 piece products (k_dwf_bx); 0 fp32 MFMA
  int hot;            // diagnostic build only (PPO_DW_HOT): every stage re-reads the chunk's first rows (L2-hot)
  // h1_recompute (k_dwf_bx, LayerNorm agent): H1 is not read; each 16-row stage recomputes it from the Xn
  // rows it stages anyway, k_upd's layer-1 chain (W1 swizzled copy, bias init, 16x16x4 fp32 MFMAs in the
  // same k order, kl1 = k-steps of the last k block) and the rows' LayerNorm statistics lns: bitwise k_upd's
  // H1
  int h1_recompute, kl1;
  const float* lns[2];
  const float* w1sw[2];                          // WSW[trunk] (W1 swizzled block first)
  const float *b1[2], *g1[2], *be1[2];           // layer-1 bias and LayerNorm affine (parameters)
};
// k_dwf output slices and dW row chunks for a minibatch of M rows: 128 chunks per trunk (one
// workgroup per CU over both trunks); below 32 K rows 64 chunks x 2 output halves instead — the
// same 256 workgroups, half the split-K partial bytes written by k_dwf and read back by k_colsum
inline int dw_slices(int M, int H, int OP, bool fused) { return (fused && H == 256 && OP <= 32 && M <= 32768) ? 2 : 1; }

struct ColsumSeg {
  const float* src;
  float* dst;
  long stride;
  int count;
  int len;
  float scale;
};
#define PPO_MAX_SEGS 40
struct ColsumArgs {
  ColsumSeg seg[PPO_MAX_SEGS];
  int tile0[PPO_MAX_SEGS + 1];  // first 64-float tile of each segment (set by launch_colsum)
  int nseg;
  // gradient-norm fold (create option gradnorm=fold): each tile of a segment that is a whole norm
  // tensor (seg_t = its NormArgs index, -1: none) stores the sum of squares of the values it wrote in
  // sq[tile]; the segment's last tile (counter cnt[seg]) adds them in tile order into
  // part[seg_t * PPO_GN_SPLIT] (the other slices 0) — k_gradnorm's output, one launch fewer
  int fold;
  int seg_t[PPO_MAX_SEGS];
  float* sq;
  unsigned* cnt;
  float* part;
};

struct NormArgs {
  const float* grad;
  int nt;
  int off[PPO_LAYOUT_MAX_TENSORS];
  int len[PPO_LAYOUT_MAX_TENSORS];
  float max_norm;
  float* out;   // [0] total norm, [1] clip coefficient, [2 + t] per-tensor norms (written by k_adam)
  float* part;  // [nt][PPO_GN_SPLIT] partial sums of squares
};
#define PPO_GN_SPLIT 16

struct AdamArgs {
  float* param;
  const float* grad;
  float *m, *v;
  long begin, n;
  float* norm_out;
  const float* part;  // k_gradnorm partials
  float* stat_out;    // optional: total norm of this step (minibatch stats slot)
  int nt;
  float max_norm;
  float step_size, sbc2, eps;
  long w2_off[2];
  float* w2t[2];
  int H;
  long w1_off[2];
  float* wsw[2];  // swizzled copies (sw_index), refreshed with the parameters
  int OP;
  // update graph (create option update_graph=1): the step size and sqrt(1 - 0.999^t) of minibatch gi
  // come from sched[2 gi], sched[2 gi + 1] (written by the host before every replay) instead of
  // step_size / sbc2, so the captured launch sequence stays valid across iterations
  const float* sched;
  int gi;
  int bx;  // also refresh the split-bf16 pieces (bx_index) after each wsw copy: 1 of W2 | W2^T, 2 of W1
};

struct GaeArgs {
  const float *rewards, *values, *dones, *next_value, *next_done;
  float *adv, *ret;
  int T, E;
  float gamma, lam;
};

struct AdvArgs {
  const int32_t* perm;  // [nmb][M]
  const float* adv;
  float* stats;         // [nmb][2]
  float* sq;            // [nmb]
  double* part;         // [nmb][PPO_ADV_SPLIT] slice partial sums
  int M, nmb, world;
};
#define PPO_ADV_SPLIT 32

// The PPO trainer's env wrapper chain behind a device vector env (ppo:41-49; include/ppo_env_wrappers.h),
// one state per env in one allocation of 2*E*O + 5*E floats (the oracle's orc_vwrap_* layout).
struct WrapArgs {
  float* om;      // [E][O] NormalizeObservation mean_ (stateful_observation.h:56-84)
  float* ov;      // [E][O] var_
  float* ocount;  // [E]    count_
  float* rmean;   // [E]    NormalizeReward mean_ / var_ / accumulated_reward_ / count_ (stateful_reward.h:55-91)
  float* rvar;
  float* racc;
  float* rcount;
  float gamma;
  int on;         // 0: no chain (the AC trainer's envs, ac:50-53)
};

#define PSYN_MAXO 384  // device synthetic env: max observation width (k_synth_step_wide above 32)
struct SynthArgs {
  WrapArgs w;  // applied inside the env's own kernels when w.on
  int E, O, A;
  float* q;
  int* t;
  int* autoreset;
  uint32_t* rseed;
  uint32_t* rcount;
  float* ep_ret;
  int* ep_len;
  float* fin_ret;
  float* fin_len;
  float* fin_cnt;
};

// Persistent device-env rollout (ppo_rollout.hip, k_rollout): all T steps of act + env step in one
// launch, one 16-env block per workgroup, the actor's weights resident in registers.
struct RolloutArgs {
  const float* P;
  PackedLayout K;
  const float* WSW;     // actor trunk's swizzled W1 | W2 | W2^T
  int E, T;
  long step0;           // Philox step counter of step 0 (iteration * T)
  uint64_t seed;
  int rank;
  float* next_obs;      // [E][O] in: the obs of step 0; out: the obs after step T-1
  float* next_done;     // [E]
  float *s_obs, *s_actions, *s_logp, *s_dones, *s_rewards;
  float* s_beta;        // AC: [T][E][A][3] (alpha, beta, sample) for k_beta_logp; null: log-probs in the loop
  SynthArgs env;
  float lo, hi;         // the env's action space (clip_actions)
  int variant;          // AC rollout kernel: 0 auto, 1 k_rollout (MFMA, 16 envs per workgroup), 2 k_rollout_v (VALU)
};
// Critic forward over n stored rows (ppo_rollout.hip, k_values): values[i] = critic(obs[i]), the
// same chain as k_act3's critic workgroups, so each value is bitwise the one the per-step act
// kernel stores.
struct ValuesArgs {
  const float* P;
  PackedLayout K;
  const float* WSW;     // critic trunk's swizzled copy
  const float* obs;     // [n][O]
  float* values;        // [n]
  long n;
  const float* WBX;     // non-null: the critic's W2 pieces (bx_index): layer 2 as split-bf16 products (k_vbx)
};
int launch_vbx(const ValuesArgs& a, hipStream_t s);  // ppo_update.hip; -1 when the shape is not covered
int rollout_supported(const PackedLayout& K);
int launch_rollout(const RolloutArgs& a, hipStream_t s);
int launch_values(const ValuesArgs& a, hipStream_t s);
int launch_beta_logp(const float* s_beta, float* logp, long n, int A, hipStream_t s);

// sets the thread-local ppo_last_error() message and returns code (ppo_capi.hip)
int ppo_fail(const std::string& msg, int code);

int launch_act(const ActArgs& a, hipStream_t s);
int launch_act3(const ActArgs& a, hipStream_t s);
int launch_act4(const ActArgs& a, hipStream_t s);  // ppo_act_narrow.hip (H = 64 tanh agent)
int launch_fwdbwd(const UpdArgs& a, int nblocks, size_t lds_bytes, hipStream_t s);
int fwdbwd_set_lds(const PackedLayout& K, size_t lds_bytes);
// bx = 1: the split-bf16 form (k_upd<..., BX = 1>; LayerNorm-Beta agent, H = 256, one head tile)
int upd_supported(const PackedLayout& K, int nh_actor, int sg0_size, int sg1_size, UpdGeoOut* g, int bx = 0);
int launch_upd(const UpdArgs& a, int nh_actor, int nblocks, size_t lds_bytes, hipStream_t s);
// k_upd32 (create option upd_mfma=32 | mix): k_upd on 32x32x2 MFMAs, LayerNorm-Beta agent at
// H = 256; mix = 1: only the critic trunk on 32x32x2, the actor on k_upd's body
int upd32_supported(const PackedLayout& K, int nh_actor, int sg0_size, int sg1_size, UpdGeoOut* g, int mix);
int launch_upd32(const UpdArgs& a, int nh_actor, int nblocks, size_t lds_bytes, hipStream_t s, int mix);
// ppo_update_narrow.hip (H = 64 tanh agent); split form: k_l1g computes layer 1 (a.Z1), k_upd2 the rest
bool upd2_split_supported(const PackedLayout& K);
// split: 0 one kernel; 2 / 3 the split form at 2 / 3 workgroups per CU; bx: layer 1 as split-bf16
// piece products (cfg2's Humanoid shape)
int upd2_supported(const PackedLayout& K, UpdGeoOut* g, int split, int bx = 0);
int launch_upd2(const UpdArgs& a, int nblocks, size_t lds_bytes, hipStream_t s, int split);
int launch_l1g(const UpdArgs& a, hipStream_t s);
int launch_dw2(const DwArgs& a, int OP, int nchunks, hipStream_t s);  // both 64-wide trunks, rows gathered once
int launch_dw(const DwArgs& a, int H, int OP, int nchunks, hipStream_t s);
size_t dw_lds_bytes(int H, int OP);
void launch_colsum(const ColsumArgs& a, int nseg, long maxlen, hipStream_t s);
void launch_gradnorm(const NormArgs& a, hipStream_t s);
// k_gradnorm + k_adam in one cooperative launch (grid barrier on *bar; *count: its arrivals so far)
int launch_gradstep(const NormArgs& na, const AdamArgs& a, unsigned* bar, unsigned* count, hipStream_t s);

// Grid-wide barrier of a cooperative launch (every workgroup resident): all stores before it are
// visible to every workgroup after it. bar counts arrivals monotonically across launches; target =
// its value once every workgroup of this barrier has arrived.
// __syncthreads orders the workgroup's stores before thread 0's agent-scope release (which writes the
// XCD's L2 back for the other XCDs); thread 0's acquire invalidates the CU's caches for the loads
// every thread issues after the second __syncthreads. (A fence in every thread instead costs an L2
// write-back per wave.)
PPO_DEV void grid_barrier(unsigned* bar, unsigned target) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    while ((int)(__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) - target) < 0)
      __builtin_amdgcn_s_sleep(2);
  }
  __syncthreads();
}
void launch_adam(const AdamArgs& a, hipStream_t s);
void launch_transpose(const float* src, float* dst, int H, hipStream_t s);
void launch_swizzle(const float* w1, const float* w2, float* dst, int H, int OP, int bx, hipStream_t s);
// scan: k_gae_scan (segmented scan over T, create option gae=scan) instead of the serial k_gae
void launch_gae(const GaeArgs& a, hipStream_t s, bool scan = false);
void launch_perm(int32_t* out, uint32_t B, const PermKey& pk, hipStream_t s);
void launch_adv_sum(const AdvArgs& a, hipStream_t s);
void launch_adv_sq(const AdvArgs& a, int with_std, hipStream_t s);
void launch_adv_finalize(const AdvArgs& a, hipStream_t s);
void launch_synth_reset(const SynthArgs& a, int seed, float* obs, float* done, hipStream_t s);
void launch_synth_step(const SynthArgs& a, int e0, int e1, const float* act, float lo, float hi, float* obs,
                       float* reward, float* done, hipStream_t s);
void launch_wrap_step(const WrapArgs& w, int O, int e0, int e1, float* obs, float* reward, const float* term,
                      const float* is_reset, hipStream_t s);
