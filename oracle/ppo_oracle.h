/*
 * ppo_oracle.h — CPU restatement of the reference's rollout -> GAE -> PPO-update hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing in the product (ppo.cpp_amd/, include/ppo_hip.h) links,
 * loads or calls this code. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may use it, and only as the checker / the timed CPU baseline.
 *
 * Every function cites the reference file:line it restates (paths relative to the reference
 * root autonomousvision/ppo.cpp). Parity of this restatement is pinned by tests/golden/,
 * fixtures produced by oracle/ref_harness.cpp, which compiles the reference's own
 * include/rl_utils.h against LibTorch and replays the reference's inline main() arithmetic.
 */
#ifndef PPO_ORACLE_H
#define PPO_ORACLE_H

#include <stdint.h>
#include "../include/ppo_layout.h"
#include "../include/ppo_carla.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- RNG contract shared with the HIP path (restated independently there) ---- */
void orc_philox4x32(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
uint32_t orc_mix32(uint32_t h);
float orc_u01(uint32_t x);
/* index of minibatch slot `i` in the epoch permutation of [0,B) */
long orc_perm_index(long i, long B, uint64_t seed, int rank, long epoch_counter);
void orc_perm(long B, uint64_t seed, int rank, long epoch_counter, int64_t* out);

/* ---- special functions (ATen calc_digamma / calc_trigamma restated) ---- */
double orc_digamma(double x);
double orc_trigamma(double x);

/* ---- agent (a1-a4, a13-a15) ---- */
/* Agent::get_action_and_value over n rows.
 *   mode 0: sample with the Philox contract (ctr env index = env_base + row, step = step_id)
 *   mode 1: given `action_in` (update path; AC rescales + clamps, ac_ppo_continuous_action.cpp:194-203)
 *   mode 2: deterministic mean action (AC "mean", ac:229-231; PPO: mean of the Normal)
 * Outputs may be NULL. value has n entries. */
void orc_get_action_and_value(const ppo_layout* L, const float* params, int n, const float* x,
                              int mode, const float* action_in, uint64_t seed, int rank,
                              long env_base, long step_id,
                              float* action_out, float* logprob, float* entropy, float* value);

typedef struct orc_loss_cfg {
  float clip_coef, ent_coef, vf_coef;
  int clip_vloss, norm_adv;
} orc_loss_cfg;

/* One minibatch: loss + raw gradient (a8-a9). Rows are already gathered (minibatch order).
 * grad has L->P entries (non-grad params get 0). stats: [pg, v, ent, old_kl, kl, clipfrac, loss].
 * adv_mean / adv_std are the (possibly distributed) minibatch statistics; scale = 1/M_total
 * is folded per rank as 1/M_local (gradients are then averaged over ranks, ac:877-885). */
void orc_minibatch_grad(const ppo_layout* L, const float* params, int M, const float* x,
                        const float* actions, const float* old_logp, const float* adv,
                        const float* ret, const float* old_v, float adv_mean, float adv_std,
                        const orc_loss_cfg* cfg, float* grad, float* stats);
/* The same over rows [r0, r1) of the M-row minibatch: adds into double G[L->P] and sums[6]
 * (pg, v, ent, old_kl, kl, clipfrac row sums); orc_minibatch_finish turns the accumulated partials
 * into grad / stats. Disjoint ranges may run on different threads. */
void orc_minibatch_grad_part(const ppo_layout* L, const float* params, int M, int r0, int r1, const float* x,
                             const float* actions, const float* old_logp, const float* adv, const float* ret,
                             const float* old_v, float adv_mean, float adv_std, const orc_loss_cfg* cfg,
                             double* G, double* sums);
void orc_minibatch_finish(const ppo_layout* L, int M, const double* G, const double* sums,
                          const orc_loss_cfg* cfg, float* grad, float* stats);

/* per-minibatch advantage statistics: mean, unbiased std (ppo:511; distributed form ac:833-846) */
void orc_adv_stats(int M, const float* adv, float* mean, float* stdv);

/* clip_grad_norm_ (norm of per-tensor norms) + optim::Adam step over the flat vector (a10-a11).
 * m, v: Adam state (P floats). step: 1-based step count. Returns the total norm. */
double orc_clip_grad_norm(const ppo_layout* L, float* grad, float max_norm);
void orc_adam_step(const ppo_layout* L, float* params, const float* grad, float* m, float* v,
                   long step, float lr, float eps);

/* GAE(lambda) (a6): ppo_continuous_action.cpp:447-467 / ac_ppo_continuous_action.cpp:759-779 */
void orc_gae(int T, int E, const float* rewards, const float* values, const float* dones,
             const float* next_value, const float* next_done, float gamma, float lam,
             float* adv, float* ret);

/* Full update (a7-a12): EP epochs x MB minibatches over a flattened [B] batch, permutation from
 * orc_perm (or `perms` [EP][B] when non-NULL). Updates params, m, v in place, step_io counts
 * Adam steps. stats_out: last minibatch stats + mean clipfrac (7 floats). */
void orc_update(const ppo_layout* L, float* params, float* m, float* v, long* step_io,
                long B, int O, int A, const float* b_obs, const float* b_actions,
                const float* b_logp, const float* b_adv, const float* b_ret, const float* b_val,
                int epochs, int minibatches, float lr, float max_grad_norm, float adam_eps,
                const orc_loss_cfg* cfg, uint64_t seed, int rank, long epoch_counter0,
                const int64_t* perms, float* stats_out);

/* ---- synthetic HalfCheetah-shaped env + next-step-autoreset vector env (bench/test env) ---- */
typedef struct orc_env_state {
  int E, O, A;
  float* q;          /* [E,O] */
  int* t;            /* [E] elapsed steps */
  int* autoreset;    /* [E] */
  uint32_t* rseed;   /* [E] */
  uint32_t* rcount;  /* [E] */
  float* ep_ret;     /* [E] RecordEpisodeStatistics */
  int* ep_len;       /* [E] */
} orc_env_state;

void orc_env_reset(orc_env_state* s, int seed, float* obs_out);
/* The sampling draws of the Philox contract, for replays that compute the distribution elsewhere
 * (oracle/ref_harness.cpp end-to-end case): the A standard-normal draws of Normal.sample for
 * (env, step), and the Beta(alpha, beta) sample in [0, 1] of action index a (Marsaglia-Tsang
 * gammas), exactly as orc_get_action_and_value draws them. */
void orc_normal_noise(uint64_t seed, int rank, long env, long step, int A, float* z);
float orc_beta_sample01(float alpha, float beta, uint64_t seed, int rank, long env, long step, int a);
/* SeqVectorEnv::step semantics (gym.h:131-163) with clip_actions and RecordEpisodeStatistics.
 * info_ret/info_len get the finished episode stats (info_len = 0 if none). */
void orc_env_step(orc_env_state* s, const float* actions, float act_lo, float act_hi,
                  float* obs_out, float* reward, float* term, float* trunc,
                  float* info_ret, int* info_len);

/* ---- PPO env wrapper chain (a20): ppo:41-49 make_env over a scripted single env ----
 * RecordEpisodeStatistics (common.h:11-66) -> NormalizeObservation kFloat32 (stateful_observation.h:
 * 56-84: Welford with batch_count 1, update BEFORE normalising, also on reset) -> clamp +-10 ->
 * NormalizeReward (stateful_reward.h:55-91: discounted-return variance) -> clamp +-10, driven with
 * SeqVectorEnv's next-step autoreset (gym.h:141-159) and a plain reset(3) at step reset_at.
 * Scripted env, call c (reset or step): obs[i] = (i - 2) + 5 u(30, c*O + i); step reward
 * -1 + 5 u(31, c); termination c % 29 == 28; truncation c % 61 == 60 (u = orc_u01 of the
 * murmur3 hash stream of tests/carla_inputs.py). Writes obs [T+1][O] (row 0 = the first reset)
 * and reward / term / trunc / info_ret / info_len [T]; mean/var of the final obs statistics. */
/* The PPO wrapper chain behind a vector env, one state per env (layout in ppo_oracle.c):
 * st has 2*E*O + 5*E floats. */
void orc_vwrap_init(float* st, int E, int O);
void orc_vwrap_reset(float* st, int E, int O, float* obs);
void orc_vwrap_step(float* st, int E, int O, float gamma, float* obs, float* reward, const float* te,
                    const float* is_reset);
void orc_wrappers_script(int O, int T, int reset_at, float* raw_obs, float* reward, float* term, float* trunc,
                         float* is_reset);
void orc_wrappers_run(int O, int T, int reset_at, float gamma, float* obs, float* reward, float* term, float* trunc,
                      float* info_ret, float* info_len, float* obs_mean, float* obs_var);

/* ---- CaRL CNN agent (a23): AgentImpl::forward, include/carla/carla_model.h:222-318 ----
 * bev uint8 [n, C, IH, IW]; meas [n, NM]; vmeas [n, NV]; mode = PPO_CARLA_* (ppo_carla.h).
 * Convolutions and Linear layers accumulate in double. Outputs may be NULL; features [n, 256]. */
int orc_carla_layout_init(ppo_carla_layout* L, int C, int IH, int IW, int NM, int NV, int A);
void orc_carla_forward(const ppo_carla_layout* L, const float* params, float beta_min, int n, const uint8_t* bev,
                       const float* meas, const float* vmeas, int mode, const float* action_in, uint64_t seed,
                       int rank, long env_base, long step_id, float* action, float* logprob, float* entropy,
                       float* value, float* alpha, float* beta, float* features);

#ifdef __cplusplus
}
#endif
#endif
