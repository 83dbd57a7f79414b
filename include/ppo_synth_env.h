/*
 * ppo_synth_env.h — device-resident synthetic HalfCheetah-shaped vector env (bench / test env).
 *
 * NOT part of the hot path: it stands in for the MuJoCo envs behind the gymcpp boundary
 * (libs/gymcpp/mujoco/half_cheetah_v5.h is unbuildable here — no libmujoco) so the GPU path can be
 * measured with inputs resident in HBM. Semantics follow SeqVectorEnv (libs/gymcpp/gym.h:131-163:
 * clip_actions, next-step autoreset with reward 0 / done 0 on the reset step, reset(seed + i))
 * wrapped in RecordEpisodeStatistics (libs/gymcpp/wrappers/common.h:48-65). Dynamics (identical,
 * bit for bit, to the host SyntheticCheetah in ppo.cpp_amd/gymcpp/synthetic/ and oracle/):
 *   q'_i = fma(0.9, q_i, fma(0.1, a_{i mod A}, 0.05 * q_{(i+1) mod O}))
 *   r    = (q'_0 - q_0) / 0.05 - sum_k (0.1 a_k) a_k ;  truncation after 1000 steps, never terminates
 */
#ifndef PPO_SYNTH_ENV_H
#define PPO_SYNTH_ENV_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct psyn_env psyn_t;

int psyn_create(int num_envs, int obs_dim, int act_dim, psyn_t** out);
int psyn_destroy(psyn_t* env);
/* reset(seed + i) for every env; writes obs [E,O] and done [E] (= 0) */
int psyn_reset(psyn_t* env, int seed, float* obs_dev, float* done_dev, void* stream);
/* The env's action space (default [-1, 1]); ppo_rollout_synth clips actions to it (clip_actions,
 * gym.h:141-144), e.g. Humanoid-v4's [-0.4, 0.4] (libs/gymcpp/mujoco/humanoid_v4.h:29-30). */
int psyn_set_action_space(psyn_t* env, float lo, float hi);
int psyn_action_space(const psyn_t* env, float* lo, float* hi);
/* one SeqVectorEnv step on envs [env_begin, env_end); actions are clipped to [lo, hi] */
int psyn_step(psyn_t* env, int env_begin, int env_end, const float* action_dev, float lo, float hi,
              float* obs_dev, float* reward_dev, float* done_dev, void* stream);
/* sums of finished-episode returns / lengths / counts since the last call (host floats) */
int psyn_episode_stats(psyn_t* env, float* sum_return, float* sum_length, float* count);
/* the same without a device-wide sync: _begin enqueues the read-out (and the reset of the sums)
 * on `stream`; _end waits for that read-out only and returns the sums (same values as above) */
int psyn_episode_stats_begin(psyn_t* env, void* stream);
int psyn_episode_stats_end(psyn_t* env, float* sum_return, float* sum_length, float* count);

/* Device-resident rollout driver: num_steps x {ppo_rollout_act, psyn_step, ppo_rollout_reward} on
 * the context stream (ppo_continuous_action.cpp:387-434 with this env behind the boundary).
 * act_scratch [E*A] and rew_scratch [E] are caller-provided device buffers. */
struct ppo_ctx;
int ppo_rollout_synth(struct ppo_ctx* ctx, psyn_t* env, float* next_obs_dev, float* next_done_dev,
                      float* act_scratch_dev, float* rew_scratch_dev);
/* How ppo_rollout_synth runs the T steps: PPO_ROLLOUT_AUTO (default) uses one persistent launch
 * (actor weights resident in registers, the env step and the PPO wrapper chain fused in; then the
 * critic over all stored observations) for the agent shapes the trainers build (AC agent H = 256
 * without wrappers, PPO agent H = 64), and per-step launches otherwise; PPO_ROLLOUT_PER_STEP always
 * launches per step. The persistent kernels run the arithmetic of the per-step act kernels k_act3
 * (AC) and k_act4 (PPO; the per-step default at O >= 112, option act_kernel=4 otherwise): storage,
 * env state and episode statistics are then bitwise identical. */
enum { PPO_ROLLOUT_AUTO = 0, PPO_ROLLOUT_PER_STEP = 1 };
int ppo_set_rollout_mode(struct ppo_ctx* ctx, int mode);

#ifdef __cplusplus
}
#endif
#endif
