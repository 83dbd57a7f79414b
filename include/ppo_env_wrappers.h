/*
 * ppo_env_wrappers.h — the PPO trainer's env wrapper chain on the device.
 *
 * The reference wraps every env of ppo_continuous_action in (src/ppo_continuous_action.cpp:41-49)
 *   RecordEpisodeStatistics -> NormalizeObservation(kFloat32) -> TransformObservation(clamp +-10)
 *   -> NormalizeReward(gamma) -> TransformReward(clamp +-10)
 * (libs/gymcpp/wrappers/stateful_observation.h:56-84, stateful_reward.h:55-91). Host envs keep
 * that chain on the CPU (ppo.cpp_amd/gymcpp/wrappers.h); a device-resident vector env runs it here,
 * with one state per env in HBM (running obs mean / var / count, discounted-return accumulator and
 * its running mean / var / count), in fp32 with the same operations in the same order, so results
 * are bit-exact against gymcpp/wrappers.h and the oracle (normalised observations within 1 ulp of
 * the LibTorch replay, whose CPU torch::sqrt is not correctly rounded).
 *
 * Semantics per vector-env step (gym.h:131-163 next-step autoreset): every observation passes the
 * observation half (statistics updated BEFORE normalising, on reset observations too); the reward
 * passes NormalizeReward unless the step was the env's autoreset (reward 0, accumulator unchanged).
 * RecordEpisodeStatistics sits inside: episode returns stay raw.
 */
#ifndef PPO_ENV_WRAPPERS_H
#define PPO_ENV_WRAPPERS_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pwrap pwrap_t;
struct psyn_env;

/* NormalizeObservation epsilon 1e-4, NormalizeReward epsilon 1e-8 (the reference defaults) */
int pwrap_create(int num_envs, int obs_dim, float gamma, pwrap_t** out);
int pwrap_destroy(pwrap_t* w);
/* obs [E,O] of a reset of envs [env_begin, env_end), normalised in place (reset_all, ppo:373) */
int pwrap_reset(pwrap_t* w, int env_begin, int env_end, float* obs_dev, void* stream);
/* one vector-env step of envs [env_begin, env_end), in place: obs [E,O] (rows by absolute env
 * index), reward [E]; term_dev [E] termination flags (NULL: none); is_reset_dev [E] != 0 where the
 * step was the env's next-step autoreset (NULL: none). */
int pwrap_step(pwrap_t* w, int env_begin, int env_end, float* obs_dev, float* reward_dev, const float* term_dev,
               const float* is_reset_dev, void* stream);
/* host copy of the state: n = 2*E*O + 5*E floats — obs mean [E,O], obs var [E,O], obs count [E],
 * reward mean [E], reward var [E], return accumulator [E], reward count [E] */
int pwrap_read_state(pwrap_t* w, float* host, long n);
/* Attach the chain to the synthetic device env (include/ppo_synth_env.h): psyn_reset / psyn_step /
 * ppo_rollout_synth then apply it inside the env's own kernels (no extra launch), with the same
 * arithmetic as pwrap_step. NULL detaches. The shapes must match. */
int psyn_attach_wrappers(struct psyn_env* env, pwrap_t* w);

#ifdef __cplusplus
}
#endif
#endif /* PPO_ENV_WRAPPERS_H */
