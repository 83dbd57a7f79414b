// ppo_wrap.hpp — the PPO env wrapper chain's per-element arithmetic on the device (ppo:41-49),
// shared by the device env kernels (ppo_kernels.hip) and the persistent rollout (ppo_rollout.hip).
// Same fp32 operations, in the same order, as gymcpp/wrappers.h and the oracle (orc_vwrap_*): no
// contraction, IEEE division and square root, so the chain is bit-exact against both.
#pragma once

#include "ppo_kernels.hpp"

// NormalizeObservation::observation of one element (stateful_observation.h:64-84: the Welford
// update with batch_count 1 BEFORE normalising) + TransformObservation clamp +-10 (ppo:44). om / ov
// point at the element's running mean / var (HBM or LDS); oc is the env's count_ as read before this
// step; the caller stores oc + 1 once per env.
PPO_DEV float wrap_obs_at(float* om, float* ov, float oc, float x) {
#pragma clang fp contract(off)
  const float batch_count = 1.0f;
  const float tot_count = oc + batch_count;
  const float delta = x - *om;
  const float new_mean = *om + delta * batch_count / tot_count;
  const float m_a = *ov * oc;
  const float m_b = 0.0f * batch_count;
  const float M2 = m_a + m_b + (delta * delta) * oc * batch_count / tot_count;
  const float new_var = M2 / tot_count;
  *om = new_mean;
  *ov = new_var;
  const float v = (x - new_mean) / sqrtf(new_var + 1e-4f);
  return v < -10.0f ? -10.0f : (v > 10.0f ? 10.0f : v);
}
// dimension i of env e of the state in HBM
PPO_DEV float wrap_obs_dim(const WrapArgs& w, long e, int O, int i, float oc, float x) {
  return wrap_obs_at(w.om + e * O + i, w.ov + e * O + i, oc, x);
}

// NormalizeReward::step (stateful_reward.h:55-91; te = termination) + TransformReward clamp +-10,
// on one env's accumulator / running mean / var / count (HBM or LDS)
PPO_DEV float wrap_reward_at(float* racc_p, float* rmean_p, float* rvar_p, float* rcount_p, float gamma, float r,
                             float te) {
#pragma clang fp contract(off)
  const float racc = *racc_p * gamma * (1.0f - te) + r;
  const float rmean = *rmean_p, rvar = *rvar_p, rcount = *rcount_p;
  const float batch_count = 1.0f;
  const float delta = racc - rmean;
  const float tot_count = rcount + batch_count;
  const float new_mean = rmean + delta * batch_count / tot_count;
  const float m_a = rvar * rcount;
  const float m_b = 0.0f * batch_count;
  const float M2 = m_a + m_b + (delta * delta) * rcount * batch_count / tot_count;
  const float new_var = M2 / tot_count;
  *racc_p = racc;
  *rcount_p = tot_count;
  *rmean_p = new_mean;
  *rvar_p = new_var;
  const float rn = r / sqrtf(new_var + 1e-8f);
  return rn < -10.0f ? -10.0f : (rn > 10.0f ? 10.0f : rn);
}
PPO_DEV float wrap_reward(const WrapArgs& w, long e, float r, float te) {
  return wrap_reward_at(w.racc + e, w.rmean + e, w.rvar + e, w.rcount + e, w.gamma, r, te);
}
