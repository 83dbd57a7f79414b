// ppo_wrap.hpp — the PPO env wrapper chain's per-element arithmetic on the device (ppo:41-49),
// shared by the device env kernels (ppo_kernels.hip) and the persistent rollout (ppo_rollout.hip).
// Same fp32 operations, in the same order, as gymcpp/wrappers.h and the oracle (orc_vwrap_*): no
// contraction, IEEE division and square root, so the chain is bit-exact against both.
#pragma once

#include "ppo_kernels.hpp"

// Correctly rounded fp32 division without the compiler's scaled sequence. IEEE `n / d` lowers to
// v_div_scale (x2, one writing VCC) -> v_rcp -> an fma refinement -> v_div_fmas (reads VCC) ->
// v_div_fixup; the single VCC makes every division in a wave wait for the previous one, which
// serialised the wrapper chain's 4 divisions per element. The refinement below is that sequence's
// own arithmetic, step for step; v_div_scale / v_div_fmas only rescale when an operand is near the
// ends of the exponent range (|n| < 2^-103, |d| or n / d near denormal or overflow), which the
// wrapper chain's operands (counts, variances >= 0 shifted by 1e-8 / 1e-4, observations and their
// differences) never are, and v_div_fixup still handles zeros, infinities and NaN. Results are
// bitwise those of `n / d` (the oracle's IEEE division; tests/test_gpu_wrappers.py, test_gpu_rollout).
struct Recip {
  float d, r;
};
PPO_DEV Recip recip_of(float d) {
  const float r0 = __builtin_amdgcn_rcpf(d);
  const float e = __builtin_fmaf(-d, r0, 1.0f);
  return Recip{d, __builtin_fmaf(e, r0, r0)};
}
PPO_DEV float div_by(float n, Recip q) {
  const float q0 = n * q.r;
  const float rem0 = __builtin_fmaf(-q.d, q0, n);
  const float q1 = __builtin_fmaf(rem0, q.r, q0);
  const float rem1 = __builtin_fmaf(-q.d, q1, n);
  const float q2 = __builtin_fmaf(rem1, q.r, q1);
  return __builtin_amdgcn_div_fixupf(q2, q.d, n);
}

// NormalizeObservation::observation of one element (stateful_observation.h:64-84: the Welford
// update with batch_count 1 BEFORE normalising) + TransformObservation clamp +-10 (ppo:44). om / ov
// point at the element's running mean / var (HBM or LDS); oc is the env's count_ as read before this
// step; the caller stores oc + 1 once per env.
// rtot = recip_of(oc + 1): one per env and step, shared by the env's elements
PPO_DEV float wrap_obs_at_r(float* om, float* ov, float oc, Recip rtot, float x) {
#pragma clang fp contract(off)
  const float batch_count = 1.0f;
  const float delta = x - *om;
  const float new_mean = *om + div_by(delta * batch_count, rtot);
  const float m_a = *ov * oc;
  const float m_b = 0.0f * batch_count;
  const float M2 = m_a + m_b + div_by((delta * delta) * oc * batch_count, rtot);
  const float new_var = div_by(M2, rtot);
  *om = new_mean;
  *ov = new_var;
  const float v = div_by(x - new_mean, recip_of(sqrtf(new_var + 1e-4f)));
  return v < -10.0f ? -10.0f : (v > 10.0f ? 10.0f : v);
}
PPO_DEV float wrap_obs_at(float* om, float* ov, float oc, float x) {
  return wrap_obs_at_r(om, ov, oc, recip_of(oc + 1.0f), x);
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
  const Recip rtot = recip_of(tot_count);
  const float new_mean = rmean + div_by(delta * batch_count, rtot);
  const float m_a = rvar * rcount;
  const float m_b = 0.0f * batch_count;
  const float M2 = m_a + m_b + div_by((delta * delta) * rcount * batch_count, rtot);
  const float new_var = div_by(M2, rtot);
  *racc_p = racc;
  *rcount_p = tot_count;
  *rmean_p = new_mean;
  *rvar_p = new_var;
  const float rn = div_by(r, recip_of(sqrtf(new_var + 1e-8f)));
  return rn < -10.0f ? -10.0f : (rn > 10.0f ? 10.0f : rn);
}
PPO_DEV float wrap_reward(const WrapArgs& w, long e, float r, float te) {
  return wrap_reward_at(w.racc + e, w.rmean + e, w.rvar + e, w.rcount + e, w.gamma, r, te);
}
