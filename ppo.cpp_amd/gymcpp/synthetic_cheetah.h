// gymcpp/synthetic_cheetah.h — deterministic HalfCheetah-shaped env (O=17, A=6, actions in [-1,1],
// 1000-step truncation, never terminates). Stands in for libs/gymcpp/mujoco/half_cheetah_v5.h
// where libmujoco is unavailable. Bit-identical to the device env (include/ppo_synth_env.h) and to
// the oracle (oracle/ppo_oracle.c): fp32, explicit fmaf, no contraction (compile with
// -ffp-contract=off), Philox4x32-10 reset noise keyed (seed, 0x5EED5EED), counter (resets, i).
#pragma once

#include <chrono>
#include <cmath>
#include <cstdint>
#include <vector>

#include "gym.h"

namespace gymcpp {

inline void philox4x32_host(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                            uint32_t out[4]) {
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0, hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

class SyntheticCheetah final : public Environment {
  static constexpr int kO = 17, kA = 6, kMaxSteps = 1000;
  std::vector<float> q_ = std::vector<float>(kO, 0.0f), nq_ = std::vector<float>(kO, 0.0f);
  uint32_t rseed_ = 1, rcount_ = 0;
  int elapsed_ = kMaxSteps + 1;
  int64_t step_cost_ns_ = 0;

 public:
  // Host CPU time each step() burns before it returns (a busy wait): stands in for the physics of the
  // MuJoCo env this replaces ("per-step host cost configurable"), so the async
  // collection's overlap of CPU stepping with GPU inference can be measured. 0: no cost.
  void set_step_cost_ns(int64_t ns) { step_cost_ns_ = ns; }
  int64_t step_cost_ns() const { return step_cost_ns_; }
  ObsView reset(int seed) override {
    if (seed > 0) { rseed_ = (uint32_t)seed; rcount_ = 0; }
    for (int i = 0; i < kO; ++i) {
      uint32_t r[4];
      philox4x32_host(rcount_, (uint32_t)i, 0u, 0u, rseed_, 0x5EED5EEDu, r);
      const float u = ((float)(r[0] >> 8) + 0.5f) * 5.9604644775390625e-8f;
      q_[i] = 0.1f * (2.0f * u - 1.0f);
    }
    rcount_ += 1;
    elapsed_ = 0;
    return ObsView{q_.data(), kO};
  }
  std::tuple<ObsView, float, bool, bool> step(const float* a) override {
    if (step_cost_ns_ > 0) {
      const auto until = std::chrono::steady_clock::now() + std::chrono::nanoseconds(step_cost_ns_);
      while (std::chrono::steady_clock::now() < until) {
      }
    }
    const float xb = q_[0];
    for (int i = 0; i < kO; ++i) nq_[i] = std::fma(0.9f, q_[i], std::fma(0.1f, a[i % kA], 0.05f * q_[(i + 1) % kO]));
    q_.swap(nq_);
    const float vel = (q_[0] - xb) / 0.05f;
    float ctrl = 0.0f;
    for (int k = 0; k < kA; ++k) ctrl = ctrl + 0.1f * a[k] * a[k];
    const float reward = vel - ctrl;
    ++elapsed_;
    return {ObsView{q_.data(), kO}, reward, false, elapsed_ >= kMaxSteps};
  }
  int get_observation_space() const override { return kO; }
  int get_action_space() const override { return kA; }
  float get_action_space_min() const override { return -1.0f; }
  float get_action_space_max() const override { return 1.0f; }
};

}  // namespace gymcpp
