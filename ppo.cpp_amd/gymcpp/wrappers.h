// gymcpp/wrappers.h — the reference's env wrappers, LibTorch-free, same constants and order.
//   RecordEpisodeStatistics  libs/gymcpp/wrappers/common.h:11-66
//   NormalizeObservation     libs/gymcpp/wrappers/stateful_observation.h:56-84  (float32 state,
//                            batch_count = 1, update BEFORE normalising, also on reset)
//   TransformObservation     libs/gymcpp/wrappers/transform_observation.h
//   NormalizeReward          libs/gymcpp/wrappers/stateful_reward.h:55-91
//   TransformReward          libs/gymcpp/wrappers/vectorize_reward.h
#pragma once

#include <algorithm>
#include <chrono>
#include <cmath>
#include <functional>
#include <memory>
#include <vector>

#include "gym.h"

namespace gymcpp {

class RecordEpisodeStatistics final : public EnvironmentWrapper {
  std::shared_ptr<Environment> env_;
  std::chrono::steady_clock::time_point start_;
  float episode_return_ = 0.0f;
  int episode_length_ = 0;

 public:
  explicit RecordEpisodeStatistics(std::shared_ptr<Environment> env) : env_(std::move(env)) {
    start_ = std::chrono::steady_clock::now();
  }
  ObsView reset(int seed) override {
    ObsView o = env_->reset(seed);
    episode_return_ = 0.0f;
    episode_length_ = 0;
    start_ = std::chrono::steady_clock::now();
    return o;
  }
  std::tuple<ObsView, float, bool, bool, std::optional<env_info>> step(const float* action) override {
    auto [o, r, te, tr] = env_->step(action);
    std::optional<env_info> info = std::nullopt;
    episode_return_ += r;
    episode_length_ += 1;
    if (te || tr) {
      const std::chrono::duration<float> dt = std::chrono::steady_clock::now() - start_;
      info = env_info{episode_return_, episode_length_, dt.count()};
    }
    return {o, r, te, tr, info};
  }
  int get_observation_space() const override { return env_->get_observation_space(); }
  int get_action_space() const override { return env_->get_action_space(); }
  float get_action_space_min() const override { return env_->get_action_space_min(); }
  float get_action_space_max() const override { return env_->get_action_space_max(); }
};

// Running mean/var of observations, batch of 1 (stateful_observation.h:64-84).
class NormalizeObservation final : public EnvironmentWrapper {
  std::shared_ptr<EnvironmentWrapper> env_;
  std::vector<float> mean_, var_, out_;
  float count_, epsilon_;

 public:
  bool update_running_mean_ = true;
  NormalizeObservation(std::shared_ptr<EnvironmentWrapper> env, int observation_space, float epsilon = 1e-4f)
      : env_(std::move(env)), mean_(observation_space, 0.0f), var_(observation_space, 1.0f),
        out_(observation_space, 0.0f), count_(epsilon), epsilon_(epsilon) {}
  ObsView reset(int seed) override { return observation(env_->reset(seed)); }
  std::tuple<ObsView, float, bool, bool, std::optional<env_info>> step(const float* action) override {
    auto [o, r, te, tr, info] = env_->step(action);
    return {observation(o), r, te, tr, info};
  }
  ObsView observation(const ObsView& x) {
    if (update_running_mean_) update(x);
    for (int i = 0; i < x.size; ++i) out_[i] = (x.data[i] - mean_[i]) / std::sqrt(var_[i] + epsilon_);
    return ObsView{out_.data(), x.size};
  }
  void update(const ObsView& x) {
    const float batch_count = 1.0f;
    const float tot_count = count_ + batch_count;
    for (int i = 0; i < x.size; ++i) {
      const float delta = x.data[i] - mean_[i];
      const float new_mean = mean_[i] + delta * batch_count / tot_count;
      const float m_a = var_[i] * count_;
      const float m_b = 0.0f * batch_count;
      const float M2 = m_a + m_b + (delta * delta) * count_ * batch_count / tot_count;
      mean_[i] = new_mean;
      var_[i] = M2 / tot_count;
    }
    count_ = tot_count;
  }
  const std::vector<float>& mean() const { return mean_; }
  const std::vector<float>& var() const { return var_; }
  int get_observation_space() const override { return env_->get_observation_space(); }
  int get_action_space() const override { return env_->get_action_space(); }
  float get_action_space_min() const override { return env_->get_action_space_min(); }
  float get_action_space_max() const override { return env_->get_action_space_max(); }
};

class TransformObservation final : public EnvironmentWrapper {
  std::shared_ptr<EnvironmentWrapper> env_;
  std::function<void(float*, int)> func_;
  std::vector<float> out_;

 public:
  TransformObservation(std::shared_ptr<EnvironmentWrapper> env, std::function<void(float*, int)> func)
      : env_(std::move(env)), func_(std::move(func)), out_(env_->get_observation_space()) {}
  ObsView reset(int seed) override { return observation(env_->reset(seed)); }
  std::tuple<ObsView, float, bool, bool, std::optional<env_info>> step(const float* action) override {
    auto [o, r, te, tr, info] = env_->step(action);
    return {observation(o), r, te, tr, info};
  }
  ObsView observation(const ObsView& x) {
    std::copy(x.data, x.data + x.size, out_.begin());
    func_(out_.data(), x.size);
    return ObsView{out_.data(), x.size};
  }
  int get_observation_space() const override { return env_->get_observation_space(); }
  int get_action_space() const override { return env_->get_action_space(); }
  float get_action_space_min() const override { return env_->get_action_space_min(); }
  float get_action_space_max() const override { return env_->get_action_space_max(); }
};

// Discounted-return variance normaliser (stateful_reward.h:55-91).
class NormalizeReward final : public EnvironmentWrapper {
  std::shared_ptr<EnvironmentWrapper> env_;
  float mean_ = 0.0f, var_ = 1.0f, accumulated_reward_ = 0.0f, count_, gamma_, epsilon_;

 public:
  bool update_running_mean_ = true;
  explicit NormalizeReward(std::shared_ptr<EnvironmentWrapper> env, float gamma = 0.99f, float epsilon = 1e-8f)
      : env_(std::move(env)), count_(epsilon), gamma_(gamma), epsilon_(epsilon) {}
  ObsView reset(int seed) override { return env_->reset(seed); }
  std::tuple<ObsView, float, bool, bool, std::optional<env_info>> step(const float* action) override {
    auto [o, r, te, tr, info] = env_->step(action);
    accumulated_reward_ = accumulated_reward_ * gamma_ * (1.0f - static_cast<float>(te)) + r;
    return {o, normalize(r), te, tr, info};
  }
  float normalize(float reward) {
    if (update_running_mean_) update(accumulated_reward_);
    return reward / std::sqrt(var_ + epsilon_);
  }
  void update(float x) {
    const float batch_count = 1.0f;
    const float delta = x - mean_;
    const float tot_count = count_ + batch_count;
    const float new_mean = mean_ + delta * batch_count / tot_count;
    const float m_a = var_ * count_;
    const float m_b = 0.0f * batch_count;
    const float M2 = m_a + m_b + (delta * delta) * count_ * batch_count / tot_count;
    count_ = tot_count;
    mean_ = new_mean;
    var_ = M2 / tot_count;
  }
  int get_observation_space() const override { return env_->get_observation_space(); }
  int get_action_space() const override { return env_->get_action_space(); }
  float get_action_space_min() const override { return env_->get_action_space_min(); }
  float get_action_space_max() const override { return env_->get_action_space_max(); }
};

class TransformReward final : public EnvironmentWrapper {
  std::shared_ptr<EnvironmentWrapper> env_;
  std::function<float(float)> func_;

 public:
  TransformReward(std::shared_ptr<EnvironmentWrapper> env, std::function<float(float)> func)
      : env_(std::move(env)), func_(std::move(func)) {}
  ObsView reset(int seed) override { return env_->reset(seed); }
  std::tuple<ObsView, float, bool, bool, std::optional<env_info>> step(const float* action) override {
    auto [o, r, te, tr, info] = env_->step(action);
    return {o, func_(r), te, tr, info};
  }
  int get_observation_space() const override { return env_->get_observation_space(); }
  int get_action_space() const override { return env_->get_action_space(); }
  float get_action_space_min() const override { return env_->get_action_space_min(); }
  float get_action_space_max() const override { return env_->get_action_space_max(); }
};

// The PPO trainer's wrapper chain (ppo_continuous_action.cpp:41-49): episode statistics on the raw
// env, running observation normalisation clamped to +-10, discounted-return reward scaling clamped
// to +-10.
inline std::shared_ptr<EnvironmentWrapper> make_env(const std::shared_ptr<Environment>& env_0, float gamma) {
  auto env_1 = std::make_shared<RecordEpisodeStatistics>(env_0);
  auto env_2 = std::make_shared<NormalizeObservation>(env_1, env_1->get_observation_space());
  auto env_3 = std::make_shared<TransformObservation>(env_2, [](float* x, int n) {
    for (int i = 0; i < n; ++i) x[i] = std::clamp(x[i], -10.0f, 10.0f);
  });
  auto env_4 = std::make_shared<NormalizeReward>(env_3, gamma);
  return std::make_shared<TransformReward>(env_4, [](float x) { return std::clamp(x, -10.0f, 10.0f); });
}

}  // namespace gymcpp
