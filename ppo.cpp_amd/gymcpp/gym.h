// gymcpp/gym.h — LibTorch-free drop-in of the reference's env interface (libs/gymcpp/gym.h).
//
// Same names and semantics as the reference:
//   env_info                         gym.h:19-24
//   Environment / EnvironmentWrapper gym.h:26-47  (step / reset / spaces)
//   SeqVectorEnv                     gym.h:75-164 (clip_actions, next-step autoreset, reset(seed + i))
//   ParVectorEnv                     gym.h:276-366 (same, env steps on a thread pool)
// Differences by design: observations are borrowed float views (ObsView: pointer + size, valid
// until the next call on that env — the reference returns its internal obs_ tensor the same way,
// half_cheetah_v5.h:86,115) instead of torch::Tensor; actions are plain float pointers; the vector
// env returns views of its own [E, O] / [E] buffers. No LibTorch, no boost.
#pragma once

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <optional>
#include <stdexcept>
#include <thread>
#include <tuple>
#include <vector>

namespace gymcpp {

struct env_info {
  float r;  // episode return
  int l;    // episode length
  float t;  // episode wall time in seconds
};

struct ObsView {
  const float* data = nullptr;
  int size = 0;
};

class Environment {
 public:
  virtual std::tuple<ObsView, float, bool, bool> step(const float* action) = 0;
  virtual ObsView reset(int seed) = 0;
  [[nodiscard]] virtual int get_observation_space() const = 0;
  [[nodiscard]] virtual int get_action_space() const = 0;
  [[nodiscard]] virtual float get_action_space_min() const = 0;
  [[nodiscard]] virtual float get_action_space_max() const = 0;
  virtual ~Environment() = default;
};

class EnvironmentWrapper {
 public:
  virtual std::tuple<ObsView, float, bool, bool, std::optional<env_info>> step(const float* action) = 0;
  virtual ObsView reset(int seed) = 0;
  [[nodiscard]] virtual int get_observation_space() const = 0;
  [[nodiscard]] virtual int get_action_space() const = 0;
  [[nodiscard]] virtual float get_action_space_min() const = 0;
  [[nodiscard]] virtual float get_action_space_max() const = 0;
  virtual ~EnvironmentWrapper() = default;
};

struct VecStep {
  const float* obs;           // [E, O]
  const float* rewards;       // [E]
  const float* terminations;  // [E] (0/1)
  const float* truncations;   // [E] (0/1)
  const std::vector<std::optional<env_info>>* infos;
};

namespace detail {
// shared per-env step body of SeqVectorEnv / ParVectorEnv (gym.h:140-160, :337-355)
struct VecState {
  std::vector<std::shared_ptr<EnvironmentWrapper>> envs;
  std::vector<float> obs, rewards, terms, truncs, clipped;
  std::vector<int> autoreset;  // int, not vector<bool>: written concurrently (gym.h:283-284)
  std::vector<std::optional<env_info>> infos;
  bool clip_actions;
  int O = 0, A = 0;

  VecState(const std::vector<std::shared_ptr<EnvironmentWrapper>>& e, bool clip) : envs(e), clip_actions(clip) {
    if (envs.empty()) throw std::runtime_error("vector env needs at least one env");
    O = envs[0]->get_observation_space();
    A = envs[0]->get_action_space();
    const size_t E = envs.size();
    obs.assign(E * O, 0.f);
    rewards.assign(E, 0.f);
    terms.assign(E, 0.f);
    truncs.assign(E, 0.f);
    clipped.assign(E * A, 0.f);
    autoreset.assign(E, 0);
    infos.assign(E, std::nullopt);
  }
  void copy_obs(size_t i, const ObsView& v) { std::copy(v.data, v.data + O, obs.begin() + i * O); }
  void reset_all(int seed) {
    for (size_t i = 0; i < envs.size(); ++i) {
      copy_obs(i, envs[i]->reset(seed + (int)i));
      autoreset[i] = 0;
    }
  }
  void prepare(const float* actions) {
    const float lo = envs[0]->get_action_space_min(), hi = envs[0]->get_action_space_max();
    for (size_t k = 0; k < envs.size() * A; ++k)
      clipped[k] = clip_actions ? std::clamp(actions[k], lo, hi) : actions[k];
  }
  void step_one(size_t i) {
    if (autoreset[i]) {
      copy_obs(i, envs[i]->reset(-1));  // -1: do not reseed
      rewards[i] = 0.f;
      terms[i] = 0.f;
      truncs[i] = 0.f;
      infos[i] = std::nullopt;
      autoreset[i] = 0;
    } else {
      auto [o, r, te, tr, info] = envs[i]->step(clipped.data() + i * A);
      copy_obs(i, o);
      rewards[i] = r;
      terms[i] = te ? 1.f : 0.f;
      truncs[i] = tr ? 1.f : 0.f;
      infos[i] = info;
      autoreset[i] = (te || tr) ? 1 : 0;
    }
  }
  VecStep view() const { return VecStep{obs.data(), rewards.data(), terms.data(), truncs.data(), &infos}; }
};
}  // namespace detail

// Comparable to gymnasium's SyncVectorEnv (gym.h:75-164).
class SeqVectorEnv {
 public:
  SeqVectorEnv(const std::vector<std::shared_ptr<EnvironmentWrapper>>& env_array, bool clip_actions)
      : s_(env_array, clip_actions), num_envs_((unsigned)env_array.size()) {}
  const float* reset(int seed) {
    s_.reset_all(seed);
    return s_.obs.data();
  }
  VecStep step(const float* actions) {
    s_.prepare(actions);
    for (size_t i = 0; i < s_.envs.size(); ++i) s_.step_one(i);
    return s_.view();
  }
  [[nodiscard]] unsigned get_num_envs() const { return num_envs_; }
  [[nodiscard]] int get_observation_space() const { return s_.O; }
  [[nodiscard]] int get_action_space() const { return s_.A; }
  [[nodiscard]] float get_action_space_min() const { return s_.envs[0]->get_action_space_min(); }
  [[nodiscard]] float get_action_space_max() const { return s_.envs[0]->get_action_space_max(); }

 private:
  detail::VecState s_;
  unsigned num_envs_;
};

// Comparable to gymnasium's AsyncVectorEnv, threads instead of processes (gym.h:276-366). The
// reference posts one task per env to a pool of num_envs threads; here a fixed pool of
// min(num_envs, hardware threads) workers takes contiguous env slices (same results: env i is
// always stepped by exactly one worker, with the same clipped action).
class ParVectorEnv {
 public:
  ParVectorEnv(const std::vector<std::shared_ptr<EnvironmentWrapper>>& env_array, bool clip_actions,
               int num_threads = 0)
      : s_(env_array, clip_actions), num_envs_((unsigned)env_array.size()) {
    int nt = num_threads > 0 ? num_threads : (int)std::max(1u, std::thread::hardware_concurrency());
    nt = std::min<int>(nt, (int)num_envs_);
    for (int w = 0; w < nt; ++w) workers_.emplace_back([this, w, nt] { worker(w, nt); });
  }
  ~ParVectorEnv() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  const float* reset(int seed) {
    s_.reset_all(seed);
    return s_.obs.data();
  }
  VecStep step(const float* actions) {
    s_.prepare(actions);
    {
      std::lock_guard<std::mutex> lk(mu_);
      pending_ = (int)workers_.size();
      ++gen_;
    }
    cv_.notify_all();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return pending_ == 0; });
    return s_.view();
  }
  [[nodiscard]] unsigned get_num_envs() const { return num_envs_; }
  [[nodiscard]] int get_observation_space() const { return s_.O; }
  [[nodiscard]] int get_action_space() const { return s_.A; }
  [[nodiscard]] float get_action_space_min() const { return s_.envs[0]->get_action_space_min(); }
  [[nodiscard]] float get_action_space_max() const { return s_.envs[0]->get_action_space_max(); }

 private:
  void worker(int w, int nt) {
    long seen = 0;
    const size_t E = s_.envs.size();
    const size_t b = E * w / nt, e = E * (w + 1) / nt;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
      }
      for (size_t i = b; i < e; ++i) s_.step_one(i);
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (--pending_ == 0) done_cv_.notify_one();
      }
    }
  }
  detail::VecState s_;
  unsigned num_envs_;
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  long gen_ = 0;
  int pending_ = 0;
  bool stop_ = false;
};

}  // namespace gymcpp
