// gymcpp/carla_gym.h — LibTorch-free drop-in of the reference's CaRL env layer:
//   EnvironmentCarla / EnvironmentWrapperCarla   libs/gymcpp/gym.h:50-69
//   RecordEpisodeStatisticsCarla                 libs/gymcpp/wrappers/common.h:69-126
//   SeqVectorEnvCarla                            libs/gymcpp/gym.h:167-270 (clip_actions, next-step autoreset)
//   CarlaEnv                                     libs/gymcpp/carla/carla_gym.h:23-148
// CarlaEnv speaks the reference's protocol with the CARLA leaderboard gym over a PAIR socket bound
// at ipc://<comm_root>/comm_files/<port>.lock (net/zmtp.h, ZMTP 3.0 — the Python side uses pyzmq):
//   first reset: receive one hello message; every reset / step: receive the 8-part multipart state
//   [bev uint8 C x H x W | measurements f32[NM] | value_measurements f32[NV] | reward f32 |
//    termination bool | truncation bool | n_steps i32 | suggest i32]; step first sends the action
//   (A float32, one frame). Observations are views of the env's own buffers (valid until the next
//   call), like the reference's obs_ tensors.
#pragma once

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <filesystem>
#include <iostream>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "../net/zmtp.h"
#include "gym.h"

namespace gymcpp {

// the GlobalConfig fields the env reads (carla_config.h:57, 84, 97-98, bev_semantics_width)
struct CarlaObsConfig {
  int obs_num_channels = 15;
  int bev_semantics_height = 192;
  int bev_semantics_width = 192;
  int obs_num_measurements = 8;
  int num_value_measurements = 3;
};

struct CarlaObsView {
  const uint8_t* bev_semantics = nullptr;   // [C, H, W]
  const float* measurements = nullptr;      // [NM]
  const float* value_measurements = nullptr;  // [NV]
};

class EnvironmentCarla {
 public:
  virtual std::tuple<CarlaObsView, float, bool, bool> step(const float* action) = 0;
  virtual CarlaObsView reset(int seed) = 0;
  [[nodiscard]] virtual std::vector<int> get_observation_space() const = 0;  // C, H, W, NM, NV
  [[nodiscard]] virtual int get_action_space() const = 0;
  [[nodiscard]] virtual float get_action_space_min() const = 0;
  [[nodiscard]] virtual float get_action_space_max() const = 0;
  virtual ~EnvironmentCarla() = default;
};

class EnvironmentWrapperCarla {
 public:
  virtual std::tuple<CarlaObsView, float, bool, bool, std::optional<env_info>> step(const float* action) = 0;
  virtual CarlaObsView reset(int seed) = 0;
  [[nodiscard]] virtual std::vector<int> get_observation_space() const = 0;
  [[nodiscard]] virtual int get_action_space() const = 0;
  [[nodiscard]] virtual float get_action_space_min() const = 0;
  [[nodiscard]] virtual float get_action_space_max() const = 0;
  virtual ~EnvironmentWrapperCarla() = default;
};

class CarlaEnv final : public EnvironmentCarla {
  zmtp::Socket socket_{zmtp::Type::PAIR};
  bool initialized_ = false;
  const int port_;
  bool termination_ = false, truncation_ = false;
  std::string comm_root_;
  std::vector<int> observation_space_;
  std::vector<uint8_t> bev_;
  std::vector<float> meas_, vmeas_;
  int32_t n_steps_ = 0, suggest_ = 0;  // Roach-only fields, received and kept (unused, as in the reference)

  float receive_state() {
    zmtp::Message m;
    socket_.recv(m);
    if (m.size() != 8) throw std::runtime_error("CarlaEnv: expected an 8-part state message, got " + std::to_string(m.size()));
    const size_t nb = (size_t)observation_space_[0] * observation_space_[1] * observation_space_[2];
    auto need = [&](int k, size_t bytes) {
      if (m[k].size() < bytes) throw std::runtime_error("CarlaEnv: state part " + std::to_string(k) + " too short");
    };
    need(0, nb); need(1, 4 * meas_.size()); need(2, 4 * vmeas_.size()); need(3, 4); need(4, 1); need(5, 1);
    need(6, 4); need(7, 4);
    std::memcpy(bev_.data(), m[0].data(), nb);
    std::memcpy(meas_.data(), m[1].data(), 4 * meas_.size());
    std::memcpy(vmeas_.data(), m[2].data(), 4 * vmeas_.size());
    float reward;
    std::memcpy(&reward, m[3].data(), 4);
    termination_ = m[4][0] != 0;
    truncation_ = m[5][0] != 0;
    std::memcpy(&n_steps_, m[6].data(), 4);
    std::memcpy(&suggest_, m[7].data(), 4);
    return reward;
  }
  CarlaObsView view() const { return CarlaObsView{bev_.data(), meas_.data(), vmeas_.data()}; }

 public:
  static constexpr int action_space_{2};
  static constexpr float action_space_min_{-1.0f};
  static constexpr float action_space_max_{1.0f};

  CarlaEnv(const CarlaObsConfig& config, const std::string& comm_root, const int port)
      : port_(port), comm_root_(comm_root),
        observation_space_{config.obs_num_channels, config.bev_semantics_height, config.bev_semantics_width,
                           config.obs_num_measurements, config.num_value_measurements} {
    bev_.assign((size_t)observation_space_[0] * observation_space_[1] * observation_space_[2], 0);
    meas_.assign(observation_space_[3], 0.f);
    vmeas_.assign(observation_space_[4], 0.f);
  }

  [[nodiscard]] std::vector<int> get_observation_space() const override { return observation_space_; }
  [[nodiscard]] int get_action_space() const override { return action_space_; }
  [[nodiscard]] float get_action_space_min() const override { return action_space_min_; }
  [[nodiscard]] float get_action_space_max() const override { return action_space_max_; }

  // the CARLA env is seeded on the Python side; seed is unused (carla_gym.h:69-70)
  CarlaObsView reset(const int seed) override {
    (void)seed;
    if (!initialized_) {
      const std::filesystem::path comm_folder = std::filesystem::path(comm_root_) / "comm_files";
      std::filesystem::create_directories(comm_folder);
      const std::filesystem::path file(std::to_string(port_) + ".lock");
      socket_.bind("ipc://" + (comm_folder / file).string());
      std::cout << "Connecting to leaderboard gym, port: " << file.string() << std::endl;
      zmtp::Message hello;
      if (!socket_.recv(hello)) throw std::runtime_error("Connection to CARLA leaderboard failed.");
      std::cout << (hello.empty() ? std::string() : hello[0]) << std::endl;
      initialized_ = true;
    }
    receive_state();
    return view();
  }

  std::tuple<CarlaObsView, float, bool, bool> step(const float* action) override {
    std::string a(sizeof(float) * action_space_, '\0');
    std::memcpy(&a[0], action, a.size());
    socket_.send(a);
    const float reward = receive_state();
    return {view(), reward, termination_, truncation_};
  }
};

class RecordEpisodeStatisticsCarla final : public EnvironmentWrapperCarla {
  std::chrono::steady_clock::time_point episode_start_time_;
  float episode_return_ = 0.0f;
  int episode_length_ = 0;
  std::shared_ptr<EnvironmentCarla> env_;

 public:
  explicit RecordEpisodeStatisticsCarla(const std::shared_ptr<EnvironmentCarla>& env)
      : episode_start_time_(std::chrono::steady_clock::now()), env_(env) {}

  CarlaObsView reset(const int seed) override {
    const CarlaObsView obs = env_->reset(seed);
    episode_return_ = 0.0f;
    episode_length_ = 0;
    episode_start_time_ = std::chrono::steady_clock::now();
    return obs;
  }
  [[nodiscard]] std::vector<int> get_observation_space() const override { return env_->get_observation_space(); }
  [[nodiscard]] int get_action_space() const override { return env_->get_action_space(); }
  [[nodiscard]] float get_action_space_min() const override { return env_->get_action_space_min(); }
  [[nodiscard]] float get_action_space_max() const override { return env_->get_action_space_max(); }

  std::tuple<CarlaObsView, float, bool, bool, std::optional<env_info>> step(const float* action) override {
    auto [obs, reward, termination, truncation] = env_->step(action);
    std::optional<env_info> info = std::nullopt;
    episode_return_ += reward;
    episode_length_ += 1;
    if (termination || truncation) {
      const std::chrono::duration<float> dt = std::chrono::steady_clock::now() - episode_start_time_;
      info = env_info{episode_return_, episode_length_, dt.count()};
    }
    return {obs, reward, termination, truncation, info};
  }
};

// ac_ppo_carla.cpp:51-60
inline std::shared_ptr<EnvironmentWrapperCarla> make_env(const std::shared_ptr<EnvironmentCarla>& env_0) {
  return std::make_shared<RecordEpisodeStatisticsCarla>(env_0);
}

// gym.h:167-270: one state row per env, clip_actions, next-step autoreset (reset(-1), reward 0)
class SeqVectorEnvCarla {
  std::vector<std::shared_ptr<EnvironmentWrapperCarla>> env_array_;
  std::vector<uint8_t> bev_;
  std::vector<float> meas_, vmeas_, rewards_, terminations_, truncations_, clipped_;
  std::vector<std::optional<env_info>> infos_;
  std::vector<int> autoreset_envs_;
  const bool clip_actions_;
  size_t nb_ = 0;
  int nm_ = 0, nv_ = 0, A_ = 0;

  void put(int i, const CarlaObsView& o) {
    std::memcpy(bev_.data() + nb_ * i, o.bev_semantics, nb_);
    std::memcpy(meas_.data() + (size_t)nm_ * i, o.measurements, sizeof(float) * nm_);
    std::memcpy(vmeas_.data() + (size_t)nv_ * i, o.value_measurements, sizeof(float) * nv_);
  }

 public:
  const unsigned int num_envs_;

  struct State {
    const uint8_t* bev_semantics;       // [E, C, H, W]
    const float* measurements;          // [E, NM]
    const float* value_measurements;    // [E, NV]
  };

  SeqVectorEnvCarla(const std::vector<std::shared_ptr<EnvironmentWrapperCarla>>& env_array, const bool clip_actions)
      : env_array_(env_array), clip_actions_(clip_actions), num_envs_((unsigned)env_array.size()) {
    if (env_array_.empty()) throw std::runtime_error("SeqVectorEnvCarla needs at least one env");
    const auto s = env_array_[0]->get_observation_space();
    nb_ = (size_t)s[0] * s[1] * s[2];
    nm_ = s[3];
    nv_ = s[4];
    A_ = env_array_[0]->get_action_space();
    bev_.assign(nb_ * num_envs_, 0);
    meas_.assign((size_t)nm_ * num_envs_, 0.f);
    vmeas_.assign((size_t)nv_ * num_envs_, 0.f);
    rewards_.assign(num_envs_, 0.f);
    terminations_.assign(num_envs_, 0.f);
    truncations_.assign(num_envs_, 0.f);
    clipped_.assign(A_, 0.f);
    infos_.assign(num_envs_, std::nullopt);
    autoreset_envs_.assign(num_envs_, 0);
  }

  State state() const { return State{bev_.data(), meas_.data(), vmeas_.data()}; }
  [[nodiscard]] unsigned int get_num_envs() const { return num_envs_; }
  [[nodiscard]] std::vector<int> get_observation_space() const { return env_array_[0]->get_observation_space(); }
  [[nodiscard]] int get_action_space() const { return A_; }
  [[nodiscard]] float get_action_space_min() const { return env_array_[0]->get_action_space_min(); }
  [[nodiscard]] float get_action_space_max() const { return env_array_[0]->get_action_space_max(); }

  State reset(const int seed) {
    for (unsigned i = 0; i < num_envs_; ++i) {
      put((int)i, env_array_[i]->reset(seed + (int)i));
      autoreset_envs_[i] = 0;
    }
    return state();
  }

  // actions [E, A]; returns the state plus per-env rewards / terminations / truncations / infos
  std::tuple<State, const float*, const float*, const float*, const std::vector<std::optional<env_info>>*> step(
      const float* actions) {
    const float lo = get_action_space_min(), hi = get_action_space_max();
    for (unsigned i = 0; i < num_envs_; ++i) {
      if (autoreset_envs_[i]) {
        put((int)i, env_array_[i]->reset(-1));  // -1: do not reseed
        rewards_[i] = 0.0f;
        terminations_[i] = 0.0f;
        truncations_[i] = 0.0f;
        infos_[i] = std::nullopt;
        autoreset_envs_[i] = 0;
        continue;
      }
      const float* a = actions + (size_t)A_ * i;
      if (clip_actions_) {
        for (int k = 0; k < A_; ++k) clipped_[k] = std::clamp(a[k], lo, hi);
        a = clipped_.data();
      }
      auto [obs, reward, termination, truncation, info] = env_array_[i]->step(a);
      put((int)i, obs);
      rewards_[i] = reward;
      terminations_[i] = termination ? 1.0f : 0.0f;
      truncations_[i] = truncation ? 1.0f : 0.0f;
      infos_[i] = info;
      autoreset_envs_[i] = (termination || truncation) ? 1 : 0;
    }
    return {state(), rewards_.data(), terminations_.data(), truncations_.data(), &infos_};
  }
};

}  // namespace gymcpp
