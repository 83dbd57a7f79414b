// trainer_common.h — shared host code of the two drop-in trainer executables: flag parsing with
// the reference's names/defaults/syntax (args.hxx "--flag value", bools as 0/1, --gpu_ids appends to
// the default {0}, args.hxx:3324-3350 / :3693-3714), parameter initialisation, checkpoints, logging,
// environment construction and the C-ABI error check. No LibTorch: the agent lives on the GPU
// behind include/ppo_hip.h.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <filesystem>
#include <fstream>
#include <functional>
#include <iostream>
#include <map>
#include <memory>
#include <random>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/ppo_hip.h"
#include "../../include/ppo_pth.h"
#include "../../include/ppo_synth_env.h"
#include "../../include/ppo_env_wrappers.h"
#include "../gymcpp/gym.h"
#include "../gymcpp/synthetic_cheetah.h"
#include "tensorboard_logger.h"
#include "../gymcpp/wrappers.h"

namespace app {

inline void check(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string(what) + ": " + ppo_last_error());
}
#define HIPCHECK(x)                                                                                  \
  do {                                                                                               \
    hipError_t e_ = (x);                                                                             \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

// ------------------------------------------------------------------------------------------------
// flags
// ------------------------------------------------------------------------------------------------
struct ParseError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct HelpRequested {};

class Flags {
 public:
  struct Def {
    std::string help;
    std::function<void(const std::string&)> set;
    std::string current;
  };
  void add(const std::string& name, const std::string& help, int* v) {
    defs_[name] = {help, [v, name](const std::string& s) { *v = parse_int(s, name); }, std::to_string(*v)};
  }
  void add(const std::string& name, const std::string& help, unsigned* v) {
    defs_[name] = {help, [v, name](const std::string& s) { *v = (unsigned)parse_int(s, name); }, std::to_string(*v)};
  }
  void add(const std::string& name, const std::string& help, float* v) {
    defs_[name] = {help, [v, name](const std::string& s) { *v = parse_float(s, name); }, std::to_string(*v)};
  }
  void add(const std::string& name, const std::string& help, bool* v) {
    // args.hxx parses bools with istream >> bool: only "0" / "1"
    defs_[name] = {help, [v, name](const std::string& s) {
                     if (s == "0") *v = false;
                     else if (s == "1") *v = true;
                     else throw ParseError("Argument '" + name + "' received invalid value type '" + s + "'");
                   }, *v ? "1" : "0"};
  }
  void add(const std::string& name, const std::string& help, std::string* v) {
    defs_[name] = {help, [v](const std::string& s) { *v = s; }, *v};
  }
  void add_list(const std::string& name, const std::string& help, std::vector<int>* v) {
    // ValueFlagList: values APPEND to the default list (args.hxx:3693-3714)
    defs_[name] = {help, [v, name](const std::string& s) { v->push_back(parse_int(s, name)); }, "list"};
  }
  void parse(int argc, const char** argv) {
    for (int i = 1; i < argc; ++i) {
      std::string a = argv[i];
      if (a == "-h" || a == "--help") throw HelpRequested{};
      if (a.rfind("--", 0) != 0) throw ParseError("Passed in argument, but no positional arguments were ready to receive it: " + a);
      std::string name = a.substr(2), val;
      const auto eq = name.find('=');
      if (eq != std::string::npos) { val = name.substr(eq + 1); name = name.substr(0, eq); }
      auto it = defs_.find(name);
      if (it == defs_.end()) throw ParseError("Flag could not be matched: " + name);
      if (eq == std::string::npos) {
        if (i + 1 >= argc) throw ParseError("Flag '" + name + "' requires an argument but received none");
        val = argv[++i];
      }
      it->second.set(val);
    }
  }
  void print_help(std::ostream& os) const {
    os << "  OPTIONS:\n\n      -h, --help                        Display this help menu\n";
    for (auto& kv : defs_) os << "      --" << kv.first << " [" << kv.first << "]    " << kv.second.help << "\n";
  }

 private:
  static int parse_int(const std::string& s, const std::string& n) {
    try { size_t p; int v = std::stoi(s, &p); if (p != s.size()) throw 1; return v; }
    catch (...) { throw ParseError("Argument '" + n + "' received invalid value type '" + s + "'"); }
  }
  static float parse_float(const std::string& s, const std::string& n) {
    try { size_t p; float v = std::stof(s, &p); if (p != s.size()) throw 1; return v; }
    catch (...) { throw ParseError("Argument '" + n + "' received invalid value type '" + s + "'"); }
  }
  std::map<std::string, Def> defs_;
};

// ------------------------------------------------------------------------------------------------
// parameter initialisation (reference order, include/ppo_layout.h)
// ------------------------------------------------------------------------------------------------
// orthogonal_(W, gain) for W [rows, cols] (nn::init::orthogonal_, used by ppo:159-164): QR of a
// Gaussian matrix via modified Gram-Schmidt, sign-corrected.
inline void orthogonal(float* W, int rows, int cols, double gain, std::mt19937& rng) {
  const bool tall = rows >= cols;
  const int n = tall ? rows : cols, k = tall ? cols : rows;  // n x k matrix with orthonormal columns
  std::normal_distribution<double> nd(0.0, 1.0);
  std::vector<double> q((size_t)n * k);
  for (auto& x : q) x = nd(rng);
  for (int c = 0; c < k; ++c) {
    for (int p = 0; p < c; ++p) {
      double d = 0;
      for (int r = 0; r < n; ++r) d += q[(size_t)r * k + c] * q[(size_t)r * k + p];
      for (int r = 0; r < n; ++r) q[(size_t)r * k + c] -= d * q[(size_t)r * k + p];
    }
    double nrm = 0;
    for (int r = 0; r < n; ++r) nrm += q[(size_t)r * k + c] * q[(size_t)r * k + c];
    nrm = std::sqrt(nrm);
    for (int r = 0; r < n; ++r) q[(size_t)r * k + c] /= nrm;
  }
  for (int r = 0; r < rows; ++r)
    for (int c = 0; c < cols; ++c) W[(size_t)r * cols + c] = (float)(gain * (tall ? q[(size_t)r * k + c] : q[(size_t)c * k + r]));
}

inline std::vector<float> init_params(const ppo_layout& L, int seed, float act_hi, float act_lo,
                                      const std::vector<float>& obs_mean, const std::vector<float>& obs_std) {
  std::vector<float> P(L.P, 0.0f);
  std::mt19937 rng(seed > 0 ? seed : 1);
  const int H = L.H, O = L.O, A = L.A;
  if (L.kind == PPO_NET_TANH_NORMAL) {
    const ppo_trunk_layout* tr[2] = {&L.critic, &L.actor};
    for (int k = 0; k < 2; ++k) {
      orthogonal(&P[tr[k]->W1], H, O, std::sqrt(2.0), rng);
      orthogonal(&P[tr[k]->W2], H, H, std::sqrt(2.0), rng);
    }
    orthogonal(&P[L.cW3], 1, H, 1.0, rng);
    orthogonal(&P[L.aW3], A, H, 0.01, rng);
  } else {
    // LibTorch defaults: Linear U(-1/sqrt(fan_in), 1/sqrt(fan_in)) for weight and bias, LN 1 / 0
    auto unif = [&](long off, long n, int fan_in) {
      std::uniform_real_distribution<float> u(-1.0f / std::sqrt((float)fan_in), 1.0f / std::sqrt((float)fan_in));
      for (long i = 0; i < n; ++i) P[off + i] = u(rng);
    };
    P[L.hi] = act_hi;
    P[L.lo] = act_lo;
    for (int i = 0; i < O; ++i) {
      P[L.omean + i] = obs_mean.empty() ? 0.0f : obs_mean[i];
      P[L.ostd + i] = obs_std.empty() ? 1.0f : obs_std[i];
    }
    const ppo_trunk_layout* tr[2] = {&L.critic, &L.actor};
    for (int k = 0; k < 2; ++k) {
      unif(tr[k]->W1, (long)H * O, O); unif(tr[k]->b1, H, O);
      for (int i = 0; i < H; ++i) { P[tr[k]->g1 + i] = 1.0f; P[tr[k]->g2 + i] = 1.0f; }
      unif(tr[k]->W2, (long)H * H, H); unif(tr[k]->b2, H, H);
    }
    unif(L.cW3, H, H); unif(L.cb3, 1, H);
    unif(L.aW3, (long)A * H, H); unif(L.ab3, A, H);
    unif(L.bW3, (long)A * H, H); unif(L.bb3, A, H);
  }
  return P;
}

// ------------------------------------------------------------------------------------------------
// checkpoints: flat fp32 parameters + Adam state (reference: torch::save(agent / optimizer) every
// iteration, ppo:173-180 / :545-563; .pth interop is a SURVEY §8f "next" item)
// ------------------------------------------------------------------------------------------------
// save_state (ppo:173-180): torch::save(agent, model_file) and torch::save(optimizer,
// optimizer_file) as LibTorch module archives (include/ppo_pth.h), loadable by torch::load in the
// reference's tools (e.g. src/carla/ppo_carla_inference.cpp:104) and by torch.jit.load
inline void save_state(ppo_t* ctx, const std::filesystem::path& folder, const std::string& model_file,
                       const std::string& optimizer_file, double lr, double adam_eps) {
  ppo_layout L;
  check(ppo_get_layout(ctx, &L), "ppo_get_layout");
  std::vector<float> p(L.P), m(L.P), v(L.P);
  long step = 0;
  check(ppo_save_params(ctx, p.data(), L.P), "ppo_save_params");
  check(ppo_save_adam(ctx, m.data(), v.data(), L.P, &step), "ppo_save_adam");
  check(ppo_pth_save_agent(&L, p.data(), (folder / model_file).string().c_str()), "ppo_pth_save_agent");
  check(ppo_pth_save_adam(&L, m.data(), v.data(), step, lr, adam_eps, (folder / optimizer_file).string().c_str()),
        "ppo_pth_save_adam");
}

// keeps only this iteration's model_latest_* / optimizer_latest_* (ppo:548-563)
inline void cleanup_checkpoints(const std::filesystem::path& folder, long iteration);

// The per-iteration checkpoint of the reference (ppo:545-563, ac:904-927: model_latest_%09d.pth +
// optimizer_latest_%09d.pth, older ones deleted) off the critical path: request()
// enqueues a device-side snapshot of parameters + Adam state behind the update just launched and
// returns; a writer thread waits for that snapshot, copies it out and writes / prunes the archives
// while the GPU runs the next iteration. One request in flight: a new one first waits until the
// writer has copied the previous snapshot out. Errors surface on the next request() / finish().
class AsyncCheckpointer {
  struct Job {
    std::filesystem::path folder;
    std::string model_file, optimizer_file;
    double lr, eps;
    long cleanup_iteration;  // < 0: no pruning
  };
  ppo_t* ctx_;
  ppo_layout L_{};
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool have_job_ = false, snapshot_free_ = true, idle_ = true, stop_ = false;
  Job job_;
  std::string error_;

  void run() {
    std::vector<float> p(L_.P), m(L_.P), v(L_.P);
    for (;;) {
      Job j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return have_job_ || stop_; });
        if (!have_job_ && stop_) return;
        j = job_;
        have_job_ = false;
        idle_ = false;
      }
      std::string err;
      long step = 0;
      if (ppo_read_snapshot(ctx_, p.data(), m.data(), v.data(), L_.P, &step) != 0) err = ppo_last_error();
      {
        std::lock_guard<std::mutex> lk(mu_);
        snapshot_free_ = true;
      }
      cv_.notify_all();
      if (err.empty() && ppo_pth_save_agent(&L_, p.data(), (j.folder / j.model_file).string().c_str()) != 0)
        err = ppo_last_error();
      if (err.empty() && ppo_pth_save_adam(&L_, m.data(), v.data(), step, j.lr, j.eps,
                                           (j.folder / j.optimizer_file).string().c_str()) != 0)
        err = ppo_last_error();
      if (err.empty() && j.cleanup_iteration >= 0) {
        try {
          cleanup_checkpoints(j.folder, j.cleanup_iteration);
        } catch (const std::exception& e) {
          err = e.what();
        }
      }
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (!err.empty() && error_.empty()) error_ = "checkpoint: " + err;
        idle_ = true;
      }
      cv_.notify_all();
    }
  }

 public:
  explicit AsyncCheckpointer(ppo_t* ctx) : ctx_(ctx) {
    check(ppo_get_layout(ctx, &L_), "ppo_get_layout");
    th_ = std::thread([this] { run(); });
  }
  ~AsyncCheckpointer() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
  }
  void request(const std::filesystem::path& folder, const std::string& model_file, const std::string& optimizer_file,
               double lr, double eps, long cleanup_iteration) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return snapshot_free_ && !have_job_; });
    if (!error_.empty()) throw std::runtime_error(error_);
    check(ppo_snapshot_state(ctx_), "ppo_snapshot_state");
    job_ = Job{folder, model_file, optimizer_file, lr, eps, cleanup_iteration};
    have_job_ = true;
    snapshot_free_ = false;
    lk.unlock();
    cv_.notify_all();
  }
  // waits until every requested checkpoint is on disk
  void finish() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return !have_job_ && idle_; });
    if (!error_.empty()) throw std::runtime_error(error_);
  }
};
inline void cleanup_checkpoints(const std::filesystem::path& folder, long iteration) {
  char keep_m[64], keep_o[64];
  std::snprintf(keep_m, sizeof keep_m, "model_latest_%09ld.pth", iteration);
  std::snprintf(keep_o, sizeof keep_o, "optimizer_latest_%09ld.pth", iteration);
  for (const auto& e : std::filesystem::directory_iterator(folder)) {
    const std::string fn = e.path().filename().string();
    const bool pth = fn.size() > 4 && fn.compare(fn.size() - 4, 4, ".pth") == 0;
    if (pth && ((fn.rfind("model_latest_", 0) == 0 && fn != keep_m) ||
                (fn.rfind("optimizer_latest_", 0) == 0 && fn != keep_o)))
      std::filesystem::remove(e.path());
  }
}

// scalar log (one JSON object per line: {"tag", "step", "value"}) — the TensorBoard event writer is
// the SURVEY §8f-1 "next" item; tag names follow the reference (ppo:426-432, :575-583)
class ScalarLog {
  std::ofstream f_;

 public:
  explicit ScalarLog(const std::filesystem::path& p) : f_(p) {}
  void add_scalar(const std::string& tag, long step, double v) {
    f_ << "{\"tag\": \"" << tag << "\", \"step\": " << step << ", \"value\": " << v << "}\n";
    f_.flush();
  }
};

// The reference's TensorBoard event file (tfevents_logs[_rank].pb, ppo:281 / ac:420) plus the same
// scalars as JSON lines. Steps go to the event file as int, as the reference's static_cast<int>.
class RunLog {
  TensorBoardLogger tb_;
  ScalarLog js_;

 public:
  RunLog(const std::filesystem::path& dir, const std::string& tfevents_name, const std::string& jsonl_name)
      : tb_((dir / tfevents_name).string()), js_(dir / jsonl_name) {}
  void add_scalar(const std::string& tag, long step, double v) {
    tb_.add_scalar(tag, static_cast<int>(step), v);
    js_.add_scalar(tag, step, v);
  }
};

// ------------------------------------------------------------------------------------------------
// environments
// ------------------------------------------------------------------------------------------------
struct EnvSpec {
  int obs_dim = 0, act_dim = 0;
  float act_min = -1, act_max = 1;
};

// Shape of the device env (--env_backend device) for an env id: the synthetic dynamics of
// include/ppo_synth_env.h at the observation / action widths and action bounds of the reference's
// MuJoCo env (libs/gymcpp/mujoco/half_cheetah_v5.h:31-34, humanoid_v4.h:27-30, ant_v5.h:38-41,
// hopper_v5.h:35-38). Returns false for an unknown id.
struct EnvShape {
  int O, A;
  float lo, hi;
};
inline bool device_env_shape(const std::string& env_id, EnvShape* s) {
  if (env_id == "HalfCheetah-v5" || env_id == "SyntheticCheetah-v0") *s = {17, 6, -1.0f, 1.0f};
  else if (env_id == "Humanoid-v4") *s = {376, 17, -0.4f, 0.4f};
  else if (env_id == "Ant-v5") *s = {105, 8, -1.0f, 1.0f};
  else if (env_id == "Hopper-v5") *s = {11, 3, -1.0f, 1.0f};
  else return false;
  return true;
}

// creates one base env; MuJoCo envs need libmujoco 3.2.0 (absent from this build)
inline std::shared_ptr<gymcpp::Environment> make_base_env(const std::string& env_id) {
  if (env_id == "SyntheticCheetah-v0") return std::make_shared<gymcpp::SyntheticCheetah>();
  if (env_id == "Humanoid-v4" || env_id == "HalfCheetah-v5" || env_id == "Ant-v5" || env_id == "Hopper-v5")
    throw std::invalid_argument("env_id: " + env_id +
                                " needs MuJoCo 3.2.0, which this build does not link; use SyntheticCheetah-v0 "
                                "or the device env (--env_backend device)");
  throw std::invalid_argument("env_id: " + env_id + " is not implemented.");
}

// Host threads this process may use: the launcher's thread budget (OMP_NUM_THREADS, set to the box's
// CPU share), else the cgroup CPU quota, else the hardware concurrency.
inline int host_threads() {
  if (const char* v = std::getenv("OMP_NUM_THREADS"))
    if (std::atoi(v) > 0) return std::atoi(v);
  std::ifstream f("/sys/fs/cgroup/cpu.max");
  std::string q, per;
  if (f >> q >> per && q != "max" && std::atol(per.c_str()) > 0)
    return std::max(1L, std::atol(q.c_str()) / std::atol(per.c_str()));
  return std::max(1u, std::thread::hardware_concurrency());
}

inline double seconds_since(std::chrono::high_resolution_clock::time_point t0) {
  return std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - t0).count();
}

}  // namespace app
