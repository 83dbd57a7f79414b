// ref_harness.cpp — golden-vector generator that runs the REFERENCE's arithmetic on LibTorch CPU.
//
// TEST INFRASTRUCTURE ONLY: built by oracle/Makefile into oracle/_ref/ (git-ignored), run once to
// write tests/golden/*. Nothing in the product links or loads it.
//
// What is the reference here:
//   * include/rl_utils.h (Normal / Dirichlet / Beta) is compiled AS-IS from /root/reference
//     (-I/root/reference/include) — the distributions are the reference's own code.
//   * The agents and the loss/update arithmetic live inline in the reference's main() functions,
//     which cannot be compiled here (boost, MPI, MuJoCo, protobuf are absent). They are replayed
//     with the same LibTorch calls, in the same order, as:
//       ppo_continuous_action.cpp:120-157 (AgentImpl), :447-467 (GAE), :489-540 (update)
//       ac_ppo_continuous_action.cpp:150-249 (AgentImpl), :803-888 (update, distributed adv norm)
//   * LibTorch is the pip wheel's 2.10 CPU build (reference pins 2.4.1); ATen formulas for addmm,
//     tanh, layer_norm, softplus, lgamma/digamma, clip_grad_norm_ and Adam are unchanged across
//     those versions. RNG streams are not used: every random input is injected.
#include <rl_utils.h>
#include <torch/torch.h>

#include "ppo_oracle.h"  // the synthetic env and the Philox sampling draws (end-to-end case only)

#include <algorithm>
#include <memory>
#include <chrono>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <filesystem>
#include <fstream>
#include <random>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

using torch::Tensor;
namespace nn = torch::nn;

static std::string g_out;
static std::ostringstream g_manifest;
static bool g_first_case = true;
static bool g_first_entry = true;

static void begin_case(const std::string& name, const std::string& meta_json) {
  g_manifest << (g_first_case ? "" : ",\n") << "  \"" << name << "\": {\"meta\": " << meta_json << ", \"arrays\": {";
  g_first_case = false;
  g_first_entry = true;
  std::filesystem::create_directories(g_out + "/" + name);
}
static void end_case() { g_manifest << "}}"; }

static void dump(const std::string& cname, const std::string& name, const Tensor& t0) {
  Tensor t = t0.detach().contiguous();
  std::string dt;
  if (t.scalar_type() == torch::kFloat32) dt = "f32";
  else if (t.scalar_type() == torch::kInt64) dt = "i64";
  else { t = t.to(torch::kFloat32); dt = "f32"; }
  std::string path = g_out + "/" + cname + "/" + name + "." + dt;
  std::ofstream f(path, std::ios::binary);
  f.write(reinterpret_cast<const char*>(t.data_ptr()), t.numel() * t.element_size());
  g_manifest << (g_first_entry ? "" : ", ") << "\"" << name << "\": {\"dtype\": \"" << dt << "\", \"shape\": [";
  for (int64_t i = 0; i < t.dim(); ++i) g_manifest << (i ? ", " : "") << t.size(i);
  g_manifest << "]}";
  g_first_entry = false;
}

// ---------------------------------------------------------------------------------------------
// Agents (same module structure / registration order as the reference, so named_parameters()
// order equals the reference's flat order).
// ---------------------------------------------------------------------------------------------
struct PPOAgentImpl : nn::Module {  // ppo_continuous_action.cpp:120-157
  nn::Sequential critic{nullptr}, actor_mean{nullptr};
  Tensor actor_logstd;
  PPOAgentImpl(int O, int A, int H) {
    critic = register_module("critic", nn::Sequential(nn::Linear(O, H), nn::Tanh(), nn::Linear(H, H), nn::Tanh(),
                                                      nn::Linear(H, 1)));
    actor_mean = register_module("actor_mean", nn::Sequential(nn::Linear(O, H), nn::Tanh(), nn::Linear(H, H),
                                                              nn::Tanh(), nn::Linear(H, A)));
    actor_logstd = register_parameter("actor_logstd", torch::zeros({1, A}, torch::kFloat32));
  }
  Tensor get_value(const Tensor& x) { return critic->forward(x); }
  std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> get_action_and_value(const Tensor& x, const Tensor& action) {
    const Tensor action_mean = actor_mean->forward(x);
    const Tensor action_logstd = actor_logstd.expand_as(action_mean);
    const Tensor action_std = torch::exp(action_logstd);
    const Normal probs(action_mean, action_std);
    Tensor logprob = probs.log_prob(action).sum(1);
    Tensor entropy = probs.entropy().sum(1);
    Tensor value = critic->forward(x);
    return {action, logprob, entropy, value, action_mean};
  }
};
TORCH_MODULE(PPOAgent);

struct ACAgentImpl : nn::Module {  // ac_ppo_continuous_action.cpp:150-249
  nn::Sequential critic{nullptr}, actor_encoder{nullptr}, dist_alpha{nullptr}, dist_beta{nullptr};
  Tensor action_space_high, action_space_low, mean_, std_;
  ACAgentImpl(int O, int A, int H, float high, float low, Tensor mean, Tensor std) {
    action_space_high = register_parameter("action_space_high", torch::tensor(high), false);
    action_space_low = register_parameter("action_space_low", torch::tensor(low), false);
    mean_ = register_parameter("mean_", mean.unsqueeze(0), false);
    std_ = register_parameter("std_", std.unsqueeze(0), false);
    critic = register_module("critic", nn::Sequential(nn::Linear(O, H), nn::LayerNorm(nn::LayerNormOptions({H})),
                                                      nn::ReLU(), nn::Linear(H, H),
                                                      nn::LayerNorm(nn::LayerNormOptions({H})), nn::ReLU(),
                                                      nn::Linear(H, 1)));
    actor_encoder = register_module(
        "actor_mean", nn::Sequential(nn::Linear(O, H), nn::LayerNorm(nn::LayerNormOptions({H})), nn::ReLU(),
                                     nn::Linear(H, H), nn::LayerNorm(nn::LayerNormOptions({H})), nn::ReLU()));
    dist_alpha = register_module("dist_alpha", nn::Sequential(nn::Linear(H, A)));
    dist_beta = register_module("dist_beta", nn::Sequential(nn::Linear(H, A)));
  }
  Tensor scale_action(const Tensor& action) const {
    constexpr float d_low = 0.0f, d_high = 1.0f, eps = 1e-7;
    Tensor s = (action - action_space_low) / (action_space_high - action_space_low) * (d_high - d_low) + d_low;
    return torch::clamp(s, d_low + eps, d_high + eps);
  }
  Tensor unscale_action(const Tensor& action) const {
    constexpr float d_low = 0.0f, d_high = 1.0f;
    return (action - d_low) / (d_high - d_low) * (action_space_high - action_space_low) + action_space_low;
  }
  // mode: "given" (update path) or "mean" (eval path)
  std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> get_action_and_value(const Tensor& x, Tensor action,
                                                                                  const std::string& mode) {
    Tensor xn = (x - mean_) / std_;
    Tensor feat = actor_encoder->forward(xn);
    Tensor alpha = nn::functional::softplus(dist_alpha->forward(feat)) + 1.0f;
    Tensor beta = nn::functional::softplus(dist_beta->forward(feat)) + 1.0f;
    const Beta probs(alpha, beta);
    if (mode == "mean") action = probs.mean();
    else action = scale_action(action);
    Tensor logprob = probs.log_prob(action).sum(1);
    action = unscale_action(action);
    Tensor entropy = probs.entropy().sum(1);
    Tensor value = critic->forward(xn);
    return {action, logprob, entropy, value, alpha, beta};
  }
};
TORCH_MODULE(ACAgent);

// ---------------------------------------------------------------------------------------------
// Deterministic inputs
// ---------------------------------------------------------------------------------------------
// CaRL CNN agent (include/carla/carla_model.h:21-318 with the carla_config.h defaults: "roach"
// encoder, no LayerNorm, no positional encoding). The reference header needs OpenCV and
// boost::format, absent here, so the module is restated with the same LibTorch modules in the same
// registration order; the Beta distribution is the reference's own rl_utils.h.
struct CarlaAgentImpl : nn::Module {
  nn::Sequential cnn{nullptr}, linear{nullptr}, state_linear{nullptr}, value_head{nullptr}, policy_head{nullptr},
      dist_mu{nullptr}, dist_sigma{nullptr};
  Tensor action_space_high, action_space_low;
  float beta_min;
  CarlaAgentImpl(int C, int NM, int NV, int A, float hi, float lo, float bmin) : beta_min(bmin) {
    auto conv = [](int i, int o, int k, int st) { return nn::Conv2d(nn::Conv2dOptions(i, o, k).stride(st)); };
    cnn = register_module("cnn", nn::Sequential(conv(C, 8, 5, 2), nn::ReLU(), conv(8, 16, 5, 2), nn::ReLU(),
                                                 conv(16, 32, 5, 2), nn::ReLU(), conv(32, 64, 3, 2), nn::ReLU(),
                                                 conv(64, 128, 3, 2), nn::ReLU(), conv(128, 256, 3, 1), nn::ReLU()));
    linear = register_module("linear", nn::Sequential(nn::Linear(1024 + 256, 512), nn::ReLU(), nn::Linear(512, 256),
                                                      nn::ReLU()));
    state_linear = register_module("state_linear", nn::Sequential(nn::Linear(NM, 256), nn::ReLU(),
                                                                  nn::Linear(256, 256), nn::ReLU()));
    value_head = register_module("value_head", nn::Sequential(nn::Linear(256 + NV, 256), nn::ReLU(),
                                                              nn::Linear(256, 256), nn::ReLU(), nn::Linear(256, 1)));
    policy_head = register_module("policy_head", nn::Sequential(nn::Linear(256, 256), nn::ReLU(),
                                                                nn::Linear(256, 256), nn::ReLU()));
    dist_mu = register_module("dist_mu", nn::Sequential(nn::Linear(256, A)));
    dist_sigma = register_module("dist_sigma", nn::Sequential(nn::Linear(256, A)));
    action_space_high = register_parameter("action_space_high", torch::tensor(hi), false);
    action_space_low = register_parameter("action_space_low", torch::tensor(lo), false);
  }
  Tensor encoder(const Tensor& bev_u8, const Tensor& meas) {  // carla_model.h:222-242
    Tensor birdview = bev_u8.to(torch::kFloat32) / 255.0f;
    Tensor x = torch::flatten(cnn->forward(birdview), 1);
    Tensor latent_state = state_linear->forward(meas);
    return linear->forward(torch::cat({x, latent_state}, 1));
  }
  // carla_model.h:270-318; sample types "mean", "roach", or a given action
  std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> forward(const Tensor& bev, const Tensor& meas,
                                                                             const Tensor& vmeas, Tensor actions,
                                                                             const std::string& mode) {
    Tensor features = encoder(bev, meas);
    Tensor values = value_head->forward(torch::cat({features, vmeas}, 1));
    Tensor latent_pi = policy_head->forward(features);
    Tensor mu = nn::functional::softplus(dist_mu->forward(latent_pi)) + beta_min;
    Tensor sigma = nn::functional::softplus(dist_sigma->forward(latent_pi)) + beta_min;
    const Beta dist(mu, sigma);
    if (mode == "mean") actions = dist.mean();
    else if (mode == "roach") actions = dist.roach_deterministic();
    else {
      actions = (actions - action_space_low) / (action_space_high - action_space_low) * (1.0f - 0.0f) + 0.0f;
      actions = torch::clamp(actions, 0.0f + 1e-7f, 1.0f + 1e-7f);
    }
    Tensor log_prob = dist.log_prob(actions).sum(1);
    actions = (actions - 0.0f) / (1.0f - 0.0f) * (action_space_high - action_space_low) + action_space_low;
    Tensor entropy = dist.entropy().sum(1);
    return {actions, log_prob, entropy, values, mu, sigma, features};
  }
};
TORCH_MODULE(CarlaAgent);

// Deterministic CaRL inputs / parameters shared with tests/carla_inputs.py (so the 1+ MB image
// batch and the 1.2 M parameters need not be stored): u = (mix32(mix32(stream * 0x9E3779B1) ^ i)
// >> 8 + 0.5) * 2^-24, mix32 = the murmur3 finalizer (oracle orc_mix32).
static uint32_t hmix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85EBCA6Bu;
  h ^= h >> 13; h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
static uint32_t hbits(uint32_t stream, uint32_t i) { return hmix32(hmix32(stream * 0x9E3779B1u) ^ i); }
static float hu01(uint32_t stream, uint32_t i) { return ((float)(hbits(stream, i) >> 8) + 0.5f) * 5.9604644775390625e-8f; }
static Tensor hunif(uint32_t stream, std::vector<int64_t> shape, float lo, float hi) {
  Tensor t = torch::empty(shape, torch::kFloat32);
  float* p = t.data_ptr<float>();
  for (int64_t i = 0; i < t.numel(); ++i) p[i] = lo + (hi - lo) * hu01(stream, (uint32_t)i);
  return t;
}

static std::mt19937 g_rng(1234);
static Tensor randn(std::vector<int64_t> shape, float scale = 1.0f) {
  std::normal_distribution<float> d(0.0f, 1.0f);
  Tensor t = torch::empty(shape, torch::kFloat32);
  float* p = t.data_ptr<float>();
  for (int64_t i = 0; i < t.numel(); ++i) p[i] = d(g_rng) * scale;
  return t;
}
static Tensor randu(std::vector<int64_t> shape, float lo, float hi) {
  std::uniform_real_distribution<float> d(lo, hi);
  Tensor t = torch::empty(shape, torch::kFloat32);
  float* p = t.data_ptr<float>();
  for (int64_t i = 0; i < t.numel(); ++i) p[i] = d(g_rng);
  return t;
}

// Fill every parameter with deterministic values of a sensible scale and return the flat vector
// in named_parameters() order (and the names, for the manifest).
static Tensor set_params(nn::Module& m, std::string& names_json) {
  torch::NoGradGuard ng;
  std::vector<Tensor> flat;
  names_json = "[";
  bool first = true;
  for (auto& kv : m.named_parameters()) {
    Tensor p = kv.value();
    const std::string& n = kv.key();
    Tensor v;
    if (n == "action_space_high") v = torch::tensor(1.0f);
    else if (n == "action_space_low") v = torch::tensor(-1.0f);
    else if (n == "mean_") v = randn(p.sizes().vec(), 0.1f);
    else if (n == "std_") v = randu(p.sizes().vec(), 0.8f, 1.5f);
    else if (n == "actor_logstd") v = randu(p.sizes().vec(), -0.7f, -0.3f);
    else if (n.find("weight") != std::string::npos && p.dim() == 1) v = randu(p.sizes().vec(), 0.8f, 1.2f);  // LN gamma
    else if (n.find("weight") != std::string::npos) v = randn(p.sizes().vec(), 1.0f / std::sqrt((float)p.size(1)));
    else v = randn(p.sizes().vec(), 0.1f);  // biases / LN beta
    p.copy_(v.reshape(p.sizes()));
    flat.push_back(p.detach().reshape({-1}).clone());
    names_json += std::string(first ? "" : ", ") + "[\"" + n + "\", " + std::to_string(p.numel()) + ", " +
                  (p.requires_grad() ? "1" : "0") + "]";
    first = false;
  }
  names_json += "]";
  return torch::cat(flat);
}

static Tensor flat_grads(nn::Module& m) {
  std::vector<Tensor> g;
  for (auto& p : m.parameters()) {
    if (p.grad().defined()) g.push_back(p.grad().detach().reshape({-1}).clone());
    else g.push_back(torch::zeros({p.numel()}));
  }
  return torch::cat(g);
}
static Tensor flat_params(nn::Module& m) {
  std::vector<Tensor> g;
  for (auto& p : m.parameters()) g.push_back(p.detach().reshape({-1}).clone());
  return torch::cat(g);
}
static Tensor flat_state(torch::optim::Adam& opt, bool sq) {
  std::vector<Tensor> out;
  for (auto& p : opt.param_groups()[0].params()) {
    auto it = opt.state().find(p.unsafeGetTensorImpl());
    if (it == opt.state().end()) { out.push_back(torch::zeros({p.numel()})); continue; }
    auto& st = static_cast<torch::optim::AdamParamState&>(*it->second);
    out.push_back((sq ? st.exp_avg_sq() : st.exp_avg()).reshape({-1}).clone());
  }
  return torch::cat(out);
}

// ---------------------------------------------------------------------------------------------
// Losses (ppo:497-535 ; ac:817-872 with world_size = G emulated by row shards)
// ---------------------------------------------------------------------------------------------
struct LossCfg { float clip_coef, ent_coef, vf_coef; bool clip_vloss, norm_adv; };

static std::tuple<Tensor, std::vector<float>> ppo_loss(const Tensor& newlogprob, const Tensor& entropy,
                                                       Tensor newvalue, const Tensor& old_logp, Tensor mb_adv,
                                                       const Tensor& ret, const Tensor& old_v, const LossCfg& c,
                                                       const Tensor* adv_mean, const Tensor* adv_std) {
  Tensor logratio = newlogprob - old_logp;
  Tensor ratio = logratio.exp();
  Tensor old_approx_kl, approx_kl;
  float clipfrac;
  {
    torch::NoGradGuard ng;
    old_approx_kl = (-logratio).mean();
    approx_kl = ((ratio - 1.0f) - logratio).mean();
    clipfrac = ((ratio - 1.0f).abs() > c.clip_coef).to(torch::kFloat).mean().item<float>();
  }
  if (c.norm_adv) {
    if (adv_mean) mb_adv = (mb_adv - *adv_mean) / (*adv_std + 1e-8);  // distributed form (ac:848)
    else mb_adv = (mb_adv - mb_adv.mean()) / (mb_adv.std() + 1e-8);   // ppo:511
  }
  Tensor pg_loss1 = -mb_adv * ratio;
  Tensor pg_loss2 = -mb_adv * torch::clamp(ratio, 1.0f - c.clip_coef, 1.0f + c.clip_coef);
  Tensor pg_loss = torch::max(pg_loss1, pg_loss2).mean();
  newvalue = newvalue.view(-1);
  Tensor v_loss;
  if (c.clip_vloss) {
    Tensor v_loss_unclipped = torch::pow(newvalue - ret, 2);
    Tensor v_clipped = old_v + torch::clamp(newvalue - old_v, -c.clip_coef, c.clip_coef);
    Tensor v_loss_clipped = torch::pow(v_clipped - ret, 2);
    v_loss = 0.5f * torch::max(v_loss_unclipped, v_loss_clipped).mean();
  } else {
    v_loss = 0.5 * torch::pow(newvalue - ret, 2).mean();
  }
  Tensor entropy_loss = entropy.mean();
  Tensor loss = pg_loss - c.ent_coef * entropy_loss + v_loss * c.vf_coef;
  std::vector<float> st = {pg_loss.item<float>(),      v_loss.item<float>(),   entropy_loss.item<float>(),
                           old_approx_kl.item<float>(), approx_kl.item<float>(), clipfrac, loss.item<float>()};
  return {loss, st};
}

// ---------------------------------------------------------------------------------------------
// Round-2 cases: the agents at the widths the reference builds (AC 2x256 LayerNorm trunks,
// ac:159-186, at HalfCheetah O=17/A=6 and Ant O=105/A=8; the PPO 2x64 tanh agent at Humanoid
// O=376/A=17, ppo:122-139), GAE at cfg2's T=2048 and at ragged T, and the PPO env wrapper chain.
// Parameters are drawn from hash streams (tests/golden_inputs.py restates the draw), so only the
// inputs and outputs are stored.
// ---------------------------------------------------------------------------------------------
// tensor t of named_parameters() from stream base + t: 2-D weights U(+-sqrt(3 / fan_in)), LayerNorm
// gamma U(0.8, 1.2), biases / LayerNorm beta U(+-0.1), mean_ U(+-0.1), std_ U(0.8, 1.5),
// actor_logstd U(-0.7, -0.3), action_space_high / low = hi / lo
static Tensor hash_params(nn::Module& m, uint32_t base, float hi, float lo, std::string& names_json) {
  torch::NoGradGuard ng;
  std::vector<Tensor> flat;
  names_json = "[";
  uint32_t t = 0;
  for (auto& kv : m.named_parameters()) {
    Tensor p = kv.value();
    const std::string& n = kv.key();
    const uint32_t s = base + t;
    const std::vector<int64_t> shape = p.sizes().vec();
    Tensor v;
    if (n == "action_space_high") v = torch::tensor(hi);
    else if (n == "action_space_low") v = torch::tensor(lo);
    else if (n == "mean_") v = hunif(s, shape, -0.1f, 0.1f);
    else if (n == "std_") v = hunif(s, shape, 0.8f, 1.5f);
    else if (n == "actor_logstd") v = hunif(s, shape, -0.7f, -0.3f);
    else if (n.find("weight") != std::string::npos && p.dim() == 1) v = hunif(s, shape, 0.8f, 1.2f);
    else if (n.find("weight") != std::string::npos) {
      const float a = std::sqrt(3.0f / (float)p.size(1));
      v = hunif(s, shape, -a, a);
    } else v = hunif(s, shape, -0.1f, 0.1f);
    p.copy_(v.reshape(p.sizes()));
    flat.push_back(p.detach().reshape({-1}).clone());
    names_json += std::string(t ? ", " : "") + "[\"" + n + "\", " + std::to_string(p.numel()) + ", " +
                  (p.requires_grad() ? "1" : "0") + "]";
    ++t;
  }
  names_json += "]";
  return torch::cat(flat);
}

// GAE exactly as ppo:447-467 / ac:759-779 (LibTorch ops, float32)
static std::pair<Tensor, Tensor> gae_ref(const Tensor& rewards, const Tensor& values, const Tensor& dones,
                                         const Tensor& next_value, const Tensor& next_done, float gamma,
                                         float gae_lambda) {
  torch::NoGradGuard ng;
  const int64_t T = rewards.size(0), E = rewards.size(1);
  Tensor advantages = torch::zeros({T, E});
  Tensor lastgaelam = torch::zeros({E});
  Tensor nextnonterminal, nextvalues;
  for (int64_t t = T - 1; t >= 0; --t) {
    if (t == T - 1) { nextnonterminal = 1.0f - next_done; nextvalues = next_value; }
    else { nextnonterminal = 1.0 - dones.index({t + 1}); nextvalues = values.index({t + 1}); }
    Tensor delta = rewards.index({t}) + gamma * nextvalues * nextnonterminal - values.index({t});
    advantages.index({t}) = delta + gamma * gae_lambda * nextnonterminal * lastgaelam;
    lastgaelam = advantages.index({t});
  }
  return {advantages, advantages + values};
}

// FNV-1a 64 over the float32 bit patterns of column e, rows t = 0 .. T-1 (bit-exact check of a
// [T, E] array without storing it; tests/golden_inputs.py computes the same)
static Tensor column_fnv(const Tensor& a) {
  Tensor c = a.contiguous();
  const int64_t T = c.size(0), E = c.size(1);
  const float* p = c.data_ptr<float>();
  Tensor out = torch::empty({E}, torch::kInt64);
  int64_t* o = out.data_ptr<int64_t>();
  for (int64_t e = 0; e < E; ++e) {
    uint64_t h = 14695981039346656037ull;
    for (int64_t t = 0; t < T; ++t) {
      uint32_t b;
      std::memcpy(&b, p + t * E + e, 4);
      h ^= b;
      h *= 1099511628211ull;
    }
    o[e] = (int64_t)h;
  }
  return out;
}

static std::string f2s(float v) {
  std::ostringstream s;
  s.precision(9);
  s << v;
  return s.str();
}

static void ppo_width_case(const std::string& pre, int O, int A, int H, int M, uint32_t base) {
  PPOAgent agent(O, A, H);
  std::string names;
  Tensor p0 = hash_params(*agent, base, 1.0f, -1.0f, names);
  Tensor x = randn({M, O});
  Tensor act = randn({M, A}, 0.5f);
  const std::string dims = "\"kind\": 0, \"O\": " + std::to_string(O) + ", \"A\": " + std::to_string(A) +
                           ", \"H\": " + std::to_string(H) + ", \"hash_base\": " + std::to_string(base);
  const std::string ca = pre + "_act";
  begin_case(ca, "{" + dims + ", \"n\": " + std::to_string(M) + ", \"params\": " + names + "}");
  {
    torch::NoGradGuard ng;
    auto [a, lp, ent, v, mu] = agent->get_action_and_value(x, act);
    dump(ca, "x", x); dump(ca, "action", act);
    dump(ca, "logprob", lp); dump(ca, "entropy", ent); dump(ca, "value", v.view(-1)); dump(ca, "mean", mu);
  }
  end_case();
  const LossCfg c{0.2f, 0.01f, 0.5f, true, true};
  Tensor old_logp, old_v, adv = randn({M}), ret = randn({M});
  {
    torch::NoGradGuard ng;
    auto [a, lp, ent, v, mu] = agent->get_action_and_value(x, act);
    old_logp = lp + randn({M}, 0.15f);
    old_v = v.view(-1) + randn({M}, 0.15f);
  }
  torch::optim::Adam opt(agent->parameters(), torch::optim::AdamOptions(3e-4).eps(1e-5));
  const std::string cu = pre + "_update";
  begin_case(cu, "{" + dims + ", \"M\": " + std::to_string(M) +
                     ", \"clip_coef\": 0.2, \"ent_coef\": 0.01, \"vf_coef\": 0.5, \"clip_vloss\": 1, \"norm_adv\": 1, "
                     "\"max_grad_norm\": 0.5, \"lr\": 0.0003, \"adam_eps\": 1e-05}");
  dump(cu, "x", x); dump(cu, "action", act); dump(cu, "old_logp", old_logp); dump(cu, "adv", adv);
  dump(cu, "ret", ret); dump(cu, "old_v", old_v);
  for (int s = 1; s <= 3; ++s) {  // ppo:497-540, Tensor::std() advantage normalisation
    auto [a, lp, ent, v, mu] = agent->get_action_and_value(x, act);
    auto [loss, st] = ppo_loss(lp, ent, v, old_logp, adv, ret, old_v, c, nullptr, nullptr);
    opt.zero_grad();
    loss.backward();
    if (s == 1) { dump(cu, "grad_raw", flat_grads(*agent)); dump(cu, "stats", torch::tensor(st)); }
    const double tn = torch::nn::utils::clip_grad_norm_(agent->parameters(), 0.5);
    if (s == 1) dump(cu, "total_norm", torch::tensor({(float)tn}));
    opt.step();
    if (s == 1) dump(cu, "params_step1", flat_params(*agent));
  }
  dump(cu, "params_step3", flat_params(*agent));
  end_case();
}

static void ac_width_case(const std::string& pre, int O, int A, int H, int M, uint32_t base, float hi, float lo) {
  ACAgent agent(O, A, H, hi, lo, torch::zeros({O}), torch::ones({O}));
  std::string names;
  Tensor p0 = hash_params(*agent, base, hi, lo, names);
  Tensor x = randn({M, O});
  Tensor act = lo + (hi - lo) * randu({M, A}, 0.01f, 0.99f);
  const std::string dims = "\"kind\": 1, \"O\": " + std::to_string(O) + ", \"A\": " + std::to_string(A) +
                           ", \"H\": " + std::to_string(H) + ", \"hi\": " + f2s(hi) + ", \"lo\": " + f2s(lo) +
                           ", \"hash_base\": " + std::to_string(base);
  const std::string ca = pre + "_act";
  begin_case(ca, "{" + dims + ", \"n\": " + std::to_string(M) + ", \"params\": " + names + "}");
  {
    torch::NoGradGuard ng;
    auto [a, lp, ent, v, al, be] = agent->get_action_and_value(x, act, "given");
    dump(ca, "x", x); dump(ca, "action", act);
    dump(ca, "logprob", lp); dump(ca, "entropy", ent); dump(ca, "value", v.view(-1));
    dump(ca, "alpha", al); dump(ca, "beta", be); dump(ca, "action_roundtrip", a);
    auto [am, lpm, entm, vm, alm, bem] = agent->get_action_and_value(x, Tensor(), "mean");
    dump(ca, "mean_action", am); dump(ca, "mean_logprob", lpm);
  }
  end_case();
  const LossCfg c{0.1f, 0.01f, 0.5f, true, true};
  Tensor old_logp, old_v, adv = randn({M}), ret = randn({M});
  {
    torch::NoGradGuard ng;
    auto [a, lp, ent, v, al, be] = agent->get_action_and_value(x, act, "given");
    old_logp = lp + randn({M}, 0.1f);
    old_v = v.view(-1) + randn({M}, 0.1f);
  }
  torch::optim::Adam opt(agent->parameters(), torch::optim::AdamOptions(2.5e-4).eps(1e-5));
  const std::string cu = pre + "_update";
  begin_case(cu, "{" + dims + ", \"M\": " + std::to_string(M) +
                     ", \"clip_coef\": 0.1, \"ent_coef\": 0.01, \"vf_coef\": 0.5, \"clip_vloss\": 1, \"norm_adv\": 1, "
                     "\"max_grad_norm\": 0.5, \"lr\": 0.00025, \"adam_eps\": 1e-05}");
  dump(cu, "x", x); dump(cu, "action", act); dump(cu, "old_logp", old_logp); dump(cu, "adv", adv);
  dump(cu, "ret", ret); dump(cu, "old_v", old_v);
  // the AC trainer's advantage statistics (ac:830-849) over G row shards
  auto dist_stats = [&](int G) {
    const int64_t Md = M / G;
    Tensor amean = torch::zeros({});
    for (int r = 0; r < G; ++r) amean = amean + adv.slice(0, r * Md, (r + 1) * Md).mean();
    amean = amean / (float)G;  // ncclAvg
    Tensor ssum = torch::zeros({});
    for (int r = 0; r < G; ++r) ssum = ssum + torch::sum(torch::square(adv.slice(0, r * Md, (r + 1) * Md) - amean));
    Tensor astd = torch::sqrt(ssum / static_cast<float>(G * Md - 1));
    return std::make_pair(amean, astd);
  };
  {  // G = 2: per-rank losses with the distributed statistics, gradients averaged (ac:877-885)
    auto [amean, astd] = dist_stats(2);
    const int64_t Md = M / 2;
    Tensor gsum;
    for (int r = 0; r < 2; ++r) {
      auto sl = [&](const Tensor& t) { return t.slice(0, r * Md, (r + 1) * Md); };
      auto [a, lp, ent, v, al, be] = agent->get_action_and_value(sl(x), sl(act), "given");
      auto [loss, st] = ppo_loss(lp, ent, v, sl(old_logp), sl(adv), sl(ret), sl(old_v), c, &amean, &astd);
      opt.zero_grad();
      loss.backward();
      Tensor g = flat_grads(*agent);
      gsum = gsum.defined() ? gsum + g : g;
    }
    dump(cu, "grad_dist2_avg", gsum / 2.0f);
    dump(cu, "dist2_adv_stats", torch::stack({amean, astd}));
  }
  auto [amean1, astd1] = dist_stats(1);
  for (int s = 1; s <= 3; ++s) {  // world_size = 1 form of ac:830-888
    auto [a, lp, ent, v, al, be] = agent->get_action_and_value(x, act, "given");
    auto [loss, st] = ppo_loss(lp, ent, v, old_logp, adv, ret, old_v, c, &amean1, &astd1);
    opt.zero_grad();
    loss.backward();
    if (s == 1) { dump(cu, "grad_raw", flat_grads(*agent)); dump(cu, "stats", torch::tensor(st)); }
    const double tn = torch::nn::utils::clip_grad_norm_(agent->parameters(), 0.5);
    if (s == 1) dump(cu, "total_norm", torch::tensor({(float)tn}));
    opt.step();
    if (s == 1) dump(cu, "params_step1", flat_params(*agent));
  }
  dump(cu, "params_step3", flat_params(*agent));
  end_case();
}

// The PPO env wrapper chain of ppo:41-49 (RecordEpisodeStatistics -> NormalizeObservation(kFloat32)
// -> TransformObservation(clamp +-10) -> NormalizeReward(gamma) -> TransformReward(clamp +-10)),
// replayed with the LibTorch calls of stateful_observation.h:56-84 / stateful_reward.h:55-91 over a
// scripted env (the reference headers include gym.h, which needs boost, absent here).
// Scripted env: call c (reset or step) returns obs[i] = U(stream 30, c*O + i) on [i - 2, i + 3),
// step reward U(stream 31, c) on [-1, 4), termination when c % 29 == 28, truncation when c % 61 == 60.
struct WrapChain {
  int O;
  int c = 0;
  float ep_ret = 0.0f;
  int ep_len = 0;
  Tensor om, ov;         // NormalizeObservation mean_ / var_ (kFloat32)
  float ocount = 1e-4f;  // count_ = epsilon
  const float oeps = 1e-4f;
  float rmean = 0.0f, rvar = 1.0f, racc = 0.0f, rcount = 1e-8f;
  const float reps = 1e-8f, gamma = 0.99f;
  explicit WrapChain(int O_) : O(O_) { om = torch::zeros({O}, torch::kFloat32); ov = torch::ones({O}, torch::kFloat32); }
  Tensor raw_obs() {
    Tensor o = torch::empty({O}, torch::kFloat32);
    float* p = o.data_ptr<float>();
    for (int i = 0; i < O; ++i) {
      const float lo = (float)i - 2.0f, hi = (float)i + 3.0f;
      p[i] = lo + (hi - lo) * hu01(30, (uint32_t)(c * O + i));
    }
    return o;
  }
  Tensor obs_wrappers(const Tensor& x) {  // NormalizeObservation::observation + clamp
    torch::NoGradGuard ng;
    {
      const Tensor batch_mean = x;
      const Tensor batch_var = torch::zeros_like(x);
      constexpr float batch_count = 1.0f;
      const Tensor delta = x - om;
      const float tot_count = ocount + batch_count;
      const Tensor new_mean = om + delta * batch_count / tot_count;
      const Tensor m_a = ov * ocount;
      const Tensor m_b = batch_var * batch_count;
      const Tensor M2 = m_a + m_b + (delta * delta) * ocount * batch_count / tot_count;
      const Tensor new_var = M2 / tot_count;
      ocount = tot_count;
      om = new_mean;
      ov = new_var;
      (void)batch_mean;
    }
    Tensor y = (x - om) / torch::sqrt(ov + oeps);
    return torch::clamp(y, -10.0f, 10.0f);
  }
  Tensor reset() {
    Tensor o = raw_obs();
    ++c;
    ep_ret = 0.0f;
    ep_len = 0;
    return obs_wrappers(o);
  }
  // -> obs, reward, term, trunc, info_ret, info_len
  std::tuple<Tensor, float, bool, bool, float, int> step() {
    Tensor o = raw_obs();
    const float r = -1.0f + 5.0f * hu01(31, (uint32_t)c);
    const bool te = (c % 29) == 28, tr = (c % 61) == 60;
    ++c;
    ep_ret += r;
    ep_len += 1;
    float ir = 0.0f;
    int il = 0;
    if (te || tr) { ir = ep_ret; il = ep_len; }
    Tensor oo = obs_wrappers(o);
    racc = racc * gamma * (1.0f - static_cast<float>(te)) + r;
    {
      constexpr float batch_var = 0.0f;
      constexpr float batch_count = 1.0f;
      const float delta = racc - rmean;
      const float tot_count = rcount + batch_count;
      const float new_mean = rmean + delta * batch_count / tot_count;
      const float m_a = rvar * rcount;
      constexpr float m_b = batch_var * batch_count;
      const float M2 = m_a + m_b + (delta * delta) * rcount * batch_count / tot_count;
      rcount = tot_count;
      rmean = new_mean;
      rvar = M2 / tot_count;
    }
    const float rn = std::clamp(r / std::sqrt(rvar + reps), -10.0f, 10.0f);
    return {oo, rn, te, tr, ir, il};
  }
};


// The PPO trainer's per-env wrapper chain (ppo:41-49) over E envs at once for the end-to-end
// replay: NormalizeObservation's LibTorch ops of stateful_observation.h:64-84 applied row-wise to the
// [E, O] observations (one mean_ / var_ / count_ per env: count_ is an [E, 1] column, every other op
// elementwise, so each element sees exactly the per-env operations), the clamp, and
// NormalizeReward's float arithmetic (stateful_reward.h:55-91, std::sqrt) per env.
struct VecWrap {
  int E, O;
  Tensor om, ov, oc;  // [E, O], [E, O], [E, 1]
  std::vector<float> rmean, rvar, racc, rcount;
  const float gamma = 0.99f;
  VecWrap(int E_, int O_) : E(E_), O(O_), rmean(E_, 0.0f), rvar(E_, 1.0f), racc(E_, 0.0f), rcount(E_, 1e-8f) {
    om = torch::zeros({E, O}, torch::kFloat32);
    ov = torch::ones({E, O}, torch::kFloat32);
    oc = torch::full({E, 1}, 1e-4f, torch::kFloat32);
  }
  Tensor obs(const Tensor& x) {
    torch::NoGradGuard ng;
    constexpr float batch_count = 1.0f;
    const Tensor batch_var = torch::zeros_like(x);
    const Tensor delta = x - om;
    const Tensor tot_count = oc + batch_count;
    const Tensor new_mean = om + delta * batch_count / tot_count;
    const Tensor m_a = ov * oc;
    const Tensor m_b = batch_var * batch_count;
    const Tensor M2 = m_a + m_b + (delta * delta) * oc * batch_count / tot_count;
    ov = M2 / tot_count;
    om = new_mean;
    oc = tot_count;
    return torch::clamp((x - om) / torch::sqrt(ov + 1e-4f), -10.0f, 10.0f);
  }
  float reward(int e, float r, float te) {
    racc[e] = racc[e] * gamma * (1.0f - te) + r;
    constexpr float batch_count = 1.0f;
    const float delta = racc[e] - rmean[e];
    const float tot_count = rcount[e] + batch_count;
    const float new_mean = rmean[e] + delta * batch_count / tot_count;
    const float m_a = rvar[e] * rcount[e];
    constexpr float m_b = 0.0f * batch_count;
    const float M2 = m_a + m_b + (delta * delta) * rcount[e] * batch_count / tot_count;
    rcount[e] = tot_count;
    rmean[e] = new_mean;
    rvar[e] = M2 / tot_count;
    return std::clamp(r / std::sqrt(rvar[e] + 1e-8f), -10.0f, 10.0f);
  }
};

// ---------------------------------------------------------------------------------------------
// End-to-end replay (SURVEY §8c "end-to-end run fixture"; north_star: episodic returns on identical
// seeds): NIT iterations of the trainer loop -- lr anneal (ppo:379-384 / ac:634-639), rollout
// (ppo:387-434), GAE, EP x MB minibatch updates with clip_grad_norm_ + Adam (ppo:489-540 /
// ac:803-888) -- with the reference's LibTorch arithmetic, on the synthetic device env's dynamics
// (oracle env, bit-identical to the device env) and the build's RNG contract injected: the
// Normal noise / Beta samples of the Philox counters and the Feistel minibatch permutations
// (LibTorch's own generators cannot be reproduced on the GPU). Records per-iteration loss
// statistics, finished-episode returns and the final parameters.
// ---------------------------------------------------------------------------------------------
template <typename AgentT>
static void e2e_case(const std::string& cname, AgentT& agent, int kind, int E, int T, int MB, int EP, int NIT,
                     float lr0, const LossCfg& c, uint32_t base, bool wrappers = false, bool teacher = false) {
  const int O = 17, A = 6;
  std::string names;
  hash_params(*agent, base, 1.0f, -1.0f, names);
  const uint64_t seed = 1;
  torch::optim::Adam opt(agent->parameters(), torch::optim::AdamOptions(lr0).eps(1e-5));
  // env
  std::vector<float> q((size_t)E * O);
  std::vector<int> et(E), ar(E), elen(E);
  std::vector<uint32_t> rs(E), rc(E);
  std::vector<float> eret(E);
  orc_env_state env{E, O, A, q.data(), et.data(), ar.data(), rs.data(), rc.data(), eret.data(), elen.data()};
  Tensor next_obs = torch::empty({E, O});
  orc_env_reset(&env, (int)seed, next_obs.data_ptr<float>());
  std::unique_ptr<VecWrap> wrap;
  if (wrappers) {
    wrap = std::make_unique<VecWrap>(E, O);
    next_obs = wrap->obs(next_obs).contiguous();
  }
  Tensor next_done = torch::zeros({E});
  const long B = (long)E * T, M = B / MB;
  std::vector<float> stats;   // per iteration: pg, v, ent, old_kl, kl (last minibatch), clipfrac (mean), ret_sum, n_ep
  // teacher forcing (verdict r04 item 1): the state every iteration starts from (parameters and Adam
  // moments for it >= 1), the rollout it collects, and its last minibatch's pre-clip gradient and
  // total norm, so the GPU trainer can run each iteration from the replay's own state
  std::vector<Tensor> tf_p, tf_m, tf_v, tf_obs, tf_act, tf_lp, tf_rew, tf_done, tf_val, tf_nv, tf_nd, tf_grad;
  std::vector<float> tf_gn;
  for (int it = 0; it < NIT; ++it) {
    if (teacher && it > 0) {
      tf_p.push_back(flat_params(*agent));
      tf_m.push_back(flat_state(opt, false));
      tf_v.push_back(flat_state(opt, true));
    }
    const float frac = 1.0f - static_cast<float>(it) / static_cast<float>(NIT);
    const float lrnow = frac * lr0;
    static_cast<torch::optim::AdamOptions&>(opt.param_groups()[0].options()).set_lr(lrnow);
    Tensor obs = torch::zeros({T, E, O}), actions = torch::zeros({T, E, A}), logprobs = torch::zeros({T, E});
    Tensor rewards = torch::zeros({T, E}), dones = torch::zeros({T, E}), values = torch::zeros({T, E});
    double ret_sum = 0.0, n_ep = 0.0;
    for (int t = 0; t < T; ++t) {
      torch::NoGradGuard ng;
      obs.index_put_({t}, next_obs);
      dones.index_put_({t}, next_done);
      const long step = (long)it * T + t;
      Tensor act, lp, v;
      if constexpr (std::is_same_v<AgentT, PPOAgent>) {
        const Tensor mu = agent->actor_mean->forward(next_obs);
        const Tensor sd = torch::exp(agent->actor_logstd.expand_as(mu));
        Tensor z = torch::empty({E, A});
        for (int e = 0; e < E; ++e) orc_normal_noise(seed, 0, e, step, A, z.data_ptr<float>() + (long)e * A);
        act = mu + z * sd;  // Normal::sample = mean + std * eps (rl_utils.h:34-37)
        const Normal probs(mu, sd);
        lp = probs.log_prob(act).sum(1);
        v = agent->critic->forward(next_obs).view(-1);
      } else {
        Tensor xn = (next_obs - agent->mean_) / agent->std_;
        Tensor feat = agent->actor_encoder->forward(xn);
        Tensor al = nn::functional::softplus(agent->dist_alpha->forward(feat)) + 1.0f;
        Tensor be = nn::functional::softplus(agent->dist_beta->forward(feat)) + 1.0f;
        Tensor s01 = torch::empty({E, A});
        for (int e = 0; e < E; ++e)
          for (int a = 0; a < A; ++a)
            s01.data_ptr<float>()[e * A + a] = orc_beta_sample01(al[e][a].item<float>(), be[e][a].item<float>(), seed, 0,
                                                                e, step, a);
        const Beta probs(al, be);
        lp = probs.log_prob(s01).sum(1);
        act = agent->unscale_action(s01);
        v = agent->critic->forward(xn).view(-1);
      }
      actions.index_put_({t}, act);
      logprobs.index_put_({t}, lp);
      values.index_put_({t}, v);
      Tensor ob = torch::empty({E, O}), r = torch::empty({E}), te = torch::empty({E}), tr = torch::empty({E});
      Tensor ir = torch::empty({E});
      std::vector<int> il(E);
      Tensor ac = act.contiguous();
      orc_env_step(&env, ac.data_ptr<float>(), -1.0f, 1.0f, ob.data_ptr<float>(), r.data_ptr<float>(),
                   te.data_ptr<float>(), tr.data_ptr<float>(), ir.data_ptr<float>(), il.data());
      for (int e = 0; e < E; ++e)
        if (il[e] > 0) { ret_sum += ir.data_ptr<float>()[e]; n_ep += 1.0; }
      if (wrap) {  // gym.h:141-149: an env whose previous step ended is reset now (reward 0, not normalised)
        ob = wrap->obs(ob).contiguous();
        for (int e = 0; e < E; ++e)
          if (next_done.data_ptr<float>()[e] == 0.0f)
            r.data_ptr<float>()[e] = wrap->reward(e, r.data_ptr<float>()[e], te.data_ptr<float>()[e]);
      }
      rewards.index_put_({t}, r);
      next_obs = ob;
      next_done = torch::maximum(te, tr);
    }
    Tensor next_value;
    {
      torch::NoGradGuard ng;
      if constexpr (std::is_same_v<AgentT, PPOAgent>) next_value = agent->get_value(next_obs).flatten();
      else next_value = agent->critic->forward((next_obs - agent->mean_) / agent->std_).flatten();
    }
    auto [adv, ret] = gae_ref(rewards, values, dones, next_value, next_done, 0.99f, 0.95f);
    if (teacher) {
      tf_obs.push_back(obs.clone()); tf_act.push_back(actions.clone()); tf_lp.push_back(logprobs.clone());
      tf_rew.push_back(rewards.clone()); tf_done.push_back(dones.clone()); tf_val.push_back(values.clone());
      tf_nv.push_back(next_value.clone()); tf_nd.push_back(next_done.clone());
    }
    if (const char* dbg = std::getenv("E2E_DEBUG_DIR")) {  // diagnostics: the rollout of every iteration
      const std::string pre = std::string(dbg) + "/" + cname + "_it" + std::to_string(it);
      for (auto& [nm, tt] : std::vector<std::pair<std::string, Tensor>>{{"actions", actions}, {"logprobs", logprobs},
                                                                         {"values", values}, {"obs", obs}}) {
        Tensor c2 = tt.contiguous();
        std::ofstream(pre + "_" + nm + ".f32", std::ios::binary)
            .write(reinterpret_cast<const char*>(c2.data_ptr<float>()), c2.numel() * 4);
      }
    }
    Tensor b_obs = obs.reshape({B, O}), b_act = actions.reshape({B, A}), b_lp = logprobs.reshape({B});
    Tensor b_adv = adv.reshape({B}), b_ret = ret.reshape({B}), b_val = values.reshape({B});
    std::vector<float> st_last;
    double cf_sum = 0.0;
    for (int ep = 0; ep < EP; ++ep) {
      std::vector<int64_t> perm(B);
      orc_perm(B, seed, 0, (long)it * EP + ep, perm.data());
      Tensor b_inds = torch::from_blob(perm.data(), {B}, torch::kInt64).clone();
      for (long start = 0; start < B; start += M) {
        Tensor mb = b_inds.index({torch::indexing::Slice(start, start + M)});
        Tensor lp, ent, v;
        if constexpr (std::is_same_v<AgentT, PPOAgent>) {
          auto [a_, lp_, ent_, v_, mu_] = agent->get_action_and_value(b_obs.index({mb}), b_act.index({mb}));
          lp = lp_; ent = ent_; v = v_;
        } else {
          auto [a_, lp_, ent_, v_, al_, be_] = agent->get_action_and_value(b_obs.index({mb}), b_act.index({mb}), "given");
          lp = lp_; ent = ent_; v = v_;
        }
        Tensor madv = b_adv.index({mb});
        std::tuple<Tensor, std::vector<float>> res;
        if (kind == 1) {  // ac:830-849 with world_size = 1
          Tensor amean, astd;
          {
            torch::NoGradGuard ng;
            amean = madv.mean();
            astd = torch::sqrt(torch::sum(torch::square(madv - amean)) / static_cast<float>(M - 1));
          }
          res = ppo_loss(lp, ent, v, b_lp.index({mb}), madv, b_ret.index({mb}), b_val.index({mb}), c, &amean, &astd);
        } else {
          res = ppo_loss(lp, ent, v, b_lp.index({mb}), madv, b_ret.index({mb}), b_val.index({mb}), c, nullptr, nullptr);
        }
        auto& [loss, st] = res;
        opt.zero_grad();
        loss.backward();
        const bool last_mb = ep == EP - 1 && start + M >= B;
        if (teacher && last_mb && (it & 1)) tf_grad.push_back(flat_grads(*agent));
        const double tn = torch::nn::utils::clip_grad_norm_(agent->parameters(), 0.5);
        if (teacher && last_mb) tf_gn.push_back((float)tn);
        opt.step();
        st_last = st;
        cf_sum += st[5];
      }
    }
    stats.insert(stats.end(), {st_last[0], st_last[1], st_last[2], st_last[3], st_last[4],
                               (float)(cf_sum / (EP * (B / M))), (float)ret_sum, (float)n_ep});
  }
  begin_case(cname, "{\"kind\": " + std::to_string(kind) + ", \"wrappers\": " + (wrappers ? "true" : "false") +
                        ", \"E\": " + std::to_string(E) + ", \"T\": " +
                        std::to_string(T) + ", \"MB\": " + std::to_string(MB) + ", \"EP\": " + std::to_string(EP) +
                        ", \"iterations\": " + std::to_string(NIT) + ", \"lr\": " + f2s(lr0) + ", \"clip_coef\": " +
                        f2s(c.clip_coef) + ", \"ent_coef\": " + f2s(c.ent_coef) + ", \"hash_base\": " +
                        std::to_string(base) + ", \"seed\": 1, \"stats\": [\"pg_loss\", \"v_loss\", \"entropy\", "
                        "\"old_approx_kl\", \"approx_kl\", \"clipfrac_mean\", \"episodic_return_sum\", \"episodes\"]}");
  dump(cname, "stats", torch::tensor(stats).view({NIT, 8}));
  dump(cname, "params_final", flat_params(*agent));
  if (teacher) {  // tf_* [it] = iteration it (tf_params / tf_adam_*: iterations 1.., tf_grad: odd iterations)
    dump(cname, "tf_params", torch::stack(tf_p)); dump(cname, "tf_adam_m", torch::stack(tf_m));
    dump(cname, "tf_adam_v", torch::stack(tf_v));
    dump(cname, "tf_obs", torch::stack(tf_obs)); dump(cname, "tf_actions", torch::stack(tf_act));
    dump(cname, "tf_logprobs", torch::stack(tf_lp)); dump(cname, "tf_rewards", torch::stack(tf_rew));
    dump(cname, "tf_dones", torch::stack(tf_done)); dump(cname, "tf_values", torch::stack(tf_val));
    dump(cname, "tf_next_value", torch::stack(tf_nv)); dump(cname, "tf_next_done", torch::stack(tf_nd));
    dump(cname, "tf_grad_last_mb", torch::stack(tf_grad)); dump(cname, "tf_grad_norm", torch::tensor(tf_gn));
  }
  end_case();
}

static void e2e_cases() {
  const int E = 8, T = 128, MB = 4, EP = 4, NIT = 8;  // 1024 steps per env: every env finishes an episode
  {
    PPOAgent agent(17, 6, 64);
    e2e_case("e2e_ppo", agent, 0, E, T, MB, EP, NIT, 3e-4f, LossCfg{0.2f, 0.0f, 0.5f, true, true}, 3300);
  }
  {  // the PPO trainer as the reference runs it: every env behind the ppo:41-49 wrapper chain
    PPOAgent agent(17, 6, 64);
    e2e_case("e2e_ppo_wrapped", agent, 0, E, T, MB, EP, NIT, 3e-4f, LossCfg{0.2f, 0.0f, 0.5f, true, true}, 3500, true);
  }
  {
    ACAgent agent(17, 6, 256, 1.0f, -1.0f, torch::zeros({17}), torch::ones({17}));
    e2e_case("e2e_ac", agent, 1, E, T, MB, EP, NIT, 2.5e-4f, LossCfg{0.1f, 0.01f, 0.5f, true, true}, 3400, false, true);
  }
}

static void width_cases() {
  ac_width_case("ac256", 17, 6, 256, 256, 3000, 1.0f, -1.0f);
  ac_width_case("ant256", 105, 8, 256, 256, 3100, 1.0f, -1.0f);
  ppo_width_case("hum376", 376, 17, 64, 256, 3200);

  {  // GAE at cfg2's T = 2048 (E = 1024): inputs from hash streams 11-15, outputs as column hashes
    const int T = 2048, E = 1024;
    Tensor rewards = hunif(11, {T, E}, -1.0f, 1.0f), values = hunif(12, {T, E}, -1.0f, 1.0f);
    Tensor dones = (hunif(13, {T, E}, 0.0f, 1.0f) < 0.002f).to(torch::kFloat32);
    dones.index_put_({0}, 1.0f);
    dones.index_put_({T - 1, torch::indexing::Slice(0, E / 2)}, 1.0f);
    Tensor next_value = hunif(14, {E}, -1.0f, 1.0f);
    Tensor next_done = (hunif(15, {E}, 0.0f, 1.0f) < 0.5f).to(torch::kFloat32);
    auto [adv, ret] = gae_ref(rewards, values, dones, next_value, next_done, 0.99f, 0.95f);
    begin_case("gae_long", "{\"T\": 2048, \"E\": 1024, \"gamma\": 0.99, \"gae_lambda\": 0.95, \"streams\": "
                           "[11, 12, 13, 14, 15], \"done_p\": 0.002}");
    dump("gae_long", "adv_fnv", column_fnv(adv)); dump("gae_long", "ret_fnv", column_fnv(ret));
    dump("gae_long", "adv_cols8", adv.slice(1, 0, 8)); dump("gae_long", "ret_cols8", ret.slice(1, 0, 8));
    end_case();
  }
  for (int T : {1, 7, 33}) {  // ragged T (k_gae loads 32-step chunks), E = 37
    const int E = 37;
    Tensor rewards = randn({T, E}), values = randn({T, E});
    Tensor dones = (randu({T, E}, 0.0f, 1.0f) < 0.1f).to(torch::kFloat32);
    Tensor next_value = randn({E});
    Tensor next_done = (randu({E}, 0.0f, 1.0f) < 0.5f).to(torch::kFloat32);
    auto [adv, ret] = gae_ref(rewards, values, dones, next_value, next_done, 0.99f, 0.95f);
    const std::string cn = "gae_t" + std::to_string(T);
    begin_case(cn, "{\"T\": " + std::to_string(T) + ", \"E\": 37, \"gamma\": 0.99, \"gae_lambda\": 0.95}");
    dump(cn, "rewards", rewards); dump(cn, "values", values); dump(cn, "dones", dones);
    dump(cn, "next_value", next_value); dump(cn, "next_done", next_done);
    dump(cn, "advantages", adv); dump(cn, "returns", ret);
    end_case();
  }
  {  // wrapper chain over the scripted env, one env with next-step autoreset (gym.h:141-159) and a
     // plain reset(3) at t = 120
    const int O = 5, T = 200;
    WrapChain w(O);
    std::vector<float> obs, rew, te, tr, ir, il;
    auto put = [&](const Tensor& o) { for (int i = 0; i < O; ++i) obs.push_back(o.data_ptr<float>()[i]); };
    put(w.reset());
    bool autoreset = false;
    for (int t = 0; t < T; ++t) {
      if (t == 120) { put(w.reset()); rew.push_back(0.0f); te.push_back(0); tr.push_back(0); ir.push_back(0); il.push_back(0); autoreset = false; continue; }
      if (autoreset) {
        put(w.reset());
        rew.push_back(0.0f); te.push_back(0); tr.push_back(0); ir.push_back(0); il.push_back(0);
        autoreset = false;
        continue;
      }
      auto [o, r, a, b, iret, ilen] = w.step();
      put(o); rew.push_back(r); te.push_back(a); tr.push_back(b); ir.push_back(iret); il.push_back((float)ilen);
      autoreset = a || b;
    }
    begin_case("wrappers", "{\"O\": 5, \"T\": 200, \"gamma\": 0.99, \"reset_at\": 120, \"obs_stream\": 30, "
                           "\"reward_stream\": 31, \"term_mod\": 29, \"trunc_mod\": 61}");
    dump("wrappers", "obs", torch::tensor(obs).view({T + 1, O})); dump("wrappers", "reward", torch::tensor(rew));
    dump("wrappers", "term", torch::tensor(te)); dump("wrappers", "trunc", torch::tensor(tr));
    dump("wrappers", "info_ret", torch::tensor(ir)); dump("wrappers", "info_len", torch::tensor(il));
    dump("wrappers", "obs_mean_final", w.om); dump("wrappers", "obs_var_final", w.ov);
    end_case();
  }
}

// ---------------------------------------------------------------------------------------------
// --bench: times the reference's CPU arithmetic for one AC-PPO iteration on a bounded sample.
// The reference runs with one intra-op thread (ac_ppo_continuous_action.cpp:288-289) and collects
// with E/G host threads, each calling the shared agent with batch 1 on its own generator
// (ac:575-618, :641-698). So:
//   * rollout inference: `threads` host threads, each making n_act batch-1
//     Agent::get_action_and_value calls ("sample", ac:655) on the same module under NoGradGuard;
//     the per-call cost is wall time / (threads * n_act) (and the 1-thread cost on its own)
//   * one full optimizer step on a minibatch of M rows (ac:815-888: forward, loss, backward,
//     clip_grad_norm_, Adam) -- single-threaded, as the reference's update is
//   * the GAE loop over [T, E] (ac:759-779)
// and prints a JSON line; bench.py extrapolates it to one iteration (E*T acts, EP*MB steps).
// --bench-ppo: the same for ppo_continuous_action (ppo:387-542; cfg1: E=1, T=2048, 32 x 10
// minibatches of 64 rows, HalfCheetah O=17 / A=6, one thread by design ppo:187).
// ---------------------------------------------------------------------------------------------
static double time_ac_acts(ACAgent& agent, int O, int n_act, int threads) {
  using clk = std::chrono::steady_clock;
  std::vector<std::thread> pool;
  std::vector<Tensor> xs;
  for (int t = 0; t < threads; ++t) xs.push_back(randn({1, O}));
  auto t0 = clk::now();
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&, t] {
      torch::NoGradGuard ng;
      auto gen = at::make_generator<at::CPUGeneratorImpl>(t);
      for (int i = 0; i < n_act; ++i) {
        Tensor xx = (xs[t] - agent->mean_) / agent->std_;
        Tensor feat = agent->actor_encoder->forward(xx);
        Tensor al = nn::functional::softplus(agent->dist_alpha->forward(feat)) + 1.0f;
        Tensor be = nn::functional::softplus(agent->dist_beta->forward(feat)) + 1.0f;
        const Beta probs(al, be);
        Tensor a = probs.sample(gen);
        Tensor lp = probs.log_prob(a).sum(1);
        a = agent->unscale_action(a);
        Tensor ent = probs.entropy().sum(1);
        Tensor v = agent->critic->forward(xx);
        (void)lp; (void)ent; (void)v;
      }
    });
  for (auto& th : pool) th.join();
  return std::chrono::duration<double>(clk::now() - t0).count() / ((double)n_act * threads);
}

static double time_gae(int T, int E) {
  using clk = std::chrono::steady_clock;
  Tensor rewards = randn({T, E}), values = randn({T, E}), dones = torch::zeros({T, E});
  Tensor next_value = randn({E}), next_done = torch::zeros({E});
  auto t0 = clk::now();
  auto r = gae_ref(rewards, values, dones, next_value, next_done, 0.99f, 0.95f);
  (void)r;
  return std::chrono::duration<double>(clk::now() - t0).count();
}

static int bench_main(int E, int T, int MB, int EP, int n_act, int threads) {
  using clk = std::chrono::steady_clock;
  const int O = 17, A = 6, H = 256;
  const long B = (long)E * T, M = B / MB;
  ACAgent agent(O, A, H, 1.0f, -1.0f, torch::zeros({O}), torch::ones({O}));
  std::string names;
  set_params(*agent, names);
  torch::optim::Adam opt(agent->parameters(), torch::optim::AdamOptions(2.5e-4).eps(1e-5));
  const double t_act1 = time_ac_acts(agent, O, n_act / 4 > 0 ? n_act / 4 : 1, 1);
  const double t_act = threads > 1 ? time_ac_acts(agent, O, n_act, threads) : t_act1;
  // one optimizer step on M rows
  Tensor bx = randn({M, O}), ba = randu({M, A}, -0.99f, 0.99f), blp = randn({M}, 0.1f) - 5.0f;
  Tensor badv = randn({M}), bret = randn({M}), bval = randn({M});
  LossCfg c{0.1f, 0.01f, 0.5f, true, true};
  double t_opt;
  {
    auto t0 = clk::now();
    auto [a, lp, ent, v, al, be] = agent->get_action_and_value(bx, ba, "given");
    Tensor amean = badv.mean();
    Tensor astd = torch::sqrt(torch::sum(torch::square(badv - amean)) / static_cast<float>(M - 1));
    auto [loss, st] = ppo_loss(lp, ent, v, blp, badv, bret, bval, c, &amean, &astd);
    opt.zero_grad();
    loss.backward();
    torch::nn::utils::clip_grad_norm_(agent->parameters(), 0.5);
    opt.step();
    t_opt = std::chrono::duration<double>(clk::now() - t0).count();
  }
  const double t_gae = time_gae(T, E);
  const double t_iter = t_act * (double)B + t_opt * (double)(EP * MB) + t_gae;
  const double t_iter1 = t_act1 * (double)B + t_opt * (double)(EP * MB) + t_gae;
  std::printf("{\"t_act_batch1_s\": %.9g, \"t_act_batch1_1thread_s\": %.9g, \"t_opt_step_s\": %.9g, \"t_gae_s\": %.9g, "
              "\"n_act\": %d, \"M\": %ld, \"t_iter_s\": %.9g, \"sps\": %.9g, \"threads\": %d, \"sps_1thread\": %.9g}\n",
              t_act, t_act1, t_opt, t_gae, n_act, M, t_iter, (double)B / t_iter, threads, (double)B / t_iter1);
  return 0;
}

static int bench_ppo_main(int E, int T, int MB, int EP, int n_act) {
  using clk = std::chrono::steady_clock;
  const int O = 17, A = 6, H = 64;
  const long B = (long)E * T, M = B / MB;
  PPOAgent agent(O, A, H);
  std::string names;
  set_params(*agent, names);
  torch::optim::Adam opt(agent->parameters(), torch::optim::AdamOptions(3e-4).eps(1e-5));
  Tensor x1 = randn({E, O});
  double t_act;
  {
    torch::NoGradGuard ng;
    auto t0 = clk::now();
    for (int i = 0; i < n_act; ++i) {  // ppo:395 with the sampling of ppo:150-151 (Normal, at::normal)
      const Tensor mu = agent->actor_mean->forward(x1);
      const Tensor sd = torch::exp(agent->actor_logstd.expand_as(mu));
      const Normal probs(mu, sd);
      Tensor a = probs.sample(std::nullopt);
      Tensor lp = probs.log_prob(a).sum(1), ent = probs.entropy().sum(1), v = agent->critic->forward(x1);
      (void)lp; (void)ent; (void)v;
    }
    t_act = std::chrono::duration<double>(clk::now() - t0).count() / n_act;
  }
  Tensor bx = randn({M, O}), ba = randn({M, A}, 0.5f), blp = randn({M}, 0.1f) - 5.0f;
  Tensor badv = randn({M}), bret = randn({M}), bval = randn({M});
  const LossCfg c{0.2f, 0.0f, 0.5f, true, true};
  const int n_opt = 64;
  auto t0 = clk::now();
  for (int i = 0; i < n_opt; ++i) {  // ppo:494-540
    auto [a, lp, ent, v, mu] = agent->get_action_and_value(bx, ba);
    auto [loss, st] = ppo_loss(lp, ent, v, blp, badv, bret, bval, c, nullptr, nullptr);
    opt.zero_grad();
    loss.backward();
    torch::nn::utils::clip_grad_norm_(agent->parameters(), 0.5);
    opt.step();
  }
  const double t_opt = std::chrono::duration<double>(clk::now() - t0).count() / n_opt;
  const double t_gae = time_gae(T, E);
  const double t_iter = t_act * (double)T + t_opt * (double)(EP * MB) + t_gae;
  std::printf("{\"t_act_s\": %.9g, \"t_opt_step_s\": %.9g, \"t_gae_s\": %.9g, \"n_act\": %d, \"M\": %ld, "
              "\"t_iter_s\": %.9g, \"sps\": %.9g, \"threads\": 1}\n",
              t_act, t_opt, t_gae, n_act, M, t_iter, (double)B / t_iter);
  return 0;
}

int main(int argc, char** argv) {
  torch::set_num_threads(1);
  if (argc > 1 && std::string(argv[1]) == "--bench") {
    // --bench E T MB EP n_act threads
    int E = argc > 2 ? std::atoi(argv[2]) : 4096, T = argc > 3 ? std::atoi(argv[3]) : 128;
    int MB = argc > 4 ? std::atoi(argv[4]) : 4, EP = argc > 5 ? std::atoi(argv[5]) : 4;
    int n_act = argc > 6 ? std::atoi(argv[6]) : 2000, threads = argc > 7 ? std::atoi(argv[7]) : 1;
    return bench_main(E, T, MB, EP, n_act, threads < 1 ? 1 : threads);
  }
  if (argc > 1 && std::string(argv[1]) == "--bench-ppo") {
    // --bench-ppo E T MB EP n_act   (cfg1 defaults: 1 2048 32 10)
    int E = argc > 2 ? std::atoi(argv[2]) : 1, T = argc > 3 ? std::atoi(argv[3]) : 2048;
    int MB = argc > 4 ? std::atoi(argv[4]) : 32, EP = argc > 5 ? std::atoi(argv[5]) : 10;
    int n_act = argc > 6 ? std::atoi(argv[6]) : 2048;
    return bench_ppo_main(E, T, MB, EP, n_act);
  }
  if (argc > 1 && std::string(argv[1]) == "--pth-load") {
    // --pth-load <ppo|ac> O A H <model.pth> <optimizer.pth> <out_dir>: torch::load both archives
    // into a fresh agent / Adam (ac_ppo_carla.cpp:236-251) and dump what LibTorch read
    if (argc < 9) { std::fprintf(stderr, "usage: --pth-load <ppo|ac> O A H model optimizer out_dir\n"); return 2; }
    const std::string kind = argv[2];
    const int O = std::atoi(argv[3]), A = std::atoi(argv[4]), H = std::atoi(argv[5]);
    g_out = argv[8];
    std::filesystem::create_directories(g_out);
    g_manifest << "{\n";
    auto run = [&](auto& agent) {
      torch::optim::Adam opt(agent->parameters(), torch::optim::AdamOptions(1e-3));
      torch::load(agent, argv[6]);
      torch::load(opt, argv[7]);
      long step = 0;
      for (auto& p : opt.param_groups()[0].params()) {
        auto it = opt.state().find(p.unsafeGetTensorImpl());
        if (it != opt.state().end()) { step = static_cast<torch::optim::AdamParamState&>(*it->second).step(); break; }
      }
      const auto& o = static_cast<torch::optim::AdamOptions&>(opt.param_groups()[0].options());
      begin_case("loaded", "{\"step\": " + std::to_string(step) + ", \"lr\": " + std::to_string(o.lr()) +
                           ", \"eps\": " + std::to_string(o.eps()) + "}");
      dump("loaded", "params", flat_params(*agent));
      dump("loaded", "adam_m", flat_state(opt, false));
      dump("loaded", "adam_v", flat_state(opt, true));
      end_case();
    };
    if (kind == "ppo") { PPOAgent agent(O, A, H); run(agent); }
    else { ACAgent agent(O, A, H, 1.0f, -1.0f, torch::zeros({O}), torch::ones({O})); run(agent); }
    g_manifest << "\n}\n";
    std::ofstream(g_out + "/manifest.json") << g_manifest.str();
    return 0;
  }
  g_out = argc > 1 ? argv[1] : "tests/golden";
  std::filesystem::create_directories(g_out);
  g_manifest << "{\n";
  const int O = 17, A = 6, H = 64, M = 64;

  // ---- PPO agent: act + update ----------------------------------------------------------
  {
    PPOAgent agent(O, A, H);
    std::string names;
    Tensor p0 = set_params(*agent, names);
    Tensor x = randn({M, O});
    Tensor act = randn({M, A}, 0.8f);
    begin_case("ppo_act", "{\"kind\": 0, \"O\": 17, \"A\": 6, \"H\": 64, \"n\": 64, \"params\": " + names + "}");
    {
      torch::NoGradGuard ng;
      auto [a, lp, ent, v, mu] = agent->get_action_and_value(x, act);
      dump("ppo_act", "params", p0); dump("ppo_act", "x", x); dump("ppo_act", "action", act);
      dump("ppo_act", "logprob", lp); dump("ppo_act", "entropy", ent); dump("ppo_act", "value", v.view(-1));
      dump("ppo_act", "mean", mu);
    }
    end_case();

    LossCfg c{0.2f, 0.01f, 0.5f, true, true};
    Tensor old_logp, adv = randn({M}), ret = randn({M}), old_v;
    {
      torch::NoGradGuard ng;
      auto [a, lp, ent, v, mu] = agent->get_action_and_value(x, act);
      old_logp = lp + randn({M}, 0.15f);
      old_v = v.view(-1) + randn({M}, 0.15f);
    }
    torch::optim::Adam opt(agent->parameters(), torch::optim::AdamOptions(3e-4).eps(1e-5));
    begin_case("ppo_update", "{\"kind\": 0, \"O\": 17, \"A\": 6, \"H\": 64, \"M\": 64, \"clip_coef\": 0.2, "
                             "\"ent_coef\": 0.01, \"vf_coef\": 0.5, \"clip_vloss\": 1, \"norm_adv\": 1, "
                             "\"max_grad_norm\": 0.5, \"lr\": 0.0003, \"adam_eps\": 1e-05}");
    dump("ppo_update", "params", p0); dump("ppo_update", "x", x); dump("ppo_update", "action", act);
    dump("ppo_update", "old_logp", old_logp); dump("ppo_update", "adv", adv); dump("ppo_update", "ret", ret);
    dump("ppo_update", "old_v", old_v);
    for (int s = 1; s <= 3; ++s) {
      auto [a, lp, ent, v, mu] = agent->get_action_and_value(x, act);
      auto [loss, st] = ppo_loss(lp, ent, v, old_logp, adv, ret, old_v, c, nullptr, nullptr);
      opt.zero_grad();
      loss.backward();
      if (s == 1) { dump("ppo_update", "grad_raw", flat_grads(*agent)); dump("ppo_update", "stats", torch::tensor(st)); }
      double tn = torch::nn::utils::clip_grad_norm_(agent->parameters(), 0.5);
      if (s == 1) { dump("ppo_update", "grad_clipped", flat_grads(*agent)); dump("ppo_update", "total_norm", torch::tensor({(float)tn})); }
      opt.step();
      if (s == 1) dump("ppo_update", "params_step1", flat_params(*agent));
    }
    dump("ppo_update", "params_step3", flat_params(*agent));
    dump("ppo_update", "adam_m_step3", flat_state(opt, false));
    dump("ppo_update", "adam_v_step3", flat_state(opt, true));
    end_case();
  }

  // ---- AC agent: act (given + mean) + update + distributed equivalence ---------------------
  {
    Tensor mean = randn({O}, 0.1f), stdv = randu({O}, 0.8f, 1.5f);
    ACAgent agent(O, A, H, 1.0f, -1.0f, mean, stdv);
    std::string names;
    Tensor p0 = set_params(*agent, names);
    Tensor x = randn({M, O});
    Tensor act = randu({M, A}, -0.98f, 0.98f);
    begin_case("ac_act", "{\"kind\": 1, \"O\": 17, \"A\": 6, \"H\": 64, \"n\": 64, \"params\": " + names + "}");
    {
      torch::NoGradGuard ng;
      auto [a, lp, ent, v, al, be] = agent->get_action_and_value(x, act, "given");
      dump("ac_act", "params", p0); dump("ac_act", "x", x); dump("ac_act", "action", act);
      dump("ac_act", "logprob", lp); dump("ac_act", "entropy", ent); dump("ac_act", "value", v.view(-1));
      dump("ac_act", "alpha", al); dump("ac_act", "beta", be); dump("ac_act", "action_roundtrip", a);
      auto [am, lpm, entm, vm, alm, bem] = agent->get_action_and_value(x, Tensor(), "mean");
      dump("ac_act", "mean_action", am); dump("ac_act", "mean_logprob", lpm);
    }
    end_case();

    LossCfg c{0.1f, 0.01f, 0.5f, true, true};
    Tensor old_logp, adv = randn({M}), ret = randn({M}), old_v;
    {
      torch::NoGradGuard ng;
      auto [a, lp, ent, v, al, be] = agent->get_action_and_value(x, act, "given");
      old_logp = lp + randn({M}, 0.1f);
      old_v = v.view(-1) + randn({M}, 0.1f);
    }
    torch::optim::Adam opt(agent->parameters(), torch::optim::AdamOptions(2.5e-4).eps(1e-5));
    begin_case("ac_update", "{\"kind\": 1, \"O\": 17, \"A\": 6, \"H\": 64, \"M\": 64, \"clip_coef\": 0.1, "
                            "\"ent_coef\": 0.01, \"vf_coef\": 0.5, \"clip_vloss\": 1, \"norm_adv\": 1, "
                            "\"max_grad_norm\": 0.5, \"lr\": 0.00025, \"adam_eps\": 1e-05}");
    dump("ac_update", "params", p0); dump("ac_update", "x", x); dump("ac_update", "action", act);
    dump("ac_update", "old_logp", old_logp); dump("ac_update", "adv", adv); dump("ac_update", "ret", ret);
    dump("ac_update", "old_v", old_v);
    // G = 2 equivalence (ac:830-849, :877-885): two row shards, distributed adv stats, avg grads
    {
      Tensor gsum;
      const int G = 2, Md = M / G;
      std::vector<Tensor> means;
      for (int r = 0; r < G; ++r) means.push_back(adv.slice(0, r * Md, (r + 1) * Md).mean());
      Tensor amean = (means[0] + means[1]) / 2.0f;  // ncclAvg
      Tensor ssum = torch::zeros({});
      for (int r = 0; r < G; ++r) ssum = ssum + torch::sum(torch::square(adv.slice(0, r * Md, (r + 1) * Md) - amean));
      Tensor astd = torch::sqrt(ssum / static_cast<float>(G * Md - 1));
      for (int r = 0; r < G; ++r) {
        auto sl = [&](const Tensor& t) { return t.slice(0, r * Md, (r + 1) * Md); };
        auto [a, lp, ent, v, al, be] = agent->get_action_and_value(sl(x), sl(act), "given");
        auto [loss, st] = ppo_loss(lp, ent, v, sl(old_logp), sl(adv), sl(ret), sl(old_v), c, &amean, &astd);
        opt.zero_grad();
        loss.backward();
        Tensor g = flat_grads(*agent);
        gsum = gsum.defined() ? gsum + g : g;
      }
      dump("ac_update", "grad_dist2_avg", gsum / 2.0f);
      dump("ac_update", "dist2_adv_stats", torch::stack({amean, astd}));
    }
    for (int s = 1; s <= 3; ++s) {
      auto [a, lp, ent, v, al, be] = agent->get_action_and_value(x, act, "given");
      auto [loss, st] = ppo_loss(lp, ent, v, old_logp, adv, ret, old_v, c, nullptr, nullptr);
      opt.zero_grad();
      loss.backward();
      if (s == 1) { dump("ac_update", "grad_raw", flat_grads(*agent)); dump("ac_update", "stats", torch::tensor(st)); }
      double tn = torch::nn::utils::clip_grad_norm_(agent->parameters(), 0.5);
      if (s == 1) { dump("ac_update", "grad_clipped", flat_grads(*agent)); dump("ac_update", "total_norm", torch::tensor({(float)tn})); }
      opt.step();
      if (s == 1) dump("ac_update", "params_step1", flat_params(*agent));
    }
    dump("ac_update", "params_step3", flat_params(*agent));
    end_case();
  }

  // ---- GAE (ppo:447-467) -------------------------------------------------------------------
  {
    const int T = 64, E = 16;
    const float gamma = 0.99f, gae_lambda = 0.95f;
    Tensor rewards = randn({T, E}), values = randn({T, E});
    Tensor dones = (randu({T, E}, 0.0f, 1.0f) < 0.05f).to(torch::kFloat32);
    dones.index_put_({0}, 1.0f);
    dones.index_put_({T - 1, torch::indexing::Slice(0, E / 2)}, 1.0f);
    Tensor next_value = randn({E});
    Tensor next_done = (randu({E}, 0.0f, 1.0f) < 0.5f).to(torch::kFloat32);
    Tensor advantages = torch::zeros({T, E});
    Tensor lastgaelam = torch::zeros({E});
    Tensor nextnonterminal, nextvalues;
    for (int t = T - 1; t >= 0; --t) {
      if (t == T - 1) { nextnonterminal = 1.0f - next_done; nextvalues = next_value; }
      else { nextnonterminal = 1.0 - dones.index({t + 1}); nextvalues = values.index({t + 1}); }
      Tensor delta = rewards.index({t}) + gamma * nextvalues * nextnonterminal - values.index({t});
      advantages.index({t}) = delta + gamma * gae_lambda * nextnonterminal * lastgaelam;
      lastgaelam = advantages.index({t});
    }
    Tensor returns = advantages + values;
    begin_case("gae", "{\"T\": 64, \"E\": 16, \"gamma\": 0.99, \"gae_lambda\": 0.95}");
    dump("gae", "rewards", rewards); dump("gae", "values", values); dump("gae", "dones", dones);
    dump("gae", "next_value", next_value); dump("gae", "next_done", next_done);
    dump("gae", "advantages", advantages); dump("gae", "returns", returns);
    end_case();
  }

  // ---- CaRL CNN agent forward (carla_model.h:270-318), SURVEY §8 a23 ----------------------------
  {
    torch::NoGradGuard ng;
    const int N = 3, C = 15, HW = 192, NM = 8, NV = 3, A = 2;
    CarlaAgent agent(C, NM, NV, A, 1.0f, -1.0f, 1.0f);
    // parameters: tensor t (named_parameters order) from stream 1000 + t; weights uniform with
    // He scale sqrt(6 / fan_in), biases uniform in [-0.1, 0.1]; action space [-1, 1]
    std::vector<Tensor> flat;
    std::string names = "[";
    int t = 0;
    for (auto& kv : agent->named_parameters()) {
      Tensor p = kv.value();
      Tensor v;
      if (kv.key() == "action_space_high") v = torch::tensor(1.0f);
      else if (kv.key() == "action_space_low") v = torch::tensor(-1.0f);
      else if (p.dim() >= 2) {
        const float fan_in = (float)(p.numel() / p.size(0));
        const float a = std::sqrt(6.0f / fan_in);
        v = hunif(1000 + t, p.sizes().vec(), -a, a);
      } else v = hunif(1000 + t, p.sizes().vec(), -0.1f, 0.1f);
      p.copy_(v.reshape(p.sizes()));
      flat.push_back(p.detach().reshape({-1}).clone());
      names += std::string(t ? ", " : "") + "[\"" + kv.key() + "\", " + std::to_string(p.numel()) + "]";
      ++t;
    }
    names += "]";
    // inputs: bev bytes = top 8 bits of hbits(1, i); meas, vmeas uniform [-1, 1) (streams 2, 3);
    // given actions uniform [-0.98, 0.98) (stream 4)
    Tensor bev = torch::empty({N, C, HW, HW}, torch::kUInt8);
    uint8_t* bp = bev.data_ptr<uint8_t>();
    for (int64_t i = 0; i < bev.numel(); ++i) bp[i] = (uint8_t)(hbits(1, (uint32_t)i) >> 24);
    Tensor meas = hunif(2, {N, NM}, -1.0f, 1.0f), vmeas = hunif(3, {N, NV}, -1.0f, 1.0f);
    Tensor act = hunif(4, {N, A}, -0.98f, 0.98f);
    begin_case("carla_act", "{\"N\": 3, \"C\": 15, \"H\": 192, \"W\": 192, \"NM\": 8, \"NV\": 3, \"A\": 2, "
                            "\"beta_min\": 1.0, \"P\": " + std::to_string(torch::cat(flat).numel()) +
                            ", \"params\": " + names + "}");
    auto [a, lp, ent, v, mu, sg, feat] = agent->forward(bev, meas, vmeas, act, "given");
    dump("carla_act", "logprob", lp); dump("carla_act", "entropy", ent); dump("carla_act", "value", v.view(-1));
    dump("carla_act", "alpha", mu); dump("carla_act", "beta", sg); dump("carla_act", "action_roundtrip", a);
    dump("carla_act", "features", feat);
    auto [am, lpm, entm, vm, mum, sgm, fm] = agent->forward(bev, meas, vmeas, Tensor(), "mean");
    dump("carla_act", "mean_action", am); dump("carla_act", "mean_logprob", lpm);
    auto [ar, lpr, entr, vr, mur, sgr, fr] = agent->forward(bev, meas, vmeas, Tensor(), "roach");
    dump("carla_act", "roach_action", ar); dump("carla_act", "roach_logprob", lpr);
    end_case();
  }

  // ---- CaRL update: loss, backward, clip_grad_norm_, Adam (ac_ppo_carla.cpp:540-619) ----------
  // Same parameters / input streams as carla_act with N=4 rows; gradients and the stepped
  // parameters are summarised per tensor (sum, sum of squares, 32 entries at hbits-drawn indices)
  // so the 1.2 M-float vectors need not be stored.
  {
    const int N = 4, C = 15, HW = 192, NM = 8, NV = 3, A = 2;
    CarlaAgent agent(C, NM, NV, A, 1.0f, -1.0f, 1.0f);
    {
      torch::NoGradGuard ng;
      int t = 0;
      for (auto& kv : agent->named_parameters()) {
        Tensor p = kv.value();
        Tensor v;
        if (kv.key() == "action_space_high") v = torch::tensor(1.0f);
        else if (kv.key() == "action_space_low") v = torch::tensor(-1.0f);
        else if (p.dim() >= 2) {
          const float a = std::sqrt(6.0f / (float)(p.numel() / p.size(0)));
          v = hunif(1000 + t, p.sizes().vec(), -a, a);
        } else v = hunif(1000 + t, p.sizes().vec(), -0.1f, 0.1f);
        p.copy_(v.reshape(p.sizes()));
        ++t;
      }
    }
    Tensor bev = torch::empty({N, C, HW, HW}, torch::kUInt8);
    uint8_t* bp = bev.data_ptr<uint8_t>();
    for (int64_t i = 0; i < bev.numel(); ++i) bp[i] = (uint8_t)(hbits(1, (uint32_t)i) >> 24);
    Tensor meas = hunif(2, {N, NM}, -1.0f, 1.0f), vmeas = hunif(3, {N, NV}, -1.0f, 1.0f);
    Tensor act = hunif(4, {N, A}, -0.98f, 0.98f);
    Tensor old_logp, old_v;
    {
      torch::NoGradGuard ng;
      auto [a0, lp0, e0, v0, m0, s0, f0] = agent->forward(bev, meas, vmeas, act, "given");
      old_logp = lp0 + (hunif(5, {N}, 0.0f, 1.0f) - 0.5f) * 0.3f;
      old_v = v0.view(-1) + (hunif(8, {N}, 0.0f, 1.0f) - 0.5f) * 0.3f;
    }
    Tensor adv = hunif(6, {N}, -1.0f, 1.0f), ret = hunif(7, {N}, -1.0f, 1.0f);
    LossCfg c{0.2f, 0.01f, 0.5f, true, true};
    auto [a, lp, ent, v, mu, sg, feat] = agent->forward(bev, meas, vmeas, act, "given");
    auto [loss, st] = ppo_loss(lp, ent, v, old_logp, adv, ret, old_v, c, nullptr, nullptr);
    loss.backward();
    const int NS = 32;
    auto summarise = [&](bool grads) {
      std::vector<Tensor> rows;
      std::vector<int64_t> idx;
      int t = 0;
      for (auto& kv : agent->named_parameters()) {
        Tensor x = grads ? (kv.value().grad().defined() ? kv.value().grad() : torch::zeros_like(kv.value()))
                         : kv.value().detach();
        x = x.reshape({-1}).to(torch::kFloat64);
        std::vector<double> r = {x.sum().item<double>(), x.square().sum().item<double>()};
        for (int i = 0; i < NS; ++i) {
          const int64_t k = (int64_t)(hbits(2000 + t, (uint32_t)i) % (uint32_t)x.numel());
          idx.push_back(k);
          r.push_back(x[k].item<double>());
        }
        rows.push_back(torch::tensor(r, torch::kFloat64));
        ++t;
      }
      return std::make_pair(torch::stack(rows).to(torch::kFloat32), torch::tensor(idx, torch::kInt64));
    };
    begin_case("carla_update", "{\"N\": 4, \"C\": 15, \"H\": 192, \"W\": 192, \"NM\": 8, \"NV\": 3, \"A\": 2, "
                               "\"beta_min\": 1.0, \"clip_coef\": 0.2, \"ent_coef\": 0.01, \"vf_coef\": 0.5, "
                               "\"clip_vloss\": 1, \"norm_adv\": 1, \"max_grad_norm\": 0.5, \"lr\": 0.0003, "
                               "\"adam_eps\": 1e-05, \"samples_per_tensor\": 32}");
    dump("carla_update", "old_logp", old_logp); dump("carla_update", "old_v", old_v);
    dump("carla_update", "adv", adv); dump("carla_update", "ret", ret);
    dump("carla_update", "logprob", lp); dump("carla_update", "value", v.view(-1));
    dump("carla_update", "stats", torch::tensor(st));
    auto [gsum, gidx] = summarise(true);
    dump("carla_update", "grad_summary", gsum); dump("carla_update", "sample_idx", gidx.view({gsum.size(0), NS}));
    torch::optim::Adam opt(agent->parameters(), torch::optim::AdamOptions(3e-4).eps(1e-5));
    const double tn = torch::nn::utils::clip_grad_norm_(agent->parameters(), 0.5);
    dump("carla_update", "total_norm", torch::tensor({(float)tn}));
    opt.step();
    auto [psum, pidx] = summarise(false);
    dump("carla_update", "param_step1_summary", psum);
    end_case();
  }

  // ---- Distribution spot values straight from rl_utils.h ------------------------------------
  {
    torch::NoGradGuard ng;
    Tensor al = randu({256}, 1.0f, 8.0f), be = randu({256}, 1.0f, 8.0f), xs = randu({256}, 0.01f, 0.99f);
    const Beta b(al, be);
    begin_case("beta_dist", "{\"n\": 256}");
    dump("beta_dist", "alpha", al); dump("beta_dist", "beta", be); dump("beta_dist", "x", xs);
    dump("beta_dist", "log_prob", b.log_prob(xs)); dump("beta_dist", "entropy", b.entropy());
    dump("beta_dist", "mean", b.mean());
    end_case();
  }

  // ---- LibTorch checkpoints: torch::save of agent + Adam (save_state, ppo:173-180), SURVEY §8 f-2 ----
  // Small agents (O=5, A=2, H=16) after two Adam steps on a surrogate loss; model.pth and
  // optimizer.pth are the fixtures, params / adam_m / adam_v their flat contents.
  {
    const int Op = 5, Ap = 2, Hp = 16, Mp = 8;
    auto pth_case = [&](const std::string& cname, auto& agent, auto&& loss_fn) {
      std::string names;
      set_params(*agent, names);
      torch::optim::Adam opt(agent->parameters(), torch::optim::AdamOptions(2.5e-4).eps(1e-5));
      for (int s = 0; s < 2; ++s) {
        opt.zero_grad();
        loss_fn().backward();
        opt.step();
      }
      begin_case(cname, "{\"O\": 5, \"A\": 2, \"H\": 16, \"steps\": 2, \"lr\": 0.00025, \"eps\": 1e-05, "
                        "\"params\": " + names + "}");
      dump(cname, "params", flat_params(*agent));
      dump(cname, "adam_m", flat_state(opt, false));
      dump(cname, "adam_v", flat_state(opt, true));
      end_case();
      torch::save(agent, g_out + "/" + cname + "/model.pth");
      torch::save(opt, g_out + "/" + cname + "/optimizer.pth");
    };
    {
      PPOAgent agent(Op, Ap, Hp);
      Tensor x = randn({Mp, Op}), act = randn({Mp, Ap}, 0.8f);
      pth_case("pth_ppo", agent, [&] {
        auto [a, lp, ent, v, mu] = agent->get_action_and_value(x, act);
        return -lp.mean() + v.square().mean() - 0.01f * ent.mean();
      });
    }
    {
      ACAgent agent(Op, Ap, Hp, 1.0f, -1.0f, torch::zeros({Op}), torch::ones({Op}));
      Tensor x = randn({Mp, Op}), act = randu({Mp, Ap}, -0.98f, 0.98f);
      pth_case("pth_ac", agent, [&] {
        auto [a, lp, ent, v, al, be] = agent->get_action_and_value(x, act, "given");
        return -lp.mean() + v.square().mean() - 0.01f * ent.mean();
      });
    }
  }

  // ---- round 2: the reference's real widths, long / ragged GAE, the PPO env wrappers ----------
  width_cases();
  e2e_cases();

  g_manifest << "\n}\n";
  std::ofstream(g_out + "/manifest.json") << g_manifest.str();
  std::printf("golden fixtures written to %s\n", g_out.c_str());
  return 0;
}
