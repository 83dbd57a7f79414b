// ppo_pth.hip — C-ABI of include/ppo_pth.h: the reference agents' module structure as pth::Spec
// over the flat layouts, and the archive reader/writer of pth_io.hpp. Host code only.
#include <exception>
#include <string>
#include <vector>

#include "../../include/ppo_pth.h"
#include "ppo_kernels.hpp"  // ppo_fail
#include "pth_io.hpp"

namespace {

using Shape = std::vector<int64_t>;

void seq(pth::Spec& s, const std::string& name, int n) {
  s.modules.push_back(name);
  for (int i = 0; i < n; ++i) s.modules.push_back(name + "." + std::to_string(i));
}
void linear(pth::Spec& s, const std::string& name, long w, long b, int out, int in) {
  s.tensors.push_back({name + ".weight", Shape{out, in}, w, true});
  s.tensors.push_back({name + ".bias", Shape{out}, b, true});
}
void norm(pth::Spec& s, const std::string& name, long g, long b, int n) {
  s.tensors.push_back({name + ".weight", Shape{n}, g, true});
  s.tensors.push_back({name + ".bias", Shape{n}, b, true});
}

// ppo_continuous_action.cpp:120-157 / ac_ppo_continuous_action.cpp:150-249
pth::Spec agent_spec(const ppo_layout& L) {
  pth::Spec s;
  s.P = L.P;
  const int O = L.O, A = L.A, H = L.H;
  if (L.kind == PPO_NET_TANH_NORMAL) {
    seq(s, "critic", 5);      // Linear Tanh Linear Tanh Linear
    seq(s, "actor_mean", 5);
    s.tensors.push_back({"actor_logstd", Shape{1, A}, L.logstd, true});
    linear(s, "critic.0", L.critic.W1, L.critic.b1, H, O);
    linear(s, "critic.2", L.critic.W2, L.critic.b2, H, H);
    linear(s, "critic.4", L.cW3, L.cb3, 1, H);
    linear(s, "actor_mean.0", L.actor.W1, L.actor.b1, H, O);
    linear(s, "actor_mean.2", L.actor.W2, L.actor.b2, H, H);
    linear(s, "actor_mean.4", L.aW3, L.ab3, A, H);
  } else {
    seq(s, "critic", 7);      // Linear LayerNorm ReLU Linear LayerNorm ReLU Linear
    seq(s, "actor_mean", 6);  // Linear LayerNorm ReLU Linear LayerNorm ReLU
    seq(s, "dist_alpha", 1);
    seq(s, "dist_beta", 1);
    s.tensors.push_back({"action_space_high", Shape{}, L.hi, false});
    s.tensors.push_back({"action_space_low", Shape{}, L.lo, false});
    s.tensors.push_back({"mean_", Shape{1, O}, L.omean, false});
    s.tensors.push_back({"std_", Shape{1, O}, L.ostd, false});
    linear(s, "critic.0", L.critic.W1, L.critic.b1, H, O);
    norm(s, "critic.1", L.critic.g1, L.critic.be1, H);
    linear(s, "critic.3", L.critic.W2, L.critic.b2, H, H);
    norm(s, "critic.4", L.critic.g2, L.critic.be2, H);
    linear(s, "critic.6", L.cW3, L.cb3, 1, H);
    linear(s, "actor_mean.0", L.actor.W1, L.actor.b1, H, O);
    norm(s, "actor_mean.1", L.actor.g1, L.actor.be1, H);
    linear(s, "actor_mean.3", L.actor.W2, L.actor.b2, H, H);
    norm(s, "actor_mean.4", L.actor.g2, L.actor.be2, H);
    linear(s, "dist_alpha.0", L.aW3, L.ab3, A, H);
    linear(s, "dist_beta.0", L.bW3, L.bb3, A, H);
  }
  return s;
}

// carla_model.h:65-192 (roach encoder, no layer norm)
pth::Spec carla_spec(const ppo_carla_layout& L) {
  pth::Spec s;
  s.P = L.P;
  seq(s, "cnn", 2 * PPO_CARLA_NCONV);  // Conv ReLU x 6
  seq(s, "linear", 4);
  seq(s, "state_linear", 4);
  seq(s, "value_head", 5);
  seq(s, "policy_head", 4);
  seq(s, "dist_mu", 1);
  seq(s, "dist_sigma", 1);
  s.tensors.push_back({"action_space_high", Shape{}, L.hi, false});
  s.tensors.push_back({"action_space_low", Shape{}, L.lo, false});
  for (int i = 0; i < PPO_CARLA_NCONV; ++i) {
    const std::string n = "cnn." + std::to_string(2 * i);
    s.tensors.push_back({n + ".weight", Shape{L.conv_oc[i], L.conv_ic[i], L.conv_k[i], L.conv_k[i]}, L.conv_w[i], true});
    s.tensors.push_back({n + ".bias", Shape{L.conv_oc[i]}, L.conv_b[i], true});
  }
  linear(s, "linear.0", L.lin_w[0], L.lin_b[0], 512, 1024 + 256);
  linear(s, "linear.2", L.lin_w[1], L.lin_b[1], 256, 512);
  linear(s, "state_linear.0", L.st_w[0], L.st_b[0], 256, L.NM);
  linear(s, "state_linear.2", L.st_w[1], L.st_b[1], 256, 256);
  linear(s, "value_head.0", L.v_w[0], L.v_b[0], 256, 256 + L.NV);
  linear(s, "value_head.2", L.v_w[1], L.v_b[1], 256, 256);
  linear(s, "value_head.4", L.v_w[2], L.v_b[2], 1, 256);
  linear(s, "policy_head.0", L.pi_w[0], L.pi_b[0], 256, 256);
  linear(s, "policy_head.2", L.pi_w[1], L.pi_b[1], 256, 256);
  linear(s, "dist_mu.0", L.mu_w, L.mu_b, L.A, 256);
  linear(s, "dist_sigma.0", L.sg_w, L.sg_b, L.A, 256);
  return s;
}

// the spec must tile the layout exactly (guards a layout / spec drift)
bool covers(const pth::Spec& s) {
  long total = 0;
  for (const auto& t : s.tensors) {
    long n = 1;
    for (int64_t d : t.shape) n *= (long)d;
    if (t.off < 0 || t.off + n > s.P) return false;
    total += n;
  }
  return total == s.P;
}

template <typename F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const std::exception& e) {
    return ppo_fail(e.what(), -1);
  }
}

}  // namespace

extern "C" int ppo_layout_fill(ppo_layout* L, int kind, int O, int A, int H) {
  if (!L || ppo_layout_init(L, kind, O, A, H) != 0) return ppo_fail("ppo_layout_fill: bad arguments", -1);
  return 0;
}

extern "C" int ppo_carla_layout_fill(ppo_carla_layout* L, int C, int IH, int IW, int NM, int NV, int A) {
  if (!L || ppo_carla_layout_init(L, C, IH, IW, NM, NV, A) != 0)
    return ppo_fail("ppo_carla_layout_fill: bad arguments (n_flatten must be 256 * 2 * 2)", -1);
  return 0;
}

extern "C" int ppo_pth_save_agent(const ppo_layout* L, const float* params, const char* path) {
  if (!L || !params || !path) return ppo_fail("ppo_pth_save_agent: null argument", -1);
  return guarded([&] {
    const pth::Spec s = agent_spec(*L);
    if (!covers(s)) return ppo_fail("ppo_pth_save_agent: layout does not match the agent structure", -1);
    pth::save_module(path, s, params);
    return 0;
  });
}

extern "C" int ppo_pth_load_agent(const ppo_layout* L, const char* path, float* params, long n) {
  if (!L || !params || !path) return ppo_fail("ppo_pth_load_agent: null argument", -1);
  if (n != L->P) return ppo_fail("ppo_pth_load_agent: n != layout P", -1);
  return guarded([&] {
    const pth::Spec s = agent_spec(*L);
    if (!covers(s)) return ppo_fail("ppo_pth_load_agent: layout does not match the agent structure", -1);
    const std::vector<float> flat = pth::load_module(path, s);
    std::copy(flat.begin(), flat.end(), params);
    return 0;
  });
}

extern "C" int ppo_pth_save_adam(const ppo_layout* L, const float* m, const float* v, long step, double lr,
                                 double eps, const char* path) {
  if (!L || !m || !v || !path) return ppo_fail("ppo_pth_save_adam: null argument", -1);
  if (step < 0) return ppo_fail("ppo_pth_save_adam: negative step", -1);
  return guarded([&] {
    const pth::Spec s = agent_spec(*L);
    pth::AdamOptions o;
    o.lr = lr;
    o.eps = eps;
    pth::save_adam(path, s, m, v, step, o);
    return 0;
  });
}

extern "C" int ppo_pth_load_adam(const ppo_layout* L, const char* path, float* m, float* v, long n, long* step,
                                 double* lr_out, double* eps_out) {
  if (!L || !m || !v || !path || !step) return ppo_fail("ppo_pth_load_adam: null argument", -1);
  if (n != L->P) return ppo_fail("ppo_pth_load_adam: n != layout P", -1);
  return guarded([&] {
    const pth::Spec s = agent_spec(*L);
    pth::AdamOptions o;
    *step = pth::load_adam(path, s, m, v, &o);
    if (lr_out) *lr_out = o.lr;
    if (eps_out) *eps_out = o.eps;
    return 0;
  });
}

extern "C" int ppo_carla_pth_save(const ppo_carla_layout* L, const float* params, const char* path) {
  if (!L || !params || !path) return ppo_fail("ppo_carla_pth_save: null argument", -1);
  return guarded([&] {
    const pth::Spec s = carla_spec(*L);
    if (!covers(s)) return ppo_fail("ppo_carla_pth_save: layout does not match the agent structure", -1);
    pth::save_module(path, s, params);
    return 0;
  });
}

extern "C" int ppo_carla_pth_load(const ppo_carla_layout* L, const char* path, float* params, long n) {
  if (!L || !params || !path) return ppo_fail("ppo_carla_pth_load: null argument", -1);
  if (n != L->P) return ppo_fail("ppo_carla_pth_load: n != layout P", -1);
  return guarded([&] {
    const pth::Spec s = carla_spec(*L);
    if (!covers(s)) return ppo_fail("ppo_carla_pth_load: layout does not match the agent structure", -1);
    const std::vector<float> flat = pth::load_module(path, s);
    std::copy(flat.begin(), flat.end(), params);
    return 0;
  });
}
