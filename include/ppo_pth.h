/*
 * ppo_pth.h — LibTorch checkpoint interop behind the ppo_hip.h C-ABI
 * conventions: int status (0 = OK, -1 = bad argument / I/O / format error), ppo_last_error() for
 * the message. Host memory only; no GPU is touched.
 *
 * The files are the TorchScript module archives torch::save writes and torch::load reads:
 *   ppo_pth_save_agent  <-> torch::save(agent, "model_*.pth")
 *                           (save_state, src/ppo_continuous_action.cpp:173-180 / :546 / :587,
 *                            src/ac_ppo_continuous_action.cpp:907-909 / :952)
 *   ppo_pth_load_agent  <-> torch::load(agent, path) (src/carla/ac_ppo_carla.cpp:236)
 *   ppo_pth_save_adam   <-> torch::save(optimizer, "optimizer_*.pth") (same save_state)
 *   ppo_pth_load_adam   <-> torch::load(optimizer, path) (src/carla/ac_ppo_carla.cpp:251)
 *   ppo_carla_pth_*     <-> the CaRL agent's model_*.pth (src/carla/ppo_carla_inference.cpp:104)
 * Flat vectors follow the layouts' named_parameters() order (ppo_layout.h, ppo_carla.h); the
 * module structure written around them (Sequential children, parameterless Tanh / ReLU modules,
 * class numbering) is the reference agents' (ppo_continuous_action.cpp:120-157,
 * ac_ppo_continuous_action.cpp:150-249, carla_model.h:65-192 with image_encoder "roach" and
 * use_layer_norm false). Loading requires every named parameter with the same shape, as
 * torch::load does; extra entries are ignored.
 */
#ifndef PPO_PTH_H
#define PPO_PTH_H

#include "ppo_carla.h"
#include "ppo_layout.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ppo_layout_init / ppo_carla_layout_init as exported symbols (for bindings that cannot use the
 * static inline header functions); -1 on bad dimensions. */
int ppo_layout_fill(ppo_layout* L, int kind, int O, int A, int H);
int ppo_carla_layout_fill(ppo_carla_layout* L, int C, int IH, int IW, int NM, int NV, int A);

int ppo_pth_save_agent(const ppo_layout* L, const float* params, const char* path);
int ppo_pth_load_agent(const ppo_layout* L, const char* path, float* params, long n);
/* Adam state in flat order (exp_avg, exp_avg_sq) with its step count; the archive's options are
 * lr, betas (0.9, 0.999), eps, weight_decay 0, amsgrad false (AdamOptions(lr).eps(eps)). Tensors
 * without gradient (AC action-space / normalisation parameters) carry no state, as in LibTorch.
 * step == 0 writes an optimizer without state (before its first step). */
int ppo_pth_save_adam(const ppo_layout* L, const float* m, const float* v, long step, double lr, double eps,
                      const char* path);
/* lr_out / eps_out may be NULL */
int ppo_pth_load_adam(const ppo_layout* L, const char* path, float* m, float* v, long n, long* step,
                      double* lr_out, double* eps_out);

int ppo_carla_pth_save(const ppo_carla_layout* L, const float* params, const char* path);
int ppo_carla_pth_load(const ppo_carla_layout* L, const char* path, float* params, long n);

#ifdef __cplusplus
}
#endif

#endif /* PPO_PTH_H */
