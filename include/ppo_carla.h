/*
 * ppo_carla.h — the CaRL CNN agent's forward pass behind the same C-ABI
 * conventions as ppo_hip.h: int status (0 = OK), ppo_last_error() for the message, device
 * pointers for every array, the handle owns its device memory.
 *
 * Reference: include/carla/carla_model.h:21-318 (AgentImpl), with the defaults of
 * include/carla/carla_config.h: image_encoder "roach" (:71), use_layer_norm false (:78),
 * use_positional_encoding false (:117), obs_num_channels 15 (:58), bev 192 x 192 (:101-102),
 * obs_num_measurements 8 (:90), num_value_measurements 3 (:103), beta_min_a_b_value 1.0 (:56).
 *
 *   bev uint8 [N, C, 192, 192] / 255
 *     -> cnn: Conv(C,8,5,s2) ReLU Conv(8,16,5,s2) ReLU Conv(16,32,5,s2) ReLU
 *             Conv(32,64,3,s2) ReLU Conv(64,128,3,s2) ReLU Conv(128,256,3,s1) ReLU   -> [N, 1024]
 *     state_linear: Linear(8,256) ReLU Linear(256,256) ReLU on measurements         -> [N, 256]
 *     linear: Linear(1024+256, 512) ReLU Linear(512, 256) ReLU                      -> features
 *   value_head: Linear(256+3, 256) ReLU Linear(256,256) ReLU Linear(256,1) on [features | vmeas]
 *   policy_head: Linear(256,256) ReLU Linear(256,256) ReLU; dist_mu / dist_sigma: Linear(256, A)
 *   alpha = softplus(mu) + beta_min, beta = softplus(sigma) + beta_min; Beta(alpha, beta)
 *   (rl_utils.h:87-132): sample | mean | roach_deterministic | given action (scaled to [0,1] and
 *   clamped to [1e-7, 1 + 1e-7], carla_model.h:251-260); log_prob and entropy summed over
 *   actions; the action is unscaled to [low, high] (:262-268).
 *
 * Parameter order = LibTorch named_parameters() of that module: action_space_high[],
 * action_space_low[] (no grad, own parameters first), then cnn.{0,2,4,6,8,10}.{weight,bias},
 * linear.{0,2}, state_linear.{0,2}, value_head.{0,2,4}, policy_head.{0,2}, dist_mu.0,
 * dist_sigma.0 (registration order, carla_model.h:108-192). Conv weights [OC, IC, k, k],
 * Linear weights [out, in].
 */
#ifndef PPO_CARLA_H
#define PPO_CARLA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PPO_CARLA_MAX_TENSORS 40
#define PPO_CARLA_NCONV 6

/* sample types: 0 "sample", 1 "mean", 2 given action, 3 "roach" (carla_model.h:287-303) */
enum { PPO_CARLA_SAMPLE = 0, PPO_CARLA_MEAN = 1, PPO_CARLA_GIVEN = 2, PPO_CARLA_ROACH = 3 };

typedef struct ppo_carla_layout {
  int C, IH, IW, NM, NV, A;
  long P;                       /* total floats */
  long hi, lo;                  /* action_space_high / low (no grad) */
  long conv_w[PPO_CARLA_NCONV], conv_b[PPO_CARLA_NCONV];
  int conv_ic[PPO_CARLA_NCONV], conv_oc[PPO_CARLA_NCONV], conv_k[PPO_CARLA_NCONV], conv_s[PPO_CARLA_NCONV];
  int conv_ih[PPO_CARLA_NCONV], conv_iw[PPO_CARLA_NCONV], conv_oh[PPO_CARLA_NCONV], conv_ow[PPO_CARLA_NCONV];
  long lin_w[2], lin_b[2];      /* linear.0: Linear(1024 + 256, 512), linear.2: Linear(512, 256) */
  long st_w[2], st_b[2];        /* state_linear.0: Linear(NM, 256), state_linear.2: Linear(256, 256) */
  long v_w[3], v_b[3];          /* value_head.{0,2,4}: Linear(256 + NV, 256), Linear(256, 256), Linear(256, 1) */
  long pi_w[2], pi_b[2];        /* policy_head.{0,2}: Linear(256, 256) x 2 */
  long mu_w, mu_b, sg_w, sg_b;  /* dist_mu.0, dist_sigma.0: Linear(256, A) */
  int ntensors;
  long t_off[PPO_CARLA_MAX_TENSORS];
  long t_len[PPO_CARLA_MAX_TENSORS];
  int t_grad[PPO_CARLA_MAX_TENSORS];
} ppo_carla_layout;

static inline long ppo_carla__add(ppo_carla_layout* L, long* cur, long n, int grad) {
  const long off = *cur;
  L->t_off[L->ntensors] = off;
  L->t_len[L->ntensors] = n;
  L->t_grad[L->ntensors] = grad;
  L->ntensors++;
  *cur += n;
  return off;
}

/* Returns 0, or -1 if the shapes do not give the reference's fixed n_flatten = 256 * 2 * 2
 * (carla_model.h:110) or are non-positive. */
static inline int ppo_carla_layout_init(ppo_carla_layout* L, int C, int IH, int IW, int NM, int NV, int A) {
  static const int oc[PPO_CARLA_NCONV] = {8, 16, 32, 64, 128, 256};
  static const int ks[PPO_CARLA_NCONV] = {5, 5, 5, 3, 3, 3};
  static const int st[PPO_CARLA_NCONV] = {2, 2, 2, 2, 2, 1};
  long cur = 0;
  int i, h = IH, w = IW, ic = C;
  if (C <= 0 || IH <= 0 || IW <= 0 || NM <= 0 || NV < 0 || A <= 0) return -1;
  L->C = C; L->IH = IH; L->IW = IW; L->NM = NM; L->NV = NV; L->A = A;
  L->ntensors = 0;
  L->hi = ppo_carla__add(L, &cur, 1, 0);
  L->lo = ppo_carla__add(L, &cur, 1, 0);
  for (i = 0; i < PPO_CARLA_NCONV; ++i) {
    L->conv_ic[i] = ic; L->conv_oc[i] = oc[i]; L->conv_k[i] = ks[i]; L->conv_s[i] = st[i];
    L->conv_ih[i] = h; L->conv_iw[i] = w;
    if (h < ks[i] || w < ks[i]) return -1;
    h = (h - ks[i]) / st[i] + 1;
    w = (w - ks[i]) / st[i] + 1;
    L->conv_oh[i] = h; L->conv_ow[i] = w;
    L->conv_w[i] = ppo_carla__add(L, &cur, (long)oc[i] * ic * ks[i] * ks[i], 1);
    L->conv_b[i] = ppo_carla__add(L, &cur, oc[i], 1);
    ic = oc[i];
  }
  if (256L * h * w != 1024) return -1;
  L->lin_w[0] = ppo_carla__add(L, &cur, 512L * (1024 + 256), 1); L->lin_b[0] = ppo_carla__add(L, &cur, 512, 1);
  L->lin_w[1] = ppo_carla__add(L, &cur, 256L * 512, 1);          L->lin_b[1] = ppo_carla__add(L, &cur, 256, 1);
  L->st_w[0] = ppo_carla__add(L, &cur, 256L * NM, 1);            L->st_b[0] = ppo_carla__add(L, &cur, 256, 1);
  L->st_w[1] = ppo_carla__add(L, &cur, 256L * 256, 1);           L->st_b[1] = ppo_carla__add(L, &cur, 256, 1);
  L->v_w[0] = ppo_carla__add(L, &cur, 256L * (256 + NV), 1);     L->v_b[0] = ppo_carla__add(L, &cur, 256, 1);
  L->v_w[1] = ppo_carla__add(L, &cur, 256L * 256, 1);            L->v_b[1] = ppo_carla__add(L, &cur, 256, 1);
  L->v_w[2] = ppo_carla__add(L, &cur, 256, 1);                   L->v_b[2] = ppo_carla__add(L, &cur, 1, 1);
  L->pi_w[0] = ppo_carla__add(L, &cur, 256L * 256, 1);           L->pi_b[0] = ppo_carla__add(L, &cur, 256, 1);
  L->pi_w[1] = ppo_carla__add(L, &cur, 256L * 256, 1);           L->pi_b[1] = ppo_carla__add(L, &cur, 256, 1);
  L->mu_w = ppo_carla__add(L, &cur, 256L * A, 1);                L->mu_b = ppo_carla__add(L, &cur, A, 1);
  L->sg_w = ppo_carla__add(L, &cur, 256L * A, 1);                L->sg_b = ppo_carla__add(L, &cur, A, 1);
  L->P = cur;
  return 0;
}

typedef struct ppo_carla_config {
  int obs_channels;            /* 15 */
  int bev_h, bev_w;            /* 192, 192 */
  int num_measurements;        /* 8 */
  int num_value_measurements;  /* 3 */
  int action_dim;              /* 2 (steer, acceleration) */
  float beta_min;              /* 1.0 */
  int max_batch;               /* largest n passed to ppo_carla_forward */
  uint64_t seed;               /* Philox sampling key (same contract as ppo_hip.h) */
  int rank;
} ppo_carla_config;

typedef struct ppo_carla ppo_carla_t;

/* carla_model.h:35-206 (the module) — allocates parameters and activation buffers on `device`. */
int ppo_carla_create(const ppo_carla_config* cfg, int device, ppo_carla_t** out);
/* options: NULL / "" (defaults) or "key=value" pairs separated by ',':
 *   conv1=packed|staged|generic  conv1 forward with packed taps (k_conv_img3, default), conv1 forward
 *                              and weight gradient with the image patch staged in LDS (staged; the
 *                              weight gradient's form for packed too), or the generic implicit-GEMM
 *                              kernels (A/B tests)
 *   conv1_mfma=auto|bx3|f32    the packed conv1 forward and the staged conv1 weight gradient with their
 *                              products as split-bf16 MFMAs (bx3, auto: the raw byte operand is exact
 *                              in bf16, the fp32 operand's three bf16 pieces make every product exact;
 *                              fp32 accumulation on 16x16x32 bf16 MFMAs) or on 16x16x4 fp32 MFMAs
 *   conv_fwd=tiled|generic     conv2 / conv3 forward from LDS-staged input patches (k_conv_t / k_conv_t2,
 *                              default) or the generic gather kernel (A/B tests; another fp32 sum order)
 *   conv_wgrad=tiled|generic   conv2 / conv3 weight gradients from LDS-staged tiles (k_wgrad_t / k_wgrad_t2,
 *                              default) or the generic k_wgrad
 *   conv_dgrad=quad|staged     conv2 / conv3 input gradients with the four stride-2 parity classes of a
 *                              quad sharing one dZ operand (k_dgrad_q / k_dgrad_q2, default) or
 *                              k_dgrad_s2 / k_dgrad (needs conv1=staged|packed)
 *   deep_dgrad=col|gather      conv6's input gradient as a dense GEMM into columns + col2im (default) or
 *                              k_dgrad
 *   tail=staged|fused|layers   forwards of n <= 64 rows: the MLP tail after the CNN as one launch per
 *                              dependency stage (default), one cooperative launch with a grid barrier
 *                              between stages, or one k_conv / k_conv_fin pair per layer (the path of
 *                              larger batches); bitwise equal
 *   wgrad_group_bytes=N        (tests) the generic fp32 weight-gradient kernel runs its samples in groups
 *                              whose input stays below N bytes, each group's sums added to the previous
 *                              ones'; without it the groups start at 0x70000000 bytes (the kernel's 32-bit
 *                              buffer offsets), so no batch size is refused */
int ppo_carla_create_ex(const ppo_carla_config* cfg, int device, const char* options, ppo_carla_t** out);
int ppo_carla_destroy(ppo_carla_t* c);
int ppo_carla_get_layout(const ppo_carla_t* c, ppo_carla_layout* out);
/* host floats in named_parameters() order (torch::load of a model_*.pth, ac_ppo_carla.cpp) */
int ppo_carla_load_params(ppo_carla_t* c, const float* host, long n);
/* AgentImpl::forward (carla_model.h:270-318) for n rows; every array is a device pointer:
 *   bev uint8 [n, C, IH, IW], meas [n, NM], vmeas [n, NV], action_in [n, A] (GIVEN only);
 *   outputs (any may be NULL): action [n, A] in [low, high], logprob [n], entropy [n],
 *   value [n], alpha [n, A], beta [n, A].
 * SAMPLE draws with the Philox contract of ppo_hip.h (env = env_base + row, step = step_id). */
int ppo_carla_forward(ppo_carla_t* c, int n, const uint8_t* bev, const float* meas, const float* vmeas,
                      int sample_type, const float* action_in, long env_base, long step_id, float* action,
                      float* logprob, float* entropy, float* value, float* alpha, float* beta, void* stream);

/* ---- training (ac_ppo_carla.cpp:529-620): one PPO minibatch step --------------------------------
 * Loss = pg_loss - ent_coef * entropy + vf_coef * v_loss exactly as the MLP agents (clipped
 * surrogate, clipped value loss, minibatch advantage normalisation with Bessel's correction),
 * backward through heads, MLPs and all six convolutions, clip_grad_norm_(max_grad_norm), Adam
 * (betas 0.9 / 0.999, eps = adam_eps, bias-corrected, weight_decay 0), all on the device. */
typedef struct ppo_carla_train_config {
  float clip_coef;      /* 0.2 */
  float ent_coef;       /* 0.0 */
  float vf_coef;        /* 0.5 */
  float max_grad_norm;  /* 0.5 */
  float adam_eps;       /* 1e-5 */
  int norm_adv;         /* 1 */
  int clip_vloss;       /* 1 */
} ppo_carla_train_config;

typedef struct ppo_carla_update_stats {
  float pg_loss, v_loss, entropy, old_approx_kl, approx_kl, clipfrac;
  float grad_norm;  /* total norm before clipping */
} ppo_carla_update_stats;

/* One minibatch of n <= max_batch rows (device pointers): bev uint8 [n, C, IH, IW], meas [n, NM],
 * vmeas [n, NV], actions [n, A] (env space), old_logp / adv / ret / old_v [n]. stats may be NULL
 * (no host synchronisation then). */
int ppo_carla_update(ppo_carla_t* c, const ppo_carla_train_config* tc, int n, const uint8_t* bev, const float* meas,
                     const float* vmeas, const float* actions, const float* old_logp, const float* adv,
                     const float* ret, const float* old_v, float lr, ppo_carla_update_stats* stats, void* stream);
/* parameters (named_parameters() order) and the raw gradient of the last update, to host */
int ppo_carla_save_params(ppo_carla_t* c, float* host, long n);
int ppo_carla_last_grad(ppo_carla_t* c, float* host, long n);
/* Adam moments in the same flat order, and the step count */
int ppo_carla_save_adam(ppo_carla_t* c, float* m_host, float* v_host, long n, long* step);
int ppo_carla_load_adam(ppo_carla_t* c, const float* m_host, const float* v_host, long n, long step);

/* ---- data parallelism (ac_ppo_carla.cpp:243, 561-616; torchfort::Comm, distributed.cpp:81-224) ----
 * One RCCL communicator per agent; id from ppo_comm_unique_id (ppo_hip.h), PPO_COMM_ID_BYTES bytes.
 * With a communicator attached (any world >= 1), every ppo_carla_update
 *   - takes the minibatch advantage mean as the rank average of the local means and the std
 *     from the all-reduced sum of squares with Bessel's correction over world * n - 1
 *     (ac_ppo_carla.cpp:561-580),
 *   - all-reduces (average) the gradient of every trainable tensor before clip_grad_norm_ (:608-616),
 *   - averages the returned loss statistics over ranks (:645-651; grad_norm is already global).
 * world = 1 runs the same collective sequence over a one-rank communicator (results equal the
 * communicator-free update bit for bit). */
int ppo_carla_comm_init(ppo_carla_t* c, const char* id, int rank, int world);
/* ac_ppo_carla.cpp:241-244: every parameter from `root` to all ranks */
int ppo_carla_comm_broadcast_params(ppo_carla_t* c, int root);

#ifdef __cplusplus
}
#endif

#endif /* PPO_CARLA_H */
