/*
 * ppo_layout.h — flat parameter layout of the two PPO agents (plain C, header-only).
 *
 * The flat vector follows LibTorch's Module::named_parameters() order for the reference agents,
 * so a parameter dump of the reference model maps 1:1 onto it:
 *
 *   PPO_NET_TANH_NORMAL  — AgentImpl of ppo_continuous_action
 *       (reference: src/ppo_continuous_action.cpp:120-171)
 *       actor_logstd[1,A],
 *       critic.0.weight[H,O] critic.0.bias[H] critic.2.weight[H,H] critic.2.bias[H]
 *       critic.4.weight[1,H] critic.4.bias[1],
 *       actor_mean.0.weight[H,O] actor_mean.0.bias[H] actor_mean.2.weight[H,H] actor_mean.2.bias[H]
 *       actor_mean.4.weight[A,H] actor_mean.4.bias[A]                         (H = 64)
 *
 *   PPO_NET_LN_BETA      — AgentImpl of ac_ppo_continuous_action
 *       (reference: src/ac_ppo_continuous_action.cpp:150-268)
 *       action_space_high[] action_space_low[] mean_[1,O] std_[1,O]           (no grad)
 *       critic.{0:Linear(O,H) 1:LayerNorm(H) 3:Linear(H,H) 4:LayerNorm(H) 6:Linear(H,1)},
 *       actor_mean.{0:Linear(O,H) 1:LayerNorm(H) 3:Linear(H,H) 4:LayerNorm(H)},
 *       dist_alpha.0:Linear(H,A), dist_beta.0:Linear(H,A)                      (H = 256)
 *
 * Weights are row-major [out, in] exactly as nn::Linear stores them (y = x W^T + b).
 * The "tensor table" lists every named parameter with its grad flag: clip_grad_norm_ and Adam
 * operate per tensor (reference: torch/nn/utils/clip_grad.h norm-of-norms, optim::Adam per param).
 */
#ifndef PPO_LAYOUT_H
#define PPO_LAYOUT_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { PPO_NET_TANH_NORMAL = 0, PPO_NET_LN_BETA = 1 };

#define PPO_LAYOUT_MAX_TENSORS 32

/* Offsets (in floats) of one 2-hidden-layer trunk. LayerNorm offsets are -1 for the tanh net. */
typedef struct ppo_trunk_layout {
  long W1, b1, g1, be1, W2, b2, g2, be2;
} ppo_trunk_layout;

typedef struct ppo_layout {
  int kind, O, A, H;
  long P;             /* total floats in the flat vector (incl. non-grad params) */
  long train_begin;   /* first trainable float (everything after it is trainable) */
  long hi, lo, omean, ostd; /* AC non-grad params (-1 for PPO) */
  long logstd;        /* PPO actor_logstd (-1 for AC) */
  ppo_trunk_layout critic, actor;
  long cW3, cb3;      /* critic head Linear(H,1) */
  long aW3, ab3;      /* PPO: actor_mean.4 Linear(H,A); AC: dist_alpha Linear(H,A) */
  long bW3, bb3;      /* AC: dist_beta Linear(H,A); -1 for PPO */
  int ntensors;
  long t_off[PPO_LAYOUT_MAX_TENSORS];
  long t_len[PPO_LAYOUT_MAX_TENSORS];
  int t_grad[PPO_LAYOUT_MAX_TENSORS];
} ppo_layout;

static inline long ppo_layout__add(ppo_layout* L, long* cur, long n, int grad) {
  long off = *cur;
  L->t_off[L->ntensors] = off;
  L->t_len[L->ntensors] = n;
  L->t_grad[L->ntensors] = grad;
  L->ntensors++;
  *cur += n;
  return off;
}

/* Fills L for the given net kind / dims. Returns 0 on success, -1 on bad arguments. */
static inline int ppo_layout_init(ppo_layout* L, int kind, int O, int A, int H) {
  long cur = 0;
  if (O <= 0 || A <= 0 || H <= 0) return -1;
  if (kind != PPO_NET_TANH_NORMAL && kind != PPO_NET_LN_BETA) return -1;
  L->kind = kind; L->O = O; L->A = A; L->H = H;
  L->ntensors = 0;
  L->hi = L->lo = L->omean = L->ostd = L->logstd = -1;
  L->bW3 = L->bb3 = -1;
  if (kind == PPO_NET_TANH_NORMAL) {
    L->logstd = ppo_layout__add(L, &cur, A, 1);
    L->train_begin = 0;
    L->critic.W1 = ppo_layout__add(L, &cur, (long)H * O, 1);
    L->critic.b1 = ppo_layout__add(L, &cur, H, 1);
    L->critic.g1 = L->critic.be1 = -1;
    L->critic.W2 = ppo_layout__add(L, &cur, (long)H * H, 1);
    L->critic.b2 = ppo_layout__add(L, &cur, H, 1);
    L->critic.g2 = L->critic.be2 = -1;
    L->cW3 = ppo_layout__add(L, &cur, H, 1);
    L->cb3 = ppo_layout__add(L, &cur, 1, 1);
    L->actor.W1 = ppo_layout__add(L, &cur, (long)H * O, 1);
    L->actor.b1 = ppo_layout__add(L, &cur, H, 1);
    L->actor.g1 = L->actor.be1 = -1;
    L->actor.W2 = ppo_layout__add(L, &cur, (long)H * H, 1);
    L->actor.b2 = ppo_layout__add(L, &cur, H, 1);
    L->actor.g2 = L->actor.be2 = -1;
    L->aW3 = ppo_layout__add(L, &cur, (long)A * H, 1);
    L->ab3 = ppo_layout__add(L, &cur, A, 1);
  } else {
    L->hi = ppo_layout__add(L, &cur, 1, 0);
    L->lo = ppo_layout__add(L, &cur, 1, 0);
    L->omean = ppo_layout__add(L, &cur, O, 0);
    L->ostd = ppo_layout__add(L, &cur, O, 0);
    L->train_begin = cur;
    ppo_trunk_layout* tr[2] = {&L->critic, &L->actor};
    for (int k = 0; k < 2; ++k) {
      tr[k]->W1 = ppo_layout__add(L, &cur, (long)H * O, 1);
      tr[k]->b1 = ppo_layout__add(L, &cur, H, 1);
      tr[k]->g1 = ppo_layout__add(L, &cur, H, 1);
      tr[k]->be1 = ppo_layout__add(L, &cur, H, 1);
      tr[k]->W2 = ppo_layout__add(L, &cur, (long)H * H, 1);
      tr[k]->b2 = ppo_layout__add(L, &cur, H, 1);
      tr[k]->g2 = ppo_layout__add(L, &cur, H, 1);
      tr[k]->be2 = ppo_layout__add(L, &cur, H, 1);
      if (k == 0) {
        L->cW3 = ppo_layout__add(L, &cur, H, 1);
        L->cb3 = ppo_layout__add(L, &cur, 1, 1);
      }
    }
    L->aW3 = ppo_layout__add(L, &cur, (long)A * H, 1);
    L->ab3 = ppo_layout__add(L, &cur, A, 1);
    L->bW3 = ppo_layout__add(L, &cur, (long)A * H, 1);
    L->bb3 = ppo_layout__add(L, &cur, A, 1);
  }
  L->P = cur;
  return 0;
}

#ifdef __cplusplus
}
#endif
#endif /* PPO_LAYOUT_H */
