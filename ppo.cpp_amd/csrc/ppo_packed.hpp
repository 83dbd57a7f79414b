// ppo_packed.hpp — HBM layout of the agent on the device.
//
// The reference's flat named_parameters() order (include/ppo_layout.h) is the external format.
// On the device every tensor starts on a 64-byte boundary and Linear(O, H) weights are stored
// [H][OP] with OP = roundup(O, 16) (zero padded), so every MFMA A-operand is one aligned 16-byte
// load. Gradients and both Adam moments use the same packed layout (padding stays exactly 0).
#pragma once

#include <string.h>

#include "../../include/ppo_layout.h"

struct TrunkDev {
  int W1, b1, g1, be1, W2, b2, g2, be2;  // packed float offsets (g*/be* = -1 for the tanh net)
};

struct PackedLayout {
  int kind, O, A, H, OP;
  int hi, lo, omean, ostd, logstd;
  TrunkDev tr[2];  // 0 = critic, 1 = actor (actor_mean / actor_encoder)
  int cW3, cb3;    // critic head Linear(H,1)
  int aW3, ab3;    // PPO actor_mean.4 [A][H] / AC dist_alpha [A][H]
  int bW3, bb3;    // AC dist_beta [A][H]
  int size;        // floats
  // tensor table in reference order: packed offset, rows, cols, leading dim, grad flag
  int nt;
  int poff[PPO_LAYOUT_MAX_TENSORS], rows[PPO_LAYOUT_MAX_TENSORS], cols[PPO_LAYOUT_MAX_TENSORS];
  int ld[PPO_LAYOUT_MAX_TENSORS], grad[PPO_LAYOUT_MAX_TENSORS];
};

inline int pk_round16(int x) { return (x + 15) & ~15; }

inline PackedLayout make_packed(const ppo_layout& L) {
  PackedLayout K;
  memset(&K, 0, sizeof(K));
  K.kind = L.kind; K.O = L.O; K.A = L.A; K.H = L.H; K.OP = pk_round16(L.O);
  int cur = 0;
  K.nt = L.ntensors;
  for (int t = 0; t < L.ntensors; ++t) {
    const long off = L.t_off[t];
    int rows = 1, cols = (int)L.t_len[t], ld = cols;
    if (off == L.critic.W1 || off == L.actor.W1) { rows = L.H; cols = L.O; ld = K.OP; }
    K.poff[t] = cur; K.rows[t] = rows; K.cols[t] = cols; K.ld[t] = ld; K.grad[t] = L.t_grad[t];
    cur += pk_round16(rows * ld);
  }
  K.size = cur;
  auto map = [&](long off) -> int {
    if (off < 0) return -1;
    for (int t = 0; t < L.ntensors; ++t)
      if (L.t_off[t] == off) return K.poff[t];
    return -1;
  };
  K.hi = map(L.hi); K.lo = map(L.lo); K.omean = map(L.omean); K.ostd = map(L.ostd); K.logstd = map(L.logstd);
  const ppo_trunk_layout* src[2] = {&L.critic, &L.actor};
  for (int k = 0; k < 2; ++k) {
    K.tr[k].W1 = map(src[k]->W1); K.tr[k].b1 = map(src[k]->b1); K.tr[k].g1 = map(src[k]->g1);
    K.tr[k].be1 = map(src[k]->be1); K.tr[k].W2 = map(src[k]->W2); K.tr[k].b2 = map(src[k]->b2);
    K.tr[k].g2 = map(src[k]->g2); K.tr[k].be2 = map(src[k]->be2);
  }
  K.cW3 = map(L.cW3); K.cb3 = map(L.cb3); K.aW3 = map(L.aW3); K.ab3 = map(L.ab3);
  K.bW3 = map(L.bW3); K.bb3 = map(L.bb3);
  return K;
}

// flat (reference order) <-> packed, host side
inline void pack_params(const PackedLayout& K, const ppo_layout& L, const float* flat, float* packed) {
  memset(packed, 0, sizeof(float) * K.size);
  for (int t = 0; t < K.nt; ++t)
    for (int r = 0; r < K.rows[t]; ++r)
      memcpy(packed + K.poff[t] + (long)r * K.ld[t], flat + L.t_off[t] + (long)r * K.cols[t], sizeof(float) * K.cols[t]);
}
inline void unpack_params(const PackedLayout& K, const ppo_layout& L, const float* packed, float* flat) {
  for (int t = 0; t < K.nt; ++t)
    for (int r = 0; r < K.rows[t]; ++r)
      memcpy(flat + L.t_off[t] + (long)r * K.cols[t], packed + K.poff[t] + (long)r * K.ld[t], sizeof(float) * K.cols[t]);
}

// Per-trunk "small gradient" vector produced by the fused forward/backward kernel (everything
// except the two Linear weight matrices, which the dW GEMM kernel produces):
//   [b1 H][g1 H][be1 H][b2 H][g2 H][be2 H][head W nh*H][head b nh][logstd A][stats 8]
struct SmallGradLayout {
  int H, nh, A;
  int b1, g1, be1, b2, g2, be2, hW, hb, ls, stats, size;
};
inline SmallGradLayout make_sg(int H, int nh, int A) {
  SmallGradLayout s;
  s.H = H; s.nh = nh; s.A = A;
  s.b1 = 0; s.g1 = H; s.be1 = 2 * H; s.b2 = 3 * H; s.g2 = 4 * H; s.be2 = 5 * H;
  s.hW = 6 * H; s.hb = s.hW + nh * H; s.ls = s.hb + nh; s.stats = s.ls + A;
  s.size = (s.stats + 8 + 3) & ~3;
  return s;
}
// loss statistic slots (sums over rows; divided by M at reduction)
enum { ST_PG = 0, ST_V = 1, ST_ENT = 2, ST_OKL = 3, ST_KL = 4, ST_CF = 5 };
