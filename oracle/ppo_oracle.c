/*
 * ppo_oracle.c — CPU restatement of the reference's rollout -> GAE -> PPO-update hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see ppo_oracle.h). Never linked into the product.
 *
 * Arithmetic: fp32 element-wise math in the reference's op order, double accumulators for the
 * reductions (dot products, LayerNorm moments, minibatch means, gradient sums) so the oracle is
 * at least as accurate as the LibTorch CPU path it restates. GAE is restated op-for-op in fp32
 * and is bit-exact with the reference formula.
 */
#include "ppo_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------ */
/* RNG contract: Philox4x32-10 + murmur3 fmix32 keyed Feistel permutation                      */
/* ------------------------------------------------------------------------------------------ */

void orc_philox4x32(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

uint32_t orc_mix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85EBCA6Bu;
  h ^= h >> 13; h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

float orc_u01(uint32_t x) { return ((float)(x >> 8) + 0.5f) * 5.9604644775390625e-8f; }

static void sample_key(uint64_t seed, int rank, uint32_t key[2]) {
  key[0] = (uint32_t)seed;
  key[1] = (uint32_t)(seed >> 32) ^ (0x85EBCA6Bu * (uint32_t)(rank + 1));
}

static void philox_draw(uint64_t seed, int rank, long env, long step, uint32_t draw, uint32_t out[4]) {
  uint32_t key[2], ctr[4];
  sample_key(seed, rank, key);
  ctr[0] = (uint32_t)env; ctr[1] = (uint32_t)step; ctr[2] = (uint32_t)((uint64_t)step >> 32); ctr[3] = draw;
  orc_philox4x32(ctr, key, out);
}

/* Box-Muller pair from two 32-bit draws. */
static void box_muller(uint32_t a, uint32_t b, float* z0, float* z1) {
  float u0 = orc_u01(a), u1 = orc_u01(b);
  float r = sqrtf(-2.0f * logf(u0));
  float th = 6.2831853071795865f * u1;
  *z0 = r * cosf(th);
  *z1 = r * sinf(th);
}

/* Feistel permutation on [0, 2^bits) (bits even), cycle-walked into [0, B).
 * Replaces torch::randperm (ppo:490, ac:804); keys depend on (seed, rank, epoch counter). */
static uint32_t perm_round_key(uint64_t seed, int rank, long epoch_counter, int r) {
  uint32_t base = orc_mix32((uint32_t)seed ^ 0x1B873593u) ^ orc_mix32((uint32_t)(seed >> 32) + 0x68E31DA4u) ^
                  orc_mix32((uint32_t)rank * 0x632BE5ABu + 0x2545F491u) ^
                  orc_mix32((uint32_t)epoch_counter * 2u + 1u);
  return orc_mix32(base + (uint32_t)r * 0x9E3779B9u);
}

long orc_perm_index(long i, long B, uint64_t seed, int rank, long epoch_counter) {
  int bits = 2;
  while ((1L << bits) < B) bits += 2;
  int half = bits / 2;
  uint32_t mask = (1u << half) - 1u;
  uint32_t k[4];
  for (int r = 0; r < 4; ++r) k[r] = perm_round_key(seed, rank, epoch_counter, r);
  uint32_t x = (uint32_t)i;
  do {
    uint32_t L = x >> half, R = x & mask;
    for (int r = 0; r < 4; ++r) {
      uint32_t F = orc_mix32(R * 0x9E3779B1u + k[r]) & mask;
      uint32_t nL = R, nR = L ^ F;
      L = nL; R = nR;
    }
    x = (L << half) | R;
  } while ((long)x >= B);
  return (long)x;
}

void orc_perm(long B, uint64_t seed, int rank, long epoch_counter, int64_t* out) {
  for (long i = 0; i < B; ++i) out[i] = orc_perm_index(i, B, seed, rank, epoch_counter);
}

/* ------------------------------------------------------------------------------------------ */
/* Special functions: restatement of ATen's calc_digamma / calc_trigamma (Math.h)              */
/* ------------------------------------------------------------------------------------------ */

double orc_digamma(double x) {
  static const double PSI_10 = 2.25175258906672110764;
  if (x == 0) return copysign(INFINITY, -x);
  int x_is_integer = (x == trunc(x));
  if (x < 0) {
    if (x_is_integer) return NAN;
    double q, r = modf(x, &q);
    return orc_digamma(1 - x) - M_PI / tan(M_PI * r);
  }
  double result = 0;
  while (x < 10) { result -= 1 / x; x += 1; }
  if (x == 10) return result + PSI_10;
  static const double A[] = {8.33333333333333333333E-2, -2.10927960927960927961E-2, 7.57575757575757575758E-3,
                             -4.16666666666666666667E-3, 3.96825396825396825397E-3, -8.33333333333333333333E-3,
                             8.33333333333333333333E-2};
  double y = 0;
  if (x < 1.0e17) {
    double z = 1.0 / (x * x);
    double p = 0;
    for (int i = 0; i < 7; ++i) p = p * z + A[i];
    y = z * p;
  }
  return result + log(x) - (0.5 / x) - y;
}

double orc_trigamma(double x) {
  double sign = +1, result = 0;
  if (x < 0.5) {
    sign = -1;
    double s = sin(M_PI * x);
    result -= (M_PI * M_PI) / (s * s);
    x = 1 - x;
  }
  for (int i = 0; i < 6; ++i) { result += 1 / (x * x); x += 1; }
  double ixx = 1 / (x * x);
  result += (1 + 1 / (2 * x) + ixx * (1. / 6 - ixx * (1. / 30 - ixx * (1. / 42)))) / x;
  return sign * result;
}

/* ATen softplus(beta=1, threshold=20) forward / backward (factor d softplus / dx). */
static float softplus_f(float x) { return x > 20.0f ? x : log1pf(expf(x)); }
static float softplus_d(float x) {
  if (x > 20.0f) return 1.0f;
  float z = expf(x);
  return z / (z + 1.0f);
}
static float xlogy_f(float a, float b) {
  if (isnan(b)) return NAN;
  if (a == 0.0f) return 0.0f;
  return a * logf(b);
}

/* ------------------------------------------------------------------------------------------ */
/* Agent forward / backward for one row                                                       */
/* ------------------------------------------------------------------------------------------ */

#define MAXH 1024
#define MAXA 64
#define MAXO 4096

typedef struct trunk_cache {
  float x[MAXO];
  float z1[MAXH], h1[MAXH], xh1[MAXH], rstd1;
  float z2[MAXH], h2[MAXH], xh2[MAXH], rstd2;
} trunk_cache;

/* Linear layer y[o] = sum_i W[o,i] x[i] + b[o], double accumulation (nn::Linear, addmm). */
static void linear(const float* W, const float* b, const float* x, int in, int out, float* y) {
  for (int o = 0; o < out; ++o) {
    double acc = 0;
    const float* w = W + (long)o * in;
    for (int i = 0; i < in; ++i) acc += (double)w[i] * (double)x[i];
    y[o] = (float)(acc + (double)b[o]);
  }
}

/* LayerNorm(H, eps=1e-5, affine) + ReLU (ac:159-174), keeping x_hat and rstd for backward. */
static void ln_relu(const float* z, const float* g, const float* be, int H, float* xh, float* rstd, float* h) {
  double mean = 0, var = 0;
  for (int i = 0; i < H; ++i) mean += z[i];
  mean /= H;
  for (int i = 0; i < H; ++i) { double d = z[i] - mean; var += d * d; }
  var /= H;
  float rs = (float)(1.0 / sqrt(var + 1e-5));
  *rstd = rs;
  for (int i = 0; i < H; ++i) {
    xh[i] = (float)((z[i] - mean) * rs);
    float y = g[i] * xh[i] + be[i];
    h[i] = y > 0.0f ? y : 0.0f;
  }
}

static void trunk_forward(const ppo_layout* L, const ppo_trunk_layout* tr, const float* P, const float* x,
                          trunk_cache* c) {
  const int O = L->O, H = L->H;
  memcpy(c->x, x, sizeof(float) * O);
  linear(P + tr->W1, P + tr->b1, x, O, H, c->z1);
  if (L->kind == PPO_NET_TANH_NORMAL) {
    for (int i = 0; i < H; ++i) c->h1[i] = tanhf(c->z1[i]);
  } else {
    ln_relu(c->z1, P + tr->g1, P + tr->be1, H, c->xh1, &c->rstd1, c->h1);
  }
  linear(P + tr->W2, P + tr->b2, c->h1, H, H, c->z2);
  if (L->kind == PPO_NET_TANH_NORMAL) {
    for (int i = 0; i < H; ++i) c->h2[i] = tanhf(c->z2[i]);
  } else {
    ln_relu(c->z2, P + tr->g2, P + tr->be2, H, c->xh2, &c->rstd2, c->h2);
  }
}

/* Backward through a trunk given d(h2); accumulates into the double gradient vector. */
static void trunk_backward(const ppo_layout* L, const ppo_trunk_layout* tr, const float* P, const trunk_cache* c,
                           const double* dh2, double* G) {
  const int O = L->O, H = L->H;
  double dz2[MAXH], dh1[MAXH], dz1[MAXH];
  if (L->kind == PPO_NET_TANH_NORMAL) {
    for (int i = 0; i < H; ++i) dz2[i] = dh2[i] * (1.0 - (double)c->h2[i] * c->h2[i]);
  } else {
    const float* g = P + tr->g2;
    double dy[MAXH], s1 = 0, s2 = 0;
    for (int i = 0; i < H; ++i) {
      float y = g[i] * c->xh2[i] + P[tr->be2 + i];
      dy[i] = y > 0.0f ? dh2[i] : 0.0;
      G[tr->g2 + i] += dy[i] * c->xh2[i];
      G[tr->be2 + i] += dy[i];
      double dx = dy[i] * g[i];
      s1 += dx; s2 += dx * c->xh2[i];
    }
    s1 /= H; s2 /= H;
    for (int i = 0; i < H; ++i) dz2[i] = c->rstd2 * (dy[i] * g[i] - s1 - c->xh2[i] * s2);
  }
  for (int o = 0; o < H; ++o) {
    G[tr->b2 + o] += dz2[o];
    double* gw = G + tr->W2 + (long)o * H;
    for (int i = 0; i < H; ++i) gw[i] += dz2[o] * c->h1[i];
  }
  for (int i = 0; i < H; ++i) dh1[i] = 0;
  for (int o = 0; o < H; ++o) {
    const float* w = P + tr->W2 + (long)o * H;
    for (int i = 0; i < H; ++i) dh1[i] += dz2[o] * w[i];
  }
  if (L->kind == PPO_NET_TANH_NORMAL) {
    for (int i = 0; i < H; ++i) dz1[i] = dh1[i] * (1.0 - (double)c->h1[i] * c->h1[i]);
  } else {
    const float* g = P + tr->g1;
    double dy[MAXH], s1 = 0, s2 = 0;
    for (int i = 0; i < H; ++i) {
      float y = g[i] * c->xh1[i] + P[tr->be1 + i];
      dy[i] = y > 0.0f ? dh1[i] : 0.0;
      G[tr->g1 + i] += dy[i] * c->xh1[i];
      G[tr->be1 + i] += dy[i];
      double dx = dy[i] * g[i];
      s1 += dx; s2 += dx * c->xh1[i];
    }
    s1 /= H; s2 /= H;
    for (int i = 0; i < H; ++i) dz1[i] = c->rstd1 * (dy[i] * g[i] - s1 - c->xh1[i] * s2);
  }
  for (int o = 0; o < H; ++o) {
    G[tr->b1 + o] += dz1[o];
    double* gw = G + tr->W1 + (long)o * O;
    for (int i = 0; i < O; ++i) gw[i] += dz1[o] * c->x[i];
  }
}

static float dot_head(const float* w, const float* b, const float* h, int H) {
  double acc = 0;
  for (int i = 0; i < H; ++i) acc += (double)w[i] * (double)h[i];
  return (float)(acc + (double)*b);
}

/* normalized input for the AC agent: (x - mean_) / std_ (ac:189, :215) */
static void agent_input(const ppo_layout* L, const float* P, const float* x, float* xn) {
  for (int i = 0; i < L->O; ++i)
    xn[i] = (L->kind == PPO_NET_LN_BETA) ? (x[i] - P[L->omean + i]) / P[L->ostd + i] : x[i];
}

/* Normal head (rl_utils.h:20-46, ppo:145-157). */
static const double kLz = 0.91893853320467274178; /* log(sqrt(2 pi)) */
static const double kEntC = 1.4189385332046727418; /* 0.5 + 0.5 log(2 pi) */

/* Gamma(alpha, 1) by Marsaglia-Tsang with the Philox contract (replaces at::_sample_dirichlet). */
static float gamma_mt(float alpha, uint64_t seed, int rank, long env, long step, uint32_t draw_base) {
  const float d = alpha - 0.33333334f;
  const float cc = 1.0f / sqrtf(9.0f * d);
  for (uint32_t t = 0; t < 64; ++t) {
    uint32_t r[4];
    philox_draw(seed, rank, env, step, draw_base + t, r);
    float z, z1;
    box_muller(r[0], r[1], &z, &z1);
    float y = 1.0f + cc * z;
    if (y <= 0.0f) continue;
    float v = y * y * y;
    float u = orc_u01(r[2]);
    float xx = z * z;
    if (u < 1.0f - 0.0331f * xx * xx) return d * v;
    if (logf(u) < 0.5f * xx + d * (1.0f - v + logf(v))) return d * v;
  }
  return d;
}

void orc_normal_noise(uint64_t seed, int rank, long env, long step, int A, float* z) {
  for (int a = 0; a < A; ++a) {
    uint32_t rr[4];
    philox_draw(seed, rank, env, step, (uint32_t)(a >> 1), rr);
    float z0, z1;
    box_muller(rr[0], rr[1], &z0, &z1);
    z[a] = (a & 1) ? z1 : z0;
  }
}

float orc_beta_sample01(float alpha, float beta, uint64_t seed, int rank, long env, long step, int a) {
  const float ga = gamma_mt(alpha, seed, rank, env, step, 0x10000u + (uint32_t)(a * 2 + 0) * 64u);
  const float gb = gamma_mt(beta, seed, rank, env, step, 0x10000u + (uint32_t)(a * 2 + 1) * 64u);
  return ga / (ga + gb);
}

void orc_get_action_and_value(const ppo_layout* L, const float* P, int n, const float* x, int mode,
                              const float* action_in, uint64_t seed, int rank, long env_base, long step_id,
                              float* action_out, float* logprob, float* entropy, float* value) {
  const int O = L->O, A = L->A, H = L->H;
  trunk_cache* cc = (trunk_cache*)malloc(sizeof(trunk_cache));
  trunk_cache* ca = (trunk_cache*)malloc(sizeof(trunk_cache));
  float xn[MAXO];
  for (int r = 0; r < n; ++r) {
    agent_input(L, P, x + (long)r * O, xn);
    trunk_forward(L, &L->critic, P, xn, cc);
    trunk_forward(L, &L->actor, P, xn, ca);
    if (value) value[r] = dot_head(P + L->cW3, P + L->cb3, cc->h2, H);
    double lp = 0, ent = 0;
    long env = env_base + r;
    if (L->kind == PPO_NET_TANH_NORMAL) {
      for (int a = 0; a < A; ++a) {
        float mu = dot_head(P + L->aW3 + (long)a * H, P + L->ab3 + a, ca->h2, H);
        float sd = expf(P[L->logstd + a]);
        float var = sd * sd, lsd = logf(sd);
        float act;
        if (mode == 1) {
          act = action_in[(long)r * A + a];
        } else if (mode == 2) {
          act = mu;
        } else {
          uint32_t rr[4];
          philox_draw(seed, rank, env, step_id, (uint32_t)(a >> 1), rr);
          float z0, z1;
          box_muller(rr[0], rr[1], &z0, &z1);
          act = mu + ((a & 1) ? z1 : z0) * sd;
        }
        if (action_out) action_out[(long)r * A + a] = act;
        float d = act - mu;
        lp += -(d * d) / (2.0f * var) - lsd - (float)kLz;
        ent += (float)kEntC + lsd;
      }
    } else {
      const float hi = P[L->hi], lo = P[L->lo];
      for (int a = 0; a < A; ++a) {
        float pa = dot_head(P + L->aW3 + (long)a * H, P + L->ab3 + a, ca->h2, H);
        float pb = dot_head(P + L->bW3 + (long)a * H, P + L->bb3 + a, ca->h2, H);
        float al = softplus_f(pa) + 1.0f, be = softplus_f(pb) + 1.0f;
        float s; /* action in [0,1] */
        if (mode == 1) {
          float av = action_in[(long)r * A + a];
          s = (av - lo) / (hi - lo) * (1.0f - 0.0f) + 0.0f;
          s = fminf(fmaxf(s, 0.0f + 1e-7f), 1.0f + 1e-7f);
        } else if (mode == 2) {
          s = al / (al + be);
        } else {
          float ga = gamma_mt(al, seed, rank, env, step_id, 0x10000u + (uint32_t)(a * 2 + 0) * 64u);
          float gb = gamma_mt(be, seed, rank, env, step_id, 0x10000u + (uint32_t)(a * 2 + 1) * 64u);
          s = ga / (ga + gb);
        }
        float ab = al + be;
        float l = xlogy_f(al - 1.0f, s) + xlogy_f(be - 1.0f, 1.0f - s);
        l += (float)(lgamma((double)ab) - (lgamma((double)al) + lgamma((double)be)));
        lp += l;
        double e = lgamma((double)al) + lgamma((double)be) - lgamma((double)ab) - (2.0 - ab) * orc_digamma(ab) -
                   ((al - 1.0) * orc_digamma(al) + (be - 1.0) * orc_digamma(be));
        ent += e;
        if (action_out) action_out[(long)r * A + a] = (s - 0.0f) / (1.0f - 0.0f) * (hi - lo) + lo;
      }
    }
    if (logprob) logprob[r] = (float)lp;
    if (entropy) entropy[r] = (float)ent;
  }
  free(cc);
  free(ca);
}

/* ------------------------------------------------------------------------------------------ */
/* Loss + backward for one minibatch (ppo:496-538; ac:816-875)                                 */
/* ------------------------------------------------------------------------------------------ */

void orc_adv_stats(int M, const float* adv, float* mean, float* stdv) {
  double s = 0;
  for (int i = 0; i < M; ++i) s += adv[i];
  double mu = s / M;
  double q = 0;
  for (int i = 0; i < M; ++i) { double d = adv[i] - (float)mu; q += d * d; }
  *mean = (float)mu;
  *stdv = (float)sqrt(q / (double)(M - 1));
}

/* Rows [r0, r1) of an M-row minibatch (ppo:497-538, ac:815-875): adds the loss gradient of those
 * rows (already scaled by 1/M) into G (double, flat layout) and the six per-row loss sums
 * (pg, v, entropy, old_kl, kl, clipfrac) into sums[6]. orc_minibatch_grad is the whole range; tests
 * run disjoint ranges on several threads and add the partials in a fixed order (large minibatches). */
void orc_minibatch_grad_part(const ppo_layout* L, const float* P, int M, int r0, int r1, const float* x,
                             const float* actions, const float* old_logp, const float* adv, const float* ret,
                             const float* old_v, float adv_mean, float adv_std, const orc_loss_cfg* cfg,
                             double* G, double* sums) {
  const int O = L->O, A = L->A, H = L->H;
  trunk_cache* cc = (trunk_cache*)malloc(sizeof(trunk_cache));
  trunk_cache* ca = (trunk_cache*)malloc(sizeof(trunk_cache));
  double s_pg = 0, s_v = 0, s_ent = 0, s_okl = 0, s_kl = 0, s_cf = 0;
  const double invM = 1.0 / M;
  const float c = cfg->clip_coef;
  float xn[MAXO];
  for (int r = r0; r < r1; ++r) {
    agent_input(L, P, x + (long)r * O, xn);
    trunk_forward(L, &L->critic, P, xn, cc);
    trunk_forward(L, &L->actor, P, xn, ca);
    const float v = dot_head(P + L->cW3, P + L->cb3, cc->h2, H);
    /* actor head */
    float mu[MAXA], pa[MAXA], pb[MAXA], al[MAXA], be[MAXA], sx[MAXA];
    double lp = 0, ent = 0;
    if (L->kind == PPO_NET_TANH_NORMAL) {
      for (int a = 0; a < A; ++a) {
        mu[a] = dot_head(P + L->aW3 + (long)a * H, P + L->ab3 + a, ca->h2, H);
        float sd = expf(P[L->logstd + a]);
        float var = sd * sd, lsd = logf(sd);
        float d = actions[(long)r * A + a] - mu[a];
        lp += -(d * d) / (2.0f * var) - lsd - (float)kLz;
        ent += (float)kEntC + lsd;
      }
    } else {
      const float hi = P[L->hi], lo = P[L->lo];
      for (int a = 0; a < A; ++a) {
        pa[a] = dot_head(P + L->aW3 + (long)a * H, P + L->ab3 + a, ca->h2, H);
        pb[a] = dot_head(P + L->bW3 + (long)a * H, P + L->bb3 + a, ca->h2, H);
        al[a] = softplus_f(pa[a]) + 1.0f;
        be[a] = softplus_f(pb[a]) + 1.0f;
        float s = (actions[(long)r * A + a] - lo) / (hi - lo) * (1.0f - 0.0f) + 0.0f;
        s = fminf(fmaxf(s, 1e-7f), 1.0f + 1e-7f);
        sx[a] = s;
        float ab = al[a] + be[a];
        float l = xlogy_f(al[a] - 1.0f, s) + xlogy_f(be[a] - 1.0f, 1.0f - s);
        l += (float)(lgamma((double)ab) - (lgamma((double)al[a]) + lgamma((double)be[a])));
        lp += l;
        ent += lgamma((double)al[a]) + lgamma((double)be[a]) - lgamma((double)ab) - (2.0 - ab) * orc_digamma(ab) -
               ((al[a] - 1.0) * orc_digamma(al[a]) + (be[a] - 1.0) * orc_digamma(be[a]));
      }
    }
    const float newlogp = (float)lp, entr = (float)ent;
    const float logratio = newlogp - old_logp[r];
    const float ratio = expf(logratio);
    s_okl += -logratio;
    s_kl += (ratio - 1.0f) - logratio;
    s_cf += (fabsf(ratio - 1.0f) > c) ? 1.0 : 0.0;
    float an = adv[r];
    if (cfg->norm_adv) an = (adv[r] - adv_mean) / (adv_std + 1e-8f);
    const float rc = fminf(fmaxf(ratio, 1.0f - c), 1.0f + c);
    const float pg1 = -an * ratio, pg2 = -an * rc;
    s_pg += fmaxf(pg1, pg2);
    /* d max(pg1,pg2)/d ratio; ties split the gradient (ATen maximum backward) */
    double dratio;
    {
      double w1 = pg1 > pg2 ? 1.0 : (pg1 == pg2 ? 0.5 : 0.0);
      double w2 = 1.0 - w1;
      double inr = (ratio >= 1.0f - c && ratio <= 1.0f + c) ? 1.0 : 0.0;
      dratio = w1 * (-an) + w2 * (-an) * inr;
    }
    const double g_logp = invM * dratio * ratio;
    double g_v;
    if (cfg->clip_vloss) {
      float vu = (v - ret[r]) * (v - ret[r]);
      float dv = v - old_v[r];
      float vcl = old_v[r] + fminf(fmaxf(dv, -c), c);
      float vc = (vcl - ret[r]) * (vcl - ret[r]);
      s_v += fmaxf(vu, vc);
      double w1 = vu > vc ? 1.0 : (vu == vc ? 0.5 : 0.0), w2 = 1.0 - w1;
      double inr = (dv >= -c && dv <= c) ? 1.0 : 0.0;
      g_v = 0.5 * cfg->vf_coef * invM * (w1 * 2.0 * (v - ret[r]) + w2 * 2.0 * (vcl - ret[r]) * inr);
    } else {
      float vu = (v - ret[r]) * (v - ret[r]);
      s_v += vu;
      g_v = 0.5 * cfg->vf_coef * invM * 2.0 * (v - ret[r]);
    }
    s_ent += entr;
    const double g_ent = -(double)cfg->ent_coef * invM;
    /* critic backward */
    double dh2[MAXH];
    G[L->cb3] += g_v;
    for (int i = 0; i < H; ++i) {
      G[L->cW3 + i] += g_v * cc->h2[i];
      dh2[i] = g_v * P[L->cW3 + i];
    }
    trunk_backward(L, &L->critic, P, cc, dh2, G);
    /* actor head backward */
    for (int i = 0; i < H; ++i) dh2[i] = 0;
    if (L->kind == PPO_NET_TANH_NORMAL) {
      for (int a = 0; a < A; ++a) {
        float sd = expf(P[L->logstd + a]);
        double var = (double)sd * sd;
        double d = actions[(long)r * A + a] - mu[a];
        double gmu = g_logp * d / var;
        G[L->logstd + a] += g_logp * (d * d / var - 1.0) + g_ent * 1.0;
        G[L->ab3 + a] += gmu;
        for (int i = 0; i < H; ++i) {
          G[L->aW3 + (long)a * H + i] += gmu * ca->h2[i];
          dh2[i] += gmu * P[L->aW3 + (long)a * H + i];
        }
      }
    } else {
      for (int a = 0; a < A; ++a) {
        double ab = (double)al[a] + be[a];
        double psab = orc_digamma(ab), tab = orc_trigamma(ab);
        double dla = ((al[a] - 1.0f) != 0.0f ? log((double)sx[a]) : 0.0) + psab - orc_digamma(al[a]);
        double dlb = ((be[a] - 1.0f) != 0.0f ? log((double)(1.0f - sx[a])) : 0.0) + psab - orc_digamma(be[a]);
        double dea = (ab - 2.0) * tab - (al[a] - 1.0) * orc_trigamma(al[a]);
        double deb = (ab - 2.0) * tab - (be[a] - 1.0) * orc_trigamma(be[a]);
        double gpa = (g_logp * dla + g_ent * dea) * softplus_d(pa[a]);
        double gpb = (g_logp * dlb + g_ent * deb) * softplus_d(pb[a]);
        G[L->ab3 + a] += gpa;
        G[L->bb3 + a] += gpb;
        for (int i = 0; i < H; ++i) {
          G[L->aW3 + (long)a * H + i] += gpa * ca->h2[i];
          G[L->bW3 + (long)a * H + i] += gpb * ca->h2[i];
          dh2[i] += gpa * P[L->aW3 + (long)a * H + i] + gpb * P[L->bW3 + (long)a * H + i];
        }
      }
    }
    trunk_backward(L, &L->actor, P, ca, dh2, G);
  }
  sums[0] += s_pg;
  sums[1] += s_v;
  sums[2] += s_ent;
  sums[3] += s_okl;
  sums[4] += s_kl;
  sums[5] += s_cf;
  free(cc);
  free(ca);
}

/* Finishes a minibatch from the accumulated partials: grad = (float)G, stats from the sums. */
void orc_minibatch_finish(const ppo_layout* L, int M, const double* G, const double* sums, const orc_loss_cfg* cfg,
                          float* grad, float* stats) {
  const double invM = 1.0 / M;
  for (long i = 0; i < L->P; ++i) grad[i] = (float)G[i];
  if (stats) {
    stats[0] = (float)(sums[0] * invM);
    stats[1] = (float)(0.5 * sums[1] * invM);
    stats[2] = (float)(sums[2] * invM);
    stats[3] = (float)(sums[3] * invM);
    stats[4] = (float)(sums[4] * invM);
    stats[5] = (float)(sums[5] * invM);
    stats[6] = (float)(stats[0] - cfg->ent_coef * stats[2] + stats[1] * cfg->vf_coef);
  }
}

void orc_minibatch_grad(const ppo_layout* L, const float* P, int M, const float* x, const float* actions,
                        const float* old_logp, const float* adv, const float* ret, const float* old_v,
                        float adv_mean, float adv_std, const orc_loss_cfg* cfg, float* grad, float* stats) {
  double* G = (double*)calloc((size_t)L->P, sizeof(double));
  double sums[6] = {0, 0, 0, 0, 0, 0};
  orc_minibatch_grad_part(L, P, M, 0, M, x, actions, old_logp, adv, ret, old_v, adv_mean, adv_std, cfg, G, sums);
  orc_minibatch_finish(L, M, G, sums, cfg, grad, stats);
  free(G);
}

/* ------------------------------------------------------------------------------------------ */
/* clip_grad_norm_ + Adam (torch/nn/utils/clip_grad.h; torch/optim/adam.cpp)                   */
/* ------------------------------------------------------------------------------------------ */

double orc_clip_grad_norm(const ppo_layout* L, float* grad, float max_norm) {
  double tot = 0;
  for (int t = 0; t < L->ntensors; ++t) {
    if (!L->t_grad[t]) continue;
    double s = 0;
    for (long i = 0; i < L->t_len[t]; ++i) { double g = grad[L->t_off[t] + i]; s += g * g; }
    float nrm = (float)sqrt(s); /* per-tensor norm is an fp32 tensor */
    tot += (double)nrm * nrm;
  }
  float total = (float)sqrt(tot);
  float coef = (float)max_norm / (total + 1e-6f);
  if (coef > 1.0f) coef = 1.0f;
  for (int t = 0; t < L->ntensors; ++t) {
    if (!L->t_grad[t]) continue;
    for (long i = 0; i < L->t_len[t]; ++i) grad[L->t_off[t] + i] *= coef;
  }
  return total;
}

void orc_adam_step(const ppo_layout* L, float* p, const float* g, float* m, float* v, long step, float lr,
                   float eps) {
  const double b1 = 0.9, b2 = 0.999;
  const double bc1 = 1.0 - pow(b1, (double)step), bc2 = 1.0 - pow(b2, (double)step);
  const float sbc2 = (float)sqrt(bc2);
  const float step_size = (float)((double)lr / bc1);
  for (int t = 0; t < L->ntensors; ++t) {
    if (!L->t_grad[t]) continue;
    for (long i = L->t_off[t]; i < L->t_off[t] + L->t_len[t]; ++i) {
      m[i] = m[i] * (float)b1 + g[i] * (float)(1.0 - b1);
      v[i] = v[i] * (float)b2 + g[i] * g[i] * (float)(1.0 - b2);
      float denom = sqrtf(v[i]) / sbc2 + eps;
      p[i] = p[i] - step_size * (m[i] / denom);
    }
  }
}

/* ------------------------------------------------------------------------------------------ */
/* GAE (ppo:447-467) — op-for-op fp32                                                          */
/* ------------------------------------------------------------------------------------------ */

void orc_gae(int T, int E, const float* rewards, const float* values, const float* dones, const float* next_value,
             const float* next_done, float gamma, float lam, float* adv, float* ret) {
  const float gl = gamma * lam;
  for (int e = 0; e < E; ++e) {
    float last = 0.0f;
    for (int t = T - 1; t >= 0; --t) {
      float nnt, nv;
      if (t == T - 1) { nnt = 1.0f - next_done[e]; nv = next_value[e]; }
      else { nnt = 1.0f - dones[(long)(t + 1) * E + e]; nv = values[(long)(t + 1) * E + e]; }
      volatile float gnv = gamma * nv;
      volatile float gnvn = gnv * nnt;
      volatile float rd = rewards[(long)t * E + e] + gnvn;
      volatile float delta = rd - values[(long)t * E + e];
      volatile float gln = gl * nnt;
      volatile float glnl = gln * last;
      volatile float a = delta + glnl;
      adv[(long)t * E + e] = a;
      last = a;
    }
    for (int t = 0; t < T; ++t) ret[(long)t * E + e] = adv[(long)t * E + e] + values[(long)t * E + e];
  }
}

/* ------------------------------------------------------------------------------------------ */
/* Update loop (ppo:489-542; ac:803-889)                                                       */
/* ------------------------------------------------------------------------------------------ */

void orc_update(const ppo_layout* L, float* params, float* m, float* v, long* step_io, long B, int O, int A,
                const float* b_obs, const float* b_actions, const float* b_logp, const float* b_adv,
                const float* b_ret, const float* b_val, int epochs, int minibatches, float lr, float max_grad_norm,
                float adam_eps, const orc_loss_cfg* cfg, uint64_t seed, int rank, long epoch_counter0,
                const int64_t* perms, float* stats_out) {
  const long Mb = B / minibatches;
  int64_t* perm = (int64_t*)malloc(sizeof(int64_t) * B);
  float* x = (float*)malloc(sizeof(float) * Mb * O);
  float* act = (float*)malloc(sizeof(float) * Mb * A);
  float* lp = (float*)malloc(sizeof(float) * Mb);
  float* ad = (float*)malloc(sizeof(float) * Mb);
  float* rt = (float*)malloc(sizeof(float) * Mb);
  float* vl = (float*)malloc(sizeof(float) * Mb);
  float* grad = (float*)malloc(sizeof(float) * L->P);
  float stats[7] = {0};
  double cf_sum = 0;
  int nmb = 0;
  for (int e = 0; e < epochs; ++e) {
    if (perms) memcpy(perm, perms + (long)e * B, sizeof(int64_t) * B);
    else orc_perm(B, seed, rank, epoch_counter0 + e, perm);
    for (long start = 0; start + Mb <= B; start += Mb) {
      for (long i = 0; i < Mb; ++i) {
        long j = perm[start + i];
        memcpy(x + i * O, b_obs + j * O, sizeof(float) * O);
        memcpy(act + i * A, b_actions + j * A, sizeof(float) * A);
        lp[i] = b_logp[j]; ad[i] = b_adv[j]; rt[i] = b_ret[j]; vl[i] = b_val[j];
      }
      float am = 0, as = 1;
      if (cfg->norm_adv) orc_adv_stats((int)Mb, ad, &am, &as);
      orc_minibatch_grad(L, params, (int)Mb, x, act, lp, ad, rt, vl, am, as, cfg, grad, stats);
      orc_clip_grad_norm(L, grad, max_grad_norm);
      *step_io += 1;
      orc_adam_step(L, params, grad, m, v, *step_io, lr, adam_eps);
      cf_sum += stats[5];
      nmb++;
    }
  }
  if (stats_out) {
    memcpy(stats_out, stats, sizeof(stats));
    stats_out[5] = (float)(cf_sum / (nmb > 0 ? nmb : 1));
  }
  free(perm); free(x); free(act); free(lp); free(ad); free(rt); free(vl); free(grad);
}

/* ------------------------------------------------------------------------------------------ */
/* Synthetic HalfCheetah-shaped env (O obs, A act, 1000-step truncation, never terminates)     */
/* wrapped as SeqVectorEnv(RecordEpisodeStatistics(env)) — gym.h:131-163, common.h:48-65       */
/* ------------------------------------------------------------------------------------------ */

static void env_reset_one(orc_env_state* s, int e, int seed, float* obs) {
  if (seed > 0) { s->rseed[e] = (uint32_t)seed; s->rcount[e] = 0; }
  for (int i = 0; i < s->O; ++i) {
    uint32_t key[2] = {s->rseed[e], 0x5EED5EEDu};
    uint32_t ctr[4] = {s->rcount[e], (uint32_t)i, 0u, 0u};
    uint32_t r[4];
    orc_philox4x32(ctr, key, r);
    s->q[(long)e * s->O + i] = 0.1f * (2.0f * orc_u01(r[0]) - 1.0f);
  }
  s->rcount[e] += 1;
  s->t[e] = 0;
  s->ep_ret[e] = 0.0f;
  s->ep_len[e] = 0;
  memcpy(obs + (long)e * s->O, s->q + (long)e * s->O, sizeof(float) * s->O);
}

void orc_env_reset(orc_env_state* s, int seed, float* obs_out) {
  for (int e = 0; e < s->E; ++e) {
    env_reset_one(s, e, seed + e, obs_out);
    s->autoreset[e] = 0;
  }
}

void orc_env_step(orc_env_state* s, const float* actions, float lo, float hi, float* obs, float* reward, float* term,
                  float* trunc, float* info_ret, int* info_len) {
  const int O = s->O, A = s->A;
  for (int e = 0; e < s->E; ++e) {
    info_ret[e] = 0.0f; info_len[e] = 0;
    if (s->autoreset[e]) {
      env_reset_one(s, e, -1, obs);
      reward[e] = 0.0f; term[e] = 0.0f; trunc[e] = 0.0f;
      s->autoreset[e] = 0;
      continue;
    }
    float a[MAXA];
    for (int k = 0; k < A; ++k) a[k] = fminf(fmaxf(actions[(long)e * A + k], lo), hi);
    float* q = s->q + (long)e * O;
    float nq[MAXO];
    const float xb = q[0];
    for (int i = 0; i < O; ++i) nq[i] = fmaf(0.9f, q[i], fmaf(0.1f, a[i % A], 0.05f * q[(i + 1) % O]));
    memcpy(q, nq, sizeof(float) * O);
    const float vel = (q[0] - xb) / 0.05f;
    float ctrl = 0.0f;
    for (int k = 0; k < A; ++k) ctrl = ctrl + 0.1f * a[k] * a[k];
    const float r = vel - ctrl;
    s->t[e] += 1;
    const int tr = s->t[e] >= 1000;
    memcpy(obs + (long)e * O, q, sizeof(float) * O);
    reward[e] = r; term[e] = 0.0f; trunc[e] = tr ? 1.0f : 0.0f;
    s->ep_ret[e] += r;
    s->ep_len[e] += 1;
    if (tr) { info_ret[e] = s->ep_ret[e]; info_len[e] = s->ep_len[e]; }
    s->autoreset[e] = tr;
  }
}

/* ------------------------------------------------------------------------------------------ */
/* CaRL CNN agent forward (include/carla/carla_model.h:222-318; carla_config.h defaults:        */
/* "roach" encoder :71, no LayerNorm :78, no positional encoding :117)                          */
/* ------------------------------------------------------------------------------------------ */

/* nn::Conv2d(IC, OC, K).stride(S), no padding, + ReLU; in [IC][IH][IW] -> out [OC][OH][OW] */
static void conv_relu(const float* in, int IC, int IH, int IW, const float* W, const float* b, int OC, int K, int S,
                      int OH, int OW, float* out) {
  for (int oc = 0; oc < OC; ++oc)
    for (int oy = 0; oy < OH; ++oy)
      for (int ox = 0; ox < OW; ++ox) {
        double acc = 0;
        for (int ic = 0; ic < IC; ++ic)
          for (int ky = 0; ky < K; ++ky) {
            const float* w = W + (((long)oc * IC + ic) * K + ky) * K;
            const float* x = in + ((long)ic * IH + (long)oy * S + ky) * IW + (long)ox * S;
            for (int kx = 0; kx < K; ++kx) acc += (double)w[kx] * (double)x[kx];
          }
        const float y = (float)(acc + (double)b[oc]);
        out[((long)oc * OH + oy) * OW + ox] = y > 0.0f ? y : 0.0f;
      }
}
static void linear_relu(const float* W, const float* b, const float* x, int in, int out, float* y) {
  linear(W, b, x, in, out, y);
  for (int o = 0; o < out; ++o) y[o] = y[o] > 0.0f ? y[o] : 0.0f;
}

int orc_carla_layout_init(ppo_carla_layout* L, int C, int IH, int IW, int NM, int NV, int A) {
  return ppo_carla_layout_init(L, C, IH, IW, NM, NV, A);
}

void orc_carla_forward(const ppo_carla_layout* L, const float* P, float beta_min, int n, const uint8_t* bev,
                       const float* meas, const float* vmeas, int mode, const float* action_in, uint64_t seed,
                       int rank, long env_base, long step_id, float* action, float* logprob, float* entropy,
                       float* value, float* alpha, float* beta, float* features) {
  const int A = L->A, NM = L->NM, NV = L->NV;
  long maxa = (long)L->C * L->IH * L->IW;
  for (int i = 0; i < PPO_CARLA_NCONV; ++i) {
    const long sz = (long)L->conv_oc[i] * L->conv_oh[i] * L->conv_ow[i];
    if (sz > maxa) maxa = sz;
  }
  float* b0 = (float*)malloc(sizeof(float) * maxa);
  float* b1 = (float*)malloc(sizeof(float) * maxa);
  float enc[1024 + 256], s1[256], l1[512], feat[256 + 64], v1[256], v2[256], p1[256], p2[256];
  const float hi = P[L->hi], lo = P[L->lo];
  for (int r = 0; r < n; ++r) {
    /* birdview = bev / 255 (carla_model.h:214-216, :223-224) */
    const long npx = (long)L->C * L->IH * L->IW;
    for (long i = 0; i < npx; ++i) b0[i] = (float)bev[(long)r * npx + i] / 255.0f;
    float* cur = b0;
    float* nxt = b1;
    for (int i = 0; i < PPO_CARLA_NCONV; ++i) {
      conv_relu(cur, L->conv_ic[i], L->conv_ih[i], L->conv_iw[i], P + L->conv_w[i], P + L->conv_b[i], L->conv_oc[i],
                L->conv_k[i], L->conv_s[i], L->conv_oh[i], L->conv_ow[i], nxt);
      float* t = cur; cur = nxt; nxt = t;
    }
    memcpy(enc, cur, sizeof(float) * 1024);                      /* flatten(x, 1): [C][H][W] order */
    linear_relu(P + L->st_w[0], P + L->st_b[0], meas + (long)r * NM, NM, 256, s1);
    linear_relu(P + L->st_w[1], P + L->st_b[1], s1, 256, 256, enc + 1024);
    linear_relu(P + L->lin_w[0], P + L->lin_b[0], enc, 1024 + 256, 512, l1);
    linear_relu(P + L->lin_w[1], P + L->lin_b[1], l1, 512, 256, feat);
    if (features) memcpy(features + (long)r * 256, feat, sizeof(float) * 256);
    /* value_head on cat(features, value_measurements) (:276-277) */
    for (int k = 0; k < NV; ++k) feat[256 + k] = vmeas[(long)r * NV + k];
    linear_relu(P + L->v_w[0], P + L->v_b[0], feat, 256 + NV, 256, v1);
    linear_relu(P + L->v_w[1], P + L->v_b[1], v1, 256, 256, v2);
    float vv;
    linear(P + L->v_w[2], P + L->v_b[2], v2, 256, 1, &vv);
    if (value) value[r] = vv;
    /* policy head, Beta(softplus + beta_min) (:279-285) */
    linear_relu(P + L->pi_w[0], P + L->pi_b[0], feat, 256, 256, p1);
    linear_relu(P + L->pi_w[1], P + L->pi_b[1], p1, 256, 256, p2);
    double lp = 0, ent = 0;
    const long env = env_base + r;
    for (int a = 0; a < A; ++a) {
      float pm, ps;
      linear(P + L->mu_w + (long)a * 256, P + L->mu_b + a, p2, 256, 1, &pm);
      linear(P + L->sg_w + (long)a * 256, P + L->sg_b + a, p2, 256, 1, &ps);
      const float al = softplus_f(pm) + beta_min, be = softplus_f(ps) + beta_min;
      if (alpha) alpha[(long)r * A + a] = al;
      if (beta) beta[(long)r * A + a] = be;
      float s;
      if (mode == PPO_CARLA_GIVEN) {                            /* scale_action (:251-260) */
        s = (action_in[(long)r * A + a] - lo) / (hi - lo) * (1.0f - 0.0f) + 0.0f;
        s = fminf(fmaxf(s, 0.0f + 1e-7f), 1.0f + 1e-7f);
      } else if (mode == PPO_CARLA_MEAN) {                      /* rl_utils.h:103-105 */
        s = al / (al + be);
      } else if (mode == PPO_CARLA_ROACH) {                     /* rl_utils.h:109-129 */
        if (al > 1.0f && be > 1.0f) s = (al - 1.0f) / (al + be - 2.0f);
        else if (al <= 1.0f && be > 1.0f) s = 0.0f;
        else if (al > 1.0f && be <= 1.0f) s = 1.0f;
        else s = al / (al + be);
      } else {                                                  /* Dirichlet sample, Philox contract */
        const float ga = gamma_mt(al, seed, rank, env, step_id, 0x10000u + (uint32_t)(a * 2 + 0) * 64u);
        const float gb = gamma_mt(be, seed, rank, env, step_id, 0x10000u + (uint32_t)(a * 2 + 1) * 64u);
        s = ga / (ga + gb);
      }
      const float ab = al + be;
      float l = xlogy_f(al - 1.0f, s) + xlogy_f(be - 1.0f, 1.0f - s);
      l += (float)(lgamma((double)ab) - (lgamma((double)al) + lgamma((double)be)));
      lp += l;
      ent += lgamma((double)al) + lgamma((double)be) - lgamma((double)ab) - (2.0 - ab) * orc_digamma(ab) -
             ((al - 1.0) * orc_digamma(al) + (be - 1.0) * orc_digamma(be));
      if (action) action[(long)r * A + a] = (s - 0.0f) / (1.0f - 0.0f) * (hi - lo) + lo;  /* unscale (:262-268) */
    }
    if (logprob) logprob[r] = (float)lp;
    if (entropy) entropy[r] = (float)ent;
  }
  free(b0);
  free(b1);
}

/* ------------------------------------------------------------------------------------------ */
/* PPO env wrapper chain over a scripted env (ppo:41-49; stateful_observation.h:56-84,          */
/* stateful_reward.h:55-91, common.h:11-66, gym.h:141-159)                                      */
/* ------------------------------------------------------------------------------------------ */
static float stream_u01(uint32_t stream, uint32_t i) { return orc_u01(orc_mix32(orc_mix32(stream * 0x9E3779B1u) ^ i)); }

typedef struct wrap_state {
  int O, c, ep_len;
  float ep_ret;
  float *om, *ov, ocount;                /* NormalizeObservation: float32 state, count_ = 1e-4 */
  float rmean, rvar, racc, rcount;       /* NormalizeReward: count_ = 1e-8 */
} wrap_state;

/* NormalizeObservation::observation of one env (stateful_observation.h:64-84: update, then
 * (x - mean) / sqrt(var + eps)) and the clamp of ppo:44; mean / var / count are that env's state. */
static void wrap_obs_one(float* om, float* ov, float* ocount, int O, const float* x, float* y) {
  const float batch_count = 1.0f;
  const float tot_count = *ocount + batch_count;
  for (int i = 0; i < O; ++i) {
    const float delta = x[i] - om[i];
    const float new_mean = om[i] + delta * batch_count / tot_count;
    const float m_a = ov[i] * *ocount;
    const float m_b = 0.0f * batch_count;
    const float M2 = m_a + m_b + (delta * delta) * *ocount * batch_count / tot_count;
    om[i] = new_mean;
    ov[i] = M2 / tot_count;
  }
  *ocount = tot_count;
  for (int i = 0; i < O; ++i) {
    float v = (x[i] - om[i]) / sqrtf(ov[i] + 1e-4f);
    y[i] = v < -10.0f ? -10.0f : (v > 10.0f ? 10.0f : v);
  }
}

/* NormalizeReward::step of one env (stateful_reward.h:55-91) and the clamp of ppo:46 */
static float wrap_rew_one(float* rmean, float* rvar, float* racc, float* rcount, float gamma, float r, float te) {
  *racc = *racc * gamma * (1.0f - te) + r;
  const float batch_count = 1.0f;
  const float delta = *racc - *rmean;
  const float tot_count = *rcount + batch_count;
  const float new_mean = *rmean + delta * batch_count / tot_count;
  const float m_a = *rvar * *rcount;
  const float m_b = 0.0f * batch_count;
  const float M2 = m_a + m_b + (delta * delta) * *rcount * batch_count / tot_count;
  *rcount = tot_count;
  *rmean = new_mean;
  *rvar = M2 / tot_count;
  const float rn = r / sqrtf(*rvar + 1e-8f);
  return rn < -10.0f ? -10.0f : (rn > 10.0f ? 10.0f : rn);
}

static void wrap_obs(wrap_state* w, const float* x, float* y) { wrap_obs_one(w->om, w->ov, &w->ocount, w->O, x, y); }

/* The chain behind a vector env (one state per env, ppo:300-354): st is [E*O] obs mean, [E*O] obs
 * var, then [E] each of obs count, reward mean, reward var, return accumulator, reward count.
 * orc_vwrap_reset: the observations of reset_all (stats updated, normalised in place);
 * orc_vwrap_step: one vector-env step in place -- every obs goes through the obs chain; where
 * is_reset[e] != 0 (the step was the env's next-step autoreset, gym.h:141-149) the reward (0) does
 * not pass NormalizeReward, otherwise it does with the termination flag te[e]. */
static void vwrap_ptrs(float* st, int E, int O, float** om, float** ov, float** oc, float** rm, float** rv, float** ra,
                       float** rc) {
  *om = st; *ov = st + (long)E * O; *oc = st + 2L * E * O;
  *rm = *oc + E; *rv = *rm + E; *ra = *rv + E; *rc = *ra + E;
}
void orc_vwrap_init(float* st, int E, int O) {
  float *om, *ov, *oc, *rm, *rv, *ra, *rc;
  vwrap_ptrs(st, E, O, &om, &ov, &oc, &rm, &rv, &ra, &rc);
  for (long k = 0; k < (long)E * O; ++k) { om[k] = 0.0f; ov[k] = 1.0f; }
  for (int e = 0; e < E; ++e) { oc[e] = 1e-4f; rm[e] = 0.0f; rv[e] = 1.0f; ra[e] = 0.0f; rc[e] = 1e-8f; }
}
void orc_vwrap_reset(float* st, int E, int O, float* obs) {
  float *om, *ov, *oc, *rm, *rv, *ra, *rc;
  vwrap_ptrs(st, E, O, &om, &ov, &oc, &rm, &rv, &ra, &rc);
  float y[MAXO];
  for (int e = 0; e < E; ++e) {
    wrap_obs_one(om + (long)e * O, ov + (long)e * O, oc + e, O, obs + (long)e * O, y);
    memcpy(obs + (long)e * O, y, sizeof(float) * O);
  }
}
void orc_vwrap_step(float* st, int E, int O, float gamma, float* obs, float* reward, const float* te,
                    const float* is_reset) {
  float *om, *ov, *oc, *rm, *rv, *ra, *rc;
  vwrap_ptrs(st, E, O, &om, &ov, &oc, &rm, &rv, &ra, &rc);
  float y[MAXO];
  for (int e = 0; e < E; ++e) {
    wrap_obs_one(om + (long)e * O, ov + (long)e * O, oc + e, O, obs + (long)e * O, y);
    memcpy(obs + (long)e * O, y, sizeof(float) * O);
    if (is_reset[e] == 0.0f) reward[e] = wrap_rew_one(rm + e, rv + e, ra + e, rc + e, gamma, reward[e], te ? te[e] : 0.0f);
  }
}

static void script_obs(const wrap_state* w, float* x) {
  for (int i = 0; i < w->O; ++i) {
    const float lo = (float)i - 2.0f, hi = (float)i + 3.0f;
    x[i] = lo + (hi - lo) * stream_u01(30, (uint32_t)(w->c * w->O + i));
  }
}

/* The raw (unwrapped) stream of orc_wrappers_run's scripted env: obs of the initial reset and of
 * every step [(T+1)*O], reward / termination / truncation per step, and is_reset[t] = 1 where step t
 * was a reset (the plain reset at reset_at or the next-step autoreset). Feeds device wrapper tests. */
void orc_wrappers_script(int O, int T, int reset_at, float* raw_obs, float* reward, float* term, float* trunc,
                         float* is_reset) {
  wrap_state w;
  memset(&w, 0, sizeof(w));
  w.O = O;
  script_obs(&w, raw_obs);
  w.c++;
  int autoreset = 0;
  for (int t = 0; t < T; ++t) {
    float* o = raw_obs + (size_t)(t + 1) * O;
    script_obs(&w, o);
    if (t == reset_at || autoreset) {
      w.c++;
      reward[t] = 0.0f; term[t] = 0.0f; trunc[t] = 0.0f; is_reset[t] = 1.0f;
      autoreset = 0;
      continue;
    }
    const int te = (w.c % 29) == 28, tr = (w.c % 61) == 60;
    reward[t] = -1.0f + 5.0f * stream_u01(31, (uint32_t)w.c);
    w.c++;
    term[t] = (float)te; trunc[t] = (float)tr; is_reset[t] = 0.0f;
    autoreset = te || tr;
  }
}

void orc_wrappers_run(int O, int T, int reset_at, float gamma, float* obs, float* reward, float* term, float* trunc,
                      float* info_ret, float* info_len, float* obs_mean, float* obs_var) {
  wrap_state w;
  memset(&w, 0, sizeof(w));
  w.O = O;
  w.om = (float*)calloc((size_t)O, sizeof(float));
  w.ov = (float*)malloc(sizeof(float) * O);
  for (int i = 0; i < O; ++i) w.ov[i] = 1.0f;
  w.ocount = 1e-4f;
  w.rvar = 1.0f;
  w.rcount = 1e-8f;
  float* x = (float*)malloc(sizeof(float) * O);
  /* reset: RecordEpisodeStatistics clears its counters; NormalizeReward keeps its accumulator */
#define WRAP_RESET(dst)                    \
  do {                                     \
    script_obs(&w, x);                     \
    w.c++;                                 \
    w.ep_ret = 0.0f;                       \
    w.ep_len = 0;                          \
    wrap_obs(&w, x, (dst));                \
  } while (0)
  WRAP_RESET(obs);
  int autoreset = 0;
  for (int t = 0; t < T; ++t) {
    float* o = obs + (size_t)(t + 1) * O;
    if (t == reset_at || autoreset) {
      WRAP_RESET(o);
      reward[t] = 0.0f; term[t] = 0.0f; trunc[t] = 0.0f; info_ret[t] = 0.0f; info_len[t] = 0.0f;
      autoreset = 0;
      continue;
    }
    script_obs(&w, x);
    const float r = -1.0f + 5.0f * stream_u01(31, (uint32_t)w.c);
    const int te = (w.c % 29) == 28, tr = (w.c % 61) == 60;
    w.c++;
    w.ep_ret += r;
    w.ep_len += 1;
    info_ret[t] = (te || tr) ? w.ep_ret : 0.0f;
    info_len[t] = (te || tr) ? (float)w.ep_len : 0.0f;
    wrap_obs(&w, x, o);
    reward[t] = wrap_rew_one(&w.rmean, &w.rvar, &w.racc, &w.rcount, gamma, r, (float)te);
    term[t] = (float)te;
    trunc[t] = (float)tr;
    autoreset = te || tr;
  }
#undef WRAP_RESET
  memcpy(obs_mean, w.om, sizeof(float) * O);
  memcpy(obs_var, w.ov, sizeof(float) * O);
  free(w.om); free(w.ov); free(x);
}
