// ppo_carla.hip — the CaRL CNN agent's forward pass (include/ppo_carla.h; reference
// include/carla/carla_model.h:222-318 with the carla_config.h defaults).
//
//  * k_conv: every convolution AND every Linear layer is one implicit GEMM on
//    mfma_f32_16x16x4f32 in the batch-on-lanes layout of the MLP kernels: a wave owns 16 output
//    pixels (flattened over samples and the output plane, so a Linear layer — a 1x1 "conv" on a
//    1x1 plane — tiles over samples) x 16·NOT output channels. The im2col offsets of the K = IC·k·k
//    reduction are a per-workgroup LDS table, so a B operand is one gathered load per lane and
//    k-step; A operands (weights [OC][IC·k·k]) stream from L2. The uint8 image is converted
//    (x / 255, carla_model.h:214-216) inside the first convolution's gather.
//  * Concatenations are strides: conv6 and state_linear.2 write the two halves of the [n, 1280]
//    linear input, linear.2 writes the first 256 columns of the [n, 256 + NV] value-head input.
//  * k_carla_head: dist_mu / dist_sigma dot products, softplus + beta_min, the Beta sample (the
//    Philox / Marsaglia-Tsang contract of the MLP agents), mean, roach_deterministic or the given
//    action, log_prob and entropy (rl_utils.h:87-132), one thread per row.
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/ppo_carla.h"
#include "../../include/ppo_hip.h"
#include "ppo_agent.hpp"
#include "ppo_kernels.hpp"

namespace {

struct ConvArgs {
  const float* in_f;
  const uint8_t* in_u8;
  long in_stride;  // elements per sample
  int IC, IH, IW;
  const float* W;  // [OC][IC * K * K]
  const float* b;
  float* out;
  long out_stride;  // elements per sample
  int OC, OH, OW;
  int K, S, relu;
  int n;
};

constexpr int kConvWaves = 4;
constexpr int kMaxKTab = 2048;  // im2col offset table entries (IC * K * K <= 1280 here)

// a wave: NP tiles of 16 output pixels x NOT tiles of 16 output channels
template <int NOT, int NP>
__global__ __launch_bounds__(256) void k_conv(ConvArgs a) {
  __shared__ int koff[kMaxKTab];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  const int KK = a.K * a.K, Kt = a.IC * KK, plane = a.IH * a.IW;
  for (int k = tid; k < Kt; k += 256) {
    const int ic = k / KK, rem = k - ic * KK, ky = rem / a.K, kx = rem - ky * a.K;
    koff[k] = ic * plane + ky * a.IW + kx;
  }
  __syncthreads();
  const int P = a.OH * a.OW;
  const long Q = (long)a.n * P;
  const long q0 = ((long)blockIdx.x * kConvWaves + wave) * 16 * NP;
  if (q0 >= Q) return;
  // this lane's output pixels (B-operand column j of each pixel tile)
  long xbase[NP], obase[NP];
  bool qv[NP];
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    const long q = q0 + 16 * u + j;
    qv[u] = q < Q;
    const long s = qv[u] ? q / P : 0;
    const int p = qv[u] ? (int)(q - s * P) : 0, oy = p / a.OW, ox = p - oy * a.OW;
    xbase[u] = s * a.in_stride + (long)oy * a.S * a.IW + (long)ox * a.S;
    obase[u] = s * a.out_stride + p;
  }
  const int oc0 = blockIdx.y * 16 * NOT;
  f4 acc[NOT][NP];
#pragma unroll
  for (int t = 0; t < NOT; ++t)
#pragma unroll
    for (int u = 0; u < NP; ++u) acc[t][u] = f4{0.f, 0.f, 0.f, 0.f};
  const float* wrow[NOT];
  bool ocv[NOT];
#pragma unroll
  for (int t = 0; t < NOT; ++t) {
    const int oc = oc0 + 16 * t + j;
    ocv[t] = oc < a.OC;
    wrow[t] = a.W + (long)(ocv[t] ? oc : 0) * Kt;
  }
#pragma unroll 8
  for (int k0 = 0; k0 < Kt; k0 += 4) {
    const int k = k0 + g;
    const bool kv = k < Kt;
    const int ko = kv ? koff[k] : 0;
    float x[NP], w[NOT];
#pragma unroll
    for (int u = 0; u < NP; ++u) {
      x[u] = 0.f;
      if (kv && qv[u]) x[u] = a.in_u8 ? (float)a.in_u8[xbase[u] + ko] / 255.0f : a.in_f[xbase[u] + ko];
    }
#pragma unroll
    for (int t = 0; t < NOT; ++t) w[t] = (kv && ocv[t]) ? wrow[t][k] : 0.f;
#pragma unroll
    for (int t = 0; t < NOT; ++t)
#pragma unroll
      for (int u = 0; u < NP; ++u) acc[t][u] = mfma16(w[t], x[u], acc[t][u]);
  }
  // lane (j, g) holds out channel oc0 + 16t + 4g + r of pixel q0 + 16u + j
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    if (!qv[u]) continue;
    float* o = a.out + obase[u];
#pragma unroll
    for (int t = 0; t < NOT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int oc = oc0 + 16 * t + 4 * g + r;
        if (oc < a.OC) {
          float y = acc[t][u][r] + a.b[oc];
          if (a.relu) y = y > 0.0f ? y : 0.0f;
          o[(long)oc * P] = y;
        }
      }
  }
}

// value_measurements -> columns [256, 256 + NV) of the value-head input (carla_model.h:276)
__global__ void k_carla_pack(const float* __restrict__ vmeas, float* __restrict__ feat, int n, int NV) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * NV) return;
  const int r = i / NV, c = i - r * NV;
  feat[(long)r * (256 + NV) + 256 + c] = vmeas[i];
}

struct HeadArgs {
  const float* P;
  long mu_w, mu_b, sg_w, sg_b, hi, lo;
  const float* latent;  // [n][256] policy_head output
  const float* val;     // [n]
  int n, A, mode;
  float beta_min;
  const float* action_in;
  uint64_t seed;
  int rank;
  long env_base, step_id;
  float *action, *logprob, *entropy, *value, *alpha, *beta;
};

__global__ __launch_bounds__(64) void k_carla_head(HeadArgs h) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= h.n) return;
  const float* P = h.P;
  const float* x = h.latent + (long)r * 256;
  const float hi = P[h.hi], lo = P[h.lo];
  const SampleKey key = sample_key(h.seed, h.rank);
  const long env = h.env_base + r;
  float lp = 0.f, ent = 0.f;
  for (int ai = 0; ai < h.A; ++ai) {
    const float* wm = P + h.mu_w + (long)ai * 256;
    const float* ws = P + h.sg_w + (long)ai * 256;
    float pm = 0.f, ps = 0.f;
    for (int k = 0; k < 256; ++k) {
      pm = fmaf(wm[k], x[k], pm);
      ps = fmaf(ws[k], x[k], ps);
    }
    pm += P[h.mu_b + ai];
    ps += P[h.sg_b + ai];
    const float al = softplusf_(pm) + h.beta_min, be = softplusf_(ps) + h.beta_min;
    float sv;
    if (h.mode == PPO_CARLA_GIVEN) {
      sv = (h.action_in[(long)r * h.A + ai] - lo) / (hi - lo) * (1.0f - 0.0f) + 0.0f;
      sv = fminf(fmaxf(sv, 0.0f + 1e-7f), 1.0f + 1e-7f);
    } else if (h.mode == PPO_CARLA_MEAN) {
      sv = al / (al + be);
    } else if (h.mode == PPO_CARLA_ROACH) {
      if (al > 1.0f && be > 1.0f) sv = (al - 1.0f) / (al + be - 2.0f);
      else if (al <= 1.0f && be > 1.0f) sv = 0.0f;
      else if (al > 1.0f && be <= 1.0f) sv = 1.0f;
      else sv = al / (al + be);
    } else {
      const float ga = gamma_mt(al, key, env, h.step_id, 0x10000u + (uint32_t)(ai * 2 + 0) * 64u);
      const float gb = gamma_mt(be, key, env, h.step_id, 0x10000u + (uint32_t)(ai * 2 + 1) * 64u);
      sv = ga / (ga + gb);
    }
    const float ab = al + be;
    const float lga = lgammaf(al), lgb = lgammaf(be), lgab = lgammaf(ab);
    lp += xlogyf_(al - 1.0f, sv) + xlogyf_(be - 1.0f, 1.0f - sv) + (lgab - (lga + lgb));
    ent += (lga + lgb) - lgab - (2.0f - ab) * digammaf_(ab) - ((al - 1.0f) * digammaf_(al) + (be - 1.0f) * digammaf_(be));
    if (h.action) h.action[(long)r * h.A + ai] = (sv - 0.0f) / (1.0f - 0.0f) * (hi - lo) + lo;
    if (h.alpha) h.alpha[(long)r * h.A + ai] = al;
    if (h.beta) h.beta[(long)r * h.A + ai] = be;
  }
  if (h.logprob) h.logprob[r] = lp;
  if (h.entropy) h.entropy[r] = ent;
  if (h.value) h.value[r] = h.val[r];
}

int launch_conv(const ConvArgs& a, hipStream_t s) {
  if (a.IC * a.K * a.K > kMaxKTab) return -1;
  const long Q = (long)a.n * a.OH * a.OW;
  // several pixel tiles per wave where there are pixels to spare (B-operand reuse of every weight
  // load), one where the layer is narrow (Linear layers, the last convolutions)
  const int np = Q >= 16L * 4 * 2048 ? 4 : 1;
  const unsigned gx = (unsigned)((Q + 16 * kConvWaves * np - 1) / (16 * kConvWaves * np));
  if (a.OC >= 64) {
    if (np == 4) hipLaunchKernelGGL((k_conv<4, 4>), dim3(gx, (a.OC + 63) / 64), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_conv<4, 1>), dim3(gx, (a.OC + 63) / 64), dim3(256), 0, s, a);
  } else if (a.OC >= 32) {
    if (np == 4) hipLaunchKernelGGL((k_conv<2, 4>), dim3(gx, (a.OC + 31) / 32), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_conv<2, 1>), dim3(gx, (a.OC + 31) / 32), dim3(256), 0, s, a);
  } else {
    if (np == 4) hipLaunchKernelGGL((k_conv<1, 4>), dim3(gx, (a.OC + 15) / 16), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_conv<1, 1>), dim3(gx, (a.OC + 15) / 16), dim3(256), 0, s, a);
  }
  return 0;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// C-ABI
// ------------------------------------------------------------------------------------------
struct ppo_carla {
  ppo_carla_config cfg;
  ppo_carla_layout L;
  int device = 0;
  hipStream_t stream = nullptr;
  float* P = nullptr;
  float* act[PPO_CARLA_NCONV - 1] = {};  // conv1..conv5 outputs
  float *enc = nullptr, *s1 = nullptr, *l1 = nullptr, *feat = nullptr, *v1 = nullptr, *v2 = nullptr, *val = nullptr;
  float *p1 = nullptr, *p2 = nullptr;
};

static int carla_alloc(float** p, size_t n) {
  if (hipMalloc((void**)p, (n ? n : 1) * sizeof(float)) != hipSuccess) return -2;
  return hipMemset(*p, 0, (n ? n : 1) * sizeof(float)) == hipSuccess ? 0 : -2;
}

extern "C" int ppo_carla_destroy(ppo_carla_t* c) {
  if (!c) return 0;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  float* bufs[] = {c->P, c->enc, c->s1, c->l1, c->feat, c->v1, c->v2, c->val, c->p1, c->p2};
  for (float* b : bufs)
    if (b) (void)hipFree(b);
  for (float* b : c->act)
    if (b) (void)hipFree(b);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return 0;
}

extern "C" int ppo_carla_create(const ppo_carla_config* cfg, int device, ppo_carla_t** out) {
  if (!cfg || !out) return ppo_fail("ppo_carla_create: null argument", -1);
  ppo_carla_layout L;
  if (ppo_carla_layout_init(&L, cfg->obs_channels, cfg->bev_h, cfg->bev_w, cfg->num_measurements,
                            cfg->num_value_measurements, cfg->action_dim) != 0)
    return ppo_fail("ppo_carla_create: the roach encoder needs a bev that ends at 256 x 2 x 2 (n_flatten = 1024, "
                    "carla_model.h:110)", -1);
  if (cfg->max_batch <= 0) return ppo_fail("ppo_carla_create: max_batch must be positive", -1);
  if ((long)L.C * L.conv_k[0] * L.conv_k[0] > kMaxKTab || 1280 > kMaxKTab)
    return ppo_fail("ppo_carla_create: too many input channels", -1);
  if (hipSetDevice(device) != hipSuccess) return ppo_fail("ppo_carla_create: hipSetDevice failed", -2);
  ppo_carla_t* c = new ppo_carla_t();
  c->cfg = *cfg;
  c->L = L;
  c->device = device;
  int rc = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess ? 0 : -2;
  const size_t B = (size_t)cfg->max_batch;
  rc |= carla_alloc(&c->P, L.P);
  for (int i = 0; i < PPO_CARLA_NCONV - 1; ++i)
    rc |= carla_alloc(&c->act[i], B * L.conv_oc[i] * L.conv_oh[i] * L.conv_ow[i]);
  rc |= carla_alloc(&c->enc, B * 1280);
  rc |= carla_alloc(&c->s1, B * 256);
  rc |= carla_alloc(&c->l1, B * 512);
  rc |= carla_alloc(&c->feat, B * (256 + L.NV));
  rc |= carla_alloc(&c->v1, B * 256);
  rc |= carla_alloc(&c->v2, B * 256);
  rc |= carla_alloc(&c->val, B);
  rc |= carla_alloc(&c->p1, B * 256);
  rc |= carla_alloc(&c->p2, B * 256);
  if (rc || hipDeviceSynchronize() != hipSuccess) {
    ppo_carla_destroy(c);
    return ppo_fail("ppo_carla_create: device allocation failed", -2);
  }
  *out = c;
  return 0;
}

extern "C" int ppo_carla_get_layout(const ppo_carla_t* c, ppo_carla_layout* out) {
  if (!c || !out) return ppo_fail("ppo_carla_get_layout: null argument", -1);
  *out = c->L;
  return 0;
}

extern "C" int ppo_carla_load_params(ppo_carla_t* c, const float* host, long n) {
  if (!c || !host) return ppo_fail("ppo_carla_load_params: null argument", -1);
  if (n != c->L.P) return ppo_fail("ppo_carla_load_params: expected " + std::to_string(c->L.P) + " floats", -1);
  if (hipSetDevice(c->device) != hipSuccess ||
      hipMemcpyAsync(c->P, host, sizeof(float) * n, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    return ppo_fail("ppo_carla_load_params: copy failed", -2);
  return 0;
}

extern "C" int ppo_carla_forward(ppo_carla_t* c, int n, const uint8_t* bev, const float* meas, const float* vmeas,
                                 int sample_type, const float* action_in, long env_base, long step_id, float* action,
                                 float* logprob, float* entropy, float* value, float* alpha, float* beta,
                                 void* stream) {
  if (!c || !bev || !meas || (!vmeas && c->L.NV > 0)) return ppo_fail("ppo_carla_forward: null argument", -1);
  if (n <= 0) return 0;
  if (n > c->cfg.max_batch) return ppo_fail("ppo_carla_forward: n exceeds max_batch", -1);
  if (sample_type < PPO_CARLA_SAMPLE || sample_type > PPO_CARLA_ROACH)
    return ppo_fail("Unsupported sample type used. Sample type: " + std::to_string(sample_type), -1);
  if (sample_type == PPO_CARLA_GIVEN && !action_in) return ppo_fail("ppo_carla_forward: GIVEN needs action_in", -1);
  const ppo_carla_layout& L = c->L;
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  const float* P = c->P;
  auto conv = [&](const float* in_f, const uint8_t* in_u8, long in_stride, int IC, int IH, int IW, long w, long b,
                  float* out, long out_stride, int OC, int OH, int OW, int K, int S, int relu) {
    ConvArgs a{in_f, in_u8, in_stride, IC, IH, IW, P + w, P + b, out, out_stride, OC, OH, OW, K, S, relu, n};
    return launch_conv(a, s);
  };
  auto linear = [&](const float* in, long in_stride, int IN, long w, long b, float* out, long out_stride, int OUT,
                    int relu) { return conv(in, nullptr, in_stride, IN, 1, 1, w, b, out, out_stride, OUT, 1, 1, 1, 1, relu); };
  int rc = 0;
  // cnn (carla_model.h:66-78, :236): conv1 reads the uint8 image, conv6 writes linear-input columns 0..1023
  const uint8_t* img = bev;
  const float* cur = nullptr;
  long cur_stride = (long)L.C * L.IH * L.IW;
  for (int i = 0; i < PPO_CARLA_NCONV; ++i) {
    const bool last = i == PPO_CARLA_NCONV - 1;
    float* out = last ? c->enc : c->act[i];
    const long out_stride = last ? 1280 : (long)L.conv_oc[i] * L.conv_oh[i] * L.conv_ow[i];
    rc |= conv(cur, img, cur_stride, L.conv_ic[i], L.conv_ih[i], L.conv_iw[i], L.conv_w[i], L.conv_b[i], out,
               out_stride, L.conv_oc[i], L.conv_oh[i], L.conv_ow[i], L.conv_k[i], L.conv_s[i], 1);
    img = nullptr;
    cur = out;
    cur_stride = out_stride;
  }
  // state_linear (:238) -> columns 1024..1279; linear (:240) -> features = value-head input columns 0..255
  const long FW = 256 + L.NV;
  rc |= linear(meas, L.NM, L.NM, L.st_w[0], L.st_b[0], c->s1, 256, 256, 1);
  rc |= linear(c->s1, 256, 256, L.st_w[1], L.st_b[1], c->enc + 1024, 1280, 256, 1);
  rc |= linear(c->enc, 1280, 1280, L.lin_w[0], L.lin_b[0], c->l1, 512, 512, 1);
  rc |= linear(c->l1, 512, 512, L.lin_w[1], L.lin_b[1], c->feat, FW, 256, 1);
  if (L.NV > 0)
    hipLaunchKernelGGL(k_carla_pack, dim3((n * L.NV + 255) / 256), dim3(256), 0, s, vmeas, c->feat, n, L.NV);
  // value_head on [features | value_measurements] (:276-277), policy_head on features (:279)
  rc |= linear(c->feat, FW, (int)FW, L.v_w[0], L.v_b[0], c->v1, 256, 256, 1);
  rc |= linear(c->v1, 256, 256, L.v_w[1], L.v_b[1], c->v2, 256, 256, 1);
  rc |= linear(c->v2, 256, 256, L.v_w[2], L.v_b[2], c->val, 1, 1, 0);
  rc |= linear(c->feat, FW, 256, L.pi_w[0], L.pi_b[0], c->p1, 256, 256, 1);
  rc |= linear(c->p1, 256, 256, L.pi_w[1], L.pi_b[1], c->p2, 256, 256, 1);
  if (rc) return ppo_fail("ppo_carla_forward: no convolution kernel for this shape", -1);
  HeadArgs h{P,          L.mu_w, L.mu_b,   L.sg_w,    L.sg_b,    L.hi,    L.lo,
             c->p2,      c->val, n,        L.A,       sample_type, c->cfg.beta_min, action_in,
             c->cfg.seed, c->cfg.rank, env_base, step_id, action, logprob, entropy, value, alpha, beta};
  hipLaunchKernelGGL(k_carla_head, dim3((n + 63) / 64), dim3(64), 0, s, h);
  if (hipGetLastError() != hipSuccess) return ppo_fail("ppo_carla_forward: launch failed", -2);
  return 0;
}
