// ppo_carla.hip — the CaRL CNN agent's forward pass (include/ppo_carla.h; reference
// include/carla/carla_model.h:222-318 with the carla_config.h defaults).
//
//  * k_conv: every convolution AND every Linear layer is one implicit GEMM on
//    mfma_f32_16x16x4f32 in the batch-on-lanes layout of the MLP kernels: a wave owns 16 output
//    pixels (flattened over samples and the output plane, so a Linear layer — a 1x1 "conv" on a
//    1x1 plane — tiles over samples) x 16·NOT output channels. The im2col offsets of the K = IC·k·k
//    reduction are a per-workgroup LDS table, so a B operand is one gathered load per lane and
//    k-step; A operands (weights [OC][IC·k·k]) stream from L2. The uint8 image is converted
//    (x / 255, carla_model.h:214-216, as x * (1/255): within 1 ulp) inside the first convolution's
//    gather.
//  * Concatenations are strides: conv6 and state_linear.2 write the two halves of the [n, 1280]
//    linear input, linear.2 writes the first 256 columns of the [n, 256 + NV] value-head input.
//  * k_carla_head: dist_mu / dist_sigma dot products, softplus + beta_min, the Beta sample (the
//    Philox / Marsaglia-Tsang contract of the MLP agents), mean, roach_deterministic or the given
//    action, log_prob and entropy (rl_utils.h:87-132), one thread per row.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

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
  float* part;  // split-K partial sums [Z][n * OH * OW][OC] (launch_conv sets kc and part)
  int kc;       // k-range per blockIdx.z (0: no split)
  float* wprep = nullptr;  // conv1 packed form (k_conv_img3): its A operands, [kImg3Blocks][4][16][4]
  int bx = 0;              // conv1 packed form: 1 runs its products as split-bf16 MFMAs (k_conv_img3<.., BX>)
  int tiled = 0;           // 1: conv2's shape runs k_conv_t (LDS-staged input patches)
};

constexpr int kConvWaves = 4;
constexpr int kMaxKTab = 2048;  // im2col offset table entries (IC * K * K <= 1280 here)
constexpr int kUK = 4;          // k-steps per loop iteration: their loads are all in flight together

// a wave: NP tiles of 16 output pixels x NOT tiles of 16 output channels
// Loads are unconditional from clamped addresses and masked with selects afterwards: a load under a
// per-lane branch is followed by its own s_waitcnt, which serialises the gather latency.
// The 4 waves of a workgroup share the output channels, so the weight tile of each 16-wide k group
// (16 NOT channels x 16 k) is loaded once per workgroup — coalesced, one float4 per thread and
// channel quarter — and staged in LDS in A-operand order: lane (j, g) of tile t reads its four
// k-steps as one ds_read_b128 (the per-wave scalar weight gathers read 16 rows x 16 B per
// instruction, 4 times over). Double-buffered, one barrier per k group; same operands and MFMA
// chain as before, so results are unchanged bit for bit.
template <int NOT, int NP, bool U8>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 4))) void k_conv(ConvArgs a) {
  __shared__ int koff[kMaxKTab + 4 * kUK];
  __shared__ __attribute__((aligned(16))) float wst[2][NOT * 256];  // [buf][t][g][j][st]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  const int KK = a.K * a.K, Kt = a.IC * KK, plane = a.IH * a.IW;
  for (int k = tid; k < Kt + 4 * kUK; k += 256) {  // padding: the last iteration reads without a branch
    const int ic = k / KK, rem = k - ic * KK, ky = rem / a.K, kx = rem - ky * a.K;
    koff[k] = k < Kt ? ic * plane + ky * a.IW + kx : 0;
  }
  const int P = a.OH * a.OW;
  const long Q = (long)a.n * P;
  // waves past the last pixel stay (masked) for the workgroup's staging and barriers
  const long q0 = ((long)blockIdx.x * kConvWaves + wave) * 16 * NP;
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
  const int kbeg = a.kc ? (int)blockIdx.z * a.kc : 0, kend = a.kc ? min(Kt, kbeg + a.kc) : Kt;
  // staging: thread (o = tid >> 2 + 64 h, c = tid & 3) owns channel oc0 + o, k-steps st = c: k0 + 4 c .. + 3
  const bool vec = (Kt & 3) == 0;  // rows start on 16-byte boundaries (uniform)
  constexpr int NH = (16 * NOT + 63) / 64;
  const int so = tid >> 2, sc = tid & 3;
  f4 wreg[NH];
  auto wload = [&](int k0) {
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int o = so + 64 * h, oc = oc0 + o, k = k0 + 4 * sc;
      const bool ocok = o < 16 * NOT && oc < a.OC;
      const float* row = a.W + (long)(ocok ? oc : 0) * Kt;
      f4 v;
      if (vec) {
        v = *reinterpret_cast<const f4*>(row + min(k, Kt - 4));
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = row[min(k + i, Kt - 1)];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] *= (ocok && k + i < kend) ? 1.0f : 0.0f;
      wreg[h] = v;
    }
  };
  auto wstore = [&](int buf) {
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int o = so + 64 * h;
      if (o < 16 * NOT) {
        const int t = o >> 4, jj = o & 15;
#pragma unroll
        for (int i = 0; i < 4; ++i) wst[buf][((t * 4 + i) * 16 + jj) * 4 + sc] = wreg[h][i];
      }
    }
  };
  wload(kbeg);
  wstore(0);
  __syncthreads();
  int buf = 0;
  for (int k0 = kbeg; k0 < kend; k0 += 4 * kUK, buf ^= 1) {
    const bool more = k0 + 4 * kUK < kend;
    if (more) wload(k0 + 4 * kUK);
    float x[kUK][NP];
#pragma unroll
    for (int st = 0; st < kUK; ++st) {
      const int k = k0 + 4 * st + g;
      const bool kv = k < kend;
      const int ko = koff[k];
#pragma unroll
      for (int u = 0; u < NP; ++u) {
        const bool ok = kv && qv[u];
        const long off = ok ? xbase[u] + ko : 0;
        if constexpr (U8) {
          // unconditional load, masked as an integer; x / 255 as x * (1 / 255) (within 1 ulp of the
          // reference's division: a division sequence serialises the gather behind VCC)
          const int raw = a.in_u8[off];
          x[st][u] = (float)(ok ? raw : 0) * (1.0f / 255.0f);
        } else {
          x[st][u] = a.in_f[off] * (ok ? 1.0f : 0.0f);  // a multiplicative mask keeps the load unconditional
        }
      }
    }
    f4 w[NOT];  // w[t][st] = W[oc0 + 16 t + j][k0 + 4 st + g]
#pragma unroll
    for (int t = 0; t < NOT; ++t) w[t] = *reinterpret_cast<const f4*>(&wst[buf][(t * 64 + lane) * 4]);
#pragma unroll
    for (int st = 0; st < kUK; ++st)
#pragma unroll
      for (int t = 0; t < NOT; ++t)
#pragma unroll
        for (int u = 0; u < NP; ++u) acc[t][u] = mfma16(w[t][st], x[st][u], acc[t][u]);
    if (more) wstore(buf ^ 1);
    __syncthreads();
  }
  // lane (j, g) holds out channel oc0 + 16t + 4g + r of pixel q0 + 16u + j
  if (a.kc) {  // split K: raw partial sums, added in z order by k_conv_fin
#pragma unroll
    for (int u = 0; u < NP; ++u) {
      if (!qv[u]) continue;
      float* o = a.part + ((size_t)blockIdx.z * Q + q0 + 16 * u + j) * a.OC;
#pragma unroll
      for (int t = 0; t < NOT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int oc = oc0 + 16 * t + 4 * g + r;
          if (oc < a.OC) o[oc] = acc[t][u][r];
        }
    }
    return;
  }
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

// ---- conv2's forward from LDS-staged input patches (create option conv_fwd=tiled, the default) ----
// k_conv gathers each B operand from global memory (one load per MFMA for conv2's 16 output
// channels). Here a persistent workgroup walks TY x TX output tiles of one sample and stages the
// tile's input patch (IC x PH x PW, zero outside the plane) in LDS, the next tile's loaded into
// registers while the current one computes. GEMM: rows = oc (A = the weights, in registers for all
// tiles), columns = the tile's pixels (16 per MFMA column tile: one output row segment), k = (tap, ic)
// with k = 4 kk + g -> ic = 4 (kk % (IC / 4)) + g, tap = kk / (IC / 4): a lane's B operand is its
// pixel's patch offset + its ic plane + an IMMEDIATE per kk (ds_read_b32 + MFMA only). Same products as
// k_conv (fp32 MFMA), another k order (tolerance tests).
constexpr int kCtTY = 8, kCtTX = 16;  // conv2: 45 x 45 -> 6 x 3 tiles
template <int IC, int OC, int TY, int TX>
__global__ __launch_bounds__(256, 3) void k_conv_t(ConvArgs a, int tiles_x, int tps, int tiles) {
  constexpr int K = 5, S = 2, PH = (TY - 1) * S + K, PW = (TX - 1) * S + K, PP = PH * PW, NX = IC * PP;
  constexpr int NRT = OC / 16, ICQ = IC / 4, KS = K * K * ICQ, RPW = TY / 4, NSX = (NX + 255) / 256;
  static_assert(OC % 16 == 0 && IC % 4 == 0 && TY % 4 == 0 && TX == 16, "tile shape");
  __shared__ float xp[NX];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  float wa[NRT][KS];  // A operands: W[16 rt + j][ic][tap], k = 4 kk + g
#pragma unroll
  for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int tap = kk / ICQ, ic = 4 * (kk - tap * ICQ) + g, oc = 16 * rt + j;
      wa[rt][kk] = a.W[(oc < a.OC ? oc * IC + ic : 0) * (K * K) + tap] * (oc < a.OC ? 1.0f : 0.0f);
    }
  float bias[NRT][4];
#pragma unroll
  for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[rt][r] = a.b[16 * rt + 4 * g + r];
  const int bb = g * PP + S * RPW * wave * PW + S * j;  // + 4 (kk % ICQ) PP + ky PW + kx + S u PW
  const long plane = (long)a.IH * a.IW;
  const int P = a.OH * a.OW;
  float sx[NSX];
  auto sload = [&](int tile) {
    const int smp = tile / tps, tt = tile - smp * tps, ty = tt / tiles_x, tx = tt - ty * tiles_x;
    const PBuf xb{__builtin_amdgcn_make_buffer_rsrc((void*)(a.in_f + (size_t)smp * a.in_stride), (short)0,
                                                    (int)(a.in_stride * 4), 0x00020000)};
    const int iy0 = S * TY * ty, ix0 = S * TX * tx;
#pragma unroll
    for (int i = 0; i < NSX; ++i) {
      const int e = tid + 256 * i, ic = e / PP, rem = e - ic * PP, r = rem / PW, c = rem - r * PW;
      const int iy = iy0 + r, ix = ix0 + c;
      const bool in = e < NX && iy < a.IH && ix < a.IW;
      const uint32_t off = in ? (uint32_t)(ic * plane + iy * a.IW + ix) * 4u : 0x7ffffff0u;
      sx[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xb.r, off, 0, 0));
    }
  };
  if ((int)blockIdx.x < tiles) sload(blockIdx.x);
  for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
#pragma unroll
    for (int i = 0; i < NSX; ++i)
      if (tid + 256 * i < NX) xp[tid + 256 * i] = sx[i];
    __syncthreads();
    const int smp = tile / tps, tt = tile - smp * tps, ty = tt / tiles_x, tx = tt - ty * tiles_x;
    if (tile + (int)gridDim.x < tiles) sload(tile + gridDim.x);
    f4 acc[NRT][RPW];
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int u = 0; u < RPW; ++u) acc[rt][u] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int tap = kk / ICQ, icq = kk - tap * ICQ, ky = tap / K, kx = tap - ky * K;
      float bv[RPW];
#pragma unroll
      for (int u = 0; u < RPW; ++u) bv[u] = xp[bb + 4 * icq * PP + ky * PW + kx + S * u * PW];
#pragma unroll
      for (int u = 0; u < RPW; ++u)
#pragma unroll
        for (int rt = 0; rt < NRT; ++rt) acc[rt][u] = mfma16(wa[rt][kk], bv[u], acc[rt][u]);
      if (kk % 10 == 9) __builtin_amdgcn_sched_barrier(0);  // bounds the LDS read hoisting (registers)
    }
    __syncthreads();  // every wave is done with the patch before the next one is stored
    // lane (j, g) holds out channel 16 rt + 4 g + r of output pixel (TY ty + RPW wave + u, TX tx + j)
    const PBuf ob{__builtin_amdgcn_make_buffer_rsrc((void*)(a.out + (size_t)smp * a.out_stride), (short)0,
                                                    (int)(a.out_stride * 4), 0x00020000)};
    const int ox = TX * tx + j;
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int u = 0; u < RPW; ++u) {
        const int oy = TY * ty + RPW * wave + u;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int oc = 16 * rt + 4 * g + r;
          const bool in = oy < a.OH && ox < a.OW && oc < a.OC;
          float y = acc[rt][u][r] + bias[rt][r];
          if (a.relu) y = y > 0.0f ? y : 0.0f;
          const uint32_t off = in ? (uint32_t)(oc * P + oy * a.OW + ox) * 4u : 0x7ffffff0u;
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y), ob.r, off, 0, 0);
        }
      }
  }
}

// ---- conv3's forward (IC 16, OC 32): k_conv_t with the two 16-channel row tiles on different waves ---
// 400 k x 32 rows of weights do not fit one wave's registers: wave w keeps row tile w & 1 (100 A
// operands) and takes half of the 8 x 8 output tile's pixels (two MFMA column tiles of 2 rows x 8
// columns). Patch rows PW = 24 floats (two output rows = 16 banks apart) and ic planes of odd length:
// a ds_read_b32 half (lane groups g = 0, 1) hits 32 distinct banks. k = 4 kk + g -> ic = 4 (kk % 4) + g,
// tap = kk / 4. Same products as k_conv (fp32 MFMA), another k order (tolerance tests).
constexpr int kCt2T = 8;  // output tile edge (conv3: 21 x 21 -> 3 x 3 tiles, 77 % used)
template <int IC, int OC>
__global__ __launch_bounds__(256, 2) void k_conv_t2(ConvArgs a, int tiles_x, int tps, int tiles) {
  constexpr int K = 5, S = 2, T = kCt2T, PH = (T - 1) * S + K, PWL = PH, PW = 24, PPA = 457, NXP = IC * PPA;
  constexpr int ICQ = IC / 4, KS = K * K * ICQ, NSX = (NXP + 255) / 256;
  static_assert(IC % 4 == 0 && OC == 32 && PW >= PWL && PPA >= PH * PW && (PPA & 1) && PW % 16 == 8, "shape");
  __shared__ float xp[NXP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  const int rt = wave & 1, ph = wave >> 1;
  float wa[KS];  // A operands: W[16 rt + j][ic][tap], k = 4 kk + g
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    const int tap = kk / ICQ, ic = 4 * (kk - tap * ICQ) + g;
    wa[kk] = a.W[((16 * rt + j) * IC + ic) * (K * K) + tap];
  }
  float bias[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) bias[r] = a.b[16 * rt + 4 * g + r];
  // lane j of column tile u: output pixel (2 (2 ph + u) + (j >> 3), j & 7) of the tile
  const int bb = g * PPA + 2 * (4 * ph + (j >> 3)) * PW + 2 * (j & 7);  // + 4 PW u + 4 (kk % ICQ) PPA + ky PW + kx
  const long plane = (long)a.IH * a.IW;
  const int P = a.OH * a.OW;
  float sx[NSX];
  auto sload = [&](int tile) {
    const int smp = tile / tps, tt = tile - smp * tps, ty = tt / tiles_x, tx = tt - ty * tiles_x;
    const PBuf xb{__builtin_amdgcn_make_buffer_rsrc((void*)(a.in_f + (size_t)smp * a.in_stride), (short)0,
                                                    (int)(a.in_stride * 4), 0x00020000)};
    const int iy0 = S * T * ty, ix0 = S * T * tx;
#pragma unroll
    for (int i = 0; i < NSX; ++i) {
      const int e = tid + 256 * i, ic = e / PPA, rem = e - ic * PPA, r = rem / PW, c = rem - r * PW;
      const int iy = iy0 + r, ix = ix0 + c;
      const bool in = e < NXP && r < PH && c < PWL && iy < a.IH && ix < a.IW;
      const uint32_t off = in ? (uint32_t)(ic * plane + iy * a.IW + ix) * 4u : 0x7ffffff0u;
      sx[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xb.r, off, 0, 0));
    }
  };
  // no register prefetch of the next patch here (the weights take 100 VGPRs): the two workgroups of a
  // CU overlap one's staging with the other's MFMAs
  for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    sload(tile);
#pragma unroll
    for (int i = 0; i < NSX; ++i)
      if (tid + 256 * i < NXP) xp[tid + 256 * i] = sx[i];
    __syncthreads();
    const int smp = tile / tps, tt = tile - smp * tps, ty = tt / tiles_x, tx = tt - ty * tiles_x;
    f4 acc[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int tap = kk / ICQ, icq = kk - tap * ICQ, ky = tap / K, kx = tap - ky * K;
      float bv[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) bv[u] = xp[bb + 4 * PW * u + 4 * icq * PPA + ky * PW + kx];
#pragma unroll
      for (int u = 0; u < 2; ++u) acc[u] = mfma16(wa[kk], bv[u], acc[u]);
      if (kk % 10 == 9) __builtin_amdgcn_sched_barrier(0);  // bounds the LDS read hoisting (registers)
    }
    __syncthreads();  // every wave is done with the patch before the next one is stored
    const PBuf ob{__builtin_amdgcn_make_buffer_rsrc((void*)(a.out + (size_t)smp * a.out_stride), (short)0,
                                                    (int)(a.out_stride * 4), 0x00020000)};
    const int ox = T * tx + (j & 7);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int oy = T * ty + 2 * (2 * ph + u) + (j >> 3);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int oc = 16 * rt + 4 * g + r;
        const bool in = oy < a.OH && ox < a.OW;
        float y = acc[u][r] + bias[r];
        if (a.relu) y = y > 0.0f ? y : 0.0f;
        const uint32_t off = in ? (uint32_t)(oc * P + oy * a.OW + ox) * 4u : 0x7ffffff0u;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y), ob.r, off, 0, 0);
      }
    }
  }
}

// split-K finish: out = relu(sum over z of the partials, in z order, + bias)
__global__ __launch_bounds__(256) void k_conv_fin(ConvArgs a, int Z) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const int P = a.OH * a.OW;
  const long Q = (long)a.n * P;
  if (i >= Q * a.OC) return;
  const long q = i / a.OC;
  const int oc = (int)(i - q * a.OC);
  float v = 0.f;
  for (int z = 0; z < Z; ++z) v += a.part[(size_t)z * Q * a.OC + i];
  float y = v + a.b[oc];
  if (a.relu) y = y > 0.0f ? y : 0.0f;
  const long smp = q / P;
  a.out[smp * a.out_stride + (long)oc * P + (q - smp * P)] = y;
}

// split-K policy, by layer shape only (so every output element sums its k range in the same
// chunks for any batch): few output pixels per sample and a deep reduction — the Linear layers,
// conv5 and conv6 — get 128-wide k chunks. With few rows (the rollout's batches) those layers
// otherwise run a handful of workgroups whose waves each walk the whole reduction as one
// latency-bound load chain.
constexpr int kSplitKC = 128;
static int conv_split_z(int Kt, int P) { return (P <= 16 && Kt >= 256) ? (Kt + kSplitKC - 1) / kSplitKC : 1; }

// ---- the first convolution (uint8 image, OC <= 16): input patch staged in LDS ----------------
// k_conv's gather issues one vector-memory byte load per lane, pixel tile and k-step (with the weight
// loads, 1.25 vector-memory instructions per MFMA), and conv1 — 15 x 25 taps per output pixel, most
// of the network's FLOPs — was bound by that instruction rate. Here a workgroup owns a 16 x 16 tile
// of output pixels of one sample (wave w: output rows 4w .. 4w + 3, lane j: column j): the
// (15 S + K)^2 x IC input patch is staged in LDS as bytes with aligned dword loads (~0.2 per MFMA),
// the weights and the im2col offsets are staged too, and every B operand is a ds_read_u8. The MFMA
// chain, the k order and the operands of every lane are those of k_conv: the outputs are bitwise
// equal (tested).
constexpr int kImgTile = 16;
template <int K, int S>
struct ImgGeo {
  static constexpr int TI = (kImgTile - 1) * S + K;  // input patch edge
  static constexpr int TIP = (TI + 3) & ~3;          // patch row pitch in bytes (whole dwords)
};
static size_t img_lds_bytes(int IC, int K, int S, int OC) {
  const int TI = (kImgTile - 1) * S + K, TIP = (TI + 3) & ~3, Kt = IC * K * K;
  const size_t patch = ((size_t)IC * TI * TIP + 15) & ~(size_t)15;
  return patch + (size_t)OC * (Kt + 64) * 4 + ((size_t)Kt + 64) * 4;
}

template <int K, int S>
__global__ __launch_bounds__(256) void k_conv_img(ConvArgs a) {
  using G = ImgGeo<K, S>;
  constexpr int TI = G::TI, TIP = G::TIP, DW = TIP / 4, UK = 4;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  const int KK = K * K, Kt = a.IC * KK, OC = a.OC;
  const size_t patch = ((size_t)a.IC * TI * TIP + 15) & ~(size_t)15;
  unsigned char* tile = smem;
  const int Ktp = Kt + 64;                                    // weight row pitch: zeros past Kt
  float* wl = reinterpret_cast<float*>(smem + patch);         // [OC][Ktp]
  int* koff = reinterpret_cast<int*>(wl + (size_t)OC * Ktp);  // [Ktp]: patch offset of tap k (0 past Kt)
  const int tiles_x = (a.OW + kImgTile - 1) / kImgTile;
  const int ty = (int)blockIdx.x / tiles_x, tx = (int)blockIdx.x - ty * tiles_x, smp = blockIdx.y;
  const int x0 = tx * kImgTile * S, y0 = ty * kImgTile * S;
  // patch rows: bytes [x0, x0 + TIP) of input rows y0 .. y0 + TI - 1 of every channel. Rows or
  // columns past the image read the next row / channel (or zeros past the buffer): they only reach
  // output pixels outside the image, which are not stored.
  {
    const unsigned char* base = a.in_u8 + (size_t)smp * a.in_stride;
    const size_t left = (size_t)(a.n - smp) * a.in_stride;
    const PBuf ib{__builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0,
                                                    (int)(left < 0xFFFFFFF0u ? left : 0xFFFFFFF0u), 0x00020000)};
    const int plane = a.IH * a.IW, total = a.IC * TI * DW;
    for (int e = tid; e < total; e += 256) {
      const int ic = e / (TI * DW), rem = e - ic * (TI * DW), r = rem / DW, d = rem - r * DW;
      const int off = ic * plane + (y0 + r) * a.IW + x0 + 4 * d;
      const unsigned v = __builtin_amdgcn_raw_buffer_load_b32(ib.r, off, 0, 0);
      *reinterpret_cast<unsigned*>(tile + (ic * TI + r) * TIP + 4 * d) = v;
    }
  }
  for (int e = tid; e < OC * Ktp; e += 256) {
    const int oc = e / Ktp, k = e - oc * Ktp;
    wl[e] = k < Kt ? a.W[oc * Kt + k] : 0.0f;
  }
  for (int k = tid; k < Kt + 64; k += 256) {
    const int ic = k / KK, rem = k - ic * KK, ky = rem / K, kx = rem - ky * K;
    koff[k] = k < Kt ? (ic * TI + ky) * TIP + kx : 0;
  }
  __syncthreads();
  int pix[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) pix[u] = S * (4 * wave + u) * TIP + S * j;
  const float* wrow = wl + (size_t)(j < OC ? j : 0) * Ktp;
  const float wm = j < OC ? 1.0f : 0.0f;
  f4 acc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) acc[u] = f4{0.f, 0.f, 0.f, 0.f};
  // taps past Kt read offset 0 of the patch (a finite value) against a zero weight: the product is
  // +0, as k_conv's masked operands give, so no per-step masks are needed
  for (int k0 = 0; k0 < Kt; k0 += 4 * UK) {
    float x[UK][4], w[UK];
#pragma unroll
    for (int st = 0; st < UK; ++st) {
      const int k = k0 + 4 * st + g;
      const int ko = koff[k];
#pragma unroll
      for (int u = 0; u < 4; ++u) x[st][u] = (float)tile[ko + pix[u]] * (1.0f / 255.0f);
      w[st] = wrow[k] * wm;
    }
#pragma unroll
    for (int st = 0; st < UK; ++st)
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = mfma16(w[st], x[st][u], acc[u]);
  }
  const int P = a.OH * a.OW;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int oy = ty * kImgTile + 4 * wave + u, ox = tx * kImgTile + j;
    if (oy >= a.OH || ox >= a.OW) continue;
    float* o = a.out + (size_t)smp * a.out_stride + (size_t)oy * a.OW + ox;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int oc = 4 * g + r;
      if (oc < OC) {
        float y = acc[u][r] + a.b[oc];
        if (a.relu) y = y > 0.0f ? y : 0.0f;
        o[(size_t)oc * P] = y;
      }
    }
  }
}

// ---- conv1 with OC <= 8: two output columns per MFMA column --------------------------------
// With OC = 8, half of every 16-row A tile of k_conv_img is padding. Here A row oc + 8 dx holds the
// weights of channel oc shifted by dx output columns (S input columns) over an extended tap row
// kx' in [0, K + S): row oc + 8 dx, tap (ic, ky, kx') = W[oc][ic][ky][kx' - S dx] (0 outside the
// kernel), and lane column j of the B tile is output column 2 j, so one MFMA yields 16 output
// columns x 2 for all 8 channels. 15 x 5 x 7 = 525 taps per 32 outputs instead of 375 per 16:
// 31 % fewer MFMAs and LDS reads per output. The f32 MFMA accumulates like a sequential fma chain
// over k, the added taps carry exact zero weights (fma(+0, x >= 0, acc) = acc) and the real taps
// keep k_conv's order, so the outputs stay bitwise equal to k_conv's (tested).
constexpr int kImg2W = 32;  // output columns per workgroup tile
template <int K, int S>
struct Img2Geo {
  static constexpr int TI = (kImgTile - 1) * S + K;  // patch rows
  static constexpr int TW = (kImg2W - 1) * S + K;    // patch columns
  static constexpr int TIP = (TW + 3) & ~3;          // patch row pitch in bytes
  static constexpr int KX = K + S;                   // extended taps per kernel row
};
static size_t img2_lds_bytes(int IC, int K, int S, int OC) {
  const int TI = (kImgTile - 1) * S + K, TW = (kImg2W - 1) * S + K, TIP = (TW + 3) & ~3;
  const int Kt = IC * K * K, Kx = IC * K * (K + S);
  const size_t patch = ((size_t)IC * TI * TIP + 15) & ~(size_t)15;
  return patch + (size_t)OC * Kt * 4 + 2 * ((size_t)Kx + 64) * 4;
}

template <int K, int S>
__global__ __launch_bounds__(256) void k_conv_img2(ConvArgs a) {
  using G = Img2Geo<K, S>;
  constexpr int TI = G::TI, TIP = G::TIP, DW = TIP / 4, UK = 4, KX = G::KX;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  const int KK = K * K, Kt = a.IC * KK, Kx = a.IC * K * KX, OC = a.OC;
  const size_t patch = ((size_t)a.IC * TI * TIP + 15) & ~(size_t)15;
  unsigned char* tile = smem;
  float* wl = reinterpret_cast<float*>(smem + patch);         // [OC][Kt]
  int* poff = reinterpret_cast<int*>(wl + (size_t)OC * Kt);   // [Kx + 64]: patch offset of tap k'
  int* wtap = poff + Kx + 64;                                 // [Kx + 64]: (ic K + ky) K << 8 | kx'
  const int tiles_x = (a.OW + kImg2W - 1) / kImg2W;
  const int ty = (int)blockIdx.x / tiles_x, tx = (int)blockIdx.x - ty * tiles_x, smp = blockIdx.y;
  const int x0 = tx * kImg2W * S, y0 = ty * kImgTile * S;
  {  // the uint8 patch, as k_conv_img (bytes past the image only reach outputs that are not stored)
    const unsigned char* base = a.in_u8 + (size_t)smp * a.in_stride;
    const size_t left = (size_t)(a.n - smp) * a.in_stride;
    const PBuf ib{__builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0,
                                                    (int)(left < 0xFFFFFFF0u ? left : 0xFFFFFFF0u), 0x00020000)};
    const int plane = a.IH * a.IW, total = a.IC * TI * DW;
    for (int e = tid; e < total; e += 256) {
      const int ic = e / (TI * DW), rem = e - ic * (TI * DW), r = rem / DW, d = rem - r * DW;
      const int off = ic * plane + (y0 + r) * a.IW + x0 + 4 * d;
      const unsigned v = __builtin_amdgcn_raw_buffer_load_b32(ib.r, off, 0, 0);
      *reinterpret_cast<unsigned*>(tile + (ic * TI + r) * TIP + 4 * d) = v;
    }
  }
  for (int e = tid; e < OC * Kt; e += 256) wl[e] = a.W[e];
  for (int k = tid; k < Kx + 64; k += 256) {
    const int ic = k / (K * KX), rem = k - ic * (K * KX), ky = rem / KX, kxp = rem - ky * KX;
    const bool in = k < Kx;
    poff[k] = in ? (ic * TI + ky) * TIP + kxp : 0;
    wtap[k] = in ? (((ic * K + ky) * K) << 8) | kxp : 255;  // kx' = 255: no tap (zero weight)
  }
  __syncthreads();
  int pix[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) pix[u] = S * (4 * wave + u) * TIP + 2 * S * j;
  const int aoc = j & 7, adx = j >> 3;  // A row j: channel aoc, shifted by adx output columns
  const bool aok = aoc < OC;
  const float* wrow = wl + (size_t)(aok ? aoc : 0) * Kt;
  f4 acc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) acc[u] = f4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < Kx; k0 += 4 * UK) {
    float x[UK][4], w[UK];
#pragma unroll
    for (int st = 0; st < UK; ++st) {
      const int k = k0 + 4 * st + g;
      const int po = poff[k], wt = wtap[k];
      const int kx = (wt & 255) - S * adx;
      const bool ok = aok && kx >= 0 && kx < K;
      const float wv = wrow[(wt >> 8) + min(max(kx, 0), K - 1)];
      w[st] = ok ? wv : 0.0f;
#pragma unroll
      for (int u = 0; u < 4; ++u) x[st][u] = (float)tile[po + pix[u]] * (1.0f / 255.0f);
    }
#pragma unroll
    for (int st = 0; st < UK; ++st)
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = mfma16(w[st], x[st][u], acc[u]);
  }
  // lane (j, g), register r: channel (4 g + r) & 7 of output column 2 j + ((4 g + r) >> 3)
  const int P = a.OH * a.OW;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int oy = ty * kImgTile + 4 * wave + u;
    if (oy >= a.OH) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ocp = 4 * g + r, oc = ocp & 7, ox = tx * kImg2W + 2 * j + (ocp >> 3);
      if (oc < OC && ox < a.OW) {
        float y = acc[u][r] + a.b[oc];
        if (a.relu) y = y > 0.0f ? y : 0.0f;
        a.out[(size_t)smp * a.out_stride + (size_t)oc * P + (size_t)oy * a.OW + ox] = y;
      }
    }
  }
}

// ---- conv1, packed taps (k_conv_img3; create option conv1=packed) -------------------------------
// k_conv_img2 spends 7.3 VALU and 1.6 LDS instructions per MFMA (SQ counters, profiles/r05/carla):
// every B operand is its own ds_read_u8 + convert + scale, every A operand an index lookup + select.
// Here the taps of one 16-wide MFMA k block are ordered so that lane group g's four k-steps are four
// CONSECUTIVE taps of one kernel row: tap (16 kb + 4 g + st) = extended column kx' = 4 (g & 1) + st of
// kernel row r = 2 kb + (g >> 1) (r = ic K + ky; kx' in [0, 8): k_conv_img2's K + S = 7 columns
// padded to 8 with a zero-weight tap). Then a lane's B operands for the four steps are the four bytes
// of ONE aligned dword of the patch row (ds_read_b32 + v_cvt_f32_ubyte0..3), and its A operands the
// four floats of one 16-byte piece of a pre-arranged weight table (wprep, built by k_conv1_wprep from
// W each call: A row i = oc + 8 dx holds W[oc][ic][ky][kx' - S dx], 0 outside the kernel), read from
// L2 one k block ahead. 38 blocks x 4 steps x 4 row tiles = 608 MFMAs per wave (k_conv_img2: 528) for
// ~8x fewer VALU and 5x fewer LDS instructions. Each product is k_conv's (x = u8 / 255, the same
// weight); only the order of the k chain differs (not bitwise k_conv's; tolerance tests).
constexpr int kImg3KX = 8;  // extended taps per kernel row, padded
constexpr int kConv1Auto = 2;  // the default conv1 form (ppo_carla_create_ex option conv1): packed (measured faster)
// conv1_mfma=auto: the split-bf16 form (bx3). cfg5's 2 048-row update 12.33 -> 10.63 ms, batch-256
// forward 0.69 -> 0.58 ms (profiles/r05/carla_bx/); gradient vs the fp32 torch reference 6.7e-7 rel-L2
// (test_conv1_split_bf16_update_vs_torch)
constexpr int kConv1BxAuto = 1;
// conv_dgrad=auto: the quad form (k_dgrad_q, one GEMM over the four parity classes)
constexpr int kDgradQuadAuto = 1;
// conv_wgrad=auto: the LDS-tiled form (k_wgrad_t)
constexpr int kWgradTiledAuto = 1;
// conv_fwd=auto: the LDS-tiled form (k_conv_t)
constexpr int kConvTiledAuto = 1;
// deep_dgrad=auto: conv6's input gradient as a dense GEMM + col2im
constexpr int kDgradColAuto = 1;
template <int K, int S>
struct Img3Geo {
  static constexpr int TI = (kImgTile - 1) * S + K;          // patch rows
  static constexpr int TW = (kImg2W - 1) * S + K;            // patch columns used by real taps
  static constexpr int TIP = ((2 * S * (kImg2W / 2 - 1) + kImg3KX) + 3) & ~3;  // incl. the padding tap
};
// 16-tap A blocks of the packed table (two kernel rows each), rounded up to an even count: the BX loop
// reads blocks in pairs (2 kk, 2 kk + 1), so an odd IC * K / 2 (e.g. obs_num_channels 1, 5, 9, 13) gets
// a zero block (k_conv1_wprep writes 0 for rows past IC * K; a zero weight adds exactly 0)
__host__ __device__ inline int img3_blocks(int IC, int K) { return (((IC * K + 1) / 2) + 1) & ~1; }
static size_t img3_lds_bytes(int IC, int K, int S) {
  const int TI = (kImgTile - 1) * S + K, TIP = ((2 * S * (kImg2W / 2 - 1) + kImg3KX) + 3) & ~3;
  return ((size_t)IC * TI * TIP + 15) & ~(size_t)15;
}
// wprep[((kb * 4 + g) * 16 + i) * 4 + st] = A[i][tap 16 kb + 4 g + st]
__global__ void k_conv1_wprep(const float* __restrict__ W, float* __restrict__ wp, int IC, int K, int S, int OC,
                              int nblk) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nblk * 256) return;
  const int st = e & 3, i = (e >> 2) & 15, g = (e >> 6) & 3, kb = e >> 8;
  const int r = 2 * kb + (g >> 1), kxp = 4 * (g & 1) + st;
  const int oc = i & 7, dx = i >> 3, kx = kxp - S * dx;
  float w = 0.0f;
  if (oc < OC && r < IC * K && kx >= 0 && kx < K) w = W[((size_t)oc * IC * K + r) * K + kx];  // W[oc][ic][ky][kx]
  wp[e] = w * (1.0f / 255.0f);  // the image's 1 / 255 moves onto the weights: B is the raw byte value
}

// A workgroup walks tiles [t0, t1) (sample-major, 18 per 192 x 192 sample) with the A-operand table
// staged in LDS once (38 KB) and one patch buffer (35 KB), refilled per tile by LDS DMA (one dword a
// lane); two workgroups per CU, so one's patch fetch runs under the other's MFMAs. The k loop issues
// no vector-memory instruction: an A operand in global memory made the compiler wait vmcnt(0) at
// every k block (the ring index is not static), a full L2 round trip per 16 MFMAs.
constexpr int kImg3WG = 512;  // workgroups: two per CU
__host__ __device__ inline size_t img3_patch_bytes(int IC, int K, int S) {
  const int TI = (kImgTile - 1) * S + K, TIP = ((2 * S * (kImg2W / 2 - 1) + kImg3KX) + 3) & ~3;
  return ((size_t)IC * TI * TIP + 1023) & ~(size_t)1023;  // whole 4-wave DMA rounds (1 KB)
}
// BX (conv1_mfma=bx3): the k loop as v_mfma_f32_16x16x32_bf16 over block pairs (2 kk, 2 kk + 1): a
// lane's slots e < 4 are block 2 kk's taps st = e, slots 4 + st block 2 kk + 1's. The byte operands
// are exact bf16 numbers; the weights (fp32, 1/255 folded in) are split into their three pieces as
// they are read (split3_pair), so every product is exact and three 16-cycle MFMAs replace eight
// 32-cycle 16x16x4 f32 ones per row tile.
template <int K, int S, bool BX = false>
__global__ __launch_bounds__(256, 2) void k_conv_img3(ConvArgs a, int tiles, int tpc) {
  using G = Img3Geo<K, S>;
  constexpr int TI = G::TI, TIP = G::TIP, DW = TIP / 4;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  const int nblk = img3_blocks(a.IC, K), nrow = a.IC * K;
  const int pbytes = (int)img3_patch_bytes(a.IC, K, S), ndma = pbytes / 1024;  // DMA instructions per wave
  unsigned char* tile = smem;
  float* wl = reinterpret_cast<float*>(smem + pbytes);  // [nblk][4][16][4]
  const int tiles_x = (a.OW + kImg2W - 1) / kImg2W, tps = tiles_x * ((a.OH + kImgTile - 1) / kImgTile);
  const int t0 = blockIdx.x * tpc, t1 = min(tiles, t0 + tpc);
  if (t0 >= t1) return;
  for (int e = tid; e < nblk * 64; e += 256)
    reinterpret_cast<f4*>(wl)[e] = reinterpret_cast<const f4*>(a.wprep)[e];
  const int plane = a.IH * a.IW, total = a.IC * TI * DW;
  const float* wlane = wl + (g * 16 + j) * 4;  // this lane's piece of an A block
  const int P = a.OH * a.OW;
  int pix[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) pix[u] = S * (4 * wave + u) * TIP + 2 * S * j + 4 * (g & 1);
  // row 2 m + (g >> 1) of a ten-row step: channel (2 m + (g >> 1)) / K of the pair, kernel row % K
  int rowoff[5], rowq[5];
#pragma unroll
  for (int m = 0; m < 5; ++m) {
    const int rr = 2 * m + (g >> 1), q = rr / K, ky = rr - q * K;
    rowq[m] = q;
    rowoff[m] = (q * TI + ky) * TIP;
  }
  for (int t = t0; t < t1; ++t) {
    const int smp = t / tps, tt = t - smp * tps, ty = tt / tiles_x, tx = tt - ty * tiles_x;
    __syncthreads();  // every wave is done with the previous tile's patch
    {  // wave w moves dwords (w ndma + q) 64 + lane of the patch, q < ndma
      const int x0 = tx * kImg2W * S, y0 = ty * kImgTile * S;
      const size_t sb = (size_t)smp * a.in_stride, left = (size_t)a.n * a.in_stride - sb;
      const PBuf ib{__builtin_amdgcn_make_buffer_rsrc((void*)(a.in_u8 + sb), (short)0,
                                                      (int)(left < 0xFFFFFFF0u ? left : 0xFFFFFFF0u), 0x00020000)};
      for (int q = 0; q < ndma; ++q) {
        const int e0 = (wave * ndma + q) * 64, e = e0 + lane;
        const int ic = e / (TI * DW), rem = e - ic * (TI * DW), r = rem / DW, d = rem - r * DW;
        const uint32_t voff = e < total ? (uint32_t)(ic * plane + (y0 + r) * a.IW + x0 + 4 * d) : 0xFFFFFFF0u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ib.r, (__attribute__((address_space(3))) void*)(tile + 4 * e0), 4,
                                                 voff, 0, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    f4 acc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = f4{0.f, 0.f, 0.f, 0.f};
    if constexpr (BX) {
      // ten blocks (four channels) per step: five block pairs whose row offsets are per-lane constants
      for (int c4 = 0; c4 < (nblk + 9) / 10; ++c4) {
#pragma unroll
        for (int h5 = 0; h5 < 5; ++h5) {
          const int kk = 5 * c4 + h5;
          if (2 * kk >= nblk) break;
          unsigned xb[2][4];
          f4 wv[2];
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const int mm = 2 * h5 + t, c2 = 2 * c4 + (mm >= 5 ? 1 : 0), m = mm >= 5 ? mm - 5 : mm;
            const unsigned char* cbase = tile + (size_t)min(2 * c2, a.IC - 1) * TI * TIP;
            const unsigned char* prow =
                (2 * c2 + 1 < a.IC || rowq[m] == 0) ? cbase + rowoff[m] : tile + rowoff[m] % (TI * TIP);
#pragma unroll
            for (int u = 0; u < 4; ++u) xb[t][u] = *reinterpret_cast<const unsigned*>(prow + pix[u]);
            wv[t] = *reinterpret_cast<const f4*>(wlane + (2 * kk + t) * 256);
          }
          u32x4 ah, amd, al;
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            unsigned h, md, l;
            split3_pair(wv[w >> 1][2 * (w & 1)], wv[w >> 1][2 * (w & 1) + 1], h, md, l);
            ah[w] = h; amd[w] = md; al[w] = l;
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            u32x4 b;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
              const unsigned x = xb[w >> 1][u], sh = 16 * (w & 1);
              b[w] = pack_bf16_exact((float)((x >> sh) & 255u), (float)((x >> (sh + 8)) & 255u));
            }
            acc[u] = mfma16bx(al, b, acc[u]);
            acc[u] = mfma16bx(amd, b, acc[u]);
            acc[u] = mfma16bx(ah, b, acc[u]);
          }
        }
      }
    } else
    // Five k blocks = ten kernel rows = two input channels per step: the patch offset of every row is
    // a per-lane constant plus 2 TI TIP per step (rows past the last channel read channel 0: their
    // weights are 0). The operands of block kb + 1 are read from LDS under block kb's MFMAs.
    for (int c2 = 0; c2 < (a.IC + 1) / 2; ++c2) {
      const unsigned char* cbase = tile + (size_t)min(2 * c2, a.IC - 1) * TI * TIP;
#pragma unroll
      for (int m = 0; m < 5; ++m) {
        const int kb = 5 * c2 + m;
        if (kb >= nblk) break;
        const unsigned char* prow = (2 * c2 + 1 < a.IC || rowq[m] == 0) ? cbase + rowoff[m] : tile + rowoff[m] % (TI * TIP);
        unsigned xb[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) xb[u] = *reinterpret_cast<const unsigned*>(prow + pix[u]);
        const f4 wv = *reinterpret_cast<const f4*>(wlane + kb * 256);
#pragma unroll
        for (int st = 0; st < 4; ++st)
#pragma unroll
          for (int u = 0; u < 4; ++u) acc[u] = mfma16(wv[st], (float)((xb[u] >> (8 * st)) & 255u), acc[u]);
      }
    }
    // lane (j, g), register r: channel (4 g + r) & 7 of output column 2 j + ((4 g + r) >> 3) (k_conv_img2's)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int oy = ty * kImgTile + 4 * wave + u;
      if (oy >= a.OH) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ocp = 4 * g + r, oc = ocp & 7, ox = tx * kImg2W + 2 * j + (ocp >> 3);
        if (oc < a.OC && ox < a.OW) {
          float y = acc[u][r] + a.b[oc];
          if (a.relu) y = y > 0.0f ? y : 0.0f;
          a.out[(size_t)smp * a.out_stride + (size_t)oc * P + (size_t)oy * a.OW + ox] = y;
        }
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
  float* hpre;  // [n][2A] dist_mu / dist_sigma pre-activations (training), may be null
};

// A value the compiler may not look through: the per-concentration results (gamma draw, lgamma,
// digamma) are computed by other threads in the fused tail's head (tail_head_rows) and reach the
// combining expressions through LDS; the same barrier here keeps the two paths' fp contraction (a
// producer's final multiply fused into its consumer's add) identical, so they agree bit for bit.
PPO_DEV float opaque_(float x) {
  asm volatile("" : "+v"(x));
  return x;
}

// The Beta head's arithmetic in two pieces shared by k_carla_head (one thread per row) and the fused
// tail (tail_head_rows: the pieces on different threads, exchanged through LDS). Every value that
// crosses from one piece to the other, and every transcendental result, passes opaque_, so both
// paths compile the same expression trees over the same leaves (no contraction into a consumer
// in one path only) and agree bit for bit.
struct BetaConc {
  float conc, draw, lg, dg;  // softplus(pre) + beta_min, its gamma draw (sampling), lgamma, digamma
};
PPO_DEV BetaConc beta_conc(const HeadArgs& h, float pre, SampleKey key, long env, int ai, int side) {
  BetaConc c;
  c.conc = opaque_(opaque_(softplusf_(pre)) + h.beta_min);
  c.draw = h.mode == PPO_CARLA_SAMPLE
               ? opaque_(gamma_mt(c.conc, key, env, h.step_id, 0x10000u + (uint32_t)(ai * 2 + side) * 64u))
               : 0.0f;
  c.lg = opaque_(lgammaf(c.conc));
  c.dg = opaque_(digammaf_(c.conc));
  return c;
}
// action ai of row r: the sample / mean / roach / given value and the action's log-prob and
// entropy terms (carla_head_row adds them over actions in action order); writes action / alpha / beta
PPO_DEV void beta_action(const HeadArgs& h, int r, int ai, const BetaConc& ca, const BetaConc& cb, float& lpt,
                         float& entt) {
  const float* P = h.P;
  const float hi = P[h.hi], lo = P[h.lo];
  const float al = ca.conc, be = cb.conc;
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
    sv = ca.draw / (ca.draw + cb.draw);
  }
  sv = opaque_(sv);
  const float ab = al + be;
  const float lgab = opaque_(lgammaf(ab)), dgab = opaque_(digammaf_(ab));
  const float xa = opaque_(xlogyf_(al - 1.0f, sv)), xb = opaque_(xlogyf_(be - 1.0f, 1.0f - sv));
  lpt = opaque_(xa + xb + (lgab - (ca.lg + cb.lg)));
  entt = opaque_((ca.lg + cb.lg) - lgab - (2.0f - ab) * dgab - ((al - 1.0f) * ca.dg + (be - 1.0f) * cb.dg));
  if (h.action) h.action[(long)r * h.A + ai] = (sv - 0.0f) / (1.0f - 0.0f) * (hi - lo) + lo;
  if (h.alpha) h.alpha[(long)r * h.A + ai] = al;
  if (h.beta) h.beta[(long)r * h.A + ai] = be;
}

// one row of k_carla_head: the dist_mu / dist_sigma dot products (or, with pre != nullptr, their
// values computed by the same loop elsewhere: pre[ai] = mu, pre[A + ai] = sigma pre-activations),
// softplus + beta_min, the sample / mean / roach / given value, log_prob, entropy
PPO_DEV void carla_head_row(const HeadArgs& h, int r, const float* pre, bool copy_value) {
  const float* P = h.P;
  const float* x = h.latent + (long)r * 256;
  const SampleKey key = sample_key(h.seed, h.rank);
  const long env = h.env_base + r;
  float lp = 0.f, ent = 0.f;
  for (int ai = 0; ai < h.A; ++ai) {
    float pm, ps;
    if (pre) {
      pm = pre[ai];
      ps = pre[h.A + ai];
    } else {
      const float* wm = P + h.mu_w + (long)ai * 256;
      const float* ws = P + h.sg_w + (long)ai * 256;
      pm = 0.f;
      ps = 0.f;
      for (int k = 0; k < 256; ++k) {
        pm = fmaf(wm[k], x[k], pm);
        ps = fmaf(ws[k], x[k], ps);
      }
      pm += P[h.mu_b + ai];
      ps += P[h.sg_b + ai];
    }
    if (h.hpre) {
      h.hpre[(long)r * 2 * h.A + ai] = pm;
      h.hpre[(long)r * 2 * h.A + h.A + ai] = ps;
    }
    const BetaConc ca = beta_conc(h, pm, key, env, ai, 0), cb = beta_conc(h, ps, key, env, ai, 1);
    float lpt, entt;
    beta_action(h, r, ai, ca, cb, lpt, entt);
    lp += lpt;
    ent += entt;
  }
  if (h.logprob) h.logprob[r] = lp;
  if (h.entropy) h.entropy[r] = ent;
  if (copy_value && h.value) h.value[r] = h.val[r];
}

__global__ __launch_bounds__(64) void k_carla_head(HeadArgs h) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= h.n) return;
  carla_head_row(h, r, nullptr, true);
}

// ==========================================================================================
// The MLP tail at rollout batch sizes (n <= kTailMaxN): state MLP, linear, value and policy heads
// and the distribution head after the CNN, as stages of ONE kernel (cooperative launch, a grid
// barrier between stages) instead of ~20 launches of k_conv / k_conv_fin / k_carla_pack /
// k_carla_head, whose fixed cost per launch dominated the 32-row forward. Every Linear output is
// bitwise k_conv's: a work item (16 rows x 16 output channels of one layer) is one workgroup, its
// waves run the same MFMA chains over the same 128-wide k chunks (same operands, same step order,
// same masked operands), and the chunk partials are added in z order from 0 as k_conv_fin does
// (one chunk: acc + bias, as k_conv). The head's dot products run one (row, action) per thread with
// k_carla_head's loop; the per-row Beta arithmetic is k_carla_head's.
// ==========================================================================================
constexpr int kTailThreads = 512, kTailMaxZ = 10, kTailMaxLin = 9, kTailMaxStage = 8, kTailMaxN = 64;
constexpr int kTailLdx = 256 + 4;  // LDS row stride of a recomputed layer's output (OC <= 256)
constexpr int kTailPreMaxK = 32;   // widest input of a layer computed inside its consumer's items

struct TailLin {
  const float* in;
  long in_stride;
  int K;
  long w, b;  // parameter offsets: W [OC][K], b [OC]
  float* out;
  long out_stride;
  int OC, relu;
  float* out2;  // optional copy of output column 0 (the value head's last layer -> value), stride 1
};
struct TailArgs {
  const float* P;
  int n;
  ConvArgs c6;  // conv6's split-K partials, finished in stage 0 as k_conv_fin (c6_Z > 1)
  int c6_Z;
  const float* vmeas;  // value measurements -> feat columns [256, 256 + NV) (stage 0)
  float* feat;
  int NV;
  TailLin lin[kTailMaxLin];
  int lin_stage[kTailMaxLin];  // stage of each layer (non-decreasing)
  int nlin, nstage, head_stage;
  HeadArgs h;
  unsigned* bar;       // grid barrier counter (monotonic across launches)
  unsigned bar_base;   // its value when this launch started
  int stage_lo, stage_hi;  // the stages this launch runs (a barrier between consecutive ones)
  int pre_lin, pre_for;    // layer pre_lin (K < 256, stage -1) is computed inside layer pre_for's items
                           // for their rows (LDS), instead of as a stage of its own; -1: none
};

PPO_DEV int tail_z(int K) { return K >= 256 ? (K + kSplitKC - 1) / kSplitKC : 1; }

// one Linear work item: rows s0 .. s0 + 15, output channels oc0 .. oc0 + 15 of layer L
// (in_row0: the row of the batch that L.in's row 0 holds — 0 for a global input, s0 for rows staged in LDS)
PPO_DEV void tail_lin_item(const float* __restrict__ P, const TailLin& L, int n, int s0, int oc0, float* part,
                           int in_row0 = 0) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  const int K = L.K, Z = tail_z(K), kc = Z > 1 ? kSplitKC : K;
  const int oc = oc0 + j, s = s0 + j;
  const float* wrow = P + L.w + (long)(oc < L.OC ? oc : 0) * K;
  const bool sv = s < n;
  const float* xrow = L.in + (long)(sv ? s - in_row0 : 0) * L.in_stride;
  // a chunk is at most 32 k-steps (128 / 4): all 64 operand loads of a lane go out together (one
  // memory latency per chunk), from clamped addresses, masked afterwards (issuing a second chunk's
  // loads before the first chunk's chain, for linear.0's ten chunks on eight waves, measured slower:
  // 236 VGPRs)
  constexpr int NW = kTailThreads / 64, NU = kSplitKC / 4;
  auto load = [&](int z, float (&av)[NU], float (&bv)[NU]) {
    const int kbeg = z * kc, kend = min(K, kbeg + kc);
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int k = kbeg + 4 * u + g;
      // k_conv's staged weight: rows of K % 4 == 0 are read as float4s from min(k, K - 4), so a
      // masked tap past the end holds W[K - 4 + (k & 3)]; other rows clamp to K - 1
      const int kw = (K & 3) == 0 ? (k < K ? k : K - 4 + (k & 3)) : min(k, K - 1);
      av[u] = wrow[kw] * ((oc < L.OC && k < kend) ? 1.0f : 0.0f);
      const bool ok = sv && k < kend;
      bv[u] = (ok ? xrow[min(k, K - 1)] : L.in[0]) * (ok ? 1.0f : 0.0f);
    }
  };
  auto chain = [&](int z, const float (&av)[NU], const float (&bv)[NU]) {
    const int kbeg = z * kc, kend = min(K, kbeg + kc);
    const int nsteps = 4 * ((kend - kbeg + 15) / 16);
    f4 acc = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < NU; ++u)
      if (u < nsteps) acc = mfma16(av[u], bv[u], acc);
    // lane (j, g) holds output channel oc0 + 4 g + r of row s0 + j
#pragma unroll
    for (int r = 0; r < 4; ++r) part[(z * 16 + 4 * g + r) * 17 + j] = acc[r];
  };
  for (int z = wave; z < Z; z += NW) {
    float av[NU], bv[NU];
    load(z, av, bv);
    chain(z, av, bv);
  }
  __syncthreads();
  if (tid < 256) {
    const int ocl = tid >> 4, sl = tid & 15, o = oc0 + ocl, r = s0 + sl;
    if (o < L.OC && r < n) {
      float y;
      if (Z == 1) {
        y = part[ocl * 17 + sl] + P[L.b + o];
      } else {
        float v = 0.f;
        for (int z = 0; z < Z; ++z) v += part[(z * 16 + ocl) * 17 + sl];
        y = v + P[L.b + o];
      }
      if (L.relu) y = y > 0.0f ? y : 0.0f;
      L.out[(long)r * L.out_stride + o] = y;
      if (L.out2 && o == 0) L.out2[r] = y;
    }
  }
  __syncthreads();  // part is reused by the next item
}

// All OC outputs of a one-chunk layer L (K < 256) for rows s0 .. s0 + 15 into LDS xs[16][ldx], with
// tail_lin_item's arithmetic (per 16x16 tile the same MFMA chain over the same masked operands, then
// + bias, relu), so a dependent layer's items can take them as their input without a stage of their
// own (the state MLP's first layer under its second). Optionally also stored to L.out (rows < n).
PPO_DEV void tail_lin_rows_lds(const float* __restrict__ P, const TailLin& L, int n, int s0, float* xs, int ldx,
                               bool store) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  constexpr int NU = kTailPreMaxK / 4;  // u-steps a K <= kTailPreMaxK layer can use (tail_lin_item loads
                                        // kSplitKC / 4 and issues the first nsteps: the same operands)
  const int K = L.K, kend = K;
  const int nsteps = 4 * ((K + 15) / 16);
  const int s = s0 + j;
  const bool sv = s < n;
  const float* xrow = L.in + (long)(sv ? s : 0) * L.in_stride;
#pragma unroll 1
  for (int ot = wave; ot < (L.OC + 15) / 16; ot += kTailThreads / 64) {
    const int oc0 = 16 * ot, oc = oc0 + j;
    const float* wrow = P + L.w + (long)(oc < L.OC ? oc : 0) * K;
    f4 acc = f4{0.f, 0.f, 0.f, 0.f};
    float av[NU], bv[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int k = 4 * u + g;
      const int kw = (K & 3) == 0 ? (k < K ? k : K - 4 + (k & 3)) : min(k, K - 1);
      av[u] = wrow[kw] * ((oc < L.OC && k < kend) ? 1.0f : 0.0f);
      const bool ok = sv && k < kend;
      bv[u] = (ok ? xrow[min(k, K - 1)] : L.in[0]) * (ok ? 1.0f : 0.0f);
    }
#pragma unroll
    for (int u = 0; u < NU; ++u)
      if (u < nsteps) acc = mfma16(av[u], bv[u], acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = oc0 + 4 * g + r;
      if (o < L.OC) {
        float y = acc[r] + P[L.b + o];
        if (L.relu) y = y > 0.0f ? y : 0.0f;
        xs[j * ldx + o] = y;
        if (store && sv) L.out[(long)s * L.out_stride + o] = y;
      }
    }
  }
  __syncthreads();
}

// The tail's Beta head for rows r0 .. r0 + rows - 1 (rows * 2A <= kTailThreads), given the dist_mu /
// dist_sigma pre-activations pre[row][2A]: carla_head_row's arithmetic spread over threads — one per
// (row, concentration) for softplus, the gamma draw, lgamma and digamma of that concentration, one
// per (row, action) for the sample value and the action's log-prob / entropy terms, one per row for
// the sums over actions in action order (lp = (0 + t_0) + t_1 ..., as carla_head_row's loop adds
// them) — so the row's serial chain is one concentration plus one action instead of 2A of each.
PPO_DEV void tail_head_rows(const HeadArgs& h, int r0, int rows, const float* pre, float* hsc) {
  const int tid = threadIdx.x, A = h.A, n = h.n;
  const SampleKey key = sample_key(h.seed, h.rank);
  BetaConc* cs = reinterpret_cast<BetaConc*>(hsc);  // [rows][2A]
  {  // (row, q): q < A the alpha side of action q, q >= A the beta side of action q - A
    const int rl = tid / (2 * A), q = tid - rl * 2 * A, r = r0 + rl;
    if (rl < rows && r < n) {
      const int side = q < A ? 0 : 1, ai = q - side * A;
      const float x = pre[rl * 2 * A + q];
      if (h.hpre) h.hpre[(long)r * 2 * A + q] = x;
      cs[rl * 2 * A + q] = beta_conc(h, x, key, h.env_base + r, ai, side);
    }
  }
  __syncthreads();
  float* terms = hsc + kTailThreads * 4;  // [rows][A][2]: log-prob term, entropy term
  {
    const int rl = tid / A, ai = tid - rl * A, r = r0 + rl;
    if (rl < rows && r < n)
      beta_action(h, r, ai, cs[rl * 2 * A + ai], cs[rl * 2 * A + A + ai], terms[tid * 2], terms[tid * 2 + 1]);
  }
  __syncthreads();
  if (tid < rows && r0 + tid < n) {
    float lp = 0.f, ent = 0.f;
    for (int ai = 0; ai < A; ++ai) {
      lp += terms[(tid * A + ai) * 2 + 0];
      ent += terms[(tid * A + ai) * 2 + 1];
    }
    if (h.logprob) h.logprob[r0 + tid] = lp;
    if (h.entropy) h.entropy[r0 + tid] = ent;
  }
  __syncthreads();
}

__global__ __launch_bounds__(kTailThreads) void k_carla_tail(TailArgs a) {
  __shared__ float part[kTailMaxZ * 16 * 17];
  __shared__ float pre[kTailThreads * 2];
  __shared__ float xs[16 * kTailLdx];            // rows of layer pre_lin, computed inside pre_for's items
  __shared__ float hsc[kTailThreads * 4 + kTailThreads * 2];  // head scratch (tail_head_rows)
  const int tid = threadIdx.x;
  const int rt_n = (a.n + 15) / 16;
  for (int stage = a.stage_lo; stage <= a.stage_hi; ++stage) {
    if (stage > a.stage_lo) grid_barrier(a.bar, a.bar_base + (unsigned)(stage - a.stage_lo) * gridDim.x);
    if (stage == 0) {  // conv6's split-K finish (k_conv_fin) and the value measurements
      const long gt = (long)blockIdx.x * kTailThreads + tid, gs = (long)gridDim.x * kTailThreads;
      if (a.c6_Z > 1) {
        const ConvArgs& c = a.c6;
        const int P6 = c.OH * c.OW;
        const long Q = (long)c.n * P6;
        for (long i = gt; i < Q * c.OC; i += gs) {
          const long q = i / c.OC;
          const int oc = (int)(i - q * c.OC);
          float v = 0.f;
          for (int z = 0; z < a.c6_Z; ++z) v += c.part[(size_t)z * Q * c.OC + i];
          float y = v + c.b[oc];
          if (c.relu) y = y > 0.0f ? y : 0.0f;
          const long smp = q / P6;
          c.out[smp * c.out_stride + (long)oc * P6 + (q - smp * P6)] = y;
        }
      }
      for (long i = gt; i < (long)a.n * a.NV; i += gs) {
        const long r = i / a.NV, cc = i - r * a.NV;
        a.feat[r * (256 + a.NV) + 256 + cc] = a.vmeas[i];
      }
    }
    // Linear work items of this stage, then (head stage) the distribution head
    int nitems = 0;
    for (int l = 0; l < a.nlin; ++l)
      if (a.lin_stage[l] == stage) nitems += rt_n * ((a.lin[l].OC + 15) / 16);
    const int head_wgs = stage == a.head_stage ? (a.n * a.h.A * 2 + kTailThreads - 1) / kTailThreads : 0;
    for (int it = blockIdx.x; it < nitems + head_wgs; it += gridDim.x) {
      if (it < nitems) {
        int rem = it, l = 0;
        for (; l < a.nlin; ++l) {
          if (a.lin_stage[l] != stage) continue;
          const int cnt = rt_n * ((a.lin[l].OC + 15) / 16);
          if (rem < cnt) break;
          rem -= cnt;
        }
        const int rt = rem % rt_n, ot = rem / rt_n;
        TailLin lx = a.lin[l];
        int row0 = 0;
        if (l == a.pre_for) {  // its input rows first, from the one-chunk layer pre_lin (ot 0 also stores them)
          tail_lin_rows_lds(a.P, a.lin[a.pre_lin], a.n, 16 * rt, xs, kTailLdx, ot == 0);
          lx.in = xs;
          lx.in_stride = kTailLdx;
          row0 = 16 * rt;
        }
        tail_lin_item(a.P, lx, a.n, 16 * rt, 16 * ot, part, row0);
      } else {
        // head: thread (row, ai, mu | sigma) runs k_carla_head's dot product loop for its
        // pre-activation; then one thread per row the rest of k_carla_head
        const HeadArgs& h = a.h;
        const int A = h.A, rows = kTailThreads / (2 * A), r0 = (it - nitems) * rows;
        const int rl = tid / (2 * A), q = tid - rl * 2 * A, r = r0 + rl;
        if (rl < rows && r < a.n) {
          const int ai = q < A ? q : q - A;
          const float* wv = a.P + (q < A ? h.mu_w : h.sg_w) + (long)ai * 256;
          const float* x = h.latent + (long)r * 256;
          float p = 0.f;
          for (int k = 0; k < 256; ++k) p = fmaf(wv[k], x[k], p);
          pre[rl * 2 * A + q] = p + a.P[(q < A ? h.mu_b : h.sg_b) + ai];
        }
        __syncthreads();
        tail_head_rows(h, r0, rows, pre, hsc);
      }
    }
  }
}

// fin = false: a split-K layer leaves its partials (k_conv_fin is the caller's, e.g. the fused
// tail's stage 0); *z_out receives the chunk count (1: not split)
int launch_conv(const ConvArgs& a, hipStream_t s, int img = 1, bool fin = true, int* z_out = nullptr) {
  if (z_out) *z_out = 1;
  if (a.IC * a.K * a.K > kMaxKTab) return -1;
  if (img == 2 && a.wprep && a.in_u8 && ((uintptr_t)a.in_u8 & 3) == 0 && a.K == 5 && a.S == 2 && a.OC <= 8 &&
      a.IW % 4 == 0 && a.in_stride % 4 == 0 && a.OH <= 16 * 64 &&
      img3_patch_bytes(a.IC, a.K, a.S) + (size_t)img3_blocks(a.IC, a.K) * 1024 <= 80 * 1024) {
    const int nblk = img3_blocks(a.IC, a.K);
    hipLaunchKernelGGL(k_conv1_wprep, dim3((nblk * 256 + 255) / 256), dim3(256), 0, s, a.W, a.wprep, a.IC, a.K, a.S,
                       a.OC, nblk);
    const int tiles = ((a.OW + kImg2W - 1) / kImg2W) * ((a.OH + kImgTile - 1) / kImgTile) * a.n;
    const int grid = std::min(tiles, kImg3WG), tpc = (tiles + grid - 1) / grid;
    const size_t lds = img3_patch_bytes(a.IC, a.K, a.S) + (size_t)nblk * 256 * sizeof(float);
    // the launch condition caps lds at 80 KB: allow that once for every later context and channel count
    static const bool attr =
        hipFuncSetAttribute((const void*)k_conv_img3<5, 2, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            80 * 1024) == hipSuccess &&
        hipFuncSetAttribute((const void*)k_conv_img3<5, 2, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            80 * 1024) == hipSuccess;
    if (!attr) return -2;
    if (a.bx)
      hipLaunchKernelGGL((k_conv_img3<5, 2, true>), dim3((tiles + tpc - 1) / tpc), dim3(256), lds, s, a, tiles, tpc);
    else
      hipLaunchKernelGGL((k_conv_img3<5, 2, false>), dim3((tiles + tpc - 1) / tpc), dim3(256), lds, s, a, tiles, tpc);
    return hipGetLastError() == hipSuccess ? 0 : -2;
  }
  if (img && a.in_u8 && ((uintptr_t)a.in_u8 & 3) == 0 && a.K == 5 && a.S == 2 && a.OC <= 8 && a.IW % 4 == 0 &&
      a.in_stride % 4 == 0 && a.OH <= 16 * 64 && img2_lds_bytes(a.IC, a.K, a.S, a.OC) <= 64 * 1024) {
    const int tiles = ((a.OW + kImg2W - 1) / kImg2W) * ((a.OH + kImgTile - 1) / kImgTile);
    hipLaunchKernelGGL((k_conv_img2<5, 2>), dim3(tiles, a.n), dim3(256), img2_lds_bytes(a.IC, a.K, a.S, a.OC), s, a);
    return 0;
  }
  if (img && a.in_u8 && ((uintptr_t)a.in_u8 & 3) == 0 && a.K == 5 && a.S == 2 && a.OC <= 16 && a.IW % 4 == 0 &&
      a.in_stride % 4 == 0 &&
      a.OH <= 16 * 64 && img_lds_bytes(a.IC, a.K, a.S, a.OC) <= 64 * 1024) {
    const int tiles = ((a.OW + kImgTile - 1) / kImgTile) * ((a.OH + kImgTile - 1) / kImgTile);
    hipLaunchKernelGGL((k_conv_img<5, 2>), dim3(tiles, a.n), dim3(256), img_lds_bytes(a.IC, a.K, a.S, a.OC), s, a);
    return 0;
  }
  if (img && a.tiled && a.in_f && a.K == 5 && a.S == 2 && a.IC == 8 && a.OC == 16 && a.in_stride < (1L << 29) &&
      a.out_stride < (1L << 29)) {
    const int tiles_x = (a.OW + kCtTX - 1) / kCtTX, tps = tiles_x * ((a.OH + kCtTY - 1) / kCtTY);
    const long tiles = (long)a.n * tps;
    if (tiles < (1L << 31)) {
      const int grid = (int)std::min<long>(tiles, 256L * 3);  // three workgroups per CU (167 VGPRs)
      hipLaunchKernelGGL((k_conv_t<8, 16, kCtTY, kCtTX>), dim3(grid), dim3(256), 0, s, a, tiles_x, tps, (int)tiles);
      return 0;
    }
  }
  if (img && a.tiled && a.in_f && a.K == 5 && a.S == 2 && a.IC == 16 && a.OC == 32 && a.in_stride < (1L << 29) &&
      a.out_stride < (1L << 29)) {
    const int tiles_x = (a.OW + kCt2T - 1) / kCt2T, tps = tiles_x * ((a.OH + kCt2T - 1) / kCt2T);
    const long tiles = (long)a.n * tps;
    if (tiles < (1L << 31)) {
      const int grid = (int)std::min<long>(tiles, 256L * 2);
      hipLaunchKernelGGL((k_conv_t2<16, 32>), dim3(grid), dim3(256), 0, s, a, tiles_x, tps, (int)tiles);
      return 0;
    }
  }
  const long Q = (long)a.n * a.OH * a.OW;
  // several pixel tiles per wave where there are pixels to spare (B-operand reuse of every weight
  // load), one where the layer is narrow (Linear layers, the last convolutions)
  const int np = Q >= 16L * 4 * 1024 ? 4 : 1;
  const unsigned gx = (unsigned)((Q + 16 * kConvWaves * np - 1) / (16 * kConvWaves * np));
  const bool u8 = a.in_u8 != nullptr;
  const int Z = (a.part && !u8) ? conv_split_z(a.IC * a.K * a.K, a.OH * a.OW) : 1;
  ConvArgs b = a;
  b.kc = Z > 1 ? kSplitKC : 0;
#define PPO_CONV_LAUNCH(NOT_, NP_)                                                                          \
  do {                                                                                                     \
    const dim3 grid(gx, (a.OC + 16 * NOT_ - 1) / (16 * NOT_), Z);                                          \
    if (u8) hipLaunchKernelGGL((k_conv<NOT_, NP_, true>), grid, dim3(256), 0, s, b);                        \
    else hipLaunchKernelGGL((k_conv<NOT_, NP_, false>), grid, dim3(256), 0, s, b);                          \
  } while (0)
  if (a.OC >= 64) {
    if (np == 4) PPO_CONV_LAUNCH(4, 4);
    else PPO_CONV_LAUNCH(4, 1);
  } else if (a.OC >= 32) {
    if (np == 4) PPO_CONV_LAUNCH(2, 4);
    else PPO_CONV_LAUNCH(2, 1);
  } else {
    if (np == 4) PPO_CONV_LAUNCH(1, 4);
    else PPO_CONV_LAUNCH(1, 1);
  }
#undef PPO_CONV_LAUNCH
  if (z_out) *z_out = Z;
  if (Z > 1 && fin) hipLaunchKernelGGL(k_conv_fin, dim3((unsigned)((Q * a.OC + 255) / 256)), dim3(256), 0, s, b, Z);
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
  float* hpre = nullptr;  // [B][2A]
  float* ksplit = nullptr;  // split-K partials of the forward's narrow layers (conv_split_z)
  // training state (allocated on the first ppo_carla_update)
  bool train_ready = false;
  float *G = nullptr, *m = nullptr, *v = nullptr;        // [P]
  float* dact[PPO_CARLA_NCONV - 1] = {};                 // d(conv1..conv5 outputs), masked
  float *denc = nullptr, *ds1 = nullptr, *dl1 = nullptr, *dfeat = nullptr, *dv1 = nullptr, *dv2 = nullptr;
  float *dp1 = nullptr, *dp2 = nullptr, *dhead = nullptr, *dval = nullptr;  // dhead [B][2A], dval [B]
  float *lp = nullptr, *ent = nullptr, *rowstat = nullptr;                    // rowstat [B][8]
  float *part = nullptr;                                 // wgrad partials
  size_t part_floats = 0;
  float* small = nullptr;  // scalars, tensor table and norm slices (carla_train_init)
  long step = 0;
  // conv1 / conv2 kernels: 2 packed conv1 taps (k_conv_img3), 1 LDS-staged (k_conv_img2 and the staged
  // wgrad / dgrad kernels), 0 generic (create option conv1=packed|staged|generic; PPO_CARLA_CONV1 in the
  // diagnostic build). The backward's staged kernels run for 1 and 2.
  int conv_img = kConv1Auto;
  // conv1 (raw-byte input) as split-bf16 products on bf16 MFMAs (create option conv1_mfma=bx3|f32):
  // k_wgrad_img2<.., BX> and k_conv_img3<.., BX>
  int c1bx = kConv1BxAuto;
  // conv2's input gradient: 1 k_dgrad_q (quad classes as GEMM columns), 0 k_dgrad_s2 (create option
  // conv_dgrad=quad|staged; both need conv1=staged|packed)
  int dgrad_q = kDgradQuadAuto;
  // conv2's weight gradient: 1 k_wgrad_t (LDS-staged tiles), 0 k_wgrad (create option conv_wgrad=tiled|generic)
  int wgrad_t = kWgradTiledAuto;
  // conv2's forward: 1 k_conv_t (LDS-staged input patches), 0 k_conv (create option conv_fwd=tiled|generic)
  int conv_t = kConvTiledAuto;
  // conv6's input gradient: 1 dense GEMM + col2im (create option deep_dgrad=col|gather)
  int dgrad_col = kDgradColAuto;
  // create option wgrad_group_bytes (tests): the generic fp32 k_wgrad runs its samples in groups whose
  // input stays below this many bytes (0: kWgradFar, the limit of its 32-bit buffer offsets)
  long wgrad_group = 0;
  float *dcol = nullptr, *wt = nullptr, *zbias = nullptr;  // carla_train_init
  float* c1w = nullptr;  // k_conv_img3's A-operand table
  // MLP tail for n <= kTailMaxN: 1 (default) one launch per stage, 0 one cooperative launch (a grid
  // barrier between stages: slower here, a cooperative launch costs more than the launches it
  // saves), 2 one k_conv / k_conv_fin pair per layer
  int tail_mode = 1;
  unsigned* tail_bar = nullptr;  // k_carla_tail's grid barrier counter
  unsigned tail_count = 0;       // arrivals so far (the counter's value between launches)
  // data parallelism (ppo_carla_comm_init): one RCCL communicator, any world >= 1
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1;
};

static int carla_alloc(float** p, size_t n) {
  if (hipMalloc((void**)p, (n ? n : 1) * sizeof(float)) != hipSuccess) return -2;
  return hipMemset(*p, 0, (n ? n : 1) * sizeof(float)) == hipSuccess ? 0 : -2;
}

extern "C" int ppo_carla_destroy(ppo_carla_t* c) {
  if (!c) return 0;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm) (void)ncclCommDestroy(c->comm);
  float* bufs[] = {c->P,    c->enc,  c->s1,  c->l1,  c->feat,  c->v1,  c->v2,      c->val,  c->p1,
                   c->p2,   c->hpre, c->G,   c->m,   c->v,     c->denc, c->ds1,     c->dl1,  c->dfeat,
                   c->dv1,  c->dv2,  c->dp1, c->dp2, c->dhead, c->dval, c->lp,      c->ent,  c->rowstat,
                   c->part, c->small,  c->ksplit, c->c1w, c->dcol, c->wt, c->zbias, reinterpret_cast<float*>(c->tail_bar)};
  for (float* b : bufs)
    if (b) (void)hipFree(b);
  for (float* b : c->act)
    if (b) (void)hipFree(b);
  for (float* b : c->dact)
    if (b) (void)hipFree(b);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return 0;
}

extern "C" int ppo_carla_create(const ppo_carla_config* cfg, int device, ppo_carla_t** out) {
  return ppo_carla_create_ex(cfg, device, nullptr, out);
}

extern "C" int ppo_carla_create_ex(const ppo_carla_config* cfg, int device, const char* options, ppo_carla_t** out) {
  if (!cfg || !out) return ppo_fail("ppo_carla_create: null argument", -1);
  int conv_img = kConv1Auto;
  int tail_mode = 1;
  int c1bx = kConv1BxAuto;
  int dgrad_q = kDgradQuadAuto;
  int wgrad_t = kWgradTiledAuto;
  int conv_t = kConvTiledAuto;
  int dgrad_col = kDgradColAuto;
  long wgrad_group = 0;
  if (options && *options) {  // comma-separated key=value
    std::string rest(options);
    while (!rest.empty()) {
      const size_t cpos = rest.find(',');
      const std::string o = rest.substr(0, cpos);
      rest = cpos == std::string::npos ? std::string() : rest.substr(cpos + 1);
      if (o == "conv1=packed") conv_img = 2;
      else if (o == "conv1=staged") conv_img = 1;
      else if (o == "conv1=generic") conv_img = 0;
      else if (o == "tail=fused") tail_mode = 0;
      else if (o == "tail=staged") tail_mode = 1;
      else if (o == "tail=layers") tail_mode = 2;
      else if (o == "conv1_mfma=bx3") c1bx = 1;
      else if (o == "conv1_mfma=f32") c1bx = 0;
      else if (o == "conv1_mfma=auto") c1bx = kConv1BxAuto;
      else if (o == "conv_dgrad=quad") dgrad_q = 1;
      else if (o == "conv_dgrad=staged") dgrad_q = 0;
      else if (o == "conv_dgrad=auto") dgrad_q = kDgradQuadAuto;
      else if (o == "conv_wgrad=tiled") wgrad_t = 1;
      else if (o == "conv_wgrad=generic") wgrad_t = 0;
      else if (o == "conv_wgrad=auto") wgrad_t = kWgradTiledAuto;
      else if (o == "conv_fwd=tiled") conv_t = 1;
      else if (o == "conv_fwd=generic") conv_t = 0;
      else if (o == "conv_fwd=auto") conv_t = kConvTiledAuto;
      else if (o == "deep_dgrad=col") dgrad_col = 1;
      else if (o == "deep_dgrad=gather") dgrad_col = 0;
      else if (o == "deep_dgrad=auto") dgrad_col = kDgradColAuto;
      else if (o.rfind("wgrad_group_bytes=", 0) == 0 && o.size() > 18 && o.size() <= 28 &&
               o.find_first_not_of("0123456789", 18) == std::string::npos)
        wgrad_group = atol(o.c_str() + 18);
      else return ppo_fail("ppo_carla_create_ex: unknown option " + o, -1);
    }
  }
  if (int rc = ppo_runtime_check()) return rc;
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
  c->conv_img = conv_img;
  c->tail_mode = tail_mode;
  c->c1bx = c1bx;
  c->dgrad_q = dgrad_q;
  c->wgrad_t = wgrad_t;
  c->conv_t = conv_t;
  c->dgrad_col = dgrad_col;
  c->wgrad_group = wgrad_group;
#ifdef PPO_DIAG
  if (const char* e = getenv("PPO_CARLA_CONV1")) c->conv_img = e[0] - '0';
#endif
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
  rc |= carla_alloc(&c->hpre, B * 2 * L.A);
  {  // the largest split-K partial buffer of the forward's layers
    size_t m = 0;
    auto need = [&](int Kt, int P, int OC) {
      const int Z = conv_split_z(Kt, P);
      if (Z > 1) m = std::max(m, (size_t)Z * B * P * OC);
    };
    for (int i = 1; i < PPO_CARLA_NCONV; ++i)
      need(L.conv_ic[i] * L.conv_k[i] * L.conv_k[i], L.conv_oh[i] * L.conv_ow[i], L.conv_oc[i]);
    need(L.NM, 1, 256); need(256, 1, 256); need(1280, 1, 512); need(512, 1, 256);
    need(256 + L.NV, 1, 256); need(256, 1, 256); need(256, 1, 1);
    if (m) rc |= carla_alloc(&c->ksplit, m);
  }
  rc |= carla_alloc(&c->c1w, (size_t)img3_blocks(L.C, L.conv_k[0]) * 256);
  rc |= carla_alloc(reinterpret_cast<float**>(&c->tail_bar), 1);
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
    ConvArgs a{in_f, in_u8, in_stride, IC, IH, IW, P + w, P + b, out, out_stride, OC, OH, OW, K, S, relu, n,
               c->ksplit, 0};
    a.wprep = c->c1w;
    a.bx = c->c1bx;
    a.tiled = c->conv_t;
    return launch_conv(a, s, c->conv_img);
  };
  auto linear = [&](const float* in, long in_stride, int IN, long w, long b, float* out, long out_stride, int OUT,
                    int relu) { return conv(in, nullptr, in_stride, IN, 1, 1, w, b, out, out_stride, OUT, 1, 1, 1, 1, relu); };
  int rc = 0;
  const bool fused_tail = c->tail_mode != 2 && n <= kTailMaxN;
  ConvArgs c6{};
  int c6_Z = 1;
  const long FW = 256 + L.NV;
  // cnn (carla_model.h:66-78, :236): conv1 reads the uint8 image, conv6 writes linear-input columns 0..1023
  const uint8_t* img = bev;
  const float* cur = nullptr;
  long cur_stride = (long)L.C * L.IH * L.IW;
  for (int i = 0; i < PPO_CARLA_NCONV; ++i) {
    const bool last = i == PPO_CARLA_NCONV - 1;
    float* out = last ? c->enc : c->act[i];
    const long out_stride = last ? 1280 : (long)L.conv_oc[i] * L.conv_oh[i] * L.conv_ow[i];
    if (last && fused_tail) {  // conv6's split-K finish moves into the tail's stage 0
      c6 = ConvArgs{cur, nullptr, cur_stride, L.conv_ic[i], L.conv_ih[i], L.conv_iw[i], P + L.conv_w[i],
                    P + L.conv_b[i], out, out_stride, L.conv_oc[i], L.conv_oh[i], L.conv_ow[i], L.conv_k[i],
                    L.conv_s[i], 1, n, c->ksplit, 0};
      rc |= launch_conv(c6, s, c->conv_img, false, &c6_Z);
    } else {
      rc |= conv(cur, img, cur_stride, L.conv_ic[i], L.conv_ih[i], L.conv_iw[i], L.conv_w[i], L.conv_b[i], out,
                 out_stride, L.conv_oc[i], L.conv_oh[i], L.conv_ow[i], L.conv_k[i], L.conv_s[i], 1);
    }
    img = nullptr;
    cur = out;
    cur_stride = out_stride;
  }
  if (fused_tail) {
    if (rc) return ppo_fail("ppo_carla_forward: no convolution kernel for this shape", -1);
    TailArgs ta{};
    ta.P = P;
    ta.n = n;
    ta.c6 = c6;
    ta.c6_Z = c6_Z;
    ta.vmeas = vmeas;
    ta.feat = c->feat;
    ta.NV = L.NV;
    auto lin = [&](int stage, const float* in, long in_stride, int K, long w, long b, float* out, long out_stride,
                   int OC, int relu, float* out2) {
      ta.lin[ta.nlin] = TailLin{in, in_stride, K, w, b, out, out_stride, OC, relu, out2};
      ta.lin_stage[ta.nlin++] = stage;
    };
    // the forward's layers in dependency stages (carla_model.h:238-279)
    // With a narrow measurement vector the state MLP's first layer runs inside its second layer's
    // items (stage 0, beside conv6's finish): one stage fewer
    const int d = L.NM <= kTailPreMaxK ? 1 : 0;
    ta.pre_lin = ta.pre_for = -1;
    if (d) ta.pre_lin = ta.nlin;
    lin(d ? -1 : 0, meas, L.NM, L.NM, L.st_w[0], L.st_b[0], c->s1, 256, 256, 1, nullptr);
    if (d) ta.pre_for = ta.nlin;
    lin(1 - d, c->s1, 256, 256, L.st_w[1], L.st_b[1], c->enc + 1024, 1280, 256, 1, nullptr);
    lin(2 - d, c->enc, 1280, 1280, L.lin_w[0], L.lin_b[0], c->l1, 512, 512, 1, nullptr);
    lin(3 - d, c->l1, 512, 512, L.lin_w[1], L.lin_b[1], c->feat, FW, 256, 1, nullptr);
    lin(4 - d, c->feat, FW, (int)FW, L.v_w[0], L.v_b[0], c->v1, 256, 256, 1, nullptr);
    lin(4 - d, c->feat, FW, 256, L.pi_w[0], L.pi_b[0], c->p1, 256, 256, 1, nullptr);
    lin(5 - d, c->v1, 256, 256, L.v_w[1], L.v_b[1], c->v2, 256, 256, 1, nullptr);
    lin(5 - d, c->p1, 256, 256, L.pi_w[1], L.pi_b[1], c->p2, 256, 256, 1, nullptr);
    lin(6 - d, c->v2, 256, 256, L.v_w[2], L.v_b[2], c->val, 1, 1, 0, value);
    ta.nstage = 7 - d;
    ta.head_stage = 6 - d;
    ta.h = HeadArgs{P,          L.mu_w, L.mu_b,   L.sg_w,    L.sg_b,    L.hi,    L.lo,
                    c->p2,      c->val, n,        L.A,       sample_type, c->cfg.beta_min, action_in,
                    c->cfg.seed, c->cfg.rank, env_base, step_id, action, logprob, entropy, value, alpha, beta,
                    c->hpre};
    ta.bar = c->tail_bar;
    const int rt_n = (n + 15) / 16;
    const unsigned G = (unsigned)(rt_n * 32);  // linear.0's work items (512 / 16 output tiles)
    if (c->tail_mode == 0) {
      ta.stage_lo = 0;
      ta.stage_hi = ta.nstage - 1;
      ta.bar_base = c->tail_count;
      void* args[] = {&ta};
      if (hipLaunchCooperativeKernel((const void*)k_carla_tail, dim3(G), dim3(kTailThreads), args, 0, s) != hipSuccess)
        return ppo_fail("ppo_carla_forward: cooperative launch of the fused tail failed", -2);
      c->tail_count += (unsigned)(ta.nstage - 1) * G;
    } else {
      for (int st = 0; st < ta.nstage; ++st) {
        ta.stage_lo = ta.stage_hi = st;
        hipLaunchKernelGGL(k_carla_tail, dim3(G), dim3(kTailThreads), 0, s, ta);
      }
    }
    if (hipGetLastError() != hipSuccess) return ppo_fail("ppo_carla_forward: launch failed", -2);
    return 0;
  }
  // state_linear (:238) -> columns 1024..1279; linear (:240) -> features = value-head input columns 0..255
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
             c->cfg.seed, c->cfg.rank, env_base, step_id, action, logprob, entropy, value, alpha, beta,
             c->hpre};
  hipLaunchKernelGGL(k_carla_head, dim3((n + 63) / 64), dim3(64), 0, s, h);
  if (hipGetLastError() != hipSuccess) return ppo_fail("ppo_carla_forward: launch failed", -2);
  return 0;
}

// ==========================================================================================
// Training (ac_ppo_carla.cpp:529-620): the loss, backward through every layer, clip_grad_norm_,
// Adam. Every convolution and Linear layer uses two kernels, both MFMA 16x16x4 in the
// batch-on-lanes layout of k_conv:
//  * k_dgrad — gradient w.r.t. the layer input, times the ReLU mask of that input (the previous
//    layer's output): a gather-GEMM over (output channel, tap). A strided convolution's input
//    pixels split into S x S parity classes (blockIdx.z); within a class the contributing taps are
//    a fixed set (ky = py + S*j), so the reduction has no zero-stuffed taps.
//  * k_wgrad — dW = dZ^T · im2col(x) with the bias as an extra all-ones column, split over
//    chunks of output pixels (blockIdx.x); k_wsum adds the chunks in order (deterministic).
// Linear layers are 1x1 convolutions on a 1x1 plane, as in the forward.
// ==========================================================================================
namespace {

struct DgradArgs {
  const float* dz;  // [n][OC][OH*OW], sample stride dz_stride
  long dz_stride;
  const float* W;   // W[oc][w_ic][K][K]
  int w_ic;
  const float* x;   // the layer input (post-ReLU) for the mask, [n][IC][IH*IW]
  long x_stride;
  float* dx;
  long dx_stride;
  int IC, IH, IW, OC, OH, OW, K, S, n, accumulate;
};

constexpr int kMaxDTab = 3072;

template <int NOT, int NP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 4))) void k_dgrad(DgradArgs a) {
  __shared__ int woff[kMaxDTab + 4 * kUK], zoff[kMaxDTab + 4 * kUK];
  __shared__ int dji[kMaxDTab + 4 * kUK];
  __shared__ __attribute__((aligned(16))) float wst[2][NOT * 256];  // staged weights, as in k_conv
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  const int S = a.S, K = a.K, KK = K * K;
  const int py = blockIdx.z / S, px = blockIdx.z - py * S;
  const int nj = (K - py + S - 1) / S, ni = (K - px + S - 1) / S;
  const int OP = a.OH * a.OW, Kt = a.OC * nj * ni;
  for (int k = tid; k < Kt + 4 * kUK; k += 256) {  // padding entries (valid offsets) for the last iteration
    const int oc = k / (nj * ni), rem = k - oc * nj * ni, jj = rem / ni, ii = rem - jj * ni;
    const bool in = k < Kt;
    woff[k] = in ? oc * a.w_ic * KK + (py + S * jj) * K + (px + S * ii) : 0;
    zoff[k] = in ? oc * OP - jj * a.OW - ii : 0;
    dji[k] = in ? (jj << 16) | ii : 0;
  }
  __syncthreads();
  const int H2 = (a.IH - py + S - 1) / S, W2 = (a.IW - px + S - 1) / S, P2 = H2 * W2;
  const long Q = (long)a.n * P2;
  const long q0 = ((long)blockIdx.x * 4 + wave) * 16 * NP;  // waves past Q stay (masked) for the staging
  long zb[NP], sv[NP];
  int pix[NP], iy2v[NP], ix2v[NP];
  bool qv[NP];
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    const long q = q0 + 16 * u + j;
    qv[u] = q < Q;
    const long s = qv[u] ? q / P2 : 0;
    const int p2 = qv[u] ? (int)(q - s * P2) : 0, iy2 = p2 / W2, ix2 = p2 - iy2 * W2;
    sv[u] = s;
    iy2v[u] = iy2;
    ix2v[u] = ix2;
    zb[u] = s * a.dz_stride + (long)iy2 * a.OW + ix2;
    pix[u] = (S * iy2 + py) * a.IW + (S * ix2 + px);
  }
  const int ic0 = blockIdx.y * 16 * NOT;
  f4 acc[NOT][NP];
#pragma unroll
  for (int t = 0; t < NOT; ++t)
#pragma unroll
    for (int u = 0; u < NP; ++u) acc[t][u] = f4{0.f, 0.f, 0.f, 0.f};
  // weight tile of each k group (16 NOT input channels x 16 (oc, tap) entries) gathered once per
  // workgroup into LDS in A-operand order (k_conv's scheme): thread (o, c) loads k0 + 4 c .. + 3
  constexpr int NH = (16 * NOT + 63) / 64;
  const int so = tid >> 2, sc = tid & 3;
  float wreg[NH][4];
  auto wload = [&](int k0) {
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int o = so + 64 * h, ic = ic0 + o;
      const bool icok = o < 16 * NOT && ic < a.IC;
      const float* wr = a.W + (long)(icok ? ic : 0) * KK;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = k0 + 4 * sc + i;
        wreg[h][i] = wr[woff[k]] * ((icok && k < Kt) ? 1.0f : 0.0f);
      }
    }
  };
  auto wstore = [&](int buf) {
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int o = so + 64 * h;
      if (o < 16 * NOT) {
        const int t = o >> 4, jo = o & 15;
#pragma unroll
        for (int i = 0; i < 4; ++i) wst[buf][((t * 4 + i) * 16 + jo) * 4 + sc] = wreg[h][i];
      }
    }
  };
  wload(0);
  wstore(0);
  __syncthreads();
  int buf = 0;
  for (int k0 = 0; k0 < Kt; k0 += 4 * kUK, buf ^= 1) {
    const bool more = k0 + 4 * kUK < Kt;
    if (more) wload(k0 + 4 * kUK);
    float xb[kUK][NP];
#pragma unroll
    for (int st = 0; st < kUK; ++st) {
      const int k = k0 + 4 * st + g;
      const bool kv = k < Kt;
      const int zo = zoff[k], d = dji[k];
      const int jj = d >> 16, ii = d & 0xFFFF;
#pragma unroll
      for (int u = 0; u < NP; ++u) {
        const bool ok =
            kv && qv[u] && (unsigned)(iy2v[u] - jj) < (unsigned)a.OH && (unsigned)(ix2v[u] - ii) < (unsigned)a.OW;
        xb[st][u] = a.dz[ok ? zb[u] + zo : 0] * (ok ? 1.0f : 0.0f);
      }
    }
    f4 wa[NOT];  // wa[t][st] = W[oc(k)][ic0 + 16 t + j][tap(k)], k = k0 + 4 st + g
#pragma unroll
    for (int t = 0; t < NOT; ++t) wa[t] = *reinterpret_cast<const f4*>(&wst[buf][(t * 64 + lane) * 4]);
#pragma unroll
    for (int st = 0; st < kUK; ++st)
#pragma unroll
      for (int t = 0; t < NOT; ++t)
#pragma unroll
        for (int u = 0; u < NP; ++u) acc[t][u] = mfma16(wa[t][st], xb[st][u], acc[t][u]);
    if (more) wstore(buf ^ 1);
    __syncthreads();
  }
  const long plane = (long)a.IH * a.IW;
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    if (!qv[u]) continue;
#pragma unroll
    for (int t = 0; t < NOT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ic = ic0 + 16 * t + 4 * g + r;
        if (ic >= a.IC) continue;
        const float xm = a.x[sv[u] * a.x_stride + ic * plane + pix[u]];
        const float gv = xm > 0.0f ? acc[t][u][r] : 0.0f;
        float* o = a.dx + sv[u] * a.dx_stride + ic * plane + pix[u];
        *o = a.accumulate ? *o + gv : gv;
      }
  }
}

// ---- stride-2 input gradient with the dZ region staged in LDS (conv2: IC 8, OC 16, K 5) --------
// k_dgrad gathers every B operand (a dZ value) from global memory per lane and k-step. Here a
// workgroup owns a 32 x 32 block of input pixels of one sample: the OC x 18 x 18 dZ region those
// pixels read (zero outside the output plane) and the weights are staged in LDS. Wave w takes rows
// 4w .. 4w + 3 of each of the four parity classes (16 x 16 pixels each), so the 9-, 6-, 6- and
// 4-tap classes are spread evenly. Per class the k order (oc, jj, ii), the k-steps and each lane's
// operands are those of k_dgrad: the results are bitwise equal (tested).
constexpr int kDs2Tile = 32;                          // input pixels per block edge
constexpr int kDs2R = kDs2Tile / 2 + 2;               // dZ region edge for K = 5, S = 2
static size_t ds2_lds_bytes(int IC, int OC) {
  return ((size_t)OC * kDs2R * kDs2R + (size_t)OC * IC * 25 + 4 * 2 * (16 * 9 + 16)) * 4;
}

__global__ __launch_bounds__(256) void k_dgrad_s2(DgradArgs a, int tiles_x, int tps) {
  constexpr int K = 5, S = 2, KK = 25, R = kDs2R;
  extern __shared__ __attribute__((aligned(16))) float dsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  const int OC = a.OC, IC = a.IC, OP = a.OH * a.OW;
  float* dzl = dsm;                                // [OC][R][R]
  float* wl = dzl + OC * R * R;                    // W[oc][ic][K][K] of this layer (w_ic == IC)
  int* woff = reinterpret_cast<int*>(wl + OC * IC * KK);  // [4][16 * 9 + 16]
  int* zoff = woff + 4 * (16 * 9 + 16);
  const int smp = blockIdx.x / tps, tt = blockIdx.x - smp * tps, ty = tt / tiles_x, tx = tt - ty * tiles_x;
  const int oy0 = ty * (kDs2Tile / 2) - 2, ox0 = tx * (kDs2Tile / 2) - 2;  // dZ region origin
  {
    const float* dz = a.dz + (size_t)smp * a.dz_stride;
    for (int e = tid; e < OC * R * R; e += 256) {
      const int oc = e / (R * R), rem = e - oc * R * R, r = rem / R, q = rem - r * R;
      const int oy = oy0 + r, ox = ox0 + q;
      const bool in = (unsigned)oy < (unsigned)a.OH && (unsigned)ox < (unsigned)a.OW;
      const float v = dz[in ? (size_t)oc * OP + oy * a.OW + ox : 0];
      dzl[e] = in ? v : 0.0f;
    }
    for (int e = tid; e < OC * IC * KK; e += 256) wl[e] = a.W[e];
    for (int e = tid; e < 4 * (16 * 9 + 16); e += 256) {
      const int c = e / (16 * 9 + 16), k = e - c * (16 * 9 + 16), py = c >> 1, px = c & 1;
      const int nj = (K - py + S - 1) / S, ni = (K - px + S - 1) / S, Kt = OC * nj * ni;
      const int oc = k / (nj * ni), rem = k - oc * nj * ni, jj = rem / ni, ii = rem - jj * ni;
      const bool in = k < Kt;
      woff[e] = in ? oc * IC * KK + (py + S * jj) * K + (px + S * ii) : 0;
      zoff[e] = in ? oc * R * R - jj * R - ii : 0;
    }
  }
  __syncthreads();
  const int icr = j < IC ? j : 0;
  const float wm = j < IC ? 1.0f : 0.0f;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int py = c >> 1, px = c & 1;
    const int nj = (K - py + S - 1) / S, ni = (K - px + S - 1) / S, Kt = OC * nj * ni;
    const int* wo_c = woff + c * (16 * 9 + 16);
    const int* zo_c = zoff + c * (16 * 9 + 16);
    // class-local pixel (ly, lx) = (4 wave + u, j): dZ row ly + 2 - jj, column lx + 2 - ii
    int zb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) zb[u] = (4 * wave + u + 2) * R + j + 2;
    f4 acc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = f4{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < Kt; k0 += 4 * kUK) {
      float xb[kUK][4], wa[kUK];
#pragma unroll
      for (int st = 0; st < kUK; ++st) {
        const int k = k0 + 4 * st + g;
        const bool kv = k < Kt;
        const int wo = wo_c[k], zo = zo_c[k];
#pragma unroll
        for (int u = 0; u < 4; ++u) xb[st][u] = dzl[zb[u] + zo] * (kv ? 1.0f : 0.0f);
        wa[st] = wl[icr * KK + wo] * (kv ? wm : 0.0f);
      }
#pragma unroll
      for (int st = 0; st < kUK; ++st)
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[u] = mfma16(wa[st], xb[st][u], acc[u]);
    }
    const long plane = (long)a.IH * a.IW;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int iy = ty * kDs2Tile + S * (4 * wave + u) + py, ix = tx * kDs2Tile + S * j + px;
      if (iy >= a.IH || ix >= a.IW) continue;
      const long pix = (long)iy * a.IW + ix;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ic = 4 * g + r;
        if (ic >= IC) continue;
        const float xm = a.x[smp * a.x_stride + ic * plane + pix];
        const float gv = xm > 0.0f ? acc[u][r] : 0.0f;
        float* o = a.dx + smp * a.dx_stride + ic * plane + pix;
        *o = a.accumulate ? *o + gv : gv;
      }
    }
  }
}

// ---- conv2's input gradient as ONE GEMM over the four parity classes (create option
// conv_dgrad=quad, the default) --------------------------------------------------------------------
// For S = 2, K = 5 the input pixel (2 qy + py, 2 qx + px) of "quad" (qy, qx) reads dZ at
// (qy - jj, qx - ii), jj, ii < 3, through the tap (py + 2 jj, px + 2 ii), which does not exist when a
// coordinate is 5: all four parity classes of a quad read the SAME 3 x 3 dZ neighbourhood. So the
// classes become columns: rows = quads (16 per MFMA tile), k = (tap, oc) (9 x OC; a class's missing
// taps are zero weights), columns = (class, ic) — 4 x IC = 32 for IC = 8, two full 16-wide tiles,
// where k_dgrad_s2 leaves half of every MFMA's rows on IC = 8's padding to 16. 72 MFMAs per 16 quads
// (k_dgrad_s2: 100 with half the rows idle). A lane's A operand (dZ) is its quad's neighbourhood in
// the LDS-staged dZ region at one base address plus an IMMEDIATE offset per k-step (k = 4 kk + g:
// oc = 4 (kk % (OC / 4)) + g, tap kk / (OC / 4)), so the k loop is ds_read_b32 + MFMA only; the B
// operands (weights, 72 per lane) stay in registers for all tiles of the persistent workgroup. The
// next tile's dZ region is loaded into registers while the current one computes. Epilogue: the
// two px-classes of a quad sit in lanes j and j ^ 8, one exchange gives each lane four consecutive
// input pixels (two 8-byte stores, the ReLU mask read the same way). The sum runs in another order
// than k_dgrad's (tolerance tests, not bitwise).
constexpr int kDqT = 16;          // quads per tile row (32 input pixels)
constexpr int kDqU = 2;           // quad rows per wave: a tile is 4 kDqU x kDqT quads
constexpr int kDqR = kDqT + 2;    // dZ region row length (ii < 3)
template <int IC, int OC>
__global__ __launch_bounds__(256, kDqU == 2 ? 3 : 2) void k_dgrad_q(DgradArgs a, int tiles_x, int tps, int tiles) {
  constexpr int U = kDqU, TQY = 4 * U, RY = TQY + 2;
  constexpr int K = 5, R = kDqR, RR = RY * R, NCT = 4 * IC / 16, OCQ = OC / 4, KS = 9 * OCQ;
  // each oc plane padded to RRP = 16 (mod 32) dwords: lane groups g = 0, 1 (one ds_read_b32 half) read
  // 16 banks apart, conflict-free
  constexpr int RRP = ((RR - 16 + 31) / 32) * 32 + 16;
  constexpr int NST = (OC * RRP + 255) / 256;  // staging runs over the padded layout (linear LDS stores)
  static_assert(IC == 8 && OC % 4 == 0 && RRP >= RR, "the paired-lane epilogue is written for IC = 8");
  __shared__ float dzl[OC * RRP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  const int OP = a.OH * a.OW;
  // B operands: bw[ct][kk] = W[oc][ic][py + 2 jj][px + 2 ii] for column 16 ct + j = (class, ic), k = 4 kk + g
  float bw[NCT][KS];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) {
    const int py = ct, px = j >> 3, ic = j & 7;  // IC = 8: column 16 ct + j = class (ct, j >> 3), channel j & 7
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int tap = kk / OCQ, oc = 4 * (kk - tap * OCQ) + g, ky = py + 2 * (tap / 3), kx = px + 2 * (tap % 3);
      const bool ok = ky < K && kx < K;
      bw[ct][kk] = ky < K ? a.W[((oc * IC + ic) * K + ky) * K + (ok ? kx : 0)] * (ok ? 1.0f : 0.0f) : 0.0f;
    }
  }
  // the lane's A base: dzl[g][4 wave][j]; step kk of row u adds 4 ocq RRP + (u + 2 - jj) R + (2 - ii)
  const int abase = g * RRP + U * wave * R + j;
  float st[NST];
  auto sload = [&](int tile) {
    const int smp = tile / tps, tt = tile - smp * tps, ty = tt / tiles_x, tx = tt - ty * tiles_x;
    const int oy0 = ty * TQY - 2, ox0 = tx * kDqT - 2;
    // a buffer descriptor over the sample's dZ: elements outside the output plane read as 0 through an
    // offset past the buffer (no select after the load, so the loads stay in flight over the tile)
    const PBuf zb{__builtin_amdgcn_make_buffer_rsrc((void*)(a.dz + (size_t)smp * a.dz_stride), (short)0,
                                                    (int)(a.dz_stride * 4), 0x00020000)};
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const int e = tid + 256 * i, oc = e / RRP, rem = e - oc * RRP, r = rem / R, q = rem - r * R;
      const int oy = oy0 + r, ox = ox0 + q;
      const bool in = e < OC * RRP && rem < RR && (unsigned)oy < (unsigned)a.OH && (unsigned)ox < (unsigned)a.OW;
      const uint32_t off = in ? (uint32_t)(oc * OP + oy * a.OW + ox) * 4u : 0x7ffffff0u;
      st[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(zb.r, off, 0, 0));
    }
  };
  if ((int)blockIdx.x < tiles) sload(blockIdx.x);
  const long plane = (long)a.IH * a.IW;
  const int px = j >> 3, icl = j & 7;
  for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const int e = tid + 256 * i;
      if (e < OC * RRP) dzl[e] = st[i];
    }
    __syncthreads();
    const int smp = tile / tps, tt = tile - smp * tps, ty = tt / tiles_x, tx = tt - ty * tiles_x;
    if (tile + (int)gridDim.x < tiles) sload(tile + gridDim.x);
    f4 acc[U][NCT];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) acc[u][ct] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int tap = kk / OCQ, ocq = kk - tap * OCQ, jj = tap / 3, ii = tap % 3;
      float av[U];
#pragma unroll
      for (int u = 0; u < U; ++u) av[u] = dzl[abase + 4 * ocq * RRP + (u + 2 - jj) * R + (2 - ii)];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
          if (ct + 2 * jj < K) acc[u][ct] = mfma16(av[u], bw[ct][kk], acc[u][ct]);  // py = 1 has no jj = 2 taps
      if (kk % 12 == 11) __builtin_amdgcn_sched_barrier(0);  // bounds the LDS read hoisting (registers)
    }
    __syncthreads();  // every wave is done with dzl before the next tile's region is stored
    // lane (j, g) holds, for quad row 4 wave + u and class (py = ct, px = j >> 3), channel j & 7 of the
    // quads 4 g + r; after the exchange with lane j ^ 8 it holds input pixels 8 g + 4 px + 0..3
    // the mask reads and the stores go through buffer descriptors: pixels past the plane read 0 and
    // their stores are dropped (an offset past the buffer), so there is no branch between the loads
    const PBuf xq{__builtin_amdgcn_make_buffer_rsrc((void*)(a.x + (size_t)smp * a.x_stride), (short)0,
                                                    (int)(a.x_stride * 4), 0x00020000)};
    const PBuf dq{__builtin_amdgcn_make_buffer_rsrc((void*)(a.dx + (size_t)smp * a.dx_stride), (short)0,
                                                    (int)(a.dx_stride * 4), 0x00020000)};
    const int ix = 2 * tx * kDqT + 8 * g + 4 * px;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        const f4 v = acc[u][ct];
        const float s0 = px ? v[0] : v[2], s1 = px ? v[1] : v[3];
        const float r0 = __shfl_xor(s0, 8), r1 = __shfl_xor(s1, 8);
        const int iy = 2 * (ty * TQY + U * wave + u) + ct;
        float o[4];
        o[0] = px ? r0 : v[0];
        o[1] = px ? v[2] : r0;
        o[2] = px ? r1 : v[1];
        o[3] = px ? v[3] : r1;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const bool in = iy < a.IH && ix + 2 * h < a.IW;
          const uint32_t off = in ? (uint32_t)(icl * plane + (long)iy * a.IW + ix + 2 * h) * 4u : 0x7ffffff0u;
          // (32-bit accesses; the compiler pairs the mask loads into one dwordx2)
          const float x0 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xq.r, off, 0, 0));
          const float x1 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xq.r, off + 4, 0, 0));
          float g0 = x0 > 0.0f ? o[2 * h] : 0.0f;
          float g1 = x1 > 0.0f ? o[2 * h + 1] : 0.0f;
          if (a.accumulate) {
            g0 += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dq.r, off, 0, 0));
            g1 += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dq.r, off + 4, 0, 0));
          }
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, g0), dq.r, off, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, g1), dq.r, off + 4, 0, 0);
        }
      }
  }
}

// ---- conv3's input gradient (IC 16, OC 32): the quad form with the classes as separate GEMMs --------
// As k_dgrad_q, the four parity classes of a quad read the same 3 x 3 dZ neighbourhood, so one B
// operand (dZ at tap (jj, ii), oc = 4 ocq + g, from the LDS-staged region at a per-lane base plus an
// IMMEDIATE offset) feeds the MFMA of every class that has that tap. Here rows = the 16 input channels
// (full MFMA rows), columns = 16 quads (2 quad rows x 8 quad columns), and the A operands are the
// classes' weights from a table built once per persistent workgroup in LDS ([class k / 4][lane][4]:
// one ds_read_b128 per class and 4 k-steps); the classes' missing taps (py = 1: jj = 2, px = 1: ii = 2)
// are skipped: 200 MFMAs per wave and tile of 8 x 8 quads (conv3: 23 x 23 quads -> 3 x 3 tiles, 92 %
// used). Lane (j, g) ends with input channel 4 g + r of quad j for every class, so the px = 0 / 1
// classes of a row give two adjacent pixels. dZ region rows are 16 floats and oc planes 168 (= 8 mod 32):
// lane groups 0 and 1 read 32 distinct banks. Another sum order than k_dgrad (tolerance tests).
constexpr int kDq2T = 8;  // quads per tile edge
template <int IC, int OC>
__global__ __launch_bounds__(256, 2) void k_dgrad_q2(DgradArgs a, int tiles_x, int tps, int tiles) {
  constexpr int K = 5, R = 16, RU = kDq2T + 2, RRP = 168, OCQ = OC / 4, NTAB = (9 + 6 + 6 + 4) * OCQ * 64;
  constexpr int NST = (OC * RRP + 255) / 256;
  static_assert(IC == 16 && OC % 8 == 0 && RRP >= RU * R && RRP % 32 == 8, "shape");
  extern __shared__ __attribute__((aligned(16))) float dq2[];
  float* tab = dq2;          // [(class base + tap index * OCQ + ocq) / 4][lane][4]
  float* dzl = dq2 + NTAB;   // [OC][RRP]: rows of R
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  // class c = (py, px) = (c >> 1, c & 1): (3 - py) (3 - px) taps; k base (in k-steps) 0, 9, 15, 21 x OCQ
  auto cbase = [](int c) { return (c == 0 ? 0 : c == 1 ? 9 : c == 2 ? 15 : 21) * OCQ; };
  for (int f = tid; f < NTAB; f += 256) {
    const int e = f & 3, ln = (f >> 2) & 63, kc = 4 * (f >> 8) + e;
    const int c = kc < 9 * OCQ ? 0 : kc < 15 * OCQ ? 1 : kc < 21 * OCQ ? 2 : 3, py = c >> 1, px = c & 1;
    const int loc = kc - cbase(c), ti = loc / OCQ, ocq = loc - ti * OCQ, jj = ti / (3 - px), ii = ti - jj * (3 - px);
    const int oc = 4 * ocq + (ln >> 4), ic = ln & 15;
    tab[f] = a.W[((oc * IC + ic) * K + py + 2 * jj) * K + px + 2 * ii];
  }
  const int bbase = g * RRP + (2 * wave + (j >> 3)) * R + (j & 7);  // + 4 ocq RRP + (2 - jj) R + (2 - ii)
  const int OP = a.OH * a.OW;
  float st[NST];
  auto sload = [&](int tile) {
    const int smp = tile / tps, tt = tile - smp * tps, ty = tt / tiles_x, tx = tt - ty * tiles_x;
    const int oy0 = ty * kDq2T - 2, ox0 = tx * kDq2T - 2;
    const PBuf zb{__builtin_amdgcn_make_buffer_rsrc((void*)(a.dz + (size_t)smp * a.dz_stride), (short)0,
                                                    (int)(a.dz_stride * 4), 0x00020000)};
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const int e = tid + 256 * i, oc = e / RRP, rem = e - oc * RRP, r = rem / R, q = rem - r * R;
      const int oy = oy0 + r, ox = ox0 + q;
      const bool in = e < OC * RRP && r < RU && q < RU && (unsigned)oy < (unsigned)a.OH && (unsigned)ox < (unsigned)a.OW;
      const uint32_t off = in ? (uint32_t)(oc * OP + oy * a.OW + ox) * 4u : 0x7ffffff0u;
      st[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(zb.r, off, 0, 0));
    }
  };
  if ((int)blockIdx.x < tiles) sload(blockIdx.x);
  const long plane = (long)a.IH * a.IW;
  for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
#pragma unroll
    for (int i = 0; i < NST; ++i)
      if (tid + 256 * i < OC * RRP) dzl[tid + 256 * i] = st[i];
    __syncthreads();
    const int smp = tile / tps, tt = tile - smp * tps, ty = tt / tiles_x, tx = tt - ty * tiles_x;
    if (tile + (int)gridDim.x < tiles) sload(tile + gridDim.x);
    f4 acc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int jj = t / 3, ii = t % 3;
#pragma unroll
      for (int h = 0; h < OCQ / 4; ++h) {
        f4 wa[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int py = c >> 1, px = c & 1;
          if (jj < 3 - py && ii < 3 - px) {
            const int kk4 = (cbase(c) + (jj * (3 - px) + ii) * OCQ) / 4 + h;
            wa[c] = *reinterpret_cast<const f4*>(&tab[(kk4 * 64 + lane) * 4]);
          }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int ocq = 4 * h + q;
          const float bv = dzl[bbase + 4 * ocq * RRP + (2 - jj) * R + (2 - ii)];
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (jj < 3 - (c >> 1) && ii < 3 - (c & 1)) acc[c] = mfma16(wa[c][q], bv, acc[c]);
        }
      }
    }
    __syncthreads();  // every wave is done with dzl before the next tile's region is stored
    // lane (j, g): channel 4 g + r of quad (2 wave + (j >> 3), j & 7) for class c; px = 0 / 1 adjacent
    const PBuf xq{__builtin_amdgcn_make_buffer_rsrc((void*)(a.x + (size_t)smp * a.x_stride), (short)0,
                                                    (int)(a.x_stride * 4), 0x00020000)};
    const PBuf dq{__builtin_amdgcn_make_buffer_rsrc((void*)(a.dx + (size_t)smp * a.dx_stride), (short)0,
                                                    (int)(a.dx_stride * 4), 0x00020000)};
    const int qy = ty * kDq2T + 2 * wave + (j >> 3), ix = 2 * (tx * kDq2T + (j & 7));
#pragma unroll
    for (int py = 0; py < 2; ++py) {
      const int iy = 2 * qy + py;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ic = 4 * g + r;
#pragma unroll
        for (int px = 0; px < 2; ++px) {
          const bool in = iy < a.IH && ix + px < a.IW;
          const uint32_t off = in ? (uint32_t)(ic * plane + (long)iy * a.IW + ix + px) * 4u : 0x7ffffff0u;
          const float xm = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xq.r, off, 0, 0));
          float gv = xm > 0.0f ? acc[2 * py + px][r] : 0.0f;
          if (a.accumulate) gv += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dq.r, off, 0, 0));
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, gv), dq.r, off, 0, 0);
        }
      }
    }
  }
}
static size_t dq2_lds_bytes(int OC) { return ((size_t)(9 + 6 + 6 + 4) * (OC / 4) * 64 + (size_t)OC * 168) * 4; }

// ---- the last convolution's input gradient as a dense GEMM + col2im (create option deep_dgrad=col) ----
// conv6 (4 x 4 -> 2 x 2, stride 1) has 4 output pixels: k_dgrad's per-pixel tap sets are mostly
// outside the output plane (2.25 of 9 taps valid on average, the rest multiply zeros). Instead dcol[n][(ic, ky, kx)][oy, ox] = sum_oc W[oc][ic, ky, kx] dZ[n][oc][oy, ox]
// is one dense GEMM (k_conv as a 1 x 1 convolution over the OH x OW plane with the transposed weights,
// no zero products), and k_col2im adds each input pixel's (at most K x K) contributions in (ky, kx)
// order and applies the ReLU mask. Another sum order than k_dgrad (tolerance tests).
__global__ void k_wtrans(const float* __restrict__ W, int OC, int Kt, float* __restrict__ Wt) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;  // Wt[k][oc] = W[oc][k]
  if (i >= (long)OC * Kt) return;
  const int k = (int)(i / OC), oc = (int)(i - (long)k * OC);
  Wt[i] = W[(long)oc * Kt + k];
}
template <int K, int S>
__global__ void k_col2im(const float* __restrict__ dcol, const float* __restrict__ x, long x_stride,
                         float* __restrict__ dx, long dx_stride, int IC, int IH, int IW, int OH, int OW, int n,
                         int accumulate) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long per = (long)IC * IH * IW;
  if (i >= per * n) return;
  const long smp = i / per;
  const int r = (int)(i - smp * per), ic = r / (IH * IW), p = r - ic * IH * IW, iy = p / IW, ix = p - iy * IW;
  const int OP = OH * OW;
  const float* col = dcol + (size_t)smp * IC * K * K * OP + (size_t)ic * K * K * OP;
  float v = 0.0f;
#pragma unroll
  for (int ky = 0; ky < K; ++ky) {
    const int dy = iy - ky, oy = dy / S;
    if (dy < 0 || dy % S || oy >= OH) continue;
#pragma unroll
    for (int kx = 0; kx < K; ++kx) {
      const int dxx = ix - kx, ox = dxx / S;
      if (dxx < 0 || dxx % S || ox >= OW) continue;
      v += col[(ky * K + kx) * OP + oy * OW + ox];
    }
  }
  const float xm = x[smp * x_stride + r];
  const float gv = xm > 0.0f ? v : 0.0f;
  float* o = dx + smp * dx_stride + r;
  *o = accumulate ? *o + gv : gv;
}
// conv6 only: for conv5 (stride 2, 10 x 10 -> 4 x 4) the col2im pass costs more than the GEMM saves
// (GEMM 77 + col2im 127 us vs k_dgrad's 182 us; conv6: 5 + 71 + 33 vs 370 us; profiles/r05/carla_tiled/)
static bool dgrad_col_layer(int OH, int OW, int K = 3, int S = 1) { return OH * OW <= 16 && K == 3 && S == 1; }

struct WgradArgs {
  const float* dz;  // [n][OC][OP], sample stride dz_stride
  long dz_stride;
  int OC, OP, OW;
  const float* x_f;
  const uint8_t* x_u8;
  long x_stride;
  int IC, IH, IW, K, S;
  int n, Kt;     // Kt = IC*K*K; column Kt is the bias (x = 1)
  long qchunk;   // output pixels per chunk (multiple of 4)
  float* part;   // [chunks][OC][Kt + 1]
  long group_bytes = 0;  // host only: launch_wgrad_generic's sample-group limit (0: kWgradFar)
};

constexpr int kMaxPTab = 9216;  // output pixels per sample (94 x 94 = 8836 for conv1)
constexpr uint32_t kWgradFar = 0x70000000u;  // k_wgrad's out-of-range byte offset (fp32 inputs stay below it)

template <int NOT, int NKT, bool U8>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 4))) void k_wgrad(WgradArgs a) {
  // U q-steps per iteration: all their loads are issued before their MFMAs (the narrow layers have
  // the longest pixel runs and the fewest MFMAs per load, so they get the deepest batch)
  constexpr int U = NOT == 1 ? 8 : 2;
  constexpr int NA = 16 * NOT * 4 * U;           // dZ tile of one iteration (channels x pixels)
  constexpr int NAT = (NA + 255) / 256;          // dZ elements staged per thread
  __shared__ int koff[kMaxKTab];
  __shared__ int pbase[kMaxPTab];
  __shared__ __attribute__((aligned(16))) float ast[2][NA];  // [buf][t][g][j][st]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  const int KK = a.K * a.K, plane = a.IH * a.IW;
  for (int k = tid; k < a.Kt; k += 256) {
    const int ic = k / KK, rem = k - ic * KK, ky = rem / a.K, kx = rem - ky * a.K;
    koff[k] = ic * plane + ky * a.IW + kx;
  }
  for (int p = tid; p < a.OP; p += 256) {
    const int oy = p / a.OW, ox = p - oy * a.OW;
    pbase[p] = oy * a.S * a.IW + ox * a.S;
  }
  const long Q = (long)a.n * a.OP;
  const long qs = (long)blockIdx.x * a.qchunk;
  const long qe = qs + a.qchunk < Q ? qs + a.qchunk : Q;
  const int oc0 = blockIdx.y * 16 * NOT;
  // waves whose columns start past Kt stay (their columns are masked) for the workgroup's staging
  const int kb = (blockIdx.z * 4 + wave) * 16 * NKT;
  f4 acc[NOT][NKT];
#pragma unroll
  for (int t = 0; t < NOT; ++t)
#pragma unroll
    for (int u = 0; u < NKT; ++u) acc[t][u] = f4{0.f, 0.f, 0.f, 0.f};
  int ko[NKT];
  int kc[NKT];  // 0: gathered column, 1: bias column, 2: past the end
  __syncthreads();
#pragma unroll
  for (int u = 0; u < NKT; ++u) {
    const int k = kb + 16 * u + j;
    kc[u] = k < a.Kt ? 0 : (k == a.Kt ? 1 : 2);
    ko[u] = k < a.Kt ? koff[k] : 0;
  }
  // fp32 input: the gathers go through a buffer descriptor with 32-bit byte offsets (the whole
  // minibatch's activations are < 4 GB, launch condition): column byte offsets ko4 (a value far past
  // the buffer for the bias / padding columns) plus the pixel's byte offset xb4 (also far past the
  // buffer for pixels past the chunk), so a column reads 0 out of range instead of through a select
  // and 64-bit address arithmetic (round 5: 15 VALU per MFMA before, SQ counters)
  constexpr uint32_t kFar = kWgradFar;
  uint32_t ko4[NKT];
#pragma unroll
  for (int u = 0; u < NKT; ++u) ko4[u] = kc[u] == 0 ? (uint32_t)ko[u] * 4u : kFar;
  const PBuf xbuf{__builtin_amdgcn_make_buffer_rsrc((void*)(U8 ? (const void*)a.x_u8 : (const void*)a.x_f), (short)0,
                                                    (int)(U8 ? 0 : (uint32_t)min((long)a.n * a.x_stride * 4, (long)kFar)),
                                                    0x00020000)};
  // The dZ operand (the A side) is the same for the workgroup's 4 waves: each iteration's
  // 16 NOT x 4 U tile is loaded once per workgroup (element e = tid + 256 h: channel e / (4 U),
  // pixel qb + e % (4 U), consecutive threads on consecutive pixels) and staged in LDS in A-operand
  // order (lane (j, g) reads its U steps of tile t as one vector). Same operands and MFMA chain as
  // the per-wave gathers: bitwise unchanged.
  long as_[NAT];
  int ap_[NAT];
  auto apos = [&](int h, long q) {  // (sample, pixel) of pixel q for staging slot h
    const long sm = q / a.OP;
    as_[h] = sm;
    ap_[h] = (int)(q - sm * a.OP);
  };
#pragma unroll
  for (int h = 0; h < NAT; ++h) apos(h, qs + (tid + 256 * h) % (4 * U));
  float areg[NAT];
  auto aload = [&](long qb) {
#pragma unroll
    for (int h = 0; h < NAT; ++h) {
      const int e = tid + 256 * h, o = e / (4 * U), pi = e - o * (4 * U), oc = oc0 + o;
      const bool ok = e < NA && oc < a.OC && qb + pi < qe;
      areg[h] = a.dz[ok ? as_[h] * a.dz_stride + (long)oc * a.OP + ap_[h] : 0] * (ok ? 1.0f : 0.0f);
      // advance to the next iteration's pixel (qb + 4 U + pi)
      long sm = as_[h];
      int pp = ap_[h] + 4 * U;
      while (pp >= a.OP) {
        pp -= a.OP;
        ++sm;
      }
      as_[h] = sm;
      ap_[h] = pp;
    }
  };
  auto astore = [&](int buf) {
#pragma unroll
    for (int h = 0; h < NAT; ++h) {
      const int e = tid + 256 * h;
      if (e < NA) {
        const int o = e / (4 * U), pi = e - o * (4 * U), t = o >> 4, jo = o & 15, st = pi >> 2, gg = pi & 3;
        ast[buf][((t * 4 + gg) * 16 + jo) * U + st] = areg[h];
      }
    }
  };
  long q = qs + g;
  long s = q / a.OP;
  int p = (int)(q - s * a.OP);
  const bool wrap1 = a.OP >= 4;
  aload(qs);
  astore(0);
  __syncthreads();
  int buf = 0;
  for (long qb = qs; qb < qe; qb += 4 * U, buf ^= 1) {
    const bool more = qb + 4 * U < qe;
    if (more) aload(qb + 4 * U);
    float bv[U][NKT];
#pragma unroll
    for (int st = 0; st < U; ++st) {
      const bool qv = q < qe;
      if constexpr (U8) {
        const long xb = s * a.x_stride + (qv ? pbase[p] : 0);
#pragma unroll
        for (int u = 0; u < NKT; ++u) {
          const bool ok = qv && kc[u] == 0;
          const long off = ok ? xb + ko[u] : 0;
          const int raw = a.x_u8[off];
          const float v = (float)(ok ? raw : 0) * (1.0f / 255.0f);
          bv[st][u] = (qv && kc[u] == 1) ? 1.0f : v;
        }
      } else {
        const uint32_t xb4 = qv ? (uint32_t)(s * a.x_stride + pbase[p]) * 4u : kFar;
#pragma unroll
        for (int u = 0; u < NKT; ++u) {
          const float v = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xbuf.r, xb4 + ko4[u], 0, 0));
          bv[st][u] = (qv && kc[u] == 1) ? 1.0f : v;
        }
      }
      q += 4;
      p += 4;
      if (wrap1) {  // OP >= 4: at most one sample boundary per step (branch-free)
        const bool w = p >= a.OP;
        p -= w ? a.OP : 0;
        s += w ? 1 : 0;
      } else {
        while (p >= a.OP) {
          p -= a.OP;
          ++s;
        }
      }
    }
    float av[NOT][U];  // av[t][st] = dZ[oc0 + 16 t + j][pixel qb + 4 st + g]
#pragma unroll
    for (int t = 0; t < NOT; ++t)
#pragma unroll
      for (int st = 0; st < U; ++st) av[t][st] = ast[buf][((t * 4 + g) * 16 + j) * U + st];
#pragma unroll
    for (int st = 0; st < U; ++st)
#pragma unroll
      for (int t = 0; t < NOT; ++t)
#pragma unroll
        for (int u = 0; u < NKT; ++u) acc[t][u] = mfma16(av[t][st], bv[st][u], acc[t][u]);
    if (more) astore(buf ^ 1);
    __syncthreads();
  }
  float* out = a.part + (long)blockIdx.x * a.OC * (a.Kt + 1);
#pragma unroll
  for (int t = 0; t < NOT; ++t)
#pragma unroll
    for (int u = 0; u < NKT; ++u) {
      const int k = kb + 16 * u + j;
      if (k > a.Kt) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int oc = oc0 + 16 * t + 4 * g + r;
        if (oc < a.OC) out[(long)oc * (a.Kt + 1) + k] = acc[t][u][r];
      }
    }
}

// ---- conv1's weight gradient (uint8 image, OC <= 16): input patch and dZ tile staged in LDS ----
// dW[oc][k] (+ the bias column k = Kt) = sum over output pixels of dZ[oc][px] * im2col(x)[px][k].
// k_wgrad gathers every B operand from global memory (a byte per lane and k-step): for conv1, with
// 18 M output pixels per 2 048-row minibatch, that instruction rate was the bound. Here workgroup c
// walks output tiles [c * tpc, (c + 1) * tpc) (16 x 16 pixels of one sample each); per tile the
// (15 S + K)^2 x IC uint8 patch and the OC x 256 dZ tile (zero outside the image) are staged in LDS,
// and wave w accumulates column tiles 6w .. 6w + 5 of the [OC] x [Kt + 1] product over the tile's
// 256 pixels (A = dZ, B = ds_read_u8 gathers), across all its tiles. Partials: part[c][OC][Kt + 1],
// reduced by k_wsum1 / k_wsum in chunk order as k_wgrad's.
constexpr int kWimgCT = 6;  // column tiles per wave: 4 waves x 6 x 16 = 384 >= Kt + 1 = 376
static size_t wimg_lds_bytes(int IC, int K, int S, int OC) {
  const int TI = (kImgTile - 1) * S + K, TIP = (TI + 3) & ~3;
  const size_t patch = ((size_t)IC * TI * TIP + 15) & ~(size_t)15;
  return patch + (size_t)OC * 260 * 4;
}

template <int K, int S>
__global__ __launch_bounds__(256) void k_wgrad_img(WgradArgs a, int tiles_x, int tps, int tiles, int tpc) {
  using G = ImgGeo<K, S>;
  constexpr int TI = G::TI, TIP = G::TIP, DW = TIP / 4, DZP = 260;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  const int KK = K * K, Kt = a.Kt, OC = a.OC, plane = a.IH * a.IW;
  const size_t patch = ((size_t)a.IC * TI * TIP + 15) & ~(size_t)15;
  unsigned char* tile = smem;
  float* dzl = reinterpret_cast<float*>(smem + patch);  // [OC][DZP]: pixel 16 ly + lx
  // this lane's B columns: patch offset of tap col (gathered), or the bias / padding column
  int ko[kWimgCT];
  float cb[kWimgCT];  // 1 for the bias column, 0 for padding columns, -1 for gathered columns
#pragma unroll
  for (int u = 0; u < kWimgCT; ++u) {
    const int col = (wave * kWimgCT + u) * 16 + j;
    const int ic = col / KK, rem = col - ic * KK, ky = rem / K, kx = rem - ky * K;
    ko[u] = col < Kt ? (ic * TI + ky) * TIP + kx : 0;
    cb[u] = col < Kt ? -1.0f : (col == Kt ? 1.0f : 0.0f);
  }
  const float* arow = dzl + (j < OC ? j : 0) * DZP;
  const float am = j < OC ? 1.0f : 0.0f;
  f4 acc[kWimgCT];
#pragma unroll
  for (int u = 0; u < kWimgCT; ++u) acc[u] = f4{0.f, 0.f, 0.f, 0.f};
  const size_t total_bytes = (size_t)a.n * a.x_stride;
  const int t0 = blockIdx.x * tpc, t1 = min(tiles, t0 + tpc);
  for (int t = t0; t < t1; ++t) {
    const int smp = t / tps, tt = t - smp * tps;
    const int ty = tt / tiles_x, tx = tt - ty * tiles_x;
    const int OH = a.OP / a.OW;
    const int x0 = tx * kImgTile * S, y0 = ty * kImgTile * S;
    __syncthreads();  // the previous tile's readers are done
    {
      const size_t sb = (size_t)smp * a.x_stride, left = total_bytes - sb;
      const PBuf ib{__builtin_amdgcn_make_buffer_rsrc((void*)(a.x_u8 + sb), (short)0,
                                                      (int)(left < 0xFFFFFFF0u ? left : 0xFFFFFFF0u), 0x00020000)};
      const int tot = a.IC * TI * DW;
      for (int e = tid; e < tot; e += 256) {
        const int ic = e / (TI * DW), rem = e - ic * (TI * DW), r = rem / DW, d = rem - r * DW;
        const unsigned v = __builtin_amdgcn_raw_buffer_load_b32(ib.r, ic * plane + (y0 + r) * a.IW + x0 + 4 * d, 0, 0);
        *reinterpret_cast<unsigned*>(tile + (ic * TI + r) * TIP + 4 * d) = v;
      }
      const float* dz = a.dz + (size_t)smp * a.dz_stride;
      for (int e = tid; e < OC * 256; e += 256) {
        const int oc = e >> 8, px = e & 255, oy = ty * kImgTile + (px >> 4), ox = tx * kImgTile + (px & 15);
        const bool in = oy < OH && ox < a.OW;
        const float v = dz[in ? (size_t)oc * a.OP + oy * a.OW + ox : 0];
        dzl[oc * DZP + px] = in ? v : 0.0f;
      }
    }
    __syncthreads();
#pragma unroll 4
    for (int st = 0; st < 64; ++st) {
      const int px = 4 * st + g, ly = px >> 4, lx = px & 15;
      const int po = S * ly * TIP + S * lx;
      const float av = arow[px] * am;
#pragma unroll
      for (int u = 0; u < kWimgCT; ++u) {
        const int raw = tile[ko[u] + po];
        const float xv = (float)raw * (1.0f / 255.0f);
        // columns >= Kt (bias, padding) exist only in the last tile of the last wave
        const float bv = u == kWimgCT - 1 ? (cb[u] < 0.0f ? xv : cb[u]) : xv;
        acc[u] = mfma16(av, bv, acc[u]);
      }
    }
  }
  float* out = a.part + (size_t)blockIdx.x * OC * (Kt + 1);
#pragma unroll
  for (int u = 0; u < kWimgCT; ++u) {
    const int col = (wave * kWimgCT + u) * 16 + j;
    if (col > Kt) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int oc = 4 * g + r;
      if (oc < OC) out[(size_t)oc * (Kt + 1) + col] = acc[u][r];
    }
  }
}

// ---- conv2's weight gradient from LDS-staged tiles (create option conv_wgrad=tiled, the default) ----
// k_wgrad gathers every B operand (an input value) from global memory, one buffer load per MFMA,
// which its counters show it waits on. Here a persistent workgroup walks output tiles of TY x TX
// pixels of one sample: the tile's dZ (OC x TY TX) and its input patch (IC x PH x PW, zero outside the
// plane) are staged in LDS, the next tile's loaded into registers while the current one computes.
// GEMM: rows = oc (A = dZ), columns = (ic, ky, kx) plus the bias column, k = the tile's pixels; wave w
// takes output rows RPW w .. + RPW - 1. For k-step kk a lane's B operand sits at its column's patch
// offset + the lane's pixel offset + an IMMEDIATE per kk, its A operand at one base + 4 kk: the k loop
// is ds_read_b32 + MFMA only. The bias column reads a block of ones. The workgroup keeps its sums in
// registers over all its tiles, adds its four waves in a fixed order through LDS and writes one
// partial per workgroup (k_wsum's layout); the sum order differs from k_wgrad's (tolerance tests).
constexpr int kWtTY = 8, kWtTX = 16;  // output tile (conv2: 45 x 45 -> 6 x 3 tiles, 88 % used)
// LDS layout (bank = dword address mod 32 for ds_read_b32, per 32-lane half = lane groups g = 0, 1):
// the patch rows are PW = 37 floats and each input channel's plane PPA = 713 floats, so column
// c = (ic, ky, kx) sits at a dword offset = c (mod 16) and a wave's 16 columns hit 16 distinct banks;
// lane group g takes the output columns kk % 4 + 8 (g & 1) + 4 (g >> 1), 16 input floats (16 banks) away
// for g = 1: the B reads are conflict-free. dZ rows are TQ + 1 floats (A reads: 2-way on half the banks).
template <int IC, int OC, int TY, int TX>
struct WtGeo {
  static constexpr int K = 5, S = 2, Kt = IC * K * K, NCT = (Kt + 1 + 15) / 16, NRT = OC / 16;
  static constexpr int PH = (TY - 1) * S + K, PWL = (TX - 1) * S + K, PW = 37, PPL = PH * PWL, TQ = TY * TX;
  static constexpr int PPA = ((PH * PW - 9 + 15) / 16) * 16 + 9;  // >= PH PW, = 9 (mod 16): ic planes step c by 25
  static constexpr int NXL = IC * PPL, NXP = IC * PPA, DZS = TQ + 1, NZ = OC * TQ, NZP = OC * DZS;
  static constexpr int RPW = TY / 4, KS = RPW * TX / 4;
  // the largest B offset a lane adds to its column base: wave rows, lane group and k-step parts
  static constexpr int BMAX = S * RPW * 3 * PW + 16 + 8 + S * (RPW - 1) * PW + S * 3;
  static constexpr int OB0 = NXP + NZP, ONES0 = OB0 + (((Kt - OB0) % 16) + 16) % 16;  // ones base = Kt (mod 16)
  static constexpr int LDS = ONES0 + BMAX + 1;
  static constexpr int RED = OC * NCT * 16;  // the wave reduction, aliased on the patch
  static_assert(PW >= PWL && PW % 16 == 5 && RED <= NXP, "layout");
};
template <int IC, int OC, int TY, int TX>
__global__ __launch_bounds__(256, 3) void k_wgrad_t(WgradArgs a, int tiles_x, int tps, int tiles) {
  using G = WtGeo<IC, OC, TY, TX>;
  constexpr int Kt = G::Kt, NCT = G::NCT, NRT = G::NRT, PW = G::PW, PWL = G::PWL, PPA = G::PPA, TQ = G::TQ,
                DZS = G::DZS, RPW = G::RPW, KS = G::KS, S = G::S;
  // staging runs over the padded layouts, so the LDS stores are linear in the thread index
  constexpr int NXP = G::NXP, NZP = G::NZP, NSX = (NXP + 255) / 256, NSZ = (NZP + 255) / 256;
  static_assert(OC % 16 == 0 && TY % 4 == 0 && TX == 16, "tile shape");
  __shared__ __attribute__((aligned(16))) float sm[G::LDS];
  float* xp = sm;                // [IC][PPA]: rows of PW
  float* dzt = sm + G::NXP;      // [OC][DZS]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  for (int i = G::OB0 + tid; i < G::LDS; i += 256) sm[i] = 1.0f;  // the bias column's B operands
  // column bases: (ic, ky, kx) -> ic PPA + ky PW + kx; the bias column -> the ones; padding -> any
  // in-patch offset = c (mod 16)
  int cb[NCT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) {
    const int c = 16 * ct + j, ic = c / 25, r = c - 25 * ic, ky = r / 5, kx = r - 5 * ky;
    cb[ct] = c < Kt ? ic * PPA + ky * PW + kx : (c == Kt ? G::ONES0 : (c & 15));
  }
  const int bb = S * RPW * wave * PW + 16 * (g & 1) + 8 * (g >> 1);  // + S (kk / 4) PW + S (kk % 4)
  const int ab = j * DZS + RPW * TX * wave + 8 * (g & 1) + 4 * (g >> 1);  // + 16 rt DZS + TX (kk / 4) + kk % 4
  const long plane = (long)a.IH * a.IW;
  const int OH = a.OP / a.OW;
  float sx[NSX], sz[NSZ];
  auto sload = [&](int tile) {
    int tidv = tid;  // opaque: the per-element offsets are recomputed per tile, not hoisted (registers)
    asm volatile("" : "+v"(tidv));
    const int smp = tile / tps, tt = tile - smp * tps, ty = tt / tiles_x, tx = tt - ty * tiles_x;
    const PBuf xb{__builtin_amdgcn_make_buffer_rsrc((void*)(a.x_f + (size_t)smp * a.x_stride), (short)0,
                                                    (int)(a.x_stride * 4), 0x00020000)};
    const PBuf zb{__builtin_amdgcn_make_buffer_rsrc((void*)(a.dz + (size_t)smp * a.dz_stride), (short)0,
                                                    (int)(a.dz_stride * 4), 0x00020000)};
    const int iy0 = S * TY * ty, ix0 = S * TX * tx, oy0 = TY * ty, ox0 = TX * tx;
#pragma unroll
    for (int i = 0; i < NSX; ++i) {
      const int e = tidv + 256 * i, ic = e / PPA, rem = e - ic * PPA, r = rem / PW, c = rem - r * PW;
      const int iy = iy0 + r, ix = ix0 + c;
      const bool in = e < NXP && r < G::PH && c < PWL && iy < a.IH && ix < a.IW;
      const uint32_t off = in ? (uint32_t)(ic * plane + iy * a.IW + ix) * 4u : 0x7ffffff0u;
      sx[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xb.r, off, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < NSZ; ++i) {
      const int e = tidv + 256 * i, oc = e / DZS, q = e - oc * DZS, oy = oy0 + q / TX, ox = ox0 + q % TX;
      const bool in = e < NZP && q < TQ && oy < OH && ox < a.OW;
      const uint32_t off = in ? (uint32_t)(oc * a.OP + oy * a.OW + ox) * 4u : 0x7ffffff0u;
      sz[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(zb.r, off, 0, 0));
    }
  };
  f4 acc[NRT][NCT];
#pragma unroll
  for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) acc[rt][ct] = f4{0.f, 0.f, 0.f, 0.f};
  if ((int)blockIdx.x < tiles) sload(blockIdx.x);
  for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
#pragma unroll
    for (int i = 0; i < NSX; ++i)
      if (tid + 256 * i < NXP) xp[tid + 256 * i] = sx[i];
#pragma unroll
    for (int i = 0; i < NSZ; ++i)
      if (tid + 256 * i < NZP) dzt[tid + 256 * i] = sz[i];
    __syncthreads();
    if (tile + (int)gridDim.x < tiles) sload(tile + gridDim.x);
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int boff = S * (kk / 4) * PW + S * (kk % 4), aoff = TX * (kk / 4) + kk % 4;
      float av[NRT];
#pragma unroll
      for (int rt = 0; rt < NRT; ++rt) av[rt] = dzt[ab + 16 * rt * DZS + aoff];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        const float bv = xp[cb[ct] + bb + boff];
#pragma unroll
        for (int rt = 0; rt < NRT; ++rt) acc[rt][ct] = mfma16(av[rt], bv, acc[rt][ct]);
      }
    }
    __syncthreads();  // every wave is done with the tile before the next one is stored
  }
  // the four waves' sums in wave order through LDS (aliasing the patch), then one partial per workgroup
  float* red = sm;  // [OC][NCT * 16]
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float* p = red + (16 * rt + 4 * g + r) * (NCT * 16) + 16 * ct + j;
            *p = w ? *p + acc[rt][ct][r] : acc[rt][ct][r];
          }
    }
    __syncthreads();
  }
  float* out = a.part + (size_t)blockIdx.x * OC * (Kt + 1);
  for (int i = tid; i < OC * (Kt + 1); i += 256) {
    const int oc = i / (Kt + 1), c = i - oc * (Kt + 1);
    out[i] = red[oc * (NCT * 16) + c];
  }
}

// ---- conv3's weight gradient (IC 16, OC 32): k_wgrad_t with the COLUMNS split over the waves ---------
// Same staging and GEMM as k_wgrad_t, but 401 columns x 32 rows do not fit one wave's registers: wave w
// takes column tiles w, w + 4, ... over all TQ pixels of the tile (no cross-wave reduction), and the
// tile is TY x TX = 8 x 8 (conv3's 21 x 21 output: 3 x 3 tiles, 77 % used). Patch rows PW = 5 (mod 16)
// and planes PPA = 9 (mod 16) floats as in k_wgrad_t; dZ rows TQ + 2 floats (A reads: lane groups 0 and
// 1 on even / odd banks). Each lane group g takes pixel 4 kk + g of k-step kk.
constexpr int kWt2TY = 8, kWt2TX = 8;
template <int IC, int OC, int TY, int TX>
struct Wt2Geo {
  static constexpr int K = 5, S = 2, Kt = IC * K * K, NCT = (Kt + 1 + 15) / 16, NCW = (NCT + 3) / 4, NRT = OC / 16;
  static constexpr int PH = (TY - 1) * S + K, PWL = (TX - 1) * S + K, PW = ((PWL - 5 + 15) / 16) * 16 + 5;
  static constexpr int PPA = ((PH * PW - 9 + 15) / 16) * 16 + 9, TQ = TY * TX, DZS = TQ + 2, KS = TQ / 4;
  static constexpr int NXP = IC * PPA, NZP = OC * DZS;
  static constexpr int BMAX = S * (KS / (TX / 4) - 1) * PW + S * 4 * (TX / 4 - 1) + S * 3;
  static constexpr int OB0 = NXP + NZP, ONES0 = OB0 + (((Kt - OB0) % 16) + 16) % 16;
  static constexpr int LDS = ONES0 + BMAX + 1;
  static_assert(PW >= PWL && PPA >= PH * PW && TX % 4 == 0 && OC % 16 == 0, "layout");
};
template <int IC, int OC, int TY, int TX>
__global__ __launch_bounds__(256, 4) void k_wgrad_t2(WgradArgs a, int tiles_x, int tps, int tiles) {
  using G = Wt2Geo<IC, OC, TY, TX>;
  constexpr int Kt = G::Kt, NCT = G::NCT, NCW = G::NCW, NRT = G::NRT, PW = G::PW, PWL = G::PWL, PPA = G::PPA,
                TQ = G::TQ, DZS = G::DZS, KS = G::KS, S = G::S, NXP = G::NXP, NZP = G::NZP;
  constexpr int NSX = (NXP + 255) / 256, NSZ = (NZP + 255) / 256;
  __shared__ __attribute__((aligned(16))) float sm[G::LDS];
  float* xp = sm;            // [IC][PPA]: rows of PW
  float* dzt = sm + NXP;     // [OC][DZS]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  for (int i = G::OB0 + tid; i < G::LDS; i += 256) sm[i] = 1.0f;  // the bias column's B operands
  int cb[NCW];
#pragma unroll
  for (int i = 0; i < NCW; ++i) {
    const int c = 16 * (wave + 4 * i) + j, ic = c / 25, r = c - 25 * ic, ky = r / 5, kx = r - 5 * ky;
    cb[i] = c < Kt ? ic * PPA + ky * PW + kx : (c == Kt ? G::ONES0 : (c & 15));
  }
  const int bb = S * g, ab = j * DZS + g;  // B: + S (kk / (TX / 4)) PW + 4 S (kk % (TX / 4)); A: + 16 rt DZS + 4 kk
  const long plane = (long)a.IH * a.IW;
  const int OH = a.OP / a.OW;
  float sx[NSX], sz[NSZ];
  auto sload = [&](int tile) {
    int tidv = tid;  // opaque: the per-element offsets are recomputed per tile, not hoisted (registers)
    asm volatile("" : "+v"(tidv));
    const int smp = tile / tps, tt = tile - smp * tps, ty = tt / tiles_x, tx = tt - ty * tiles_x;
    const PBuf xb{__builtin_amdgcn_make_buffer_rsrc((void*)(a.x_f + (size_t)smp * a.x_stride), (short)0,
                                                    (int)(a.x_stride * 4), 0x00020000)};
    const PBuf zb{__builtin_amdgcn_make_buffer_rsrc((void*)(a.dz + (size_t)smp * a.dz_stride), (short)0,
                                                    (int)(a.dz_stride * 4), 0x00020000)};
    const int iy0 = S * TY * ty, ix0 = S * TX * tx, oy0 = TY * ty, ox0 = TX * tx;
#pragma unroll
    for (int i = 0; i < NSX; ++i) {
      const int e = tidv + 256 * i, ic = e / PPA, rem = e - ic * PPA, r = rem / PW, c = rem - r * PW;
      const int iy = iy0 + r, ix = ix0 + c;
      const bool in = e < NXP && r < G::PH && c < PWL && iy < a.IH && ix < a.IW;
      const uint32_t off = in ? (uint32_t)(ic * plane + iy * a.IW + ix) * 4u : 0x7ffffff0u;
      sx[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xb.r, off, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < NSZ; ++i) {
      const int e = tidv + 256 * i, oc = e / DZS, q = e - oc * DZS, oy = oy0 + q / TX, ox = ox0 + q % TX;
      const bool in = e < NZP && q < TQ && oy < OH && ox < a.OW;
      const uint32_t off = in ? (uint32_t)(oc * a.OP + oy * a.OW + ox) * 4u : 0x7ffffff0u;
      sz[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(zb.r, off, 0, 0));
    }
  };
  f4 acc[NRT][NCW];
#pragma unroll
  for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
    for (int i = 0; i < NCW; ++i) acc[rt][i] = f4{0.f, 0.f, 0.f, 0.f};
  if ((int)blockIdx.x < tiles) sload(blockIdx.x);
  for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
#pragma unroll
    for (int i = 0; i < NSX; ++i)
      if (tid + 256 * i < NXP) xp[tid + 256 * i] = sx[i];
#pragma unroll
    for (int i = 0; i < NSZ; ++i)
      if (tid + 256 * i < NZP) dzt[tid + 256 * i] = sz[i];
    __syncthreads();
    if (tile + (int)gridDim.x < tiles) sload(tile + gridDim.x);
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int boff = S * (kk / (TX / 4)) * PW + 4 * S * (kk % (TX / 4));
      float av[NRT];
#pragma unroll
      for (int rt = 0; rt < NRT; ++rt) av[rt] = dzt[ab + 16 * rt * DZS + 4 * kk];
#pragma unroll
      for (int i = 0; i < NCW; ++i) {
        if (wave + 4 * i >= NCT) continue;  // wave-uniform
        const float bv = xp[cb[i] + bb + boff];
#pragma unroll
        for (int rt = 0; rt < NRT; ++rt) acc[rt][i] = mfma16(av[rt], bv, acc[rt][i]);
      }
    }
    __syncthreads();  // every wave is done with the tile before the next one is stored
  }
  float* out = a.part + (size_t)blockIdx.x * OC * (Kt + 1);
#pragma unroll
  for (int i = 0; i < NCW; ++i) {
    const int c = 16 * (wave + 4 * i) + j;
    if (c > Kt) continue;
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(size_t)(16 * rt + 4 * g + r) * (Kt + 1) + c] = acc[rt][i][r];
  }
}

// G[w + oc*Kt + k] / G[b + oc] = sum over chunks. Level 1 (k_wsum1) adds groups of kSumGroup
// consecutive chunks in parallel (blockIdx.y = group), level 2 (k_wsum) adds the group sums in order:
// a fixed order, so the result is deterministic.
constexpr int kSumGroup = 32;

__global__ void k_wsum1(const float* __restrict__ part, int chunks, long per, float* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= per) return;
  const int c0 = blockIdx.y * kSumGroup, c1 = c0 + kSumGroup < chunks ? c0 + kSumGroup : chunks;
  float acc = 0.f;
  for (int c = c0; c < c1; ++c) acc += part[(long)c * per + i];
  out[(long)blockIdx.y * per + i] = acc;
}

__global__ void k_wsum(const float* __restrict__ part, int chunks, int OC, int Kt, float* __restrict__ Gw,
                       float* __restrict__ Gb, int accum) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long per = (long)OC * (Kt + 1);
  if (i >= per) return;
  float acc = 0.f;
  for (int c = 0; c < chunks; ++c) acc += part[(long)c * per + i];
  const int oc = (int)(i / (Kt + 1)), k = (int)(i - (long)oc * (Kt + 1));
  float* o = k < Kt ? Gw + (long)oc * Kt + k : Gb + oc;
  *o = accum ? *o + acc : acc;  // accum: a later sample group of launch_wgrad's split
}

// the same statistics in the distributed order of ac_ppo_carla.cpp:561-580, one block each:
// phase 0: out[0] = local mean; phase 1: out[2] = sum (adv - out[0])^2 about the (all-reduced) mean
__global__ __launch_bounds__(256) void k_carla_adv_part(const float* __restrict__ adv, int n, float* __restrict__ out,
                                                        int phase) {
  __shared__ float red[256];
  float s = 0.f;
  if (phase == 0) {
    for (int i = threadIdx.x; i < n; i += 256) s += adv[i];
  } else {
    const float mean = out[0];
    for (int i = threadIdx.x; i < n; i += 256) s += (adv[i] - mean) * (adv[i] - mean);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (phase == 0) out[0] = red[0] / (float)n;
    else out[2] = red[0];
  }
}
// out[1] = sqrt(sum of squares over all ranks / (world * n - 1))
__global__ void k_carla_adv_fin(float* __restrict__ out, float denom) {
  if (threadIdx.x == 0) out[1] = sqrtf(out[2] / denom);
}

// minibatch advantage mean / std (Bessel), one block, fixed summation order
__global__ __launch_bounds__(256) void k_carla_advstats(const float* __restrict__ adv, int n, float* __restrict__ out) {
  __shared__ float red[256];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += adv[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  const float mean = red[0] / (float)n;
  __syncthreads();
  float q = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) q += (adv[i] - mean) * (adv[i] - mean);
  red[threadIdx.x] = q;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = mean;
    out[1] = sqrtf(red[0] / (float)(n - 1));
  }
}

struct HeadBwdArgs {
  const float* P;
  long hi, lo;
  const float* hpre;  // [n][2A]
  const float* actions;
  const float *lp, *ent, *val, *old_logp, *adv, *ret, *old_v;
  const float* advstat;  // mean, std
  int n, A;
  float beta_min, clip, ent_coef, vf_coef;
  int norm_adv, clip_vloss;
  float* dhead;    // [n][2A]
  float* dval;     // [n]
  float* rowstat;  // [n][8]
};

PPO_DEV float softplus_grad(float x) {
  if (x > 20.0f) return 1.0f;
  const float e = expf(x);
  return e / (e + 1.0f);
}

// loss -> d(dist_mu, dist_sigma pre-activations), d(value); the terms of the minibatch stats
__global__ __launch_bounds__(64) void k_carla_head_bwd(HeadBwdArgs h) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= h.n) return;
  const float invM = 1.0f / (float)h.n, c = h.clip;
  const float logratio = h.lp[r] - h.old_logp[r];
  const float ratio = expf(logratio);
  float an = h.adv[r];
  if (h.norm_adv) an = (an - h.advstat[0]) / (h.advstat[1] + 1e-8f);
  const float rc = fminf(fmaxf(ratio, 1.0f - c), 1.0f + c);
  const float pg1 = -an * ratio, pg2 = -an * rc;
  // d max(pg1, pg2) / d ratio; ties split the gradient (ATen maximum backward)
  const float w1 = pg1 > pg2 ? 1.0f : (pg1 == pg2 ? 0.5f : 0.0f);
  const float inr = (ratio >= 1.0f - c && ratio <= 1.0f + c) ? 1.0f : 0.0f;
  const float dratio = w1 * (-an) + (1.0f - w1) * (-an) * inr;
  const float g_logp = invM * dratio * ratio;
  const float v = h.val[r], R = h.ret[r];
  float g_v, vterm;
  if (h.clip_vloss) {
    const float vu = (v - R) * (v - R);
    const float dv = v - h.old_v[r];
    const float vcl = h.old_v[r] + fminf(fmaxf(dv, -c), c);
    const float vc = (vcl - R) * (vcl - R);
    vterm = fmaxf(vu, vc);
    const float u1 = vu > vc ? 1.0f : (vu == vc ? 0.5f : 0.0f);
    const float in2 = (dv >= -c && dv <= c) ? 1.0f : 0.0f;
    g_v = 0.5f * h.vf_coef * invM * (u1 * 2.0f * (v - R) + (1.0f - u1) * 2.0f * (vcl - R) * in2);
  } else {
    vterm = (v - R) * (v - R);
    g_v = 0.5f * h.vf_coef * invM * 2.0f * (v - R);
  }
  const float g_ent = -h.ent_coef * invM;
  const float hi = h.P[h.hi], lo = h.P[h.lo];
  for (int ai = 0; ai < h.A; ++ai) {
    const float pm = h.hpre[(long)r * 2 * h.A + ai], ps = h.hpre[(long)r * 2 * h.A + h.A + ai];
    const float al = softplusf_(pm) + h.beta_min, be = softplusf_(ps) + h.beta_min, ab = al + be;
    float sv = (h.actions[(long)r * h.A + ai] - lo) / (hi - lo) * (1.0f - 0.0f) + 0.0f;
    sv = fminf(fmaxf(sv, 0.0f + 1e-7f), 1.0f + 1e-7f);
    const float psab = digammaf_(ab), tab = trigammaf_(ab);
    const float dla = ((al - 1.0f) != 0.0f ? logf(sv) : 0.0f) + psab - digammaf_(al);
    const float dlb = ((be - 1.0f) != 0.0f ? logf(1.0f - sv) : 0.0f) + psab - digammaf_(be);
    const float dea = (ab - 2.0f) * tab - (al - 1.0f) * trigammaf_(al);
    const float deb = (ab - 2.0f) * tab - (be - 1.0f) * trigammaf_(be);
    h.dhead[(long)r * 2 * h.A + ai] = (g_logp * dla + g_ent * dea) * softplus_grad(pm);
    h.dhead[(long)r * 2 * h.A + h.A + ai] = (g_logp * dlb + g_ent * deb) * softplus_grad(ps);
  }
  h.dval[r] = g_v;
  float* st = h.rowstat + (long)r * 8;
  st[0] = fmaxf(pg1, pg2);
  st[1] = vterm;
  st[2] = h.ent[r];
  st[3] = -logratio;
  st[4] = (ratio - 1.0f) - logratio;
  st[5] = fabsf(ratio - 1.0f) > c ? 1.0f : 0.0f;
}

// row means of the stats, one block, fixed order: pg, 0.5*v, entropy, old_kl, kl, clipfrac
__global__ __launch_bounds__(256) void k_carla_stats(const float* __restrict__ rowstat, int n, float* __restrict__ out) {
  __shared__ float red[6][256];
  float a[6] = {0, 0, 0, 0, 0, 0};
  for (int i = threadIdx.x; i < n; i += 256)
    for (int k = 0; k < 6; ++k) a[k] += rowstat[(long)i * 8 + k];
  for (int k = 0; k < 6; ++k) red[k][threadIdx.x] = a[k];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w)
      for (int k = 0; k < 6; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x < 6) out[threadIdx.x] = red[threadIdx.x][0] / (float)n * (threadIdx.x == 1 ? 0.5f : 1.0f);
}

constexpr int kNormSplit = 32;

// per-tensor sums of squares of the gradient, kNormSplit slices per tensor (blockIdx.y)
__global__ __launch_bounds__(256) void k_carla_tnorm(const float* __restrict__ G, const long* __restrict__ off,
                                                     const long* __restrict__ len, float* __restrict__ part) {
  __shared__ float red[256];
  const int t = blockIdx.x, sp = blockIdx.y;
  const long n = len[t], per = (n + kNormSplit - 1) / kNormSplit, b = sp * per, e = b + per < n ? b + per : n;
  float q = 0.f;
  for (long i = b + threadIdx.x; i < e; i += 256) {
    const float x = G[off[t] + i];
    q += x * x;
  }
  red[threadIdx.x] = q;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[t * kNormSplit + sp] = red[0];
}

// clip_grad_norm_ (clip_grad.h): norm_t = ||g_t|| (slices added in order), total = ||(norm_t)||,
// coef = clamp(max_norm / (total + 1e-6), max = 1); out = {total, coef}
__global__ void k_carla_tsum(const float* __restrict__ part, int nt, float max_norm, float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  float tot = 0.f;
  for (int t = 0; t < nt; ++t) {
    float q = 0.f;
    for (int sp = 0; sp < kNormSplit; ++sp) q += part[t * kNormSplit + sp];
    const float nrm = sqrtf(q);
    tot += nrm * nrm;
  }
  const float total = sqrtf(tot);
  const float coef = max_norm / (total + 1e-6f);
  out[0] = total;
  out[1] = coef > 1.0f ? 1.0f : coef;
}

struct CarlaAdamArgs {
  float *P, *G, *m, *v;
  long begin, n;        // trainable range [begin, begin + n)
  const float* clip;    // {total, coef} from k_carla_tsum
  float step_size, sbc2, eps;
};

__global__ __launch_bounds__(256) void k_carla_adam(CarlaAdamArgs a) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  const long p = a.begin + i;
  const float gv = a.G[p] * a.clip[1];
  const float m = a.m[p] * 0.9f + gv * 0.1f;
  const float v = a.v[p] * 0.999f + gv * gv * 0.001f;
  a.m[p] = m;
  a.v[p] = v;
  a.P[p] = a.P[p] - a.step_size * (m / (sqrtf(v) / a.sbc2 + a.eps));
}

int launch_dgrad(const DgradArgs& a, hipStream_t s, bool staged = true, bool quad = false) {
  if (staged && quad && a.K == 5 && a.S == 2 && a.IC == 16 && a.OC == 32 && a.w_ic == a.IC) {
    const int tiles_x = ((a.IW + 1) / 2 + kDq2T - 1) / kDq2T, tps = tiles_x * (((a.IH + 1) / 2 + kDq2T - 1) / kDq2T);
    const long tiles = (long)a.n * tps;
    const size_t lds = dq2_lds_bytes(a.OC);
    static const bool attr = hipFuncSetAttribute((const void*)k_dgrad_q2<16, 32>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess;
    if (attr && tiles < (1L << 31) && a.dz_stride < (1L << 29) && a.x_stride < (1L << 29) && a.dx_stride < (1L << 29)) {
      const int grid = (int)std::min<long>(tiles, 256L * 2);  // two workgroups per CU (LDS)
      hipLaunchKernelGGL((k_dgrad_q2<16, 32>), dim3(grid), dim3(256), lds, s, a, tiles_x, tps, (int)tiles);
      return 0;
    }
  }
  if (staged && quad && a.K == 5 && a.S == 2 && a.IC == 8 && a.OC == 16 && a.w_ic == a.IC && a.IW % 2 == 0) {
    const int tiles_x = ((a.IW + 1) / 2 + kDqT - 1) / kDqT, tps = tiles_x * (((a.IH + 1) / 2 + 4 * kDqU - 1) / (4 * kDqU));
    const long tiles = (long)a.n * tps;
    if (tiles >= (1L << 31) || a.dz_stride >= (1L << 29) || a.x_stride >= (1L << 29) || a.dx_stride >= (1L << 29))
      return -1;
    // one round of resident workgroups (kDqU = 2: three per CU; 4: two): a larger grid would run a
    // second, partial round
    const int grid = (int)std::min<long>(tiles, 256L * (kDqU == 2 ? 3 : 2));
    hipLaunchKernelGGL((k_dgrad_q<8, 16>), dim3(grid), dim3(256), 0, s, a, tiles_x, tps, (int)tiles);
    return 0;
  }
  if (staged && a.K == 5 && a.S == 2 && a.IC <= 16 && a.OC <= 16 && a.w_ic == a.IC &&
      ds2_lds_bytes(a.IC, a.OC) <= 64 * 1024) {
    const int tiles_x = (a.IW + kDs2Tile - 1) / kDs2Tile, tps = tiles_x * ((a.IH + kDs2Tile - 1) / kDs2Tile);
    hipLaunchKernelGGL(k_dgrad_s2, dim3(a.n * tps), dim3(256), ds2_lds_bytes(a.IC, a.OC), s, a, tiles_x, tps);
    return 0;
  }
  const int nj = (a.K + a.S - 1) / a.S;
  if ((long)a.OC * nj * nj > kMaxDTab) return -1;
  const int H2 = (a.IH + a.S - 1) / a.S, W2 = (a.IW + a.S - 1) / a.S;
  const long Q = (long)a.n * H2 * W2;
  const int np = Q >= 16L * 4 * 1024 ? 4 : 1;
  const unsigned gx = (unsigned)((Q + 64L * np - 1) / (64L * np));
  const unsigned gz = (unsigned)(a.S * a.S);
  if (a.IC >= 64) {
    if (np == 4) hipLaunchKernelGGL((k_dgrad<4, 4>), dim3(gx, (a.IC + 63) / 64, gz), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_dgrad<4, 1>), dim3(gx, (a.IC + 63) / 64, gz), dim3(256), 0, s, a);
  } else if (a.IC >= 32) {
    if (np == 4) hipLaunchKernelGGL((k_dgrad<2, 4>), dim3(gx, (a.IC + 31) / 32, gz), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_dgrad<2, 1>), dim3(gx, (a.IC + 31) / 32, gz), dim3(256), 0, s, a);
  } else {
    if (np == 4) hipLaunchKernelGGL((k_dgrad<1, 4>), dim3(gx, (a.IC + 15) / 16, gz), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_dgrad<1, 1>), dim3(gx, (a.IC + 15) / 16, gz), dim3(256), 0, s, a);
  }
  return 0;
}

constexpr int kWgradNKT = 2;  // a wave: 32 gathered columns; a workgroup: 128

struct WgradPlan {
  int not_, ocg, kg, chunks;
  long qchunk;
  size_t part_floats;
};

WgradPlan plan_wgrad(int OC, int Kt, long Q) {
  WgradPlan p;
  p.not_ = OC >= 64 ? 4 : (OC >= 32 ? 2 : 1);
  p.ocg = (OC + 16 * p.not_ - 1) / (16 * p.not_);
  p.kg = (Kt + 1 + 64 * kWgradNKT - 1) / (64 * kWgradNKT);
  long chunks = (8192 + (long)p.ocg * p.kg - 1) / ((long)p.ocg * p.kg);
  chunks = chunks < 1 ? 1 : (chunks > 4096 ? 4096 : chunks);
  const long cap = (32L << 20) / ((long)OC * (Kt + 1));  // partials <= 32 M floats
  if (chunks > cap) chunks = cap < 1 ? 1 : cap;
  // at least 64 pixels / rows per chunk: the Linear layers (2 048 rows) then need <= 32 chunks and
  // one k_wsum pass instead of k_wsum1 + k_wsum
  const long maxc = (Q + 63) / 64;
  if (chunks > maxc) chunks = maxc < 1 ? 1 : maxc;
  p.qchunk = ((Q + chunks - 1) / chunks + 3) / 4 * 4;
  p.chunks = (int)((Q + p.qchunk - 1) / p.qchunk);
  const int groups = (p.chunks + kSumGroup - 1) / kSumGroup;
  p.part_floats = (size_t)(p.chunks + (p.chunks > kSumGroup ? groups : 0)) * OC * (Kt + 1);
  return p;
}

// ---- conv1's weight gradient with OC <= 8: two output columns per A row pair ------------------
// As k_conv_img2: A row oc + 8 dx is dZ[oc] at the odd (dx = 1) or even (dx = 0) output column of
// each column pair, the k dimension is the tile's 128 column pairs, and the B columns are the
// extended taps (ic, ky, kx'), kx' in [0, K + S), plus the bias column: D[oc + 8 dx][(ic, ky, kx')]
// sums dZ x input over the even (dx = 0) or odd (dx = 1) output columns, and
// dW[oc][ic, ky, kx] = D[oc][(ic, ky, kx)] + D[oc + 8][(ic, ky, kx + S)] (bias: both halves).
// 25 % fewer MFMAs than k_wgrad_img; the pixel sum is split into its even and odd halves, so the
// result differs from k_wgrad's in rounding only. The combine runs once per workgroup through LDS.
// The B operands are the raw byte values (exact in fp32) and the workgroup's tap sums are scaled by
// 1 / 255 once in the combine (round 5: one VALU fewer per MFMA; the bias column is not scaled).
constexpr int kWimg2CT = 9;  // column tiles per wave: 4 x 9 x 16 = 576 >= IC K (K + S) + 1 = 526
static size_t wimg2_lds_bytes(int IC, int K, int S, int OC) {
  const int TI = (kImgTile - 1) * S + K, TIP = (TI + 3) & ~3;
  const size_t patch = ((size_t)IC * TI * TIP + 15) & ~(size_t)15;
  const size_t stage = patch + (size_t)OC * 260 * 4, comb = (size_t)16 * 4 * kWimg2CT * 16 * 4;
  return stage > comb ? stage : comb;
}

// BX (create option conv1_mfma=bx3): the pixel sums as v_mfma_f32_16x16x32_bf16 — the B operands
// (raw bytes 0..255, and the bias column's 1) are exact bf16 numbers, so every fp32 product dZ.x is
// the exact sum of three: dZ's split-bf16 pieces (hi, mid, lo; split3_pair) times x. Three 16-cycle
// MFMAs per 32 pixel pairs instead of eight 32-cycle 16x16x4 f32 ones; lane group g's k slot e of
// step q is pixel pair 32 q + 4 e + g (the f32 loop's step 8 q + e).
template <int K, int S, bool BX = false>
__global__ __launch_bounds__(256, 3) void k_wgrad_img2(WgradArgs a, int tiles_x, int tps, int tiles, int tpc) {
  using G = ImgGeo<K, S>;
  constexpr int TI = G::TI, TIP = G::TIP, DW = TIP / 4, DZP = 260, KX = K + S, NC = 4 * kWimg2CT * 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  const int Kt = a.Kt, OC = a.OC, plane = a.IH * a.IW, Kx = a.IC * K * KX;
  const size_t patch = ((size_t)a.IC * TI * TIP + 15) & ~(size_t)15;
  unsigned char* tile = smem;
  float* dzl = reinterpret_cast<float*>(smem + patch);  // [OC][DZP]: pixel 16 ly + lx
  // B columns: extended tap col (gathered), the bias column (col == Kx) or padding
  int ko[kWimg2CT];
  float cb[kWimg2CT];  // 1 for the bias column, 0 for padding columns, -1 for gathered columns
#pragma unroll
  for (int u = 0; u < kWimg2CT; ++u) {
    const int col = (wave * kWimg2CT + u) * 16 + j;
    const int ic = col / (K * KX), rem = col - ic * (K * KX), ky = rem / KX, kxp = rem - ky * KX;
    ko[u] = col < Kx ? (ic * TI + ky) * TIP + kxp : 0;
    cb[u] = col < Kx ? -1.0f : (col == Kx ? 1.0f : 0.0f);
  }
  // A row j: channel j & 7 at the odd (j >= 8) or even column of each pair
  const int aoc = j & 7, adx = j >> 3;
  const float* arow = dzl + (aoc < OC ? aoc : 0) * DZP + adx;
  const float am = aoc < OC ? 1.0f : 0.0f;
  f4 acc[kWimg2CT];
#pragma unroll
  for (int u = 0; u < kWimg2CT; ++u) acc[u] = f4{0.f, 0.f, 0.f, 0.f};
  const size_t total_bytes = (size_t)a.n * a.x_stride;
  const int t0 = blockIdx.x * tpc, t1 = min(tiles, t0 + tpc);
  // staging (round 5): every load of a tile is issued at once into registers through buffer
  // descriptors (out-of-range offsets read 0), then stored, so no load waits on the previous one's
  // store (the loop form serialised ~27 load round trips per tile: 0.15 MFMA-pipe busy, 70 % of wave
  // cycles waiting). Prefetching the next tile during the MFMAs instead took 268 VGPRs (92 now).
  constexpr int NPE = (16 * TI * DW + 255) / 256, NZE = 8;  // launch condition: IC <= 16, OC <= 8
  const int tot = a.IC * TI * DW, OH = a.OP / a.OW;
  unsigned pv[NPE];
  float zv[NZE];
  auto sload = [&](int t) {
    const int smp = t / tps, tt = t - smp * tps, ty = tt / tiles_x, tx = tt - ty * tiles_x;
    const int x0 = tx * kImgTile * S, y0 = ty * kImgTile * S;
    const size_t sb = (size_t)smp * a.x_stride, left = total_bytes - sb;
    const PBuf ib{__builtin_amdgcn_make_buffer_rsrc((void*)(a.x_u8 + sb), (short)0,
                                                    (int)(left < 0xFFFFFFF0u ? left : 0xFFFFFFF0u), 0x00020000)};
#pragma unroll
    for (int i = 0; i < NPE; ++i) {
      const int e = tid + 256 * i, ic = e / (TI * DW), rem = e - ic * (TI * DW), r = rem / DW, d = rem - r * DW;
      const uint32_t off = e < tot ? (uint32_t)(ic * plane + (y0 + r) * a.IW + x0 + 4 * d) : 0xFFFFFFF0u;
      pv[i] = __builtin_amdgcn_raw_buffer_load_b32(ib.r, off, 0, 0);
    }
    const PBuf zb{__builtin_amdgcn_make_buffer_rsrc((void*)(a.dz + (size_t)smp * a.dz_stride), (short)0,
                                                    (int)(a.dz_stride * 4), 0x00020000)};
#pragma unroll
    for (int i = 0; i < NZE; ++i) {
      const int e = tid + 256 * i, oc = e >> 8, px = e & 255, oy = ty * kImgTile + (px >> 4),
                ox = tx * kImgTile + (px & 15);
      const bool in = oc < OC && oy < OH && ox < a.OW;
      const uint32_t off = in ? (uint32_t)(oc * a.OP + oy * a.OW + ox) * 4u : 0x7ffffff0u;
      zv[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(zb.r, off, 0, 0));
    }
  };
  for (int t = t0; t < t1; ++t) {
    sload(t);
    __syncthreads();  // the previous tile's readers are done
#pragma unroll
    for (int i = 0; i < NPE; ++i) {
      const int e = tid + 256 * i, ic = e / (TI * DW), rem = e - ic * (TI * DW), r = rem / DW, d = rem - r * DW;
      if (e < tot) *reinterpret_cast<unsigned*>(tile + (ic * TI + r) * TIP + 4 * d) = pv[i];
    }
#pragma unroll
    for (int i = 0; i < NZE; ++i) {
      const int e = tid + 256 * i;
      if ((e >> 8) < OC) dzl[(e >> 8) * DZP + (e & 255)] = zv[i];
    }
    __syncthreads();
    if constexpr (BX) {
#pragma unroll 1
      for (int q = 0; q < 4; ++q) {
        u32x4 ah, amd, al;
#pragma unroll
        for (int w = 0; w < 4; ++w) {  // slots e = 2 w, 2 w + 1: rows 4 q + w, column pairs g, 4 + g
          const float* ar = arow + 16 * (4 * q + w) + 2 * g;
          unsigned h, md, l;
          split3_pair(ar[0] * am, ar[8] * am, h, md, l);
          ah[w] = h; amd[w] = md; al[w] = l;
        }
        const int po0 = S * 4 * q * TIP + 2 * S * g;
#pragma unroll
        for (int u = 0; u < kWimg2CT; ++u) {
          u32x4 b;
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const int po = po0 + S * w * TIP;  // slot 2 w: column pair g; slot 2 w + 1: pair 4 + g
            float x0 = (float)tile[ko[u] + po], x1 = (float)tile[ko[u] + po + 8 * S];
            if (u >= kWimg2CT - 4 && cb[u] >= 0.0f) { x0 = cb[u]; x1 = cb[u]; }
            b[w] = pack_bf16_exact(x0, x1);
          }
          acc[u] = mfma16bx(al, b, acc[u]);
          acc[u] = mfma16bx(amd, b, acc[u]);
          acc[u] = mfma16bx(ah, b, acc[u]);
        }
      }
    } else {
#pragma unroll 4
    for (int st = 0; st < 32; ++st) {
      const int m = 4 * st + g, ly = m >> 3, lx2 = m & 7;  // column pair (2 lx2, 2 lx2 + 1) of row ly
      const int po = S * ly * TIP + 2 * S * lx2;
      const float av = arow[16 * ly + 2 * lx2] * am;
#pragma unroll
      for (int u = 0; u < kWimg2CT; ++u) {
        const int raw = tile[ko[u] + po];
        const float xv = (float)raw;  // the image's 1 / 255 is applied once, in the combine below
        // the bias and padding columns lie in the last 4 tiles of the last wave (launch condition)
        const float bv = u >= kWimg2CT - 4 ? (cb[u] < 0.0f ? xv : cb[u]) : xv;
        acc[u] = mfma16(av, bv, acc[u]);
      }
    }
    }
  }
  // combine through LDS: D[16][NC] (row 4 g + r, column (wave 9 + u) 16 + j), then
  // dW[oc][(ic, ky, kx)] = D[oc][(ic, ky, kx)] + D[oc + 8][(ic, ky, kx + S)]
  __syncthreads();
  float* dl = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int u = 0; u < kWimg2CT; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) dl[(4 * g + r) * NC + (wave * kWimg2CT + u) * 16 + j] = acc[u][r];
  __syncthreads();
  float* out = a.part + (size_t)blockIdx.x * OC * (Kt + 1);
  for (int e = tid; e < OC * (Kt + 1); e += 256) {
    const int oc = e / (Kt + 1), k = e - oc * (Kt + 1);
    float v;
    if (k == Kt) {
      v = dl[oc * NC + Kx] + dl[(oc + 8) * NC + Kx];
    } else {
      const int ic = k / (K * K), rem = k - ic * (K * K), ky = rem / K, kx = rem - ky * K;
      const int c = (ic * K + ky) * KX + kx;
      v = (dl[oc * NC + c] + dl[(oc + 8) * NC + c + S]) * (1.0f / 255.0f);
    }
    out[e] = v;
  }
}

static int launch_wgrad_generic(WgradArgs a, float* Gw, float* Gb, float* part, size_t part_cap, hipStream_t s,
                                int accum = 0);
int launch_wgrad(WgradArgs a, float* Gw, float* Gb, float* part, size_t part_cap, hipStream_t s, bool img = true,
                 bool bx = false, bool tiled = false) {
  if (a.Kt > kMaxKTab || a.OP > kMaxPTab) return -1;
  const long per = (long)a.OC * (a.Kt + 1);
  const int OH = a.OP / a.OW;
  const bool c2 = a.IC == 8 && a.OC == 16, c3 = a.IC == 16 && a.OC == 32;
  if (img && tiled && a.x_f && a.K == 5 && a.S == 2 && (c2 || c3) && a.dz_stride < (1L << 29) && a.x_stride < (1L << 29)) {
    const int TY = c2 ? kWtTY : kWt2TY, TX = c2 ? kWtTX : kWt2TX;
    const int tiles_x = (a.OW + TX - 1) / TX, tps = tiles_x * ((OH + TY - 1) / TY);
    const long tiles = (long)a.n * tps;
    // one round of resident workgroups: k_wgrad_t three per CU (137 VGPRs), k_wgrad_t2 four (112)
    const int chunks = (int)std::min<long>(tiles, c2 ? 768 : 1024);
    const int groups = (chunks + kSumGroup - 1) / kSumGroup;
    if (tiles < (1L << 31) && (size_t)(chunks + (chunks > kSumGroup ? groups : 0)) * per <= part_cap) {
      a.part = part;
      if (c2)
        hipLaunchKernelGGL((k_wgrad_t<8, 16, kWtTY, kWtTX>), dim3(chunks), dim3(256), 0, s, a, tiles_x, tps, (int)tiles);
      else
        hipLaunchKernelGGL((k_wgrad_t2<16, 32, kWt2TY, kWt2TX>), dim3(chunks), dim3(256), 0, s, a, tiles_x, tps,
                           (int)tiles);
      const unsigned gb = (unsigned)((per + 255) / 256);
      if (chunks > kSumGroup) {
        float* lvl = part + (size_t)chunks * per;
        hipLaunchKernelGGL(k_wsum1, dim3(gb, groups), dim3(256), 0, s, part, chunks, per, lvl);
        hipLaunchKernelGGL(k_wsum, dim3(gb), dim3(256), 0, s, lvl, groups, a.OC, a.Kt, Gw, Gb, 0);
      } else {
        hipLaunchKernelGGL(k_wsum, dim3(gb), dim3(256), 0, s, part, chunks, a.OC, a.Kt, Gw, Gb, 0);
      }
      return 0;
    }
  }
  if (img && a.x_u8 && ((uintptr_t)a.x_u8 & 3) == 0 && a.K == 5 && a.S == 2 && a.OC <= 8 &&
      a.IC * a.K * (a.K + a.S) + 1 <= 4 * kWimg2CT * 16 && a.IC * a.K * (a.K + a.S) >= (4 * kWimg2CT - 4) * 16 &&
      a.IW % 4 == 0 && a.x_stride % 4 == 0 &&
      wimg2_lds_bytes(a.IC, a.K, a.S, a.OC) <= 64 * 1024) {
    const int tiles_x = (a.OW + kImgTile - 1) / kImgTile, tiles_y = (OH + kImgTile - 1) / kImgTile;
    const int tiles = a.n * tiles_x * tiles_y;
    int chunks = std::min(tiles, 768);  // three workgroups per CU (168 VGPRs): one round
    const int tpc = (tiles + chunks - 1) / chunks;
    chunks = (tiles + tpc - 1) / tpc;
    const int groups = (chunks + kSumGroup - 1) / kSumGroup;
    if ((size_t)(chunks + (chunks > kSumGroup ? groups : 0)) * per <= part_cap) {
      a.part = part;
      if (bx)
        hipLaunchKernelGGL((k_wgrad_img2<5, 2, true>), dim3(chunks), dim3(256), wimg2_lds_bytes(a.IC, a.K, a.S, a.OC),
                           s, a, tiles_x, tiles_x * tiles_y, tiles, tpc);
      else
        hipLaunchKernelGGL((k_wgrad_img2<5, 2, false>), dim3(chunks), dim3(256), wimg2_lds_bytes(a.IC, a.K, a.S, a.OC),
                           s, a, tiles_x, tiles_x * tiles_y, tiles, tpc);
      const unsigned gb = (unsigned)((per + 255) / 256);
      if (chunks > kSumGroup) {
        float* lvl = part + (size_t)chunks * per;
        hipLaunchKernelGGL(k_wsum1, dim3(gb, groups), dim3(256), 0, s, part, chunks, per, lvl);
        hipLaunchKernelGGL(k_wsum, dim3(gb), dim3(256), 0, s, lvl, groups, a.OC, a.Kt, Gw, Gb, 0);
      } else {
        hipLaunchKernelGGL(k_wsum, dim3(gb), dim3(256), 0, s, part, chunks, a.OC, a.Kt, Gw, Gb, 0);
      }
      return 0;
    }
  }
  if (img && a.x_u8 && ((uintptr_t)a.x_u8 & 3) == 0 && a.K == 5 && a.S == 2 && a.OC <= 16 &&
      a.Kt + 1 <= 4 * kWimgCT * 16 &&
      a.Kt >= (4 * kWimgCT - 1) * 16 && a.IW % 4 == 0 &&
      a.x_stride % 4 == 0 && wimg_lds_bytes(a.IC, a.K, a.S, a.OC) <= 64 * 1024) {
    const int tiles_x = (a.OW + kImgTile - 1) / kImgTile, tiles_y = (OH + kImgTile - 1) / kImgTile;
    const int tiles = a.n * tiles_x * tiles_y;
    int chunks = std::min(tiles, 1024);
    const int tpc = (tiles + chunks - 1) / chunks;
    chunks = (tiles + tpc - 1) / tpc;
    const int groups = (chunks + kSumGroup - 1) / kSumGroup;
    if ((size_t)(chunks + (chunks > kSumGroup ? groups : 0)) * per <= part_cap) {
      a.part = part;
      hipLaunchKernelGGL((k_wgrad_img<5, 2>), dim3(chunks), dim3(256), wimg_lds_bytes(a.IC, a.K, a.S, a.OC), s, a,
                         tiles_x, tiles_x * tiles_y, tiles, tpc);
      const unsigned gb = (unsigned)((per + 255) / 256);
      if (chunks > kSumGroup) {
        float* lvl = part + (size_t)chunks * per;
        hipLaunchKernelGGL(k_wsum1, dim3(gb, groups), dim3(256), 0, s, part, chunks, per, lvl);
        hipLaunchKernelGGL(k_wsum, dim3(gb), dim3(256), 0, s, lvl, groups, a.OC, a.Kt, Gw, Gb, 0);
      } else {
        hipLaunchKernelGGL(k_wsum, dim3(gb), dim3(256), 0, s, part, chunks, a.OC, a.Kt, Gw, Gb, 0);
      }
      return 0;
    }
  }
  return launch_wgrad_generic(a, Gw, Gb, part, part_cap, s);
}

// the generic gather kernel k_wgrad (+ its chunk sums). Its fp32 gathers use 32-bit buffer offsets
// over the whole input, so an input of >= 0x70000000 bytes runs as consecutive sample groups below
// that size, each group's sums added to the previous ones' (accum)
static int launch_wgrad_generic(WgradArgs a, float* Gw, float* Gb, float* part, size_t part_cap, hipStream_t s,
                                int accum) {
  const long lim = a.group_bytes > 0 && a.group_bytes < (long)kWgradFar ? a.group_bytes : (long)kWgradFar;
  if (!a.x_u8 && (long)a.n * a.x_stride * 4 >= lim) {
    const long ns = (lim / 4 - 1) / (a.x_stride > 0 ? a.x_stride : 1);
    if (ns < 1) return -1;
    for (long s0 = 0; s0 < a.n; s0 += ns) {
      WgradArgs b = a;
      b.n = (int)std::min<long>(ns, a.n - s0);
      b.x_f = a.x_f + s0 * a.x_stride;
      b.dz = a.dz + s0 * a.dz_stride;
      if (launch_wgrad_generic(b, Gw, Gb, part, part_cap, s, accum || s0 > 0)) return -1;
    }
    return 0;
  }
  const long per = (long)a.OC * (a.Kt + 1);
  const WgradPlan p = plan_wgrad(a.OC, a.Kt, (long)a.n * a.OP);
  if (p.part_floats > part_cap) return -1;
  a.qchunk = p.qchunk;
  a.part = part;
  const dim3 grid(p.chunks, p.ocg, p.kg);
  if (a.x_u8) {
    if (p.not_ == 4) hipLaunchKernelGGL((k_wgrad<4, kWgradNKT, true>), grid, dim3(256), 0, s, a);
    else if (p.not_ == 2) hipLaunchKernelGGL((k_wgrad<2, kWgradNKT, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_wgrad<1, kWgradNKT, true>), grid, dim3(256), 0, s, a);
  } else {
    if (p.not_ == 4) hipLaunchKernelGGL((k_wgrad<4, kWgradNKT, false>), grid, dim3(256), 0, s, a);
    else if (p.not_ == 2) hipLaunchKernelGGL((k_wgrad<2, kWgradNKT, false>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_wgrad<1, kWgradNKT, false>), grid, dim3(256), 0, s, a);
  }
  const unsigned gb = (unsigned)((per + 255) / 256);
  if (p.chunks > kSumGroup) {
    // level 1 writes its group sums after the chunk partials (sized by plan_wgrad)
    const int groups = (p.chunks + kSumGroup - 1) / kSumGroup;
    float* lvl = part + (size_t)p.chunks * per;
    hipLaunchKernelGGL(k_wsum1, dim3(gb, groups), dim3(256), 0, s, part, p.chunks, per, lvl);
    hipLaunchKernelGGL(k_wsum, dim3(gb), dim3(256), 0, s, lvl, groups, a.OC, a.Kt, Gw, Gb, accum);
  } else {
    hipLaunchKernelGGL(k_wsum, dim3(gb), dim3(256), 0, s, part, p.chunks, a.OC, a.Kt, Gw, Gb, accum);
  }
  return 0;
}

}  // namespace

// the largest wgrad partial buffer any layer needs at max_batch rows
static size_t carla_part_floats(const ppo_carla_layout& L, long B) {
  size_t m = 0;
  auto need = [&](int OC, int Kt, long Q) {
    const size_t f = plan_wgrad(OC, Kt, Q).part_floats;
    if (f > m) m = f;
  };
  for (int i = 0; i < PPO_CARLA_NCONV; ++i)
    need(L.conv_oc[i], L.conv_ic[i] * L.conv_k[i] * L.conv_k[i], B * L.conv_oh[i] * L.conv_ow[i]);
  need(512, 1280, B);
  need(256, 512, B);
  need(256, L.NM, B);
  need(256, 256, B);
  need(256, 256 + L.NV, B);
  need(1, 256, B);
  need(L.A, 256, B);
  return m;
}

static int carla_train_init(ppo_carla_t* c) {
  if (c->train_ready) return 0;
  const ppo_carla_layout& L = c->L;
  const size_t B = (size_t)c->cfg.max_batch;
  int rc = 0;
  rc |= carla_alloc(&c->G, L.P);
  rc |= carla_alloc(&c->m, L.P);
  rc |= carla_alloc(&c->v, L.P);
  for (int i = 0; i < PPO_CARLA_NCONV - 1; ++i)
    rc |= carla_alloc(&c->dact[i], B * L.conv_oc[i] * L.conv_oh[i] * L.conv_ow[i]);
  rc |= carla_alloc(&c->denc, B * 1280);
  rc |= carla_alloc(&c->ds1, B * 256);
  rc |= carla_alloc(&c->dl1, B * 512);
  rc |= carla_alloc(&c->dfeat, B * 256);
  rc |= carla_alloc(&c->dv1, B * 256);
  rc |= carla_alloc(&c->dv2, B * 256);
  rc |= carla_alloc(&c->dp1, B * 256);
  rc |= carla_alloc(&c->dp2, B * 256);
  rc |= carla_alloc(&c->dhead, B * 2 * L.A);
  rc |= carla_alloc(&c->dval, B);
  rc |= carla_alloc(&c->lp, B);
  rc |= carla_alloc(&c->ent, B);
  rc |= carla_alloc(&c->rowstat, B * 8);
  c->part_floats = carla_part_floats(L, (long)B);
  rc |= carla_alloc(&c->part, c->part_floats);
  size_t dcol_f = 1, wt_f = 1, zb_f = 1;
  for (int i = 1; i < PPO_CARLA_NCONV; ++i)
    if (dgrad_col_layer(L.conv_oh[i], L.conv_ow[i], L.conv_k[i], L.conv_s[i])) {
      const size_t kt = (size_t)L.conv_ic[i] * L.conv_k[i] * L.conv_k[i];
      dcol_f = std::max(dcol_f, B * kt * L.conv_oh[i] * L.conv_ow[i]);
      wt_f = std::max(wt_f, kt * L.conv_oc[i]);
      zb_f = std::max(zb_f, kt);
    }
  rc |= carla_alloc(&c->dcol, dcol_f);
  rc |= carla_alloc(&c->wt, wt_f);
  rc |= carla_alloc(&c->zbias, zb_f);
  // [0,2) adv mean/std, [64,71) stats + {total, coef}, [128,288) int64 tensor table, [320,...) norm slices
  rc |= carla_alloc(&c->small, 320 + PPO_CARLA_MAX_TENSORS * kNormSplit);
  if (rc) return ppo_fail("ppo_carla_update: device allocation failed", -2);
  // tensor table (offsets / lengths as int64) after the scalars
  std::vector<long> tab(2 * PPO_CARLA_MAX_TENSORS, 0);
  for (int t = 0; t < L.ntensors; ++t) {
    tab[t] = L.t_off[t];
    tab[PPO_CARLA_MAX_TENSORS + t] = L.t_grad[t] ? L.t_len[t] : 0;
  }
  if (hipMemcpy(c->small + 128, tab.data(), tab.size() * sizeof(long), hipMemcpyHostToDevice) != hipSuccess)
    return ppo_fail("ppo_carla_update: copy failed", -2);
  c->train_ready = true;
  return 0;
}

extern "C" int ppo_carla_update(ppo_carla_t* c, const ppo_carla_train_config* tc, int n, const uint8_t* bev,
                                const float* meas, const float* vmeas, const float* actions, const float* old_logp,
                                const float* adv, const float* ret, const float* old_v, float lr,
                                ppo_carla_update_stats* stats, void* stream) {
  if (!c || !tc || !bev || !meas || !actions || !old_logp || !adv || !ret || !old_v || (!vmeas && c->L.NV > 0))
    return ppo_fail("ppo_carla_update: null argument", -1);
  if (n <= 1 && tc->norm_adv) return ppo_fail("ppo_carla_update: advantage normalisation needs n >= 2", -1);
  if (n <= 0 || n > c->cfg.max_batch) return ppo_fail("ppo_carla_update: n must be in [1, max_batch]", -1);
  if (hipSetDevice(c->device) != hipSuccess) return ppo_fail("ppo_carla_update: hipSetDevice failed", -2);
  int rc = carla_train_init(c);
  if (rc) return rc;
  const ppo_carla_layout& L = c->L;
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  // forward with the given actions (ac_ppo_carla.cpp:543-546); activations stay in the context
  rc = ppo_carla_forward(c, n, bev, meas, vmeas, PPO_CARLA_GIVEN, actions, 0, 0, nullptr, c->lp, c->ent, nullptr,
                         nullptr, nullptr, s);
  if (rc) return rc;
  float* P = c->P;
  float* G = c->G;
  float* sm = c->small;
  if (tc->norm_adv) {
    if (c->comm) {  // ac_ppo_carla.cpp:564-578: averaged mean, summed squares, Bessel over world * n
      hipLaunchKernelGGL(k_carla_adv_part, dim3(1), dim3(256), 0, s, adv, n, sm, 0);
      if (ncclAllReduce(sm, sm, 1, ncclFloat, ncclAvg, c->comm, s) != ncclSuccess)
        return ppo_fail("ppo_carla_update: advantage mean all-reduce failed", -3);
      hipLaunchKernelGGL(k_carla_adv_part, dim3(1), dim3(256), 0, s, adv, n, sm, 1);
      if (ncclAllReduce(sm + 2, sm + 2, 1, ncclFloat, ncclSum, c->comm, s) != ncclSuccess)
        return ppo_fail("ppo_carla_update: advantage variance all-reduce failed", -3);
      hipLaunchKernelGGL(k_carla_adv_fin, dim3(1), dim3(64), 0, s, sm, (float)(c->world * n - 1));
    } else {
      hipLaunchKernelGGL(k_carla_advstats, dim3(1), dim3(256), 0, s, adv, n, sm);
    }
  }
  HeadBwdArgs hb{P,      L.hi,    L.lo,      c->hpre,   actions,     c->lp,        c->ent,        c->val,
                 old_logp, adv,   ret,       old_v,     sm,          n,            L.A,           c->cfg.beta_min,
                 tc->clip_coef, tc->ent_coef, tc->vf_coef, tc->norm_adv, tc->clip_vloss, c->dhead, c->dval, c->rowstat};
  hipLaunchKernelGGL(k_carla_head_bwd, dim3((n + 63) / 64), dim3(64), 0, s, hb);
  int bad = 0;
  // y = x W^T + b on rows: dz [n][OUT] (stride dzs), x [n][IN] (stride xs)
  auto lin_w = [&](const float* dz, long dzs, int OUT, const float* x, long xs, int IN, long w, long b) {
    WgradArgs a{dz, dzs, OUT, 1, 1, x, nullptr, xs, IN, 1, 1, 1, 1, n, IN, 0, nullptr, c->wgrad_group};
    bad |= launch_wgrad(a, G + w, G + b, c->part, c->part_floats, s);
  };
  auto lin_d = [&](const float* dz, long dzs, int OUT, long w, int w_in, const float* x, long xs, float* dx, long dxs,
                   int IN, int accumulate) {
    DgradArgs a{dz, dzs, P + w, w_in, x, xs, dx, dxs, IN, 1, 1, OUT, 1, 1, 1, 1, n, accumulate};
    bad |= launch_dgrad(a, s);
  };
  const long FW = 256 + L.NV;
  const int A = L.A;
  // heads (carla_model.h:279-284): dist_mu / dist_sigma on the policy latent
  lin_w(c->dhead, 2 * A, A, c->p2, 256, 256, L.mu_w, L.mu_b);
  lin_w(c->dhead + A, 2 * A, A, c->p2, 256, 256, L.sg_w, L.sg_b);
  lin_d(c->dhead, 2 * A, A, L.mu_w, 256, c->p2, 256, c->dp2, 256, 256, 0);
  lin_d(c->dhead + A, 2 * A, A, L.sg_w, 256, c->p2, 256, c->dp2, 256, 256, 1);
  // policy_head (:279)
  lin_w(c->dp2, 256, 256, c->p1, 256, 256, L.pi_w[1], L.pi_b[1]);
  lin_d(c->dp2, 256, 256, L.pi_w[1], 256, c->p1, 256, c->dp1, 256, 256, 0);
  lin_w(c->dp1, 256, 256, c->feat, FW, 256, L.pi_w[0], L.pi_b[0]);
  lin_d(c->dp1, 256, 256, L.pi_w[0], 256, c->feat, FW, c->dfeat, 256, 256, 0);
  // value_head (:276-277)
  lin_w(c->dval, 1, 1, c->v2, 256, 256, L.v_w[2], L.v_b[2]);
  lin_d(c->dval, 1, 1, L.v_w[2], 256, c->v2, 256, c->dv2, 256, 256, 0);
  lin_w(c->dv2, 256, 256, c->v1, 256, 256, L.v_w[1], L.v_b[1]);
  lin_d(c->dv2, 256, 256, L.v_w[1], 256, c->v1, 256, c->dv1, 256, 256, 0);
  lin_w(c->dv1, 256, 256, c->feat, FW, (int)FW, L.v_w[0], L.v_b[0]);
  lin_d(c->dv1, 256, 256, L.v_w[0], (int)FW, c->feat, FW, c->dfeat, 256, 256, 1);
  // linear (:240) and state_linear (:238)
  lin_w(c->dfeat, 256, 256, c->l1, 512, 512, L.lin_w[1], L.lin_b[1]);
  lin_d(c->dfeat, 256, 256, L.lin_w[1], 512, c->l1, 512, c->dl1, 512, 512, 0);
  lin_w(c->dl1, 512, 512, c->enc, 1280, 1280, L.lin_w[0], L.lin_b[0]);
  lin_d(c->dl1, 512, 512, L.lin_w[0], 1280, c->enc, 1280, c->denc, 1280, 1280, 0);
  lin_w(c->denc + 1024, 1280, 256, c->s1, 256, 256, L.st_w[1], L.st_b[1]);
  lin_d(c->denc + 1024, 1280, 256, L.st_w[1], 256, c->s1, 256, c->ds1, 256, 256, 0);
  lin_w(c->ds1, 256, 256, meas, L.NM, L.NM, L.st_w[0], L.st_b[0]);
  // cnn (:236), last layer first; conv i reads act[i-1] (the image for i = 0)
  for (int i = PPO_CARLA_NCONV - 1; i >= 0; --i) {
    const float* dz = i == PPO_CARLA_NCONV - 1 ? c->denc : c->dact[i];
    const long dzs = i == PPO_CARLA_NCONV - 1 ? 1280 : (long)L.conv_oc[i] * L.conv_oh[i] * L.conv_ow[i];
    const float* xf = i > 0 ? c->act[i - 1] : nullptr;
    const long xs = (long)L.conv_ic[i] * L.conv_ih[i] * L.conv_iw[i];
    WgradArgs wa{dz,          dzs,         L.conv_oc[i], L.conv_oh[i] * L.conv_ow[i], L.conv_ow[i], xf,
                 i ? nullptr : bev, xs,    L.conv_ic[i], L.conv_ih[i],                L.conv_iw[i], L.conv_k[i],
                 L.conv_s[i], n,           L.conv_ic[i] * L.conv_k[i] * L.conv_k[i], 0, nullptr, c->wgrad_group};
    bad |= launch_wgrad(wa, G + L.conv_w[i], G + L.conv_b[i], c->part, c->part_floats, s, c->conv_img, c->c1bx,
                        c->wgrad_t);
    if (i > 0) {
      DgradArgs da{dz,           dzs,          P + L.conv_w[i], L.conv_ic[i], xf,           xs,
                   c->dact[i - 1], xs,         L.conv_ic[i],    L.conv_ih[i], L.conv_iw[i], L.conv_oc[i],
                   L.conv_oh[i], L.conv_ow[i], L.conv_k[i],     L.conv_s[i],  n,            0};
      if (c->dgrad_col && dgrad_col_layer(L.conv_oh[i], L.conv_ow[i], L.conv_k[i], L.conv_s[i])) {
        const int kt = L.conv_ic[i] * L.conv_k[i] * L.conv_k[i], OP = L.conv_oh[i] * L.conv_ow[i];
        hipLaunchKernelGGL(k_wtrans, dim3((unsigned)(((long)kt * L.conv_oc[i] + 255) / 256)), dim3(256), 0, s,
                           P + L.conv_w[i], L.conv_oc[i], kt, c->wt);
        ConvArgs ca{dz,     nullptr, dzs, L.conv_oc[i], L.conv_oh[i], L.conv_ow[i], c->wt, c->zbias, c->dcol,
                    (long)kt * OP, kt, L.conv_oh[i], L.conv_ow[i], 1, 1, 0, n, nullptr, 0};
        bad |= launch_conv(ca, s, 0);
        const long tot = (long)n * xs;
        const dim3 cg((unsigned)((tot + 255) / 256));
        if (L.conv_s[i] == 1)
          hipLaunchKernelGGL((k_col2im<3, 1>), cg, dim3(256), 0, s, c->dcol, xf, xs, c->dact[i - 1], xs, L.conv_ic[i],
                             L.conv_ih[i], L.conv_iw[i], L.conv_oh[i], L.conv_ow[i], n, 0);
        else
          hipLaunchKernelGGL((k_col2im<3, 2>), cg, dim3(256), 0, s, c->dcol, xf, xs, c->dact[i - 1], xs, L.conv_ic[i],
                             L.conv_ih[i], L.conv_iw[i], L.conv_oh[i], L.conv_ow[i], n, 0);
      } else {
        bad |= launch_dgrad(da, s, c->conv_img, c->dgrad_q);
      }
    }
  }
  if (bad) return ppo_fail("ppo_carla_update: no gradient kernel for this shape", -1);
  const long begin = 2;  // action_space_high / _low carry no gradient (registered with requires_grad false)
  // gradient average over ranks before clipping (ac_ppo_carla.cpp:608-616)
  if (c->comm && ncclAllReduce(G + begin, G + begin, (size_t)(L.P - begin), ncclFloat, ncclAvg, c->comm, s) != ncclSuccess)
    return ppo_fail("ppo_carla_update: gradient all-reduce failed", -3);
  // clip_grad_norm_ + Adam (ac_ppo_carla.cpp:618-619)
  const long* toff = (const long*)(sm + 128);
  hipLaunchKernelGGL(k_carla_tnorm, dim3(L.ntensors, kNormSplit), dim3(256), 0, s, G, toff,
                     toff + PPO_CARLA_MAX_TENSORS, sm + 320);
  hipLaunchKernelGGL(k_carla_tsum, dim3(1), dim3(64), 0, s, sm + 320, L.ntensors, tc->max_grad_norm, sm + 70);
  c->step += 1;
  const double bc1 = 1.0 - std::pow(0.9, (double)c->step), bc2 = 1.0 - std::pow(0.999, (double)c->step);
  CarlaAdamArgs ad{P, G, c->m, c->v, begin, L.P - begin, sm + 70, (float)((double)lr / bc1), (float)std::sqrt(bc2),
                   tc->adam_eps};
  hipLaunchKernelGGL(k_carla_adam, dim3((unsigned)((L.P - begin + 255) / 256)), dim3(256), 0, s, ad);
  hipLaunchKernelGGL(k_carla_stats, dim3(1), dim3(256), 0, s, c->rowstat, n, sm + 64);
  if (hipGetLastError() != hipSuccess) return ppo_fail("ppo_carla_update: launch failed", -2);
  if (stats) {
    // loss statistics averaged over ranks (ac_ppo_carla.cpp:645-651); the total norm is global already
    if (c->comm && ncclAllReduce(sm + 64, sm + 64, 6, ncclFloat, ncclAvg, c->comm, s) != ncclSuccess)
      return ppo_fail("ppo_carla_update: statistics all-reduce failed", -3);
    float h[8];
    if (hipMemcpyAsync(h, sm + 64, sizeof h, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
      return ppo_fail("ppo_carla_update: stats copy failed", -2);
    stats->pg_loss = h[0];
    stats->v_loss = h[1];
    stats->entropy = h[2];
    stats->old_approx_kl = h[3];
    stats->approx_kl = h[4];
    stats->clipfrac = h[5];
    stats->grad_norm = h[6];
  }
  return 0;
}

static int carla_d2h(ppo_carla_t* c, const float* dev, float* host, long n, const char* what) {
  if (!c || !host) return ppo_fail(std::string(what) + ": null argument", -1);
  if (n != c->L.P) return ppo_fail(std::string(what) + ": expected " + std::to_string(c->L.P) + " floats", -1);
  if (!dev) return ppo_fail(std::string(what) + ": no training state yet (call ppo_carla_update first)", -1);
  if (hipSetDevice(c->device) != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess || hipMemcpy(host, dev, sizeof(float) * n, hipMemcpyDeviceToHost) != hipSuccess)
    return ppo_fail(std::string(what) + ": copy failed", -2);
  return 0;
}

extern "C" int ppo_carla_save_params(ppo_carla_t* c, float* host, long n) {
  return carla_d2h(c, c ? c->P : nullptr, host, n, "ppo_carla_save_params");
}

extern "C" int ppo_carla_last_grad(ppo_carla_t* c, float* host, long n) {
  return carla_d2h(c, c ? c->G : nullptr, host, n, "ppo_carla_last_grad");
}

extern "C" int ppo_carla_save_adam(ppo_carla_t* c, float* m_host, float* v_host, long n, long* step) {
  if (!c || !step) return ppo_fail("ppo_carla_save_adam: null argument", -1);
  if (!c->train_ready) {  // a fresh optimizer
    if (!m_host || !v_host || n != c->L.P) return ppo_fail("ppo_carla_save_adam: bad arguments", -1);
    std::fill(m_host, m_host + n, 0.0f);
    std::fill(v_host, v_host + n, 0.0f);
    *step = 0;
    return 0;
  }
  int rc = carla_d2h(c, c->m, m_host, n, "ppo_carla_save_adam");
  if (!rc) rc = carla_d2h(c, c->v, v_host, n, "ppo_carla_save_adam");
  *step = c->step;
  return rc;
}

extern "C" int ppo_carla_load_adam(ppo_carla_t* c, const float* m_host, const float* v_host, long n, long step) {
  if (!c || !m_host || !v_host) return ppo_fail("ppo_carla_load_adam: null argument", -1);
  if (n != c->L.P || step < 0) return ppo_fail("ppo_carla_load_adam: bad arguments", -1);
  if (hipSetDevice(c->device) != hipSuccess) return ppo_fail("ppo_carla_load_adam: hipSetDevice failed", -2);
  int rc = carla_train_init(c);
  if (rc) return rc;
  if (hipMemcpy(c->m, m_host, sizeof(float) * n, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->v, v_host, sizeof(float) * n, hipMemcpyHostToDevice) != hipSuccess)
    return ppo_fail("ppo_carla_load_adam: copy failed", -2);
  c->step = step;
  return 0;
}

// ------------------------------------------------------------------------------------------
// data parallelism: RCCL communicator (replaces torchfort::Comm, distributed.cpp:81-224)
// ------------------------------------------------------------------------------------------
extern "C" int ppo_carla_comm_init(ppo_carla_t* c, const char* id, int rank, int world) {
  if (!c || !id) return ppo_fail("ppo_carla_comm_init: null argument", -1);
  if (world < 1 || rank < 0 || rank >= world) return ppo_fail("ppo_carla_comm_init: bad rank / world", -1);
  if (hipSetDevice(c->device) != hipSuccess) return ppo_fail("ppo_carla_comm_init: hipSetDevice failed", -2);
  if (c->comm) {
    (void)ncclCommDestroy(c->comm);
    c->comm = nullptr;
  }
  ncclUniqueId uid;
  static_assert(sizeof(ncclUniqueId) <= PPO_COMM_ID_BYTES, "ncclUniqueId size");
  memcpy(&uid, id, sizeof(uid));
  const ncclResult_t r = ncclCommInitRank(&c->comm, world, uid, rank);
  if (r != ncclSuccess) {
    c->comm = nullptr;
    return ppo_fail(std::string("ppo_carla_comm_init: ncclCommInitRank: ") + ncclGetErrorString(r), -3);
  }
  c->rank = rank;
  c->world = world;
  return 0;
}

extern "C" int ppo_carla_comm_broadcast_params(ppo_carla_t* c, int root) {
  if (!c) return ppo_fail("ppo_carla_comm_broadcast_params: null argument", -1);
  if (!c->comm) return 0;
  if (hipSetDevice(c->device) != hipSuccess) return ppo_fail("ppo_carla_comm_broadcast_params: hipSetDevice failed", -2);
  if (ncclBroadcast(c->P, c->P, (size_t)c->L.P, ncclFloat, root, c->comm, c->stream) != ncclSuccess)
    return ppo_fail("ppo_carla_comm_broadcast_params: ncclBroadcast failed", -3);
  return hipStreamSynchronize(c->stream) == hipSuccess ? 0 : ppo_fail("ppo_carla_comm_broadcast_params: sync failed", -2);
}
