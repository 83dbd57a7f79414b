// ppo_update_narrow.hip — k_upd2: the fused minibatch forward / PPO loss / backward of the PPO
// agent (two 64-wide tanh trunks + Normal head, ppo:120-157; loss and backward ppo:495-538) with
// BOTH trunks in one workgroup, for any observation width (cfg1 HalfCheetah O = 17, cfg2
// Humanoid O = 376).
//
// Why a separate kernel: at H = 64 the work is dominated by layer 1 (K = O = 376 against N = 64),
// and the wave-per-16-rows k_fwdbwd re-streams each trunk's 96 KB W1 per 64 rows through a
// barrier per 16-column k-tile and then recomputes layer 1 for the backward. Here:
//  * a workgroup (4 waves) owns 32 rows per tile; waves 0-1 are the critic, 2-3 the actor, and
//    each wave owns 32 output features x 32 rows (2 x 2 accumulator tiles of 16x16x4 f32 MFMA),
//    so every W1 A-operand load feeds 8 MFMAs;
//  * the gathered observation rows are staged ONCE in LDS for both trunks, in 128-column chunks
//    moved by LDS DMA (buffer_load ... lds: no staging registers; out-of-range columns and rows
//    read as 0), double-buffered (the next chunk's gather is in flight under the current chunk's
//    MFMAs, the last chunk prefetches the next tile's first one), 16-byte units XOR-swizzled by
//    row so the B-operand ds_read_b128 stay conflict-free without row padding;
//  * the next tile's per-row data (return, value, old log-prob, advantage, actions) is DMA'd into
//    LDS once this tile's loss no longer needs it, through permutation entries loaded a tile ahead:
//    no dependent perm -> data round trip at a tile's start;
//  * tanh' needs only h1, which stays in registers: no layer-1 recompute;
//  * bias / head-weight / logstd gradients and the loss statistics accumulate in registers over
//    all of a workgroup's tiles and are reduced across lanes once, in a fixed order, at the end.
// The dW1 / dW2 GEMMs stay in k_dw, which gathers the observation rows through the permutation
// itself (no Xn round trip: the PPO agent has no input normalisation).
#include "ppo_agent.hpp"
#include "ppo_kernels.hpp"

#ifdef PPO_STAMPS
// diagnostic build only: per-wave shader-clock stamps at the phase ends of the first 16 tiles of
// every workgroup ([wg][wave][tile][start, 12 phase ends, hardware wave id]), read by
// ppo_diag_read_stamps2 (scripts/diag_stamps2.py)
#define PPO2_NSTAMP 12
#define PPO2_TILES 16
#define PPO2_REC (PPO2_NSTAMP + 2)
__device__ unsigned long long g_upd2_stamps[512 * 4 * PPO2_TILES * PPO2_REC];
#define PPO2_STAMP(k)                                                                                \
  do {                                                                                               \
    const int tt_ = (it - (int)blockIdx.x) / (int)gridDim.x;                                         \
    if (tt_ >= 0 && tt_ < PPO2_TILES && blockIdx.x < 512 && lane == 0)                              \
      g_upd2_stamps[((blockIdx.x * 4 + wave) * PPO2_TILES + tt_) * PPO2_REC + (k)] =                \
          __builtin_amdgcn_s_memtime();                                                              \
  } while (0)
#define PPO2_STAMP_ID()                                                                              \
  do {                                                                                               \
    const int tt_ = (it - (int)blockIdx.x) / (int)gridDim.x;                                         \
    if (tt_ >= 0 && tt_ < PPO2_TILES && blockIdx.x < 512 && lane == 0)                              \
      g_upd2_stamps[((blockIdx.x * 4 + wave) * PPO2_TILES + tt_) * PPO2_REC + PPO2_NSTAMP + 1] =    \
          (unsigned long long)__builtin_amdgcn_s_getreg(0xF804) |                                    \
          ((unsigned long long)__builtin_amdgcn_s_getreg(0xF814) << 32);                             \
  } while (0)
#else
#define PPO2_STAMP(k) do {} while (0)
#define PPO2_STAMP_ID() do {} while (0)
#endif

typedef float f16v2 __attribute__((ext_vector_type(16)));

namespace {

// tanh of the update's forward recompute: (1 - e) / (1 + e) with e = exp(-2|x|) on v_exp_f32 /
// v_rcp_f32, sign restored — 8 instructions instead of the device library's 27 (a third of this
// kernel's VALU went to tanhf). Absolute error about 1e-7 for every x (the relative error grows as
// |x| -> 0: 3e-5 at |x| = 1e-3); the update tests' gradient bars (rel-L2 2e-4 against LibTorch,
// 2e-5 against k_fwdbwd) are far above what this moves.
// The rollout's act kernels keep tanhf: their samples are compared with the oracle.
PPO_DEV float tanh_upd(float x) {
  const float e = __builtin_amdgcn_exp2f(-2.8853900817779268f * __builtin_fabsf(x));
  const float t = (1.0f - e) * __builtin_amdgcn_rcpf(1.0f + e);
  return __builtin_copysignf(t, x);
}

constexpr int H2 = 64, FT2 = 2, RT2 = 2, R2 = 32, LDA2 = H2 + 4;

template <int NTO, int NHT, int VEC, int NUA, int SPLIT = 0>
struct Geo2 {
  static constexpr int OP = NTO * 16;
  static constexpr int CKB = NTO < 8 ? NTO : 8;      // k-blocks (16 columns) per staged X chunk
  static constexpr int NCH = (NTO + CKB - 1) / CKB;  // chunks per tile
  static constexpr int CW = CKB * 16;                // columns per chunk
  static constexpr int LDX = CW;                     // unpadded rows (DMA writes 64 lanes x VEC floats)
  static constexpr int UPR = CW / 4;                 // 16-byte units per row
  static constexpr int SWZ = (UPR % 16 == 0) ? 16 : (UPR % 8 == 0) ? 8 : 4;  // unit XOR swizzle span
  static constexpr int NB = 2;  // X chunk buffers, alternating by running chunk count (a DMA lands at once)
  static constexpr int NHP = NHT * 16, LDG = NHP + 4;
  static constexpr int PERROW = VEC == 4 ? UPR : CW;     // DMA lanes per row and chunk
  static constexpr int NGI = R2 * PERROW / 256;          // DMA instructions per wave per chunk
  static_assert(R2 * PERROW % 256 == 0, "chunk must be a whole number of DMA instructions per wave");
  static constexpr int NU = NUA;                         // (row, action) items per thread: ceil(R A / 256)
  // LDS carve (floats); the (row, action) item and action regions follow at runtime offsets
  static constexpr int oXS = 0;
  // split form (k_l1g computed layer 1): no X staging
  static constexpr int oACT = oXS + (SPLIT ? 0 : NB * R2 * LDX);  // [2 trunks][R][LDA]: h1, then h2, then dz2
  static constexpr int oSCR = oACT + 2 * R2 * LDA2;    // actor head partials [2][NHP][R] | critic [2][R]
  static constexpr int oGG = oSCR + 2 * NHP * R2 + 2 * R2;  // [R][LDG] d loss / d mu
  static constexpr int oROWS = oGG + R2 * LDG;          // [R][8] per-row scalars computed by the loss
  static constexpr int oRD = oROWS + R2 * 8;            // [4][64] DMA'd return | value | old log-prob | advantage
  static constexpr int oSP = oRD + 4 * 64;              // head biases | sd | var | log sd (NHP each) | critic bias
  static constexpr int oITM = oSP + 4 * NHP + 4;        // [R*A][4] items, then [64 ceil(R*A / 64)] actions
};

// k_upd2 BX: W1 piece units (32 k x FT feature tiles) in flight ahead; 2 spills 31 VGPRs and runs
// slower (profiles/r05/bx6_cfg2/split_once)
constexpr int kBx2Ring = 1;
PPO_DEV float lf(const float* p) { return *p; }
PPO_DEV f4 lf4(const float* p) { return *reinterpret_cast<const f4*>(p); }
PPO_DEV void sf4(float* p, f4 v) { *reinterpret_cast<f4*>(p) = v; }
PPO_DEV float bl1(PBuf b, int lane_floats, int uni_floats) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(b.r, lane_floats * 4, uni_floats * 4, 0));
}

// buffer resource over `bytes` bytes (offsets at or past the end read as 0)
PPO_DEV PBuf make_pbuf_b(const void* base, uint32_t bytes) {
  return PBuf{__builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000)};
}
constexpr uint32_t kOOB = 0xFFFFFFF0u;  // a byte offset past every buffer: the DMA writes zeros
// LDS DMA: every lane of the wave loads `size` bytes at its byte offset into lds_wave + lane * size
// (lds_wave must be wave-uniform); completion is counted by vmcnt
template <int SIZE, int AUX = 0>
PPO_DEV void dma(PBuf b, float* lds_wave, uint32_t voff) {
  auto* l = (__attribute__((address_space(3))) void*)lds_wave;
  if constexpr (SIZE == 16) __builtin_amdgcn_raw_ptr_buffer_load_lds(b.r, l, 16, voff, 0, 0, AUX);
  else __builtin_amdgcn_raw_ptr_buffer_load_lds(b.r, l, 4, voff, 0, 0, AUX);
}
// cache policy of k_dw2_dma's read-once streams (gathered X rows, DZ1 / DZ2 / H1 blocks): 2 non-temporal
// (cfg2 88.8 -> 88.3 ms per iteration: k_colsum then finds more of the split-K partials in cache; bitwise
// the same; profiles/r06/dw2_nt/), 0 the default policy
#ifndef PPO_DW2_AUX
#define PPO_DW2_AUX 2
#endif

// Column sums over the 16 rows j of a lane group: x[4 ft + r] (feature 16 ft + 4 g + r of this lane's
// row) is reduce-scattered with DPP partners j ^ 8 (row_ror:8), the mirror in each half, the mirror in
// each quad, then summed with j ^ 1: lane j returns slot s = j >> 1 summed over all 16 rows
// (feature 16 (s >> 2) + 4 g + (s & 3)); lanes j and j ^ 1 hold the same value. Fixed order.
template <int CTRL, int LEN, int MB>
PPO_DEV void rs8_stage(float (&x)[8], int j) {
  const bool bit = (j & MB) != 0;
#pragma unroll
  for (int i = 0; i < LEN / 2; ++i) {
    const float lo = x[i], hi = x[i + LEN / 2];
    const float keep = bit ? hi : lo, send = bit ? lo : hi;
    x[i] = keep + dpp_f<CTRL>(send);
  }
}
PPO_DEV float colsum8(float (&x)[8], int j) {
  rs8_stage<kDppRowRor8, 8, 8>(x, j);
  rs8_stage<kDppHalfMirror, 4, 4>(x, j);
  rs8_stage<kDppQuadMirror, 2, 2>(x, j);
  return x[0] + dpp_f<kDppQuadXor1>(x[0]);
}

// out[ft][rt] (+)= sum_k W[fbase + 16 ft + i][k] * IN[16 rt + j][k] for a 64-wide input in LDS;
// A operands from the swizzled copy (sw_index: feature tile ft, k-block kb at wlane + 1024 ft + 256 kb)
PPO_DEV void mm64(f4 (&out)[FT2][RT2], PBuf wb, int wlane, const float* in) {
  f4 w[2][FT2];
#pragma unroll
  for (int ft = 0; ft < FT2; ++ft) w[0][ft] = pld4(wb, wlane, 1024 * ft);
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    if (kb + 1 < 4) {
#pragma unroll
      for (int ft = 0; ft < FT2; ++ft) w[(kb + 1) & 1][ft] = pld4(wb, wlane, 1024 * ft + 256 * (kb + 1));
    }
    __builtin_amdgcn_sched_barrier(0);
    f4 b[RT2];
#pragma unroll
    for (int rt = 0; rt < RT2; ++rt) b[rt] = lf4(in + 16 * rt * LDA2 + 16 * kb);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int ft = 0; ft < FT2; ++ft)
#pragma unroll
        for (int rt = 0; rt < RT2; ++rt) out[ft][rt] = mfma16(w[kb & 1][ft][c], b[rt][c], out[ft][rt]);
  }
}

}  // namespace

// SPLIT (2 or 3: workgroups per CU): layer 1's pre-activations come from k_l1g (a.Z1 rows, bias
// included) instead of the staged X chunks and W1: the kernel is the tail only (tanh onwards), with
// a smaller LDS / register footprint (3 per CU: 168 VGPRs, a few spilled registers).
// BX: layer 1 as split-bf16 piece products (upd_mfma=bx6, k_upd's scheme): each staged
// 128-column chunk is split ONCE into bf16 pieces (XP: [32 rows][3 pieces x 128 bf16 + 16 B], in the
// space of ACT and SCR, which layer 1 does not use) by all 256 threads between two barriers; the MFMAs
// then read 3 ds_read_b128 per row tile and 32 k, the W1 pieces come from their bx_index copy
// (k_adam), and six v_mfma_f32_16x16x32_bf16 replace eight x four 16x16x4 f32 ones per (feature
// tile, row tile) and 32 k.
template <int NTO, int NHT, int VEC, int NUA, int SPLIT, int BX = 0>
__global__ __launch_bounds__(256, SPLIT ? SPLIT : 2) void k_upd2(UpdArgs a) {
  using GE = Geo2<NTO, NHT, VEC, NUA, SPLIT>;
  static_assert(!BX || (GE::CW == 128 && NTO % 8 == 0 && !SPLIT), "k_upd2 BX: whole 128-column chunks");
  constexpr int OP = GE::OP, CKB = GE::CKB, NCH = GE::NCH, CW = GE::CW, LDX = GE::LDX, NHP = GE::NHP;
  constexpr int LDG = GE::LDG, PERROW = GE::PERROW, NGI = GE::NGI, NU = GE::NU, UPR = GE::UPR, SWZ = GE::SWZ;
  constexpr int W1D = 3;  // W1 A-operand prefetch depth (k-blocks; 2 -> 3: cfg2 k_upd2 44.05 -> 43.88 ms)
  constexpr int R = R2, FT = FT2, RT = RT2, LDA = LDA2, H = H2;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* XS = lds + GE::oXS;
  float* SCR = lds + GE::oSCR;
  float* GG = lds + GE::oGG;
  float* ROWS = lds + GE::oROWS;
  float* RD = lds + GE::oRD;   // [0] return [64] value [128] old log-prob [192] advantage (DMA)
  float* SHB = lds + GE::oSP;  // actor head biases
  float* SSD = SHB + NHP;      // exp(logstd)
  float* SVAR = SSD + NHP;     // sd^2
  float* SLSD = SVAR + NHP;    // log(sd)
  float* SCB = SLSD + NHP;     // critic head bias
  float* ITM = lds + GE::oITM;
  float* ACTN = lds + a.actn_off;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  const int trunk = wave >> 1, wf = wave & 1, fbase = 32 * wf;
  const PackedLayout& K = a.K;
  const TrunkDev& T = K.tr[trunk];
  const float* __restrict__ P = a.P;
  const PBuf pb = make_pbuf(P, K.size);
  const PBuf wsw = make_pbuf(a.WSW[trunk], (int)sw_size(H, OP));
  const int O = K.O, A = K.A, M = a.M;
  const float c = a.clip_coef;
  const float adv_mean = a.adv_stats[0], adv_std = a.adv_stats[1];
  float* ACT = lds + GE::oACT + trunk * R * LDA;

  for (int i = tid; i < R * LDG; i += 256) GG[i] = 0.f;  // padding heads stay exactly 0
  if (tid < NHP) {
    const bool real = tid < A;
    const float sd = real ? expf(P[K.logstd + tid]) : 1.f;
    SHB[tid] = real ? P[K.ab3 + tid] : 0.f;
    SSD[tid] = sd;
    SVAR[tid] = sd * sd;
    SLSD[tid] = logf(sd);
  }
  if (tid == 0) SCB[0] = P[K.cb3];

  // per-lane A-operand offsets into the swizzled W1 | W2 | W2^T (sw_index)
  const int w1lane = ((fbase >> 4) * NTO * 64 + lane) * 4;
  const int w2lane = H * OP + ((fbase >> 4) * 4 * 64 + lane) * 4;
  const int w2tlane = H * OP + H * H + ((fbase >> 4) * 4 * 64 + lane) * 4;
  const float* act_in = ACT + j * LDA + 4 * g;
  // head operands (loaded per tile from L1/L2): actor forward A = W3[16 ht + j][fbase + 16 ft + 4 g + c],
  // backward A = W3^T: W3[16 ht + 4 g + c][fbase + 16 ft + j]; critic w3[fbase + 16 ft + 4 g + c]
  auto head_fwd = [&](int ht, int ft) -> f4 {
    const int hf = 16 * ht + j;
    return hf < A ? pld4(pb, K.aW3 + hf * H + fbase + 4 * g, 16 * ft) : f4{0.f, 0.f, 0.f, 0.f};
  };
  auto head_bwd = [&](int ht, int ft) -> f4 {
    f4 w;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int hb = 16 * ht + 4 * g + r;
      w[r] = hb < A ? bl1(pb, K.aW3 + hb * H + fbase + j, 16 * ft) : 0.f;
    }
    return w;
  };
  const int ntiles = (M + R - 1) / R;

  // ---- gather of the observation rows, chunk by chunk, through the permutation, by LDS DMA ----
  // DMA lane (u, lane) of wave w covers chunk element e = (w NGI + u) 64 + lane: VEC 4: 16-byte unit
  // e, VEC 1: float e (unit e / 4, component e % 4). Physical unit p of row r holds logical unit
  // p ^ (r & (SWZ - 1)).
  const PBuf ob = make_pbuf_b(a.obs, (uint32_t)min(a.obs_n * 4, (long)0xFFFFFFFF));
  int pcur[NGI], pnext[NGI];
  auto perms_of = [&](int itn, int (&pm)[NGI]) {
#pragma unroll
    for (int u = 0; u < NGI; ++u) {
      const int e = (wave * NGI + u) * 64 + lane, row = e / PERROW, m = itn * R + row;
#ifdef PPO_DIAG
      const int p = a.perm[min(a.hot ? m % (8 * R) : m, M - 1)];  // diagnostic: L2-resident rows
#else
      const int p = a.perm[min(m, M - 1)];  // unconditional (clamped), masked below
#endif
      pm[u] = (itn < ntiles && m < M) ? p : -1;
    }
  };
  // column chunk ch of the rows in pm into X buffer buf
  auto issue = [&](const int (&pm)[NGI], int ch, int buf) {
    float* xs = XS + buf * R * LDX;
#pragma unroll
    for (int u = 0; u < NGI; ++u) {
      const int e = (wave * NGI + u) * 64 + lane;
      const int unit = VEC == 4 ? e : e >> 2, comp = VEC == 4 ? 0 : e & 3;
      const int row = unit / UPR, pu = unit - row * UPR, lu = pu ^ (row & (SWZ - 1));
      const int col = ch * CW + 4 * lu + comp;
      const uint32_t voff = (pm[u] >= 0 && col < O) ? (uint32_t)(pm[u] * O + col) * 4u : kOOB;
      dma<4 * VEC>(ob, xs + (wave * NGI + u) * 64 * VEC, voff);
    }
  };
  // ---- per-row data of a tile into LDS by DMA (RD, ACTN), through permutation entries held a tile ahead ----
  const int NV = (R * A + 63) / 64;  // action DMA instructions (wave w issues v = w, w + 4, ...)
  constexpr int NVW = (R * NHP + 255) / 256;
  const PBuf bret = make_pbuf_b(a.ret, (uint32_t)(a.rows_n * 4)), bval = make_pbuf_b(a.val, (uint32_t)(a.rows_n * 4));
  const PBuf blogp = make_pbuf_b(a.logp, (uint32_t)(a.rows_n * 4)), badv = make_pbuf_b(a.adv, (uint32_t)(a.rows_n * 4));
  const PBuf bact = make_pbuf_b(a.actions, (uint32_t)min(a.rows_n * A * 4, (long)0xFFFFFFFF));
  int prow = -1, pact[NVW];
  auto row_perms = [&](int itn) {
    const int m = itn * R + lane;
    const int p = a.perm[min(m, M - 1)];
    prow = (wave == 0 && lane < R && itn < ntiles && m < M) ? p : -1;
#pragma unroll
    for (int k = 0; k < NVW; ++k) {
      const int idx = (wave + 4 * k) * 64 + lane, row = min(idx, R * A - 1) / A, mm = itn * R + row;
      const int q = a.perm[min(mm, M - 1)];
      pact[k] = (idx < R * A && itn < ntiles && mm < M) ? q : -1;
    }
  };
  auto row_dma = [&]() {
    if (wave == 0) {
      const uint32_t voff = prow >= 0 ? (uint32_t)prow * 4u : kOOB;
      dma<4>(bret, RD, voff);
      dma<4>(bval, RD + 64, voff);
      dma<4>(blogp, RD + 128, voff);
      dma<4>(badv, RD + 192, voff);
    }
#pragma unroll
    for (int k = 0; k < NVW; ++k) {
      const int v = wave + 4 * k;
      if (v < NV) {  // wave-uniform
        const int idx = v * 64 + lane, ai = idx - (min(idx, R * A - 1) / A) * A;
        dma<4>(bact, ACTN + v * 64, pact[k] >= 0 ? (uint32_t)(pact[k] * A + ai) * 4u : kOOB);
      }
    }
  };

  // register accumulators over all of this workgroup's tiles
  // column sums: one slot per lane (colsum8), feature fbase + 16 (s >> 2) + 4 g + (s & 3), s = j >> 1
  float acc_b1 = 0.f, acc_b2 = 0.f, acc_hw = 0.f;
  f4 d3acc[NHT][FT];  // actor dW3 tiles (rows already contracted)
#pragma unroll
  for (int ft = 0; ft < FT; ++ft)
#pragma unroll
    for (int ht = 0; ht < NHT; ++ht) d3acc[ht][ft] = f4{0.f, 0.f, 0.f, 0.f};
  float gacc[NU], lacc[NU];  // per (row, action) item: head-bias and logstd gradient sums
#pragma unroll
  for (int u = 0; u < NU; ++u) { gacc[u] = 0.f; lacc[u] = 0.f; }
  float cbacc = 0.f;                        // critic head bias (tid < R)
  float lst[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // pg, v, ent, old kl, kl, clipfrac (tid < R)

  // split form: this lane's layer-1 pre-activations of a tile (rows 16 rt + j, clamped; masked at use)
  auto z1_load = [&](int itn, f4 (&zz)[FT][RT]) {
#pragma unroll
    for (int ft = 0; ft < FT; ++ft)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const long m = min((long)itn * R + 16 * rt + j, (long)M - 1);
        zz[ft][rt] = ld4(a.Z1 + m * 128 + 64 * trunk + fbase + 16 * ft + 4 * g);
      }
  };
  f4 zn[FT][RT];
  constexpr bool PREF_Z = false;  // next tile's Z1 rows prefetched mid-tile (16 VGPRs: spills at 3 WGs / CU)
  if constexpr (SPLIT) {
    if constexpr (PREF_Z) z1_load(blockIdx.x, zn);
  } else {
    perms_of(blockIdx.x, pcur);
    issue(pcur, 0, 0);
  }
  row_perms(blockIdx.x);
  row_dma();

  int tp = 0;  // buffer of this tile's chunk 0: the running chunk count's parity
  for (int it = blockIdx.x; it < ntiles; it += gridDim.x, tp ^= NCH & 1) {
    const int m0 = it * R;
    PPO2_STAMP(0);
    PPO2_STAMP_ID();
    // chunk 0 and the row data of this tile were DMA'd during the previous tile
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    PPO2_STAMP(1);
    if constexpr (!SPLIT) perms_of(it + gridDim.x, pnext);
    row_perms(it + gridDim.x);
    // ---------------- layer 1 (both trunks share the staged rows) ----------------
    f4 z[FT][RT];
    if constexpr (SPLIT) {
      if constexpr (!PREF_Z) z1_load(it, zn);
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) z[ft][rt] = zn[ft][rt];
    } else {
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      const f4 bv = pld4(pb, T.b1 + fbase + 4 * g, 16 * ft);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) z[ft][rt] = bv;
    }
    if constexpr (BX) {
      constexpr int LDB = 3 * (CW / 2) + 4;  // floats per XP row (row stride 4 mod 64 banks)
      static_assert(R * LDB <= GE::oGG - GE::oACT, "XP must fit in ACT + SCR");
      float* XP = lds + GE::oACT;
      constexpr int NKK = NTO / 2, KPC = CW / 32, D2 = kBx2Ring;  // 32-k units: per tile, per chunk
      const PBuf w1b = make_pbuf(a.WSW[trunk] + sw_size(H, OP), (int)bx_w1_size(H, OP));
      const int w1blane = ((fbase >> 4) * NKK * 3 * 64 + lane) * 4;
      u32x4 wr[D2 + 1][FT][3];
      auto load_w = [&](int kk, u32x4 (&dst)[FT][3]) {
#pragma unroll
        for (int ft = 0; ft < FT; ++ft)
#pragma unroll
          for (int p = 0; p < 3; ++p) dst[ft][p] = __builtin_bit_cast(u32x4, pld4(w1b, w1blane, 256 * ((ft * NKK + kk) * 3 + p)));
      };
      // the chunk in X buffer buf -> its pieces in XP: unit (row, lu) = columns 4 lu .. + 3 at bf16
      // position 32 (lu >> 3) + 8 (lu & 3) + 4 ((lu >> 2) & 1) of each piece (mm_bx's k slots)
      auto split_chunk = [&](int buf) {
        const float* xs = XS + buf * R * LDX;
#pragma unroll
        for (int q = 0; q < R * UPR / 256; ++q) {
          const int un = tid + 256 * q, row = un / UPR, lu = un - row * UPR;
          const f4 x = lf4(xs + row * LDX + 4 * (lu ^ (row & (SWZ - 1))));
          float* qp = XP + row * LDB + 16 * (lu >> 3) + 4 * (lu & 3) + 2 * ((lu >> 2) & 1);
          unsigned h0, m0, l0, h1, m1, l1;
          split3_pair(x[0], x[1], h0, m0, l0);
          split3_pair(x[2], x[3], h1, m1, l1);
          typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
          *reinterpret_cast<u32x2*>(qp) = u32x2{h0, h1};
          *reinterpret_cast<u32x2*>(qp + CW / 2) = u32x2{m0, m1};
          *reinterpret_cast<u32x2*>(qp + CW) = u32x2{l0, l1};
        }
      };
      if (NCH > 1) issue(pcur, 1, tp ^ 1);
      else issue(pnext, 0, tp ^ 1);
#pragma unroll
      for (int q = 0; q < D2 && q < NKK; ++q) load_w(q, wr[q]);
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        const int kp = kk % KPC;
        if (kp == 0) {
          const int ch = kk / KPC;
          if (ch > 0) {
            // chunk ch landed: only the W1 piece loads of units kk .. kk + D2 - 1 may still be in flight
            if constexpr (D2 == 1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            else if constexpr (D2 == 2) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
            else static_assert(D2 == 1 || D2 == 2, "vmcnt: D2 x FT2 x 3 piece loads");
          }
          lds_barrier();  // every wave is done reading XP (the previous chunk) and chunk ch is visible
          split_chunk(tp ^ (ch & 1));
          lds_barrier();
          if (ch > 0) {
            if (ch + 1 < NCH) issue(pcur, ch + 1, tp ^ ((ch + 1) & 1));
            else issue(pnext, 0, tp ^ (NCH & 1));
          }
        }
        if (kk + D2 < NKK) load_w(kk + D2, wr[(kk + D2) % (D2 + 1)]);
        __builtin_amdgcn_sched_barrier(0);
        u32x4 bs[RT][3];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int p = 0; p < 3; ++p)
            bs[rt][p] = __builtin_bit_cast(u32x4, lf4(XP + (16 * rt + j) * LDB + (CW / 2) * p + 16 * kp + 4 * g));
        const u32x4(&av)[FT][3] = wr[kk % (D2 + 1)];
#pragma unroll
        for (int ft = 0; ft < FT; ++ft)
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) {
            f4 acc = z[ft][rt];
            acc = mfma16bx(av[ft][2], bs[rt][0], acc);
            acc = mfma16bx(av[ft][0], bs[rt][2], acc);
            acc = mfma16bx(av[ft][1], bs[rt][1], acc);
            acc = mfma16bx(av[ft][1], bs[rt][0], acc);
            acc = mfma16bx(av[ft][0], bs[rt][1], acc);
            z[ft][rt] = mfma16bx(av[ft][0], bs[rt][0], acc);
          }
      }
      lds_barrier();  // XP (ACT / SCR) is read by no wave any more: h1 goes to ACT next
    } else {
      if (NCH > 1) issue(pcur, 1, tp ^ 1);
      else issue(pnext, 0, tp ^ 1);
      f4 w[W1D + 1][FT];
#pragma unroll
      for (int q = 0; q < W1D && q < NTO; ++q)
#pragma unroll
        for (int ft = 0; ft < FT; ++ft) w[q][ft] = pld4(wsw, w1lane, 256 * NTO * ft + 256 * q);
#pragma unroll
      for (int kb = 0; kb < NTO; ++kb) {
        if (kb > 0 && kb % CKB == 0) {
          // chunk kb / CKB landed: only the W1 loads of k-blocks kb .. kb + 2 may still be in flight
          static_assert(W1D * FT2 == 6, "vmcnt below");
          asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
          lds_barrier();
          const int ch = kb / CKB;
          if (ch + 1 < NCH) issue(pcur, ch + 1, tp ^ ((ch + 1) & 1));
          else issue(pnext, 0, tp ^ (NCH & 1));
        }
        if (kb + W1D < NTO) {
#pragma unroll
          for (int ft = 0; ft < FT; ++ft)
            w[(kb + W1D) % (W1D + 1)][ft] = pld4(wsw, w1lane, 256 * NTO * ft + 256 * (kb + W1D));
        }
        __builtin_amdgcn_sched_barrier(0);
        const int lu = 4 * (kb % CKB) + g;
        const float* xs = XS + (tp ^ ((kb / CKB) & 1)) * R * LDX + j * LDX + 4 * (lu ^ (j & (SWZ - 1)));
        f4 b[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) b[rt] = lf4(xs + 16 * rt * LDX);  // (16 rt + j) & (SWZ - 1) = j & (SWZ - 1)
        const int wq = kb % (W1D + 1);
        // k-step c outermost: 4 independent accumulator chains back to back (16x16x4 f32: 32-cycle
        // issue, 40-cycle dependent latency); each chain's order is unchanged
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int ft = 0; ft < FT; ++ft)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) z[ft][rt] = mfma16(w[wq][ft][c], b[rt][c], z[ft][rt]);
      }
    }
#pragma unroll
    for (int u = 0; u < NGI; ++u) pcur[u] = pnext[u];
    }  // !SPLIT
    PPO2_STAMP(2);
    // h1 = tanh(z1): kept in registers for the backward, stored for dW2 and as layer 2's input
#pragma unroll
    for (int ft = 0; ft < FT; ++ft)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) z[ft][rt][r] = tanh_upd(z[ft][rt][r]);
        const int row = 16 * rt + j, m = m0 + row;
        sf4(ACT + row * LDA + fbase + 16 * ft + 4 * g, z[ft][rt]);
        if (m < M) st4(a.H1[trunk] + (size_t)m * H + fbase + 16 * ft + 4 * g, z[ft][rt]);
      }
    lds_barrier();
    PPO2_STAMP(3);

    // ---------------- layer 2 ----------------
    f4 h2[FT][RT];
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      const f4 bv = pld4(pb, T.b2 + fbase + 4 * g, 16 * ft);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) h2[ft][rt] = bv;
    }
    mm64(h2, wsw, w2lane, act_in);
#pragma unroll
    for (int ft = 0; ft < FT; ++ft)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) h2[ft][rt][r] = tanh_upd(h2[ft][rt][r]);
    lds_barrier();  // every wave is done reading h1
#pragma unroll
    for (int ft = 0; ft < FT; ++ft)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) sf4(ACT + (16 * rt + j) * LDA + fbase + 16 * ft + 4 * g, h2[ft][rt]);
    PPO2_STAMP(4);

    // ---------------- heads: partial sums over this wave's 32 features ----------------
    if (trunk == 0) {
      f4 cw3[FT];
#pragma unroll
      for (int ft = 0; ft < FT; ++ft) cw3[ft] = pld4(pb, K.cW3 + fbase + 4 * g, 16 * ft);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        float pv = 0.f;
#pragma unroll
        for (int ft = 0; ft < FT; ++ft)
#pragma unroll
          for (int r = 0; r < 4; ++r) pv = fmaf(cw3[ft][r], h2[ft][rt][r], pv);
        pv = row_allreduce(pv);
        if (g == 0) SCR[2 * NHP * R + wf * R + 16 * rt + j] = pv;
      }
    } else {
      f4 hp[NHT][RT];
#pragma unroll
      for (int ht = 0; ht < NHT; ++ht) {
        f4 hw[FT];
#pragma unroll
        for (int ft = 0; ft < FT; ++ft) hw[ft] = head_fwd(ht, ft);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) hp[ht][rt] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ft = 0; ft < FT; ++ft)
#pragma unroll
          for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) hp[ht][rt] = mfma16(hw[ft][c], h2[ft][rt][c], hp[ht][rt]);
      }
#pragma unroll
      for (int ht = 0; ht < NHT; ++ht)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) SCR[(wf * NHP + 16 * ht + 4 * g + r) * R + 16 * rt + j] = hp[ht][rt][r];
    }
    lds_barrier();
    PPO2_STAMP(5);
    if constexpr (SPLIT && PREF_Z) z1_load(it + gridDim.x, zn);  // the next tile's rows, a half tile ahead

    // ---------------- loss, pass 1: per (row, action) Normal log-prob / entropy terms ----------------
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int idx = tid + 256 * u;
      if (idx < R * A) {
        const int row = idx / A, ai = idx - row * A;
        const bool valid = m0 + row < M;
        const float mu = (SCR[ai * R + row] + SCR[(NHP + ai) * R + row]) + SHB[ai];
        const float var = SVAR[ai], lsd = SLSD[ai];
        const float act = valid ? ACTN[idx] : mu;
        const float d = act - mu;
        float* it_ = ITM + 4 * idx;
        it_[0] = -(d * d) / (2.0f * var) - lsd - kLz;
        it_[1] = kEntC + lsd;
        it_[2] = d / var;
        it_[3] = d * d / var - 1.0f;
      }
    }
    // critic rows: value loss and d loss / d value (ppo:515-527)
    if (tid < R) {
      const bool valid = m0 + tid < M;
      const float v = (SCR[2 * NHP * R + tid] + SCR[2 * NHP * R + R + tid]) + SCB[0];
      const float rt_ = RD[tid], ov = RD[64 + tid];
      float gv, sv;
      if (a.clip_vloss) {
        const float vu = (v - rt_) * (v - rt_);
        const float dv = v - ov;
        const float vcl = ov + fminf(fmaxf(dv, -c), c);
        const float vc = (vcl - rt_) * (vcl - rt_);
        sv = fmaxf(vu, vc);
        const float w1 = vu > vc ? 1.0f : (vu == vc ? 0.5f : 0.0f);
        const float inr = (dv >= -c && dv <= c) ? 1.0f : 0.0f;
        gv = 0.5f * a.vf_coef * a.inv_m * (w1 * 2.0f * (v - rt_) + (1.0f - w1) * 2.0f * (vcl - rt_) * inr);
      } else {
        sv = (v - rt_) * (v - rt_);
        gv = 0.5f * a.vf_coef * a.inv_m * 2.0f * (v - rt_);
      }
      if (!valid) { gv = 0.f; sv = 0.f; }
      ROWS[tid * 8 + 6] = gv;
      cbacc += gv;
      lst[1] += sv;
    }
    lds_barrier();
    PPO2_STAMP(6);
    // ---------------- loss, per row: clipped surrogate (ppo:497-513) ----------------
    if (tid < R) {
      const bool valid = m0 + tid < M;
      float lp = 0.f, ent = 0.f;
      for (int ai = 0; ai < A; ++ai) {
        lp += ITM[4 * (tid * A + ai) + 0];
        ent += ITM[4 * (tid * A + ai) + 1];
      }
      const float oldlp = valid ? RD[128 + tid] : lp;
      const float logratio = lp - oldlp;
      const float ratio = expf(logratio);
      float an = valid ? RD[192 + tid] : 0.f;
      if (a.norm_adv) an = (an - adv_mean) / (adv_std + 1e-8f);
      const float rc = fminf(fmaxf(ratio, 1.0f - c), 1.0f + c);
      const float pg1 = -an * ratio, pg2 = -an * rc;
      const float w1 = pg1 > pg2 ? 1.0f : (pg1 == pg2 ? 0.5f : 0.0f);
      const float inr = (ratio >= 1.0f - c && ratio <= 1.0f + c) ? 1.0f : 0.0f;
      float g_logp = a.inv_m * (w1 * (-an) + (1.0f - w1) * (-an) * inr) * ratio;
      float g_ent = -a.ent_coef * a.inv_m;
      if (valid) {
        lst[0] += fmaxf(pg1, pg2);
        lst[2] += ent;
        lst[3] += -logratio;
        lst[4] += (ratio - 1.0f) - logratio;
        lst[5] += fabsf(ratio - 1.0f) > c ? 1.0f : 0.0f;
      } else {
        g_logp = 0.f;
        g_ent = 0.f;
      }
      ROWS[tid * 8 + 4] = g_logp;
      ROWS[tid * 8 + 5] = g_ent;
    }
    lds_barrier();
    PPO2_STAMP(7);
    // every read of this tile's RD / ACTN is done: DMA the next tile's
    row_dma();
    // ---------------- loss, pass 2: d loss / d mu and d loss / d logstd ----------------
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int idx = tid + 256 * u;
      if (idx < R * A) {
        const int row = idx / A, ai = idx - row * A;
        const float g_logp = ROWS[row * 8 + 4], g_ent = ROWS[row * 8 + 5];
        const float* it_ = ITM + 4 * idx;
        const float gmu = g_logp * it_[2];
        GG[row * LDG + ai] = gmu;
        gacc[u] += gmu;
        lacc[u] += g_logp * it_[3] + g_ent;
      }
    }
    lds_barrier();
    PPO2_STAMP(8);

    // ---------------- head backward: dh2, dW3 ----------------
    f4 dh[FT][RT];
    if (trunk == 0) {
      float gr[RT], x[8];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) gr[rt] = lf(ROWS + (16 * rt + j) * 8 + 6);
#pragma unroll
      for (int ft = 0; ft < FT; ++ft) {
        const f4 cw = pld4(pb, K.cW3 + fbase + 4 * g, 16 * ft);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float s = 0.f;
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) {
            dh[ft][rt][r] = cw[r] * gr[rt];
            s = fmaf(gr[rt], h2[ft][rt][r], s);
          }
          x[4 * ft + r] = s;
        }
      }
      acc_hw += colsum8(x, j);
    } else {
#pragma unroll
      for (int ft = 0; ft < FT; ++ft) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) dh[ft][rt] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ht = 0; ht < NHT; ++ht) {
          const f4 hw = head_bwd(ht, ft);
          f4 gvv[RT];
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) gvv[rt] = lf4(GG + (16 * rt + j) * LDG + 16 * ht + 4 * g);
#pragma unroll
          for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) dh[ft][rt] = mfma16(hw[c], gvv[rt][c], dh[ft][rt]);
          // dW3 tile (heads 16 ht.., features fbase + 16 ft ..), contracted over the tile's rows
#pragma unroll
          for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = 16 * rt + 4 * g + r;
              d3acc[ht][ft] = mfma16(lf(GG + row * LDG + 16 * ht + j), lf(ACT + row * LDA + fbase + 16 * ft + j),
                                     d3acc[ht][ft]);
            }
        }
      }
    }
    PPO2_STAMP(9);
    // dz2 = dh2 * (1 - h2^2)
    {
      float x[8];
#pragma unroll
      for (int ft = 0; ft < FT; ++ft) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const f4 dz = dh[ft][rt] * (1.0f - h2[ft][rt] * h2[ft][rt]);
          dh[ft][rt] = dz;
          const int m = m0 + 16 * rt + j;
          if (m < M) st4(a.DZ2[trunk] + (size_t)m * H + fbase + 16 * ft + 4 * g, dz);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) x[4 * ft + r] = dh[ft][0][r] + dh[ft][1][r];
      }
      acc_b2 += colsum8(x, j);
    }
    lds_barrier();  // the actor's dW3 readers of h2 are done
#pragma unroll
    for (int ft = 0; ft < FT; ++ft)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) sf4(ACT + (16 * rt + j) * LDA + fbase + 16 * ft + 4 * g, dh[ft][rt]);
    lds_barrier();
    PPO2_STAMP(10);

    // ---------------- dh1 = W2^T dz2, dz1 = dh1 * (1 - h1^2) ----------------
    f4 d1[FT][RT];
#pragma unroll
    for (int ft = 0; ft < FT; ++ft)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) d1[ft][rt] = f4{0.f, 0.f, 0.f, 0.f};
    mm64(d1, wsw, w2tlane, act_in);
    PPO2_STAMP(11);
    {
      float x[8];
#pragma unroll
      for (int ft = 0; ft < FT; ++ft) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          d1[ft][rt] = d1[ft][rt] * (1.0f - z[ft][rt] * z[ft][rt]);
          const int m = m0 + 16 * rt + j;
          if (m < M) st4(a.DZ1[trunk] + (size_t)m * H + fbase + 16 * ft + 4 * g, d1[ft][rt]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) x[4 * ft + r] = d1[ft][0][r] + d1[ft][1][r];
      }
      acc_b1 += colsum8(x, j);
    }
    PPO2_STAMP(12);
  }

  // ---------------- workgroup result: one slab row per trunk (fixed-order reductions) ----------------
  const SmallGradLayout sg = a.sg[trunk];
  float* out = a.slab[trunk] + (size_t)blockIdx.x * sg.size;
  if ((j & 1) == 0) {
    const int s = j >> 1, f = fbase + 16 * (s >> 2) + 4 * g + (s & 3);
    out[sg.b1 + f] = acc_b1;
    out[sg.b2 + f] = acc_b2;
    if (trunk == 0) out[sg.hW + f] = acc_hw;
  }
  if (trunk == 1) {
#pragma unroll
    for (int ht = 0; ht < NHT; ++ht)
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int h = 16 * ht + 4 * g + r;
          if (h < A) out[sg.hW + h * H + fbase + 16 * ft + j] = d3acc[ht][ft][r];
        }
  }
  // per-item head-bias / logstd sums -> LDS, then summed over rows per action in row order
  lds_barrier();
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int idx = tid + 256 * u;
    if (idx < R * A) {
      ITM[2 * idx] = gacc[u];
      ITM[2 * idx + 1] = lacc[u];
    }
  }
  if (wave == 0) {
#pragma unroll
    for (int mm = 32; mm >= 1; mm >>= 1) {
      cbacc += __shfl_xor(cbacc, mm, 64);
#pragma unroll
      for (int k = 0; k < 6; ++k) lst[k] += __shfl_xor(lst[k], mm, 64);
    }
  }
  lds_barrier();
  if (tid < A) {
    float s = 0.f, q = 0.f;
    for (int row = 0; row < R; ++row) {
      s += ITM[2 * (row * A + tid)];
      q += ITM[2 * (row * A + tid) + 1];
    }
    float* o1 = a.slab[1] + (size_t)blockIdx.x * a.sg[1].size;
    o1[a.sg[1].hb + tid] = s;
    o1[a.sg[1].ls + tid] = q;
  }
  if (tid == 0) {
    float* o0 = a.slab[0] + (size_t)blockIdx.x * a.sg[0].size;
    float* o1 = a.slab[1] + (size_t)blockIdx.x * a.sg[1].size;
    o0[a.sg[0].hb] = cbacc;
    o0[a.sg[0].stats + ST_V] = lst[1];
    o1[a.sg[1].stats + ST_PG] = lst[0];
    o1[a.sg[1].stats + ST_ENT] = lst[2];
    o1[a.sg[1].stats + ST_OKL] = lst[3];
    o1[a.sg[1].stats + ST_KL] = lst[4];
    o1[a.sg[1].stats + ST_CF] = lst[5];
  }
}

// =============================================================================================
// k_l1g — layer 1 of BOTH 64-wide trunks over the minibatch's gathered observation rows, as one
// GEMM: Z1[m][o] = b1[o] + sum_k X[perm[m]][k] W1[o][k], o < 64 the critic, o >= 64 the actor
// (ppo:124-135: actor_mean.0 / critic.0), for wide inputs (cfg2 Humanoid: K = 376 of 384 padded).
// k_upd2 then runs in its split form (SPLIT): tanh of these rows onwards, no X staging, no W1.
// At K = 384 layer 1 is 73 % of the update forward/backward's MFMAs; inside k_upd2 it ran beside
// the tail's barrier / VALU phases of the co-resident workgroup at ~0.8 of the pipe while the
// tails themselves left it idle. Here it is a plain GEMM, and the tail kernel gets occupancy of its
// own.
//  * workgroup: 128 rows x 128 outputs, 4 waves; wave w: trunk w >> 1, rows 64 (w & 1) .. + 64
//    (2 tiles of 32), outputs 64 trunk .. + 64 (2 tiles of 32): 4 accumulators of
//    v_mfma_f32_32x32x2_f32 (64-cycle issue = dependent latency: no chain stalls);
//  * D[m][o] orientation: A = X rows (lane = row), B = W1^T (lane = output), so a result register
//    holds 32 consecutive outputs of one row (128-byte row segments on store);
//  * k in groups of 8: lane half h holds k = 8 q + 4 h .. + 3 as one f4 of each operand; MFMA step
//    c takes component c (k = 8 q + c and 8 q + 4 + c);
//  * X: 32-column chunks of the 128 gathered rows by LDS DMA (16 bytes a lane; columns >= O and
//    rows >= M out of range, hence 0) into three buffers, two chunks ahead; 16-byte unit u of row r
//    stored at unit u ^ ((r >> 1) & 7): conflict-free ds_read_b128 A operands (64 banks, 32-float
//    rows, the b128 lane groups of MI355X_MICROARCH.md's LDS table);
//  * W1^T: f4 buffer loads from the packed parameters (L2-resident), one chunk ahead;
//  * one s_waitcnt vmcnt(4) per chunk: everything but the newest chunk's 4 DMAs has landed.
// =============================================================================================
template <int OP>
__global__ __launch_bounds__(256, 2) void k_l1g(UpdArgs a) {
  constexpr int H = 64, RW = 128, CK = 32, NCH = OP / CK, NBUF = 3, UPR = CK / 4;
  static_assert(OP % CK == 0, "k_l1g: OP must be a multiple of 32");
  constexpr int DPW = RW * UPR / 64 / 4;  // DMA instructions per wave per chunk (4)
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int trunk = wave >> 1, rh = wave & 1;
  const int M = a.M, O = a.K.O;
  const long m0 = (long)blockIdx.x * RW;
  const PBuf ob = make_pbuf_b(a.obs, (uint32_t)min(a.obs_n * 4, (long)0xFFFFFFFF));
  const PBuf pb = make_pbuf(a.P, a.K.size);
  // this lane's rows of its DMA instructions (the same rows every chunk): instruction i covers rows
  // 8 i .. 8 i + 7, lane -> row 8 i + (lane >> 3), physical unit lane & 7
  int prow[DPW];
#pragma unroll
  for (int d = 0; d < DPW; ++d) {
    const int row = 8 * (wave * DPW + d) + (lane >> 3);
    const long m = m0 + row;
    const int p = a.perm[min(m, (long)M - 1)];
    prow[d] = m < M ? p : -1;
  }
  auto issue = [&](int ch) {
    float* b = lds + (ch % NBUF) * RW * CK;
#pragma unroll
    for (int d = 0; d < DPW; ++d) {
      const int i = wave * DPW + d, row = 8 * i + (lane >> 3), pu = lane & 7;
      const int u = pu ^ ((row >> 1) & 7), col = ch * CK + 4 * u;
      const uint32_t voff = (ch < NCH && prow[d] >= 0 && col < O) ? (uint32_t)(prow[d] * O + col) * 4u : kOOB;
      dma<16>(ob, b + i * 256, voff);
    }
  };
  // W1^T operands: lane (output j, half h): W1[64 trunk + 32 ot + j][8 q + 4 h .. + 3]
  const int wl = (a.K.tr[trunk].W1 + l32 * OP + 4 * h);
  f4 wc[2][4][2];  // [chunk parity][q][ot]
  auto wload = [&](int ch, f4 (&w)[4][2]) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int ot = 0; ot < 2; ++ot)
        w[q][ot] = ch < NCH ? pld4(pb, wl, 32 * ot * OP + ch * CK + 8 * q) : f4{0.f, 0.f, 0.f, 0.f};
  };
  f16v2 acc[2][2];  // [rt][ot]
#pragma unroll
  for (int ot = 0; ot < 2; ++ot) {
    const float bv = a.P[a.K.tr[trunk].b1 + 32 * ot + l32];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[rt][ot][r] = bv;
  }
  wload(0, wc[0]);
  issue(0);
  issue(1);
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    // chunk ch's rows (every wave's DMAs) and W1 of chunk ch have landed; chunk ch + 1's DMAs may
    // stay in flight
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DPW) : "memory");
    lds_barrier();
    wload(ch + 1, wc[(ch + 1) & 1]);
    issue(ch + 2);
    __builtin_amdgcn_sched_barrier(0);
    const float* b = lds + (ch % NBUF) * RW * CK;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f4 x[2];
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const int row = 64 * rh + 32 * rt + l32, u = 2 * q + h;
        x[rt] = *reinterpret_cast<const f4*>(b + row * CK + 4 * (u ^ ((row >> 1) & 7)));
      }
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
          for (int ot = 0; ot < 2; ++ot)
            acc[rt][ot] = __builtin_amdgcn_mfma_f32_32x32x2f32(x[rt][c], wc[ch & 1][q][ot][c], acc[rt][ot], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS DMA may land after the workgroup ends
  // result register r of tile (rt, ot): row 64 rh + 32 rt + (r & 3) + 8 (r >> 2) + 4 h, output 32 ot + l32
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const long m = m0 + 64 * rh + 32 * rt + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (m < M) {
#pragma unroll
        for (int ot = 0; ot < 2; ++ot) a.Z1[m * 128 + 64 * trunk + 32 * ot + l32] = acc[rt][ot][r];
      }
    }
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
size_t l1g_lds_bytes();

// the split form (k_l1g + the tail) where layer 1 is wide: OP a multiple of 32 from 128 on, whole
// 16-byte units per row (O % 4 == 0) — cfg2's Humanoid O = 376 / OP = 384
bool upd2_split_supported(const PackedLayout& K) { return K.H == 64 && K.OP == 384 && K.O % 4 == 0; }

template <typename F>
static int dispatch_upd2(const PackedLayout& K, int split, F&& f) {
  if (K.H != 64 || K.kind != PPO_NET_TANH_NORMAL || K.A > 32) return -1;
  if (split && !upd2_split_supported(K)) return -1;
  const int nto = K.OP / 16, nht = (K.A + 15) / 16, nu = (R2 * K.A + 255) / 256;
  const int vec = (K.O % 4 == 0 && nto >= 2) ? 4 : 1;  // 16-byte DMA needs >= 8 units per row (256 per chunk)
  if (split && nto == 24 && nht == 2 && vec == 4 && nu == 3) {
    if (split == 3)
      return f(std::integral_constant<int, 24>{}, std::integral_constant<int, 2>{}, std::integral_constant<int, 4>{},
               std::integral_constant<int, 3>{}, std::integral_constant<int, 3>{});
    return f(std::integral_constant<int, 24>{}, std::integral_constant<int, 2>{}, std::integral_constant<int, 4>{},
             std::integral_constant<int, 3>{}, std::integral_constant<int, 2>{});
  }
  if (split) return -1;
#define PPO_UPD2_CASE(NTO_, NHT_, VEC_, NU_)                                                         \
  if (nto == NTO_ && nht == NHT_ && vec == VEC_ && nu == NU_)                                        \
    return f(std::integral_constant<int, NTO_>{}, std::integral_constant<int, NHT_>{},               \
             std::integral_constant<int, VEC_>{}, std::integral_constant<int, NU_>{}, std::integral_constant<int, 0>{});
  // NU = 1: A <= 8; 2: A <= 16; 3: A <= 24; 4: A <= 32
  PPO_UPD2_CASE(1, 1, 1, 1) PPO_UPD2_CASE(2, 1, 1, 1) PPO_UPD2_CASE(2, 1, 1, 2) PPO_UPD2_CASE(7, 1, 1, 1)
  PPO_UPD2_CASE(24, 2, 4, 3) PPO_UPD2_CASE(2, 2, 1, 3) PPO_UPD2_CASE(24, 2, 1, 3)
  PPO_UPD2_CASE(2, 1, 4, 1) PPO_UPD2_CASE(24, 1, 4, 2) PPO_UPD2_CASE(24, 2, 4, 4)
#undef PPO_UPD2_CASE
  return -1;
}

// the split-bf16 layer 1 is instantiated for cfg2's shape (Humanoid O = 376: OP = 384, 17 actions)
template <int NTO, int NHT, int VEC, int NU, int SP>
constexpr bool upd2_bx_ok() { return NTO == 24 && NHT == 2 && VEC == 4 && NU == 3 && SP == 0; }

int upd2_supported(const PackedLayout& K, UpdGeoOut* g, int split, int bx) {
  if (split) {
    const auto k = k_l1g<384>;
    if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l1g_lds_bytes()) !=
        hipSuccess)
      return -2;
  }
  return dispatch_upd2(K, split, [&](auto NTO_, auto NHT_, auto VEC_, auto NU_, auto SP_) {
    using GE = Geo2<decltype(NTO_)::value, decltype(NHT_)::value, decltype(VEC_)::value, decltype(NU_)::value,
                    decltype(SP_)::value>;
    int off = GE::oITM + 4 * R2 * K.A;
    g->actn_off = off;
    off += 64 * ((R2 * K.A + 63) / 64);
    g->acc_off = 0;
    g->spar_off = 0;
    g->lds_bytes = (size_t)off * sizeof(float);
    g->rows = R2;
    constexpr int N = decltype(NTO_)::value, T = decltype(NHT_)::value, V = decltype(VEC_)::value,
                  U = decltype(NU_)::value, S = decltype(SP_)::value;
    const void* k = (const void*)k_upd2<N, T, V, U, S, 0>;
    if (bx) {
      if constexpr (upd2_bx_ok<N, T, V, U, S>()) k = (const void*)k_upd2<N, T, V, U, S, 1>;
      else return -1;
    }
    return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)g->lds_bytes) == hipSuccess ? 0 : -2;
  });
}

#ifdef PPO_STAMPS
extern "C" int ppo_diag_read_stamps2(unsigned long long* host, long n) {
  const long cap = (long)(sizeof(g_upd2_stamps) / sizeof(g_upd2_stamps[0]));
  if (n > cap) n = cap;
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_upd2_stamps), n * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? (int)n : -2;
}
#endif

int launch_upd2(const UpdArgs& a, int nblocks, size_t lds_bytes, hipStream_t s, int split) {
  return dispatch_upd2(a.K, split, [&](auto NTO_, auto NHT_, auto VEC_, auto NU_, auto SP_) {
    constexpr int N = decltype(NTO_)::value, T = decltype(NHT_)::value, V = decltype(VEC_)::value,
                  U = decltype(NU_)::value, S = decltype(SP_)::value;
    if (a.bx == 2) {
      if constexpr (upd2_bx_ok<N, T, V, U, S>()) {
        hipLaunchKernelGGL((k_upd2<N, T, V, U, S, 1>), dim3(nblocks), dim3(256), lds_bytes, s, a);
        return 0;
      }
      return -1;
    }
    hipLaunchKernelGGL((k_upd2<N, T, V, U, S, 0>), dim3(nblocks), dim3(256), lds_bytes, s, a);
    return 0;
  });
}

size_t l1g_lds_bytes() { return (size_t)3 * 128 * 32 * sizeof(float); }

int launch_l1g(const UpdArgs& a, hipStream_t s) {
  if (!upd2_split_supported(a.K)) return -1;
  hipLaunchKernelGGL((k_l1g<384>), dim3((a.M + 127) / 128), dim3(256), l1g_lds_bytes(), s, a);
  return 0;
}

// =============================================================================================
// k_dw2 — the weight gradients of BOTH 64-wide trunks for one chunk of minibatch rows:
//   dW1[t][o][i] = sum_m DZ1[t][m][o] * X[perm[m]][i]   (2 x 64 x OP; X gathered ONCE for both)
//   dW2[t][o][i] = sum_m DZ2[t][m][o] * H1[t][m][i]     (2 x 64 x 64)
// 8 waves, MFMA 32x32x2 f32. dW1 is one 128 x OP GEMM (o = 64 t + feature): wave (wo, wi) owns
// o-tile wo and i-tiles [TIW wi, TIW wi + TIW); dW2 is 8 tiles of 32 x 32, one per wave. 16-row
// stages go through one LDS buffer; the next stage's rows (and the permutation two stages ahead)
// are in flight in registers under the current stage's MFMAs. Partials per chunk go to the slab
// (k_colsum adds the chunks in a fixed order).
// =============================================================================================
template <int OP, int VEC>
__global__ __launch_bounds__(512) void k_dw2(DwArgs a) {
  constexpr int H = 64, KS = 16, NTH = 512;
  constexpr int LDXS = OP + 4, LDZ = 2 * H + 4;
  constexpr int TI = (OP + 31) / 32, TIW = (TI + 1) / 2;
  constexpr int XPR = VEC == 4 ? OP / 4 : OP;             // X items per row
  constexpr int NXI = (KS * XPR + NTH - 1) / NTH;         // X items per thread
  constexpr int NZ = KS * 2 * H / 4;                      // f4 per 128-wide row block (DZ1 | DZ2 | H1)
  constexpr int NZI = (NZ + NTH - 1) / NTH;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* XS = lds;
  float* Z1 = XS + KS * LDXS;
  float* Z2 = Z1 + KS * LDZ;
  float* HH = Z2 + KS * LDZ;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, hs = lane >> 5;
  const long m0 = (long)blockIdx.x * a.rows_per_chunk;
  const long m1 = min((long)a.M, m0 + a.rows_per_chunk);
  if (m0 >= m1) return;
  const int nst = (int)((m1 - m0 + KS - 1) / KS);
  const int O = a.O;
  const int wo = wave & 3, wi = wave >> 2;                // dW1 tiles
  const int t2 = wave >> 2, ot2 = (wave >> 1) & 1, it2 = wave & 1;  // dW2 tile

  f16v2 acc1[TIW], acc2;
#pragma unroll
  for (int v = 0; v < TIW; ++v)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc1[v][r] = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc2[r] = 0.f;

  int pr[NXI];     // permutation of the rows of the stage being loaded
  int pn[NXI];     // ... of the stage after it
  f4 xv[NXI];
  f4 zv[3][NZI];   // DZ1 | DZ2 | H1 (both trunks)
  // unconditional loads (clamped addresses, masked values): a per-lane branch around a load costs
  // it its own s_waitcnt vmcnt(0)
  auto perm_of = [&](int st, int (&p)[NXI]) {
#pragma unroll
    for (int u = 0; u < NXI; ++u) {
      const int idx = tid + NTH * u, row = idx / XPR;
      const long m = m0 + (long)st * KS + row;
      const int v = a.perm[min(m, m1 - 1)];
      p[u] = (st < nst && idx < KS * XPR && m < m1) ? v : -1;
    }
  };
  const float* dz1[2] = {a.dz1[0], a.dz1[1]};
  const float* dz2[2] = {a.dz2[0], a.dz2[1]};
  const float* h1[2] = {a.h1[0], a.h1[1]};
  auto load = [&](int st) {
#pragma unroll
    for (int u = 0; u < NXI; ++u) {
      const int idx = tid + NTH * u, row = idx / XPR, q = idx - row * XPR;
      (void)row;
      const long b = (long)(pr[u] >= 0 ? pr[u] : 0) * O;
      if constexpr (VEC == 4) {
        const f4 v = ld4(a.obs + b + min(4 * q, O - 4));
        xv[u] = (pr[u] >= 0 && 4 * q < O) ? v : f4{0.f, 0.f, 0.f, 0.f};
      } else {
        const float v = a.obs[b + min(q, O - 1)];
        xv[u].x = (pr[u] >= 0 && q < O) ? v : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < NZI; ++u) {
      const int c = tid + NTH * u, row = c / 32, q = c - row * 32, f = 4 * (q & 15);
      const bool t = (q >> 4) != 0;
      const long m = m0 + (long)st * KS + row;
      const bool ok = c < NZ && st < nst && m < m1;
      const long o = min(m, m1 - 1) * H + f;
      const f4 v0 = ld4((t ? dz1[1] : dz1[0]) + o);
      const f4 v1 = ld4((t ? dz2[1] : dz2[0]) + o);
      const f4 v2 = ld4((t ? h1[1] : h1[0]) + o);
      const f4 zz = f4{0.f, 0.f, 0.f, 0.f};
      zv[0][u] = ok ? v0 : zz;
      zv[1][u] = ok ? v1 : zz;
      zv[2][u] = ok ? v2 : zz;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < NXI; ++u) {
      const int idx = tid + NTH * u, row = idx / XPR, q = idx - row * XPR;
      if (idx < KS * XPR) {
        if constexpr (VEC == 4) *reinterpret_cast<f4*>(XS + row * LDXS + 4 * q) = xv[u];
        else XS[row * LDXS + q] = xv[u].x;
      }
    }
#pragma unroll
    for (int u = 0; u < NZI; ++u) {
      const int c = tid + NTH * u, row = c / 32, q = c - row * 32;
      if (c < NZ) {
        const int o = row * LDZ + 4 * q;
        *reinterpret_cast<f4*>(Z1 + o) = zv[0][u];
        *reinterpret_cast<f4*>(Z2 + o) = zv[1][u];
        *reinterpret_cast<f4*>(HH + o) = zv[2][u];
      }
    }
  };

  perm_of(0, pr);
  perm_of(1, pn);
  load(0);
  store();
  lds_barrier();
#pragma unroll
  for (int u = 0; u < NXI; ++u) pr[u] = pn[u];
  perm_of(2, pn);
  load(1);
  for (int st = 0; st < nst; ++st) {
    __builtin_amdgcn_sched_barrier(0);
    // operands of k-step k + 2 are read while k-step k's MFMAs run
    float opn[TIW + 3];
    auto rd_ops = [&](int k, float (&o)[TIW + 3]) {
      const int row = k + hs;
      o[0] = Z1[row * LDZ + 32 * wo + l32];
#pragma unroll
      for (int v = 0; v < TIW; ++v) {
        const int col = min(32 * (TIW * wi + v) + l32, OP + 3);  // cols >= OP read the zero pad / row end
        o[1 + v] = XS[row * LDXS + col];
      }
      o[TIW + 1] = Z2[row * LDZ + 64 * t2 + 32 * ot2 + l32];
      o[TIW + 2] = HH[row * LDZ + 64 * t2 + 32 * it2 + l32];
    };
    rd_ops(0, opn);
#pragma unroll
    for (int k = 0; k < KS; k += 2) {
      float op[TIW + 3];
#pragma unroll
      for (int q = 0; q < TIW + 3; ++q) op[q] = opn[q];
      if (k + 2 < KS) rd_ops(k + 2, opn);
#pragma unroll
      for (int v = 0; v < TIW; ++v) {
        const int col = 32 * (TIW * wi + v) + l32;
        acc1[v] = __builtin_amdgcn_mfma_f32_32x32x2f32(op[0], col < OP ? op[1 + v] : 0.f, acc1[v], 0, 0, 0);
      }
      acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(op[TIW + 1], op[TIW + 2], acc2, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    lds_barrier();  // every wave is done with this stage
    if (st + 1 < nst) {
      store();
#pragma unroll
      for (int u = 0; u < NXI; ++u) pr[u] = pn[u];
      perm_of(st + 3, pn);
      lds_barrier();
      if (st + 2 < nst) load(st + 2);
    }
  }
  // ---- partials of this chunk ----
#pragma unroll
  for (int v = 0; v < TIW; ++v)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = 32 * wo + (r & 3) + 8 * (r >> 2) + 4 * hs, t = o >> 6;
      const int i = 32 * (TIW * wi + v) + l32;
      if (i < OP) a.slab[t][(size_t)blockIdx.x * a.slab_stride + H * H + (size_t)(o & 63) * OP + i] = acc1[v][r];
    }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int o = 32 * ot2 + (r & 3) + 8 * (r >> 2) + 4 * hs, i = 32 * it2 + l32;
    a.slab[t2][(size_t)blockIdx.x * a.slab_stride + o * H + i] = acc2[r];
  }
}

// k_dw2_dma — k_dw2 with the stage rows moved by LDS DMA (16 bytes a lane) into three stage buffers,
// two stages ahead of the MFMAs, instead of through registers into one buffer between two barriers
// (OP % 128 == 0 and O % 4 == 0: Humanoid's 376 / 384). The gathered X rows are [16][OP] unpadded
// (columns O .. OP-1 and rows past the chunk read as 0 through out-of-range offsets); DZ1 / DZ2 / H1
// of each trunk are [16][64] blocks. Each wave issues the same number of DMA instructions per stage
// (OP / 128 X + 3 row-block instructions) and loads the permutation entries of its X rows four
// stages ahead, so one constant s_waitcnt keeps exactly the next stage in flight. Every stage past
// the last is issued too (all out of range) to keep that count; the operand values and the MFMA
// order are k_dw2's: bitwise k_dw2.
// BX (dw_mfma=bf16x6 / x9 / x8, k_dwf_bx's scheme): a 16-row stage is one v_mfma_f32_32x32x16_bf16
// k block; lane (l32, hs) reads its operand column at rows 8 hs .. 8 hs + 7 (the same LDS reads as
// the eight 32x32x2 steps) and splits each value into its three bf16 pieces; NP piece products per
// stage and accumulator, fp32 accumulation. Not bitwise the fp32 form (the bf16 MFMA's internal sums).
template <int OP, int BX = 0>
__global__ __launch_bounds__(512) void k_dw2_dma(DwArgs a) {
  constexpr int H = 64, KS = 16, NBUF = 3;
  constexpr int TI = (OP + 31) / 32, TIW = (TI + 1) / 2;
  constexpr int UPR = OP / 4;                      // 16-byte units per X row
  constexpr int XI = KS * OP / 256, XPW = XI / 8;  // X DMA instructions per stage / per wave
  static_assert(OP % 128 == 0 && XPW >= 1, "k_dw2_dma: X rows must be whole instructions per wave");
  constexpr int oZ = KS * OP, STG = oZ + 6 * KS * H;  // X | DZ1 t0,t1 | DZ2 t0,t1 | H1 t0,t1
  // every dW1 column tile is a real one (OP = 32 TI, two waves' TIW tiles cover them exactly): no
  // operand clamping or masking in the MFMA loop
  constexpr bool FULL = TI * 32 == OP && 2 * TIW == TI;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hs = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar DMA descriptors
  const long m0 = (long)blockIdx.x * a.rows_per_chunk;
  const long m1 = min((long)a.M, m0 + a.rows_per_chunk);
  if (m0 >= m1) return;
  const int nst = (int)((m1 - m0 + KS - 1) / KS);
  const int O = a.O;
  const int wo = wave & 3, wi = wave >> 2;
  const int t2 = wave >> 2, ot2 = (wave >> 1) & 1, it2 = wave & 1;
  const PBuf ob = make_pbuf_b(a.obs, (uint32_t)min(a.obs_n * 4, (long)0xFFFFFFFF));
  const uint32_t zb = (uint32_t)((long)a.M * H * 4);
  const PBuf bz0 = make_pbuf_b(a.dz1[0], zb), bz1 = make_pbuf_b(a.dz1[1], zb);
  const PBuf bz2 = make_pbuf_b(a.dz2[0], zb), bz3 = make_pbuf_b(a.dz2[1], zb);
  const PBuf bz4 = make_pbuf_b(a.h1[0], zb), bz5 = make_pbuf_b(a.h1[1], zb);

  f16v2 acc1[TIW], acc2;
#pragma unroll
  for (int v = 0; v < TIW; ++v)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc1[v][r] = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc2[r] = 0.f;

  // The permutation entries of a stage's 16 rows also arrive by LDS DMA (4 bytes a lane), each wave
  // fetching those of its own two X rows (2 w, 2 w + 1) into its slot of a three-stage ring, so no
  // register waits on a load: per stage every wave issues X (XPW) + row-block (3) + entry (1) DMAs.
  static_assert(XPW * 64 == 2 * UPR, "each wave's X instructions cover its two rows");
  const PBuf bperm = make_pbuf_b(a.perm, (uint32_t)((long)a.M * 4));
  int* PR = reinterpret_cast<int*>(lds + NBUF * STG);  // [3 stages][8 waves][64]
  auto perm_dma = [&](int st) {
    const long m = m0 + (long)st * KS + 2 * wave + lane;
    const uint32_t voff = lane < 2 ? (uint32_t)(min(m, m1 - 1) * 4) : kOOB;  // clamped; masked at use
    dma<4>(bperm, reinterpret_cast<float*>(PR + ((st % NBUF) * 8 + wave) * 64), voff);
  };
  auto issue = [&](int st) {
    float* b = lds + (st % NBUF) * STG;
    const int* pw = PR + ((st % NBUF) * 8 + wave) * 64;
#pragma unroll
    for (int x = 0; x < XPW; ++x) {
      const int i = wave * XPW + x, u = i * 64 + lane, row = u / UPR, q = u - row * UPR;
      const long m = m0 + (long)st * KS + row;
      const int pr = pw[row - 2 * wave];
      const uint32_t voff = (m < m1 && 4 * q < O) ? (uint32_t)(pr * O + 4 * q) * 4u : kOOB;
      dma<16, PPO_DW2_AUX>(ob, b + i * 256, voff);
    }
#pragma unroll
    for (int y = 0; y < 3; ++y) {  // row-block instruction i: source i / 4, rows 4 (i % 4) .. + 3
      const int i = wave * 3 + y, src = i >> 2, r0 = 4 * (i & 3), row = r0 + (lane >> 4);
      const long m = m0 + (long)st * KS + row;
      const uint32_t voff = m < m1 ? (uint32_t)((m * H + 4 * (lane & 15)) * 4) : kOOB;
      const PBuf bs = src == 0 ? bz0 : src == 1 ? bz1 : src == 2 ? bz2 : src == 3 ? bz3 : src == 4 ? bz4 : bz5;
      dma<16, PPO_DW2_AUX>(bs, b + oZ + src * KS * H + r0 * H, voff);
    }
  };
  perm_dma(0);
  perm_dma(1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // each wave reads only its own entries
  issue(0);
  perm_dma(2);
  issue(1);
  perm_dma(3);
  for (int st = 0; st < nst; ++st) {
    // stage st's rows and stage st + 2's entries have landed; stage st + 1's rows and stage st + 3's
    // entries may stay in flight
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(XPW + 3 + 1) : "memory");
    lds_barrier();
    issue(st + 2);
    perm_dma(st + 4);
    __builtin_amdgcn_sched_barrier(0);
    const float* b = lds + (st % NBUF) * STG;
    const float* XS = b;
    const float* Z = b + oZ;
    if constexpr (BX) {
      float v8[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v8[e] = Z[(wo >> 1) * KS * H + (8 * hs + e) * H + 32 * (wo & 1) + l32];
      const Split3 az = split3(v8);
#pragma unroll
      for (int v = 0; v < TIW; ++v) {
        const int col = 32 * (TIW * wi + v) + l32;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float x = XS[(8 * hs + e) * OP + (FULL ? col : min(col, OP - 1))];
          v8[e] = (FULL || col < OP) ? x : 0.f;
        }
        acc1[v] = mfma_split<BX>(az, split3(v8), acc1[v]);
      }
      float w8[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v8[e] = Z[(2 + t2) * KS * H + (8 * hs + e) * H + 32 * ot2 + l32];
        w8[e] = Z[(4 + t2) * KS * H + (8 * hs + e) * H + 32 * it2 + l32];
      }
      acc2 = mfma_split<BX>(split3(v8), split3(w8), acc2);
      continue;
    }
    float opn[TIW + 3];
    auto rd_ops = [&](int k, float (&o)[TIW + 3]) {
      const int row = k + hs;
      o[0] = Z[(wo >> 1) * KS * H + row * H + 32 * (wo & 1) + l32];
#pragma unroll
      for (int v = 0; v < TIW; ++v) {
        const int col = 32 * (TIW * wi + v) + l32;
        o[1 + v] = XS[row * OP + (FULL ? col : min(col, OP - 1))];  // cols >= OP are masked below
      }
      o[TIW + 1] = Z[(2 + t2) * KS * H + row * H + 32 * ot2 + l32];
      o[TIW + 2] = Z[(4 + t2) * KS * H + row * H + 32 * it2 + l32];
    };
    rd_ops(0, opn);
#pragma unroll
    for (int k = 0; k < KS; k += 2) {
      float op[TIW + 3];
#pragma unroll
      for (int q = 0; q < TIW + 3; ++q) op[q] = opn[q];
      if (k + 2 < KS) rd_ops(k + 2, opn);
#pragma unroll
      for (int v = 0; v < TIW; ++v) {
        const int col = 32 * (TIW * wi + v) + l32;
        acc1[v] = __builtin_amdgcn_mfma_f32_32x32x2f32(op[0], (FULL || col < OP) ? op[1 + v] : 0.f, acc1[v], 0, 0, 0);
      }
      acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(op[TIW + 1], op[TIW + 2], acc2, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS DMA may land after the workgroup ends
  // ---- partials of this chunk (k_dw2's layout) ----
#pragma unroll
  for (int v = 0; v < TIW; ++v)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = 32 * wo + (r & 3) + 8 * (r >> 2) + 4 * hs, t = o >> 6;
      const int i = 32 * (TIW * wi + v) + l32;
      if (i < OP) a.slab[t][(size_t)blockIdx.x * a.slab_stride + H * H + (size_t)(o & 63) * OP + i] = acc1[v][r];
    }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int o = 32 * ot2 + (r & 3) + 8 * (r >> 2) + 4 * hs, i = 32 * it2 + l32;
    a.slab[t2][(size_t)blockIdx.x * a.slab_stride + o * H + i] = acc2[r];
  }
}

size_t dw2_lds_bytes(int OP) { return (size_t)(16 * (OP + 4) + 3 * 16 * (2 * 64 + 4)) * sizeof(float); }

template <int OP, int VEC>
static int launch_dw2_t(const DwArgs& a, int nchunks, hipStream_t s) {
  const size_t lds = dw2_lds_bytes(OP);
  static const bool ok = hipFuncSetAttribute((const void*)k_dw2<OP, VEC>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)lds) == hipSuccess;
  if (!ok) return -2;
  hipLaunchKernelGGL((k_dw2<OP, VEC>), dim3(nchunks), dim3(512), lds, s, a);
  return 0;
}

int launch_dw2(const DwArgs& a, int OP, int nchunks, hipStream_t s) {
  const bool v4 = (a.O % 4) == 0;
  // 32-bit buffer descriptors: the observation buffer and the row blocks must stay below 4 GB
  if (a.dma && v4 && OP == 384 && a.obs_n * 4 < 0xFFFFFFF0L && (long)a.M * 64 * 4 < 0xFFFFFFF0L) {
    constexpr size_t lds = (size_t)3 * (16 * 384 + 6 * 16 * 64) * sizeof(float) + 3 * 8 * 64 * sizeof(int);
    const void* k = a.bx == 6   ? (const void*)k_dw2_dma<384, 6>
                    : a.bx == 8 ? (const void*)k_dw2_dma<384, 8>
                    : a.bx == 9 ? (const void*)k_dw2_dma<384, 9>
                                : (const void*)k_dw2_dma<384, 0>;
    static bool attr[10] = {};
    const int ai = a.bx >= 0 && a.bx < 10 ? a.bx : 0;
    if (!attr[ai]) {
      if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return -2;
      attr[ai] = true;
    }
    if (a.bx == 6) hipLaunchKernelGGL((k_dw2_dma<384, 6>), dim3(nchunks), dim3(512), lds, s, a);
    else if (a.bx == 8) hipLaunchKernelGGL((k_dw2_dma<384, 8>), dim3(nchunks), dim3(512), lds, s, a);
    else if (a.bx == 9) hipLaunchKernelGGL((k_dw2_dma<384, 9>), dim3(nchunks), dim3(512), lds, s, a);
    else hipLaunchKernelGGL((k_dw2_dma<384, 0>), dim3(nchunks), dim3(512), lds, s, a);
    return 0;
  }
  if (OP == 16) return v4 ? launch_dw2_t<16, 4>(a, nchunks, s) : launch_dw2_t<16, 1>(a, nchunks, s);
  if (OP == 32) return v4 ? launch_dw2_t<32, 4>(a, nchunks, s) : launch_dw2_t<32, 1>(a, nchunks, s);
  if (OP == 112) return v4 ? launch_dw2_t<112, 4>(a, nchunks, s) : launch_dw2_t<112, 1>(a, nchunks, s);
  if (OP == 384) return v4 ? launch_dw2_t<384, 4>(a, nchunks, s) : launch_dw2_t<384, 1>(a, nchunks, s);
  return -1;
}
