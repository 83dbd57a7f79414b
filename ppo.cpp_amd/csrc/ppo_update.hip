// ppo_update.hip — k_upd: the fused minibatch forward / PPO loss / backward kernel, feature-split.
//
// Same contract as k_fwdbwd (ppo_kernels.hip) — gather through the permutation, forward of one
// trunk, heads, clipped-surrogate / value / entropy loss and its gradient, backward to dz2 / dz1,
// the "small gradient" slab (biases, LayerNorm affine, head weights and biases, logstd, loss
// stats) and the Xn / H1 / DZ1 / DZ2 activations the dW GEMM reads — but laid out so that the
// VALU work stays small next to the MFMA work (reference: ppo:495-538, ac:815-875):
//
//  * a workgroup (4 waves) owns R rows per iteration; the rows' activations live in LDS
//    ([R][H+4] fp32, row stride = 4 mod 64 banks so every ds_read_b128 B-operand load is
//    conflict-free); each wave owns FT 16-feature output tiles x RT 16-row tiles, so a 256-wide
//    layer needs 64 accumulator registers per wave instead of 256;
//  * weight A-operands stream from L2 with buffer loads, double-buffered one k-block ahead;
//  * heads are MFMAs (split-K over the waves' features, partials reduced through LDS), the head
//    backward dh2 = W3^T G^T and the head weight gradient G^T h2 are MFMAs too;
//  * LayerNorm row statistics: in-lane sums + 2 lane shuffles + a cross-wave LDS exchange;
//    column sums (bias / LN-affine gradients) are a 15-shuffle reduce-scatter per vector per
//    iteration instead of per 16 rows;
//  * R = 32 rows keep LDS under 80 KB, so two workgroups (8 waves) share a CU and one's VALU /
//    barrier phases overlap the other's MFMA phases;
//  * BX (create option upd_mfma=bx6, the default for the LayerNorm-Beta agent at H = 256): layer 2
//    and dh1 = W2^T dz2 run as six split-bf16 piece products per fp32 product on
//    v_mfma_f32_16x16x32_bf16 (mm_bx: weight pieces from k_adam's bx_index copies, activation
//    pieces split once when the tile is written to LDS) — 0.375 of the fp32 MFMA cycles, the same
//    accumulator layout, as exact against the fp64 oracle as the fp32 form.
// Everything is reduced in a fixed order: results are bitwise reproducible run to run.
#include "ppo_agent.hpp"
#include <cstdlib>
#include "ppo_kernels.hpp"

// 1: a tile's gathered rows are committed to LDS by the previous tile (EARLY in upd16_body); 0: at the
// tile top (A/B builds)
#ifndef PPO_UPD_EARLY
#define PPO_UPD_EARLY 0
#endif
// A/B switches of round-6 k_upd changes (each 1 = on; all off = the round-5 kernel): merged
// LayerNorm statistics (one exchange per LayerNorm), the two barriers other exchange barriers cover,
// head partials summed inside the loss, branch-free prefetch loads, no LDS copy of the critic's h2,
// the tile top's first barrier (covered by the previous tile's layer-1 backward exchange), the next
// tile's rows committed in the layer-1 backward (EARLY). Measured per launch against all-off
// (profiles/r06/kupd_ab/): EARLY +9.6 %, BF +1.4 %; CHAN -1.0 %, BAR -1.0 %, PRE -0.5 %, CH2 0 one at
// a time on one box, but CHAN + BAR + PRE + CH2 together +1.2 % and with TOP +1.5 % on another (the
// critic's tile 75 K -> 67 K cycles, the actor's 79 K -> 81 K: the launch is the actor's, and the
// critic's shorter phases leave the actor's loss with fewer partner MFMA gaps). Not kept: all off.
// 1: the H1 / DZ2 hand-off rows are stored from inside the next GEMM (read back from the LDS pieces,
// issued after its first weight prefetches) instead of from registers before it (A/B builds). Measured
// +11 % per launch (spills 31 -> 53, profiles/r06/kupd_defer/): off
#ifndef PPO_UPD_DEFER
#define PPO_UPD_DEFER 0
#endif
// 1: the head weights (NHT = 1) held in registers from the tile top (16 VGPRs); 0: loaded at each use.
// Measured 0: k_upd 0.610 -> 0.602 ms per launch (spills 31 -> 28; results bitwise equal, profiles/r06/kupd_hwb/)
#ifndef PPO_V_HWB
#define PPO_V_HWB 0
#endif
// 1: the next tile's permutation entries requested after the layer-2 GEMM and its rows after the dh1 GEMM
// (shorter register live ranges), 0: at the tile top and after the layer-2 GEMM (A/B)
// 1: no register prefetch of the next tile's rows (each tile gathers its rows at its top; A/B)
#ifndef PPO_V_NOPREF
#define PPO_V_NOPREF 0
#endif
#ifndef PPO_V_PLATE
#define PPO_V_PLATE 0
#endif
#ifndef PPO_V_CHAN
#define PPO_V_CHAN 0
#endif
#ifndef PPO_V_BAR
#define PPO_V_BAR 0
#endif
#ifndef PPO_V_PRE
#define PPO_V_PRE 0
#endif
#ifndef PPO_V_BF
#define PPO_V_BF 0
#endif
#ifndef PPO_V_TOP
#define PPO_V_TOP 0
#endif
#ifndef PPO_V_CH2
#define PPO_V_CH2 0
#endif

#ifdef PPO_STAMPS
// diagnostic build only: per-wave shader-clock stamps at phase ends of the first 16 tiles of every workgroup
#define PPO_NSTAMP 13
#define PPO_STAMP_TILES 16
#define PPO_STAMP_REC (PPO_NSTAMP + 2)  // start, 13 phase ends, hardware wave id (HW_ID | XCC_ID << 32)
__device__ unsigned long long g_upd_stamps[1024 * 4 * PPO_STAMP_TILES * PPO_STAMP_REC];
#define PPO_STAMP(k)                                                                                 \
  do {                                                                                               \
    const int tt_ = (it - (int)blockIdx.x) / (int)gridDim.x;                                     \
    if (tt_ >= 0 && tt_ < PPO_STAMP_TILES) {                                                         \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                    \
      const int wg_ = trunk * 512 + blockIdx.x;                                            \
      if (lane == 0 && blockIdx.x < 512)                                                                    \
        g_upd_stamps[((wg_ * 4 + wave) * PPO_STAMP_TILES + tt_) * PPO_STAMP_REC + (k) + 1] = t_;      \
    }                                                                                                \
  } while (0)
#define PPO_STAMP_START()                                                                            \
  do {                                                                                               \
    const int tt_ = (it - (int)blockIdx.x) / (int)gridDim.x;                                     \
    if (tt_ >= 0 && tt_ < PPO_STAMP_TILES) {                                                         \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                    \
      const int wg_ = trunk * 512 + blockIdx.x;                                            \
      const unsigned long long id_ = (unsigned long long)__builtin_amdgcn_s_getreg(0xF804) |          \
                                     ((unsigned long long)__builtin_amdgcn_s_getreg(0xF814) << 32);  \
      if (lane == 0 && blockIdx.x < 512) {                                                           \
        g_upd_stamps[((wg_ * 4 + wave) * PPO_STAMP_TILES + tt_) * PPO_STAMP_REC] = t_;               \
        g_upd_stamps[((wg_ * 4 + wave) * PPO_STAMP_TILES + tt_) * PPO_STAMP_REC + PPO_NSTAMP + 1] = id_; \
      }                                                                                              \
    }                                                                                                \
  } while (0)
// a.sched bits 4..7 skip the H1 / DZ2 / DZ1 / Xn stores, bit 12 the column sums (bias / LayerNorm-affine /
// critic head weight gradients), bit 13 reads every split-bf16 weight unit from the wave's first one
// (timing experiments only: the gradient is then wrong)
#define PPO_DIAG_SKIP(bit) ((a.sched >> (bit)) & 1)
#else
#define PPO_STAMP(k) do {} while (0)
#define PPO_STAMP_START() do {} while (0)
#define PPO_DIAG_SKIP(bit) false
#endif

namespace {

template <int H_, int NTO_, int NHT_, bool BX_ = false>
struct Geo {
  static constexpr int H = H_, NT = H / 16;
  static constexpr bool BX = BX_;
  static constexpr int WF = (H >= 256) ? 4 : 1;  // wave feature groups
  static constexpr int WR = 4 / WF;              // wave row groups
  static constexpr int FT = NT / WF;             // 16-feature tiles per wave
  static constexpr int RT = (WF == 4) ? 2 : 1;   // 16-row tiles per wave
  static constexpr int R = 16 * RT * WR;         // rows per workgroup iteration
  static constexpr int NTO = NTO_, OP = NTO * 16;
  static constexpr int NHT = NHT_, NHP = 16 * NHT;
  static constexpr int LDX = OP + 4;  // layer-1 B operands: 2 k-blocks per pass, a 2-way conflict is noise
  static constexpr int LDA = ((H + 63) / 64) * 64 + 4;
  static constexpr int LDG = NHP + 4;
  static constexpr int ITS = 10;  // floats per (row, action) item
  // BX: split-bf16 activation rows (3 pieces x H bf16 + 16 B, row stride 4 mod 64 banks like LDA),
  // in the same region as the fp32 h2 rows the actor's head backward reads
  static constexpr int LDB = 3 * (H / 2) + 4;
  static constexpr int LDU = (BX && LDB > LDA) ? LDB : LDA;
  // static part of the LDS carve (floats); the runtime part (items, rows, accumulators) follows
  static constexpr int oXN = 0;
  static constexpr int oACT = oXN + R * LDX;
  static constexpr int oRED = oACT + R * LDU;        // 4 slots x WF x R
  // BX: the per-tile regions whose lifetime lies between the layer-2 GEMM's last piece read and the
  // dz2 piece writes — head partials / loss items (SCR), head pre-activations (PRE) and gradients
  // (GG, re-zeroed every tile) — sit in the activation region behind the fp32 h2 rows, which keeps
  // two workgroups and the LDS accumulators on a CU
  static constexpr int SCRB = (WF * NHP * R > R * (NHP / 2) * ITS) ? WF * NHP * R : R * (NHP / 2) * ITS;
  static constexpr int oSCR = BX ? oACT + R * LDA : oRED + 4 * WF * R + 2 * R * LDG + R * 8;
  static constexpr int oPRE = BX ? oSCR + SCRB : oRED + 4 * WF * R;  // R x LDG head pre-activations
  static constexpr int oG = oPRE + R * LDG;                          // R x LDG head gradients
  static constexpr int oROW = BX ? oRED + 4 * WF * R : oG + R * LDG; // R x 8 per-row scalars
  static constexpr int SCR_MAX = BX ? SCRB : 1 << 30;  // floats SCR (head partials / items) may take
  // staged small parameters: LayerNorm gamma/beta of both layers, head biases, observation
  // mean / std (placed after the runtime-sized regions)
  static constexpr int NSPAR = 4 * H + NHP + 2 * OP;
  static_assert(!BX || oG + R * LDG <= oACT + R * LDU, "BX: SCR / PRE / GG must fit behind the h2 rows");
  static_assert(BX || oSCR == oROW + R * 8, "carve");
};

PPO_DEV float lds_f(const float* p) { return *p; }
PPO_DEV f4 lds_f4(const float* p) { return *reinterpret_cast<const f4*>(p); }
PPO_DEV void lds_st4(float* p, f4 v) { *reinterpret_cast<f4*>(p) = v; }
PPO_DEV float bld1(PBuf b, int lane_floats, int uni_floats) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(b.r, lane_floats * 4, uni_floats * 4, 0));
}

// out[ft][rt] (+)= sum_k W[fbase + 16 ft + i][k] * IN[rbase + 16 rt + j][k], k in [0, 16 NKB)
//   in = IN + (rbase + j) * LDI + 4 g (LDS, per lane)
// A (weights) double-buffered one 16-wide k-block ahead; B (activations) one ds_read_b128 per row tile.
// KL (1 or 4): k-steps of the last 16-wide k-block that hold a real column — step c covers columns
// 16 kb + 4 g + c, so with KL = 1 (K = 16 (NKB - 1) + 1, layer 1 at O = 17) the last block's y / z / w
// steps are all padding and are skipped (5 of 8 steps).
// A operands come from the swizzled copy (sw_index): feature tile ft, k-block kb of this wave at
// wlane + FS ft + KS kb with FS = 256 NKB, KS = 256 (one contiguous 1 KB per wave-load)
template <int FT, int RT, int NKB, int LDI, int KL = 4>
PPO_DEV void mm_fr(f4 (&out)[FT][RT], PBuf wb, int wlane, const float* in) {
  constexpr int FS = 256 * NKB, KS = 256;
  f4 w[2][FT];
#pragma unroll
  for (int ft = 0; ft < FT; ++ft) w[0][ft] = pld4(wb, wlane, FS * ft);
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) {
    if (kb + 1 < NKB) {
#pragma unroll
      for (int ft = 0; ft < FT; ++ft) w[(kb + 1) & 1][ft] = pld4(wb, wlane, FS * ft + KS * (kb + 1));
    }
    // pin the prefetch here: the scheduler otherwise sinks it next to its use (vmcnt(0) per block)
    __builtin_amdgcn_sched_barrier(0);
    f4 b[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) b[rt] = lds_f4(in + 16 * rt * LDI + 16 * kb);
    const bool full = kb + 1 < NKB || KL >= 4;
    // k-step c outermost: consecutive MFMAs go to different accumulators (FT x RT independent
    // chains), so none waits out the 40-cycle dependent latency of 16x16x4 f32 (32-cycle issue)
    // when the partner wave is not streaming MFMAs; each accumulator's chain order is unchanged
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c > 0 && !full) break;
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) out[ft][rt] = mfma16(w[kb & 1][ft][c], b[rt][c], out[ft][rt]);
    }
  }
}

// Split-bf16 form of the 256-wide GEMMs (create option upd_mfma=bx6, BX = 1): out[ft][rt] (+)= the
// same sum as mm_fr over k in [0, 16 NKB), as v_mfma_f32_16x16x32_bf16 piece products. A = the
// weights' pieces (bx_index copies: hi, mid, lo of every fp32 weight, written by k_adam), B = the
// activations' pieces (split once when the tile is written to LDS, lds_store_pieces). Of the nine
// piece products six are kept: lo.hi, hi.lo, mid.mid, mid.hi, hi.mid, hi.hi (smallest first); the
// dropped mid.lo + lo.mid + lo.lo are < 2^-21 |a b| (|mid| < 2^-7 |x|, |lo| < 2^-15 |x|): the order of
// an fp32 accumulation's rounding over K = 256 terms, and measured as exact as the fp32 MFMA form
// against the fp64 oracle (test_upd_bx6_is_as_accurate_as_fp32_mfma). One 16x16x32 MFMA takes 16 cycles for 32 k against 8 x 32 cycles of 16x16x4 f32:
// six are 0.375 of the fp32 MFMA time. Lane (j, g) k slot 8 g + e <-> column 32 kk + 16 (e >> 2) +
// 4 g + (e & 3), the columns mm_fr gives lane group g in k-blocks 2 kk and 2 kk + 1, so the
// accumulator layout is mm_fr's.
//   inb = ACTB + (rbase + j) LDB + 4 g (floats; row = 3 pieces x H bf16 + 16 B, piece p at 128 p floats)
//   weight unit (kk, ft): 3 x 16 B per lane at wlane + 256 ((ft NKK + kk) 3 + p) floats
// A pieces stream through a ring of NS units (D = NS - 1 ahead, ~ one 32-k block of every feature tile).
// weight-piece ring depth (32-k units in flight ahead): 2 / 3 / 4 / 5 measured 0.62 / 0.61 / 0.65 /
// 0.69 ms per launch (deeper rings spill; profiles/r05/bx6/abm2, abm3)
#ifndef PPO_BX_RING
#define PPO_BX_RING 3
#endif
constexpr int kBxRing = PPO_BX_RING;
PPO_DEV u32x4 pld4u(PBuf b, int lane_floats, int uni_floats) { return __builtin_bit_cast(u32x4, pld4(b, lane_floats, uni_floats)); }
// diag_unit0 (stamps build, timing only): every weight unit read from the wave's first unit, so the
// wave streams 3 KB from the L1 instead of 96 KB from L2 (is the weight stream the GEMMs' bound?)
struct NoMid {
  PPO_DEV void operator()() const {}
};
// mid (PPO_UPD_DEFER): called once, right after the first in-loop weight prefetch — vector-memory work
// (the hand-off stores) issued there is older than only the weight loads of units D + 1 .., so the
// wave first waits on it D + 1 units later instead of at the GEMM's first unit
template <int FT, int RT, int NKB, int LDB, class Mid = NoMid>
PPO_DEV void mm_bx(f4 (&out)[FT][RT], PBuf wb, int wlane, const float* inb, bool diag_unit0 = false, Mid mid = Mid{}) {
  static_assert(NKB % 2 == 0, "mm_bx: 32-wide k blocks");
  constexpr int NKK = NKB / 2, U = NKK * FT, D = kBxRing, NS = D + 1, PS = 8 * NKB;
  u32x4 ar[NS][3];
  auto load_unit = [&](int u, u32x4 (&dst)[3]) {
#ifdef PPO_STAMPS
    if (diag_unit0) u = 0;
#else
    (void)diag_unit0;
#endif
    const int kk = u / FT, ft = u - kk * FT;
#pragma unroll
    for (int p = 0; p < 3; ++p) dst[p] = pld4u(wb, wlane, 256 * ((ft * NKK + kk) * 3 + p));
  };
#pragma unroll
  for (int u = 0; u < D; ++u) load_unit(u, ar[u]);
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) {
    u32x4 bs[RT][3];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int p = 0; p < 3; ++p) bs[rt][p] = __builtin_bit_cast(u32x4, lds_f4(inb + 16 * rt * LDB + PS * p + 16 * kk));
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      const int u = kk * FT + ft;
      if (u + D < U) load_unit(u + D, ar[(u + D) % NS]);
      if (u == 0) mid();
      // pin the prefetch here: the scheduler otherwise sinks it next to its use
      __builtin_amdgcn_sched_barrier(0);
      const u32x4(&av)[3] = ar[u % NS];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        f4 acc = out[ft][rt];
        acc = mfma16bx(av[2], bs[rt][0], acc);
        acc = mfma16bx(av[0], bs[rt][2], acc);
        acc = mfma16bx(av[1], bs[rt][1], acc);
        acc = mfma16bx(av[1], bs[rt][0], acc);
        acc = mfma16bx(av[0], bs[rt][1], acc);
        out[ft][rt] = mfma16bx(av[0], bs[rt][0], acc);
      }
    }
  }
}
// the tile's activations as split-bf16 pieces: lane (j, g) holds row rbase + 16 rt + j, features
// f = fbase + 16 ft + 4 g + r; feature f of a row sits at bf16 position 32 (f >> 5) + 8 g + 4 ((f >> 4) & 1)
// + r of each piece (mm_bx's k slots), so a lane writes 8 bytes per piece
template <int FT, int RT, int LDB, int PS>
PPO_DEV void lds_store_pieces(float* actb, const f4 (&v)[FT][RT], int rbase, int fbase, int j, int g) {
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      const int f0 = fbase + 16 * ft;
      float* q = actb + (rbase + 16 * rt + j) * LDB + 16 * (f0 >> 5) + 4 * g + 2 * ((f0 >> 4) & 1);
      unsigned h0, m0, l0, h1, m1, l1;
      split3_pair(v[ft][rt][0], v[ft][rt][1], h0, m0, l0);
      split3_pair(v[ft][rt][2], v[ft][rt][3], h1, m1, l1);
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      *reinterpret_cast<u32x2*>(q) = u32x2{h0, h1};
      *reinterpret_cast<u32x2*>(q + PS) = u32x2{m0, m1};
      *reinterpret_cast<u32x2*>(q + 2 * PS) = u32x2{l0, l1};
    }
}

// the hand-off rows store_tile_rows writes, read back from lds_store_pieces' split-bf16 pieces:
// x = hi + (mid + lo) exactly (hi, mid, lo are consecutive 8-bit slices of x's significand), so the
// bytes are store_tile_rows' (a -0 comes back as +0)
template <int FT, int RT, int LDB, int PS>
PPO_DEV void store_rows_from_pieces(float* __restrict__ dst, int ld, const float* actb, int m0, int M, int rbase,
                                    int fbase, int j, int g) {
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int m = m0 + rbase + 16 * rt + j;
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      const int f0 = fbase + 16 * ft;
      const float* q = actb + (rbase + 16 * rt + j) * LDB + 16 * (f0 >> 5) + 4 * g + 2 * ((f0 >> 4) & 1);
      const u32x2 h = *reinterpret_cast<const u32x2*>(q);
      const u32x2 md = *reinterpret_cast<const u32x2*>(q + PS);
      const u32x2 lo = *reinterpret_cast<const u32x2*>(q + 2 * PS);
      f4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int w = r >> 1, sh = (r & 1) ? 0 : 16;
        const float fh = __uint_as_float(((h[w] << sh) & 0xffff0000u));
        const float fm = __uint_as_float(((md[w] << sh) & 0xffff0000u));
        const float fl = __uint_as_float(((lo[w] << sh) & 0xffff0000u));
        v[r] = fh + (fm + fl);
      }
      if (m < M) st4(dst + (size_t)m * ld + f0 + 4 * g, v);
    }
  }
}

// bias init: out[ft][rt] = b[fbase + 16 ft + 4 g + r]
template <int FT, int RT>
PPO_DEV void init_bias(f4 (&out)[FT][RT], PBuf pb, int boff_lane) {
#pragma unroll
  for (int ft = 0; ft < FT; ++ft) {
    const f4 bv = pld4(pb, boff_lane, 16 * ft);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) out[ft][rt] = bv;
  }
}
template <int FT, int RT>
PPO_DEV void zero(f4 (&out)[FT][RT]) {
#pragma unroll
  for (int ft = 0; ft < FT; ++ft)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) out[ft][rt] = f4{0.f, 0.f, 0.f, 0.f};
}

// per-row sums over all H features of (row tile rt, lane's row j): in-lane over the wave's
// FT x 4 features, then the 4 lane groups, then (WF > 1) the WF feature-group waves via LDS.
// red: a [WF][R] LDS slot. Must be called by every thread (contains a barrier when WF > 1).
template <int WF, int RT, int R>
PPO_DEV void rows_total(float (&s)[RT], float* red, int wf, int rbase, int j, int g) {
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) s[rt] = row_allreduce(s[rt]);
  if constexpr (WF > 1) {
    if (g == 0) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) red[wf * R + rbase + 16 * rt + j] = s[rt];
    }
    lds_barrier();
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < WF; ++w) t += red[w * R + rbase + 16 * rt + j];
      s[rt] = t;
    }
  }
}
// two row sums at once (one barrier)
template <int WF, int RT, int R>
PPO_DEV void rows_total2(float (&s)[RT], float (&q)[RT], float* red0, float* red1, int wf, int rbase, int j, int g) {
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    s[rt] = row_allreduce(s[rt]);
    q[rt] = row_allreduce(q[rt]);
  }
  if constexpr (WF > 1) {
    if (g == 0) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        red0[wf * R + rbase + 16 * rt + j] = s[rt];
        red1[wf * R + rbase + 16 * rt + j] = q[rt];
      }
    }
    lds_barrier();
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      float t = 0.f, u = 0.f;
#pragma unroll
      for (int w = 0; w < WF; ++w) {
        t += red0[w * R + rbase + 16 * rt + j];
        u += red1[w * R + rbase + 16 * rt + j];
      }
      s[rt] = t;
      q[rt] = u;
    }
  }
}

// LayerNorm statistics of z (eps 1e-5, biased variance as torch::layer_norm). One wave holds H / WF
// features of a row: it computes their sum and their squared deviations about its OWN mean (two-pass
// within the wave), and the WF waves' (sum, M2) pairs are merged after ONE cross-wave exchange with
// Chan's parallel formula, M2 = sum_w M2_w + n_w (mean_w - mean)^2 (exactly the two-pass variance in
// exact arithmetic, as stable in fp32): one barrier per LayerNorm instead of two. WF = 1 is the plain
// two-pass form.
template <int FT, int RT, int WF, int R, int H>
PPO_DEV void ln_rows(const f4 (&z)[FT][RT], float (&mu)[RT], float (&rs)[RT], float* red0, float* red1, int wf,
                     int rbase, int j, int g) {
  constexpr float invH = 1.0f / H;
#if !PPO_V_CHAN
  {
    float s[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      float t = 0.f;
#pragma unroll
      for (int ft = 0; ft < FT; ++ft) t += (z[ft][rt].x + z[ft][rt].y) + (z[ft][rt].z + z[ft][rt].w);
      s[rt] = t;
    }
    rows_total<WF, RT, R>(s, red0, wf, rbase, j, g);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      mu[rt] = s[rt] * invH;
      float t = 0.f;
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = z[ft][rt][r] - mu[rt];
          t += d * d;
        }
      s[rt] = t;
    }
    rows_total<WF, RT, R>(s, red1, wf, rbase, j, g);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) rs[rt] = 1.0f / sqrtf(s[rt] * invH + 1e-5f);
    return;
  }
#endif
  constexpr int HW = H / WF;
  constexpr float invW = 1.0f / HW;
  float s[RT], q[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    float t = 0.f;
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) t += (z[ft][rt].x + z[ft][rt].y) + (z[ft][rt].z + z[ft][rt].w);
    s[rt] = row_allreduce(t);
  }
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const float mw = s[rt] * invW;
    float t = 0.f;
#pragma unroll
    for (int ft = 0; ft < FT; ++ft)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d = z[ft][rt][r] - mw;
        t += d * d;
      }
    q[rt] = row_allreduce(t);
  }
  if constexpr (WF > 1) {
    if (g == 0) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        red0[wf * R + rbase + 16 * rt + j] = s[rt];
        red1[wf * R + rbase + 16 * rt + j] = q[rt];
      }
    }
    lds_barrier();
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      float sw[WF], tot = 0.f;
#pragma unroll
      for (int w = 0; w < WF; ++w) {
        sw[w] = red0[w * R + rbase + 16 * rt + j];
        tot += sw[w];
      }
      mu[rt] = tot * invH;
      float m2 = 0.f;
#pragma unroll
      for (int w = 0; w < WF; ++w) {
        const float dm = sw[w] * invW - mu[rt];
        m2 += red1[w * R + rbase + 16 * rt + j] + (float)HW * (dm * dm);
      }
      rs[rt] = 1.0f / sqrtf(m2 * invH + 1e-5f);
    }
  } else {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      mu[rt] = s[rt] * invH;
      rs[rt] = 1.0f / sqrtf(q[rt] * invH + 1e-5f);
    }
  }
}

template <int CTRL, int LEN, int M>
PPO_DEV void rs_stage(float (&x)[16], int j) {
  const bool bit = (j & M) != 0;
#pragma unroll
  for (int i = 0; i < LEN / 2; ++i) {
    const float lo = x[i], hi = x[i + LEN / 2];
    const float keep = bit ? hi : lo, send = bit ? lo : hi;
    x[i] = keep + dpp_f<CTRL>(send);
  }
}

// Stages j ^ 8 and half-mirror (bit 2 of j) of the reduce-scatter with bank-masked DPP adds: lanes
// whose bit is 0 (banks 0-1, resp. 0 and 2) keep slot i and add the partner's slot i; lanes whose
// bit is 1 keep slot i + LEN / 2 and add the partner's, written into slot i. The second add of a
// pair reads only upper slots, which the first does not write. s_nop 1: the DPP sources may have
// been written by the instruction just before the block.
PPO_DEV void rs_stage_banked(float (&x)[16]) {
#define PPO_RS_A(i, C, B) "v_add_f32_dpp %" #i ", %" #i ", %" #i " " C " row_mask:0xf bank_mask:" B "\n\t"
#define PPO_RS_B(i, k, C, B) "v_add_f32_dpp %" #i ", %" #k ", %" #k " " C " row_mask:0xf bank_mask:" B "\n\t"
  asm("s_nop 1\n\t"
      PPO_RS_A(0, "row_ror:8", "0x3") PPO_RS_A(1, "row_ror:8", "0x3") PPO_RS_A(2, "row_ror:8", "0x3")
      PPO_RS_A(3, "row_ror:8", "0x3") PPO_RS_A(4, "row_ror:8", "0x3") PPO_RS_A(5, "row_ror:8", "0x3")
      PPO_RS_A(6, "row_ror:8", "0x3") PPO_RS_A(7, "row_ror:8", "0x3")
      PPO_RS_B(0, 8, "row_ror:8", "0xc") PPO_RS_B(1, 9, "row_ror:8", "0xc") PPO_RS_B(2, 10, "row_ror:8", "0xc")
      PPO_RS_B(3, 11, "row_ror:8", "0xc") PPO_RS_B(4, 12, "row_ror:8", "0xc") PPO_RS_B(5, 13, "row_ror:8", "0xc")
      PPO_RS_B(6, 14, "row_ror:8", "0xc") PPO_RS_B(7, 15, "row_ror:8", "0xc")
      : "+&v"(x[0]), "+&v"(x[1]), "+&v"(x[2]), "+&v"(x[3]), "+&v"(x[4]), "+&v"(x[5]), "+&v"(x[6]), "+&v"(x[7])
      : "v"(x[8]), "v"(x[9]), "v"(x[10]), "v"(x[11]), "v"(x[12]), "v"(x[13]), "v"(x[14]), "v"(x[15]));
  asm("s_nop 1\n\t"
      PPO_RS_A(0, "row_half_mirror", "0x5") PPO_RS_A(1, "row_half_mirror", "0x5")
      PPO_RS_A(2, "row_half_mirror", "0x5") PPO_RS_A(3, "row_half_mirror", "0x5")
      PPO_RS_B(0, 4, "row_half_mirror", "0xa") PPO_RS_B(1, 5, "row_half_mirror", "0xa")
      PPO_RS_B(2, 6, "row_half_mirror", "0xa") PPO_RS_B(3, 7, "row_half_mirror", "0xa")
      : "+&v"(x[0]), "+&v"(x[1]), "+&v"(x[2]), "+&v"(x[3])
      : "v"(x[4]), "v"(x[5]), "v"(x[6]), "v"(x[7]));
#undef PPO_RS_A
#undef PPO_RS_B
}

// column sums over this wave's rows of v(ft, rt, r), added to acc[fbase + feature]:
// sum over rt in lane, then a 16-lane reduce-scatter (lane j ends with slot j).
template <int FT, int RT, typename Fn>
PPO_DEV void col_sums(Fn v, float* acc, int fbase, int j, int g) {
  static_assert(FT == 4, "col_sums assumes 16 slots per lane");
  float x[16];
#pragma unroll
  for (int ft = 0; ft < FT; ++ft)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float t = v(ft, 0, r);
#pragma unroll
      for (int rt = 1; rt < RT; ++rt) t += v(ft, rt, r);
      x[4 * ft + r] = t;
    }
  // recursive halving over the 16 lanes j of each lane group with DPP partners: j ^ 8 (row_ror:8),
  // the mirror in each half (row_half_mirror), the mirror in each quad, j ^ 1. Each stage pairs
  // lanes of opposite bit m, so lane j still ends with slot j summed over all 16 lanes.
  // The first two stages split the lanes by DPP bank (bank = j >> 2): one bank-masked add per slot
  // and half, own + partner exactly as the select form, without the two selects per slot.
  rs_stage_banked(x);
  rs_stage<kDppQuadMirror, 4, 2>(x, j);
  rs_stage<kDppQuadXor1, 2, 1>(x, j);
  // slot j <-> feature 16 (j >> 2) + 4 g + (j & 3)
  acc[fbase + 16 * (j >> 2) + 4 * g + (j & 3)] += x[0];
}

// PPO_UPD_NT (A/B): the hand-off rows (H1 / DZ2 / DZ1) as non-temporal stores
#ifndef PPO_UPD_NT
#define PPO_UPD_NT 0
#endif
template <int FT, int RT>
PPO_DEV void store_tile_rows(float* __restrict__ dst, int ld, const f4 (&v)[FT][RT], int m0, int M, int rbase,
                             int fbase, int j, int g, bool diag_blocked = false) {
#ifdef PPO_STAMPS
  if (diag_blocked) {  // timing only: the same bytes as 16-row x 64-feature blocks, 1 KB per store instruction
    const int lane = j + 16 * g;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const long blk = (long)((m0 + rbase) / 16 + rt) * (ld / 64) + fbase / 64;
      if (m0 + rbase + 16 * rt < M) {
#pragma unroll
        for (int ft = 0; ft < FT; ++ft) st4(dst + blk * 1024 + (ft * 64 + lane) * 4, v[ft][rt]);
      }
    }
    return;
  }
#else
  (void)diag_blocked;
#endif
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int m = m0 + rbase + 16 * rt + j;
    if (m < M) {
#pragma unroll
      for (int ft = 0; ft < FT; ++ft) {
#if PPO_UPD_NT
        __builtin_nontemporal_store(v[ft][rt], reinterpret_cast<f4*>(dst + (size_t)m * ld + fbase + 16 * ft + 4 * g));
#else
        st4(dst + (size_t)m * ld + fbase + 16 * ft + 4 * g, v[ft][rt]);
#endif
      }
    }
  }
}
template <int FT, int RT, int LDA>
PPO_DEV void lds_store_tile(float* act, const f4 (&v)[FT][RT], int rbase, int fbase, int j, int g) {
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) lds_st4(act + (rbase + 16 * rt + j) * LDA + fbase + 16 * ft + 4 * g, v[ft][rt]);
}

// packed offset of head h's weight row / bias, -1 if h is padding
PPO_DEV int head_row(const PackedLayout& K, int trunk, int h, int H) {
  if (trunk == 0) return h == 0 ? K.cW3 : -1;
  if (K.kind == PPO_NET_LN_BETA) {
    if (h < K.A) return K.aW3 + h * H;
    if (h < 2 * K.A) return K.bW3 + (h - K.A) * H;
    return -1;
  }
  return h < K.A ? K.aW3 + h * H : -1;
}
PPO_DEV int head_bias(const PackedLayout& K, int trunk, int h) {
  if (trunk == 0) return K.cb3;
  if (K.kind == PPO_NET_LN_BETA) return h < K.A ? K.ab3 + h : K.bb3 + (h - K.A);
  return K.ab3 + h;
}

}  // namespace

// The PPO loss of one tile and its gradient wrt the head pre-activations: PRE -> GG (critic: the
// clipped value loss, ppo:520-533; actor: Beta or Normal log-prob / entropy, the clipped surrogate,
// ppo:497-519, ac:815-875), the per-lane loss statistics added to lst. Shared by k_upd and k_upd32.
// pre(row, h): a head pre-activation for the critic and the one-row-per-8-lanes Beta loss (k_upd sums the
// head partials there directly); the other losses read the materialised PRE array.
template <bool LN, int R, int ITS, int LDG, typename PreFn>
PPO_DEV void upd_loss(const UpdArgs& a, int trunk, int tid, int m0, float c, float adv_mean, float adv_std,
                      PreFn pre, const float* PRE, float* GG, float* ROWS, const float* ACTN, float* ITM,
                      float (&lst)[6]) {
  const PackedLayout& K = a.K;
  const float* __restrict__ P = a.P;
  const int A = K.A;
  float st_a = 0.f, st_b = 0.f, st_c = 0.f, st_d = 0.f, st_e = 0.f, st_f = 0.f;  // per-row stats (tid < R)
  if (trunk == 0) {
    if (tid < R) {
      const bool valid = m0 + tid < a.M;
      const float v = pre(tid, 0);
      const float rt_ = ROWS[tid * 8 + 1], ov = ROWS[tid * 8 + 2];
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
      GG[tid * LDG] = gv;
      st_b = sv;
    }
  } else if (LN && R == 32 && A <= 8) {
    // Beta actor, one row per 8-lane group (32 rows x 8 lanes = the workgroup), one (row, action)
    // item per lane: the row's log-prob / entropy sums are DPP sums inside the group, every lane
    // of the group evaluates the row's surrogate, and the head gradients are written straight to
    // GG — no item scratch in LDS and one barrier instead of three
    const int row = tid >> 3, ai = tid & 7;
    const bool item = ai < A;
    const bool valid = m0 + row < a.M;
    const int ac = item ? ai : 0;  // lanes past A evaluate item 0 and drop it (uniform control flow)
    const float hi = P[K.hi], lo = P[K.lo];
    const float pa = pre(row, ac), pbv = pre(row, A + ac);
    const float al = softplusf_(pa) + 1.0f, be = softplusf_(pbv) + 1.0f;
    const float av = valid ? ACTN[row * A + ac] : 0.5f * (hi + lo);
    float s = (av - lo) / (hi - lo) * (1.0f - 0.0f) + 0.0f;
    s = fminf(fmaxf(s, 1e-7f), 1.0f + 1e-7f);
    const float ab = al + be;
    float lga, lgb, lgab, psa, psb, psab, ta, tb, tab;
    lgamma_digamma_trigamma(al, lga, psa, ta);
    lgamma_digamma_trigamma(be, lgb, psb, tb);
    lgamma_digamma_trigamma(ab, lgab, psab, tab);
    const float lpi = xlogyf_(al - 1.0f, s) + xlogyf_(be - 1.0f, 1.0f - s) + (lgab - (lga + lgb));
    const float eni = (lga + lgb) - lgab - (2.0f - ab) * psab - ((al - 1.0f) * psa + (be - 1.0f) * psb);
    const float lp = group8_sum(item ? lpi : 0.0f), ent = group8_sum(item ? eni : 0.0f);
    const float oldlp = valid ? ROWS[row * 8 + 1] : lp;
    const float logratio = lp - oldlp;
    const float ratio = expf(logratio);
    float an = valid ? ROWS[row * 8 + 2] : 0.f;
    if (a.norm_adv) an = (an - adv_mean) / (adv_std + 1e-8f);
    const float rc = fminf(fmaxf(ratio, 1.0f - c), 1.0f + c);
    const float pg1 = -an * ratio, pg2 = -an * rc;
    const float w1 = pg1 > pg2 ? 1.0f : (pg1 == pg2 ? 0.5f : 0.0f);
    const float inr = (ratio >= 1.0f - c && ratio <= 1.0f + c) ? 1.0f : 0.0f;
    float g_logp = a.inv_m * (w1 * (-an) + (1.0f - w1) * (-an) * inr) * ratio;
    float g_ent = -a.ent_coef * a.inv_m;
    if (!valid) { g_logp = 0.f; g_ent = 0.f; }
    if (ai == 0 && valid) {  // the row's statistics, once per row
      st_a = fmaxf(pg1, pg2);
      st_c = ent;
      st_d = -logratio;
      st_e = (ratio - 1.0f) - logratio;
      st_f = fabsf(ratio - 1.0f) > c ? 1.0f : 0.0f;
    }
    if (item) {
      const float dla = ((al - 1.0f) != 0.0f ? logf(s) : 0.0f) + psab - psa;         // d lp / d alpha
      const float dea = (ab - 2.0f) * tab - (al - 1.0f) * ta;                         // d ent / d alpha
      const float dlb = ((be - 1.0f) != 0.0f ? logf(1.0f - s) : 0.0f) + psab - psb;  // d lp / d beta
      const float deb = (ab - 2.0f) * tab - (be - 1.0f) * tb;                         // d ent / d beta
      GG[row * LDG + ai] = (g_logp * dla + g_ent * dea) * softplus_d(pa);
      GG[row * LDG + A + ai] = (g_logp * dlb + g_ent * deb) * softplus_d(pbv);
    }
  } else {
    // pass 1: per (row, action) log-prob / entropy terms and derivative pieces
    for (int idx = tid; idx < R * A; idx += 256) {
      const int row = idx / A, ai = idx - row * A;
      const bool valid = m0 + row < a.M;
      float* it_ = ITM + idx * ITS;
      if constexpr (LN) {
        const float hi = P[K.hi], lo = P[K.lo];
        const float pa = PRE[row * LDG + ai], pbv = PRE[row * LDG + A + ai];
        const float al = softplusf_(pa) + 1.0f, be = softplusf_(pbv) + 1.0f;
        const float av = valid ? ACTN[idx] : 0.5f * (hi + lo);
        float s = (av - lo) / (hi - lo) * (1.0f - 0.0f) + 0.0f;
        s = fminf(fmaxf(s, 1e-7f), 1.0f + 1e-7f);
        const float ab = al + be;
        float lga, lgb, lgab, psa, psb, psab, ta, tb, tab;
        lgamma_digamma_trigamma(al, lga, psa, ta);
        lgamma_digamma_trigamma(be, lgb, psb, tb);
        lgamma_digamma_trigamma(ab, lgab, psab, tab);
        it_[0] = xlogyf_(al - 1.0f, s) + xlogyf_(be - 1.0f, 1.0f - s) + (lgab - (lga + lgb));
        it_[1] = (lga + lgb) - lgab - (2.0f - ab) * psab - ((al - 1.0f) * psa + (be - 1.0f) * psb);
        it_[2] = ((al - 1.0f) != 0.0f ? logf(s) : 0.0f) + psab - psa;            // d lp / d alpha
        it_[3] = (ab - 2.0f) * tab - (al - 1.0f) * ta;                            // d ent / d alpha
        it_[4] = softplus_d(pa);
        it_[5] = ((be - 1.0f) != 0.0f ? logf(1.0f - s) : 0.0f) + psab - psb;     // d lp / d beta
        it_[6] = (ab - 2.0f) * tab - (be - 1.0f) * tb;                            // d ent / d beta
        it_[7] = softplus_d(pbv);
      } else {
        const float mu = PRE[row * LDG + ai];
        const float sd = expf(P[K.logstd + ai]);
        const float var = sd * sd, lsd = logf(sd);
        const float act = valid ? ACTN[idx] : mu;
        const float d = act - mu;
        it_[0] = -(d * d) / (2.0f * var) - lsd - kLz;
        it_[1] = kEntC + lsd;
        it_[2] = d / var;
        it_[3] = d * d / var - 1.0f;
      }
    }
    lds_barrier();
    // per row: log-prob / entropy sums, clipped surrogate, d loss / d logp, d loss / d ent
    if (tid < R) {
      const bool valid = m0 + tid < a.M;
      float lp = 0.f, ent = 0.f;
      for (int ai = 0; ai < A; ++ai) {
        lp += ITM[(tid * A + ai) * ITS + 0];
        ent += ITM[(tid * A + ai) * ITS + 1];
      }
      const float oldlp = valid ? ROWS[tid * 8 + 1] : lp;
      const float logratio = lp - oldlp;
      const float ratio = expf(logratio);
      float an = valid ? ROWS[tid * 8 + 2] : 0.f;
      if (a.norm_adv) an = (an - adv_mean) / (adv_std + 1e-8f);
      const float rc = fminf(fmaxf(ratio, 1.0f - c), 1.0f + c);
      const float pg1 = -an * ratio, pg2 = -an * rc;
      const float w1 = pg1 > pg2 ? 1.0f : (pg1 == pg2 ? 0.5f : 0.0f);
      const float inr = (ratio >= 1.0f - c && ratio <= 1.0f + c) ? 1.0f : 0.0f;
      float g_logp = a.inv_m * (w1 * (-an) + (1.0f - w1) * (-an) * inr) * ratio;
      float g_ent = -a.ent_coef * a.inv_m;
      st_a = fmaxf(pg1, pg2);
      st_c = ent;
      st_d = -logratio;
      st_e = (ratio - 1.0f) - logratio;
      st_f = fabsf(ratio - 1.0f) > c ? 1.0f : 0.0f;
      if (!valid) { g_logp = 0.f; g_ent = 0.f; st_a = st_c = st_d = st_e = st_f = 0.f; }
      ROWS[tid * 8 + 3] = g_logp;
      ROWS[tid * 8 + 4] = g_ent;
    }
    lds_barrier();
    // pass 2: head gradients
    for (int idx = tid; idx < R * A; idx += 256) {
      const int row = idx / A, ai = idx - row * A;
      const float g_logp = ROWS[row * 8 + 3], g_ent = ROWS[row * 8 + 4];
      float* it_ = ITM + idx * ITS;
      if constexpr (LN) {
        GG[row * LDG + ai] = (g_logp * it_[2] + g_ent * it_[3]) * it_[4];
        GG[row * LDG + A + ai] = (g_logp * it_[5] + g_ent * it_[6]) * it_[7];
      } else {
        GG[row * LDG + ai] = g_logp * it_[2];
        it_[4] = g_logp * it_[3] + g_ent;  // d loss / d logstd (per row)
      }
    }
  }
  // loss statistics: summed per lane over the tiles, reduced across lanes and waves once after
  // the tile loop (reported values only, no gradient depends on them)
  lst[0] += st_a; lst[1] += st_b; lst[2] += st_c; lst[3] += st_d; lst[4] += st_e; lst[5] += st_f;
}

// k_upd's body (a device function so that k_upd32's mixed form can run it for the actor trunk)
template <int H, int KIND, int NTO, int NHT, int KL1, bool BX = false>
PPO_DEV void upd16_body(const UpdArgs& a) {
  using GE = Geo<H, NTO, NHT, BX>;
  static_assert(!BX || (H == 256 && KIND == PPO_NET_LN_BETA), "split-bf16 form: LayerNorm-Beta agent, H = 256");
  constexpr int FT = GE::FT, RT = GE::RT, WF = GE::WF, R = GE::R, NT = GE::NT, OP = GE::OP;
  constexpr int LDX = GE::LDX, LDA = GE::LDA, LDG = GE::LDG, NHP = GE::NHP, ITS = GE::ITS;
  constexpr bool LN = KIND == PPO_NET_LN_BETA;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* XN = lds + GE::oXN;
  float* ACT = lds + GE::oACT;
  float* RED = lds + GE::oRED;
  float* PRE = lds + GE::oPRE;
  float* GG = lds + GE::oG;
  float* ROWS = lds + GE::oROW;
  float* SCR = lds + GE::oSCR;   // head partials, then per-item scratch
  float* ACTN = lds + a.actn_off;  // R x A stored actions
  float* ACC = lds + a.acc_off;    // WR x sg.size accumulators
  float* SPAR = lds + a.spar_off;  // staged gamma1 | beta1 | gamma2 | beta2 | head biases
  float* SG1 = SPAR;
  float* SBE1 = SPAR + H;
  float* SG2 = SPAR + 2 * H;
  float* SBE2 = SPAR + 3 * H;
  float* SHB = SPAR + 4 * H;
  float* SOM = SHB + NHP;
  float* SOS = SOM + OP;
  float* RED0 = RED;
  float* RED1 = RED + WF * R;
  float* RED2 = RED + 2 * WF * R;
  float* RED3 = RED + 3 * WF * R;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  const int wf = wave % WF, wr = wave / WF;
  const int fbase = wf * FT * 16, rbase = wr * RT * 16;
  // The actor's tile is the longer one (Beta loss, larger head); the hardware issues the oldest
  // wave first, so the actor workgroups are dispatched first (grid row 0) and, with sched bit 1,
  // also raise their wave priority; the critic's MFMA stream fills the actor's latency gaps.
  const int trunk = (a.sched & 1) ? 1 - (int)blockIdx.y : (int)blockIdx.y;
  if (!((a.trunk_mask >> trunk) & 1)) return;
  if ((a.sched & 2) && trunk == 1) __builtin_amdgcn_s_setprio(1);
#ifdef PPO_STAMPS
  // timing experiment: start the actor workgroups (a.sched >> 8) x ~8 K cycles late
  if (trunk == 1)
    for (int i = 0; i < (a.sched >> 8); ++i) __builtin_amdgcn_s_sleep(127);
#endif
  const PackedLayout& K = a.K;
  const TrunkDev& T = K.tr[trunk];
  const float* __restrict__ P = a.P;
  const PBuf pb = make_pbuf(P, K.size);
  const PBuf wsw = make_pbuf(a.WSW[trunk], (int)sw_size(H, OP));
  const SmallGradLayout sg = a.sg[trunk];
  const int O = K.O, A = K.A, nh = sg.nh;
  const float c = a.clip_coef;
  const float adv_mean = a.adv_stats[0], adv_std = a.adv_stats[1];
  // sl: the LDS accumulators' layout — sg's, or (hw_global, actor) sg without the head-weight
  // block, whose nh x H sums then accumulate in this workgroup's slab row (upd_geo)
  const bool hwg = a.hw_global && trunk == 1;
  SmallGradLayout sl = sg;
  if (hwg) {
    const int d = sg.nh * H;
    sl.hb -= d; sl.ls -= d; sl.stats -= d; sl.size -= d;
  }
  float* slab_row = a.slab[trunk] + (size_t)blockIdx.x * sg.size;
  float* acc = ACC + wr * sl.size;
  float* hwacc = hwg ? slab_row + sg.hW : acc + sg.hW;
  for (int i = tid; i < GE::WR * sl.size; i += 256) ACC[i] = 0.f;
  for (int i = tid; i < R * LDG; i += 256) GG[i] = 0.f;  // padding heads stay exactly 0
  if (hwg) {  // each owning lane zeroes the slab entries it will accumulate (see the head backward)
#pragma unroll
    for (int ht = 0; ht < NHT; ++ht)
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int h = 16 * ht + 4 * g + r;
          if (h < nh) hwacc[h * H + fbase + 16 * ft + j] = 0.f;
        }
  }

  // per-lane A-operand offsets into the swizzled W1 | W2 | W2^T (sw_index): this wave's feature blocks
  const int w1lane = ((fbase >> 4) * NTO * 64 + lane) * 4;
  const int w2lane = H * OP + ((fbase >> 4) * NT * 64 + lane) * 4;
  const int w2tlane = H * OP + H * H + ((fbase >> 4) * NT * 64 + lane) * 4;
  const float* xn_in = XN + (rbase + j) * LDX + 4 * g;
  const float* act_in = ACT + (rbase + j) * LDA + 4 * g;
  // BX: the pieces of W2 | W2^T (bx_index, after the fp32 copies) and of the activation rows
  constexpr int LDB = GE::LDB;
  const PBuf wbx = make_pbuf(a.WSW[trunk] + sw_size(H, OP), BX ? (int)bx_size(H) : 0);
  const int w2blane = ((fbase >> 4) * (NT / 2) * 3 * 64 + lane) * 4;
  const int w2tblane = 3 * H * H / 2 + w2blane;
  const float* actb_in = ACT + (rbase + j) * LDB + 4 * g;
  // head rows for the forward (A = W3[16 ht + i][..]) and the backward (A = W3^T: heads 16 ht + 4 g + r)
  int hrow_f[NHT], hrow_b[NHT][4];
#pragma unroll
  for (int ht = 0; ht < NHT; ++ht) {
    hrow_f[ht] = head_row(K, trunk, 16 * ht + j, H);
#pragma unroll
    for (int r = 0; r < 4; ++r) hrow_b[ht][r] = head_row(K, trunk, 16 * ht + 4 * g + r, H);
  }
  const int ntiles = (a.M + R - 1) / R;

  // Gather prefetch, two stages one tile ahead: permutation indices at the top of a tile, the
  // rows' data after its forward pass; committed to LDS at the top of the next tile.
  // (register-staged only for narrow inputs; wide ones (O > 32) gather synchronously)
  constexpr bool PREF = (R * OP + 255) / 256 <= 4 && !PPO_V_NOPREF;
  constexpr int NG = PREF ? (R * OP + 255) / 256 : 1;   // gather items per thread
  constexpr int NAI = PREF ? (R * PPO_UPD_MAXA + 255) / 256 : 1;  // action items per thread
  int pg[NG], pra, pac[NAI];
  float vg[NG], vr1 = 0.f, vr2 = 0.f, vac[NAI];
#if PPO_V_BF
  // every load is unconditional from a clamped (valid) address and masked by a select afterwards: a
  // load under a per-lane branch gets its own branch and, at the loop head, a vmcnt(0) wait
  auto pref_idx = [&](int itn) {
    const int mb = itn * R;
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      const int idx = tid + 256 * k, row = idx / OP, f = idx - row * OP, m = mb + row;
      const bool ok = itn < ntiles && idx < R * OP && m < a.M && f < O;
      const int pv = a.perm[ok ? m : 0];
      pg[k] = ok ? pv : -1;
    }
    {
      const bool ok = itn < ntiles && tid < R && mb + tid < a.M;
      const int pv = a.perm[ok ? mb + tid : 0];
      pra = ok ? pv : -1;
    }
#pragma unroll
    for (int k = 0; k < NAI; ++k) {
      const int idx = tid + 256 * k, row = idx / (A > 0 ? A : 1), m = mb + row;
      const bool ok = trunk == 1 && itn < ntiles && idx < R * A && m < a.M;
      const int pv = a.perm[ok ? m : 0];
      pac[k] = ok ? pv : -1;
    }
  };
  auto pref_data = [&](int itn) {
    (void)itn;
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      const int idx = tid + 256 * k, row = idx / OP, f = idx - row * OP;
      (void)row;
      const float v = a.obs[(long)(pg[k] >= 0 ? pg[k] : 0) * O + (f < O ? f : 0)];
      vg[k] = pg[k] >= 0 ? v : 0.f;
    }
    {
      const int pr = pra >= 0 ? pra : 0;
      const float x1 = trunk == 0 ? a.ret[pr] : a.logp[pr];
      const float x2 = trunk == 0 ? a.val[pr] : a.adv[pr];
      vr1 = pra >= 0 ? x1 : 0.f;
      vr2 = pra >= 0 ? x2 : 0.f;
    }
#pragma unroll
    for (int k = 0; k < NAI; ++k) {
      const int idx = tid + 256 * k, ai = idx - (idx / (A > 0 ? A : 1)) * A;
      const float v = a.actions[(long)(pac[k] >= 0 ? pac[k] : 0) * A + ai];
      vac[k] = pac[k] >= 0 ? v : 0.f;
    }
  };
#else
  auto pref_idx = [&](int itn) {
    const int mb = itn * R;
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      const int idx = tid + 256 * k, row = idx / OP, f = idx - row * OP, m = mb + row;
      pg[k] = (itn < ntiles && idx < R * OP && m < a.M && f < O) ? a.perm[m] : -1;
    }
    pra = (itn < ntiles && tid < R && mb + tid < a.M) ? a.perm[mb + tid] : -1;
#pragma unroll
    for (int k = 0; k < NAI; ++k) {
      const int idx = tid + 256 * k, row = idx / (A > 0 ? A : 1), m = mb + row;
      pac[k] = (trunk == 1 && itn < ntiles && idx < R * A && m < a.M) ? a.perm[m] : -1;
    }
  };
  auto pref_data = [&](int itn) {
    const int mb = itn * R;
    (void)mb;
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      const int idx = tid + 256 * k, row = idx / OP, f = idx - row * OP;
      (void)row;
      vg[k] = pg[k] >= 0 ? a.obs[(long)pg[k] * O + f] : 0.f;
    }
    if (pra >= 0) {
      if (trunk == 0) { vr1 = a.ret[pra]; vr2 = a.val[pra]; }
      else { vr1 = a.logp[pra]; vr2 = a.adv[pra]; }
    } else {
      vr1 = 0.f; vr2 = 0.f;
    }
#pragma unroll
    for (int k = 0; k < NAI; ++k) {
      const int idx = tid + 256 * k, ai = idx - (idx / (A > 0 ? A : 1)) * A;
      vac[k] = pac[k] >= 0 ? a.actions[(long)pac[k] * A + ai] : 0.f;
    }
  };
#endif
  auto commit = [&](int itc) {
    const int mb = itc * R;
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      const int idx = tid + 256 * k, row = idx / OP, f = idx - row * OP, m = mb + row;
      if (idx < R * OP) {
        float v = vg[k];
        if (LN && pg[k] >= 0) v = (v - SOM[f]) / SOS[f];
        XN[row * LDX + f] = v;
        if (trunk == 0 && m < a.M && !PPO_DIAG_SKIP(7)) a.Xn[(size_t)m * OP + f] = v;
      }
    }
    if (tid < R) {
      ROWS[tid * 8 + 1] = vr1;
      ROWS[tid * 8 + 2] = vr2;
    }
#pragma unroll
    for (int k = 0; k < NAI; ++k) {
      const int idx = tid + 256 * k;
      if (trunk == 1 && idx < R * A) ACTN[idx] = vac[k];
    }
  };
  // wide inputs: the tile's loads go out in chunks of GC items from clamped indices (the chunk's
  // permutation entries, then its observation values), masked afterwards — a load under a per-lane
  // branch would wait for itself, one dependent round trip pair per item
  // (the tile's permutation entries are in ROWS slot 0, loaded a tile ahead: only the data loads
  // are on the tile's critical path)
  auto perm_of = [&](int r) { return __float_as_int(ROWS[r * 8]); };
  auto gather_sync = [&](int itc) {
    const int mb = itc * R;
    constexpr int NGS = (R * OP + 255) / 256, GC = 4;
#pragma unroll 1
    for (int k0 = 0; k0 < NGS; k0 += GC) {
      int rp[GC];
      float v[GC];
#pragma unroll
      for (int c = 0; c < GC; ++c) {
        const int idx = tid + 256 * (k0 + c), row = min(idx / OP, R - 1);
        rp[c] = perm_of(row);
      }
#pragma unroll
      for (int c = 0; c < GC; ++c) {
        const int idx = tid + 256 * (k0 + c), f = idx - (idx / OP) * OP;
        v[c] = a.obs[(long)rp[c] * O + min(f, O - 1)];
      }
#pragma unroll
      for (int c = 0; c < GC; ++c) {
        const int idx = tid + 256 * (k0 + c), row = idx / OP, f = idx - row * OP, m = mb + row;
        if (k0 + c < NGS && idx < R * OP) {
          const bool ok = m < a.M && f < O;
          float x = ok ? v[c] : 0.f;
          if constexpr (LN)
            if (ok) x = (x - SOM[f]) / SOS[f];
          XN[row * LDX + f] = x;
          if (trunk == 0 && m < a.M && !PPO_DIAG_SKIP(7)) a.Xn[(size_t)m * OP + f] = x;
        }
      }
    }
    {
      const int rrow = perm_of(min(tid, R - 1));
      const float r1 = trunk == 0 ? a.ret[rrow] : a.logp[rrow];
      const float r2 = trunk == 0 ? a.val[rrow] : a.adv[rrow];
      if (tid < R) {
        const bool ok = mb + tid < a.M;
        ROWS[tid * 8 + 1] = ok ? r1 : 0.f;
        ROWS[tid * 8 + 2] = ok ? r2 : 0.f;
      }
    }
    if (trunk == 1) {
      constexpr int NAS = (R * PPO_UPD_MAXA + 255) / 256;
      int ap[NAS];
#pragma unroll
      for (int k = 0; k < NAS; ++k) {
        const int idx = tid + 256 * k, row = min(idx / (A > 0 ? A : 1), R - 1);
        ap[k] = perm_of(row);
      }
      float av[NAS];
#pragma unroll
      for (int k = 0; k < NAS; ++k) {
        const int idx = tid + 256 * k, ai = idx - (idx / (A > 0 ? A : 1)) * A;
        av[k] = a.actions[(long)ap[k] * A + ai];
      }
#pragma unroll
      for (int k = 0; k < NAS; ++k) {
        const int idx = tid + 256 * k, m = mb + idx / (A > 0 ? A : 1);
        if (idx < R * A) ACTN[idx] = m < a.M ? av[k] : 0.f;
      }
    }
  };
  // the first tile's permutation entries are requested before the staging loads below, so their
  // round trip overlaps the staging instead of following it
  if constexpr (PREF) pref_idx(blockIdx.x);
  // the per-tile LayerNorm / head-bias reads come from LDS instead of an L2 round trip each
  for (int i = tid; i < GE::NSPAR; i += 256) {
    const int v = i / H, f = i - v * H;
    float x = 0.f;
    if (v < 4) {
      if constexpr (LN) x = P[(v == 0 ? T.g1 : v == 1 ? T.be1 : v == 2 ? T.g2 : T.be2) + f];
    } else if (i < 4 * H + NHP) {
      if (i - 4 * H < nh) x = P[head_bias(K, trunk, i - 4 * H)];
    } else {
      const int q = i - 4 * H - NHP, o = q % OP;
      x = q < OP ? 0.f : 1.f;
      if constexpr (LN)
        if (o < O) x = P[(q < OP ? K.omean : K.ostd) + o];
    }
    SPAR[i] = x;
  }
  if constexpr (PREF) pref_data(blockIdx.x);
  // EARLY (narrow inputs, LayerNorm trunks over several waves): a tile's gathered rows are committed to
  // LDS by the PREVIOUS tile, right after its layer-1 backward exchange barrier (every wave is past its
  // last XN / ROWS / ACTN read of that tile by then), so the tile top is one barrier and a few loads;
  // the first tile's rows are committed here
  constexpr bool EARLY = PPO_UPD_EARLY && PREF && LN && WF > 1;
  constexpr bool DEFER = PPO_UPD_DEFER != 0;
  if constexpr (EARLY) {
    lds_barrier();  // SPAR (observation mean / std) is staged
    commit(blockIdx.x);
  }
  // TOP: the tile top writes XN / ROWS / ACTN without a barrier first: the previous tile's last readers
  // of them (layer-1 recompute, loss) all precede its layer-1 backward exchange barrier (rows_total2)
  constexpr bool TOP = PPO_V_TOP && !EARLY && PREF && LN && WF > 1;
  if constexpr (TOP) lds_barrier();  // SPAR (observation mean / std) is staged for the first commit
  // wide inputs: row tid's permutation entry of the next tile (clamped, as the gather clamps rows)
  int nperm = 0;
  if constexpr (!PREF) nperm = tid < R ? a.perm[min((int)blockIdx.x * R + tid, a.M - 1)] : 0;

  float lst[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // per-lane loss statistics over this workgroup's tiles
  for (int it = blockIdx.x; it < ntiles; it += gridDim.x) {
    const int m0 = it * R;
    PPO_STAMP_START();
    if constexpr (!PREF)
      if (tid < R) ROWS[tid * 8] = __int_as_float(nperm);  // slot 0 is read only by gather_sync
    if constexpr (!TOP) lds_barrier();  // the previous iteration's LDS readers are done (EARLY: rows committed)
    if constexpr (EARLY) {
      pref_idx(it + gridDim.x);
    } else if constexpr (PREF) {
      commit(it);
      if constexpr (!PPO_V_PLATE) pref_idx(it + gridDim.x);
    } else {
      if (tid < R) nperm = a.perm[min((it + (int)gridDim.x) * R + tid, a.M - 1)];
      gather_sync(it);
    }
    // one head tile (NHT == 1): its weights, in the layout the head backward reads them (critic: w3
    // features 4 g + r, which the forward dot product uses too; actor: heads 4 g + r of feature j),
    // are requested here, a whole forward pass before their first use, instead of in the head
    // phases (where they were the only loads a wave waited on outside the matrix phases)
    f4 hwb[FT];
    if constexpr (NHT == 1 && PPO_V_HWB) {
#pragma unroll
      for (int ft = 0; ft < FT; ++ft) {
        if (trunk == 0) {
          hwb[ft] = pld4(pb, K.cW3 + fbase + 4 * g, 16 * ft);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
#if PPO_V_BF
            const float v = bld1(pb, (hrow_b[0][r] >= 0 ? hrow_b[0][r] : 0) + fbase + j, 16 * ft);
            hwb[ft][r] = hrow_b[0][r] >= 0 ? v : 0.0f;
#else
            hwb[ft][r] = hrow_b[0][r] >= 0 ? bld1(pb, hrow_b[0][r] + fbase + j, 16 * ft) : 0.0f;
#endif
          }
        }
      }
    }
    if constexpr (!EARLY) lds_barrier();
    PPO_STAMP(0);

    // ---------------- layer 1 ----------------
    f4 z[FT][RT];
    init_bias<FT, RT>(z, pb, T.b1 + fbase + 4 * g);
    mm_fr<FT, RT, NTO, LDX, KL1>(z, wsw, w1lane, xn_in);
    PPO_STAMP(1);
    float mu1[RT], rs1[RT];
    if constexpr (LN) {
      ln_rows<FT, RT, WF, R, H>(z, mu1, rs1, RED0, RED1, wf, rbase, j, g);
#pragma unroll
      for (int ft = 0; ft < FT; ++ft) {
        const f4 gm = lds_f4(SG1 + fbase + 4 * g + 16 * ft), bt = lds_f4(SBE1 + fbase + 4 * g + 16 * ft);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float xh = (z[ft][rt][r] - mu1[rt]) * rs1[rt];
            const float y = __fmaf_rn(gm[r], xh, bt[r]);
            z[ft][rt][r] = y > 0.0f ? y : 0.0f;
          }
      }
    } else {
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) z[ft][rt][r] = tanhf(z[ft][rt][r]);
    }
    if (a.h1_skip) {
      // h1_handoff=recompute: no H1 rows; k_dwf_bx recomputes them from Xn, W1 and these statistics
      if constexpr (LN) {
        if (wf == 0 && g == 0) {
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) {
            const int m = m0 + rbase + 16 * rt + j;
            typedef float fl2 __attribute__((ext_vector_type(2)));
            if (m < a.M) *reinterpret_cast<fl2*>(a.LNS[trunk] + 2 * (size_t)m) = fl2{mu1[rt], rs1[rt]};
          }
        }
      }
    } else if (!PPO_DIAG_SKIP(4) && !(DEFER && BX)) {
      store_tile_rows<FT, RT>(a.H1[trunk], H, z, m0, a.M, rbase, fbase, j, g, PPO_DIAG_SKIP(14));
    }
    if constexpr (BX) lds_store_pieces<FT, RT, LDB, H / 2>(ACT, z, rbase, fbase, j, g);
    else lds_store_tile<FT, RT, LDA>(ACT, z, rbase, fbase, j, g);
    lds_barrier();
    PPO_STAMP(2);

    // ---------------- layer 2 ----------------
    f4 x2[FT][RT];  // LN: x_hat2; tanh: h2
    init_bias<FT, RT>(x2, pb, T.b2 + fbase + 4 * g);
    if constexpr (BX && DEFER) {
      const bool st_h1 = !a.h1_skip && !PPO_DIAG_SKIP(4);
      mm_bx<FT, RT, NT, LDB>(x2, wbx, w2blane, actb_in, PPO_DIAG_SKIP(13), [&]() {
        if (st_h1) store_rows_from_pieces<FT, RT, LDB, H / 2>(a.H1[trunk], H, ACT, m0, a.M, rbase, fbase, j, g);
      });
    } else if constexpr (BX) {
      mm_bx<FT, RT, NT, LDB>(x2, wbx, w2blane, actb_in, PPO_DIAG_SKIP(13));
    } else {
      mm_fr<FT, RT, NT, LDA>(x2, wsw, w2lane, act_in);
    }
    PPO_STAMP(3);
    if constexpr (PREF && (!PPO_V_PLATE || EARLY)) pref_data(it + gridDim.x);
    if constexpr (PREF && PPO_V_PLATE && !EARLY) pref_idx(it + gridDim.x);
    float rs2[RT];
    if constexpr (LN) {
      float mu2[RT];
      ln_rows<FT, RT, WF, R, H>(x2, mu2, rs2, RED2, RED3, wf, rbase, j, g);
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) x2[ft][rt] = (x2[ft][rt] - mu2[rt]) * rs2[rt];
    } else {
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) x2[ft][rt][r] = tanhf(x2[ft][rt][r]);
    }
    auto h2_of = [&](int ft, int rt) -> f4 {
      if constexpr (LN) {
        const f4 gm = lds_f4(SG2 + fbase + 4 * g + 16 * ft), bt = lds_f4(SBE2 + fbase + 4 * g + 16 * ft);
        f4 y;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = __fmaf_rn(gm[r], x2[ft][rt][r], bt[r]);
          y[r] = v > 0.0f ? v : 0.0f;
        }
        return y;
      } else {
        return x2[ft][rt];
      }
    };
    PPO_STAMP(4);
    // ---------------- heads (split-K over this wave's features) ----------------
    f4 hp[NHT][RT];
#pragma unroll
    for (int ht = 0; ht < NHT; ++ht)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) hp[ht][rt] = f4{0.f, 0.f, 0.f, 0.f};
    // every wave is done reading h1 from ACT: LN2's exchange barrier (ln_rows) already follows every
    // wave's layer-2 GEMM; tanh trunks and one-wave rows (WF = 1) have no exchange, so they wait here
    if constexpr (!PPO_V_BAR || !LN || WF == 1) lds_barrier();
    if constexpr (BX) {  // GG shares the activation region: padding heads must read exactly 0
      for (int i = tid; i < R * LDG; i += 256) GG[i] = 0.f;
    }
    if (trunk == 0) {
      // critic: one real head of NHP — a per-row dot product on the VALU (in-lane over the wave's
      // features, then the 4 lane groups) instead of 15/16-padding MFMAs
      float pv[RT];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) pv[rt] = 0.f;
#pragma unroll
      for (int ft = 0; ft < FT; ++ft) {
        const f4 w = (NHT == 1 && PPO_V_HWB) ? hwb[ft] : pld4(pb, K.cW3 + fbase + 4 * g, 16 * ft);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          // no LDS copy of the critic's h2: its head backward and dW3 column sums read registers
          const f4 h2 = h2_of(ft, rt);
          if constexpr (!PPO_V_CH2) lds_st4(ACT + (rbase + 16 * rt + j) * LDA + fbase + 16 * ft + 4 * g, h2);
#pragma unroll
          for (int r = 0; r < 4; ++r) pv[rt] = fmaf(w[r], h2[r], pv[rt]);
        }
      }
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        pv[rt] = row_allreduce(pv[rt]);
        if (g == 0) SCR[(wf * NHP) * R + rbase + 16 * rt + j] = pv[rt];
      }
    } else {
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      f4 wv[NHT];
#pragma unroll
      for (int ht = 0; ht < NHT; ++ht) {
        wv[ht] = hrow_f[ht] >= 0 ? pld4(pb, hrow_f[ht] + fbase + 4 * g, 16 * ft) : f4{0.f, 0.f, 0.f, 0.f};
      }
      f4 h2v[RT];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        h2v[rt] = h2_of(ft, rt);
        lds_st4(ACT + (rbase + 16 * rt + j) * LDA + fbase + 16 * ft + 4 * g, h2v[rt]);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int ht = 0; ht < NHT; ++ht) hp[ht][rt] = mfma16(wv[ht][c], h2v[rt][c], hp[ht][rt]);
    }
    // partial head sums -> SCR[wf][head][row]
#pragma unroll
    for (int ht = 0; ht < NHT; ++ht)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) SCR[(wf * NHP + 16 * ht + 4 * g + r) * R + rbase + 16 * rt + j] = hp[ht][rt][r];
    }  // actor heads
    lds_barrier();
    PPO_STAMP(5);
    float* ITM = SCR;  // R x A x ITS (head partials are consumed)
    // the critic and the one-row-per-8-lanes Beta loss read each pre-activation straight from the WF
    // partial sums (same order, bitwise the materialised PRE): no PRE pass and no barrier; the other
    // losses reuse SCR as item scratch, so they need PRE first
    auto psum = [&](int row, int h) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < WF; ++w) s += SCR[(w * NHP + h) * R + row];
      return s + SHB[h];
    };
    auto pre = [&](int row, int h) {
      if constexpr (PPO_V_PRE) return psum(row, h);
      else return PRE[row * LDG + h];
    };
    if (!PPO_V_PRE || !(trunk == 0 || (LN && R == 32 && A <= 8))) {
      for (int idx = tid; idx < R * nh; idx += 256) {
        const int row = idx / nh, h = idx - row * nh;
        PRE[row * LDG + h] = psum(row, h);
      }
      lds_barrier();
    }
    PPO_STAMP(6);
    // ---------------- loss and its gradient wrt the head pre-activations ----------------
    upd_loss<LN, R, ITS, LDG>(a, trunk, tid, m0, c, adv_mean, adv_std, pre, PRE, GG, ROWS, ACTN, ITM, lst);
    lds_barrier();
    PPO_STAMP(7);
    // head bias (and logstd) gradients: fixed-order sums over the workgroup's rows
    if (tid < nh) {
      float s = 0.f;
      for (int row = 0; row < R; ++row) s += GG[row * LDG + tid];
      ACC[sl.hb + tid] += s;
    }
    if (!LN && trunk == 1 && tid >= 64 && tid < 64 + A) {
      const int ai = tid - 64;
      float s = 0.f;
      for (int row = 0; row < R; ++row) s += ITM[(row * A + ai) * ITS + 4];
      ACC[sl.ls + ai] += s;
    }

    // ---------------- head backward: dh2 = W3^T G^T, dW3 += G^T h2 ----------------
    f4 dh[FT][RT];
    zero<FT, RT>(dh);
    if (trunk == 0) {
      // critic: dh2 = w3 g (outer product), dW3 = column sums of g h2 over the rows (VALU)
      float gr[RT];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) gr[rt] = lds_f(GG + (rbase + 16 * rt + j) * LDG);
#pragma unroll
      for (int ft = 0; ft < FT; ++ft) {
        const f4 w = (NHT == 1 && PPO_V_HWB) ? hwb[ft] : pld4(pb, K.cW3 + fbase + 4 * g, 16 * ft);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) dh[ft][rt][r] = w[r] * gr[rt];
      }
      if (!PPO_DIAG_SKIP(12)) col_sums<FT, RT>([&](int ft, int rt, int r) { return gr[rt] * h2_of(ft, rt)[r]; }, acc + sg.hW, fbase, j, g);
    } else {
#pragma unroll
    for (int ht = 0; ht < NHT; ++ht) {
#pragma unroll
      for (int ft = 0; ft < FT; ++ft) {
        f4 wT;
        if constexpr (NHT == 1 && PPO_V_HWB) {
          wT = hwb[ft];
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            wT[r] = hrow_b[ht][r] >= 0 ? bld1(pb, hrow_b[ht][r] + fbase + j, 16 * ft) : 0.0f;
        }
        f4 gvv[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) gvv[rt] = lds_f4(GG + (rbase + 16 * rt + j) * LDG + 16 * ht + 4 * g);
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) dh[ft][rt] = mfma16(wT[c], gvv[rt][c], dh[ft][rt]);
        // dW3 tile (heads 16 ht.., features fbase + 16 ft ..): contract over this wave's rows
        f4 d3 = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = rbase + 16 * rt + 4 * g + r;
            d3 = mfma16(lds_f(GG + row * LDG + 16 * ht + j), lds_f(ACT + row * LDA + fbase + 16 * ft + j), d3);
          }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int h = 16 * ht + 4 * g + r;
          if (h < nh) hwacc[h * H + fbase + 16 * ft + j] += d3[r];
        }
      }
    }
    }  // actor head backward

    PPO_STAMP(8);
    // ---------------- layer-2 backward: dz2 ----------------
    if constexpr (LN) {
      float s1[RT], s2[RT];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) { s1[rt] = 0.f; s2[rt] = 0.f; }
#pragma unroll
      for (int ft = 0; ft < FT; ++ft) {
        const f4 gm = lds_f4(SG2 + fbase + 4 * g + 16 * ft), bt = lds_f4(SBE2 + fbase + 4 * g + 16 * ft);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float y = __fmaf_rn(gm[r], x2[ft][rt][r], bt[r]);
            const float dy = y > 0.0f ? dh[ft][rt][r] : 0.0f;
            dh[ft][rt][r] = dy;
            const float dx = dy * gm[r];
            s1[rt] += dx;
            s2[rt] += dx * x2[ft][rt][r];
          }
      }
      rows_total2<WF, RT, R>(s1, s2, RED0, RED1, wf, rbase, j, g);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) { s1[rt] *= (1.0f / H); s2[rt] *= (1.0f / H); }
      if (!PPO_DIAG_SKIP(12)) col_sums<FT, RT>([&](int ft, int rt, int r) { return dh[ft][rt][r]; }, acc + sg.be2, fbase, j, g);
      if (!PPO_DIAG_SKIP(12)) col_sums<FT, RT>([&](int ft, int rt, int r) { return dh[ft][rt][r] * x2[ft][rt][r]; }, acc + sg.g2, fbase, j, g);
#pragma unroll
      for (int ft = 0; ft < FT; ++ft) {
        const f4 gm = lds_f4(SG2 + fbase + 4 * g + 16 * ft);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) x2[ft][rt] = rs2[rt] * (dh[ft][rt] * gm - s1[rt] - x2[ft][rt] * s2[rt]);
      }
    } else {
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) x2[ft][rt] = dh[ft][rt] * (1.0f - x2[ft][rt] * x2[ft][rt]);
    }
    // x2 = dz2
    if (!PPO_DIAG_SKIP(12)) col_sums<FT, RT>([&](int ft, int rt, int r) { return x2[ft][rt][r]; }, acc + sg.b2, fbase, j, g);
    if (!PPO_DIAG_SKIP(5) && !(DEFER && BX)) store_tile_rows<FT, RT>(a.DZ2[trunk], H, x2, m0, a.M, rbase, fbase, j, g, PPO_DIAG_SKIP(14));
    // the head backward's readers of h2 / GG (ACT) are done: LN2-backward's exchange barrier (rows_total2)
    // follows every wave's head backward; without it (tanh, WF = 1) wait here
    if constexpr (!PPO_V_BAR || !LN || WF == 1) lds_barrier();
    if constexpr (BX) lds_store_pieces<FT, RT, LDB, H / 2>(ACT, x2, rbase, fbase, j, g);
    else lds_store_tile<FT, RT, LDA>(ACT, x2, rbase, fbase, j, g);
    lds_barrier();
    PPO_STAMP(9);

    // ---------------- dh1 = W2^T dz2 ----------------
    zero<FT, RT>(dh);
    if constexpr (BX && DEFER) {
      mm_bx<FT, RT, NT, LDB>(dh, wbx, w2tblane, actb_in, PPO_DIAG_SKIP(13), [&]() {
        if (!PPO_DIAG_SKIP(5)) store_rows_from_pieces<FT, RT, LDB, H / 2>(a.DZ2[trunk], H, ACT, m0, a.M, rbase, fbase, j, g);
      });
    } else if constexpr (BX) {
      mm_bx<FT, RT, NT, LDB>(dh, wbx, w2tblane, actb_in, PPO_DIAG_SKIP(13));
    } else {
      mm_fr<FT, RT, NT, LDA>(dh, wsw, w2tlane, act_in);
    }
    PPO_STAMP(10);
    if constexpr (PREF && PPO_V_PLATE && !EARLY) pref_data(it + gridDim.x);
    // ---------------- recompute layer 1, layer-1 backward ----------------
    init_bias<FT, RT>(z, pb, T.b1 + fbase + 4 * g);
    mm_fr<FT, RT, NTO, LDX, KL1>(z, wsw, w1lane, xn_in);
    PPO_STAMP(11);
    if constexpr (LN) {
      float s1[RT], s2[RT];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) { s1[rt] = 0.f; s2[rt] = 0.f; }
#pragma unroll
      for (int ft = 0; ft < FT; ++ft) {
        const f4 gm = lds_f4(SG1 + fbase + 4 * g + 16 * ft), bt = lds_f4(SBE1 + fbase + 4 * g + 16 * ft);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float xh = (z[ft][rt][r] - mu1[rt]) * rs1[rt];
            z[ft][rt][r] = xh;
            const float y = __fmaf_rn(gm[r], xh, bt[r]);
            const float dy = y > 0.0f ? dh[ft][rt][r] : 0.0f;
            dh[ft][rt][r] = dy;
            const float dx = dy * gm[r];
            s1[rt] += dx;
            s2[rt] += dx * xh;
          }
      }
      rows_total2<WF, RT, R>(s1, s2, RED2, RED3, wf, rbase, j, g);
      if constexpr (EARLY) commit(it + gridDim.x);  // the next tile's rows (see EARLY)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) { s1[rt] *= (1.0f / H); s2[rt] *= (1.0f / H); }
      if (!PPO_DIAG_SKIP(12)) col_sums<FT, RT>([&](int ft, int rt, int r) { return dh[ft][rt][r]; }, acc + sg.be1, fbase, j, g);
      if (!PPO_DIAG_SKIP(12)) col_sums<FT, RT>([&](int ft, int rt, int r) { return dh[ft][rt][r] * z[ft][rt][r]; }, acc + sg.g1, fbase, j, g);
#pragma unroll
      for (int ft = 0; ft < FT; ++ft) {
        const f4 gm = lds_f4(SG1 + fbase + 4 * g + 16 * ft);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) z[ft][rt] = rs1[rt] * (dh[ft][rt] * gm - s1[rt] - z[ft][rt] * s2[rt]);
      }
    } else {
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float h1 = tanhf(z[ft][rt][r]);
            z[ft][rt][r] = dh[ft][rt][r] * (1.0f - h1 * h1);
          }
    }
    // z = dz1
    if (!PPO_DIAG_SKIP(12)) col_sums<FT, RT>([&](int ft, int rt, int r) { return z[ft][rt][r]; }, acc + sg.b1, fbase, j, g);
    if (!PPO_DIAG_SKIP(6)) store_tile_rows<FT, RT>(a.DZ1[trunk], H, z, m0, a.M, rbase, fbase, j, g, PPO_DIAG_SKIP(14));
    PPO_STAMP(12);
  }
  // ---------------- workgroup result (row groups summed in a fixed order) ----------------
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1)
#pragma unroll
    for (int k = 0; k < 6; ++k) lst[k] += shfl_xor(lst[k], m);
  lds_barrier();  // RED is free
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 6; ++k) RED[wave * 8 + k] = lst[k];
  }
  lds_barrier();
  if (tid == 0) {
    float t[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) t[k] = (RED[k] + RED[8 + k]) + (RED[16 + k] + RED[24 + k]);
    float* st = ACC + sl.stats;  // row group 0's accumulator
    st[ST_PG] += t[0]; st[ST_V] += t[1]; st[ST_ENT] += t[2];
    st[ST_OKL] += t[3]; st[ST_KL] += t[4]; st[ST_CF] += t[5];
  }
  lds_barrier();
  // LDS accumulators -> the slab row (sg's layout); with hwg the head-weight block is already there
  for (int i = tid; i < sl.size; i += 256) {
    float s = ACC[i];
#pragma unroll
    for (int w = 1; w < GE::WR; ++w) s += ACC[w * sl.size + i];
    slab_row[hwg && i >= sg.hW ? i + sg.nh * H : i] = s;
  }
}

// =============================================================================================
// k_upd32: k_upd on v_mfma_f32_32x32x2_f32 (create option upd_mfma=32; LayerNorm-Beta agent, H = 256).
//
// Same contract, LDS carve, gather, loss and accumulators as k_upd; the three 256-wide GEMMs of a
// tile (layer 2, dh1 = W2^T dz2, layer 1 twice) and the actor's head backward run as 32 x 32 x 2
// MFMAs on a 32-row tile per wave, so every activation is 2 feature tiles x 16 registers per lane:
// lane (j = row, h = lane >> 5), register r of tile ft = feature fbase + 32 ft + 8 (r >> 2) + 4 h + (r & 3).
// Why: a 32x32x2 f32 MFMA issues for 64 cycles, and a partner wave on the same SIMD co-issues 6.2
// VALU instructions beside it against 2.2 beside a 16x16x4 (32 cycles) — 1.4x the VALU per FLOP
// (profiles/r02/probe/mfma_valu_coissue.jsonl), and k_upd's latency-bound phases (LayerNorm
// backward, loss, column sums) run beside the partner trunk's GEMMs. Row statistics are in-lane
// sums over 32 features plus one v_permlane32_swap; column sums a 32-lane reduce-scatter (one
// v_permlane16_swap stage ahead of k_upd's four DPP stages). The A operands come from the same
// swizzled copies (16-byte pieces of the 16 x 16 blocks, four 256-byte runs per wave-load); the B
// operand of a k-block is one ds_read_b128 of the lane's row (conflict-free at row stride 4 mod 64).
// The forward heads and the head-weight gradient stay 16x16x4 MFMAs reading h2 from LDS (padding the
// 12 heads to 32 would double them). Summation orders differ from k_upd (not bitwise equal to it);
// the parity tests compare both with the oracle.
// =============================================================================================
namespace {
typedef float f16v __attribute__((ext_vector_type(16)));
PPO_DEV f16v mfma32(float a, float b, f16v c) { return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0); }
PPO_DEV f4 quad(const f16v& v, int q) { return f4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]}; }
PPO_DEV void set_quad(f16v& v, int q, f4 x) {
  v[4 * q] = x.x;
  v[4 * q + 1] = x.y;
  v[4 * q + 2] = x.z;
  v[4 * q + 3] = x.w;
}

// out[ft] (+)= sum_k W[fbase + 32 ft + i][k] IN[j][k] over NKB 8-wide k-blocks (the last one: KLAST
// k-steps). alane: this lane's float offset of the wave's first A piece in the swizzled copy (the
// matrix base, the wave's 32-row block, (i >> 4) NC/16 blocks, lane group h, row i & 15);
// in = IN + j LDI + 4 h. Step c of k-block kb covers columns 8 kb + c (h = 0) and 8 kb + 4 + c.
template <int NKB, int KLAST, int NC>
PPO_DEV void mm32(f16v (&out)[2], PBuf wb, int alane, const float* in) {
  constexpr int FS = 32 * NC;  // floats between the wave's two 32-row feature tiles
  constexpr int PD = 2;        // A pieces requested two k-blocks (2 x 512 MFMA cycles) ahead
  auto ko = [](int kb) { return (kb >> 1) * 256 + (kb & 1) * 128; };
  f4 w[PD + 1][2];
#pragma unroll
  for (int p = 0; p < PD && p < NKB; ++p)
#pragma unroll
    for (int ft = 0; ft < 2; ++ft) w[p][ft] = pld4(wb, alane, FS * ft + ko(p));
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) {
    if (kb + PD < NKB) {
#pragma unroll
      for (int ft = 0; ft < 2; ++ft) w[(kb + PD) % (PD + 1)][ft] = pld4(wb, alane, FS * ft + ko(kb + PD));
    }
    __builtin_amdgcn_sched_barrier(0);
    const f4 b = lds_f4(in + 8 * kb);
    const int nc = kb + 1 < NKB ? 4 : KLAST;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c >= nc) break;
#pragma unroll
      for (int ft = 0; ft < 2; ++ft) out[ft] = mfma32(w[kb % (PD + 1)][ft][c], b[c], out[ft]);
    }
  }
}

// out = the bias vector in the 32x32 layout (boff_lane = bias + fbase + 4 h)
PPO_DEV void init_bias32(f16v (&out)[2], PBuf pb, int boff_lane) {
#pragma unroll
  for (int ft = 0; ft < 2; ++ft)
#pragma unroll
    for (int q = 0; q < 4; ++q) set_quad(out[ft], q, pld4(pb, boff_lane, 32 * ft + 8 * q));
}

PPO_DEV float lane_sum32(const f16v (&v)[2]) {
  float t = 0.f;
#pragma unroll
  for (int ft = 0; ft < 2; ++ft)
#pragma unroll
    for (int q = 0; q < 4; ++q) t += (v[ft][4 * q] + v[ft][4 * q + 1]) + (v[ft][4 * q + 2] + v[ft][4 * q + 3]);
  return t;
}

// row j's total over the 256 features from the lane partials: + the other lane half, then the four
// waves through LDS (red: [4][32]); contains a barrier
PPO_DEV float rows32(float s, float* red, int wave, int j, int h) {
  s = xor32_sum(s);
  if (h == 0) red[wave * 32 + j] = s;
  lds_barrier();
  float t = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w) t += red[w * 32 + j];
  return t;
}
PPO_DEV void rows32x2(float& s, float& q, float* red0, float* red1, int wave, int j, int h) {
  s = xor32_sum(s);
  q = xor32_sum(q);
  if (h == 0) {
    red0[wave * 32 + j] = s;
    red1[wave * 32 + j] = q;
  }
  lds_barrier();
  float t = 0.f, u = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    t += red0[w * 32 + j];
    u += red1[w * 32 + j];
  }
  s = t;
  q = u;
}

// LayerNorm statistics of row j (two-pass, eps 1e-5, biased variance as torch::layer_norm)
PPO_DEV void ln32(const f16v (&z)[2], float& mu, float& rs, float* red0, float* red1, int wave, int j, int h) {
  mu = rows32(lane_sum32(z), red0, wave, j, h) * (1.0f / 256);
  float t = 0.f;
#pragma unroll
  for (int ft = 0; ft < 2; ++ft)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float d = z[ft][r] - mu;
      t = __fmaf_rn(d, d, t);
    }
  rs = 1.0f / sqrtf(__fmaf_rn(rows32(t, red1, wave, j, h), 1.0f / 256, 1e-5f));
}

// column sums over the tile's 32 rows of v(ft, r), added to acc[feature]: the j / j + 16 halves by
// v_permlane16_swap (rows 0 | 2 keep tile 0, rows 1 | 3 tile 1), then k_upd's 16-lane
// reduce-scatter; lane j ends with register j & 15 of tile j >> 4 summed over all rows
template <typename Fn>
PPO_DEV void col_sums32(Fn v, float* acc, int fbase, int j, int h) {
  float x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const auto p = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v(0, i)),
                                                    __builtin_bit_cast(unsigned, v(1, i)), false, false);
    x[i] = __builtin_bit_cast(float, (unsigned)p[0]) + __builtin_bit_cast(float, (unsigned)p[1]);
  }
  const int jj = j & 15;
  rs_stage_banked(x);
  rs_stage<kDppQuadMirror, 4, 2>(x, jj);
  rs_stage<kDppQuadXor1, 2, 1>(x, jj);
  acc[fbase + 32 * (j >> 4) + 8 * (jj >> 2) + 4 * h + (jj & 3)] += x[0];
}

PPO_DEV void store_rows32(float* __restrict__ dst, int ld, const f16v (&v)[2], int m, int M, int fh) {
  if (m < M) {
#pragma unroll
    for (int ft = 0; ft < 2; ++ft)
#pragma unroll
      for (int q = 0; q < 4; ++q) st4(dst + (size_t)m * ld + fh + 32 * ft + 8 * q, quad(v[ft], q));
  }
}
template <int LDA>
PPO_DEV void lds_store32(float* act, const f16v (&v)[2], int j, int fh) {
#pragma unroll
  for (int ft = 0; ft < 2; ++ft)
#pragma unroll
    for (int q = 0; q < 4; ++q) lds_st4(act + j * LDA + fh + 32 * ft + 8 * q, quad(v[ft], q));
}
PPO_DEV void zero32(f16v (&v)[2]) {
#pragma unroll
  for (int ft = 0; ft < 2; ++ft)
#pragma unroll
    for (int r = 0; r < 16; ++r) v[ft][r] = 0.f;
}
}  // namespace

template <int NTO, int NHT, int KL1>
PPO_DEV void upd32_body(const UpdArgs& a) {
  constexpr int H = 256;
  using GE = Geo<H, NTO, NHT>;
  constexpr int R = GE::R, OP = GE::OP, NHP = GE::NHP, ITS = GE::ITS;
  constexpr int LDX = GE::LDX, LDA = GE::LDA, LDG = GE::LDG;
  static_assert(R == 32 && GE::WF == 4, "k_upd32: 32-row tiles, 4 feature waves");
  // layer 1's 8-wide k-blocks: with K = 16 (NTO - 1) + 1 (KL1 == 1) only column 16 (NTO - 1) of the
  // last 16-wide block is real, i.e. step 0 of its first 8-wide block
  constexpr int NKB1 = KL1 == 1 ? 2 * (NTO - 1) + 1 : 2 * NTO, KLAST1 = KL1 == 1 ? 1 : 4;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* XN = lds + GE::oXN;
  float* ACT = lds + GE::oACT;
  float* RED = lds + GE::oRED;
  float* PRE = lds + GE::oPRE;
  float* GG = lds + GE::oG;
  float* ROWS = lds + GE::oROW;
  float* SCR = lds + GE::oSCR;
  float* ACTN = lds + a.actn_off;
  float* ACC = lds + a.acc_off;
  float* SPAR = lds + a.spar_off;  // gamma1 | beta1 | gamma2 | beta2 | head biases | obs mean | std
  float* SG1 = SPAR;
  float* SBE1 = SPAR + H;
  float* SG2 = SPAR + 2 * H;
  float* SBE2 = SPAR + 3 * H;
  float* SHB = SPAR + 4 * H;
  float* SOM = SHB + NHP;
  float* SOS = SOM + OP;
  float* RED0 = RED;
  float* RED1 = RED + 4 * R;
  float* RED2 = RED + 8 * R;
  float* RED3 = RED + 12 * R;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = lane & 31, h = lane >> 5;    // 32x32 layout: row, lane half
  const int j16 = lane & 15, g = lane >> 4;  // 16x16 layout (forward heads, head-weight gradient)
  const int fbase = 64 * wave, fh = fbase + 4 * h;
  const int trunk = (a.sched & 1) ? 1 - (int)blockIdx.y : (int)blockIdx.y;
  if (!((a.trunk_mask >> trunk) & 1)) return;
  if ((a.sched & 2) && trunk == 1) __builtin_amdgcn_s_setprio(1);
  const PackedLayout& K = a.K;
  const TrunkDev& T = K.tr[trunk];
  const float* __restrict__ P = a.P;
  const PBuf pb = make_pbuf(P, K.size);
  const PBuf wsw = make_pbuf(a.WSW[trunk], (int)sw_size(H, OP));
  const SmallGradLayout sg = a.sg[trunk];
  const int O = K.O, A = K.A, nh = sg.nh;
  const float c = a.clip_coef;
  const float adv_mean = a.adv_stats[0], adv_std = a.adv_stats[1];
  const bool hwg = a.hw_global && trunk == 1;
  SmallGradLayout sl = sg;
  if (hwg) {
    const int d = sg.nh * H;
    sl.hb -= d; sl.ls -= d; sl.stats -= d; sl.size -= d;
  }
  float* slab_row = a.slab[trunk] + (size_t)blockIdx.x * sg.size;
  float* acc = ACC;
  float* hwacc = hwg ? slab_row + sg.hW : acc + sg.hW;
  for (int i = tid; i < sl.size; i += 256) ACC[i] = 0.f;
  for (int i = tid; i < R * LDG; i += 256) GG[i] = 0.f;
  if (hwg) {  // each owning lane zeroes the slab entries it accumulates (head-weight gradient, 16x16)
#pragma unroll
    for (int ht = 0; ht < NHT; ++ht)
#pragma unroll
      for (int ft = 0; ft < 4; ++ft)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int hh = 16 * ht + 4 * g + r;
          if (hh < nh) hwacc[hh * H + fbase + 16 * ft + j16] = 0.f;
        }
  }
  for (int i = tid; i < GE::NSPAR; i += 256) {
    const int v = i / H, f = i - v * H;
    float x = 0.f;
    if (v < 4) {
      x = P[(v == 0 ? T.g1 : v == 1 ? T.be1 : v == 2 ? T.g2 : T.be2) + f];
    } else if (i < 4 * H + NHP) {
      if (i - 4 * H < nh) x = P[head_bias(K, trunk, i - 4 * H)];
    } else {
      const int q = i - 4 * H - NHP, o = q % OP;
      x = q < OP ? 0.f : 1.f;
      if (o < O) x = P[(q < OP ? K.omean : K.ostd) + o];
    }
    SPAR[i] = x;
  }

  // A-operand lane offsets into the swizzled W1 | W2 | W2^T (mm32)
  const int w1lane = (fbase / 32) * 32 * OP + ((j >> 4) * (OP / 16) * 64 + h * 16 + (j & 15)) * 4;
  const int w2lane = H * OP + (fbase / 32) * 32 * H + ((j >> 4) * 16 * 64 + h * 16 + (j & 15)) * 4;
  const int w2tlane = w2lane + H * H;
  const float* xn_in = XN + j * LDX + 4 * h;
  const float* act_in = ACT + j * LDA + 4 * h;
  // forward head rows (16x16: A = W3[16 ht + j16][..]); head-backward rows (32x32: heads
  // 16 ht + 8 q2 + 4 h + c of feature fbase + 32 ft + j)
  int hrow_f[NHT], hrow_b[NHT][2][4];
#pragma unroll
  for (int ht = 0; ht < NHT; ++ht) {
    hrow_f[ht] = head_row(K, trunk, 16 * ht + j16, H);
#pragma unroll
    for (int q2 = 0; q2 < 2; ++q2)
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) hrow_b[ht][q2][cc] = head_row(K, trunk, 16 * ht + 8 * q2 + 4 * h + cc, H);
  }
  const int ntiles = (a.M + R - 1) / R;

  // ---- gather (as k_upd) ----
  constexpr bool PREF = (R * OP + 255) / 256 <= 4;
  constexpr int NG = PREF ? (R * OP + 255) / 256 : 1;
  constexpr int NAI = PREF ? (R * PPO_UPD_MAXA + 255) / 256 : 1;
  int pg[NG], pra, pac[NAI];
  float vg[NG], vr1 = 0.f, vr2 = 0.f, vac[NAI];
  auto pref_idx = [&](int itn) {
    const int mb = itn * R;
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      const int idx = tid + 256 * k, row = idx / OP, f = idx - row * OP, m = mb + row;
      pg[k] = (itn < ntiles && idx < R * OP && m < a.M && f < O) ? a.perm[m] : -1;
    }
    pra = (itn < ntiles && tid < R && mb + tid < a.M) ? a.perm[mb + tid] : -1;
#pragma unroll
    for (int k = 0; k < NAI; ++k) {
      const int idx = tid + 256 * k, row = idx / (A > 0 ? A : 1), m = mb + row;
      pac[k] = (trunk == 1 && itn < ntiles && idx < R * A && m < a.M) ? a.perm[m] : -1;
    }
  };
  auto pref_data = [&]() {
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      const int idx = tid + 256 * k, f = idx - (idx / OP) * OP;
      vg[k] = pg[k] >= 0 ? a.obs[(long)pg[k] * O + f] : 0.f;
    }
    if (pra >= 0) {
      if (trunk == 0) { vr1 = a.ret[pra]; vr2 = a.val[pra]; }
      else { vr1 = a.logp[pra]; vr2 = a.adv[pra]; }
    } else {
      vr1 = 0.f; vr2 = 0.f;
    }
#pragma unroll
    for (int k = 0; k < NAI; ++k) {
      const int idx = tid + 256 * k, ai = idx - (idx / (A > 0 ? A : 1)) * A;
      vac[k] = pac[k] >= 0 ? a.actions[(long)pac[k] * A + ai] : 0.f;
    }
  };
  auto commit = [&](int itc) {
    const int mb = itc * R;
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      const int idx = tid + 256 * k, row = idx / OP, f = idx - row * OP, m = mb + row;
      if (idx < R * OP) {
        float v = vg[k];
        if (pg[k] >= 0) v = (v - SOM[f]) / SOS[f];
        XN[row * LDX + f] = v;
        if (trunk == 0 && m < a.M) a.Xn[(size_t)m * OP + f] = v;
      }
    }
    if (tid < R) {
      ROWS[tid * 8 + 1] = vr1;
      ROWS[tid * 8 + 2] = vr2;
    }
#pragma unroll
    for (int k = 0; k < NAI; ++k) {
      const int idx = tid + 256 * k;
      if (trunk == 1 && idx < R * A) ACTN[idx] = vac[k];
    }
  };
  auto perm_of = [&](int r) { return __float_as_int(ROWS[r * 8]); };
  auto gather_sync = [&](int itc) {
    const int mb = itc * R;
    constexpr int NGS = (R * OP + 255) / 256, GC = 4;
#pragma unroll 1
    for (int k0 = 0; k0 < NGS; k0 += GC) {
      int rp[GC];
      float v[GC];
#pragma unroll
      for (int cc = 0; cc < GC; ++cc) {
        const int idx = tid + 256 * (k0 + cc), row = min(idx / OP, R - 1);
        rp[cc] = perm_of(row);
      }
#pragma unroll
      for (int cc = 0; cc < GC; ++cc) {
        const int idx = tid + 256 * (k0 + cc), f = idx - (idx / OP) * OP;
        v[cc] = a.obs[(long)rp[cc] * O + min(f, O - 1)];
      }
#pragma unroll
      for (int cc = 0; cc < GC; ++cc) {
        const int idx = tid + 256 * (k0 + cc), row = idx / OP, f = idx - row * OP, m = mb + row;
        if (k0 + cc < NGS && idx < R * OP) {
          const bool ok = m < a.M && f < O;
          float x = ok ? v[cc] : 0.f;
          if (ok) x = (x - SOM[f]) / SOS[f];
          XN[row * LDX + f] = x;
          if (trunk == 0 && m < a.M) a.Xn[(size_t)m * OP + f] = x;
        }
      }
    }
    {
      const int rrow = perm_of(min(tid, R - 1));
      const float r1 = trunk == 0 ? a.ret[rrow] : a.logp[rrow];
      const float r2 = trunk == 0 ? a.val[rrow] : a.adv[rrow];
      if (tid < R) {
        const bool ok = mb + tid < a.M;
        ROWS[tid * 8 + 1] = ok ? r1 : 0.f;
        ROWS[tid * 8 + 2] = ok ? r2 : 0.f;
      }
    }
    if (trunk == 1) {
      constexpr int NAS = (R * PPO_UPD_MAXA + 255) / 256;
      int ap[NAS];
#pragma unroll
      for (int k = 0; k < NAS; ++k) {
        const int idx = tid + 256 * k, row = min(idx / (A > 0 ? A : 1), R - 1);
        ap[k] = perm_of(row);
      }
      float av[NAS];
#pragma unroll
      for (int k = 0; k < NAS; ++k) {
        const int idx = tid + 256 * k, ai = idx - (idx / (A > 0 ? A : 1)) * A;
        av[k] = a.actions[(long)ap[k] * A + ai];
      }
#pragma unroll
      for (int k = 0; k < NAS; ++k) {
        const int idx = tid + 256 * k, m = mb + idx / (A > 0 ? A : 1);
        if (idx < R * A) ACTN[idx] = m < a.M ? av[k] : 0.f;
      }
    }
  };
  if constexpr (PREF) {
    pref_idx(blockIdx.x);
    pref_data();
  }
  int nperm = 0;
  if constexpr (!PREF) nperm = tid < R ? a.perm[min((int)blockIdx.x * R + tid, a.M - 1)] : 0;

  float lst[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int it = blockIdx.x; it < ntiles; it += gridDim.x) {
    const int m0 = it * R, m = m0 + j;
    PPO_STAMP_START();
    if constexpr (!PREF)
      if (tid < R) ROWS[tid * 8] = __int_as_float(nperm);
    lds_barrier();
    if constexpr (PREF) {
      commit(it);
      pref_idx(it + gridDim.x);
    } else {
      if (tid < R) nperm = a.perm[min((it + (int)gridDim.x) * R + tid, a.M - 1)];
      gather_sync(it);
    }
    // the actor's head-backward A operands (one head tile), requested a forward pass ahead
    f4 hwb[2][2];
    if constexpr (NHT == 1) {
      if (trunk == 1) {
#pragma unroll
        for (int ft = 0; ft < 2; ++ft)
#pragma unroll
          for (int q2 = 0; q2 < 2; ++q2)
#pragma unroll
            for (int cc = 0; cc < 4; ++cc)
              hwb[ft][q2][cc] = hrow_b[0][q2][cc] >= 0 ? bld1(pb, hrow_b[0][q2][cc] + fbase + j, 32 * ft) : 0.0f;
      }
    }
    lds_barrier();
    PPO_STAMP(0);

    // ---------------- layer 1 ----------------
    f16v z[2];
    init_bias32(z, pb, T.b1 + fh);
    mm32<NKB1, KLAST1, OP>(z, wsw, w1lane, xn_in);
    PPO_STAMP(1);
    float mu1, rs1;
    ln32(z, mu1, rs1, RED0, RED1, wave, j, h);
#pragma unroll
    for (int ft = 0; ft < 2; ++ft)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f4 gm = lds_f4(SG1 + fh + 32 * ft + 8 * q), bt = lds_f4(SBE1 + fh + 32 * ft + 8 * q);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float xh = (z[ft][4 * q + r] - mu1) * rs1;
          const float y = __fmaf_rn(gm[r], xh, bt[r]);
          z[ft][4 * q + r] = y > 0.0f ? y : 0.0f;
        }
      }
    store_rows32(a.H1[trunk], H, z, m, a.M, fh);
    lds_store32<LDA>(ACT, z, j, fh);
    lds_barrier();
    PPO_STAMP(2);

    // ---------------- layer 2 ----------------
    f16v x2[2];  // x_hat2
    init_bias32(x2, pb, T.b2 + fh);
    mm32<32, 4, H>(x2, wsw, w2lane, act_in);
    PPO_STAMP(3);
    if constexpr (PREF) pref_data();
    float mu2, rs2;
    ln32(x2, mu2, rs2, RED2, RED3, wave, j, h);
#pragma unroll
    for (int ft = 0; ft < 2; ++ft) x2[ft] = (x2[ft] - mu2) * rs2;
    auto h2_of = [&](int ft, int q) -> f4 {
      const f4 gm = lds_f4(SG2 + fh + 32 * ft + 8 * q), bt = lds_f4(SBE2 + fh + 32 * ft + 8 * q);
      f4 y;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = __fmaf_rn(gm[r], x2[ft][4 * q + r], bt[r]);
        y[r] = v > 0.0f ? v : 0.0f;
      }
      return y;
    };
    PPO_STAMP(4);
    // ---------------- heads ----------------
    lds_barrier();  // every wave is done reading h1 from ACT
    if (trunk == 0) {
      // critic: one real head — per-row dot product over the lane's 32 features, + the other half
      float pv = 0.f;
#pragma unroll
      for (int ft = 0; ft < 2; ++ft)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f4 w = pld4(pb, K.cW3 + fh, 32 * ft + 8 * q);
          const f4 h2 = h2_of(ft, q);
          lds_st4(ACT + j * LDA + fh + 32 * ft + 8 * q, h2);
#pragma unroll
          for (int r = 0; r < 4; ++r) pv = __fmaf_rn(w[r], h2[r], pv);
        }
      pv = xor32_sum(pv);
      if (h == 0) SCR[(wave * NHP) * R + j] = pv;
    } else {
#pragma unroll
      for (int ft = 0; ft < 2; ++ft)
#pragma unroll
        for (int q = 0; q < 4; ++q) lds_st4(ACT + j * LDA + fh + 32 * ft + 8 * q, h2_of(ft, q));
      // 16x16x4 heads over this wave's 64 features, h2 read back from ACT (the wave's own columns:
      // LDS keeps one wave's accesses in order)
      f4 hp[NHT][2];
#pragma unroll
      for (int ht = 0; ht < NHT; ++ht)
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) hp[ht][rt] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ft = 0; ft < 4; ++ft) {
        f4 wv[NHT];
#pragma unroll
        for (int ht = 0; ht < NHT; ++ht)
          wv[ht] = hrow_f[ht] >= 0 ? pld4(pb, hrow_f[ht] + fbase + 4 * g, 16 * ft) : f4{0.f, 0.f, 0.f, 0.f};
        f4 h2v[2];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) h2v[rt] = lds_f4(ACT + (16 * rt + j16) * LDA + fbase + 16 * ft + 4 * g);
#pragma unroll
        for (int cc = 0; cc < 4; ++cc)
#pragma unroll
          for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int ht = 0; ht < NHT; ++ht) hp[ht][rt] = mfma16(wv[ht][cc], h2v[rt][cc], hp[ht][rt]);
      }
#pragma unroll
      for (int ht = 0; ht < NHT; ++ht)
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) SCR[(wave * NHP + 16 * ht + 4 * g + r) * R + 16 * rt + j16] = hp[ht][rt][r];
    }
    lds_barrier();
    PPO_STAMP(5);
    for (int idx = tid; idx < R * nh; idx += 256) {
      const int row = idx / nh, hh = idx - row * nh;
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) s += SCR[(w * NHP + hh) * R + row];
      PRE[row * LDG + hh] = s + SHB[hh];
    }
    lds_barrier();
    PPO_STAMP(6);

    // ---------------- loss and its gradient wrt the head pre-activations (k_upd's) ----------------
    float* ITM = SCR;
    upd_loss<true, R, ITS, LDG>(a, trunk, tid, m0, c, adv_mean, adv_std,
                                [&](int row, int h) { return PRE[row * LDG + h]; }, PRE, GG, ROWS, ACTN, ITM, lst);
    lds_barrier();
    PPO_STAMP(7);
    if (tid < nh) {
      float s = 0.f;
      for (int row = 0; row < R; ++row) s += GG[row * LDG + tid];
      ACC[sl.hb + tid] += s;
    }

    // ---------------- head backward: dh2 = W3^T G^T, dW3 += G^T h2 ----------------
    f16v dh[2];
    zero32(dh);
    if (trunk == 0) {
      const float gr = lds_f(GG + j * LDG);
#pragma unroll
      for (int ft = 0; ft < 2; ++ft)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f4 w = pld4(pb, K.cW3 + fh, 32 * ft + 8 * q);
#pragma unroll
          for (int r = 0; r < 4; ++r) dh[ft][4 * q + r] = w[r] * gr;
        }
      f16v hv[2];  // h2 back from ACT (stored by this lane above)
#pragma unroll
      for (int ft = 0; ft < 2; ++ft)
#pragma unroll
        for (int q = 0; q < 4; ++q) set_quad(hv[ft], q, lds_f4(ACT + j * LDA + fh + 32 * ft + 8 * q));
      col_sums32([&](int ft, int r) { return gr * hv[ft][r]; }, acc + sg.hW, fbase, j, h);
    } else {
#pragma unroll
      for (int ht = 0; ht < NHT; ++ht)
#pragma unroll
        for (int q2 = 0; q2 < 2; ++q2) {
          const f4 gq = lds_f4(GG + j * LDG + 16 * ht + 8 * q2 + 4 * h);
#pragma unroll
          for (int cc = 0; cc < 4; ++cc)
#pragma unroll
            for (int ft = 0; ft < 2; ++ft) {
              float wv;
              if constexpr (NHT == 1) wv = hwb[ft][q2][cc];
              else wv = hrow_b[ht][q2][cc] >= 0 ? bld1(pb, hrow_b[ht][q2][cc] + fbase + j, 32 * ft) : 0.0f;
              dh[ft] = mfma32(wv, gq[cc], dh[ft]);
            }
        }
      // dW3 tiles (heads 16 ht .., features fbase + 16 ft ..), 16x16x4 over the 32 rows from LDS
#pragma unroll
      for (int ht = 0; ht < NHT; ++ht)
#pragma unroll
        for (int ft = 0; ft < 4; ++ft) {
          f4 d3 = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = 16 * rt + 4 * g + r;
              d3 = mfma16(lds_f(GG + row * LDG + 16 * ht + j16), lds_f(ACT + row * LDA + fbase + 16 * ft + j16), d3);
            }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int hh = 16 * ht + 4 * g + r;
            if (hh < nh) hwacc[hh * H + fbase + 16 * ft + j16] += d3[r];
          }
        }
    }
    PPO_STAMP(8);

    // ---------------- layer-2 backward: dz2 ----------------
    {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int ft = 0; ft < 2; ++ft)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f4 gm = lds_f4(SG2 + fh + 32 * ft + 8 * q), bt = lds_f4(SBE2 + fh + 32 * ft + 8 * q);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int k = 4 * q + r;
            const float y = __fmaf_rn(gm[r], x2[ft][k], bt[r]);
            const float dy = y > 0.0f ? dh[ft][k] : 0.0f;
            dh[ft][k] = dy;
            const float dx = dy * gm[r];
            s1 += dx;
            s2 += dx * x2[ft][k];
          }
        }
      rows32x2(s1, s2, RED0, RED1, wave, j, h);
      s1 *= (1.0f / H);
      s2 *= (1.0f / H);
      col_sums32([&](int ft, int r) { return dh[ft][r]; }, acc + sg.be2, fbase, j, h);
      col_sums32([&](int ft, int r) { return dh[ft][r] * x2[ft][r]; }, acc + sg.g2, fbase, j, h);
#pragma unroll
      for (int ft = 0; ft < 2; ++ft)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f4 gm = lds_f4(SG2 + fh + 32 * ft + 8 * q);
          set_quad(x2[ft], q, rs2 * (quad(dh[ft], q) * gm - s1 - quad(x2[ft], q) * s2));
        }
    }
    // x2 = dz2
    col_sums32([&](int ft, int r) { return x2[ft][r]; }, acc + sg.b2, fbase, j, h);
    store_rows32(a.DZ2[trunk], H, x2, m, a.M, fh);
    lds_barrier();  // dW3 readers of h2 are done
    lds_store32<LDA>(ACT, x2, j, fh);
    lds_barrier();
    PPO_STAMP(9);

    // ---------------- dh1 = W2^T dz2 ----------------
    zero32(dh);
    mm32<32, 4, H>(dh, wsw, w2tlane, act_in);
    PPO_STAMP(10);
    // ---------------- recompute layer 1, layer-1 backward ----------------
    init_bias32(z, pb, T.b1 + fh);
    mm32<NKB1, KLAST1, OP>(z, wsw, w1lane, xn_in);
    PPO_STAMP(11);
    {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int ft = 0; ft < 2; ++ft)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f4 gm = lds_f4(SG1 + fh + 32 * ft + 8 * q), bt = lds_f4(SBE1 + fh + 32 * ft + 8 * q);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int k = 4 * q + r;
            const float xh = (z[ft][k] - mu1) * rs1;
            z[ft][k] = xh;
            const float y = __fmaf_rn(gm[r], xh, bt[r]);
            const float dy = y > 0.0f ? dh[ft][k] : 0.0f;
            dh[ft][k] = dy;
            const float dx = dy * gm[r];
            s1 += dx;
            s2 += dx * xh;
          }
        }
      rows32x2(s1, s2, RED2, RED3, wave, j, h);
      s1 *= (1.0f / H);
      s2 *= (1.0f / H);
      col_sums32([&](int ft, int r) { return dh[ft][r]; }, acc + sg.be1, fbase, j, h);
      col_sums32([&](int ft, int r) { return dh[ft][r] * z[ft][r]; }, acc + sg.g1, fbase, j, h);
#pragma unroll
      for (int ft = 0; ft < 2; ++ft)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f4 gm = lds_f4(SG1 + fh + 32 * ft + 8 * q);
          set_quad(z[ft], q, rs1 * (quad(dh[ft], q) * gm - s1 - quad(z[ft], q) * s2));
        }
    }
    // z = dz1
    col_sums32([&](int ft, int r) { return z[ft][r]; }, acc + sg.b1, fbase, j, h);
    store_rows32(a.DZ1[trunk], H, z, m, a.M, fh);
    PPO_STAMP(12);
  }
  // ---------------- workgroup result ----------------
#pragma unroll
  for (int mm = 32; mm >= 1; mm >>= 1)
#pragma unroll
    for (int k = 0; k < 6; ++k) lst[k] += shfl_xor(lst[k], mm);
  lds_barrier();
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 6; ++k) RED[wave * 8 + k] = lst[k];
  }
  lds_barrier();
  if (tid == 0) {
    float t[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) t[k] = (RED[k] + RED[8 + k]) + (RED[16 + k] + RED[24 + k]);
    float* st = ACC + sl.stats;
    st[ST_PG] += t[0]; st[ST_V] += t[1]; st[ST_ENT] += t[2];
    st[ST_OKL] += t[3]; st[ST_KL] += t[4]; st[ST_CF] += t[5];
  }
  lds_barrier();
  for (int i = tid; i < sl.size; i += 256) slab_row[hwg && i >= sg.hW ? i + sg.nh * H : i] = ACC[i];
}

template <int H, int KIND, int NTO, int NHT, int KL1, bool BX>
__global__ __launch_bounds__(256, 2) void k_upd(UpdArgs a) {
  upd16_body<H, KIND, NTO, NHT, KL1, BX>(a);
}
// the split-bf16 form is instantiated for the LayerNorm-Beta agent at H = 256 with one head tile
template <int H, int KIND, int NHT>
constexpr bool upd_bx_ok() { return H == 256 && KIND == PPO_NET_LN_BETA && NHT == 1; }

// MIX = 0: both trunks on 32x32x2 MFMAs; MIX = 1: the critic on 32x32x2, the actor on k_upd's
// 16x16x4 body (the actor's loss and LayerNorm phases are VALU chains that co-issue beside the
// partner's MFMAs: 6.2 VALU per 32x32x2 against 2.2 per 16x16x4)
template <int NTO, int NHT, int KL1, int MIX>
__global__ __launch_bounds__(256, 2) void k_upd32(UpdArgs a) {
  const int trunk = (a.sched & 1) ? 1 - (int)blockIdx.y : (int)blockIdx.y;
  if (MIX && trunk == 1) upd16_body<256, PPO_NET_LN_BETA, NTO, NHT, KL1>(a);
  else upd32_body<NTO, NHT, KL1>(a);
}

// =============================================================================================
// k_vbx: the rollout's critic pass (values[i] = critic(obs[i]) over n stored rows, ac:641-698's
// value per step and ac:761's bootstrap; the agent module ac:150-249) with k_upd's forward
// arithmetic: layer 1 on 16x16x4 fp32 MFMAs, LayerNorm statistics merged across the four feature
// waves (ln_rows), layer 2 as six split-bf16 piece products (mm_bx over the critic's W2 pieces that
// k_adam / k_swizzle keep), the value head as k_upd's per-row VALU dot product and head-partial sum.
// A workgroup of 4 waves walks 32-row tiles (each wave 64 features); the next tile's observations
// are loaded into registers under the current tile's GEMMs. Every row is computed by the same code
// wherever it sits in a tile, so a row's value does not depend on n or on the other rows (the
// per-step host-env rollout and the persistent rollout agree bitwise). Against the fp64 oracle as
// the act kernels are (test_values_bx_vs_oracle).
// =============================================================================================
template <int NTO, int KL1>
__global__ __launch_bounds__(256, 2) void k_vbx(ValuesArgs a) {
  using GE = Geo<256, NTO, 1, true>;
  constexpr int H = 256, FT = GE::FT, RT = GE::RT, WF = GE::WF, R = GE::R, NT = GE::NT, OP = GE::OP;
  constexpr int LDX = GE::LDX, LDB = GE::LDB;
  static_assert(GE::WR == 1 && R == 32, "k_vbx: 4 feature waves, 32-row tiles");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* XN = lds;
  float* ACT = XN + R * LDX;
  float* RED = ACT + R * LDB;
  float* SPAR = RED + 4 * WF * R;  // gamma1 | beta1 | gamma2 | beta2 | w3 | obs mean | obs std
  float *RED0 = RED, *RED1 = RED + WF * R, *RED2 = RED + 2 * WF * R, *RED3 = RED + 3 * WF * R;
  float *SG1 = SPAR, *SBE1 = SPAR + H, *SG2 = SPAR + 2 * H, *SBE2 = SPAR + 3 * H, *SW3 = SPAR + 4 * H;
  float *SOM = SPAR + 5 * H, *SOS = SOM + OP;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  const int wf = wave, fbase = wf * FT * 16;
  const PackedLayout& K = a.K;
  const TrunkDev& T = K.tr[0];
  const float* __restrict__ P = a.P;
  const PBuf pb = make_pbuf(P, K.size);
  const PBuf wsw = make_pbuf(a.WSW, (int)sw_size(H, OP));
  const PBuf wbx = make_pbuf(a.WBX, (int)bx_size(H));
  const int O = K.O;
  const int w1lane = ((fbase >> 4) * NTO * 64 + lane) * 4;
  const int w2blane = ((fbase >> 4) * (NT / 2) * 3 * 64 + lane) * 4;
  const float* xn_in = XN + j * LDX + 4 * g;
  const float* actb_in = ACT + j * LDB + 4 * g;
  const long ntiles = (a.n + R - 1) / R;
  constexpr int NG = (R * OP + 255) / 256;
  float vg[NG];
  auto load_obs = [&](long it) {
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      const int idx = tid + 256 * k, row = idx / OP, f = idx - row * OP;
      const long m = it * R + row;
      const bool ok = it < ntiles && idx < R * OP && m < a.n && f < O;
      const float v = a.obs[(ok ? m : 0) * O + (ok ? f : 0)];
      vg[k] = ok ? v : 0.f;
    }
  };
  load_obs(blockIdx.x);
  for (int i = tid; i < 5 * H + 2 * OP; i += 256) {
    const int v = i / H, f = i - v * H;
    float x;
    if (v < 4) x = P[(v == 0 ? T.g1 : v == 1 ? T.be1 : v == 2 ? T.g2 : T.be2) + f];
    else if (v == 4) x = P[K.cW3 + f];
    else {
      const int q = i - 5 * H, o = q % OP;
      x = q < OP ? 0.f : 1.f;
      if (o < O) x = P[(q < OP ? K.omean : K.ostd) + o];
    }
    SPAR[i] = x;
  }
  const float cb3 = P[K.cb3];
  for (long it = blockIdx.x; it < ntiles; it += gridDim.x) {
    const long m0 = it * R;
    lds_barrier();  // the previous tile's XN / ACT / RED readers are done; SPAR staged (first tile)
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      const int idx = tid + 256 * k, row = idx / OP, f = idx - row * OP;
      if (idx < R * OP) {
        float v = vg[k];
        if (m0 + row < a.n && f < O) v = (v - SOM[f]) / SOS[f];
        XN[row * LDX + f] = v;
      }
    }
    load_obs(it + gridDim.x);
    lds_barrier();
    // layer 1, LayerNorm, ReLU -> split-bf16 pieces in LDS
    f4 z[FT][RT];
    init_bias<FT, RT>(z, pb, T.b1 + fbase + 4 * g);
    mm_fr<FT, RT, NTO, LDX, KL1>(z, wsw, w1lane, xn_in);
    {
      float mu1[RT], rs1[RT];
      ln_rows<FT, RT, WF, R, H>(z, mu1, rs1, RED0, RED1, wf, 0, j, g);
#pragma unroll
      for (int ft = 0; ft < FT; ++ft) {
        const f4 gm = lds_f4(SG1 + fbase + 4 * g + 16 * ft), bt = lds_f4(SBE1 + fbase + 4 * g + 16 * ft);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float xh = (z[ft][rt][r] - mu1[rt]) * rs1[rt];
            const float y = __fmaf_rn(gm[r], xh, bt[r]);
            z[ft][rt][r] = y > 0.0f ? y : 0.0f;
          }
      }
    }
    lds_store_pieces<FT, RT, LDB, H / 2>(ACT, z, 0, fbase, j, g);
    lds_barrier();
    // layer 2 (split-bf16), LayerNorm, ReLU, value head
    f4 x2[FT][RT];
    init_bias<FT, RT>(x2, pb, T.b2 + fbase + 4 * g);
    mm_bx<FT, RT, NT, LDB>(x2, wbx, w2blane, actb_in);
    float mu2[RT], rs2[RT];
    ln_rows<FT, RT, WF, R, H>(x2, mu2, rs2, RED2, RED3, wf, 0, j, g);
    float pv[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) pv[rt] = 0.f;
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      const f4 gm = lds_f4(SG2 + fbase + 4 * g + 16 * ft), bt = lds_f4(SBE2 + fbase + 4 * g + 16 * ft);
      const f4 w = lds_f4(SW3 + fbase + 4 * g + 16 * ft);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float xh = (x2[ft][rt][r] - mu2[rt]) * rs2[rt];
          const float v = __fmaf_rn(gm[r], xh, bt[r]);
          pv[rt] = fmaf(w[r], v > 0.0f ? v : 0.0f, pv[rt]);
        }
    }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      pv[rt] = row_allreduce(pv[rt]);
      if (g == 0) RED0[wf * R + 16 * rt + j] = pv[rt];  // LN1's reads of RED0 precede LN2's exchange
    }
    lds_barrier();
    if (tid < R && m0 + tid < a.n) {
      float sv = 0.f;
#pragma unroll
      for (int w = 0; w < WF; ++w) sv += RED0[w * R + tid];
      a.values[m0 + tid] = sv + cb3;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// host side: geometry, LDS size, dispatch
// ---------------------------------------------------------------------------------------------
// LDS of one workgroup; two must fit one CU (160 KB) so that a critic and an actor workgroup
// share it. Where the actor's accumulators would break that (wide inputs: Ant's O = 105 takes
// 95 KB), its head-weight gradient (nh x H floats) accumulates in its own slab row instead: every
// element has one owning lane, which adds the tile contributions in tile order (bitwise the LDS
// result).
template <int H, int NTO, int NHT, bool BX = false>
static void upd_geo(const PackedLayout& K, int nh_actor, int sg0_size, int sg1_size, UpdGeoOut* g) {
  using GE = Geo<H, NTO, NHT, BX>;
  auto carve = [&](int sg_lds) {
    const int scr = std::max(GE::WF * GE::NHP * GE::R, GE::R * K.A * GE::ITS);
    int off = GE::BX ? GE::oROW + GE::R * 8 : GE::oSCR + scr;
    if (scr > GE::SCR_MAX) off = 1 << 20;  // BX: SCR does not fit its region (refused)
    g->actn_off = off;
    off += GE::R * K.A;
    off = (off + 3) & ~3;
    g->acc_off = off;
    off += GE::WR * sg_lds;
    g->spar_off = off;
    off += GE::NSPAR;
    g->lds_bytes = (size_t)off * sizeof(float);
  };
  g->hw_global = 0;
  carve(std::max(sg0_size, sg1_size));
  if (GE::WR == 1 && 2 * g->lds_bytes > 160 * 1024) {
    const size_t full = g->lds_bytes;
    carve(std::max(sg0_size, sg1_size - nh_actor * H));
    if (2 * g->lds_bytes <= 160 * 1024) g->hw_global = 1;
    else carve(std::max(sg0_size, sg1_size)), (void)full;  // one workgroup per CU either way
  }
  g->rows = GE::R;
}

template <typename F>
static int dispatch_upd(const PackedLayout& K, int nh, F&& f) {
  const int nto = K.OP / 16, nht = (nh + 15) / 16;
  const int kl = (K.O == 16 * (nto - 1) + 1) ? 1 : 4;  // layer 1: one real column in the last k-block
#define PPO_UPD_CASE(H_, KIND_, NTO_, NHT_, KL_)                                                             \
  if (K.H == H_ && K.kind == KIND_ && nto == NTO_ && nht == NHT_ && kl == KL_)                               \
    return f(std::integral_constant<int, H_>{}, std::integral_constant<int, KIND_>{},                        \
             std::integral_constant<int, NTO_>{}, std::integral_constant<int, NHT_>{},                       \
             std::integral_constant<int, KL_>{});
  PPO_UPD_CASE(256, PPO_NET_LN_BETA, 1, 1, 4) PPO_UPD_CASE(256, PPO_NET_LN_BETA, 2, 1, 4)
  PPO_UPD_CASE(256, PPO_NET_LN_BETA, 2, 1, 1) PPO_UPD_CASE(256, PPO_NET_LN_BETA, 7, 1, 4)
  PPO_UPD_CASE(256, PPO_NET_LN_BETA, 24, 3, 4) PPO_UPD_CASE(256, PPO_NET_LN_BETA, 2, 3, 4)
  PPO_UPD_CASE(256, PPO_NET_LN_BETA, 2, 3, 1) PPO_UPD_CASE(256, PPO_NET_TANH_NORMAL, 2, 1, 4)
  PPO_UPD_CASE(256, PPO_NET_TANH_NORMAL, 2, 1, 1)
#undef PPO_UPD_CASE
  return -1;
}

int upd_supported(const PackedLayout& K, int nh_actor, int sg0_size, int sg1_size, UpdGeoOut* g, int bx) {
  // both trunks run in one launch: the geometry must cover the actor's head count (critic: 1)
  return dispatch_upd(K, nh_actor, [&](auto H_, auto KIND_, auto NTO_, auto NHT_, auto KL_) {
    constexpr int H = decltype(H_)::value, KIND = decltype(KIND_)::value, NTO = decltype(NTO_)::value,
                  NHT = decltype(NHT_)::value, KL = decltype(KL_)::value;
    const void* k = nullptr;
    if (bx) {
      if constexpr (upd_bx_ok<H, KIND, NHT>()) {
        upd_geo<H, NTO, NHT, true>(K, nh_actor, sg0_size, sg1_size, g);
        if (2 * g->lds_bytes > 160 * 1024) return -1;  // one workgroup per CU: not this form
        k = (const void*)k_upd<H, KIND, NTO, NHT, KL, true>;
      } else {
        return -1;
      }
    } else {
      upd_geo<H, NTO, NHT>(K, nh_actor, sg0_size, sg1_size, g);
      k = (const void*)k_upd<H, KIND, NTO, NHT, KL, false>;
    }
    return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)g->lds_bytes) == hipSuccess ? 0 : -2;
  });
}

// k_upd32: the LayerNorm-Beta agent at H = 256 (the instantiations k_upd has for it)
template <typename F>
static int dispatch_upd32(const PackedLayout& K, int nh, F&& f) {
  const int nto = K.OP / 16, nht = (nh + 15) / 16;
  const int kl = (K.O == 16 * (nto - 1) + 1) ? 1 : 4;
  if (K.H != 256 || K.kind != PPO_NET_LN_BETA) return -1;
#define PPO_UPD32_CASE(NTO_, NHT_, KL_)                                                              \
  if (nto == NTO_ && nht == NHT_ && kl == KL_)                                                       \
    return f(std::integral_constant<int, NTO_>{}, std::integral_constant<int, NHT_>{}, std::integral_constant<int, KL_>{});
  PPO_UPD32_CASE(1, 1, 4) PPO_UPD32_CASE(2, 1, 4) PPO_UPD32_CASE(2, 1, 1) PPO_UPD32_CASE(7, 1, 4)
  PPO_UPD32_CASE(24, 3, 4) PPO_UPD32_CASE(2, 3, 4) PPO_UPD32_CASE(2, 3, 1)
#undef PPO_UPD32_CASE
  return -1;
}

int upd32_supported(const PackedLayout& K, int nh_actor, int sg0_size, int sg1_size, UpdGeoOut* g, int mix) {
  return dispatch_upd32(K, nh_actor, [&](auto NTO_, auto NHT_, auto KL_) {
    upd_geo<256, decltype(NTO_)::value, decltype(NHT_)::value>(K, nh_actor, sg0_size, sg1_size, g);
    constexpr int N = decltype(NTO_)::value, T = decltype(NHT_)::value, L = decltype(KL_)::value;
    const void* k = mix ? (const void*)k_upd32<N, T, L, 1> : (const void*)k_upd32<N, T, L, 0>;
    return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)g->lds_bytes) == hipSuccess ? 0 : -2;
  });
}

int launch_upd32(const UpdArgs& a, int nh_actor, int nblocks, size_t lds_bytes, hipStream_t s, int mix) {
  UpdArgs b = a;
#ifndef PPO_DIAG
  b.trunk_mask = 3;
#endif
  return dispatch_upd32(a.K, nh_actor, [&](auto NTO_, auto NHT_, auto KL_) {
    constexpr int N = decltype(NTO_)::value, T = decltype(NHT_)::value, L = decltype(KL_)::value;
    if (mix) hipLaunchKernelGGL((k_upd32<N, T, L, 1>), dim3(nblocks, 2), dim3(256), lds_bytes, s, b);
    else hipLaunchKernelGGL((k_upd32<N, T, L, 0>), dim3(nblocks, 2), dim3(256), lds_bytes, s, b);
    return 0;
  });
}

int launch_upd(const UpdArgs& a, int nh_actor, int nblocks, size_t lds_bytes, hipStream_t s) {
  // trunk_mask / sched come from the context (ppo_create); a trunk mask other than 3 exists only in
  // the diagnostic build (PPO_DIAG), where it times the two trunks apart
  UpdArgs b = a;
#ifndef PPO_DIAG
  b.trunk_mask = 3;
#endif
  const dim3 grid(nblocks, 2);
  return dispatch_upd(a.K, nh_actor, [&](auto H_, auto KIND_, auto NTO_, auto NHT_, auto KL_) {
    constexpr int H = decltype(H_)::value, KIND = decltype(KIND_)::value, NTO = decltype(NTO_)::value,
                  NHT = decltype(NHT_)::value, KL = decltype(KL_)::value;
    if (a.bx) {
      if constexpr (upd_bx_ok<H, KIND, NHT>()) {
        hipLaunchKernelGGL((k_upd<H, KIND, NTO, NHT, KL, true>), grid, dim3(256), lds_bytes, s, b);
        return 0;
      }
      return -1;
    }
    hipLaunchKernelGGL((k_upd<H, KIND, NTO, NHT, KL, false>), grid, dim3(256), lds_bytes, s, b);
    return 0;
  });
}

// k_vbx for the LayerNorm-Beta agent at H = 256 (the critic pass of the persistent and per-step
// rollouts when the bx pieces exist); -1: not covered here (the caller runs k_values)
int launch_vbx(const ValuesArgs& a, hipStream_t s) {
  if (!a.WBX || a.K.H != 256 || a.K.kind != PPO_NET_LN_BETA || a.n <= 0) return -1;
  const int nto = a.K.OP / 16, kl = (a.K.O == 16 * (nto - 1) + 1) ? 1 : 4;
  auto go = [&](auto kern, int nto_) {
    using GE = Geo<256, 1, 1, true>;
    const int OP = 16 * nto_, LDX = OP + 4;
    const size_t lds = (size_t)(GE::R * LDX + GE::R * GE::LDB + 4 * GE::WF * GE::R + 5 * 256 + 2 * OP) * sizeof(float);
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return -2;
    int dev = 0, ncu = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const long ntiles = (a.n + GE::R - 1) / GE::R;
    const long grid = ntiles < 2L * ncu ? ntiles : 2L * ncu;  // two resident workgroups per CU
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(256), lds, s, a);
    return 0;
  };
  if (nto == 1) return go(k_vbx<1, 4>, 1);
  if (nto == 2 && kl == 1) return go(k_vbx<2, 1>, 2);
  if (nto == 2) return go(k_vbx<2, 4>, 2);
  if (nto == 7) return go(k_vbx<7, 4>, 7);
  return -1;
}

#ifdef PPO_STAMPS
extern "C" int ppo_diag_read_stamps(unsigned long long* host, long n) {
  const long cap = (long)(sizeof(g_upd_stamps) / sizeof(g_upd_stamps[0]));
  if (n > cap) n = cap;
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_upd_stamps), n * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? (int)n : -2;
}
#endif
