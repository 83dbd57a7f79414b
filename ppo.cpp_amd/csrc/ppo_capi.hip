// ppo_capi.hip — C-ABI of libppo_hip.so (include/ppo_hip.h, include/ppo_synth_env.h).
//
// Host runtime around the gfx950 kernels: device memory for the agent (packed params, grads,
// Adam moments), the [T, E, *] rollout storage, minibatch scratch, the per-minibatch launch
// sequence of the PPO update, and the RCCL communicator that replaces torchfort::Comm
// (reference src/distributed.cpp). Everything runs asynchronously on the context stream; the only
// host synchronisation in an update is the optional stats read-back at its end.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>
#include <link.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ppo_hip.h"
#include "../../include/ppo_synth_env.h"
#include "../../include/ppo_env_wrappers.h"
#include "ppo_kernels.hpp"

// ------------------------------------------------------------------------------------------
// errors
// ------------------------------------------------------------------------------------------
static thread_local std::string g_err;
static int fail(const std::string& msg, int code = -1) {
  g_err = msg;
  return code;
}
#define HIP_TRY(expr)                                                                           \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess) return fail(std::string(#expr) + ": " + hipGetErrorString(e_), -2);   \
  } while (0)
#define NCCL_TRY(expr)                                                                          \
  do {                                                                                          \
    ncclResult_t r_ = (expr);                                                                   \
    if (r_ != ncclSuccess) return fail(std::string(#expr) + ": " + ncclGetErrorString(r_), -3); \
  } while (0)

extern "C" const char* ppo_last_error(void) { return g_err.c_str(); }

// ------------------------------------------------------------------------------------------
// one HIP runtime per process
// ------------------------------------------------------------------------------------------
// libppo_hip.so links /opt/rocm's libamdhip64.so.7. A PyTorch-ROCm wheel bundles its own copy and
// its libraries ask for it as "libamdhip64.so"; if libppo_hip.so is loaded first, `import torch`
// then maps a second HIP runtime, and the two tear each other down at exit (free(): invalid
// pointer, exit 134). Every runtime-initialising entry point checks for that and fails with a
// clear message; the first failed check also installs an exit guard that ends the process with
// status 70 before either runtime's teardown runs. The guard is permanent for the process (a host
// that handles the -4 still exits 70: its teardown would crash otherwise); it flushes every stdio
// stream first.
static int hip_runtime_paths(std::vector<std::string>* out) {
  out->clear();
  dl_iterate_phdr(
      [](struct dl_phdr_info* info, size_t, void* data) -> int {
        auto* v = static_cast<std::vector<std::string>*>(data);
        const char* name = info->dlpi_name;
        if (!name || !strstr(name, "libamdhip64.so")) return 0;
        char buf[4096];
        std::string path = realpath(name, buf) ? std::string(buf) : std::string(name);
        if (std::find(v->begin(), v->end(), path) == v->end()) v->push_back(path);
        return 0;
      },
      out);
  return (int)out->size();
}

static std::string g_runtime_msg;
static void runtime_exit_guard() {
  fprintf(stderr, "libppo_hip: %s -- exiting (70) before the HIP runtimes' teardown\n", g_runtime_msg.c_str());
  fflush(nullptr);  // every stdio stream (stdout, log files) before _exit skips the C library's flush
  _exit(70);
}

extern "C" int ppo_runtime_check(void) {
  std::vector<std::string> paths;
  if (hip_runtime_paths(&paths) <= 1) return 0;
  std::string msg = "two HIP runtimes are mapped in this process (";
  for (size_t i = 0; i < paths.size(); ++i) msg += (i ? ", " : "") + paths[i];
  msg += "): load libppo_hip.so after `import torch` (ppo_amd does), or do not import torch";
  static std::once_flag guard;
  std::call_once(guard, [&] {
    g_runtime_msg = msg;
    atexit(runtime_exit_guard);
  });
  return fail(msg, -4);
}

// ------------------------------------------------------------------------------------------
// per-env-id observation normalisation of the AC agent (ac:480-534)
// ------------------------------------------------------------------------------------------
#include "ppo_obs_norm.inc"

extern "C" int ppo_obs_norm(const char* env_id, const float** mean, const float** stdv, int* n) {
  if (!env_id || !mean || !stdv || !n) return fail("ppo_obs_norm: null argument");
  *mean = *stdv = nullptr;
  *n = 0;
  if (!strcmp(env_id, "HalfCheetah-v5")) return 0;  // zeros / ones (ac:510-511): identity
  for (const ObsNormEntry& e : k_obs_norm)
    if (!strcmp(env_id, e.env_id)) {
      *mean = e.mean;
      *stdv = e.std;
      *n = e.n;
      return 0;
    }
  return fail(std::string("ppo_obs_norm: env_id ") + env_id + " is not implemented.", -1);
}
int ppo_fail(const std::string& msg, int code) { return fail(msg, code); }
extern "C" const char* ppo_version(void) { return "ppo_hip 0.1 (gfx950)"; }

// ------------------------------------------------------------------------------------------
// profiling (HIP events around the context's launches)
// ------------------------------------------------------------------------------------------
enum {
  PK_ACT = 0, PK_FWDBWD, PK_DW2, PK_DW1, PK_COLSUM, PK_GRADNORM, PK_ADAM, PK_GAE, PK_PERM, PK_ADV, PK_ALLREDUCE,
  PK_SYNTH, PK_ROLLOUT, PK_VALUES, PK_L1G, PK_COUNT
};
static const char* kProfNames[PK_COUNT] = {"act", "fwdbwd", "dw", "dw_l1", "colsum", "gradnorm",
                                           "adam", "gae", "perm", "adv_stats", "allreduce", "synth_env",
                                           "rollout", "values", "l1g"};

struct ProfEvent {
  int id;
  hipEvent_t a, b;
};

struct ppo_ctx {
  ppo_hip_config cfg;
  int device = 0;
  hipStream_t stream = nullptr;
  ppo_layout L;
  PackedLayout K;
  SmallGradLayout sg[2];
  long B = 0;
  int M = 0, nmb = 0;
  float *P = nullptr, *G = nullptr, *Am = nullptr, *Av = nullptr, *W2T[2] = {nullptr, nullptr};
  float* WSW[2] = {nullptr, nullptr};  // swizzled W1 | W2 | W2^T per trunk (sw_index)
  float* buf[PPO_BUF_COUNT] = {};
  float* next_value = nullptr;
  int32_t* perms = nullptr;
  float *advstats = nullptr, *advsq = nullptr;
  double* advpart = nullptr;
  float *Xn = nullptr, *H1[2] = {}, *DZ1[2] = {}, *DZ2[2] = {};
  float* slab[2] = {};
  int tiles_per_block = 1, nblk = 1;
  bool use_upd = false;  // feature-split k_upd (ppo_update.hip) instead of k_fwdbwd
  bool use_upd32 = false;  // k_upd32 (32x32x2 MFMAs) instead of k_upd (create option upd_mfma)
  int upd_bx = 0;          // 1: k_upd's 256-wide GEMMs as split-bf16 piece products (upd_mfma=bx6)
  int gae_scan = -1;       // 1: GAE as k_gae_scan (create option gae=scan); 0: the bit-exact serial k_gae; -1 auto
  // 1: the rollout's critic pass is k_vbx (layer 2 as split-bf16 products; create option values_mfma),
  // run once over the stored rows: the per-step act kernels skip the critic and leave it pending
  int values_bx = 0;
  std::atomic<int> values_pending{0};  // steps [0, n) of the rollout storage whose values are not computed yet
  // the minibatch's k_upd + dW in msplit launch pairs of Mq rows each (create option upd_split): the
  // hand-off rows (H1 / DZ1 / DZ2 / Xn) of one pair are ~M / msplit x 6 KB, small enough to stay in the
  // 256 MB Infinity Cache between k_upd's stores and k_dwf's reads
  int msplit = 1, Mq = 0;
  // 1: k_upd writes no H1 rows, only each row's layer-1 LayerNorm (mean, 1 / std) into LNS[trunk]
  // ([M][2]), and k_dwf_bx recomputes H1 bitwise (create option h1_handoff)
  int h1_recomp = 0;
  float* LNS[2] = {nullptr, nullptr};
  int upd32_mix = 0;       // k_upd32 with the actor trunk on k_upd's body (upd_mfma=mix)
  bool use_upd2 = false;  // two-trunk k_upd2 (ppo_update_narrow.hip, H = 64 tanh agent)
  int rollout_kernel = 0;   // AC persistent rollout: 0 auto, 1 k_rollout (MFMA), 2 k_rollout_v (VALU)
  int upd2_split = 0;       // k_l1g (layer 1 as a gathered GEMM into Z1) + k_upd2's split form at 2 / 3 per CU
  float* Z1 = nullptr;      // [Mr][128] layer-1 pre-activations of the minibatch (split form)
  UpdGeoOut upd = {};
  int upd_nblk = 0;
  size_t lds_bytes = 0;
  int wlds_off = 0;
  float* dwslab[4] = {};
  int nchunks = 1, rows_per_chunk = 64, dw_slices = 1;
  float* normout = nullptr;
  float* gnpart = nullptr;
  float* cs_sq = nullptr;               // gradnorm=fold: k_colsum's per-tile sums of squares
  unsigned* cs_cnt = nullptr;           // ... and its per-segment arrival counters (reset by each last arriver)
  int gn_fold = 0;                      // create option gradnorm: 1 fold the norm slices into k_colsum
  float* mbstats = nullptr;  // [EP*MB][8]
  float* snap = nullptr;     // ppo_snapshot_state: P | Am | Av (packed)
  hipEvent_t snap_ev = nullptr;
  hipStream_t snap_stream = nullptr;
  long snap_step = 0;
  long adam_step = 0;
  long iteration = 0;
  ncclComm_t comm = nullptr;
  ppo_host_allreduce_fn host_ar = nullptr;  // host transport (ppo_comm_init_host)
  void* host_user = nullptr;
  std::vector<float> host_stage;
  int world = 1, rank = 0;  // data-parallel group of the attached communicator (1 / cfg.rank without one)
  int act_kernel = 0;  // 0: the fastest act kernel for the shape; 2 / 4: force k_act2 / k_act4 (PPO_ACT_KERNEL, A/B)
  int upd_trunk_mask = 3, upd_sched = 1;   // k_upd launch options (PPO_UPD_TRUNK: PPO_DIAG builds only)
  int dw_fused = 1;
  int dw_dma = 1;                       // create option dw_dma: k_dwf stages by LDS DMA (k_dwf_dma)
  int dw_bx = 0;                        // create option dw_mfma: 0 fp32 MFMA, 8 / 9 exact bf16 piece products (k_dwf_bx)
  int rollout_mode = PPO_ROLLOUT_AUTO;  // ppo_set_rollout_mode
  int gradstep = 0;                     // create option gradstep=fused|split (default split)
  unsigned* gs_bar = nullptr;           // k_gradstep's grid barrier counter
  unsigned gs_count = 0;                // its arrivals so far
  int update_graph = 0;                 // create option update_graph: replay the minibatch loop as a hipGraph
  bool update_graph_auto = false;       // ... chosen by update_graph=auto (then off once snapshots are taken)
  hipGraphExec_t upd_exec = nullptr;    // the captured loop (all epochs x minibatches)
  const int32_t* upd_exec_perms = nullptr;
  long upd_calls = 0;
  float* sched = nullptr;               // per-minibatch (step size, sqrt(bc2)), AdamArgs::sched
  float* sched_host[2] = {};            // pinned staging of that table, alternating per replay
  hipEvent_t sched_ev[2] = {};          // the H2D copy out of sched_host[i] has completed
  int sched_flip = 0;
  float* beta_store = nullptr;          // persistent AC rollout: (alpha, beta, sample) per (t, env, action)
  // profiling
  unsigned prof_mask = 0;
  std::mutex prof_mu;
  std::vector<ProfEvent> pending;
  std::vector<hipEvent_t> free_events;
  double prof_ms[PK_COUNT] = {};
  long prof_cnt[PK_COUNT] = {};
};

static hipEvent_t prof_event(ppo_t* c) {
  if (!c->free_events.empty()) {
    hipEvent_t e = c->free_events.back();
    c->free_events.pop_back();
    return e;
  }
  hipEvent_t e;
  (void)hipEventCreate(&e);
  return e;
}
struct ProfScope {
  ppo_t* c;
  int id;
  hipStream_t s;
  hipEvent_t a = nullptr, b = nullptr;
  ProfScope(ppo_t* c_, int id_, hipStream_t s_) : c(c_), id(id_), s(s_) {
    if (c->prof_mask & (1u << id)) {
      std::lock_guard<std::mutex> lk(c->prof_mu);
      a = prof_event(c);
      b = prof_event(c);
      (void)hipEventRecord(a, s);
    }
  }
  ~ProfScope() {
    if (a) {
      (void)hipEventRecord(b, s);
      std::lock_guard<std::mutex> lk(c->prof_mu);
      c->pending.push_back({id, a, b});
    }
  }
};
static void prof_drain(ppo_t* c) {
  std::lock_guard<std::mutex> lk(c->prof_mu);
  for (auto& p : c->pending) {
    (void)hipEventSynchronize(p.b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, p.a, p.b);
    c->prof_ms[p.id] += ms;
    c->prof_cnt[p.id] += 1;
    c->free_events.push_back(p.a);
    c->free_events.push_back(p.b);
  }
  c->pending.clear();
}

static hipStream_t S(ppo_t* c, void* s) { return s ? (hipStream_t)s : c->stream; }
static void comm_detach(ppo_t* c);

// ------------------------------------------------------------------------------------------
// create / destroy
// ------------------------------------------------------------------------------------------
template <typename T>
static int dmalloc(T** p, size_t n) {
  if (n == 0) n = 1;
  hipError_t e = hipMalloc((void**)p, n * sizeof(T));
  if (e != hipSuccess) return fail(std::string("hipMalloc: ") + hipGetErrorString(e), -2);
  (void)hipMemset(*p, 0, n * sizeof(T));
  return 0;
}

// Kernel selection options of ppo_create_ex: "key=value" pairs separated by ',' (include/ppo_hip.h).
struct CreateOptions {
  int upd_kernel = 0;   // 0 auto, 1 the wave-per-16-rows k_fwdbwd
  int act_kernel = 0;   // 0 auto, 2 / 4 force k_act2 / k_act4
  int dw_fused = 1;
  int rollout = PPO_ROLLOUT_AUTO;
  // 1: grad norm + Adam in one cooperative launch (k_gradstep); 0 (default): two launches. A
  // cooperative launch costs ~30 us on this stack (measured: cfg1 +8.5 ms per iteration), more
  // than the launch it saves.
  int gradstep = 0;
  int gradnorm = -1;   // gradnorm=auto|slices|fold: clip_grad_norm_'s sums of squares by k_gradnorm or inside k_colsum
  int dw_rows = 0;     // dW split-K rows per chunk (multiple of 16; 0: auto, ~128 chunks per trunk)
  int dw_slices = 0;   // k_dwf output slices per chunk (1 / 2; 0: auto, dw_slices())
  int dw_dma = 1;      // 1 (default): k_dwf_dma (LDS-DMA staging, three stage buffers); 0: k_dwf
  int dw_bx = -1;      // dw_mfma: -1 auto, 0 f32 (fp32 MFMA), 9 / 8 / 6 bf16x9 / x8 / x6 (k_dwf_bx: exact bf16 splits)
  int gae_scan = -1;   // gae=auto (scan from kGaeScanMinT steps) | serial (bit-exact with the reference's loop) | scan
  int values_mfma = -1;  // values_mfma=auto (bx6 where k_upd's bx6 pieces exist) | f32 | bx6
  int upd_split = 0;     // upd_split=auto|1|2|4|8: minibatch rows per k_upd + dW launch pair (M / n)
  int h1_handoff = -1;   // h1_handoff=auto|store|recompute: H1 rows from k_upd, or recomputed by k_dwf_bx
  // 1: ppo_update replays its minibatch launches as one captured hipGraph; 0 (default): eager.
  // Snapshots work with it on (ppo_read_snapshot waits for the snapshot's event on the host).
  int update_graph = -1;  // -1 auto (kUpdGraphAutoRows), 0 eager, 1 graph
  int rollout_kernel = 0;  // 0 auto, 1 mfma (k_rollout), 2 valu (k_rollout_v)
  int upd2_split = -1;  // -1 auto (= kUpd2SplitAuto: the single k_upd2), 0 one k_upd2, 2 / 3 split at 2 / 3 workgroups per CU
  int upd_mfma = 0;     // 0 auto (bx6 where it applies, else 16), 16: k_upd (16x16x4 fp32 MFMAs),
                        // 32: k_upd32 (32x32x2; LayerNorm-Beta agent, H = 256),
                        // 1: k_upd32's mixed form (critic 32x32x2, actor 16x16x4),
                        // 6: bx6, k_upd with its 256-wide GEMMs as split-bf16 piece products (k_upd<.., BX>)
};
// auto = the single k_upd2: the split form measured slower on cfg2 (round 4, profiles/r04/cfg2_split/:
// 101.3 vs 92.9 ms per iteration; k_l1g 66 us = 0.61 of peak per launch, the tail 94 us at 3 per CU)
static constexpr int kUpd2SplitAuto = 0;
// dw_mfma=auto: the fused dW as six exact bf16 piece products (k_dwf_bx, bf16x6: k_upd's six; the
// dropped mid.lo + lo.mid + lo.lo are < 2^-21 of each product). With k_upd on its split-bf16 form the
// metric iteration runs 17.32 (fp32 MFMA dW) -> 16.65 (bf16x9) ms, and bf16x9 17.02 -> bf16x6 16.55 ms
// on another box (profiles/r05/bx6/); against the fp64 oracle every dW tensor stays within 1.5x of the
// fp32 MFMA's error (test_split_bf16_dw_is_as_accurate_as_fp32_mfma)
static constexpr int kDwBxAuto = 6;
// upd_mfma=auto: k_upd's split-bf16 form (bx6) wherever it is instantiated (LayerNorm-Beta agent,
// H = 256, one head tile): as exact as the fp32 MFMA form against the oracle
// (test_upd_bx6_is_as_accurate_as_fp32_mfma), k_upd 0.775 -> 0.606 ms per launch at the metric config
static constexpr int kUpdBxAuto = 1;
// upd_mfma=auto for the 64-wide agent: k_upd2's layer 1 as split-bf16 piece products where instantiated
static constexpr int kUpd2BxAuto = 1;
// gae=auto: k_gae_scan from this many steps on (cfg1 / cfg2's T = 2 048: 16 segments per env; within
// 1e-5 of the serial recurrence and of the golden vectors, test_gae_scan_vs_golden), the bit-exact serial
// k_gae below it (the metric's T = 128: 13 us, < 0.1 % of the iteration). cfg2: 0.186 -> 0.107 ms
// (profiles/r05/gae_scan/)
static constexpr int kGaeScanMinT = 512;
// upd_split=auto: launch pairs per minibatch (see ppo_ctx::msplit); 1 until measured
static int kUpdSplitAuto(int M) { (void)M; return 1; }
// h1_handoff=auto: H1 stored. Recomputing it in k_dwf_bx (bitwise the same, test_h1_recompute_is_bitwise_the_
// stored_h1) took k_upd 0.605 -> 0.573 ms per launch but k_dwf_bx 217 -> 255 us (its extra fp32 MFMAs and a
// barrier per stage): 15.97 -> 16.04 ms per metric iteration (profiles/r06/h1_recompute/)
static constexpr bool kH1RecomputeAuto = false;
static constexpr int kUpdGraphAutoRows = 4096;  // update_graph=auto: minibatches of at most this many rows
// gradnorm=auto: k_gradnorm. The fold measured slower everywhere (E = 512 shard 3.44 -> 3.78 ms, cfg2 87.5 -> 88.7,
// cfg1 17.4 -> 17.9: each tile's write-through store + counter round trip costs more than the launch it
// saves; profiles/r06/gradnorm_fold/)
static constexpr int kGradnormFoldAuto = 0;
static int parse_create_options(const char* opts, CreateOptions* o) {
  if (!opts) return 0;
  std::string s(opts);
  size_t pos = 0;
  while (pos < s.size()) {
    size_t end = s.find(',', pos);
    if (end == std::string::npos) end = s.size();
    const std::string kv = s.substr(pos, end - pos);
    pos = end + 1;
    if (kv.empty()) continue;
    const size_t eq = kv.find('=');
    if (eq == std::string::npos) return fail("ppo_create_ex: option without '=': " + kv);
    const std::string k = kv.substr(0, eq), v = kv.substr(eq + 1);
    if (k == "upd_kernel" && (v == "auto" || v == "fwdbwd")) o->upd_kernel = v == "fwdbwd";
    else if (k == "act_kernel" && (v == "auto" || v == "2" || v == "4")) o->act_kernel = v == "auto" ? 0 : v[0] - '0';
    else if (k == "dw_fused" && (v == "0" || v == "1")) o->dw_fused = v[0] - '0';
    else if (k == "rollout" && (v == "auto" || v == "per_step"))
      o->rollout = v == "auto" ? PPO_ROLLOUT_AUTO : PPO_ROLLOUT_PER_STEP;
    else if (k == "gradstep" && (v == "fused" || v == "split")) o->gradstep = v == "fused";
    else if (k == "gradnorm" && (v == "auto" || v == "slices" || v == "fold")) o->gradnorm = v == "auto" ? -1 : v == "fold";
    else if (k == "dw_rows" && !v.empty() && v.size() <= 5 && v.find_first_not_of("0123456789") == std::string::npos &&
             atoi(v.c_str()) % 16 == 0 && atoi(v.c_str()) >= 16 && atoi(v.c_str()) <= 65536)
      o->dw_rows = atoi(v.c_str());  // at most 5 digits: no overflow, no exception across the C-ABI
    else if (k == "dw_slices" && (v == "1" || v == "2")) o->dw_slices = v[0] - '0';
    else if (k == "dw_dma" && (v == "0" || v == "1")) o->dw_dma = v[0] - '0';
    else if (k == "gae" && (v == "auto" || v == "serial" || v == "scan")) o->gae_scan = v == "auto" ? -1 : v == "scan";
    else if (k == "h1_handoff" && (v == "auto" || v == "store" || v == "recompute"))
      o->h1_handoff = v == "auto" ? -1 : v == "recompute";
    else if (k == "upd_split" && (v == "auto" || v == "1" || v == "2" || v == "4" || v == "8"))
      o->upd_split = v == "auto" ? 0 : v[0] - '0';
    else if (k == "values_mfma" && (v == "auto" || v == "f32" || v == "bx6"))
      o->values_mfma = v == "auto" ? -1 : v == "f32" ? 0 : 6;
    else if (k == "dw_mfma" && (v == "auto" || v == "f32" || v == "bf16x9" || v == "bf16x8" || v == "bf16x6"))
      o->dw_bx = v == "auto" ? -1 : v == "f32" ? 0 : v == "bf16x9" ? 9 : v == "bf16x8" ? 8 : 6;
    else if (k == "update_graph" && (v == "auto" || v == "0" || v == "1")) o->update_graph = v == "auto" ? -1 : v[0] - '0';
    else if (k == "rollout_kernel" && (v == "auto" || v == "mfma" || v == "valu"))
      o->rollout_kernel = v == "auto" ? 0 : v == "mfma" ? 1 : 2;
    else if (k == "upd2_split" && (v == "auto" || v == "0" || v == "2" || v == "3")) o->upd2_split = v == "auto" ? -1 : v[0] - '0';
    else if (k == "upd_mfma" && (v == "auto" || v == "16" || v == "32" || v == "mix" || v == "bx6"))
      o->upd_mfma = v == "auto" ? 0 : v == "mix" ? 1 : v == "bx6" ? 6 : atoi(v.c_str());
    else return fail("ppo_create_ex: unknown option or value: " + kv);
  }
  return 0;
}

extern "C" int ppo_create(const ppo_hip_config* cfg, int device, ppo_t** out) {
  return ppo_create_ex(cfg, device, nullptr, out);
}

extern "C" int ppo_create_ex(const ppo_hip_config* cfg, int device, const char* options, ppo_t** out) {
  if (!cfg || !out) return fail("ppo_create: null argument");
  CreateOptions opt;
  if (parse_create_options(options, &opt)) return -1;
  if (int rc = ppo_runtime_check()) return rc;
  ppo_layout L;
  if (ppo_layout_init(&L, cfg->net_kind, cfg->obs_dim, cfg->act_dim, cfg->hidden) != 0)
    return fail("ppo_create: bad net kind / dims");
  if (cfg->hidden != 64 && cfg->hidden != 256) return fail("ppo_create: hidden must be 64 or 256");
  if (cfg->act_dim > 20) return fail("ppo_create: act_dim > 20 not supported");
  if (cfg->num_envs <= 0 || cfg->num_steps <= 0 || cfg->num_minibatches <= 0 || cfg->update_epochs <= 0)
    return fail("ppo_create: sizes must be positive");
  const long B = (long)cfg->num_envs * cfg->num_steps;
  if (B % cfg->num_minibatches) return fail("ppo_create: num_steps*num_envs must divide by num_minibatches");
  if (B >= (1L << 31)) return fail("ppo_create: batch too large");
  {
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev)  // the reference's gpu_ids.at(local_rank) throws here (ac:447)
      return fail("ppo_create: device " + std::to_string(device) + " requested but " + std::to_string(ndev) +
                  " HIP device(s) are visible");
  }
  HIP_TRY(hipSetDevice(device));
  ppo_t* c = new ppo_t();
  c->cfg = *cfg;
  c->device = device;
  c->L = L;
  c->K = make_packed(L);
  {
    int nto = c->K.OP / 16;
    bool ok = false;
    const int H = cfg->hidden, kind = cfg->net_kind;
    const int sup[][3] = {{256, 1, 1}, {256, 1, 2}, {256, 1, 7}, {256, 1, 24}, {64, 0, 1}, {64, 0, 2},
                          {64, 0, 7}, {64, 0, 24}, {64, 1, 2}, {256, 0, 2}};
    for (auto& s3 : sup)
      if (s3[0] == H && s3[1] == kind && s3[2] == nto) ok = true;
    if (!ok) {
      delete c;
      return fail("ppo_create: no kernel instantiation for this (hidden, net_kind, obs_dim)");
    }
  }
  c->B = B;
  c->nmb = cfg->num_minibatches;
  c->M = (int)(B / cfg->num_minibatches);
  c->rank = cfg->rank;
  c->world = 1;  // statistics and collectives span the communicator attached later (ppo_comm_init*)
  // kernel selection: the options of ppo_create_ex (A/B comparisons of complete, tested kernels);
  // the diagnostic build (PPO_DIAG) also reads the measurement scripts' environment switches
  c->act_kernel = opt.act_kernel;
  c->dw_fused = opt.dw_fused;
  c->dw_dma = opt.dw_dma;
  c->gae_scan = opt.gae_scan;
  c->dw_bx = opt.dw_bx >= 0 ? opt.dw_bx : kDwBxAuto;
  c->rollout_mode = opt.rollout;
  c->gradstep = opt.gradstep;
  c->gn_fold = opt.gradnorm >= 0 ? opt.gradnorm : kGradnormFoldAuto;
  // auto: the graph where the minibatches are small enough that launch overhead shows (cfg1's 64 rows:
  // 17.9 -> 17.4 ms per iteration); at cfg2 / cfg4 / the shards / the metric config it measured equal or
  // 0.5-1 % slower (profiles/r06/update_graph/)
  c->update_graph = opt.update_graph >= 0 ? opt.update_graph : (c->M <= kUpdGraphAutoRows ? 1 : 0);
  c->update_graph_auto = opt.update_graph < 0;
  c->rollout_kernel = opt.rollout_kernel;
  if (opt.rollout_kernel == 2 && (cfg->net_kind != PPO_NET_LN_BETA || c->K.OP > 32)) {
    delete c;  // nothing allocated yet
    return fail("ppo_create: rollout_kernel=valu needs the LayerNorm-Beta agent with obs_dim <= 32");
  }
  int upd_kernel = opt.upd_kernel;
#ifdef PPO_DIAG
  {
    const char* es = getenv("PPO_UPD_SCHED");
    if (es && es[0] >= '0' && es[0] <= '3') c->upd_sched = es[0] - '0';
#ifdef PPO_STAMPS
    if (es) c->upd_sched = atoi(es);  // diagnostic build: bits 4..7 skip stores (ppo_update.hip)
    const char* eg = getenv("PPO_ACT_DIAG");  // diagnostic build: phases of k_act3 to skip (bits, << 8)
    if (eg) c->act_kernel |= atoi(eg) << 8;
#endif
    const char* ea = getenv("PPO_ACT_KERNEL");
    if (ea && (ea[0] == '2' || ea[0] == '4')) c->act_kernel = ea[0] - '0';
    const char* ed = getenv("PPO_DW_FUSED");
    if (ed) c->dw_fused = !(ed[0] == '0');
    const char* ev = getenv("PPO_UPD_KERNEL");
    if (ev && ev[0] == '0') upd_kernel = 1;
    const char* et = getenv("PPO_UPD_TRUNK");
    if (et && (et[0] == '0' || et[0] == '1')) c->upd_trunk_mask = 1 << (et[0] - '0');
  }
#endif
  const int H = cfg->hidden, A = cfg->act_dim, O = cfg->obs_dim, OP = c->K.OP;
  c->sg[0] = make_sg(H, 1, A);
  c->sg[1] = make_sg(H, cfg->net_kind == PPO_NET_LN_BETA ? 2 * A : A, A);
  int rc = 0;
  HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  const size_t PS = c->K.size;
  rc |= dmalloc(&c->P, PS); rc |= dmalloc(&c->G, PS); rc |= dmalloc(&c->Am, PS); rc |= dmalloc(&c->Av, PS);
  for (int k = 0; k < 2; ++k) rc |= dmalloc(&c->W2T[k], (size_t)H * H);
  // room for the split-bf16 pieces after the fp32 copies (upd_mfma=bx6): W2 | W2^T at H = 256, W1 at 64
  for (int k = 0; k < 2; ++k) rc |= dmalloc(&c->WSW[k], (size_t)(sw_size(H, c->K.OP) + bx_region(H, c->K.OP)));
  const size_t E = cfg->num_envs, T = cfg->num_steps;
  rc |= dmalloc(&c->buf[PPO_BUF_OBS], T * E * O);
  rc |= dmalloc(&c->buf[PPO_BUF_ACTIONS], T * E * A);
  for (int b = PPO_BUF_LOGPROBS; b < PPO_BUF_COUNT; ++b)
    if (b != PPO_BUF_ACTIONS) rc |= dmalloc(&c->buf[b], T * E);
  rc |= dmalloc(&c->next_value, E);
  const int EP = cfg->update_epochs;
  rc |= dmalloc(&c->perms, (size_t)EP * B);
  rc |= dmalloc(&c->advstats, (size_t)2 * EP * c->nmb);
  rc |= dmalloc(&c->advsq, (size_t)EP * c->nmb);
  rc |= dmalloc(&c->advpart, (size_t)EP * c->nmb * PPO_ADV_SPLIT);
  const size_t Mr = ((size_t)c->M + 63) / 64 * 64;
  rc |= dmalloc(&c->Xn, Mr * OP + 64);
  for (int k = 0; k < 2; ++k) {
    rc |= dmalloc(&c->H1[k], Mr * H);
    rc |= dmalloc(&c->DZ1[k], Mr * H);
    rc |= dmalloc(&c->DZ2[k], Mr * H);
  }
  const int tiles = (int)(Mr / 64);
  c->tiles_per_block = std::max(1, (tiles + 255) / 256);
  c->nblk = (tiles + c->tiles_per_block - 1) / c->tiles_per_block;
  {
    const int sgmax = std::max(c->sg[0].size, c->sg[1].size);
    // k_upd2 addresses the rollout storage with 32-bit buffer offsets
    const bool fits32 = (double)B * (double)std::max(O, A) * 4.0 < 4294967040.0;
    const int split = !fits32 ? 0 : opt.upd2_split >= 0 ? opt.upd2_split : upd2_split_supported(c->K) ? kUpd2SplitAuto : 0;
    if ((opt.upd_mfma == 32 || opt.upd_mfma == 1) && (H != 256 || cfg->net_kind != PPO_NET_LN_BETA)) {
      ppo_destroy(c);
      return fail("ppo_create: upd_mfma=32 / mix needs the LayerNorm-Beta agent at hidden 256");
    }
    const char* bx_refusal = "ppo_create: upd_mfma=bx6 needs the LayerNorm-Beta agent at hidden 256 with at most 16 "
                             "heads, or the 64-wide agent's single k_upd2 at OP = 384";
    if (opt.upd_mfma == 6 && !((H == 256 && cfg->net_kind == PPO_NET_LN_BETA) || H == 64)) {
      ppo_destroy(c);
      return fail(bx_refusal);
    }
    if (opt.upd2_split > 0 && (upd_kernel || !fits32 || !upd2_split_supported(c->K))) {
      ppo_destroy(c);
      return fail("ppo_create: upd2_split needs the 64-wide agent with O % 4 == 0, OP = 384 and 32-bit storage offsets");
    }
    if (!upd_kernel && fits32 && upd2_supported(c->K, &c->upd, split) == 0) {
      c->use_upd = c->use_upd2 = true;
      c->upd2_split = split;
      // layer 1 as split-bf16 piece products (the single kernel at cfg2's shape)
      const bool want_bx = opt.upd_mfma == 6 || (opt.upd_mfma == 0 && kUpd2BxAuto);
      if (want_bx && split == 0 && upd2_supported(c->K, &c->upd, 0, 1) == 0) {
        c->upd_bx = 2;
      } else if (opt.upd_mfma == 6) {
        ppo_destroy(c);
        return fail(bx_refusal);
      } else if (want_bx) {
        upd2_supported(c->K, &c->upd, split);  // the fp32 form's geometry again
      }
      const int ut = (c->M + c->upd.rows - 1) / c->upd.rows;
      // both trunks per workgroup, 2 workgroups per CU x 256 CUs (split form: 3 per CU)
      c->upd_nblk = std::min(ut, split ? 256 * split : 512);
    } else if (opt.upd_mfma == 32 || opt.upd_mfma == 1) {
      c->upd32_mix = opt.upd_mfma == 1;
      if (upd_kernel || upd32_supported(c->K, c->sg[1].nh, c->sg[0].size, c->sg[1].size, &c->upd, c->upd32_mix) != 0) {
        ppo_destroy(c);
        return fail("ppo_create: upd_mfma=32 / mix needs the LayerNorm-Beta agent at hidden 256");
      }
      c->use_upd = c->use_upd32 = true;
      c->upd_nblk = std::min((c->M + c->upd.rows - 1) / c->upd.rows, 256);
    } else if (opt.upd_mfma == 6 ||
               (opt.upd_mfma == 0 && kUpdBxAuto && !upd_kernel &&
                upd_supported(c->K, c->sg[1].nh, c->sg[0].size, c->sg[1].size, &c->upd, 1) == 0)) {
      if (upd_kernel || upd_supported(c->K, c->sg[1].nh, c->sg[0].size, c->sg[1].size, &c->upd, 1) != 0) {
        ppo_destroy(c);
        return fail(bx_refusal);
      }
      c->use_upd = true;
      c->upd_bx = 1;
      c->upd_nblk = std::min((c->M + c->upd.rows - 1) / c->upd.rows, 256);
    } else if (!upd_kernel && upd_supported(c->K, c->sg[1].nh, c->sg[0].size, c->sg[1].size, &c->upd) == 0) {
      c->use_upd = true;
      const int ut = (c->M + c->upd.rows - 1) / c->upd.rows;
      c->upd_nblk = std::min(ut, 256);  // 2 workgroups per CU x 256 CUs over the two trunks
    }
  }
  // the critic pass on split-bf16 products wherever k_upd keeps the critic's W2 pieces (bx6)
  c->values_bx = (c->upd_bx == 1 && opt.values_mfma != 0 && rollout_supported(c->K) == 0) ? 1 : 0;
  if (opt.values_mfma == 6 && !c->values_bx) {
    ppo_destroy(c);
    return fail("ppo_create: values_mfma=bx6 needs the LayerNorm-Beta agent at hidden 256 with upd_mfma=bx6 (auto)");
  }
  {
    const bool split_ok = c->use_upd && !c->use_upd2 && !c->use_upd32 && H == 256 && OP <= 32 && c->dw_fused;
    int S = opt.upd_split > 0 ? opt.upd_split : kUpdSplitAuto(c->M);
    if (!split_ok) {
      if (opt.upd_split > 1) {
        ppo_destroy(c);
        return fail("ppo_create: upd_split > 1 needs the fused k_upd + k_dwf path (hidden 256, obs_dim <= 32)");
      }
      S = 1;
    }
    while (S > 1 && c->M < S * 32 * 64) S /= 2;  // keep >= 64 tiles of 32 rows per launch
    c->msplit = S;
    c->Mq = S == 1 ? c->M : (((c->M + S - 1) / S + 31) & ~31);
    while (c->msplit > 1 && (long)(c->msplit - 1) * c->Mq >= c->M) --c->msplit;  // no empty split
  }
  for (int k = 0; k < 2; ++k)
    rc |= dmalloc(&c->slab[k], (size_t)c->msplit * std::max(c->nblk, c->upd_nblk) * c->sg[k].size);
  c->wlds_off = 4 * std::max(c->sg[0].size, c->sg[1].size);
  c->wlds_off = (c->wlds_off + 63) & ~63;
  c->lds_bytes = ((size_t)c->wlds_off + 2 * (size_t)H * 16) * sizeof(float);
  // dW split-K: ~128 row chunks per trunk (256 workgroups for the two trunks), 16-row multiples
  // (the chunking does not depend on dw_fused, so k_dwf and the two-phase k_dw sum the same chunks)
  // (with upd_split: the geometry of one Mq-row pair; every pair writes its own nchunks partial rows)
  c->dw_slices = dw_slices(c->Mq, H, OP, true);
  if (opt.dw_slices && H == 256 && OP <= 32) c->dw_slices = opt.dw_slices;  // k_dwf geometry only
  c->rows_per_chunk = std::max(64, (((c->Mq + 128 / c->dw_slices - 1) / (128 / c->dw_slices)) + 15) & ~15);
  if (c->use_upd2) c->rows_per_chunk = std::max(32, (((c->M + 255) / 256) + 31) & ~31);  // k_dw2: both trunks
  if (opt.dw_rows && (!c->use_upd2 || opt.dw_rows % 32 == 0)) c->rows_per_chunk = opt.dw_rows;  // k_dw2: 32-row steps
  c->nchunks = (c->Mq + c->rows_per_chunk - 1) / c->rows_per_chunk;
  {
    const bool rc_ok = c->use_upd && !c->use_upd2 && !c->use_upd32 && cfg->net_kind == PPO_NET_LN_BETA && H == 256 &&
                       OP <= 32 && c->dw_fused && c->dw_dma && c->dw_bx;
    if (opt.h1_handoff == 1 && !rc_ok) {
      ppo_destroy(c);
      return fail("ppo_create: h1_handoff=recompute needs the LayerNorm-Beta agent at hidden 256 (obs_dim <= 32) with "
                  "the fused split-bf16 dW (dw_mfma bf16x6/x8/x9)");
    }
    c->h1_recomp = rc_ok && (opt.h1_handoff == 1 || (opt.h1_handoff < 0 && kH1RecomputeAuto));
    if (c->h1_recomp)
      for (int k = 0; k < 2; ++k) rc |= dmalloc(&c->LNS[k], 2 * (size_t)c->M);
  }
  for (int k = 0; k < 2; ++k) rc |= dmalloc(&c->dwslab[k], (size_t)c->msplit * c->nchunks * (H * H + H * OP));
  if (c->upd2_split) rc |= dmalloc(&c->Z1, Mr * 128);
  rc |= dmalloc(&c->normout, 2 + PPO_LAYOUT_MAX_TENSORS + 2);
  rc |= dmalloc(&c->gnpart, (size_t)PPO_LAYOUT_MAX_TENSORS * PPO_GN_SPLIT);
  rc |= dmalloc(reinterpret_cast<float**>(&c->gs_bar), 1);
  rc |= dmalloc(&c->cs_sq, (size_t)c->K.size / 64 + 2 * PPO_MAX_SEGS + 64);
  rc |= dmalloc(reinterpret_cast<float**>(&c->cs_cnt), PPO_MAX_SEGS);
  rc |= dmalloc(&c->mbstats, (size_t)8 * EP * c->nmb);
  if (rc) {
    ppo_destroy(c);
    return -2;
  }
  if (fwdbwd_set_lds(c->K, c->lds_bytes) != 0) {
    ppo_destroy(c);
    return fail("ppo_create: cannot set LDS size for the fused update kernel");
  }
  HIP_TRY(hipDeviceSynchronize());
  *out = c;
  return 0;
}

extern "C" int ppo_destroy(ppo_t* c) {
  if (!c) return 0;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  prof_drain(c);
  for (auto e : c->free_events) (void)hipEventDestroy(e);
  float* ptrs[] = {c->P, c->G, c->Am, c->Av, c->W2T[0], c->W2T[1], c->WSW[0], c->WSW[1], c->next_value, c->advstats, c->advsq, c->Xn, c->Z1,
                   c->normout, c->gnpart, c->mbstats, c->beta_store, reinterpret_cast<float*>(c->gs_bar), c->cs_sq,
                   reinterpret_cast<float*>(c->cs_cnt)};
  for (float* p : ptrs)
    if (p) (void)hipFree(p);
  for (int b = 0; b < PPO_BUF_COUNT; ++b)
    if (c->buf[b]) (void)hipFree(c->buf[b]);
  for (int k = 0; k < 2; ++k) {
    float* q[] = {c->H1[k], c->DZ1[k], c->DZ2[k], c->slab[k], c->LNS[k]};
    for (float* p : q)
      if (p) (void)hipFree(p);
  }
  for (int k = 0; k < 4; ++k)
    if (c->dwslab[k]) (void)hipFree(c->dwslab[k]);
  if (c->perms) (void)hipFree(c->perms);
  if (c->upd_exec) (void)hipGraphExecDestroy(c->upd_exec);
  if (c->sched) (void)hipFree(c->sched);
  for (int i = 0; i < 2; ++i) {
    if (c->sched_host[i]) (void)hipHostFree(c->sched_host[i]);
    if (c->sched_ev[i]) (void)hipEventDestroy(c->sched_ev[i]);
  }
  if (c->advpart) (void)hipFree(c->advpart);
  comm_detach(c);
  if (c->snap) (void)hipFree(c->snap);
  if (c->snap_ev) (void)hipEventDestroy(c->snap_ev);
  if (c->snap_stream) (void)hipStreamDestroy(c->snap_stream);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return 0;
}

extern "C" int ppo_get_layout(const ppo_t* c, ppo_layout* out) {
  if (!c || !out) return fail("ppo_get_layout: null argument");
  *out = c->L;
  return 0;
}
extern "C" void* ppo_stream(ppo_t* c) { return c ? (void*)c->stream : nullptr; }
extern "C" long ppo_iteration(const ppo_t* c) { return c ? c->iteration : -1; }
extern "C" int ppo_set_iteration(ppo_t* c, long it) {
  if (!c) return fail("null ctx");
  c->iteration = it;
  return 0;
}
#ifdef PPO_DIAG
// diagnostic build only (not part of the C-ABI header): internal device buffers by name
// ("beta_store": the AC rollout's (alpha, beta, sample) per (t, env, action); scripts/debug_rollout_v.py)
extern "C" float* ppo_debug_buffer(ppo_t* c, const char* name) {
  if (!c || !name) return nullptr;
  if (!strcmp(name, "beta_store")) return c->beta_store;
  return nullptr;
}
#endif
extern "C" float* ppo_buffer(ppo_t* c, int which) {
  if (!c || which < 0 || which >= PPO_BUF_COUNT) return nullptr;
  return c->buf[which];
}

// ------------------------------------------------------------------------------------------
// parameters / optimizer state
// ------------------------------------------------------------------------------------------
static int refresh_weight_copies(ppo_t* c) {
  for (int k = 0; k < 2; ++k) launch_transpose(c->P + c->K.tr[k].W2, c->W2T[k], c->K.H, c->stream);
  for (int k = 0; k < 2; ++k)
    launch_swizzle(c->P + c->K.tr[k].W1, c->P + c->K.tr[k].W2, c->WSW[k], c->K.H, c->K.OP, c->upd_bx, c->stream);
  HIP_TRY(hipGetLastError());
  return 0;
}

extern "C" int ppo_load_params(ppo_t* c, const float* host, long n) {
  if (!c || !host) return fail("ppo_load_params: null argument");
  if (n != c->L.P) return fail("ppo_load_params: expected " + std::to_string(c->L.P) + " floats");
  HIP_TRY(hipSetDevice(c->device));
  std::vector<float> packed(c->K.size);
  pack_params(c->K, c->L, host, packed.data());
  HIP_TRY(hipMemcpyAsync(c->P, packed.data(), sizeof(float) * c->K.size, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemsetAsync(c->Am, 0, sizeof(float) * c->K.size, c->stream));
  HIP_TRY(hipMemsetAsync(c->Av, 0, sizeof(float) * c->K.size, c->stream));
  c->adam_step = 0;
  if (refresh_weight_copies(c)) return -2;
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

extern "C" int ppo_save_params(ppo_t* c, float* host, long n) {
  if (!c || !host) return fail("ppo_save_params: null argument");
  if (n != c->L.P) return fail("ppo_save_params: expected " + std::to_string(c->L.P) + " floats");
  HIP_TRY(hipSetDevice(c->device));
  std::vector<float> packed(c->K.size);
  HIP_TRY(hipMemcpyAsync(packed.data(), c->P, sizeof(float) * c->K.size, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  unpack_params(c->K, c->L, packed.data(), host);
  return 0;
}

extern "C" int ppo_save_adam(ppo_t* c, float* m_host, float* v_host, long n, long* step) {
  if (!c) return fail("null ctx");
  if (n != c->L.P) return fail("ppo_save_adam: size mismatch");
  std::vector<float> pm(c->K.size), pv(c->K.size);
  HIP_TRY(hipMemcpyAsync(pm.data(), c->Am, sizeof(float) * c->K.size, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(pv.data(), c->Av, sizeof(float) * c->K.size, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (m_host) unpack_params(c->K, c->L, pm.data(), m_host);
  if (v_host) unpack_params(c->K, c->L, pv.data(), v_host);
  if (step) *step = c->adam_step;
  return 0;
}

extern "C" int ppo_load_adam(ppo_t* c, const float* m_host, const float* v_host, long n, long step) {
  if (!c || !m_host || !v_host) return fail("ppo_load_adam: null argument");
  if (n != c->L.P) return fail("ppo_load_adam: size mismatch");
  std::vector<float> pm(c->K.size), pv(c->K.size);
  pack_params(c->K, c->L, m_host, pm.data());
  pack_params(c->K, c->L, v_host, pv.data());
  HIP_TRY(hipMemcpyAsync(c->Am, pm.data(), sizeof(float) * c->K.size, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->Av, pv.data(), sizeof(float) * c->K.size, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->adam_step = step;
  return 0;
}

// ------------------------------------------------------------------------------------------
// agent calls
// ------------------------------------------------------------------------------------------
static ActArgs base_act(ppo_t* c) {
  ActArgs a;
  memset(&a, 0, sizeof(a));
  a.P = c->P;
  a.K = c->K;
  a.seed = c->cfg.seed;
  a.rank = c->rank;
  a.store_step = -1;
  a.E = c->cfg.num_envs;
  a.kernel = c->act_kernel;
  a.WSW[0] = c->WSW[0];
  a.WSW[1] = c->WSW[1];
  return a;
}

extern "C" int ppo_get_action_and_value(ppo_t* c, int n, const float* x, int sample_type, const float* action_in,
                                        long env_base, long step_id, float* action, float* logprob, float* entropy,
                                        float* value, void* stream) {
  if (!c || !x) return fail("ppo_get_action_and_value: null argument");
  if (n <= 0) return 0;
  if (sample_type == PPO_GIVEN && !action_in) return fail("ppo_get_action_and_value: GIVEN needs action_in");
  if (sample_type < 0 || sample_type > 2) return fail("Unsupported sample type used. Sample type: " + std::to_string(sample_type));
  ActArgs a = base_act(c);
  a.n = n;
  a.x = x;
  a.ldx = c->K.O;
  a.mode = sample_type;
  a.need_actor = (action || logprob || entropy) ? 1 : 0;
  a.action_in = action_in;
  a.env_base = env_base;
  a.step_id = step_id;
  a.action_out = action;
  a.logprob_out = logprob;
  a.entropy_out = entropy;
  a.value_out = value;
  hipStream_t s = S(c, stream);
  ProfScope ps(c, PK_ACT, s);
  if (launch_act(a, s) != 0) return fail("no act kernel for this configuration");
  HIP_TRY(hipGetLastError());
  return 0;
}

extern "C" int ppo_get_value(ppo_t* c, int n, const float* x, float* value, void* stream) {
  return ppo_get_action_and_value(c, n, x, PPO_MEAN, nullptr, 0, 0, nullptr, nullptr, nullptr, value, stream);
}

extern "C" int ppo_rollout_act(ppo_t* c, int step, int e0, int e1, const float* next_obs, const float* next_done,
                               float* action_out, void* stream) {
  if (!c || !next_obs) return fail("ppo_rollout_act: null argument");
  if (step < 0 || step >= c->cfg.num_steps || e0 < 0 || e1 > c->cfg.num_envs || e0 >= e1)
    return fail("ppo_rollout_act: step / env range out of bounds");
  ActArgs a = base_act(c);
  a.n = e1 - e0;
  a.x = next_obs;
  a.ldx = c->K.O;
  a.mode = PPO_SAMPLE;
  a.need_actor = 1;
  a.env_base = e0;
  a.step_id = c->iteration * (long)c->cfg.num_steps + step;
  a.action_out = action_out;
  a.store_step = step;
  a.next_done = next_done;
  a.s_obs = c->buf[PPO_BUF_OBS];
  a.s_actions = c->buf[PPO_BUF_ACTIONS];
  a.s_logp = c->buf[PPO_BUF_LOGPROBS];
  a.s_dones = c->buf[PPO_BUF_DONES];
  a.s_values = c->buf[PPO_BUF_VALUES];
  // values_bx: the critic runs later, once over the stored rows (flush_values: ppo_compute_gae,
  // ppo_rollout_values), with the persistent rollout's kernel, so both collection paths store the
  // same values bit for bit
  a.skip_critic = c->values_bx;
  hipStream_t s = S(c, stream);
  ProfScope ps(c, PK_ACT, s);
  if (launch_act(a, s) != 0) return fail("no act kernel for this configuration");
  if (c->values_bx) {  // groups act concurrently from host threads: an atomic maximum
    int cur = c->values_pending.load();
    while (cur < step + 1 && !c->values_pending.compare_exchange_weak(cur, step + 1)) {
    }
  }
  HIP_TRY(hipGetLastError());
  return 0;
}

extern "C" int ppo_rollout_reward(ppo_t* c, int step, int e0, int e1, const float* reward, void* stream) {
  if (!c || !reward) return fail("ppo_rollout_reward: null argument");
  if (step < 0 || step >= c->cfg.num_steps || e0 < 0 || e1 > c->cfg.num_envs || e0 >= e1)
    return fail("ppo_rollout_reward: step / env range out of bounds");
  HIP_TRY(hipMemcpyAsync(c->buf[PPO_BUF_REWARDS] + (size_t)step * c->cfg.num_envs + e0, reward,
                         sizeof(float) * (e1 - e0), hipMemcpyDeviceToDevice, S(c, stream)));
  return 0;
}

static int gae_launch(ppo_t* c, const float* next_value, const float* next_done, int nsteps, hipStream_t s);

// the critic over n contiguous observation rows (k_vbx with the critic's W2 pieces, else k_values)
static int run_values(ppo_t* c, const float* obs, float* values, long n, hipStream_t s) {
  ValuesArgs v;
  v.P = c->P;
  v.K = c->K;
  v.WSW = c->WSW[0];
  v.obs = obs;
  v.values = values;
  v.n = n;
  v.WBX = c->values_bx ? c->WSW[0] + sw_size(c->K.H, c->K.OP) : nullptr;
  ProfScope ps(c, PK_VALUES, s);
  if (v.WBX) return launch_vbx(v, s) == 0 ? 0 : -1;
  return launch_values(v, s);
}
// the deferred critic pass of per-step rollouts (ppo_rollout_act with values_bx): values[t] for every
// step acted so far, over the stored observations
static int flush_values(ppo_t* c, hipStream_t s) {
  const int steps = c->values_pending.exchange(0);
  if (steps <= 0) return 0;
  if (run_values(c, c->buf[PPO_BUF_OBS], c->buf[PPO_BUF_VALUES], (long)steps * c->cfg.num_envs, s) != 0)
    return fail("ppo_rollout_values: critic kernel launch failed");
  HIP_TRY(hipGetLastError());
  return 0;
}
extern "C" int ppo_rollout_values(ppo_t* c, void* stream) {
  if (!c) return fail("ppo_rollout_values: null argument");
  return flush_values(c, S(c, stream));
}

extern "C" int ppo_compute_gae(ppo_t* c, const float* next_obs, const float* next_done, int nsteps, void* stream) {
  if (!c || !next_obs || !next_done) return fail("ppo_compute_gae: null argument");
  if (nsteps <= 0 || nsteps > c->cfg.num_steps) return fail("ppo_compute_gae: bad step count");
  hipStream_t s = S(c, stream);
  if (int rc = flush_values(c, s)) return rc;
  if (rollout_supported(c->K) == 0) {
    // the bootstrap value with the critic pass that fills values[t] on the persistent path
    if (run_values(c, next_obs, c->next_value, c->cfg.num_envs, s) != 0)
      return fail("ppo_compute_gae: values kernel launch failed");
  } else {
    int rc = ppo_get_value(c, c->cfg.num_envs, next_obs, c->next_value, s);
    if (rc) return rc;
  }
  return gae_launch(c, c->next_value, next_done, nsteps, s);
}

extern "C" int ppo_gae_from_values(ppo_t* c, const float* next_value, const float* next_done, int nsteps,
                                   void* stream) {
  if (!c || !next_value || !next_done) return fail("ppo_gae_from_values: null argument");
  if (nsteps <= 0 || nsteps > c->cfg.num_steps) return fail("ppo_gae_from_values: bad step count");
  if (int rc = flush_values(c, S(c, stream))) return rc;
  return gae_launch(c, next_value, next_done, nsteps, S(c, stream));
}

static int gae_launch(ppo_t* c, const float* next_value, const float* next_done, int nsteps, hipStream_t s) {
  // a partial collection (DD-PPO preemption, nsteps < num_steps): the reference's recurrence bootstraps
  // the last collected step from the STORED step nsteps (values[t + 1], dones[t + 1] whenever
  // t != num_steps - 1, ac:765-774), which every env executed before it stopped; next_value and
  // next_done are not read then
  if (nsteps < c->cfg.num_steps) {
    next_value = c->buf[PPO_BUF_VALUES] + (size_t)nsteps * c->cfg.num_envs;
    next_done = c->buf[PPO_BUF_DONES] + (size_t)nsteps * c->cfg.num_envs;
  }
  GaeArgs g;
  g.rewards = c->buf[PPO_BUF_REWARDS];
  g.values = c->buf[PPO_BUF_VALUES];
  g.dones = c->buf[PPO_BUF_DONES];
  g.next_value = next_value;
  g.next_done = next_done;
  g.adv = c->buf[PPO_BUF_ADVANTAGES];
  g.ret = c->buf[PPO_BUF_RETURNS];
  g.T = nsteps;
  g.E = c->cfg.num_envs;
  g.gamma = c->cfg.gamma;
  g.lam = c->cfg.gae_lambda;
  ProfScope ps(c, PK_GAE, s);
  launch_gae(g, s, c->gae_scan > 0 || (c->gae_scan < 0 && nsteps >= kGaeScanMinT));
  HIP_TRY(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------------------------------
// update
// ------------------------------------------------------------------------------------------
static bool distributed(const ppo_t* c) { return c->comm != nullptr || c->host_ar != nullptr; }

// In-place all-reduce over the attached communicator (no communicator: identity). RCCL runs on the
// context stream; the host transport synchronises the stream, hands the values to the caller's
// function in host memory and copies the result back.
static int allreduce(ppo_t* c, float* buf, long n, int average, hipStream_t s) {
  if (c->comm) {
    ProfScope ps(c, PK_ALLREDUCE, s);
    NCCL_TRY(ncclAllReduce(buf, buf, (size_t)n, ncclFloat, average ? ncclAvg : ncclSum, c->comm, s));
    return 0;
  }
  if (c->host_ar) {
    if ((long)c->host_stage.size() < n) c->host_stage.resize((size_t)n);
    float* h = c->host_stage.data();
    HIP_TRY(hipMemcpyAsync(h, buf, sizeof(float) * n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (c->host_ar(h, n, average, c->host_user) != 0) return fail("ppo host all-reduce callback failed", -3);
    HIP_TRY(hipMemcpyAsync(buf, h, sizeof(float) * n, hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));  // the staging buffer is reused by the next call
  }
  return 0;
}

extern "C" int ppo_update(ppo_t* c, float lr, const int32_t* perms_dev, ppo_update_stats* out) {
  if (!c) return fail("ppo_update: null ctx");
  return ppo_update_ex(c, lr, c->cfg.num_steps, perms_dev, out);
}

extern "C" int ppo_update_ex(ppo_t* c, float lr, int nsteps, const int32_t* perms_dev, ppo_update_stats* out) {
  if (!c) return fail("ppo_update: null ctx");
  if (nsteps <= 0 || nsteps > c->cfg.num_steps) return fail("ppo_update: bad collected step count");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const ppo_hip_config& cfg = c->cfg;
  const int EP = cfg.update_epochs, MB = c->nmb, M = c->M, H = c->K.H, OP = c->K.OP, A = c->K.A;
  const long B = c->B;
  const bool multi = distributed(c);
  if (cfg.world_size > 1 && !multi)
    return fail("ppo_update: world_size " + std::to_string(cfg.world_size) +
                " but no communicator attached (ppo_comm_init / ppo_comm_init_host)");
  if (int rc = flush_values(c, s)) return rc;  // old values of a per-step rollout whose GAE came from elsewhere
  // ---- permutations (torch::randperm per epoch, ppo:490 / ac:804) ----
  // A partial collection of nsteps < num_steps (DD-PPO preemption, ac:803-810): the permutation runs
  // over the Bc = nsteps * E collected samples (the first nsteps rows of the [T, E] storage) and is
  // repeated and truncated to the per-device batch, b_inds.repeat(ceil(B / Bc))[:B]
  const int32_t* perms = perms_dev;
  if (!perms) {
    ProfScope ps(c, PK_PERM, s);
    const long Bc = (long)nsteps * cfg.num_envs;
    for (int e = 0; e < EP; ++e) {
      int32_t* dst = c->perms + (size_t)e * B;
      launch_perm(dst, (uint32_t)Bc, make_perm_key(cfg.seed, c->rank, c->iteration * (long)EP + e, Bc), s);
      for (long have = Bc; have < B;) {  // doubling copies of the periodic prefix
        const long n = std::min(have, B - have);
        HIP_TRY(hipMemcpyAsync(dst + have, dst, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, s));
        have += n;
      }
    }
    perms = c->perms;
  }
  // ---- advantage statistics of every minibatch (ppo:511; distributed ac:833-846) ----
  AdvArgs aa;
  aa.perm = perms;
  aa.adv = c->buf[PPO_BUF_ADVANTAGES];
  aa.stats = c->advstats;
  aa.sq = c->advsq;
  aa.part = c->advpart;
  aa.M = M;
  aa.nmb = EP * MB;
  aa.world = multi ? c->world : 1;
  if (cfg.norm_adv) {
    ProfScope ps(c, PK_ADV, s);
    launch_adv_sum(aa, s);
    if (multi && allreduce(c, c->advstats, 2L * EP * MB, 1, s)) return -3;
    launch_adv_sq(aa, multi ? 0 : 1, s);
    if (multi) {
      if (allreduce(c, c->advsq, (long)EP * MB, 0, s)) return -3;
      launch_adv_finalize(aa, s);
    }
  }
  // ---- per-minibatch launch sequence ----
  UpdArgs u;
  memset(&u, 0, sizeof(u));
  u.P = c->P;
  u.W2T[0] = c->W2T[0];
  u.W2T[1] = c->W2T[1];
  u.WSW[0] = c->WSW[0];
  u.WSW[1] = c->WSW[1];
  u.bx = c->upd_bx;
  u.K = c->K;
  u.sg[0] = c->sg[0];
  u.sg[1] = c->sg[1];
  u.M = M;
  u.tiles_per_block = c->tiles_per_block;
  u.wlds_off = c->wlds_off;
  u.obs = c->buf[PPO_BUF_OBS];
  u.actions = c->buf[PPO_BUF_ACTIONS];
  u.logp = c->buf[PPO_BUF_LOGPROBS];
  u.adv = c->buf[PPO_BUF_ADVANTAGES];
  u.ret = c->buf[PPO_BUF_RETURNS];
  u.val = c->buf[PPO_BUF_VALUES];
  u.rows_n = B;
  u.obs_n = B * c->K.O;
  u.clip_coef = cfg.clip_coef;
  u.ent_coef = cfg.ent_coef;
  u.vf_coef = cfg.vf_coef;
  u.inv_m = 1.0f / (float)M;
  u.clip_vloss = cfg.clip_vloss;
  u.norm_adv = cfg.norm_adv;
  u.Xn = c->Xn;
  u.Z1 = c->Z1;
  u.actn_off = c->upd.actn_off;
  u.acc_off = c->upd.acc_off;
  u.spar_off = c->upd.spar_off;
  u.hw_global = c->upd.hw_global;
  u.trunk_mask = c->upd_trunk_mask;
  u.sched = c->upd_sched;
  u.h1_skip = c->h1_recomp;
#ifdef PPO_DIAG
  {
    static const int hot = [] { const char* e = getenv("PPO_UPD2_HOT"); return e ? atoi(e) : 0; }();
    u.hot = hot;
  }
#endif
  const int nblk = c->use_upd ? c->upd_nblk : c->nblk;  // workgroups that wrote a slab row (per launch)
  const int nsrow = c->msplit * nblk;                     // slab rows of one minibatch (msplit launches)
  for (int k = 0; k < 2; ++k) {
    u.H1[k] = c->H1[k];
    u.LNS[k] = c->LNS[k];
    u.DZ1[k] = c->DZ1[k];
    u.DZ2[k] = c->DZ2[k];
    u.slab[k] = c->slab[k];
  }
  DwArgs dw;
  memset(&dw, 0, sizeof(dw));
  dw.M = M;
  dw.rows_per_chunk = c->rows_per_chunk;
  dw.slices = c->dw_slices;
  dw.fused = c->dw_fused;
  dw.dma = c->dw_dma;
  dw.bx = c->dw_dma ? c->dw_bx : 0;
  dw.h1_recompute = c->h1_recomp;
  dw.kl1 = (c->K.O == 16 * (c->K.OP / 16 - 1) + 1) ? 1 : 4;
  dw.xn = c->Xn;
  dw.obs = c->buf[PPO_BUF_OBS];
  dw.O = c->K.O;
  dw.obs_n = B * c->K.O;
  dw.slab_stride = (long)H * H + (long)H * OP;
  for (int k = 0; k < 2; ++k) {
    dw.dz2[k] = c->DZ2[k];
    dw.h1[k] = c->H1[k];
    dw.lns[k] = c->LNS[k];
    dw.w1sw[k] = c->WSW[k];
    dw.b1[k] = c->P + c->K.tr[k].b1;
    dw.g1[k] = c->P + c->K.tr[k].g1;
    dw.be1[k] = c->P + c->K.tr[k].be1;
    dw.dz1[k] = c->DZ1[k];
    dw.slab[k] = c->dwslab[k];
  }
  // slab -> packed gradient segments
  ColsumArgs cs;
  memset(&cs, 0, sizeof(cs));
  int ns = 0;
  long maxlen = 0;
  auto seg = [&](const float* src, long stride, int count, int len, float* dst, float scale) {
    cs.seg[ns++] = ColsumSeg{src, dst, stride, count, len, scale};
    maxlen = std::max(maxlen, (long)len);
  };
  const bool ln = cfg.net_kind == PPO_NET_LN_BETA;
  for (int k = 0; k < 2; ++k) {
    const TrunkDev& T = c->K.tr[k];
    seg(c->dwslab[k], dw.slab_stride, c->msplit * c->nchunks, H * H, c->G + T.W2, 1.f);
    seg(c->dwslab[k] + (long)H * H, dw.slab_stride, c->msplit * c->nchunks, H * OP, c->G + T.W1, 1.f);
    const SmallGradLayout& g = c->sg[k];
    const float* sl = c->slab[k];
    seg(sl + g.b1, g.size, nsrow, H, c->G + T.b1, 1.f);
    seg(sl + g.b2, g.size, nsrow, H, c->G + T.b2, 1.f);
    if (ln) {
      seg(sl + g.g1, g.size, nsrow, H, c->G + T.g1, 1.f);
      seg(sl + g.be1, g.size, nsrow, H, c->G + T.be1, 1.f);
      seg(sl + g.g2, g.size, nsrow, H, c->G + T.g2, 1.f);
      seg(sl + g.be2, g.size, nsrow, H, c->G + T.be2, 1.f);
    }
    if (k == 0) {
      seg(sl + g.hW, g.size, nsrow, H, c->G + c->K.cW3, 1.f);
      seg(sl + g.hb, g.size, nsrow, 1, c->G + c->K.cb3, 1.f);
    } else if (!ln) {
      seg(sl + g.hW, g.size, nsrow, A * H, c->G + c->K.aW3, 1.f);
      seg(sl + g.hb, g.size, nsrow, A, c->G + c->K.ab3, 1.f);
      seg(sl + g.ls, g.size, nsrow, A, c->G + c->K.logstd, 1.f);
    } else {
      seg(sl + g.hW, g.size, nsrow, A * H, c->G + c->K.aW3, 1.f);
      seg(sl + g.hW + A * H, g.size, nsrow, A * H, c->G + c->K.bW3, 1.f);
      seg(sl + g.hb, g.size, nsrow, A, c->G + c->K.ab3, 1.f);
      seg(sl + g.hb + A, g.size, nsrow, A, c->G + c->K.bb3, 1.f);
    }
  }
  const int stats_seg0 = ns;  // filled per minibatch below
  ns += 3;
  NormArgs na;
  memset(&na, 0, sizeof(na));
  na.grad = c->G;
  na.max_norm = cfg.max_grad_norm;
  na.out = c->normout;
  na.part = c->gnpart;
  for (int t = 0; t < c->K.nt; ++t)
    if (c->K.grad[t]) {
      na.off[na.nt] = c->K.poff[t];
      na.len[na.nt] = c->K.rows[t] * c->K.ld[t];
      na.nt++;
    }
  // gradnorm=fold: every norm tensor must be exactly one gradient segment of the column sums (and no
  // all-reduce may change the gradient between them and the norm); otherwise k_gradnorm runs
  bool fold = c->gn_fold && !multi && !c->gradstep;
  if (fold) {
    int hits[PPO_LAYOUT_MAX_TENSORS] = {};
    for (int k = 0; k < stats_seg0; ++k) {
      cs.seg_t[k] = -1;
      const long off = (long)(cs.seg[k].dst - c->G);
      for (int t = 0; t < na.nt; ++t)
        if (na.off[t] == off && na.len[t] == cs.seg[k].len) { cs.seg_t[k] = t; hits[t]++; }
    }
    for (int t = 0; t < na.nt; ++t) fold = fold && hits[t] == 1;
    long tiles = 0;
    for (int k = 0; k < stats_seg0 + 3; ++k) tiles += (k < stats_seg0 ? (cs.seg[k].len + 63) / 64 : 1);
    fold = fold && tiles <= (long)c->K.size / 64 + 2 * PPO_MAX_SEGS + 64;
  }
  for (int k = stats_seg0; k < stats_seg0 + 3; ++k) cs.seg_t[k] = -1;
  cs.fold = fold ? 1 : 0;
  cs.sq = c->cs_sq;
  cs.cnt = c->cs_cnt;
  cs.part = c->gnpart;
  int tb = -1;
  for (int t = 0; t < c->K.nt; ++t)
    if (c->K.grad[t]) { tb = c->K.poff[t]; break; }
  AdamArgs ad;
  memset(&ad, 0, sizeof(ad));
  ad.param = c->P;
  ad.grad = c->G;
  ad.m = c->Am;
  ad.v = c->Av;
  ad.begin = tb;
  ad.n = c->K.size - tb;
  ad.norm_out = c->normout;
  ad.part = c->gnpart;
  ad.nt = na.nt;
  ad.max_norm = cfg.max_grad_norm;
  ad.eps = cfg.adam_eps;
  ad.H = H;
  ad.OP = c->K.OP;
  for (int k = 0; k < 2; ++k) {
    ad.w2_off[k] = c->K.tr[k].W2;
    ad.w2t[k] = c->W2T[k];
    ad.w1_off[k] = c->K.tr[k].W1;
    ad.wsw[k] = c->WSW[k];
  }
  ad.bx = c->upd_bx;
  const long trainable_n = c->K.size - tb;

  // the minibatch launch sequence; with graph, the Adam step constants come from c->sched[gi]
  auto enqueue = [&](bool graph) -> int {
  for (int e = 0; e < EP; ++e) {
    for (int mb = 0; mb < MB; ++mb) {
      const int gi = e * MB + mb;
      u.perm = perms + (size_t)e * B + (size_t)mb * M;
      u.adv_stats = c->advstats + 2 * gi;
      if (c->use_upd2) dw.perm = u.perm;  // k_dw gathers dW1's input rows itself
      if (c->upd2_split) {
        ProfScope ps(c, PK_L1G, s);
        if (launch_l1g(u, s) != 0) return fail("k_l1g: unsupported configuration");
      }
      // msplit > 1: launch pairs over consecutive Mq-row ranges of the minibatch's permutation; each pair's
      // hand-off rows start at row 0 of the hand-off buffers (reused while cache-resident), its slab rows
      // and dW partial rows follow the previous pair's (the column sums add them all, in pair order);
      // the loss scale stays 1 / M of the whole minibatch
      for (int q = 0; q < c->msplit; ++q) {
        const int mq = std::min(c->Mq, M - q * c->Mq);
        UpdArgs uq = u;
        DwArgs dq = dw;
        if (c->msplit > 1) {
          uq.perm = u.perm + (size_t)q * c->Mq;
          uq.M = mq;
          dq.M = mq;
          for (int k = 0; k < 2; ++k) {
            uq.slab[k] = c->slab[k] + (size_t)q * nblk * c->sg[k].size;
            dq.slab[k] = c->dwslab[k] + (size_t)q * c->nchunks * dw.slab_stride;
          }
        }
        {
          ProfScope ps(c, PK_FWDBWD, s);
          const int rc_ = c->use_upd2  ? launch_upd2(uq, c->upd_nblk, c->upd.lds_bytes, s, c->upd2_split)
                          : c->use_upd32 ? launch_upd32(uq, c->sg[1].nh, c->upd_nblk, c->upd.lds_bytes, s, c->upd32_mix)
                          : c->use_upd ? launch_upd(uq, c->sg[1].nh, c->upd_nblk, c->upd.lds_bytes, s)
                                       : launch_fwdbwd(uq, nblk, c->lds_bytes, s);
          if (rc_ != 0) return fail("no update kernel for this configuration");
        }
        {
          ProfScope ps(c, PK_DW2, s);
          const int nch = (mq + c->rows_per_chunk - 1) / c->rows_per_chunk;
          const int rc_ = c->use_upd2 ? launch_dw2(dq, OP, c->nchunks, s) : launch_dw(dq, H, OP, nch, s);
          if (rc_ != 0) return fail("no dW kernel for this configuration");
          if (nch < c->nchunks && !c->use_upd2)  // a shorter last pair: its unused partial rows must add 0
            for (int k = 0; k < 2; ++k)
              HIP_TRY(hipMemsetAsync(dq.slab[k] + (size_t)nch * dw.slab_stride, 0,
                                     sizeof(float) * (size_t)(c->nchunks - nch) * dw.slab_stride, s));
        }
      }
      float* st = c->mbstats + 8 * gi;
      cs.seg[stats_seg0 + 0] = ColsumSeg{c->slab[1] + c->sg[1].stats + ST_PG, st + ST_PG, c->sg[1].size, nsrow, 1, 1.f / M};
      cs.seg[stats_seg0 + 1] = ColsumSeg{c->slab[0] + c->sg[0].stats + ST_V, st + ST_V, c->sg[0].size, nsrow, 1, 0.5f / M};
      cs.seg[stats_seg0 + 2] = ColsumSeg{c->slab[1] + c->sg[1].stats + ST_ENT, st + ST_ENT, c->sg[1].size, nsrow, 4, 1.f / M};
      {
        ProfScope ps(c, PK_COLSUM, s);
        launch_colsum(cs, ns, maxlen, s);
      }
      if (multi && allreduce(c, c->G + tb, trainable_n, 1, s)) return -3;  // ac:877-885, before the clip
      if (graph) {
        ad.sched = c->sched;
        ad.gi = gi;
      } else {
        c->adam_step += 1;
        const double bc1 = 1.0 - std::pow(0.9, (double)c->adam_step);
        const double bc2 = 1.0 - std::pow(0.999, (double)c->adam_step);
        ad.step_size = (float)((double)lr / bc1);
        ad.sbc2 = (float)std::sqrt(bc2);
      }
      ad.stat_out = st + 6;  // the total norm of this minibatch next to its loss stats
      if (c->gradstep) {  // clip_grad_norm_ + Adam: one cooperative launch (profile class "adam")
        ProfScope ps(c, PK_ADAM, s);
        if (launch_gradstep(na, ad, c->gs_bar, &c->gs_count, s) != 0) return fail("k_gradstep launch failed");
      } else {
        if (!cs.fold) {
          ProfScope ps(c, PK_GRADNORM, s);
          launch_gradnorm(na, s);
        }
        ProfScope ps(c, PK_ADAM, s);
        launch_adam(ad, s);
      }
    }
  }
  return 0;
  };
  // hipGraph replay (update_graph=1, one process, split clip + Adam, no profiling events): captured
  // on the second call (the first warms the launchers' one-time attribute calls), re-captured when
  // the permutation buffer changes; every captured kernel argument is fixed across iterations
  // auto stays eager for a caller that takes snapshots (the CLIs' checkpoint writer thread reads them
  // while the next update runs: a capture then failed on the GPU box, "operation failed due to a previous
  // error during capture"); update_graph=1 keeps the graph with snapshots (single-threaded callers)
  const bool use_graph = c->update_graph && !multi && !c->gradstep && c->prof_mask == 0 && !(c->update_graph_auto && c->snap);
  if (use_graph && c->upd_calls > 0) {
    const int n = EP * MB;
    if (!c->sched) {
      if (dmalloc(&c->sched, 2 * (size_t)n)) return -2;
      for (int i = 0; i < 2; ++i) {
        HIP_TRY(hipHostMalloc((void**)&c->sched_host[i], sizeof(float) * 2 * n, hipHostMallocDefault));
        HIP_TRY(hipEventCreateWithFlags(&c->sched_ev[i], hipEventDisableTiming));
      }
    }
    // the staging buffer alternates per replay; before refilling one, wait until the copy that last
    // read it (two replays ago) has completed — back-to-back replays never overwrite a pending copy
    float* sh = c->sched_host[c->sched_flip];
    HIP_TRY(hipEventSynchronize(c->sched_ev[c->sched_flip]));
    for (int gi = 0; gi < n; ++gi) {  // the eager path's per-step constants, same expressions
      const long t = c->adam_step + 1 + gi;
      const double bc1 = 1.0 - std::pow(0.9, (double)t);
      const double bc2 = 1.0 - std::pow(0.999, (double)t);
      sh[2 * gi] = (float)((double)lr / bc1);
      sh[2 * gi + 1] = (float)std::sqrt(bc2);
    }
    HIP_TRY(hipMemcpyAsync(c->sched, sh, sizeof(float) * 2 * n, hipMemcpyHostToDevice, s));
    HIP_TRY(hipEventRecord(c->sched_ev[c->sched_flip], s));
    c->sched_flip ^= 1;
    if (!c->upd_exec || c->upd_exec_perms != perms) {
      if (c->upd_exec) (void)hipGraphExecDestroy(c->upd_exec);
      c->upd_exec = nullptr;
      HIP_TRY(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      const int rc = enqueue(true);
      hipGraph_t g = nullptr;
      const hipError_t ec = hipStreamEndCapture(s, &g);
      if (rc != 0) {
        if (g) (void)hipGraphDestroy(g);
        return rc;
      }
      if (ec != hipSuccess) return fail(std::string("ppo_update: graph capture: ") + hipGetErrorString(ec));
      const hipError_t ei = hipGraphInstantiate(&c->upd_exec, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      if (ei != hipSuccess) {
        c->upd_exec = nullptr;
        return fail(std::string("ppo_update: graph instantiate: ") + hipGetErrorString(ei));
      }
      c->upd_exec_perms = perms;
    }
    HIP_TRY(hipGraphLaunch(c->upd_exec, s));
    c->adam_step += n;
  } else {
    const int rc = enqueue(false);
    if (rc != 0) return rc;
  }
  c->upd_calls += 1;
  HIP_TRY(hipGetLastError());
  c->iteration += 1;
  if (out) {
    std::vector<float> h((size_t)8 * EP * MB);
    if (multi && allreduce(c, c->mbstats, 8L * EP * MB, 1, s)) return -3;  // logging averages, ac:895-901
    HIP_TRY(hipMemcpyAsync(h.data(), c->mbstats, sizeof(float) * h.size(), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const float* last = h.data() + 8 * (EP * MB - 1);
    out->pg_loss = last[ST_PG];
    out->v_loss = last[ST_V];
    out->entropy = last[ST_ENT];
    out->old_approx_kl = last[ST_OKL];
    out->approx_kl = last[ST_KL];
    double cf = 0;
    for (int i = 0; i < EP * MB; ++i) cf += h[8 * i + ST_CF];
    out->clipfrac = (float)(cf / (EP * MB));
    out->grad_norm = last[6];
    out->minibatches = EP * MB;
  }
  return 0;
}

extern "C" int ppo_debug_last_grad(ppo_t* c, float* host, long n) {
  if (!c || !host) return fail("ppo_debug_last_grad: null argument");
  if (n != c->L.P) return fail("ppo_debug_last_grad: size mismatch");
  std::vector<float> packed(c->K.size);
  HIP_TRY(hipMemcpyAsync(packed.data(), c->G, sizeof(float) * c->K.size, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  unpack_params(c->K, c->L, packed.data(), host);
  return 0;
}

extern "C" int ppo_snapshot_state(ppo_t* c) {
  if (!c) return fail("null ctx");
  HIP_TRY(hipSetDevice(c->device));
  const size_t n = c->K.size;
  if (!c->snap) {
    HIP_TRY(hipMalloc(&c->snap, 3 * n * sizeof(float)));
    HIP_TRY(hipEventCreateWithFlags(&c->snap_ev, hipEventDisableTiming));
    HIP_TRY(hipStreamCreateWithFlags(&c->snap_stream, hipStreamNonBlocking));
  }
  HIP_TRY(hipMemcpyAsync(c->snap, c->P, n * sizeof(float), hipMemcpyDeviceToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->snap + n, c->Am, n * sizeof(float), hipMemcpyDeviceToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->snap + 2 * n, c->Av, n * sizeof(float), hipMemcpyDeviceToDevice, c->stream));
  HIP_TRY(hipEventRecord(c->snap_ev, c->stream));
  c->snap_step = c->adam_step;
  return 0;
}

extern "C" int ppo_read_snapshot(ppo_t* c, float* p, float* m, float* v, long n, long* step) {
  if (!c) return fail("null ctx");
  if (!c->snap) return fail("ppo_read_snapshot: no snapshot taken");
  if (n != c->L.P) return fail("ppo_read_snapshot: size mismatch");
  HIP_TRY(hipSetDevice(c->device));
  const size_t K = c->K.size;
  std::vector<float> h(3 * K);
  // a host wait, not hipStreamWaitEvent: a cross-stream dependency on the context stream is refused
  // while the owner thread captures that stream into the update hipGraph (update_graph=1)
  HIP_TRY(hipEventSynchronize(c->snap_ev));
  HIP_TRY(hipMemcpyAsync(h.data(), c->snap, 3 * K * sizeof(float), hipMemcpyDeviceToHost, c->snap_stream));
  HIP_TRY(hipStreamSynchronize(c->snap_stream));
  if (p) unpack_params(c->K, c->L, h.data(), p);
  if (m) unpack_params(c->K, c->L, h.data() + K, m);
  if (v) unpack_params(c->K, c->L, h.data() + 2 * K, v);
  if (step) *step = c->snap_step;
  return 0;
}

extern "C" int ppo_sync(ppo_t* c) {
  if (!c) return fail("null ctx");
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

// ------------------------------------------------------------------------------------------
// communicator (RCCL)
// ------------------------------------------------------------------------------------------
extern "C" int ppo_comm_unique_id(char id_out[PPO_COMM_ID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) <= PPO_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  memset(id_out, 0, PPO_COMM_ID_BYTES);
  memcpy(id_out, &id, sizeof(id));
  return 0;
}

static void comm_detach(ppo_t* c) {
  if (c->comm) (void)ncclCommDestroy(c->comm);
  c->comm = nullptr;
  c->host_ar = nullptr;
  c->host_user = nullptr;
  c->world = 1;
}

// A real RCCL communicator for every world size, world = 1 included: a one-rank group runs the
// same distributed update sequence (advantage statistics, gradient and stats all-reduces) as a
// multi-GPU job, which is how the single-GPU tests exercise it.
extern "C" int ppo_comm_init(ppo_t* c, const char id[PPO_COMM_ID_BYTES], int rank, int world) {
  if (!c || !id) return fail("ppo_comm_init: null argument");
  if (world < 1 || rank < 0 || rank >= world) return fail("ppo_comm_init: bad rank / world size");
  HIP_TRY(hipSetDevice(c->device));
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  comm_detach(c);
  NCCL_TRY(ncclCommInitRank(&c->comm, world, uid, rank));
  c->rank = rank;
  c->world = world;
  return 0;
}

extern "C" int ppo_comm_init_host(ppo_t* c, int rank, int world, ppo_host_allreduce_fn fn, void* user) {
  if (!c || !fn) return fail("ppo_comm_init_host: null argument");
  if (world < 1 || rank < 0 || rank >= world) return fail("ppo_comm_init_host: bad rank / world size");
  comm_detach(c);
  c->host_ar = fn;
  c->host_user = user;
  c->rank = rank;
  c->world = world;
  return 0;
}

extern "C" int ppo_comm_destroy(ppo_t* c) {
  if (!c) return fail("null ctx");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  comm_detach(c);
  return 0;
}

extern "C" int ppo_comm_broadcast_params(ppo_t* c, int root) {
  if (!c) return fail("null ctx");
  if (!distributed(c)) return 0;
  if (root < 0 || root >= c->world) return fail("ppo_comm_broadcast_params: bad root");
  HIP_TRY(hipSetDevice(c->device));
  if (c->comm) {
    NCCL_TRY(ncclBroadcast(c->P, c->P, (size_t)c->K.size, ncclFloat, root, c->comm, c->stream));
  } else {  // host transport: sum with zeros from every rank but the root (x + 0 == x exactly)
    if (c->rank != root) HIP_TRY(hipMemsetAsync(c->P, 0, sizeof(float) * c->K.size, c->stream));
    if (allreduce(c, c->P, (long)c->K.size, 0, c->stream)) return -3;
  }
  if (refresh_weight_copies(c)) return -2;
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

extern "C" int ppo_comm_allreduce(ppo_t* c, float* buf, long n, int average) {
  if (!c || !buf) return fail("null argument");
  return allreduce(c, buf, n, average, c->stream);
}

extern "C" int ppo_comm_info(const ppo_t* c, int* kind, int* rank, int* world) {
  if (!c || !kind || !rank || !world) return fail("ppo_comm_info: null argument");
  if (c->comm) {
    *kind = PPO_COMM_RCCL;
    NCCL_TRY(ncclCommCount(c->comm, world));
    NCCL_TRY(ncclCommUserRank(c->comm, rank));
  } else if (c->host_ar) {
    *kind = PPO_COMM_HOST;
    *rank = c->rank;
    *world = c->world;
  } else {
    *kind = PPO_COMM_NONE;
    *rank = c->rank;
    *world = c->world;
  }
  return 0;
}

// ------------------------------------------------------------------------------------------
// device helpers
// ------------------------------------------------------------------------------------------
extern "C" int ppo_get_device(const ppo_t* c, int* device, char* pci_bus_id, int len) {
  if (!c || !device) return fail("ppo_get_device: null argument");
  *device = c->device;
  if (pci_bus_id && len > 0) HIP_TRY(hipDeviceGetPCIBusId(pci_bus_id, len, c->device));
  return 0;
}

extern "C" int ppo_kernel_info(const ppo_t* c, char* buf, int len) {
  if (!c || !buf || len <= 0) return fail("ppo_kernel_info: null argument");
  std::string upd = c->use_upd2    ? (c->upd2_split ? "k_l1g+k_upd2" : c->upd_bx ? "k_upd2/bx6" : "k_upd2/f32")
                    : c->use_upd32 ? (c->upd32_mix ? "k_upd32/mix" : "k_upd32")
                    : c->use_upd   ? (c->upd_bx ? "k_upd/bx6" : "k_upd/f32")
                                   : "k_fwdbwd";
  if (c->use_upd && !c->use_upd2 && c->upd.hw_global) upd += "/hwg";  // actor dW3 sums in its slab row
  const int H = c->K.H, OP = c->K.OP;
  const bool fused = c->dw_fused && H == 256 && (OP == 16 || OP == 32);  // launch_dw's dispatch
  const std::string bxs = c->dw_bx ? "/bf16x" + std::to_string(c->dw_bx) : "/f32";
  std::string dw = c->use_upd2 ? (c->dw_dma && OP == 384 && c->K.O % 4 == 0 ? "k_dw2_dma" + bxs : "k_dw2")
                   : fused ? (!c->dw_dma ? "k_dwf" : c->dw_bx ? "k_dwf_bx/bf16x" + std::to_string(c->dw_bx) + (c->h1_recomp ? "/h1rc" : "")
                                                        : "k_dwf_dma/f32")
                   : (c->dw_dma && H == 256 && OP == 112) ? "k_dw_dma" + bxs
                                                          : "k_dw";
  const std::string vals = rollout_supported(c->K) != 0 ? "k_act" : c->values_bx ? "k_vbx/bx6"
                           : c->K.kind == PPO_NET_TANH_NORMAL ? "k_values4/f32" : "k_values/f32";
  const std::string s = "update=" + upd + " dw=" + dw + " values=" + vals +
                        (c->gn_fold && !c->gradstep ? " norm=k_colsum" : c->gradstep ? " norm=k_gradstep" : " norm=k_gradnorm");
  snprintf(buf, (size_t)len, "%s", s.c_str());
  return 0;
}

extern "C" int ppo_set_device(int d) {
  if (int rc = ppo_runtime_check()) return rc;
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (d < 0 || d >= ndev)
    return fail("ppo_set_device: device " + std::to_string(d) + " requested but " + std::to_string(ndev) +
                " HIP device(s) are visible");
  HIP_TRY(hipSetDevice(d));
  return 0;
}
extern "C" int ppo_device_count(int* n) { HIP_TRY(hipGetDeviceCount(n)); return 0; }
// The helpers are host-synchronous and device-wide ordered: contexts run on non-blocking streams,
// which are NOT ordered against the legacy null stream that plain hipMemcpy/hipMemset use.
extern "C" int ppo_dev_malloc(void** p, size_t bytes) {
  if (int rc = ppo_runtime_check()) return rc;
  HIP_TRY(hipMalloc(p, bytes ? bytes : 1));
  HIP_TRY(hipMemset(*p, 0, bytes ? bytes : 1));
  HIP_TRY(hipDeviceSynchronize());
  return 0;
}
extern "C" int ppo_dev_free(void* p) {
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipFree(p));
  return 0;
}
extern "C" int ppo_memcpy_h2d(void* d, const void* h, size_t n) {
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(d, h, n, hipMemcpyHostToDevice));
  HIP_TRY(hipDeviceSynchronize());
  return 0;
}
extern "C" int ppo_memcpy_d2h(void* h, const void* d, size_t n) {
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(h, d, n, hipMemcpyDeviceToHost));
  return 0;
}
extern "C" int ppo_memset_dev(void* d, int v, size_t n) {
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemset(d, v, n));
  HIP_TRY(hipDeviceSynchronize());
  return 0;
}
extern "C" int ppo_device_sync(void) { HIP_TRY(hipDeviceSynchronize()); return 0; }

// ------------------------------------------------------------------------------------------
// profiling API
// ------------------------------------------------------------------------------------------
extern "C" int ppo_profile_enable(ppo_t* c, int mask) {
  if (!c) return fail("null ctx");
  c->prof_mask = (unsigned)mask;
  return 0;
}
extern "C" int ppo_profile_read(ppo_t* c, double* ms, long* count, int cap) {
  if (!c) return fail("null ctx");
  prof_drain(c);
  for (int i = 0; i < PK_COUNT && i < cap; ++i) {
    if (ms) ms[i] = c->prof_ms[i];
    if (count) count[i] = c->prof_cnt[i];
  }
  return PK_COUNT;
}
extern "C" const char* ppo_profile_name(int id) { return (id >= 0 && id < PK_COUNT) ? kProfNames[id] : ""; }
extern "C" int ppo_profile_reset(ppo_t* c) {
  if (!c) return fail("null ctx");
  prof_drain(c);
  for (int i = 0; i < PK_COUNT; ++i) {
    c->prof_ms[i] = 0;
    c->prof_cnt[i] = 0;
  }
  return 0;
}

// ------------------------------------------------------------------------------------------
// synthetic device env
// ------------------------------------------------------------------------------------------
struct psyn_env {
  SynthArgs a;
  float act_lo = -1.0f, act_hi = 1.0f;  // the env's action space (clip_actions, gym.h:141-144)
  int device;
  float* host_stats = nullptr;  // pinned [3][E]: psyn_episode_stats_begin / _end
  hipEvent_t stats_ev = nullptr;
};

extern "C" int psyn_create(int E, int O, int A, psyn_t** out) {
  if (!out || E <= 0 || O <= 0 || A <= 0) return fail("psyn_create: bad arguments");
  if (O > PSYN_MAXO) return fail("psyn_create: obs_dim > 384 is not supported by the device env");
  psyn_t* env = new psyn_t();
  memset(&env->a, 0, sizeof(env->a));
  (void)hipGetDevice(&env->device);
  SynthArgs& a = env->a;
  a.E = E; a.O = O; a.A = A;
  int rc = 0;
  rc |= dmalloc(&a.q, (size_t)E * O);
  rc |= dmalloc(&a.t, E);
  rc |= dmalloc(&a.autoreset, E);
  rc |= dmalloc(&a.rseed, E);
  rc |= dmalloc(&a.rcount, E);
  rc |= dmalloc(&a.ep_ret, E);
  rc |= dmalloc(&a.ep_len, E);
  rc |= dmalloc(&a.fin_ret, E);
  rc |= dmalloc(&a.fin_len, E);
  rc |= dmalloc(&a.fin_cnt, E);
  if (rc) {
    psyn_destroy(env);
    return -2;
  }
  HIP_TRY(hipDeviceSynchronize());
  *out = env;
  return 0;
}

extern "C" int psyn_destroy(psyn_t* env) {
  if (!env) return 0;
  SynthArgs& a = env->a;
  void* ptrs[] = {a.q, a.t, a.autoreset, a.rseed, a.rcount, a.ep_ret, a.ep_len, a.fin_ret, a.fin_len, a.fin_cnt};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (env->host_stats) (void)hipHostFree(env->host_stats);
  if (env->stats_ev) (void)hipEventDestroy(env->stats_ev);
  delete env;
  return 0;
}

extern "C" int psyn_reset(psyn_t* env, int seed, float* obs, float* done, void* stream) {
  if (!env || !obs) return fail("psyn_reset: null argument");
  launch_synth_reset(env->a, seed, obs, done, (hipStream_t)stream);
  HIP_TRY(hipGetLastError());
  return 0;
}

extern "C" int psyn_step(psyn_t* env, int e0, int e1, const float* act, float lo, float hi, float* obs, float* reward,
                         float* done, void* stream) {
  if (!env || !act || !obs || !reward || !done) return fail("psyn_step: null argument");
  if (e0 < 0 || e1 > env->a.E || e0 >= e1) return fail("psyn_step: env range out of bounds");
  launch_synth_step(env->a, e0, e1, act, lo, hi, obs, reward, done, (hipStream_t)stream);
  HIP_TRY(hipGetLastError());
  return 0;
}

// One full device-resident rollout (ppo:387-434 with the env behind the gymcpp boundary replaced by
// the synthetic device env): T x {agent act + store, env step, reward store}. next_obs / next_done
// carry the env state across iterations exactly like the reference's next_obs / next_done tensors.
extern "C" int ppo_rollout_synth(ppo_t* c, psyn_t* env, float* next_obs, float* next_done, float* act_scratch,
                                 float* rew_scratch) {
  if (!c || !env || !next_obs || !next_done || !act_scratch || !rew_scratch) return fail("ppo_rollout_synth: null argument");
  const int E = c->cfg.num_envs;
  if (env->a.E != E || env->a.O != c->K.O || env->a.A != c->K.A) return fail("ppo_rollout_synth: env shape mismatch");
  const float lo = env->act_lo, hi = env->act_hi;
  // the AC kernel has no wrapper chain (the AC trainer's envs carry none, ac:50-53); the PPO kernel
  // runs k_act4's arithmetic (the per-step path's kernel at O >= 112, or with act_kernel=4)
  const bool persistent = c->rollout_mode == PPO_ROLLOUT_AUTO && rollout_supported(c->K) == 0 &&
                          (c->K.kind == PPO_NET_TANH_NORMAL || !env->a.w.on);
  if (persistent) {
    // one persistent launch for all T steps (k_rollout), then the critic over the stored rows
    RolloutArgs r;
    memset(&r, 0, sizeof(r));
    r.P = c->P;
    r.K = c->K;
    r.WSW = c->WSW[1];
    r.E = E;
    r.T = c->cfg.num_steps;
    r.step0 = c->iteration * (long)c->cfg.num_steps;
    r.seed = c->cfg.seed;
    r.rank = c->rank;
    r.next_obs = next_obs;
    r.next_done = next_done;
    r.s_obs = c->buf[PPO_BUF_OBS];
    r.s_actions = c->buf[PPO_BUF_ACTIONS];
    r.s_logp = c->buf[PPO_BUF_LOGPROBS];
    r.s_dones = c->buf[PPO_BUF_DONES];
    r.s_rewards = c->buf[PPO_BUF_REWARDS];
    r.env = env->a;
    r.lo = lo;
    r.hi = hi;
    r.variant = c->rollout_kernel;
    if (c->K.kind == PPO_NET_LN_BETA) {  // Beta log-probs after the rollout (off the env's path)
      if (!c->beta_store && dmalloc(&c->beta_store, (size_t)E * c->cfg.num_steps * c->K.A * 3)) return -2;
      r.s_beta = c->beta_store;
    }
    {
      ProfScope ps(c, PK_ROLLOUT, c->stream);
      if (const int lrc = launch_rollout(r, c->stream))
        return fail(lrc == -3 ? "ppo_rollout_synth: rollout_kernel=valu needs the LayerNorm-Beta agent, O <= 32 and no "
                                "device env wrappers"
                              : "ppo_rollout_synth: rollout kernel launch failed");
      if (r.s_beta) launch_beta_logp(r.s_beta, c->buf[PPO_BUF_LOGPROBS], (long)E * c->cfg.num_steps, c->K.A, c->stream);
    }
    c->values_pending.store(0);  // every stored row's value comes from this pass
    if (run_values(c, c->buf[PPO_BUF_OBS], c->buf[PPO_BUF_VALUES], (long)E * c->cfg.num_steps, c->stream) != 0)
      return fail("ppo_rollout_synth: values kernel launch failed");
    HIP_TRY(hipGetLastError());
    return 0;
  }
  for (int t = 0; t < c->cfg.num_steps; ++t) {
    int rc = ppo_rollout_act(c, t, 0, E, next_obs, next_done, act_scratch, nullptr);
    if (rc) return rc;
    {
      ProfScope ps(c, PK_SYNTH, c->stream);
      // the env's reward output IS rewards[t] of the rollout storage (ppo:406) — no extra copy
      launch_synth_step(env->a, 0, E, act_scratch, lo, hi, next_obs, c->buf[PPO_BUF_REWARDS] + (size_t)t * E,
                        next_done, c->stream);
    }
  }
  if (int rc = flush_values(c, c->stream)) return rc;  // the rollout's values, as the persistent path leaves them
  HIP_TRY(hipGetLastError());
  return 0;
}

extern "C" int psyn_episode_stats_begin(psyn_t* env, void* stream) {
  if (!env) return fail("null env");
  const int E = env->a.E;
  hipStream_t s = (hipStream_t)stream;
  if (!env->host_stats) {
    HIP_TRY(hipHostMalloc(&env->host_stats, sizeof(float) * 3 * E));
    HIP_TRY(hipEventCreateWithFlags(&env->stats_ev, hipEventDisableTiming));
  }
  float* src[3] = {env->a.fin_ret, env->a.fin_len, env->a.fin_cnt};
  for (int k = 0; k < 3; ++k) {
    HIP_TRY(hipMemcpyAsync(env->host_stats + (size_t)k * E, src[k], sizeof(float) * E, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemsetAsync(src[k], 0, sizeof(float) * E, s));
  }
  HIP_TRY(hipEventRecord(env->stats_ev, s));
  return 0;
}

extern "C" int psyn_episode_stats_end(psyn_t* env, float* sr, float* sl, float* sc) {
  if (!env || !env->stats_ev) return fail("psyn_episode_stats_end: no read-out pending");
  HIP_TRY(hipEventSynchronize(env->stats_ev));
  const int E = env->a.E;
  double R = 0, Lsum = 0, N = 0;
  const float* h = env->host_stats;
  for (int i = 0; i < E; ++i) { R += h[i]; Lsum += h[E + i]; N += h[2 * E + i]; }
  if (sr) *sr = (float)R;
  if (sl) *sl = (float)Lsum;
  if (sc) *sc = (float)N;
  return 0;
}

extern "C" int psyn_episode_stats(psyn_t* env, float* sr, float* sl, float* sc) {
  if (!env) return fail("null env");
  const int E = env->a.E;
  std::vector<float> r(E), l(E), n(E);
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(r.data(), env->a.fin_ret, sizeof(float) * E, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(l.data(), env->a.fin_len, sizeof(float) * E, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(n.data(), env->a.fin_cnt, sizeof(float) * E, hipMemcpyDeviceToHost));
  double R = 0, Lsum = 0, N = 0;
  for (int i = 0; i < E; ++i) { R += r[i]; Lsum += l[i]; N += n[i]; }
  HIP_TRY(hipMemset(env->a.fin_ret, 0, sizeof(float) * E));
  HIP_TRY(hipMemset(env->a.fin_len, 0, sizeof(float) * E));
  HIP_TRY(hipMemset(env->a.fin_cnt, 0, sizeof(float) * E));
  HIP_TRY(hipDeviceSynchronize());
  if (sr) *sr = (float)R;
  if (sl) *sl = (float)Lsum;
  if (sc) *sc = (float)N;
  return 0;
}

extern "C" int psyn_set_action_space(psyn_t* env, float lo, float hi) {
  if (!env || !(lo < hi)) return fail("psyn_set_action_space: bad arguments");
  env->act_lo = lo;
  env->act_hi = hi;
  return 0;
}

extern "C" int psyn_action_space(const psyn_t* env, float* lo, float* hi) {
  if (!env || !lo || !hi) return fail("psyn_action_space: null argument");
  *lo = env->act_lo;
  *hi = env->act_hi;
  return 0;
}

// ------------------------------------------------------------------------------------------
// PPO env wrapper chain on the device (include/ppo_env_wrappers.h)
// ------------------------------------------------------------------------------------------
struct pwrap {
  WrapArgs w;
  int E, O;
  float* state = nullptr;  // 2*E*O + 5*E floats (orc_vwrap_* layout)
};

extern "C" int pwrap_create(int E, int O, float gamma, pwrap_t** out) {
  if (!out || E <= 0 || O <= 0) return fail("pwrap_create: bad arguments");
  pwrap_t* p = new pwrap_t();
  p->E = E;
  p->O = O;
  const size_t n = 2 * (size_t)E * O + 5 * (size_t)E;
  if (dmalloc(&p->state, n)) {
    delete p;
    return -2;
  }
  std::vector<float> h(n, 0.0f);  // mean 0, var 1, obs count 1e-4; reward mean 0, var 1, acc 0, count 1e-8
  for (size_t k = (size_t)E * O; k < 2 * (size_t)E * O; ++k) h[k] = 1.0f;
  float* tail = h.data() + 2 * (size_t)E * O;
  for (int e = 0; e < E; ++e) {
    tail[e] = 1e-4f;
    tail[2 * E + e] = 1.0f;
    tail[4 * E + e] = 1e-8f;
  }
  HIP_TRY(hipMemcpy(p->state, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
  WrapArgs& w = p->w;
  w.om = p->state;
  w.ov = p->state + (size_t)E * O;
  w.ocount = p->state + 2 * (size_t)E * O;
  w.rmean = w.ocount + E;
  w.rvar = w.rmean + E;
  w.racc = w.rvar + E;
  w.rcount = w.racc + E;
  w.gamma = gamma;
  w.on = 1;
  *out = p;
  return 0;
}

extern "C" int pwrap_destroy(pwrap_t* p) {
  if (!p) return 0;
  if (p->state) (void)hipFree(p->state);
  delete p;
  return 0;
}

extern "C" int pwrap_reset(pwrap_t* p, int e0, int e1, float* obs, void* stream) {
  if (!p || !obs) return fail("pwrap_reset: null argument");
  if (e0 < 0 || e1 > p->E || e0 >= e1) return fail("pwrap_reset: env range out of bounds");
  launch_wrap_step(p->w, p->O, e0, e1, obs, nullptr, nullptr, nullptr, (hipStream_t)stream);
  HIP_TRY(hipGetLastError());
  return 0;
}

extern "C" int pwrap_step(pwrap_t* p, int e0, int e1, float* obs, float* reward, const float* term,
                          const float* is_reset, void* stream) {
  if (!p || !obs || !reward) return fail("pwrap_step: null argument");
  if (e0 < 0 || e1 > p->E || e0 >= e1) return fail("pwrap_step: env range out of bounds");
  launch_wrap_step(p->w, p->O, e0, e1, obs, reward, term, is_reset, (hipStream_t)stream);
  HIP_TRY(hipGetLastError());
  return 0;
}

extern "C" int pwrap_read_state(pwrap_t* p, float* host, long n) {
  if (!p || !host) return fail("pwrap_read_state: null argument");
  if (n != 2L * p->E * p->O + 5L * p->E) return fail("pwrap_read_state: size mismatch");
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(host, p->state, n * sizeof(float), hipMemcpyDeviceToHost));
  return 0;
}

extern "C" int psyn_attach_wrappers(psyn_t* env, pwrap_t* p) {
  if (!env) return fail("psyn_attach_wrappers: null env");
  if (!p) {
    env->a.w = WrapArgs{};
    return 0;
  }
  if (p->E != env->a.E || p->O != env->a.O) return fail("psyn_attach_wrappers: shape mismatch");
  env->a.w = p->w;
  return 0;
}

extern "C" int ppo_set_rollout_mode(ppo_t* c, int mode) {
  if (!c) return fail("null ctx");
  if (mode != PPO_ROLLOUT_AUTO && mode != PPO_ROLLOUT_PER_STEP) return fail("ppo_set_rollout_mode: bad mode");
  c->rollout_mode = mode;
  return 0;
}
