/*
 * ppo_hip.h — C-ABI of libppo_hip.so: the MI355X-native rollout -> GAE -> PPO-update hot path.
 *
 * Plain C: opaque handles, plain pointers and sizes, int status codes (0 = OK; on error
 * ppo_last_error() returns a thread-local message). All `*_dev` pointers are HIP device pointers
 * (allocate with ppo_dev_malloc or hipMalloc); `stream` arguments are hipStream_t passed as
 * void* (NULL = the context's own stream). No LibTorch / torch types cross this boundary.
 *
 * What each entry point replaces in the reference (autonomousvision/ppo.cpp):
 *   ppo_create / ppo_destroy         AgentImpl ctor + optim::Adam ctor + storage zeros
 *                                    (ppo_continuous_action.cpp:338-364, ac_ppo_continuous_action.cpp:542-596)
 *   ppo_load_params / ppo_save_params  torch::save(agent) / parameter broadcast source (ppo:173-180, ac:551-553)
 *   ppo_get_action_and_value         Agent::get_action_and_value (ppo:145-157, ac:212-249) + Normal/Beta
 *                                    (include/rl_utils.h:20-132)
 *   ppo_get_value                    Agent::get_value (ppo:140-143, ac:188-192)
 *   ppo_rollout_act                  one rollout step's agent half: obs/dones/actions/logprobs/values stores
 *                                    (ppo:387-400, ac:649-660) for envs [env_begin, env_end)
 *   ppo_rollout_reward               rewards[step] store (ppo:406, ac:668)
 *   ppo_compute_gae                  next_value + GAE(lambda) + returns (ppo:447-467, ac:759-779)
 *   ppo_rollout_values               the rollout's deferred critic pass (ac:655 values[step])
 *   ppo_update                       epochs x minibatches: randperm, gather, loss, backward, grad all-reduce,
 *                                    clip_grad_norm_, Adam (ppo:489-542, ac:803-889)
 *   ppo_comm_*                       torchfort::Comm (include/distributed.h:41-60, src/distributed.cpp:81-224)
 *                                    re-designed as one RCCL communicator over xGMI
 */
#ifndef PPO_HIP_H
#define PPO_HIP_H

#include <stddef.h>
#include <stdint.h>

#include "ppo_layout.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ppo_ctx ppo_t;

typedef struct ppo_hip_config {
  int net_kind;         /* PPO_NET_TANH_NORMAL (ppo_continuous_action) / PPO_NET_LN_BETA (ac_ppo_...) */
  int obs_dim, act_dim; /* environment observation / action space */
  int hidden;           /* 64 (PPO agent) or 256 (AC agent) */
  int num_envs;         /* envs on THIS device (num_envs_per_device, ac:399) */
  int num_steps;        /* T (rollout length) */
  int num_minibatches;  /* minibatch_per_device = T*num_envs / num_minibatches (ac:407) */
  int update_epochs;
  float gamma, gae_lambda;
  float clip_coef, ent_coef, vf_coef, max_grad_norm, adam_eps;
  int norm_adv, clip_vloss;
  uint64_t seed;        /* Philox key for action sampling and minibatch permutations */
  int rank, world_size; /* data-parallel position (envs sharded per rank, ac:398-407) */
} ppo_hip_config;

typedef struct ppo_update_stats {
  float pg_loss, v_loss, entropy, old_approx_kl, approx_kl, clipfrac; /* last minibatch; clipfrac = mean */
  float grad_norm;    /* total norm of the last minibatch (pre-clip) */
  int minibatches;
} ppo_update_stats;

/* sample types for ppo_get_action_and_value (ac:225-238) */
enum { PPO_SAMPLE = 0, PPO_MEAN = 1, PPO_GIVEN = 2 };

/* storage buffers, all [T, E, *] row-major fp32 (ppo:357-364) */
enum { PPO_BUF_OBS = 0, PPO_BUF_ACTIONS, PPO_BUF_LOGPROBS, PPO_BUF_REWARDS, PPO_BUF_DONES, PPO_BUF_VALUES,
       PPO_BUF_ADVANTAGES, PPO_BUF_RETURNS, PPO_BUF_COUNT };

const char* ppo_last_error(void);
const char* ppo_version(void);
/* 0 if exactly one HIP runtime (libamdhip64) is mapped in the process; otherwise an error naming
 * them (a second one appears when a PyTorch-ROCm wheel is imported AFTER libppo_hip.so is loaded)
 * and an exit guard that ends the process with status 70 instead of a corrupted-heap abort at exit.
 * ppo_create / ppo_set_device / ppo_dev_malloc run this check first. */
int ppo_runtime_check(void);

/* The AC agent's fixed observation normalisation for env_id (AgentImpl mean_ / std_; reference
 * ac_ppo_continuous_action.cpp Humanoid-v4 :496-497, Ant-v5 :521-522, Hopper-v5 :533-534).
 * HalfCheetah-v5 uses zeros / ones (:510-511): returns 0 with *n = 0. Unknown env id: error.
 * The arrays are static (owned by the library). */
int ppo_obs_norm(const char* env_id, const float** mean, const float** std, int* n);

int ppo_create(const ppo_hip_config* cfg, int device, ppo_t** out);
/* ppo_create with kernel-selection options, "key=value" pairs separated by ',' (NULL or "": the
 * defaults ppo_create uses). Every choice is a complete, tested kernel path; results differ only in
 * summation order (A/B comparisons, tests). Split-bf16 forms: every fp32 operand x is the exact sum
 * of three bf16 pieces (hi = x truncated to bf16, mid = (x - hi) truncated, lo = the rest), so an
 * fp32 product is the sum of nine exact piece products, accumulated in fp32 on the bf16 MFMA (16x
 * the fp32 MFMA rate). The default forms keep six of the nine (the dropped mid*lo + lo*mid + lo*lo are
 * < ~2^-21 |ab|) with fp32 accumulation: tested within 1.5x of the fp32 MFMA form's distance from the
 * fp64 oracle, and not bitwise equal to the fp32 MFMA form (upd_mfma=16,dw_mfma=f32 selects it):
 *   upd_kernel=auto|fwdbwd   minibatch forward/backward: the feature-split k_upd / k_upd2 (auto) or
 *                            the wave-per-16-rows k_fwdbwd
 *   act_kernel=auto|2|4      64-wide agent act: by shape (auto), k_act2, or k_act4
 *   dw_fused=1|0             dW1 / dW2 in one pass (k_dwf) or two (k_dw)
 *   dw_dma=1|0               k_dwf's rows staged by LDS DMA in three buffers (k_dwf_dma, default)
 *                            or through registers in two (k_dwf); bitwise the same
 *   dw_mfma=auto|f32|bf16x9|bf16x8|bf16x6  the fused dW's products as split-bf16 piece products on
 *                            32x32x16 bf16 MFMAs (k_dwf_bx: all 9; 8 without lo*lo < 2^-30 |ab|; 6
 *                            without mid*lo + lo*mid + lo*lo < 2^-21 |ab|, auto) or on fp32 MFMAs
 *                            (k_dwf_dma, f32); not bitwise the fp32 path (rounding of the bf16 MFMA's
 *                            internal sums)
 *   dw_rows=<n>, dw_slices=1|2  dW split-K geometry: rows per chunk (multiple of 16; 32 for the
 *                            64-wide agent) and k_dwf output slices; default: automatic
 *   update_graph=auto|0|1  ppo_update's minibatch launches eager or replayed as one (auto: the graph for
 *                            minibatches of at most 4 096 rows, where launch overhead shows, e.g. cfg1; eager
 *                            once the context has taken a snapshot: the CLIs read snapshots from a writer thread)
 *                            hipGraph captured on the second call (one process, gradstep=split,
 *                            no profiling); the Adam step constants come from a device table, so
 *                            the result is bitwise the eager one. Checkpoint snapshots work with it
 *                            (ppo_read_snapshot waits on the host, never across streams)
 *   upd2_split=auto|0|2|3    64-wide agent with wide inputs (O % 4 == 0, OP = 384: Humanoid): layer 1
 *                            of both trunks as one gathered GEMM (k_l1g) and k_upd2's tail in its own
 *                            launch at 2 / 3 workgroups per CU, or the single k_upd2 (0; auto: the
 *                            single kernel, measured faster)
 *   upd_mfma=auto|bx6|16|32|mix  LayerNorm-Beta agent at hidden 256: the fused minibatch kernel
 *                            with its 256-wide GEMMs (layer 2, dh1 = W2^T dz2) as six split-bf16
 *                            piece products per fp32 product on 16x16x32 bf16 MFMAs (k_upd bx6;
 *                            auto where it applies: at most 16 heads; the dropped mid*lo + lo*mid +
 *                            lo*lo are < 2^-21 |ab|), on 16x16x4 fp32 MFMAs (k_upd, 16), on 32x32x2
 *                            (k_upd32), or mixed (critic trunk 32x32x2, actor 16x16x4); the same
 *                            results up to summation order
 *   rollout=auto|per_step    ppo_rollout_synth: persistent launch where supported, or per step
 *   rollout_kernel=auto|mfma|valu  the AC agent's persistent rollout: k_rollout (16 envs per
 *                            workgroup, MFMA) or k_rollout_v (2 envs per workgroup, VALU; O <= 32);
 *                            auto: k_rollout_v at E <= 512. Bitwise the same results. valu on an
 *                            agent it cannot serve (the PPO agent, O > 32, device env wrappers) fails
 *   gae=auto|serial|scan     GAE as the reference's serial recurrence per env (k_gae: bit-exact with
 *                            ppo:447-467, ac:759-779) or as a segmented scan over the steps (k_gae_scan: 16
 *                            segments per 64 envs, within 1e-5 of the serial form and of the golden
 *                            vectors); auto: the scan from 512 steps (cfg1 / cfg2's T = 2 048), serial below
 *   upd_split=auto|1|2|4|8   the minibatch's fused update (k_upd + k_dwf; hidden 256, obs_dim <= 32) as
 *                            n launch pairs over consecutive M / n rows of its permutation: one pair's
 *                            hand-off rows (H1 / DZ1 / DZ2 / Xn, ~6 KB per row) stay cache-resident
 *                            between k_upd's stores and k_dwf's reads; the pairs' partial sums are added
 *                            together (the same gradient up to summation order); auto = 1 (measured slower)
 *   h1_handoff=auto|store|recompute  the H1 rows of k_upd's hand-off: stored by k_upd (store, auto) or
 *                            recomputed inside the fused split-bf16 dW from Xn, W1 and 8 bytes of LayerNorm
 *                            statistics per row (recompute: bitwise the stored rows; measured slower overall)
 *   values_mfma=auto|bx6|f32 the rollout's critic pass (values of the stored rows and the bootstrap,
 *                            ac:655 / :761): k_vbx, layer 2 as k_upd's six split-bf16 piece products
 *                            (bx6; auto where upd_mfma=bx6 applies: the per-step act kernels then skip
 *                            the critic and one batched pass runs before GAE) or the fp32 MFMA
 *                            k_values / per-step critic (f32)
 *   gradstep=split|fused     clip_grad_norm_ + Adam: two launches (k_gradnorm, k_adam; default) or
 *                            one cooperative launch (k_gradstep: slower on ROCm 7, whose cooperative
 *                            launch costs ~30 us); bitwise the same as gradstep=split,gradnorm=slices
 *   gradnorm=auto|fold|slices  clip_grad_norm_'s per-tensor sums of squares: folded into k_colsum (fold:
 *                            per-tile sums, each tensor's last tile adds them in tile order; one launch
 *                            fewer per minibatch, but measured slower) or k_gradnorm's 16 slices per tensor (slices; auto). Fold needs one
 *                            rank (with an all-reduce between the column sums and the norm, or
 *                            gradstep=fused, k_gradnorm runs). Deterministic either way; the two differ in
 *                            the summation order of the squares only
 * An unknown key or value is an error, and so is an option the agent cannot use (upd_mfma=32 / mix /
 * bx6 off the LayerNorm-Beta agent, upd2_split > 0 off the 64-wide Humanoid shape): such a create
 * fails and releases everything it had allocated. */
int ppo_create_ex(const ppo_hip_config* cfg, int device, const char* options, ppo_t** out);
int ppo_destroy(ppo_t* ctx);
int ppo_get_layout(const ppo_t* ctx, ppo_layout* out);
void* ppo_stream(ppo_t* ctx);

/* parameters in the reference's flat named_parameters() order (ppo_layout.h); loading also
 * resets the Adam state (fresh optimizer, as after the reference's ctor). */
int ppo_load_params(ppo_t* ctx, const float* host, long n);
int ppo_save_params(ppo_t* ctx, float* host, long n);
/* Adam state in the same flat order (exp_avg, exp_avg_sq) and its step count */
int ppo_save_adam(ppo_t* ctx, float* m_host, float* v_host, long n, long* step);
int ppo_load_adam(ppo_t* ctx, const float* m_host, const float* v_host, long n, long step);

int ppo_get_action_and_value(ppo_t* ctx, int n, const float* x_dev, int sample_type,
                             const float* action_in_dev, long env_base, long step_id,
                             float* action_dev, float* logprob_dev, float* entropy_dev, float* value_dev,
                             void* stream);
int ppo_get_value(ppo_t* ctx, int n, const float* x_dev, float* value_dev, void* stream);

/* rollout step `step` for envs [env_begin, env_end): stores obs/dones, samples actions with the
 * Philox key (seed, rank, env, iteration*T + step), writes actions into storage and (if non-NULL)
 * into action_out_dev[e - env_begin]. Several host threads may call it concurrently on distinct
 * env ranges and streams (AC-PPO async collection, ac:641-698). The value of each row (ac:655,
 * `values[step] = value`) is stored either here or, for the LayerNorm-Beta agent with the split-bf16
 * critic pass (create option values_mfma, default where upd_mfma=bx6 applies), by one batched critic
 * launch over the stored observations that ppo_compute_gae / ppo_gae_from_values / ppo_update run
 * first (the persistent rollout's kernel: both collection paths store the same values bit for bit);
 * ppo_rollout_values runs that pass now. */
int ppo_rollout_act(ppo_t* ctx, int step, int env_begin, int env_end, const float* next_obs_dev,
                    const float* next_done_dev, float* action_out_dev, void* stream);
/* the deferred critic pass of ppo_rollout_act (values[t] for every step acted since the last pass),
 * on `stream` after the act launches; a no-op when nothing is pending (ac:655). */
int ppo_rollout_values(ppo_t* ctx, void* stream);
int ppo_rollout_reward(ppo_t* ctx, int step, int env_begin, int env_end, const float* reward_dev, void* stream);
/* GAE over steps [0, num_steps_collected) using next_obs/next_done after the last step (ac:759-779).
 * num_steps_collected < num_steps (DD-PPO preemption): the last collected step is bootstrapped from
 * the stored step num_steps_collected (values / dones), as the reference's loop does; next_obs and
 * next_done are then unused. */
int ppo_compute_gae(ppo_t* ctx, const float* next_obs_dev, const float* next_done_dev, int num_steps_collected,
                    void* stream);
/* GAE with a caller-supplied bootstrap value next_value[E] (skips the critic call). */
int ppo_gae_from_values(ppo_t* ctx, const float* next_value_dev, const float* next_done_dev, int num_steps_collected,
                        void* stream);
/* Runs update_epochs x num_minibatches optimizer steps with learning rate lr. Asynchronous on the
 * context stream; stats (if non-NULL) are copied back after a stream sync. Advances the iteration
 * counter used by the rollout RNG. perms_dev (optional, int32 [epochs][T*E]) overrides the
 * Philox/Feistel minibatch permutation (tests inject the reference's randperm). */
int ppo_update(ppo_t* ctx, float lr, const int32_t* perms_dev, ppo_update_stats* stats);
/* ppo_update over a partial collection (DD-PPO preemption, ac:803-810): the first
 * num_steps_collected steps of every env are the samples; each epoch's permutation runs over those
 * num_steps_collected * E samples and is repeated and truncated to T * E (b_inds.repeat(...)[:B]),
 * so the minibatch count and size are those of a full collection. GAE for such a collection:
 * ppo_compute_gae with the same step count, which bootstraps from the stored step
 * num_steps_collected as the reference does (ac:765-774). ppo_update = ppo_update_ex(..., T, ...). */
int ppo_update_ex(ppo_t* ctx, float lr, int num_steps_collected, const int32_t* perms_dev, ppo_update_stats* stats);
int ppo_sync(ppo_t* ctx);
/* test hook: raw (pre-clip, post all-reduce) gradient of the last minibatch, flat reference order */
int ppo_debug_last_grad(ppo_t* ctx, float* host, long n);
/* Asynchronous checkpoint source (the reference saves agent + optimizer every iteration inside its
 * SPS span, ppo:545-563 / ac:904-927): ppo_snapshot_state enqueues a device-side copy of the
 * parameters and the Adam state on the context stream (ordered after the last update, before the
 * next) and returns at once; ppo_read_snapshot, callable from another host thread, waits (on the
 * host, hipEventSynchronize) for that copy only and unpacks it in the flat reference order — no
 * cross-stream dependency, so it is safe while the context stream is being captured into a hipGraph
 * (update_graph=1). One snapshot buffer: call
 * ppo_read_snapshot before the next ppo_snapshot_state. */
int ppo_snapshot_state(ppo_t* ctx);
int ppo_read_snapshot(ppo_t* ctx, float* params_host, float* m_host, float* v_host, long n, long* step);
long ppo_iteration(const ppo_t* ctx);
int ppo_set_iteration(ppo_t* ctx, long iteration);
float* ppo_buffer(ppo_t* ctx, int which);

/* ---- data-parallel communicator (RCCL over xGMI) ---- */
#define PPO_COMM_ID_BYTES 128
int ppo_comm_unique_id(char id_out[PPO_COMM_ID_BYTES]);
/* attaches an RCCL communicator for (rank, world) to the context (world = 1 included: a one-rank
 * group runs the distributed sequence). While one is attached, ppo_update computes the advantage
 * statistics over the group (mean averaged, sum of squares summed, Bessel over world * M;
 * ac:830-849), averages the flat gradient before clip_grad_norm_ (ac:877-885) and averages the
 * logged stats (ac:895-901). A context created with world_size > 1 refuses ppo_update until a
 * communicator is attached. */
int ppo_comm_init(ppo_t* ctx, const char id[PPO_COMM_ID_BYTES], int rank, int world);
/* Host-transport communicator: the same sequence with every all-reduce handed to fn in host memory
 * (in place over n floats; average != 0: mean over ranks, else sum; return 0 on success) — the
 * reference Comm's MPI path for CPU tensors (distributed.cpp:134-148). Lets MPI / gloo callers
 * drive the data-parallel update without RCCL. */
typedef int (*ppo_host_allreduce_fn)(float* host_buf, long n, int average, void* user);
int ppo_comm_init_host(ppo_t* ctx, int rank, int world, ppo_host_allreduce_fn fn, void* user);
int ppo_comm_destroy(ppo_t* ctx);
/* comm->broadcast of every parameter from root (ac:551-553) */
int ppo_comm_broadcast_params(ppo_t* ctx, int root);
int ppo_comm_allreduce(ppo_t* ctx, float* buf_dev, long n, int average);
/* The attached communicator as its transport sees it: kind 0 = none, 1 = RCCL (rank and world
 * from ncclCommUserRank / ncclCommCount), 2 = host transport. comm->rank / comm->size
 * (distributed.cpp:66-79). */
enum { PPO_COMM_NONE = 0, PPO_COMM_RCCL = 1, PPO_COMM_HOST = 2 };
int ppo_comm_info(const ppo_t* ctx, int* kind, int* rank, int* world);
/* The HIP device the context lives on (the `device` of ppo_create, the reference's
 * cudaSetDevice(gpu_ids.at(local_rank)), ac:447-448 / :459-460) and that device's PCI bus id
 * (hipDeviceGetPCIBusId, e.g. "0000:05:00.0"; pass NULL / 0 to skip). Launchers compare the bus ids
 * of all ranks: two ranks on one GPU is an error under RCCL. */
int ppo_get_device(const ppo_t* ctx, int* device, char* pci_bus_id, int len);
/* The kernels the context selected for its update (create options and shape; no reference
 * counterpart — a report for benchmarks and logs), as "update=<kernel>[/<form>] dw=<kernel>[/<form>]",
 * e.g. "update=k_upd/bx6 dw=k_dwf_dma/f32" (bx6: k_upd's 256-wide GEMMs as split-bf16 piece
 * products, upd_mfma). NUL-terminated, truncated to len. */
int ppo_kernel_info(const ppo_t* ctx, char* buf, int len);

/* ---- device memory helpers (so C / ctypes callers need no HIP headers) ---- */
int ppo_set_device(int device);
int ppo_device_count(int* n);
int ppo_dev_malloc(void** p, size_t bytes);
int ppo_dev_free(void* p);
int ppo_memcpy_h2d(void* dst_dev, const void* src_host, size_t bytes);
int ppo_memcpy_d2h(void* dst_host, const void* src_dev, size_t bytes);
int ppo_memset_dev(void* dst_dev, int value, size_t bytes);
int ppo_device_sync(void);

/* ---- profiling hooks: per-kernel HIP-event timing of the context's launches ---- */
int ppo_profile_enable(ppo_t* ctx, int on);
/* returns (into host arrays of length cap) accumulated ms and launch counts per kernel id; names
 * via ppo_profile_name(). Returns the number of kernel ids. */
int ppo_profile_read(ppo_t* ctx, double* ms, long* count, int cap);
const char* ppo_profile_name(int id);
int ppo_profile_reset(ppo_t* ctx);

#ifdef __cplusplus
}
#endif
#endif /* PPO_HIP_H */
