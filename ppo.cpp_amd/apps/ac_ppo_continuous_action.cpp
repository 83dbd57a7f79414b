// ac_ppo_continuous_action — drop-in for the reference executable of the same name
// (src/ac_ppo_continuous_action.cpp): same flags and defaults, one process per GPU, envs sharded
// per rank (num_envs_per_device = num_envs / world_size, ac:398-407), gradients averaged over ranks
// every minibatch — here with one RCCL communicator (replacing torchfort::Comm's MPI + NCCL) inside
// ppo_update.
//
// Asynchronous collection (ac:641-698): the reference runs one host thread + one CUDA stream +
// batch-1 inference per env. Here the per-device envs are split into --num_collect_groups groups;
// each group has a host thread and a HIP stream and runs the batched act kernel for its env slice,
// copies the actions back, steps its envs on the CPU and copies obs/reward/done up — so the GPU
// inference of one group overlaps the CPU env stepping of the others. Per-env trajectories are
// identical to the reference's per-env threads (counter-based Philox sampling is independent of
// grouping). --env_backend device runs the device-resident synthetic env instead (no PCIe).
// --num_collect_groups 0 (default) = two groups per host thread, so one group's GPU round trip hides
// under another's CPU stepping; --host_step_us gives the host env a per-step CPU cost (the MuJoCo
// physics it stands in for), and each group's env stepping is a roctx range ("host_env_step"), so a
// rocprofv3 --kernel-trace --marker-trace timeline shows the act kernels under the stepping.
//
// DD-PPO preemption (--use_dd_ppo_preempt 1, ac:568-583, :629, :680-693, :803-810): rank 0 serves the
// TCP store (apps/tcp_store.h), every collection group has a client; a group stops collecting once
// more than dd_ppo_preempt_threshold of all groups (over all ranks) are done and it is past
// dd_ppo_min_perc of the steps. A group stands in for the reference's per-env thread: the store
// counts finished groups. The update trains on the minimum step count over the groups, its
// permutations repeated and truncated to the full batch (ppo_update_ex).
//
// Launch: one process per GPU with RANK / WORLD_SIZE / LOCAL_RANK (torchrun or any launcher) or
// OMPI_COMM_WORLD_{RANK,SIZE,LOCAL_RANK} (mpirun); the RCCL id is exchanged through --rdzv_file.
#include "trainer_common.h"
#include "tcp_store.h"

#include <rocprofiler-sdk-roctx/roctx.h>

#include <atomic>
#include <iomanip>
#include <thread>

using namespace app;
namespace fs = std::filesystem;

struct GlobalConfig {  // ac_ppo_continuous_action.cpp:55-148
  int seed = 1;
  int eval_seed = 2;
  unsigned total_timesteps = 10'000'000;
  float learning_rate = 2.5e-4f;
  unsigned num_envs = 8;
  unsigned num_steps = 128;
  float gamma = 0.99f;
  float gae_lambda = 0.95f;
  unsigned num_minibatches = 4;
  unsigned update_epochs = 4;
  bool norm_adv = true;
  float clip_coef = 0.1f;
  bool clip_vloss = true;
  float ent_coef = 0.01f;
  float vf_coef = 0.5f;
  float max_grad_norm = 0.5f;
  float adam_eps = 1e-5f;
  bool anneal_lr = true;
  unsigned num_eval_runs = 128;
  bool clip_actions = true;
  bool torch_deterministic = true;
  std::string exp_name_stem = "Ant-v5_AC_PPO_Atari";
  std::string env_id = "Ant-v5";
  std::string render = "rgb_array";
  std::vector<int> gpu_ids = {0};
  std::string collect_device = "cpu";
  std::string train_device = "cpu";
  std::string rdzv_addr = "localhost";
  int tcp_store_port = 29500;
  int use_dd_ppo_preempt = 0;
  float dd_ppo_min_perc = 0.25f;
  float dd_ppo_preempt_threshold = 0.6f;
  bool estimate_mean_std = false;
  // MI355X build additions
  std::string env_backend = "host";  // host | device
  int num_collect_groups = 0;        // 0: two per host thread
  float host_step_us = 0.0f;         // host env: CPU time per env step (busy wait)
  float straggler_us = 0.0f;         // host env: extra CPU time per env step for the last group (test knob)
  std::string rdzv_file = "";
  unsigned num_devices = 1, num_envs_per_device = 0, batch_size = 0, minibatch_size = 0, num_iterations = 0;
  unsigned batch_size_per_device = 0, minibatch_per_device = 0;
  std::string exp_name;
};

static int env_int(const char* a, const char* b, int def) {
  if (const char* v = std::getenv(a)) return std::atoi(v);
  if (const char* v = std::getenv(b)) return std::atoi(v);
  return def;
}

int main(int argc, const char** argv) {
  std::ios_base::sync_with_stdio(false);
  const auto process_start = std::filesystem::file_time_type::clock::now();
  const int rank = env_int("RANK", "OMPI_COMM_WORLD_RANK", 0);
  const int world_size = env_int("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", 1);
  const int local_rank = env_int("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", rank);

  GlobalConfig config;
  Flags flags;
  flags.add("seed", "Training seed", &config.seed);
  flags.add("eval_seed", "Seed of final evaluation run", &config.eval_seed);
  flags.add("total_timesteps", "Number of environment steps", &config.total_timesteps);
  flags.add("learning_rate", "Adam learning rate", &config.learning_rate);
  flags.add("num_steps", "Num environment steps per iteration", &config.num_steps);
  flags.add("gamma", "Discount factor", &config.gamma);
  flags.add("gae_lambda", "Lambda of generalized advantage estimation", &config.gae_lambda);
  flags.add("num_minibatches", "Number of training iterations per epoch", &config.num_minibatches);
  flags.add("update_epochs", "Number of training epochs per iteration", &config.update_epochs);
  flags.add("norm_adv", "Whether to normalize the advantage", &config.norm_adv);
  flags.add("clip_coef", "PPO clip coefficient", &config.clip_coef);
  flags.add("clip_vloss", "Whether to apply clipping to the value loss", &config.clip_vloss);
  flags.add("ent_coef", "Weigth of entropy loss.", &config.ent_coef);
  flags.add("vf_coef", "Weigth of value loss.", &config.vf_coef);
  flags.add("max_grad_norm", "Factor for gradient clipping.", &config.max_grad_norm);
  flags.add("adam_eps", "Epsilon of adam.", &config.adam_eps);
  flags.add("anneal_lr", "Whether to anneal the learning rate linearly.", &config.anneal_lr);
  flags.add("num_eval_runs", "How many environments to evaluate", &config.num_eval_runs);
  flags.add("clip_actions", "Whether to clip action into the valid range.", &config.clip_actions);
  flags.add("torch_deterministic", "Whether to use deterministic algorithms (always deterministic here)",
            &config.torch_deterministic);
  flags.add("exp_name_stem", "Name of the experiment.", &config.exp_name_stem);
  flags.add("env_id", "Name of the env to be executed.", &config.env_id);
  flags.add("render", "rgb_array (human rendering needs MuJoCo/GLFW)", &config.render);
  flags.add("num_envs", "Number of environments to be used.", &config.num_envs);
  flags.add_list("gpu_ids", "The ids of the GPUs used for training. Usage: --gpu_ids 0 --gpu_ids 1 ...", &config.gpu_ids);
  flags.add("collect_device", "Whether to collect data on gpu or cpu. Options: cpu, gpu", &config.collect_device);
  flags.add("train_device", "Whether to train on gpu or cpu. Options: cpu, gpu", &config.train_device);
  flags.add("rdzv_addr", "IP adress of master node. Default: localhost", &config.rdzv_addr);
  flags.add("tcp_store_port", "Port for the TCP store. Default: 29500", &config.tcp_store_port);
  flags.add("use_dd_ppo_preempt", "Flag to toggle the dd_ppo pre-emption trick", &config.use_dd_ppo_preempt);
  flags.add("dd_ppo_min_perc", "Percentage of envs that need to finish before preemtion.", &config.dd_ppo_min_perc);
  flags.add("dd_ppo_preempt_threshold", "Percentage of envs that need to finish before preemtion.",
            &config.dd_ppo_preempt_threshold);
  flags.add("estimate_mean_std", "Print the mean / std of env 0's observations at the end", &config.estimate_mean_std);
  flags.add("env_backend", "host (gymcpp envs on the CPU) or device (synthetic env in HBM)", &config.env_backend);
  flags.add("num_collect_groups", "host envs: number of async collection groups (threads + HIP streams); 0: two "
            "per host thread", &config.num_collect_groups);
  flags.add("host_step_us", "host envs: CPU time burnt per env step (stands in for the physics)", &config.host_step_us);
  flags.add("straggler_us", "host envs: extra CPU time per env step in the last collection group", &config.straggler_us);
  flags.add("rdzv_file", "file used to exchange the RCCL id between ranks", &config.rdzv_file);
  try {
    flags.parse(argc, argv);
  } catch (const HelpRequested&) {
    flags.print_help(std::cout);
    return 0;
  } catch (const ParseError& e) {
    std::cerr << e.what() << std::endl;
    flags.print_help(std::cerr);
    return 1;
  }
  if (config.use_dd_ppo_preempt && config.env_backend == "device") {
    std::cerr << "use_dd_ppo_preempt needs host envs (--env_backend host): the device rollout has no per-env "
                 "collection threads to preempt\n";
    return 1;
  }
  // derived fields (ac:398-407)
  config.num_devices = world_size;
  config.num_envs_per_device = config.num_envs / config.num_devices;
  if (config.num_envs % config.num_devices != 0) {
    std::cerr << "num_envs must be a multiple of num_devices.\n";
    return 1;
  }
  config.exp_name = config.exp_name_stem + "_" + std::to_string(config.seed);
  config.batch_size = config.num_steps * config.num_envs;
  config.minibatch_size = config.batch_size / config.num_minibatches;
  config.num_iterations = config.total_timesteps / config.batch_size;
  config.batch_size_per_device = config.batch_size / config.num_devices;
  config.minibatch_per_device = config.minibatch_size / config.num_devices;
  std::cout << "world_size: " << world_size << "\nrank: " << rank << "\nlocal_rank: " << local_rank << std::endl;
  if (config.collect_device != "cpu" && config.collect_device != "gpu") {
    std::cerr << "Unsupported Collect device selected. Options: cpu, gpu. Selected Device: " << config.collect_device << std::endl;
    return 2;
  }
  if (config.train_device != "cpu" && config.train_device != "gpu") {
    std::cerr << "Unsupported train device selected. Options: cpu, gpu. Selected device: " << config.train_device << std::endl;
    return 3;
  }
  // The agent always runs on the MI355X (the reference's cpu options exist for LibTorch CPU runs).
  // gpu_ids.at(local_rank) as the reference indexes it (ac:447-448 / :459-460): a list shorter than
  // the local rank count is an error, never a silent wrap onto another rank's GPU
  if ((size_t)local_rank >= config.gpu_ids.size()) {
    std::cerr << "local rank " << local_rank << " has no entry in --gpu_ids (" << config.gpu_ids.size()
              << " given): pass one --gpu_ids per local rank\n";
    return 2;
  }
  const int device = config.gpu_ids.at((size_t)local_rank);

  const fs::path exe = fs::canonical(argv[0]);
  const fs::path exp_folder = exe.parent_path() / ".." / "models" / config.exp_name;
  fs::create_directories(exp_folder);
  RunLog logger(exp_folder, "tfevents_logs_" + std::to_string(rank) + ".pb", "scalars_" + std::to_string(rank) + ".jsonl");

  const int E = (int)config.num_envs_per_device, T = (int)config.num_steps;
  const bool device_env = config.env_backend == "device";
  // DD-PPO store (ac:568-573): rank 0 serves it from before the communicator exists, so the other
  // ranks' clients (created once every rank has joined) always find it
  std::unique_ptr<TCPStoreServer> store_server;
  if (config.use_dd_ppo_preempt && rank == 0) {
    store_server = std::make_unique<TCPStoreServer>(config.rdzv_addr, config.tcp_store_port, (int)config.num_envs);
    store_server->start();
  }
  int O = 17, A = 6;
  float act_lo = -1.f, act_hi = 1.f;
  std::vector<std::shared_ptr<gymcpp::SeqVectorEnv>> envs;  // one SeqVectorEnv per env, as the reference
  if (!device_env) {
    try {
      const int G0 = config.num_collect_groups > 0 ? config.num_collect_groups : 2 * host_threads();
      const int Gs = std::max(1, std::min(G0, E));
      for (int i = 0; i < E; ++i) {
        auto base = make_base_env(config.env_id);
        // the last collection group (envs [E (G-1) / G, E)) carries the straggler cost
        const float us = config.host_step_us + (i >= (long)E * (Gs - 1) / Gs ? config.straggler_us : 0.0f);
        if (us > 0.0f) {
          auto sc = std::dynamic_pointer_cast<gymcpp::SyntheticCheetah>(base);
          if (!sc) throw std::invalid_argument("host_step_us / straggler_us apply to SyntheticCheetah-v0 only");
          sc->set_step_cost_ns((int64_t)std::llround(us * 1000.0));
        }
        std::vector<std::shared_ptr<gymcpp::EnvironmentWrapper>> arr{
            std::make_shared<gymcpp::RecordEpisodeStatistics>(base)};
        envs.push_back(std::make_shared<gymcpp::SeqVectorEnv>(arr, config.clip_actions));
      }
    } catch (const std::invalid_argument& e) {
      std::cerr << e.what() << std::endl;
      return 1;
    }
    O = envs[0]->get_observation_space();
    A = envs[0]->get_action_space();
    act_lo = envs[0]->get_action_space_min();
    act_hi = envs[0]->get_action_space_max();
  } else {
    EnvShape sh;
    if (!device_env_shape(config.env_id, &sh)) {
      std::cerr << "env_backend device: unknown env_id " << config.env_id
                << " (HalfCheetah-v5, Humanoid-v4, Ant-v5, Hopper-v5, SyntheticCheetah-v0)\n";
      return 1;
    }
    O = sh.O; A = sh.A; act_lo = sh.lo; act_hi = sh.hi;
  }

  ppo_hip_config hc{};
  hc.net_kind = PPO_NET_LN_BETA; hc.obs_dim = O; hc.act_dim = A; hc.hidden = 256;
  hc.num_envs = E; hc.num_steps = T; hc.num_minibatches = (int)config.num_minibatches;
  hc.update_epochs = (int)config.update_epochs; hc.gamma = config.gamma; hc.gae_lambda = config.gae_lambda;
  hc.clip_coef = config.clip_coef; hc.ent_coef = config.ent_coef; hc.vf_coef = config.vf_coef;
  hc.max_grad_norm = config.max_grad_norm; hc.adam_eps = config.adam_eps; hc.norm_adv = config.norm_adv;
  hc.clip_vloss = config.clip_vloss; hc.seed = (uint64_t)config.seed; hc.rank = rank; hc.world_size = world_size;
  ppo_t* agent = nullptr;
  psyn_t* denv = nullptr;
  try {
    check(ppo_create(&hc, device, &agent), "ppo_create");
    ppo_layout L;
    check(ppo_get_layout(agent, &L), "ppo_get_layout");
    std::vector<float> obs_mean, obs_std;  // per-env-id constants (ac:480-534)
    {
      const float *m = nullptr, *sd = nullptr;
      int n = 0;
      if (ppo_obs_norm(config.env_id.c_str(), &m, &sd, &n) == 0 && n == O) {
        obs_mean.assign(m, m + n);
        obs_std.assign(sd, sd + n);
      }
    }
    auto p0 = init_params(L, config.seed, act_hi, act_lo, obs_mean, obs_std);
    check(ppo_load_params(agent, p0.data(), L.P), "ppo_load_params");
    if (world_size > 1) {  // ncclUniqueId exchange through a file (no MPI in this build)
      // The file carries a per-launch key (PPO_RUN_ID / TORCHELASTIC_RUN_ID / the MPI job id, when
      // the launcher sets one) and must be newer than this process: a file left behind by an
      // earlier launch on the same port is never taken for this one's. Rank 0 removes it once the
      // communicator is up (ncclCommInitRank returns only after every rank has joined).
      const std::string path = config.rdzv_file.empty()
                                   ? "/tmp/ppo_rdzv_" + std::to_string(config.tcp_store_port) + ".id"
                                   : config.rdzv_file;
      std::string key;
      for (const char* v : {"PPO_RUN_ID", "TORCHELASTIC_RUN_ID", "OMPI_MCA_ess_base_jobid", "SLURM_JOB_ID"})
        if (const char* e = getenv(v)) { key = e; break; }
      // torchrun keeps the run id across elastic restarts: the attempt number makes the key per attempt
      if (const char* rc = getenv("TORCHELASTIC_RESTART_COUNT")) key += std::string("#") + rc;
      char id[PPO_COMM_ID_BYTES];
      if (rank == 0) {
        std::error_code rm_ec;
        fs::remove(path, rm_ec);  // a file a crashed earlier attempt left behind is never read again
        check(ppo_comm_unique_id(id), "ppo_comm_unique_id");
        {
          std::ofstream f(path + ".tmp", std::ios::binary | std::ios::trunc);
          const uint32_t kl = (uint32_t)key.size();
          f.write(reinterpret_cast<const char*>(&kl), sizeof(kl));
          f.write(key.data(), kl);
          f.write(id, PPO_COMM_ID_BYTES);
        }
        fs::rename(path + ".tmp", path);
      } else {
        const auto not_before = process_start - std::chrono::seconds(30);
        for (int tries = 0;; ++tries) {
          if (tries > 6000) throw std::runtime_error("timed out waiting for " + path + " (rank 0's communicator id)");
          std::error_code ec;
          if (fs::exists(path, ec) && fs::last_write_time(path, ec) >= not_before && !ec) {
            std::ifstream f(path, std::ios::binary);
            uint32_t kl = 0;
            std::string k;
            if (f.read(reinterpret_cast<char*>(&kl), sizeof(kl)) && kl < 4096) {
              k.resize(kl);
              if (f.read(k.data(), kl) && k == key && f.read(id, PPO_COMM_ID_BYTES)) break;
            }
          }
          std::this_thread::sleep_for(std::chrono::milliseconds(10));
        }
      }
      check(ppo_comm_init(agent, id, rank, world_size), "ppo_comm_init");
      if (rank == 0) {
        std::error_code ec;
        fs::remove(path, ec);
      }
      check(ppo_comm_broadcast_params(agent, 0), "ppo_comm_broadcast_params");  // ac:551-553
    }
    if (rank == 0) std::cout << "Number of parameters in model: " << (L.P - L.train_begin) << std::endl;

    hipStream_t s = (hipStream_t)ppo_stream(agent);
    float *d_obs, *d_done, *d_act, *d_rew;
    HIPCHECK(hipMalloc(&d_obs, sizeof(float) * E * O));
    HIPCHECK(hipMalloc(&d_done, sizeof(float) * E));
    HIPCHECK(hipMalloc(&d_act, sizeof(float) * E * A));
    HIPCHECK(hipMalloc(&d_rew, sizeof(float) * E));
    HIPCHECK(hipMemset(d_done, 0, sizeof(float) * E));
    float *h_obs = nullptr, *h_act = nullptr, *h_rew = nullptr, *h_done = nullptr;
    const int G = std::max(1, std::min(config.num_collect_groups > 0 ? config.num_collect_groups : 2 * host_threads(), E));
    if (!device_env && rank == 0)
      std::cout << "collection groups: " << G << " (" << host_threads() << " host threads)" << std::endl;
    std::vector<std::unique_ptr<TCPStoreClient>> store_clients;  // one per group (ac:576-582: one per env thread)
    if (config.use_dd_ppo_preempt)
      for (int gi = 0; gi < G; ++gi)
        store_clients.push_back(std::make_unique<TCPStoreClient>(config.rdzv_addr, config.tcp_store_port));
    const long dd_min_steps = std::lround(config.dd_ppo_min_perc * static_cast<float>(config.num_steps));
    const int dd_groups = G * world_size;  // every rank runs G groups
    std::vector<float> obs_mean_std;       // env 0's observations (ac:663, estimate_mean_std)
    std::vector<hipStream_t> gstreams(G);
    if (device_env) {
      check(psyn_create(E, O, A, &denv), "psyn_create");
      check(psyn_set_action_space(denv, act_lo, act_hi), "psyn_set_action_space");
      check(psyn_reset(denv, config.seed, d_obs, d_done, s), "psyn_reset");  // env i: seed + i on every rank (ac:606)
    } else {
      HIPCHECK(hipHostMalloc(&h_obs, sizeof(float) * E * O));
      HIPCHECK(hipHostMalloc(&h_act, sizeof(float) * E * A));
      HIPCHECK(hipHostMalloc(&h_rew, sizeof(float) * E));
      HIPCHECK(hipHostMalloc(&h_done, sizeof(float) * E));
      for (int i = 0; i < E; ++i) {  // env i reset with seed + i (ac:606)
        const float* o = envs[i]->reset(config.seed + i);
        std::copy(o, o + O, h_obs + (size_t)i * O);
      }
      HIPCHECK(hipMemcpy(d_obs, h_obs, sizeof(float) * E * O, hipMemcpyHostToDevice));
      for (auto& gs : gstreams) HIPCHECK(hipStreamCreateWithFlags(&gs, hipStreamNonBlocking));
    }
    HIPCHECK(hipDeviceSynchronize());

    long global_step = 0;
    float* d_stats = nullptr;  // episode sums all-reduced over ranks (ac:700-727)
    HIPCHECK(hipMalloc(&d_stats, sizeof(float) * 3));
    AsyncCheckpointer ckpt(agent);
    const auto start_time = std::chrono::high_resolution_clock::now();
    ppo_update_stats st{};
    double last_lr = config.learning_rate;  // the optimizer's lr at save time
    for (unsigned iteration = 0; iteration < config.num_iterations; ++iteration) {
      float lrnow = config.learning_rate;
      if (config.anneal_lr) {  // ac:634-639
        const float frac = 1.0f - static_cast<float>(iteration) / static_cast<float>(config.num_iterations);
        lrnow = frac * config.learning_rate;
      }
      double sum_r = 0, sum_l = 0, n_ep = 0;
      int steps_collected = T;  // min over the collection groups (ac:703-707, :723)
      if (config.use_dd_ppo_preempt) {
        if (rank == 0) store_clients[0]->reset();  // ac:628-630
        if (world_size > 1) {  // comm->allreduce(sychronize) (ac:631): every rank starts after the reset
          HIPCHECK(hipMemsetAsync(d_stats, 0, sizeof(float), s));
          check(ppo_comm_allreduce(agent, d_stats, 1, 0), "ppo_comm_allreduce");
          HIPCHECK(hipStreamSynchronize(s));
        }
      }
      if (device_env) {
        check(ppo_rollout_synth(agent, denv, d_obs, d_done, d_act, d_rew), "ppo_rollout_synth");
        if (config.estimate_mean_std) {  // env 0's next observation after every step: obs[1..T-1][0], next_obs[0]
          const float* sobs = ppo_buffer(agent, PPO_BUF_OBS);
          std::vector<float> o((size_t)T * O);
          for (int t = 1; t < T; ++t)
            HIPCHECK(hipMemcpyAsync(o.data() + (size_t)(t - 1) * O, sobs + (size_t)t * E * O, sizeof(float) * O,
                                    hipMemcpyDeviceToHost, s));
          HIPCHECK(hipMemcpyAsync(o.data() + (size_t)(T - 1) * O, d_obs, sizeof(float) * O, hipMemcpyDeviceToHost, s));
          HIPCHECK(hipStreamSynchronize(s));
          obs_mean_std.insert(obs_mean_std.end(), o.begin(), o.end());
        }
        // episode sums read out behind the rollout, without a device-wide sync; collected after
        // the update has been enqueued (the values are those of this rollout)
        check(psyn_episode_stats_begin(denv, s), "psyn_episode_stats_begin");
      } else {
        // asynchronous collection: one host thread + HIP stream per env group
        std::vector<std::thread> th;
        std::vector<double> gr(G, 0), gl(G, 0), gn(G, 0);
        std::vector<int> gsteps(G, T);
        std::atomic<int> failed{0};
        for (int gi = 0; gi < G; ++gi) {
          th.emplace_back([&, gi] {
            const int e0 = E * gi / G, e1 = E * (gi + 1) / G, n = e1 - e0;
            hipStream_t gs = gstreams[gi];
            try {
              int step;
              for (step = 0; step < T; ++step) {
                check(ppo_rollout_act(agent, step, e0, e1, d_obs + (size_t)e0 * O, d_done + e0, d_act + (size_t)e0 * A, gs),
                      "ppo_rollout_act");
                HIPCHECK(hipMemcpyAsync(h_act + (size_t)e0 * A, d_act + (size_t)e0 * A, sizeof(float) * n * A,
                                        hipMemcpyDeviceToHost, gs));
                HIPCHECK(hipStreamSynchronize(gs));
                roctxRangePushA("host_env_step");
                for (int i = e0; i < e1; ++i) {
                  gymcpp::VecStep r = envs[i]->step(h_act + (size_t)i * A);
                  if (i == 0 && config.estimate_mean_std) obs_mean_std.insert(obs_mean_std.end(), r.obs, r.obs + O);
                  std::copy(r.obs, r.obs + O, h_obs + (size_t)i * O);
                  h_rew[i] = r.rewards[0];
                  h_done[i] = (r.terminations[0] != 0.f || r.truncations[0] != 0.f) ? 1.f : 0.f;
                  if ((*r.infos)[0].has_value()) {
                    gr[gi] += (*r.infos)[0]->r;
                    gl[gi] += (*r.infos)[0]->l;
                    gn[gi] += 1;
                  }
                }
                roctxRangePop();
                HIPCHECK(hipMemcpyAsync(d_rew + e0, h_rew + e0, sizeof(float) * n, hipMemcpyHostToDevice, gs));
                check(ppo_rollout_reward(agent, step, e0, e1, d_rew + e0, gs), "ppo_rollout_reward");
                HIPCHECK(hipMemcpyAsync(d_obs + (size_t)e0 * O, h_obs + (size_t)e0 * O, sizeof(float) * n * O,
                                        hipMemcpyHostToDevice, gs));
                HIPCHECK(hipMemcpyAsync(d_done + e0, h_done + e0, sizeof(float) * n, hipMemcpyHostToDevice, gs));
                if (config.use_dd_ppo_preempt) {  // ac:680-689 (the step just taken is stored, not trained on)
                  const int num_done = store_clients[gi]->get();
                  if (static_cast<float>(num_done) / static_cast<float>(dd_groups) > config.dd_ppo_preempt_threshold &&
                      step > dd_min_steps)
                    break;
                }
              }
              HIPCHECK(hipStreamSynchronize(gs));
              if (config.use_dd_ppo_preempt) store_clients[gi]->increment();  // ac:692-694
              gsteps[gi] = step;
            } catch (const std::exception& e) {
              std::cerr << e.what() << std::endl;
              failed = 1;
            }
          });
        }
        for (auto& t : th) t.join();
        if (failed) throw std::runtime_error("collection failed");
        for (int gi = 0; gi < G; ++gi) {
          sum_r += gr[gi]; sum_l += gl[gi]; n_ep += gn[gi];
          steps_collected = std::min(steps_collected, gsteps[gi]);
        }
        if (steps_collected < T)
          std::cout << "dd_ppo: rank " << rank << " trains on " << steps_collected << " of " << T
                    << " steps per env (preempted)" << std::endl;
      }
      check(ppo_compute_gae(agent, d_obs, d_done, steps_collected, s), "ppo_compute_gae");
      // a preempted collection: the permutations over the collected samples, repeated to the batch (ac:803-810)
      check(ppo_update_ex(agent, lrnow, steps_collected, nullptr, &st), "ppo_update");  // stats rank-averaged inside
      if (device_env) {
        float r, l, n;
        check(psyn_episode_stats_end(denv, &r, &l, &n), "psyn_episode_stats_end");
        sum_r = r; sum_l = l; n_ep = n;
      }
      global_step += (long)config.num_envs * config.num_steps;  // ac:730
      // episode statistics summed over ranks (ac:700-727), through the RCCL communicator
      float h_stats[3] = {(float)sum_r, (float)sum_l, (float)n_ep};
      if (world_size > 1) {
        HIPCHECK(hipMemcpyAsync(d_stats, h_stats, sizeof(h_stats), hipMemcpyHostToDevice, s));
        check(ppo_comm_allreduce(agent, d_stats, 3, 0), "ppo_comm_allreduce");
        HIPCHECK(hipMemcpyAsync(h_stats, d_stats, sizeof(h_stats), hipMemcpyDeviceToHost, s));
        HIPCHECK(hipStreamSynchronize(s));
      }
      if (rank == 0 && h_stats[2] > 0) {
        const float avg_return = h_stats[0] / h_stats[2], avg_length = h_stats[1] / h_stats[2];
        logger.add_scalar("charts/episodic_return", global_step, avg_return);
        logger.add_scalar("charts/episodic_length", global_step, avg_length);
        std::cout << "global_step=" << global_step << ", avg_episodic_return=" << std::fixed << std::setprecision(2)
                  << avg_return << " \n";
        logger.add_scalar("charts/episodic_return_per_sec", std::lround(seconds_since(start_time)), avg_return);
      }
      if (rank == 0) {
        char mf[64], of[64];
        std::snprintf(mf, sizeof mf, "model_latest_%09u.pth", iteration);
        std::snprintf(of, sizeof of, "optimizer_latest_%09u.pth", iteration);
        ckpt.request(exp_folder, mf, of, lrnow, config.adam_eps, iteration);  // written while the GPU runs on
        last_lr = lrnow;
        const double secs = seconds_since(start_time);
        float sps = 0.f;
        if (secs > 0) {
          sps = (float)(global_step / secs);
          std::cout << std::fixed << std::setprecision(0) << "SPS: " << sps << std::endl;
        }
        logger.add_scalar("charts/learning_rate", global_step, lrnow);
        logger.add_scalar("losses/value_loss", global_step, st.v_loss);
        logger.add_scalar("losses/policy_loss", global_step, st.pg_loss);
        logger.add_scalar("losses/entropy", global_step, st.entropy);
        logger.add_scalar("losses/old_approx_kl", global_step, st.old_approx_kl);
        logger.add_scalar("losses/approx_kl", global_step, st.approx_kl);
        logger.add_scalar("losses/clipfrac", global_step, st.clipfrac);
        logger.add_scalar("charts/SPS", global_step, sps);
      }
      std::cout << std::flush;
    }
    ckpt.finish();
    if (rank == 0) save_state(agent, exp_folder, "model_final.pth", "optimizer_final.pth", last_lr, config.adam_eps);
    if (config.estimate_mean_std && !obs_mean_std.empty()) {  // ac:954-963: mean and population std of env 0's obs
      const size_t n = obs_mean_std.size() / O;
      std::vector<double> mu(O, 0.0), var(O, 0.0);
      for (size_t k = 0; k < n; ++k)
        for (int f = 0; f < O; ++f) mu[f] += obs_mean_std[k * O + f];
      for (int f = 0; f < O; ++f) mu[f] /= (double)n;
      for (size_t k = 0; k < n; ++k)
        for (int f = 0; f < O; ++f) {
          const double d = obs_mean_std[k * O + f] - mu[f];
          var[f] += d * d;
        }
      std::cout << "Mean obs:\n";
      for (int f = 0; f < O; ++f) std::cout << std::setprecision(6) << " " << (float)mu[f] << "\n";
      std::cout << "[ CPUFloatType{" << O << "} ]\n\nStd obs:\n";
      for (int f = 0; f < O; ++f) std::cout << " " << (float)std::sqrt(var[f] / (double)n) << "\n";
      std::cout << "[ CPUFloatType{" << O << "} ]\n" << std::endl;
    }
    // rank 0 evaluation with the Beta mean action on env 0 (ac:965-1001)
    if (rank == 0 && !device_env) {
      std::vector<float> episodic_returns;
      const float* o = envs[0]->reset(config.eval_seed);
      std::copy(o, o + O, h_obs);
      long guard = 0;
      while (episodic_returns.size() < config.num_eval_runs && guard++ < 100000000L) {
        HIPCHECK(hipMemcpy(d_obs, h_obs, sizeof(float) * O, hipMemcpyHostToDevice));
        check(ppo_get_action_and_value(agent, 1, d_obs, PPO_MEAN, nullptr, 0, 0, d_act, nullptr, nullptr, nullptr, s),
              "ppo_get_action_and_value");
        HIPCHECK(hipStreamSynchronize(s));
        HIPCHECK(hipMemcpy(h_act, d_act, sizeof(float) * A, hipMemcpyDeviceToHost));
        gymcpp::VecStep r = envs[0]->step(h_act);
        std::copy(r.obs, r.obs + O, h_obs);
        if ((*r.infos)[0].has_value()) {
          std::cout << "Evaluation result: episode=" << episodic_returns.size() << " episodic_return=" << std::fixed
                    << std::setprecision(2) << (*r.infos)[0]->r << " \n";
          episodic_returns.push_back((*r.infos)[0]->r);
        }
      }
      for (size_t i = 0; i < episodic_returns.size(); ++i) logger.add_scalar("eval/episodic_return", (long)i, episodic_returns[i]);
      double avg = 0;
      for (float x : episodic_returns) avg += x;
      avg /= std::max<size_t>(1, episodic_returns.size());
      logger.add_scalar("eval/avg_return", (long)episodic_returns.size(), avg);
      std::cout << "Average evaluation return=" << std::fixed << std::setprecision(2) << avg << " over "
                << episodic_returns.size() << " episodes" << std::endl;
    }
    for (auto gs : gstreams)
      if (gs) (void)hipStreamDestroy(gs);
    if (denv) psyn_destroy(denv);
    (void)hipFree(d_stats);
    (void)hipFree(d_obs); (void)hipFree(d_done); (void)hipFree(d_act); (void)hipFree(d_rew);
    if (h_obs) { (void)hipHostFree(h_obs); (void)hipHostFree(h_act); (void)hipHostFree(h_rew); (void)hipHostFree(h_done); }
    ppo_destroy(agent);
  } catch (const std::exception& e) {
    std::cerr << e.what() << std::endl;
    if (denv) psyn_destroy(denv);
    if (agent) ppo_destroy(agent);
    return 6;
  }
  return 0;
}
