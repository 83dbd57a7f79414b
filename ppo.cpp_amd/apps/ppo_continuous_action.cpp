// ppo_continuous_action — drop-in for the reference executable of the same name
// (src/ppo_continuous_action.cpp): same flags, defaults, stdout lines and per-iteration flow
// (lr anneal -> rollout -> GAE -> epochs x minibatches -> checkpoint -> SPS/log), with the agent,
// GAE and the whole update running as gfx950 kernels behind include/ppo_hip.h. The envs stay on
// the host behind the gymcpp interface (ParVectorEnv + the reference's wrapper chain, ppo:41-49),
// or, with --env_backend device, are the synthetic device env at the env id's shapes with the same
// wrapper chain on the device (include/ppo_env_wrappers.h): nothing crosses PCIe per step.
#include "trainer_common.h"

#include <algorithm>
#include <iomanip>

using namespace app;
namespace fs = std::filesystem;

struct GlobalConfig {  // ppo_continuous_action.cpp:51-118
  int seed = 1;
  int eval_seed = 2;
  int total_timesteps = 1'000'000;
  float learning_rate = 3e-4f;
  int num_envs = 1;
  int num_steps = 2048;
  float gamma = 0.99f;
  float gae_lambda = 0.95f;
  int num_minibatches = 32;
  int update_epochs = 10;
  bool norm_adv = true;
  float clip_coef = 0.2f;
  bool clip_vloss = true;
  float ent_coef = 0.0f;
  float vf_coef = 0.5f;
  float max_grad_norm = 0.5f;
  float adam_eps = 1e-5f;
  bool anneal_lr = true;
  int num_eval_runs = 10;
  bool clip_actions = true;
  bool torch_deterministic = true;
  std::string exp_name_stem = "PPO_002";
  std::string env_id = "Humanoid-v4";
  std::string render = "rgb_array";
  int device = 0;
  std::string env_backend = "host";
  std::string exp_name;
  int batch_size = 0, minibatch_size = 0, num_iterations = 0;
  void derive() {  // ppo:268-272
    exp_name = exp_name_stem + "_" + std::to_string(seed);
    batch_size = num_steps * num_envs;
    minibatch_size = batch_size / num_minibatches;
    num_iterations = total_timesteps / batch_size;
  }
};

int main(int argc, const char** argv) {
  std::ios_base::sync_with_stdio(false);
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
  flags.add("num_envs", "Number of environments to be used.", &config.num_envs);
  flags.add("render", "Set to human for Visualizing the training with OpenGL, rgb_array for no visualization",
            &config.render);
  flags.add("device", "HIP device index", &config.device);
  flags.add("env_backend", "host (gymcpp envs on the CPU) or device (synthetic env + wrapper chain in HBM)",
            &config.env_backend);
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
  config.derive();
  if (config.num_iterations <= 0)
    std::cerr << "warning: total_timesteps / (num_steps * num_envs) = 0 iterations; pass --total_timesteps explicitly\n";

  const fs::path exe = fs::canonical(argv[0]);
  const fs::path exp_folder = exe.parent_path() / ".." / "models" / config.exp_name;
  fs::create_directories(exp_folder);
  RunLog logger(exp_folder, "tfevents_logs.pb", "scalars.jsonl");

  const bool device_env = config.env_backend == "device";
  if (!device_env && config.env_backend != "host") {
    std::cerr << "env_backend must be host or device\n";
    return 1;
  }
  std::vector<std::shared_ptr<gymcpp::EnvironmentWrapper>> env_array;
  EnvShape sh{0, 0, -1.0f, 1.0f};
  if (device_env) {
    if (!device_env_shape(config.env_id, &sh)) {
      std::cerr << "env_backend device: unknown env_id " << config.env_id
                << " (HalfCheetah-v5, Humanoid-v4, Ant-v5, Hopper-v5, SyntheticCheetah-v0)\n";
      return 1;
    }
  } else {
    try {
      for (int i = 0; i < config.num_envs; ++i) env_array.push_back(gymcpp::make_env(make_base_env(config.env_id), config.gamma));
    } catch (const std::invalid_argument& e) {
      std::cerr << e.what() << std::endl;
      return 1;
    }
    sh = {env_array[0]->get_observation_space(), env_array[0]->get_action_space(),
          env_array[0]->get_action_space_min(), env_array[0]->get_action_space_max()};
  }
  const int O = sh.O, A = sh.A;
  const int E = config.num_envs, T = config.num_steps;

  ppo_hip_config hc{};
  hc.net_kind = PPO_NET_TANH_NORMAL; hc.obs_dim = O; hc.act_dim = A; hc.hidden = 64;
  hc.num_envs = E; hc.num_steps = T; hc.num_minibatches = config.num_minibatches; hc.update_epochs = config.update_epochs;
  hc.gamma = config.gamma; hc.gae_lambda = config.gae_lambda; hc.clip_coef = config.clip_coef;
  hc.ent_coef = config.ent_coef; hc.vf_coef = config.vf_coef; hc.max_grad_norm = config.max_grad_norm;
  hc.adam_eps = config.adam_eps; hc.norm_adv = config.norm_adv; hc.clip_vloss = config.clip_vloss;
  hc.seed = (uint64_t)config.seed; hc.rank = 0; hc.world_size = 1;
  ppo_t* agent = nullptr;
  psyn_t* denv = nullptr;
  pwrap_t* dwrap = nullptr;
  try {
    check(ppo_create(&hc, config.device, &agent), "ppo_create");
    ppo_layout L;
    check(ppo_get_layout(agent, &L), "ppo_get_layout");
    auto p0 = init_params(L, config.seed, sh.hi, sh.lo, {}, {});
    check(ppo_load_params(agent, p0.data(), L.P), "ppo_load_params");
    std::cout << "Number of parameters in model: " << (L.P - L.train_begin) << std::endl;

    std::shared_ptr<gymcpp::ParVectorEnv> envs;
    if (!device_env) envs = std::make_shared<gymcpp::ParVectorEnv>(env_array, config.clip_actions);
    float *d_obs, *d_done, *d_act, *d_rew;
    HIPCHECK(hipMalloc(&d_obs, sizeof(float) * E * O));
    HIPCHECK(hipMalloc(&d_done, sizeof(float) * E));
    HIPCHECK(hipMalloc(&d_act, sizeof(float) * E * A));
    HIPCHECK(hipMalloc(&d_rew, sizeof(float) * E));
    float *h_act, *h_done;
    HIPCHECK(hipHostMalloc(&h_act, sizeof(float) * E * A));
    HIPCHECK(hipHostMalloc(&h_done, sizeof(float) * E));
    hipStream_t s = (hipStream_t)ppo_stream(agent);

    if (device_env) {  // ParVectorEnv(make_env(...)) on the device: synthetic env + the ppo:41-49 chain
      check(psyn_create(E, O, A, &denv), "psyn_create");
      if (config.clip_actions) check(psyn_set_action_space(denv, sh.lo, sh.hi), "psyn_set_action_space");
      else check(psyn_set_action_space(denv, -3.0e38f, 3.0e38f), "psyn_set_action_space");
      check(pwrap_create(E, O, config.gamma, &dwrap), "pwrap_create");
      check(psyn_attach_wrappers(denv, dwrap), "psyn_attach_wrappers");
      check(psyn_reset(denv, config.seed, d_obs, d_done, s), "psyn_reset");
    } else {
      const float* obs0 = envs->reset(config.seed);
      HIPCHECK(hipMemcpyAsync(d_obs, obs0, sizeof(float) * E * O, hipMemcpyHostToDevice, s));
      HIPCHECK(hipMemsetAsync(d_done, 0, sizeof(float) * E, s));
    }

    long global_step = 0;
    AsyncCheckpointer ckpt(agent);
    const auto start_time = std::chrono::high_resolution_clock::now();
    ppo_update_stats st{};
    double last_lr = config.learning_rate;  // the optimizer's lr at save time
    for (int iteration = 0; iteration < config.num_iterations; ++iteration) {
      float lrnow = config.learning_rate;
      if (config.anneal_lr) {  // ppo:379-384
        const float frac = 1.0f - static_cast<float>(iteration) / static_cast<float>(config.num_iterations);
        lrnow = frac * config.learning_rate;
      }
      double env_time = 0;
      if (device_env) {  // T x {act, env step + wrappers, reward store} on the device (ppo:387-434)
        global_step += (long)E * T;
        check(ppo_rollout_synth(agent, denv, d_obs, d_done, d_act, d_rew), "ppo_rollout_synth");
        check(psyn_episode_stats_begin(denv, s), "psyn_episode_stats_begin");
      }
      for (int step = 0; step < T && !device_env; ++step) {
        global_step += E;
        check(ppo_rollout_act(agent, step, 0, E, d_obs, d_done, d_act, s), "ppo_rollout_act");
        HIPCHECK(hipMemcpyAsync(h_act, d_act, sizeof(float) * E * A, hipMemcpyDeviceToHost, s));
        HIPCHECK(hipStreamSynchronize(s));
        const auto t0 = std::chrono::high_resolution_clock::now();
        gymcpp::VecStep r = envs->step(h_act);
        env_time += seconds_since(t0);
        for (int e = 0; e < E; ++e) h_done[e] = (r.terminations[e] != 0.f || r.truncations[e] != 0.f) ? 1.f : 0.f;
        HIPCHECK(hipMemcpyAsync(d_rew, r.rewards, sizeof(float) * E, hipMemcpyHostToDevice, s));
        check(ppo_rollout_reward(agent, step, 0, E, d_rew, s), "ppo_rollout_reward");
        HIPCHECK(hipMemcpyAsync(d_obs, r.obs, sizeof(float) * E * O, hipMemcpyHostToDevice, s));
        HIPCHECK(hipMemcpyAsync(d_done, h_done, sizeof(float) * E, hipMemcpyHostToDevice, s));
        HIPCHECK(hipStreamSynchronize(s));  // host env buffers are reused by the next step
        float total_reward = 0.f;
        int total_length = 0, finished = 0;
        for (const auto& info : *r.infos)
          if (info.has_value()) {
            std::cout << "global_step=" << global_step << ", episodic_return=" << std::fixed << std::setprecision(2)
                      << info->r << " \n";
            total_reward += info->r;
            total_length += info->l;
            ++finished;
          }
        if (finished > 0) {
          logger.add_scalar("charts/episodic_return", global_step, total_reward / finished);
          logger.add_scalar("charts/episodic_length", global_step, (float)total_length / finished);
          logger.add_scalar("charts/episodic_return_per_sec", std::lround(seconds_since(start_time)), total_reward / finished);
        }
      }
      std::cout << std::fixed << std::setprecision(6) << "Total env step time " << env_time << " seconds \n";
      check(ppo_compute_gae(agent, d_obs, d_done, T, s), "ppo_compute_gae");
      check(ppo_update(agent, lrnow, nullptr, &st), "ppo_update");
      if (device_env) {  // finished episodes of this rollout (raw returns: RecordEpisodeStatistics is innermost)
        float sr = 0.f, sl = 0.f, n = 0.f;
        check(psyn_episode_stats_end(denv, &sr, &sl, &n), "psyn_episode_stats_end");
        if (n > 0) {
          std::cout << "global_step=" << global_step << ", episodic_return=" << std::fixed << std::setprecision(2)
                    << sr / n << " (mean of " << (long)n << " episodes)\n";
          logger.add_scalar("charts/episodic_return", global_step, sr / n);
          logger.add_scalar("charts/episodic_length", global_step, sl / n);
          logger.add_scalar("charts/episodic_return_per_sec", std::lround(seconds_since(start_time)), sr / n);
        }
      }
      char mf[64], of[64];
      std::snprintf(mf, sizeof mf, "model_latest_%09d.pth", iteration);
      std::snprintf(of, sizeof of, "optimizer_latest_%09d.pth", iteration);
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
    ckpt.finish();
    save_state(agent, exp_folder, "model_final.pth", "optimizer_final.pth", last_lr, config.adam_eps);
    // final evaluation on the training envs (normalisation statistics live there, ppo:589-626)
    if (device_env) {
      check(psyn_reset(denv, config.eval_seed, d_obs, d_done, s), "psyn_reset");
      float sr0, sl0, n0;
      check(psyn_episode_stats(denv, &sr0, &sl0, &n0), "psyn_episode_stats");  // clears the sums
      double sum_r = 0, n_ep = 0;
      long eval_step = 0;
      while (n_ep < config.num_eval_runs && eval_step < 100000000L) {
        check(ppo_get_action_and_value(agent, E, d_obs, PPO_SAMPLE, nullptr, 0, (1L << 40) + eval_step++, d_act,
                                       nullptr, nullptr, nullptr, s), "ppo_get_action_and_value");
        check(psyn_step(denv, 0, E, d_act, config.clip_actions ? sh.lo : -3.0e38f, config.clip_actions ? sh.hi : 3.0e38f,
                        d_obs, d_rew, d_done, s), "psyn_step");
        if (eval_step % 50 == 0) {
          float sr, sl, n;
          check(psyn_episode_stats(denv, &sr, &sl, &n), "psyn_episode_stats");
          sum_r += sr;
          n_ep += n;
        }
      }
      const double avg = n_ep > 0 ? sum_r / n_ep : 0.0;
      logger.add_scalar("eval/avg_return", (long)n_ep, avg);
      std::cout << "Average evaluation return=" << std::fixed << std::setprecision(2) << avg << " over " << (long)n_ep
                << " episodes" << std::endl;
    }
    const float* eobs = device_env ? nullptr : envs->reset(config.eval_seed);
    if (!device_env) {
    HIPCHECK(hipMemcpyAsync(d_obs, eobs, sizeof(float) * E * O, hipMemcpyHostToDevice, s));
    std::vector<float> episodic_returns;
    long eval_step = 0;
    while ((int)episodic_returns.size() < config.num_eval_runs) {
      check(ppo_get_action_and_value(agent, E, d_obs, PPO_SAMPLE, nullptr, 0, (1L << 40) + eval_step++, d_act, nullptr,
                                     nullptr, nullptr, s), "ppo_get_action_and_value");
      HIPCHECK(hipMemcpyAsync(h_act, d_act, sizeof(float) * E * A, hipMemcpyDeviceToHost, s));
      HIPCHECK(hipStreamSynchronize(s));
      gymcpp::VecStep r = envs->step(h_act);
      HIPCHECK(hipMemcpyAsync(d_obs, r.obs, sizeof(float) * E * O, hipMemcpyHostToDevice, s));
      HIPCHECK(hipStreamSynchronize(s));
      for (const auto& info : *r.infos)
        if (info.has_value()) {
          std::cout << "Evaluation result: episode=" << episodic_returns.size() << " episodic_return=" << std::fixed
                    << std::setprecision(2) << info->r << " \n";
          episodic_returns.push_back(info->r);
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
    if (denv) psyn_destroy(denv);
    if (dwrap) pwrap_destroy(dwrap);
    (void)hipFree(d_obs); (void)hipFree(d_done); (void)hipFree(d_act); (void)hipFree(d_rew);
    (void)hipHostFree(h_act); (void)hipHostFree(h_done);
    ppo_destroy(agent);
  } catch (const std::exception& e) {
    std::cerr << e.what() << std::endl;
    if (denv) psyn_destroy(denv);
    if (dwrap) pwrap_destroy(dwrap);
    if (agent) ppo_destroy(agent);
    return 2;
  }
  return 0;
}
