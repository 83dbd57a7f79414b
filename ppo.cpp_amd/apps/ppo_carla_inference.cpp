// apps/ppo_carla_inference.cpp — drop-in of src/carla/ppo_carla_inference.cpp: serves CaRL driving
// actions to eval_agent.py (CARLA leaderboard) from an ensemble of trained model_*.pth files.
//
// Same flags (--path_to_conf_file, --ipc_path, --port; all required), same protocol on a PAIR socket
// bound at ipc://<ipc_path>/<port>.lock (net/zmtp.h speaks ZMTP 3.0 to pyzmq):
//   send "Connected to eval_agent.py."; receive the sample type ("sample" | "mean" | "roach");
//   per step: receive a keepalive ("" = one more observation, anything else = route finished, exit 0),
//   then the 3-part observation [bev uint8 C x H x W | measurements f32[NM] | value_measurements f32[NV]],
//   answer 4 frames [action f32[A] | value f32 | mu f32[A] | sigma f32[A]], each the ensemble mean
//   over the models (ppo_carla_inference.cpp:163-194).
// Exit codes as the reference: 1 handshake failed, 2 no model file, 3 connection interrupted.
// The agent is the repo's CaRL forward on the GPU (include/ppo_carla.h: implicit-GEMM MFMA
// convolutions, Beta head); model files are read by the LibTorch-compatible reader (ppo_pth.h).
// Sampling per model i uses the Philox contract with seed config.seed + i (the reference seeds a
// CUDA generator with seed + i, ppo_carla_inference.cpp:118-126), step counter = query index.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <iostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/ppo_carla.h"
#include "../../include/ppo_hip.h"
#include "../../include/ppo_pth.h"
#include "../net/zmtp.h"
#include "json_flat.h"
#include "trainer_common.h"

using namespace app;

int main(int argc, const char** argv) {
  std::ios_base::sync_with_stdio(false);
  std::string path_to_conf_file, ipc_path;
  int port = -1;
  Flags flags;
  flags.add("path_to_conf_file", "Path to the folder containing model weights and config.json.", &path_to_conf_file);
  flags.add("ipc_path", "Path to folder that is used to sync inter process communication.", &ipc_path);
  flags.add("port", "Port to connect to eval_agent.py with.", &port);
  try {
    flags.parse(argc, argv);
    if (path_to_conf_file.empty() || ipc_path.empty() || port < 0) throw ParseError("Option 'path_to_conf_file', 'ipc_path' and 'port' are required");
  } catch (const HelpRequested&) {
    flags.print_help(std::cout);
    throw std::runtime_error("Display help.");
  } catch (const ParseError& e) {
    std::cerr << e.what() << std::endl;
    flags.print_help(std::cerr);
    throw std::runtime_error("Could not parse arguments.");
  }

  // config.json next to the models (carla_config.h update_from_json): the fields the agent needs
  const std::filesystem::path model_folder(path_to_conf_file);
  const FlatJson cfg = FlatJson::parse_file((model_folder / "config.json").string());
  if (cfg.get_string("image_encoder", "roach") != "roach")
    throw std::runtime_error("ppo_carla_inference: only the 'roach' image encoder is built (carla_model.h:65-127)");
  ppo_carla_config cc;
  std::memset(&cc, 0, sizeof(cc));
  cc.obs_channels = cfg.get_int("obs_num_channels", 15);
  cc.bev_h = cfg.get_int("bev_semantics_height", 192);
  cc.bev_w = cfg.get_int("bev_semantics_width", 192);
  cc.num_measurements = cfg.get_int("obs_num_measurements", 8);
  cc.num_value_measurements = cfg.get_int("num_value_measurements", 3);
  cc.action_dim = 2;  // CarlaEnv::action_space_
  cc.beta_min = cfg.get_float("beta_min_a_b_value", 1.0f);
  cc.max_batch = 1;
  const int seed = cfg.get_int("seed", 1);

  zmtp::Socket socket(zmtp::Type::PAIR);
  std::filesystem::create_directories(ipc_path);
  socket.bind("ipc://" + (std::filesystem::path(ipc_path) / (std::to_string(port) + ".lock")).string());
  socket.send(std::string("Connected to eval_agent.py."));
  std::cout << "Connecting to eval_agent.py, port: " << port << std::endl;
  zmtp::Message answer;
  if (!socket.recv(answer) || answer.empty()) {
    std::cerr << "Establishing connected to eval_agent.py failed." << std::endl;
    return 1;
  }
  std::cout << "Connected to eval_agent.py, port: " << port << std::endl;
  std::cout << "Deterministic actions: " << answer[0] << std::endl;
  const std::string sample_type = answer[0];
  int mode;
  if (sample_type == "sample") mode = PPO_CARLA_SAMPLE;
  else if (sample_type == "mean") mode = PPO_CARLA_MEAN;
  else if (sample_type == "roach") mode = PPO_CARLA_ROACH;
  else throw std::runtime_error("Unsupported sample type used. Sample type: " + sample_type);

  HIPCHECK(hipSetDevice(0));
  std::vector<ppo_carla_t*> agents;
  ppo_carla_layout L;
  for (const auto& entry : std::filesystem::recursive_directory_iterator(model_folder)) {
    const std::string fn = entry.path().filename().string();
    if (fn.rfind("model", 0) == 0 && fn.size() >= 4 && fn.compare(fn.size() - 4, 4, ".pth") == 0) {
      ppo_carla_config ci = cc;
      ci.seed = (uint64_t)(seed + (int)agents.size());
      ppo_carla_t* a = nullptr;
      check(ppo_carla_create(&ci, 0, &a), "ppo_carla_create");
      check(ppo_carla_get_layout(a, &L), "ppo_carla_get_layout");
      std::vector<float> p(L.P);
      check(ppo_carla_pth_load(&L, entry.path().string().c_str(), p.data(), L.P), "torch::load of the model");
      check(ppo_carla_load_params(a, p.data(), L.P), "ppo_carla_load_params");
      agents.push_back(a);
    }
  }
  if (agents.empty()) {
    std::cerr << "No model file was found in the selected path:" << model_folder.string() << std::endl;
    return 2;
  }

  const int A = cc.action_dim, NM = cc.num_measurements, NV = cc.num_value_measurements;
  const size_t nb = (size_t)cc.obs_channels * cc.bev_h * cc.bev_w;
  uint8_t* d_bev = nullptr;
  float *d_meas = nullptr, *d_vmeas = nullptr, *d_out = nullptr;
  HIPCHECK(hipMalloc(&d_bev, nb));
  HIPCHECK(hipMalloc(&d_meas, sizeof(float) * std::max(NM, 1)));
  HIPCHECK(hipMalloc(&d_vmeas, sizeof(float) * std::max(NV, 1)));
  HIPCHECK(hipMalloc(&d_out, sizeof(float) * (3 * A + 1) * agents.size()));
  std::vector<float> h_out((3 * A + 1) * agents.size());

  long step = 0;
  int rc = 0;
  for (;;) {
    zmtp::Message keepalive;
    if (!socket.recv(keepalive)) {
      std::cerr << "Connection to eval_agent.py interrupted." << std::endl;
      rc = 3;
      break;
    }
    if (!keepalive.empty() && !keepalive[0].empty()) {
      std::cout << "Finished route." << std::endl;
      break;
    }
    zmtp::Message obs;
    if (!socket.recv(obs) || obs.size() < 3 || obs[0].size() < nb || obs[1].size() < 4u * NM || obs[2].size() < 4u * NV) {
      std::cerr << "Connection to eval_agent.py interrupted." << std::endl;
      rc = 3;
      break;
    }
    HIPCHECK(hipMemcpy(d_bev, obs[0].data(), nb, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(d_meas, obs[1].data(), sizeof(float) * NM, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(d_vmeas, obs[2].data(), sizeof(float) * NV, hipMemcpyHostToDevice));
    for (size_t i = 0; i < agents.size(); ++i) {  // per model: action | value | mu | sigma
      float* o = d_out + (3 * A + 1) * i;
      check(ppo_carla_forward(agents[i], 1, d_bev, d_meas, d_vmeas, mode, nullptr, 0, step, o, nullptr, nullptr,
                              o + A, o + A + 1, o + 2 * A + 1, nullptr),
            "ppo_carla_forward");
    }
    // the forwards run on each context's own (non-blocking) stream
    check(ppo_device_sync(), "ppo_device_sync");
    HIPCHECK(hipMemcpy(h_out.data(), d_out, sizeof(float) * h_out.size(), hipMemcpyDeviceToHost));
    // torch::mean(torch::stack(x, 0), 0): sum over the models in order, divided by their count
    std::vector<float> mean(3 * A + 1, 0.f);
    for (size_t i = 0; i < agents.size(); ++i)
      for (int k = 0; k < 3 * A + 1; ++k) mean[k] += h_out[(3 * A + 1) * i + k];
    for (auto& v : mean) v /= (float)agents.size();
    auto part = [&](int off, int n) { return std::string((const char*)(mean.data() + off), sizeof(float) * n); };
    socket.send(zmtp::Message{part(0, A), part(A, 1), part(A + 1, A), part(2 * A + 1, A)});
    ++step;
  }
  for (auto* a : agents) ppo_carla_destroy(a);
  (void)hipFree(d_bev);
  (void)hipFree(d_meas);
  (void)hipFree(d_vmeas);
  (void)hipFree(d_out);
  socket.close();
  return rc;
}
