// Test driver: steps gymcpp::SeqVectorEnv / ParVectorEnv over SyntheticCheetah (+ the wrappers)
// with actions read from a file and writes obs / reward / term / trunc / info per step, so that
// tests/test_host_env.py can compare the host env stack with the oracle bit for bit.
//   host_env_driver <seq|par> E T seed actions.f32 out.f32
// out layout per step: obs[E*O], reward[E], term[E], trunc[E], info_ret[E], info_len[E] (float)
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "../../ppo.cpp_amd/gymcpp/gym.h"
#include "../../ppo.cpp_amd/gymcpp/synthetic_cheetah.h"
#include "../../ppo.cpp_amd/gymcpp/wrappers.h"

template <class V>
static int run(V& venv, int E, int T, int seed, const std::vector<float>& act, FILE* out) {
  const int O = venv.get_observation_space(), A = venv.get_action_space();
  const float* o = venv.reset(seed);
  fwrite(o, sizeof(float), (size_t)E * O, out);
  std::vector<float> ir(E), il(E);
  for (int t = 0; t < T; ++t) {
    gymcpp::VecStep r = venv.step(act.data() + (size_t)t * E * A);
    for (int e = 0; e < E; ++e) {
      const auto& inf = (*r.infos)[e];
      ir[e] = inf ? inf->r : 0.f;
      il[e] = inf ? (float)inf->l : 0.f;
    }
    fwrite(r.obs, sizeof(float), (size_t)E * O, out);
    fwrite(r.rewards, sizeof(float), E, out);
    fwrite(r.terminations, sizeof(float), E, out);
    fwrite(r.truncations, sizeof(float), E, out);
    fwrite(ir.data(), sizeof(float), E, out);
    fwrite(il.data(), sizeof(float), E, out);
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc != 7) return 2;
  const std::string mode = argv[1];
  const int E = std::atoi(argv[2]), T = std::atoi(argv[3]), seed = std::atoi(argv[4]);
  const int A = 6;
  std::vector<float> act((size_t)T * E * A);
  FILE* f = fopen(argv[5], "rb");
  if (!f || fread(act.data(), sizeof(float), act.size(), f) != act.size()) return 3;
  fclose(f);
  std::vector<std::shared_ptr<gymcpp::EnvironmentWrapper>> envs;
  for (int e = 0; e < E; ++e)
    envs.push_back(std::make_shared<gymcpp::RecordEpisodeStatistics>(std::make_shared<gymcpp::SyntheticCheetah>()));
  FILE* out = fopen(argv[6], "wb");
  if (!out) return 4;
  int rc;
  if (mode == "seq") {
    gymcpp::SeqVectorEnv v(envs, true);
    rc = run(v, E, T, seed, act, out);
  } else {
    gymcpp::ParVectorEnv v(envs, true, 4);
    rc = run(v, E, T, seed, act, out);
  }
  fclose(out);
  return rc;
}
