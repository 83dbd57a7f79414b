// apps/zmtp_tool.cpp — host-only driver of the ZMTP layer for tests (tests/test_zmtp.py) and manual
// checks: the reference's DD-PPO store (tcp_store.h) and CaRL env (carla_gym.h) run exactly as the
// trainer uses them, against peers in other processes (the Python side speaks ZMTP on its own).
//   zmtp_tool greeting                                   hex of the greeting and READY commands
//   zmtp_tool store-server <addr> <port> <seconds>       TCPStoreServer for <seconds>
//   zmtp_tool store-client <addr> <port> <ops>           ops: i (increment) r (reset) g (print get())
//                                                        s (sleep 50 ms) w<n> (poll get() until == n)
//   zmtp_tool store-selftest <port> <threads> <rounds>   server + <threads> client threads in-process
//   zmtp_tool carla-env <comm_root> <port> <steps> <C> <H> <W> <NM> <NV> <clip>
//                                                        SeqVectorEnvCarla(RecordEpisodeStatisticsCarla(
//                                                        CarlaEnv)): reset, then <steps> steps with
//                                                        actions a_t = (1.5 sin t, 1.5 cos t); one line
//                                                        per step (reward, term, trunc, obs checksums, info)
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../gymcpp/carla_gym.h"
#include "../net/zmtp.h"
#include "tcp_store.h"

static void hex(const std::string& s) {
  for (unsigned char c : s) std::printf("%02x", c);
  std::printf("\n");
}

static uint64_t fnv(const void* p, size_t n) {
  const unsigned char* b = (const unsigned char*)p;
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: zmtp_tool <greeting|store-server|store-client|store-selftest|carla-env> ...\n");
    return 2;
  }
  const std::string cmd = argv[1];
  try {
    if (cmd == "greeting") {
      hex(zmtp::greeting());
      for (auto t : {zmtp::Type::PAIR, zmtp::Type::REQ, zmtp::Type::REP, zmtp::Type::PUB, zmtp::Type::SUB})
        hex(zmtp::ready_command(t));
      return 0;
    }
    if (cmd == "store-server" && argc >= 5) {
      TCPStoreServer server(argv[2], std::stoi(argv[3]), 64);
      server.start();
      std::printf("ready\n");
      std::fflush(stdout);
      std::this_thread::sleep_for(std::chrono::milliseconds((long)(std::stod(argv[4]) * 1000)));
      return 0;
    }
    if (cmd == "store-client" && argc >= 5) {
      TCPStoreClient client(argv[2], std::stoi(argv[3]));
      for (const char* op = argv[4]; *op; ++op) {
        if (*op == 'i') client.increment();
        else if (*op == 'r') client.reset();
        else if (*op == 'g') std::printf("%d\n", client.get());
        else if (*op == 's') std::this_thread::sleep_for(std::chrono::milliseconds(50));
        else if (*op == 'w') {
          const int want = std::atoi(op + 1);
          while (*(op + 1) >= '0' && *(op + 1) <= '9') ++op;
          const auto t0 = std::chrono::steady_clock::now();
          int v = client.get();
          while (v != want) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
              std::printf("timeout waiting for %d (last %d)\n", want, v);
              return 3;
            }
            std::this_thread::sleep_for(std::chrono::milliseconds(5));
            v = client.get();
          }
          std::printf("%d\n", v);
        }
        std::fflush(stdout);
      }
      return 0;
    }
    if (cmd == "store-selftest" && argc >= 5) {
      // ac_ppo_carla.cpp:267-282, :343-345, :399-412: rank 0 resets, every collection thread
      // increments once per iteration, every thread sees the count through get()
      const int port = std::stoi(argv[2]), nt = std::stoi(argv[3]), rounds = std::stoi(argv[4]);
      TCPStoreServer server("127.0.0.1", port, nt);
      server.start();
      std::vector<std::unique_ptr<TCPStoreClient>> clients;
      for (int i = 0; i < nt; ++i) clients.push_back(std::make_unique<TCPStoreClient>("127.0.0.1", port));
      for (int r = 0; r < rounds; ++r) {
        clients[0]->reset();
        std::vector<std::thread> th;
        for (int i = 0; i < nt; ++i) th.emplace_back([&, i] { clients[i]->increment(); });
        for (auto& t : th) t.join();
        // every client's subscription converges to the final count
        for (int i = 0; i < nt; ++i) {
          const auto t0 = std::chrono::steady_clock::now();
          int v = clients[i]->get();
          while (v != nt && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(10)) {
            std::this_thread::sleep_for(std::chrono::milliseconds(2));
            v = clients[i]->get();
          }
          if (v != nt) {
            std::printf("round %d client %d saw %d, expected %d\n", r, i, v, nt);
            return 3;
          }
        }
      }
      std::printf("ok %d rounds x %d threads\n", rounds, nt);
      return 0;
    }
    if (cmd == "carla-env" && argc >= 11) {
      gymcpp::CarlaObsConfig c;
      c.obs_num_channels = std::stoi(argv[5]);
      c.bev_semantics_height = std::stoi(argv[6]);
      c.bev_semantics_width = std::stoi(argv[7]);
      c.obs_num_measurements = std::stoi(argv[8]);
      c.num_value_measurements = std::stoi(argv[9]);
      const bool clip = std::stoi(argv[10]) != 0;
      const int steps = std::stoi(argv[4]);
      auto env0 = std::make_shared<gymcpp::CarlaEnv>(c, argv[2], std::stoi(argv[3]));
      std::vector<std::shared_ptr<gymcpp::EnvironmentWrapperCarla>> arr{gymcpp::make_env(env0)};
      gymcpp::SeqVectorEnvCarla env(arr, clip);
      const size_t nb = (size_t)c.obs_num_channels * c.bev_semantics_height * c.bev_semantics_width;
      auto s = env.reset(1);
      std::printf("reset bev %016llx meas %016llx vmeas %016llx\n", (unsigned long long)fnv(s.bev_semantics, nb),
                  (unsigned long long)fnv(s.measurements, 4 * c.obs_num_measurements),
                  (unsigned long long)fnv(s.value_measurements, 4 * c.num_value_measurements));
      std::fflush(stdout);
      for (int t = 0; t < steps; ++t) {
        const float a[2] = {1.5f * std::sin((float)t), 1.5f * std::cos((float)t)};
        auto [st, rew, term, trunc, infos] = env.step(a);
        const auto& info = (*infos)[0];
        std::printf("step %d reward %.9g term %d trunc %d bev %016llx meas %016llx vmeas %016llx info %s %.9g %d\n", t,
                    rew[0], (int)term[0], (int)trunc[0], (unsigned long long)fnv(st.bev_semantics, nb),
                    (unsigned long long)fnv(st.measurements, 4 * c.obs_num_measurements),
                    (unsigned long long)fnv(st.value_measurements, 4 * c.num_value_measurements),
                    info ? "yes" : "no", info ? info->r : 0.0f, info ? info->l : 0);
        std::fflush(stdout);
      }
      return 0;
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
  std::fprintf(stderr, "bad arguments\n");
  return 2;
}
