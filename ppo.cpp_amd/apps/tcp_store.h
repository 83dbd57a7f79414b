// apps/tcp_store.h — the DD-PPO preemption store (include/tcp_store.h) over the repo's ZMTP sockets
// (net/zmtp.h) instead of libzmq: same classes, methods, wire protocol and error behaviour.
//
//   TCPStoreServer(rdvz_addr, port, max_connections)   tcp_store.h:16-98
//     start(): REP on tcp://*:port receives 'i' (num_done += 1) or 'r' (num_done = 0), answers one
//     byte ' ', then PUBlishes the new count (the raw int) on tcp://rdvz_addr:port+1; any other
//     command is an error that ends the process (the reference throws from the server thread).
//   TCPStoreClient(rdvz_addr, port)                      tcp_store.h:100-158
//     increment() / reset(): REQ round trip; get(): the latest published count (SUB, conflate),
//     or the previous value when nothing new arrived.
// Used by the CaRL trainer (ac_ppo_carla.cpp:267-282, :343-345, :399-412): each collection thread
// counts itself done and stops early once more than dd_ppo_preempt_threshold of all envs are done.
#pragma once

#include <atomic>
#include <cstring>
#include <iostream>
#include <stdexcept>
#include <string>
#include <thread>

#include "../net/zmtp.h"

class TCPStoreServer {
  int num_done_;
  std::string rdvz_addr_;
  int port_;
  int max_connections_;
  std::thread server_thread_;
  const char empty_ = ' ';

 public:
  std::atomic_bool running_ = false;

  TCPStoreServer(const std::string& rdvz_addr, const int port, const int max_connections)
      : num_done_(0), rdvz_addr_(rdvz_addr), port_(port), max_connections_(max_connections) {}

  void start() {
    // bound here (not in the thread) so that a client constructed right after start() finds them
    auto rep = std::make_shared<zmtp::Socket>(zmtp::Type::REP);   // change requests
    auto pub = std::make_shared<zmtp::Socket>(zmtp::Type::PUB);   // current state
    rep->set_max_msg_size(1 << 16);  // the store's commands are one byte; the port is open to the network
    rep->bind("tcp://*:" + std::to_string(port_));
    pub->bind("tcp://" + rdvz_addr_ + ":" + std::to_string(port_ + 1));
    std::cout << "Server started, waiting for requests..." << std::endl;
    running_ = true;
    server_thread_ = std::thread([this, rep, pub] {
      while (running_) {
        zmtp::Message request;
        pub->pump(0);  // accept subscribers between requests
        if (!rep->recv(request, false, 100)) continue;
        const std::string command = request.empty() ? std::string() : request[0];
        if (!command.empty() && command[0] == 'i') {
          num_done_ += 1;
        } else if (!command.empty() && command[0] == 'r') {
          num_done_ = 0;
        } else {
          std::cerr << "Invalid command: " << command << std::endl;
          throw std::runtime_error("Invalid command: " + command);
        }
        rep->send(std::string(&empty_, 1));
        std::string value(sizeof(num_done_), '\0');
        std::memcpy(&value[0], &num_done_, sizeof(num_done_));
        pub->send(value);  // publish the new value to all workers
      }
      std::cout << "TCP socket closed, exiting thread..." << std::endl;
    });
  }

  ~TCPStoreServer() {
    if (running_) {
      running_ = false;
      server_thread_.join();
    }
  }
};

class TCPStoreClient {
  std::string rdvz_addr_;
  int port_;
  int num_done_ = 0;
  zmtp::Socket socket_0_{zmtp::Type::REQ};
  zmtp::Socket socket_1_{zmtp::Type::SUB};

  void request(char command) {
    socket_0_.send(std::string(1, command));
    zmtp::Message reply;
    if (!socket_0_.recv(reply)) {
      std::cerr << "Invalid message receiveced: " << std::endl;
      throw std::runtime_error("Invalid message receiveced: ");
    }
  }

 public:
  TCPStoreClient(const std::string& rdvz_addr, const int port) : rdvz_addr_(rdvz_addr), port_(port) {
    socket_1_.set_conflate(true);
    socket_0_.connect("tcp://" + rdvz_addr_ + ":" + std::to_string(port_));
    socket_1_.connect("tcp://" + rdvz_addr_ + ":" + std::to_string(port_ + 1));
    socket_1_.subscribe("");  // all topics
    // libzmq completes the subscription on its I/O thread right after connect; without one, finish
    // the handshake here so the first publications after construction are not missed
    socket_1_.wait_ready(-1);
  }

  void increment() { request('i'); }
  void reset() { request('r'); }

  int get() {
    zmtp::Message reply;
    if (!socket_1_.recv(reply, /*dontwait=*/true) || reply.empty() || reply[0].size() < sizeof(int))
      return num_done_;  // nothing new: the previous value (tcp_store.h:150-153)
    std::memcpy(&num_done_, reply[0].data(), sizeof(int));
    return num_done_;
  }
};
