// net/zmtp.h — the ZeroMQ wire protocol (ZMTP 3.0, https://rfc.zeromq.org/spec/23/, NULL security)
// for the socket patterns the reference uses through libzmq / cppzmq:
//   PAIR over ipc://   CaRL env <-> CARLA leaderboard (libs/gymcpp/carla/carla_gym.h:49-141),
//                      inference server <-> eval_agent.py (src/carla/ppo_carla_inference.cpp:71-196)
//   REQ / REP, PUB / SUB with conflate over tcp://   DD-PPO preemption store (include/tcp_store.h)
// libzmq is not in this image; the bytes on the wire are the ones a libzmq / pyzmq peer sends and
// expects (greeting, READY handshake, frames, REQ/REP envelope, 3.0 subscription messages), so the
// Python side of the reference (leaderboard gym, eval_agent.py) can talk to these sockets unchanged.
//
// Model: one Socket owns its listening fd (bind) or its one outgoing connection (connect, retried
// until the peer exists, as libzmq does), every accepted peer, and per-peer inboxes of complete
// multipart messages. All fds are non-blocking; progress happens inside send / recv (poll-driven),
// no background thread. Blocking calls take an optional timeout. Not thread-safe (neither is a zmq
// socket).
#pragma once

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstring>
#include <deque>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace zmtp {

enum class Type { PAIR, PUB, SUB, REQ, REP };
using Message = std::vector<std::string>;  // frames of one multipart message

inline const char* type_name(Type t) {
  switch (t) {
    case Type::PAIR: return "PAIR";
    case Type::PUB: return "PUB";
    case Type::SUB: return "SUB";
    case Type::REQ: return "REQ";
    case Type::REP: return "REP";
  }
  return "?";
}
// RFC 23 "Socket-Type" compatibility (the subset of patterns implemented here)
inline bool compatible(Type t, const std::string& peer) {
  switch (t) {
    case Type::PAIR: return peer == "PAIR";
    case Type::PUB: return peer == "SUB" || peer == "XSUB";
    case Type::SUB: return peer == "PUB" || peer == "XPUB";
    case Type::REQ: return peer == "REP" || peer == "ROUTER";
    case Type::REP: return peer == "REQ" || peer == "DEALER";
  }
  return false;
}

class Error : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

// ---- wire encoding (RFC 23 §"Formal Grammar") ----
enum : uint8_t { kMore = 0x01, kLong = 0x02, kCommand = 0x04 };

// 64-octet greeting: signature %xFF 8*%x00 %x7F, version 3.0, mechanism "NULL" (20 octets, zero
// padded), as-server 0, filler 31*%x00
inline std::string greeting() {
  std::string g(64, '\0');
  g[0] = '\xFF';
  g[9] = '\x7F';
  g[10] = 3;
  g[11] = 0;
  std::memcpy(&g[12], "NULL", 4);
  return g;
}
inline void put_frame(std::string& out, uint8_t flags, const std::string& body) {
  if (body.size() > 255) {
    out.push_back((char)(flags | kLong));
    const uint64_t n = body.size();
    for (int i = 7; i >= 0; --i) out.push_back((char)((n >> (8 * i)) & 0xFF));
  } else {
    out.push_back((char)flags);
    out.push_back((char)body.size());
  }
  out += body;
}
// READY command: name-size "READY" then properties name-size name value-size(4, network order) value
inline std::string ready_command(Type t) {
  auto prop = [](std::string& b, const std::string& name, const std::string& value) {
    b.push_back((char)name.size());
    b += name;
    const uint32_t n = (uint32_t)value.size();
    for (int i = 3; i >= 0; --i) b.push_back((char)((n >> (8 * i)) & 0xFF));
    b += value;
  };
  std::string body;
  body.push_back(5);
  body += "READY";
  prop(body, "Socket-Type", type_name(t));
  if (t == Type::REQ) prop(body, "Identity", "");  // libzmq sends Identity for REQ / DEALER / ROUTER
  std::string out;
  put_frame(out, kCommand, body);
  return out;
}
inline std::string encode(const Message& m) {
  std::string out;
  for (size_t i = 0; i < m.size(); ++i) put_frame(out, i + 1 < m.size() ? kMore : 0, m[i]);
  return out;
}

class Socket {
  struct Peer {
    int fd = -1;
    std::string rbuf;
    bool greeted = false, ready = false;
    Message partial;
    std::deque<Message> inbox;
    std::vector<std::string> subs;  // PUB side: subscriptions of this SUB peer
  };

 public:
  explicit Socket(Type t) : type_(t) {}
  Socket(const Socket&) = delete;
  Socket& operator=(const Socket&) = delete;
  ~Socket() { close(); }

  Type type() const { return type_; }
  // SUB options (zmq::sockopt::subscribe / conflate)
  void subscribe(const std::string& prefix) {
    subs_.push_back(prefix);
    std::vector<Peer*> dead;
    for (auto& p : peers_)
      if (p->ready && !send_raw(*p, encode({std::string(1, '\x01') + prefix}))) dead.push_back(p.get());
    for (Peer* d : dead) drop(d);
  }
  void set_conflate(bool on) { conflate_ = on; }
  // ZMQ_MAXMSGSIZE: a peer announcing a larger frame is disconnected (0: no limit, libzmq's default)
  void set_max_msg_size(size_t bytes) { max_msg_size_ = bytes; }

  // "tcp://*:port", "tcp://host:port", "ipc:///path"
  void bind(const std::string& endpoint) {
    if (listen_fd_ >= 0) throw Error("zmtp: socket already bound");
    listen_fd_ = open_endpoint(endpoint, true);
  }
  void connect(const std::string& endpoint) {
    connect_ep_ = endpoint;
    try_connect();
  }
  void close() {
    for (auto& p : peers_)
      if (p->fd >= 0) ::close(p->fd);
    peers_.clear();
    if (listen_fd_ >= 0) {
      ::close(listen_fd_);
      listen_fd_ = -1;
      if (!ipc_path_.empty()) ::unlink(ipc_path_.c_str());
    }
  }

  // Send one multipart message. PAIR / REQ wait for the peer (timeout_ms < 0: forever); REP replies
  // to the peer of the last request; PUB fans out to the matching subscribers present (none: dropped,
  // as zmq). Returns false on timeout.
  // A peer that has gone (EPIPE, ECONNRESET, ...) is dropped, as libzmq does, instead of failing
  // the socket: PUB keeps serving its other subscribers; REP / REQ / PAIR return false.
  bool send(const Message& m, int timeout_ms = -1) {
    if (type_ == Type::SUB) throw Error("zmtp: SUB sockets do not send");
    if (type_ == Type::PUB) {
      pump(0);
      const std::string bytes = encode(m);
      std::vector<Peer*> dead;
      for (auto& p : peers_)
        if (p->ready && matches(*p, m.empty() ? std::string() : m[0]) && !send_raw(*p, bytes, true))
          dead.push_back(p.get());
      for (Peer* d : dead) drop(d);
      return true;
    }
    if (type_ == Type::REP) {
      if (!reply_to_) throw Error("zmtp: REP send without a pending request");
      Message e = reply_env_;
      e.insert(e.end(), m.begin(), m.end());
      Peer* p = reply_to_;
      reply_to_ = nullptr;
      if (!send_raw(*p, encode(e))) {
        drop(p);
        return false;
      }
      return true;
    }
    Peer* p = wait_peer(timeout_ms);
    if (!p) return false;
    if (type_ == Type::REQ) {
      if (awaiting_reply_) throw Error("zmtp: REQ send while a reply is pending");
      Message e{std::string()};  // empty delimiter frame
      e.insert(e.end(), m.begin(), m.end());
      if (!send_raw(*p, encode(e))) {
        drop(p);
        return false;
      }
      awaiting_reply_ = true;
      return true;
    }
    if (!send_raw(*p, encode(m))) {
      drop(p);
      return false;
    }
    return true;
  }
  bool send(const std::string& single, int timeout_ms = -1) { return send(Message{single}, timeout_ms); }

  // Receive one multipart message. dontwait: return false at once when none is queued; otherwise
  // wait up to timeout_ms (< 0: forever). SUB with conflate returns the newest queued message.
  bool recv(Message& out, bool dontwait = false, int timeout_ms = -1) {
    if (type_ == Type::PUB) throw Error("zmtp: PUB sockets do not receive");
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      pump(0);
      if (take(out)) return true;
      if (dontwait) return false;
      int left = -1;
      if (timeout_ms >= 0) {
        const long el = (long)std::chrono::duration_cast<std::chrono::milliseconds>(
                            std::chrono::steady_clock::now() - t0).count();
        if (el >= timeout_ms) return false;
        left = (int)(timeout_ms - el);
      }
      pump(left < 0 ? 100 : std::min(left, 100));
    }
  }

  // drive the connection until a peer finished the handshake (and, for SUB, got our
  // subscriptions); libzmq does this on its I/O thread right after connect. false on timeout.
  bool wait_ready(int timeout_ms) { return wait_peer(timeout_ms) != nullptr; }

  int num_ready_peers() const {
    int n = 0;
    for (const auto& p : peers_) n += p->ready;
    return n;
  }
  // drive accepts / handshakes / reads for up to timeout_ms (0: non-blocking)
  void pump(int timeout_ms) {
    if (!connect_ep_.empty() && peers_.empty()) try_connect();
    std::vector<pollfd> fds;
    if (listen_fd_ >= 0) fds.push_back({listen_fd_, POLLIN, 0});
    for (auto& p : peers_) fds.push_back({p->fd, POLLIN, 0});
    if (fds.empty()) {
      if (timeout_ms > 0) ::poll(nullptr, 0, std::min(timeout_ms, 20));
      return;
    }
    const int rc = ::poll(fds.data(), fds.size(), timeout_ms);
    if (rc <= 0) return;
    size_t k = 0;
    if (listen_fd_ >= 0) {
      if (fds[0].revents & POLLIN) accept_all();
      k = 1;
    }
    std::vector<Peer*> dead;
    for (size_t i = 0; k + i < fds.size() && i < peers_.size(); ++i)
      if (fds[k + i].revents & (POLLIN | POLLHUP | POLLERR))
        if (!read_peer(*peers_[i])) dead.push_back(peers_[i].get());
    for (Peer* d : dead) drop(d);
  }

 private:
  Type type_;
  int listen_fd_ = -1;
  std::string ipc_path_, connect_ep_;
  std::vector<std::unique_ptr<Peer>> peers_;
  std::vector<std::string> subs_;
  bool conflate_ = false, awaiting_reply_ = false;
  size_t max_msg_size_ = 0;
  static constexpr int kStallMs = 5000;  // a peer that stops reading in the middle of a message is dropped
  size_t rr_ = 0;  // REP fair queueing
  Peer* reply_to_ = nullptr;
  Message reply_env_;
  std::chrono::steady_clock::time_point next_try_{};

  static void nonblock(int fd) { ::fcntl(fd, F_SETFL, ::fcntl(fd, F_GETFL, 0) | O_NONBLOCK); }

  int open_endpoint(const std::string& ep, bool do_bind) {
    if (ep.rfind("ipc://", 0) == 0) {
      const std::string path = ep.substr(6);
      sockaddr_un a{};
      a.sun_family = AF_UNIX;
      if (path.size() >= sizeof(a.sun_path)) throw Error("zmtp: ipc path too long: " + path);
      std::memcpy(a.sun_path, path.c_str(), path.size() + 1);
      const int fd = ::socket(AF_UNIX, SOCK_STREAM, 0);
      if (fd < 0) throw Error("zmtp: socket() failed");
      if (do_bind) {
        ::unlink(path.c_str());  // libzmq replaces a stale socket file
        if (::bind(fd, (sockaddr*)&a, sizeof(a)) != 0 || ::listen(fd, 64) != 0) {
          ::close(fd);
          throw Error("zmtp: cannot bind " + ep + ": " + std::strerror(errno));
        }
        ipc_path_ = path;
        nonblock(fd);
        return fd;
      }
      if (::connect(fd, (sockaddr*)&a, sizeof(a)) != 0) {
        ::close(fd);
        return -1;
      }
      nonblock(fd);
      return fd;
    }
    if (ep.rfind("tcp://", 0) != 0) throw Error("zmtp: unsupported endpoint " + ep);
    const std::string hp = ep.substr(6);
    const size_t c = hp.rfind(':');
    if (c == std::string::npos) throw Error("zmtp: endpoint without port: " + ep);
    std::string host = hp.substr(0, c);
    const std::string port = hp.substr(c + 1);
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (do_bind && (host == "*" || host.empty())) {
      hints.ai_flags = AI_PASSIVE;
      if (::getaddrinfo(nullptr, port.c_str(), &hints, &res) != 0) throw Error("zmtp: bad endpoint " + ep);
    } else if (::getaddrinfo(host.c_str(), port.c_str(), &hints, &res) != 0) {
      if (do_bind) throw Error("zmtp: cannot resolve " + ep);
      return -1;
    }
    const int fd = ::socket(res->ai_family, SOCK_STREAM, 0);
    if (fd < 0) {
      ::freeaddrinfo(res);
      throw Error("zmtp: socket() failed");
    }
    int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    if (do_bind) {
      ::setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
      const int ok = ::bind(fd, res->ai_addr, res->ai_addrlen) == 0 && ::listen(fd, 64) == 0;
      ::freeaddrinfo(res);
      if (!ok) {
        ::close(fd);
        throw Error("zmtp: cannot bind " + ep + ": " + std::strerror(errno));
      }
      nonblock(fd);
      return fd;
    }
    const int ok = ::connect(fd, res->ai_addr, res->ai_addrlen) == 0;
    ::freeaddrinfo(res);
    if (!ok) {
      ::close(fd);
      return -1;
    }
    nonblock(fd);
    return fd;
  }

  void try_connect() {
    const auto now = std::chrono::steady_clock::now();
    if (now < next_try_) return;
    const int fd = open_endpoint(connect_ep_, false);
    if (fd < 0) {  // not there yet: retry (libzmq reconnects in the background the same way)
      next_try_ = now + std::chrono::milliseconds(50);
      return;
    }
    add_peer(fd);
  }
  void accept_all() {
    for (;;) {
      const int fd = ::accept(listen_fd_, nullptr, nullptr);
      if (fd < 0) return;
      if (type_ == Type::PAIR && !peers_.empty()) {  // PAIR is exclusive: refuse a second peer
        ::close(fd);
        continue;
      }
      nonblock(fd);
      int one = 1;
      ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      add_peer(fd);
    }
  }
  void add_peer(int fd) {
    auto p = std::make_unique<Peer>();
    p->fd = fd;
    Peer& r = *p;
    peers_.push_back(std::move(p));
    if (!send_raw(r, greeting())) drop(&r);  // the whole greeting at once (RFC 23 allows it)
  }
  void drop(Peer* d) {
    if (reply_to_ == d) reply_to_ = nullptr;
    for (size_t i = 0; i < peers_.size(); ++i)
      if (peers_[i].get() == d) {
        ::close(d->fd);
        peers_.erase(peers_.begin() + (long)i);
        break;
      }
    if (type_ == Type::REQ) awaiting_reply_ = false;
  }

  // Writes one encoded message to a peer. false: the peer is gone (any send error but EAGAIN /
  // EINTR) or stopped reading for kStallMs in the middle of the message -- the caller drops it.
  // hwm_drop (PUB): a subscriber whose socket buffer is full when the message starts does not get
  // it (libzmq drops messages for a subscriber at its high-water mark) and stays connected.
  bool send_raw(Peer& p, const std::string& bytes, bool hwm_drop = false) {
    size_t off = 0;
    const auto t0 = std::chrono::steady_clock::now();
    while (off < bytes.size()) {
      const ssize_t n = ::send(p.fd, bytes.data() + off, bytes.size() - off, MSG_NOSIGNAL);
      if (n > 0) {
        off += (size_t)n;
        continue;
      }
      if (n < 0 && errno == EINTR) continue;
      if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        if (hwm_drop && off == 0) return true;
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(kStallMs)) return false;
        pollfd f{p.fd, POLLOUT, 0};
        ::poll(&f, 1, 100);
        continue;
      }
      return false;
    }
    return true;
  }

  // read what is available and parse it; false when the peer closed or broke the protocol
  bool read_peer(Peer& p) {
    char buf[65536];
    for (;;) {
      const ssize_t n = ::recv(p.fd, buf, sizeof(buf), 0);
      if (n > 0) {
        p.rbuf.append(buf, (size_t)n);
        continue;
      }
      if (n == 0) return false;
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      if (errno == EINTR) continue;
      return false;
    }
    return parse(p);
  }
  bool parse(Peer& p) {
    size_t pos = 0;
    if (!p.greeted) {
      if (p.rbuf.size() < 64) return true;
      const std::string& g = p.rbuf;
      if ((uint8_t)g[0] != 0xFF || (uint8_t)g[9] != 0x7F || (uint8_t)g[10] < 3) return false;  // ZMTP >= 3.0
      if (std::memcmp(&g[12], "NULL", 4) != 0) return false;
      p.greeted = true;
      pos = 64;
      if (!send_raw(p, ready_command(type_))) return false;
    }
    for (;;) {
      if (p.rbuf.size() - pos < 2) break;
      const uint8_t flags = (uint8_t)p.rbuf[pos];
      size_t hdr = 2, len = (uint8_t)p.rbuf[pos + 1];
      if (flags & kLong) {
        if (p.rbuf.size() - pos < 9) break;
        len = 0;
        for (int i = 0; i < 8; ++i) len = (len << 8) | (uint8_t)p.rbuf[pos + 1 + i];
        hdr = 9;
      }
      if (max_msg_size_ && len > max_msg_size_) return false;  // ZMQ_MAXMSGSIZE: drop the peer
      if (p.rbuf.size() - pos - hdr < len) break;
      std::string body = p.rbuf.substr(pos + hdr, len);
      pos += hdr + len;
      if (flags & kCommand) {
        if (!on_command(p, body)) return false;
        continue;
      }
      if (!p.ready) return false;  // a message before READY
      p.partial.push_back(std::move(body));
      if (!(flags & kMore)) {
        on_message(p, std::move(p.partial));
        p.partial.clear();
      }
    }
    p.rbuf.erase(0, pos);
    return true;
  }
  bool on_command(Peer& p, const std::string& body) {
    if (body.empty()) return false;
    const size_t nl = (uint8_t)body[0];
    if (body.size() < 1 + nl) return false;
    const std::string name = body.substr(1, nl);
    if (name == "READY") {
      size_t q = 1 + nl;
      std::string peer_type;
      while (q < body.size()) {
        const size_t kn = (uint8_t)body[q];
        if (q + 1 + kn + 4 > body.size()) return false;
        const std::string key = body.substr(q + 1, kn);
        q += 1 + kn;
        size_t vn = 0;
        for (int i = 0; i < 4; ++i) vn = (vn << 8) | (uint8_t)body[q + i];
        q += 4;
        if (q + vn > body.size()) return false;
        if (key == "Socket-Type") peer_type = body.substr(q, vn);
        q += vn;
      }
      if (!compatible(type_, peer_type)) return false;
      p.ready = true;
      if (type_ == Type::SUB)
        for (const auto& s : subs_)
          if (!send_raw(p, encode({std::string(1, '\x01') + s}))) return false;
      return true;
    }
    if (name == "SUBSCRIBE" && type_ == Type::PUB) {  // ZMTP 3.1 form
      p.subs.push_back(body.substr(1 + nl));
      return true;
    }
    if (name == "CANCEL" && type_ == Type::PUB) {
      cancel(p, body.substr(1 + nl));
      return true;
    }
    if (name == "ERROR") return false;
    return true;  // PING / PONG and others: nothing to do for these patterns
  }
  void cancel(Peer& p, const std::string& topic) {
    for (size_t i = 0; i < p.subs.size(); ++i)
      if (p.subs[i] == topic) {
        p.subs.erase(p.subs.begin() + (long)i);
        return;
      }
  }
  void on_message(Peer& p, Message m) {
    if (type_ == Type::PUB) {  // ZMTP 3.0 subscriptions: %x01 topic / %x00 topic
      if (m.size() == 1 && !m[0].empty()) {
        if (m[0][0] == '\x01') p.subs.push_back(m[0].substr(1));
        else if (m[0][0] == '\x00') cancel(p, m[0].substr(1));
      }
      return;
    }
    if (type_ == Type::SUB && conflate_) p.inbox.clear();
    p.inbox.push_back(std::move(m));
  }
  static bool matches(const Peer& p, const std::string& first) {
    for (const auto& s : p.subs)
      if (first.compare(0, s.size(), s) == 0) return true;
    return false;
  }
  Peer* wait_peer(int timeout_ms) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      for (auto& p : peers_)
        if (p->ready) return p.get();
      if (timeout_ms >= 0 && std::chrono::duration_cast<std::chrono::milliseconds>(
                                 std::chrono::steady_clock::now() - t0).count() >= timeout_ms)
        return nullptr;
      pump(50);
    }
  }
  bool take(Message& out) {
    if (peers_.empty()) return false;
    if (type_ == Type::SUB && conflate_) {  // the newest message of any publisher
      Peer* best = nullptr;
      for (auto& p : peers_)
        if (!p->inbox.empty()) best = p.get();
      if (!best) return false;
      out = std::move(best->inbox.back());
      for (auto& p : peers_) p->inbox.clear();
      return true;
    }
    for (size_t k = 0; k < peers_.size(); ++k) {
      Peer& p = *peers_[(rr_ + k) % peers_.size()];
      if (p.inbox.empty()) continue;
      Message m = std::move(p.inbox.front());
      p.inbox.pop_front();
      rr_ = (rr_ + k + 1) % peers_.size();
      if (type_ == Type::REP) {  // strip the envelope up to and including the empty delimiter
        size_t d = 0;
        while (d < m.size() && !m[d].empty()) ++d;
        if (d == m.size()) continue;  // malformed request: dropped, as libzmq does
        reply_env_.assign(m.begin(), m.begin() + (long)d + 1);
        m.erase(m.begin(), m.begin() + (long)d + 1);
        reply_to_ = &p;
      } else if (type_ == Type::REQ) {
        if (!awaiting_reply_) continue;
        if (m.empty() || !m[0].empty()) continue;  // replies carry the empty delimiter
        m.erase(m.begin());
        awaiting_reply_ = false;
      }
      out = std::move(m);
      return true;
    }
    return false;
  }
};

}  // namespace zmtp
