// tensorboard_logger.h — TensorBoard event-file writer without protobuf.
//
// Drop-in for the reference's libs/tensorboard_logger TensorBoardLogger as the trainers use it
// (src/ppo_continuous_action.cpp:281, src/ac_ppo_continuous_action.cpp:420): same class name,
// constructor contract (the basename must contain "tfevents"), and add_scalar(tag, int step,
// value). The reference serializes tensorflow.Event with libprotobuf (tensorboard_logger.cc:
// 305-335); here the three messages it uses are hand-encoded in protobuf wire format, fields in
// field-number order as libprotobuf emits them:
//   Event   { double wall_time = 1; int64 step = 2; Summary summary = 5; }   (proto3: zero
//           wall_time / step are omitted)
//   Summary { repeated Value value = 1; }
//   Value   { string tag = 1; float simple_value = 2; }                     (oneof: always written)
// Record framing (TFRecord): uint64 length, masked CRC32C of the length, payload, masked CRC32C
// of the payload; mask = ((crc >> 15) | (crc << 17)) + 0xa282ead8 (crc.h / crc.cc:237).
#pragma once

#include <cstdint>
#include <cstring>
#include <ctime>
#include <fstream>
#include <mutex>
#include <stdexcept>
#include <string>

namespace tb {

// CRC32C (Castagnoli, reflected polynomial 0x82F63B78), table-driven
inline uint32_t crc32c(const char* buf, size_t len) {
  static uint32_t table[256];
  static bool init = false;
  if (!init) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
      table[i] = c;
    }
    init = true;
  }
  uint32_t crc = 0xFFFFFFFFu;
  for (size_t i = 0; i < len; ++i) crc = table[(crc ^ (uint8_t)buf[i]) & 0xFF] ^ (crc >> 8);
  return crc ^ 0xFFFFFFFFu;
}
inline uint32_t masked_crc32c(const char* buf, size_t len) {
  const uint32_t crc = crc32c(buf, len);
  return ((crc >> 15) | (crc << 17)) + 0xa282ead8u;
}

inline void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back((char)((v & 0x7F) | 0x80));
    v >>= 7;
  }
  s.push_back((char)v);
}
inline void put_key(std::string& s, int field, int wire) { put_varint(s, ((uint64_t)field << 3) | (uint64_t)wire); }
inline void put_bytes(std::string& s, int field, const std::string& b) {
  put_key(s, field, 2);
  put_varint(s, b.size());
  s += b;
}
template <typename T>
inline void put_fixed(std::string& s, int field, T v) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "fixed32 / fixed64");
  put_key(s, field, sizeof(T) == 8 ? 1 : 5);
  char b[sizeof(T)];
  std::memcpy(b, &v, sizeof(T));  // little-endian host, as the wire format
  s.append(b, sizeof(T));
}

// serialized tensorflow.Event carrying one scalar summary value
inline std::string scalar_event(double wall_time, int64_t step, const std::string& tag, float value) {
  std::string val, summary, ev;
  put_bytes(val, 1, tag);
  put_fixed(val, 2, value);
  put_bytes(summary, 1, val);
  if (wall_time != 0.0) put_fixed(ev, 1, wall_time);
  if (step != 0) {
    put_key(ev, 2, 0);
    put_varint(ev, (uint64_t)step);  // int64: two's complement, 10 bytes when negative
  }
  put_bytes(ev, 5, summary);
  return ev;
}

}  // namespace tb

class TensorBoardLogger {
  std::ofstream ofs_;
  std::mutex mu_;

 public:
  explicit TensorBoardLogger(const std::string& log_file) {
    const auto slash = log_file.find_last_of("/\\");
    const std::string base = slash == std::string::npos ? log_file : log_file.substr(slash + 1);
    if (base.find("tfevents") == std::string::npos)
      throw std::runtime_error("A valid event file must contain substring \"tfevents\" in its basename, got " + base);
    ofs_.open(log_file, std::ios::out | std::ios::trunc | std::ios::binary);
    if (!ofs_.is_open()) throw std::runtime_error("failed to open log_file " + log_file);
  }

  // tensorboard_logger.cc:58-64 / :305-312 (wall_time = time(nullptr), the event's step)
  int add_scalar(const std::string& tag, int step, double value) {
    write(tb::scalar_event((double)time(nullptr), step, tag, (float)value));
    return 0;
  }

  void write(const std::string& buf) {
    const uint64_t len = buf.size();
    const uint32_t len_crc = tb::masked_crc32c(reinterpret_cast<const char*>(&len), sizeof(len));
    const uint32_t data_crc = tb::masked_crc32c(buf.data(), buf.size());
    std::lock_guard<std::mutex> lk(mu_);
    ofs_.write(reinterpret_cast<const char*>(&len), sizeof(len));
    ofs_.write(reinterpret_cast<const char*>(&len_crc), sizeof(len_crc));
    ofs_.write(buf.data(), (std::streamsize)buf.size());
    ofs_.write(reinterpret_cast<const char*>(&data_crc), sizeof(data_crc));
    ofs_.flush();
  }
};
