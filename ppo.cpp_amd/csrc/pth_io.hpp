// pth_io.h — LibTorch checkpoints (torch::save(agent / optimizer, "*.pth")) without LibTorch
// (SURVEY §8(f)-2). Host-only C++.
//
// torch::save of an nn::Module or an optimizer (reference: save_state in
// src/ppo_continuous_action.cpp:173-180 and src/ac_ppo_continuous_action.cpp; torch::load in
// src/carla/ppo_carla_inference.cpp:104 and src/carla/ac_ppo_carla.cpp:236-251) writes a
// TorchScript module archive: an uncompressed zip whose entries sit under one top-level folder,
//   data.pkl            pickle (protocol 2) of nested `__torch__[.___torch_mangle_k] Module`
//                       objects; each object's state is a dict of its attributes in slot order:
//                       tensors (torch._utils._rebuild_tensor_v2 over a persistent storage id),
//                       int / str / float / bool / tuple values and child objects
//   data/<key>          raw little-endian storage of each tensor (float32 or int64)
//   code/__torch__.py, code/__torch__/___torch_mangle_k.py (+ .debug_pkl)
//                       the TorchScript class of every object: its parameter list and members
//   constants.pkl, version, byteorder, .data/serialization_id
// archive_bytes() emits that layout from an Obj tree: data.pkl and the class files are
// byte-identical to torch::save's for the same tree (same memo sequence, same class numbering —
// tests/test_pth_io.py checks both against archives the reference's LibTorch wrote);
// read_archive() parses any such archive back into an Obj tree.
//
// Agent-level helpers: an agent is described by a Spec (every submodule path in registration
// order, parameterless Tanh / ReLU included, and the parameters in named_parameters() order with
// their flat offsets); save_module / load_module and save_adam / load_adam convert between that
// and the flat vectors of the C-ABI (ppo_save_params, ppo_save_adam).
#pragma once

#include <algorithm>
#include <cctype>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <iterator>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace pth {

// ------------------------------------------------------------------------------------------
// object model
// ------------------------------------------------------------------------------------------
struct Obj;
struct Value {
  enum Kind { TENSOR, INT, STR, DOUBLE, DOUBLE_TUPLE, BOOL, OBJ, NONE } kind = NONE;
  // TENSOR
  std::vector<int64_t> shape;
  std::string bytes;  // contiguous little-endian data
  bool is_long = false, requires_grad = false, is_param = false;
  // scalars
  int64_t i = 0;
  double d = 0.0;
  std::vector<double> dt;
  std::string s;
  bool b = false;
  std::shared_ptr<Obj> obj;

  int64_t numel() const {
    int64_t n = 1;
    for (int64_t x : shape) n *= x;
    return n;
  }
  std::vector<float> floats() const {
    if (kind != TENSOR || is_long) throw std::runtime_error("pth: not a float tensor");
    std::vector<float> v((size_t)numel());
    std::memcpy(v.data(), bytes.data(), v.size() * 4);
    return v;
  }
  int64_t long_scalar() const {
    if (kind != TENSOR || !is_long || numel() != 1) throw std::runtime_error("pth: not an int64 scalar tensor");
    int64_t v;
    std::memcpy(&v, bytes.data(), 8);
    return v;
  }
};

struct Obj {
  std::vector<std::pair<std::string, Value>> attrs;
  const Value* find(const std::string& k) const {
    for (const auto& a : attrs)
      if (a.first == k) return &a.second;
    return nullptr;
  }
  const Value& at(const std::string& k) const {
    const Value* v = find(k);
    if (!v) throw std::runtime_error("pth: missing attribute " + k);
    return *v;
  }
  Obj& child(const std::string& k) {
    for (auto& a : attrs)
      if (a.first == k && a.second.kind == Value::OBJ) return *a.second.obj;
    Value v;
    v.kind = Value::OBJ;
    v.obj = std::make_shared<Obj>();
    attrs.push_back({k, v});
    return *attrs.back().second.obj;
  }
  void add(const std::string& k, Value v) { attrs.push_back({k, std::move(v)}); }
};

inline Value tensor_f32(const std::vector<int64_t>& shape, const float* data, bool requires_grad, bool is_param) {
  Value v;
  v.kind = Value::TENSOR;
  v.shape = shape;
  v.bytes.assign(reinterpret_cast<const char*>(data), (size_t)v.numel() * 4);
  v.requires_grad = requires_grad;
  v.is_param = is_param;
  return v;
}
inline Value tensor_i64_scalar(int64_t x, bool is_param) {
  Value v;
  v.kind = Value::TENSOR;
  v.is_long = true;
  v.bytes.assign(reinterpret_cast<const char*>(&x), 8);
  v.is_param = is_param;
  return v;
}
inline Value int_value(int64_t x) { Value v; v.kind = Value::INT; v.i = x; return v; }
inline Value str_value(const std::string& x) { Value v; v.kind = Value::STR; v.s = x; return v; }
inline Value double_value(double x) { Value v; v.kind = Value::DOUBLE; v.d = x; return v; }
inline Value bool_value(bool x) { Value v; v.kind = Value::BOOL; v.b = x; return v; }
inline Value double_tuple(const std::vector<double>& x) { Value v; v.kind = Value::DOUBLE_TUPLE; v.dt = x; return v; }

// ------------------------------------------------------------------------------------------
// zip (stored entries, data 64-byte aligned like PyTorch's writer)
// ------------------------------------------------------------------------------------------
inline uint32_t crc32(const char* p, size_t n) {
  static uint32_t table[256];
  static bool init = false;
  if (!init) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
      table[i] = c;
    }
    init = true;
  }
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) c = table[(c ^ (uint8_t)p[i]) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

class ZipWriter {
  std::string out_;
  struct Entry {
    std::string name;
    uint32_t crc, size, offset;
  };
  std::vector<Entry> entries_;
  template <typename T>
  void put(T v) {
    out_.append(reinterpret_cast<const char*>(&v), sizeof(T));
  }

 public:
  void add(const std::string& name, const std::string& data) {
    if (out_.size() + data.size() > 0xFFFFFFF0u) throw std::runtime_error("pth: archive above 4 GiB (zip64) not supported");
    const uint32_t offset = (uint32_t)out_.size();
    const uint32_t crc = crc32(data.data(), data.size());
    const size_t start = offset + 30 + name.size() + 4;
    const uint16_t pad = (uint16_t)((64 - start % 64) % 64);
    put<uint32_t>(0x04034b50u); put<uint16_t>(20); put<uint16_t>(0); put<uint16_t>(0);
    put<uint16_t>(0); put<uint16_t>(0x21);  // 1980-01-01 00:00
    put<uint32_t>(crc); put<uint32_t>((uint32_t)data.size()); put<uint32_t>((uint32_t)data.size());
    put<uint16_t>((uint16_t)name.size()); put<uint16_t>((uint16_t)(4 + pad));
    out_ += name;
    put<uint16_t>(0x4246);  // "FB" padding field, as PyTorch's writer
    put<uint16_t>(pad);
    out_.append(pad, 'Z');
    out_ += data;
    entries_.push_back({name, crc, (uint32_t)data.size(), offset});
  }
  std::string finish() {
    const uint32_t cd = (uint32_t)out_.size();
    for (const Entry& e : entries_) {
      put<uint32_t>(0x02014b50u); put<uint16_t>(20); put<uint16_t>(20); put<uint16_t>(0); put<uint16_t>(0);
      put<uint16_t>(0); put<uint16_t>(0x21); put<uint32_t>(e.crc); put<uint32_t>(e.size); put<uint32_t>(e.size);
      put<uint16_t>((uint16_t)e.name.size()); put<uint16_t>(0); put<uint16_t>(0); put<uint16_t>(0);
      put<uint16_t>(0); put<uint32_t>(0); put<uint32_t>(e.offset);
      out_ += e.name;
    }
    const uint32_t cd_size = (uint32_t)out_.size() - cd;
    put<uint32_t>(0x06054b50u); put<uint16_t>(0); put<uint16_t>(0);
    put<uint16_t>((uint16_t)entries_.size()); put<uint16_t>((uint16_t)entries_.size());
    put<uint32_t>(cd_size); put<uint32_t>(cd); put<uint16_t>(0);
    return out_;
  }
};

// name -> data of every stored entry (via the central directory, so data descriptors are fine).
// torch::save deflates some class files (code/...py); their names go to `deflated` (tensor data
// and data.pkl are always stored), any other compressed entry is an error.
inline std::map<std::string, std::string> zip_read(const std::string& z, std::vector<std::string>* deflated = nullptr) {
  auto u16 = [&](size_t o) {
    if (o + 2 > z.size()) throw std::runtime_error("pth: truncated zip");
    uint16_t v;
    std::memcpy(&v, z.data() + o, 2);
    return (size_t)v;
  };
  auto u32 = [&](size_t o) {
    if (o + 4 > z.size()) throw std::runtime_error("pth: truncated zip");
    uint32_t v;
    std::memcpy(&v, z.data() + o, 4);
    return (size_t)v;
  };
  if (z.size() < 22) throw std::runtime_error("pth: not a zip archive");
  size_t eocd = z.size() - 22;
  while (eocd > 0 && u32(eocd) != 0x06054b50u) --eocd;
  if (u32(eocd) != 0x06054b50u) throw std::runtime_error("pth: zip end record not found");
  const size_t n = u16(eocd + 10);
  size_t p = u32(eocd + 16);
  std::map<std::string, std::string> out;
  for (size_t i = 0; i < n; ++i) {
    if (u32(p) != 0x02014b50u) throw std::runtime_error("pth: bad zip central directory");
    const size_t method = u16(p + 10);
    const size_t csize = u32(p + 20), nlen = u16(p + 28), xlen = u16(p + 30), clen = u16(p + 32);
    const size_t loc = u32(p + 42);
    if (csize == 0xFFFFFFFFu || loc == 0xFFFFFFFFu) throw std::runtime_error("pth: zip64 archives are not supported");
    const std::string name = z.substr(p + 46, nlen);
    if (method != 0) {
      if (method != 8 || !deflated || name.find("/code/") == std::string::npos)
        throw std::runtime_error("pth: compressed zip entry " + name + " is not supported");
      deflated->push_back(name);
      p += 46 + nlen + xlen + clen;
      continue;
    }
    const size_t data = loc + 30 + u16(loc + 26) + u16(loc + 28);
    if (data + csize > z.size()) throw std::runtime_error("pth: zip entry out of range: " + name);
    out[name] = z.substr(data, csize);
    p += 46 + nlen + xlen + clen;
  }
  return out;
}

// ------------------------------------------------------------------------------------------
// pickle writer: LibTorch's Pickler memoizes every string and global by value (BINPUT on first
// use, BINGET after), every persistent-id and tensor result, and the root object after BUILD.
// ------------------------------------------------------------------------------------------
class PickleWriter {
  std::map<std::string, uint32_t> memo_;
  uint32_t next_ = 0;
  bool get_memo(const std::string& key) {
    auto it = memo_.find(key);
    if (it == memo_.end()) return false;
    const uint32_t i = it->second;
    if (i < 256) {
      op('h');
      s.push_back((char)i);
    } else {
      op('j');
      s.append(reinterpret_cast<const char*>(&i), 4);
    }
    return true;
  }

 public:
  std::string s = std::string("\x80\x02", 2);
  void op(char c) { s.push_back(c); }
  void memoize() {
    const uint32_t i = next_++;
    if (i < 256) {
      op('q');
      s.push_back((char)i);
    } else {
      op('r');
      s.append(reinterpret_cast<const char*>(&i), 4);
    }
  }
  void global(const std::string& mod, const std::string& name) {
    const std::string key = "g" + mod + "\n" + name;
    if (get_memo(key)) return;
    s += 'c' + mod + '\n' + name + '\n';
    memo_[key] = next_;
    memoize();
  }
  void str(const std::string& v) {
    const std::string key = "s" + v;
    if (get_memo(key)) return;
    op('X');
    const uint32_t n = (uint32_t)v.size();
    s.append(reinterpret_cast<const char*>(&n), 4);
    s += v;
    memo_[key] = next_;
    memoize();
  }
  void integer(int64_t v) {
    if (v >= 0 && v < 256) {
      op('K');
      s.push_back((char)v);
    } else if (v >= 0 && v < 65536) {
      op('M');
      const uint16_t x = (uint16_t)v;
      s.append(reinterpret_cast<const char*>(&x), 2);
    } else if (v >= INT32_MIN && v <= INT32_MAX) {
      op('J');
      const int32_t x = (int32_t)v;
      s.append(reinterpret_cast<const char*>(&x), 4);
    } else {
      op('\x8a');  // LONG1
      s.push_back(8);
      s.append(reinterpret_cast<const char*>(&v), 8);
    }
  }
  void dbl(double v) {  // BINFLOAT, big-endian
    op('G');
    uint64_t u;
    std::memcpy(&u, &v, 8);
    for (int k = 7; k >= 0; --k) s.push_back((char)((u >> (8 * k)) & 0xFF));
  }
  void tuple(const std::vector<int64_t>& v) {
    op('(');
    for (int64_t x : v) integer(x);
    op('t');
  }
};

namespace detail {
// the (empty) source-range table torch::save writes next to every class file
inline std::string debug_pkl() {
  static const char b[] =
      "\x80\x02X\x18\x00\x00\x00" "FORMAT_WITH_STRING_TABLEq\x00X\x00\x00\x00\x00q\x01\x85q\x02K\x00"
      "ctorch.jit._pickle\nbuild_intlist\nq\x03(](etRK\x00K\x00\x87q\x04K\x00K\x00\x87K\x00\x87\x85q\x05\x87.";
  return std::string(b, sizeof(b) - 1);
}
inline bool is_ident(const std::string& s) {
  if (s.empty() || !(std::isalpha((unsigned char)s[0]) || s[0] == '_')) return false;
  for (char c : s)
    if (!(std::isalnum((unsigned char)c) || c == '_')) return false;
  return true;
}
inline std::string cls_name(int mangle) {
  return mangle < 0 ? "__torch__.Module" : "__torch__.___torch_mangle_" + std::to_string(mangle) + ".Module";
}
}  // namespace detail

// The archive of `root` with its entries under `folder` (torch::save uses the file's stem).
inline std::string archive_bytes(const Obj& root, const std::string& folder) {
  // class numbering: DFS pre-order over child objects, as the TorchScript exporter numbers them
  std::map<const Obj*, int> mangle;
  std::vector<const Obj*> dfs;
  std::function<void(const Obj*)> visit = [&](const Obj* o) {
    mangle[o] = o == &root ? -1 : (int)dfs.size() - 1;
    dfs.push_back(o);
    for (const auto& a : o->attrs)
      if (a.second.kind == Value::OBJ) visit(a.second.obj.get());
  };
  visit(&root);

  ZipWriter zip;
  PickleWriter pk;
  std::vector<const Value*> storages;
  std::function<void(const Value&)> emit_value;
  std::function<void(const Obj&)> emit_obj = [&](const Obj& o) {
    const std::string c = detail::cls_name(mangle.at(&o));
    const auto d = c.rfind('.');
    pk.global(c.substr(0, d), c.substr(d + 1));
    pk.op(')'); pk.op('\x81'); pk.op('}'); pk.op('(');
    for (const auto& a : o.attrs) {
      pk.str(a.first);
      emit_value(a.second);
    }
    pk.op('u'); pk.op('b');
  };
  emit_value = [&](const Value& v) {
    switch (v.kind) {
      case Value::TENSOR: {
        std::vector<int64_t> stride(v.shape.size());
        int64_t st = 1;
        for (size_t i = v.shape.size(); i-- > 0;) { stride[i] = st; st *= v.shape[i]; }
        const std::string key = std::to_string(storages.size());
        storages.push_back(&v);
        pk.global("torch._utils", "_rebuild_tensor_v2");
        pk.op('(');
        pk.op('(');
        pk.str("storage");
        pk.global("torch", v.is_long ? "LongStorage" : "FloatStorage");
        pk.str(key);
        pk.str("cpu");
        pk.integer(v.numel());
        pk.op('t');
        pk.op('Q');
        pk.memoize();
        pk.integer(0);
        pk.tuple(v.shape);
        pk.tuple(stride);
        pk.op(v.requires_grad ? '\x88' : '\x89');
        pk.global("collections", "OrderedDict"); pk.op(')'); pk.op('R');
        pk.op('t');
        pk.op('R');
        pk.memoize();
        break;
      }
      case Value::INT: pk.integer(v.i); break;
      case Value::STR: pk.str(v.s); break;
      case Value::DOUBLE: pk.dbl(v.d); break;
      case Value::BOOL: pk.op(v.b ? '\x88' : '\x89'); break;
      case Value::DOUBLE_TUPLE:
        for (double x : v.dt) pk.dbl(x);
        if (v.dt.empty()) pk.op(')');
        else if (v.dt.size() <= 3) pk.op("\x85\x86\x87"[v.dt.size() - 1]);
        else throw std::runtime_error("pth: tuples above 3 elements not supported");
        break;
      case Value::OBJ: emit_obj(*v.obj); break;
      default: throw std::runtime_error("pth: cannot serialize a None attribute");
    }
  };
  emit_obj(root);
  pk.memoize();
  pk.op('.');
  for (size_t k = 0; k < storages.size(); ++k) zip.add(folder + "/data/" + std::to_string(k), storages[k]->bytes);
  zip.add(folder + "/data.pkl", pk.s);
  // the TorchScript class of every object
  for (const Obj* o : dfs) {
    std::string code = "class Module(Module):\n  __parameters__ = [";
    for (const auto& a : o->attrs)
      if (a.second.kind == Value::TENSOR && a.second.is_param) code += "\"" + a.first + "\", ";
    code += "]\n  __buffers__ = []\n";
    bool header = false;
    for (const auto& a : o->attrs) {
      std::string type;
      switch (a.second.kind) {
        case Value::TENSOR: type = "Tensor"; break;
        case Value::INT: type = "int"; break;
        case Value::STR: type = "str"; break;
        case Value::DOUBLE: type = "float"; break;
        case Value::BOOL: type = "bool"; break;
        case Value::DOUBLE_TUPLE: {
          type = "Tuple[";
          for (size_t k = 0; k < a.second.dt.size(); ++k) type += k ? ", float" : "float";
          type += "]";
          break;
        }
        case Value::OBJ: type = detail::cls_name(mangle.at(a.second.obj.get())); break;
        default: break;
      }
      if (detail::is_ident(a.first)) {
        code += "  " + a.first + " : " + type + "\n";
      } else {
        if (!header) code += "  __annotations__ = []\n";
        header = true;
        code += "  __annotations__[\"" + a.first + "\"] = " + type + "\n";
      }
    }
    const int m = mangle.at(o);
    const std::string file = m < 0 ? folder + "/code/__torch__.py"
                                   : folder + "/code/__torch__/___torch_mangle_" + std::to_string(m) + ".py";
    zip.add(file, code);
    zip.add(file + ".debug_pkl", detail::debug_pkl());
  }
  zip.add(folder + "/constants.pkl", std::string("\x80\x02).", 4));
  zip.add(folder + "/version", "3\n");
  zip.add(folder + "/byteorder", "little");
  // a fixed-width decimal id (torch::save draws a random one)
  char id[48];
  std::snprintf(id, sizeof id, "%020u%020u", crc32(pk.s.data(), pk.s.size()), (unsigned)storages.size());
  zip.add(folder + "/.data/serialization_id", std::string(id, 40));
  return zip.finish();
}

inline void write_archive(const std::string& path, const Obj& root) {
  std::string stem = path;
  const auto slash = stem.find_last_of('/');
  if (slash != std::string::npos) stem = stem.substr(slash + 1);
  const auto ext = stem.rfind('.');
  if (ext != std::string::npos && ext > 0) stem = stem.substr(0, ext);
  if (stem.empty()) stem = "archive";
  const std::string bytes = archive_bytes(root, stem);
  std::ofstream f(path, std::ios::binary | std::ios::trunc);
  if (!f) throw std::runtime_error("pth: cannot open " + path);
  f.write(bytes.data(), (std::streamsize)bytes.size());
  if (!f) throw std::runtime_error("pth: write failed for " + path);
}

// ------------------------------------------------------------------------------------------
// pickle reader (the opcodes LibTorch's Pickler emits for module archives)
// ------------------------------------------------------------------------------------------
namespace detail {
struct PV;
using PVP = std::shared_ptr<PV>;
struct PV {  // pickle VM value
  enum Kind { NONE, BOOL, INT, DOUBLE, STR, TUPLE, LIST, DICT, GLOBAL, OBJ, PERSID, TENSOR } kind = NONE;
  int64_t i = 0;
  double d = 0;
  std::string s;
  std::vector<PVP> items;
  std::vector<std::pair<PVP, PVP>> dict;
  Value tensor;
};
inline PVP mk(PV::Kind k) {
  auto v = std::make_shared<PV>();
  v->kind = k;
  return v;
}
}  // namespace detail

inline Obj read_archive_bytes(const std::string& z) {
  using namespace detail;
  std::vector<std::string> deflated;  // class files only; parameter flags then default to false
  const auto files = zip_read(z, &deflated);
  std::string prefix;  // "<folder>/" of the top-level data.pkl
  for (const auto& kv : files) {
    const auto slash = kv.first.find('/');
    if (slash != std::string::npos && kv.first.substr(slash + 1) == "data.pkl") prefix = kv.first.substr(0, slash + 1);
  }
  if (!files.count(prefix + "data.pkl")) throw std::runtime_error("pth: no data.pkl in archive");
  const std::string& pkl = files.at(prefix + "data.pkl");
  std::vector<PVP> st;
  std::vector<size_t> marks;
  std::map<int64_t, PVP> memo;
  size_t p = 0;
  auto rd = [&](size_t n) {
    if (p + n > pkl.size()) throw std::runtime_error("pth: truncated pickle");
    const std::string r = pkl.substr(p, n);
    p += n;
    return r;
  };
  auto rdint = [&](size_t n) {  // little-endian, unsigned
    uint64_t v = 0;
    const std::string b = rd(n);
    for (size_t k = n; k-- > 0;) v = (v << 8) | (uint8_t)b[k];
    return (int64_t)v;
  };
  auto line = [&]() {
    const size_t e = pkl.find('\n', p);
    if (e == std::string::npos) throw std::runtime_error("pth: bad GLOBAL");
    const std::string r = pkl.substr(p, e - p);
    p = e + 1;
    return r;
  };
  auto pop_mark = [&]() {
    if (marks.empty()) throw std::runtime_error("pth: MARK expected");
    const size_t m = marks.back();
    marks.pop_back();
    if (m > st.size()) throw std::runtime_error("pth: bad MARK");
    std::vector<PVP> items(st.begin() + (long)m, st.end());
    st.resize(m);
    return items;
  };
  auto pop = [&]() {
    if (st.empty()) throw std::runtime_error("pth: pickle stack underflow");
    PVP v = st.back();
    st.pop_back();
    return v;
  };
  auto top = [&]() -> PVP& {
    if (st.empty()) throw std::runtime_error("pth: pickle stack underflow");
    return st.back();
  };
  auto memo_at = [&](int64_t k) {
    auto it = memo.find(k);
    if (it == memo.end()) throw std::runtime_error("pth: bad memo reference");
    return it->second;
  };
  auto push_int = [&](int64_t x) { auto v = mk(PV::INT); v->i = x; st.push_back(v); };
  bool done = false;
  while (!done) {
    const char o = rd(1)[0];
    switch (o) {
      case '\x80': rd(1); break;  // PROTO
      case 'c': { auto v = mk(PV::GLOBAL); v->s = line(); v->s += " " + line(); st.push_back(v); break; }
      case 'q': memo[(uint8_t)rd(1)[0]] = top(); break;  // BINPUT
      case 'r': memo[rdint(4)] = top(); break;           // LONG_BINPUT
      case 'h': st.push_back(memo_at((uint8_t)rd(1)[0])); break;
      case 'j': st.push_back(memo_at(rdint(4))); break;
      case ')': st.push_back(mk(PV::TUPLE)); break;
      case ']': st.push_back(mk(PV::LIST)); break;
      case '}': st.push_back(mk(PV::DICT)); break;
      case 'N': st.push_back(mk(PV::NONE)); break;
      case '(': marks.push_back(st.size()); break;
      case 'X': { const int64_t n = rdint(4); auto v = mk(PV::STR); v->s = rd((size_t)n); st.push_back(v); break; }
      case '\x8c': { const size_t n = (uint8_t)rd(1)[0]; auto v = mk(PV::STR); v->s = rd(n); st.push_back(v); break; }
      case 'K': push_int((uint8_t)rd(1)[0]); break;
      case 'M': push_int(rdint(2)); break;
      case 'J': push_int((int32_t)(uint32_t)rdint(4)); break;
      case '\x8a': {  // LONG1
        const size_t n = (uint8_t)rd(1)[0];
        if (n > 8) throw std::runtime_error("pth: integer above 64 bits");
        int64_t x = n ? rdint(n) : 0;
        if (n > 0 && n < 8 && ((x >> (8 * n - 1)) & 1)) x -= int64_t(1) << (8 * n);
        push_int(x);
        break;
      }
      case 'G': {  // BINFLOAT, big-endian
        const std::string b = rd(8);
        uint64_t u = 0;
        for (int k = 0; k < 8; ++k) u = (u << 8) | (uint8_t)b[k];
        auto v = mk(PV::DOUBLE);
        std::memcpy(&v->d, &u, 8);
        st.push_back(v);
        break;
      }
      case '\x88': { auto v = mk(PV::BOOL); v->i = 1; st.push_back(v); break; }
      case '\x89': { auto v = mk(PV::BOOL); v->i = 0; st.push_back(v); break; }
      case 't': { auto v = mk(PV::TUPLE); v->items = pop_mark(); st.push_back(v); break; }
      case '\x85': { auto v = mk(PV::TUPLE); v->items = {pop()}; st.push_back(v); break; }
      case '\x86': { auto b = pop(), a = pop(); auto v = mk(PV::TUPLE); v->items = {a, b}; st.push_back(v); break; }
      case '\x87': { auto c = pop(), b = pop(), a = pop(); auto v = mk(PV::TUPLE); v->items = {a, b, c}; st.push_back(v); break; }
      case 'Q': { auto t = pop(); auto v = mk(PV::PERSID); v->items = {t}; st.push_back(v); break; }
      case 'a': { auto x = pop(); top()->items.push_back(x); break; }
      case 'e': { auto items = pop_mark(); for (auto& x : items) top()->items.push_back(x); break; }
      case 's': { auto v = pop(), k = pop(); top()->dict.push_back({k, v}); break; }
      case 'u': {
        auto items = pop_mark();
        for (size_t i = 0; i + 1 < items.size(); i += 2) top()->dict.push_back({items[i], items[i + 1]});
        break;
      }
      case '\x81': {  // NEWOBJ
        pop();
        auto cls = pop();
        auto v = mk(PV::OBJ);
        v->s = cls->s;
        st.push_back(v);
        break;
      }
      case 'b': { auto state = pop(); top()->dict = state->dict; break; }  // BUILD
      case 'R': {  // REDUCE
        auto args = pop(), fn = pop();
        if (fn->s == "torch._utils _rebuild_tensor_v2") {
          const auto& a = args->items;
          if (a.size() < 5 || a[0]->kind != PV::PERSID || a[0]->items.empty() || a[0]->items[0]->items.size() < 5)
            throw std::runtime_error("pth: bad tensor record");
          const auto& pid = a[0]->items[0]->items;  // ('storage', <Type>Storage, key, location, numel)
          auto v = mk(PV::TENSOR);
          Value& t = v->tensor;
          t.kind = Value::TENSOR;
          if (pid[1]->s == "torch FloatStorage") t.is_long = false;
          else if (pid[1]->s == "torch LongStorage") t.is_long = true;
          else throw std::runtime_error("pth: unsupported storage type " + pid[1]->s);
          const size_t es = t.is_long ? 8 : 4;
          auto fit = files.find(prefix + "data/" + pid[2]->s);
          if (fit == files.end()) throw std::runtime_error("pth: missing storage " + pid[2]->s);
          const std::string& data = fit->second;
          const int64_t offset = a[1]->i;
          std::vector<int64_t> stride;
          for (auto& x : a[2]->items) t.shape.push_back(x->i);
          for (auto& x : a[3]->items) stride.push_back(x->i);
          if (stride.size() != t.shape.size()) throw std::runtime_error("pth: bad tensor strides");
          t.requires_grad = a[4]->i != 0;
          int64_t expect = 1;  // contiguous row-major (how torch::save writes parameters)
          for (size_t i = t.shape.size(); i-- > 0;) {
            if (t.shape[i] != 1 && stride[i] != expect) throw std::runtime_error("pth: non-contiguous tensor");
            expect *= t.shape[i];
          }
          if (offset < 0 || (size_t)(offset + t.numel()) * es > data.size()) throw std::runtime_error("pth: storage too small");
          t.bytes = data.substr((size_t)offset * es, (size_t)t.numel() * es);
          st.push_back(v);
        } else {
          auto v = mk(PV::DICT);  // collections.OrderedDict() and other empty containers
          v->s = fn->s;
          st.push_back(v);
        }
        break;
      }
      case '.': done = true; break;
      default: {
        char buf[64];
        std::snprintf(buf, sizeof buf, "pth: unsupported pickle opcode 0x%02x", (unsigned)(uint8_t)o);
        throw std::runtime_error(buf);
      }
    }
  }
  if (st.empty() || st.back()->kind != PV::OBJ) throw std::runtime_error("pth: root is not a module object");
  // parameter names from the class files: `__parameters__ = ["a", "b", ]`
  auto params_of = [&](const std::string& cls) {
    std::vector<std::string> names;
    std::string file;
    if (cls == "__torch__ Module") file = "code/__torch__.py";
    else if (cls.rfind("__torch__.", 0) == 0) file = "code/__torch__/" + cls.substr(10, cls.find(' ') - 10) + ".py";
    auto it = files.find(prefix + file);
    if (file.empty() || it == files.end()) return names;
    const std::string& c = it->second;
    const auto b = c.find("__parameters__ = [");
    if (b == std::string::npos) return names;
    const auto e = c.find(']', b);
    size_t q = c.find('"', b);
    while (q != std::string::npos && q < e) {
      const size_t q2 = c.find('"', q + 1);
      if (q2 == std::string::npos) break;
      names.push_back(c.substr(q + 1, q2 - q - 1));
      q = c.find('"', q2 + 1);
    }
    return names;
  };
  std::function<Obj(const PVP&)> conv = [&](const PVP& o) {
    Obj out;
    const auto params = params_of(o->s);
    for (const auto& [k, v] : o->dict) {
      Value val;
      switch (v->kind) {
        case PV::TENSOR:
          val = v->tensor;
          for (const auto& n : params) val.is_param |= n == k->s;
          break;
        case PV::INT: val = int_value(v->i); break;
        case PV::STR: val = str_value(v->s); break;
        case PV::DOUBLE: val = double_value(v->d); break;
        case PV::BOOL: val = bool_value(v->i != 0); break;
        case PV::TUPLE: {
          std::vector<double> dt;
          for (auto& x : v->items) dt.push_back(x->kind == PV::DOUBLE ? x->d : (double)x->i);
          val = double_tuple(dt);
          break;
        }
        case PV::OBJ:
          val.kind = Value::OBJ;
          val.obj = std::make_shared<Obj>(conv(v));
          break;
        default: val.kind = Value::NONE; break;
      }
      out.add(k->s, std::move(val));
    }
    return out;
  };
  return conv(st.back());
}

inline std::string read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("pth: cannot open " + path);
  return std::string((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}
inline Obj read_archive(const std::string& path) { return read_archive_bytes(read_file(path)); }

// ------------------------------------------------------------------------------------------
// agents: module archives and Adam archives over the flat C-ABI vectors
// ------------------------------------------------------------------------------------------
struct Spec {
  struct Tensor {
    std::string name;  // dotted, e.g. "critic.0.weight"
    std::vector<int64_t> shape;
    long off;          // offset in the flat vector
    bool grad;         // requires_grad (false: registered with requires_grad = false)
  };
  std::vector<std::string> modules;  // every submodule path, registration (DFS) order
  std::vector<Tensor> tensors;       // named_parameters() order
  long P = 0;
};

// Module::save: the module's own parameters, then its children (recursively), in registration order.
inline Obj module_tree(const Spec& spec, const float* flat) {
  auto parent_of = [](const std::string& n) {
    const auto dot = n.rfind('.');
    return dot == std::string::npos ? std::string() : n.substr(0, dot);
  };
  auto leaf_of = [](const std::string& n) {
    const auto dot = n.rfind('.');
    return dot == std::string::npos ? n : n.substr(dot + 1);
  };
  std::map<std::string, bool> known{{"", true}};
  for (const std::string& m : spec.modules) {
    if (!known.count(parent_of(m))) throw std::runtime_error("pth: module " + m + " listed before its parent");
    known[m] = true;
  }
  for (const auto& t : spec.tensors)
    if (!known.count(parent_of(t.name))) throw std::runtime_error("pth: parameter " + t.name + " has no module");
  std::function<void(const std::string&, Obj&)> fill = [&](const std::string& path, Obj& o) {
    for (const auto& t : spec.tensors)
      if (parent_of(t.name) == path) o.add(leaf_of(t.name), tensor_f32(t.shape, flat + t.off, t.grad, true));
    for (const std::string& m : spec.modules)
      if (parent_of(m) == path) fill(m, o.child(leaf_of(m)));
  };
  Obj root;
  fill("", root);
  return root;
}

inline void save_module(const std::string& path, const Spec& spec, const float* flat) {
  write_archive(path, module_tree(spec, flat));
}

// torch::load(agent, path): every named parameter must be present with the same shape.
inline std::vector<float> load_module(const std::string& path, const Spec& spec) {
  const Obj root = read_archive(path);
  std::vector<float> flat((size_t)spec.P, 0.0f);
  for (const auto& t : spec.tensors) {
    const Obj* o = &root;
    std::string rest = t.name;
    for (auto dot = rest.find('.'); dot != std::string::npos; dot = rest.find('.')) {
      const Value* c = o->find(rest.substr(0, dot));
      if (!c || c->kind != Value::OBJ) throw std::runtime_error("pth: " + path + " has no module for " + t.name);
      o = c->obj.get();
      rest = rest.substr(dot + 1);
    }
    const Value* v = o->find(rest);
    if (!v || v->kind != Value::TENSOR) throw std::runtime_error("pth: " + path + " has no parameter " + t.name);
    if (v->shape != t.shape) throw std::runtime_error("pth: shape mismatch for " + t.name + " in " + path);
    const auto f = v->floats();
    std::copy(f.begin(), f.end(), flat.begin() + t.off);
  }
  return flat;
}

// Adam archive (torch::optim::Adam::save): state/<key>/{step, exp_avg, exp_avg_sq} for every
// parameter with state, param_groups/size, param_groups/0/params/{size, 0..n-1} = the keys of all
// group parameters in parameters() order, param_groups/0/options. LibTorch's keys are the decimal
// TensorImpl addresses at save time; loading only needs them to match within the file.
struct AdamOptions {
  double lr = 3e-4, beta1 = 0.9, beta2 = 0.999, eps = 1e-8, weight_decay = 0.0;
  bool amsgrad = false;
};

inline std::string adam_key(size_t i) { return std::to_string(94000000000000ull + 64ull * i); }

inline void save_adam(const std::string& path, const Spec& spec, const float* m, const float* v, long step,
                      const AdamOptions& opt) {
  Obj root;
  root.add("pytorch_version", str_value("1.5.0"));
  Obj& state = root.child("state");
  if (step > 0)
    for (size_t i = 0; i < spec.tensors.size(); ++i) {
      const auto& t = spec.tensors[i];
      if (!t.grad) continue;  // no gradient, no Adam state (Adam::step skips it)
      Obj& s = state.child(adam_key(i));
      s.add("step", int_value(step));
      s.add("exp_avg", tensor_f32(t.shape, m + t.off, false, false));
      s.add("exp_avg_sq", tensor_f32(t.shape, v + t.off, false, false));
    }
  Obj& groups = root.child("param_groups");
  groups.add("param_groups/size", tensor_i64_scalar(1, true));
  Obj& g = groups.child("param_groups/0");
  g.add("params/size", tensor_i64_scalar((int64_t)spec.tensors.size(), true));
  for (size_t i = 0; i < spec.tensors.size(); ++i) g.add("params/" + std::to_string(i), str_value(adam_key(i)));
  Obj& o = g.child("options");
  o.add("lr", double_value(opt.lr));
  o.add("betas", double_tuple({opt.beta1, opt.beta2}));
  o.add("eps", double_value(opt.eps));
  o.add("weight_decay", double_value(opt.weight_decay));
  o.add("amsgrad", bool_value(opt.amsgrad));
  write_archive(path, root);
}

// torch::load(optimizer, path): the group's parameter count must match; state is mapped back by
// position in the group. Returns the step of the first parameter with state (0 if none).
inline long load_adam(const std::string& path, const Spec& spec, float* m, float* v, AdamOptions* opt_out = nullptr) {
  const Obj root = read_archive(path);
  const Obj& groups = *root.at("param_groups").obj;
  if (groups.at("param_groups/size").long_scalar() != 1) throw std::runtime_error("pth: expected one param group");
  const Obj& g = *groups.at("param_groups/0").obj;
  const int64_t n = g.at("params/size").long_scalar();
  if (n != (int64_t)spec.tensors.size())
    throw std::runtime_error("pth: optimizer has " + std::to_string(n) + " parameters, the agent " +
                             std::to_string(spec.tensors.size()));
  if (opt_out) {
    const Obj& o = *g.at("options").obj;
    opt_out->lr = o.at("lr").d;
    opt_out->beta1 = o.at("betas").dt.at(0);
    opt_out->beta2 = o.at("betas").dt.at(1);
    opt_out->eps = o.at("eps").d;
    opt_out->weight_decay = o.at("weight_decay").d;
    opt_out->amsgrad = o.at("amsgrad").b;
  }
  std::fill(m, m + spec.P, 0.0f);
  std::fill(v, v + spec.P, 0.0f);
  const Obj& state = *root.at("state").obj;
  long step = 0;
  for (int64_t i = 0; i < n; ++i) {
    const std::string key = g.at("params/" + std::to_string(i)).s;
    const Value* s = state.find(key);
    if (!s) continue;
    const auto& t = spec.tensors[(size_t)i];
    const Value& ea = s->obj->at("exp_avg");
    const Value& es = s->obj->at("exp_avg_sq");
    if (ea.shape != t.shape || es.shape != t.shape) throw std::runtime_error("pth: Adam state shape mismatch for " + t.name);
    const auto fa = ea.floats(), fs = es.floats();
    std::copy(fa.begin(), fa.end(), m + t.off);
    std::copy(fs.begin(), fs.end(), v + t.off);
    const Value& sv = s->obj->at("step");
    const long stp = sv.kind == Value::TENSOR ? (long)(sv.is_long ? sv.long_scalar() : sv.floats().at(0)) : (long)sv.i;
    if (step == 0) step = stp;
  }
  return step;
}

}  // namespace pth
