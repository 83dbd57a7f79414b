// apps/json_flat.h — reader for the flat config.json the CaRL tools write and read
// (carla_config.h:379-497 to_json / update_from_json with json_spirit): a top-level object whose
// values are numbers, strings, booleans, null, or arrays / objects (kept as raw text). No LibTorch,
// no json_spirit; enough for GlobalConfig-style files.
#pragma once

#include <cctype>
#include <fstream>
#include <map>
#include <sstream>
#include <stdexcept>
#include <string>

namespace app {

class FlatJson {
 public:
  static FlatJson parse_file(const std::string& path) {
    std::ifstream f(path);
    if (!f) throw std::runtime_error("Could not open the file: " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    return parse(ss.str());
  }
  static FlatJson parse(const std::string& text) {
    FlatJson j;
    size_t i = 0;
    ws(text, i);
    expect(text, i, '{');
    ws(text, i);
    if (peek(text, i) == '}') return j;
    for (;;) {
      ws(text, i);
      const std::string key = string_lit(text, i);
      ws(text, i);
      expect(text, i, ':');
      ws(text, i);
      j.values_[key] = value_text(text, i);
      ws(text, i);
      const char c = peek(text, i);
      ++i;
      if (c == '}') break;
      if (c != ',') throw std::runtime_error("config json: expected ',' or '}'");
    }
    return j;
  }

  bool has(const std::string& k) const { return values_.count(k) != 0; }
  // raw JSON text of a value (strings keep their quotes)
  const std::string& raw(const std::string& k) const { return values_.at(k); }
  int get_int(const std::string& k, int def) const { return has(k) ? (int)std::stol(raw(k)) : def; }
  float get_float(const std::string& k, float def) const { return has(k) ? std::stof(raw(k)) : def; }
  bool get_bool(const std::string& k, bool def) const {
    if (!has(k)) return def;
    const std::string& v = raw(k);
    return v == "true" || v == "1";
  }
  std::string get_string(const std::string& k, const std::string& def) const {
    if (!has(k)) return def;
    size_t i = 0;
    const std::string& v = raw(k);
    return v.empty() || v[0] != '"' ? v : string_lit(v, i);
  }

 private:
  std::map<std::string, std::string> values_;

  static char peek(const std::string& s, size_t i) {
    if (i >= s.size()) throw std::runtime_error("config json: unexpected end");
    return s[i];
  }
  static void ws(const std::string& s, size_t& i) {
    while (i < s.size() && std::isspace((unsigned char)s[i])) ++i;
  }
  static void expect(const std::string& s, size_t& i, char c) {
    if (peek(s, i) != c) throw std::runtime_error(std::string("config json: expected '") + c + "'");
    ++i;
  }
  static std::string string_lit(const std::string& s, size_t& i) {
    expect(s, i, '"');
    std::string out;
    for (;;) {
      const char c = peek(s, i++);
      if (c == '"') return out;
      if (c == '\\') {
        const char e = peek(s, i++);
        switch (e) {
          case 'n': out += '\n'; break;
          case 't': out += '\t'; break;
          case 'r': out += '\r'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'u': i += 4; out += '?'; break;  // non-ASCII escapes are not needed by these configs
          default: out += e;
        }
      } else {
        out += c;
      }
    }
  }
  // the raw text of one value (balanced for arrays / objects)
  static std::string value_text(const std::string& s, size_t& i) {
    const size_t b = i;
    const char c = peek(s, i);
    if (c == '"') {
      string_lit(s, i);
      return s.substr(b, i - b);
    }
    if (c == '[' || c == '{') {
      int depth = 0;
      bool in_str = false;
      for (; i < s.size(); ++i) {
        const char d = s[i];
        if (in_str) {
          if (d == '\\') ++i;
          else if (d == '"') in_str = false;
          continue;
        }
        if (d == '"') in_str = true;
        else if (d == '[' || d == '{') ++depth;
        else if (d == ']' || d == '}') {
          if (--depth == 0) {
            ++i;
            return s.substr(b, i - b);
          }
        }
      }
      throw std::runtime_error("config json: unbalanced value");
    }
    while (i < s.size() && s[i] != ',' && s[i] != '}' && !std::isspace((unsigned char)s[i])) ++i;
    return s.substr(b, i - b);
  }
};

}  // namespace app
