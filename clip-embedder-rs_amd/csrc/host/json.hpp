// Minimal JSON reader for the model-dir files (open_clip_config.json,
// model_config.json, tokenizer.json, safetensors headers).  Replaces the
// reference's serde_json use (src/config.rs:16-21, :66-71).
#pragma once
#include <cstdint>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace clipgpu {
namespace json {

struct Value;
typedef std::shared_ptr<Value> ValuePtr;

struct Value {
  enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
  bool b = false;
  double num = 0.0;
  std::string str;
  std::vector<ValuePtr> arr;
  // insertion-ordered object (tokenizer.json vocab order does not matter, but
  // keep keys unique and lookups O(log n))
  std::vector<std::pair<std::string, ValuePtr>> items;
  std::map<std::string, size_t> index;

  bool is_null() const { return kind == NUL; }
  const Value* get(const std::string& k) const {
    if (kind != OBJ) return nullptr;
    auto it = index.find(k);
    return it == index.end() ? nullptr : items[it->second].second.get();
  }
  double as_num(double dflt) const { return kind == NUM ? num : dflt; }
  std::string as_str(const std::string& dflt) const { return kind == STR ? str : dflt; }
  bool as_bool(bool dflt) const { return kind == BOOL ? b : dflt; }
};

class Parser {
 public:
  explicit Parser(const std::string& s) : s_(s), i_(0) {}
  ValuePtr parse() {
    ValuePtr v = value();
    ws();
    if (i_ != s_.size()) fail("trailing characters");
    return v;
  }

 private:
  const std::string& s_;
  size_t i_;

  [[noreturn]] void fail(const char* what) {
    throw std::runtime_error(std::string("JSON parse error: ") + what + " at offset " + std::to_string(i_));
  }
  void ws() {
    while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\n' || s_[i_] == '\r' || s_[i_] == '\t')) ++i_;
  }
  char peek() {
    ws();
    if (i_ >= s_.size()) fail("unexpected end");
    return s_[i_];
  }
  void expect(char c) {
    if (peek() != c) fail("unexpected character");
    ++i_;
  }
  static void put_utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) {
      out += (char)cp;
    } else if (cp < 0x800) {
      out += (char)(0xC0 | (cp >> 6));
      out += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      out += (char)(0xE0 | (cp >> 12));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    } else {
      out += (char)(0xF0 | (cp >> 18));
      out += (char)(0x80 | ((cp >> 12) & 0x3F));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (i_ + 4 > s_.size()) fail("bad \\u escape");
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = s_[i_++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex digit");
    }
    return v;
  }
  std::string string_lit() {
    expect('"');
    std::string out;
    while (true) {
      if (i_ >= s_.size()) fail("unterminated string");
      char c = s_[i_++];
      if (c == '"') break;
      if (c != '\\') {
        out += c;
        continue;
      }
      if (i_ >= s_.size()) fail("bad escape");
      char e = s_[i_++];
      switch (e) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && i_ + 1 < s_.size() && s_[i_] == '\\' && s_[i_ + 1] == 'u') {
            i_ += 2;
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    return out;
  }
  ValuePtr value() {
    char c = peek();
    auto v = std::make_shared<Value>();
    if (c == '{') {
      ++i_;
      v->kind = Value::OBJ;
      if (peek() == '}') { ++i_; return v; }
      while (true) {
        std::string k = string_lit();
        expect(':');
        ValuePtr item = value();
        auto it = v->index.find(k);
        if (it == v->index.end()) {
          v->index[k] = v->items.size();
          v->items.emplace_back(k, item);
        } else {
          v->items[it->second].second = item;
        }
        char d = peek();
        ++i_;
        if (d == '}') break;
        if (d != ',') fail("expected , or }");
      }
    } else if (c == '[') {
      ++i_;
      v->kind = Value::ARR;
      if (peek() == ']') { ++i_; return v; }
      while (true) {
        v->arr.push_back(value());
        char d = peek();
        ++i_;
        if (d == ']') break;
        if (d != ',') fail("expected , or ]");
      }
    } else if (c == '"') {
      v->kind = Value::STR;
      v->str = string_lit();
    } else if (c == 't' && s_.compare(i_, 4, "true") == 0) {
      i_ += 4; v->kind = Value::BOOL; v->b = true;
    } else if (c == 'f' && s_.compare(i_, 5, "false") == 0) {
      i_ += 5; v->kind = Value::BOOL; v->b = false;
    } else if (c == 'n' && s_.compare(i_, 4, "null") == 0) {
      i_ += 4; v->kind = Value::NUL;
    } else {
      const char* start = s_.c_str() + i_;
      char* end = nullptr;
      v->num = std::strtod(start, &end);
      if (end == start) fail("bad value");
      i_ += (size_t)(end - start);
      v->kind = Value::NUM;
    }
    return v;
  }
};

inline ValuePtr parse(const std::string& s) { return Parser(s).parse(); }
ValuePtr parse_file(const std::string& path);  // host/config.cpp

}  // namespace json
}  // namespace clipgpu
