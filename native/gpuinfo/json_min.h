// Minimal JSON reader used by the fake SMI backend (no third-party headers in the image).
// Supports objects, arrays, strings (with \" \\ \n \t \uXXXX->'?'), numbers, true/false/null.
#pragma once
#include <cctype>
#include <cstdlib>
#include <map>
#include <string>
#include <vector>

namespace jsonmin {

struct Value {
  enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
  bool b = false;
  double num = 0;
  std::string str;
  std::vector<Value> arr;
  std::map<std::string, Value> obj;

  bool is_array() const { return kind == Arr; }
  bool is_string() const { return kind == Str; }
  const Value* get(const std::string& k) const {
    if (kind != Obj) return nullptr;
    auto it = obj.find(k);
    return it == obj.end() ? nullptr : &it->second;
  }
  double num_or(const std::string& k, double d) const {
    const Value* v = get(k);
    return (v && v->kind == Num) ? v->num : d;
  }
};

class Parser {
 public:
  explicit Parser(const std::string& s) : s_(s) {}
  bool parse(Value* v, std::string* err) {
    if (!value(v, 0)) {
      *err = err_ + " at offset " + std::to_string(i_);
      return false;
    }
    ws();
    if (i_ != s_.size()) {
      *err = "trailing characters at offset " + std::to_string(i_);
      return false;
    }
    return true;
  }

 private:
  void ws() {
    while (i_ < s_.size() && isspace((unsigned char)s_[i_])) ++i_;
  }
  bool fail(const char* m) {
    err_ = m;
    return false;
  }
  bool lit(const char* w) {
    size_t n = std::char_traits<char>::length(w);
    if (s_.compare(i_, n, w) != 0) return false;
    i_ += n;
    return true;
  }
  bool string(std::string* out) {
    if (s_[i_] != '"') return fail("expected string");
    ++i_;
    while (i_ < s_.size() && s_[i_] != '"') {
      char c = s_[i_++];
      if (c == '\\') {
        if (i_ >= s_.size()) return fail("bad escape");
        char e = s_[i_++];
        switch (e) {
          case 'n': out->push_back('\n'); break;
          case 't': out->push_back('\t'); break;
          case 'r': out->push_back('\r'); break;
          case 'b': out->push_back('\b'); break;
          case 'f': out->push_back('\f'); break;
          case 'u':
            if (i_ + 4 > s_.size()) return fail("bad \\u escape");
            i_ += 4;
            out->push_back('?');
            break;
          default: out->push_back(e);
        }
      } else {
        out->push_back(c);
      }
    }
    if (i_ >= s_.size()) return fail("unterminated string");
    ++i_;
    return true;
  }
  bool value(Value* v, int depth) {
    if (depth > 64) return fail("nesting too deep");
    ws();
    if (i_ >= s_.size()) return fail("unexpected end");
    char c = s_[i_];
    if (c == '{') {
      v->kind = Value::Obj;
      ++i_;
      ws();
      if (i_ < s_.size() && s_[i_] == '}') return ++i_, true;
      while (true) {
        ws();
        std::string k;
        if (i_ >= s_.size() || !string(&k)) return fail("expected key");
        ws();
        if (i_ >= s_.size() || s_[i_] != ':') return fail("expected ':'");
        ++i_;
        if (!value(&v->obj[k], depth + 1)) return false;
        ws();
        if (i_ < s_.size() && s_[i_] == ',') {
          ++i_;
          continue;
        }
        if (i_ < s_.size() && s_[i_] == '}') return ++i_, true;
        return fail("expected ',' or '}'");
      }
    }
    if (c == '[') {
      v->kind = Value::Arr;
      ++i_;
      ws();
      if (i_ < s_.size() && s_[i_] == ']') return ++i_, true;
      while (true) {
        v->arr.emplace_back();
        if (!value(&v->arr.back(), depth + 1)) return false;
        ws();
        if (i_ < s_.size() && s_[i_] == ',') {
          ++i_;
          continue;
        }
        if (i_ < s_.size() && s_[i_] == ']') return ++i_, true;
        return fail("expected ',' or ']'");
      }
    }
    if (c == '"') {
      v->kind = Value::Str;
      return string(&v->str);
    }
    if (lit("true")) return v->kind = Value::Bool, v->b = true, true;
    if (lit("false")) return v->kind = Value::Bool, v->b = false, true;
    if (lit("null")) return v->kind = Value::Null, true;
    const char* start = s_.c_str() + i_;
    char* end = nullptr;
    double d = strtod(start, &end);
    if (end == start) return fail("unexpected character");
    i_ += (size_t)(end - start);
    v->kind = Value::Num;
    v->num = d;
    return true;
  }
  const std::string& s_;
  size_t i_ = 0;
  std::string err_;
};

inline bool parse(const std::string& s, Value* v, std::string* err) { return Parser(s).parse(v, err); }

inline std::string escape(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '"' || c == '\\') o.push_back('\\'), o.push_back(c);
    else if ((unsigned char)c < 0x20) o.push_back(' ');
    else o.push_back(c);
  }
  return o;
}

}  // namespace jsonmin
