// toml.h — the subset of TOML the reference's res/*.toml files use: [tables],
// [[arrays of tables]], bare or quoted keys, basic/literal strings, integers, floats, booleans
// and (multi-line) arrays. toml-f, the reference's parser, is an un-vendored dependency;
// only its lookup semantics are restated here (get_value with a default, integer -> real
// promotion).
#pragma once
#include <cctype>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace smcrt {
namespace toml {

struct Value;
using Table = std::map<std::string, Value>;

struct Value {
  enum Kind { NONE, STRING, INT, FLOAT, BOOL, ARRAY, TABLE, TABLE_ARRAY } kind = NONE;
  std::string s;
  int64_t i = 0;
  double f = 0.0;
  bool b = false;
  std::vector<Value> arr;          // ARRAY, TABLE_ARRAY (elements are TABLE)
  std::shared_ptr<Table> table;    // TABLE
  int line = 0;

  bool is_number() const { return kind == INT || kind == FLOAT; }
  double number() const { return kind == INT ? (double)i : f; }
};

struct ParseError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class Parser {
 public:
  explicit Parser(const std::string& text) : t_(text) {}

  Table parse() {
    Table root;
    Table* cur = &root;
    while (skip_ws_nl(), pos_ < t_.size()) {
      if (t_[pos_] == '[') {
        const bool arr = pos_ + 1 < t_.size() && t_[pos_ + 1] == '[';
        pos_ += arr ? 2 : 1;
        skip_ws();
        std::vector<std::string> path = key_path();
        skip_ws();
        expect(']');
        if (arr) expect(']');
        end_of_line();
        cur = open_table(root, path, arr);
      } else {
        std::vector<std::string> path = key_path();
        skip_ws();
        expect('=');
        skip_ws();
        Value v = value();
        Table* t = cur;
        for (size_t k = 0; k + 1 < path.size(); ++k) t = sub_table(*t, path[k]);
        if (t->count(path.back())) fail("duplicate key '" + path.back() + "'");
        (*t)[path.back()] = std::move(v);
        end_of_line();
      }
    }
    return root;
  }

 private:
  const std::string& t_;
  size_t pos_ = 0;
  int line_ = 1;

  [[noreturn]] void fail(const std::string& m) const {
    throw ParseError("TOML line " + std::to_string(line_) + ": " + m);
  }
  void expect(char c) {
    if (pos_ >= t_.size() || t_[pos_] != c) fail(std::string("expected '") + c + "'");
    ++pos_;
  }
  void skip_ws() {
    while (pos_ < t_.size() && (t_[pos_] == ' ' || t_[pos_] == '\t')) ++pos_;
  }
  void skip_comment() {
    if (pos_ < t_.size() && t_[pos_] == '#')
      while (pos_ < t_.size() && t_[pos_] != '\n') ++pos_;
  }
  void skip_ws_nl() {
    for (;;) {
      skip_ws();
      skip_comment();
      if (pos_ < t_.size() && (t_[pos_] == '\n' || t_[pos_] == '\r')) {
        if (t_[pos_] == '\n') ++line_;
        ++pos_;
        continue;
      }
      return;
    }
  }
  void end_of_line() {
    skip_ws();
    skip_comment();
    if (pos_ < t_.size() && t_[pos_] == '\r') ++pos_;
    if (pos_ < t_.size()) {
      if (t_[pos_] != '\n') fail("unexpected text after value");
      ++pos_;
      ++line_;
    }
  }
  static bool bare(char c) { return std::isalnum((unsigned char)c) || c == '_' || c == '-'; }
  std::string key() {
    if (pos_ < t_.size() && (t_[pos_] == '"' || t_[pos_] == '\'')) return string_value();
    const size_t b = pos_;
    while (pos_ < t_.size() && bare(t_[pos_])) ++pos_;
    if (b == pos_) fail("expected a key");
    return t_.substr(b, pos_ - b);
  }
  std::vector<std::string> key_path() {
    std::vector<std::string> p{key()};
    for (;;) {
      skip_ws();
      if (pos_ < t_.size() && t_[pos_] == '.') {
        ++pos_;
        skip_ws();
        p.push_back(key());
      } else {
        return p;
      }
    }
  }
  std::string string_value() {
    const char q = t_[pos_++];
    std::string out;
    while (pos_ < t_.size() && t_[pos_] != q) {
      char c = t_[pos_++];
      if (c == '\n') fail("newline in string");
      if (q == '"' && c == '\\') {
        if (pos_ >= t_.size()) fail("bad escape");
        const char e = t_[pos_++];
        switch (e) {
          case 'n': c = '\n'; break;
          case 't': c = '\t'; break;
          case '"': c = '"'; break;
          case '\\': c = '\\'; break;
          default: fail(std::string("unsupported escape \\") + e);
        }
      }
      out += c;
    }
    expect(q);
    return out;
  }
  Value value() {
    Value v;
    v.line = line_;
    if (pos_ >= t_.size()) fail("missing value");
    const char c = t_[pos_];
    if (c == '"' || c == '\'') {
      v.kind = Value::STRING;
      v.s = string_value();
      return v;
    }
    if (c == '[') {
      ++pos_;
      v.kind = Value::ARRAY;
      for (;;) {
        skip_ws_nl();
        if (pos_ < t_.size() && t_[pos_] == ']') { ++pos_; return v; }
        v.arr.push_back(value());
        skip_ws_nl();
        if (pos_ < t_.size() && t_[pos_] == ',') { ++pos_; continue; }
        skip_ws_nl();
        expect(']');
        return v;
      }
    }
    const size_t b = pos_;
    while (pos_ < t_.size() && !std::strchr(" \t\r\n,]#", t_[pos_])) ++pos_;
    std::string tok = t_.substr(b, pos_ - b);
    if (tok == "true" || tok == "false") {
      v.kind = Value::BOOL;
      v.b = tok == "true";
      return v;
    }
    std::string clean;
    for (char ch : tok)
      if (ch != '_') clean += ch;
    if (clean == "inf" || clean == "+inf" || clean == "-inf" || clean == "nan" || clean == "+nan" || clean == "-nan") {
      v.kind = Value::FLOAT;
      v.f = clean.find("nan") != std::string::npos ? NAN : (clean[0] == '-' ? -INFINITY : INFINITY);
      return v;
    }
    const bool is_float = clean.find_first_of(".eE") != std::string::npos;
    char* end = nullptr;
    if (is_float) {
      v.kind = Value::FLOAT;
      v.f = std::strtod(clean.c_str(), &end);
    } else {
      v.kind = Value::INT;
      v.i = std::strtoll(clean.c_str(), &end, 10);
    }
    if (clean.empty() || end != clean.c_str() + clean.size()) fail("cannot read value '" + tok + "'");
    return v;
  }
  Table* sub_table(Table& t, const std::string& k) {
    Value& v = t[k];
    if (v.kind == Value::NONE) {
      v.kind = Value::TABLE;
      v.table = std::make_shared<Table>();
    }
    if (v.kind == Value::TABLE_ARRAY) return v.arr.back().table.get();
    if (v.kind != Value::TABLE) fail("'" + k + "' is not a table");
    return v.table.get();
  }
  Table* open_table(Table& root, const std::vector<std::string>& path, bool arr) {
    Table* t = &root;
    for (size_t k = 0; k + 1 < path.size(); ++k) t = sub_table(*t, path[k]);
    Value& v = (*t)[path.back()];
    if (!arr) {
      if (v.kind == Value::NONE) {
        v.kind = Value::TABLE;
        v.table = std::make_shared<Table>();
      } else if (v.kind != Value::TABLE) {
        fail("'" + path.back() + "' redefined");
      }
      return v.table.get();
    }
    if (v.kind == Value::NONE) v.kind = Value::TABLE_ARRAY;
    if (v.kind != Value::TABLE_ARRAY) fail("'" + path.back() + "' is not an array of tables");
    Value e;
    e.kind = Value::TABLE;
    e.table = std::make_shared<Table>();
    v.arr.push_back(e);
    return v.arr.back().table.get();
  }
};

// get_value(table, key, var, default): the value if present (an integer is accepted where a
// real is asked for, as toml-f does), else the default.
inline const Value* find(const Table* t, const std::string& k) {
  if (!t) return nullptr;
  auto it = t->find(k);
  return it == t->end() ? nullptr : &it->second;
}
inline double get_real(const Table* t, const std::string& k, double def) {
  const Value* v = find(t, k);
  if (!v) return def;
  if (!v->is_number()) throw ParseError("'" + k + "' must be a number");
  return v->number();
}
inline int64_t get_int(const Table* t, const std::string& k, int64_t def) {
  const Value* v = find(t, k);
  if (!v) return def;
  if (v->kind != Value::INT) throw ParseError("'" + k + "' must be an integer");
  return v->i;
}
inline bool get_bool(const Table* t, const std::string& k, bool def) {
  const Value* v = find(t, k);
  if (!v) return def;
  if (v->kind != Value::BOOL) throw ParseError("'" + k + "' must be true or false");
  return v->b;
}
inline std::string get_string(const Table* t, const std::string& k, const std::string& def) {
  const Value* v = find(t, k);
  if (!v) return def;
  if (v->kind != Value::STRING) throw ParseError("'" + k + "' must be a string");
  return v->s;
}
inline const Table* get_table(const Table* t, const std::string& k) {
  const Value* v = find(t, k);
  return v && v->kind == Value::TABLE ? v->table.get() : nullptr;
}

}  // namespace toml
}  // namespace smcrt
