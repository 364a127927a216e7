#include "core/caps.h"

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <numeric>

#include "core/util.h"

namespace nnsx {

// ---------------------------------------------------------------- Value ----

namespace {

int frac_cmp(int64_t an, int64_t ad, int64_t bn, int64_t bd) {
  // compare an/ad vs bn/bd, denominators positive
  if (ad < 0) { an = -an; ad = -ad; }
  if (bd < 0) { bn = -bn; bd = -bd; }
  __int128 l = static_cast<__int128>(an) * bd;
  __int128 r = static_cast<__int128>(bn) * ad;
  return l < r ? -1 : (l > r ? 1 : 0);
}

bool is_tensor_dim_field(const std::string& f) { return f == "dimension" || f == "dimensions"; }
bool is_tensor_type_field(const std::string& f) { return f == "type" || f == "types"; }

// "float32.int32" and "float32,int32" name the same type list
bool type_string_equal(const std::string& a, const std::string& b) {
  auto pa = split_any(a, ",."), pb = split_any(b, ",.");
  if (pa.size() != pb.size()) return false;
  for (size_t i = 0; i < pa.size(); ++i)
    if (lower(strip(pa[i])) != lower(strip(pb[i]))) return false;
  return true;
}

bool needs_quotes(const std::string& s) {
  if (s.empty()) return true;
  for (char c : s) {
    if (!(std::isalnum(static_cast<unsigned char>(c)) || c == '_' || c == '-' || c == '+' || c == '.' || c == '/' ||
          c == ':'))
      return true;
  }
  return false;
}

std::string quote(const std::string& s) {
  std::string r = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') r += '\\';
    r += c;
  }
  r += '"';
  return r;
}

}  // namespace

bool Value::is_fixed() const {
  switch (kind) {
    case Kind::INT_RANGE:
    case Kind::FRACTION_RANGE:
    case Kind::DOUBLE_RANGE:
    case Kind::NONE:
      return false;
    case Kind::LIST:
      return list.size() == 1 && list[0].is_fixed();
    default:
      return true;
  }
}

static std::string frac_str(int64_t n, int64_t d) {
  if (n == INT_MAX && d == 1) return "2147483647/1";
  return std::to_string(n) + "/" + std::to_string(d);
}

std::string Value::to_string(bool with_type) const {
  switch (kind) {
    case Kind::INT: return (with_type ? "(int)" : "") + std::to_string(i);
    case Kind::DOUBLE: {
      char buf[64];
      snprintf(buf, sizeof(buf), "%g", d);
      return (with_type ? "(double)" : "") + std::string(buf);
    }
    case Kind::BOOL: return (with_type ? "(boolean)" : "") + std::string(b ? "true" : "false");
    case Kind::STRING: return (with_type ? "(string)" : "") + (needs_quotes(s) ? quote(s) : s);
    case Kind::FRACTION: return (with_type ? "(fraction)" : "") + frac_str(i, i2);
    case Kind::INT_RANGE:
      return (with_type ? "(int)" : "") + std::string("[ ") + std::to_string(i) + ", " + std::to_string(i2) + " ]";
    case Kind::DOUBLE_RANGE: {
      char buf[128];
      snprintf(buf, sizeof(buf), "[ %g, %g ]", d, d2);
      return (with_type ? "(double)" : "") + std::string(buf);
    }
    case Kind::FRACTION_RANGE:
      return (with_type ? "(fraction)" : "") + std::string("[ ") + frac_str(f1n, f1d) + ", " + frac_str(f2n, f2d) +
             " ]";
    case Kind::LIST: {
      std::string prefix;
      if (with_type && !list.empty()) {
        switch (list[0].kind) {
          case Kind::INT: prefix = "(int)"; break;
          case Kind::STRING: prefix = "(string)"; break;
          case Kind::FRACTION: prefix = "(fraction)"; break;
          case Kind::DOUBLE: prefix = "(double)"; break;
          case Kind::BOOL: prefix = "(boolean)"; break;
          default: break;
        }
      }
      std::string r = prefix + "{ ";
      for (size_t k = 0; k < list.size(); ++k) {
        if (k) r += ", ";
        r += list[k].to_string(false);
      }
      return r + " }";
    }
    default: return "";
  }
}

bool Value::operator==(const Value& o) const {
  if (kind != o.kind) return false;
  switch (kind) {
    case Kind::INT: return i == o.i;
    case Kind::DOUBLE: return d == o.d;
    case Kind::BOOL: return b == o.b;
    case Kind::STRING: return s == o.s;
    case Kind::FRACTION: return frac_cmp(i, i2, o.i, o.i2) == 0;
    case Kind::INT_RANGE: return i == o.i && i2 == o.i2;
    case Kind::DOUBLE_RANGE: return d == o.d && d2 == o.d2;
    case Kind::FRACTION_RANGE:
      return frac_cmp(f1n, f1d, o.f1n, o.f1d) == 0 && frac_cmp(f2n, f2d, o.f2n, o.f2d) == 0;
    case Kind::LIST: return list == o.list;
    default: return true;
  }
}

bool Value::intersect(const Value& a, const Value& b, Value* out, const std::string& field) {
  if (a.kind == Kind::LIST || b.kind == Kind::LIST) {
    const Value& l = a.kind == Kind::LIST ? a : b;
    const Value& o = a.kind == Kind::LIST ? b : a;
    std::vector<Value> res;
    for (const auto& e : l.list) {
      Value r;
      if (intersect(e, o, &r, field)) {
        if (r.kind == Kind::LIST)
          for (auto& x : r.list) res.push_back(x);
        else
          res.push_back(r);
      }
    }
    if (res.empty()) return false;
    *out = res.size() == 1 ? res[0] : Value::List(res);
    return true;
  }
  // make a the "fixed" side when one is a range
  auto is_range = [](const Value& v) {
    return v.kind == Kind::INT_RANGE || v.kind == Kind::FRACTION_RANGE || v.kind == Kind::DOUBLE_RANGE;
  };
  if (is_range(a) && !is_range(b)) return intersect(b, a, out, field);

  switch (a.kind) {
    case Kind::INT:
      if (b.kind == Kind::INT) {
        if (a.i != b.i) return false;
        *out = a;
        return true;
      }
      if (b.kind == Kind::INT_RANGE) {
        if (a.i < b.i || a.i > b.i2) return false;
        *out = a;
        return true;
      }
      if (b.kind == Kind::DOUBLE && static_cast<double>(a.i) == b.d) {
        *out = a;
        return true;
      }
      return false;
    case Kind::DOUBLE:
      if (b.kind == Kind::DOUBLE) {
        if (a.d != b.d) return false;
        *out = a;
        return true;
      }
      if (b.kind == Kind::DOUBLE_RANGE) {
        if (a.d < b.d || a.d > b.d2) return false;
        *out = a;
        return true;
      }
      if (b.kind == Kind::INT && static_cast<double>(b.i) == a.d) {
        *out = b;
        return true;
      }
      return false;
    case Kind::BOOL:
      if (b.kind != Kind::BOOL || a.b != b.b) return false;
      *out = a;
      return true;
    case Kind::STRING:
      if (b.kind != Kind::STRING) return false;
      if (is_tensor_dim_field(field)) {
        if (!dimension_string_equal(a.s, b.s)) return false;
      } else if (is_tensor_type_field(field)) {
        if (!type_string_equal(a.s, b.s)) return false;
      } else if (a.s != b.s) {
        return false;
      }
      *out = a;
      return true;
    case Kind::FRACTION:
      if (b.kind == Kind::FRACTION) {
        if (frac_cmp(a.i, a.i2, b.i, b.i2) != 0) return false;
        *out = a;
        return true;
      }
      if (b.kind == Kind::FRACTION_RANGE) {
        if (frac_cmp(a.i, a.i2, b.f1n, b.f1d) < 0 || frac_cmp(a.i, a.i2, b.f2n, b.f2d) > 0) return false;
        *out = a;
        return true;
      }
      if (b.kind == Kind::INT && a.i2 != 0 && a.i == b.i * a.i2) {
        *out = a;
        return true;
      }
      return false;
    case Kind::INT_RANGE:
      if (b.kind == Kind::INT_RANGE) {
        int64_t lo = std::max(a.i, b.i), hi = std::min(a.i2, b.i2);
        if (lo > hi) return false;
        *out = lo == hi ? Value::Int(lo) : Value::IntRange(lo, hi);
        return true;
      }
      return false;
    case Kind::DOUBLE_RANGE:
      if (b.kind == Kind::DOUBLE_RANGE) {
        double lo = std::max(a.d, b.d), hi = std::min(a.d2, b.d2);
        if (lo > hi) return false;
        *out = lo == hi ? Value::Double(lo) : Value::DoubleRange(lo, hi);
        return true;
      }
      return false;
    case Kind::FRACTION_RANGE:
      if (b.kind == Kind::FRACTION_RANGE) {
        int64_t ln = a.f1n, ld = a.f1d, hn = a.f2n, hd = a.f2d;
        if (frac_cmp(b.f1n, b.f1d, ln, ld) > 0) { ln = b.f1n; ld = b.f1d; }
        if (frac_cmp(b.f2n, b.f2d, hn, hd) < 0) { hn = b.f2n; hd = b.f2d; }
        int c = frac_cmp(ln, ld, hn, hd);
        if (c > 0) return false;
        *out = c == 0 ? Value::Fraction(ln, ld) : Value::FractionRange(ln, ld, hn, hd);
        return true;
      }
      return false;
    default:
      return false;
  }
}

Value Value::fixate() const {
  switch (kind) {
    case Kind::LIST: return list.empty() ? Value() : list[0].fixate();
    case Kind::INT_RANGE: return Value::Int(i);
    case Kind::DOUBLE_RANGE: return Value::Double(d);
    case Kind::FRACTION_RANGE: return Value::Fraction(f1n, f1d);
    default: return *this;
  }
}

// ------------------------------------------------------------ Structure ----

bool Structure::has_feature(const std::string& f) const {
  return std::find(features_.begin(), features_.end(), f) != features_.end();
}

bool Structure::has(const std::string& field) const { return get(field) != nullptr; }

const Value* Structure::get(const std::string& field) const {
  for (const auto& kv : fields_)
    if (kv.first == field) return &kv.second;
  return nullptr;
}

void Structure::set(const std::string& field, Value v) {
  for (auto& kv : fields_) {
    if (kv.first == field) {
      kv.second = std::move(v);
      return;
    }
  }
  fields_.emplace_back(field, std::move(v));
}

void Structure::remove(const std::string& field) {
  fields_.erase(std::remove_if(fields_.begin(), fields_.end(), [&](auto& kv) { return kv.first == field; }),
                fields_.end());
}

bool Structure::get_int(const std::string& f, int64_t* v) const {
  const Value* x = get(f);
  if (!x) return false;
  if (x->kind == Value::Kind::INT) {
    *v = x->i;
    return true;
  }
  if (x->kind == Value::Kind::LIST && x->list.size() == 1 && x->list[0].kind == Value::Kind::INT) {
    *v = x->list[0].i;
    return true;
  }
  return false;
}

bool Structure::get_string(const std::string& f, std::string* v) const {
  const Value* x = get(f);
  if (!x) return false;
  if (x->kind == Value::Kind::STRING) {
    *v = x->s;
    return true;
  }
  if (x->kind == Value::Kind::LIST && x->list.size() == 1 && x->list[0].kind == Value::Kind::STRING) {
    *v = x->list[0].s;
    return true;
  }
  return false;
}

bool Structure::get_fraction(const std::string& f, int* n, int* d) const {
  const Value* x = get(f);
  if (!x) return false;
  if (x->kind == Value::Kind::FRACTION) {
    *n = static_cast<int>(x->i);
    *d = static_cast<int>(x->i2);
    return true;
  }
  return false;
}

bool Structure::get_bool(const std::string& f, bool* v) const {
  const Value* x = get(f);
  if (!x || x->kind != Value::Kind::BOOL) return false;
  *v = x->b;
  return true;
}

bool Structure::get_double(const std::string& f, double* v) const {
  const Value* x = get(f);
  if (!x) return false;
  if (x->kind == Value::Kind::DOUBLE) {
    *v = x->d;
    return true;
  }
  if (x->kind == Value::Kind::INT) {
    *v = static_cast<double>(x->i);
    return true;
  }
  return false;
}

std::string Structure::get_string_or(const std::string& f, const std::string& def) const {
  std::string v;
  return get_string(f, &v) ? v : def;
}

int64_t Structure::get_int_or(const std::string& f, int64_t def) const {
  int64_t v;
  return get_int(f, &v) ? v : def;
}

bool Structure::is_fixed() const {
  for (const auto& kv : fields_)
    if (!kv.second.is_fixed()) return false;
  return true;
}

std::string Structure::to_string(bool with_types) const {
  std::string r = name_;
  if (!features_.empty()) r += "(" + join(features_, ", ") + ")";
  for (const auto& kv : fields_) {
    Value v = kv.second;
    if (v.kind == Value::Kind::LIST && v.list.size() == 1) v = v.list[0];
    r += ", " + kv.first + "=" + v.to_string(with_types);
  }
  return r;
}

bool Structure::intersect(const Structure& a, const Structure& b, Structure* out) {
  if (a.name_ != b.name_) return false;
  Structure r(a.name_);
  // features are informative for placement (runtime maps memory on demand): union them
  r.features_ = a.features_;
  for (const auto& f : b.features_)
    if (!r.has_feature(f)) r.features_.push_back(f);
  for (const auto& kv : a.fields_) {
    const Value* bv = b.get(kv.first);
    if (!bv) {
      r.fields_.push_back(kv);
      continue;
    }
    Value res;
    if (!Value::intersect(kv.second, *bv, &res, kv.first)) return false;
    r.fields_.emplace_back(kv.first, res);
  }
  for (const auto& kv : b.fields_)
    if (!a.get(kv.first)) r.fields_.push_back(kv);
  *out = std::move(r);
  return true;
}

void Structure::fixate() {
  for (auto& kv : fields_) kv.second = kv.second.fixate();
}

void Structure::fixate_nearest_int(const std::string& f, int64_t target) {
  const Value* v = get(f);
  if (!v) return;
  if (v->kind == Value::Kind::INT_RANGE) {
    set(f, Value::Int(std::min(std::max(target, v->i), v->i2)));
  } else if (v->kind == Value::Kind::LIST) {
    int64_t best = 0;
    int64_t bestd = INT64_MAX;
    bool found = false;
    for (const auto& e : v->list) {
      int64_t cand;
      if (e.kind == Value::Kind::INT)
        cand = e.i;
      else if (e.kind == Value::Kind::INT_RANGE)
        cand = std::min(std::max(target, e.i), e.i2);
      else
        continue;
      int64_t dd = std::llabs(cand - target);
      if (dd < bestd) {
        bestd = dd;
        best = cand;
        found = true;
      }
    }
    if (found) set(f, Value::Int(best));
  }
}

void Structure::fixate_nearest_fraction(const std::string& f, int n, int d) {
  const Value* v = get(f);
  if (!v) return;
  if (v->kind == Value::Kind::FRACTION_RANGE) {
    if (frac_cmp(n, d, v->f1n, v->f1d) < 0)
      set(f, Value::Fraction(v->f1n, v->f1d));
    else if (frac_cmp(n, d, v->f2n, v->f2d) > 0)
      set(f, Value::Fraction(v->f2n, v->f2d));
    else
      set(f, Value::Fraction(n, d));
  } else if (v->kind == Value::Kind::LIST) {
    for (const auto& e : v->list) {
      if (e.kind == Value::Kind::FRACTION && frac_cmp(e.i, e.i2, n, d) == 0) {
        set(f, e);
        return;
      }
    }
    set(f, v->fixate());
  }
}

void Structure::fixate_string(const std::string& f, const std::string& target) {
  const Value* v = get(f);
  if (!v || v->kind != Value::Kind::LIST) return;
  for (const auto& e : v->list) {
    if (e.kind == Value::Kind::STRING && e.s == target) {
      set(f, e);
      return;
    }
  }
  set(f, v->fixate());
}

// ----------------------------------------------------------------- Caps ----

namespace {

struct CapsParser {
  const std::string& s;
  size_t p = 0;
  explicit CapsParser(const std::string& str) : s(str) {}

  [[noreturn]] void fail(const std::string& msg) {
    throw Error("caps parse error at " + std::to_string(p) + " in '" + s + "': " + msg);
  }
  void ws() {
    while (p < s.size() && std::isspace(static_cast<unsigned char>(s[p]))) ++p;
  }
  bool eat(char c) {
    ws();
    if (p < s.size() && s[p] == c) {
      ++p;
      return true;
    }
    return false;
  }
  std::string name_token() {
    ws();
    size_t b = p;
    while (p < s.size()) {
      char c = s[p];
      if (std::isalnum(static_cast<unsigned char>(c)) || c == '/' || c == '-' || c == '_' || c == '.' || c == '+' ||
          c == ':')
        ++p;
      else
        break;
    }
    return s.substr(b, p - b);
  }
  std::string quoted() {
    // s[p] == '"'
    ++p;
    std::string r;
    while (p < s.size() && s[p] != '"') {
      if (s[p] == '\\' && p + 1 < s.size()) ++p;
      r += s[p++];
    }
    if (p >= s.size()) fail("unterminated string");
    ++p;
    return r;
  }
  std::string bare() {
    ws();
    size_t b = p;
    while (p < s.size()) {
      char c = s[p];
      if (c == ',' || c == ';' || c == '}' || c == ']' || c == '>' || c == ')') break;
      ++p;
    }
    return strip(s.substr(b, p - b));
  }

  Value typed_scalar(const std::string& type, const std::string& tok, bool was_quoted) {
    std::string t = lower(type);
    if (was_quoted || t == "string" || t == "str" || t == "s") return Value::String(tok);
    if (t == "int" || t == "i" || t == "uint" || t == "gint" || t == "int64" || t == "guint") {
      if (tok == "max" || tok == "MAX") return Value::Int(INT_MAX);
      if (tok == "min" || tok == "MIN") return Value::Int(INT_MIN);
      return Value::Int(to_int(tok));
    }
    if (t == "fraction") {
      if (tok == "max") return Value::Fraction(INT_MAX, 1);
      if (tok == "min") return Value::Fraction(0, 1);
      int n = 0, d = 1;
      if (!parse_fraction(tok, &n, &d)) fail("bad fraction '" + tok + "'");
      return Value::Fraction(n, d);
    }
    if (t == "double" || t == "float" || t == "d" || t == "f") return Value::Double(to_double(tok));
    if (t == "boolean" || t == "bool" || t == "b") return Value::Bool(to_bool(tok));
    if (!t.empty()) return Value::String(tok);  // unknown type name (e.g. GstVideoFormat) -> string
    // infer
    if (tok == "max") return Value::Fraction(INT_MAX, 1);
    char* end = nullptr;
    long long iv = std::strtoll(tok.c_str(), &end, 10);
    if (!tok.empty() && end && *end == '\0') return Value::Int(iv);
    auto slash = tok.find('/');
    if (slash != std::string::npos) {
      std::string a = tok.substr(0, slash), b = tok.substr(slash + 1);
      char *e1 = nullptr, *e2 = nullptr;
      long long n = std::strtoll(a.c_str(), &e1, 10);
      long long d = std::strtoll(b.c_str(), &e2, 10);
      if (!a.empty() && !b.empty() && *e1 == '\0' && *e2 == '\0') return Value::Fraction(n, d);
    }
    double dv = std::strtod(tok.c_str(), &end);
    if (!tok.empty() && end && *end == '\0') return Value::Double(dv);
    std::string lt = lower(tok);
    if (lt == "true" || lt == "false") return Value::Bool(lt == "true");
    return Value::String(tok);
  }

  Value value(const std::string& outer_type) {
    ws();
    std::string type = outer_type;
    if (p < s.size() && s[p] == '(') {
      ++p;
      size_t e = s.find(')', p);
      if (e == std::string::npos) fail("unterminated type");
      type = strip(s.substr(p, e - p));
      p = e + 1;
      ws();
    }
    if (p >= s.size()) fail("missing value");
    char c = s[p];
    if (c == '{' || c == '<') {
      char close = c == '{' ? '}' : '>';
      ++p;
      std::vector<Value> items;
      ws();
      if (p < s.size() && s[p] == close) {
        ++p;
        return Value::List(items);
      }
      while (true) {
        items.push_back(value(type));
        ws();
        if (eat(',')) continue;
        if (eat(close)) break;
        fail("bad list");
      }
      return Value::List(items);
    }
    if (c == '[') {
      ++p;
      Value a = value(type);
      if (!eat(',')) fail("bad range");
      Value b = value(type);
      if (eat(',')) value(type);  // step (ignored)
      if (!eat(']')) fail("unterminated range");
      if (a.kind == Value::Kind::INT && b.kind == Value::Kind::INT) return Value::IntRange(a.i, b.i);
      if (a.kind == Value::Kind::FRACTION || b.kind == Value::Kind::FRACTION) {
        auto tofrac = [](const Value& v, int64_t* n, int64_t* d) {
          if (v.kind == Value::Kind::FRACTION) {
            *n = v.i;
            *d = v.i2;
          } else if (v.kind == Value::Kind::INT) {
            *n = v.i;
            *d = 1;
          } else {
            *n = 0;
            *d = 1;
          }
        };
        int64_t an, ad, bn, bd;
        tofrac(a, &an, &ad);
        tofrac(b, &bn, &bd);
        return Value::FractionRange(an, ad, bn, bd);
      }
      if (a.kind == Value::Kind::DOUBLE || b.kind == Value::Kind::DOUBLE) {
        double x = a.kind == Value::Kind::DOUBLE ? a.d : static_cast<double>(a.i);
        double y = b.kind == Value::Kind::DOUBLE ? b.d : static_cast<double>(b.i);
        return Value::DoubleRange(x, y);
      }
      fail("unsupported range");
    }
    if (c == '"') {
      std::string q = quoted();
      return typed_scalar(type, q, lower(type) != "fraction" && lower(type) != "int" && lower(type) != "double" &&
                                       lower(type) != "boolean" && lower(type) != "bool");
    }
    std::string tok = bare();
    return typed_scalar(type, tok, false);
  }

  Structure structure() {
    ws();
    std::string name = name_token();
    if (name.empty()) fail("missing structure name");
    Structure st(name);
    ws();
    if (p < s.size() && s[p] == '(') {
      ++p;
      size_t e = s.find(')', p);
      if (e == std::string::npos) fail("unterminated features");
      std::vector<std::string> feats;
      for (auto& f : split(s.substr(p, e - p), ',')) {
        std::string t = strip(f);
        if (!t.empty() && t != "ANY") feats.push_back(t);
      }
      st.set_features(feats);
      p = e + 1;
    }
    while (true) {
      ws();
      if (p >= s.size() || s[p] == ';') break;
      if (!eat(',')) fail("expected ','");
      ws();
      if (p >= s.size()) break;  // trailing comma
      std::string field = name_token();
      if (field.empty()) fail("missing field name");
      if (!eat('=')) fail("expected '=' after " + field);
      Value v = value("");
      if (field == "framerate" && v.kind == Value::Kind::INT) v = Value::Fraction(v.i, 1);
      // tensor dimension / type strings that happen to look numeric ("dimensions=10")
      if ((field == "dimension" || field == "dimensions" || field == "type" || field == "types") &&
          (v.kind == Value::Kind::INT || v.kind == Value::Kind::DOUBLE))
        v = Value::String(v.kind == Value::Kind::INT ? std::to_string(v.i) : strip(v.to_string(false)));
      st.set(field, v);
    }
    return st;
  }
};

}  // namespace

Caps Caps::from_string(const std::string& str) {
  std::string t = strip(str);
  if (t == "ANY") return Caps::Any();
  if (t.empty() || t == "EMPTY" || t == "NONE") return Caps();
  Caps caps;
  CapsParser cp(t);
  while (true) {
    cp.ws();
    if (cp.p >= t.size()) break;
    caps.structs_.push_back(cp.structure());
    cp.ws();
    if (!cp.eat(';')) break;
  }
  cp.ws();
  if (cp.p != t.size()) cp.fail("trailing characters");
  return caps;
}

bool Caps::try_parse(const std::string& s, Caps* out, std::string* err) {
  try {
    *out = from_string(s);
    return true;
  } catch (const std::exception& e) {
    if (err) *err = e.what();
    return false;
  }
}

bool Caps::is_fixed() const {
  if (any_ || structs_.size() != 1) return false;
  return structs_[0].is_fixed();
}

void Caps::append(const Caps& c) {
  if (c.any_) {
    any_ = true;
    return;
  }
  for (const auto& s : c.structs_) structs_.push_back(s);
}

Caps Caps::intersect(const Caps& other) const {
  if (any_) return other;
  if (other.any_) return *this;
  Caps r;
  for (const auto& a : structs_) {
    for (const auto& b : other.structs_) {
      Structure s;
      if (Structure::intersect(a, b, &s)) r.structs_.push_back(std::move(s));
    }
  }
  return r;
}

Caps Caps::fixate() const {
  Caps r;
  if (any_ || structs_.empty()) return r;
  Structure s = structs_[0];
  s.fixate();
  r.structs_.push_back(s);
  return r;
}

std::string Caps::to_string() const {
  if (any_) return "ANY";
  if (structs_.empty()) return "EMPTY";
  std::string r;
  for (size_t i = 0; i < structs_.size(); ++i) {
    if (i) r += "; ";
    r += structs_[i].to_string(true);
  }
  return r;
}

// --------------------------------------------------------- tensor caps ----

bool structure_is_tensor_stream(const Structure& s) { return s.name() == kMimeTensor || s.name() == kMimeTensors; }

MediaType structure_media_type(const Structure& s) {
  const std::string& n = s.name();
  if (starts_with(n, "video/")) return MediaType::VIDEO;
  if (starts_with(n, "audio/")) return MediaType::AUDIO;
  if (starts_with(n, "text/")) return MediaType::TEXT;
  if (n == "application/octet-stream") return MediaType::OCTET;
  if (structure_is_tensor_stream(s)) return MediaType::TENSOR;
  return MediaType::ANY;
}

bool config_from_structure(const Structure& st_in, TensorsConfig* config) {
  *config = TensorsConfig();
  // `dimensions=10` parses as an int in untyped caps strings: read it as text
  Structure st = st_in;
  for (const char* f : {"dimension", "dimensions", "types", "type"}) {
    const Value* v = st.get(f);
    if (v && v->kind == Value::Kind::INT) st.set(f, Value::String(std::to_string(v->i)));
  }
  const std::string& name = st.name();
  if (name == kMimeTensor) {
    config->info.resize(1);
    std::string v;
    if (st.get_string("dimension", &v)) parse_dimension(v, config->info.at(0).dim);
    if (st.get_string("type", &v)) config->info.at(0).type = dtype_from_string(v);
  } else if (name == kMimeTensors) {
    std::string v;
    if (st.get_string("format", &v)) {
      Format f = format_from_string(v);
      if (f != Format::END) config->info.format = f;
    }
    if (config->info.format == Format::STATIC) {
      int64_t n = 0;
      if (st.get_int("num_tensors", &n)) {
        if (n > kSizeLimit + kSizeExtraLimit) n = kSizeLimit + kSizeExtraLimit;
        config->info.resize(static_cast<unsigned>(n));
      }
      if (st.get_string("dimensions", &v)) {
        unsigned nd = config->info.parse_dimensions(v);
        if (config->info.num_tensors == 0) config->info.num_tensors = nd;
      }
      if (st.get_string("types", &v)) config->info.parse_types(v);
      if (st.get_string("names", &v)) config->info.parse_names(v);
    }
  } else {
    return false;
  }
  int n, d;
  if (st.get_fraction("framerate", &n, &d)) {
    config->rate_n = n;
    config->rate_d = d;
  }
  return true;
}

static std::string dims_for_caps(const TensorsInfo& info) {
  std::string out;
  for (unsigned i = 0; i < info.num_tensors; ++i) {
    if (i) out += ',';
    const auto& t = info.at(i);
    unsigned r = static_cast<unsigned>(std::max(t.rank(), kRankLimitPrev));
    out += dimension_valid(t.dim) ? rank_dimension_string(t.dim, r) : dimension_string(t.dim);
  }
  return out;
}

Caps caps_from_config(const TensorsConfig& config, bool device) {
  Structure st(kMimeTensors);
  if (device) st.set_features({kFeatureHIP});
  st.set("format", Value::String(format_name(config.info.format) ? format_name(config.info.format) : "static"));
  if (config.info.format == Format::STATIC && config.info.num_tensors > 0) {
    st.set("num_tensors", Value::Int(config.info.num_tensors));
    st.set("dimensions", Value::String(dims_for_caps(config.info)));
    st.set("types", Value::String(config.info.types_string()));
  }
  if (config.rate_n >= 0 && config.rate_d > 0)
    st.set("framerate", Value::Fraction(config.rate_n, config.rate_d));
  else
    st.set("framerate", Value::FractionRange(0, 1, INT_MAX, 1));
  Caps c;
  c.append(st);
  return c;
}

Caps pad_caps_from_config(const TensorsConfig& config, const Caps* peer, bool device) {
  bool peer_flexible = false;
  bool peer_only_legacy = false;
  if (peer && !peer->is_any() && peer->size() > 0) {
    TensorsConfig pc;
    if (config_from_structure(peer->at(0), &pc)) peer_flexible = pc.is_flexible() && peer->at(0).has("format") &&
                                                                 peer->at(0).get("format")->is_fixed();
    Caps tensors = Caps::from_string("other/tensors");
    Caps legacy = Caps::from_string("other/tensor");
    peer_only_legacy = !peer->can_intersect(tensors) && peer->can_intersect(legacy);
  }
  if (config.is_flexible() || peer_flexible) {
    TensorsConfig c = config;
    c.info.format = Format::FLEXIBLE;
    return caps_from_config(c, device);
  }
  if (peer_only_legacy && config.info.num_tensors == 1) {
    Structure st(kMimeTensor);
    if (device) st.set_features({kFeatureHIP});
    st.set("dimension", Value::String(dims_for_caps(config.info)));
    st.set("type", Value::String(dtype_name(config.info.at(0).type) ? dtype_name(config.info.at(0).type) : ""));
    if (config.rate_n >= 0 && config.rate_d > 0) st.set("framerate", Value::Fraction(config.rate_n, config.rate_d));
    Caps c;
    c.append(st);
    return c;
  }
  return caps_from_config(config, device);
}

std::string tensor_caps_template_static() {
  return "other/tensors, format=(string)static, num_tensors=(int)[ 1, 16 ], framerate=(fraction)[ 0/1, 2147483647/1 ]; "
         "other/tensor, framerate=(fraction)[ 0/1, 2147483647/1 ]";
}

std::string tensor_caps_template_flexible() {
  return "other/tensors, format=(string)flexible, framerate=(fraction)[ 0/1, 2147483647/1 ]";
}

std::string tensor_caps_template_all() {
  return "other/tensors, format=(string){ static, flexible, sparse }, framerate=(fraction)[ 0/1, 2147483647/1 ]; "
         "other/tensor, framerate=(fraction)[ 0/1, 2147483647/1 ]";
}

}  // namespace nnsx
