// Lua 5.1 subset interpreter (see lua_vm.h): lexer -> recursive-descent parser
// -> resolved AST (locals as frame slots, upvalues as (depth, slot) through the
// lexical frame chain) -> tree-walking evaluator.
#include "filter/lua_vm.h"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <random>
#include <sstream>

namespace nnsx {
namespace lua {

// ================================================================ values ====
Value Value::string(std::string s) {
  auto o = std::make_shared<StrObj>();
  o->hash = std::hash<std::string>()(s);
  o->s = std::move(s);
  Value r;
  r.t = STR;
  r.o = std::move(o);
  return r;
}
Value Value::table(std::shared_ptr<Table> t) {
  Value r;
  r.t = TABLE;
  r.o = std::move(t);
  return r;
}
Value Value::native(std::string name, std::function<std::vector<Value>(std::vector<Value>&)> fn) {
  auto o = std::make_shared<Native>();
  o->name = std::move(name);
  o->fn = std::move(fn);
  Value r;
  r.t = NATIVE;
  r.o = std::move(o);
  return r;
}
Value Value::userdata(std::shared_ptr<Userdata> u) {
  Value r;
  r.t = USERDATA;
  r.o = std::move(u);
  return r;
}
const std::string& Value::str() const { return static_cast<StrObj*>(o.get())->s; }
Table* Value::tab() const { return static_cast<Table*>(o.get()); }
Userdata* Value::ud() const { return static_cast<Userdata*>(o.get()); }
std::string Value::type_name() const {
  switch (t) {
    case NIL: return "nil";
    case BOOL: return "boolean";
    case NUM: return "number";
    case STR: return "string";
    case TABLE: return "table";
    case FUNC:
    case NATIVE: return "function";
    case USERDATA: return "userdata";
  }
  return "?";
}

size_t ValueHash::operator()(const Value& v) const {
  switch (v.t) {
    case Value::NUM: return std::hash<double>()(v.n);
    case Value::BOOL: return v.b ? 1 : 2;
    case Value::STR: return static_cast<StrObj*>(v.o.get())->hash;
    default: return std::hash<const void*>()(v.o.get());
  }
}
bool ValueEq::operator()(const Value& a, const Value& b) const {
  if (a.t != b.t) return false;
  switch (a.t) {
    case Value::NIL: return true;
    case Value::BOOL: return a.b == b.b;
    case Value::NUM: return a.n == b.n;
    case Value::STR: return a.o == b.o || a.str() == b.str();
    default: return a.o == b.o;
  }
}

static bool array_index(const Value& k, size_t* i) {
  if (k.t != Value::NUM) return false;
  const double d = k.n;
  if (d < 1 || d != std::floor(d) || d > 4e9) return false;
  *i = static_cast<size_t>(d);
  return true;
}

Value Table::get(const Value& k) const {
  size_t i;
  if (array_index(k, &i) && i <= arr.size()) return arr[i - 1];
  if (k.t == Value::NIL) return Value();
  auto it = hash.find(k);
  return it == hash.end() ? Value() : it->second;
}

void Table::set(const Value& k, Value v) {
  if (k.t == Value::NIL) throw LuaError("table index is nil");
  if (k.t == Value::NUM && std::isnan(k.n)) throw LuaError("table index is NaN");
  size_t i;
  if (array_index(k, &i)) {
    if (i <= arr.size()) {
      arr[i - 1] = std::move(v);
      if (i == arr.size())
        while (!arr.empty() && arr.back().t == Value::NIL) arr.pop_back();
      return;
    }
    if (i == arr.size() + 1 && v.t != Value::NIL) {
      arr.push_back(std::move(v));
      // migrate following keys from the hash part
      for (;;) {
        auto it = hash.find(Value::number(static_cast<double>(arr.size() + 1)));
        if (it == hash.end()) break;
        arr.push_back(std::move(it->second));
        hash.erase(it);
      }
      return;
    }
  }
  if (v.t == Value::NIL)
    hash.erase(k);
  else
    hash[k] = std::move(v);
}

size_t Table::length() const { return arr.size(); }

std::string fmt_number(double d) {
  if (d == std::floor(d) && std::fabs(d) < 1e15) {
    char b[32];
    std::snprintf(b, sizeof(b), "%.0f", d);
    return b;
  }
  char b[48];
  std::snprintf(b, sizeof(b), "%.14g", d);
  return b;
}

std::string tostring(const Value& v) {
  char b[64];
  switch (v.t) {
    case Value::NIL: return "nil";
    case Value::BOOL: return v.b ? "true" : "false";
    case Value::NUM: return fmt_number(v.n);
    case Value::STR: return v.str();
    default:
      std::snprintf(b, sizeof(b), "%s: %p", v.type_name().c_str(), v.o.get());
      return b;
  }
}

bool tonumber(const Value& v, double* out) {
  if (v.t == Value::NUM) {
    *out = v.n;
    return true;
  }
  if (v.t != Value::STR) return false;
  const std::string& s = v.str();
  const char* p = s.c_str();
  while (std::isspace(static_cast<unsigned char>(*p))) ++p;
  if (!*p) return false;
  char* end = nullptr;
  double d;
  if (p[0] == '0' && (p[1] == 'x' || p[1] == 'X'))
    d = static_cast<double>(std::strtoull(p, &end, 16));
  else
    d = std::strtod(p, &end);
  if (end == p) return false;
  while (std::isspace(static_cast<unsigned char>(*end))) ++end;
  if (*end) return false;
  *out = d;
  return true;
}

// ================================================================= lexer ====
namespace {

enum Tok {
  T_EOF, T_NAME, T_NUM, T_STR,
  // keywords
  K_AND, K_BREAK, K_DO, K_ELSE, K_ELSEIF, K_END, K_FALSE, K_FOR, K_FUNCTION, K_GOTO, K_IF, K_IN, K_LOCAL,
  K_NIL, K_NOT, K_OR, K_REPEAT, K_RETURN, K_THEN, K_TRUE, K_UNTIL, K_WHILE,
  // symbols
  S_PLUS, S_MINUS, S_STAR, S_SLASH, S_DSLASH, S_PCT, S_CARET, S_HASH, S_EQ, S_NE, S_LE, S_GE, S_LT, S_GT,
  S_ASSIGN, S_LPAREN, S_RPAREN, S_LBRACE, S_RBRACE, S_LBRACK, S_RBRACK, S_SEMI, S_COLON, S_COMMA, S_DOT,
  S_CONCAT, S_DOTS, S_DCOLON
};

struct Token {
  Tok t = T_EOF;
  std::string s;
  double n = 0;
  int line = 1;
};

const std::unordered_map<std::string, Tok>& keywords() {
  static const std::unordered_map<std::string, Tok> k = {
      {"and", K_AND},       {"break", K_BREAK}, {"do", K_DO},         {"else", K_ELSE},     {"elseif", K_ELSEIF},
      {"end", K_END},       {"false", K_FALSE}, {"for", K_FOR},       {"function", K_FUNCTION},
      {"goto", K_GOTO},     {"if", K_IF},       {"in", K_IN},         {"local", K_LOCAL},   {"nil", K_NIL},
      {"not", K_NOT},       {"or", K_OR},       {"repeat", K_REPEAT}, {"return", K_RETURN}, {"then", K_THEN},
      {"true", K_TRUE},     {"until", K_UNTIL}, {"while", K_WHILE}};
  return k;
}

class Lexer {
 public:
  Lexer(const std::string& src, const std::string& chunk) : s_(src), chunk_(chunk) {}

  Token next() {
    skip_space();
    Token tk;
    tk.line = line_;
    if (i_ >= s_.size()) return tk;
    const char c = s_[i_];
    if (std::isalpha(static_cast<unsigned char>(c)) || c == '_') {
      size_t j = i_;
      while (j < s_.size() && (std::isalnum(static_cast<unsigned char>(s_[j])) || s_[j] == '_')) ++j;
      tk.s = s_.substr(i_, j - i_);
      i_ = j;
      auto it = keywords().find(tk.s);
      tk.t = it == keywords().end() ? T_NAME : it->second;
      return tk;
    }
    if (std::isdigit(static_cast<unsigned char>(c)) ||
        (c == '.' && i_ + 1 < s_.size() && std::isdigit(static_cast<unsigned char>(s_[i_ + 1])))) {
      tk.t = T_NUM;
      tk.n = number();
      return tk;
    }
    if (c == '"' || c == '\'') {
      tk.t = T_STR;
      tk.s = quoted(c);
      return tk;
    }
    if (c == '[') {
      size_t lvl;
      if (long_open(&lvl)) {
        tk.t = T_STR;
        tk.s = long_body(lvl);
        return tk;
      }
    }
    ++i_;
    auto two = [&](char nx) {
      if (i_ < s_.size() && s_[i_] == nx) {
        ++i_;
        return true;
      }
      return false;
    };
    switch (c) {
      case '+': tk.t = S_PLUS; break;
      case '-': tk.t = S_MINUS; break;
      case '*': tk.t = S_STAR; break;
      case '/': tk.t = two('/') ? S_DSLASH : S_SLASH; break;
      case '%': tk.t = S_PCT; break;
      case '^': tk.t = S_CARET; break;
      case '#': tk.t = S_HASH; break;
      case '=': tk.t = two('=') ? S_EQ : S_ASSIGN; break;
      case '~':
        if (!two('=')) error("unexpected symbol near '~'");
        tk.t = S_NE;
        break;
      case '<': tk.t = two('=') ? S_LE : S_LT; break;
      case '>': tk.t = two('=') ? S_GE : S_GT; break;
      case '(': tk.t = S_LPAREN; break;
      case ')': tk.t = S_RPAREN; break;
      case '{': tk.t = S_LBRACE; break;
      case '}': tk.t = S_RBRACE; break;
      case '[': tk.t = S_LBRACK; break;
      case ']': tk.t = S_RBRACK; break;
      case ';': tk.t = S_SEMI; break;
      case ':': tk.t = two(':') ? S_DCOLON : S_COLON; break;
      case ',': tk.t = S_COMMA; break;
      case '.':
        if (two('.'))
          tk.t = two('.') ? S_DOTS : S_CONCAT;
        else
          tk.t = S_DOT;
        break;
      default: error(std::string("unexpected symbol near '") + c + "'");
    }
    return tk;
  }

  [[noreturn]] void error(const std::string& m) const {
    throw LuaError(chunk_ + ":" + std::to_string(line_) + ": " + m);
  }

 private:
  void skip_space() {
    for (;;) {
      while (i_ < s_.size() && std::isspace(static_cast<unsigned char>(s_[i_]))) {
        if (s_[i_] == '\n') ++line_;
        ++i_;
      }
      if (i_ + 1 < s_.size() && s_[i_] == '-' && s_[i_ + 1] == '-') {
        i_ += 2;
        size_t lvl;
        if (i_ < s_.size() && s_[i_] == '[' && long_open(&lvl)) {
          long_body(lvl);
          continue;
        }
        while (i_ < s_.size() && s_[i_] != '\n') ++i_;
        continue;
      }
      if (i_ == 0 && s_.size() > 1 && s_[0] == '#' && s_[1] == '!') {  // shebang line
        while (i_ < s_.size() && s_[i_] != '\n') ++i_;
        continue;
      }
      return;
    }
  }

  // at '[': '[' '='* '[' -> level; the position moves past it
  bool long_open(size_t* lvl) {
    size_t j = i_ + 1, l = 0;
    while (j < s_.size() && s_[j] == '=') ++j, ++l;
    if (j < s_.size() && s_[j] == '[') {
      i_ = j + 1;
      *lvl = l;
      return true;
    }
    return false;
  }

  std::string long_body(size_t lvl) {
    if (i_ < s_.size() && s_[i_] == '\r') ++i_;
    if (i_ < s_.size() && s_[i_] == '\n') ++line_, ++i_;  // a first newline is skipped
    std::string close = "]" + std::string(lvl, '=') + "]";
    const size_t e = s_.find(close, i_);
    if (e == std::string::npos) error("unfinished long string/comment");
    std::string body = s_.substr(i_, e - i_);
    line_ += static_cast<int>(std::count(body.begin(), body.end(), '\n'));
    i_ = e + close.size();
    return body;
  }

  double number() {
    const char* p = s_.c_str() + i_;
    char* end = nullptr;
    double d;
    if (p[0] == '0' && (p[1] == 'x' || p[1] == 'X'))
      d = static_cast<double>(std::strtoull(p, &end, 16));
    else
      d = std::strtod(p, &end);
    if (end == p) error("malformed number");
    i_ += static_cast<size_t>(end - p);
    if (i_ < s_.size() && (std::isalnum(static_cast<unsigned char>(s_[i_])) || s_[i_] == '_'))
      error("malformed number");
    return d;
  }

  std::string quoted(char q) {
    ++i_;
    std::string out;
    for (;;) {
      if (i_ >= s_.size() || s_[i_] == '\n') error("unfinished string");
      char c = s_[i_++];
      if (c == q) break;
      if (c != '\\') {
        out += c;
        continue;
      }
      if (i_ >= s_.size()) error("unfinished string");
      c = s_[i_++];
      switch (c) {
        case 'n': out += '\n'; break;
        case 't': out += '\t'; break;
        case 'r': out += '\r'; break;
        case 'a': out += '\a'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'v': out += '\v'; break;
        case '\\': out += '\\'; break;
        case '"': out += '"'; break;
        case '\'': out += '\''; break;
        case '\n': out += '\n'; ++line_; break;
        default:
          if (std::isdigit(static_cast<unsigned char>(c))) {
            int v = c - '0', k = 1;
            while (k < 3 && i_ < s_.size() && std::isdigit(static_cast<unsigned char>(s_[i_]))) v = v * 10 + (s_[i_++] - '0'), ++k;
            if (v > 255) error("escape sequence too large");
            out += static_cast<char>(v);
          } else {
            error(std::string("invalid escape sequence '\\") + c + "'");
          }
      }
    }
    return out;
  }

  const std::string& s_;
  std::string chunk_;
  size_t i_ = 0;
  int line_ = 1;
};

}  // namespace

// =================================================================== AST ====
struct Frame;
struct Exec;

struct Expr {
  int line = 0;
  virtual ~Expr() = default;
  virtual Value eval(Exec& x, Frame& f) const = 0;
  // calls and '...' yield several values
  virtual bool multi() const { return false; }
  virtual void eval_multi(Exec& x, Frame& f, std::vector<Value>* out) const { out->push_back(eval(x, f)); }
  // variables: where the value lives (no copy, no refcount traffic); else nullptr
  virtual Value* ref(Exec&, Frame&) const { return nullptr; }
};
using ExprP = std::unique_ptr<Expr>;

struct Stmt {
  int line = 0;
  virtual ~Stmt() = default;
  enum Flow { NORMAL, BREAK, RETURN };
  virtual Flow exec(Exec& x, Frame& f) const = 0;
};
using StmtP = std::unique_ptr<Stmt>;
using Block = std::vector<StmtP>;

// a local variable; `captured` (set while parsing the rest of its scope) puts
// its value in a heap cell that closures share, made fresh each time the
// declaration runs -- so a closure created in a loop body keeps that
// iteration's value, as in Lua 5.1
struct VarInfo {
  int slot = 0;
  bool captured = false;
};

struct UpDesc {
  bool from_local;         // the enclosing function's local ...
  const VarInfo* var;      // ... this one
  int index;               // else the enclosing function's upvalue #index
};

struct FuncProto {
  int nparams = 0;
  bool vararg = false;
  bool has_self = false;
  int nslots = 0;
  Block body;
  std::string name;
  int line = 0;
  std::vector<std::unique_ptr<VarInfo>> vars;
  std::vector<const VarInfo*> params;
  std::vector<UpDesc> upvals;
};

struct Chunk {
  std::vector<std::unique_ptr<FuncProto>> protos;
  FuncProto* main = nullptr;
};

using Cell = std::shared_ptr<Value>;

struct Closure : Obj {
  const FuncProto* proto = nullptr;
  std::vector<Cell> upvals;
};

struct Frame {
  std::vector<Value> slots;
  std::vector<Cell> cells;  // captured locals (VarInfo::captured)
  std::vector<Value> varargs;
  std::vector<Value> ret;
  const Closure* cl = nullptr;
};

struct Exec {
  VM& vm;  // (its depth_ counts nested Lua calls across every Exec: pcall, gsub, sort callbacks)
  std::string chunk;
  [[noreturn]] void error(int line, const std::string& m) const {
    throw LuaError(chunk + ":" + std::to_string(line) + ": " + m);
  }
  void step(int line) {
    if (vm.step_limit_ && ++vm.steps_ > vm.step_limit_) error(line, "script exceeded its step limit");
  }
  std::vector<Value> call(const Value& fn, std::vector<Value>& args, int line);
};

static inline Value& local_ref(Frame& f, const VarInfo* v) {
  if (!v->captured) return f.slots[v->slot];
  Cell& c = f.cells[v->slot];
  if (!c) c = std::make_shared<Value>();
  return *c;
}
// a declaration ran: captured locals get a fresh cell
static inline void bind_local(Frame& f, const VarInfo* v, Value val) {
  if (v->captured)
    f.cells[v->slot] = std::make_shared<Value>(std::move(val));
  else
    f.slots[v->slot] = std::move(val);
}

// ---------------------------------------------------------------- exprs ----
struct ConstE : Expr {
  Value v;
  Value eval(Exec&, Frame&) const override { return v; }
};
struct LocalE : Expr {
  const VarInfo* var = nullptr;
  Value eval(Exec&, Frame& f) const override { return local_ref(f, var); }
  Value* ref(Exec&, Frame& f) const override { return &local_ref(f, var); }
};
struct UpvalE : Expr {
  int index = 0;
  Value eval(Exec&, Frame& f) const override { return *f.cl->upvals[static_cast<size_t>(index)]; }
  Value* ref(Exec&, Frame& f) const override { return f.cl->upvals[static_cast<size_t>(index)].get(); }
};
// the AST belongs to one VM and VM::globals_ never erases, so the map node
// (stable across rehashing) is looked up once
struct GlobalE : Expr {
  std::string name;
  mutable Value* slot = nullptr;
  Value* ref(Exec& x, Frame&) const override {
    if (!slot) slot = &x.vm.globals_[name];
    return slot;
  }
  Value eval(Exec& x, Frame& f) const override { return *ref(x, f); }
};
struct VarargE : Expr {
  Value eval(Exec&, Frame& f) const override { return f.varargs.empty() ? Value() : f.varargs[0]; }
  bool multi() const override { return true; }
  void eval_multi(Exec&, Frame& f, std::vector<Value>* out) const override {
    out->insert(out->end(), f.varargs.begin(), f.varargs.end());
  }
};

// ---- metatables
enum MetaEvent { M_INDEX, M_NEWINDEX, M_CALL, M_ADD, M_SUB, M_MUL, M_DIV, M_MOD, M_POW, M_IDIV, M_UNM, M_CONCAT,
                 M_EQ, M_LT, M_LE, M_TOSTRING, M_METATABLE, M_COUNT };
static const Value& meta_name(MetaEvent e) {
  static const Value names[M_COUNT] = {
      Value::string("__index"), Value::string("__newindex"), Value::string("__call"), Value::string("__add"),
      Value::string("__sub"),   Value::string("__mul"),      Value::string("__div"),  Value::string("__mod"),
      Value::string("__pow"),   Value::string("__idiv"),     Value::string("__unm"),  Value::string("__concat"),
      Value::string("__eq"),    Value::string("__lt"),       Value::string("__le"),   Value::string("__tostring"),
      Value::string("__metatable")};
  return names[e];
}
static Value metamethod(const Value& v, MetaEvent e) {
  if (v.t != Value::TABLE || !v.tab()->meta) return Value();
  return v.tab()->meta->get(meta_name(e));
}
static Value call1(Exec& x, const Value& fn, std::vector<Value> args, int line) {
  std::vector<Value> r = x.call(fn, args, line);
  return r.empty() ? Value() : r[0];
}

static Value index_value(Exec& x, const Value& o, const Value& k, int line, int depth = 0) {
  if (o.t == Value::TABLE) {
    Value r = o.tab()->get(k);
    if (r.t != Value::NIL || !o.tab()->meta) return r;
    const Value h = o.tab()->meta->get(meta_name(M_INDEX));
    if (h.t == Value::NIL) return r;
    if (h.t == Value::FUNC || h.t == Value::NATIVE) return call1(x, h, {o, k}, line);
    if (depth > 100) x.error(line, "'__index' chain too long; possible loop");
    return index_value(x, h, k, line, depth + 1);
  }
  if (o.t == Value::USERDATA) return o.ud()->index(k);
  if (o.t == Value::STR) {  // ("abc"):upper() etc. go through the string library
    auto it = x.vm.globals_.find("string");
    if (it != x.vm.globals_.end() && it->second.t == Value::TABLE) return it->second.tab()->get(k);
  }
  x.error(line, "attempt to index a " + o.type_name() + " value");
}

static void newindex_value(Exec& x, const Value& o, const Value& k, Value v, int line, int depth = 0) {
  if (o.t == Value::TABLE) {
    if (o.tab()->meta && o.tab()->get(k).t == Value::NIL) {
      const Value h = o.tab()->meta->get(meta_name(M_NEWINDEX));
      if (h.t == Value::FUNC || h.t == Value::NATIVE) {
        std::vector<Value> args{o, k, std::move(v)};
        x.call(h, args, line);
        return;
      }
      if (h.t != Value::NIL) {
        if (depth > 100) x.error(line, "'__newindex' chain too long; possible loop");
        newindex_value(x, h, k, std::move(v), line, depth + 1);
        return;
      }
    }
    try {
      o.tab()->set(k, std::move(v));
    } catch (const LuaError& e) {
      x.error(line, e.what());
    }
    return;
  }
  if (o.t == Value::USERDATA) {
    o.ud()->newindex(k, v);
    return;
  }
  x.error(line, "attempt to index a " + o.type_name() + " value");
}

struct IndexE : Expr {
  ExprP obj, key;
  Value eval(Exec& x, Frame& f) const override {
    if (const Value* o = obj->ref(x, f)) {
      const Value k = key->eval(x, f);  // (may not reassign the variable: keys are evaluated after)
      return index_value(x, *o, k, line);
    }
    Value o = obj->eval(x, f);
    return index_value(x, o, key->eval(x, f), line);
  }
};

struct CallE : Expr {
  ExprP fn;
  std::string method;  // obj:method(args)
  std::vector<ExprP> args;
  bool multi() const override { return true; }
  std::vector<Value> run(Exec& x, Frame& f) const {
    std::vector<Value> a;
    a.reserve(args.size() + 1);
    Value callee;
    if (!method.empty()) {
      Value self = fn->eval(x, f);
      callee = index_value(x, self, Value::string(method), line);
      a.push_back(std::move(self));
    } else {
      callee = fn->eval(x, f);
    }
    for (size_t i = 0; i < args.size(); ++i) {
      if (i + 1 == args.size() && args[i]->multi())
        args[i]->eval_multi(x, f, &a);
      else
        a.push_back(args[i]->eval(x, f));
    }
    return x.call(callee, a, line);
  }
  Value eval(Exec& x, Frame& f) const override {
    auto r = run(x, f);
    return r.empty() ? Value() : r[0];
  }
  void eval_multi(Exec& x, Frame& f, std::vector<Value>* out) const override {
    auto r = run(x, f);
    out->insert(out->end(), std::make_move_iterator(r.begin()), std::make_move_iterator(r.end()));
  }
};

struct FunctionE : Expr {
  const FuncProto* proto = nullptr;
  Value eval(Exec&, Frame& f) const override;
};

Value FunctionE::eval(Exec&, Frame& f) const {
  auto c = std::make_shared<Closure>();
  c->proto = proto;
  c->upvals.reserve(proto->upvals.size());
  for (const UpDesc& u : proto->upvals) {
    if (u.from_local) {
      Cell& cell = f.cells[u.var->slot];
      if (!cell) cell = std::make_shared<Value>();
      c->upvals.push_back(cell);
    } else {
      c->upvals.push_back(f.cl->upvals[static_cast<size_t>(u.index)]);
    }
  }
  Value r;
  r.t = Value::FUNC;
  r.o = std::move(c);
  return r;
}

static double arith_num(Exec& x, const Value& v, int line, const char* what) {
  double d;
  if (tonumber(v, &d)) return d;
  x.error(line, std::string("attempt to perform arithmetic on a ") + v.type_name() + " value" + what);
}

// a binary metamethod from either operand (Lua 5.1 order: first, then second)
static bool try_bin_meta(Exec& x, MetaEvent e, const Value& a, const Value& b, int line, Value* out) {
  Value h = metamethod(a, e);
  if (h.t == Value::NIL) h = metamethod(b, e);
  if (h.t == Value::NIL) return false;
  *out = call1(x, h, {a, b}, line);
  return true;
}

static bool lua_lt(Exec& x, const Value& a, const Value& b, int line) {
  if (a.t == Value::NUM && b.t == Value::NUM) return a.n < b.n;
  if (a.t == Value::STR && b.t == Value::STR) return a.str() < b.str();
  Value r;
  if (a.t == b.t && try_bin_meta(x, M_LT, a, b, line, &r)) return r.truthy();
  x.error(line, "attempt to compare " + a.type_name() + " with " + b.type_name());
}
static bool lua_le(Exec& x, const Value& a, const Value& b, int line) {
  if (a.t == Value::NUM && b.t == Value::NUM) return a.n <= b.n;
  if (a.t == Value::STR && b.t == Value::STR) return a.str() <= b.str();
  Value r;
  if (a.t == b.t) {
    if (try_bin_meta(x, M_LE, a, b, line, &r)) return r.truthy();
    if (try_bin_meta(x, M_LT, b, a, line, &r)) return !r.truthy();  // a <= b as not (b < a)
  }
  x.error(line, "attempt to compare " + a.type_name() + " with " + b.type_name());
}
static bool lua_eq(Exec& x, const Value& a, const Value& b, int line) {
  if (ValueEq()(a, b)) return true;
  if (a.t != Value::TABLE || b.t != Value::TABLE) return false;
  const Value ha = metamethod(a, M_EQ), hb = metamethod(b, M_EQ);
  if (ha.t == Value::NIL || !ValueEq()(ha, hb)) return false;  // 5.1: the same __eq on both
  return call1(x, ha, {a, b}, line).truthy();
}

enum BinOp { B_ADD, B_SUB, B_MUL, B_DIV, B_IDIV, B_MOD, B_POW, B_CONCAT, B_EQ, B_NE, B_LT, B_LE, B_GT, B_GE };

struct BinE : Expr {
  BinOp op;
  ExprP a, b;
  Value eval(Exec& x, Frame& f) const override {
    Value va = a->eval(x, f), vb = b->eval(x, f);
    if (va.t == Value::NUM && vb.t == Value::NUM) {  // fast path
      const double p = va.n, q = vb.n;
      switch (op) {
        case B_ADD: return Value::number(p + q);
        case B_SUB: return Value::number(p - q);
        case B_MUL: return Value::number(p * q);
        case B_DIV: return Value::number(p / q);
        case B_IDIV: return Value::number(std::floor(p / q));
        case B_MOD: return Value::number(p - std::floor(p / q) * q);
        case B_POW: return Value::number(std::pow(p, q));
        case B_EQ: return Value::boolean(p == q);
        case B_NE: return Value::boolean(p != q);
        case B_LT: return Value::boolean(p < q);
        case B_LE: return Value::boolean(p <= q);
        case B_GT: return Value::boolean(p > q);
        case B_GE: return Value::boolean(p >= q);
        case B_CONCAT: break;
      }
    }
    switch (op) {
      case B_EQ: return Value::boolean(lua_eq(x, va, vb, line));
      case B_NE: return Value::boolean(!lua_eq(x, va, vb, line));
      case B_LT: return Value::boolean(lua_lt(x, va, vb, line));
      case B_LE: return Value::boolean(lua_le(x, va, vb, line));
      case B_GT: return Value::boolean(lua_lt(x, vb, va, line));
      case B_GE: return Value::boolean(lua_le(x, vb, va, line));
      case B_CONCAT: {
        auto plain = [](const Value& v) { return v.t == Value::STR || v.t == Value::NUM; };
        if (!plain(va) || !plain(vb)) {
          Value r;
          if (try_bin_meta(x, M_CONCAT, va, vb, line, &r)) return r;
          x.error(line, "attempt to concatenate a " + (plain(va) ? vb : va).type_name() + " value");
        }
        return Value::string((va.t == Value::STR ? va.str() : fmt_number(va.n)) +
                             (vb.t == Value::STR ? vb.str() : fmt_number(vb.n)));
      }
      default: break;
    }
    double p, q;
    if (!tonumber(va, &p) || !tonumber(vb, &q)) {
      static const MetaEvent ev[] = {M_ADD, M_SUB, M_MUL, M_DIV, M_IDIV, M_MOD, M_POW};
      Value r;
      if (op <= B_POW && try_bin_meta(x, ev[op], va, vb, line, &r)) return r;
      p = arith_num(x, va, line, "");
      q = arith_num(x, vb, line, "");
    }
    switch (op) {
      case B_ADD: return Value::number(p + q);
      case B_SUB: return Value::number(p - q);
      case B_MUL: return Value::number(p * q);
      case B_DIV: return Value::number(p / q);
      case B_IDIV: return Value::number(std::floor(p / q));
      case B_MOD: return Value::number(p - std::floor(p / q) * q);
      case B_POW: return Value::number(std::pow(p, q));
      default: return Value();
    }
  }
};

struct AndE : Expr {
  ExprP a, b;
  Value eval(Exec& x, Frame& f) const override {
    Value v = a->eval(x, f);
    return v.truthy() ? b->eval(x, f) : v;
  }
};
struct OrE : Expr {
  ExprP a, b;
  Value eval(Exec& x, Frame& f) const override {
    Value v = a->eval(x, f);
    return v.truthy() ? v : b->eval(x, f);
  }
};

enum UnOp { U_NEG, U_NOT, U_LEN };
struct UnE : Expr {
  UnOp op;
  ExprP a;
  Value eval(Exec& x, Frame& f) const override {
    Value v = a->eval(x, f);
    switch (op) {
      case U_NEG: {
        double d;
        if (tonumber(v, &d)) return Value::number(-d);
        const Value h = metamethod(v, M_UNM);
        if (h.t != Value::NIL) return call1(x, h, {v, v}, line);
        return Value::number(-arith_num(x, v, line, ""));
      }
      case U_NOT: return Value::boolean(!v.truthy());
      case U_LEN:
        if (v.t == Value::STR) return Value::number(static_cast<double>(v.str().size()));
        if (v.t == Value::TABLE) return Value::number(static_cast<double>(v.tab()->length()));
        if (v.t == Value::USERDATA) return Value::number(static_cast<double>(v.ud()->length()));
        x.error(line, "attempt to get length of a " + v.type_name() + " value");
    }
    return Value();
  }
};

struct TableE : Expr {
  std::vector<ExprP> items;                         // positional
  std::vector<std::pair<ExprP, ExprP>> keyed;       // [k] = v / name = v
  std::vector<int> order;                           // >= 0: items[i]; < 0: keyed[-i-1]
  Value eval(Exec& x, Frame& f) const override {
    auto t = std::make_shared<Table>();
    double n = 1;
    for (size_t k = 0; k < order.size(); ++k) {
      const int o = order[k];
      if (o >= 0) {
        const Expr& e = *items[static_cast<size_t>(o)];
        if (k + 1 == order.size() && e.multi()) {
          std::vector<Value> vs;
          e.eval_multi(x, f, &vs);
          for (auto& v : vs) t->set(Value::number(n++), std::move(v));
        } else {
          t->set(Value::number(n++), e.eval(x, f));
        }
      } else {
        const auto& kv = keyed[static_cast<size_t>(-o - 1)];
        Value key = kv.first->eval(x, f);
        if (key.t == Value::NIL) x.error(line, "table index is nil");
        t->set(key, kv.second->eval(x, f));
      }
    }
    return Value::table(std::move(t));
  }
};

// ---------------------------------------------------------------- stmts ----
static Stmt::Flow exec_block(Exec& x, Frame& f, const Block& b) {
  for (const auto& s : b) {
    x.step(s->line);
    const Stmt::Flow r = s->exec(x, f);
    if (r != Stmt::NORMAL) return r;
  }
  return Stmt::NORMAL;
}

static void eval_list(Exec& x, Frame& f, const std::vector<ExprP>& es, size_t want, std::vector<Value>* out) {
  for (size_t i = 0; i < es.size(); ++i) {
    if (i + 1 == es.size() && es[i]->multi())
      es[i]->eval_multi(x, f, out);
    else
      out->push_back(es[i]->eval(x, f));
  }
  if (want) out->resize(std::max(want, out->size()));
}

struct LocalS : Stmt {
  std::vector<const VarInfo*> vars;
  std::vector<ExprP> exprs;
  bool function_decl = false;  // local function f: f is in scope (and may be captured) in its body
  Flow exec(Exec& x, Frame& f) const override {
    if (function_decl) {
      bind_local(f, vars[0], Value());
      Value fn = exprs[0]->eval(x, f);
      local_ref(f, vars[0]) = std::move(fn);
      return NORMAL;
    }
    if (vars.size() == 1 && exprs.size() == 1 && !exprs[0]->multi()) {
      bind_local(f, vars[0], exprs[0]->eval(x, f));
      return NORMAL;
    }
    std::vector<Value> vs;
    eval_list(x, f, exprs, vars.size(), &vs);
    for (size_t i = 0; i < vars.size(); ++i) bind_local(f, vars[i], vs[i]);
    return NORMAL;
  }
};

struct AssignS : Stmt {
  std::vector<ExprP> targets;  // LocalE / GlobalE / IndexE
  std::vector<ExprP> exprs;
  static void store(Exec& x, Frame& f, const Expr& t, Value v) {
    if (Value* slot = t.ref(x, f)) {
      *slot = std::move(v);
    } else {
      auto* ix = static_cast<const IndexE*>(&t);
      Value o = ix->obj->eval(x, f);
      newindex_value(x, o, ix->key->eval(x, f), std::move(v), ix->line);
    }
  }
  const IndexE* single_index = nullptr;  // set by the parser for `t[k] = v`
  Flow exec(Exec& x, Frame& f) const override {
    if (targets.size() == 1 && exprs.size() == 1 && !exprs[0]->multi()) {
      if (const IndexE* ix = single_index) {  // t[k] = v: table and key first (Lua order)
        Value o = ix->obj->eval(x, f);
        Value k = ix->key->eval(x, f);
        newindex_value(x, o, k, exprs[0]->eval(x, f), ix->line);
      } else {
        store(x, f, *targets[0], exprs[0]->eval(x, f));
      }
      return NORMAL;
    }
    std::vector<Value> vs;
    eval_list(x, f, exprs, targets.size(), &vs);
    for (size_t i = 0; i < targets.size(); ++i) store(x, f, *targets[i], vs[i]);
    return NORMAL;
  }
};

struct CallS : Stmt {
  std::unique_ptr<CallE> call;
  Flow exec(Exec& x, Frame& f) const override {
    call->run(x, f);
    return NORMAL;
  }
};

struct DoS : Stmt {
  Block body;
  Flow exec(Exec& x, Frame& f) const override { return exec_block(x, f, body); }
};

struct WhileS : Stmt {
  ExprP cond;
  Block body;
  Flow exec(Exec& x, Frame& f) const override {
    while (cond->eval(x, f).truthy()) {
      x.step(line);
      const Flow r = exec_block(x, f, body);
      if (r == BREAK) break;
      if (r == RETURN) return r;
    }
    return NORMAL;
  }
};

struct RepeatS : Stmt {
  Block body;
  ExprP cond;
  Flow exec(Exec& x, Frame& f) const override {
    for (;;) {
      x.step(line);
      const Flow r = exec_block(x, f, body);
      if (r == BREAK) break;
      if (r == RETURN) return r;
      if (cond->eval(x, f).truthy()) break;
    }
    return NORMAL;
  }
};

struct IfS : Stmt {
  std::vector<ExprP> conds;
  std::vector<Block> blocks;  // blocks.size() == conds.size() (+1 with else)
  Flow exec(Exec& x, Frame& f) const override {
    for (size_t i = 0; i < conds.size(); ++i)
      if (conds[i]->eval(x, f).truthy()) return exec_block(x, f, blocks[i]);
    if (blocks.size() > conds.size()) return exec_block(x, f, blocks.back());
    return NORMAL;
  }
};

struct NumForS : Stmt {
  const VarInfo* var = nullptr;
  ExprP start, limit, step;
  Block body;
  Flow exec(Exec& x, Frame& f) const override {
    double a, b, s = 1;
    if (!tonumber(start->eval(x, f), &a)) x.error(line, "'for' initial value must be a number");
    if (!tonumber(limit->eval(x, f), &b)) x.error(line, "'for' limit must be a number");
    if (step && !tonumber(step->eval(x, f), &s)) x.error(line, "'for' step must be a number");
    if (s == 0) x.error(line, "'for' step is zero");
    for (double v = a; s > 0 ? v <= b : v >= b; v += s) {
      bind_local(f, var, Value::number(v));
      const Flow r = exec_block(x, f, body);
      if (r == BREAK) break;
      if (r == RETURN) return r;
    }
    return NORMAL;
  }
};

struct GenForS : Stmt {
  std::vector<const VarInfo*> vars;
  std::vector<ExprP> exprs;
  Block body;
  Flow exec(Exec& x, Frame& f) const override {
    std::vector<Value> init;
    eval_list(x, f, exprs, 3, &init);
    Value fn = init[0], state = init[1], ctl = init[2];
    for (;;) {
      x.step(line);
      std::vector<Value> args{state, ctl};
      std::vector<Value> r = x.call(fn, args, line);
      if (r.empty() || r[0].t == Value::NIL) break;
      ctl = r[0];
      for (size_t i = 0; i < vars.size(); ++i) bind_local(f, vars[i], i < r.size() ? r[i] : Value());
      const Flow fl = exec_block(x, f, body);
      if (fl == BREAK) break;
      if (fl == RETURN) return fl;
    }
    return NORMAL;
  }
};

struct ReturnS : Stmt {
  std::vector<ExprP> exprs;
  Flow exec(Exec& x, Frame& f) const override {
    f.ret.clear();
    eval_list(x, f, exprs, 0, &f.ret);
    return RETURN;
  }
};

struct BreakS : Stmt {
  Flow exec(Exec&, Frame&) const override { return BREAK; }
};

// ------------------------------------------------------------------ call ----
std::vector<Value> Exec::call(const Value& fn, std::vector<Value>& args, int line) {
  if (fn.t == Value::NATIVE) {
    auto* n = static_cast<Native*>(fn.o.get());
    try {
      return n->fn(args);
    } catch (const LuaError& e) {
      const std::string m = e.what();
      if (m.find(':') != std::string::npos && m.rfind(chunk, 0) == 0) throw;
      error(line, m);
    } catch (const std::exception& e) {
      error(line, std::string(n->name) + ": " + e.what());
    }
  }
  if (fn.t == Value::TABLE) {  // __call: the table is the first argument
    const Value h = metamethod(fn, M_CALL);
    if (h.t == Value::NIL) error(line, "attempt to call a table value");
    args.insert(args.begin(), fn);
    return call(h, args, line);
  }
  if (fn.t != Value::FUNC) error(line, "attempt to call a " + fn.type_name() + " value");
  if (++vm.depth_ > 200) {
    --vm.depth_;
    error(line, "stack overflow");
  }
  auto* c = static_cast<Closure*>(fn.o.get());
  const FuncProto* p = c->proto;
  Frame fr;
  fr.cl = c;
  fr.slots.resize(static_cast<size_t>(p->nslots));
  fr.cells.resize(static_cast<size_t>(p->nslots));
  const size_t np = p->params.size();
  for (size_t i = 0; i < np; ++i) bind_local(fr, p->params[i], i < args.size() ? args[i] : Value());
  if (p->vararg && args.size() > np) fr.varargs.assign(args.begin() + static_cast<std::ptrdiff_t>(np), args.end());
  std::vector<Value> out;
  try {
    if (exec_block(*this, fr, p->body) == Stmt::RETURN) out = std::move(fr.ret);
  } catch (...) {
    --vm.depth_;
    throw;
  }
  --vm.depth_;
  return out;
}

// ================================================================ parser ====
namespace {

struct FuncState {
  FuncProto* proto;
  FuncState* parent;
  std::vector<std::vector<std::pair<std::string, VarInfo*>>> blocks;  // scopes: name -> variable
  int next_slot = 0;
  std::vector<std::string> upnames;  // proto->upvals[i] is upnames[i]
};

class Parser {
 public:
  Parser(const std::string& src, const std::string& chunk, Chunk* out) : lx_(src, chunk), chunk_(chunk), out_(out) {
    advance();
  }

  void parse_chunk() {
    auto* p = new_proto("main chunk", 1);
    p->vararg = true;
    FuncState fs{p, nullptr, {}, 0, {}};
    fs_ = &fs;
    open_scope();
    p->body = block();
    if (tk_.t != T_EOF) error("'<eof>' expected near '" + tok_text() + "'");
    close_scope();
    p->nslots = fs.next_slot;
    out_->main = p;
  }

 private:
  // ---- tokens
  void advance() {
    if (has_ahead_) {
      tk_ = ahead_;
      has_ahead_ = false;
    } else {
      tk_ = lx_.next();
    }
  }
  const Token& peek() {
    if (!has_ahead_) {
      ahead_ = lx_.next();
      has_ahead_ = true;
    }
    return ahead_;
  }
  std::string tok_text() const {
    if (tk_.t == T_EOF) return "<eof>";
    if (tk_.t == T_NAME || tk_.t == T_STR) return tk_.s;
    if (tk_.t == T_NUM) return fmt_number(tk_.n);
    for (const auto& kv : keywords())
      if (kv.second == tk_.t) return kv.first;
    static const char* sym[] = {"+", "-", "*", "/", "//", "%", "^", "#", "==", "~=", "<=", ">=", "<", ">", "=", "(",
                                ")", "{", "}", "[", "]", ";", ":", ",", ".", "..", "...", "::"};
    return sym[tk_.t - S_PLUS];
  }
  [[noreturn]] void error(const std::string& m) const {
    throw LuaError(chunk_ + ":" + std::to_string(tk_.line) + ": " + m);
  }
  void expect(Tok t, const char* what) {
    if (tk_.t != t) error(std::string("'") + what + "' expected near '" + tok_text() + "'");
    advance();
  }
  bool accept(Tok t) {
    if (tk_.t != t) return false;
    advance();
    return true;
  }
  std::string name() {
    if (tk_.t != T_NAME) error("<name> expected near '" + tok_text() + "'");
    std::string s = tk_.s;
    advance();
    return s;
  }

  // ---- scopes
  FuncProto* new_proto(const std::string& name, int line) {
    out_->protos.push_back(std::make_unique<FuncProto>());
    auto* p = out_->protos.back().get();
    p->name = name;
    p->line = line;
    return p;
  }
  void open_scope() { fs_->blocks.emplace_back(); }
  void close_scope() { fs_->blocks.pop_back(); }
  VarInfo* declare(const std::string& n) {
    fs_->proto->vars.push_back(std::make_unique<VarInfo>());
    VarInfo* v = fs_->proto->vars.back().get();
    v->slot = fs_->next_slot++;
    fs_->blocks.back().emplace_back(n, v);
    return v;
  }
  static VarInfo* find_local(FuncState* fs, const std::string& n) {
    for (auto b = fs->blocks.rbegin(); b != fs->blocks.rend(); ++b)
      for (auto v = b->rbegin(); v != b->rend(); ++v)
        if (v->first == n) return v->second;
    return nullptr;
  }
  // index of `n` among fs's upvalues, adding it (and the chain above) on first use; -1 = global
  static int find_upval(FuncState* fs, const std::string& n) {
    for (size_t i = 0; i < fs->upnames.size(); ++i)
      if (fs->upnames[i] == n) return static_cast<int>(i);
    if (!fs->parent) return -1;
    UpDesc d{false, nullptr, -1};
    if (VarInfo* v = find_local(fs->parent, n)) {
      v->captured = true;
      d.from_local = true;
      d.var = v;
    } else {
      d.index = find_upval(fs->parent, n);
      if (d.index < 0) return -1;
    }
    fs->proto->upvals.push_back(d);
    fs->upnames.push_back(n);
    return static_cast<int>(fs->upnames.size()) - 1;
  }
  ExprP var_ref(const std::string& n, int line) {
    if (VarInfo* v = find_local(fs_, n)) {
      auto e = std::make_unique<LocalE>();
      e->var = v;
      e->line = line;
      return e;
    }
    const int up = find_upval(fs_, n);
    if (up >= 0) {
      auto e = std::make_unique<UpvalE>();
      e->index = up;
      e->line = line;
      return e;
    }
    auto g = std::make_unique<GlobalE>();
    g->name = n;
    g->line = line;
    return g;
  }

  // ---- statements
  static bool block_end(Tok t) { return t == T_EOF || t == K_END || t == K_ELSE || t == K_ELSEIF || t == K_UNTIL; }

  Block block() {
    Nest guard(*this);
    Block b;
    while (!block_end(tk_.t)) {
      if (tk_.t == K_RETURN) {
        b.push_back(return_stat());
        break;
      }
      if (StmtP s = statement()) b.push_back(std::move(s));
    }
    return b;
  }

  StmtP return_stat() {
    auto r = std::make_unique<ReturnS>();
    r->line = tk_.line;
    advance();
    if (!block_end(tk_.t) && tk_.t != S_SEMI) r->exprs = expr_list();
    accept(S_SEMI);
    return r;
  }

  StmtP statement() {
    const int line = tk_.line;
    switch (tk_.t) {
      case S_SEMI: advance(); return nullptr;
      case K_IF: return if_stat();
      case K_WHILE: {
        advance();
        auto s = std::make_unique<WhileS>();
        s->line = line;
        s->cond = expr();
        expect(K_DO, "do");
        open_scope();
        s->body = block();
        close_scope();
        expect(K_END, "end");
        return s;
      }
      case K_DO: {
        advance();
        auto s = std::make_unique<DoS>();
        s->line = line;
        open_scope();
        s->body = block();
        close_scope();
        expect(K_END, "end");
        return s;
      }
      case K_FOR: return for_stat();
      case K_REPEAT: {
        advance();
        auto s = std::make_unique<RepeatS>();
        s->line = line;
        open_scope();
        s->body = block();
        expect(K_UNTIL, "until");
        s->cond = expr();  // (sees the body's locals, as in Lua)
        close_scope();
        return s;
      }
      case K_FUNCTION: return function_stat();
      case K_LOCAL:
        advance();
        if (accept(K_FUNCTION)) return local_function();
        return local_stat(line);
      case K_BREAK: {
        advance();
        auto s = std::make_unique<BreakS>();
        s->line = line;
        return s;
      }
      case K_GOTO:
      case S_DCOLON: error("goto / labels are not supported by this interpreter");
      default: return expr_stat();
    }
  }

  StmtP if_stat() {
    auto s = std::make_unique<IfS>();
    s->line = tk_.line;
    advance();
    s->conds.push_back(expr());
    expect(K_THEN, "then");
    open_scope();
    s->blocks.push_back(block());
    close_scope();
    while (tk_.t == K_ELSEIF) {
      advance();
      s->conds.push_back(expr());
      expect(K_THEN, "then");
      open_scope();
      s->blocks.push_back(block());
      close_scope();
    }
    if (accept(K_ELSE)) {
      open_scope();
      s->blocks.push_back(block());
      close_scope();
    }
    expect(K_END, "end");
    return s;
  }

  StmtP for_stat() {
    const int line = tk_.line;
    advance();
    std::string n1 = name();
    if (tk_.t == S_ASSIGN) {
      advance();
      auto s = std::make_unique<NumForS>();
      s->line = line;
      s->start = expr();
      expect(S_COMMA, ",");
      s->limit = expr();
      if (accept(S_COMMA)) s->step = expr();
      expect(K_DO, "do");
      open_scope();
      s->var = declare(n1);
      s->body = block();
      close_scope();
      expect(K_END, "end");
      return s;
    }
    std::vector<std::string> names{n1};
    while (accept(S_COMMA)) names.push_back(name());
    expect(K_IN, "in");
    auto s = std::make_unique<GenForS>();
    s->line = line;
    s->exprs = expr_list();
    expect(K_DO, "do");
    open_scope();
    for (auto& n : names) s->vars.push_back(declare(n));
    s->body = block();
    close_scope();
    expect(K_END, "end");
    return s;
  }

  // function a.b.c:m(...) body end
  StmtP function_stat() {
    const int line = tk_.line;
    advance();
    std::string n = name();
    ExprP target = var_ref(n, line);
    std::string full = n;
    bool method = false;
    while (tk_.t == S_DOT || tk_.t == S_COLON) {
      method = tk_.t == S_COLON;
      advance();
      std::string k = name();
      full += (method ? ":" : ".") + k;
      auto ix = std::make_unique<IndexE>();
      ix->line = line;
      ix->obj = std::move(target);
      auto key = std::make_unique<ConstE>();
      key->v = Value::string(k);
      ix->key = std::move(key);
      target = std::move(ix);
      if (method) break;
    }
    auto s = std::make_unique<AssignS>();
    s->line = line;
    s->targets.push_back(std::move(target));
    s->single_index = dynamic_cast<const IndexE*>(s->targets[0].get());
    s->exprs.push_back(function_body(full, method, line));
    return s;
  }

  StmtP local_function() {
    const int line = tk_.line;
    std::string n = name();
    auto s = std::make_unique<LocalS>();
    s->line = line;
    s->vars.push_back(declare(n));  // visible inside its own body (recursion)
    s->function_decl = true;
    s->exprs.push_back(function_body(n, false, line));
    return s;
  }

  StmtP local_stat(int line) {
    std::vector<std::string> names{name()};
    while (accept(S_COMMA)) names.push_back(name());
    auto s = std::make_unique<LocalS>();
    s->line = line;
    if (accept(S_ASSIGN)) s->exprs = expr_list();  // evaluated before the names are visible
    for (auto& n : names) s->vars.push_back(declare(n));
    return s;
  }

  StmtP expr_stat() {
    const int line = tk_.line;
    ExprP e = suffixed_expr();
    if (tk_.t == S_ASSIGN || tk_.t == S_COMMA) {
      auto s = std::make_unique<AssignS>();
      s->line = line;
      check_assignable(*e);
      s->targets.push_back(std::move(e));
      while (accept(S_COMMA)) {
        ExprP t = suffixed_expr();
        check_assignable(*t);
        s->targets.push_back(std::move(t));
      }
      expect(S_ASSIGN, "=");
      s->exprs = expr_list();
      if (s->targets.size() == 1) s->single_index = dynamic_cast<const IndexE*>(s->targets[0].get());
      return s;
    }
    auto* call = dynamic_cast<CallE*>(e.get());
    if (!call) error("syntax error near '" + tok_text() + "'");
    auto s = std::make_unique<CallS>();
    s->line = line;
    e.release();
    s->call.reset(call);
    return s;
  }

  void check_assignable(const Expr& e) {
    if (!dynamic_cast<const LocalE*>(&e) && !dynamic_cast<const UpvalE*>(&e) && !dynamic_cast<const GlobalE*>(&e) &&
        !dynamic_cast<const IndexE*>(&e))
      error("syntax error: cannot assign to this expression");
  }

  // ---- expressions
  std::vector<ExprP> expr_list() {
    std::vector<ExprP> v;
    v.push_back(expr());
    while (accept(S_COMMA)) v.push_back(expr());
    return v;
  }

  ExprP function_body(const std::string& fname, bool self, int line) {
    auto* p = new_proto(fname, line);
    FuncState fs{p, fs_, {}, 0, {}};
    fs_ = &fs;
    open_scope();
    if (self) p->params.push_back(declare("self"));
    expect(S_LPAREN, "(");
    if (tk_.t != S_RPAREN) {
      do {
        if (tk_.t == S_DOTS) {
          advance();
          p->vararg = true;
          break;
        }
        p->params.push_back(declare(name()));
      } while (accept(S_COMMA));
    }
    p->nparams = static_cast<int>(p->params.size());
    p->has_self = self;
    expect(S_RPAREN, ")");
    p->body = block();
    expect(K_END, "end");
    close_scope();
    p->nslots = fs.next_slot;
    fs_ = fs.parent;
    auto e = std::make_unique<FunctionE>();
    e->line = line;
    e->proto = p;
    return e;
  }

  ExprP primary_expr() {
    const int line = tk_.line;
    if (tk_.t == T_NAME) return var_ref(name(), line);
    if (accept(S_LPAREN)) {
      ExprP e = expr();
      expect(S_RPAREN, ")");
      if (e->multi()) return one_value(std::move(e));  // (f()) truncates to one value
      return e;
    }
    error("unexpected symbol near '" + tok_text() + "'");
  }

  struct OneE : Expr {
    ExprP e;
    Value eval(Exec& x, Frame& f) const override { return e->eval(x, f); }
  };
  ExprP one_value(ExprP e) {
    auto o = std::make_unique<OneE>();
    o->line = e->line;
    o->e = std::move(e);
    return o;
  }

  ExprP suffixed_expr() {
    ExprP e = primary_expr();
    for (;;) {
      const int line = tk_.line;
      switch (tk_.t) {
        case S_DOT: {
          advance();
          auto ix = std::make_unique<IndexE>();
          ix->line = line;
          ix->obj = std::move(e);
          auto k = std::make_unique<ConstE>();
          k->v = Value::string(name());
          ix->key = std::move(k);
          e = std::move(ix);
          break;
        }
        case S_LBRACK: {
          advance();
          auto ix = std::make_unique<IndexE>();
          ix->line = line;
          ix->obj = std::move(e);
          ix->key = expr();
          expect(S_RBRACK, "]");
          e = std::move(ix);
          break;
        }
        case S_COLON: {
          advance();
          auto c = std::make_unique<CallE>();
          c->line = line;
          c->method = name();
          c->fn = std::move(e);
          c->args = call_args();
          e = std::move(c);
          break;
        }
        case S_LPAREN:
        case T_STR:
        case S_LBRACE: {
          auto c = std::make_unique<CallE>();
          c->line = line;
          c->fn = std::move(e);
          c->args = call_args();
          e = std::move(c);
          break;
        }
        default: return e;
      }
    }
  }

  std::vector<ExprP> call_args() {
    std::vector<ExprP> a;
    if (tk_.t == T_STR) {
      auto c = std::make_unique<ConstE>();
      c->v = Value::string(tk_.s);
      advance();
      a.push_back(std::move(c));
      return a;
    }
    if (tk_.t == S_LBRACE) {
      a.push_back(table_cons());
      return a;
    }
    expect(S_LPAREN, "(");
    if (tk_.t != S_RPAREN) a = expr_list();
    expect(S_RPAREN, ")");
    return a;
  }

  ExprP table_cons() {
    auto t = std::make_unique<TableE>();
    t->line = tk_.line;
    expect(S_LBRACE, "{");
    while (tk_.t != S_RBRACE) {
      if (tk_.t == S_LBRACK) {
        advance();
        ExprP k = expr();
        expect(S_RBRACK, "]");
        expect(S_ASSIGN, "=");
        t->keyed.emplace_back(std::move(k), expr());
        t->order.push_back(-static_cast<int>(t->keyed.size()));
      } else if (tk_.t == T_NAME && peek().t == S_ASSIGN) {
        auto k = std::make_unique<ConstE>();
        k->v = Value::string(name());
        advance();  // '='
        t->keyed.emplace_back(std::move(k), expr());
        t->order.push_back(-static_cast<int>(t->keyed.size()));
      } else {
        t->items.push_back(expr());
        t->order.push_back(static_cast<int>(t->items.size()) - 1);
      }
      if (!accept(S_COMMA) && !accept(S_SEMI)) break;
    }
    expect(S_RBRACE, "}");
    return t;
  }

  ExprP simple_expr() {
    const int line = tk_.line;
    auto cnst = [&](Value v) {
      auto c = std::make_unique<ConstE>();
      c->line = line;
      c->v = std::move(v);
      advance();
      return c;
    };
    switch (tk_.t) {
      case T_NUM: return cnst(Value::number(tk_.n));
      case T_STR: return cnst(Value::string(tk_.s));
      case K_NIL: return cnst(Value());
      case K_TRUE: return cnst(Value::boolean(true));
      case K_FALSE: return cnst(Value::boolean(false));
      case S_DOTS: {
        if (!fs_->proto->vararg) error("cannot use '...' outside a vararg function");
        advance();
        auto v = std::make_unique<VarargE>();
        v->line = line;
        return v;
      }
      case S_LBRACE: return table_cons();
      case K_FUNCTION: advance(); return function_body("anonymous", false, line);
      default: return suffixed_expr();
    }
  }

  // precedence climbing (Lua 5.1 priorities)
  struct Prio {
    int left, right;
  };
  bool binop(Tok t, BinOp* op, Prio* p, int* kind) const {
    *kind = 0;
    switch (t) {
      case S_PLUS: *op = B_ADD; *p = {6, 6}; return true;
      case S_MINUS: *op = B_SUB; *p = {6, 6}; return true;
      case S_STAR: *op = B_MUL; *p = {7, 7}; return true;
      case S_SLASH: *op = B_DIV; *p = {7, 7}; return true;
      case S_DSLASH: *op = B_IDIV; *p = {7, 7}; return true;
      case S_PCT: *op = B_MOD; *p = {7, 7}; return true;
      case S_CARET: *op = B_POW; *p = {10, 9}; return true;  // right assoc
      case S_CONCAT: *op = B_CONCAT; *p = {5, 4}; return true;  // right assoc
      case S_EQ: *op = B_EQ; *p = {3, 3}; return true;
      case S_NE: *op = B_NE; *p = {3, 3}; return true;
      case S_LT: *op = B_LT; *p = {3, 3}; return true;
      case S_LE: *op = B_LE; *p = {3, 3}; return true;
      case S_GT: *op = B_GT; *p = {3, 3}; return true;
      case S_GE: *op = B_GE; *p = {3, 3}; return true;
      case K_AND: *kind = 1; *p = {2, 2}; return true;
      case K_OR: *kind = 2; *p = {1, 1}; return true;
      default: return false;
    }
  }
  static constexpr int kUnaryPrio = 8;

  // (nesting depth of expressions / blocks: a pathological script cannot
  // recurse the parser off the C++ stack)
  struct Nest {
    Parser& p;
    explicit Nest(Parser& x) : p(x) {
      if (++p.nest_ > 200) p.error("chunk has too many syntax levels");
    }
    ~Nest() { --p.nest_; }
  };

  ExprP expr(int limit = 0) {
    Nest guard(*this);
    ExprP e;
    const int line = tk_.line;
    if (tk_.t == K_NOT || tk_.t == S_MINUS || tk_.t == S_HASH) {
      const Tok t = tk_.t;
      advance();
      auto u = std::make_unique<UnE>();
      u->line = line;
      u->op = t == K_NOT ? U_NOT : t == S_MINUS ? U_NEG : U_LEN;
      u->a = expr(kUnaryPrio);
      // fold a negative literal
      if (u->op == U_NEG)
        if (auto* c = dynamic_cast<ConstE*>(u->a.get()))
          if (c->v.t == Value::NUM) {
            c->v.n = -c->v.n;
            e = std::move(u->a);
          }
      if (!e) e = std::move(u);
    } else {
      e = simple_expr();
    }
    BinOp op;
    Prio p;
    int kind;
    while (binop(tk_.t, &op, &p, &kind) && p.left > limit) {
      const int l2 = tk_.line;
      advance();
      ExprP rhs = expr(p.right);
      if (kind == 1) {
        auto a = std::make_unique<AndE>();
        a->line = l2;
        a->a = std::move(e);
        a->b = std::move(rhs);
        e = std::move(a);
      } else if (kind == 2) {
        auto o = std::make_unique<OrE>();
        o->line = l2;
        o->a = std::move(e);
        o->b = std::move(rhs);
        e = std::move(o);
      } else {
        auto b = std::make_unique<BinE>();
        b->line = l2;
        b->op = op;
        b->a = std::move(e);
        b->b = std::move(rhs);
        e = std::move(b);
      }
    }
    return e;
  }

  Lexer lx_;
  std::string chunk_;
  Chunk* out_;
  Token tk_, ahead_;
  bool has_ahead_ = false;
  FuncState* fs_ = nullptr;
  int nest_ = 0;
};

}  // namespace

// ==================================================================== VM ====
VM::VM() { open_libs(); }
VM::~VM() = default;

Value VM::global(const std::string& name) const {
  auto it = globals_.find(name);
  return it == globals_.end() ? Value() : it->second;
}

void VM::set_global(const std::string& name, Value v) { globals_[name] = std::move(v); }

void VM::run(const std::string& source, const std::string& chunkname) {
  auto chunk = std::make_unique<Chunk>();
  Parser(source, chunkname, chunk.get()).parse_chunk();
  chunkname_ = chunkname;
  auto c = std::make_shared<Closure>();
  c->proto = chunk->main;
  chunks_.push_back(std::move(chunk));
  Value fn;
  fn.t = Value::FUNC;
  fn.o = std::move(c);
  call(fn, {});
}

std::vector<Value> VM::call(const Value& fn, std::vector<Value> args) {
  Exec x{*this, chunkname_};
  steps_ = 0;
  return x.call(fn, args, 0);
}

// ------------------------------------------------------------- libraries ----
namespace {

const Value& arg(std::vector<Value>& a, size_t i) {
  static const Value nil;
  return i < a.size() ? a[i] : nil;
}
double num_arg(std::vector<Value>& a, size_t i, const char* fn) {
  double d;
  if (!tonumber(arg(a, i), &d))
    throw LuaError(std::string("bad argument #") + std::to_string(i + 1) + " to '" + fn + "' (number expected, got " +
                   arg(a, i).type_name() + ")");
  return d;
}
std::string str_arg(std::vector<Value>& a, size_t i, const char* fn) {
  const Value& v = arg(a, i);
  if (v.t == Value::STR) return v.str();
  if (v.t == Value::NUM) return fmt_number(v.n);
  throw LuaError(std::string("bad argument #") + std::to_string(i + 1) + " to '" + fn + "' (string expected, got " +
                 v.type_name() + ")");
}
Table* tab_arg(std::vector<Value>& a, size_t i, const char* fn) {
  if (arg(a, i).t != Value::TABLE)
    throw LuaError(std::string("bad argument #") + std::to_string(i + 1) + " to '" + fn + "' (table expected, got " +
                   arg(a, i).type_name() + ")");
  return a[i].tab();
}

using Fn = std::function<std::vector<Value>(std::vector<Value>&)>;

// next(t, k) over the array part, then the hash part (insertion-independent
// but stable while the table is not modified)
std::vector<Value> table_next(Table* t, const Value& k) {
  size_t i = 0;
  if (k.t == Value::NIL) {
    i = 0;
  } else if (array_index(k, &i) && i <= t->arr.size()) {
    // continue in the array part
  } else {
    auto it = t->hash.find(k);
    if (it == t->hash.end()) throw LuaError("invalid key to 'next'");
    for (++it; it != t->hash.end(); ++it)
      if (it->second.t != Value::NIL) return {it->first, it->second};
    return {Value()};
  }
  for (; i < t->arr.size(); ++i)
    if (t->arr[i].t != Value::NIL) return {Value::number(static_cast<double>(i + 1)), t->arr[i]};
  for (auto it = t->hash.begin(); it != t->hash.end(); ++it)
    if (it->second.t != Value::NIL) return {it->first, it->second};
  return {Value()};
}

// ---- Lua patterns (string.find / match / gmatch / gsub): backtracking
// matcher over single-char classes (. %a %d %l %s %u %w %x %p %c and their
// complements), sets [...], quantifiers * + - ?, anchors, captures (incl.
// position captures), back-references %1-%9, %b and %f
class Pattern {
 public:
  static constexpr int kMaxCaps = 32;
  static constexpr std::ptrdiff_t kPos = -2, kOpen = -1;

  Pattern(const std::string& s, const std::string& p)
      : src_(s.data()), src_end_(s.data() + s.size()), pat_(p.data()), pat_end_(p.data() + p.size()) {}

  // match at s (an offset into the subject): end offset, or -1
  std::ptrdiff_t match_at(std::ptrdiff_t s, std::ptrdiff_t p) {
    level_ = 0;
    depth_ = 0;
    const char* e = match(src_ + s, pat_ + p);
    return e ? e - src_ : -1;
  }
  int captures() const { return level_; }
  // capture i (or the whole match s..e when the pattern has none and i == 0)
  Value capture(int i, std::ptrdiff_t s, std::ptrdiff_t e) const {
    if (i >= level_) {
      if (i == 0) return Value::string(std::string(src_ + s, static_cast<size_t>(e - s)));
      throw LuaError("invalid capture index");
    }
    if (cap_[i].len == kPos) return Value::number(static_cast<double>(cap_[i].init - src_ + 1));
    if (cap_[i].len == kOpen) throw LuaError("unfinished capture");
    return Value::string(std::string(cap_[i].init, static_cast<size_t>(cap_[i].len)));
  }
  std::vector<Value> all_captures(std::ptrdiff_t s, std::ptrdiff_t e, bool whole_if_none) const {
    std::vector<Value> r;
    const int n = (level_ == 0 && whole_if_none) ? 1 : level_;
    for (int i = 0; i < n; ++i) r.push_back(capture(i, s, e));
    return r;
  }

 private:
  struct Cap {
    const char* init;
    std::ptrdiff_t len;
  };

  static bool in_class(int c, int cl) {
    bool r;
    switch (std::tolower(cl)) {
      case 'a': r = std::isalpha(c); break;
      case 'c': r = std::iscntrl(c); break;
      case 'd': r = std::isdigit(c); break;
      case 'l': r = std::islower(c); break;
      case 'p': r = std::ispunct(c); break;
      case 's': r = std::isspace(c); break;
      case 'u': r = std::isupper(c); break;
      case 'w': r = std::isalnum(c); break;
      case 'x': r = std::isxdigit(c); break;
      default: return cl == c;  // %. %% %( ...: the character itself
    }
    return std::isupper(cl) ? !r : r;
  }
  // one past the class item starting at p
  const char* item_end(const char* p) const {
    const char c = *p++;
    if (c == '%') {
      if (p >= pat_end_) throw LuaError("malformed pattern (ends with '%')");
      return p + 1;
    }
    if (c == '[') {
      if (p < pat_end_ && *p == '^') ++p;
      do {  // (a ']' right after '[' or '[^' is a member)
        if (p >= pat_end_) throw LuaError("malformed pattern (missing ']')");
        const char d = *p++;
        if (d == '%' && p < pat_end_) ++p;
      } while (p >= pat_end_ || *p != ']');
      return p + 1;
    }
    return p;
  }
  // set [..] from p ('[') to close (its ']')
  static bool in_set(int c, const char* p, const char* close) {
    bool yes = true;
    if (p[1] == '^') {
      yes = false;
      ++p;
    }
    while (++p < close) {
      if (*p == '%' && p + 1 < close) {
        ++p;
        if (in_class(c, static_cast<unsigned char>(*p))) return yes;
      } else if (p + 2 < close && p[1] == '-') {
        if (static_cast<unsigned char>(p[0]) <= c && c <= static_cast<unsigned char>(p[2])) return yes;
        p += 2;
      } else if (static_cast<unsigned char>(*p) == c) {
        return yes;
      }
    }
    return !yes;
  }
  bool single(const char* s, const char* p, const char* ep) const {
    if (s >= src_end_) return false;
    const int c = static_cast<unsigned char>(*s);
    switch (*p) {
      case '.': return true;
      case '%': return in_class(c, static_cast<unsigned char>(p[1]));
      case '[': return in_set(c, p, ep - 1);
      default: return static_cast<unsigned char>(*p) == c;
    }
  }

  const char* match(const char* s, const char* p) {
    struct Depth {
      int& d;
      explicit Depth(int& x) : d(x) {
        if (++d > 220) throw LuaError("pattern too complex");
      }
      ~Depth() { --d; }
    } guard(depth_);
    while (p < pat_end_) {
      switch (*p) {
        case '(':
          if (p + 1 < pat_end_ && p[1] == ')') return open_capture(s, p + 2, kPos);
          return open_capture(s, p + 1, kOpen);
        case ')': return close_capture(s, p + 1);
        case '$':
          if (p + 1 == pat_end_) return s == src_end_ ? s : nullptr;
          break;
        case '%':
          if (p + 1 < pat_end_ && p[1] == 'b') {
            s = balance(s, p + 2);
            if (!s) return nullptr;
            p += 4;
            continue;
          }
          if (p + 1 < pat_end_ && p[1] == 'f') {
            p += 2;
            if (p >= pat_end_ || *p != '[') throw LuaError("missing '[' after '%f' in pattern");
            const char* ep = item_end(p);
            const int prev = s == src_ ? 0 : static_cast<unsigned char>(s[-1]);
            const int cur = s < src_end_ ? static_cast<unsigned char>(*s) : 0;
            if (in_set(prev, p, ep - 1) || !in_set(cur, p, ep - 1)) return nullptr;
            p = ep;
            continue;
          }
          if (p + 1 < pat_end_ && std::isdigit(static_cast<unsigned char>(p[1]))) {
            s = backref(s, p[1]);
            if (!s) return nullptr;
            p += 2;
            continue;
          }
          break;
        default: break;
      }
      const char* ep = item_end(p);
      const char q = ep < pat_end_ ? *ep : '\0';
      if (q == '?') {
        if (single(s, p, ep))
          if (const char* r = match(s + 1, ep + 1)) return r;
        p = ep + 1;
        continue;
      }
      if (q == '+') return single(s, p, ep) ? greedy(s + 1, p, ep) : nullptr;
      if (q == '*') return greedy(s, p, ep);
      if (q == '-') return lazy(s, p, ep);
      if (!single(s, p, ep)) return nullptr;
      ++s;
      p = ep;
    }
    return s;
  }
  const char* greedy(const char* s, const char* p, const char* ep) {
    std::ptrdiff_t n = 0;
    while (single(s + n, p, ep)) ++n;
    for (; n >= 0; --n)
      if (const char* r = match(s + n, ep + 1)) return r;
    return nullptr;
  }
  const char* lazy(const char* s, const char* p, const char* ep) {
    for (;;) {
      if (const char* r = match(s, ep + 1)) return r;
      if (!single(s, p, ep)) return nullptr;
      ++s;
    }
  }
  const char* open_capture(const char* s, const char* p, std::ptrdiff_t what) {
    if (level_ >= kMaxCaps) throw LuaError("too many captures");
    cap_[level_] = {s, what};
    ++level_;
    const char* r = match(s, p);
    if (!r) --level_;
    return r;
  }
  const char* close_capture(const char* s, const char* p) {
    int l = level_ - 1;
    while (l >= 0 && cap_[l].len != kOpen) --l;
    if (l < 0) throw LuaError("invalid pattern capture");
    cap_[l].len = s - cap_[l].init;
    const char* r = match(s, p);
    if (!r) cap_[l].len = kOpen;
    return r;
  }
  const char* balance(const char* s, const char* p) const {
    if (p + 1 >= pat_end_) throw LuaError("missing arguments to '%b'");
    if (s >= src_end_ || *s != p[0]) return nullptr;
    int open = 1;
    while (++s < src_end_) {
      if (*s == p[1]) {
        if (--open == 0) return s + 1;
      } else if (*s == p[0]) {
        ++open;
      }
    }
    return nullptr;
  }
  const char* backref(const char* s, char d) const {
    const int l = d - '1';
    if (l < 0 || l >= level_ || cap_[l].len == kOpen) throw LuaError("invalid capture index");
    const size_t n = static_cast<size_t>(cap_[l].len);
    if (static_cast<size_t>(src_end_ - s) >= n && std::memcmp(cap_[l].init, s, n) == 0) return s + n;
    return nullptr;
  }

  const char *src_, *src_end_, *pat_, *pat_end_;
  int level_ = 0, depth_ = 0;
  Cap cap_[kMaxCaps];
};

bool has_specials(const std::string& p) { return p.find_first_of("^$*+?.([%-") != std::string::npos; }

// 1-based (negative from the end) string position -> 0-based offset in [0, n]
std::ptrdiff_t str_start(double i, size_t n) {
  std::ptrdiff_t k = static_cast<std::ptrdiff_t>(i);
  if (k < 0) k = static_cast<std::ptrdiff_t>(n) + k + 1;
  if (k < 1) k = 1;
  return k - 1;
}

// string.find (find = true) / string.match
std::vector<Value> str_find(std::vector<Value>& a, bool find) {
  const char* fn = find ? "find" : "match";
  const std::string s = str_arg(a, 0, fn), p = str_arg(a, 1, fn);
  const std::ptrdiff_t init = str_start(a.size() > 2 && a[2].t != Value::NIL ? num_arg(a, 2, fn) : 1, s.size());
  if (init > static_cast<std::ptrdiff_t>(s.size())) return {Value()};
  if (find && ((a.size() > 3 && a[3].truthy()) || !has_specials(p))) {
    const size_t at = s.find(p, static_cast<size_t>(init));
    if (at == std::string::npos) return {Value()};
    return {Value::number(static_cast<double>(at + 1)), Value::number(static_cast<double>(at + p.size()))};
  }
  Pattern m(s, p);
  const bool anchor = !p.empty() && p[0] == '^';
  for (std::ptrdiff_t i = init; i <= static_cast<std::ptrdiff_t>(s.size()); ++i) {
    const std::ptrdiff_t e = m.match_at(i, anchor ? 1 : 0);
    if (e >= 0) {
      if (!find) return m.all_captures(i, e, true);
      std::vector<Value> r{Value::number(static_cast<double>(i + 1)), Value::number(static_cast<double>(e))};
      for (auto& c : m.all_captures(i, e, false)) r.push_back(c);
      return r;
    }
    if (anchor) break;
  }
  return {Value()};
}

std::string lua_format(std::vector<Value>& a) {
  const std::string f = str_arg(a, 0, "format");
  std::string out;
  size_t ai = 1;
  for (size_t i = 0; i < f.size(); ++i) {
    if (f[i] != '%') {
      out += f[i];
      continue;
    }
    if (++i >= f.size()) throw LuaError("invalid option '%' to 'format'");
    if (f[i] == '%') {
      out += '%';
      continue;
    }
    std::string spec = "%";
    while (i < f.size() && std::strchr("-+ #0123456789.", f[i])) spec += f[i++];
    if (i >= f.size()) throw LuaError("invalid conversion to 'format'");
    const char c = f[i];
    char buf[512];
    switch (c) {
      case 'd':
      case 'i':
        std::snprintf(buf, sizeof(buf), (spec + "lld").c_str(), static_cast<long long>(num_arg(a, ai++, "format")));
        break;
      case 'x':
      case 'X':
      case 'o':
      case 'u':
      case 'c':
        std::snprintf(buf, sizeof(buf), (spec + (c == 'c' ? "c" : std::string("ll") + c)).c_str(),
                      static_cast<long long>(num_arg(a, ai++, "format")));
        break;
      case 'e':
      case 'E':
      case 'f':
      case 'g':
      case 'G':
        std::snprintf(buf, sizeof(buf), (spec + c).c_str(), num_arg(a, ai++, "format"));
        break;
      case 's':
        std::snprintf(buf, sizeof(buf), (spec + "s").c_str(), tostring(arg(a, ai++)).c_str());
        break;
      case 'q': {
        std::string s = "\"";
        for (char ch : str_arg(a, ai++, "format")) {
          if (ch == '"' || ch == '\\') s += '\\';
          if (ch == '\n') {
            s += "\\n";
            continue;
          }
          s += ch;
        }
        out += s + "\"";
        continue;
      }
      default: throw LuaError(std::string("invalid option '%") + c + "' to 'format'");
    }
    out += buf;
  }
  return out;
}

}  // namespace

void VM::open_libs() {
  auto reg = [&](Table* t, const std::string& n, Fn f) { t->set(Value::string(n), Value::native(n, std::move(f))); };
  auto& G = globals_;
  auto g = [&](const std::string& n, Fn f) { G[n] = Value::native(n, std::move(f)); };

  // tostring honouring __tostring
  auto to_str = [this](const Value& v) {
    const Value h = metamethod(v, M_TOSTRING);
    if (h.t == Value::NIL) return tostring(v);
    Exec x{*this, chunkname_};
    const Value r = call1(x, h, {v}, 0);
    if (r.t != Value::STR && r.t != Value::NUM) throw LuaError("'__tostring' must return a string");
    return tostring(r);
  };
  g("print", [to_str](std::vector<Value>& a) {
    std::string s;
    for (size_t i = 0; i < a.size(); ++i) s += (i ? "\t" : "") + to_str(a[i]);
    std::fprintf(stdout, "%s\n", s.c_str());
    std::fflush(stdout);
    return std::vector<Value>{};
  });
  g("type", [](std::vector<Value>& a) {
    if (a.empty()) throw LuaError("bad argument #1 to 'type' (value expected)");
    return std::vector<Value>{Value::string(a[0].type_name())};
  });
  g("tostring", [to_str](std::vector<Value>& a) { return std::vector<Value>{Value::string(to_str(arg(a, 0)))}; });
  g("setmetatable", [](std::vector<Value>& a) {
    Table* t = tab_arg(a, 0, "setmetatable");
    const Value& mt = arg(a, 1);
    if (mt.t != Value::NIL && mt.t != Value::TABLE)
      throw LuaError("bad argument #2 to 'setmetatable' (nil or table expected)");
    if (t->meta && t->meta->get(meta_name(M_METATABLE)).t != Value::NIL)
      throw LuaError("cannot change a protected metatable");
    t->meta = mt.t == Value::TABLE ? std::static_pointer_cast<Table>(mt.o) : nullptr;
    return std::vector<Value>{a[0]};
  });
  g("getmetatable", [](std::vector<Value>& a) {
    const Value& v = arg(a, 0);
    if (v.t != Value::TABLE || !v.tab()->meta) return std::vector<Value>{Value()};
    const Value prot = v.tab()->meta->get(meta_name(M_METATABLE));
    if (prot.t != Value::NIL) return std::vector<Value>{prot};
    return std::vector<Value>{Value::table(v.tab()->meta)};
  });
  g("tonumber", [](std::vector<Value>& a) {
    const Value& v = arg(a, 0);
    if (a.size() > 1 && arg(a, 1).t == Value::NUM) {
      const int base = static_cast<int>(arg(a, 1).n);
      const std::string s = tostring(v);
      char* end = nullptr;
      const long long r = std::strtoll(s.c_str(), &end, base);
      if (end == s.c_str() || *end) return std::vector<Value>{Value()};
      return std::vector<Value>{Value::number(static_cast<double>(r))};
    }
    double d;
    return std::vector<Value>{tonumber(v, &d) ? Value::number(d) : Value()};
  });
  g("error", [](std::vector<Value>& a) -> std::vector<Value> { throw LuaError(tostring(arg(a, 0))); });
  g("assert", [](std::vector<Value>& a) {
    if (!arg(a, 0).truthy()) throw LuaError(a.size() > 1 ? tostring(a[1]) : "assertion failed!");
    return a;
  });
  g("next", [](std::vector<Value>& a) { return table_next(tab_arg(a, 0, "next"), arg(a, 1)); });
  Value next_fn = G["next"];
  g("pairs", [next_fn](std::vector<Value>& a) {
    tab_arg(a, 0, "pairs");
    return std::vector<Value>{next_fn, a[0], Value()};
  });
  Value inext = Value::native("ipairs_iter", [](std::vector<Value>& a) {
    const double i = num_arg(a, 1, "ipairs") + 1;
    Value v = arg(a, 0).t == Value::TABLE ? a[0].tab()->get(Value::number(i))
              : arg(a, 0).t == Value::USERDATA && i <= a[0].ud()->length() ? a[0].ud()->index(Value::number(i))
                                                                            : Value();
    if (v.t == Value::NIL) return std::vector<Value>{Value()};
    return std::vector<Value>{Value::number(i), v};
  });
  g("ipairs", [inext](std::vector<Value>& a) {
    if (arg(a, 0).t != Value::TABLE && arg(a, 0).t != Value::USERDATA)
      throw LuaError("bad argument #1 to 'ipairs' (table expected)");
    return std::vector<Value>{inext, a[0], Value::number(0)};
  });
  g("select", [](std::vector<Value>& a) {
    if (arg(a, 0).t == Value::STR && a[0].str() == "#")
      return std::vector<Value>{Value::number(static_cast<double>(a.size() - 1))};
    const double n = num_arg(a, 0, "select");
    if (n < 1) throw LuaError("bad argument #1 to 'select' (index out of range)");
    std::vector<Value> r;
    for (size_t i = static_cast<size_t>(n); i < a.size(); ++i) r.push_back(a[i]);
    return r;
  });
  g("unpack", [](std::vector<Value>& a) {
    Table* t = tab_arg(a, 0, "unpack");
    const double i0 = a.size() > 1 && a[1].t != Value::NIL ? num_arg(a, 1, "unpack") : 1;
    const double i1 = a.size() > 2 && a[2].t != Value::NIL ? num_arg(a, 2, "unpack") : static_cast<double>(t->length());
    std::vector<Value> r;
    for (double i = i0; i <= i1; ++i) r.push_back(t->get(Value::number(i)));
    return r;
  });
  g("rawget", [](std::vector<Value>& a) { return std::vector<Value>{tab_arg(a, 0, "rawget")->get(arg(a, 1))}; });
  g("rawset", [](std::vector<Value>& a) {
    tab_arg(a, 0, "rawset")->set(arg(a, 1), arg(a, 2));
    return std::vector<Value>{a[0]};
  });
  g("rawequal", [](std::vector<Value>& a) { return std::vector<Value>{Value::boolean(ValueEq()(arg(a, 0), arg(a, 1)))}; });
  g("pcall", [this](std::vector<Value>& a) {
    if (a.empty()) throw LuaError("bad argument #1 to 'pcall' (value expected)");
    std::vector<Value> rest(a.begin() + 1, a.end());
    Exec x{*this, chunkname_};
    try {
      std::vector<Value> r = x.call(a[0], rest, 0);
      r.insert(r.begin(), Value::boolean(true));
      return r;
    } catch (const LuaError& e) {
      return std::vector<Value>{Value::boolean(false), Value::string(e.what())};
    }
  });
  G["_G"] = Value();  // (no first-class globals table)

  // math
  auto math = std::make_shared<Table>();
  auto m1 = [&](const std::string& n, double (*f)(double)) {
    reg(math.get(), n, [f, n](std::vector<Value>& a) { return std::vector<Value>{Value::number(f(num_arg(a, 0, n.c_str())))}; });
  };
  m1("floor", std::floor);
  m1("ceil", std::ceil);
  m1("abs", std::fabs);
  m1("sqrt", std::sqrt);
  m1("exp", std::exp);
  m1("sin", std::sin);
  m1("cos", std::cos);
  m1("tan", std::tan);
  m1("asin", std::asin);
  m1("acos", std::acos);
  m1("atan", std::atan);
  m1("sinh", std::sinh);
  m1("cosh", std::cosh);
  m1("tanh", std::tanh);
  m1("log10", std::log10);
  reg(math.get(), "log", [](std::vector<Value>& a) {
    const double x = num_arg(a, 0, "log");
    if (a.size() > 1 && a[1].t != Value::NIL) return std::vector<Value>{Value::number(std::log(x) / std::log(num_arg(a, 1, "log")))};
    return std::vector<Value>{Value::number(std::log(x))};
  });
  reg(math.get(), "atan2", [](std::vector<Value>& a) {
    return std::vector<Value>{Value::number(std::atan2(num_arg(a, 0, "atan2"), num_arg(a, 1, "atan2")))};
  });
  reg(math.get(), "pow", [](std::vector<Value>& a) {
    return std::vector<Value>{Value::number(std::pow(num_arg(a, 0, "pow"), num_arg(a, 1, "pow")))};
  });
  reg(math.get(), "fmod", [](std::vector<Value>& a) {
    return std::vector<Value>{Value::number(std::fmod(num_arg(a, 0, "fmod"), num_arg(a, 1, "fmod")))};
  });
  reg(math.get(), "modf", [](std::vector<Value>& a) {
    double ip;
    const double fp = std::modf(num_arg(a, 0, "modf"), &ip);
    return std::vector<Value>{Value::number(ip), Value::number(fp)};
  });
  reg(math.get(), "max", [](std::vector<Value>& a) {
    double m = num_arg(a, 0, "max");
    for (size_t i = 1; i < a.size(); ++i) m = std::max(m, num_arg(a, i, "max"));
    return std::vector<Value>{Value::number(m)};
  });
  reg(math.get(), "min", [](std::vector<Value>& a) {
    double m = num_arg(a, 0, "min");
    for (size_t i = 1; i < a.size(); ++i) m = std::min(m, num_arg(a, i, "min"));
    return std::vector<Value>{Value::number(m)};
  });
  auto rng = std::make_shared<std::mt19937_64>(0x5eed);
  reg(math.get(), "random", [rng](std::vector<Value>& a) {
    const double u = std::uniform_real_distribution<double>(0.0, 1.0)(*rng);
    if (a.empty()) return std::vector<Value>{Value::number(u)};
    double lo = 1, hi = num_arg(a, 0, "random");
    if (a.size() > 1) {
      lo = hi;
      hi = num_arg(a, 1, "random");
    }
    if (lo > hi) throw LuaError("bad argument to 'random' (interval is empty)");
    return std::vector<Value>{Value::number(std::floor(lo + u * (std::floor(hi) - std::floor(lo) + 1)))};
  });
  reg(math.get(), "randomseed", [rng](std::vector<Value>& a) {
    rng->seed(static_cast<uint64_t>(static_cast<int64_t>(num_arg(a, 0, "randomseed"))));
    return std::vector<Value>{};
  });
  math->set(Value::string("pi"), Value::number(M_PI));
  math->set(Value::string("huge"), Value::number(HUGE_VAL));
  G["math"] = Value::table(math);

  // string
  auto str = std::make_shared<Table>();
  reg(str.get(), "len", [](std::vector<Value>& a) {
    return std::vector<Value>{Value::number(static_cast<double>(str_arg(a, 0, "len").size()))};
  });
  reg(str.get(), "sub", [](std::vector<Value>& a) {
    const std::string s = str_arg(a, 0, "sub");
    const long n = static_cast<long>(s.size());
    long i = a.size() > 1 ? static_cast<long>(num_arg(a, 1, "sub")) : 1;
    long j = a.size() > 2 && a[2].t != Value::NIL ? static_cast<long>(num_arg(a, 2, "sub")) : -1;
    if (i < 0) i = std::max(n + i + 1, 1L);
    if (i == 0) i = 1;
    if (j < 0) j = n + j + 1;
    if (j > n) j = n;
    return std::vector<Value>{Value::string(i > j ? "" : s.substr(static_cast<size_t>(i - 1), static_cast<size_t>(j - i + 1)))};
  });
  reg(str.get(), "upper", [](std::vector<Value>& a) {
    std::string s = str_arg(a, 0, "upper");
    for (auto& c : s) c = static_cast<char>(std::toupper(static_cast<unsigned char>(c)));
    return std::vector<Value>{Value::string(s)};
  });
  reg(str.get(), "lower", [](std::vector<Value>& a) {
    std::string s = str_arg(a, 0, "lower");
    for (auto& c : s) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
    return std::vector<Value>{Value::string(s)};
  });
  reg(str.get(), "rep", [](std::vector<Value>& a) {
    const std::string s = str_arg(a, 0, "rep");
    std::string r;
    for (long k = static_cast<long>(num_arg(a, 1, "rep")); k > 0; --k) r += s;
    return std::vector<Value>{Value::string(r)};
  });
  reg(str.get(), "reverse", [](std::vector<Value>& a) {
    std::string s = str_arg(a, 0, "reverse");
    std::reverse(s.begin(), s.end());
    return std::vector<Value>{Value::string(s)};
  });
  reg(str.get(), "byte", [](std::vector<Value>& a) {
    const std::string s = str_arg(a, 0, "byte");
    const long n = static_cast<long>(s.size());
    long i = a.size() > 1 && a[1].t != Value::NIL ? static_cast<long>(num_arg(a, 1, "byte")) : 1;
    long j = a.size() > 2 && a[2].t != Value::NIL ? static_cast<long>(num_arg(a, 2, "byte")) : i;
    if (i < 0) i = n + i + 1;
    if (j < 0) j = n + j + 1;
    if (i < 1) i = 1;
    if (j > n) j = n;
    std::vector<Value> r;
    for (long k = i; k <= j; ++k) r.push_back(Value::number(static_cast<unsigned char>(s[static_cast<size_t>(k - 1)])));
    return r;
  });
  reg(str.get(), "char", [](std::vector<Value>& a) {
    std::string s;
    for (size_t i = 0; i < a.size(); ++i) s += static_cast<char>(static_cast<int>(num_arg(a, i, "char")));
    return std::vector<Value>{Value::string(s)};
  });
  reg(str.get(), "format", [](std::vector<Value>& a) { return std::vector<Value>{Value::string(lua_format(a))}; });
  reg(str.get(), "find", [](std::vector<Value>& a) { return str_find(a, true); });
  reg(str.get(), "match", [](std::vector<Value>& a) { return str_find(a, false); });
  reg(str.get(), "gmatch", [](std::vector<Value>& a) {
    struct State {
      std::string s, p;
      std::ptrdiff_t pos = 0;
    };
    auto st = std::make_shared<State>();
    st->s = str_arg(a, 0, "gmatch");
    st->p = str_arg(a, 1, "gmatch");
    return std::vector<Value>{Value::native("gmatch_iter", [st](std::vector<Value>&) {
      Pattern m(st->s, st->p);
      for (std::ptrdiff_t i = st->pos; i <= static_cast<std::ptrdiff_t>(st->s.size()); ++i) {
        const std::ptrdiff_t e = m.match_at(i, 0);
        if (e >= 0) {
          st->pos = e == i ? e + 1 : e;  // an empty match steps one character on
          return m.all_captures(i, e, true);
        }
      }
      st->pos = static_cast<std::ptrdiff_t>(st->s.size()) + 1;
      return std::vector<Value>{Value()};
    })};
  });
  reg(str.get(), "gsub", [this](std::vector<Value>& a) {
    const std::string s = str_arg(a, 0, "gsub"), p = str_arg(a, 1, "gsub");
    const Value repl = arg(a, 2);
    if (repl.t != Value::STR && repl.t != Value::NUM && repl.t != Value::TABLE && repl.t != Value::FUNC &&
        repl.t != Value::NATIVE)
      throw LuaError("bad argument #3 to 'gsub' (string/function/table expected)");
    const double max_n = a.size() > 3 && a[3].t != Value::NIL ? num_arg(a, 3, "gsub") : 1e300;
    const bool anchor = !p.empty() && p[0] == '^';
    Pattern m(s, p);
    Exec x{*this, chunkname_};
    std::string out;
    double n = 0;
    std::ptrdiff_t i = 0;
    const std::ptrdiff_t len = static_cast<std::ptrdiff_t>(s.size());
    while (n < max_n) {
      const std::ptrdiff_t e = m.match_at(i, anchor ? 1 : 0);
      if (e >= 0) {
        ++n;
        const std::string whole = s.substr(static_cast<size_t>(i), static_cast<size_t>(e - i));
        Value v;
        if (repl.t == Value::STR || repl.t == Value::NUM) {
          const std::string r = repl.t == Value::STR ? repl.str() : fmt_number(repl.n);
          std::string add;
          for (size_t k = 0; k < r.size(); ++k) {
            if (r[k] != '%') {
              add += r[k];
              continue;
            }
            if (++k >= r.size()) throw LuaError("invalid use of '%' in replacement string");
            if (r[k] == '%') {
              add += '%';
            } else if (std::isdigit(static_cast<unsigned char>(r[k]))) {
              add += r[k] == '0' ? whole : tostring(m.capture(r[k] - '1', i, e));
            } else {
              throw LuaError("invalid use of '%' in replacement string");
            }
          }
          v = Value::string(add);
        } else {
          const Value key = m.capture(0, i, e);
          if (repl.t == Value::TABLE) {
            v = index_value(x, repl, key, 0);
          } else {
            std::vector<Value> caps = m.all_captures(i, e, true);
            std::vector<Value> r = x.call(repl, caps, 0);
            v = r.empty() ? Value() : r[0];
          }
        }
        if (!v.truthy())
          out += whole;  // false / nil: keep the match
        else if (v.t == Value::STR || v.t == Value::NUM)
          out += tostring(v);
        else
          throw LuaError("invalid replacement value (a " + v.type_name() + ")");
      }
      if (e >= 0 && e > i)
        i = e;
      else if (i < len)
        out += s[static_cast<size_t>(i++)];
      else
        break;
      if (anchor) break;
    }
    if (i < len) out += s.substr(static_cast<size_t>(i));
    return std::vector<Value>{Value::string(out), Value::number(n)};
  });
  G["string"] = Value::table(str);

  // table
  auto tab = std::make_shared<Table>();
  reg(tab.get(), "insert", [](std::vector<Value>& a) {
    Table* t = tab_arg(a, 0, "insert");
    if (a.size() == 2) {
      t->set(Value::number(static_cast<double>(t->length() + 1)), a[1]);
    } else if (a.size() == 3) {
      const size_t n = t->length();
      const size_t pos = static_cast<size_t>(num_arg(a, 1, "insert"));
      if (pos < 1 || pos > n + 1) throw LuaError("bad argument #2 to 'insert' (position out of bounds)");
      for (size_t i = n; i >= pos; --i) t->set(Value::number(static_cast<double>(i + 1)), t->get(Value::number(static_cast<double>(i))));
      t->set(Value::number(static_cast<double>(pos)), a[2]);
    } else {
      throw LuaError("wrong number of arguments to 'insert'");
    }
    return std::vector<Value>{};
  });
  reg(tab.get(), "remove", [](std::vector<Value>& a) {
    Table* t = tab_arg(a, 0, "remove");
    const size_t n = t->length();
    if (n == 0) return std::vector<Value>{Value()};
    const size_t pos = a.size() > 1 ? static_cast<size_t>(num_arg(a, 1, "remove")) : n;
    Value v = t->get(Value::number(static_cast<double>(pos)));
    for (size_t i = pos; i < n; ++i) t->set(Value::number(static_cast<double>(i)), t->get(Value::number(static_cast<double>(i + 1))));
    t->set(Value::number(static_cast<double>(n)), Value());
    return std::vector<Value>{v};
  });
  reg(tab.get(), "concat", [](std::vector<Value>& a) {
    Table* t = tab_arg(a, 0, "concat");
    const std::string sep = a.size() > 1 ? str_arg(a, 1, "concat") : "";
    std::string r;
    for (size_t i = 1; i <= t->length(); ++i) {
      if (i > 1) r += sep;
      r += tostring(t->get(Value::number(static_cast<double>(i))));
    }
    return std::vector<Value>{Value::string(r)};
  });
  reg(tab.get(), "getn", [](std::vector<Value>& a) {
    return std::vector<Value>{Value::number(static_cast<double>(tab_arg(a, 0, "getn")->length()))};
  });
  // table.sort: a merge sort (well defined even for an inconsistent comparator)
  reg(tab.get(), "sort", [this](std::vector<Value>& a) {
    Table* t = tab_arg(a, 0, "sort");
    const Value cmp = arg(a, 1);
    if (cmp.t != Value::NIL && cmp.t != Value::FUNC && cmp.t != Value::NATIVE)
      throw LuaError("bad argument #2 to 'sort' (function expected)");
    Exec x{*this, chunkname_};
    const size_t n = t->length();
    std::vector<Value> v(t->arr.begin(), t->arr.begin() + static_cast<std::ptrdiff_t>(n)), tmp(n);
    auto less = [&](const Value& p, const Value& q) {
      if (cmp.t == Value::NIL) return lua_lt(x, p, q, 0);
      return call1(x, cmp, {p, q}, 0).truthy();
    };
    for (size_t w = 1; w < n; w *= 2)
      for (size_t lo = 0; lo + w < n; lo += 2 * w) {
        const size_t mid = lo + w, hi = std::min(n, lo + 2 * w);
        size_t i = lo, j = mid, k = lo;
        while (i < mid && j < hi) tmp[k++] = less(v[j], v[i]) ? v[j++] : v[i++];
        while (i < mid) tmp[k++] = v[i++];
        while (j < hi) tmp[k++] = v[j++];
        std::copy(tmp.begin() + static_cast<std::ptrdiff_t>(lo), tmp.begin() + static_cast<std::ptrdiff_t>(hi),
                  v.begin() + static_cast<std::ptrdiff_t>(lo));
      }
    for (size_t i = 0; i < n; ++i) t->set(Value::number(static_cast<double>(i + 1)), v[i]);
    return std::vector<Value>{};
  });
  tab->set(Value::string("unpack"), G["unpack"]);
  G["table"] = Value::table(tab);

  // os: the clock / time / date subset (no process or file access)
  auto os = std::make_shared<Table>();
  reg(os.get(), "clock", [](std::vector<Value>&) {
    return std::vector<Value>{Value::number(static_cast<double>(std::clock()) / CLOCKS_PER_SEC)};
  });
  reg(os.get(), "time", [](std::vector<Value>&) {
    return std::vector<Value>{Value::number(static_cast<double>(std::time(nullptr)))};
  });
  reg(os.get(), "date", [](std::vector<Value>& a) {
    const std::string f = a.empty() || a[0].t == Value::NIL ? "%c" : str_arg(a, 0, "date");
    const std::time_t t = a.size() > 1 ? static_cast<std::time_t>(num_arg(a, 1, "date")) : std::time(nullptr);
    std::tm tm{};
    if (!f.empty() && f[0] == '!')
      gmtime_r(&t, &tm);
    else
      localtime_r(&t, &tm);
    char buf[256];
    const size_t n = std::strftime(buf, sizeof(buf), f.c_str() + (!f.empty() && f[0] == '!' ? 1 : 0), &tm);
    return std::vector<Value>{Value::string(std::string(buf, n))};
  });
  G["os"] = Value::table(os);
  G["_VERSION"] = Value::string("Lua 5.1 (nnsx)");
}

}  // namespace lua
}  // namespace nnsx
