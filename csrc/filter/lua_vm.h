// A small Lua 5.1 interpreter for tensor_filter framework=lua -- the image
// ships no Lua library, so the language is implemented here (reference
// ext/nnstreamer/tensor_filter/tensor_filter_lua.cc embeds liblua 5.1).
//
// Covered: numbers (doubles, as Lua 5.1), strings, booleans, nil, tables
// (array + hash parts), first-class functions and closures, varargs, multiple
// assignment / returns, local / global variables, if / while / repeat /
// numeric and generic for / break / return, method calls, long strings and
// comments, and the base / math / string / table library functions that
// tensor scripts use, metatables (__index, __newindex, __call, arithmetic,
// comparison, __concat, __unm, __tostring, __metatable) and Lua patterns
// (string.find / match / gmatch / gsub).  Not covered: coroutines, goto, the
// io / debug libraries and most of os (a script using them fails to load or
// run with a LuaError naming the construct).
//
// Host objects (the input / output tensors) are Userdata with virtual
// index / newindex / length.
#pragma once

#include <cstdint>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace nnsx {
namespace lua {

struct LuaError : std::runtime_error {
  explicit LuaError(const std::string& m) : std::runtime_error(m) {}
};

struct Obj {
  virtual ~Obj() = default;
};

struct Value;
struct Table;
struct Closure;
struct Native;
struct Userdata;

struct Value {
  enum Type : uint8_t { NIL = 0, BOOL, NUM, STR, TABLE, FUNC, NATIVE, USERDATA };
  Type t = NIL;
  bool b = false;
  double n = 0;
  std::shared_ptr<Obj> o;

  Value() = default;
  static Value boolean(bool v) {
    Value r;
    r.t = BOOL;
    r.b = v;
    return r;
  }
  static Value number(double v) {
    Value r;
    r.t = NUM;
    r.n = v;
    return r;
  }
  static Value string(std::string s);
  static Value table(std::shared_ptr<Table> t);
  static Value native(std::string name, std::function<std::vector<Value>(std::vector<Value>&)> fn);
  static Value userdata(std::shared_ptr<Userdata> u);

  bool truthy() const { return !(t == NIL || (t == BOOL && !b)); }
  const std::string& str() const;
  Table* tab() const;
  Userdata* ud() const;
  std::string type_name() const;
};

struct StrObj : Obj {
  std::string s;
  size_t hash = 0;
};

struct ValueHash {
  size_t operator()(const Value& v) const;
};
struct ValueEq {
  bool operator()(const Value& a, const Value& b) const;
};

struct Table : Obj {
  std::vector<Value> arr;  // keys 1..arr.size()
  std::unordered_map<Value, Value, ValueHash, ValueEq> hash;
  std::shared_ptr<Table> meta;  // setmetatable()
  Value get(const Value& k) const;
  void set(const Value& k, Value v);
  size_t length() const;  // the border of the array part (Lua's # on sequences)
};

struct Native : Obj {
  std::string name;
  std::function<std::vector<Value>(std::vector<Value>&)> fn;
};

// host object: tensors (1-based element index, number values)
struct Userdata : Obj {
  virtual Value index(const Value& key) = 0;
  virtual void newindex(const Value& key, const Value& v) = 0;
  virtual size_t length() const { return 0; }
  virtual std::string type_name() const { return "userdata"; }
};

struct FuncProto;
struct Chunk;

class VM {
 public:
  VM();
  ~VM();
  // compile and run a chunk (script text); throws LuaError
  void run(const std::string& source, const std::string& chunkname);
  Value global(const std::string& name) const;
  void set_global(const std::string& name, Value v);
  // call a function value; throws LuaError
  std::vector<Value> call(const Value& fn, std::vector<Value> args);
  // a cap on executed statements per run/call (0 = none): a runaway script
  // (while true do end) ends with a LuaError instead of hanging the pipeline
  void set_step_limit(uint64_t steps) { step_limit_ = steps; }

  // (interpreter internals)
  std::unordered_map<std::string, Value> globals_;
  uint64_t steps_ = 0, step_limit_ = 0;
  int depth_ = 0;  // nested Lua calls (capped: "stack overflow")
  std::vector<std::unique_ptr<Chunk>> chunks_;
  std::string chunkname_;

 private:
  void open_libs();
};

std::string tostring(const Value& v);
std::string fmt_number(double d);  // Lua 5.1 number formatting (%.14g, integers without a point)
bool tonumber(const Value& v, double* out);

}  // namespace lua
}  // namespace nnsx
