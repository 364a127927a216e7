// Caps: the stream-format negotiation language (GstCaps/GstStructure/GValue
// subset).  Parses and prints the gst-launch caps syntax, intersects and
// fixates.  Tensor-aware rules (dimension-string spelling, flexible wins)
// follow gst/nnstreamer/nnstreamer_plugin_api_impl.c:713-1405.
//
// nnsx extension: a caps structure may carry the feature "memory:HIP"
// (device-resident payload), written `other/tensors(memory:HIP),...`.
#pragma once

#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "core/types.h"

namespace nnsx {

struct Value {
  enum class Kind { NONE, INT, DOUBLE, BOOL, STRING, FRACTION, INT_RANGE, FRACTION_RANGE, DOUBLE_RANGE, LIST };
  Kind kind = Kind::NONE;
  int64_t i = 0, i2 = 0;        // INT / INT_RANGE(i..i2) / FRACTION(i/i2)
  int64_t f1n = 0, f1d = 1, f2n = 0, f2d = 1;  // FRACTION_RANGE
  double d = 0, d2 = 0;
  bool b = false;
  std::string s;
  std::vector<Value> list;

  static Value Int(int64_t v) { Value x; x.kind = Kind::INT; x.i = v; return x; }
  static Value Double(double v) { Value x; x.kind = Kind::DOUBLE; x.d = v; return x; }
  static Value Bool(bool v) { Value x; x.kind = Kind::BOOL; x.b = v; return x; }
  static Value String(std::string v) { Value x; x.kind = Kind::STRING; x.s = std::move(v); return x; }
  static Value Fraction(int64_t n, int64_t dd) { Value x; x.kind = Kind::FRACTION; x.i = n; x.i2 = dd; return x; }
  static Value IntRange(int64_t a, int64_t b) { Value x; x.kind = Kind::INT_RANGE; x.i = a; x.i2 = b; return x; }
  static Value DoubleRange(double a, double b) { Value x; x.kind = Kind::DOUBLE_RANGE; x.d = a; x.d2 = b; return x; }
  static Value FractionRange(int64_t an, int64_t ad, int64_t bn, int64_t bd) {
    Value x; x.kind = Kind::FRACTION_RANGE; x.f1n = an; x.f1d = ad; x.f2n = bn; x.f2d = bd; return x;
  }
  static Value List(std::vector<Value> v) { Value x; x.kind = Kind::LIST; x.list = std::move(v); return x; }

  bool is_fixed() const;
  std::string to_string(bool with_type = false) const;
  bool operator==(const Value& o) const;
  // Intersection; returns false if empty.  `field` enables tensor-aware string compare.
  static bool intersect(const Value& a, const Value& b, Value* out, const std::string& field = "");
  Value fixate() const;
};

class Structure {
 public:
  Structure() = default;
  explicit Structure(std::string name) : name_(std::move(name)) {}

  const std::string& name() const { return name_; }
  void set_name(const std::string& n) { name_ = n; }
  const std::vector<std::string>& features() const { return features_; }
  void set_features(std::vector<std::string> f) { features_ = std::move(f); }
  bool has_feature(const std::string& f) const;

  bool has(const std::string& field) const;
  const Value* get(const std::string& field) const;
  void set(const std::string& field, Value v);
  void remove(const std::string& field);
  const std::vector<std::pair<std::string, Value>>& fields() const { return fields_; }

  // typed getters (false if absent or not fixed of that type)
  bool get_int(const std::string& f, int64_t* v) const;
  bool get_string(const std::string& f, std::string* v) const;
  bool get_fraction(const std::string& f, int* n, int* d) const;
  bool get_bool(const std::string& f, bool* v) const;
  bool get_double(const std::string& f, double* v) const;
  std::string get_string_or(const std::string& f, const std::string& def) const;
  int64_t get_int_or(const std::string& f, int64_t def) const;

  bool is_fixed() const;
  std::string to_string(bool with_types = true) const;
  static bool intersect(const Structure& a, const Structure& b, Structure* out);
  void fixate();
  // Fixation helpers used by sources (gst_structure_fixate_field_nearest_*).
  void fixate_nearest_int(const std::string& f, int64_t target);
  void fixate_nearest_fraction(const std::string& f, int n, int d);
  void fixate_string(const std::string& f, const std::string& target);

 private:
  std::string name_;
  std::vector<std::string> features_;
  std::vector<std::pair<std::string, Value>> fields_;
};

class Caps {
 public:
  Caps() = default;  // EMPTY
  static Caps Any() { Caps c; c.any_ = true; return c; }
  static Caps Empty() { return Caps(); }
  static Caps from_string(const std::string& s);  // throws Error on syntax error
  static bool try_parse(const std::string& s, Caps* out, std::string* err = nullptr);

  bool is_any() const { return any_; }
  bool is_empty() const { return !any_ && structs_.empty(); }
  bool is_fixed() const;
  size_t size() const { return structs_.size(); }
  Structure& at(size_t i) { return structs_[i]; }
  const Structure& at(size_t i) const { return structs_[i]; }
  void append(Structure s) { structs_.push_back(std::move(s)); }
  void append(const Caps& c);

  Caps intersect(const Caps& other) const;
  bool can_intersect(const Caps& other) const { return !intersect(other).is_empty(); }
  Caps fixate() const;  // first structure, every field fixated
  std::string to_string() const;
  bool operator==(const Caps& o) const { return to_string() == o.to_string(); }

 private:
  bool any_ = false;
  std::vector<Structure> structs_;
};

// ----- tensor caps helpers (nnstreamer_plugin_api_impl.c) -----
constexpr const char* kMimeTensor = "other/tensor";
constexpr const char* kMimeTensors = "other/tensors";
constexpr const char* kFeatureHIP = "memory:HIP";

bool structure_is_tensor_stream(const Structure& s);
MediaType structure_media_type(const Structure& s);
// Parse an other/tensor(s) structure into config.  Returns false if not a tensor stream.
bool config_from_structure(const Structure& s, TensorsConfig* config);
// Caps describing config; `flexible` forces format=flexible, legacy emits other/tensor.
Caps caps_from_config(const TensorsConfig& config, bool device = false);
// Pad caps from config given peer caps (flexible wins if either side is flexible).
Caps pad_caps_from_config(const TensorsConfig& config, const Caps* peer, bool device = false);
// Template caps strings
std::string tensor_caps_template_static();
std::string tensor_caps_template_flexible();
std::string tensor_caps_template_all();

}  // namespace nnsx
