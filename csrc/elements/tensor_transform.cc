// tensor_transform: dimchg / typecast / arithmetic / transpose / stand / clamp
// on every (or the `apply`-selected) tensor of a stream.
// Reference: gst/nnstreamer/elements/gsttensor_transform.c (option grammar
// :70-80,653-958; kernels :1121-1658; caps :1851-2186).
//
// Device-resident inputs (or `device>=0`) run the fused CDNA4 kernels of
// csrc/kernels/transform.hip on this element's stream; host inputs run the C
// reference loops below (also the numerics oracle of the kernels).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <regex>
#include <vector>

#include "core/cpu_ops.h"
#include "core/log.h"
#include "elements/elements.h"
#include "elements/tensor_common.h"
#include "kernels/kernels.h"
#include "runtime/base.h"
#include "runtime/fusion.h"
#include "runtime/pipeline.h"

namespace nnsx {

namespace cpu {

double read_as_double(const void* p, DType t, uint64_t i) {
  double r = 0;
#define NNSX_R(T) r = as_double<T>(static_cast<const T*>(p)[i])
  NNSX_CPU_DTYPE_CASES(t, NNSX_R)
#undef NNSX_R
  return r;
}

void write_from_double(void* p, DType t, uint64_t i, double v) {
#define NNSX_W(T) static_cast<T*>(p)[i] = Cast<T>::from(v)
  NNSX_CPU_DTYPE_CASES(t, NNSX_W)
#undef NNSX_W
}

}  // namespace cpu

namespace {

enum Mode { DIMCHG = 0, TYPECAST, ARITHMETIC, TRANSPOSE, STAND, CLAMP, MODE_UNKNOWN };

template <typename T>
struct is_int_t {
  static constexpr bool value = std::is_integral<T>::value;
};

template <typename T>
inline T cpu_apply(T v, const kernels::ArithOp& op) {
  using namespace cpu;
  if constexpr (std::is_integral<T>::value) {
    using W = typename std::conditional<std::is_unsigned<T>::value, uint64_t, int64_t>::type;
    if (op.kind == kernels::OP_CLAMP) {
      double d = static_cast<double>(v);
      d = d < op.fval ? op.fval : (d > op.fval2 ? op.fval2 : d);
      return static_cast<T>(d);
    }
    W a = static_cast<W>(v);
    W b = static_cast<W>(static_cast<T>(op.ival));
    switch (op.kind) {
      case kernels::OP_ADD: return static_cast<T>(a + b);
      case kernels::OP_MUL: return static_cast<T>(a * b);
      default: return b == 0 ? static_cast<T>(0) : static_cast<T>(a / b);
    }
  } else if constexpr (std::is_same<T, half_t>::value || std::is_same<T, bhalf_t>::value) {
    float a = static_cast<float>(as_double(v));
    float b = static_cast<float>(as_double(Cast<T>::from(op.fval)));
    float r;
    switch (op.kind) {
      case kernels::OP_ADD: r = a + b; break;
      case kernels::OP_MUL: r = a * b; break;
      case kernels::OP_DIV: r = a / b; break;
      default: r = a < op.fval ? static_cast<float>(op.fval) : (a > op.fval2 ? static_cast<float>(op.fval2) : a); break;
    }
    return Cast<T>::from(r);
  } else {
    T b = static_cast<T>(op.fval);
    switch (op.kind) {
      case kernels::OP_ADD: return v + b;
      case kernels::OP_MUL: return v * b;
      case kernels::OP_DIV: return v / b;
      default: {
        double d = static_cast<double>(v);
        d = d < op.fval ? op.fval : (d > op.fval2 ? op.fval2 : d);
        return static_cast<T>(d);
      }
    }
  }
}

// one element through the whole op chain (the definition every path below
// reproduces bit for bit)
template <typename InT, typename OutT>
inline OutT cpu_arith_one(InT x, int ch, const kernels::ArithParams& p) {
  OutT v = cpu::Cast<OutT>::from(x);
  for (int k = 0; k < p.nops; ++k)
    if (!p.ch_count || p.ops[k].ch < 0 || p.ops[k].ch == ch) v = cpu_apply<OutT>(v, p.ops[k]);
  return v;
}

// one op over a run of elements, the op kind resolved outside the loop (the
// loop vectorises; fp32 division stays a division)
template <typename T>
void cpu_apply_run(T* v, size_t n, const kernels::ArithOp& op) {
  if constexpr (std::is_same<T, float>::value || std::is_same<T, double>::value) {
    const T c = static_cast<T>(op.fval);
    switch (op.kind) {
      case kernels::OP_ADD: for (size_t i = 0; i < n; ++i) v[i] = v[i] + c; return;
      case kernels::OP_MUL: for (size_t i = 0; i < n; ++i) v[i] = v[i] * c; return;
      case kernels::OP_DIV: for (size_t i = 0; i < n; ++i) v[i] = v[i] / c; return;
      default: break;
    }
  }
  for (size_t i = 0; i < n; ++i) v[i] = cpu_apply<T>(v[i], op);
}

template <typename InT, typename OutT>
void cpu_arith_t(const void* in, void* out, uint64_t n, const kernels::ArithParams& p) {
  const InT* a = static_cast<const InT*>(in);
  OutT* b = static_cast<OutT*>(out);
  const int nch = p.ch_count > 0 ? p.ch_count : 1;
  if constexpr (sizeof(InT) == 1) {
    // 8-bit input (camera frames): every distinct (channel, value) through the
    // chain once, then a table lookup per element -- identical results
    if (p.nops > 0 && n >= static_cast<uint64_t>(1024) * nch) {
      std::vector<OutT> lut(static_cast<size_t>(256) * nch);
      for (int c = 0; c < nch; ++c)
        for (int x = 0; x < 256; ++x) {
          InT xv;
          const uint8_t byte = static_cast<uint8_t>(x);
          std::memcpy(&xv, &byte, 1);
          lut[static_cast<size_t>(c) * 256 + byte] = cpu_arith_one<InT, OutT>(xv, p.ch_count ? c : -1, p);
        }
      if (!p.ch_count) {
        const OutT* t = lut.data();
        for (uint64_t i = 0; i < n; ++i) {
          uint8_t byte;
          std::memcpy(&byte, &a[i], 1);
          b[i] = t[byte];
        }
      } else {
        for (uint64_t i = 0; i < n; ++i) {
          uint8_t byte;
          std::memcpy(&byte, &a[i], 1);
          b[i] = lut[static_cast<size_t>((i / p.ch_size) % p.ch_count) * 256 + byte];
        }
      }
      return;
    }
  }
  if (!p.ch_count) {
    // op at a time over cache-sized runs
    constexpr uint64_t kRun = 2048;
    for (uint64_t i0 = 0; i0 < n; i0 += kRun) {
      const size_t m = static_cast<size_t>(std::min<uint64_t>(kRun, n - i0));
      OutT* v = b + i0;
      for (size_t i = 0; i < m; ++i) v[i] = cpu::Cast<OutT>::from(a[i0 + i]);
      for (int k = 0; k < p.nops; ++k) cpu_apply_run<OutT>(v, m, p.ops[k]);
    }
    return;
  }
  for (uint64_t i = 0; i < n; ++i)
    b[i] = cpu_arith_one<InT, OutT>(a[i], static_cast<int>((i / p.ch_size) % p.ch_count), p);
}

template <typename InT>
void cpu_arith_in(DType out_t, const void* in, void* out, uint64_t n, const kernels::ArithParams& p) {
#define NNSX_O(T) cpu_arith_t<InT, T>(in, out, n, p)
  NNSX_CPU_DTYPE_CASES(out_t, NNSX_O)
#undef NNSX_O
}

void cpu_arith(const void* in, DType in_t, void* out, DType out_t, uint64_t n, const kernels::ArithParams& p) {
#define NNSX_I(T) cpu_arith_in<T>(out_t, in, out, n, p)
  NNSX_CPU_DTYPE_CASES(in_t, NNSX_I)
#undef NNSX_I
}

void cpu_permute(const void* in, void* out, size_t es, const Dims& in_dim, const int perm[8]) {
  uint64_t in_stride[8], acc = 1;
  for (int k = 0; k < 8; ++k) {
    in_stride[k] = acc;
    acc *= in_dim[k];
  }
  uint64_t out_dim[8], st[8];
  for (int k = 0; k < 8; ++k) {
    out_dim[k] = in_dim[perm[k]];
    st[k] = in_stride[perm[k]];
  }
  const char* src = static_cast<const char*>(in);
  char* dst = static_cast<char*>(out);
  uint64_t c[8] = {0};
  uint64_t off = 0;
  for (uint64_t o = 0; o < acc; ++o) {
    std::memcpy(dst + o * es, src + off * es, es);
    for (int k = 0; k < 8; ++k) {
      ++c[k];
      off += st[k];
      if (c[k] < out_dim[k]) break;
      off -= st[k] * c[k];
      c[k] = 0;
    }
  }
}

void cpu_stand(const void* in, DType in_t, void* out, DType out_t, uint64_t n, uint32_t C, int mode, bool per_ch) {
  uint32_t nch = per_ch ? C : 1;
  uint64_t cnt = per_ch ? n / C : n;
  std::vector<double> mean(nch, 0.0), stdv(nch, 1e-10);
  for (uint32_t ch = 0; ch < nch; ++ch) {
    double avg = 0;
    for (uint64_t i = 0; i < cnt; ++i) {
      double x = cpu::read_as_double(in, in_t, per_ch ? i * C + ch : i);
      avg = (x - avg) / static_cast<double>(i + 1) + avg;  // running mean, as the reference
    }
    mean[ch] = avg;
    if (mode == 0) {
      double sd = 0;
      for (uint64_t i = 0; i < cnt; ++i) {
        double x = cpu::read_as_double(in, in_t, per_ch ? i * C + ch : i);
        sd += std::pow(x - avg, 2) / static_cast<double>(cnt);
      }
      stdv[ch] = sd != 0.0 ? std::sqrt(sd) : 1e-10;
    }
  }
  for (uint64_t i = 0; i < n; ++i) {
    uint32_t ch = per_ch ? static_cast<uint32_t>(i % C) : 0;
    double x = cpu::read_as_double(in, in_t, i);
    double r = mode == 0 ? std::fabs((x - mean[ch]) / stdv[ch]) : x - mean[ch];
    cpu::write_from_double(out, out_t, i, r);
  }
}

class TensorTransform : public BaseTransform, public AbsorbableElement {
 public:
  explicit TensorTransform(const std::string& name)
      : BaseTransform("tensor_transform", name,
                      Caps::from_string(tensor_caps_template_static() + "; " + tensor_caps_template_flexible()),
                      Caps::from_string(tensor_caps_template_static() + "; " + tensor_caps_template_flexible())) {
    prop_enum("mode", &mode_, {"dimchg", "typecast", "arithmetic", "transpose", "stand", "clamp"},
              "Mode used for transforming tensor", [this] { parse_option(); });
    prop_string("option", &option_, "Option for the tensor transform mode ?", [this] { parse_option(); });
    prop_bool("acceleration", &accel_, "Orc acceleration in the reference; here: allow the GPU path when data is device-resident");
    prop_string("apply", &apply_str_, "Select tensors to apply, separated with ',' in case of multiple tensors. Default to apply all tensors.",
                [this] {
                  apply_.clear();
                  for (auto& s : split(apply_str_, ','))
                    if (!strip(s).empty()) apply_.push_back(static_cast<int>(to_int(s)));
                });
    prop_uint("transpose-rank-limit", &transpose_rank_limit_, "The rank limit of transpose, which varies per version of nnstreamer and may be lower than the global rank limit if it is over 4.");
    prop_int("device", &device_, "nnsx: -2 follow input placement, -1 CPU, N run on GPU N");
    prop_bool("absorbable", &absorbable_,
              "nnsx: let a downstream tensor_filter whose model takes uint8 frames fold this elementwise arithmetic "
              "into the model (the transform then passes the frames through)");
    prop_readonly("absorbed-by", [this] { return absorbed_ ? absorbed_by_ : std::string(); },
                  "nnsx: the element that absorbed this transform at caps negotiation (empty: runs its own kernel)");
    mode_ = MODE_UNKNOWN;
  }

  // ---- AbsorbableElement (runtime/fusion.h) ----
  void set_absorber(TransformAbsorber* a) override {
    std::lock_guard<std::mutex> lk(absorb_mu_);
    absorber_ = a;
    if (!a) {
      absorbed_ = false;
      absorbed_by_.clear();
    }
  }
  bool absorbed() const override { return absorbed_; }

 protected:
  bool applies(unsigned i) const {
    if (apply_.empty()) return true;
    for (int a : apply_)
      if (static_cast<unsigned>(a) == i) return true;
    return false;
  }

  void parse_option() {
    loaded_ = false;
    if (mode_ == MODE_UNKNOWN || option_.empty()) return;
    std::string opt = strip(option_);
    switch (mode_) {
      case DIMCHG: {
        static const std::regex re("^([0-7]):([0-7])$", std::regex::icase);
        std::smatch m;
        if (!std::regex_match(opt, m, re)) throw Error("dimchg: '" + opt + "' is not valid option string");
        from_ = std::stoi(m[1]);
        to_ = std::stoi(m[2]);
        break;
      }
      case TYPECAST: {
        static const std::regex re("(^[u]?int(8|16|32|64)$|^float(16|32|64)$|^bfloat16$)", std::regex::icase);
        if (!std::regex_match(opt, re)) throw Error("typecast: '" + opt + "' is not valid data type");
        cast_to_ = dtype_from_string(opt);
        break;
      }
      case ARITHMETIC: {
        params_ = kernels::ArithParams();
        arith_out_ = DType::END;
        per_channel_ = false;
        ch_dim_ = 0;
        auto ops = split(opt, ',');
        bool first = true;
        for (auto& raw : ops) {
          std::string o = strip(raw);
          if (o.empty()) continue;
          auto kv = split(o, ':');
          std::string op = lower(strip(kv[0]));
          if (op == "typecast") {
            if (!first) {
              NNSX_LOGE(name(), "arithmetic: [typecast:TYPE,] should be located at the first; ignored: ", o);
              continue;
            }
            if (kv.size() < 2) throw Error("arithmetic: invalid typecast");
            arith_out_ = dtype_from_string(kv[1]);
            if (arith_out_ == DType::END) throw Error("arithmetic: invalid type " + kv[1]);
            first = false;
            continue;
          }
          first = false;
          if (op == "per-channel") {
            if (kv.size() > 1) {
              auto v = split(kv[1], '@');
              if (lower(strip(v[0])) == "true" && v.size() > 1) {
                per_channel_ = true;
                ch_dim_ = static_cast<unsigned>(to_uint(v[1]));
              }
            }
            continue;
          }
          int kind;
          if (op == "add") kind = kernels::OP_ADD;
          else if (op == "mul") kind = kernels::OP_MUL;
          else if (op == "div") kind = kernels::OP_DIV;
          else throw Error("arithmetic: unknown operator '" + op + "' in '" + opt + "'");
          if (kv.size() < 2) throw Error("arithmetic: missing operand in '" + o + "'");
          auto v = split(kv[1], '@');
          std::string num = strip(v[0]);
          if (params_.nops >= kernels::kMaxArithOps) throw Error("arithmetic: too many operators");
          kernels::ArithOp a{};
          a.kind = kind;
          if (num.find_first_of(".eE") != std::string::npos) {
            a.fval = to_double(num);
            a.ival = static_cast<int64_t>(a.fval);
          } else {
            a.ival = to_int(num);
            a.fval = static_cast<double>(a.ival);
          }
          a.ch = (per_channel_ && v.size() > 1) ? static_cast<int>(to_int(v[1])) : -1;
          params_.ops[params_.nops++] = a;
        }
        if (params_.nops == 0 && arith_out_ == DType::END) throw Error("arithmetic: no operator in '" + opt + "'");
        break;
      }
      case TRANSPOSE: {
        auto parts = split(opt, ':');
        if (parts.size() != 4) throw Error("transpose: '" + opt + "' is not valid option string");
        bool used[3] = {false, false, false};
        for (int i = 0; i < 4; ++i) {
          int v = static_cast<int>(to_int(parts[i], -1));
          if (i < 3 && (v < 0 || v > 2 || used[v])) throw Error("transpose: invalid order " + opt);
          if (i == 3 && v != 3) throw Error("transpose: the last dim must be fixed to 3");
          if (i < 3) used[v] = true;
          order_[i] = v;
        }
        break;
      }
      case STAND: {
        static const std::regex re(
            "^(default|dc-average)(:([u]?int(8|16|32|64)|float(16|32|64)|bfloat16))?(,per-channel:(true|false))?$",
            std::regex::icase);
        if (!std::regex_match(opt, re)) throw Error("stand: '" + opt + "' is not a valid option string");
        stand_out_ = DType::END;
        stand_per_ch_ = false;
        for (auto& o : split(opt, ',')) {
          auto kv = split(o, ':');
          std::string k = lower(strip(kv[0]));
          if (k == "default" || k == "dc-average") {
            stand_mode_ = k == "default" ? 0 : 1;
            if (kv.size() > 1) stand_out_ = dtype_from_string(kv[1]);
          } else if (k == "per-channel") {
            stand_per_ch_ = kv.size() > 1 && lower(strip(kv[1])) == "true";
          }
        }
        break;
      }
      case CLAMP: {
        auto parts = split(opt, ':');
        if (parts.size() != 2) throw Error("clamp: '" + opt + "' is not valid option string");
        clamp_min_ = to_double(parts[0]);
        clamp_max_ = to_double(parts[1]);
        if (clamp_min_ > clamp_max_) throw Error("clamp: CLAMP_MIN is larger than CLAMP_MAX");
        break;
      }
      default:
        return;
    }
    loaded_ = true;
  }

  // output tensor info for one input tensor
  bool convert_info(const TensorInfo& in, TensorInfo* out) const {
    *out = in;
    switch (mode_) {
      case DIMCHG: {
        if (from_ == to_) return true;
        if (from_ > to_) {
          NNSX_LOGE(name(), "tensor-transform/dimchg operation is not permitted if from >= to.");
          return false;
        }
        Dims d = in.dim;
        uint32_t moving = d[from_];
        for (int i = from_; i < to_; ++i) d[i] = d[i + 1];
        d[to_] = moving;
        out->dim = d;
        return true;
      }
      case TYPECAST: out->type = cast_to_; return true;
      case ARITHMETIC: if (arith_out_ != DType::END) out->type = arith_out_; return true;
      case TRANSPOSE:
        for (int i = 0; i < 4; ++i) out->dim[i] = in.dim[order_[i]];
        return true;
      case STAND: if (stand_out_ != DType::END) out->type = stand_out_; return true;
      case CLAMP: return true;
      default: return false;
    }
  }

  // An elementwise uint8 -> float32 arithmetic / typecast on a single static
  // tensor, offered to the downstream absorber once per negotiation.
  bool try_absorb(const TensorsConfig& in) {
    std::lock_guard<std::mutex> lk(absorb_mu_);
    if (!absorber_ || !absorbable_ || !loaded_) return false;
    if (mode_ != ARITHMETIC && mode_ != TYPECAST) return false;
    if (!in.is_static() || in.info.num_tensors != 1 || !applies(0)) return false;
    const TensorInfo& ti = in.info.at(0);
    if (ti.type != DType::UINT8) return false;
    if (mode_ == ARITHMETIC && per_channel_) return false;
    const DType out = mode_ == TYPECAST ? cast_to_ : (arith_out_ == DType::END ? ti.type : arith_out_);
    if (out != DType::FLOAT32) return false;
    if (absorbed_) return true;
    ArithPrefix p;
    p.tensor = 0;
    p.in_type = ti.type;
    p.out_type = out;
    p.params = effective_params(ti);
    if (!absorber_->absorb_arith(p, name())) return false;
    absorbed_ = true;
    Element* e = dynamic_cast<Element*>(absorber_);
    absorbed_by_ = e ? e->name() : std::string("?");
    NNSX_LOGI(name(), "arithmetic absorbed by ", absorbed_by_, ": uint8 frames pass through");
    return true;
  }

  Caps transform_caps(PadDirection dir, const Caps& caps, const Caps* filter) override {
    Caps r;
    for (size_t i = 0; i < caps.size(); ++i) {
      const Structure& st = caps.at(i);
      TensorsConfig in;
      if (!config_from_structure(st, &in) || !loaded_) {
        r.append(st);
        continue;
      }
      if (dir == PadDirection::SINK && try_absorb(in)) {  // pass-through caps
        r.append(st);
        continue;
      }
      if (in.is_flexible()) {
        r.append(st);
        continue;
      }
      if (dir == PadDirection::SRC) {
        // reverse direction: we cannot invert every mode exactly; offer the template
        r.append(Caps::from_string(tensor_caps_template_static()));
        continue;
      }
      TensorsConfig out = in;
      bool ok = in.info.num_tensors > 0;
      for (unsigned t = 0; t < in.info.num_tensors && ok; ++t) {
        if (!applies(t)) continue;
        const TensorInfo& ti = in.info.at(t);
        if (!dimension_valid(ti.dim) && mode_ != TYPECAST && mode_ != ARITHMETIC && mode_ != STAND && mode_ != CLAMP) {
          ok = false;
          break;
        }
        ok = convert_info(ti, &out.info.at(t));
      }
      if (!ok) {
        r.append(Caps::from_string(tensor_caps_template_static()));
        continue;
      }
      Caps c = caps_from_config(out);
      if (st.name() == kMimeTensor && out.info.num_tensors == 1) {
        Structure s(kMimeTensor);
        s.set("dimension", Value::String(rank_dimension_string(out.info.at(0).dim, std::max(4, out.info.at(0).rank()))));
        s.set("type", Value::String(dtype_name(out.info.at(0).type)));
        if (const Value* fr = st.get("framerate")) s.set("framerate", *fr);
        r.append(s);
      }
      r.append(c);
    }
    if (filter) r = r.intersect(*filter);
    return r;
  }

  Caps fixate_caps(PadDirection, const Caps& caps, Caps othercaps) override {
    TensorsConfig in;
    if (caps.size() && config_from_structure(caps.at(0), &in) && !in.is_flexible() && loaded_) {
      if (absorbed_) {  // pass-through: the output is the input
        Caps peer = src_pad()->peer_query_caps(nullptr);
        return pad_caps_from_config(in, &peer);
      }
      TensorsConfig out = in;
      for (unsigned t = 0; t < in.info.num_tensors; ++t)
        if (applies(t)) convert_info(in.info.at(t), &out.info.at(t));
      Caps peer = src_pad()->peer_query_caps(nullptr);
      return pad_caps_from_config(out, &peer);
    }
    return othercaps.fixate();
  }

  bool set_caps(const Caps& incaps, const Caps& outcaps) override {
    if (!loaded_) {
      NNSX_LOGE(name(), "tensor_transform: mode/option are not configured");
      return false;
    }
    if (!tensor_config_from_caps(incaps, &in_config_) || !tensor_config_from_caps(outcaps, &out_config_)) return false;
    in_flexible_ = in_config_.is_flexible();
    out_flexible_ = out_config_.is_flexible();
    if (absorbed_) return true;  // pass-through
    if (!in_flexible_) {
      // validate the output config against the conversion
      for (unsigned t = 0; t < in_config_.info.num_tensors; ++t) {
        TensorInfo o;
        if (!applies(t)) continue;
        if (!convert_info(in_config_.info.at(t), &o)) return false;
      }
    }
    return true;
  }

  FlowReturn transform(const BufferPtr& inbuf, BufferPtr* outbuf) override {
    if (!loaded_) return FlowReturn::ERROR;
    if (absorbed_) {  // the downstream filter applies this arithmetic inside its model
      *outbuf = inbuf;
      return FlowReturn::OK;
    }
    BufferPtr in;
    if (!buffer_from_config(inbuf, in_config_, &in)) {
      post_error("tensor_transform: input buffer does not match the negotiated caps");
      return FlowReturn::ERROR;
    }
    int dev = accel_ ? resolve_device(device_, *in) : -1;
    hipStream_t s = dev >= 0 ? streams_.get(dev) : nullptr;
    auto out = make_buffer();
    out->copy_metadata_from(*in);
    for (size_t t = 0; t < in->n_memory(); ++t) {
      MemoryPtr m = in->mems[t];
      TensorInfo ti;
      MemoryPtr payload = m;
      if (in_flexible_) {
        MetaInfo meta;
        if (!parse_flexible(m, &meta, &payload) || !meta.to_info(&ti)) {
          post_error("tensor_transform: invalid flexible header");
          return FlowReturn::ERROR;
        }
      } else {
        ti = in_config_.info.at(static_cast<unsigned>(t));
      }
      if (!applies(static_cast<unsigned>(t))) {
        out->mems.push_back(m);
        continue;
      }
      TensorInfo to;
      if (!convert_info(ti, &to)) return FlowReturn::ERROR;
      MemoryPtr res = dev >= 0 ? run_gpu(payload, ti, to, dev, s) : run_cpu(payload, ti, to);
      if (!res) return FlowReturn::ERROR;
      if (out_flexible_) res = make_flexible(res, MetaInfo::from_info(to));
      out->mems.push_back(res);
    }
    *outbuf = out;
    return FlowReturn::OK;
  }

  kernels::ArithParams effective_params(const TensorInfo& in) const {
    kernels::ArithParams p = params_;
    if (mode_ == CLAMP) {
      p = kernels::ArithParams();
      p.nops = 1;
      p.ops[0] = kernels::ArithOp{kernels::OP_CLAMP, clamp_min_, 0, clamp_max_, -1};
    }
    if (mode_ == TYPECAST) p = kernels::ArithParams();
    if (mode_ == ARITHMETIC && per_channel_) {
      uint64_t chs = 1;
      for (unsigned i = 0; i < ch_dim_ && i < 8; ++i) chs *= in.dim[i];
      p.ch_size = chs;
      p.ch_count = ch_dim_ < 8 ? in.dim[ch_dim_] : 1;
    }
    return p;
  }

  MemoryPtr run_cpu(const MemoryPtr& m, const TensorInfo& ti, const TensorInfo& to) {
    const void* src = m->map_host();
    uint64_t n = element_count(ti.dim);
    auto outm = Memory::alloc_host(to.size());
    switch (mode_) {
      case TYPECAST:
      case ARITHMETIC:
      case CLAMP:
        cpu_arith(src, ti.type, outm->data(), to.type, n, effective_params(ti));
        break;
      case DIMCHG:
      case TRANSPOSE: {
        int perm[8];
        perm_for(ti, perm);
        cpu_permute(src, outm->data(), dtype_size(ti.type), ti.dim, perm);
        break;
      }
      case STAND:
        cpu_stand(src, ti.type, outm->data(), to.type, n, ti.dim[0], stand_mode_, stand_per_ch_);
        break;
      default:
        return nullptr;
    }
    return outm;
  }

  void perm_for(const TensorInfo& ti, int perm[8]) const {
    (void)ti;
    for (int i = 0; i < 8; ++i) perm[i] = i;
    if (mode_ == TRANSPOSE) {
      for (int i = 0; i < 4; ++i) perm[i] = order_[i];
    } else if (mode_ == DIMCHG && from_ < to_) {
      // out dims: d[from] moves to `to`, the ones in between shift down
      for (int i = from_; i < to_; ++i) perm[i] = i + 1;
      perm[to_] = from_;
    }
  }

  MemoryPtr run_gpu(const MemoryPtr& m, const TensorInfo& ti, const TensorInfo& to, int dev, hipStream_t s) {
    hip::DeviceGuard g(dev);
    const void* src = m->map_device(dev, s);
    uint64_t n = element_count(ti.dim);
    auto outm = Memory::alloc_device(to.size(), dev, s);
    switch (mode_) {
      case TYPECAST:
      case ARITHMETIC:
      case CLAMP:
        kernels::arith(src, ti.type, outm->data(), to.type, n, effective_params(ti), s);
        break;
      case DIMCHG:
      case TRANSPOSE: {
        int perm[8];
        perm_for(ti, perm);
        if (mode_ == DIMCHG && from_ == to_) {
          hip::check(hipMemcpyAsync(outm->data(), src, to.size(), hipMemcpyDeviceToDevice, s), "D2D");
        } else {
          kernels::permute(src, outm->data(), dtype_size(ti.type), ti.dim.data(), perm, s);
        }
        break;
      }
      case STAND: {
        size_t wsz = kernels::stand_workspace_bytes(ti.dim[0]);
        auto ws = Memory::alloc_device(wsz, dev, s);
        kernels::stand(src, ti.type, outm->data(), to.type, n, ti.dim[0], stand_mode_, stand_per_ch_, ws->data(), s);
        break;
      }
      default:
        return nullptr;
    }
    hip::check(hipGetLastError(), "tensor_transform kernel launch");
    m->record_use(s, dev);
    outm->mark_ready(s);
    return outm;
  }

  int mode_;
  std::string option_;
  bool accel_ = true;
  std::string apply_str_;
  std::vector<int> apply_;
  unsigned transpose_rank_limit_ = 4;
  int device_ = -2;
  bool loaded_ = false;
  int from_ = 0, to_ = 0;
  DType cast_to_ = DType::END;
  kernels::ArithParams params_;
  DType arith_out_ = DType::END;
  bool per_channel_ = false;
  unsigned ch_dim_ = 0;
  int order_[4] = {0, 1, 2, 3};
  int stand_mode_ = 0;
  DType stand_out_ = DType::END;
  bool stand_per_ch_ = false;
  double clamp_min_ = 0, clamp_max_ = 0;
  TensorsConfig in_config_, out_config_;
  bool in_flexible_ = false, out_flexible_ = false;
  StreamSet streams_;
  std::mutex absorb_mu_;
  TransformAbsorber* absorber_ = nullptr;
  bool absorbable_ = true;
  std::atomic<bool> absorbed_{false};
  std::string absorbed_by_;
};

}  // namespace

bool arith_table_u8(const kernels::ArithParams& p, DType out, std::vector<float>* lut) {
  if (out != DType::FLOAT32) return false;
  uint8_t in[256];
  for (int i = 0; i < 256; ++i) in[i] = static_cast<uint8_t>(i);
  lut->assign(256, 0.f);
  cpu_arith(in, DType::UINT8, lut->data(), DType::FLOAT32, 256, p);
  return true;
}

void register_tensor_transform() {
  register_element("tensor_transform", "Filter/Tensor", "Transforms other/tensor dimensions for different models or frameworks",
                   [](const std::string& n) { return std::make_unique<TensorTransform>(n); });
}

}  // namespace nnsx
