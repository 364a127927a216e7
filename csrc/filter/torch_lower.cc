// Load-time lowering of a plain TorchScript model onto the CDNA4 engine.
//
// The reference filter runs whatever torch::jit::load returns, op by op on the
// framework's own kernels (tensor_filter_pytorch.cc:205-230, invoke :517-557).
// nnsx does the same for any model, and in addition rewrites the frozen
// forward graph once, at load, so that the layers its hand-written MI355X
// kernels cover run on them -- a user's own TorchScript MobileNet-style model
// gets the engine without nnsx's model builders:
//
//   conv 1x1 (+ ReLU6/ReLU)                  -> nnsx::pw_conv            (x3 GEMM)
//   depthwise 3x3 (stride 1/2, dilation d)   -> nnsx::dw_conv
//   1x1 + ReLU6 -> dw 3x3 + ReLU6 -> 1x1 [+ x] (the inverted residual, with or
//     without the expand)                    -> nnsx::ir_block_any       (one fused kernel)
//   3x3/2 stem conv on 3 channels (+ a t = 1 first block)
//                                            -> nnsx::stem_any / stem_ir1_any
//   1x1 + act -> mean over H, W              -> nnsx::pw_conv_pool
//   mean over H, W / adaptive_avg_pool2d(1)  -> nnsx::avgpool
//   linear                                   -> nnsx::pw_conv (2-D)
//   add / ReLU6 / ReLU / dropout(eval) / flatten on lowered values: NHWC forms
//
// Activations are NHWC between lowered ops (the NNStreamer video tensor is
// NHWC already: an entry `x.permute(0, 3, 1, 2)` is dropped, an NCHW input is
// permuted once); any node left on ATen reads an NCHW view of a lowered value,
// so unmatched layers keep running unchanged.  Weights are re-laid-out, padded
// and split into their bf16 parts (kernels/x3.h) here, once, as graph
// constants on the model's device.  A model whose first layer is the stem gets
// an `in_lut` table, so tensor_filter can absorb an upstream tensor_transform
// and feed uint8 frames (runtime/fusion.h), exactly as for nnsx's own models.
// tensor_filter verifies the lowered module against the original at load (a
// 2-frame random input) and keeps the original when they disagree
// (filter/pytorch.cc).
#include "filter/torch_lower.h"

#include <torch/csrc/jit/ir/ir.h>
#include <torch/csrc/jit/passes/dead_code_elimination.h>
#include <torch/csrc/jit/passes/freeze_module.h>

#include <algorithm>
#include <unordered_map>
#include <unordered_set>

#include "core/util.h"

namespace nnsx {

using torch::jit::Graph;
using torch::jit::NamedValue;
using torch::jit::Node;
using torch::jit::Value;
using torch::jit::WithInsertPoint;

std::string LowerReport::summary() const {
  return strfmt(lowered, "/", convs, " convs", linears ? strfmt(" + ", linears, " linear") : std::string(),
                " on nnsx kernels, ", ir_blocks, " fused inverted residuals",
                stem_block ? ", stem + block 1 fused" : "", head_pool ? ", head + pool fused" : "",
                lut ? ", uint8 input table" : "");
}

namespace {

c10::Symbol nnsx_op(const char* name) { return c10::Symbol::fromQualString(std::string("nnsx::") + name); }

bool const_tensor(Value* v, at::Tensor* t) {
  auto iv = torch::jit::toIValue(v);
  if (!iv || !iv->isTensor()) return false;
  *t = iv->toTensor();
  return true;
}
bool const_none(Value* v) {
  auto iv = torch::jit::toIValue(v);
  return iv && iv->isNone();
}
bool const_ints(Value* v, std::vector<int64_t>* out) {
  auto iv = torch::jit::toIValue(v);
  if (!iv || !iv->isIntList()) return false;
  *out = iv->toIntVector();
  return true;
}
bool const_int(Value* v, int64_t* out) {
  auto iv = torch::jit::toIValue(v);
  if (!iv || !iv->isInt()) return false;
  *out = iv->toInt();
  return true;
}
bool const_double(Value* v, double* out) {
  auto iv = torch::jit::toIValue(v);
  if (!iv) return false;
  if (iv->isDouble()) *out = iv->toDouble();
  else if (iv->isInt()) *out = static_cast<double>(iv->toInt());
  else return false;
  return true;
}
bool const_bool(Value* v, bool* out) {
  auto iv = torch::jit::toIValue(v);
  if (!iv || !iv->isBool()) return false;
  *out = iv->toBool();
  return true;
}

Node* single_user(Value* v) { return v->uses().size() == 1 ? v->uses()[0].user : nullptr; }

// 0 none, 1 ReLU6, 2 ReLU; -1 not an activation
int act_code(Node* n) {
  const std::string k = n->kind().toQualString();
  if (k == "aten::relu" || k == "aten::relu_") return 2;
  if (k == "aten::relu6" || k == "aten::relu6_") return 1;
  if (k == "aten::hardtanh" || k == "aten::hardtanh_" || k == "aten::clamp" || k == "aten::clamp_") {
    double lo = 0, hi = 0;
    if (n->inputs().size() >= 3 && const_double(n->input(1), &lo) && const_double(n->input(2), &hi) && lo == 0.0 &&
        hi == 6.0)
      return 1;
  }
  return -1;
}

struct Conv {
  Node* node = nullptr;
  Value* in = nullptr;
  at::Tensor w, b;  // w [cout, cin/groups, kh, kw]; b may be undefined
  int64_t stride = 1, pad = 0, dil = 1, groups = 1;
  int64_t cin = 0, cout = 0, kh = 0, kw = 0;
  Node* act_node = nullptr;
  int act = 0;
  Value* result = nullptr;  // the activation's output when fused, else the conv's
  bool pw() const { return kh == 1 && kw == 1 && stride == 1 && pad == 0 && groups == 1; }
  bool dw() const { return kh == 3 && kw == 3 && groups == cin && cin == cout && pad == dil && dil >= 1; }
};

bool symmetric(const std::vector<int64_t>& v, int64_t* out) {
  if (v.empty()) return false;
  for (int64_t x : v)
    if (x != v[0]) return false;
  *out = v[0];
  return true;
}

// aten::conv2d(input, weight, bias, stride, padding, dilation, groups) or
// aten::_convolution(input, weight, bias, stride, padding, dilation, transposed, output_padding, groups, ...)
bool parse_conv(Node* n, Conv* c) {
  const std::string k = n->kind().toQualString();
  const bool conv2d = k == "aten::conv2d", conv_ = k == "aten::_convolution";
  if (!conv2d && !conv_) return false;
  std::vector<int64_t> st, pd, dl;
  int64_t groups = 1;
  if (!const_tensor(n->input(1), &c->w) || c->w.dim() != 4 || c->w.scalar_type() != at::kFloat) return false;
  if (!const_none(n->input(2)) && !const_tensor(n->input(2), &c->b)) return false;
  if (!const_ints(n->input(3), &st) || !const_ints(n->input(5), &dl)) return false;
  if (!const_ints(n->input(4), &pd)) return false;  // (string padding "same" is not lowered)
  if (conv_) {
    bool transposed = false;
    if (!const_bool(n->input(6), &transposed) || transposed || !const_int(n->input(8), &groups)) return false;
  } else if (!const_int(n->input(6), &groups)) {
    return false;
  }
  if (!symmetric(st, &c->stride) || !symmetric(pd, &c->pad) || !symmetric(dl, &c->dil)) return false;
  c->node = n;
  c->in = n->input(0);
  c->groups = groups;
  c->cout = c->w.size(0);
  c->cin = c->w.size(1) * groups;
  c->kh = c->w.size(2);
  c->kw = c->w.size(3);
  c->result = n->output();
  if (Node* u = single_user(n->output())) {
    const int a = act_code(u);
    if (a >= 0) {
      c->act_node = u;
      c->act = a;
      c->result = u->output();
    }
  }
  return true;
}

at::Tensor bias_of(const Conv& c, int64_t pad_to) {
  at::Tensor b = at::zeros({pad_to}, at::kFloat);
  if (c.b.defined()) b.slice(0, 0, c.cout).copy_(c.b.to(at::kCPU).to(at::kFloat));
  return b;
}

// fp32 [rows, cols] weights of the fp32 GEMMs: rows padded to 16, cols to 8
at::Tensor pw_matrix(const at::Tensor& w2, int64_t rpad, int64_t cpad) {
  at::Tensor out = at::zeros({rpad, cpad}, at::kFloat);
  out.slice(0, 0, w2.size(0)).slice(1, 0, w2.size(1)).copy_(w2.to(at::kCPU).to(at::kFloat));
  return out;
}

// the split-bf16 form [3, rows, cols] of an fp32 matrix (models/fused.py x3_split)
at::Tensor x3_split(const at::Tensor& w2, int64_t rows, int64_t cols) {
  at::Tensor wp = at::zeros({rows, cols}, at::kFloat);
  wp.slice(0, 0, w2.size(0)).slice(1, 0, w2.size(1)).copy_(w2.to(at::kCPU).to(at::kFloat));
  at::Tensor hi = wp.to(at::kBFloat16);
  at::Tensor r = wp - hi.to(at::kFloat);
  at::Tensor mid = r.to(at::kBFloat16);
  at::Tensor lo = (r - mid.to(at::kFloat)).to(at::kBFloat16);
  return at::stack({hi, mid, lo}).contiguous();
}

int64_t up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

class Lowering {
 public:
  Lowering(torch::jit::Module& m, const torch::Device& dev, LowerReport* rep)
      : m_(m), g_(m.get_method("forward").graph()), dev_(dev), rep_(rep) {}

  bool run(std::string* err) {
    if (g_->inputs().size() < 2) {
      *err = "forward takes no input";
      return false;
    }
    self_ = g_->inputs()[0];
    input_ = g_->inputs()[1];
    std::vector<Node*> nodes(g_->nodes().begin(), g_->nodes().end());
    for (Node* n : nodes) {
      Conv c;
      if (parse_conv(n, &c)) ++rep_->convs;
    }
    if (rep_->convs == 0) {
      *err = "no conv2d with constant weights (not a frozen conv model)";
      return false;
    }
    for (Node* n : nodes) {
      if (consumed_.count(n)) continue;
      WithInsertPoint ip(n);
      if (!lower(n)) rewire_inputs(n);
    }
    // graph outputs: NCHW views of lowered 4-D values, lowered 2-D values as they are
    for (size_t i = 0; i < g_->outputs().size(); ++i) {
      Value* o = g_->outputs()[i];
      auto f = flat_.find(o);
      if (f != flat_.end()) {
        g_->return_node()->replaceInput(i, f->second);
        continue;
      }
      auto h = nhwc_.find(o);
      if (h != nhwc_.end()) {
        WithInsertPoint ip(g_->return_node());
        g_->return_node()->replaceInput(i, nchw_view(h->second));
      }
    }
    torch::jit::EliminateDeadCode(g_);
    if (rep_->lowered == 0 && rep_->linears == 0) {
      *err = "no layer matched";
      return false;
    }
    return true;
  }

 private:
  Value* cst(const at::Tensor& t) { return g_->insertConstant(t.to(dev_).contiguous()); }

  Value* call(const char* op, std::vector<NamedValue> args) { return g_->insert(nnsx_op(op), args); }

  Value* nchw_view(Value* v) {
    return g_->insert(c10::aten::permute, {v, std::vector<int64_t>{0, 3, 1, 2}});
  }

  // the NHWC lowered form of a 4-D NCHW value (permuted once when it comes from ATen)
  Value* nhwc(Value* v) {
    auto it = nhwc_.find(v);
    if (it != nhwc_.end()) return it->second;
    Value* p = g_->insert(c10::aten::permute, {v, std::vector<int64_t>{0, 2, 3, 1}});
    Value* c = g_->insert(c10::aten::contiguous, {p});
    nhwc_[v] = c;
    return c;
  }

  Value* lut() {
    if (lut_) return lut_;
    if (!m_.hasattr("in_lut")) {
      // default table: the byte value itself (a bare typecast); an absorbed
      // tensor_transform rewrites it (filter/pytorch.cc apply_lut)
      m_.register_attribute("in_lut", c10::TensorType::get(), at::arange(256, at::kFloat).to(dev_));
      rep_->lut = true;
    }
    WithInsertPoint ip(*g_->nodes().begin());
    lut_ = g_->insertGetAttr(self_, "in_lut");
    return lut_;
  }

  Value* tickets() {
    const std::string name = strfmt("nnsx_tickets_", ntickets_++);
    m_.register_attribute(name, c10::TensorType::get(), at::zeros({768}, at::TensorOptions().dtype(at::kInt).device(dev_)));
    Node* first = *g_->nodes().begin();
    Value* v;
    {
      WithInsertPoint ip(first);
      v = g_->insertGetAttr(self_, name);
    }
    return v;
  }

  // is this value the NNStreamer video tensor seen as NCHW (the NHWC wrapper's
  // entry permute), or already lowered?
  bool lowered4(Value* v) const { return nhwc_.count(v) != 0; }

  bool lower(Node* n) {
    const std::string k = n->kind().toQualString();
    if (k == "aten::permute" && n->input(0) == input_) {
      std::vector<int64_t> d;
      if (const_ints(n->input(1), &d) && d == std::vector<int64_t>{0, 3, 1, 2}) {
        nhwc_[n->output()] = input_;  // the frame is NHWC already
        return true;
      }
      return false;
    }
    Conv c;
    if (parse_conv(n, &c)) return lower_conv(c);
    if ((k == "aten::add" || k == "aten::add_") && n->inputs().size() >= 3) {
      double alpha = 0;
      if (lowered4(n->input(0)) && lowered4(n->input(1)) && const_double(n->input(2), &alpha) && alpha == 1.0) {
        nhwc_[n->output()] = g_->insert(c10::aten::add, {nhwc_[n->input(0)], nhwc_[n->input(1)]});
        return true;
      }
      return false;
    }
    const int a = act_code(n);
    if (a > 0 && lowered4(n->input(0))) {
      Value* x = nhwc_[n->input(0)];
      nhwc_[n->output()] =
          a == 1 ? g_->insert(c10::aten::clamp, {x, 0.0, 6.0}) : g_->insert(c10::aten::relu, {x});
      return true;
    }
    if (a > 0 && flat_.count(n->input(0))) {
      Value* x = flat_[n->input(0)];
      flat_[n->output()] = a == 1 ? g_->insert(c10::aten::clamp, {x, 0.0, 6.0}) : g_->insert(c10::aten::relu, {x});
      return true;
    }
    if (k == "aten::mean" && lowered4(n->input(0)) && spatial_mean(n)) {
      flat_[n->output()] = call("avgpool", {nhwc_[n->input(0)]});
      return true;
    }
    if (k == "aten::adaptive_avg_pool2d" && lowered4(n->input(0))) {
      std::vector<int64_t> os;
      if (const_ints(n->input(1), &os) && (os == std::vector<int64_t>{1, 1} || os == std::vector<int64_t>{1})) {
        pooled_[n->output()] = call("avgpool", {nhwc_[n->input(0)]});  // [B, C] standing for [B, C, 1, 1]
        return true;
      }
      return false;
    }
    if ((k == "aten::flatten" || k == "aten::reshape" || k == "aten::view") && pooled_.count(n->input(0))) {
      int64_t s = 0;
      if (k == "aten::flatten" && const_int(n->input(1), &s) && s == 1) {
        flat_[n->output()] = pooled_[n->input(0)];
        return true;
      }
      return false;
    }
    if ((k == "aten::dropout" || k == "aten::dropout_" || k == "aten::feature_dropout") && n->inputs().size() >= 3) {
      bool train = true;
      if (!const_bool(n->input(2), &train) || train) return false;
      if (flat_.count(n->input(0))) {
        flat_[n->output()] = flat_[n->input(0)];
        return true;
      }
      if (lowered4(n->input(0))) {
        nhwc_[n->output()] = nhwc_[n->input(0)];
        return true;
      }
      return false;
    }
    if (k == "aten::flatten" && flat_.count(n->input(0))) {
      flat_[n->output()] = flat_[n->input(0)];
      return true;
    }
    if (k == "aten::linear" && flat_.count(n->input(0))) {
      at::Tensor w, b;
      if (!const_tensor(n->input(1), &w) || w.dim() != 2 || w.scalar_type() != at::kFloat) return false;
      if (!const_none(n->input(2)) && !const_tensor(n->input(2), &b)) return false;
      const int64_t N = w.size(0), K = w.size(1);
      if (N % 4 || K % 4) return false;
      at::Tensor bias = at::zeros({up(N, 16)}, at::kFloat);
      if (b.defined()) bias.slice(0, 0, N).copy_(b.to(at::kCPU));
      flat_[n->output()] = call("pw_conv", {flat_[n->input(0)], cst(pw_matrix(w, up(N, 16), up(K, 8))), cst(bias),
                                            c10::IValue(), N, int64_t{0}, true});
      ++rep_->linears;
      return true;
    }
    return false;
  }

  bool spatial_mean(Node* n) const {
    std::vector<int64_t> d;
    bool keep = true;
    if (n->inputs().size() < 3 || !const_ints(n->input(1), &d) || !const_bool(n->input(2), &keep) || keep) return false;
    if (n->inputs().size() >= 4 && !const_none(n->input(3))) return false;
    std::sort(d.begin(), d.end());
    return d == std::vector<int64_t>{2, 3} || d == std::vector<int64_t>{-2, -1};
  }

  // a 1x1 conv whose result feeds only the spatial mean (head + pool)
  Node* pooled_by(const Conv& c) const {
    Node* u = single_user(c.result);
    if (!u) return nullptr;
    const std::string k = u->kind().toQualString();
    if (k == "aten::mean" && spatial_mean(u)) return u;
    return nullptr;
  }

  // ---- conv chains ----
  bool lower_conv(Conv& c) {
    // stem: 3x3/2 on the 3-channel frame, 32 outputs
    if (c.kh == 3 && c.kw == 3 && c.cin == 3 && c.cout == 32 && c.stride == 2 && c.pad == 1 && c.dil == 1 &&
        c.groups == 1 && (c.in == input_ || lowered4(c.in)))
      return lower_stem(c);
    // inverted residual (with expand)
    if (c.pw() && c.act == 1) {
      Conv d, p;
      if (next_conv(c, &d) && d.dw() && d.act == 1 && d.cin == c.cout && next_conv(d, &p) && p.pw() && p.act == 0 &&
          p.cin == d.cout)
        return emit_ir(&c, d, p);
    }
    // inverted residual without expand (dw -> pw)
    if (c.dw() && c.act == 1 && lowered4(c.in)) {
      Conv p;
      if (next_conv(c, &p) && p.pw() && p.act == 0 && p.cin == c.cout) return emit_ir(nullptr, c, p);
    }
    // head 1x1 + act + global average pool
    if (c.pw() && c.cin % 4 == 0 && c.cout % 4 == 0) {
      if (Node* mean = pooled_by(c)) {
        Value* y = call("pw_conv_pool", {nhwc(c.in), cst(pw_matrix(c.w.reshape({c.cout, c.cin}), up(c.cout, 16),
                                                                   up(c.cin, 8))),
                                         cst(bias_of(c, up(c.cout, 16))), c.cout, static_cast<int64_t>(c.act)});
        consume(c);
        consumed_.insert(mean);
        flat_[mean->output()] = y;
        rep_->head_pool = true;
        ++rep_->lowered;
        return true;
      }
      nhwc_[c.result] =
          call("pw_conv", {nhwc(c.in), cst(pw_matrix(c.w.reshape({c.cout, c.cin}), up(c.cout, 16), up(c.cin, 8))),
                           cst(bias_of(c, up(c.cout, 16))), c10::IValue(), c.cout, static_cast<int64_t>(c.act), true});
      consume(c);
      ++rep_->lowered;
      return true;
    }
    if (c.dw() && c.cin % 4 == 0) {
      nhwc_[c.result] = call("dw_conv", {nhwc(c.in), cst(c.w.reshape({c.cin, 9}).t().contiguous().to(at::kFloat)),
                                         cst(bias_of(c, c.cout)), c.stride, static_cast<int64_t>(c.act == 1 ? 1 : 0), c.dil});
      if (c.act == 2) nhwc_[c.result] = g_->insert(c10::aten::relu, {nhwc_[c.result]});  // (dw_conv fuses ReLU6 only)
      consume(c);
      ++rep_->lowered;
      return true;
    }
    return false;
  }

  // the conv that alone consumes c's result
  bool next_conv(const Conv& c, Conv* out) const {
    Node* u = single_user(c.result);
    return u && parse_conv(u, out) && out->in == c.result;
  }

  void consume(const Conv& c) {
    consumed_.insert(c.node);
    if (c.act_node) consumed_.insert(c.act_node);
  }

  bool emit_ir(Conv* e, Conv& d, Conv& p) {
    Value* xin = e ? e->in : d.in;
    const int64_t hid = d.cout, cin = e ? e->cin : d.cin, cout = p.cout;
    if (hid % 16 || cin % 4 || cout % 4) return false;
    // residual: the project's result consumed only by `x + y` (either order) with x the block input
    Node* add = single_user(p.result);
    bool residual = false;
    if (add && (std::string(add->kind().toQualString()) == "aten::add" ||
                std::string(add->kind().toQualString()) == "aten::add_")) {
      double alpha = 0;
      Value* other = add->input(0) == p.result ? add->input(1) : add->input(0);
      residual = add->inputs().size() >= 3 && const_double(add->input(2), &alpha) && alpha == 1.0 && other == xin &&
                 d.stride == 1 && cin == cout;
    }
    at::Tensor we = e ? pw_matrix(e->w.reshape({hid, cin}), hid, up(cin, 8)) : at::zeros({1}, at::kFloat);
    at::Tensor be = e ? bias_of(*e, hid) : at::zeros({1}, at::kFloat);
    at::Tensor wd = d.w.reshape({hid, 9}).t().contiguous().to(at::kFloat);
    at::Tensor bd = bias_of(d, hid);
    at::Tensor wp = pw_matrix(p.w.reshape({cout, hid}), up(cout, 16), hid);
    at::Tensor bp = bias_of(p, up(cout, 16));
    std::vector<NamedValue> args = {nhwc(xin), cst(we), cst(be), cst(wd), cst(bd), cst(wp), cst(bp), d.stride,
                                    cout, e != nullptr, residual, d.dil, tickets()};
    if (e) {
      args.push_back(cst(x3_split(e->w.reshape({hid, cin}), hid, up(cin, 32))));
      args.push_back(cst(x3_split(p.w.reshape({cout, hid}), up(cout, 32), hid)));
    } else {
      args.push_back(c10::IValue());
      args.push_back(c10::IValue());
    }
    Value* y = call("ir_block_any", args);
    if (e) consume(*e);
    consume(d);
    consume(p);
    if (residual) {
      consumed_.insert(add);
      nhwc_[add->output()] = y;
    } else {
      nhwc_[p.result] = y;
    }
    ++rep_->ir_blocks;
    rep_->lowered += e ? 3 : 2;
    return true;
  }

  bool lower_stem(Conv& c) {
    Value* x = c.in == input_ && !lowered4(c.in) ? nullptr : nhwc(c.in);
    if (!x) {
      // an NCHW frame straight into the stem: one permute to NHWC
      x = nhwc(input_);
    }
    at::Tensor ws = c.w.permute({2, 3, 1, 0}).contiguous().to(at::kFloat);  // [ky, kx, ci, co]
    at::Tensor bs = bias_of(c, 32);
    // + a t = 1 first block: dw 3x3/1 + ReLU6 on the 32 channels -> 1x1 -> 16, no residual
    Conv d, p;
    if (c.act == 1 && next_conv(c, &d) && d.dw() && d.stride == 1 && d.dil == 1 && d.act == 1 && d.cin == 32 &&
        next_conv(d, &p) && p.pw() && p.act == 0 && p.cin == 32 && p.cout == 16) {
      Node* add = single_user(p.result);
      const bool plain_end = !add || std::string(add->kind().toQualString()) != "aten::add";
      if (plain_end) {
        Value* y = call("stem_ir1_any", {x, cst(ws), cst(bs), cst(d.w.reshape({32, 9}).t().contiguous().to(at::kFloat)),
                                         cst(bias_of(d, 32)), cst(pw_matrix(p.w.reshape({16, 32}), 16, 32)),
                                         cst(bias_of(p, 16)), lut(), int64_t{16}});
        consume(c);
        consume(d);
        consume(p);
        nhwc_[p.result] = y;
        rep_->stem_block = true;
        rep_->lowered += 3;
        return true;
      }
    }
    Value* y = call("stem_any", {x, cst(ws), cst(bs), lut(), static_cast<int64_t>(c.act)});
    consume(c);
    nhwc_[c.result] = y;
    ++rep_->lowered;
    return true;
  }

  // a node left on ATen: every lowered operand is handed over in its original layout
  void rewire_inputs(Node* n) {
    for (size_t i = 0; i < n->inputs().size(); ++i) {
      Value* v = n->input(i);
      if (flat_.count(v)) {
        n->replaceInput(i, flat_[v]);
      } else if (pooled_.count(v)) {
        n->replaceInput(i, g_->insert(c10::aten::unsqueeze,
                                      {g_->insert(c10::aten::unsqueeze, {pooled_[v], int64_t{-1}}), int64_t{-1}}));
      } else if (nhwc_.count(v) && nhwc_[v] != v) {
        n->replaceInput(i, nchw_view(nhwc_[v]));
      }
    }
  }

  torch::jit::Module& m_;
  std::shared_ptr<Graph> g_;
  torch::Device dev_;
  LowerReport* rep_;
  Value* self_ = nullptr;
  Value* input_ = nullptr;
  Value* lut_ = nullptr;
  int ntickets_ = 0;
  std::unordered_map<Value*, Value*> nhwc_;    // original 4-D NCHW value -> its NHWC lowered form
  std::unordered_map<Value*, Value*> flat_;    // original 2-D value -> its lowered form (same layout)
  std::unordered_map<Value*, Value*> pooled_;  // original [B, C, 1, 1] -> lowered [B, C]
  std::unordered_set<Node*> consumed_;
};

}  // namespace

// tools / tests: load, freeze, lower and save a TorchScript file; returns the
// report ("not lowered: <why>" when nothing matched, the file then unchanged)
std::string lower_torchscript_file(const std::string& in, const std::string& out, int device) {
  const torch::Device dev = device >= 0 ? torch::Device(torch::kCUDA, device) : torch::Device(torch::kCPU);
  torch::jit::Module m = torch::jit::load(in, dev);
  m.eval();
  m = torch::jit::freeze(m);
  LowerReport rep;
  std::string why;
  if (!lower_to_engine(m, dev, &rep, &why)) {
    m.save(out);
    return "not lowered: " + why;
  }
  m.save(out);
  return rep.summary();
}

bool lower_to_engine(torch::jit::Module& m, const torch::Device& device, LowerReport* rep, std::string* err) {
  LowerReport r;
  try {
    Lowering l(m, device, &r);
    if (!l.run(err)) return false;
  } catch (const std::exception& e) {
    if (err) *err = e.what();
    return false;
  }
  if (rep) *rep = r;
  return true;
}

}  // namespace nnsx
