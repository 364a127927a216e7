// tensor_filter framework=pytorch on PyTorch-ROCm (libtorch C++, TorchScript).
//
// Reference behaviour: ext/nnstreamer/tensor_filter/tensor_filter_pytorch.cc
// (load :197-237, reversed dims + input ranks :517-536, forward :544/557,
// tensor/tuple/list outputs flattened :415-492).  The reference stages every
// frame H2D and D2H (:532, :423); here inputs are wrapped zero-copy from the
// device Memory (torch::from_blob on the element's HIP stream), outputs stay
// in HBM as allocate-in-invoke tensors whose lifetime ends with the output
// Memory (DESTROY_NOTIFY), and `custom=hipgraph:true` replays the whole
// forward as one captured hipGraph per input shape.
//
// custom= options (comma separated key:value):
//   hipgraph:true|false   capture/replay the forward (static shapes)
//   dtype:bfloat16|float16|float32   cast floating inputs before forward
//   channels_last:true    pass 4-D inputs in channels-last memory format
//   broadcast:<rank>      load the model once: <rank> broadcasts the file's bytes
//                         to every rank of the job (RCCL / TCP), see load_broadcast
//   broadcast-backend:auto|rccl|tcp, broadcast-store:host:port, broadcast-name:<channel>
//   lower:auto|off        load-time lowering of a plain model onto the nnsx kernels
//                         (filter/torch_lower.cc): auto = on a GPU, verified against
//                         the original on a 2-frame input at load (NNSX_LOWER=0: off)
//   lanes:<n>|auto        replay lanes (hipgraph): consecutive frames go round robin
//                         to n streams, each with its own graphs and memory pool, so
//                         the forwards of small batches overlap on the GPU (auto: 3
//                         for a leading dimension of 2..32 and <= 8 MB of input, else 1)
#include <ATen/hip/HIPGraph.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/script.h>

#include <atomic>
#include <cstdlib>
#include <fstream>
#include <set>
#include <sstream>

#include "comm/group.h"
#include "core/log.h"
#include "filter/filter.h"
#include "filter/torch_lower.h"
#include "filter/torch_util.h"
#include "kernels/kernels.h"
#include "kernels/mbv2.h"
#include "runtime/fusion.h"
#include "runtime/hip_util.h"
#include "runtime/plugin_api.h"

namespace nnsx {

namespace ops {
void x3_retire_flush();  // ops/torch_ops.cc
}  // namespace ops

namespace {

std::vector<int64_t> torch_sizes(const TensorInfo& ti, int rank_override) {
  int rank = rank_override > 0 ? rank_override : ti.rank();
  std::vector<int64_t> s;
  for (int i = rank - 1; i >= 0; --i) s.push_back(ti.dim[i]);
  return s;
}

TensorInfo info_from_tensor(const at::Tensor& t) {
  TensorInfo ti;
  ti.type = from_torch(t.scalar_type());
  ti.dim.fill(1);
  int r = static_cast<int>(t.dim());
  if (r > kRankLimit) throw Error("pytorch: output rank > 8");
  for (int i = 0; i < r; ++i) ti.dim[i] = static_cast<uint32_t>(t.size(r - 1 - i));
  if (r == 0) ti.dim[0] = 1;
  return ti;
}

void flatten(const c10::IValue& v, std::vector<at::Tensor>* out) {
  if (v.isTensor()) {
    out->push_back(v.toTensor());
  } else if (v.isTuple()) {
    for (const auto& e : v.toTupleRef().elements()) flatten(e, out);
  } else if (v.isList()) {
    for (const auto& e : v.toListRef()) flatten(e, out);
  } else if (v.isTensorList()) {
    for (const auto& t : v.toTensorVector()) out->push_back(t);
  } else {
    throw Error("pytorch: unsupported model output type");
  }
}

// GPU model instances alive per device: with more than one, replays of
// different filters may run at the same time, so kernels must not wait inside
// a launch for workgroups that may not be resident (kernels::SharedDeviceScope)
std::atomic<int> g_device_instances[64];

int device_instances(int dev) { return dev >= 0 && dev < 64 ? g_device_instances[dev].load() : 0; }

struct GraphState {
  std::unique_ptr<at::cuda::CUDAGraph> graph;
  std::vector<at::Tensor> static_in;  // the stable input slot the frame is copied into
  std::vector<at::Tensor> static_out;
  // downstream holders of static_out handed out without a copy (0 = free)
  std::shared_ptr<std::atomic<int>> out_held = std::make_shared<std::atomic<int>>(0);
  // in place: static_in IS a pooled upstream block (DeviceBufferPool), replayed
  // whenever that block comes back -- no input copy
  bool in_place = false;
  // small outputs are copied out after each replay, so the instance is free
  // again at once (no instance count driven by downstream queue depth)
  bool copy_out = false;
};

class TorchInstance : public FilterInstance {
 public:
  explicit TorchInstance(FilterProperties& p) : props_(p) {
    parse_custom(p.custom_properties);
    device_ = p.device;
    load(p.model_files.at(0));
    if (device_ >= 0 && device_ < 64) g_device_instances[device_].fetch_add(1);
  }
  ~TorchInstance() override {
    if (device_ >= 0 && device_ < 64) g_device_instances[device_].fetch_sub(1);
    print_trace_wait();
    clear_graphs();
    for (Lane& l : lanes_) {
      hip::DeviceGuard g(l.dev);
      if (l.last_ev) {
        (void)hipEventSynchronize(l.last_ev);
        (void)hipEventDestroy(l.last_ev);
      }
      if (l.in_ev) (void)hipEventDestroy(l.in_ev);
      if (l.stream) {
        (void)hipStreamSynchronize(l.stream);
        (void)hipStreamDestroy(l.stream);
      }
    }
    if (cap_stream_) {
      hip::DeviceGuard g(device_);
      (void)hipStreamSynchronize(cap_stream_);
      (void)hipStreamDestroy(cap_stream_);
    }
  }

  bool wants_host_input() const override { return device_ < 0; }

  std::string info(const std::string& key) const override {
    if (key == "model-broadcast" && !bcast_group_.empty()) return bcast_group_;
    if (key == "lowered") return lowered_;
    return std::string();
  }

  // models exposing a float32 [256] attribute `in_lut` map a uint8 input 0
  // through it (nnstreamer_amd.models.fused: the fused stems); an upstream
  // tensor_transform's arithmetic is folded into that table (runtime/fusion.h)
  bool accepts_input_table(unsigned index) const override { return index == 0 && has_lut_; }

  bool set_input_table(unsigned index, const std::vector<float>& lut) override {
    if (index != 0 || !has_lut_ || lut.size() != 256) return false;
    std::lock_guard<std::mutex> lk(mu_);
    try {
      apply_lut(module_, lut);
    } catch (const std::exception& e) {
      NNSX_LOGE("pytorch", "set_input_table failed: ", e.what());
      return false;
    }
    lut_ = lut;
    if (props_.input_info.num_tensors > 0) props_.input_info.at(0).type = DType::UINT8;
    clear_graphs();
    return true;
  }

  // the absorbing element released the transform (stop, re-link): back to the
  // table the model file shipped with
  bool reset_input_table(unsigned index) override {
    if (index != 0 || !has_lut_) return false;
    std::lock_guard<std::mutex> lk(mu_);
    if (lut_.empty()) return true;
    try {
      apply_lut(module_, default_lut_);
    } catch (const std::exception& e) {
      NNSX_LOGE("pytorch", "reset_input_table failed: ", e.what());
      return false;
    }
    lut_.clear();
    clear_graphs();
    return true;
  }

  // a downstream image_labeling decoder's argmax, run at the end of the
  // forward (inside the captured graph): output `index` becomes the int32
  // index of the largest score along its last dimension (runtime/fusion.h)
  bool accepts_output_argmax(unsigned index) const override { return index == 0; }
  bool set_output_argmax(unsigned index, bool on) override {
    if (index != 0) return false;
    std::lock_guard<std::mutex> lk(mu_);
    argmax_out_ = on ? 0 : -1;
    clear_graphs();
    return true;
  }

  // a downstream decoder's device post-processing, appended to the forward
  // (inside the captured graph): the stage's outputs replace the model's
  // (runtime/fusion.h DecodeStage)
  int stage_device() const override { return device_; }
  bool set_output_stage(std::shared_ptr<DecodeStage> stage) override {
    if (device_ < 0) return false;
    std::lock_guard<std::mutex> lk(mu_);
    stage_ = std::move(stage);
    clear_graphs();
    return true;
  }

  bool get_model_info(TensorsInfo* in, TensorsInfo* out) override {
    if (props_.input_info.num_tensors > 0 && props_.input_info.valid() && props_.output_info.num_tensors > 0 &&
        props_.output_info.valid()) {
      *in = props_.input_info;
      *out = props_.output_info;
      return true;
    }
    if (props_.input_info.num_tensors > 0 && props_.input_info.valid()) {
      // outputs unknown: discover them with one dry run
      if (!set_input_info(props_.input_info, out)) return false;
      *in = props_.input_info;
      return true;
    }
    return false;
  }

  bool set_input_info(const TensorsInfo& in, TensorsInfo* out) override {
    try {
      torch::InferenceMode guard;
      std::vector<c10::IValue> inputs;
      for (unsigned i = 0; i < in.num_tensors; ++i) {
        int rk = i < props_.input_ranks.size() ? props_.input_ranks[i] : 0;
        auto t = torch::zeros(torch_sizes(in.at(i), rk), torch::TensorOptions().dtype(to_torch(in.at(i).type)).device(dev()));
        inputs.push_back(prepare(t));
      }
      std::vector<at::Tensor> outs;
      flatten(module_.forward(inputs), &outs);
      TensorsInfo r;
      r.resize(static_cast<unsigned>(outs.size()));
      for (size_t k = 0; k < outs.size(); ++k) r.at(static_cast<unsigned>(k)) = info_from_tensor(outs[k]);
      *out = r;
      if (device_ >= 0) hip::check(hipDeviceSynchronize(), "sync dry run");
      // the caller now feeds this input (SET_INPUT_INFO): invoke wraps buffers with it
      std::lock_guard<std::mutex> lk(mu_);
      props_.input_info = in;
      props_.output_info = r;
      return true;
    } catch (const std::exception& e) {
      NNSX_LOGE("pytorch", "set_input_info failed: ", e.what());
      return false;
    }
  }

  int invoke(const std::vector<MemoryPtr>& in, std::vector<MemoryPtr>* out, InvokeContext& ctx) override {
    try {
      return do_invoke(in, out, ctx);
    } catch (const std::exception& e) {
      NNSX_LOGE("pytorch", "invoke failed: ", e.what());
      return -1;
    }
  }

  // hot reload (is-updatable, tensor_filter_common.c:1404-1462): the new
  // module is loaded and placed on the device next to the running one, then
  // swapped in under the invoke lock -- frames keep flowing during the load and
  // no frame ever sees a half-loaded model
  bool reload_model(const FilterProperties& p) override {
    try {
      torch::jit::Module fresh = load_module(p.model_files.at(0));
      if (!lut_.empty()) apply_lut(fresh, lut_);  // keep an absorbed transform
      std::lock_guard<std::mutex> lk(mu_);
      module_ = std::move(fresh);
      clear_graphs();  // captured graphs point at the old weights
      return true;
    } catch (const std::exception& e) {
      NNSX_LOGE("pytorch", "reload failed: ", e.what());
      return false;
    }
  }

 private:
  torch::Device dev() const { return device_ >= 0 ? torch::Device(torch::kCUDA, device_) : torch::Device(torch::kCPU); }

  void parse_custom(const std::string& c) {
    for (auto& kv : split(c, ',')) {
      auto p = split(strip(kv), ':', 2);
      if (p.size() != 2) continue;
      std::string k = lower(strip(p[0])), v = strip(p[1]);
      if (k == "hipgraph" || k == "graph") use_graph_ = to_bool(v, false);
      else if (k == "dtype") compute_dtype_ = dtype_from_string(v);
      else if (k == "channels_last") channels_last_ = to_bool(v, false);
      else if (k == "broadcast") bcast_root_ = static_cast<int>(to_int(v));
      else if (k == "broadcast-backend") bcast_backend_ = v;
      else if (k == "broadcast-store") bcast_store_ = v;
      else if (k == "broadcast-name") bcast_name_ = v;
      else if (k == "lower") lower_opt_ = lower(v);
      else if (k == "lanes") lanes_opt_ = lower(v) == "auto" ? 0 : std::max(1, std::min(kMaxLanes, static_cast<int>(to_int(v))));
    }
  }

  torch::jit::Module load_module(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw Error("pytorch: cannot read " + path);
    return load_bytes(std::string((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>()));
  }

  torch::jit::Module load_bytes(const std::string& bytes) {
    hip::DeviceGuard g(device_);
    std::istringstream is(bytes);
    torch::jit::Module m = finish_module(torch::jit::load(is, dev()));
    lowered_.clear();
    if (!want_lowering(m)) return m;
    // a second, independent copy is rewritten; the original stays the fallback
    std::istringstream is2(bytes);
    torch::jit::Module low = finish_module(torch::jit::load(is2, dev()));
    LowerReport rep;
    std::string why;
    if (!lower_to_engine(low, dev(), &rep, &why)) {
      NNSX_LOGI("pytorch", "model not lowered onto the nnsx kernels: ", why);
      return m;
    }
    if (!verify_lowering(m, low, &why)) {
      NNSX_LOGW("pytorch", "lowered model rejected (", why, "); running the model as loaded");
      lowered_ = "rejected: " + why;
      return m;
    }
    lowered_ = rep.summary();
    NNSX_LOGI("pytorch", "model lowered onto the nnsx kernels: ", lowered_);
    has_lut_ = low.hasattr("in_lut");
    if (has_lut_ && default_lut_.empty()) {
      at::Tensor t = low.attr("in_lut").toTensor().detach().to(torch::kCPU).contiguous();
      default_lut_.assign(t.data_ptr<float>(), t.data_ptr<float>() + 256);
    }
    return low;
  }

  // plain models on a GPU: not nnsx's own exports (those call torch.ops.nnsx
  // already, or expose in_lut), and only with a known input shape to verify on
  bool want_lowering(const torch::jit::Module& m) const {
    if (device_ < 0 || lower_opt_ == "off" || lower_opt_ == "false" || has_lut_) return false;
    if (const char* e = std::getenv("NNSX_LOWER"))
      if (e[0] == '0') return false;
    if (props_.input_info.num_tensors != 1 || !props_.input_info.valid()) return false;
    try {
      for (const torch::jit::Node* n : m.get_method("forward").graph()->nodes())
        if (std::string(n->kind().toQualString()).rfind("nnsx::", 0) == 0) return false;
    } catch (...) {
      return false;
    }
    return true;
  }

  // the lowered module must reproduce the original on a 2-frame random input
  // (max |diff| <= 1e-3 of the output scale, every output)
  bool verify_lowering(torch::jit::Module& orig, torch::jit::Module& low, std::string* why) {
    try {
      torch::InferenceMode guard;
      const TensorInfo& ti = props_.input_info.at(0);
      if (ti.type != DType::FLOAT32) {
        *why = "input type is not float32";
        return false;
      }
      const int rk = !props_.input_ranks.empty() ? props_.input_ranks[0] : 0;
      std::vector<int64_t> sz = torch_sizes(ti, rk);
      if (sz.size() == 4) sz[0] = 2;
      at::Tensor x = torch::randn(sz, torch::TensorOptions().dtype(torch::kFloat).device(dev()));
      std::vector<at::Tensor> a, b;
      flatten(orig.forward({x}), &a);
      flatten(low.forward({x}), &b);
      if (device_ >= 0) hip::check(hipDeviceSynchronize(), "lowering check");
      if (a.size() != b.size()) {
        *why = "output count differs";
        return false;
      }
      for (size_t i = 0; i < a.size(); ++i) {
        if (a[i].sizes() != b[i].sizes()) {
          *why = strfmt("output ", i, " shape differs");
          return false;
        }
        const double scale = std::max(1.0, a[i].abs().max().item<double>());
        const double d = (a[i].to(torch::kFloat) - b[i].to(torch::kFloat)).abs().max().item<double>() / scale;
        if (!(d <= 1e-3)) {
          *why = strfmt("output ", i, " differs by ", d, " of its scale");
          return false;
        }
      }
      return true;
    } catch (const std::exception& e) {
      *why = e.what();
      return false;
    }
  }

  // eval + freeze (constant-folds attributes); `in_lut` stays a mutable
  // attribute so an absorbed transform can rewrite it in place
  torch::jit::Module finish_module(torch::jit::Module m) {
    m.eval();
    has_lut_ = false;
    if (m.hasattr("in_lut")) {
      const c10::IValue v = m.attr("in_lut");
      has_lut_ = v.isTensor() && v.toTensor().scalar_type() == torch::kFloat && v.toTensor().numel() == 256;
      if (has_lut_ && default_lut_.empty()) {
        at::Tensor t = v.toTensor().detach().to(torch::kCPU).contiguous();
        default_lut_.assign(t.data_ptr<float>(), t.data_ptr<float>() + 256);
      }
    }
    try {
      if (has_lut_)
        m = torch::jit::freeze(m, std::vector<std::string>{"in_lut"});
      else
        m = torch::jit::freeze(m);
    } catch (...) {
    }
    return m;
  }

  void apply_lut(torch::jit::Module& m, const std::vector<float>& lut) {
    torch::NoGradGuard ng;
    hip::DeviceGuard g(device_);
    at::Tensor t = m.attr("in_lut").toTensor();
    at::Tensor src = torch::from_blob(const_cast<float*>(lut.data()), {256}, torch::kFloat).clone();
    t.copy_(src.to(t.device()));
    if (device_ >= 0) hip::check(hipDeviceSynchronize(), "in_lut upload");
  }
  void load(const std::string& path) {
    if (bcast_root_ < 0) {
      module_ = load_module(path);
      return;
    }
    try {
      module_ = load_broadcast(path);
    } catch (const std::exception& e) {
      // the data plane must never cost a rank its model: when the broadcast
      // fails (a member missing, an aborted communicator) and this rank has
      // the file itself, it loads it and reports the failure in model-broadcast
      std::ifstream f(path, std::ios::binary);
      if (!f) throw;
      NNSX_LOGW("pytorch", e.what(), "; loading ", path, " locally");
      bcast_group_ = strfmt("failed:", e.what());
      module_ = load_module(path);
    }
  }

  // custom=broadcast:<root rank>: one-process-per-GPU deployments load the
  // model once -- rank <root> reads the TorchScript file and broadcasts its
  // bytes to every rank of the job (comm::Group: RCCL over xGMI between GPUs,
  // the TCP store on hosts), and every rank deserialises the same bytes onto
  // its own device.  Other ranks' model= paths are not read.  Multi-rank
  // counterpart of the reference's in-process shared model table
  // (tensor_filter_common.c:2911-3076).  Group membership comes from the job
  // environment (RANK / WORLD_SIZE / MASTER_ADDR:MASTER_PORT, or
  // broadcast-store:host:port).
  torch::jit::Module load_broadcast(const std::string& path) {
    comm::GroupSpec spec;
    spec.name = "model-broadcast/" + (bcast_name_.empty() ? std::string("default") : bcast_name_);
    spec.device = device_;
    spec.backend = bcast_backend_;
    spec.store = bcast_store_;
    std::string err;
    auto g = comm::Group::open(spec, &err);
    if (!g) throw Error("model broadcast: cannot join the rank group: " + err);
    int root = -1;
    for (int i = 0; i < g->size(); ++i)
      if (g->global_rank(i) == bcast_root_) root = i;
    if (root < 0) throw Error("model broadcast: root rank " + std::to_string(bcast_root_) + " is not in the job");
    comm::Packet pkt;
    if (g->rank() == root) {
      std::ifstream f(path, std::ios::binary);
      if (!f) throw Error("model broadcast: cannot read " + path);
      std::string bytes((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
      pkt.blobs.push_back(Memory::from_bytes(bytes.data(), bytes.size()));
    }
    if (!g->broadcast(root, &pkt, &err) || pkt.blobs.empty()) throw Error("model broadcast failed: " + err);
    const MemoryPtr& blob = pkt.blobs[0];
    std::string bytes(static_cast<const char*>(blob->map_host()), blob->size());
    bcast_bytes_ = bytes.size();
    bcast_group_ = strfmt(g->backend_name(), ":", g->size(), ":", bytes.size());
    NNSX_LOGI("pytorch", "model of rank ", bcast_root_, " received over ", g->backend_name(), " (", bytes.size(),
              " bytes, group rank ", g->rank(), "/", g->size(), ")");
    return load_bytes(bytes);
  }

  // outs[argmax_out_] -> int32 index of the first largest value along the last
  // dimension (the decoder's rule), on the device with kernels::argmax_rows
  void apply_argmax(std::vector<at::Tensor>* outs, hipStream_t s) {
    if (argmax_out_ < 0 || static_cast<size_t>(argmax_out_) >= outs->size()) return;
    at::Tensor t = (*outs)[static_cast<size_t>(argmax_out_)].contiguous();
    if (t.dim() == 0 || t.numel() == 0) return;
    std::vector<int64_t> sizes = t.sizes().vec();
    const int64_t n = sizes.back();
    sizes.back() = 1;
    at::Tensor idx;
    if (t.is_cuda()) {
      idx = at::empty(sizes, t.options().dtype(at::kInt));
      kernels::argmax_rows(t.data_ptr(), from_torch(t.scalar_type()), static_cast<uint64_t>(n),
                           static_cast<uint32_t>(t.numel() / n), idx.data_ptr<int32_t>(), s);
    } else {
      idx = t.argmax(-1, /*keepdim=*/true).to(at::kInt);
    }
    (*outs)[static_cast<size_t>(argmax_out_)] = idx;
  }

  // outs (model outputs on the device) -> the decode stage's outputs, enqueued
  // on s (the capture stream while capturing: kernels and memsets only)
  void apply_stage(std::vector<at::Tensor>* outs, hipStream_t s) {
    if (!stage_) return;
    const TensorsInfo& oi = stage_->out_info();
    std::vector<const void*> in;
    std::vector<at::Tensor> keep;
    for (auto& t : *outs) {
      at::Tensor c = t.contiguous();
      keep.push_back(c);
      in.push_back(c.data_ptr());
    }
    std::vector<at::Tensor> res;
    std::vector<void*> optr;
    for (unsigned k = 0; k < oi.num_tensors; ++k) {
      at::Tensor o = at::empty(torch_sizes(oi.at(k), 0),
                               keep.empty() ? at::TensorOptions() : keep[0].options().dtype(to_torch(oi.at(k).type)));
      optr.push_back(o.data_ptr());
      res.push_back(o);
    }
    if (!stage_->enqueue(in, optr, s)) throw Error("pytorch: the decoder stage rejected the model outputs");
    *outs = std::move(res);
  }

  at::Tensor prepare(at::Tensor t) {
    if (compute_dtype_ != DType::END && at::isFloatingType(t.scalar_type())) t = t.to(to_torch(compute_dtype_));
    if (channels_last_ && t.dim() == 4) t = t.contiguous(at::MemoryFormat::ChannelsLast);
    return t;
  }

  MemoryPtr wrap_output(at::Tensor t, int dev_idx, hipStream_t s, std::shared_ptr<std::atomic<int>> held = nullptr) {
    t = t.contiguous();
    auto holder = std::make_shared<at::Tensor>(t);
    size_t bytes = t.numel() * t.element_size();
    if (dev_idx >= 0) {
      auto m = Memory::wrap(t.data_ptr(), bytes, MemPlace::DEVICE, dev_idx, [holder, s, dev_idx, held](Memory* mm) {
        // the caching allocator (or the next graph replay, for a static output)
        // reuses the block in the order of its stream: make that stream wait for
        // every downstream reader before dropping the tensor
        hip::DeviceGuard g(dev_idx);
        mm->wait_uses(s);
        holder->reset();
        if (held) held->fetch_sub(1);
      });
      m->mark_ready(s);
      return m;
    }
    return Memory::wrap(t.data_ptr(), bytes, MemPlace::HOST, -1, [holder](Memory*) { holder->reset(); });
  }

  int do_invoke(const std::vector<MemoryPtr>& in, std::vector<MemoryPtr>* out, InvokeContext& ctx) {
    std::lock_guard<std::mutex> lk(mu_);
    torch::InferenceMode guard;
    const TensorsInfo& info = props_.input_info;
    int dev_idx = device_ >= 0 ? (ctx.device >= 0 ? ctx.device : device_) : -1;
    hipStream_t s = ctx.stream;
    std::unique_ptr<c10::hip::HIPStreamGuardMasqueradingAsCUDA> sg;
    if (dev_idx >= 0) {
      if (!s) s = hip::thread_copy_stream(dev_idx);
      sg = std::make_unique<c10::hip::HIPStreamGuardMasqueradingAsCUDA>(
          c10::hip::getStreamFromExternalMasqueradingAsCUDA(s, static_cast<c10::DeviceIndex>(dev_idx)));
    }
    // NNSX_TRACE_WAIT=1 (diagnostics): events at the invoke's start on the
    // stream, before the replay and after it -- printed at teardown as the
    // device time spent waiting for the inputs and in the graph, per invoke
    hipEvent_t tw_a = nullptr, tw_b = nullptr, tw_c = nullptr;
    if (trace_wait() && dev_idx >= 0) {
      for (hipEvent_t* e : {&tw_a, &tw_b, &tw_c}) hip::check(hipEventCreate(e), "trace event");
      hip::check(hipEventRecord(tw_a, s), "trace event");
    }
    std::vector<at::Tensor> inputs;
    for (size_t i = 0; i < in.size(); ++i) {
      TensorInfo ti = i < info.num_tensors ? info.at(static_cast<unsigned>(i)) : TensorInfo();
      if (!ti.valid()) {
        ti.type = DType::UINT8;
        ti.dim = make_dims({static_cast<uint32_t>(in[i]->size())});
      }
      int rk = i < props_.input_ranks.size() ? props_.input_ranks[i] : 0;
      auto sizes = torch_sizes(ti, rk);
      auto opts = torch::TensorOptions().dtype(to_torch(ti.type));
      void* ptr;
      if (dev_idx >= 0) {
        ptr = const_cast<void*>(in[i]->map_device(dev_idx, s));
        opts = opts.device(torch::kCUDA, dev_idx);
      } else {
        ptr = const_cast<void*>(in[i]->map_host());
      }
      inputs.push_back(torch::from_blob(ptr, sizes, opts));
    }

    // replay lane: lane 0 runs on the element's stream, lane k > 0 on a private
    // stream ordered after the inputs' arrival on s; everything below (replay,
    // copy-out, output readiness, input release) is on that lane's stream
    const int nl = dev_idx >= 0 && use_graph_ ? lane_count(inputs) : 1;
    const int lane = nl > 1 ? static_cast<int>(invokes_++ % static_cast<uint64_t>(nl)) : 0;
    if (lane > 0) {
      Lane& l = lane_state(lane, dev_idx);
      hip::check(hipEventRecord(l.in_ev, s), "lane input event");
      hip::check(hipStreamWaitEvent(l.stream, l.in_ev, 0), "lane input wait");
      s = l.stream;
      ctx.done_stream = s;
      sg.reset();  // (restores the caller's stream before the lane's guard records it)
      sg = std::make_unique<c10::hip::HIPStreamGuardMasqueradingAsCUDA>(
          c10::hip::getStreamFromExternalMasqueradingAsCUDA(s, static_cast<c10::DeviceIndex>(dev_idx)));
    }
    // more than one lane, or other model instances on the device: kernels must
    // not assume the device to themselves.  Graphs captured under the other
    // assumption are dropped and captured again
    const bool shared_dev = dev_idx >= 0 && (nl > 1 || device_instances(dev_idx) > 1);
    if (shared_dev != graphs_shared_) {
      for (Lane& l : lanes_)
        if (l.last_ev) hip::check(hipEventSynchronize(l.last_ev), "replays done");  // (graphs die below)
      clear_graphs();
      graphs_shared_ = shared_dev;
    }
    kernels::SharedDeviceScope shared(shared_dev);
    Lane& ln = lane_state(lane, dev_idx);

    std::vector<at::Tensor> outs;
    std::vector<MemoryPtr> host_outs;        // outputs already copied to pinned host memory
    std::shared_ptr<std::atomic<int>> held;  // static outputs handed out as they are
    bool pooled = dev_idx >= 0 && !in.empty();
    for (auto& m : in) pooled = pooled && m->on_device() && m->root()->tags().count(DeviceBufferPool::kPoolTag);
    PoolRef pref;
    if (pooled && in.size() == 1) {
      Memory* root = in[0]->root();
      pref.id = static_cast<uint64_t>(root->tags().at(DeviceBufferPool::kPoolTag));
      pref.offset = static_cast<size_t>(static_cast<const char*>(in[0]->data()) - static_cast<const char*>(root->data()));
    }
    GraphState* gs = use_graph_ && dev_idx >= 0 ? graph_for(inputs, s, dev_idx, pooled, pref, lane) : nullptr;
    if (gs) {
      // an instance whose static outputs no downstream element holds: the replay
      // rewrites them and hands them out as they are (no copy); they return to
      // the instance when their last reader is done
      // every graph of this instance shares one memory pool (capture) and a
      // copy-out instance is handed back at once: replays must not overlap, nor
      // a replay the previous one's copy-out.  Elements sharing the instance
      // (shared-tensor-filter-key), or invokes from another thread, bring another
      // stream, so work on a new stream first waits for the last replay -- before
      // the static inputs are rewritten below: issued ahead of this wait, the
      // copy could overwrite an instance's inputs while its previous replay on
      // the old stream had not read them yet (that frame's outputs then carried
      // the next frame's result: test_gpu_filter_graph.py, static outputs, appsrc)
      if (ln.last_ev && ln.last_stream != s) hip::check(hipStreamWaitEvent(s, ln.last_ev, 0), "replay order wait");
      if (!gs->in_place)
        for (size_t i = 0; i < gs->static_in.size(); ++i) gs->static_in[i].copy_(inputs[i], /*non_blocking=*/true);
      // the captured executable on the element's stream (CUDAGraph::replay would
      // first refresh RNG offsets with two fill kernels: the models here draw no
      // random numbers)
      if (tw_b) hip::check(hipEventRecord(tw_b, s), "trace event");
      hip::check(hipGraphLaunch(gs->graph->raw_cuda_graph_exec(), s), "hipGraphLaunch");
      if (tw_c) {
        hip::check(hipEventRecord(tw_c, s), "trace event");
        trace_.push_back({tw_a, tw_b, tw_c});
        tw_a = tw_b = tw_c = nullptr;
      }
      if (copy_out_ || gs->copy_out) {  // private copies of the outputs: the instance is free again
        for (size_t k = 0; k < gs->static_out.size(); ++k) {
          const at::Tensor& t = gs->static_out[k];
          if (static_cast<int>(k) == argmax_out_ && host_argmax_ && t.scalar_type() == at::kInt && t.is_contiguous()) {
            // the absorbed decoder's int32 label indices go straight to pinned host
            // memory on this stream (the decoder reads them on the host): no device
            // clone and no second copy by the decoder
            const size_t bytes = t.numel() * t.element_size();
            auto hm = Memory::alloc_pinned(bytes);
            if (bytes) hip::check(hipMemcpyAsync(hm->data(), t.data_ptr(), bytes, hipMemcpyDeviceToHost, s), "argmax D2H");
            hm->mark_ready(s);
            host_outs.resize(gs->static_out.size());
            host_outs[k] = hm;
            outs.push_back(t);  // (shape and type only)
          } else {
            outs.push_back(t.clone());
          }
        }
      } else {
        held = gs->out_held;
        held->store(1);
        outs = gs->static_out;
      }
      if (!ln.last_ev) hip::check(hipEventCreateWithFlags(&ln.last_ev, hipEventDisableTiming), "replay event");
      hip::check(hipEventRecord(ln.last_ev, s), "replay event record");
      ln.last_stream = s;
    } else {
      std::vector<c10::IValue> iv;
      for (auto& t : inputs) iv.push_back(prepare(t));
      flatten(module_.forward(iv), &outs);
      apply_argmax(&outs, s);
      apply_stage(&outs, s);
    }
    for (auto& m : in)
      if (dev_idx >= 0) m->record_use(s, dev_idx);
    if (ctx.out_info) {
      ctx.out_info->resize(static_cast<unsigned>(outs.size()));
      for (size_t k = 0; k < outs.size(); ++k) ctx.out_info->at(static_cast<unsigned>(k)) = info_from_tensor(outs[k]);
    }
    if (held) held->store(static_cast<int>(outs.size()));  // one count per handed-out tensor
    for (size_t k = 0; k < outs.size(); ++k) {
      if (k < host_outs.size() && host_outs[k]) {
        out->push_back(host_outs[k]);
        continue;
      }
      at::Tensor& t = outs[k];
      if (dev_idx < 0 && t.is_cuda()) t = t.cpu();
      out->push_back(wrap_output(t, dev_idx, s, held));
    }
    for (hipEvent_t e : {tw_a, tw_b, tw_c})  // (an eager invoke: not traced)
      if (e) (void)hipEventDestroy(e);
    return 0;
  }

  // Capture runs on a private stream of this filter, ordered after the element
  // stream `s` by events.  `s` itself is never in capture mode, so other threads
  // may keep enqueueing on it meanwhile -- e.g. the release of an earlier output
  // still queued downstream makes `s` wait for that output's readers
  // (wrap_output) -- which would otherwise invalidate a capture that starts
  // after a hot reload or a new input shape.
  //
  // A replay rewrites its instance's static outputs, so an instance is only
  // replayed when downstream holds none of them (double/triple buffering of the
  // outputs); each input shape keeps up to kInstances instances -- created in
  // the first frames, while the downstream queues fill -- and when all are
  // held the frame runs eagerly (nullptr).
  //
  // Pooled inputs (blocks of an upstream DeviceBufferPool) get in-place
  // instances: one per block address, capturing the block itself as the graph
  // input, so a replay reads the frame where the upstream element wrote it (no
  // input copy; the block stays allocated for the pool's life and recurs only
  // after its previous use was released).  Up to kInPlace per shape, then the
  // copying instances take over.
  static constexpr size_t kInstances = 6;
  static constexpr size_t kInPlace = 12;
  static constexpr size_t kCopyOutBytes = 64u << 20;
  // the pool a single pooled input came from (id 0: none) and its offset in the block
  struct PoolRef {
    uint64_t id = 0;
    size_t offset = 0;
  };

  GraphState* graph_for(const std::vector<at::Tensor>& inputs, hipStream_t s, int dev_idx, bool pooled,
                        const PoolRef& pref, int lane) {
    std::string key = lane ? "L" + std::to_string(lane) + "|" : std::string();
    for (auto& t : inputs) {
      for (auto d : t.sizes()) key += std::to_string(d) + "x";
      key += std::string(c10::toString(t.scalar_type())) + ";";
    }
    if (pooled) {
      std::string pkey = key + "@";
      for (auto& t : inputs) pkey += std::to_string(reinterpret_cast<uintptr_t>(t.data_ptr())) + ";";
      auto it = graphs_.find(pkey);
      if (it != graphs_.end() && !it->second.empty()) {
        GraphState* g = it->second.front().get();
        if (g->copy_out || copy_out_ || g->out_held->load() == 0) return g;
      } else if (in_place_count_[key] < kInPlace) {
        ++in_place_count_[key];
        GraphState* g = capture(graphs_[pkey], inputs, s, dev_idx, pkey, true, lane);
        precapture_pool(inputs, key, s, dev_idx, pref, lane);
        return g;
      }
    }
    auto& set = graphs_[key];
    for (auto& g : set)
      if (g->copy_out || g->out_held->load() == 0) return g.get();  // (never held with copy_out_)
    if (set.size() >= kInstances) return nullptr;
    return capture(set, inputs, s, dev_idx, key, false, lane);
  }

  // the other blocks of the input's pool get their in-place instances now, at
  // the first frame of this shape (a capture costs ~1 ms of host time: taken
  // lazily, each new block address stalled the stream once in steady state)
  void precapture_pool(const std::vector<at::Tensor>& inputs, const std::string& key, hipStream_t s, int dev_idx,
                       const PoolRef& pref, int lane) {
    if (!pref.id || inputs.size() != 1) return;
    auto pool = DeviceBufferPool::find(pref.id);
    if (!pool) return;
    const size_t bytes = inputs[0].numel() * inputs[0].element_size();
    if (pref.offset + bytes > pool->block_size()) return;
    for (void* base : pool->block_addresses()) {
      if (in_place_count_[key] >= kInPlace) break;
      void* p = static_cast<char*>(base) + pref.offset;
      const std::string pk = key + "@" + std::to_string(reinterpret_cast<uintptr_t>(p)) + ";";
      auto it = graphs_.find(pk);
      if (it != graphs_.end() && !it->second.empty()) continue;
      std::vector<at::Tensor> t{torch::from_blob(p, inputs[0].sizes(), inputs[0].options())};
      ++in_place_count_[key];
      capture(graphs_[pk], t, s, dev_idx, pk, true, lane);
    }
  }

  GraphState* capture(std::vector<std::unique_ptr<GraphState>>& set, const std::vector<at::Tensor>& inputs,
                      hipStream_t s, int dev_idx, const std::string& key, bool in_place, int lane) {
    hip::DeviceGuard dg(dev_idx);
    if (!cap_stream_) hip::check(hipStreamCreateWithFlags(&cap_stream_, hipStreamNonBlocking), "capture stream");
    hipEvent_t ev;
    hip::check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "capture event");
    hip::check(hipEventRecord(ev, s), "capture event record");  // inputs were produced on s
    hip::check(hipStreamWaitEvent(cap_stream_, ev, 0), "capture stream wait");
    // and after the lane's last replay, wherever it ran: the warm-up and the
    // capture allocate from the lane's graph pool, whose activations that replay
    // may still be using (an invoke on another stream than the last one)
    if (lanes_[static_cast<size_t>(lane)].last_ev)
      hip::check(hipStreamWaitEvent(cap_stream_, lanes_[static_cast<size_t>(lane)].last_ev, 0), "capture order wait");
    auto gs = std::make_unique<GraphState>();
    {
      c10::hip::HIPStreamGuardMasqueradingAsCUDA cg(
          c10::hip::getStreamFromExternalMasqueradingAsCUDA(cap_stream_, static_cast<c10::DeviceIndex>(dev_idx)));
      gs->in_place = in_place;
      for (auto& t : inputs) gs->static_in.push_back(in_place ? t : torch::empty_like(t, t.options()).copy_(t));
      const std::vector<at::Tensor>& src = gs->static_in;
      std::vector<c10::IValue> iv;
      // warm up on the capture stream (lazy init, autotuning) before the first
      // capture of this module, one pass before a copying instance; an in-place
      // instance (one more pooled block address of a shape already run) captures
      // straight away -- the extra eager forward cost a whole step of GPU time
      const size_t bar = key.find('|'), at = key.find('@');
      const size_t b0 = bar == std::string::npos ? 0 : bar + 1;
      const std::string shape = key.substr(b0, at == std::string::npos ? std::string::npos : at - b0);
      const int warm = graphs_captured_ == 0 ? 3 : (in_place && warmed_.count(shape)) ? 0 : 1;
      warmed_.insert(shape);
      for (int w = 0; w < warm; ++w) {
        iv.clear();
        for (auto& t : src) iv.push_back(prepare(t));
        std::vector<at::Tensor> tmp;
        flatten(module_.forward(iv), &tmp);
      }
      hip::check(hipStreamSynchronize(cap_stream_), "graph warmup sync");
      gs->graph = std::make_unique<at::cuda::CUDAGraph>();
      // one memory pool for every graph of a lane: replays of a lane never
      // overlap (one stream + replay order, do_invoke), so the activations of its
      // forward are allocated once, not once per pooled input block and output
      // buffer; lanes replay concurrently, so each has its own
      at::cuda::MempoolId_t& pool = lanes_[static_cast<size_t>(lane)].pool;
      if (pool.first == 0 && pool.second == 0) pool = at::cuda::graph_pool_handle();
      gs->graph->capture_begin(pool, hipStreamCaptureModeThreadLocal);
      iv.clear();
      for (auto& t : src) iv.push_back(prepare(t));
      flatten(module_.forward(iv), &gs->static_out);
      apply_argmax(&gs->static_out, cap_stream_);
      apply_stage(&gs->static_out, cap_stream_);
      gs->graph->capture_end();
      size_t out_bytes = 0;
      for (auto& t : gs->static_out) out_bytes += t.numel() * t.element_size();
      gs->copy_out = out_bytes <= kCopyOutBytes;
    }
    ++graphs_captured_;
    hip::check(hipEventDestroy(ev), "capture event destroy");
    // the replay runs on s, after the capture stream's work (the static outputs'
    // first contents are not handed out, but keep the streams ordered)
    hipEvent_t done;
    hip::check(hipEventCreateWithFlags(&done, hipEventDisableTiming), "capture done event");
    hip::check(hipEventRecord(done, cap_stream_), "capture done record");
    hip::check(hipStreamWaitEvent(s, done, 0), "capture done wait");
    hip::check(hipEventDestroy(done), "capture done destroy");
    NNSX_LOGI("pytorch", "captured hipGraph for input ", key, in_place ? " (in place)" : "", ", instance ", set.size());
    set.push_back(std::move(gs));
    return set.back().get();
  }

  FilterProperties props_;
  int device_ = -1;
  torch::jit::script::Module module_;
  bool use_graph_ = false;
  int bcast_root_ = -1;  // custom=broadcast:<rank>
  std::string bcast_backend_ = "auto", bcast_store_, bcast_name_;
  size_t bcast_bytes_ = 0;
  std::string bcast_group_;  // "<data plane>:<members>:<bytes>" of the load-time broadcast
  std::string lower_opt_ = "auto";  // custom=lower:auto|off
  std::string lowered_;             // what the load-time lowering did ("" = not lowered)
  const bool copy_out_ = [] {
    const char* e = std::getenv("NNSX_GRAPH_COPY_OUT");
    return e && e[0] == '1';
  }();
  bool channels_last_ = false;
  DType compute_dtype_ = DType::END;
  std::mutex mu_;
  int argmax_out_ = -1;        // output replaced by its argmax (absorbed decoder), -1: none
  std::shared_ptr<DecodeStage> stage_;  // absorbed decoder's device stage (runtime/fusion.h)
  // the absorbed argmax's indices are copied to pinned host memory after each
  // graph replay (a device clone read back by the decoder measured slower: batch 1
  // at a live 500 fps camera p50 308 vs 362-366 us, profiles/r3_b1_host_argmax_ab.txt)
  const bool host_argmax_ = true;
  bool has_lut_ = false;       // the model maps uint8 input 0 through attribute in_lut
  std::vector<float> lut_;     // the absorbed table (re-applied on hot reload)
  std::vector<float> default_lut_;  // the table of the loaded model file (reset_input_table)
  std::map<std::string, std::vector<std::unique_ptr<GraphState>>> graphs_;
  std::map<std::string, size_t> in_place_count_;  // in-place instances per input shape
  std::set<std::string> warmed_;                   // input shapes run eagerly before a capture
  void clear_graphs() {
    graphs_.clear();
    ops::x3_retire_flush();  // (x3 weight parts the dropped graphs baked in: ops/torch_ops.cc)
    for (Lane& l : lanes_) l.pool = {0, 0};  // a pool goes with its last graph
    in_place_count_.clear();
    warmed_.clear();  // a reloaded module runs eagerly again before its first capture
  }
  size_t graphs_captured_ = 0;
  // replay lanes (custom=lanes): lane 0 replays on the element's stream
  static constexpr int kMaxLanes = 4;
  struct Lane {
    int dev = 0;
    hipStream_t stream = nullptr;           // lanes > 0: private stream
    hipEvent_t in_ev = nullptr;             // lanes > 0: inputs arrived on the element's stream
    at::cuda::MempoolId_t pool{0, 0};       // shared by every graph of the lane (capture)
    hipEvent_t last_ev = nullptr;           // end of the lane's latest replay (+ copy-out)
    hipStream_t last_stream = nullptr;
  };
  std::vector<Lane> lanes_ = std::vector<Lane>(kMaxLanes);
  static bool trace_wait() {
    static const bool on = [] {
      const char* e = std::getenv("NNSX_TRACE_WAIT");
      return e && e[0] == '1';
    }();
    return on;
  }
  struct TraceWait {
    hipEvent_t a, b, c;
  };
  std::vector<TraceWait> trace_;  // NNSX_TRACE_WAIT: (invoke start, replay start, replay end) per replay
  void print_trace_wait() {
    if (trace_.empty()) return;
    std::string w = "input-wait ms", g = "graph ms", gap = "start-after-prev-end ms";
    for (size_t i = 0; i < trace_.size(); ++i) {
      auto& t = trace_[i];
      if (hipEventSynchronize(t.c) != hipSuccess) break;
      float x = 0.f, y = 0.f, z = 0.f;
      (void)hipEventElapsedTime(&x, t.a, t.b);
      (void)hipEventElapsedTime(&y, t.b, t.c);
      if (i > 0) (void)hipEventElapsedTime(&z, trace_[i - 1].c, t.b);
      w += strfmt(" ", static_cast<int>(x * 1000));
      g += strfmt(" ", static_cast<int>(y * 1000));
      gap += strfmt(" ", static_cast<int>(z * 1000));
    }
    std::fprintf(stderr, "pytorch filter (us per replay)\n%s\n%s\n%s\n", w.c_str(), g.c_str(), gap.c_str());
    for (auto& t : trace_)
      for (hipEvent_t e : {t.a, t.b, t.c}) (void)hipEventDestroy(e);
    trace_.clear();
  }
  int lanes_opt_ = 0;  // custom=lanes:<n>; 0 = auto
  bool graphs_shared_ = false;  // graphs_ were captured under kernels::SharedDeviceScope
  uint64_t invokes_ = 0;
  int lane_count(const std::vector<at::Tensor>& inputs) const {
    static const int forced = [] {
      const char* e = std::getenv("NNSX_TORCH_LANES");
      return e ? std::max(0, std::min(kMaxLanes, std::atoi(e))) : 0;
    }();
    // an absorbed decoder stage with scratch of its own (candidate lists,
    // keypoint buffers) would have every lane's graph capture the same buffers:
    // concurrent replays on two lanes would share them.  One lane then, whatever
    // custom=lanes asks for; stages that write only their outputs may have lanes.
    if (stage_ && !stage_->lane_safe()) return 1;
    if (forced > 0) return forced;
    if (lanes_opt_ > 0) return lanes_opt_;
    if (inputs.empty() || inputs[0].dim() < 1) return 1;
    size_t bytes = 0;
    for (auto& t : inputs) bytes += t.numel() * t.element_size();
    const int64_t b = inputs[0].size(0);
    // (MobileNetV2 batch 8: 1 / 2 / 3 lanes 20.8k / 20.0k / 26.6k frames/s, batch 32 50.0k / 49.3k /
    // 54.2k; DeepLab batch 8, 6.3 MB of frames, 1 / 3 lanes 7.64k / 7.21k: its forward is long
    // enough to fill the chip alone -- profiles/r4_lanes_ab.txt)
    return b >= 2 && b <= 32 && bytes <= (5u << 20) ? 3 : 1;
  }
  Lane& lane_state(int lane, int dev_idx) {
    Lane& l = lanes_[static_cast<size_t>(lane)];
    if (lane > 0 && !l.stream) {
      hip::DeviceGuard g(dev_idx);
      l.dev = dev_idx;
      hip::check(hipStreamCreateWithFlags(&l.stream, hipStreamNonBlocking), "lane stream");
      hip::check(hipEventCreateWithFlags(&l.in_ev, hipEventDisableTiming), "lane event");
    }
    if (!l.last_ev) l.dev = dev_idx;
    return l;
  }
  hipStream_t cap_stream_ = nullptr;  // private capture stream (graph_for)
};

class TorchFw : public FilterFramework {
 public:
  std::string name() const override { return "pytorch"; }
  std::unique_ptr<FilterInstance> open(FilterProperties& p) override { return std::make_unique<TorchInstance>(p); }
  bool check_availability(Accelerator a) const override {
    if (a == Accelerator::GPU) return hip::available();
    return true;
  }
  std::vector<std::string> model_extensions() const override { return {".pt", ".pth", ".ptl"}; }
  std::string accelerators() const override { return "cpu,gpu"; }
};

}  // namespace

void register_torch_frameworks() { register_filter_framework(std::make_shared<TorchFw>()); }

}  // namespace nnsx
