// Python-backed sub-plugins and data exchange:
//   framework=python3   model=<script>.py with class CustomFilter
//                       (ext/nnstreamer/tensor_filter/tensor_filter_python3.cc)
//   tensor_decoder mode=python3 option1=<script>.py with class CustomDecoder
//   tensor_converter mode=custom-script:<script>.py with class CustomConverter
//   register_custom_easy / register_decoder_custom / register_converter_custom /
//   register_if_custom from Python callables.
// Inputs reach Python as zero-copy numpy views (host) -- the GIL is taken
// only around the callback.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "core/log.h"
#include "decoders/decoders.h"
#include "runtime/hip_util.h"
#include "runtime/plugin_api.h"
#include "single/single.h"

namespace py = pybind11;

namespace nnsx {

namespace {

struct DLDevice {
  int32_t device_type;
  int32_t device_id;
};
struct DLDataType {
  uint8_t code;
  uint8_t bits;
  uint16_t lanes;
};
struct DLTensor {
  void* data;
  DLDevice device;
  int32_t ndim;
  DLDataType dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
};
struct DLManagedTensor {
  DLTensor dl_tensor;
  void* manager_ctx;
  void (*deleter)(DLManagedTensor*);
};
constexpr int32_t kDLCPU = 1, kDLROCM = 10;

struct DLCtx {
  MemoryPtr mem;
  std::vector<int64_t> shape;
  DLManagedTensor mt;
};

DLDataType dl_dtype(DType t) {
  switch (t) {
    case DType::INT8: return {0, 8, 1};
    case DType::INT16: return {0, 16, 1};
    case DType::INT32: return {0, 32, 1};
    case DType::INT64: return {0, 64, 1};
    case DType::UINT8: return {1, 8, 1};
    case DType::UINT16: return {1, 16, 1};
    case DType::UINT32: return {1, 32, 1};
    case DType::UINT64: return {1, 64, 1};
    case DType::FLOAT16: return {2, 16, 1};
    case DType::FLOAT32: return {2, 32, 1};
    case DType::FLOAT64: return {2, 64, 1};
    case DType::BFLOAT16: return {4, 16, 1};
    default: throw Error("dlpack: unsupported dtype");
  }
}

std::string np_dtype_name(DType t) {
  switch (t) {
    case DType::BFLOAT16: return "uint16";
    default: return dtype_name(t) ? dtype_name(t) : "uint8";
  }
}

DType dtype_from_numpy(const py::dtype& d) {
  std::string k(1, d.kind());
  size_t sz = d.itemsize();
  if (k == "f") return sz == 2 ? DType::FLOAT16 : (sz == 4 ? DType::FLOAT32 : DType::FLOAT64);
  if (k == "i") return sz == 1 ? DType::INT8 : sz == 2 ? DType::INT16 : sz == 4 ? DType::INT32 : DType::INT64;
  if (k == "u" || k == "b") return sz == 1 ? DType::UINT8 : sz == 2 ? DType::UINT16 : sz == 4 ? DType::UINT32 : DType::UINT64;
  throw Error("unsupported numpy dtype");
}

}  // namespace

py::object memory_to_numpy(const MemoryPtr& m, const std::string& dtype, std::vector<int64_t> shape) {
  const void* p;
  {
    py::gil_scoped_release r;
    p = m->map_host();
  }
  py::dtype dt(dtype);
  size_t n = m->size() / dt.itemsize();
  if (shape.empty()) shape.push_back(static_cast<int64_t>(n));
  // zero-copy view; the capsule keeps the Memory (or its host mirror) alive
  auto* holder = new MemoryPtr(m);
  py::capsule base(holder, [](void* x) { delete static_cast<MemoryPtr*>(x); });
  return py::array(dt, shape, {}, p, base);
}

py::capsule memory_to_dlpack(const MemoryPtr& m, const TensorInfo& ti) {
  auto* ctx = new DLCtx();
  ctx->mem = m;
  int r = ti.rank();
  for (int i = r - 1; i >= 0; --i) ctx->shape.push_back(ti.dim[i]);
  if (m->on_device()) m->sync_ready();
  DLTensor& t = ctx->mt.dl_tensor;
  t.data = m->on_device() ? m->data() : const_cast<void*>(m->map_host());
  t.device = m->on_device() ? DLDevice{kDLROCM, m->device()} : DLDevice{kDLCPU, 0};
  t.ndim = static_cast<int32_t>(ctx->shape.size());
  t.dtype = dl_dtype(ti.type);
  t.shape = ctx->shape.data();
  t.strides = nullptr;
  t.byte_offset = 0;
  ctx->mt.manager_ctx = ctx;
  ctx->mt.deleter = [](DLManagedTensor* self) { delete static_cast<DLCtx*>(self->manager_ctx); };
  return py::capsule(&ctx->mt, "dltensor", [](PyObject* cap) {
    if (PyCapsule_IsValid(cap, "dltensor")) {
      auto* mt = static_cast<DLManagedTensor*>(PyCapsule_GetPointer(cap, "dltensor"));
      if (mt && mt->deleter) mt->deleter(mt);
    }
  });
}

// numpy array / bytes / torch tensor (via __dlpack__) -> Memory
MemoryPtr memory_from_python(py::handle obj) {
  if (py::isinstance<Memory>(obj)) return obj.cast<MemoryPtr>();
  if (py::isinstance<py::bytes>(obj)) {
    std::string s = obj.cast<py::bytes>();
    return Memory::from_bytes(s.data(), s.size());
  }
  if (py::hasattr(obj, "__cuda_array_interface__") || (py::hasattr(obj, "is_cuda") && obj.attr("is_cuda").cast<bool>())) {
    // torch CUDA(HIP) tensor: zero-copy, the tensor object stays referenced
    py::object t = py::reinterpret_borrow<py::object>(obj);
    if (!t.attr("is_contiguous")().cast<bool>()) t = t.attr("contiguous")();
    uintptr_t ptr = t.attr("data_ptr")().cast<uintptr_t>();
    size_t bytes = t.attr("numel")().cast<size_t>() * t.attr("element_size")().cast<size_t>();
    int dev = t.attr("device").attr("index").cast<int>();
    auto* ref = new py::object(t);
    auto m = Memory::wrap(reinterpret_cast<void*>(ptr), bytes, MemPlace::DEVICE, dev, [ref](Memory*) {
      py::gil_scoped_acquire g;
      delete ref;
    });
    // order after the producer: record on the tensor's current stream
    py::object torch = py::module_::import("torch");
    uintptr_t s = torch.attr("cuda").attr("current_stream")(dev).attr("cuda_stream").cast<uintptr_t>();
    m->mark_ready(reinterpret_cast<hipStream_t>(s));
    return m;
  }
  if (py::hasattr(obj, "numpy") && py::hasattr(obj, "detach")) {
    return memory_from_python(obj.attr("detach")().attr("cpu")().attr("numpy")());
  }
  py::array a = py::array::ensure(obj, py::array::c_style);
  if (!a) throw Error("cannot convert object to tensor memory");
  return Memory::from_bytes(a.data(), static_cast<size_t>(a.nbytes()));
}

namespace {

py::object tensor_shape_class() {
  return py::module_::import("nnstreamer_python").attr("TensorShape");
}

TensorInfo info_from_shape(py::handle shp) {
  TensorInfo ti;
  ti.dim.fill(1);
  auto dims = shp.attr("getDims")().cast<std::vector<int64_t>>();
  for (size_t i = 0; i < dims.size() && i < 8; ++i) ti.dim[i] = static_cast<uint32_t>(dims[i]);
  py::object t = shp.attr("getType")();
  ti.type = dtype_from_numpy(py::dtype::from_args(t));
  return ti;
}

py::object shape_from_info(const TensorInfo& ti) {
  std::vector<int64_t> d(ti.dim.begin(), ti.dim.end());
  py::module_ np = py::module_::import("numpy");
  return tensor_shape_class()(d, np.attr("dtype")(np_dtype_name(ti.type)));
}

TensorsInfo infos_from_list(py::handle lst) {
  TensorsInfo r;
  unsigned i = 0;
  for (auto it : lst) r.at(i++) = info_from_shape(it);
  r.num_tensors = i;
  return r;
}

py::list list_from_infos(const TensorsInfo& in) {
  py::list l;
  for (unsigned i = 0; i < in.num_tensors; ++i) l.append(shape_from_info(in.at(i)));
  return l;
}

py::object load_script_class(const std::string& path, const std::string& cls) {
  py::module_ ilu = py::module_::import("importlib.util");
  std::string modname = "nnsx_script_" + std::to_string(std::hash<std::string>()(path));
  py::object spec = ilu.attr("spec_from_file_location")(modname, path);
  if (spec.is_none()) throw Error("cannot load python script " + path);
  py::object mod = ilu.attr("module_from_spec")(spec);
  spec.attr("loader").attr("exec_module")(mod);
  if (!py::hasattr(mod, cls.c_str())) throw Error(path + " does not define class " + cls);
  return mod.attr(cls.c_str());
}

// ------------------------------------------------------------ python3 filter ----
class PyFilter : public FilterInstance {
 public:
  explicit PyFilter(FilterProperties& p) {
    py::gil_scoped_acquire g;
    py::object cls = load_script_class(p.model_files.at(0), "CustomFilter");
    py::tuple args;
    if (!p.custom_properties.empty()) {
      py::list l;
      for (auto& a : split(p.custom_properties, ' '))
        if (!a.empty()) l.append(a);
      args = py::tuple(l);
    }
    obj_ = std::make_shared<py::object>(cls(*args));
  }
  ~PyFilter() override {
    py::gil_scoped_acquire g;
    obj_.reset();
  }
  bool get_model_info(TensorsInfo* in, TensorsInfo* out) override {
    py::gil_scoped_acquire g;
    if (!py::hasattr(*obj_, "getInputDim") || !py::hasattr(*obj_, "getOutputDim")) return false;
    *in = infos_from_list(obj_->attr("getInputDim")());
    *out = infos_from_list(obj_->attr("getOutputDim")());
    in_ = *in;
    out_ = *out;
    return true;
  }
  bool set_input_info(const TensorsInfo& in, TensorsInfo* out) override {
    py::gil_scoped_acquire g;
    if (!py::hasattr(*obj_, "setInputDim")) return false;
    py::object r = obj_->attr("setInputDim")(list_from_infos(in));
    if (r.is_none()) return false;
    *out = infos_from_list(r);
    in_ = in;
    out_ = *out;
    return true;
  }
  int invoke(const std::vector<MemoryPtr>& in, std::vector<MemoryPtr>* out, InvokeContext&) override {
    std::vector<const void*> ptrs;
    for (auto& m : in) ptrs.push_back(m->map_host());
    py::gil_scoped_acquire g;
    py::list args;
    for (size_t i = 0; i < in.size(); ++i) {
      DType t = i < in_.num_tensors ? in_.at(static_cast<unsigned>(i)).type : DType::UINT8;
      py::dtype dt(np_dtype_name(t));
      size_t n = in[i]->size() / dt.itemsize();
      auto* holder = new MemoryPtr(in[i]);
      py::capsule base(holder, [](void* x) { delete static_cast<MemoryPtr*>(x); });
      args.append(py::array(dt, {static_cast<int64_t>(n)}, {}, ptrs[i], base));
    }
    py::object r;
    try {
      r = obj_->attr("invoke")(args);
    } catch (py::error_already_set& e) {
      NNSX_LOGE("python3", "invoke raised: ", e.what());
      return -1;
    }
    if (r.is_none()) return 1;  // drop
    for (auto it : r) out->push_back(memory_from_python(it));
    return 0;
  }

 private:
  std::shared_ptr<py::object> obj_;
  TensorsInfo in_, out_;
};

class PyFilterFw : public FilterFramework {
 public:
  std::string name() const override { return "python3"; }
  std::unique_ptr<FilterInstance> open(FilterProperties& p) override { return std::make_unique<PyFilter>(p); }
  std::vector<std::string> model_extensions() const override { return {".py"}; }
};

// ------------------------------------------------------------ python3 decoder ----
class PyDecoder : public DecoderInstance {
 public:
  ~PyDecoder() override {
    py::gil_scoped_acquire g;
    obj_.reset();
  }
  bool set_option(int idx, const std::string& v) override {
    if (idx != 0) return true;
    py::gil_scoped_acquire g;
    obj_ = std::make_shared<py::object>(load_script_class(v, "CustomDecoder")());
    return true;
  }
  Caps get_out_caps(const TensorsConfig& config) override {
    if (!obj_) return Caps();
    py::gil_scoped_acquire g;
    py::object r = obj_->attr("getOutCaps")();
    std::string s = py::isinstance<py::bytes>(r) ? std::string(r.cast<py::bytes>()) : r.cast<std::string>();
    while (!s.empty() && s.back() == '\0') s.pop_back();
    Caps c = Caps::from_string(s);
    set_framerate_from_config(c, config);
    return c;
  }
  FlowReturn decode(const TensorsConfig& config, const std::vector<MemoryPtr>& in, Buffer* out,
                    InvokeContext&) override {
    std::vector<const void*> ptrs;
    for (auto& m : in) ptrs.push_back(m->map_host());
    py::gil_scoped_acquire g;
    py::list raw;
    for (size_t i = 0; i < in.size(); ++i) {
      auto* holder = new MemoryPtr(in[i]);
      py::capsule base(holder, [](void* x) { delete static_cast<MemoryPtr*>(x); });
      raw.append(py::array(py::dtype("uint8"), {static_cast<int64_t>(in[i]->size())}, {}, ptrs[i], base));
    }
    py::object r = obj_->attr("decode")(raw, list_from_infos(config.info), config.rate_n, config.rate_d);
    if (r.is_none()) return FlowReturn::ERROR;
    out->mems.push_back(memory_from_python(r));
    return FlowReturn::OK;
  }

 private:
  std::shared_ptr<py::object> obj_;
};

class PyDecoderPlugin : public DecoderSubplugin {
 public:
  std::string name() const override { return "python3"; }
  std::unique_ptr<DecoderInstance> create() override { return std::make_unique<PyDecoder>(); }
};

// ---------------------------------------------------------- python converter ----
class PyConverter : public ConverterSubplugin {
 public:
  explicit PyConverter(const std::string& path) {
    py::gil_scoped_acquire g;
    obj_ = std::make_shared<py::object>(load_script_class(path, "CustomConverter")());
  }
  ~PyConverter() override {
    py::gil_scoped_acquire g;
    obj_.reset();
  }
  std::string name() const override { return "python3"; }
  Caps query_caps() const override { return Caps::Any(); }
  BufferPtr convert(const BufferPtr& in, TensorsConfig* config) override {
    std::vector<const void*> ptrs;
    for (auto& m : in->mems) ptrs.push_back(m->map_host());
    py::gil_scoped_acquire g;
    py::list raw;
    for (size_t i = 0; i < in->mems.size(); ++i) {
      auto* holder = new MemoryPtr(in->mems[i]);
      py::capsule base(holder, [](void* x) { delete static_cast<MemoryPtr*>(x); });
      raw.append(py::array(py::dtype("uint8"), {static_cast<int64_t>(in->mems[i]->size())}, {}, ptrs[i], base));
    }
    py::tuple r = obj_->attr("convert")(raw);
    // (tensors_info, raw_data, rate_n, rate_d)
    TensorsInfo info = infos_from_list(r[0]);
    auto out = make_buffer();
    for (auto it : r[1]) out->mems.push_back(memory_from_python(it));
    config->info = info;
    config->info.format = Format::STATIC;
    config->rate_n = r[2].cast<int>();
    config->rate_d = r[3].cast<int>();
    return out;
  }

 private:
  std::shared_ptr<py::object> obj_;
};

struct PyCallable {
  py::object fn;
  explicit PyCallable(py::object f) : fn(std::move(f)) {}
  ~PyCallable() {
    py::gil_scoped_acquire g;
    fn = py::object();
  }
};

py::list numpy_views(const std::vector<MemoryPtr>& in, const TensorsInfo* info) {
  py::list l;
  for (size_t i = 0; i < in.size(); ++i) {
    DType t = info && i < info->num_tensors ? info->at(static_cast<unsigned>(i)).type : DType::UINT8;
    l.append(memory_to_numpy(in[i], np_dtype_name(t), {}));
  }
  return l;
}

}  // namespace

TensorInfo tensor_info_from_py(py::handle o) { return info_from_shape(o); }

void register_python_bridge(py::module_& m) {
  py::register_exception<TimeoutError>(m, "NnsxTimeout", PyExc_TimeoutError);
  // single-shot (ml_single_*): Python wrapper in nnstreamer_amd/single.py
  py::class_<SingleShot>(m, "SingleShot")
      .def(py::init([](const std::string& fw, std::vector<std::string> models, py::object in, py::object out,
                       const std::string& accl, const std::string& custom, int device) {
             SingleOptions o;
             o.framework = fw;
             o.models = std::move(models);
             if (!in.is_none()) o.input_info = infos_from_list(in);
             if (!out.is_none()) o.output_info = infos_from_list(out);
             o.accelerator = accl;
             o.custom = custom;
             o.device = device;
             py::gil_scoped_release nogil;  // opening may run Python frameworks on other threads
             return std::make_unique<SingleShot>(o);
           }),
           py::arg("framework"), py::arg("models"), py::arg("input") = py::none(), py::arg("output") = py::none(),
           py::arg("accelerator") = "", py::arg("custom") = "", py::arg("device") = -1)
      .def("input_info", [](SingleShot& s) { return list_from_infos(s.input_info()); })
      .def("output_info", [](SingleShot& s) { return list_from_infos(s.output_info()); })
      .def("set_input_info", [](SingleShot& s, py::list in) {
        TensorsInfo i = infos_from_list(in);
        py::gil_scoped_release nogil;
        s.set_input_info(i);
      })
      .def("invoke", [](SingleShot& s, py::list inputs) {
        std::vector<MemoryPtr> in;
        for (auto o : inputs) in.push_back(memory_from_python(o));
        std::vector<MemoryPtr> out;
        TensorsInfo oi;
        {
          py::gil_scoped_release nogil;
          out = s.invoke(in, &oi);
        }
        return py::make_tuple(out, list_from_infos(oi));
      })
      .def("set_timeout", &SingleShot::set_timeout)
      .def("timeout", &SingleShot::timeout)
      .def("framework", &SingleShot::framework)
      .def("device", &SingleShot::device)
      .def("close", [](SingleShot& s) {
        py::gil_scoped_release nogil;
        s.close();
      });

  register_filter_framework(std::make_shared<PyFilterFw>());
  register_decoder(std::make_shared<PyDecoderPlugin>());
  set_script_converter_factory([](const std::string& path) -> std::shared_ptr<ConverterSubplugin> {
    return std::make_shared<PyConverter>(path);
  });

  m.def("register_custom_easy", [](const std::string& name, py::function fn, py::list in, py::list out) {
    auto ref = std::make_shared<PyCallable>(fn);
    TensorsInfo ii = infos_from_list(in), oo = infos_from_list(out);
    return custom_easy_register(
        name,
        [ref](const std::vector<MemoryPtr>& inm, std::vector<MemoryPtr>* outm, const TensorsInfo& iinfo,
              const TensorsInfo&) -> int {
          for (auto& x : inm) x->map_host();
          py::gil_scoped_acquire g;
          try {
            py::object r = ref->fn(numpy_views(inm, &iinfo));
            if (r.is_none()) return 1;
            for (auto it : r) outm->push_back(memory_from_python(it));
            return 0;
          } catch (py::error_already_set& e) {
            NNSX_LOGE("custom-easy", e.what());
            return -1;
          }
        },
        ii, oo);
  });
  m.def("unregister_custom_easy", &custom_easy_unregister);
  m.def("register_decoder_custom", [](const std::string& name, py::function fn) {
    auto ref = std::make_shared<PyCallable>(fn);
    return decoder_custom_register(name, [ref](const std::vector<MemoryPtr>& in, const TensorsConfig& cfg, Buffer* out) {
      for (auto& x : in) x->map_host();
      py::gil_scoped_acquire g;
      py::object r = ref->fn(numpy_views(in, &cfg.info));
      if (r.is_none()) return FlowReturn::ERROR;
      out->mems.push_back(memory_from_python(r));
      return FlowReturn::OK;
    });
  });
  m.def("unregister_decoder_custom", &decoder_custom_unregister);
  m.def("register_converter_custom", [](const std::string& name, py::function fn) {
    auto ref = std::make_shared<PyCallable>(fn);
    return converter_custom_register(name, [ref](const BufferPtr& in, TensorsConfig* cfg) -> BufferPtr {
      for (auto& x : in->mems) x->map_host();
      py::gil_scoped_acquire g;
      py::tuple r = ref->fn(numpy_views(in->mems, nullptr));
      TensorsInfo info = infos_from_list(r[0]);
      auto out = make_buffer();
      for (auto it : r[1]) out->mems.push_back(memory_from_python(it));
      cfg->info = info;
      cfg->info.format = Format::STATIC;
      if (r.size() > 2) {
        cfg->rate_n = r[2].cast<int>();
        cfg->rate_d = r[3].cast<int>();
      }
      return out;
    });
  });
  m.def("unregister_converter_custom", &converter_custom_unregister);
  m.def("register_if_custom", [](const std::string& name, py::function fn) {
    auto ref = std::make_shared<PyCallable>(fn);
    return if_custom_register(name, [ref](const TensorsInfo& info, const std::vector<MemoryPtr>& in) {
      for (auto& x : in) x->map_host();
      py::gil_scoped_acquire g;
      return ref->fn(numpy_views(in, &info)).cast<bool>();
    });
  });
  m.def("unregister_if_custom", &if_custom_unregister);
}

}  // namespace nnsx
