// Python bindings (pybind11) of the nnsx runtime: pipelines, elements,
// buffers/memories (numpy + DLPack zero-copy), signals, appsrc/appsink,
// registration of Python callbacks, and raw kernel entry points for tests.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "comm/group.h"
#include "comm/hpack.h"
#include "comm/mqtt.h"
#include "core/caps.h"
#include "core/log.h"
#include "core/registry.h"
#include "elements/elements.h"
#include "filter/filter.h"
#include "kernels/kernels.h"
#include "runtime/hip_util.h"
#include "runtime/pbtxt.h"
#include "runtime/tracer.h"
#include "runtime/pipeline.h"
#include "runtime/plugin_api.h"

namespace py = pybind11;
using namespace nnsx;

namespace nnsx {
std::string memory_selftest(const std::string& name, int dev);  // runtime/selftest.cc
std::string lower_torchscript_file(const std::string& in, const std::string& out, int device);  // filter/torch_lower.cc
}  // namespace nnsx

namespace nnsx {
void register_python_bridge(py::module_& m);  // python_bridge.cc
py::object memory_to_numpy(const MemoryPtr& m, const std::string& dtype, std::vector<int64_t> shape);
py::capsule memory_to_dlpack(const MemoryPtr& m, const TensorInfo& ti);
MemoryPtr memory_from_python(py::handle obj);
TensorInfo tensor_info_from_py(py::handle o);
}  // namespace nnsx

namespace {

State state_from(const py::object& o) {
  if (py::isinstance<py::str>(o)) {
    std::string s = lower(o.cast<std::string>());
    if (s == "null") return State::NULL_;
    if (s == "ready") return State::READY;
    if (s == "paused") return State::PAUSED;
    if (s == "playing") return State::PLAYING;
    throw Error("unknown state " + s);
  }
  return static_cast<State>(o.cast<int>());
}

// Python object holders released under the GIL from any thread
struct PyRef {
  py::object obj;
  explicit PyRef(py::object o) : obj(std::move(o)) {}
  ~PyRef() {
    py::gil_scoped_acquire g;
    obj = py::object();
  }
};

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "nnsx: MI355X-native NNStreamer-compatible streaming runtime";

  py::register_exception<Error>(m, "NnsxError", PyExc_RuntimeError);

  m.def("version", [] { return std::string(version_string()); });
  m.def("version_tuple", [] {
    unsigned a, b, c;
    version_fetch(&a, &b, &c);
    return py::make_tuple(a, b, c);
  });
  m.def("gpu_count", [] { return hip::device_count(); });
  m.def("memory_selftest", [](const std::string& name, int dev) {
    py::gil_scoped_release nogil;
    return memory_selftest(name, dev);
  }, py::arg("name"), py::arg("device") = 0,
        "Deterministic device-memory lifetime regression case (runtime/selftest.cc): '' = pass");
  m.def("memory_check_enabled", [] { return Memory::check_enabled(); });
  m.def("memory_test_mutation", [](int m) { return Memory::set_test_mutation(m); }, py::arg("mutation"),
        "Lifetime self-tests only: 1 = undo the pageable-H2D use (7ba8684), 2 = undo the mirror hold (ee80b24), "
        "0 = none; returns the previous value");
  m.def("memory_drain_deferred", [] {
    py::gil_scoped_release nogil;
    Memory::drain_deferred();
  });
  m.def("gpu_numa_node", [](int d) { return hip::numa_node(d); }, py::arg("device") = 0);
  m.def("bind_numa", [](int d) { return hip::bind_numa(d); }, py::arg("device"),
        "Pin the process to the GPU's NUMA node (CPUs + preferred memory); call before building pipelines");
  m.def("gpu_arch", [](int d) { return hip::device_arch(d); }, py::arg("device") = 0);
  m.def("set_debug", [](const std::string& s) { log::set_threshold(s); });
  m.def("last_error", [] { return log::last_error(); });
  m.def("list_elements", [] {
    std::vector<std::tuple<std::string, std::string, std::string>> v;
    for (auto& f : list_elements()) v.emplace_back(f.name, f.klass, f.description);
    return v;
  });
  m.def("element_exists", &element_exists);
  m.def("subplugins", [](const std::string& kind) {
    static const std::map<std::string, SubpluginKind> k = {{"filter", SubpluginKind::FILTER},
                                                           {"decoder", SubpluginKind::DECODER},
                                                           {"converter", SubpluginKind::CONVERTER},
                                                           {"trainer", SubpluginKind::TRAINER}};
    auto it = k.find(kind);
    if (it == k.end()) throw Error("unknown sub-plugin kind " + kind);
    ensure_builtin_elements();
    return Registry::get().names(it->second, true);
  });
  m.def("load_subplugin_library", [](const std::string& path) {
    std::string err;
    if (!Registry::get().load_library(path, &err)) throw Error(err);
  });
  m.def("config_dump", [] { return Config::get().dump(); });
  m.def("config_reload", [](const std::string& p) { Config::get().load(p); }, py::arg("path") = "");
  m.def("config_value", [](const std::string& g, const std::string& k, const std::string& d) {
    return Config::get().custom_value(g, k, d);
  }, py::arg("group"), py::arg("key"), py::arg("default") = "");

  // ---------------------------------------------------------- data model ----
  m.def("parse_dimension", [](const std::string& s) {
    Dims d{};
    unsigned r = parse_dimension(s, d);
    return py::make_tuple(r, std::vector<uint32_t>(d.begin(), d.end()));
  });
  m.def("dimension_string", [](std::vector<uint32_t> d, unsigned rank) {
    Dims x{};
    for (size_t i = 0; i < x.size(); ++i) x[i] = i < d.size() ? d[i] : 1;
    return rank ? rank_dimension_string(x, rank) : dimension_string(x);
  }, py::arg("dims"), py::arg("rank") = 0);
  m.def("dimension_string_equal", &dimension_string_equal);
  m.def("dtype_from_string", [](const std::string& s) { return static_cast<int>(dtype_from_string(s)); });
  m.def("dtype_name", [](int t) {
    const char* n = dtype_name(static_cast<DType>(t));
    return n ? std::string(n) : std::string();
  });
  m.def("dtype_size", [](int t) { return dtype_size(static_cast<DType>(t)); });
  m.def("meta_header", [](int type, std::vector<uint32_t> dims, int format, int media, uint32_t nnz) {
    MetaInfo mi;
    mi.type = static_cast<uint32_t>(type);
    for (size_t i = 0; i < dims.size() && i < static_cast<size_t>(kMetaRankLimit); ++i) mi.dimension[i] = dims[i];
    mi.format = static_cast<uint32_t>(format);
    mi.media_type = static_cast<uint32_t>(media);
    mi.nnz = nnz;
    std::string out(kMetaHeaderSize, '\0');
    mi.write(out.data());
    return py::bytes(out);
  }, py::arg("type"), py::arg("dims"), py::arg("format") = 1, py::arg("media") = 4, py::arg("nnz") = 0);
  m.def("parse_meta_header", [](py::bytes b) {
    std::string s = b;
    MetaInfo mi;
    bool ok = MetaInfo::parse(s.data(), s.size(), &mi);
    py::dict d;
    d["valid"] = ok;
    d["version"] = mi.version;
    d["type"] = mi.type;
    d["dims"] = std::vector<uint32_t>(mi.dimension, mi.dimension + kMetaRankLimit);
    d["format"] = mi.format;
    d["media_type"] = mi.media_type;
    d["nnz"] = mi.nnz;
    d["header_size"] = mi.header_size();
    d["data_size"] = mi.data_size();
    return d;
  });

  py::class_<Caps>(m, "Caps")
      .def(py::init([](const std::string& s) { return Caps::from_string(s); }))
      .def("__str__", &Caps::to_string)
      .def("__repr__", [](const Caps& c) { return "<Caps " + c.to_string() + ">"; })
      .def("intersect", &Caps::intersect)
      .def("can_intersect", &Caps::can_intersect)
      .def("fixate", &Caps::fixate)
      .def("is_fixed", &Caps::is_fixed)
      .def("is_any", &Caps::is_any)
      .def("is_empty", &Caps::is_empty)
      .def("__len__", &Caps::size)
      .def("structure_name", [](const Caps& c, size_t i) { return c.at(i).name(); })
      .def("get", [](const Caps& c, const std::string& field, size_t i) -> py::object {
        if (i >= c.size()) return py::none();
        const Value* v = c.at(i).get(field);
        if (!v) return py::none();
        switch (v->kind) {
          case Value::Kind::INT: return py::int_(v->i);
          case Value::Kind::STRING: return py::str(v->s);
          case Value::Kind::BOOL: return py::bool_(v->b);
          case Value::Kind::DOUBLE: return py::float_(v->d);
          case Value::Kind::FRACTION: return py::make_tuple(v->i, v->i2);
          default: return py::str(v->to_string());
        }
      }, py::arg("field"), py::arg("index") = 0)
      .def("tensors_config", [](const Caps& c) -> py::object {
        TensorsConfig cfg;
        if (c.size() == 0 || !config_from_structure(c.at(0), &cfg)) return py::none();
        py::dict d;
        d["format"] = format_name(cfg.info.format) ? format_name(cfg.info.format) : "";
        d["num_tensors"] = cfg.info.num_tensors;
        d["dimensions"] = cfg.info.dimensions_string();
        d["types"] = cfg.info.types_string();
        d["rate"] = py::make_tuple(cfg.rate_n, cfg.rate_d);
        return d;
      });

  // ------------------------------------------------------------- memory ----
  py::class_<Memory, MemoryPtr>(m, "Memory")
      .def_property_readonly("size", &Memory::size)
      .def_property_readonly("on_device", &Memory::on_device)
      .def_property_readonly("device", &Memory::device)
      .def_property_readonly("place", [](const Memory& mm) {
        return mm.place() == MemPlace::DEVICE ? "device" : (mm.place() == MemPlace::PINNED ? "pinned" : "host");
      })
      .def_property_readonly("data_ptr", [](const Memory& mm) { return reinterpret_cast<uintptr_t>(mm.data()); })
      .def_property_readonly("has_meta", &Memory::has_meta)
      .def("bytes", [](MemoryPtr mm) {
        const void* p;
        {
          py::gil_scoped_release r;
          p = mm->map_host();
        }
        return py::bytes(static_cast<const char*>(p), mm->size());
      })
      .def("serialize", [](MemoryPtr mm) {
        auto v = serialize_with_header(mm);
        return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
      })
      .def("numpy", &memory_to_numpy, py::arg("dtype") = "uint8", py::arg("shape") = std::vector<int64_t>{})
      .def("dlpack", [](MemoryPtr mm, const std::string& dtype, std::vector<uint32_t> dims) {
        TensorInfo ti;
        ti.type = dtype_from_string(dtype);
        ti.dim.fill(1);
        for (size_t i = 0; i < dims.size() && i < 8; ++i) ti.dim[i] = dims[i];
        return memory_to_dlpack(mm, ti);
      }, py::arg("dtype"), py::arg("dims"))
      .def("sync", [](MemoryPtr mm) {
        py::gil_scoped_release r;
        mm->sync_ready();
      })
      .def("meta", [](MemoryPtr mm) -> py::object {
        if (!mm->has_meta()) return py::none();
        const MetaInfo& mi = mm->meta();
        py::dict d;
        d["type"] = mi.type;
        d["dims"] = std::vector<uint32_t>(mi.dimension, mi.dimension + kMetaRankLimit);
        d["format"] = mi.format;
        d["media_type"] = mi.media_type;
        return d;
      });
  m.def("memory_from", &memory_from_python, "Wrap/copy a numpy array, bytes or torch tensor into a Memory");

  py::class_<Buffer, BufferPtr>(m, "Buffer")
      .def(py::init([] { return make_buffer(); }))
      .def_readwrite("pts", &Buffer::pts)
      .def_readwrite("dts", &Buffer::dts)
      .def_readwrite("duration", &Buffer::duration)
      .def_readwrite("offset", &Buffer::offset)
      .def_property("client_id", [](const Buffer& b) { return b.meta.client_id; },
                    [](Buffer& b, int64_t v) { b.meta.client_id = v; })
      .def_property_readonly("n_memory", &Buffer::n_memory)
      .def("memory", [](Buffer& b, size_t i) { return b.mems.at(i); })
      .def_property_readonly("memories", [](Buffer& b) { return b.mems; })
      .def("append", [](Buffer& b, py::handle o) { b.mems.push_back(memory_from_python(o)); })
      .def_property_readonly("size", &Buffer::total_size);

  // ------------------------------------------------------------ element ----
  py::class_<Element>(m, "Element")
      .def_property_readonly("name", &Element::name)
      .def_property_readonly("factory", &Element::factory)
      .def("set_property", [](Element& e, const std::string& k, py::object v) {
        std::string s;
        if (py::isinstance<py::bool_>(v))
          s = v.cast<bool>() ? "true" : "false";
        else if (py::isinstance<py::str>(v))
          s = v.cast<std::string>();
        else
          s = py::str(v).cast<std::string>();
        e.set_property(k, s);
      })
      .def("get_property", [](Element& e, const std::string& k) -> py::object {
        const PropSpec* p = e.find_property(k);
        if (!p) throw Error("no property " + k);
        std::string v = e.get_property(k);
        switch (p->type) {
          case PropType::BOOL: return py::bool_(to_bool(v));
          case PropType::INT:
          case PropType::UINT:
          case PropType::INT64:
          case PropType::UINT64: return py::int_(to_int(v));
          case PropType::DOUBLE: return py::float_(to_double(v));
          default: return py::str(v);
        }
      })
      .def("query_latency", [](Element& e) -> py::object {
        // latency query from this element's first sink pad upstream (GST_QUERY_LATENCY)
        Pad* sp = e.sink_pad(0);
        if (!sp) return py::none();
        bool live = false;
        int64_t mn = 0, mx = -1;
        bool ok;
        {
          py::gil_scoped_release r;
          ok = e.query_latency(sp, &live, &mn, &mx);
        }
        if (!ok) return py::none();
        return py::make_tuple(live, mn, mx);
      }, "Latency query from this element's sink pad: (live, min_ns, max_ns) or None")
      .def("properties", [](Element& e) {
        std::vector<std::tuple<std::string, std::string, std::string>> v;
        for (auto& p : e.properties()) v.emplace_back(p.name, p.blurb, p.default_value);
        return v;
      })
      .def("connect", [](Element& e, const std::string& sig, py::function cb) {
        auto ref = std::make_shared<PyRef>(cb);
        return e.connect(sig, [ref](Element* el, const SignalArgs& a) {
          py::gil_scoped_acquire g;
          try {
            if (a.buffer)
              ref->obj(a.buffer);
            else
              ref->obj();
          } catch (py::error_already_set& err) {
            NNSX_LOGE(el->name(), "python signal handler raised: ", err.what());
          }
        });
      })
      .def("disconnect", &Element::disconnect)
      .def("pad_names", [](Element& e) {
        std::vector<std::string> v;
        for (auto& p : e.pads()) v.push_back(p->name());
        return v;
      })
      .def("pad_caps", [](Element& e, const std::string& pad) -> py::object {
        Pad* p = e.get_pad(pad);
        if (!p || !p->has_current_caps()) return py::none();
        return py::cast(p->current_caps());
      })
      .def("send_event", [](Element& e, const std::string& name, py::dict fields, bool upstream) {
        Structure s(name);
        for (auto kv : fields) {
          std::string k = py::str(kv.first);
          py::handle v = kv.second;
          if (py::isinstance<py::bool_>(v)) s.set(k, Value::Bool(v.cast<bool>()));
          else if (py::isinstance<py::int_>(v)) s.set(k, Value::Int(v.cast<int64_t>()));
          else if (py::isinstance<py::float_>(v)) s.set(k, Value::Double(v.cast<double>()));
          else s.set(k, Value::String(py::str(v)));
        }
        Event ev = Event::make_custom(upstream ? EventType::CUSTOM_UPSTREAM : EventType::CUSTOM_DOWNSTREAM, s);
        py::gil_scoped_release r;
        if (upstream) {
          for (Pad* p : e.src_pads()) p->push_event(ev);
        } else {
          for (Pad* p : e.sink_pads())
            if (p->peer()) p->peer()->parent()->src_event(p->peer(), ev);
          // downstream custom events injected at this element's src
          for (Pad* p : e.src_pads()) p->push_event(ev);
        }
      }, py::arg("name"), py::arg("fields") = py::dict(), py::arg("upstream") = false)
      // appsrc
      .def("push_buffer", [](Element& e, py::object data, int64_t pts, int64_t duration) {
        auto* a = dynamic_cast<AppSrcIface*>(&e);
        if (!a) throw Error(e.name() + " is not an appsrc");
        BufferPtr b;
        if (py::isinstance<Buffer>(data)) {
          b = data.cast<BufferPtr>();
        } else {
          b = make_buffer();
          if (py::isinstance<py::list>(data) || py::isinstance<py::tuple>(data)) {
            for (auto it : data) b->mems.push_back(memory_from_python(it));
          } else {
            b->mems.push_back(memory_from_python(data));
          }
          b->pts = pts;
          b->duration = duration;
        }
        py::gil_scoped_release r;
        return static_cast<int>(a->push(b));
      }, py::arg("data"), py::arg("pts") = -1, py::arg("duration") = -1)
      .def("end_of_stream", [](Element& e) {
        auto* a = dynamic_cast<AppSrcIface*>(&e);
        if (!a) throw Error(e.name() + " is not an appsrc");
        return static_cast<int>(a->end_of_stream());
      })
      // appsink
      .def("pull", [](Element& e, double timeout_s) -> py::object {
        auto* a = dynamic_cast<AppSinkIface*>(&e);
        if (!a) throw Error(e.name() + " is not an appsink");
        BufferPtr b;
        {
          py::gil_scoped_release r;
          b = a->pull(timeout_s < 0 ? -1 : static_cast<int64_t>(timeout_s * 1e9));
        }
        if (!b) return py::none();
        return py::cast(b);
      }, py::arg("timeout") = -1.0)
      .def("is_eos", [](Element& e) {
        auto* a = dynamic_cast<AppSinkIface*>(&e);
        if (!a) throw Error(e.name() + " is not an appsink");
        return a->is_eos();
      });

  py::class_<Pipeline, Element>(m, "Pipeline")
      .def(py::init<const std::string&>(), py::arg("name") = "pipeline0")
      .def("get_by_name", &Pipeline::get_by_name, py::return_value_policy::reference_internal)
      .def("elements", [](Pipeline& p) {
        std::vector<Element*> v = p.elements();
        return v;
      }, py::return_value_policy::reference_internal)
      .def("add", [](Pipeline& p, const std::string& factory, const std::string& name) {
        return p.add(make_element(factory, name));
      }, py::arg("factory"), py::arg("name") = "", py::return_value_policy::reference_internal)
      .def("link", [](Pipeline& p, const std::string& a, const std::string& b, const std::string& caps) {
        auto parse = [](const std::string& s, std::string* el, std::string* pad) {
          auto dot = s.find('.');
          *el = dot == std::string::npos ? s : s.substr(0, dot);
          *pad = dot == std::string::npos ? "" : s.substr(dot + 1);
        };
        std::string ea, pa, eb, pb;
        parse(a, &ea, &pa);
        parse(b, &eb, &pb);
        Element* x = p.get_by_name(ea);
        Element* y = p.get_by_name(eb);
        if (!x || !y) throw Error("link: unknown element");
        if (!p.link(x, pa, y, pb, caps)) throw Error("link failed: " + a + " -> " + b);
      }, py::arg("src"), py::arg("sink"), py::arg("caps") = "")
      .def("set_state", [](Pipeline& p, py::object s) {
        State st = state_from(s);
        py::gil_scoped_release r;
        return p.set_state(st);
      })
      .def("get_state", [](Pipeline& p) { return std::string(state_name(p.get_state())); })
      .def("run", [](Pipeline& p, double timeout_s) {
        std::string err;
        bool ok;
        {
          py::gil_scoped_release r;
          ok = p.run_until_eos(timeout_s < 0 ? -1 : static_cast<int64_t>(timeout_s * 1e9), &err);
        }
        if (!ok) throw Error("pipeline did not reach EOS: " + err);
        return true;
      }, py::arg("timeout") = -1.0)
      .def("wait", [](Pipeline& p, double timeout_s) -> py::object {
        Message msg;
        bool got;
        {
          py::gil_scoped_release r;
          got = p.bus().pop(&msg, timeout_s < 0 ? -1 : static_cast<int64_t>(timeout_s * 1e9),
                            {MessageType::EOS, MessageType::ERROR});
        }
        if (!got) return py::none();
        return py::make_tuple(message_type_name(msg.type), msg.src, msg.text);
      }, py::arg("timeout") = -1.0)
      .def("send_eos", [](Pipeline& p) {
        py::gil_scoped_release r;
        p.send_eos();
      })
      .def("messages", [](Pipeline& p) {
        std::vector<std::tuple<std::string, std::string, std::string>> v;
        for (auto& msg : p.bus().drain()) v.emplace_back(message_type_name(msg.type), msg.src, msg.text);
        return v;
      })
      .def("dot", &Pipeline::dot)
      .def("running_time", [](Pipeline& p) { return now_ns() - p.base_time_ns(); },
           "Pipeline running time (ns): the clock buffer PTS are compared against")
      .def("stop", [](Pipeline& p) {
        py::gil_scoped_release r;
        p.set_state(State::NULL_);
      });

  // in-process MQTT broker (mqttsink / mqttsrc / connect-type=HYBRID without an external broker)
  // rank groups (comm/group.h): the multi-GPU data plane the among-device
  // elements use, for direct tests of each collective and of p2p
  py::class_<comm::Packet>(m, "Packet")
      .def(py::init([](py::list blobs, int64_t pts, bool eos, const std::string& caps) {
             comm::Packet p;
             for (auto b : blobs) p.blobs.push_back(memory_from_python(b));
             p.pts = pts;
             p.eos = eos;
             p.caps = caps;
             return p;
           }),
           py::arg("blobs") = py::list(), py::arg("pts") = -1, py::arg("eos") = false, py::arg("caps") = "")
      .def_readonly("src", &comm::Packet::src)
      .def_readonly("pts", &comm::Packet::pts)
      .def_readonly("eos", &comm::Packet::eos)
      .def_readonly("caps", &comm::Packet::caps)
      .def_property_readonly("blobs", [](const comm::Packet& p) { return p.blobs; });
  py::class_<comm::Group, std::shared_ptr<comm::Group>>(m, "Group")
      .def(py::init([](const std::string& name, int rank, int world, const std::string& store, int device,
                       const std::string& backend, int timeout_ms) {
             comm::GroupSpec s;
             s.name = name;
             s.rank = rank;
             s.world = world;
             s.store = store;
             s.device = device;
             s.backend = backend;
             s.timeout_ms = timeout_ms;
             std::string err;
             std::shared_ptr<comm::Group> g;
             {
               py::gil_scoped_release r;
               g = comm::Group::open(s, &err);
             }
             if (!g) throw Error("Group: " + err);
             return g;
           }),
           py::arg("name"), py::arg("rank"), py::arg("world"), py::arg("store"), py::arg("device") = -1,
           py::arg("backend") = "auto", py::arg("timeout_ms") = 60000)
      .def_property_readonly("rank", &comm::Group::rank)
      .def_property_readonly("size", &comm::Group::size)
      .def_property_readonly("backend", [](const comm::Group& g) { return std::string(g.backend_name()); })
      .def_property_readonly("bytes_sent", &comm::Group::bytes_sent)
      .def_property_readonly("bytes_received", &comm::Group::bytes_received)
      .def("allgather", [](comm::Group& g, const comm::Packet& mine) {
        std::vector<comm::Packet> all;
        MemoryPtr stacked;
        std::string err;
        bool ok;
        {
          py::gil_scoped_release r;
          ok = g.allgather(mine, &all, &err, &stacked);
        }
        if (!ok) throw Error("allgather: " + err);
        return py::make_tuple(all, stacked);
      }, "-> (per-member packets, stacked buffer or None)")
      .def("broadcast", [](comm::Group& g, int root, comm::Packet pkt) {
        std::string err;
        bool ok;
        {
          py::gil_scoped_release r;
          ok = g.broadcast(root, &pkt, &err);
        }
        if (!ok) throw Error("broadcast: " + err);
        return pkt;
      })
      .def("scatter", [](comm::Group& g, int root, std::vector<comm::Packet> parts) {
        comm::Packet mine;
        std::string err;
        bool ok;
        {
          py::gil_scoped_release r;
          ok = g.scatter(root, g.rank() == root ? &parts : nullptr, &mine, &err);
        }
        if (!ok) throw Error("scatter: " + err);
        return mine;
      }, py::arg("root"), py::arg("parts") = std::vector<comm::Packet>())
      .def("send", [](comm::Group& g, int peer, const comm::Packet& p) {
        std::string err;
        bool ok;
        {
          py::gil_scoped_release r;
          ok = g.send(peer, p, &err);
        }
        if (!ok) throw Error("send: " + err);
      })
      .def("recv", [](comm::Group& g, int timeout_ms) -> py::object {
        comm::Packet p;
        bool to = false, ok;
        std::string err;
        {
          py::gil_scoped_release r;
          ok = g.recv(&p, timeout_ms, &to, &err);
        }
        if (!ok) {
          if (to) return py::none();
          throw Error("recv: " + err);
        }
        return py::cast(p);
      }, py::arg("timeout_ms") = 60000);

  py::class_<comm::MqttBroker, std::shared_ptr<comm::MqttBroker>>(m, "MqttBroker")
      .def(py::init([](int port, const std::string& host) {
             std::string err;
             auto b = comm::mqtt_broker_start(host, port, &err);
             if (!b) throw Error(err);
             return b;
           }),
           py::arg("port") = 0, py::arg("host") = "127.0.0.1")
      .def_property_readonly("port", &comm::MqttBroker::port)
      .def_property_readonly("clients", &comm::MqttBroker::clients)
      .def_property_readonly("messages", &comm::MqttBroker::messages)
      .def("stop", [](comm::MqttBroker& b) {
        py::gil_scoped_release r;
        b.stop();
      });

  m.def("parse_launch", [](const std::string& d) { return parse_launch(d); });
  m.def("lower_torchscript", [](const std::string& in, const std::string& out, int device) {
    py::gil_scoped_release r;
    return lower_torchscript_file(in, out, device);
  }, py::arg("path"), py::arg("out"), py::arg("device") = -1,
        "Freeze and lower a TorchScript file onto the nnsx kernels (what tensor_filter framework=pytorch does at "
        "load); saves the result and returns the report");
  m.def("tracer_enable", [](const std::string& spec) { trace::enable(spec); }, py::arg("spec"),
        "Enable built-in tracers: 'proctime;interlatency;framerate;roctx' ('' disables)");
  m.def("tracer_reset", [] { trace::reset(); });
  m.def("tracer_report", [] { return trace::report_json(); }, "Tracer statistics as a JSON string");
  m.def("to_pbtxt", [](const Pipeline& p, bool with_options) { return pipeline_to_pbtxt(p, with_options); },
        py::arg("pipeline"), py::arg("with_options") = false,
        "MediaPipe-style pbtxt of a pipeline (tools/development/parser/convert.c)");
  m.def("pbtxt_to_launch", [](const std::string& t) {
    std::string err;
    std::string d = pbtxt_to_launch(t, &err);
    if (d.empty()) throw Error(err);
    return d;
  }, py::arg("pbtxt"), "Launch description of a pbtxt graph (the reverse conversion)");
  // the reference's >16-tensor buffer form (GstTensorExtraInfo in the 16th memory)
  m.def("pack_extra", [](py::list arrays, std::vector<std::string> dims, std::vector<std::string> types) {
    std::vector<MemoryPtr> mems;
    for (auto a : arrays) mems.push_back(memory_from_python(a));
    TensorsInfo info;
    info.num_tensors = static_cast<unsigned>(mems.size());
    for (size_t i = 0; i < mems.size() && i < dims.size() && i < types.size(); ++i) {
      parse_dimension(dims[i], info.at(static_cast<unsigned>(i)).dim);
      info.at(static_cast<unsigned>(i)).type = dtype_from_string(types[i]);
    }
    return pack_extra(mems, info);
  }, "Pack >16 tensors into 16 memories (reference GstTensorExtraInfo layout)");
  m.def("unpack_extra", [](std::vector<MemoryPtr> mems) {
    TensorsInfo info;
    info.num_tensors = static_cast<unsigned>(mems.size());
    auto out = unpack_extra(mems, &info);
    std::vector<std::pair<std::string, std::string>> ti;
    for (size_t i = mems.size(); i < out.size(); ++i) {
      const auto& t = info.at(static_cast<unsigned>(i));
      std::string d;
      for (int k = 0; k < kRankLimit; ++k) d += (k ? ":" : "") + std::to_string(t.dim[k]);
      ti.emplace_back(d, dtype_name(t.type) ? dtype_name(t.type) : "");
    }
    return py::make_tuple(out, ti);
  }, "Inverse of pack_extra: one memory per tensor, plus (dims, type) of the extra ones");
  // HPACK codec of the native gRPC transport (comm/hpack.h), for its tests
  m.def("hpack_huffman_encode", [](const std::string& s) { return py::bytes(hpack::huffman_encode(s)); });
  m.def("hpack_huffman_decode", [](const py::bytes& b) {
    const std::string in = b;
    std::string out;
    if (!hpack::huffman_decode(reinterpret_cast<const uint8_t*>(in.data()), in.size(), &out))
      throw std::invalid_argument("invalid HPACK Huffman string");
    return out;
  });
  m.def("hpack_decode_blocks", [](const std::vector<py::bytes>& blocks) {
    hpack::Decoder d;  // one connection's decoder: the dynamic table carries over between blocks
    std::vector<hpack::Headers> out;
    for (const auto& b : blocks) {
      const std::string in = b;
      hpack::Headers h;
      std::string err;
      if (!d.decode(reinterpret_cast<const uint8_t*>(in.data()), in.size(), &h, &err)) throw std::invalid_argument(err);
      out.push_back(std::move(h));
    }
    return out;
  });
  m.def("make_element", [](const std::string& f, const std::string& n) { return make_element(f, n); },
        py::arg("factory"), py::arg("name") = "");

  // ---------------------------------------------------------- kernels ----
  auto k = m.def_submodule("kernels", "Raw CDNA4 kernel entry points (device pointers as ints)");
  k.def("arith", [](uintptr_t in, int in_t, uintptr_t out, int out_t, uint64_t n,
                    std::vector<std::tuple<int, double, int64_t, double, int>> ops, uint64_t ch_size,
                    uint32_t ch_count, uintptr_t stream) {
    kernels::ArithParams p;
    p.nops = static_cast<int>(ops.size());
    for (size_t i = 0; i < ops.size() && i < static_cast<size_t>(kernels::kMaxArithOps); ++i) {
      auto& o = ops[i];
      p.ops[i] = kernels::ArithOp{std::get<0>(o), std::get<1>(o), std::get<2>(o), std::get<3>(o), std::get<4>(o)};
    }
    p.ch_size = ch_size;
    p.ch_count = ch_count;
    kernels::arith(reinterpret_cast<const void*>(in), static_cast<DType>(in_t), reinterpret_cast<void*>(out),
                   static_cast<DType>(out_t), n, p, reinterpret_cast<hipStream_t>(stream));
    hip::check(hipGetLastError(), "arith");
  });
  k.def("permute", [](uintptr_t in, uintptr_t out, size_t es, std::vector<uint32_t> dims, std::vector<int> perm,
                      uintptr_t stream) {
    uint32_t d[8];
    int pm[8];
    for (int i = 0; i < 8; ++i) {
      d[i] = i < static_cast<int>(dims.size()) ? dims[i] : 1;
      pm[i] = i < static_cast<int>(perm.size()) ? perm[i] : i;
    }
    kernels::permute(reinterpret_cast<const void*>(in), reinterpret_cast<void*>(out), es, d, pm,
                     reinterpret_cast<hipStream_t>(stream));
    hip::check(hipGetLastError(), "permute");
  });
  k.def("argmax_rows", [](uintptr_t in, int t, uint64_t n, uint32_t batch, uintptr_t out, uintptr_t stream) {
    kernels::argmax_rows(reinterpret_cast<const void*>(in), static_cast<DType>(t), n, batch,
                         reinterpret_cast<int32_t*>(out), reinterpret_cast<hipStream_t>(stream));
    hip::check(hipGetLastError(), "argmax");
  });
  k.def("stand", [](uintptr_t in, int in_t, uintptr_t out, int out_t, uint64_t n, uint32_t ch, int mode, bool per_ch,
                    uintptr_t ws, uintptr_t stream) {
    kernels::stand(reinterpret_cast<const void*>(in), static_cast<DType>(in_t), reinterpret_cast<void*>(out),
                   static_cast<DType>(out_t), n, ch, mode, per_ch, reinterpret_cast<void*>(ws),
                   reinterpret_cast<hipStream_t>(stream));
    hip::check(hipGetLastError(), "stand");
  });
  k.def("stand_workspace_bytes", &kernels::stand_workspace_bytes);

  register_python_bridge(m);
}
