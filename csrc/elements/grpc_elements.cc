// tensor_sink_grpc / tensor_src_grpc (reference ext/nnstreamer/tensor_sink/
// tensor_sink_grpc.c, tensor_source/tensor_src_grpc.c, extra/
// nnstreamer_grpc_common.cc:83-200).  Properties: silent, server, blocking,
// idl (protobuf | flatbuf), host, port, out.  Defaults as the reference: the
// sink is a client, the source a server, port 55115.  Each buffer is one
// `Tensors` message (serial/serial.h); the source's output caps come from
// downstream (a capsfilter), like the reference push-src.  Transport: the
// native HTTP/2 gRPC endpoint (comm/grpc_native.cc).
#include <atomic>
#include <mutex>

#include "comm/grpc_bridge.h"
#include "core/log.h"
#include "elements/elements.h"
#include "elements/tensor_common.h"
#include "runtime/base.h"
#include "runtime/pipeline.h"
#include "serial/serial.h"

namespace nnsx {

namespace comm {
namespace {
std::mutex g_grpc_mu;
GrpcFactory g_grpc;
}  // namespace
void set_grpc_factory(GrpcFactory f) {
  std::lock_guard<std::mutex> lk(g_grpc_mu);
  g_grpc = std::move(f);
}
GrpcFactory grpc_factory() {
  std::lock_guard<std::mutex> lk(g_grpc_mu);
  if (g_grpc) return g_grpc;
  return make_native_grpc_endpoint;
}
}  // namespace comm

namespace {

serial::Wire wire_of(const std::string& idl) {
  return lower(idl) == "flatbuf" ? serial::Wire::FLATBUF : serial::Wire::PROTOBUF;
}

// shared properties / state of both elements
template <class Base>
class GrpcElement : public Base {
 public:
  using Base::Base;

 protected:
  void add_grpc_props() {
    this->prop_bool("silent", &silent_, "Dont' produce verbose output");
    this->prop_bool("server", &opt_.server, "Specify its working mode either server or client");
    this->prop_bool("blocking", &opt_.blocking, "Specify its working mode either blocking or non-blocking");
    this->prop_string("idl", &opt_.idl, "Specify Interface Description Language (IDL): protobuf or flatbuf");
    this->prop_string("host", &opt_.host, "The hostname to listen as or connect");
    PropSpec p;
    p.name = "port";
    p.type = PropType::INT;
    p.blurb = "The port to listen to (server, 0 = ephemeral, reads back the bound port) or connect (client)";
    p.set = [this](const std::string& v) { opt_.port = static_cast<int>(to_int(v)); };
    p.get = [this] { return std::to_string(ep_ && opt_.server ? ep_->port() : opt_.port); };
    this->add_prop(p);
    this->prop_readonly("out", [this] { return std::to_string(out_.load()); }, "The number of buffers sent / received");
    PropSpec m;
    m.name = "max-recv-message-size";
    m.type = PropType::INT64;
    m.blurb = "nnsx: largest gRPC message accepted in bytes (gRPC's default 4 MiB; -1 = unlimited); a larger one "
              "ends its call with RESOURCE_EXHAUSTED";
    m.default_value = std::to_string(4 << 20);
    m.set = [this](const std::string& v) { opt_.max_recv_bytes = to_int(v); };
    m.get = [this] { return std::to_string(opt_.max_recv_bytes); };
    this->add_prop(m);
  }

  comm::GrpcOptions opt_;
  bool silent_ = true;
  std::atomic<uint64_t> out_{0};
  std::shared_ptr<comm::GrpcEndpoint> ep_;
  TensorsConfig config_;
};

std::shared_ptr<comm::GrpcEndpoint> open_endpoint(Element* e, const comm::GrpcOptions& o) {
  auto f = comm::grpc_factory();
  const std::string idl = lower(o.idl);
  if (idl != "protobuf" && idl != "flatbuf") {
    e->post_error("unknown idl " + o.idl + " (protobuf or flatbuf)");
    return nullptr;
  }
  auto ep = f(o);
  std::string err;
  if (!ep || !ep->start(&err)) {
    e->post_error("gRPC " + std::string(o.server ? "server" : "client") + " start failed: " + err);
    return nullptr;
  }
  return ep;
}

class TensorSinkGrpc : public GrpcElement<BaseSink> {
 public:
  explicit TensorSinkGrpc(const std::string& name)
      : GrpcElement<BaseSink>("tensor_sink_grpc", name, Caps::from_string(tensor_caps_template_all())) {
    opt_.server = false;
    opt_.sending = true;
    add_grpc_props();
  }

 protected:
  bool start() override {
    BaseSink::start();
    out_ = 0;
    ep_ = open_endpoint(this, opt_);
    return ep_ != nullptr;
  }
  bool stop() override {
    if (ep_) ep_->stop();
    ep_.reset();
    return true;
  }
  bool set_caps(const Caps& caps) override {
    return tensor_config_from_caps(caps, &config_);
  }
  FlowReturn render(const BufferPtr& buf) override {
    auto m = serial::encode(wire_of(opt_.idl), config_, buf->mems);
    if (!ep_->send(std::string(static_cast<const char*>(m->data()), m->size()))) {
      post_error("tensor_sink_grpc: send failed");
      return FlowReturn::ERROR;
    }
    ++out_;
    return FlowReturn::OK;
  }
  void on_eos() override {
    if (ep_) ep_->stop();  // finishes the client stream / the server's RecvTensors streams
  }

};

class TensorSrcGrpc : public GrpcElement<BaseSrc> {
 public:
  explicit TensorSrcGrpc(const std::string& name)
      : GrpcElement<BaseSrc>("tensor_src_grpc", name, Caps::from_string(tensor_caps_template_all())) {
    opt_.server = true;
    opt_.sending = false;
    add_grpc_props();
    is_live_ = true;
  }

 protected:
  bool on_start() override {
    out_ = 0;
    ep_ = open_endpoint(this, opt_);
    return ep_ != nullptr;
  }
  void on_stop() override {
    if (ep_) ep_->stop();
  }
  void on_unlock() override {
    if (ep_) ep_->stop();
  }
  bool set_caps(const Caps& caps) override {
    tensor_config_from_caps(caps, &config_);
    return true;
  }
  FlowReturn create(BufferPtr* out) override {
    std::string msg;
    while (true) {
      const int r = ep_->recv(&msg, 100);
      if (r > 0) break;
      if (r < 0 || flushing_.load()) return flushing_.load() ? FlowReturn::FLUSHING : FlowReturn::EOS;
    }
    TensorsConfig c;
    auto b = make_buffer();
    if (!serial::decode(wire_of(opt_.idl), msg.data(), msg.size(), &c, &b->mems)) {
      post_error("tensor_src_grpc: malformed Tensors message");
      return FlowReturn::ERROR;
    }
    // timestamps: frame count scaled by the negotiated framerate (tensor_src_grpc.c:264)
    const uint64_t n = out_++;
    if (config_.rate_n > 0 && config_.rate_d > 0) {
      b->pts = static_cast<int64_t>(n) * kSecond * config_.rate_d / config_.rate_n;
      b->duration = kSecond * config_.rate_d / config_.rate_n;
    } else {
      b->pts = running_time();
    }
    *out = b;
    return FlowReturn::OK;
  }

};

}  // namespace

void register_grpc_elements() {
  register_element("tensor_sink_grpc", "Sink/Network", "Send nnstreamer protocal buffers as a gRPC server/client",
                   [](const std::string& n) { return std::make_unique<TensorSinkGrpc>(n); });
  register_element("tensor_src_grpc", "Source/Network", "Receive nnstreamer protocal buffers as a gRPC server/client",
                   [](const std::string& n) { return std::make_unique<TensorSrcGrpc>(n); });
}

}  // namespace nnsx
