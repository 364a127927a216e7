// gRPC endpoint interface for tensor_src_grpc / tensor_sink_grpc.
//
// The reference links grpc++ (ext/nnstreamer/extra/nnstreamer_grpc_*.cc);
// no C++ gRPC library exists in this image, so the transport is our own
// HTTP/2 (h2c) + HPACK + gRPC-framing implementation (comm/grpc_native.cc),
// wire-compatible with grpc++ / grpcio peers.  The Tensors payloads are the
// protobuf or flatbuf IDL bytes of serial/serial.h; service names / paths:
//   /nnstreamer.<idl>.TensorService/SendTensors  (client -> server stream)
//   /nnstreamer.<idl>.TensorService/RecvTensors  (server -> client stream)
#pragma once

#include <functional>
#include <memory>
#include <string>

namespace nnsx {
namespace comm {

struct GrpcOptions {
  bool server = false;   // run the service (else call it)
  bool sending = false;  // sink side (else source side)
  std::string idl = "protobuf";
  std::string host = "localhost";
  int port = 55115;  // 0: ephemeral (server), read back with port()
  bool blocking = true;
  // largest gRPC message accepted (gRPC's default receive limit is 4 MiB;
  // < 0 = unlimited); a larger one ends its call with RESOURCE_EXHAUSTED
  int64_t max_recv_bytes = 4 << 20;
};

class GrpcEndpoint {
 public:
  virtual ~GrpcEndpoint() = default;
  virtual bool start(std::string* err) = 0;
  virtual bool send(const std::string& msg) = 0;
  // 1: got a message, 0: timeout, -1: stream finished / endpoint stopped
  virtual int recv(std::string* msg, int timeout_ms) = 0;
  virtual void stop() = 0;
  virtual int port() = 0;
};

// the native HTTP/2 endpoint (comm/grpc_native.cc)
std::shared_ptr<GrpcEndpoint> make_native_grpc_endpoint(const GrpcOptions& o);

using GrpcFactory = std::function<std::shared_ptr<GrpcEndpoint>(const GrpcOptions&)>;
void set_grpc_factory(GrpcFactory f);  // replaces the native endpoint (tests, other transports)
GrpcFactory grpc_factory();            // the replacement, else make_native_grpc_endpoint

}  // namespace comm
}  // namespace nnsx
