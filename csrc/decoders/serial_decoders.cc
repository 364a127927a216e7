// tensor_decoder mode=protobuf|flatbuf|flexbuf and the matching
// tensor_converter sub-plugins (reference ext/nnstreamer/tensor_decoder/
// tensordec-{protobuf,flatbuf,flexbuf}.cc, tensor_converter/
// tensor_converter_{protobuf,flatbuf,flexbuf}.cc).  Host-only: the frame is
// serialized into one application buffer (serial/serial.h).
#include "decoders/decoders.h"
#include "serial/serial.h"

namespace nnsx {

namespace {

class WireDecoder : public DecoderInstance {
 public:
  explicit WireDecoder(serial::Wire w) : w_(w) {}
  Caps get_out_caps(const TensorsConfig& config) override {
    Caps c = Caps::from_string(serial::wire_caps(w_));
    set_framerate_from_config(c, config);
    return c;
  }
  FlowReturn decode(const TensorsConfig& config, const std::vector<MemoryPtr>& in, Buffer* out,
                    InvokeContext&) override {
    if (in.empty() || in.size() > static_cast<size_t>(kSizeLimit)) return FlowReturn::ERROR;
    out->mems.push_back(serial::encode(w_, config, in));
    return FlowReturn::OK;
  }

 private:
  serial::Wire w_;
};

class WireDecoderPlugin : public DecoderSubplugin {
 public:
  explicit WireDecoderPlugin(serial::Wire w) : w_(w) {}
  std::string name() const override { return serial::wire_name(w_); }
  std::unique_ptr<DecoderInstance> create() override { return std::make_unique<WireDecoder>(w_); }

 private:
  serial::Wire w_;
};

class WireConverter : public ConverterSubplugin {
 public:
  explicit WireConverter(serial::Wire w) : w_(w) {}
  std::string name() const override { return serial::wire_name(w_); }
  Caps query_caps() const override { return Caps::from_string(serial::wire_caps(w_)); }
  BufferPtr convert(const BufferPtr& in, TensorsConfig* config) override {
    if (in->mems.empty()) return nullptr;
    const MemoryPtr& m = in->mems[0];
    TensorsConfig c;
    std::vector<MemoryPtr> tensors;
    if (!serial::decode(w_, m->map_host(), m->size(), &c, &tensors)) return nullptr;
    auto out = make_buffer();
    out->mems = std::move(tensors);
    *config = c;
    return out;
  }

 private:
  serial::Wire w_;
};

}  // namespace

void register_serial_decoders() {
  for (auto w : {serial::Wire::PROTOBUF, serial::Wire::FLATBUF, serial::Wire::FLEXBUF}) {
    register_decoder(std::make_shared<WireDecoderPlugin>(w));
    register_converter(std::make_shared<WireConverter>(w));
  }
}

}  // namespace nnsx
