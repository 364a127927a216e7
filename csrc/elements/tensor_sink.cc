// tensor_sink: application sink with `new-data`, `stream-start` and `eos`
// signals (gst/nnstreamer/elements/gsttensor_sink.c:207-229, render :479-533).
// nnsx adds per-buffer latency statistics (source PTS -> render wall clock)
// read by the benchmark harness, and `sync-device` to wait for the device
// payloads before signalling (end-to-end timing).
#include <algorithm>

#include "elements/elements.h"
#include "elements/tensor_common.h"
#include "runtime/base.h"
#include "runtime/pipeline.h"

namespace nnsx {

namespace {

class TensorSink : public BaseSink {
 public:
  explicit TensorSink(const std::string& name)
      : BaseSink("tensor_sink", name,
                 Caps::from_string(tensor_caps_template_all() + "; other/tensors(memory:HIP)")) {
    sink_pad()->set_template_caps(Caps::Any());
    prop_uint("signal-rate", &signal_rate_, "New data signals per second (0 for unlimited, max 500)");
    prop_bool("emit-signal", &emit_signal_, "Emit signal for new data, stream start, eos");
    prop_bool("sync-device", &sync_device_, "nnsx: wait until device-resident payloads are produced before signalling");
    prop_readonly("frames", [this] { return std::to_string(frames_.load()); }, "nnsx: number of rendered frames");
    sync_ = false;
    qos_ = true;
  }

 protected:
  bool start() override {
    BaseSink::start();
    last_emit_ = -1;
    frames_ = 0;
    return true;
  }

  bool event(Event& ev) override {
    if (ev.type == EventType::STREAM_START && emit_signal_) emit("stream-start", SignalArgs{});
    if (ev.type == EventType::EOS && emit_signal_) emit("eos", SignalArgs{});
    if (ev.type == EventType::CAPS) caps_ = ev.caps;
    return true;
  }

  FlowReturn render(const BufferPtr& buf) override {
    if (sync_device_)
      for (auto& m : buf->mems) m->sync_ready();
    ++frames_;
    if (!emit_signal_) return FlowReturn::OK;
    if (signal_rate_ > 0) {
      int64_t now = now_ns();
      int64_t interval = kSecond / std::min(500u, signal_rate_);
      if (last_emit_ >= 0 && now - last_emit_ < interval) return FlowReturn::OK;
      last_emit_ = now;
    }
    SignalArgs a;
    a.buffer = buf;
    a.caps = caps_;
    emit("new-data", a);
    return FlowReturn::OK;
  }

 private:
  unsigned signal_rate_ = 0;
  bool emit_signal_ = true;
  bool sync_device_ = false;
  int64_t last_emit_ = -1;
  std::atomic<int64_t> frames_{0};
  Caps caps_;
};

}  // namespace

void register_tensor_sink() {
  register_element("tensor_sink", "Sink/Tensor", "Sink element to handle tensor stream",
                   [](const std::string& n) { return std::make_unique<TensorSink>(n); });
}

}  // namespace nnsx
