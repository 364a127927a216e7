// tensor_sink: application sink with `new-data`, `stream-start` and `eos`
// signals (gst/nnstreamer/elements/gsttensor_sink.c:207-229, render :479-533).
// nnsx adds per-buffer latency statistics (source PTS -> render wall clock)
// (`stats-every=N`: every N-th buffer's arrival on the monotonic clock and its
// source-PTS -> render latency, read back through the `stats` property without
// a Python callback per frame), and `sync-device` to wait for the device
// payloads before signalling (end-to-end timing).
#include <algorithm>
#include <mutex>
#include <vector>

#include <rocprofiler-sdk-roctx/roctx.h>

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
    prop_uint("stats-every", &stats_every_, "nnsx: record every N-th buffer's arrival time and latency (0 = off)");
    PropSpec mk;
    mk.name = "roctx-marks";
    mk.blurb = "nnsx: comma-separated buffer counts at whose arrival a roctx mark 'nnsx:<name>:<count>' is emitted "
               "(profilers window their kernel statistics to a timed region with them)";
    mk.set = [this](const std::string& v) {
      marks_.clear();
      for (auto& t : split(v, ','))
        if (!strip(t).empty()) marks_.push_back(std::stoll(strip(t)));
    };
    mk.get = [this] {
      std::string r;
      for (int64_t m : marks_) r += (r.empty() ? "" : ",") + std::to_string(m);
      return r;
    };
    add_prop(mk);
    prop_readonly(
        "stats",
        [this] {
          std::lock_guard<std::mutex> lk(stats_mu_);
          std::string r;
          for (auto& e : stats_) r += std::to_string(e.first) + ":" + std::to_string(e.second) + ",";
          return r;
        },
        "nnsx: 'monotonic_ns:latency_ns,' per recorded buffer (latency -1 without a PTS)");
    sync_ = false;
    qos_ = true;
  }

 protected:
  bool start() override {
    BaseSink::start();
    last_emit_ = -1;
    frames_ = 0;
    std::lock_guard<std::mutex> lk(stats_mu_);
    stats_.clear();
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
    const int64_t n = ++frames_;
    for (int64_t m : marks_)
      if (m == n) roctxMarkA(strfmt("nnsx:", name(), ":", n).c_str());
    if (stats_every_ > 0 && n % stats_every_ == 0) {
      const int64_t lat = buf->pts >= 0 ? running_time() - buf->pts : -1;
      std::lock_guard<std::mutex> lk(stats_mu_);
      stats_.emplace_back(now_ns(), lat);
    }
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
  unsigned stats_every_ = 0;
  std::vector<int64_t> marks_;  // roctx-marks
  std::mutex stats_mu_;
  std::vector<std::pair<int64_t, int64_t>> stats_;
  Caps caps_;
};

}  // namespace

void register_tensor_sink() {
  register_element("tensor_sink", "Sink/Tensor", "Sink element to handle tensor stream",
                   [](const std::string& n) { return std::make_unique<TensorSink>(n); });
}

}  // namespace nnsx
