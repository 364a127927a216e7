// Built-in utility elements the reference pipelines rely on from stock
// GStreamer (queue, tee, capsfilter, identity, fakesrc/fakesink, appsrc/
// appsink, videotestsrc, audiotestsrc, filesrc/filesink, multifilesrc/
// multifilesink, videoconvert).  GStreamer is absent from this image, so nnsx
// ships its own.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>
#include <deque>
#include <fstream>
#include <random>

#include "comm/shm.h"
#include "core/log.h"
#include "elements/elements.h"
#include "runtime/base.h"
#include "runtime/hip_util.h"
#include "runtime/pipeline.h"
#include "runtime/video.h"

namespace nnsx {

namespace {

std::string format_location(const std::string& pattern, int64_t index) {
  char buf[4096];
  if (pattern.find('%') == std::string::npos) return pattern;
  snprintf(buf, sizeof(buf), pattern.c_str(), static_cast<int>(index));
  return buf;
}

// ------------------------------------------------------------------ queue ----
class Queue : public Element {
 public:
  explicit Queue(const std::string& name) : Element("queue", name) {
    add_template("sink", PadDirection::SINK, PadPresence::ALWAYS, Caps::Any());
    add_template("src", PadDirection::SRC, PadPresence::ALWAYS, Caps::Any());
    prop_uint("max-size-buffers", &max_buffers_, "Max. number of buffers in the queue (0=disable)");
    prop_uint("max-size-bytes", &max_bytes_, "Max. amount of data in the queue (bytes, 0=disable)");
    prop_int("max-size-time", &max_time_, "Max. amount of data in the queue (in ns, 0=disable)");
    prop_enum("leaky", &leaky_, {"no", "upstream", "downstream"}, "Where the queue leaks, if at all");
    prop_readonly("current-level-buffers", [this] {
      std::lock_guard<std::mutex> lk(mu_);
      return std::to_string(nbuf_);
    }, "Current number of buffers in the queue");
  }

  bool start() override {
    std::lock_guard<std::mutex> lk(mu_);
    q_.clear();
    nbuf_ = 0;
    bytes_ = 0;
    flushing_local_ = false;
    last_ret_ = FlowReturn::OK;
    task_ = std::make_unique<Task>([this] { return loop(); });
    task_->start();
    return true;
  }
  void unlock() override {
    {
      std::lock_guard<std::mutex> lk(mu_);
      flushing_local_ = true;
    }
    cv_.notify_all();
    if (task_) task_->request_stop();
  }
  bool stop() override {
    unlock();
    if (task_) {
      task_->join();
      task_.reset();
    }
    std::lock_guard<std::mutex> lk(mu_);
    q_.clear();
    return true;
  }

  FlowReturn chain(Pad*, BufferPtr buf) override {
    std::unique_lock<std::mutex> lk(mu_);
    if (flushing_local_) return FlowReturn::FLUSHING;
    if (!flow_ok(last_ret_) && last_ret_ != FlowReturn::NOT_LINKED) return last_ret_;
    size_t sz = buf->total_size();
    while (full()) {
      if (leaky_ == 1) return FlowReturn::OK;  // upstream: drop the new buffer
      if (leaky_ == 2) {                       // downstream: drop the oldest buffer
        for (auto it = q_.begin(); it != q_.end(); ++it) {
          if (it->buf) {
            bytes_ -= it->buf->total_size();
            --nbuf_;
            q_.erase(it);
            break;
          }
        }
        continue;
      }
      cv_.wait(lk);
      if (flushing_local_) return FlowReturn::FLUSHING;
    }
    q_.push_back(Item{std::move(buf), Event(), false});
    ++nbuf_;
    bytes_ += sz;
    cv_.notify_all();
    return FlowReturn::OK;
  }

  bool sink_event(Pad* pad, Event& ev) override {
    (void)pad;
    if (ev.type == EventType::FLUSH_START) {
      {
        std::lock_guard<std::mutex> lk(mu_);
        q_.clear();
        nbuf_ = 0;
        bytes_ = 0;
      }
      cv_.notify_all();
      return forward_event_downstream(ev);
    }
    if (!event_is_serialized(ev.type)) return forward_event_downstream(ev);
    std::lock_guard<std::mutex> lk(mu_);
    q_.push_back(Item{nullptr, ev, true});
    cv_.notify_all();
    return true;
  }

  Caps query_caps(Pad* pad, const Caps* filter) override {
    Pad* other = pad->direction() == PadDirection::SINK ? src_pad() : sink_pad();
    Caps c = other->is_linked() ? other->peer_query_caps(filter) : Caps::Any();
    return filter ? c.intersect(*filter) : c;
  }

 private:
  struct Item {
    BufferPtr buf;
    Event ev;
    bool is_event;
  };
  bool full() const {
    if (max_buffers_ && nbuf_ >= max_buffers_) return true;
    if (max_bytes_ && bytes_ >= max_bytes_) return true;
    return false;
  }
  bool loop() {
    Item it;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return flushing_local_ || !q_.empty(); });
      if (flushing_local_) return false;
      it = std::move(q_.front());
      q_.pop_front();
      if (!it.is_event) {
        --nbuf_;
        bytes_ -= it.buf->total_size();
      }
      cv_.notify_all();
    }
    if (it.is_event) {
      bool is_eos = it.ev.type == EventType::EOS;
      src_pad()->push_event(it.ev);
      return true;
      (void)is_eos;
    }
    FlowReturn r = src_pad()->push(it.buf);
    if (!flow_ok(r)) {
      std::lock_guard<std::mutex> lk(mu_);
      last_ret_ = r;
      if (r == FlowReturn::EOS || r == FlowReturn::FLUSHING) {
        // keep draining events (an EOS must still reach the sink) but drop data
        return true;
      }
      if (r == FlowReturn::NOT_LINKED) return true;
      post_error(strfmt("internal data stream error: ", flow_name(r)));
      return true;
    }
    return true;
  }

  unsigned max_buffers_ = 200;
  unsigned max_bytes_ = 10 * 1024 * 1024;
  int64_t max_time_ = 1000000000;
  int leaky_ = 0;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Item> q_;
  unsigned nbuf_ = 0;
  size_t bytes_ = 0;
  bool flushing_local_ = false;
  FlowReturn last_ret_ = FlowReturn::OK;
  std::unique_ptr<Task> task_;
};

// -------------------------------------------------------------------- tee ----
class Tee : public Element {
 public:
  explicit Tee(const std::string& name) : Element("tee", name) {
    add_template("sink", PadDirection::SINK, PadPresence::ALWAYS, Caps::Any());
    add_template("src_%u", PadDirection::SRC, PadPresence::REQUEST, Caps::Any());
    prop_bool("allow-not-linked", &allow_not_linked_, "Return GST_FLOW_OK even if there are no source pads or they are all unlinked");
  }
  FlowReturn chain(Pad*, BufferPtr buf) override {
    FlowReturn agg = FlowReturn::NOT_LINKED;
    bool any_ok = false;
    for (Pad* p : src_pads()) {
      FlowReturn r = p->push(buf);
      if (flow_ok(r)) any_ok = true;
      else if (r != FlowReturn::NOT_LINKED && r != FlowReturn::EOS) agg = r;
      else if (r == FlowReturn::EOS && agg == FlowReturn::NOT_LINKED) agg = FlowReturn::EOS;
    }
    if (any_ok) return FlowReturn::OK;
    if (agg == FlowReturn::NOT_LINKED && allow_not_linked_) return FlowReturn::OK;
    return agg;
  }
  Caps query_caps(Pad* pad, const Caps* filter) override {
    Caps r = Caps::Any();
    if (pad->direction() == PadDirection::SINK) {
      for (Pad* p : src_pads())
        if (p->is_linked()) r = r.intersect(p->peer_query_caps(nullptr));
    } else if (sink_pad()->is_linked()) {
      r = sink_pad()->peer_query_caps(nullptr);
    }
    return filter ? r.intersect(*filter) : r;
  }

 private:
  bool allow_not_linked_ = false;
};

// ------------------------------------------------------------- capsfilter ----
class CapsFilter : public Element {
 public:
  explicit CapsFilter(const std::string& name) : Element("capsfilter", name) {
    add_template("sink", PadDirection::SINK, PadPresence::ALWAYS, Caps::Any());
    add_template("src", PadDirection::SRC, PadPresence::ALWAYS, Caps::Any());
    PropSpec s;
    s.name = "caps";
    s.type = PropType::CAPS;
    s.blurb = "Restrict the possible allowed capabilities";
    s.set = [this](const std::string& v) { caps_ = Caps::from_string(v); };
    s.get = [this] { return caps_.to_string(); };
    add_prop(s);
  }
  FlowReturn chain(Pad*, BufferPtr buf) override { return src_pad()->push(std::move(buf)); }
  Caps query_caps(Pad* pad, const Caps* filter) override {
    Pad* other = pad->direction() == PadDirection::SINK ? src_pad() : sink_pad();
    Caps r = caps_;
    if (other->is_linked()) {
      Caps peer = other->peer_query_caps(&caps_);
      r = caps_.intersect(peer);
    }
    return filter ? r.intersect(*filter) : r;
  }
  bool sink_event(Pad*, Event& ev) override {
    if (ev.type == EventType::CAPS && !caps_.can_intersect(ev.caps)) {
      post_error(strfmt("not-negotiated: caps ", ev.caps.to_string(), " do not match filter ", caps_.to_string()));
      return false;
    }
    return forward_event_downstream(ev);
  }

 private:
  Caps caps_ = Caps::Any();
};

// --------------------------------------------------------------- identity ----
class Identity : public Element {
 public:
  explicit Identity(const std::string& name) : Element("identity", name) {
    add_template("sink", PadDirection::SINK, PadPresence::ALWAYS, Caps::Any());
    add_template("src", PadDirection::SRC, PadPresence::ALWAYS, Caps::Any());
    prop_int("sleep-time", &sleep_us_, "Microseconds to sleep between processing");
    prop_int("error-after", &error_after_, "Error after N buffers (-1 = never)");
    prop_double("drop-probability", &drop_prob_, "The Probability a buffer is dropped");
    prop_bool("signal-handoffs", &signal_, "Send a signal before pushing the buffer");
    prop_bool("sync", &sync_, "Synchronize to pipeline clock");
  }
  FlowReturn chain(Pad*, BufferPtr buf) override {
    ++count_;
    if (error_after_ >= 0 && count_ > error_after_) {
      post_error("Failed because of \"error-after\" property");
      return FlowReturn::ERROR;
    }
    if (drop_prob_ > 0 && dist_(rng_) < drop_prob_) return FlowReturn::OK;
    if (sleep_us_ > 0) std::this_thread::sleep_for(std::chrono::microseconds(sleep_us_));
    if (sync_ && buf->pts >= 0) wait_until_running_time(buf->pts);
    if (signal_) {
      SignalArgs a;
      a.buffer = buf;
      emit("handoff", a);
    }
    return src_pad()->push(std::move(buf));
  }

 private:
  int64_t sleep_us_ = 0, error_after_ = -1, count_ = 0;
  double drop_prob_ = 0;
  bool signal_ = true, sync_ = false;
  std::mt19937 rng_{1234};
  std::uniform_real_distribution<double> dist_{0.0, 1.0};
};

// --------------------------------------------------------------- fakesink ----
class FakeSink : public BaseSink {
 public:
  explicit FakeSink(const std::string& name) : BaseSink("fakesink", name, Caps::Any()) {
    prop_bool("signal-handoffs", &signal_, "Send a signal before unreffing the buffer");
    prop_bool("dump", &dump_, "Dump buffer contents to stdout");
    prop_bool("sync-device", &sync_device_, "Wait for device-resident payloads to be produced (end-to-end timing)");
  }

 protected:
  FlowReturn render(const BufferPtr& buf) override {
    if (sync_device_)
      for (auto& m : buf->mems) m->sync_ready();
    if (dump_) {
      for (auto& m : buf->mems) {
        const uint8_t* p = static_cast<const uint8_t*>(m->map_host());
        for (size_t i = 0; i < m->size(); ++i) std::printf("%02x%s", p[i], (i % 16 == 15) ? "\n" : " ");
        std::printf("\n");
      }
    }
    if (signal_) {
      SignalArgs a;
      a.buffer = buf;
      emit("handoff", a);
    }
    return FlowReturn::OK;
  }

 private:
  bool signal_ = false, dump_ = false, sync_device_ = false;
};

// ---------------------------------------------------------------- fakesrc ----
class FakeSrc : public BaseSrc {
 public:
  explicit FakeSrc(const std::string& name) : BaseSrc("fakesrc", name, Caps::Any()) {
    prop_int("sizemax", &size_, "Size of the buffers");
    prop_enum("filltype", &fill_, {"nothing", "zero", "random", "pattern", "pattern-span"}, "How to fill the buffer");
    prop_enum("sizetype", &sizetype_, {"empty", "fixed", "random"}, "How to determine buffer sizes");
    num_buffers_ = -1;
  }

 protected:
  Caps get_caps(const Caps* filter) override {
    Caps c = Caps::Any();
    return filter ? c.intersect(*filter) : c;
  }
  Caps fixate(Caps caps) override { return caps.is_any() ? Caps::from_string("application/octet-stream") : caps.fixate(); }
  FlowReturn create(BufferPtr* out) override {
    auto b = make_buffer();
    size_t sz = sizetype_ == 0 ? 0 : static_cast<size_t>(size_);
    auto m = Memory::alloc_host(sz);
    if (fill_ == 1) std::memset(m->data(), 0, sz);
    if (fill_ == 2)
      for (size_t i = 0; i < sz; ++i) static_cast<uint8_t*>(m->data())[i] = static_cast<uint8_t>(rng_());
    if (fill_ >= 3)
      for (size_t i = 0; i < sz; ++i) static_cast<uint8_t*>(m->data())[i] = static_cast<uint8_t>(i);
    b->mems.push_back(m);
    b->offset = produced_;
    *out = b;
    return FlowReturn::OK;
  }

 private:
  int64_t size_ = 4096;
  int fill_ = 1, sizetype_ = 1;
  std::mt19937 rng_{7};
};

// ----------------------------------------------------------------- appsrc ----
class AppSrc : public BaseSrc, public AppSrcIface {
 public:
  explicit AppSrc(const std::string& name) : BaseSrc("appsrc", name, Caps::Any()) {
    PropSpec s;
    s.name = "caps";
    s.type = PropType::CAPS;
    s.blurb = "The allowed caps for the src pad";
    s.set = [this](const std::string& v) { caps_prop_ = Caps::from_string(v); };
    s.get = [this] { return caps_prop_.to_string(); };
    add_prop(s);
    prop_int("max-buffers", &max_buffers_, "The maximum number of buffers to queue internally (0 = unlimited)");
    prop_bool("block", &block_, "Block push-buffer when max-buffers are queued");
    prop_enum("format", &format_, {"undefined", "default", "bytes", "time", "buffers"}, "The format of the segment events");
    prop_enum("stream-type", &stream_type_, {"stream", "seekable", "random-access"}, "the type of the stream");
    prop_bool("emit-signals", &emit_signals_, "Emit need-data, enough-data and seek-data signals");
  }

  FlowReturn push(BufferPtr buf) override {
    // an application buffer in the reference's >16-tensor form (16 memories,
    // the last one a GstTensorExtraInfo block): one memory per tensor downstream
    if (buf && buf->mems.size() == static_cast<size_t>(kSizeLimit)) buf->mems = unpack_extra(buf->mems, nullptr);
    std::unique_lock<std::mutex> lk(mu_);
    if (eos_) return FlowReturn::EOS;
    if (flushing_.load() || unlocked_) return FlowReturn::FLUSHING;
    if (max_buffers_ > 0 && static_cast<int64_t>(q_.size()) >= max_buffers_) {
      if (!block_) {
        if (emit_signals_) {
          lk.unlock();
          emit("enough-data", SignalArgs{});
          lk.lock();
        }
      } else {
        cv_.wait(lk, [&] { return unlocked_ || static_cast<int64_t>(q_.size()) < max_buffers_; });
        if (unlocked_) return FlowReturn::FLUSHING;
      }
    }
    q_.push_back(std::move(buf));
    cv_.notify_all();
    return FlowReturn::OK;
  }
  FlowReturn end_of_stream() override {
    std::lock_guard<std::mutex> lk(mu_);
    eos_ = true;
    cv_.notify_all();
    return FlowReturn::OK;
  }
  void set_caps_string(const std::string& c) override { caps_prop_ = Caps::from_string(c); }
  size_t queued() override {
    std::lock_guard<std::mutex> lk(mu_);
    return q_.size();
  }

 protected:
  bool on_start() override {
    std::lock_guard<std::mutex> lk(mu_);
    unlocked_ = false;
    eos_ = false;
    q_.clear();
    return true;
  }
  void on_unlock() override {
    std::lock_guard<std::mutex> lk(mu_);
    unlocked_ = true;
    cv_.notify_all();
  }
  Caps get_caps(const Caps* filter) override {
    Caps c = caps_prop_;
    return filter ? c.intersect(*filter) : c;
  }
  FlowReturn create(BufferPtr* out) override {
    std::unique_lock<std::mutex> lk(mu_);
    if (q_.empty() && emit_signals_ && !eos_) {
      lk.unlock();
      emit("need-data", SignalArgs{});
      lk.lock();
    }
    cv_.wait(lk, [&] { return unlocked_ || eos_ || !q_.empty(); });
    if (unlocked_) return FlowReturn::FLUSHING;
    if (q_.empty() && eos_) return FlowReturn::EOS;
    *out = q_.front();
    q_.pop_front();
    cv_.notify_all();
    return FlowReturn::OK;
  }

 private:
  Caps caps_prop_ = Caps::Any();
  int64_t max_buffers_ = 0;
  bool block_ = false, emit_signals_ = true;
  int format_ = 3, stream_type_ = 0;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<BufferPtr> q_;
  bool eos_ = false, unlocked_ = false;
};

// ---------------------------------------------------------------- appsink ----
class AppSink : public BaseSink, public AppSinkIface {
 public:
  explicit AppSink(const std::string& name) : BaseSink("appsink", name, Caps::Any()) {
    PropSpec s;
    s.name = "caps";
    s.type = PropType::CAPS;
    s.blurb = "The allowed caps for the sink pad";
    s.set = [this](const std::string& v) {
      caps_prop_ = Caps::from_string(v);
      sink_pad()->set_template_caps(caps_prop_);
    };
    s.get = [this] { return caps_prop_.to_string(); };
    add_prop(s);
    prop_int("max-buffers", &max_buffers_, "The maximum number of buffers to queue internally (0 = unlimited)");
    prop_bool("drop", &drop_, "Drop old buffers when the buffer queue is filled");
    prop_bool("emit-signals", &emit_signals_, "Emit new-sample signal");
  }
  BufferPtr pull(int64_t timeout_ns) override {
    std::unique_lock<std::mutex> lk(mu_);
    auto pred = [&] { return !q_.empty() || eos_ || flushing_.load(); };
    if (timeout_ns < 0)
      cv_.wait(lk, pred);
    else
      cv_.wait_for(lk, std::chrono::nanoseconds(timeout_ns), pred);
    if (q_.empty()) return nullptr;
    auto b = q_.front();
    q_.pop_front();
    cv_.notify_all();
    return b;
  }
  bool is_eos() override {
    std::lock_guard<std::mutex> lk(mu_);
    return eos_ && q_.empty();
  }
  Caps negotiated_caps() override { return sink_pad()->current_caps(); }

 protected:
  bool start() override {
    BaseSink::start();
    std::lock_guard<std::mutex> lk(mu_);
    q_.clear();
    eos_ = false;
    return true;
  }
  void unlock() override { cv_.notify_all(); }
  FlowReturn render(const BufferPtr& buf) override {
    {
      std::unique_lock<std::mutex> lk(mu_);
      if (max_buffers_ > 0 && static_cast<int64_t>(q_.size()) >= max_buffers_) {
        if (drop_) {
          q_.pop_front();
        } else {
          cv_.wait(lk, [&] { return flushing_.load() || static_cast<int64_t>(q_.size()) < max_buffers_; });
          if (flushing_.load()) return FlowReturn::FLUSHING;
        }
      }
      q_.push_back(buf);
    }
    cv_.notify_all();
    if (emit_signals_) {
      SignalArgs a;
      a.buffer = buf;
      emit("new-sample", a);
    }
    return FlowReturn::OK;
  }
  void on_eos() override {
    std::lock_guard<std::mutex> lk(mu_);
    eos_ = true;
    cv_.notify_all();
  }

 private:
  Caps caps_prop_ = Caps::Any();
  int64_t max_buffers_ = 0;
  bool drop_ = false, emit_signals_ = false;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<BufferPtr> q_;
  bool eos_ = false;
};

// ----------------------------------------------------------- videotestsrc ----
class VideoTestSrc : public BaseSrc {
 public:
  explicit VideoTestSrc(const std::string& name)
      : BaseSrc("videotestsrc", name,
                Caps::from_string("video/x-raw, format=(string){ RGB, BGR, RGBx, BGRx, xRGB, xBGR, RGBA, BGRA, ARGB, "
                                  "ABGR, GRAY8, I420, NV12 }, width=(int)[ 1, 2147483647 ], height=(int)[ 1, "
                                  "2147483647 ], framerate=(fraction)[ 0/1, 2147483647/1 ]")) {
    prop_enum("pattern", &pattern_,
              {"smpte", "snow", "black", "white", "red", "green", "blue", "checkers-1", "checkers-2", "checkers-4",
               "checkers-8", "circular", "blink", "smpte75", "zone-plate", "gamut", "chroma-zone-plate",
               "solid-color", "ball", "smpte100", "bar", "pinwheel", "spokes", "gradient", "colors", "random"},
              "Type of test pattern to generate");
    prop_uint("foreground-color", &fg_, "Foreground color to use (big-endian ARGB)");
    prop_uint("background-color", &bg_, "Background color to use (big-endian ARGB)");
    prop_int("pool-size", &pool_size_, "Number of distinct pre-rendered frames cycled for animated patterns (nnsx)");
    prop_string("pool-shm", &pool_shm_,
                "nnsx: render the frame ring into this named POSIX shared-memory segment, so edgesink "
                "connect-type=SHM hands frames to other processes by reference ('' = private pinned memory)");
  }

 protected:
  Caps fixate(Caps caps) override {
    if (caps.size() == 0) return caps;
    Structure s = caps.at(0);
    s.fixate_nearest_int("width", 320);
    s.fixate_nearest_int("height", 240);
    s.fixate_nearest_fraction("framerate", 30, 1);
    s.fixate_string("format", "RGB");
    s.fixate();
    Caps r;
    r.append(s);
    return r;
  }
  bool set_caps(const Caps& caps) override {
    if (!info_.from_structure(caps.at(0))) return false;
    frames_.clear();
    // pre-render the whole frame ring up front (in parallel) so producing a frame
    // is O(1) and no rendering lands inside a measured run
    const bool animated = pattern_ == 1 || pattern_ == 12 || pattern_ == 18 || pattern_ == 25;
    int64_t n = animated ? std::max<int64_t>(1, pool_size_) : 1;
    if (num_buffers_ >= 0) n = std::min<int64_t>(n, std::max<int64_t>(1, num_buffers_));  // frames ever shown
    frames_.resize(static_cast<size_t>(n));
    // one pinned block holds the whole ring (a camera's mmap'ed capture ring):
    // consecutive frames are adjacent, so a batching consumer uploads a run of
    // them with one DMA copy
    if (!pool_shm_.empty()) {
      // the ring in shared memory: consumers in other processes map it and
      // DMA their frames over their own GPU's link (comm/shm.h)
      std::string err;
      shm_ = comm::ShmSegment::create(pool_shm_, static_cast<size_t>(n) * info_.size, &err);
      if (!shm_) {
        post_error("videotestsrc: pool-shm: " + err);
        return false;
      }
      ring_ = shm_->view(0, static_cast<size_t>(n) * info_.size);
    } else {
      ring_ = Memory::alloc_pinned(static_cast<size_t>(n) * info_.size);
    }
    for (int64_t i = 0; i < n; ++i)
      frames_[static_cast<size_t>(i)] = Memory::view(ring_, static_cast<size_t>(i) * info_.size, info_.size);
    const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
      th.emplace_back([this, t, nt, n] {
        for (int64_t i = t; i < n; i += nt) render(i, frames_[static_cast<size_t>(i)]);
      });
    for (auto& x : th) x.join();
    return true;
  }
  FlowReturn create(BufferPtr* out) override {
    bool animated = pattern_ == 1 || pattern_ == 12 || pattern_ == 18 || pattern_ == 25;
    int64_t nframes = animated ? std::max<int64_t>(1, pool_size_) : 1;
    size_t idx = static_cast<size_t>(produced_ % nframes);
    if (frames_.size() <= idx) frames_.resize(idx + 1);
    if (!frames_[idx]) frames_[idx] = render(produced_);
    auto b = make_buffer();
    b->mems.push_back(frames_[idx]);  // immutable frames are shared zero-copy
    if (info_.fps_n > 0) {
      b->pts = produced_ * kSecond * info_.fps_d / info_.fps_n;
      b->duration = kSecond * info_.fps_d / info_.fps_n;
    } else {
      // no framerate: stamp the capture time (running time) so sinks can
      // measure per-frame end-to-end latency
      b->pts = running_time();
      b->duration = -1;
    }
    b->offset = produced_;
    if (is_live_ && info_.fps_n > 0 && !wait_until_running_time(b->pts)) return FlowReturn::FLUSHING;
    *out = b;
    return FlowReturn::OK;
  }

 private:
  void color_of(int x, int y, int64_t frame, uint8_t rgb[3]) {
    int w = info_.width, h = info_.height;
    switch (pattern_) {
      case 0: case 13: case 19: {  // smpte-like colour bars
        static const uint8_t bars[7][3] = {{192, 192, 192}, {192, 192, 0}, {0, 192, 192}, {0, 192, 0},
                                          {192, 0, 192},   {192, 0, 0},   {0, 0, 192}};
        int i = std::min(6, x * 7 / std::max(1, w));
        std::memcpy(rgb, bars[i], 3);
        return;
      }
      case 1: case 25: {  // snow / random
        uint32_t v = static_cast<uint32_t>((x * 1103515245u) ^ (y * 12345u) ^ (frame * 2654435761u));
        v ^= v >> 13; v *= 0x5bd1e995u; v ^= v >> 15;
        rgb[0] = v & 255; rgb[1] = (v >> 8) & 255; rgb[2] = (v >> 16) & 255;
        if (pattern_ == 1) rgb[1] = rgb[2] = rgb[0];
        return;
      }
      case 2: rgb[0] = rgb[1] = rgb[2] = 0; return;
      case 3: rgb[0] = rgb[1] = rgb[2] = 255; return;
      case 4: rgb[0] = 255; rgb[1] = rgb[2] = 0; return;
      case 5: rgb[1] = 255; rgb[0] = rgb[2] = 0; return;
      case 6: rgb[2] = 255; rgb[0] = rgb[1] = 0; return;
      case 7: case 8: case 9: case 10: {
        int sz = 1 << (pattern_ - 7);
        bool on = ((x / sz) + (y / sz)) & 1;
        rgb[0] = on ? 255 : 0; rgb[1] = on ? 255 : 0; rgb[2] = on ? 255 : 0;
        if (!on) { rgb[0] = 0; rgb[1] = 255; rgb[2] = 0; }
        return;
      }
      case 17: {
        rgb[0] = (fg_ >> 16) & 255; rgb[1] = (fg_ >> 8) & 255; rgb[2] = fg_ & 255;
        return;
      }
      case 23: {
        uint8_t v = static_cast<uint8_t>(y * 255 / std::max(1, h - 1));
        rgb[0] = rgb[1] = rgb[2] = v;
        return;
      }
      default: {  // gradient-ish colours for the remaining patterns
        rgb[0] = static_cast<uint8_t>(x * 255 / std::max(1, w - 1));
        rgb[1] = static_cast<uint8_t>(y * 255 / std::max(1, h - 1));
        rgb[2] = static_cast<uint8_t>((frame * 8) & 255);
        return;
      }
    }
  }

  MemoryPtr render(int64_t frame, MemoryPtr m = nullptr) {
    if (!m) m = Memory::alloc_pinned(info_.size);
    uint8_t* p = static_cast<uint8_t*>(m->data());
    std::memset(p, 0, info_.size);
    const std::string& f = info_.format;
    if (f == "RGB" && info_.packed()) {  // fast path (benchmarks render large frame rings)
      for (int y = 0; y < info_.height; ++y) {
        uint8_t* row = p + y * info_.stride[0];
        for (int x = 0; x < info_.width; ++x) color_of(x, y, frame, row + 3 * x);
      }
      return m;
    }
    for (int y = 0; y < info_.height; ++y) {
      for (int x = 0; x < info_.width; ++x) {
        uint8_t c[3];
        color_of(x, y, frame, c);
        if (info_.packed()) {
          uint8_t* px = p + y * info_.stride[0] + x * info_.bpp;
          if (f == "RGB") { px[0] = c[0]; px[1] = c[1]; px[2] = c[2]; }
          else if (f == "BGR") { px[0] = c[2]; px[1] = c[1]; px[2] = c[0]; }
          else if (f == "RGBx" || f == "RGBA") { px[0] = c[0]; px[1] = c[1]; px[2] = c[2]; px[3] = 255; }
          else if (f == "BGRx" || f == "BGRA") { px[0] = c[2]; px[1] = c[1]; px[2] = c[0]; px[3] = 255; }
          else if (f == "xRGB" || f == "ARGB") { px[0] = 255; px[1] = c[0]; px[2] = c[1]; px[3] = c[2]; }
          else if (f == "xBGR" || f == "ABGR") { px[0] = 255; px[1] = c[2]; px[2] = c[1]; px[3] = c[0]; }
          else if (f == "GRAY8") { px[0] = static_cast<uint8_t>((c[0] * 77 + c[1] * 150 + c[2] * 29) >> 8); }
          else if (f == "GRAY16_LE") { uint16_t g = static_cast<uint16_t>((c[0] * 77 + c[1] * 150 + c[2] * 29)); std::memcpy(px, &g, 2); }
        } else {
          int yy = (66 * c[0] + 129 * c[1] + 25 * c[2] + 128) / 256 + 16;
          p[y * info_.stride[0] + x] = static_cast<uint8_t>(yy);
          if ((x % 2 == 0) && (y % 2 == 0)) {
            int u = (-38 * c[0] - 74 * c[1] + 112 * c[2] + 128) / 256 + 128;
            int v = (112 * c[0] - 94 * c[1] - 18 * c[2] + 128) / 256 + 128;
            if (f == "I420") {
              p[info_.offset[1] + (y / 2) * info_.stride[1] + x / 2] = static_cast<uint8_t>(u);
              p[info_.offset[2] + (y / 2) * info_.stride[2] + x / 2] = static_cast<uint8_t>(v);
            } else {
              uint8_t* uv = p + info_.offset[1] + (y / 2) * info_.stride[1] + (x / 2) * 2;
              uv[0] = static_cast<uint8_t>(f == "NV12" ? u : v);
              uv[1] = static_cast<uint8_t>(f == "NV12" ? v : u);
            }
          }
        }
      }
    }
    return m;
  }

  int pattern_ = 0;
  unsigned fg_ = 0xffffffff, bg_ = 0xff000000;
  int64_t pool_size_ = 8;
  std::string pool_shm_;
  std::shared_ptr<comm::ShmSegment> shm_;
  VideoInfo info_;
  std::vector<MemoryPtr> frames_;
  MemoryPtr ring_;
};

// ----------------------------------------------------------- audiotestsrc ----
class AudioTestSrc : public BaseSrc {
 public:
  explicit AudioTestSrc(const std::string& name)
      : BaseSrc("audiotestsrc", name,
                Caps::from_string("audio/x-raw, format=(string){ S16LE, S32LE, F32LE, F64LE, S8, U8 }, "
                                  "rate=(int)[ 1, 2147483647 ], channels=(int)[ 1, 256 ], layout=(string)interleaved")) {
    prop_int("samplesperbuffer", &spb_, "Number of samples in each outgoing buffer");
    prop_enum("wave", &wave_, {"sine", "square", "saw", "triangle", "silence", "white-noise"}, "Oscillator waveform");
    prop_double("freq", &freq_, "Frequency of test signal");
    prop_double("volume", &volume_, "Volume of test signal");
  }

 protected:
  Caps fixate(Caps caps) override {
    Structure s = caps.at(0);
    s.fixate_nearest_int("rate", 44100);
    s.fixate_nearest_int("channels", 1);
    s.fixate_string("format", "S16LE");
    s.fixate();
    Caps r;
    r.append(s);
    return r;
  }
  bool set_caps(const Caps& caps) override { return info_.from_structure(caps.at(0)); }
  FlowReturn create(BufferPtr* out) override {
    auto m = Memory::alloc_host(static_cast<size_t>(spb_) * info_.bpf);
    for (int64_t i = 0; i < spb_; ++i) {
      double t = static_cast<double>(sample_ + i) / info_.rate;
      double v = 0;
      switch (wave_) {
        case 0: v = std::sin(2 * M_PI * freq_ * t); break;
        case 1: v = std::sin(2 * M_PI * freq_ * t) >= 0 ? 1 : -1; break;
        case 2: v = 2 * (freq_ * t - std::floor(freq_ * t + 0.5)); break;
        case 3: v = 2 * std::fabs(2 * (freq_ * t - std::floor(freq_ * t + 0.5))) - 1; break;
        case 4: v = 0; break;
        default: v = dist_(rng_); break;
      }
      v *= volume_;
      for (int c = 0; c < info_.channels; ++c) {
        uint8_t* px = static_cast<uint8_t*>(m->data()) + (i * info_.channels + c) * info_.sample_size;
        const std::string& f = info_.format;
        if (f == "S16LE") { int16_t s = static_cast<int16_t>(v * 32767); std::memcpy(px, &s, 2); }
        else if (f == "S32LE") { int32_t s = static_cast<int32_t>(v * 2147483647.0); std::memcpy(px, &s, 4); }
        else if (f == "F32LE") { float s = static_cast<float>(v); std::memcpy(px, &s, 4); }
        else if (f == "F64LE") { std::memcpy(px, &v, 8); }
        else if (f == "S8") { int8_t s = static_cast<int8_t>(v * 127); std::memcpy(px, &s, 1); }
        else if (f == "U8") { uint8_t s = static_cast<uint8_t>(v * 127 + 128); std::memcpy(px, &s, 1); }
      }
    }
    auto b = make_buffer();
    b->mems.push_back(m);
    b->pts = sample_ * kSecond / info_.rate;
    b->duration = spb_ * kSecond / info_.rate;
    b->offset = sample_;
    sample_ += spb_;
    *out = b;
    return FlowReturn::OK;
  }
  bool on_start() override {
    sample_ = 0;
    return true;
  }

 private:
  int64_t spb_ = 1024, sample_ = 0;
  int wave_ = 0;
  double freq_ = 440, volume_ = 0.8;
  AudioInfo info_;
  std::mt19937 rng_{3};
  std::uniform_real_distribution<double> dist_{-1.0, 1.0};
};

// ---------------------------------------------------------------- filesrc ----
class FileSrc : public BaseSrc {
 public:
  explicit FileSrc(const std::string& name) : BaseSrc("filesrc", name, Caps::Any()) {
    prop_string("location", &location_, "Location of the file to read");
    prop_uint("blocksize", &blocksize_, "Size in bytes to read per buffer (-1 = default)");
  }

 protected:
  Caps fixate(Caps caps) override { return caps.is_any() ? Caps::from_string("application/octet-stream") : caps.fixate(); }
  bool on_start() override {
    f_.close();
    f_.clear();
    f_.open(location_, std::ios::binary);
    if (!f_) {
      post_error("Could not open file \"" + location_ + "\" for reading.");
      return false;
    }
    offset_ = 0;
    return true;
  }
  void on_stop() override { f_.close(); }
  FlowReturn create(BufferPtr* out) override {
    auto m = Memory::alloc_host(blocksize_);
    f_.read(static_cast<char*>(m->data()), blocksize_);
    std::streamsize n = f_.gcount();
    if (n <= 0) return FlowReturn::EOS;
    auto b = make_buffer();
    b->mems.push_back(n == static_cast<std::streamsize>(blocksize_) ? m : Memory::view(m, 0, static_cast<size_t>(n)));
    b->offset = offset_;
    offset_ += n;
    b->offset_end = offset_;
    *out = b;
    return FlowReturn::OK;
  }

 private:
  std::string location_;
  unsigned blocksize_ = 4096;
  std::ifstream f_;
  int64_t offset_ = 0;
};

// ----------------------------------------------------------- multifilesrc ----
class MultiFileSrc : public BaseSrc {
 public:
  explicit MultiFileSrc(const std::string& name) : BaseSrc("multifilesrc", name, Caps::Any()) {
    prop_string("location", &location_, "Pattern to create file names of input files.  File names are created by calling sprintf() with the pattern and the current index.");
    prop_int("index", &index_, "Index to use with location property to create file names");
    prop_int("start-index", &start_index_, "Start value of index");
    prop_int("stop-index", &stop_index_, "Stop value of index (-1 = unlimited)");
    prop_bool("loop", &loop_, "Whether to repeat from the beginning when all files have been read");
    PropSpec s;
    s.name = "caps";
    s.type = PropType::CAPS;
    s.blurb = "Caps describing the format of the data";
    s.set = [this](const std::string& v) { caps_prop_ = Caps::from_string(v); };
    s.get = [this] { return caps_prop_.to_string(); };
    add_prop(s);
  }

 protected:
  Caps get_caps(const Caps* filter) override {
    Caps c = caps_prop_;
    return filter ? c.intersect(*filter) : c;
  }
  Caps fixate(Caps caps) override {
    if (caps.is_any()) return Caps::from_string("application/octet-stream");
    return caps.fixate();
  }
  bool set_caps(const Caps& caps) override {
    fps_n_ = 0;
    fps_d_ = 1;
    if (caps.size() > 0) caps.at(0).get_fraction("framerate", &fps_n_, &fps_d_);
    return true;
  }
  bool on_start() override {
    cur_ = index_ > 0 ? index_ : start_index_;
    count_ = 0;
    return true;
  }
  FlowReturn create(BufferPtr* out) override {
    if (stop_index_ >= 0 && cur_ > stop_index_) {
      if (!loop_) return FlowReturn::EOS;
      cur_ = start_index_;
    }
    std::string fn = format_location(location_, cur_);
    std::ifstream f(fn, std::ios::binary);
    if (!f) {
      if (loop_ && cur_ != start_index_) {
        cur_ = start_index_;
        return create(out);
      }
      if (count_ == 0) post_error("Could not open file \"" + fn + "\" for reading.");
      return FlowReturn::EOS;
    }
    std::vector<char> data((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    auto b = make_buffer();
    b->mems.push_back(Memory::from_bytes(data.data(), data.size()));
    if (fps_n_ > 0) {
      b->pts = count_ * kSecond * fps_d_ / fps_n_;
      b->duration = kSecond * fps_d_ / fps_n_;
    }
    b->offset = count_;
    ++cur_;
    ++count_;
    *out = b;
    return FlowReturn::OK;
  }

 private:
  std::string location_ = "%05d";
  int64_t index_ = 0, start_index_ = 0, stop_index_ = -1, cur_ = 0, count_ = 0;
  bool loop_ = false;
  Caps caps_prop_ = Caps::Any();
  int fps_n_ = 0, fps_d_ = 1;
};

// --------------------------------------------------------------- filesink ----
class FileSink : public BaseSink {
 public:
  explicit FileSink(const std::string& name) : BaseSink("filesink", name, Caps::Any()) {
    prop_string("location", &location_, "Location of the file to write");
    prop_bool("append", &append_, "Append to an already existing file");
  }

 protected:
  bool start() override {
    BaseSink::start();
    f_.open(location_, std::ios::binary | (append_ ? std::ios::app : std::ios::trunc));
    if (!f_) {
      post_error("Could not open file \"" + location_ + "\" for writing.");
      return false;
    }
    return true;
  }
  bool stop() override {
    f_.close();
    return true;
  }
  FlowReturn render(const BufferPtr& buf) override {
    for (auto& m : buf->mems) {
      auto bytes = serialize_with_header(m);
      f_.write(reinterpret_cast<const char*>(bytes.data()), static_cast<std::streamsize>(bytes.size()));
    }
    f_.flush();
    return FlowReturn::OK;
  }

 private:
  std::string location_;
  bool append_ = false;
  std::ofstream f_;
};

// ---------------------------------------------------------- multifilesink ----
class MultiFileSink : public BaseSink {
 public:
  explicit MultiFileSink(const std::string& name) : BaseSink("multifilesink", name, Caps::Any()) {
    prop_string("location", &location_, "Location of the file to write");
    prop_int("index", &index_, "Index to use with location property to create file names");
    prop_int("max-files", &max_files_, "Maximum number of files to keep on disk (0 = unlimited)");
  }

 protected:
  bool start() override {
    BaseSink::start();
    cur_ = index_;
    return true;
  }
  FlowReturn render(const BufferPtr& buf) override {
    std::string fn = format_location(location_, cur_++);
    std::ofstream f(fn, std::ios::binary | std::ios::trunc);
    if (!f) {
      post_error("Could not open file \"" + fn + "\" for writing.");
      return FlowReturn::ERROR;
    }
    for (auto& m : buf->mems) {
      auto bytes = serialize_with_header(m);
      f.write(reinterpret_cast<const char*>(bytes.data()), static_cast<std::streamsize>(bytes.size()));
    }
    if (max_files_ > 0 && cur_ - index_ > max_files_) std::remove(format_location(location_, cur_ - max_files_ - 1).c_str());
    return FlowReturn::OK;
  }

 private:
  std::string location_ = "%05d";
  int64_t index_ = 0, cur_ = 0, max_files_ = 0;
};

// ----------------------------------------------------------- videoconvert ----
class VideoConvert : public BaseTransform {
 public:
  explicit VideoConvert(const std::string& name)
      : BaseTransform("videoconvert", name, templ(), templ()) {}

 protected:
  static Caps templ() {
    return Caps::from_string(
        "video/x-raw, format=(string){ RGB, BGR, RGBx, BGRx, xRGB, xBGR, RGBA, BGRA, ARGB, ABGR, GRAY8 }, "
        "width=(int)[ 1, 2147483647 ], height=(int)[ 1, 2147483647 ], framerate=(fraction)[ 0/1, 2147483647/1 ]");
  }
  Caps transform_caps(PadDirection, const Caps& caps, const Caps* filter) override {
    Caps r;
    for (size_t i = 0; i < caps.size(); ++i) {
      Structure s = caps.at(i);
      s.remove("format");
      s.set("format", Value::List({Value::String("RGB"), Value::String("BGR"), Value::String("RGBx"),
                                   Value::String("BGRx"), Value::String("xRGB"), Value::String("xBGR"),
                                   Value::String("RGBA"), Value::String("BGRA"), Value::String("ARGB"),
                                   Value::String("ABGR"), Value::String("GRAY8")}));
      r.append(s);
    }
    if (filter) r = r.intersect(*filter);
    return r;
  }
  Caps fixate_caps(PadDirection, const Caps& caps, Caps other) override {
    // keep the input format when possible
    std::string f;
    if (caps.size() && caps.at(0).get_string("format", &f) && other.size()) {
      Structure s = other.at(0);
      s.fixate_string("format", f);
      s.fixate();
      Caps r;
      r.append(s);
      return r;
    }
    return other.fixate();
  }
  bool set_caps(const Caps& in, const Caps& out) override {
    return in_.from_structure(in.at(0)) && out_.from_structure(out.at(0));
  }
  static void unpack(const std::string& f, const uint8_t* px, uint8_t rgba[4]) {
    rgba[3] = 255;
    if (f == "RGB") { rgba[0] = px[0]; rgba[1] = px[1]; rgba[2] = px[2]; }
    else if (f == "BGR") { rgba[0] = px[2]; rgba[1] = px[1]; rgba[2] = px[0]; }
    else if (f == "RGBx") { rgba[0] = px[0]; rgba[1] = px[1]; rgba[2] = px[2]; }
    else if (f == "RGBA") { rgba[0] = px[0]; rgba[1] = px[1]; rgba[2] = px[2]; rgba[3] = px[3]; }
    else if (f == "BGRx") { rgba[0] = px[2]; rgba[1] = px[1]; rgba[2] = px[0]; }
    else if (f == "BGRA") { rgba[0] = px[2]; rgba[1] = px[1]; rgba[2] = px[0]; rgba[3] = px[3]; }
    else if (f == "xRGB") { rgba[0] = px[1]; rgba[1] = px[2]; rgba[2] = px[3]; }
    else if (f == "ARGB") { rgba[3] = px[0]; rgba[0] = px[1]; rgba[1] = px[2]; rgba[2] = px[3]; }
    else if (f == "xBGR") { rgba[0] = px[3]; rgba[1] = px[2]; rgba[2] = px[1]; }
    else if (f == "ABGR") { rgba[3] = px[0]; rgba[0] = px[3]; rgba[1] = px[2]; rgba[2] = px[1]; }
    else if (f == "GRAY8") { rgba[0] = rgba[1] = rgba[2] = px[0]; }
  }
  static void pack(const std::string& f, const uint8_t rgba[4], uint8_t* px) {
    if (f == "RGB") { px[0] = rgba[0]; px[1] = rgba[1]; px[2] = rgba[2]; }
    else if (f == "BGR") { px[0] = rgba[2]; px[1] = rgba[1]; px[2] = rgba[0]; }
    else if (f == "RGBx") { px[0] = rgba[0]; px[1] = rgba[1]; px[2] = rgba[2]; px[3] = 255; }
    else if (f == "RGBA") { px[0] = rgba[0]; px[1] = rgba[1]; px[2] = rgba[2]; px[3] = rgba[3]; }
    else if (f == "BGRx") { px[0] = rgba[2]; px[1] = rgba[1]; px[2] = rgba[0]; px[3] = 255; }
    else if (f == "BGRA") { px[0] = rgba[2]; px[1] = rgba[1]; px[2] = rgba[0]; px[3] = rgba[3]; }
    else if (f == "xRGB") { px[0] = 255; px[1] = rgba[0]; px[2] = rgba[1]; px[3] = rgba[2]; }
    else if (f == "ARGB") { px[0] = rgba[3]; px[1] = rgba[0]; px[2] = rgba[1]; px[3] = rgba[2]; }
    else if (f == "xBGR") { px[0] = 255; px[1] = rgba[2]; px[2] = rgba[1]; px[3] = rgba[0]; }
    else if (f == "ABGR") { px[0] = rgba[3]; px[1] = rgba[2]; px[2] = rgba[1]; px[3] = rgba[0]; }
    else if (f == "GRAY8") { px[0] = static_cast<uint8_t>((rgba[0] * 77 + rgba[1] * 150 + rgba[2] * 29) >> 8); }
  }
  FlowReturn transform(const BufferPtr& in, BufferPtr* out) override {
    if (in_.format == out_.format) {
      *out = in;
      return FlowReturn::OK;
    }
    const uint8_t* src = static_cast<const uint8_t*>(in->mems.at(0)->map_host());
    auto m = Memory::alloc_host(out_.size);
    uint8_t* dst = static_cast<uint8_t*>(m->data());
    std::memset(dst, 0, out_.size);
    for (int y = 0; y < in_.height; ++y)
      for (int x = 0; x < in_.width; ++x) {
        uint8_t c[4];
        unpack(in_.format, src + y * in_.stride[0] + x * in_.bpp, c);
        pack(out_.format, c, dst + y * out_.stride[0] + x * out_.bpp);
      }
    auto b = make_buffer();
    b->copy_metadata_from(*in);
    b->mems.push_back(m);
    *out = b;
    return FlowReturn::OK;
  }

 private:
  VideoInfo in_, out_;
};

}  // namespace

void register_basic_elements() {
  register_element("queue", "Generic", "Simple data queue", [](const std::string& n) { return std::make_unique<Queue>(n); });
  register_element("tee", "Generic", "1-to-N pipe fitting", [](const std::string& n) { return std::make_unique<Tee>(n); });
  register_element("capsfilter", "Generic", "Pass data without modification, limiting formats",
                   [](const std::string& n) { return std::make_unique<CapsFilter>(n); });
  register_element("identity", "Generic", "Pass data without modification",
                   [](const std::string& n) { return std::make_unique<Identity>(n); });
  register_element("fakesink", "Sink", "Black hole for data", [](const std::string& n) { return std::make_unique<FakeSink>(n); });
  register_element("fakesrc", "Source", "Push empty (no data) buffers around",
                   [](const std::string& n) { return std::make_unique<FakeSrc>(n); });
  register_element("appsrc", "Generic/Source", "Allow the application to feed buffers to a pipeline",
                   [](const std::string& n) { return std::make_unique<AppSrc>(n); });
  register_element("appsink", "Generic/Sink", "Allow the application to get access to raw buffer",
                   [](const std::string& n) { return std::make_unique<AppSink>(n); });
  register_element("videotestsrc", "Source/Video", "Creates a test video stream",
                   [](const std::string& n) { return std::make_unique<VideoTestSrc>(n); });
  register_element("audiotestsrc", "Source/Audio", "Creates audio test signals of given frequency and volume",
                   [](const std::string& n) { return std::make_unique<AudioTestSrc>(n); });
  register_element("filesrc", "Source/File", "Read from arbitrary point in a file",
                   [](const std::string& n) { return std::make_unique<FileSrc>(n); });
  register_element("multifilesrc", "Source/File", "Read a sequentially named set of files into buffers",
                   [](const std::string& n) { return std::make_unique<MultiFileSrc>(n); });
  register_element("filesink", "Sink/File", "Write stream to a file",
                   [](const std::string& n) { return std::make_unique<FileSink>(n); });
  register_element("multifilesink", "Sink/File", "Write buffers to a sequentially named set of files",
                   [](const std::string& n) { return std::make_unique<MultiFileSink>(n); });
  register_element("videoconvert", "Filter/Converter/Video", "Converts packed RGB/gray video formats",
                   [](const std::string& n) { return std::make_unique<VideoConvert>(n); });
}

}  // namespace nnsx
