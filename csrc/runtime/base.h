// Base classes for the three element shapes (GstBaseSrc/GstPushSrc,
// GstBaseSink, GstBaseTransform) plus the collect-pads aggregator used by
// tensor_mux / tensor_merge / tensor_crop (GstCollectPads).
#pragma once

#include <deque>

#include "runtime/element.h"

namespace nnsx {

// ---------------------------------------------------------------- BaseSrc ----
class BaseSrc : public Element {
 public:
  BaseSrc(const std::string& factory, const std::string& name, const Caps& src_templ);
  ~BaseSrc() override;

  bool start() override;
  bool stop() override;
  void play() override;
  void unlock() override;
  bool src_event(Pad* pad, Event& ev) override;
  Caps query_caps(Pad* pad, const Caps* filter) override;
  bool query_latency(Pad* pad, bool* live, int64_t* min_lat, int64_t* max_lat) override;

 protected:
  // negotiation: default = template ∩ peer, then fixate()
  virtual bool negotiate();
  virtual Caps get_caps(const Caps* filter) { return filter ? src_pad()->template_caps().intersect(*filter) : src_pad()->template_caps(); }
  virtual Caps fixate(Caps caps) { return caps.fixate(); }
  virtual bool set_caps(const Caps& caps) { (void)caps; return true; }
  // produce one buffer; return EOS to finish
  virtual FlowReturn create(BufferPtr* out) = 0;
  virtual bool on_start() { return true; }
  virtual void on_stop() {}
  virtual void on_unlock() {}
  virtual bool handle_upstream_event(Event& ev) { (void)ev; return true; }
  virtual Segment make_segment() { return Segment(); }
  // push (for sources that want to emit several buffers per create)
  FlowReturn push_buffer(BufferPtr buf);
  bool ensure_negotiated();
  void send_eos();
  bool loop();

  int64_t num_buffers_ = -1;
  bool is_live_ = false;
  bool do_timestamp_ = false;
  int64_t produced_ = 0;
  bool negotiated_ = false;
  bool started_stream_ = false;
  Caps caps_;
  std::unique_ptr<Task> task_;
  std::atomic<bool> eos_sent_{false};
  std::atomic<bool> eos_requested_{false};
};

// --------------------------------------------------------------- BaseSink ----
class BaseSink : public Element {
 public:
  BaseSink(const std::string& factory, const std::string& name, const Caps& sink_templ);

  FlowReturn chain(Pad* pad, BufferPtr buf) override;
  bool sink_event(Pad* pad, Event& ev) override;
  bool start() override;
  bool query_latency(Pad* pad, bool* live, int64_t* min_lat, int64_t* max_lat) override;

 protected:
  virtual bool set_caps(const Caps& caps) { (void)caps; return true; }
  virtual FlowReturn render(const BufferPtr& buf) = 0;
  virtual bool event(Event& ev) { (void)ev; return true; }
  virtual void on_eos() {}

  bool sync_ = false;
  bool qos_ = false;
  int64_t ts_offset_ = 0;
  int64_t max_lateness_ = -1;
  Segment segment_;
  int64_t rendered_ = 0;
  int64_t dropped_ = 0;
};

// ---------------------------------------------------------- BaseTransform ----
class BaseTransform : public Element {
 public:
  BaseTransform(const std::string& factory, const std::string& name, const Caps& sink_templ,
                const Caps& src_templ);

  FlowReturn chain(Pad* pad, BufferPtr buf) override;
  bool sink_event(Pad* pad, Event& ev) override;
  bool src_event(Pad* pad, Event& ev) override;
  Caps query_caps(Pad* pad, const Caps* filter) override;
  bool query_latency(Pad* pad, bool* live, int64_t* min_lat, int64_t* max_lat) override;

 protected:
  // Caps on the other side of `dir` (dir = SINK: caps are sink caps -> src caps)
  virtual Caps transform_caps(PadDirection dir, const Caps& caps, const Caps* filter);
  virtual Caps fixate_caps(PadDirection dir, const Caps& caps, Caps othercaps);
  virtual bool set_caps(const Caps& incaps, const Caps& outcaps) {
    (void)incaps;
    (void)outcaps;
    return true;
  }
  // transform; *out = nullptr with OK means "drop silently"
  virtual FlowReturn transform(const BufferPtr& in, BufferPtr* out) = 0;
  virtual bool handle_sink_event(Event& ev) { (void)ev; return true; }  // return false to swallow
  virtual bool handle_src_event(Event& ev) { (void)ev; return true; }   // return false to swallow
  virtual void before_transform(const BufferPtr& in) { (void)in; }
  // latency this element adds (for latency queries)
  virtual int64_t own_latency() const { return 0; }

  bool negotiated_ = false;
  Caps in_caps_, out_caps_;
  std::mutex caps_mu_;
};

// ---------------------------------------------------------- CollectPads ----
// Per-sink-pad one-deep queues with blocking hand-off; `collected` runs on the
// thread of the pad that completed the set.
class CollectPads {
 public:
  struct PadData {
    Pad* pad = nullptr;
    std::deque<BufferPtr> queue;
    bool eos = false;
    int64_t base_ts = -1;  // time-sync helpers
    BufferPtr last;        // "refresh"/"slowest" policies keep the previous buffer
  };

  explicit CollectPads(Element* owner) : owner_(owner) {}
  void add_pad(Pad* pad);
  void remove_pad(Pad* pad);
  void set_flushing(bool f);
  void reset();
  // called from a sink pad's chain: enqueue and maybe run the collect callback
  FlowReturn chain(Pad* pad, BufferPtr buf, const std::function<FlowReturn()>& collected, size_t depth = 1);
  // EOS on a pad: mark and maybe collect (returns true if everything is EOS)
  bool set_eos(Pad* pad, const std::function<FlowReturn()>& collected);
  // inside `collected` (lock held)
  std::vector<PadData*> pads();
  PadData* data(Pad* pad);
  BufferPtr peek(PadData* d) { return d->queue.empty() ? nullptr : d->queue.front(); }
  BufferPtr pop(PadData* d);
  bool all_have_data_or_eos();
  bool all_eos();
  bool any_has_data();
  void notify() { cv_.notify_all(); }
  std::mutex& lock() { return mu_; }

 private:
  Element* owner_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<std::unique_ptr<PadData>> pads_;
  bool flushing_ = false;
  bool collecting_ = false;
};

}  // namespace nnsx
