#include "runtime/base.h"

#include "core/log.h"
#include "runtime/pipeline.h"

namespace nnsx {

// ---------------------------------------------------------------- BaseSrc ----

BaseSrc::BaseSrc(const std::string& factory, const std::string& name, const Caps& src_templ)
    : Element(factory, name) {
  flags_ |= ELEM_SOURCE;
  add_template("src", PadDirection::SRC, PadPresence::ALWAYS, src_templ);
  prop_int("num-buffers", &num_buffers_, "Number of buffers to output before sending EOS (-1 = unlimited)");
  prop_bool("is-live", &is_live_, "Whether to act as a live source");
  prop_bool("do-timestamp", &do_timestamp_, "Apply current stream time to buffers");
}

BaseSrc::~BaseSrc() {
  if (task_) {
    task_->request_stop();
    task_->join();
  }
}

bool BaseSrc::start() {
  produced_ = 0;
  negotiated_ = false;
  started_stream_ = false;
  eos_sent_ = false;
  eos_requested_ = false;
  return on_start();
}

void BaseSrc::play() {
  if (!task_) task_ = std::make_unique<Task>([this] { return loop(); });
  if (!task_->running()) {
    task_->join();
    task_->start();
  }
}

void BaseSrc::unlock() {
  if (task_) task_->request_stop();
  on_unlock();
}

bool BaseSrc::stop() {
  if (task_) {
    task_->request_stop();
    on_unlock();
    task_->join();
    task_.reset();
  }
  on_stop();
  return true;
}

Caps BaseSrc::query_caps(Pad* pad, const Caps* filter) {
  (void)pad;
  if (negotiated_ && src_pad()->has_current_caps()) {
    Caps c = src_pad()->current_caps();
    return filter ? c.intersect(*filter) : c;
  }
  return get_caps(filter);
}

bool BaseSrc::query_latency(Pad*, bool* live, int64_t*, int64_t*) {
  *live = *live || is_live_;
  return true;
}

bool BaseSrc::negotiate() {
  Caps thiscaps = get_caps(nullptr);
  Caps peer = src_pad()->peer_query_caps(&thiscaps);
  Caps caps = thiscaps.intersect(peer);
  if (caps.is_empty()) {
    post_error(strfmt("not-negotiated: ", thiscaps.to_string(), " vs peer ", peer.to_string()));
    return false;
  }
  if (caps.is_any()) caps = thiscaps;
  caps = fixate(caps);
  if (caps.is_empty() || (!caps.is_fixed() && !caps.is_any())) {
    caps = caps.fixate();
  }
  if (!set_caps(caps)) {
    post_error("set_caps failed: " + caps.to_string());
    return false;
  }
  caps_ = caps;
  return src_pad()->push_event(Event::make_caps(caps));
}

bool BaseSrc::ensure_negotiated() {
  if (!started_stream_) {
    src_pad()->push_event(Event::make_stream_start(name() + "-stream"));
    started_stream_ = true;
  }
  if (!negotiated_) {
    if (!negotiate()) return false;
    negotiated_ = true;
    src_pad()->push_event(Event::make_segment(make_segment()));
  }
  return true;
}

FlowReturn BaseSrc::push_buffer(BufferPtr buf) { return src_pad()->push(std::move(buf)); }

void BaseSrc::send_eos() {
  if (eos_sent_.exchange(true)) return;
  Event ev = Event::make_eos();
  src_pad()->push_event(ev);
}

bool BaseSrc::loop() {
  if (flushing_.load()) return false;
  if (!ensure_negotiated()) {
    send_eos();
    return false;
  }
  if (eos_requested_.load() || (num_buffers_ >= 0 && produced_ >= num_buffers_)) {
    send_eos();
    return false;
  }
  BufferPtr buf;
  FlowReturn r = create(&buf);
  if (r == FlowReturn::EOS) {
    send_eos();
    return false;
  }
  if (r == FlowReturn::FLUSHING) return false;
  if (!flow_ok(r)) {
    post_error(strfmt("internal data stream error: create returned ", flow_name(r)));
    send_eos();
    return false;
  }
  if (!buf) return true;  // nothing this round
  if (do_timestamp_ && buf->pts < 0) buf->pts = running_time();
  ++produced_;
  r = push_buffer(std::move(buf));
  if (r == FlowReturn::EOS) {
    send_eos();
    return false;
  }
  if (r == FlowReturn::FLUSHING) return false;
  if (!flow_ok(r) && r != FlowReturn::NOT_LINKED) {
    post_error(strfmt("internal data stream error: streaming stopped, reason ", flow_name(r)));
    send_eos();
    return false;
  }
  return true;
}

bool BaseSrc::src_event(Pad*, Event& ev) {
  if (ev.type == EventType::EOS) {
    eos_requested_ = true;
    return true;
  }
  return handle_upstream_event(ev);
}

// --------------------------------------------------------------- BaseSink ----

BaseSink::BaseSink(const std::string& factory, const std::string& name, const Caps& sink_templ)
    : Element(factory, name) {
  flags_ |= ELEM_SINK;
  add_template("sink", PadDirection::SINK, PadPresence::ALWAYS, sink_templ);
  prop_bool("sync", &sync_, "Sync on the clock");
  prop_bool("qos", &qos_, "Generate Quality-of-Service events upstream");
  prop_int("ts-offset", &ts_offset_, "Timestamp offset in nanoseconds");
  prop_int("max-lateness", &max_lateness_, "Maximum number of nanoseconds that a buffer can be late before it is dropped (-1 unlimited)");
  prop_readonly("rendered", [this] { return std::to_string(rendered_); }, "Number of rendered buffers");
}

bool BaseSink::start() {
  rendered_ = 0;
  dropped_ = 0;
  segment_ = Segment();
  return true;
}

FlowReturn BaseSink::chain(Pad*, BufferPtr buf) {
  if (flushing_.load()) return FlowReturn::FLUSHING;
  if (sync_ && buf->pts >= 0) {
    int64_t rt = buf->pts - segment_.start + segment_.base + ts_offset_;
    if (!wait_until_running_time(rt)) return FlowReturn::FLUSHING;
    if (max_lateness_ >= 0 && running_time() - rt > max_lateness_) {
      ++dropped_;
      return FlowReturn::OK;
    }
  }
  FlowReturn r = render(buf);
  if (flow_ok(r)) ++rendered_;
  return r;
}

bool BaseSink::sink_event(Pad* pad, Event& ev) {
  switch (ev.type) {
    case EventType::CAPS:
      if (!set_caps(ev.caps)) {
        post_error("sink refused caps " + ev.caps.to_string());
        return false;
      }
      pad->set_current_caps(ev.caps);
      return event(ev);
    case EventType::SEGMENT:
      segment_ = ev.segment;
      return event(ev);
    case EventType::EOS: {
      bool r = event(ev);
      on_eos();
      if (pipeline_) pipeline_->sink_reached_eos(this);
      return r;
    }
    case EventType::STREAM_START:
      if (pipeline_)
        pipeline_->bus().post(Message{MessageType::STREAM_START, name(), "", Structure("stream-start"), now_ns()});
      return event(ev);
    default:
      return event(ev);
  }
}

bool BaseSink::query_latency(Pad* pad, bool* live, int64_t* min_lat, int64_t* max_lat) {
  return Element::query_latency(pad, live, min_lat, max_lat);
}

// ---------------------------------------------------------- BaseTransform ----

BaseTransform::BaseTransform(const std::string& factory, const std::string& name, const Caps& sink_templ,
                             const Caps& src_templ)
    : Element(factory, name) {
  add_template("sink", PadDirection::SINK, PadPresence::ALWAYS, sink_templ);
  add_template("src", PadDirection::SRC, PadPresence::ALWAYS, src_templ);
}

Caps BaseTransform::transform_caps(PadDirection dir, const Caps& caps, const Caps* filter) {
  (void)dir;
  Caps r = caps;
  if (filter) r = r.intersect(*filter);
  return r;
}

Caps BaseTransform::fixate_caps(PadDirection dir, const Caps& caps, Caps othercaps) {
  (void)dir;
  (void)caps;
  return othercaps.fixate();
}

Caps BaseTransform::query_caps(Pad* pad, const Caps* filter) {
  // caps on `pad` = this pad's template ∩ transform(peer of the other pad's caps)
  Pad* other = pad->direction() == PadDirection::SINK ? src_pad() : sink_pad();
  Caps peer = other->is_linked() ? other->peer_query_caps(nullptr) : other->template_caps();
  Caps peer_t = peer.is_any() ? other->template_caps() : other->template_caps().intersect(peer);
  Caps r = transform_caps(other->direction(), peer_t, nullptr);
  r = pad->template_caps().intersect(r);
  if (filter) r = r.intersect(*filter);
  return r;
}

bool BaseTransform::sink_event(Pad* pad, Event& ev) {
  (void)pad;
  if (ev.type == EventType::CAPS) {
    const Caps& incaps = ev.caps;
    Caps peer = src_pad()->peer_query_caps(nullptr);
    Caps othercaps = transform_caps(PadDirection::SINK, incaps, nullptr);
    othercaps = src_pad()->template_caps().intersect(othercaps);
    Caps narrowed = othercaps.intersect(peer);
    if (!narrowed.is_empty()) othercaps = narrowed;
    if (othercaps.is_empty()) {
      post_error(strfmt("not-negotiated: cannot transform ", incaps.to_string()));
      return false;
    }
    Caps out = fixate_caps(PadDirection::SINK, incaps, othercaps);
    if (!out.is_fixed()) out = out.fixate();
    {
      std::lock_guard<std::mutex> lk(caps_mu_);
      if (!set_caps(incaps, out)) {
        post_error(strfmt("not-negotiated: set_caps failed in=", incaps.to_string(), " out=", out.to_string()));
        negotiated_ = false;
        return false;
      }
      in_caps_ = incaps;
      out_caps_ = out;
      negotiated_ = true;
    }
    return src_pad()->push_event(Event::make_caps(out));
  }
  if (!handle_sink_event(ev)) return true;
  return forward_event_downstream(ev);
}

bool BaseTransform::src_event(Pad*, Event& ev) {
  if (!handle_src_event(ev)) return true;
  return forward_event_upstream(ev);
}

FlowReturn BaseTransform::chain(Pad*, BufferPtr buf) {
  if (!negotiated_) {
    post_error("not-negotiated: buffer before caps");
    return FlowReturn::NOT_NEGOTIATED;
  }
  before_transform(buf);
  BufferPtr out;
  FlowReturn r;
  try {
    r = transform(buf, &out);
  } catch (const std::exception& e) {
    post_error(e.what());
    return FlowReturn::ERROR;
  }
  if (r == FlowReturn::CUSTOM_SUCCESS) return FlowReturn::OK;  // dropped on purpose
  if (!flow_ok(r)) return r;
  if (!out) return FlowReturn::OK;
  return src_pad()->push(std::move(out));
}

bool BaseTransform::query_latency(Pad* pad, bool* live, int64_t* min_lat, int64_t* max_lat) {
  bool ok = Element::query_latency(pad, live, min_lat, max_lat);
  int64_t own = own_latency();
  *min_lat += own;
  if (*max_lat >= 0) *max_lat += own;
  return ok;
}

// ---------------------------------------------------------- CollectPads ----

void CollectPads::add_pad(Pad* pad) {
  std::lock_guard<std::mutex> lk(mu_);
  auto d = std::make_unique<PadData>();
  d->pad = pad;
  pads_.push_back(std::move(d));
}

void CollectPads::remove_pad(Pad* pad) {
  std::lock_guard<std::mutex> lk(mu_);
  pads_.erase(std::remove_if(pads_.begin(), pads_.end(), [&](auto& d) { return d->pad == pad; }), pads_.end());
  cv_.notify_all();
}

void CollectPads::set_flushing(bool f) {
  std::lock_guard<std::mutex> lk(mu_);
  flushing_ = f;
  if (f)
    for (auto& d : pads_) d->queue.clear();
  cv_.notify_all();
}

void CollectPads::reset() {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& d : pads_) {
    d->queue.clear();
    d->eos = false;
    d->last.reset();
    d->base_ts = -1;
  }
  flushing_ = false;
  collecting_ = false;
}

std::vector<CollectPads::PadData*> CollectPads::pads() {
  std::vector<PadData*> v;
  for (auto& d : pads_) v.push_back(d.get());
  return v;
}

CollectPads::PadData* CollectPads::data(Pad* pad) {
  for (auto& d : pads_)
    if (d->pad == pad) return d.get();
  return nullptr;
}

BufferPtr CollectPads::pop(PadData* d) {
  if (d->queue.empty()) return nullptr;
  BufferPtr b = d->queue.front();
  d->queue.pop_front();
  cv_.notify_all();
  return b;
}

bool CollectPads::all_have_data_or_eos() {
  for (auto& d : pads_)
    if (d->queue.empty() && !d->eos) return false;
  return !pads_.empty();
}

bool CollectPads::all_eos() {
  for (auto& d : pads_)
    if (!d->eos || !d->queue.empty()) return false;
  return true;
}

bool CollectPads::any_has_data() {
  for (auto& d : pads_)
    if (!d->queue.empty()) return true;
  return false;
}

static size_t total_queued(const std::vector<std::unique_ptr<CollectPads::PadData>>& pads) {
  size_t n = 0;
  for (auto& d : pads) n += d->queue.size();
  return n;
}

FlowReturn CollectPads::chain(Pad* pad, BufferPtr buf, const std::function<FlowReturn()>& collected,
                              size_t depth) {
  std::unique_lock<std::mutex> lk(mu_);
  PadData* d = data(pad);
  if (!d) return FlowReturn::NOT_LINKED;
  cv_.wait(lk, [&] { return flushing_ || d->queue.size() < depth; });
  if (flushing_) return FlowReturn::FLUSHING;
  if (d->eos) return FlowReturn::EOS;
  d->queue.push_back(std::move(buf));
  FlowReturn ret = FlowReturn::OK;
  while (!collecting_ && !flushing_ && all_have_data_or_eos() && any_has_data()) {
    size_t before = total_queued(pads_);
    collecting_ = true;
    ret = collected();
    collecting_ = false;
    cv_.notify_all();
    if (!flow_ok(ret)) break;
    if (total_queued(pads_) >= before) break;  // nothing consumed: wait for more input
  }
  return ret;
}

bool CollectPads::set_eos(Pad* pad, const std::function<FlowReturn()>& collected) {
  std::unique_lock<std::mutex> lk(mu_);
  PadData* d = data(pad);
  if (!d) return false;
  d->eos = true;
  while (!collecting_ && !flushing_ && all_have_data_or_eos() && any_has_data()) {
    size_t before = total_queued(pads_);
    collecting_ = true;
    FlowReturn r = collected();
    collecting_ = false;
    cv_.notify_all();
    if (!flow_ok(r)) break;
    if (total_queued(pads_) >= before) break;
  }
  return all_eos();
}

}  // namespace nnsx
