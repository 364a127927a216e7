#include "runtime/element.h"
#include "runtime/tracer.h"

#include <algorithm>

#include "core/log.h"
#include "runtime/pipeline.h"

namespace nnsx {

const char* flow_name(FlowReturn r) {
  switch (r) {
    case FlowReturn::CUSTOM_SUCCESS: return "custom-success";
    case FlowReturn::OK: return "ok";
    case FlowReturn::NOT_LINKED: return "not-linked";
    case FlowReturn::FLUSHING: return "flushing";
    case FlowReturn::EOS: return "eos";
    case FlowReturn::NOT_NEGOTIATED: return "not-negotiated";
    case FlowReturn::ERROR: return "error";
  }
  return "?";
}

const char* event_type_name(EventType t) {
  switch (t) {
    case EventType::STREAM_START: return "stream-start";
    case EventType::CAPS: return "caps";
    case EventType::SEGMENT: return "segment";
    case EventType::EOS: return "eos";
    case EventType::FLUSH_START: return "flush-start";
    case EventType::FLUSH_STOP: return "flush-stop";
    case EventType::QOS: return "qos";
    case EventType::LATENCY: return "latency";
    case EventType::RECONFIGURE: return "reconfigure";
    case EventType::CUSTOM_DOWNSTREAM: return "custom-downstream";
    case EventType::CUSTOM_UPSTREAM: return "custom-upstream";
    case EventType::GAP: return "gap";
    case EventType::TAG: return "tag";
  }
  return "?";
}

const char* state_name(State s) {
  switch (s) {
    case State::NULL_: return "NULL";
    case State::READY: return "READY";
    case State::PAUSED: return "PAUSED";
    case State::PLAYING: return "PLAYING";
  }
  return "?";
}

// ------------------------------------------------------------------ Pad ----

Pad::Pad(Element* parent, std::string name, PadDirection dir, Caps templ)
    : parent_(parent), name_(std::move(name)), dir_(dir), templ_(std::move(templ)) {}

Caps Pad::current_caps() const {
  std::lock_guard<std::mutex> lk(caps_mu_);
  return caps_;
}

bool Pad::has_current_caps() const {
  std::lock_guard<std::mutex> lk(caps_mu_);
  return has_caps_;
}

void Pad::set_current_caps(const Caps& c) {
  std::lock_guard<std::mutex> lk(caps_mu_);
  caps_ = c;
  has_caps_ = true;
}

FlowReturn Pad::push(BufferPtr buf) {
  if (dir_ != PadDirection::SRC) return FlowReturn::ERROR;
  if (!peer_) {
    last_flow_.store(FlowReturn::NOT_LINKED);
    return FlowReturn::NOT_LINKED;
  }
  if (flushing_.load() || peer_->flushing_.load()) return FlowReturn::FLUSHING;
  if (peer_->eos_.load()) return FlowReturn::EOS;
  Element* sink = peer_->parent();
  FlowReturn r;
  const bool traced = trace::flags() != 0;
  try {
    if (traced) {  // built-in tracers (runtime/tracer.h)
      if (buf->origin_ns < 0) buf->origin_ns = now_ns();
      trace::src_push(parent());
      trace::chain_enter(sink, buf->origin_ns);
      r = sink->chain(peer_, std::move(buf));
      trace::chain_exit(sink);
    } else {
      r = sink->chain(peer_, std::move(buf));
    }
  } catch (const std::exception& e) {
    // failure detection: anything thrown downstream (a HIP error, a framework
    // exception) becomes an error message of the element that threw, not a
    // silently dead streaming thread
    if (traced) trace::chain_exit(sink);
    sink->post_error(e.what());
    r = FlowReturn::ERROR;
  }
  last_flow_.store(r);
  return r;
}

void Pad::store_sticky(const Event& e) {
  if (e.type != EventType::STREAM_START && e.type != EventType::CAPS && e.type != EventType::SEGMENT) return;
  std::lock_guard<std::mutex> lk(sticky_mu_);
  for (auto& s : sticky_) {
    if (s.type == e.type) {
      s = e;
      return;
    }
  }
  sticky_.push_back(e);
}

std::vector<Event> Pad::sticky_events() const {
  std::lock_guard<std::mutex> lk(sticky_mu_);
  return sticky_;
}

bool Pad::push_event(Event ev) {
  if (dir_ == PadDirection::SRC) {
    // downstream
    if (ev.type == EventType::CAPS) set_current_caps(ev.caps);
    if (ev.type == EventType::FLUSH_START) flushing_.store(true);
    if (ev.type == EventType::FLUSH_STOP) {
      flushing_.store(false);
      eos_.store(false);
    }
    store_sticky(ev);
    if (!peer_) return ev.type == EventType::EOS || ev.type == EventType::STREAM_START ||
                        ev.type == EventType::SEGMENT || ev.type == EventType::CAPS;
    Pad* sink = peer_;
    if (ev.type == EventType::EOS) {
      if (sink->eos_.exchange(true)) return true;  // already EOS
    }
    if (ev.type == EventType::FLUSH_START) sink->flushing_.store(true);
    if (ev.type == EventType::FLUSH_STOP) {
      sink->flushing_.store(false);
      sink->eos_.store(false);
    }
    if (ev.type == EventType::CAPS) sink->set_current_caps(ev.caps);
    sink->store_sticky(ev);
    return sink->parent()->sink_event(sink, ev);
  }
  // sink pad: upstream
  if (!peer_) return false;
  return peer_->parent()->src_event(peer_, ev);
}

Caps Pad::peer_query_caps(const Caps* filter) {
  if (!peer_) return filter ? *filter : Caps::Any();
  return peer_->query_caps(filter);
}

bool Pad::peer_accept_caps(const Caps& caps) {
  if (!peer_) return true;
  return peer_->parent()->accept_caps(peer_, caps);
}

Caps Pad::query_caps(const Caps* filter) { return parent_->query_caps(this, filter); }

bool Pad::link(Pad* src, Pad* sink) {
  if (!src || !sink) return false;
  if (src->dir_ != PadDirection::SRC || sink->dir_ != PadDirection::SINK) return false;
  if (src->peer_ || sink->peer_) return false;
  src->peer_ = sink;
  sink->peer_ = src;
  return true;
}

void Pad::unlink(Pad* src, Pad* sink) {
  if (src && src->peer_ == sink) src->peer_ = nullptr;
  if (sink && sink->peer_ == src) sink->peer_ = nullptr;
}

// -------------------------------------------------------------- Element ----

Element::Element(const std::string& factory, const std::string& name) : name_(name), factory_(factory) {
  prop_string("name", &name_, "The name of the object");
  prop_bool("silent", &silent_, "Produce verbose output");
}

Element::~Element() = default;

Pad* Element::get_pad(const std::string& name) const {
  for (const auto& p : pads_)
    if (p->name() == name) return p.get();
  return nullptr;
}

std::vector<Pad*> Element::src_pads() const {
  std::vector<Pad*> v;
  for (const auto& p : pads_)
    if (p->direction() == PadDirection::SRC) v.push_back(p.get());
  return v;
}

std::vector<Pad*> Element::sink_pads() const {
  std::vector<Pad*> v;
  for (const auto& p : pads_)
    if (p->direction() == PadDirection::SINK) v.push_back(p.get());
  return v;
}

Pad* Element::src_pad(size_t i) const {
  auto v = src_pads();
  return i < v.size() ? v[i] : nullptr;
}

Pad* Element::sink_pad(size_t i) const {
  auto v = sink_pads();
  return i < v.size() ? v[i] : nullptr;
}

Pad* Element::add_pad(const std::string& name, PadDirection dir, const Caps& caps) {
  pads_.push_back(std::make_unique<Pad>(this, name, dir, caps));
  return pads_.back().get();
}

void Element::remove_pad(Pad* pad) {
  if (pad->peer()) {
    if (pad->direction() == PadDirection::SRC)
      Pad::unlink(pad, pad->peer());
    else
      Pad::unlink(pad->peer(), pad);
  }
  pads_.erase(std::remove_if(pads_.begin(), pads_.end(), [&](auto& p) { return p.get() == pad; }), pads_.end());
}

void Element::add_template(const std::string& name_template, PadDirection dir, PadPresence pres, const Caps& caps) {
  templates_.push_back(PadTemplate{name_template, dir, pres, caps});
  if (pres == PadPresence::ALWAYS) add_pad(name_template, dir, caps);
}

const PadTemplate* Element::find_template(const std::string& name, PadDirection dir) const {
  for (const auto& t : templates_) {
    if (t.direction != dir) continue;
    if (t.name_template == name) return &t;
    auto pct = t.name_template.find('%');
    if (pct != std::string::npos && starts_with(name, t.name_template.substr(0, pct))) return &t;
  }
  return nullptr;
}

Pad* Element::request_pad(const PadTemplate& templ, const std::string& name) {
  std::string n = name;
  if (n.empty()) {
    auto pct = templ.name_template.find('%');
    std::string prefix = templ.name_template.substr(0, pct);
    // lowest unused index
    for (int i = 0;; ++i) {
      std::string cand = prefix + std::to_string(i);
      if (!get_pad(cand)) {
        n = cand;
        break;
      }
    }
  } else if (get_pad(n)) {
    return nullptr;
  }
  return add_pad(n, templ.direction, templ.caps);
}

void Element::release_pad(Pad* pad) { remove_pad(pad); }

Pad* Element::get_compatible_pad(PadDirection dir, const std::string& hint) {
  if (!hint.empty()) {
    if (Pad* p = get_pad(hint)) return (p->direction() == dir && !p->is_linked()) ? p : nullptr;
    if (const PadTemplate* t = find_template(hint, dir)) {
      // request pads, and sometimes-pads named explicitly in a link (delayed linking)
      if (t->presence != PadPresence::ALWAYS) return request_pad(*t, hint.find('%') == std::string::npos ? hint : "");
    }
    return nullptr;
  }
  for (const auto& p : pads_)
    if (p->direction() == dir && !p->is_linked()) return p.get();
  for (const auto& t : templates_)
    if (t.direction == dir && t.presence == PadPresence::REQUEST) return request_pad(t, "");
  return nullptr;
}

// ----------------------------------------------------------- properties ----

PropSpec& Element::add_prop(PropSpec spec) {
  for (auto& p : props_) {
    if (p.name == spec.name) {
      p = std::move(spec);
      return p;
    }
  }
  props_.push_back(std::move(spec));
  return props_.back();
}

const PropSpec* Element::find_property(const std::string& name) const {
  std::string n = replace_all(name, "_", "-");
  for (const auto& p : props_)
    if (p.name == n || p.name == name) return &p;
  return nullptr;
}

bool Element::has_property(const std::string& name) const { return find_property(name) != nullptr; }

std::vector<std::string> Element::property_names() const {
  std::vector<std::string> v;
  for (const auto& p : props_) v.push_back(p.name);
  return v;
}

void Element::set_property(const std::string& name, const std::string& value) {
  const PropSpec* p = find_property(name);
  if (!p) throw Error(strfmt("no property \"", name, "\" in element \"", name_, "\" (", factory_, ")"));
  if (!p->writable || !p->set) throw Error(strfmt("property \"", name, "\" of ", name_, " is not writable"));
  p->set(value);
}

std::string Element::get_property(const std::string& name) const {
  const PropSpec* p = find_property(name);
  if (!p) throw Error(strfmt("no property \"", name, "\" in element \"", name_, "\" (", factory_, ")"));
  if (!p->get) return "";
  return p->get();
}

void Element::prop_string(const std::string& name, std::string* target, const std::string& blurb,
                          std::function<void()> on_change) {
  PropSpec s;
  s.name = name;
  s.type = PropType::STRING;
  s.blurb = blurb;
  s.default_value = *target;
  s.set = [target, on_change](const std::string& v) {
    *target = v;
    if (on_change) on_change();
  };
  s.get = [target] { return *target; };
  add_prop(std::move(s));
}

void Element::prop_int(const std::string& name, int64_t* target, const std::string& blurb,
                       std::function<void()> on_change) {
  PropSpec s;
  s.name = name;
  s.type = PropType::INT64;
  s.blurb = blurb;
  s.default_value = std::to_string(*target);
  s.set = [target, on_change, name](const std::string& v) {
    *target = to_int(v, *target);
    if (on_change) on_change();
  };
  s.get = [target] { return std::to_string(*target); };
  add_prop(std::move(s));
}

void Element::prop_int(const std::string& name, int* target, const std::string& blurb,
                       std::function<void()> on_change) {
  PropSpec s;
  s.name = name;
  s.type = PropType::INT;
  s.blurb = blurb;
  s.default_value = std::to_string(*target);
  s.set = [target, on_change](const std::string& v) {
    *target = static_cast<int>(to_int(v, *target));
    if (on_change) on_change();
  };
  s.get = [target] { return std::to_string(*target); };
  add_prop(std::move(s));
}

void Element::prop_uint(const std::string& name, unsigned* target, const std::string& blurb,
                        std::function<void()> on_change) {
  PropSpec s;
  s.name = name;
  s.type = PropType::UINT;
  s.blurb = blurb;
  s.default_value = std::to_string(*target);
  s.set = [target, on_change](const std::string& v) {
    *target = static_cast<unsigned>(to_uint(v, *target));
    if (on_change) on_change();
  };
  s.get = [target] { return std::to_string(*target); };
  add_prop(std::move(s));
}

void Element::prop_bool(const std::string& name, bool* target, const std::string& blurb,
                        std::function<void()> on_change) {
  PropSpec s;
  s.name = name;
  s.type = PropType::BOOL;
  s.blurb = blurb;
  s.default_value = *target ? "true" : "false";
  s.set = [target, on_change](const std::string& v) {
    *target = to_bool(v, *target);
    if (on_change) on_change();
  };
  s.get = [target] { return std::string(*target ? "true" : "false"); };
  add_prop(std::move(s));
}

void Element::prop_double(const std::string& name, double* target, const std::string& blurb,
                          std::function<void()> on_change) {
  PropSpec s;
  s.name = name;
  s.type = PropType::DOUBLE;
  s.blurb = blurb;
  s.default_value = std::to_string(*target);
  s.set = [target, on_change](const std::string& v) {
    *target = to_double(v, *target);
    if (on_change) on_change();
  };
  s.get = [target] {
    char buf[64];
    snprintf(buf, sizeof(buf), "%g", *target);
    return std::string(buf);
  };
  add_prop(std::move(s));
}

void Element::prop_enum(const std::string& name, int* target, const std::vector<std::string>& nicks,
                        const std::string& blurb, std::function<void()> on_change) {
  PropSpec s;
  s.name = name;
  s.type = PropType::ENUM;
  s.blurb = blurb;
  s.choices = nicks;
  s.default_value = (*target >= 0 && *target < static_cast<int>(nicks.size())) ? nicks[*target] : "";
  s.set = [target, nicks, on_change, name](const std::string& v) {
    std::string t = strip(v);
    for (size_t i = 0; i < nicks.size(); ++i) {
      if (lower(nicks[i]) == lower(t)) {
        *target = static_cast<int>(i);
        if (on_change) on_change();
        return;
      }
    }
    char* end = nullptr;
    long iv = std::strtol(t.c_str(), &end, 10);
    if (!t.empty() && *end == '\0' && iv >= 0 && iv < static_cast<long>(nicks.size())) {
      *target = static_cast<int>(iv);
      if (on_change) on_change();
      return;
    }
    throw Error(strfmt("invalid value '", v, "' for enum property ", name));
  };
  s.get = [target, nicks] {
    return (*target >= 0 && *target < static_cast<int>(nicks.size())) ? nicks[*target] : std::string();
  };
  add_prop(std::move(s));
}

void Element::prop_readonly(const std::string& name, std::function<std::string()> get, const std::string& blurb) {
  PropSpec s;
  s.name = name;
  s.type = PropType::STRING;
  s.blurb = blurb;
  s.writable = false;
  s.get = std::move(get);
  add_prop(std::move(s));
}

// -------------------------------------------------------------- signals ----

int Element::connect(const std::string& signal, SignalHandler h) {
  std::lock_guard<std::mutex> lk(sig_mu_);
  int id = next_sig_id_++;
  signals_[signal].emplace_back(id, std::move(h));
  return id;
}

void Element::disconnect(int id) {
  std::lock_guard<std::mutex> lk(sig_mu_);
  for (auto& kv : signals_) {
    auto& v = kv.second;
    v.erase(std::remove_if(v.begin(), v.end(), [id](auto& x) { return x.first == id; }), v.end());
  }
}

bool Element::has_handlers(const std::string& signal) const {
  std::lock_guard<std::mutex> lk(sig_mu_);
  auto it = signals_.find(signal);
  return it != signals_.end() && !it->second.empty();
}

void Element::emit(const std::string& signal, const SignalArgs& args) {
  std::vector<SignalHandler> hs;
  {
    std::lock_guard<std::mutex> lk(sig_mu_);
    auto it = signals_.find(signal);
    if (it == signals_.end()) return;
    for (auto& x : it->second) hs.push_back(x.second);
  }
  for (auto& h : hs) h(this, args);
}

// ------------------------------------------------------------ lifecycle ----

bool Element::change_state(State target) {
  while (state_ != target) {
    if (target > state_) {
      State next = static_cast<State>(static_cast<int>(state_) + 1);
      bool ok = true;
      if (next == State::READY) {
        ok = open();
      } else if (next == State::PAUSED) {
        flushing_.store(false);
        for (auto& p : pads_) {
          p->set_flushing(false);
          p->set_eos(false);
        }
        unlock_stop();
        ok = start();
      } else if (next == State::PLAYING) {
        play();
      }
      if (!ok) return false;
      state_ = next;
    } else {
      State next = static_cast<State>(static_cast<int>(state_) - 1);
      if (next == State::PAUSED) {
        pause();
      } else if (next == State::READY) {
        flushing_.store(true);
        for (auto& p : pads_) p->set_flushing(true);
        unlock();
        stop();
      } else if (next == State::NULL_) {
        close();
      }
      state_ = next;
    }
  }
  return true;
}

FlowReturn Element::chain(Pad*, BufferPtr) { return FlowReturn::NOT_LINKED; }

bool Element::sink_event(Pad*, Event& ev) {
  if (ev.type == EventType::CAPS) {
    // default pass-through: same caps on every src pad
    bool ok = true;
    for (Pad* p : src_pads()) ok &= p->push_event(ev);
    return ok;
  }
  return forward_event_downstream(ev);
}

bool Element::src_event(Pad*, Event& ev) { return forward_event_upstream(ev); }

Caps Element::query_caps(Pad* pad, const Caps* filter) {
  // default: pass-through elements intersect the far side's caps with the template
  Caps result = pad->template_caps();
  std::vector<Pad*> others = pad->direction() == PadDirection::SINK ? src_pads() : sink_pads();
  for (Pad* o : others) {
    if (!o->is_linked()) continue;
    Caps peer = o->peer_query_caps(nullptr);
    result = result.intersect(peer);
  }
  if (filter) result = result.intersect(*filter);
  return result;
}

bool Element::accept_caps(Pad* pad, const Caps& caps) { return query_caps(pad, nullptr).can_intersect(caps); }

bool Element::query_latency(Pad* pad, bool* live, int64_t* min_lat, int64_t* max_lat) {
  // default: forward upstream through the first sink pad
  (void)pad;
  Pad* s = sink_pad(0);
  if (!s || !s->peer()) return true;
  return s->peer()->parent()->query_latency(s->peer(), live, min_lat, max_lat);
}

bool Element::forward_event_downstream(Event& ev) {
  bool ok = true;
  for (Pad* p : src_pads()) {
    Event e = ev;
    ok &= p->push_event(e);
  }
  return ok;
}

bool Element::forward_event_upstream(Event& ev) {
  bool ok = true;
  for (Pad* p : sink_pads()) {
    Event e = ev;
    ok &= p->push_event(e);
  }
  return ok;
}

FlowReturn Element::push_all(BufferPtr buf) {
  FlowReturn ret = FlowReturn::NOT_LINKED;
  bool any_ok = false;
  for (Pad* p : src_pads()) {
    FlowReturn r = p->push(buf);
    if (flow_ok(r)) any_ok = true;
    else if (r != FlowReturn::NOT_LINKED) ret = r;
  }
  return any_ok ? FlowReturn::OK : ret;
}

void Element::post_error(const std::string& msg) {
  NNSX_LOGE(name_, msg);
  if (pipeline_) pipeline_->bus().post(Message{MessageType::ERROR, name_, msg, Structure("error"), now_ns()});
}

void Element::post_warning(const std::string& msg) {
  NNSX_LOGW(name_, msg);
  if (pipeline_) pipeline_->bus().post(Message{MessageType::WARNING, name_, msg, Structure("warning"), now_ns()});
}

void Element::post_info(const std::string& msg) {
  if (pipeline_) pipeline_->bus().post(Message{MessageType::INFO, name_, msg, Structure("info"), now_ns()});
}

void Element::post_element_message(const Structure& s) {
  if (pipeline_) pipeline_->bus().post(Message{MessageType::ELEMENT, name_, s.to_string(), s, now_ns()});
}

void Element::post_latency() {
  if (pipeline_) pipeline_->bus().post(Message{MessageType::LATENCY, name_, "", Structure("latency"), now_ns()});
}

int64_t Element::base_time() const { return pipeline_ ? pipeline_->base_time_ns() : 0; }

int64_t Element::running_time() const { return pipeline_ ? now_ns() - pipeline_->base_time_ns() : now_ns(); }

bool Element::wait_until_running_time(int64_t t) {
  if (t < 0) return true;
  // sleep to within kSpinNs of the deadline, then yield-spin: a plain sleep
  // overshoots by the timer slack (50 us by default on Linux) plus the
  // wake-up latency, which a live source would add to every frame's latency
  constexpr int64_t kSpinNs = 150000;
  while (!flushing_.load()) {
    int64_t now = running_time();
    if (now >= t) return true;
    if (t - now <= kSpinNs) {
      std::this_thread::yield();
      continue;
    }
    int64_t d = std::min<int64_t>(t - now - kSpinNs, 5000000);  // re-check flushing every 5 ms
    std::this_thread::sleep_for(std::chrono::nanoseconds(d));
  }
  return false;
}

// ----------------------------------------------------------------- Task ----

void Task::start() {
  if (running_.load()) return;
  stop_.store(false);
  running_.store(true);
  th_ = std::thread([this] {
    while (!stop_.load()) {
      bool cont = false;
      try {
        cont = fn_();
      } catch (const std::exception& e) {
        NNSX_LOGE("task", e.what());
        cont = false;
      }
      if (!cont) break;
    }
    running_.store(false);
  });
}

void Task::join() {
  if (th_.joinable()) {
    if (th_.get_id() == std::this_thread::get_id()) {
      th_.detach();
    } else {
      th_.join();
    }
  }
  running_.store(false);
}

}  // namespace nnsx
