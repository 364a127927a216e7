#include "runtime/pipeline.h"

#include <algorithm>
#include <set>

#include "core/log.h"

namespace nnsx {

const char* message_type_name(MessageType t) {
  switch (t) {
    case MessageType::EOS: return "eos";
    case MessageType::ERROR: return "error";
    case MessageType::WARNING: return "warning";
    case MessageType::INFO: return "info";
    case MessageType::ELEMENT: return "element";
    case MessageType::STATE_CHANGED: return "state-changed";
    case MessageType::LATENCY: return "latency";
    case MessageType::STREAM_START: return "stream-start";
    case MessageType::APPLICATION: return "application";
    case MessageType::QOS: return "qos";
  }
  return "?";
}

// ------------------------------------------------------------------ Bus ----

void Bus::post(Message m) {
  if (sync_handler_) sync_handler_(m);
  {
    std::lock_guard<std::mutex> lk(mu_);
    q_.push_back(std::move(m));
    if (q_.size() > 100000) q_.pop_front();  // unbounded posting must not eat memory
  }
  cv_.notify_all();
}

bool Bus::pop(Message* out, int64_t timeout_ns, const std::vector<MessageType>& types) {
  std::unique_lock<std::mutex> lk(mu_);
  auto match = [&](const Message& m) {
    return types.empty() || std::find(types.begin(), types.end(), m.type) != types.end();
  };
  auto find = [&]() -> bool {
    for (auto it = q_.begin(); it != q_.end(); ++it) {
      if (match(*it)) {
        *out = *it;
        q_.erase(it);
        return true;
      }
    }
    return false;
  };
  if (timeout_ns < 0) {
    cv_.wait(lk, [&] { return find(); });
    return true;
  }
  return cv_.wait_for(lk, std::chrono::nanoseconds(timeout_ns), [&] { return find(); });
}

bool Bus::peek_any(const std::vector<MessageType>& types) const {
  std::lock_guard<std::mutex> lk(mu_);
  for (const auto& m : q_)
    if (std::find(types.begin(), types.end(), m.type) != types.end()) return true;
  return false;
}

std::vector<Message> Bus::drain() {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<Message> v(q_.begin(), q_.end());
  q_.clear();
  return v;
}

void Bus::clear() {
  std::lock_guard<std::mutex> lk(mu_);
  q_.clear();
}

// ------------------------------------------------------------- Pipeline ----

Pipeline::Pipeline(const std::string& name) : Element("pipeline", name) {}

Pipeline::~Pipeline() {
  try {
    set_state(State::NULL_);
  } catch (...) {
  }
  // break links before elements die (pads reference each other)
  for (auto& e : elems_)
    for (const auto& p : e->pads())
      if (p->peer() && p->direction() == PadDirection::SRC) Pad::unlink(p.get(), p->peer());
  elems_.clear();
}

Element* Pipeline::add(std::unique_ptr<Element> e) {
  if (e->name().empty() || get_by_name(e->name())) {
    // auto-name like GStreamer: factory + counter
    int i = 0;
    std::string base = e->factory();
    while (get_by_name(base + std::to_string(i))) ++i;
    e->set_name(base + std::to_string(i));
  }
  e->set_pipeline(this);
  elems_.push_back(std::move(e));
  return elems_.back().get();
}

Element* Pipeline::get_by_name(const std::string& name) const {
  for (const auto& e : elems_)
    if (e->name() == name) return e.get();
  return nullptr;
}

std::vector<Element*> Pipeline::elements() const {
  std::vector<Element*> v;
  for (const auto& e : elems_) v.push_back(e.get());
  return v;
}

bool Pipeline::link(Element* src, const std::string& srcpad, Element* sink, const std::string& sinkpad,
                    const std::string& caps_filter) {
  if (!caps_filter.empty()) {
    auto cf = make_element("capsfilter");
    cf->set_property("caps", caps_filter);
    Element* c = add(std::move(cf));
    return link(src, srcpad, c, "", "") && link(c, "", sink, sinkpad, "");
  }
  Pad* sp = src->get_compatible_pad(PadDirection::SRC, srcpad);
  if (!sp) {
    NNSX_LOGE("pipeline", "no src pad '", srcpad, "' available on ", src->name());
    return false;
  }
  Pad* kp = sink->get_compatible_pad(PadDirection::SINK, sinkpad);
  if (!kp) {
    NNSX_LOGE("pipeline", "no sink pad '", sinkpad, "' available on ", sink->name());
    return false;
  }
  return Pad::link(sp, kp);
}

namespace {
// order: sinks first (downstream before upstream), by distance from the sinks
std::vector<Element*> sink_first_order(const std::vector<Element*>& elems) {
  std::map<Element*, int> depth;
  std::function<int(Element*, std::set<Element*>&)> dist = [&](Element* e, std::set<Element*>& seen) -> int {
    auto it = depth.find(e);
    if (it != depth.end()) return it->second;
    if (seen.count(e)) return 0;  // cycle (repo loops)
    seen.insert(e);
    int d = 0;
    for (Pad* p : e->src_pads())
      if (p->peer()) d = std::max(d, 1 + dist(p->peer()->parent(), seen));
    seen.erase(e);
    depth[e] = d;
    return d;
  };
  for (Element* e : elems) {
    std::set<Element*> seen;
    dist(e, seen);
  }
  std::vector<Element*> v = elems;
  std::stable_sort(v.begin(), v.end(), [&](Element* a, Element* b) { return depth[a] < depth[b]; });
  return v;
}
}  // namespace

bool Pipeline::set_state(State target) {
  std::vector<Element*> order = sink_first_order(elements());
  while (state_ != target) {
    if (target > state_) {
      State next = static_cast<State>(static_cast<int>(state_) + 1);
      if (next == State::PAUSED) {
        std::lock_guard<std::mutex> lk(eos_mu_);
        eos_sinks_.clear();
        eos_posted_ = false;
        for (Element* e : order)
          if (e->is_sink()) eos_sinks_[e->name()] = false;
      }
      if (next == State::PLAYING) base_time_ = now_ns();
      for (Element* e : order) {
        if (!e->change_state(next)) {
          post_error(strfmt("state change of ", e->name(), " to ", state_name(next), " failed"));
          return false;
        }
      }
      state_ = next;
      dump_dot();
    } else {
      State next = static_cast<State>(static_cast<int>(state_) - 1);
      if (next == State::READY) {
        // unblock everything first, then stop from the sources downwards
        for (Element* e : order) {
          for (const auto& p : e->pads()) p->set_flushing(true);
          e->unlock();
        }
        for (auto it = order.rbegin(); it != order.rend(); ++it) (*it)->change_state(next);
      } else {
        for (auto it = order.rbegin(); it != order.rend(); ++it) (*it)->change_state(next);
      }
      state_ = next;
    }
  }
  return true;
}

void Pipeline::sink_reached_eos(Element* sink) {
  bool post = false;
  {
    std::lock_guard<std::mutex> lk(eos_mu_);
    eos_sinks_[sink->name()] = true;
    bool all = true;
    for (auto& kv : eos_sinks_) all &= kv.second;
    if (all && !eos_posted_) {
      eos_posted_ = true;
      post = true;
    }
  }
  if (post) bus_.post(Message{MessageType::EOS, name(), "end of stream", Structure("eos"), now_ns()});
}

bool Pipeline::run_until_eos(int64_t timeout_ns, std::string* error) {
  if (state_ != State::PLAYING && !set_state(State::PLAYING)) {
    Message m;
    if (error && bus_.pop(&m, 0, {MessageType::ERROR})) *error = m.src + ": " + m.text;
    return false;
  }
  Message m;
  if (!bus_.pop(&m, timeout_ns, {MessageType::EOS, MessageType::ERROR})) {
    if (error) *error = "timeout";
    return false;
  }
  if (m.type == MessageType::ERROR) {
    if (error) *error = m.src + ": " + m.text;
    return false;
  }
  return true;
}

void Pipeline::send_eos() {
  for (auto& e : elems_) {
    if (e->is_source()) {
      Event ev = Event::make_eos();
      for (Pad* p : e->src_pads()) p->push_event(ev);
    }
  }
}

// NNSX_DEBUG_DUMP_DOT_DIR=<dir>: <dir>/<pipeline>.<state>.dot after each upward state change
void Pipeline::dump_dot() const {
  const char* dir = std::getenv("NNSX_DEBUG_DUMP_DOT_DIR");
  if (!dir || !*dir) return;
  const std::string path = strfmt(dir, "/", name(), ".", state_name(state_), ".dot");
  if (FILE* f = std::fopen(path.c_str(), "w")) {
    const std::string d = dot();
    std::fwrite(d.data(), 1, d.size(), f);
    std::fclose(f);
  }
}

std::string Pipeline::dot() const {
  std::string r = "digraph pipeline {\n  rankdir=LR;\n";
  for (const auto& e : elems_) r += strfmt("  \"", e->name(), "\" [label=\"", e->factory(), "\\n", e->name(), "\"];\n");
  for (const auto& e : elems_)
    for (Pad* p : e->src_pads())
      if (p->peer()) {
        std::string caps = p->has_current_caps() ? replace_all(p->current_caps().to_string(), "\"", "'") : "";
        r += strfmt("  \"", e->name(), "\" -> \"", p->peer()->parent()->name(), "\" [label=\"", p->name(), "->",
                    p->peer()->name(), "\\n", caps, "\"];\n");
      }
  return r + "}\n";
}

// ------------------------------------------------------------- registry ----

namespace {
std::mutex& reg_mu() {
  static std::mutex* m = new std::mutex();
  return *m;
}
std::map<std::string, FactoryInfo>& reg() {
  static auto* m = new std::map<std::string, FactoryInfo>();
  return *m;
}
}  // namespace

void register_element(const std::string& name, const std::string& klass, const std::string& desc,
                      ElementFactory f) {
  std::lock_guard<std::mutex> lk(reg_mu());
  reg()[name] = FactoryInfo{name, klass, desc, std::move(f)};
}

std::unique_ptr<Element> make_element(const std::string& factory, const std::string& name) {
  ensure_builtin_elements();
  ElementFactory f;
  {
    std::lock_guard<std::mutex> lk(reg_mu());
    auto it = reg().find(factory);
    if (it == reg().end()) throw Error("no element \"" + factory + "\"");
    f = it->second.make;
  }
  return f(name);
}

std::vector<FactoryInfo> list_elements() {
  ensure_builtin_elements();
  std::lock_guard<std::mutex> lk(reg_mu());
  std::vector<FactoryInfo> v;
  for (auto& kv : reg()) v.push_back(kv.second);
  return v;
}

bool element_exists(const std::string& factory) {
  ensure_builtin_elements();
  std::lock_guard<std::mutex> lk(reg_mu());
  return reg().count(factory) > 0;
}

}  // namespace nnsx
