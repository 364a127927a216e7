// Element / Pad / Event / Property: nnsx's own streaming runtime, replacing
// the GStreamer core the reference is built on (GstElement, GstPad,
// GstEvent, GObject properties and signals).  Push model: a source's
// streaming thread calls Pad::push, which runs the peer's chain() on the same
// thread; `queue` (and the collect-pads aggregators) start new threads.
#pragma once

#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "core/caps.h"
#include "core/util.h"
#include "runtime/memory.h"

namespace nnsx {

class Element;
class Pipeline;
class Pad;

enum class FlowReturn {
  CUSTOM_SUCCESS = 100,  // dropped on purpose (GST_BASE_TRANSFORM_FLOW_DROPPED)
  OK = 0,
  NOT_LINKED = -1,
  FLUSHING = -2,
  EOS = -3,
  NOT_NEGOTIATED = -4,
  ERROR = -5,
};
const char* flow_name(FlowReturn r);
inline bool flow_ok(FlowReturn r) { return r == FlowReturn::OK || r == FlowReturn::CUSTOM_SUCCESS; }

struct Segment {
  double rate = 1.0;
  int64_t start = 0;
  int64_t stop = -1;
  int64_t time = 0;
  int64_t position = 0;
  int64_t base = 0;
};

enum class EventType {
  STREAM_START,
  CAPS,
  SEGMENT,
  EOS,
  FLUSH_START,
  FLUSH_STOP,
  QOS,          // upstream
  LATENCY,      // upstream
  RECONFIGURE,  // upstream
  CUSTOM_DOWNSTREAM,
  CUSTOM_UPSTREAM,
  GAP,
  TAG,
};
const char* event_type_name(EventType t);
inline bool event_is_upstream(EventType t) {
  return t == EventType::QOS || t == EventType::LATENCY || t == EventType::RECONFIGURE ||
         t == EventType::CUSTOM_UPSTREAM;
}
inline bool event_is_serialized(EventType t) {
  return t != EventType::FLUSH_START && t != EventType::FLUSH_STOP && !event_is_upstream(t);
}

struct Event {
  EventType type = EventType::EOS;
  Caps caps;             // CAPS
  Segment segment;       // SEGMENT
  std::string stream_id; // STREAM_START
  // QOS: throttle/overflow/underflow
  std::string qos_type = "throttle";
  double proportion = 1.0;
  int64_t diff = 0;
  int64_t timestamp = -1;
  int64_t latency = 0;   // LATENCY
  Structure data;        // CUSTOM_* payload (name identifies it, e.g. "evt_update_model")

  static Event make_caps(const Caps& c) { Event e; e.type = EventType::CAPS; e.caps = c; return e; }
  static Event make_eos() { Event e; e.type = EventType::EOS; return e; }
  static Event make_segment(const Segment& s) { Event e; e.type = EventType::SEGMENT; e.segment = s; return e; }
  static Event make_stream_start(const std::string& id) {
    Event e; e.type = EventType::STREAM_START; e.stream_id = id; return e;
  }
  static Event make_custom(EventType t, const Structure& s) { Event e; e.type = t; e.data = s; return e; }
};

enum class PadDirection { SRC, SINK };
enum class PadPresence { ALWAYS, SOMETIMES, REQUEST };

struct PadTemplate {
  std::string name_template;  // "src", "sink_%u", "src_%u"
  PadDirection direction;
  PadPresence presence;
  Caps caps;
};

class Pad {
 public:
  Pad(Element* parent, std::string name, PadDirection dir, Caps templ);
  const std::string& name() const { return name_; }
  PadDirection direction() const { return dir_; }
  Element* parent() const { return parent_; }
  Pad* peer() const { return peer_; }
  bool is_linked() const { return peer_ != nullptr; }
  const Caps& template_caps() const { return templ_; }
  void set_template_caps(const Caps& c) { templ_ = c; }
  Caps current_caps() const;
  bool has_current_caps() const;
  void set_current_caps(const Caps& c);

  // src pads: push data/event downstream; sink pads: push_event goes upstream
  FlowReturn push(BufferPtr buf);
  bool push_event(Event ev);
  // Ask what the peer accepts (filter optional).
  Caps peer_query_caps(const Caps* filter = nullptr);
  // Ask the peer to accept caps
  bool peer_accept_caps(const Caps& caps);
  Caps query_caps(const Caps* filter = nullptr);  // this pad (delegates to the element)

  static bool link(Pad* src, Pad* sink);
  static void unlink(Pad* src, Pad* sink);

  bool eos() const { return eos_.load(); }
  void set_eos(bool v) { eos_.store(v); }
  bool flushing() const { return flushing_.load(); }
  void set_flushing(bool v) { flushing_.store(v); }
  FlowReturn last_flow() const { return last_flow_.load(); }
  // Sticky events replayed to a newly linked peer
  void store_sticky(const Event& e);
  std::vector<Event> sticky_events() const;
  int64_t user_data = 0;  // per-pad element scratch (pad index etc.)

 private:
  Element* parent_;
  std::string name_;
  PadDirection dir_;
  Caps templ_;
  Pad* peer_ = nullptr;
  mutable std::mutex caps_mu_;
  Caps caps_;
  bool has_caps_ = false;
  std::atomic<bool> eos_{false};
  std::atomic<bool> flushing_{false};
  std::atomic<FlowReturn> last_flow_{FlowReturn::OK};
  mutable std::mutex sticky_mu_;
  std::vector<Event> sticky_;
};

// --------------------------------------------------------------- props ----

enum class PropType { STRING, INT, UINT, INT64, UINT64, BOOL, DOUBLE, ENUM, FLAGS, FRACTION, CAPS, POINTER };

struct PropSpec {
  std::string name;
  PropType type = PropType::STRING;
  std::string blurb;
  std::string default_value;
  bool readable = true;
  bool writable = true;
  std::vector<std::string> choices;  // ENUM / FLAGS nicks
  std::function<void(const std::string&)> set;
  std::function<std::string()> get;
};

// Values handed to signal handlers
struct SignalArgs {
  BufferPtr buffer;
  std::string text;
  int64_t value = 0;
  Caps caps;
};
using SignalHandler = std::function<void(Element*, const SignalArgs&)>;

// -------------------------------------------------------------- element ----

enum class State { NULL_ = 0, READY = 1, PAUSED = 2, PLAYING = 3 };
const char* state_name(State s);

enum ElementFlags : uint32_t { ELEM_SOURCE = 1u << 0, ELEM_SINK = 1u << 1 };

class Element {
 public:
  Element(const std::string& factory, const std::string& name);
  virtual ~Element();

  const std::string& name() const { return name_; }
  void set_name(const std::string& n) { name_ = n; }
  const std::string& factory() const { return factory_; }
  Pipeline* pipeline() const { return pipeline_; }
  void set_pipeline(Pipeline* p) { pipeline_ = p; }
  uint32_t flags() const { return flags_; }
  bool is_source() const { return flags_ & ELEM_SOURCE; }
  bool is_sink() const { return flags_ & ELEM_SINK; }

  // pads
  const std::vector<std::unique_ptr<Pad>>& pads() const { return pads_; }
  Pad* get_pad(const std::string& name) const;
  Pad* get_static_pad(const std::string& name) const { return get_pad(name); }
  std::vector<Pad*> src_pads() const;
  std::vector<Pad*> sink_pads() const;
  Pad* src_pad(size_t i = 0) const;
  Pad* sink_pad(size_t i = 0) const;
  const std::vector<PadTemplate>& pad_templates() const { return templates_; }
  const PadTemplate* find_template(const std::string& name, PadDirection dir) const;
  // Request pad (sink_%u etc.); name may be empty to auto-number
  virtual Pad* request_pad(const PadTemplate& templ, const std::string& name);
  virtual void release_pad(Pad* pad);
  // Find or create a pad compatible for linking
  Pad* get_compatible_pad(PadDirection dir, const std::string& hint = "");

  // properties
  void set_property(const std::string& name, const std::string& value);
  std::string get_property(const std::string& name) const;
  bool has_property(const std::string& name) const;
  const PropSpec* find_property(const std::string& name) const;
  std::vector<std::string> property_names() const;
  const std::vector<PropSpec>& properties() const { return props_; }

  // signals
  int connect(const std::string& signal, SignalHandler h);
  void disconnect(int id);
  void emit(const std::string& signal, const SignalArgs& args);
  bool has_handlers(const std::string& signal) const;

  // ---- lifecycle (called by Pipeline) ----
  State state() const { return state_; }
  bool change_state(State target);
  virtual bool start() { return true; }   // READY -> PAUSED
  virtual bool stop() { return true; }    // PAUSED -> READY
  virtual bool open() { return true; }    // NULL -> READY
  virtual void close() {}                 // READY -> NULL
  virtual void play() {}                  // PAUSED -> PLAYING (sources start tasks)
  virtual void pause() {}                 // PLAYING -> PAUSED
  // unblock every wait in this element (flush / shutdown)
  virtual void unlock() {}
  virtual void unlock_stop() {}
  bool flushing() const { return flushing_.load(); }

  // ---- dataflow (overridden by elements) ----
  virtual FlowReturn chain(Pad* sinkpad, BufferPtr buf);
  virtual bool sink_event(Pad* sinkpad, Event& ev);  // downstream events arriving at a sink pad
  virtual bool src_event(Pad* srcpad, Event& ev);    // upstream events arriving at a src pad
  // caps this pad can handle given the far side's constraints
  virtual Caps query_caps(Pad* pad, const Caps* filter);
  virtual bool accept_caps(Pad* pad, const Caps& caps);
  // latency query: (live, min, max) accumulated
  virtual bool query_latency(Pad* pad, bool* live, int64_t* min_lat, int64_t* max_lat);

  // helpers for subclasses
  bool forward_event_downstream(Event& ev);  // to every src pad
  bool forward_event_upstream(Event& ev);    // to every sink pad
  FlowReturn push_all(BufferPtr buf);        // to every src pad
  void post_error(const std::string& msg);
  void post_warning(const std::string& msg);
  void post_info(const std::string& msg);
  void post_element_message(const Structure& s);
  void post_latency();
  // time (ns) of the pipeline clock relative to base time (running time)
  int64_t running_time() const;
  int64_t base_time() const;
  // pipeline-wide sync helper: wait until running-time `t` (for sync=true sinks)
  bool wait_until_running_time(int64_t t);

  bool silent() const { return silent_; }
  std::mutex& object_lock() { return obj_mu_; }

 protected:
  Pad* add_pad(const std::string& name, PadDirection dir, const Caps& caps);
  void add_template(const std::string& name_template, PadDirection dir, PadPresence pres, const Caps& caps);
  void remove_pad(Pad* pad);
  // property registration helpers
  PropSpec& add_prop(PropSpec spec);
  void prop_string(const std::string& name, std::string* target, const std::string& blurb,
                   std::function<void()> on_change = nullptr);
  void prop_int(const std::string& name, int64_t* target, const std::string& blurb,
                std::function<void()> on_change = nullptr);
  void prop_int(const std::string& name, int* target, const std::string& blurb,
                std::function<void()> on_change = nullptr);
  void prop_uint(const std::string& name, unsigned* target, const std::string& blurb,
                 std::function<void()> on_change = nullptr);
  void prop_bool(const std::string& name, bool* target, const std::string& blurb,
                 std::function<void()> on_change = nullptr);
  void prop_double(const std::string& name, double* target, const std::string& blurb,
                   std::function<void()> on_change = nullptr);
  void prop_enum(const std::string& name, int* target, const std::vector<std::string>& nicks,
                 const std::string& blurb, std::function<void()> on_change = nullptr);
  void prop_readonly(const std::string& name, std::function<std::string()> get, const std::string& blurb);

  std::string name_;
  std::string factory_;
  Pipeline* pipeline_ = nullptr;
  uint32_t flags_ = 0;
  std::vector<std::unique_ptr<Pad>> pads_;
  std::vector<PadTemplate> templates_;
  std::vector<PropSpec> props_;
  std::atomic<bool> flushing_{false};
  State state_ = State::NULL_;
  bool silent_ = true;
  mutable std::mutex obj_mu_;
  mutable std::mutex sig_mu_;
  std::map<std::string, std::vector<std::pair<int, SignalHandler>>> signals_;
  int next_sig_id_ = 1;
  int request_counter_ = 0;
};

// A streaming thread (GstTask).  The loop function runs until stop() or until it
// returns false.
class Task {
 public:
  explicit Task(std::function<bool()> iteration) : fn_(std::move(iteration)) {}
  ~Task() { join(); }
  void start();
  void request_stop() { stop_.store(true); }
  bool stop_requested() const { return stop_.load(); }
  void join();
  bool running() const { return running_.load(); }

 private:
  std::function<bool()> fn_;
  std::thread th_;
  std::atomic<bool> stop_{false};
  std::atomic<bool> running_{false};
};

}  // namespace nnsx
