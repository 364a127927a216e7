// Pipeline (bin + clock + bus + state machine) and the element factory
// registry.  `parse_launch` accepts gst-launch syntax (see launch.cc).
#pragma once

#include <chrono>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "runtime/element.h"

namespace nnsx {

enum class MessageType { EOS, ERROR, WARNING, INFO, ELEMENT, STATE_CHANGED, LATENCY, STREAM_START, APPLICATION, QOS };
const char* message_type_name(MessageType t);

struct Message {
  MessageType type = MessageType::INFO;
  std::string src;
  std::string text;
  Structure structure;
  int64_t timestamp = 0;
};

class Bus {
 public:
  void post(Message m);
  // Wait for a message whose type is in mask (empty = any).  timeout_ns < 0 waits forever.
  bool pop(Message* out, int64_t timeout_ns, const std::vector<MessageType>& types = {});
  bool peek_any(const std::vector<MessageType>& types) const;
  std::vector<Message> drain();
  void set_sync_handler(std::function<void(const Message&)> h) { sync_handler_ = std::move(h); }
  void clear();

 private:
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Message> q_;
  std::function<void(const Message&)> sync_handler_;
};

class Pipeline : public Element {
 public:
  explicit Pipeline(const std::string& name = "pipeline0");
  ~Pipeline() override;

  Element* add(std::unique_ptr<Element> e);
  Element* get_by_name(const std::string& name) const;
  std::vector<Element*> elements() const;
  // link with pad names (empty = any compatible) and optional caps filter string
  bool link(Element* src, const std::string& srcpad, Element* sink, const std::string& sinkpad,
            const std::string& caps_filter = "");

  bool set_state(State s);
  State get_state() const { return state_; }
  Bus& bus() { return bus_; }

  // run until EOS or error; returns true on EOS.  timeout_ns < 0 = forever.
  bool run_until_eos(int64_t timeout_ns = -1, std::string* error = nullptr);
  void send_eos();  // inject EOS at every source

  int64_t base_time_ns() const { return base_time_; }
  int64_t clock_time_ns() const { return now_ns(); }

  // called by sinks
  void sink_reached_eos(Element* sink);
  std::string dot() const;  // graph description (GST_DEBUG_DUMP_DOT_DIR analogue)
  void dump_dot() const;    // to $NNSX_DEBUG_DUMP_DOT_DIR when set

 private:
  std::vector<std::unique_ptr<Element>> elems_;
  Bus bus_;
  int64_t base_time_ = 0;
  std::mutex eos_mu_;
  std::map<std::string, bool> eos_sinks_;
  bool eos_posted_ = false;
};

// ------------------------------------------------------------- registry ----

using ElementFactory = std::function<std::unique_ptr<Element>(const std::string& name)>;

struct FactoryInfo {
  std::string name;
  std::string klass;        // "Filter/Tensor", "Source", ...
  std::string description;
  ElementFactory make;
};

void register_element(const std::string& name, const std::string& klass, const std::string& desc,
                      ElementFactory f);
std::unique_ptr<Element> make_element(const std::string& factory, const std::string& name = "");
std::vector<FactoryInfo> list_elements();
bool element_exists(const std::string& factory);
void ensure_builtin_elements();  // idempotent registration of everything built in

// gst_parse_launch equivalent
std::unique_ptr<Pipeline> parse_launch(const std::string& description);

}  // namespace nnsx
