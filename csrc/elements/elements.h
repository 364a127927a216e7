// Registration entry points and application-facing interfaces of built-in
// elements.
#pragma once

#include "runtime/element.h"

namespace nnsx {

void register_basic_elements();
void register_tensor_elements();   // converter/transform/sink/mux/demux/merge/split/...
void register_filter_elements();   // tensor_filter
void register_decoder_elements();  // tensor_decoder
void register_comm_elements();
void register_mqtt_elements();     // mqttsink / mqttsrc
void register_fault_inject();      // fault_inject (testing)
void register_grpc_elements();     // tensor_src_grpc / tensor_sink_grpc     // tensor_query_* / edge / mqtt-like
void register_extra_elements();    // crop/if/rate/repo/sparse/debug/trainer/iio/join/datarepo

// appsrc / appsink application API (implemented by the element classes)
class AppSrcIface {
 public:
  virtual ~AppSrcIface() = default;
  virtual FlowReturn push(BufferPtr buf) = 0;
  virtual FlowReturn end_of_stream() = 0;
  virtual void set_caps_string(const std::string& c) = 0;
  virtual size_t queued() = 0;
};

class AppSinkIface {
 public:
  virtual ~AppSinkIface() = default;
  virtual BufferPtr pull(int64_t timeout_ns) = 0;
  virtual bool is_eos() = 0;
  virtual Caps negotiated_caps() = 0;
};

// tensor_repo (global slot repository, gsttensor_repo.c) -- defined in repo.cc
class TensorRepo {
 public:
  static TensorRepo& get();
  // blocks while the slot is full (one-deep mailbox) unless flushing
  bool set_buffer(unsigned slot, BufferPtr buf, const Caps& caps);
  // blocks until data or EOS; returns nullptr on EOS/flush
  BufferPtr get_buffer(unsigned slot, Caps* caps, bool* eos, int64_t timeout_ns = -1);
  void set_eos(unsigned slot);
  void set_changed(unsigned slot, bool pushing);
  void reset(unsigned slot);
  void remove(unsigned slot);
  void flush(unsigned slot);
  size_t num_slots();

 private:
  TensorRepo() = default;
  struct Slot;
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<unsigned, std::shared_ptr<Slot>> slots_;
  std::shared_ptr<Slot> slot(unsigned i);
};

}  // namespace nnsx
