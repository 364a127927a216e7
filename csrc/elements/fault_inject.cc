// fault_inject: pass-through element that injects the failures the reference
// tests provoke with fake filters (tests/nnstreamer_example/custom_example_
// framecounter `custom=delay-N`, drop_buffer, invalid hosts in
// unittest_edge.cc:88): latency, dropped frames, a failing element, an early
// EOS and a thrown exception (which the runtime must turn into a bus error).
//
//   ... ! fault_inject delay-ms=5 drop-every=10 fail-after=100 ! ...
#include <chrono>
#include <random>
#include <thread>

#include "elements/elements.h"
#include "runtime/base.h"
#include "runtime/pipeline.h"

namespace nnsx {

namespace {

class FaultInject : public BaseTransform {
 public:
  explicit FaultInject(const std::string& name)
      : BaseTransform("fault_inject", name, Caps::Any(), Caps::Any()) {
    prop_uint("delay-ms", &delay_ms_, "Sleep this long before passing each buffer (latency injection)");
    prop_uint("drop-every", &drop_every_, "Drop every N-th buffer (0 = never)");
    prop_double("drop-probability", &drop_p_, "Drop each buffer with this probability");
    prop_uint("seed", &seed_, "Random seed for drop-probability");
    prop_int("fail-after", &fail_after_, "Post an error and fail after N buffers (-1 = never)");
    prop_int("throw-after", &throw_after_, "Throw a C++ exception after N buffers (-1 = never)");
    prop_int("eos-after", &eos_after_, "End the stream after N buffers (-1 = never)");
    prop_readonly("passed", [this] { return std::to_string(passed_); }, "Buffers passed");
    prop_readonly("dropped", [this] { return std::to_string(dropped_); }, "Buffers dropped");
  }

 protected:
  Caps transform_caps(PadDirection, const Caps& caps, const Caps* filter) override {
    return filter ? caps.intersect(*filter) : caps;
  }
  bool set_caps(const Caps&, const Caps&) override {
    rng_.seed(seed_);
    seen_ = passed_ = dropped_ = 0;
    return true;
  }
  FlowReturn transform(const BufferPtr& in, BufferPtr* out) override {
    const int64_t n = seen_++;
    if (fail_after_ >= 0 && n >= fail_after_) {
      post_error(strfmt("fault_inject: injected failure at buffer ", n));
      return FlowReturn::ERROR;
    }
    if (throw_after_ >= 0 && n >= throw_after_) throw Error(strfmt("fault_inject: injected exception at buffer ", n));
    if (eos_after_ >= 0 && n >= eos_after_) return FlowReturn::EOS;
    if (delay_ms_) std::this_thread::sleep_for(std::chrono::milliseconds(delay_ms_));
    const bool drop = (drop_every_ && (n + 1) % drop_every_ == 0) ||
                      (drop_p_ > 0 && std::uniform_real_distribution<double>(0, 1)(rng_) < drop_p_);
    if (drop) {
      ++dropped_;
      *out = nullptr;
      return FlowReturn::OK;
    }
    ++passed_;
    *out = in;  // zero-copy pass-through
    return FlowReturn::OK;
  }

 private:
  unsigned delay_ms_ = 0, drop_every_ = 0, seed_ = 0;
  double drop_p_ = 0.0;
  int64_t fail_after_ = -1, throw_after_ = -1, eos_after_ = -1;
  int64_t seen_ = 0, passed_ = 0, dropped_ = 0;
  std::mt19937 rng_;
};

}  // namespace

void register_fault_inject() {
  register_element("fault_inject", "Filter/Debug", "Injects latency, drops, errors and early EOS (testing)",
                   [](const std::string& n) { return std::make_unique<FaultInject>(n); });
}

}  // namespace nnsx
