// Single-shot inference API (ML API "single": ml_single_open / invoke /
// set_input_info / set_timeout / close; reference tensor_filter_single.c and
// SURVEY.md section 3.6).  No pipeline: the filter framework is opened
// directly and invoked synchronously on the caller's buffers.
//
// MI355X notes: a GPU model keeps its weights resident in HBM for the life of
// the handle; each handle owns one HIP stream, and invoke() returns only after
// that stream has drained (outputs are ready on return, wherever they live).
// With a timeout the invoke runs on the handle's worker thread and the caller
// stops waiting after `timeout_ms` (the reference behaviour: the late result
// is discarded, the next invoke waits for the worker).
#pragma once

#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "runtime/plugin_api.h"

namespace nnsx {

struct SingleOptions {
  std::string framework = "auto";
  std::vector<std::string> models;
  TensorsInfo input_info, output_info;  // optional: the model's own info wins when it has one
  std::string accelerator;
  std::string custom;
  int device = -1;  // -1: LOCAL_RANK % #GPUs when the framework runs on the GPU
};

class SingleShot {
 public:
  explicit SingleShot(const SingleOptions& opt);
  ~SingleShot();
  SingleShot(const SingleShot&) = delete;
  SingleShot& operator=(const SingleShot&) = delete;

  const TensorsInfo& input_info() const { return in_; }
  const TensorsInfo& output_info() const { return out_; }
  const std::string& framework() const { return props_.fwname; }
  int device() const { return props_.device; }

  // ml_single_set_input_info: reconfigure for new input dims (SET_INPUT_INFO)
  void set_input_info(const TensorsInfo& in);
  // ml_single_invoke: one memory per input tensor, sizes checked against
  // input_info(); returns one memory per output tensor.  `out_info` receives the
  // actual output info (ml_single_invoke_dynamic).
  std::vector<MemoryPtr> invoke(const std::vector<MemoryPtr>& in, TensorsInfo* out_info = nullptr);
  void set_timeout(unsigned ms) { timeout_ms_ = ms; }
  unsigned timeout() const { return timeout_ms_; }
  void close();

 private:
  std::vector<MemoryPtr> run(const std::vector<MemoryPtr>& in, TensorsInfo* out_info);
  void worker_loop();

  FilterProperties props_;
  std::shared_ptr<FilterFramework> fw_;
  std::unique_ptr<FilterInstance> inst_;
  TensorsInfo in_, out_;
  hipStream_t stream_ = nullptr;
  unsigned timeout_ms_ = 0;
  std::mutex invoke_mu_;  // one invoke at a time per handle

  // timed invokes run here
  std::thread worker_;
  std::mutex wmu_;
  std::condition_variable wcv_;
  std::function<void()> job_;
  bool busy_ = false, quit_ = false;
};

}  // namespace nnsx
