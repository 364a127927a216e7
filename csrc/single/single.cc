#include "single/single.h"

#include <sys/stat.h>

#include <chrono>
#include <exception>

#include "core/log.h"
#include "core/util.h"
#include "runtime/pipeline.h"
#include "runtime/hip_util.h"

namespace nnsx {

SingleShot::SingleShot(const SingleOptions& opt) {
  ensure_builtin_elements();  // registers the built-in filter frameworks
  props_.model_files = opt.models;
  props_.input_info = opt.input_info;
  props_.output_info = opt.output_info;
  props_.input_configured = opt.input_info.num_tensors > 0;
  props_.output_configured = opt.output_info.num_tensors > 0;
  props_.accl_str = opt.accelerator;
  props_.custom_properties = opt.custom;
  std::string err;
  fw_ = resolve_filter_framework(opt.framework, &props_, opt.device, &err);
  if (!fw_) throw Error("single: " + err);
  if (fw_->verify_model_path())
    for (auto& m : props_.model_files)
      if (struct stat st; ::stat(m.c_str(), &st) != 0) throw Error("single: model file '" + m + "' does not exist");
  {
    hip::DeviceGuard g(props_.device);
    inst_ = fw_->open(props_);
  }
  if (!inst_) throw Error("single: framework '" + props_.fwname + "' failed to open the model");
  TensorsInfo in, out;
  if (inst_->get_model_info(&in, &out)) {
    in_ = in;
    out_ = out;
  } else {
    in_ = props_.input_info;
    out_ = props_.output_info;
  }
  // the model cannot tell its input: the user-given input info decides the output one
  if (props_.input_configured && !(in_ == props_.input_info)) {
    TensorsInfo o;
    if (inst_->set_input_info(props_.input_info, &o)) {
      in_ = props_.input_info;
      out_ = o;
    }
  }
  if (props_.device >= 0) stream_ = hip::stream_create(props_.device);
}

SingleShot::~SingleShot() {
  try {
    close();
  } catch (...) {
  }
}

void SingleShot::close() {
  {
    std::lock_guard<std::mutex> lk(wmu_);
    quit_ = true;
  }
  wcv_.notify_all();
  if (worker_.joinable()) worker_.join();
  std::lock_guard<std::mutex> lk(invoke_mu_);
  inst_.reset();
  if (stream_) {
    hip::stream_destroy(props_.device, stream_);
    stream_ = nullptr;
  }
}

void SingleShot::set_input_info(const TensorsInfo& in) {
  std::lock_guard<std::mutex> lk(invoke_mu_);
  if (!inst_) throw Error("single: handle is closed");
  if (in == in_) return;
  TensorsInfo out;
  if (!inst_->set_input_info(in, &out)) throw Error("single: the model does not accept input " + in.to_string());
  in_ = in;
  out_ = out;
}

std::vector<MemoryPtr> SingleShot::run(const std::vector<MemoryPtr>& in, TensorsInfo* out_info) {
  std::lock_guard<std::mutex> lk(invoke_mu_);
  if (!inst_) throw Error("single: handle is closed");
  if (in_.num_tensors > 0) {
    if (in.size() != in_.num_tensors)
      throw Error(strfmt("single: expected ", in_.num_tensors, " input tensors, got ", in.size()));
    for (unsigned i = 0; i < in_.num_tensors; ++i)
      if (in_.at(i).valid() && in[i]->size() != in_.size(static_cast<int>(i)))
        throw Error(strfmt("single: input ", i, " has ", in[i]->size(), " bytes, the model expects ",
                           in_.size(static_cast<int>(i))));
  }
  InvokeContext ctx;
  ctx.device = props_.device;
  ctx.stream = stream_;
  TensorsInfo dyn;
  ctx.out_info = &dyn;
  std::vector<MemoryPtr> outs;
  int ret;
  {
    hip::DeviceGuard g(props_.device);
    ret = inst_->invoke(in, &outs, ctx);
    if (stream_) hip::check(hipStreamSynchronize(stream_), "single: invoke sync");
  }
  if (ret < 0) throw Error(strfmt("single: invoke failed (", ret, ")"));
  if (out_info) *out_info = dyn.num_tensors ? dyn : out_;
  return outs;
}

void SingleShot::worker_loop() {
  std::unique_lock<std::mutex> lk(wmu_);
  while (true) {
    wcv_.wait(lk, [&] { return quit_ || job_; });
    if (!job_) return;  // quit with nothing pending
    auto job = std::move(job_);
    job_ = nullptr;
    lk.unlock();
    job();
    lk.lock();
    busy_ = false;
    wcv_.notify_all();
  }
}

std::vector<MemoryPtr> SingleShot::invoke(const std::vector<MemoryPtr>& in, TensorsInfo* out_info) {
  if (timeout_ms_ == 0) return run(in, out_info);
  struct Result {
    std::vector<MemoryPtr> out;
    TensorsInfo info;
    std::exception_ptr err;
    bool done = false;
  };
  auto res = std::make_shared<Result>();
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms_);
  std::unique_lock<std::mutex> lk(wmu_);
  if (!worker_.joinable()) worker_ = std::thread([this] { worker_loop(); });
  // a previous timed-out invoke may still be running: wait for it within the budget
  if (!wcv_.wait_until(lk, deadline, [&] { return !busy_; }))
    throw TimeoutError("single: the previous invoke is still running");
  busy_ = true;
  job_ = [this, in, res] {
    try {
      res->out = run(in, &res->info);
    } catch (...) {
      res->err = std::current_exception();
    }
    std::lock_guard<std::mutex> g(wmu_);
    res->done = true;
  };
  wcv_.notify_all();
  if (!wcv_.wait_until(lk, deadline, [&] { return res->done; }))
    throw TimeoutError(strfmt("single: invoke timed out after ", timeout_ms_, " ms"));
  if (res->err) std::rethrow_exception(res->err);
  if (out_info) *out_info = res->info;
  return res->out;
}

}  // namespace nnsx
