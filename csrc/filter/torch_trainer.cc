// tensor_trainer framework=pytorch: on-device training of a TorchScript
// module with libtorch optimizers on PyTorch-ROCm.
//
// Reference behaviour: the trainer sub-plugin contract of
// gst/nnstreamer/include/nnstreamer_plugin_api_trainer.h:66-127 (create /
// start / push_data / getFrameworkInfo, completion signalled through a
// condition) and the nntrainer sub-plugin's sample accounting
// (ext/nnstreamer/tensor_trainer/tensor_trainer_nntrainer.cc: samples of one
// epoch = num-training-samples then num-validation-samples, repeated
// num-epochs times).  Samples are staged into a device batch; each full batch
// is one forward/backward/optimizer step on the GPU.
//
// model-config is a key=value file ([sections] and # comments ignored):
//   model = path/to/module.pt     TorchScript module: forward(x...) -> logits
//   loss = cross_entropy | mse | bce           (default cross_entropy)
//   optimizer = sgd | adam | adamw             (default sgd)
//   learning_rate = 0.01, momentum = 0, weight_decay = 0, batch_size = 32
//   seed = 0
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <torch/nn/functional/loss.h>
#include <torch/optim/adam.h>
#include <torch/optim/adamw.h>
#include <torch/optim/sgd.h>
#include <torch/script.h>

#include <condition_variable>
#include <fstream>

#include "core/log.h"
#include "filter/filter.h"
#include "filter/torch_util.h"
#include "runtime/hip_util.h"
#include "runtime/plugin_api.h"

namespace nnsx {

namespace {

namespace F = torch::nn::functional;

std::map<std::string, std::string> read_kv(const std::string& path) {
  std::map<std::string, std::string> kv;
  std::ifstream f(path);
  if (!f) throw Error("pytorch trainer: cannot read model-config '" + path + "'");
  std::string line;
  while (std::getline(f, line)) {
    auto h = line.find('#');
    if (h != std::string::npos) line = line.substr(0, h);
    line = strip(line);
    if (line.empty() || line[0] == '[') continue;
    auto eq = line.find('=');
    if (eq == std::string::npos) continue;
    kv[lower(strip(line.substr(0, eq)))] = strip(line.substr(eq + 1));
  }
  return kv;
}

class TorchTrainer : public TrainerInstance {
 public:
  explicit TorchTrainer(const TrainerProperties& p) : props_(p) {
    auto kv = read_kv(p.model_config);
    auto get = [&](const std::string& k, const std::string& d) {
      auto it = kv.find(k);
      return it == kv.end() ? d : it->second;
    };
    std::string model = get("model", "");
    if (!p.model_load_path.empty()) model = p.model_load_path;
    if (model.empty()) throw Error("pytorch trainer: model-config has no 'model' entry");
    if (model[0] != '/') {
      auto slash = p.model_config.rfind('/');
      if (slash != std::string::npos && !std::ifstream(model)) model = p.model_config.substr(0, slash + 1) + model;
    }
    loss_ = lower(get("loss", "cross_entropy"));
    batch_ = std::max<int64_t>(1, to_int(get("batch_size", "32")));
    double lr = to_double(get("learning_rate", "0.01"));
    double wd = to_double(get("weight_decay", "0"));
    torch::manual_seed(static_cast<uint64_t>(to_int(get("seed", "0"))));
    device_ = p.device >= 0 ? torch::Device(torch::kCUDA, static_cast<int8_t>(p.device)) : torch::Device(torch::kCPU);
    guard();
    module_ = torch::jit::load(model, device_);
    module_.train();
    std::vector<at::Tensor> params;
    for (const auto& t : module_.parameters()) {
      t.requires_grad_(true);
      params.push_back(t);
    }
    if (params.empty()) throw Error("pytorch trainer: module has no parameters");
    std::string opt = lower(get("optimizer", "sgd"));
    if (opt == "adam")
      optim_ = std::make_unique<torch::optim::Adam>(params, torch::optim::AdamOptions(lr).weight_decay(wd));
    else if (opt == "adamw")
      optim_ = std::make_unique<torch::optim::AdamW>(params, torch::optim::AdamWOptions(lr).weight_decay(wd));
    else if (opt == "sgd")
      optim_ = std::make_unique<torch::optim::SGD>(
          params, torch::optim::SGDOptions(lr).momentum(to_double(get("momentum", "0"))).weight_decay(wd));
    else
      throw Error("pytorch trainer: unknown optimizer '" + opt + "'");
    if (loss_ != "cross_entropy" && loss_ != "mse" && loss_ != "bce")
      throw Error("pytorch trainer: unknown loss '" + loss_ + "'");
  }

  bool start() override { return true; }
  bool stop() override {
    std::lock_guard<std::mutex> lk(mu_);
    stopped_ = true;
    cv_.notify_all();
    return true;
  }

  bool push_data(const std::vector<MemoryPtr>& tensors, bool is_validation) override {
    unsigned ni = props_.num_inputs, nl = props_.num_labels;
    if (tensors.size() < ni + nl) return false;
    guard();
    if (is_validation != staging_validation_) flush();  // phase change ends a partial batch
    staging_validation_ = is_validation;
    if (staged_.empty()) staged_.resize(ni + nl);
    for (unsigned i = 0; i < ni + nl; ++i) staged_[i].push_back(to_tensor(tensors[i], props_.input_info.at(i)));
    if (static_cast<int64_t>(staged_[0].size()) >= batch_) flush();
    ++seen_;
    int64_t per_epoch = static_cast<int64_t>(props_.num_training_samples) + props_.num_validation_samples;
    if (per_epoch > 0 && seen_ % per_epoch == 0) end_epoch();
    return true;
  }

  TrainerStatus status() override {
    std::lock_guard<std::mutex> lk(mu_);
    return status_;
  }

  bool save(const std::string& path) override {
    if (path.empty()) return false;
    guard();
    module_.save(path);
    return true;
  }

  bool wait_complete(int64_t timeout_ns) override {
    std::unique_lock<std::mutex> lk(mu_);
    auto pred = [&] { return status_.complete || stopped_; };
    if (timeout_ns < 0) {
      cv_.wait(lk, pred);
      return status_.complete;
    }
    return cv_.wait_for(lk, std::chrono::nanoseconds(timeout_ns), pred) && status_.complete;
  }

 private:
  void guard() {
    if (device_.is_cuda()) hip::check(hipSetDevice(device_.index()), "hipSetDevice");
  }

  at::Tensor to_tensor(const MemoryPtr& m, const TensorInfo& ti) {
    int rank = std::max(1, ti.rank());
    auto shape = torch_shape(ti, rank);
    auto opts = at::TensorOptions().dtype(to_torch(ti.type));
    if (m->on_device()) {
      m->sync_ready();
      return torch::from_blob(m->data(), shape, opts.device(torch::kCUDA, m->device())).to(device_, false, true);
    }
    return torch::from_blob(const_cast<void*>(m->map_host()), shape, opts).to(device_, false, true);
  }

  // one optimizer step (training) or evaluation (validation) over the staged samples
  void flush() {
    if (staged_.empty() || staged_[0].empty()) return;
    unsigned ni = props_.num_inputs;
    std::vector<torch::jit::IValue> inputs;
    for (unsigned i = 0; i < ni; ++i) {
      auto x = torch::stack(staged_[i]);
      if (!at::isFloatingType(x.scalar_type())) x = x.to(torch::kFloat);
      inputs.emplace_back(x);
    }
    at::Tensor label = torch::stack(staged_[ni]);
    int64_t n = label.size(0);
    for (auto& v : staged_) v.clear();

    auto run = [&](bool train) {
      at::Tensor out = module_.forward(inputs).toTensor().reshape({n, -1});
      at::Tensor loss, correct;
      if (loss_ == "cross_entropy") {
        at::Tensor target_idx;
        if (label.numel() == n) {  // class indices
          target_idx = label.reshape({n}).to(torch::kLong);
          loss = F::cross_entropy(out, target_idx);
        } else {  // one-hot / soft targets
          at::Tensor soft = label.reshape({n, -1}).to(out.scalar_type());
          loss = F::cross_entropy(out, soft);
          target_idx = soft.argmax(1);
        }
        correct = (out.argmax(1) == target_idx).sum();
      } else if (loss_ == "mse") {
        loss = F::mse_loss(out, label.reshape(out.sizes()).to(out.scalar_type()));
        correct = torch::zeros({}, out.options());
      } else {
        at::Tensor t = label.reshape(out.sizes()).to(out.scalar_type());
        loss = F::binary_cross_entropy_with_logits(out, t);
        correct = ((out > 0) == (t > 0.5)).all(1).sum();
      }
      if (train) {
        optim_->zero_grad();
        loss.backward();
        optim_->step();
      }
      return std::make_pair(loss.detach().item<double>() * n, correct.item<double>());
    };
    std::pair<double, double> r;
    if (staging_validation_) {
      torch::NoGradGuard ng;
      module_.eval();
      r = run(false);
      module_.train();
      val_loss_ += r.first;
      val_correct_ += r.second;
      val_n_ += n;
    } else {
      r = run(true);
      train_loss_ += r.first;
      train_correct_ += r.second;
      train_n_ += n;
    }
  }

  void end_epoch() {
    flush();
    std::lock_guard<std::mutex> lk(mu_);
    status_.training_loss = train_n_ ? train_loss_ / train_n_ : 0;
    status_.training_accuracy = train_n_ ? train_correct_ / train_n_ : 0;
    status_.validation_loss = val_n_ ? val_loss_ / val_n_ : 0;
    status_.validation_accuracy = val_n_ ? val_correct_ / val_n_ : 0;
    status_.epoch_count++;
    NNSX_LOGI("pytorch-trainer", strfmt("epoch ", status_.epoch_count, " loss=", status_.training_loss,
                                        " acc=", status_.training_accuracy, " val_loss=", status_.validation_loss,
                                        " val_acc=", status_.validation_accuracy));
    train_loss_ = train_correct_ = val_loss_ = val_correct_ = 0;
    train_n_ = val_n_ = 0;
    if (status_.epoch_count >= props_.epochs) {
      if (!props_.model_save_path.empty()) module_.save(props_.model_save_path);
      status_.complete = true;
      cv_.notify_all();
    }
  }

  TrainerProperties props_;
  torch::Device device_{torch::kCPU};
  torch::jit::Module module_;
  std::unique_ptr<torch::optim::Optimizer> optim_;
  std::string loss_;
  int64_t batch_ = 32, seen_ = 0;
  std::vector<std::vector<at::Tensor>> staged_;
  bool staging_validation_ = false;
  double train_loss_ = 0, train_correct_ = 0, val_loss_ = 0, val_correct_ = 0;
  int64_t train_n_ = 0, val_n_ = 0;
  std::mutex mu_;
  std::condition_variable cv_;
  TrainerStatus status_;
  bool stopped_ = false;
};

class TorchTrainerFw : public TrainerFramework {
 public:
  std::string name() const override { return "pytorch"; }
  std::unique_ptr<TrainerInstance> create(const TrainerProperties& p) override {
    return std::make_unique<TorchTrainer>(p);
  }
};

}  // namespace

void register_torch_trainer() { register_trainer(std::make_shared<TorchTrainerFw>()); }

}  // namespace nnsx
