// tensor_src_iio: Linux Industrial-I/O sensor source (sysfs + buffered char
// device), producing float32 tensors.
//
// Reference: gst/nnstreamer/elements/gsttensor_srciio.c -- channel type
// strings "[be|le]:[s|u]bits/storagebits>>shift" (:720-790), scan layout with
// per-channel natural alignment (:1503-1525), value = (raw + offset) * scale
// with sign extension (:106-133), merged [channels x capacity] or one tensor
// per channel (:2560-2585), framerate = sampling_frequency / buffer-capacity.
// Sysfs state changed by start() (enables, trigger, buffer length/enable,
// sampling frequency) is restored by stop().
#include <fcntl.h>
#include <poll.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <dirent.h>
#include <fstream>
#include <sstream>
#include <thread>

#include "core/log.h"
#include "elements/elements.h"
#include "elements/tensor_common.h"
#include "runtime/base.h"
#include "runtime/pipeline.h"

namespace nnsx {

namespace {

bool read_file(const std::string& path, std::string* out) {
  std::ifstream f(path);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  *out = strip(ss.str());
  return true;
}

bool write_file(const std::string& path, const std::string& v) {
  std::ofstream f(path, std::ios::trunc);
  if (!f) return false;
  f << v;
  return static_cast<bool>(f);
}

std::vector<std::string> list_dir(const std::string& path) {
  std::vector<std::string> v;
  DIR* d = opendir(path.c_str());
  if (!d) return v;
  while (dirent* e = readdir(d)) {
    std::string n = e->d_name;
    if (n != "." && n != "..") v.push_back(n);
  }
  closedir(d);
  std::sort(v.begin(), v.end());
  return v;
}

struct IioChannel {
  std::string name, generic;
  int index = 0;
  bool enabled = false, was_enabled = false;
  bool big_endian = false, is_signed = false;
  unsigned used_bits = 0, storage_bits = 0, storage_bytes = 0, shift = 0;
  uint64_t mask = 0;
  double scale = 1.0, offset = 0.0;
  unsigned location = 0;
};

bool parse_channel_type(const std::string& s, IioChannel* c) {
  // [be|le]:[s|u]bits/storagebits[Xrepeat]>>shift
  if (s.size() < 8 || (s[0] != 'b' && s[0] != 'l') || s[1] != 'e' || s[2] != ':') return false;
  c->big_endian = s[0] == 'b';
  if (s[3] != 's' && s[3] != 'u') return false;
  c->is_signed = s[3] == 's';
  char* end = nullptr;
  c->used_bits = static_cast<unsigned>(std::strtoul(s.c_str() + 4, &end, 10));
  if (*end != '/') return false;
  c->storage_bits = static_cast<unsigned>(std::strtoul(end + 1, &end, 10));
  if (end[0] == 'X') std::strtoul(end + 1, &end, 10);  // repeat count is unused
  if (end[0] != '>' || end[1] != '>') return false;
  c->shift = static_cast<unsigned>(std::strtoul(end + 2, &end, 10));
  if (c->used_bits == 0 || c->used_bits > 64 || c->storage_bits < c->used_bits || c->storage_bits > 64) return false;
  if (c->shift >= c->storage_bits) return false;
  c->storage_bytes = ((c->storage_bits - 1) >> 3) + 1;
  c->mask = c->used_bits == 64 ? ~0ull : ((1ull << c->used_bits) - 1);
  return true;
}

// generic name used for shared scale/offset attributes: in_voltage0 -> in_voltage
std::string generic_name(const std::string& n) {
  size_t e = n.size();
  while (e > 0 && std::isdigit(static_cast<unsigned char>(n[e - 1]))) --e;
  return n.substr(0, e);
}

float convert_sample(const IioChannel& c, const uint8_t* scan) {
  uint64_t v = 0;
  const uint8_t* p = scan + c.location;
  if (c.big_endian) {
    for (unsigned i = 0; i < c.storage_bytes; ++i) v = (v << 8) | p[i];
    v >>= (c.storage_bytes * 8 - c.storage_bits);
  } else {
    for (unsigned i = 0; i < c.storage_bytes; ++i) v |= static_cast<uint64_t>(p[i]) << (8 * i);
    if (c.storage_bits < 64) v &= (1ull << c.storage_bits) - 1;
  }
  v >>= c.shift;
  v &= c.mask;
  double x;
  if (c.is_signed) {
    unsigned sh = 64 - c.used_bits;
    x = static_cast<double>(static_cast<int64_t>(v << sh) >> sh);
  } else {
    x = static_cast<double>(v);
  }
  return static_cast<float>((x + c.offset) * c.scale);
}

class TensorSrcIio : public BaseSrc {
 public:
  explicit TensorSrcIio(const std::string& name)
      : BaseSrc("tensor_src_iio", name, Caps::from_string(tensor_caps_template_static())) {
    prop_string("mode", &mode_, "Operating mode: continuous (buffered) or one-shot (sysfs _raw reads)");
    prop_string("iio-base-dir", &base_dir_, "Base directory of IIO devices");
    prop_string("dev-dir", &dev_dir_, "Directory of the IIO character devices");
    prop_string("device", &device_, "Device name");
    prop_int("device-number", &device_num_, "Device number (used when device is unset)");
    prop_string("trigger", &trigger_, "Trigger name");
    prop_int("trigger-number", &trigger_num_, "Trigger number (used when trigger is unset)");
    prop_string("channels", &channels_prop_, "Channels to enable: auto, all, or comma separated indices");
    prop_uint("buffer-capacity", &capacity_, "Samples per output buffer");
    prop_int("frequency", &frequency_, "Sampling frequency (0 = keep the device's)");
    prop_bool("merge-channels-data", &merge_, "Merge all channels into one tensor");
    prop_int("poll-timeout", &poll_timeout_ms_, "Poll timeout in ms");
    prop_bool("silent", &silent_, "Suppress verbose output");
  }

 protected:
  bool on_start() override {
    try {
      setup();
    } catch (const std::exception& e) {
      post_error(std::string("tensor_src_iio: ") + e.what());
      restore();
      return false;
    }
    return true;
  }
  void on_stop() override { restore(); }

  Caps get_caps(const Caps* filter) override {
    Caps c = caps_from_config(config_);
    return filter ? c.intersect(*filter) : c;
  }

  FlowReturn create(BufferPtr* out) override {
    const size_t n = enabled_.size();
    std::vector<uint8_t> raw(scan_size_ * capacity_);
    std::vector<float> merged(merge_ ? n * capacity_ : 0);
    if (mode_ == "one-shot") {
      // read each channel's _raw attribute `capacity_` times
      for (unsigned s = 0; s < capacity_; ++s)
        for (size_t c = 0; c < n; ++c) {
          std::string v;
          if (!read_file(dev_path_ + "/" + enabled_[c].name + "_raw", &v)) return FlowReturn::ERROR;
          float f = static_cast<float>((to_double(v) + enabled_[c].offset) * enabled_[c].scale);
          oneshot_store(&merged, c, s, f);
        }
    } else {
      if (trigger_name_.empty()) {
        int64_t us = frequency_ > 0 ? static_cast<int64_t>(1000000.0 * capacity_ / frequency_) : 1;
        std::this_thread::sleep_for(std::chrono::microseconds(std::max<int64_t>(1, us)));
      } else {
        pollfd pfd{fd_, POLLIN, 0};
        int st = poll(&pfd, 1, poll_timeout_ms_);
        if (st <= 0 || !(pfd.revents & POLLIN)) {
          post_error("tensor_src_iio: timeout or error while polling the buffer");
          return FlowReturn::ERROR;
        }
      }
      size_t need = raw.size(), got = 0;
      int64_t deadline = now_ns() + static_cast<int64_t>(poll_timeout_ms_) * 1000000;
      while (got < need) {
        ssize_t r = read(fd_, raw.data() + got, need - got);
        if (r > 0) {
          got += static_cast<size_t>(r);
          continue;
        }
        if (r == 0) return FlowReturn::EOS;  // regular-file backed device: end of data
        if (errno == EAGAIN && now_ns() < deadline) {
          std::this_thread::sleep_for(std::chrono::microseconds(100));
          continue;
        }
        post_error(strfmt("tensor_src_iio: read ", got, "/", need, " bytes from the buffer"));
        return FlowReturn::ERROR;
      }
    }
    auto b = make_buffer();
    if (merge_) {
      auto m = Memory::alloc_host(n * capacity_ * sizeof(float));
      float* o = static_cast<float*>(m->data());
      if (mode_ == "one-shot")
        std::memcpy(o, merged.data(), m->size());
      else
        for (unsigned s = 0; s < capacity_; ++s)
          for (size_t c = 0; c < n; ++c) o[s * n + c] = convert_sample(enabled_[c], raw.data() + s * scan_size_);
      b->mems.push_back(m);
    } else {
      for (size_t c = 0; c < n; ++c) {
        auto m = Memory::alloc_host(capacity_ * sizeof(float));
        float* o = static_cast<float*>(m->data());
        for (unsigned s = 0; s < capacity_; ++s)
          o[s] = mode_ == "one-shot" ? oneshot_[c * capacity_ + s]
                                     : convert_sample(enabled_[c], raw.data() + s * scan_size_);
        b->mems.push_back(m);
      }
    }
    if (frequency_ > 0) {
      b->pts = produced_ * static_cast<int64_t>(kSecond * static_cast<double>(capacity_) / frequency_);
      b->duration = static_cast<int64_t>(kSecond * static_cast<double>(capacity_) / frequency_);
    }
    *out = b;
    return FlowReturn::OK;
  }

 private:
  void oneshot_store(std::vector<float>* merged, size_t c, unsigned s, float f) {
    size_t n = enabled_.size();
    if (merge_)
      (*merged)[s * n + c] = f;
    else {
      oneshot_.resize(n * capacity_);
      oneshot_[c * capacity_ + s] = f;
    }
  }

  int find_numbered(const std::string& prefix, const std::string& want, int num) {
    for (auto& e : list_dir(base_dir_)) {
      if (!starts_with(e, prefix)) continue;
      int id = static_cast<int>(to_int(e.substr(prefix.size()), -1));
      if (id < 0) continue;
      std::string n;
      read_file(base_dir_ + "/" + e + "/name", &n);
      if (!want.empty() ? n == want : id == num) return id;
    }
    return -1;
  }

  void setup() {
    if (mode_ != "continuous" && mode_ != "one-shot") throw Error("unknown mode '" + mode_ + "'");
    if (capacity_ == 0) throw Error("buffer-capacity must be > 0");
    dev_id_ = find_numbered("iio:device", device_, device_num_);
    if (dev_id_ < 0) throw Error("cannot find the IIO device");
    dev_path_ = base_dir_ + "/iio:device" + std::to_string(dev_id_);
    // trigger
    trigger_name_.clear();
    if (!trigger_.empty() || trigger_num_ >= 0) {
      int tid = find_numbered("trigger", trigger_, trigger_num_);
      if (tid < 0) throw Error("cannot find the IIO trigger");
      read_file(base_dir_ + "/trigger" + std::to_string(tid) + "/name", &trigger_name_);
      read_file(dev_path_ + "/trigger/current_trigger", &saved_trigger_);
      if (!write_file(dev_path_ + "/trigger/current_trigger", trigger_name_))
        throw Error("cannot set the device trigger");
    }
    // sampling frequency
    saved_freq_.clear();
    std::string f;
    if (read_file(dev_path_ + "/sampling_frequency", &f)) {
      saved_freq_ = f;
      if (frequency_ > 0) {
        if (!write_file(dev_path_ + "/sampling_frequency", std::to_string(frequency_)))
          throw Error("cannot set the sampling frequency");
      } else {
        frequency_ = static_cast<int>(to_int(f));
        if (frequency_ <= 0) {
          std::string avail;
          if (read_file(dev_path_ + "/sampling_frequency_available", &avail)) {
            auto p = split_any(avail, " \t");
            if (!p.empty()) frequency_ = static_cast<int>(to_int(p[0]));
          }
        }
      }
    }
    // channels
    channels_.clear();
    std::string scan = dev_path_ + "/scan_elements";
    for (auto& e : list_dir(scan)) {
      if (!ends_with(e, "_en")) continue;
      IioChannel c;
      c.name = e.substr(0, e.size() - 3);
      c.generic = generic_name(c.name);
      std::string v;
      if (!read_file(scan + "/" + c.name + "_index", &v)) continue;
      c.index = static_cast<int>(to_int(v));
      if (!read_file(scan + "/" + c.name + "_type", &v) || !parse_channel_type(v, &c))
        throw Error("invalid type for channel " + c.name);
      if (read_file(scan + "/" + e, &v)) c.was_enabled = c.enabled = to_int(v) != 0;
      // per-channel, then digit-stripped generic (reference), then axis-stripped
      // shared attribute (in_accel_x -> in_accel_scale, Linux IIO ABI)
      std::string axis_less = c.name.substr(0, c.name.rfind('_') == std::string::npos ? c.name.size() : c.name.rfind('_'));
      for (const std::string& base : {c.name, c.generic, axis_less}) {
        if (read_file(dev_path_ + "/" + base + "_scale", &v)) {
          c.scale = to_double(v, 1.0);
          break;
        }
      }
      for (const std::string& base : {c.name, c.generic, axis_less}) {
        if (read_file(dev_path_ + "/" + base + "_offset", &v)) {
          c.offset = to_double(v);
          break;
        }
      }
      channels_.push_back(c);
    }
    if (channels_.empty()) throw Error("no channels in " + scan);
    std::sort(channels_.begin(), channels_.end(), [](auto& a, auto& b) { return a.index < b.index; });
    std::string cp = lower(strip(channels_prop_));
    bool any_enabled = std::any_of(channels_.begin(), channels_.end(), [](auto& c) { return c.enabled; });
    for (auto& c : channels_) {
      if (cp == "all" || (cp == "auto" && !any_enabled))
        c.enabled = true;
      else if (cp != "auto") {
        c.enabled = false;
        for (auto& t : split(cp, ','))
          if (!strip(t).empty() && to_int(t) == c.index) c.enabled = true;
      }
      if (c.enabled != c.was_enabled && !write_file(scan + "/" + c.name + "_en", c.enabled ? "1" : "0"))
        throw Error("cannot enable channel " + c.name);
    }
    enabled_.clear();
    scan_size_ = 0;
    for (auto& c : channels_) {
      if (!c.enabled) continue;
      unsigned rem = c.storage_bytes ? scan_size_ % c.storage_bytes : 0;
      c.location = rem == 0 ? scan_size_ : scan_size_ - rem + c.storage_bytes;
      scan_size_ = c.location + c.storage_bytes;
      enabled_.push_back(c);
    }
    if (enabled_.empty()) throw Error("no channel enabled");
    // buffer
    if (mode_ == "continuous") {
      read_file(dev_path_ + "/buffer/length", &saved_len_);
      write_file(dev_path_ + "/buffer/length", std::to_string(capacity_));
      write_file(dev_path_ + "/buffer/enable", "1");
      std::string dev = dev_dir_ + "/iio:device" + std::to_string(dev_id_);
      fd_ = ::open(dev.c_str(), O_RDONLY | O_NONBLOCK);
      if (fd_ < 0) throw Error("cannot open " + dev);
    }
    // output config
    config_ = TensorsConfig();
    unsigned n = static_cast<unsigned>(enabled_.size());
    if (merge_) {
      config_.info.num_tensors = 1;
      config_.info.at(0).type = DType::FLOAT32;
      config_.info.at(0).dim = {n, capacity_, 1, 1, 1, 1, 1, 1};
    } else {
      config_.info.num_tensors = n;
      for (unsigned i = 0; i < n; ++i) {
        config_.info.at(i).type = DType::FLOAT32;
        config_.info.at(i).dim = {capacity_, 1, 1, 1, 1, 1, 1, 1};
      }
    }
    config_.rate_n = std::max(frequency_, 0);
    config_.rate_d = static_cast<int>(capacity_);
  }

  void restore() {
    if (fd_ >= 0) {
      ::close(fd_);
      fd_ = -1;
    }
    if (dev_path_.empty()) return;
    if (mode_ == "continuous") {
      write_file(dev_path_ + "/buffer/enable", "0");
      if (!saved_len_.empty()) write_file(dev_path_ + "/buffer/length", saved_len_);
    }
    for (auto& c : channels_)
      if (c.enabled != c.was_enabled) write_file(dev_path_ + "/scan_elements/" + c.name + "_en", c.was_enabled ? "1" : "0");
    if (!trigger_name_.empty()) write_file(dev_path_ + "/trigger/current_trigger", saved_trigger_);
    if (!saved_freq_.empty()) write_file(dev_path_ + "/sampling_frequency", saved_freq_);
    dev_path_.clear();
  }

  std::string mode_ = "continuous", base_dir_ = "/sys/bus/iio/devices", dev_dir_ = "/dev";
  std::string device_, trigger_, channels_prop_ = "auto";
  int device_num_ = -1, trigger_num_ = -1, frequency_ = 0, poll_timeout_ms_ = 10000;
  unsigned capacity_ = 1;
  bool merge_ = true, silent_ = true;
  // runtime
  int dev_id_ = -1, fd_ = -1;
  std::string dev_path_, trigger_name_, saved_trigger_, saved_freq_, saved_len_;
  std::vector<IioChannel> channels_, enabled_;
  unsigned scan_size_ = 0;
  std::vector<float> oneshot_;
  TensorsConfig config_;
};

}  // namespace

void register_src_iio() {
  register_element("tensor_src_iio", "Source/Tensor/Device", "Creates tensors from Linux IIO sensor devices",
                   [](const std::string& n) { return std::make_unique<TensorSrcIio>(n); });
}

}  // namespace nnsx
