// tensor_if, tensor_rate, tensor_reposink / tensor_reposrc (+ TensorRepo),
// tensor_sparse_enc / tensor_sparse_dec, tensor_debug, join, datareposrc /
// datareposink.
//
// Reference: gst/nnstreamer/elements/gsttensor_if.c (:145-220,:812-1200),
// gsttensor_rate.c (:455-632), gsttensor_repo.c (:49-394),
// gsttensor_reposink.c / gsttensor_reposrc.c, gsttensor_sparseutil.c
// (:20-255), gsttensor_debug.c, gst/join/gstjoin.c, gst/datarepo/*.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <fstream>
#include <random>
#include <set>

#include "core/cpu_ops.h"
#include "core/log.h"
#include "elements/elements.h"
#include "elements/tensor_common.h"
#include "kernels/kernels.h"
#include "runtime/base.h"
#include "runtime/pipeline.h"
#include "runtime/plugin_api.h"

namespace nnsx {

// ============================================================== TensorRepo ====
struct TensorRepo::Slot {
  BufferPtr buffer;
  Caps caps;
  bool eos = false;
  bool src_changed = false, sink_changed = false;
  bool flushing = false;
};

TensorRepo& TensorRepo::get() {
  static TensorRepo* r = new TensorRepo();
  return *r;
}

std::shared_ptr<TensorRepo::Slot> TensorRepo::slot(unsigned i) {
  auto it = slots_.find(i);
  if (it != slots_.end()) return it->second;
  auto s = std::make_shared<Slot>();
  slots_[i] = s;
  return s;
}

bool TensorRepo::set_buffer(unsigned i, BufferPtr buf, const Caps& caps) {
  std::unique_lock<std::mutex> lk(mu_);
  auto s = slot(i);
  // one-deep mailbox: wait until the previous buffer was pulled
  cv_.wait(lk, [&] { return !s->buffer || s->eos || s->flushing; });
  if (s->flushing) return false;
  s->buffer = std::move(buf);
  s->caps = caps;
  cv_.notify_all();
  return true;
}

BufferPtr TensorRepo::get_buffer(unsigned i, Caps* caps, bool* eos, int64_t timeout_ns) {
  std::unique_lock<std::mutex> lk(mu_);
  auto s = slot(i);
  auto pred = [&] { return s->buffer || s->eos || s->flushing; };
  if (timeout_ns < 0)
    cv_.wait(lk, pred);
  else if (!cv_.wait_for(lk, std::chrono::nanoseconds(timeout_ns), pred)) {
    *eos = false;
    return nullptr;
  }
  *eos = s->eos && !s->buffer;
  if (s->flushing) return nullptr;
  BufferPtr b = std::move(s->buffer);
  s->buffer.reset();
  if (caps) *caps = s->caps;
  cv_.notify_all();
  return b;
}

void TensorRepo::set_eos(unsigned i) {
  std::lock_guard<std::mutex> lk(mu_);
  slot(i)->eos = true;
  cv_.notify_all();
}

void TensorRepo::set_changed(unsigned i, bool pushing) {
  std::lock_guard<std::mutex> lk(mu_);
  if (pushing)
    slot(i)->sink_changed = true;
  else
    slot(i)->src_changed = true;
}

void TensorRepo::reset(unsigned i) {
  std::lock_guard<std::mutex> lk(mu_);
  auto s = slot(i);
  s->buffer.reset();
  s->eos = false;
  s->flushing = false;
  cv_.notify_all();
}

void TensorRepo::flush(unsigned i) {
  std::lock_guard<std::mutex> lk(mu_);
  slot(i)->flushing = true;
  cv_.notify_all();
}

void TensorRepo::remove(unsigned i) {
  std::lock_guard<std::mutex> lk(mu_);
  slots_.erase(i);
  cv_.notify_all();
}

size_t TensorRepo::num_slots() {
  std::lock_guard<std::mutex> lk(mu_);
  return slots_.size();
}

namespace {

// ================================================================ tensor_if ====
enum IfCV { CV_A_VALUE = 0, CV_TENSOR_AVERAGE, CV_CUSTOM };
enum IfOp { OP_EQ = 0, OP_NE, OP_GT, OP_GE, OP_LT, OP_LE, OP_RANGE_IN, OP_RANGE_EX, OP_NOT_RANGE_IN, OP_NOT_RANGE_EX };
enum IfAct { ACT_PASSTHROUGH = 0, ACT_SKIP, ACT_TENSORPICK };

class TensorIf : public Element {
 public:
  explicit TensorIf(const std::string& name) : Element("tensor_if", name) {
    add_template("sink", PadDirection::SINK, PadPresence::ALWAYS, Caps::from_string(tensor_caps_template_static()));
    add_template("src_%u", PadDirection::SRC, PadPresence::SOMETIMES, Caps::from_string(tensor_caps_template_static()));
    prop_enum("compared-value", &cv_, {"A_VALUE", "TENSOR_AVERAGE_VALUE", "CUSTOM"}, "Compared value from input tensor(s)");
    prop_string("compared-value-option", &cv_opt_, "Specify an element of the nth tensor or the nth tensor (or custom name)");
    prop_string("supplied-value", &sv_str_, "Supplied value(s) for comparison (one, or two for ranges)", [this] {
      sv_.clear();
      for (auto& v : split(sv_str_, ','))
        if (!strip(v).empty()) sv_.push_back(to_double(v));
    });
    prop_enum("operator", &op_, {"EQ", "NE", "GT", "GE", "LT", "LE", "RANGE_INCLUSIVE", "RANGE_EXCLUSIVE",
                                 "NOT_IN_RANGE_INCLUSIVE", "NOT_IN_RANGE_EXCLUSIVE"},
              "Comparison operator");
    prop_enum("then", &then_, {"PASSTHROUGH", "SKIP", "TENSORPICK"}, "Action when the condition is TRUE");
    prop_string("then-option", &then_opt_, "Tensors picked when then=TENSORPICK");
    prop_enum("else", &else_, {"PASSTHROUGH", "SKIP", "TENSORPICK"}, "Action when the condition is FALSE");
    prop_string("else-option", &else_opt_, "Tensors picked when else=TENSORPICK");
  }

  bool sink_event(Pad*, Event& ev) override {
    if (ev.type == EventType::CAPS) {
      if (!tensor_config_from_caps(ev.caps, &config_)) return false;
      for (int branch = 0; branch < 2; ++branch) {
        Pad* p = pad_for(branch);
        if (!p->is_linked()) continue;
        int act = branch == 0 ? then_ : else_;
        if (act == ACT_SKIP) continue;
        TensorsConfig oc = config_;
        if (act == ACT_TENSORPICK) {
          auto picks = parse_picks(branch == 0 ? then_opt_ : else_opt_);
          oc.info.resize(static_cast<unsigned>(picks.size()));
          oc.info.num_tensors = static_cast<unsigned>(picks.size());
          for (size_t i = 0; i < picks.size(); ++i) oc.info.at(static_cast<unsigned>(i)) = config_.info.at(picks[i]);
        }
        p->push_event(Event::make_stream_start(name() + std::to_string(branch)));
        p->push_event(Event::make_caps(tensor_src_caps(p, oc)));
        p->push_event(Event::make_segment(Segment()));
      }
      return true;
    }
    if (ev.type == EventType::STREAM_START || ev.type == EventType::SEGMENT) return true;
    return forward_event_downstream(ev);
  }

  FlowReturn chain(Pad*, BufferPtr buf) override {
    BufferPtr in;
    if (!buffer_from_config(buf, config_, &in)) return FlowReturn::ERROR;
    bool cond;
    if (!evaluate(*in, &cond)) {
      post_error("tensor_if: failed to evaluate the condition");
      return FlowReturn::ERROR;
    }
    int branch = cond ? 0 : 1;
    int act = cond ? then_ : else_;
    if (act == ACT_SKIP) return FlowReturn::OK;
    Pad* p = pad_for(branch);
    if (!p->is_linked()) return FlowReturn::OK;
    BufferPtr out = in;
    if (act == ACT_TENSORPICK) {
      out = make_buffer();
      out->copy_metadata_from(*in);
      for (unsigned k : parse_picks(cond ? then_opt_ : else_opt_)) {
        if (k >= in->n_memory()) return FlowReturn::ERROR;
        out->mems.push_back(in->mems[k]);
      }
    }
    FlowReturn r = p->push(out);
    return r == FlowReturn::NOT_LINKED ? FlowReturn::OK : r;
  }

  Caps query_caps(Pad* pad, const Caps* filter) override {
    Caps c = pad->template_caps();
    return filter ? c.intersect(*filter) : c;
  }

 private:
  Pad* pad_for(int branch) {
    std::string n = "src_" + std::to_string(branch);
    Pad* p = get_pad(n);
    if (!p) p = Element::request_pad(templates_[1], n);
    return p;
  }

  static std::vector<unsigned> parse_picks(const std::string& s) {
    std::vector<unsigned> v;
    for (auto& x : split(s, ','))
      if (!strip(x).empty()) v.push_back(static_cast<unsigned>(to_uint(x)));
    return v;
  }

  bool evaluate(const Buffer& in, bool* out) {
    double v = 0;
    if (cv_ == CV_CUSTOM) {
      auto fn = find_if_custom(cv_opt_);
      if (!fn) return false;
      *out = fn(config_.info, in.mems);
      return true;
    }
    if (cv_ == CV_A_VALUE) {
      // "d1:d2:...:d8,nth" (missing dims are 0)
      auto parts = split(cv_opt_, ',');
      if (parts.size() != 2) return false;
      unsigned nth = static_cast<unsigned>(to_uint(parts[1]));
      if (nth >= in.n_memory()) return false;
      auto idx_s = split(parts[0], ':');
      const TensorInfo& ti = config_.info.at(nth);
      uint64_t idx = 0, stride = 1;
      for (int d = 0; d < kRankLimit; ++d) {
        uint64_t c = d < static_cast<int>(idx_s.size()) ? to_uint(idx_s[d]) : 0;
        idx += c * stride;
        stride *= ti.dim[d];
      }
      if (idx >= element_count(ti.dim)) return false;
      const MemoryPtr& m = in.mems[nth];
      if (m->on_device()) {
        // single-element D2H (K22)
        size_t es = dtype_size(ti.type);
        uint8_t tmp[8];
        m->sync_ready();
        hip::check(hipMemcpy(tmp, static_cast<const char*>(m->data()) + idx * es, es, hipMemcpyDeviceToHost), "D2H");
        v = cpu::read_as_double(tmp, ti.type, 0);
      } else {
        v = cpu::read_as_double(m->map_host(), ti.type, idx);
      }
    } else {
      unsigned nth = static_cast<unsigned>(to_uint(cv_opt_));
      if (nth >= in.n_memory()) return false;
      const TensorInfo& ti = config_.info.at(nth);
      const MemoryPtr& m = in.mems[nth];
      uint64_t n = element_count(ti.dim);
      double avg = 0;
      if (m->on_device()) {
        // K22: reduce on the GPU, only the 8-byte mean crosses to the host
        const int dev = m->device();
        hip::DeviceGuard g(dev);
        hipStream_t s = streams_.get(dev);
        if (!mean_ws_ || mean_ws_->device() != dev) {  // (a buffer from another GPU: its own workspace)
          mean_ws_ = Memory::alloc_device(kernels::mean_workspace_bytes(), dev, s);
          if (!mean_host_) mean_host_ = Memory::alloc_pinned(8);
        }
        double* ws = static_cast<double*>(mean_ws_->data());
        if (!kernels::tensor_mean(m->map_device(dev, s), ti.type, n, ws, s)) return false;
        hip::check(hipMemcpyAsync(mean_host_->data(), ws + kernels::mean_workspace_bytes() / 8 - 1, 8,
                                  hipMemcpyDeviceToHost, s),
                   "tensor_if mean D2H");
        hip::check(hipStreamSynchronize(s), "tensor_if mean sync");
        m->record_use(s, dev);
        std::memcpy(&avg, mean_host_->data(), 8);
      } else {
        const void* p = m->map_host();
        for (uint64_t i = 0; i < n; ++i) avg = (cpu::read_as_double(p, ti.type, i) - avg) / (i + 1) + avg;
      }
      // the reference casts the average to the tensor type before comparing
      uint8_t tmp[8];
      cpu::write_from_double(tmp, ti.type, 0, avg);
      v = cpu::read_as_double(tmp, ti.type, 0);
    }
    double a = sv_.empty() ? 0 : sv_[0];
    double b = sv_.size() > 1 ? sv_[1] : a;
    switch (op_) {
      case OP_EQ: *out = v == a; break;
      case OP_NE: *out = v != a; break;
      case OP_GT: *out = v > a; break;
      case OP_GE: *out = v >= a; break;
      case OP_LT: *out = v < a; break;
      case OP_LE: *out = v <= a; break;
      case OP_RANGE_IN: *out = a <= v && v <= b; break;
      case OP_RANGE_EX: *out = a < v && v < b; break;
      case OP_NOT_RANGE_IN: *out = v < a || v > b; break;
      case OP_NOT_RANGE_EX: *out = v <= a || v >= b; break;
      default: return false;
    }
    return true;
  }

  int cv_ = CV_A_VALUE, op_ = OP_EQ, then_ = ACT_PASSTHROUGH, else_ = ACT_SKIP;
  std::string cv_opt_, sv_str_, then_opt_, else_opt_;
  std::vector<double> sv_;
  TensorsConfig config_;
  StreamSet streams_;             // device average (K22)
  MemoryPtr mean_ws_, mean_host_;
};


// ============================================================= tensor_crop ====
// gsttensor_crop.c:540-760: `raw` (NHWC-style [ch, w, h, ...] tensor) is cropped
// by the [x, y, w, h] regions carried in the flexible `info` tensor; output is
// one flexible tensor per region.  HBM-resident inputs are cropped with pitched
// device copies on the element's stream (no host round trip).
class TensorCrop : public Element {
 public:
  explicit TensorCrop(const std::string& name) : Element("tensor_crop", name), cp_(this) {
    add_template("raw", PadDirection::SINK, PadPresence::ALWAYS, Caps::from_string(tensor_caps_template_all()));
    add_template("info", PadDirection::SINK, PadPresence::ALWAYS, Caps::from_string(tensor_caps_template_all()));
    add_template("src", PadDirection::SRC, PadPresence::ALWAYS, Caps::from_string(tensor_caps_template_flexible()));
    cp_.add_pad(get_pad("raw"));
    cp_.add_pad(get_pad("info"));
    prop_int("lateness", &lateness_ms_, "Max time difference between raw and info buffers in ms (-1 = no sync)");
  }

  bool start() override {
    cp_.reset();
    sent_caps_ = false;
    stream_started_ = false;
    eos_sent_ = false;
    return true;
  }
  void unlock() override { cp_.set_flushing(true); }
  bool stop() override {
    cp_.set_flushing(true);
    return true;
  }

  FlowReturn chain(Pad* pad, BufferPtr buf) override {
    return cp_.chain(pad, std::move(buf), [this] { return collected(); });
  }

  bool sink_event(Pad* pad, Event& ev) override {
    switch (ev.type) {
      case EventType::CAPS: {
        TensorsConfig c;
        if (!tensor_config_from_caps(ev.caps, &c)) return false;
        if (pad->name() == "raw")
          raw_cfg_ = c;
        else
          info_cfg_ = c;
        return true;
      }
      case EventType::EOS:
        if (cp_.set_eos(pad, [this] { return collected(); })) send_eos();
        return true;
      case EventType::STREAM_START:
      case EventType::SEGMENT:
        return true;
      default:
        return forward_event_downstream(ev);
    }
  }

  Caps query_caps(Pad* pad, const Caps* filter) override {
    Caps c = pad->template_caps();
    return filter ? c.intersect(*filter) : c;
  }

 private:
  void send_eos() {
    if (eos_sent_) return;
    eos_sent_ = true;
    Event e = Event::make_eos();
    src_pad()->push_event(e);
  }

  FlowReturn collected() {
    auto* draw = cp_.data(get_pad("raw"));
    auto* dinfo = cp_.data(get_pad("info"));
    BufferPtr raw = cp_.peek(draw), info = cp_.peek(dinfo);
    if (!raw || !info) {
      if ((!raw && draw->eos) || (!info && dinfo->eos)) {
        send_eos();
        return FlowReturn::EOS;
      }
      return FlowReturn::OK;
    }
    if (lateness_ms_ >= 0 && raw->pts >= 0 && info->pts >= 0 &&
        std::llabs(raw->pts - info->pts) > lateness_ms_ * 1000000LL) {
      // drop the older buffer and wait for the next one
      if (raw->pts > info->pts)
        cp_.pop(dinfo);
      else
        cp_.pop(draw);
      return FlowReturn::OK;
    }
    cp_.pop(draw);
    cp_.pop(dinfo);
    std::vector<std::array<uint32_t, 4>> regions;
    if (!parse_info(info, &regions)) {
      post_error("tensor_crop: failed to parse the crop info");
      return FlowReturn::ERROR;
    }
    BufferPtr out;
    if (!crop(raw, regions, &out)) {
      post_error("tensor_crop: failed to crop the raw tensor");
      return FlowReturn::ERROR;
    }
    if (!stream_started_) {
      src_pad()->push_event(Event::make_stream_start(name()));
      stream_started_ = true;
    }
    if (!sent_caps_) {
      TensorsConfig oc;
      oc.info.format = Format::FLEXIBLE;
      oc.rate_n = raw_cfg_.rate_n;
      oc.rate_d = raw_cfg_.rate_d;
      src_pad()->push_event(Event::make_caps(caps_from_config(oc)));
      src_pad()->push_event(Event::make_segment(Segment()));
      sent_caps_ = true;
    }
    return src_pad()->push(out);
  }

  bool parse_info(const BufferPtr& info, std::vector<std::array<uint32_t, 4>>* regions) {
    if (info->n_memory() == 0) return false;
    MemoryPtr m = info->mems[0];
    MetaInfo meta;
    MemoryPtr payload;
    TensorInfo ti;
    if (parse_flexible(m, &meta, &payload)) {
      if (!meta.to_info(&ti)) return false;
    } else if (info_cfg_.is_static() && info_cfg_.info.num_tensors > 0) {
      ti = info_cfg_.info.at(0);
      payload = m;
    } else {
      return false;
    }
    size_t es = dtype_size(ti.type);
    const void* p = payload->map_host();
    size_t n = payload->size() / (es * 4);
    n = std::min<size_t>(n, kSizeLimit);
    for (size_t i = 0; i < n; ++i) {
      std::array<uint32_t, 4> r;
      for (int j = 0; j < 4; ++j) {
        double v = cpu::read_as_double(p, ti.type, i * 4 + static_cast<size_t>(j));
        r[static_cast<size_t>(j)] = v <= 0 ? 0u : static_cast<uint32_t>(v);
      }
      regions->push_back(r);
    }
    return true;
  }

  bool crop(const BufferPtr& raw, const std::vector<std::array<uint32_t, 4>>& regions, BufferPtr* outp) {
    if (raw->n_memory() == 0) return false;
    MemoryPtr m = raw->mems[0];
    TensorInfo ti;
    MemoryPtr payload;
    MetaInfo meta;
    if (raw_cfg_.is_flexible() || (m->has_meta() && !raw_cfg_.is_static())) {
      if (!parse_flexible(m, &meta, &payload) || !meta.to_info(&ti)) return false;
    } else {
      ti = raw_cfg_.info.at(0);
      payload = m;
    }
    if (payload->size() != ti.size()) return false;
    uint32_t ch = ti.dim[0], mw = ti.dim[1], mh = ti.dim[2];
    size_t es = dtype_size(ti.type);
    int dev = payload->on_device() ? payload->device() : -1;
    hipStream_t s = dev >= 0 ? streams_.get(dev) : nullptr;
    const uint8_t* src = dev >= 0 ? static_cast<const uint8_t*>(payload->map_device(dev, s))
                                  : static_cast<const uint8_t*>(payload->map_host());
    auto out = make_buffer();
    out->copy_metadata_from(*raw);
    for (auto& r : regions) {
      uint32_t x = std::min(r[0], mw), y = std::min(r[1], mh);
      uint32_t w = (x + r[2] - 1 < mw) ? r[2] : mw - x;
      uint32_t h = (y + r[3] - 1 < mh) ? r[3] : mh - y;
      if (w == 0 || h == 0) continue;
      size_t row = es * ch * w, pitch = es * ch * mw;
      const uint8_t* base = src + es * ch * (x + static_cast<size_t>(y) * mw);
      MemoryPtr o = alloc_output(row * h, dev, s);
      if (dev >= 0) {
        hip::check(hipMemcpy2DAsync(o->data(), row, base, pitch, row, h, hipMemcpyDeviceToDevice, s), "crop 2D");
        o->mark_ready(s);
      } else {
        for (uint32_t j = 0; j < h; ++j) std::memcpy(static_cast<uint8_t*>(o->data()) + row * j, base + pitch * j, row);
      }
      TensorInfo oi = ti;
      oi.dim[1] = w;
      oi.dim[2] = h;
      oi.dim[3] = 1;
      out->mems.push_back(make_flexible(o, MetaInfo::from_info(oi, Format::FLEXIBLE)));
    }
    if (dev >= 0) payload->record_use(s, dev);
    *outp = out;
    return true;
  }

  CollectPads cp_;
  int64_t lateness_ms_ = -1;
  TensorsConfig raw_cfg_, info_cfg_;
  StreamSet streams_;
  bool sent_caps_ = false, stream_started_ = false, eos_sent_ = false;
};

// ============================================================== tensor_rate ====
class TensorRate : public BaseTransform {
 public:
  explicit TensorRate(const std::string& name)
      : BaseTransform("tensor_rate", name, Caps::from_string(tensor_caps_template_all()),
                      Caps::from_string(tensor_caps_template_all())) {
    prop_string("framerate", &rate_str_, "Target framerate (e.g. 15/1)", [this] {
      if (!parse_fraction(rate_str_, &tn_, &td_) || tn_ < 0 || td_ <= 0) throw Error("tensor_rate: bad framerate");
    });
    prop_bool("throttle", &throttle_, "Send QoS throttling events upstream so tensor_filter drops frames early");
    prop_readonly("in", [this] { return std::to_string(in_); }, "Number of input frames");
    prop_readonly("out", [this] { return std::to_string(out_); }, "Number of output frames");
    prop_readonly("duplicate", [this] { return std::to_string(dup_); }, "Number of duplicated frames");
    prop_readonly("drop", [this] { return std::to_string(drop_); }, "Number of dropped frames");
  }

 protected:
  bool start() override {
    in_ = out_ = dup_ = drop_ = 0;
    next_ts_ = -1;
    prev_.reset();
    return true;
  }

  Caps transform_caps(PadDirection dir, const Caps& caps, const Caps* filter) override {
    Caps r;
    for (size_t i = 0; i < caps.size(); ++i) {
      Structure s = caps.at(i);
      if (dir == PadDirection::SINK && tn_ > 0)
        s.set("framerate", Value::Fraction(tn_, td_));
      else
        s.set("framerate", Value::FractionRange(0, 1, INT32_MAX, 1));
      r.append(s);
    }
    if (filter) r = r.intersect(*filter);
    return r;
  }

  bool set_caps(const Caps&, const Caps&) override { return true; }

  // videorate-style selection (gsttensor_rate.c:530-605): hold the previous
  // frame, emit it for every output slot it is closest to (ties go to the
  // previous frame), then keep the new one.
  FlowReturn transform(const BufferPtr& in, BufferPtr* out) override {
    *out = nullptr;  // frames are pushed from here
    ++in_;
    if (tn_ <= 0 || in->pts < 0) {
      ++out_;
      *out = in;
      return FlowReturn::OK;
    }
    int64_t intime = in->pts;
    if (!prev_) {
      prev_ = in;
      if (next_ts_ < 0) {
        next_ts_ = intime;
        base_ts_ = intime;
        out_frames_ = 0;
      }
      return FlowReturn::OK;
    }
    if (intime < prev_->pts) {
      ++drop_;
      return FlowReturn::OK;
    }
    int count = 0;
    int64_t d1, d2;
    FlowReturn r = FlowReturn::OK;
    do {
      d1 = std::llabs(prev_->pts - next_ts_);
      d2 = std::llabs(intime - next_ts_);
      if (d1 <= d2) {
        ++count;
        r = flush_prev();
        if (!flow_ok(r)) return r;
      }
    } while (d1 < d2);
    if (count > 1)
      dup_ += count - 1;
    else if (count == 0) {
      ++drop_;
      send_throttle(intime);
    }
    prev_ = in;
    return r;
  }

  bool handle_sink_event(Event& ev) override {
    if (ev.type == EventType::EOS && prev_ && tn_ > 0) flush_prev();
    if (ev.type == EventType::FLUSH_STOP || ev.type == EventType::SEGMENT) {
      prev_.reset();
      next_ts_ = -1;
    }
    return true;
  }

  FlowReturn flush_prev() {
    auto b = make_buffer();
    *b = *prev_;
    int64_t push_ts = next_ts_;
    ++out_;
    ++out_frames_;
    next_ts_ = base_ts_ + static_cast<int64_t>(static_cast<__int128>(kSecond) * td_ * out_frames_ / tn_);
    b->pts = push_ts;
    b->duration = next_ts_ - push_ts;
    b->offset = out_ - 1;
    return src_pad()->push(b);
  }

  // upstream QoS(throttle) so a tensor_filter in front skips frames that would be dropped here
  void send_throttle(int64_t ts) {
    if (!throttle_) return;
    Event qos;
    qos.type = EventType::QOS;
    qos.qos_type = "throttle";
    qos.diff = static_cast<int64_t>(static_cast<double>(kSecond) * td_ / tn_ * 0.999);
    qos.timestamp = ts;
    sink_pad()->push_event(qos);
  }

 private:
  std::string rate_str_;
  int tn_ = -1, td_ = 1;
  bool throttle_ = true;
  int64_t in_ = 0, out_ = 0, dup_ = 0, drop_ = 0, next_ts_ = -1, base_ts_ = 0, out_frames_ = 0;
  BufferPtr prev_;
};

// ====================================================== tensor_repo sink/src ====
class TensorRepoSink : public BaseSink {
 public:
  explicit TensorRepoSink(const std::string& name)
      : BaseSink("tensor_reposink", name, Caps::from_string(tensor_caps_template_all())) {
    prop_uint("slot-index", &slot_, "Slot index of the tensor repository");
    prop_uint("signal-rate", &signal_rate_, "New data signals per second (0 for unlimited)");
    prop_bool("emit-signal", &emit_signal_, "Emit signal for new data");
  }

 protected:
  bool start() override {
    BaseSink::start();
    TensorRepo::get().reset(slot_);
    return true;
  }
  void unlock() override { TensorRepo::get().flush(slot_); }
  bool set_caps(const Caps& caps) override {
    caps_ = caps;
    return true;
  }
  FlowReturn render(const BufferPtr& buf) override {
    auto copy = make_buffer();
    *copy = *buf;  // shares memories (immutable); the reference deep-copies
    if (!TensorRepo::get().set_buffer(slot_, copy, caps_)) return FlowReturn::FLUSHING;
    if (emit_signal_) {
      SignalArgs a;
      a.buffer = buf;
      emit("new-data", a);
    }
    return FlowReturn::OK;
  }
  void on_eos() override { TensorRepo::get().set_eos(slot_); }

 private:
  unsigned slot_ = 0, signal_rate_ = 0;
  bool emit_signal_ = false;
  Caps caps_;
};

class TensorRepoSrc : public BaseSrc {
 public:
  explicit TensorRepoSrc(const std::string& name)
      : BaseSrc("tensor_reposrc", name, Caps::from_string(tensor_caps_template_all())) {
    prop_uint("slot-index", &slot_, "Slot index of the tensor repository");
    PropSpec s;
    s.name = "caps";
    s.type = PropType::CAPS;
    s.blurb = "Caps of the tensors (the first frame before the loop is closed is a zero tensor of these caps)";
    s.set = [this](const std::string& v) { caps_prop_ = Caps::from_string(v); };
    s.get = [this] { return caps_prop_.to_string(); };
    add_prop(s);
  }

 protected:
  bool on_start() override {
    first_ = true;
    return true;
  }
  void on_unlock() override { TensorRepo::get().flush(slot_); }
  Caps get_caps(const Caps* filter) override {
    Caps c = caps_prop_.is_empty() ? Caps::from_string(tensor_caps_template_all()) : caps_prop_;
    return filter ? c.intersect(*filter) : c;
  }
  bool set_caps(const Caps& caps) override { return tensor_config_from_caps(caps, &config_); }
  FlowReturn create(BufferPtr* out) override {
    if (first_) {
      // recurrence: the loop's first iteration reads a zero state
      first_ = false;
      auto b = make_buffer();
      for (unsigned i = 0; i < config_.info.num_tensors; ++i) {
        auto m = Memory::alloc_host(config_.info.size(static_cast<int>(i)));
        std::memset(m->data(), 0, m->size());
        b->mems.push_back(m);
      }
      b->pts = 0;
      *out = b;
      return FlowReturn::OK;
    }
    bool eos = false;
    Caps c;
    BufferPtr b = TensorRepo::get().get_buffer(slot_, &c, &eos);
    if (eos) return FlowReturn::EOS;
    if (!b) return FlowReturn::FLUSHING;
    *out = b;
    return FlowReturn::OK;
  }

 private:
  unsigned slot_ = 0;
  Caps caps_prop_;
  TensorsConfig config_;
  bool first_ = true;
};

// ======================================================== sparse enc / dec ====
// sparse payload: nnz values followed by nnz uint32 flat indices (gsttensor_sparseutil.c)
MemoryPtr sparse_encode(const MemoryPtr& m, const TensorInfo& ti) {
  const uint8_t* p = static_cast<const uint8_t*>(m->map_host());
  size_t es = dtype_size(ti.type);
  uint64_t n = element_count(ti.dim);
  std::vector<uint32_t> idx;
  idx.reserve(n / 4);
  static const uint8_t zero[8] = {0};
  for (uint64_t i = 0; i < n; ++i)
    if (std::memcmp(p + i * es, zero, es) != 0) idx.push_back(static_cast<uint32_t>(i));
  MetaInfo meta = MetaInfo::from_info(ti, Format::SPARSE);
  meta.nnz = static_cast<uint32_t>(idx.size());
  auto out = Memory::alloc_host(kMetaHeaderSize + idx.size() * (es + 4));
  uint8_t* o = static_cast<uint8_t*>(out->data());
  meta.write(o);
  uint8_t* vals = o + kMetaHeaderSize;
  for (size_t k = 0; k < idx.size(); ++k) std::memcpy(vals + k * es, p + static_cast<size_t>(idx[k]) * es, es);
  if (!idx.empty()) std::memcpy(vals + idx.size() * es, idx.data(), idx.size() * 4);
  return out;
}

bool sparse_decode(const MemoryPtr& m, MemoryPtr* out, TensorInfo* ti) {
  const uint8_t* p = static_cast<const uint8_t*>(m->map_host());
  MetaInfo meta;
  if (!MetaInfo::parse(p, m->size(), &meta) || meta.format != static_cast<uint32_t>(Format::SPARSE)) return false;
  if (!meta.to_info(ti)) return false;
  size_t es = dtype_size(ti->type);
  if (kMetaHeaderSize + meta.nnz * (es + 4) > m->size()) return false;
  auto o = Memory::alloc_host(ti->size());
  std::memset(o->data(), 0, o->size());
  const uint8_t* vals = p + kMetaHeaderSize;
  const uint8_t* idxp = vals + meta.nnz * es;
  uint64_t n = element_count(ti->dim);
  for (uint32_t k = 0; k < meta.nnz; ++k) {
    uint32_t i;
    std::memcpy(&i, idxp + k * 4, 4);
    if (i >= n) return false;
    std::memcpy(static_cast<uint8_t*>(o->data()) + static_cast<size_t>(i) * es, vals + k * es, es);
  }
  *out = o;
  return true;
}


// Device-resident tensors stay on the GPU (kernels/sparse.hip, K21): encode =
// count + scan, one 4-byte read-back of nnz to size the output, then the
// order-preserving compaction; decode = read back the 128-B header, zero-fill,
// scatter.  Small pinned read-back slots per element.
struct SparseDeviceCtx {
  StreamSet streams;
  MemoryPtr pinned;  // [0..3] nnz / bad flag, [128..255] header
  uint8_t* host(int dev, hipStream_t) {
    (void)dev;
    if (!pinned) pinned = Memory::alloc_pinned(256);
    return static_cast<uint8_t*>(pinned->data());
  }
};

MemoryPtr sparse_encode_device(const MemoryPtr& m, const TensorInfo& ti, int dev, SparseDeviceCtx& c) {
  hip::DeviceGuard g(dev);
  hipStream_t s = c.streams.get(dev);
  const void* x = m->map_device(dev, s);
  const int es = static_cast<int>(dtype_size(ti.type));
  const uint64_t n = element_count(ti.dim);
  const uint32_t nt = kernels::sparse_tiles(n);
  auto counts = Memory::alloc_device(std::max<size_t>(1, nt) * 4 + 4, dev, s);
  uint32_t* d_counts = static_cast<uint32_t*>(counts->data());
  uint32_t* d_nnz = d_counts + std::max<uint32_t>(1, nt);
  if (!kernels::sparse_count(x, es, n, d_counts, d_nnz, s)) return nullptr;
  uint8_t* h = c.host(dev, s);
  hip::check(hipMemcpyAsync(h, d_nnz, 4, hipMemcpyDeviceToHost, s), "sparse nnz D2H");
  hip::check(hipStreamSynchronize(s), "sparse nnz sync");
  uint32_t nnz;
  std::memcpy(&nnz, h, 4);
  MetaInfo meta = MetaInfo::from_info(ti, Format::SPARSE);
  meta.nnz = nnz;
  uint8_t hdr[kMetaHeaderSize];
  meta.write(hdr);
  auto out = Memory::alloc_device(kMetaHeaderSize + static_cast<size_t>(nnz) * (es + 4), dev, s);
  if (!kernels::sparse_compact(x, es, n, d_counts, out->data(), nnz, hdr, s)) return nullptr;
  m->record_use(s, dev);
  counts->record_use(s, dev);
  out->mark_ready(s);
  return out;
}

bool sparse_decode_device(const MemoryPtr& m, MemoryPtr* out, TensorInfo* ti, int dev, SparseDeviceCtx& c) {
  hip::DeviceGuard g(dev);
  hipStream_t s = c.streams.get(dev);
  if (m->size() < kMetaHeaderSize) return false;
  const uint8_t* src = static_cast<const uint8_t*>(m->map_device(dev, s));
  uint8_t* h = c.host(dev, s);
  hip::check(hipMemcpyAsync(h + 128, src, kMetaHeaderSize, hipMemcpyDeviceToHost, s), "sparse header D2H");
  hip::check(hipStreamSynchronize(s), "sparse header sync");
  MetaInfo meta;
  if (!MetaInfo::parse(h + 128, kMetaHeaderSize, &meta) || meta.format != static_cast<uint32_t>(Format::SPARSE))
    return false;
  if (!meta.to_info(ti)) return false;
  const size_t es = dtype_size(ti->type);
  if (kMetaHeaderSize + static_cast<size_t>(meta.nnz) * (es + 4) > m->size()) return false;
  auto o = Memory::alloc_device(ti->size(), dev, s);
  auto flag = Memory::alloc_device(4, dev, s);
  int* d_bad = static_cast<int*>(flag->data());
  hip::check(hipMemsetAsync(o->data(), 0, o->size(), s), "sparse zero fill");
  hip::check(hipMemsetAsync(d_bad, 0, 4, s), "sparse flag clear");
  if (!kernels::sparse_scatter(src + kMetaHeaderSize, static_cast<int>(es), meta.nnz, o->data(),
                               element_count(ti->dim), d_bad, s))
    return false;
  hip::check(hipMemcpyAsync(h, d_bad, 4, hipMemcpyDeviceToHost, s), "sparse flag D2H");
  hip::check(hipStreamSynchronize(s), "sparse decode sync");
  int bad;
  std::memcpy(&bad, h, 4);
  if (bad) return false;
  m->record_use(s, dev);
  o->mark_ready(s);
  *out = o;
  return true;
}

class TensorSparseEnc : public BaseTransform {
 public:
  explicit TensorSparseEnc(const std::string& name)
      : BaseTransform("tensor_sparse_enc", name, Caps::from_string(tensor_caps_template_static()),
                      Caps::from_string("other/tensors, format=(string)sparse, framerate=(fraction)[ 0/1, 2147483647/1 ]")) {}

 protected:
  Caps transform_caps(PadDirection dir, const Caps& caps, const Caps* filter) override {
    Caps r;
    for (size_t i = 0; i < caps.size(); ++i) {
      Structure s(kMimeTensors);
      s.set("format", Value::String(dir == PadDirection::SINK ? "sparse" : "static"));
      if (const Value* fr = caps.at(i).get("framerate")) s.set("framerate", *fr);
      r.append(s);
    }
    if (dir == PadDirection::SRC) r = Caps::from_string(tensor_caps_template_static());
    if (filter) r = r.intersect(*filter);
    return r;
  }
  bool set_caps(const Caps& in, const Caps&) override { return tensor_config_from_caps(in, &config_); }
  FlowReturn transform(const BufferPtr& inbuf, BufferPtr* outbuf) override {
    BufferPtr in;
    if (!buffer_from_config(inbuf, config_, &in)) return FlowReturn::ERROR;
    auto out = make_buffer();
    out->copy_metadata_from(*in);
    for (size_t i = 0; i < in->n_memory(); ++i) {
      const MemoryPtr& m = in->mems[i];
      const TensorInfo& ti = config_.info.at(static_cast<unsigned>(i));
      MemoryPtr o = m->on_device() ? sparse_encode_device(m, ti, m->device(), dev_) : sparse_encode(m, ti);
      if (!o) return FlowReturn::ERROR;
      out->mems.push_back(o);
    }
    *outbuf = out;
    return FlowReturn::OK;
  }

 private:
  TensorsConfig config_;
  SparseDeviceCtx dev_;
};

class TensorSparseDec : public BaseTransform {
 public:
  explicit TensorSparseDec(const std::string& name)
      : BaseTransform("tensor_sparse_dec", name,
                      Caps::from_string("other/tensors, format=(string)sparse, framerate=(fraction)[ 0/1, 2147483647/1 ]"),
                      Caps::from_string(tensor_caps_template_static() + "; " + tensor_caps_template_flexible())) {}

 protected:
  Caps transform_caps(PadDirection dir, const Caps& caps, const Caps* filter) override {
    Caps r = dir == PadDirection::SINK ? Caps::from_string(tensor_caps_template_flexible())
                                       : Caps::from_string("other/tensors, format=(string)sparse, framerate=(fraction)[ 0/1, 2147483647/1 ]");
    (void)caps;
    if (filter) r = r.intersect(*filter);
    return r;
  }
  Caps fixate_caps(PadDirection, const Caps& caps, Caps) override {
    // shapes are only known per buffer: negotiate flexible, refine to static at the first buffer
    Caps c = Caps::from_string(tensor_caps_template_flexible());
    Structure s = c.at(0);
    if (caps.size() && caps.at(0).get("framerate")) s.set("framerate", *caps.at(0).get("framerate"));
    s.fixate();
    Caps r;
    r.append(s);
    return r;
  }
  FlowReturn transform(const BufferPtr& in, BufferPtr* outbuf) override {
    auto out = make_buffer();
    out->copy_metadata_from(*in);
    TensorsConfig cfg;
    cfg.info.format = Format::STATIC;
    TensorsConfig inc;
    inc.info.format = Format::SPARSE;
    BufferPtr split_in;
    if (!buffer_from_config(in, inc, &split_in)) return FlowReturn::ERROR;
    for (auto& m : split_in->mems) {
      MemoryPtr o;
      TensorInfo ti;
      const bool ok = m->on_device() ? sparse_decode_device(m, &o, &ti, m->device(), dev_) : sparse_decode(m, &o, &ti);
      if (!ok) {
        post_error("tensor_sparse_dec: invalid sparse tensor");
        return FlowReturn::ERROR;
      }
      cfg.info.at(cfg.info.num_tensors) = ti;
      cfg.info.num_tensors++;
      out->mems.push_back(o);
    }
    int n, d;
    if (in_caps_.size() && in_caps_.at(0).get_fraction("framerate", &n, &d)) {
      cfg.rate_n = n;
      cfg.rate_d = d;
    } else {
      cfg.rate_n = 0;
      cfg.rate_d = 1;
    }
    if (!(cfg == last_)) {
      last_ = cfg;
      src_pad()->push_event(Event::make_caps(tensor_src_caps(src_pad(), cfg)));
    }
    *outbuf = out;
    return FlowReturn::OK;
  }

 private:
  TensorsConfig last_;
  SparseDeviceCtx dev_;
};

// ============================================================= tensor_debug ====
class TensorDebug : public BaseTransform {
 public:
  explicit TensorDebug(const std::string& name)
      : BaseTransform("tensor_debug", name, Caps::from_string(tensor_caps_template_all()),
                      Caps::from_string(tensor_caps_template_all())) {
    prop_string("output-method", &method_, "Output methods: console-info, console-warn, console-error, gstdebug-*");
    prop_enum("capability", &cap_mode_, {"disabled", "update", "update-F", "always"}, "How to print caps");
    prop_string("metadata", &meta_, "Print metadata: disabled, timestamps, queryserver");
    cap_mode_ = 2;
  }

 protected:
  bool set_caps(const Caps& in, const Caps&) override {
    if (cap_mode_ == 1 || cap_mode_ == 2 || cap_mode_ == 3) print("caps: " + in.to_string());
    return tensor_config_from_caps(in, &config_);
  }
  FlowReturn transform(const BufferPtr& in, BufferPtr* out) override {
    if (cap_mode_ == 3) print("caps: " + in_caps_.to_string());
    if (meta_.find("timestamp") != std::string::npos)
      print(strfmt("pts=", in->pts, " dts=", in->dts, " duration=", in->duration));
    if (meta_.find("queryserver") != std::string::npos) print(strfmt("client_id=", in->meta.client_id));
    if (!silent_) {
      std::string s = strfmt("buffer: ", in->n_memory(), " memories [");
      for (auto& m : in->mems) s += strfmt(m->size(), m->on_device() ? "@dev " : " ");
      print(s + "]");
    }
    *out = in;
    return FlowReturn::OK;
  }

 private:
  void print(const std::string& s) {
    if (method_.find("warn") != std::string::npos)
      NNSX_LOGW(name(), s);
    else if (method_.find("error") != std::string::npos)
      NNSX_LOGE(name(), s);
    else
      std::fprintf(stdout, "[%s] %s\n", name().c_str(), s.c_str());
  }
  std::string method_ = "console-info", meta_ = "disabled";
  int cap_mode_ = 2;
  TensorsConfig config_;
};

// ===================================================================== join ====
class Join : public Element {
 public:
  explicit Join(const std::string& name) : Element("join", name) {
    add_template("sink_%u", PadDirection::SINK, PadPresence::REQUEST, Caps::Any());
    add_template("src", PadDirection::SRC, PadPresence::ALWAYS, Caps::Any());
    prop_readonly("active-pad", [this] {
      std::lock_guard<std::mutex> lk(mu_);
      return active_;
    }, "The currently active sink pad");
    // gst/join/gstjoin.c:448 (read-only; counts the requested sink pads)
    prop_readonly("n-pads", [this] {
      size_t n = 0;
      for (Pad* p : sink_pads()) n += p != nullptr;
      return std::to_string(n);
    }, "The number of sink pads");
  }
  FlowReturn chain(Pad* pad, BufferPtr buf) override {
    std::lock_guard<std::mutex> lk(mu_);
    if (active_ != pad->name()) {
      active_ = pad->name();
      if (pad->has_current_caps()) src_pad()->push_event(Event::make_caps(pad->current_caps()));
    }
    return src_pad()->push(std::move(buf));
  }
  bool sink_event(Pad* pad, Event& ev) override {
    std::lock_guard<std::mutex> lk(mu_);
    if (ev.type == EventType::EOS) {
      eos_pads_++;
      if (eos_pads_ < sink_pads().size()) return true;
      return forward_event_downstream(ev);
    }
    if (ev.type == EventType::CAPS) {
      if (active_.empty() || active_ == pad->name()) {
        active_ = pad->name();
        return forward_event_downstream(ev);
      }
      return true;
    }
    if (ev.type == EventType::STREAM_START || ev.type == EventType::SEGMENT) {
      if (sent_start_.count(ev.type)) return true;
      sent_start_.insert(ev.type);
    }
    return forward_event_downstream(ev);
  }
  bool start() override {
    eos_pads_ = 0;
    active_.clear();
    sent_start_.clear();
    return true;
  }

 private:
  std::mutex mu_;
  std::string active_;
  size_t eos_pads_ = 0;
  std::set<EventType> sent_start_;
};

// ============================================================ datarepo src ====
// Reads fixed-size tensor records from a file (gst/datarepo/gstdatareposrc.c);
// record layout is given by `caps` (static tensors), or a JSON sidecar.
class DataRepoSrc : public BaseSrc {
 public:
  explicit DataRepoSrc(const std::string& name) : BaseSrc("datareposrc", name, Caps::Any()) {
    prop_string("location", &location_, "Location of the file to read");
    prop_string("json", &json_, "Sidecar JSON written by datareposink (gst_caps, total_samples, sample_size)");
    prop_int("start-sample-index", &start_, "Start index of the samples to read");
    prop_int("stop-sample-index", &stop_, "Stop index of the samples to read (-1 = all)");
    prop_int("epochs", &epochs_, "Repetitions over the selected samples");
    prop_bool("is-shuffle", &shuffle_, "Shuffle the samples every epoch");
    PropSpec s;
    s.name = "caps";
    s.type = PropType::CAPS;
    s.blurb = "Caps of the records (other/tensors static)";
    s.set = [this](const std::string& v) { caps_prop_ = Caps::from_string(v); };
    s.get = [this] { return caps_prop_.to_string(); };
    add_prop(s);
  }

 protected:
  Caps get_caps(const Caps* filter) override {
    Caps c = caps_prop_;
    return filter ? c.intersect(*filter) : c;
  }
  bool set_caps(const Caps& caps) override {
    if (!tensor_config_from_caps(caps, &config_)) return false;
    record_ = config_.info.size();
    return record_ > 0;
  }
  bool on_start() override {
    if (!json_.empty()) {
      std::ifstream jf(json_);
      std::string js((std::istreambuf_iterator<char>(jf)), std::istreambuf_iterator<char>());
      auto cpos = js.find("\"gst_caps\"");
      if (cpos != std::string::npos) {
        auto q1 = js.find('"', js.find(':', cpos) + 1);
        auto q2 = js.find('"', q1 + 1);
        if (q1 != std::string::npos && q2 != std::string::npos) caps_prop_ = Caps::from_string(js.substr(q1 + 1, q2 - q1 - 1));
      }
    }
    f_.close();
    f_.clear();
    f_.open(location_, std::ios::binary);
    if (!f_) {
      post_error("Could not open file \"" + location_ + "\" for reading.");
      return false;
    }
    f_.seekg(0, std::ios::end);
    file_size_ = static_cast<int64_t>(f_.tellg());
    epoch_ = 0;
    cursor_ = -1;
    return true;
  }
  FlowReturn create(BufferPtr* out) override {
    int64_t total = record_ ? file_size_ / static_cast<int64_t>(record_) : 0;
    int64_t last = stop_ < 0 ? total - 1 : std::min(stop_, total - 1);
    if (cursor_ < 0) {
      build_order(last);
      cursor_ = 0;
    }
    if (cursor_ >= static_cast<int64_t>(order_.size())) {
      if (++epoch_ >= epochs_) return FlowReturn::EOS;
      build_order(last);
      cursor_ = 0;
    }
    int64_t idx = order_[cursor_++];
    f_.seekg(idx * static_cast<int64_t>(record_));
    auto b = make_buffer();
    for (unsigned i = 0; i < config_.info.num_tensors; ++i) {
      auto m = Memory::alloc_host(config_.info.size(static_cast<int>(i)));
      f_.read(static_cast<char*>(m->data()), static_cast<std::streamsize>(m->size()));
      b->mems.push_back(m);
    }
    b->offset = idx;
    *out = b;
    return FlowReturn::OK;
  }

 private:
  void build_order(int64_t last) {
    order_.clear();
    for (int64_t i = start_; i <= last; ++i) order_.push_back(i);
    if (shuffle_) {
      std::mt19937_64 rng(static_cast<uint64_t>(epoch_) * 7919 + 17);
      std::shuffle(order_.begin(), order_.end(), rng);
    }
  }
  std::string location_, json_;
  int64_t start_ = 0, stop_ = -1, epochs_ = 1, epoch_ = 0, cursor_ = -1, file_size_ = 0;
  bool shuffle_ = false;
  Caps caps_prop_ = Caps::Any();
  TensorsConfig config_;
  size_t record_ = 0;
  std::ifstream f_;
  std::vector<int64_t> order_;
};

class DataRepoSink : public BaseSink {
 public:
  explicit DataRepoSink(const std::string& name) : BaseSink("datareposink", name, Caps::Any()) {
    prop_string("location", &location_, "Location of the file to write");
    prop_string("json", &json_, "Sidecar JSON describing the records");
  }

 protected:
  bool start() override {
    BaseSink::start();
    count_ = 0;
    f_.open(location_, std::ios::binary | std::ios::trunc);
    return static_cast<bool>(f_);
  }
  bool set_caps(const Caps& c) override {
    caps_ = c;
    return true;
  }
  FlowReturn render(const BufferPtr& buf) override {
    size_t sz = 0;
    for (auto& m : buf->mems) {
      f_.write(static_cast<const char*>(m->map_host()), static_cast<std::streamsize>(m->size()));
      sz += m->size();
    }
    sample_size_ = sz;
    ++count_;
    return FlowReturn::OK;
  }
  void on_eos() override {
    f_.flush();
    if (!json_.empty()) {
      std::ofstream j(json_);
      j << "{\"gst_caps\":\"" << replace_all(caps_.to_string(), "\"", "\\\"") << "\",\"total_samples\":" << count_
        << ",\"sample_size\":" << sample_size_ << "}\n";
    }
  }
  bool stop() override {
    f_.close();
    return true;
  }

 private:
  std::string location_, json_;
  std::ofstream f_;
  Caps caps_;
  int64_t count_ = 0;
  size_t sample_size_ = 0;
};


// ========================================================== tensor_trainer ====
// gsttensor_trainer.c: samples (inputs then labels, one buffer each) go to the
// trainer sub-plugin; a 1:1:4 float64 status tensor (loss, accuracy, val_loss,
// val_accuracy) is pushed on the first sample and at every epoch end; EOS waits
// for the sub-plugin to finish training (gsttensor_trainer.c:713-724).
class TensorTrainer : public BaseTransform {
 public:
  explicit TensorTrainer(const std::string& name)
      : BaseTransform("tensor_trainer", name, Caps::from_string(tensor_caps_template_static()),
                      Caps::from_string(tensor_caps_template_static())) {
    prop_string("framework", &framework_, "Neural network framework to be used for model training");
    prop_string("model-config", &props_.model_config, "Model configuration file path");
    prop_string("model-save-path", &props_.model_save_path, "Path to save the trained model");
    prop_string("model-load-path", &props_.model_load_path, "Path of a model to continue training from");
    prop_string("input-dim", &input_dim_, "Input tensors dimension from inner array");
    prop_string("input-type", &input_type_, "Type of each element of the input tensors");
    prop_uint("num-inputs", &props_.num_inputs, "Number of input tensors in a sample");
    prop_uint("num-labels", &props_.num_labels, "Number of label tensors in a sample");
    prop_uint("num-training-samples", &props_.num_training_samples, "Training samples per epoch");
    prop_uint("num-validation-samples", &props_.num_validation_samples, "Validation samples per epoch");
    prop_uint("epochs", &props_.epochs, "Number of epochs");
    prop_int("device", &device_, "GPU used for training (-1 = CPU, -2 = follow input placement)");
    prop_readonly("epoch-count", [this] { return std::to_string(last_.epoch_count); }, "Completed epochs");
    prop_readonly("training-loss", [this] { return strfmt(last_.training_loss); }, "Last training loss");
    prop_readonly("training-accuracy", [this] { return strfmt(last_.training_accuracy); }, "Last training accuracy");
    prop_readonly("validation-loss", [this] { return strfmt(last_.validation_loss); }, "Last validation loss");
    prop_readonly("validation-accuracy", [this] { return strfmt(last_.validation_accuracy); },
                  "Last validation accuracy");
    props_.num_training_samples = 1;
    props_.num_validation_samples = 0;
  }

 protected:
  bool start() override {
    total_ = 0;
    last_ = TrainerStatus();
    reported_epoch_ = 0;
    instance_.reset();
    return true;
  }
  bool stop() override {
    if (instance_) instance_->stop();
    instance_.reset();
    return true;
  }
  void unlock() override {
    if (instance_) instance_->stop();
  }

  Caps transform_caps(PadDirection dir, const Caps&, const Caps* filter) override {
    Caps r;
    if (dir == PadDirection::SINK) {
      TensorsConfig c;
      c.info.num_tensors = 1;
      c.info.at(0).type = DType::FLOAT64;
      c.info.at(0).dim = {1, 1, 4, 1, 1, 1, 1, 1};
      c.rate_n = 0;
      c.rate_d = 1;
      r = caps_from_config(c);
    } else if (!input_dim_.empty() && !input_type_.empty()) {
      TensorsConfig c;
      c.info.num_tensors = c.info.parse_dimensions(input_dim_);
      c.info.parse_types(input_type_);
      r = caps_from_config(c);
      Structure s = r.at(0);
      s.set("framerate", Value::FractionRange(0, 1, INT32_MAX, 1));
      r = Caps();
      r.append(s);
    } else {
      r = Caps::from_string(tensor_caps_template_static());
    }
    if (filter) r = r.intersect(*filter);
    return r;
  }

  bool set_caps(const Caps& in, const Caps&) override {
    if (!tensor_config_from_caps(in, &config_)) return false;
    if (!input_dim_.empty()) {
      TensorsInfo want;
      want.num_tensors = want.parse_dimensions(input_dim_);
      if (!input_type_.empty()) want.parse_types(input_type_);
      if (!(want == config_.info)) {
        post_error("tensor_trainer: the input tensors info differs from input-dim/input-type");
        return false;
      }
    }
    if (config_.info.num_tensors != props_.num_inputs + props_.num_labels) {
      post_error("tensor_trainer: num-inputs + num-labels must equal the number of incoming tensors");
      return false;
    }
    if (instance_) return true;
    auto fw = find_trainer(framework_);
    if (!fw) {
      post_error("tensor_trainer: unknown framework '" + framework_ + "'");
      return false;
    }
    props_.input_info = config_.info;
    props_.device = device_ == -2 ? -1 : device_;
    try {
      instance_ = fw->create(props_);
      if (!instance_->start()) throw Error("start failed");
    } catch (const std::exception& e) {
      post_error(std::string("tensor_trainer: ") + e.what());
      instance_.reset();
      return false;
    }
    return true;
  }

  FlowReturn transform(const BufferPtr& inbuf, BufferPtr* out) override {
    *out = nullptr;
    if (!instance_) return FlowReturn::NOT_NEGOTIATED;
    BufferPtr in;
    if (!buffer_from_config(inbuf, config_, &in)) return FlowReturn::ERROR;
    if (in->n_memory() != config_.info.num_tensors) {
      post_error("tensor_trainer: invalid number of memory blocks");
      return FlowReturn::ERROR;
    }
    for (unsigned i = 0; i < config_.info.num_tensors; ++i) {
      if (in->mems[i]->size() != config_.info.size(static_cast<int>(i))) {
        post_error(strfmt("tensor_trainer: invalid tensor size (", i, "'th memory chunk: ", in->mems[i]->size(), ")"));
        return FlowReturn::ERROR;
      }
    }
    uint64_t per_epoch = static_cast<uint64_t>(props_.num_training_samples) + props_.num_validation_samples;
    bool is_val = per_epoch && (total_ % per_epoch) >= props_.num_training_samples;
    bool ok;
    try {
      ok = instance_->push_data(in->mems, is_val);
    } catch (const std::exception& e) {
      post_error(std::string("tensor_trainer: ") + e.what());
      return FlowReturn::ERROR;
    }
    if (!ok) {
      post_error("tensor_trainer: push_data failed");
      return FlowReturn::ERROR;
    }
    ++total_;
    TrainerStatus st = instance_->status();
    if (total_ == 1 || st.epoch_count != reported_epoch_) {
      reported_epoch_ = st.epoch_count;
      last_ = st;
      auto m = Memory::alloc_host(4 * sizeof(double));
      double* d = static_cast<double*>(m->data());
      d[0] = st.training_loss;
      d[1] = st.training_accuracy;
      d[2] = st.validation_loss;
      d[3] = st.validation_accuracy;
      auto b = make_buffer();
      b->copy_metadata_from(*in);
      b->mems.push_back(m);
      if (pad_caps_is_flexible(src_pad())) {
        TensorInfo ti;
        ti.type = DType::FLOAT64;
        ti.dim = {1, 1, 4, 1, 1, 1, 1, 1};
        b->mems[0] = make_flexible(m, MetaInfo::from_info(ti, Format::FLEXIBLE));
      }
      *out = b;
    }
    return FlowReturn::OK;
  }

  bool handle_sink_event(Event& ev) override {
    if (ev.type == EventType::EOS && instance_) {
      if (!instance_->status().complete) {
        NNSX_LOGI(name(), "EOS before training completed: waiting");
        instance_->wait_complete(-1);
      }
      last_ = instance_->status();
    }
    return true;
  }

 private:
  std::string framework_ = "pytorch", input_dim_, input_type_;
  int device_ = -2;
  TrainerProperties props_;
  TensorsConfig config_;
  std::unique_ptr<TrainerInstance> instance_;
  uint64_t total_ = 0;
  unsigned reported_epoch_ = 0;
  TrainerStatus last_;
};

}  // namespace

void register_src_iio();  // tensor_src_iio.cc

void register_extra_elements() {
  register_src_iio();
  register_element("tensor_if", "Filter/Tensor", "Controls streams based on tensor(s) values",
                   [](const std::string& n) { return std::make_unique<TensorIf>(n); });
  register_element("tensor_crop", "Filter/Tensor", "Crops the raw tensor with the regions of the info tensor",
                   [](const std::string& n) { return std::make_unique<TensorCrop>(n); });
  register_element("tensor_rate", "Filter/Tensor", "Adjusts the framerate of tensor streams (QoS throttling)",
                   [](const std::string& n) { return std::make_unique<TensorRate>(n); });
  register_element("tensor_reposink", "Sink/Tensor", "Pushes tensors into the tensor repository slot",
                   [](const std::string& n) { return std::make_unique<TensorRepoSink>(n); });
  register_element("tensor_reposrc", "Source/Tensor", "Pops tensors from the tensor repository slot (recurrence)",
                   [](const std::string& n) { return std::make_unique<TensorRepoSrc>(n); });
  register_element("tensor_sparse_enc", "Filter/Tensor", "Encodes static tensors into sparse tensors",
                   [](const std::string& n) { return std::make_unique<TensorSparseEnc>(n); });
  register_element("tensor_sparse_dec", "Filter/Tensor", "Decodes sparse tensors into static tensors",
                   [](const std::string& n) { return std::make_unique<TensorSparseDec>(n); });
  register_element("tensor_debug", "Filter/Tensor", "Prints tensor stream information",
                   [](const std::string& n) { return std::make_unique<TensorDebug>(n); });
  register_element("join", "Generic", "N-to-1 pass-through of whichever pad is active",
                   [](const std::string& n) { return std::make_unique<Join>(n); });
  register_element("datareposrc", "Source/File", "Reads fixed-size tensor records from a data repository file",
                   [](const std::string& n) { return std::make_unique<DataRepoSrc>(n); });
  register_element("datareposink", "Sink/File", "Writes tensor records into a data repository file",
                   [](const std::string& n) { return std::make_unique<DataRepoSink>(n); });
  register_element("tensor_trainer", "Trainer/Tensor", "Trains a model on the incoming tensor samples",
                   [](const std::string& n) { return std::make_unique<TensorTrainer>(n); });
}

}  // namespace nnsx
