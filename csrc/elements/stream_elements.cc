// Multi-stream tensor elements: tensor_mux, tensor_demux, tensor_merge,
// tensor_split, tensor_aggregator, plus the collect-pads time-sync policies.
//
// Reference: gst/nnstreamer/nnstreamer_plugin_api_impl.c:20-441 (time sync:
// nosync / slowest / basepad / refresh), gsttensor_mux.c:360-540,
// gsttensor_demux.c:343-556, gsttensor_merge.c:380-604,
// gsttensor_split.c:414-532, gsttensor_aggregator.c:540-946.
//
// Zero-copy: mux/demux/split pass Memory references or sub-views; merge and
// aggregator concatenate with pitched copies (hipMemcpy2DAsync on the
// element's stream for HBM-resident tensors, memcpy on the host).
#include <algorithm>
#include <cstring>
#include <deque>

#include "core/log.h"
#include "elements/elements.h"
#include "elements/tensor_common.h"
#include "runtime/base.h"
#include "runtime/pipeline.h"

namespace nnsx {

namespace {

// ------------------------------------------------------------- time sync ----
enum SyncMode { SYNC_NOSYNC = 0, SYNC_SLOWEST, SYNC_BASEPAD, SYNC_REFRESH, SYNC_END };

struct PadState {
  BufferPtr last;  // GstTensorCollectPadData::buffer
};

// GstClockTime semantics: an unset timestamp (GST_CLOCK_TIME_NONE) compares as
// the largest time, so untimestamped streams (multifilesrc) still pair up.
inline int64_t sync_ts(const BufferPtr& b) { return b->pts < 0 ? INT64_MAX : b->pts; }

class TimeSync {
 public:
  int mode = SYNC_SLOWEST;
  std::string option;
  unsigned basepad_id = 0;
  int64_t basepad_duration = INT32_MAX;

  bool parse() {
    if (mode == SYNC_BASEPAD) {
      auto p = split(option, ':', 2);
      basepad_id = p.size() > 0 && !strip(p[0]).empty() ? static_cast<unsigned>(to_uint(p[0])) : 0;
      basepad_duration = p.size() > 1 ? static_cast<int64_t>(to_uint(p[1])) : INT32_MAX;
    }
    return true;
  }

  bool is_eos(size_t total, size_t empty) const {
    if (mode == SYNC_REFRESH) return empty == total;
    return empty > 0;
  }

  // returns true on EOS; updates current and copies metadata of the chosen buffer
  bool get_current_time(CollectPads& cp, int64_t* current, Buffer* meta_out) {
    size_t count = 0, empty = 0;
    auto pads = cp.pads();
    for (auto* d : pads) {
      BufferPtr b = cp.peek(d);
      if (b) {
        bool upd = false;
        switch (mode) {
          case SYNC_NOSYNC:
          case SYNC_SLOWEST:
          case SYNC_REFRESH:
            if (*current < sync_ts(b)) upd = true;
            break;
          case SYNC_BASEPAD:
            if (count == basepad_id) upd = true;
            break;
        }
        if (upd) {
          *current = sync_ts(b);
          meta_out->copy_metadata_from(*b);
        }
      } else {
        ++empty;
      }
      ++count;
    }
    return is_eos(pads.size(), empty);
  }

  // GstTensorCollectPadData update (returns false: "popped an old buffer, not ready")
  bool buffer_update(CollectPads& cp, CollectPads::PadData* d, int64_t current, int64_t base) {
    BufferPtr b = cp.peek(d);
    if (!b) return true;
    if (sync_ts(b) < current) {
      d->last = cp.pop(d);
      return false;
    }
    auto absdiff = [](int64_t a, int64_t c) { return a > c ? a - c : c - a; };
    bool keep = (mode == SYNC_SLOWEST && d->last && absdiff(current, sync_ts(d->last)) < absdiff(current, sync_ts(b))) ||
                (mode == SYNC_BASEPAD && d->last && absdiff(current, sync_ts(b)) > base);
    if (!keep) d->last = cp.pop(d);
    return true;
  }

  // Collect one memory list from every pad; fills mems + per-tensor configs.
  // returns false when not ready or EOS (*eos says which)
  bool collect(CollectPads& cp, int64_t current, std::vector<MemoryPtr>* mems, TensorsConfig* out_cfg,
               std::vector<Format>* in_formats, bool* eos) {
    *eos = false;
    auto pads = cp.pads();
    int64_t base = 0;
    if (mode == SYNC_BASEPAD) {
      if (basepad_id >= pads.size()) return false;
      auto* d = pads[basepad_id];
      BufferPtr b = cp.peek(d);
      if (b && d->last) {
        int64_t diff = b->pts - d->last->pts;
        if (diff < 0) diff = -diff;
        base = std::min<int64_t>(basepad_duration, diff - 1);
      }
    }
    int rate_n = INT32_MAX, rate_d = INT32_MAX;
    size_t empty = 0;
    out_cfg->info = TensorsInfo();
    out_cfg->info.format = Format::STATIC;
    for (auto* d : pads) {
      TensorsConfig in;
      if (!d->pad->has_current_caps() || !tensor_config_from_caps(d->pad->current_caps(), &in) || !in.valid())
        return false;
      rate_d = std::min(rate_d, in.rate_d);
      rate_n = std::min(rate_n, in.rate_n);
      BufferPtr b;
      bool is_empty = false;
      switch (mode) {
        case SYNC_SLOWEST:
        case SYNC_BASEPAD:
          if (!buffer_update(cp, d, current, base)) return false;
          b = d->last;
          is_empty = !b;
          break;
        case SYNC_NOSYNC:
          b = cp.pop(d);
          is_empty = !b;
          break;
        case SYNC_REFRESH:
          b = cp.pop(d);
          if (b) {
            d->last = b;
          } else {
            if (!d->last) return false;  // not all buffers arrived yet
            is_empty = true;
            b = d->last;
          }
          break;
      }
      if (b) {
        BufferPtr bb;
        if (!buffer_from_config(b, in, &bb)) return false;
        if (in.is_flexible()) out_cfg->info.format = Format::FLEXIBLE;
        for (size_t i = 0; i < bb->n_memory(); ++i) {
          unsigned idx = out_cfg->info.num_tensors;
          out_cfg->info.at(idx) = in.is_flexible() ? TensorInfo() : in.info.at(static_cast<unsigned>(i));
          out_cfg->info.num_tensors = idx + 1;
          mems->push_back(bb->mems[i]);
          in_formats->push_back(in.info.format);
        }
      }
      if (is_empty) ++empty;
    }
    out_cfg->rate_n = rate_n;
    out_cfg->rate_d = rate_d;
    *eos = is_eos(pads.size(), empty);
    return !*eos;
  }
};

// Base for collect-pads aggregators (mux / merge)
class CollectElement : public Element {
 public:
  CollectElement(const std::string& factory, const std::string& name, const Caps& sink_caps, const Caps& src_caps)
      : Element(factory, name), cp_(this) {
    add_template("sink_%u", PadDirection::SINK, PadPresence::REQUEST, sink_caps);
    add_template("src", PadDirection::SRC, PadPresence::ALWAYS, src_caps);
    prop_enum("sync-mode", &sync_.mode, {"nosync", "slowest", "basepad", "refresh"},
              "Time synchronization mode", [this] { sync_.parse(); });
    prop_string("sync-option", &sync_.option, "Option for the time synchronization mode ?", [this] { sync_.parse(); });
  }

  Pad* request_pad(const PadTemplate& t, const std::string& name) override {
    Pad* p = Element::request_pad(t, name);
    if (p && p->direction() == PadDirection::SINK) cp_.add_pad(p);
    return p;
  }
  void release_pad(Pad* p) override {
    cp_.remove_pad(p);
    Element::release_pad(p);
  }

  bool start() override {
    cp_.reset();
    need_set_time_ = true;
    current_ = 0;
    negotiated_ = false;
    need_segment_ = true;
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
      case EventType::EOS: {
        bool all = cp_.set_eos(pad, [this] { return collected(); });
        if (all) send_eos();
        return true;
      }
      case EventType::CAPS:
        return true;  // output caps are decided at the first collect
      case EventType::SEGMENT:
      case EventType::STREAM_START:
        return true;
      case EventType::FLUSH_START:
        cp_.set_flushing(true);
        return forward_event_downstream(ev);
      case EventType::FLUSH_STOP:
        cp_.reset();
        return forward_event_downstream(ev);
      default:
        return forward_event_downstream(ev);
    }
  }

  Caps query_caps(Pad* pad, const Caps* filter) override {
    Caps c = pad->template_caps();
    return filter ? c.intersect(*filter) : c;
  }

 protected:
  // called with the collect-pads lock held; implementations push downstream
  virtual FlowReturn collected() = 0;

  void send_eos() {
    if (eos_sent_) return;
    eos_sent_ = true;
    Event e = Event::make_eos();
    src_pad()->push_event(e);
  }

  void ensure_stream_start(int64_t pts) {
    if (!stream_started_) {
      src_pad()->push_event(Event::make_stream_start(name()));
      stream_started_ = true;
    }
    if (need_segment_) {
      Segment s;
      s.start = pts >= 0 ? pts : 0;
      src_pad()->push_event(Event::make_segment(s));
      need_segment_ = false;
    }
  }

  bool set_src_caps(const TensorsConfig& cfg) {
    if (negotiated_ && cfg == last_cfg_) return true;
    Caps c = tensor_src_caps(src_pad(), cfg);
    if (!src_pad()->push_event(Event::make_caps(c))) return false;
    negotiated_ = true;
    last_cfg_ = cfg;
    out_flexible_ = c.size() && c.at(0).get_string_or("format", "static") == "flexible";
    return true;
  }

  // returns (buffer collected?, eos?)
  bool collect_buffer(std::vector<MemoryPtr>* mems, TensorsConfig* cfg, std::vector<Format>* fmts, Buffer* meta,
                      bool* eos) {
    *eos = false;
    if (need_set_time_) {
      if (sync_.get_current_time(cp_, &current_, meta)) {
        *eos = true;
        return false;
      }
      need_set_time_ = false;
    } else {
      meta->pts = current_;
    }
    bool ok = sync_.collect(cp_, current_, mems, cfg, fmts, eos);
    meta->pts = current_;
    return ok;
  }

  CollectPads cp_;
  TimeSync sync_;
  bool need_set_time_ = true;
  int64_t current_ = 0;
  bool negotiated_ = false, need_segment_ = true, eos_sent_ = false, stream_started_ = false;
  bool out_flexible_ = false;
  TensorsConfig last_cfg_;
  StreamSet streams_;
};

// -------------------------------------------------------------- tensor_mux ----
class TensorMux : public CollectElement {
 public:
  explicit TensorMux(const std::string& name)
      : CollectElement("tensor_mux", name, Caps::from_string(tensor_caps_template_all()),
                       Caps::from_string(tensor_caps_template_static() + "; " + tensor_caps_template_flexible())) {}

 protected:
  FlowReturn collected() override {
    std::vector<MemoryPtr> mems;
    std::vector<Format> fmts;
    TensorsConfig cfg;
    Buffer meta;
    bool eos;
    bool ok = collect_buffer(&mems, &cfg, &fmts, &meta, &eos);
    if (!ok) {
      if (eos) {
        send_eos();
        return FlowReturn::EOS;
      }
      return FlowReturn::OK;
    }
    if (!set_src_caps(cfg)) {
      post_error("tensor_mux: failed to set caps");
      return FlowReturn::NOT_NEGOTIATED;
    }
    ensure_stream_start(meta.pts);
    auto out = make_buffer();
    out->copy_metadata_from(meta);
    out->pts = current_;
    for (size_t i = 0; i < mems.size(); ++i) {
      if (out_flexible_ && fmts[i] != Format::FLEXIBLE)
        out->mems.push_back(make_flexible(mems[i], MetaInfo::from_info(cfg.info.at(static_cast<unsigned>(i)))));
      else
        out->mems.push_back(mems[i]);
    }
    need_set_time_ = true;
    return src_pad()->push(out);
  }
};

// ------------------------------------------------------------ tensor_merge ----
class TensorMerge : public CollectElement {
 public:
  explicit TensorMerge(const std::string& name)
      : CollectElement("tensor_merge", name, Caps::from_string(tensor_caps_template_static()),
                       Caps::from_string(tensor_caps_template_static())) {
    prop_enum("mode", &mode_, {"linear"}, "Tensor Merge mode ?");
    prop_string("option", &option_, "Option for the tensor Merge mode ?", [this] {
      axis_ = static_cast<int>(to_int(option_, 0));
      if (axis_ < 0 || axis_ >= kRankLimit) throw Error("tensor_merge: invalid option (axis) " + option_);
    });
  }

 protected:
  FlowReturn collected() override {
    std::vector<MemoryPtr> mems;
    std::vector<Format> fmts;
    TensorsConfig cfg;
    Buffer meta;
    bool eos;
    if (!collect_buffer(&mems, &cfg, &fmts, &meta, &eos)) {
      if (eos) {
        send_eos();
        return FlowReturn::EOS;
      }
      return FlowReturn::OK;
    }
    // merged config: same type, dims equal except the merge axis (summed)
    TensorsConfig out;
    out.rate_n = cfg.rate_n;
    out.rate_d = cfg.rate_d;
    out.info.resize(1);
    TensorInfo o = cfg.info.at(0);
    for (unsigned i = 1; i < cfg.info.num_tensors; ++i) {
      const auto& t = cfg.info.at(i);
      if (t.type != o.type) {
        post_error("tensor_merge: all tensors must have the same type");
        return FlowReturn::ERROR;
      }
      for (int d = 0; d < kRankLimit; ++d) {
        if (d == axis_) continue;
        if (t.dim[d] != o.dim[d]) {
          post_error("tensor_merge: dimensions other than the merge axis must match");
          return FlowReturn::ERROR;
        }
      }
      o.dim[axis_] += t.dim[axis_];
    }
    out.info.at(0) = o;
    if (!set_src_caps(out)) return FlowReturn::NOT_NEGOTIATED;
    ensure_stream_start(meta.pts);
    // concatenation: for each outer index, copy each input's [inner x dim_axis] block
    size_t es = dtype_size(o.type);
    size_t inner = es;
    for (int d = 0; d < axis_; ++d) inner *= o.dim[d];
    size_t outer = 1;
    for (int d = axis_ + 1; d < kRankLimit; ++d) outer *= o.dim[d];
    size_t out_row = inner * o.dim[axis_];
    int dev = -1;
    for (auto& m : mems)
      if (m->on_device()) dev = m->device();
    hipStream_t s = dev >= 0 ? streams_.get(dev) : nullptr;
    MemoryPtr om = alloc_output(o.size(), dev, s);
    size_t col = 0;
    for (size_t i = 0; i < mems.size(); ++i) {
      size_t blk = inner * cfg.info.at(static_cast<unsigned>(i)).dim[axis_];
      char* dst = static_cast<char*>(om->data()) + col;
      if (dev >= 0) {
        const void* src = mems[i]->map_device(dev, s);
        hip::check(hipMemcpy2DAsync(dst, out_row, src, blk, blk, outer, hipMemcpyDeviceToDevice, s), "merge 2D");
        mems[i]->record_use(s, dev);
      } else {
        const char* src = static_cast<const char*>(mems[i]->map_host());
        for (size_t r = 0; r < outer; ++r) std::memcpy(dst + r * out_row, src + r * blk, blk);
      }
      col += blk;
    }
    if (dev >= 0) om->mark_ready(s);
    auto b = make_buffer();
    b->copy_metadata_from(meta);
    b->pts = current_;
    b->mems.push_back(om);
    need_set_time_ = true;
    return src_pad()->push(b);
  }

 private:
  int mode_ = 0;
  std::string option_ = "0";
  int axis_ = 0;
};

// ------------------------------------------------------------ tensor_demux ----
class TensorDemux : public Element {
 public:
  explicit TensorDemux(const std::string& name) : Element("tensor_demux", name) {
    add_template("sink", PadDirection::SINK, PadPresence::ALWAYS, Caps::from_string(tensor_caps_template_all()));
    add_template("src_%u", PadDirection::SRC, PadPresence::SOMETIMES, Caps::from_string(tensor_caps_template_all()));
    prop_string("tensorpick", &pick_str_, "Choose nth tensor among tensors ?", [this] {
      picks_.clear();
      for (auto& g : split(pick_str_, ',')) {
        std::vector<unsigned> grp;
        for (auto& x : split_any(g, ":+"))
          if (!strip(x).empty()) grp.push_back(static_cast<unsigned>(to_uint(x)));
        if (!grp.empty()) picks_.push_back(grp);
      }
    });
  }

  Pad* request_pad(const PadTemplate& t, const std::string& name) override { return Element::request_pad(t, name); }

  bool sink_event(Pad*, Event& ev) override {
    if (ev.type == EventType::CAPS) {
      if (!tensor_config_from_caps(ev.caps, &config_)) return false;
      unsigned n = config_.is_flexible() ? 0 : config_.info.num_tensors;
      unsigned nout = picks_.empty() ? n : static_cast<unsigned>(picks_.size());
      for (unsigned i = 0; i < nout; ++i) {
        Pad* p = get_pad("src_" + std::to_string(i));
        if (!p) p = Element::request_pad(templates_[1], "src_" + std::to_string(i));
        if (!config_.is_flexible()) {
          TensorsConfig oc;
          oc.rate_n = config_.rate_n;
          oc.rate_d = config_.rate_d;
          std::vector<unsigned> grp = picks_.empty() ? std::vector<unsigned>{i} : picks_[i];
          oc.info.resize(static_cast<unsigned>(grp.size()));
          for (size_t k = 0; k < grp.size(); ++k) {
            if (grp[k] >= n) {
              post_error("tensor_demux: tensorpick index out of range");
              return false;
            }
            oc.info.at(static_cast<unsigned>(k)) = config_.info.at(grp[k]);
          }
          if (p->is_linked()) {
            p->push_event(Event::make_stream_start(name() + "_" + std::to_string(i)));
            p->push_event(Event::make_caps(tensor_src_caps(p, oc)));
            p->push_event(Event::make_segment(Segment()));
          }
        } else if (p->is_linked()) {
          p->push_event(Event::make_caps(ev.caps));
        }
      }
      return true;
    }
    if (ev.type == EventType::STREAM_START || ev.type == EventType::SEGMENT) return true;
    return forward_event_downstream(ev);
  }

  FlowReturn chain(Pad*, BufferPtr buf) override {
    BufferPtr in;
    if (!buffer_from_config(buf, config_, &in)) return FlowReturn::ERROR;
    unsigned n = static_cast<unsigned>(in->n_memory());
    unsigned nout = picks_.empty() ? n : static_cast<unsigned>(picks_.size());
    FlowReturn agg = FlowReturn::NOT_LINKED;
    bool any_ok = false;
    for (unsigned i = 0; i < nout; ++i) {
      Pad* p = get_pad("src_" + std::to_string(i));
      if (!p) {
        p = Element::request_pad(templates_[1], "src_" + std::to_string(i));
      }
      if (!p->is_linked()) continue;
      if (!p->has_current_caps() && config_.is_flexible()) {
        p->push_event(Event::make_stream_start(name() + "_" + std::to_string(i)));
        p->push_event(Event::make_caps(Caps::from_string(tensor_caps_template_flexible()).fixate()));
        p->push_event(Event::make_segment(Segment()));
      }
      auto b = make_buffer();
      b->copy_metadata_from(*in);
      std::vector<unsigned> grp = picks_.empty() ? std::vector<unsigned>{i} : picks_[i];
      for (unsigned k : grp) {
        if (k >= n) return FlowReturn::ERROR;
        b->mems.push_back(in->mems[k]);
      }
      FlowReturn r = p->push(b);
      if (flow_ok(r)) any_ok = true;
      else if (r != FlowReturn::NOT_LINKED) agg = r;
    }
    return any_ok ? FlowReturn::OK : (agg == FlowReturn::NOT_LINKED ? FlowReturn::OK : agg);
  }

  Caps query_caps(Pad* pad, const Caps* filter) override {
    Caps c = pad->template_caps();
    return filter ? c.intersect(*filter) : c;
  }

 private:
  std::string pick_str_;
  std::vector<std::vector<unsigned>> picks_;
  TensorsConfig config_;
};

// ------------------------------------------------------------ tensor_split ----
class TensorSplit : public Element {
 public:
  explicit TensorSplit(const std::string& name) : Element("tensor_split", name) {
    add_template("sink", PadDirection::SINK, PadPresence::ALWAYS, Caps::from_string(tensor_caps_template_static()));
    add_template("src_%u", PadDirection::SRC, PadPresence::SOMETIMES, Caps::from_string(tensor_caps_template_static()));
    prop_string("tensorpick", &pick_str_, "Choose nth tensor among tensors ?", [this] {
      picks_.clear();
      for (auto& x : split(pick_str_, ','))
        if (!strip(x).empty()) picks_.push_back(static_cast<unsigned>(to_uint(x)));
    });
    prop_string("tensorseg", &seg_str_, "Manually Segment Tensor (d1:d2:...,d1:d2:...)", [this] {
      segs_.clear();
      for (auto& s : split_any(seg_str_, ",.")) {
        if (strip(s).empty()) continue;
        Dims d{};
        parse_dimension(s, d);
        segs_.push_back(d);
      }
    });
  }

  bool sink_event(Pad*, Event& ev) override {
    if (ev.type == EventType::CAPS) {
      if (!tensor_config_from_caps(ev.caps, &config_) || config_.info.num_tensors != 1) {
        post_error("tensor_split: expects a single static tensor");
        return false;
      }
      size_t total = 0;
      for (auto& d : segs_) total += element_count(d) * dtype_size(config_.info.at(0).type);
      if (total != config_.info.at(0).size()) {
        post_error("tensor_split: tensorseg does not add up to the input tensor size");
        return false;
      }
      for (unsigned i = 0; i < segs_.size(); ++i) {
        if (!picked(i)) continue;
        Pad* p = out_pad(i);
        TensorsConfig oc;
        oc.rate_n = config_.rate_n;
        oc.rate_d = config_.rate_d;
        oc.info.resize(1);
        oc.info.at(0).type = config_.info.at(0).type;
        oc.info.at(0).dim = segs_[i];
        if (p->is_linked()) {
          p->push_event(Event::make_stream_start(name() + std::to_string(i)));
          p->push_event(Event::make_caps(tensor_src_caps(p, oc)));
          p->push_event(Event::make_segment(Segment()));
        }
      }
      return true;
    }
    if (ev.type == EventType::STREAM_START || ev.type == EventType::SEGMENT) return true;
    return forward_event_downstream(ev);
  }

  FlowReturn chain(Pad*, BufferPtr buf) override {
    BufferPtr in;
    if (!buffer_from_config(buf, config_, &in)) return FlowReturn::ERROR;
    size_t off = 0;
    size_t es = dtype_size(config_.info.at(0).type);
    bool any_ok = false;
    for (unsigned i = 0; i < segs_.size(); ++i) {
      size_t sz = element_count(segs_[i]) * es;
      if (picked(i)) {
        Pad* p = out_pad(i);
        if (p->is_linked()) {
          auto b = make_buffer();
          b->copy_metadata_from(*in);
          b->mems.push_back(Memory::view(in->mems[0], off, sz));  // zero-copy slice (K19)
          if (flow_ok(p->push(b))) any_ok = true;
        }
      }
      off += sz;
    }
    (void)any_ok;
    return FlowReturn::OK;
  }

  Caps query_caps(Pad* pad, const Caps* filter) override {
    Caps c = pad->template_caps();
    return filter ? c.intersect(*filter) : c;
  }

 private:
  bool picked(unsigned i) const {
    if (picks_.empty()) return true;
    return std::find(picks_.begin(), picks_.end(), i) != picks_.end();
  }
  Pad* out_pad(unsigned i) {
    // pads are numbered by output order among picked segments
    unsigned idx = 0;
    if (!picks_.empty()) {
      for (size_t k = 0; k < picks_.size(); ++k)
        if (picks_[k] == i) idx = static_cast<unsigned>(k);
    } else {
      idx = i;
    }
    std::string n = "src_" + std::to_string(idx);
    Pad* p = get_pad(n);
    if (!p) p = Element::request_pad(templates_[1], n);
    return p;
  }
  std::string pick_str_, seg_str_;
  std::vector<unsigned> picks_;
  std::vector<Dims> segs_;
  TensorsConfig config_;
};

// ------------------------------------------------------- tensor_aggregator ----
class TensorAggregator : public Element {
 public:
  explicit TensorAggregator(const std::string& name) : Element("tensor_aggregator", name) {
    add_template("sink", PadDirection::SINK, PadPresence::ALWAYS, Caps::from_string(tensor_caps_template_static()));
    add_template("src", PadDirection::SRC, PadPresence::ALWAYS, Caps::from_string(tensor_caps_template_static()));
    prop_uint("frames-in", &frames_in_, "The number of frames in incoming buffer");
    prop_uint("frames-out", &frames_out_, "The number of frames in outgoing buffer");
    prop_uint("frames-flush", &frames_flush_, "The number of frames to flush (0 to flush all output)");
    prop_uint("frames-dim", &frames_dim_, "The dimension index of frames in tensor");
    prop_bool("concat", &concat_, "Concatenate incoming buffers");
  }

  bool start() override {
    adapters_.clear();
    return true;
  }

  bool sink_event(Pad*, Event& ev) override {
    if (ev.type == EventType::CAPS) {
      if (!tensor_config_from_caps(ev.caps, &in_) || in_.info.num_tensors != 1) {
        post_error("tensor_aggregator: expects a single static tensor");
        return false;
      }
      out_ = in_;
      TensorInfo& t = out_.info.at(0);
      if (frames_dim_ >= static_cast<unsigned>(kRankLimit) || t.dim[frames_dim_] % frames_in_ != 0) {
        post_error("tensor_aggregator: frames-in does not divide the frames dimension");
        return false;
      }
      uint32_t per = t.dim[frames_dim_] / frames_in_;
      t.dim[frames_dim_] = per * frames_out_;
      return src_pad()->push_event(Event::make_caps(tensor_src_caps(src_pad(), out_)));
    }
    if (ev.type == EventType::FLUSH_STOP) adapters_.clear();
    return forward_event_downstream(ev);
  }

  FlowReturn chain(Pad*, BufferPtr buf) override {
    size_t buf_size = buf->total_size();
    if (buf_size == 0) return FlowReturn::ERROR;
    size_t frame_size = buf_size / frames_in_;
    if (frames_in_ == frames_out_) return push(buf, frame_size);
    auto& ad = adapters_[buf->meta.client_id];  // per query-client adapter
    int64_t duration = buf->duration >= 0 ? buf->duration * frames_out_ / frames_in_ : -1;
    for (auto& m : buf->mems) {
      ad.pieces.push_back(Piece{m, 0, buf->pts, buf->dts});
      ad.avail += m->size();
      buf->pts = -1;
    }
    size_t out_size = frame_size * frames_out_;
    FlowReturn ret = FlowReturn::OK;
    while (ad.avail >= out_size && flow_ok(ret)) {
      // timestamp of the first byte (+ distance when frames-in > 1)
      int64_t pts = -1, dts = -1;
      size_t dist = 0;
      for (auto& p : ad.pieces) {
        if (p.pts >= 0 || &p == &ad.pieces.front()) {
          pts = p.pts;
          dts = p.dts;
          dist = p.off;
          break;
        }
      }
      if (frames_in_ > 1 && in_.rate_n > 0 && in_.rate_d > 0 && pts >= 0)
        pts += static_cast<int64_t>(dist) * in_.rate_d * kSecond / (static_cast<int64_t>(in_.rate_n) * frame_size);
      auto out = make_buffer();
      out->pts = pts;
      out->dts = dts;
      out->duration = duration;
      out->meta.client_id = buf->meta.client_id;
      out->mems.push_back(peek_bytes(ad, out_size));
      ret = push(out, frame_size);
      size_t flush = frames_flush_ > 0 ? std::min(frame_size * frames_flush_, ad.avail) : out_size;
      flush_bytes(ad, flush);
    }
    return ret;
  }

 private:
  struct Piece {
    MemoryPtr mem;
    size_t off;
    int64_t pts, dts;
  };
  struct Adapter {
    std::deque<Piece> pieces;
    size_t avail = 0;
  };

  MemoryPtr peek_bytes(Adapter& ad, size_t size) {
    Piece& f = ad.pieces.front();
    if (f.mem->size() - f.off >= size) return Memory::view(f.mem, f.off, size);
    int dev = f.mem->on_device() ? f.mem->device() : -1;
    hipStream_t s = dev >= 0 ? streams_.get(dev) : nullptr;
    MemoryPtr out = alloc_output(size, dev, s);
    size_t done = 0;
    for (auto& p : ad.pieces) {
      if (done >= size) break;
      size_t n = std::min(size - done, p.mem->size() - p.off);
      char* dst = static_cast<char*>(out->data()) + done;
      if (dev >= 0) {
        const char* src = static_cast<const char*>(p.mem->map_device(dev, s)) + p.off;
        hip::check(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, s), "aggregator copy");
        p.mem->record_use(s, dev);
      } else {
        std::memcpy(dst, static_cast<const char*>(p.mem->map_host()) + p.off, n);
      }
      done += n;
    }
    if (dev >= 0) out->mark_ready(s);
    return out;
  }

  void flush_bytes(Adapter& ad, size_t n) {
    while (n > 0 && !ad.pieces.empty()) {
      Piece& f = ad.pieces.front();
      size_t k = std::min(n, f.mem->size() - f.off);
      f.off += k;
      n -= k;
      ad.avail -= k;
      if (f.off == f.mem->size()) ad.pieces.pop_front();
    }
  }

  FlowReturn push(BufferPtr out, size_t frame_size) {
    TensorInfo frame = out_.info.at(0);
    frame.dim[frames_dim_] /= frames_out_;
    if (frame_size != frame.size()) {
      post_error("tensor_aggregator: invalid output frame size");
      return FlowReturn::ERROR;
    }
    bool need_concat = false;
    if (concat_ && frames_out_ > 1)
      for (unsigned i = frames_dim_ + 1; i < static_cast<unsigned>(kRankLimit); ++i)
        if (frame.dim[i] > 1) need_concat = true;
    if (need_concat) {
      // interleave frames along frames-dim (K8): block = dims[0..frames_dim] of one frame
      MemoryPtr src = out->mems.size() == 1 ? out->mems[0] : nullptr;
      if (!src) return FlowReturn::ERROR;
      size_t block = dtype_size(frame.type);
      for (unsigned f = 0; f <= frames_dim_; ++f) block *= frame.dim[f];
      size_t outer = frame_size / block;
      int dev = src->on_device() ? src->device() : -1;
      hipStream_t s = dev >= 0 ? streams_.get(dev) : nullptr;
      MemoryPtr dst = alloc_output(src->size(), dev, s);
      for (unsigned f = 0; f < frames_out_; ++f) {
        // frame f's slabs go to dst at (outer_i * frames_out + f) * block
        if (dev >= 0) {
          const char* sp = static_cast<const char*>(src->map_device(dev, s)) + frame_size * f;
          hip::check(hipMemcpy2DAsync(static_cast<char*>(dst->data()) + block * f, block * frames_out_, sp, block, block,
                                      outer, hipMemcpyDeviceToDevice, s),
                     "aggregator concat");
        } else {
          const char* sp = static_cast<const char*>(src->map_host()) + frame_size * f;
          for (size_t o = 0; o < outer; ++o)
            std::memcpy(static_cast<char*>(dst->data()) + (o * frames_out_ + f) * block, sp + o * block, block);
        }
      }
      if (dev >= 0) {
        src->record_use(s, dev);
        dst->mark_ready(s);
      }
      out->mems[0] = dst;
    }
    return src_pad()->push(out);
  }

  unsigned frames_in_ = 1, frames_out_ = 1, frames_flush_ = 0, frames_dim_ = kRankLimit - 1;
  bool concat_ = true;
  TensorsConfig in_, out_;
  std::map<int64_t, Adapter> adapters_;
  StreamSet streams_;
};

}  // namespace

void register_tensor_stream_elements() {
  register_element("tensor_mux", "Muxer/Tensor", "Creates other/tensors from other/tensor(s) streams (with time sync)",
                   [](const std::string& n) { return std::make_unique<TensorMux>(n); });
  register_element("tensor_merge", "Muxer/Tensor", "Merges (concatenates) single-tensor streams along an axis",
                   [](const std::string& n) { return std::make_unique<TensorMerge>(n); });
  register_element("tensor_demux", "Demuxer/Tensor", "Splits other/tensors into separate streams (tensorpick)",
                   [](const std::string& n) { return std::make_unique<TensorDemux>(n); });
  register_element("tensor_split", "Demuxer/Tensor", "Splits one tensor into several tensors (tensorseg)",
                   [](const std::string& n) { return std::make_unique<TensorSplit>(n); });
  register_element("tensor_aggregator", "Filter/Tensor", "Aggregates frames into a sliding window",
                   [](const std::string& n) { return std::make_unique<TensorAggregator>(n); });
}

}  // namespace nnsx
