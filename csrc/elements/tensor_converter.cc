// tensor_converter: media (video/audio/text/octet/flexible tensors/custom)
// -> other/tensors.  Behaviour follows gst/nnstreamer/elements/
// gsttensor_converter.c (chain :1015-1312, parse_* :1422-1833, timestamps
// :783-841, chunking :946-1013).
//
// MI355X path (nnsx extension, property `device`): frames are uploaded into
// stream-ordered device memory right here -- padded video rows are stripped by
// hipMemcpy2DAsync during the H2D copy (K7), and `frames-per-tensor` batches
// are assembled directly in one device block (K8) -- so everything
// downstream stays HBM-resident.
#include <cstring>
#include <deque>

#include "core/log.h"
#include "elements/elements.h"
#include "elements/tensor_common.h"
#include "kernels/kernels.h"
#include "runtime/pipeline.h"
#include "runtime/plugin_api.h"
#include "runtime/video.h"

namespace nnsx {

namespace {

Caps converter_sink_templ() {
  return Caps::from_string(
      "video/x-raw, format=(string){ RGB, BGR, RGBx, BGRx, xRGB, xBGR, RGBA, BGRA, ARGB, ABGR, GRAY8 }, "
      "width=(int)[ 1, 2147483647 ], height=(int)[ 1, 2147483647 ], framerate=(fraction)[ 0/1, 2147483647/1 ]; "
      "audio/x-raw, format=(string){ S8, U8, S16LE, U16LE, S32LE, U32LE, F32LE, F64LE }, "
      "rate=(int)[ 1, 2147483647 ], channels=(int)[ 1, 2147483647 ], layout=(string)interleaved; "
      "text/x-raw, format=(string)utf8; application/octet-stream; "
      "other/tensors, format=(string)flexible, framerate=(fraction)[ 0/1, 2147483647/1 ]");
}

class TensorConverter : public Element {
 public:
  explicit TensorConverter(const std::string& name) : Element("tensor_converter", name) {
    add_template("sink", PadDirection::SINK, PadPresence::ALWAYS, Caps::Any());
    add_template("src", PadDirection::SRC, PadPresence::ALWAYS,
                 Caps::from_string(tensor_caps_template_static() + "; " + tensor_caps_template_flexible()));
    prop_string("input-dim", &input_dim_, "Input tensor dimension from inner array, up to 8 dimensions (text/octet)", [this] {
      prop_info_.parse_dimensions(input_dim_);
      unsigned n = static_cast<unsigned>(split_any(input_dim_, ",.").size());
      if (prop_info_.num_tensors < n) prop_info_.num_tensors = n;
    });
    prop_string("input-type", &input_type_, "Type of each element of the input tensor (octet)", [this] {
      prop_info_.parse_types(input_type_);
      unsigned n = static_cast<unsigned>(split_any(input_type_, ",.").size());
      if (prop_info_.num_tensors < n) prop_info_.num_tensors = n;
    });
    prop_uint("frames-per-tensor", &frames_per_tensor_, "The number of frames in output tensor");
    prop_bool("set-timestamp", &set_timestamp_, "The flag to set timestamp when received a buffer with invalid timestamp");
    prop_string("mode", &mode_, "Converter mode: custom-code:<registered callback> or custom-script:<python script>", [this] { parse_mode(); });
    prop_readonly("sub-plugins", [] { return join(Registry::get().names(SubpluginKind::CONVERTER), ","); },
                  "Registrable sub-plugins list");
    prop_int("device", &device_, "nnsx: -1 keep tensors on the host, N upload into GPU N's HBM (zero-copy downstream)");
    prop_int("pool-size", &pool_blocks_,
             "nnsx: device tensors come from a pool of this many recycled HBM blocks (0: one allocation per tensor)");
  }

  bool start() override {
    configured_ = false;
    adapter_.clear();
    avail_ = 0;
    old_pts_ = -1;
    need_segment_ = true;
    return true;
  }

  Caps query_caps(Pad* pad, const Caps* filter) override {
    if (pad->direction() == PadDirection::SINK) {
      Caps t = converter_sink_templ();
      if (!mode_.empty() || !Registry::get().names(SubpluginKind::CONVERTER).empty()) t = Caps::Any();
      if (filter) t = t.intersect(*filter);
      return t;
    }
    Caps c = pad->template_caps();
    if (configured_) c = caps_from_config(config_);
    return filter ? c.intersect(*filter) : c;
  }

  bool sink_event(Pad* pad, Event& ev) override {
    (void)pad;
    switch (ev.type) {
      case EventType::CAPS:
        if (!parse_caps(ev.caps)) {
          post_error("not-negotiated: tensor_converter cannot handle " + ev.caps.to_string());
          return false;
        }
        return update_src_caps();
      case EventType::SEGMENT:
        in_segment_ = ev.segment;
        need_segment_ = true;
        return true;  // re-sent in TIME format at the next buffer
      case EventType::EOS: {
        // flush a partial chunk? the reference drops incomplete frames-per-tensor chunks
        return forward_event_downstream(ev);
      }
      case EventType::FLUSH_STOP:
        adapter_.clear();
        avail_ = 0;
        return forward_event_downstream(ev);
      default:
        return forward_event_downstream(ev);
    }
  }

  FlowReturn chain(Pad*, BufferPtr buf) override {
    try {
      return do_chain(std::move(buf));
    } catch (const std::exception& e) {
      post_error(e.what());
      return FlowReturn::ERROR;
    }
  }

 private:
  void parse_mode() {
    custom_fn_ = nullptr;
    external_.reset();
    if (mode_.empty()) return;
    auto parts = split(mode_, ':', 2);
    if (parts.size() != 2) throw Error("invalid mode " + mode_);
    if (parts[0] == "custom-code") {
      auto fn = Registry::get().find_as<ConverterCustomFn>(SubpluginKind::CUSTOM_CONVERTER, parts[1], false);
      if (!fn) throw Error("custom-code converter '" + parts[1] + "' is not registered");
      custom_fn_ = *fn;
    } else if (parts[0] == "custom-script") {
      external_ = make_script_converter(parts[1]);
      if (!external_) throw Error("cannot load converter script " + parts[1]);
    } else {
      throw Error("unknown converter mode " + parts[0]);
    }
  }

  bool parse_caps(const Caps& caps) {
    if (caps.size() == 0) return false;
    const Structure& st = caps.at(0);
    media_ = structure_media_type(st);
    TensorsConfig cfg;
    remove_padding_ = false;
    if (custom_fn_ || external_) {
      media_ = MediaType::ANY;
    }
    switch (media_) {
      case MediaType::VIDEO: {
        if (!vinfo_.from_structure(st) || !vinfo_.packed() || vinfo_.format == "YUY2" || vinfo_.format == "GRAY16_LE") {
          NNSX_LOGE(name(), "unsupported video caps ", caps.to_string());
          return false;
        }
        cfg.info.resize(1);
        auto& t = cfg.info.at(0);
        t.type = DType::UINT8;
        t.dim = make_dims({static_cast<uint32_t>(vinfo_.channels), static_cast<uint32_t>(vinfo_.width),
                           static_cast<uint32_t>(vinfo_.height), frames_per_tensor_});
        cfg.rate_n = vinfo_.fps_n;
        cfg.rate_d = vinfo_.fps_d;
        size_t row = static_cast<size_t>(vinfo_.width) * vinfo_.channels;
        remove_padding_ = (row % 4) != 0;
        frame_size_ = row * vinfo_.height;  // tensor bytes per frame (padding stripped)
        in_frame_size_ = vinfo_.size;
        break;
      }
      case MediaType::AUDIO: {
        AudioInfo ai;
        if (!ai.from_structure(st)) return false;
        static const std::map<std::string, DType> fmt = {
            {"S8", DType::INT8},     {"U8", DType::UINT8},     {"S16LE", DType::INT16},   {"U16LE", DType::UINT16},
            {"S32LE", DType::INT32}, {"U32LE", DType::UINT32}, {"F32LE", DType::FLOAT32}, {"F64LE", DType::FLOAT64}};
        auto it = fmt.find(ai.format);
        if (it == fmt.end()) return false;
        cfg.info.resize(1);
        cfg.info.at(0).type = it->second;
        cfg.info.at(0).dim = make_dims({static_cast<uint32_t>(ai.channels), frames_per_tensor_});
        cfg.rate_n = ai.rate;
        cfg.rate_d = 1;
        frame_size_ = in_frame_size_ = ai.bpf;
        break;
      }
      case MediaType::TEXT: {
        uint32_t text_size = prop_info_.num_tensors > 0 ? prop_info_.at(0).dim[0] : 0;
        if (text_size == 0) {
          NNSX_LOGE(name(), "tensor_converter: set input-dim for text streams (e.g. input-dim=30)");
          return false;
        }
        std::string f;
        if (st.get_string("format", &f) && lower(f) != "utf8") return false;
        cfg.info.resize(1);
        cfg.info.at(0).type = DType::UINT8;
        cfg.info.at(0).dim = make_dims({text_size, frames_per_tensor_});
        if (!st.get_fraction("framerate", &cfg.rate_n, &cfg.rate_d)) {
          cfg.rate_n = 0;
          cfg.rate_d = 1;
        }
        frame_size_ = in_frame_size_ = text_size;
        break;
      }
      case MediaType::OCTET: {
        Caps peer = src_pad()->peer_query_caps(nullptr);
        TensorsConfig pc;
        bool peer_flex = peer.size() > 0 && config_from_structure(peer.at(0), &pc) && pc.is_flexible() &&
                         peer.at(0).get("format") && peer.at(0).get("format")->is_fixed();
        bool configured = prop_info_.num_tensors > 0 && prop_info_.valid();
        if (!configured && peer.size() > 0 && config_from_structure(peer.at(0), &pc) && pc.info.valid() &&
            peer.is_fixed()) {
          prop_info_ = pc.info;
          configured = true;
        }
        if (peer_flex || !configured) {
          cfg.info.format = Format::FLEXIBLE;
          cfg.info.resize(1);
          cfg.info.at(0).type = DType::UINT8;
          cfg.info.at(0).dim = make_dims({1});
          frame_size_ = in_frame_size_ = 0;
        } else {
          cfg.info = prop_info_;
          if (frames_per_tensor_ > 1 && cfg.info.num_tensors == 1) {
            int r = cfg.info.at(0).rank();
            if (r < kRankLimit) cfg.info.at(0).dim[r] = frames_per_tensor_;
          }
          frame_size_ = in_frame_size_ = prop_info_.size();
        }
        if (!st.get_fraction("framerate", &cfg.rate_n, &cfg.rate_d)) {
          cfg.rate_n = 0;
          cfg.rate_d = 1;
        }
        break;
      }
      case MediaType::TENSOR: {
        // flexible -> static: config comes from the first buffer's headers
        TensorsConfig in;
        config_from_structure(st, &in);
        cfg = in;
        cfg.info.format = Format::STATIC;
        cfg.info.num_tensors = 0;
        if (prop_info_.num_tensors > 0) cfg.info = prop_info_;
        frame_size_ = in_frame_size_ = 0;
        break;
      }
      default: {
        if (!custom_fn_ && !external_) {
          external_ = find_converter_for_caps(caps);
          if (!external_) {
            NNSX_LOGE(name(), "no converter sub-plugin for ", caps.to_string());
            return false;
          }
        }
        media_ = MediaType::ANY;
        if (external_ && external_->get_out_config(caps, &cfg)) {
          // known in advance
        } else {
          cfg.info.num_tensors = 0;
        }
        int n = 0, d = 1;
        if (st.get_fraction("framerate", &n, &d)) {
          cfg.rate_n = n;
          cfg.rate_d = d;
        } else {
          cfg.rate_n = 0;
          cfg.rate_d = 1;
        }
        break;
      }
    }
    config_ = cfg;
    configured_ = true;
    return true;
  }

  bool update_src_caps() {
    if (config_.is_static() && config_.info.num_tensors == 0) return true;  // decided at first buffer
    Caps c = tensor_src_caps(src_pad(), config_, device_ >= 0);
    out_flexible_ = c.size() > 0 && c.at(0).get_string_or("format", "static") == "flexible";
    return src_pad()->push_event(Event::make_caps(c));
  }

  void push_segment() {
    if (!need_segment_) return;
    Segment seg;
    bool have_fr = config_.rate_n > 0 && config_.rate_d > 0;
    if (have_fr && in_segment_.start > 0 && frame_size_ > 0 && media_ == MediaType::AUDIO) {
      int64_t start = in_segment_.start * config_.rate_d * kSecond / (static_cast<int64_t>(frame_size_) * config_.rate_n);
      seg.start = seg.time = start;
    } else {
      seg = in_segment_;
    }
    out_segment_ = seg;
    need_segment_ = false;
    src_pad()->push_event(Event::make_segment(seg));
  }

  void set_timestamp(Buffer& b, unsigned frames_in) {
    if (set_timestamp_) {
      bool have_fr = config_.rate_n > 0 && config_.rate_d > 0;
      if (b.duration < 0 && have_fr)
        b.duration = static_cast<int64_t>(frames_in) * config_.rate_d * kSecond / config_.rate_n;
      if (b.pts < 0) {
        int64_t pts = out_segment_.start;
        if (have_fr) {
          if (old_pts_ >= 0) pts = old_pts_ + (b.duration > 0 ? b.duration : 0);
        } else {
          pts = running_time();
          if (pts < 0) pts = 0;
        }
        b.pts = pts;
      }
    }
    old_pts_ = b.pts;
  }

  // strip row padding (K7) and optionally upload (device path: one 2D H2D copy)
  MemoryPtr video_frame(const MemoryPtr& m, int dev, hipStream_t s) {
    size_t row = static_cast<size_t>(vinfo_.width) * vinfo_.channels;
    if (!remove_padding_) {
      if (dev >= 0 && frames_per_tensor_ == 1) {
        auto out = dev_alloc(frame_size_, dev, s);
        if (m->on_device()) {
          m->wait_ready(s);
          hip::check(hipMemcpyAsync(out->data(), m->data(), frame_size_, hipMemcpyDeviceToDevice, s), "D2D");
        } else {
          hip::check(hipMemcpyAsync(out->data(), m->data(), frame_size_, hipMemcpyHostToDevice, s), "H2D frame");
        }
        m->record_use(s, dev);
        out->mark_ready(s);
        return out;
      }
      return m->size() == frame_size_ ? m : Memory::view(m, 0, frame_size_);
    }
    size_t stride = vinfo_.stride[0];
    if (dev >= 0 && m->place() != MemPlace::HOST && stride <= kernels::kGatherMaxStride && stride % 4 == 0 &&
        m->size() >= stride * (vinfo_.height - 1) + row) {
      // the padded frame goes to HBM as it is (one DMA, padded_dma) and one
      // unpad_rows launch strips the padding -- batch 1 too: a 2D copy (one
      // DMA descriptor per row) took 3.6 ms for a 513 x 513 RGB frame
      // (scripts/b1_pipeline_probe.py: DeepLab batch-1 p50 4.2 ms, of which the
      // converter 3.6)
      padded_frame_ = true;
      return m;
    }
    if (dev >= 0 && frames_per_tensor_ == 1 && !m->on_device()) {
      auto out = dev_alloc(frame_size_, dev, s);
      hip::check(hipMemcpy2DAsync(out->data(), row, m->data(), stride, row, vinfo_.height, hipMemcpyHostToDevice, s),
                 "H2D 2D frame");
      m->record_use(s, dev);
      out->mark_ready(s);
      return out;
    }
    const uint8_t* src = static_cast<const uint8_t*>(m->map_host());
    auto out = Memory::alloc_host(frame_size_);
    uint8_t* dst = static_cast<uint8_t*>(out->data());
    for (int y = 0; y < vinfo_.height; ++y) std::memcpy(dst + y * row, src + y * stride, row);
    return out;
  }

  struct Piece {
    MemoryPtr mem;
    size_t off;
    int64_t pts, dts;
    size_t row = 0, stride = 0, rows = 0;  // padded video frame (packed size row * rows)
    bool padded() const { return row != 0; }
    size_t size() const { return padded() ? row * rows : mem->size(); }
  };

  // a padded piece that cannot go through the gather kernel whole: pack it on the host
  void unpad(Piece& p) {
    if (!p.padded()) return;
    const uint8_t* src = static_cast<const uint8_t*>(p.mem->map_host());
    auto out = Memory::alloc_host(p.row * p.rows);
    for (size_t y = 0; y < p.rows; ++y)
      std::memcpy(static_cast<uint8_t*>(out->data()) + y * p.row, src + y * p.stride, p.row);
    p.mem = out;
    p.row = p.stride = p.rows = 0;
  }

  // take `size` bytes from the adapter: zero-copy view when inside one piece,
  // otherwise gathered into one block (on the device when uploading)
  MemoryPtr adapter_take(size_t size, int dev, hipStream_t s, int64_t* pts, int64_t* dts, size_t* pts_dist) {
    Piece& f = adapter_.front();
    *pts = f.pts;
    *dts = f.dts;
    *pts_dist = f.off;
    MemoryPtr out;
    if (!f.padded() && f.size() - f.off >= size && dev < 0) {
      out = Memory::view(f.mem, f.off, size);
      f.off += size;
      if (f.off == f.size()) adapter_.pop_front();
      avail_ -= size;
      return out;
    }
    out = dev >= 0 ? dev_alloc(size, dev, s) : Memory::alloc_host(size);
    size_t done = 0;
    std::vector<std::pair<const char*, size_t>> runs;
    if (dev >= 0 && dma_runs(size, &runs)) {
      // adjacent frames (a capture ring): a few DMA copies, no CU time spent on the upload
      for (auto& r : runs) {
        hip::check(hipMemcpyAsync(static_cast<char*>(out->data()) + done, r.first, r.second, hipMemcpyDefault, s),
                   "ring upload");
        done += r.second;
      }
      // one use record per source allocation: the frames of a ring are views
      // of one block, whose use event is re-recorded by every record_use on the
      // same stream (Memory::record_use_self) -- 512 per batch cost ~2.5-4 ms of
      // converter-thread time in hipEventRecord, the sustained headline's
      // bottleneck on slower hosts (profiles/r6_host_bound_converter.txt)
      const Memory* last_root = nullptr;
      for (size_t left = size; left > 0;) {
        Piece& p = adapter_.front();
        const size_t n = std::min(left, p.size() - p.off);
        if (p.mem->root() != last_root) {
          p.mem->record_use(s, dev);
          last_root = p.mem->root();
        }
        p.off += n;
        left -= n;
        if (p.off == p.size()) adapter_.pop_front();
      }
    }
    if (dev >= 0 && done < size && padded_dma(size, dev, s, out)) done = size;
    if (dev >= 0 && done < size && gather_eligible(size)) {
      // one gather launch per <=128 pieces instead of one hipMemcpyAsync per frame
      kernels::GatherArgs g;
      auto flush = [&]() {
        kernels::gather_copy(g, out->data(), s);
        g.n = 0;
      };
      while (done < size) {
        Piece& p = adapter_.front();
        size_t n = std::min(size - done, p.size() - p.off);
        if (p.mem->on_device()) p.mem->wait_ready(s);
        if (p.padded()) {  // whole frame (gather_eligible checked)
          g.row = static_cast<uint32_t>(p.row);
          g.stride = static_cast<uint32_t>(p.stride);
          g.seg[g.n++] = kernels::GatherSeg{p.mem->data(), done, n | kernels::kGatherPadded};
        } else {
          g.seg[g.n++] = kernels::GatherSeg{static_cast<const char*>(p.mem->data()) + p.off, done, n};
        }
        p.mem->record_use(s, dev);
        if (g.n == kernels::kGatherMax) flush();
        done += n;
        p.off += n;
        if (p.off == p.size()) adapter_.pop_front();
      }
      flush();
    }
    while (done < size) {
      Piece& p = adapter_.front();
      unpad(p);
      size_t n = std::min(size - done, p.mem->size() - p.off);
      char* dst = static_cast<char*>(out->data()) + done;
      const char* srcp = static_cast<const char*>(p.mem->data()) + p.off;
      if (dev >= 0) {
        if (p.mem->on_device()) p.mem->wait_ready(s);
        hip::check(hipMemcpyAsync(dst, srcp, n, p.mem->on_device() ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s),
                   "adapter copy");
        p.mem->record_use(s, dev);
      } else {
        std::memcpy(dst, static_cast<const char*>(p.mem->map_host()) + p.off, n);
      }
      done += n;
      p.off += n;
      if (p.off == p.mem->size()) adapter_.pop_front();
    }
    if (dev >= 0) out->mark_ready(s);
    avail_ -= size;
    return out;
  }

  // Padded video frames (row stride > W*C, e.g. 513x513 RGB: 1539-byte rows 1540
  // apart; reference: gsttensor_converter.c:1062-1107) in pinned host memory:
  // the padded bytes go to HBM on the copy engine as they are -- one DMA for a
  // ring of equally spaced frames, else one per frame -- and one unpad_rows
  // launch packs the rows device-side.  (The bus-reading gather kernel moved
  // them at ~5 GB/s with 1-byte stores on a few workgroups:
  // profiles/r3_config_trace_deeplab_b8.txt.)  Every piece must be a whole
  // padded pinned frame of one geometry.
  bool padded_dma(size_t size, int dev, hipStream_t s, const MemoryPtr& out) {
    std::vector<Piece*> ps;
    size_t seen = 0;
    for (Piece& p : adapter_) {
      if (!p.padded() || p.off != 0 || p.mem->place() != MemPlace::PINNED) return false;
      if (!ps.empty() && (p.row != ps[0]->row || p.stride != ps[0]->stride || p.rows != ps[0]->rows)) return false;
      ps.push_back(&p);
      seen += p.size();
      if (seen >= size) break;
    }
    if (ps.empty() || seen != size) return false;
    const size_t row = ps[0]->row, stride = ps[0]->stride, rows = ps[0]->rows;
    const size_t sf = stride * (rows - 1) + row;  // padded bytes of one frame (the last row's padding may be absent)
    // Frames of a capture ring sit `spacing` apart: the staging copy keeps that
    // spacing and every run of adjacent frames goes up as ONE DMA -- a batch
    // that wraps around the ring is two.  A lone frame is one DMA of its own.
    // (Per-frame DMAs of 790 KB ran at ~23 GB/s with the queue gaps between
    // them, one 25 MB ring DMA at the 50 GB/s link rate:
    // profiles/r5_fan_ingest_1gpu.txt.)
    auto at = [&](size_t i) { return static_cast<const char*>(ps[i]->mem->data()); };
    size_t spacing = 0;
    for (size_t i = 1; i < ps.size() && !spacing; ++i)
      if (at(i) > at(i - 1) && static_cast<size_t>(at(i) - at(i - 1)) >= sf &&
          static_cast<size_t>(at(i) - at(i - 1)) <= 2 * sf)
        spacing = static_cast<size_t>(at(i) - at(i - 1));
    if (!spacing) spacing = (sf + 255) / 256 * 256;
    auto stg = stage_alloc(spacing * (ps.size() - 1) + sf, dev, s);
    char* sp = static_cast<char*>(stg->data());
    // (splitting the upload over 2-4 copy streams did not help: profiles/r4_upload_bench.txt)
    // (a run never spans two allocations: frames of separate pinned blocks can
    // be adjacent in virtual memory, and a copy across them fails HIP's bounds
    // check on the source allocation)
    for (size_t i = 0; i < ps.size();) {
      size_t j = i + 1;
      while (j < ps.size() && at(j) == at(i) + (j - i) * spacing &&
             ps[j]->mem->allocation() == ps[i]->mem->allocation())
        ++j;
      hip::check(hipMemcpyAsync(sp + i * spacing, at(i), spacing * (j - i - 1) + sf, hipMemcpyHostToDevice, s),
                 "padded DMA");
      i = j;
    }
    kernels::unpad_rows(sp, out->data(), static_cast<uint32_t>(ps.size()), static_cast<uint32_t>(row),
                        static_cast<uint32_t>(stride), static_cast<uint32_t>(rows), spacing, s);
    stg->record_use(s, dev);
    const Memory* last_root = nullptr;  // (one use record per source allocation, as above)
    for (size_t i = 0; i < ps.size(); ++i) {
      if (adapter_.front().mem->root() != last_root) {
        adapter_.front().mem->record_use(s, dev);
        last_root = adapter_.front().mem->root();
      }
      adapter_.pop_front();
    }
    return true;
  }

  // the next `size` bytes as at most kMaxRuns address-contiguous runs of unpadded
  // pinned-host pieces
  bool dma_runs(size_t size, std::vector<std::pair<const char*, size_t>>* runs) const {
    constexpr size_t kMaxRuns = 4;
    size_t seen = 0;
    for (const Piece& p : adapter_) {
      // pinned host pieces only (device pieces keep the kernel path, which waits on them)
      if (p.padded() || p.mem->place() != MemPlace::PINNED) return runs->clear(), false;
      const char* d = static_cast<const char*>(p.mem->data()) + p.off;
      const size_t n = std::min(size - seen, p.size() - p.off);
      if (!runs->empty() && runs->back().first + runs->back().second == d)
        runs->back().second += n;
      else if (runs->size() == kMaxRuns)
        return runs->clear(), false;
      else
        runs->emplace_back(d, n);
      seen += n;
      if (seen >= size) break;
    }
    if (seen < size) return runs->clear(), false;
    return true;
  }

  // every piece that feeds the next `size` bytes is device-readable in place (pinned host or HBM)
  bool gather_eligible(size_t size) const {
    size_t seen = 0;
    for (const Piece& p : adapter_) {
      if (p.mem->place() == MemPlace::HOST) return false;
      // a padded frame goes through the kernel whole
      if (p.padded() && (p.off != 0 || seen + p.size() > size)) return false;
      seen += p.size() - p.off;
      if (seen >= size) return true;
    }
    return false;
  }

  FlowReturn push_out(BufferPtr b) {
    // octet: split one memory into N static tensors (zero-copy views)
    if (media_ == MediaType::OCTET && !config_.is_flexible() && config_.info.num_tensors > 1 && b->n_memory() == 1) {
      auto nb = make_buffer();
      nb->copy_metadata_from(*b);
      size_t off = 0;
      for (unsigned i = 0; i < config_.info.num_tensors; ++i) {
        size_t sz = config_.info.size(static_cast<int>(i));
        nb->mems.push_back(Memory::view(b->mems[0], off, sz));
        off += sz;
      }
      b = nb;
    }
    if (out_flexible_ && !skip_header_) {
      auto nb = make_buffer();
      nb->copy_metadata_from(*b);
      for (size_t i = 0; i < b->n_memory(); ++i) {
        TensorInfo ti = config_.info.at(static_cast<unsigned>(i));
        if (config_.is_flexible() && media_ == MediaType::OCTET) {
          ti.type = DType::UINT8;
          ti.dim = make_dims({static_cast<uint32_t>(b->mems[i]->size())});
        }
        MediaType mt = (media_ == MediaType::VIDEO || media_ == MediaType::AUDIO || media_ == MediaType::TEXT ||
                        media_ == MediaType::OCTET)
                           ? media_
                           : MediaType::TENSOR;
        nb->mems.push_back(make_flexible(b->mems[i], MetaInfo::from_info(ti, Format::FLEXIBLE, mt)));
      }
      b = nb;
    }
    return src_pad()->push(std::move(b));
  }

  FlowReturn do_chain(BufferPtr buf) {
    if (!configured_) {
      post_error("tensor_converter: buffer before caps");
      return FlowReturn::NOT_NEGOTIATED;
    }
    size_t buf_size = buf->total_size();
    if (buf_size == 0 && media_ != MediaType::ANY) return FlowReturn::OK;
    int dev = device_ >= 0 && hip::available() ? device_ : -1;
    hipStream_t s = dev >= 0 ? streams_.get(dev) : nullptr;
    unsigned frames_out = frames_per_tensor_;
    unsigned frames_in = 1;
    size_t frame_size = frame_size_;
    BufferPtr in = buf;
    skip_header_ = false;

    switch (media_) {
      case MediaType::VIDEO: {
        if (buf->n_memory() != 1) {
          auto m = Memory::alloc_host(buf_size);
          size_t off = 0;
          for (auto& mm : buf->mems) {
            std::memcpy(static_cast<char*>(m->data()) + off, mm->map_host(), mm->size());
            off += mm->size();
          }
          buf = make_buffer();
          buf->copy_metadata_from(*in);
          buf->mems.push_back(m);
        }
        if (buf_size < in_frame_size_) {
          post_error(strfmt("video buffer too small: ", buf_size, " < ", in_frame_size_));
          return FlowReturn::ERROR;
        }
        auto nb = make_buffer();
        nb->copy_metadata_from(*buf);
        nb->mems.push_back(video_frame(buf->mems[0], dev, s));
        in = nb;
        break;
      }
      case MediaType::AUDIO:
        frames_in = static_cast<unsigned>(buf_size / frame_size_);
        break;
      case MediaType::TEXT:
        if (buf_size != frame_size_) {
          auto m = Memory::alloc_host(frame_size_);
          std::memset(m->data(), 0, frame_size_);
          size_t off = 0;
          for (auto& mm : buf->mems) {
            size_t n = std::min(mm->size(), frame_size_ - off);
            std::memcpy(static_cast<char*>(m->data()) + off, mm->map_host(), n);
            off += n;
            if (off >= frame_size_) break;
          }
          in = make_buffer();
          in->copy_metadata_from(*buf);
          in->mems.push_back(m);
        }
        break;
      case MediaType::OCTET:
        if (config_.is_flexible()) {
          frame_size = buf_size;
        } else {
          if (frame_size_ == 0 || buf_size % frame_size_ != 0) {
            post_error(strfmt("octet stream size ", buf_size, " is not a multiple of the tensor size ", frame_size_));
            return FlowReturn::ERROR;
          }
          frames_in = static_cast<unsigned>(buf_size / frame_size_);
        }
        break;
      case MediaType::TENSOR: {
        // flexible -> static: strip headers, check against configured info
        TensorsConfig tmp;
        tmp.rate_n = config_.rate_n;
        tmp.rate_d = config_.rate_d;
        tmp.info.format = Format::FLEXIBLE;
        BufferPtr fb;
        if (!buffer_from_config(buf, tmp, &fb)) {
          post_error("invalid flexible tensor buffer");
          return FlowReturn::ERROR;
        }
        auto nb = make_buffer();
        nb->copy_metadata_from(*buf);
        tmp.info.format = Format::STATIC;
        tmp.info.resize(static_cast<unsigned>(fb->n_memory()));
        for (size_t i = 0; i < fb->n_memory(); ++i) {
          MetaInfo meta;
          MemoryPtr payload;
          if (!parse_flexible(fb->mems[i], &meta, &payload) || !meta.to_info(&tmp.info.at(static_cast<unsigned>(i)))) {
            post_error("invalid flexible header");
            return FlowReturn::ERROR;
          }
          if (payload->size() != tmp.info.at(static_cast<unsigned>(i)).size()) {
            post_error(strfmt("flexible->static: data size ", payload->size(), " != expected ",
                              tmp.info.at(static_cast<unsigned>(i)).size()));
            return FlowReturn::ERROR;
          }
          if (dev >= 0 && !payload->on_device()) {
            auto d = Memory::alloc_device(payload->size(), dev, s);
            hip::check(hipMemcpyAsync(d->data(), payload->data(), payload->size(), hipMemcpyHostToDevice, s), "H2D");
            payload->record_use(s, dev);
            d->mark_ready(s);
            payload = d;
          }
          nb->mems.push_back(payload);
        }
        if (!(tmp.info == config_.info)) {
          if (prop_info_.num_tensors > 0 && prop_info_.valid()) {
            post_error("incoming flexible buffer does not match the given input-dim/input-type");
            return FlowReturn::ERROR;
          }
          config_ = tmp;
          update_src_caps();
        }
        push_segment();
        set_timestamp(*nb, 1);
        return push_out(nb);
      }
      case MediaType::ANY: {
        TensorsConfig nc = config_;
        BufferPtr out;
        if (custom_fn_)
          out = custom_fn_(buf, &nc);
        else if (external_)
          out = external_->convert(buf, &nc);
        if (!out) {
          post_error("converter returned no buffer");
          return FlowReturn::ERROR;
        }
        out->copy_metadata_from(*buf);
        skip_header_ = nc.is_flexible();
        if (!(nc == config_) || !src_pad()->has_current_caps()) {
          config_ = nc;
          update_src_caps();
        }
        if (dev >= 0) {
          for (auto& m : out->mems) {
            if (m->on_device()) continue;
            auto d = Memory::alloc_device(m->size(), dev, s);
            hip::check(hipMemcpyAsync(d->data(), m->data(), m->size(), hipMemcpyHostToDevice, s), "H2D");
            m->record_use(s, dev);
            d->mark_ready(s);
            m = d;
          }
        }
        push_segment();
        set_timestamp(*out, 1);
        return push_out(out);
      }
      default:
        post_error("tensor_converter: unknown media type");
        return FlowReturn::ERROR;
    }

    push_segment();
    set_timestamp(*in, frames_in);

    if (frames_in == frames_out && !padded_frame_) {  // (a padded frame is unpacked through the adapter)
      if (dev >= 0) {
        auto nb = make_buffer();
        nb->copy_metadata_from(*in);
        for (auto& m : in->mems) {
          if (m->on_device()) {
            nb->mems.push_back(m);
            continue;
          }
          auto d = Memory::alloc_device(m->size(), dev, s);
          hip::check(hipMemcpyAsync(d->data(), m->data(), m->size(), hipMemcpyHostToDevice, s), "H2D");
          m->record_use(s, dev);
          d->mark_ready(s);
          nb->mems.push_back(d);
        }
        in = nb;
      }
      return push_out(in);
    }

    // chunking through the adapter (frames-per-tensor)
    int64_t duration = in->duration;
    if (duration >= 0) duration = duration * frames_out / std::max(1u, frames_in);
    for (auto& m : in->mems) {
      Piece pc{m, 0, in->pts, in->dts};
      if (padded_frame_) {
        pc.row = static_cast<size_t>(vinfo_.width) * vinfo_.channels;
        pc.stride = vinfo_.stride[0];
        pc.rows = static_cast<size_t>(vinfo_.height);
        padded_frame_ = false;
      }
      avail_ += pc.size();
      adapter_.push_back(pc);
      // only the first memory carries the timestamp
      in->pts = -1;
      in->dts = -1;
    }
    size_t out_size = static_cast<size_t>(frames_out) * frame_size;
    FlowReturn ret = FlowReturn::OK;
    bool have_fr = config_.rate_n > 0 && config_.rate_d > 0;
    while (avail_ >= out_size && flow_ok(ret)) {
      int64_t pts, dts;
      size_t dist;
      auto m = adapter_take(out_size, dev, s, &pts, &dts, &dist);
      if (frames_in > 1 && have_fr && frame_size > 0) {
        if (pts >= 0) pts += static_cast<int64_t>(dist) * config_.rate_d * kSecond / (config_.rate_n * static_cast<int64_t>(frame_size));
        if (dts >= 0) dts += static_cast<int64_t>(dist) * config_.rate_d * kSecond / (config_.rate_n * static_cast<int64_t>(frame_size));
      }
      auto ob = make_buffer();
      ob->pts = pts;
      ob->dts = dts;
      ob->duration = duration;
      ob->mems.push_back(m);
      ret = push_out(ob);
    }
    return ret;
  }

  std::string input_dim_, input_type_, mode_;
  TensorsInfo prop_info_;
  unsigned frames_per_tensor_ = 1;
  bool set_timestamp_ = true;
  int device_ = -1;
  int pool_blocks_ = 8;
  std::shared_ptr<DeviceBufferPool> pool_;
  // device tensors of the steady size come from the recycled block pool
  MemoryPtr dev_alloc(size_t size, int dev, hipStream_t s) {
    if (pool_blocks_ <= 0) return Memory::alloc_device(size, dev, s);
    if (!pool_ || pool_->device() != dev || pool_->block_size() != size) {
      pool_ = DeviceBufferPool::create(dev, size, static_cast<size_t>(pool_blocks_));
      // every block up front: a consumer keying per-address state (in-place
      // hipGraph instances) can prepare all of it at the first frame
      pool_->preallocate(s);
    }
    return pool_->acquire(s);
  }
  // the padded upload's staging blocks: recycled too (a hipFreeAsync per batch
  // held the converter thread 90-210 us, a third of a batch-8 camera's budget:
  // profiles/r5_fan_ingest_1gpu.txt)
  std::shared_ptr<DeviceBufferPool> stage_pool_;
  MemoryPtr stage_alloc(size_t size, int dev, hipStream_t s) {
    if (pool_blocks_ <= 0) return Memory::alloc_device(size, dev, s);
    if (!stage_pool_ || stage_pool_->device() != dev || stage_pool_->block_size() != size)
      stage_pool_ = DeviceBufferPool::create(dev, size, static_cast<size_t>(pool_blocks_));
    return stage_pool_->acquire(s);
  }
  bool configured_ = false;
  TensorsConfig config_;
  MediaType media_ = MediaType::INVALID;
  VideoInfo vinfo_;
  bool remove_padding_ = false;
  bool padded_frame_ = false;  // video_frame() handed back a padded frame for the gather kernel
  size_t frame_size_ = 0, in_frame_size_ = 0;
  bool out_flexible_ = false, skip_header_ = false;
  int64_t old_pts_ = -1;
  bool need_segment_ = true;
  Segment in_segment_, out_segment_;
  std::deque<Piece> adapter_;
  size_t avail_ = 0;
  ConverterCustomFn custom_fn_;
  std::shared_ptr<ConverterSubplugin> external_;
  StreamSet streams_;
};

}  // namespace

void register_tensor_converter() {
  register_element("tensor_converter", "Converter/Tensor", "Converts audio/video/text/octet streams to tensors",
                   [](const std::string& n) { return std::make_unique<TensorConverter>(n); });
}

}  // namespace nnsx
