// tensor_decoder mode=bounding_boxes: detection heads -> RGBA overlay frames.
//
// Reference: ext/nnstreamer/tensor_decoder/tensordec-boundingbox.c -- modes
// mobilenet-ssd (+tflite-ssd alias), mobilenet-ssd-postprocess (+tf-ssd),
// ov-person-detection, ov-face-detection, yolov5, mp-palm-detection; options
// option1 mode, option2 labels, option3 per-mode parameters (:26-83,
// :700-780), option4 output WIDTH:HEIGHT, option5 model input WIDTH:HEIGHT;
// first-passing-class SSD decode (:1145-1185), greedy NMS with the +1 integer
// IoU convention (:1206-1262), box + label drawing (:1466-1536).
//
// MI355X path (HBM-resident float32 heads of mobilenet-ssd / yolov5): candidate
// extraction, sort, bitmask NMS and rasterisation run as kernels
// (kernels/detect.hip) on the element's stream; a leading batch dimension
// ([4:1:N:B] / [C:N:B]) is decoded in one launch and emitted as B frames.
// The host path implements the same algorithm for every mode and type.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>

#include "core/cpu_ops.h"
#include "core/log.h"
#include "decoders/decoders.h"
#include "decoders/font.h"
#include "kernels/detect.h"
#include "runtime/hip_util.h"

namespace nnsx {

namespace {

enum BBMode { SSD = 0, SSD_PP, OV_PERSON, OV_FACE, OLD_SSD, OLD_SSD_PP, YOLOV5, MP_PALM, UNKNOWN };
const char* kModeNames[] = {"mobilenet-ssd", "mobilenet-ssd-postprocess", "ov-person-detection", "ov-face-detection",
                            "tflite-ssd",    "tf-ssd",                    "yolov5",              "mp-palm-detection"};

constexpr int kBoxSize = 4;
constexpr unsigned kSsdMax = 2034;
constexpr unsigned kSsdPpMax = 100;
constexpr unsigned kOvMax = 200;
constexpr float kOvConf = 0.8f;
constexpr float kYoloConf = 0.25f, kYoloIou = 0.45f;
constexpr unsigned kPalmMax = 2016;
constexpr int kNmsCap = 4096;  // device NMS capacity per frame (top-scoring candidates)

const uint8_t kFont[95][13] = NNSX_FONT8X13_DATA;

struct Det {
  bool valid = false;
  int cls = 0, x = 0, y = 0, w = 0, h = 0;
  float prob = 0;
};

float logit(float x) {
  if (x <= 0.f) return -INFINITY;
  if (x >= 1.f) return INFINITY;
  return static_cast<float>(std::log(x / (1.0 - x)));
}

float iou(const Det& a, const Det& b) {
  int x1 = std::max(a.x, b.x), y1 = std::max(a.y, b.y);
  int x2 = std::min(a.x + a.w, b.x + b.w), y2 = std::min(a.y + a.h, b.y + b.h);
  int w = std::max(0, x2 - x1 + 1), h = std::max(0, y2 - y1 + 1);
  float inter = static_cast<float>(w * h);
  float aa = static_cast<float>(a.w * a.h), ab = static_cast<float>(b.w * b.h);
  float o = inter / (aa + ab - inter);
  return o >= 0 ? o : 0;
}

void nms(std::vector<Det>* r, float thr) {
  std::stable_sort(r->begin(), r->end(), [](const Det& a, const Det& b) { return a.prob > b.prob; });
  for (size_t i = 0; i < r->size(); ++i) {
    if (!(*r)[i].valid) continue;
    for (size_t j = i + 1; j < r->size(); ++j)
      if ((*r)[j].valid && iou((*r)[i], (*r)[j]) > thr) (*r)[j].valid = false;
  }
  r->erase(std::remove_if(r->begin(), r->end(), [](const Det& d) { return !d.valid; }), r->end());
}

struct Anchor {
  float xc, yc, w, h;
};

class BoundingBoxes : public DecoderInstance {
 public:
  bool set_option(int idx, const std::string& v) override {
    switch (idx) {
      case 0: {
        int m = UNKNOWN;
        for (int i = 0; i < UNKNOWN; ++i)
          if (v == kModeNames[i]) m = i;
        if (v.empty()) return false;
        if (m != mode_ && m != UNKNOWN) {
          mode_ = m;
          init_mode();
        }
        mode_ = m;
        return true;
      }
      case 1:
        if (mode_ == MP_PALM) return true;
        labels_ = load_labels(v);
        dev_labels_.reset();
        return !labels_.empty();
      case 2:
        return set_mode_option(v);
      case 3:
      case 4: {
        Dims d;
        unsigned& w = idx == 3 ? width_ : i_width_;
        unsigned& h = idx == 3 ? height_ : i_height_;
        w = h = 0;
        if (v.empty()) return true;
        int rank = parse_dimension(v, d);
        if (rank < 2) return true;  // ignored like the reference
        w = d[0];
        h = d[1];
        return true;
      }
      case 8:  // nnsx: label rendering style (font | solid | none); solid marks the label cells
        label_style_ = v == "solid" ? 2 : (v == "none" ? 0 : 1);
        return true;
      default:
        return true;
    }
  }

  bool supports_device() const override { return true; }

  Caps get_out_caps(const TensorsConfig& config) override {
    unsigned batch = 1;
    if (!check_config(config, &batch)) return Caps();
    Caps c = Caps::from_string(strfmt("video/x-raw, format=(string)RGBA, width=(int)", width_, ", height=(int)", height_));
    set_framerate_from_config(c, config);
    return c;
  }

  FlowReturn decode(const TensorsConfig& config, const std::vector<MemoryPtr>& in, Buffer* out,
                    InvokeContext& ctx) override {
    unsigned batch = 1;
    if (!check_config(config, &batch)) return FlowReturn::ERROR;
    if (width_ == 0 || height_ == 0 || i_width_ == 0 || i_height_ == 0) {
      NNSX_LOGE("bounding_boxes", "option4 (output size) and option5 (input size) must be set");
      return FlowReturn::ERROR;
    }
    use_labels_ = !labels_.empty();
    // every mode has a device path for float32 tensors (K9-K12 + ov-*); other
    // element types decode on the host
    const bool gpu_mode = config.info.at(0).type == DType::FLOAT32 && ctx.device >= 0;
    ctx.out_frames = batch;
    if (gpu_mode) return decode_device(config, in, out, ctx, batch);
    const size_t fsize = static_cast<size_t>(width_) * height_ * 4;
    for (unsigned b = 0; b < batch; ++b) {
      std::vector<Det> res;
      if (!candidates_host(config, in, b, &res)) return FlowReturn::ERROR;
      auto m = Memory::alloc_host(fsize);
      std::memset(m->data(), 0, fsize);
      draw_host(static_cast<uint32_t*>(m->data()), res);
      out->mems.push_back(m);
      last_ = res;
    }
    return FlowReturn::OK;
  }

  // for tests / introspection: boxes of the last host decode
  const std::vector<Det>& last() const { return last_; }

 private:
  bool is_ssd() const { return mode_ == SSD || mode_ == OLD_SSD; }
  bool is_ssd_pp() const { return mode_ == SSD_PP || mode_ == OLD_SSD_PP; }

  void init_mode() {
    if (is_ssd()) {
      ssd_params_[0] = 0.5f;
      ssd_params_[1] = 10.f;
      ssd_params_[2] = 10.f;
      ssd_params_[3] = 5.f;
      ssd_params_[4] = 5.f;
      ssd_params_[5] = 0.5f;
      sig_thr_ = logit(ssd_params_[0]);
    } else if (is_ssd_pp()) {
      pp_map_[0] = 3;  // locations
      pp_map_[1] = 1;  // classes
      pp_map_[2] = 2;  // scores
      pp_map_[3] = 0;  // num
      pp_thr_ = 1.17549435e-38f;
    } else if (mode_ == YOLOV5) {
      yolo_scaled_ = 0;
    } else if (mode_ == MP_PALM) {
      palm_layers_ = 4;
      palm_min_scale_ = palm_max_scale_ = 1.f;
      palm_off_x_ = palm_off_y_ = 0.5f;
      palm_strides_ = {8, 16, 16, 16};
      palm_thr_ = 0.5f;
      anchors_.clear();
    }
    max_detection_ = 0;
  }

  bool set_mode_option(const std::string& v) {
    if (mode_ == YOLOV5) {
      yolo_scaled_ = static_cast<int>(to_int(v));
      return true;
    }
    if (is_ssd()) {
      auto opts = split(v, ':');
      if (opts.empty()) return false;
      if (!load_priors(opts[0])) return false;
      for (size_t i = 1; i < opts.size() && i <= 6; ++i)
        if (!opts[i].empty()) ssd_params_[i - 1] = static_cast<float>(to_double(opts[i]));
      sig_thr_ = logit(ssd_params_[0]);
      return true;
    }
    if (is_ssd_pp()) {
      int a, b, c, d, t;
      if (std::sscanf(v.c_str(), "%i:%i:%i:%i,%i", &a, &b, &c, &d, &t) < 5) {
        NNSX_LOGE("bounding_boxes", "option3 must be \"locations:classes:scores:num,threshold%\"");
        return false;
      }
      pp_map_[0] = a;
      pp_map_[1] = b;
      pp_map_[2] = c;
      pp_map_[3] = d;
      if (t >= 0 && t <= 100) pp_thr_ = t / 100.f;
      return true;
    }
    if (mode_ == MP_PALM) {
      auto opts = split(v, ':');
      if (opts.size() > 13) return false;
      auto f = [&](size_t i, float* dst) {
        if (i < opts.size() && !opts[i].empty()) *dst = static_cast<float>(to_double(opts[i]));
      };
      f(0, &palm_thr_);
      if (opts.size() > 1) palm_layers_ = static_cast<int>(to_int(opts[1]));
      f(2, &palm_min_scale_);
      f(3, &palm_max_scale_);
      f(4, &palm_off_x_);
      f(5, &palm_off_y_);
      palm_strides_.resize(std::max(palm_layers_, 0), 16);
      for (int i = 0; i < palm_layers_ && 6 + i < static_cast<int>(opts.size()); ++i)
        palm_strides_[static_cast<size_t>(i)] = static_cast<int>(to_int(opts[static_cast<size_t>(6 + i)]));
      gen_anchors();
      return true;
    }
    return true;
  }

  bool load_priors(const std::string& path) {
    std::ifstream f(path);
    if (!f) {
      NNSX_LOGE("bounding_boxes", "box prior file ", path, " cannot be read");
      return false;
    }
    priors_.assign(kBoxSize, {});
    std::string line;
    int prev = -1;
    for (int row = 0; row < kBoxSize; ++row) {
      if (!std::getline(f, line)) {
        NNSX_LOGE("bounding_boxes", "prior file needs ", kBoxSize, " lines");
        return false;
      }
      for (auto& w : split_any(line, " \t,")) {
        if (strip(w).empty()) continue;
        if (priors_[static_cast<size_t>(row)].size() > kSsdMax) break;
        priors_[static_cast<size_t>(row)].push_back(static_cast<float>(std::strtod(w.c_str(), nullptr)));
      }
      int reg = static_cast<int>(priors_[static_cast<size_t>(row)].size());
      if (prev != -1 && prev != reg) {
        NNSX_LOGE("bounding_boxes", "box prior data file is not consistent");
        return false;
      }
      prev = reg;
    }
    dev_priors_.reset();
    return true;
  }

  static float calc_scale(float mn, float mx, int idx, int n) {
    if (n == 1) return (mn + mx) * 0.5f;
    return static_cast<float>(mn + (mx - mn) * 1.0 * idx / (n - 1.0f));
  }

  void gen_anchors() {
    anchors_.clear();
    int layer = 0;
    const int n = palm_layers_;
    while (layer < n) {
      std::vector<float> ratios, scales;
      int last = layer;
      while (last < n && palm_strides_[static_cast<size_t>(last)] == palm_strides_[static_cast<size_t>(layer)]) {
        ratios.push_back(1.f);
        ratios.push_back(1.f);
        scales.push_back(calc_scale(palm_min_scale_, palm_max_scale_, last, n));
        scales.push_back(calc_scale(palm_min_scale_, palm_max_scale_, last + 1, n));
        ++last;
      }
      std::vector<float> ah, aw;
      for (size_t i = 0; i < ratios.size(); ++i) {
        float r = std::sqrt(ratios[i]);
        ah.push_back(scales[i] / r);
        aw.push_back(scales[i] * r);
      }
      const int stride = palm_strides_[static_cast<size_t>(layer)];
      const int fh = static_cast<int>(std::ceil(192.0f / stride)), fw = fh;
      for (int y = 0; y < fh; ++y)
        for (int x = 0; x < fw; ++x)
          for (size_t a = 0; a < ratios.size(); ++a)
            anchors_.push_back({(x + palm_off_x_) / fw, (y + palm_off_y_) / fh, aw[a], ah[a]});
      layer = last;
    }
  }

  static bool rest_ones(const uint32_t* d, int from) {
    for (int i = from; i < kRankLimit; ++i)
      if (d[i] != 1) return false;
    return true;
  }

  bool set_max_detection(unsigned md, unsigned limit) {
    if (max_detection_ == 0)
      max_detection_ = md;
    else if (md != max_detection_)
      return false;
    return max_detection_ <= limit;
  }

  bool check_config(const TensorsConfig& config, unsigned* batch) {
    const TensorsInfo& ti = config.info;
    auto same_types = [&](unsigned limit) {
      if (ti.num_tensors < limit) return false;
      for (unsigned i = 1; i < ti.num_tensors; ++i)
        if (ti.at(i).type != ti.at(i - 1).type) return false;
      return true;
    };
    *batch = 1;
    if (is_ssd()) {
      if (!same_types(2)) return false;
      const uint32_t* d1 = ti.at(0).dim.data();
      const uint32_t* d2 = ti.at(1).dim.data();
      if (d1[0] != kBoxSize || d1[1] != 1 || d1[2] == 0) return false;
      unsigned md = d1[2];
      *batch = d1[3];
      if (!rest_ones(d1, 4)) return false;
      if (d2[0] > labels_.size() || d2[1] != md || d2[2] != *batch || !rest_ones(d2, 3)) return false;
      if (priors_.empty() || priors_[0].size() < md) return false;
      return set_max_detection(md, kSsdMax);
    }
    if (is_ssd_pp()) {
      if (!same_types(4)) return false;
      const uint32_t* dn = ti.at(static_cast<unsigned>(pp_map_[3])).dim.data();
      const uint32_t* dc = ti.at(static_cast<unsigned>(pp_map_[1])).dim.data();
      const uint32_t* ds = ti.at(static_cast<unsigned>(pp_map_[2])).dim.data();
      const uint32_t* dl = ti.at(static_cast<unsigned>(pp_map_[0])).dim.data();
      if (dn[0] != 1 || !rest_ones(dn, 1)) return false;
      if (ds[0] != dc[0] || !rest_ones(dc, 1) || !rest_ones(ds, 1)) return false;
      if (dl[0] != kBoxSize || dl[1] != dc[0] || !rest_ones(dl, 2)) return false;
      return set_max_detection(dc[0], kSsdPpMax);
    }
    if (mode_ == OV_PERSON || mode_ == OV_FACE) {
      if (!same_types(1)) return false;
      const uint32_t* d = ti.at(0).dim.data();
      return d[0] == 7 && d[1] == kOvMax && rest_ones(d, 2);
    }
    if (mode_ == YOLOV5) {
      if (!same_types(1)) return false;
      const uint32_t* d = ti.at(0).dim.data();
      max_detection_ = ((i_width_ / 32) * (i_height_ / 32) + (i_width_ / 16) * (i_height_ / 16) +
                        (i_width_ / 8) * (i_height_ / 8)) * 3;
      *batch = d[2];
      return d[0] == labels_.size() + 5 && d[1] == max_detection_ && rest_ones(d, 3) && *batch >= 1;
    }
    if (mode_ == MP_PALM) {
      if (!same_types(2)) return false;
      const uint32_t* d1 = ti.at(0).dim.data();
      const uint32_t* d2 = ti.at(1).dim.data();
      if (d1[0] != 18 || d1[1] == 0 || d1[2] != 1 || !rest_ones(d1, 3)) return false;
      if (d2[0] != 1 || d2[1] != d1[1] || !rest_ones(d2, 2)) return false;
      if (anchors_.size() < d1[1]) {
        if (anchors_.empty()) gen_anchors();
        if (anchors_.size() < d1[1]) return false;
      }
      return set_max_detection(d1[1], kPalmMax);
    }
    return false;
  }

  // -------------------------------------------------------------- host ----
  bool candidates_host(const TensorsConfig& config, const std::vector<MemoryPtr>& in, unsigned b,
                       std::vector<Det>* res) {
    const TensorsInfo& ti = config.info;
    if (is_ssd()) {
      const DType t = ti.at(0).type;
      const void* boxes = in[0]->map_host();
      const void* dets = in[1]->map_host();
      const unsigned n = std::min(max_detection_, kSsdMax);
      const unsigned c = ti.at(1).dim[0];
      const size_t bo = static_cast<size_t>(b) * n * 4, so = static_cast<size_t>(b) * n * c;
      for (unsigned d = 0; d < n; ++d) {
        for (unsigned cl = 1; cl < c; ++cl) {
          float v = static_cast<float>(cpu::read_as_double(dets, t, so + static_cast<size_t>(d) * c + cl));
          if (v < sig_thr_) continue;
          float bx[4];
          for (int k = 0; k < 4; ++k)
            bx[k] = static_cast<float>(cpu::read_as_double(boxes, t, bo + static_cast<size_t>(d) * 4 + static_cast<size_t>(k)));
          float score = 1.f / (1.f + std::exp(-v));
          float ycenter = bx[0] / ssd_params_[1] * priors_[2][d] + priors_[0][d];
          float xcenter = bx[1] / ssd_params_[2] * priors_[3][d] + priors_[1][d];
          float h = std::exp(bx[2] / ssd_params_[3]) * priors_[2][d];
          float w = std::exp(bx[3] / ssd_params_[4]) * priors_[3][d];
          float ymin = ycenter - h / 2.f, xmin = xcenter - w / 2.f;
          Det o;
          o.cls = static_cast<int>(cl);
          o.x = std::max(0, static_cast<int>(xmin * i_width_));
          o.y = std::max(0, static_cast<int>(ymin * i_height_));
          o.w = static_cast<int>(w * i_width_);
          o.h = static_cast<int>(h * i_height_);
          o.prob = score;
          o.valid = true;
          res->push_back(o);
          break;
        }
      }
      nms(res, ssd_params_[5]);
      return true;
    }
    if (is_ssd_pp()) {
      const DType t = ti.at(static_cast<unsigned>(pp_map_[3])).type;
      const void* num = in[static_cast<size_t>(pp_map_[3])]->map_host();
      const void* cls = in[static_cast<size_t>(pp_map_[1])]->map_host();
      const void* sc = in[static_cast<size_t>(pp_map_[2])]->map_host();
      const void* bx = in[static_cast<size_t>(pp_map_[0])]->map_host();
      const unsigned bpi = ti.at(static_cast<unsigned>(pp_map_[0])).dim[0];
      int n = static_cast<int>(cpu::read_as_double(num, t, 0));
      n = std::min(n, static_cast<int>(max_detection_));
      auto clamp01 = [](double v) { return std::min(std::max(v, 0.0), 1.0); };
      for (int d = 0; d < n; ++d) {
        double score = cpu::read_as_double(sc, t, static_cast<size_t>(d));
        if (score < pp_thr_) continue;
        double x1 = clamp01(cpu::read_as_double(bx, t, static_cast<size_t>(d) * bpi + 1));
        double y1 = clamp01(cpu::read_as_double(bx, t, static_cast<size_t>(d) * bpi));
        double x2 = clamp01(cpu::read_as_double(bx, t, static_cast<size_t>(d) * bpi + 3));
        double y2 = clamp01(cpu::read_as_double(bx, t, static_cast<size_t>(d) * bpi + 2));
        if (t == DType::FLOAT32) {  // reference arithmetic runs in the tensor type
          float fx1 = static_cast<float>(x1), fy1 = static_cast<float>(y1), fx2 = static_cast<float>(x2),
                fy2 = static_cast<float>(y2);
          Det o;
          o.valid = true;
          o.cls = static_cast<int>(cpu::read_as_double(cls, t, static_cast<size_t>(d)));
          o.x = static_cast<int>(fx1 * static_cast<float>(i_width_));
          o.y = static_cast<int>(fy1 * static_cast<float>(i_height_));
          o.w = static_cast<int>((fx2 - fx1) * static_cast<float>(i_width_));
          o.h = static_cast<int>((fy2 - fy1) * static_cast<float>(i_height_));
          o.prob = static_cast<float>(score);
          res->push_back(o);
        } else {
          Det o;
          o.valid = true;
          o.cls = static_cast<int>(cpu::read_as_double(cls, t, static_cast<size_t>(d)));
          o.x = static_cast<int>(x1 * i_width_);
          o.y = static_cast<int>(y1 * i_height_);
          o.w = static_cast<int>((x2 - x1) * i_width_);
          o.h = static_cast<int>((y2 - y1) * i_height_);
          o.prob = static_cast<float>(score);
          res->push_back(o);
        }
      }
      return true;
    }
    if (mode_ == OV_PERSON || mode_ == OV_FACE) {
      const DType t = ti.at(0).type;
      const void* p = in[0]->map_host();
      for (unsigned d = 0; d < kOvMax; ++d) {
        double v[7];
        for (int k = 0; k < 7; ++k) v[k] = cpu::read_as_double(p, t, static_cast<size_t>(d) * 7 + static_cast<size_t>(k));
        if (static_cast<int>(v[0]) < 0) break;
        if (v[2] < kOvConf) continue;
        Det o;
        o.cls = -1;
        o.x = static_cast<int>(v[3] * i_width_);
        o.y = static_cast<int>(v[4] * i_height_);
        o.w = static_cast<int>((v[5] - v[3]) * i_width_);
        o.h = static_cast<int>((v[6] - v[4]) * i_height_);
        o.prob = 1;
        o.valid = true;
        res->push_back(o);
      }
      return true;
    }
    if (mode_ == YOLOV5) {
      if (ti.at(0).type != DType::FLOAT32) return false;
      const float* p = static_cast<const float*>(in[0]->map_host());
      const int classes = static_cast<int>(labels_.size());
      const int row = classes + 5;
      const float* base = p + static_cast<size_t>(b) * max_detection_ * row;
      for (unsigned i = 0; i < max_detection_; ++i) {
        const float* r = base + static_cast<size_t>(i) * row;
        float best = -INFINITY;
        int bi = -1;
        for (int c = 0; c < classes; ++c)
          if (r[5 + c] > best) {
            best = r[5 + c];
            bi = c;
          }
        float score = best * r[4];
        if (!(score > kYoloConf)) continue;
        float cx = r[0], cy = r[1], w = r[2], h = r[3];
        if (!yolo_scaled_) {
          cx *= static_cast<float>(i_width_);
          cy *= static_cast<float>(i_height_);
          w *= static_cast<float>(i_width_);
          h *= static_cast<float>(i_height_);
        }
        Det o;
        o.x = static_cast<int>(std::max(0.f, cx - w / 2.f));
        o.y = static_cast<int>(std::max(0.f, cy - h / 2.f));
        o.w = static_cast<int>(std::min(static_cast<float>(i_width_), w));
        o.h = static_cast<int>(std::min(static_cast<float>(i_height_), h));
        o.prob = score;
        o.cls = bi;
        o.valid = true;
        res->push_back(o);
      }
      nms(res, kYoloIou);
      return true;
    }
    if (mode_ == MP_PALM) {
      const DType t = ti.at(0).type;
      const void* boxes = in[0]->map_host();
      const void* scores = in[1]->map_host();
      const unsigned bpi = ti.at(0).dim[0];
      for (unsigned d = 0; d < max_detection_; ++d) {
        float score = static_cast<float>(cpu::read_as_double(scores, t, d));
        score = std::min(std::max(score, -100.f), 100.f);
        score = 1.0f / (1.0f + std::exp(-score));
        if (score < palm_thr_) continue;
        const Anchor& a = anchors_[d];
        float bx[4];
        for (int k = 0; k < 4; ++k)
          bx[k] = static_cast<float>(cpu::read_as_double(boxes, t, static_cast<size_t>(d) * bpi + static_cast<size_t>(k)));
        float yc = bx[0] / i_height_ * a.h + a.yc;
        float xc = bx[1] / i_width_ * a.w + a.xc;
        float h = bx[2] / i_height_ * a.h;
        float w = bx[3] / i_width_ * a.w;
        float ymin = yc - h / 2.f, xmin = xc - w / 2.f;
        Det o;
        o.cls = 0;
        o.x = std::max(0, static_cast<int>(xmin * i_width_));
        o.y = std::max(0, static_cast<int>(ymin * i_height_));
        o.w = static_cast<int>(w * i_width_);
        o.h = static_cast<int>(h * i_height_);
        o.prob = score;
        o.valid = true;
        res->push_back(o);
      }
      nms(res, 0.05f);
      return true;
    }
    return false;
  }

  void draw_host(uint32_t* f, const std::vector<Det>& res) {
    const int64_t W = width_, H = height_;
    auto put = [&](int64_t y, int64_t x, uint32_t v) {
      if (y >= 0 && y < H && x >= 0 && x < W) f[y * W + x] = v;
    };
    for (const Det& a : res) {
      if (use_labels_ && (a.cls < 0 || a.cls >= static_cast<int>(labels_.size()))) continue;
      int64_t x1 = (W * a.x) / i_width_;
      int64_t x2 = std::min(W - 1, (W * (a.x + a.w)) / static_cast<int64_t>(i_width_));
      int64_t y1 = (H * a.y) / i_height_;
      int64_t y2 = std::min(H - 1, (H * (a.y + a.h)) / static_cast<int64_t>(i_height_));
      for (int64_t x = x1; x <= x2; ++x) {
        put(y1, x, font::kPixel);
        put(y2, x, font::kPixel);
      }
      for (int64_t y = y1 + 1; y < y2; ++y) {
        put(y, x1, font::kPixel);
        put(y, x2, font::kPixel);
      }
      if (use_labels_ && label_style_ != 0) {
        const std::string& lab = labels_[static_cast<size_t>(a.cls)];
        int64_t ly = std::max<int64_t>(0, y1 - font::kAboveBox);
        int64_t lx = x1;
        for (unsigned char ch : lab) {
          if (lx + 8 > W) break;
          for (int r = 0; r < font::kCellH; ++r)
            for (int c = 0; c < font::kCellW; ++c)
              put(ly + r, lx + c, (label_style_ == 2 || font::cell_on(kFont, ch, r, c)) ? font::kPixel : 0u);
          lx += font::kAdvance;
        }
      }
    }
  }

  // ------------------------------------------------------------ device ----
  // Device decode in two parts: prepare (scratch, priors / anchors / labels
  // uploaded once; may sync) and enqueue (kernels + one memset on `s`, no host
  // work, no allocation) -- so the same enqueue also runs inside an upstream
  // filter's hipGraph capture (stage_enqueue, runtime/fusion.h).
  bool prepare_device(const TensorsConfig& config, int dev, hipStream_t s, unsigned batch) {
    const int n = det_count();
    const int k = std::min(kNmsCap, (n + 63) / 64 * 64);
    const size_t need = kernels::det_scratch_bytes(n, k, static_cast<int>(batch));
    if (!scratch_ || scratch_->size() < need || scratch_->device() != dev) {
      // a decode still queued on the old block keeps it alive (record_use)
      scratch_ = Memory::alloc_device(need, dev, s);
    }
    ensure_labels(dev, s);
    if (is_ssd() && (!dev_priors_ || dev_priors_->device() != dev)) {
      // rows of n priors (the kernel's stride: the decoded box count)
      std::vector<float> flat(4 * static_cast<size_t>(n));
      for (int r = 0; r < 4; ++r)
        std::memcpy(flat.data() + static_cast<size_t>(r) * n, priors_[static_cast<size_t>(r)].data(), sizeof(float) * n);
      dev_priors_ = Memory::alloc_device(flat.size() * sizeof(float), dev, s);
      hip::check(hipMemcpyAsync(dev_priors_->data(), flat.data(), flat.size() * sizeof(float), hipMemcpyHostToDevice, s),
                 "priors H2D");
      hip::check(hipStreamSynchronize(s), "priors sync");
    }
    if (mode_ == MP_PALM && (!dev_anchors_ || dev_anchors_->device() != dev || dev_anchor_count_ != anchors_.size())) {
      std::vector<float> flat;
      for (const Anchor& a : anchors_) flat.insert(flat.end(), {a.xc, a.yc, a.w, a.h});
      dev_anchors_ = Memory::alloc_device(flat.size() * sizeof(float), dev, s);
      hip::check(hipMemcpyAsync(dev_anchors_->data(), flat.data(), flat.size() * sizeof(float), hipMemcpyHostToDevice, s),
                 "anchors H2D");
      hip::check(hipStreamSynchronize(s), "anchors sync");
      dev_anchor_count_ = anchors_.size();
    }
    dev_cfg_ = config;
    dev_batch_ = batch;
    return true;
  }
  int det_count() const {
    return static_cast<int>(is_ssd()                                  ? std::min(max_detection_, kSsdMax)
                            : (mode_ == OV_PERSON || mode_ == OV_FACE) ? kOvMax
                                                                       : max_detection_);
  }
  // in: device pointers of the input tensors (config order); frames: B RGBA frames
  void enqueue_device(const std::vector<const void*>& in, uint32_t* frames, hipStream_t s) {
    const TensorsConfig& config = dev_cfg_;
    const unsigned batch = dev_batch_;
    const int n = det_count();
    const int k = std::min(kNmsCap, (n + 63) / 64 * 64);
    kernels::DetScratch ds = kernels::det_scratch_carve(scratch_->data(), n, k, static_cast<int>(batch));
    auto f = [&](size_t i) { return static_cast<const float*>(in[i]); };
    if (is_ssd()) {
      kernels::SsdParams p{sig_thr_, ssd_params_[1], ssd_params_[2], ssd_params_[3], ssd_params_[4],
                           static_cast<int>(i_width_), static_cast<int>(i_height_)};
      kernels::ssd_candidates(f(0), f(1), static_cast<const float*>(dev_priors_->data()),
                              static_cast<int>(config.info.at(1).dim[0]), static_cast<int>(batch), p, ds, s);
      kernels::sort_nms(ds, static_cast<int>(batch), ssd_params_[5], s);
    } else if (is_ssd_pp()) {
      kernels::pp_candidates(f(static_cast<size_t>(pp_map_[0])), f(static_cast<size_t>(pp_map_[1])),
                             f(static_cast<size_t>(pp_map_[2])), f(static_cast<size_t>(pp_map_[3])),
                             static_cast<int>(config.info.at(static_cast<unsigned>(pp_map_[0])).dim[0]), pp_thr_,
                             static_cast<int>(i_width_), static_cast<int>(i_height_), ds, s);
      kernels::sort_keep_all(ds, 1, s);
    } else if (mode_ == OV_PERSON || mode_ == OV_FACE) {
      kernels::ov_candidates(f(0), kOvConf, static_cast<int>(i_width_), static_cast<int>(i_height_), ds, s);
      kernels::sort_keep_all(ds, 1, s);
    } else if (mode_ == MP_PALM) {
      kernels::palm_candidates(f(0), f(1), static_cast<const float*>(dev_anchors_->data()),
                               static_cast<int>(config.info.at(0).dim[0]), palm_thr_, static_cast<int>(i_width_),
                               static_cast<int>(i_height_), ds, s);
      kernels::sort_nms(ds, 1, 0.05f, s);
    } else {
      kernels::yolov5_candidates(f(0), static_cast<int>(labels_.size()), static_cast<int>(batch), kYoloConf,
                                 yolo_scaled_, static_cast<int>(i_width_), static_cast<int>(i_height_), ds, s);
      kernels::sort_nms(ds, static_cast<int>(batch), kYoloIou, s);
    }
    const size_t fsize = static_cast<size_t>(width_) * height_ * 4;
    hip::check(hipMemsetAsync(frames, 0, fsize * batch, s), "clear frames");
    kernels::draw_boxes(ds, static_cast<int>(batch), frames, static_cast<int>(width_), static_cast<int>(height_),
                        static_cast<int>(i_width_), static_cast<int>(i_height_),
                        dev_labels_ ? static_cast<const char*>(dev_labels_->data()) : nullptr,
                        dev_label_offs_ ? static_cast<const int*>(dev_label_offs_->data()) : nullptr,
                        static_cast<int>(labels_.size()), use_labels_, label_style_, s);
  }

  FlowReturn decode_device(const TensorsConfig& config, const std::vector<MemoryPtr>& in, Buffer* out,
                           InvokeContext& ctx, unsigned batch) {
    const int dev = ctx.device;
    hipStream_t s = ctx.stream;
    prepare_device(config, dev, s, batch);
    std::vector<const void*> ptrs;
    for (auto& m : in) ptrs.push_back(m->map_device(dev, s));
    const size_t fsize = static_cast<size_t>(width_) * height_ * 4;
    MemoryPtr frames = Memory::alloc_device(fsize * batch, dev, s);
    enqueue_device(ptrs, static_cast<uint32_t*>(frames->data()), s);
    frames->mark_ready(s);
    scratch_->record_use(s, dev);
    for (unsigned b = 0; b < batch; ++b) out->mems.push_back(Memory::view(frames, b * fsize, fsize));
    return FlowReturn::OK;
  }

 public:
  // ---- device stage (runtime/fusion.h): candidates + sort + NMS + raster in
  // the filter's graph; output = the B RGBA frames [4:W:H:B] ----
  bool stage_prepare(const TensorsConfig& config, int dev, hipStream_t s, TensorsInfo* out) override {
    unsigned batch = 1;
    if (dev < 0 || !check_config(config, &batch) || config.info.at(0).type != DType::FLOAT32 || width_ == 0 ||
        height_ == 0 || i_width_ == 0 || i_height_ == 0)
      return false;
    for (unsigned i = 0; i < config.info.num_tensors; ++i)
      if (config.info.at(i).type != DType::FLOAT32) return false;
    use_labels_ = !labels_.empty();
    if (!prepare_device(config, dev, s, batch)) return false;
    out->resize(1);
    TensorInfo& t = out->at(0);
    t.type = DType::UINT8;
    t.dim = make_dims({4, width_, height_, batch});
    return true;
  }
  bool stage_enqueue(const std::vector<const void*>& in, const std::vector<void*>& out, hipStream_t s) override {
    if (in.size() != dev_cfg_.info.num_tensors || out.size() != 1) return false;
    enqueue_device(in, static_cast<uint32_t*>(out[0]), s);
    return true;
  }

 private:
  void ensure_labels(int dev, hipStream_t s) {
    if (labels_.empty() || (dev_labels_ && dev_labels_->device() == dev)) return;
    std::string blob;
    std::vector<int> offs;
    for (auto& l : labels_) {
      offs.push_back(static_cast<int>(blob.size()));
      blob += l;
      blob.push_back('\0');
    }
    dev_labels_ = Memory::alloc_device(blob.size(), dev, s);
    dev_label_offs_ = Memory::alloc_device(offs.size() * sizeof(int), dev, s);
    hip::check(hipMemcpyAsync(dev_labels_->data(), blob.data(), blob.size(), hipMemcpyHostToDevice, s), "labels");
    hip::check(hipMemcpyAsync(dev_label_offs_->data(), offs.data(), offs.size() * sizeof(int), hipMemcpyHostToDevice, s),
               "label offsets");
    hip::check(hipStreamSynchronize(s), "labels sync");
  }

  int mode_ = UNKNOWN;
  std::vector<std::string> labels_;
  bool use_labels_ = false;
  int label_style_ = 1;
  unsigned width_ = 0, height_ = 0, i_width_ = 0, i_height_ = 0, max_detection_ = 0;
  // mobilenet-ssd
  std::vector<std::vector<float>> priors_;
  float ssd_params_[6] = {0.5f, 10.f, 10.f, 5.f, 5.f, 0.5f};
  float sig_thr_ = 0;
  // mobilenet-ssd-postprocess
  int pp_map_[4] = {3, 1, 2, 0};
  float pp_thr_ = 1.17549435e-38f;
  // yolov5
  int yolo_scaled_ = 0;
  // mp-palm-detection
  int palm_layers_ = 4;
  float palm_min_scale_ = 1.f, palm_max_scale_ = 1.f, palm_off_x_ = 0.5f, palm_off_y_ = 0.5f, palm_thr_ = 0.5f;
  std::vector<int> palm_strides_ = {8, 16, 16, 16};
  std::vector<Anchor> anchors_;
  // device state
  MemoryPtr scratch_, dev_priors_, dev_labels_, dev_label_offs_, dev_anchors_;
  size_t dev_anchor_count_ = 0;
  TensorsConfig dev_cfg_;  // the input config prepare_device sized the scratch for
  unsigned dev_batch_ = 1;
  std::vector<Det> last_;
};

class BoundingBoxesPlugin : public DecoderSubplugin {
 public:
  std::string name() const override { return "bounding_boxes"; }
  std::unique_ptr<DecoderInstance> create() override { return std::make_unique<BoundingBoxes>(); }
};

}  // namespace

void register_bbox_decoder() { register_decoder(std::make_shared<BoundingBoxesPlugin>()); }

}  // namespace nnsx
