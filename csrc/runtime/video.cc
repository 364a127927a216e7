#include "runtime/video.h"

#include "core/util.h"

namespace nnsx {

const std::vector<std::string>& video_formats_all() {
  static const std::vector<std::string> v = {"RGB",  "BGR",  "RGBx", "BGRx", "xRGB",      "xBGR", "RGBA", "BGRA",
                                             "ARGB", "ABGR", "GRAY8", "GRAY16_LE", "I420", "NV12", "NV21", "YUY2"};
  return v;
}

bool video_format_info(const std::string& f, int* bpp, int* channels) {
  if (f == "RGB" || f == "BGR") {
    *bpp = 3;
    *channels = 3;
  } else if (f == "RGBx" || f == "BGRx" || f == "xRGB" || f == "xBGR" || f == "RGBA" || f == "BGRA" ||
             f == "ARGB" || f == "ABGR") {
    *bpp = 4;
    *channels = 4;
  } else if (f == "GRAY8") {
    *bpp = 1;
    *channels = 1;
  } else if (f == "GRAY16_LE" || f == "GRAY16_BE") {
    *bpp = 2;
    *channels = 1;
  } else if (f == "YUY2") {
    *bpp = 2;
    *channels = 2;
  } else if (f == "I420" || f == "NV12" || f == "NV21" || f == "YV12") {
    *bpp = 0;
    *channels = 1;
  } else {
    return false;
  }
  return true;
}

bool VideoInfo::from_structure(const Structure& s) {
  if (s.name() != "video/x-raw") return false;
  if (!s.get_string("format", &format)) return false;
  int64_t w, h;
  if (!s.get_int("width", &w) || !s.get_int("height", &h)) return false;
  width = static_cast<int>(w);
  height = static_cast<int>(h);
  if (!s.get_fraction("framerate", &fps_n, &fps_d)) {
    fps_n = 0;
    fps_d = 1;
  }
  if (!video_format_info(format, &bpp, &channels)) return false;
  if (bpp > 0) {
    stride[0] = round_up4(static_cast<size_t>(width) * bpp);
    offset[0] = 0;
    size = stride[0] * height;
  } else {
    // 4:2:0 planar (GStreamer default strides)
    size_t cw = (width + 1) / 2, ch = (height + 1) / 2;
    stride[0] = round_up4(width);
    if (format == "I420" || format == "YV12") {
      stride[1] = stride[2] = round_up4(cw);
      offset[1] = stride[0] * round_up4(height) / 1;  // GStreamer: stride0 * GST_ROUND_UP_2(height)
      offset[1] = stride[0] * ((height + 1) & ~1);
      offset[2] = offset[1] + stride[1] * ch;
      size = offset[2] + stride[2] * ch;
    } else {  // NV12 / NV21
      stride[1] = round_up4(width);
      offset[1] = stride[0] * ((height + 1) & ~1);
      size = offset[1] + stride[1] * ch;
    }
  }
  return true;
}

Structure VideoInfo::to_structure() const {
  Structure s("video/x-raw");
  s.set("format", Value::String(format));
  s.set("width", Value::Int(width));
  s.set("height", Value::Int(height));
  s.set("framerate", Value::Fraction(fps_n, fps_d));
  return s;
}

bool audio_format_info(const std::string& f, int* ss) {
  if (f == "S8" || f == "U8") *ss = 1;
  else if (f == "S16LE" || f == "U16LE" || f == "S16BE" || f == "U16BE") *ss = 2;
  else if (f == "S32LE" || f == "U32LE" || f == "F32LE" || f == "S32BE" || f == "U32BE" || f == "F32BE") *ss = 4;
  else if (f == "F64LE" || f == "F64BE") *ss = 8;
  else return false;
  return true;
}

bool AudioInfo::from_structure(const Structure& s) {
  if (s.name() != "audio/x-raw") return false;
  if (!s.get_string("format", &format)) return false;
  int64_t r = 0, c = 0;
  if (!s.get_int("rate", &r) || !s.get_int("channels", &c)) return false;
  rate = static_cast<int>(r);
  channels = static_cast<int>(c);
  if (!audio_format_info(format, &sample_size)) return false;
  bpf = sample_size * channels;
  return true;
}

}  // namespace nnsx
