// Raw video / audio format helpers (GstVideoInfo / GstAudioInfo subset).
#pragma once

#include <string>
#include <vector>

#include "core/caps.h"

namespace nnsx {

struct VideoInfo {
  std::string format;  // RGB, BGR, RGBx, BGRx, xRGB, xBGR, RGBA, BGRA, ARGB, ABGR, GRAY8, GRAY16_LE, I420, NV12, NV21, YUY2
  int width = 0;
  int height = 0;
  int fps_n = 0;
  int fps_d = 1;
  int bpp = 0;              // bytes per pixel for packed formats (0 for planar)
  int channels = 0;         // tensor channel count (3 or 4 or 1)
  size_t stride[3] = {0, 0, 0};
  size_t offset[3] = {0, 0, 0};
  size_t size = 0;          // padded frame size

  bool from_structure(const Structure& s);
  bool packed() const { return bpp > 0; }
  Structure to_structure() const;
};

// Packed-RGB family and gray formats the tensor_converter handles.
const std::vector<std::string>& video_formats_all();
bool video_format_info(const std::string& fmt, int* bpp, int* channels);
// Round up to 4 (GST_ROUND_UP_4)
inline size_t round_up4(size_t v) { return (v + 3) & ~static_cast<size_t>(3); }

struct AudioInfo {
  std::string format;  // S8 U8 S16LE U16LE S32LE U32LE F32LE F64LE
  int rate = 0;
  int channels = 0;
  int bpf = 0;         // bytes per frame
  int sample_size = 0;
  bool from_structure(const Structure& s);
};
bool audio_format_info(const std::string& fmt, int* sample_size);

}  // namespace nnsx
