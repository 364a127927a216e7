// Segmentation / pose post-processing kernels (kernels/vision.hip), used by
// the image_segment and pose_estimation decoders.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

namespace nnsx {
namespace kernels {

// tflite-deeplab: prob [pixels][labels] -> RGBA; label = argmax (first max),
// background when max <= threshold; colour = rgb_modifier * label | alpha.
void segment_argmax_color(const float* prob, int labels, uint64_t pixels, uint32_t rgb_modifier, float threshold,
                          uint32_t* out, hipStream_t s);
// tflite-deeplab on a low-resolution score map: logits [B][h][w][labels] are
// bilinearly resized (align_corners) to H x W per label, then argmax / threshold
// / colour as above -> out [B][H][W]; the H x W x labels map is never stored.
void segment_upsample_argmax_color(const float* logits, int labels, int h, int w, int batch, int H, int W,
                                   uint32_t rgb_modifier, float threshold, uint32_t* out, hipStream_t s);
// NHWC bilinear resize with align_corners: x [B][h][w][C] -> y [B][H][W][C]
void upsample_bilinear_nhwc(const float* x, int batch, int h, int w, int C, int H, int W, float* y, hipStream_t s);
// snpe-deeplab: label index map (float) -> RGBA
void segment_index_color(const float* index_map, uint64_t pixels, int max_labels, uint32_t rgb_modifier,
                         uint32_t* out, hipStream_t s);
// snpe-depth: grayscale normalised by the per-frame maximum; ws holds `batch` uint32
void segment_depth_gray(const float* in, uint64_t pixels_per_frame, int batch, uint32_t* ws, uint32_t* out,
                        hipStream_t s);
// pose: heat [B][gh][gw][K] -> out [B][K][3] = (grid x, grid y, score)
void pose_heatmap_argmax(const float* heat, int keypoints, int grid_w, int grid_h, int batch, bool sigmoid,
                         float* out, hipStream_t s);

// pose: keypoint positions (+ offsets) and skeleton / dot / label raster into
// zeroed RGBA frames [B][H][W]; edges = (i, k) pairs with k > i; <= 64 keypoints
struct PoseDrawArgs {
  const float* kp = nullptr;       // [B][K][3] from pose_heatmap_argmax
  const float* offsets = nullptr;  // heatmap-offset mode: [B][gh][gw][2K], else null
  int keypoints = 0, gw = 0, gh = 0, i_w = 0, i_h = 0, W = 0, H = 0;
  const int* edges = nullptr;
  int n_edges = 0;
  const char* labels = nullptr;
  const int* label_offs = nullptr;
  uint32_t* frames = nullptr;
};
void pose_draw(const PoseDrawArgs& a, int batch, hipStream_t s);

}  // namespace kernels
}  // namespace nnsx
