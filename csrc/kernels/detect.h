// Object-detection post-processing on CDNA4: candidate extraction for SSD /
// YOLO heads, per-frame sort + bitmask NMS, and RGBA box/label rasterisation.
// Used by the bounding_boxes decoder (csrc/decoders/bounding_boxes.cc).
//
// Data flow per batch of B frames (all on one stream, no host sync):
//   *_candidates  -> keys/boxes per frame (atomic slot per passing anchor)
//   sort_nms      -> bitonic sort by (score desc, anchor asc), IoU bit matrix,
//                    one-wave greedy reduction == the reference's sequential NMS
//   draw_boxes    -> RGBA frames (box outlines + label sprites, drawn in order)
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

namespace nnsx {
namespace kernels {

struct DetScratch {
  int n = 0;            // anchors per frame (stride of the per-anchor arrays)
  int k = 0;            // NMS capacity per frame (multiple of 64)
  int key_cap = 0;      // power-of-two key capacity per frame (>= n)
  int* count = nullptr;        // [B] candidates passing the threshold
  uint64_t* keys = nullptr;    // [B][key_cap]
  int4* box = nullptr;         // [B][n]  x, y, w, h (input-model pixels)
  int* cls = nullptr;          // [B][n]
  float* prob = nullptr;       // [B][n]
  int4* sbox = nullptr;        // [B][k] sorted candidates
  int* scls = nullptr;         // [B][k]
  float* sprob = nullptr;      // [B][k]
  uint64_t* mask = nullptr;    // [B][k][k/64]
  int* kept = nullptr;         // [B][k] indices into the sorted arrays
  int* nkept = nullptr;        // [B]
};

// bytes of scratch for B frames of n anchors (k = NMS capacity)
size_t det_scratch_bytes(int n, int k, int batch);
DetScratch det_scratch_carve(void* base, int n, int k, int batch);

struct SsdParams {
  float sigmoid_threshold;
  float y_scale, x_scale, h_scale, w_scale;
  int i_width, i_height;
};

// mobilenet-ssd: boxes [B][n][4], scores [B][n][c] (logits), priors [4][n]
// (ycenter, xcenter, h, w).  First class >= threshold wins (reference order).
void ssd_candidates(const float* boxes, const float* scores, const float* priors, int c, int batch,
                    const SsdParams& p, const DetScratch& s, hipStream_t stream);

// yolov5: in [B][n][5 + classes]; score = max class conf * objectness
void yolov5_candidates(const float* in, int classes, int batch, float conf_threshold, int scaled_output,
                       int i_width, int i_height, const DetScratch& s, hipStream_t stream);

// mobilenet-ssd-postprocess / tf-ssd (one frame): loc [n][bpi] (ymin, xmin,
// ymax, xmax), cls [n], score [n], num [1]; drawn in input order, no NMS
void pp_candidates(const float* loc, const float* cls, const float* score, const float* num, int bpi, float thr,
                   int i_width, int i_height, const DetScratch& s, hipStream_t stream);
// ov-person / ov-face (one frame): in [n <= 256][7]; drawn in input order, no NMS
void ov_candidates(const float* in, float conf, int i_width, int i_height, const DetScratch& s, hipStream_t stream);
// mp-palm-detection (one frame): boxes [n][bpi], scores [n] (logits), anchors [n][4] (xc, yc, w, h)
void palm_candidates(const float* boxes, const float* scores, const float* anchors, int bpi, float thr, int i_width,
                     int i_height, const DetScratch& s, hipStream_t stream);
// order-preserving modes: sort by the candidates' order keys, keep all
void sort_keep_all(const DetScratch& s, int batch, hipStream_t stream);

// sort + NMS (suppress when IoU > iou_threshold, reference integer-box IoU)
void sort_nms(const DetScratch& s, int batch, float iou_threshold, hipStream_t stream);

// Draw kept boxes into B RGBA frames (frames must be zeroed by the caller).
// labels: concatenated NUL-terminated strings with offsets; use_labels
// skips out-of-range classes and draws the label sprite above the box
// (label_style: 0 none, 1 font, 2 solid cells).
void draw_boxes(const DetScratch& s, int batch, uint32_t* frames, int width, int height, int i_width,
                int i_height, const char* labels, const int* label_offsets, int n_labels, bool use_labels,
                int label_style, hipStream_t stream);

}  // namespace kernels
}  // namespace nnsx
