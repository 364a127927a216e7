// Cross-element fusion at caps negotiation.
//
// The reference classification pipeline normalises frames in a separate
// element: `tensor_converter ! tensor_transform mode=arithmetic
// option=typecast:float32,add:-127.5,div:127.5 ! tensor_filter ...`
// (gsttensor_transform.c:1241-1412).  Run as written, that is one more kernel
// and a 4x larger tensor (uint8 -> float32) between the two elements.  nnsx
// lets the consumer absorb the transform instead: when the filter's model maps
// a uint8 input through a 256-entry table (the fused CDNA4 stems do), the
// filter registers itself as the transform's absorber; at caps negotiation the
// transform describes its per-element arithmetic, the filter folds it into the
// model's table (computed in the transform's own fp32 arithmetic, so results
// are bit-identical) and the transform passes the uint8 frames through.  Any
// arithmetic the model cannot take (per-channel ops, stand, transpose, other
// input types) keeps running in the transform's own kernel.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "core/types.h"
#include "kernels/kernels.h"

namespace nnsx {

// The per-element arithmetic an upstream tensor_transform applies to one tensor.
struct ArithPrefix {
  unsigned tensor = 0;           // tensor index in the stream
  DType in_type = DType::END;    // element type entering the transform
  DType out_type = DType::END;   // element type it produces
  kernels::ArithParams params;   // add/mul/div chain in order (nops == 0: typecast only)
};

class TransformAbsorber {
 public:
  virtual ~TransformAbsorber() = default;
  // Called by the transform while it negotiates.  true = the absorber now
  // applies `p` itself and accepts `p.in_type` data; the transform passes
  // buffers through unchanged.  `by` names the transform (logs, properties).
  virtual bool absorb_arith(const ArithPrefix& p, const std::string& by) = 0;
};

// Implemented by elements whose work a downstream consumer may absorb.
class AbsorbableElement {
 public:
  virtual ~AbsorbableElement() = default;
  virtual void set_absorber(TransformAbsorber* a) = 0;
  virtual bool absorbed() const = 0;
};

// Downstream: `tensor_filter ! [queue !] tensor_decoder mode=image_labeling`
// classifies by an argmax over the scores.  A filter whose framework can run
// that argmax at the end of its own device work (inside its captured hipGraph)
// asks the decoder to take the int32 indices instead: the scores never leave
// the graph (no copy-out of [classes x B] floats, no separate argmax launch
// between the graph and the decoder), only B indices cross to the host.
class ArgmaxConsumer {  // implemented by tensor_decoder
 public:
  virtual ~ArgmaxConsumer() = default;
  // the producer would hand over indices of tensor `tensor` ([classes:B]
  // scores -> int32 [1:B]); true = accepted (the decoder now expects them)
  virtual bool take_argmax(unsigned tensor, uint32_t classes, const std::string& by) = 0;
  virtual void drop_argmax() = 0;
};

// Downstream, generalised: the WHOLE device post-processing of a decoder
// (bounding_boxes: candidates + sort + NMS + raster; image_segment: resize +
// argmax + colour map; pose_estimation: heatmap argmax + skeleton raster) as
// one capturable stage that the filter appends to its captured forward, so
// model outputs -> decoded RGBA frames is one hipGraph replay and only the
// frames leave it.  The decoder prepares the stage at caps negotiation
// (scratch, uploaded tables: all allocated up front, so the captured kernels
// keep valid pointers across replays); the filter allocates the outputs per
// graph instance and calls enqueue() while capturing (kernels and memsets
// only).  The decoder then receives the stage outputs and only slices them
// into per-frame media buffers.
class DecodeStage {
 public:
  virtual ~DecodeStage() = default;
  virtual const TensorsInfo& out_info() const = 0;  // the tensors enqueue() writes
  // in = device pointers of the model outputs (the decoder's normal input),
  // out = device buffers sized by out_info(); capturable work on s only
  virtual bool enqueue(const std::vector<const void*>& in, const std::vector<void*>& out, void* stream) = 0;
  // true once the decoder's mode or options changed after this stage was
  // prepared: graphs captured with it run the old post-processing.  The filter
  // checks it before every invoke and re-takes a fresh stage (re-capturing).
  virtual bool stale() const { return false; }
  // true when enqueue() touches no buffer of the stage's own (only `in` and
  // `out`): graphs captured with it on several replay lanes may then run
  // concurrently.  Stages with scratch (candidate lists, keypoints) say false.
  virtual bool lane_safe() const { return false; }
};

class DecodeStageConsumer {  // implemented by tensor_decoder
 public:
  virtual ~DecodeStageConsumer() = default;
  // the producer's outputs (`model_out`, on GPU `dev`) would go through the
  // decoder's device stage upstream; nullptr = the decoder has none / declines
  virtual std::shared_ptr<DecodeStage> take_stage(const TensorsConfig& model_out, int dev, const std::string& by) = 0;
  virtual void drop_stage() = 0;
};

// The transform's output for every uint8 value 0..255 (out must be FLOAT32):
// the table an absorbing model applies.  Computed with the transform's own
// host arithmetic (tensor_transform.cc), which its device kernel matches.
bool arith_table_u8(const kernels::ArithParams& p, DType out, std::vector<float>* lut);

}  // namespace nnsx
