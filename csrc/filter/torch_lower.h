// Load-time lowering of a plain TorchScript model onto the CDNA4 engine
// (tensor_filter framework=pytorch): see torch_lower.cc.
#pragma once

#include <torch/script.h>

#include <string>

namespace nnsx {

struct LowerReport {
  int convs = 0;          // conv2d nodes in the frozen graph
  int lowered = 0;        // of them, now on nnsx ops
  int linears = 0;        // aten::linear nodes on the nnsx GEMM
  int ir_blocks = 0;      // inverted residuals fused into one op
  bool stem_block = false;  // stem + first block fused (stem_ir1)
  bool head_pool = false;   // head 1x1 conv + global average pool fused
  bool lut = false;         // the module got an `in_lut` input table (uint8 frames)
  std::string summary() const;
};

// Rewrites the frozen module's forward graph in place: conv2d / BatchNorm-
// folded conv chains become torch.ops.nnsx ops on NHWC activations, with
// weights re-laid-out (and split into their bf16 parts) once, here.  Returns
// false (module untouched) when nothing matched or the graph is not frozen.
// `device` is where the new weight constants live.
bool lower_to_engine(torch::jit::Module& m, const torch::Device& device, LowerReport* rep, std::string* err);

}  // namespace nnsx
