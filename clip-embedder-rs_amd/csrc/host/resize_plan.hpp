// Crop + resize plan of one image (src/vision.rs:164-198, resize_with_fast_image_resize),
// shared by the host resize (preprocess.cpp) and the GPU resize (kernels/resize.hip) so
// both apply the very same fixed-point coefficients: the GPU output is bit-identical
// to the host's, which the tests pin to the CPU restatement of the reference.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace clipgpu {

constexpr int kResizePrecisionBits = 32 - 8 - 2;  // Pillow's 22-bit coefficients

// One separable axis: output i reads input [bounds[2i], bounds[2i] + bounds[2i+1]) with
// weights k[i*ksize ..] (fixed point, sum ~= 1 << kResizePrecisionBits).
struct AxisPlan {
  int ksize = 0;
  std::vector<int> bounds;
  std::vector<int32_t> k;
};

// Horizontal pass (need_h): rows [yfirst, yfirst + th) of the source -> tmp [th][S][3];
// vertical pass (need_v): tmp (or the source when !need_h) -> out [S][S][3], with v.bounds
// relative to the pass input.  A pass that is not needed is a straight copy (the source
// already has that axis at S with an identity box).  Nearest is the same two passes with
// one unit tap per output (exact: (p << 22 + 2^21) >> 22 == p).
struct ResizePlan {
  int W = 0, H = 0, S = 0;
  bool need_h = false, need_v = false;
  int yfirst = 0, th = 0;
  AxisPlan h, v;
};

ResizePlan make_resize_plan(int W, int H, int S, const std::string& interp, const std::string& mode);
// Host application of a plan (the reference's resize, on the CPU).
void apply_resize_plan(const ResizePlan& p, const uint8_t* src, uint8_t* dst);

}  // namespace clipgpu
