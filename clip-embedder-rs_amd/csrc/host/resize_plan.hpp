// Crop + resize plan of one image (src/vision.rs:164-198, resize_with_fast_image_resize),
// shared by the host resize (preprocess.cpp) and the GPU resize (kernels/resize.hip) so
// both apply the very same fixed-point coefficients: the GPU output is bit-identical
// to the host's, which the tests pin to the CPU restatement of the reference.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace clipgpu {

// fast_image_resize 6.0.0's u8 convolution (its Normalizer16, a port of Pillow-SIMD): the
// normalised f64 weights of an axis become i16 fixed point at the largest precision p < 22 for
// which round(max weight * 2^p) still fits under 2^15 (the identity's unit tap: p = 14;
// test_fast_image_resize_coefficient_precision); a pass sums 2^(p-1) + pixel * k in i32 and stores
// clamp(sum >> p, 0, 255).
constexpr int kResizeMaxPrecision = 32 - 8 - 2;  // PRECISION_BITS (the precision search's bound)
constexpr int kResizeCoefBits = 16 - 1;          // MAX_COEFS_PRECISION (i16 coefficients)

// One separable axis: output i reads input [bounds[2i], bounds[2i] + bounds[2i+1]) with
// weights k[i*ksize ..] (fixed point at `prec` bits, sum ~= 1 << prec).
struct AxisPlan {
  int ksize = 0;
  int prec = kResizeMaxPrecision;
  std::vector<int> bounds;
  std::vector<int32_t> k;
};

// Horizontal pass (need_h): rows [yfirst, yfirst + th) of the source -> tmp [th][S][3];
// vertical pass (need_v): tmp (or the source when !need_h) -> out [S][S][3], with v.bounds
// relative to the pass input.  A pass that is not needed is a straight copy (the source
// already has that axis at S with an identity box).  Nearest is the same two passes with
// one unit tap per output (exact: (p << prec + 2^(prec-1)) >> prec == p).
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
