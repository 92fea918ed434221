// Clip facade scores on the host, with the reference's own f32 arithmetic bit for bit
// (src/clip.rs:79-185, kept as-is by the north star; Rust is absent here, so the host mirror
// calls this instead of re-deriving the math in numpy):
//   sim    = emb . query        ndarray 0.17.2 without BLAS (Cargo.toml:14): Array2.dot(Array1)
//                               -> general_mat_vec_mul -> row.dot(x) -> numeric_util::unrolled_dot
//                               (eight f32 partial sums, combined (p0+p4), (p1+p5), (p2+p6),
//                               (p3+p7), then the < 8-element tail; Array1.dot(Array1) is the
//                               same function, :85)
//   logit  = sim.mul_add(scale, bias)                    fused multiply-add (:89, :108, :150)
//   softmax: max by f32::max fold from -inf, exp (libm expf, as Rust's f32::exp), a sequential
//            f32 sum (Iterator::sum), then x / sum            (:174-179)
//   sigmoid: 1 / (1 + exp(-l))                                (:183-185)
// Built with -ffp-contract=off: no other multiply-add is fused.
#include <cmath>
#include <cstdint>

#include "../../../include/clipgpu.h"
#include "api_util.hpp"

namespace clipgpu {

float unrolled_dot(const float* xs, const float* ys, int64_t n) {
  float p0 = 0.f, p1 = 0.f, p2 = 0.f, p3 = 0.f, p4 = 0.f, p5 = 0.f, p6 = 0.f, p7 = 0.f;
  int64_t i = 0;
  for (; i + 8 <= n; i += 8) {
    p0 = p0 + xs[i + 0] * ys[i + 0];
    p1 = p1 + xs[i + 1] * ys[i + 1];
    p2 = p2 + xs[i + 2] * ys[i + 2];
    p3 = p3 + xs[i + 3] * ys[i + 3];
    p4 = p4 + xs[i + 4] * ys[i + 4];
    p5 = p5 + xs[i + 5] * ys[i + 5];
    p6 = p6 + xs[i + 6] * ys[i + 6];
    p7 = p7 + xs[i + 7] * ys[i + 7];
  }
  float sum = 0.f;
  sum = sum + (p0 + p4);
  sum = sum + (p1 + p5);
  sum = sum + (p2 + p6);
  sum = sum + (p3 + p7);
  for (; i < n; ++i) sum = sum + xs[i] * ys[i];
  return sum;
}

}  // namespace clipgpu

using namespace clipgpu;

extern "C" int clipgpu_facade_scores(const float* embs, int64_t n, const float* query, int64_t E, float logit_scale,
                                     float logit_bias, int activation, float* out) {
  return guarded([&]() {
    if (n <= 0) throw ClipErr(CLIPGPU_ERR_INVALID, "Empty batch");
    if (E <= 0 || !embs || !query || !out) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL buffer / bad dim");
    if (activation < CLIPGPU_SIM_SOFTMAX || activation > CLIPGPU_SIM_LOGITS)
      throw ClipErr(CLIPGPU_ERR_INVALID, "bad activation");
    for (int64_t i = 0; i < n; ++i) out[i] = std::fmaf(unrolled_dot(embs + i * E, query, E), logit_scale, logit_bias);
    if (activation == CLIPGPU_SIM_SIGMOID) {
      for (int64_t i = 0; i < n; ++i) out[i] = 1.0f / (1.0f + std::exp(-out[i]));
    } else if (activation == CLIPGPU_SIM_SOFTMAX) {
      float m = -INFINITY;
      for (int64_t i = 0; i < n; ++i) m = std::fmax(m, out[i]);  // f32::max: NaN-ignoring
      float sum = -0.0f;
      for (int64_t i = 0; i < n; ++i) {
        out[i] = std::exp(out[i] - m);
        sum = sum + out[i];
      }
      for (int64_t i = 0; i < n; ++i) out[i] = out[i] / sum;
    }
  });
}
