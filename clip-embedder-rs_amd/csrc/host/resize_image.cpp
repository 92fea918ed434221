// VisionEmbedder::resize_with_image (src/vision.rs:200-233), the crate's
// non-default preprocessing path (built without the `fast_image_resize` feature, Cargo.toml:27):
//   filter: "bicubic" -> FilterType::CatmullRom, "bilinear" -> Triangle, else Nearest (:206-210)
//   "squash": image.resize_exact(S, S)                                                  (:219)
//   else:    scale = S / min(W, H) (f32); resize_exact(round(W*scale), round(H*scale)); crop_imm
//            at (round((W' - S) / 2), round((H' - S) / 2)), S x S                        (:221-228)
// resize_exact is the `image` crate 0.25.9 (Cargo.lock:1317-1318) imageops::resize, restated
// from its published sample.rs (the crate is not in this image):
//   * same size: a copy;
//   * vertical_sample to the new height into an f32 intermediate, then horizontal_sample to the
//     new width into u8 (clamp to [0, 255], f32::round);
//   * per output coordinate: ratio = in / out (f32), sratio = max(ratio, 1), support scaled by
//     sratio; centre = (o + 0.5) * ratio; taps [floor(centre - support), ceil(centre + support))
//     clamped to the image (at least one tap); weight = kernel((i - (centre - 0.5)) / sratio),
//     normalised by their f32 sum; t += pixel * w in tap order, f32 throughout;
//   * kernels: CatmullRom = cubic_bc(b 0, c 0.5) (support 2), Triangle (support 1), Nearest = box
//     (support 0: one tap, floor of the centre).
// Built with -ffp-contract=off, so no multiply-add is fused (Rust does not contract either).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/clipgpu.h"
#include "api_util.hpp"

namespace clipgpu {

namespace {

enum Filt { F_NEAREST = 0, F_TRIANGLE = 1, F_CATMULLROM = 2 };

float filt_support(int f) { return f == F_CATMULLROM ? 2.0f : (f == F_TRIANGLE ? 1.0f : 0.0f); }

// image::imageops::sample::cubic_bc(0.0, 0.5, x): a.powi(3) = a * (a * a), a.powi(2) = a * a
float catmullrom(float x) {
  const float b = 0.0f, c = 0.5f;
  const float a = std::fabs(x);
  float k;
  if (a < 1.0f) {
    k = (12.0f - 9.0f * b - 6.0f * c) * (a * (a * a)) + (-18.0f + 12.0f * b + 6.0f * c) * (a * a) + (6.0f - 2.0f * b);
  } else if (a < 2.0f) {
    k = (-b - 6.0f * c) * (a * (a * a)) + (6.0f * b + 30.0f * c) * (a * a) + (-12.0f * b - 48.0f * c) * a +
        (8.0f * b + 24.0f * c);
  } else {
    k = 0.0f;
  }
  return k / 6.0f;
}

float kernel(int f, float x) {
  if (f == F_CATMULLROM) return catmullrom(x);
  if (f == F_TRIANGLE) return std::fabs(x) < 1.0f ? 1.0f - std::fabs(x) : 0.0f;
  return 1.0f;  // box
}

struct Taps {
  std::vector<int> left, count;
  std::vector<float> w;  // count[o] weights per output, concatenated
  std::vector<int> off;
};

// The tap window and normalised weights of one axis (vertical_sample / horizontal_sample).
Taps make_taps(int in, int out, int f) {
  Taps t;
  const float ratio = (float)in / (float)out;
  const float sratio = ratio < 1.0f ? 1.0f : ratio;
  const float src_support = filt_support(f) * sratio;
  t.left.resize(out);
  t.count.resize(out);
  t.off.resize(out);
  for (int o = 0; o < out; ++o) {
    const float centre = ((float)o + 0.5f) * ratio;
    int64_t left = (int64_t)std::floor(centre - src_support);
    left = std::min<int64_t>(std::max<int64_t>(left, 0), (int64_t)in - 1);
    int64_t right = (int64_t)std::ceil(centre + src_support);
    right = std::min<int64_t>(std::max<int64_t>(right, left + 1), (int64_t)in);
    const float c = centre - 0.5f;
    t.left[o] = (int)left;
    t.count[o] = (int)(right - left);
    t.off[o] = (int)t.w.size();
    float sum = 0.0f;
    for (int64_t i = left; i < right; ++i) {
      const float w = kernel(f, ((float)i - c) / sratio);
      t.w.push_back(w);
      sum += w;
    }
    for (int64_t i = 0; i < right - left; ++i) t.w[t.off[o] + i] /= sum;
  }
  return t;
}

inline uint8_t round_clamp_u8(float v) {
  v = v < 0.0f ? 0.0f : (v > 255.0f ? 255.0f : v);
  return (uint8_t)std::round(v);  // FloatNearest: f32::round (half away from zero)
}

// imageops::resize(Rgb<u8>) -> [nh][nw][3] u8
void image_resize(const uint8_t* src, int W, int H, int nw, int nh, int f, std::vector<uint8_t>& dst) {
  dst.assign((size_t)nw * nh * 3, 0);
  if (nw == W && nh == H) {
    std::memcpy(dst.data(), src, dst.size());
    return;
  }
  // vertical_sample: [nh][W][3] f32 (the crate's Rgba32F intermediate; alpha is not used for Rgb)
  const Taps v = make_taps(H, nh, f);
  std::vector<float> tmp((size_t)nh * W * 3);
  for (int oy = 0; oy < nh; ++oy) {
    const float* w = &v.w[v.off[oy]];
    for (int x = 0; x < W; ++x) {
      float t0 = 0.0f, t1 = 0.0f, t2 = 0.0f;
      for (int i = 0; i < v.count[oy]; ++i) {
        const uint8_t* p = src + ((size_t)(v.left[oy] + i) * W + x) * 3;
        t0 += (float)p[0] * w[i];
        t1 += (float)p[1] * w[i];
        t2 += (float)p[2] * w[i];
      }
      float* o = &tmp[((size_t)oy * W + x) * 3];
      o[0] = t0;
      o[1] = t1;
      o[2] = t2;
    }
  }
  // horizontal_sample: [nh][nw][3] u8
  const Taps h = make_taps(W, nw, f);
  for (int ox = 0; ox < nw; ++ox) {
    const float* w = &h.w[h.off[ox]];
    for (int y = 0; y < nh; ++y) {
      float t0 = 0.0f, t1 = 0.0f, t2 = 0.0f;
      for (int i = 0; i < h.count[ox]; ++i) {
        const float* p = &tmp[((size_t)y * W + h.left[ox] + i) * 3];
        t0 += p[0] * w[i];
        t1 += p[1] * w[i];
        t2 += p[2] * w[i];
      }
      uint8_t* o = &dst[((size_t)y * nw + ox) * 3];
      o[0] = round_clamp_u8(t0);
      o[1] = round_clamp_u8(t1);
      o[2] = round_clamp_u8(t2);
    }
  }
}

inline uint32_t f32_to_u32_sat(float v) {  // Rust `as u32`: saturating, NaN -> 0
  if (!(v > 0.0f)) return 0;
  if (v >= 4294967296.0f) return 0xffffffffu;
  return (uint32_t)v;
}

}  // namespace

// resize_with_image (src/vision.rs:200-233) for an RGB8 image: out [S][S][3] u8.
void resize_rgb8_image_crate(const uint8_t* rgb, int W, int H, int S, const std::string& interp,
                             const std::string& mode, uint8_t* out) {
  if (!rgb || !out) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL buffer");
  if (W <= 0 || H <= 0 || S <= 0) throw ClipErr(CLIPGPU_ERR_INVALID, "Resize error: empty image");
  const int f = interp == "bicubic" ? F_CATMULLROM : (interp == "bilinear" ? F_TRIANGLE : F_NEAREST);
  std::vector<uint8_t> r;
  if (mode == "squash") {
    image_resize(rgb, W, H, S, S, f, r);
    std::memcpy(out, r.data(), r.size());
    return;
  }
  const float scale = (float)S / (float)std::min(W, H);
  const uint32_t sw = f32_to_u32_sat(std::round((float)W * scale));
  const uint32_t sh = f32_to_u32_sat(std::round((float)H * scale));
  if (sw == 0 || sh == 0) throw ClipErr(CLIPGPU_ERR_INVALID, "Resize error: empty resized image");
  image_resize(rgb, W, H, (int)sw, (int)sh, f, r);
  uint32_t x = f32_to_u32_sat(std::round(((float)sw - (float)S) / 2.0f));
  uint32_t y = f32_to_u32_sat(std::round(((float)sh - (float)S) / 2.0f));
  // crop_imm clamps the window to the image; an image smaller than S x S would make the
  // reference's normalize_pixels index past its buffer (a panic there): an error here
  x = std::min(x, sw);
  y = std::min(y, sh);
  if (sw - x < (uint32_t)S || sh - y < (uint32_t)S)
    throw ClipErr(CLIPGPU_ERR_INVALID, "Resize error: resized image smaller than the crop");
  for (int yy = 0; yy < S; ++yy)
    std::memcpy(out + (size_t)yy * S * 3, r.data() + ((size_t)(y + yy) * sw + x) * 3, (size_t)S * 3);
}

}  // namespace clipgpu
