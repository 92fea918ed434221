// Host image preprocessing: centre-crop + resize + normalise.
//
// Restates VisionEmbedder::preprocess_batch / preprocess_into /
// resize_with_fast_image_resize / normalize_pixels (src/vision.rs:119-259):
//   * crop box (f64, source pixels) unless resize_mode == "squash":
//       scale = S / min(W,H); crop_w = crop_h = S / scale;
//       crop_x = (W - crop_w) / 2; crop_y = (H - crop_h) / 2      (src/vision.rs:184-192)
//   * resampling: "bicubic" -> CatmullRom (Keys cubic, a = -0.5, support 2),
//     "bilinear" -> triangle (support 1), anything else -> nearest   (src/vision.rs:176-180)
//     as fast_image_resize 6.0.0's u8 convolution (the crate the reference's default feature
//     builds, Cargo.toml; restated from its published algorithm, a port of Pillow-SIMD's
//     Resample): per output pixel in_center = in0 + (i + 0.5) * scale, taps
//     floor(in_center - r) .. ceil(in_center + r) clamped to the image, r = support * max(scale,
//     1), weights filter((x - (in_center - 0.5)) / max(scale, 1)) divided by their sum; the
//     axis's weights become i16 fixed point at precision p (the largest p < 22 with
//     round(max weight * 2^p) < 2^15, p = 14 for a unit tap; Normalizer16), each rounded half away from zero;
//     a pass sums 2^(p-1) + pixel * k in i32 and stores clamp(sum >> p, 0, 255); horizontal
//     pass first, over the source rows the vertical pass reads, into a u8 intermediate.
//   * normalize_pixels: out[c][i] = (px[i*3+c] / 255 - mean[c]) / std[c]   in f32
//     (src/vision.rs:235-259; divide, not reciprocal-multiply).
// Parity: bit-exact vs oracle/preprocess_ref.py (the same restatement in Python); vs Pillow 12.2
// within 1 u8 level (Pillow's 22-bit coefficients, f32 crop box).  The crate itself cannot be
// built here (no Rust toolchain), so the restatement is pinned by its published algorithm.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/clipgpu.h"
#include "api_util.hpp"
#include "resize_plan.hpp"

namespace clipgpu {

namespace {

double bicubic_filter(double x) {  // Keys cubic, a = -0.5 (CatmullRom)
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}
double bilinear_filter(double x) {
  if (x < 0.0) x = -x;
  if (x < 1.0) return 1.0 - x;
  return 0.0;
}

// Rust's f64::round (half away from zero) then `as i16` (saturating).
int32_t round_i16(double v) {
  const double r = std::round(v);
  return (int32_t)std::min(32767.0, std::max(-32768.0, r));
}

// precompute_coefficients + Normalizer16::new of fast_image_resize (header above).
AxisPlan precompute(int in_size, double in0, double in1, int out_size, double (*filter)(double), double support0) {
  AxisPlan c;
  const double scale = (in1 - in0) / out_size;
  const double filter_scale = scale < 1.0 ? 1.0 : scale;
  const double radius = support0 * filter_scale;
  const double recip = 1.0 / filter_scale;
  c.ksize = (int)std::ceil(radius) * 2 + 1;
  c.bounds.resize((size_t)out_size * 2);
  std::vector<double> w((size_t)out_size * c.ksize, 0.0);
  for (int xx = 0; xx < out_size; ++xx) {
    const double in_center = in0 + (xx + 0.5) * scale;
    const int xmin = (int)std::max(std::floor(in_center - radius), 0.0);
    const int xmax = std::min((int)std::ceil(in_center + radius), in_size);
    const double center = in_center - 0.5;
    double* wx = &w[(size_t)xx * c.ksize];
    double ww = 0.0;
    for (int x = xmin; x < xmax; ++x) {
      wx[x - xmin] = filter(((double)x - center) * recip);
      ww += wx[x - xmin];
    }
    if (ww != 0.0)
      for (int x = 0; x < xmax - xmin; ++x) wx[x] /= ww;
    c.bounds[(size_t)xx * 2] = xmin;
    c.bounds[(size_t)xx * 2 + 1] = xmax - xmin;
  }
  double wmax = 0.0;
  bool first = true;
  for (double v : w)
    if (first || v > wmax) {
      wmax = v;
      first = false;
    }
  int prec = 0;
  for (int p = 0; p < kResizeMaxPrecision; ++p) {
    prec = p;
    if ((int64_t)std::round(wmax * (double)(1 << (p + 1))) >= (1 << kResizeCoefBits)) break;
  }
  c.prec = prec;
  c.k.resize(w.size());
  const double sc = (double)(1 << prec);
  for (size_t i = 0; i < w.size(); ++i) c.k[i] = round_i16(w[i] * sc);
  return c;
}

// Nearest: output i reads input index floor(in0 + (i + 0.5) * scale), clamped.
AxisPlan nearest_axis(int in_size, double in0, double in1, int out_size) {
  AxisPlan c;
  c.ksize = 1;
  c.bounds.resize((size_t)out_size * 2);
  c.k.assign((size_t)out_size, 1 << c.prec);
  const double sc = (in1 - in0) / out_size;
  for (int i = 0; i < out_size; ++i) {
    int x = (int)(in0 + (i + 0.5) * sc);
    x = std::min(std::max(x, 0), in_size - 1);
    c.bounds[(size_t)i * 2] = x;
    c.bounds[(size_t)i * 2 + 1] = 1;
  }
  return c;
}

inline uint8_t clip8(int32_t in, int prec) {
  const int32_t q = in >> prec;  // arithmetic shift (i32, as the crate)
  return (uint8_t)(q < 0 ? 0 : (q > 255 ? 255 : q));
}

}  // namespace

namespace {
ResizePlan compute_resize_plan(int W, int H, int S, const std::string& interp, const std::string& mode);
}

// Plans depend only on (W, H, S, interpolation, mode), and a batch of photos repeats a few sizes: the
// tables are computed once per key (f64 filter weights and the precision search were ~40 us per image,
// ~10 ms of a 256-image 640x480 call before round 6) and copied out of a small process-wide cache.
ResizePlan make_resize_plan(int W, int H, int S, const std::string& interp, const std::string& mode) {
  if (W <= 0 || H <= 0 || S <= 0) throw ClipErr(CLIPGPU_ERR_INVALID, "Resize error: empty image");
  struct Key {
    int W, H, S;
    std::string interp, mode;
    bool operator==(const Key& o) const {
      return W == o.W && H == o.H && S == o.S && interp == o.interp && mode == o.mode;
    }
  };
  static std::mutex mu;
  static std::vector<std::pair<Key, ResizePlan>> cache;  // most recent last; a handful of sizes
  const Key k{W, H, S, interp, mode};
  {
    std::lock_guard<std::mutex> lk(mu);
    for (size_t i = cache.size(); i-- > 0;)
      if (cache[i].first == k) return cache[i].second;
  }
  ResizePlan p = compute_resize_plan(W, H, S, interp, mode);
  std::lock_guard<std::mutex> lk(mu);
  if (cache.size() >= 64) cache.erase(cache.begin());
  cache.emplace_back(k, p);
  return p;
}

namespace {
ResizePlan compute_resize_plan(int W, int H, int S, const std::string& interp, const std::string& mode) {
  double x0 = 0, y0 = 0, x1 = W, y1 = H;
  if (mode != "squash") {  // src/vision.rs:184-192
    const double scale = (double)S / (double)std::min(W, H);
    const double cw = (double)S / scale, chh = (double)S / scale;
    x0 = ((double)W - cw) / 2.0;
    y0 = ((double)H - chh) / 2.0;
    x1 = x0 + cw;
    y1 = y0 + chh;
    // f64 round-off can place the box ~1e-14 outside the image (e.g. 517x389 -> 224): clamp.
    x0 = std::max(0.0, x0);
    y0 = std::max(0.0, y0);
    x1 = std::min((double)W, x1);
    y1 = std::min((double)H, y1);
  }
  ResizePlan p;
  p.W = W;
  p.H = H;
  p.S = S;
  if (interp == "bicubic" || interp == "bilinear") {
    double (*f)(double) = interp == "bicubic" ? bicubic_filter : bilinear_filter;
    const double support = interp == "bicubic" ? 2.0 : 1.0;
    p.h = precompute(W, x0, x1, S, f, support);
    p.v = precompute(H, y0, y1, S, f, support);
    p.need_h = S != W || x0 != 0.0 || x1 != (double)S;
    p.need_v = S != H || y0 != 0.0 || y1 != (double)S;
  } else {  // "nearest" and anything else (src/vision.rs:176-180)
    p.h = nearest_axis(W, x0, x1, S);
    p.v = nearest_axis(H, y0, y1, S);
    p.need_h = p.need_v = true;
  }
  p.yfirst = 0;
  p.th = H;
  if (p.need_h) {  // the horizontal pass only produces the rows the vertical pass reads
    p.yfirst = p.v.bounds[0];
    int ylast = 0;
    for (int i = 0; i < S; ++i) ylast = std::max(ylast, p.v.bounds[(size_t)i * 2] + p.v.bounds[(size_t)i * 2 + 1]);
    p.th = ylast - p.yfirst;
    for (int i = 0; i < S; ++i) p.v.bounds[(size_t)i * 2] -= p.yfirst;
  }
  return p;
}
}  // namespace

void apply_resize_plan(const ResizePlan& p, const uint8_t* src, uint8_t* dst) {
  const int S = p.S, W = p.W;
  std::vector<uint8_t> tmp;
  const uint8_t* vin = src;
  int vin_w = W;
  if (p.need_h) {
    tmp.resize((size_t)S * p.th * 3);
    for (int yy = 0; yy < p.th; ++yy) {
      const uint8_t* row = src + (size_t)(yy + p.yfirst) * W * 3;
      for (int xx = 0; xx < S; ++xx) {
        const int xmin = p.h.bounds[(size_t)xx * 2], cnt = p.h.bounds[(size_t)xx * 2 + 1];
        const int32_t* k = &p.h.k[(size_t)xx * p.h.ksize];
        int32_t s0 = 1 << (p.h.prec - 1), s1 = s0, s2 = s0;
        for (int x = 0; x < cnt; ++x) {
          const uint8_t* q = row + (size_t)(x + xmin) * 3;
          s0 += (int32_t)q[0] * k[x];
          s1 += (int32_t)q[1] * k[x];
          s2 += (int32_t)q[2] * k[x];
        }
        uint8_t* o = &tmp[((size_t)yy * S + xx) * 3];
        o[0] = clip8(s0, p.h.prec);
        o[1] = clip8(s1, p.h.prec);
        o[2] = clip8(s2, p.h.prec);
      }
    }
    vin = tmp.data();
    vin_w = S;
  }
  if (p.need_v) {
    for (int yy = 0; yy < S; ++yy) {
      const int ymin = p.v.bounds[(size_t)yy * 2], cnt = p.v.bounds[(size_t)yy * 2 + 1];
      const int32_t* k = &p.v.k[(size_t)yy * p.v.ksize];
      for (int xx = 0; xx < S; ++xx) {
        int32_t s0 = 1 << (p.v.prec - 1), s1 = s0, s2 = s0;
        for (int y = 0; y < cnt; ++y) {
          const uint8_t* q = vin + ((size_t)(y + ymin) * vin_w + xx) * 3;
          s0 += (int32_t)q[0] * k[y];
          s1 += (int32_t)q[1] * k[y];
          s2 += (int32_t)q[2] * k[y];
        }
        uint8_t* o = dst + ((size_t)yy * S + xx) * 3;
        o[0] = clip8(s0, p.v.prec);
        o[1] = clip8(s1, p.v.prec);
        o[2] = clip8(s2, p.v.prec);
      }
    }
  } else {
    for (int yy = 0; yy < S; ++yy) std::memcpy(dst + (size_t)yy * S * 3, vin + (size_t)yy * vin_w * 3, (size_t)S * 3);
  }
}

// resize_image.cpp: resize_with_image (src/vision.rs:200-233), the non-default resize
void resize_rgb8_image_crate(const uint8_t* rgb, int W, int H, int S, const std::string& interp,
                             const std::string& mode, uint8_t* out);

namespace {

void resize_rgb8(const uint8_t* rgb, int W, int H, int S, const std::string& interp, const std::string& mode,
                 uint8_t* out) {
  if (!rgb || !out) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL buffer");
  apply_resize_plan(make_resize_plan(W, H, S, interp, mode), rgb, out);
}

void normalize_pixels(const uint8_t* px, int S, const float* mean, const float* stdv, float* out) {
  const size_t n = (size_t)S * S;
  for (int c = 0; c < 3; ++c) {
    float* o = out + c * n;
    for (size_t i = 0; i < n; ++i) {
      const float val = (float)px[i * 3 + c] / 255.0f;
      o[i] = (val - mean[c]) / stdv[c];
    }
  }
}

// image_crate: resize with resize_with_image (the crate built without `fast_image_resize`)
// instead of the default resize_with_fast_image_resize (src/vision.rs:149-157).
void preprocess_one(const uint8_t* rgb, int W, int H, int S, const std::string& interp, const std::string& mode,
                    const float* mean, const float* stdv, float* out, bool image_crate = false) {
  std::vector<uint8_t> resized((size_t)S * S * 3);
  if (image_crate) resize_rgb8_image_crate(rgb, W, H, S, interp, mode, resized.data());
  else resize_rgb8(rgb, W, H, S, interp, mode, resized.data());
  normalize_pixels(resized.data(), S, mean, stdv, out);
}

void preprocess_batch(const uint8_t* const* images, const int* widths, const int* heights, int64_t n, int size,
                      const char* interpolation, const char* resize_mode, const float* mean, const float* stdv,
                      float* out, bool image_crate) {
  if (n <= 0) throw ClipErr(CLIPGPU_ERR_INVALID, "Empty batch");  // src/vision.rs:121-123
  if (!images || !widths || !heights || !mean || !stdv || !out) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL buffer");
  const std::string interp = interpolation ? interpolation : "bicubic";
  const std::string mode = resize_mode ? resize_mode : "shortest";
  const size_t per = (size_t)3 * size * size;
  unsigned nt = std::thread::hardware_concurrency();
  if (nt == 0) nt = 1;
  nt = (unsigned)std::min<int64_t>(nt, 16);
  nt = (unsigned)std::min<int64_t>(nt, n);
  std::vector<std::thread> th;
  std::vector<std::string> errs(nt);
  for (unsigned t = 0; t < nt; ++t) {
    th.emplace_back([&, t]() {
      try {
        for (int64_t i = t; i < n; i += nt)
          preprocess_one(images[i], widths[i], heights[i], size, interp, mode, mean, stdv, out + i * per,
                         image_crate);
      } catch (const std::exception& ex) {
        errs[t] = ex.what();
      }
    });
  }
  for (auto& x : th) x.join();
  for (auto& e : errs)
    if (!e.empty()) throw ClipErr(CLIPGPU_ERR_INVALID, e);
}

}  // namespace
}  // namespace clipgpu

using namespace clipgpu;

extern "C" {

int clipgpu_resize_rgb8(const uint8_t* rgb, int width, int height, int size, const char* interpolation,
                        const char* resize_mode, uint8_t* out_rgb) {
  return guarded([&]() {
    resize_rgb8(rgb, width, height, size, interpolation ? interpolation : "bicubic",
                resize_mode ? resize_mode : "shortest", out_rgb);
  });
}

int clipgpu_preprocess_rgb8(const uint8_t* rgb, int width, int height, int size, const char* interpolation,
                            const char* resize_mode, const float mean[3], const float stdv[3], float* out_chw) {
  return guarded([&]() {
    if (!mean || !stdv || !out_chw) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL buffer");
    preprocess_one(rgb, width, height, size, interpolation ? interpolation : "bicubic",
                   resize_mode ? resize_mode : "shortest", mean, stdv, out_chw);
  });
}

int clipgpu_preprocess_batch(const uint8_t* const* images, const int* widths, const int* heights, int64_t n,
                             int size, const char* interpolation, const char* resize_mode, const float mean[3],
                             const float stdv[3], float* out) {
  return guarded([&]() {
    preprocess_batch(images, widths, heights, n, size, interpolation, resize_mode, mean, stdv, out, false);
  });
}

int clipgpu_resize_rgb8_image(const uint8_t* rgb, int width, int height, int size, const char* interpolation,
                              const char* resize_mode, uint8_t* out_rgb) {
  return guarded([&]() {
    resize_rgb8_image_crate(rgb, width, height, size, interpolation ? interpolation : "bicubic",
                            resize_mode ? resize_mode : "shortest", out_rgb);
  });
}

int clipgpu_preprocess_batch_image(const uint8_t* const* images, const int* widths, const int* heights, int64_t n,
                                   int size, const char* interpolation, const char* resize_mode, const float mean[3],
                                   const float stdv[3], float* out) {
  return guarded([&]() {
    preprocess_batch(images, widths, heights, n, size, interpolation, resize_mode, mean, stdv, out, true);
  });
}

}  // extern "C"
