// GPU crop + resize of decoded RGB8 images of any size to the model's S x S
// (a5 on the device: resize_with_fast_image_resize, src/vision.rs:164-198).
//
// The coefficients come from the host's make_resize_plan (csrc/host/resize_plan.hpp),
// the same fixed-point tables the host resize applies, so the output is bit-identical
// to the host path: a separable convolution, horizontal pass into a u8 intermediate
// holding only the source rows the vertical pass reads, then the vertical pass into
// u8 NHWC [n][S][S][3] -- the input of the u8 embedding path, which normalises
// (normalize_pixels) while staging the patch rows.  fast_image_resize's integer rounding
// (resize_plan.hpp): 2^(p-1) + sum(pixel * k) in i32, clamp(sum >> p, 0, 255), p per axis.
//
// One thread = one output pixel (3 channels); grid.y = image.  Memory-bound: a
// 224 x 224 output reads its source rows once per tap column, from L2.
#include "common.hpp"
#include "kernels.hpp"

namespace clipgpu {

namespace {

__device__ __forceinline__ uint8_t clip8(int v, int prec) {
  const int q = v >> prec;  // arithmetic shift, as the crate's i32 `>>`
  return (uint8_t)(q < 0 ? 0 : (q > 255 ? 255 : q));
}

__global__ __launch_bounds__(256) void resize_h_kernel(const uint8_t* __restrict__ raw, uint8_t* __restrict__ tmp,
                                                       const int* __restrict__ ints,
                                                       const ResizeImage* __restrict__ imgs, int S) {
  const ResizeImage d = imgs[blockIdx.y];
  if (!d.need_h) return;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)d.th * S) return;
  const int yy = (int)(t / S), xx = (int)(t - (long)yy * S);
  const int* b = ints + d.h_bounds + 2 * xx;
  const int xmin = b[0], cnt = b[1];
  const int* k = ints + d.h_coef + (long)xx * d.h_ksize;
  const uint8_t* row = raw + d.src + ((long)(yy + d.yfirst) * d.W + xmin) * 3;
  int s0 = 1 << (d.h_prec - 1), s1 = s0, s2 = s0;
  for (int x = 0; x < cnt; ++x) {
    const int kx = k[x];
    s0 += (int)row[3 * x] * kx;
    s1 += (int)row[3 * x + 1] * kx;
    s2 += (int)row[3 * x + 2] * kx;
  }
  uint8_t* o = tmp + d.tmp + t * 3;
  o[0] = clip8(s0, d.h_prec);
  o[1] = clip8(s1, d.h_prec);
  o[2] = clip8(s2, d.h_prec);
}

__global__ __launch_bounds__(256) void resize_v_kernel(const uint8_t* __restrict__ raw,
                                                       const uint8_t* __restrict__ tmp, const int* __restrict__ ints,
                                                       const ResizeImage* __restrict__ imgs, uint8_t* __restrict__ out,
                                                       int S) {
  const ResizeImage d = imgs[blockIdx.y];
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)S * S) return;
  const int yy = (int)(t / S), xx = (int)(t - (long)yy * S);
  // pass input: the horizontal pass output [th][S] or the source itself (W == S)
  const uint8_t* in = d.need_h ? tmp + d.tmp : raw + d.src;
  const int in_w = d.need_h ? S : d.W;
  uint8_t* o = out + ((long)blockIdx.y * S * S + t) * 3;
  if (!d.need_v) {
    const uint8_t* q = in + ((long)yy * in_w + xx) * 3;
    o[0] = q[0];
    o[1] = q[1];
    o[2] = q[2];
    return;
  }
  const int* b = ints + d.v_bounds + 2 * yy;
  const int ymin = b[0], cnt = b[1];
  const int* k = ints + d.v_coef + (long)yy * d.v_ksize;
  const uint8_t* col = in + ((long)ymin * in_w + xx) * 3;
  const long stride = (long)in_w * 3;
  int s0 = 1 << (d.v_prec - 1), s1 = s0, s2 = s0;
  for (int y = 0; y < cnt; ++y) {
    const int ky = k[y];
    const uint8_t* q = col + y * stride;
    s0 += (int)q[0] * ky;
    s1 += (int)q[1] * ky;
    s2 += (int)q[2] * ky;
  }
  o[0] = clip8(s0, d.v_prec);
  o[1] = clip8(s1, d.v_prec);
  o[2] = clip8(s2, d.v_prec);
}

}  // namespace

hipError_t launch_resize(const uint8_t* raw, uint8_t* tmp, const int* ints, const ResizeImage* d_imgs, int n,
                         int max_th, int S, uint8_t* out, hipStream_t s) {
  if (n <= 0 || S <= 0 || n > 65535) return hipErrorInvalidValue;
  if (max_th > 0) {
    const long px = (long)max_th * S;
    hipLaunchKernelGGL(resize_h_kernel, dim3((unsigned)((px + 255) / 256), n), dim3(256), 0, s, raw, tmp, ints,
                       d_imgs, S);
  }
  const long px = (long)S * S;
  hipLaunchKernelGGL(resize_v_kernel, dim3((unsigned)((px + 255) / 256), n), dim3(256), 0, s, raw, tmp, ints, d_imgs,
                     out, S);
  return hipGetLastError();
}

}  // namespace clipgpu
