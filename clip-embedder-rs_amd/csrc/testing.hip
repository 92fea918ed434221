// Kernel-level test hooks (include/clipgpu_testing.h): each runs one kernel on
// device 0 over host f32 buffers so tests/ can check it against numpy.
#include <hip/hip_runtime.h>

#include <chrono>
#include <csignal>
#include <cstdio>
#include <dlfcn.h>
#include <execinfo.h>
#include <unistd.h>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <vector>

#include "../../include/clipgpu.h"
#include "../../include/clipgpu_testing.h"
#include "bounce.hpp"
#include "host/copy_pool.hpp"
#include "host/api_util.hpp"
#include "kernels/common.hpp"
#include "kernels/kernels.hpp"

using namespace clipgpu;

namespace {

#define TCHECK(expr)                                                                                  \
  do {                                                                                                \
    hipError_t _e = (expr);                                                                           \
    if (_e != hipSuccess) throw ClipErr(CLIPGPU_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  explicit DevBuf(size_t n) {
    TCHECK(hipMalloc(&p, n ? n : 16));
    TCHECK(hipMemset(p, 0, n ? n : 16));
  }
  ~DevBuf() { (void)hipFree(p); }
  template <typename T> T* as() const { return (T*)p; }
};

DType dt_of(int dtype) {
  if (dtype != CLIPGPU_DTYPE_BF16 && dtype != CLIPGPU_DTYPE_F16) throw ClipErr(CLIPGPU_ERR_INVALID, "bad dtype");
  return dtype == CLIPGPU_DTYPE_BF16 ? DT_BF16 : DT_F16;
}

// CLIPGPU_TEST_TILE forces a GEMM tile in the kernel-level test hooks below (tile-config coverage; the
// engine itself reads no environment): a built GemmTile id (kernels.hpp kGemmTiles), 0 auto, 100 skinny;
// the MX hooks take MxTile ids.
int tile_override() {
  const char* e = getenv("CLIPGPU_TEST_TILE");
  const int t = e ? atoi(e) : 0;
  if (t != 0 && t != TILE_SKINNY && t != TILE_GENERAL && !gemm_tile_built(t))
    throw ClipErr(CLIPGPU_ERR_INVALID, "CLIPGPU_TEST_TILE: " + std::to_string(t) + " is not a built GEMM tile");
  return t;
}

// One wave: sleep-poll s_memrealtime (100 MHz) for `ticks`, counting shader clocks (s_memtime) over the
// same span.  Lanes 0 / 1 store the two counts (vector stores of lane-dependent addresses).
__global__ void clock_probe_kernel(unsigned long long* out, unsigned long long ticks) {
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r = r0;
  while (r - r0 < ticks) {
    __builtin_amdgcn_s_sleep(32);
    r = __builtin_amdgcn_s_memrealtime();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const int lane = threadIdx.x;
  if (lane < 2) out[lane] = lane == 0 ? t1 - t0 : r - r0;
}

void up(void* d, const void* h, size_t n) { TCHECK(copy_h2d(d, h, n)); }
void down(void* h, const void* d, size_t n) { TCHECK(copy_d2h(h, d, n)); }

// f32 host -> 16-bit device
void up16(DType dt, void* d16, const float* h, size_t n) {
  DevBuf tmp(n * 4);
  up(tmp.p, h, n * 4);
  TCHECK(launch_cast_f32(dt, tmp.as<float>(), d16, (long)n, nullptr));
  TCHECK(hipDeviceSynchronize());
}

template <typename T>
__global__ void widen(const T* in, float* out, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = (float)in[i];
}

void down16(DType dt, float* h, const void* d16, size_t n) {
  DevBuf tmp(n * 4);
  if (dt == DT_BF16) hipLaunchKernelGGL(widen<__bf16>, dim3(1024), dim3(256), 0, nullptr, (const __bf16*)d16, tmp.as<float>(), (long)n);
  else hipLaunchKernelGGL(widen<_Float16>, dim3(1024), dim3(256), 0, nullptr, (const _Float16*)d16, tmp.as<float>(), (long)n);
  TCHECK(hipGetLastError());
  TCHECK(hipDeviceSynchronize());
  down(h, tmp.p, n * 4);
}

}  // namespace

extern "C" {

int clipgpu_test_gemm(int dtype, int mode, int act, int64_t M, int64_t N, int64_t K, const float* A, const float* W,
                      const float* bias, const float* resid, float* out) {
  return guarded([&]() {
    const DType dt = dt_of(dtype);
    if (M <= 0 || N <= 0 || K <= 0 || K % 64) throw ClipErr(CLIPGPU_ERR_INVALID, "bad GEMM shape (K % 64 == 0)");
    DevBuf dA(M * K * 2), dW(N * K * 2), dB(N * 4), dO(M * N * 4);
    up16(dt, dA.p, A, M * K);
    up16(dt, dW.p, W, N * K);
    if (bias) up(dB.p, bias, N * 4);
    GemmParams g{};
    g.tile = tile_override();
    g.A = dA.p; g.lda = K; g.W = dW.p; g.ldw = K; g.bias = bias ? dB.as<float>() : nullptr;
    g.out = dO.p; g.ldo = N; g.M = (int)M; g.N = (int)N; g.K = (int)K;
    int epi = EPI_STORE16;
    if (mode == 1) {
      epi = EPI_RESID;
      if (resid) up(dO.p, resid, M * N * 4);
    } else if (mode == 2) {
      epi = EPI_STORE32;
    } else if (mode == 3) {  // the f16 residual stream (GemmParams.x16)
      epi = EPI_RESID;
      g.x16 = 1;
      if (resid) up16(DT_F16, dO.p, resid, M * N);
    } else if (mode != 0) {
      throw ClipErr(CLIPGPU_ERR_INVALID, "bad mode");
    }
    TCHECK(launch_gemm(dt, A_ROWS, epi, mode == 0 ? act : 0, g, nullptr));
    TCHECK(hipDeviceSynchronize());
    if (mode == 0) down16(dt, out, dO.p, M * N);
    else if (mode == 3) down16(DT_F16, out, dO.p, M * N);
    else down(out, dO.p, M * N * 4);
  });
}

int clipgpu_test_gemm_chunk_rows(int64_t rows) {
  return guarded([&]() {
    if (rows < 0) throw ClipErr(CLIPGPU_ERR_INVALID, "rows < 0");
    g_gemm_chunk_cap = (long)rows;
  });
}

int clipgpu_test_gemm_lnf(int dtype, int act, int64_t M, int64_t N, int64_t K, const float* x, const float* wf,
                          const float* cs, const float* bias, float eps, int tile, float* out) {
  return guarded([&]() {
    const DType dt = dt_of(dtype);
    if (M <= 0 || N <= 0 || K <= 0 || K % 64 || N % 4) throw ClipErr(CLIPGPU_ERR_INVALID, "bad GEMM shape");
    if (tile != 0 && tile != TILE_SKINNY && tile != TILE_GENERAL && !gemm_tile_built(tile))
      throw ClipErr(CLIPGPU_ERR_INVALID, "bad tile");
    DevBuf dA(M * K * 2), dW(N * K * 2), dB(N * 4), dC(N * 4), dO(M * N * 2), dS((M + 256) * 8);
    up16(DT_F16, dA.p, x, M * K);
    up16(DT_F16, dW.p, wf, N * K);
    up(dB.p, bias, N * 4);
    up(dC.p, cs, N * 4);
    TCHECK(launch_ln_stats(dA.p, 1, eps, dS.as<float>(), (int)M, (int)K, nullptr));  // the rows' (mean, rstd)
    GemmParams g{};
    g.tile = tile;
    g.A = dA.p; g.lda = K; g.W = dW.p; g.ldw = K; g.bias = dB.as<float>(); g.cs = dC.as<float>();
    g.rowstats = dS.as<float>();
    g.out = dO.p; g.ldo = N; g.M = (int)M; g.N = (int)N; g.K = (int)K;
    TCHECK(launch_gemm(dt, A_ROWS, EPI_LNF, act, g, nullptr));
    TCHECK(hipDeviceSynchronize());
    down16(dt, out, dO.p, M * N);
  });
}

int clipgpu_test_attention(int dtype, int64_t B, int64_t N, int64_t H, int64_t HD, int causal, const float* qkv,
                           float* out) {
  return guarded([&]() {
    const DType dt = dt_of(dtype);
    const int64_t D = H * HD;
    DevBuf dq(B * N * 3 * D * 2), dO(B * N * D * 2);
    up16(dt, dq.p, qkv, B * N * 3 * D);
    TCHECK(launch_attention(dt, dq.p, dO.p, (int)B, (int)N, (int)H, (int)D, causal, nullptr));
    TCHECK(hipDeviceSynchronize());
    down16(dt, out, dO.p, B * N * D);
  });
}

int clipgpu_test_layernorm(int dtype, int64_t rows, int64_t D, float eps, const float* x, const float* w,
                           const float* b, float* out) {
  return guarded([&]() {
    const DType dt = dt_of(dtype);
    DevBuf dx(rows * D * 4), dw(D * 4), db(D * 4), dO(rows * D * 2);
    up(dx.p, x, rows * D * 4);
    up(dw.p, w, D * 4);
    up(db.p, b, D * 4);
    TCHECK(launch_ln_rows(dt, dx.as<float>(), 0, dw.as<float>(), db.as<float>(), eps, dO.p, (int)rows, (int)D, nullptr));
    TCHECK(hipDeviceSynchronize());
    down16(dt, out, dO.p, rows * D);
  });
}

int clipgpu_test_patch_embed(int dtype, int mode, int64_t B, int64_t S, int64_t P, int64_t D, const void* pixels,
                             const float mean[3], const float stdv[3], const float* conv_w, const float* pos,
                             float* x_out) {
  return guarded([&]() {
    const DType dt = dt_of(dtype);
    const int64_t G = S / P, K = 3 * P * P, Kp = (K + 63) / 64 * 64, tokens = G * G + 1;
    const size_t pix_bytes = mode == 0 ? (size_t)B * 3 * S * S * 4 : (size_t)B * S * S * 3;
    DevBuf dpix(pix_bytes), dw(D * Kp * 2), dpos(tokens * D * 4), dx(B * tokens * D * 4);
    up(dpix.p, pixels, pix_bytes);
    std::vector<float> wpad((size_t)(D * Kp), 0.f);  // conv weight zero-padded to K % 64 == 0 (as the engine does)
    for (int64_t r = 0; r < D; ++r)
      for (int64_t k = 0; k < K; ++k) wpad[(size_t)(r * Kp + k)] = conv_w[r * K + k];
    up16(dt, dw.p, wpad.data(), D * Kp);
    up(dpos.p, pos, tokens * D * 4);
    // the engine's stem: patch rows (16-bit) -> row GEMM with the patch epilogue
    DevBuf drows(B * G * G * Kp * 2);
    TCHECK(launch_patch_rows(dt, mode == 0 ? A_IMG_F32 : A_IMG_U8, dpix.p, mean, stdv, drows.p, (int)B, (int)S,
                             (int)P, (int)K, (int)Kp, nullptr));
    GemmParams g{};
    g.A = drows.p; g.lda = Kp;
    g.W = dw.p; g.ldw = Kp; g.out = dx.p; g.ldo = D; g.M = (int)(B * G * G); g.N = (int)D; g.K = (int)Kp;
    g.cls = 1;
    g.G = (int)G; g.pos = dpos.as<float>();
    g.tile = tile_override();
    TCHECK(launch_gemm(dt, A_ROWS, EPI_PATCH, 0, g, nullptr));
    TCHECK(hipDeviceSynchronize());
    down(x_out, dx.p, B * tokens * D * 4);
  });
}

int clipgpu_test_patch_rows(int dtype, int mode, int64_t B, int64_t S, int64_t P, const void* pixels,
                            const float mean[3], const float stdv[3], float* rows_out) {
  return guarded([&]() {
    const DType dt = dt_of(dtype);
    const int64_t G = S / P, K = 3 * P * P, Kp = (K + 63) / 64 * 64;
    const size_t pix_bytes = mode == 0 ? (size_t)B * 3 * S * S * 4 : (size_t)B * S * S * 3;
    DevBuf dpix(pix_bytes), drows(B * G * G * Kp * 2);
    up(dpix.p, pixels, pix_bytes);
    TCHECK(launch_patch_rows(dt, mode == 0 ? A_IMG_F32 : A_IMG_U8, dpix.p, mean, stdv, drows.p, (int)B, (int)S,
                             (int)P, (int)K, (int)Kp, nullptr));
    TCHECK(hipDeviceSynchronize());
    down16(dt, rows_out, drows.p, B * G * G * Kp);
  });
}

namespace {
__global__ void fill_random(float* out, long n, uint32_t seed) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint32_t z = (uint32_t)i * 2654435761u ^ seed;
    z ^= z >> 15; z *= 2246822519u; z ^= z >> 13; z *= 3266489917u; z ^= z >> 16;
    out[i] = ((float)(z >> 8) * (1.0f / 16777216.0f)) * 2.0f - 1.0f;
  }
}
}  // namespace

namespace {
__global__ void lane_reduce_kernel(const float* in, float* out) {
  const int l = threadIdx.x;
  const float v = in[l];
  out[0 * 64 + l] = wave_sum(v);
  out[1 * 64 + l] = wave_max(v);
  out[2 * 64 + l] = xsum16(v);
  out[3 * 64 + l] = xsum32(v);
  out[4 * 64 + l] = group16_sum(v);
  out[5 * 64 + l] = group16_max(v);
  float a = v, b = v;
  swap16(a, b);
  out[6 * 64 + l] = a;
  out[7 * 64 + l] = b;
}
}  // namespace

int clipgpu_test_lane_reduce(const float* in64, float* out512) {
  return guarded([&]() {
    DevBuf di(64 * 4), dO(512 * 4);
    up(di.p, in64, 64 * 4);
    hipLaunchKernelGGL(lane_reduce_kernel, dim3(1), dim3(64), 0, nullptr, di.as<float>(), dO.as<float>());
    TCHECK(hipGetLastError());
    TCHECK(hipDeviceSynchronize());
    down(out512, dO.p, 512 * 4);
  });
}

int clipgpu_test_clock_probe(void* stream, int64_t duration_us, uint64_t* d_out) {
  return guarded([&]() {
    if (!d_out || duration_us <= 0 || duration_us > 10000000) throw ClipErr(CLIPGPU_ERR_INVALID, "bad clock probe");
    hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (unsigned long long*)d_out,
                       (unsigned long long)duration_us * 100ull);
    TCHECK(hipGetLastError());
  });
}

int clipgpu_test_gemm_grid(int tile, int64_t M, int64_t N, int64_t K, int* grid) {
  return guarded([&]() {
    if (M <= 0 || N <= 0 || K <= 0 || K % 64 || !grid || M > INT32_MAX || N > INT32_MAX || K > INT32_MAX)
      throw ClipErr(CLIPGPU_ERR_INVALID, "bad GEMM grid arguments");
    if (tile != 0 && tile != TILE_SKINNY && !gemm_tile_built(tile)) throw ClipErr(CLIPGPU_ERR_INVALID, "not a built tile");
    *grid = gemm_grid(tile, (int)M, (int)N, (int)K);
  });
}

int clipgpu_test_gemm_bench(int dtype, int epi, int act, int64_t M, int64_t N, int64_t K, int tile, int iters,
                            double* us_per_launch) {
  return clipgpu_test_gemm_bench_ld(dtype, epi, act, M, N, K, K, K, tile, iters, us_per_launch);
}

int clipgpu_test_gemm_bench_ld(int dtype, int epi, int act, int64_t M, int64_t N, int64_t K, int64_t lda,
                               int64_t ldw, int tile, int iters, double* us_per_launch) {
  return guarded([&]() {
    const DType dt = dt_of(dtype);
    if (M <= 0 || N <= 0 || K <= 0 || K % 64 || iters <= 0 || !us_per_launch || lda < K || ldw < K ||
        lda % 8 || ldw % 8)
      throw ClipErr(CLIPGPU_ERR_INVALID, "bad GEMM bench arguments");
    // A [M][lda], W [N][ldw] (row pitch in elements; the pad columns hold random values the GEMM
    // never reads)
    DevBuf fA(M * lda * 4), fW(N * ldw * 4), dA(M * lda * 2), dW(N * ldw * 2), dB(N * 4), dO(M * N * 4);
    hipLaunchKernelGGL(fill_random, dim3(2048), dim3(256), 0, nullptr, fA.as<float>(), (long)(M * lda), 1u);
    hipLaunchKernelGGL(fill_random, dim3(2048), dim3(256), 0, nullptr, fW.as<float>(), (long)(N * ldw), 2u);
    hipLaunchKernelGGL(fill_random, dim3(64), dim3(256), 0, nullptr, dB.as<float>(), (long)N, 3u);
    TCHECK(launch_cast_f32(dt, fA.as<float>(), dA.p, (long)(M * lda), nullptr));
    TCHECK(launch_cast_f32(dt, fW.as<float>(), dW.p, (long)(N * ldw), nullptr));
    TCHECK(hipDeviceSynchronize());
    GemmParams g{};
    g.A = dA.p; g.lda = lda; g.W = dW.p; g.ldw = ldw; g.bias = dB.as<float>();
    g.out = dO.p; g.ldo = N; g.M = (int)M; g.N = (int)N; g.K = (int)K; g.tile = tile;
    if (tile != 0 && tile != TILE_SKINNY && !gemm_tile_built(tile)) throw ClipErr(CLIPGPU_ERR_INVALID, "not a built tile");
    const int e = (epi == 1 || epi == 3) ? EPI_RESID : (epi == 2 ? EPI_STORE32 : EPI_STORE16);
    g.x16 = epi == 3;  // the f16 residual stream (its random f32 fill read as f16: timing only)
    for (int i = 0; i < 3; ++i) TCHECK(launch_gemm(dt, A_ROWS, e, epi == 0 ? act : 0, g, nullptr));
    hipEvent_t a, b;
    TCHECK(hipEventCreate(&a));
    TCHECK(hipEventCreate(&b));
    TCHECK(hipEventRecord(a, nullptr));
    for (int i = 0; i < iters; ++i) TCHECK(launch_gemm(dt, A_ROWS, e, epi == 0 ? act : 0, g, nullptr));
    TCHECK(hipEventRecord(b, nullptr));
    TCHECK(hipEventSynchronize(b));
    float ms = 0.f;
    TCHECK(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    *us_per_launch = (double)ms * 1000.0 / iters;
  });
}

int clipgpu_test_attention_bench(int dtype, int64_t B, int64_t N, int64_t H, int64_t HD, int causal, int iters,
                                 double* us_per_launch) {
  return guarded([&]() {
    const DType dt = dt_of(dtype);
    if (B <= 0 || N <= 0 || H <= 0 || iters <= 0 || !us_per_launch)
      throw ClipErr(CLIPGPU_ERR_INVALID, "bad attention bench arguments");
    const int64_t D = H * HD;
    DevBuf f(B * N * 3 * D * 4), dq(B * N * 3 * D * 2), dO(B * N * D * 2);
    hipLaunchKernelGGL(fill_random, dim3(2048), dim3(256), 0, nullptr, f.as<float>(), (long)(B * N * 3 * D), 7u);
    TCHECK(launch_cast_f32(dt, f.as<float>(), dq.p, (long)(B * N * 3 * D), nullptr));
    for (int i = 0; i < 3; ++i)
      TCHECK(launch_attention(dt, dq.p, dO.p, (int)B, (int)N, (int)H, (int)D, causal, nullptr));
    hipEvent_t a, b;
    TCHECK(hipEventCreate(&a));
    TCHECK(hipEventCreate(&b));
    TCHECK(hipEventRecord(a, nullptr));
    for (int i = 0; i < iters; ++i)
      TCHECK(launch_attention(dt, dq.p, dO.p, (int)B, (int)N, (int)H, (int)D, causal, nullptr));
    TCHECK(hipEventRecord(b, nullptr));
    TCHECK(hipEventSynchronize(b));
    float ms = 0.f;
    TCHECK(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    *us_per_launch = (double)ms * 1000.0 / iters;
  });
}

int clipgpu_test_quant_rows(int64_t rows, int64_t cols, const float* in, uint8_t* q, uint8_t* qs) {
  return guarded([&]() {
    if (rows <= 0 || cols <= 0 || cols % 32) throw ClipErr(CLIPGPU_ERR_INVALID, "bad quant shape (cols % 32 == 0)");
    DevBuf dx(rows * cols * 4), dq(rows * cols), ds(rows * cols / 32);
    up(dx.p, in, rows * cols * 4);
    TCHECK(launch_quant_rows(-1, dx.p, cols, dq.as<uint8_t>(), cols, ds.as<uint8_t>(), cols / 32, (int)rows, (int)cols,
                             nullptr));
    TCHECK(hipDeviceSynchronize());
    down(q, dq.p, rows * cols);
    down(qs, ds.p, rows * cols / 32);
  });
}

int clipgpu_test_layernorm_mx(int64_t rows, int64_t D, float eps, const float* x, const float* w, const float* b,
                              uint8_t* q, uint8_t* qs) {
  return guarded([&]() {
    if (rows <= 0 || D <= 0 || D % 32) throw ClipErr(CLIPGPU_ERR_INVALID, "bad LN shape (D % 32 == 0)");
    DevBuf dx(rows * D * 4), dw(D * 4), db(D * 4), dq(rows * D), ds(rows * D / 32);
    up(dx.p, x, rows * D * 4);
    up(dw.p, w, D * 4);
    up(db.p, b, D * 4);
    TCHECK(launch_ln_rows(DT_BF16, dx.as<float>(), 0, dw.as<float>(), db.as<float>(), eps, dq.p, (int)rows, (int)D,
                          nullptr, ds.as<uint8_t>()));
    TCHECK(hipDeviceSynchronize());
    down(q, dq.p, rows * D);
    down(qs, ds.p, rows * D / 32);
  });
}

int clipgpu_test_gemm_mx(int dtype, int mode, int act, int64_t M, int64_t N, int64_t K, const uint8_t* Aq,
                         const uint8_t* As, const uint8_t* Wq, const uint8_t* Ws, const float* bias, const float* resid,
                         float* out, uint8_t* outq, uint8_t* outs) {
  return guarded([&]() {
    const DType dt = dt_of(dtype);
    if (M <= 0 || N <= 0 || K <= 0 || K % 128 || N % 32 || mode < 0 || mode > 3)
      throw ClipErr(CLIPGPU_ERR_INVALID, "bad MX GEMM shape (K % 128 == 0, N % 32 == 0)");
    DevBuf dA(M * K), dAs(M * K / 32), dW(N * K), dWs(N * K / 32), dB(N * 4), dO(M * N * 4), dOs(M * N / 32);
    up(dA.p, Aq, M * K);
    up(dAs.p, As, M * K / 32);
    up(dW.p, Wq, N * K);
    up(dWs.p, Ws, N * K / 32);
    if (bias) up(dB.p, bias, N * 4);
    MxGemmParams g{};
    g.A = dA.as<uint8_t>(); g.lda = K; g.As = dAs.as<uint8_t>(); g.ldas = K / 32;
    g.W = dW.as<uint8_t>(); g.ldw = K; g.Ws = dWs.as<uint8_t>(); g.ldws = K / 32;
    g.bias = bias ? dB.as<float>() : nullptr;
    g.out = dO.p; g.M = (int)M; g.N = (int)N; g.K = (int)K; g.tile = tile_override();
    static const int epis[4] = {EPI_STORE16, EPI_RESID, EPI_STORE32, EPI_STOREQ};
    const int epi = epis[mode];
    g.ldo = N;
    if (epi == EPI_STOREQ) {
      g.outs = dOs.as<uint8_t>();
      g.ldos = N / 32;
    }
    if (epi == EPI_RESID && resid) up(dO.p, resid, M * N * 4);
    TCHECK(launch_gemm_mx(dt, epi, (epi == EPI_STORE16 || epi == EPI_STOREQ) ? act : 0, g, nullptr));
    TCHECK(hipDeviceSynchronize());
    if (epi == EPI_STORE16) down16(dt, out, dO.p, M * N);
    else if (epi == EPI_STOREQ) {
      down(outq, dO.p, M * N);
      down(outs, dOs.p, M * N / 32);
    } else down(out, dO.p, M * N * 4);
  });
}

int clipgpu_test_gemm_mx_bench(int epi, int act, int64_t M, int64_t N, int64_t K, int tile, int iters,
                               double* us_per_launch) {
  return guarded([&]() {
    if (M <= 0 || N <= 0 || K <= 0 || K % 128 || N % 32 || iters <= 0 || !us_per_launch || epi < 0 || epi > 3)
      throw ClipErr(CLIPGPU_ERR_INVALID, "bad MX GEMM bench arguments");
    DevBuf fA(M * K * 4), fW(N * K * 4), dA(M * K), dAs(M * K / 32), dW(N * K), dWs(N * K / 32), dB(N * 4),
        dO(M * N * 4), dOs(M * N / 32);
    hipLaunchKernelGGL(fill_random, dim3(2048), dim3(256), 0, nullptr, fA.as<float>(), (long)(M * K), 1u);
    hipLaunchKernelGGL(fill_random, dim3(2048), dim3(256), 0, nullptr, fW.as<float>(), (long)(N * K), 2u);
    hipLaunchKernelGGL(fill_random, dim3(64), dim3(256), 0, nullptr, dB.as<float>(), (long)N, 3u);
    TCHECK(launch_quant_rows(-1, fA.p, K, dA.as<uint8_t>(), K, dAs.as<uint8_t>(), K / 32, (int)M, (int)K, nullptr));
    TCHECK(launch_quant_rows(-1, fW.p, K, dW.as<uint8_t>(), K, dWs.as<uint8_t>(), K / 32, (int)N, (int)K, nullptr));
    TCHECK(hipDeviceSynchronize());
    MxGemmParams g{};
    g.A = dA.as<uint8_t>(); g.lda = K; g.As = dAs.as<uint8_t>(); g.ldas = K / 32;
    g.W = dW.as<uint8_t>(); g.ldw = K; g.Ws = dWs.as<uint8_t>(); g.ldws = K / 32;
    g.bias = dB.as<float>(); g.out = dO.p; g.ldo = N; g.M = (int)M; g.N = (int)N; g.K = (int)K; g.tile = tile;
    static const int epis[4] = {EPI_STORE16, EPI_RESID, EPI_STORE32, EPI_STOREQ};
    const int e = epis[epi];
    if (e == EPI_STOREQ) {
      g.outs = dOs.as<uint8_t>();
      g.ldos = N / 32;
    }
    const int a = (e == EPI_STORE16 || e == EPI_STOREQ) ? act : 0;
    for (int i = 0; i < 3; ++i) TCHECK(launch_gemm_mx(DT_BF16, e, a, g, nullptr));
    hipEvent_t ea, eb;
    TCHECK(hipEventCreate(&ea));
    TCHECK(hipEventCreate(&eb));
    TCHECK(hipEventRecord(ea, nullptr));
    for (int i = 0; i < iters; ++i) TCHECK(launch_gemm_mx(DT_BF16, e, a, g, nullptr));
    TCHECK(hipEventRecord(eb, nullptr));
    TCHECK(hipEventSynchronize(eb));
    float ms = 0.f;
    TCHECK(hipEventElapsedTime(&ms, ea, eb));
    (void)hipEventDestroy(ea);
    (void)hipEventDestroy(eb);
    *us_per_launch = (double)ms * 1000.0 / iters;
  });
}

// Crash diagnostics for GPU-box runs (no debugger there): a SIGSEGV / SIGABRT handler that prints each
// frame's object file and offset (map offsets to functions with addr2line -f -C -e <object> <offset>),
// then re-raises with the default action.
static void crash_handler(int sig) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  char line[512];
  int len = snprintf(line, sizeof(line), "clipgpu crash handler: signal %d, %d frames\n", sig, n);
  if (write(2, line, (size_t)len) < 0) {}
  for (int i = 0; i < n; ++i) {
    Dl_info info{};
    if (dladdr(frames[i], &info) && info.dli_fname) {
      len = snprintf(line, sizeof(line), "  #%d %s +0x%lx (%s)\n", i, info.dli_fname,
                     (unsigned long)((char*)frames[i] - (char*)info.dli_fbase), info.dli_sname ? info.dli_sname : "?");
    } else {
      len = snprintf(line, sizeof(line), "  #%d %p\n", i, frames[i]);
    }
    if (write(2, line, (size_t)len) < 0) {}
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

int clipgpu_test_install_crash_handler(void) {
  static char alt[1 << 16];  // the handler runs on its own stack, so a stack overflow is reported too
  stack_t ss{};
  ss.ss_sp = alt;
  ss.ss_size = sizeof(alt);
  sigaltstack(&ss, nullptr);
  struct sigaction sa{};
  sa.sa_handler = crash_handler;
  sa.sa_flags = SA_ONSTACK;
  sigaction(SIGSEGV, &sa, nullptr);
  sigaction(SIGABRT, &sa, nullptr);
  return 0;
}

int clipgpu_test_host_copy(int64_t bytes, int mode, int iters, double* us_per_copy) {
  return guarded([&]() {
    if (bytes <= 0 || iters <= 0 || !us_per_copy || mode < 0 || mode > 3)
      throw ClipErr(CLIPGPU_ERR_INVALID, "bad host copy arguments");
    // source: page-aligned malloc'd memory; destination: malloc'd (mode 0 / 1) or pinned hipHostMalloc
    // memory (mode 2 / 3, the host path's staging); one thread (0 / 2) or the copy pool (1 / 3)
    void* src = nullptr;
    if (posix_memalign(&src, 4096, (size_t)bytes) != 0) throw ClipErr(CLIPGPU_ERR_INVALID, "host alloc");
    std::memset(src, 3, (size_t)bytes);
    void* dst = nullptr;
    if (mode >= 2) TCHECK(hipHostMalloc(&dst, (size_t)bytes, hipHostMallocDefault));
    else if (posix_memalign(&dst, 4096, (size_t)bytes) != 0) throw ClipErr(CLIPGPU_ERR_INVALID, "host alloc");
    std::memset(dst, 0, (size_t)bytes);
    auto once = [&]() {
      if (mode & 1) pool_memcpy(dst, src, (size_t)bytes);
      else std::memcpy(dst, src, (size_t)bytes);
    };
    once();
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; ++i) once();
    const auto t1 = std::chrono::steady_clock::now();
    *us_per_copy = std::chrono::duration<double, std::micro>(t1 - t0).count() / iters;
    if (mode >= 2) (void)hipHostFree(dst);
    else std::free(dst);
    std::free(src);
  });
}

int clipgpu_test_h2d_bench(int64_t bytes, int mode, int iters, double* us_per_copy) {
  return guarded([&]() {
    const int src = mode >> 2;
    mode &= 3;
    if (bytes <= 0 || bytes % 32 || src > 1 || iters <= 0 || !us_per_copy)
      throw ClipErr(CLIPGPU_ERR_INVALID, "bad H2D bench arguments");
    // src 0: hipHostMalloc; 1: page-aligned malloc'd memory registered as clipgpu_host_register does
    void* host = nullptr;
    if (src == 0) {
      TCHECK(hipHostMalloc(&host, (size_t)bytes, hipHostMallocMapped | hipHostMallocPortable));
    } else {
      if (posix_memalign(&host, 4096, (size_t)bytes) != 0) throw ClipErr(CLIPGPU_ERR_INVALID, "host alloc");
      std::memset(host, 1, (size_t)bytes);
      const hipError_t e = hipHostRegister(host, (size_t)bytes, hipHostRegisterMapped | hipHostRegisterPortable);
      if (e != hipSuccess) {
        std::free(host);
        TCHECK(e);
      }
    }
    std::memset(host, 1, (size_t)bytes);
    void* mapped = nullptr;
    hipStream_t s0 = nullptr, s1 = nullptr;
    hipEvent_t a = nullptr, b = nullptr, j = nullptr;
    DevBuf dst(bytes);
    auto run = [&]() {
      const size_t h = (size_t)bytes / 2;
      switch (mode) {
        case 0: TCHECK(hipMemcpyAsync(dst.p, host, (size_t)bytes, hipMemcpyHostToDevice, s0)); break;
        case 1: TCHECK(launch_pull_copy(mapped, dst.p, (size_t)bytes, s0)); break;
        default:  // halves on two streams: 2 = two SDMA copies, 3 = the pull kernel beside one SDMA copy
          TCHECK(hipEventRecord(j, s0));
          TCHECK(hipStreamWaitEvent(s1, j, 0));
          if (mode == 2) TCHECK(hipMemcpyAsync(dst.p, host, h, hipMemcpyHostToDevice, s0));
          else TCHECK(launch_pull_copy(mapped, dst.p, h, s0));
          TCHECK(hipMemcpyAsync((char*)dst.p + h, (char*)host + h, (size_t)bytes - h, hipMemcpyHostToDevice, s1));
          TCHECK(hipEventRecord(j, s1));
          TCHECK(hipStreamWaitEvent(s0, j, 0));
      }
    };
    std::exception_ptr err;
    try {
      TCHECK(hipHostGetDevicePointer(&mapped, host, 0));
      TCHECK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
      TCHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
      TCHECK(hipEventCreate(&a));
      TCHECK(hipEventCreate(&b));
      TCHECK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
      for (int i = 0; i < 3; ++i) run();
      TCHECK(hipEventRecord(a, s0));
      for (int i = 0; i < iters; ++i) run();
      TCHECK(hipEventRecord(b, s0));
      TCHECK(hipEventSynchronize(b));
      float ms = 0.f;
      TCHECK(hipEventElapsedTime(&ms, a, b));
      *us_per_copy = (double)ms * 1000.0 / iters;
    } catch (...) {
      err = std::current_exception();
    }
    (void)hipStreamSynchronize(s0);
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
    if (j) (void)hipEventDestroy(j);
    if (s0) (void)hipStreamDestroy(s0);
    if (s1) (void)hipStreamDestroy(s1);
    if (src == 0) {
      (void)hipHostFree(host);
    } else {
      (void)hipHostUnregister(host);
      std::free(host);
    }
    if (err) std::rethrow_exception(err);
  });
}

#ifdef CLIPGPU_GEMM_STAMPS
// Diagnostic build only (not in the headers): one timed-after-warmup GEMM launch
// with s_memtime stamps; out receives nblocks x 64 u64 (see gemm.hip slots).
int clipgpu_diag_gemm_stamps(int dtype, int epi, int act, int64_t M, int64_t N, int64_t K, int tile,
                             unsigned long long* out, int nblocks, int diag) {
  return guarded([&]() {
    const DType dt = dt_of(dtype);
    DevBuf fA(M * K * 4), fW(N * K * 4), dA(M * K * 2), dW(N * K * 2), dB(N * 4), dO(M * N * 4);
    hipLaunchKernelGGL(fill_random, dim3(2048), dim3(256), 0, nullptr, fA.as<float>(), (long)(M * K), 1u);
    hipLaunchKernelGGL(fill_random, dim3(2048), dim3(256), 0, nullptr, fW.as<float>(), (long)(N * K), 2u);
    hipLaunchKernelGGL(fill_random, dim3(64), dim3(256), 0, nullptr, dB.as<float>(), (long)N, 3u);
    TCHECK(launch_cast_f32(dt, fA.as<float>(), dA.p, (long)(M * K), nullptr));
    TCHECK(launch_cast_f32(dt, fW.as<float>(), dW.p, (long)(N * K), nullptr));
    GemmParams g{};
    g.A = dA.p; g.lda = K; g.W = dW.p; g.ldw = K; g.bias = dB.as<float>();
    g.out = dO.p; g.ldo = N; g.M = (int)M; g.N = (int)N; g.K = (int)K; g.tile = tile; g.diag = diag;
    const int e = (epi == 1 || epi == 3) ? EPI_RESID : (epi == 2 ? EPI_STORE32 : EPI_STORE16);
    g.x16 = epi == 3;  // the f16 residual stream (timing only)
    for (int i = 0; i < 20; ++i) TCHECK(launch_gemm(dt, A_ROWS, e, epi == 0 ? act : 0, g, nullptr));
    TCHECK(hipDeviceSynchronize());
    TCHECK(read_gemm_stamps(nullptr, nblocks, true));
    TCHECK(launch_gemm(dt, A_ROWS, e, epi == 0 ? act : 0, g, nullptr));
    TCHECK(hipDeviceSynchronize());
    TCHECK(read_gemm_stamps(out, nblocks, false));
  });
}

#endif

}  // extern "C"
