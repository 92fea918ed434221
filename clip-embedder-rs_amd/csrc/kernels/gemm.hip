// MFMA GEMM for the transformer towers, gfx950.
//
//   C[M][N] = A[M][K] . W[N][K]^T  (+ fused epilogue)
//
// Replaces the MatMul/Gemm/Conv nodes ONNX Runtime executes for the exported
// graphs (pull_onnx.py:53-68 -> src/vision.rs:108, src/text.rs:158-160):
// QKV in_proj, out_proj, c_fc (+activation), c_proj (+residual), the
// conv1 patch embedding (im2col-free: A rows are gathered straight from the
// image) and the final projection.
//
// Tile 128x128x64, 256 threads = 4 waves in 2x2, each wave 64x64 outputs as
// 4x4 v_mfma_f32_16x16x32_{bf16,f16} tiles (f32 accumulate).  Operand tiles
// are staged global->LDS by global_load_lds_dwordx4 (lane-linear LDS image,
// the XOR swizzle applied on the SOURCE address and on the ds_read_b128
// address: cdna_hip_programming.md §5.4 rule 21), double-buffered, one
// barrier per K-step.  Image-sourced A tiles are register-staged (f32/u8 ->
// 16-bit conversion on the way into LDS).  Block ids are remapped XCD-aware.
// M and N tails are handled by clamping source rows and masking stores; K must
// be a multiple of 64.
#include "common.hpp"
#include "kernels.hpp"

namespace clipgpu {

namespace {

constexpr int BM = 128, BN = 128, BK = 64, NTHREADS = 256;
constexpr int TILE_BYTES = BM * BK * 2;  // 16 KiB per operand tile

// Byte offset of 16-byte chunk c (0..7) of row r in a [rows][64] 16-bit tile.
// Conflict-free for the 16x16x32 fragment reads (16 rows x 4 chunks per
// ds_read_b128 lane group).
__device__ __forceinline__ int tile_off(int r, int c) {
  return r * 128 + ((c ^ ((r >> 1) & 7)) << 4);
}

template <typename T>
__device__ __forceinline__ T to16(float v) { return (T)v; }

template <typename T, int ASRC, int EPI, int ACT>
__global__ __launch_bounds__(NTHREADS, 2) void gemm_bt_kernel(GemmParams p) {
  typedef typename Vec8<T>::type V8;
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nTn = (p.N + BN - 1) / BN;
  const int nTm = (p.M + BM - 1) / BM;
  const int wg = xcd_remap(blockIdx.x, nTn * nTm);
  const int m0 = (wg / nTn) * BM;
  const int n0 = (wg % nTn) * BN;

  char* const sA0 = smem;
  char* const sB0 = smem + TILE_BYTES;
  char* const sA1 = smem + 2 * TILE_BYTES;
  char* const sB1 = smem + 3 * TILE_BYTES;

  // ---- staging setup -------------------------------------------------------
  // glds: wave w, instruction i writes rows w*32 + i*8 .. +7 (1 KiB); lane l
  // lands at row +(l>>3), 16-byte slot (l&7), which holds global chunk
  // slot ^ f(row) (source-side swizzle).
  const T* wsrc[4];
  const T* asrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = wave * 32 + i * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int gn = min(n0 + r, p.N - 1);
    wsrc[i] = (const T*)p.W + (long)gn * p.ldw + c * 8;
    if constexpr (ASRC == A_ROWS) {
      const int gm = min(m0 + r, p.M - 1);
      asrc[i] = (const T*)p.A + (long)gm * p.lda + c * 8;
    }
  }
  // Register-staged image A: thread owns chunks q = tid + 256*i (row q>>3, chunk q&7).
  long img_base[4];
  int img_row[4];
  if constexpr (ASRC != A_ROWS) {
    const int G2 = p.G * p.G;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + NTHREADS * i;
      const int r = q >> 3;
      img_row[i] = r;
      const int gm = min(m0 + r, p.M - 1);
      const int b = gm / G2, pp = gm % G2;
      const int py = pp / p.G, px = pp % p.G;
      if constexpr (ASRC == A_IMG_F32)
        img_base[i] = ((long)b * 3 * p.S + (long)py * p.P) * p.S + (long)px * p.P;
      else  // NHWC u8
        img_base[i] = (((long)b * p.S + (long)py * p.P) * p.S + (long)px * p.P) * 3;
    }
  }

  auto stage_w = [&](int kt, char* sB) {
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(wsrc[i] + kt * BK, sB + wave * 4096 + i * 1024);
  };
  auto stage_a_rows = [&](int kt, char* sA) {
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(asrc[i] + kt * BK, sA + wave * 4096 + i * 1024);
  };

  // Image-sourced A: load 8 consecutive k (same channel / image row, P % 8 == 0).
  float areg[4][8];
  auto load_a_img = [&](int kt) {
    const int PP = p.P * p.P;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = (tid + NTHREADS * i) & 7;
      const int k = kt * BK + c * 8;
      const int ch = k / PP, rem = k - ch * PP;
      const int ky = rem / p.P, kx = rem - ky * p.P;
      if constexpr (ASRC == A_IMG_F32) {
        const float* src = (const float*)p.img + img_base[i] + ((long)ch * p.S + ky) * p.S + kx;
        const float4 v0 = *(const float4*)src;
        const float4 v1 = *(const float4*)(src + 4);
        areg[i][0] = v0.x; areg[i][1] = v0.y; areg[i][2] = v0.z; areg[i][3] = v0.w;
        areg[i][4] = v1.x; areg[i][5] = v1.y; areg[i][6] = v1.z; areg[i][7] = v1.w;
      } else {
        const uint8_t* src = (const uint8_t*)p.img + img_base[i] + ((long)ky * p.S + kx) * 3 + ch;
        const float mu = p.mean[0] * (ch == 0) + p.mean[1] * (ch == 1) + p.mean[2] * (ch == 2);
        const float sd = p.stdv[0] * (ch == 0) + p.stdv[1] * (ch == 1) + p.stdv[2] * (ch == 2);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          // src/vision.rs:254-255: (p / 255 - mean[c]) / std[c]
          const float val = (float)src[e * 3] / 255.0f;
          areg[i][e] = (val - mu) / sd;
        }
      }
    }
  };
  auto store_a_img = [&](char* sA) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = (tid + NTHREADS * i) & 7;
      V8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = to16<T>(areg[i][e]);
      *(V8*)(sA + tile_off(img_row[i], c)) = v;
    }
  };

  // ---- fragment addressing -------------------------------------------------
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int fr = lane & 15, fq = lane >> 4;
  int offA[2], offB[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int sw = ((kk * 4 + fq) ^ (fr >> 1)) << 4;
    offA[kk] = (wm + fr) * 128 + sw;
    offB[kk] = (wn + fr) * 128 + sw;
  }

  f32x4 acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const char* sA, const char* sB) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      V8 a[4], b[4];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) a[mi] = *(const V8*)(sA + offA[kk] + mi * 2048);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) b[ni] = *(const V8*)(sB + offB[kk] + ni * 2048);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = mfma_16x16x32(a[mi], b[ni], acc[mi][ni]);
    }
  };

  // ---- main loop: 2-stage, one barrier per K-step ---------------------------
  const int nk = p.K / BK;
  stage_w(0, sB0);
  if constexpr (ASRC == A_ROWS) {
    stage_a_rows(0, sA0);
  } else {
    load_a_img(0);
    store_a_img(sA0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const bool odd = kt & 1;
    char* const sAc = odd ? sA1 : sA0;
    char* const sBc = odd ? sB1 : sB0;
    char* const sAn = odd ? sA0 : sA1;
    char* const sBn = odd ? sB0 : sB1;
    const bool more = kt + 1 < nk;
    if (more) {
      stage_w(kt + 1, sBn);
      if constexpr (ASRC == A_ROWS) stage_a_rows(kt + 1, sAn);
      else load_a_img(kt + 1);
    }
    compute(sAc, sBc);
    if constexpr (ASRC != A_ROWS) {
      if (more) store_a_img(sAn);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue --------------------------------------------------------------
  // acc[mi][ni][j] = C[m0 + wm + mi*16 + fq*4 + j][n0 + wn + ni*16 + fr]
  float bv[4];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int n = n0 + wn + ni * 16 + fr;
    bv[ni] = (p.bias != nullptr && n < p.N) ? p.bias[n] : 0.f;
  }
  const int G2 = p.G * p.G;
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + wm + mi * 16 + fq * 4 + j;
      if (m >= p.M) continue;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int n = n0 + wn + ni * 16 + fr;
        if (n >= p.N) continue;
        const float v = acc[mi][ni][j] + bv[ni];
        if constexpr (EPI == EPI_STORE16) {
          ((T*)p.out)[(long)m * p.ldo + n] = to16<T>(apply_act<ACT>(v));
        } else if constexpr (EPI == EPI_RESID) {
          float* o = (float*)p.out + (long)m * p.ldo + n;
          *o = *o + v;
        } else if constexpr (EPI == EPI_STORE32) {
          ((float*)p.out)[(long)m * p.ldo + n] = v;
        } else {  // EPI_PATCH
          const int b = m / G2, pp = m - b * G2;
          const long row = (long)b * (G2 + 1) + 1 + pp;
          ((float*)p.out)[row * p.ldo + n] = v + p.pos[(long)(1 + pp) * p.N + n];
        }
      }
    }
  }
}

template <typename T, int ASRC, int EPI, int ACT>
hipError_t launch_t(const GemmParams& p, hipStream_t s) {
  const int nTn = (p.N + BN - 1) / BN, nTm = (p.M + BM - 1) / BM;
  hipLaunchKernelGGL((gemm_bt_kernel<T, ASRC, EPI, ACT>), dim3(nTn * nTm), dim3(NTHREADS), 0, s, p);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_typed(int asrc, int epi, int act, const GemmParams& p, hipStream_t s) {
  if (asrc == A_ROWS) {
    if (epi == EPI_STORE16) {
      switch (act) {
        case ACT_NONE: return launch_t<T, A_ROWS, EPI_STORE16, ACT_NONE>(p, s);
        case ACT_QUICK_GELU: return launch_t<T, A_ROWS, EPI_STORE16, ACT_QUICK_GELU>(p, s);
        case ACT_GELU: return launch_t<T, A_ROWS, EPI_STORE16, ACT_GELU>(p, s);
        case ACT_GELU_TANH: return launch_t<T, A_ROWS, EPI_STORE16, ACT_GELU_TANH>(p, s);
      }
    } else if (epi == EPI_RESID) {
      return launch_t<T, A_ROWS, EPI_RESID, ACT_NONE>(p, s);
    } else if (epi == EPI_STORE32) {
      return launch_t<T, A_ROWS, EPI_STORE32, ACT_NONE>(p, s);
    }
  } else if (asrc == A_IMG_F32 && epi == EPI_PATCH) {
    return launch_t<T, A_IMG_F32, EPI_PATCH, ACT_NONE>(p, s);
  } else if (asrc == A_IMG_U8 && epi == EPI_PATCH) {
    return launch_t<T, A_IMG_U8, EPI_PATCH, ACT_NONE>(p, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace

hipError_t launch_gemm(DType dt, int asrc, int epi, int act, const GemmParams& p, hipStream_t s) {
  if (p.K % BK != 0 || p.M <= 0 || p.N <= 0) return hipErrorInvalidValue;
  if (asrc != A_ROWS && (p.P % 8 != 0)) return hipErrorInvalidValue;
  return dt == DT_BF16 ? launch_typed<__bf16>(asrc, epi, act, p, s)
                       : launch_typed<_Float16>(asrc, epi, act, p, s);
}

}  // namespace clipgpu
