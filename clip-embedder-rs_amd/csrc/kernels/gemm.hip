// MFMA GEMM for the transformer towers, gfx950.
//
//   C[M][N] = A[M][K] . W[N][K]^T  (+ fused epilogue)
//
// Replaces the MatMul/Gemm/Conv nodes ONNX Runtime executes for the exported
// graphs (pull_onnx.py:53-68 -> src/vision.rs:108, src/text.rs:158-160):
// QKV in_proj, out_proj, c_fc (+activation), c_proj (+residual), the conv1
// patch embedding (im2col-free: A rows are gathered straight from the image)
// and the final projection.
//
// One kernel template, three tile shapes (GemmTile):
//   128x128  4 waves (2x2, 64x64 per wave), 64 KiB LDS, 2 blocks / CU
//   256x128  8 waves (2x4, 128x32 per wave), 96 KiB LDS
//   256x256  8 waves (2x4, 128x64 per wave), 128 KiB LDS
// Each wave issues v_mfma_f32_16x16x32_{bf16,f16} (f32 accumulate).  Operand
// tiles (BK = 64) are staged global->LDS by global_load_lds_dwordx4 into a
// lane-linear image with the XOR swizzle applied on the SOURCE address and on
// the ds_read_b128 address (cdna_hip_programming.md §5.4 rule 21),
// double-buffered: the next K-tile's loads are issued before the current one's
// MFMAs, one vmcnt(0) + barrier per K-step.  Image-sourced A tiles are
// register-staged (f32 / u8 -> 16-bit in flight).  Block ids are remapped
// XCD-aware, then grouped 8 row-panels at a time for L2 reuse.  Persistent:
// the grid is the resident block count and each block walks its tiles, the
// next tile's first K-slice staged under the current tile's last K-step.  MFMA
// operands are swapped so each lane owns 4 consecutive output columns (8 / 16 B
// epilogue stores).  M and N tails: clamped source rows + masked stores; K must
// be a multiple of 64.
#include "common.hpp"
#include "kernels.hpp"

namespace clipgpu {

namespace {

constexpr int BK = 64;

// Byte offset of 16-byte chunk c (0..7) of row r in a [rows][64] 16-bit tile.
// Conflict-free for the 16x16x32 fragment reads (16 rows x 4 chunks per
// ds_read_b128 lane group).
__device__ __forceinline__ int tile_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

template <typename T>
__device__ __forceinline__ T to16(float v) { return (T)v; }

// Tile order shared by all blocks: tiles are grouped 8 row panels at a time
// (walk M first inside a group) so that concurrently running tiles share A and W
// panels in L2.
__device__ __forceinline__ void tile_coords(int t, int nTm, int nTn, int BM, int BN, int& m0, int& n0) {
  constexpr int GROUP = 8;
  const int per_group = GROUP * nTn;
  const int first_m = (t / per_group) * GROUP;
  const int gsize = min(nTm - first_m, GROUP);
  m0 = (first_m + (t % per_group) % gsize) * BM;
  n0 = ((t % per_group) / gsize) * BN;
}

template <typename T, int BM, int BN, int WGM, int WGN, int ASRC, int EPI, int ACT>
__global__ __launch_bounds__(WGM* WGN * 64, 2) void gemm_bt_kernel(GemmParams p) {
  typedef typename Vec8<T>::type V8;
  typedef typename Vec4<T>::type V4;
  constexpr int NW = WGM * WGN, NT = NW * 64;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int A_INSTR = BM / 8 / NW, B_INSTR = BN / 8 / NW;  // 1 KiB glds per wave-instruction
  constexpr int TM = BM / WGM, TN = BN / WGN, MI = TM / 16, NI = TN / 16;
  constexpr int A_CHUNKS = BM * 8 / NT;  // register-staged image A: 16-byte chunks per thread
  static_assert(A_INSTR >= 1 && B_INSTR >= 1 && MI >= 1 && NI >= 1, "bad tile");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nTn = (p.N + BN - 1) / BN;
  const int nTm = (p.M + BM - 1) / BM;
  const int ntiles = nTn * nTm;
  const int nk = p.K / BK;

  // Persistent schedule: the grid is <= the resident block count.  With a grid
  // that is a multiple of 8, XCD x (blocks b = x mod 8) walks a contiguous range
  // of tiles; otherwise every block owns one tile (grid == ntiles).
  const int nb = gridDim.x;
  int t_first, t_stride, t_end;
  if (nb % 8 == 0 && nb < ntiles) {
    const int x = blockIdx.x & 7, nbx = nb >> 3;
    const int q = ntiles >> 3, r = ntiles & 7;
    const int start = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
    t_first = start + (blockIdx.x >> 3);
    t_stride = nbx;
    t_end = start + q + (x < r ? 1 : 0);
  } else {
    t_first = xcd_remap(blockIdx.x, nb);
    t_stride = ntiles;  // single tile
    t_end = t_first + 1;
  }
  if (t_first >= t_end) return;

  char* const sA0 = smem;
  char* const sB0 = smem + A_BYTES;
  char* const sA1 = smem + STAGE;
  char* const sB1 = smem + STAGE + A_BYTES;

  // ---- per-tile staging sources ----------------------------------------------
  // glds: wave w, instruction i writes rows (w*INSTR + i)*8 .. +7 (1 KiB); lane
  // l lands at row +(l>>3), slot (l&7), which holds global chunk slot ^ f(row).
  // 32-bit per-lane element offsets from the kernel-argument base pointers
  // (host checks that every operand fits in 2^31 elements).
  int woff[B_INSTR];
  int aoff[A_INSTR];
  long img_base[A_CHUNKS];
  int img_row[A_CHUNKS];
  const T* const Wb = (const T*)p.W;
  const T* const Ab = (const T*)p.A;
  auto set_tile = [&](int m0, int n0) {
#pragma unroll
    for (int i = 0; i < B_INSTR; ++i) {
      const int r = (wave * B_INSTR + i) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      woff[i] = min(n0 + r, p.N - 1) * (int)p.ldw + c * 8;
    }
    if constexpr (ASRC == A_ROWS) {
#pragma unroll
      for (int i = 0; i < A_INSTR; ++i) {
        const int r = (wave * A_INSTR + i) * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        aoff[i] = min(m0 + r, p.M - 1) * (int)p.lda + c * 8;
      }
    } else {
      const int G2 = p.G * p.G;
#pragma unroll
      for (int i = 0; i < A_CHUNKS; ++i) {
        const int q = tid + NT * i;
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
  };

  auto stage_w = [&](int kt, char* sB) {
#pragma unroll
    for (int i = 0; i < B_INSTR; ++i) glds16(Wb + (woff[i] + kt * BK), sB + (wave * B_INSTR + i) * 1024);
  };
  auto stage_a_rows = [&](int kt, char* sA) {
#pragma unroll
    for (int i = 0; i < A_INSTR; ++i) glds16(Ab + (aoff[i] + kt * BK), sA + (wave * A_INSTR + i) * 1024);
  };

  // Image-sourced A: 8 consecutive k (same channel and image row; P % 8 == 0).
  float areg[A_CHUNKS][8];
  auto load_a_img = [&](int kt) {
    const int PP = p.P * p.P;
#pragma unroll
    for (int i = 0; i < A_CHUNKS; ++i) {
      const int c = (tid + NT * i) & 7;
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
    for (int i = 0; i < A_CHUNKS; ++i) {
      const int c = (tid + NT * i) & 7;
      V8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = to16<T>(areg[i][e]);
      *(V8*)(sA + tile_off(img_row[i], c)) = v;
    }
  };
  // Issue the loads of K-step kt of the current tile into buffer (sA, sB).
  auto stage = [&](int kt, char* sA, char* sB) {
    stage_w(kt, sB);
    if constexpr (ASRC == A_ROWS) stage_a_rows(kt, sA);
    else load_a_img(kt);
  };

  // ---- fragment addressing -------------------------------------------------
  const int wm = (wave / WGN) * TM, wn = (wave % WGN) * TN;
  const int fr = lane & 15, fq = lane >> 4;
  int offA[2], offB[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int sw = ((kk * 4 + fq) ^ (fr >> 1)) << 4;  // rows are 16-aligned + fr
    offA[kk] = (wm + fr) * 128 + sw;
    offB[kk] = (wn + fr) * 128 + sw;
  }

  // Operands swapped (W rows as the MFMA "A" operand): acc[ni][mi][j] =
  // C[m = wm + mi*16 + fr][n = wn + ni*16 + fq*4 + j], i.e. each lane owns 4
  // consecutive output columns of one row -> 8 / 16-byte epilogue stores.
  f32x4 acc[NI][MI];
  auto compute = [&](const char* sA, const char* sB) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      V8 a[MI], b[NI];
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) b[ni] = *(const V8*)(sB + offB[kk] + ni * 2048);
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) a[mi] = *(const V8*)(sA + offA[kk] + mi * 2048);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) acc[ni][mi] = mfma_16x16x32(b[ni], a[mi], acc[ni][mi]);
    }
  };

  auto epilogue = [&](int m0, int n0) {
    const int G2 = p.G * p.G;
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int n = n0 + wn + ni * 16 + fq * 4;
      const bool nfull = n + 4 <= p.N;
      float bv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[j] = (p.bias != nullptr && n + j < p.N) ? p.bias[n + j] : 0.f;
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        const int m = m0 + wm + mi * 16 + fr;
        if (m >= p.M) continue;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = acc[ni][mi][j] + bv[j];
        if constexpr (EPI == EPI_STORE16) {
          T* o = (T*)p.out + (long)m * p.ldo + n;
          if (nfull) {
            V4 w;
#pragma unroll
            for (int j = 0; j < 4; ++j) w[j] = to16<T>(apply_act<ACT>(v[j]));
            *(V4*)o = w;
          } else {
            for (int j = 0; j < 4; ++j)
              if (n + j < p.N) o[j] = to16<T>(apply_act<ACT>(v[j]));
          }
        } else {
          float* o;
          const float* ps = nullptr;
          if constexpr (EPI == EPI_PATCH) {
            const int b = m / G2, pp = m - b * G2;
            o = (float*)p.out + ((long)b * (G2 + 1) + 1 + pp) * p.ldo + n;
            ps = p.pos + (long)(1 + pp) * p.N + n;
          } else {
            o = (float*)p.out + (long)m * p.ldo + n;
          }
          if (nfull) {
            float4 w = make_float4(v[0], v[1], v[2], v[3]);
            if constexpr (EPI == EPI_RESID) {
              const float4 x = *(const float4*)o;
              w.x += x.x; w.y += x.y; w.z += x.z; w.w += x.w;
            } else if constexpr (EPI == EPI_PATCH) {
              const float4 x = *(const float4*)ps;
              w.x += x.x; w.y += x.y; w.z += x.z; w.w += x.w;
            }
            *(float4*)o = w;
          } else {
            for (int j = 0; j < 4; ++j) {
              if (n + j >= p.N) continue;
              float r = v[j];
              if constexpr (EPI == EPI_RESID) r += o[j];
              if constexpr (EPI == EPI_PATCH) r += ps[j];
              o[j] = r;
            }
          }
        }
      }
    }
  };

  // ---- persistent tile loop: 2-stage K pipeline, next tile's first K-step
  //      prefetched under the current tile's last K-step and epilogue ----------
  int m0, n0;
  tile_coords(t_first, nTm, nTn, BM, BN, m0, n0);
  set_tile(m0, n0);
  stage(0, sA0, sB0);
  if constexpr (ASRC != A_ROWS) store_a_img(sA0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  int parity = 0;  // buffer holding K-step 0 of the current tile
  for (int t = t_first; t < t_end; t += t_stride) {
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) acc[ni][mi] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt + 1 < nk; ++kt) {
      const bool cur1 = (kt & 1) ^ parity;
      char* const sAn = cur1 ? sA0 : sA1;
      char* const sBn = cur1 ? sB0 : sB1;
      stage(kt + 1, sAn, sBn);
      compute(cur1 ? sA1 : sA0, cur1 ? sB1 : sB0);
      if constexpr (ASRC != A_ROWS) store_a_img(sAn);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    // last K-step: prefetch the next tile's first K-step under it and the epilogue
    const bool cur1 = ((nk - 1) & 1) ^ parity;
    const int tn = t + t_stride;
    const bool has_next = tn < t_end;
    int nm0 = m0, nn0 = n0;
    if (has_next) {
      tile_coords(tn, nTm, nTn, BM, BN, nm0, nn0);
      set_tile(nm0, nn0);
      stage(0, cur1 ? sA0 : sA1, cur1 ? sB0 : sB1);
    }
    compute(cur1 ? sA1 : sA0, cur1 ? sB1 : sB0);
    if constexpr (ASRC != A_ROWS) {
      if (has_next) store_a_img(cur1 ? sA0 : sA1);
    }
    epilogue(m0, n0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    parity ^= (nk & 1);
    m0 = nm0;
    n0 = nn0;
  }
}

int device_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
      cus = prop.multiProcessorCount;
    if (cus <= 0) cus = 256;
  }
  return cus;
}

template <typename T, int BM, int BN, int WGM, int WGN, int ASRC, int EPI, int ACT>
hipError_t launch_cfg(const GemmParams& p, hipStream_t s) {
  const int nTn = (p.N + BN - 1) / BN, nTm = (p.M + BM - 1) / BM;
  const int ntiles = nTn * nTm;
  // resident blocks: one 8-wave block (96-128 KiB LDS) or two 4-wave blocks (64 KiB) per CU
  const int resident = device_cus() * (WGM * WGN == 4 ? 2 : 1);
  const int grid = ntiles <= resident ? ntiles : resident;
  hipLaunchKernelGGL((gemm_bt_kernel<T, BM, BN, WGM, WGN, ASRC, EPI, ACT>), dim3(grid), dim3(WGM * WGN * 64), 0, s,
                     p);
  return hipGetLastError();
}

template <typename T, int ASRC, int EPI, int ACT>
hipError_t launch_tile(const GemmParams& p, hipStream_t s) {
  if constexpr (ASRC != A_ROWS) {
    return launch_cfg<T, 128, 128, 2, 2, ASRC, EPI, ACT>(p, s);  // register-staged A: spill-free tile
  } else {
    const int tile = p.tile == TILE_AUTO ? pick_gemm_tile(p.M, p.N, p.K) : p.tile;
    switch (tile) {
      case TILE_256x256: return launch_cfg<T, 256, 256, 2, 4, ASRC, EPI, ACT>(p, s);
      case TILE_256x128: return launch_cfg<T, 256, 128, 2, 4, ASRC, EPI, ACT>(p, s);
      default: return launch_cfg<T, 128, 128, 2, 2, ASRC, EPI, ACT>(p, s);
    }
  }
}

template <typename T>
hipError_t launch_typed(int asrc, int epi, int act, const GemmParams& p, hipStream_t s) {
  if (asrc == A_ROWS) {
    if (epi == EPI_STORE16) {
      switch (act) {
        case ACT_NONE: return launch_tile<T, A_ROWS, EPI_STORE16, ACT_NONE>(p, s);
        case ACT_QUICK_GELU: return launch_tile<T, A_ROWS, EPI_STORE16, ACT_QUICK_GELU>(p, s);
        case ACT_GELU: return launch_tile<T, A_ROWS, EPI_STORE16, ACT_GELU>(p, s);
        case ACT_GELU_TANH: return launch_tile<T, A_ROWS, EPI_STORE16, ACT_GELU_TANH>(p, s);
      }
    } else if (epi == EPI_RESID) {
      return launch_tile<T, A_ROWS, EPI_RESID, ACT_NONE>(p, s);
    } else if (epi == EPI_STORE32) {
      return launch_tile<T, A_ROWS, EPI_STORE32, ACT_NONE>(p, s);
    }
  } else if (asrc == A_IMG_F32 && epi == EPI_PATCH) {
    return launch_tile<T, A_IMG_F32, EPI_PATCH, ACT_NONE>(p, s);
  } else if (asrc == A_IMG_U8 && epi == EPI_PATCH) {
    return launch_tile<T, A_IMG_U8, EPI_PATCH, ACT_NONE>(p, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace

// Tile choice: large-M GEMMs use the 256-row tiles (128 FLOP per staged byte
// instead of 64); among those, the column tile that wastes the least of the
// last wave of blocks over the 256 CUs (one 8-wave block per CU).
int pick_gemm_tile(int M, int N, int K) {
  (void)K;
  if (M < 2048) return TILE_128x128;
  const int cus = 256;
  auto eff = [&](int bm, int bn) {
    const long tiles = (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
    const long rounds = (tiles + cus - 1) / cus;
    return (double)tiles / (double)(rounds * cus);
  };
  // 256x128 stages 1.5x the bytes per FLOP of 256x256: prefer 256x256 unless it idles
  // noticeably more CUs in the tail.
  return eff(256, 256) >= 0.85 * eff(256, 128) ? TILE_256x256 : TILE_256x128;
}

hipError_t launch_gemm(DType dt, int asrc, int epi, int act, const GemmParams& p, hipStream_t s) {
  if (p.K % BK != 0 || p.M <= 0 || p.N <= 0) return hipErrorInvalidValue;
  // 32-bit staging offsets
  if ((long)p.M * p.lda >= (1L << 31) || (long)p.N * p.ldw >= (1L << 31)) return hipErrorInvalidValue;
  if (asrc != A_ROWS && (p.P % 8 != 0)) return hipErrorInvalidValue;
  return dt == DT_BF16 ? launch_typed<__bf16>(asrc, epi, act, p, s)
                       : launch_typed<_Float16>(asrc, epi, act, p, s);
}

}  // namespace clipgpu
