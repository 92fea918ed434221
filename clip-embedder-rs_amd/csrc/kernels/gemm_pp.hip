// Ping-pong MFMA GEMM for the large trunk tiles, gfx950.
//
//   C[M][N] = A[M][K] . W[N][K]^T  (+ the fused epilogues of gemm.hip)
//
// Same arithmetic as gemm_pipe_kernel (gemm.hip) -- the same LDS images and swizzles, MFMA operand
// roles, k -> lane map, per-output MFMA chain (K-steps ascending, kk0 then kk1) and epilogue float
// ops -- so every output is bit-identical to the other tiles' (test_gemm_tile_choice_is_bit_exact);
// only the schedule differs.
//
// gemm_pipe_kernel runs its 8 waves in lockstep: one block barrier per 64-deep K-step, where both
// waves of every SIMD stop issuing MFMAs at once (the round-2 stamps: 256x256 K-steps 2,787 cycles,
// 2,139 with the barrier removed, 2,048 MFMA floor; 192x256 2,488 vs 1,478).  Here the block is two
// groups of 4 waves -- group 0 owns rows 0 .. BM/2-1, group 1 rows BM/2 .. BM-1, each wave a
// (BM/2) x 64 output tile -- and every K-step is four sections separated by block barriers:
//   L0  read the kk0 fragments of step g (buffer g % 2); issue this wave's LDS-DMA pieces of
//       step g + 1 into the other buffer; wait the fragment reads
//   M0  the kk0 MFMAs (MI * NI)
//   L1  read the kk1 fragments; wait this wave's DMA pieces of step g + 1 (vmcnt 0)
//   M1  the kk1 MFMAs
// and after a tile's last step an E section runs the epilogue.  Group 1 starts one barrier late,
// so in every interval between two barriers one wave of each SIMD issues MFMAs while the other
// reads fragments, issues DMA or runs its epilogue (the 8-phase template of
// cdna_hip_programming.md §5, with this kernel's sections).
// Hazards (G0's section s shares an interval with G1's section s - 1):
//   WAR  the DMA of step g + 1 into buffer (g + 1) % 2 is issued in L0(g); that buffer's last
//        readers (L1(g - 1) of both groups) finished before the barrier ahead of G0's L0(g);
//   RAW  every wave waits its own DMA of step g + 1 in its L1(g); the first reader, G0's
//        L0(g + 1), starts after the barrier that ends G1's L1(g).
// Barrier counts: every wave runs 1 + 4 per K-step + 1 per tile, plus one extra (group 1 at the
// start, group 0 at the end).
#include <algorithm>
#include <type_traits>

#include "common.hpp"
#include "gemm_util.hpp"
#include "kernels.hpp"

namespace clipgpu {

namespace {

using namespace gemm_detail;

constexpr int PBK = 64;

// Race-check build (make poison: the product objects with this file and gemm.hip rebuilt with
// CLIPGPU_GEMM_POISON): every wave fills the 1 KiB destination of each of its LDS-DMAs with NaN
// bytes before issuing it, so a fragment read ahead of its DMA reads NaN (test_gpu_kernels.py).
#if CLIPGPU_GEMM_POISON
__device__ __forceinline__ void pp_poison(char* dst) { gemm_detail::lds_poison_piece(dst); }
#define PP_POISON(dst) pp_poison(dst)
#else
#define PP_POISON(dst) do {} while (0)
#endif

template <typename T>
__device__ __forceinline__ T to16pp(float v) { return (T)v; }

template <typename T, int BM, int EPI, int ACT>
__global__ __launch_bounds__(512, 2) void gemm_pp_kernel(GemmParams p) {
  typedef typename Vec8<T>::type V8;
  constexpr int BN = 256, NW = 8, WGN = 4;
  constexpr int A_BYTES = BM * PBK * 2, B_BYTES = BN * PBK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int PW = BN / 8, PA = BM / 8, PT = PW + PA, NP = PT / NW;
  static_assert(PT % NW == 0 && PW % NW == 0, "even DMA piece split, W pieces first");
  constexpr int TM = BM / 2, TN = BN / WGN, MI = TM / 16, NI = TN / 16, LG = 2;
  static_assert(NI == 4 && TM % 16 == 0, "tile");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + 2048];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave / WGN;
  const int nTn = (p.N + BN - 1) / BN;
  const int nTm = (p.M + BM - 1) / BM;
  const int ntiles = nTn * nTm;
  const int nk = p.K / PBK;

  // persistent schedule (gemm_pipe_kernel's): XCD x walks a contiguous range of tiles
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
    t_stride = ntiles;
    t_end = t_first + 1;
  }
  if (t_first >= t_end) return;
  const int total = ((t_end - t_first + t_stride - 1) / t_stride) * nk;

  auto swW = [](int r) { return (r & 2) | (((r >> (2 + LG)) & 1) << 2); };

  // ---- LDS-DMA cursor (step d_g = tile d_t, K-step d_kt), pieces q = wave + NW * i -----------
  uint32_t poff[NP];
  const char* const Wb = (const char*)p.W;
  const char* const Ab = (const char*)p.A;
  auto set_tile = [&](int m0, int n0) {
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int q = wave + NW * i;
      if (i < PW / NW) {
        const int r = q * 8 + (lane >> 3);
        const int c = (lane & 7) ^ swW(r);
        poff[i] = (uint32_t)(min(n0 + r, p.N - 1) * (int)p.ldw + c * 8) * 2u;
      } else {
        const int r = (q - PW) * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        poff[i] = (uint32_t)(min(m0 + r, p.M - 1) * (int)p.lda + c * 8) * 2u;
      }
    }
  };
  int d_g = 0, d_kt = 0, d_t = t_first, d_n0 = 0, d_ti = 0;
  {
    int m0, n0;
    tile_coords(d_t, nTm, nTn, BM, BN, m0, n0);
    set_tile(m0, n0);
    d_n0 = n0;
  }
  auto dma_step = [&]() {
    if (d_g < total) {
      char* const st = smem + (d_g & 1) * STAGE;
      static_for<NP>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const int q = wave + NW * i;
        char* const dst = i < PW / NW ? st + A_BYTES + q * 1024 : st + (q - PW) * 1024;
        PP_POISON(dst);
        if constexpr (i < PW / NW) glds16(Wb + (size_t)d_kt * (PBK * 2) + poff[i], dst);
        else glds16(Ab + (size_t)d_kt * (PBK * 2) + poff[i], dst);
      });
      if (p.bias != nullptr && wave == 0 && d_kt == 0) {  // the tile's bias slice (tile-parity slot)
        const int n = min(d_n0 + lane * 4, ((p.N - 1) / 4) * 4);
        PP_POISON(smem + 2 * STAGE + (d_ti & 1) * 1024);
        glds16(p.bias + n, smem + 2 * STAGE + (d_ti & 1) * 1024);
      }
    }
    ++d_g;
    if (++d_kt == nk) {
      d_kt = 0;
      d_t += t_stride;
      ++d_ti;
      if (d_t < t_end) {
        int m0, n0;
        tile_coords(d_t, nTm, nTn, BM, BN, m0, n0);
        set_tile(m0, n0);
        d_n0 = n0;
      }
    }
  };

  // ---- fragments (gemm_pipe_kernel's offsets) -------------------------------------------------
  const int wm = grp * TM, wn = (wave % WGN) * TN;
  const int fr = lane & 15, fq = lane >> 4;
  const int rowB = wn + (fr >> 2) * (4 * NI) + (fr & 3);
  uint32_t offA[2], offB[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    offA[kk] = (uint32_t)((wm + fr) * 128 + (((kk * 4 + fq) ^ (fr >> 1)) << 4));
    offB[kk] = (uint32_t)(A_BYTES + rowB * 128 + (((kk * 4 + fq) ^ swW(rowB)) << 4));
  }
  const uint32_t lds0 = lds_addr(smem);
  f32x4 acc[NI][MI];
  V8 a[MI], b[NI];
  auto read_frags = [&](uint32_t buf, int kk) {
    static_for<NI>([&](auto ni) { ds_read_b128<(int)ni * 512>(b[ni], buf + offB[kk]); });
    static_for<MI>([&](auto mi) { ds_read_b128<(int)mi * 2048>(a[mi], buf + offA[kk]); });
  };
  auto mfmas = [&](auto zero) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
        acc[ni][mi] = mfma_16x16x32(b[ni], a[mi], decltype(zero)::value ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[ni][mi]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto bar = []() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // ---- epilogue (gemm_pipe_kernel's float ops): lane owns row wm+mi*16+fr, columns nc .. +4NI-1
  auto epilogue = [&](int m0, int n0, int bpar) {
    const int nc = n0 + wn + fq * (4 * NI);
    const bool nfull = nc + 4 * NI <= p.N;
    f32x4 bias[NI];
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) bias[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (p.bias != nullptr) {
      const uint32_t ba = lds0 + 2 * STAGE + bpar * 1024 + (wn + fq * (4 * NI)) * 4;
      static_for<NI>([&](auto ni) { ds_read_b128<(int)ni * 16>(bias[ni], ba); });
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) asm volatile("" : "+v"(bias[ni]));
    }
    constexpr bool ADDX = EPI == EPI_RESID || EPI == EPI_PATCH;
    const int G2 = p.G * p.G;
    auto out_row = [&](int m) -> long {
      if constexpr (EPI == EPI_PATCH) {
        const int bb = m / G2;
        return ((long)bb * (G2 + p.cls) + p.cls + (m - bb * G2)) * p.ldo;
      } else {
        return (long)m * p.ldo;
      }
    };
    auto add_src = [&](int m) -> const float* {
      if constexpr (EPI == EPI_PATCH) return p.pos + (long)(p.cls + m % G2) * p.N + nc;
      else return (const float*)p.out + (long)m * p.ldo + nc;
    };
    // residual / positional rows: a ring of 2 row blocks loaded one ahead
    float4 xr[2][NI];
    auto load_x = [&](int mi, float4(&dst)[NI]) {
      const int m = m0 + wm + mi * 16 + fr;
      if (m < p.M && nfull) {
        const float* src = add_src(m);
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) dst[ni] = *(const float4*)(src + ni * 4);
      }
    };
    if constexpr (ADDX) load_x(0, xr[0]);
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      if constexpr (ADDX) {
        if (mi + 1 < MI) load_x(mi + 1, xr[(mi + 1) & 1]);
      }
      const int m = m0 + wm + mi * 16 + fr;
      if (m >= p.M) continue;
      float v[NI][4];
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int j = 0; j < 4; ++j) v[ni][j] = acc[ni][mi][j] + bias[ni][j];
      if constexpr (EPI == EPI_STORE16) {
        T* o = (T*)p.out + (long)m * p.ldo + nc;
        if (nfull) {
#pragma unroll
          for (int h = 0; h < NI / 2; ++h) {
            V8 w;
#pragma unroll
            for (int e = 0; e < 8; ++e) w[e] = to16pp<T>(apply_act<ACT>(v[2 * h + e / 4][e % 4]));
            *(V8*)(o + h * 8) = w;
          }
        } else {
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (nc + ni * 4 + j < p.N) o[ni * 4 + j] = to16pp<T>(apply_act<ACT>(v[ni][j]));
        }
      } else {
        float* o = (float*)p.out + out_row(m) + nc;
        if (nfull) {
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) {
            float4 w = make_float4(v[ni][0], v[ni][1], v[ni][2], v[ni][3]);
            if constexpr (ADDX) {
              const float4 x = xr[mi & 1][ni];
              w.x += x.x; w.y += x.y; w.z += x.z; w.w += x.w;
            }
            *(float4*)(o + ni * 4) = w;
          }
        } else {
          const float* xs = ADDX ? add_src(m) : nullptr;
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              if (nc + ni * 4 + j >= p.N) continue;
              float r = v[ni][j];
              if constexpr (ADDX) r += xs[ni * 4 + j];
              o[ni * 4 + j] = r;
            }
        }
      }
    }
  };

  // ---- prologue: step 0 landed in buffer 0; group 1 one barrier behind ------------------------
  dma_step();
  vm_wait<0>();
  bar();
  if (grp == 1) bar();

  int g = 0, ti = 0;
  for (int t = t_first; t < t_end; t += t_stride, ++ti) {
    int m0, n0;
    tile_coords(t, nTm, nTn, BM, BN, m0, n0);
    for (int kt = 0; kt < nk; ++kt, ++g) {
      const uint32_t buf = lds0 + (g & 1) * STAGE;
      // L0
      read_frags(buf, 0);
      dma_step();
      lgkm_wait_all(a, b);
      bar();
      // M0
      if (kt == 0) mfmas(std::true_type{});
      else mfmas(std::false_type{});
      bar();
      // L1
      read_frags(buf, 1);
      lgkm_wait_all(a, b);
      vm_wait<0>();
      bar();
      // M1
      mfmas(std::false_type{});
      bar();
    }
    // E
    epilogue(m0, n0, ti & 1);
    bar();
  }
  if (grp == 0) bar();
}

template <typename T, int BM, int EPI, int ACT>
hipError_t launch_pp_t(const GemmParams& p, hipStream_t s) {
  const int ntiles = ((p.N + 255) / 256) * ((p.M + BM - 1) / BM);
  const int resident = device_cus();
  const int grid = ntiles <= resident ? ntiles : resident;
  gemm_launch(gemm_pp_kernel<T, BM, EPI, ACT>, grid, 512, s, p);
  return hipGetLastError();
}

template <typename T, int BM>
hipError_t launch_pp_epi(int epi, int act, const GemmParams& p, hipStream_t s) {
  switch (epi) {
    case EPI_STORE16:
      switch (act) {
        case ACT_NONE: return launch_pp_t<T, BM, EPI_STORE16, ACT_NONE>(p, s);
        case ACT_QUICK_GELU: return launch_pp_t<T, BM, EPI_STORE16, ACT_QUICK_GELU>(p, s);
        case ACT_GELU: return launch_pp_t<T, BM, EPI_STORE16, ACT_GELU>(p, s);
        case ACT_GELU_TANH: return launch_pp_t<T, BM, EPI_STORE16, ACT_GELU_TANH>(p, s);
      }
      break;
    case EPI_RESID: return launch_pp_t<T, BM, EPI_RESID, ACT_NONE>(p, s);
    case EPI_STORE32: return launch_pp_t<T, BM, EPI_STORE32, ACT_NONE>(p, s);
    case EPI_PATCH: return launch_pp_t<T, BM, EPI_PATCH, ACT_NONE>(p, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace

// bm: 256 or 192 rows per tile (256 columns).  Preconditions (launch_tile): K % 64 == 0, K >= 128,
// no split-K, 16-bit outputs 16-byte aligned (ldo % 8 == 0), every operand within the 32-bit DMA
// offsets (launch_gemm's row chunks).
hipError_t launch_gemm_pp(DType dt, int bm, int epi, int act, const GemmParams& p, hipStream_t s) {
  if (p.ksplit > 1 || p.K % PBK || p.K < 2 * PBK) return hipErrorInvalidValue;
  if (bm == 256) return dt == DT_BF16 ? launch_pp_epi<__bf16, 256>(epi, act, p, s) : launch_pp_epi<_Float16, 256>(epi, act, p, s);
  if (bm == 192) return dt == DT_BF16 ? launch_pp_epi<__bf16, 192>(epi, act, p, s) : launch_pp_epi<_Float16, 192>(epi, act, p, s);
  return hipErrorInvalidValue;
}

}  // namespace clipgpu
