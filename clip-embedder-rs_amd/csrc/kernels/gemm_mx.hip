// MX-fp8 GEMM for the fp8 weight path (BASELINE.json configs[4]: DFN5B ViT-H/14-378 "fp8
// MFMA weight path").
//
//   C[M][N] = A[M][K] . W[N][K]^T  (+ fused epilogue)
//
// A and W are MX-fp8: OCP e4m3 elements with one E8M0 scale per 32 consecutive K
// elements of a row (kernels.hpp MxGemmParams).  The products run on the gfx950
// block-scaled MFMA v_mfma_scale_f32_32x32x64_f8f6f4, which applies the scales in
// hardware at twice the bf16 rate (MI355X_MICROARCH.md: the non-scaled fp8 MFMAs run at
// the bf16 rate, so only the scaled form pays).  Same machine as gemm.hip's pipelined
// kernel: one 128-byte K-step per LDS stage (128 fp8 elements instead of 64 bf16 --
// the same bytes and the same MFMA cycles per step, twice the K), staged by
// global_load_lds_dwordx4 into an XOR-swizzled lane-linear image, two MFMA phases of 64 K
// per step with one barrier between them, next step's fragments read under the current
// step's second phase, persistent XCD-aware tile walk.  The scale dwords of the step
// (4 blocks x rows) ride along as one global_load_lds_dword piece per wave.
//
// Operand maps of v_mfma_scale_f32_32x32x64_f8f6f4 (tools/mx_probe.hip, measured): lane l
// holds row l & 31 of its operand; its 32 bytes pair with the other operand's by (l >> 5,
// byte).  Bytes 0-15 of both lane halves form scale block 0 (scale from lane row), bytes
// 16-31 block 1 (scale from lane row + 32).  So for K-phase kk (64 elements) lane half h
// takes memory elements 16h..16h+15 into bytes 0-15 and 32+16h..+15 into bytes 16-31: the
// hardware blocks are then the memory blocks 2kk and 2kk+1, and lane half h supplies the
// scale of memory block 2kk + h (byte 2kk + h of the row's step dword; pre-shifted by 8h,
// selected with op_sel 2kk).
//
// Operands swapped as in gemm.hip: W rows are the MFMA "A" operand.  C/D: lane l holds
// output row m = l & 31 and W-fragment rows i = (r & 3) + 8 (r >> 2) + 4 (l >> 5); the W
// LDS image stores W row perm(i) = 16 ((i >> 2) & 1) + (i & 3) + 4 (i >> 3) at row i of
// each 32-row group, so register r of lane half h is output column 16 h + r: 16
// consecutive columns per lane (64-byte f32 / 32-byte 16-bit / 16-byte fp8 stores).
#include <algorithm>
#include <type_traits>
#include <utility>

#include "common.hpp"
#include "kernels.hpp"
#include "gemm_util.hpp"

namespace clipgpu {

namespace {

using namespace gemm_detail;

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));

constexpr int KB = 128;  // K-step: 128 e4m3 bytes per row

__device__ __forceinline__ int wperm(int i) { return 16 * ((i >> 2) & 1) + (i & 3) + 4 * (i >> 3); }

template <int OFF>
__device__ __forceinline__ void ds_read_b32(uint32_t& r, uint32_t addr) {
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
}

template <int OPS>
__device__ __forceinline__ f32x16 mfma_mx(const v4i (&w)[2], const v4i (&a)[2], f32x16 c, int sw, int sa) {
  const v8i wv = __builtin_shufflevector(w[0], w[1], 0, 1, 2, 3, 4, 5, 6, 7);
  const v8i av = __builtin_shufflevector(a[0], a[1], 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(wv, av, c, 0, 0, OPS, sw, OPS, sa);
}

template <typename T, int BM, int BN, int WGM, int WGN, int EPI, int ACT>
__global__ __launch_bounds__(WGM* WGN * 64, 2)
void gemm_mx_kernel(MxGemmParams p) {
  typedef typename Vec8<T>::type V8;
  constexpr int NW = WGM * WGN;
  constexpr int A_BYTES = BM * KB, B_BYTES = BN * KB, S_OFF = A_BYTES + B_BYTES;
  constexpr int STAGE = S_OFF + (BM + BN) * 4;
  constexpr int A_INSTR = BM / 8 / NW, B_INSTR = BN / 8 / NW;
  constexpr int NSC = (BM + BN) / 64;     // scale pieces (64 rows each): piece w + NW*j on wave w
  constexpr int SPW = (NSC + NW - 1) / NW;
  constexpr int NP = A_INSTR + B_INSTR + SPW;
  constexpr int TM = BM / WGM, TN = BN / WGN, MI = TM / 32, NI = TN / 32;
  static_assert(A_INSTR >= 1 && B_INSTR >= 1 && MI >= 1 && NI >= 1 && BN <= 256, "bad tile");
  static_assert(STAGE % 16 == 0, "stage alignment");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + 2048];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nTn = (p.N + BN - 1) / BN;
  const int nTm = (p.M + BM - 1) / BM;
  const int ntiles = nTn * nTm;
  const int nk = p.K / KB;

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

  // ---- LDS-DMA cursor ----------------------------------------------------------
  // 32-bit byte offsets from the kernel-argument bases (the DMA takes SGPR base + VGPR
  // offset; the host checks every operand fits in 2^31 bytes)
  uint32_t woff[B_INSTR], aoff[A_INSTR], soff[SPW];
  const char* const Wb = (const char*)p.W;
  const char* const Ab = (const char*)p.A;
  auto sbase = [&](int j) {  // wave-uniform: piece wave + NW*j stages A scales (< BM/64) or W scales
    return wave + NW * j < BM / 64 ? (const char*)p.As : (const char*)p.Ws;
  };
  auto set_tile = [&](int m0, int n0) {
#pragma unroll
    for (int i = 0; i < B_INSTR; ++i) {
      const int r = (wave * B_INSTR + i) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      const int n = min(n0 + (r & ~31) + wperm(r & 31), p.N - 1);
      woff[i] = (uint32_t)n * (uint32_t)p.ldw + (uint32_t)(c * 16);
    }
#pragma unroll
    for (int i = 0; i < A_INSTR; ++i) {
      const int r = (wave * A_INSTR + i) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      aoff[i] = (uint32_t)min(m0 + r, p.M - 1) * (uint32_t)p.lda + (uint32_t)(c * 16);
    }
#pragma unroll
    for (int j = 0; j < SPW; ++j) {
      const int pc = wave + NW * j;
      soff[j] = 0;
      if (pc < BM / 64) {
        soff[j] = (uint32_t)min(m0 + pc * 64 + lane, p.M - 1) * (uint32_t)p.ldas;
      } else if (pc < NSC) {
        const int r = (pc - BM / 64) * 64 + lane;
        soff[j] = (uint32_t)min(n0 + (r & ~31) + wperm(r & 31), p.N - 1) * (uint32_t)p.ldws;
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
  auto dma_piece = [&](auto jc) {  // W pieces, A pieces, then the scale piece
    constexpr int j = decltype(jc)::value;
    char* const st = smem + (d_g & 1) * STAGE;
    if constexpr (j < B_INSTR) {
      glds16(Wb + (size_t)d_kt * KB + woff[j], st + A_BYTES + (wave * B_INSTR + j) * 1024);
    } else if constexpr (j < B_INSTR + A_INSTR) {
      constexpr int i = j - B_INSTR;
      glds16(Ab + (size_t)d_kt * KB + aoff[i], st + (wave * A_INSTR + i) * 1024);
    } else {
      constexpr int jj = j - B_INSTR - A_INSTR;
      if (wave + NW * jj < NSC) glds4(sbase(jj) + (size_t)d_kt * 4 + soff[jj], st + S_OFF + (wave + NW * jj) * 256);
    }
  };
  auto dma_bias = [&]() {
    if (p.bias != nullptr && wave == 0 && d_kt == 0) {
      const int n = min(d_n0 + lane * 4, ((p.N - 1) / 4) * 4);
      glds16(p.bias + n, smem + 2 * STAGE + (d_ti & 1) * 1024);
    }
  };
  auto dma_advance = [&]() {
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
  auto dma_step = [&]() {
    if (d_g < total) {
      static_for<NP>([&](auto j) { dma_piece(j); });
      dma_bias();
    }
    dma_advance();
  };

  // ---- fragments ---------------------------------------------------------------
  const int wm = (wave / WGN) * TM, wn = (wave % WGN) * TN;
  const int r32 = lane & 31, h = lane >> 5;
  uint32_t offA[2][2], offB[2][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int part = 0; part < 2; ++part) {
      const int c = 4 * kk + 2 * part + h;
      offA[kk][part] = (uint32_t)((wm + r32) * KB + ((c ^ ((r32 >> 1) & 7)) << 4));
      offB[kk][part] = (uint32_t)(A_BYTES + (wn + r32) * KB + ((c ^ ((r32 >> 1) & 7)) << 4));
    }
  const uint32_t offSA = (uint32_t)(S_OFF + (wm + r32) * 4), offSB = (uint32_t)(S_OFF + BM * 4 + (wn + r32) * 4);
  const uint32_t hshift = 8u * (uint32_t)h;
  const uint32_t lds0 = lds_addr(smem);
  f32x16 acc[NI][MI];
  v4i a0[MI][2], b0[NI][2], a1[MI][2], b1[NI][2];
  // One scale dword per fragment row and K-step serves both phases (after the shift by 8h:
  // byte 0 = block 2*0 + h for phase 0, byte 2 = block 2 + h for phase 1), so the scales of
  // step g+1 are read in phase 1 of step g right after the last MFMA that uses step g's.
  uint32_t sa[MI], sb[NI];

  auto read_a = [&](v4i (&a)[2], uint32_t buf, int kk, auto mic) {
    constexpr int mi = decltype(mic)::value;
    ds_read_b128<mi * 32 * KB>(a[0], buf + offA[kk][0]);
    ds_read_b128<mi * 32 * KB>(a[1], buf + offA[kk][1]);
  };
  auto read_b = [&](v4i (&b)[NI][2], uint32_t buf, int kk) {
    static_for<NI>([&](auto ni) {
      ds_read_b128<(int)ni * 32 * KB>(b[ni][0], buf + offB[kk][0]);
      ds_read_b128<(int)ni * 32 * KB>(b[ni][1], buf + offB[kk][1]);
    });
  };
  auto read_sb = [&](uint32_t buf) {
    static_for<NI>([&](auto ni) { ds_read_b32<(int)ni * 128>(sb[ni], buf + offSB); });
  };
  // lgkmcnt(0) naming every fragment register (nothing reads them above it); with the
  // step's scales: each lane's scale bytes moved to the op_sel positions
  auto wait_frags = [&](v4i (&a)[MI][2], v4i (&b)[NI][2], bool scales) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < MI; ++i) asm volatile("" : "+v"(a[i][0]), "+v"(a[i][1]));
#pragma unroll
    for (int i = 0; i < NI; ++i) asm volatile("" : "+v"(b[i][0]), "+v"(b[i][1]));
    if (scales) {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        asm volatile("" : "+v"(sa[i]));
        sa[i] >>= hshift;
      }
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        asm volatile("" : "+v"(sb[i]));
        sb[i] >>= hshift;
      }
    }
  };
  auto read_step0 = [&](uint32_t buf) {  // kk0 fragments and the scales of a landed step
    read_b(b0, buf, 0);
    read_sb(buf);
    static_for<MI>([&](auto mi) {
      read_a(a0[mi], buf, 0, mi);
      ds_read_b32<(int)mi * 128>(sa[mi], buf + offSA);
    });
    wait_frags(a0, b0, true);
  };
  auto phase0 = [&](auto zero, uint32_t buf) {
    read_b(b1, buf, 1);
    static_for<MI>([&](auto mi) {
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        f32x16 c = {};
        if constexpr (!decltype(zero)::value) c = acc[ni][mi];
        acc[ni][mi] = mfma_mx<0>(b0[ni], a0[mi], c, (int)sb[ni], (int)sa[mi]);
      }
      __builtin_amdgcn_sched_barrier(0);
      read_a(a1[mi], buf, 1, mi);
    });
    wait_frags(a1, b1, false);
  };
  auto phase1 = [&](bool next, uint32_t nbuf) {
    const bool dma = d_g < total;
    // the next step's kk0 fragments are read unconditionally (on a tile's last step from
    // the other buffer, unused): a conditional read made the compiler keep a second copy
    // of the fragment registers across the branch
    read_b(b0, nbuf, 0);
    if (dma) dma_bias();
    static_for<MI>([&](auto mi) {
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
        acc[ni][mi] = mfma_mx<2>(b1[ni], a1[mi], acc[ni][mi], (int)sb[ni], (int)sa[mi]);
      __builtin_amdgcn_sched_barrier(0);
      {
        read_a(a0[mi], nbuf, 0, mi);
        ds_read_b32<(int)mi * 128>(sa[mi], nbuf + offSA);
        if constexpr ((int)mi + 1 == MI) read_sb(nbuf);
      }
      static_for<NP>([&](auto j) {
        if constexpr (((int)j * MI) / NP == (int)mi) {
          if (dma) dma_piece(j);
        }
      });
      __builtin_amdgcn_sched_barrier(0);
    });
    dma_advance();
    wait_frags(a0, b0, true);
    (void)next;
  };

  // ---- epilogue: lane owns row wm + mi*32 + r32, columns wn + ni*32 + 16h .. +15 ------
  auto epilogue = [&](int m0, int n0, int bpar) {
    // the tile's bias slice (LDS, staged with its first K-step), read per 16-column group
    const float* const bsl = (const float*)(smem + 2 * STAGE + bpar * 1024) + wn + 16 * h;
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int m = m0 + wm + mi * 32 + r32;
      if (m >= p.M) continue;  // (lanes l and l ^ 32 share m: the STOREQ swap stays paired)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const int nc = n0 + wn + ni * 32 + 16 * h;
        if (nc >= p.N) continue;  // N % 32 == 0: both halves of a 32-column block agree
        float v[16];
        if (p.bias != nullptr) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 bq = *(const float4*)(bsl + ni * 32 + 4 * q);
            v[4 * q] = acc[ni][mi][4 * q] + bq.x;
            v[4 * q + 1] = acc[ni][mi][4 * q + 1] + bq.y;
            v[4 * q + 2] = acc[ni][mi][4 * q + 2] + bq.z;
            v[4 * q + 3] = acc[ni][mi][4 * q + 3] + bq.w;
          }
        } else {
#pragma unroll
          for (int j = 0; j < 16; ++j) v[j] = acc[ni][mi][j];
        }
        if constexpr (EPI == EPI_STORE16) {
          T* o = (T*)p.out + (long)m * p.ldo + nc;
#pragma unroll
          for (int half = 0; half < 2; ++half) {
            V8 w;
#pragma unroll
            for (int e = 0; e < 8; ++e) w[e] = (T)apply_act<ACT>(v[8 * half + e]);
            *(V8*)(o + 8 * half) = w;
          }
        } else if constexpr (EPI == EPI_STOREQ) {
          float amax = 0.f;
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            v[j] = apply_act<ACT>(v[j]);
            amax = fmaxf(amax, fabsf(v[j]));
          }
          amax = xmax32(amax);  // the 32-column block: this lane's 16 and lane ^ 32's
          const int e = mx_exp(amax);
          const float inv = mx_inv(e);
          uint4 w;
          w.x = mx_pack4(v[0], v[1], v[2], v[3], inv);
          w.y = mx_pack4(v[4], v[5], v[6], v[7], inv);
          w.z = mx_pack4(v[8], v[9], v[10], v[11], inv);
          w.w = mx_pack4(v[12], v[13], v[14], v[15], inv);
          *(uint4*)((uint8_t*)p.out + (long)m * p.ldo + nc) = w;
          if (h == 0) p.outs[(long)m * p.ldos + (nc >> 5)] = (uint8_t)(e + 127);
        } else {
          // (EPI_RESID16: the residual stream in f16)
          typedef typename std::conditional<EPI == EPI_RESID16, _Float16, float>::type XE;
          XE* o = (XE*)p.out + (long)m * p.ldo + nc;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float4 w = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
            if constexpr (epi_resid(EPI)) {
              const float4 x = ldx4(o + 4 * q);
              w.x += x.x; w.y += x.y; w.z += x.z; w.w += x.w;
            }
            stx4(o + 4 * q, w);
          }
        }
      }
    }
  };
  // vm ops a full tile's epilogue leaves in flight behind the DMA of the step after it
  constexpr int EPI_VM = EPI == EPI_STORE16 ? 2 * MI * NI
                         : EPI == EPI_STOREQ ? 2 * MI * NI
                         : epi_resid(EPI)    ? 8 * MI * NI
                                             : 4 * MI * NI;

  // ---- prologue: steps 0 and 1 in flight, step 0 landed, its kk0 fragments read ----
  dma_step();
  vm_wait<0>();
  __builtin_amdgcn_s_barrier();
  dma_step();
  read_step0(lds0);

  int g = 0;
  bool after_full_epi = false;
  int ti = 0;
  for (int t = t_first; t < t_end; t += t_stride, ++ti) {
    int m0, n0;
    tile_coords(t, nTm, nTn, BM, BN, m0, n0);
    for (int kt = 0; kt < nk; ++kt, ++g) {
      const uint32_t buf = lds0 + (g & 1) * STAGE;
      if (kt == 0) phase0(std::true_type{}, buf);
      else phase0(std::false_type{}, buf);
      if (after_full_epi) vm_wait<(EPI_VM < 63 ? EPI_VM : 63)>();
      else vm_wait<0>();
      after_full_epi = false;
      __builtin_amdgcn_s_barrier();
      phase1(kt + 1 < nk, lds0 + ((g + 1) & 1) * STAGE);
    }
    vm_wait<0>();  // the next step's LDS-DMA lands before the epilogue's stores (gemm.hip gemm_pipe_kernel)
    epilogue(m0, n0, ti & 1);
    after_full_epi = m0 + BM <= p.M && n0 + BN <= p.N;
    if (!after_full_epi) vm_wait<0>();
    if (t + t_stride < t_end) {  // the next tile's step 0 landed at the last barrier
      read_step0(lds0 + (g & 1) * STAGE);
    }
  }
}

template <typename T, int BM, int BN, int WGM, int WGN, int EPI, int ACT>
hipError_t launch_mx_cfg(const MxGemmParams& p, hipStream_t s) {
  const int ntiles = ((p.N + BN - 1) / BN) * ((p.M + BM - 1) / BM);
  const int lds = 2 * ((BM + BN) * KB + (BM + BN) * 4) + 2048;
  const int per_cu = WGM * WGN == 8 ? 1 : std::min(2, (160 * 1024) / lds);
  const int resident = device_cus() * per_cu;
  const int grid = ntiles <= resident ? ntiles : resident;
  gemm_launch(gemm_mx_kernel<T, BM, BN, WGM, WGN, EPI, ACT>, grid, WGM * WGN * 64, s, p);
  return hipGetLastError();
}

// 128x128 (two 4-wave blocks per CU) measured faster than 256x128 at every trunk shape
// (profiles/r01_v11_mx_sweep.jsonl: 1.2-1.5 vs 1.0-1.3 PFLOP/s); the engine autotunes per site.
int pick_mx_tile(int M, int N) {
  (void)M;
  (void)N;
  return MX_TILE_128x128;
}

template <typename T, int EPI, int ACT>
hipError_t launch_mx_tile(const MxGemmParams& p, hipStream_t s) {
  switch (p.tile == MX_TILE_AUTO ? pick_mx_tile(p.M, p.N) : p.tile) {
    case MX_TILE_256x128: return launch_mx_cfg<T, 256, 128, 4, 2, EPI, ACT>(p, s);
    default: return launch_mx_cfg<T, 128, 128, 2, 2, EPI, ACT>(p, s);
  }
}

template <typename T, int EPI>
hipError_t launch_mx_act(int act, const MxGemmParams& p, hipStream_t s) {
  switch (act) {
    case ACT_NONE: return launch_mx_tile<T, EPI, ACT_NONE>(p, s);
    case ACT_QUICK_GELU: return launch_mx_tile<T, EPI, ACT_QUICK_GELU>(p, s);
    case ACT_GELU: return launch_mx_tile<T, EPI, ACT_GELU>(p, s);
    case ACT_GELU_TANH: return launch_mx_tile<T, EPI, ACT_GELU_TANH>(p, s);
  }
  return hipErrorInvalidValue;
}

template <typename T>
hipError_t launch_mx_typed(int epi, int act, const MxGemmParams& p, hipStream_t s) {
  switch (epi) {
    case EPI_STORE16: return launch_mx_act<T, EPI_STORE16>(act, p, s);
    case EPI_STOREQ: return launch_mx_act<T, EPI_STOREQ>(act, p, s);
    case EPI_RESID:  // the residual stream: f32, or f16 (MxGemmParams.x16)
      if (act != ACT_NONE) return hipErrorInvalidValue;
      return p.x16 ? launch_mx_tile<T, EPI_RESID16, ACT_NONE>(p, s) : launch_mx_tile<T, EPI_RESID, ACT_NONE>(p, s);
    case EPI_STORE32: return act == ACT_NONE ? launch_mx_tile<T, EPI_STORE32, ACT_NONE>(p, s) : hipErrorInvalidValue;
  }
  return hipErrorInvalidValue;
}

// One thread per 32-element block: amax -> E8M0 exponent -> 32 e4m3 bytes + 1 scale byte.
template <typename S>
__global__ __launch_bounds__(256) void quant_rows_kernel(const S* __restrict__ src, long ld, uint8_t* __restrict__ q,
                                                         long ldq, uint8_t* __restrict__ qs, long ldqs, int rows,
                                                         int cols) {
  const int nbk = cols >> 5;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)rows * nbk) return;
  const int r = (int)(t / nbk), bk = (int)(t - (long)r * nbk);
  const S* x = src + (long)r * ld + bk * 32;
  float v[32];
  float amax = 0.f;
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    v[j] = (float)x[j];
    amax = fmaxf(amax, fabsf(v[j]));
  }
  const int e = mx_exp(amax);
  const float inv = mx_inv(e);
  uint4* o = (uint4*)(q + (long)r * ldq + bk * 32);
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    uint4 w;
    w.x = mx_pack4(v[16 * c + 0], v[16 * c + 1], v[16 * c + 2], v[16 * c + 3], inv);
    w.y = mx_pack4(v[16 * c + 4], v[16 * c + 5], v[16 * c + 6], v[16 * c + 7], inv);
    w.z = mx_pack4(v[16 * c + 8], v[16 * c + 9], v[16 * c + 10], v[16 * c + 11], inv);
    w.w = mx_pack4(v[16 * c + 12], v[16 * c + 13], v[16 * c + 14], v[16 * c + 15], inv);
    o[c] = w;
  }
  qs[(long)r * ldqs + bk] = (uint8_t)(e + 127);
}

}  // namespace

hipError_t launch_gemm_mx(DType dt, int epi, int act, const MxGemmParams& p, hipStream_t s) {
  if (p.M <= 0 || p.N <= 0 || p.K <= 0 || p.K % KB != 0 || p.N % 32 != 0) return hipErrorInvalidValue;
  if (p.tile < MX_TILE_AUTO || p.tile > MX_TILE_LAST || p.tile == MX_TILE_256x256) return hipErrorInvalidValue;
  // 16-byte row DMA, dword scale DMA, 32-bit staging offsets
  if (p.lda % 16 || p.ldw % 16 || p.ldas % 4 || p.ldws % 4 || p.lda < p.K || p.ldw < p.K || p.ldas < p.K / 32 ||
      p.ldws < p.K / 32)
    return hipErrorInvalidValue;
  if ((long)p.N * p.ldw >= (1L << 31)) return hipErrorInvalidValue;
  if (epi == EPI_STOREQ && (p.outs == nullptr || p.ldo % 16 || p.ldos < p.N / 32)) return hipErrorInvalidValue;
  if (epi == EPI_STORE16 && p.ldo % 8) return hipErrorInvalidValue;
  if ((epi == EPI_RESID || epi == EPI_STORE32) && p.ldo % 4) return hipErrorInvalidValue;
  if ((long)p.M * p.lda >= (1L << 31)) {
    // 32-bit per-lane staging offsets (as launch_gemm): consecutive row chunks of whole 256-row
    // tiles, bit-invisible (per-row scales, per-row MFMA chains)
    long chunk = ((1L << 31) - 1) / p.lda;
    chunk -= chunk % 256;
    const long osz = epi == EPI_STORE16 || (epi == EPI_RESID && p.x16) ? 2 : (epi == EPI_STOREQ ? 1 : 4);
    for (long m0 = 0; m0 < p.M; m0 += chunk) {
      MxGemmParams q = p;
      q.M = (int)std::min<long>(chunk, p.M - m0);
      q.A = p.A + m0 * p.lda;
      q.As = p.As + m0 * p.ldas;
      q.out = (char*)p.out + m0 * p.ldo * osz;
      if (p.outs) q.outs = p.outs + m0 * p.ldos;
      const hipError_t err =
          dt == DT_BF16 ? launch_mx_typed<__bf16>(epi, act, q, s) : launch_mx_typed<_Float16>(epi, act, q, s);
      if (err != hipSuccess) return err;
    }
    return hipSuccess;
  }
  return dt == DT_BF16 ? launch_mx_typed<__bf16>(epi, act, p, s) : launch_mx_typed<_Float16>(epi, act, p, s);
}

hipError_t launch_quant_rows(int src_dt, const void* src, long ld, uint8_t* q, long ldq, uint8_t* qs, long ldqs,
                             int rows, int cols, hipStream_t s) {
  if (rows <= 0 || cols <= 0 || cols % 32 || ldq % 16 || ldq < cols || ldqs < cols / 32 || ld < cols)
    return hipErrorInvalidValue;
  const long n = (long)rows * (cols / 32);
  const dim3 grid((unsigned)((n + 255) / 256));
  if (src_dt < 0)
    hipLaunchKernelGGL(quant_rows_kernel<float>, grid, dim3(256), 0, s, (const float*)src, ld, q, ldq, qs, ldqs, rows,
                       cols);
  else if (src_dt == DT_BF16)
    hipLaunchKernelGGL(quant_rows_kernel<__bf16>, grid, dim3(256), 0, s, (const __bf16*)src, ld, q, ldq, qs, ldqs,
                       rows, cols);
  else
    hipLaunchKernelGGL(quant_rows_kernel<_Float16>, grid, dim3(256), 0, s, (const _Float16*)src, ld, q, ldq, qs, ldqs,
                       rows, cols);
  return hipGetLastError();
}

}  // namespace clipgpu
