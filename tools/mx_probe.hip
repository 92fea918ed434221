// Probe of the gfx950 block-scaled MFMA and fp8 conversions the MX-fp8 GEMM relies on
// (run on the GPU box: hipcc --offload-arch=gfx950 -O3 tools/mx_probe.hip -o /tmp/mx_probe).
//   1. v_mfma_scale_f32_32x32x64_f8f6f4 operand map: lane l holds row (A) / column (B)
//      l & 31, k = 32 (l >> 5) + byte j; C/D: col = l & 31, row = (r & 3) + 8 (r >> 2) + 4 (l >> 5).
//   2. its E8M0 scales: lane l's scale register, byte `opsel`, scales row/column l & 31 of
//      k-block l >> 5.
//   3. v_cvt_pk_fp8_f32 against a host round-to-nearest-even e4m3fn encoder, and what
//      v_cvt_scalef32_pk_fp8_f32 does with its scale.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef short v2s __attribute__((ext_vector_type(2)));

template <int OA, int OB>
__global__ void mfma_k(const v8i* a, const v8i* b, const int* sa, const int* sb, v16f* c) {
  const int l = threadIdx.x;
  v16f acc = {};
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[l], b[l], acc, 0, 0, OA, sa[l], OB, sb[l]);
  c[l] = acc;
}

__global__ void cvt_k(const float* f, int n, int* o, int* os) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  o[i] = __builtin_amdgcn_cvt_pk_fp8_f32(f[i], f[i], 0, false) & 0xff;
  v2s z = {0, 0};
  os[i] = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(z, f[i], f[i], 4.0f, false)[0] & 0xff;
}

static float dec(uint8_t v) {  // e4m3fn
  const int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  if (e == 15 && m == 7) return NAN;
  const float x = e == 0 ? std::ldexp((float)m, -9) : std::ldexp(1.0f + m / 8.0f, e - 7);
  return s ? -x : x;
}
static uint8_t enc(float x) {  // RNE, saturate to 448 (inputs here are in range)
  uint8_t best = 0;
  float bd = INFINITY;
  for (int v = 0; v < 256; ++v) {
    const float d = dec((uint8_t)v);
    if (std::isnan(d)) continue;
    const float err = std::fabs(d - x);
    if (err < bd || (err == bd && (v & 1) == 0 && (best & 1))) {
      bd = err;
      best = (uint8_t)v;
    }
  }
  if (dec(best) == 0.0f && std::signbit(x)) return 0x80;  // RNE to zero keeps the sign
  return best;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e_)); return 1; } } while (0)

template <int OA, int OB>
int run_mfma(const uint8_t (&A)[32][64], const uint8_t (&B)[64][32], const int* sa, const int* sb, int& bad) {
  uint8_t ha[64][32], hb[64][32];
  for (int l = 0; l < 64; ++l)
    for (int j = 0; j < 32; ++j) {
      ha[l][j] = A[l & 31][32 * (l >> 5) + j];
      hb[l][j] = B[32 * (l >> 5) + j][l & 31];
    }
  void *da, *db, *dsa, *dsb, *dc;
  CK(hipMalloc(&da, sizeof ha)); CK(hipMalloc(&db, sizeof hb)); CK(hipMalloc(&dsa, 256)); CK(hipMalloc(&dsb, 256));
  CK(hipMalloc(&dc, 64 * 64 * 4));
  CK(hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice));
  CK(hipMemcpy(dsa, sa, 256, hipMemcpyHostToDevice));
  CK(hipMemcpy(dsb, sb, 256, hipMemcpyHostToDevice));
  hipLaunchKernelGGL((mfma_k<OA, OB>), dim3(1), dim3(64), 0, 0, (const v8i*)da, (const v8i*)db, (const int*)dsa,
                     (const int*)dsb, (v16f*)dc);
  float c[64][16];
  CK(hipMemcpy(c, dc, sizeof c, hipMemcpyDeviceToHost));
  bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 16; ++r) {
      const int col = l & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
      double ref = 0;
      for (int k = 0; k < 64; ++k) {
        // the scale block of the element in byte j = k & 31 of lane half k >> 5: bytes 0-15
        // of both halves are block 0, bytes 16-31 block 1 (MX_H1: block = lane half)
        const int blk = getenv("MX_H1") ? k >> 5 : (k & 31) >> 4;
        const int ea = ((sa[row + 32 * blk] >> (8 * OA)) & 255) - 127;
        const int eb = ((sb[col + 32 * blk] >> (8 * OB)) & 255) - 127;
        ref += (double)dec(A[row][k]) * std::ldexp(1.0, ea) * dec(B[k][col]) * std::ldexp(1.0, eb);
      }
      if (std::fabs(ref - c[l][r]) > 1e-6 * (1 + std::fabs(ref))) ++bad;
    }
  (void)hipFree(da); (void)hipFree(db); (void)hipFree(dsa); (void)hipFree(dsb); (void)hipFree(dc);
  return 0;
}

int main() {
  srand(7);
  static uint8_t A[32][64], B[64][32];
  const float vals[] = {-2.f, -1.5f, -1.f, -0.5f, 0.f, 0.5f, 1.f, 1.5f, 2.f, 3.f};
  for (auto& row : A) for (auto& v : row) v = enc(vals[rand() % 10]);
  for (auto& row : B) for (auto& v : row) v = enc(vals[rand() % 10]);
  int sa[64], sb[64], one[64];
  for (int l = 0; l < 64; ++l) {
    one[l] = 0x7f7f7f7f;
    sa[l] = sb[l] = 0;
    for (int byte = 0; byte < 4; ++byte) {
      sa[l] |= (127 + rand() % 5 - 2) << (8 * byte);
      sb[l] |= (127 + rand() % 5 - 2) << (8 * byte);
    }
  }
  int bad = 0, fails = 0;
  if (getenv("MX_DISCOVER")) {
    // all-ones operands, one lane's scale byte doubled: which rows / columns change
    static uint8_t O[32][64], OB[64][32];
    memset(O, 0x38, sizeof O);
    memset(OB, 0x38, sizeof OB);
    for (int side = 0; side < 2; ++side)
      for (int byte = 0; byte < 4; ++byte) {
        printf("%s byte %d:", side ? "B" : "A", byte);
        for (int L = 0; L < 64; L += 1) {
          int s1[64];
          for (int l = 0; l < 64; ++l) s1[l] = 0x7f7f7f7f;
          s1[L] = (int)((0x7f7f7f7fu & ~(0xffu << (8 * byte))) | (0x80u << (8 * byte)));
          void *da, *db, *dsa, *dsb, *dc;
          uint8_t ha[64][32], hb[64][32];
          memset(ha, 0x38, sizeof ha); memset(hb, 0x38, sizeof hb);
          CK(hipMalloc(&da, 2048)); CK(hipMalloc(&db, 2048)); CK(hipMalloc(&dsa, 256)); CK(hipMalloc(&dsb, 256)); CK(hipMalloc(&dc, 4096));
          CK(hipMemcpy(da, ha, 2048, hipMemcpyHostToDevice)); CK(hipMemcpy(db, hb, 2048, hipMemcpyHostToDevice));
          CK(hipMemcpy(dsa, side ? one : s1, 256, hipMemcpyHostToDevice)); CK(hipMemcpy(dsb, side ? s1 : one, 256, hipMemcpyHostToDevice));
          switch (byte) {
            case 0: hipLaunchKernelGGL((mfma_k<0, 0>), dim3(1), dim3(64), 0, 0, (const v8i*)da, (const v8i*)db, (const int*)dsa, (const int*)dsb, (v16f*)dc); break;
            case 1: hipLaunchKernelGGL((mfma_k<1, 1>), dim3(1), dim3(64), 0, 0, (const v8i*)da, (const v8i*)db, (const int*)dsa, (const int*)dsb, (v16f*)dc); break;
            case 2: hipLaunchKernelGGL((mfma_k<2, 2>), dim3(1), dim3(64), 0, 0, (const v8i*)da, (const v8i*)db, (const int*)dsa, (const int*)dsb, (v16f*)dc); break;
            default: hipLaunchKernelGGL((mfma_k<3, 3>), dim3(1), dim3(64), 0, 0, (const v8i*)da, (const v8i*)db, (const int*)dsa, (const int*)dsb, (v16f*)dc); break;
          }
          float c[64][16];
          CK(hipMemcpy(c, dc, sizeof c, hipMemcpyDeviceToHost));
          (void)hipFree(da); (void)hipFree(db); (void)hipFree(dsa); (void)hipFree(dsb); (void)hipFree(dc);
          // summarise: changed entries as row/col sets and the value
          int rows[32] = {0}, cols[32] = {0}; float val = 0; int nch = 0;
          for (int l = 0; l < 64; ++l) for (int r = 0; r < 16; ++r) {
            const int col = l & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
            if (c[l][r] != 64.f) { rows[row] = 1; cols[col] = 1; val = c[l][r]; ++nch; }
          }
          printf(" L%d:", L);
          if (!nch) { printf("-"); continue; }
          int nr = 0, nc = 0, r0 = -1, c0 = -1;
          for (int i = 0; i < 32; ++i) { if (rows[i]) { ++nr; if (r0 < 0) r0 = i; } if (cols[i]) { ++nc; if (c0 < 0) c0 = i; } }
          printf("r%d(%d)c%d(%d)=%g", r0, nr, c0, nc, val);
        }
        printf("\n");
      }
    return 0;
  }
  if (run_mfma<0, 0>(A, B, one, one, bad)) return 1;
  printf("layout (unit scales): %d / 1024 mismatches\n", bad); fails += bad != 0;
  if (getenv("MX_DISCOVER2")) {
    int hi[64], ra[64];
    for (int l = 0; l < 64; ++l) { hi[l] = l >= 32 ? 0x80808080 : 0x7f7f7f7f; ra[l] = sa[l]; }
    if (run_mfma<0, 0>(A, B, hi, one, bad)) return 1;
    printf("A: lanes 32-63 x2: %d mismatches\n", bad);
    if (run_mfma<0, 0>(A, B, one, hi, bad)) return 1;
    printf("B: lanes 32-63 x2: %d mismatches\n", bad);
    if (run_mfma<0, 0>(A, B, ra, one, bad)) return 1;
    printf("A random, B unit: %d mismatches\n", bad);
    if (run_mfma<0, 0>(A, B, one, sb, bad)) return 1;
    printf("A unit, B random: %d mismatches\n", bad);
    for (int l = 0; l < 64; ++l) ra[l] = 0x7f7f7f00 | (127 + (l & 1));
    if (run_mfma<0, 0>(A, B, ra, one, bad)) return 1;
    printf("A odd lanes x2: %d mismatches\n", bad);
    for (int l = 0; l < 64; ++l) ra[l] = 0x7f7f7f00 | (127 + ((l >> 3) & 1));
    if (run_mfma<0, 0>(A, B, ra, one, bad)) return 1;
    printf("A lanes with bit 3 x2: %d mismatches\n", bad);
    for (int l = 0; l < 64; ++l) ra[l] = 0x7f7f7f00 | (126 + (l & 3));
    if (run_mfma<0, 0>(A, B, ra, one, bad)) return 1;
    printf("A lanes scale 2^((l&3)-1): %d mismatches\n", bad);
  }
  if (run_mfma<0, 0>(A, B, sa, sb, bad)) return 1;
  printf("scales opsel 0/0: %d mismatches\n", bad); fails += bad != 0;
  if (run_mfma<2, 1>(A, B, sa, sb, bad)) return 1;
  printf("scales opsel 2/1: %d mismatches\n", bad); fails += bad != 0;
  if (run_mfma<3, 3>(A, B, sa, sb, bad)) return 1;
  printf("scales opsel 3/3: %d mismatches\n", bad); fails += bad != 0;

  // conversions: every e4m3 value, midpoints between neighbours, and out-of-range inputs
  std::vector<float> f;
  for (int v = 0; v < 256; ++v) {
    const float d = dec((uint8_t)v);
    if (std::isnan(d)) continue;
    f.push_back(d);
    const float d2 = dec((uint8_t)(v + 1));
    if ((v & 0x7f) < 0x7e && !std::isnan(d2)) f.push_back(0.5f * (d + d2));
    f.push_back(d * 1.03f);
  }
  const int n = (int)f.size();
  float* df; int *dout, *douts;
  CK(hipMalloc(&df, n * 4)); CK(hipMalloc(&dout, n * 4)); CK(hipMalloc(&douts, n * 4));
  CK(hipMemcpy(df, f.data(), n * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(cvt_k, dim3((n + 255) / 256), dim3(256), 0, 0, df, n, dout, douts);
  std::vector<int> o(n), os(n);
  CK(hipMemcpy(o.data(), dout, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(os.data(), douts, n * 4, hipMemcpyDeviceToHost));
  int cbad = 0, smul = 0, sdiv = 0, inr = 0;
  for (int i = 0; i < n; ++i) {
    if (std::fabs(f[i]) <= 448.f) {
      ++inr;
      if (o[i] != enc(f[i])) {
        if (cbad < 5) printf("cvt %.8g -> %02x, host %02x\n", f[i], o[i], enc(f[i]));
        ++cbad;
      }
    }
    if (std::fabs(f[i] * 4.f) <= 448.f && os[i] == enc(f[i] * 4.f)) ++smul;
    if (os[i] == enc(f[i] / 4.f)) ++sdiv;
  }
  int sat = 0;
  for (int i = 0; i < n; ++i) if (std::fabs(f[i]) > 448.f && i < 4000) { printf("out of range %.6g -> %02x\n", f[i], o[i]); if (++sat > 3) break; }
  printf("cvt_pk_fp8_f32: %d / %d in-range mismatches vs RNE\n", cbad, inr); fails += cbad != 0;
  printf("cvt_scalef32 (scale 4): matches x*4 on %d, x/4 on %d of %d\n", smul, sdiv, n);
  printf(fails ? "PROBE FAILED\n" : "PROBE OK\n");
  return fails ? 1 : 0;
}
