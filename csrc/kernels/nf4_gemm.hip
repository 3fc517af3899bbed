// K8 (part 2): fused NF4-dequant + bf16 MFMA GEMM for QLoRA, y[M, N] = x[M, K] . W^T with W kept as
// 4-bit NormalFloat codes (nf4.hip format: blocks of 64 along K, high nibble first, double-quantised
// absmax).  The bf16 weight never exists in memory: codes are decoded straight into MFMA B fragments.
//
// Used for small M (decode / evaluation / tiny micro-batches, ops/nf4.py FUSED_MAX_ROWS) where the
// GEMM is bound by the weight stream: 0.52 B/param instead of 2 B/param (bf16) or 4.5 B/param
// (dequantise to bf16, then a library GEMM).
//
// Geometry: a 512-thread workgroup owns 32 output features (n) x 32*MT rows (m); its 8 waves split the
// K blocks 8 ways (wave w takes blocks w, w+8, ...) and are summed through LDS at the end.
// Per 64-wide K block a lane (n = lane&31, half h = lane>>5) loads the 16 packed bytes of
// W[n][64kb + 32h .. +32) and decodes them into four bf16x8 B fragments.  MFMA k order is permuted
// (k-step s, half h covers k = 32h + 8s + j): the A fragments read x with the same permutation, so
// each lane's x reads are 64 contiguous bytes and the sum is unchanged.
#include "common.h"

using namespace ftc;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int WAVES = 8;

__constant__ float kCode[16] = {-1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f,
                                -0.28444138169288635f, -0.18477343022823334f, -0.09105003625154495f, 0.0f,
                                0.07958029955625534f, 0.16093020141124725f, 0.24611230194568634f,
                                0.33791524171829224f, 0.44070982933044434f, 0.5626170039176941f,
                                0.7229568362236023f, 1.0f};

template <int MT>
__global__ __launch_bounds__(512) void nf4_gemm_kernel(const uint16_t* __restrict__ x, const uint8_t* __restrict__ packed,
                                                       const uint8_t* __restrict__ aq, const float* __restrict__ s2,
                                                       float off, uint16_t* __restrict__ y, int M, int N, int K,
                                                       int block2) {
  __shared__ float code[16];
  extern __shared__ __attribute__((aligned(16))) float red[];  // [WAVES][MT][16][64]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5, lr = lane & 31;
  if (tid < 16) code[tid] = kCode[tid];
  __syncthreads();

  const int n0 = blockIdx.x * 32;
  const int m0 = blockIdx.y * 32 * MT;
  const int n = n0 + lr;
  const int nkb = K >> 6;
  const long long row_bytes = K >> 1;

  f32x16 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;

  // this lane's x rows (clamped; rows >= M contribute zeros)
  const uint16_t* xrow[MT];
  bool mval[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    const int m = m0 + t * 32 + lr;
    mval[t] = m < M;
    xrow[t] = x + (long long)(mval[t] ? m : 0) * K + 32 * hh;
  }
  const uint8_t* wrow = packed + (long long)n * row_bytes + 16 * hh;

  for (int kb = wave; kb < nkb; kb += WAVES) {
    // ---- B: decode 32 codes of W[n][64kb + 32h ..] into 4 bf16x8 fragments
    const uint4 p = *reinterpret_cast<const uint4*>(wrow + (long long)kb * 32);
    const long long bi = (long long)n * nkb + kb;
    const float a = off + ((float)aq[bi] - 128.0f) * (1.0f / 127.0f) * s2[bi / block2];
    bf16x8 bf[4];
    const uint32_t words[4] = {p.x, p.y, p.z, p.w};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const uint32_t wd = words[s];  // 4 bytes = 8 codes = k 32h + 8s + [0, 8)
      uint4 u;
      u.x = pack_bf2(code[(wd >> 4) & 15] * a, code[wd & 15] * a);
      u.y = pack_bf2(code[(wd >> 12) & 15] * a, code[(wd >> 8) & 15] * a);
      u.z = pack_bf2(code[(wd >> 20) & 15] * a, code[(wd >> 16) & 15] * a);
      u.w = pack_bf2(code[(wd >> 28) & 15] * a, code[(wd >> 24) & 15] * a);
      bf[s] = __builtin_bit_cast(bf16x8, u);
    }
    // ---- A: x[m][64kb + 32h + 8s .. +8] (same permuted k order), 4 MFMAs per row tile
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const uint4* xp = reinterpret_cast<const uint4*>(xrow[t] + kb * 64);
      uint4 xa[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) xa[s] = mval[t] ? xp[s] : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int s = 0; s < 4; ++s)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, xa[s]), bf[s], acc[t], 0, 0, 0);
    }
  }

  // ---- sum the 8 K-slices through LDS, write bf16
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) red[((wave * MT + t) * 16 + i) * 64 + lane] = acc[t][i];
  __syncthreads();
  for (int idx = tid; idx < MT * 16 * 64; idx += 512) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) v += red[w * MT * 16 * 64 + idx];
    const int l = idx & 63, i = (idx >> 6) & 15, t = idx >> 10;
    const int m = m0 + t * 32 + (i & 3) + 8 * (i >> 2) + 4 * (l >> 5);
    if (m < M) y[(long long)m * N + n0 + (l & 31)] = f2bf(v);
  }
}

}  // namespace

extern "C" int ftc_nf4_gemm(const void* x, const uint8_t* packed, const uint8_t* absmax_q, const float* absmax_scale,
                            float absmax_offset, void* y, int M, int N, int K, int block, int block2,
                            hipStream_t stream) {
  if (block != 64 || K % 64 != 0 || N % 32 != 0 || M <= 0) return -1;
  auto X = (const uint16_t*)x;
  auto Y = (uint16_t*)y;
  static bool attr = false;  // 64 KiB dynamic reduction buffer + the static codebook
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)nf4_gemm_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        WAVES * 2 * 16 * 64 * 4);
    attr = true;
  }
  if (M <= 32) {
    dim3 grid(N / 32, 1);
    hipLaunchKernelGGL(nf4_gemm_kernel<1>, grid, dim3(512), WAVES * 1 * 16 * 64 * 4, stream, X, packed, absmax_q,
                       absmax_scale, absmax_offset, Y, M, N, K, block2);
  } else {
    dim3 grid(N / 32, (M + 63) / 64);
    hipLaunchKernelGGL(nf4_gemm_kernel<2>, grid, dim3(512), WAVES * 2 * 16 * 64 * 4, stream, X, packed, absmax_q,
                       absmax_scale, absmax_offset, Y, M, N, K, block2);
  }
  return (int)hipGetLastError();
}
