// K8 (part 1): NF4 quantisation / dequantisation for QLoRA base weights.
//
// Format: 4-bit NormalFloat codes, blocks of `block` (=64) consecutive
// elements share an fp32 absmax; two codes per byte, FIRST element in the HIGH nibble (the
// bitsandbytes packing order).  Double quantisation stores the absmax vector itself as uint8:
//     absmax[i] = offset + (q2[i] - 128) / 127 * scale2[i / block2]        (block2 = 256)
// The nested step is done on the host-side tensor (finetune_controller_amd/ops/nf4.py) because it
// is a one-time O(n/64) operation; these kernels do the O(n) parts.
#include "common.h"

using namespace ftc;

__constant__ float kNF4[16] = {-1.0f,
                               -0.6961928009986877f,
                               -0.5250730514526367f,
                               -0.39491748809814453f,
                               -0.28444138169288635f,
                               -0.18477343022823334f,
                               -0.09105003625154495f,
                               0.0f,
                               0.07958029955625534f,
                               0.16093020141124725f,
                               0.24611230194568634f,
                               0.33791524171829224f,
                               0.44070982933044434f,
                               0.5626170039176941f,
                               0.7229568362236023f,
                               1.0f};

// The codebook indexed per lane from __constant__ memory compiles to one global load per element (16
// vector-memory loads per 8 bytes of codes: the dequant kernels ran at 2.5 TB/s).  Each workgroup
// copies it to LDS once; a lookup is then one conflict-free ds_read (16 entries, 16 banks).
DEV_INLINE void nf4_lut_load(float* lut) {
  if (threadIdx.x < 16) lut[threadIdx.x] = kNF4[threadIdx.x];
  __syncthreads();
}

DEV_INLINE int nf4_encode(float x) {
  // nearest codebook entry (midpoints between consecutive codes)
  int best = 0;
  float bd = fabsf(x - kNF4[0]);
#pragma unroll
  for (int i = 1; i < 16; ++i) {
    const float dd = fabsf(x - kNF4[i]);
    if (dd < bd) { bd = dd; best = i; }
  }
  return best;
}

// The rank-r parts of the augmented QLoRA operands (ops/nf4.py _QScratch), written by extra workgroups
// of the same dequant launch instead of 2-3 small copy / scale kernels per projection call:
//   out_b[n * ldob + r] = B[n * ldb + r]                     (n < N, r < R; B copy)
//   out_a[r * ldoa + k] = bf16(s * A[r * lda + k])           (forward: rows N.. of [W ; s A])
//   out_a[k * ldoa + r] = bf16(s * A[r * lda + k])           (a_t: the transposed backward operand)
// Same rounding as torch.mul on bf16 (fp32 product, round to nearest even).
struct AugTail {
  const uint16_t* B;
  long long ldb;
  uint16_t* out_b;
  long long ldob;
  const uint16_t* A;
  long long lda;
  uint16_t* out_a;
  long long ldoa;
  float s;
  int N, R, K, a_t;
};

DEV_INLINE void aug_tail_fill(const AugTail& t, long long i0, long long stride) {
  const long long nb = t.B ? (long long)t.N * t.R : 0;
  const long long na = t.A ? (long long)t.R * t.K : 0;
  for (long long i = i0; i < nb + na; i += stride) {
    if (i < nb) {
      const long long n = i / t.R;
      const int r = (int)(i - n * t.R);
      t.out_b[n * t.ldob + r] = t.B[n * t.ldb + r];
    } else {
      const long long j = i - nb;
      const int r = (int)(j / t.K), k = (int)(j - (long long)r * t.K);
      const uint16_t v = f2bf(t.s * bf2f(t.A[(long long)r * t.lda + k]));
      if (t.a_t)
        t.out_a[(long long)k * t.ldoa + r] = v;
      else
        t.out_a[(long long)r * t.ldoa + k] = v;
    }
  }
}

constexpr int kTailBlocks = 64;  // extra workgroups of a dequant launch that carry an AugTail

// one wave per block of 64 elements: lane j handles element j
__global__ __launch_bounds__(256) void nf4_quant_kernel(const uint16_t* __restrict__ w, uint8_t* __restrict__ packed,
                                                        float* __restrict__ absmax, long long nblocks, int block) {
  const int lane = threadIdx.x & 63;
  for (long long b = (long long)blockIdx.x * 4 + (threadIdx.x >> 6); b < nblocks; b += (long long)gridDim.x * 4) {
    float mx = 0.f;
    for (int i = lane; i < block; i += 64) mx = fmaxf(mx, fabsf(bf2f(w[b * block + i])));
    mx = wave_max(mx);
    const float inv = mx > 0.f ? 1.0f / mx : 0.f;
    for (int i = lane * 2; i < block; i += 128) {
      const int q0 = nf4_encode(bf2f(w[b * block + i]) * inv);
      const int q1 = nf4_encode(bf2f(w[b * block + i + 1]) * inv);
      packed[(b * block + i) >> 1] = (uint8_t)((q0 << 4) | q1);
    }
    if (lane == 0) absmax[b] = mx;
  }
}

__global__ __launch_bounds__(256) void nf4_dequant_kernel(const uint8_t* __restrict__ packed,
                                                          const uint8_t* __restrict__ aq,
                                                          const float* __restrict__ s2, float off,
                                                          uint16_t* __restrict__ out, long long n, int block,
                                                          int block2) {
  // each thread: 16 codes (8 bytes) -> 16 bf16 (32 bytes)
  __shared__ float lut[16];
  nf4_lut_load(lut);
  const long long n16 = n >> 4;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n16; i += (long long)gridDim.x * 256) {
    const uint2 p = reinterpret_cast<const uint2*>(packed)[i];
    const long long e0 = i << 4;
    const long long bi = e0 / block;  // block >= 16 and a multiple of 16: one absmax per thread
    const float a = off + ((float)aq[bi] - 128.0f) * (1.0f / 127.0f) * s2[bi / block2];
    float f[16];
    uint32_t words[2] = {p.x, p.y};
#pragma unroll
    for (int wd = 0; wd < 2; ++wd) {
#pragma unroll
      for (int bt = 0; bt < 4; ++bt) {
        const uint32_t byte = (words[wd] >> (8 * bt)) & 0xffu;
        f[wd * 8 + bt * 2] = lut[byte >> 4] * a;
        f[wd * 8 + bt * 2 + 1] = lut[byte & 0xf] * a;
      }
    }
    uint4* o = reinterpret_cast<uint4*>(out + e0);
    o[0] = pack8(f);
    o[1] = pack8(f + 8);
  }
}

DEV_INLINE float nf4_absmax(const uint8_t* aq, const float* s2, float off, long long bi, int block2) {
  return off + ((float)aq[bi] - 128.0f) * (1.0f / 127.0f) * s2[bi / block2];
}

// dequantise into a row view: out[n * ldo + k] (a column block of an augmented GEMM operand).  (Measured
// and kept over a lane-contiguous rewrite -- 4-byte code words, 16-byte stores, four chunks per thread in
// flight: 14.3 / 74.7 vs 13.6 / 71.1 us at the qkv / gate_up shapes, profiles/r5/followup/.)
__global__ __launch_bounds__(256) void nf4_dequant_rows_kernel(const uint8_t* __restrict__ packed,
                                                               const uint8_t* __restrict__ aq,
                                                               const float* __restrict__ s2, float off,
                                                               uint16_t* __restrict__ out, long long n, int cols,
                                                               long long ldo, int block, int block2, int main_blocks,
                                                               AugTail tail) {
  if ((int)blockIdx.x >= main_blocks) {  // block-uniform: the rank-r operand parts
    aug_tail_fill(tail, (long long)(blockIdx.x - main_blocks) * 256 + threadIdx.x,
                  (long long)(gridDim.x - main_blocks) * 256);
    return;
  }
  __shared__ float lut[16];
  nf4_lut_load(lut);
  const long long n16 = n >> 4;
  const int c16 = cols >> 4;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n16; i += (long long)main_blocks * 256) {
    const uint2 p = reinterpret_cast<const uint2*>(packed)[i];
    const long long e0 = i << 4;
    const long long bi = e0 / block;
    const float a = off + ((float)aq[bi] - 128.0f) * (1.0f / 127.0f) * s2[bi / block2];
    float f[16];
    const uint32_t words[2] = {p.x, p.y};
#pragma unroll
    for (int wd = 0; wd < 2; ++wd)
#pragma unroll
      for (int bt = 0; bt < 4; ++bt) {
        const uint32_t byte = (words[wd] >> (8 * bt)) & 0xffu;
        f[wd * 8 + bt * 2] = lut[byte >> 4] * a;
        f[wd * 8 + bt * 2 + 1] = lut[byte & 0xf] * a;
      }
    const long long row = i / c16;
    const int c = (int)(i - row * c16) * 16;
    uint4* o = reinterpret_cast<uint4*>(out + row * ldo + c);
    o[0] = pack8(f);
    o[1] = pack8(f + 8);
  }
}

// dequantise TRANSPOSED: outT[k * ldo + n] = W[n][k] -- the K-contiguous right operand of the backward
// GEMM dx = dy . W (TN layout).  A 64 (n) x 128 (k) tile per workgroup through LDS as [k][n]:
//   decode: thread (n pair 2m, 2m + 1; 16 k) loads the two rows' 8-byte code runs, and writes each k's
//           (W[2m][k], W[2m+1][k]) pair as ONE 32-bit LDS word (16 ds_write_b32, not 32 ds_write_b16);
//   store:  each output row segment (64 n = 128 bytes) is 8 lanes x 16 bytes of one store instruction, a wave
//           instruction covers 8 whole rows (ds_read_b128 from a 16-byte-aligned padded LDS row).
// (Round 4: 64 x 64 tiles, 16-bit LDS writes and reads, 3.6 TB/s.)
constexpr int kTN = 64, kTK = 128, kTPad = 8;  // LDS row = kTN + kTPad bf16 = 144 bytes
__global__ __launch_bounds__(256) void nf4_dequant_t_kernel(const uint8_t* __restrict__ packed,
                                                            const uint8_t* __restrict__ aq,
                                                            const float* __restrict__ s2, float off,
                                                            uint16_t* __restrict__ outT, int N, int K, long long ldo,
                                                            int block2, AugTail tail) {
  if ((int)blockIdx.y == (K + kTK - 1) / kTK) {  // the extra row of workgroups: the rank-r operand parts
    aug_tail_fill(tail, (long long)blockIdx.x * 256 + threadIdx.x, (long long)gridDim.x * 256);
    return;
  }
  __shared__ __attribute__((aligned(16))) uint16_t tile[kTK][kTN + kTPad];
  __shared__ float lut[16];
  nf4_lut_load(lut);
  const int n0 = blockIdx.x * kTN, k0 = blockIdx.y * kTK;
  const int kvalid = min(kTK, K - k0);  // K % 128 == 64: a half tile at the end
  const int t = threadIdx.x;
  if ((t >> 5) * 16 < kvalid) {
    const int m = t & 31, seg = t >> 5;  // rows n0 + 2m, 2m + 1; k in [16 seg, 16 seg + 16)
    const int kq = seg * 16;
    const long long e0 = (long long)(n0 + 2 * m) * K + k0 + kq;  // first element of row 2m's run
    const long long e1 = e0 + K;
    const uint2 p0 = *reinterpret_cast<const uint2*>(packed + (e0 >> 1));
    const uint2 p1 = *reinterpret_cast<const uint2*>(packed + (e1 >> 1));
    const float a0 = nf4_absmax(aq, s2, off, e0 >> 6, block2), a1 = nf4_absmax(aq, s2, off, e1 >> 6, block2);
    const uint32_t w0[2] = {p0.x, p0.y}, w1[2] = {p1.x, p1.y};
#pragma unroll
    for (int wd = 0; wd < 2; ++wd)
#pragma unroll
      for (int bt = 0; bt < 4; ++bt) {
        const uint32_t b0 = (w0[wd] >> (8 * bt)) & 0xffu, b1 = (w1[wd] >> (8 * bt)) & 0xffu;
        const int kk = kq + wd * 8 + bt * 2;
        *reinterpret_cast<uint32_t*>(&tile[kk][2 * m]) = pack_bf2(lut[b0 >> 4] * a0, lut[b1 >> 4] * a1);
        *reinterpret_cast<uint32_t*>(&tile[kk + 1][2 * m]) = pack_bf2(lut[b0 & 0xf] * a0, lut[b1 & 0xf] * a1);
      }
  }
  __syncthreads();
  {
    const int lane = t & 63, wave = t >> 6, ch = lane & 7;
#pragma unroll
    for (int j = 0; j < kTK / 32; ++j) {
      const int kr = wave * (kTK / 4) + j * 8 + (lane >> 3);
      if (kr >= kvalid) break;
      const uint4 v = *reinterpret_cast<const uint4*>(&tile[kr][ch * 8]);
      *reinterpret_cast<uint4*>(outT + (long long)(k0 + kr) * ldo + n0 + ch * 8) = v;
    }
  }
}

extern "C" int ftc_nf4_dequant_aug(const uint8_t* packed, const uint8_t* absmax_q, const float* absmax_scale,
                                   float absmax_offset, void* out, int rows, int cols, long long ldo, int block,
                                   int block2, int transpose, const void* B, long long ldb, void* out_b,
                                   long long ldob, const void* A, long long lda, void* out_a, long long ldoa, float s,
                                   int R, hipStream_t stream);

extern "C" int ftc_nf4_dequant_into(const uint8_t* packed, const uint8_t* absmax_q, const float* absmax_scale,
                                    float absmax_offset, void* out, int rows, int cols, long long ldo, int block,
                                    int block2, int transpose, hipStream_t stream) {
  return ftc_nf4_dequant_aug(packed, absmax_q, absmax_scale, absmax_offset, out, rows, cols, ldo, block, block2,
                             transpose, nullptr, 0, nullptr, 0, nullptr, 0, nullptr, 0, 0.f, 0, stream);
}

// As ftc_nf4_dequant_into, plus the AugTail writes (B -> out_b, s A -> out_a, transposed when a_t) in the
// same launch; B / A may be null (that part is skipped).  R = rank rows of A / columns of B.
extern "C" int ftc_nf4_dequant_aug(const uint8_t* packed, const uint8_t* absmax_q, const float* absmax_scale,
                                   float absmax_offset, void* out, int rows, int cols, long long ldo, int block,
                                   int block2, int transpose, const void* B, long long ldb, void* out_b,
                                   long long ldob, const void* A, long long lda, void* out_a, long long ldoa, float s,
                                   int R, hipStream_t stream) {
  if (cols % 64 != 0 || block != 64 || ldo % 8 != 0) return -1;
  AugTail t{(const uint16_t*)B, ldb, (uint16_t*)out_b, ldob, (const uint16_t*)A, lda, (uint16_t*)out_a, ldoa, s,
            rows, R, cols, transpose};
  const bool has_tail = R > 0 && (B || A);
  if (!has_tail) t.B = t.A = nullptr;
  if (transpose) {
    if (rows % kTN != 0) return -1;
    const int ky = (cols + kTK - 1) / kTK;
    hipLaunchKernelGGL(nf4_dequant_t_kernel, dim3(rows / kTN, ky + (has_tail ? 1 : 0)), dim3(256), 0, stream,
                       packed, absmax_q, absmax_scale, absmax_offset, (uint16_t*)out, rows, cols, ldo, block2, t);
  } else {
    const long long n = (long long)rows * cols;
    const int grid = ftc::oneshot_grid(n / 16, 256);
    hipLaunchKernelGGL(nf4_dequant_rows_kernel, dim3(grid + (has_tail ? kTailBlocks : 0)), dim3(256), 0, stream,
                       packed, absmax_q, absmax_scale, absmax_offset, (uint16_t*)out, n, cols, ldo, block, block2, grid,
                       t);
  }
  return (int)hipGetLastError();
}

extern "C" int ftc_nf4_quant(const void* w, uint8_t* packed, float* absmax, long long n, int block,
                             hipStream_t stream) {
  if (block % 2 != 0 || n % block != 0) return -1;
  const long long nb = n / block;
  const int grid = ftc::stream_grid(nb, 4);
  hipLaunchKernelGGL(nf4_quant_kernel, dim3(grid), dim3(256), 0, stream, (const uint16_t*)w, packed, absmax, nb, block);
  return (int)hipGetLastError();
}

extern "C" int ftc_nf4_dequant(const uint8_t* packed, const uint8_t* absmax_q, const float* absmax_scale,
                               float absmax_offset, void* out, long long n, int block, int block2,
                               hipStream_t stream) {
  if (n % 16 != 0 || block % 16 != 0) return -1;
  const int grid = ftc::oneshot_grid(n / 16, 256);
  hipLaunchKernelGGL(nf4_dequant_kernel, dim3(grid), dim3(256), 0, stream, packed, absmax_q, absmax_scale,
                     absmax_offset, (uint16_t*)out, n, block, block2);
  return (int)hipGetLastError();
}
