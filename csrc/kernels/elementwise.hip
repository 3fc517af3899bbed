// K4 RoPE (in place, forward and inverse rotation) and K9 SwiGLU forward/backward.
// Memory-bound: 16-byte vector loads per lane, cos/sin from host-precomputed fp32 tables
// (no on-device trig: guide Appendix B "Element-wise"); grid-stride loops launched one-shot
// (common.h oneshot_grid: one work item per thread).
#include "common.h"

#include <algorithm>

using namespace ftc;

// qkv: [rows, ld] bf16; the first (n_rot_heads * head_dim) columns are rotated in place, half-split
// (rotate_half) convention: (x1, x2) -> (x1 c - x2 s, x2 c + x1 s) with x1 = x[:D/2], x2 = x[D/2:].
// pos = positions ? positions[row] : row % seq_len, clamped to the table (positions are device data:
// no host read of them, so a step with explicit positions stays sync-free and graph-capturable).
// cos/sin tables: [max_pos, D/2] fp32.
__global__ __launch_bounds__(256) void rope_kernel(uint16_t* __restrict__ qkv, const float* __restrict__ cosT,
                                                   const float* __restrict__ sinT,
                                                   const int* __restrict__ positions, long long rows, int ld,
                                                   int n_rot_heads, int head_dim, int seq_len, float sign,
                                                   int max_pos) {
  const int half = head_dim >> 1;
  const int chunks = half >> 3;  // 8 pairs per work item
  const long long per_row = (long long)n_rot_heads * chunks;
  const long long total = rows * per_row;
  for (long long it = (long long)blockIdx.x * 256 + threadIdx.x; it < total; it += (long long)gridDim.x * 256) {
    const long long row = it / per_row;
    const int rem = (int)(it - row * per_row);
    const int head = rem / chunks;
    const int c = rem - head * chunks;
    const int pos = positions ? min(max(positions[row], 0), max_pos - 1) : (int)(row % seq_len);
    uint16_t* base = qkv + row * ld + (long long)head * head_dim + c * 8;
    uint4* p1 = reinterpret_cast<uint4*>(base);
    uint4* p2 = reinterpret_cast<uint4*>(base + half);
    float x1[8], x2[8], cs[8], sn[8];
    unpack8(*p1, x1);
    unpack8(*p2, x2);
    const float4* cr = reinterpret_cast<const float4*>(cosT + (long long)pos * half + c * 8);
    const float4* sr = reinterpret_cast<const float4*>(sinT + (long long)pos * half + c * 8);
    float4 c0 = cr[0], c1 = cr[1], s0 = sr[0], s1 = sr[1];
    cs[0] = c0.x; cs[1] = c0.y; cs[2] = c0.z; cs[3] = c0.w; cs[4] = c1.x; cs[5] = c1.y; cs[6] = c1.z; cs[7] = c1.w;
    sn[0] = s0.x; sn[1] = s0.y; sn[2] = s0.z; sn[3] = s0.w; sn[4] = s1.x; sn[5] = s1.y; sn[6] = s1.z; sn[7] = s1.w;
    float o1[8], o2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float s = sign * sn[j];
      o1[j] = x1[j] * cs[j] - x2[j] * s;
      o2[j] = x2[j] * cs[j] + x1[j] * s;
    }
    *p1 = pack8(o1);
    *p2 = pack8(o2);
  }
}

extern "C" int ftc_rope(void* qkv, const float* cosT, const float* sinT, const int* positions, long long rows,
                        int ld, int n_rot_heads, int head_dim, int seq_len, int inverse, int max_pos,
                        hipStream_t stream) {
  if (head_dim % 16 != 0 || ld % 8 != 0) return -1;
  const long long total = rows * n_rot_heads * (head_dim / 16);
  const int grid = ftc::oneshot_grid(total, 256);
  hipLaunchKernelGGL(rope_kernel, dim3(grid), dim3(256), 0, stream, (uint16_t*)qkv, cosT, sinT, positions, rows, ld,
                     n_rot_heads, head_dim, seq_len, inverse ? -1.0f : 1.0f, max_pos);
  return (int)hipGetLastError();
}

DEV_INLINE float silu_f(float g) { return g / (1.0f + __expf(-g)); }

// gu: [rows, 2F] (gate | up), a: [rows, F]
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const uint16_t* __restrict__ gu, uint16_t* __restrict__ a,
                                                         long long rows, int F, long long a_rs) {
  const int fv = F >> 3;
  const long long total = rows * fv;
  for (long long it = (long long)blockIdx.x * 256 + threadIdx.x; it < total; it += (long long)gridDim.x * 256) {
    const long long row = it / fv;
    const int c = (int)(it - row * fv);
    const uint4* r = reinterpret_cast<const uint4*>(gu + row * 2 * F);
    float g[8], u[8], o[8];
    unpack8(r[c], g);
    unpack8(r[fv + c], u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = silu_f(g[j]) * u[j];
    reinterpret_cast<uint4*>(a + row * a_rs)[c] = pack8(o);
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const uint16_t* __restrict__ da,
                                                         const uint16_t* __restrict__ gu, uint16_t* __restrict__ dgu,
                                                         long long rows, int F, long long dgu_rs) {
  const int fv = F >> 3;
  const long long total = rows * fv;
  for (long long it = (long long)blockIdx.x * 256 + threadIdx.x; it < total; it += (long long)gridDim.x * 256) {
    const long long row = it / fv;
    const int c = (int)(it - row * fv);
    const uint4* r = reinterpret_cast<const uint4*>(gu + row * 2 * F);
    float g[8], u[8], d[8], dg[8], du[8];
    unpack8(r[c], g);
    unpack8(r[fv + c], u);
    unpack8(reinterpret_cast<const uint4*>(da + row * F)[c], d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float sg = 1.0f / (1.0f + __expf(-g[j]));
      const float sl = g[j] * sg;
      du[j] = d[j] * sl;
      dg[j] = d[j] * u[j] * sg * (1.0f + g[j] * (1.0f - sg));
    }
    uint4* o = reinterpret_cast<uint4*>(dgu + row * dgu_rs);
    o[c] = pack8(dg);
    o[fv + c] = pack8(du);
  }
}

// a / dgu may be padded row views (row strides a_rs >= F, dgu_rs >= 2F; multiples of 8)
extern "C" int ftc_swiglu_fwd(const void* gu, void* a, long long rows, int F, long long a_rs, hipStream_t stream) {
  if (F % 8 != 0 || a_rs % 8 != 0) return -1;
  const int grid = ftc::oneshot_grid(rows * (F / 8), 256);
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(grid), dim3(256), 0, stream, (const uint16_t*)gu, (uint16_t*)a, rows, F,
                     a_rs);
  return (int)hipGetLastError();
}

extern "C" int ftc_swiglu_bwd(const void* da, const void* gu, void* dgu, long long rows, int F, long long dgu_rs,
                              hipStream_t stream) {
  if (F % 8 != 0 || dgu_rs % 8 != 0) return -1;
  const int grid = ftc::oneshot_grid(rows * (F / 8), 256);
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(grid), dim3(256), 0, stream, (const uint16_t*)da, (const uint16_t*)gu,
                     (uint16_t*)dgu, rows, F, dgu_rs);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- batched strided 2-D copy / scale
// dst[r, c] = bf16(scale * src[r, c]) for a table of small strided jobs in ONE launch: the LoRA operand
// refresh after each optimizer step (A, B, s A^T, B^T into the augmented GEMM buffers of every layer)
// was ~400 separate ~5 us copy / mul launches per Llama-3-8B step.  blockIdx.y = job; the job record
// is read by scalar loads; columns are the fast index (the host orients every job so the destination
// row is contiguous, dcs == 1).  Rounding = torch's bf16 mul (fp32 product, round-to-nearest-even).
struct Copy2DJob {
  long long src, dst;            // byte addresses of element (0, 0)
  long long srs, scs, drs, dcs;  // element strides
  int rows, cols;
  float scale;
  int pad;
};
static_assert(sizeof(Copy2DJob) == 64, "job record layout (mirrored in ops/linear.py)");

__global__ __launch_bounds__(256) void copy2d_batched_kernel(const Copy2DJob* __restrict__ jobs) {
  const Copy2DJob j = jobs[blockIdx.y];
  const uint16_t* src = reinterpret_cast<const uint16_t*>(j.src);
  uint16_t* dst = reinterpret_cast<uint16_t*>(j.dst);
  const long long n = (long long)j.rows * j.cols;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    const int r = (int)(e / j.cols), c = (int)(e - (long long)r * j.cols);
    const float v = bf2f(src[r * j.srs + c * j.scs]);
    dst[r * j.drs + c * j.dcs] = j.scale == 1.0f ? src[r * j.srs + c * j.scs] : f2bf(v * j.scale);
  }
}

extern "C" int ftc_copy2d_batched(const void* jobs, int njobs, long long max_elems, hipStream_t stream) {
  if (njobs <= 0) return 0;
  if (njobs > 65535) return -1;
  const int gx = (int)std::min<long long>(256, std::max<long long>(1, (max_elems + 2047) / 2048));
  hipLaunchKernelGGL(copy2d_batched_kernel, dim3(gx, njobs), dim3(256), 0, stream, (const Copy2DJob*)jobs);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- split-K partial sum
// C[r, c] = beta C + sum_s P[s][r, c]: the fp32 partials of a weight-gradient GEMM split along the token
// dimension (ops/linear.py `_dw_split`) folded into the (bf16 or fp32) gradient in one pass -- 8 columns
// per work item, 16-byte (bf16 C) / 2 x 16-byte (fp32 C) accesses, the partials read once.
template <bool F32C>
__global__ __launch_bounds__(256) void splitk_sum_kernel(const float* __restrict__ parts, int nsplit,
                                                         long long pstride, void* __restrict__ c, long long rows,
                                                         int cols, long long ldc, float beta) {
  const int cv = cols >> 3;
  const long long total = rows * cv;
  for (long long it = (long long)blockIdx.x * 256 + threadIdx.x; it < total; it += (long long)gridDim.x * 256) {
    const long long row = it / cv;
    const int col = (int)(it - row * cv) * 8;
    float acc[8];
    {
      const float4* p = reinterpret_cast<const float4*>(parts + row * cols + col);
      const float4 a0 = p[0], a1 = p[1];
      acc[0] = a0.x; acc[1] = a0.y; acc[2] = a0.z; acc[3] = a0.w;
      acc[4] = a1.x; acc[5] = a1.y; acc[6] = a1.z; acc[7] = a1.w;
    }
    for (int s = 1; s < nsplit; ++s) {
      const float4* p = reinterpret_cast<const float4*>(parts + s * pstride + row * cols + col);
      const float4 a0 = p[0], a1 = p[1];
      acc[0] += a0.x; acc[1] += a0.y; acc[2] += a0.z; acc[3] += a0.w;
      acc[4] += a1.x; acc[5] += a1.y; acc[6] += a1.z; acc[7] += a1.w;
    }
    if constexpr (F32C) {
      float4* q = reinterpret_cast<float4*>(reinterpret_cast<float*>(c) + row * ldc + col);
      if (beta != 0.f) {
        const float4 o0 = q[0], o1 = q[1];
        acc[0] += beta * o0.x; acc[1] += beta * o0.y; acc[2] += beta * o0.z; acc[3] += beta * o0.w;
        acc[4] += beta * o1.x; acc[5] += beta * o1.y; acc[6] += beta * o1.z; acc[7] += beta * o1.w;
      }
      q[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
      q[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
    } else {
      uint4* q = reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(c) + row * ldc + col);
      if (beta != 0.f) {
        float o[8];
        unpack8(*q, o);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += beta * o[j];
      }
      *q = pack8(acc);
    }
  }
}

extern "C" int ftc_splitk_sum(const float* parts, int nsplit, long long pstride, void* c, int c_fp32, long long rows,
                              int cols, long long ldc, float beta, hipStream_t stream) {
  if (nsplit < 1 || cols % 8 != 0 || ldc % 8 != 0 || (reinterpret_cast<uintptr_t>(parts) & 15) ||
      (reinterpret_cast<uintptr_t>(c) & 15) || pstride % 8 != 0)
    return -1;
  const int grid = ftc::oneshot_grid(rows * (cols / 8), 256);
  if (c_fp32)
    hipLaunchKernelGGL(splitk_sum_kernel<true>, dim3(grid), dim3(256), 0, stream, parts, nsplit, pstride, c, rows, cols,
                       ldc, beta);
  else
    hipLaunchKernelGGL(splitk_sum_kernel<false>, dim3(grid), dim3(256), 0, stream, parts, nsplit, pstride, c, rows,
                       cols, ldc, beta);
  return (int)hipGetLastError();
}
