// K3: RMSNorm forward / backward with the residual add fused in.
//
//   fwd:  h = x (+ res)            (bf16, written back when res is given: the residual stream)
//         rstd = rsqrt(mean(h^2) + eps)   (fp32, saved for backward)
//         y = bf16(h * rstd * w)
//   bwd:  xhat = h*rstd, g = dy*w
//         dx = rstd*(g - xhat*mean(g*xhat)) (+ dres: gradient arriving along the residual stream)
//         dw = sum_rows dy*xhat   (optional: frozen in LoRA runs)
//
// Layout: one wave64 per row, the row held in registers (NV x 16-byte vectors per lane) so the
// reduction is a pure wave shuffle -- no LDS, no barrier on the row path.  4 waves per 256-thread
// block, grid-stride over rows with the grid capped at 2048 blocks (8 per CU).  The dw partials
// are reduced across the 4 waves of a block in LDS and across blocks by a second tiny kernel
// (deterministic: no float atomics).
#include "common.h"

#include <cstdlib>

using namespace ftc;

template <int NV, bool RES>
__global__ __launch_bounds__(256) void rmsnorm_fwd_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ res, const uint16_t* __restrict__ w,
    uint16_t* __restrict__ h_out, uint16_t* __restrict__ y, float* __restrict__ rstd, int rows, int d,
    float eps, long long y_rs) {
  const int lane = threadIdx.x & 63;
  const int nvec = d >> 3;
  const float inv_d = 1.0f / (float)d;
  for (long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6); row < rows;
       row += (long long)gridDim.x * 4) {
    const uint4* xr = reinterpret_cast<const uint4*>(x + row * d);
    float v[NV][8];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int idx = lane + i * 64;
      if (idx < nvec) {
        uint4 a = xr[idx];
        unpack8(a, v[i]);
        if constexpr (RES) {
          float r8[8];
          unpack8(reinterpret_cast<const uint4*>(res + row * d)[idx], r8);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[i][j] += r8[j];
          uint4 hv = pack8(v[i]);
          reinterpret_cast<uint4*>(h_out + row * d)[idx] = hv;
          unpack8(hv, v[i]);  // statistics on the stored (rounded) residual stream
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
      }
    }
    ss = wave_sum(ss);
    const float r = rsqrtf(ss * inv_d + eps);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int idx = lane + i * 64;
      if (idx < nvec) {
        float w8[8], o[8];
        unpack8(reinterpret_cast<const uint4*>(w)[idx], w8);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = v[i][j] * r * w8[j];
        reinterpret_cast<uint4*>(y + row * y_rs)[idx] = pack8(o);
      }
    }
    if (lane == 0) rstd[row] = r;
  }
}

// Forward with TWO waves per row (each lane NV2 16-byte chunks): half the registers of the one-wave
// layout, so twice the rows in flight for this HBM-bound pass; the sum of squares meets in LDS.
template <int NV2, bool RES>
__global__ __launch_bounds__(256) void rmsnorm_fwd2_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ res, const uint16_t* __restrict__ w,
    uint16_t* __restrict__ h_out, uint16_t* __restrict__ y, float* __restrict__ rstd, int rows, int d,
    float eps, long long y_rs) {
  __shared__ float part[4];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int pair = wid >> 1, half = wid & 1;
  const int nvec = d >> 3;
  const float inv_d = 1.0f / (float)d;
  const int lane2 = half * 64 + lane;
  for (long long base = (long long)blockIdx.x * 2; base < rows; base += (long long)gridDim.x * 2) {
    const long long row = base + pair;
    const bool ok = row < rows;
    float v[NV2][8];
    float ss = 0.f;
    if (ok) {
      uint4 xv[NV2], rv[RES ? NV2 : 1];
#pragma unroll
      for (int i = 0; i < NV2; ++i) {
        const int idx = lane2 + i * 128;
        if (idx < nvec) {
          xv[i] = reinterpret_cast<const uint4*>(x + row * d)[idx];
          if constexpr (RES) rv[i] = reinterpret_cast<const uint4*>(res + row * d)[idx];
        }
      }
#pragma unroll
      for (int i = 0; i < NV2; ++i) {
        const int idx = lane2 + i * 128;
        if (idx < nvec) {
          unpack8(xv[i], v[i]);
          if constexpr (RES) {
            float r8[8];
            unpack8(rv[i], r8);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[i][j] += r8[j];
            const uint4 hv = pack8(v[i]);
            reinterpret_cast<uint4*>(h_out + row * d)[idx] = hv;
            unpack8(hv, v[i]);  // statistics on the stored (rounded) residual stream
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
        }
      }
    }
    ss = wave_sum(ss);
    if (lane == 0) part[wid] = ss;
    __syncthreads();
    const float r = rsqrtf((part[2 * pair] + part[2 * pair + 1]) * inv_d + eps);
    __syncthreads();
    if (ok) {
#pragma unroll
      for (int i = 0; i < NV2; ++i) {
        const int idx = lane2 + i * 128;
        if (idx < nvec) {
          float w8[8], o[8];
          unpack8(reinterpret_cast<const uint4*>(w)[idx], w8);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = v[i][j] * r * w8[j];
          reinterpret_cast<uint4*>(y + row * y_rs)[idx] = pack8(o);
        }
      }
      if (half == 0 && lane == 0) rstd[row] = r;
    }
  }
}

// One wave per row.  dy / h rows stay in registers as packed bf16 (4 VGPRs per 8 elements) and are
// re-expanded in the second pass, and w is loaded once per wave: ~100 VGPRs at d = 4096 instead of
// ~180 for fp32 copies, i.e. twice the waves in flight for this HBM-bound kernel.
// dres (gradient of the residual stream from the next layer) and dx may be row-padded views
// (row strides dres_rs / dx_rs): dx's spare columns take the next projection's LoRA term (ops/linear.py).
template <int NV, bool DW, bool DRES>
__global__ __launch_bounds__(256) void rmsnorm_bwd_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ h, const uint16_t* __restrict__ w,
    const float* __restrict__ rstd, const uint16_t* __restrict__ dres, uint16_t* __restrict__ dx,
    float* __restrict__ dw_part, int rows, int d, long long dres_rs, long long dx_rs) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nvec = d >> 3;
  const float inv_d = 1.0f / (float)d;
  float acc[DW ? NV : 1][8];
  if constexpr (DW) {
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
  }
  uint4 wv[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int idx = lane + i * 64;
    wv[i] = idx < nvec ? reinterpret_cast<const uint4*>(w)[idx] : make_uint4(0, 0, 0, 0);
  }
  for (long long row = (long long)blockIdx.x * 4 + wid; row < rows; row += (long long)gridDim.x * 4) {
    const float r = rstd[row];
    uint4 dyv[NV], hv[NV];
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int idx = lane + i * 64;
      if (idx < nvec) {
        dyv[i] = reinterpret_cast<const uint4*>(dy + row * d)[idx];
        hv[i] = reinterpret_cast<const uint4*>(h + row * d)[idx];
        float dy8[8], h8[8], w8[8];
        unpack8(dyv[i], dy8);
        unpack8(hv[i], h8);
        unpack8(wv[i], w8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = h8[j] * r;
          dot += dy8[j] * w8[j] * xh;
          if constexpr (DW) acc[i][j] += dy8[j] * xh;
        }
      }
    }
    dot = wave_sum(dot) * inv_d;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int idx = lane + i * 64;
      if (idx < nvec) {
        float dy8[8], h8[8], w8[8], o[8];
        unpack8(dyv[i], dy8);
        unpack8(hv[i], h8);
        unpack8(wv[i], w8);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = r * (dy8[j] * w8[j] - h8[j] * r * dot);
        if constexpr (DRES) {
          float d8[8];
          unpack8(reinterpret_cast<const uint4*>(dres + row * dres_rs)[idx], d8);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += d8[j];
        }
        reinterpret_cast<uint4*>(dx + row * dx_rs)[idx] = pack8(o);
      }
    }
  }
  if constexpr (DW) {
    // reduce the 4 waves' partial dw rows in LDS: lds[4][d]
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int idx = lane + i * 64;
      if (idx < nvec) {
#pragma unroll
        for (int j = 0; j < 8; ++j) lds[wid * d + idx * 8 + j] = acc[i][j];
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < d; c += 256) {
      float s = lds[c] + lds[d + c] + lds[2 * d + c] + lds[3 * d + c];
      dw_part[(long long)blockIdx.x * d + c] = s;
    }
  }
}

// Frozen-weight backward (no dw: LoRA / QLoRA norms), tuned for occupancy: TWO waves per row (each
// lane holds NV2 16-byte chunks, half of the one-wave layout), w staged once per workgroup in LDS, and
// dres loaded together with dy / h so each row needs a single memory round trip.  The row dot product
// meets in LDS (one barrier per pair of rows).  ~100 VGPRs instead of 178: 4+ waves per SIMD.
template <int NV2, bool DRES>
__global__ __launch_bounds__(256) void rmsnorm_bwd2_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ h, const uint16_t* __restrict__ w,
    const float* __restrict__ rstd, const uint16_t* __restrict__ dres, uint16_t* __restrict__ dx, int rows, int d,
    long long dres_rs, long long dx_rs) {
  extern __shared__ __attribute__((aligned(16))) uint4 wl[];  // w: d / 8 chunks, then 4 floats of partial dots
  float* part = reinterpret_cast<float*>(wl + (d >> 3));
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int pair = wid >> 1, half = wid & 1;  // rows: 2 per iteration, 2 waves per row
  const int nvec = d >> 3;
  const float inv_d = 1.0f / (float)d;
  for (int i = tid; i < nvec; i += 256) wl[i] = reinterpret_cast<const uint4*>(w)[i];
  __syncthreads();
  const int lane2 = half * 64 + lane;  // 0..127 within the row
  for (long long base = (long long)blockIdx.x * 2; base < rows; base += (long long)gridDim.x * 2) {
    const long long row = base + pair;
    const bool ok = row < rows;
    uint4 dyv[NV2], hv[NV2], drv[DRES ? NV2 : 1];
    float dot = 0.f, r = 0.f;
    if (ok) {
      r = rstd[row];
#pragma unroll
      for (int i = 0; i < NV2; ++i) {
        const int idx = lane2 + i * 128;
        if (idx < nvec) {
          dyv[i] = reinterpret_cast<const uint4*>(dy + row * d)[idx];
          hv[i] = reinterpret_cast<const uint4*>(h + row * d)[idx];
          if constexpr (DRES) drv[i] = reinterpret_cast<const uint4*>(dres + row * dres_rs)[idx];
        }
      }
#pragma unroll
      for (int i = 0; i < NV2; ++i) {
        const int idx = lane2 + i * 128;
        if (idx < nvec) {
          float dy8[8], h8[8], w8[8];
          unpack8(dyv[i], dy8);
          unpack8(hv[i], h8);
          unpack8(wl[idx], w8);
#pragma unroll
          for (int j = 0; j < 8; ++j) dot += dy8[j] * w8[j] * (h8[j] * r);
        }
      }
    }
    dot = wave_sum(dot);
    if (lane == 0) part[wid] = dot;
    __syncthreads();
    dot = (part[2 * pair] + part[2 * pair + 1]) * inv_d;
    __syncthreads();  // part is rewritten next iteration
    if (ok) {
#pragma unroll
      for (int i = 0; i < NV2; ++i) {
        const int idx = lane2 + i * 128;
        if (idx < nvec) {
          float dy8[8], h8[8], w8[8], o[8];
          unpack8(dyv[i], dy8);
          unpack8(hv[i], h8);
          unpack8(wl[idx], w8);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = r * (dy8[j] * w8[j] - h8[j] * r * dot);
          if constexpr (DRES) {
            float d8[8];
            unpack8(drv[i], d8);
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] += d8[j];
          }
          reinterpret_cast<uint4*>(dx + row * dx_rs)[idx] = pack8(o);
        }
      }
    }
  }
}

// dw[c] = sum_b part[b][c].  A workgroup owns 64 columns; its 4 waves take every 4th partial row with
// 8 independent accumulators each (enough loads in flight to hide HBM latency), then reduce through
// LDS.  Deterministic (fixed summation order), d/64 workgroups.
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ part, float* __restrict__ out,
                                                     int nrows, int d) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  if (c < d) {
    int b = wv;
    for (; b + 28 < nrows; b += 32) {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += part[(long long)(b + 4 * j) * d + c];
    }
    for (; b < nrows; b += 4) acc[0] += part[(long long)b * d + c];
  }
  red[wv][lane] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  if (wv == 0 && c < d) out[c] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// frozen-weight launches: one row group per workgroup (common.h oneshot_grid); bwd 0.097 vs 0.101 ms,
// fwd equal (profiles/r4/oneshot/rms.log).  The dw backward keeps its capped grid (partials per block).
static int rms_grid(long long rows, int per_block) { return ftc::oneshot_grid(rows, per_block); }

static int pick_nv(int d) {
  const int per_lane = (d / 8 + 63) / 64;
  int nv = 1;
  while (nv < per_lane) nv <<= 1;
  return nv;
}

// y is written with row stride y_rs (>= d): a padded buffer lets the next projection append its LoRA
// activations as extra GEMM columns (ops/linear.py "augmented" path)
extern "C" int ftc_rmsnorm_fwd(const void* x, const void* res, const void* w, void* h_out, void* y, float* rstd,
                               int rows, int d, float eps, long long y_rs, hipStream_t stream) {
  if (d % 8 != 0 || d > 16 * 512) return -1;
  const int nv = pick_nv(d);
  const int grid = rms_grid(rows, 4);
  auto X = (const uint16_t*)x;
  auto R = (const uint16_t*)res;
  auto W = (const uint16_t*)w;
  auto H = (uint16_t*)h_out;
  auto Y = (uint16_t*)y;
#define LAUNCH_FWD(NV)                                                                                    \
  if (res)                                                                                                    \
    hipLaunchKernelGGL((rmsnorm_fwd_kernel<NV, true>), dim3(grid), dim3(256), 0, stream, X, R, W, H, Y, rstd, \
                       rows, d, eps, y_rs);                                                                         \
  else                                                                                                        \
    hipLaunchKernelGGL((rmsnorm_fwd_kernel<NV, false>), dim3(grid), dim3(256), 0, stream, X, R, W, H, Y,     \
                       rstd, rows, d, eps, y_rs);
  // two waves per row wherever a row has >= 2 vectors per lane (the one-wave kernel: d <= 512)
  if (nv >= 2) {
    const int g2 = rms_grid(rows, 2);
#define LAUNCH_FWD2(NV2)                                                                                     \
  if (res)                                                                                                       \
    hipLaunchKernelGGL((rmsnorm_fwd2_kernel<NV2, true>), dim3(g2), dim3(256), 0, stream, X, R, W, H, Y, rstd, rows, \
                       d, eps, y_rs);                                                                            \
  else                                                                                                           \
    hipLaunchKernelGGL((rmsnorm_fwd2_kernel<NV2, false>), dim3(g2), dim3(256), 0, stream, X, R, W, H, Y, rstd,     \
                       rows, d, eps, y_rs);
    switch (nv) {
      case 2: LAUNCH_FWD2(1); break;
      case 4: LAUNCH_FWD2(2); break;
      case 8: LAUNCH_FWD2(4); break;
      case 16: LAUNCH_FWD2(8); break;
      default: return -1;
    }
#undef LAUNCH_FWD2
    return (int)hipGetLastError();
  }
  switch (nv) {
    case 1: LAUNCH_FWD(1); break;
    case 2: LAUNCH_FWD(2); break;
    case 4: LAUNCH_FWD(4); break;
    case 8: LAUNCH_FWD(8); break;
    case 16: LAUNCH_FWD(16); break;
    default: return -1;
  }
#undef LAUNCH_FWD
  return (int)hipGetLastError();
}

// dw_part must hold grid*d floats where grid = ftc_rmsnorm_bwd_grid(rows); dw (fp32, d) may be null.
extern "C" int ftc_rmsnorm_bwd_grid(int rows) { return ftc::stream_grid(rows, 4) > 512 ? 512 : ftc::stream_grid(rows, 4); }

extern "C" int ftc_rmsnorm_bwd(const void* dy, const void* h, const void* w, const float* rstd, const void* dres,
                               void* dx, float* dw_part, float* dw, int rows, int d, long long dres_rs,
                               long long dx_rs, hipStream_t stream) {
  if (d % 8 != 0 || d > 16 * 512) return -1;
  const int nv = pick_nv(d);
  const bool need_dw = dw != nullptr;
  // the dw path keeps per-wave accumulators: fewer, longer-lived blocks
  const int grid = need_dw ? ftc_rmsnorm_bwd_grid(rows) : rms_grid(rows, 4);
  const size_t lds = need_dw ? (size_t)4 * d * sizeof(float) : 0;
  auto DY = (const uint16_t*)dy;
  auto Hh = (const uint16_t*)h;
  auto W = (const uint16_t*)w;
  auto DR = (const uint16_t*)dres;
  auto DX = (uint16_t*)dx;
#define LAUNCH_BWD(NV, DWB, DRB)                                                                       \
  hipLaunchKernelGGL((rmsnorm_bwd_kernel<NV, DWB, DRB>), dim3(grid), dim3(256), lds, stream, DY, Hh, W, rstd, \
                     DR, DX, dw_part, rows, d, dres_rs, dx_rs)
#define LAUNCH_BWD_NV(NV)                     \
  if (need_dw) {                                  \
    if (dres) LAUNCH_BWD(NV, true, true);     \
    else LAUNCH_BWD(NV, true, false);         \
  } else {                                        \
    if (dres) LAUNCH_BWD(NV, false, true);    \
    else LAUNCH_BWD(NV, false, false);        \
  }
  // frozen norms: the two-waves-per-row kernel (the weight-gradient path keeps per-wave accumulators)
  if (!need_dw && nv >= 2) {
    const int g2 = rms_grid(rows, 2);
    const size_t l2 = (size_t)(d / 8) * 16 + 4 * sizeof(float);
#define LAUNCH_BWD2(NV2)                                                                                  \
  if (dres)                                                                                                   \
    hipLaunchKernelGGL((rmsnorm_bwd2_kernel<NV2, true>), dim3(g2), dim3(256), l2, stream, DY, Hh, W, rstd, DR, DX, \
                       rows, d, dres_rs, dx_rs);                                                              \
  else                                                                                                        \
    hipLaunchKernelGGL((rmsnorm_bwd2_kernel<NV2, false>), dim3(g2), dim3(256), l2, stream, DY, Hh, W, rstd, DR,  \
                       DX, rows, d, dres_rs, dx_rs);
    switch (nv) {
      case 2: LAUNCH_BWD2(1); break;
      case 4: LAUNCH_BWD2(2); break;
      case 8: LAUNCH_BWD2(4); break;
      case 16: LAUNCH_BWD2(8); break;
      default: return -1;
    }
#undef LAUNCH_BWD2
    return (int)hipGetLastError();
  }
  switch (nv) {
    case 1: LAUNCH_BWD_NV(1); break;
    case 2: LAUNCH_BWD_NV(2); break;
    case 4: LAUNCH_BWD_NV(4); break;
    case 8: LAUNCH_BWD_NV(8); break;
    case 16: LAUNCH_BWD_NV(16); break;
    default: return -1;
  }
#undef LAUNCH_BWD_NV
#undef LAUNCH_BWD
  if (need_dw) {
    hipLaunchKernelGGL(colsum_kernel, dim3((d + 63) / 64), dim3(256), 0, stream, dw_part, dw, grid, d);
  }
  return (int)hipGetLastError();
}
