// K5b: LoRA weight gradients as one streaming MFMA pass over the long operand.
//
//   dB [N, r]  += alpha * dy^T (s x A^T)      X = dy [T, N], Y = s x A^T [T, r]
//   dA [r, K]  += alpha * (dy B)^T x          X = x  [T, K], Y = dy B    [T, r]   (written transposed)
//
// i.e. out[m][r] = beta * out[m][r] + alpha * sum_t X[t][m] Y[t][r] with T = tokens (16k) and r <= 64.
// These GEMMs are pure HBM streams of X (r is tiny); hipBLASLt picks 16/64-wide tiles with no split
// of the 16k-deep reduction and runs the 4096-wide ones at ~1.5 TB/s.  Here every workgroup owns 128
// columns of X for one slice of the rows (split-T sized so the grid has ~1k workgroups), streams
// 64-row tiles through a double-buffered LDS image and reduces them with v_mfma_f32_32x32x16_bf16:
// both operands have the reduction dim (t) as their row index, so both are read with
// ds_read_b64_tr_b16 from the XOR-swizzled row-major images (same permuted k order on A and B).
// Each split writes an fp32 partial [M, r]; a second launch sums the splits and applies
// beta/alpha into the bf16 gradient (deterministic order, no atomics).
#include "common.h"

using namespace ftc;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int MB = 128;  // X columns per workgroup (32 per wave)
constexpr int TT = 64;   // rows per LDS tile
constexpr int RW = 64;   // Y image width (r padded to 64, zero-filled past r)

DEV_INLINE int swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
template <int W>
DEV_INLINE int img_off(int row, int chunk) {  // byte offset of 16-byte chunk `chunk` of image row `row`
  constexpr int NCH = W / 8;
  return row * (W * 2) + 16 * ((chunk ^ swz(row)) & (NCH - 1));
}
// Lane's two tr_b16 byte offsets for the 32-wide operand block starting at column colbase (k base 0):
// lane l gets column colbase + (l & 31), rows {4h..4h+3} then {4h+8..4h+11} (h = l >> 5).  The
// swizzle depends on row & 15 only, so a k base that is a multiple of 16 is a plain row offset.
template <int W>
DEV_INLINE int2 tr_offsets(int colbase, int lane) {
  const int hh = lane >> 5, gi = (lane >> 4) & 3, li = lane & 15;
  const int col = colbase + 16 * (gi & 1) + 4 * (li & 3);
  const int chunk = col >> 3, half8 = (col & 7) ? 8 : 0;
  const int r1 = 4 * hh + (li >> 2);
  return make_int2(img_off<W>(r1, chunk) + half8, img_off<W>(r1 + 8, chunk) + half8);
}
template <int W>
DEV_INLINE bf16x8 tr_read(const char* img, int kb, int2 off) {
  s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + off.x + kb * W * 2));
  s16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + off.y + kb * W * 2));
  s16x8 va = {v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
  return __builtin_bit_cast(bf16x8, va);
}

// Column segments of X (block-diagonal B of a packed projection: q|k|v or gate|up rows of dB): rows
// [m_end[i-1], m_end[i]) of the output use Y columns [ycol[i], ycol[i]+R) and output columns
// [ocol[i], ocol[i]+R).  One segment (m_end = M, ycol = ocol = 0) is the plain product.
struct Segs {
  int n;
  int m_end[4];
  int ycol[4];
  int ocol[4];
};
DEV_INLINE int seg_of(const Segs& sg, int m) {
  int i = 0;
#pragma unroll
  for (int k = 0; k < 3; ++k) i += (k + 1 < sg.n && m >= sg.m_end[k]) ? 1 : 0;
  return i;
}

// grid = ncb * splits; block b: column block b % ncb, row slice b / ncb (rows_per_split rows)
template <int NRB>
__global__ __launch_bounds__(256) void lora_wgrad_kernel(const uint16_t* __restrict__ X, long long ldx,
                                                         const uint16_t* __restrict__ Y, long long ldy,
                                                         float* __restrict__ ws, int M, int R, int rows_per_split,
                                                         int ncb, Segs sg) {
  __shared__ __attribute__((aligned(16))) char Xs0[TT * MB * 2];
  __shared__ __attribute__((aligned(16))) char Xs1[TT * MB * 2];
  __shared__ __attribute__((aligned(16))) char Ys0[TT * RW * 2];
  __shared__ __attribute__((aligned(16))) char Ys1[TT * RW * 2];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cb = blockIdx.x % ncb, sp = blockIdx.x / ncb;
  const int m0 = cb * MB;
  const long long t0 = (long long)sp * rows_per_split;
  const int ntiles = rows_per_split / TT;

  // global -> register staging: X tile = 64 rows x 16 chunks (4 per thread), Y tile = 64 rows x 8
  // chunks (2 per thread; chunks at or past r are zero)
  const int xc = tid & 15, xr0 = tid >> 4;
  const int yc = tid & 7, yr0 = tid >> 3;
  const bool yon = 8 * yc < R;
  const uint16_t* xp = X + (t0 + xr0) * ldx + m0 + 8 * xc;
  const uint16_t* yp = Y + (t0 + yr0) * ldy + sg.ycol[seg_of(sg, m0)] + 8 * yc;
  u32x4 xs[4], ys[2];
  auto gload = [&](int tile) {
    const long long tr = (long long)tile * TT;
#pragma unroll
    for (int i = 0; i < 4; ++i) xs[i] = *reinterpret_cast<const u32x4*>(xp + (tr + 16 * i) * ldx);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      ys[i] = yon ? *reinterpret_cast<const u32x4*>(yp + (tr + 32 * i) * ldy) : u32x4{0u, 0u, 0u, 0u};
  };
  auto lstore = [&](char* xs_img, char* ys_img) {
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<u32x4*>(xs_img + img_off<MB>(xr0 + 16 * i, xc)) = xs[i];
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<u32x4*>(ys_img + img_off<RW>(yr0 + 32 * i, yc)) = ys[i];
  };

  f32x16 acc[NRB];
#pragma unroll
  for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[rb][i] = 0.f;

  const int2 xo = tr_offsets<MB>(wave * 32, lane);
  int2 yo[NRB];
#pragma unroll
  for (int rb = 0; rb < NRB; ++rb) yo[rb] = tr_offsets<RW>(rb * 32, lane);

  auto compute = [&](const char* xs_img, const char* ys_img) {
#pragma unroll
    for (int ks = 0; ks < TT / 16; ++ks) {
      const bf16x8 a = tr_read<MB>(xs_img, 16 * ks, xo);
#pragma unroll
      for (int rb = 0; rb < NRB; ++rb) {
        const bf16x8 b = tr_read<RW>(ys_img, 16 * ks, yo[rb]);
        acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[rb], 0, 0, 0);
      }
    }
  };

  gload(0);
  lstore(Xs0, Ys0);
  __syncthreads();
  for (int it = 0; it < ntiles; it += 2) {
    if (it + 1 < ntiles) gload(it + 1);
    compute(Xs0, Ys0);
    if (it + 1 < ntiles) lstore(Xs1, Ys1);
    __syncthreads();
    if (it + 1 >= ntiles) break;
    if (it + 2 < ntiles) gload(it + 2);
    compute(Xs1, Ys1);
    if (it + 2 < ntiles) lstore(Xs0, Ys0);
    __syncthreads();
  }

  // partial [M, R] of this split: lane owns column r = rb*32 + (lane & 31) and 16 rows m
  float* w = ws + (long long)sp * M * R;
#pragma unroll
  for (int rb = 0; rb < NRB; ++rb) {
    const int r = rb * 32 + (lane & 31);
    if (r < R) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int m = m0 + wave * 32 + 8 * (i >> 2) + 4 * (lane >> 5) + (i & 3);
        w[(long long)m * R + r] = acc[rb][i];
      }
    }
  }
}

// out[m * out_sm + (ocol(m) + r) * out_sr] = beta * out + alpha * sum_s ws[s][m][r]; each thread owns 4
// consecutive (m, r) entries (R % 8 == 0, so they share m).  SPLITS is a compile-time power of two: all
// of a thread's split loads are issued before the first add (one memory round trip, not SPLITS / 8).
template <int SPLITS>
__global__ __launch_bounds__(256) void lora_wgrad_reduce_kernel(const float* __restrict__ ws, int M, int R,
                                                                uint16_t* __restrict__ out, long long out_sm,
                                                                long long out_sr, float alpha, float beta, Segs sg) {
  const long long n = (long long)M * R;
  const long long idx = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (idx >= n) return;
  f32x4 v[SPLITS];
#pragma unroll
  for (int k = 0; k < SPLITS; ++k) v[k] = *reinterpret_cast<const f32x4*>(ws + (long long)k * n + idx);
#pragma unroll
  for (int w = SPLITS / 2; w > 0; w /= 2)
#pragma unroll
    for (int k = 0; k < w; ++k) v[k] += v[k + w];
  const f32x4 s = v[0];
  const int m = (int)(idx / R), r = (int)(idx - (long long)m * R);
  uint16_t* o = out + (long long)m * out_sm + (long long)(sg.ocol[seg_of(sg, m)] + r) * out_sr;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float prev = beta != 0.f ? beta * bf2f(o[j * out_sr]) : 0.f;
    o[j * out_sr] = f2bf(prev + alpha * s[j]);
  }
}

}  // namespace

// Number of row splits for a [T, M] operand (power of two, >= 256 rows per split, ~1k workgroups).
extern "C" int ftc_lora_wgrad_splits(int T, int M) {
  const int ncb = M / MB;
  int s = 1;
  while (s < 64 && s * 2 * ncb <= 1024 && T % (s * 2 * TT) == 0 && T / (s * 2) >= 256) s *= 2;
  return s;
}

// Requirements (checked by the binding): T % 64 == 0, M % 128 == 0, R % 8 == 0, R <= 64, 16-byte
// aligned rows (ld % 8 == 0, base pointers 16-byte aligned); ws holds splits * M * R floats.
// nseg segments (<= 4; m_end ascending, multiples of 128, last = M), see Segs.
extern "C" int ftc_lora_wgrad(const void* x, long long ldx, const void* y, long long ldy, float* ws, int T, int M,
                              int R, void* out, long long out_sm, long long out_sr, float alpha, float beta, int nseg,
                              const int* m_end, const int* ycol, const int* ocol, hipStream_t stream) {
  if (T % TT != 0 || M % MB != 0 || R % 8 != 0 || R <= 0 || R > 64 || nseg < 1 || nseg > 4) return -1;
  Segs sg{};
  sg.n = nseg;
  for (int i = 0; i < nseg; ++i) {
    if (m_end[i] % MB != 0 || (i > 0 && m_end[i] <= m_end[i - 1]) || ycol[i] % 8 != 0) return -1;
    sg.m_end[i] = m_end[i];
    sg.ycol[i] = ycol[i];
    sg.ocol[i] = ocol[i];
  }
  if (sg.m_end[nseg - 1] != M) return -1;
  const int splits = ftc_lora_wgrad_splits(T, M);
  const int ncb = M / MB;
  const int rows = T / splits;
  if (R > 32)
    hipLaunchKernelGGL(lora_wgrad_kernel<2>, dim3(ncb * splits), dim3(256), 0, stream, (const uint16_t*)x, ldx,
                       (const uint16_t*)y, ldy, ws, M, R, rows, ncb, sg);
  else
    hipLaunchKernelGGL(lora_wgrad_kernel<1>, dim3(ncb * splits), dim3(256), 0, stream, (const uint16_t*)x, ldx,
                       (const uint16_t*)y, ldy, ws, M, R, rows, ncb, sg);
  const long long n = (long long)M * R;
  const dim3 rg((unsigned)((n / 4 + 255) / 256));
  auto out16 = (uint16_t*)out;
#define RED_CASE(SP)                                                                                       \
  case SP:                                                                                                \
    hipLaunchKernelGGL(lora_wgrad_reduce_kernel<SP>, rg, dim3(256), 0, stream, ws, M, R, out16, out_sm, out_sr, \
                       alpha, beta, sg);                                                                  \
    break;
  switch (splits) {
    RED_CASE(1) RED_CASE(2) RED_CASE(4) RED_CASE(8) RED_CASE(16) RED_CASE(32) RED_CASE(64)
    default: return -1;
  }
#undef RED_CASE
  return (int)hipGetLastError();
}
