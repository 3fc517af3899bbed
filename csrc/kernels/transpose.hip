// bf16 2-D transpose through LDS: Y[C, R] = X[R, C]^T (X with row stride ldx, Y with row stride ldy).
//
// Used to hand hipBLASLt the operand layouts it runs fastest (tools/bench_dw_gemm.py,
// tools/bench_gemms.py): the full fine-tune weight gradient dW += dy^T x with x transposed ("tn",
// 14-24 % faster than both operands T-major) and the input gradient dx = dy W with a per-step W^T copy
// (TN, 14-16 % faster than NN).  torch's generic transpose copy runs at ~1 TB/s on these shapes; this
// one streams at HBM rate:
//   * one 256-thread workgroup per 64 x 64 tile, 16-byte row loads (8 bf16 per lane, 128 contiguous
//     bytes per tile row) into an LDS tile padded to 66 columns,
//   * transposed gathers of 8 elements per lane (2-byte LDS reads: with the pad, the 64 lanes of a
//     read hit 32 distinct dwords -- conflict-free) and 16-byte stores along the output rows,
//   * consecutive workgroups take consecutive row tiles of one 64-column panel of X, i.e. adjacent
//     128-byte segments of the same 64 output rows.
#include "common.h"

using namespace ftc;

namespace {

constexpr int TS = 64;       // tile edge
constexpr int LDP = TS + 2;  // padded LDS row (elements)

__global__ __launch_bounds__(256) void transpose_kernel(const uint16_t* __restrict__ X, long long ldx,
                                                        uint16_t* __restrict__ Y, long long ldy, int R, int C,
                                                        int tiles_r) {
  __shared__ uint16_t t[TS * LDP];
  const int tid = threadIdx.x;
  const int tr = blockIdx.x % tiles_r, tc = blockIdx.x / tiles_r;
  const long long r0 = (long long)tr * TS, c0 = (long long)tc * TS;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = tid + 256 * i;
    const int row = e >> 3, cg = e & 7;
    const long long r = r0 + row, c = c0 + 8 * cg;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (r < R && c < C) v = *reinterpret_cast<const uint4*>(X + r * ldx + c);
    uint32_t* dst = reinterpret_cast<uint32_t*>(t + row * LDP + 8 * cg);  // 4-byte aligned (LDP even)
    dst[0] = v.x;
    dst[1] = v.y;
    dst[2] = v.z;
    dst[3] = v.w;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = tid + 256 * i;
    const int oc = e >> 3, og = e & 7;  // output row (= input column) and 8-element group
    const long long yr = c0 + oc, yc = r0 + 8 * og;
    uint16_t g[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = t[(8 * og + j) * LDP + oc];
    if (yr < C && yc < R) {
      uint4 v;
      v.x = (uint32_t)g[0] | ((uint32_t)g[1] << 16);
      v.y = (uint32_t)g[2] | ((uint32_t)g[3] << 16);
      v.z = (uint32_t)g[4] | ((uint32_t)g[5] << 16);
      v.w = (uint32_t)g[6] | ((uint32_t)g[7] << 16);
      *reinterpret_cast<uint4*>(Y + yr * ldy + yc) = v;
    }
  }
}

}  // namespace

// R, C multiples of 8; ldx, ldy multiples of 8 (16-byte rows); partial edge tiles are guarded.
extern "C" int ftc_transpose(const void* x, long long ldx, void* y, long long ldy, int R, int C, hipStream_t stream) {
  if (R <= 0 || C <= 0 || R % 8 != 0 || C % 8 != 0 || ldx % 8 != 0 || ldy % 8 != 0 || ldx < C || ldy < R) return -1;
  const int tiles_r = (R + TS - 1) / TS, tiles_c = (C + TS - 1) / TS;
  const long long nt = (long long)tiles_r * tiles_c;
  if (nt > 0x7fffffffLL) return -1;
  hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)nt), dim3(256), 0, stream, (const uint16_t*)x, ldx,
                     (uint16_t*)y, ldy, R, C, tiles_r);
  return (int)hipGetLastError();
}
