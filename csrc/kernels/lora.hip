// K6: LoRA merge / unmerge   W[out,in] += scale * B[out,r] @ A[r,in]   (bf16 out, fp32 accumulate).
//
// Used at adapter export / inference hand-off (one launch per projection, 224 projections for an
// all-linear Llama-3-8B adapter).  The rank is tiny (r*segments <= 192), so this is a streaming
// read-modify-write of W with the rank-r product formed in registers: each lane owns 8 consecutive
// columns of one output row (16-byte W access), keeps its B row slice in registers (broadcast
// loads) and streams the matching A columns, which are shared by all rows and stay in L2.
//
// seg_rows > 0 selects the packed-projection layout: output rows [s*seg_rows, (s+1)*seg_rows) use
// only rank slice s of A/B (the block-diagonal B of a packed qkv / gate_up projection), so a packed
// merge costs the same as merging the segments one by one.
#include "common.h"

using namespace ftc;

__global__ __launch_bounds__(256) void lora_merge_kernel(uint16_t* __restrict__ W, const uint16_t* __restrict__ A,
                                                         const uint16_t* __restrict__ Bm, int out_f, int in_f,
                                                         int r_total, int r_seg, int seg_rows, float scale) {
  const int cv = in_f >> 3;
  const long long total = (long long)out_f * cv;
  for (long long it = (long long)blockIdx.x * 256 + threadIdx.x; it < total; it += (long long)gridDim.x * 256) {
    const int o = (int)(it / cv);
    const int c = (int)(it - (long long)o * cv);
    const int r0 = seg_rows > 0 ? (o / seg_rows) * r_seg : 0;
    const int r1 = seg_rows > 0 ? r0 + r_seg : r_total;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = r0; r < r1; ++r) {
      const float b = bf2f(Bm[(long long)o * r_total + r]);
      float a8[8];
      unpack8(reinterpret_cast<const uint4*>(A + (long long)r * in_f)[c], a8);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += b * a8[j];
    }
    uint4* wp = reinterpret_cast<uint4*>(W + (long long)o * in_f) + c;
    float w8[8];
    unpack8(*wp, w8);
#pragma unroll
    for (int j = 0; j < 8; ++j) w8[j] += scale * acc[j];
    *wp = pack8(w8);
  }
}

extern "C" int ftc_lora_merge(void* w, const void* a, const void* b, int out_f, int in_f, int r, int seg_rows,
                              float scale, hipStream_t stream) {
  if (in_f % 8 != 0) return -1;
  int r_seg = r;
  if (seg_rows > 0) {
    if (out_f % seg_rows != 0) return -1;
    const int nseg = out_f / seg_rows;
    if (r % nseg != 0) return -1;
    r_seg = r / nseg;
  }
  const int grid = ftc::stream_grid((long long)out_f * (in_f / 8), 256);
  hipLaunchKernelGGL(lora_merge_kernel, dim3(grid), dim3(256), 0, stream, (uint16_t*)w, (const uint16_t*)a,
                     (const uint16_t*)b, out_f, in_f, r, r_seg, seg_rows, scale);
  return (int)hipGetLastError();
}
