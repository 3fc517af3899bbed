// Shared device helpers of the LoRA "tail" producers: kernels that form the rank-r product of the tensor
// they write, straight into that tensor's spare columns (swiglu_lora.hip, rmsnorm.hip).  A wave-private
// swizzled LDS tile turns coalesced row data into v_mfma_f32_16x16x32_bf16 A fragments; the four waves'
// 16 x 16 fp32 partials meet in LDS (write_tail).  Included (after common.h) inside each file's
// anonymous namespace.
#pragma once

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kRows = 16;
constexpr int kWaves = 4;

DEV_INLINE bf16x8 as_frag(const uint4& v) { return __builtin_bit_cast(bf16x8, v); }

DEV_INLINE f32x4 mfma16(const uint4& a, const uint4& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(a), as_frag(b), c, 0, 0, 0);
}

// Sum the four waves' [16 x 16] partials per column tile and write the bf16 tail (+ zero padding).
template <int NCT>
DEV_INLINE void write_tail(f32x4 (&acc)[NCT], float* red, uint16_t* base, long long rs, long long r0, long long rows,
                        int col0, int Rp) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int t = 0; t < NCT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[((wave * NCT + t) * 4 + i) * 64 + lane] = acc[t][i];
  __syncthreads();
  // 16 rows x (NCT*16) values; thread -> (t, lane, i) over the first wave-set of the reduction image
  for (int idx = tid; idx < NCT * 4 * 64; idx += 256) {
    const int t = idx / 256, rem = idx % 256, i = rem / 64, ln = rem % 64;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) s += red[((w * NCT + t) * 4 + i) * 64 + ln];
    const long long row = r0 + 4 * (ln >> 4) + i;
    if (row < rows) base[row * rs + col0 + t * 16 + (ln & 15)] = f2bf(s);
  }
  const int zc = (Rp - NCT * 16) / 8;  // zero 16-byte chunks per row
  for (int idx = tid; idx < kRows * zc; idx += 256) {
    const long long row = r0 + idx / zc;
    if (row < rows)
      *reinterpret_cast<uint4*>(base + row * rs + col0 + NCT * 16 + 8 * (idx % zc)) = make_uint4(0u, 0u, 0u, 0u);
  }
}

// Wave-private LDS tile [RT*16 rows][128 cols] bf16 with the 16-byte chunk index XOR-swizzled by
// (row & 15): the coalesced row writes (16 lanes x 16 B per row) and the MFMA fragment reads (16 rows
// x one chunk per quarter-wave) are both conflict-free.
DEV_INLINE __amdgpu_buffer_rsrc_t make_rsrc_n(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
DEV_INLINE uint4 bload16(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
  return make_uint4(v[0], v[1], v[2], v[3]);
}
DEV_INLINE void bstore16(const uint4& v, __amdgpu_buffer_rsrc_t r, int voff, int soff) {
  const u32x4 d = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(d, r, voff, soff, 0);
}

DEV_INLINE int tile_off(int row, int chunk) { return row * 256 + ((chunk ^ (row & 15)) << 4); }

