// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels of finetune_controller_amd.
//
// Conventions used by every kernel in csrc/kernels:
//   * wave64: lane = threadIdx.x & 63, wave reductions over 64 lanes with __shfl_xor;
//   * bf16 is moved as raw 16-bit words, 8 per 16-byte vector (uint4) -- hipcc does not
//     auto-vectorise bf16 loads (guide: Guideline 13), so every memory-bound kernel loads
//     16 B per lane;
//   * float -> bf16 goes through the __bf16 cast, which hipcc lowers to v_cvt_pk_bf16_f32
//     (round-to-nearest-even, NaN preserving);
//   * launchers are extern "C" host functions taking raw pointers + hipStream_t so that the
//     kernels compile without torch headers; csrc/binding.cpp adapts them to at::Tensor.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DEV_INLINE __device__ __forceinline__

namespace ftc {

constexpr int kWave = 64;

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

// Raw buffer resource over a wave-uniform base pointer (guide T8): loads then take one 32-bit VGPR
// offset + an SGPR offset instead of a 64-bit VGPR address per row.
DEV_INLINE __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
DEV_INLINE u32x4 buf_load16(__amdgpu_buffer_rsrc_t r, int voff_bytes, int soff_bytes) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, voff_bytes, soff_bytes, 0);
}

// One LDS-DMA piece (buffer_load_dwordx4 ... lds: 16 B per lane, lane-linear at M0 = lds) as inline
// asm, so hipcc keeps it out of its own s_waitcnt bookkeeping (through the builtin, every ds_read of
// ANOTHER stage gets a compiler vmcnt(0) in front of it and the prefetch drains).  The caller counts
// completion with explicit vmcnt waits.  M0 is saved / restored inside the statement (compiler-
// reserved).  The operands must come from SALU (kernel arguments, blockIdx / readfirstlane-derived
// values computed well before): no VALU-written SGPR hazard is padded here.
DEV_INLINE void lds_dma16_at(__amdgpu_buffer_rsrc_t r, unsigned dst, int voff, int soff) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(r), "s"(dst), "s"(soff)
      : "memory");
}
// the same without saving M0 (two SALU fewer per piece): only for a kernel whose compiled code has no M0
// use of its own -- the "m0-owned" marker lets tools/check_asm_hazards.py prove that on every build
DEV_INLINE void lds_dma16_m0(__amdgpu_buffer_rsrc_t r, unsigned dst, int voff, int soff) {
  asm volatile("s_mov_b32 m0, %2 ; m0-owned\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
               :
               : "v"(voff), "s"(r), "s"(dst), "s"(soff)
               : "memory");
}
DEV_INLINE unsigned lds_addr(const void* lds) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)lds;
}
DEV_INLINE void lds_dma16(__amdgpu_buffer_rsrc_t r, const void* lds, int voff, int soff) {
  lds_dma16_at(r, lds_addr(lds), voff, soff);
}
// the same with the LDS destination made provably wave-uniform (readfirstlane: an SGPR for the M0 write,
// which is an SALU read of it -- no VALU-written-SGPR wait states needed, guide §5.7 item 2)
DEV_INLINE void lds_dma16_u(__amdgpu_buffer_rsrc_t r, const void* lds, int voff, int soff) {
  lds_dma16_at(r, __builtin_amdgcn_readfirstlane(lds_addr(lds)), voff, soff);
}

DEV_INLINE float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
DEV_INLINE float bf_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
DEV_INLINE float bf2f(uint16_t u) { return __uint_as_float(((uint32_t)u) << 16); }

DEV_INLINE uint16_t f2bf(float x) {
  __bf16 b = (__bf16)x;
  return __builtin_bit_cast(uint16_t, b);
}
// pack two floats into one dword of 2 x bf16 (lo in bits 0..15)
DEV_INLINE uint32_t pack_bf2(float lo, float hi) {
  f32x2 v = {lo, hi};
  bf16x2 b = __builtin_convertvector(v, bf16x2);
  return __builtin_bit_cast(uint32_t, b);
}

// 8 bf16 <-> 8 floats
DEV_INLINE void unpack8(const uint4& v, float* f) {
  f[0] = bf_lo(v.x); f[1] = bf_hi(v.x);
  f[2] = bf_lo(v.y); f[3] = bf_hi(v.y);
  f[4] = bf_lo(v.z); f[5] = bf_hi(v.z);
  f[6] = bf_lo(v.w); f[7] = bf_hi(v.w);
}
DEV_INLINE uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack_bf2(f[0], f[1]);
  v.y = pack_bf2(f[2], f[3]);
  v.z = pack_bf2(f[4], f[5]);
  v.w = pack_bf2(f[6], f[7]);
  return v;
}

DEV_INLINE float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
DEV_INLINE float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `red` needs NT/64 floats of LDS.
template <int NT>
DEV_INLINE float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += red[i];
  __syncthreads();
  return r;
}
template <int NT>
DEV_INLINE float block_max(float v, float* red) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r = fmaxf(r, red[i]);
  __syncthreads();
  return r;
}

// Grid size for grid-stride memory-bound kernels: enough blocks to fill 256 CUs x 8,
// never more than the work needs (guide Guideline 11).
inline int stream_grid(long long work_items, int block) {
  long long g = (work_items + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

// One work item per thread: the grid-stride element-wise kernels launched this way run their loop once.
// At the Llama-3-8B SwiGLU shape a one-shot grid streams 5.90 TB/s against 5.0-5.3 for 2-8 workgroups
// per CU walking the tensor (profiles/r4/hbm/stream.log), AdamW 6.07 vs 5.62 (profiles/r4/adamw/); plain
// SwiGLU fwd / bwd 0.241 / 0.423 vs 0.277 / 0.465 ms, split-K fold 0.104 vs 0.112 (profiles/r4/oneshot/).
inline int oneshot_grid(long long work_items, int block) {
  long long g = (work_items + block - 1) / block;
  if (g > 0x7fffffffLL) g = 0x7fffffffLL;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace ftc
