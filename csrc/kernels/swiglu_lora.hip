// K9 + K5 fusion: SwiGLU forward / backward that also form the LoRA rank-r product of the tensor they
// produce, straight into the spare columns of its row-padded buffer (ops/linear.py "augmented GEMMs").
//
//   forward   h = silu(g) * u                 [T, F]   and   h (s A_down)^T   [T, Rp]  (tail of h's rows)
//   backward  dgu = dSwiGLU(da; g, u)         [T, 2F]  and   dgu B_gu         [T, Rp]  (tail of dgu's rows)
//
// Without the fusion each tail product is a separate skinny GEMM that re-reads the whole producer
// output from HBM (h: 470 MB, dgu: 940 MB per Llama-3-8B layer at 16k tokens; 0.10 + 0.17 ms).  Here
// the product is formed from the values while they are still in registers:
//
// * one workgroup = 32 (forward) / 16 (backward) token rows x 4 waves; wave w owns a contiguous
//   quarter of the F columns and walks it in 128-column chunks;
// * operands are loaded coalesced (256 contiguous bytes per row per instruction), the outputs are
//   computed and stored, and the SAME rounded bf16 values go through a wave-private swizzled LDS tile
//   into the v_mfma_f32_16x16x32_bf16 A-fragment layout (lane l: row l & 15, k-octet l >> 4) -- so the
//   tail has the inputs of the two-GEMM path (fp32 accumulation, bf16 result).  (A first version that
//   loaded straight in fragment layout -- 16 rows x 64 B per instruction -- ran 25-50 % slower than
//   the plain SwiGLU kernel + the skinny GEMM: tools/bench_swiglu_tail.py);
// * the B fragment is a 16-byte row slice of (s A) [Rp, F] (forward) or of B^T [Rp, 2F] (backward),
//   a few MB that stay L2-resident across the 1k workgroups;
// * the four waves' 16 x 16 fp32 partials meet in LDS; columns past the NCT*16 formed ones are
//   written as zeros (the augmented GEMM reads all Rp spare columns).
#include "common.h"

using namespace ftc;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kRows = 16;
constexpr int kWaves = 4;

FTC_DEV float silu_f(float g) { return g / (1.0f + __expf(-g)); }

FTC_DEV bf16x8 as_frag(const uint4& v) { return __builtin_bit_cast(bf16x8, v); }

FTC_DEV f32x4 mfma16(const uint4& a, const uint4& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(a), as_frag(b), c, 0, 0, 0);
}

// Sum the four waves' [16 x 16] partials per column tile and write the bf16 tail (+ zero padding).
template <int NCT>
FTC_DEV void write_tail(f32x4 (&acc)[NCT], float* red, uint16_t* base, long long rs, long long r0, long long rows,
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
FTC_DEV __amdgpu_buffer_rsrc_t make_rsrc_n(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
FTC_DEV uint4 bload16(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
  return make_uint4(v[0], v[1], v[2], v[3]);
}
FTC_DEV void bstore16(const uint4& v, __amdgpu_buffer_rsrc_t r, int voff, int soff) {
  const u32x4 d = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(d, r, voff, soff, 0);
}

FTC_DEV int tile_off(int row, int chunk) { return row * 256 + ((chunk ^ (row & 15)) << 4); }

// Coalesced layout of a [RT*16, 128] chunk: load i of a lane covers row 4 i + (lane >> 4), columns
// 8 (lane & 15) .. +8 -- 256 contiguous bytes per row per instruction.
//
// MODE 0 (forward):  X = h = silu(g) u written to out, tail += h . Bm[t]^T over the F columns
// MODE 1 (backward): X = dg | du written to out, tail += dg . Bm[t]^T (gate columns) + du . Bm[t]^T (up
//                    columns of Bm, offset F); SPLIT: gate uses tiles [0, NCT/2), up [NCT/2, NCT)
template <int MODE, int NCT, int RT, bool SPLIT>
__global__ __launch_bounds__(256) void swiglu_lora_kernel(const uint16_t* __restrict__ gu,
                                                          const uint16_t* __restrict__ da, long long da_rs,
                                                          uint16_t* __restrict__ out, long long out_rs, long long rows,
                                                          int F, const uint16_t* __restrict__ Bm, long long ldb,
                                                          int Rp) {
  constexpr int NH = MODE == 0 ? 1 : 2;            // produced halves: h, or dg | du
  constexpr int NL = RT * 4;                        // coalesced loads per operand per chunk
  constexpr int TG0 = 0, TG1 = SPLIT ? NCT / 2 : NCT;  // tiles fed by the first half
  constexpr int TU0 = SPLIT ? NCT / 2 : 0, TU1 = NCT;  // tiles fed by the second half (MODE 1)
  __shared__ __attribute__((aligned(16))) char lds[kWaves * NH * RT * 16 * 256];
  __shared__ float red[kWaves * RT * NCT * 4 * 64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  char* my = lds + wave * (NH * RT * 16 * 256);
  const long long r0 = (long long)blockIdx.x * (RT * 16);
  const int cq = lane & 15, rq = lane >> 4;  // coalesced: chunk within the 128 columns, row within 4
  const int fr = lane & 15, fq = lane >> 4;  // fragment: row (A) / column (B), k-octet

  // Buffer resources over this block's rows (host guarantees < 2 GiB per tensor): one 32-bit VGPR
  // offset per lane, the load index i in the scalar offset; rows past the end read as zero and their
  // stores are dropped by the range check (no clamping, no per-row pointers).
  const long long nrows = rows - r0 < RT * 16 ? rows - r0 : RT * 16;
  const __amdgpu_buffer_rsrc_t rg = make_rsrc_n(gu + r0 * 2LL * F, (unsigned)(nrows * 4LL * F));
  const __amdgpu_buffer_rsrc_t ro = make_rsrc_n(out + r0 * out_rs, (unsigned)(nrows * out_rs * 2LL));
  const __amdgpu_buffer_rsrc_t rd =
      make_rsrc_n(MODE == 1 ? da + r0 * da_rs : gu, MODE == 1 ? (unsigned)(nrows * da_rs * 2LL) : 0u);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc_n(Bm, 0x7fffffffu);
  const int vg = (rq * 2 * F + 8 * cq) * 2, vo = (int)(rq * out_rs + 8 * cq) * 2;
  const int vd = MODE == 1 ? (int)(rq * da_rs + 8 * cq) * 2 : 0;
  const int vb = (int)(fr * ldb + 8 * fq) * 2;

  f32x4 acc[RT][NCT];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int t = 0; t < NCT; ++t) acc[r][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nch = F / 128;
  const int c0 = (nch * wave) / kWaves, c1 = (nch * (wave + 1)) / kWaves;
  for (int c = c0; c < c1; ++c) {
    const int k0 = c * 128;
    uint4 gv[NL], uv[NL], dv[MODE == 1 ? NL : 1];
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      gv[i] = bload16(rg, vg + 2 * k0, i * 16 * F);
      uv[i] = bload16(rg, vg + 2 * (F + k0), i * 16 * F);
      if constexpr (MODE == 1) dv[i] = bload16(rd, vd + 2 * k0, (int)(i * 8 * da_rs));
    }
    // B fragments of the 4 k-steps of this chunk (L2-resident operand)
    uint4 bf[4][NCT];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int t = 0; t < NCT; ++t) {
        const bool need_g = t >= TG0 && t < TG1, need_u = MODE == 1 && t >= TU0 && t < TU1;
        const int soff = (int)(t * 16 * ldb * 2);
        if (need_g) bf[m][t] = bload16(rb, vb + 2 * (k0 + 32 * m), soff);
        else if (need_u) bf[m][t] = bload16(rb, vb + 2 * (F + k0 + 32 * m), soff);
      }
    asm volatile("" ::: "memory");  // the previous chunk's fragment reads stay above these writes
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      float g[8], u[8];
      unpack8(gv[i], g);
      unpack8(uv[i], u);
      const int trow = 4 * i + rq;
      if constexpr (MODE == 0) {
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = silu_f(g[e]) * u[e];
        const uint4 ov = pack8(o);
        bstore16(ov, ro, vo + 2 * k0, (int)(i * 8 * out_rs));
        *reinterpret_cast<uint4*>(my + tile_off(trow, cq)) = ov;
      } else {
        float d[8], dg[8], du[8];
        unpack8(dv[i], d);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float sg = 1.0f / (1.0f + __expf(-g[e]));
          const float sl = g[e] * sg;
          du[e] = d[e] * sl;
          dg[e] = d[e] * u[e] * sg * (1.0f + g[e] * (1.0f - sg));
        }
        const uint4 gq = pack8(dg), uq = pack8(du);
        bstore16(gq, ro, vo + 2 * k0, (int)(i * 8 * out_rs));
        bstore16(uq, ro, vo + 2 * (F + k0), (int)(i * 8 * out_rs));
        *reinterpret_cast<uint4*>(my + tile_off(trow, cq)) = gq;
        *reinterpret_cast<uint4*>(my + RT * 16 * 256 + tile_off(trow, cq)) = uq;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-private tile complete
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        const int off = tile_off(r * 16 + fr, 4 * m + fq);
        const uint4 ag = *reinterpret_cast<const uint4*>(my + off);
#pragma unroll
        for (int t = TG0; t < TG1; ++t) acc[r][t] = mfma16(ag, bf[m][t], acc[r][t]);
        if constexpr (MODE == 1) {
          const uint4 au = *reinterpret_cast<const uint4*>(my + RT * 16 * 256 + off);
#pragma unroll
          for (int t = TU0; t < TU1; ++t) {
            if constexpr (!SPLIT) {
              // generic: the up half pairs with the up columns of B^T (loaded separately below)
              const uint4 bu = bload16(rb, vb + 2 * (F + k0 + 32 * m), (int)(t * 16 * ldb * 2));
              acc[r][t] = mfma16(au, bu, acc[r][t]);
            } else {
              acc[r][t] = mfma16(au, bf[m][t], acc[r][t]);
            }
          }
        }
      }
  }
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    write_tail<NCT>(acc[r], red + r * (kWaves * NCT * 4 * 64), out, out_rs, r0 + 16 * r, rows, NH * F, Rp);
  }
}

}  // namespace

// h / dgu are row-padded buffers: h_rs >= F + Rp, dgu_rs >= 2F + Rp.  nct = ceil(R / 16) column tiles
// are formed (1..4), the remaining Rp - 16 nct tail columns are zeroed.  Backward with split = 1: the
// gate rows of B feed tail tiles [0, nct/2) and the up rows [nct/2, nct) (block-diagonal B of the packed
// gate|up projection with 16-aligned ranks).
namespace {
template <int MODE, int NCT, int RT, bool SPLIT>
void launch(const void* gu, const void* da, long long da_rs, void* out, long long out_rs, long long rows, int F,
            const void* Bm, long long ldb, int Rp, hipStream_t stream) {
  const dim3 grid((unsigned)((rows + RT * 16 - 1) / (RT * 16))), block(256);
  hipLaunchKernelGGL((swiglu_lora_kernel<MODE, NCT, RT, SPLIT>), grid, block, 0, stream, (const uint16_t*)gu,
                     (const uint16_t*)da, da_rs, (uint16_t*)out, out_rs, rows, F, (const uint16_t*)Bm, ldb, Rp);
}
}  // namespace

extern "C" int ftc_swiglu_fwd_lora(const void* gu, void* h, long long rows, int F, long long h_rs, const void* Am,
                                   long long lda, int nct, int Rp, hipStream_t stream) {
  if (F % 128 != 0 || h_rs % 8 != 0 || lda % 8 != 0 || nct < 1 || nct > 4 || Rp < 16 * nct || Rp % 16 != 0 ||
      h_rs < F + Rp || rows <= 0)
    return -1;
  switch (nct) {
    case 1: launch<0, 1, 2, false>(gu, nullptr, 0, h, h_rs, rows, F, Am, lda, Rp, stream); break;
    case 2: launch<0, 2, 2, false>(gu, nullptr, 0, h, h_rs, rows, F, Am, lda, Rp, stream); break;
    case 3: launch<0, 3, 2, false>(gu, nullptr, 0, h, h_rs, rows, F, Am, lda, Rp, stream); break;
    default: launch<0, 4, 2, false>(gu, nullptr, 0, h, h_rs, rows, F, Am, lda, Rp, stream); break;
  }
  return (int)hipGetLastError();
}

extern "C" int ftc_swiglu_bwd_lora(const void* da, long long da_rs, const void* gu, void* dgu, long long rows, int F,
                                   long long dgu_rs, const void* Bt, long long ldb, int nct, int split, int Rp,
                                   hipStream_t stream) {
  if (F % 128 != 0 || da_rs % 8 != 0 || dgu_rs % 8 != 0 || ldb % 8 != 0 || nct < 1 || nct > 4 || Rp < 16 * nct ||
      Rp % 16 != 0 || dgu_rs < 2LL * F + Rp || rows <= 0 || (split && nct % 2 != 0))
    return -1;
  if (split) {
    if (nct == 2) launch<1, 2, 1, true>(gu, da, da_rs, dgu, dgu_rs, rows, F, Bt, ldb, Rp, stream);
    else launch<1, 4, 1, true>(gu, da, da_rs, dgu, dgu_rs, rows, F, Bt, ldb, Rp, stream);
  } else {
    switch (nct) {
      case 1: launch<1, 1, 1, false>(gu, da, da_rs, dgu, dgu_rs, rows, F, Bt, ldb, Rp, stream); break;
      case 2: launch<1, 2, 1, false>(gu, da, da_rs, dgu, dgu_rs, rows, F, Bt, ldb, Rp, stream); break;
      case 3: launch<1, 3, 1, false>(gu, da, da_rs, dgu, dgu_rs, rows, F, Bt, ldb, Rp, stream); break;
      default: launch<1, 4, 1, false>(gu, da, da_rs, dgu, dgu_rs, rows, F, Bt, ldb, Rp, stream); break;
    }
  }
  return (int)hipGetLastError();
}
