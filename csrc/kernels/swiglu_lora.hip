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

#include <cstdlib>

using namespace ftc;

namespace {

#include "lora_tail.h"

DEV_INLINE float silu_f(float g) { return g / (1.0f + __expf(-g)); }

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

// ====================================================================================================
// SwiGLU backward fused with the LoRA weight-gradient partials of BOTH neighbouring projections.
//
// Besides dgu and its row tail dgu B_gu (above), the weight gradients that need the MLP's big
// tensors are formed here from the values in registers / LDS instead of by separate streaming passes
// (csrc/kernels/lora_wgrad.hip re-reading dgu, 940 MB, and h, 470 MB, per Llama-3-8B layer):
//
//   dB_gu[c, r]   = sum_t dgu[t, c] xa[t, seg(c) * 16 + r]     xa = s x A_gu^T (gate | up tails, 2 x 16)
//   dA_down^T[f, r] = sum_t h[t, f] dyb[t, r]                  h = silu(g) u recomputed, dyb = dy_down B_down
//
// Both reduce over tokens, the row tail over columns, so the grid tiles BOTH: a workgroup owns RB
// token rows x 512 gate|up column pairs (4 waves x 128) and writes fp32 partials -- row tail per
// column block, dB / dA per row block -- that two small reduction launches fold (deterministic, no
// atomics).  Per 16-row sub-tile and wave: coalesced g / u / da loads (256 B per row and
// instruction), dg / du / h into wave-private swizzled LDS tiles, then
//   * row tail:  v_mfma_f32_16x16x32_bf16, A = dg / du row fragments, B = B^T rows held in registers
//                for the whole row loop (the wave's columns never change),
//   * dB, dA:    v_mfma_f32_16x16x16_bf16 with BOTH operands read column-wise by ds_read_b64_tr_b16
//                (4 rows x 16 columns per 16-lane group: k = token) from the dg / du / h tiles and
//                from the wave's small xa / dyb tiles.
// Per-segment LoRA rank 16 (the all-linear r = 16 configuration); other ranks take the unfused path.
namespace {

typedef short s16x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4v lds_s16x4v;

DEV_INLINE f32x4 mfma16k16(const s16x4v& a, const s16x4v& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
// transposed 4-row x 16-column read: lane 4q+p of each 16-lane group addresses row q, columns 4p..4p+3
DEV_INLINE s16x4v tr4(const char* p) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4v*)p); }

struct WgArgs {
  const uint16_t* gu;
  const uint16_t* da;
  long long da_rs;
  uint16_t* dgu;
  long long dgu_rs;
  const uint16_t* bt;  // B^T [32, 2F]: rows 0..15 gate (over gate columns), 16..31 up (over up columns)
  long long ldb;
  const uint16_t* xa;  // [T, 32] (row stride xa_rs): s x A_gu^T, gate tail | up tail
  long long xa_rs;
  const uint16_t* dyb;  // [T, 16] (row stride dyb_rs): dy_down B_down
  long long dyb_rs;
  float* p_tail;  // [ncb][T][32]
  float* p_b;     // [nrb][2F][16]
  float* p_a;     // [nrb][F][16]
  int T, F, RB, ncb;
};

constexpr int kCB = 512;  // gate|up column pairs per workgroup (128 per wave)

// byte offset of (row, col) in a wave tile [16][128] bf16 with the 16-byte chunk swizzle of tile_off
DEV_INLINE int tcol_off(int row, int col) { return row * 256 + ((((col >> 3) ^ (row & 15)) & 15) << 4) + (col & 7) * 2; }

// The next 16-row sub-tile's loads are issued before the current one is consumed (0.517 vs 0.528 ms at the
// Llama-3-8B MLP shape, profiles/r3/swiglu_pf*.log; the load-at-the-top schedule is in git history).
__global__ __launch_bounds__(256, 2) void swiglu_bwd_wgrad_kernel(WgArgs a) {
  __shared__ __attribute__((aligned(16))) char tiles[kWaves][3][16 * 256];  // dg, du, h
  __shared__ __attribute__((aligned(16))) char xat[kWaves][16 * 64];       // xa sub-tile [16][32]
  __shared__ __attribute__((aligned(16))) char dyt[kWaves][16 * 32];       // dyb sub-tile [16][16]
  __shared__ float red[2][kWaves * 2 * 4 * 64];                            // row-tail partials, 2 buffers
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int F = a.F;
  const int cb = blockIdx.x % a.ncb, rb = blockIdx.x / a.ncb;
  const int cw = cb * kCB + 128 * wave;  // this wave's first gate column
  const long long rbeg = (long long)rb * a.RB;
  const long long rend = rbeg + a.RB < a.T ? rbeg + a.RB : a.T;
  const int cq = lane & 15, rq = lane >> 4;  // coalesced: 16-byte chunk, row within 4
  const int fr = lane & 15, fq = lane >> 4;  // fragment: row / column, k group
  char* my = tiles[wave][0];

  // row-tail B fragments (16x16x32): lane holds bt[tile][col = k0 + 8 fq .. +8] with tile row fr
  uint4 bfg[4], bfu[4];
  {
    const __amdgpu_buffer_rsrc_t rb_ = make_rsrc_n(a.bt, 0x7fffffffu);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      bfg[m] = bload16(rb_, (int)((fr * a.ldb + cw + 32 * m + 8 * fq) * 2), 0);
      bfu[m] = bload16(rb_, (int)(((16 + fr) * a.ldb + F + cw + 32 * m + 8 * fq) * 2), 0);
    }
  }
  f32x4 accb[16], acca[8];
#pragma unroll
  for (int j = 0; j < 16; ++j) accb[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 8; ++j) acca[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // The g / u loads (2/3 of the streamed bytes) are issued one sub-tile ahead: rows r0 + 16.. leave
  // right after the element-wise pass of rows r0.. has consumed their registers, so they fly under this
  // sub-tile's MFMAs and row-tail reduction (whose barrier waits on LDS only, never on these loads).
  // da stays in-iteration: prefetching it too spills at two workgroups per CU.
  uint4 gv[4], uv[4];
  auto issue = [&](long long r) __attribute__((always_inline)) {
    const long long nr = rend - r < 16 ? rend - r : 16;
    // this sub-tile's rows as buffer resources: rows past the block read as zero
    const __amdgpu_buffer_rsrc_t rg = make_rsrc_n(a.gu + r * 2LL * F, (unsigned)(nr * 4LL * F));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 4 * i + rq;
      gv[i] = bload16(rg, (int)((row * 2LL * F + cw + 8 * cq) * 2), 0);
      uv[i] = bload16(rg, (int)((row * 2LL * F + F + cw + 8 * cq) * 2), 0);
    }
  };
  if (rbeg < rend) issue(rbeg);
  int sub = 0;
  for (long long r0 = rbeg; r0 < rend; r0 += 16, ++sub) {
    const long long nrows = rend - r0 < 16 ? rend - r0 : 16;
    // stores past the block's rows are dropped
    const __amdgpu_buffer_rsrc_t ro = make_rsrc_n(a.dgu + r0 * a.dgu_rs, (unsigned)(nrows * a.dgu_rs * 2));
    const __amdgpu_buffer_rsrc_t rx = make_rsrc_n(a.xa + r0 * a.xa_rs, (unsigned)(nrows * a.xa_rs * 2));
    const __amdgpu_buffer_rsrc_t ry = make_rsrc_n(a.dyb + r0 * a.dyb_rs, (unsigned)(nrows * a.dyb_rs * 2));
    const __amdgpu_buffer_rsrc_t rd = make_rsrc_n(a.da + r0 * a.da_rs, (unsigned)(nrows * a.da_rs * 2));
    uint4 dv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) dv[i] = bload16(rd, (int)(((4 * i + rq) * a.da_rs + cw + 8 * cq) * 2), 0);
    // xa [16][32]: lane -> row lane >> 2, chunk lane & 3;  dyb [16][16]: lanes 0..31 -> row lane >> 1, chunk lane & 1
    const uint4 xv = bload16(rx, (int)(((lane >> 2) * a.xa_rs + 8 * (lane & 3)) * 2), 0);
    const uint4 yv = lane < 32 ? bload16(ry, (int)(((lane >> 1) * a.dyb_rs + 8 * (lane & 1)) * 2), 0)
                               : make_uint4(0u, 0u, 0u, 0u);
    asm volatile("" ::: "memory");  // previous sub-tile's LDS reads stay above these writes
    *reinterpret_cast<uint4*>(xat[wave] + (lane >> 2) * 64 + 16 * (lane & 3)) = xv;
    if (lane < 32) *reinterpret_cast<uint4*>(dyt[wave] + (lane >> 1) * 32 + 16 * (lane & 1)) = yv;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 4 * i + rq;
      float g[8], u[8], d[8], dg[8], du[8], h[8];
      unpack8(gv[i], g);
      unpack8(uv[i], u);
      unpack8(dv[i], d);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float sg = 1.0f / (1.0f + __expf(-g[e]));
        const float sl = g[e] * sg;
        du[e] = d[e] * sl;
        dg[e] = d[e] * u[e] * sg * (1.0f + g[e] * (1.0f - sg));
        h[e] = silu_f(g[e]) * u[e];  // the forward's h, bit for bit
      }
      const uint4 gq = pack8(dg), uq = pack8(du), hq = pack8(h);
      bstore16(gq, ro, (int)((row * a.dgu_rs + cw + 8 * cq) * 2), 0);
      bstore16(uq, ro, (int)((row * a.dgu_rs + F + cw + 8 * cq) * 2), 0);
      const int off = tile_off(row, cq);
      *reinterpret_cast<uint4*>(my + off) = gq;
      *reinterpret_cast<uint4*>(my + 16 * 256 + off) = uq;
      *reinterpret_cast<uint4*>(my + 2 * 16 * 256 + off) = hq;
    }
    if (r0 + 16 < rend) issue(r0 + 16);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-private tiles complete

    // ---- row tail: [16 rows] x (gate tile 0, up tile 1)
    f32x4 tg = f32x4{0.f, 0.f, 0.f, 0.f}, tu = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int off = tile_off(fr, 4 * m + fq);
      tg = mfma16(*reinterpret_cast<const uint4*>(my + off), bfg[m], tg);
      tu = mfma16(*reinterpret_cast<const uint4*>(my + 16 * 256 + off), bfu[m], tu);
    }
    // ---- dB (gate / up) and dA: k = the 16 token rows, operands read column-wise
    const int q = (lane & 15) >> 2, p = lane & 3, g4 = lane >> 4;
    const int trow = 4 * g4 + q;  // the row this lane addresses in a tr read
    const s16x4v xg = tr4(xat[wave] + trow * 64 + (4 * p) * 2);
    const s16x4v xu = tr4(xat[wave] + trow * 64 + (16 + 4 * p) * 2);
    const s16x4v yb = tr4(dyt[wave] + trow * 32 + (4 * p) * 2);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int off = tcol_off(trow, 16 * j + 4 * p);
      accb[j] = mfma16k16(tr4(my + off), xg, accb[j]);
      accb[8 + j] = mfma16k16(tr4(my + 16 * 256 + off), xu, accb[8 + j]);
      acca[j] = mfma16k16(tr4(my + 2 * 16 * 256 + off), yb, acca[j]);
    }
    // ---- row-tail reduction over the 4 waves (double-buffered LDS, one barrier per sub-tile)
    float* rbuf = red[sub & 1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      rbuf[((wave * 2 + 0) * 4 + i) * 64 + lane] = tg[i];
      rbuf[((wave * 2 + 1) * 4 + i) * 64 + lane] = tu[i];
    }
    // LDS-only barrier: __syncthreads' release fence would also drain the prefetch loads (vmcnt(0))
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    for (int idx = tid; idx < 2 * 4 * 64; idx += 256) {  // (tile, i, lane) -> row 4 (ln >> 4) + i, col tile*16 + (ln & 15)
      const int t = idx >> 8, i = (idx >> 6) & 3, ln = idx & 63;
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) s += rbuf[((w * 2 + t) * 4 + i) * 64 + ln];
      const long long row = r0 + 4 * (ln >> 4) + i;
      if (row < rend) a.p_tail[((long long)cb * a.T + row) * 32 + t * 16 + (ln & 15)] = s;
    }
  }
  // ---- dB / dA partials of this row block: C[m = column][n = r], lane: r = lane & 15, m = 4 (lane >> 4) + i
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = cw + 16 * j + 4 * (lane >> 4) + i;
      a.p_b[((long long)rb * 2 * F + c) * 16 + (lane & 15)] = accb[j][i];
      a.p_b[((long long)rb * 2 * F + F + c) * 16 + (lane & 15)] = accb[8 + j][i];
      a.p_a[((long long)rb * F + c) * 16 + (lane & 15)] = acca[j][i];
    }
}

// dgu tail[t][r] = bf16(sum_cb p_tail[cb][t][r]) for r < 32, zeros for 32 <= r < Rp
__global__ __launch_bounds__(256) void wgrad_tail_reduce_kernel(const float* __restrict__ p, int ncb, int T,
                                                                uint16_t* __restrict__ dgu, long long dgu_rs,
                                                                int col0, int Rp) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;  // one (t, 8-column chunk)
  const int nch = Rp / 8;
  if (idx >= (long long)T * nch) return;
  const long long t = idx / nch;
  const int ch = (int)(idx - t * nch);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (ch < 4) {
    for (int k = 0; k < ncb; ++k) {
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(p + ((long long)k * T + t) * 32 + 8 * ch);
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(p + ((long long)k * T + t) * 32 + 8 * ch + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s[e] += v0[e];
        s[4 + e] += v1[e];
      }
    }
  }
  *reinterpret_cast<uint4*>(dgu + t * dgu_rs + col0 + 8 * ch) = pack8(s);
}

// mgB[c][seg(c) * 16 + r] += alpha * sum_rb p_b[rb][c][r]   (c < 2F; seg = c >= F)
// mgA[r][f] (row stride ldA)  += alphaA * sum_rb p_a[rb][f][r]
__global__ __launch_bounds__(256) void wgrad_col_reduce_kernel(const float* __restrict__ pb, const float* __restrict__ pa,
                                                               int nrb, int F, uint16_t* __restrict__ mgB,
                                                               long long ldB, float alphaB, uint16_t* __restrict__ mgA,
                                                               long long ldA, float alphaA) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;  // one (row, 4 r) of B then of A
  const long long nB = 2LL * F * 4, nA = (long long)F * 4;
  if (idx < nB) {
    const long long c = idx >> 2;
    const int r = 4 * (int)(idx & 3);
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < nrb; ++k) s += *reinterpret_cast<const f32x4*>(pb + ((long long)k * 2 * F + c) * 16 + r);
    uint16_t* o = mgB + c * ldB + (c >= F ? 16 : 0) + r;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = f2bf(bf2f(o[e]) + alphaB * s[e]);
  } else if (idx < nB + nA) {
    const long long i2 = idx - nB;
    const long long f = i2 >> 2;
    const int r = 4 * (int)(i2 & 3);
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < nrb; ++k) s += *reinterpret_cast<const f32x4*>(pa + ((long long)k * F + f) * 16 + r);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      uint16_t* o = mgA + (long long)(r + e) * ldA + f;
      *o = f2bf(bf2f(*o) + alphaA * s[e]);
    }
  }
}

}  // namespace

// Row-block size and workspace (floats) of the fused backward for T tokens and F = ffn width.
extern "C" int ftc_swiglu_wgrad_plan(long long T, int F, int* rb, long long* ws_floats) {
  if (F % kCB != 0 || T <= 0) return -1;
  const int ncb = F / kCB;
  // workgroup target: partial traffic grows with ncb + nrb, balance wants whole rounds of the
  // 2-per-CU residency (512 = one round on 256 CUs; profiles/r3/wgrad_wgs/)
  constexpr int target = 512;
  long long nrb = target / ncb > 0 ? target / ncb : 1;
  long long r = (T + nrb - 1) / nrb;
  r = (r + 15) / 16 * 16;
  if (r < 64) r = 64;
  nrb = (T + r - 1) / r;
  *rb = (int)r;
  *ws_floats = (long long)ncb * T * 32 + nrb * 2LL * F * 16 + nrb * (long long)F * 16;
  return 0;
}

extern "C" int ftc_swiglu_bwd_wgrad(const void* da, long long da_rs, const void* gu, void* dgu, long long dgu_rs,
                                    long long T, int F, const void* bt, long long ldb, const void* xa, long long xa_rs,
                                    const void* dyb, long long dyb_rs, float* ws, void* mgB, long long ldB,
                                    float alphaB, void* mgA, long long ldA, float alphaA, int Rp, hipStream_t stream) {
  int RB;
  long long wsf;
  if (ftc_swiglu_wgrad_plan(T, F, &RB, &wsf) != 0) return -1;
  // buffer resources are made per 16-row sub-tile: no 2 GiB limit on the tensors themselves
  if (Rp < 32 || Rp % 8 != 0 || dgu_rs < 2LL * F + Rp || da_rs % 8 || dgu_rs % 8 || ldb % 8 || xa_rs % 8 ||
      dyb_rs % 8 || T >= (1LL << 31))
    return -1;
  const int ncb = F / kCB;
  const int nrb = (int)((T + RB - 1) / RB);
  WgArgs a{(const uint16_t*)gu, (const uint16_t*)da, da_rs, (uint16_t*)dgu, dgu_rs, (const uint16_t*)bt, ldb,
           (const uint16_t*)xa, xa_rs, (const uint16_t*)dyb, dyb_rs, ws, ws + (long long)ncb * T * 32,
           ws + (long long)ncb * T * 32 + (long long)nrb * 2 * F * 16, (int)T, F, RB, ncb};
  hipLaunchKernelGGL(swiglu_bwd_wgrad_kernel, dim3(ncb * nrb), dim3(256), 0, stream, a);
  const long long nt = T * (Rp / 8);
  hipLaunchKernelGGL(wgrad_tail_reduce_kernel, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, stream, a.p_tail,
                     ncb, (int)T, (uint16_t*)dgu, dgu_rs, 2 * F, Rp);
  const long long nc = 2LL * F * 4 + (long long)F * 4;
  hipLaunchKernelGGL(wgrad_col_reduce_kernel, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, stream, a.p_b, a.p_a,
                     nrb, F, (uint16_t*)mgB, ldB, alphaB, (uint16_t*)mgA, ldA, alphaA);
  return (int)hipGetLastError();
}

// ====================================================================================================
// Skinny "tail" GEMM: tail[t, 0:Rp] = X[t, 0:K] . Bm[0:Rp, 0:K]^T written into X's own spare columns
// (X row stride ldx >= K + Rp; rows of Bm past 16 * nct are treated as zero and their columns written
// as zeros).  This is the rank-r product of an augmented LoRA GEMM when its producer is a kernel that
// cannot form it (flash attention output, RMSNorm output / residual gradient, ...): a pure stream of X
// at HBM rate -- hipBLASLt's 64x64 tiles run these [T, K] x [K, 64] shapes at ~4.3 TB/s.  Same
// structure as the SwiGLU kernels above: 32 rows x 4 waves (K split in 128-column chunks), coalesced
// 256-byte row loads, a wave-private swizzled LDS tile into 16x16x32 MFMA fragments, LDS reduction.
namespace {

template <int NCT>
__global__ __launch_bounds__(256) void tail_gemm_kernel(uint16_t* __restrict__ X, long long ldx, long long rows, int K,
                                                        const uint16_t* __restrict__ Bm, long long ldb, int Rp) {
  constexpr int RT = 2, NL = RT * 4;
  __shared__ __attribute__((aligned(16))) char lds[kWaves * RT * 16 * 256];
  __shared__ float red[kWaves * RT * NCT * 4 * 64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  char* my = lds + wave * (RT * 16 * 256);
  const long long r0 = (long long)blockIdx.x * (RT * 16);
  const int cq = lane & 15, rq = lane >> 4;
  const int fr = lane & 15, fq = lane >> 4;
  const long long nrows = rows - r0 < RT * 16 ? rows - r0 : RT * 16;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc_n(X + r0 * ldx, (unsigned)(nrows * ldx * 2LL));
  const __amdgpu_buffer_rsrc_t rb = make_rsrc_n(Bm, 0x7fffffffu);
  const int vx = (int)(rq * ldx + 8 * cq) * 2;
  const int vb = (int)(fr * ldb + 8 * fq) * 2;
  f32x4 acc[RT][NCT];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int t = 0; t < NCT; ++t) acc[r][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nch = K / 128;
  const int c0 = (nch * wave) / kWaves, c1 = (nch * (wave + 1)) / kWaves;
  for (int c = c0; c < c1; ++c) {
    const int k0 = c * 128;
    uint4 xv[NL];
#pragma unroll
    for (int i = 0; i < NL; ++i) xv[i] = bload16(rx, vx + 2 * k0, (int)(i * 8 * ldx));
    uint4 bf[4][NCT];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int t = 0; t < NCT; ++t) bf[m][t] = bload16(rb, vb + 2 * (k0 + 32 * m), (int)(t * 16 * ldb * 2));
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < NL; ++i) *reinterpret_cast<uint4*>(my + tile_off(4 * i + rq, cq)) = xv[i];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        const uint4 a = *reinterpret_cast<const uint4*>(my + tile_off(r * 16 + fr, 4 * m + fq));
#pragma unroll
        for (int t = 0; t < NCT; ++t) acc[r][t] = mfma16(a, bf[m][t], acc[r][t]);
      }
  }
#pragma unroll
  for (int r = 0; r < RT; ++r)
    write_tail<NCT>(acc[r], red + r * (kWaves * NCT * 4 * 64), X, ldx, r0 + 16 * r, rows, K, Rp);
}

}  // namespace

extern "C" int ftc_tail_gemm(void* x, long long ldx, long long rows, int K, const void* Bm, long long ldb, int nct,
                             int Rp, hipStream_t stream) {
  if (K % 128 != 0 || ldx % 8 != 0 || ldb % 8 != 0 || ldx < (long long)K + Rp || nct < 1 || nct > 4 ||
      Rp < 16 * nct || Rp % 16 != 0 || rows <= 0)  // per-block buffer resources: no 2 GiB limit
    return -1;
  const dim3 grid((unsigned)((rows + 31) / 32)), block(256);
  auto X = (uint16_t*)x;
  auto B = (const uint16_t*)Bm;
  switch (nct) {
    case 1: hipLaunchKernelGGL(tail_gemm_kernel<1>, grid, block, 0, stream, X, ldx, rows, K, B, ldb, Rp); break;
    case 2: hipLaunchKernelGGL(tail_gemm_kernel<2>, grid, block, 0, stream, X, ldx, rows, K, B, ldb, Rp); break;
    case 3: hipLaunchKernelGGL(tail_gemm_kernel<3>, grid, block, 0, stream, X, ldx, rows, K, B, ldb, Rp); break;
    default: hipLaunchKernelGGL(tail_gemm_kernel<4>, grid, block, 0, stream, X, ldx, rows, K, B, ldb, Rp); break;
  }
  return (int)hipGetLastError();
}
