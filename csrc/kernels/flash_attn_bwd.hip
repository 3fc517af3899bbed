// K2: flash-attention backward for gfx950 (causal / sliding window, GQA, bf16, recompute P from LSE).
//
// Two launches, no float atomics anywhere (bitwise reproducible):
//   1. dQ (below, launched first): also forms delta[b,h,q] = sum_d dO*O for its rows from the dO
//      fragments it holds, and writes the [-delta | -lse/scale] row constants of the workspace
//   2. dK/dV: one workgroup = 128 keys of one (batch, kv head); it sweeps ALL G = H/KV query heads
//      of the group and every 32-row query slice that can see its keys, so dK and dV are complete
//      when the workgroup ends (GQA summation inside the kernel, no cross-workgroup reduction).
//         S  [q][k] = Q K^T    - LSE/scale   (accumulator pre-loaded with the row constant)
//         dP'[q][k] = dO V^T   - delta
//         P = exp2(c S), dS = P * dP'
//         dV^T[d][k] += dO^T P        dK^T[d][k] += Q^T dS
//      "key on the lane": S and dP' accumulators have the key on the MFMA lane, so they ARE the
//      B operands of the two accumulating products (permuted-k order, guide §3), and the dO^T / Q^T
//      A operands come from one LDS image each through ds_read_b64_tr_b16.
//   dQ: one workgroup = 128 query rows of one (batch, q head); K/V tiles stream through LDS like the
//      forward:  S^T = K Q^T, dP^T = V dO^T (query on the lane: LSE/delta are per-lane scalars),
//      dQ^T[d][q] += K^T dS^T with K^T read by tr_b16 from the same K image.
// The dQ pass recomputes S and dP (7 MFMA products per tile pair instead of 5) -- on MI355X the
// alternative, summing dQ over key blocks with fp32 atomics, is bound by the ≈1.3 TB/s atomic rate
// (≈4.3 GB of adds per Llama-3-8B layer at 16k tokens), slower than the extra MFMAs.
#include "common.h"

#include <cstdlib>

using namespace ftc;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr float LOG2E = 1.4426950408889634f;

DEV_INLINE int swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
template <int D>
DEV_INLINE int lds_off(int r, int chunk) {
  constexpr int NCH = D / 8;
  return r * (D * 2) + 16 * ((chunk ^ swz(r)) & (NCH - 1));
}
DEV_INLINE bf16x8 as_bf8(const uint4& v) { return __builtin_bit_cast(bf16x8, v); }
DEV_INLINE bf16x8 pack8_bf(const f32x16& p, int base) {
  uint4 u;
  u.x = pack_bf2(p[base + 0], p[base + 1]);
  u.y = pack_bf2(p[base + 2], p[base + 3]);
  u.z = pack_bf2(p[base + 4], p[base + 5]);
  u.w = pack_bf2(p[base + 6], p[base + 7]);
  return as_bf8(u);
}
// Epilogue rows (lanes l and l ^ 32 hold the same row, d runs {8 g4 + 4 hh + 0..3} of each 32-wide tile):
// WIDE swaps dword pairs across the lane halves (v_permlane32_swap) so each lane stores 16 contiguous
// d as 2 x dwordx4 per tile instead of 4 x dwordx2 (the store tail is issue-bound; forward: -1 %).
#ifndef BWD_WIDE_STORE
#define BWD_WIDE_STORE 1
#endif
template <int DT>
DEV_INLINE void store_rows(uint16_t* p, const f32x16* acc, float sc, int hh, bool wide) {
  if (BWD_WIDE_STORE && wide) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      uint32_t w[4][2];
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        w[g4][0] = pack_bf2(acc[dt][4 * g4 + 0] * sc, acc[dt][4 * g4 + 1] * sc);
        w[g4][1] = pack_bf2(acc[dt][4 * g4 + 2] * sc, acc[dt][4 * g4 + 3] * sc);
      }
      const auto a0 = __builtin_amdgcn_permlane32_swap(w[0][0], w[2][0], false, false);
      const auto a1 = __builtin_amdgcn_permlane32_swap(w[0][1], w[2][1], false, false);
      const auto b0 = __builtin_amdgcn_permlane32_swap(w[1][0], w[3][0], false, false);
      const auto b1 = __builtin_amdgcn_permlane32_swap(w[1][1], w[3][1], false, false);
      const int d = dt * 32 + 16 * hh;
      *reinterpret_cast<uint4*>(p + d) = make_uint4(a0[0], a1[0], a0[1], a1[1]);
      *reinterpret_cast<uint4*>(p + d + 8) = make_uint4(b0[0], b1[0], b0[1], b1[1]);
    }
  } else {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        uint2 w;
        w.x = pack_bf2(acc[dt][4 * g4 + 0] * sc, acc[dt][4 * g4 + 1] * sc);
        w.y = pack_bf2(acc[dt][4 * g4 + 2] * sc, acc[dt][4 * g4 + 3] * sc);
        *reinterpret_cast<uint2*>(p + dt * 32 + 8 * g4 + 4 * hh) = w;
      }
  }
}
// A operand (32 rows x 16 k, permuted k) via two transposed reads of an LDS image whose rows are k
// and columns are the A rows: elements 0..3 <- image rows kb+4h+0..3, elements 4..7 <- +8.
// tr_offsets() gives the lane's two byte offsets for kb = 0; since the swizzle depends on r & 15 only,
// kb (a multiple of 16) is a plain immediate on top (few live address VGPRs).
template <int D>
DEV_INLINE int2 tr_offsets(int colbase, int lane) {
  const int hh = lane >> 5, gi = (lane >> 4) & 3, li = lane & 15;
  const int trq = li >> 2, trp = li & 3;
  const int col = colbase + 16 * (gi & 1) + 4 * trp;
  const int chunk = col >> 3, half8 = (col & 7) ? 8 : 0;
  const int r1 = 4 * hh + trq;
  return make_int2(lds_off<D>(r1, chunk) + half8, lds_off<D>(r1 + 8, chunk) + half8);
}
template <int D>
DEV_INLINE bf16x8 tr_read(const char* img, int kb, int2 off) {
  s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + off.x + kb * D * 2));
  s16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + off.y + kb * D * 2));
  s16x8 va = {v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
  return __builtin_bit_cast(bf16x8, va);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
// dQ pass: packed-fp32 scale / shift ahead of the exponentials -- off: the forward's packed form measured
// slower (tools/pk_softmax_ab.sh, profiles/r3/pk_softmax/)
#ifndef BWD_PK_EXP
#define BWD_PK_EXP 0
#endif

struct BwdArgs {
  const uint16_t *q, *k, *v, *o, *dout;
  const float* lse;
  float* delta;
  uint16_t *dq, *dk, *dv;
  long long q_rs, kv_rs, o_rs, dq_rs, dkv_rs, do_rs;
  int B, S, H, KV;
  float scale, c;  // c = scale * log2(e)
  int causal, window;
  const int* doc_start;  // [B*S] packed-sequence document bounds (null: one document per sequence):
  const int* doc_end;    //   key k visible to query q iff doc_start[q] <= k, i.e. q < doc_end[k]
  // keys >= kv_valid are masked for every query (right-padded tail of non-causal attention).  Only
  // the dQ pass masks them: dK / dV rows of those keys are discarded by the caller, and a masked key
  // never reaches a valid key's dK / dV.
  int kv_valid;
  // RoPE folded into the epilogues (D = 128): q and k were rotated (HF rotate_half, fp32 cos / sin
  // [max_pos, 64]) by their producer, so dQ and dK leave as the gradients of the UN-rotated q / k --
  // the inverse rotation the producer's backward would otherwise run as a separate pass over dq / dk.
  // pos = rpos[token] or (token % S); rcos == null: no rotation
  const float* rcos;
  const float* rsin;
  const int* rpos;
};

// Inverse rotation of one row's gradient held as store_rows' accumulators: element i of tile dt is
// d = 32 dt + 8 (i >> 2) + 4 hh + (i & 3), so d and d + 64 are tiles dt and dt + 2 of the same lane.
// (y1, y2) = (u1 c - u2 s, u2 c + u1 s)  =>  (du1, du2) = (g1 c + g2 s, g2 c - g1 s)
template <int DT>
DEV_INLINE void rope_inv_rows(f32x16* acc, const BwdArgs& a, long long token, int hh) {
  static_assert(DT == 4, "RoPE epilogue: head_dim 128");
  const int pos = a.rpos ? a.rpos[token] : (int)(token % a.S);
  const float* cr = a.rcos + (long long)pos * 64 + 4 * hh;
  const float* sr = a.rsin + (long long)pos * 64 + 4 * hh;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const float4 c = *reinterpret_cast<const float4*>(cr + 32 * dt + 8 * g4);
      const float4 sn = *reinterpret_cast<const float4*>(sr + 32 * dt + 8 * g4);
      const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {sn.x, sn.y, sn.z, sn.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = 4 * g4 + e;
        const float g1 = acc[dt][i], g2 = acc[dt + 2][i];
        acc[dt][i] = g1 * cc[e] + g2 * ss[e];
        acc[dt + 2][i] = g2 * cc[e] - g1 * ss[e];
      }
    }
}

// (Removed in round 5: the separate delta = rowsum(dO * O) pass -- bwd_dq_kernel forms delta from the
// operands it already loads and runs first; 1.892 vs 1.933 ms per layer backward, profiles/r5/attn_ab2/.)

// ---------------------------------------------------------------- 1. dK / dV
// One workgroup = 4 waves = 256 keys of one (batch, kv head); each wave owns 64 keys as two 32-key
// halves and keeps their dK^T / dV^T accumulators (2 x 2 x D/32 tiles = 256 VGPRs at D=128) for the
// whole sweep over the G query heads x 32-row query slices, so the 512-register single-wave budget
// (launch_bounds(256, 1)) is used.  Per slice and wave: 64 MFMAs between barriers, the Q/dO slice is
// read from LDS once for both halves (dV/dK tr-operands shared), the next slice's global loads fly
// under them (register staging into the other LDS slot, one barrier per slice).
// Block order: heavy (early, causal) key blocks first; the key blocks of one (batch, kv head) pair
// share an XCD so its Q/dO slices are L2 hits for the co-running blocks.
// One slice's LDS-DMA for a dK/dV wave: NG 1 KiB pieces of Q and of dO (lane-linear destinations,
// pre-swizzled per-lane source offsets qvo/dvo) and the 256-byte row-constant piece.  A device-only
// function rather than a lambda in the kernel: the host pass cannot instantiate these builtins.
// SPLIT (a slice of fewer 1 KiB pieces per matrix than waves, D = 64 with 8 waves): each wave DMAs ONE
// piece -- waves [0, P) a piece of Q, waves [P, 2P) the same piece of dO -- so every wave still issues
// the same number of DMA instructions per slice (the counted vmcnt stays wave-uniform).
// QR = 2 (64-row slices): the row constants are two 256-byte pieces (-lse/scale rows, then -delta rows).
// one 4-byte-per-lane LDS-DMA piece (the row constants), inline asm like common.h lds_dma16
DEV_INLINE void lds_dma4(__amdgpu_buffer_rsrc_t r, const void* lds, int voff, int soff) {
  const unsigned dst = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)lds;
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "buffer_load_dword %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(r), "s"(dst), "s"(soff)
      : "memory");
}

template <int D, int NG, int RPG, int QBYTES, bool SPLIT = false, int QR = 1>
DEV_INLINE void dkdv_dma(__amdgpu_buffer_rsrc_t qr, __amdgpu_buffer_rsrc_t dr, __amdgpu_buffer_rsrc_t cr, const int* qvo,
                      const int* dvo, int cvo, int cvo2, int qso, int dso, int cso, char* base, int wave) {
  // inline asm (lds_dma16 / lds_dma4), not the builtin: hipcc tracks builtin LDS-DMA and, unable to prove
  // the ring slots disjoint from the row-constant reads, drained every in-flight slice (vmcnt(0)) at the
  // start of each phase A -- the counted waits in sync_slice are the only ones the ring needs
  if constexpr (SPLIT) {
    constexpr int P = QBYTES / 1024;
    if (wave < P)
      lds_dma16(qr, base + wave * 1024, qvo[0], qso);
    else
      lds_dma16(dr, base + QBYTES + (wave - P) * 1024, dvo[0], dso);
  } else {
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      const int r0 = (wave * NG + i) * RPG;
      lds_dma16(qr, base + r0 * D * 2, qvo[i], qso);
      lds_dma16(dr, base + QBYTES + r0 * D * 2, dvo[i], dso);
    }
  }
  lds_dma4(cr, base + 2 * QBYTES, cvo, cso);
  if constexpr (QR == 2)  // second piece: -delta of the 64 rows (cvo addressed the -lse/scale rows)
    lds_dma4(cr, base + 2 * QBYTES + 256, cvo2, cso);
}

// 8 waves x 32 keys (HW = one 32-key half per wave), two waves per SIMD (256 registers each).
// "Ping-pong": the two waves sharing a SIMD (w, w + 4) run each query slice's two phases in opposite
// order between the same pair of barriers: half 0 does A(j) then B(j), half 1 does B(j - 1) then A(j),
// where A = the S / dP' MFMA chains and B = softmax / masking VALU + the dV / dK MFMAs.  One wave's exp /
// mask / pack work then issues under its partner's MFMAs instead of both waves idling the matrix pipe at
// the same time (guide: MI355X_MICROARCH.md "Two waves per SIMD").  Q/dO slices are DMA'd three slices
// ahead (DIST) into a 5-slot ring.
// QR = 32-row query blocks per slice: QR = 2 (D = 64) doubles the MFMA work between two barriers,
// which at D = 64 is otherwise half of D = 128's (the per-slice barrier / DMA cost stays the same).
// Measured and removed (git history, profiles/): 4 waves x 64 keys at one wave per SIMD (backward 2.094
// vs 1.788 ms), the round-4 in-wave interleaved 4-wave kernel "IL" (1.890 ms, profiles/r4/attn_final/),
// no ping-pong (2.00 vs 1.97 ms), DMA distance 2 (1.99 vs 1.96 ms), 32-row slices at D = 64, and a
// B1 B2 A order for half 1 carrying the raw S / dP' across the barrier (2.03 vs 1.96 ms).
template <int D, int QR = 1>
__global__ __launch_bounds__(512, 1) void bwd_dkdv8_kernel(BwdArgs a) {
  constexpr int HW = 1, DIST = 3;
  static_assert(QR == 1 || QR == 2, "one or two 32-row query blocks per slice");
  constexpr int NCH = D / 8, DSTEPS = D / 16, DT = D / 32;
  constexpr int BKV = 256, BQ2 = 32 * QR;
  constexpr int WAVES = 8 / HW, NT = 64 * WAVES;
  constexpr int KBYTES = BKV * D * 2, QBYTES = BQ2 * D * 2;
  constexpr int SLICE = 2 * QBYTES + 2 * BQ2 * 4;  // Q | dO | -lse/scale | -delta
  // K and the three ring slots are DISTINCT __shared__ objects: the compiler then knows (LDS alias
  // scopes) that reading one slot does not depend on the DMA still writing the others, instead of
  // draining every DMA (vmcnt(0)) before the first ds_read of each slice
  __shared__ __attribute__((aligned(16))) char Ks[KBYTES];
  __shared__ __attribute__((aligned(16))) char slot0[SLICE];
  __shared__ __attribute__((aligned(16))) char slot1[SLICE];
  __shared__ __attribute__((aligned(16))) char slot2[SLICE];
  __shared__ __attribute__((aligned(16))) char slot3[SLICE];
  __shared__ __attribute__((aligned(16))) char slot4[SLICE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5, lr = lane & 31;
  const int S = a.S, G = a.H / a.KV;
  const int nkb = S / BKV;
  const int npairs = a.B * a.KV;
  int kb, pair;
  {
    const int bid = blockIdx.x;
    if ((npairs & 7) == 0) {
      const int xcd = bid & 7, slot = bid >> 3, ppx = npairs >> 3;
      kb = slot / ppx;
      pair = (slot % ppx) * 8 + xcd;
    } else {
      kb = bid / npairs;
      pair = bid % npairs;
    }
  }
  const int kvh = pair % a.KV, b = pair / a.KV;
  const int kv0 = kb * BKV;
  const int wkey0 = kv0 + wave * 32 * HW;  // this wave's first key

  // stage the block's K rows into LDS; V^T fragments (B operand of dP) to registers
  const uint16_t* kbase = a.k + ((long long)b * S) * a.kv_rs + (long long)kvh * D;
  {
    constexpr int RPP = NT / NCH;
    const int lrow = tid / NCH, lch = tid % NCH;
    const auto krs = make_rsrc(kbase + (long long)kv0 * a.kv_rs);
    const int voff = (lrow * (int)a.kv_rs + lch * 8) * 2;
#pragma unroll
    for (int p = 0; p < BKV / RPP; ++p)
      *reinterpret_cast<u32x4*>(Ks + lds_off<D>(p * RPP + lrow, lch)) = buf_load16(krs, voff, p * RPP * (int)a.kv_rs * 2);
  }
  bf16x8 vf[HW][DSTEPS];
#pragma unroll
  for (int j = 0; j < HW; ++j) {
    const uint16_t* vp = a.v + ((long long)b * S + wkey0 + 32 * j + lr) * a.kv_rs + (long long)kvh * D + 8 * hh;
#pragma unroll
    for (int s = 0; s < DSTEPS; ++s) vf[j][s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(vp + 16 * s));
  }

  f32x16 dv[HW][DT], dk[HW][DT];
#pragma unroll
  for (int j = 0; j < HW; ++j)
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) { dv[j][t][i] = 0.f; dk[j][t][i] = 0.f; }

  // query range that can see this key block
  int qbeg = a.causal ? kv0 : 0;
  int qend = S;
  if (a.window > 0) qend = min(S, kv0 + BKV - 1 + a.window);
  // packed documents: queries past the end of the block's last key's document see none of its keys;
  // per half, the smallest doc_end of its keys (dmin, wave-uniform: per-element masks needed beyond
  // it).  The lane's own doc_end is loaded only inside the masked branch (no loop-long register).
  int dmin[HW];
#pragma unroll
  for (int j = 0; j < HW; ++j) dmin[j] = 0x3fffffff;
  const int* de_row = a.doc_end ? a.doc_end + (long long)b * S : nullptr;
  if (de_row) {
    qend = min(qend, de_row[kv0 + BKV - 1]);
#pragma unroll
    for (int j = 0; j < HW; ++j) dmin[j] = de_row[wkey0 + 32 * j];
  }
  qbeg = (qbeg / BQ2) * BQ2;
  const int nqt = (qend - qbeg + BQ2 - 1) / BQ2;
  // Q / dO / row-constant slices arrive by LDS-DMA (global_load_lds_dwordx4: no staging VGPRs) into a
  // 5-slot ring, three slices ahead of the compute; one raw barrier per slice with a COUNTED vmcnt so the
  // next slice's DMA stays in flight across it (guide §5 "Pipelining across barriers").  The swizzled
  // LDS image is produced by pre-swizzling the per-lane global source (the DMA writes lane-linearly).
  constexpr int PIECES = BQ2 * D * 2 / 1024;         // 1 KiB pieces per matrix per slice
  constexpr bool SPLIT = PIECES < WAVES;             // D = 64, 8 waves: one piece of Q OR dO per wave
  static_assert(!SPLIT || 2 * PIECES == WAVES, "split DMA: one piece per wave");
  constexpr int NG = SPLIT ? 1 : PIECES / WAVES;     // 1 KiB DMA pieces per wave per matrix
  static_assert(NG >= 1, "each wave DMAs at least one 1 KiB piece of Q and of dO");
  constexpr int PER_SLICE = (SPLIT ? 1 : 2 * NG) + QR;  // DMA instructions per wave per slice (+ row constants)
  constexpr int RPG = 1024 / (D * 2);                // rows per 1 KiB piece
  // DMA sources as buffer resources (SGPRs) + per-lane loop-invariant 32-bit offsets: the slice's head
  // and row position go into the scalar offset, so no 64-bit address VGPRs stay live in the loop
  const auto qrsrc = make_rsrc(a.q + (long long)b * S * a.q_rs);
  const auto drsrc = make_rsrc(a.dout + (long long)b * S * a.do_rs);
  const auto crsrc = make_rsrc(a.delta);  // workspace [-delta | -lse/scale]
  int qvo[NG], dvo[NG];
#pragma unroll
  for (int i = 0; i < NG; ++i) {
    const int row = ((SPLIT ? wave % PIECES : wave * NG) + i) * RPG + lane / NCH, pc = lane % NCH;
    const int lc = (pc ^ swz(row)) & (NCH - 1);  // pre-swizzled source, lane-linear destination
    qvo[i] = (row * (int)a.q_rs + lc * 8) * 2;
    dvo[i] = (row * (int)a.do_rs + lc * 8) * 2;
  }
  // QR = 1: lanes 0..31 -lse/scale of the 32 rows, lanes 32..63 -delta (every wave issues the same
  // piece); QR = 2: one piece of the 64 rows' -lse/scale (cvo) and one of their -delta (cvo2)
  const int cvo = QR == 1 ? (lr + (hh ? 0 : a.B * a.H * S)) * 4 : (lane + a.B * a.H * S) * 4;
  const int cvo2 = lane * 4;
  auto issue = [&](int it_, char* base_) {
    const int g_ = it_ / nqt, qt_ = qbeg + (it_ % nqt) * BQ2;
    const int hq_ = kvh * G + g_;
    dkdv_dma<D, NG, RPG, QBYTES, SPLIT, QR>(qrsrc, drsrc, crsrc, qvo, dvo, cvo, cvo2, (hq_ * D + qt_ * (int)a.q_rs) * 2,
                                 (hq_ * D + qt_ * (int)a.do_rs) * 2, ((b * a.H + hq_) * S + qt_) * 4, base_, wave);
  };
  constexpr int VM_ONE = 0x0F70 | (PER_SLICE & 15) | ((PER_SLICE >> 4) << 14);  // vmcnt(PER_SLICE)
  constexpr int VM_TWO = 0x0F70 | ((2 * PER_SLICE) & 15) | (((2 * PER_SLICE) >> 4) << 14);  // vmcnt(2 PER_SLICE)
  constexpr int VM_ZERO = 0x0F70;                                               // vmcnt(0)
  constexpr int LGKM_ZERO = 0xC07F;                                             // lgkmcnt(0)

  const int total = G * nqt;
  // K staging and the V fragments are ordinary loads: retire them before the first DMA so no
  // compiler-inserted wait inside the loop has to count them
  __builtin_amdgcn_s_waitcnt(VM_ZERO);
  __syncthreads();  // K staged (no DMA in flight yet: a plain barrier is fine here)
  if (total > 0) issue(0, slot0);
  if (total > 1) issue(1, slot1);
  if (total > 2) issue(2, slot2);
  f32x16 s[QR][HW], dp[QR][HW];  // S / dP' of the slice between phase A and phase B (registers)
  // phase A: S[q][k], dP'[q][k] for both 32-key halves in one k-loop (rows q in registers, key on the
  // lane): the Q / dO A-fragments are read once for both halves, the K fragments once for all row
  // blocks -- 2 QR HW independent MFMA chains
  auto phaseA = [&](const char* Qs) __attribute__((always_inline)) {
    const char* Ds = Qs + QBYTES;
    const float* lse_s = reinterpret_cast<const float*>(Ds + QBYTES);
    const float* dlt_s = lse_s + BQ2;
#pragma unroll
    for (int r = 0; r < QR; ++r)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const float4 lv = *reinterpret_cast<const float4*>(lse_s + 32 * r + 8 * g4 + 4 * hh);
        const float4 dv4 = *reinterpret_cast<const float4*>(dlt_s + 32 * r + 8 * g4 + 4 * hh);
#pragma unroll
        for (int j = 0; j < HW; ++j) {
          s[r][j][4 * g4 + 0] = lv.x; s[r][j][4 * g4 + 1] = lv.y; s[r][j][4 * g4 + 2] = lv.z; s[r][j][4 * g4 + 3] = lv.w;
          dp[r][j][4 * g4 + 0] = dv4.x; dp[r][j][4 * g4 + 1] = dv4.y; dp[r][j][4 * g4 + 2] = dv4.z;
          dp[r][j][4 * g4 + 3] = dv4.w;
        }
      }
#pragma unroll
    for (int st = 0; st < DSTEPS; ++st) {
      u32x4 qa[QR], da[QR];
#pragma unroll
      for (int r = 0; r < QR; ++r) {
        qa[r] = *reinterpret_cast<const u32x4*>(Qs + lds_off<D>(32 * r + lr, 2 * st + hh));
        da[r] = *reinterpret_cast<const u32x4*>(Ds + lds_off<D>(32 * r + lr, 2 * st + hh));
      }
      u32x4 kk[HW];
#pragma unroll
      for (int j = 0; j < HW; ++j)
        kk[j] = *reinterpret_cast<const u32x4*>(Ks + lds_off<D>(wave * 32 * HW + 32 * j + lr, 2 * st + hh));
#pragma unroll
      for (int r = 0; r < QR; ++r)
#pragma unroll
        for (int j = 0; j < HW; ++j)
          s[r][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, qa[r]), __builtin_bit_cast(bf16x8, kk[j]),
                                                            s[r][j], 0, 0, 0);
#pragma unroll
      for (int r = 0; r < QR; ++r)
#pragma unroll
        for (int j = 0; j < HW; ++j)
          dp[r][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, da[r]), vf[j][st], dp[r][j], 0, 0, 0);
    }
    // fragment reads of two k-steps in flight ahead of the MFMA chain, the rest interleaved
    {
      constexpr int NDS = (2 * QR + HW) * DSTEPS, NMF = 2 * HW * QR * DSTEPS, PRE = (HW == 1 ? 1 : 2) * (2 * QR + HW);
      constexpr int REM = NDS - PRE, Q = REM / NMF, X = REM % NMF;
      __builtin_amdgcn_sched_group_barrier(0x100, PRE, 0);
#pragma unroll
      for (int i = 0; i < X; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, Q + 1, 0);
      }
#pragma unroll
      for (int i = X; i < NMF; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if constexpr (Q > 0) __builtin_amdgcn_sched_group_barrier(0x100, Q, 0);
      }
    }
  };
  // phase B1: P, dS (bf16 B operands of the accumulating products) -- exp / mask / pack VALU work
  bf16x8 pb[QR][HW][2], sb[QR][HW][2];
  auto phaseB1 = [&](const int it) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < QR; ++r) {
      const int qt = qbeg + (it % nqt) * BQ2 + 32 * r;
#pragma unroll
      for (int j = 0; j < HW; ++j) {
        const int key = wkey0 + 32 * j + lr;
        const int kmin = wkey0 + 32 * j;
        const bool need_mask = (a.causal && qt < kmin + 31) || (a.window > 0 && qt + 31 - kmin >= a.window) ||
                               qt + 31 >= dmin[j];
#pragma unroll
        for (int i = 0; i < 16; ++i) s[r][j][i] = __builtin_amdgcn_exp2f(a.c * s[r][j][i]);
        if (need_mask) {  // wave-uniform; query q = qt + (i&3) + 8(i>>2) + 4hh valid iff key <= q < key + window
          const int base = qt + 4 * hh;
          const int lo = (a.causal ? key : -0x3fffffff) - base;
          const int dend = de_row ? de_row[key] : 0x40000000;
          const int hi = min(a.window > 0 ? key + a.window - 1 : 0x3fffffff, dend - 1) - base;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int off = (i & 3) + 8 * (i >> 2);
            s[r][j][i] = (off >= lo && off <= hi) ? s[r][j][i] : 0.f;
          }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) dp[r][j][i] = s[r][j][i] * dp[r][j][i];
        pb[r][j][0] = pack8_bf(s[r][j], 0);
        pb[r][j][1] = pack8_bf(s[r][j], 8);
        sb[r][j][0] = pack8_bf(dp[r][j], 0);
        sb[r][j][1] = pack8_bf(dp[r][j], 8);
      }
    }
  };
  // phase B2: dV^T += dO^T P ; dK^T += Q^T dS for both halves (k of these MFMAs = the slice's query
  // rows); the dO^T / Q^T tr-operands are read once and used by both halves
  auto phaseB2 = [&](const char* Qs) __attribute__((always_inline)) {
    const char* Ds = Qs + QBYTES;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int2 to = tr_offsets<D>(dt * 32, lane);
#pragma unroll
      for (int r = 0; r < QR; ++r) {
        const bf16x8 a0 = tr_read<D>(Ds, 32 * r, to);
        const bf16x8 a1 = tr_read<D>(Ds, 32 * r + 16, to);
        const bf16x8 q0v = tr_read<D>(Qs, 32 * r, to);
        const bf16x8 q1v = tr_read<D>(Qs, 32 * r + 16, to);
#pragma unroll
        for (int j = 0; j < HW; ++j) {
          dv[j][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, pb[r][j][0], dv[j][dt], 0, 0, 0);
          dv[j][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, pb[r][j][1], dv[j][dt], 0, 0, 0);
          dk[j][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(q0v, sb[r][j][0], dk[j][dt], 0, 0, 0);
          dk[j][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(q1v, sb[r][j][1], dk[j][dt], 0, 0, 0);
        }
      }
    }
  };
  // one barrier per slice: slice it is in LDS for every wave, the DMA of slice it + 2 goes out
  auto sync_slice = [&](const int it, char* dma_slot) __attribute__((always_inline)) {
    if (it + 2 < total) {
      __builtin_amdgcn_s_waitcnt(VM_TWO);  // slices it+1, it+2 may fly on
    } else if (it + 1 < total) {
      __builtin_amdgcn_s_waitcnt(VM_ONE);  // slice it landed, it+1 may fly on
    } else {
      __builtin_amdgcn_s_waitcnt(VM_ZERO);
    }
    __builtin_amdgcn_s_waitcnt(LGKM_ZERO);
    __builtin_amdgcn_s_barrier();  // every wave's pieces of slice it are in
    if (it + DIST < total) issue(it + DIST, dma_slot);
  };
  // ping-pong over a 5-slot ring, DMA three slices ahead: slice it in slot it % 5; the DMA of slice it + 3
  // reuses the slot of slice it - 2, whose last reader (half 1's phase B2) finished before this slice's
  // barrier.  Half 1 carries only the packed P / dS operands (16 VGPRs) across the barrier:
  // ... [B2(it-1) A(it) B1(it)] ...; the halves run separate straight-line loops (one branch outside the
  // loop, not one per slice: the register allocator then sees two independent paths) with the same
  // barrier count
  if (wave < 4) {  // waves w and w + 4 share a SIMD
    auto body = [&](const int it, const char* Qs, char* dma_slot) __attribute__((always_inline)) {
      sync_slice(it, dma_slot);
      phaseA(Qs);
      phaseB1(it);
      phaseB2(Qs);
    };
    for (int it = 0; it < total; it += 5) {
      body(it, slot0, slot3);
      if (it + 1 < total) body(it + 1, slot1, slot4);
      if (it + 2 < total) body(it + 2, slot2, slot0);
      if (it + 3 < total) body(it + 3, slot3, slot1);
      if (it + 4 < total) body(it + 4, slot4, slot2);
    }
  } else {
    auto body = [&](const int it, const char* Qs, const char* Qprev, char* dma_slot) __attribute__((always_inline)) {
      sync_slice(it, dma_slot);
      if (it > 0) phaseB2(Qprev);
      phaseA(Qs);
      phaseB1(it);
    };
    for (int it = 0; it < total; it += 5) {
      body(it, slot0, slot4, slot3);
      if (it + 1 < total) body(it + 1, slot1, slot0, slot4);
      if (it + 2 < total) body(it + 2, slot2, slot1, slot0);
      if (it + 3 < total) body(it + 3, slot3, slot2, slot1);
      if (it + 4 < total) body(it + 4, slot4, slot3, slot2);
    }
    if (total > 0) {
      const int r = (total - 1) % 5;
      phaseB2(r == 0 ? slot0 : r == 1 ? slot1 : r == 2 ? slot2 : r == 3 ? slot3 : slot4);
    }
  }

  // ---- epilogue: dK = scale * dK^T^T, dV; lane owns one key row per half
#pragma unroll
  for (int j = 0; j < HW; ++j) {
    const int key = wkey0 + 32 * j + lr;
    uint16_t* dkp = a.dk + ((long long)b * S + key) * a.dkv_rs + (long long)kvh * D;
    uint16_t* dvp = a.dv + ((long long)b * S + key) * a.dkv_rs + (long long)kvh * D;
    const bool wide = (a.dkv_rs & 7) == 0;
    if constexpr (D == 128) {
      if (a.rcos) rope_inv_rows<DT>(dk[j], a, (long long)b * S + key, hh);
    }
    store_rows<DT>(dkp, dk[j], a.scale, hh, wide);
    store_rows<DT>(dvp, dv[j], 1.0f, hh, wide);
  }
}

// ---------------------------------------------------------------- dQ (launched first: forms delta)
#ifndef DQ_CINIT
#define DQ_CINIT 1
#endif
// One K/V tile by LDS-DMA: NGT 1 KiB pieces per matrix per wave (device-only: see dkdv_dma)
template <int D, int NGT, int RPG>
DEV_INLINE void kv_dma(__amdgpu_buffer_rsrc_t kr, __amdgpu_buffer_rsrc_t vr, const int* voff, int toff, char* kdst,
                    char* vdst, int wave) {
#pragma unroll
  for (int i = 0; i < NGT; ++i) {
    const int r0 = (wave * NGT + i) * RPG;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(kr, (__attribute__((address_space(3))) void*)(kdst + r0 * D * 2), 16,
                                             voff[i], toff, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(vr, (__attribute__((address_space(3))) void*)(vdst + r0 * D * 2), 16,
                                             voff[i], toff, 0, 0);
  }
}

template <int D, int OCC>
__global__ __launch_bounds__(256, OCC) void bwd_dq_kernel(BwdArgs a) {
  constexpr int NCH = D / 8, DSTEPS = D / 16, DT = D / 32;
  constexpr int BQ = 128, BK = 64;
  constexpr int TILE = BK * D * 2;
  // K/V tiles arrive by LDS-DMA (global_load_lds_dwordx4) into two distinct buffer pairs: no staging
  // registers (the register-staged version spilled at D=128) and no ds_write pass
  __shared__ __attribute__((aligned(16))) char Kt0[TILE];
  __shared__ __attribute__((aligned(16))) char Vt0[TILE];
  __shared__ __attribute__((aligned(16))) char Kt1[TILE];
  __shared__ __attribute__((aligned(16))) char Vt1[TILE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform -> scalar branches
  const int hh = lane >> 5, lr = lane & 31;
  const int S = a.S, G = a.H / a.KV;
  const int nqb = S / BQ;
  // heaviest (latest) query blocks first; q heads of one kv group adjacent
  const int qr = blockIdx.x / (a.B * a.H);
  const int rem = blockIdx.x % (a.B * a.H);
  const int b = rem / a.H, hq = rem % a.H;
  const int kvh = hq / G;
  const int qb = nqb - 1 - qr;
  const int q0 = qb * BQ;
  const int qrow = q0 + wave * 32 + lr;

  bf16x8 qf[DSTEPS], df[DSTEPS];
  {
    const uint16_t* qp = a.q + ((long long)b * S + qrow) * a.q_rs + (long long)hq * D + 8 * hh;
    const uint16_t* dp = a.dout + ((long long)b * S + qrow) * a.do_rs + (long long)hq * D + 8 * hh;
#pragma unroll
    for (int s = 0; s < DSTEPS; ++s) {
      qf[s] = as_bf8(*reinterpret_cast<const uint4*>(qp + 16 * s));
      df[s] = as_bf8(*reinterpret_cast<const uint4*>(dp + 16 * s));
    }
  }
  const long long sidx = ((long long)b * a.H + hq) * S + qrow;
  const float lse = a.lse[sidx];
  const float lse2 = lse * LOG2E;
  // delta = rowsum(dO * O) for this lane's query row, formed here from the dO fragments already in
  // registers (lane halves hh = 0 / 1 hold the two interleaved halves of the row) -- the separate delta
  // pass over dO and O is gone.  The row constants the dK/dV kernel DMAs ([-delta | -lse/scale] in the
  // workspace) are written here too: this kernel runs first.
  float dsum = 0.f;
  {
    const uint16_t* op = a.o + ((long long)b * S + qrow) * a.o_rs + (long long)hq * D + 8 * hh;
#pragma unroll
    for (int s = 0; s < DSTEPS; ++s) {
      float fo[8], fd[8];
      unpack8(*reinterpret_cast<const uint4*>(op + 16 * s), fo);
      unpack8(__builtin_bit_cast(uint4, df[s]), fd);
#pragma unroll
      for (int j = 0; j < 8; ++j) dsum += fo[j] * fd[j];
    }
  }
  dsum += __shfl_xor(dsum, 32, 64);
  const float ndlt = -dsum;
  if (hh == 0) {
    a.delta[sidx] = ndlt;
    a.delta[(long long)a.B * S * a.H + sidx] = -lse / a.scale;
  }

  int kv_end = min(a.causal ? q0 + BQ : S, a.kv_valid);
  int kv_begin = 0;
  if (a.window > 0) kv_begin = (max(0, q0 - a.window + 1) / BK) * BK;
  int dlo = -0x3fffffff, wdmax = -0x3fffffff;  // packed documents: as in the forward
  if (a.doc_start) {
    const int* ds = a.doc_start + (long long)b * S;
    dlo = ds[qrow];
    wdmax = ds[q0 + wave * 32 + 31];
    kv_begin = max(kv_begin, (ds[q0] / BK) * BK);
  }
  const int ntiles = (kv_end - kv_begin + BK - 1) / BK;
  const uint16_t* kbase = a.k + (long long)b * S * a.kv_rs + (long long)kvh * D;
  const uint16_t* vbase = a.v + (long long)b * S * a.kv_rs + (long long)kvh * D;
  constexpr int NGT = TILE / 1024 / 4;  // 1 KiB DMA pieces per wave per matrix
  constexpr int RPG = 1024 / (D * 2);  // rows per piece
  // buffer resources + per-lane loop-invariant 32-bit offsets (pre-swizzled source, lane-linear
  // destination); the tile's first row goes into the scalar offset
  const auto krs = make_rsrc(kbase), vrs = make_rsrc(vbase);
  int voff[NGT];
#pragma unroll
  for (int i = 0; i < NGT; ++i) {
    const int row = (wave * NGT + i) * RPG + lane / NCH, pc = lane % NCH;
    voff[i] = (row * (int)a.kv_rs + ((pc ^ swz(row)) & (NCH - 1)) * 8) * 2;
  }
  auto issue = [&](int kv0_, char* kdst, char* vdst) {
    kv_dma<D, NGT, RPG>(krs, vrs, voff, kv0_ * (int)a.kv_rs * 2, kdst, vdst, wave);
  };

  f32x16 dq[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) dq[t][i] = 0.f;
  // DQ_CINIT: the dP^T chains start from -delta (the query is on the lane, so one loop-invariant
  // accumulator image serves every tile as the first MFMA's C operand): dS^T = P (dP - delta) then
  // needs no per-element add (32 VALU per tile)
  f32x16 ndv;
#pragma unroll
  for (int i = 0; i < 16; ++i) ndv[i] = DQ_CINIT ? ndlt : 0.f;

  __builtin_amdgcn_s_waitcnt(0x0F70);  // retire the Q/dO/lse loads before any DMA (vmcnt(0))
  if (ntiles > 0) issue(kv_begin, Kt0, Vt0);
  auto tile = [&](const int t, const char* Kc, const char* Vc, char* Kn, char* Vn) __attribute__((always_inline)) {
    const int kv0 = kv_begin + t * BK;
    __builtin_amdgcn_s_waitcnt(0x0F70);  // this wave's pieces of tile t landed (vmcnt(0))
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();        // ... everyone's; and tile t-1's buffers are free
    if (t + 1 < ntiles) issue(kv0 + BK, Kn, Vn);  // flies under this tile's compute
    f32x16 s[2], dp[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
      for (int i = 0; i < 16; ++i) s[kt][i] = 0.f;
      dp[kt] = ndv;
      const int r = kt * 32 + lr;
#pragma unroll
      for (int st = 0; st < DSTEPS; ++st) {
        const u32x4 kv = *reinterpret_cast<const u32x4*>(Kc + lds_off<D>(r, 2 * st + hh));
        const u32x4 vv = *reinterpret_cast<const u32x4*>(Vc + lds_off<D>(r, 2 * st + hh));
        s[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kv), qf[st], s[kt], 0, 0, 0);
        dp[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, vv), df[st], dp[kt], 0, 0, 0);
      }
    }
    // keep 2 K/V fragment reads in flight against the MFMA chain (deeper ones spill at D=128)
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
    for (int i = 0; i < 4 * DSTEPS - 2; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    if constexpr (BWD_PK_EXP) {
      // scale / shift as packed fp32 pairs (v_pk_fma_f32: 16 instead of 32), exponentials scalar
      const f32x2 c2 = {a.c, a.c}, l2 = {-lse2, -lse2};
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          const f32x2 y = __builtin_elementwise_fma((f32x2){s[kt][i], s[kt][i + 1]}, c2, l2);
          s[kt][i] = __builtin_amdgcn_exp2f(y[0]);
          s[kt][i + 1] = __builtin_amdgcn_exp2f(y[1]);
        }
    } else {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i = 0; i < 16; ++i) s[kt][i] = __builtin_amdgcn_exp2f(__builtin_fmaf(a.c, s[kt][i], -lse2));
    }
    const int qmin_w = q0 + wave * 32;
    const bool need_mask = (a.causal && kv0 + BK - 1 > qmin_w) || (a.window > 0 && qmin_w + 31 - kv0 >= a.window) ||
                           kv0 + BK > a.kv_valid ||
                           kv0 < wdmax;
    if (need_mask) {  // wave-uniform; selects inside
      const int base = kv0 + 4 * hh;
      const int hi = min(a.causal ? qrow : 0x3fffffff, a.kv_valid - 1) - base;
      const int lo = max(a.window > 0 ? qrow - a.window + 1 : -0x3fffffff, dlo) - base;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int off = kt * 32 + (i & 3) + 8 * (i >> 2);
          s[kt][i] = (off >= lo && off <= hi) ? s[kt][i] : 0.f;
        }
    }
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i) dp[kt][i] = DQ_CINIT ? s[kt][i] * dp[kt][i] : s[kt][i] * (dp[kt][i] + ndlt);  // dS^T
    bf16x8 sb[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) sb[ks] = pack8_bf(dp[ks >> 1], 8 * (ks & 1));
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      bf16x8 ka[4];
      const int2 to = tr_offsets<D>(dt * 32, lane);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) ka[ks] = tr_read<D>(Kc, 16 * ks, to);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) dq[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka[ks], sb[ks], dq[dt], 0, 0, 0);
    }
  };
  for (int t = 0; t < ntiles; t += 2) {
    tile(t, Kt0, Vt0, Kt1, Vt1);
    if (t + 1 < ntiles) tile(t + 1, Kt1, Vt1, Kt0, Vt0);
  }
  uint16_t* op = a.dq + ((long long)b * S + qrow) * a.dq_rs + (long long)hq * D;
  if constexpr (D == 128) {
    if (a.rcos) rope_inv_rows<DT>(dq, a, (long long)b * S + qrow, hh);
  }
  store_rows<DT>(op, dq, a.scale, hh, (a.dq_rs & 7) == 0);
}


}  // namespace

// (Removed in round 5: skipping the causal slices / tiles a wave sees fully masked, in dK/dV and dQ -- the
// wave-uniform branch cost more than the diagonal work it saved: forward + backward 2.478 vs 2.437 ms,
// headline -0.75 %, profiles/r5/attn_skip/.)
// (Removed in round 5: a dS spill -- dK/dV stores dS^T (bf16), a third kernel forms dQ = scale dS K from
// it instead of recomputing S and dP.  dK/dV 1.435 vs 1.119 ms (2.15 GB of dS stores at the Llama-3-8B
// layer, B4 S4096) and the dS-reading dQ 0.586 vs 0.773: 2.079 vs 1.892 ms per layer, memory bound on both
// sides, profiles/r5/attn_ab2/; git history has the kernels.)
extern "C" int ftc_flash_bwd_workspace(int B, int S, int H, int D, long long* bytes) {
  *bytes = 2LL * B * H * S * sizeof(float);  // -delta, -lse/scale
  return 0;
}

// (Removed: dQ on a second stream beside dK/dV -- 2.017 vs 2.016 ms,
// profiles/r2/s8_*conc*.log: dK/dV holds every CU's registers until its last workgroups retire.)
extern "C" int ftc_flash_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                             const float* lse, void* dq, void* dk, void* dv, void* workspace, int B, int S, int H,
                             int KV, int D, long long q_rs, long long kv_rs, long long o_rs, long long do_rs,
                             long long dq_rs, long long dkv_rs, float scale, int causal, int window,
                             const int* doc_start, const int* doc_end, int kv_valid, const float* rope_cos,
                             const float* rope_sin, const int* rope_pos, hipStream_t stream) {
  if (S % 256 != 0 || H % KV != 0 || (D != 128 && D != 64)) return -1;
  if (rope_cos && (D != 128 || !rope_sin || ((reinterpret_cast<uintptr_t>(rope_cos) |
                                               reinterpret_cast<uintptr_t>(rope_sin)) & 15)))
    return -1;
  if (kv_valid <= 0 || kv_valid > S) kv_valid = S;
  // the dK/dV kernel addresses one batch's Q / dO rows and the workspace with 32-bit buffer offsets
  const long long max_rs = q_rs > do_rs ? (q_rs > kv_rs ? q_rs : kv_rs) : (do_rs > kv_rs ? do_rs : kv_rs);
  if ((long long)S * max_rs * 2 >= (1LL << 31) || 2LL * B * H * S * 4 >= (1LL << 31)) return -1;
  BwdArgs a{(const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const uint16_t*)o, (const uint16_t*)dout,
            lse, (float*)workspace, (uint16_t*)dq, (uint16_t*)dk, (uint16_t*)dv, q_rs, kv_rs, o_rs, dq_rs, dkv_rs, do_rs,
            B, S, H, KV, scale, scale * LOG2E, causal, window, doc_start, doc_end, kv_valid,
            rope_cos, rope_sin, rope_pos};
  const int g_kv = B * KV * (S / 256);
  const int g_q = B * H * (S / 128);
  // dQ first: it forms delta for its rows and writes the workspace row constants the dK/dV kernel reads
  // (the separate delta pass is gone: -41 us per layer, profiles/r5/attn_ab2/).  dQ at 2 waves per SIMD (one wave per SIMD, 512 registers: +0.2 ms at
  // the Llama-3-8B layer shape, profiles/r4/attn_final/); D = 64 dK/dV takes two 32-row query blocks per slice
  if (D == 128) {
    hipLaunchKernelGGL((bwd_dq_kernel<128, 2>), dim3(g_q), dim3(256), 0, stream, a);
    hipLaunchKernelGGL((bwd_dkdv8_kernel<128, 1>), dim3(g_kv), dim3(512), 0, stream, a);
  } else {
    hipLaunchKernelGGL((bwd_dq_kernel<64, 2>), dim3(g_q), dim3(256), 0, stream, a);
    hipLaunchKernelGGL((bwd_dkdv8_kernel<64, 2>), dim3(g_kv), dim3(512), 0, stream, a);
  }
  return (int)hipGetLastError();
}
