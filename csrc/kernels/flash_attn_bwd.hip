// K2: flash-attention backward for gfx950 (causal / sliding window, GQA, bf16, recompute P from LSE).
//
// Three launches, no float atomics anywhere (bitwise reproducible):
//   1. delta[b,h,q] = sum_d dO*O                                   (streaming, one wave per row)
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
//   3. dQ: one workgroup = 128 query rows of one (batch, q head); K/V tiles stream through LDS like the
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

// Diagnostic build only (tools/stamp_dkdv.hip defines FTC_STAMPS; the extension never does): per-wave
// cycle sums of the dK/dV loop's segments for one workgroup, read through g_stamps (guide "In-kernel
// stamps": shares, not lengths -- the stamps' waits forbid some overlap).
#ifdef FTC_STAMPS
__device__ unsigned long long g_stamps[8][6];  // [wave][sync, A, B1, B2, loop total, slices]
__device__ int g_stamp_block;
#define FTC_STAMP(t)                                                                          \
  do {                                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");                 \
    __builtin_amdgcn_sched_barrier(0);                                                        \
  } while (0)
#endif

FTC_DEV int swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
template <int D>
FTC_DEV int lds_off(int r, int chunk) {
  constexpr int NCH = D / 8;
  return r * (D * 2) + 16 * ((chunk ^ swz(r)) & (NCH - 1));
}
FTC_DEV bf16x8 as_bf8(const uint4& v) { return __builtin_bit_cast(bf16x8, v); }
FTC_DEV bf16x8 pack8_bf(const f32x16& p, int base) {
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
FTC_DEV void store_rows(uint16_t* p, const f32x16* acc, float sc, int hh, bool wide) {
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
FTC_DEV int2 tr_offsets(int colbase, int lane) {
  const int hh = lane >> 5, gi = (lane >> 4) & 3, li = lane & 15;
  const int trq = li >> 2, trp = li & 3;
  const int col = colbase + 16 * (gi & 1) + 4 * trp;
  const int chunk = col >> 3, half8 = (col & 7) ? 8 : 0;
  const int r1 = 4 * hh + trq;
  return make_int2(lds_off<D>(r1, chunk) + half8, lds_off<D>(r1 + 8, chunk) + half8);
}
template <int D>
FTC_DEV bf16x8 tr_read(const char* img, int kb, int2 off) {
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
FTC_DEV void rope_inv_rows(f32x16* acc, const BwdArgs& a, long long token, int hh) {
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

// ---------------------------------------------------------------- 1. delta
template <int D>
__global__ __launch_bounds__(256) void bwd_delta_kernel(BwdArgs a) {
  constexpr int CPH = D / 8;  // 16-byte chunks per head
  const int lane = threadIdx.x & 63;
  const long long rows = (long long)a.B * a.S;
  const int nch = a.H * CPH;
  for (long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6); row < rows; row += (long long)gridDim.x * 4) {
    const uint16_t* orow = a.o + row * a.o_rs;
    const uint16_t* drow = a.dout + row * a.do_rs;
    const int b = (int)(row / a.S), s = (int)(row % a.S);
    for (int c0 = 0; c0 < nch; c0 += 64) {
      const int c = c0 + lane;
      float acc = 0.f;
      if (c < nch) {
        float x[8], y[8];
        unpack8(reinterpret_cast<const uint4*>(orow)[c], x);
        unpack8(reinterpret_cast<const uint4*>(drow)[c], y);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += x[j] * y[j];
      }
#pragma unroll
      for (int off = CPH / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
      if (c < nch && (c % CPH) == 0) {
        const int h = c / CPH;
        // workspace rows: [-delta | -lse/scale] -- the dK/dV kernel's accumulator start values, DMA'd as is
        const long long ri = ((long long)b * a.H + h) * a.S + s;
        a.delta[ri] = -acc;
        a.delta[rows * a.H + ri] = -a.lse[ri] / a.scale;
      }
    }
  }
}

// ---------------------------------------------------------------- 2. dK / dV
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
FTC_DEV void lds_dma4(__amdgpu_buffer_rsrc_t r, const void* lds, int voff, int soff) {
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
FTC_DEV void dkdv_dma(__amdgpu_buffer_rsrc_t qr, __amdgpu_buffer_rsrc_t dr, __amdgpu_buffer_rsrc_t cr, const int* qvo,
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

// HW = 32-key halves per wave: HW = 2 -> 4 waves x 64 keys, one wave per SIMD (512-register budget);
// HW = 1 -> 8 waves x 32 keys, two waves per SIMD (256 registers each): one wave's softmax VALU then
// runs under the other wave's MFMAs.
// PP (8 waves only): "ping-pong" -- the two waves sharing a SIMD (w, w + 4) run each query slice's
// two phases in opposite order between the same pair of barriers: half 0 does A(j) then B(j), half 1
// does B(j - 1) then A(j), where A = the S / dP' MFMA chains and B = softmax / masking VALU + the
// dV / dK MFMAs.  One wave's exp / mask / pack work then issues under its partner's MFMAs instead of
// both waves idling the matrix pipe at the same time (guide: MI355X_MICROARCH.md "Two waves per
// SIMD").  Slice j is read by half 1 one barrier interval later, so the Q/dO ring has 4 slots.
// QR = 32-row query blocks per slice: QR = 2 (D = 64) doubles the MFMA work between two barriers,
// which at D = 64 is otherwise half of D = 128's (the per-slice barrier / DMA cost stays the same).
// (Measured and removed, git history / profiles/r2/stamp_dkdv.md: a B1 B2 A order for half 1 carrying the
// raw S / dP' across the barrier -- bwd 2.03 vs 1.96 ms: the MFMA phases wait on the 8 waves' LDS reads,
// not on the partner's VALU.)
template <int D, int HW, bool PP = false, int DIST = 2, int QR = 1>
__global__ __launch_bounds__(64 * (8 / HW), 1) void bwd_dkdv_kernel(BwdArgs a) {
  static_assert(DIST == 2 || (PP && DIST == 3), "DMA distance 3 needs the ping-pong 5-slot ring");
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
  __shared__ __attribute__((aligned(16))) char slot3[PP ? SLICE : 16];
  __shared__ __attribute__((aligned(16))) char slot4[DIST == 3 ? SLICE : 16];

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
  // 3-slot ring, two slices ahead of the compute; one raw barrier per slice with a COUNTED vmcnt so the
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
  if (DIST == 3 && total > 2) issue(2, slot2);
  // slice it computes from slot it % 3 and DMAs slice it + 2 into slot (it + 2) % 3, which held
  // slice it - 1 (finished by every wave before this slice's barrier)
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
    if (DIST == 3 && it + 2 < total) __builtin_amdgcn_s_waitcnt(VM_TWO);  // slices it+1, it+2 may fly on
    else if (it + 1 < total) __builtin_amdgcn_s_waitcnt(VM_ONE);       // slice it landed, it+1 may fly on
    else __builtin_amdgcn_s_waitcnt(VM_ZERO);
    __builtin_amdgcn_s_waitcnt(LGKM_ZERO);
    __builtin_amdgcn_s_barrier();  // every wave's pieces of slice it are in
    if (it + DIST < total) issue(it + DIST, dma_slot);
  };
  if constexpr (!PP) {
    // slice it computes from slot it % 3 and DMAs slice it + 2 into slot (it + 2) % 3, which held
    // slice it - 1 (finished by every wave before this slice's barrier)
    auto body = [&](const int it, const char* Qs, char* dma_slot) __attribute__((always_inline)) {
      sync_slice(it, dma_slot);
      phaseA(Qs);
      phaseB1(it);
      phaseB2(Qs);
    };
    for (int it = 0; it < total; it += 3) {
      body(it, slot0, slot2);
      if (it + 1 < total) body(it + 1, slot1, slot0);
      if (it + 2 < total) body(it + 2, slot2, slot1);
    }
  } else {
    // 4-slot ring: slice it in slot it % 4; the DMA of slice it + 2 reuses the slot of slice it - 2,
    // whose last reader (half 1's phase B2) finished before this slice's barrier.  Half 1 carries only
    // the packed P / dS operands (16 VGPRs) across the barrier: A2 ... [B2(it-1) A(it) B1(it)] ...
    // the halves run separate straight-line loops (one branch outside the loop, not one per slice:
    // the register allocator then sees two independent paths) with the same barrier count
    if constexpr (DIST == 3) {
#ifdef FTC_STAMPS
      const bool stamping = blockIdx.x == g_stamp_block;
      unsigned long long st_acc[4] = {0, 0, 0, 0}, st_prev = 0, st_now = 0, st_t0 = 0, st_t1 = 0;
#define SEG_START()            \
  do {                         \
    if (stamping) FTC_STAMP(st_prev); \
  } while (0)
#define SEG_END(i)                                                  \
  do {                                                              \
    if (stamping) {                                                 \
      FTC_STAMP(st_now);                                            \
      st_acc[i] += st_now - st_prev;                                \
      st_prev = st_now;                                             \
    }                                                               \
  } while (0)
      if (stamping) FTC_STAMP(st_t0);
#else
#define SEG_START() \
  do {              \
  } while (0)
#define SEG_END(i) \
  do {             \
  } while (0)
#endif
      // 5-slot ring, DMA three slices ahead: slice it + 3 reuses the slot of slice it - 2
      if (wave < 4) {
        auto body = [&](const int it, const char* Qs, char* dma_slot) __attribute__((always_inline)) {
          SEG_START();
          sync_slice(it, dma_slot);
          SEG_END(0);
          phaseA(Qs);
          SEG_END(1);
          phaseB1(it);
          SEG_END(2);
          phaseB2(Qs);
          SEG_END(3);
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
          SEG_START();
          sync_slice(it, dma_slot);
          SEG_END(0);
          if (it > 0) phaseB2(Qprev);
          SEG_END(3);
          phaseA(Qs);
          SEG_END(1);
          phaseB1(it);
          SEG_END(2);
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
#ifdef FTC_STAMPS
      if (stamping) {
        FTC_STAMP(st_t1);
        if (lane == 0) {
#pragma unroll
          for (int i = 0; i < 4; ++i) g_stamps[wave][i] = st_acc[i];
          g_stamps[wave][4] = st_t1 - st_t0;
          g_stamps[wave][5] = (unsigned long long)total;
        }
      }
#endif
#undef SEG_START
#undef SEG_END
    } else if (wave < 4) {  // waves w and w + 4 share a SIMD
      auto body = [&](const int it, const char* Qs, char* dma_slot) __attribute__((always_inline)) {
        sync_slice(it, dma_slot);
        phaseA(Qs);
        phaseB1(it);
        phaseB2(Qs);
      };
      for (int it = 0; it < total; it += 4) {
        body(it, slot0, slot2);
        if (it + 1 < total) body(it + 1, slot1, slot3);
        if (it + 2 < total) body(it + 2, slot2, slot0);
        if (it + 3 < total) body(it + 3, slot3, slot1);
      }
    } else {
      auto body = [&](const int it, const char* Qs, const char* Qprev, char* dma_slot) __attribute__((always_inline)) {
        sync_slice(it, dma_slot);
        if (it > 0) phaseB2(Qprev);
        phaseA(Qs);
        phaseB1(it);
      };
      for (int it = 0; it < total; it += 4) {
        body(it, slot0, slot3, slot2);
        if (it + 1 < total) body(it + 1, slot1, slot0, slot3);
        if (it + 2 < total) body(it + 2, slot2, slot1, slot0);
        if (it + 3 < total) body(it + 3, slot3, slot2, slot1);
      }
      if (total > 0) {
        const int last = total - 1;
        phaseB2((last & 3) == 0 ? slot0 : (last & 3) == 1 ? slot1 : (last & 3) == 2 ? slot2 : slot3);
      }
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

// ---- IL (round 4): 4 waves x 64 keys, one wave per SIMD, fenced in-wave interleave --------------------
// profiles/r2/stamp_dkdv.md: the 8-wave kernel spends ~4,070 cycles per 32-row slice on 2,048 cycles of
// MFMA work per SIMD because its 8 waves each re-read the slice's Q / dO from LDS (~1,280 LDS-array
// cycles per slice interval at 256 B/clk).  Here each wave owns 64 keys as two 32-key halves, so every
// Q / dO fragment it reads feeds both halves (half the LDS bytes per MFMA), and the softmax VALU that
// the second wave of a SIMD used to hide is interleaved by hand with the wave's OWN MFMAs
// (sched_barrier fences; values pinned so the compiler cannot sink them past the fences):
//
//   sync(it)  A(it): S, dP' of both halves (32 MFMAs, next k-step's reads between them;
//                    the row constants -lse/scale, -delta are the first MFMA's C operand, with -inf
//                    at masked positions on diagonal / window / document slices)
//   X:  dV, dK += B2(it - 1, half 1)  (16 MFMAs)  x  P, dS of (it, half 0)   (exp / mul / pack)
//   Y:  dV, dK += B2(it,     half 0)  (16 MFMAs)  x  P, dS of (it, half 1)   (carried to slice it + 1)
//
// The transposed dO^T / Q^T reads of each d tile go out one d tile ahead.  Slice it - 1 is still read in
// X of slice it, so the Q / dO ring has 4 slots (DMA two slices ahead into the slot of slice it - 2).
// The DMA is inline asm (common.h lds_dma16) and counted with explicit vmcnt waits.  Slice 0's X runs
// its 16 MFMAs on zero P / dS carried from "slice -1" (exact: K rows x 0 adds 0).

#ifndef IL_TV2
#define IL_TV2 1
#endif
// timing-only ablations of the stamp build (tools/stamp_dkdv.hip -DIL_DIAG=N; wrong results): 1 no softmax
// VALU in X / Y, 2 no transposed reads in X / Y, 3 no fragment reads in A, 4 = 3 + no row-constant loads /
// masks, 5 = 4 + no A MFMAs, 6 = 3 + no masks, 7 = 3 + no row-constant loads
#if defined(FTC_STAMPS) && defined(IL_DIAG)
constexpr int kIlDiag = IL_DIAG;
#else
constexpr int kIlDiag = 0;
#endif
#ifndef IL_PIPE
#define IL_PIPE 1
#endif
template <int D>
__global__ __launch_bounds__(256, 1) void bwd_dkdv_il_kernel(BwdArgs a) {
  static_assert(D == 128, "IL dK/dV: head_dim 128");
  constexpr int NCH = D / 8, DSTEPS = D / 16, DT = D / 32;
  constexpr int BKV = 256, BQ2 = 32, WAVES = 4;
  constexpr int KBYTES = BKV * D * 2, QBYTES = BQ2 * D * 2;
  constexpr int SLICE = 2 * QBYTES + 2 * BQ2 * 4;  // Q | dO | -lse/scale | -delta
  constexpr int NG = QBYTES / 1024 / WAVES;         // 1 KiB pieces per matrix per wave per slice
  constexpr int RPG = 1024 / (D * 2);
  constexpr int PER_SLICE = 2 * NG + 1;             // DMA instructions per wave per slice
  __shared__ __attribute__((aligned(16))) char Ks[KBYTES];
  __shared__ __attribute__((aligned(16))) char ring[4 * SLICE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5, lr = lane & 31;
  const int S = a.S, G = a.H / a.KV;
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
  const int wkey0 = kv0 + wave * 64;

  const uint16_t* kbase = a.k + ((long long)b * S) * a.kv_rs + (long long)kvh * D;
  {
    constexpr int RPP = 256 / NCH;
    const int lrow = tid / NCH, lch = tid % NCH;
    const auto krs = make_rsrc(kbase + (long long)kv0 * a.kv_rs);
    const int voff = (lrow * (int)a.kv_rs + lch * 8) * 2;
#pragma unroll
    for (int p = 0; p < BKV / RPP; ++p)
      *reinterpret_cast<u32x4*>(Ks + lds_off<D>(p * RPP + lrow, lch)) = buf_load16(krs, voff, p * RPP * (int)a.kv_rs * 2);
  }
  bf16x8 vf[2][DSTEPS];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const uint16_t* vp = a.v + ((long long)b * S + wkey0 + 32 * j + lr) * a.kv_rs + (long long)kvh * D + 8 * hh;
#pragma unroll
    for (int st = 0; st < DSTEPS; ++st) vf[j][st] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(vp + 16 * st));
  }

  int qbeg = a.causal ? kv0 : 0;
  int qend = S;
  if (a.window > 0) qend = min(S, kv0 + BKV - 1 + a.window);
  int dmin[2] = {0x3fffffff, 0x3fffffff};
  // the lane's own keys' document ends, loaded once: a global load inside the loop's mask branch made
  // the compiler drain every in-flight DMA (vmcnt(0)) at the branch join on every slice
  int dend[2] = {0x40000000, 0x40000000};
  const int* de_row = a.doc_end ? a.doc_end + (long long)b * S : nullptr;
  if (de_row) {
    qend = min(qend, de_row[kv0 + BKV - 1]);
    dmin[0] = de_row[wkey0];
    dmin[1] = de_row[wkey0 + 32];
    dend[0] = de_row[wkey0 + lr];
    dend[1] = de_row[wkey0 + 32 + lr];
  }
  qbeg = (qbeg / BQ2) * BQ2;
  const int nqt = (qend - qbeg + BQ2 - 1) / BQ2;
  const int total = G * nqt;

  const auto qrsrc = make_rsrc(a.q + (long long)b * S * a.q_rs);
  const auto drsrc = make_rsrc(a.dout + (long long)b * S * a.do_rs);
  const auto crsrc = make_rsrc(a.delta);
  int qvo[NG], dvo[NG];
#pragma unroll
  for (int i = 0; i < NG; ++i) {
    const int row = (wave * NG + i) * RPG + lane / NCH, pc = lane % NCH;
    const int lc = (pc ^ swz(row)) & (NCH - 1);
    qvo[i] = (row * (int)a.q_rs + lc * 8) * 2;
    dvo[i] = (row * (int)a.do_rs + lc * 8) * 2;
  }
  const int cvo = (lr + (hh ? 0 : a.B * a.H * S)) * 4;  // lanes 0-31: -lse/scale rows, 32-63: -delta rows
  auto slot = [&](int it_) __attribute__((always_inline)) -> char* { return ring + (it_ & 3) * SLICE; };
  // slices in order it = g nqt + i (query head g of the group, 32-row block i): the DMA cursor walks them
  // with counters (no integer division per slice)
  int dg = 0, di = 0;
  auto issue = [&](int it_) __attribute__((always_inline)) {
    const int qt_ = qbeg + di * BQ2;
    const int hq_ = kvh * G + dg;
    if (++di == nqt) {
      di = 0;
      ++dg;
    }
    char* base = slot(it_);
    const int qso = (hq_ * D + qt_ * (int)a.q_rs) * 2, dso = (hq_ * D + qt_ * (int)a.do_rs) * 2;
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      const int r0 = (wave * NG + i) * RPG;
      lds_dma16(qrsrc, base + r0 * D * 2, qvo[i], qso);
      lds_dma16(drsrc, base + QBYTES + r0 * D * 2, dvo[i], dso);
    }
    lds_dma4(crsrc, base + 2 * QBYTES, cvo, ((b * a.H + hq_) * S + qt_) * 4);
  };
  constexpr int VM_ONE = 0x0F70 | (PER_SLICE & 15) | ((PER_SLICE >> 4) << 14);  // vmcnt(PER_SLICE)

  f32x16 dv[2][DT], dk[2][DT];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) { dv[j][t][i] = 0.f; dk[j][t][i] = 0.f; }

  __builtin_amdgcn_s_waitcnt(0x0F70);  // K staging, V fragments, doc bounds retired (vmcnt(0))
  __syncthreads();
  if (total > 0) issue(0);
  if (total > 1) issue(1);

  auto fence = []() __attribute__((always_inline)) { __builtin_amdgcn_sched_barrier(0); };
  const int2 to[DT] = {tr_offsets<D>(0, lane), tr_offsets<D>(32, lane), tr_offsets<D>(64, lane), tr_offsets<D>(96, lane)};
  f32x16 s[2], dp[2];
  bf16x8 pb0[2], sb0[2];  // P / dS of half 0 of the current slice
  bf16x8 pbc[2], sbc[2];  // P / dS of half 1, carried into the next slice's X
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    pbc[k] = __builtin_bit_cast(bf16x8, make_uint4(0, 0, 0, 0));
    sbc[k] = pbc[k];
  }
  // B1 of half j, software-pipelined over the 16 MFMA gaps of a region so no VALU waits on a fresh
  // exponential: gap g computes P_g = exp2(c S_g) and dS_(g-1) = P_(g-1) dP'_(g-1); P's first 8 elements
  // pack in gap 8, dS's in gap 9; the tail (dS_15, the second packs) follows the region's last MFMA
  auto b1_gap = [&](int j, int g, bf16x8* pbo, bf16x8* sbo) __attribute__((always_inline)) {
    if (kIlDiag == 1) return;
    if (!IL_PIPE) {  // unpipelined: P and dS of element g in gap g, packs after elements 7 / 15
      if (g < 16) {
        const float p = __builtin_amdgcn_exp2f(a.c * s[j][g]);
        const float d = p * dp[j][g];
        asm volatile("" ::"v"(p), "v"(d));
        s[j][g] = p;
        dp[j][g] = d;
        if ((g & 7) == 7) {
          pbo[g >> 3] = pack8_bf(s[j], g & 8);
          sbo[g >> 3] = pack8_bf(dp[j], g & 8);
        }
      }
      return;
    }
    if (g < 16) {
      const float p = __builtin_amdgcn_exp2f(a.c * s[j][g]);
      asm volatile("" ::"v"(p));  // pin: pure arithmetic would otherwise sink past the fences
      s[j][g] = p;
    }
    if (g >= 1) {
      const float d = s[j][g - 1] * dp[j][g - 1];
      asm volatile("" ::"v"(d));
      dp[j][g - 1] = d;
    }
    if (g == 8) pbo[0] = pack8_bf(s[j], 0);
    if (g == 9) sbo[0] = pack8_bf(dp[j], 0);
    if (g == 16) {
      pbo[1] = pack8_bf(s[j], 8);
      sbo[1] = pack8_bf(dp[j], 8);
    }
  };
  // the four transposed operands of a d tile (dO^T rows 0-15 / 16-31, Q^T rows 0-15 / 16-31), two register
  // sets by d-tile parity: d tile dt + 1 is read during the first two MFMAs of d tile dt (>= 6 MFMAs of
  // latency cover)
  bf16x8 tv[2][4];
  constexpr int TVM = IL_TV2 ? 1 : 0;
  auto tr_op = [&](const char* Qs, int dt, int m) __attribute__((always_inline)) {
    if (kIlDiag == 2) return;
    tv[dt & TVM][m] = tr_read<D>((m < 2 ? Qs + QBYTES : Qs), 16 * (m & 1), to[dt]);
  };
  // B2 of half j on d tile dt, MFMA m (0..3) of its four.  The dV / dK accumulators (256 registers) are
  // pinned to the AGPR half by inline asm ("+a"): left to itself the compiler spreads them and the S / dP'
  // chains over both halves and pays ~220 v_accvgpr moves per slice to feed the softmax VALU.  Wait
  // states (guide §5.7 item 2): an MFMA's D feeding the next MFMA's C is 0 states; the operands are LDS
  // reads (lgkmcnt-waited by the compiler) or packs made at least one MFMA earlier, covered by the
  // s_nop 1; the epilogue's readers follow a padding statement after the loop.
  auto b2_mfma = [&](int j, int dt, int m, const bf16x8* pbs, const bf16x8* sbs) __attribute__((always_inline)) {
    if (m < 2)
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(dv[j][dt]) : "v"(tv[dt & TVM][m]), "v"(pbs[m]));
    else
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(dk[j][dt]) : "v"(tv[dt & TVM][m]), "v"(sbs[m - 2]));
  };
  // X / Y region: B2 of half j from slice image Qs (pbs / sbs) with B1 of half jv of the current slice
  // (into pbo / sbo), one gap per MFMA; the next d tile's operands (d tile 0 of Qnext after the last)
  // are read in the first two gaps of each d tile.  Operands of d tile 0 are read by the caller.
  auto region = [&](int j, const char* Qs, const bf16x8* pbs, const bf16x8* sbs, int jv, bf16x8* pbo, bf16x8* sbo,
                    const char* Qnext) __attribute__((always_inline)) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        b2_mfma(j, dt, m, pbs, sbs);
        fence();
        b1_gap(jv, dt * 4 + m, pbo, sbo);
        const char* src = dt + 1 < DT ? Qs : Qnext;
        if (IL_TV2 && m < 2 && src) {
          tr_op(src, (dt + 1) & 3, 2 * m);
          tr_op(src, (dt + 1) & 3, 2 * m + 1);
        }
        if (!IL_TV2 && src) tr_op(src, (dt + 1) & 3, m);
        fence();
      }
    b1_gap(jv, 16, pbo, sbo);
    fence();
  };

#ifdef FTC_STAMPS  // diagnostic build (tools/stamp_dkdv.hip with FTC_FLASH_DKDV_WAVES=il): segments sync / A / X / Y
  const bool stamping = blockIdx.x == g_stamp_block;
  unsigned long long st_acc[4] = {0, 0, 0, 0}, st_prev = 0, st_now = 0, st_t0 = 0, st_t1 = 0;
  if (stamping) FTC_STAMP(st_t0);
#define IL_SEG_START()              \
  do {                              \
    if (stamping) FTC_STAMP(st_prev); \
  } while (0)
#define IL_SEG_END(i)                \
  do {                               \
    if (stamping) {                  \
      FTC_STAMP(st_now);             \
      st_acc[i] += st_now - st_prev; \
      st_prev = st_now;              \
    }                                \
  } while (0)
#else
#define IL_SEG_START() \
  do {                 \
  } while (0)
#define IL_SEG_END(i) \
  do {                \
  } while (0)
#endif
  int ci = 0;  // 32-row block of the current slice
  for (int it = 0; it < total; ++it) {
    IL_SEG_START();
    // ---- sync: slice it landed (it + 1 may fly), every wave is past slice it - 1's Y; DMA it + 2
    if (it + 1 < total) __builtin_amdgcn_s_waitcnt(VM_ONE);
    else __builtin_amdgcn_s_waitcnt(0x0F70);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    if (it + 2 < total) issue(it + 2);
    fence();
    IL_SEG_END(0);
    const char* Qs = slot(it);
    const char* Ds = Qs + QBYTES;
    const char* Qprev = it > 0 ? slot(it - 1) : Ks;  // slice -1: K rows x zero P / dS
    // ---- A: S = Q K^T - lse/scale, dP' = dO V^T - delta for both halves
    {
      // the chains start from the row constants (-lse/scale for S, -delta for dP'), read from the slice's
      // LDS image straight into the accumulators (one copy per half: no separate start tile whose
      // registers an in-flight MFMA would still be reading as C); masks (diagonal / window / document
      // slices, wave-uniform branches) put -inf into S's start values, so P = exp2(c S) = 0 and dS = 0
      const float* cst = reinterpret_cast<const float*>(Qs + 2 * QBYTES);
      // a second, opaque copy of the address: the S / dP' chains of both halves get their own LDS reads
      // of the row constants (4 ds_read each) instead of one read + 32 v_mov copies
      typedef __attribute__((address_space(3))) const float lds_f32;
      unsigned cst_off = (unsigned)(uintptr_t)(lds_f32*)cst;  // (an opaque generic pointer would turn into
      asm volatile("" : "+v"(cst_off));                      //  flat loads, counted by vmcnt: DMA drain)
      lds_f32* cst_b = (lds_f32*)(uintptr_t)cst_off;
      auto ld_const = [&](f32x16& t, auto src) __attribute__((always_inline)) {
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
#pragma unroll
          for (int e = 0; e < 4; ++e) t[4 * g4 + e] = src[8 * g4 + 4 * hh + e];
        }
      };
      if (kIlDiag < 4 || kIlDiag == 6) {
        ld_const(s[0], (lds_f32*)cst);
        ld_const(dp[0], (lds_f32*)cst + BQ2);
        ld_const(s[1], cst_b);
        ld_const(dp[1], cst_b + BQ2);
      }
      if (kIlDiag < 4 || kIlDiag == 7) {
        const int qt = qbeg + ci * BQ2;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int kmin = wkey0 + 32 * j;
          const bool need_mask = (a.causal && qt < kmin + 31) || (a.window > 0 && qt + 31 - kmin >= a.window) ||
                                 qt + 31 >= dmin[j];
          if (need_mask) {
            const int key = kmin + lr;
            const int base = qt + 4 * hh;
            const int lo = (a.causal ? key : -0x3fffffff) - base;
            const int hi = min(a.window > 0 ? key + a.window - 1 : 0x3fffffff, dend[j] - 1) - base;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int off = (i & 3) + 8 * (i >> 2);
              s[j][i] = (off >= lo && off <= hi) ? s[j][i] : -INFINITY;
            }
          }
        }
      }
      // k-step fragments [qa, da, k0, k1], double-buffered: k-step st + 1 is read under k-step st's MFMAs
      u32x4 fr[2][4];
      auto rd = [&](int st) __attribute__((always_inline)) {
        if (kIlDiag >= 3 && st > 0) return;  // (6, 7: as 3)
        fr[st & 1][0] = *reinterpret_cast<const u32x4*>(Qs + lds_off<D>(lr, 2 * st + hh));
        fr[st & 1][1] = *reinterpret_cast<const u32x4*>(Ds + lds_off<D>(lr, 2 * st + hh));
        fr[st & 1][2] = *reinterpret_cast<const u32x4*>(Ks + lds_off<D>(wave * 64 + lr, 2 * st + hh));
        fr[st & 1][3] = *reinterpret_cast<const u32x4*>(Ks + lds_off<D>(wave * 64 + 32 + lr, 2 * st + hh));
      };
      rd(0);
      fence();
#pragma unroll
      for (int st = 0; st < DSTEPS; ++st) {
        const bool more = st + 1 < DSTEPS;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const u32x4* f = fr[st & 1];
          const bf16x8 qa = __builtin_bit_cast(bf16x8, f[0]), da = __builtin_bit_cast(bf16x8, f[1]);
          const bf16x8 bop = m == 0 ? __builtin_bit_cast(bf16x8, f[2]) : m == 1 ? __builtin_bit_cast(bf16x8, f[3]) : vf[m - 2][st];
          f32x16& acc = m == 0 ? s[0] : m == 1 ? s[1] : m == 2 ? dp[0] : dp[1];
          // (s_nop 1 at k-step 0: the start values may come from the mask's VALU selects)
          if (kIlDiag == 5)
            asm volatile("" : "+v"(acc) : "v"(m < 2 ? qa : da), "v"(bop));
          else if (st == 0)
            asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(m < 2 ? qa : da), "v"(bop));
          else
            asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(m < 2 ? qa : da), "v"(bop));
          fence();
          if (more && m == 0) rd(st + 1);
          if (st == DSTEPS - 1 && m < 2) {  // X's first d tile
            tr_op(Qprev, 0, 2 * m);
            tr_op(Qprev, 0, 2 * m + 1);
          }
          fence();
        }
      }
    }
    // the S / dP' results (8-pass XDL, asm: not padded by the compiler) before the first VALU reader
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    fence();
    IL_SEG_END(1);
    // ---- X: B2(it - 1, half 1) x B1(it, half 0);  Y: B2(it, half 0) x B1(it, half 1)
    region(1, Qprev, pbc, sbc, 0, pb0, sb0, Qs);
    IL_SEG_END(2);
    region(0, Qs, pb0, sb0, 1, pbc, sbc, nullptr);
    IL_SEG_END(3);
    if (++ci == nqt) ci = 0;
  }
#ifdef FTC_STAMPS
  if (stamping) {
    FTC_STAMP(st_t1);
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) g_stamps[wave][i] = st_acc[i];
      g_stamps[wave][4] = st_t1 - st_t0;
      g_stamps[wave][5] = (unsigned long long)total;
    }
  }
#endif
#undef IL_SEG_START
#undef IL_SEG_END
  // ---- the last slice's half 1
  if (total > 0) {
    const char* Ql = slot(total - 1);
#pragma unroll
    for (int m = 0; m < 4; ++m) tr_op(Ql, 0, m);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      if (dt + 1 < DT)
#pragma unroll
        for (int m = 0; m < 4; ++m) tr_op(Ql, dt + 1, m);
#pragma unroll
      for (int m = 0; m < 4; ++m) b2_mfma(1, dt, m, pbc, sbc);
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // no DMA outlives the workgroup
  asm volatile("s_nop 15" ::: "memory");  // the last asm MFMAs' results before any reader (16-pass XDL)

#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int key = wkey0 + 32 * j + lr;
    uint16_t* dkp = a.dk + ((long long)b * S + key) * a.dkv_rs + (long long)kvh * D;
    uint16_t* dvp = a.dv + ((long long)b * S + key) * a.dkv_rs + (long long)kvh * D;
    const bool wide = (a.dkv_rs & 7) == 0;
    if (a.rcos) rope_inv_rows<DT>(dk[j], a, (long long)b * S + key, hh);
    store_rows<DT>(dkp, dk[j], a.scale, hh, wide);
    store_rows<DT>(dvp, dv[j], 1.0f, hh, wide);
  }
}

// ---------------------------------------------------------------- 3. dQ
#ifndef DQ_CINIT
#define DQ_CINIT 1
#endif
// One K/V tile by LDS-DMA: NGT 1 KiB pieces per matrix per wave (device-only: see dkdv_dma)
template <int D, int NGT, int RPG>
FTC_DEV void kv_dma(__amdgpu_buffer_rsrc_t kr, __amdgpu_buffer_rsrc_t vr, const int* voff, int toff, char* kdst,
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
  const float lse2 = a.lse[sidx] * LOG2E;
  const float ndlt = a.delta[sidx];  // -delta

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


// dK/dV variant: 8 waves x 32 keys (2 waves/SIMD) with ping-pong and the 5-slot ring by default, or
// 4 waves x 64 keys (1 wave/SIMD)
template <int D>
void launch_dkdv(const BwdArgs& a, int grid, int waves, bool pp, bool dist3, hipStream_t stream) {
  // D = 64: 64-row query slices (FTC_FLASH_DKDV_QR=1 for 32)
  static const bool qr2 = [] {
    const char* e = getenv("FTC_FLASH_DKDV_QR");
    return !(e && e[0] == '1');
  }();
  if (D == 64 && qr2 && waves == 8 && pp && dist3)
    hipLaunchKernelGGL((bwd_dkdv_kernel<64, 1, true, 3, 2>), dim3(grid), dim3(512), 0, stream, a);
  else if (waves == 8 && pp && dist3)
    hipLaunchKernelGGL((bwd_dkdv_kernel<D, 1, true, 3>), dim3(grid), dim3(512), 0, stream, a);
  else if (waves == 8 && pp)
    hipLaunchKernelGGL((bwd_dkdv_kernel<D, 1, true>), dim3(grid), dim3(512), 0, stream, a);
  else if (waves == 8)
    hipLaunchKernelGGL((bwd_dkdv_kernel<D, 1>), dim3(grid), dim3(512), 0, stream, a);
  else if (D == 128 && waves == 1)
    hipLaunchKernelGGL((bwd_dkdv_il_kernel<128>), dim3(grid), dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL((bwd_dkdv_kernel<D, 2>), dim3(grid), dim3(256), 0, stream, a);
}

// dK/dV variant: 8 (8 waves x 32 keys, ping-pong), 4 (4 waves x 64 keys), 1 (IL: 4 waves x 64 keys,
// fenced interleave, D = 128); FTC_FLASH_DKDV_WAVES=8|4|il, or ftc_flash_dkdv_config (tests / tools)
int& dkdv_variant() {
  static int v = [] {
    const char* e = getenv("FTC_FLASH_DKDV_WAVES");
    return (e && e[0] == '4') ? 4 : (e && e[0] == 'i') ? 1 : 8;
  }();
  return v;
}

}  // namespace

extern "C" void ftc_flash_dkdv_config(int waves) { dkdv_variant() = (waves == 4 || waves == 1) ? waves : 8; }

extern "C" int ftc_flash_bwd_workspace(int B, int S, int H, int D, long long* bytes) {
  (void)D;
  *bytes = 2LL * B * H * S * sizeof(float);  // -delta, -lse/scale
  return 0;
}

// (Removed: dQ on a second stream beside dK/dV, FTC_FLASH_BWD_CONCURRENT -- 2.017 vs 2.016 ms,
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
  const int grid_d = ftc::oneshot_grid((long long)B * S, 4);
  const int g_kv = B * KV * (S / 256);
  const int g_q = B * H * (S / 128);
  // occupancy variant of the two main kernels: 2 waves/SIMD (256-VGPR budget, spills a few staging
  // registers at D=128) or 1 wave/SIMD (512 VGPR+AGPR, no spills); FTC_FLASH_BWD_OCC=1|2
  static const int occ = [] {
    const char* e = getenv("FTC_FLASH_BWD_OCC");
    return (e && e[0] == '1') ? 1 : 2;
  }();
  // dK/dV workgroup shape at D=128: 8 waves x 32 keys (2 waves/SIMD, default: 1.20 vs 1.52 ms at the
  // Llama-3-8B layer shape, profiles/) or 4 waves x 64 keys (1 wave/SIMD); FTC_FLASH_DKDV_WAVES=8|4
  // FTC_FLASH_DKDV_WAVES=il: the round-4 interleaved 4-wave kernel (bwd_dkdv_il_kernel, D = 128)
  const int dkdv_waves = dkdv_variant();
  // ping-pong phase order for the two waves of a SIMD (default; FTC_FLASH_DKDV_PP=0 turns it off):
  // bwd 2.00 -> 1.97 ms at the Llama-3-8B layer shape (profiles/r1_attn_dkdv_pp.log)
  static const bool pp = [] {
    const char* e = getenv("FTC_FLASH_DKDV_PP");
    return !(e && e[0] == '0');
  }();
  // Q/dO slices DMA'd three slices ahead (5-slot ring; default, FTC_FLASH_DKDV_DIST=2 for two):
  // bwd 1.99 -> 1.96 ms at the Llama-3-8B layer shape (profiles/r1_attn_dkdv_pp.log)
  static const bool dist3 = [] {
    const char* e = getenv("FTC_FLASH_DKDV_DIST");
    return !(e && e[0] == '2');
  }();
  hipStream_t qs = stream;
  if (D == 128) {
    hipLaunchKernelGGL(bwd_delta_kernel<128>, dim3(grid_d), dim3(256), 0, stream, a);
  } else {
    hipLaunchKernelGGL(bwd_delta_kernel<64>, dim3(grid_d), dim3(256), 0, stream, a);
  }
  if (D == 128) {
    launch_dkdv<128>(a, g_kv, dkdv_waves, pp, dist3, stream);
    if (occ == 1) {
      hipLaunchKernelGGL((bwd_dq_kernel<128, 1>), dim3(g_q), dim3(256), 0, qs, a);
    } else {
      hipLaunchKernelGGL((bwd_dq_kernel<128, 2>), dim3(g_q), dim3(256), 0, qs, a);
    }
  } else {
    launch_dkdv<64>(a, g_kv, dkdv_waves, pp, dist3, stream);
    hipLaunchKernelGGL((bwd_dq_kernel<64, 2>), dim3(g_q), dim3(256), 0, qs, a);
  }
  return (int)hipGetLastError();
}
