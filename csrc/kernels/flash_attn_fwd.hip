// K1: flash-attention forward for gfx950 -- causal / sliding-window, GQA, bf16 in/out, fp32 LSE.
//
// Geometry: one 256-thread workgroup (4 waves) = 128 query rows of one (batch, q-head); each wave
// owns 32 rows.  K/V stream through LDS in 64-key tiles, double buffered; the next tile arrives by
// LDS-DMA (buffer_load ... lds, pre-swizzled sources) issued right after the current tile's barrier,
// so it flies under the whole tile's compute with no staging registers and no ds_write pass.
//
// MFMA orientation (v_mfma_f32_32x32x16_bf16, wave64):
//   S^T[key][q] = K . Q^T      A = K rows from LDS (ds_read_b128), B = Q^T kept in registers.
//                             The accumulator has the query on the lane and 16 keys per lane half
//                             in registers, so softmax row statistics are lane-local (+1 xor-32
//                             exchange) -- no LDS traffic for softmax.
//   O^T[d][q]  += V^T . P^T    B = P^T straight from the S^T accumulator (bf16-packed): the
//                             accumulator's permuted row order is used as the k order of this
//                             MFMA, and the V^T A-operand is read in that same order with
//                             ds_read_b64_tr_b16 (hardware transpose), two 4-key reads per step.
//                             O^T keeps the query on the lane, so the online-softmax rescale is a
//                             per-lane scalar multiply.
// LDS image (K and V, [64 keys][D] bf16, 256-byte rows for D=128): 16-byte chunk c of row r lives
// at chunk c ^ (((r&3)<<2) | ((r>>2)&3)) -- conflict-free for both the b128 row reads of K and the
// tr_b16 column reads of V (guide T10 "one image for row reads and transposed reads").
// Block order: heaviest causal q-blocks first; the G = H/KV query heads that share a kv head are
// placed on the same XCD (blockIdx % 8 group) so their K/V tiles are L2 hits.
#include "common.h"

#include <cstdlib>
#include <type_traits>

using namespace ftc;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// query rows per workgroup = 32 x 4 waves (256 threads, two workgroups per CU).  Measured and removed
// (git history, profiles/r1_attn_fwd_pp.log, profiles/r2/s9_attn_pipe*.log): 8 waves per workgroup
// (0.617 vs 0.604 ms), an 8-wave ping-pong phase order (0.64 ms) and an in-wave software pipeline across
// tiles (0.626 ms at 2 waves/SIMD, 0.85 at 1) at the Llama-3-8B layer shape.
constexpr int WAVES = 4;
constexpr int BK = 64;   // keys per tile
// build-time A/B knobs (tools/fwd_knobs_ab.sh): K-fragment reads issued ahead of the S MFMA chain, and a
// raised wave priority over the S MFMA phase
#ifndef FWD_KPRE
#define FWD_KPRE 4
#endif
#ifndef FWD_PRIO
#define FWD_PRIO 0
#endif
#ifndef FWD_EARLY_DMA  // tile 0's DMA issued before the Q loads (tools/fwd_knobs_ab.sh)
#define FWD_EARLY_DMA 0
#endif
#ifndef FWD_WIDE_STORE  // 16-byte O stores in the epilogue (tools/fwd_knobs_ab.sh)
#define FWD_WIDE_STORE 1
#endif
// packed-fp32 scale / row-sum in the online softmax (phase B1).  Measured slower (tools/pk_softmax_ab.sh,
// profiles/r3/pk_softmax/: forward 0.605 / 0.615 vs 0.589 / 0.578 ms, headline 35,376 / 35,429 vs
// 35,533 / 35,527 tok/s, one box) -> off
#ifndef FWD_PIN
#define FWD_PIN 0
#endif
#ifndef FWD_PK_SOFTMAX
#define FWD_PK_SOFTMAX 0
#endif
typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

DEV_INLINE int swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

template <int D>
DEV_INLINE int lds_off(int r, int chunk) {  // byte offset of 16-byte chunk `chunk` of row r
  constexpr int NCH = D / 8;
  return r * (D * 2) + 16 * ((chunk ^ swz(r)) & (NCH - 1));
}

DEV_INLINE bf16x8 as_bf8(const uint4& v) { return __builtin_bit_cast(bf16x8, v); }

// max over lanes l and l ^ 32: v_permlane32_swap (gfx950 VALU, one instruction) instead of
// ds_bpermute -- the row max sits on the softmax's dependency chain every tile, and the LDS permute's
// round trip was part of it.
DEV_INLINE float xhalf_max(float v) {
  const auto pr = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float a = __uint_as_float(pr[0]), b = __uint_as_float(pr[1]);
  return a > b ? a : b;  // lane l holds {v_l, v_(l^32)} in some order
}

DEV_INLINE bf16x8 pack_p(const f32x16& p, int base) {
  f32x4 lo = {p[base + 0], p[base + 1], p[base + 2], p[base + 3]};
  f32x4 hi = {p[base + 4], p[base + 5], p[base + 6], p[base + 7]};
  uint4 u;
  u.x = pack_bf2(lo[0], lo[1]);
  u.y = pack_bf2(lo[2], lo[3]);
  u.z = pack_bf2(hi[0], hi[1]);
  u.w = pack_bf2(hi[2], hi[3]);
  return as_bf8(u);
}

struct FwdArgs {
  const uint16_t* q;
  const uint16_t* k;
  const uint16_t* v;
  uint16_t* o;
  float* lse;
  long long q_rs, kv_rs, o_rs;
  int B, S, H, KV, nqb;
  float scale_log2;
  int causal, window;
  const int* doc_start;  // [B*S] first position of each token's document (packed sequences), or null
  int kv_valid;          // keys >= kv_valid are masked for every query (a right-padded tail; S: none)
};

// logical block -> (qb, b, kvh, g) with heavy-first order and GQA groups co-located on one XCD
DEV_INLINE void decode_block(const FwdArgs& a, int& qb, int& b, int& hq, int& kvh, const int bid_in = -1) {
  const int G = a.H / a.KV;
  const int bid = bid_in < 0 ? (int)blockIdx.x : bid_in;
  const int ngroups = a.nqb * a.B * a.KV;
  int j, g;
  if ((ngroups & 7) == 0) {
    const int xcd = bid & 7, slot = bid >> 3;
    g = slot % G;
    j = (slot / G) * 8 + xcd;
  } else {
    g = bid % G;
    j = bid / G;
  }
  kvh = j % a.KV;
  const int t = j / a.KV;
  b = t % a.B;
  const int qr = t / a.B;
  qb = a.nqb - 1 - qr;  // heaviest (latest) query blocks first
  hq = kvh * G + g;
}

// One tile's K and V by LDS-DMA (buffer_load ... lds): NGT 1 KiB pieces per matrix per wave, the
// lane's 16 bytes landing lane-linearly, the source pre-swizzled (voff) so the LDS image is the
// XOR-swizzled one; toff = the tile's first row (scalar).  A device-only function: the host pass of
// hipcc cannot instantiate these builtins inside a kernel lambda.
template <int D, int NGT, int RPG>
DEV_INLINE void fwd_dma(__amdgpu_buffer_rsrc_t kr, __amdgpu_buffer_rsrc_t vr, const int* voff, int toff, char* kdst,
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

template <int D>
__global__ __launch_bounds__(64 * WAVES, 8 / WAVES) void flash_fwd_kernel(FwdArgs a) {
  constexpr int BQ = 32 * WAVES;
  constexpr int NCH = D / 8;           // 16-byte chunks per row
  constexpr int DSTEPS = D / 16;       // k-steps of the S MFMA
  constexpr int DT = D / 32;           // 32-wide d tiles of O
  constexpr int TILE_BYTES = BK * D * 2;
  constexpr int NGT = TILE_BYTES / 1024 / WAVES;  // 1 KiB DMA pieces per wave per matrix
  constexpr int RPG = 1024 / (D * 2);             // rows per piece
  static_assert(NGT >= 1, "tile too small for the wave count");
  // K/V tiles double-buffered in four DISTINCT __shared__ objects: reading one does not make the
  // compiler drain the DMA still filling the other pair (LDS alias scopes)
  __shared__ __attribute__((aligned(16))) char K0[TILE_BYTES];
  __shared__ __attribute__((aligned(16))) char V0[TILE_BYTES];
  __shared__ __attribute__((aligned(16))) char K1[TILE_BYTES];
  __shared__ __attribute__((aligned(16))) char V1[TILE_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform -> scalar branches
  const int hh = lane >> 5, lr = lane & 31;
  int qb, b, hq, kvh;
  decode_block(a, qb, b, hq, kvh);
  const int S = a.S;
  const int q0 = qb * BQ;
  const int qrow = q0 + wave * 32 + lr;
  const bool qvalid = qrow < S;
  static_assert(BQ == 32 * WAVES, "geometry");

  bf16x8 qf[DSTEPS];
  auto load_q = [&]() __attribute__((always_inline)) {
    // ---- Q^T fragments (B operand of S^T = K Q^T): lane holds Q[qrow][16s + 8hh .. +8)
    const uint16_t* qp = a.q + ((long long)b * S + (qvalid ? qrow : 0)) * a.q_rs + (long long)hq * D + 8 * hh;
#pragma unroll
    for (int s = 0; s < DSTEPS; ++s) {
      uint4 v = qvalid ? *reinterpret_cast<const uint4*>(qp + 16 * s) : make_uint4(0, 0, 0, 0);
      qf[s] = as_bf8(v);
    }
  };
  if constexpr (!FWD_EARLY_DMA) load_q();

  // ---- key range
  const int q_last = min(S, q0 + BQ) - 1;
  int kv_end = min(a.causal ? q_last + 1 : S, a.kv_valid);
  int kv_begin = 0;
  if (a.window > 0) {
    kv_begin = max(0, q0 - a.window + 1);
    kv_begin = (kv_begin / BK) * BK;
  }
  // document-masked packing: key k is visible to query q only when doc_start[q] <= k.  doc_start is
  // non-decreasing along a sequence, so the block's first row bounds the key range and the wave's
  // last row tells whether a tile needs the per-element mask.
  int dlo = -0x3fffffff, wdmax = -0x3fffffff;
  if (a.doc_start) {
    const int* ds = a.doc_start + (long long)b * S;
    dlo = ds[qvalid ? qrow : S - 1];
    wdmax = ds[min(S - 1, q0 + wave * 32 + 31)];
    kv_begin = max(kv_begin, (ds[q0] / BK) * BK);
  }
  const int ntiles = (kv_end - kv_begin + BK - 1) / BK;

  const uint16_t* kbase = a.k + (long long)b * S * a.kv_rs + (long long)kvh * D;
  const uint16_t* vbase = a.v + (long long)b * S * a.kv_rs + (long long)kvh * D;
  // rows of one (b, kv head) span < 2 GiB (S * kv_rs * 2 bytes): 32-bit buffer offsets
  const auto krs = make_rsrc(kbase), vrs = make_rsrc(vbase);
  int voff[NGT];
#pragma unroll
  for (int i = 0; i < NGT; ++i) {
    const int row = (wave * NGT + i) * RPG + lane / NCH, pc = lane % NCH;
    voff[i] = (row * (int)a.kv_rs + ((pc ^ swz(row)) & (NCH - 1)) * 8) * 2;
  }

  f32x16 o[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[t][i] = 0.f;
  float m = -INFINITY, l = 0.f;
  const float c = a.scale_log2;

  if constexpr (FWD_EARLY_DMA) {
    // tile 0's K/V DMA first, then the Q loads: both latencies overlap (the first tile's vmcnt(0)
    // covers the two) instead of Q retiring before the DMA is issued
    if (ntiles > 0) fwd_dma<D, NGT, RPG>(krs, vrs, voff, kv_begin * (int)a.kv_rs * 2, K0, V0, wave);
    load_q();
  } else {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // Q fragments (plain loads) retired before any DMA: vmcnt(0)
    if (ntiles > 0) fwd_dma<D, NGT, RPG>(krs, vrs, voff, kv_begin * (int)a.kv_rs * 2, K0, V0, wave);
  }

  // tr-read addressing (V^T A operand): 16-lane group gi = lane>>4 covers d cols [16*(gi&1), +16)
  // of the 32-wide d tile and key rows [16ks + 4*hh (+8), +4)
  const int gi = lane >> 4, li = lane & 15;
  const int trq = li >> 2, trp = li & 3;
  // lane byte offsets of the transposed V reads, hoisted out of the tile loop: row r1 = 16 ks + 4 hh
  // + trq has swizzle (trq << 2) | hh for every ks (r1 + 8: | (hh + 2)), so ks only moves the row by
  // a compile-time 16 * D * 2 bytes (the ds_read's immediate offset) and the 2 * DT lane offsets below
  // are the only per-lane addressing left in phase B2 (was ~20 address adds per tile)
  int vto[DT][2];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    const int col = dt * 32 + 16 * (gi & 1) + 4 * trp;
    const int chunk = col >> 3, half8 = (col & 7) ? 8 : 0;
    vto[dt][0] = lds_off<D>(4 * hh + trq, chunk) + half8;
    vto[dt][1] = lds_off<D>(4 * hh + trq + 8, chunk) + half8;
  }

  f32x16 s[2];   // S^T of the current tile, then its P (registers between the phases)
  bf16x8 pf[4];  // packed P^T operand of the PV MFMAs
  // wait for tile t, barrier, then DMA tile t+1 into the slots that held tile t-1
  auto sync_tile = [&](const int t, char* Kn, char* Vn) __attribute__((always_inline)) {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // this wave's pieces of tile t landed (vmcnt(0))
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();        // ... and everyone's
    if (t + 1 < ntiles) fwd_dma<D, NGT, RPG>(krs, vrs, voff, (kv_begin + (t + 1) * BK) * (int)a.kv_rs * 2, Kn, Vn, wave);
  };
  // ---- phase A: S^T = K Q^T, two 32-key blocks
  auto phaseA = [&](const char* Kc) __attribute__((always_inline)) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      // issue all LDS reads of this 32-key block before its MFMA chain (no read->wait->mfma serialisation)
      const int r = kt * 32 + lr;
      uint4 kf[DSTEPS];
#pragma unroll
      for (int st = 0; st < DSTEPS; ++st) kf[st] = *reinterpret_cast<const uint4*>(Kc + lds_off<D>(r, 2 * st + hh));
      f32x16 acc;
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
      for (int st = 0; st < DSTEPS; ++st) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf8(kf[st]), qf[st], acc, 0, 0, 0);
      s[kt] = acc;
    }
    // software pipeline of the 2*DSTEPS K-fragment reads against the MFMA chain, 4 reads in flight
    // (the default scheduler serialises read -> wait -> mfma to save registers)
    __builtin_amdgcn_sched_group_barrier(0x100, FWD_KPRE, 0);
#pragma unroll
    for (int i = 0; i < 2 * DSTEPS - FWD_KPRE; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, FWD_KPRE, 0);
  };
  // ---- phase B1: mask (wave-uniform branch, branch-free selects inside) + online softmax in the log2
  // domain; P packed as the bf16 B operand of the PV MFMAs
  auto phaseB1 = [&](const int t) __attribute__((always_inline)) {
    const int kv0 = kv_begin + t * BK;
    const int qmin_w = q0 + wave * 32;
    const bool need_mask = (a.causal && kv0 + BK - 1 > qmin_w) || (a.window > 0 && qmin_w + 31 - kv0 >= a.window) ||
                           kv0 + BK > a.kv_valid ||
                           kv0 < wdmax;
    if (need_mask) {
      // key k of element (kt, i) = kv0 + kt*32 + (i&3) + 8*(i>>2) + 4*hh; valid iff lo <= k <= hi
      const int base = kv0 + 4 * hh;
      const int hi = min(a.causal ? qrow : 0x3fffffff, a.kv_valid - 1) - base;
      const int lo = max(a.window > 0 ? qrow - a.window + 1 : -0x3fffffff, dlo) - base;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int off = kt * 32 + (i & 3) + 8 * (i >> 2);
          s[kt][i] = (off >= lo && off <= hi) ? s[kt][i] : -INFINITY;
        }
    }
    float mt = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i) mt = fmaxf(mt, s[kt][i]);  // (a depth-5 fmaxf tree measured 3-4 % slower)
    mt = xhalf_max(mt) * c;  // c > 0: max commutes with the scale
    // deferred rescale (guide T13): the running reference m moves -- and O, l are rescaled -- only
    // when some row's max grew by more than 2^8; otherwise P <= 256 (exact in bf16's exponent range,
    // fp32 accumulation) and the 64 multiplies of O are skipped.  Wave-uniform branch.
    if (__builtin_amdgcn_ballot_w64(mt > m + 8.0f) != 0) {
      const float mn = fmaxf(m, mt);
      const float alpha = __builtin_amdgcn_exp2f(m - ((mn == -INFINITY) ? 0.f : mn));
      m = mn;
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[dt][i] *= alpha;
    }
    const float mref = (m == -INFINITY) ? 0.f : m;
#if FWD_PK_SOFTMAX
    // element pairs through packed fp32 VALU: v_pk_fma_f32 for the scale / shift and v_pk_add_f32 for
    // the row sum (16 + 16 instructions instead of 32 + 32, and a 16-deep instead of a 32-deep add
    // chain); the exponentials stay scalar
    f32x2 rs2 = {0.f, 0.f};
    const f32x2 c2 = {c, c}, m2 = {-mref, -mref};
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        const f32x2 x = {s[kt][i], s[kt][i + 1]};
        const f32x2 y = __builtin_elementwise_fma(x, c2, m2);
        const f32x2 pp = {__builtin_amdgcn_exp2f(y[0]), __builtin_amdgcn_exp2f(y[1])};
        s[kt][i] = pp[0];
        s[kt][i + 1] = pp[1];
        rs2 += pp;
      }
    l += rs2[0] + rs2[1];
#else
    float rs = 0.f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[kt][i], c, -mref));
        s[kt][i] = p;
        rs += p;
        if (FWD_PIN) asm volatile("" : "+v"(rs));  // lab: keep the row sum in B1 (see W64_PIN)
      }
    l += rs;
#endif
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) pf[ks] = pack_p(s[ks >> 1], 8 * (ks & 1));
  };
  // ---- phase B2: O^T += V^T P^T, 4 k-steps of 16 keys
  auto phaseB2 = [&](const char* Vc) __attribute__((always_inline)) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      s16x4 vt[8];  // all 8 transposed reads of this 32-wide d tile in flight before the MFMA chain
      const char* v0 = Vc + vto[dt][0];
      const char* v8 = Vc + vto[dt][1];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        vt[2 * ks] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(v0 + ks * 16 * D * 2));
        vt[2 * ks + 1] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(v8 + ks * 16 * D * 2));
      }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const s16x4 v1 = vt[2 * ks], v2 = vt[2 * ks + 1];
        s16x8 va = {v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
        o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, va), pf[ks], o[dt], 0, 0, 0);
      }
    }
  };
  // tile t reads (Kc, Vc); tile t+1 is DMA'd into (Kn, Vn), which held tile t-1 -- free once every
  // wave passed this tile's barrier
  auto tile = [&](const int t, const char* Kc, const char* Vc, char* Kn, char* Vn) __attribute__((always_inline)) {
    sync_tile(t, Kn, Vn);
    if constexpr (FWD_PRIO) __builtin_amdgcn_s_setprio(1);  // S MFMA phase ahead of the partner wave's VALU
    phaseA(Kc);
    if constexpr (FWD_PRIO) __builtin_amdgcn_s_setprio(0);
    phaseB1(t);
    phaseB2(Vc);
  };
  for (int t = 0; t < ntiles; t += 2) {
    tile(t, K0, V0, K1, V1);
    if (t + 1 < ntiles) tile(t + 1, K1, V1, K0, V0);
  }

  // ---- epilogue: normalise, store O (bf16) and LSE (natural log)
  const float ltot = l + __shfl_xor(l, 32, 64);
  const float inv = ltot > 0.f ? 1.0f / ltot : 0.f;
  uint16_t* op = a.o + ((long long)b * S + (qvalid ? qrow : 0)) * a.o_rs + (long long)hq * D;
  if (FWD_WIDE_STORE && (a.o_rs & 7) == 0) {
    // 16-byte stores (guide T21: the store tail is issue-bound): lanes l and l ^ 32 hold the same
    // query row, d runs {8 g4 + 4 hh + 0..3}; two v_permlane32_swap per dword pair give lane half hh
    // the 16 contiguous d [16 hh, 16 hh + 16) of each 32-wide tile -> 2 x dwordx4 instead of 4 x dwordx2
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      uint32_t w[4][2];
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        w[g4][0] = pack_bf2(o[dt][4 * g4 + 0] * inv, o[dt][4 * g4 + 1] * inv);
        w[g4][1] = pack_bf2(o[dt][4 * g4 + 2] * inv, o[dt][4 * g4 + 3] * inv);
      }
      // swap(x, y): lanes 0-31 keep x and receive the upper half's x; lanes 32-63 receive the lower
      // half's y and keep y -> (x_own | x_partner) below, (y_partner | y_own) above
      const auto a0 = __builtin_amdgcn_permlane32_swap(w[0][0], w[2][0], false, false);
      const auto a1 = __builtin_amdgcn_permlane32_swap(w[0][1], w[2][1], false, false);
      const auto b0 = __builtin_amdgcn_permlane32_swap(w[1][0], w[3][0], false, false);
      const auto b1 = __builtin_amdgcn_permlane32_swap(w[1][1], w[3][1], false, false);
      if (qvalid) {
        const int d = dt * 32 + 16 * hh;
        *reinterpret_cast<uint4*>(op + d) = make_uint4(a0[0], a1[0], a0[1], a1[1]);
        *reinterpret_cast<uint4*>(op + d + 8) = make_uint4(b0[0], b1[0], b0[1], b1[1]);
      }
    }
  } else if (qvalid) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = dt * 32 + 8 * g4 + 4 * hh;
        uint2 w;
        w.x = pack_bf2(o[dt][4 * g4 + 0] * inv, o[dt][4 * g4 + 1] * inv);
        w.y = pack_bf2(o[dt][4 * g4 + 2] * inv, o[dt][4 * g4 + 3] * inv);
        *reinterpret_cast<uint2*>(op + d) = w;
      }
  }
  if (qvalid) {
    if (hh == 0) {
      const float lse2 = (m == -INFINITY) ? -INFINITY : m + __log2f(ltot);
      a.lse[((long long)b * a.H + hq) * S + qrow] = lse2 * LN2;
    }
  }
}


// ==== W64 (round 6): the one-wave-per-SIMD, 64-rows-per-wave forward lives in the lab
// (tools/w64_lab/w64_fwd_kernel.inc, compiled only with W64_LAB: it lost in the headline step).
#ifndef W64_LAB
#define W64_LAB 0
#endif
#if W64_LAB
#include "../../tools/w64_lab/w64_fwd_kernel.inc"
#endif  // W64_LAB

}  // namespace

// (Removed in round 5: skipping a tile a wave sees fully masked (causal diagonal) -- 0.566 / 0.559 vs
// 0.558 / 0.556 ms, profiles/r5/followup/.)
// (Removed in round 5: the row sum l on the matrix pipe -- a fifth O^T tile with an all-ones A operand,
// 4 MFMAs per tile instead of 32 f32 adds: forward 0.570 vs 0.553 ms, profiles/r5/attn_skip/.)
// (Removed in round 4: QB2 -- two 32-row query blocks per wave, one wave per SIMD, the softmax of one
// block fenced between the other block's MFMAs, asm-DMA 3-slot ring: 0.740 vs 0.554 ms at the Llama-3-8B
// layer, profiles/r4/attn/fwd_qb6.log; git history has the kernel.)

#if W64_LAB
// lab: the forward variant of every later call (W64_DEFAULT), switched in one process by the lab's
// timing / numerics scripts (ftc_flash_fwd_config)
#ifndef W64_DEFAULT
#define W64_DEFAULT 1
#endif
namespace {
int& fwd_variant() {
  static int v = W64_DEFAULT;
  return v;
}
int& fwd_persistent() {
  static int v = 1;
  return v;
}
}  // namespace

// variant: 1 = W64 (persistent grid), 2 = W64 with one workgroup per block, 0 = the 32-row kernel everywhere,
// negative = the build default
#if W64_STAMPS
extern "C" int ftc_w64_stamps(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(w64_stamps), sizeof(w64_stamps));
}
extern "C" int ftc_w64_bstamps(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(w64_bstamps), sizeof(w64_bstamps));
}
#endif
extern "C" void ftc_flash_fwd_config(int variant) {
  if (variant < 0) variant = W64_DEFAULT;  // back to the build's default
  fwd_variant() = variant ? 1 : 0;
  fwd_persistent() = variant == 2 ? 0 : 1;
}
#endif  // W64_LAB

extern "C" int ftc_flash_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int S, int H,
                             int KV, int D, long long q_rs, long long kv_rs, long long o_rs, float scale, int causal,
                             int window, const int* doc_start, int kv_valid, hipStream_t stream) {
  if (S % BK != 0 || H % KV != 0 || (D != 128 && D != 64)) return -1;
  if (kv_valid <= 0 || kv_valid > S) kv_valid = S;
#if W64_LAB
  if (fwd_variant() == 1 && D == 128 && S % W64_BQ == 0 && window <= 0 && doc_start == nullptr && kv_valid == S &&
      (o_rs & 7) == 0) {
    FwdArgs a{(const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (uint16_t*)o, lse, q_rs, kv_rs, o_rs,
              B, S, H, KV, S / W64_BQ, scale * LOG2E, causal, 0, nullptr, S};
    // persistent: one workgroup per CU (LDS and registers allow no second), each walking its share of the
    // blocks heaviest-first; fewer workgroups than blocks only when there are more blocks than CUs
    static int n_cu[64] = {0};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev >= 0 && dev < 64 && n_cu[dev] == 0) {
      int v = 0;
      if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
      n_cu[dev] = v;
    }
    const int cus = (dev >= 0 && dev < 64) ? n_cu[dev] : 256;
    const int total = a.nqb * B * H;
    const int grid = fwd_persistent() ? (total < cus ? total : cus) : total;
    hipLaunchKernelGGL((flash_fwd_w64_kernel<128>), dim3(grid), dim3(256), 0, stream, a);
    return (int)hipGetLastError();
  }
#endif
  constexpr int BQ = 32 * WAVES;
  FwdArgs a{(const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (uint16_t*)o, lse, q_rs, kv_rs, o_rs,
            B, S, H, KV, (S + BQ - 1) / BQ, scale * LOG2E, causal, window, doc_start, kv_valid};
  const int nblocks = a.nqb * B * H;
  if (D == 128) {
    hipLaunchKernelGGL((flash_fwd_kernel<128>), dim3(nblocks), dim3(256), 0, stream, a);
  } else {
    hipLaunchKernelGGL((flash_fwd_kernel<64>), dim3(nblocks), dim3(256), 0, stream, a);
  }
  return (int)hipGetLastError();
}
