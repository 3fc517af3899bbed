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


// ==== W64: one wave per SIMD, 64 query rows per wave, software-pipelined across tiles (round 6) =========
//
// LAB ONLY (compiled when W64_LAB is 1: tools/w64_lab/build.sh, tests/test_build.py's audit; the package
// build leaves it out -- it measured 0.5 % slower in the headline step than flash_fwd_kernel,
// profiles/r6/w64/README.md).
//
// A workgroup = 4 waves = 256 query rows of one (batch, q head); wave w owns rows q0 + 64 w + [0, 64) as two
// 32-row blocks j = 0, 1 (one wave per SIMD: the whole 512-register file).  Every K / V^T fragment feeds
// BOTH blocks' MFMAs, and each wave runs its softmax one phase behind its own matrix work:
//
//   iteration i:  sync (vmcnt + barrier) | O rescale if the last start asked for it (rare)
//     X_i  32 MFMAs  S(i) = K(i) Q^T (block-major)  || finish softmax(i-1) (keys 32-63, one exp per gap);
//                                                    V(i-1)^T fragments 0-7; LDS-DMA of K(i+2) (and V);
//                                                    block 0's row max / statistics of tile i
//     seam           K(i+1) -> a[64:127] (16 asm ds_read_b128: also the S results' wait states)
//     Y_i  32 MFMAs  O += V(i-1)^T P(i-1)^T         || start softmax(i): block 1's row max / statistics,
//                                                    keys 0-31 of both blocks (one exp per gap);
//                                                    V(i-1)^T fragments 8-15
//
// Registers: the whole accumulator file is kernel-owned -- Q a[0:63] and K a[64:127] loaded by asm
// ds_read_b128, O a[128:255] accumulated by asm MFMAs; S lands in VGPRs from asm MFMAs (this file is built
// with -mllvm -amdgpu-mfma-vgpr-form, tools/build.py).  tools/check_asm_hazards.py audits every build: no
// compiler instruction touches a[0:255] or M0, no VALU write feeds an asm MFMA operand unpadded, no
// instruction reads an asm S result within 12 wait states.  Gaps are fenced by sched_barrier AND their VALU
// results pinned by empty volatile asm (the IR passes otherwise move work across the fences).  Persistent
// grid, heaviest causal blocks first, K / V / Q streamed across block seams; one barrier per tile; the
// deferred rescale (a row max moves only when it grew by more than 2^8) is applied at the next seam.
// Covers head_dim 128, no window / document mask / padded tail, S % 256 == 0; otherwise ftc_flash_fwd
// runs flash_fwd_kernel.
#ifndef W64_LAB
#define W64_LAB 0
#endif
#if W64_LAB
constexpr int W64_BQ = 256;
// timing-only ablations for tools/w64_lab (wrong results; never set by tools/build.py): no barrier in the
// per-tile sync, no LDS-DMA in the loop, no exponentials (P packed from raw S)
#ifndef W64_ABL_NOBAR
#define W64_ABL_NOBAR 0
#endif
#ifndef W64_ABL_NODMA
#define W64_ABL_NODMA 0
#endif
#ifndef W64_ABL_NOEXP
#define W64_ABL_NOEXP 0
#endif
#ifndef W64_ABL_NOLDS  // K / Q / V^T fragments not read from LDS (lane-constant registers instead)
#define W64_ABL_NOLDS 0
#endif
#ifndef W64_TAIL_J1FIRST
#define W64_TAIL_J1FIRST 0
#endif
#ifndef W64_TAIL_NOP
#define W64_TAIL_NOP 0
#endif
#ifndef W64_XB  // 0: no cross-block prefetch (the next block's Q, K(0), K(1) DMA'd at its start)
#define W64_XB 1
#endif
#ifndef W64_V3  // 1: a 3-slot V ring streamed one tile ahead (the whole 160 KiB of LDS); 0: 2 slots, same tile
#define W64_V3 0
#endif
#ifndef W64_SEAM  // 1: the last wave carries its final tile into the next block's first body (no tail)
#define W64_SEAM 1
#endif
#ifndef W64_QEARLY
#define W64_QEARLY 1
#endif
#ifndef W64_PIN
#define W64_PIN 1
#endif
#ifndef W64_STAMPS  // lab only: s_memtime stamps of workgroup 0's first block, tiles 20-23 (ftc_w64_stamps)
#define W64_STAMPS 0
#endif
#if W64_STAMPS
__device__ unsigned long long w64_stamps[4][4][6];
__device__ unsigned long long w64_bstamps[8][4][6];  // workgroup 0, blocks 0-7: per-block phase boundaries
#endif
#ifndef W64_DEFER
#define W64_DEFER 8.0f
#endif

// O lives in accumulator registers the kernel OWNS: a[128:255], tile (j, dt) at a[128 + 16 (4 j + dt) ..+15],
// written and read only by the inline asm below (MFMAs, zeroing, rescale, epilogue reads), which lists them as
// clobbers (that also makes the kernel descriptor allocate all 256).  The compiler never holds O, so it can
// neither copy nor spill it: copies of "+a" operands it had inserted right after an asm MFMA read the
// accumulators before the MFMA had written them (no hazard padding across asm) and corrupted block 1 on
// ~0.1 % of rows.  The compiler's own accumulator use (VGPR spill slots) stays in a[0:127];
// tools/check_asm_hazards.py --owned 128 fails the build audit if any compiler instruction touches a[128:255].
// clobber lists of the eight 16-register O tiles (a128-a143, ..., a240-a255)
#define W64_CLOB_T0 "a128", "a129", "a130", "a131", "a132", "a133", "a134", "a135", "a136", "a137", "a138", "a139", "a140", "a141", "a142", "a143"
#define W64_CLOB_T1 "a144", "a145", "a146", "a147", "a148", "a149", "a150", "a151", "a152", "a153", "a154", "a155", "a156", "a157", "a158", "a159"
#define W64_CLOB_T2 "a160", "a161", "a162", "a163", "a164", "a165", "a166", "a167", "a168", "a169", "a170", "a171", "a172", "a173", "a174", "a175"
#define W64_CLOB_T3 "a176", "a177", "a178", "a179", "a180", "a181", "a182", "a183", "a184", "a185", "a186", "a187", "a188", "a189", "a190", "a191"
#define W64_CLOB_T4 "a192", "a193", "a194", "a195", "a196", "a197", "a198", "a199", "a200", "a201", "a202", "a203", "a204", "a205", "a206", "a207"
#define W64_CLOB_T5 "a208", "a209", "a210", "a211", "a212", "a213", "a214", "a215", "a216", "a217", "a218", "a219", "a220", "a221", "a222", "a223"
#define W64_CLOB_T6 "a224", "a225", "a226", "a227", "a228", "a229", "a230", "a231", "a232", "a233", "a234", "a235", "a236", "a237", "a238", "a239"
#define W64_CLOB_T7 "a240", "a241", "a242", "a243", "a244", "a245", "a246", "a247", "a248", "a249", "a250", "a251", "a252", "a253", "a254", "a255"
#define W64_CLOB_ALL W64_CLOB_T0, W64_CLOB_T1, W64_CLOB_T2, W64_CLOB_T3, W64_CLOB_T4, W64_CLOB_T5, W64_CLOB_T6, W64_CLOB_T7

// O tile T (= 4 j + dt) += V^T . P^T
template <int T>
DEV_INLINE void w64_pv(const bf16x8& va, const bf16x8& p) {
  constexpr int B = 128 + 16 * T;
  if constexpr (T == 0)
    asm volatile("v_mfma_f32_32x32x16_bf16 a[%c2:%c3], %0, %1, a[%c2:%c3]" ::"v"(va), "v"(p), "i"(B), "i"(B + 15) : W64_CLOB_T0);
  if constexpr (T == 1)
    asm volatile("v_mfma_f32_32x32x16_bf16 a[%c2:%c3], %0, %1, a[%c2:%c3]" ::"v"(va), "v"(p), "i"(B), "i"(B + 15) : W64_CLOB_T1);
  if constexpr (T == 2)
    asm volatile("v_mfma_f32_32x32x16_bf16 a[%c2:%c3], %0, %1, a[%c2:%c3]" ::"v"(va), "v"(p), "i"(B), "i"(B + 15) : W64_CLOB_T2);
  if constexpr (T == 3)
    asm volatile("v_mfma_f32_32x32x16_bf16 a[%c2:%c3], %0, %1, a[%c2:%c3]" ::"v"(va), "v"(p), "i"(B), "i"(B + 15) : W64_CLOB_T3);
  if constexpr (T == 4)
    asm volatile("v_mfma_f32_32x32x16_bf16 a[%c2:%c3], %0, %1, a[%c2:%c3]" ::"v"(va), "v"(p), "i"(B), "i"(B + 15) : W64_CLOB_T4);
  if constexpr (T == 5)
    asm volatile("v_mfma_f32_32x32x16_bf16 a[%c2:%c3], %0, %1, a[%c2:%c3]" ::"v"(va), "v"(p), "i"(B), "i"(B + 15) : W64_CLOB_T5);
  if constexpr (T == 6)
    asm volatile("v_mfma_f32_32x32x16_bf16 a[%c2:%c3], %0, %1, a[%c2:%c3]" ::"v"(va), "v"(p), "i"(B), "i"(B + 15) : W64_CLOB_T6);
  if constexpr (T == 7)
    asm volatile("v_mfma_f32_32x32x16_bf16 a[%c2:%c3], %0, %1, a[%c2:%c3]" ::"v"(va), "v"(p), "i"(B), "i"(B + 15) : W64_CLOB_T7);
}
// zero all of O (block start); the trailing nops cover v_accvgpr_write -> MFMA SrcC
DEV_INLINE void w64_o_zero() {
  asm volatile("v_accvgpr_write_b32 a128, 0\n\tv_accvgpr_write_b32 a129, 0\n\tv_accvgpr_write_b32 a130, 0\n\tv_accvgpr_write_b32 a131, 0\n\tv_accvgpr_write_b32 a132, 0\n\tv_accvgpr_write_b32 a133, 0\n\tv_accvgpr_write_b32 a134, 0\n\tv_accvgpr_write_b32 a135, 0\n\tv_accvgpr_write_b32 a136, 0\n\tv_accvgpr_write_b32 a137, 0\n\tv_accvgpr_write_b32 a138, 0\n\tv_accvgpr_write_b32 a139, 0\n\tv_accvgpr_write_b32 a140, 0\n\tv_accvgpr_write_b32 a141, 0\n\tv_accvgpr_write_b32 a142, 0\n\tv_accvgpr_write_b32 a143, 0\n\tv_accvgpr_write_b32 a144, 0\n\tv_accvgpr_write_b32 a145, 0\n\tv_accvgpr_write_b32 a146, 0\n\tv_accvgpr_write_b32 a147, 0\n\tv_accvgpr_write_b32 a148, 0\n\tv_accvgpr_write_b32 a149, 0\n\tv_accvgpr_write_b32 a150, 0\n\tv_accvgpr_write_b32 a151, 0\n\tv_accvgpr_write_b32 a152, 0\n\tv_accvgpr_write_b32 a153, 0\n\tv_accvgpr_write_b32 a154, 0\n\tv_accvgpr_write_b32 a155, 0\n\tv_accvgpr_write_b32 a156, 0\n\tv_accvgpr_write_b32 a157, 0\n\tv_accvgpr_write_b32 a158, 0\n\tv_accvgpr_write_b32 a159, 0\n\tv_accvgpr_write_b32 a160, 0\n\tv_accvgpr_write_b32 a161, 0\n\tv_accvgpr_write_b32 a162, 0\n\tv_accvgpr_write_b32 a163, 0\n\tv_accvgpr_write_b32 a164, 0\n\tv_accvgpr_write_b32 a165, 0\n\tv_accvgpr_write_b32 a166, 0\n\tv_accvgpr_write_b32 a167, 0\n\tv_accvgpr_write_b32 a168, 0\n\tv_accvgpr_write_b32 a169, 0\n\tv_accvgpr_write_b32 a170, 0\n\tv_accvgpr_write_b32 a171, 0\n\tv_accvgpr_write_b32 a172, 0\n\tv_accvgpr_write_b32 a173, 0\n\tv_accvgpr_write_b32 a174, 0\n\tv_accvgpr_write_b32 a175, 0\n\tv_accvgpr_write_b32 a176, 0\n\tv_accvgpr_write_b32 a177, 0\n\tv_accvgpr_write_b32 a178, 0\n\tv_accvgpr_write_b32 a179, 0\n\tv_accvgpr_write_b32 a180, 0\n\tv_accvgpr_write_b32 a181, 0\n\tv_accvgpr_write_b32 a182, 0\n\tv_accvgpr_write_b32 a183, 0\n\tv_accvgpr_write_b32 a184, 0\n\tv_accvgpr_write_b32 a185, 0\n\tv_accvgpr_write_b32 a186, 0\n\tv_accvgpr_write_b32 a187, 0\n\tv_accvgpr_write_b32 a188, 0\n\tv_accvgpr_write_b32 a189, 0\n\tv_accvgpr_write_b32 a190, 0\n\tv_accvgpr_write_b32 a191, 0\n\tv_accvgpr_write_b32 a192, 0\n\tv_accvgpr_write_b32 a193, 0\n\tv_accvgpr_write_b32 a194, 0\n\tv_accvgpr_write_b32 a195, 0\n\tv_accvgpr_write_b32 a196, 0\n\tv_accvgpr_write_b32 a197, 0\n\tv_accvgpr_write_b32 a198, 0\n\tv_accvgpr_write_b32 a199, 0\n\tv_accvgpr_write_b32 a200, 0\n\tv_accvgpr_write_b32 a201, 0\n\tv_accvgpr_write_b32 a202, 0\n\tv_accvgpr_write_b32 a203, 0\n\tv_accvgpr_write_b32 a204, 0\n\tv_accvgpr_write_b32 a205, 0\n\tv_accvgpr_write_b32 a206, 0\n\tv_accvgpr_write_b32 a207, 0\n\tv_accvgpr_write_b32 a208, 0\n\tv_accvgpr_write_b32 a209, 0\n\tv_accvgpr_write_b32 a210, 0\n\tv_accvgpr_write_b32 a211, 0\n\tv_accvgpr_write_b32 a212, 0\n\tv_accvgpr_write_b32 a213, 0\n\tv_accvgpr_write_b32 a214, 0\n\tv_accvgpr_write_b32 a215, 0\n\tv_accvgpr_write_b32 a216, 0\n\tv_accvgpr_write_b32 a217, 0\n\tv_accvgpr_write_b32 a218, 0\n\tv_accvgpr_write_b32 a219, 0\n\tv_accvgpr_write_b32 a220, 0\n\tv_accvgpr_write_b32 a221, 0\n\tv_accvgpr_write_b32 a222, 0\n\tv_accvgpr_write_b32 a223, 0\n\tv_accvgpr_write_b32 a224, 0\n\tv_accvgpr_write_b32 a225, 0\n\tv_accvgpr_write_b32 a226, 0\n\tv_accvgpr_write_b32 a227, 0\n\tv_accvgpr_write_b32 a228, 0\n\tv_accvgpr_write_b32 a229, 0\n\tv_accvgpr_write_b32 a230, 0\n\tv_accvgpr_write_b32 a231, 0\n\tv_accvgpr_write_b32 a232, 0\n\tv_accvgpr_write_b32 a233, 0\n\tv_accvgpr_write_b32 a234, 0\n\tv_accvgpr_write_b32 a235, 0\n\tv_accvgpr_write_b32 a236, 0\n\tv_accvgpr_write_b32 a237, 0\n\tv_accvgpr_write_b32 a238, 0\n\tv_accvgpr_write_b32 a239, 0\n\tv_accvgpr_write_b32 a240, 0\n\tv_accvgpr_write_b32 a241, 0\n\tv_accvgpr_write_b32 a242, 0\n\tv_accvgpr_write_b32 a243, 0\n\tv_accvgpr_write_b32 a244, 0\n\tv_accvgpr_write_b32 a245, 0\n\tv_accvgpr_write_b32 a246, 0\n\tv_accvgpr_write_b32 a247, 0\n\tv_accvgpr_write_b32 a248, 0\n\tv_accvgpr_write_b32 a249, 0\n\tv_accvgpr_write_b32 a250, 0\n\tv_accvgpr_write_b32 a251, 0\n\tv_accvgpr_write_b32 a252, 0\n\tv_accvgpr_write_b32 a253, 0\n\tv_accvgpr_write_b32 a254, 0\n\tv_accvgpr_write_b32 a255, 0\n\ts_nop 4" ::: W64_CLOB_ALL);
}
// O tile T *= alpha (per lane).  The caller put the MFMA -> v_accvgpr_read wait states in front
// (w64_o_wait); the chain runs through one scratch VGPR; the trailing nops cover v_accvgpr_write -> MFMA SrcC
template <int T>
DEV_INLINE void w64_o_scale(const float alpha) {
  float t;
  if constexpr (T == 0) asm volatile("v_accvgpr_read_b32 %0, a128\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a128, %0\n\tv_accvgpr_read_b32 %0, a129\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a129, %0\n\tv_accvgpr_read_b32 %0, a130\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a130, %0\n\tv_accvgpr_read_b32 %0, a131\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a131, %0\n\tv_accvgpr_read_b32 %0, a132\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a132, %0\n\tv_accvgpr_read_b32 %0, a133\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a133, %0\n\tv_accvgpr_read_b32 %0, a134\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a134, %0\n\tv_accvgpr_read_b32 %0, a135\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a135, %0\n\tv_accvgpr_read_b32 %0, a136\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a136, %0\n\tv_accvgpr_read_b32 %0, a137\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a137, %0\n\tv_accvgpr_read_b32 %0, a138\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a138, %0\n\tv_accvgpr_read_b32 %0, a139\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a139, %0\n\tv_accvgpr_read_b32 %0, a140\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a140, %0\n\tv_accvgpr_read_b32 %0, a141\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a141, %0\n\tv_accvgpr_read_b32 %0, a142\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a142, %0\n\tv_accvgpr_read_b32 %0, a143\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a143, %0\n\ts_nop 2" : "=&v"(t) : "v"(alpha) : W64_CLOB_T0);
  if constexpr (T == 1) asm volatile("v_accvgpr_read_b32 %0, a144\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a144, %0\n\tv_accvgpr_read_b32 %0, a145\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a145, %0\n\tv_accvgpr_read_b32 %0, a146\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a146, %0\n\tv_accvgpr_read_b32 %0, a147\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a147, %0\n\tv_accvgpr_read_b32 %0, a148\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a148, %0\n\tv_accvgpr_read_b32 %0, a149\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a149, %0\n\tv_accvgpr_read_b32 %0, a150\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a150, %0\n\tv_accvgpr_read_b32 %0, a151\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a151, %0\n\tv_accvgpr_read_b32 %0, a152\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a152, %0\n\tv_accvgpr_read_b32 %0, a153\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a153, %0\n\tv_accvgpr_read_b32 %0, a154\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a154, %0\n\tv_accvgpr_read_b32 %0, a155\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a155, %0\n\tv_accvgpr_read_b32 %0, a156\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a156, %0\n\tv_accvgpr_read_b32 %0, a157\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a157, %0\n\tv_accvgpr_read_b32 %0, a158\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a158, %0\n\tv_accvgpr_read_b32 %0, a159\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a159, %0\n\ts_nop 2" : "=&v"(t) : "v"(alpha) : W64_CLOB_T1);
  if constexpr (T == 2) asm volatile("v_accvgpr_read_b32 %0, a160\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a160, %0\n\tv_accvgpr_read_b32 %0, a161\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a161, %0\n\tv_accvgpr_read_b32 %0, a162\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a162, %0\n\tv_accvgpr_read_b32 %0, a163\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a163, %0\n\tv_accvgpr_read_b32 %0, a164\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a164, %0\n\tv_accvgpr_read_b32 %0, a165\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a165, %0\n\tv_accvgpr_read_b32 %0, a166\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a166, %0\n\tv_accvgpr_read_b32 %0, a167\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a167, %0\n\tv_accvgpr_read_b32 %0, a168\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a168, %0\n\tv_accvgpr_read_b32 %0, a169\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a169, %0\n\tv_accvgpr_read_b32 %0, a170\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a170, %0\n\tv_accvgpr_read_b32 %0, a171\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a171, %0\n\tv_accvgpr_read_b32 %0, a172\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a172, %0\n\tv_accvgpr_read_b32 %0, a173\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a173, %0\n\tv_accvgpr_read_b32 %0, a174\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a174, %0\n\tv_accvgpr_read_b32 %0, a175\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a175, %0\n\ts_nop 2" : "=&v"(t) : "v"(alpha) : W64_CLOB_T2);
  if constexpr (T == 3) asm volatile("v_accvgpr_read_b32 %0, a176\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a176, %0\n\tv_accvgpr_read_b32 %0, a177\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a177, %0\n\tv_accvgpr_read_b32 %0, a178\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a178, %0\n\tv_accvgpr_read_b32 %0, a179\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a179, %0\n\tv_accvgpr_read_b32 %0, a180\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a180, %0\n\tv_accvgpr_read_b32 %0, a181\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a181, %0\n\tv_accvgpr_read_b32 %0, a182\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a182, %0\n\tv_accvgpr_read_b32 %0, a183\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a183, %0\n\tv_accvgpr_read_b32 %0, a184\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a184, %0\n\tv_accvgpr_read_b32 %0, a185\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a185, %0\n\tv_accvgpr_read_b32 %0, a186\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a186, %0\n\tv_accvgpr_read_b32 %0, a187\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a187, %0\n\tv_accvgpr_read_b32 %0, a188\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a188, %0\n\tv_accvgpr_read_b32 %0, a189\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a189, %0\n\tv_accvgpr_read_b32 %0, a190\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a190, %0\n\tv_accvgpr_read_b32 %0, a191\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a191, %0\n\ts_nop 2" : "=&v"(t) : "v"(alpha) : W64_CLOB_T3);
  if constexpr (T == 4) asm volatile("v_accvgpr_read_b32 %0, a192\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a192, %0\n\tv_accvgpr_read_b32 %0, a193\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a193, %0\n\tv_accvgpr_read_b32 %0, a194\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a194, %0\n\tv_accvgpr_read_b32 %0, a195\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a195, %0\n\tv_accvgpr_read_b32 %0, a196\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a196, %0\n\tv_accvgpr_read_b32 %0, a197\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a197, %0\n\tv_accvgpr_read_b32 %0, a198\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a198, %0\n\tv_accvgpr_read_b32 %0, a199\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a199, %0\n\tv_accvgpr_read_b32 %0, a200\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a200, %0\n\tv_accvgpr_read_b32 %0, a201\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a201, %0\n\tv_accvgpr_read_b32 %0, a202\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a202, %0\n\tv_accvgpr_read_b32 %0, a203\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a203, %0\n\tv_accvgpr_read_b32 %0, a204\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a204, %0\n\tv_accvgpr_read_b32 %0, a205\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a205, %0\n\tv_accvgpr_read_b32 %0, a206\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a206, %0\n\tv_accvgpr_read_b32 %0, a207\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a207, %0\n\ts_nop 2" : "=&v"(t) : "v"(alpha) : W64_CLOB_T4);
  if constexpr (T == 5) asm volatile("v_accvgpr_read_b32 %0, a208\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a208, %0\n\tv_accvgpr_read_b32 %0, a209\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a209, %0\n\tv_accvgpr_read_b32 %0, a210\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a210, %0\n\tv_accvgpr_read_b32 %0, a211\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a211, %0\n\tv_accvgpr_read_b32 %0, a212\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a212, %0\n\tv_accvgpr_read_b32 %0, a213\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a213, %0\n\tv_accvgpr_read_b32 %0, a214\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a214, %0\n\tv_accvgpr_read_b32 %0, a215\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a215, %0\n\tv_accvgpr_read_b32 %0, a216\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a216, %0\n\tv_accvgpr_read_b32 %0, a217\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a217, %0\n\tv_accvgpr_read_b32 %0, a218\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a218, %0\n\tv_accvgpr_read_b32 %0, a219\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a219, %0\n\tv_accvgpr_read_b32 %0, a220\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a220, %0\n\tv_accvgpr_read_b32 %0, a221\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a221, %0\n\tv_accvgpr_read_b32 %0, a222\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a222, %0\n\tv_accvgpr_read_b32 %0, a223\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a223, %0\n\ts_nop 2" : "=&v"(t) : "v"(alpha) : W64_CLOB_T5);
  if constexpr (T == 6) asm volatile("v_accvgpr_read_b32 %0, a224\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a224, %0\n\tv_accvgpr_read_b32 %0, a225\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a225, %0\n\tv_accvgpr_read_b32 %0, a226\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a226, %0\n\tv_accvgpr_read_b32 %0, a227\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a227, %0\n\tv_accvgpr_read_b32 %0, a228\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a228, %0\n\tv_accvgpr_read_b32 %0, a229\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a229, %0\n\tv_accvgpr_read_b32 %0, a230\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a230, %0\n\tv_accvgpr_read_b32 %0, a231\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a231, %0\n\tv_accvgpr_read_b32 %0, a232\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a232, %0\n\tv_accvgpr_read_b32 %0, a233\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a233, %0\n\tv_accvgpr_read_b32 %0, a234\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a234, %0\n\tv_accvgpr_read_b32 %0, a235\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a235, %0\n\tv_accvgpr_read_b32 %0, a236\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a236, %0\n\tv_accvgpr_read_b32 %0, a237\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a237, %0\n\tv_accvgpr_read_b32 %0, a238\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a238, %0\n\tv_accvgpr_read_b32 %0, a239\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a239, %0\n\ts_nop 2" : "=&v"(t) : "v"(alpha) : W64_CLOB_T6);
  if constexpr (T == 7) asm volatile("v_accvgpr_read_b32 %0, a240\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a240, %0\n\tv_accvgpr_read_b32 %0, a241\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a241, %0\n\tv_accvgpr_read_b32 %0, a242\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a242, %0\n\tv_accvgpr_read_b32 %0, a243\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a243, %0\n\tv_accvgpr_read_b32 %0, a244\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a244, %0\n\tv_accvgpr_read_b32 %0, a245\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a245, %0\n\tv_accvgpr_read_b32 %0, a246\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a246, %0\n\tv_accvgpr_read_b32 %0, a247\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a247, %0\n\tv_accvgpr_read_b32 %0, a248\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a248, %0\n\tv_accvgpr_read_b32 %0, a249\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a249, %0\n\tv_accvgpr_read_b32 %0, a250\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a250, %0\n\tv_accvgpr_read_b32 %0, a251\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a251, %0\n\tv_accvgpr_read_b32 %0, a252\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a252, %0\n\tv_accvgpr_read_b32 %0, a253\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a253, %0\n\tv_accvgpr_read_b32 %0, a254\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a254, %0\n\tv_accvgpr_read_b32 %0, a255\n\tv_mul_f32 %0, %0, %1\n\tv_accvgpr_write_b32 a255, %0\n\ts_nop 2" : "=&v"(t) : "v"(alpha) : W64_CLOB_T7);
  (void)t;
}
// Q (a[0:63]: block j, k-step st at a[4 (8 j + st)]) and K (a[64:127]: 32-key half kt, k-step st at
// a[64 + 4 (8 kt + st)]) also live in kernel-owned accumulator registers: the S MFMA reads both operands from
// there, its result lands in VGPRs (the softmax's), and K(i+1) is loaded a whole phase ahead (during Y_i)
// by asm ds_reads the compiler neither counts nor sees -- the per-tile sync's lgkmcnt(0) covers them.
#define W64_CLOB_G0 "a0", "a1", "a2", "a3"
#define W64_CLOB_G1 "a4", "a5", "a6", "a7"
#define W64_CLOB_G2 "a8", "a9", "a10", "a11"
#define W64_CLOB_G3 "a12", "a13", "a14", "a15"
#define W64_CLOB_G4 "a16", "a17", "a18", "a19"
#define W64_CLOB_G5 "a20", "a21", "a22", "a23"
#define W64_CLOB_G6 "a24", "a25", "a26", "a27"
#define W64_CLOB_G7 "a28", "a29", "a30", "a31"
#define W64_CLOB_G8 "a32", "a33", "a34", "a35"
#define W64_CLOB_G9 "a36", "a37", "a38", "a39"
#define W64_CLOB_G10 "a40", "a41", "a42", "a43"
#define W64_CLOB_G11 "a44", "a45", "a46", "a47"
#define W64_CLOB_G12 "a48", "a49", "a50", "a51"
#define W64_CLOB_G13 "a52", "a53", "a54", "a55"
#define W64_CLOB_G14 "a56", "a57", "a58", "a59"
#define W64_CLOB_G15 "a60", "a61", "a62", "a63"
#define W64_CLOB_G16 "a64", "a65", "a66", "a67"
#define W64_CLOB_G17 "a68", "a69", "a70", "a71"
#define W64_CLOB_G18 "a72", "a73", "a74", "a75"
#define W64_CLOB_G19 "a76", "a77", "a78", "a79"
#define W64_CLOB_G20 "a80", "a81", "a82", "a83"
#define W64_CLOB_G21 "a84", "a85", "a86", "a87"
#define W64_CLOB_G22 "a88", "a89", "a90", "a91"
#define W64_CLOB_G23 "a92", "a93", "a94", "a95"
#define W64_CLOB_G24 "a96", "a97", "a98", "a99"
#define W64_CLOB_G25 "a100", "a101", "a102", "a103"
#define W64_CLOB_G26 "a104", "a105", "a106", "a107"
#define W64_CLOB_G27 "a108", "a109", "a110", "a111"
#define W64_CLOB_G28 "a112", "a113", "a114", "a115"
#define W64_CLOB_G29 "a116", "a117", "a118", "a119"
#define W64_CLOB_G30 "a120", "a121", "a122", "a123"
#define W64_CLOB_G31 "a124", "a125", "a126", "a127"
template <int G>
DEV_INLINE void w64_lda(const unsigned addr) {  // a[4 G .. 4 G + 3] = the 16 bytes at LDS addr
  if constexpr (G == 0) asm volatile("ds_read_b128 a[0:3], %0" ::"v"(addr) : W64_CLOB_G0);
  if constexpr (G == 1) asm volatile("ds_read_b128 a[4:7], %0" ::"v"(addr) : W64_CLOB_G1);
  if constexpr (G == 2) asm volatile("ds_read_b128 a[8:11], %0" ::"v"(addr) : W64_CLOB_G2);
  if constexpr (G == 3) asm volatile("ds_read_b128 a[12:15], %0" ::"v"(addr) : W64_CLOB_G3);
  if constexpr (G == 4) asm volatile("ds_read_b128 a[16:19], %0" ::"v"(addr) : W64_CLOB_G4);
  if constexpr (G == 5) asm volatile("ds_read_b128 a[20:23], %0" ::"v"(addr) : W64_CLOB_G5);
  if constexpr (G == 6) asm volatile("ds_read_b128 a[24:27], %0" ::"v"(addr) : W64_CLOB_G6);
  if constexpr (G == 7) asm volatile("ds_read_b128 a[28:31], %0" ::"v"(addr) : W64_CLOB_G7);
  if constexpr (G == 8) asm volatile("ds_read_b128 a[32:35], %0" ::"v"(addr) : W64_CLOB_G8);
  if constexpr (G == 9) asm volatile("ds_read_b128 a[36:39], %0" ::"v"(addr) : W64_CLOB_G9);
  if constexpr (G == 10) asm volatile("ds_read_b128 a[40:43], %0" ::"v"(addr) : W64_CLOB_G10);
  if constexpr (G == 11) asm volatile("ds_read_b128 a[44:47], %0" ::"v"(addr) : W64_CLOB_G11);
  if constexpr (G == 12) asm volatile("ds_read_b128 a[48:51], %0" ::"v"(addr) : W64_CLOB_G12);
  if constexpr (G == 13) asm volatile("ds_read_b128 a[52:55], %0" ::"v"(addr) : W64_CLOB_G13);
  if constexpr (G == 14) asm volatile("ds_read_b128 a[56:59], %0" ::"v"(addr) : W64_CLOB_G14);
  if constexpr (G == 15) asm volatile("ds_read_b128 a[60:63], %0" ::"v"(addr) : W64_CLOB_G15);
  if constexpr (G == 16) asm volatile("ds_read_b128 a[64:67], %0" ::"v"(addr) : W64_CLOB_G16);
  if constexpr (G == 17) asm volatile("ds_read_b128 a[68:71], %0" ::"v"(addr) : W64_CLOB_G17);
  if constexpr (G == 18) asm volatile("ds_read_b128 a[72:75], %0" ::"v"(addr) : W64_CLOB_G18);
  if constexpr (G == 19) asm volatile("ds_read_b128 a[76:79], %0" ::"v"(addr) : W64_CLOB_G19);
  if constexpr (G == 20) asm volatile("ds_read_b128 a[80:83], %0" ::"v"(addr) : W64_CLOB_G20);
  if constexpr (G == 21) asm volatile("ds_read_b128 a[84:87], %0" ::"v"(addr) : W64_CLOB_G21);
  if constexpr (G == 22) asm volatile("ds_read_b128 a[88:91], %0" ::"v"(addr) : W64_CLOB_G22);
  if constexpr (G == 23) asm volatile("ds_read_b128 a[92:95], %0" ::"v"(addr) : W64_CLOB_G23);
  if constexpr (G == 24) asm volatile("ds_read_b128 a[96:99], %0" ::"v"(addr) : W64_CLOB_G24);
  if constexpr (G == 25) asm volatile("ds_read_b128 a[100:103], %0" ::"v"(addr) : W64_CLOB_G25);
  if constexpr (G == 26) asm volatile("ds_read_b128 a[104:107], %0" ::"v"(addr) : W64_CLOB_G26);
  if constexpr (G == 27) asm volatile("ds_read_b128 a[108:111], %0" ::"v"(addr) : W64_CLOB_G27);
  if constexpr (G == 28) asm volatile("ds_read_b128 a[112:115], %0" ::"v"(addr) : W64_CLOB_G28);
  if constexpr (G == 29) asm volatile("ds_read_b128 a[116:119], %0" ::"v"(addr) : W64_CLOB_G29);
  if constexpr (G == 30) asm volatile("ds_read_b128 a[120:123], %0" ::"v"(addr) : W64_CLOB_G30);
  if constexpr (G == 31) asm volatile("ds_read_b128 a[124:127], %0" ::"v"(addr) : W64_CLOB_G31);
}
DEV_INLINE void w64_lda_t(const int G, const unsigned addr) {
  switch (G) {
    case 0: w64_lda<0>(addr); break;
    case 1: w64_lda<1>(addr); break;
    case 2: w64_lda<2>(addr); break;
    case 3: w64_lda<3>(addr); break;
    case 4: w64_lda<4>(addr); break;
    case 5: w64_lda<5>(addr); break;
    case 6: w64_lda<6>(addr); break;
    case 7: w64_lda<7>(addr); break;
    case 8: w64_lda<8>(addr); break;
    case 9: w64_lda<9>(addr); break;
    case 10: w64_lda<10>(addr); break;
    case 11: w64_lda<11>(addr); break;
    case 12: w64_lda<12>(addr); break;
    case 13: w64_lda<13>(addr); break;
    case 14: w64_lda<14>(addr); break;
    case 15: w64_lda<15>(addr); break;
    case 16: w64_lda<16>(addr); break;
    case 17: w64_lda<17>(addr); break;
    case 18: w64_lda<18>(addr); break;
    case 19: w64_lda<19>(addr); break;
    case 20: w64_lda<20>(addr); break;
    case 21: w64_lda<21>(addr); break;
    case 22: w64_lda<22>(addr); break;
    case 23: w64_lda<23>(addr); break;
    case 24: w64_lda<24>(addr); break;
    case 25: w64_lda<25>(addr); break;
    case 26: w64_lda<26>(addr); break;
    case 27: w64_lda<27>(addr); break;
    case 28: w64_lda<28>(addr); break;
    case 29: w64_lda<29>(addr); break;
    case 30: w64_lda<30>(addr); break;
    case 31: w64_lda<31>(addr); break;
  }
}
// S^T(j, kt) (+)= K(kt, st) . Q(j, st)^T from the owned operands into a VGPR accumulator
template <int KR, int QR, bool FIRST>
DEV_INLINE void w64_s(f32x16& acc) {
  if constexpr (FIRST)
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, a[%c1:%c2], a[%c3:%c4], 0" : "=v"(acc) : "i"(KR), "i"(KR + 3), "i"(QR), "i"(QR + 3));
  else
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, a[%c1:%c2], a[%c3:%c4], %0" : "+v"(acc) : "i"(KR), "i"(KR + 3), "i"(QR), "i"(QR + 3));
}
DEV_INLINE void w64_s_t(const int kt, const int st, const int j, f32x16& acc) {
  const int idx = (kt * 8 + st) * 2 + j;
  switch (idx) {
    case 0: w64_s<64, 0, true>(acc); break;
    case 1: w64_s<64, 32, true>(acc); break;
    case 2: w64_s<68, 4, false>(acc); break;
    case 3: w64_s<68, 36, false>(acc); break;
    case 4: w64_s<72, 8, false>(acc); break;
    case 5: w64_s<72, 40, false>(acc); break;
    case 6: w64_s<76, 12, false>(acc); break;
    case 7: w64_s<76, 44, false>(acc); break;
    case 8: w64_s<80, 16, false>(acc); break;
    case 9: w64_s<80, 48, false>(acc); break;
    case 10: w64_s<84, 20, false>(acc); break;
    case 11: w64_s<84, 52, false>(acc); break;
    case 12: w64_s<88, 24, false>(acc); break;
    case 13: w64_s<88, 56, false>(acc); break;
    case 14: w64_s<92, 28, false>(acc); break;
    case 15: w64_s<92, 60, false>(acc); break;
    case 16: w64_s<96, 0, true>(acc); break;
    case 17: w64_s<96, 32, true>(acc); break;
    case 18: w64_s<100, 4, false>(acc); break;
    case 19: w64_s<100, 36, false>(acc); break;
    case 20: w64_s<104, 8, false>(acc); break;
    case 21: w64_s<104, 40, false>(acc); break;
    case 22: w64_s<108, 12, false>(acc); break;
    case 23: w64_s<108, 44, false>(acc); break;
    case 24: w64_s<112, 16, false>(acc); break;
    case 25: w64_s<112, 48, false>(acc); break;
    case 26: w64_s<116, 20, false>(acc); break;
    case 27: w64_s<116, 52, false>(acc); break;
    case 28: w64_s<120, 24, false>(acc); break;
    case 29: w64_s<120, 56, false>(acc); break;
    case 30: w64_s<124, 28, false>(acc); break;
    case 31: w64_s<124, 60, false>(acc); break;
  }
}

DEV_INLINE void w64_pv_t(const int T, const bf16x8& va, const bf16x8& p) {
  switch (T) {
    case 0: w64_pv<0>(va, p); break;
    case 1: w64_pv<1>(va, p); break;
    case 2: w64_pv<2>(va, p); break;
    case 3: w64_pv<3>(va, p); break;
    case 4: w64_pv<4>(va, p); break;
    case 5: w64_pv<5>(va, p); break;
    case 6: w64_pv<6>(va, p); break;
    default: w64_pv<7>(va, p); break;
  }
}
// wait states between the last PV MFMA writing O and any read of it (8-pass XDL: 12; padded to 24)
DEV_INLINE void w64_o_wait() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory"); }
// read O tile T into registers (after w64_o_wait)
template <int T>
DEV_INLINE f32x16 w64_o_read() {
  float r[16];
  if constexpr (T == 0) asm volatile("v_accvgpr_read_b32 %0, a128\n\tv_accvgpr_read_b32 %1, a129\n\tv_accvgpr_read_b32 %2, a130\n\tv_accvgpr_read_b32 %3, a131\n\tv_accvgpr_read_b32 %4, a132\n\tv_accvgpr_read_b32 %5, a133\n\tv_accvgpr_read_b32 %6, a134\n\tv_accvgpr_read_b32 %7, a135\n\tv_accvgpr_read_b32 %8, a136\n\tv_accvgpr_read_b32 %9, a137\n\tv_accvgpr_read_b32 %10, a138\n\tv_accvgpr_read_b32 %11, a139\n\tv_accvgpr_read_b32 %12, a140\n\tv_accvgpr_read_b32 %13, a141\n\tv_accvgpr_read_b32 %14, a142\n\tv_accvgpr_read_b32 %15, a143\n\t" : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3]), "=v"(r[4]), "=v"(r[5]), "=v"(r[6]), "=v"(r[7]), "=v"(r[8]), "=v"(r[9]), "=v"(r[10]), "=v"(r[11]), "=v"(r[12]), "=v"(r[13]), "=v"(r[14]), "=v"(r[15]));
  if constexpr (T == 1) asm volatile("v_accvgpr_read_b32 %0, a144\n\tv_accvgpr_read_b32 %1, a145\n\tv_accvgpr_read_b32 %2, a146\n\tv_accvgpr_read_b32 %3, a147\n\tv_accvgpr_read_b32 %4, a148\n\tv_accvgpr_read_b32 %5, a149\n\tv_accvgpr_read_b32 %6, a150\n\tv_accvgpr_read_b32 %7, a151\n\tv_accvgpr_read_b32 %8, a152\n\tv_accvgpr_read_b32 %9, a153\n\tv_accvgpr_read_b32 %10, a154\n\tv_accvgpr_read_b32 %11, a155\n\tv_accvgpr_read_b32 %12, a156\n\tv_accvgpr_read_b32 %13, a157\n\tv_accvgpr_read_b32 %14, a158\n\tv_accvgpr_read_b32 %15, a159\n\t" : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3]), "=v"(r[4]), "=v"(r[5]), "=v"(r[6]), "=v"(r[7]), "=v"(r[8]), "=v"(r[9]), "=v"(r[10]), "=v"(r[11]), "=v"(r[12]), "=v"(r[13]), "=v"(r[14]), "=v"(r[15]));
  if constexpr (T == 2) asm volatile("v_accvgpr_read_b32 %0, a160\n\tv_accvgpr_read_b32 %1, a161\n\tv_accvgpr_read_b32 %2, a162\n\tv_accvgpr_read_b32 %3, a163\n\tv_accvgpr_read_b32 %4, a164\n\tv_accvgpr_read_b32 %5, a165\n\tv_accvgpr_read_b32 %6, a166\n\tv_accvgpr_read_b32 %7, a167\n\tv_accvgpr_read_b32 %8, a168\n\tv_accvgpr_read_b32 %9, a169\n\tv_accvgpr_read_b32 %10, a170\n\tv_accvgpr_read_b32 %11, a171\n\tv_accvgpr_read_b32 %12, a172\n\tv_accvgpr_read_b32 %13, a173\n\tv_accvgpr_read_b32 %14, a174\n\tv_accvgpr_read_b32 %15, a175\n\t" : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3]), "=v"(r[4]), "=v"(r[5]), "=v"(r[6]), "=v"(r[7]), "=v"(r[8]), "=v"(r[9]), "=v"(r[10]), "=v"(r[11]), "=v"(r[12]), "=v"(r[13]), "=v"(r[14]), "=v"(r[15]));
  if constexpr (T == 3) asm volatile("v_accvgpr_read_b32 %0, a176\n\tv_accvgpr_read_b32 %1, a177\n\tv_accvgpr_read_b32 %2, a178\n\tv_accvgpr_read_b32 %3, a179\n\tv_accvgpr_read_b32 %4, a180\n\tv_accvgpr_read_b32 %5, a181\n\tv_accvgpr_read_b32 %6, a182\n\tv_accvgpr_read_b32 %7, a183\n\tv_accvgpr_read_b32 %8, a184\n\tv_accvgpr_read_b32 %9, a185\n\tv_accvgpr_read_b32 %10, a186\n\tv_accvgpr_read_b32 %11, a187\n\tv_accvgpr_read_b32 %12, a188\n\tv_accvgpr_read_b32 %13, a189\n\tv_accvgpr_read_b32 %14, a190\n\tv_accvgpr_read_b32 %15, a191\n\t" : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3]), "=v"(r[4]), "=v"(r[5]), "=v"(r[6]), "=v"(r[7]), "=v"(r[8]), "=v"(r[9]), "=v"(r[10]), "=v"(r[11]), "=v"(r[12]), "=v"(r[13]), "=v"(r[14]), "=v"(r[15]));
  if constexpr (T == 4) asm volatile("v_accvgpr_read_b32 %0, a192\n\tv_accvgpr_read_b32 %1, a193\n\tv_accvgpr_read_b32 %2, a194\n\tv_accvgpr_read_b32 %3, a195\n\tv_accvgpr_read_b32 %4, a196\n\tv_accvgpr_read_b32 %5, a197\n\tv_accvgpr_read_b32 %6, a198\n\tv_accvgpr_read_b32 %7, a199\n\tv_accvgpr_read_b32 %8, a200\n\tv_accvgpr_read_b32 %9, a201\n\tv_accvgpr_read_b32 %10, a202\n\tv_accvgpr_read_b32 %11, a203\n\tv_accvgpr_read_b32 %12, a204\n\tv_accvgpr_read_b32 %13, a205\n\tv_accvgpr_read_b32 %14, a206\n\tv_accvgpr_read_b32 %15, a207\n\t" : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3]), "=v"(r[4]), "=v"(r[5]), "=v"(r[6]), "=v"(r[7]), "=v"(r[8]), "=v"(r[9]), "=v"(r[10]), "=v"(r[11]), "=v"(r[12]), "=v"(r[13]), "=v"(r[14]), "=v"(r[15]));
  if constexpr (T == 5) asm volatile("v_accvgpr_read_b32 %0, a208\n\tv_accvgpr_read_b32 %1, a209\n\tv_accvgpr_read_b32 %2, a210\n\tv_accvgpr_read_b32 %3, a211\n\tv_accvgpr_read_b32 %4, a212\n\tv_accvgpr_read_b32 %5, a213\n\tv_accvgpr_read_b32 %6, a214\n\tv_accvgpr_read_b32 %7, a215\n\tv_accvgpr_read_b32 %8, a216\n\tv_accvgpr_read_b32 %9, a217\n\tv_accvgpr_read_b32 %10, a218\n\tv_accvgpr_read_b32 %11, a219\n\tv_accvgpr_read_b32 %12, a220\n\tv_accvgpr_read_b32 %13, a221\n\tv_accvgpr_read_b32 %14, a222\n\tv_accvgpr_read_b32 %15, a223\n\t" : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3]), "=v"(r[4]), "=v"(r[5]), "=v"(r[6]), "=v"(r[7]), "=v"(r[8]), "=v"(r[9]), "=v"(r[10]), "=v"(r[11]), "=v"(r[12]), "=v"(r[13]), "=v"(r[14]), "=v"(r[15]));
  if constexpr (T == 6) asm volatile("v_accvgpr_read_b32 %0, a224\n\tv_accvgpr_read_b32 %1, a225\n\tv_accvgpr_read_b32 %2, a226\n\tv_accvgpr_read_b32 %3, a227\n\tv_accvgpr_read_b32 %4, a228\n\tv_accvgpr_read_b32 %5, a229\n\tv_accvgpr_read_b32 %6, a230\n\tv_accvgpr_read_b32 %7, a231\n\tv_accvgpr_read_b32 %8, a232\n\tv_accvgpr_read_b32 %9, a233\n\tv_accvgpr_read_b32 %10, a234\n\tv_accvgpr_read_b32 %11, a235\n\tv_accvgpr_read_b32 %12, a236\n\tv_accvgpr_read_b32 %13, a237\n\tv_accvgpr_read_b32 %14, a238\n\tv_accvgpr_read_b32 %15, a239\n\t" : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3]), "=v"(r[4]), "=v"(r[5]), "=v"(r[6]), "=v"(r[7]), "=v"(r[8]), "=v"(r[9]), "=v"(r[10]), "=v"(r[11]), "=v"(r[12]), "=v"(r[13]), "=v"(r[14]), "=v"(r[15]));
  if constexpr (T == 7) asm volatile("v_accvgpr_read_b32 %0, a240\n\tv_accvgpr_read_b32 %1, a241\n\tv_accvgpr_read_b32 %2, a242\n\tv_accvgpr_read_b32 %3, a243\n\tv_accvgpr_read_b32 %4, a244\n\tv_accvgpr_read_b32 %5, a245\n\tv_accvgpr_read_b32 %6, a246\n\tv_accvgpr_read_b32 %7, a247\n\tv_accvgpr_read_b32 %8, a248\n\tv_accvgpr_read_b32 %9, a249\n\tv_accvgpr_read_b32 %10, a250\n\tv_accvgpr_read_b32 %11, a251\n\tv_accvgpr_read_b32 %12, a252\n\tv_accvgpr_read_b32 %13, a253\n\tv_accvgpr_read_b32 %14, a254\n\tv_accvgpr_read_b32 %15, a255\n\t" : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3]), "=v"(r[4]), "=v"(r[5]), "=v"(r[6]), "=v"(r[7]), "=v"(r[8]), "=v"(r[9]), "=v"(r[10]), "=v"(r[11]), "=v"(r[12]), "=v"(r[13]), "=v"(r[14]), "=v"(r[15]));
  f32x16 v;
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = r[i];
  return v;
}
DEV_INLINE f32x16 w64_o_read_t(const int T) {
  switch (T) {
    case 0: return w64_o_read<0>();
    case 1: return w64_o_read<1>();
    case 2: return w64_o_read<2>();
    case 3: return w64_o_read<3>();
    case 4: return w64_o_read<4>();
    case 5: return w64_o_read<5>();
    case 6: return w64_o_read<6>();
    default: return w64_o_read<7>();
  }
}
#define W64_GAP() __builtin_amdgcn_sched_barrier(0)

template <int D>
__global__ __launch_bounds__(256, 1) void flash_fwd_w64_kernel(FwdArgs a) {
  static_assert(D == 128, "W64 forward: head_dim 128");
  constexpr int NCH = D / 8, DSTEPS = D / 16, DT = D / 32;
  constexpr int TILE = BK * D * 2;             // 16 KiB per K or V tile
  constexpr int NGT = TILE / 1024 / 4;         // LDS-DMA pieces per wave per tile (4)
  constexpr int RPG = 1024 / (D * 2);          // rows per piece (4)
  constexpr int HALF = 32 * D * 2;             // byte offset of rows 32-63 of a tile (same swizzle)
  __shared__ __attribute__((aligned(16))) char Qs[W64_BQ * D * 2];  // 64 KiB
  __shared__ __attribute__((aligned(16))) char Kr[3 * TILE];        // K ring, 3 slots
  __shared__ __attribute__((aligned(16))) char Vr[(2 + W64_V3) * TILE];  // V ring

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5, lr = lane & 31;
  const int S = a.S;
  const float c = a.scale_log2;
  // persistent schedule: this workgroup's n-th block.  Rounds of gridDim blocks in decode_block's order
  // (heaviest causal blocks first, the q heads of one kv head on one XCD); odd rounds run mirrored inside
  // each XCD column (low three bits kept), so the causal weights even out over the rounds
  const int total = a.nqb * a.B * a.H;
  const int G = gridDim.x;
  auto sched = [&](const int n) __attribute__((always_inline)) -> int {
    const int p = blockIdx.x;
    int pos = p;
    if (n & 1) pos = (G & 7) == 0 ? (((G >> 3) - 1 - (p >> 3)) << 3) | (p & 7) : G - 1 - p;
    return n * G + pos;
  };
  // block variables are loop-carried through the persistent loop: readfirstlane keeps them (and every DMA
  // descriptor / offset derived from them by SALU) provably wave-uniform
  auto rfl = [](const int x) __attribute__((always_inline)) { return __builtin_amdgcn_readfirstlane(x); };
  int qb, b, hq, kvh;
  decode_block(a, qb, b, hq, kvh, sched(0));
  qb = rfl(qb);
  b = rfl(b);
  hq = rfl(hq);
  kvh = rfl(kvh);
  int q0 = qb * W64_BQ, wq0 = q0 + 64 * wave;
  int ntiles = a.causal ? (q0 + W64_BQ) / BK : S / BK;
  int wtiles = a.causal ? (wq0 + 64) / BK : ntiles;
  int stamp_blk = 1;  // W64_STAMPS: the first block of the workgroup
  // W64_SEAM: the previous block's last tile, carried into this block's first body
  bool carry = false;
  int tp_ = 0, wq0p_ = 0, bp_ = 0, hqp_ = 0;
  float mp_[2] = {0.f, 0.f}, lp_[2] = {0.f, 0.f}, rsp_[2] = {0.f, 0.f};
  static_assert(!(W64_SEAM && W64_V3), "the seam body reads the carried tile's V from slot (t & 1)");
  int vslot0 = 0;  // V ring slot of this block's tile 0 (W64_V3: the V stream runs on across blocks too)
  int kslot0 = 0;  // K ring slot of this block's tile 0: the K stream runs on across blocks
  // the next block (its K(0), K(1) and Q stream in under this block's last iterations)
  int nqb_ = 0, nb_ = 0, nhq_ = 0, nkvh_ = 0;
  int has_next = 0;

  // K / V element offsets of this block's and the next block's (b, kv head), set once per block; LDS
  // destinations as plain 32-bit addresses (SALU arithmetic, no generic-pointer casts per piece)
  auto kv_of = [&](const int bb, const int kh) __attribute__((always_inline)) -> long long {
    return (long long)bb * S * a.kv_rs + (long long)kh * D;
  };
  long long kof_c = kv_of(b, kvh), kof_n = 0;
  const unsigned kr0 = lds_addr(Kr) + wave * NGT * RPG * D * 2, vr0 = lds_addr(Vr) + wave * NGT * RPG * D * 2;
  const unsigned qs0 = lds_addr(Qs) + 64 * wave * D * 2;
  int voff[NGT];
#pragma unroll
  for (int i = 0; i < NGT; ++i) {
    const int row = (wave * NGT + i) * RPG + lane / NCH, pc = lane % NCH;
    voff[i] = (row * (int)a.kv_rs + ((pc ^ swz(row)) & (NCH - 1)) * 8) * 2;
  }
  const int tstride = BK * (int)a.kv_rs * 2;  // global bytes per 64-key tile
  // LDS-DMA of K stream tile t (t >= ntiles: the next block's tile t - ntiles; past the last block a
  // harmless repeat into the slot it would have used: that slot held K(t - 3), read by nobody again)
  auto dma_k = [&](const int t, const int p) __attribute__((always_inline)) {
    const int slot = (kslot0 + t) % 3;
    const int nxt = (t >= ntiles) & has_next & W64_XB;  // integer selects (SALU), never a select of descriptors
    const int tt = t < ntiles ? t : (nxt ? t - ntiles : 0);
    lds_dma16_m0(make_rsrc(a.k + (nxt ? kof_n : kof_c)), rfl(kr0 + slot * TILE + p * RPG * D * 2), voff[p], tt * tstride);
  };
  // LDS-DMA of V stream tile t (W64_V3: as the K stream, one tile ahead of its use instead of two)
  auto dma_v = [&](const int t, const int p) __attribute__((always_inline)) {
    if (W64_V3) {
      const int nxt = (t >= ntiles) & has_next & W64_XB;
      const int tt = t < ntiles ? t : (nxt ? t - ntiles : 0);
      lds_dma16_m0(make_rsrc(a.v + (nxt ? kof_n : kof_c)), rfl(vr0 + ((vslot0 + t) % 3) * TILE + p * RPG * D * 2),
                   voff[p], tt * tstride);
    } else {
      lds_dma16_m0(make_rsrc(a.v + kof_c), rfl(vr0 + (t & 1) * TILE + p * RPG * D * 2), voff[p], t * tstride);
    }
  };
  // this wave's 64 Q rows of block (qb', b', hq') -> Qs (swizzled row image).  The lane id is re-derived per
  // call by volatile asm: hoisted as loop-invariant, the sixteen lane offsets were spilled and every reload's
  // vmcnt(0) serialised the pieces behind the whole DMA stream (0.13 ms of the kernel at the 8B shape)
  // pieces [p0, p1) of the 16 (four rows each)
  auto dma_q = [&](const int qbx, const int bx, const int hqx, const int p0, const int p1) __attribute__((always_inline)) {
    const uint16_t* qbase = a.q + ((long long)bx * S + qbx * W64_BQ + 64 * wave) * a.q_rs + (long long)hqx * D;
    const auto qrs = make_rsrc(qbase);
    int ln;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
#pragma unroll
    for (int p = p0; p < p1; ++p) {
      const int row = p * RPG + ln / NCH, pc = ln % NCH;
      const int qo = (row * (int)a.q_rs + ((pc ^ swz(row)) & (NCH - 1)) * 8) * 2;
      lds_dma16_m0(qrs, rfl(qs0 + p * RPG * D * 2), qo, 0);
    }
  };
  // prologue of the first block: Q, K(0), K(1)
  dma_q(qb, b, hq, 0, 16);
#pragma unroll
  for (int p = 0; p < NGT; ++p) dma_k(0, p);
#pragma unroll
  for (int p = 0; p < NGT; ++p) dma_k(1, p);
  if (W64_V3) {
#pragma unroll
    for (int p = 0; p < NGT; ++p) dma_v(0, p);
  }

  // lane-constant LDS offsets: K / Q fragment (row lr, chunk 2 st + hh); V^T tr-read (as flash_fwd_kernel).
  // Re-derived at every block start from a volatile-asm lane id, so they are dead across the epilogue and
  // the idle iterations (kept live there, they pushed the compiler into spilling through owned registers)
  int ko[DSTEPS], vto[DT][2];
  auto lane_offsets = [&]() __attribute__((always_inline)) {
    int ln;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
    const int lh = ln >> 5, ll = ln & 31;
#pragma unroll
    for (int st = 0; st < DSTEPS; ++st) ko[st] = lds_off<D>(ll, 2 * st + lh);
    const int gi = ln >> 4, li = ln & 15;
    const int trq = li >> 2, trp = li & 3;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int col = dt * 32 + 16 * (gi & 1) + 4 * trp;
      const int chunk = col >> 3, half8 = (col & 7) ? 8 : 0;
      vto[dt][0] = lds_off<D>(4 * lh + trq, chunk) + half8;
      vto[dt][1] = lds_off<D>(4 * lh + trq + 8, chunk) + half8;
    }
  };
  const char* Qw = Qs + 64 * wave * D * 2;
  const uint4 fake = make_uint4(0x3c003c00u ^ lane, 0x3c003c00u, 0x3c003c00u ^ (lane << 3), 0x3c003c00u);
  // K fragment (kt, st) of stream tile t / Q fragment (j, st) into their owned accumulator registers
  auto ld_k = [&](const int t, const int kt, const int st) __attribute__((always_inline)) {
    if (!W64_ABL_NOLDS) w64_lda_t(16 + 8 * kt + st, lds_addr(Kr + ((kslot0 + t) % 3) * TILE) + kt * HALF + ko[st]);
  };
  auto ld_q = [&](const int j, const int st) __attribute__((always_inline)) {
    if (!W64_ABL_NOLDS) w64_lda_t(8 * j + st, lds_addr(Qw) + j * HALF + ko[st]);
  };
  auto rd_v = [&](const int t, const int f, const int h) __attribute__((always_inline)) -> s16x4 {
    if (W64_ABL_NOLDS) return s16x4{(short)lane, (short)f, (short)h, (short)t};
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4*)(Vr + (W64_V3 ? (vslot0 + t) % 3 : (t & 1)) * TILE + vto[f >> 2][h] + (f & 3) * 16 * D * 2));
  };

  w64_o_zero();  // O: a[128:255], owned by the asm helpers above
  float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f}, alpha[2] = {1.f, 1.f}, rs[2] = {0.f, 0.f};
  bool resc = false;
  f32x16 sA[2][2], sB[2][2];  // S of the tile being started / finished (parity buffers)
  uint4 pA[2][4], pB[2][4];   // P^T fragments as packed bf16 words (parity buffers)
  // V(i-1)^T fragments (two tr-reads each), a ring of eight: fragments 0-7 read during X_i, fragments 8-15
  // during Y_i's first half into the slots fragments 0-7 free (each 14+ gaps before its MFMAs)
  s16x4 vf[8][2];

  auto sync = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's DMA pieces of the last iteration landed
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    if (!W64_ABL_NOBAR) __builtin_amdgcn_s_barrier();  // ... everyone's; every read of a slot about to be refilled is done
  };
  // a body's sync (W64_V3): the V pieces the last Y phase issued (its last NGT vector-memory operations, read
  // only in the tile after next) stay in flight; everything older -- K(i+1), V(i) -- has landed
  auto sync_body = [&]() __attribute__((always_inline)) {
    if (W64_V3) {
      static_assert(NGT == 4, "vmcnt(4) below counts the four V pieces of one Y phase");
      __builtin_amdgcn_s_waitcnt(0x0F74);  // vmcnt(4)
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      if (!W64_ABL_NOBAR) __builtin_amdgcn_s_barrier();
    } else {
      sync();
    }
  };
  auto rescale = [&]() __attribute__((always_inline)) {
    if (resc) {
      w64_o_wait();  // the last PV MFMA's result is readable
      w64_o_scale<0>(alpha[0]);
      w64_o_scale<1>(alpha[0]);
      w64_o_scale<2>(alpha[0]);
      w64_o_scale<3>(alpha[0]);
      w64_o_scale<4>(alpha[1]);
      w64_o_scale<5>(alpha[1]);
      w64_o_scale<6>(alpha[1]);
      w64_o_scale<7>(alpha[1]);
      resc = false;
    }
  };
  auto masked = [&](const float x, const int j, const int e, const int t, const bool mask, const int wq)
      __attribute__((always_inline)) -> float {
    if (!mask) return x;
    const int kt = e >> 4, i = e & 15;
    const int off = t * BK + kt * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;  // key of element (kt, i)
    return off <= wq + 32 * j + lr ? x : -INFINITY;  // wq: the first query row of the wave's block
  };
  // one exponential of element (kt, i) of block j into the packed P word; r = row-sum partial
  auto exp_el = [&](const f32x16 (&sv)[2][2], uint4 (&pw)[2][4], float (&r)[2], const int j, const int e,
                    const int t, const bool mask, const float mref, float (&ev)[2][2]) __attribute__((always_inline)) {
    const int kt = e >> 4, i = e & 15;
    const float p = W64_ABL_NOEXP ? sv[j][kt][i] : __builtin_amdgcn_exp2f(__builtin_fmaf(masked(sv[j][kt][i], j, e, t, mask, wq0), c, -mref));
    r[j] += p;
    ev[j][i & 1] = p;
    if (i & 1) {
      const uint32_t w = pack_bf2(ev[j][0], ev[j][1]);
      const int f = 2 * kt + (i >> 3), dw = (i & 7) >> 1;
      if (dw == 0) pw[j][f].x = w; else if (dw == 1) pw[j][f].y = w; else if (dw == 2) pw[j][f].z = w; else pw[j][f].w = w;
    }
  };
  // the phases' exponential pipeline: element (j, e)'s exponential in one gap, its consumers (the row-sum add,
  // the bf16 pack) in the next -- a VALU read right behind a v_exp_f32 costs a wait state (an s_nop per
  // element).  pr: the last four exponentials by i & 3 (at most two per gap, so four are live at most)
  float pr[4];
  auto exp_p = [&](const f32x16 (&sv)[2][2], const int j, const int e, const int t, const bool mask, const float mref,
                   const int wq) __attribute__((always_inline)) {
    const int kt = e >> 4, i = e & 15;
    pr[i & 3] = W64_ABL_NOEXP ? sv[j][kt][i] : __builtin_amdgcn_exp2f(__builtin_fmaf(masked(sv[j][kt][i], j, e, t, mask, wq), c, -mref));
  };
  // W64_PIN: an empty volatile asm that takes a result as "+v" keeps its computation in the gap that
  // produced it -- sched_barrier fences only the machine scheduler; without the pins the IR passes sank the
  // row-sum adds to the end of Y and a whole phase's exponentials into the next tile's X
  auto consume = [&](uint4 (&pw)[2][4], float (&r)[2], const int j, const int e) __attribute__((always_inline)) {
    const int kt = e >> 4, i = e & 15;
    r[j] += pr[i & 3];
    if (W64_PIN) asm volatile("" : "+v"(r[j]));
    if (i & 1) {
      uint32_t w = pack_bf2(pr[(i - 1) & 3], pr[i & 3]);
      if (W64_PIN) asm volatile("" : "+v"(w));
      const int f = 2 * kt + (i >> 3), dw = (i & 7) >> 1;
      if (dw == 0) pw[j][f].x = w; else if (dw == 1) pw[j][f].y = w; else if (dw == 2) pw[j][f].z = w; else pw[j][f].w = w;
    }
  };

  // ---- one iteration (tile i).  first: no finish / PV (tile 0); mask: tile i is the wave's diagonal; more:
  // the wave computes tile i + 1 (read its first K fragments in Y_i)
  auto stamp = [&](const int i, const int k) __attribute__((always_inline)) {
#if W64_STAMPS
    if (blockIdx.x == 0 && stamp_blk && i >= 20 && i < 24) {
      W64_GAP();
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (lane == 0) w64_stamps[wave][i - 20][k] = t;
      W64_GAP();
    }
#endif
  };
  auto bstamp = [&](const int n, const int k) __attribute__((always_inline)) {
#if W64_STAMPS
    if (blockIdx.x == 0 && n < 8) {
      W64_GAP();
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (lane == 0) w64_bstamps[n][wave][k] = t;
      W64_GAP();
    }
#endif
  };
  // fin: the tile being finished and PV'd (not first): tile tp of the block whose first query row (this
  // wave's) is wqp, under the causal diagonal mask maskp, with that block's row statistics mf / lf / rsf --
  // the previous tile of this block (tp = i - 1, no mask, m / l / rs), or, in a seam body (W64_SEAM), the
  // last tile of the previous block; q0b: the block's body 0 (issues the next block's Q)
  auto body = [&](const int i, f32x16 (&sn)[2][2], f32x16 (&so)[2][2], uint4 (&pn)[2][4], uint4 (&po)[2][4],
                  const bool first, const bool mask, const bool more, const int tp, const int wqp, const bool maskp,
                  const float (&mf)[2], float (&lf)[2], const float (&rsf)[2], const bool q0b)
      __attribute__((always_inline)) {
    stamp(i, 0);
    sync_body();
    stamp(i, 1);
    rescale();
    stamp(i, 2);
    float mref_o[2], r[2] = {rsf[0], rsf[1]};
#pragma unroll
    for (int j = 0; j < 2; ++j) mref_o[j] = (mf[j] == -INFINITY) ? 0.f : mf[j];
    float mt[2] = {-INFINITY, -INFINITY}, mref_n[2] = {0.f, 0.f};
    bool need_any = false;
    // row statistics of block jj for tile i (l is rescaled where its tile i - 1 sum is complete)
    auto stats = [&](const int jj) __attribute__((always_inline)) {
      const bool need = mt[jj] > m[jj] + W64_DEFER;
      const float mn = need ? fmaxf(m[jj], mt[jj]) : m[jj];
      alpha[jj] = __builtin_amdgcn_exp2f(m[jj] - ((mn == -INFINITY) ? 0.f : mn));
      m[jj] = mn;
      mref_n[jj] = (mn == -INFINITY) ? 0.f : mn;
      need_any |= need;
    };
    auto rowmax4 = [&](const int jj, const int e0) __attribute__((always_inline)) {
#pragma unroll
      for (int e = e0; e < e0 + 4; ++e) mt[jj] = fmaxf(mt[jj], masked(sn[jj][e >> 4][e & 15], jj, e, i, mask, wq0));
      if (W64_PIN) asm volatile("" : "+v"(mt[jj]));
    };
    // ---------------- X_i: S(i) block-major (block 0's chains complete at gap 15, so its row maximum and
    // statistics run in gaps 19-28 and Y_i can exponentiate from its first gap: one exponential per gap in
    // both phases)
    W64_GAP();
#pragma unroll
    for (int gq = 0; gq < 8; ++gq)
#pragma unroll
    for (int gu = 0; gu < 4; ++gu) {
      const int g = 4 * gq + gu;
      const int j = g >> 4, st = (g & 15) >> 1, kt = g & 1;
      w64_s_t(kt, st, j, sn[j][kt]);  // operands K(i), Q in owned accumulator registers
      // V^T fragments 0-7, one read per gap in gaps 8-23 (after the DMA gaps, landed well before the seam)
      if (!first && g >= 8 && g < 24) vf[(g - 8) >> 1][g & 1] = rd_v(tp, (g - 8) >> 1, g & 1);
      if (!first) {
        exp_p(so, g >> 4, 16 + (g & 15), tp, maskp, mref_o[g >> 4], wqp);
        if (g > 0) consume(po, r, (g - 1) >> 4, 16 + ((g - 1) & 15));
      }
      if (W64_ABL_NODMA) {
      } else if (W64_V3 ? (g < 2 * NGT && !(g & 1)) : g < NGT) {
        dma_k(i + 2, W64_V3 ? g >> 1 : g);
      } else if (!W64_V3 && g < 2 * NGT) {
        dma_v(i, g - NGT);
      }
      if (first && g == 19) {  // tile 0's gaps carry no fillers
        asm volatile("s_nop 7\n\ts_nop 3" ::: "memory");
        W64_GAP();
      }
      if (g >= 19 && g < 27) rowmax4(0, 4 * (g - 19));
      if (g == 27) mt[0] = xhalf_max(mt[0]) * c;
      if (g == 28) stats(0);
      W64_GAP();
    }
    if (!first) {
      consume(po, r, 1, 31);
      lf[0] += r[0];
      lf[1] += r[1];
    }
    l[0] *= alpha[0];
    stamp(i, 3);
    // seam: every V^T fragment landed (a compiler-known wait: no further waits in Y_i); then K(i+1) a phase
    // ahead (landed two tiles ahead), all sixteen reads issued before any of the compiler's LDS reads of Y_i --
    // LDS returns in order, so the compiler's lgkmcnt waits (which do not count these asm reads) are neither
    // short nor inflated by them -- and they are the wait states between the last asm S MFMAs and the
    // softmax's VALU reads of their (VGPR) results (nops when there is no next tile)
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if (more) {
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) ld_k(i + 1, kk >> 3, kk & 7);
    } else {
      asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    }
    W64_GAP();
    stamp(i, 4);
    // ---------------- Y_i
    r[0] = r[1] = 0.f;
#pragma unroll
    for (int f = 0; f < 16; ++f) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int g = 2 * f + j;
        if (!first) {
          const s16x4 v1 = vf[f & 7][0], v2 = vf[f & 7][1];
          const s16x8 va = {v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
          w64_pv_t(4 * j + (f >> 2), __builtin_bit_cast(bf16x8, va), as_bf8(po[j][f & 3]));
        }
        // after this gap's MFMA: fragment 8 + k into the slot fragment k freed (gaps 2-17)
        if (!first && g >= 2 && g < 18) {
          const int fr = 8 + ((g - 2) >> 1), h = (g - 2) & 1;
          vf[fr & 7][h] = rd_v(tp, fr, h);
        }
        // W64_V3: V(i+1) by LDS-DMA in the LDS-read-free gaps 22, 24, 26, 28 (its slot held V(i-2), whose last
        // reads were Y_{i-1}'s); waited two syncs later (sync_body)
        if (W64_V3 && !W64_ABL_NODMA && g >= 22 && g < 22 + 2 * NGT && !(g & 1)) dma_v(i + 1, (g - 22) >> 1);
        // W64_QEARLY: the next block's Q by LDS-DMA in the first body's Y (no PV there; this wave's Q rows were
        // read at block start; before the V pieces, so the counted body sync still leaves only V in flight) --
        // off the last wave's critical tail
        if (W64_QEARLY && W64_XB && !W64_ABL_NODMA && q0b && g >= 2 && g < 18 && has_next)
          dma_q(nqb_, nb_, nhq_, g - 2, g - 1);
        // start softmax(i): block 0's keys 0-31 exponentiated in gaps 0-15; block 1's row maximum in gaps 0-7,
        // its statistics in 8-9, its exponentials in 16-31 (consumers one gap behind)
        if (g < 8) rowmax4(1, 4 * g);
        if (g == 8) mt[1] = xhalf_max(mt[1]) * c;
        if (g == 9) {
          stats(1);
          l[1] *= alpha[1];
        }
        exp_p(sn, g >> 4, g & 15, i, mask, mref_n[g >> 4], wq0);
        if (g > 0) consume(pn, r, (g - 1) >> 4, (g - 1) & 15);
        W64_GAP();
      }
    }
    consume(pn, r, 1, 15);
    stamp(i, 5);
    rs[0] = r[0];
    rs[1] = r[1];
    resc = __builtin_amdgcn_ballot_w64(need_any) != 0;
  };
  auto tail = [&](const int i, f32x16 (&so)[2][2], uint4 (&po)[2][4], const bool mask) __attribute__((always_inline)) {
    sync_body();  // V(i) (the last Y's pieces) is read only in the next block or never
    rescale();
#pragma unroll
    for (int p = 0; p < NGT; ++p) dma_k(i + 2, p);
    if (W64_V3 || i < ntiles) {
#pragma unroll
      for (int p = 0; p < NGT; ++p) dma_v(i + W64_V3, p);
    }
    // the next block's Q pieces its bodies 1-4 did not issue (this wave's Q rows were read at block start only)
    if (has_next && W64_XB) {
      if (!W64_QEARLY) dma_q(nqb_, nb_, nhq_, 0, 16);
    }
    float r[2] = {rs[0], rs[1]}, ev[2][2];
#pragma unroll
    for (int jo = 0; jo < 2; ++jo) {
      const int j = W64_TAIL_J1FIRST ? 1 - jo : jo;
      const float mref = (m[j] == -INFINITY) ? 0.f : m[j];
#pragma unroll
      for (int e = 16; e < 32; ++e) exp_el(so, po, r, j, e, i - 1, mask, mref, ev);
      l[j] += r[j];
    }
    if (W64_TAIL_NOP) {
      W64_GAP();
      asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
      W64_GAP();
    }
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      vf[f][0] = rd_v(i - 1, f, 0);
      vf[f][1] = rd_v(i - 1, f, 1);
    }
#pragma unroll
    for (int f = 0; f < 16; ++f) {
      W64_GAP();
      if (f >= 1 && f + 7 < 16) {  // fragment f + 7 into the slot fragment f - 1 freed
        vf[(f + 7) & 7][0] = rd_v(i - 1, f + 7, 0);
        vf[(f + 7) & 7][1] = rd_v(i - 1, f + 7, 1);
      }
      const s16x4 v1 = vf[f & 7][0], v2 = vf[f & 7][1];
      const s16x8 va = {v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
      w64_pv_t(f >> 2, __builtin_bit_cast(bf16x8, va), as_bf8(po[0][f & 3]));
      w64_pv_t(4 + (f >> 2), __builtin_bit_cast(bf16x8, va), as_bf8(po[1][f & 3]));
    }
  };

  // O / LSE of the wave's rows of block (bb, hqq) whose first row is wq, with its statistics mm / ll
  auto epilogue = [&](const float (&mm)[2], const float (&ll)[2], const int wq, const int bb, const int hqq)
      __attribute__((always_inline)) {
    w64_o_wait();  // the last PV MFMA's result is readable
  #pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int qrow = wq + 32 * j + lr;
      const float ltot = ll[j] + __shfl_xor(ll[j], 32, 64);
      const float inv = ltot > 0.f ? 1.0f / ltot : 0.f;
      uint16_t* op = a.o + ((long long)bb * S + qrow) * a.o_rs + (long long)hqq * D;
  #pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const f32x16 ov = w64_o_read_t(4 * j + dt);
        uint32_t w[4][2];
  #pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          w[g4][0] = pack_bf2(ov[4 * g4 + 0] * inv, ov[4 * g4 + 1] * inv);
          w[g4][1] = pack_bf2(ov[4 * g4 + 2] * inv, ov[4 * g4 + 3] * inv);
        }
        const auto a0 = __builtin_amdgcn_permlane32_swap(w[0][0], w[2][0], false, false);
        const auto a1 = __builtin_amdgcn_permlane32_swap(w[0][1], w[2][1], false, false);
        const auto b0 = __builtin_amdgcn_permlane32_swap(w[1][0], w[3][0], false, false);
        const auto b1 = __builtin_amdgcn_permlane32_swap(w[1][1], w[3][1], false, false);
        const int d = dt * 32 + 16 * hh;
        *reinterpret_cast<uint4*>(op + d) = make_uint4(a0[0], a1[0], a0[1], a1[1]);
        *reinterpret_cast<uint4*>(op + d + 8) = make_uint4(b0[0], b1[0], b0[1], b1[1]);
      }
      if (hh == 0) {
        const float lse2 = (mm[j] == -INFINITY) ? -INFINITY : mm[j] + __log2f(ltot);
        a.lse[((long long)bb * a.H + hqq) * S + qrow] = lse2 * LN2;
      }
    }
  };

  for (int n = 0;; ++n) {
    {  // the next block of this workgroup, if any
      const int nx = sched(n + 1);
      has_next = rfl(nx < total ? 1 : 0);
      if (has_next) {
        decode_block(a, nqb_, nb_, nhq_, nkvh_, nx);
        nqb_ = rfl(nqb_);
        nb_ = rfl(nb_);
        nhq_ = rfl(nhq_);
        nkvh_ = rfl(nkvh_);
        kof_n = kv_of(nb_, nkvh_);
      }
    }
    // block start: Q, K(0), K(1) landed; X_0's first K / Q fragments
    bstamp(n, 0);
    lane_offsets();
    if (!W64_XB && n > 0) {
      sync();  // every read of the Q rows and K slots of the last block is done
      dma_q(qb, b, hq, 0, 16);
#pragma unroll
      for (int p = 0; p < NGT; ++p) dma_k(0, p);
#pragma unroll
      for (int p = 0; p < NGT; ++p) dma_k(1, p);
      if (W64_V3) {
#pragma unroll
        for (int p = 0; p < NGT; ++p) dma_v(0, p);
      }
    }
    sync();
#pragma unroll
    for (int st = 0; st < DSTEPS; ++st) {
      ld_q(0, st);
      ld_q(1, st);
      ld_k(0, 0, st);
      ld_k(0, 1, st);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // the asm loads above (the compiler does not count them)
    bstamp(n, 1);
    if (carry) {
      // seam body: S(0) of this block while the last tile of the previous block is finished and PV'd; that
      // block's O is complete after it and stored here, before this block's first PV (body 1)
      body(0, sA, sB, pA, pB, false, a.causal && wtiles == 1, wtiles > 1, tp_, wq0p_, a.causal != 0, mp_, lp_, rsp_,
           true);
      epilogue(mp_, lp_, wq0p_, bp_, hqp_);
      w64_o_zero();
      carry = false;
    } else {
      body(0, sA, sB, pA, pB, true, a.causal && wtiles == 1, wtiles > 1, -1, wq0, false, m, l, rs, true);
    }
    int i = 1;
    // steady iterations 1 .. wtiles - 2 in parity pairs; the state is back in (sA, pA) after each pair
    for (; i + 2 < wtiles; i += 2) {
      body(i, sB, sA, pB, pA, false, false, true, i - 1, wq0, false, m, l, rs, false);
      body(i + 1, sA, sB, pA, pB, false, false, true, i, wq0, false, m, l, rs, false);
    }
    if (i + 1 < wtiles) {  // one more steady iteration (odd i); then the state moves back to (sA, pA)
      body(i, sB, sA, pB, pA, false, false, true, i - 1, wq0, false, m, l, rs, false);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        sA[j][1] = sB[j][1];
        pA[j][0] = pB[j][0];
        pA[j][1] = pB[j][1];
      }
      ++i;
    }
    // W64_SEAM with a next block: the wave whose rows run to the block's last tile (every wave without the causal
    // mask, the last one with it) hands that tile to the next block's first body instead of a tail here, and
    // the block loses its step ntiles (its DMA -- the next block's K(2) -- is re-issued by that body anyway)
    const bool seam_blk = W64_SEAM && has_next;
    const bool carry_now = seam_blk && wtiles == ntiles;
    if (i < wtiles) {  // the wave's last tile: the diagonal under the causal mask
      body(i, sB, sA, pB, pA, false, a.causal != 0, false, i - 1, wq0, false, m, l, rs, false);
      ++i;
      bstamp(n, 2);
      if (!carry_now) tail(i, sB, pB, a.causal != 0);
    } else {  // wtiles == 1
      bstamp(n, 2);
      tail(i, sA, pA, a.causal != 0);
    }
    bstamp(n, 3);
    if (carry_now) {
      tp_ = wtiles - 1;
      wq0p_ = wq0;
      bp_ = b;
      hqp_ = hq;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        mp_[j] = m[j];
        lp_[j] = l[j];
        rsp_[j] = rs[j];
        m[j] = -INFINITY;  // alpha / resc stay: the seam body rescales the carried O first
        l[j] = 0.f;
        rs[j] = 0.f;
      }
      carry = true;
    } else {
      // this wave's rows are done: store them now, under the other waves' remaining tiles
      epilogue(m, l, wq0, b, hq);
      w64_o_zero();
      m[0] = m[1] = -INFINITY;
      l[0] = l[1] = 0.f;
      rs[0] = rs[1] = 0.f;
      alpha[0] = alpha[1] = 1.f;
      resc = false;
    }
    bstamp(n, 4);
    // waves whose rows ended keep joining the workgroup's DMA / barriers
    for (++i; i <= ntiles - (seam_blk ? 1 : 0); ++i) {
      sync();
#pragma unroll
      for (int p = 0; p < NGT; ++p) dma_k(i + 2, p);
      if (W64_V3 || i < ntiles) {
#pragma unroll
        for (int p = 0; p < NGT; ++p) dma_v(i + W64_V3, p);
      }
    }
    bstamp(n, 5);
    if (!has_next) break;
    stamp_blk = 0;
    kslot0 = rfl((kslot0 + ntiles) % 3);
    vslot0 = rfl((vslot0 + ntiles) % 3);
    qb = nqb_;
    b = nb_;
    hq = nhq_;
    kvh = nkvh_;
    kof_c = kof_n;
    q0 = qb * W64_BQ;
    wq0 = q0 + 64 * wave;
    ntiles = rfl(a.causal ? (q0 + W64_BQ) / BK : S / BK);
    wtiles = rfl(a.causal ? (wq0 + 64) / BK : ntiles);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // no LDS-DMA may outlive the workgroup

}
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
