// Lab kernel (VERDICT r4 "Next" 1a): the projection GEMM C[M, N] = alpha A[M, K] . B[N, K]^T as an 8-wave
// PING-PONG on the 256 x 256 tile -- two waves per SIMD, one in a pure-MFMA compute phase while its
// partner reads its next fragments and issues its share of the operand DMA, swapped at every s_barrier.
//
//   waves: w = 4 g + s; group g = w >> 2 owns rows [128 g, +128) of the tile, s owns columns [64 s, +64);
//          waves w and w + 4 share a SIMD (dispatch order; correctness never depends on it).
//   wave tile 128 x 64 = 8 x 4 accumulators of v_mfma_f32_16x16x32_bf16 (128 registers), ONE fragment
//          set (8 A + 4 B = 48 VGPRs): a wave's load phase fills it, its next compute phase consumes it.
//   phases (one barrier each), stage t = 64 deep, h = 32-deep half:
//          P0: G0 computes (t, h0) | G1 reads (t, h0), DMA A_hi(t+1)
//          P1: G1 computes (t, h0) | G0 reads (t, h1), DMA B_lo(t+2)
//          P2: G0 computes (t, h1) | G1 reads (t, h1), DMA B_hi(t+2)
//          P3: G1 computes (t, h1) | G0 reads (t+1, h0), DMA A_lo(t+2)
//   LDS: a ring of 5 slots of 32 KiB (one operand of one stage, [256 rows][64 k] bf16, 128-byte rows,
//          16-byte chunk c of row r at c ^ f5(r)); stage g: B in slot 2g mod 5, A in slot 2g+1 mod 5.  Every
//          DMA job then has >= 3 phases to land: B(t+2) goes into stage t-1's A slot (free from P3 of t-1),
//          A(t+2) into stage t's B slot (free from P3 of t), A_hi(t+1) into stage t-1's B slot.
//   waits: G0 vmcnt(4) at the end of P2 (B_lo(t+1), A_lo(t+1) landed; B_lo(t+2) flies on); G1 vmcnt(8)
//          at the end of P2 (B_hi(t+1)) and vmcnt(4) at the end of P3 (A_hi(t+1)).  Epilogue stores are
//          issued BEFORE the phase's DMA pieces, so the same counted waits cover them.
//   persistent grid: one workgroup per CU walking tiles lw + i G, the stage stream running across tiles
//          (stages past the end re-load the last one into a slot nobody reads again).
#include "common.h"

using namespace ftc;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#ifndef PPM
#define PPM 0  // lab ablations (wrong results, timing only): 1 no loop DMA / waits, 2 + no loop reads, 3 no waits
#endif
constexpr bool kLoopDma = PPM == 0 || PPM == 3, kLoopRead = PPM != 2, kLoopWait = PPM == 0;
// where a wave's 4 DMA pieces per load phase go: 0 after its fragment reads, 1 before them, 2 two before
// them + two inside its next compute phase, 3 all four inside its next compute phase (spread over the MFMAs)
#ifndef DMAP
#define DMAP 0
#endif
constexpr int kLoadPieces = DMAP == 2 ? 2 : DMAP == 3 ? 0 : 4;  // pieces issued in the load phase
constexpr int kG1P2Wait = DMAP == 2 ? 6 : DMAP == 3 ? 4 : 8;     // G1's count at the end of P2
constexpr int BM = 256, BN = 256, BK = 64;
constexpr int SLOT = 256 * BK * 2;  // 32 KiB
constexpr int NSLOT = 5;

struct PPArgs {
  const uint16_t* a;
  const uint16_t* b;
  uint16_t* c;
  long long lda, ldb, ldc;
  int K, nm, nn, group, xcc;
  float alpha;
};

DEV_INLINE int f5(int r) { return (r & 1) | (r & 2) | ((r >> 1) & 4); }

DEV_INLINE void tile_of(const PPArgs& p, int l, int& mb, int& nb) {
  const bool mfast = p.group > 0;
  const int g = mfast ? p.group : -p.group;
  const int nf = mfast ? p.nm : p.nn, ns = mfast ? p.nn : p.nm;
  const int grp = l / (g * ns), first = grp * g, gsz = min(nf - first, g);
  const int rem = l - grp * g * ns;
  const int f = first + rem % gsz, sl = rem / gsz;
  mb = mfast ? f : sl;
  nb = mfast ? sl : f;
}

DEV_INLINE int xmap(int w, int xcc) {
  const int run = 8 * xcc, within = w & (run - 1);
  return (w - within) + (within & 7) * xcc + (within >> 3);
}

DEV_INLINE bf16x8 rd(const char* s, int off) { return *reinterpret_cast<const bf16x8*>(s + off); }

DEV_INLINE void barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}
DEV_INLINE void lgkm0() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_sched_barrier(0);
}
template <int N>
DEV_INLINE void vmcnt() {
  static_assert(N < 16, "vmcnt field");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(0x0F70 | N);
  __builtin_amdgcn_sched_barrier(0);
}

// DMA cursor over the global stage stream (clamped to the last stage)
struct Cursor {
  int g, s, i;
  const uint16_t* pa;
  const uint16_t* pb;
};

#define PP_CAT2(a, b) a##b
#define PP_CAT(a, b) PP_CAT2(a, b)
#define PP_KERNEL PP_CAT(PP_CAT(gemm_pp_kernel_m, PPM), PP_CAT(_d, DMAP))
__global__ __launch_bounds__(512, 1) void PP_KERNEL(PPArgs p) {
  __shared__ __attribute__((aligned(16))) char S[NSLOT * SLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, ws = wave & 3;
  const int G = gridDim.x, ntiles = p.nm * p.nn;
  const int lw = xmap(blockIdx.x, p.xcc);
  const int my = lw < ntiles ? (ntiles - lw + G - 1) / G : 0;
  if (my == 0) return;
  const int ns = p.K / BK;
  const int total = my * ns;

  auto bases = [&](int i, const uint16_t*& ta, const uint16_t*& tb) __attribute__((always_inline)) {
    int mb, nb;
    tile_of(p, lw + i * G, mb, nb);
    mb = __builtin_amdgcn_readfirstlane(mb);
    nb = __builtin_amdgcn_readfirstlane(nb);
    ta = p.a + (long long)mb * BM * p.lda;
    tb = p.b + (long long)nb * BN * p.ldb;
  };
  auto cur_init = [&](Cursor& c, int g0) __attribute__((always_inline)) {
    c.g = min(g0, total - 1);
    c.i = c.g / ns;
    c.s = c.g - c.i * ns;
    bases(c.i, c.pa, c.pb);
    c.pa += c.s * BK;
    c.pb += c.s * BK;
  };
  auto cur_adv = [&](Cursor& c) __attribute__((always_inline)) {
    if (c.g + 1 < total) {
      ++c.g;
      if (++c.s == ns) {
        c.s = 0;
        ++c.i;
        bases(c.i, c.pa, c.pb);
      } else {
        c.pa += BK;
        c.pb += BK;
      }
    }
  };

  // per-lane DMA source offsets: piece j of a wave's 4 = rows 32 ws + 8 j + (lane >> 3) of a job's 128; the
  // chunk swizzle f5 sees row bits 0-1 (lane >> 3) and bit 3 (j & 1)
  int voa[2], vob[2];
  {
    const int rr = lane >> 3, pc = lane & 7;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int lc = pc ^ f5(rr + 8 * q);
      voa[q] = (int)((rr * p.lda + 8 * lc) * 2);
      vob[q] = (int)((rr * p.ldb + 8 * lc) * 2);
    }
  }
  const unsigned lds_base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)S;
  // one job share: 4 pieces (8 rows x 128 B each) of rows [row0 + 32 ws, +32) of operand A (op 0) or B
  // (op 1) of cursor c's stage, into slot `slot`
  // one job share: 4 pieces (8 rows x 128 B each) of rows [row0 + 32 ws, +32) of operand A (op 0) or B
  // (op 1) of cursor c's stage, into slot `slot`; described first (jobd), issued later (pieces j0..j1-1)
  struct JobD {
    __amdgpu_buffer_rsrc_t rs;
    int s0, st, v0, v1;
    unsigned dst;
  };
  auto jobd = [&](const Cursor& c, int op, int row0, int slot) __attribute__((always_inline)) {
    const long long ld = op == 0 ? p.lda : p.ldb;
    const int r0 = row0 + 32 * ws;
    JobD d;
    d.rs = make_rsrc(op == 0 ? c.pa : c.pb);
    d.s0 = (int)(r0 * ld * 2);
    d.st = (int)(8 * ld * 2);
    d.v0 = op == 0 ? voa[0] : vob[0];
    d.v1 = op == 0 ? voa[1] : vob[1];
    d.dst = lds_base + (unsigned)(slot * SLOT + r0 * 128);
    return d;
  };
  auto piece = [&](const JobD& d, int j) __attribute__((always_inline)) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %3, %4 offen sc0 lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"((j & 1) ? d.v1 : d.v0), "s"(d.dst + 1024u * j), "s"(d.rs), "s"(d.s0 + j * d.st)
        : "memory");
  };
  auto job = [&](const Cursor& c, int op, int row0, int slot) __attribute__((always_inline)) {
    const JobD d = jobd(c, op, row0, slot);
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %4, %5 offen sc0 lds\n\t"
        "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %2, %4, %6 offen sc0 lds\n\t"
        "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %4, %7 offen sc0 lds\n\t"
        "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %2, %4, %8 offen sc0 lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(d.v0), "v"(d.v1), "s"(d.dst), "s"(d.rs), "s"(d.s0), "s"(d.s0 + d.st), "s"(d.s0 + 2 * d.st),
          "s"(d.s0 + 3 * d.st)
        : "memory");
  };

  // the lane index behind an opaque statement: the per-lane fragment / epilogue offsets are recomputed
  // where they are used (a few VALU per phase) instead of being hoisted out of the loops and spilled
  auto opaque_lane = []() __attribute__((always_inline)) {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
  };
  auto bnt = [](int nt) { return (32 * (nt >> 1) + 4 * (nt & 1)) * 128; };
  auto slotB = [](int g) { return (2 * g) % NSLOT; };
  auto slotA = [](int g) { return (2 * g + 1) % NSLOT; };

  f32x4 acc[8][4];
  bf16x8 fa[8], fb[4];

  // fragments of stage g, K-half h: A rows 128 grp + 16 mt + li, B rows 64 ws + bnt(nt) + 8 (li >> 2) + (li & 3)
  // (so that lane holds columns n = 64 ws + 32 (nt >> 1) + 8 kc + 4 (nt & 1) + r), chunk (4 h + kc) ^ f5(row)
  auto read = [&](int g, int h) __attribute__((always_inline)) {
    const int l = opaque_lane(), li = l & 15, kc = l >> 4;
    const int rb = 64 * ws + 8 * (li >> 2) + (li & 3);
    const int ao = (128 * grp + li) * 128 + 16 * ((4 * h + kc) ^ f5(li));
    const int bo = rb * 128 + 16 * ((4 * h + kc) ^ f5(rb));
    const char* A = S + slotA(g) * SLOT + ao;
    const char* B = S + slotB(g) * SLOT + bo;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) fb[nt] = rd(B, bnt(nt));
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) fa[mt] = rd(A, mt * 2048);
  };
  // one 32-deep half of the wave's 128 x 64 block: 32 MFMAs, B fragment outer (src0 constant per group of 8)
  auto compute = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int mt = 0; mt < 8; ++mt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[nt], fa[mt], acc[mt][nt], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // the same 32 MFMAs with n pieces of a deferred job (j0 ..) spread over them
  auto compute_dma = [&](const JobD& d, int j0, int n) __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) {
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[nt], fa[mt], acc[mt][nt], 0, 0, 0);
        const int idx = nt * 8 + mt;
        if (n > 0 && idx % (32 / (n > 0 ? n : 1)) == 16 / (n > 0 ? n : 1) - 1) {
          __builtin_amdgcn_sched_barrier(0);
          if (kLoopDma) piece(d, j0 + idx / (32 / n));
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    __builtin_amdgcn_s_setprio(0);
  };
  // a new tile: clear the accumulators in a load phase (128 v_mov once per tile; ONE loop body keeps the
  // accumulators in one register assignment -- separate first-stage bodies made hipcc shuffle and spill them)
  // (the zero is opaque: a known-zero accumulator lets hipcc peel the first iteration into a zero-C
  // MFMA copy with its own register assignment, which spilled)
  auto clear = [&]() __attribute__((always_inline)) {
    float z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
#pragma unroll
    for (int mt = 0; mt < 8; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = f32x4{z, z, z, z};
  };
  // lane holds C[128 grp + 16 mt + li][64 ws + 32 pr + 8 kc + 0..7] in acc[mt][2 pr] (+0..3), acc[mt][2 pr + 1]
  // (+4..7): one 16-byte buffer store per (mt, pr), the wave's C block as the buffer base (SGPRs), the row /
  // pair as the scalar offset
  auto store = [&](int ti) __attribute__((always_inline)) {
    int mb, nb;
    tile_of(p, lw + ti * G, mb, nb);
    mb = __builtin_amdgcn_readfirstlane(mb);
    nb = __builtin_amdgcn_readfirstlane(nb);
    const auto rc = make_rsrc(p.c + ((long long)mb * BM + 128 * grp) * p.ldc + (long long)nb * BN + 64 * ws);
    const int l = opaque_lane(), li = l & 15, kc = l >> 4;
    const int vo = (int)((li * p.ldc + 8 * kc) * 2);
#pragma unroll
    for (int mt = 0; mt < 8; ++mt)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = p.alpha * acc[mt][2 * pr][j];
          v[4 + j] = p.alpha * acc[mt][2 * pr + 1][j];
        }
        const uint4 q = pack8(v);
        // inline asm: a compiler-visible store made hipcc drain every in-flight DMA (vmcnt(0)) before the
        // next DMA statement of EVERY iteration (its waitcnt merge at the loop join); the counted waits
        // of the loop cover these stores (issued before the phase's pieces)
        // (s_nop 1: a VALU may not overwrite a >8-byte store's data VGPRs in the next wait state -- hipcc
        // pads its own stores, never an asm statement)
        asm volatile("buffer_store_dwordx4 %0, %1, %2, %3 offen\n\ts_nop 1" ::"v"(u32x4{q.x, q.y, q.z, q.w}), "v"(vo), "s"(rc),
                     "s"((int)((16 * mt * p.ldc + 32 * pr) * 2))
                     : "memory");
      }
  };

  Cursor c1, c2;  // stages t + 1 and t + 2 (clamped)
  // prologue: stage 0 complete, stage 1 except A_hi (G1 issues that in P0 of stage 0); all landed
  {
    Cursor c0;
    cur_init(c0, 0);
    cur_init(c1, 1);
    if (grp == 0) {
      job(c0, 1, 0, slotB(0));
      job(c0, 0, 0, slotA(0));
      job(c1, 1, 0, slotB(1));
      job(c1, 0, 0, slotA(1));
    } else {
      job(c0, 1, 128, slotB(0));
      job(c0, 0, 128, slotA(0));
      job(c1, 1, 128, slotB(1));
    }
    cur_init(c2, 2);
    vmcnt<0>();
    barrier();
    if (grp == 0) read(0, 0);
    lgkm0();
    barrier();
  }

  clear();
  constexpr int kDef = 4 - kLoadPieces;  // pieces deferred into the next compute phase
  auto load_pieces = [&](const JobD& d) __attribute__((always_inline)) {
    if (!kLoopDma) return;
#pragma unroll
    for (int j = 0; j < kLoadPieces; ++j) piece(d, j);
  };
  if (grp == 0) {
    int s = 0, ti = 0;
    JobD dA = jobd(c2, 0, 0, slotA(1));  // (no deferred pieces before stage 0: the prologue loaded stage 1)
    for (int t = 0; t < total; ++t) {
      if (kDef > 0 && t > 0) compute_dma(dA, kLoadPieces, kDef);  // P0: (t, h0)
      else compute();
      barrier();
      const JobD dB = jobd(c2, 1, 0, slotB(t + 2));  // P1
      if (DMAP == 0) {
        if (kLoopRead) read(t, 1);
        if (kLoopDma) job(c2, 1, 0, slotB(t + 2));
      } else {
        load_pieces(dB);
        if (kLoopRead) read(t, 1);
      }
      lgkm0();
      barrier();
      if (kDef > 0) compute_dma(dB, kLoadPieces, kDef);  // P2: (t, h1)
      else compute();
      if (kLoopWait) vmcnt<4>();
      barrier();
      if (s == ns - 1) {                     // P3
        store(ti);
        clear();
        s = 0;
        ++ti;
      } else {
        ++s;
      }
      dA = jobd(c2, 0, 0, slotA(t + 2));
      if (DMAP == 0) {
        if (kLoopRead && t + 1 < total) read(t + 1, 0);
        if (kLoopDma) job(c2, 0, 0, slotA(t + 2));
      } else {
        load_pieces(dA);
        if (kLoopRead && t + 1 < total) read(t + 1, 0);
      }
      lgkm0();
      barrier();
      cur_adv(c1);
      cur_adv(c2);
    }
  } else {
    int s = 0, ti = 0, pend = 0;  // pend: a finished tile's accumulators await their store
    // one extra pass after the last stage runs only the last tile's store: every store of the accumulators
    // stays inside the loop (a store after the loop made hipcc re-assign and spill them at the exit)
    for (int t = 0;; ++t) {
      asm volatile("" : "+v"(pend));         // opaque: no peeled first iteration (it spilled)
      pend = __builtin_amdgcn_readfirstlane(pend);
      if (pend) {                            // P0
        pend = 0;
        store(ti - 1);
        clear();
      }
      if (t == total) break;
      const JobD dA = jobd(c1, 0, 128, slotA(t + 1));
      if (DMAP == 0) {
        if (kLoopRead) read(t, 0);
        if (kLoopDma) job(c1, 0, 128, slotA(t + 1));
      } else {
        load_pieces(dA);
        if (kLoopRead) read(t, 0);
      }
      lgkm0();
      barrier();
      if (kDef > 0) compute_dma(dA, kLoadPieces, kDef);  // P1: (t, h0)
      else compute();
      barrier();
      const JobD dB = jobd(c2, 1, 128, slotB(t + 2));  // P2
      if (DMAP == 0) {
        if (kLoopRead) read(t, 1);
        if (kLoopDma) job(c2, 1, 128, slotB(t + 2));
      } else {
        load_pieces(dB);
        if (kLoopRead) read(t, 1);
      }
      lgkm0();
      if (kLoopWait) vmcnt<kG1P2Wait>();
      barrier();
      if (kDef > 0) compute_dma(dB, kLoadPieces, kDef);  // P3: (t, h1)
      else compute();
      if (kLoopWait) vmcnt<4>();
      barrier();
      cur_adv(c1);
      cur_adv(c2);
      if (++s == ns) {
        s = 0;
        ++ti;
        pend = 1;
      }
    }
  }
  vmcnt<0>();  // no LDS-DMA may outlive the workgroup
}

int num_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

}  // namespace

// bf16 C[M, N] (ldc) = alpha A B^T; A [M, K] (lda), B [N, K] (ldb) bf16, K contiguous.  -1: outside the contract.
extern "C" int ftc_gemm_pp(const void* a, long long lda, const void* b, long long ldb, void* c, long long ldc, int M,
                           int N, int K, float alpha, int grid_cap, int group, int xcc, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || M % BM || N % BN || K % BK) return -1;
  if (lda % 8 || ldb % 8 || ldc % 8 || lda < K || ldb < K || ldc < N) return -1;
  if ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) | reinterpret_cast<uintptr_t>(c)) & 15) return -1;
  if ((long long)(BM - 1) * (lda > ldb ? lda : ldb) * 2 + 2 * BK * 2 >= (1LL << 31)) return -1;
  PPArgs p{(const uint16_t*)a, (const uint16_t*)b, (uint16_t*)c, lda, ldb, ldc, K, M / BM, N / BN, group ? group : -8, 1,
           alpha};
  const int ntiles = p.nm * p.nn;
  int grid = grid_cap > 0 ? grid_cap : num_cus();
  if (grid > ntiles) grid = ntiles;
  int x = xcc > 0 ? xcc : 32;
  while (x > 1 && grid % (8 * x)) x >>= 1;
  if (grid % 8) x = 1;
  p.xcc = x;
  hipLaunchKernelGGL(PP_KERNEL, dim3(grid), dim3(512), 0, stream, p);
  return (int)hipGetLastError();
}
