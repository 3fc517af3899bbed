// Projection GEMM for gfx950:  C[M, N] = alpha A[M, K] . B[N, K]^T (+ beta C) with a fused epilogue.
//
// Both operands are stored K-contiguous (activations [tokens, in], weights [out, in]; the backward
// input-gradient GEMM hands the transposed frozen weight, also K-contiguous) -- every base GEMM of
// a LoRA / QLoRA step has this form (ops/linear.py).  Reference workload: the projections of the
// LoRA job spec the control plane launches (/root/reference/app/models/base/finetuning.py:51-145 --
// the reference itself ships no training code).
//
// Geometry: one 256-thread workgroup (4 waves, ONE per SIMD, one workgroup per CU) owns a 256 x 256
// tile of C; wave w = (wm, wn) = (w >> 1, w & 1) owns 128 x 128 as 8 x 8 accumulators of
// v_mfma_f32_16x16x32_bf16 (256 accumulator registers; the 16x16 shape holds a higher clock than
// 32x32 on random data at equal cycles per FLOP -- MI355X_MICROARCH "DVFS give-back" item 7).
//
// Pipeline: K advances in 64-deep "super-stages" through two LDS buffers (A [256][64] | B [256][64]
// bf16 = 64 KiB each, 128-byte rows = whole cache lines per DMA row), filled by LDS-DMA
// (buffer_load_dwordx4 ... lds, 16 B per lane, 8 rows x 128 B per 1 KiB piece) two super-stages
// ahead.  Each wave holds two full fragment sets: X (first 32 of the stage's K) and Y (second 32).
// Iteration g (one super-stage) runs 128 MFMAs as 16 groups of 8 (group = one B fragment against the
// 8 A fragments, src0 constant across the group); the LDS reads of Y, the DMA pieces of stage g+2 and
// the reads of X for stage g+1 sit between the MFMAs of the dense chain, with three barriers per
// stage: A region released (its DMA starts), B region released (its DMA starts), stage g+1 landed.
//
// PERSISTENT grid (round-4 change, profiles/r4/gemm_nt.md): gridDim.x <= number of CUs and each
// workgroup walks its tiles l = xmap(blockIdx) + i * gridDim.x.  The super-stage stream runs across
// tile boundaries -- the first two stages of tile i+1 are prefetched under the last two of tile i --
// so a tile change costs only its epilogue stores (no workgroup launch, no cold pipeline refill from
// HBM on every CU at once).  The first super-stage of every tile feeds a zero accumulator into the
// MFMA instead of clearing 256 registers.
//
// Tile order: logical id l -> (M block, N block) by groups of |group| blocks along M (group > 0) or N
// (group < 0), fastest inside the group; xmap puts `xcc` consecutive logical ids of every 8 * xcc on
// one hardware XCD slot (workgroups are dealt round-robin over the 8 XCDs: blocks b and b + 8 share an
// L2 -- speed only, never correctness).
//
// LDS image: [row][64 k] bf16 = 128-byte rows, 16-byte chunk c of row r stored at c ^ f5(r),
// f5(r) = r0 | r1 << 1 | r3 << 2 -- conflict-free for the ds_read_b128 fragment reads of both operands
// (brute-forced over the lane groups).  The swizzle is applied to the per-lane DMA SOURCE address so
// the LDS side stays lane-linear (guide rule 21).
//
// Output layout: the MFMA is fed (A operand = B rows, B operand = A rows), so lane l ends up holding
// C[m = l & 15][n = 4 (l >> 4) + 0..3] of each 16x16 tile; B fragment rows are read permuted inside each
// 32-column pair so that the two tiles of a pair give every lane 8 CONSECUTIVE columns: one 16-byte
// store per lane per (m tile, pair).
#include "common.h"

#include <cstdio>
#include <cstdlib>
#include <type_traits>

using namespace ftc;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int BM = 256, BN = 256, BKS = 64;
constexpr int IMG = 256 * BKS * 2;  // one operand image of a super-stage: 32 KiB
constexpr int SS = 2 * IMG;         // one LDS buffer: A | B
constexpr int PSTRIDE = 1024;       // LDS bytes between a wave's consecutive DMA pieces (8 rows x 128 B)

enum Epi : int {
  EPI_STORE = 0,  // C = alpha acc (+ beta C), bf16 or fp32
  EPI_ROPE = 1,   // bf16 C = rope(alpha acc) on the q / k heads (the packed qkv projection), beta 0
};

struct NTArgs {
  const uint16_t* a;  // [M, lda]
  const uint16_t* b;  // [N, ldb]
  void* c;            // [M, ldc]
  long long lda, ldb, ldc;
  int K, nm, nn;
  int group;  // > 0: groups of `group` M blocks (M fastest); < 0: groups of -group N blocks (N fastest)
  int xcc;    // logical ids per XCD slot in each run of 8 * xcc (power of two; gridDim.x % (8 xcc) == 0)
  float alpha, beta;
  // EPI_ROPE (head_dim 128): rotate the first rot_heads 128-column heads of every output row by
  // (cos, sin)[pos] (fp32 [max_pos, 64], HF rotate_half pairs (i, i + 64)); pos = positions[row] or
  // row % seq_len
  const float* cos_t;
  const float* sin_t;
  const int* positions;
  int seq_len, rot_heads;
};

DEV_INLINE int f5(int r) { return (r & 1) | (r & 2) | ((r >> 1) & 4); }

// logical tile id -> (M block, N block)
DEV_INLINE void tile_of(const NTArgs& p, int l, int& mb, int& nb) {
  const bool mfast = p.group > 0;
  const int g = mfast ? p.group : -p.group;
  const int nf = mfast ? p.nm : p.nn, ns = mfast ? p.nn : p.nm;  // fast / slow block counts
  const int grp = l / (g * ns), first = grp * g, gsz = min(nf - first, g);
  const int rem = l - grp * g * ns;
  const int f = first + rem % gsz, sl = rem / gsz;
  mb = mfast ? f : sl;
  nb = mfast ? sl : f;
}

// hardware workgroup id -> first logical tile id (bijective on [0, gridDim.x))
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

// Epilogue of one wave's 128 x 128: lane holds C[row0 + 16 mt + (lane & 15)][c0 + 32 pr + 8 kc + 0..7] in
// acc[mt][2 pr] (columns +0..3) and acc[mt][2 pr + 1] (+4..7), kc = lane >> 4: one 16-byte (bf16) / two
// (fp32) stores per (mt, pr).  With c0 % 128 == 0 the wave's columns are a whole 128-wide head, so
// RoPE's rotate_half partners (d, d + 64) are pairs pr / pr + 2 of the same lane.
template <bool F32C, int EPI, bool BETA>
DEV_INLINE void store_w128(const NTArgs& p, const f32x4 (&acc)[8][8], long long row0, long long c0) {
  // the lane index is re-derived here behind an opaque statement, so the per-lane epilogue addresses
  // are computed at the epilogue instead of being kept live (and spilled) across the K loop
  int lane;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
  const int li = lane & 15, kc = lane >> 4;
  if constexpr (EPI == EPI_STORE) {
#pragma unroll
    for (int mt = 0; mt < 8; ++mt)
#pragma unroll
      for (int pr = 0; pr < 4; ++pr) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = p.alpha * acc[mt][2 * pr][j];
          v[4 + j] = p.alpha * acc[mt][2 * pr + 1][j];
        }
        const long long off = (row0 + li + 16 * mt) * p.ldc + c0 + 8 * kc + 32 * pr;
        if constexpr (F32C) {
          f32x4* cp = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.c) + off);
          if constexpr (BETA) {
            const f32x4 o0 = cp[0], o1 = cp[1];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              v[j] += p.beta * o0[j];
              v[4 + j] += p.beta * o1[j];
            }
          }
          *cp = f32x4{v[0], v[1], v[2], v[3]};
          cp[1] = f32x4{v[4], v[5], v[6], v[7]};
        } else {
          u32x4* cp = reinterpret_cast<u32x4*>(reinterpret_cast<uint16_t*>(p.c) + off);
          if constexpr (BETA) {
            const u32x4 o = *cp;
            float f[8];
            unpack8(uint4{o[0], o[1], o[2], o[3]}, f);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] += p.beta * f[j];
          }
          const uint4 q = pack8(v);
          *cp = u32x4{q.x, q.y, q.z, q.w};
        }
        __builtin_amdgcn_sched_barrier(0);  // one store at a time: no register pile-up beside the live X set
      }
  } else {
    static_assert(!F32C, "RoPE epilogue is bf16");
    const bool rope = (int)(c0 >> 7) < p.rot_heads;  // wave-uniform
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      const long long row = row0 + li + 16 * mt;
      int pos = 0;
      if (rope) pos = p.positions ? p.positions[row] : (int)(row % p.seq_len);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float v[2][8];
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[q][j] = p.alpha * acc[mt][2 * (h + 2 * q)][j];
            v[q][4 + j] = p.alpha * acc[mt][2 * (h + 2 * q) + 1][j];
          }
        if (rope) {
          const int ri = 32 * h + 8 * kc;
          const f32x4* cp = reinterpret_cast<const f32x4*>(p.cos_t + (long long)pos * 64 + ri);
          const f32x4* sp = reinterpret_cast<const f32x4*>(p.sin_t + (long long)pos * 64 + ri);
          const f32x4 c0v = cp[0], c1v = cp[1], s0v = sp[0], s1v = sp[1];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float cs = j < 4 ? c0v[j & 3] : c1v[j & 3], sn = j < 4 ? s0v[j & 3] : s1v[j & 3];
            const float x1 = v[0][j], x2 = v[1][j];
            v[0][j] = x1 * cs - x2 * sn;
            v[1][j] = x2 * cs + x1 * sn;
          }
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const uint4 w = pack8(v[q]);
          *reinterpret_cast<u32x4*>(reinterpret_cast<uint16_t*>(p.c) + row * p.ldc + c0 + 64 * q + 32 * h + 8 * kc) =
              u32x4{w.x, w.y, w.z, w.w};
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
}

// stores per lane of one wave epilogue (they sit in vmcnt between two DMA stages, see the kernel)
template <bool F32C>
constexpr int kEpiStores = F32C ? 64 : 32;

template <bool F32C, int EPI, bool BETA>
__global__ __launch_bounds__(256, 1) void gemm_nt_kernel(NTArgs p) {
  __shared__ __attribute__((aligned(16))) char S[2 * SS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int G = gridDim.x, ntiles = p.nm * p.nn;
  const int lw = xmap(blockIdx.x, p.xcc);
  const int my = lw < ntiles ? (ntiles - lw + G - 1) / G : 0;
  if (my == 0) return;  // (the launcher sizes the grid <= ntiles: never taken)
  const int ns = p.K / BKS;
  const int total = my * ns;

  // DMA: wave w fills rows [64 w, 64 w + 64) of both images; piece j = rows 64 w + 8 j + (lane >> 3),
  // lane chunk (lane & 7) ^ f5(row) -- f5 sees row bits 0-2 (lane >> 3) and 3 (j & 1).
  int vo[2][2];
  {
    const int rr = lane >> 3, pc = lane & 7;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int r0 = 64 * wave + rr;
      const int lc = pc ^ f5(rr + 8 * q);
      vo[0][q] = (int)((r0 * p.lda + 8 * lc) * 2);
      vo[1][q] = (int)((r0 * p.ldb + 8 * lc) * 2);
    }
  }
  int so[2][8];  // scalar offsets of the 8 pieces (8 rows each)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    so[0][j] = (int)(j * 8 * p.lda * 2);
    so[1][j] = (int)(j * 8 * p.ldb * 2);
  }
  char* const wbase = S + 64 * wave * 128;
  const unsigned lds0 = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)wbase;
  // One piece.  M0 (the LDS destination) walks with the pieces: every piece's statement advances it by
  // one piece after its load (s_add, like the library's loop), the last piece of a chain loads M0 with
  // the first destination of the NEXT chain (A -> B of the same stage, B -> A of the next stage), so the
  // loop never writes M0 right before a DMA (MFMAs separate them: the SALU-write -> LDS-DMA hazard) and
  // needs one SALU per piece.  NOP: a wait state before the load (back-to-back pieces, prologue only).
  // M0 has no other user in this kernel (tests/test_build.py checks the ISA).
  // `sc0` cache policy on the pieces (profiles/r4/gemm_nt/policy.log)
  auto dma = [&](int op, __amdgpu_buffer_rsrc_t r, int j, unsigned next, bool nop) __attribute__((always_inline)) {
    if (nop) asm volatile("s_nop 0" ::: "memory");
    if (j < 7)
      asm volatile("buffer_load_dwordx4 %0, %1, %2 offen sc0 lds\n\ts_add_u32 m0, m0, 0x400"
                   ::"v"(vo[op][j & 1]), "s"(r), "s"(so[op][j]) : "memory");
    else
      asm volatile("buffer_load_dwordx4 %0, %1, %2 offen sc0 lds\n\ts_mov_b32 m0, %3"
                   ::"v"(vo[op][1]), "s"(r), "s"(so[op][7]), "s"(next) : "memory");
  };
  static_assert(PSTRIDE == 0x400, "the M0 walk adds one 1 KiB piece");

  // prefetch cursor: global stage pg = (tile pi, stage ps); pa / pb = the operands at stage ps of tile pi
  int pg = 0, pi = 0, ps = 0;
  const uint16_t* pa;
  const uint16_t* pb;
  auto tile_bases = [&](int i, const uint16_t*& ta, const uint16_t*& tb) __attribute__((always_inline)) {
    int mb, nb;
    tile_of(p, lw + i * G, mb, nb);
    mb = __builtin_amdgcn_readfirstlane(mb);  // uniform by construction; keeps the bases in SGPRs
    nb = __builtin_amdgcn_readfirstlane(nb);
    ta = p.a + (long long)mb * BM * p.lda;
    tb = p.b + (long long)nb * BN * p.ldb;
  };
  tile_bases(0, pa, pb);
  // past the last stage the cursor stays put: the repeated stage lands in a buffer nobody reads again
  auto advance = [&]() __attribute__((always_inline)) {
    if (pg + 1 < total) {
      ++pg;
      if (++ps == ns) {
        ps = 0;
        ++pi;
        tile_bases(pi, pa, pb);
      } else {
        pa += BKS;
        pb += BKS;
      }
    }
  };

  const int li = lane & 15, kc = lane >> 4;
  int a_off[2], b_off[2];
  {
    const int ra_ = wm * 128 + li;
    const int rb_ = 128 * wn + 8 * (li >> 2) + (li & 3);  // store_w128's column mapping
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      a_off[h] = ra_ * 128 + 16 * ((4 * h + kc) ^ f5(li));
      b_off[h] = IMG + rb_ * 128 + 16 * ((4 * h + kc) ^ f5(rb_));
    }
  }
  auto bnt = [](int nt) { return (32 * (nt >> 1) + 4 * (nt & 1)) * 128; };

  f32x4 acc[8][8];
  bf16x8 xa[8], xb[8], ya[8], yb[8];
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};

  // one MFMA group: B fragment g against the 8 A fragments, side operation k after MFMAs 1, 3, 5, 7;
  // FIRST: the tile's first K-half, accumulators start from zero
  auto group = [&](const bf16x8 (&fa)[8], const bf16x8 (&fb)[8], int g, auto first, auto&& side)
      __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if constexpr (decltype(first)::value)
        acc[q][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[g], fa[q], zero, 0, 0, 0);
      else
        acc[q][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[g], fa[q], acc[q][g], 0, 0, 0);
      if (q & 1) {
        __builtin_amdgcn_sched_barrier(0);
        side(q >> 1);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  auto nop = [](int) __attribute__((always_inline)) {};

  // one super-stage.  first: the tile's first stage (zero accumulators); after_epi: an epilogue's
  // stores were issued between the DMA of stage g+1 and this iteration's pieces, so the wait for stage
  // g+1 leaves them in flight too (vmcnt counts loads, stores and LDS-DMA together, in issue order).
  auto iteration = [&](int g, auto first, bool after_epi) __attribute__((always_inline)) {
    const char* cur = S + (g & 1) * SS;
    const char* nxt = S + ((g + 1) & 1) * SS;
    const auto ras = make_rsrc(pa);
    const auto rbs = make_rsrc(pb);
    const unsigned dB = lds0 + (unsigned)((g & 1) * SS) + IMG;      // M0 after the A chain
    const unsigned dA_next = lds0 + (unsigned)(((g + 1) & 1) * SS);  // M0 after the B chain
    // half 0 on X: Y.A in groups 0-1, release A after group 2; A pieces and Y.B in groups 3-6;
    // release B after group 7.  Every wait sits at least one group after the reads it covers.
#pragma unroll
    for (int gi = 0; gi < 2; ++gi)
      group(xa, xb, gi, first, [&](int k) __attribute__((always_inline)) {
        ya[4 * gi + k] = rd(cur, a_off[1] + (4 * gi + k) * 2048);
      });
    group(xa, xb, 2, first, nop);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    barrier();
#pragma unroll
    for (int gi = 3; gi < 7; ++gi)
      group(xa, xb, gi, first, [&](int k) __attribute__((always_inline)) {
        const int i = 2 * (gi - 3) + (k >> 1);
        if (k & 1) yb[i] = rd(cur, b_off[1] + bnt(i));
        else dma(0, ras, i, dB, false);
      });
    group(xa, xb, 7, first, nop);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    barrier();
    // half 1 on Y: B pieces in groups 0-3, wait for stage g+1, X of g+1 in groups 4-5 (A first: the
    // next iteration's first group needs all of X.A but only X.B[0])
#pragma unroll
    for (int gi = 0; gi < 4; ++gi)
      group(ya, yb, gi, std::false_type{}, [&](int k) __attribute__((always_inline)) {
        if (!(k & 1)) dma(1, rbs, 2 * gi + (k >> 1), dA_next, false);
      });
    if (after_epi) {
      constexpr int n = 16 + kEpiStores<F32C> > 63 ? 63 : 16 + kEpiStores<F32C>;
      __builtin_amdgcn_s_waitcnt(0x0F70 | (n & 15) | ((n >> 4) << 14));
    } else {
      __builtin_amdgcn_s_waitcnt(0x4F70);  // vmcnt(16): the 16 pieces of g+1 landed
    }
    barrier();
    group(ya, yb, 4, std::false_type{}, [&](int k) __attribute__((always_inline)) {
      xa[2 * k] = rd(nxt, a_off[0] + 2 * k * 2048);
      xa[2 * k + 1] = rd(nxt, a_off[0] + (2 * k + 1) * 2048);
    });
    group(ya, yb, 5, std::false_type{}, [&](int k) __attribute__((always_inline)) {
      xb[2 * k] = rd(nxt, b_off[0] + bnt(2 * k));
      xb[2 * k + 1] = rd(nxt, b_off[0] + bnt(2 * k + 1));
    });
#pragma unroll
    for (int gi = 6; gi < 8; ++gi) group(ya, yb, gi, std::false_type{}, nop);
    advance();
  };

  // prologue: global stages 0 and 1 (back-to-back pieces: a wait state before each load)
  {
    const unsigned d0 = lds0, d1 = lds0 + (unsigned)SS;
    asm volatile("s_mov_b32 m0, %0" :: "s"(d0) : "memory");
#pragma unroll
    for (int j = 0; j < 8; ++j) dma(0, make_rsrc(pa), j, d0 + IMG, true);
#pragma unroll
    for (int j = 0; j < 8; ++j) dma(1, make_rsrc(pb), j, d1, true);
    advance();
#pragma unroll
    for (int j = 0; j < 8; ++j) dma(0, make_rsrc(pa), j, d1 + IMG, true);
#pragma unroll
    for (int j = 0; j < 8; ++j) dma(1, make_rsrc(pb), j, d0, true);  // M0 = iteration 0's A chain (buffer 0)
    advance();
    __builtin_amdgcn_s_waitcnt(0x4F70);  // vmcnt(16): stage 0 landed
  }
  barrier();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    xa[i] = rd(S, a_off[0] + i * 2048);
    xb[i] = rd(S, b_off[0] + bnt(i));
  }

  int g = 0;
  for (int ti = 0; ti < my; ++ti) {
    iteration(g++, std::true_type{}, ti > 0);
    for (int s = 1; s < ns; ++s) iteration(g++, std::false_type{}, false);
    int mb, nb;
    tile_of(p, lw + ti * G, mb, nb);
    store_w128<F32C, EPI, BETA>(p, acc, (long long)mb * BM + wm * 128, (long long)nb * BN + wn * 128);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): no LDS-DMA may outlive the workgroup
}

// ---- launch configuration ----------------------------------------------------------------------------
// Measured and fixed (profiles/r4/gemm_nt.md, gemm_nt/policy.log): one persistent workgroup per CU, N-fast
// groups of 8 blocks, XCD runs of 32 logical ids, plain C stores (non-temporal: no gain), `sc0` on the
// operand DMA (+0.1-2.4 % over the default policy; sc1 / sc0 sc1 equal, nt -20-30 %).  The grid cap / order
// stay settable for tools/bench_gemm_nt.py and the multi-tile tests (ftc_gemm_nt_config).
struct Config {
  int grid_cap;  // persistent grid: min(tiles, grid_cap) workgroups (0: number of CUs)
  int group;     // tile order, see NTArgs
  int xcc;
};

Config& config() {
  static Config c{0, -8, 32};
  return c;
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

template <bool F32C, int EPI>
int launch(NTArgs& p, hipStream_t stream) {
  const Config& c = config();
  const int ntiles = p.nm * p.nn;
  int grid = c.grid_cap > 0 ? c.grid_cap : num_cus();
  if (grid > ntiles) grid = ntiles;
  int xcc = c.xcc > 0 ? c.xcc : 1;
  while (xcc > 1 && grid % (8 * xcc)) xcc >>= 1;  // xmap must be a bijection on [0, grid)
  if (grid % 8) xcc = 1;
  p.group = c.group == 0 ? 1 : c.group;
  p.xcc = xcc;
  if (EPI == EPI_STORE && p.beta != 0.f)  // accumulating calls: tests / rare paths
    hipLaunchKernelGGL((gemm_nt_kernel<F32C, EPI, true>), dim3(grid), dim3(256), 0, stream, p);
  else
    hipLaunchKernelGGL((gemm_nt_kernel<F32C, EPI, false>), dim3(grid), dim3(256), 0, stream, p);
  return (int)hipGetLastError();
}

}  // namespace

// Launch configuration of every later call (tools/bench_gemm_nt.py, tests): grid_cap (0 = CU count),
// group (> 0 M-fast, < 0 N-fast), xcc.
extern "C" void ftc_gemm_nt_config(int grid_cap, int group, int xcc) { config() = Config{grid_cap, group, xcc}; }

// C[M, N] (ldc) = alpha A B^T + beta C; A [M, K] (lda), B [N, K] (ldb) bf16 row-major, K contiguous.
// Returns 0 when the shape / alignment is outside the kernel's contract.
extern "C" int ftc_gemm_nt_ok(const void* a, long long lda, const void* b, long long ldb, const void* c, long long ldc,
                              int c_fp32, int M, int N, int K) {
  if (M <= 0 || N <= 0 || K <= 0 || M % BM || N % BN || K % BKS) return 0;
  if (lda % 8 || ldb % 8 || ldc % 8 || lda < K || ldb < K || ldc < N) return 0;
  if ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) | reinterpret_cast<uintptr_t>(c)) & 15) return 0;
  // 32-bit per-lane / scalar DMA offsets inside one tile: 255 rows + 128 bytes of K
  if ((long long)(BM - 1) * (lda > ldb ? lda : ldb) * 2 + 2 * BKS * 2 >= (1LL << 31)) return 0;
  if ((long long)(M / BM) * (N / BN) > 0x7fffffffLL) return 0;
  (void)c_fp32;
  return 1;
}

extern "C" int ftc_gemm_nt(const void* a, long long lda, const void* b, long long ldb, void* c, long long ldc,
                           int c_fp32, int M, int N, int K, float alpha, float beta, hipStream_t stream) {
  if (!ftc_gemm_nt_ok(a, lda, b, ldb, c, ldc, c_fp32, M, N, K)) return -1;
  NTArgs p{(const uint16_t*)a, (const uint16_t*)b, c, lda, ldb, ldc, K, M / BM, N / BN, 1, 1, alpha, beta};
  return c_fp32 ? launch<true, EPI_STORE>(p, stream) : launch<false, EPI_STORE>(p, stream);
}

// qkv projection with RoPE fused into the epilogue: c[M, N] bf16 = rope(a b^T) on the first rot_heads
// 128-wide heads (q then k), the rest (v) stored as is.  cos / sin: fp32 [max_pos, 64]; positions: int32
// [M] or null (row % seq_len).
extern "C" int ftc_gemm_nt_rope(const void* a, long long lda, const void* b, long long ldb, void* c, long long ldc,
                                int M, int N, int K, const float* cos_t, const float* sin_t, const int* positions,
                                int seq_len, int rot_heads, hipStream_t stream) {
  if (!ftc_gemm_nt_ok(a, lda, b, ldb, c, ldc, 0, M, N, K)) return -1;
  if (!cos_t || !sin_t || (reinterpret_cast<uintptr_t>(cos_t) | reinterpret_cast<uintptr_t>(sin_t)) & 15) return -1;
  if (!positions && seq_len <= 0) return -1;
  if (rot_heads < 0 || rot_heads * 128 > N) return -1;
  NTArgs p{(const uint16_t*)a, (const uint16_t*)b, c, lda, ldb, ldc, K, M / BM, N / BN, 1, 1, 1.f, 0.f,
           cos_t, sin_t, positions, seq_len, rot_heads};
  return launch<false, EPI_ROPE>(p, stream);
}
