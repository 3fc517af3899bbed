// Weight-gradient GEMM for gfx950 (full fine-tuning):  C[M, N] = beta C + alpha A^T B
//
//   A = dy [K, M] and B = x [K, N], both row-major with the reduction dimension K (= tokens) as the
//   SLOW one -- the "TT" form of dW += dy^T x that hipBLASLt / rocBLAS run at 1.24-1.36 PF/s on the
//   Llama-3-8B shapes (profiles/r2/tune_full: every TunableOp candidate timed) against 1.56 PF/s for
//   the same FLOPs in the forward's K-contiguous form.  The library wants K-contiguous operands; here
//   the transposition happens for free in the LDS read: both operands are staged as [k][col] images
//   and read with ds_read_b64_tr_b16, which hands every lane 4 consecutive k of one column -- exactly
//   the MFMA A/B fragment layout (the trick the flash backward already uses for dO^T / Q^T).  No
//   transposed copy of x (or dy) is ever written.
//
// Geometry: one 512-thread workgroup (8 waves, 2 per SIMD, one workgroup per CU) = a 256 x 256 C
// tile; wave (wm, wn) = (w >> 2, w & 3) owns 128 x 64 (4 x 2 accumulators of
// v_mfma_f32_32x32x16_bf16, 128 VGPRs).  K advances in 64-row steps:
//   * each K-step's A and B tiles ([64 k][256 col] bf16, 32 KiB each) arrive by LDS-DMA
//     (buffer_load_dwordx4 ... lds, 8 per wave) as four [64][128] half images with 256-byte rows,
//     16-byte chunks XOR-swizzled by (r & 3) << 2 -- conflict-free for the tr_b16 reads.  The swizzle
//     is applied to the per-lane GLOBAL source, the LDS side stays lane-linear;
//   * double buffered; the DMA is issued as inline asm so that hipcc does not drain it (vmcnt(0))
//     before every read of the other buffer; one barrier per K-step, placed before its last k-step
//     (see `step`), after which the DMA of step k+2 flies under a whole step of MFMAs;
//   * software pipelined by 16-deep k-steps: the tr reads of the next k-step go out beside the
//     MFMAs of the current one (two register sets of fragments);
//   * block -> tile: XCD-bijective remap (each XCD gets a contiguous run of logical tiles), then
//     groups of group_m M-blocks x all N-blocks (M fastest) so the 32 tiles resident on one XCD share
//     a few dy and x panels in its L2.
// Epilogue: alpha * acc (+ beta * C) rounded once, into bf16 or fp32 C (the fp32 gradient buffer of
// the precise accumulation mode).  Shapes: M, N multiples of 256, K of 64 (every Llama / Mistral
// projection and the vocab-chunked lm_head); anything else stays on the library.
#include "common.h"

#include <cstdlib>
#include <type_traits>

using namespace ftc;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int IMG = BK * 128 * 2;  // one [64 k][128 col] bf16 half image: 16 KiB
constexpr int STAGE = 4 * IMG;     // A lo | A hi | B lo | B hi

// Only tr_b16 reads touch these images (no row reads): XOR-ing the 16-byte chunk with (r & 3) << 2
// spreads the 4 rows a 32-lane half reads over the 4 quarters of the bank row -- conflict-free -- and
// rows r and r + 8 (the two reads of a fragment) share one swizzle, so a fragment costs ONE address
// register (+2048 immediate) and a DMA piece's source columns do not depend on its row block.
DEV_INLINE int swz(int r) { return (r & 3) << 2; }
DEV_INLINE int img_off(int r, int chunk) { return r * 256 + 16 * ((chunk ^ swz(r)) & 15); }

// A/B fragment (32 cols x 16 k, permuted k) by two transposed reads: lane l gets column colbase +
// (l & 31), k = kb + 4 (l >> 5) + {0..3} from the first read and + 8 + {0..3} from the second; both
// operands use the same permutation, so the MFMA's k-sum is unchanged.
DEV_INLINE int tr_offset(int colbase, int lane) {
  const int hh = lane >> 5, gi = (lane >> 4) & 3, li = lane & 15;
  const int trq = li >> 2, trp = li & 3;
  const int col = colbase + 16 * (gi & 1) + 4 * trp;
  const int chunk = col >> 3, half8 = (col & 7) ? 8 : 0;
  return img_off(4 * hh + trq, chunk) + half8;  // row r1; row r1 + 8 is +2048 (same swizzle)
}
DEV_INLINE bf16x8 tr_read(const char* img, int kb, int off) {
  s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + off + kb * 256));
  s16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + off + kb * 256 + 2048));
  s16x8 va = {v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
  return __builtin_bit_cast(bf16x8, va);
}

struct GemmTNArgs {
  const uint16_t* a;  // [K, lda] dy
  const uint16_t* b;  // [K, ldb] x
  void* c;            // [M, ldc] bf16 or fp32
  long long lda, ldb, ldc;
  int K, nm, nn;
  float alpha, beta;
  int group_m;  // M-blocks per tile group (XCD-local operand reuse)
  long long cstride;  // split-K: elements between the splits' C (fp32 partial) matrices; K = one split's rows
};

// One LDS-DMA instruction (buffer_load_dwordx4 ... lds) as inline asm: hipcc then keeps it out of its
// s_waitcnt bookkeeping.  Issued through the builtin, every ds_read of the OTHER buffer got a
// compiler-inserted vmcnt(0) in front of it (the merged LDS allocation defeats the alias scopes),
// draining the DMA that is meant to fly under the MFMAs; here the one explicit vmcnt(0) before each
// barrier is the only wait.  M0 is saved / restored inside the statement (guide: compiler-reserved);
// s_nop 4 covers an SGPR operand written by v_readfirstlane just before.
DEV_INLINE void glds16(__amdgpu_buffer_rsrc_t r, const char* lds, int voff, int soff) {
  const unsigned dst = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)lds;
  unsigned keep;
  asm volatile(
      "s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(r), "s"(dst), "s"(soff)
      : "memory");
}

// The same piece without the leading s_nop 4 (its operands are SALU-computed long before: no
// readfirstlane -> SGPR hazard to cover); used inside the K loop of the spread schedule.
DEV_INLINE void glds16_fast(__amdgpu_buffer_rsrc_t r, const char* lds, int voff, int soff) {
  const unsigned dst = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)lds;
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(r), "s"(dst), "s"(soff)
      : "memory");
}

// One K-step's DMA for this wave: PW = 32 / NW pieces of each matrix (32 KiB = 32 x 1 KiB per K-step);
// piece c = PW wave + j covers half image c >> 4, rows 4 (c & 15) .. +4 (lane-linear).  With the
// (r & 3) << 2 swizzle every lane's row phase is lane >> 4 whatever the piece, so one source offset
// per matrix serves all PW pieces (+ 4 j rows as the scalar offset).
template <int NW>
DEV_INLINE void tn_dma(__amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb, int voa, int vob, int sa4, int sb4,
                    char* stage, int wave) {
  constexpr int PW = 32 / NW;
  const int c0 = wave * PW;
  const int dst = (c0 >> 4) * IMG + (c0 & 15) * 1024;
#pragma unroll
  for (int j = 0; j < PW; ++j) {
    glds16(ra, stage + dst + j * 1024, voa, j * sa4);
    glds16(rb, stage + 2 * IMG + dst + j * 1024, vob, j * sb4);
  }
}

// 2 x 2 waves of 128 x 128, one wave per SIMD (512 registers; the 256 accumulator registers live in
// AGPRs): per MFMA a wave reads 1 fragment instead of 1.5 for 8 waves of 128 x 64 (measured slower and
// removed), which takes the LDS array (tr reads + the DMA's writes) from ~90 % to ~60 % of the MFMA
// time per K-step.  The K-step's DMA is spread over its four 16-deep phases (the round-2 schedule -- one
// 16-piece burst behind the step's single barrier -- is in git history).  Rows 16 q .. 16 q + 15 of an image feed only k-step q, so once every wave has read k-step q
// (lgkmcnt(0) + a barrier at the start of phase q + 1) the pieces covering those rows may be refilled
// with step kt + 2: 4 pieces at phase 1 (k-step 0's rows), 4 at phase 2, 8 at phase 3, each one
// between MFMAs instead of a 16-piece burst behind the step's single barrier (whose issue cost -- M0
// save / restore, s_nop -- left the matrix pipe idle); the next step's buffer is waited for with a
// counted vmcnt (this step's pieces stay in flight) before the last phase reads its k-step 0.
template <bool F32C>
__global__ __launch_bounds__(256, 1) void gemm_tn_kernel(GemmTNArgs p) {
  constexpr int NW = 4;
  constexpr int WN = NW / 2;         // waves along N
  constexpr int WNC = BN / WN;       // columns per wave: 64 or 128
  constexpr int NT = WNC / 32;       // 32-wide accumulator tiles along N: 2 or 4
  constexpr int PW = 32 / NW;        // DMA pieces per wave per matrix
  // both stages in ONE array: the DMA is inline asm, invisible to hipcc's alias analysis and waits,
  // so nothing is gained from distinct objects, and a rolled K loop (runtime stage offset) keeps the
  // register allocation of the 512-register variant sane
  __shared__ __attribute__((aligned(16))) char S[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5, lr = lane & 31;
  const int wm = wave / WN, wn = wave % WN;

  // ---- block -> tile
  int mb, nb;
  // split-K (grid = splits x tiles, split-major): split `ks` reduces rows [ks K, ks K + K) of A and B
  // into its own C matrix (fp32 partials, summed by splitk_sum_kernel)
  const int ks = blockIdx.x / (p.nm * p.nn);
  {
    const int nblk = p.nm * p.nn, bid = blockIdx.x - ks * nblk;
    const int xcd = bid & 7, q = nblk >> 3, rr = nblk & 7;
    const int t = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
    const int gm = p.group_m;
    const int grp = t / (gm * p.nn);
    const int first = grp * gm;
    const int gsz = min(p.nm - first, gm);
    const int rem = t - grp * gm * p.nn;
    mb = first + rem % gsz;
    nb = rem / gsz;
  }
  const long long m0 = (long long)mb * BM, n0 = (long long)nb * BN;

  // ---- per-lane DMA source offsets (pre-swizzled columns), loop invariant
  int voa, vob;
  {
    const int c0 = wave * PW;
    const int r = 4 * (c0 & 15) + (lane >> 4);  // row of piece 0; piece j: + 4 j
    const int col = (c0 >> 4) * 128 + 8 * ((lane & 15) ^ swz(r));
    voa = (r * (int)p.lda + col) * 2;
    vob = (r * (int)p.ldb + col) * 2;
  }
  const int sa4 = 4 * (int)p.lda * 2, sb4 = 4 * (int)p.ldb * 2;
  const uint16_t* abase = p.a + m0 + (long long)ks * p.K * p.lda;
  const uint16_t* bbase = p.b + n0 + (long long)ks * p.K * p.ldb;
  auto issue = [&](int kt, char* stage) {
    const auto ra = make_rsrc(abase + (long long)kt * BK * p.lda);
    const auto rb = make_rsrc(bbase + (long long)kt * BK * p.ldb);
    tn_dma<NW>(ra, rb, voa, vob, sa4, sb4, stage, wave);
  };

  // fragment offsets: A = half image wm, columns mt 32; B = the wave's WNC columns of half image
  // (wn WNC) >> 7
  int toa[4], tob[NT];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) toa[mt] = tr_offset(mt * 32, lane);
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) tob[nt] = tr_offset((wn * WNC) % 128 + nt * 32, lane);
  const int bhalf = (wn * WNC) >> 7;

  f32x16 acc[4][NT];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[mt][nt][i] = 0.f;

  // Fragments of one 16-deep k-step: 4 A + NT B.  Two named register sets P / Q alternate: the reads
  // of k-step q + 1 go out beside the MFMAs of k-step q (each phase: wait for the previous phase's
  // reads, issue the next reads, run 4 NT MFMAs), so the LDS traffic runs under the matrix pipe.
  auto read_k = [&](const char* stage, int kk, bf16x8 (&fa)[4], bf16x8 (&fb)[NT]) __attribute__((always_inline)) {
    const char* Ai = stage + wm * IMG;
    const char* Bi = stage + 2 * IMG + bhalf * IMG;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) fb[nt] = tr_read(Bi, 16 * kk, tob[nt]);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) fa[mt] = tr_read(Ai, 16 * kk, toa[mt]);
  };
  auto mfma_k = [&](const bf16x8 (&fa)[4], const bf16x8 (&fb)[NT]) __attribute__((always_inline)) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[mt], fb[nt], acc[mt][nt], 0, 0, 0);
    // pin the phase boundary: the MFMAs are register-only, so without it the scheduler moves them
    // across the next wait / barrier and the reads' latency is waited out with an idle matrix pipe
    __builtin_amdgcn_sched_barrier(0);
  };
  auto lgkm0 = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the previous phase's reads are in
    __builtin_amdgcn_sched_barrier(0);
  };
  const int nk = p.K / BK;
  bf16x8 pa[4], pb[NT], qa[4], qb[NT];
  {
    // refill mapping: the 8 pieces (4 rows each) of k-step q's 16 rows across both half images are
    // split 2 per wave -- wave w takes half image w >> 1, rows 16 q + 8 (w & 1) + 4 e (e = 0, 1) -- so
    // every wave issues the same pieces in the same phase (no wave-dependent branch around the
    // accumulators).  The (r & 3) << 2 swizzle is q / e independent: one source offset per matrix.
    int va2, vb2;
    {
      const int r = 8 * (wave & 1) + (lane >> 4);
      const int col = (wave >> 1) * 128 + 8 * ((lane & 15) ^ swz(r));
      va2 = (r * (int)p.lda + col) * 2;
      vb2 = (r * (int)p.ldb + col) * 2;
    }
    const int dst2 = (wave >> 1) * IMG + 2 * (wave & 1) * 1024;
    // piece (q, e) of step kt2 into `stage`
    auto piece = [&](int kt2, char* stage, int q, int e) __attribute__((always_inline)) {
      if (kt2 >= nk) return;
      const int kk = kt2;
      const auto ra = make_rsrc(abase + (long long)kk * BK * p.lda);
      const auto rb = make_rsrc(bbase + (long long)kk * BK * p.ldb);
      const int off = (4 * q + e) * 1024;
      glds16_fast(ra, stage + dst2 + off, va2, (16 * q + 4 * e) * (int)p.lda * 2);
      glds16_fast(rb, stage + 2 * IMG + dst2 + off, vb2, (16 * q + 4 * e) * (int)p.ldb * 2);
    };
    // the 16 MFMAs of a phase (rows mt_lo .. mt_hi of the 4 x 4 tile grid) with piece pairs after
    // MFMAs 3, 7, 11, 15 (slot k gets pieces[k] if k < npc)
    auto mfma_pieces = [&](const bf16x8 (&fa)[4], const bf16x8 (&fb)[4], int mt_lo, int mt_hi, int kt2,
                           char* stage, const int (&pq)[4], const int (&pe)[4], int npc) __attribute__((always_inline)) {
#pragma unroll
      for (int mt = mt_lo; mt < mt_hi; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[mt], fb[nt], acc[mt][nt], 0, 0, 0);
          if (nt == 3 && (mt - mt_lo) < npc) {
            __builtin_amdgcn_sched_barrier(0);
            piece(kt2, stage, pq[mt - mt_lo], pe[mt - mt_lo]);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      __builtin_amdgcn_sched_barrier(0);
    };
    issue(0, S);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __builtin_amdgcn_s_barrier();
    if (nk > 1) issue(1, S + STAGE);
    read_k(S, 0, pa, pb);
    const int q0[4] = {0, 0, 0, 0}, e01[4] = {0, 1, 0, 0};
    const int q1[4] = {1, 1, 0, 0};
    const int q23[4] = {2, 2, 3, 3}, e23[4] = {0, 1, 0, 1};
    for (int kt = 0; kt < nk; ++kt) {
      const int so = (kt & 1) * STAGE;
      char* cur = S + so;
      const char* nxt = S + (STAGE - so);
      // phase 0: k-step 0 (P), read k-step 1 -> Q
      lgkm0();
      read_k(cur, 1, qa, qb);
      mfma_k(pa, pb);
      // phase 1: every wave has read k-steps 0 and 1 -> refill k-step 0's rows with step kt + 2
      lgkm0();
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      read_k(cur, 2, pa, pb);
      mfma_pieces(qa, qb, 0, 4, kt + 2, cur, q0, e01, 2);
      // phase 2: k-step 2 read -> refill k-step 1's rows
      lgkm0();
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      read_k(cur, 3, qa, qb);
      mfma_pieces(pa, pb, 0, 4, kt + 2, cur, q1, e01, 2);
      // phase 3: k-step 3 read -> refill k-steps 2 and 3 over the first half of the MFMAs; then step
      // kt + 1's buffer (16 pieces issued during step kt - 1) must have landed: only this step's 16
      // may still fly
      lgkm0();
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      mfma_pieces(qa, qb, 0, 2, kt + 2, cur, q23, e23, 2);
      {
        // the other two piece pairs of k-steps 2 / 3 between MFMAs of rows 2 .. 3 would follow the
        // wait below; issue them here, back to back with the last two of the first half
        const int q23b[4] = {3, 3, 0, 0}, e23b[4] = {0, 1, 0, 0};
        piece(kt + 2, cur, q23b[0], e23b[0]);
        piece(kt + 2, cur, q23b[1], e23b[1]);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 2 < nk) __builtin_amdgcn_s_waitcnt(0x4F70);  // vmcnt(16)
      else __builtin_amdgcn_s_waitcnt(0x0F70);             // vmcnt(0)
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 1 < nk) read_k(nxt, 0, pa, pb);
      mfma_pieces(qa, qb, 2, 4, kt + 2, cur, q23, e23, 0);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // no DMA may land after the workgroup ends
  }

  // ---- epilogue: lane holds C[m0 + wm 128 + mt 32 + 8 (r >> 2) + 4 hh + (r & 3)][n0 + wn WNC + nt 32 + lr];
  // per accumulator tile, the 16 old C values are loaded together (one latency, not 16) -- beta is
  // tested once, outside the loops (a per-element branch around a load serialises the round trips)
  using CT = typename std::conditional<F32C, float, uint16_t>::type;
  CT* cbase = reinterpret_cast<CT*>(p.c) + ks * p.cstride + (m0 + wm * 128 + 4 * hh) * p.ldc + n0 + wn * WNC + lr;
  const bool accumulate = p.beta != 0.f;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      CT* ct = cbase + (long long)(mt * 32) * p.ldc + nt * 32;
      float old[16];
      if (accumulate) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const CT x = ct[(long long)(8 * (r >> 2) + (r & 3)) * p.ldc];
          if constexpr (F32C) old[r] = p.beta * x;
          else old[r] = p.beta * bf2f(x);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) old[r] = 0.f;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = p.alpha * acc[mt][nt][r] + old[r];
        CT* cp = ct + (long long)(8 * (r >> 2) + (r & 3)) * p.ldc;
        if constexpr (F32C) *cp = v;
        else *cp = f2bf(v);
      }
    }
}

}  // namespace

// C[M, N] (ldc) = beta C + alpha A^T B; A [K, M] (lda), B [K, N] (ldb) bf16 row-major; C bf16 or fp32.
// Returns -1 (nothing launched) when the shape / alignment is outside the kernel's contract.
extern "C" int ftc_gemm_tn_ok(const void* a, long long lda, const void* b, long long ldb, const void* c, long long ldc,
                              int M, int N, int K) {
  if (M <= 0 || N <= 0 || K <= 0 || M % BM || N % BN || K % BK) return 0;
  if (lda % 8 || ldb % 8 || lda < M || ldb < N || ldc < N) return 0;
  if ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15) return 0;
  if ((long long)(BK - 1) * (lda > ldb ? lda : ldb) * 2 + 512 >= (1LL << 31)) return 0;  // 32-bit lane offsets
  if ((long long)(M / BM) * (N / BN) > 0x7fffffffLL) return 0;
  (void)c;
  return 1;
}

extern "C" int ftc_gemm_tn(const void* a, long long lda, const void* b, long long ldb, void* c, long long ldc,
                           int c_fp32, int M, int N, int K, float alpha, float beta, hipStream_t stream) {
  if (!ftc_gemm_tn_ok(a, lda, b, ldb, c, ldc, M, N, K)) return -1;
  GemmTNArgs p{(const uint16_t*)a, (const uint16_t*)b, c, lda, ldb, ldc, K, M / BM, N / BN, alpha, beta, 4, 0};
  const int grid = p.nm * p.nn;
  if (c_fp32)
    hipLaunchKernelGGL((gemm_tn_kernel<true>), dim3(grid), dim3(256), 0, stream, p);
  else
    hipLaunchKernelGGL((gemm_tn_kernel<false>), dim3(grid), dim3(256), 0, stream, p);
  return (int)hipGetLastError();
}

// Split-K weight gradient: parts[s] (fp32 [M, N], contiguous) = A[s K' : (s + 1) K']^T B[s K' : (s + 1) K']
// for s < splits, K' = K / splits -- one launch of splits x tiles workgroups (whole waves where the tile
// grid alone is not: qkv dW 384 -> 768, down dW 896 -> 1792); the caller folds the partials into the
// gradient with splitk_sum.
extern "C" int ftc_gemm_tn_split(const void* a, long long lda, const void* b, long long ldb, float* parts, int M, int N,
                                 int K, int splits, hipStream_t stream) {
  if (splits < 1 || K % splits || !ftc_gemm_tn_ok(a, lda, b, ldb, parts, N, M, N, K / splits)) return -1;
  GemmTNArgs p{(const uint16_t*)a, (const uint16_t*)b, parts, lda, ldb, N, K / splits, M / BM, N / BN, 1.0f, 0.0f, 4,
               (long long)M * N};
  const long long grid = (long long)p.nm * p.nn * splits;
  if (grid > 0x7fffffffLL) return -1;
  hipLaunchKernelGGL((gemm_tn_kernel<true>), dim3((unsigned)grid), dim3(256), 0, stream, p);
  return (int)hipGetLastError();
}
