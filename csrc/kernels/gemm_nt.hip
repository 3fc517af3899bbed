// Projection GEMM for gfx950:  C[M, N] = alpha A[M, K] . B[N, K]^T (+ beta C) with a fused epilogue.
//
// Both operands are stored K-contiguous (activations [tokens, in], weights [out, in]; the backward
// input-gradient GEMM hands the transposed frozen weight, also K-contiguous) -- every base GEMM of
// a LoRA / QLoRA step has this form (ops/linear.py).  Reference workload: the projections of the
// LoRA job spec the control plane launches (/root/reference/app/models/base/finetuning.py:51-145 --
// the reference itself ships no training code).
//
// Geometry: one 512-thread workgroup (8 waves, two per SIMD, one workgroup per CU) owns a 256 x 256
// tile of C; wave w = (wm, wn) = (w >> 2, w & 3) owns 128 (M) x 64 (N) as 8 x 4 accumulators of
// v_mfma_f32_16x16x32_bf16 (the 16x16 shape holds a higher clock than 32x32 on random data at equal
// cycles per FLOP -- MI355X_MICROARCH "DVFS give-back" item 7).
//
// Pipeline: K advances in 32-deep tiles through a 4-stage LDS ring (4 x [A 256x32 | B 256x32] bf16 =
// 128 KiB), filled by LDS-DMA (buffer_load_dwordx4 ... lds, 16 B per lane) two tiles ahead.  Each
// tile is two phases per wave (rows 0-63 / 64-127 of the wave's M range, 16 MFMAs each):
//     [ds_read fragments for phase | 2 DMA pieces of tile t+2] barrier [16 MFMA] barrier
// and the two waves of every SIMD run half a phase apart (waves 4-7 pass one extra barrier first), so
// at every barrier interval one wave of each SIMD reads LDS / issues DMA while its partner keeps the
// matrix pipe busy (ping-pong).  DMA completion is counted per wave (vmcnt(4) = tile t+1 landed, tile
// t+2 still flying) and published by the next barrier; a stage is re-filled only after the barrier
// that follows the last wave's lgkmcnt(0) on it (four intervals of margin).
//
// LDS image: [row][32 k] bf16 = 64-byte rows, 16-byte chunk c stored at c ^ ((row >> 2) & 2) --
// conflict-free for the ds_read_b128 fragment reads of both operands (lane groups of MI355X_MICROARCH
// §LDS; checked by tools/lds_banks.py).  The swizzle is applied to the per-lane DMA SOURCE address so
// the LDS side stays lane-linear (guide rule 21).
//
// Output layout: the MFMA is fed (A operand = B rows, B operand = A rows), so lane l ends up holding
// C[m = l & 15][n = 4 (l >> 4) + 0..3] of each 16x16 tile; B fragment rows are read permuted inside each
// 32-column pair so that the two tiles of a pair give every lane 8 CONSECUTIVE columns: one 16-byte
// store per lane per (m tile, pair).
//
// Block -> tile: XCD-bijective remap (each XCD owns a contiguous run of logical tiles), then groups of
// group_m M-blocks x all N-blocks with M fastest, so the ~32 tiles resident on one XCD share a few A
// and B panels in its L2.
#include "common.h"

#include <cstdlib>
#include <type_traits>

using namespace ftc;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int BM = 256, BN = 256, BK = 32;
constexpr int IMG = 256 * BK * 2;  // one operand image: 16 KiB
constexpr int STAGE = 2 * IMG;     // A | B
constexpr int NSTAGE = 4;

enum Epi : int {
  EPI_STORE = 0,  // C = alpha acc (+ beta C), bf16 or fp32
  EPI_ROPE = 1,   // bf16 C = rope(alpha acc) on the q / k heads (the packed qkv projection), beta 0
};

struct NTArgs {
  const uint16_t* a;  // [M, lda]
  const uint16_t* b;  // [N, ldb]
  void* c;            // [M, ldc]
  long long lda, ldb, ldc;
  int K, nm, nn, group_m;
  float alpha, beta;
  // EPI_ROPE (head_dim 128): rotate the first rot_heads 128-column heads of every output row by
  // (cos, sin)[pos] (fp32 [max_pos, 64], HF rotate_half pairs (i, i + 64)); pos = positions[row] or
  // row % seq_len
  const float* cos_t;
  const float* sin_t;
  const int* positions;
  int seq_len, rot_heads;
  // variant 7: K-loop stagger -- workgroup b starts at super-stage ((b & stagger_mask) * stagger_step) % ns
  // and wraps, so co-running tiles do not stream the same K columns (the same HBM channel offsets) in
  // lockstep
  int stagger_mask, stagger_step;
};

FTC_DEV int swz(int row) { return (row >> 2) & 2; }

// ---- pieces shared by the kernel variants --------------------------------------------------------

// block -> (M block, N block): XCD-bijective remap, then group_m M-blocks x all N-blocks, M fastest
FTC_DEV void tile_of(const NTArgs& p, int& mb, int& nb) {
  const int nblk = p.nm * p.nn, bid = blockIdx.x;
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

// LDS-DMA of one K-tile: wave w fills rows [32 w, 32 w + 32) of both images, 2 pieces of 16 rows each.
// Lane i of a piece lands at row r0 + (i >> 2), physical chunk i & 3, which holds logical chunk
// (i & 3) ^ swz(row); swz only sees row bits 2-3, so both pieces share one per-lane source offset (+16
// rows as the scalar offset).
struct Dma {
  __amdgpu_buffer_rsrc_t ra, rb;
  int voa, vob, sa16, sb16;
  char* da;  // this wave's rows of the A image of stage 0 (B image = + IMG)

  FTC_DEV Dma(const NTArgs& p, long long m0, long long n0, char* S, int wave, int lane) {
    const int r = 32 * wave + (lane >> 2);
    const int c = (lane & 3) ^ swz(r);
    voa = (int)((r * p.lda + 8 * c) * 2);
    vob = (int)((r * p.ldb + 8 * c) * 2);
    sa16 = (int)(16 * p.lda * 2);
    sb16 = (int)(16 * p.ldb * 2);
    ra = make_rsrc(p.a + m0 * p.lda);
    rb = make_rsrc(p.b + n0 * p.ldb);
    da = S + 32 * wave * 64;
  }
  // piece j (0..3) of tile kt: A rows +0 / +16, B rows +0 / +16
  FTC_DEV void piece(int kt, int j, int stage_of) const {
    char* d = da + (stage_of & (NSTAGE - 1)) * STAGE + (j >> 1) * IMG + (j & 1) * 1024;
    const int so = kt * BK * 2 + ((j & 1) ? ((j >> 1) ? sb16 : sa16) : 0);
    lds_dma16((j >> 1) ? rb : ra, d, (j >> 1) ? vob : voa, so);
  }
  FTC_DEV void piece(int kt, int j) const { piece(kt, j, kt); }
  // register staging of the same piece: a 16-byte load per lane, then a lane-linear ds_write_b128
  FTC_DEV u32x4 load(int kt, int j) const {
    const int so = kt * BK * 2 + ((j & 1) ? ((j >> 1) ? sb16 : sa16) : 0);
    return buf_load16((j >> 1) ? rb : ra, (j >> 1) ? vob : voa, so);
  }
  FTC_DEV void store(int stage, int j, const u32x4& v, int lane) const {
    char* d = da + (stage & (NSTAGE - 1)) * STAGE + (j >> 1) * IMG + (j & 1) * 1024 + lane * 16;
    *reinterpret_cast<u32x4*>(d) = v;
  }
  FTC_DEV void tile(int kt) const {
#pragma unroll
    for (int j = 0; j < 4; ++j) piece(kt, j);
  }
};

FTC_DEV bf16x8 rd(const char* s, int off) { return *reinterpret_cast<const bf16x8*>(s + off); }

// Epilogue: lane holds C[m0 + wm 128 + 16 mt + li][n0 + wn 64 + 32 pr + 8 kc + 0..7] in acc[mt][2 pr]
// (columns +0..3) and acc[mt][2 pr + 1] (+4..7): one 16-byte (bf16) / two 16-byte (fp32) stores.
template <bool F32C, int MT, int NT>
FTC_DEV void store_wave(const NTArgs& p, const f32x4 (&acc)[MT][NT], long long row0, long long col0, int lane) {
  const int li = lane & 15, kc = lane >> 4;
  const long long mrow = row0 + li;
  const long long ncol = col0 + 8 * kc;
  const bool accumulate = p.beta != 0.f;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int pr = 0; pr < NT / 2; ++pr) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = p.alpha * acc[mt][2 * pr][j];
        v[4 + j] = p.alpha * acc[mt][2 * pr + 1][j];
      }
      const long long off = (mrow + 16 * mt) * p.ldc + ncol + 32 * pr;
      if constexpr (F32C) {
        float4* cp = reinterpret_cast<float4*>(reinterpret_cast<float*>(p.c) + off);
        if (accumulate) {
          const float4 o0 = cp[0], o1 = cp[1];
          v[0] += p.beta * o0.x; v[1] += p.beta * o0.y; v[2] += p.beta * o0.z; v[3] += p.beta * o0.w;
          v[4] += p.beta * o1.x; v[5] += p.beta * o1.y; v[6] += p.beta * o1.z; v[7] += p.beta * o1.w;
        }
        cp[0] = make_float4(v[0], v[1], v[2], v[3]);
        cp[1] = make_float4(v[4], v[5], v[6], v[7]);
      } else {
        uint4* cp = reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(p.c) + off);
        if (accumulate) {
          float o[8];
          unpack8(*cp, o);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] += p.beta * o[j];
        }
        *cp = pack8(v);
      }
    }
}

// Epilogue of the 8-wave kernels: lane holds C[m0 + wm 128 + 16 mt + li][n0 + wn 64 + 32 pr + 8 kc + 0..7] in
// acc[mt][2 pr] (columns +0..3) and acc[mt][2 pr + 1] (+4..7): one 16-byte (bf16) / two (fp32) stores.
template <bool F32C>
FTC_DEV void store_tile(const NTArgs& p, const f32x4 (&acc)[8][4], long long m0, long long n0, int wm, int wn,
                        int lane) {
  store_wave<F32C, 8, 4>(p, acc, m0 + wm * 128, n0 + wn * 64, lane);
}

FTC_DEV void barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// Fragment read offsets (bytes inside a stage).  A: rows wm 128 + 16 mt + (lane & 15) at a_off + mt 1024.
// B: tile nt of the wave reads rows wn 64 + 32 (nt >> 1) + 4 (nt & 1) + 8 ((lane & 15) >> 2) + (lane & 3),
// so that the MFMA output row 4 q + j of tiles 2 p and 2 p + 1 is column 32 p + 8 q + j and + 4 + j.
FTC_DEV int a_frag_off(int wm, int lane) {
  const int li = lane & 15, kc = lane >> 4;
  return (wm * 128 + li) * 64 + 16 * (kc ^ swz(li));
}
FTC_DEV int b_frag_off(int wn, int lane) {
  const int li = lane & 15, kc = lane >> 4;
  const int brow = wn * 64 + 8 * (li >> 2) + (li & 3);
  return IMG + brow * 64 + 16 * (kc ^ swz(brow));
}
FTC_DEV constexpr int b_nt(int nt) { return (32 * (nt >> 1) + 4 * (nt & 1)) * 64; }

// ---- variant 1 (default): register-double-buffered fragments, one barrier per K-tile ------------------
//
// Iteration t: DMA tile t+3 into stage (t+3) % 4 (held tile t-1, whose fragments every wave read before
// the previous barrier), 32 MFMAs of tile t from register set X interleaved with the ds_reads of tile
// t+1 into set Y, then vmcnt (tile t+2 landed: only tile t+3's 4 pieces may still fly) and ONE barrier
// that publishes tile t+2.  The two waves of a SIMD interleave freely; the barrier costs only the
// arrival skew once per 32 MFMAs per wave.  Two named register sets, loop unrolled by 2 (guide rule 20).
// MODE (diagnostics only, FTC_GEMM_NT_MODE; results are garbage): bit 0 skips the DMA wait, bit 1 the
// loop's DMA, bit 2 the loop's barrier; bit 3 makes every DMA re-read K-tile 0 (L2-resident operands).
template <bool F32C, int MODE = 0>
__global__ __launch_bounds__(512, 1) void gemm_nt_kernel(NTArgs p) {
  __shared__ __attribute__((aligned(16))) char S[NSTAGE * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  int mb, nb;
  tile_of(p, mb, nb);
  const long long m0 = (long long)mb * BM, n0 = (long long)nb * BN;
  const Dma dma(p, m0, n0, S, wave, lane);
  const int a_off = a_frag_off(wm, lane), b_off = b_frag_off(wn, lane);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / BK;  // even (host contract)
  bf16x8 xa[8], xb[4], ya[8], yb[4];

  // one iteration: compute from (ca, cb), read tile t+1 into (na, nb_)
  // No branches in the body: past the last tile the reads fetch a dead stage (discarded) and the DMA
  // re-fetches tile nk-1 into the dead stage (t+3) % 4 (never read; keeps the vmcnt count uniform).
  auto iter = [&](int t, const bf16x8 (&ca)[8], const bf16x8 (&cb)[4], bf16x8 (&na)[8], bf16x8 (&nb_)[4])
      __attribute__((always_inline)) {
    const int tdma = min(t + 3, nk - 1);
    const int sdma = t + 3;
    const char* st = S + ((t + 1) & (NSTAGE - 1)) * STAGE;
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cb[nt], ca[mt], acc[mt][nt], 0, 0, 0);
      na[mt] = rd(st, a_off + mt * 1024);
      if (mt < 4) nb_[mt] = rd(st, b_off + b_nt(mt));
      if (!(MODE & 2)) {
        if constexpr (MODE & 16) {
          // the two waves of a SIMD (wm 0 / 1) issue their DMA pieces after different MFMA groups, so
          // one wave's DMA issue stall falls where its partner is issuing MFMAs
          if ((mt & 1) == wm) dma.piece((MODE & 8) ? 0 : tdma, mt >> 1, sdma);
        } else if ((mt & 1) == 0 && (!(MODE & 32) || mt < 4)) {  // MODE 32: A pieces only
          dma.piece((MODE & 8) ? 0 : tdma, mt >> 1, sdma);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (!(MODE & 1)) __builtin_amdgcn_s_waitcnt(0x0F74);  // vmcnt(4): tile t+2 landed, only the 4 pieces just issued fly
    if (!(MODE & 4)) barrier();
  };

  // prologue: tiles 0, 1, 2 in flight; tiles 0 and 1 landed and published; tile 0 into set X
  dma.tile(0);
  dma.tile(1);  // nk >= 2 (even)
#pragma unroll
  for (int j = 0; j < 4; ++j) dma.piece(min(2, nk - 1), j, 2);
  __builtin_amdgcn_s_waitcnt(0x0F74);  // vmcnt(4): tiles 0 and 1 landed
  barrier();
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) xa[mt] = rd(S, a_off + mt * 1024);
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) xb[nt] = rd(S, b_off + b_nt(nt));

  for (int t = 0; t < nk; t += 2) {
    iter(t, xa, xb, ya, yb);
    iter(t + 1, ya, yb, xa, xb);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): no DMA may land in LDS after the workgroup ends
  store_tile<F32C>(p, acc, m0, n0, wm, wn, lane);
}

// ---- variant 2: as variant 1, with the K-tiles staged through registers instead of LDS-DMA ----------
// An LDS-DMA piece costs its wave ~60-185 issue cycles among MFMAs (MI355X_MICROARCH cycle table): at 4
// pieces per 32 MFMAs that was a 25 % loss (variant 1 with the loop's DMA switched off: 1.60 PF vs
// 1.27).  Here iteration t ds_writes tile t+2 (loaded into 16 staging VGPRs during iteration t-1) into
// stage (t+2) % 4 and re-issues the staging loads for tile t+3; lgkmcnt(0) before the barrier makes
// the writes visible to the reads of iteration t+1.
template <bool F32C>
__global__ __launch_bounds__(512, 1) void gemm_nt_rs_kernel(NTArgs p) {
  __shared__ __attribute__((aligned(16))) char S[NSTAGE * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  int mb, nb;
  tile_of(p, mb, nb);
  const long long m0 = (long long)mb * BM, n0 = (long long)nb * BN;
  const Dma dma(p, m0, n0, S, wave, lane);
  const int a_off = a_frag_off(wm, lane), b_off = b_frag_off(wn, lane);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / BK;  // even (host contract)
  // A fragments: ONE set -- the next tile's fragment mt is read into fa[mt] right after the 4 MFMAs that
  // consume it; B fragments (read by all 8 groups): two named sets alternating per iteration
  bf16x8 fa[8], xb[4], yb[4];
  u32x4 rs[4];

  auto iter = [&](int t, const bf16x8 (&cb)[4], bf16x8 (&nb_)[4]) __attribute__((always_inline)) {
    const int tld = min(t + 3, nk - 1);
    const char* st = S + ((t + 1) & (NSTAGE - 1)) * STAGE;
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cb[nt], fa[mt], acc[mt][nt], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);  // the MFMAs read fa[mt] before it is reloaded (same registers)
      fa[mt] = rd(st, a_off + mt * 1024);
      if (mt < 4) nb_[mt] = rd(st, b_off + b_nt(mt));
      if (mt & 1) {
        const int j = mt >> 1;
        dma.store(t + 2, j, rs[j], lane);  // tile t+2 (past the end: a dead stage)
        rs[j] = dma.load(tld, j);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's writes of tile t+2 are in LDS
    barrier();
  };

  // prologue: tiles 0 and 1 through registers into stages 0 / 1, tile 2 into the staging registers
#pragma unroll
  for (int j = 0; j < 4; ++j) rs[j] = dma.load(0, j);
#pragma unroll
  for (int j = 0; j < 4; ++j) dma.store(0, j, rs[j], lane);
#pragma unroll
  for (int j = 0; j < 4; ++j) rs[j] = dma.load(1, j);
#pragma unroll
  for (int j = 0; j < 4; ++j) dma.store(1, j, rs[j], lane);
#pragma unroll
  for (int j = 0; j < 4; ++j) rs[j] = dma.load(min(2, nk - 1), j);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  barrier();
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) fa[mt] = rd(S, a_off + mt * 1024);
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) xb[nt] = rd(S, b_off + b_nt(nt));

  for (int t = 0; t < nk; t += 2) {
    iter(t, xb, yb);
    iter(t + 1, yb, xb);
  }
  store_tile<F32C>(p, acc, m0, n0, wm, wn, lane);
}

// ---- packed-B kernel: the weight operand never touches LDS ---------------------------------------------
// Variant 1 with the loop's DMA switched off runs 1.60 PF against 1.27 with it: the LDS, not the matrix
// pipe, is the limiter -- per 32-deep tile a CU writes 32 KiB (ds_write_b128 ~79 B/clk) and reads 96 KiB.
// Here B (the frozen projection weight -- or its transposed copy for the input-gradient GEMM) is stored
// once in MFMA fragment order ("packed", pack_b_nt in ops/gemm.py): [N/32][K/32][2][64 lanes][8], so a
// wave's 16x32 B fragment is ONE coalesced 1 KiB buffer_load straight into VGPRs.  Only A goes through
// LDS (register-staged: buffer_load -> ds_write_b128 two tiles ahead), halving the LDS write traffic and
// cutting the reads by a third.  Every memory op is compiler-visible, so hipcc counts vmcnt exactly.
//
// Iteration t: the MFMAs of tile t (A fragments of tile t in fa, B fragments in cb) interleaved with
//   the A fragment reads of tile t+1 (LDS) into fa (each after its last use), the B fragment loads of
//   tile t+1 (global) into nb_, the ds_writes of A tile t+2 from the staging registers and their
//   re-load with A tile t+3; lgkmcnt(0) and one barrier publish tile t+2.
struct PBArgs {
  const uint16_t* a;   // [M, lda]
  const uint16_t* bp;  // packed [N/32][K/32][2][64][8]
  void* c;             // [M, ldc]
  long long lda, ldc;
  int K, nm, nn, group_m;
  float alpha, beta;
};

// MODE (diagnostics, FTC_GEMM_NT_MODE; garbage results): bit 0 -- B loads re-read K-tile 0; bit 1 -- no A
// staging in the loop.
template <bool F32C, int MODE = 0>
__global__ __launch_bounds__(512, 1) void gemm_nt_pb_kernel(PBArgs p) {
  __shared__ __attribute__((aligned(16))) char S[NSTAGE * IMG];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  int mb, nb;
  {
    NTArgs q{};
    q.nm = p.nm;
    q.nn = p.nn;
    q.group_m = p.group_m;
    tile_of(q, mb, nb);
  }
  const long long m0 = (long long)mb * BM, n0 = (long long)nb * BN;
  const int nk = p.K / BK;  // even (host contract)

  // A staging: wave w owns rows [32 w, 32 w + 32) of the A image, 2 pieces of 16 rows
  int voa;
  {
    const int r = 32 * wave + (lane >> 2);
    voa = (int)((r * p.lda + 8 * ((lane & 3) ^ swz(r))) * 2);
  }
  const int sa16 = (int)(16 * p.lda * 2);
  const auto ra = make_rsrc(p.a + m0 * p.lda);
  char* const wa = S + 32 * wave * 64 + lane * 16;
  // B fragments: wave wn reads 32-column groups n0/32 + 2 wn + {0, 1}, 2 fragments each
  const int grp_bytes = nk * 2048;
  const auto rbp = make_rsrc(p.bp + (n0 >> 5) * (long long)nk * 1024);
  const int vob = lane * 16 + 2 * wn * grp_bytes;
  const int a_off = a_frag_off(wm, lane) - 0;  // A image at the stage base (no B image here)

  auto ldA = [&](int kt, int j) __attribute__((always_inline)) { return buf_load16(ra, voa, kt * BK * 2 + j * sa16); };
  auto stA = [&](int kt, int j, const u32x4& v) __attribute__((always_inline)) {
    *reinterpret_cast<u32x4*>(wa + (kt & (NSTAGE - 1)) * IMG + j * 1024) = v;
  };
  auto ldB = [&](int kt, int nt) __attribute__((always_inline)) {
    const bf16x8 v = __builtin_bit_cast(bf16x8, buf_load16(rbp, vob, kt * 2048 + (nt >> 1) * grp_bytes + (nt & 1) * 1024));
    return v;
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa[8], xb[4], yb[4];
  u32x4 rs[2];

  auto iter = [&](int t, const bf16x8 (&cb)[4], bf16x8 (&nb_)[4]) __attribute__((always_inline)) {
    const int tB = (MODE & 1) ? 0 : min(t + 1, nk - 1);
    const int tA = min(t + 3, nk - 1);
    const char* st = S + ((t + 1) & (NSTAGE - 1)) * IMG;
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cb[nt], fa[mt], acc[mt][nt], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);  // the MFMAs read fa[mt] before it is reloaded (same registers)
      fa[mt] = rd(st, a_off + mt * 1024);
      if (mt < 4) nb_[mt] = ldB(tB, mt);
      if ((mt == 1 || mt == 5) && !(MODE & 2)) {
        const int j = mt >> 2;
        stA(t + 2, j, rs[j]);  // A tile t+2 (past the end: a dead stage)
        rs[j] = ldA(tA, j);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's A writes of tile t+2 are in LDS
    barrier();
  };

  // prologue: A tiles 0, 1 into stages 0, 1; A tile 2 into the staging registers; B tile 0 into xb
#pragma unroll
  for (int j = 0; j < 2; ++j) rs[j] = ldA(0, j);
#pragma unroll
  for (int j = 0; j < 2; ++j) stA(0, j, rs[j]);
#pragma unroll
  for (int j = 0; j < 2; ++j) rs[j] = ldA(1, j);
#pragma unroll
  for (int j = 0; j < 2; ++j) stA(1, j, rs[j]);
#pragma unroll
  for (int j = 0; j < 2; ++j) rs[j] = ldA(min(2, nk - 1), j);
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) xb[nt] = ldB(0, nt);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  barrier();
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) fa[mt] = rd(S, a_off + mt * 1024);

  for (int t = 0; t < nk; t += 2) {
    iter(t, xb, yb);
    iter(t + 1, yb, xb);
  }
  NTArgs q{};
  q.c = p.c;
  q.ldc = p.ldc;
  q.alpha = p.alpha;
  q.beta = p.beta;
  store_tile<F32C>(q, acc, m0, n0, wm, wn, lane);
}

// ---- variant 4: one wave per SIMD, 128 x 128 per wave, register-staged loads -------------------------
// The LDS is the shared resource of the 8-wave kernels (per 32-deep tile a CU reads 96 KiB of fragments
// and writes 32 KiB): with 4 waves of 128 x 128 each fragment read feeds 8 MFMAs instead of 4 / 8, so
// the reads drop to 64 KiB.  One wave per SIMD (512 registers: 256 accumulators + fragments + staging)
// hides its own latencies: fragment reads of tile t+1 and the global loads of tile t+3 are issued
// between the MFMAs of tile t (register staging: a global_load / ds_write pair issues in a few cycles
// inside an MFMA's shadow, where an LDS-DMA piece would stall the wave ~60+ cycles with no partner wave
// to fill the pipe).
template <bool F32C>
__global__ __launch_bounds__(256, 1) void gemm_nt_w4_kernel(NTArgs p) {
  __shared__ __attribute__((aligned(16))) char S[NSTAGE * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  int mb, nb;
  tile_of(p, mb, nb);
  const long long m0 = (long long)mb * BM, n0 = (long long)nb * BN;
  const int nk = p.K / BK;  // even (host contract)

  // staging: wave w loads rows [64 w, 64 w + 64) of both images, 4 pieces of 16 rows each per operand
  int voa, vob;
  {
    const int r = 64 * wave + (lane >> 2);
    const int c = (lane & 3) ^ swz(r);
    voa = (int)((r * p.lda + 8 * c) * 2);
    vob = (int)((r * p.ldb + 8 * c) * 2);
  }
  const int sa16 = (int)(16 * p.lda * 2), sb16 = (int)(16 * p.ldb * 2);
  const auto ra = make_rsrc(p.a + m0 * p.lda);
  const auto rb = make_rsrc(p.b + n0 * p.ldb);
  char* const wdst = S + 64 * wave * 64 + lane * 16;
  // piece j: operand j >> 2, rows + 16 (j & 3)
  auto ld = [&](int kt, int j) __attribute__((always_inline)) {
    return buf_load16((j >> 2) ? rb : ra, (j >> 2) ? vob : voa, kt * BK * 2 + (j & 3) * ((j >> 2) ? sb16 : sa16));
  };
  auto st = [&](int kt, int j, const u32x4& v) __attribute__((always_inline)) {
    *reinterpret_cast<u32x4*>(wdst + (kt & (NSTAGE - 1)) * STAGE + (j >> 2) * IMG + (j & 3) * 1024) = v;
  };
  const int li = lane & 15, kc = lane >> 4;
  const int a_off = (wm * 128 + li) * 64 + 16 * (kc ^ swz(li));
  const int brow = wn * 128 + 8 * (li >> 2) + (li & 3);
  const int b_off = IMG + brow * 64 + 16 * (kc ^ swz(brow));

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa[8], xb[8], yb[8];
  u32x4 rs[8];

  auto iter = [&](int t, const bf16x8 (&cb)[8], bf16x8 (&nb_)[8]) __attribute__((always_inline)) {
    const int tld = min(t + 3, nk - 1);
    const char* sr = S + ((t + 1) & (NSTAGE - 1)) * STAGE;
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
#pragma unroll
      for (int nt = 0; nt < 8; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cb[nt], fa[mt], acc[mt][nt], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      fa[mt] = rd(sr, a_off + mt * 1024);
      nb_[mt] = rd(sr, b_off + b_nt(mt));
      st(t + 2, mt, rs[mt]);  // tile t+2 (past the end: a dead stage)
      rs[mt] = ld(tld, mt);
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's writes of tile t+2 are in LDS
    barrier();
  };

#pragma unroll
  for (int j = 0; j < 8; ++j) rs[j] = ld(0, j);
#pragma unroll
  for (int j = 0; j < 8; ++j) st(0, j, rs[j]);
#pragma unroll
  for (int j = 0; j < 8; ++j) rs[j] = ld(1, j);
#pragma unroll
  for (int j = 0; j < 8; ++j) st(1, j, rs[j]);
#pragma unroll
  for (int j = 0; j < 8; ++j) rs[j] = ld(min(2, nk - 1), j);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  barrier();
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) fa[mt] = rd(S, a_off + mt * 1024);
#pragma unroll
  for (int nt = 0; nt < 8; ++nt) xb[nt] = rd(S, b_off + b_nt(nt));

  for (int t = 0; t < nk; t += 2) {
    iter(t, xb, yb);
    iter(t + 1, yb, xb);
  }
  store_wave<F32C, 8, 8>(p, acc, m0 + wm * 128, n0 + wn * 128, lane);
}

// Epilogue of the head-aligned mapping: lane holds, for m tile mt, columns c0 + 8 kc + [0, 8) (pair 0:
// acc[mt][0..1]) and c0 + 64 + 8 kc + [0, 8) (pair 1: acc[mt][2..3]), c0 = n0 + 128 (wn >> 1) + 32 (wn & 1).
template <bool F32C, int EPI>
FTC_DEV void store_v5(const NTArgs& p, const f32x4 (&acc)[8][4], long long m0, long long n0, int wm, int wn,
                      int lane) {
  const int li = lane & 15, kc = lane >> 4;
  const long long mrow = m0 + wm * 128 + li;
  const long long c0 = n0 + 128 * (wn >> 1) + 32 * (wn & 1);
  const long long ncol = c0 + 8 * kc;
  const bool accumulate = p.beta != 0.f;
  bool rope = false;
  if constexpr (EPI == EPI_ROPE) rope = (int)(c0 >> 7) < p.rot_heads;  // wave-uniform
  const int ri = 32 * (wn & 1) + 8 * kc;  // rotation-pair index of this lane's first column (0..63)
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    float v[2][8];
#pragma unroll
    for (int pr = 0; pr < 2; ++pr)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[pr][j] = p.alpha * acc[mt][2 * pr][j];
        v[pr][4 + j] = p.alpha * acc[mt][2 * pr + 1][j];
      }
    const long long row = mrow + 16 * mt;
    if constexpr (EPI == EPI_ROPE) {
      if (rope) {
        const int pos = p.positions ? p.positions[row] : (int)(row % p.seq_len);
        const float4* cp = reinterpret_cast<const float4*>(p.cos_t + (long long)pos * 64 + ri);
        const float4* sp = reinterpret_cast<const float4*>(p.sin_t + (long long)pos * 64 + ri);
        const float4 c0v = cp[0], c1v = cp[1], s0v = sp[0], s1v = sp[1];
        const float cs[8] = {c0v.x, c0v.y, c0v.z, c0v.w, c1v.x, c1v.y, c1v.z, c1v.w};
        const float sn[8] = {s0v.x, s0v.y, s0v.z, s0v.w, s1v.x, s1v.y, s1v.z, s1v.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x1 = v[0][j], x2 = v[1][j];
          v[0][j] = x1 * cs[j] - x2 * sn[j];
          v[1][j] = x2 * cs[j] + x1 * sn[j];
        }
      }
    }
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const long long off = row * p.ldc + ncol + 64 * pr;
      if constexpr (F32C) {
        float4* cp = reinterpret_cast<float4*>(reinterpret_cast<float*>(p.c) + off);
        if (accumulate) {
          const float4 o0 = cp[0], o1 = cp[1];
          v[pr][0] += p.beta * o0.x; v[pr][1] += p.beta * o0.y; v[pr][2] += p.beta * o0.z; v[pr][3] += p.beta * o0.w;
          v[pr][4] += p.beta * o1.x; v[pr][5] += p.beta * o1.y; v[pr][6] += p.beta * o1.z; v[pr][7] += p.beta * o1.w;
        }
        cp[0] = make_float4(v[pr][0], v[pr][1], v[pr][2], v[pr][3]);
        cp[1] = make_float4(v[pr][4], v[pr][5], v[pr][6], v[pr][7]);
      } else {
        uint4* cp = reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(p.c) + off);
        if (accumulate) {
          float o[8];
          unpack8(*cp, o);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[pr][j] += p.beta * o[j];
        }
        *cp = pack8(v[pr]);
      }
    }
  }
}

// ---- variant 5 (default): 64-deep super-stages, full 128-byte lines per DMA row --------------------------
// rocprofv3 on variants 1-4 (profiles/r3/gemm_nt.md): the texture addresser was 95 % busy (hipBLASLt:
// 60 %) -- with 32-deep tiles every DMA row is a 64-byte HALF line, so a 1 KiB piece touches 16 cache
// lines instead of 8.  Here the LDS ring holds two 64-deep "super-stages" (A [256][64] | B [256][64],
// 64 KiB each, 128-byte rows), each DMA piece is 8 rows x 128 B, and the MFMA loop still walks 32-deep
// tiles (tile t = half t & 1 of super-stage t >> 1).  The 128-byte-row image is swizzled by
// f(R) = R0 | R1 << 1 | R3 << 2 on the 16-byte chunk (conflict-free for both fragment reads).
//
// Iteration t (32 MFMAs of tile t, fragment reads of tile t+1 into the other register set):
//   odd t:  8 DMA pieces of super-stage (t+3)/2 (tiles t+3, t+4) into the stage tiles t-1 / t held --
//           tile t's fragments are already in registers and every wave's reads of tile t-1 completed
//           before the previous barrier;
//   even t: vmcnt(0) (super-stage t/2+1 landed) + lgkmcnt(0) + barrier.
FTC_DEV int f5(int r) { return (r & 1) | (r & 2) | ((r >> 1) & 4); }

// Column mapping: wave wn owns columns 128 (wn >> 1) + 32 (wn & 1) + [0, 32) and the same + 64 -- the two
// halves of one 128-wide head that HF's rotate_half pairs up -- so a RoPE epilogue finds both elements
// of every rotation pair in one lane, one register apart.
// MODE (FTC_GEMM_NT_V5_MODE): bit 0 skips the DMA wait and bit 1 the loop's DMA (diagnostics: garbage
// results); bit 2 issues an odd iteration's 8 DMA pieces up front instead of one per MFMA group (real);
// bit 3 stages through registers instead of LDS-DMA (real): odd iteration t loads super-stage
// (t+3)/2 into 8 x 16 B per lane, even iteration t+1 ds_writes them (the stage is dead by then) before
// its barrier.
template <bool F32C, int EPI = EPI_STORE, int MODE = 0>
__global__ __launch_bounds__(512, 1) void gemm_nt_v5_kernel(NTArgs p) {
  constexpr int IMG2 = 256 * 64 * 2;  // one operand image of a super-stage: 32 KiB
  constexpr int SS = 2 * IMG2;        // super-stage: A | B
  __shared__ __attribute__((aligned(16))) char S[2 * SS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  int mb, nb;
  tile_of(p, mb, nb);
  const long long m0 = (long long)mb * BM, n0 = (long long)nb * BN;
  const int nk = p.K / BK;  // even (host contract)
  const int ns = nk >> 1;   // super-stages

  // DMA: wave w fills rows [32 w, 32 w + 32) of both images as 4 pieces of 8 rows x 128 B; lane i -> row
  // +(i >> 3), physical chunk i & 7 = logical chunk (i & 7) ^ f5(row).  Piece sub's rows start at 8 sub,
  // so row bit 3 = sub & 1: one per-lane source offset per parity.
  int vo[2][2];  // [operand][parity]
  {
    const int rr = lane >> 3, pc = lane & 7;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int lc = pc ^ f5(rr + 8 * q);
      vo[0][q] = (int)(((32 * wave + rr) * p.lda + 8 * lc) * 2);
      vo[1][q] = (int)(((32 * wave + rr) * p.ldb + 8 * lc) * 2);
    }
  }
  const int s8a = (int)(8 * p.lda * 2), s8b = (int)(8 * p.ldb * 2);
  const auto ra = make_rsrc(p.a + m0 * p.lda);
  const auto rb = make_rsrc(p.b + n0 * p.ldb);
  char* const ddst = S + 32 * wave * 128;
  // piece j (0..7) of super-stage ss: operand j >> 2, rows 32 w + 8 (j & 3)
  auto piece = [&](int ss_src, int ss_dst, int j) __attribute__((always_inline)) {
    const int op = j >> 2, sub = j & 3;
    char* d = ddst + (ss_dst & 1) * SS + op * IMG2 + sub * 1024;
    const int so = ss_src * 128 + sub * (op ? s8b : s8a);
    lds_dma16(op ? rb : ra, d, vo[op][sub & 1], so);
  };

  const int li = lane & 15, kc = lane >> 4;
  int a_off[2], b_off[2];
  {
    const int ra_ = wm * 128 + li;
    const int rb_ = 128 * (wn >> 1) + 32 * (wn & 1) + 8 * (li >> 2) + (li & 3);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      a_off[h] = ra_ * 128 + 16 * ((4 * h + kc) ^ f5(li));
      b_off[h] = IMG2 + rb_ * 128 + 16 * ((4 * h + kc) ^ f5(rb_));
    }
  }
  auto bnt = [](int nt) { return (64 * (nt >> 1) + 4 * (nt & 1)) * 128; };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa[8], xb[4], yb[4];
  constexpr bool RS = (MODE & 8) != 0;
  u32x4 rs[RS ? 8 : 1];
  auto rs_load = [&](int ss_src, int j) __attribute__((always_inline)) {
    const int op = j >> 2, sub = j & 3;
    return buf_load16(op ? rb : ra, vo[op][sub & 1], ss_src * 128 + sub * (op ? s8b : s8a));
  };
  auto rs_store = [&](int ss_dst, int j, const u32x4& v) __attribute__((always_inline)) {
    const int op = j >> 2, sub = j & 3;
    *reinterpret_cast<u32x4*>(ddst + (ss_dst & 1) * SS + op * IMG2 + sub * 1024 + lane * 16) = v;
  };

  // ODD: compile-time parity of t (the loop is unrolled by 2)
  auto iter = [&](int t, auto odd_c, const bf16x8 (&cb)[4], bf16x8 (&nb_)[4]) __attribute__((always_inline)) {
    constexpr bool ODD = decltype(odd_c)::value;
    const int tn = t + 1;  // fragments of tile t+1 (past the end: a dead read)
    const char* st = S + ((tn >> 1) & 1) * SS;
    const int h = ODD ? 0 : 1;  // tn & 1
    const int dsrc = min((t + 3) >> 1, ns - 1), ddst_ss = (t + 3) >> 1;
    if constexpr (ODD && (MODE & 4) && !(MODE & 2)) {
#pragma unroll
      for (int j = 0; j < 8; ++j) piece(dsrc, ddst_ss, j);
    }
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      if constexpr (MODE & 32) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cb[nt], fa[mt], acc[mt][nt], 0, 0, 0);
      if constexpr (MODE & 32) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);  // the MFMAs read fa[mt] before it is reloaded (same registers)
      fa[mt] = rd(st, a_off[h] + mt * 2048);
      if (mt < 4) nb_[mt] = rd(st, b_off[h] + bnt(mt));
      if constexpr (RS) {
        if constexpr (ODD)
          rs[mt] = rs_load(dsrc, mt);
        else
          rs_store((t + 2) >> 1, mt, rs[mt]);  // super-stage t/2+1 (past the end: a dead stage)
      } else if constexpr (ODD && (MODE & 16)) {
        // the two waves of a SIMD (wm 0 / 1) issue their pieces in different halves of the iteration, so
        // one wave's DMA issue never coincides with its partner's
        if ((mt >> 2) == wm) {
          piece(dsrc, ddst_ss, 2 * (mt & 3));
          piece(dsrc, ddst_ss, 2 * (mt & 3) + 1);
        }
      } else if constexpr (ODD && !(MODE & 6)) {
        piece(dsrc, ddst_ss, mt);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (!ODD) {
      if constexpr (MODE & 1)
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only
      else
        __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) + lgkmcnt(0): super-stage t/2+1 landed, reads done
      barrier();
    }
  };

  // prologue: super-stages 0 and 1 in flight, wait for 0
  if constexpr (RS) {
#pragma unroll
    for (int j = 0; j < 8; ++j) rs[j] = rs_load(0, j);
#pragma unroll
    for (int j = 0; j < 8; ++j) rs_store(0, j, rs[j]);
#pragma unroll
    for (int j = 0; j < 8; ++j) rs[j] = rs_load(min(1, ns - 1), j);
#pragma unroll
    for (int j = 0; j < 8; ++j) rs_store(1, j, rs[j]);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) piece(0, 0, j);
#pragma unroll
    for (int j = 0; j < 8; ++j) piece(min(1, ns - 1), 1, j);
    __builtin_amdgcn_s_waitcnt(0x0F78);  // vmcnt(8)
  }
  barrier();
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) fa[mt] = rd(S, a_off[0] + mt * 2048);
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) xb[nt] = rd(S, b_off[0] + bnt(nt));

  for (int t = 0; t < nk; t += 2) {
    iter(t, std::false_type{}, xb, yb);
    iter(t + 1, std::true_type{}, yb, xb);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): no DMA may land in LDS after the workgroup ends
  store_v5<F32C, EPI>(p, acc, m0, n0, wm, wn, lane);
}

// ---- variant 6: one wave per SIMD, 128 x 128 per wave, 64-deep super-stages, register staging ---------
// The 8-wave kernels pay ~17 % for moving operands into LDS even once the texture addresser is relieved
// (variant 5 with the loop's DMA removed: 1.59-1.63 PF, above hipBLASLt).  Here 4 waves own 128 x 128 each
// (256 accumulators in AGPRs): a fragment read feeds 8 MFMAs, per 64-deep super-stage a wave issues 16
// global_load_dwordx4 (odd iteration) and 16 ds_write_b128 (even iteration) into the shadows of 128
// MFMAs -- a register-staging load issues in a few cycles where an LDS-DMA piece would stall the lone
// wave ~60-185 cycles.  Same 128-byte-row image and swizzle as variant 5.
template <bool F32C>
__global__ __launch_bounds__(256, 1) void gemm_nt_w4s_kernel(NTArgs p) {
  constexpr int IMG2 = 256 * 64 * 2;
  constexpr int SS = 2 * IMG2;
  __shared__ __attribute__((aligned(16))) char S[2 * SS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  int mb, nb;
  tile_of(p, mb, nb);
  const long long m0 = (long long)mb * BM, n0 = (long long)nb * BN;
  const int nk = p.K / BK;
  const int ns = nk >> 1;

  // staging: wave w fills rows [64 w, 64 w + 64) of both images: 8 pieces of 8 rows x 128 B per operand
  int vo[2][2];
  {
    const int rr = lane >> 3, pc = lane & 7;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int lc = pc ^ f5(rr + 8 * q);
      vo[0][q] = (int)(((64 * wave + rr) * p.lda + 8 * lc) * 2);
      vo[1][q] = (int)(((64 * wave + rr) * p.ldb + 8 * lc) * 2);
    }
  }
  const int s8a = (int)(8 * p.lda * 2), s8b = (int)(8 * p.ldb * 2);
  const auto ra = make_rsrc(p.a + m0 * p.lda);
  const auto rb = make_rsrc(p.b + n0 * p.ldb);
  char* const wdst = S + 64 * wave * 128 + lane * 16;
  // piece j (0..15): operand j >> 3, rows 64 w + 8 (j & 7)
  auto ld = [&](int ss_src, int j) __attribute__((always_inline)) {
    const int op = j >> 3, sub = j & 7;
    return buf_load16(op ? rb : ra, vo[op][sub & 1], ss_src * 128 + sub * (op ? s8b : s8a));
  };
  auto st = [&](int ss_dst, int j, const u32x4& v) __attribute__((always_inline)) {
    const int op = j >> 3, sub = j & 7;
    *reinterpret_cast<u32x4*>(wdst + (ss_dst & 1) * SS + op * IMG2 + sub * 1024) = v;
  };

  const int li = lane & 15, kc = lane >> 4;
  int a_off[2], b_off[2];
  {
    const int ra_ = wm * 128 + li;
    // store_wave's mapping: tiles 2 p, 2 p + 1 give columns 128 wn + 32 p + 8 kc + [0, 8)
    const int rb_ = 128 * wn + 8 * (li >> 2) + (li & 3);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      a_off[h] = ra_ * 128 + 16 * ((4 * h + kc) ^ f5(li));
      b_off[h] = IMG2 + rb_ * 128 + 16 * ((4 * h + kc) ^ f5(rb_));
    }
  }
  // B fragment nt (0..7): 32-column group g = nt >> 1 at offset 32 g, rows +4 (nt & 1)
  auto bnt = [](int nt) { return (32 * (nt >> 1) + 4 * (nt & 1)) * 128; };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa[8], xb[8], yb[8];
  u32x4 rs[16];

  auto iter = [&](int t, auto odd_c, const bf16x8 (&cb)[8], bf16x8 (&nb_)[8]) __attribute__((always_inline)) {
    constexpr bool ODD = decltype(odd_c)::value;
    const int tn = t + 1;
    const char* sr = S + ((tn >> 1) & 1) * SS;
    const int h = ODD ? 0 : 1;
    const int lsrc = min((t + 3) >> 1, ns - 1);
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
#pragma unroll
      for (int nt = 0; nt < 8; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cb[nt], fa[mt], acc[mt][nt], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      fa[mt] = rd(sr, a_off[h] + mt * 2048);
      nb_[mt] = rd(sr, b_off[h] + bnt(mt));
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        if constexpr (ODD)
          rs[2 * mt + k] = ld(lsrc, 2 * mt + k);
        else
          st((t + 2) >> 1, 2 * mt + k, rs[2 * mt + k]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (!ODD) {
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's writes of super-stage t/2+1 landed
      barrier();
    }
  };

#pragma unroll
  for (int j = 0; j < 16; ++j) rs[j] = ld(0, j);
#pragma unroll
  for (int j = 0; j < 16; ++j) st(0, j, rs[j]);
#pragma unroll
  for (int j = 0; j < 16; ++j) rs[j] = ld(min(1, ns - 1), j);
#pragma unroll
  for (int j = 0; j < 16; ++j) st(1, j, rs[j]);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  barrier();
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) fa[mt] = rd(S, a_off[0] + mt * 2048);
#pragma unroll
  for (int nt = 0; nt < 8; ++nt) xb[nt] = rd(S, b_off[0] + bnt(nt));

  for (int t = 0; t < nk; t += 2) {
    iter(t, std::false_type{}, xb, yb);
    iter(t + 1, std::true_type{}, yb, xb);
  }
  store_wave<F32C, 8, 8>(p, acc, m0 + wm * 128, n0 + wn * 128, lane);
}

// Epilogue of the 128 x 128 wave tile (store_wave's mapping): lane holds, for m tile mt, columns
// c0 + 32 pr + 8 kc + [0, 8) in acc[mt][2 pr .. 2 pr + 1], c0 = the wave's first column -- a whole
// 128-wide head when c0 % 128 == 0, so RoPE's rotate_half partners (d, d + 64) are pairs pr / pr + 2 of
// the same lane.
template <bool F32C, int EPI>
FTC_DEV void store_w128(const NTArgs& p, const f32x4 (&acc)[8][8], long long row0, long long c0, int lane) {
  if constexpr (EPI == EPI_STORE) {
    store_wave<F32C, 8, 8>(p, acc, row0, c0, lane);
  } else {
    static_assert(!F32C, "RoPE epilogue is bf16");
    const int li = lane & 15, kc = lane >> 4;
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
          const float4* cp = reinterpret_cast<const float4*>(p.cos_t + (long long)pos * 64 + ri);
          const float4* sp = reinterpret_cast<const float4*>(p.sin_t + (long long)pos * 64 + ri);
          const float4 c0v = cp[0], c1v = cp[1], s0v = sp[0], s1v = sp[1];
          const float cs[8] = {c0v.x, c0v.y, c0v.z, c0v.w, c1v.x, c1v.y, c1v.z, c1v.w};
          const float sn[8] = {s0v.x, s0v.y, s0v.z, s0v.w, s1v.x, s1v.y, s1v.z, s1v.w};
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float x1 = v[0][j], x2 = v[1][j];
            v[0][j] = x1 * cs[j] - x2 * sn[j];
            v[1][j] = x2 * cs[j] + x1 * sn[j];
          }
        }
#pragma unroll
        for (int q = 0; q < 2; ++q)
          *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(p.c) + row * p.ldc + c0 + 64 * q + 32 * h + 8 * kc) =
              pack8(v[q]);
      }
    }
  }
}

// ---- variant 7: one wave per SIMD with LDS-DMA, A/B-split release barriers -----------------------------
// 4 waves own 128 x 128 each (256 AGPR accumulators, two full fragment sets X / Y of 8 A + 8 B), two
// 64 KiB LDS buffers in variant 5's 128-byte-row image.  Iteration s computes super-stage s from buffer
// s & 1 in two 32-deep halves and refills THAT buffer with super-stage s + 2 as soon as its regions are
// released: half 0 reads Y.A, then (lgkmcnt + barrier: every wave is done with the A region) the 8 A
// pieces of s + 2 go out between the MFMAs while Y.B is read; the barrier at the end of half 0 frees the
// B region for its 8 pieces in half 1; a vmcnt + barrier in the middle of half 1 makes super-stage s + 1
// (issued one iteration earlier) visible and the X fragments of s + 1 are read under the last 32 MFMAs.
// Every DMA / LDS read sits between MFMAs of a dense 128-MFMA chain.  Three barriers per 64-deep step.
// Spread schedule (variant 7, MODE bit 7): the 16 pieces of super-stage s + 2 sit after MFMAs
// 41, 47, ..., 127 of the iteration's 128 (one per ~5.5 MFMAs instead of bursts of one per 4), piece i
// after MFMA 41 + 2 floor(43 i / 15); the 10 issued before MFMA 96 are what the s + 1 wait skips.
FTC_DEV constexpr int v7_piece(int idx) {
  if (idx < 41 || !(idx & 1)) return -1;
  const int d = (idx - 41) / 2;
  for (int i = 0; i < 16; ++i)
    if ((43 * i) / 15 == d) return i;
  return -1;
}

// MODE (FTC_GEMM_NT_V7_MODE, diagnostics): bit 0 sets M0 without saving it (the kernel's only M0 user;
// audited in the ISA), bit 3 runs each MFMA group as one B fragment against the 8 A fragments; timing
// only (results garbage): bit 1 drops the loop's DMA, bit 2 its barriers, bit 4 the DMA wait, bit 5
// re-reads K-tile 0 in every DMA (L2-resident).
template <bool F32C, int MODE = 0, int EPI = EPI_STORE>
__global__ __launch_bounds__(256, 1) void gemm_nt_w4d_kernel(NTArgs p) {
  constexpr int IMG2 = 256 * 64 * 2;
  constexpr int SS = 2 * IMG2;
  __shared__ __attribute__((aligned(16))) char S[2 * SS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  int mb, nb;
  tile_of(p, mb, nb);
  const long long m0 = (long long)mb * BM, n0 = (long long)nb * BN;
  const int ns = p.K / (2 * BK);
  const int st0 = ((int)(blockIdx.x & p.stagger_mask) * p.stagger_step) % ns;
  auto phys = [&](int ss) { const int q = ss + st0; return q >= ns ? q - ns : q; };

  // DMA: wave w fills rows [64 w, 64 w + 64) of both images, piece j = rows 64 w + 8 j + (lane >> 3);
  // MODE bit 8 (interleaved): piece j of wave w = rows 32 j + 8 w + (lane >> 3), i.e. the 4 waves'
  // j-th pieces cover 32 consecutive rows (the library's order)
  constexpr bool IL = (MODE & 256) != 0;
  constexpr int PSTRIDE = IL ? 4096 : 1024;  // LDS bytes between a wave's consecutive pieces
  int vo[2][2];
  {
    const int rr = lane >> 3, pc = lane & 7;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int r0 = IL ? 8 * wave + rr : 64 * wave + rr;
      const int lc = pc ^ f5(IL ? rr + 8 * (wave & 1) : rr + 8 * q);
      vo[0][q] = (int)((r0 * p.lda + 8 * lc) * 2);
      vo[1][q] = (int)((r0 * p.ldb + 8 * lc) * 2);
    }
  }
  const int s8a = (int)((IL ? 32 : 8) * p.lda * 2), s8b = (int)((IL ? 32 : 8) * p.ldb * 2);
  const auto ra = make_rsrc(p.a + m0 * p.lda);
  const auto rb = make_rsrc(p.b + n0 * p.ldb);
  char* const wbase = S + (IL ? 8 : 64) * wave * 128;
  auto dma = [&](int op, int ss, int j) __attribute__((always_inline)) {
    if constexpr (MODE & 2) return;
    const void* dst = wbase + (ss & 1) * SS + op * IMG2 + j * PSTRIDE;
    const int soff = ((MODE & 32) ? 0 : phys(ss) * 128) + j * (op ? s8b : s8a);
    if constexpr (MODE & 1) {
      const unsigned d = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)dst;
      asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
                   :: "v"(vo[op][j & 1]), "s"(op ? rb : ra), "s"(d), "s"(soff) : "memory");
    } else {
      lds_dma16(op ? rb : ra, dst, vo[op][j & 1], soff);
    }
  };
  auto sync = [&]() __attribute__((always_inline)) {
    if constexpr (!(MODE & 4)) barrier();
  };
  // MODE bit 6, the lean loop DMA: the descriptor base walks K (once per operand and iteration), so
  // the per-piece soffsets are loop-invariant SGPRs; each piece's statement sets M0 for the NEXT piece
  // after its load, so MFMAs separate every M0 write from the DMA reading it (no s_nop, no save).
  int so[2][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    so[0][j] = j * s8a;
    so[1][j] = j * s8b;
  }
  auto dmal = [&](int op, __amdgpu_buffer_rsrc_t r, unsigned base, int j) __attribute__((always_inline)) {
    if (j == 0)
      asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds\n\ts_mov_b32 m0, %4"
                   :: "v"(vo[op][0]), "s"(r), "s"(base), "s"(so[op][0]), "s"(base + (unsigned)PSTRIDE) : "memory");
    else if (j < 7)
      asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds\n\ts_mov_b32 m0, %3"
                   :: "v"(vo[op][j & 1]), "s"(r), "s"(so[op][j]), "s"(base + (unsigned)((j + 1) * PSTRIDE)) : "memory");
    else
      asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" :: "v"(vo[op][1]), "s"(r), "s"(so[op][7]) : "memory");
  };
  const unsigned lds0 = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)wbase;

  const int li = lane & 15, kc = lane >> 4;
  int a_off[2], b_off[2];
  {
    const int ra_ = wm * 128 + li;
    const int rb_ = 128 * wn + 8 * (li >> 2) + (li & 3);  // store_wave's column mapping
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      a_off[h] = ra_ * 128 + 16 * ((4 * h + kc) ^ f5(li));
      b_off[h] = IMG2 + rb_ * 128 + 16 * ((4 * h + kc) ^ f5(rb_));
    }
  }
  auto bnt = [](int nt) { return (32 * (nt >> 1) + 4 * (nt & 1)) * 128; };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 xa[8], xb[8], ya[8], yb[8];

  // one MFMA group (A fragment mt against the 8 B fragments) with up to 4 side operations after
  // MFMAs 1, 3, 5, 7
  // (MODE bit 3: B fragment g against the 8 A fragments instead -- src0 of consecutive MFMAs constant)
  auto group = [&](const bf16x8 (&fa)[8], const bf16x8 (&fb)[8], int g, auto&& side) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int mt = (MODE & 8) ? q : g, nt = (MODE & 8) ? g : q;
      acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[nt], fa[mt], acc[mt][nt], 0, 0, 0);
      if (q & 1) {
        __builtin_amdgcn_sched_barrier(0);
        side(q >> 1);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  // prologue: super-stages 0 and 1
#pragma unroll
  for (int j = 0; j < 8; ++j) { dma(0, 0, j); dma(1, 0, j); }
  if (ns > 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { dma(0, 1, j); dma(1, 1, j); }
    __builtin_amdgcn_s_waitcnt(0x4F70);  // vmcnt(16) (bits 15:14 carry vmcnt[5:4])
  } else {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  }
  barrier();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    xa[i] = rd(S, a_off[0] + i * 2048);
    xb[i] = rd(S, b_off[0] + bnt(i));
  }

  if constexpr (MODE & 128) {
    for (int s = 0; s < ns; ++s) {
      const char* cur = S + (s & 1) * SS;
      const char* nxt = S + ((s + 1) & 1) * SS;
      const int sp = min(s + 2, ns - 1);
      const auto ras = make_rsrc(p.a + m0 * p.lda + 64 * phys(sp));
      const auto rbs = make_rsrc(p.b + n0 * p.ldb + 64 * phys(sp));
      const unsigned dA = lds0 + (unsigned)((s & 1) * SS), dB = dA + IMG2;
      auto piece = [&](int pc) __attribute__((always_inline)) {
        if (pc < 0) return;
        if constexpr (MODE & 64) dmal(pc >> 3, (pc >> 3) ? rbs : ras, (pc >> 3) ? dB : dA, pc & 7);
        else dma(pc >> 3, sp, pc & 7);
      };
      // half 0 on X: all of Y (A then B) in groups 0-3, release the buffer after group 4
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        group(xa, xb, g, [&](int k) __attribute__((always_inline)) {
          if (g < 4) {
            const int r = 4 * g + k;
            if (r < 8) ya[r] = rd(cur, a_off[1] + r * 2048);
            else yb[r - 8] = rd(cur, b_off[1] + bnt(r - 8));
          }
          piece(v7_piece(8 * g + 2 * k + 1));
        });
        if (g == 4) {
          __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
          sync();
        }
      }
      // half 1 on Y: wait for s + 1 after group 3, X of s + 1 in groups 4-5
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        group(ya, yb, g, [&](int k) __attribute__((always_inline)) {
          if (g == 4 || g == 5) {
            const bool a_first = (MODE & 8) != 0;
            if ((g == 4) == a_first) {
              xa[2 * k] = rd(nxt, a_off[0] + 2 * k * 2048);
              xa[2 * k + 1] = rd(nxt, a_off[0] + (2 * k + 1) * 2048);
            } else {
              xb[2 * k] = rd(nxt, b_off[0] + bnt(2 * k));
              xb[2 * k + 1] = rd(nxt, b_off[0] + bnt(2 * k + 1));
            }
          }
          piece(v7_piece(64 + 8 * g + 2 * k + 1));
        });
        if (g == 3) {
          if constexpr (!(MODE & 16)) __builtin_amdgcn_s_waitcnt(0x0F7A);  // vmcnt(10): s + 1 landed
          sync();
        }
      }
    }
  } else {
  for (int s = 0; s < ns; ++s) {
    const char* cur = S + (s & 1) * SS;
    const char* nxt = S + ((s + 1) & 1) * SS;
    const int sp = min(s + 2, ns - 1);  // past the end: reload the last super-stage into a dead region
    const auto ras = make_rsrc(p.a + m0 * p.lda + 64 * phys(sp));
    const auto rbs = make_rsrc(p.b + n0 * p.ldb + 64 * phys(sp));
    const unsigned dA = lds0 + (unsigned)((s & 1) * SS), dB = dA + IMG2;
    // Every wait sits at least one MFMA group (8 MFMAs) after the last LDS read it covers, so the
    // read latency hides under the matrix pipe instead of stalling the lone wave.
    // half 0 on X: Y.A in groups 0-1, release A after group 2; A pieces of s + 2 and Y.B in groups 3-6;
    // release B after group 7
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
      group(xa, xb, mt, [&](int k) __attribute__((always_inline)) { ya[4 * mt + k] = rd(cur, a_off[1] + (4 * mt + k) * 2048); });
    group(xa, xb, 2, [&](int) __attribute__((always_inline)) {});
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    sync();
#pragma unroll
    for (int mt = 3; mt < 7; ++mt)
      group(xa, xb, mt, [&](int k) __attribute__((always_inline)) {
        const int i = 2 * (mt - 3) + (k >> 1);
        if (k & 1) yb[i] = rd(cur, b_off[1] + bnt(i));
        else if constexpr (MODE & 64) dmal(0, ras, dA, i);
        else dma(0, sp, i);
      });
    group(xa, xb, 7, [&](int) __attribute__((always_inline)) {});
    __builtin_amdgcn_s_waitcnt(0xC07F);
    sync();
    // half 1 on Y: B pieces of s + 2 in groups 0-3, wait for s + 1, X of s + 1 in groups 4-6 (B first:
    // the next iteration's first group needs all of X.B but only X.A[0])
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
      group(ya, yb, mt, [&](int k) __attribute__((always_inline)) {
        if (!(k & 1)) {
          if constexpr (MODE & 64) dmal(1, rbs, dB, 2 * mt + (k >> 1));
          else dma(1, sp, 2 * mt + (k >> 1));
        }
      });
    if constexpr (!(MODE & 16)) __builtin_amdgcn_s_waitcnt(0x4F70);  // vmcnt(16): the 16 pieces of s + 1 landed
    sync();
    group(ya, yb, 4, [&](int k) __attribute__((always_inline)) {
      if constexpr (MODE & 8) {
        xa[2 * k] = rd(nxt, a_off[0] + 2 * k * 2048);
        xa[2 * k + 1] = rd(nxt, a_off[0] + (2 * k + 1) * 2048);
      } else {
        xb[2 * k] = rd(nxt, b_off[0] + bnt(2 * k));
        xb[2 * k + 1] = rd(nxt, b_off[0] + bnt(2 * k + 1));
      }
    });
    group(ya, yb, 5, [&](int k) __attribute__((always_inline)) {
      if constexpr (MODE & 8) {
        xb[2 * k] = rd(nxt, b_off[0] + bnt(2 * k));
        xb[2 * k + 1] = rd(nxt, b_off[0] + bnt(2 * k + 1));
      } else {
        xa[2 * k] = rd(nxt, a_off[0] + 2 * k * 2048);
        xa[2 * k + 1] = rd(nxt, a_off[0] + (2 * k + 1) * 2048);
      }
    });
#pragma unroll
    for (int mt = 6; mt < 8; ++mt) group(ya, yb, mt, [&](int) __attribute__((always_inline)) {});
  }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // no LDS-DMA may outlive the workgroup
  store_w128<F32C, EPI>(p, acc, m0 + wm * 128, n0 + wn * 128, lane);
}

// ---- variant 0: ping-pong ---------------------------------------------------------------------------
// Each tile is two phases per wave (rows 0-63 / 64-127 of the wave's M range, 16 MFMAs each):
//     [ds_read fragments for phase | 2 DMA pieces of tile t+2] barrier [16 MFMA] barrier
// and the two waves of every SIMD run half a phase apart (waves 4-7 pass one extra barrier first), so at
// every barrier interval one wave of each SIMD reads LDS / issues DMA while its partner keeps the matrix
// pipe busy.  Measured 0.78-0.82x hipBLASLt: 31 % of wave cycles parked on the barriers
// (profiles/r3/gemm_nt.md) -- kept as the A/B baseline (FTC_GEMM_NT_VARIANT=0).
template <bool F32C>
__global__ __launch_bounds__(512, 1) void gemm_nt_pp_kernel(NTArgs p) {
  __shared__ __attribute__((aligned(16))) char S[NSTAGE * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  int mb, nb;
  tile_of(p, mb, nb);
  const long long m0 = (long long)mb * BM, n0 = (long long)nb * BN;
  const Dma dma(p, m0, n0, S, wave, lane);
  const int a_off = a_frag_off(wm, lane), b_off = b_frag_off(wn, lane);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa[4], fb[4];
  auto mfma16 = [&](int h) __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        acc[4 * h + mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[nt], fa[mt], acc[4 * h + mt][nt], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  const int nk = p.K / BK;
  dma.tile(0);
  if (nk > 1) {
    dma.tile(1);
    __builtin_amdgcn_s_waitcnt(0x0F74);  // vmcnt(4)
  } else {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  }
  barrier();
  if (wm) barrier();  // stagger: waves 4-7 run one interval behind waves 0-3

  for (int kt = 0; kt < nk; ++kt) {
    const char* st = S + (kt & (NSTAGE - 1)) * STAGE;
    const bool pre = kt + 2 < nk;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) fb[nt] = rd(st, b_off + b_nt(nt));
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) fa[mt] = rd(st, a_off + mt * 1024);
    if (pre) {
      dma.piece(kt + 2, 0);
      dma.piece(kt + 2, 1);
    }
    barrier();
    mfma16(0);
    barrier();
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) fa[mt] = rd(st, a_off + 4096 + mt * 1024);
    if (pre) {
      dma.piece(kt + 2, 2);
      dma.piece(kt + 2, 3);
      __builtin_amdgcn_s_waitcnt(0x0F74);  // vmcnt(4): only tile kt + 2 may still fly
    } else {
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    }
    barrier();
    mfma16(1);
    barrier();
  }
  if (!wm) barrier();  // equal barrier counts for both halves
  store_tile<F32C>(p, acc, m0, n0, wm, wn, lane);
}

}  // namespace

// C[M, N] (ldc) = alpha A B^T + beta C; A [M, K] (lda), B [N, K] (ldb) bf16 row-major, K contiguous.
// Returns 0 when the shape / alignment is outside the kernel's contract.
extern "C" int ftc_gemm_nt_ok(const void* a, long long lda, const void* b, long long ldb, const void* c, long long ldc,
                              int c_fp32, int M, int N, int K) {
  if (M <= 0 || N <= 0 || K <= 0 || M % BM || N % BN || K % (2 * BK)) return 0;  // even tile count
  if (lda % 8 || ldb % 8 || ldc % 8 || lda < K || ldb < K || ldc < N) return 0;
  if ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) | reinterpret_cast<uintptr_t>(c)) & 15) return 0;
  // 32-bit per-lane DMA offsets: 255 rows + one K extent
  if ((long long)(BM - 1) * (lda > ldb ? lda : ldb) * 2 + (long long)K * 2 + 64 >= (1LL << 31)) return 0;
  if ((long long)(M / BM) * (N / BN) > 0x7fffffffLL) return 0;
  (void)c_fp32;
  return 1;
}

extern "C" int ftc_gemm_nt(const void* a, long long lda, const void* b, long long ldb, void* c, long long ldc,
                           int c_fp32, int M, int N, int K, float alpha, float beta, hipStream_t stream) {
  if (!ftc_gemm_nt_ok(a, lda, b, ldb, c, ldc, c_fp32, M, N, K)) return -1;
  static const int group_m = [] {
    const char* e = getenv("FTC_GEMM_NT_GROUP");
    return e ? atoi(e) : 4;
  }();
  NTArgs p{(const uint16_t*)a, (const uint16_t*)b, c, lda, ldb, ldc, K, M / BM, N / BN, group_m > 0 ? group_m : 4,
           alpha, beta};
  static const int variant = [] {
    const char* e = getenv("FTC_GEMM_NT_VARIANT");
    return e ? atoi(e) : 5;
  }();
  const int grid = p.nm * p.nn;
  {
    static const int su = [] {
      const char* e = getenv("FTC_GEMM_NT_STAGGER");
      return e ? atoi(e) : 0;
    }();
    static const int sus = [] {
      const char* e = getenv("FTC_GEMM_NT_STAGGER_STEP");
      return e ? atoi(e) : 2;
    }();
    p.stagger_mask = su > 1 ? su - 1 : 0;
    p.stagger_step = sus;
  }
  if (variant == 7) {
    static const int v7mode = [] {
      const char* e = getenv("FTC_GEMM_NT_V7_MODE");
      return e ? atoi(e) : 0;
    }();
    if (c_fp32)
      hipLaunchKernelGGL((gemm_nt_w4d_kernel<true>), dim3(grid), dim3(256), 0, stream, p);
    else if (v7mode == 1)
      hipLaunchKernelGGL((gemm_nt_w4d_kernel<false, 1>), dim3(grid), dim3(256), 0, stream, p);
    else if (v7mode == 2)
      hipLaunchKernelGGL((gemm_nt_w4d_kernel<false, 2>), dim3(grid), dim3(256), 0, stream, p);
    else if (v7mode == 6)
      hipLaunchKernelGGL((gemm_nt_w4d_kernel<false, 6>), dim3(grid), dim3(256), 0, stream, p);
    else if (v7mode == 456)
      hipLaunchKernelGGL((gemm_nt_w4d_kernel<false, 456>), dim3(grid), dim3(256), 0, stream, p);
    else if (v7mode == 329)
      hipLaunchKernelGGL((gemm_nt_w4d_kernel<false, 329>), dim3(grid), dim3(256), 0, stream, p);
    else if (v7mode == 200)
      hipLaunchKernelGGL((gemm_nt_w4d_kernel<false, 200>), dim3(grid), dim3(256), 0, stream, p);
    else if (v7mode == 137)
      hipLaunchKernelGGL((gemm_nt_w4d_kernel<false, 137>), dim3(grid), dim3(256), 0, stream, p);
    else if (v7mode == 72)
      hipLaunchKernelGGL((gemm_nt_w4d_kernel<false, 72>), dim3(grid), dim3(256), 0, stream, p);
    else if (v7mode == 73)
      hipLaunchKernelGGL((gemm_nt_w4d_kernel<false, 73>), dim3(grid), dim3(256), 0, stream, p);
    else if (v7mode == 25)
      hipLaunchKernelGGL((gemm_nt_w4d_kernel<false, 25>), dim3(grid), dim3(256), 0, stream, p);
    else if (v7mode == 41)
      hipLaunchKernelGGL((gemm_nt_w4d_kernel<false, 41>), dim3(grid), dim3(256), 0, stream, p);
    else if (v7mode == 13)
      hipLaunchKernelGGL((gemm_nt_w4d_kernel<false, 13>), dim3(grid), dim3(256), 0, stream, p);
    else if (v7mode == 9)
      hipLaunchKernelGGL((gemm_nt_w4d_kernel<false, 9>), dim3(grid), dim3(256), 0, stream, p);
    else if (v7mode == 10)
      hipLaunchKernelGGL((gemm_nt_w4d_kernel<false, 10>), dim3(grid), dim3(256), 0, stream, p);
    else
      hipLaunchKernelGGL((gemm_nt_w4d_kernel<false>), dim3(grid), dim3(256), 0, stream, p);
  } else if (variant == 6) {
    if (c_fp32)
      hipLaunchKernelGGL((gemm_nt_w4s_kernel<true>), dim3(grid), dim3(256), 0, stream, p);
    else
      hipLaunchKernelGGL((gemm_nt_w4s_kernel<false>), dim3(grid), dim3(256), 0, stream, p);
  } else if (variant == 5) {
    static const int v5mode = [] {
      const char* e = getenv("FTC_GEMM_NT_V5_MODE");
      return e ? atoi(e) : 0;
    }();
    if (c_fp32)
      hipLaunchKernelGGL((gemm_nt_v5_kernel<true>), dim3(grid), dim3(512), 0, stream, p);
    else if (v5mode == 1)
      hipLaunchKernelGGL((gemm_nt_v5_kernel<false, EPI_STORE, 1>), dim3(grid), dim3(512), 0, stream, p);
    else if (v5mode == 2)
      hipLaunchKernelGGL((gemm_nt_v5_kernel<false, EPI_STORE, 2>), dim3(grid), dim3(512), 0, stream, p);
    else if (v5mode == 4)
      hipLaunchKernelGGL((gemm_nt_v5_kernel<false, EPI_STORE, 4>), dim3(grid), dim3(512), 0, stream, p);
    else if (v5mode == 8)
      hipLaunchKernelGGL((gemm_nt_v5_kernel<false, EPI_STORE, 8>), dim3(grid), dim3(512), 0, stream, p);
    else if (v5mode == 16)
      hipLaunchKernelGGL((gemm_nt_v5_kernel<false, EPI_STORE, 16>), dim3(grid), dim3(512), 0, stream, p);
    else if (v5mode == 32)
      hipLaunchKernelGGL((gemm_nt_v5_kernel<false, EPI_STORE, 32>), dim3(grid), dim3(512), 0, stream, p);
    else if (v5mode == 17)
      hipLaunchKernelGGL((gemm_nt_v5_kernel<false, EPI_STORE, 17>), dim3(grid), dim3(512), 0, stream, p);
    else
      hipLaunchKernelGGL((gemm_nt_v5_kernel<false>), dim3(grid), dim3(512), 0, stream, p);
  } else if (variant == 4) {
    if (c_fp32)
      hipLaunchKernelGGL((gemm_nt_w4_kernel<true>), dim3(grid), dim3(256), 0, stream, p);
    else
      hipLaunchKernelGGL((gemm_nt_w4_kernel<false>), dim3(grid), dim3(256), 0, stream, p);
  } else if (variant == 2) {
    if (c_fp32)
      hipLaunchKernelGGL((gemm_nt_rs_kernel<true>), dim3(grid), dim3(512), 0, stream, p);
    else
      hipLaunchKernelGGL((gemm_nt_rs_kernel<false>), dim3(grid), dim3(512), 0, stream, p);
  } else if (variant == 0) {
    if (c_fp32)
      hipLaunchKernelGGL((gemm_nt_pp_kernel<true>), dim3(grid), dim3(512), 0, stream, p);
    else
      hipLaunchKernelGGL((gemm_nt_pp_kernel<false>), dim3(grid), dim3(512), 0, stream, p);
  } else if (c_fp32) {
    hipLaunchKernelGGL((gemm_nt_kernel<true>), dim3(grid), dim3(512), 0, stream, p);
  } else {
    static const int mode = [] {
      const char* e = getenv("FTC_GEMM_NT_MODE");
      return e ? atoi(e) : 0;
    }();
    switch (mode) {
      case 1: hipLaunchKernelGGL((gemm_nt_kernel<false, 1>), dim3(grid), dim3(512), 0, stream, p); break;
      case 2: hipLaunchKernelGGL((gemm_nt_kernel<false, 2>), dim3(grid), dim3(512), 0, stream, p); break;
      case 3: hipLaunchKernelGGL((gemm_nt_kernel<false, 3>), dim3(grid), dim3(512), 0, stream, p); break;
      case 7: hipLaunchKernelGGL((gemm_nt_kernel<false, 7>), dim3(grid), dim3(512), 0, stream, p); break;
      case 8: hipLaunchKernelGGL((gemm_nt_kernel<false, 8>), dim3(grid), dim3(512), 0, stream, p); break;
      case 16: hipLaunchKernelGGL((gemm_nt_kernel<false, 16>), dim3(grid), dim3(512), 0, stream, p); break;
      case 32: hipLaunchKernelGGL((gemm_nt_kernel<false, 32>), dim3(grid), dim3(512), 0, stream, p); break;
      default: hipLaunchKernelGGL((gemm_nt_kernel<false>), dim3(grid), dim3(512), 0, stream, p);
    }
  }
  return (int)hipGetLastError();
}

// C[M, N] (ldc) = alpha A Bp^T + beta C with Bp the packed [N/32][K/32][2][64][8] form of B [N, K].
extern "C" int ftc_gemm_nt_pb_ok(const void* a, long long lda, const void* bp, const void* c, long long ldc, int M,
                                 int N, int K) {
  if (M <= 0 || N <= 0 || K <= 0 || M % BM || N % BN || K % (2 * BK)) return 0;
  if (lda % 8 || ldc % 8 || lda < K || ldc < N) return 0;
  if ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(bp) | reinterpret_cast<uintptr_t>(c)) & 15) return 0;
  if ((long long)(BM - 1) * lda * 2 + (long long)K * 2 + 64 >= (1LL << 31)) return 0;
  if ((long long)8 * (K / BK) * 2048 >= (1LL << 31)) return 0;  // B offsets inside one block's panel
  return 1;
}

extern "C" int ftc_gemm_nt_pb(const void* a, long long lda, const void* bp, void* c, long long ldc, int c_fp32, int M,
                              int N, int K, float alpha, float beta, hipStream_t stream) {
  if (!ftc_gemm_nt_pb_ok(a, lda, bp, c, ldc, M, N, K)) return -1;
  static const int group_m = [] {
    const char* e = getenv("FTC_GEMM_NT_GROUP");
    return e ? atoi(e) : 4;
  }();
  PBArgs p{(const uint16_t*)a, (const uint16_t*)bp, c, lda, ldc, K, M / BM, N / BN, group_m > 0 ? group_m : 4, alpha,
           beta};
  const int grid = p.nm * p.nn;
  static const int mode = [] {
    const char* e = getenv("FTC_GEMM_NT_PB_MODE");
    return e ? atoi(e) : 0;
  }();
  if (c_fp32)
    hipLaunchKernelGGL((gemm_nt_pb_kernel<true>), dim3(grid), dim3(512), 0, stream, p);
  else if (mode == 1)
    hipLaunchKernelGGL((gemm_nt_pb_kernel<false, 1>), dim3(grid), dim3(512), 0, stream, p);
  else if (mode == 2)
    hipLaunchKernelGGL((gemm_nt_pb_kernel<false, 2>), dim3(grid), dim3(512), 0, stream, p);
  else if (mode == 3)
    hipLaunchKernelGGL((gemm_nt_pb_kernel<false, 3>), dim3(grid), dim3(512), 0, stream, p);
  else
    hipLaunchKernelGGL((gemm_nt_pb_kernel<false>), dim3(grid), dim3(512), 0, stream, p);
  return (int)hipGetLastError();
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
  static const int group_m = [] {
    const char* e = getenv("FTC_GEMM_NT_GROUP");
    return e ? atoi(e) : 4;
  }();
  NTArgs p{(const uint16_t*)a, (const uint16_t*)b, c, lda, ldb, ldc, K, M / BM, N / BN, group_m > 0 ? group_m : 4,
           1.f, 0.f, cos_t, sin_t, positions, seq_len, rot_heads};
  static const int variant = [] {
    const char* e = getenv("FTC_GEMM_NT_VARIANT");
    return e ? atoi(e) : 5;
  }();
  if (variant == 7)
    hipLaunchKernelGGL((gemm_nt_w4d_kernel<false, 72, EPI_ROPE>), dim3(p.nm * p.nn), dim3(256), 0, stream, p);
  else
    hipLaunchKernelGGL((gemm_nt_v5_kernel<false, EPI_ROPE>), dim3(p.nm * p.nn), dim3(512), 0, stream, p);
  return (int)hipGetLastError();
}
