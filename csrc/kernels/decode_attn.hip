// Decode attention for generation: one new query token per sequence against its KV cache (GQA,
// optional sliding window), split over the key axis so a batch of long caches fills the 256 CUs.
//
// Decode is bound by HBM (every cached K/V byte is read once per generated token), so the layout is
// chosen for coalesced 16-byte loads, not for MFMA:
//   * partial kernel: workgroup = (sequence, kv head, key chunk).  The chunk (64..256 keys) is sized
//     on the host so that batch x kv heads x chunks gives >= ~512 workgroups: a single sequence's
//     short cache still spreads over the CUs instead of a few latency-bound workgroups.  A key row (D bf16) is read by
//     D/8 adjacent lanes, 16 bytes each, so one wave instruction covers 64/(D/8) whole rows; the G
//     query heads of the kv group are scored against the row at once (the row is read once for all
//     G heads).  Scores go through LDS for the chunk softmax (running max / sum per head), then the
//     same lane layout streams V and accumulates P V.  Output: unnormalised partial O per head and
//     chunk plus its (max, sum).
//   * combine kernel: per (sequence, head), rescales the chunk partials to the global max and
//     normalises -- the split-K reduction of flash decoding, deterministic (no atomics).
// Cache layout: [B, Lmax, KV*D] bf16 rows (row stride kv_rs elements, batch stride b_rs);
// lens[b] = valid keys of sequence b (the current token included).  The current token's K/V come
// from the projection output (knew / vnew rows): the workgroup whose chunk holds position lens[b]-1
// uses them directly and appends them to the cache -- no separate append launch.
#include "common.h"

using namespace ftc;

namespace {

constexpr int CHUNK_MAX = 256;  // keys per partial workgroup (at most)
constexpr int GMAX = 8;         // query heads per kv head (Llama-3-70B: 64 / 8)
constexpr float LOG2E = 1.4426950408889634f;

struct DecArgs {
  const uint16_t* q;
  uint16_t* kc;
  uint16_t* vc;
  const uint16_t* knew;  // [B, new_rs] rows: the current token's K (KV*D) ...
  const uint16_t* vnew;  // ... and V
  const int* lens;
  float* opart;  // [B*H, nsplit, D]
  float* ml;     // [B*H, nsplit, 2]
  uint16_t* out;
  long long q_rs, kv_rs, b_rs, o_rs, new_rs;
  int B, H, KV, nsplit, window, chunk;
  float c;  // scale * log2(e)
};

template <int D>
__global__ __launch_bounds__(256) void decode_partial_kernel(DecArgs a) {
  constexpr int CPR = D / 8;        // 16-byte chunks per row = lanes per key row
  constexpr int KPW = 64 / CPR;     // key rows per wave instruction
  __shared__ float sc[GMAX][CHUNK_MAX];
  __shared__ float red[4][GMAX][D];
  __shared__ float stat[2][4][GMAX];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c8 = lane % CPR, kq = lane / CPR;
  const int bk = blockIdx.x, split = blockIdx.y;
  const int b = bk / a.KV, kvh = bk % a.KV;
  const int G = a.H / a.KV;
  const int len = a.lens[b];
  const int lo = a.window > 0 ? max(0, len - a.window) : 0;
  const int chunk = a.chunk, iters = chunk / (4 * KPW);
  const int k0 = split * chunk;
  if (k0 >= len || k0 + chunk <= lo) return;  // the combine kernel skips this chunk too
  const int cur = len - 1;  // the current token: K / V from the projection output

  // the lane's 8-element slice of each query head of the group, pre-scaled into the log2 domain
  float qv[GMAX][8];
#pragma unroll
  for (int g = 0; g < GMAX; ++g) {
    if (g < G) {
      const uint4 u = *reinterpret_cast<const uint4*>(a.q + (long long)b * a.q_rs + (long long)(kvh * G + g) * D + c8 * 8);
      unpack8(u, qv[g]);
#pragma unroll
      for (int j = 0; j < 8; ++j) qv[g][j] *= a.c;
    }
  }
  const uint16_t* kbase = a.kc + (long long)b * a.b_rs + (long long)kvh * D + c8 * 8;
  const uint16_t* vbase = a.vc + (long long)b * a.b_rs + (long long)kvh * D + c8 * 8;
  const long long noff = (long long)b * a.new_rs + (long long)kvh * D + c8 * 8;

  // ---- scores of the chunk: CPR lanes per key row, shuffle-reduced
  for (int it = 0; it < iters; ++it) {
    const int kl = (it * 4 + wave) * KPW + kq;  // key within the chunk
    const int key = k0 + kl;
    const bool ok = key >= lo && key < len;
    float kf[8];
    uint4 u = make_uint4(0, 0, 0, 0);
    if (key == cur) {  // append the new row while using it
      u = *reinterpret_cast<const uint4*>(a.knew + noff);
      *reinterpret_cast<uint4*>(const_cast<uint16_t*>(kbase) + (long long)key * a.kv_rs) = u;
    } else if (ok) {
      u = *reinterpret_cast<const uint4*>(kbase + (long long)key * a.kv_rs);
    }
    unpack8(u, kf);
#pragma unroll
    for (int g = 0; g < GMAX; ++g) {
      if (g < G) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s += qv[g][j] * kf[j];
#pragma unroll
        for (int off = CPR / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
        if (c8 == 0) sc[g][kl] = ok ? s : -INFINITY;
      }
    }
  }
  __syncthreads();

  // ---- chunk softmax per head: thread t owns key t
  float mx[GMAX], sm[GMAX];
#pragma unroll
  for (int g = 0; g < GMAX; ++g) {
    if (g < G) {
      const float v = wave_max(tid < chunk ? sc[g][tid] : -INFINITY);
      if (lane == 0) stat[0][wave][g] = v;
    }
  }
  __syncthreads();
#pragma unroll
  for (int g = 0; g < GMAX; ++g) {
    if (g < G) {
      mx[g] = fmaxf(fmaxf(stat[0][0][g], stat[0][1][g]), fmaxf(stat[0][2][g], stat[0][3][g]));
      const float s = tid < chunk ? sc[g][tid] : -INFINITY;
      const float p = (s == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(s - mx[g]);
      if (tid < chunk) sc[g][tid] = p;
      const float ws = wave_sum(p);
      if (lane == 0) stat[1][wave][g] = ws;
    }
  }
  __syncthreads();
#pragma unroll
  for (int g = 0; g < GMAX; ++g)
    if (g < G) sm[g] = stat[1][0][g] + stat[1][1][g] + stat[1][2][g] + stat[1][3][g];

  // ---- P V over the chunk, same lane layout as the scores
  float acc[GMAX][8];
#pragma unroll
  for (int g = 0; g < GMAX; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[g][j] = 0.f;
  for (int it = 0; it < iters; ++it) {
    const int kl = (it * 4 + wave) * KPW + kq;
    const int key = k0 + kl;
    const bool ok = key >= lo && key < len;
    float vf[8];
    uint4 u = make_uint4(0, 0, 0, 0);
    if (key == cur) {
      u = *reinterpret_cast<const uint4*>(a.vnew + noff);
      *reinterpret_cast<uint4*>(const_cast<uint16_t*>(vbase) + (long long)key * a.kv_rs) = u;
    } else if (ok) {
      u = *reinterpret_cast<const uint4*>(vbase + (long long)key * a.kv_rs);
    }
    unpack8(u, vf);
#pragma unroll
    for (int g = 0; g < GMAX; ++g) {
      if (g < G) {
        const float p = sc[g][kl];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[g][j] += p * vf[j];
      }
    }
  }
  // reduce over the KPW key rows of a wave instruction (lanes that share c8), then over the 4 waves
#pragma unroll
  for (int g = 0; g < GMAX; ++g) {
    if (g < G) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = acc[g][j];
#pragma unroll
        for (int off = CPR; off < 64; off <<= 1) v += __shfl_xor(v, off, 64);
        acc[g][j] = v;
      }
      if (kq == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) red[wave][g][c8 * 8 + j] = acc[g][j];
      }
    }
  }
  __syncthreads();
  for (int e = tid; e < G * D; e += 256) {
    const int g = e / D, d = e % D;
    const float o = red[0][g][d] + red[1][g][d] + red[2][g][d] + red[3][g][d];
    const long long row = ((long long)b * a.H + kvh * G + g) * a.nsplit + split;
    a.opart[row * D + d] = o;
    if (d == 0) {
      a.ml[row * 2] = mx[g];
      a.ml[row * 2 + 1] = sm[g];
    }
  }
}

template <int D>
__global__ __launch_bounds__(D) void decode_combine_kernel(DecArgs a) {
  const int bh = blockIdx.x, d = threadIdx.x;
  const int b = bh / a.H;
  const int len = a.lens[b];
  const int lo = a.window > 0 ? max(0, len - a.window) : 0;
  const int s0 = lo / a.chunk, s1 = min(a.nsplit, (len + a.chunk - 1) / a.chunk);
  const long long base = (long long)bh * a.nsplit;
  float M = -INFINITY;
  for (int s = s0; s < s1; ++s) M = fmaxf(M, a.ml[(base + s) * 2]);
  float L = 0.f, o = 0.f;
  for (int s = s0; s < s1; ++s) {
    const float w = __builtin_amdgcn_exp2f(a.ml[(base + s) * 2] - M);
    L += w * a.ml[(base + s) * 2 + 1];
    o += w * a.opart[(base + s) * D + d];
  }
  a.out[(long long)b * a.o_rs + (long long)(bh % a.H) * D + d] = f2bf(L > 0.f ? o / L : 0.f);
}

}  // namespace

// chunk: a multiple of 64 in [64, 256] giving >= ~512 partial workgroups where the caches allow
static int decode_chunk(int B, int KV, int max_len) {
  const long long want = 512;
  long long c = ((long long)B * KV * max_len + want - 1) / want;
  c = (c + 63) / 64 * 64;
  return (int)(c < 64 ? 64 : (c > CHUNK_MAX ? CHUNK_MAX : c));
}

extern "C" long long ftc_decode_workspace_floats(int B, int H, int KV, int D, int max_len) {
  const int chunk = decode_chunk(B, KV, max_len);
  const long long nsplit = (max_len + chunk - 1) / chunk;
  return (long long)B * H * nsplit * (D + 2);
}

extern "C" int ftc_decode_attention(const void* q, void* kc, void* vc, const void* knew, const void* vnew,
                                    long long new_rs, const int* lens, void* out, float* workspace, int B, int H,
                                    int KV, int D, int max_len, long long q_rs, long long kv_rs, long long b_rs,
                                    long long o_rs, float scale, int window, hipStream_t stream) {
  if ((D != 128 && D != 64) || H % KV != 0 || H / KV > GMAX || max_len < 1) return -1;
  const int chunk = decode_chunk(B, KV, max_len);
  const int nsplit = (max_len + chunk - 1) / chunk;
  DecArgs a{(const uint16_t*)q, (uint16_t*)kc, (uint16_t*)vc, (const uint16_t*)knew, (const uint16_t*)vnew, lens,
            workspace, workspace + (long long)B * H * nsplit * D, (uint16_t*)out,
            q_rs, kv_rs, b_rs, o_rs, new_rs, B, H, KV, nsplit, window, chunk, scale * LOG2E};
  if (D == 128) {
    hipLaunchKernelGGL(decode_partial_kernel<128>, dim3(B * KV, nsplit), dim3(256), 0, stream, a);
    hipLaunchKernelGGL(decode_combine_kernel<128>, dim3(B * H), dim3(128), 0, stream, a);
  } else {
    hipLaunchKernelGGL(decode_partial_kernel<64>, dim3(B * KV, nsplit), dim3(256), 0, stream, a);
    hipLaunchKernelGGL(decode_combine_kernel<64>, dim3(B * H), dim3(64), 0, stream, a);
  }
  return (int)hipGetLastError();
}
