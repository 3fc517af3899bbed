// K10 (softmax/NLL half): fused cross-entropy forward + gradient, IN PLACE on a bf16 logits chunk.
//
// The chunked linear+CE driver (finetune_controller_amd/ops/cross_entropy.py) runs the lm_head
// GEMM for a chunk of rows (hipBLASLt), then this kernel turns each logits row into
//     loss[row] = logsumexp(row) - row[label]          (fp32)
//     row      <- (softmax(row) - onehot(label)) * gscale   (bf16, written over the logits)
// so the [rows, vocab] fp32 logits of a naive CE are never materialised and the dlogits needed
// by the two backward GEMMs are produced in the same pass.  Rows whose label == ignore_index get
// loss 0 and a zero gradient row.
//
// One 256-thread block per row: pass 1 is an online (max, sum-exp) reduction with 16-byte loads,
// pass 2 re-reads the row (an L2 / Infinity-Cache hit: 256 KB per row at vocab 128256) and writes
// the gradient.  vocab % 8 != 0 (GPT-2's 50257) takes the scalar path.
#include "common.h"

using namespace ftc;

DEV_INLINE void ms_merge(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  if (mn == -INFINITY) return;
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

template <bool VEC>
__global__ __launch_bounds__(256) void ce_fwd_bwd_kernel(uint16_t* __restrict__ logits, const long long* __restrict__ labels,
                                                         float* __restrict__ loss, float* __restrict__ lse_out,
                                                         int V, long long ld, float gscale, long long ignore_index) {
  __shared__ float red_m[4], red_s[4];
  const long long row = blockIdx.x;
  uint16_t* rp = logits + row * ld;
  const long long lab = labels[row];
  const int tid = threadIdx.x;
  float m = -INFINITY, s = 0.f;
  if constexpr (VEC) {
    const int nv = V >> 3;
    const uint4* r4 = reinterpret_cast<const uint4*>(rp);
    for (int i = tid; i < nv; i += 256) {
      float f[8];
      unpack8(r4[i], f);
      float lm = f[0];
#pragma unroll
      for (int j = 1; j < 8; ++j) lm = fmaxf(lm, f[j]);
      float ls = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) ls += __expf(f[j] - lm);
      ms_merge(m, s, lm, ls);
    }
  } else {
    for (int i = tid; i < V; i += 256) ms_merge(m, s, bf2f(rp[i]), 1.0f);
  }
  // wave merge
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    ms_merge(m, s, m2, s2);
  }
  if ((tid & 63) == 0) {
    red_m[tid >> 6] = m;
    red_s[tid >> 6] = s;
  }
  __syncthreads();
  m = red_m[0];
  s = red_s[0];
#pragma unroll
  for (int w = 1; w < 4; ++w) ms_merge(m, s, red_m[w], red_s[w]);
  const float lse = m + __logf(s);
  const bool valid = lab != ignore_index;
  if (tid == 0) {
    const float xl = (valid && lab >= 0 && lab < V) ? bf2f(rp[lab]) : 0.f;
    loss[row] = valid ? (lse - xl) : 0.f;
    if (lse_out) lse_out[row] = lse;
  }
  __syncthreads();  // the label logit is read before pass 2 overwrites it
  const float gs = valid ? gscale : 0.f;
  if constexpr (VEC) {
    const int nv = V >> 3;
    uint4* r4 = reinterpret_cast<uint4*>(rp);
    for (int i = tid; i < nv; i += 256) {
      float f[8];
      unpack8(r4[i], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float p = __expf(f[j] - lse);
        if ((long long)(i * 8 + j) == lab) p -= 1.0f;
        f[j] = p * gs;
      }
      r4[i] = pack8(f);
    }
  } else {
    for (int i = tid; i < V; i += 256) {
      float p = __expf(bf2f(rp[i]) - lse);
      if ((long long)i == lab) p -= 1.0f;
      rp[i] = f2bf(p * gs);
    }
  }
}

extern "C" int ftc_ce_fwd_bwd(void* logits, const long long* labels, float* loss, float* lse, long long rows, int V,
                              long long ld, float gscale, long long ignore_index, hipStream_t stream) {
  if (rows <= 0) return 0;
  const bool vec = (V % 8 == 0) && (ld % 8 == 0);
  if (vec)
    hipLaunchKernelGGL((ce_fwd_bwd_kernel<true>), dim3((unsigned)rows), dim3(256), 0, stream, (uint16_t*)logits, labels,
                       loss, lse, V, ld, gscale, ignore_index);
  else
    hipLaunchKernelGGL((ce_fwd_bwd_kernel<false>), dim3((unsigned)rows), dim3(256), 0, stream, (uint16_t*)logits,
                       labels, loss, lse, V, ld, gscale, ignore_index);
  return (int)hipGetLastError();
}
