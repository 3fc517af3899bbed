// K7: fused AdamW over ONE flat parameter buffer, plus the global grad-norm reduction it uses.
//
// The trainer keeps every trainable parameter as a view into one flat bf16 buffer, its gradient
// as a view into one flat grad buffer, and the fp32 master copy + Adam moments as flat fp32
// buffers (finetune_controller_amd/train/optim.py).  One launch therefore updates all of them --
// 13.6-42 M LoRA params or 8.03 B full-FT params -- with no multi-tensor list walking.  HBM bound:
// per element it reads master/m/v (12 B) + grad (2 or 4 B) and writes master/m/v + bf16 param
// (14 B), moved as 16-byte vectors (4 elements per lane per step).
//
// The grad scale (1/world for averaging x clip coefficient) is read from DEVICE memory so the
// whole optimizer step runs with no host synchronisation (and can be captured in a hipGraph).
#include "common.h"

using namespace ftc;

template <typename G>
DEV_INLINE void load_grad4(const G* g, long long i, float* o);
template <>
DEV_INLINE void load_grad4<float>(const float* g, long long i, float* o) {
  const float4 v = reinterpret_cast<const float4*>(g)[i];
  o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
template <>
DEV_INLINE void load_grad4<uint16_t>(const uint16_t* g, long long i, float* o) {
  const uint2 v = reinterpret_cast<const uint2*>(g)[i];
  o[0] = bf_lo(v.x); o[1] = bf_hi(v.x); o[2] = bf_lo(v.y); o[3] = bf_hi(v.y);
}
template <typename G>
DEV_INLINE float load_grad1(const G* g, long long i);
template <>
DEV_INLINE float load_grad1<float>(const float* g, long long i) { return g[i]; }
template <>
DEV_INLINE float load_grad1<uint16_t>(const uint16_t* g, long long i) { return bf2f(g[i]); }

struct AdamHP {
  float lr, b1, b2, eps, wd, bc1, bc2;  // bc = 1 - beta^t
};

DEV_INLINE void adam_elem(float& p, float& m, float& v, float g, const AdamHP& hp) {
  m = hp.b1 * m + (1.f - hp.b1) * g;
  v = hp.b2 * v + (1.f - hp.b2) * g * g;
  const float mh = m / hp.bc1;
  const float vh = v / hp.bc2;
  p = p * (1.f - hp.lr * hp.wd) - hp.lr * mh / (sqrtf(vh) + hp.eps);
}

template <typename G>
__global__ __launch_bounds__(256) void adamw_kernel(uint16_t* __restrict__ param, float* __restrict__ master,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    const G* __restrict__ grad, long long n, AdamHP hp,
                                                    const float* __restrict__ gscale,
                                                    const float* __restrict__ hpdev) {
  const float sc = gscale ? gscale[0] : 1.0f;
  if (hpdev) {  // [lr, 1 - b1^t, 1 - b2^t] from device memory: a captured step replays with new values
    hp.lr = hpdev[0];
    hp.bc1 = hpdev[1];
    hp.bc2 = hpdev[2];
  }
  // one 4-element group per thread over a one-shot grid: 5.91 vs 5.62 TB/s for the grid-stride loop
  // (2048 workgroups) at 8.03 B elements, 38.1 vs 40.0 ms (profiles/r4/adamw/; an 8-wide group read
  // 5.67)
  // one pass when the launch covers the tensor (the usual case); the loop keeps a capped grid correct
  // (ftc_adamw caps it so grid x 256 stays below HIP's 2^32 work items per launch)
  const long long i0 = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = i0; i < n4; i += stride) {
    float g[4];
    load_grad4<G>(grad, i, g);
    float4 P = reinterpret_cast<float4*>(master)[i];
    float4 M = reinterpret_cast<float4*>(m)[i];
    float4 Vv = reinterpret_cast<float4*>(v)[i];
    adam_elem(P.x, M.x, Vv.x, g[0] * sc, hp);
    adam_elem(P.y, M.y, Vv.y, g[1] * sc, hp);
    adam_elem(P.z, M.z, Vv.z, g[2] * sc, hp);
    adam_elem(P.w, M.w, Vv.w, g[3] * sc, hp);
    reinterpret_cast<float4*>(master)[i] = P;
    reinterpret_cast<float4*>(m)[i] = M;
    reinterpret_cast<float4*>(v)[i] = Vv;
    if (param) {
      uint2 o;
      o.x = pack_bf2(P.x, P.y);
      o.y = pack_bf2(P.z, P.w);
      reinterpret_cast<uint2*>(param)[i] = o;
    }
  }
  const long long t = (n4 << 2) + i0;  // tail (n % 4): the first threads of the grid
  if (t < n) {
    float P = master[t], M = m[t], Vv = v[t];
    adam_elem(P, M, Vv, load_grad1<G>(grad, t) * sc, hp);
    master[t] = P; m[t] = M; v[t] = Vv;
    if (param) param[t] = f2bf(P);
  }
}

extern "C" int ftc_adamw(void* param_bf16, float* master, float* m, float* v, const void* grad, int grad_is_fp32,
                         long long n, float lr, float b1, float b2, float eps, float wd, float bc1, float bc2,
                         const float* gscale, const float* hpdev, hipStream_t stream) {
  AdamHP hp{lr, b1, b2, eps, wd, bc1, bc2};
  const long long groups = n >> 2 > 0 ? n >> 2 : 1;
  long long blocks = (groups + 255) / 256;
  if (blocks > (1LL << 24) - 1) blocks = (1LL << 24) - 1;  // grid x 256 < 2^32: larger tensors loop
  const dim3 grid((unsigned)blocks);
  if (grad_is_fp32)
    hipLaunchKernelGGL((adamw_kernel<float>), dim3(grid), dim3(256), 0, stream, (uint16_t*)param_bf16, master, m, v,
                       (const float*)grad, n, hp, gscale, hpdev);
  else
    hipLaunchKernelGGL((adamw_kernel<uint16_t>), dim3(grid), dim3(256), 0, stream, (uint16_t*)param_bf16, master, m,
                       v, (const uint16_t*)grad, n, hp, gscale, hpdev);
  return (int)hipGetLastError();
}

// ---- sum of squares (grad-norm) : deterministic two-stage reduction ----
// 16-byte loads (8 bf16 / 4 fp32 per lane), two independent loads in flight per lane per iteration:
// the full-FT gradient (16 GB bf16) streams at HBM rate (the 8-byte-per-lane version read 3.7 TB/s).
DEV_INLINE float sumsq16(const uint4 v, const uint16_t*) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float lo = bf_lo(w[j]), hi = bf_hi(w[j]);
    s += lo * lo + hi * hi;
  }
  return s;
}
DEV_INLINE float sumsq16(const uint4 v, const float*) {
  const float a = __uint_as_float(v.x), b = __uint_as_float(v.y), c = __uint_as_float(v.z),
              d = __uint_as_float(v.w);
  return a * a + b * b + c * c + d * d;
}

template <typename G, bool VEC>
__global__ __launch_bounds__(256) void sumsq_partial_kernel(const G* __restrict__ x, long long n,
                                                            float* __restrict__ partial) {
  __shared__ float red[4];
  constexpr int EPV = VEC ? 16 / sizeof(G) : 1;  // elements per 16-byte vector (VEC: x 16-byte aligned)
  float s0 = 0.f, s1 = 0.f;
  const long long nv = VEC ? n / EPV : 0;
  const uint4* xv = reinterpret_cast<const uint4*>(x);
  const long long stride = (long long)gridDim.x * 256;
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  for (; i + stride < nv; i += 2 * stride) {
    const uint4 a = xv[i], b = xv[i + stride];
    s0 += sumsq16(a, x);
    s1 += sumsq16(b, x);
  }
  if (i < nv) s0 += sumsq16(xv[i], x);
  // tail (n % EPV; the whole range when x is not 16-byte aligned)
  for (long long t = nv * EPV + (long long)blockIdx.x * 256 + threadIdx.x; t < n; t += stride) {
    const float g = load_grad1<G>(x, t);
    s0 += g * g;
  }
  const float s = block_sum<256>(s0 + s1, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// out[0] = sum(partial); coef[0] = scale * min(1, max_norm / (sqrt(out)+1e-6)) (max_norm<=0: no clip)
__global__ __launch_bounds__(256) void sumsq_final_kernel(const float* __restrict__ partial, int np,
                                                          float* __restrict__ out, float* __restrict__ coef,
                                                          float max_norm, float scale) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < np; i += 256) s += partial[i];
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) {
    out[0] = s;
    if (coef) {
      float c = 1.0f;
      // the norm is measured on the unscaled (summed) grads: scale first
      const float norm = sqrtf(s) * scale;
      if (max_norm > 0.f && norm > max_norm) c = max_norm / (norm + 1e-6f);
      coef[0] = c * scale;
    }
  }
}

extern "C" int ftc_sumsq_partials() { return 1024; }

extern "C" int ftc_sumsq(const void* x, int is_fp32, long long n, float* partial, float* out, float* coef,
                         float max_norm, float scale, hipStream_t stream) {
  const int grid = ftc::stream_grid((n + 7) / 8, 256) > 1024 ? 1024 : ftc::stream_grid((n + 7) / 8, 256);
  const bool vec = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  if (is_fp32 && vec)
    hipLaunchKernelGGL((sumsq_partial_kernel<float, true>), dim3(grid), dim3(256), 0, stream, (const float*)x, n,
                       partial);
  else if (is_fp32)
    hipLaunchKernelGGL((sumsq_partial_kernel<float, false>), dim3(grid), dim3(256), 0, stream, (const float*)x, n,
                       partial);
  else if (vec)
    hipLaunchKernelGGL((sumsq_partial_kernel<uint16_t, true>), dim3(grid), dim3(256), 0, stream,
                       (const uint16_t*)x, n, partial);
  else
    hipLaunchKernelGGL((sumsq_partial_kernel<uint16_t, false>), dim3(grid), dim3(256), 0, stream,
                       (const uint16_t*)x, n, partial);
  hipLaunchKernelGGL(sumsq_final_kernel, dim3(1), dim3(256), 0, stream, partial, grid, out, coef, max_norm, scale);
  return (int)hipGetLastError();
}
