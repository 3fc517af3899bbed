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
FTC_DEV void load_grad4(const G* g, long long i, float* o);
template <>
FTC_DEV void load_grad4<float>(const float* g, long long i, float* o) {
  const float4 v = reinterpret_cast<const float4*>(g)[i];
  o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
template <>
FTC_DEV void load_grad4<uint16_t>(const uint16_t* g, long long i, float* o) {
  const uint2 v = reinterpret_cast<const uint2*>(g)[i];
  o[0] = bf_lo(v.x); o[1] = bf_hi(v.x); o[2] = bf_lo(v.y); o[3] = bf_hi(v.y);
}
template <typename G>
FTC_DEV float load_grad1(const G* g, long long i);
template <>
FTC_DEV float load_grad1<float>(const float* g, long long i) { return g[i]; }
template <>
FTC_DEV float load_grad1<uint16_t>(const uint16_t* g, long long i) { return bf2f(g[i]); }

struct AdamHP {
  float lr, b1, b2, eps, wd, bc1, bc2;  // bc = 1 - beta^t
};

FTC_DEV void adam_elem(float& p, float& m, float& v, float g, const AdamHP& hp) {
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
  const long long n4 = n >> 2;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
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
  // tail (n % 4)
  const long long t = (n4 << 2) + (long long)blockIdx.x * 256 + threadIdx.x;
  if (t < n && t >= (n4 << 2)) {
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
  const int grid = ftc::stream_grid((n + 3) / 4, 256);
  if (grad_is_fp32)
    hipLaunchKernelGGL((adamw_kernel<float>), dim3(grid), dim3(256), 0, stream, (uint16_t*)param_bf16, master, m, v,
                       (const float*)grad, n, hp, gscale, hpdev);
  else
    hipLaunchKernelGGL((adamw_kernel<uint16_t>), dim3(grid), dim3(256), 0, stream, (uint16_t*)param_bf16, master, m,
                       v, (const uint16_t*)grad, n, hp, gscale, hpdev);
  return (int)hipGetLastError();
}

// ---- sum of squares (grad-norm) : deterministic two-stage reduction ----
template <typename G>
__global__ __launch_bounds__(256) void sumsq_partial_kernel(const G* __restrict__ x, long long n,
                                                            float* __restrict__ partial) {
  __shared__ float red[4];
  float s = 0.f;
  const long long n4 = n >> 2;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    float g[4];
    load_grad4<G>(x, i, g);
    s += g[0] * g[0] + g[1] * g[1] + g[2] * g[2] + g[3] * g[3];
  }
  const long long t = (n4 << 2) + (long long)blockIdx.x * 256 + threadIdx.x;
  if (t < n && t >= (n4 << 2)) {
    const float g = load_grad1<G>(x, t);
    s += g * g;
  }
  s = block_sum<256>(s, red);
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
  const int grid = ftc::stream_grid((n + 3) / 4, 256) > 1024 ? 1024 : ftc::stream_grid((n + 3) / 4, 256);
  if (is_fp32)
    hipLaunchKernelGGL((sumsq_partial_kernel<float>), dim3(grid), dim3(256), 0, stream, (const float*)x, n, partial);
  else
    hipLaunchKernelGGL((sumsq_partial_kernel<uint16_t>), dim3(grid), dim3(256), 0, stream, (const uint16_t*)x, n,
                       partial);
  hipLaunchKernelGGL(sumsq_final_kernel, dim3(1), dim3(256), 0, stream, partial, grid, out, coef, max_norm, scale);
  return (int)hipGetLastError();
}
