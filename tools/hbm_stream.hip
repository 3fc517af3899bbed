// Streaming roof for the SwiGLU shapes (Llama-3-8B MLP, T = 16384, F = 14336): how close can a
// 2-read : 1-write (forward, h = silu(g) u) and a 3-read : 2-write (backward, dg | du) element-wise
// pass get to HBM3E peak on MI355X, and which structure gets there.  Standalone:
//   hipcc --offload-arch=gfx950 -O3 -o tools/hbm_stream tools/hbm_stream.hip && tools/hbm_stream
// Variants (all bit-identical outputs, checked against variant 0):
//   copy11   plain 1:1 copy (calibration, same bytes as the torch unary functor probe)
//   fwd_u1   one 16-byte chunk of g and u per thread, one-shot grid
//   fwd_uN   N chunks per thread, all loads issued before any math (more bytes in flight per wave)
//   *_nt     non-temporal stores (the output is not re-read by this kernel)
//   *_gs     grid-stride over 4 x CUs workgroups instead of a one-shot grid
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                 \
      exit(1);                                                                                  \
    }                                                                                           \
  } while (0)

__device__ __forceinline__ float bf2f(unsigned short v) { return __uint_as_float((unsigned)v << 16); }
__device__ __forceinline__ unsigned short f2bf(float f) {
  unsigned u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}
__device__ __forceinline__ unsigned pk(float a, float b) { return (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16); }
__device__ __forceinline__ float lo(unsigned v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float hi(unsigned v) { return __uint_as_float(v & 0xffff0000u); }
__device__ __forceinline__ float silu(float g) { return g / (1.0f + __expf(-g)); }

__device__ __forceinline__ uint4 fwd_math(uint4 g, uint4 u) {
  uint4 o;
  o.x = pk(silu(lo(g.x)) * lo(u.x), silu(hi(g.x)) * hi(u.x));
  o.y = pk(silu(lo(g.y)) * lo(u.y), silu(hi(g.y)) * hi(u.y));
  o.z = pk(silu(lo(g.z)) * lo(u.z), silu(hi(g.z)) * hi(u.z));
  o.w = pk(silu(lo(g.w)) * lo(u.w), silu(hi(g.w)) * hi(u.w));
  return o;
}

template <bool NT>
__device__ __forceinline__ void st16(uint4* p, uint4 v) {
  if constexpr (NT) {
    __builtin_nontemporal_store(v.x, &reinterpret_cast<unsigned*>(p)[0]);
    __builtin_nontemporal_store(v.y, &reinterpret_cast<unsigned*>(p)[1]);
    __builtin_nontemporal_store(v.z, &reinterpret_cast<unsigned*>(p)[2]);
    __builtin_nontemporal_store(v.w, &reinterpret_cast<unsigned*>(p)[3]);
  } else {
    *p = v;
  }
}

__global__ __launch_bounds__(256) void copy11(const uint4* __restrict__ a, uint4* __restrict__ b, long long n) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  constexpr int U = 4;
  const long long base = (long long)blockIdx.x * 256 * U + threadIdx.x;
  uint4 v[U];
#pragma unroll
  for (int k = 0; k < U; ++k)
    if (base + k * 256 < n) v[k] = a[base + k * 256];
#pragma unroll
  for (int k = 0; k < U; ++k)
    if (base + k * 256 < n) b[base + k * 256] = v[k];
  (void)i;
}

// gu [T][2F] (gate | up), h [T][hs]; chunks of 8 bf16; nc = F / 8 chunks per row.
// One-shot: thread -> U chunks spaced 256 apart within a row-major chunk index space of T * nc.
template <int U, bool NT>
__global__ __launch_bounds__(256) void fwd_oneshot(const uint4* __restrict__ gu, uint4* __restrict__ h, long long T,
                                                   int nc, long long hs16) {
  const long long base = (long long)blockIdx.x * 256 * U + threadIdx.x;
  const long long n = T * nc;
  uint4 g[U], u[U];
  long long t[U];
  int c[U];
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const long long idx = base + k * 256;
    t[k] = idx / nc;
    c[k] = (int)(idx - t[k] * nc);
    if (idx < n) {
      g[k] = gu[t[k] * 2 * nc + c[k]];
      u[k] = gu[t[k] * 2 * nc + nc + c[k]];
    }
  }
#pragma unroll
  for (int k = 0; k < U; ++k)
    if (base + k * 256 < n) st16<NT>(h + t[k] * hs16 + c[k], fwd_math(g[k], u[k]));
}

// Grid-stride, software-pipelined: the next U chunks are loaded before this U are computed/stored.
template <int U, bool NT>
__global__ __launch_bounds__(256) void fwd_gs(const uint4* __restrict__ gu, uint4* __restrict__ h, long long T, int nc,
                                              long long hs16) {
  const long long n = T * nc;
  const long long step = (long long)gridDim.x * 256 * U;
  long long base = (long long)blockIdx.x * 256 * U + threadIdx.x;
  uint4 g[U], u[U];
  auto load = [&](long long b) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const long long idx = b + k * 256;
      if (idx < n) {
        const long long tt = idx / nc;
        const int cc = (int)(idx - tt * nc);
        g[k] = gu[tt * 2 * nc + cc];
        u[k] = gu[tt * 2 * nc + nc + cc];
      }
    }
  };
  load(base);
  for (; base < n; base += step) {
    uint4 gc[U], uc[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      gc[k] = g[k];
      uc[k] = u[k];
    }
    if (base + step < n) load(base + step);
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const long long idx = base + k * 256;
      if (idx < n) {
        const long long tt = idx / nc;
        const int cc = (int)(idx - tt * nc);
        st16<NT>(h + tt * hs16 + cc, fwd_math(gc[k], uc[k]));
      }
    }
  }
}

// Row-tile shape of the production kernel: a workgroup owns 32 rows, wave w a quarter of the columns,
// 128-column chunks, loads of chunk c+1 issued before chunk c is computed (PF) or not.
template <bool PF, bool NT>
__global__ __launch_bounds__(256) void fwd_rowtile(const uint4* __restrict__ gu, uint4* __restrict__ h, long long T,
                                                   int nc, long long hs16) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long r0 = (long long)blockIdx.x * 32;
  const int cq = lane & 15, rq = lane >> 4;
  const int nch = nc / 16;  // 128-column chunks
  const int c0 = nch * wave / 4, c1 = nch * (wave + 1) / 4;
  uint4 g[8], u[8];
  auto load = [&](int c) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const long long row = r0 + 4 * i + rq;
      g[i] = gu[row * 2 * nc + c * 16 + cq];
      u[i] = gu[row * 2 * nc + nc + c * 16 + cq];
    }
  };
  if (PF) load(c0);
  for (int c = c0; c < c1; ++c) {
    if (!PF) load(c);
    uint4 gc[8], uc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      gc[i] = g[i];
      uc[i] = u[i];
    }
    if (PF && c + 1 < c1) load(c + 1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const long long row = r0 + 4 * i + rq;
      st16<NT>(h + row * hs16 + c * 16 + cq, fwd_math(gc[i], uc[i]));
    }
  }
}

__device__ __forceinline__ void bwd_math(uint4 g, uint4 u, uint4 d, uint4& dg, uint4& du) {
  const unsigned* gp = reinterpret_cast<const unsigned*>(&g);
  const unsigned* up = reinterpret_cast<const unsigned*>(&u);
  const unsigned* dp = reinterpret_cast<const unsigned*>(&d);
  unsigned* o1 = reinterpret_cast<unsigned*>(&dg);
  unsigned* o2 = reinterpret_cast<unsigned*>(&du);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float gg[2] = {lo(gp[k]), hi(gp[k])}, uu[2] = {lo(up[k]), hi(up[k])}, dd[2] = {lo(dp[k]), hi(dp[k])};
    float a[2], b[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const float sg = 1.0f / (1.0f + __expf(-gg[e]));
      b[e] = dd[e] * gg[e] * sg;
      a[e] = dd[e] * uu[e] * sg * (1.0f + gg[e] * (1.0f - sg));
    }
    o1[k] = pk(a[0], a[1]);
    o2[k] = pk(b[0], b[1]);
  }
}

// Backward structure of the production fused kernel: a workgroup owns 512 columns (wave: 128) and RB
// rows walked in 16-row sub-tiles.  PFG: g/u of sub-tile s+1 issued before s is computed; PFD: da too.
template <bool PFG, bool PFD, bool NT>
__global__ __launch_bounds__(256, 2) void bwd_colwalk(const uint4* __restrict__ gu, const uint4* __restrict__ da,
                                                      uint4* __restrict__ dgu, long long T, int nc, long long ds16,
                                                      int RB, int ncb) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int cb = blockIdx.x % ncb, rb = blockIdx.x / ncb;
  const int cw = cb * 64 + 16 * wave;  // chunk index of this wave's first 8-column chunk
  const int cq = lane & 15, rq = lane >> 4;
  const long long rbeg = (long long)rb * RB, rend = rbeg + RB < T ? rbeg + RB : T;
  uint4 g[4], u[4], d[4];
  auto ld_gu = [&](long long r) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const long long row = r + 4 * i + rq;
      g[i] = gu[row * 2 * nc + cw + cq];
      u[i] = gu[row * 2 * nc + nc + cw + cq];
    }
  };
  auto ld_d = [&](long long r) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] = da[(r + 4 * i + rq) * nc + cw + cq];
  };
  if (PFG) ld_gu(rbeg);
  if (PFD) ld_d(rbeg);
  for (long long r0 = rbeg; r0 < rend; r0 += 16) {
    if (!PFG) ld_gu(r0);
    if (!PFD) ld_d(r0);
    uint4 gc[4], uc[4], dc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      gc[i] = g[i];
      uc[i] = u[i];
      dc[i] = d[i];
    }
    if (PFG && r0 + 16 < rend) ld_gu(r0 + 16);
    if (PFD && r0 + 16 < rend) ld_d(r0 + 16);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const long long row = r0 + 4 * i + rq;
      uint4 a, b;
      bwd_math(gc[i], uc[i], dc[i], a, b);
      st16<NT>(dgu + row * ds16 + cw + cq, a);
      st16<NT>(dgu + row * ds16 + nc + cw + cq, b);
    }
  }
}

int main(int argc, char** argv) {
  const long long T = argc > 1 ? atoll(argv[1]) : 16384;
  const int F = 14336, Rp = 64;
  const int nc = F / 8;
  const long long hs = F + Rp, hs16 = hs / 8;
  const size_t gu_bytes = (size_t)T * 2 * F * 2, h_bytes = (size_t)T * hs * 2;
  void *gu, *h, *h0;
  CK(hipMalloc(&gu, gu_bytes));
  CK(hipMalloc(&h, h_bytes));
  CK(hipMalloc(&h0, h_bytes));
  {
    std::vector<unsigned short> host(gu_bytes / 2);
    unsigned s = 12345u;
    for (auto& v : host) {
      s = s * 1664525u + 1013904223u;
      float f = ((s >> 8) & 0xffff) / 16384.0f - 2.0f;
      unsigned bits;
      memcpy(&bits, &f, 4);
      v = (unsigned short)(bits >> 16);
    }
    CK(hipMemcpy(gu, host.data(), gu_bytes, hipMemcpyHostToDevice));
  }
  CK(hipMemset(h, 0, h_bytes));
  CK(hipMemset(h0, 0, h_bytes));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double fwd_bytes = (double)T * 2 * F * 2 + (double)T * F * 2;
  const long long n = T * nc;
  auto run = [&](const char* name, auto launch, double bytes, bool check) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0.f;
    const int reps = 20;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
      sum += ms;
    }
    int ok = -1;
    if (check) {
      std::vector<unsigned short> a(h_bytes / 2), b(h_bytes / 2);
      CK(hipMemcpy(a.data(), h, h_bytes, hipMemcpyDeviceToHost));
      CK(hipMemcpy(b.data(), h0, h_bytes, hipMemcpyDeviceToHost));
      ok = 1;
      for (long long t = 0; t < T && ok; ++t)
        if (memcmp(&a[t * hs], &b[t * hs], (size_t)F * 2)) ok = 0;
      CK(hipMemset(h, 0, h_bytes));
    }
    printf("{\"variant\": \"%s\", \"us_best\": %.1f, \"us_mean\": %.1f, \"TBps_best\": %.3f, \"match\": %d}\n", name,
           best * 1e3, sum / reps * 1e3, bytes / (best * 1e-3) / 1e12, ok);
    fflush(stdout);
  };
  const uint4* G = (const uint4*)gu;
  uint4* H = (uint4*)h;
  // reference output (variant 0) into h0
  hipLaunchKernelGGL((fwd_oneshot<1, false>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, G, (uint4*)h0, T, nc,
                     hs16);
  CK(hipDeviceSynchronize());
  const long long n11 = (long long)(gu_bytes / 2) / 16;  // copy half of gu (1:1, = h-sized x 2 read / write)
  run("copy11_940MB", [&] {
        hipLaunchKernelGGL(copy11, dim3((unsigned)((n11 + 1023) / 1024)), dim3(256), 0, 0, G, H, n11 < (long long)(h_bytes / 16) ? n11 : (long long)(h_bytes / 16));
      }, 2.0 * (double)((n11 < (long long)(h_bytes / 16) ? n11 : (long long)(h_bytes / 16)) * 16), false);
  CK(hipMemset(h, 0, h_bytes));
  run("fwd_u1", [&] { hipLaunchKernelGGL((fwd_oneshot<1, false>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, G, H, T, nc, hs16); }, fwd_bytes, true);
  run("fwd_u2", [&] { hipLaunchKernelGGL((fwd_oneshot<2, false>), dim3((unsigned)((n + 511) / 512)), dim3(256), 0, 0, G, H, T, nc, hs16); }, fwd_bytes, true);
  run("fwd_u4", [&] { hipLaunchKernelGGL((fwd_oneshot<4, false>), dim3((unsigned)((n + 1023) / 1024)), dim3(256), 0, 0, G, H, T, nc, hs16); }, fwd_bytes, true);
  run("fwd_u8", [&] { hipLaunchKernelGGL((fwd_oneshot<8, false>), dim3((unsigned)((n + 2047) / 2048)), dim3(256), 0, 0, G, H, T, nc, hs16); }, fwd_bytes, true);
  run("fwd_u1_nt", [&] { hipLaunchKernelGGL((fwd_oneshot<1, true>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, G, H, T, nc, hs16); }, fwd_bytes, true);
  run("fwd_u4_nt", [&] { hipLaunchKernelGGL((fwd_oneshot<4, true>), dim3((unsigned)((n + 1023) / 1024)), dim3(256), 0, 0, G, H, T, nc, hs16); }, fwd_bytes, true);
  for (int mult : {2, 4, 8}) {
    char nm[64];
    snprintf(nm, sizeof nm, "fwd_gs4_x%d", mult);
    run(nm, [&] { hipLaunchKernelGGL((fwd_gs<4, false>), dim3(cus * mult), dim3(256), 0, 0, G, H, T, nc, hs16); }, fwd_bytes, true);
    snprintf(nm, sizeof nm, "fwd_gs4_nt_x%d", mult);
    run(nm, [&] { hipLaunchKernelGGL((fwd_gs<4, true>), dim3(cus * mult), dim3(256), 0, 0, G, H, T, nc, hs16); }, fwd_bytes, true);
    snprintf(nm, sizeof nm, "fwd_gs2_x%d", mult);
    run(nm, [&] { hipLaunchKernelGGL((fwd_gs<2, false>), dim3(cus * mult), dim3(256), 0, 0, G, H, T, nc, hs16); }, fwd_bytes, true);
  }
  const unsigned rt = (unsigned)(T / 32);
  run("fwd_rowtile", [&] { hipLaunchKernelGGL((fwd_rowtile<false, false>), dim3(rt), dim3(256), 0, 0, G, H, T, nc, hs16); }, fwd_bytes, true);
  run("fwd_rowtile_pf", [&] { hipLaunchKernelGGL((fwd_rowtile<true, false>), dim3(rt), dim3(256), 0, 0, G, H, T, nc, hs16); }, fwd_bytes, true);
  run("fwd_rowtile_nt", [&] { hipLaunchKernelGGL((fwd_rowtile<false, true>), dim3(rt), dim3(256), 0, 0, G, H, T, nc, hs16); }, fwd_bytes, true);
  run("fwd_rowtile_pf_nt", [&] { hipLaunchKernelGGL((fwd_rowtile<true, true>), dim3(rt), dim3(256), 0, 0, G, H, T, nc, hs16); }, fwd_bytes, true);
  // ---- backward: da [T][F], dgu [T][2F + Rp]
  const long long ds = 2LL * F + Rp, ds16 = ds / 8;
  const size_t da_bytes = (size_t)T * F * 2, dgu_bytes = (size_t)T * ds * 2;
  void *da, *dgu, *dgu0;
  CK(hipMalloc(&da, da_bytes));
  CK(hipMalloc(&dgu, dgu_bytes));
  CK(hipMalloc(&dgu0, dgu_bytes));
  CK(hipMemcpy(da, gu, da_bytes, hipMemcpyDeviceToDevice));  // any finite bf16 values
  CK(hipMemset(dgu, 0, dgu_bytes));
  CK(hipMemset(dgu0, 0, dgu_bytes));
  const double bwd_bytes = (double)T * 2 * F * 2 + (double)T * F * 2 + (double)T * 2 * F * 2;
  const int ncb = F / 512;
  auto bwd_run = [&](const char* name, auto kern, int wgs, bool ref) {
    long long nrb = wgs / ncb, rb = (T + nrb - 1) / nrb;
    rb = (rb + 15) / 16 * 16;
    nrb = (T + rb - 1) / rb;
    const dim3 grid((unsigned)(ncb * nrb));
    void* out = ref ? dgu0 : dgu;
    auto launch = [&] {
      hipLaunchKernelGGL(kern, grid, dim3(256), 0, 0, (const uint4*)gu, (const uint4*)da, (uint4*)out, T, nc, ds16,
                         (int)rb, ncb);
    };
    if (ref) {
      launch();
      CK(hipDeviceSynchronize());
      return;
    }
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0.f;
    const int reps = 20;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
      sum += ms;
    }
    std::vector<unsigned short> a(dgu_bytes / 2), b(dgu_bytes / 2);
    CK(hipMemcpy(a.data(), dgu, dgu_bytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), dgu0, dgu_bytes, hipMemcpyDeviceToHost));
    int ok = 1;
    for (long long t = 0; t < T && ok; ++t)
      if (memcmp(&a[t * ds], &b[t * ds], (size_t)F * 4)) ok = 0;
    CK(hipMemset(dgu, 0, dgu_bytes));
    printf("{\"variant\": \"%s_wgs%d\", \"us_best\": %.1f, \"us_mean\": %.1f, \"TBps_best\": %.3f, \"match\": %d}\n", name,
           wgs, best * 1e3, sum / reps * 1e3, bwd_bytes / (best * 1e-3) / 1e12, ok);
    fflush(stdout);
  };
  bwd_run("ref", bwd_colwalk<false, false, false>, 512, true);
  for (int wgs : {512, 1024}) {
    bwd_run("bwd_nopf", bwd_colwalk<false, false, false>, wgs, false);
    bwd_run("bwd_pfgu", bwd_colwalk<true, false, false>, wgs, false);
    bwd_run("bwd_pfall", bwd_colwalk<true, true, false>, wgs, false);
    bwd_run("bwd_pfgu_nt", bwd_colwalk<true, false, true>, wgs, false);
    bwd_run("bwd_pfall_nt", bwd_colwalk<true, true, true>, wgs, false);
  }
  CK(hipFree(da));
  CK(hipFree(dgu));
  CK(hipFree(dgu0));
  CK(hipFree(gu));
  CK(hipFree(h));
  CK(hipFree(h0));
  return 0;
}
