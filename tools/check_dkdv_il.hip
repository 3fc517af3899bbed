// Numerics bisect for the IL dK/dV kernel: runs the backward with the 8-wave kernel and with IL on the same
// random inputs and prints max |dK_il - dK_8| / max |dK_8| (and dV).  Build variants with -DIL_TV2=0/1
// -DIL_PIPE=0/1:  hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc/kernels tools/check_dkdv_il.hip -o X
#include "../csrc/kernels/flash_attn_bwd.hip"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

static void fill(std::vector<uint16_t>& v, unsigned seed, float amp) {
  unsigned x = seed * 2654435761u + 1;
  for (auto& e : v) {
    x = x * 1664525u + 1013904223u;
    const float f = ((x >> 8) * (1.0f / 16777216.0f) * 2.f - 1.f) * amp;
    unsigned u;
    std::memcpy(&u, &f, 4);
    e = (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
  }
}
static float b2f(uint16_t h) {
  unsigned u = (unsigned)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

int main() {
  const int B = 2, S = 512, H = 8, KV = 2, D = 128;
  const long long rows = (long long)B * S;
  std::vector<uint16_t> hq(rows * H * D), hk(rows * KV * D), hv(rows * KV * D), ho(rows * H * D), hdo(rows * H * D);
  fill(hq, 1, 1.f); fill(hk, 2, 1.f); fill(hv, 3, 1.f); fill(ho, 4, 0.5f); fill(hdo, 5, 0.5f);
  std::vector<float> hl((size_t)B * H * S, 3.0f);
  uint16_t *q, *k, *v, *o, *dout, *dq, *dk, *dv;
  float* lse;
  void* ws;
  long long wsb = 0;
  ftc_flash_bwd_workspace(B, S, H, D, &wsb);
  hipMalloc(&q, hq.size() * 2); hipMalloc(&k, hk.size() * 2); hipMalloc(&v, hv.size() * 2);
  hipMalloc(&o, ho.size() * 2); hipMalloc(&dout, hdo.size() * 2); hipMalloc(&dq, hq.size() * 2);
  hipMalloc(&dk, hk.size() * 2); hipMalloc(&dv, hv.size() * 2); hipMalloc(&lse, hl.size() * 4); hipMalloc(&ws, wsb);
  hipMemcpy(q, hq.data(), hq.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(k, hk.data(), hk.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(v, hv.data(), hv.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(o, ho.data(), ho.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dout, hdo.data(), hdo.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(lse, hl.data(), hl.size() * 4, hipMemcpyHostToDevice);
  std::vector<uint16_t> r8k(hk.size()), r8v(hk.size()), rik(hk.size()), riv(hk.size());
  for (int variant : {8, 1}) {
    ftc_flash_dkdv_config(variant);
    const int rc = ftc_flash_bwd(q, k, v, o, dout, lse, dq, dk, dv, ws, B, S, H, KV, D, H * D, KV * D, H * D, H * D,
                                 H * D, KV * D, 0.08838834764831845f, 1, 0, nullptr, nullptr, 0, nullptr, nullptr,
                                 nullptr, 0);
    if (rc != 0 || hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
    hipMemcpy(variant == 8 ? r8k.data() : rik.data(), dk, hk.size() * 2, hipMemcpyDeviceToHost);
    hipMemcpy(variant == 8 ? r8v.data() : riv.data(), dv, hk.size() * 2, hipMemcpyDeviceToHost);
  }
  double mk = 0, ek = 0, mv = 0, ev = 0;
  long long bad = -1;
  for (size_t i = 0; i < r8k.size(); ++i) {
    mk = fmax(mk, fabs(b2f(r8k[i]))); mv = fmax(mv, fabs(b2f(r8v[i])));
    const double dk_ = fabs(b2f(r8k[i]) - b2f(rik[i])), dv_ = fabs(b2f(r8v[i]) - b2f(riv[i]));
    if (dk_ > ek) { ek = dk_; bad = (long long)i; }
    ev = fmax(ev, dv_);
  }
  printf("IL_TV2=%d IL_PIPE=%d  dK rel %.4g  dV rel %.4g  (worst dK row %lld col %lld)\n", IL_TV2, IL_PIPE, ek / mk,
         ev / mv, bad / (KV * D), bad % (KV * D));
  return 0;
}
