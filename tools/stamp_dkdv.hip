// Diagnostic: where the dK/dV kernel's loop spends its cycles (in-kernel s_memtime stamps, guide
// "In-kernel stamps").  Builds the backward kernels with FTC_STAMPS, runs the Llama-3-8B layer shape
// (B4 S4096 H32 KV8 D128 causal) and prints, for the stamped workgroup, each wave's share of the loop
// in: sync (counted vmcnt + lgkmcnt(0) + barrier + next DMA issue), A (S / dP' MFMA chains), B1
// (exp / mask / pack VALU), B2 (dV / dK MFMAs).  Read shares, not lengths: the stamps' own waits
// forbid some of the real kernel's overlap.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DFTC_STAMPS -Icsrc/kernels tools/stamp_dkdv.hip -o tools/stamp_dkdv
//   tools/stamp_dkdv [block ...]        (default: blocks 0 (heaviest key block) and 256)
// FTC_FLASH_DKDV_WAVES=il stamps the interleaved 4-wave kernel instead: its columns are sync / A (S, dP'
// MFMAs) / X (B2 of the previous slice's half 1 + B1 of half 0) / Y (B2 of half 0 + B1 of half 1).
#include "../csrc/kernels/flash_attn_bwd.hip"

#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

static void fill_bf16(std::vector<uint16_t>& v, unsigned seed, float amp) {
  unsigned x = seed * 2654435761u + 1;
  for (auto& e : v) {
    x = x * 1664525u + 1013904223u;
    const float f = ((x >> 8) * (1.0f / 16777216.0f) * 2.f - 1.f) * amp;
    unsigned u;
    std::memcpy(&u, &f, 4);
    e = (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
  }
}

int main(int argc, char** argv) {
  const int B = 4, S = 4096, H = 32, KV = 8, D = 128;
  const long long rows = (long long)B * S;
  std::vector<uint16_t> hq(rows * H * D), hk(rows * KV * D), hv(rows * KV * D), ho(rows * H * D), hdo(rows * H * D);
  fill_bf16(hq, 1, 1.f);
  fill_bf16(hk, 2, 1.f);
  fill_bf16(hv, 3, 1.f);
  fill_bf16(ho, 4, 0.5f);
  fill_bf16(hdo, 5, 0.1f);
  std::vector<float> hl((size_t)B * H * S, 6.0f);
  uint16_t *q, *k, *v, *o, *dout, *dq, *dk, *dv;
  float* lse;
  void* ws;
  long long wsb = 0;
  ftc_flash_bwd_workspace(B, S, H, D, &wsb);
  CK(hipMalloc(&q, hq.size() * 2));
  CK(hipMalloc(&k, hk.size() * 2));
  CK(hipMalloc(&v, hv.size() * 2));
  CK(hipMalloc(&o, ho.size() * 2));
  CK(hipMalloc(&dout, hdo.size() * 2));
  CK(hipMalloc(&dq, hq.size() * 2));
  CK(hipMalloc(&dk, hk.size() * 2));
  CK(hipMalloc(&dv, hv.size() * 2));
  CK(hipMalloc(&lse, hl.size() * 4));
  CK(hipMalloc(&ws, wsb));
  CK(hipMemcpy(q, hq.data(), hq.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(k, hk.data(), hk.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(v, hv.data(), hv.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(o, ho.data(), ho.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dout, hdo.data(), hdo.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(lse, hl.data(), hl.size() * 4, hipMemcpyHostToDevice));
  std::vector<int> blocks;
  for (int i = 1; i < argc; ++i) blocks.push_back(atoi(argv[i]));
  if (blocks.empty()) blocks = {0, 256};
  const int g_kv = B * KV * (S / 256);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int blk : blocks) {
    if (blk < 0 || blk >= g_kv) continue;
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_block), &blk, sizeof(int)));
    {
      unsigned long long z[8][6];
      memset(z, 0, sizeof(z));
      CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z)));
    }
    float ms = 0.f;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0, 0));
      const int rc = ftc_flash_bwd(q, k, v, o, dout, lse, dq, dk, dv, ws, B, S, H, KV, D, H * D, KV * D, H * D, H * D,
                                   H * D, KV * D, 0.08838834764831845f, 1, 0, nullptr, nullptr, 0, nullptr, nullptr, nullptr,
                                   0);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      if (rc != 0) {
        fprintf(stderr, "ftc_flash_bwd rc=%d\n", rc);
        return 1;
      }
      CK(hipEventElapsedTime(&ms, e0, e1));
    }
    unsigned long long st[8][6];
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof(st)));
    printf("block %d (delta + dK/dV + dQ, stamp build): %.3f ms\n", blk, ms);
    printf("| wave | slices | loop cycles | cyc/slice | sync | A (S,dP MFMA) | B1 (VALU) | B2 (dV,dK MFMA) |\n");
    printf("|---:|---:|---:|---:|---:|---:|---:|---:|\n");
    for (int w = 0; w < 8; ++w) {
      const double tot = (double)st[w][4], n = (double)st[w][5];
      if (tot <= 0) continue;
      if (n <= 0) continue;
      printf("| %d | %.0f | %.0f | %.0f | %.1f %% | %.1f %% | %.1f %% | %.1f %% |\n", w, n, tot, tot / n,
             100.0 * st[w][0] / tot, 100.0 * st[w][1] / tot, 100.0 * st[w][2] / tot, 100.0 * st[w][3] / tot);
    }
  }
  return 0;
}
