// Stand-alone stress driver of the native token loader (csrc/runtime/token_loader.h) for the host
// sanitizer builds in tests/test_native_sanitizers.py (ASan + UBSan, TSan): several ranks' loaders on
// one token file, worker pools racing the consumer over a small buffer ring, full and aborted epochs
// (stop() while workers are mid-fill), every delivered batch checked against the file.
//
// usage: token_loader_stress <file> <itemsize> <seq_len> <batch> <world> <threads> <depth> <epochs>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <vector>

#include "../token_loader.h"

int main(int argc, char** argv) {
  if (argc != 9) {
    std::fprintf(stderr, "usage: %s file itemsize seq batch world threads depth epochs\n", argv[0]);
    return 2;
  }
  const std::string path = argv[1];
  const int itemsize = std::atoi(argv[2]);
  const int64_t seq = std::atoll(argv[3]), batch = std::atoll(argv[4]);
  const int world = std::atoi(argv[5]), threads = std::atoi(argv[6]), depth = std::atoi(argv[7]);
  const int epochs = std::atoi(argv[8]);
  // the file itself, for checking
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return 2;
  std::fseek(f, 0, SEEK_END);
  const long bytes = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  std::vector<unsigned char> raw((size_t)bytes);
  if (std::fread(raw.data(), 1, raw.size(), f) != raw.size()) return 2;
  std::fclose(f);
  auto tok = [&](int64_t i) -> int64_t {
    if (itemsize == 2) return reinterpret_cast<const uint16_t*>(raw.data())[i];
    return reinterpret_cast<const uint32_t*>(raw.data())[i];
  };
  const int64_t w = seq + 1;
  uint64_t lcg = 12345;
  long checked = 0;
  for (int rank = 0; rank < world; ++rank) {
    ftc_rt::TokenLoader ld(path, itemsize, seq, batch, rank, world, threads);
    const int64_t nwin = ld.n_windows();
    std::vector<std::vector<int64_t>> bufs(depth, std::vector<int64_t>((size_t)(batch * w), -1));
    std::vector<uintptr_t> ptrs;
    for (auto& b : bufs) ptrs.push_back(reinterpret_cast<uintptr_t>(b.data()));
    ld.set_buffers(ptrs);
    std::vector<int64_t> order((size_t)nwin);
    for (int e = 0; e < epochs; ++e) {
      std::iota(order.begin(), order.end(), 0);
      for (int64_t i = nwin - 1; i > 0; --i) {  // deterministic shuffle
        lcg = lcg * 6364136223846793005ULL + 1442695040888963407ULL;
        std::swap(order[(size_t)i], order[(size_t)((lcg >> 33) % (uint64_t)(i + 1))]);
      }
      const int64_t nb = std::max<int64_t>(1, nwin / (batch * world));
      const bool abort_early = (e % 3) == 2;  // stop() with workers still filling
      ld.start(order.data(), order.size(), 0, nb);
      for (int64_t b = 0; b < nb; ++b) {
        if (abort_early && b == nb / 2) break;
        const int slot = ld.acquire();
        if (slot < 0) {
          std::fprintf(stderr, "premature end at batch %lld\n", (long long)b);
          return 1;
        }
        const int64_t* out = bufs[(size_t)slot].data();
        for (int64_t i = 0; i < batch; ++i) {
          const int64_t j = order[(size_t)(((b * world + rank) * batch + i) % nwin)];
          for (int64_t k = 0; k < w; ++k) {
            if (out[i * w + k] != tok(j * seq + k)) {
              std::fprintf(stderr, "mismatch rank %d batch %lld row %lld col %lld\n", rank, (long long)b,
                           (long long)i, (long long)k);
              return 1;
            }
          }
        }
        ++checked;
        ld.release(slot);
      }
      if (!abort_early && ld.acquire() != -1) {
        std::fprintf(stderr, "batches past the range\n");
        return 1;
      }
      ld.stop();
    }
  }
  std::printf("OK %ld batches checked\n", checked);
  return 0;
}
