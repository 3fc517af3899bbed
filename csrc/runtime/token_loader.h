// Native token loader core (no Python: also built stand-alone under ASan/UBSan and TSan by
// tests/test_native_sanitizers.py) for the worker runtime (SURVEY.md §7.1 "data/"): memory-mapped token file,
// a pool of worker threads gathering fixed [batch, seq_len + 1] windows into a ring of caller-owned
// (pinned) int64 buffers ahead of the training loop, delivered strictly in batch order.
//
// Division of labour with train/data.py: Python draws the per-epoch window permutation (numpy, so the
// native and the fallback path produce identical batches) and owns the buffers (torch pinned host
// tensors, so the H2D copy is an async DMA); this file does the O(tokens) work -- page-faulting the
// mmap, the uint16/uint32 -> int64 widening and the window gather -- off the Python thread.
//
// Batch b of an epoch for rank r of w ranks takes windows order[((b * w + r) * batch + i) % n_windows],
// i < batch; window j covers tokens [j * seq_len, j * seq_len + seq_len] (seq_len + 1 tokens).
#pragma once

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace ftc_rt {

class TokenLoader {
 public:
  // offset: bytes before the first token (a .npy header); vocab > 0: every gathered id is checked
  // against it and a batch holding an id >= vocab fails with an error instead of reaching the GPU
  // (an out-of-range id would make the embedding gather fault the device)
  TokenLoader(const std::string& path, int itemsize, int64_t seq_len, int64_t batch, int rank, int world, int threads,
              int64_t offset = 0, int64_t vocab = 0)
      : itemsize_(itemsize), seq_(seq_len), batch_(batch), rank_(rank), world_(world), offset_(offset), vocab_(vocab) {
    if (itemsize != 2 && itemsize != 4) throw std::runtime_error("token_loader: itemsize must be 2 or 4");
    if (offset < 0 || offset % itemsize) throw std::runtime_error("token_loader: offset must be a multiple of itemsize");
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw std::runtime_error("token_loader: cannot open " + path);
    struct stat st;
    if (fstat(fd_, &st) != 0) throw std::runtime_error("token_loader: fstat failed");
    bytes_ = (size_t)st.st_size;
    if ((int64_t)bytes_ <= offset) throw std::runtime_error("token_loader: file shorter than its header");
    ntok_ = (int64_t)((bytes_ - (size_t)offset) / itemsize);
    if (ntok_ <= seq_) throw std::runtime_error("token_loader: file shorter than one window");
    map_ = ::mmap(nullptr, bytes_, PROT_READ, MAP_SHARED, fd_, 0);
    if (map_ == MAP_FAILED) throw std::runtime_error("token_loader: mmap failed");
    ::madvise(map_, bytes_, MADV_RANDOM);
    n_windows_ = (ntok_ - 1) / seq_;
    nthreads_ = threads > 0 ? threads : 2;
  }

  ~TokenLoader() {
    stop();
    if (map_ && map_ != MAP_FAILED) ::munmap(map_, bytes_);
    if (fd_ >= 0) ::close(fd_);
  }

  int64_t n_windows() const { return n_windows_; }
  int64_t n_tokens() const { return ntok_; }

  // ring of caller-owned int64 buffers, each batch * (seq_len + 1) elements
  void set_buffers(const std::vector<uintptr_t>& ptrs) {
    stop();
    bufs_.assign(ptrs.begin(), ptrs.end());
    state_.assign(bufs_.size(), kFree);
  }

  // (re)start producing batches [first, last) of an epoch with window order `order`
  void start(const int64_t* order, size_t n, int64_t first, int64_t last) {
    stop();
    if (bufs_.empty()) throw std::runtime_error("token_loader: set_buffers first");
    order_.assign(order, order + n);
    if ((int64_t)order_.size() != n_windows_) throw std::runtime_error("token_loader: order length != n_windows");
    first_ = first;
    last_ = last;
    next_fill_ = first;
    next_take_ = first;
    for (auto& s : state_) s = kFree;
    running_ = true;
    for (int t = 0; t < nthreads_; ++t) workers_.emplace_back([this] { work(); });
  }

  // blocks until the next batch (in order) is in its buffer; returns the buffer index (-1 when the
  // range is exhausted)
  int acquire() {
    std::unique_lock<std::mutex> lk(mu_);
    if (next_take_ >= last_) return -1;
    const int slot = (int)(next_take_ % (int64_t)bufs_.size());
    cv_.wait(lk, [&] { return state_[slot] == kReady || !error_.empty(); });
    if (!error_.empty()) throw std::runtime_error(error_);
    state_[slot] = kTaken;
    ++next_take_;
    return slot;
  }

  // the caller is done with the buffer (its device copy completed)
  void release(int slot) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (slot < 0 || slot >= (int)state_.size()) throw std::runtime_error("token_loader: bad slot");
      state_[slot] = kFree;
    }
    cv_.notify_all();
  }

  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      running_ = false;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
    workers_.clear();
  }

 private:
  enum : int { kFree = 0, kFilling = 1, kReady = 2, kTaken = 3 };

  void work() {
    for (;;) {
      int64_t b;
      int slot;
      {
        std::unique_lock<std::mutex> lk(mu_);
        // batch b goes to slot b % depth once that slot is free; batches are claimed in order so a
        // slot is never claimed by two batches at once
        cv_.wait(lk, [&] {
          if (!running_ || next_fill_ >= last_) return true;
          return state_[next_fill_ % (int64_t)bufs_.size()] == kFree;
        });
        if (!running_ || next_fill_ >= last_) return;
        b = next_fill_++;
        slot = (int)(b % (int64_t)bufs_.size());
        state_[slot] = kFilling;
      }
      try {
        fill(b, reinterpret_cast<int64_t*>(bufs_[slot]));
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> lk(mu_);
        error_ = e.what();
      }
      {
        std::lock_guard<std::mutex> lk(mu_);
        state_[slot] = kReady;
      }
      cv_.notify_all();
    }
  }

  void fill(int64_t b, int64_t* out) const {
    const int64_t w = seq_ + 1;
    const char* base = static_cast<const char*>(map_) + offset_;
    for (int64_t i = 0; i < batch_; ++i) {
      const int64_t j = order_[(size_t)(((b * world_ + rank_) * batch_ + i) % n_windows_)];
      const int64_t t0 = j * seq_;
      int64_t* dst = out + i * w;
      uint32_t hi = 0;
      if (itemsize_ == 2) {
        const uint16_t* src = reinterpret_cast<const uint16_t*>(base) + t0;
        for (int64_t k = 0; k < w; ++k) {
          dst[k] = src[k];
          hi = src[k] > hi ? src[k] : hi;
        }
      } else {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(base) + t0;
        for (int64_t k = 0; k < w; ++k) {
          dst[k] = src[k];
          hi = src[k] > hi ? src[k] : hi;
        }
      }
      if (vocab_ > 0 && (int64_t)hi >= vocab_)  // (int32 ids read as uint32: negatives land here too)
        throw std::runtime_error("token_loader: token id " + std::to_string(hi) + " >= vocab " +
                                 std::to_string(vocab_) + " in window " + std::to_string(j));
    }
  }

  int itemsize_;
  int64_t seq_, batch_;
  int rank_, world_;
  int64_t offset_ = 0, vocab_ = 0;
  int fd_ = -1;
  void* map_ = nullptr;
  size_t bytes_ = 0;
  int64_t ntok_ = 0, n_windows_ = 0;
  int nthreads_ = 2;
  std::vector<uintptr_t> bufs_;
  std::vector<int> state_;
  std::vector<int64_t> order_;
  int64_t first_ = 0, last_ = 0, next_fill_ = 0, next_take_ = 0;
  bool running_ = false;
  std::string error_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<std::thread> workers_;
};

}  // namespace ftc_rt
