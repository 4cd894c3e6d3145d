// Host <-> HBM transfers of batches that arrive in pageable host memory
// (SURVEY.md §8(d) tier 2: packed host CSR -> H2D -> kernels -> D2H).
//
// A pageable hipMemcpy stages through the runtime's own small bounce buffers on
// one thread (~8 GB/s measured, profiles/r02_v3_tiers.json).  Here T host threads
// each own two pinned staging buffers and a slice of the chunks: a thread copies
// chunk k into a free buffer (memcpy at host-memory speed, T in parallel), issues
// its DMA on the caller's stream and moves on to its next chunk while that DMA
// runs; a buffer is reused only after the event recorded behind its DMA.  So the
// PCIe link, not the staging copy, bounds the transfer.  D2H is the mirror image:
// DMA into a buffer, wait for it, copy out.
//
// Unlike the compute entry points these calls use host threads and one
// process-wide staging pool (allocated on first use, serialised by a mutex).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace spx {

constexpr size_t kStageChunk = size_t(8) << 20;  // bytes per DMA
constexpr int kStageThreads = 8;                // staging threads (2 pinned buffers each)

struct StagePool {
  std::mutex mu;
  int device = -1;
  std::vector<void*> buf;          // 2 per thread, pinned, portable
  std::vector<hipEvent_t> ev;      // the DMA last issued from each buffer (this device)
  std::vector<char> used;          // ev[i] has been recorded
  ~StagePool() {}                  // left to process teardown (the runtime may be gone)

  hipError_t ready() {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (buf.empty()) {
      buf.assign(2 * kStageThreads, nullptr);
      for (auto& b : buf)
        if ((e = hipHostMalloc(&b, kStageChunk, hipHostMallocPortable)) != hipSuccess) return e;
    }
    if (dev != device) {  // events belong to a device
      for (size_t i = 0; i < ev.size(); ++i) {
        if (used[i]) (void)hipEventSynchronize(ev[i]);
        (void)hipEventDestroy(ev[i]);
      }
      ev.assign(buf.size(), nullptr);
      used.assign(buf.size(), 0);
      for (auto& x : ev)
        if ((e = hipEventCreateWithFlags(&x, hipEventDisableTiming)) != hipSuccess) return e;
      device = dev;
    }
    return hipSuccess;
  }
};

inline StagePool& stage_pool() {
  static StagePool* p = new StagePool();  // never destroyed: outlives static teardown order
  return *p;
}

// Chunks k = t, t + T, ... of [0, n) on thread t; buffer slot alternates.
// h2d: memcpy(src chunk -> pinned), DMA pinned -> dst.  d2h: DMA src -> pinned,
// wait, memcpy pinned -> dst.
inline hipError_t staged_copy(char* dst, const char* src, size_t n, hipStream_t s, bool h2d) {
  StagePool& P = stage_pool();
  std::lock_guard<std::mutex> lock(P.mu);
  hipError_t e = P.ready();
  if (e != hipSuccess) return e;
  int dev = P.device;
  const size_t nchunks = (n + kStageChunk - 1) / kStageChunk;
  const int T = (int)std::min<size_t>(kStageThreads, std::max<size_t>(nchunks, 1));
  std::atomic<int> err{(int)hipSuccess};
  auto work = [&](int t) {
    if (hipSetDevice(dev) != hipSuccess) { err = (int)hipErrorInvalidDevice; return; }
    int slot = 0;
    for (size_t k = (size_t)t; k < nchunks && err.load() == (int)hipSuccess; k += (size_t)T, slot ^= 1) {
      const int b = 2 * t + slot;
      const size_t off = k * kStageChunk, len = std::min(kStageChunk, n - off);
      if (P.used[b] && hipEventSynchronize(P.ev[b]) != hipSuccess) { err = (int)hipErrorUnknown; return; }
      hipError_t r;
      if (h2d) {
        std::memcpy(P.buf[b], src + off, len);
        r = hipMemcpyAsync(dst + off, P.buf[b], len, hipMemcpyHostToDevice, s);
        if (r == hipSuccess) r = hipEventRecord(P.ev[b], s);
        P.used[b] = 1;
      } else {
        r = hipMemcpyAsync(P.buf[b], src + off, len, hipMemcpyDeviceToHost, s);
        if (r == hipSuccess) r = hipEventRecord(P.ev[b], s);
        if (r == hipSuccess) r = hipEventSynchronize(P.ev[b]);
        if (r == hipSuccess) std::memcpy(dst + off, P.buf[b], len);
        P.used[b] = 0;
      }
      if (r != hipSuccess) { err = (int)r; return; }
    }
  };
  if (T == 1) {
    work(0);
  } else {
    std::vector<std::thread> pool;
    for (int t = 0; t < T; ++t) pool.emplace_back(work, t);
    for (auto& th : pool) th.join();
  }
  return (hipError_t)err.load();
}

}  // namespace spx
