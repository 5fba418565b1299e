// host_io.hpp -- how the library moves bytes between caller host memory and HBM (api.hip).
//
// The cgo caller hands the library the bytes of an OpenTable'd .sst: a Go heap buffer under the
// default LoadToRAM mode (options.go:76, table/table.go:117-123,329-338) or an mmap (MemoryMap,
// y/mmap.go:11-21), and pageable output arrays.  The HIP runtime never sees such a pointer:
//  * memory the runtime itself page-locked (hipHostMalloc -- lsmgpu_host_alloc, torch's pinned
//    allocator -- or a caller's own hipHostRegister) is DMA'd directly;
//  * everything else is staged through page-locked buffers this library allocated once per
//    context with hipHostMalloc, filled / drained with memcpy by a small per-context thread pool.
// Until ABI 3 the library page-locked caller ranges with hipHostRegister around each call.  Under
// register / unregister cycles at re-used heap addresses (exactly what compaction's OpenTable /
// DecrRef churn produces, levels.go:281-298) the runtime's registration bookkeeping went stale: a
// later pageable copy into a re-used address faulted (round 5, GPUTEST_r05: illegal address on a
// pageable D2H, hipPointerGetAttributes already at 700).  With staging, no caller address is ever
// registered with or passed to the runtime, so that whole class of state is gone.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <thread>

#include "copy_pool.hpp"

namespace lsmgpu {

// A page-locked host buffer owned by the library (hipHostMalloc), grown on demand.  Growing
// frees the old buffer: callers grow only when no DMA into or out of it is in flight.
struct PinnedBuf {
  uint8_t* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t need) {
    if (need <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    const size_t n = std::max<size_t>((need + 4095) / 4096 * 4096, 1u << 16);
    hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p), n, hipHostMallocPortable);
    if (e == hipSuccess) cap = n;
    else p = nullptr;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Whether [p, p + n) is host memory the HIP runtime already knows as page-locked (both ends
// checked).  Pageable memory answers with an error or "unregistered": staged.
inline bool runtime_pinned(const void* p, uint64_t n) {
  if (!p || !n) return false;
  for (const void* q : {p, static_cast<const void*>(static_cast<const uint8_t*>(p) + n - 1)}) {
    hipPointerAttribute_t a{};
    const hipError_t e = hipPointerGetAttributes(&a, q);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    if (a.type != hipMemoryTypeHost) return false;
  }
  return true;
}

// Whether p is device memory (a data_on_device = 0 call handed a device pointer: staging it with
// memcpy would fault on the host)
inline bool device_memory(const void* p) {
  hipPointerAttribute_t a{};
  const hipError_t e = hipPointerGetAttributes(&a, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeDevice;
}

// The staging pair of one context: two page-locked pieces used alternately, each guarded by an
// event on the stream of the DMA that last used it, so host memcpy of one piece overlaps the
// DMA of the other.
class Stager {
 public:
  static constexpr uint64_t kPiece = 16ull << 20;
  explicit Stager(CopyPool* pool) : pool_(pool) {}
  void release() {
    for (int b = 0; b < 2; b++) {
      if (ev_[b]) (void)hipEventSynchronize(ev_[b]);
      buf_[b].release();
      if (ev_[b]) (void)hipEventDestroy(ev_[b]);
      ev_[b] = nullptr;
      armed_[b] = false;
    }
  }

  // Host -> HBM.  On return the caller's src may be reused (staged bytes already copied out of
  // it); a direct DMA (runtime-pinned src) may still be in flight on s.
  hipError_t h2d(void* dst, const void* src, uint64_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    if (runtime_pinned(src, n)) {
      const hipError_t e = hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, s);
      if (e != hipErrorInvalidValue) return e;  // refused (spans two allocations): staged below
      (void)hipGetLastError();
    }
    hipError_t e = init();
    for (uint64_t o = 0; o < n && e == hipSuccess; o += kPiece) {
      const uint64_t m = std::min(kPiece, n - o);
      const int b = next_;
      next_ ^= 1;
      if (armed_[b] && (e = hipEventSynchronize(ev_[b])) != hipSuccess) break;
      pool_->copy(buf_[b].p, static_cast<const uint8_t*>(src) + o, m);
      e = hipMemcpyAsync(static_cast<uint8_t*>(dst) + o, buf_[b].p, m, hipMemcpyHostToDevice, s);
      if (e == hipSuccess) e = hipEventRecord(ev_[b], s);
      armed_[b] = e == hipSuccess;
    }
    return e;
  }

  // HBM -> host, after the work already on s.  Staged: returns when dst holds the bytes.  Direct
  // (runtime-pinned dst): enqueued on s; the caller synchronizes s before reading dst.
  hipError_t d2h(void* dst, const void* src, uint64_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    if (runtime_pinned(dst, n)) {
      const hipError_t e = hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, s);
      if (e != hipErrorInvalidValue) return e;
      (void)hipGetLastError();
    }
    hipError_t e = init();
    uint64_t pend_o = 0, pend_m = 0;
    int pend_b = -1;
    const uint64_t np = (n + kPiece - 1) / kPiece;
    for (uint64_t k = 0; k <= np && e == hipSuccess; k++) {  // piece k issued, piece k-1 drained
      const uint64_t o = k * kPiece;
      const uint64_t m = k < np ? std::min(kPiece, n - o) : 0;
      int b = -1;
      if (m) {
        b = next_;
        next_ ^= 1;
        if (armed_[b] && (e = hipEventSynchronize(ev_[b])) != hipSuccess) break;
        e = hipMemcpyAsync(buf_[b].p, static_cast<const uint8_t*>(src) + o, m, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipEventRecord(ev_[b], s);
        armed_[b] = e == hipSuccess;
        if (e != hipSuccess) break;
      }
      if (pend_b >= 0) {  // the previous piece: wait for its DMA, then drain it
        if ((e = hipEventSynchronize(ev_[pend_b])) != hipSuccess) break;
        pool_->copy(static_cast<uint8_t*>(dst) + pend_o, buf_[pend_b].p, pend_m);
      }
      pend_o = o;
      pend_m = m;
      pend_b = b;
      if (!m) break;
    }
    return e;
  }

 private:
  hipError_t init() {
    for (int b = 0; b < 2; b++) {
      if (!ev_[b]) {
        const hipError_t e = hipEventCreateWithFlags(&ev_[b], hipEventDisableTiming);
        if (e != hipSuccess) return e;
      }
      const hipError_t e = buf_[b].ensure(kPiece);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  CopyPool* pool_;
  PinnedBuf buf_[2];
  hipEvent_t ev_[2] = {nullptr, nullptr};
  bool armed_[2] = {false, false};
  int next_ = 0;
};

// The process's CPU quota (cgroup v2 cpu.max, or v1 cfs quota / period), 0 if none
inline unsigned cgroup_cpus() {
  long long q = -1, per = 0;
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char a[32] = {0};
    if (fscanf(f, "%31s %lld", a, &per) == 2 && a[0] != 'm') q = atoll(a);
    fclose(f);
  } else if (FILE* f1 = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
    if (fscanf(f1, "%lld", &q) != 1) q = -1;
    fclose(f1);
    if (FILE* f2 = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
      if (fscanf(f2, "%lld", &per) != 1) per = 0;
      fclose(f2);
    }
  }
  return q > 0 && per > 0 ? (unsigned)std::max(1ll, q / per) : 0u;
}

// Copy-pool size: LSMGPU_COPY_THREADS, else half the hardware threads, at most 16, and at most
// one less than the CPU quota (the calling thread memcpys too).  C2 1 GiB from pageable memory,
// materialize: 8 threads 0.035 s, 16 threads 0.026 s against a 0.0186 s PCIe bound (profiles/r06b)
// -- on a box whose job quota is 16 CPUs, so the 16 threads of the default then oversubscribed it.
inline unsigned copy_threads() {
  if (const char* e = getenv("LSMGPU_COPY_THREADS")) return (unsigned)std::max(1, atoi(e));
  const unsigned hw = std::thread::hardware_concurrency();
  unsigned n = std::max(1u, std::min(16u, hw / 2));
  if (const unsigned q = cgroup_cpus()) n = std::max(1u, std::min(n, q > 1 ? q - 1 : 1u));
  return n;
}

}  // namespace lsmgpu
