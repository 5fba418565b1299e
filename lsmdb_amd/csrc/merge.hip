// merge.hip -- y.MergeIterator (y/iterator.go:74-202) over K sorted runs on gfx950: the
// merge step of compactBuildTables (levels.go:239-258) between the device decode of the input
// tables and the device encode of the output tables.
//
// MergeIterator always emits the least head under elemHeap.Less (y.CompareKeys, then the lower
// `nice` = run index) and Next() drops every head equal to the last emitted key.  For sorted
// runs (SSTs are) that is: the runs' stable merge under (CompareKeys, run), keeping the first
// entry of each group of equal keys.  Computed without a heap, every entry in parallel:
//   check  (lane = entry)   runs in CompareKeys order? keys > 8 B (CompareKeys asserts it)?
//   split  (lane = tile x run) for the first entry of every 256-entry tile of a run, its rank
//                           in every other run (full binary search)
//   rank   (lane = entry)   merged position = own index in its run + for every other run the
//                           number of entries that precede it: binary search between the
//                           tile's splitters (ranks are monotone in a sorted run), upper bound
//                           for lower-index runs (equal keys of a lower nice come first),
//                           lower bound for higher-index runs
//   keep   (lane = merged position)  first of its equal-key group (bytes.Equal with the
//                           predecessor, y/iterator.go:172-181)
//   scan   (rocPRIM)        output entry index, key and value byte offsets of the kept entries
//   gather (8 lanes / entry) 16-B piece copies of key and raw vs-enc bytes, end offsets, source
// Unsorted runs (the heap would interleave them differently) and keys <= 8 B are reported in
// result[3] and produce no output.
#include <rocprim/device/device_scan.hpp>

#include "codec_common.hpp"
#include "kernels.hpp"

namespace lsmgpu {

namespace {

constexpr uint32_t M_UNSORTED = 1, M_KEY_LEN = 2, M_CAPACITY = 4;
constexpr uint32_t kMergeTile = 256;  // entries per splitter tile

struct MTri {
  uint64_t n, k, v;
};
struct MTriPlus {
  __device__ __host__ MTri operator()(const MTri& a, const MTri& b) const {
    return MTri{a.n + b.n, a.k + b.k, a.v + b.v};
  }
};

__device__ __forceinline__ const uint8_t* key_of(const MergeParams& p, uint32_t i, uint32_t& len) {
  const uint32_t s = i ? p.ke[i - 1] : 0u;
  len = p.ke[i] - s;
  return p.kd + s;
}

__device__ __forceinline__ uint32_t run_of(const MergeParams& p, uint32_t i) {
  uint32_t lo = 0, hi = p.nruns - 1;  // largest r with run_first[r] <= i
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (p.run_first[mid] <= i) lo = mid; else hi = mid - 1;
  }
  return lo;
}

}  // namespace

__global__ void merge_check_kernel(MergeParams p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  uint32_t li;
  const uint8_t* ki = key_of(p, i, li);
  uint32_t fl = 0;
  if (li <= 8) {
    fl = M_KEY_LEN;
  } else {
    const uint32_t r = run_of(p, i);
    if (i > p.run_first[r]) {
      uint32_t lp;
      const uint8_t* kp = key_of(p, i - 1, lp);
      if (lp > 8 && compare_keys(kp, lp, ki, li) > 0) fl = M_UNSORTED;
    }
  }
  if (fl) atomicOr(p.flags, fl);
}

// Entries of run s that precede key x of run r (key < x, or == x with s < r: lower nice
// first), searched in [lo, hi) of run s.
__device__ __forceinline__ uint32_t rank_in(const MergeParams& p, uint32_t s, uint32_t r,
                                            const uint8_t* kx, uint32_t lx, uint32_t lo,
                                            uint32_t hi) {
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    uint32_t lm;
    const uint8_t* km = key_of(p, mid, lm);
    const int c = compare_keys(km, lm, kx, lx);
    if (c < 0 || (c == 0 && s < r)) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// tile_base[r] = first tile of run r (tiles of kMergeTile entries never span runs)
__global__ void merge_tiles_kernel(MergeParams p) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint32_t t = 0;
  for (uint32_t r = 0; r < p.nruns; r++) {
    p.tile_base[r] = t;
    t += (p.run_first[r + 1] - p.run_first[r] + kMergeTile - 1) / kMergeTile;
  }
  p.tile_base[p.nruns] = t;
}

// Splitters: for the first entry of every tile, its absolute rank position in every other run
// (a full binary search); entries then only search between their tile's splitters.
__global__ void merge_split_kernel(MergeParams p) {
  const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t g = x / p.nruns, s = x % p.nruns;
  if (*p.flags || g >= p.tile_base[p.nruns]) return;
  uint32_t r = 0;  // run of tile g
  while (p.tile_base[r + 1] <= g) r++;
  const uint32_t i = p.run_first[r] + (g - p.tile_base[r]) * kMergeTile;
  uint32_t li;
  const uint8_t* ki = key_of(p, i, li);
  p.spl[(uint64_t)g * p.nruns + s] =
      s == r ? i : rank_in(p, s, r, ki, li, p.run_first[s], p.run_first[s + 1]);
}

__global__ void merge_rank_kernel(MergeParams p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n || *p.flags) return;
  const uint32_t r = run_of(p, i);
  const uint32_t j = i - p.run_first[r];
  const uint32_t g = p.tile_base[r] + j / kMergeTile;
  const bool last_tile = g + 1 == p.tile_base[r + 1];
  uint32_t li;
  const uint8_t* ki = key_of(p, i, li);
  uint32_t pos = j;
  for (uint32_t s = 0; s < p.nruns; s++) {
    if (s == r) continue;
    const uint32_t lo = p.spl[(uint64_t)g * p.nruns + s];
    const uint32_t hi = last_tile ? p.run_first[s + 1] : p.spl[(uint64_t)(g + 1) * p.nruns + s];
    pos += rank_in(p, s, r, ki, li, lo, hi) - p.run_first[s];
  }
  p.dst[pos] = i;
}

__global__ void merge_keep_kernel(MergeParams p) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= p.n) return;
  MTri t{0, 0, 0};
  if (!*p.flags) {
    const uint32_t i = p.dst[q];
    uint32_t li;
    const uint8_t* ki = key_of(p, i, li);
    bool keep = true;
    if (q > 0) {  // bytes.Equal(key, curKey): the merged predecessor is the last candidate
      uint32_t lp;
      const uint8_t* kp = key_of(p, p.dst[q - 1], lp);
      if (lp == li) keep = bytes_compare(kp, lp, ki, li) != 0;
    }
    if (keep) t = MTri{1, li, (uint64_t)(p.ve[i] - (i ? p.ve[i - 1] : 0u))};
  }
  reinterpret_cast<MTri*>(p.tri)[q] = t;
}

// 8 lanes per merged position
__global__ void __launch_bounds__(256) merge_gather_kernel(MergeParams p) {
  constexpr uint32_t J = 8;
  const uint32_t lane = threadIdx.x & (J - 1);
  const uint32_t q = (blockIdx.x * blockDim.x + threadIdx.x) / J;
  if (q >= p.n || *p.flags) return;
  const MTri t = reinterpret_cast<const MTri*>(p.tri)[q];
  const MTri b = reinterpret_cast<const MTri*>(p.base)[q];
  if (q == p.n - 1 && lane == 0) {  // totals
    p.result[0] = b.n + t.n;
    p.result[1] = b.k + t.k;
    p.result[2] = b.v + t.v;
    if (b.n + t.n > p.ent_cap || (p.okd && b.k + t.k > p.key_cap) ||
        (p.ovd && b.v + t.v > p.val_cap) || b.k + t.k > 0xffffffffull || b.v + t.v > 0xffffffffull)
      atomicOr(p.flags + 1, M_CAPACITY);
  }
  if (!t.n) return;
  if (b.n >= p.ent_cap || (p.okd && b.k + t.k > p.key_cap) || (p.ovd && b.v + t.v > p.val_cap))
    return;
  const uint32_t i = p.dst[q];
  const uint32_t ks = i ? p.ke[i - 1] : 0u, vs = i ? p.ve[i - 1] : 0u;
  const uint32_t kl = (uint32_t)t.k, vl = (uint32_t)t.v;
  if (lane == 0) {
    if (p.oke) p.oke[b.n] = (uint32_t)(b.k + kl);
    if (p.ove) p.ove[b.n] = (uint32_t)(b.v + vl);
    if (p.osrc) p.osrc[b.n] = i;
  }
  const uint32_t kp = p.okd ? pieces16(kl) : 0u, np = kp + (p.ovd ? pieces16(vl) : 0u);
  for (uint32_t c = lane; c < np; c += J) {
    const bool key = c < kp;
    copy_piece16(key ? p.okd + b.k : p.ovd + b.v, key ? p.kd + ks : p.vd + vs, key ? kl : vl,
                 key ? c : c - kp);
  }
}

__global__ void merge_flags_kernel(MergeParams p) {
  if (threadIdx.x == 0) p.result[3] = (uint64_t)(p.flags[0] | p.flags[1]);
}

size_t merge_scan_bytes(uint32_t n) {
  size_t bytes = 0;
  (void)rocprim::exclusive_scan(nullptr, bytes, (const MTri*)nullptr, (MTri*)nullptr,
                                MTri{0, 0, 0}, (size_t)n, MTriPlus());
  return bytes;
}

hipError_t launch_merge(const MergeParams& p, void* scan_tmp, size_t scan_bytes, hipStream_t s) {
  hipError_t e;
  if ((e = hipMemsetAsync(p.flags, 0, 8, s)) != hipSuccess) return e;
  if (p.n) {
    const dim3 g((p.n + 255) / 256), g8((uint32_t)(((uint64_t)p.n * 8 + 255) / 256));
    hipLaunchKernelGGL(merge_check_kernel, g, dim3(256), 0, s, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(merge_tiles_kernel, dim3(1), dim3(64), 0, s, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const uint64_t tiles = p.n / kMergeTile + p.nruns;  // >= the tile count
    hipLaunchKernelGGL(merge_split_kernel, dim3((uint32_t)((tiles * p.nruns + 255) / 256)),
                       dim3(256), 0, s, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(merge_rank_kernel, g, dim3(256), 0, s, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(merge_keep_kernel, g, dim3(256), 0, s, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    size_t bytes = scan_bytes;
    e = rocprim::exclusive_scan(scan_tmp, bytes, reinterpret_cast<const MTri*>(p.tri),
                                reinterpret_cast<MTri*>(p.base), MTri{0, 0, 0}, (size_t)p.n,
                                MTriPlus(), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(merge_gather_kernel, g8, dim3(256), 0, s, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  hipLaunchKernelGGL(merge_flags_kernel, dim3(1), dim3(64), 0, s, p);
  return hipGetLastError();
}

}  // namespace lsmgpu
