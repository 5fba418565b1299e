// codec_common.hpp -- device helpers shared by the CDNA4 (gfx950) SST block decode/encode
// kernels.  Wave64-only code: every "wave" idiom here assumes 64 lanes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lsmgpu.h"

namespace lsmgpu {

constexpr int kWave = 64;

// ---------------------------------------------------------------- wave primitives
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint32_t uniform(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
  uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
  return ((uint64_t)hi << 32) | lo;
}
// Orders this wave's LDS accesses for the compiler (the hardware already runs one wave's
// DS instructions in order).
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    uint32_t lo = __shfl_xor((uint32_t)v, o);
    uint32_t hi = __shfl_xor((uint32_t)(v >> 32), o);
    v += ((uint64_t)hi << 32) | lo;
  }
  return v;
}

// ---------------------------------------------------------------- agent-scope granules
// Prefix state: 8-byte {tag:32 | value:32} granules written by ONE atomic (sc1) store and
// read by relaxed agent-scope loads (MI355X_MICROARCH: R2 granule hand-off).  Values are
// u32 with saturating adds (a key stream past 4 GiB - 1 saturates and fails the capacity
// check; entries and value bytes are bounded by the <= 4 GiB - 1 input).
constexpr int kTagShift = 32;
constexpr uint64_t kValMask = 0xffffffffull;
__device__ __forceinline__ uint32_t sat_add(uint32_t a, uint32_t b) {
  const uint32_t s = a + b;
  return s < a ? 0xffffffffu : s;
}
__device__ __forceinline__ uint64_t gload(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gstore(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------- byte helpers
__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
// 4 bytes starting at byte p of an LDS buffer (any alignment): 2 aligned dword reads.
__device__ __forceinline__ uint32_t lds_u32(const uint8_t* lds, uint32_t p) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(lds + (p & ~3u));
  return __builtin_amdgcn_alignbyte(w[1], w[0], p & 3u);
}
// 16 bytes starting at byte p of an LDS buffer (any alignment): 5 aligned dword reads.
__device__ __forceinline__ uint4 lds_u128(const uint8_t* lds, uint32_t p) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(lds + (p & ~3u));
  uint32_t r = p & 3u;
  uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
  uint4 o;
  o.x = __builtin_amdgcn_alignbyte(w1, w0, r);
  o.y = __builtin_amdgcn_alignbyte(w2, w1, r);
  o.z = __builtin_amdgcn_alignbyte(w3, w2, r);
  o.w = __builtin_amdgcn_alignbyte(w4, w3, r);
  return o;
}
__device__ __forceinline__ void set_byte(uint4& v, int i, uint32_t b) {
  uint32_t sh = (uint32_t)(i & 3) * 8;
  uint32_t m = ~(0xffu << sh);
  switch (i >> 2) {
    case 0: v.x = (v.x & m) | (b << sh); break;
    case 1: v.y = (v.y & m) | (b << sh); break;
    case 2: v.z = (v.z & m) | (b << sh); break;
    default: v.w = (v.w & m) | (b << sh); break;
  }
}

// bytes.Compare on global memory, 8-B big-endian words at a time (unaligned loads); the tail
// bytewise.  Returns -1 / 0 / 1.
__device__ __forceinline__ int bytes_compare(const uint8_t* a, uint32_t la, const uint8_t* b,
                                             uint32_t lb) {
  const uint32_t n = la < lb ? la : lb;
  uint32_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t x, y;
    __builtin_memcpy(&x, a + i, 8);
    __builtin_memcpy(&y, b + i, 8);
    if (x != y) return __builtin_bswap64(x) < __builtin_bswap64(y) ? -1 : 1;
  }
  for (; i < n; i++)
    if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  return la == lb ? 0 : (la < lb ? -1 : 1);
}
// y.CompareKeys (y/y.go:84-90) for keys longer than 8 B: the user key, then the 8-B suffix
__device__ __forceinline__ int compare_keys(const uint8_t* a, uint32_t la, const uint8_t* b,
                                            uint32_t lb) {
  const int c = bytes_compare(a, la - 8, b, lb - 8);
  return c ? c : bytes_compare(a + la - 8, 8, b + lb - 8, 8);
}

// Range-checked buffer accesses (raw buffer loads / stores over a resource of `bytes` bytes at a
// wave-uniform base): an offset at or past the end reads zeros and drops the store without a
// memory access, so every lane can issue the instruction and none needs a branch around it.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
constexpr uint32_t kNoStore = 0xfffffff0u;  // an offset past any resource (resources are < 4 GiB - 16)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buffer_rsrc(const void* base, uint64_t bytes) {
  // word 3: gfx9 32-bit data format, the range check on raw offsets
  return __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(uniform64(reinterpret_cast<uint64_t>(base))), 0,
      (int)(uint32_t)(bytes < kNoStore ? bytes : kNoStore), 0x00020000);
}

// A stream of `len` bytes copied global -> global (any alignment) as independent pieces:
// 16-B pieces, the last one overlapping back inside the stream; below 16 B two overlapping
// 8-B or 4-B pieces; below 4 B single bytes.  No piece touches a byte outside the stream, so
// neighbouring streams can be written concurrently.  pieces16 = the piece count, copy_piece16
// copies piece q.
__device__ __forceinline__ uint32_t pieces16(uint32_t len) {
  return len >= 16 ? (len + 15) >> 4 : (len >= 4 ? 2u : len);
}
__device__ __forceinline__ void copy_piece16(uint8_t* dst, const uint8_t* src, uint32_t len,
                                          uint32_t q) {
  if (len >= 16) {
    const uint32_t o = min(16 * q, len - 16);
    uint4 v;
    __builtin_memcpy(&v, src + o, 16);
    __builtin_memcpy(dst + o, &v, 16);
  } else if (len >= 8) {
    const uint32_t o = q ? len - 8 : 0;
    uint2 v;
    __builtin_memcpy(&v, src + o, 8);
    __builtin_memcpy(dst + o, &v, 8);
  } else if (len >= 4) {
    const uint32_t o = q ? len - 4 : 0;
    uint32_t v;
    __builtin_memcpy(&v, src + o, 4);
    __builtin_memcpy(dst + o, &v, 4);
  } else {
    dst[q] = src[q];
  }
}


// Copies [src, src+n) of global memory (any alignment, n = multiple-of-16 region base given)
// into LDS as 16-B chunks: lds[16c .. 16c+16) = global[a0+16c ..], a0 = src & ~15.
// Bytes past `limit` (end of the readable global buffer) are never read (zero-filled).
// Returns the byte shift (src - a0) of src inside LDS.
__device__ __forceinline__ uint32_t stage_to_lds(uint8_t* lds, const uint8_t* base, uint64_t src,
                                                 uint32_t n, uint64_t limit, uint32_t lane) {
  uint64_t a0 = src & ~15ull;
  uint32_t sh = (uint32_t)(src - a0);
  uint32_t nchunk = (sh + n + 15) >> 4;
  for (uint32_t c = lane; c < nchunk; c += kWave) {
    uint64_t a = a0 + 16ull * c;
    uint4 v;
    if (a + 16 <= limit) {
      v = *reinterpret_cast<const uint4*>(base + a);
    } else {
      v = make_uint4(0, 0, 0, 0);
      for (int i = 0; i < 16; i++)
        if (a + i < limit) set_byte(v, i, base[a + i]);
    }
    *reinterpret_cast<uint4*>(lds + 16 * c) = v;
  }
  return sh;
}

// Largest e in [0, n-1] with o(e) <= t, where o is a non-decreasing u16 column of the
// per-entry metadata (stride 4 u16s).  Requires n >= 1 and o(0) <= t.
__device__ __forceinline__ uint32_t meta_search(const uint16_t* col, uint32_t n, uint32_t t) {
  uint32_t lo = 0, hi = n - 1;
  while (lo < hi) {
    uint32_t mid = (lo + hi + 1) >> 1;
    if (col[4 * mid] <= t) lo = mid; else hi = mid - 1;
  }
  return lo;
}

}  // namespace lsmgpu
