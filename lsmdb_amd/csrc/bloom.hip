// bloom.hip -- the SST bloom tail on the device: Builder.Finish's filter build and JSON, and
// batched Table.DoesNotHave probes (table/builder.go:164-195, table/table.go:180-186,301).
// The reference uses github.com/AndreasBriese/bbloom v0.0.0-20190825152654-46b345b51c96 (not
// vendored); its algorithm is restated in oracle/bbloom.c (the checker) and DESIGN.md:
// SipHash-2-4 keyed (0xdeadbeaf, 0xfaebdaed), h = hash >> shift, l = hash << shift >> shift,
// bit (h + i * l) & (bits - 1) for i < setLocs, bit idx = bit idx % 64 of little-endian u64
// word idx / 64, JSON {"FilterSet":"<base64 std>","SetLocs":N}.
//
// One thread per key: the hash is ~8 SipRounds of 64-bit ALU work on 1-2 message words, then
// setLocs (7) scattered 64-bit atomic ORs into the filter (C4: 519,540 keys into a 1 MiB filter).
#include "codec_common.hpp"
#include "kernels.hpp"

namespace lsmgpu {

namespace {

__device__ __forceinline__ uint64_t rotl64(uint64_t x, int b) { return (x << b) | (x >> (64 - b)); }

#define LSMGPU_SIPROUND                                                   \
  do {                                                                    \
    v0 += v1; v1 = rotl64(v1, 13); v1 ^= v0; v0 = rotl64(v0, 32);         \
    v2 += v3; v3 = rotl64(v3, 16); v3 ^= v2;                              \
    v0 += v3; v3 = rotl64(v3, 21); v3 ^= v0;                              \
    v2 += v1; v1 = rotl64(v1, 17); v1 ^= v2; v2 = rotl64(v2, 32);         \
  } while (0)

// bbloom's sipHash over key [p, p + n); `limit` = first byte past the readable buffer (the
// last word is read as one unaligned 8-B load when it stays below limit)
__device__ __forceinline__ uint64_t bbloom_sip(const uint8_t* p, uint32_t n, const uint8_t* limit) {
  uint64_t v0 = 8317987320269560794ull, v1 = 7237128889637516672ull;
  uint64_t v2 = 7816392314733513934ull, v3 = 8387220255325274014ull;
  uint32_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t m;
    __builtin_memcpy(&m, p + i, 8);  // little-endian word (binary.LittleEndian order)
    v3 ^= m;
    LSMGPU_SIPROUND;
    LSMGPU_SIPROUND;
    v0 ^= m;
  }
  uint64_t t = (uint64_t)n << 56;
  const uint32_t r = n - i;
  if (r) {
    uint64_t w = 0;
    if (p + i + 8 <= limit) {
      __builtin_memcpy(&w, p + i, 8);
    } else {
      for (uint32_t k = 0; k < r; k++) w |= (uint64_t)p[i + k] << (8 * k);
    }
    t |= w & ((1ull << (8 * r)) - 1);
  }
  v3 ^= t;
  LSMGPU_SIPROUND;
  LSMGPU_SIPROUND;
  v0 ^= t;
  v2 ^= 0xff;
  LSMGPU_SIPROUND;
  LSMGPU_SIPROUND;
  LSMGPU_SIPROUND;
  LSMGPU_SIPROUND;
  return v0 ^ v1 ^ v2 ^ v3;
}

// Builder.Finish: key i (with its 8-B ts) adds ParseKey(key) = key[:len - 8]
__global__ void __launch_bounds__(256) bloom_build_kernel(BloomParams p) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= p.n) return;
  const uint32_t s = i ? p.key_end[i - 1] : (p.key_base ? *p.key_base : 0u), e = p.key_end[i];
  if (e - s <= 8 || e < s) {  // y.go:98 AssertTruef(len(key) > 8): a panic in Go
    atomicOr(p.flags, 1u);
    return;
  }
  const uint8_t* k = p.keys + s;
  // the key's last word is followed by its 8-B ts: a whole 8-B read never leaves key i
  const uint64_t hash = bbloom_sip(k, e - s - 8, k + (e - s));
  // equal hashes set equal bits: a lane whose hash equals the wave's first active lane's
  // leaves the bits to that lane (keys sharing ParseKey(key) -- e.g. 16-B keys without a ts,
  // whose first 8 B repeat -- would otherwise serialize on the same words' atomics)
  const uint32_t lo = (uint32_t)hash, hi = (uint32_t)(hash >> 32);
  const bool same = __builtin_amdgcn_readfirstlane(lo) == lo && __builtin_amdgcn_readfirstlane(hi) == hi;
  if (same && __lane_id() != (uint32_t)__builtin_ctzll(__ballot(1))) return;
  const uint64_t h = hash >> p.shift, l = (hash << p.shift) >> p.shift;
  unsigned long long* w = reinterpret_cast<unsigned long long*>(p.bitset);
  for (uint64_t j = 0; j < p.locs; j++) {
    const uint64_t idx = (h + j * l) & p.mask;
    const unsigned long long bit = 1ull << (idx & 63);
    // a bit another key already set needs no atomic (a stale read only costs the atomic)
    if (!(__hip_atomic_load(w + (idx >> 6), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit))
      atomicOr(w + (idx >> 6), bit);
  }
}

// Table.DoesNotHave batch: has[i] = bf.Has(key i); keys as given (level_handler.go:221-224
// passes ParseKey(key))
__global__ void __launch_bounds__(256) bloom_has_kernel(BloomParams p) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= p.n) return;
  const uint32_t s = i ? p.key_end[i - 1] : 0, e = p.key_end[i];
  const uint8_t* k = p.keys + s;
  const uint64_t hash = bbloom_sip(k, e - s, p.keys + p.key_end[p.n - 1]);
  const uint64_t h = hash >> p.shift, l = (hash << p.shift) >> p.shift;
  uint32_t res = 1;
  for (uint64_t j = 0; j < p.locs && res; j++) {
    const uint64_t idx = (h + j * l) & p.mask;
    res = (uint32_t)(p.bitset[idx >> 6] >> (idx & 63)) & 1u;
  }
  p.has[i] = (uint8_t)res;
}

// JSONMarshal: base64 (std alphabet, '=' padding) of the filter's bytes between the fixed head
// and the "SetLocs" tail.  Thread g < groups writes the 4 characters of bytes [3g, 3g + 3).
__global__ void __launch_bounds__(256) bloom_json_kernel(BloomJson p) {
  const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t groups = (p.nbytes + 2) / 3;
  const uint8_t* s = reinterpret_cast<const uint8_t*>(p.bitset);
  if (g < groups) {
    const uint64_t i = 3 * g;
    const uint32_t a = s[i], b = i + 1 < p.nbytes ? s[i + 1] : 0u, c = i + 2 < p.nbytes ? s[i + 2] : 0u;
    const uint32_t w = (a << 16) | (b << 8) | c;
    auto enc = [](uint32_t x) -> uint8_t {
      return (uint8_t)(x < 26 ? 'A' + x : x < 52 ? 'a' + (x - 26) : x < 62 ? '0' + (x - 52) : x == 62 ? '+' : '/');
    };
    uint8_t* o = p.out + p.head_len + 4 * g;
    o[0] = enc((w >> 18) & 63);
    o[1] = enc((w >> 12) & 63);
    o[2] = i + 1 < p.nbytes ? enc((w >> 6) & 63) : (uint8_t)'=';
    o[3] = i + 2 < p.nbytes ? enc(w & 63) : (uint8_t)'=';
  } else if (g < groups + p.head_len + p.tail_len) {
    const uint32_t k = (uint32_t)(g - groups);
    if (k < p.head_len) p.out[k] = p.text[k];
    else p.out[p.head_len + 4 * groups + (k - p.head_len)] = p.text[k];
  }
}

// ---- many tables at once (compaction: Finish for every output table)
__device__ __forceinline__ uint32_t seg_of_key(const BloomTables& p, uint32_t i) {
  uint32_t lo = 0, hi = p.nseg - 1;  // largest t with seg[t].first <= i
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (p.seg[mid].first <= i) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__global__ void __launch_bounds__(256) bloom_tables_build_kernel(BloomTables p) {
  const uint64_t gi = (uint64_t)blockIdx.x * 256 + threadIdx.x + p.seg[0].first;
  if (gi >= p.end) return;
  const uint32_t i = (uint32_t)gi;
  const BloomSeg& sg = p.seg[seg_of_key(p, i)];
  const uint32_t ki = p.src ? p.src[i] : i;  // gather mode: the merged entry's source key
  const uint32_t s = ki ? p.key_end[ki - 1] : 0u, e = p.key_end[ki];
  if (e - s <= 8 || e < s) {  // y.go:98 AssertTruef(len(key) > 8)
    atomicOr(p.flags, 1u);
    return;
  }
  const uint8_t* k = p.keys + s;
  const uint64_t hash = bbloom_sip(k, e - s - 8, k + (e - s));
  const uint32_t lo32 = (uint32_t)hash, hi32 = (uint32_t)(hash >> 32);
  const uint64_t wo = sg.word_off;
  // lanes repeating the first active lane's hash in the same table leave the bits to it
  const bool same = __builtin_amdgcn_readfirstlane(lo32) == lo32 &&
                    __builtin_amdgcn_readfirstlane(hi32) == hi32 &&
                    __builtin_amdgcn_readfirstlane((uint32_t)wo) == (uint32_t)wo;
  if (same && __lane_id() != (uint32_t)__builtin_ctzll(__ballot(1))) return;
  const uint64_t h = hash >> sg.shift, l = (hash << sg.shift) >> sg.shift;
  unsigned long long* w = reinterpret_cast<unsigned long long*>(p.scratch + wo);
  for (uint32_t j = 0; j < sg.locs; j++) {
    const uint64_t idx = (h + (uint64_t)j * l) & sg.mask;
    const unsigned long long bit = 1ull << (idx & 63);
    if (!(__hip_atomic_load(w + (idx >> 6), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit))
      atomicOr(w + (idx >> 6), bit);
  }
}

// thread g < groups: 4 base64 characters of its table; then 64 threads per table write the
// head / tail text bytes
__global__ void __launch_bounds__(256) bloom_tables_json_kernel(BloomTables p, uint64_t groups) {
  const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  static constexpr char kHead[] = "{\"FilterSet\":\"";
  if (g < groups) {
    uint32_t lo = 0, hi = p.nseg - 1;
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (p.seg[mid].group_off <= g) lo = mid; else hi = mid - 1;
    }
    const BloomSeg& sg = p.seg[lo];
    const uint64_t gl = g - sg.group_off, nbytes = (sg.mask + 1) / 8, i = 3 * gl;
    const uint8_t* src = reinterpret_cast<const uint8_t*>(p.scratch + sg.word_off);
    const uint32_t a = src[i], b = i + 1 < nbytes ? src[i + 1] : 0u, c = i + 2 < nbytes ? src[i + 2] : 0u;
    const uint32_t w = (a << 16) | (b << 8) | c;
    auto enc = [](uint32_t x) -> uint8_t {
      return (uint8_t)(x < 26 ? 'A' + x : x < 52 ? 'a' + (x - 26) : x < 62 ? '0' + (x - 52) : x == 62 ? '+' : '/');
    };
    uint8_t* o = p.out + sg.json_out + 14 + 4 * gl;
    o[0] = enc((w >> 18) & 63);
    o[1] = enc((w >> 12) & 63);
    o[2] = i + 1 < nbytes ? enc((w >> 6) & 63) : (uint8_t)'=';
    o[3] = i + 2 < nbytes ? enc(w & 63) : (uint8_t)'=';
  } else if (g < groups + 64ull * p.nseg) {
    const uint32_t t = (uint32_t)((g - groups) >> 6), k = (uint32_t)((g - groups) & 63);
    const BloomSeg& sg = p.seg[t];
    const uint64_t nb64 = 4 * (((sg.mask + 1) / 8 + 2) / 3);
    if (k < 14) p.out[sg.json_out + k] = (uint8_t)kHead[k];
    else if (k - 14 < sg.tail_len) p.out[sg.json_out + 14 + nb64 + (k - 14)] = sg.tail[k - 14];
  }
}

}  // namespace

hipError_t launch_bloom_tables(const BloomTables& p, uint64_t groups, hipStream_t s) {
  if (p.nseg == 0) return hipSuccess;
  const uint64_t keys = p.end - p.seg[0].first;
  if (keys) {
    hipLaunchKernelGGL(bloom_tables_build_kernel, dim3((unsigned)((keys + 255) / 256)), dim3(256),
                       0, s, p);
  }
  const uint64_t threads = groups + 64ull * p.nseg;
  hipLaunchKernelGGL(bloom_tables_json_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256),
                     0, s, p, groups);
  return hipGetLastError();
}

hipError_t launch_bloom_build(const BloomParams& p, hipStream_t s) {
  if (p.n == 0) return hipSuccess;
  hipLaunchKernelGGL(bloom_build_kernel, dim3((unsigned)((p.n + 255) / 256)), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_bloom_has(const BloomParams& p, hipStream_t s) {
  if (p.n == 0) return hipSuccess;
  hipLaunchKernelGGL(bloom_has_kernel, dim3((unsigned)((p.n + 255) / 256)), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_bloom_json(const BloomJson& p, hipStream_t s) {
  const uint64_t threads = (p.nbytes + 2) / 3 + p.head_len + p.tail_len;
  hipLaunchKernelGGL(bloom_json_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace lsmgpu
