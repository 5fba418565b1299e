// decode_wsc.hip -- "walk, scan, copy" SST block decode for LARGE or irregular blocks
// (BASELINE C5: Zipf 16-264 B keys in 32 KiB blocks; 100-entry blocks of C1/C4).
//
// The speculative in-LDS walk of decode.hip confirms a whole run of equal-size entries per
// round; with Zipf key lengths every entry has its own size, so it degenerates to one entry
// per round and one 32 KiB block per wave (LDS).  Here the serial header chain is walked by
// ONE LANE PER BLOCK straight from global memory -- 64 blocks per wave, thousands of blocks in
// flight, each hop one dependent 8-B load -- and the bytes are then moved by a separate,
// fully parallel copy with known output bases:
//   K1 walk_kernel : lane b walks block b exactly like blockIterator.Next/parseKV
//                    (table/iterator.go:93-135), writing per entry {pos | plen << 16,
//                    key offset | value offset << 16} into the block's metadata region and
//                    {entries, key bytes, value bytes} + status per block
//   scan           : rocPRIM exclusive scan of the per-block triples (device-wide)
//   K2 copy_kernel : one wave per block; lane groups copy each entry's key and value as
//                    unaligned 16-B pieces (the last overlapping back inside the entry, so
//                    no store leaves it) global -> global, plus end offsets / view records
// Traffic: the input is read twice (walk touches every line; copy reads the bytes) -- the
// price of taking the serial walk off the critical path.  Blocks must be < 64 KiB.
#include <rocprim/device/device_scan.hpp>

#include "codec_common.hpp"
#include "kernels.hpp"

namespace lsmgpu {

namespace {

// big-endian u16 fields of the 10-B header at g (table/builder.go:23-45), unaligned global read
__device__ __forceinline__ void read_hdr(const uint8_t* g, uint32_t& plen, uint32_t& klen,
                                         uint32_t& vlen) {
  uint2 w;
  __builtin_memcpy(&w, g, 8);  // one unaligned global_load_dwordx2
  plen = __builtin_amdgcn_perm(0u, w.x, 0x0c0c0001u);
  klen = __builtin_amdgcn_perm(0u, w.x, 0x0c0c0203u);
  vlen = __builtin_amdgcn_perm(0u, w.y, 0x0c0c0001u);
}

}  // namespace

// K1: lane = block.
__global__ void __launch_bounds__(256) wsc_walk_kernel(DecodeParams p) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= p.nblk) return;
  const uint32_t off = p.blk_off[b], len = p.blk_len[b];
  uint32_t n = 0, K = 0, V = 0, st = LSMGPU_BLK_OK;
  if ((uint64_t)off + len > p.data_len) {
    st = LSMGPU_BLK_RANGE;
  } else {
    const uint8_t* blk = p.data + off;
    uint32_t* meta = p.wmeta + 2ull * p.wcap * b;
    uint32_t pos = 0, base_pos = 0;
    bool have_base = false;
    for (;;) {
      if (pos >= len) break;                                   // iterator.go:115-118
      if (len - pos < 10) { st = LSMGPU_BLK_TRUNC_HEADER; break; }
      uint32_t plen, klen, vlen;
      read_hdr(blk + pos, plen, klen, vlen);
      const uint32_t hp = pos;
      pos += 10;                                               // iterator.go:121
      if ((klen | plen) == 0) break;                           // iterator.go:124-127
      if (!have_base) {                                        // iterator.go:129-133
        if (plen != 0) { st = LSMGPU_BLK_FIRST_PLEN; break; }
        base_pos = pos;
        have_base = true;
      }
      if (base_pos + plen > len) { st = LSMGPU_BLK_PREFIX_OOB; break; }
      pos += klen;                                             // iterator.go:101
      if (pos + vlen > len) { st = LSMGPU_BLK_VALUE_OVERFLOW; break; }  // iterator.go:103
      pos += vlen;                                             // iterator.go:109
      if (n < p.wcap && !(p.ablate & 32)) {  // (ablation 32: timing without the metadata)
        meta[2 * n] = hp | (plen << 16);
        meta[2 * n + 1] = K | (V << 16);                       // exclusive offsets (< 64 KiB)
      }
      K += plen + klen;
      V += vlen;
      n++;
    }
  }
  uint64_t* t = p.wstat + 3ull * b;
  t[0] = n;
  t[1] = K;
  t[2] = V;
  p.wstatus[b] = st;
}

// Copy `len` bytes from src to dst (both global, any alignment) with the J lanes of a group:
// lane j writes pieces j, j + J, ...; 16-B pieces, the last overlapping back inside the range,
// or two overlapping 8/4-B pieces below 16 B, bytes below 4 B.
__device__ __forceinline__ void group_copy(uint8_t* dst, const uint8_t* src, uint32_t len,
                                           uint32_t j, uint32_t J) {
  if (len >= 16) {
    const uint32_t np = (len + 15) >> 4;
    for (uint32_t q = j; q < np; q += J) {
      const uint32_t o = min(16 * q, len - 16);
      uint4 v;
      __builtin_memcpy(&v, src + o, 16);
      __builtin_memcpy(dst + o, &v, 16);
    }
  } else if (len >= 8) {
    if (j < 2) {
      const uint32_t o = j ? len - 8 : 0;
      uint2 v;
      __builtin_memcpy(&v, src + o, 8);
      __builtin_memcpy(dst + o, &v, 8);
    }
  } else if (len >= 4) {
    if (j < 2) {
      const uint32_t o = j ? len - 4 : 0;
      uint32_t v;
      __builtin_memcpy(&v, src + o, 4);
      __builtin_memcpy(dst + o, &v, 4);
    }
  } else if (j < len) {
    dst[j] = src[j];
  }
}

// Pieces of a stream of `len` bytes (see group_copy) and piece q of it.
__device__ __forceinline__ uint32_t n_pieces16(uint32_t len) {
  return len >= 16 ? (len + 15) >> 4 : (len >= 4 ? 2u : len);
}
__device__ __forceinline__ void piece_copy(uint8_t* dst, const uint8_t* src, uint32_t len,
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

// K2: one wave per block, J = 8 lanes per entry.
__global__ void __launch_bounds__(256) wsc_copy_kernel(DecodeParams p) {
  const uint32_t lane = lane_id();
  const uint32_t b = uniform(blockIdx.x * (blockDim.x / kWave) + (threadIdx.x >> 6));
  if (b >= p.nblk) return;
  const uint64_t* t = p.wstat + 3ull * b;
  const uint32_t n = uniform((uint32_t)t[0]), K = uniform((uint32_t)t[1]),
                 V = uniform((uint32_t)t[2]);
  const uint32_t st = uniform(p.wstatus[b]);
  const uint64_t* bs = p.wbase + 3ull * b;
  const uint64_t en = uniform64(bs[0]), ek = uniform64(bs[1]), ev = uniform64(bs[2]);
  const uint32_t off = uniform(p.blk_off[b]);
  if (lane == 0) {
    if (p.blk_first) p.blk_first[b] = (uint32_t)en;
    if (p.blk_status) p.blk_status[b] = (int32_t)st;
    if (st != LSMGPU_BLK_OK) {
      atomicAdd(reinterpret_cast<unsigned long long*>(p.result + 4), 1ull);
      atomicMax(reinterpret_cast<unsigned long long*>(p.result + 3),
                (unsigned long long)(p.nblk - b));
    }
    if (b == p.nblk - 1) {  // totals of the whole batch
      if (p.blk_first) p.blk_first[p.nblk] = (uint32_t)(en + n);
      p.result[0] = en + n;
      p.result[1] = ek + K;
      p.result[2] = ev + V;
    }
  }
  const bool mat = (p.mode & LSMGPU_MODE_MATERIALIZE) != 0;
  const bool view = (p.mode & LSMGPU_MODE_VIEW) != 0 && p.view;
  bool ok = en + n <= p.ent_cap && en + n <= 0xffffffffull;
  if (mat) {
    const uint64_t kend = ek + K, vend = ev + V;
    ok = ok && (kend <= p.key_cap || !p.key_data) && (vend <= p.val_cap || !p.val_data);
    ok = ok && kend < 0xffffffffull && vend <= 0xffffffffull;
  }
  if (!ok) {
    if (lane == 0) atomicOr(reinterpret_cast<unsigned long long*>(p.result + 5), 1ull);
    return;
  }
  if (n == 0 || (p.ablate & 2)) return;
  const uint8_t* blk = p.data + off;
  const uint32_t* meta = p.wmeta + 2ull * p.wcap * b;
  uint8_t* kbase = p.key_data ? p.key_data + ek : nullptr;
  uint8_t* vbase = p.val_data ? p.val_data + ev : nullptr;
  // J = 8 lanes per entry; an entry's pieces are [key pieces | value pieces] (16 B, the last
  // overlapping back inside its stream, or two overlapping 8/4/2/1-B pieces below 16 B) and
  // lane j takes pieces j, j + 8, ...  Four entry groups per pass, all loads issued first.
  constexpr uint32_t J = 8, G = 4;
  const uint32_t j = lane & (J - 1);
  bool any_plen = false;
  for (uint32_t e0 = 0; e0 < n; e0 += G * (kWave / J)) {
    uint32_t hp[G], kl[G], vl[G], ko[G], vo[G], np[G], kp[G];
    bool on[G];
#pragma unroll
    for (int i = 0; i < G; i++) {
      const uint32_t e = e0 + i * (kWave / J) + (lane >> 3);
      const uint32_t ec = min(e, n - 1);
      const uint32_t a0 = meta[2 * ec], a1 = meta[2 * ec + 1];
      const uint32_t b1 = ec + 1 < n ? meta[2 * ec + 3] : (K | (V << 16));
      const uint32_t plen = a0 >> 16;
      hp[i] = a0 & 0xffffu;
      ko[i] = a1 & 0xffffu;
      vo[i] = a1 >> 16;
      const uint32_t ko1 = b1 & 0xffffu, vo1 = b1 >> 16;
      kl[i] = ko1 - ko[i] - plen;  // stored key bytes
      vl[i] = vo1 - vo[i];
      on[i] = e < n;
      any_plen = any_plen || (on[i] && plen != 0);
      kp[i] = plen ? 0u : n_pieces16(kl[i]);  // prefix-compressed keys: bytewise pass below
      np[i] = kp[i] + n_pieces16(vl[i]);
      if (on[i] && j == 0) {
        if (mat) {
          if (p.key_end) p.key_end[en + e] = (uint32_t)(ek + ko1);
          if (p.val_end) p.val_end[en + e] = (uint32_t)(ev + vo1);
        }
        if (view)
          p.view[en + e] = (uint64_t)(off + hp[i] + 10) | ((uint64_t)kl[i] << 32) |
                           ((uint64_t)vl[i] << 48);
      }
    }
    if (!mat) continue;
#pragma unroll
    for (int i = 0; i < G; i++) {
      if (!on[i]) continue;
      for (uint32_t q = j; q < np[i]; q += J) {
        const bool key = q < kp[i];
        const uint32_t len = key ? kl[i] : vl[i];
        uint8_t* dst = key ? kbase : vbase;
        if (!dst) continue;
        const uint32_t s0 = key ? hp[i] + 10 : hp[i] + 10 + kl[i];
        piece_copy(dst + (key ? ko[i] : vo[i]), blk + s0, len, key ? q : q - kp[i]);
      }
    }
  }
  if (any_plen && kbase && mat) {  // baseKey[:plen] ++ diff (iterator.go:98-100): bytewise
    for (uint32_t e = lane >> 3; e < n; e += kWave / J) {
      const uint32_t a0 = meta[2 * e], a1 = meta[2 * e + 1];
      const uint32_t plen = a0 >> 16;
      if (plen == 0) continue;
      const uint32_t hp = a0 & 0xffffu, ko = a1 & 0xffffu;
      const uint32_t ko1 = e + 1 < n ? (meta[2 * e + 3] & 0xffffu) : K;
      const uint32_t kl = ko1 - ko;
      for (uint32_t i = j; i < kl; i += J)
        kbase[ko + i] = i < plen ? blk[10 + i] : blk[hp + 10 + i - plen];
    }
  }
}

namespace {
struct Tri64 {
  uint64_t n, k, v;
};
struct Tri64Plus {
  __device__ __host__ Tri64 operator()(const Tri64& a, const Tri64& b) const {
    return Tri64{a.n + b.n, a.k + b.k, a.v + b.v};
  }
};
}  // namespace

size_t wsc_scan_bytes(uint32_t nblk) {
  size_t bytes = 0;
  (void)rocprim::exclusive_scan(nullptr, bytes, (const Tri64*)nullptr, (Tri64*)nullptr,
                                Tri64{0, 0, 0}, (size_t)nblk, Tri64Plus());
  return bytes;
}

hipError_t launch_decode_wsc(const DecodeParams& p, void* scan_tmp, size_t scan_bytes,
                             hipStream_t s) {
  const uint32_t nblk = p.nblk;
  hipLaunchKernelGGL(wsc_walk_kernel, dim3((nblk + 255) / 256), dim3(256), 0, s, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  size_t bytes = scan_bytes;
  e = rocprim::exclusive_scan(scan_tmp, bytes, reinterpret_cast<const Tri64*>(p.wstat),
                              reinterpret_cast<Tri64*>(p.wbase), Tri64{0, 0, 0}, (size_t)nblk,
                              Tri64Plus(), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(wsc_copy_kernel, dim3((nblk + 3) / 4), dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace lsmgpu
