// decode_common.hpp -- pieces shared by the gfx950 decode kernels (decode.hip: the persistent
// LDS-lag / register-lag kernels; decode_wsc.hip: walk-scan-copy and the fused tile kernel):
// the header readers and serial walk (table/iterator.go:93-135), the epoch-tagged prefix
// granules with their decoupled look-back, and the LDS-DMA block stager.
#pragma once
#include "codec_common.hpp"
#include "kernels.hpp"

namespace lsmgpu {

struct Hdr {
  uint32_t plen, klen, vlen;
};

// ---- header readers (the 10-B BE header of table/builder.go:23-45; prev is unused here)
struct LdsSrc {
  const uint8_t* slot;  // 16-B aligned LDS slot (block byte 0 at slot + sh)
  uint32_t sh;
  __device__ __forceinline__ Hdr hdr(uint32_t pos) const {
    // three ALIGNED dword reads + v_alignbyte: a misaligned ds_read_b64/b128 costs ~10x the
    // LDS cycles of an aligned one on gfx950 (scripts/lds_probe.hip)
    const uint32_t p = sh + pos;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(slot + (p & ~3u));
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
    const uint32_t x0 = __builtin_amdgcn_alignbyte(w1, w0, p & 3u);  // plen:klen (BE)
    const uint32_t x1 = __builtin_amdgcn_alignbyte(w2, w1, p & 3u);  // vlen:..   (BE)
    // v_perm byte selects: BE u16 -> u32
    return Hdr{__builtin_amdgcn_perm(0u, x0, 0x0c0c0001u), __builtin_amdgcn_perm(0u, x0, 0x0c0c0203u),
               __builtin_amdgcn_perm(0u, x1, 0x0c0c0001u)};
  }
};
struct GlobalSrc {
  const uint8_t* blk;  // global pointer to block byte 0
  __device__ __forceinline__ Hdr hdr(uint32_t pos) const {
    const uint8_t* h = blk + pos;
    return Hdr{((uint32_t)h[0] << 8) | h[1], ((uint32_t)h[2] << 8) | h[3],
               ((uint32_t)h[4] << 8) | h[5]};
  }
};

struct WalkResult {
  uint32_t n, K, V, status;
};

// The blockIterator forward walk, serial (count only: oversize blocks from global memory,
// blocks with more entries than the metadata holds from LDS).  Values identical in every lane.
template <class Src>
__device__ __forceinline__ WalkResult walk_block(const Src& src, uint32_t len) {
  uint32_t pos = 0, n = 0, K = 0, V = 0, st = LSMGPU_BLK_OK, base_pos = 0;
  bool have_base = false;
  for (;;) {
    if (pos >= len) break;                                   // iterator.go:115-118
    if (len - pos < 10) { st = LSMGPU_BLK_TRUNC_HEADER; break; }
    Hdr h = src.hdr(pos);
    pos += 10;                                               // iterator.go:121
    if ((h.klen | h.plen) == 0) break;                       // iterator.go:124-127
    if (!have_base) {                                        // iterator.go:129-133
      if (h.plen != 0) { st = LSMGPU_BLK_FIRST_PLEN; break; }
      base_pos = pos;
      have_base = true;
    }
    if (base_pos + h.plen > len) { st = LSMGPU_BLK_PREFIX_OOB; break; }
    pos += h.klen;                                           // iterator.go:101
    if (pos + h.vlen > len) { st = LSMGPU_BLK_VALUE_OVERFLOW; break; }  // iterator.go:103
    pos += h.vlen;                                           // iterator.go:109
    K += h.plen + h.klen;
    V += h.vlen;
    n++;
  }
  return WalkResult{n, K, V, st};
}

// ---- wave primitives: DPP row_shr inside each 16-lane row, the four rows combined through
// v_readlane (scalar).  (No row_bcast: its row-masked forms are not relied on here.)
__device__ __forceinline__ uint32_t readlane(uint32_t v, uint32_t l) {
  return __builtin_amdgcn_readlane(v, l);
}

// ---------------------------------------------------------------------------------- prefix
struct Tot {
  uint32_t n, k, v;
};

// Poll bound: wall-clock, not a poll count -- a legal but slow predecessor (a block of
// thousands of prefix-compressed entries with megabytes of output keys) may take milliseconds;
// only a real deadlock runs into the bound, which then ends the wait with an error flag.
constexpr uint64_t kSpinTimeoutTicks = 200000000ull;  // 2 s of the 100 MHz s_memrealtime clock
struct SpinBound {
  uint64_t t0 = 0;
  uint32_t polls = 0;
  __device__ __forceinline__ bool expired() {  // call once per unsuccessful poll
    if ((++polls & 255u) != 0) return false;   // read the clock every 256 polls
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    if (t0 == 0) t0 = t;
    return t - t0 > kSpinTimeoutTicks;
  }
};

__device__ __forceinline__ void flag_timeout(uint64_t* result, uint32_t lane) {
  if (lane == 0) atomicOr(reinterpret_cast<unsigned long long*>(result + 5), 2ull);
}

// Saturating (u32) wave scan / sum: DPP row_shr inside 16-lane rows, rows combined through
// v_readlane (the prefix protocol's values saturate instead of wrapping).
__device__ __forceinline__ uint32_t row_incl_sat(uint32_t v) {
  v = sat_add(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true));
  v = sat_add(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, true));
  v = sat_add(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, true));
  v = sat_add(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, true));
  return v;
}
__device__ __forceinline__ uint32_t wave_scan_sat(uint32_t v, uint32_t lane) {
  v = row_incl_sat(v);
  const uint32_t r0 = __builtin_amdgcn_readlane(v, 15);
  const uint32_t r1 = sat_add(r0, __builtin_amdgcn_readlane(v, 31));
  const uint32_t r2 = sat_add(r1, __builtin_amdgcn_readlane(v, 47));
  const uint32_t row = lane >> 4;
  return sat_add(v, row == 0 ? 0u : row == 1 ? r0 : row == 2 ? r1 : r2);
}
// Inclusive max-scan over the wave (DPP row_shr inside 16-lane rows, rows through v_readlane).
__device__ __forceinline__ uint32_t wave_scan_max(uint32_t v, uint32_t lane) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, true));
  const uint32_t r0 = __builtin_amdgcn_readlane(v, 15);
  const uint32_t r1 = max(r0, __builtin_amdgcn_readlane(v, 31));
  const uint32_t r2 = max(r1, __builtin_amdgcn_readlane(v, 47));
  const uint32_t row = lane >> 4;
  return max(v, row == 0 ? 0u : row == 1 ? r0 : row == 2 ? r1 : r2);
}
__device__ __forceinline__ uint32_t wave_sum_sat(uint32_t v) {  // uniform result
  v = row_incl_sat(v);
  return sat_add(sat_add(__builtin_amdgcn_readlane(v, 15), __builtin_amdgcn_readlane(v, 31)),
                 sat_add(__builtin_amdgcn_readlane(v, 47), __builtin_amdgcn_readlane(v, 63)));
}
__device__ __forceinline__ bool read3(const uint64_t* r, uint64_t tag, uint32_t& a, uint32_t& b,
                                      uint32_t& c) {
  const uint64_t x0 = gload(r), x1 = gload(r + 1), x2 = gload(r + 2);
  a = (uint32_t)x0;
  b = (uint32_t)x1;
  c = (uint32_t)x2;
  return (x0 >> kTagShift) == tag && (x1 >> kTagShift) == tag && (x2 >> kTagShift) == tag;
}
__device__ __forceinline__ void store3(uint64_t* r, uint64_t tag, uint32_t a, uint32_t b,
                                       uint32_t c, uint32_t lane) {
  if (lane < 3) gstore(r + lane, (tag << kTagShift) | (lane == 0 ? a : (lane == 1 ? b : c)));
}

// Decoupled look-back over group records (aggregate [0..2], inclusive [4..6]): exclusive
// {entries, key bytes, value bytes} of every group before g.
__device__ inline Tot lookback(const uint64_t* rec, uint32_t g, uint64_t tag, uint32_t lane,
                        uint64_t* result) {
  Tot ex{0, 0, 0};
  int64_t j0 = (int64_t)g - 1;
  uint32_t wsize = 8;
  SpinBound bound;
  while (j0 >= 0) {
    const int64_t j = j0 - (int64_t)lane;
    bool inc = false, ready = false;
    uint32_t a = 0, b = 0, c = 0;
    if (lane < wsize) {
      if (j < 0) {
        inc = ready = true;
      } else {
        const uint64_t* r = rec + (uint64_t)j * 8;
        inc = ready = read3(r + 4, tag, a, b, c);
        if (!inc) ready = read3(r, tag, a, b, c);
      }
    }
    const uint64_t im = __ballot(inc);
    const uint64_t rm = __ballot(ready);
    const uint32_t first = im ? (uint32_t)__builtin_ctzll(im) : wsize;
    const uint32_t last = first < wsize ? first : wsize - 1;
    const uint64_t need = (last >= 63) ? ~0ull : ((1ull << (last + 1)) - 1);
    if ((rm & need) != need) {
      if (bound.expired()) {
        flag_timeout(result, lane);
        return ex;
      }
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    const bool contrib = lane < wsize && lane <= last;
    ex.n = sat_add(ex.n, wave_sum_sat(contrib ? a : 0u));
    ex.k = sat_add(ex.k, wave_sum_sat(contrib ? b : 0u));
    ex.v = sat_add(ex.v, wave_sum_sat(contrib ? c : 0u));
    if (first < wsize) break;
    j0 -= (int64_t)wsize;
    wsize = 64;
  }
  return ex;
}

// Look-back by every thread of the workgroup (round 5, the default; LSMGPU_WSC_LOOKBACK=window
// selects the windowed one above): thread i sums
// the AGGREGATES of predecessor tiles i, i + nthreads, ... (waiting for each to be published),
// so the exclusive prefix costs about one round trip however many tiles finish together --
// the windowed look-back above walks back 64 tiles per round trip while no inclusive prefix is
// published yet (1,041 tiles finishing at once: ~35 us, profiles/r05q).  Returns this thread's
// partial sums; the caller reduces them over the workgroup.  A timeout sets result[5] bit 2.
__device__ inline Tot lookback_partial(const uint64_t* rec, uint32_t g, uint64_t tag, uint32_t tid,
                                       uint32_t nthreads, uint64_t* result) {
  Tot s{0, 0, 0};
  for (uint32_t j = tid; j < g; j += nthreads) {
    const uint64_t* r = rec + (uint64_t)j * 8;
    uint32_t a, b, c;
    SpinBound bound;
    while (!read3(r, tag, a, b, c)) {
      if (bound.expired()) {
        atomicOr(reinterpret_cast<unsigned long long*>(result + 5), 2ull);
        return s;
      }
      __builtin_amdgcn_s_sleep(8);
    }
    s.n = sat_add(s.n, a);
    s.k = sat_add(s.k, b);
    s.v = sat_add(s.v, c);
  }
  return s;
}

// ------------------------------------------------------------------------ LDS-DMA staging
typedef __attribute__((address_space(3))) void lds_void_t;
// One LDS-DMA piece: lane l's 16 bytes at gptr -> LDS lds + 16 * l (global_load_lds_dwordx4,
// M0 = LDS base).  Inline asm ON PURPOSE: the compiler treats an LDS-DMA it can see as a
// writer of every LDS byte and drains vmcnt before the next LDS read -- which would make
// each walk wait for the NEXT block's prefetch.  The kernel's own `s_waitcnt vmcnt(0)` at the
// top of each iteration is what orders a block's DMA before its reads.
__device__ __forceinline__ void dma16(const uint8_t* gptr, uint8_t* lds) {
  const uint32_t m0 = uniform((uint32_t)(uintptr_t)(lds_void_t*)lds);
  uint32_t saved;  // M0 is reserved to the compiler: restore it
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(saved)
      : "v"(gptr), "s"(m0)
      : "memory");
}

struct BlockRef {
  uint32_t off, len, sh;
  bool fits, tail;  // tail: a chunk crosses the end of the data buffer (loaded by lanes)
};

// Block [off, off + len): if it fits the slot, its bytes are issued into `buf` by LDS-DMA
// (global_load_lds_dwordx4: 1 KiB per wave instruction, no VGPRs), 16-B aligned source; the
// chunk crossing the end of the data buffer (last block only) is left for land_tail().
template <int SLOT, int ITERS>
__device__ __forceinline__ BlockRef prefetch_block(const DecodeParams& p, uint32_t off,
                                                   uint32_t len, uint8_t* buf, uint32_t lane) {
  BlockRef r{off, len, 0, false, false};
  r.fits = r.len <= (uint32_t)SLOT && (uint64_t)r.off + r.len <= p.data_len;
  if (!r.fits) return r;
  const uint64_t a0 = r.off & ~15ull;
  r.sh = (uint32_t)(r.off - a0);
  const uint32_t nchunk = (r.sh + r.len + 15) >> 4;
  r.tail = a0 + 16ull * nchunk > p.data_len;
#pragma unroll
  for (int i = 0; i < ITERS; i++) {
    const uint32_t c = lane + i * kWave;
    const uint64_t a = a0 + 16ull * c;
    if (c < nchunk && a + 16 <= p.data_len) dma16(p.data + a, buf + i * 1024);
  }
  return r;
}

__device__ __forceinline__ void land_tail(const DecodeParams& p, const BlockRef& r, uint8_t* buf,
                                          uint32_t lane) {
  const uint64_t a0 = r.off & ~15ull;
  const uint32_t c = (uint32_t)((p.data_len - a0) >> 4);  // the chunk crossing data_len
  if (lane == c % kWave) {
    const uint64_t a = a0 + 16ull * c;
    uint4 v = make_uint4(0, 0, 0, 0);
    for (int i = 0; i < 16; i++)
      if (a + i < p.data_len) set_byte(v, i, p.data[a + i]);
    *reinterpret_cast<uint4*>(buf + 16 * c) = v;
  }
}

}  // namespace lsmgpu
