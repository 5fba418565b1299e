// decode_wsc.hip -- "walk, scan, copy" SST block decode: the default path for batches of
// >= 1,024 blocks < 64 KiB (BASELINE C2-C5), plus the fused tile kernel (a forced path).
//
// The serial header chain is walked by ONE LANE PER BLOCK straight from global memory -- 64
// blocks per wave, every block of the batch in flight, each hop one dependent 8-B load -- and
// the bytes are then moved by a separate, fully parallel copy with known output bases:
//   K1 walk_kernel : lane b walks block b exactly like blockIterator.Next/parseKV
//                    (table/iterator.go:93-135), writing per entry {pos | value offset << 16,
//                    key offset} (full-line chunks, see flush_meta) and {entries, key
//                    bytes, value bytes} + status per block; each 256-block workgroup then
//                    scans its blocks and finds its base by decoupled look-back, so K1 ends
//                    with every block's output base
//   K2 copy_kernel : one wave per block (two above 8 KiB); lane groups copy each entry's key
//                    and value as unaligned 16-B pieces (the last overlapping back inside the
//                    entry, so no store leaves it) global -> global, plus end offsets / view
// Traffic: the input is read twice (walk touches every line; copy reads the bytes) -- the
// price of taking the serial walk off the critical path.  Blocks must be < 64 KiB.
#include <cstdlib>
#include <type_traits>


#include "codec_common.hpp"
#include "decode_common.hpp"
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

// Per-entry metadata of the walk: uint2 {header pos | value offset << 16, key offset} (key
// offsets count plen + stored bytes: u32, prefix-compressed blocks may pass 64 KiB), entry n
// = the sentinel {stop pos | V << 16, K}.  Block b's entries are contiguous at b * wcap
// (wcap a multiple of 16: 128-B aligned chunks of 16 entries).  The walking lane stages 16
// entries in LDS and writes each chunk as one full 128-B line -- 8-B stores straight from
// 64 lanes at 64 different blocks were evicted from L2 as partial lines (4x the bytes).
constexpr uint32_t kWalkStage = 17;  // uint2 per lane row: 16 entries + 1 pad (bank spread)

__device__ __forceinline__ void flush_meta(uint2* dst, const uint2* row, uint32_t cnt) {
  if (cnt == 16) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      uint4 v;
      v.x = row[2 * i].x;
      v.y = row[2 * i].y;
      v.z = row[2 * i + 1].x;
      v.w = row[2 * i + 1].y;
      reinterpret_cast<uint4*>(dst)[i] = v;
    }
  } else {
    for (uint32_t i = 0; i < cnt; i++) dst[i] = row[i];
  }
}

// One block's walk (blockIterator.Next/parseKV, table/iterator.go:93-135) over `src` (LDS slot
// or global bytes), writing the metadata records {header pos | value offset << 16, key offset}
// + the sentinel straight to `meta`.  A fast loop takes plen == 0 entries (all Builder writes,
// SURVEY F1) with one 8-B header read each; the general loop continues from wherever it stops
// and applies every stop rule in the iterator's order.
template <class Src>
__device__ __forceinline__ WalkResult walk_meta(const Src& src, const uint8_t* fast, uint32_t len,
                                                uint2* meta) {
  uint32_t pos = 0, n = 0, K = 0, V = 0, st = LSMGPU_BLK_OK;
  if (fast) {
    for (;;) {
      uint2 hw;
      __builtin_memcpy(&hw, fast + pos, 8);  // pos <= len keeps the read inside the block's span
      const uint32_t plen = __builtin_amdgcn_perm(0u, hw.x, 0x0c0c0001u);
      const uint32_t klen = __builtin_amdgcn_perm(0u, hw.x, 0x0c0c0203u);
      const uint32_t vlen = __builtin_amdgcn_perm(0u, hw.y, 0x0c0c0001u);
      const uint32_t end = pos + 10 + klen + vlen;
      if ((len - pos < 10) | (klen == 0) | (plen != 0) | (end > len)) break;
      meta[n] = make_uint2(pos | (V << 16), K);
      K += klen;
      V += vlen;
      n++;
      pos = end;
    }
  }
  for (;;) {
    if (pos >= len) break;                                   // iterator.go:115-118
    if (len - pos < 10) { st = LSMGPU_BLK_TRUNC_HEADER; break; }
    const Hdr h = src.hdr(pos);                              // iterator.go:121
    if ((h.klen | h.plen) == 0) break;                       // iterator.go:124-127
    if (n == 0 && h.plen != 0) { st = LSMGPU_BLK_FIRST_PLEN; break; }  // iterator.go:129-133
    if (10 + h.plen > len) { st = LSMGPU_BLK_PREFIX_OOB; break; }      // base key = entry 0's
    const uint32_t end = pos + 10 + h.klen + h.vlen;         // iterator.go:101-109
    if (end > len) { st = LSMGPU_BLK_VALUE_OVERFLOW; break; }
    meta[n] = make_uint2(pos | (V << 16), K);
    K += h.plen + h.klen;
    V += h.vlen;
    n++;
    pos = end;
  }
  meta[n] = make_uint2(pos | (V << 16), K);  // sentinel
  return WalkResult{n, K, V, st};
}

// ---------------------------------------------------------------------------- scan walk
// kWalkScan: the walk of the other modes is a chain of dependent header reads (one HBM round
// trip per entry, or per same-shape run).  Here a wave takes a block and finds its headers
// without a chain:
//  1. candidates: the block streams through registers in 1 KiB chunks, all issued at once
//     (lane l: bytes 16l .. 16l + 23 of the chunk); position q is a candidate when bytes q,
//     q+1 (plen) and q+6, q+7 (the high half of prev) are zero.  Builder writes plen = 0
//      and prev = the block-relative offset of the previous header (< 64 KiB), so
//     every header it writes is a candidate, except the first (prev = 0xffffffff), which is
//     added;
//  2. each candidate's header is read (L2-warm) and a candidate is kept when one of the 4
//     candidates before it is the entry its prev names and ends exactly at it (drops the
//     false candidates inside keys and values, e.g. at h + 1 when prev < 256);
//  3. the kept list is accepted only if it IS the iterator's walk: it starts at 0, every kept
//     entry passes the fast checks (plen == 0, klen != 0, fits the block) and ends at the next
//     kept position, and the first one that does not is a terminator or ends at len
//     (iterator.go:115-127).  Anything else -- a false candidate that survived, a header with
//     plen != 0 or a wild prev, a malformed block, more than kScanCap candidates -- takes
//     walk_meta, the serial walk with every stop rule, from lane 0.
// The metadata records are the other walks' (the copy is unchanged).  The VALU is the budget
// (a wave64 instruction holds its SIMD for 4 cycles): ~45 instructions per 1 KiB chunk.
constexpr uint32_t kScanCap = 256;   // candidate headers per block held in LDS
// one wave's LDS: the candidates, then (blocks of <= SG KiB) the block's bytes, so that step 2
// reads the headers from LDS instead of a second HBM round trip per block
template <uint32_t SG>
constexpr uint32_t scan_slot_bytes() { return (kScanCap + 2) * 8 + SG * 1024 + 32; }  // 16-B aligned

// 0x80 in every byte of x that is zero
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) {
  return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
}

// the 24-B window of chunk c at lane l: bytes q0 .. q0 + 23 of the block (a = its address in
// the data buffer, q0 = 1024c + 16l).  A window past data_len is read from the buffer's last
// 24 B and shifted into place by scan_fix (registers only: no wait on later chunks' loads).
__device__ __forceinline__ void scan_issue(const DecodeParams& p, uint64_t a, uint32_t (&w)[6]) {
  const uint64_t ac = a + 24 <= p.data_len ? a : p.data_len - 24;
  uint4 x;
  uint2 y;
  __builtin_memcpy(&x, p.data + ac, 16);
  __builtin_memcpy(&y, p.data + ac + 16, 8);
  w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w; w[4] = y.x; w[5] = y.y;
}
__device__ __forceinline__ void scan_fix(const DecodeParams& p, uint64_t a, uint32_t (&w)[6]) {
  if (a + 24 <= p.data_len) return;
  const uint64_t sh64 = a - (p.data_len - 24);
  const uint32_t sh = sh64 < 24 ? (uint32_t)sh64 : 24u;
  uint32_t x[7];
#pragma unroll
  for (int d = 0; d < 6; d++) x[d] = w[d];
  x[6] = 0;
  const uint32_t ds = sh >> 2, bs = sh & 3u;
  auto sel = [&](uint32_t i) {
    uint32_t r = 0;
#pragma unroll
    for (uint32_t k = 0; k < 7; k++) r = i == k ? x[k] : r;
    return r;
  };
#pragma unroll
  for (uint32_t d = 0; d < 6; d++) w[d] = __builtin_amdgcn_alignbyte(sel(d + ds + 1), sel(d + ds), bs);
}

// Candidates of the window's 16 positions as byte flags: byte k of dword d is 0x80 when
// position 4d + k is a candidate (bytes q, q+1, q+6, q+7 zero).
__device__ __forceinline__ void scan_flags(const uint32_t (&w)[6], uint32_t (&c)[4]) {
  uint32_t z[6], pz[6];
#pragma unroll
  for (int d = 0; d < 6; d++) z[d] = zero_bytes(w[d]);
#pragma unroll
  for (int d = 0; d < 5; d++) pz[d] = z[d] & __builtin_amdgcn_alignbyte(z[d + 1], z[d], 1);
  pz[5] = z[5] & (z[5] >> 8);  // positions 20..22: all the (q + 6) pairs needed below
#pragma unroll
  for (int d = 0; d < 4; d++) c[d] = pz[d] & __builtin_amdgcn_alignbyte(pz[d + 2], pz[d + 1], 2);
}
// the flags as 16 bits in position order (bit i = position q0 + i)
__device__ __forceinline__ uint32_t flags_ordered(const uint32_t (&c)[4]) {
  uint32_t m = 0;
#pragma unroll
  for (int d = 0; d < 4; d++) m |= ((((c[d] >> 7) * 0x00204081u) >> 21) & 0xfu) << (4 * d);
  return m;
}
// bits i >= rem cleared (0 <= rem)
__device__ __forceinline__ void flags_limit(uint32_t (&c)[4], uint32_t rem) {
#pragma unroll
  for (int d = 0; d < 4; d++) {
    const uint32_t r = rem > 4u * d ? rem - 4u * d : 0u;  // valid bytes of dword d
    c[d] &= r >= 4 ? 0xffffffffu : (1u << (8 * r)) - 1u;
  }
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Step 1: the candidates of the block, in position order, into cand[].x; returns their count.
// G chunks at a time: all G windows are loaded first, then processed in straight-line code,
// so the compiler waits on each with an exact partial vmcnt (a prefetch carried around a loop
// made it drain to vmcnt(0)); every window is processed (a guard would let the compiler sink
// each load into its guarded use; a chunk past the block has no candidates).  Chunks past
// the block re-read its last chunk (same lines, no traffic).  TAIL: a window may cross the
// end of the data buffer (the last blocks of a buffer).
template <bool TAIL, uint32_t G>
__device__ __forceinline__ uint32_t scan_candidates(const DecodeParams& p, uint32_t off,
                                                    uint32_t len, uint2* cand, uint8_t* bbuf,
                                                    uint32_t lane) {
  const uint32_t nch = (len + 1023) >> 10;
  const uint64_t a0 = (uint64_t)off + 16 * lane;
  const uint64_t below = (1ull << lane) - 1ull;
  uint32_t m = 0;
  for (uint32_t c0 = 0; c0 < nch; c0 += G) {
    uint32_t w[G][6];
#pragma unroll
    for (uint32_t s = 0; s < G; s++) scan_issue(p, a0 + 1024 * min(c0 + s, nch - 1), w[s]);
#pragma unroll
    for (uint32_t s = 0; s < G; s++) {
      const uint32_t c = c0 + s;
      const uint32_t q0 = 1024 * c + 16 * lane;
      if constexpr (TAIL) scan_fix(p, a0 + 1024 * min(c, nch - 1), w[s]);
      if (nch <= G)  // the whole block fits the LDS slot (uniform): keep its bytes
        *reinterpret_cast<uint4*>(bbuf + 1024 * s + 16 * lane) = make_uint4(w[s][0], w[s][1], w[s][2], w[s][3]);
      uint32_t f[4];
      scan_flags(w[s], f);
      if (1024 * c + 1024 > len) flags_limit(f, len > q0 ? len - q0 : 0u);  // uniform
      // permuted bits: bit 8k + d = position 4d + k
      uint32_t x = (f[0] >> 7) | (f[1] >> 6) | (f[2] >> 5) | (f[3] >> 4);
      if (c == 0) x |= lane == 0 ? 1u : 0u;  // position 0: the first header
      const uint64_t b1 = __ballot(x != 0);
      const uint64_t b2 = __ballot((x & (x - 1)) != 0);
      if (b2 == 0) {  // at most one candidate per lane: its rank is a ballot count
        if (x) {
          const uint32_t bit = __builtin_ctz(x);
          const uint32_t idx = m + (uint32_t)__popcll(b1 & below);
          if (idx < kScanCap) cand[idx].x = q0 + 4 * (bit & 7) + (bit >> 3);
        }
        m += (uint32_t)__popcll(b1);
      } else {        // several in one lane (e.g. a header and a false one at h + 1)
        uint32_t cm = flags_ordered(f);
        if (c == 0 && lane == 0) cm |= 1u;
        const uint32_t cnt = __popc(cm);
        const uint32_t incl = wave_scan_sat(cnt, lane);
        uint32_t idx = m + incl - cnt;
        while (cm) {
          if (idx < kScanCap) cand[idx].x = q0 + __builtin_ctz(cm);
          idx++;
          cm &= cm - 1;
        }
        m += __builtin_amdgcn_readlane(incl, 63);
      }
    }
  }
  return m;
}

__device__ __forceinline__ WalkResult scan_serial(const uint8_t* blk, uint32_t len, uint2* meta,
                                                  uint32_t lane) {
  WalkResult r{0, 0, 0, LSMGPU_BLK_OK};
  if (lane == 0) r = walk_meta(GlobalSrc{blk}, blk, len, meta);
  return WalkResult{(uint32_t)__shfl((int)r.n, 0), (uint32_t)__shfl((int)r.K, 0),
                    (uint32_t)__shfl((int)r.V, 0), (uint32_t)__shfl((int)r.status, 0)};
}

// One block by the scan walk (whole wave; the result is uniform).  cand: kScanCap + 1 uint2 of
// this wave's LDS -- {pos | prev << 16, info}, info = klen | vlen << 16 for an entry that passes
// the fast checks, 0 for a terminator, ~0u otherwise.  G: chunks loaded at once.
template <uint32_t G>
__device__ __forceinline__ WalkResult scan_block(const DecodeParams& p, uint32_t off, uint32_t len,
                                                 uint2* meta, uint2* cand, uint32_t lane) {
  const uint8_t* blk = p.data + off;
  if (len < 10 || p.data_len < 24) return scan_serial(blk, len, meta, lane);
  // 1. candidates
  const bool tail = (uint64_t)off + (((len + 1023) >> 10) << 10) + 24 > p.data_len;
  uint8_t* const bbuf = reinterpret_cast<uint8_t*>(cand + kScanCap + 2);  // 16-B aligned
  const uint32_t m = tail ? scan_candidates<true, G>(p, off, len, cand, bbuf, lane)
                          : scan_candidates<false, G>(p, off, len, cand, bbuf, lane);
  if (m > kScanCap) return scan_serial(blk, len, meta, lane);
  wave_lds_fence();
  const bool staged = len <= G * 1024;  // uniform: the block's bytes are in bbuf
  // 2a. every candidate's header: from LDS, or from global memory (the lines were just read)
  for (uint32_t i = lane; i < m; i += kWave) {
    const uint32_t q = cand[i].x;
    uint32_t info = ~0u, prev = 0xffffu;
    if (q + 10 <= len) {
      uint2 hw;
      uint32_t lo;
      if (staged) {  // three aligned dword reads
        const uint32_t* wp = reinterpret_cast<const uint32_t*>(bbuf + (q & ~3u));
        const uint32_t w0 = wp[0], w1 = wp[1], w2 = wp[2], w3 = wp[3];
        hw.x = __builtin_amdgcn_alignbyte(w1, w0, q & 3u);
        hw.y = __builtin_amdgcn_alignbyte(w2, w1, q & 3u);
        lo = __builtin_amdgcn_alignbyte(w3, w2, q & 3u);
      } else {
        uint16_t l16;
        __builtin_memcpy(&hw, blk + q, 8);
        __builtin_memcpy(&l16, blk + q + 8, 2);
        lo = l16;
      }
      const uint32_t plen = __builtin_amdgcn_perm(0u, hw.x, 0x0c0c0001u);
      const uint32_t klen = __builtin_amdgcn_perm(0u, hw.x, 0x0c0c0203u);
      const uint32_t vlen = __builtin_amdgcn_perm(0u, hw.y, 0x0c0c0001u);
      prev = __builtin_amdgcn_perm(0u, lo, 0x0c0c0001u);  // bytes q+8, q+9 (BE); q+6, q+7 are
                                                         // zero for every candidate but q = 0
      if (plen == 0) {
        if (klen == 0) info = 0;                               // terminator
        else if (q + 10 + klen + vlen <= len) info = klen | (vlen << 16);
      }
    }
    cand[i] = make_uint2(q | (prev << 16), info);
  }
  wave_lds_fence();
  // 2b. keep: position 0, or a candidate that one of the 4 before it names as prev and that
  // entry ends here
  uint32_t keep = 0;  // bit r: candidate r * 64 + lane
  for (uint32_t r = 0; r * kWave < m; r++) {
    const uint32_t i = r * kWave + lane;
    bool k = i == 0;
    if (i < m && i > 0) {
      const uint2 ci = cand[i];
      const uint32_t q = ci.x & 0xffffu, pv = ci.x >> 16;
#pragma unroll
      for (uint32_t d = 1; d <= 4; d++) {
        const uint2 cj = cand[i >= d ? i - d : 0];
        const uint32_t pj = cj.x & 0xffffu;
        const bool fast = cj.y != 0 && cj.y != ~0u;
        k = k || (i >= d && fast && pj == pv && pj + 10 + (cj.y & 0xffffu) + (cj.y >> 16) == q);
      }
    }
    keep |= (uint32_t)k << r;
  }
  wave_lds_fence();
  // 2c. compact the kept candidates to the front (in order; a round reads only slots its own
  // writes and the later rounds' do not reach)
  uint32_t mk = 0;
  for (uint32_t r = 0; r * kWave < m; r++) {
    const uint32_t i = r * kWave + lane;
    const bool k = i < m && ((keep >> r) & 1u);
    const uint2 v = cand[min(i, m - 1)];
    const uint64_t bal = __ballot(k);
    wave_lds_fence();
    if (k) cand[mk + lanes_below(bal)] = v;
    mk += (uint32_t)__popcll(bal);
  }
  wave_lds_fence();
  // 3. the kept list must be the iterator's walk: the first kept candidate that does not link
  // to the next one is the stop (a terminator, or an entry ending at len); records
  // {pos | value offset << 16, key offset} of the entries before it, K | V << 16 scanned as
  // one word (both < 64 KiB in a block < 64 KiB)
  uint32_t t = ~0u, KV = 0;
  for (uint32_t r = 0; r * kWave < mk && t == ~0u; r++) {
    const uint32_t i = r * kWave + lane;
    const uint2 ci = cand[min(i, mk - 1)];
    const uint32_t nx = i + 1 < mk ? (cand[i + 1].x & 0xffffu) : ~0u;
    const bool fast = ci.y != 0 && ci.y != ~0u;
    const uint32_t end = (ci.x & 0xffffu) + 10 + (ci.y & 0xffffu) + (ci.y >> 16);
    const bool brk = i < mk && !(fast && end == nx);
    const uint64_t bb = __ballot(brk);
    const uint32_t tr = bb ? (uint32_t)__builtin_ctzll(bb) : 64u;  // first break in this round
    const uint32_t kv = lane < tr && fast ? ci.y : 0u;
    const uint32_t incl = wave_scan_sat(kv, lane);  // no saturation: the sums are < 2^32
    if (lane < tr && i < mk)
      meta[i] = make_uint2((ci.x & 0xffffu) | ((((KV + incl - kv) >> 16)) << 16),
                           (KV + incl - kv) & 0xffffu);
    KV += __builtin_amdgcn_readlane(incl, 63);
    if (bb) t = r * kWave + tr;
  }
  // the stop: cand[t] is a terminator (n = t) or an entry ending the block (n = t + 1)
  const uint2 ct = cand[t];
  const uint32_t pt = ct.x & 0xffffu, kl = ct.y & 0xffffu, vl = ct.y >> 16;
  uint32_t n, stop;
  if ((cand[0].x & 0xffffu) != 0) return scan_serial(blk, len, meta, lane);
  if (ct.y == 0) {
    n = t;
    stop = pt;
  } else if (ct.y != ~0u && pt + 10 + kl + vl == len) {
    n = t + 1;
    stop = len;
    if (lane == 0) meta[t] = make_uint2(pt | ((KV >> 16) << 16), KV & 0xffffu);
    KV += ct.y;
  } else {
    return scan_serial(blk, len, meta, lane);
  }
  const uint32_t K = KV & 0xffffu, V = KV >> 16;
  if (lane == 0) meta[n] = make_uint2(stop | (V << 16), K);
  return WalkResult{n, K, V, LSMGPU_BLK_OK};
}

__device__ __forceinline__ void copy_block(const DecodeParams& p, uint32_t b, uint32_t n,
                                           uint32_t K, uint32_t V, uint32_t st, uint64_t en,
                                           uint64_t ek, uint64_t ev, uint32_t off,
                                           const uint2* meta, uint32_t sub, uint32_t split,
                                           uint32_t lane);

// K1: lane = block; a workgroup = a tile of 256 consecutive blocks, tiles taken in ticket order
// (p.gcnt[0]).  After the walk the workgroup scans its blocks' {entries, key bytes, value
// bytes}, publishes the tile aggregate and finds the tile's output base by decoupled look-back
// over the tile records (epoch-tagged granules in p.lb), then writes every block's exclusive
// base: the output bases are known when the walk ends, with no separate scan launch.  The
// ticket makes every predecessor tile already running, so the look-back always progresses.
// MODE kWalkGroup (p.wwalk, the default when nblk <= 64 per CU: the lane walk would leave the
// machine idle): 256 / TB lanes per block guess same-shape runs (see the branch).
// MODE kWalkLane: lane b walks block b straight from HBM, one dependent 8-B header load per
// entry (every 128-B line of the input is fetched on its own, as scattered requests).
template <int MODE, uint32_t TB, uint32_t SG = 4>  // TB = blocks per tile (<= 256 threads:
// thread t owns block t); SG = the scan walk's chunks loaded at once (4 or 16 KiB)
__global__ void __launch_bounds__(256) wsc_walk_kernel(DecodeParams p) {
  static_assert(TB <= 256, "one thread per block of the tile");
  constexpr uint32_t kStageBytes = 256 * kWalkStage * sizeof(uint2);
  // group walk: a 32-record ring per block (the walk's LDS also serves the view epilogue's
  // owner map)
  // scan walk: one wave per block (TB = 4), kScanCap + 1 candidate slots per wave
  constexpr uint32_t kLdsBytes = MODE == kWalkGroup  ? TB * 16 * sizeof(uint2)
                                 : MODE == kWalkScan ? 4 * scan_slot_bytes<SG>()
                                                     : kStageBytes;
  static_assert(MODE != kWalkLane || kLdsBytes == kStageBytes,
                "the lane walk stages 16 records per lane");
  static_assert(MODE != kWalkScan || (TB % 4 == 0 && TB <= 256), "the scan walk: TB / 4 blocks per wave");
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
  uint2* const stage = reinterpret_cast<uint2*>(lds);
  __shared__ uint32_t s_tile;
  __shared__ uint32_t s_wave[4][3];
  __shared__ uint32_t s_ex[3];
  __shared__ uint32_t s_first[257];  // p.wfuse: tile-relative first entry of each block
  __shared__ uint32_t s_off[MODE == kWalkLane ? 256 : TB];  // each block's input offset
  constexpr uint32_t kRes = MODE == kWalkLane ? 1 : TB;
  __shared__ uint32_t s_res[4][kRes];  // group / scan walk: n, K, V, status per block
  __shared__ uint32_t s_base[3][MODE == kWalkScan ? TB : 1];  // scan walk + copy: output bases
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint32_t ntiles = (p.nblk + TB - 1) / TB;
  if (tid == 0) {
    const uint32_t t = atomicAdd(p.gcnt, 1u);
    if (t == ntiles - 1) atomicExch(p.gcnt, 0u);  // every ticket is taken
    s_tile = t;
  }
  if (p.zero_result && blockIdx.x == 0 && tid < 8) p.result[tid] = 0;  // see api.hip
  __syncthreads();
  const uint32_t tile = s_tile;
  // thread t owns block tile * TB + t (threads past TB own none: zero entries)
  const uint32_t b = tid < TB ? tile * TB + tid : 0xffffffffu;
  uint32_t n = 0, K = 0, V = 0, st = LSMGPU_BLK_OK;
  if constexpr (MODE == kWalkScan) {
    // wave w scans blocks tile * TB + w * BPW + j, j < BPW, one after the other
    constexpr uint32_t BPW = TB / 4;
    uint2* cand = reinterpret_cast<uint2*>(lds + wave * scan_slot_bytes<SG>());
    for (uint32_t j = 0; j < BPW; j++) {
      const uint32_t t = wave * BPW + j, bw = tile * TB + t;
      if (bw >= p.nblk) break;
      const uint32_t off = uniform(p.blk_off[bw]), len = uniform(p.blk_len[bw]);
      uint2* meta = reinterpret_cast<uint2*>(p.wmeta) + (uint64_t)bw * p.wcap;
      WalkResult r{0, 0, 0, LSMGPU_BLK_RANGE};
      if ((uint64_t)off + len <= p.data_len)
        r = scan_block<SG>(p, off, len, meta, cand, lane);
      else if (lane == 0)
        meta[0] = make_uint2(0, 0);  // sentinel of an empty walk
      if (lane == 0) {
        s_res[0][t] = r.n;
        s_res[1][t] = r.K;
        s_res[2][t] = r.V;
        s_res[3][t] = r.status;
        s_off[t] = off;
      }
    }
    __syncthreads();
    if (b < p.nblk) {
      n = s_res[0][tid];
      K = s_res[1][tid];
      V = s_res[2][tid];
      st = s_res[3][tid];
      uint64_t* t = p.wstat + 3ull * b;
      t[0] = n;
      t[1] = K;
      t[2] = V;
      p.wstatus[b] = st;
    }
  } else if constexpr (MODE == kWalkGroup) {
    // L lanes per block: each round the group reads the headers at pos + k * stride (stride =
    // the last accepted entry's size) and accepts the leading run whose guesses were right --
    // lane k is entry n + k iff entries n .. n + k - 1 all had the previous entry's shape.  The
    // guessed lines belong to the next entries of the same block (no extra traffic), the group
    // fetches neighbouring lines together, and the dependent chain shrinks by the run length.
    constexpr uint32_t L = 256 / TB;
    static_assert(L >= 2 && L <= 16 && (L & (L - 1)) == 0, "2..16 lanes per block");
    constexpr uint32_t kMask = (1u << L) - 1;
    constexpr uint32_t kGroupProbe = 16;
    const uint32_t g = tid / L, k = tid & (L - 1), gb = lane & ~(L - 1);
    const uint32_t bg = tile * TB + g;
    uint2* row = stage + g * 16;  // the block's current 16-record chunk (one 128-B line)
    if (p.wprefetch) {
      // The group walk is a chain of dependent rounds (~20 per C4 block), each an HBM round
      // trip.  First touch every 128-B line of this wave's blocks once, coalesced (one dword per
      // lane per line, all in flight together), so the rounds hit L2 / the Infinity Cache.
      constexpr uint32_t BW = TB / 4;  // blocks per wave
      const uint32_t b0 = tile * TB + wave * BW;
      if (b0 < p.nblk) {
        const uint32_t b1 = min(b0 + BW, p.nblk) - 1;
        const uint64_t lo = uniform(p.blk_off[b0]) & ~127ull;
        const uint64_t hi = (uint64_t)uniform(p.blk_off[b1]) + uniform(p.blk_len[b1]);
        if (hi > lo && hi - lo <= (uint64_t)BW * 65536 && hi <= p.data_len) {
          uint32_t sink = 0;
          for (uint64_t a = lo + 128ull * lane; a < hi; a += 128ull * kWave)
            asm volatile("global_load_dword %0, %1, off" : "+v"(sink) : "v"(p.data + a) : "memory");
          // the loads write `sink` asynchronously: drain them before its register is reused
          asm volatile("s_waitcnt vmcnt(0)" : "+v"(sink) : : "memory");
        }
      }
    }
    if (bg < p.nblk) {
      const uint32_t off = p.blk_off[bg], len = p.blk_len[bg];
      uint2* meta = reinterpret_cast<uint2*>(p.wmeta) + (uint64_t)bg * p.wcap;
      uint32_t pos = 0, gn = 0, gK = 0, gV = 0, gst = LSMGPU_BLK_OK;
      if ((uint64_t)off + len > p.data_len) {
        gst = LSMGPU_BLK_RANGE;
      } else {
        const uint8_t* blk = p.data + off;
        uint32_t kref = 0xffffffffu, vref = 0, stride = 0;  // no shape yet: round 1 takes one
        uint32_t rounds = 0;
        for (;;) {
          const uint32_t q = pos + k * stride;  // < 2^21: pos, stride < 2^17, k < 16
          uint32_t plen = 1, klen = 0, vlen = 0;
          if (q + 10 <= len) read_hdr(blk + q, plen, klen, vlen);
          const uint32_t endq = q + 10 + klen + vlen;
          const bool fast = (klen != 0) & (plen == 0) & (endq <= len);
          const bool same = fast & (klen == kref) & (vlen == vref);
          const uint32_t fb = (uint32_t)(__ballot(fast) >> gb) & kMask;
          const uint32_t sb = (uint32_t)(__ballot(same) >> gb) & kMask;
          if (!(fb & 1u)) break;  // entry n itself needs the general loop (or the block ended)
          const uint32_t t = __builtin_ctz(~sb);                          // leading same-shape run
          const uint32_t m = t + ((t < L && ((fb >> t) & 1u)) ? 1u : 0u);  // + one new shape
          const uint2 rec = make_uint2(q | ((gV + k * vref) << 16), gK + k * kref);
          const uint32_t idx = gn + k, cend = (gn | 15u) + 1;  // end of the current chunk
          if (k < m && idx < cend) row[idx & 15] = rec;
          const uint32_t src = gb + m - 1;  // the last accepted entry
          pos = (uint32_t)__shfl((int)endq, (int)src);
          const uint32_t shape = (uint32_t)__shfl((int)(klen | (vlen << 16)), (int)src);
          gK += t * kref + (m > t ? (shape & 0xffffu) : 0u);
          gV += t * vref + (m > t ? (shape >> 16) : 0u);
          gn += m;
          // The guess keeps the run's shape across a single odd entry (a value pointer, a longer
          // ExpiresAt varint: the next entry usually has the common shape again) and adopts a
          // new shape only when entry n itself broke the run (C4 walk: 0.069 -> 0.038 ms).
          if (t == 0) {
            kref = shape & 0xffffu;
            vref = shape >> 16;
            stride = 10 + kref + vref;
          }
          rounds++;
          if (gn >= cend) {  // chunk [cend - 16, cend) complete: one full 128-B line
            __builtin_amdgcn_wave_barrier();
            for (uint32_t i = k; i < 8; i += L) {
              const uint2 a = row[2 * i], c = row[2 * i + 1];
              reinterpret_cast<uint4*>(meta + cend - 16)[i] = make_uint4(a.x, a.y, c.x, c.y);
            }
            __builtin_amdgcn_wave_barrier();  // the chunk is read before the next one fills
            if (k < m && idx >= cend) row[idx & 15] = rec;
          }
          // shapes do not repeat in this block (< 1.25 entries per round after 16 rounds): the
          // rest entry by entry.  A rate over many rounds, not a streak -- with thousands of
          // blocks some block always starts unluckily, and the slowest block sets the kernel's
          // time (C4 shapes, simulated: 2 per round after 8 rounds gives up on 13 % of blocks)
          if (rounds >= kGroupProbe && 4 * gn < 5 * rounds) break;
        }
        if (k == 0) {  // general loop: every stop rule in the iterator's order (as the lane walk)
          for (;;) {
            if (pos >= len) break;                                   // iterator.go:115-118
            if (len - pos < 10) { gst = LSMGPU_BLK_TRUNC_HEADER; break; }
            uint32_t plen, klen, vlen;
            read_hdr(blk + pos, plen, klen, vlen);                   // iterator.go:121
            if ((klen | plen) == 0) break;                           // iterator.go:124-127
            if (gn == 0 && plen != 0) { gst = LSMGPU_BLK_FIRST_PLEN; break; }  // :129-133
            if (10 + plen > len) { gst = LSMGPU_BLK_PREFIX_OOB; break; }
            const uint32_t end = pos + 10 + klen + vlen;             // iterator.go:101-109
            if (end > len) { gst = LSMGPU_BLK_VALUE_OVERFLOW; break; }
            row[gn & 15] = make_uint2(pos | (gV << 16), gK);
            if ((gn & 15) == 15) flush_meta(meta + (gn - 15), row, 16);
            gK += plen + klen;
            gV += vlen;
            gn++;
            pos = end;
          }
        }
      }
      if (k == 0) {
        row[gn & 15] = make_uint2(pos | (gV << 16), gK);  // sentinel
        flush_meta(meta + (gn & ~15u), row, (gn & 15) + 1);
        s_res[0][g] = gn;
        s_res[1][g] = gK;
        s_res[2][g] = gV;
        s_res[3][g] = gst;
        s_off[g] = off;
      }
    }
    __syncthreads();
    if (b < p.nblk) {  // from here on thread t owns block tile * TB + t, as in the other walks
      n = s_res[0][tid];
      K = s_res[1][tid];
      V = s_res[2][tid];
      st = s_res[3][tid];
      uint64_t* t = p.wstat + 3ull * b;
      t[0] = n;
      t[1] = K;
      t[2] = V;
      p.wstatus[b] = st;
    }
  } else if (b < p.nblk) {
    uint2* row = stage + tid * kWalkStage;
    const uint32_t off = p.blk_off[b], len = p.blk_len[b];
    uint32_t pos = 0;
    s_off[tid] = off;
    uint2* meta = reinterpret_cast<uint2*>(p.wmeta) + (uint64_t)b * p.wcap;
    if ((uint64_t)off + len > p.data_len) {
      st = LSMGPU_BLK_RANGE;
    } else {
      const uint8_t* blk = p.data + off;
      for (;;) {
        if (pos >= len) break;                                   // iterator.go:115-118
        if (len - pos < 10) { st = LSMGPU_BLK_TRUNC_HEADER; break; }
        uint32_t plen, klen, vlen;
        read_hdr(blk + pos, plen, klen, vlen);                   // iterator.go:121
        if ((klen | plen) == 0) break;                           // iterator.go:124-127
        if (n == 0 && plen != 0) { st = LSMGPU_BLK_FIRST_PLEN; break; }  // iterator.go:129-133
        if (10 + plen > len) { st = LSMGPU_BLK_PREFIX_OOB; break; }      // base key = entry 0's
        const uint32_t end = pos + 10 + klen + vlen;             // iterator.go:101-109
        if (end > len) { st = LSMGPU_BLK_VALUE_OVERFLOW; break; }
        row[n & 15] = make_uint2(pos | (V << 16), K);  // n < wcap - 1: >= 10 B per entry
        if ((n & 15) == 15) flush_meta(meta + (n - 15), row, 16);
        K += plen + klen;
        V += vlen;
        n++;
        pos = end;
      }
    }
    row[n & 15] = make_uint2(pos | (V << 16), K);
    flush_meta(meta + (n & ~15u), row, (n & 15) + 1);
    uint64_t* t = p.wstat + 3ull * b;
    t[0] = n;
    t[1] = K;
    t[2] = V;
    p.wstatus[b] = st;
  }
  // tile scan (saturating u32: a key stream past 4 GiB - 1 fails the copy's capacity check)
  const uint32_t in_ = wave_scan_sat(n, lane), ik = wave_scan_sat(K, lane),
                 iv = wave_scan_sat(V, lane);
  if (lane == 63) {
    s_wave[wave][0] = in_;
    s_wave[wave][1] = ik;
    s_wave[wave][2] = iv;
  }
  __syncthreads();
  if (wave == 0) {
    uint32_t tn = 0, tk = 0, tv = 0;
    for (int w = 0; w < 4; w++) {
      tn = sat_add(tn, s_wave[w][0]);
      tk = sat_add(tk, s_wave[w][1]);
      tv = sat_add(tv, s_wave[w][2]);
    }
    uint64_t* R = p.lb + (uint64_t)tile * 8;
    Tot ex{0, 0, 0};
    if (tile > 0 && !(p.ablate & 1)) {  // LSMGPU_ABLATE bit 1: timing only, wrong bases
      store3(R, p.tag, tn, tk, tv, lane);
      ex = lookback(p.lb, tile, p.tag, lane, p.result);
    }
    store3(R + 4, p.tag, sat_add(ex.n, tn), sat_add(ex.k, tk), sat_add(ex.v, tv), lane);
    if (lane == 0) {
      s_ex[0] = ex.n;
      s_ex[1] = ex.k;
      s_ex[2] = ex.v;
    }
  }
  __syncthreads();
  if (b < p.nblk) {
    uint32_t on = s_ex[0], ok = s_ex[1], ov = s_ex[2];
    for (uint32_t w = 0; w < wave; w++) {
      on = sat_add(on, s_wave[w][0]);
      ok = sat_add(ok, s_wave[w][1]);
      ov = sat_add(ov, s_wave[w][2]);
    }
    const uint32_t en = sat_add(on, in_ - n), ek = sat_add(ok, ik == 0xffffffffu ? ik : ik - K),
                   ev = sat_add(ov, iv - V);
    if (MODE == kWalkScan && p.wcopy) {  // this workgroup copies its blocks (below)
      s_base[0][tid] = en;
      s_base[1][tid] = ek;
      s_base[2][tid] = ev;
    } else if (!p.wfuse) {
      uint64_t* bs = p.wbase + 3ull * b;
      bs[0] = en;
      bs[1] = ek;
      bs[2] = ev;
    } else {  // view-only decode: the copy kernel's per-block duties, done here
      if (p.blk_first) p.blk_first[b] = en;
      if (p.blk_status) p.blk_status[b] = (int32_t)st;
      if (st != LSMGPU_BLK_OK) {
        atomicAdd(reinterpret_cast<unsigned long long*>(p.result + 4), 1ull);
        atomicMax(reinterpret_cast<unsigned long long*>(p.result + 3),
                  (unsigned long long)(p.nblk - b));
      }
      if (b == p.nblk - 1) {  // totals of the whole batch
        if (p.blk_first) p.blk_first[p.nblk] = (uint32_t)((uint64_t)en + n);
        p.result[0] = (uint64_t)en + n;
        p.result[1] = (uint64_t)ek + K;
        p.result[2] = (uint64_t)ev + V;
      }
      if (!((uint64_t)en + n <= p.ent_cap && (uint64_t)en + n <= 0xffffffffull))
        atomicOr(reinterpret_cast<unsigned long long*>(p.result + 5), 1ull);
    }
  }
  if constexpr (MODE == kWalkScan) {
    // scan walk, p.wcopy: wave w copies block tile * 4 + w as the copy kernel would (its
    // metadata records were written by this same wave; the barrier orders them)
    if (p.wcopy) {
      __syncthreads();
      constexpr uint32_t BPW = TB / 4;
      for (uint32_t j = 0; j < BPW; j++) {
        const uint32_t t = wave * BPW + j, bw = tile * TB + t;
        if (bw >= p.nblk) break;
        copy_block(p, bw, s_res[0][t], s_res[1][t], s_res[2][t], s_res[3][t], s_base[0][t],
                   s_base[1][t], s_base[2][t], s_off[t],
                   reinterpret_cast<const uint2*>(p.wmeta) + (uint64_t)bw * p.wcap, 0, 1, lane);
      }
      return;
    }
  }
  if (!p.wfuse) return;
  // View-only decode (p.wfuse): the workgroup writes its tile's dense view records itself, so
  // no copy launch follows.  Output entry e of the tile belongs to the last block whose first
  // entry is <= e (binary search over s_first); its record comes from the walk metadata this
  // workgroup just wrote (L2-hot), and consecutive threads write consecutive 8-B records.
  {
    uint32_t rel = in_ - n;  // entries of the tile never saturate (<= 256 x 6,554)
    for (uint32_t w = 0; w < wave; w++) rel += s_wave[w][0];
    s_first[tid] = rel;
    if (tid == 255) s_first[256] = rel + n;
  }
  __syncthreads();
  if (!((p.mode & LSMGPU_MODE_VIEW) && p.view) || (p.ablate & 2)) return;  // mode 0: no view
  const uint32_t nt = s_first[256];
  const uint64_t e0 = s_ex[0];
  // entry -> block map in the walk's staging rows (free now): each thread marks its block's
  // entries, so the lookup is one LDS read (tiles of more entries: binary search)
  using Owner = uint16_t;
  Owner* owner = reinterpret_cast<Owner*>(lds);  // the walk's LDS is free now (from its start)
  static_assert(TB - 1 <= (uint32_t)(Owner)~Owner(0), "tile width must fit the owner slot");
  const bool mapped = nt <= kLdsBytes / sizeof(Owner);  // owner slots in the walk's LDS
  if (mapped) {
    const uint32_t f = s_first[tid];
    for (uint32_t i = 0; i < n; i++) owner[f + i] = (Owner)tid;
    __syncthreads();
  }
  for (uint32_t e = tid; e < nt; e += 256) {
    uint32_t lo = 0, hi = 255;
    if (mapped) {
      lo = owner[e];
    } else {
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (s_first[mid] <= e) lo = mid; else hi = mid - 1;
      }
    }
    const uint64_t bend = e0 + s_first[lo + 1];
    if (bend > p.ent_cap || bend > 0xffffffffull) continue;  // reported above (result[5])
    const uint32_t i = e - s_first[lo];
    const uint2* meta = reinterpret_cast<const uint2*>(p.wmeta) + (uint64_t)(tile * TB + lo) * p.wcap;
    const uint2 m0 = meta[i], m1 = meta[i + 1];
    const uint32_t hp = m0.x & 0xffffu, vl = (m1.x >> 16) - (m0.x >> 16);
    const uint32_t kl = (m1.x & 0xffffu) - hp - 10 - vl;  // stored key bytes
    p.view[e0 + e] = (uint64_t)(s_off[lo] + hp + 10) | ((uint64_t)kl << 32) | ((uint64_t)vl << 48);
  }
}

// The entries of one block: J lanes per entry; an entry's pieces are [key pieces | value
// pieces] (16 B, the last overlapping back inside its stream, or two overlapping 8/4/2/1-B
// pieces below 16 B) and lane j takes pieces j, j + J, ...  G entry groups per pass, all
// metadata loads issued first.
template <uint32_t J, uint32_t G>
__device__ __forceinline__ void copy_entries(const DecodeParams& p, const uint2* meta,
                                             const uint8_t* blk, uint8_t* kbase, uint8_t* vbase,
                                             uint32_t n, uint64_t en, uint64_t ek, uint64_t ev,
                                             uint32_t off, uint32_t sub, uint32_t split,
                                             bool mat, bool view, uint32_t lane, uint2 pre) {
  const uint32_t j = lane & (J - 1);
  bool any_plen = false;
  for (uint32_t e0 = sub * G * (kWave / J); e0 < n; e0 += split * G * (kWave / J)) {
    uint32_t hp[G], kl[G], vl[G], ko[G], vo[G], np[G], kp[G];
    bool on[G];
    // a pass whose entries (and their successors) are all below 64 reads the metadata the
    // kernel preloaded one record per lane (`pre`) by lane shuffle, not from memory
    const bool shuffled = e0 + G * (kWave / J) < kWave;
#pragma unroll
    for (int i = 0; i < G; i++) {
      const uint32_t e = e0 + i * (kWave / J) + (lane / J);
      const uint32_t ec = min(e, n - 1);
      uint2 m0, m1;
      if (shuffled) {
        m0.x = (uint32_t)__shfl((int)pre.x, (int)ec);
        m0.y = (uint32_t)__shfl((int)pre.y, (int)ec);
        m1.x = (uint32_t)__shfl((int)pre.x, (int)ec + 1);
        m1.y = (uint32_t)__shfl((int)pre.y, (int)ec + 1);
      } else {
        m0 = meta[ec];
        m1 = meta[ec + 1];
      }
      hp[i] = m0.x & 0xffffu;
      vo[i] = m0.x >> 16;
      ko[i] = m0.y;
      const uint32_t ko1 = m1.y, vo1 = m1.x >> 16;
      vl[i] = vo1 - vo[i];
      kl[i] = (m1.x & 0xffffu) - hp[i] - 10 - vl[i];  // stored key bytes
      const uint32_t plen = ko1 - ko[i] - kl[i];
      on[i] = e < n;
      any_plen = any_plen || (on[i] && plen != 0);
      kp[i] = plen ? 0u : pieces16(kl[i]);  // prefix-compressed keys: bytewise pass below
      np[i] = kp[i] + pieces16(vl[i]);
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
        copy_piece16(dst + (key ? ko[i] : vo[i]), blk + s0, len, key ? q : q - kp[i]);
      }
    }
  }
  if (any_plen && kbase && mat) {  // baseKey[:plen] ++ diff (iterator.go:98-100): bytewise
    // the same passes as above (any_plen covers only this wave's entries)
    for (uint32_t e = sub * G * (kWave / J) + (lane / J); e < n;
         e += ((e / (kWave / J)) % G == G - 1) ? (split - 1) * G * (kWave / J) + kWave / J
                                              : kWave / J) {
      const uint2 m0 = meta[e], m1 = meta[e + 1];
      const uint32_t hp = m0.x & 0xffffu, ko = m0.y;
      const uint32_t vl = (m1.x >> 16) - (m0.x >> 16);
      const uint32_t kl = m1.y - ko;                                // output key bytes
      const uint32_t plen = kl - ((m1.x & 0xffffu) - hp - 10 - vl);
      if (plen == 0) continue;
      for (uint32_t i = j; i < kl; i += J)
        kbase[ko + i] = i < plen ? blk[10 + i] : blk[hp + 10 + i - plen];
    }
  }
}

// One block's share of the copy (wave `sub` of `split`): the per-block outputs (first entry,
// status, error counters, totals, capacity check) and the entries' bytes / end offsets / view
// records.  n, K, V, st = the walk's results; en, ek, ev = the block's output bases.
__device__ __forceinline__ void copy_block(const DecodeParams& p, uint32_t b, uint32_t n,
                                           uint32_t K, uint32_t V, uint32_t st, uint64_t en,
                                           uint64_t ek, uint64_t ev, uint32_t off,
                                           const uint2* meta, uint32_t sub, uint32_t split,
                                           uint32_t lane) {
  // the first 64 metadata records, one per lane, requested before the per-block stores
  // (one round trip fewer before the piece loads; records past the sentinel are never used)
  const uint2 pre = meta[min(lane, p.wcap - 1)];
  if (lane == 0 && sub == 0) {
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
    if (lane == 0 && sub == 0) atomicOr(reinterpret_cast<unsigned long long*>(p.result + 5), 1ull);
    return;
  }
  if (n == 0 || (p.ablate & 2)) return;
  const uint8_t* blk = p.data + off;
  uint8_t* kbase = p.key_data ? p.key_data + ek : nullptr;
  uint8_t* vbase = p.val_data ? p.val_data + ev : nullptr;
  // lanes per entry from this block's average entry (known after the walk): 8 for C2-like
  // 119-B entries, 16 above 128 B (C5 Zipf keys: 0.96 vs 1.10 ms); p.wj forces 8 or 16.
  // 8 lanes x 5 groups = 40 entries per trip: every C2 block (31-37 entries) in one trip
  // (same-box A/B vs 4 groups: 0.799 -> 0.781 ms)
  const uint32_t avg = (K + V) / n;
  if (p.wj == 16 || (p.wj == 0 && avg > 128))
    copy_entries<16, 2>(p, meta, blk, kbase, vbase, n, en, ek, ev, off, sub, split, mat, view, lane, pre);
  else
    copy_entries<8, 5>(p, meta, blk, kbase, vbase, n, en, ek, ev, off, sub, split, mat, view, lane, pre);
}

// K2: one wave per block (p.wsplit waves above 8 KiB).
__global__ void __launch_bounds__(256) wsc_copy_kernel(DecodeParams p) {
  const uint32_t lane = lane_id();
  // p.wsplit waves share a block (large blocks): wave `sub` takes passes sub, sub + wsplit, ...
  const uint32_t wave = threadIdx.x >> 6, split = p.wsplit;
  const uint32_t sub = wave % split;
  const uint32_t b = uniform(blockIdx.x * (4 / split) + wave / split);
  if (b >= p.nblk) return;
  const uint2* meta = reinterpret_cast<const uint2*>(p.wmeta) + (uint64_t)b * p.wcap;
  const uint64_t* t = p.wstat + 3ull * b;
  const uint32_t n = uniform((uint32_t)t[0]), K = uniform((uint32_t)t[1]),
                 V = uniform((uint32_t)t[2]);
  const uint32_t st = uniform(p.wstatus[b]);
  const uint64_t* bs = p.wbase + 3ull * b;
  const uint64_t en = uniform64(bs[0]), ek = uniform64(bs[1]), ev = uniform64(bs[2]);
  const uint32_t off = uniform(p.blk_off[b]);
  copy_block(p, b, n, K, V, st, en, ek, ev, off, meta, sub, split, lane);
}


hipError_t launch_decode_wsc(const DecodeParams& p, hipStream_t s, hipEvent_t mid) {
  const uint32_t nblk = p.nblk;
  // scan walk: blocks per tile (wlanes: wlanes / 4 per wave) x chunks loaded at once
  if (p.wwalk == kWalkScan && p.wchunks <= 4 && p.wlanes == 64)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkScan, 64, 4>), dim3((nblk + 63) / 64), dim3(256), 0, s, p);
  else if (p.wwalk == kWalkScan && p.wchunks <= 4)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkScan, 16, 4>), dim3((nblk + 15) / 16), dim3(256), 0, s, p);
  else if (p.wwalk == kWalkScan && p.wlanes == 64)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkScan, 64, 16>), dim3((nblk + 63) / 64), dim3(256), 0, s, p);
  else if (p.wwalk == kWalkScan && p.wlanes == 16)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkScan, 16, 16>), dim3((nblk + 15) / 16), dim3(256), 0, s, p);
  else if (p.wwalk == kWalkScan)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkScan, 4, 16>), dim3((nblk + 3) / 4), dim3(256), 0, s, p);
  else if (p.wwalk == kWalkGroup && p.wlanes == 2)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkGroup, 128>), dim3((nblk + 127) / 128), dim3(256), 0, s, p);
  else if (p.wwalk == kWalkGroup && p.wlanes == 4)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkGroup, 64>), dim3((nblk + 63) / 64), dim3(256), 0, s, p);
  else if (p.wwalk == kWalkGroup && p.wlanes == 16)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkGroup, 16>), dim3((nblk + 15) / 16), dim3(256), 0, s, p);
  else if (p.wwalk == kWalkGroup)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkGroup, 32>), dim3((nblk + 31) / 32), dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkLane, 256>), dim3((nblk + 255) / 256), dim3(256), 0, s, p);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && mid) e = hipEventRecord(mid, s);
  if (e != hipSuccess || p.wfuse || (p.wwalk == kWalkScan && p.wcopy))
    return e;  // view-only (wfuse) or scan walk with the copy: the walk kernel wrote everything
  const uint32_t per_wg = 4 / p.wsplit;  // blocks per 4-wave workgroup
  hipLaunchKernelGGL(wsc_copy_kernel, dim3((nblk + per_wg - 1) / per_wg), dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace lsmgpu
