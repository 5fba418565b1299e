// decode_wsc.hip -- "walk, scan, copy" SST block decode: the default path for batches of
// >= 1,024 blocks < 64 KiB (BASELINE C2-C5), plus the fused tile kernel (a forced path).
//
// The serial header chain is walked by ONE LANE PER BLOCK straight from global memory -- 64
// blocks per wave, every block of the batch in flight, each hop one dependent 8-B load -- and
// the bytes are then moved by a separate, fully parallel copy with known output bases:
//   K1 walk_kernel : lane b walks block b exactly like blockIterator.Next/parseKV
//                    (table/iterator.go:93-135), writing per entry a 4-B record {pos | value
//                    offset << 16} (full-line chunks, see flush_meta) and {entries, key
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

// the same with a non-temporal load (the walks' dependent header reads).  Inline asm with the
// wait inside: the value is needed at once anyway, and the compiler does not turn an unaligned
// nontemporal builtin into one dwordx2.  C2 1 GiB, same box: walk 0.288 -> 0.233 ms, view decode
// 0.313 -> 0.270 ms, materialize 0.772 -> 0.737 ms (the copy after it 0.478 -> 0.501 ms).
__device__ __forceinline__ void read_hdr_nt(const uint8_t* g, uint32_t& plen, uint32_t& klen,
                                            uint32_t& vlen) {
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  u32x2 w;
  asm volatile("global_load_dwordx2 %0, %1, off nt\n\ts_waitcnt vmcnt(0)" : "=v"(w) : "v"(g) : "memory");
  plen = __builtin_amdgcn_perm(0u, w.x, 0x0c0c0001u);
  klen = __builtin_amdgcn_perm(0u, w.x, 0x0c0c0203u);
  vlen = __builtin_amdgcn_perm(0u, w.y, 0x0c0c0001u);
}

// the same from a block staged in LDS at byte offset o (any alignment): three aligned dword
// reads and two byte-aligns
[[maybe_unused]] __device__ __forceinline__ void read_hdr_lds(const uint32_t* d, uint32_t o, uint32_t& plen,
                                             uint32_t& klen, uint32_t& vlen) {
  const uint32_t i = o >> 2, sh = o & 3u;
  const uint32_t w0 = d[i], w1 = d[i + 1], w2 = d[i + 2];
  const uint32_t x = __builtin_amdgcn_alignbyte(w1, w0, sh), y = __builtin_amdgcn_alignbyte(w2, w1, sh);
  plen = __builtin_amdgcn_perm(0u, x, 0x0c0c0001u);
  klen = __builtin_amdgcn_perm(0u, x, 0x0c0c0203u);
  vlen = __builtin_amdgcn_perm(0u, y, 0x0c0c0001u);
}

// OR over each aligned group of L (2..16) lanes, every lane of the group receiving it: DPP
// quad_perm [1,0,3,2] and [2,3,0,1], row_half_mirror (lane i <-> 7 - i), row_mirror (i <-> 15 - i)
template <uint32_t L>
__device__ __forceinline__ uint32_t group_or(uint32_t x) {
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0xB1, 0xf, 0xf, true);
  if constexpr (L >= 4) x |= (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x4E, 0xf, 0xf, true);
  if constexpr (L >= 8) x |= (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x141, 0xf, 0xf, true);
  if constexpr (L >= 16) x |= (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x140, 0xf, 0xf, true);
  return x;
}

}  // namespace

// Device-coherent record traffic for the group walk's fused copy (p.wcopyfuse): the records and
// descriptors a walk workgroup writes are read by copy workgroups on other XCDs inside the same
// launch, and the XCDs' L2s are not coherent with each other.  Agent-scope relaxed atomics (sc1)
// write them through and read them past the L2s; an agent-scope release / acquire per tile
// instead writes back / invalidates a whole L2 (measured: C4 0.121 ms against 0.067 for the
// walk and copy launches).
// (Measured and not adopted, so the product library stores the records plainly and never
// fuses the copy: C4 0.081 ms fused against 0.068 ms for the two launches -- every tile of a
// group walk finishes at about the same time, so the copy cannot start much earlier, and the
// copy workgroups slow the walk's dependent rounds; profiles/r06e.)
__device__ __forceinline__ void st_rec4(uint32_t* dst, uint4 v) {  // 16-B aligned
#ifdef LSMGPU_DIAG
  uint64_t* d = reinterpret_cast<uint64_t*>(dst);
  __hip_atomic_store(d, (uint64_t)v.x | ((uint64_t)v.y << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(d + 1, (uint64_t)v.z | ((uint64_t)v.w << 32), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
#else
  *reinterpret_cast<uint4*>(dst) = v;
#endif
}
template <bool COH>
__device__ __forceinline__ uint32_t ldm(const uint32_t* a) {
  if constexpr (COH) return __hip_atomic_load(const_cast<uint32_t*>(a), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *a;
}
template <bool COH>
__device__ __forceinline__ uint4 ld_desc(const uint4* a) {
  if constexpr (COH) {
    uint64_t* d = reinterpret_cast<uint64_t*>(const_cast<uint4*>(a));
    const uint64_t x = __hip_atomic_load(d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t y = __hip_atomic_load(d + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_uint4((uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32));
  } else {
    return *a;
  }
}

// Per-entry metadata of the walk: one u32 record {header pos | value offset << 16} per entry
// (both < 64 KiB in a block < 64 KiB), entry n = the sentinel {stop pos | V << 16}.  The copy
// derives the rest: value length = the next record's value offset minus this one's, stored key
// length = the next header position - this one - 10 - the value length, and (no entry with
// plen > 0, i.e. every block Builder writes) the key offset = pos - 10 e - value offset;
// a block whose K differs from that sum has plen > 0 entries and takes a header-reading path.
// Block b's records are contiguous at b * wcap (wcap a multiple of 32: 128-B aligned chunks of 32
// records).  The walk stages 32 records per block in LDS and writes each chunk as one full
// 128-B line -- 8-B stores straight from 64 lanes at 64 different blocks were evicted from L2 as
// partial lines (4x the bytes).  Round 3: 4-B records instead of {pos | V << 16, K} (8 B).
// The descriptor's status word (wdesc[2b].w) = the block's status | kPlenFlag when the block holds
// prefix-compressed entries (the walk's K exceeds the stored key bytes, stop pos - 10 n - V): the
// copy's header-reading path
constexpr uint32_t kPlenFlag = 1u << 16;  // u32 per lane row: 32 records + 1 pad (bank spread)

// (group walks only: coherent stores, see st_rec4)
__device__ __forceinline__ void flush_meta(uint32_t* dst, const uint32_t* row, uint32_t cnt) {
  if (cnt == 32) {
#pragma unroll
    for (int i = 0; i < 8; i++)
      st_rec4(dst + 4 * i, make_uint4(row[4 * i], row[4 * i + 1], row[4 * i + 2], row[4 * i + 3]));
  } else {
    for (uint32_t i = 0; i < cnt; i++) {
#ifdef LSMGPU_DIAG
      __hip_atomic_store(dst + i, row[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
      dst[i] = row[i];
#endif
    }
  }
}

// kWalkGroupBi (LSMGPU_WSC_BIDIR=1, round 5): the group walk plus a BACKWARD walk of each block,
// in other waves of the workgroup, from the terminator finishBlock writes (builder.go:121-123:
// header {0, 0, 3, prev = the last entry}) over the headers' prev fields (builder.go:95-109),
// so each block's dependent chain is about halved (C4: 23.3 -> 12.4 rounds per block on
// average, 46 -> 25 at most, profiles/r05y).  Waves 0-1 walk 16 blocks forward, 8 lanes each,
// exactly as the group walk; waves 2-3 walk the same blocks backward.  They meet through LDS
// (BiState): the backward waves push each accepted entry (pos | vlen << 16) on the block's
// stack, then publish the stack depth and the lowest entry B; the forward walk accepts only
// entries starting below the B it last read.  A backward entry is accepted only as the forward
// walk would take it: it starts at or above the forward position, has plen 0 and klen > 0, and
// ends exactly where the entry after it starts (the first at the terminator; a guessed one,
// bnext - k * stride, by having the guessed shape).  Once the forward position reaches B it must
// be one of the stacked starts -- then the chains are one (the forward walk from there would
// step through exactly the stacked entries and stop at the terminator) and the stacked entries
// above it become records in forward order; if it is not, the chains disagree and the forward
// walk goes on alone.  (Round 4 ran both directions in the same lanes, and a first round-5
// version in the same wave in lockstep: the rounds halved but each cost twice as much.)
struct BiState {
  uint32_t B;     // lowest published backward entry start (kBiNone: none)
  uint32_t bn;    // entries on the stack (stack[0] the highest)
  uint32_t pos;   // the forward position
  uint32_t done;  // the forward walk has finished, or gone on alone: the backward walk stops
};
constexpr uint32_t kBiNone = 0xffffffffu, kBiCap = 64;
__device__ __forceinline__ uint32_t lds_ld(const uint32_t* a) {
  return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t* a, uint32_t v) {
  __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <uint32_t L>
__device__ __forceinline__ void bidir_bwd(const uint8_t* blk, uint32_t len, uint32_t* bst,
                                          BiState* st, uint32_t k, uint32_t gb, bool b16) {
  constexpr uint64_t kMask = (1ull << L) - 1;
  if (len < 23) return;
  uint32_t tp, tk, tv;
  read_hdr(blk + (len - 13), tp, tk, tv);
  uint32_t bnext;
  __builtin_memcpy(&bnext, blk + (len - 13) + 6, 4);
  bnext = __builtin_bswap32(bnext);
  if ((tp | tk) != 0 || bnext >= len - 13) return;
  uint32_t B = len - 13, bn = 0, bkref = kBiNone, bvref = 0, bstride = 0;
  for (;;) {
    if (lds_ld(&st->done)) break;
    const uint32_t posf = lds_ld(&st->pos);
    if (B <= posf) break;  // the forward walk is here already
    const bool act = (uint64_t)k * bstride <= bnext;
    const uint32_t q = bnext - k * bstride;
    uint32_t plen = 1, klen = 0, vlen = 0, prv = kBiNone;
    if (act && q + 10 <= len && q >= 6 && b16) {
      // one load: the 16 B ending with the header (bytes 6-15: plen, klen, vlen, prev)
      uint4 w;
      __builtin_memcpy(&w, blk + q - 6, 16);
      plen = __builtin_amdgcn_perm(0u, w.y, 0x0c0c0203u);
      klen = __builtin_amdgcn_perm(0u, w.z, 0x0c0c0001u);
      vlen = __builtin_amdgcn_perm(0u, w.z, 0x0c0c0203u);
      prv = __builtin_bswap32(w.w);
    } else if (act && q + 10 <= len) {
      uint2 w;
      __builtin_memcpy(&w, blk + q, 8);
      uint16_t lo;
      __builtin_memcpy(&lo, blk + q + 8, 2);
      plen = __builtin_amdgcn_perm(0u, w.x, 0x0c0c0001u);
      klen = __builtin_amdgcn_perm(0u, w.x, 0x0c0c0203u);
      vlen = __builtin_amdgcn_perm(0u, w.y, 0x0c0c0001u);
      prv = (__builtin_amdgcn_perm(0u, w.y, 0x0c0c0203u) << 16) | bswap16(lo);
    }
    const uint32_t endq = q + 10 + klen + vlen;
    const bool ok = act && q + 10 <= len && q >= posf && plen == 0 && klen != 0 &&
                    (k == 0 ? endq == B : (klen == bkref && vlen == bvref));
    const uint64_t bb = (__ballot(ok) >> gb) & kMask;
    uint32_t cnt = bb == kMask ? L : (uint32_t)__builtin_ctzll(~bb);
    if (bn + cnt > kBiCap) cnt = kBiCap - bn;
    if (cnt == 0) break;
    const uint32_t src = gb + cnt - 1;
    const uint32_t lc = (uint32_t)__shfl((int)q, (int)src), nx = (uint32_t)__shfl((int)prv, (int)src);
    const uint32_t sh0 = (uint32_t)__shfl((int)(klen | (vlen << 16)), (int)gb);
    if (k < cnt) bst[bn + k] = q | (vlen << 16);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // the entries before the depth
    bn += cnt;
    if (k == 0) lds_st(&st->bn, bn);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // the depth before B
    B = lc;
    if (k == 0) lds_st(&st->B, B);
    if (cnt == 1) {  // the guessed shape: lane 0's, unless a run of the old one followed it
      bkref = sh0 & 0xffffu;
      bvref = sh0 >> 16;
      bstride = 10 + bkref + bvref;
    }
    bnext = nx;
    if (bn == kBiCap || bnext >= lc) break;
  }
}

template <uint32_t L>
__device__ __forceinline__ void bidir_fwd(const DecodeParams& p, const uint8_t* blk, uint32_t len,
                                          uint32_t* meta, uint32_t* row, const uint32_t* bst,
                                          BiState* st, uint32_t k, uint32_t gb, uint32_t& pos,
                                          uint32_t& gn, uint32_t& gK, uint32_t& gV, uint32_t& gst) {
  constexpr uint64_t kMask = (1ull << L) - 1;
  constexpr uint32_t kGroupProbe = 16;
  uint32_t kref = kBiNone, vref = 0, stride = 0, rounds = 0, depth = 0;
  bool alone = false, met = false;
  for (;;) {
    uint32_t Bc = alone ? kBiNone : lds_ld(&st->B);
    if (Bc != kBiNone && pos >= Bc) {
      // the forward position must be one of the stacked starts (stack[0] the highest)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      const uint32_t nb = lds_ld(&st->bn);
      uint32_t hit = kBiNone;
      for (uint32_t i = k; i < nb; i += L)
        if ((bst[i] & 0xffffu) == pos) hit = i;
      const uint64_t hm = (__ballot(hit != kBiNone) >> gb) & kMask;
      if (hm) {
        depth = (uint32_t)__shfl((int)hit, (int)(gb + __builtin_ctzll(hm))) + 1;
        met = true;
        break;
      }
      alone = true;  // the chains disagree: the forward walk alone from here
      if (k == 0) lds_st(&st->done, 1);
      Bc = kBiNone;
    }
    const uint32_t q = pos + k * stride;
    uint32_t plen = 1, klen = 0, vlen = 0;
    if (q + 10 <= len) read_hdr(blk + q, plen, klen, vlen);
    const uint32_t endq = q + 10 + klen + vlen;
    const bool fast = (klen != 0) & (plen == 0) & (endq <= len) & (q < Bc);
    const bool same = fast & (klen == kref) & (vlen == vref);
    const uint64_t fb = (__ballot(fast) >> gb) & kMask, sb = (__ballot(same) >> gb) & kMask;
    if (!(fb & 1)) break;  // entry n needs the general loop (or the block ended)
    const uint32_t t = sb == kMask ? L : (uint32_t)__builtin_ctzll(~sb);
    const uint32_t m = t + ((t < L && ((fb >> t) & 1u)) ? 1u : 0u);
    const uint32_t rec = q | ((gV + k * vref) << 16);
    const uint32_t idx = gn + k, cend = (gn | 31u) + 1;
    const bool acc = k < m;
    if (acc && idx < cend) row[idx & 31] = rec;
    const uint32_t src = gb + m - 1;
    pos = (uint32_t)__shfl((int)endq, (int)src);
    const uint32_t shape = (uint32_t)__shfl((int)(klen | (vlen << 16)), (int)src);
    if (k == 0) lds_st(&st->pos, pos);
    gK += t * kref + (m > t ? (shape & 0xffffu) : 0u);
    gV += t * vref + (m > t ? (shape >> 16) : 0u);
    gn += m;
    if (t == 0) {
      kref = shape & 0xffffu;
      vref = shape >> 16;
      stride = 10 + kref + vref;
    }
    rounds++;
    if (gn >= cend) {  // chunk [cend - 32, cend) complete: one full 128-B line
      __builtin_amdgcn_wave_barrier();
      st_rec4(meta + cend - 32 + 4 * k,
              make_uint4(row[4 * k], row[4 * k + 1], row[4 * k + 2], row[4 * k + 3]));
      __builtin_amdgcn_wave_barrier();  // the chunk is read before the next one fills
      if (acc && idx >= cend) row[idx & 31] = rec;
    }
    if (rounds >= kGroupProbe && 4 * gn < 5 * rounds && lds_ld(&st->bn) < 8) break;
  }
  if (k == 0) lds_st(&st->done, 1);
#ifdef LSMGPU_STAMPS
  if (p.stamps && k == 0) {  // diagnostics: forward rounds per block, blocks whose chains met
    atomicAdd(reinterpret_cast<unsigned long long*>(p.stamps + 8), (unsigned long long)rounds);
    atomicMax(reinterpret_cast<unsigned long long*>(p.stamps + 9), (unsigned long long)rounds);
    atomicAdd(reinterpret_cast<unsigned long long*>(p.stamps + 10), 1ull);
    atomicAdd(reinterpret_cast<unsigned long long*>(p.stamps + 11), met ? 1ull : 0ull);
  }
#endif
  if (met) {
    // the stacked entries stack[depth - 1] (at pos) .. stack[0] in forward order, L per trip
    // through the record ring: value offsets by a scan of their value lengths, key lengths from
    // the next entry's start (stack[i - 1], the terminator above stack[0])
    for (uint32_t i0 = 0; i0 < depth; i0 += L) {
      const uint32_t i = i0 + k;
      const bool on = i < depth;
      const uint32_t si = depth - 1 - i;
      const uint32_t sv = on ? bst[si] : 0u;
      const uint32_t nxt = on ? (si ? (bst[si - 1] & 0xffffu) : len - 13) : 0u;
      const uint32_t pe = sv & 0xffffu, vl = sv >> 16;
      const uint32_t kl = on ? nxt - pe - 10 - vl : 0u;
      uint32_t x = vl, y = kl;  // inclusive scans over the group
#pragma unroll
      for (uint32_t d = 1; d < L; d <<= 1) {
        const uint32_t xv = (uint32_t)__shfl_up((int)x, d, L), yv = (uint32_t)__shfl_up((int)y, d, L);
        if (k >= d) {
          x += xv;
          y += yv;
        }
      }
      const uint32_t rec = pe | ((gV + x - vl) << 16);
      const uint32_t mc = min(L, depth - i0);
      const uint32_t idx = gn + k, cend = (gn | 31u) + 1;
      if (on && idx < cend) row[idx & 31] = rec;
      gV += (uint32_t)__shfl((int)x, (int)(gb + mc - 1));
      gK += (uint32_t)__shfl((int)y, (int)(gb + mc - 1));
      gn += mc;
      if (gn >= cend) {
        __builtin_amdgcn_wave_barrier();
        st_rec4(meta + cend - 32 + 4 * k,
                make_uint4(row[4 * k], row[4 * k + 1], row[4 * k + 2], row[4 * k + 3]));
        __builtin_amdgcn_wave_barrier();
        if (on && idx >= cend) row[idx & 31] = rec;
      }
    }
    pos = len - 13;  // at the terminator, where the forward walk stops (iterator.go:124-127)
    return;
  }
  if (k == 0) {  // general loop: every stop rule in the iterator's order (as the group walk)
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
      row[gn & 31] = pos | (gV << 16);
      if ((gn & 31) == 31) flush_meta(meta + (gn - 31), row, 32);
      gK += plen + klen;
      gV += vlen;
      gn++;
      pos = end;
    }
  }
  (void)p;
}

// Where the copy reads a block's bytes: global memory (the copy kernel), or the walk's LDS slot
// holding the block at byte sh (the 64-lane staged walk copying its own block, p.wscopy).
// piece(dst, s0, len, q) = copy_piece16(dst, block + s0, len, q).
struct GlobalBytes {
  const uint8_t* b;
  __device__ __forceinline__ void piece(uint8_t* dst, uint32_t s0, uint32_t len, uint32_t q) const {
    copy_piece16(dst, b + s0, len, q);
  }
};
struct LdsBytes {
  const uint8_t* l;
  uint32_t sh;
  __device__ __forceinline__ void piece(uint8_t* dst, uint32_t s0, uint32_t len, uint32_t q) const {
    const uint32_t a = sh + s0;
    if (len >= 16) {
      const uint32_t o = min(16 * q, len - 16);
      const uint4 v = lds_u128(l, a + o);
      __builtin_memcpy(dst + o, &v, 16);
    } else if (len >= 8) {
      const uint32_t o = q ? len - 8 : 0;
      const uint2 v = make_uint2(lds_u32(l, a + o), lds_u32(l, a + o + 4));
      __builtin_memcpy(dst + o, &v, 8);
    } else if (len >= 4) {
      const uint32_t o = q ? len - 4 : 0;
      const uint32_t v = lds_u32(l, a + o);
      __builtin_memcpy(dst + o, &v, 4);
    } else {
      dst[q] = l[a + q];
    }
  }
};

template <typename Src, bool COH = false>  // COH: records read with coherent loads (ldm)
__device__ __forceinline__ void copy_block(const DecodeParams& p, uint32_t b, const uint32_t* meta,
                                           uint32_t pre, uint32_t n, uint32_t K, uint32_t V,
                                           uint32_t sw, uint64_t en, uint64_t ek, uint64_t ev,
                                           uint32_t off, uint32_t sub, uint32_t split,
                                           uint32_t lane, const Src& src, uint32_t* tab = nullptr,
                                           bool duties = true, uint8_t* mk = nullptr);

// A copy workgroup inside a group walk's launch (p.wcopyfuse): copier c of ncop takes 4-wave
// groups of blocks c, c + ncop, ... (p.wsplit waves per block, as wsc_copy_kernel) and copies
// each block once the walk workgroup of its tile has published the tile's descriptors (granule
// 7 of the tile record = the launch tag, stored once every record and descriptor store of the
// tile -- coherent stores, st_rec4 -- has completed).  Copiers exist only past the last walk ticket, so every tile they wait for
// is already being walked by a running workgroup: no deadlock, whatever the residency.
__device__ __forceinline__ void fused_copier(const DecodeParams& p, uint32_t c, uint32_t ncop,
                                          uint32_t tb);

// K1: lane = block; a workgroup = a tile of 256 consecutive blocks, tiles taken in ticket order
// (p.gcnt[0]).  After the walk the workgroup scans its blocks' {entries, key bytes, value
// bytes}, publishes the tile aggregate and finds the tile's output base by decoupled look-back
// over the tile records (epoch-tagged granules in p.lb), then writes every block's exclusive
// base: the output bases are known when the walk ends, with no separate scan launch.  The
// ticket makes every predecessor tile already running, so the look-back always progresses.
// MODE kWalkGroup (p.wwalk, the default when nblk <= 64 per CU: the lane walk would leave the
// machine idle): 256 / TB lanes per block guess same-shape runs (see the branch).
// MODE kWalkLane: lane b walks block b straight from HBM, one dependent 8-B non-temporal header
// load per entry (every 128-B line of the input is fetched on its own, as scattered requests);
// the records leave in whole 128-B lines written by 8 lanes each.
// CH (lane walk): records per flushed chunk -- 32 (whole 128-B lines) or 16 (64-B halves: half
// the LDS, twice the workgroups per CU)
// MODE kWalkLaneView (view-only decodes, round 4): the lane walk keeping each block's first
// kViewRec records in its LDS row for the whole kernel -- no flush during the walk, no re-read:
// after the look-back each wave writes its 64 blocks' view records from LDS (records past
// kViewRec, rare, go to / come from p.wmeta)
// SLOT: the staged walk's LDS bytes per block
// WIDE (TB = 576, lane walks): 9-wave workgroups of 576 blocks, 2 per CU = 1,152 blocks per CU in
// flight, against 4 x 256 = 1,024 for TB = 256 (LDS-bound: 33 words per lane).  (384-block tiles,
// 51 KB, are not 3 per CU: walk 0.267 ms, profiles/r05e -- as if a workgroup's LDS had to lie in
// one 80 KB half of the CU's 160 KB, which also fits round 4's census of 3 x 54 KB.)  C2 at 2^30 B has
// 266,403 blocks: 1,041 tiles of 256 for 1,024 resident slots, and the 17-tile second wave cost
// the walk 0.030 ms and the view decode 0.045 ms (same-box A/B, profiles/r05c); 463 tiles of 576
// are all resident.  WIDE keeps no per-lane tables besides the rows (no s_first / s_off).
// Diagnostic build only (LSMGPU_BUILD_DIAG=1, run with LSMGPU_STAMPS=1): per tile, the
// s_memrealtime (100 MHz) of its start, its walk's end (every wave), its look-back's end and its
// epilogue's end (wave 0), written to p.stamps[16 + 4 tile ..] and summarized by the host.
#ifdef LSMGPU_STAMPS
#define WSC_STAMP(slot, v)                                                                  \
  do {                                                                                      \
    if (p.stamps && tid == 0) p.stamps[16 + (uint64_t)tile * 4 + (slot)] = (v);             \
  } while (0)
#else
#define WSC_STAMP(slot, v) \
  do {                     \
  } while (0)
#endif

template <int MODE, uint32_t TB, uint32_t CH = 32, uint32_t SLOT = kStageSlot>  // TB = blocks per tile
__global__ void __launch_bounds__(MODE == kWalkGroup || MODE == kWalkGroupBi || TB <= 256 ? 256 : TB)
    wsc_walk_kernel(DecodeParams p) {
  // group walks: kWalkGroup, or kWalkGroupBi (a second lane group per block walks backward)
  constexpr bool GW = MODE == kWalkGroup || MODE == kWalkGroupBi;
  constexpr bool BI = MODE == kWalkGroupBi;
  constexpr bool WIDE = !GW && TB > 256;
  static_assert(TB <= 256 || (WIDE && TB <= 1024 && CH == 32), "one thread per block of the tile");
  static_assert(CH == 16 || CH == 32, "16 or 32 records per chunk");
  constexpr bool KEEP = MODE == kWalkLaneView;
  // lane walks: one thread per block, TB = 192, 256 or 576 threads; the group walk: 256 threads
  constexpr uint32_t kThreads = GW ? 256 : TB;
  constexpr uint32_t kWaves = kThreads / 64;
  static_assert(kThreads % 64 == 0, "whole waves");
  // LDS row per lane: CH records (+ 1 pad, bank spread), or kViewRec kept records (+ 1; WIDE:
  // none, the 33-word stride is odd already)
  // kept records per block: 41 for the 576-block tiles (one workgroup per CU whatever their LDS;
  // C2: 23 % of blocks have 33-37 entries and spilled to p.wmeta with 33), 33 for 256-block tiles
  // (4 per CU)
  constexpr uint32_t kRec = WIDE ? 41u : kViewRec;
  constexpr uint32_t kStage = KEEP ? (WIDE ? kRec : kRec + 1) : CH + 1;
  constexpr uint32_t kStageBytes = kThreads * kStage * sizeof(uint32_t);
  // group walk: a 32-record ring per block (the walk's LDS also serves the view epilogue's
  // owner map)
  // group walk of 64 lanes (TB = 4, one wave per block): the wave first copies its block into an
  // LDS slot with every load in flight, then walks it there (kStaged; blocks too long for a
  // slot walk from global memory)
  // (SLOT = 0: the 64-lane walk reads global memory; its round is all scalar -- ballots,
  // s_ff1, v_readlane -- instead of the narrower groups' LDS lane shuffles)
  constexpr bool kWave64 = MODE == kWalkGroup && TB == 4;
  constexpr bool kStaged = kWave64 && SLOT > 0;
  constexpr uint32_t kSlot = kStaged ? SLOT : 0u;
  static_assert(SLOT % 16 == 0, "16-B chunks (0: no staging)");
  constexpr uint32_t kLdsBytes =
      GW ? TB * 32 * sizeof(uint32_t) + TB * kSlot : kStageBytes;
  static_assert(GW || kLdsBytes == kStageBytes,
                "the lane walk stages its records per lane");
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
  uint32_t* const stage = reinterpret_cast<uint32_t*>(lds);
  __shared__ uint32_t s_tile;
  __shared__ uint32_t s_wave[kWaves][3];
  __shared__ uint32_t s_ex[3];
  __shared__ uint32_t s_part[kWaves][3];  // p.wlbfull: each wave's share of the predecessors' sums
  __shared__ uint32_t s_first[KEEP || WIDE ? 1 : kThreads + 1];  // p.wfuse: tile-relative first entry
  // each block's input offset (group walks; the lane walk's non-kept view epilogue)
  __shared__ uint32_t s_off[GW ? TB : (KEEP || WIDE ? 1 : kThreads)];
  constexpr uint32_t kRes = GW ? TB : 1;
  // kWalkGroupBi: each block's backward-walked entries (pos | vlen << 16), lowest last, and
  // the state the forward and backward waves share
  __shared__ uint32_t s_bstack[BI ? TB : 1][BI ? kBiCap : 1];
  __shared__ BiState s_bi[BI ? TB : 1];
  __shared__ uint32_t s_res[4][kRes];  // group / wave walk: n, K, V, status per block
  __shared__ uint32_t s_stg[kRes];  // group walk: the block is in its LDS slot (kStaged)
  __shared__ uint32_t s_cb[3][kWave64 ? TB : 1];  // p.wscopy: each block's output bases
  __shared__ uint8_t s_mark[KEEP || !GW ? kWaves : 1][128];  // kWalkLaneView, p.wview: owner marks (lane + 1)
  // the staged walk copying its own blocks (p.wscopy): no records for a copy launch
  const bool scopy = kWave64 && LSMGPU_KNOB(p.wscopy, 0u) && !p.wfuse;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  // blocks per tile: TB, or for the wide lane walks p.wtbe <= TB (threads past it hold no block):
  // tiles sized so the two waves of tiles (one workgroup per CU) carry equal shares
  const uint32_t TBe = WIDE && p.wtbe ? p.wtbe : TB;
  const uint32_t ntiles = (p.nblk + TBe - 1) / TBe;
#ifdef LSMGPU_STAMPS
  const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
  // group walks with the copy fused (p.wcopyfuse): gridDim.x = tiles + copiers
  const bool fcopy = GW && !kWave64 && LSMGPU_KNOB(p.wcopyfuse, 0u) && !p.wfuse;  // (diag)
  const uint32_t draws = fcopy ? gridDim.x : ntiles;
  if (tid == 0) {
    const uint32_t t = atomicAdd(p.gcnt, 1u);
    if (t == draws - 1) atomicExch(p.gcnt, 0u);  // every ticket is taken
    s_tile = t;
  }
  __syncthreads();
  const uint32_t tile = s_tile;
  if constexpr (GW && !kWave64) {
    if (fcopy && tile >= ntiles) {  // (uniform) a copy workgroup
      fused_copier(p, tile - ntiles, draws - ntiles, TB);
      return;
    }
  }
#ifdef LSMGPU_STAMPS
  WSC_STAMP(0, t_start);
#endif
  // the result block is zeroed by the workgroup holding ticket 0 (see api.hip), before anything
  // else: every other tile's look-back ends only on a record chained to tile 0's, so no flag
  // (the look-back timeout, result[5] |= 2) can be set before this and then erased
  if (p.zero_result && tile == 0 && tid < 8)
    atomicExch(reinterpret_cast<unsigned long long*>(p.result + tid), 0ull);
  // thread t owns block tile * TBe + t (threads past TBe own none: zero entries)
  const uint32_t b = tid < TBe ? tile * TBe + tid : 0xffffffffu;
  uint32_t n = 0, K = 0, V = 0, st = LSMGPU_BLK_OK;
  uint32_t lane_off = 0;  // lane walks: this thread's block offset
  bool plen_b = false;    // lane walks: the block holds prefix-compressed entries
  if constexpr (GW) {
    // L lanes per block: each round the group reads the headers at pos + k * stride (stride =
    // the last accepted entry's size) and accepts the leading run whose guesses were right --
    // lane k is entry n + k iff entries n .. n + k - 1 all had the previous entry's shape.  The
    // guessed lines belong to the next entries of the same block (no extra traffic), the group
    // fetches neighbouring lines together, and the dependent chain shrinks by the run length.
    // (kWalkGroupBi: waves 0-1 walk the tile's 16 blocks forward, 8 lanes each, as below; waves
    // 2-3 the same blocks backward: bidir_fwd / bidir_bwd)
    constexpr uint32_t L = BI ? 128 / TB : 256 / TB;  // lanes per block (per direction)
    constexpr uint32_t LB = L;
    static_assert((BI ? 2 : 1) * L * TB == 256, "one tile of blocks per 256-thread workgroup");
    static_assert(L >= 2 && L <= 64 && (L & (L - 1)) == 0, "2..64 lanes per block");
    constexpr uint64_t kMask = L == 64 ? ~0ull : (1ull << (L & 63)) - 1;
    constexpr uint32_t kGroupProbe = 16;
    const uint32_t g = BI ? (tid & 127) / L : tid / L, k = tid & (L - 1), gb = lane & ~(L - 1);
    const uint32_t kk = k;
    const bool bw = BI && tid >= 128;  // a backward lane (waves 2-3)
    if constexpr (BI) {
      if (tid < TB) s_bi[tid] = BiState{kBiNone, 0u, 0u, 0u};
      __syncthreads();
    }
    const uint32_t bg = tile * TB + g;
    uint32_t* row = stage + g * 32;  // the block's current 32-record chunk (one 128-B line)
    if (bg < p.nblk) {
      const uint32_t off = p.blk_off[bg], len = p.blk_len[bg];
      uint32_t* meta = p.wmeta + (uint64_t)bg * p.wcap;
      uint32_t pos = 0, gn = 0, gK = 0, gV = 0, gst = LSMGPU_BLK_OK;
      bool staged = false;
      if ((uint64_t)off + len > p.data_len) {
        gst = LSMGPU_BLK_RANGE;
      } else if ABLATE(p, 4) {  // (timing-only ablation: no walk, every block empty)
      } else {
        const uint8_t* blk = p.data + off;
        // kStaged: the block's bytes [off, off + len) as (unaligned) 16-B chunks in the wave's
        // slot, header q at byte q.  Nothing before off is read: the host pipeline's data
        // pointer is biased (only [chunk start, data_len) is readable); a chunk past data_len
        // loads byte by byte.
        const uint32_t sh = 0;
        staged = kStaged && len + 16 <= kSlot;
        const uint32_t* sd = reinterpret_cast<const uint32_t*>(lds + TB * 32 * sizeof(uint32_t) + g * kSlot);
        if constexpr (kStaged) {
          if (staged) {
            const uint64_t a0 = off;
            const uint32_t n16 = (len + 15) >> 4;
            const uint8_t* src = p.data + a0;
            uint4* dst = reinterpret_cast<uint4*>(lds + TB * 32 * sizeof(uint32_t) + g * kSlot);
            for (uint32_t c0 = 0; c0 < n16; c0 += 8 * L) {
              uint4 v[8];
#pragma unroll
              for (uint32_t u = 0; u < 8; u++) {
                const uint32_t c = c0 + u * L + k;
                v[u] = make_uint4(0, 0, 0, 0);
                if (c < n16) {
                  if (a0 + 16ull * c + 16 <= p.data_len) {
                    __builtin_memcpy(&v[u], src + 16 * c, 16);
                  } else {  // the input's last partial chunk
                    uint8_t t[16] = {};
                    for (uint32_t j = 0; j < 16 && a0 + 16ull * c + j < p.data_len; j++) t[j] = src[16 * c + j];
                    __builtin_memcpy(&v[u], t, 16);
                  }
                }
              }
#pragma unroll
              for (uint32_t u = 0; u < 8; u++)
                if (c0 + u * L + k < n16) dst[c0 + u * L + k] = v[u];
            }
            wave_lds_fence();
          }
        }
        if constexpr (BI) {
          if (bw) bidir_bwd<L>(blk, len, s_bstack[g], &s_bi[g], k, gb, LSMGPU_KNOB(p.wb16, 0u) != 0);
          else bidir_fwd<L>(p, blk, len, meta, row, s_bstack[g], &s_bi[g], k, gb, pos, gn, gK, gV, gst);
        } else {
        uint32_t kref = 0xffffffffu, vref = 0, stride = 0;  // no shape yet: round 1 takes one
        uint32_t rounds = 0;
        // p.wsub: a round is a window of L entries; after an odd-shaped entry only the lanes
        // past the accepted ones guess again (sub-round), from the corrected position -- their
        // guesses move by the odd entry's size difference, so the lines are already in L1 --
        // and a new window (new lines) starts once all L lanes are accepted.  Lane k guesses
        // window entry j = k - a (lanes below a idle).
        uint32_t a = 0;
        for (;;) {
          const bool act = k >= a;
          const uint32_t j = k - a;
          const uint32_t q = pos + j * stride;  // < 2^24 for active lanes: stride < 2^17, j < 64
          uint32_t plen = 1, klen = 0, vlen = 0;
          // default loads here: the copy after a small batch re-reads the lines from the
          // Infinity Cache (nt guesses: C4 walk 0.038 -> 0.043 ms, copy 0.032 -> 0.042 ms)
          if (act && q + 10 <= len) {
            if (staged) read_hdr_lds(sd, sh + q, plen, klen, vlen);
            else read_hdr(blk + q, plen, klen, vlen);
          }
          const uint32_t endq = q + 10 + klen + vlen;
          const bool fast = (klen != 0) & (plen == 0) & (endq <= len);
          const bool same = fast & (klen == kref) & (vlen == vref);
          const uint64_t wm = kMask >> a;  // the window's remaining lanes
          const uint32_t La = L - a;
          const uint64_t fb = (__ballot(fast) >> (gb + a)) & wm;
          const uint64_t sb = (__ballot(same) >> (gb + a)) & wm;
          if (!(fb & 1u)) break;  // entry n itself needs the general loop (or the block ended)
          uint32_t t = sb == wm ? La : (uint32_t)__builtin_ctzll(~sb);  // leading same-shape run
          uint32_t m = t + ((t < La && ((fb >> t) & 1u)) ? 1u : 0u);  // + one new shape
          const uint32_t rec = q | ((gV + j * vref) << 16);
          const uint32_t idx = gn + j, cend = (gn | 31u) + 1;  // end of the current chunk
          // 64 lanes: the run may cross one chunk boundary but must not complete the next chunk
          // too (only the chunk ending at cend is flushed below)
          if (L > 32 && gn + m >= cend + 32) {
            m = cend + 31 - gn;
            t = min(t, m);
          }
          const bool acc = act && j < m;  // this lane's entry is accepted
          if (acc && idx < cend) row[idx & 31] = rec;
          const uint32_t src = gb + a + m - 1;  // the last accepted entry
          uint32_t shape;
          if constexpr (L == 64) {  // src is wave-uniform (from ballots)
            pos = __builtin_amdgcn_readlane(endq, src);
            shape = __builtin_amdgcn_readlane(klen | (vlen << 16), src);
          } else if (L <= 16 && LSMGPU_KNOB(p.wdpp, 0u)) {
            // the group's OR of the one lane's values by DPP (quad swaps, half-row / row
            // mirrors) -- no LDS round trip on the round's dependent chain
            const bool me = k == src - gb;
            pos = group_or<L>(me ? endq : 0u);
            shape = group_or<L>(me ? (klen | (vlen << 16)) : 0u);
          } else {
            pos = (uint32_t)__shfl((int)endq, (int)src);
            shape = (uint32_t)__shfl((int)(klen | (vlen << 16)), (int)src);
          }
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
          if (gn >= cend) {  // chunk [cend - 32, cend) complete: one full 128-B line
            __builtin_amdgcn_wave_barrier();
            for (uint32_t i = k; i < 8; i += L)
              st_rec4(meta + cend - 32 + 4 * i,
                      make_uint4(row[4 * i], row[4 * i + 1], row[4 * i + 2], row[4 * i + 3]));
            __builtin_amdgcn_wave_barrier();  // the chunk is read before the next one fills
            if (acc && idx >= cend) row[idx & 31] = rec;
          }
          if (LSMGPU_KNOB(p.wsub, 0u)) {
            a += m;
            if (a >= L) a = 0;
          }
          // shapes do not repeat in this block (< 1.25 entries per round after 16 rounds): the
          // rest entry by entry.  A rate over many rounds, not a streak -- with thousands of
          // blocks some block always starts unluckily, and the slowest block sets the kernel's
          // time (C4 shapes, simulated: 2 per round after 8 rounds gives up on 13 % of blocks)
          if (rounds >= kGroupProbe && 4 * gn < 5 * rounds) break;
        }
#ifdef LSMGPU_STAMPS
        if (p.stamps && k == 0) {  // diagnostics: rounds per block
          atomicAdd(reinterpret_cast<unsigned long long*>(p.stamps + 8), (unsigned long long)rounds);
          atomicMax(reinterpret_cast<unsigned long long*>(p.stamps + 9), (unsigned long long)rounds);
          atomicAdd(reinterpret_cast<unsigned long long*>(p.stamps + 10), 1ull);
        }
#endif
        if (k == 0) {  // general loop: every stop rule in the iterator's order (as the lane walk)
          for (;;) {
            if (pos >= len) break;                                   // iterator.go:115-118
            if (len - pos < 10) { gst = LSMGPU_BLK_TRUNC_HEADER; break; }
            uint32_t plen, klen, vlen;
            if (staged) read_hdr_lds(sd, sh + pos, plen, klen, vlen);  // iterator.go:121
            else read_hdr(blk + pos, plen, klen, vlen);
            if ((klen | plen) == 0) break;                           // iterator.go:124-127
            if (gn == 0 && plen != 0) { gst = LSMGPU_BLK_FIRST_PLEN; break; }  // :129-133
            if (10 + plen > len) { gst = LSMGPU_BLK_PREFIX_OOB; break; }
            const uint32_t end = pos + 10 + klen + vlen;             // iterator.go:101-109
            if (end > len) { gst = LSMGPU_BLK_VALUE_OVERFLOW; break; }
            row[gn & 31] = pos | (gV << 16);
            if ((gn & 31) == 31) flush_meta(meta + (gn - 31), row, 32);
            gK += plen + klen;
            gV += vlen;
            gn++;
            pos = end;
          }
        }
        }  // !BI
      }
      // the last chunk (the sentinel last) as whole 16-B parts of its 128-B line, by the group's
      // L lanes (the general loop ran in lane 0: its count is the group's)
      if (!bw) {  // (kWalkGroupBi: the forward lanes hold the block's results)
      const uint32_t gbl = lane & ~(LB - 1);  // the block's first lane (forward lane 0)
      if (kk == 0) row[gn & 31] = pos | (gV << 16);  // sentinel
      const uint32_t gnl = (uint32_t)__shfl((int)gn, (int)gbl);
      wave_lds_fence();
      for (uint32_t i = kk; i < 8; i += LB)
        st_rec4(meta + (gnl & ~31u) + 4 * i,
                make_uint4(row[4 * i], row[4 * i + 1], row[4 * i + 2], row[4 * i + 3]));
      if (kk == 0) {
        s_res[0][g] = gn;
        s_res[1][g] = gK;
        s_res[2][g] = gV;
        // + kPlenFlag: the block holds prefix-compressed entries (K exceeds the stored key bytes)
        s_res[3][g] = gst | (gK != pos - 10 * gn - gV ? kPlenFlag : 0u);
        s_off[g] = off;
        s_stg[g] = staged;
      }
      }  // !bw
    }
    __syncthreads();
    if (b < p.nblk) {  // from here on thread t owns block tile * TB + t, as in the other walks
      n = s_res[0][tid];
      K = s_res[1][tid];
      V = s_res[2][tid];
      const uint32_t sw = s_res[3][tid];
      st = sw & ~kPlenFlag;
    }
  } else {
    // Lane walk, records flushed cooperatively: every lane walks in lockstep (a lane that
    // stopped idles), so after iteration k with k % 32 == 31 every lane still walking holds
    // records k-31 .. k in its LDS row; the wave then writes those rows as whole 128-B lines,
    // 8 lanes per line -- 8 lines per store instruction instead of 64 partial ones (C2 1 GiB,
    // same box: walk 0.233 -> 0.222 ms, view decode 0.271 -> 0.261 ms).
    const bool valid = b < p.nblk;
    uint32_t* row = stage + tid * kStage;
    uint32_t off = 0, len = 0, pos = 0;
    if (valid) {
      off = p.blk_off[b];
      len = p.blk_len[b];
      if constexpr (!KEEP && !WIDE) s_off[tid] = off;  // the non-kept view epilogue's table
      lane_off = off;
    }
    bool done = !valid || ABLATE(p, 4);  // (timing-only ablation 4: no walk)
    if (valid && (uint64_t)off + len > p.data_len) {
      st = LSMGPU_BLK_RANGE;
      done = true;
    }
    const uint8_t* blk = p.data + off;
    const uint32_t wb0 = tile * TBe + wave * 64;  // the block of this wave's lane 0
    for (uint32_t k = 0;; k++) {
      if (__ballot(!done) == 0) break;
      bool rec = false;
      if (!done) {
        do {
          if (pos >= len) { done = true; break; }                  // iterator.go:115-118
          if (len - pos < 10) { st = LSMGPU_BLK_TRUNC_HEADER; done = true; break; }
          uint32_t plen, klen, vlen;
          read_hdr_nt(blk + pos, plen, klen, vlen);                // iterator.go:121
          if ((klen | plen) == 0) { done = true; break; }          // iterator.go:124-127
          if (n == 0 && plen != 0) { st = LSMGPU_BLK_FIRST_PLEN; done = true; break; }
          if (10 + plen > len) { st = LSMGPU_BLK_PREFIX_OOB; done = true; break; }
          const uint32_t end = pos + 10 + klen + vlen;             // iterator.go:101-109
          if (end > len) { st = LSMGPU_BLK_VALUE_OVERFLOW; done = true; break; }
          if constexpr (KEEP) {
            if (n < kRec) row[n] = pos | (V << 16);
            else p.wmeta[(uint64_t)b * p.wcap + n] = pos | (V << 16);
          } else {
            row[n & (CH - 1)] = pos | (V << 16);
          }
          K += plen + klen;
          V += vlen;
          n++;
          pos = end;
          rec = true;
        } while (false);
      }
      // (timing-only ablation 128: no record flush; honoured only with ablation 2, under which
      // the copy reads no record -- a copy of stale records writes out of bounds)
      if (!KEEP && (k & (CH - 1)) == CH - 1 && ABLATE(p, 130) != 130) {
        const uint64_t fl = __ballot(rec);  // lanes holding records k-CH+1 .. k
        if (fl) {
          wave_lds_fence();
          constexpr uint32_t kPer = CH / 4;  // lanes per row: one 16-B part each
#pragma unroll
          for (uint32_t r = 0; r < kPer; r++) {
            const uint32_t L = (64 / kPer) * r + lane / kPer, part = lane % kPer;
            if ((fl >> L) & 1ull) {
              const uint32_t* rw = stage + (wave * 64 + L) * kStage + 4 * part;
              uint32_t* mL = p.wmeta + (uint64_t)(wb0 + L) * p.wcap + (k - (CH - 1));
              reinterpret_cast<uint4*>(mL)[part] = make_uint4(rw[0], rw[1], rw[2], rw[3]);
            }
          }
          wave_lds_fence();
        }
      }
    }
    // the last chunk (records n & ~31 .. n, the sentinel last) of every block, cooperatively as
    // well: whole 128-B lines (the slot holds wcap records, a multiple of 32; words past the
    // sentinel are never read)
    if constexpr (KEEP) {  // the sentinel; the rows stay in LDS
      if (valid) {
        if (n < kRec) row[n] = pos | (V << 16);
        else p.wmeta[(uint64_t)b * p.wcap + n] = pos | (V << 16);
      }
    }
    if (valid && !KEEP) row[n & (CH - 1)] = pos | (V << 16);
    const uint64_t vm = KEEP || ABLATE(p, 258) == 258 ? 0ull : __ballot(valid);  // (ablation 256: as 128)
    if (!KEEP) wave_lds_fence();
    constexpr uint32_t kPer = CH / 4;
#pragma unroll
    for (uint32_t r = 0; r < (KEEP ? 0u : kPer); r++) {
      const uint32_t L = (64 / kPer) * r + lane / kPer, part = lane % kPer;
      const uint32_t nL = (uint32_t)__shfl((int)n, (int)L);
      if ((vm >> L) & 1ull) {
        const uint32_t* rw = stage + (wave * 64 + L) * kStage + 4 * part;
        uint32_t* mL = p.wmeta + (uint64_t)(wb0 + L) * p.wcap + (nL & ~(CH - 1));
        reinterpret_cast<uint4*>(mL)[part] = make_uint4(rw[0], rw[1], rw[2], rw[3]);
      }
    }
    if (valid && !KEEP) plen_b = K != pos - 10 * n - V;  // see kPlenFlag
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
  WSC_STAMP(1, __builtin_amdgcn_s_memrealtime());
  if (LSMGPU_KNOB(p.wlbfull, 1u)) {
    // every tile publishes its aggregate; every thread sums some predecessors' (lookback_partial)
    uint32_t tn = 0, tk = 0, tv = 0;
    for (uint32_t w = 0; w < kWaves; w++) {
      tn = sat_add(tn, s_wave[w][0]);
      tk = sat_add(tk, s_wave[w][1]);
      tv = sat_add(tv, s_wave[w][2]);
    }
    uint64_t* R = p.lb + (uint64_t)tile * 8;
    if (wave == 0) store3(R, p.tag, tn, tk, tv, lane);
    Tot part{0, 0, 0};
    if (tile > 0 && !ABLATE(p, 1)) part = lookback_partial(p.lb, tile, p.tag, tid, kThreads, p.result);
    const uint32_t pn = wave_sum_sat(part.n), pk = wave_sum_sat(part.k), pv = wave_sum_sat(part.v);
    if (lane == 0) {
      s_part[wave][0] = pn;
      s_part[wave][1] = pk;
      s_part[wave][2] = pv;
    }
    __syncthreads();
    if (wave == 0) {
      Tot ex{0, 0, 0};
      for (uint32_t w = 0; w < kWaves; w++) {
        ex.n = sat_add(ex.n, s_part[w][0]);
        ex.k = sat_add(ex.k, s_part[w][1]);
        ex.v = sat_add(ex.v, s_part[w][2]);
      }
      if (lane == 0) {
        s_ex[0] = ex.n;
        s_ex[1] = ex.k;
        s_ex[2] = ex.v;
      }
    }
  } else if (wave == 0) {
    uint32_t tn = 0, tk = 0, tv = 0;
    for (uint32_t w = 0; w < kWaves; w++) {
      tn = sat_add(tn, s_wave[w][0]);
      tk = sat_add(tk, s_wave[w][1]);
      tv = sat_add(tv, s_wave[w][2]);
    }
    uint64_t* R = p.lb + (uint64_t)tile * 8;
    Tot ex{0, 0, 0};
    if (tile > 0 && !ABLATE(p, 1)) {  // (timing-only ablation 1: no look-back)
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
  WSC_STAMP(2, __builtin_amdgcn_s_memrealtime());
  uint32_t en_b = 0;  // this thread's block's first entry (kWalkLaneView's view loop)
  uint32_t ek_b = 0, ev_b = 0;  // and its key / value stream bases (p.weo)
  const uint32_t off_b = !GW ? lane_off : 0u;
  if (b < p.nblk) {
    uint32_t on = s_ex[0], ok = s_ex[1], ov = s_ex[2];
    for (uint32_t w = 0; w < wave; w++) {
      on = sat_add(on, s_wave[w][0]);
      ok = sat_add(ok, s_wave[w][1]);
      ov = sat_add(ov, s_wave[w][2]);
    }
    const uint32_t en = sat_add(on, in_ - n), ek = sat_add(ok, ik == 0xffffffffu ? ik : ik - K),
                   ev = sat_add(ov, iv - V);
    en_b = en;
    ek_b = ek;
    ev_b = ev;
    if (scopy) {
      s_cb[0][tid] = en;
      s_cb[1][tid] = ek;
      s_cb[2][tid] = ev;
    } else {
      if (!p.wfuse) {  // the copy kernel's descriptor
        uint32_t swb, offb;
        if constexpr (GW) {
          swb = s_res[3][tid];
          offb = s_off[tid];
        } else {
          swb = st | (plen_b ? kPlenFlag : 0u);
          offb = lane_off;
        }
        if (fcopy) {  // read by copy workgroups of this launch (st_rec4)
          st_rec4(reinterpret_cast<uint32_t*>(p.wdesc + 2ull * b), make_uint4(n, K, V, swb));
          st_rec4(reinterpret_cast<uint32_t*>(p.wdesc + 2ull * b + 1), make_uint4(en, ek, ev, offb));
        } else {
          p.wdesc[2ull * b] = make_uint4(n, K, V, swb);
          p.wdesc[2ull * b + 1] = make_uint4(en, ek, ev, offb);
        }
      }
      // The per-block outputs, here for every decode (round 5; view-only decodes have no copy):
      // one thread per block writes consecutive words -- from the copy kernel, one lane per
      // block, they were scattered 4-B stores into lines shared by workgroups on other XCDs
      // (C2 copy 0.50 -> 0.465 ms without them, profiles/r05s)
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
      bool fits = (uint64_t)en + n <= p.ent_cap && (uint64_t)en + n <= 0xffffffffull;
      if (!p.wfuse && (p.mode & LSMGPU_MODE_MATERIALIZE)) {  // the copy's output streams
        const uint64_t kend = (uint64_t)ek + K, vend = (uint64_t)ev + V;
        fits = fits && (kend <= p.key_cap || !p.key_data) && (vend <= p.val_cap || !p.val_data) &&
               kend < 0xffffffffull && vend <= 0xffffffffull;
      }
      if (!fits) atomicOr(reinterpret_cast<unsigned long long*>(p.result + 5), 1ull);
    }
  }
  if (!p.wfuse) {
    if constexpr (kWave64) {
      // the 64-lane walk's copy (p.wscopy): wave w copies block tile * 4 + w from its LDS slot
      // (its records were flushed to p.wmeta by this wave), so the input is read once and no
      // copy launch follows
      if (scopy) {
        __syncthreads();  // the bases (s_cb); the records in p.wmeta (workgroup scope)
        const uint32_t bw = tile * TB + wave;
        if (bw < p.nblk) {
          const uint32_t* meta = p.wmeta + (uint64_t)bw * p.wcap;
          const uint32_t pre = meta[min(lane, p.wcap - 1)];
          const uint32_t off = s_off[wave];
          const uint32_t nw = s_res[0][wave], Kw = s_res[1][wave], Vw = s_res[2][wave],
                         sw = s_res[3][wave];
          const uint64_t enw = s_cb[0][wave], ekw = s_cb[1][wave], evw = s_cb[2][wave];
          if (kStaged && s_stg[wave])
            copy_block(p, bw, meta, pre, nw, Kw, Vw, sw, enw, ekw, evw, off, 0, 1, lane,
                       LdsBytes{lds + TB * 32 * sizeof(uint32_t) + wave * kSlot, 0u});
          else
            copy_block(p, bw, meta, pre, nw, Kw, Vw, sw, enw, ekw, evw, off, 0, 1, lane,
                       GlobalBytes{p.data + off});
        }
      }
    }
    if constexpr (!GW && !KEEP) {
      // p.weo (lane walks, materialize): the per-entry outputs -- key_end, val_end and the view
      // records -- written here, each wave its 64 blocks' entries (consecutive in the output),
      // one lane per entry, from the records this wave flushed (L2-hot).  From the copy kernel
      // (entry_outputs) the 68 MB cost 0.044 ms of C2's copy (profiles/r05r): its stores start
      // at every block's first entry, into lines shared with blocks copied on other XCDs.
      // Blocks with prefix-compressed entries keep them in the copy (copy_entries_plen).
      if (LSMGPU_KNOB(p.weo, 0u) && (p.mode & LSMGPU_MODE_MATERIALIZE)) {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // this wave's record flushes
        __builtin_amdgcn_wave_barrier();
        const bool valid = b < p.nblk;
        const uint32_t wb0 = tile * TBe + wave * 64;
        const uint32_t pw = in_ - n;  // wave-exclusive first entry of this lane's block
        const uint32_t T = __builtin_amdgcn_readlane(in_, 63);  // the wave's entries
        const uint64_t ew = __builtin_amdgcn_readlane(en_b, 0);  // the wave's first output entry
        const bool view = (p.mode & LSMGPU_MODE_VIEW) && p.view;
        auto emit = [&](uint32_t f, uint32_t L) {
          const uint32_t pL = (uint32_t)__shfl((int)pw, (int)L), nL = (uint32_t)__shfl((int)n, (int)L);
          const uint32_t ekL = (uint32_t)__shfl((int)ek_b, (int)L), evL = (uint32_t)__shfl((int)ev_b, (int)L);
          const uint32_t offL = (uint32_t)__shfl((int)off_b, (int)L);
          const uint32_t plL = (uint32_t)__shfl((int)(plen_b ? 1u : 0u), (int)L);
          if (f >= T || plL) return;
          const uint64_t bend = ew + pL + nL;
          if (!(bend <= p.ent_cap && bend <= 0xffffffffull)) return;  // reported (result[5])
          const uint32_t e = f - pL;
          const uint32_t* meta = p.wmeta + (uint64_t)(wb0 + L) * p.wcap;
          const uint32_t m0 = meta[e], m1 = meta[e + 1];
          const uint32_t hp1 = m1 & 0xffffu, vo1 = m1 >> 16;
          if (p.key_end) p.key_end[ew + f] = ekL + hp1 - 10 * (e + 1) - vo1;
          if (p.val_end) p.val_end[ew + f] = evL + vo1;
          if (view) {
            const uint32_t hp = m0 & 0xffffu, vl = vo1 - (m0 >> 16), kl = hp1 - hp - 10 - vl;
            p.view[ew + f] = (uint64_t)(offL + hp + 10) | ((uint64_t)kl << 32) | ((uint64_t)vl << 48);
          }
        };
        // owners by one scatter and a max-scan (as the view epilogue below), 128 entries a trip
        uint8_t* const mk = s_mark[wave];
        mk[lane] = 0;
        mk[64 + lane] = 0;
        wave_lds_fence();
        uint32_t carry = 0;
        for (uint32_t c0 = 0; c0 < T; c0 += 128) {
          if (valid && n > 0 && pw >= c0 && pw < c0 + 128) mk[pw - c0] = lane + 1;
          wave_lds_fence();
          const uint32_t a0 = mk[lane], a1 = mk[64 + lane];
          mk[lane] = 0;
          mk[64 + lane] = 0;
          const uint32_t v0 = max(wave_scan_max(a0, lane), carry);
          const uint32_t v1 = max(wave_scan_max(a1, lane), __builtin_amdgcn_readlane(v0, 63));
          carry = __builtin_amdgcn_readlane(v1, 63);
          wave_lds_fence();
          emit(c0 + lane, v0 - 1);
          emit(c0 + 64 + lane, v1 - 1);
        }
      }
    }
    if constexpr (GW && !kWave64) {
      if (fcopy) {  // the tile's descriptors and records are complete: release them to the copiers
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // every wave's stores complete
        __syncthreads();
        if (tid == 0)  // (every record / descriptor store was coherent and has completed)
          __hip_atomic_store(p.lb + (uint64_t)tile * 8 + 7, (uint64_t)p.tag, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    WSC_STAMP(3, __builtin_amdgcn_s_memrealtime());
    return;
  }
  if constexpr (KEEP) {
    if (!((p.mode & LSMGPU_MODE_VIEW) && p.view) || ABLATE(p, 2)) return;  // mode 0: no view
    // each wave writes its 64 blocks' records -- consecutive in the output -- one lane per
    // entry, 64 consecutive 8-B records per store instruction, from the rows its lanes filled
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // rows (and any spill) written
    __builtin_amdgcn_wave_barrier();
    const uint32_t wb0 = tile * TBe + wave * 64;
    const uint32_t pw = in_ - n;  // wave-exclusive first entry of this lane's block
    const uint32_t T = __builtin_amdgcn_readlane(in_, 63);  // the wave's entries (no saturation:
                                                           // <= 64 x 6,554)
    const uint64_t ew = __builtin_amdgcn_readlane(en_b, 0);  // the wave's first output entry
    // entry f of the wave (owner lane L): its 8-B view record from L's LDS row (or the spill)
    auto emit = [&](uint32_t f, uint32_t L) {
      const uint32_t pL = (uint32_t)__shfl((int)pw, (int)L), nL = (uint32_t)__shfl((int)n, (int)L);
      const uint32_t offL = (uint32_t)__shfl((int)off_b, (int)L);
      if (f >= T) return;
      const uint64_t bend = ew + pL + nL;
      if (!(bend <= p.ent_cap && bend <= 0xffffffffull)) return;  // reported (result[5])
      const uint32_t e = f - pL;
      const uint32_t* rw = stage + (wave * 64 + L) * kStage;
      const uint32_t* gl = p.wmeta + (uint64_t)(wb0 + L) * p.wcap;
      const uint32_t m0 = e < kRec ? rw[e] : gl[e];
      const uint32_t m1 = e + 1 < kRec ? rw[e + 1] : gl[e + 1];
      const uint32_t hp = m0 & 0xffffu, vl = (m1 >> 16) - (m0 >> 16);
      const uint32_t kl = (m1 & 0xffffu) - hp - 10 - vl;  // stored key bytes
      p.view[ew + f] = (uint64_t)(offL + hp + 10) | ((uint64_t)kl << 32) | ((uint64_t)vl << 48);
    };
    if (LSMGPU_KNOB(p.wview, 1u)) {
      // owners by one scatter and a max-scan, two passes (128 entries) per trip: every block
      // with entries marks (lane + 1) at its first entry's slot, a DPP max-scan carries the
      // marks forward (the previous pass's last owner carried in)
      uint8_t* const mk = s_mark[KEEP ? wave : 0];
      mk[lane] = 0;
      mk[64 + lane] = 0;
      wave_lds_fence();
      uint32_t carry = 0;
      for (uint32_t c0 = 0; c0 < T; c0 += 128) {
        if (n > 0 && pw >= c0 && pw < c0 + 128) mk[pw - c0] = lane + 1;
        wave_lds_fence();
        const uint32_t a0 = mk[lane], a1 = mk[64 + lane];
        mk[lane] = 0;  // for the next trip (this lane read its slots above)
        mk[64 + lane] = 0;
        const uint32_t v0 = max(wave_scan_max(a0, lane), carry);
        const uint32_t v1 = max(wave_scan_max(a1, lane), __builtin_amdgcn_readlane(v0, 63));
        carry = __builtin_amdgcn_readlane(v1, 63);
        wave_lds_fence();
        emit(c0 + lane, v0 - 1);
        emit(c0 + 64 + lane, v1 - 1);
      }
    } else {
      // the owner of entry f: the last block L whose wave-exclusive first entry (pw, lane L) is
      // <= f (6 lane-shuffle steps)
      for (uint32_t c0 = 0; c0 < T; c0 += 64) {
        const uint32_t f = c0 + lane;
        uint32_t L = 0;
#pragma unroll
        for (uint32_t st = 32; st >= 1; st >>= 1) {
          const uint32_t cand = L + st;
          const uint32_t pc = (uint32_t)__shfl((int)pw, (int)min(cand, 63u));
          if (cand < 64 && pc <= f) L = cand;
        }
        emit(f, L);
      }
    }
    WSC_STAMP(3, __builtin_amdgcn_s_memrealtime());
    return;
  }
  if constexpr (WIDE) return;  // (never launched with the non-kept view epilogue below)
  // View-only decode (p.wfuse): the workgroup writes its tile's dense view records itself, so
  // no copy launch follows.  Output entry e of the tile belongs to the last block whose first
  // entry is <= e (binary search over s_first); its record comes from the walk metadata this
  // workgroup just wrote (L2-hot), and consecutive threads write consecutive 8-B records.
  {
    uint32_t rel = in_ - n;  // entries of the tile never saturate (<= 256 x 6,554)
    for (uint32_t w = 0; w < wave; w++) rel += s_wave[w][0];
    s_first[tid] = rel;
    if (tid == kThreads - 1) s_first[kThreads] = rel + n;
  }
  __syncthreads();
  if (!((p.mode & LSMGPU_MODE_VIEW) && p.view) || ABLATE(p, 2)) return;  // mode 0: no view
  const uint32_t nt = s_first[kThreads];
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
  // 4 entries per thread per trip, every record load issued before any view store (the
  // compiler keeps a load behind an earlier store it cannot prove apart)
  constexpr uint32_t kVB = 4;
  for (uint32_t eb = tid; eb < nt; eb += kThreads * kVB) {
    uint32_t m0[kVB], m1[kVB], lo[kVB];
    bool on[kVB];
#pragma unroll
    for (uint32_t u = 0; u < kVB; u++) {
      const uint32_t e = eb + kThreads * u;
      uint32_t l = 0, hi = kThreads - 1;
      if (e < nt) {
        if (mapped) {
          l = owner[e];
        } else {
          while (l < hi) {
            const uint32_t mid = (l + hi + 1) >> 1;
            if (s_first[mid] <= e) l = mid; else hi = mid - 1;
          }
        }
      }
      lo[u] = l;
      const uint64_t bend = e0 + s_first[l + 1];
      on[u] = e < nt && bend <= p.ent_cap && bend <= 0xffffffffull;  // else reported (result[5])
      const uint32_t i = on[u] ? e - s_first[l] : 0u;
      const uint32_t* meta = p.wmeta + (uint64_t)(tile * TB + l) * p.wcap;
      m0[u] = meta[i];
      m1[u] = meta[i + 1];
    }
#pragma unroll
    for (uint32_t u = 0; u < kVB; u++) {
      if (!on[u]) continue;
      const uint32_t hp = m0[u] & 0xffffu, vl = (m1[u] >> 16) - (m0[u] >> 16);
      const uint32_t kl = (m1[u] & 0xffffu) - hp - 10 - vl;  // stored key bytes
      p.view[e0 + eb + kThreads * u] =
          (uint64_t)(s_off[lo[u]] + hp + 10) | ((uint64_t)kl << 32) | ((uint64_t)vl << 48);
    }
  }
}

// The entries of one block with no prefix-compressed entry: J lanes per entry; an entry's
// pieces are [key pieces | value pieces] (16 B, the last overlapping back inside its stream, or
// two overlapping 8/4/2/1-B pieces below 16 B) and lane j takes pieces j, j + J, ...  G entry
// groups per pass, all metadata loads issued first.  Key offset of entry e = pos - 10 e - value
// offset (every earlier entry contributed its 10-B header, its stored key and its value).
// The per-entry outputs of a block with no prefix-compressed entry -- key_end, val_end and the
// view records -- with one lane per entry, 64 consecutive entries per store instruction (the
// copy's J-lane entry groups wrote 8 consecutive words per instruction: C2 1 GiB, that cost
// 0.06 ms of the copy's 0.51).  Wave `sub` of `split` takes chunks sub, sub + split, ...
template <bool COH>
__device__ __forceinline__ void entry_outputs(const DecodeParams& p, const uint32_t* meta,
                                              uint32_t n, uint64_t en, uint64_t ek, uint64_t ev,
                                              uint32_t off, uint32_t sub, uint32_t split,
                                              bool mat, bool view, uint32_t lane, uint32_t pre) {
  for (uint32_t c0 = sub * kWave; c0 < n; c0 += split * kWave) {
    const uint32_t e = c0 + lane;
    const uint32_t m0 = c0 == 0 ? pre : ldm<COH>(meta + min(e, n));
    const uint32_t nx = (uint32_t)__shfl((int)m0, (int)min(lane + 1, kWave - 1));
    const uint32_t m1 = lane + 1 < kWave ? nx : ldm<COH>(meta + min(e + 1, n));
    if (e >= n) continue;
    const uint32_t hp = m0 & 0xffffu, vo = m0 >> 16, hp1 = m1 & 0xffffu, vo1 = m1 >> 16;
    const uint32_t vl = vo1 - vo, kl = hp1 - hp - 10 - vl;
    if (mat) {
      if (p.key_end) p.key_end[en + e] = (uint32_t)(ek + hp1 - 10 * (e + 1) - vo1);
      if (p.val_end) p.val_end[en + e] = (uint32_t)(ev + vo1);
    }
    if (view) p.view[en + e] = (uint64_t)(off + hp + 10) | ((uint64_t)kl << 32) | ((uint64_t)vl << 48);
  }
}

template <uint32_t J, uint32_t G, bool EO, typename Src, bool COH = false>  // EO: also the per-entry outputs
__device__ __forceinline__ void copy_entries(const DecodeParams& p, const uint32_t* meta,
                                             const Src& blk, uint8_t* kbase, uint8_t* vbase,
                                             uint32_t n, uint64_t en, uint64_t ek, uint64_t ev,
                                             uint32_t off, uint32_t sub, uint32_t split,
                                             bool mat, bool view, uint32_t lane, uint32_t pre) {
  const uint32_t j = lane & (J - 1);
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
      uint32_t m0, m1;
      if (shuffled) {
        m0 = (uint32_t)__shfl((int)pre, (int)ec);
        m1 = (uint32_t)__shfl((int)pre, (int)ec + 1);
      } else {
        m0 = ldm<COH>(meta + ec);
        m1 = ldm<COH>(meta + ec + 1);
      }
      hp[i] = m0 & 0xffffu;
      vo[i] = m0 >> 16;
      const uint32_t hp1 = m1 & 0xffffu, vo1 = m1 >> 16;
      vl[i] = vo1 - vo[i];
      kl[i] = hp1 - hp[i] - 10 - vl[i];  // stored key bytes
      ko[i] = hp[i] - 10 * ec - vo[i];
      const uint32_t ko1 = ko[i] + kl[i];
      on[i] = e < n;
      kp[i] = pieces16(kl[i]);
      np[i] = kp[i] + pieces16(vl[i]);
      if (EO && on[i] && j == 0) {
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
        blk.piece(dst + (key ? ko[i] : vo[i]), s0, len, key ? q : q - kp[i]);
      }
    }
  }
}

// Aligned output chunks (round 5).  The copy's unaligned, overlapping 16-B pieces reach L2 as
// ~54-B write requests (19.9 M per C2 1 GiB copy vs 8.4 M 128-B ones for a streaming copy of the
// same bytes, profiles/r05g); written as aligned 16-B chunks, every store instruction covers
// whole lines (per-block probe, scripts/align_probe.hip: 0.41-0.44 vs 0.49-0.56 ms).  A stream
// (keys or values) of a block starts at address B and holds S bytes; its 16-B grid starts at u0
// (B + u0 aligned) and has nfull whole chunks [u0 + 16 i, +16) ending at gend.  Entry e holds
// stream bytes [so_e, so_e1) from block byte src_e on; the lanes of e's group write the chunks
// that START inside [so_e, so_e1) -- no search, as the pieces do -- loading 16 bytes from e's
// source and, when the chunk runs into the next entries, 16 more from each, starting k bytes
// before that entry's first byte (k = bytes taken so far), merged under byte masks.  Loads stay
// in the block: from e at offset >= 0, from later entries at most 15 bytes before their first
// byte (their header and key precede it), never past a whole chunk's last byte.  The bytes before
// u0 and from gend on share their chunks with the neighbouring blocks' streams: one lane a byte.
__device__ __forceinline__ uint32_t bytes_below(uint32_t k, uint32_t d) {  // mask of dword d's bytes < k
  const int32_t t = (int32_t)k - 4 * (int32_t)d;
  return t >= 4 ? 0xffffffffu : t <= 0 ? 0u : (1u << (8 * t)) - 1u;
}
__device__ __forceinline__ uint32_t grid0(const uint8_t* B, uint32_t S) {
  return min((uint32_t)((16u - ((uintptr_t)B & 15u)) & 15u), S);
}
// stream position and source of entry e from its record and the next one (no prefix-compressed
// entry: the key offset is pos - 10 e - value offset)
struct StreamPos {
  uint32_t so, so1, src;
};
__device__ __forceinline__ StreamPos stream_pos(bool key, uint32_t e, uint32_t m0, uint32_t m1) {
  const uint32_t hp = m0 & 0xffffu, vo = m0 >> 16, hp1 = m1 & 0xffffu, vo1 = m1 >> 16;
  const uint32_t vl = vo1 - vo, kl = hp1 - hp - 10 - vl;
  if (key) {
    const uint32_t ko = hp - 10 * e - vo;
    return StreamPos{ko, ko + kl, hp + 10};
  }
  return StreamPos{vo, vo1, hp + 10 + kl};
}
__device__ __forceinline__ uint4 merge_from(uint4 w, uint4 w2, uint32_t k) {  // bytes >= k from w2
  w.x = (w.x & bytes_below(k, 0)) | (w2.x & ~bytes_below(k, 0));
  w.y = (w.y & bytes_below(k, 1)) | (w2.y & ~bytes_below(k, 1));
  w.z = (w.z & bytes_below(k, 2)) | (w2.z & ~bytes_below(k, 2));
  w.w = (w.w & bytes_below(k, 3)) | (w2.w & ~bytes_below(k, 3));
  return w;
}
// the whole chunk of stream positions [g, g + 16), its first bytes from entry e (records m0, m1;
// m2 = record e + 2): both loads are issued before either is used; a chunk running past entry
// e + 1 (entries < 16 B) takes the rest entry by entry
__device__ __forceinline__ void chunk_out(bool key, uint8_t* B, uint32_t g, uint32_t e, uint32_t m1,
                                          uint32_t m2, const StreamPos& sp, const uint32_t* meta,
                                          const uint8_t* blk) {
  uint4 w;
  __builtin_memcpy(&w, blk + sp.src + (g - sp.so), 16);
  uint32_t k = sp.so1 - g;
  if (k < 16u) {
    const StreamPos fp = stream_pos(key, e + 1, m1, m2);
    uint4 w2;
    __builtin_memcpy(&w2, blk + fp.src - k, 16);
    w = merge_from(w, w2, k);
    k = fp.so1 - g;
    uint32_t f = e + 2, mf = m2;
    while (k < 16u) {  // rare
      const uint32_t mf1 = meta[f + 1];
      const StreamPos hp = stream_pos(key, f, mf, mf1);
      __builtin_memcpy(&w2, blk + hp.src - k, 16);
      w = merge_from(w, w2, k);
      k = hp.so1 - g;
      f++;
      mf = mf1;
    }
  }
  *reinterpret_cast<uint4*>(B + g) = w;
}
// the chunk starts of [so, so1) on the grid (u0, gend): the first and the count
__device__ __forceinline__ void chunk_starts(uint32_t so, uint32_t so1, uint32_t u0, uint32_t gend,
                                             uint32_t& g0, uint32_t& nc) {
  g0 = so <= u0 ? u0 : u0 + ((so - u0 + 15u) & ~15u);
  const uint32_t hi = min(so1, gend);
  nc = g0 < hi ? (hi - g0 + 15u) >> 4 : 0u;
}

// The bytes of both streams outside their whole chunks (< 16 before u0, < 16 from gend on): lanes
// 0-15 the key stream's head, 16-31 its tail, 32-47 / 48-63 the value stream's.  The byte is
// loaded here (before the chunks) and stored by store_edge after them.  Usually the head lies in
// entry 0 and the tail in entry n - 1 (records from `pre` when n < 64); else the entry is found by
// stepping through the records.
struct EdgeByte {
  uint8_t* dst;
  uint32_t v;
};
__device__ __forceinline__ EdgeByte load_edge(const uint32_t* meta, const uint8_t* blk, uint8_t* kbase,
                                              uint8_t* vbase, uint32_t n, uint32_t K, uint32_t V,
                                              uint32_t lane, uint32_t pre) {
  const bool key = lane < 32, tail = (lane & 16) != 0;
  // records 0, 1 and n - 1, n (uniform shuffles: every lane takes part)
  const uint32_t r0 = (uint32_t)__shfl((int)pre, 0), r1 = (uint32_t)__shfl((int)pre, 1);
  uint32_t rl0, rl1;
  if (n < kWave) {
    rl0 = (uint32_t)__shfl((int)pre, (int)n - 1);
    rl1 = (uint32_t)__shfl((int)pre, (int)n);
  } else {
    rl0 = meta[n - 1];
    rl1 = meta[n];
  }
  uint8_t* B = key ? kbase : vbase;
  const uint32_t S = key ? K : V;
  if (!B || S == 0) return EdgeByte{nullptr, 0};
  const uint32_t u0 = grid0(B, S), gend = u0 + ((S - u0) & ~15u);
  const uint32_t q = tail ? gend + (lane & 15) : (lane & 15);
  if (tail ? q >= S : q >= u0) return EdgeByte{nullptr, 0};
  uint32_t e = tail ? n - 1 : 0;
  StreamPos sp = tail ? stream_pos(key, e, rl0, rl1) : stream_pos(key, 0, r0, r1);
  if (tail) {
    while (sp.so > q || sp.so1 <= q) {  // (empty entries: so == so1)
      e--;
      sp = stream_pos(key, e, meta[e], meta[e + 1]);
    }
  } else {
    while (sp.so1 <= q) {
      e++;
      sp = stream_pos(key, e, meta[e], meta[e + 1]);
    }
  }
  return EdgeByte{B + q, blk[sp.src + (q - sp.so)]};
}

template <uint32_t J, uint32_t G>
__device__ __forceinline__ void copy_entries_aligned(const uint32_t* meta, const uint8_t* blk,
                                                     uint8_t* kbase, uint8_t* vbase, uint32_t n,
                                                     uint32_t K, uint32_t V, uint32_t sub,
                                                     uint32_t split, uint32_t lane, uint32_t pre) {
  const uint32_t j = lane & (J - 1);
  const EdgeByte eb = load_edge(meta, blk, kbase, vbase, n, K, V, lane, pre);
  const uint32_t ku0 = kbase ? grid0(kbase, K) : 0u, vu0 = vbase ? grid0(vbase, V) : 0u;
  const uint32_t kend = kbase ? ku0 + ((K - ku0) & ~15u) : 0u;  // no key chunks without kbase
  const uint32_t vend = vbase ? vu0 + ((V - vu0) & ~15u) : 0u;
  for (uint32_t e0 = sub * G * (kWave / J); e0 < n; e0 += split * G * (kWave / J)) {
    // records e, e + 1, e + 2 by lane shuffle while e + 2 < 64 (`pre` holds records 0 .. 63)
    const bool shuffled = e0 + G * (kWave / J) + 1 < kWave;
#pragma unroll 1
    for (int i = 0; i < (int)G; i++) {
      const uint32_t e = e0 + i * (kWave / J) + (lane / J);
      const uint32_t ec = min(e, n - 1);
      uint32_t m0, m1, m2;
      if (shuffled) {
        m0 = (uint32_t)__shfl((int)pre, (int)ec);
        m1 = (uint32_t)__shfl((int)pre, (int)ec + 1);
        m2 = (uint32_t)__shfl((int)pre, (int)min(ec + 2, n));
      } else {
        m0 = meta[ec];
        m1 = meta[ec + 1];
        m2 = meta[min(ec + 2, n)];
      }
      if (e >= n) continue;
      const StreamPos kp = stream_pos(true, e, m0, m1), vp = stream_pos(false, e, m0, m1);
      uint32_t kg, nkc, vg, nvc;
      chunk_starts(kp.so, kp.so1, ku0, kend, kg, nkc);
      chunk_starts(vp.so, vp.so1, vu0, vend, vg, nvc);
      for (uint32_t q = j; q < nkc + nvc; q += J) {
        if (q < nkc) chunk_out(true, kbase, kg + 16 * q, e, m1, m2, kp, meta, blk);
        else chunk_out(false, vbase, vg + 16 * (q - nkc), e, m1, m2, vp, meta, blk);
      }
    }
  }
  if (eb.dst) *eb.dst = (uint8_t)eb.v;
}

// Dense aligned output chunks (LSMGPU_WSC_ALIGN=2, blocks of <= 63 entries whose two streams
// span <= kChunkOwn chunks): the key and value streams of the block as ALIGNED 16-B chunks over
// one combined chunk index (key chunks, then value chunks), 64 consecutive chunks per store
// instruction.  Each entry lane publishes its stream ends and input bases in LDS and marks the
// chunks whose first byte it holds (an LDS owner table); a chunk lane loads 16 B from its owner
// and 16 more from each following entry it runs into, merged under byte masks (input byte of
// stream byte x in entry e: D_e + x, so a later entry's load starts < 16 B before its first
// byte: its own header / key, inside the block).  A stream's partial head and tail chunks
// (shared with the neighbouring blocks' streams) are stored as naturally aligned 8/4/2/1-B parts.
constexpr uint32_t kChunkOwn = 512;  // owner-table bytes per wave
constexpr uint32_t kChunkLds = 4 * 64 + kChunkOwn / 4;  // u32 per wave: so1 / D per stream + owners

__device__ __forceinline__ uint32_t bytes_from(uint32_t k, uint32_t d) {  // dword d's bytes >= k
  const int32_t t = (int32_t)k - 4 * (int32_t)d;
  return t <= 0 ? 0xffffffffu : t >= 4 ? 0u : ~((1u << (8 * t)) - 1u);
}
// 16 bytes at block byte q; past `lim` (the readable end) bytes are zero (the batch's last block)
__device__ __forceinline__ uint4 load16_lim(const uint8_t* blk, uint32_t q, uint32_t lim) {
  uint4 v;
  if (q + 16 <= lim) {
    __builtin_memcpy(&v, blk + q, 16);
  } else {
    v = make_uint4(0, 0, 0, 0);
    for (uint32_t i = 0; i < 16 && q + i < lim; i++) set_byte(v, (int)i, blk[q + i]);
  }
  return v;
}
// the first len (< 16) bytes of v at d as naturally aligned 8/4/2/1-B stores
__device__ __forceinline__ void store_head(uint8_t* d, uint4 v, uint32_t len) {
  uint32_t s = 0;
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  while (len) {
    const uintptr_t a = (uintptr_t)d;
    uint32_t sz = 8;
    while (sz > len || (a & (sz - 1))) sz >>= 1;
    uint64_t x = 0;
    for (uint32_t i = 0; i < sz; i++)
      x |= (uint64_t)((w[(s + i) >> 2] >> (8 * ((s + i) & 3))) & 0xffu) << (8 * i);
    if (sz == 8) *reinterpret_cast<uint64_t*>(d) = x;
    else if (sz == 4) *reinterpret_cast<uint32_t*>(d) = (uint32_t)x;
    else if (sz == 2) *reinterpret_cast<uint16_t*>(d) = (uint16_t)x;
    else *d = (uint8_t)x;
    d += sz;
    s += sz;
    len -= sz;
  }
}
__device__ __forceinline__ bool chunks_fit(const uint8_t* kbase, const uint8_t* vbase, uint32_t K, uint32_t V) {
  const uint32_t ak = (uint32_t)((uintptr_t)kbase & 15u), av = (uint32_t)((uintptr_t)vbase & 15u);
  return (kbase ? (K + ak + 15) >> 4 : 0u) + (vbase ? (V + av + 15) >> 4 : 0u) <= kChunkOwn;
}
__device__ __forceinline__ void copy_chunks(const uint8_t* blk, uint32_t lim, uint8_t* kbase,
                                            uint8_t* vbase, uint32_t n, uint32_t K, uint32_t V,
                                            uint32_t lane, uint32_t pre, uint32_t* tab) {
  uint32_t* const so1 = tab;            // [2][64]: key / value stream end of entry e
  uint32_t* const dd = tab + 128;       // [2][64]: input base D_e of each stream
  uint8_t* const own = reinterpret_cast<uint8_t*>(tab + 256);
  const uint32_t ak = kbase ? (uint32_t)((uintptr_t)kbase & 15u) : 0u;
  const uint32_t av = vbase ? (uint32_t)((uintptr_t)vbase & 15u) : 0u;
  const uint32_t CK = kbase ? (K + ak + 15) >> 4 : 0u, CV = vbase ? (V + av + 15) >> 4 : 0u;
  const uint32_t m0 = pre, m1 = (uint32_t)__shfl((int)pre, (int)min(lane + 1, kWave - 1));
  const uint32_t hp = m0 & 0xffffu, vo = m0 >> 16, hp1 = m1 & 0xffffu, vo1 = m1 >> 16;
  const uint32_t vl = vo1 - vo, kl = hp1 - hp - 10 - vl, ko = hp - 10 * lane - vo, ko1 = ko + kl;
  if (lane < n) {
    so1[lane] = ko1;
    dd[lane] = hp + 10 - ko;
    so1[64 + lane] = vo1;
    dd[64 + lane] = hp1 - vo1;
    // chunk c >= 1 of a stream starts at stream byte 16 c - a, chunk 0 at byte 0
    if (CK) {
      const uint32_t lo = ko == 0 ? 0u : (ko + ak + 15) >> 4, hi = kl ? (ko1 + ak + 15) >> 4 : lo;
      for (uint32_t c = lo; c < hi; c++) own[c] = (uint8_t)lane;
    }
    if (CV) {
      const uint32_t lo = vo == 0 ? 0u : (vo + av + 15) >> 4, hi = vl ? (vo1 + av + 15) >> 4 : lo;
      for (uint32_t c = lo; c < hi; c++) own[CK + c] = (uint8_t)lane;
    }
  }
  wave_lds_fence();
  for (uint32_t c = lane; c < CK + CV; c += kWave) {
    const bool key = c < CK;
    const uint32_t cc = key ? c : c - CK, a = key ? ak : av, S = key ? K : V, s = key ? 0u : 64u;
    const uint32_t x0 = cc ? 16 * cc - a : 0u;           // the chunk's first stream byte
    const uint32_t L = min(cc ? 16u : 16u - a, S - x0);  // and its byte count
    uint32_t e = own[c];
    uint4 v = load16_lim(blk, dd[s + e] + x0, lim);
    uint32_t k = so1[s + e] - x0;
    while (k < L) {  // the chunk runs into entry e + 1
      e++;
      const uint4 w = load16_lim(blk, dd[s + e] + x0, lim);
      v.x = (v.x & ~bytes_from(k, 0)) | (w.x & bytes_from(k, 0));
      v.y = (v.y & ~bytes_from(k, 1)) | (w.y & bytes_from(k, 1));
      v.z = (v.z & ~bytes_from(k, 2)) | (w.z & bytes_from(k, 2));
      v.w = (v.w & ~bytes_from(k, 3)) | (w.w & bytes_from(k, 3));
      k = so1[s + e] - x0;
    }
    uint8_t* d = (key ? kbase : vbase) + x0;
    if (L == 16) *reinterpret_cast<uint4*>(d) = v;
    else store_head(d, v, L);
  }
}

// A block with prefix-compressed entries (plen > 0: never written by Builder; the
// format the iterator accepts): entries 64 at a time, lane = entry, plen read from the header,
// key offsets by a wave scan of plen + stored key bytes; keys bytewise as baseKey[:plen] ++ diff
// (iterator.go:98-100), values as 16-B pieces.  Whole wave; `sub` / `split` share the entries.
template <bool COH>
__device__ __forceinline__ void copy_entries_plen(const DecodeParams& p, const uint32_t* meta,
                                               const uint8_t* blk, uint8_t* kbase, uint8_t* vbase,
                                               uint32_t n, uint64_t en, uint64_t ek, uint64_t ev,
                                               uint32_t off, uint32_t sub, uint32_t split,
                                               bool mat, bool view, uint32_t lane) {
  uint32_t carry = 0;  // key bytes of the entries before this chunk
  for (uint32_t e0 = 0; e0 < n; e0 += kWave) {
    const uint32_t e = e0 + lane;
    const bool on = e < n;
    const uint32_t m0 = ldm<COH>(meta + min(e, n)), m1 = ldm<COH>(meta + min(e + 1, n));
    const uint32_t hp = m0 & 0xffffu, vo = m0 >> 16;
    const uint32_t vl = (m1 >> 16) - vo, kl = (m1 & 0xffffu) - hp - 10 - vl;
    const uint32_t plen = on ? ((uint32_t)blk[hp] << 8) | blk[hp + 1] : 0u;
    const uint32_t kout = on ? plen + kl : 0u;
    const uint32_t incl = wave_scan_sat(kout, lane);
    const uint32_t ko = carry + incl - kout;
    carry += __builtin_amdgcn_readlane(incl, 63);
    if (!on || (e / kWave) % split != sub) continue;
    if (mat) {
      if (p.key_end) p.key_end[en + e] = (uint32_t)(ek + ko + kout);
      if (p.val_end) p.val_end[en + e] = (uint32_t)(ev + vo + vl);
      if (kbase)
        for (uint32_t i = 0; i < kout; i++)
          kbase[ko + i] = i < plen ? blk[10 + i] : blk[hp + 10 + i - plen];
      if (vbase)
        for (uint32_t q = 0; q < pieces16(vl); q++) copy_piece16(vbase + vo, blk + hp + 10 + kl, vl, q);
    }
    if (view)
      p.view[en + e] = (uint64_t)(off + hp + 10) | ((uint64_t)kl << 32) | ((uint64_t)vl << 48);
  }
}

// The entries of one block with no prefix-compressed entry, DENSE (round 6; blocks of large
// entries, average > 128 B: C5's Zipf keys, C3): 64 entries at a time, one per lane, write their
// per-entry outputs (64 consecutive words per store instruction) and count their 16-B pieces
// (key pieces then value pieces, pieces16); a wave scan gives each entry its first piece, and
// then every lane takes one piece of the run -- piece P's entry is the last one starting at or
// before P: each entry marks (lane + 1) at its first piece's slot of the 64-piece window (mk:
// 64 B of LDS per wave) and a DPP max-scan carries the owners forward.  The 16-lane groups this
// replaces left a Zipf entry's idle lanes empty in every store (C5: 4.73 M store instructions
// per 1 GiB copy against C2's 2.00 M for the same bytes).
template <bool COH, typename Src>
__device__ __forceinline__ void copy_entries_dense(const DecodeParams& p, const uint32_t* meta,
                                                   const Src& blk, uint8_t* kbase, uint8_t* vbase,
                                                   uint32_t n, uint64_t en, uint64_t ek, uint64_t ev,
                                                   uint32_t off, uint32_t sub, uint32_t split,
                                                   bool mat, bool view, uint32_t lane, uint32_t pre,
                                                   uint8_t* mk) {
  for (uint32_t c0 = sub * kWave; c0 < n; c0 += split * kWave) {
    const uint32_t e = c0 + lane;
    const uint32_t m0 = c0 == 0 ? pre : ldm<COH>(meta + min(e, n));
    const uint32_t nx = (uint32_t)__shfl((int)m0, (int)min(lane + 1, kWave - 1));
    const uint32_t m1 = lane + 1 < kWave ? nx : ldm<COH>(meta + min(e + 1, n));
    const bool on = e < n;
    const uint32_t hp = m0 & 0xffffu, vo = m0 >> 16, hp1 = m1 & 0xffffu, vo1 = m1 >> 16;
    const uint32_t vl = vo1 - vo, kl = hp1 - hp - 10 - vl;  // stored key bytes
    const uint32_t ko = hp - 10 * e - vo;                   // (no prefix-compressed entry here)
    if (on) {
      if (mat) {
        if (p.key_end) p.key_end[en + e] = (uint32_t)(ek + ko + kl);
        if (p.val_end) p.val_end[en + e] = (uint32_t)(ev + vo1);
      }
      if (view) p.view[en + e] = (uint64_t)(off + hp + 10) | ((uint64_t)kl << 32) | ((uint64_t)vl << 48);
    }
    if (!mat) continue;
    const uint32_t kp = on && kbase ? pieces16(kl) : 0u;
    const uint32_t pc = on ? kp + (vbase ? pieces16(vl) : 0u) : 0u;
    const uint32_t ps = wave_scan_sat(pc, lane), ex = ps - pc;
    const uint32_t T = __builtin_amdgcn_readlane(ps, 63);
    uint32_t carry = 0;
    for (uint32_t r0 = 0; r0 < T; r0 += kWave) {
      mk[lane] = 0;
      wave_lds_fence();
      if (pc > 0 && ex >= r0 && ex < r0 + kWave) mk[ex - r0] = (uint8_t)(lane + 1);
      wave_lds_fence();
      const uint32_t own = max(wave_scan_max(mk[lane], lane), carry);  // 1 + the owner lane
      carry = __builtin_amdgcn_readlane(own, 63);
      wave_lds_fence();  // (the marks are read before the next window clears them)
      const uint32_t L = own - 1;  // own >= 1: entry 0's first piece is piece 0
      // the owner's fields, packed 16 + 16 bits (every one < 64 KiB in a block < 64 KiB)
      const uint32_t a = (uint32_t)__shfl((int)(hp | (kl << 16)), (int)L);
      const uint32_t c = (uint32_t)__shfl((int)(ko | (vo << 16)), (int)L);
      const uint32_t d = (uint32_t)__shfl((int)(vl | (kp << 16)), (int)L);
      const uint32_t exL = (uint32_t)__shfl((int)ex, (int)L);
      const uint32_t hL = a & 0xffffu, kL = a >> 16, koL = c & 0xffffu, voL = c >> 16;
      const uint32_t vL = d & 0xffffu, kpL = d >> 16;
      const uint32_t P = r0 + lane;
      if (P >= T) continue;
      const uint32_t q = P - exL;
      if (q < kpL)
        blk.piece(kbase + koL, hL + 10, kL, q);
      else
        blk.piece(vbase + voL, hL + 10 + kL, vL, q - kpL);
    }
  }
}

// copy_entries_pipe with D - 1 entry groups' pieces in flight ahead of the stores (diag
// LSMGPU_WSC_PDEPTH = D >= 3; one wave, one record window: at most 8 groups), the groups fully
// unrolled so the ring of D piece registers needs no copies.
template <int D, int NG, typename Pc, typename PF, typename LF, typename SF, typename OF>
__device__ __forceinline__ void pipe_deep(uint32_t ng, PF&& piece, LF&& load, SF&& store, OF&& outputs) {
  Pc c[D];
  u32x4 v[D];
#pragma unroll
  for (int g = 0; g < D - 1; g++) {
    c[g] = piece((uint32_t)g, ng);
    v[g] = load(c[g]);
  }
  outputs();
#pragma unroll
  for (int g = 0; g < NG; g++) {
    if ((uint32_t)g >= ng) break;  // (uniform)
    if (g + D - 1 < NG) {
      c[(g + D - 1) % D] = piece((uint32_t)(g + D - 1), ng);
      v[(g + D - 1) % D] = load(c[(g + D - 1) % D]);
    }
    store(c[g % D], v[g % D]);
  }
}

// The entries of a block with no prefix-compressed entry, PIPELINED (materialize without view;
// the encoder's scheme, encode.hip encode_pipe_kernel): J lanes per entry, entry groups
// g = sub, sub + split, ... of 64 / J entries (wave `sub` of `split`).  Each lane's first piece
// of the wave's next group is loaded before this group's stores, and every load and store of the
// pipeline is a range-checked buffer access all lanes issue (a lane with nothing to move gives an
// offset past the resource: zeros read, store dropped), so the compiler's wait for the next
// group's pieces counts this group's stores and leaves them in flight -- the plain copy waits
// (vmcnt counts stores too) for every earlier store before each piece.  In the pipeline: 16-B
// pieces of either stream and 8-B value pieces (a 15-B value pointer's); the other pieces (key
// streams under 16 B, value streams under 8 B, pieces past a lane's first) follow it in the
// plain order.  Records come by lane shuffle from a window of 64 (`pre` for entries 0-63, then
// loaded and waited for once per 64 entries, so no other wait sits in the pipeline);
// key_end / val_end: one lane per entry, two buffer stores per window (by wave window % split).
template <uint32_t J, bool COH>
__device__ __forceinline__ void copy_entries_pipe(const DecodeParams& p, const uint32_t* meta,
                                                  const uint8_t* blk, uint8_t* kbase, uint8_t* vbase,
                                                  uint32_t n, uint32_t K, uint32_t V, uint64_t en,
                                                  uint64_t ek, uint64_t ev, uint32_t off,
                                                  uint32_t sub, uint32_t split, uint32_t lane,
                                                  uint32_t pre) {
  constexpr uint32_t EPP = kWave / J;
  const uint32_t j = lane & (J - 1);
  const __amdgpu_buffer_rsrc_t in = buffer_rsrc(blk, p.data_len - off);
  const __amdgpu_buffer_rsrc_t kr = buffer_rsrc(kbase, kbase ? K : 0u);
  const __amdgpu_buffer_rsrc_t vr = buffer_rsrc(vbase, vbase ? V : 0u);
  const __amdgpu_buffer_rsrc_t ker = buffer_rsrc(p.key_end ? p.key_end + en : nullptr, p.key_end ? 4ull * n : 0ull);
  const __amdgpu_buffer_rsrc_t ver = buffer_rsrc(p.val_end ? p.val_end + en : nullptr, p.val_end ? 4ull * n : 0ull);
  // the record window: lane l holds record w0 + l, wx record w0 + 64
  uint32_t w0 = 0, wr = pre, wx = n >= kWave ? ldm<COH>(meta + kWave) : 0u;
  auto fields = [&](uint32_t e, uint32_t& hp, uint32_t& kl, uint32_t& vl, uint32_t& ko, uint32_t& vo) {
    const uint32_t ec = min(e, n - 1), i = (ec - w0) & (kWave - 1);  // (off lanes: garbage, unused)
    const uint32_t m0 = (uint32_t)__shfl((int)wr, (int)i);
    const uint32_t nx = (uint32_t)__shfl((int)wr, (int)((i + 1) & (kWave - 1)));
    const uint32_t m1 = i + 1 < kWave ? nx : wx;
    hp = m0 & 0xffffu;
    vo = m0 >> 16;
    vl = (m1 >> 16) - vo;
    kl = (m1 & 0xffffu) - hp - 10 - vl;  // stored key bytes
    ko = hp - 10 * ec - vo;              // (no prefix-compressed entry here)
  };
  // key_end / val_end of the window's entries (lane = entry), written by one wave of the block's
  // (the others issue the same stores with every offset past the end: no branch, see below)
  auto outputs = [&]() {
    const uint32_t e = w0 + lane;
    uint32_t hp, kl, vl, ko, vo;
    fields(e, hp, kl, vl, ko, vo);
    const uint32_t o = e < n && (w0 / kWave) % split == sub ? 4 * e : kNoStore;
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)(ek + ko + kl), ker, o, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)(ev + vo + vl), ver, o, 0, 0);
  };
  // group g's pipelined piece of this lane (g past the window or the block: none): input offset
  // (kNoStore: none) and destinations
  struct Pc {
    uint32_t src, k16, v16, v8;
  };
  auto piece = [&](uint32_t g, uint32_t g_end) -> Pc {
    const uint32_t e = g * EPP + lane / J;
    uint32_t hp, kl, vl, ko, vo;
    fields(e, hp, kl, vl, ko, vo);
    const uint32_t kp = pieces16(kl), np = kp + pieces16(vl);
    Pc c{kNoStore, kNoStore, kNoStore, kNoStore};
    if (g < g_end && e < n && j < np) {
      if (j < kp) {
        if (kl >= 16) {
          const uint32_t o = min(16 * j, kl - 16);
          c.src = hp + 10 + o;
          c.k16 = ko + o;
        }
      } else if (vl >= 8) {
        const uint32_t q = j - kp, o = vl >= 16 ? min(16 * q, vl - 16) : (q ? vl - 8 : 0u);
        // (an 8-B piece is read as the upper half of the 16 B ending at its last byte: the read
        // never passes the stream's end, which may be the end of the data)
        c.src = hp + 10 + kl + o - (vl >= 16 ? 0u : 8u);
        if (vl >= 16) c.v16 = vo + o;
        else c.v8 = vo + o;
      }
    }
    return c;
  };
  auto load = [&](const Pc& c) -> u32x4 { return __builtin_amdgcn_raw_buffer_load_b128(in, c.src, 0, 0); };
  auto store = [&](const Pc& c, const u32x4& v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, kr, c.k16, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(v, vr, c.v16, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{v.z, v.w}, vr, c.v8, 0, 0);
  };
  const uint32_t ng = (n + EPP - 1) / EPP;
  // blocks of one record window: two groups' pieces in flight ahead of the stores (same box,
  // C2 copy 0.447-0.450 -> 0.440-0.441 ms; three groups ahead: 0.448, profiles/r06u)
  const uint32_t depth = LSMGPU_KNOB(p.wpdepth, 3u);
  if (depth >= 3 && n < kWave && split == 1) {
    if (depth == 3) pipe_deep<3, kWave / EPP, Pc>(ng, piece, load, store, outputs);
    else pipe_deep<4, kWave / EPP, Pc>(ng, piece, load, store, outputs);
  } else
  for (uint32_t b0 = 0; b0 < n; b0 += kWave) {  // (uniform) the record windows
    if (b0) {
      w0 = b0;
      wr = ldm<COH>(meta + min(b0 + lane, n));
      wx = ldm<COH>(meta + min(b0 + kWave, n));
    }
    // the wave's groups of this window: g0, g0 + split, ... < g1
    const uint32_t gw = b0 / EPP, g1 = min(ng, (b0 + kWave) / EPP);
    const uint32_t g0 = gw + (sub + split - gw % split) % split;
    Pc ca = piece(g0, g1);
    u32x4 va = load(ca);
    outputs();
    // (a store with nothing to write: the loop is then entered with as many buffer accesses
    // issued after the pending pieces as it loops with, so one wait count serves both entries)
    store(Pc{kNoStore, kNoStore, kNoStore, kNoStore}, u32x4{0u, 0u, 0u, 0u});
    for (uint32_t g = g0; g < g1; g += 2 * split) {  // two groups per trip: no register copy
      const Pc cb = piece(g + split, g1);
      const u32x4 vb = load(cb);
      store(ca, va);
      if (g + split >= g1) break;
      ca = piece(g + 2 * split, g1);
      va = load(ca);
      store(cb, vb);
    }
  }
  // the pieces outside the pipeline
  for (uint32_t g = sub; g < ng; g += split) {
    if (((g * EPP) & ~(kWave - 1)) != w0) {  // (uniform)
      w0 = (g * EPP) & ~(kWave - 1);
      wr = ldm<COH>(meta + min(w0 + lane, n));
      wx = ldm<COH>(meta + min(w0 + kWave, n));
    }
    const uint32_t e = g * EPP + lane / J;
    uint32_t hp, kl, vl, ko, vo;
    fields(e, hp, kl, vl, ko, vo);
    if (e >= n) continue;
    const uint32_t kp = pieces16(kl), np = kp + pieces16(vl);
    const bool first_in = j < np && (j < kp ? kl >= 16 : vl >= 8);
    for (uint32_t q = first_in ? j + J : j; q < np; q += J) {
      const bool key = q < kp;
      uint8_t* dst = key ? kbase : vbase;
      if (!dst) continue;
      copy_piece16(dst + (key ? ko : vo), blk + (key ? hp + 10 : hp + 10 + kl), key ? kl : vl,
                   key ? q : q - kp);
    }
  }
}

// copy_entries_dense, PIPELINED (materialize without view; the scheme of copy_entries_pipe):
// each 64-piece window's owners and piece are found (LDS marks + max-scan) and its piece loaded
// before the previous window's stores; every pipelined load and store is a range-checked buffer
// access all lanes issue.  Pieces of 16 B and 8 B go through the pipeline, shorter ones (streams
// under 8 B) are copied in the plain order where they fall.
template <bool COH>
__device__ __forceinline__ void copy_entries_dense_pipe(const DecodeParams& p, const uint32_t* meta,
                                                        const uint8_t* blk, uint8_t* kbase,
                                                        uint8_t* vbase, uint32_t n, uint32_t K,
                                                        uint32_t V, uint64_t en, uint64_t ek,
                                                        uint64_t ev, uint32_t off, uint32_t sub,
                                                        uint32_t split, uint32_t lane, uint32_t pre,
                                                        uint8_t* mk) {
  const __amdgpu_buffer_rsrc_t in = buffer_rsrc(blk, p.data_len - off);
  const __amdgpu_buffer_rsrc_t kr = buffer_rsrc(kbase, kbase ? K : 0u);
  const __amdgpu_buffer_rsrc_t vr = buffer_rsrc(vbase, vbase ? V : 0u);
  const __amdgpu_buffer_rsrc_t ker = buffer_rsrc(p.key_end ? p.key_end + en : nullptr, p.key_end ? 4ull * n : 0ull);
  const __amdgpu_buffer_rsrc_t ver = buffer_rsrc(p.val_end ? p.val_end + en : nullptr, p.val_end ? 4ull * n : 0ull);
  struct Pc {
    uint32_t src, dst;  // dst: stream offset; which stream and width in `kind`
    uint32_t kind;      // 0 none, 1 key 16 B, 2 value 16 B, 3 key 8 B, 4 value 8 B
  };
  auto load = [&](const Pc& c) -> u32x4 {
    return __builtin_amdgcn_raw_buffer_load_b128(in, c.kind ? c.src : kNoStore, 0, 0);
  };
  auto store = [&](const Pc& c, const u32x4& v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, kr, c.kind == 1 ? c.dst : kNoStore, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(v, vr, c.kind == 2 ? c.dst : kNoStore, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{v.z, v.w}, kr, c.kind == 3 ? c.dst : kNoStore, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{v.z, v.w}, vr, c.kind == 4 ? c.dst : kNoStore, 0, 0);
  };
  for (uint32_t c0 = sub * kWave; c0 < n; c0 += split * kWave) {
    const uint32_t e = c0 + lane;
    const uint32_t m0 = c0 == 0 ? pre : ldm<COH>(meta + min(e, n));
    const uint32_t nx = (uint32_t)__shfl((int)m0, (int)min(lane + 1, kWave - 1));
    const uint32_t m1 = lane + 1 < kWave ? nx : ldm<COH>(meta + min(e + 1, n));
    const bool on = e < n;
    const uint32_t hp = m0 & 0xffffu, vo = m0 >> 16, hp1 = m1 & 0xffffu, vo1 = m1 >> 16;
    const uint32_t vl = vo1 - vo, kl = hp1 - hp - 10 - vl;  // stored key bytes
    const uint32_t ko = hp - 10 * e - vo;                   // (no prefix-compressed entry here)
    const uint32_t kp = on && kbase ? pieces16(kl) : 0u;
    const uint32_t pc = on ? kp + (vbase ? pieces16(vl) : 0u) : 0u;
    const uint32_t ps = wave_scan_sat(pc, lane), ex = ps - pc;
    const uint32_t T = __builtin_amdgcn_readlane(ps, 63);
    uint32_t carry = 0;
    // window r0's piece of this lane (its owner by LDS marks + max-scan, as copy_entries_dense)
    auto win = [&](uint32_t r0) -> Pc {
      mk[lane] = 0;
      wave_lds_fence();
      if (pc > 0 && ex >= r0 && ex < r0 + kWave) mk[ex - r0] = (uint8_t)(lane + 1);
      wave_lds_fence();
      const uint32_t own = max(wave_scan_max(mk[lane], lane), carry);  // 1 + the owner lane
      carry = __builtin_amdgcn_readlane(own, 63);
      wave_lds_fence();
      const uint32_t L = own - 1;
      const uint32_t a = (uint32_t)__shfl((int)(hp | (kl << 16)), (int)L);
      const uint32_t c = (uint32_t)__shfl((int)(ko | (vo << 16)), (int)L);
      const uint32_t d = (uint32_t)__shfl((int)(vl | (kp << 16)), (int)L);
      const uint32_t exL = (uint32_t)__shfl((int)ex, (int)L);
      const uint32_t hL = a & 0xffffu, kL = a >> 16, koL = c & 0xffffu, voL = c >> 16;
      const uint32_t vL = d & 0xffffu, kpL = d >> 16;
      const uint32_t P = r0 + lane;
      Pc r{0u, 0u, 0u};
      if (P < T) {
        const uint32_t q = P - exL;
        const bool key = q < kpL;
        const uint32_t len = key ? kL : vL, qq = key ? q : q - kpL;
        const uint32_t s0 = key ? hL + 10 : hL + 10 + kL, d0 = key ? koL : voL;
        if (len >= 16) {
          const uint32_t o = min(16 * qq, len - 16);
          r = Pc{s0 + o, d0 + o, key ? 1u : 2u};
        } else if (len >= 8) {
          const uint32_t o = qq ? len - 8 : 0u;
          r = Pc{s0 + o - 8, d0 + o, key ? 3u : 4u};  // (the upper half of the 16 B ending here)
        } else {
          copy_piece16((key ? kbase : vbase) + d0, blk + s0, len, qq);
        }
      }
      return r;
    };
    Pc ca = win(0);
    u32x4 va = load(ca);
    {  // key_end / val_end (lane = entry), then a store with nothing to write: the loop is entered
       // with as many buffer accesses after the pending piece as it loops with
      const uint32_t o = on ? 4 * e : kNoStore;
      __builtin_amdgcn_raw_buffer_store_b32((uint32_t)(ek + ko + kl), ker, o, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32((uint32_t)(ev + vo1), ver, o, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{0u, 0u, 0u, 0u}, vr, kNoStore, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{0u, 0u, 0u, 0u}, vr, kNoStore, 0, 0);
    }
    for (uint32_t r0 = 0; r0 < T; r0 += 2 * kWave) {  // two windows per trip: no register copy
      const Pc cb = win(r0 + kWave);
      const u32x4 vb = load(cb);
      store(ca, va);
      if (r0 + kWave >= T) break;
      ca = win(r0 + 2 * kWave);
      va = load(ca);
      store(cb, vb);
    }
  }
}

// One block's share of the copy (wave `sub` of `split`): per-block outputs and result totals,
// the capacity check, then the entries -- from the walk's records `meta` (`pre` = record `lane`),
// the block's bytes read through `src` (prefix-compressed blocks always from global memory).
template <typename Src, bool COH>
__device__ __forceinline__ void copy_block(const DecodeParams& p, uint32_t b, const uint32_t* meta,
                                           uint32_t pre, uint32_t n, uint32_t K, uint32_t V,
                                           uint32_t sw, uint64_t en, uint64_t ek, uint64_t ev,
                                           uint32_t off, uint32_t sub, uint32_t split,
                                           uint32_t lane, const Src& src, uint32_t* tab,
                                           bool duties, uint8_t* mk) {
  const uint32_t st = sw & ~kPlenFlag;
  // duties: the per-block outputs, unless the walk kernel wrote them (every copy launch)
  if (duties && lane == 0 && sub == 0 && !ABLATE(p, 32)) {  // (timing-only ablation 32)
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
    if (duties && lane == 0 && sub == 0) atomicOr(reinterpret_cast<unsigned long long*>(p.result + 5), 1ull);
    return;
  }
  if (n == 0 || ABLATE(p, 2)) return;
  const uint8_t* blk = p.data + off;  // (prefix-compressed blocks)
  uint8_t* kbase = p.key_data ? p.key_data + ek : nullptr;
  uint8_t* vbase = p.val_data ? p.val_data + ev : nullptr;
  // lanes per entry from this block's average entry (known after the walk): 8 for C2-like
  // 119-B entries, 16 above 128 B (C5 Zipf keys: 0.96 vs 1.10 ms); p.wj forces 8 or 16.
  // 8 lanes x 5 groups = 40 entries per trip: every C2 block (31-37 entries) in one trip
  // (same-box A/B vs 4 groups: 0.799 -> 0.781 ms)
  // a block with prefix-compressed entries (flagged by the walk: no load of the sentinel here)
  if (sw & kPlenFlag) {
    copy_entries_plen<COH>(p, meta, blk, kbase, vbase, n, en, ek, ev, off, sub, split, mat, view, lane);
    return;
  }
  // small entries (8 lanes each): the per-entry outputs first, 64 entries per store instruction
  // (C2: copy 0.504 -> 0.485 ms; C5 / C3 blocks of fewer, larger entries lose 3 % that way, so
  // their 16-lane groups keep writing them)
  const uint32_t avg = (K + V) / n;
  // dense pieces for entries of > 128 B on average.  Pipelined (materialize without view): every
  // such block (C5 copy 0.550 -> 0.475 ms, profiles/r06r; C3's 1.1 KB entries 0.509 -> 0.469-0.474,
  // profiles/r06s); in the plain order only up to 512 B (C5 copy 0.593 -> 0.547 ms; C3 lost,
  // 0.525 vs 0.496 ms, profiles/r06h), above which the 16-lane groups fill their lanes
  const bool dpipe = !COH && LSMGPU_KNOB(p.wdpipe, 1u) && mat && !view;
  if (mk && avg > LSMGPU_KNOB(p.wdmin, 128u) && (dpipe ? avg <= LSMGPU_KNOB(p.wdmax, 0xffffffffu) : avg <= 512) &&
      !LSMGPU_KNOB(p.wj, 0u) && !LSMGPU_KNOB(p.weo, 0u) && LSMGPU_KNOB(p.wdense, 1u)) {
    // (diag build: LSMGPU_WSC_DPIPE=0 keeps copy_entries_dense, LSMGPU_WSC_DMAX caps the pipelined
    // mapping's average entry)
    if (dpipe)
      copy_entries_dense_pipe<COH>(p, meta, blk, kbase, vbase, n, K, V, en, ek, ev, off, sub, split,
                                   lane, pre, mk);
    else
      copy_entries_dense<COH>(p, meta, src, kbase, vbase, n, en, ek, ev, off, sub, split, mat, view,
                              lane, pre, mk);
    return;
  }
  // (round 4: each lane's first piece of every entry of a pass loaded before any store left
  // the copy unchanged, 0.6038 vs 0.6042 ms, profiles/r04c; compiled into this kernel it also
  // raised the VGPRs from 44 to 90, 8 -> 5 waves per SIMD: removed)
  if (!COH && LSMGPU_KNOB(p.walign, 0u) == 2 && mat && split == 1 && n < kWave && tab && chunks_fit(kbase, vbase, K, V)) {
    // dense aligned chunks over both streams (copy_chunks)
    if (!LSMGPU_KNOB(p.weo, 0u)) entry_outputs<COH>(p, meta, n, en, ek, ev, off, sub, split, mat, view, lane, pre);
    const uint64_t lim = p.data_len - off;
    copy_chunks(blk, lim < 0xffffffffull ? (uint32_t)lim : 0xffffffffu, kbase, vbase, n, K, V, lane, pre, tab);
  } else if (!COH && LSMGPU_KNOB(p.walign, 0u) == 1 && mat && split == 1) {
    // aligned output chunks + the stream edges byte by byte (copy_entries_aligned)
    if (!LSMGPU_KNOB(p.weo, 0u)) entry_outputs<COH>(p, meta, n, en, ek, ev, off, sub, split, mat, view, lane, pre);
    if (LSMGPU_KNOB(p.wj, 0u) == 16 || (LSMGPU_KNOB(p.wj, 0u) == 0 && avg > 128))
      copy_entries_aligned<16, 2>(meta, blk, kbase, vbase, n, K, V, sub, split, lane, pre);
    else
      copy_entries_aligned<8, 5>(meta, blk, kbase, vbase, n, K, V, sub, split, lane, pre);
  } else if ((LSMGPU_KNOB(p.wj, 0u) == 16 || (LSMGPU_KNOB(p.wj, 0u) == 0 && avg > 128)) && (LSMGPU_KNOB(p.weo, 0u) || LSMGPU_KNOB(p.weosep, 0u) || !mat)) {
    // (outputs: the walk wrote them, or one lane per entry first: a view-only decode through
    // the copy kernel (C5 view 0.270 -> 0.238 ms, profiles/r05ae), or LSMGPU_WSC_EOSEP=1 -- for
    // materialize the 16-lane groups' own writes stay faster: C5 copy 0.607 vs 0.617 ms, C3
    // 0.494-0.498 vs 0.508-0.510)
    if (!LSMGPU_KNOB(p.weo, 0u) && !ABLATE(p, 8)) entry_outputs<COH>(p, meta, n, en, ek, ev, off, sub, split, mat, view, lane, pre);
    copy_entries<16, 2, false, Src, COH>(p, meta, src, kbase, vbase, n, en, ek, ev, off, sub, split, mat, view, lane, pre);
  } else if (LSMGPU_KNOB(p.wj, 0u) == 16 || (LSMGPU_KNOB(p.wj, 0u) == 0 && avg > 128)) {
    copy_entries<16, 2, true, Src, COH>(p, meta, src, kbase, vbase, n, en, ek, ev, off, sub, split, mat, view, lane, pre);
  } else if (!COH && p.wpipe && mat && !view && (n < kWave || p.wpipe == 2) &&
             !LSMGPU_KNOB(p.weo, 0u) && !ABLATE(p, 8) && !ABLATE(p, 16)) {
    // (same box, C2 copy 0.485-0.487 -> 0.447-0.450 ms, decode 1,482 -> 1,558-1,564 GiB/s,
    // profiles/r06p; diag build: LSMGPU_WSC_PIPE=0 keeps copy_entries below, =2 takes blocks of
    // >= 64 entries too -- C4's 100-entry blocks, two waves each, lose: copy 0.0307 -> 0.0335 ms,
    // profiles/r06q)
    copy_entries_pipe<8, COH>(p, meta, blk, kbase, vbase, n, K, V, en, ek, ev, off, sub, split, lane, pre);
  } else {
    // (timing-only ablations: 8 no per-entry outputs, 16 no pieces)
    if (!ABLATE(p, 8) && !LSMGPU_KNOB(p.weo, 0u)) entry_outputs<COH>(p, meta, n, en, ek, ev, off, sub, split, mat, view, lane, pre);
    if (mat && !ABLATE(p, 16))
      copy_entries<8, 5, false, Src, COH>(p, meta, src, kbase, vbase, n, en, ek, ev, off, sub, split, mat, view, lane, pre);
  }
}

// K2: one wave per block (p.wsplit waves above 8 KiB).
// (Measured against it: two blocks per wave with the second block's words loaded during the first
// block's pieces.  C2 copy 0.492 -> 0.598 ms at 64 VGPRs with 21 spilled, and -> 0.706 ms at 99
// VGPRs, occupancy 4: the copy needs waves in flight more than it needs fewer metadata round
// trips.  Profiles r05aj, r05ak.)
__global__ void __launch_bounds__(256) wsc_copy_kernel(DecodeParams p) {
  const uint32_t lane = lane_id();
  // p.wsplit waves share a block (large blocks): wave `sub` takes passes sub, sub + wsplit, ...
  const uint32_t wave = threadIdx.x >> 6, split = p.wsplit;
  const uint32_t sub = wave % split;
  const uint32_t b = uniform(blockIdx.x * (4 / split) + wave / split);
  if (b >= p.nblk) return;
  const uint32_t* meta = p.wmeta + (uint64_t)b * p.wcap;
  // the first 64 metadata records, one per lane, requested beside the per-block loads below
  // (one round trip fewer before the piece loads; records past the sentinel are never used)
  const uint32_t pre = meta[min(lane, p.wcap - 1)];
  const uint4 d0 = p.wdesc[2ull * b], d1 = p.wdesc[2ull * b + 1];  // the walk's descriptor
  const uint32_t n = uniform(d0.x), K = uniform(d0.y), V = uniform(d0.z), sw = uniform(d0.w);
  const uint64_t en = uniform(d1.x), ek = uniform(d1.y), ev = uniform(d1.z);
  const uint32_t off = uniform(d1.w);
  __shared__ uint32_t s_chunk[4][kChunkLds];  // copy_chunks' per-wave tables (diag)
  __shared__ uint8_t s_mk[4][kWave];           // copy_entries_dense's owner marks
  copy_block(p, b, meta, pre, n, K, V, sw, en, ek, ev, off, sub, split, lane, GlobalBytes{p.data + off},
             s_chunk[threadIdx.x >> 6], false, s_mk[threadIdx.x >> 6]);
}


__device__ __forceinline__ void fused_copier(const DecodeParams& p, uint32_t c, uint32_t ncop,
                                             uint32_t tb) {
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6, split = p.wsplit;
  const uint32_t sub = wave % split, per = 4 / split;  // blocks per 4-wave group
  const uint32_t ngroups = (p.nblk + per - 1) / per;
  for (uint32_t g = c; g < ngroups; g += ncop) {
    const uint32_t b = g * per + wave / split;
    if (b >= p.nblk) break;  // (wave-uniform; later groups are further out)
    // relaxed polls (an acquiring poll invalidates the XCD's L2 each time: C4 1.0 ms instead of
    // 0.067); the tile's records and descriptors are then read with coherent loads (st_rec4)
    const uint64_t* flag = p.lb + (uint64_t)(b / tb) * 8 + 7;
    if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != (uint64_t)p.tag) {
      SpinBound bound;
      do {
        if (bound.expired()) {
          flag_timeout(p.result, lane);
          return;
        }
        __builtin_amdgcn_s_sleep(20);
      } while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != (uint64_t)p.tag);
    }
    const uint32_t* meta = p.wmeta + (uint64_t)b * p.wcap;
    const uint32_t pre = ldm<true>(meta + min(lane, p.wcap - 1));
    const uint4 d0 = ld_desc<true>(p.wdesc + 2ull * b), d1 = ld_desc<true>(p.wdesc + 2ull * b + 1);
    const uint32_t n = uniform(d0.x), K = uniform(d0.y), V = uniform(d0.z), sw = uniform(d0.w);
    const uint64_t en = uniform(d1.x), ek = uniform(d1.y), ev = uniform(d1.z);
    const uint32_t off = uniform(d1.w);
    copy_block<GlobalBytes, true>(p, b, meta, pre, n, K, V, sw, en, ek, ev, off, sub, split, lane,
                                  GlobalBytes{p.data + off}, nullptr, false);
  }
}

// The wide lane walk with two tiles per workgroup (LSMGPU_WSC_PERSIST=1, materialize decodes of
// 576-thread tiles).  In wsc_walk_kernel each tile's workgroup waits for its predecessors'
// aggregates after walking (the census: 5-7 us per tile, profiles/r05q) and only then frees the
// CU for a second-wave tile.  Here a workgroup takes a ticket, walks that tile and publishes its
// aggregate, takes a second ticket and walks that tile, and only then runs the look-back and the
// per-block epilogue of both -- by which time the first tile's predecessors have long finished.
// Every ticket is taken by a running workgroup, and a workgroup publishes both aggregates
// before it waits on anything, so every look-back ends whatever the residency.  Each
// workgroup makes exactly two ticket draws (the grid is ceil(tiles / 2)); draws past the last
// tile walk nothing, and the last draw of the launch resets the counter.  The walk loop, the
// records and the epilogue are those of wsc_walk_kernel's lane walk.
template <uint32_t TB>
__global__ void __launch_bounds__(TB) wsc_walk_persist_kernel(DecodeParams p) {
  constexpr uint32_t CH = 32, kThreads = TB, kWaves = TB / kWave, kStage = CH + 1;
  __shared__ __attribute__((aligned(16))) uint32_t stage[kThreads * kStage];
  __shared__ uint32_t s_tile[2];
  __shared__ uint32_t s_wave[2][kWaves][3];
  __shared__ uint32_t s_part[kWaves][3];
  __shared__ uint32_t s_ex[3];
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint32_t TBe = p.wtbe, ntiles = (p.nblk + TBe - 1) / TBe, draws = 2 * gridDim.x;
  uint32_t tl[2], nn[2], KK[2], VV[2], ss[2], oo[2], in_[2], ik[2], iv[2];
#pragma unroll
  for (uint32_t r = 0; r < 2; r++) {
    if (tid == 0) {
      const uint32_t t = atomicAdd(p.gcnt, 1u);
      if (t == draws - 1) atomicExch(p.gcnt, 0u);  // the launch's last draw
      s_tile[r] = t;
    }
    __syncthreads();
    const uint32_t tile = s_tile[r];
    tl[r] = tile;
    nn[r] = KK[r] = VV[r] = oo[r] = 0;
    ss[r] = LSMGPU_BLK_OK;
    in_[r] = ik[r] = iv[r] = 0;
    if (tile >= ntiles) continue;  // (uniform)
    if (p.zero_result && tile == 0 && tid < 8)  // as wsc_walk_kernel: before anything else
      atomicExch(reinterpret_cast<unsigned long long*>(p.result + tid), 0ull);
    const uint32_t b = tid < TBe ? tile * TBe + tid : 0xffffffffu;
    uint32_t n = 0, K = 0, V = 0, st = LSMGPU_BLK_OK;
    const bool valid = b < p.nblk;
    uint32_t* row = stage + tid * kStage;
    uint32_t off = 0, len = 0, pos = 0;
    if (valid) {
      off = p.blk_off[b];
      len = p.blk_len[b];
    }
    bool done = !valid || ABLATE(p, 4);
    if (valid && (uint64_t)off + len > p.data_len) {
      st = LSMGPU_BLK_RANGE;
      done = true;
    }
    const uint8_t* blk = p.data + off;
    const uint32_t wb0 = tile * TBe + wave * 64;
    for (uint32_t k = 0;; k++) {
      if (__ballot(!done) == 0) break;
      bool rec = false;
      if (!done) {
        do {
          if (pos >= len) { done = true; break; }                  // iterator.go:115-118
          if (len - pos < 10) { st = LSMGPU_BLK_TRUNC_HEADER; done = true; break; }
          uint32_t plen, klen, vlen;
          read_hdr_nt(blk + pos, plen, klen, vlen);                // iterator.go:121
          if ((klen | plen) == 0) { done = true; break; }          // iterator.go:124-127
          if (n == 0 && plen != 0) { st = LSMGPU_BLK_FIRST_PLEN; done = true; break; }
          if (10 + plen > len) { st = LSMGPU_BLK_PREFIX_OOB; done = true; break; }
          const uint32_t end = pos + 10 + klen + vlen;             // iterator.go:101-109
          if (end > len) { st = LSMGPU_BLK_VALUE_OVERFLOW; done = true; break; }
          row[n & (CH - 1)] = pos | (V << 16);
          K += plen + klen;
          V += vlen;
          n++;
          pos = end;
          rec = true;
        } while (false);
      }
      if ((k & (CH - 1)) == CH - 1) {  // whole 128-B record lines, 8 lanes per line
        const uint64_t fl = __ballot(rec);
        if (fl) {
          wave_lds_fence();
          constexpr uint32_t kPer = CH / 4;
#pragma unroll
          for (uint32_t q = 0; q < kPer; q++) {
            const uint32_t L = (64 / kPer) * q + lane / kPer, part = lane % kPer;
            if ((fl >> L) & 1ull) {
              const uint32_t* rw = stage + (wave * 64 + L) * kStage + 4 * part;
              uint32_t* mL = p.wmeta + (uint64_t)(wb0 + L) * p.wcap + (k - (CH - 1));
              reinterpret_cast<uint4*>(mL)[part] = make_uint4(rw[0], rw[1], rw[2], rw[3]);
            }
          }
          wave_lds_fence();
        }
      }
    }
    if (valid) row[n & (CH - 1)] = pos | (V << 16);  // the sentinel
    const uint64_t vm = __ballot(valid);
    wave_lds_fence();
    {
      constexpr uint32_t kPer = CH / 4;
#pragma unroll
      for (uint32_t q = 0; q < kPer; q++) {
        const uint32_t L = (64 / kPer) * q + lane / kPer, part = lane % kPer;
        const uint32_t nL = (uint32_t)__shfl((int)n, (int)L);
        if ((vm >> L) & 1ull) {
          const uint32_t* rw = stage + (wave * 64 + L) * kStage + 4 * part;
          uint32_t* mL = p.wmeta + (uint64_t)(wb0 + L) * p.wcap + (nL & ~(CH - 1));
          reinterpret_cast<uint4*>(mL)[part] = make_uint4(rw[0], rw[1], rw[2], rw[3]);
        }
      }
    }
    wave_lds_fence();  // the rows are read before the next tile's walk refills them
    if (valid && K != pos - 10 * n - V) st |= kPlenFlag;  // (the descriptor's status word)
    // tile scan, and the tile's aggregate published at once
    in_[r] = wave_scan_sat(n, lane);
    ik[r] = wave_scan_sat(K, lane);
    iv[r] = wave_scan_sat(V, lane);
    if (lane == 63) {
      s_wave[r][wave][0] = in_[r];
      s_wave[r][wave][1] = ik[r];
      s_wave[r][wave][2] = iv[r];
    }
    __syncthreads();
    if (wave == 0) {
      uint32_t tn = 0, tk = 0, tv = 0;
      for (uint32_t w = 0; w < kWaves; w++) {
        tn = sat_add(tn, s_wave[r][w][0]);
        tk = sat_add(tk, s_wave[r][w][1]);
        tv = sat_add(tv, s_wave[r][w][2]);
      }
      store3(p.lb + (uint64_t)tile * 8, p.tag, tn, tk, tv, lane);
    }
    nn[r] = n;
    KK[r] = K;
    VV[r] = V;
    ss[r] = st;
    oo[r] = off;
  }
#pragma unroll
  for (uint32_t r = 0; r < 2; r++) {
    const uint32_t tile = tl[r];
    if (tile >= ntiles) continue;  // (uniform)
    Tot part{0, 0, 0};
    if (tile > 0 && !ABLATE(p, 1)) part = lookback_partial(p.lb, tile, p.tag, tid, kThreads, p.result);
    const uint32_t pn = wave_sum_sat(part.n), pk = wave_sum_sat(part.k), pv = wave_sum_sat(part.v);
    if (lane == 0) {
      s_part[wave][0] = pn;
      s_part[wave][1] = pk;
      s_part[wave][2] = pv;
    }
    __syncthreads();
    if (wave == 0 && lane == 0) {
      Tot ex{0, 0, 0};
      for (uint32_t w = 0; w < kWaves; w++) {
        ex.n = sat_add(ex.n, s_part[w][0]);
        ex.k = sat_add(ex.k, s_part[w][1]);
        ex.v = sat_add(ex.v, s_part[w][2]);
      }
      s_ex[0] = ex.n;
      s_ex[1] = ex.k;
      s_ex[2] = ex.v;
    }
    __syncthreads();
    const uint32_t b = tid < TBe ? tile * TBe + tid : 0xffffffffu;
    const uint32_t n = nn[r], K = KK[r], V = VV[r], sw = ss[r], st = sw & ~kPlenFlag;
    if (b < p.nblk) {  // the epilogue of wsc_walk_kernel's lane walk
      uint32_t on = s_ex[0], ok = s_ex[1], ov = s_ex[2];
      for (uint32_t w = 0; w < wave; w++) {
        on = sat_add(on, s_wave[r][w][0]);
        ok = sat_add(ok, s_wave[r][w][1]);
        ov = sat_add(ov, s_wave[r][w][2]);
      }
      const uint32_t en = sat_add(on, in_[r] - n),
                     ek = sat_add(ok, ik[r] == 0xffffffffu ? ik[r] : ik[r] - K), ev = sat_add(ov, iv[r] - V);
      p.wdesc[2ull * b] = make_uint4(n, K, V, sw);
      p.wdesc[2ull * b + 1] = make_uint4(en, ek, ev, oo[r]);
      if (p.blk_first) p.blk_first[b] = en;
      if (p.blk_status) p.blk_status[b] = (int32_t)st;
      if (st != LSMGPU_BLK_OK) {
        atomicAdd(reinterpret_cast<unsigned long long*>(p.result + 4), 1ull);
        atomicMax(reinterpret_cast<unsigned long long*>(p.result + 3), (unsigned long long)(p.nblk - b));
      }
      if (b == p.nblk - 1) {  // totals of the whole batch
        if (p.blk_first) p.blk_first[p.nblk] = (uint32_t)((uint64_t)en + n);
        p.result[0] = (uint64_t)en + n;
        p.result[1] = (uint64_t)ek + K;
        p.result[2] = (uint64_t)ev + V;
      }
      bool fits = (uint64_t)en + n <= p.ent_cap && (uint64_t)en + n <= 0xffffffffull;
      if (p.mode & LSMGPU_MODE_MATERIALIZE) {  // the copy's output streams
        const uint64_t kend = (uint64_t)ek + K, vend = (uint64_t)ev + V;
        fits = fits && (kend <= p.key_cap || !p.key_data) && (vend <= p.val_cap || !p.val_data) &&
               kend < 0xffffffffull && vend <= 0xffffffffull;
      }
      if (!fits) atomicOr(reinterpret_cast<unsigned long long*>(p.result + 5), 1ull);
    }
    __syncthreads();  // s_part / s_ex are reused by the second tile
  }
}

// The lane walk with a second lane per block walking it BACKWARD (round 6; materialize or view
// through the copy launch; batches of long blocks: C5's 150-entry chains).  A wave holds 32
// blocks: lane l < 32 walks block l forward exactly as the lane walk does, lane l + 32 walks it
// backward from the terminator T = len - 13 along the headers' `prev` fields (builder.go:95-99,
// 121-123).  The iterator never reads `prev`, so a backward step is accepted only when the
// entry it names is one the iterator would accept there: not a terminator, 10 + plen <= len,
// plen == 0 if it is at 0, and ending exactly where the last accepted one starts
// (pos + 10 + klen + vlen == bx).  Every accepted entry therefore lies on the forward chain once
// the forward walk reaches the lowest one, bx: the forward lane stops walking when its position
// equals its partner's bx and takes the backward entries from the partner's LDS stack instead
// (one LDS read per entry, no HBM round trip), then ends at T as the iterator does.  Partners
// meet through lane shuffles, once per step; both directions' header loads go out before one
// wait.  A backward lane stops when its stack is full (kBackCap), when a candidate fails, or when
// the forward lane has passed the candidate; if the forward walk never lands on bx (a block the
// Builder did not write) it simply walks on to its end: the result is always the forward
// iterator's.  Records, flushes, tile scan, look-back and epilogue are the lane walk's.
constexpr uint32_t kBackCap = 96;  // backward entries per block (LDS stack)

// non-temporal header reads the compiler sees (so it places one wait for both directions'
// loads before their first use): 8 B at g, or the 16 B at g (any alignment)
typedef uint32_t u32x2u __attribute__((ext_vector_type(2), aligned(1)));
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
__device__ __forceinline__ u32x2u ld8_nt(const uint8_t* g) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x2u*>(g));
}
__device__ __forceinline__ u32x4u ld16_nt(const uint8_t* g) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4u*>(g));
}

template <uint32_t TB>
__global__ void __launch_bounds__(2 * TB) wsc_walk_bidir_kernel(DecodeParams p) {
  constexpr uint32_t CH = 32, kThreads = 2 * TB, kWaves = kThreads / kWave, kStage = CH + 1;
  constexpr uint32_t kHalf = kWave / 2;  // blocks per wave
  static_assert(TB % kHalf == 0, "whole waves");
  __shared__ __attribute__((aligned(16))) uint32_t stage[TB * kStage];
  __shared__ uint32_t bstk[TB * kBackCap];
  __shared__ uint32_t s_tile;
  __shared__ uint32_t s_wave[kWaves][3];
  __shared__ uint32_t s_part[kWaves][3];
  __shared__ uint32_t s_ex[3];
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const bool fwd = lane < kHalf;
  const uint32_t tb = wave * kHalf + (lane & (kHalf - 1)), partner = lane ^ kHalf;
  const uint32_t ntiles = (p.nblk + TB - 1) / TB;
  if (tid == 0) {
    const uint32_t t = atomicAdd(p.gcnt, 1u);
    if (t == ntiles - 1) atomicExch(p.gcnt, 0u);  // every ticket is taken
    s_tile = t;
  }
  __syncthreads();
  const uint32_t tile = s_tile;
  if (p.zero_result && tile == 0 && tid < 8)  // (as wsc_walk_kernel: before anything else)
    atomicExch(reinterpret_cast<unsigned long long*>(p.result + tid), 0ull);
  const uint32_t b = tile * TB + tb;
  const bool valid = b < p.nblk;
  uint32_t off = 0, len = 0, st = LSMGPU_BLK_OK;
  if (valid) {
    off = p.blk_off[b];
    len = p.blk_len[b];
  }
  bool done = !valid;
  if (valid && (uint64_t)off + len > p.data_len) {
    st = LSMGPU_BLK_RANGE;
    done = true;
  }
  const uint8_t* blk = p.data + off;
  uint32_t* const row = stage + tb * kStage;
  uint32_t* const stk = bstk + tb * kBackCap;
  const uint32_t wb0 = tile * TB + wave * kHalf;
  // forward: the lane walk's state; met: it reached the partner's lowest backward entry
  uint32_t n = 0, K = 0, V = 0, pos = 0;
  bool met = false;
  // backward: lowest accepted position bx (T before the first entry), its prev `by`, entries bn
  // on the stack, their key bytes bk; bstart: the terminator has been read
  uint32_t bx = len - 13, by = 0, bn = 0, bk = 0;
  bool bact = !fwd && !done && len >= 23, bstart = false;
  if (fwd) bx = 0;
  [[maybe_unused]] uint32_t steps = 0;
  for (uint32_t k = 0;; k++) {
    if (__ballot(fwd && !done && !met) == 0) break;  // (the backward lanes only serve the forward ones)
    steps = k + 1;
    // partners, one shuffle: the forward lane sees the backward chain's lowest entry and its
    // size, the backward lane the forward position and whether that walk has stopped (positions
    // are < 64 KiB, stacks < 32 K entries)
    const uint32_t mine = fwd ? pos | ((done || met) ? 1u << 16 : 0u)
                              : bx | ((bstart ? bn : 0u) << 16);
    const uint32_t his = (uint32_t)__shfl((int)mine, (int)partner);
    bool gl = false;
    uint32_t ga = 0;
    if (fwd && !done && !met) {
      if ((his >> 16) != 0 && pos == (his & 0xffffu)) {  // met: the rest are the partner's entries
        met = true;
      } else if (pos >= len) {
        done = true;                                                               // iterator.go:115-118
      } else if (len - pos < 10) {
        st = LSMGPU_BLK_TRUNC_HEADER;
        done = true;
      } else {
        gl = true;
        ga = pos;
      }
    }
    if (!fwd && bact) {
      const uint32_t s_pos = his & 0xffffu;
      if ((his >> 16) != 0 || bn == kBackCap) bact = false;
      // (no entry fits; or the forward walk reads the candidate this step or has passed it: it
      // lands on bx by itself if the chains agree)
      else if (bstart && (by > bx || bx - by < 10 || by <= s_pos || by < 6)) bact = false;
      else { gl = true; ga = bstart ? by : bx; }
    }
    // one load instruction for the wave: every lane reads the 16 B that end with its header
    // (bytes 6-15: plen, klen, vlen, prev), inside the block; a header at 0 (a forward lane's
    // first step) from the block's first 16 B, or, in a block under 16 B, as 8 B of its own
    uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
    const bool at0 = ga < 6;
    if (gl && (!at0 || len >= 16)) {
      const u32x4u v = ld16_nt(blk + (at0 ? 0u : ga - 6));
      w0 = v.x;
      w1 = v.y;
      w2 = v.z;
      w3 = v.w;
    } else if (gl) {
      const u32x2u v = ld8_nt(blk + ga);
      w0 = v.x;
      w1 = v.y;
    }
    const uint32_t plen = at0 ? __builtin_amdgcn_perm(0u, w0, 0x0c0c0001u) : __builtin_amdgcn_perm(0u, w1, 0x0c0c0203u);
    const uint32_t klen = at0 ? __builtin_amdgcn_perm(0u, w0, 0x0c0c0203u) : __builtin_amdgcn_perm(0u, w2, 0x0c0c0001u);
    const uint32_t vlen = at0 ? __builtin_amdgcn_perm(0u, w1, 0x0c0c0001u) : __builtin_amdgcn_perm(0u, w2, 0x0c0c0203u);
    const uint32_t x1 = w3;  // (backward lanes: never at 0)
    bool rec = false;
    if (fwd && gl) {
      do {
        if ((klen | plen) == 0) { done = true; break; }          // iterator.go:124-127
        if (n == 0 && plen != 0) { st = LSMGPU_BLK_FIRST_PLEN; done = true; break; }
        if (10 + plen > len) { st = LSMGPU_BLK_PREFIX_OOB; done = true; break; }
        const uint32_t end = pos + 10 + klen + vlen;             // iterator.go:101-109
        if (end > len) { st = LSMGPU_BLK_VALUE_OVERFLOW; done = true; break; }
        row[n & (CH - 1)] = pos | (V << 16);
        K += plen + klen;
        V += vlen;
        n++;
        pos = end;
        rec = true;
      } while (false);
    }
    if (!fwd && gl) {
      const uint32_t prev = __builtin_bswap32(x1);
      if (!bstart) {  // the terminator: T's prev names the last entry
        bstart = true;
        if ((klen | plen) == 0 && prev != 0xffffffffu && prev + 10 <= bx) by = prev;
        else bact = false;
      } else if ((klen | plen) != 0 && by + 10 + klen + vlen == bx && 10 + plen <= len &&
                 (by != 0 || plen == 0)) {
        stk[bn] = by | (vlen << 16);
        bn++;
        bk += plen + klen;
        bx = by;
        by = prev;
      } else {
        bact = false;
      }
    }
    if ((k & (CH - 1)) == CH - 1) {  // whole 128-B record lines of the forward rows, 8 lanes per line
      const uint64_t fl = __ballot(rec);
      if (fl) {
        wave_lds_fence();
        constexpr uint32_t kPer = CH / 4;
#pragma unroll
        for (uint32_t q = 0; q < kHalf / (kWave / kPer); q++) {
          const uint32_t L = (kWave / kPer) * q + lane / kPer, part = lane % kPer;
          if ((fl >> L) & 1ull) {
            const uint32_t* rw = stage + (wave * kHalf + L) * kStage + 4 * part;
            uint32_t* mL = p.wmeta + (uint64_t)(wb0 + L) * p.wcap + (k - (CH - 1));
            reinterpret_cast<uint4*>(mL)[part] = make_uint4(rw[0], rw[1], rw[2], rw[3]);
          }
        }
        wave_lds_fence();
      }
    }
  }
  // a forward lane that met its partner takes the backward entries (ascending: the stack's top is
  // the block's last entry) into its row, writing each full 32-record chunk out as it fills, and
  // ends at the terminator as the iterator does
  const uint32_t pbn = (uint32_t)__shfl((int)bn, (int)partner), pbk = (uint32_t)__shfl((int)bk, (int)partner);
  wave_lds_fence();
  if (fwd && met) {
    uint32_t* const m0 = p.wmeta + (uint64_t)b * p.wcap;
    for (uint32_t i = 0; i < pbn; i++) {
      const uint32_t e = stk[pbn - 1 - i];
      row[n & (CH - 1)] = (e & 0xffffu) | (V << 16);
      V += e >> 16;
      n++;
      if ((n & (CH - 1)) == 0) {
        uint4* d = reinterpret_cast<uint4*>(m0 + (n - CH));
#pragma unroll
        for (uint32_t q = 0; q < CH / 4; q++) d[q] = make_uint4(row[4 * q], row[4 * q + 1], row[4 * q + 2], row[4 * q + 3]);
      }
    }
    K += pbk;
    pos = len - 13;
    done = true;
  }
#ifdef LSMGPU_DIAG
  // (diagnostics: blocks whose walks met, in result[6]; the longest lane's steps, in result[7])
  if (fwd && met && (p.ablate & 1024u)) atomicAdd(reinterpret_cast<unsigned long long*>(p.result + 6), 1ull);
  if (lane == 0 && (p.ablate & 1024u)) atomicAdd(reinterpret_cast<unsigned long long*>(p.result + 7), (unsigned long long)steps);
#endif
  const bool own = fwd && valid;  // the lane that reports the block
  if (own) row[n & (CH - 1)] = pos | (V << 16);  // the sentinel
  const uint64_t vm = __ballot(own);
  wave_lds_fence();
  {
    constexpr uint32_t kPer = CH / 4;
#pragma unroll
    for (uint32_t q = 0; q < kHalf / (kWave / kPer); q++) {
      const uint32_t L = (kWave / kPer) * q + lane / kPer, part = lane % kPer;
      const uint32_t nL = (uint32_t)__shfl((int)n, (int)L);
      if ((vm >> L) & 1ull) {
        const uint32_t* rw = stage + (wave * kHalf + L) * kStage + 4 * part;
        uint32_t* mL = p.wmeta + (uint64_t)(wb0 + L) * p.wcap + (nL & ~(CH - 1));
        reinterpret_cast<uint4*>(mL)[part] = make_uint4(rw[0], rw[1], rw[2], rw[3]);
      }
    }
  }
  if (!fwd) n = K = V = 0;
  if (own && K != pos - 10 * n - V) st |= kPlenFlag;  // (the descriptor's status word)
  // tile scan (backward lanes add nothing), the tile's aggregate, look-back, epilogue
  const uint32_t in = wave_scan_sat(n, lane), ik = wave_scan_sat(K, lane), iv = wave_scan_sat(V, lane);
  if (lane == 63) {
    s_wave[wave][0] = in;
    s_wave[wave][1] = ik;
    s_wave[wave][2] = iv;
  }
  __syncthreads();
  if (wave == 0) {
    uint32_t tn = 0, tk = 0, tv = 0;
    for (uint32_t w = 0; w < kWaves; w++) {
      tn = sat_add(tn, s_wave[w][0]);
      tk = sat_add(tk, s_wave[w][1]);
      tv = sat_add(tv, s_wave[w][2]);
    }
    store3(p.lb + (uint64_t)tile * 8, p.tag, tn, tk, tv, lane);
  }
  Tot part{0, 0, 0};
  if (tile > 0) part = lookback_partial(p.lb, tile, p.tag, tid, kThreads, p.result);
  const uint32_t pn = wave_sum_sat(part.n), pk = wave_sum_sat(part.k), pv = wave_sum_sat(part.v);
  if (lane == 0) {
    s_part[wave][0] = pn;
    s_part[wave][1] = pk;
    s_part[wave][2] = pv;
  }
  __syncthreads();
  if (tid == 0) {
    Tot ex{0, 0, 0};
    for (uint32_t w = 0; w < kWaves; w++) {
      ex.n = sat_add(ex.n, s_part[w][0]);
      ex.k = sat_add(ex.k, s_part[w][1]);
      ex.v = sat_add(ex.v, s_part[w][2]);
    }
    s_ex[0] = ex.n;
    s_ex[1] = ex.k;
    s_ex[2] = ex.v;
  }
  __syncthreads();
  if (own) {
    uint32_t on = s_ex[0], ok = s_ex[1], ov = s_ex[2];
    for (uint32_t w = 0; w < wave; w++) {
      on = sat_add(on, s_wave[w][0]);
      ok = sat_add(ok, s_wave[w][1]);
      ov = sat_add(ov, s_wave[w][2]);
    }
    const uint32_t sw = st, stc = sw & ~kPlenFlag;
    const uint32_t en = sat_add(on, in - n), ek = sat_add(ok, ik == 0xffffffffu ? ik : ik - K),
                   ev = sat_add(ov, iv - V);
    p.wdesc[2ull * b] = make_uint4(n, K, V, sw);
    p.wdesc[2ull * b + 1] = make_uint4(en, ek, ev, off);
    if (p.blk_first) p.blk_first[b] = en;
    if (p.blk_status) p.blk_status[b] = (int32_t)stc;
    if (stc != LSMGPU_BLK_OK) {
      atomicAdd(reinterpret_cast<unsigned long long*>(p.result + 4), 1ull);
      atomicMax(reinterpret_cast<unsigned long long*>(p.result + 3), (unsigned long long)(p.nblk - b));
    }
    if (b == p.nblk - 1) {  // totals of the whole batch
      if (p.blk_first) p.blk_first[p.nblk] = (uint32_t)((uint64_t)en + n);
      p.result[0] = (uint64_t)en + n;
      p.result[1] = (uint64_t)ek + K;
      p.result[2] = (uint64_t)ev + V;
    }
    bool fits = (uint64_t)en + n <= p.ent_cap && (uint64_t)en + n <= 0xffffffffull;
    if (p.mode & LSMGPU_MODE_MATERIALIZE) {  // the copy's output streams
      const uint64_t kend = (uint64_t)ek + K, vend = (uint64_t)ev + V;
      fits = fits && (kend <= p.key_cap || !p.key_data) && (vend <= p.val_cap || !p.val_data) &&
             kend < 0xffffffffull && vend <= 0xffffffffull;
    }
    if (!fits) atomicOr(reinterpret_cast<unsigned long long*>(p.result + 5), 1ull);
  }
}

hipError_t launch_decode_wsc(const DecodeParams& p, hipStream_t s, hipEvent_t mid) {
  const uint32_t nblk = p.nblk;
  // the adopted walks (api.hip picks one per batch; the parity suite runs each of them):
  //   materialize, wide tiles (> 4 x 256-block tiles per CU): two 576-thread tiles per workgroup
  //   view-only fused into the walk: kWalkLaneView, 576- or 256-block tiles
  //   <= 64 blocks per CU: 8 lanes forward + 8 backward per block (kWalkGroupBi)
  //   blocks above 8 KiB: one lane forward + one backward per block (wsc_walk_bidir_kernel)
  //   otherwise one lane per block, 256-block tiles
  const bool persist = LSMGPU_KNOB(p.wpersist, 1u) && !p.wfuse && p.wwalk != kWalkGroup && p.wwide == 576 &&
                       LSMGPU_KNOB(p.wchunk, 32u) == 32 && !LSMGPU_KNOB(p.weo, 0u);
  if (persist)
    hipLaunchKernelGGL(wsc_walk_persist_kernel<576>, dim3(((nblk + p.wtbe - 1) / p.wtbe + 1) / 2), dim3(576), 0, s, p);
#ifdef LSMGPU_DIAG
  else if (p.wwalk == kWalkGroup && p.wlanes == 8 && p.wbidir == 2)  // 16 lanes forward + 16 backward
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkGroupBi, 8>), dim3((nblk + 7) / 8), dim3(256), 0, s, p);
#endif
  else if (p.wwalk == kWalkGroup && p.wlanes == 8 && LSMGPU_KNOB(p.wbidir, 1u))  // 8 lanes forward + 8 backward
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkGroupBi, 16>),
                       dim3((nblk + 15) / 16 + (LSMGPU_KNOB(p.wcopyfuse, 0u) && !p.wfuse ? p.wncop : 0u)),
                       dim3(256), 0, s, p);
#ifdef LSMGPU_DIAG
  else if (p.wwalk == kWalkGroup && p.wlanes == 2)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkGroup, 128>), dim3((nblk + 127) / 128), dim3(256), 0, s, p);
  else if (p.wwalk == kWalkGroup && p.wlanes == 4)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkGroup, 64>), dim3((nblk + 63) / 64), dim3(256), 0, s, p);
  else if (p.wwalk == kWalkGroup && p.wlanes == 64 && p.wslot == 2)  // from global memory
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkGroup, 4, 32, 0>), dim3((nblk + 3) / 4), dim3(256), 0, s, p);
  else if (p.wwalk == kWalkGroup && p.wlanes == 64 && p.wslot == 1)  // 4 KiB blocks: 7 WGs per CU
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkGroup, 4, 32, kStageSlotSmall>), dim3((nblk + 3) / 4), dim3(256), 0, s, p);
  else if (p.wwalk == kWalkGroup && p.wlanes == 64)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkGroup, 4>), dim3((nblk + 3) / 4), dim3(256), 0, s, p);
  else if (p.wwalk == kWalkGroup && p.wlanes == 32)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkGroup, 8>), dim3((nblk + 7) / 8), dim3(256), 0, s, p);
  else if (p.wwalk == kWalkGroup && p.wlanes == 16)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkGroup, 16>), dim3((nblk + 15) / 16), dim3(256), 0, s, p);
  else if (p.wwalk == kWalkGroup)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkGroup, 32>), dim3((nblk + 31) / 32), dim3(256), 0, s, p);
#endif
  else if (p.wfuse && LSMGPU_KNOB(p.wkeep, 1u) && p.wwide == 576)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkLaneView, 576>), dim3((nblk + p.wtbe - 1) / p.wtbe), dim3(576), 0, s, p);
#ifdef LSMGPU_DIAG
  else if (!p.wfuse && p.wwide == 576 && p.wchunk == 32)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkLane, 576>), dim3((nblk + p.wtbe - 1) / p.wtbe), dim3(576), 0, s, p);
  else if (p.wfuse && p.wkeep && p.wtile == 192)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkLaneView, 192>), dim3((nblk + 191) / 192), dim3(192), 0, s, p);
#endif
  else if (p.wfuse && LSMGPU_KNOB(p.wkeep, 1u))
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkLaneView, 256>), dim3((nblk + 255) / 256), dim3(256), 0, s, p);
#ifdef LSMGPU_DIAG
  else if (p.wchunk == 16)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkLane, 256, 16>), dim3((nblk + 255) / 256), dim3(256), 0, s, p);
  else if (p.wtile == 192)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkLane, 192>), dim3((nblk + 191) / 192), dim3(192), 0, s, p);
  else if (p.wpad) {  // (residency experiments: unused dynamic LDS limits the tiles per CU)
    (void)hipFuncSetAttribute((const void*)wsc_walk_kernel<kWalkLane, 256>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.wpad);
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkLane, 256>), dim3((nblk + 255) / 256), dim3(256), p.wpad, s, p);
  }
#endif
  // a backward lane per block (batches of long blocks: C5 walk 0.183-0.185 -> 0.170-0.172 ms,
  // decode 1,529-1,536 -> 1,557-1,564 GiB/s, view 0.213 -> 0.199 ms, profiles/r06ai)
  else if (p.wlbidir && !p.wfuse && !LSMGPU_KNOB(p.weo, 0u))
    hipLaunchKernelGGL(wsc_walk_bidir_kernel<128>, dim3((nblk + 127) / 128), dim3(256), 0, s, p);
#ifdef LSMGPU_DIAG
  // fewer 256-block tiles than CUs (C5 2^30 B: 32 K blocks of 32 KiB, 128 tiles): smaller tiles
  // so that every CU walks (measured equal, profiles/r06z)
  else if (p.wtile == 128)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkLane, 128>), dim3((nblk + 127) / 128), dim3(128), 0, s, p);
  else if (p.wtile == 64)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkLane, 64>), dim3((nblk + 63) / 64), dim3(64), 0, s, p);
#endif
  else
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkLane, 256>), dim3((nblk + 255) / 256), dim3(256), 0, s, p);
  hipError_t e = hipGetLastError();
#ifdef LSMGPU_STAMPS
  if (e == hipSuccess && p.stamps && !persist) {  // diagnostics: the walk's per-tile timeline
    const uint32_t tb = p.wwalk == kWalkGroup ? (p.wbidir && p.wlanes == 8 ? 16 / p.wbidir : 256 / p.wlanes)
                      : (p.wwide ? p.wtbe : (p.wfuse && p.wkeep && p.wtile == 192) || p.wtile == 192 ? 192
                         : p.wtile == 128 || p.wtile == 64 ? p.wtile : 256);
    const uint32_t nt = (nblk + tb - 1) / tb;
    std::vector<uint64_t> h((size_t)nt * 4);
    uint64_t cnt[4];
    (void)hipMemcpyAsync(cnt, p.stamps + 8, sizeof(cnt), hipMemcpyDeviceToHost, s);
    (void)hipMemcpyAsync(h.data(), p.stamps + 16, h.size() * 8, hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    uint64_t t0 = ~0ull, t1 = 0;
    double walk = 0, look = 0, epi = 0;
    std::vector<double> starts, ends;
    for (uint32_t t = 0; t < nt; t++) {
      const uint64_t* r = &h[4 * (size_t)t];
      t0 = std::min(t0, r[0]);
      t1 = std::max(t1, r[3]);
      walk += (double)(r[1] - r[0]);
      look += (double)(r[2] - r[1]);
      epi += (double)(r[3] - r[2]);
    }
    for (uint32_t t = 0; t < nt; t++) {
      starts.push_back((h[4 * (size_t)t] - t0) / 100.0);
      ends.push_back((h[4 * (size_t)t + 3] - t0) / 100.0);
    }
    std::sort(starts.begin(), starts.end());
    std::sort(ends.begin(), ends.end());
    auto pct = [](const std::vector<double>& v, double q) { return v[(size_t)(q * (v.size() - 1))]; };
    fprintf(stderr, "[lsmgpu] walk stamps (us, %u tiles of %u): span %.2f | per tile: walk %.2f, scan + "
            "look-back %.2f, epilogue %.2f | starts p50 %.2f p90 %.2f max %.2f | ends p10 %.2f p50 %.2f "
            "p90 %.2f max %.2f\n", nt, tb, (t1 - t0) / 100.0, walk / nt / 100.0, look / nt / 100.0,
            epi / nt / 100.0, pct(starts, 0.5), pct(starts, 0.9), starts.back(), pct(ends, 0.1),
            pct(ends, 0.5), pct(ends, 0.9), ends.back());
    if (cnt[2])
      fprintf(stderr, "[lsmgpu] group walk rounds per block: mean %.2f max %llu over %llu blocks, "
              "chains met in %llu\n", (double)cnt[0] / cnt[2], (unsigned long long)cnt[1],
              (unsigned long long)cnt[2], (unsigned long long)cnt[3]);
    if (const char* f = getenv("LSMGPU_STAMPS_FILE")) {
      if (FILE* o = fopen(f, "a")) {
        for (uint32_t t = 0; t < nt; t++)
          fprintf(o, "%u %llu %llu %llu %llu\n", t, (unsigned long long)(h[4 * (size_t)t] - t0),
                  (unsigned long long)(h[4 * (size_t)t + 1] - t0), (unsigned long long)(h[4 * (size_t)t + 2] - t0),
                  (unsigned long long)(h[4 * (size_t)t + 3] - t0));
        fclose(o);
      }
    }
  }
#endif
  if (e == hipSuccess && mid) e = hipEventRecord(mid, s);
  // view-only, or the staged walk copying its blocks: the walk wrote everything
  if (e != hipSuccess || p.wfuse || LSMGPU_KNOB(p.wscopy, 0u) || LSMGPU_KNOB(p.wcopyfuse, 0u)) return e;
  const uint32_t per_wg = 4 / p.wsplit;  // blocks per 4-wave workgroup
  hipLaunchKernelGGL(wsc_copy_kernel, dim3((nblk + per_wg - 1) / per_wg), dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace lsmgpu
