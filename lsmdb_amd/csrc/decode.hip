// decode.hip -- gfx950 SST block decode: the device restatement of blockIterator.Next/parseKV
// (table/iterator.go:93-135) driven over every block of a batch (Iterator.seekToFirst/next,
// iterator.go:201-217,301-326).
//
// Work decomposition ("decode kernel"):
//   tile   = WPB consecutive blocks, one per wave of a workgroup; a persistent, fully
//            resident grid walks the tiles round-robin (tile = blockIdx.x + k * gridDim.x)
//   stage  : each wave's block -> an LDS slot by LDS-DMA (global_load_lds_dwordx4); with
//            NS = 3 slots the next tile's block is in flight during the current iteration
//   walk   : the serial header chain (pos += 10 + klen + vlen), speculated a whole run of
//            equal-size entries per LDS round trip; per entry {header pos, key offset}
//   prefix : tile aggregates -> groups of 64 tiles; the last tile of a group to arrive scans
//            the group, looks back over earlier GROUPS and publishes every member's exclusive
//            output base (8-B {tag, value} granules, agent scope)
//   emit   : SOFTWARE-PIPELINED one tile behind the walk: iteration k walks tile k and
//            publishes its aggregate, then waits for tile k-1's base (published a whole
//            iteration earlier) and writes tile k-1's streams.  Lanes map to aligned 16-B
//            output chunks (J lanes per entry); a chunk is one or two unaligned LDS windows
//            blended at the entry boundary and one dwordx4 store; the stream's partial head /
//            tail chunks are scattered byte-wise (the neighbouring blocks own the rest).
// Blocks larger than the slot, with more entries than the metadata holds, or with prefix-
// compressed keys (plen > 0: never written by table.Builder) take a global-memory
// path with identical semantics.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <mutex>

#include "codec_common.hpp"
#include "decode_common.hpp"
#include "kernels.hpp"

namespace lsmgpu {


// ---- wave primitives: DPP row_shr inside each 16-lane row, the four rows combined through
// v_readlane (scalar).  (No row_bcast: its row-masked forms are not relied on here.)
__device__ __forceinline__ uint32_t row_incl_add(uint32_t v) {
  v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true);   // row_shr:1
  v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, true);   // row_shr:2
  v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, true);   // row_shr:4
  v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, true);   // row_shr:8
  return v;
}
// inclusive scan over the wave; `total` = the wave's sum (uniform)
__device__ __forceinline__ uint32_t wave_incl_add(uint32_t v, uint32_t lane, uint32_t& total) {
  v = row_incl_add(v);
  const uint32_t r0 = readlane(v, 15), r1 = r0 + readlane(v, 31), r2 = r1 + readlane(v, 47);
  total = r2 + readlane(v, 63);
  const uint32_t row = lane >> 4;
  return v + (row == 0 ? 0u : row == 1 ? r0 : row == 2 ? r1 : r2);
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {  // uniform result
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, true));
  return max(max(readlane(v, 15), readlane(v, 31)), max(readlane(v, 47), readlane(v, 63)));
}

// ---- speculative walk of a block held in LDS, exactly equivalent to the iterator's walk.
// The chain pos_{e+1} = pos_e + 10 + klen_e + vlen_e is serial, but SST entries of a block
// mostly share one size: each round lane i reads the header guessed at pos + i*stride, a
// ballot finds the first lane whose entry stops the iterator (end, terminator, error) or
// whose size differs from the stride, and every lane before it is a confirmed entry.  A
// round therefore advances over a whole run of equal-size entries with ONE LDS round trip.
// meta[e] = header pos | klen << 16 for e < maxe.
struct SpecResult {
  uint32_t n, status, stop;  // stop = position just after the last entry (its successor's header)
  bool any_plen;
  uint32_t rounds;
};
// Status of the iterator at a position where no entry was confirmed.
__device__ __forceinline__ uint32_t stop_status(const LdsSrc& src, uint32_t pf, uint32_t len,
                                                uint32_t base_pos, bool first) {
  if (pf >= len) return LSMGPU_BLK_OK;                    // io.EOF (iterator.go:115-118)
  if (len - pf < 10) return LSMGPU_BLK_TRUNC_HEADER;
  const Hdr h = src.hdr(pf);
  if ((h.klen | h.plen) == 0) return LSMGPU_BLK_OK;       // terminator (iterator.go:124-127)
  if (first && h.plen != 0) return LSMGPU_BLK_FIRST_PLEN; // iterator.go:131
  if (base_pos + h.plen > len) return LSMGPU_BLK_PREFIX_OOB;
  return LSMGPU_BLK_VALUE_OVERFLOW;                       // iterator.go:103-106
}

__device__ __forceinline__ SpecResult walk_spec(const uint8_t* slot, uint32_t sh, uint32_t len,
                                                uint32_t* meta, uint32_t maxe, uint32_t lane) {
  const LdsSrc src{slot, sh};
  // first entry (uniform): defines baseKey (iterator.go:129-133) and the first stride guess
  if (len < 10) return SpecResult{0, stop_status(src, 0, len, 10, true), 0, false, 0};
  const Hdr h0 = src.hdr(0);
  const uint32_t base_pos = 10;
  const uint32_t sz0 = 10 + h0.klen + h0.vlen;
  if ((h0.klen | h0.plen) == 0 || h0.plen != 0 || sz0 > len)
    return SpecResult{0, stop_status(src, 0, len, base_pos, true), 0, false, 0};
  if (lane == 0 && maxe > 0) meta[0] = h0.klen << 16;
  uint32_t pos = sz0, stride = sz0, n = 1, ls = lane * sz0;
  uint64_t plen_m = 0;
  uint32_t rounds = 0;
  for (;;) {
    rounds++;
    // lane i checks the entry guessed at pos + i * stride (branch-free)
    const uint32_t p = pos + ls;
    const bool has = p + 10 <= len;
    const Hdr h = src.hdr(has ? p : 0u);
    const uint32_t sz = 10 + h.klen + h.vlen;
    const bool ok = has & ((h.klen | h.plen) != 0) & (base_pos + h.plen <= len) & (p + sz <= len);
    const uint64_t okm = __builtin_amdgcn_ballot_w64(ok);
    const uint64_t run = okm & __builtin_amdgcn_ballot_w64(sz == stride);
    const uint64_t brk = ~run;  // the first lane that does not continue the run
    const uint32_t f = brk ? (uint32_t)__builtin_ctzll(brk) : 64u;
    const uint32_t fok = f < 64 ? (uint32_t)(okm >> f) & 1u : 0u;
    const uint32_t m = f + fok;  // confirmed entries: lanes [0, m)
    const bool conf = lane < m;
    if (conf & (n + lane < maxe)) meta[n + lane] = p | (h.klen << 16);
    plen_m |= __builtin_amdgcn_ballot_w64(conf & (h.plen != 0));
    n += m;
    if (f == 64) {  // 64 entries of exactly `stride` bytes
      pos += 64 * stride;
      continue;
    }
    const uint32_t pf = readlane(p, f);
    if (!fok) return SpecResult{n, stop_status(src, pf, len, base_pos, false), pf, plen_m != 0, rounds};
    const uint32_t szf = readlane(sz, f);  // entry f has another size: continue after it
    pos = pf + szf;
    if (f == 0) {  // the guess failed at once: adopt the new size
      stride = szf;
      ls = lane * szf;
    }
  }
}

// Per-block emit plan (uniform).  kind: 0 nothing to write, 1 LDS fast path, 2 global path.
struct Plan {
  uint32_t n, K, V, status;
  uint32_t off, len, sh;
  uint32_t kind;
  uint32_t jk, jv;       // log2(lanes per entry) of the key / value streams
  uint32_t ku;           // the common key length of every entry, 0 if they differ
  uint32_t big;          // every key and every value is >= 16 B (16-B pieces only)
  uint32_t jkv;          // log2(lanes per entry) for key + value pieces together
};

// After walk_spec: meta[e] := header pos | key offset << 16 (wave scan of klen), sentinel
// meta[n] = stop | K << 16; derives the stream sizes, lanes-per-entry and the 2-run flags.
// Requires n <= maxe (meta holds maxe + 2 words).
// Pieces of an entry stream of `len` bytes: 16-B pieces (the last overlapping back inside the
// entry) from 16 B up; below that two overlapping pieces of the largest power of two <= len.
__device__ __forceinline__ uint32_t n_pieces(uint32_t len) {
  return len >= 16 ? (len + 15) >> 4 : (len >= 2 ? 2u : len);
}
__device__ __forceinline__ uint32_t piece_log2(uint32_t len) {  // log2 of the piece size
  return len >= 16 ? 4u : len >= 8 ? 3u : len >= 4 ? 2u : len >= 2 ? 1u : 0u;
}

__device__ __forceinline__ void finish_meta(uint32_t* meta, const SpecResult& r, uint32_t lane,
                                            Plan& pl) {
  if (lane == 0) meta[r.n] = r.stop;  // klen field 0: the walk's successor position
  wave_lds_fence();
  uint32_t K = 0, kl0 = 0;
  bool nonuni = false, small = false;
  uint32_t jk = 0, jv = 0, jkv = 0;
  // lanes per entry = pieces of the longest entry, rounded up to a power of two (ballots)
  auto jl_of = [](uint32_t len, bool on) -> uint32_t {
    const uint32_t pc = len >= 16 ? (len + 15) >> 4 : 2u;
    uint32_t j = 0;
    j = __ballot(on && pc > 1) ? 1u : j;
    j = __ballot(on && pc > 2) ? 2u : j;
    j = __ballot(on && pc > 4) ? 3u : j;
    j = __ballot(on && pc > 8) ? 4u : j;
    j = __ballot(on && pc > 16) ? 5u : j;
    j = __ballot(on && pc > 32) ? 6u : j;
    return j;
  };
  for (uint32_t e0 = 0; e0 < r.n; e0 += kWave) {
    const uint32_t e = e0 + lane;
    const bool on = e < r.n;
    uint2 w = make_uint2(0, 0);
    if (on) __builtin_memcpy(&w, meta + e, 8);  // meta[e], meta[e + 1]
    const uint32_t p = w.x & 0xffffu, kl = w.x >> 16, p1 = w.y & 0xffffu;
    const uint32_t vl = on ? p1 - p - 10 - kl : 0u;
    uint32_t ksum;
    const uint32_t inc = wave_incl_add(kl, lane, ksum);
    wave_lds_fence();  // every lane has read meta[e + 1] before it is rewritten
    if (on) meta[e] = p | ((K + inc - kl) << 16);
    K += ksum;
    if (e0 == 0) kl0 = readlane(kl, 0);
    nonuni = nonuni || __ballot(on && kl != kl0) != 0;
    small = small || __ballot(on && (kl < 16 || vl < 16)) != 0;
    jk = max(jk, jl_of(kl, on));
    jv = max(jv, jl_of(vl, on));
    jkv = max(jkv, jl_of(16 * (n_pieces(kl) + n_pieces(vl)), on));
  }
  if (lane == 0) meta[r.n] = r.stop | (K << 16);
  wave_lds_fence();
  pl.n = r.n;
  pl.K = K;
  pl.V = r.stop - 10 * r.n - K;
  pl.jk = jk;
  pl.jv = jv;
  pl.ku = nonuni ? 0u : kl0;
  pl.big = small ? 0u : 1u;
  pl.jkv = jkv;
}


// A group = 64 consecutive blocks (all in one round of the persistent grid).  Every block
// publishes its aggregate {entries, key bytes, value bytes} (lb[b][0..2], fire and forget);
// one member per group and round -- rotating with the round, so no workgroup is always the
// slow one -- collects the group's aggregates, scans them, looks back over earlier groups
// and publishes every member's exclusive prefix (lb[b][4..6]).  No returning atomics.
__device__ void group_lead(const DecodeParams& p, uint32_t b, uint64_t tag, uint32_t lane) {
  const uint32_t g = b >> 6;
  const uint32_t g0 = g << 6;
  const uint32_t gsize = (p.nblk - g0 < 64u) ? (p.nblk - g0) : 64u;
  uint32_t a = 0, bk = 0, c = 0;
  for (SpinBound bound;;) {
    bool ok = true;
    if (lane < gsize) ok = read3(p.lb + (uint64_t)(g0 + lane) * 8, tag, a, bk, c);
    if (__all(ok)) break;
    if (bound.expired()) {
      flag_timeout(p.result, lane);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  const uint32_t ia = wave_scan_sat(a, lane), ib = wave_scan_sat(bk, lane),
                 ic = wave_scan_sat(c, lane);
  const uint32_t ta = readlane(ia, gsize - 1), tb = readlane(ib, gsize - 1),
                 tc = readlane(ic, gsize - 1);
  uint64_t* Gr = p.glb + (uint64_t)g * 8;
  Tot pg{0, 0, 0};
  if (g > 0) {
    store3(Gr, tag, ta, tb, tc, lane);
    pg = lookback(p.glb, g, tag, lane, p.result);
  }
  store3(Gr + 4, tag, sat_add(pg.n, ta), sat_add(pg.k, tb), sat_add(pg.v, tc), lane);
  // exclusive = group prefix + inclusive - own (own <= inclusive unless saturated)
  const uint32_t ea = sat_add(pg.n, ia - a), eb = sat_add(pg.k, ib == 0xffffffffu ? ib : ib - bk),
                 ec = sat_add(pg.v, ic - c);
  if (lane < gsize) {
    uint64_t* Xj = p.lb + (uint64_t)(g0 + lane) * 8 + 4;
    gstore(Xj + 0, (tag << kTagShift) | ea);
    gstore(Xj + 1, (tag << kTagShift) | eb);
    gstore(Xj + 2, (tag << kTagShift) | ec);
  }
}

// Block b's exclusive prefix from a granule poll issued earlier (lanes 0..2 hold x); polls
// again until the group leader has published it.
__device__ __forceinline__ Tot prefix_of(const DecodeParams& p, uint32_t b, uint64_t x,
                                         uint64_t tag, uint32_t lane) {
  const uint64_t* X = p.lb + (uint64_t)b * 8 + 4;
  for (SpinBound bound;;) {
    const bool ok = lane >= 3 || (x >> kTagShift) == tag;
    if (__all(ok)) {
      const uint32_t v = (uint32_t)x;
      return Tot{readlane(v, 0), readlane(v, 1), readlane(v, 2)};
    }
    if (bound.expired()) {
      flag_timeout(p.result, lane);
      return Tot{0, 0, 0};
    }
    __builtin_amdgcn_s_sleep(1);
    if (lane < 3) x = gload(X + lane);
  }
}

// ---------------------------------------------------------------------------------- emit
// Entry e of one stream: output range [o, o1) comes from block bytes starting at s.
// meta[e] = header pos | key offset << 16 (sentinel at n).
template <bool IS_KEY>
__device__ __forceinline__ void entry_span(const uint32_t* meta, uint32_t e, uint32_t& o,
                                           uint32_t& o1, uint32_t& s) {
  uint2 w;
  __builtin_memcpy(&w, meta + e, 8);  // meta[e], meta[e + 1]: one ds_read_b64
  const uint32_t p0 = w.x & 0xffffu, k0 = w.x >> 16, p1 = w.y & 0xffffu, k1 = w.y >> 16;
  if (IS_KEY) {
    o = k0;
    o1 = k1;
    s = p0 + 10;
  } else {
    o = p0 - 10 * e - k0;
    o1 = p1 - 10 * (e + 1) - k1;
    s = p0 + 10 + (k1 - k0);
  }
}

// One stream (keys or values) of one block.  Entry e's bytes [o, o1) are copied as pieces of
// `sz` bytes (16, or 8/4/2/1 for entries shorter than 16): piece j covers entry bytes
// [min(j*sz, len - sz), +sz) -- the last piece overlaps back inside the entry, so no store
// ever touches a byte outside it (no read-modify-write, no cross-block ownership).  Loads
// and stores are unaligned (one ds_read_b128 + one global_store_dwordx4 for a 16-B piece).
// J = 2^jl lanes per entry; pieces beyond J are looped.
template <bool IS_KEY>
__device__ __forceinline__ void emit_pieces(uint8_t* dst, const uint8_t* src, const uint32_t* meta,
                                            uint32_t n, uint32_t jl, uint32_t lane) {
  const uint32_t J = 1u << jl;
  const uint32_t epi = kWave >> jl;  // entries per wave iteration
  const uint32_t j0 = lane & (J - 1);
  for (uint32_t e0 = 0; e0 < n; e0 += epi) {
    const uint32_t e = e0 + (lane >> jl);
    if (e >= n) continue;
    uint32_t o, o1, s;
    entry_span<IS_KEY>(meta, e, o, o1, s);
    const uint32_t len = o1 - o;
    const uint32_t sz = len >= 16 ? 16u : len >= 8 ? 8u : len >= 4 ? 4u : len >= 2 ? 2u : len;
    const uint32_t np = len >= 16 ? (len + 15) >> 4 : (len > sz ? 2u : (len ? 1u : 0u));
    for (uint32_t j = j0; j < np; j += J) {
      const uint32_t off = min(j * sz, len - sz);
      const uint8_t* sp = src + s + off;
      uint8_t* dp = dst + o + off;
      if (sz == 16) {
        uint4 v;
        __builtin_memcpy(&v, sp, 16);
        __builtin_memcpy(dp, &v, 16);
      } else if (sz == 8) {
        uint2 v;
        __builtin_memcpy(&v, sp, 8);
        __builtin_memcpy(dp, &v, 8);
      } else if (sz == 4) {
        uint32_t v;
        __builtin_memcpy(&v, sp, 4);
        __builtin_memcpy(dp, &v, 4);
      } else if (sz == 2) {
        uint16_t v;
        __builtin_memcpy(&v, sp, 2);
        __builtin_memcpy(dp, &v, 2);
      } else {
        *dp = *sp;
      }
    }
  }
}

// Global-memory path with the same semantics: re-walks the block and copies every entry's
// key and value with the wave's lanes (byte granular).  Oversize / prefix-compressed blocks.
__device__ void emit_slow(const DecodeParams& p, const uint8_t* blk, uint32_t n, uint64_t ebase,
                          uint64_t kbase, uint64_t vbase, uint64_t off, uint32_t lane) {
  GlobalSrc src{blk};
  uint32_t pos = 0, base_pos = 0;
  uint64_t kb = kbase, vb = vbase;
  for (uint32_t e = 0; e < n; e++) {
    const Hdr hd = src.hdr(pos);
    pos += 10;
    if (e == 0) base_pos = pos;
    const uint32_t ks = pos, vs = pos + hd.klen;
    if (p.mode & LSMGPU_MODE_MATERIALIZE) {
      const uint32_t kl = hd.plen + hd.klen;
      if (p.key_data)
        for (uint32_t i = lane; i < kl; i += kWave)
          p.key_data[kb + i] = (i < hd.plen) ? blk[base_pos + i] : blk[ks + i - hd.plen];
      if (p.val_data)
        for (uint32_t i = lane; i < hd.vlen; i += kWave) p.val_data[vb + i] = blk[vs + i];
      kb += kl;
      vb += hd.vlen;
      if (lane == 0) {
        if (p.key_end) p.key_end[ebase + e] = (uint32_t)kb;
        if (p.val_end) p.val_end[ebase + e] = (uint32_t)vb;
      }
    }
    if ((p.mode & LSMGPU_MODE_VIEW) && p.view && lane == 0)
      p.view[ebase + e] = (uint64_t)(uint32_t)(off + ks) | ((uint64_t)hd.klen << 32) |
                          ((uint64_t)hd.vlen << 48);
    pos = vs + hd.vlen;
  }
}

typedef __attribute__((address_space(1))) void glb_void_t;


// Walk one block (its bytes already in `slot` when it fits): the emit plan + meta.
template <int SLOT, int MAXE, bool NO_GLOBAL = false>
__device__ __forceinline__ Plan walk_stage(const DecodeParams& p, const BlockRef& ref, bool valid,
                                           uint8_t* slot, uint32_t* meta, uint32_t lane,
                                           uint64_t* spec_acc = nullptr) {
  Plan pl{};
  if (!valid) return pl;
  pl.off = ref.off;
  pl.len = ref.len;
  pl.sh = ref.sh;
  if ((uint64_t)ref.off + ref.len > p.data_len) {
    pl.status = LSMGPU_BLK_RANGE;
    return pl;
  }
  if ABLATE(p, 4) return pl;
  if (ref.fits) {
    if (ref.tail) land_tail(p, ref, slot, lane);
    wave_lds_fence();
#ifdef LSMGPU_STAMPS
    const uint64_t t0 = spec_acc ? __builtin_amdgcn_s_memtime() : 0;
#endif
    const SpecResult r = walk_spec(slot, ref.sh, ref.len, meta, MAXE, lane);
#ifdef LSMGPU_STAMPS
    if (spec_acc) {
      spec_acc[0] += __builtin_amdgcn_s_memtime() - t0;
      spec_acc[1] += r.rounds;
    }
#endif
    pl.status = r.status;
    if (r.n <= (uint32_t)MAXE && !r.any_plen) {
      finish_meta(meta, r, lane, pl);
      pl.kind = pl.n ? 1u : 0u;
      return pl;
    }
    if (NO_GLOBAL) {  // rare: counts from a serial walk of the LDS copy; global emit path
      const WalkResult w = walk_block(LdsSrc{slot, ref.sh}, ref.len);
      pl.n = w.n;
      pl.K = w.K;
      pl.V = w.V;
      pl.kind = w.n ? 2u : 0u;
      return pl;
    }
  }
  if constexpr (NO_GLOBAL) return pl;  // (never: every block of this kernel fits its slot)
  const WalkResult w = walk_block(GlobalSrc{p.data + ref.off}, ref.len);
  pl.n = w.n;
  pl.K = w.K;
  pl.V = w.V;
  pl.status = w.status;
  pl.kind = w.n ? 2u : 0u;
  return pl;
}

// Write one block's outputs at its global bases.
__device__ __forceinline__ void emit_block(const DecodeParams& p, const Plan& pl, uint32_t b,
                                           Tot ex, const uint8_t* slot, const uint32_t* meta,
                                           uint32_t lane) {
  if (lane == 0) {
    if (p.blk_first) p.blk_first[b] = ex.n;
    if (p.blk_status) p.blk_status[b] = (int32_t)pl.status;
    if (pl.status != LSMGPU_BLK_OK) {
      atomicAdd(reinterpret_cast<unsigned long long*>(p.result + 4), 1ull);
      atomicMax(reinterpret_cast<unsigned long long*>(p.result + 3),
                (unsigned long long)(p.nblk - b));
    }
  }
  const bool mat = (p.mode & LSMGPU_MODE_MATERIALIZE) != 0;
  const bool view = (p.mode & LSMGPU_MODE_VIEW) != 0 && p.view;
  bool ok = (uint64_t)ex.n + pl.n <= p.ent_cap;
  if (mat) {
    const uint64_t kend = (uint64_t)ex.k + pl.K, vend = (uint64_t)ex.v + pl.V;
    ok = ok && (kend <= p.key_cap || !p.key_data) && (vend <= p.val_cap || !p.val_data);
    ok = ok && kend < 0xffffffffull && vend <= 0xffffffffull;
  }
  if (!ok && lane == 0) atomicOr(reinterpret_cast<unsigned long long*>(p.result + 5), 1ull);
  if (!ok || pl.kind == 0 || ABLATE(p, 2)) return;
  if (pl.kind == 2) {
    emit_slow(p, p.data + pl.off, pl.n, ex.n, ex.k, ex.v, pl.off, lane);
    return;
  }
  // per-entry end offsets / view records (lane per entry)
  for (uint32_t e = lane; e < pl.n; e += kWave) {
    const uint32_t w0 = meta[e], w1 = meta[e + 1];
    const uint32_t p0 = w0 & 0xffffu, k0 = w0 >> 16, p1 = w1 & 0xffffu, k1 = w1 >> 16;
    const uint32_t vo1 = p1 - 10 * (e + 1) - k1;
    if (mat) {
      if (p.key_end) p.key_end[ex.n + e] = ex.k + k1;
      if (p.val_end) p.val_end[ex.n + e] = ex.v + vo1;
    }
    if (view) {
      const uint32_t klen = k1 - k0, vlen = vo1 - (p0 - 10 * e - k0);
      p.view[ex.n + e] = (uint64_t)(pl.off + p0 + 10) | ((uint64_t)klen << 32) |
                         ((uint64_t)vlen << 48);
    }
  }
  if (!mat) return;
  const uint8_t* src = slot + pl.sh;  // block byte 0
  if (p.key_data) emit_pieces<true>(p.key_data + ex.k, src, meta, pl.n, pl.jk, lane);
  if (p.val_data) emit_pieces<false>(p.val_data + ex.v, src, meta, pl.n, pl.jv, lane);
}

// The walk's plan of a block, parked in LDS next to its metadata until the block is emitted
// (two iterations later).
constexpr int kPlanWords = 12;
__device__ __forceinline__ void plan_store(uint32_t* rec, const Plan& pl, uint32_t lane) {
  const uint32_t v[kPlanWords] = {pl.n, pl.K, pl.V, pl.status, pl.off, pl.len, pl.sh, pl.kind, pl.jk, pl.jv, pl.ku, pl.big};
  if (lane < (uint32_t)kPlanWords) {
    uint32_t x = v[0];
#pragma unroll
    for (int i = 1; i < kPlanWords; i++) x = lane == (uint32_t)i ? v[i] : x;
    rec[lane] = x;
  }
}
__device__ __forceinline__ Plan plan_load(const uint32_t* rec) {
  Plan pl;
  pl.n = uniform(rec[0]);
  pl.K = uniform(rec[1]);
  pl.V = uniform(rec[2]);
  pl.status = uniform(rec[3]);
  pl.off = uniform(rec[4]);
  pl.len = uniform(rec[5]);
  pl.sh = uniform(rec[6]);
  pl.kind = uniform(rec[7]);
  pl.jk = uniform(rec[8]);
  pl.jv = uniform(rec[9]);
  pl.ku = uniform(rec[10]);
  pl.big = uniform(rec[11]);
  return pl;
}

template <int SLOT, int MAXE, int NS>
struct DecodeCfg {
  static_assert(NS >= 3, "the emit lags the walk by NS - 2 >= 1 blocks");
  static constexpr int kLag = NS - 2;
  static constexpr int kBuf = SLOT + 16;                  // block at shift < 16, 16-B DMA pieces
  static constexpr int kNM = NS - 1;                      // metadata of blocks k-kLag .. k
  static constexpr int kMetaWords = MAXE + 2 + kPlanWords + 2;  // {pos|koff<<16}[n+1], plan
  static constexpr int kLds = NS * kBuf + kNM * kMetaWords * 4;
  static constexpr int kIters = (SLOT + 16 + 16 * kWave - 1) / (16 * kWave);  // 1-KiB DMA pieces
};

// Residency census: every workgroup arrives and waits (bounded, 2 ms) for the whole grid.
__device__ void census(uint32_t* c, uint32_t lane) {
  if (lane != 0) return;
  atomicAdd(c, 1u);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  while (__builtin_amdgcn_s_memrealtime() - t0 < 200000ull) {
    if (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= gridDim.x) {
      atomicAdd(c + 1, 1u);
      return;
    }
    __builtin_amdgcn_s_sleep(8);
  }
}

__device__ __forceinline__ uint64_t stamp() { return __builtin_amdgcn_s_memtime(); }

// One wave per workgroup; workgroup w decodes blocks w, w + G, w + 2G, ... (G = grid size, a
// multiple of 64, fully resident).  Iteration k (one vmcnt drain per iteration):
//   a. s_waitcnt vmcnt(0): block k's LDS-DMA, block k-L's prefix poll and block k-L-1's
//      stores, all issued one iteration (a whole walk) ago
//   b. emit block k-L (its base from the poll; L = NS - 2 = 2 blocks behind the walk)
//   c. issue block k+1's LDS-DMA (into block k-L-1's slot) and block k-L+1's prefix poll
//   d. walk block k from LDS, park its plan, publish its aggregate; the round's group leader
//      publishes its group's prefixes
template <int SLOT, int MAXE, int NS>
__global__ void __launch_bounds__(64) decode_kernel(DecodeParams p) {
  using Cfg = DecodeCfg<SLOT, MAXE, NS>;
  constexpr uint32_t L = Cfg::kLag;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = lane_id();
  if (p.census) {
    census(p.census, lane);
    return;
  }
  const uint32_t G = gridDim.x, w = blockIdx.x, nblk = p.nblk;
  const uint64_t tag = p.tag;
  const uint32_t K = w < nblk ? (nblk - 1 - w) / G + 1 : 0;  // this workgroup's blocks
  uint32_t* meta_base = reinterpret_cast<uint32_t*>(smem + NS * Cfg::kBuf);
  auto slot_of = [&](uint32_t k) -> uint8_t* { return smem + (k % NS) * Cfg::kBuf; };
  auto meta_of = [&](uint32_t k) -> uint32_t* { return meta_base + (k % Cfg::kNM) * Cfg::kMetaWords; };
  auto blk_of = [&](uint32_t k) -> uint32_t { return w + k * G; };
  // lane i holds [off, len) of block k0 + i of this workgroup: 64 iterations per load
  uint32_t ring_k0 = 0, ring_off = 0, ring_len = 0;
  auto ring_load = [&](uint32_t k0) {
    ring_k0 = k0;
    const uint64_t b = (uint64_t)w + (uint64_t)(k0 + lane) * G;
    ring_off = b < nblk ? p.blk_off[b] : 0u;
    ring_len = b < nblk ? p.blk_len[b] : 0u;
  };
#ifdef LSMGPU_STAMPS
  // diagnostic build only (LSMGPU_BUILD_DIAG=1): per-phase s_memtime totals
  const bool st = p.stamps != nullptr;
  uint64_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t tprev = st ? stamp() : 0;
  auto mark = [&](int i) {
    if (st) {
      const uint64_t t = stamp();
      acc[i] += t - tprev;
      tprev = t;
    }
  };
  uint64_t* spec_acc = st ? &acc[6] : nullptr;
#else
  auto mark = [](int) {};
  uint64_t* spec_acc = nullptr;
#endif

  BlockRef ref_next{0, 0, 0, false, false};
  if (K > 0) {
    ring_load(0);
    ref_next = prefetch_block<SLOT, Cfg::kIters>(p, readlane(ring_off, 0), readlane(ring_len, 0),
                                                 slot_of(0), lane);
  }
  uint64_t poll = 0;
  for (uint32_t k = 0; k < K + L; k++) {
    // a. one drain for everything issued an iteration ago
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const BlockRef ref = ref_next;
    mark(0);
    // b. emit block k - L
    if (k >= L) {
      const uint32_t ke = k - L, be = blk_of(ke);
      Tot ex{0, 0, 0};
      if (!ABLATE(p, 1)) ex = prefix_of(p, be, poll, tag, lane);
      mark(5);
      const uint32_t* rec = meta_of(ke);
      const Plan pl = plan_load(rec + MAXE + 2);
      if (be == nblk - 1 && lane == 0) {  // totals of the whole batch
        if (p.blk_first) p.blk_first[nblk] = ex.n + pl.n;
        p.result[0] = sat_add(ex.n, pl.n);
        p.result[1] = sat_add(ex.k, pl.K);
        p.result[2] = sat_add(ex.v, pl.V);
      }
      emit_block(p, pl, be, ex, slot_of(ke), rec, lane);
    }
    mark(1);
    // c. next block's bytes, the next emit's prefix poll
    if (k + 1 < K) {
      if (k + 1 - ring_k0 >= (uint32_t)kWave) ring_load(k + 1);
      const uint32_t i = k + 1 - ring_k0;
      ref_next = prefetch_block<SLOT, Cfg::kIters>(p, readlane(ring_off, i), readlane(ring_len, i),
                                                   slot_of(k + 1), lane);
    }
    if (k + 1 >= L && k + 1 - L < K && lane < 3 && !ABLATE(p, 1))
      poll = gload(p.lb + (uint64_t)blk_of(k + 1 - L) * 8 + 4 + lane);
    mark(2);
    // d. walk block k
    if (k < K) {
      const uint32_t b = blk_of(k);
      uint32_t* rec = meta_of(k);
      wave_lds_fence();
      const Plan pl = walk_stage<SLOT, MAXE>(p, ref, true, slot_of(k), rec, lane, spec_acc);
      plan_store(rec + MAXE + 2, pl, lane);
      mark(3);
      if (!ABLATE(p, 1)) {
        store3(p.lb + (uint64_t)b * 8, tag, pl.n, pl.K, pl.V, lane);
        const uint32_t g0 = b & ~63u;
        const uint32_t gsize = (nblk - g0 < 64u) ? (nblk - g0) : 64u;
        if ((b - g0) == (b / G) % gsize) group_lead(p, b, tag, lane);
      }
      mark(4);
    }
    wave_lds_fence();
  }
#ifdef LSMGPU_STAMPS
  if (st && lane == 0) {
#pragma unroll
    for (int i = 0; i < 8; i++) atomicAdd(reinterpret_cast<unsigned long long*>(p.stamps + i), acc[i]);
    atomicAdd(reinterpret_cast<unsigned long long*>(p.stamps + 8), (unsigned long long)(K + L));
    atomicAdd(reinterpret_cast<unsigned long long*>(p.stamps + 9), 1ull);
  }
#endif
}

// ====================================================================== 4 KiB blocks
// Register-lag variant (blocks <= 4 KiB: the BASELINE C2 shape).  After block k is walked
// its key and value streams are compacted into an LDS staging buffer (overlapping unaligned
// pieces) and read back as <= 5 16-B chunks per lane: the block's OUTPUT then waits for its
// prefix in VGPRs, not in LDS, so the emit can lag the walk by L = 3 blocks with only two
// block slots + one staging buffer of LDS per wave (~12.9 KB -> 12 waves/CU).  The emit is
// then <= 5 contiguous global_store_dwordx4 (the stream's last chunk overlaps back inside it)
// plus the per-entry end offsets, with no LDS traffic.
constexpr int kRegChunks = 5;  // 320 chunks per block >= (4096 + 16 + 16) / 16
struct Pend {
  uint4 c[kRegChunks];          // chunk mode: chunk q = 64 s + lane of [key stream | value stream]
                                // piece mode: this lane's s-th 16-B piece
  uint32_t po[(kRegChunks + 1) / 2];  // piece mode, 16 bits per piece: stream offset (12 b) |
                                      // log2 size << 12 | value stream << 15; 0xffff = none
  uint32_t end0, end1;          // entries lane, 64 + lane: key end | value end << 16 (in-block)
  uint32_t sc;                  // lane i = field i: n, K, V, status, off, len, kind, mode
};
constexpr uint32_t kValueBit = 0x8000u;
constexpr uint32_t kNoPiece = 0xffffu;

// Entry e's exclusive ends within its block: key end | value end << 16 (both < 4 KiB).
__device__ __forceinline__ uint32_t ends_word(const uint32_t* meta, uint32_t e) {
  const uint32_t w1 = meta[e + 1];
  const uint32_t k1 = w1 >> 16, vo1 = (w1 & 0xffffu) - 10 * (e + 1) - k1;
  return (k1 & 0xffffu) | (vo1 << 16);
}

template <int MAXE>
struct RegCfg {
  static_assert(MAXE >= 128, "entry meta words for 128 entries are held in registers");
  static constexpr int kSlot = 4096;
  static constexpr int kBuf = kSlot + 16;
  static constexpr int kStage = kSlot + 32;
  static constexpr int kMetaWords = MAXE + 2;
  static constexpr int kMetaBytes = (kMetaWords * 4 + 15) & ~15;
  static constexpr int kLds = kMetaBytes + kStage + 2 * kBuf;
  static constexpr int kIters = (kSlot + 16 + 16 * kWave - 1) / (16 * kWave);
};

__device__ __forceinline__ uint32_t chunk_off(uint32_t q, uint32_t Q, uint32_t L) {
  return q + 1 == Q ? L - 16 : 16 * q;  // the last chunk overlaps back inside the stream
}

// Bytes [0, x) from a, [x, 16) from b (0 <= x <= 16).
__device__ __forceinline__ uint32_t lo_mask(int32_t x, int32_t d) {
  int32_t sft = 32 - 8 * (x - 4 * d);  // bytes of dword d below x -> keep mask
  sft = sft < 0 ? 0 : (sft > 32 ? 32 : sft);
  return (uint32_t)(0xffffffffull >> sft);
}
__device__ __forceinline__ uint4 blend_at(const uint4& a, const uint4& b, int32_t x) {
  uint4 r;
  uint32_t m;
  m = lo_mask(x, 0); r.x = (a.x & m) | (b.x & ~m);
  m = lo_mask(x, 1); r.y = (a.y & m) | (b.y & ~m);
  m = lo_mask(x, 2); r.z = (a.z & m) | (b.z & ~m);
  m = lo_mask(x, 3); r.w = (a.w & m) | (b.w & ~m);
  return r;
}

// One stream (keys or values) of one block assembled into `stage` (16-B aligned) as aligned
// 16-B chunks: chunk q = stream bytes [16q, 16q + 16).  Entry e owns the chunks whose first
// byte lies in [o(e), o(e+1)); J = 2^jl lanes per entry.  A chunk is one dword-aligned
// window of its owner (5 ds_read_b32 + v_alignbyte; `win` has >= 16 addressable bytes before
// the block) blended at the entry boundary with its successor's window (`two`: every entry
// >= 16 B, so two runs suffice) or run by run (general).  Every LDS access is aligned.
template <bool IS_KEY>
__device__ __forceinline__ void assemble_stream(uint8_t* stage, const uint8_t* win, uint32_t wsh,
                                                const uint32_t* meta, uint32_t n, uint32_t L,
                                                uint32_t jl, bool two, uint32_t lane) {
  const uint32_t Q = (L + 15) >> 4;
  const uint32_t J = 1u << jl;
  const uint32_t epi = kWave >> jl;
  const uint32_t j0 = lane & (J - 1);
  if (two && jl < 6) {
    // every entry >= 16 B and <= J chunks per entry: batches of NB entries per lane.  Every
    // LDS read is UNCONDITIONAL (indices clamped into [0, n]; results selected afterwards):
    // a read under a divergent branch gets its own lgkmcnt wait and serialises the batch.
    constexpr int NB = 2;
    for (uint32_t e0 = 0; e0 < n; e0 += NB * epi) {
      uint32_t m0[NB], m1[NB], m2[NB], eidx[NB];
#pragma unroll
      for (int i = 0; i < NB; i++) {
        const uint32_t e = e0 + i * epi + (lane >> jl);
        eidx[i] = e;
        const uint32_t ec = min(e, n - 1);
        m0[i] = meta[ec];
        m1[i] = meta[ec + 1];
        m2[i] = meta[min(ec + 2, n)];
      }
      uint32_t t0[NB], x[NB], a1[NB], a2[NB];
      bool on[NB];
#pragma unroll
      for (int i = 0; i < NB; i++) {
        const uint32_t e = eidx[i];
        const uint32_t p0 = m0[i] & 0xffffu, k0 = m0[i] >> 16, p1 = m1[i] & 0xffffu,
                       k1 = m1[i] >> 16, k2 = m2[i] >> 16;
        uint32_t o, o1, sp, s1;
        if (IS_KEY) {
          o = k0;
          o1 = k1;
          sp = p0 + 10;
          s1 = p1 + 10;
        } else {
          o = p0 - 10 * e - k0;
          o1 = p1 - 10 * (e + 1) - k1;
          sp = p0 + 10 + (k1 - k0);
          s1 = p1 + 10 + (k2 - k1);
        }
        const uint32_t qa = (o + 15) >> 4;
        const uint32_t qb = (e + 1 >= n) ? Q : (o1 + 15) >> 4;
        const uint32_t q = qa + j0;
        on[i] = e < n && q < qb;
        t0[i] = 16 * q;
        const int32_t xi = (int32_t)o1 - (int32_t)(16 * q);
        x[i] = (e + 1 >= n || xi >= 16) ? 16u : (uint32_t)xi;
        a1[i] = on[i] ? wsh + sp + (16 * q - o) : wsh;
        a2[i] = on[i] && x[i] < 16 ? wsh + s1 - x[i] : wsh;
      }
      uint4 w1[NB], w2[NB];
#pragma unroll
      for (int i = 0; i < NB; i++) {
        w1[i] = lds_u128(win, a1[i]);
        w2[i] = lds_u128(win, a2[i]);
      }
#pragma unroll
      for (int i = 0; i < NB; i++)
        if (on[i]) *reinterpret_cast<uint4*>(stage + t0[i]) = blend_at(w1[i], w2[i], (int32_t)x[i]);
    }
    return;
  }
  for (uint32_t e0 = 0; e0 < n; e0 += epi) {
    const uint32_t e = e0 + (lane >> jl);
    if (e >= n) continue;
    uint32_t o, o1, sp;
    entry_span<IS_KEY>(meta, e, o, o1, sp);
    const uint32_t qa = (o + 15) >> 4;
    const uint32_t qb = (e + 1 == n) ? Q : (o1 + 15) >> 4;
    for (uint32_t q = qa + j0; q < qb; q += J) {
      const uint32_t t0 = 16 * q;  // >= o
      uint4 v;
      if (two) {
        const uint4 w1 = lds_u128(win, wsh + sp + (t0 - o));
        const int32_t x = (int32_t)o1 - (int32_t)t0;
        if (x >= 16 || e + 1 >= n) {
          v = w1;
        } else {
          uint32_t oo, oo1, s1;
          entry_span<IS_KEY>(meta, e + 1, oo, oo1, s1);
          const uint4 w2 = lds_u128(win, wsh + s1 - (uint32_t)x);
          v = blend_at(w1, w2, x);
        }
      } else {  // general: entries shorter than 16 B, run by run
        v = make_uint4(0, 0, 0, 0);
        uint32_t ee = e, eo = o, eo1 = o1, es = sp;
        uint32_t t = t0;
        const uint32_t hi = min(t0 + 16, L);
        while (t < hi) {
          while (eo1 <= t) {
            ee++;
            entry_span<IS_KEY>(meta, ee, eo, eo1, es);
          }
          const uint4 w = lds_u128(win, wsh + es + (t0 - eo));
          const uint32_t rend = min(eo1, hi);
          v = blend_at(blend_at(v, w, (int32_t)(t - t0)), v, (int32_t)(rend - t0));
          t = rend;
        }
      }
      *reinterpret_cast<uint4*>(stage + t0) = v;  // aligned ds_write_b128
    }
  }
}

// Walk + stage block k: fills `pd` (registers) from the block in `slot`.
template <int MAXE>
__device__ __forceinline__ void stage_block(const DecodeParams& p, const BlockRef& ref,
                                            uint8_t* slot, uint8_t* stage, uint32_t* meta,
                                            Pend& pd, uint32_t lane, uint64_t* spec_acc) {
#ifdef LSMGPU_STAMPS
  uint64_t t0 = spec_acc ? __builtin_amdgcn_s_memtime() : 0;
  auto sub = [&](int i) {
    if (spec_acc) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      spec_acc[i] += t - t0;
      t0 = t;
    }
  };
#else
  auto sub = [](int) {};
#endif
  Plan pl = walk_stage<4096, MAXE, true>(p, ref, true, slot, meta, lane, spec_acc);
  sub(2);
  if (pl.kind == 1 && (pl.n > 128 || pl.K < 16 || pl.V < 16)) pl.kind = 2;  // n, K, V exact
  // piece mode: every entry >= 16 B and its key + value pieces (one group of J = 2^jkv lanes
  // per entry) fit kRegChunks passes
  const uint32_t passes = pl.jkv < 6 ? (pl.n + (kWave >> pl.jkv) - 1) >> (6 - pl.jkv) : 99u;
  const uint32_t mode = (pl.kind == 1 && passes <= (uint32_t)kRegChunks) ? 1u : 0u;
  const uint32_t f[8] = {pl.n, pl.K, pl.V, pl.status, pl.off, pl.len, pl.kind, mode};
  uint32_t x = f[0];
#pragma unroll
  for (int i = 1; i < 8; i++) x = lane == (uint32_t)i ? f[i] : x;
  pd.sc = x;
  if (pl.kind != 1) return;
  if (mode == 1) {
    // lane group (e, j), e = s * 64 / J + lane / J: pieces j < kpc are entry e's key pieces,
    // the rest its value pieces.  Piece j of a stream covers entry bytes
    // [min(16 j, len - 16), +16): the last piece overlaps back inside the entry, so the emit's
    // unaligned stores never touch a byte outside it.  Every LDS read is unconditional and
    // dword-aligned (window = 5 ds_read_b32 + v_alignbyte).
    const uint8_t* wn = slot - 64;
    const uint32_t ws = pl.sh + 64;
    const uint32_t jl = pl.jkv;
#pragma unroll
    for (int s = 0; s < kRegChunks; s++) {
      const uint32_t e = (uint32_t)s * (kWave >> jl) + (lane >> jl);
      const uint32_t j = lane & ((1u << jl) - 1);
      const uint32_t ec = min(e, pl.n - 1);
      const uint32_t w0 = meta[ec], w1 = meta[ec + 1];
      const uint32_t p0 = w0 & 0xffffu, k0 = w0 >> 16, p1 = w1 & 0xffffu, k1 = w1 >> 16;
      const uint32_t klen = k1 - k0, vlen = p1 - p0 - 10 - klen;
      const uint32_t kpc = n_pieces(klen);
      const bool key = j < kpc;
      const uint32_t jj = key ? j : j - kpc;
      const uint32_t len = key ? klen : vlen;
      const uint32_t o = key ? k0 : p0 - 10 * ec - k0;
      const uint32_t sp = key ? p0 + 10 : p0 + 10 + klen;
      const uint32_t lg = piece_log2(len), sz = 1u << lg;
      const bool on = (uint32_t)s < passes && e < pl.n && jj < n_pieces(len);
      const uint32_t off = min(jj << lg, len - sz);
      pd.c[s] = lds_u128(wn, ws + (on ? sp + off : 0u));
      const uint32_t f16 = on ? ((o + off) | (lg << 12) | (key ? 0u : kValueBit)) : kNoPiece;
      if (s & 1) pd.po[s >> 1] |= f16 << 16;
      else pd.po[s >> 1] = f16;
    }
    pd.end0 = ends_word(meta, lane);
    pd.end1 = ends_word(meta, 64 + lane);
    sub(3);
    return;
  }
  // windows may start up to 15 B before block byte 0: `win` = slot - 64 (the slots follow the
  // meta words and the staging buffer in LDS, so those bytes are addressable)
  const uint8_t* win = slot - 64;
  const uint32_t wsh = pl.sh + 64;
  const uint32_t Qk = (pl.K + 15) >> 4, Qv = (pl.V + 15) >> 4;
  // keys of one length that is a multiple of 16 B (16-B hex keys, 64-B keys, ...) go straight
  // from the block into registers; otherwise both streams are staged
  const uint32_t kr = pl.ku >> 4;  // 16-B pieces per key
  const bool kdirect = pl.ku && (pl.ku & 15) == 0 && (kr & (kr - 1)) == 0;
  const uint32_t vbase = kdirect ? 0u : 16 * Qk;  // value stream's 16-aligned staging offset
  if (!ABLATE(p, 8)) {  // (timing-only ablation: 8 = no stream assembly)
    if (!kdirect) assemble_stream<true>(stage, win, wsh, meta, pl.n, pl.K, pl.jk, pl.big, lane);
    assemble_stream<false>(stage + vbase, win, wsh, meta, pl.n, pl.V, pl.jv, pl.big, lane);
  }
  sub(3);
  if ABLATE(p, 16) return;  // (timing-only ablation: 16 = no register readback)
  wave_lds_fence();
  const uint32_t ksh = kdirect ? __builtin_ctz(kr) : 0u;
  // chunk addresses (window coordinates): key chunks straight from the block (kdirect) or
  // from the staging buffer; value chunks from the staging buffer; each stream's last chunk
  // overlaps back inside it.  Reads are unconditional (see assemble_stream).
  const uint32_t sbase = (uint32_t)(stage - win);  // staging byte 0 in window coordinates
  uint32_t km[kRegChunks];
#pragma unroll
  for (int s = 0; s < kRegChunks; s++) km[s] = meta[min((64u * s + lane) >> ksh, pl.n)];
#pragma unroll
  for (int s = 0; s < kRegChunks; s++) {
    const uint32_t q = 64 * s + lane;
    uint32_t a;
    if (q < Qk)
      a = kdirect ? wsh + (km[s] & 0xffffu) + 10 + 16 * (q & (kr - 1))
                  : sbase + (q + 1 < Qk ? 16 * q : pl.K - 16);
    else if (q < Qk + Qv)
      a = sbase + vbase + (q - Qk + 1 < Qv ? 16 * (q - Qk) : pl.V - 16);
    else
      a = sbase;
    pd.c[s] = lds_u128(win, a);
  }
  pd.end0 = ends_word(meta, lane);
  pd.end1 = ends_word(meta, 64 + lane);
  sub(4);
}

// Per-entry end offsets / view record of entry e from its ends word and its predecessor's.
__device__ __forceinline__ void entry_out(const DecodeParams& p, uint32_t e, uint32_t we,
                                          uint32_t wprev, Tot ex, uint32_t off, bool mat,
                                          bool view) {
  const uint32_t k1 = we & 0xffffu, vo1 = we >> 16;
  if (mat) {
    if (p.key_end) p.key_end[ex.n + e] = ex.k + k1;
    if (p.val_end) p.val_end[ex.n + e] = ex.v + vo1;
  }
  if (view) {
    const uint32_t k0 = e ? (wprev & 0xffffu) : 0u, vo0 = e ? (wprev >> 16) : 0u;
    const uint32_t p0 = vo0 + 10 * e + k0;  // header position (vo = pos - 10 e - ko)
    p.view[ex.n + e] = (uint64_t)(off + p0 + 10) | ((uint64_t)(k1 - k0) << 32) |
                       ((uint64_t)(vo1 - vo0) << 48);
  }
}

__device__ __forceinline__ void emit_pend(const DecodeParams& p, const Pend& pd, uint32_t b, Tot ex,
                                          uint32_t lane) {
  const uint32_t n = readlane(pd.sc, 0), K = readlane(pd.sc, 1), V = readlane(pd.sc, 2),
                 status = readlane(pd.sc, 3), off = readlane(pd.sc, 4), kind = readlane(pd.sc, 6),
                 mode = readlane(pd.sc, 7);
  if (lane == 0) {
    if (p.blk_first) p.blk_first[b] = ex.n;
    if (p.blk_status) p.blk_status[b] = (int32_t)status;
    if (status != LSMGPU_BLK_OK) {
      atomicAdd(reinterpret_cast<unsigned long long*>(p.result + 4), 1ull);
      atomicMax(reinterpret_cast<unsigned long long*>(p.result + 3),
                (unsigned long long)(p.nblk - b));
    }
  }
  const bool mat = (p.mode & LSMGPU_MODE_MATERIALIZE) != 0;
  const bool view = (p.mode & LSMGPU_MODE_VIEW) != 0 && p.view;
  bool ok = (uint64_t)ex.n + n <= p.ent_cap;
  if (mat) {
    const uint64_t kend = (uint64_t)ex.k + K, vend = (uint64_t)ex.v + V;
    ok = ok && (kend <= p.key_cap || !p.key_data) && (vend <= p.val_cap || !p.val_data);
    ok = ok && kend < 0xffffffffull && vend <= 0xffffffffull;
  }
  if (!ok && lane == 0) atomicOr(reinterpret_cast<unsigned long long*>(p.result + 5), 1ull);
#ifdef LSMGPU_STAMPS
  if (p.stamps && lane == 0)  // blocks per emit path: [13] chunk mode, [14] piece mode, [15] global
    atomicAdd(reinterpret_cast<unsigned long long*>(p.stamps + (kind == 2 ? 15 : 13 + mode)), 1ull);
#endif
  if (!ok || kind == 0 || ABLATE(p, 2)) return;
  if (kind == 2) {
    emit_slow(p, p.data + off, n, ex.n, ex.k, ex.v, off, lane);
    return;
  }
  uint32_t pr0 = 0, pr1 = 0;  // predecessor ends (view mode only)
  if (view) {
    pr0 = __shfl_up(pd.end0, 1);
    pr1 = __shfl_up(pd.end1, 1);
    if (lane == 0) pr1 = __builtin_amdgcn_readlane(pd.end0, 63);
  }
  if (lane < n) entry_out(p, lane, pd.end0, pr0, ex, off, mat, view);
  if (64 + lane < n) entry_out(p, 64 + lane, pd.end1, pr1, ex, off, mat, view);
  if (!mat) return;
  uint8_t* kd = p.key_data + ex.k;
  uint8_t* vd = p.val_data + ex.v;
  if (mode == 1) {  // unaligned 16-B piece stores (overlapping only inside one entry)
#pragma unroll
    for (int s = 0; s < kRegChunks; s++) {
      const uint32_t po = (pd.po[s >> 1] >> (16 * (s & 1))) & 0xffffu;
      const bool val = (po & kValueBit) != 0;
      uint8_t* base = val ? p.val_data : p.key_data;
      if (po != kNoPiece && base) {
        const uint4 v = pd.c[s];
        uint8_t* d = (val ? vd : kd) + (po & 0xfffu);
        const uint32_t lg = (po >> 12) & 7u;
        if (lg == 4) {
          __builtin_memcpy(d, &v, 16);
        } else if (lg == 3) {
          const uint2 h = make_uint2(v.x, v.y);
          __builtin_memcpy(d, &h, 8);
        } else if (lg == 2) {
          __builtin_memcpy(d, &v.x, 4);
        } else if (lg == 1) {
          const uint16_t h = (uint16_t)v.x;
          __builtin_memcpy(d, &h, 2);
        } else {
          *d = (uint8_t)v.x;
        }
      }
    }
    return;
  }
  const uint32_t Qk = (K + 15) >> 4, Qv = (V + 15) >> 4;
#pragma unroll
  for (int s = 0; s < kRegChunks; s++) {
    const uint32_t q = 64 * s + lane;
    const uint4 v = pd.c[s];
    if (q < Qk) {
      if (p.key_data) __builtin_memcpy(kd + chunk_off(q, Qk, K), &v, 16);
    } else if (q < Qk + Qv) {
      if (p.val_data) __builtin_memcpy(vd + chunk_off(q - Qk, Qv, V), &v, 16);
    }
  }
}

// One wave per workgroup, blocks w, w + G, ...  Iteration k (one vmcnt drain):
//   a. s_waitcnt vmcnt(0): block k's LDS-DMA, block k-L's prefix poll, old stores
//   b. emit block k-L from registers (its base from the poll)
//   c. issue block k+1-L's prefix poll and block k+1's LDS-DMA (the slot of block k-1)
//   d. walk + stage block k into registers, publish its aggregate, lead its group if due
template <int MAXE, int L>
__global__ void __launch_bounds__(64, 3) decode_reg_kernel(DecodeParams p) {  // <= 168 VGPRs
  static_assert(L == 3, "three named pending slots");
  using Cfg = RegCfg<MAXE>;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = lane_id();
  if (p.census) {
    census(p.census, lane);
    return;
  }
  const uint32_t G = gridDim.x, w = blockIdx.x, nblk = p.nblk;
  const uint64_t tag = p.tag;
  const uint32_t KW = w < nblk ? (nblk - 1 - w) / G + 1 : 0;  // this workgroup's blocks
  uint32_t* meta = reinterpret_cast<uint32_t*>(smem);
  uint8_t* stage = smem + Cfg::kMetaBytes;
  auto slot_of = [&](uint32_t k) -> uint8_t* { return smem + Cfg::kMetaBytes + Cfg::kStage + (k & 1) * Cfg::kBuf; };
  auto blk_of = [&](uint32_t k) -> uint32_t { return w + k * G; };
  uint32_t ring_k0 = 0, ring_off = 0, ring_len = 0;
  auto ring_load = [&](uint32_t k0) {
    ring_k0 = k0;
    const uint64_t b = (uint64_t)w + (uint64_t)(k0 + lane) * G;
    ring_off = b < nblk ? p.blk_off[b] : 0u;
    ring_len = b < nblk ? p.blk_len[b] : 0u;
  };
#ifdef LSMGPU_STAMPS
  const bool st = p.stamps != nullptr;
  uint64_t acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t tprev = st ? stamp() : 0;
  auto mark = [&](int i) {
    if (st) {
      const uint64_t t = stamp();
      acc[i] += t - tprev;
      tprev = t;
    }
  };
  uint64_t* spec_acc = st ? &acc[6] : nullptr;
#else
  auto mark = [](int) {};
  uint64_t* spec_acc = nullptr;
#endif
  BlockRef ref_next{0, 0, 0, false, false};
  if (KW > 0) {
    ring_load(0);
    ref_next = prefetch_block<4096, Cfg::kIters>(p, readlane(ring_off, 0), readlane(ring_len, 0),
                                                 slot_of(0), lane);
  }
  Pend pa, pb, pc;  // blocks k-3, k-2, k-1 (pc: after the walk, block k)
  uint64_t poll = 0;  // block k-L's prefix granules, polled one iteration ahead
  for (uint32_t k = 0; k < KW + L; k++) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const BlockRef ref = ref_next;
    mark(0);
    // b. emit block k - L
    if (k >= L) {
      const uint32_t be = blk_of(k - L);
      Tot ex{0, 0, 0};
      if (!ABLATE(p, 1)) ex = prefix_of(p, be, poll, tag, lane);
      mark(5);
      if (be == nblk - 1 && lane == 0) {  // totals of the whole batch
        const uint32_t n = readlane(pa.sc, 0), K = readlane(pa.sc, 1), V = readlane(pa.sc, 2);
        if (p.blk_first) p.blk_first[nblk] = ex.n + n;
        p.result[0] = sat_add(ex.n, n);
        p.result[1] = sat_add(ex.k, K);
        p.result[2] = sat_add(ex.v, V);
      }
      emit_pend(p, pa, be, ex, lane);
    }
    pa = pb;
    pb = pc;
    mark(1);
    // c. next prefix poll, next block's bytes
    if (k + 1 >= L && k + 1 - L < KW && lane < 3 && !ABLATE(p, 1))
      poll = gload(p.lb + (uint64_t)blk_of(k + 1 - L) * 8 + 4 + lane);
    if (k + 1 < KW) {
      if (k + 1 - ring_k0 >= (uint32_t)kWave) ring_load(k + 1);
      const uint32_t i = k + 1 - ring_k0;
      ref_next = prefetch_block<4096, Cfg::kIters>(p, readlane(ring_off, i), readlane(ring_len, i),
                                                   slot_of(k + 1), lane);
    }
    mark(2);
    // d. walk + stage block k
    if (k < KW) {
      const uint32_t b = blk_of(k);
      wave_lds_fence();
      stage_block<MAXE>(p, ref, slot_of(k), stage, meta, pc, lane, spec_acc);
      mark(3);
      if (!ABLATE(p, 1))
        store3(p.lb + (uint64_t)b * 8, tag, readlane(pc.sc, 0), readlane(pc.sc, 1),
               readlane(pc.sc, 2), lane);
    }
    // e. group duty for the PREVIOUS block, one iteration late: its group's aggregates are
    // published by now (no spinning), and the duty never delays this block's aggregate
    if (k >= 1 && k - 1 < KW && !ABLATE(p, 1)) {
      const uint32_t b = blk_of(k - 1);
      const uint32_t g0 = b & ~63u;
      const uint32_t gsize = (nblk - g0 < 64u) ? (nblk - g0) : 64u;
      if ((b - g0) == (b / G) % gsize) group_lead(p, b, tag, lane);
    }
    mark(4);
    wave_lds_fence();
  }
#ifdef LSMGPU_STAMPS
  if (st && lane == 0) {
#pragma unroll
    for (int i = 0; i < 8; i++) atomicAdd(reinterpret_cast<unsigned long long*>(p.stamps + i), acc[i]);
    atomicAdd(reinterpret_cast<unsigned long long*>(p.stamps + 8), (unsigned long long)(KW + L));
    atomicAdd(reinterpret_cast<unsigned long long*>(p.stamps + 9), 1ull);
    for (int i = 8; i < 11; i++) atomicAdd(reinterpret_cast<unsigned long long*>(p.stamps + 2 + i), acc[i]);
  }
#endif
}

// Upper bound on the decode kernels' SGPR count (hipcc -Rpass-analysis=kernel-resource-usage),
// checked by tests/test_abi.py::test_decode_resource_budget.
constexpr int kDecodeSgprs = 112;

// Persistent grid = workgroups per CU x CUs, the per-CU count MEASURED once per configuration
// by a residency census (the occupancy API over-reports on MI355X: 3 x 54,112 B of LDS per CU
// are admitted by the API but not by the hardware -- scripts/residency_probe.hip).
// Kernel traits: the LDS-lag kernel for a slot size, the register-lag kernel for 4 KiB.
template <int SLOT, int MAXE, int NS>
struct LdsLag {
  static constexpr int kSlot = SLOT;
  static constexpr int kLds = DecodeCfg<SLOT, MAXE, NS>::kLds;
  static constexpr const char* kName = "lds-lag";
  static void (*kernel())(DecodeParams) { return decode_kernel<SLOT, MAXE, NS>; }
};
template <int MAXE, int L>
struct RegLag {
  static constexpr int kSlot = 4096;
  static constexpr int kLds = RegCfg<MAXE>::kLds;
  static constexpr const char* kName = "reg-lag";
  static void (*kernel())(DecodeParams) { return decode_reg_kernel<MAXE, L>; }
};

template <class T>
static int resident_per_cu(const DecodeParams& p, int num_cus, hipStream_t s) {
  using Cfg = T;
  auto k = T::kernel();
  const int SLOT = T::kSlot;
  static std::atomic<int> per_cu_cached{0};
  if (int v = per_cu_cached.load(std::memory_order_acquire)) return v;
  // one census per configuration and process, even with contexts on several threads
  static std::mutex census_mu;
  std::lock_guard<std::mutex> lock(census_mu);
  if (int v = per_cu_cached.load(std::memory_order_acquire)) return v;
  int per_cu = 0;
  if (Cfg::kLds > 64 * 1024 &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                          hipFuncAttributeMaxDynamicSharedMemorySize, Cfg::kLds) != hipSuccess)
    return -1;
  int api = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&api, k, 64, Cfg::kLds) != hipSuccess) return -1;
  const int waves_per_simd = 800 / (((kDecodeSgprs + 15) / 16) * 16 + 16);
  int cand = api;
  const int lds_bound = (160 * 1024) / Cfg::kLds;
  if (cand > lds_bound) cand = lds_bound;
  if (cand > waves_per_simd * 4) cand = waves_per_simd * 4;
  uint32_t* c = nullptr;
  if (hipMalloc(&c, 8) != hipSuccess) return -1;
  int found = 1;
  for (; cand >= 1; cand--) {
    const uint32_t grid = (uint32_t)cand * (uint32_t)num_cus;
    uint32_t h[2] = {0, 0};
    DecodeParams q = p;
    q.census = c;
    q.stamps = nullptr;
    if (hipMemsetAsync(c, 0, 8, s) != hipSuccess) break;
    hipLaunchKernelGGL(k, dim3(grid), dim3(64), Cfg::kLds, s, q);
    if (hipMemcpyAsync(h, c + 0, 8, hipMemcpyDeviceToHost, s) != hipSuccess) break;
    if (hipStreamSynchronize(s) != hipSuccess) break;
    if (h[1] == grid) {
      found = cand;
      break;
    }
  }
  (void)hipFree(c);
  per_cu = found;
  per_cu_cached.store(per_cu, std::memory_order_release);
  if (getenv("LSMGPU_DEBUG_ERR"))
    fprintf(stderr, "[lsmgpu] decode SLOT=%d census: api %d lds %d -> resident %d per CU\n", SLOT,
            api, Cfg::kLds, per_cu);
  return per_cu;
}

template <class T>
static hipError_t launch_cfg(const DecodeParams& p, int num_cus, hipStream_t s,
                             uint64_t* waves_launched) {
  using Cfg = T;
  auto k = T::kernel();
  const int per_cu = resident_per_cu<T>(p, num_cus, s);
  if (per_cu < 1) return hipErrorLaunchFailure;
  // a multiple of 64 workgroups (each 64-block group sits in one round), never more than what
  // is resident at once, never more than the blocks
  uint64_t grid = (uint64_t)per_cu * (uint64_t)num_cus;
  grid = grid / 64 * 64;
  if (grid < 64) grid = 64;
  // LSMGPU_GRID (tests/diagnostics): a smaller multiple of 64 workgroups -> many rounds
  const uint64_t grid_cap = getenv("LSMGPU_GRID") ? (uint64_t)atoll(getenv("LSMGPU_GRID")) : 0;
  if (grid_cap >= 64 && grid_cap / 64 * 64 < grid) grid = grid_cap / 64 * 64;
  if (grid > p.nblk) grid = p.nblk;  // one round: every block has its own workgroup
  if (grid < 1) grid = 1;
  *waves_launched = grid;
  DecodeParams q = p;
  q.census = nullptr;
  q.stamps = nullptr;
#ifdef LSMGPU_DIAG
  q.ablate = getenv("LSMGPU_ABLATE") ? (uint32_t)atoi(getenv("LSMGPU_ABLATE")) : 0u;
  static uint64_t* stamps = nullptr;
  const bool want_stamps = getenv("LSMGPU_STAMPS") != nullptr;
  if (want_stamps) {
    if (!stamps && hipMalloc(&stamps, 16 * sizeof(uint64_t)) != hipSuccess) stamps = nullptr;
    if (stamps) {
      (void)hipMemsetAsync(stamps, 0, 16 * sizeof(uint64_t), s);
      q.stamps = stamps;
    }
  }
  if (getenv("LSMGPU_DEBUG"))
    fprintf(stderr, "[lsmgpu] decode %s SLOT=%d lds=%d per_cu=%d cus=%d grid=%llu nblk=%u\n",
            T::kName, T::kSlot, Cfg::kLds, per_cu, num_cus, (unsigned long long)grid, p.nblk);
#endif
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(64), Cfg::kLds, s, q);
  hipError_t e = hipGetLastError();
#ifdef LSMGPU_DIAG
  if (e == hipSuccess && q.stamps) {
    uint64_t h[16] = {0};
    (void)hipMemcpyAsync(h, stamps, sizeof(h), hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    const double it = h[8] ? (double)h[8] : 1.0;
    fprintf(stderr, "[lsmgpu] stamps per wave-iteration (s_memtime cycles): drain %.0f prefix-wait %.0f "
            "emit %.0f issue %.0f walk %.0f (spec %.0f, rounds %.2f; reg-lag: walk total %.0f, stage %.0f, "
            "readback %.0f) publish %.0f | iterations %llu waves %llu\n", h[0] / it, h[5] / it,
            h[1] / it, h[2] / it, h[3] / it, h[6] / it, h[7] / it, h[10] / it, h[11] / it,
            h[12] / it, h[4] / it, (unsigned long long)h[8], (unsigned long long)h[9]);
    fprintf(stderr, "[lsmgpu] blocks by emit path: chunk %llu piece %llu global %llu\n",
            (unsigned long long)h[13], (unsigned long long)h[14], (unsigned long long)h[15]);
  }
#endif
  return e;
}

int decode_path(uint32_t max_blk_len, uint32_t nblk) {
  // LSMGPU_DECODE_PATH=reg|lds|wsc forces a path (A/B diagnostics and tests)
  const char* f = getenv("LSMGPU_DECODE_PATH");
  if (f && f[0] == 'w' && max_blk_len < 65536) return 2;
  if (f && f[0] == 'l') return 1;
  if (f && f[0] == 'r' && max_blk_len <= 4096) return 0;
  // walk-scan-copy is three launches (walk, scan, copy): it wins from ~1k blocks up; small
  // batches stay on the single persistent kernel
  if (max_blk_len < 65536 && nblk >= kWscMinBlocks) return 2;
  return max_blk_len <= 4096 ? 0 : 1;
}

hipError_t launch_decode(const DecodeParams& p, uint32_t max_blk_len, int num_cus,
                         hipStream_t s, uint64_t* waves_launched) {
  if (decode_path(max_blk_len, p.nblk) == 0) return launch_cfg<RegLag<128, 3>>(p, num_cus, s, waves_launched);
  if (max_blk_len <= 4096) return launch_cfg<LdsLag<4096, 100, 4>>(p, num_cus, s, waves_launched);
  if (max_blk_len <= 8192) return launch_cfg<LdsLag<8192, 256, 4>>(p, num_cus, s, waves_launched);
  if (max_blk_len <= 16384) return launch_cfg<LdsLag<16384, 512, 3>>(p, num_cus, s, waves_launched);
  // 32 KiB slot; larger blocks run the global-memory path inside the same kernel
  return launch_cfg<LdsLag<32768, 1024, 3>>(p, num_cus, s, waves_launched);
}

}  // namespace lsmgpu
