// decode.hip -- gfx950 SST block decode: the device restatement of blockIterator.Next/parseKV
// (table/iterator.go:93-135) driven over every block of a batch (Iterator.seekToFirst/next,
// iterator.go:201-217,301-326).
//
// Work decomposition ("decode kernel"):
//   tile   = WPB consecutive blocks, one per wave of a workgroup; a persistent, fully
//            resident grid walks the tiles round-robin (tile = blockIdx.x + k * gridDim.x)
//   stage  : each wave's block -> its LDS slot with 16-B loads; the NEXT tile's loads are
//            issued into registers before the current tile waits on its prefix (the wait is
//            hidden behind HBM latency), and land in LDS after the current emit
//   walk   : the serial header chain (pos += 10 + klen + vlen) in LDS on the VALU (the CU's
//            single scalar unit would serialise every wave's chain), recording per entry
//            {key pos, key out offset, value pos, value out offset}
//   prefix : tile aggregates -> groups of 64 tiles; the last tile of a group to arrive
//            scans the group, looks back over earlier GROUPS and publishes every member's
//            exclusive output base (8-B {tag, value} granules, agent scope)
//   emit   : per-entry end offsets (coalesced u32), key and value streams written as
//            aligned 16-B chunks gathered from LDS (a chunk may blend several entries' runs)
// Blocks larger than the slot, or with more entries than the metadata holds, take a
// global-memory path with identical semantics.
#include <cstdio>
#include <cstdlib>

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
  uint32_t n, K, V, status, base_pos, end_pos;
};

// The blockIterator forward walk.  `meta` (LDS, stride 4 u16) gets {ks, ko, vs, vo} for
// entries < maxe when record is set.  Values are identical in every lane (VALU, no SALU).
template <class Src>
__device__ __forceinline__ WalkResult walk_block(const Src& src, uint32_t len, uint16_t* meta,
                                                 uint32_t maxe, bool record, uint32_t lane) {
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
    const uint32_t ks = pos;
    pos += h.klen;                                           // iterator.go:101
    if (pos + h.vlen > len) { st = LSMGPU_BLK_VALUE_OVERFLOW; break; }  // iterator.go:103
    const uint32_t vs = pos;
    pos += h.vlen;                                           // iterator.go:109
    if (record && n < maxe && lane == 0) {
      ushort4 m = make_ushort4((uint16_t)ks, (uint16_t)K, (uint16_t)vs, (uint16_t)V);
      *reinterpret_cast<ushort4*>(meta + 4 * n) = m;
    }
    K += h.plen + h.klen;
    V += h.vlen;
    n++;
  }
  return WalkResult{n, K, V, st, base_pos, pos};
}

__device__ __forceinline__ uint32_t wave_scan_incl32(uint32_t v, uint32_t lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t x = __shfl_up(v, o);
    if (lane >= (uint32_t)o) v += x;
  }
  return v;
}

// Speculative parallel walk of a block held in LDS, exactly equivalent to walk_block.
// The chain pos_{e+1} = pos_e + 10 + klen_e + vlen_e is serial, but SST entries of a block
// mostly share one size: each round lane i reads the header guessed at pos + i*stride, a
// ballot finds the first lane whose entry stops the iterator (end, terminator, error) or
// whose size differs from the stride, and every lane before it is a confirmed entry.  A
// round therefore advances over a whole run of equal-size entries with ONE LDS round trip;
// a size change simply starts the next round at the mismatching entry's successor.
struct SpecResult {
  uint32_t n, status, base_pos, end_pos;
};
__device__ __forceinline__ uint32_t readlane(uint32_t v, uint32_t l) {
  return __builtin_amdgcn_readlane(v, l);
}
// Status of the iterator at a position where no entry was confirmed (walk_block's rules).
__device__ __forceinline__ SpecResult stop_at(const LdsSrc& src, uint32_t pf, uint32_t len,
                                              uint32_t n, uint32_t base_pos, bool first) {
  uint32_t st = LSMGPU_BLK_OK, end = pf;
  if (pf < len) {                                          // else: pos >= len, io.EOF
    if (len - pf < 10) {
      st = LSMGPU_BLK_TRUNC_HEADER;
    } else {
      const Hdr h = src.hdr(pf);
      if ((h.klen | h.plen) == 0) end = pf + 10;            // terminator
      else if (first && h.plen != 0) st = LSMGPU_BLK_FIRST_PLEN;
      else if (base_pos + h.plen > len) st = LSMGPU_BLK_PREFIX_OOB;
      else st = LSMGPU_BLK_VALUE_OVERFLOW;                  // p + 10 + klen + vlen > len
    }
  }
  return SpecResult{n, st, base_pos, end};
}

__device__ __forceinline__ SpecResult walk_spec(const uint8_t* slot, uint32_t sh, uint32_t len,
                                                uint16_t* meta, uint32_t maxe, uint32_t lane) {
  const LdsSrc src{slot, sh};
  // first entry (uniform): defines baseKey (iterator.go:129-133) and the first stride guess
  if (len < 10) return stop_at(src, 0, len, 0, 10, true);
  const Hdr h0 = src.hdr(0);
  const uint32_t base_pos = 10;
  const uint32_t sz0 = 10 + h0.klen + h0.vlen;
  if ((h0.klen | h0.plen) == 0 || h0.plen != 0 || base_pos + h0.plen > len || sz0 > len)
    return stop_at(src, 0, len, 0, base_pos, true);
  if (lane == 0 && maxe > 0) meta[0] = 0;
  uint32_t pos = sz0, stride = sz0, n = 1;
  for (;;) {
    // lane i checks the entry guessed at pos + i*stride (branch-free)
    const uint32_t p = pos + lane * stride;
    const bool has_hdr = p + 10 <= len;
    const Hdr h = src.hdr(has_hdr ? p : 0u);
    const uint32_t sz = 10 + h.klen + h.vlen;
    const bool bad = !has_hdr || (h.klen | h.plen) == 0 || base_pos + h.plen > len || p + sz > len;
    const uint64_t any = __ballot(bad || sz != stride);
    if (any == 0) {  // 64 entries of exactly `stride` bytes
      if (n + lane < maxe) meta[4 * (n + lane)] = (uint16_t)p;
      n += 64;
      pos += 64 * stride;
      continue;
    }
    const uint32_t f = (uint32_t)__builtin_ctzll(any);
    const bool fbad = (__ballot(bad) >> f) & 1ull;
    const uint32_t m = f + (fbad ? 0u : 1u);  // confirmed entries: lanes [0, m)
    if (lane < m && n + lane < maxe) meta[4 * (n + lane)] = (uint16_t)p;
    n += m;
    const uint32_t pf = readlane(p, f);
    if (fbad) return stop_at(src, pf, len, n, base_pos, false);
    const uint32_t szf = readlane(sz, f);  // entry f has another size: continue after it
    pos = pf + szf;
    if (f == 0) stride = szf;  // the guess failed at once: adopt the new size
  }
}

// After walk_spec: lane e turns row e's header position into {ks, ko, vs, vo} (wave scans of
// the key / value output sizes) and row n into the totals sentinel.  Requires n <= maxe.
__device__ __forceinline__ WalkResult finish_meta(const uint8_t* slot, uint32_t sh,
                                                  const SpecResult& r, uint16_t* meta,
                                                  uint32_t lane, bool& any_plen) {
  const LdsSrc src{slot, sh};
  uint32_t K = 0, V = 0;
  any_plen = false;
  for (uint32_t e0 = 0; e0 < r.n; e0 += kWave) {
    const uint32_t e = e0 + lane;
    const bool on = e < r.n;
    uint32_t hp = 0;
    Hdr h{0, 0, 0};
    if (on) {
      hp = meta[4 * e];
      h = src.hdr(hp);
    }
    const uint32_t kl = on ? h.plen + h.klen : 0u, vl = on ? h.vlen : 0u;
    any_plen = any_plen || __any(on && h.plen != 0);
    const uint32_t ki = wave_scan_incl32(kl, lane), vi = wave_scan_incl32(vl, lane);
    if (on)
      *reinterpret_cast<ushort4*>(meta + 4 * e) =
          make_ushort4((uint16_t)(hp + 10), (uint16_t)(K + ki - kl), (uint16_t)(hp + 10 + h.klen),
                       (uint16_t)(V + vi - vl));
    K += __shfl(ki, 63);
    V += __shfl(vi, 63);
  }
  if (lane == 0)
    *reinterpret_cast<ushort4*>(meta + 4 * r.n) =
        make_ushort4((uint16_t)r.end_pos, (uint16_t)K, 0, (uint16_t)V);
  return WalkResult{r.n, K, V, r.status, r.base_pos, r.end_pos};
}

struct Tot {
  uint32_t n, k, v;
};

constexpr uint32_t kMaxSpins = 1u << 20;  // ~1 s of polling: a hard bound, never expected

__device__ __forceinline__ void flag_timeout(uint64_t* result, uint32_t lane) {
  if (lane == 0) atomicOr(reinterpret_cast<unsigned long long*>(result + 5), 2ull);
}

__device__ __forceinline__ uint32_t wave_sum_sat(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = sat_add(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ uint32_t wave_scan_sat(uint32_t v, uint32_t lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t x = __shfl_up(v, o);
    if (lane >= (uint32_t)o) v = sat_add(v, x);
  }
  return v;
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
__device__ Tot lookback(const uint64_t* rec, uint32_t g, uint64_t tag, uint32_t lane,
                        uint64_t* result) {
  Tot ex{0, 0, 0};
  int64_t j0 = (int64_t)g - 1;
  uint32_t wsize = 8;
  uint32_t spins = 0;
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
      if (++spins > kMaxSpins) {
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

// Exclusive {entries, key bytes, value bytes} of every tile before `tile`, given this tile's
// aggregate (already published).  Called by ONE wave of the tile's workgroup.
__device__ Tot tile_prefix(const DecodeParams& p, uint32_t tile, uint32_t ntiles, uint64_t tag,
                           uint32_t lane) {
  const uint32_t g = tile >> 6;
  const uint32_t g0 = g << 6;
  const uint32_t gsize = (ntiles - g0 < 64u) ? (ntiles - g0) : 64u;
  uint32_t old = 0;
  if (lane == 0) old = atomicAdd(p.gcnt + g, 1u);
  old = uniform(old);
  if (old != gsize - 1) {
    // a member: wait for the group's last arriver to publish this tile's exclusive prefix
    const uint64_t* X = p.lb + (uint64_t)tile * 8 + 4;
    for (uint32_t spins = 0;; ++spins) {
      uint64_t x = 0;
      bool ok = true;
      if (lane < 3) {
        x = gload(X + lane);
        ok = (x >> kTagShift) == tag;
      }
      if (__all(ok)) {
        const uint32_t v = (uint32_t)x;
        return Tot{__shfl(v, 0), __shfl(v, 1), __shfl(v, 2)};
      }
      if (spins > kMaxSpins) {
        flag_timeout(p.result, lane);
        return Tot{0, 0, 0};
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  // the last arriver of group g: lane j reads tile g0+j's aggregate
  uint32_t a = 0, b = 0, c = 0;
  for (uint32_t spins = 0;; ++spins) {
    bool ok = true;
    if (lane < gsize) ok = read3(p.lb + (uint64_t)(g0 + lane) * 8, tag, a, b, c);
    if (__all(ok)) break;
    if (spins > kMaxSpins) {
      flag_timeout(p.result, lane);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  const uint32_t ia = wave_scan_sat(a, lane), ib = wave_scan_sat(b, lane),
                 ic = wave_scan_sat(c, lane);
  uint64_t* G = p.glb + (uint64_t)g * 8;
  Tot pg{0, 0, 0};
  if (g > 0) {
    store3(G, tag, __shfl(ia, gsize - 1), __shfl(ib, gsize - 1), __shfl(ic, gsize - 1), lane);
    pg = lookback(p.glb, g, tag, lane, p.result);
  }
  store3(G + 4, tag, sat_add(pg.n, __shfl(ia, gsize - 1)), sat_add(pg.k, __shfl(ib, gsize - 1)),
         sat_add(pg.v, __shfl(ic, gsize - 1)), lane);
  // exclusive = group prefix + inclusive - own (own <= inclusive unless saturated)
  const uint32_t ea = sat_add(pg.n, ia - a), eb = sat_add(pg.k, ib == 0xffffffffu ? ib : ib - b),
                 ec = sat_add(pg.v, ic - c);
  if (lane < gsize) {
    uint64_t* Xj = p.lb + (uint64_t)(g0 + lane) * 8 + 4;
    gstore(Xj + 0, (tag << kTagShift) | ea);
    gstore(Xj + 1, (tag << kTagShift) | eb);
    gstore(Xj + 2, (tag << kTagShift) | ec);
  }
  const uint32_t me = tile - g0;
  return Tot{__shfl(ea, me), __shfl(eb, me), __shfl(ec, me)};
}

// Blend bytes [a, b) (0 <= a < b <= 16) of w into acc (v_bfi per dword).
__device__ __forceinline__ uint32_t byte_mask(uint32_t a, uint32_t b, uint32_t d) {
  const uint32_t lo = a > 4 * d ? (a - 4 * d > 4 ? 4 : a - 4 * d) : 0;
  const uint32_t hi = b > 4 * d ? (b - 4 * d > 4 ? 4 : b - 4 * d) : 0;
  return (uint32_t)((1ull << (8 * hi)) - 1) & ~(uint32_t)((1ull << (8 * lo)) - 1);
}
__device__ __forceinline__ void blend16(uint4& acc, const uint4& w, uint32_t a, uint32_t b) {
  uint32_t m;
  m = byte_mask(a, b, 0); acc.x = (acc.x & ~m) | (w.x & m);
  m = byte_mask(a, b, 1); acc.y = (acc.y & ~m) | (w.y & m);
  m = byte_mask(a, b, 2); acc.z = (acc.z & ~m) | (w.z & m);
  m = byte_mask(a, b, 3); acc.w = (acc.w & ~m) | (w.w & m);
}

// Stream bytes [t, hi) of one block assembled into a 16-B register image whose byte i is
// stream byte t0 + i, starting from entry e (o(e) <= t).  Stream byte t of entry e: values
// -> block byte vs(e) + (t - vo(e)); keys -> u = t - ko(e) < plen(e) ? baseKey prefix
// (block byte base_pos + u) : stored diff (ks(e) + u - plen(e)) -- blockIterator.parseKV,
// iterator.go:98-100.  Each contiguous run is one unaligned 16-B LDS window + a byte blend.
template <bool IS_KEY>
__device__ __forceinline__ uint4 assemble(const uint8_t* slot, uint32_t sh, const uint16_t* meta,
                                          uint32_t e, uint32_t base_pos, int32_t t0, uint32_t t,
                                          uint32_t hi) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  ushort4 me = *reinterpret_cast<const ushort4*>(meta + 4 * e);
  ushort4 mn = *reinterpret_cast<const ushort4*>(meta + 4 * e + 4);
  while (t < hi) {
    uint32_t o0 = IS_KEY ? me.y : me.w, o1 = IS_KEY ? mn.y : mn.w;
    while (o1 <= t) {  // next entry (skips empty ones); never passes the sentinel since t < L
      e++;
      me = mn;
      mn = *reinterpret_cast<const ushort4*>(meta + 4 * e + 4);
      o0 = o1;
      o1 = IS_KEY ? mn.y : mn.w;
    }
    const uint32_t u = t - o0;
    uint32_t src, rend;
    if (!IS_KEY) {
      src = me.z + u;
      rend = o1;
    } else {
      const uint32_t plen = (o1 - o0) - ((uint32_t)me.z - me.x);
      if (u < plen) {
        src = base_pos + u;
        rend = o0 + plen;
      } else {
        src = me.x + (u - plen);
        rend = o1;
      }
    }
    if (rend > hi) rend = hi;
    const uint32_t a = t - (uint32_t)t0;  // chunk byte of this run's start (0..15)
    // window whose byte a is block byte src (>= 16 addressable LDS bytes precede the block)
    const uint4 w = lds_u128(slot - 16, sh + src + 16 - a);
    blend16(acc, w, a, rend - (uint32_t)t0);
    t = rend;
  }
  return acc;
}

__device__ __forceinline__ void store_bytes(uint8_t* dst, const uint4& v, uint32_t a, uint32_t b) {
  const uint32_t words[4] = {v.x, v.y, v.z, v.w};
  for (uint32_t i = a; i < b; i++) dst[i] = (uint8_t)(words[i >> 2] >> (8 * (i & 3)));
}

// Writes stream bytes [0, L) of one block to dst (global, any alignment): lane e owns every
// aligned 16-B output chunk whose first byte lies inside entry e's output range -- interior
// chunks are one LDS window and one dwordx4 store; a chunk that crosses into later entries is
// assembled run by run.  Entry 0's lane also writes the stream's leading partial chunk, and
// the chunk past the stream end is written byte-wise (the neighbouring block owns the rest).
template <bool IS_KEY>
__device__ void emit_stream(uint8_t* dst, uint32_t L, const uint8_t* slot, uint32_t sh,
                            const uint16_t* meta, uint32_t n, uint32_t base_pos, uint32_t lane) {
  if (L == 0) return;
  const uint32_t h = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 15u);
  uint8_t* dal = dst - h;  // chunk q covers stream bytes [16q - h, 16q - h + 16)
  for (uint32_t e = lane; e < n; e += kWave) {
    const ushort4 me = *reinterpret_cast<const ushort4*>(meta + 4 * e);
    const ushort4 mn = *reinterpret_cast<const ushort4*>(meta + 4 * e + 4);
    const uint32_t o0 = IS_KEY ? me.y : me.w, o1 = IS_KEY ? mn.y : mn.w;
    if (e == 0 && h != 0) {  // leading partial chunk: stream bytes [0, min(16 - h, L))
      const uint32_t hi = (16 - h < L) ? 16 - h : L;
      const uint4 v = assemble<IS_KEY>(slot, sh, meta, 0, base_pos, -(int32_t)h, 0, hi);
      store_bytes(dal, v, h, h + hi);
    }
    if (o0 == o1) continue;
    const uint32_t plen = IS_KEY ? (o1 - o0) - ((uint32_t)me.z - me.x) : 0u;
    for (uint32_t q = (o0 + h + 15) >> 4; 16 * q < o1 + h; q++) {
      const int32_t t0 = (int32_t)(16 * q) - (int32_t)h;  // >= o0 >= 0
      const uint32_t ut0 = (uint32_t)t0;
      if (ut0 + 16 > L) {  // trailing partial chunk
        const uint4 v = assemble<IS_KEY>(slot, sh, meta, e, base_pos, t0, ut0, L);
        store_bytes(dal + 16 * q, v, 0, L - ut0);
        continue;
      }
      uint4 v;
      const uint32_t u0 = ut0 - o0;
      if (ut0 + 16 <= o1 && (!IS_KEY || u0 >= plen)) {        // inside the value / key diff
        v = lds_u128(slot, sh + (IS_KEY ? me.x + (u0 - plen) : me.z + u0));
      } else if (IS_KEY && u0 + 16 <= plen) {                  // inside the baseKey prefix
        v = lds_u128(slot, sh + base_pos + u0);
      } else {
        v = assemble<IS_KEY>(slot, sh, meta, e, base_pos, t0, ut0, ut0 + 16);
      }
      *reinterpret_cast<uint4*>(dal + 16 * q) = v;
    }
  }
}

// Bytes [lo, hi) of the 16-B chunk that starts at stream byte t0, for a stream whose entry e
// occupies [o(e), o(e+1)) and comes from block bytes starting at src(e) (no prefixes: keys of
// a plen == 0 block or values).  Entry e must contain lo.  One window + blend per entry run.
template <int OCOL, int SCOL>
__device__ __forceinline__ uint4 assemble_plain(const uint8_t* slot, uint32_t sh,
                                                const uint16_t* meta, uint32_t e, int32_t t0,
                                                uint32_t lo, uint32_t hi) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  uint32_t t = lo;
  uint32_t o0 = meta[4 * e + OCOL], s0 = meta[4 * e + SCOL];
  while (t < hi) {
    const uint32_t o1 = meta[4 * (e + 1) + OCOL];
    const uint32_t rend = o1 < hi ? o1 : hi;
    if (rend > t) {
      const uint32_t a = t - (uint32_t)t0;
      const uint4 w = lds_u128(slot - 16, sh + s0 + (t - o0) + 16 - a);
      blend16(acc, w, a, rend - (uint32_t)t0);
      t = rend;
    }
    e++;
    o0 = o1;
    s0 = meta[4 * e + SCOL];
  }
  return acc;
}

// One stream (OCOL = output-offset column, SCOL = block-position column) of one block,
// lane-per-entry: interior chunks are one window + one aligned dwordx4 store; the chunk that
// crosses the entry's end is assembled; the stream's partial head / tail chunks are stored
// byte-wise (the neighbouring blocks own the other bytes of those chunks).
template <int OCOL, int SCOL>
__device__ __forceinline__ void emit_plain(uint8_t* dst, uint32_t L, const uint8_t* slot,
                                           uint32_t sh, const uint16_t* meta, uint32_t e,
                                           uint32_t o0, uint32_t o1, uint32_t s0, uint32_t h) {
  uint8_t* dal = dst - h;  // chunk q covers stream bytes [16q - h, 16q - h + 16)
  if (e == 0 && h != 0) {
    const uint32_t hi = (16 - h < L) ? 16 - h : L;
    const uint4 v = assemble_plain<OCOL, SCOL>(slot, sh, meta, 0, -(int32_t)h, 0, hi);
    store_bytes(dal, v, h, h + hi);
  }
  // chunks fully inside [o0, o1)
  const uint32_t qa = (o0 + h + 15) >> 4, qb = (o1 + h) >> 4;  // [qa, qb)
  for (uint32_t q = qa; q < qb; q++)
    *reinterpret_cast<uint4*>(dal + 16 * q) = lds_u128(slot, sh + s0 + (16 * q - h - o0));
  // the chunk starting inside [o0, o1) that crosses o1 (or the stream end)
  const uint32_t qc = qb > qa ? qb : qa;
  const int32_t t0 = (int32_t)(16 * qc) - (int32_t)h;
  if ((uint32_t)t0 < o1 && t0 >= (int32_t)o0) {
    const uint32_t hi = ((uint32_t)t0 + 16 < L) ? (uint32_t)t0 + 16 : L;
    const uint4 v = assemble_plain<OCOL, SCOL>(slot, sh, meta, e, t0, (uint32_t)t0, hi);
    if (hi == (uint32_t)t0 + 16) *reinterpret_cast<uint4*>(dal + 16 * qc) = v;
    else store_bytes(dal + 16 * qc, v, 0, hi - (uint32_t)t0);
  }
}

// Global-memory path with the same semantics: re-walks the block and copies every entry's
// key and value with the wave's lanes (byte granular).  Used for oversize blocks only.
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

// Workgroup rendezvous for LDS data only: unlike __syncthreads() it does not drain vmcnt,
// so the next tile's prefetch loads and this tile's stream stores stay in flight.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int SLOT, int MAXE, int WPB>
struct DecodeCfg {
  static constexpr int kPad = 16;                  // addressable bytes before the block
  static constexpr int kBuf = kPad + SLOT + 32;    // block (<= SLOT) at shift < 16 + over-read
  static constexpr int kMeta = (MAXE + 1) * 8;
  static constexpr int kWaveBytes = (2 * kBuf + kMeta + 15) & ~15;  // double-buffered slot
  static constexpr int kShared = 64 + WPB * 16;    // tile base + per-wave aggregates
  static constexpr int kLds = kWaveBytes * WPB + kShared;
  static constexpr int kIters = (SLOT + 16 + 16 * kWave - 1) / (16 * kWave);  // 1-KiB DMA pieces
};

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

struct BlockRef {
  uint64_t off;
  uint32_t len, sh;
  bool fits, tail;  // tail: a chunk crosses the end of the data buffer (loaded by lanes)
};

// Issue block b's bytes into `buf` by LDS-DMA (global_load_lds_dwordx4: 1 KiB per wave
// instruction, no VGPRs), 16-B aligned source; the chunk crossing the end of the data buffer
// (last block only) is left for land_tail().
template <int SLOT, int ITERS>
__device__ __forceinline__ BlockRef prefetch_block(const DecodeParams& p, uint32_t b, uint8_t* buf,
                                                   uint32_t lane) {
  BlockRef r{0, 0, 0, false, false};
  if (b >= p.nblk) return r;
  r.off = uniform(p.blk_off[b]);
  r.len = uniform(p.blk_len[b]);
  r.fits = r.len <= (uint32_t)SLOT && r.off + r.len <= p.data_len;
  if (!r.fits) return r;
  const uint64_t a0 = r.off & ~15ull;
  r.sh = (uint32_t)(r.off - a0);
  const uint32_t nchunk = (r.sh + r.len + 15) >> 4;
  r.tail = a0 + 16ull * nchunk > p.data_len;
#pragma unroll
  for (int i = 0; i < ITERS; i++) {
    const uint32_t c = lane + i * kWave;
    const uint64_t a = a0 + 16ull * c;
    if (c < nchunk && a + 16 <= p.data_len)
      __builtin_amdgcn_global_load_lds((glb_void_t*)(p.data + a), (lds_void_t*)(buf + i * 1024),
                                       16, 0, 0);
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

template <int SLOT, int MAXE, int WPB>
__global__ void __launch_bounds__(WPB * 64) decode_kernel(DecodeParams p) {
  using Cfg = DecodeCfg<SLOT, MAXE, WPB>;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = lane_id();
  const uint32_t wv = uniform(threadIdx.x >> 6);
  uint8_t* wbase = smem + wv * Cfg::kWaveBytes;
  uint16_t* meta = reinterpret_cast<uint16_t*>(wbase + 2 * Cfg::kBuf);
  uint32_t* s_base = reinterpret_cast<uint32_t*>(smem + WPB * Cfg::kWaveBytes);  // [3]
  uint32_t* s_agg = s_base + 16;                                                // [WPB][4]
  const uint64_t tag = p.tag;
  const uint32_t ntiles = (p.nblk + WPB - 1) / WPB;

  // Static round-robin over a fully resident grid (gridDim.x a multiple of 64 workgroups, or
  // >= the tile count): a 64-tile group lies inside one round, every wait points at an
  // earlier group or at a member of the same group in the same round -> no deadlock; spins
  // are bounded anyway.  (A shared ticket counter would serialise at ~88 atomics/us.)
  uint32_t tile = blockIdx.x;
  uint32_t cur = 0;
  BlockRef ref = prefetch_block<SLOT, Cfg::kIters>(p, tile * WPB + wv, wbase + Cfg::kPad, lane);
  for (; tile < ntiles; tile += gridDim.x) {
    uint8_t* slot = wbase + cur * Cfg::kBuf + Cfg::kPad;
    const uint32_t b = tile * WPB + wv;
    const bool valid = b < p.nblk;
    WalkResult w{0, 0, 0, LSMGPU_BLK_OK, 0, 0};
    bool fast = false, any_plen = false;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this block's DMA has landed
    if (valid) {
      if (ref.off + ref.len > p.data_len) {
        w.status = LSMGPU_BLK_RANGE;
      } else if (ref.fits) {
        if (ref.tail) land_tail(p, ref, slot, lane);
        wave_lds_fence();
        if (p.ablate & 4) {
          w = WalkResult{0, 0, 0, 0, 0, 0};
        } else {
          const SpecResult r = walk_spec(slot, ref.sh, ref.len, meta, MAXE, lane);
          if (r.n <= (uint32_t)MAXE) {
            wave_lds_fence();
            w = finish_meta(slot, ref.sh, r, meta, lane, any_plen);
            fast = (w.K <= 0xffffu) && (w.V <= 0xffffu);
          } else {  // too many entries for the metadata: count on the global path
            w = walk_block(GlobalSrc{p.data + ref.off}, ref.len, meta, 0, false, lane);
          }
        }
      } else {
        w = walk_block(GlobalSrc{p.data + ref.off}, ref.len, meta, 0, false, lane);
      }
    }
    // ---- tile scan of the per-block aggregates (LDS)
    if (lane == 0) {
      s_agg[4 * wv + 0] = w.n;
      s_agg[4 * wv + 1] = w.K;
      s_agg[4 * wv + 2] = w.V;
    }
    lds_barrier();
    // next tile's block -> the other buffer, now: the DMA overlaps the prefix wait and the emit
    const uint32_t next = tile + gridDim.x;
    const BlockRef nref = prefetch_block<SLOT, Cfg::kIters>(
        p, next * WPB + wv, wbase + (cur ^ 1) * Cfg::kBuf + Cfg::kPad, lane);
    if (wv == 0) {
      uint32_t a = 0, bk = 0, c = 0;
      if (lane < (uint32_t)WPB) {
        a = s_agg[4 * lane];
        bk = s_agg[4 * lane + 1];
        c = s_agg[4 * lane + 2];
      }
      const uint32_t ia = wave_scan_sat(a, lane), ib = wave_scan_sat(bk, lane),
                     ic = wave_scan_sat(c, lane);
      const uint32_t ta = __shfl(ia, WPB - 1), tb = __shfl(ib, WPB - 1), tc = __shfl(ic, WPB - 1);
      Tot ex{0, 0, 0};
      if (!(p.ablate & 1)) {
        store3(p.lb + (uint64_t)tile * 8, tag, ta, tb, tc, lane);
        ex = tile_prefix(p, tile, ntiles, tag, lane);
      }
      if (lane < (uint32_t)WPB) {  // per-block exclusive bases within the tile
        s_agg[4 * lane] = ia - a;
        s_agg[4 * lane + 1] = ib == 0xffffffffu ? ib : ib - bk;
        s_agg[4 * lane + 2] = ic - c;
      }
      if (lane == 0) {
        s_base[0] = ex.n;
        s_base[1] = ex.k;
        s_base[2] = ex.v;
        if (tile == ntiles - 1) {
          if (p.blk_first) p.blk_first[p.nblk] = ex.n + ta;
          p.result[0] = sat_add(ex.n, ta);
          p.result[1] = sat_add(ex.k, tb);
          p.result[2] = sat_add(ex.v, tc);
        }
      }
    }
    lds_barrier();
    if (valid) {
      const Tot ex{s_base[0] + s_agg[4 * wv], sat_add(s_base[1], s_agg[4 * wv + 1]),
                   s_base[2] + s_agg[4 * wv + 2]};
      if (lane == 0) {
        if (p.blk_first) p.blk_first[b] = (uint32_t)ex.n;
        if (p.blk_status) p.blk_status[b] = (int32_t)w.status;
        if (w.status != LSMGPU_BLK_OK) {
          atomicAdd(reinterpret_cast<unsigned long long*>(p.result + 4), 1ull);
          atomicMax(reinterpret_cast<unsigned long long*>(p.result + 3),
                    (unsigned long long)(p.nblk - b));
        }
      }
      const bool mat = (p.mode & LSMGPU_MODE_MATERIALIZE) != 0;
      const bool view = (p.mode & LSMGPU_MODE_VIEW) != 0 && p.view;
      bool ok = (uint64_t)ex.n + w.n <= p.ent_cap;
      if (mat) {
        const uint64_t kend = (uint64_t)ex.k + w.K, vend = (uint64_t)ex.v + w.V;
        ok = ok && (kend <= p.key_cap || !p.key_data) && (vend <= p.val_cap || !p.val_data);
        ok = ok && kend < 0xffffffffull && vend <= 0xffffffffull;
      }
      if (!ok && lane == 0) atomicOr(reinterpret_cast<unsigned long long*>(p.result + 5), 1ull);
      if (ok && w.n > 0 && !(p.ablate & 2)) {
        if (!fast) {
          emit_slow(p, p.data + ref.off, w.n, ex.n, ex.k, ex.v, ref.off, lane);
        } else {
          const uint32_t en = ex.n, ek = ex.k, evv = ex.v;
          const bool keys_plain = !any_plen;
          const uint32_t hk = (uint32_t)(reinterpret_cast<uintptr_t>(p.key_data + ek) & 15u);
          const uint32_t hv = (uint32_t)(reinterpret_cast<uintptr_t>(p.val_data + evv) & 15u);
          // lane e: entry e's offsets / view record and the stream chunks starting inside it
          for (uint32_t e = lane; e < w.n; e += kWave) {
            const ushort4 me = *reinterpret_cast<const ushort4*>(meta + 4 * e);
            const ushort4 mn = *reinterpret_cast<const ushort4*>(meta + 4 * e + 4);
            if (mat) {
              if (p.key_end) p.key_end[en + e] = ek + mn.y;
              if (p.val_end) p.val_end[en + e] = evv + mn.w;
              if (p.val_data)
                emit_plain<3, 2>(p.val_data + evv, w.V, slot, ref.sh, meta, e, me.w, mn.w, me.z, hv);
              if (p.key_data && keys_plain)
                emit_plain<1, 0>(p.key_data + ek, w.K, slot, ref.sh, meta, e, me.y, mn.y, me.x, hk);
            }
            if (view) {
              const uint32_t klen = (uint32_t)me.z - me.x, vlen = (uint32_t)mn.w - me.w;
              p.view[en + e] = (uint64_t)(uint32_t)(ref.off + me.x) | ((uint64_t)klen << 32) |
                               ((uint64_t)vlen << 48);
            }
          }
          if (mat && p.key_data && !keys_plain)  // prefix-compressed keys (plen > 0)
            emit_stream<true>(p.key_data + ek, w.K, slot, ref.sh, meta, w.n, w.base_pos, lane);
        }
      }
    }
    ref = nref;
    cur ^= 1;
    wave_lds_fence();
  }
}

// Upper bound on the decode kernels' SGPR count (hipcc -Rpass-analysis=kernel-resource-usage),
// checked by tests/test_abi.py::test_decode_resource_budget.
constexpr int kDecodeSgprs = 112;

template <int SLOT, int MAXE, int WPB>
static hipError_t launch_cfg(const DecodeParams& p, int num_cus, hipStream_t s,
                             uint64_t* waves_launched) {
  using Cfg = DecodeCfg<SLOT, MAXE, WPB>;
  auto k = decode_kernel<SLOT, MAXE, WPB>;
  static int per_cu = 0;
  if (per_cu == 0) {
    if (Cfg::kLds > 64 * 1024) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, Cfg::kLds);
      if (e != hipSuccess) return e;
    }
    // residency = min(occupancy API, LDS, SGPR-file bound) (MI355X_MICROARCH: the API can
    // over-report by one block per CU for SGPR-heavy kernels)
    int api = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&api, k, WPB * 64, Cfg::kLds);
    if (e != hipSuccess) return e;
    const int waves_per_simd = 800 / (((kDecodeSgprs + 15) / 16) * 16 + 16);
    const int waves_per_cu = (waves_per_simd > 8 ? 8 : waves_per_simd) * 4;
    const int sg_bound = waves_per_cu / WPB;
    const int lds_bound = (160 * 1024) / Cfg::kLds;
    per_cu = api;
    if (per_cu > lds_bound) per_cu = lds_bound;
    if (per_cu > sg_bound) per_cu = sg_bound;
    if (per_cu < 1) per_cu = 1;
  }
  // a multiple of 64 workgroups (each 64-tile group sits in one round), never more than what
  // is resident at once, never more than the tiles
  uint64_t grid = (uint64_t)per_cu * (uint64_t)num_cus;
  grid = grid / 64 * 64;
  if (grid < 64) grid = 64;
  const uint64_t ntiles = ((uint64_t)p.nblk + WPB - 1) / WPB;
  if (grid > ntiles) grid = ntiles;  // one round: every tile has its own workgroup
  if (grid < 1) grid = 1;
  *waves_launched = grid * WPB;
  static const bool dbg = getenv("LSMGPU_DEBUG") != nullptr;
  static const uint32_t ablate =
      getenv("LSMGPU_ABLATE") ? (uint32_t)atoi(getenv("LSMGPU_ABLATE")) : 0u;
  DecodeParams q = p;
  q.ablate = ablate;
  if (dbg)
    fprintf(stderr, "[lsmgpu] decode SLOT=%d MAXE=%d WPB=%d lds=%d per_cu=%d cus=%d grid=%llu nblk=%u\n",
            SLOT, MAXE, WPB, Cfg::kLds, per_cu, num_cus, (unsigned long long)grid, p.nblk);
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(WPB * 64), Cfg::kLds, s, q);
  return hipGetLastError();
}

hipError_t launch_decode(const DecodeParams& p, uint32_t max_blk_len, int num_cus,
                         hipStream_t s, uint64_t* waves_launched) {
  if (max_blk_len <= 4096) return launch_cfg<4096, 128, 4>(p, num_cus, s, waves_launched);
  if (max_blk_len <= 8192) return launch_cfg<8192, 256, 4>(p, num_cus, s, waves_launched);
  if (max_blk_len <= 16384) return launch_cfg<16384, 512, 2>(p, num_cus, s, waves_launched);
  // 32 KiB slot; larger blocks run the global-memory path inside the same kernel
  return launch_cfg<32768, 1024, 1>(p, num_cus, s, waves_launched);
}

}  // namespace lsmgpu
