// decode_onepass.hip -- one-pass SST block decode: HBM sees the input once.
//
// Walk-scan-copy (decode_wsc.hip) walks every block from HBM and then copies it in a second
// launch that reads the input again (2.19x the algorithmic reads).  Here each wave
// is a worker that takes tiles of TB consecutive blocks in ticket order (p.gcnt) and, per tile:
//   1. fetches every 128-B line of the tile once with independent byte loads -- the only HBM
//      read of the input; the lines land in L2 and the 256 MiB Infinity Cache;
//   2. walks each block with L lanes guessing same-shape runs, exactly blockIterator.Next /
//      parseKV (table/iterator.go:93-135), from those cached lines; the per-entry records
//      {header pos | value offset << 16} stay in LDS (entries past R spill to p.wmeta);
//   3. publishes the tile's {entries, key bytes, value bytes} and finds its output base by
//      decoupled look-back over the tile records (decode_common.hpp);
//   4. copies every entry's key and value from the cached lines (16-B pieces, the last
//      overlapping back inside its stream, as the walk-scan-copy copy does) and writes the end
//      offsets / view records, one lane per entry.
// A tile lives a few tens of microseconds between 1 and 4; with ~8-16 workers per CU the live
// set is ~100 MB, inside the Infinity Cache.  Blocks must be < 64 KiB (u16 record fields).
#include <algorithm>
#include <cstdlib>

#include "codec_common.hpp"
#include "decode_common.hpp"
#include "kernels.hpp"

namespace lsmgpu {

namespace {

// big-endian u16 fields of the 10-B header at g (table/builder.go:23-45), unaligned global read
__device__ __forceinline__ void hdr_at(const uint8_t* g, uint32_t& plen, uint32_t& klen,
                                       uint32_t& vlen) {
  uint2 w;
  __builtin_memcpy(&w, g, 8);  // one unaligned global_load_dwordx2
  plen = __builtin_amdgcn_perm(0u, w.x, 0x0c0c0001u);
  klen = __builtin_amdgcn_perm(0u, w.x, 0x0c0c0203u);
  vlen = __builtin_amdgcn_perm(0u, w.y, 0x0c0c0001u);
}

constexpr uint32_t kPlen = 1u << 16;  // status word flag: the block has prefix-compressed entries

// the records of one block: 0 .. R-1 in the worker's LDS slot, the rest in the global spill
template <uint32_t R>
struct Recs {
  const uint32_t* lds;
  const uint32_t* ovf;
  __device__ __forceinline__ uint32_t operator()(uint32_t i) const { return i < R ? lds[i] : ovf[i]; }
};

// key_end / val_end / view of a block with no prefix-compressed entry, one lane per entry (64
// consecutive words per store instruction).  Stored key length = next pos - pos - 10 - value
// length; key offset = pos - 10 e - value offset (every earlier entry contributed its header,
// key and value).
template <class Rec>
__device__ __forceinline__ void entry_outputs(const DecodeParams& p, const Rec& rec, uint32_t n,
                                              uint64_t en, uint64_t ek, uint64_t ev, uint32_t off,
                                              bool mat, bool view, uint32_t lane) {
  for (uint32_t c0 = 0; c0 < n; c0 += kWave) {
    const uint32_t e = c0 + lane;
    if (e >= n) continue;
    const uint32_t m0 = rec(e), m1 = rec(e + 1);
    const uint32_t hp = m0 & 0xffffu, vo = m0 >> 16, hp1 = m1 & 0xffffu, vo1 = m1 >> 16;
    const uint32_t vl = vo1 - vo, kl = hp1 - hp - 10 - vl;
    if (mat) {
      if (p.key_end) p.key_end[en + e] = (uint32_t)(ek + hp1 - 10 * (e + 1) - vo1);
      if (p.val_end) p.val_end[en + e] = (uint32_t)(ev + vo1);
    }
    if (view) p.view[en + e] = (uint64_t)(off + hp + 10) | ((uint64_t)kl << 32) | ((uint64_t)vl << 48);
  }
}

// the key and value bytes of a block with no prefix-compressed entry: J lanes per entry, G entry
// groups per pass with every record read first; lane j copies pieces j, j + J, ... of
// [key pieces | value pieces]
template <uint32_t J, uint32_t G, class Rec>
__device__ __forceinline__ void copy_bytes(const Rec& rec, const uint8_t* blk, uint8_t* kbase,
                                           uint8_t* vbase, uint32_t n, uint32_t lane) {
  const uint32_t j = lane & (J - 1);
  for (uint32_t e0 = 0; e0 < n; e0 += G * (kWave / J)) {
    uint32_t hp[G], kl[G], vl[G], ko[G], vo[G], np[G], kp[G];
    bool on[G];
#pragma unroll
    for (int i = 0; i < (int)G; i++) {
      const uint32_t e = e0 + i * (kWave / J) + lane / J;
      const uint32_t ec = min(e, n - 1);
      const uint32_t m0 = rec(ec), m1 = rec(ec + 1);
      hp[i] = m0 & 0xffffu;
      vo[i] = m0 >> 16;
      vl[i] = (m1 >> 16) - vo[i];
      kl[i] = (m1 & 0xffffu) - hp[i] - 10 - vl[i];
      ko[i] = hp[i] - 10 * ec - vo[i];
      on[i] = e < n;
      kp[i] = pieces16(kl[i]);
      np[i] = kp[i] + pieces16(vl[i]);
    }
#pragma unroll
    for (int i = 0; i < (int)G; i++) {
      if (!on[i]) continue;
      for (uint32_t q = j; q < np[i]; q += J) {
        const bool key = q < kp[i];
        uint8_t* dst = key ? kbase : vbase;
        if (!dst) continue;
        const uint32_t len = key ? kl[i] : vl[i];
        const uint32_t s0 = key ? hp[i] + 10 : hp[i] + 10 + kl[i];
        copy_piece16(dst + (key ? ko[i] : vo[i]), blk + s0, len, key ? q : q - kp[i]);
      }
    }
  }
}

// the same, with every lane's first piece of each of the G entries loaded before any is stored
// (one wait for the pass instead of a load -> store round trip per piece: the lines come from
// L2 / the Infinity Cache, so the copy is latency-bound per worker); further pieces (entries
// wider than J 16-B pieces) take the piecewise loop
__device__ __forceinline__ void piece_at(const uint8_t* src, uint8_t* dst, uint32_t len, uint32_t q,
                                         const uint8_t*& s, uint8_t*& d, uint32_t& w) {
  if (len >= 16) {
    const uint32_t o = min(16 * q, len - 16);
    s = src + o; d = dst + o; w = 16;
  } else if (len >= 8) {
    const uint32_t o = q ? len - 8 : 0;
    s = src + o; d = dst + o; w = 8;
  } else if (len >= 4) {
    const uint32_t o = q ? len - 4 : 0;
    s = src + o; d = dst + o; w = 4;
  } else {
    s = src + q; d = dst + q; w = 1;
  }
}
__device__ __forceinline__ uint4 load_w(const uint8_t* s, uint32_t w) {
  uint4 v = make_uint4(0, 0, 0, 0);
  if (w == 16) __builtin_memcpy(&v, s, 16);
  else if (w == 8) __builtin_memcpy(&v, s, 8);
  else if (w == 4) __builtin_memcpy(&v, s, 4);
  else v.x = *s;
  return v;
}
__device__ __forceinline__ void store_w(uint8_t* d, uint4 v, uint32_t w) {
  if (w == 16) __builtin_memcpy(d, &v, 16);
  else if (w == 8) __builtin_memcpy(d, &v, 8);
  else if (w == 4) __builtin_memcpy(d, &v, 4);
  else *d = (uint8_t)v.x;
}
template <uint32_t J, uint32_t G, class Rec>
__device__ __forceinline__ void copy_bytes_batched(const Rec& rec, const uint8_t* blk, uint8_t* kbase,
                                                   uint8_t* vbase, uint32_t n, uint32_t lane) {
  const uint32_t j = lane & (J - 1);
  for (uint32_t e0 = 0; e0 < n; e0 += G * (kWave / J)) {
    uint32_t hp[G], kl[G], vl[G], ko[G], vo[G], np[G], kp[G];
    bool on[G];
#pragma unroll
    for (int i = 0; i < (int)G; i++) {
      const uint32_t e = e0 + i * (kWave / J) + lane / J;
      const uint32_t ec = min(e, n - 1);
      const uint32_t m0 = rec(ec), m1 = rec(ec + 1);
      hp[i] = m0 & 0xffffu;
      vo[i] = m0 >> 16;
      vl[i] = (m1 >> 16) - vo[i];
      kl[i] = (m1 & 0xffffu) - hp[i] - 10 - vl[i];
      ko[i] = hp[i] - 10 * ec - vo[i];
      on[i] = e < n;
      kp[i] = pieces16(kl[i]);
      np[i] = kp[i] + pieces16(vl[i]);
    }
    uint4 v[G];
    uint8_t* d[G];
    uint32_t w[G];
#pragma unroll
    for (int i = 0; i < (int)G; i++) {  // piece j of every entry: all loads first
      const uint8_t* sp = blk;
      d[i] = nullptr;
      w[i] = 0;
      if (on[i] && j < np[i]) {
        const bool key = j < kp[i];
        uint8_t* dst = key ? kbase : vbase;
        if (dst) {
          piece_at(blk + (key ? hp[i] + 10 : hp[i] + 10 + kl[i]), dst + (key ? ko[i] : vo[i]),
                   key ? kl[i] : vl[i], key ? j : j - kp[i], sp, d[i], w[i]);
          v[i] = load_w(sp, w[i]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < (int)G; i++)
      if (d[i]) store_w(d[i], v[i], w[i]);
#pragma unroll
    for (int i = 0; i < (int)G; i++) {  // pieces j + J, j + 2J, ... (entries wider than J pieces)
      if (!on[i]) continue;
      for (uint32_t q = j + J; q < np[i]; q += J) {
        const bool key = q < kp[i];
        uint8_t* dst = key ? kbase : vbase;
        if (!dst) continue;
        const uint32_t len = key ? kl[i] : vl[i];
        const uint32_t s0 = key ? hp[i] + 10 : hp[i] + 10 + kl[i];
        copy_piece16(dst + (key ? ko[i] : vo[i]), blk + s0, len, key ? q : q - kp[i]);
      }
    }
  }
}

// a block with prefix-compressed entries (plen > 0: never written by Builder; the
// format the iterator accepts): entries 64 at a time, lane = entry, plen read from the header,
// key offsets by a wave scan of plen + stored key bytes; keys bytewise as baseKey[:plen] ++ diff
// (iterator.go:98-100), values as 16-B pieces
template <class Rec>
__device__ __forceinline__ void copy_plen(const DecodeParams& p, const Rec& rec, const uint8_t* blk,
                                          uint8_t* kbase, uint8_t* vbase, uint32_t n, uint64_t en,
                                          uint64_t ek, uint64_t ev, uint32_t off, bool mat,
                                          bool view, uint32_t lane) {
  uint32_t carry = 0;  // key bytes of the entries before this chunk
  for (uint32_t e0 = 0; e0 < n; e0 += kWave) {
    const uint32_t e = e0 + lane;
    const bool on = e < n;
    const uint32_t m0 = rec(min(e, n)), m1 = rec(min(e + 1, n));
    const uint32_t hp = m0 & 0xffffu, vo = m0 >> 16;
    const uint32_t vl = (m1 >> 16) - vo, kl = (m1 & 0xffffu) - hp - 10 - vl;
    const uint32_t plen = on ? ((uint32_t)blk[hp] << 8) | blk[hp + 1] : 0u;
    const uint32_t kout = on ? plen + kl : 0u;
    const uint32_t incl = wave_scan_sat(kout, lane);
    const uint32_t ko = carry + incl - kout;
    carry += __builtin_amdgcn_readlane(incl, 63);
    if (!on) continue;
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

}  // namespace

// One wave per workgroup; workers loop over ticket-ordered tiles until the tickets run out (the
// worker drawing the last exit ticket resets p.gcnt for the next launch).  Lower tickets are
// always held by running workers, so every look-back progresses without a residency assumption.
template <uint32_t TB, uint32_t L, uint32_t R>
__global__ void __launch_bounds__(64) onepass_kernel(DecodeParams p) {
  static_assert(TB * L == kWave, "L lanes for each of the tile's TB blocks");
  static_assert(L >= 2 && L <= 16 && (L & (L - 1)) == 0, "2..16 lanes per block");
  constexpr uint32_t kMask = (1u << L) - 1;
  constexpr uint32_t kGroupProbe = 16;
  __shared__ __attribute__((aligned(16))) uint32_t recs[TB * R];
  const uint32_t lane = lane_id();
  const uint32_t ntiles = (p.nblk + TB - 1) / TB;
  const bool mat = (p.mode & LSMGPU_MODE_MATERIALIZE) != 0;
  const bool view = (p.mode & LSMGPU_MODE_VIEW) != 0 && p.view;
  const uint32_t g = lane / L, k = lane & (L - 1), gb = lane & ~(L - 1);
  for (;;) {
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(p.gcnt, 1u);
    t = uniform((uint32_t)__shfl((int)t, 0));
    if (t >= ntiles) {
      if (lane == 0 && t == ntiles + gridDim.x - 1) atomicExch(p.gcnt, 0u);
      return;
    }
    // ---- 1 + 2: fetch the block's lines, then walk it (L lanes per block) ----
    const uint32_t b = t * TB + g;
    const bool valid = b < p.nblk;
    uint32_t off = 0, len = 0;
    if (valid) {
      off = p.blk_off[b];
      len = p.blk_len[b];
    }
    const bool inrange = valid && (uint64_t)off + len <= p.data_len;
    const uint8_t* blk = p.data + off;
    uint32_t* row = recs + g * R;
    uint32_t* ovf = p.wmeta + (uint64_t)(valid ? b : 0) * p.wcap;
    uint32_t pos = 0, gn = 0, gK = 0, gV = 0, gst = valid && !inrange ? LSMGPU_BLK_RANGE : LSMGPU_BLK_OK;
    if (p.wprefetch && inrange && len) {
      // one byte of every 128-B line of the block (the first at the block's first byte): the
      // L2 fetches whole lines; independent loads, one wait
      const uintptr_t a0 = (uintptr_t)blk, first = a0 & ~(uintptr_t)127;
      const uint32_t nl = (uint32_t)((a0 + len - 1 - first) >> 7) + 1;
      uint32_t acc = 0;
      for (uint32_t i0 = 0; i0 < nl; i0 += 8 * L) {
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const uint32_t i = i0 + u * L + k;
          const uintptr_t a = first + ((uintptr_t)i << 7);
          v[u] = i < nl ? *reinterpret_cast<const uint8_t*>(a < a0 ? a0 : a) : 0u;
        }
#pragma unroll
        for (int u = 0; u < 8; u++) acc += v[u];
      }
      if (acc == 0xffffffffu) p.result[7] = acc;  // keeps the loads; never true (< 2^16 * 255)
    }
    if (inrange) {
      uint32_t kref = 0xffffffffu, vref = 0, stride = 0;  // no shape yet: round 1 takes one
      uint32_t rounds = 0;
      for (;;) {
        const uint32_t q = pos + k * stride;  // < 2^21
        uint32_t plen = 1, klen = 0, vlen = 0;
        if (q + 10 <= len) hdr_at(blk + q, plen, klen, vlen);
        const uint32_t endq = q + 10 + klen + vlen;
        const bool fast = (klen != 0) & (plen == 0) & (endq <= len);
        const bool same = fast & (klen == kref) & (vlen == vref);
        const uint32_t fb = (uint32_t)(__ballot(fast) >> gb) & kMask;
        const uint32_t sb = (uint32_t)(__ballot(same) >> gb) & kMask;
        if (!(fb & 1u)) break;  // entry gn itself needs the general loop (or the block ended)
        const uint32_t tr = __builtin_ctz(~sb);                             // same-shape run
        const uint32_t m = tr + ((tr < L && ((fb >> tr) & 1u)) ? 1u : 0u);  // + one new shape
        const uint32_t idx = gn + k;
        if (k < m) {
          const uint32_t rec = q | ((gV + k * vref) << 16);
          if (idx < R) row[idx] = rec; else ovf[idx] = rec;
        }
        const uint32_t src = gb + m - 1;  // the last accepted entry
        pos = (uint32_t)__shfl((int)endq, (int)src);
        const uint32_t shape = (uint32_t)__shfl((int)(klen | (vlen << 16)), (int)src);
        gK += tr * kref + (m > tr ? (shape & 0xffffu) : 0u);
        gV += tr * vref + (m > tr ? (shape >> 16) : 0u);
        gn += m;
        if (tr == 0) {  // entry gn broke the run: adopt its shape (one odd entry keeps the old)
          kref = shape & 0xffffu;
          vref = shape >> 16;
          stride = 10 + kref + vref;
        }
        rounds++;
        if (rounds >= kGroupProbe && 4 * gn < 5 * rounds) break;  // shapes do not repeat
      }
      if (k == 0) {  // general loop: every stop rule in the iterator's order
        for (;;) {
          if (pos >= len) break;                                   // iterator.go:115-118
          if (len - pos < 10) { gst = LSMGPU_BLK_TRUNC_HEADER; break; }
          uint32_t plen, klen, vlen;
          hdr_at(blk + pos, plen, klen, vlen);                     // iterator.go:121
          if ((klen | plen) == 0) break;                           // iterator.go:124-127
          if (gn == 0 && plen != 0) { gst = LSMGPU_BLK_FIRST_PLEN; break; }  // :129-133
          if (10 + plen > len) { gst = LSMGPU_BLK_PREFIX_OOB; break; }
          const uint32_t end = pos + 10 + klen + vlen;             // iterator.go:101-109
          if (end > len) { gst = LSMGPU_BLK_VALUE_OVERFLOW; break; }
          const uint32_t rec = pos | (gV << 16);
          if (gn < R) row[gn] = rec; else ovf[gn] = rec;
          gK += plen + klen;
          gV += vlen;
          gn++;
          pos = end;
        }
        const uint32_t sent = pos | (gV << 16);  // sentinel: stop pos, V
        if (gn < R) row[gn] = sent; else ovf[gn] = sent;
      }
    }
    // the block's {n, K, V, status} live in lane gb (k == 0); the others contribute zeros
    const bool own = k == 0 && valid;
    const uint32_t n = own ? gn : 0u, K = own ? gK : 0u, V = own ? gV : 0u;
    const uint32_t sw = own ? (gst | (gK != pos - 10 * gn - gV ? kPlen : 0u)) : 0u;
    // ---- 3: tile scan, publish, decoupled look-back ----
    const uint32_t in_ = wave_scan_sat(n, lane), ik = wave_scan_sat(K, lane),
                   iv = wave_scan_sat(V, lane);
    const uint32_t tn = __builtin_amdgcn_readlane(in_, 63), tk = __builtin_amdgcn_readlane(ik, 63),
                   tv = __builtin_amdgcn_readlane(iv, 63);
    uint64_t* Rt = p.lb + (uint64_t)t * 8;
    Tot ex{0, 0, 0};
    if (t > 0) {
      store3(Rt, p.tag, tn, tk, tv, lane);
      ex = lookback(p.lb, t, p.tag, lane, p.result);
    }
    store3(Rt + 4, p.tag, sat_add(ex.n, tn), sat_add(ex.k, tk), sat_add(ex.v, tv), lane);
    const uint32_t en = sat_add(ex.n, in_ - n), ek = sat_add(ex.k, ik == 0xffffffffu ? ik : ik - K),
                   ev = sat_add(ex.v, iv - V);
    // per-block outputs (the lane that owns the block)
    bool ok = (uint64_t)en + n <= p.ent_cap && (uint64_t)en + n <= 0xffffffffull;
    if (mat) {
      const uint64_t kend = (uint64_t)ek + K, vend = (uint64_t)ev + V;
      ok = ok && (kend <= p.key_cap || !p.key_data) && (vend <= p.val_cap || !p.val_data);
      ok = ok && kend < 0xffffffffull && vend <= 0xffffffffull;
    }
    if (own) {
      const uint32_t st = sw & ~kPlen;
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
      if (!ok) atomicOr(reinterpret_cast<unsigned long long*>(p.result + 5), 1ull);
    }
    // every record (LDS, and the global spill) written before other lanes read it
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
    // ---- 4: copy, block by block, the whole wave on each ----
    for (uint32_t gg = 0; gg < TB; gg++) {
      const uint32_t s = gg * L;
      const uint32_t bb = t * TB + gg;
      if (bb >= p.nblk) break;
      const uint32_t nb = __builtin_amdgcn_readlane(n, s);
      if (nb == 0 || !__builtin_amdgcn_readlane((uint32_t)ok, s) || (p.ablate & 2)) continue;
      const uint32_t swb = __builtin_amdgcn_readlane(sw, s);
      const uint64_t enb = __builtin_amdgcn_readlane(en, s), ekb = __builtin_amdgcn_readlane(ek, s),
                     evb = __builtin_amdgcn_readlane(ev, s);
      const uint32_t offb = __builtin_amdgcn_readlane(off, s);
      const Recs<R> rec{recs + gg * R, p.wmeta + (uint64_t)bb * p.wcap};
      const uint8_t* bp = p.data + offb;
      uint8_t* kbase = mat && p.key_data ? p.key_data + ekb : nullptr;
      uint8_t* vbase = mat && p.val_data ? p.val_data + evb : nullptr;
      if (swb & kPlen) {
        copy_plen(p, rec, bp, kbase, vbase, nb, enb, ekb, evb, offb, mat, view, lane);
        continue;
      }
      entry_outputs(p, rec, nb, enb, ekb, evb, offb, mat, view, lane);
      if (!mat) continue;
      const uint32_t Kb = __builtin_amdgcn_readlane(K, s), Vb = __builtin_amdgcn_readlane(V, s);
      if (p.wbatch) {
        if ((Kb + Vb) / nb > 128)
          copy_bytes_batched<16, 4>(rec, bp, kbase, vbase, nb, lane);
        else
          copy_bytes_batched<8, 8>(rec, bp, kbase, vbase, nb, lane);
      } else if ((Kb + Vb) / nb > 128) {
        copy_bytes<16, 2>(rec, bp, kbase, vbase, nb, lane);
      } else {
        copy_bytes<8, 5>(rec, bp, kbase, vbase, nb, lane);
      }
    }
    wave_lds_fence();  // the next tile's walk overwrites the records
  }
}

hipError_t launch_decode_onepass(const DecodeParams& p, uint32_t max_blk_len, int num_cus,
                                 hipStream_t s) {
  const int wpc_env = getenv("LSMGPU_ONEPASS_WPC") ? atoi(getenv("LSMGPU_ONEPASS_WPC")) : 0;
  const uint32_t wpc = wpc_env > 0 && wpc_env <= 32 ? (uint32_t)wpc_env : 12u;  // workers per CU
  uint32_t tb = max_blk_len <= 4096 ? 16u : max_blk_len <= 16384 ? 8u : 4u;
  const int tb_env = getenv("LSMGPU_ONEPASS_TB") ? atoi(getenv("LSMGPU_ONEPASS_TB")) : 0;
  if (tb_env == 4 || tb_env == 8 || tb_env == 16) tb = (uint32_t)tb_env;
  const uint32_t ntiles = (p.nblk + tb - 1) / tb;
  const uint32_t grid = std::min<uint32_t>(ntiles, wpc * (uint32_t)num_cus);
  if (tb == 16)
    hipLaunchKernelGGL((onepass_kernel<16, 4, 64>), dim3(grid), dim3(64), 0, s, p);
  else if (tb == 8)
    hipLaunchKernelGGL((onepass_kernel<8, 8, 128>), dim3(grid), dim3(64), 0, s, p);
  else
    hipLaunchKernelGGL((onepass_kernel<4, 16, 256>), dim3(grid), dim3(64), 0, s, p);
  return hipGetLastError();
}

}  // namespace lsmgpu
