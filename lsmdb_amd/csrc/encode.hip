// encode.hip -- gfx950 SST block encode: the device restatement of Builder.Add/addHelper/
// finishBlock/blockIndex (table/builder.go:84-160) for a sorted batch of entries.
//
// Every output position is closed-form, so the encoder needs no scan and no staging:
//   entry e of block b starts at  10*e + key_start(e) + vs_start(e) + 13*b
// (each earlier entry contributes its 10-B header, its full key -- keyDiff always returns the
// whole key, builder.go:74-82 -- and its ValueStruct bytes; each earlier block its 13-B
// terminator, builder.go:121-123).  One wave per block; groups of J lanes take one entry each:
// lane 0 of the group writes the synthesised header (with the key's first 6 bytes, one 16-B
// store), and the J lanes copy the key and the vs-enc bytes global -> global as unaligned 16-B
// pieces (the last piece overlapping back inside its stream, two overlapping 8/4-B pieces or
// single bytes below 16 B), so no store crosses into a neighbour's bytes.  J follows the
// average entry size.  The product kernel is encode_pipe_kernel (each lane's first piece of the
// next entry pass loaded before this pass's stores); encode_kernel, the unpipelined order with
// G groups per trip, is kept for the diagnostic build's A/Bs.
#include <cstdlib>

#include "codec_common.hpp"
#include "decode_common.hpp"
#include "kernels.hpp"

namespace lsmgpu {

__device__ __forceinline__ uint64_t key_start(const EncodeParams& p, uint64_t e) {
  return e ? p.key_end[e - 1] : 0;
}
__device__ __forceinline__ uint64_t vs_start(const EncodeParams& p, uint64_t e) {
  return e ? p.vs_end[e - 1] : 0;
}
__device__ __forceinline__ void block_range(const EncodeParams& p, uint32_t b, uint64_t& f,
                                            uint64_t& l) {
  if (p.blk_first) {
    f = p.blk_first[b];
    l = p.blk_first[b + 1];
  } else {
    f = (uint64_t)b * p.epb;
    l = f + p.epb;
    if (l > p.n) l = p.n;
    if (f > p.n) f = p.n;
  }
}

// big-endian stores at any alignment
__device__ __forceinline__ void store_be32(uint8_t* d, uint32_t v) {
  const uint32_t be = __builtin_bswap32(v);
  __builtin_memcpy(d, &be, 4);
}
// header{plen = 0, klen, vlen, prev} (builder.go:23-45): 10 bytes as one 8-B + one 2-B store
__device__ __forceinline__ void store_header(uint8_t* d, uint32_t klen, uint32_t vlen,
                                             uint32_t prev) {
  uint2 w;
  w.x = (bswap16(klen) << 16);                    // plen 00 00 | klen BE
  w.y = bswap16(vlen) | (bswap16(prev >> 16) << 16);  // vlen BE | prev[31:16] BE
  __builtin_memcpy(d, &w, 8);
  const uint16_t lo = (uint16_t)bswap16(prev & 0xffffu);
  __builtin_memcpy(d + 8, &lo, 2);
}

// One output block's table context: its entries [f, l), the output image, the image's data
// length and block count, and the entry / key / vs bases positions are relative to (one table,
// or table t of a compaction's output in tbl_* mode).  False: past the last block, or a block of
// no entries (its terminator written here).
struct EncBlock {
  uint64_t f, l, e0b, kb0, vb0, dl;
  uint32_t lb, tnb;
  uint8_t* out;
  // entry e's position in its table: 10 (e - e0b) + key bytes + vs bytes before it + 13 per block
  __device__ __forceinline__ uint32_t position(uint64_t e, uint64_t ks, uint64_t vs0) const {
    return (uint32_t)(10 * (e - e0b) + (ks - kb0) + (vs0 - vb0)) + 13u * lb;
  }
};

__device__ __forceinline__ bool enc_block(const EncodeParams& p, uint32_t b, uint32_t lane,
                                          EncBlock& k) {
  uint64_t f, l, e0b = 0, kb0 = 0, vb0 = 0, dl = p.data_len;
  uint32_t lb = b, tnb = p.nblocks;
  uint8_t* out = p.out;
  if (p.tbl_first) {
    if (b >= p.tbl_blk[p.ntables]) return false;
    uint32_t lo = 0, hi = p.ntables - 1;  // table of block b: largest t with tbl_blk[t] <= b
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (p.tbl_blk[mid] <= b) lo = mid; else hi = mid - 1;
    }
    const uint32_t t = uniform(lo);
    lb = b - p.tbl_blk[t];
    tnb = p.tbl_blk[t + 1] - p.tbl_blk[t];
    e0b = p.tbl_first[t];
    const uint64_t ee = p.tbl_first[t + 1];
    f = e0b + (uint64_t)lb * p.epb;
    l = f + p.epb < ee ? f + p.epb : ee;
    kb0 = key_start(p, e0b);
    vb0 = vs_start(p, e0b);
    out = p.out + p.tbl_out[t];
    dl = 10 * (ee - e0b) + (key_start(p, ee) - kb0) + (vs_start(p, ee) - vb0) + 13ull * tnb;
  } else {
    if (b >= p.nblocks) return false;
    block_range(p, b, f, l);
  }
  k.f = uniform64(f);
  k.l = uniform64(l);
  k.e0b = uniform64(e0b);
  k.kb0 = uniform64(kb0);
  k.vb0 = uniform64(vb0);
  k.dl = uniform64(dl);
  k.lb = lb;
  k.tnb = tnb;
  k.out = out;
  if (k.l == k.f) {  // a block of no entries: the terminator alone (table_test.go:514)
    if (lane == 0) {
      const uint32_t bs = k.position(k.f, key_start(p, k.f), vs_start(p, k.f));
      uint8_t* t = out + bs;
      store_header(t, 0, 3, 0xffffffffu);
      t[10] = 0;
      t[11] = 0;
      t[12] = 0;
      store_be32(out + k.dl + 4ull * lb, bs + 13);
    }
    if (lane == 1 && lb == tnb - 1) store_be32(out + k.dl + 4ull * tnb, tnb);
    return false;
  }
  if (lane == 1 && lb == tnb - 1) store_be32(out + k.dl + 4ull * tnb, tnb);
  return true;
}

template <uint32_t J, uint32_t G>
__global__ void __launch_bounds__(256) encode_kernel(EncodeParams p) {
  constexpr uint32_t EPP = kWave / J;      // entries per group pass; G group passes per loop
                                           // trip, every offset load issued first
  const uint32_t lane = lane_id();
  const uint32_t b = uniform(blockIdx.x * 4 + (threadIdx.x >> 6));
  EncBlock k;
  if (!enc_block(p, b, lane, k)) return;
  const uint64_t f = k.f, m = k.l - k.f, dl = k.dl;
  const uint32_t lb = k.lb;
  uint8_t* const out = k.out;
  auto position = [&](uint64_t e, uint64_t ks, uint64_t vs0) { return k.position(e, ks, vs0); };

  // Absolute entry positions are closed-form (no block base needed to place bytes); the block
  // start is entry f's position (lane 0, first pass), a header's prev is the previous entry's
  // position (the neighbouring lane group, or the previous pass), and the lane group holding
  // the block's last entry writes the terminator and the restart.
  const uint32_t j = lane & (J - 1);
  uint32_t bad = 0, bs = 0, carry = 0;
  // the starts of the block's first 64 entries, one per lane (key_end / vs_end of entry
  // f + lane - 1), in one round trip: passes over entries < 63 take offsets by lane shuffle
  const uint64_t pidx = f + lane;
  const uint64_t pc = pidx - 1 < p.n - 1 ? pidx - 1 : p.n - 1;
  const uint32_t pk = pidx ? p.key_end[pc] : 0u, pv = pidx ? p.vs_end[pc] : 0u;
  // gather mode: the source starts of the same entries (entry f + lane)
  uint32_t psk = 0, psv = 0;
  if (p.src) {
    const uint32_t si = p.src[pidx < p.n ? pidx : p.n - 1];
    psk = si ? p.src_key_end[si - 1] : 0u;
    psv = si ? p.src_vs_end[si - 1] : 0u;
  }
  for (uint64_t e0 = 0; e0 < m; e0 += (uint64_t)G * EPP) {
    uint32_t klen[G], vlen[G], pos[G], np[G], kp[G];
    uint64_t ks[G], vs0[G], sk[G], sv[G];  // sk / sv: where the bytes are read (gather mode)
    bool on[G];
    const bool shuffled = e0 + (uint64_t)G * EPP < kWave;
#pragma unroll
    for (uint32_t i = 0; i < G; i++) {
      const uint64_t r = e0 + i * EPP + lane / J;  // entry index inside the block
      on[i] = r < m;
      const uint64_t e = f + (on[i] ? r : m - 1);
      uint64_t ke, ve;
      if (shuffled) {
        const int rr = (int)(on[i] ? r : m - 1);
        ks[i] = (uint32_t)__shfl((int)pk, rr);
        ke = (uint32_t)__shfl((int)pk, rr + 1);
        vs0[i] = (uint32_t)__shfl((int)pv, rr);
        ve = (uint32_t)__shfl((int)pv, rr + 1);
        sk[i] = (uint32_t)__shfl((int)psk, rr);
        sv[i] = (uint32_t)__shfl((int)psv, rr);
      } else {
        ks[i] = key_start(p, e);
        vs0[i] = vs_start(p, e);
        ke = p.key_end[e];
        ve = p.vs_end[e];
        if (p.src) {
          const uint32_t si = p.src[e];
          sk[i] = si ? p.src_key_end[si - 1] : 0u;
          sv[i] = si ? p.src_vs_end[si - 1] : 0u;
        }
      }
      if (!p.src) {
        sk[i] = ks[i];
        sv[i] = vs0[i];
      }
      const uint64_t kl64 = ke - ks[i], vl64 = ve - vs0[i];
      klen[i] = (uint32_t)kl64;
      vlen[i] = (uint32_t)vl64;
      pos[i] = position(e, ks[i], vs0[i]);
      if (on[i] && j == 0) {
        if (kl64 <= 8 || kl64 > 0xffff) bad |= 1;  // ParseKey needs len(key) > 8 (y.go:93-100)
        if (vl64 > 0xffff) bad |= 2;                // header vlen is a uint16
      }
      kp[i] = pieces16(klen[i]);
      np[i] = on[i] ? kp[i] + pieces16(vlen[i]) : 0u;
    }
    if (e0 == 0) bs = readlane(pos[0], 0);
#pragma unroll
    for (uint32_t i = 0; i < G; i++) {
      // previous entry's position: the lane group below, else the previous group / pass
      const uint32_t below = __shfl_up(pos[i], J);
      const uint32_t edge = i == 0 ? carry : readlane(pos[i - 1], kWave - J);
      const uint64_t r = e0 + i * EPP + lane / J;
      const uint32_t prev = r == 0 ? 0xffffffffu : (lane < J ? edge : below) - bs;  // builder.go:95-99
      if (on[i] && j == 0) {
        if (LSMGPU_KNOB(p.hdr16, 1u) && klen[i] >= 8) {  // (8-B key read inside the key)
          // the header and the key's first 6 bytes as one 16-B store (the key's first piece
          // rewrites those 6 bytes with the same values): one store instruction per pass instead
          // of an 8-B and a 2-B one
          uint2 k8;
          __builtin_memcpy(&k8, p.keys + sk[i], 8);
          uint4 w;
          w.x = bswap16(klen[i]) << 16;                               // plen 00 00 | klen BE
          w.y = bswap16(vlen[i]) | (bswap16(prev >> 16) << 16);       // vlen BE | prev[31:16] BE
          w.z = bswap16(prev & 0xffffu) | (k8.x << 16);               // prev[15:0] BE | key[0..1]
          w.w = (k8.x >> 16) | (k8.y << 16);                          // key[2..5]
          __builtin_memcpy(out + pos[i], &w, 16);
        } else {
          store_header(out + pos[i], klen[i], vlen[i], prev);
        }
      }
      if (on[i] && j == 1 && r == m - 1) {  // terminator + restart (builder.go:121-123,146-160)
        const uint32_t te = pos[i] + 10 + klen[i] + vlen[i];
        uint8_t* t = out + te;
        store_header(t, 0, 3, pos[i] - bs);
        t[10] = 0;
        t[11] = 0;
        t[12] = 0;
        store_be32(out + dl + 4ull * lb, te + 13);
      }
    }
    carry = readlane(pos[G - 1], kWave - J);
#pragma unroll
    for (uint32_t i = 0; i < G; i++) {
      for (uint32_t q = j; q < np[i]; q += J) {  // one (non-divergent) copy per piece
        const bool key = q < kp[i];
        copy_piece16(out + pos[i] + 10 + (key ? 0u : klen[i]), key ? p.keys + sk[i] : p.vs + sv[i],
                  key ? klen[i] : vlen[i], key ? q : q - kp[i]);
      }
    }
  }
  if (bad) atomicOr(p.flags, bad);
}

// encode_pipe_kernel<J, U2> (the product encoder): encode_kernel<J, 1> with each lane's first
// 16-B piece of the next entry pass loaded before this pass's stores.  The compiled
// encode_kernel issues every piece as load -> s_waitcnt vmcnt(0) -> store, and the header's 8-B
// key read the same way; on gfx950 vmcnt counts stores as well as loads, so each wait also drains
// the pass's earlier stores, and a pass costs load and store round trips back to back.  Here:
//  * the header's key bytes come from the lane's own first piece (key piece 0 whenever the key
//    is >= 16 B): no separate read;
//  * the wait for pass i + 1's pieces leaves pass i's stores in flight.  For the compiler to
//    count those stores they must not sit in a branch: the header and first-piece stores are
//    buffer stores every lane issues, a lane with nothing to write giving an offset past the
//    image (the range check drops it).  The offsets come from a window of 64 entries held one
//    per lane, loaded (and waited for) once per 64 entries, so no other wait stays in the loop;
//  * U2: two passes per loop trip, each loading into the other's registers (no register copy,
//    and so no wait, at the back edge), the first pass peeled so that the loop is entered as it
//    loops.
// Pieces past a lane's first (entries of more than J pieces) and streams under 16 B keep the
// plain load -> store order.  Same bytes as encode_kernel.
struct EncPass {
  uint64_t sk, sv;              // where the key / vs bytes are read
  uint32_t klen, vlen, pos, kp, np, r;
  bool on;
};

template <uint32_t J, bool U2>
__global__ void __launch_bounds__(256) encode_pipe_kernel(EncodeParams p) {
  constexpr uint32_t EPP = kWave / J;
  const uint32_t lane = lane_id();
  const uint32_t b = uniform(blockIdx.x * 4 + (threadIdx.x >> 6));
  EncBlock k;
  if (!enc_block(p, b, lane, k)) return;
  const uint64_t f = k.f, m = k.l - k.f, dl = k.dl;
  const uint32_t lb = k.lb;
  uint8_t* const out = k.out;
  const uint32_t j = lane & (J - 1);
  uint32_t bad = 0, carry = 0, bs = 0;
  // offsets of a window of 64 entries [w0, w0 + 64) of the block, one entry per lane: its key /
  // vs start and end, and in gather mode the source starts.  A pass (EPP | 64 entries) lies in
  // one window; off lanes (past the block's end) read garbage that nothing uses.
  uint32_t wks, wke, wvs, wve, wsk = 0, wsv = 0;
  uint64_t w0 = 0;
  auto window = [&](uint64_t b0) {
    w0 = b0;
    const uint64_t r = b0 + lane, e = f + (r < m ? r : m - 1);
    wks = (uint32_t)key_start(p, e);
    wvs = (uint32_t)vs_start(p, e);
    wke = p.key_end[e];
    wve = p.vs_end[e];
    if (p.src) {
      const uint32_t si = p.src[e];
      wsk = si ? p.src_key_end[si - 1] : 0u;
      wsv = si ? p.src_vs_end[si - 1] : 0u;
    }
    // the window lands here, so no wait for it stays inside the passes (vmcnt counts stores too:
    // such a wait would drain the previous pass's stores on every trip)
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
  };
  // the pass over entries [e0, e0 + EPP): offsets by lane shuffle from the window, lengths,
  // positions, piece counts
  auto meta = [&](uint64_t e0, EncPass& s) {
    const uint64_t r = e0 + lane / J;
    s.r = (uint32_t)r;
    s.on = r < m;
    const uint64_t e = f + (s.on ? r : m - 1);
    const int i = (int)((r - w0) & (kWave - 1));
    const uint64_t ks = (uint32_t)__shfl((int)wks, i), ke = (uint32_t)__shfl((int)wke, i);
    const uint64_t vs0 = (uint32_t)__shfl((int)wvs, i), ve = (uint32_t)__shfl((int)wve, i);
    if (p.src) {
      s.sk = (uint32_t)__shfl((int)wsk, i);
      s.sv = (uint32_t)__shfl((int)wsv, i);
    } else {
      s.sk = ks;
      s.sv = vs0;
    }
    const uint64_t kl64 = ke - ks, vl64 = ve - vs0;
    s.klen = (uint32_t)kl64;
    s.vlen = (uint32_t)vl64;
    s.pos = k.position(e, ks, vs0);
    if (s.on && j == 0) {
      if (kl64 <= 8 || kl64 > 0xffff) bad |= 1;  // ParseKey needs len(key) > 8 (y.go:93-100)
      if (vl64 > 0xffff) bad |= 2;                // header vlen is a uint16
    }
    s.kp = pieces16(s.klen);
    s.np = s.on ? s.kp + pieces16(s.vlen) : 0u;
  };
  // the lane's first piece (q = j) when its stream is >= 16 B: source and destination offsets
  auto first = [&](const EncPass& s, const uint8_t*& src, uint32_t& dst) -> bool {
    if (j >= s.np) return false;
    const bool key = j < s.kp;
    const uint32_t len = key ? s.klen : s.vlen;
    if (len < 16) return false;
    const uint32_t o = min(16 * (key ? j : j - s.kp), len - 16);
    src = (key ? p.keys + s.sk : p.vs + s.sv) + o;
    dst = s.pos + 10 + (key ? 0u : s.klen) + o;
    return true;
  };

  // The header and first-piece stores go out as buffer stores over the table image, issued by
  // every lane (a lane with nothing to write gives an offset past the image's end, and the
  // hardware's range check drops it): with no branch around them the compiler counts them, so the
  // wait for the next pass's first pieces leaves them in flight (a store in a branch counts as
  // possibly absent, and the wait then drains it).  Offsets are 32-bit: an image is < 4 GiB.
  const __amdgpu_buffer_rsrc_t orsrc = buffer_rsrc(out, dl);
  auto put16 = [&](const u32x4& v, uint32_t o) {
    __builtin_amdgcn_raw_buffer_store_b128(v, orsrc, o, 0, 0);
  };
  // one pass: the next pass's offsets and first pieces into (nx, nv, n16, nd) -- loaded before
  // any store of this one, unconditionally (from p.pad when the lane has no such piece) -- then
  // this pass's header, terminator and pieces from (cu, av, a16, ad)
  auto step = [&](const EncPass& cu, const uint4& av, bool a16, uint32_t ad, uint64_t e0,
                  EncPass& nx, uint4& nv, bool& n16, uint32_t& nd) {
    if (((e0 + EPP) & (kWave - 1)) == 0 && e0 + EPP < m) window(e0 + EPP);  // (uniform)
    meta(e0 + EPP, nx);  // past the block's end: every entry off, no pieces
    const uint8_t* nsrc = p.pad;
    n16 = first(nx, nsrc, nd);
    __builtin_memcpy(&nv, nsrc, 16);
    // headers (prev = the lane group below, else the previous pass)
    const uint32_t below = __shfl_up(cu.pos, J);
    const uint32_t prev = cu.r == 0 ? 0xffffffffu : (lane < J ? carry : below) - bs;  // builder.go:95-99
    // header + the key's first 6 bytes as one 16-B store, the key bytes from this lane's first
    // piece (key piece 0: the key is >= 16 B); shorter keys: 8-B + 2-B header stores
    const u32x4 w = {bswap16(cu.klen) << 16,                                // plen 00 00 | klen BE
                     bswap16(cu.vlen) | (bswap16(prev >> 16) << 16),       // vlen BE | prev[31:16] BE
                     bswap16(prev & 0xffffu) | (av.x << 16),               // prev[15:0] BE | key[0..1]
                     (av.x >> 16) | (av.y << 16)};                         // key[2..5]
    const bool hdr = cu.on && j == 0;
    put16(w, hdr && a16 ? cu.pos : kNoStore);
    if (hdr && !a16) store_header(out + cu.pos, cu.klen, cu.vlen, prev);
    if (cu.on && j == 1 && cu.r == m - 1) {  // terminator + restart (builder.go:121-123,146-160)
      const uint32_t te = cu.pos + 10 + cu.klen + cu.vlen;
      uint8_t* t = out + te;
      store_header(t, 0, 3, cu.pos - bs);
      t[10] = 0;
      t[11] = 0;
      t[12] = 0;
      store_be32(out + dl + 4ull * lb, te + 13);
    }
    carry = readlane(cu.pos, kWave - J);
    // pieces: the preloaded first one, then the rest in load -> store order
    put16(u32x4{av.x, av.y, av.z, av.w}, a16 ? ad : kNoStore);
    for (uint32_t q = a16 ? j + J : j; q < cu.np; q += J) {
      const bool key = q < cu.kp;
      copy_piece16(out + cu.pos + 10 + (key ? 0u : cu.klen), key ? p.keys + cu.sk : p.vs + cu.sv,
                   key ? cu.klen : cu.vlen, key ? q : q - cu.kp);
    }
  };
  EncPass pa, pb;
  uint4 va, vb;
  bool fa, fb;
  uint32_t da = 0, db = 0;
  window(0);
  meta(0, pa);
  bs = readlane(pa.pos, 0);
  const uint8_t* src0 = p.pad;
  fa = first(pa, src0, da);
  __builtin_memcpy(&va, src0, 16);
  if (U2) {
    // two passes per trip, each loading into the other's registers: no register copy (and so no
    // wait for the loads in flight) at the loop's back edge
    // (the first pass peeled: the loop is then entered, as it loops, with the previous pass's two
    // buffer stores issued after the pending pieces, so one wait count serves both entries)
    step(pa, va, fa, da, 0, pb, vb, fb, db);
    for (uint64_t e0 = EPP; e0 < m; e0 += 2 * EPP) {
      step(pb, vb, fb, db, e0, pa, va, fa, da);
      if (e0 + EPP >= m) break;
      step(pa, va, fa, da, e0 + EPP, pb, vb, fb, db);
    }
  } else {
    for (uint64_t e0 = 0; e0 < m; e0 += EPP) {
      step(pa, va, fa, da, e0, pb, vb, fb, db);
      pa = pb;
      va = vb;
      fa = fb;
      da = db;
    }
  }
  if (bad) atomicOr(p.flags, bad);
}

// encode_dense_kernel (blocks of large entries, > 128 B on average: C5's Zipf keys, C3): the
// block's output as one run of 16-B pieces spread densely over the wave, as the copy's
// copy_entries_dense_pipe does for the decode.  Entries 64 at a time, one per lane: offsets,
// position, header fields; each entry counts its pieces -- the header piece (header + the key's
// first 6 bytes, as encode_pipe_kernel writes it) when the key is >= 16 B, its key and value
// pieces (16 B, the last overlapping back) -- and a wave scan gives each its first.  Then every
// lane takes one piece of each 64-piece window: its entry found by LDS marks + a max-scan, the
// next window's piece loaded before this window's store, every store a range-checked buffer
// store over the table image.  Streams under 16 B (keys of 9-15 B and their headers, value
// pointers' 15-B values) are written by the entry's lane in the plain order before the windows.
__global__ void __launch_bounds__(256) encode_dense_kernel(EncodeParams p) {
  __shared__ uint8_t s_mk[4][kWave];
  const uint32_t lane = lane_id();
  const uint32_t b = uniform(blockIdx.x * 4 + (threadIdx.x >> 6));
  uint8_t* const mk = s_mk[threadIdx.x >> 6];
  EncBlock k;
  if (!enc_block(p, b, lane, k)) return;
  const uint64_t f = k.f, m = k.l - k.f, dl = k.dl;
  const uint32_t lb = k.lb;
  uint8_t* const out = k.out;
  const __amdgpu_buffer_rsrc_t orsrc = buffer_rsrc(out, dl);
  uint32_t bad = 0, bs = 0, carry = 0, tpos = 0, tend = 0;
  struct Pc {
    const uint8_t* src;
    uint32_t dst;                  // kNoStore: none
    uint32_t hdr, hprev;           // header piece: klen | vlen << 16, prev
  };
  for (uint64_t c0 = 0; c0 < m; c0 += kWave) {
    const uint64_t r = c0 + lane;
    const bool on = r < m;
    const uint64_t e = f + (on ? r : m - 1);
    const uint64_t ks = key_start(p, e), vs0 = vs_start(p, e), ke = p.key_end[e], ve = p.vs_end[e];
    uint64_t sk = ks, sv = vs0;
    if (p.src) {
      const uint32_t si = p.src[e];
      sk = si ? p.src_key_end[si - 1] : 0u;
      sv = si ? p.src_vs_end[si - 1] : 0u;
    }
    const uint32_t klen = (uint32_t)(ke - ks), vlen = (uint32_t)(ve - vs0);
    const uint32_t pos = k.position(e, ks, vs0);
    if (c0 == 0) bs = readlane(pos, 0);
    const uint32_t below = (uint32_t)__shfl_up((int)pos, 1u);
    const uint32_t prev = r == 0 ? 0xffffffffu : (lane == 0 ? carry : below) - bs;  // builder.go:95-99
    carry = readlane(pos, kWave - 1);
    if (on) {
      if (ke - ks <= 8 || ke - ks > 0xffff) bad |= 1;  // ParseKey needs len(key) > 8 (y.go:93-100)
      if (ve - vs0 > 0xffff) bad |= 2;                  // header vlen is a uint16
      if (r == m - 1) {
        tpos = pos;
        tend = pos + 10 + klen + vlen;
      }
      // short streams, plain: the header (8 + 2 B) and the key's pieces of a key under 16 B, the
      // pieces of a value under 16 B
      if (klen < 16) {
        store_header(out + pos, klen, vlen, prev);
        for (uint32_t q = 0; q < pieces16(klen); q++) copy_piece16(out + pos + 10, p.keys + sk, klen, q);
      }
      if (vlen < 16)
        for (uint32_t q = 0; q < pieces16(vlen); q++) copy_piece16(out + pos + 10 + klen, p.vs + sv, vlen, q);
    }
    const uint32_t hp = on && klen >= 16 ? 1u : 0u, kp = on && klen >= 16 ? pieces16(klen) : 0u;
    const uint32_t pc = hp + kp + (on && vlen >= 16 ? pieces16(vlen) : 0u);
    const uint32_t ps = wave_scan_sat(pc, lane), ex = ps - pc;
    const uint32_t T = __builtin_amdgcn_readlane(ps, 63);
    uint32_t wcarry = 0;
    auto win = [&](uint32_t r0) -> Pc {
      mk[lane] = 0;
      wave_lds_fence();
      if (pc > 0 && ex >= r0 && ex < r0 + kWave) mk[ex - r0] = (uint8_t)(lane + 1);
      wave_lds_fence();
      const uint32_t own = max(wave_scan_max(mk[lane], lane), wcarry);  // 1 + the owner lane
      wcarry = __builtin_amdgcn_readlane(own, 63);
      wave_lds_fence();
      const int L = (int)own - 1;
      const uint32_t kv = (uint32_t)__shfl((int)(klen | (vlen << 16)), L);
      const uint32_t posL = (uint32_t)__shfl((int)pos, L), prevL = (uint32_t)__shfl((int)prev, L);
      const uint32_t exL = (uint32_t)__shfl((int)ex, L), hkL = (uint32_t)__shfl((int)(hp | (kp << 8)), L);
      const uint64_t skL = (uint32_t)__shfl((int)sk, L), svL = (uint32_t)__shfl((int)sv, L);
      const uint32_t kL = kv & 0xffffu, vL = kv >> 16, hL = hkL & 0xffu, kpL = hkL >> 8;
      Pc c{p.pad, kNoStore, 0u, 0u};
      const uint32_t P = r0 + lane;
      if (P < T) {
        const uint32_t q = P - exL;
        if (q < hL) {  // the header piece: the key's first 16 B
          c = Pc{p.keys + skL, posL, kv, prevL};
        } else if (q < hL + kpL) {
          const uint32_t o = min(16 * (q - hL), kL - 16);
          c = Pc{p.keys + skL + o, posL + 10 + o, 0u, 0u};
        } else {
          const uint32_t o = min(16 * (q - hL - kpL), vL - 16);
          c = Pc{p.vs + svL + o, posL + 10 + kL + o, 0u, 0u};
        }
      }
      return c;
    };
    auto load = [&](const Pc& c) -> uint4 {
      uint4 v;
      __builtin_memcpy(&v, c.src, 16);
      return v;
    };
    auto store = [&](const Pc& c, const uint4& v) {
      const uint32_t kl = c.hdr & 0xffffu, vl = c.hdr >> 16, pr = c.hprev;
      const u32x4 h = {bswap16(kl) << 16,                               // plen 00 00 | klen BE
                       bswap16(vl) | (bswap16(pr >> 16) << 16),          // vlen BE | prev[31:16] BE
                       bswap16(pr & 0xffffu) | (v.x << 16),              // prev[15:0] BE | key[0..1]
                       (v.x >> 16) | (v.y << 16)};                       // key[2..5]
      const u32x4 w = {v.x, v.y, v.z, v.w};
      __builtin_amdgcn_raw_buffer_store_b128(c.hdr ? h : w, orsrc, c.dst, 0, 0);
    };
    Pc ca = win(0);
    uint4 va = load(ca);
    for (uint32_t r0 = 0; r0 < T; r0 += 2 * kWave) {  // two windows per trip: no register copy
      const Pc cb = win(r0 + kWave);
      const uint4 vb = load(cb);
      store(ca, va);
      if (r0 + kWave >= T) break;
      ca = win(r0 + 2 * kWave);
      va = load(ca);
      store(cb, vb);
    }
  }
  // terminator + restart (builder.go:121-123,146-160), by the lane of the block's last entry
  if (lane == (uint32_t)((m - 1) & (kWave - 1))) {
    uint8_t* t = out + tend;
    store_header(t, 0, 3, tpos - bs);
    t[10] = 0;
    t[11] = 0;
    t[12] = 0;
    store_be32(out + dl + 4ull * lb, tend + 13);
  }
  if (bad) atomicOr(p.flags, bad);
}

// Builder.ReachedCapacity (builder.go:140-143) as compactBuildTables applies it before every
// Add (levels.go:265-271): a table holding e entries [s, s + e) is closed when
//   10e + K + V + 13 fb + 8 + 4 fb + 8 > cap,   fb = (e - 1) / epb finished blocks
// (buf.Len() = every entry + each finished block's 13-B terminator; len(restarts) = fb), K, V
// the key / vs bytes of those entries.  The predicate grows with e, so each cut is a search:
// one wave, 64 candidate counts per round trip.  A table ends at the first e >= 1 where it
// holds, or takes every remaining entry.  Image size = data + 4 (blocks) + 4 (block count).
// Finish's bloom tail for a table of cnt keys: JSONMarshal of bbloom.New(cnt, 0.01) + its BE32
// length.  The float64 sizing follows Go's operation order (-1 * n * ln(w) / ln2^2, then
// ceil(ln2 * size / n)) with the host's constants, so it rounds exactly like the host.
__device__ __forceinline__ uint64_t bloom_tail_bytes(const CutParams& p, uint64_t cnt) {
  const double n = (double)cnt;
  const double size = -1 * n * p.logw / p.ln2sq;
  const double locs = ceil(p.ln2 * size / n);
  uint64_t entries = (uint64_t)size, bits = 1;
  if (entries < 512) entries = 512;
  while (bits < entries) bits <<= 1;
  uint64_t l = (uint64_t)locs, digits = 1;
  while (l >= 10) {
    l /= 10;
    digits++;
  }
  // {"FilterSet":"  base64   ","SetLocs":  digits  }   BE32
  return 14 + 4 * ((bits / 8 + 2) / 3) + 12 + digits + 1 + 4;
}

__global__ void cut_tables_kernel(CutParams p) {
  const uint32_t lane = lane_id();
  uint64_t s = 0, blocks = 0, bytes = 0;
  uint32_t t = 0;
  auto kstart = [&](uint64_t e) -> uint64_t { return e ? p.key_end[e - 1] : 0; };
  auto vstart = [&](uint64_t e) -> uint64_t { return e ? p.vs_end[e - 1] : 0; };
  while (s < p.n) {
    if (t >= p.tables_cap) {
      if (lane == 0) p.result[3] = 1;
      break;
    }
    const uint64_t ks = kstart(s), vs = vstart(s), rest = p.n - s;
    // first e in [1, rest - 1] with the predicate, or `rest` (all of them)
    uint64_t lo = 1, hi = rest;
    while (lo < hi) {
      const uint64_t step = (hi - lo + 62) / 63;  // lane 63 reaches hi: the ballot is never empty
      const uint64_t e = lo + lane * step < hi ? lo + lane * step : hi;
      bool over = true;  // e == hi: the sentinel
      if (e < hi) {
        const uint64_t fb = (e - 1) / p.epb;
        const int64_t est = (int64_t)(10 * e + (kstart(s + e) - ks) + (vstart(s + e) - vs) +
                                      13 * fb + 8 + 4 * fb + 8);
        over = est > p.cap;
      }
      const uint64_t mask = __ballot(over);
      const uint32_t first = (uint32_t)__builtin_ctzll(mask);  // lane 63 or the clamp is true
      const uint64_t ef = lo + (uint64_t)first * step < hi ? lo + (uint64_t)first * step : hi;
      lo = first ? lo + (uint64_t)(first - 1) * step + 1 : lo;
      hi = ef;
    }
    const uint64_t cnt = lo;
    const uint64_t nb = (cnt + p.epb - 1) / p.epb;
    if (lane == 0) {
      p.tbl_first[t] = (uint32_t)s;
      p.tbl_blk[t] = (uint32_t)blocks;
      p.tbl_out[t] = bytes;
    }
    bytes += 10 * cnt + (kstart(s + cnt) - ks) + (vstart(s + cnt) - vs) + 13 * nb + 4 * nb + 4;
    if (p.bloom) bytes += bloom_tail_bytes(p, cnt);
    blocks += nb;
    s += cnt;
    t++;
  }
  for (uint32_t k = t + lane; k <= p.tables_cap; k += kWave) {  // close through tables_cap
    p.tbl_first[k] = (uint32_t)s;
    p.tbl_blk[k] = (uint32_t)blocks;
    p.tbl_out[k] = bytes;
  }
  if (lane == 0) {
    p.result[0] = t;
    p.result[1] = blocks;
    p.result[2] = bytes;
  }
}

hipError_t launch_cut_tables(const CutParams& p, hipStream_t s) {
  hipLaunchKernelGGL(cut_tables_kernel, dim3(1), dim3(64), 0, s, p);
  return hipGetLastError();
}

template <uint32_t J, uint32_t G>
static hipError_t launch_enc(const EncodeParams& p, hipStream_t s) {
  // tbl_* mode: p.nblocks is an upper bound on the blocks of all tables (grid size)
#ifdef LSMGPU_DIAG
  if (G > 1 || !p.pipe) {  // encode_kernel: G entry groups per trip, or the unpipelined order
    hipLaunchKernelGGL((encode_kernel<J, G>), dim3((p.nblocks + 3) / 4), dim3(256), 0, s, p);
    return hipGetLastError();
  }
#endif
#ifdef LSMGPU_DIAG
  if (p.pipe == 1) {  // one pass per loop trip (register copies at the back edge)
    hipLaunchKernelGGL((encode_pipe_kernel<J, false>), dim3((p.nblocks + 3) / 4), dim3(256), 0, s, p);
    return hipGetLastError();
  }
#endif
  hipLaunchKernelGGL((encode_pipe_kernel<J, true>), dim3((p.nblocks + 3) / 4), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_encode(const EncodeParams& p0, int num_cus, hipStream_t s) {
  (void)num_cus;
  EncodeParams p = p0;
  // one 16-B store for the header and the key's first 6 bytes (same box, C2 encode 0.5864-0.5895
  // -> 0.5627-0.5667 ms, profiles/r05ae); diag build: LSMGPU_ENC_HDR16=0 keeps the 8-B + 2-B stores
  p.hdr16 = 1u;
  // encode_pipe_kernel, two passes per trip: same box, C2 encode 0.565-0.566 -> 0.480-0.481 ms,
  // C5 0.760-0.762 -> 0.558-0.560 ms, C3 0.545-0.549 -> 0.441-0.447 ms (profiles/r06o); diag
  // build: LSMGPU_ENC_PIPE=0 keeps encode_kernel, 1 the one-pass-per-trip loop
  p.pipe = 2u;
  // J = lanes per entry ~ the average entry's 16-B pieces (C2: 129 B -> 8; C3: ~1.1 KB -> 64)
  const uint64_t avg = p.n ? (p.key_total + p.vs_total) / p.n : 120;
  // blocks of > 128-B entries: encode_dense_kernel (same box, C5 encode 0.560-0.562 -> 0.489-0.490
  // ms, C3 0.448-0.460 -> 0.430-0.442, profiles/r06ab); diag build: LSMGPU_ENC_DENSE=0 keeps the
  // J-lane passes; the LSMGPU_ENC_J test hook selects those too
  p.dense = 1u;
#ifdef LSMGPU_DIAG
  if (const char* de = getenv("LSMGPU_ENC_DENSE")) p.dense = atoi(de) != 0;
#endif
  if (LSMGPU_KNOB(p.dense, 1u) && avg > 128 && !getenv("LSMGPU_ENC_J")) {
    hipLaunchKernelGGL(encode_dense_kernel, dim3((p.nblocks + 3) / 4), dim3(256), 0, s, p);
    return hipGetLastError();
  }
  // LSMGPU_ENC_J (test hook): one of the compiled J (4, 8, 16) whatever the entry size
  if (const char* je = getenv("LSMGPU_ENC_J")) {
    const int jj = atoi(je);
    if (jj == 4) return launch_enc<4, 1>(p, s);
    if (jj == 16) return launch_enc<16, 1>(p, s);
    if (jj == 8) return launch_enc<8, 1>(p, s);
  }
#ifdef LSMGPU_DIAG
  if (const char* h16 = getenv("LSMGPU_ENC_HDR16")) p.hdr16 = atoi(h16) == 0 ? 0u : 1u;
  if (const char* pe = getenv("LSMGPU_ENC_PIPE")) p.pipe = (uint32_t)atoi(pe);  // 0, 1, 2 (unrolled)
  const char* ge = getenv("LSMGPU_ENC_G");  // A/B: entry-group passes per loop trip
  const int g = ge ? atoi(ge) : 1;           // measured: C2 G=1 0.61 ms, 2 0.68, 4 0.72
  if (g == 4) return avg <= 128 ? launch_enc<8, 4>(p, s) : launch_enc<16, 4>(p, s);
  if (g == 2) return avg <= 128 ? launch_enc<8, 2>(p, s) : launch_enc<16, 2>(p, s);
#endif
  // measured (1 GiB): C2 (119 B entries) J=8 0.57 ms vs J=4 0.63 / J=16 0.73; C5 (~141 B)
  // J=16 0.88 ms vs J=8 0.96
  if (avg <= 48) return launch_enc<4, 1>(p, s);
  if (avg <= 128) return launch_enc<8, 1>(p, s);
  if (avg <= 496) return launch_enc<16, 1>(p, s);
  if (avg <= 1008) return launch_enc<32, 1>(p, s);
  return launch_enc<64, 1>(p, s);
}

// ---------------------------------------------------------------- ValueStruct columns
// sizes: vs_end[i] = 2 + uvarint_len(expires_at[i]) + len(value i)  (y/iterator.go:31-38,
// without the uint16 truncation: the caller checks <= 65535 before building a table)
__global__ void values_sizes_kernel(ValuesParams p) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < p.n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t x = p.expires_at[i];
    uint32_t vn = 1;
    while (x >= 0x80) { x >>= 7; vn++; }
    uint32_t v0 = i ? p.value_end[i - 1] : 0;
    p.vs_end[i] = 2 + vn + (p.value_end[i] - v0);
  }
}

// write (after the inclusive scan turned sizes into end offsets): y/iterator.go:55-62
__global__ void values_write_kernel(ValuesParams p) {
  const uint32_t lane = lane_id();
  const uint64_t w = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) / kWave;
  for (uint64_t i = w; i < p.n; i += nw) {
    uint64_t o = i ? p.vs_end[i - 1] : 0;
    uint64_t v0 = i ? p.value_end[i - 1] : 0;
    uint32_t vlen = (uint32_t)(p.value_end[i] - v0);
    uint64_t x = p.expires_at[i];
    uint8_t var[10];
    uint32_t vn = 0;
    while (x >= 0x80) { var[vn++] = (uint8_t)(x | 0x80); x >>= 7; }
    var[vn++] = (uint8_t)x;
    uint32_t total = 2 + vn + vlen;
    for (uint32_t j = lane; j < total; j += kWave) {
      uint8_t byte;
      if (j == 0) byte = p.meta[i];
      else if (j == 1) byte = p.user_meta[i];
      else if (j < 2 + vn) {
        uint32_t q = j - 2;
        byte = 0;
        for (uint32_t z = 0; z < 10; z++) if (z == q) byte = var[z];
      } else byte = p.values[v0 + (j - 2 - vn)];
      p.vs[o + j] = byte;
    }
  }
}

hipError_t launch_values_sizes(const ValuesParams& p, hipStream_t s) {
  uint64_t g = (p.n + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(values_sizes_kernel, dim3((unsigned)g), dim3(256), 0, s, p);
  return hipGetLastError();
}
hipError_t launch_values_write(const ValuesParams& p, hipStream_t s) {
  uint64_t g = (p.n + 3) / 4;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(values_write_kernel, dim3((unsigned)g), dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace lsmgpu
