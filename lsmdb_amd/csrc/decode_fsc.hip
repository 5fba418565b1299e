// decode_fsc.hip -- fused, persistent SST block decode for batches of blocks <= 4 KiB (BASELINE
// C2 / C3): ONE launch that reads the block bytes from HBM once and copies them out of LDS.
//
// One 512-thread workgroup per CU (grid G <= 256, all resident: ~152 KiB of LDS each).  The
// batch is cut into chunks of kChunk = 12 consecutive blocks; in round r workgroup w owns chunk
// r * G + w.  Iteration r of every workgroup, after one barrier:
//   wave 0   : LDS-DMA of chunk r + 1 into ring slot (r + 1) % 3 (global_load_lds_dwordx4,
//              coalesced 1 KiB per instruction, no registers), then the walk of chunk r from
//              slot r % 3: one lane per block, blockIterator.Next/parseKV (table/iterator.go:
//              93-135) with its exact stop rules, each header read issued before the previous
//              entry's checks.  Per entry one u32 record {header pos | stored key bytes before
//              it << 16} (+ a sentinel) goes to the LDS pool (records 0..63 of a block; later
//              ones to global scratch).  Last, the chunk's {entries, key bytes, value bytes} are
//              published as an epoch-tagged granule record (p.lb).
//   wave 1   : reads the G records of round r - 1 (all published one iteration ago), which
//              gives chunk (r - 1, w)'s output base as P + sum of the records before it (P =
//              the running total of earlier rounds, kept in registers) -- no chained look-back,
//              so no tile waits on a slow predecessor's predecessor; then the per-block outputs
//              (blk_first, blk_status, totals, capacity) and the per-block bases in LDS.
//   waves 2-7: copy chunk r - 1 out of slot (r - 1) % 3: 8 lanes per entry, 16-B pieces read from
//              LDS at any byte offset, unaligned 16-B global stores, + key_end / val_end / view.
// So one chunk's DMA, another's walk and a third's copy overlap in every iteration, and the input
// crosses HBM once.  Blocks with prefix-compressed entries (plen > 0: never written by Builder,
// SURVEY F1) are copied by a serial per-block path from global memory with u32 offsets.
#include <cstdio>
#include <cstdlib>

#include "codec_common.hpp"
#include "decode_common.hpp"
#include "kernels.hpp"

namespace lsmgpu {

namespace {

constexpr uint32_t kFscMaxLen = 4096;   // blocks of this path
constexpr uint32_t kFscSlot = 4128;     // 258 16-B chunks: 4096 B at any 16-B shift + the walk's
                                        // 12-B header over-read
constexpr uint32_t kFscChunks = kFscSlot / 16;
constexpr uint32_t kChunk = 12;         // blocks per chunk
constexpr uint32_t kRing = 3;           // slots: DMA (r + 1), walk (r), copy (r - 1)
constexpr uint32_t kPoolRec = 64;       // records per block kept in LDS
constexpr uint32_t kMaxGrid = 256;      // wave 1 gathers <= 4 round records per lane
constexpr uint32_t kCopyWaves = 6;      // waves 2..7, two blocks each
static_assert(kChunk == 2 * kCopyWaves, "copy waves take two blocks each");
static_assert(kChunk <= 64, "one walking lane per block");

// Piece q of a `len`-byte stream (copy_piece16's cut): 16-B pieces, the last overlapping back
// inside the stream; below 16 B two overlapping 8/4-B pieces; below 4 B single bytes.
__device__ __forceinline__ uint32_t piece_at(uint32_t len, uint32_t q, uint32_t& sz) {
  if (len >= 16) { sz = 16; return min(16 * q, len - 16); }
  if (len >= 8) { sz = 8; return q ? len - 8 : 0; }
  if (len >= 4) { sz = 4; return q ? len - 4 : 0; }
  sz = 1;
  return q;
}
// sz bytes at byte x of an LDS slot (any alignment; aligned dword reads + v_alignbyte)
__device__ __forceinline__ uint4 lds_piece(const uint8_t* lds, uint32_t x, uint32_t sz) {
  if (sz == 16) return lds_u128(lds, x);
  uint4 v = make_uint4(0, 0, 0, 0);
  if (sz == 8) {
    v.x = lds_u32(lds, x);
    v.y = lds_u32(lds, x + 4);
  } else if (sz == 4) {
    v.x = lds_u32(lds, x);
  } else if (sz == 1) {
    v.x = lds[x];
  }
  return v;
}
__device__ __forceinline__ void store_piece(uint8_t* d, uint4 v, uint32_t sz) {
  if (sz == 16) __builtin_memcpy(d, &v, 16);
  else if (sz == 8) __builtin_memcpy(d, &v, 8);
  else if (sz == 4) __builtin_memcpy(d, &v, 4);
  else if (sz == 1) *d = (uint8_t)v.x;
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}

// Entries of one block (plen == 0 throughout) from its LDS slot: J lanes per entry, G entry
// groups per pass.  Records r_i = {header pos | S_i << 16}, S_i = stored key bytes of entries
// < i, r_n = the sentinel {stop pos | S_n << 16}; r_i is in the LDS pool for i < 64, in global
// scratch after.  So klen_i = S_{i+1} - S_i, vlen_i = hp_{i+1} - hp_i - 10 - klen_i, and the
// value offset in the block's value stream is hp_i - 10 i - S_i.
template <uint32_t J, uint32_t G>
__device__ __forceinline__ void copy_block_lds(const DecodeParams& p, const uint32_t* pool,
                                               const uint32_t* gm, const uint8_t* slot,
                                               uint32_t sh, uint8_t* kbase, uint8_t* vbase,
                                               uint32_t n, uint64_t en, uint64_t ek, uint64_t ev,
                                               uint32_t off, bool mat, bool view, uint32_t lane) {
  constexpr uint32_t kPass = G * (kWave / J);  // entries per pass (<= 64)
  static_assert(kPass <= kWave, "one lane per entry for the end offsets");
  const uint32_t j = lane & (J - 1);
  const uint32_t pre = pool[min(lane, n)];  // records 0..63 are in the pool
  auto rec = [&](uint32_t e, bool shuffled) -> uint32_t {
    if (shuffled) return (uint32_t)__shfl((int)pre, (int)e);
    return e < kPoolRec ? pool[e] : gm[e];
  };
  for (uint32_t e0 = 0; e0 < n; e0 += kPass) {
    const bool shuffled = e0 + kPass < kWave;  // every record of the pass is in `pre`
    // end offsets / view records: one lane per entry
    {
      const uint32_t e = e0 + lane;
      const uint32_t ec = min(e, n - 1);
      const uint32_t r0 = rec(ec, shuffled), r1 = rec(ec + 1, shuffled);
      const uint32_t hp = r0 & 0xffffu, ko = r0 >> 16, kl = (r1 >> 16) - ko;
      const uint32_t vl = (r1 & 0xffffu) - hp - 10 - kl, vo = hp - 10 * ec - ko;
      if (lane < kPass && e < n) {
        if (mat) {
          if (p.key_end) p.key_end[en + e] = (uint32_t)(ek + ko + kl);
          if (p.val_end) p.val_end[en + e] = (uint32_t)(ev + vo + vl);
        }
        if (view)
          p.view[en + e] = (uint64_t)(off + hp + 10) | ((uint64_t)kl << 32) | ((uint64_t)vl << 48);
      }
    }
    if (!mat) continue;
    // pieces: J lanes per entry, G entries per lane
    uint32_t hp[G], kl[G], vl[G], ko[G], vo[G], np[G], kp[G];
    uint32_t npmax = 0;
    bool all16 = true;
#pragma unroll
    for (int i = 0; i < G; i++) {
      const uint32_t e = e0 + i * (kWave / J) + (lane / J);
      const uint32_t ec = min(e, n - 1);
      const uint32_t r0 = rec(ec, shuffled), r1 = rec(ec + 1, shuffled);
      hp[i] = r0 & 0xffffu;
      ko[i] = r0 >> 16;
      kl[i] = (r1 >> 16) - ko[i];
      vl[i] = (r1 & 0xffffu) - hp[i] - 10 - kl[i];
      vo[i] = hp[i] - 10 * ec - ko[i];
      const bool on = e < n;
      kp[i] = kbase ? pieces16(kl[i]) : 0u;
      np[i] = on ? kp[i] + (vbase ? pieces16(vl[i]) : 0u) : 0u;
      npmax = max(npmax, np[i]);
      all16 = all16 && (!on || ((!kbase || kl[i] >= 16) && (!vbase || vl[i] >= 16)));
    }
    npmax = wave_max(npmax);
    if (__all(all16)) {
      // every piece is 16 B: one (misaligned) ds_read_b128 each, all reads before the stores
      for (uint32_t qb = 0; qb < npmax; qb += J) {
        const uint32_t q = qb + j;
        uint4 v[G];
        uint8_t* d[G];
#pragma unroll
        for (int i = 0; i < G; i++) {
          // every lane reads (an inactive piece reads slot byte 0): v[i] is defined on every
          // path, so it stays in registers
          const bool act = q < np[i];
          const bool key = q < kp[i];
          const uint32_t len = key ? kl[i] : vl[i];
          const uint32_t o = min(16 * (key ? q : q - kp[i]), len - 16);
          const uint32_t x = act ? sh + hp[i] + 10 + (key ? 0u : kl[i]) + o : 0u;
          // a typed (misaligned) ds_read_b128: taking v[i]'s address for memcpy would keep
          // the array in scratch
          v[i] = *reinterpret_cast<const uint4*>(slot + x);
          d[i] = act ? (key ? kbase + ko[i] : vbase + vo[i]) + o : nullptr;
        }
#pragma unroll
        for (int i = 0; i < G; i++)
          if (d[i]) {
            const uint4 t = v[i];
            __builtin_memcpy(d[i], &t, 16);
          }
      }
      continue;
    }
    for (uint32_t qb = 0; qb < npmax; qb += J) {
      const uint32_t q = qb + j;
#pragma unroll
      for (int i = 0; i < G; i++) {
        if (q >= np[i]) continue;
        const bool key = q < kp[i];
        uint32_t sz;
        const uint32_t o = piece_at(key ? kl[i] : vl[i], key ? q : q - kp[i], sz);
        const uint32_t x = sh + hp[i] + 10 + (key ? 0u : kl[i]) + o;
        store_piece((key ? kbase + ko[i] : vbase + vo[i]) + o, lds_piece(slot, x, sz), sz);
      }
    }
  }
}

// A block with prefix-compressed entries: the wave replays the walk serially (uniform) from
// global memory with u32 output offsets; key = baseKey[:plen] ++ diff (iterator.go:98-100),
// baseKey = entry 0's key (bytes from block offset 10, as Go's slice of the block).
__device__ void copy_block_slow(const DecodeParams& p, const uint8_t* blk, uint32_t n,
                                uint64_t en, uint64_t ek, uint64_t ev, uint32_t off, bool mat,
                                bool view, uint32_t lane) {
  const GlobalSrc src{blk};
  uint32_t pos = 0;
  uint64_t K = 0, V = 0;
  for (uint32_t i = 0; i < n; i++) {
    const Hdr h = src.hdr(pos);
    const uint32_t ks = pos + 10, kout = h.plen + h.klen;
    if (mat) {
      if (p.key_data)
        for (uint32_t x = lane; x < kout; x += kWave)
          p.key_data[ek + K + x] = x < h.plen ? blk[10 + x] : blk[ks + x - h.plen];
      if (p.val_data)
        for (uint32_t x = lane; x < h.vlen; x += kWave) p.val_data[ev + V + x] = blk[ks + h.klen + x];
      if (lane == 0) {
        if (p.key_end) p.key_end[en + i] = (uint32_t)(ek + K + kout);
        if (p.val_end) p.val_end[en + i] = (uint32_t)(ev + V + h.vlen);
      }
    }
    if (view && lane == 0)
      p.view[en + i] = (uint64_t)(off + ks) | ((uint64_t)h.klen << 32) | ((uint64_t)h.vlen << 48);
    K += kout;
    V += h.vlen;
    pos = ks + h.klen + h.vlen;
  }
}


// A copy wave's two blocks (lanes 0, 1) of round r's chunk: [off, len); len ~0 = no block
__device__ __forceinline__ void load_ol2(const DecodeParams& p, uint32_t r, uint32_t R,
                                         uint32_t G, uint32_t w, uint32_t bi0, uint32_t lane,
                                         uint32_t& o, uint32_t& l) {
  o = 0;
  l = 0xffffffffu;
  const uint64_t b = ((uint64_t)r * G + w) * kChunk + bi0 + lane;
  if (r < R && lane < 2 && b < p.nblk) {
    o = p.blk_off[b];
    l = p.blk_len[b];
  }
}

__device__ __forceinline__ bool blk_fits(const DecodeParams& p, uint32_t off, uint32_t len) {
  return len <= kFscMaxLen && (uint64_t)off + len <= p.data_len;
}

// LDS-DMA of one block into its slot: 5 x 1 KiB (chunks 0..257 of its 16-B aligned span).
// Lanes past the block (or past the data) load an in-bounds line into the slot's unused tail,
// so every instruction keeps its lanes.  (Register staging -- global_load_dwordx4 + ds_write --
// measured slower here: the in-flight registers of this three-role kernel went to scratch.)
__device__ __forceinline__ void dma_block(const DecodeParams& p, uint8_t* dst, uint32_t off,
                                          uint32_t len, uint32_t lane) {
  const uint64_t last = p.data_len >= 16 ? ((p.data_len - 16) & ~15ull) : 0ull;
  const uint64_t a0 = blk_fits(p, off, len) ? (uint64_t)(off & ~15u) : 0ull;
#pragma unroll
  for (uint32_t q = 0; q < 5; q++) {
    const uint32_t c = lane + q * kWave;
    if (q < 4 || c < kFscChunks) {
      uint64_t a = a0 + 16ull * c;
      a = a < last ? a : last;
      dma16(p.data + a, dst + q * 1024);
    }
  }
}

// The 16-B line crossing the end of the data buffer (DMA moves whole lines): bytewise.  Only
// the block holding the buffer's last byte can have one.
__device__ __forceinline__ void fix_tail(const DecodeParams& p, uint8_t* dst, uint32_t off,
                                         uint32_t len, uint32_t lane) {
  if (!blk_fits(p, off, len)) return;
  const uint64_t a0 = off & ~15ull;
  const uint32_t nch = ((off & 15u) + len + 15) >> 4;
  if (a0 + 16ull * nch <= p.data_len) return;
  const uint64_t ct = (p.data_len - a0) >> 4;  // the crossing chunk
  const uint64_t a = a0 + 16 * ct + lane;
  if (lane < 16) dst[16 * ct + lane] = a < p.data_len ? p.data[a] : 0;
}

}  // namespace

// LSMGPU_STAMPS diagnostics: s_memtime cycles per phase of wave 0 / wave 1 / wave 2, summed over
// workgroups and iterations
#define FSC_STAMP(i)                                                                   \
  if (p.stamps && lane == 0 && wave <= 2) {                                            \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();                                  \
    atomicAdd(reinterpret_cast<unsigned long long*>(p.stamps + (i)), t_ - t_prev);     \
    t_prev = t_;                                                                       \
  }

__global__ void __launch_bounds__(512) fsc_kernel(DecodeParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t slots[kRing * kChunk * kFscSlot];
  __shared__ uint32_t pool[2][kChunk * kPoolRec];
  __shared__ uint32_t s_n[2][kChunk], s_k[2][kChunk], s_v[2][kChunk], s_st[2][kChunk];
  __shared__ uint32_t s_off[kRing][kChunk], s_len[kRing][kChunk], s_slow[2];
  __shared__ uint32_t s_bn[kChunk], s_bk[kChunk], s_bv[kChunk], s_ok;
  __shared__ uint32_t s_ready;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint32_t G = gridDim.x, w = blockIdx.x, nblk = p.nblk;
  const uint32_t nchunks = (nblk + kChunk - 1) / kChunk;
  const uint32_t R = (nchunks + G - 1) / G;  // rounds
  const uint64_t tag = p.tag;
  uint32_t* const wm = p.wmeta;
  uint64_t t_prev = p.stamps ? __builtin_amdgcn_s_memtime() : 0;
  if (tid == 0) s_ready = 0xffffffffu;
  // copy waves: their two blocks of the chunk being DMA'd (cur) and of the next (nxt)
  const uint32_t bi0 = 2 * (wave - 2);
  uint32_t cur_o = 0, cur_l = 0xffffffffu, nxt_o = 0, nxt_l = 0xffffffffu;
  if (wave >= 2) {
    load_ol2(p, 0, R, G, w, bi0, lane, cur_o, cur_l);
    load_ol2(p, 1, R, G, w, bi0, lane, nxt_o, nxt_l);
    if (R > 0) {
#pragma unroll
      for (uint32_t x = 0; x < 2; x++) {
        const uint32_t o = readlane(cur_o, x), l = readlane(cur_l, x);
        dma_block(p, slots + (bi0 + x) * kFscSlot, o, l, lane);
        if (lane == 0) {
          s_off[0][bi0 + x] = o;
          s_len[0][bi0 + x] = l;
        }
      }
    }
  }
  uint32_t Pn = 0, Pk = 0, Pv = 0;  // wave 1: totals of the rounds gathered so far

  for (uint32_t r = 0; r <= R; r++) {
    // every wave's global stores and the copy waves' DMA of chunk r are complete
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (wave >= 2 && r < R) {
#pragma unroll
      for (uint32_t x = 0; x < 2; x++)
        fix_tail(p, slots + ((r % kRing) * kChunk + bi0 + x) * kFscSlot, readlane(cur_o, x),
                 readlane(cur_l, x), lane);
    }
    __syncthreads();
    if (wave == 0) {
      // ---- walk chunk r: lane = block (the walk is one instruction stream: run it first)
      __builtin_amdgcn_s_setprio(3);
      if (r >= R) continue;
      FSC_STAMP(0)  // barrier
      const uint32_t s = r % kRing, par = r & 1;
      const uint32_t cid = r * G + w;
      const uint64_t b = (uint64_t)cid * kChunk + lane;
      const bool has = lane < kChunk && cid < nchunks && b < nblk;
      uint32_t n = 0, K = 0, V = 0, S = 0, pos = 0, st = LSMGPU_BLK_OK;
      bool any_plen = false;
      if (has) {
        const uint32_t off = s_off[s][lane], len = s_len[s][lane];
        uint32_t* const pr = &pool[par][lane * kPoolRec];
        uint32_t* const gr = wm + b * p.wcap;
        if (!blk_fits(p, off, len)) {
          st = LSMGPU_BLK_RANGE;
        } else if (!(p.ablate & 4)) {
          const uint8_t* const sb = slots + (s * kChunk + lane) * kFscSlot + (off & 15u);
          // fast loop: plen == 0 entries (every entry Builder writes) while the
          // records fit the LDS pool; one misaligned 8-B LDS read per header, no branch but the
          // exit.  Anything else -- a stop rule, plen > 0, entry 63 -- leaves the rest of the
          // block to the general loop below.
          for (;;) {
            uint2 hw;
            __builtin_memcpy(&hw, sb + pos, 8);  // pos <= len keeps the read inside the slot
            const uint32_t plen = __builtin_amdgcn_perm(0u, hw.x, 0x0c0c0001u);
            const uint32_t klen = __builtin_amdgcn_perm(0u, hw.x, 0x0c0c0203u);
            const uint32_t vlen = __builtin_amdgcn_perm(0u, hw.y, 0x0c0c0001u);
            const uint32_t end = pos + 10 + klen + vlen;
            if ((len - pos < 10) | (klen == 0) | (plen != 0) | (end > len) | (n >= kPoolRec - 1))
              break;
            pr[n] = pos | (S << 16);
            S += klen;
            n++;
            pos = end;
          }
          K = S;
          V = pos - 10 * n - S;
          // general loop from here: prefix-compressed entries (plen > 0) and every stop rule
          // of table/iterator.go:93-135 in the iterator's order
          const LdsSrc src{slots + (s * kChunk + lane) * kFscSlot, off & 15u};
          for (;;) {
            const Hdr h = src.hdr(pos);  // pos <= len keeps the read inside the slot
            const uint32_t end = pos + 10 + h.klen + h.vlen;
            const bool eof = pos >= len;                              // iterator.go:115-118
            const bool trunc = len - pos < 10;
            const bool term = (h.klen | h.plen) == 0;                 // iterator.go:124-127
            const bool fplen = n == 0 && h.plen != 0;                 // iterator.go:129-133
            const bool poob = 10 + h.plen > len;                      // base key = entry 0's
            const bool vovf = end > len;                              // iterator.go:101-106
            if (eof | trunc | term | fplen | poob | vovf) {
              st = (eof | (!trunc & term)) ? LSMGPU_BLK_OK
                   : trunc                 ? LSMGPU_BLK_TRUNC_HEADER
                   : fplen                 ? LSMGPU_BLK_FIRST_PLEN
                   : poob                  ? LSMGPU_BLK_PREFIX_OOB
                                           : LSMGPU_BLK_VALUE_OVERFLOW;
              break;
            }
            const uint32_t rec = pos | (S << 16);
            if (n < kPoolRec) pr[n] = rec;
            else gr[n] = rec;
            any_plen = any_plen || h.plen != 0;
            K += h.plen + h.klen;
            S += h.klen;
            V += h.vlen;
            n++;
            pos = end;
          }
        }
        const uint32_t rec = pos | (S << 16);  // sentinel
        if (n < kPoolRec) pr[n] = rec;
        else gr[n] = rec;
        s_n[par][lane] = n;
        s_k[par][lane] = K;
        s_v[par][lane] = V;
        s_st[par][lane] = st;
      }
      const uint64_t sm = __ballot(has && any_plen);
      if (lane == 0) s_slow[par] = (uint32_t)sm;
      // publish the chunk's aggregate (read by every workgroup next iteration)
      const uint32_t an = wave_sum_sat(n), ak = wave_sum_sat(K), av = wave_sum_sat(V);
      if (cid < nchunks) store3(p.lb + (uint64_t)cid * 8, tag, an, ak, av, lane);
      FSC_STAMP(2)  // walk + publish
      continue;
    }
    if (wave == 1) {
      if (r == 0) continue;
      const uint32_t rp = r - 1, par = rp & 1;
      const uint32_t cid = rp * G + w;
      // ---- prefix of chunk (r - 1, w): the G records of round r - 1
      FSC_STAMP(4)  // barrier
      uint32_t a[4][3];
      bool got[4];
#pragma unroll
      for (int x = 0; x < 4; x++) {
        const uint32_t wx = lane + 64 * x;
        got[x] = !(wx < G && (uint64_t)rp * G + wx < nchunks) || (p.ablate & 1);
        a[x][0] = a[x][1] = a[x][2] = 0;
      }
      for (SpinBound bound;;) {
#pragma unroll
        for (int x = 0; x < 4; x++)
          if (!got[x])
            got[x] = read3(p.lb + ((uint64_t)rp * G + lane + 64 * x) * 8, tag, a[x][0], a[x][1],
                           a[x][2]);
        if (__all(got[0] && got[1] && got[2] && got[3])) break;
        if (bound.expired()) {
          flag_timeout(p.result, lane);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      uint32_t bn = 0, bk = 0, bv = 0, tn = 0, tk = 0, tv = 0;
#pragma unroll
      for (int x = 0; x < 4; x++) {
        tn = sat_add(tn, a[x][0]);
        tk = sat_add(tk, a[x][1]);
        tv = sat_add(tv, a[x][2]);
        if (lane + 64 * x < w) {
          bn = sat_add(bn, a[x][0]);
          bk = sat_add(bk, a[x][1]);
          bv = sat_add(bv, a[x][2]);
        }
      }
      const uint32_t exn = sat_add(Pn, wave_sum_sat(bn)), exk = sat_add(Pk, wave_sum_sat(bk)),
                     exv = sat_add(Pv, wave_sum_sat(bv));
      Pn = sat_add(Pn, wave_sum_sat(tn));
      Pk = sat_add(Pk, wave_sum_sat(tk));
      Pv = sat_add(Pv, wave_sum_sat(tv));
      FSC_STAMP(5)  // gather
      // ---- per-block outputs of chunk (r - 1, w)
      const uint64_t b = (uint64_t)cid * kChunk + lane;
      const bool has = cid < nchunks && lane < kChunk && b < nblk;
      const uint32_t n = has ? s_n[par][lane] : 0u, K = has ? s_k[par][lane] : 0u,
                     V = has ? s_v[par][lane] : 0u;
      const uint32_t in_ = wave_scan_sat(n, lane), ik = wave_scan_sat(K, lane),
                     iv = wave_scan_sat(V, lane);
      bool ok = false;
      if (has) {
        const uint32_t st = s_st[par][lane];
        const uint32_t en = sat_add(exn, in_ - n),
                       ek = sat_add(exk, ik == 0xffffffffu ? ik : ik - K),
                       ev = sat_add(exv, iv - V);
        s_bn[lane] = en;
        s_bk[lane] = ek;
        s_bv[lane] = ev;
        ok = (uint64_t)en + n <= p.ent_cap && (uint64_t)en + n <= 0xffffffffull;
        if (p.mode & LSMGPU_MODE_MATERIALIZE) {
          const uint64_t kend = (uint64_t)ek + K, vend = (uint64_t)ev + V;
          ok = ok && (kend <= p.key_cap || !p.key_data) && (vend <= p.val_cap || !p.val_data);
          ok = ok && kend < 0xffffffffull && vend <= 0xffffffffull;
        }
        const uint64_t okm = __ballot(ok);
        if (lane == 0) {
          s_ok = (uint32_t)okm;
          __hip_atomic_store(&s_ready, r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (p.blk_first) p.blk_first[b] = en;
        if (p.blk_status) p.blk_status[b] = (int32_t)st;
        if (st != LSMGPU_BLK_OK) {
          atomicAdd(reinterpret_cast<unsigned long long*>(p.result + 4), 1ull);
          atomicMax(reinterpret_cast<unsigned long long*>(p.result + 3),
                    (unsigned long long)(nblk - b));
        }
        if (b == nblk - 1) {  // totals of the whole batch
          if (p.blk_first) p.blk_first[nblk] = (uint32_t)((uint64_t)en + n);
          p.result[0] = (uint64_t)en + n;
          p.result[1] = (uint64_t)ek + K;
          p.result[2] = (uint64_t)ev + V;
        }
        if (!ok) atomicOr(reinterpret_cast<unsigned long long*>(p.result + 5), 1ull);
      }
      FSC_STAMP(6)  // per-block outputs
      continue;
    }
    // ---- waves 2..7: DMA their two blocks of chunk r + 1, then copy their two of chunk r - 1
    FSC_STAMP(8)  // barrier
    if (r + 1 < R) {
      const uint32_t s1 = (r + 1) % kRing;
#pragma unroll
      for (uint32_t x = 0; x < 2; x++) {
        const uint32_t o = readlane(nxt_o, x), l = readlane(nxt_l, x);
        dma_block(p, slots + (s1 * kChunk + bi0 + x) * kFscSlot, o, l, lane);
        if (lane == 0) {
          s_off[s1][bi0 + x] = o;
          s_len[s1][bi0 + x] = l;
        }
      }
    }
    cur_o = nxt_o;
    cur_l = nxt_l;
    load_ol2(p, r + 2, R, G, w, bi0, lane, nxt_o, nxt_l);
    FSC_STAMP(9)  // DMA issue
    if (r == 0) continue;
    const uint32_t rp = r - 1, par = rp & 1, s = rp % kRing;
    const uint32_t cid = rp * G + w;
    if (cid >= nchunks) continue;
    for (SpinBound bound;;) {
      if (__hip_atomic_load(&s_ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == r) break;
      if (bound.expired()) {
        flag_timeout(p.result, lane);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    FSC_STAMP(10)  // wait for the prefix
    if (p.ablate & 2) continue;
    const bool mat = (p.mode & LSMGPU_MODE_MATERIALIZE) != 0;
    const bool view = (p.mode & LSMGPU_MODE_VIEW) != 0 && p.view;
    if (!mat && !view) continue;
    const uint32_t okm = s_ok, slowm = s_slow[par];
#pragma unroll
    for (uint32_t x = 0; x < 2; x++) {
      const uint32_t bi = bi0 + x;
      const uint64_t b = (uint64_t)cid * kChunk + bi;
      if (b >= nblk) break;
      const uint32_t n = uniform(s_n[par][bi]);
      if (n == 0 || !((okm >> bi) & 1)) continue;
      const uint64_t en = uniform(s_bn[bi]), ek = uniform(s_bk[bi]), ev = uniform(s_bv[bi]);
      const uint32_t off = uniform(s_off[s][bi]);
      if ((slowm >> bi) & 1) {
        copy_block_slow(p, p.data + off, n, en, ek, ev, off, mat, view, lane);
        continue;
      }
      uint8_t* kbase = (mat && p.key_data) ? p.key_data + ek : nullptr;
      uint8_t* vbase = (mat && p.val_data) ? p.val_data + ev : nullptr;
      copy_block_lds<8, 5>(p, &pool[par][bi * kPoolRec], wm + b * p.wcap,
                           slots + (s * kChunk + bi) * kFscSlot, off & 15u, kbase, vbase, n, en,
                           ek, ev, off, mat, view, lane);
    }
    FSC_STAMP(11)  // copy
  }
  if (p.stamps && tid == 0) atomicAdd(reinterpret_cast<unsigned long long*>(p.stamps + 12), (unsigned long long)R);
}

// ============================================================ wave-owned blocks (default)
// A 512-thread workgroup takes the next tile of 16 consecutive blocks from an ordered ticket
// (p.gcnt[0]); each wave OWNS two of them for the workgroup's whole life:
//   load   : both blocks' 16-B aligned spans into registers (coalesced, 1 KiB per instruction),
//            then into the wave's two LDS slots;
//   walk   : lanes 0 and 1 walk the two blocks from LDS (blockIterator.Next/parseKV,
//            table/iterator.go:93-135), records {header pos | stored key bytes << 16} to the LDS
//            pool (entries 0..63; later ones to global scratch);
//   scan   : after a barrier wave 0 scans the 16 blocks, publishes the tile aggregate and finds
//            the tile's output base by decoupled look-back over the earlier tiles' records (the
//            ticket makes every earlier tile already running, so it always progresses);
//   copy   : after a barrier every wave copies its two blocks out of LDS (8 lanes per entry,
//            16-B pieces, unaligned global stores) + key_end / val_end / view records.
// An LDS walk is latency-bound (~210 cycles per entry whatever the number of lanes walking,
// scripts/walk_probe.hip), so what sets its throughput is how many blocks walk at once: here
// every resident block does -- 32 per CU at two workgroups per CU -- against 12-16 in the
// slot-ring designs, where only one slot of the ring is being walked.
constexpr uint32_t kWbWaves = 8;  // waves per workgroup (4: 0.90 vs 0.86 ms, C2 1 GiB)
constexpr uint32_t kWbPer = 2;    // blocks per wave
constexpr uint32_t kWbTile = kWbWaves * kWbPer;  // blocks per tile

__device__ __forceinline__ void walk_block_lds(const DecodeParams& p, const uint8_t* slot,
                                               uint32_t off, uint32_t len, uint32_t* pr,
                                               uint32_t* gr, uint32_t& n_, uint32_t& K_,
                                               uint32_t& V_, uint32_t& st_, bool& any_plen) {
  uint32_t n = 0, K = 0, V = 0, S = 0, pos = 0, st = LSMGPU_BLK_OK;
  if (!blk_fits(p, off, len)) {
    st = LSMGPU_BLK_RANGE;
  } else {
    const uint8_t* const sb = slot + (off & 15u);
    // fast loop: plen == 0 entries (every entry Builder writes) while the records
    // fit the LDS pool; anything else leaves the rest of the block to the general loop
    for (;;) {
      uint2 hw;
      __builtin_memcpy(&hw, sb + pos, 8);  // pos <= len keeps the read inside the slot
      const uint32_t plen = __builtin_amdgcn_perm(0u, hw.x, 0x0c0c0001u);
      const uint32_t klen = __builtin_amdgcn_perm(0u, hw.x, 0x0c0c0203u);
      const uint32_t vlen = __builtin_amdgcn_perm(0u, hw.y, 0x0c0c0001u);
      const uint32_t end = pos + 10 + klen + vlen;
      if ((len - pos < 10) | (klen == 0) | (plen != 0) | (end > len) | (n >= kPoolRec - 1)) break;
      pr[n] = pos | (S << 16);
      S += klen;
      n++;
      pos = end;
    }
    K = S;
    V = pos - 10 * n - S;
    // general loop: prefix-compressed entries and every stop rule, in the iterator's order
    const LdsSrc src{slot, off & 15u};
    for (;;) {
      const Hdr h = src.hdr(pos);
      const uint32_t end = pos + 10 + h.klen + h.vlen;
      const bool eof = pos >= len;                              // iterator.go:115-118
      const bool trunc = len - pos < 10;
      const bool term = (h.klen | h.plen) == 0;                 // iterator.go:124-127
      const bool fplen = n == 0 && h.plen != 0;                 // iterator.go:129-133
      const bool poob = 10 + h.plen > len;                      // base key = entry 0's
      const bool vovf = end > len;                              // iterator.go:101-106
      if (eof | trunc | term | fplen | poob | vovf) {
        st = (eof | (!trunc & term)) ? LSMGPU_BLK_OK
             : trunc                 ? LSMGPU_BLK_TRUNC_HEADER
             : fplen                 ? LSMGPU_BLK_FIRST_PLEN
             : poob                  ? LSMGPU_BLK_PREFIX_OOB
                                     : LSMGPU_BLK_VALUE_OVERFLOW;
        break;
      }
      const uint32_t rec = pos | (S << 16);
      if (n < kPoolRec) pr[n] = rec;
      else gr[n] = rec;
      any_plen = any_plen || h.plen != 0;
      K += h.plen + h.klen;
      S += h.klen;
      V += h.vlen;
      n++;
      pos = end;
    }
  }
  const uint32_t rec = pos | (S << 16);  // sentinel
  if (n < kPoolRec) pr[n] = rec;
  else gr[n] = rec;
  n_ = n;
  K_ = K;
  V_ = V;
  st_ = st;
}

__global__ void __launch_bounds__(kWbWaves * 64) fsw_kernel(DecodeParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t slots[kWbTile * kFscSlot];
  __shared__ uint32_t pool[kWbTile * kPoolRec];
  __shared__ uint32_t s_n[kWbTile], s_k[kWbTile], s_v[kWbTile], s_st[kWbTile], s_off[kWbTile];
  __shared__ uint32_t s_bn[kWbTile], s_bk[kWbTile], s_bv[kWbTile];
  __shared__ uint32_t s_slow, s_ok, s_tile;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint32_t nblk = p.nblk;
  uint64_t t_prev = p.stamps ? __builtin_amdgcn_s_memtime() : 0;
#define FSW_STAMP(i)                                                                       \
  if (p.stamps && lane == 0 && wave <= 1) {                                                \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();                                      \
    atomicAdd(reinterpret_cast<unsigned long long*>(p.stamps + (i) + 8 * wave), t_ - t_prev); \
    t_prev = t_;                                                                           \
  }
  const uint32_t ntiles = (nblk + kWbTile - 1) / kWbTile;
  if (tid == 0) {
    const uint32_t t = atomicAdd(p.gcnt, 1u);
    if (t == ntiles - 1) atomicExch(p.gcnt, 0u);  // every ticket is taken
    s_tile = t;
    s_slow = 0;
  }
  __syncthreads();
  FSW_STAMP(0)  // ticket
  const uint32_t tile = s_tile;
  const uint32_t b0 = tile * kWbTile;
  const uint32_t nb = min(kWbTile, nblk - b0);
  uint32_t* const wm = p.wmeta;

  // ---- load: the wave's two blocks, registers -> its LDS slots
  const uint32_t wb = kWbPer * wave;  // the wave's first block in the tile
  uint32_t o = 0, l = 0xffffffffu;
  if (lane < kWbPer && wb + lane < nb) {
    o = p.blk_off[b0 + wb + lane];
    l = p.blk_len[b0 + wb + lane];
  }
  {
    const uint64_t last = p.data_len >= 16 ? ((p.data_len - 16) & ~15ull) : 0ull;
    uint4 v[kWbPer][5];
#pragma unroll
    for (uint32_t x = 0; x < kWbPer; x++) {
      const uint32_t off = readlane(o, x), len = readlane(l, x);
      const uint64_t a0 = blk_fits(p, off, len) ? (uint64_t)(off & ~15u) : 0ull;
#pragma unroll
      for (uint32_t q = 0; q < 5; q++) {  // unconditional, clamped: no register merge, no wait
        uint64_t a = a0 + 16ull * (lane + q * kWave);
        a = a < last ? a : last;
        v[x][q] = *reinterpret_cast<const uint4*>(p.data + a);
      }
    }
    FSW_STAMP(1)  // [off, len) + load issue
#pragma unroll
    for (uint32_t x = 0; x < kWbPer; x++) {
      uint8_t* dst = slots + (wb + x) * kFscSlot;
#pragma unroll
      for (uint32_t q = 0; q < 5; q++) {
        const uint32_t c = lane + q * kWave;
        if (c < kFscChunks) *reinterpret_cast<uint4*>(dst + 16 * c) = v[x][q];
      }
      fix_tail(p, dst, readlane(o, x), readlane(l, x), lane);
    }
  }
  FSW_STAMP(2)  // load wait + LDS writes
  // ---- walk: lanes 0, 1 (a wave's LDS operations complete in order: no fence needed)
  {
    const uint32_t bi = wb + lane;
    const bool has = lane < kWbPer && bi < nb;
    bool any_plen = false;
    if (has) {
      uint32_t n, K, V, st;
      walk_block_lds(p, slots + bi * kFscSlot, o, l, pool + bi * kPoolRec,
                     wm + (uint64_t)(b0 + bi) * p.wcap, n, K, V, st, any_plen);
      s_n[bi] = n;
      s_k[bi] = K;
      s_v[bi] = V;
      s_st[bi] = st;
      s_off[bi] = o;
    }
    const uint64_t sm = __ballot(has && any_plen);
    if (lane == 0 && sm) atomicOr(&s_slow, (uint32_t)sm << wb);
  }
  FSW_STAMP(3)  // walk
  // records past 63 went to global scratch: complete them before other waves may read them
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  FSW_STAMP(4)  // barrier (the slowest walk)

  // ---- scan + look-back + per-block outputs (wave 0: lane = block)
  if (wave == 0) {
    const bool has = lane < nb;
    const uint32_t n = has ? s_n[lane] : 0u, K = has ? s_k[lane] : 0u, V = has ? s_v[lane] : 0u;
    const uint32_t in_ = wave_scan_sat(n, lane), ik = wave_scan_sat(K, lane),
                   iv = wave_scan_sat(V, lane);
    const uint32_t tn = readlane(in_, 63), tk = readlane(ik, 63), tv = readlane(iv, 63);
    uint64_t* Rr = p.lb + (uint64_t)tile * 8;
    Tot ex{0, 0, 0};
    if (tile > 0 && !(p.ablate & 1)) {  // (ablate 1, timing only: every tile at base 0)
      store3(Rr, p.tag, tn, tk, tv, lane);
      ex = lookback(p.lb, tile, p.tag, lane, p.result);
    }
    store3(Rr + 4, p.tag, sat_add(ex.n, tn), sat_add(ex.k, tk), sat_add(ex.v, tv), lane);
    bool ok = false;
    if (has) {
      const uint32_t b = b0 + lane, st = s_st[lane];
      const uint32_t en = sat_add(ex.n, in_ - n),
                     ek = sat_add(ex.k, ik == 0xffffffffu ? ik : ik - K),
                     ev = sat_add(ex.v, iv - V);
      s_bn[lane] = en;
      s_bk[lane] = ek;
      s_bv[lane] = ev;
      ok = (uint64_t)en + n <= p.ent_cap && (uint64_t)en + n <= 0xffffffffull;
      if (p.mode & LSMGPU_MODE_MATERIALIZE) {
        const uint64_t kend = (uint64_t)ek + K, vend = (uint64_t)ev + V;
        ok = ok && (kend <= p.key_cap || !p.key_data) && (vend <= p.val_cap || !p.val_data);
        ok = ok && kend < 0xffffffffull && vend <= 0xffffffffull;
      }
      if (p.blk_first) p.blk_first[b] = en;
      if (p.blk_status) p.blk_status[b] = (int32_t)st;
      if (st != LSMGPU_BLK_OK) {
        atomicAdd(reinterpret_cast<unsigned long long*>(p.result + 4), 1ull);
        atomicMax(reinterpret_cast<unsigned long long*>(p.result + 3),
                  (unsigned long long)(nblk - b));
      }
      if (b == nblk - 1) {  // totals of the whole batch
        if (p.blk_first) p.blk_first[nblk] = (uint32_t)((uint64_t)en + n);
        p.result[0] = (uint64_t)en + n;
        p.result[1] = (uint64_t)ek + K;
        p.result[2] = (uint64_t)ev + V;
      }
      if (!ok) atomicOr(reinterpret_cast<unsigned long long*>(p.result + 5), 1ull);
    }
    const uint64_t okm = __ballot(ok);
    if (lane == 0) s_ok = (uint32_t)okm;
  }
  __syncthreads();
  FSW_STAMP(5)  // scan + look-back + outputs
  if (p.ablate & 2) return;

  // ---- copy: each wave its two blocks, out of LDS
  const bool mat = (p.mode & LSMGPU_MODE_MATERIALIZE) != 0;
  const bool view = (p.mode & LSMGPU_MODE_VIEW) != 0 && p.view;
  if (!mat && !view) return;
  const uint32_t okm = s_ok, slowm = s_slow;
#pragma unroll
  for (uint32_t x = 0; x < kWbPer; x++) {
    const uint32_t bi = wb + x;
    if (bi >= nb) break;
    const uint32_t n = uniform(s_n[bi]);
    if (n == 0 || !((okm >> bi) & 1)) continue;
    const uint64_t en = uniform(s_bn[bi]), ek = uniform(s_bk[bi]), ev = uniform(s_bv[bi]);
    const uint32_t off = uniform(s_off[bi]);
    if ((slowm >> bi) & 1) {
      copy_block_slow(p, p.data + off, n, en, ek, ev, off, mat, view, lane);
      continue;
    }
    uint8_t* kbase = (mat && p.key_data) ? p.key_data + ek : nullptr;
    uint8_t* vbase = (mat && p.val_data) ? p.val_data + ev : nullptr;
    copy_block_lds<8, 5>(p, pool + bi * kPoolRec, wm + (uint64_t)(b0 + bi) * p.wcap,
                         slots + bi * kFscSlot, off & 15u, kbase, vbase, n, en, ek, ev, off, mat,
                         view, lane);
  }
  FSW_STAMP(6)  // copy
  if (p.stamps && tid == 0) atomicAdd(reinterpret_cast<unsigned long long*>(p.stamps + 7), 1ull);
#undef FSW_STAMP
}

hipError_t launch_decode_fsc(const DecodeParams& p, int num_cus, hipStream_t s) {
  const uint32_t nchunks = (p.nblk + kChunk - 1) / kChunk;
  uint32_t G = (uint32_t)(num_cus < (int)kMaxGrid ? num_cus : (int)kMaxGrid);
  if (G > nchunks) G = nchunks;
  if (G < 1) G = 1;
  static uint64_t* stamps = nullptr;
  DecodeParams q = p;
  q.stamps = nullptr;
  if (getenv("LSMGPU_STAMPS")) {  // diagnostics: per-phase cycle totals on stderr
    if (!stamps && hipMalloc(&stamps, 16 * sizeof(uint64_t)) != hipSuccess) stamps = nullptr;
    if (stamps) {
      (void)hipMemsetAsync(stamps, 0, 16 * sizeof(uint64_t), s);
      q.stamps = stamps;
    }
  }
  // LSMGPU_FSC=ring: the persistent slot-ring kernel; default: wave-owned blocks
  static const bool ring = getenv("LSMGPU_FSC") && getenv("LSMGPU_FSC")[0] == 'r';
  if (!ring) {
    hipLaunchKernelGGL(fsw_kernel, dim3((p.nblk + kWbTile - 1) / kWbTile), dim3(kWbWaves * 64), 0, s, q);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && q.stamps) {
      uint64_t h[16] = {0};
      (void)hipMemcpyAsync(h, stamps, sizeof(h), hipMemcpyDeviceToHost, s);
      (void)hipStreamSynchronize(s);
      const double t = h[7] ? (double)h[7] : 1.0;
      fprintf(stderr, "[lsmgpu] fsw stamps per tile (cycles) wave0|wave1: ticket %.0f|%.0f "
              "issue %.0f|%.0f loadwait %.0f|%.0f walk %.0f|%.0f barrier %.0f|%.0f scan %.0f|%.0f "
              "copy %.0f|%.0f | tiles %llu\n", h[0] / t, h[8] / t, h[1] / t, h[9] / t, h[2] / t,
              h[10] / t, h[3] / t, h[11] / t, h[4] / t, h[12] / t, h[5] / t, h[13] / t, h[6] / t,
              h[14] / t, (unsigned long long)h[7]);
    }
    return e;
  }
  hipLaunchKernelGGL(fsc_kernel, dim3(G), dim3(512), 0, s, q);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && q.stamps) {
    uint64_t h[16] = {0};
    (void)hipMemcpyAsync(h, stamps, sizeof(h), hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    const double it = h[12] ? (double)h[12] : 1.0;  // workgroup-iterations
    fprintf(stderr, "[lsmgpu] fsc stamps per iteration (cycles): wave0 barrier %.0f walk %.0f | "
            "wave1 barrier %.0f gather %.0f outputs %.0f | wave2 barrier %.0f dma %.0f "
            "prefix-wait %.0f copy %.0f | rounds x grid %llu\n", h[0] / it, h[2] / it, h[4] / it,
            h[5] / it, h[6] / it, h[8] / it, h[9] / it, h[10] / it, h[11] / it,
            (unsigned long long)h[12]);
  }
  return e;
}

}  // namespace lsmgpu
