// decode_fsc.hip -- "stream, walk, scan, copy": a ONE-launch SST block decode for batches of
// blocks <= 4 KiB (BASELINE C2 / C3) that reads the block bytes from HBM once.
//
// A 256-thread workgroup takes the next tile of TILE consecutive blocks from an ordered ticket
// (p.gcnt[0]) and runs three phases:
//   1. stream + walk: the tile goes through LDS SUB = 8 blocks at a time.  Every thread loads
//      one 16-B chunk of each block of the NEXT sub-batch into registers (coalesced, 1 KiB per
//      wave instruction) while wave 0 walks the CURRENT sub-batch from LDS.  The walk is
//      blockIterator.Next/parseKV (table/iterator.go:93-135) with 8 lanes per block: lane k
//      reads the header guessed at pos + k * stride (stride = the last entry's size), so a run
//      of same-shaped entries -- the common case, fixed-size keys and values -- resolves up to
//      8 entries per LDS round trip; the first lane whose guess breaks the run ends the round
//      with exactly the serial walk's result.  Per entry it writes one u32 record
//      {header pos | stored key bytes before it << 16} (+ a sentinel) into the tile's LDS pool
//      (records 0..63 of each block; later ones go to global scratch).
//   2. scan: the tile's {entries, key bytes, value bytes} are scanned in wave 0, published as a
//      tile aggregate, and the tile's output base comes from a decoupled look-back over the
//      earlier tiles (epoch-tagged granules, p.lb).  The ticket makes every earlier tile already
//      running, so the look-back always progresses.
//   3. copy: wave w takes blocks w, w + 4, ...: groups of 8 lanes per entry move the key and the
//      value as 16-B pieces global -> global (the source lines were streamed in phase 1 a few
//      microseconds earlier: cache hits, not HBM), every piece of a pass loaded before any is
//      stored, and write key_end / val_end / view records.
// LDS holds only the sub-batch being walked and the records, so the time a tile spends on its
// look-back and copy does not pin block bytes in LDS -- the limit that kept the earlier fused
// kernels (tile_decode_kernel, decode_kernel) below walk-scan-copy.
// Blocks with prefix-compressed entries (plen > 0: never written by Builder) are
// copied by a serial per-block path with u32 offsets.
#include <cstdio>
#include <cstdlib>

#include "codec_common.hpp"
#include "decode_common.hpp"
#include "kernels.hpp"

namespace lsmgpu {

namespace {

constexpr uint32_t kFscMaxLen = 4096;              // blocks of this path
constexpr uint32_t kFscSlot = 4128;                // 258 16-B chunks: 4096 B at any 16-B shift
                                                   // + the walk's 12-B header over-read
constexpr uint32_t kFscChunks = kFscSlot / 16;
static_assert(kFscChunks == 258, "two tail chunks past the 256 loaded by the workgroup's threads");
constexpr uint32_t kPoolRec = 64;                  // records per block kept in LDS

__device__ __forceinline__ uint4 load_chunk(const DecodeParams& p, uint64_t a) {
  if (a + 16 <= p.data_len) return *reinterpret_cast<const uint4*>(p.data + a);
  uint4 v = make_uint4(0, 0, 0, 0);  // the chunk crossing the end of the data buffer
  for (int i = 0; i < 16; i++)
    if (a + i < p.data_len) set_byte(v, i, p.data[a + i]);
  return v;
}

// Chunk c (0..257) of block [off, off + len) as it lands in its LDS slot (16-B aligned source,
// shift off & 15); zero past the block's last chunk or for a block outside the data.
__device__ __forceinline__ uint4 block_chunk(const DecodeParams& p, uint32_t off, uint32_t len,
                                             uint32_t c) {
  if (len > kFscMaxLen || (uint64_t)off + len > p.data_len) return make_uint4(0, 0, 0, 0);
  const uint32_t a0 = off & ~15u;
  const uint32_t nch = ((off - a0) + len + 15) >> 4;
  if (c >= nch) return make_uint4(0, 0, 0, 0);
  return load_chunk(p, (uint64_t)a0 + 16ull * c);
}

// Piece q of a `len`-byte stream (copy_piece16's cut): 16-B pieces, the last overlapping back
// inside the stream; below 16 B two overlapping 8/4-B pieces; below 4 B single bytes.
__device__ __forceinline__ uint32_t piece_at(uint32_t len, uint32_t q, uint32_t& sz) {
  if (len >= 16) { sz = 16; return min(16 * q, len - 16); }
  if (len >= 8) { sz = 8; return q ? len - 8 : 0; }
  if (len >= 4) { sz = 4; return q ? len - 4 : 0; }
  sz = 1;
  return q;
}
__device__ __forceinline__ uint4 load_piece(const uint8_t* s, uint32_t sz) {
  uint4 v = make_uint4(0, 0, 0, 0);
  if (sz == 16) __builtin_memcpy(&v, s, 16);
  else if (sz == 8) __builtin_memcpy(&v, s, 8);
  else if (sz == 4) __builtin_memcpy(&v, s, 4);
  else if (sz == 1) v.x = *s;
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

// Entries of one block (plen == 0 throughout): J lanes per entry, G entry groups per pass.
// Records r_i = {header pos | S_i << 16}, S_i = stored key bytes of entries < i, entry n = the
// sentinel {stop pos | S_n << 16}; record i is in the LDS pool for i < 64, in global scratch
// after.  So klen_i = S_{i+1} - S_i, vlen_i = hp_{i+1} - hp_i - 10 - klen_i, and the value
// offset in the block's value stream is hp_i - 10 i - S_i.  `pre` = record min(lane, n).
template <uint32_t J, uint32_t G>
__device__ __forceinline__ void fsc_copy_block(const DecodeParams& p, const uint32_t* pool,
                                               const uint32_t* gm, uint32_t pre,
                                               const uint8_t* blk, uint8_t* kbase, uint8_t* vbase,
                                               uint32_t n, uint64_t en, uint64_t ek, uint64_t ev,
                                               uint32_t off, bool mat, bool view, uint32_t lane) {
  const uint32_t j = lane & (J - 1);
  for (uint32_t e0 = 0; e0 < n; e0 += G * (kWave / J)) {
    uint32_t hp[G], kl[G], vl[G], ko[G], vo[G], np[G], kp[G];
    bool on[G];
    const bool shuffled = e0 + G * (kWave / J) < kWave;
    uint32_t npmax = 0;
#pragma unroll
    for (int i = 0; i < G; i++) {
      const uint32_t e = e0 + i * (kWave / J) + (lane / J);
      const uint32_t ec = min(e, n - 1);
      uint32_t r0, r1;
      if (shuffled) {
        r0 = (uint32_t)__shfl((int)pre, (int)ec);
        r1 = (uint32_t)__shfl((int)pre, (int)ec + 1);
      } else {
        r0 = ec < kPoolRec ? pool[ec] : gm[ec];
        r1 = ec + 1 < kPoolRec ? pool[ec + 1] : gm[ec + 1];
      }
      hp[i] = r0 & 0xffffu;
      ko[i] = r0 >> 16;
      kl[i] = (r1 >> 16) - ko[i];
      vl[i] = (r1 & 0xffffu) - hp[i] - 10 - kl[i];
      vo[i] = hp[i] - 10 * ec - ko[i];
      on[i] = e < n;
      kp[i] = kbase ? pieces16(kl[i]) : 0u;
      np[i] = on[i] ? kp[i] + (vbase ? pieces16(vl[i]) : 0u) : 0u;
      npmax = max(npmax, np[i]);
      if (on[i] && j == 0) {
        if (mat) {
          if (p.key_end) p.key_end[en + e] = (uint32_t)(ek + ko[i] + kl[i]);
          if (p.val_end) p.val_end[en + e] = (uint32_t)(ev + vo[i] + vl[i]);
        }
        if (view)
          p.view[en + e] = (uint64_t)(off + hp[i] + 10) | ((uint64_t)kl[i] << 32) |
                           ((uint64_t)vl[i] << 48);
      }
    }
    if (!mat) continue;
    npmax = wave_max(npmax);
    // every piece of the round is loaded before any is stored (G loads in flight per lane)
    for (uint32_t qb = 0; qb < npmax; qb += J) {
      const uint32_t q = qb + j;
      uint4 v[G];
      uint8_t* d[G];
      uint32_t sz[G];
#pragma unroll
      for (int i = 0; i < G; i++) {
        sz[i] = 0;
        d[i] = nullptr;
        if (q < np[i]) {
          const bool key = q < kp[i];
          const uint32_t o = piece_at(key ? kl[i] : vl[i], key ? q : q - kp[i], sz[i]);
          const uint32_t s0 = hp[i] + 10 + (key ? 0u : kl[i]) + o;
          d[i] = (key ? kbase + ko[i] : vbase + vo[i]) + o;
          v[i] = load_piece(blk + s0, sz[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < G; i++)
        if (sz[i]) store_piece(d[i], v[i], sz[i]);
    }
  }
}

// A block with prefix-compressed entries: the wave replays the walk serially (uniform) from
// global memory with u32 output offsets; key = baseKey[:plen] ++ diff (iterator.go:98-100),
// baseKey = entry 0's key (bytes from block offset 10, as Go's slice of the block).
__device__ void fsc_copy_block_slow(const DecodeParams& p, const uint8_t* blk, uint32_t n,
                                    uint64_t en, uint64_t ek, uint64_t ev, uint32_t off,
                                    bool mat, bool view, uint32_t lane) {
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

}  // namespace

// LSMGPU_STAMPS diagnostics: wave 0's s_memtime cycles per phase, summed over workgroups
#define FSC_STAMP(i)                                                                   \
  if (p.stamps && tid == 0) {                                                          \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();                                  \
    atomicAdd(reinterpret_cast<unsigned long long*>(p.stamps + (i)), t_ - t_prev);     \
    t_prev = t_;                                                                       \
  }

template <uint32_t TILE>
__global__ void __launch_bounds__(256) fsc_kernel(DecodeParams p) {
  constexpr uint32_t SUB = 8;  // one 8-lane walking group per block: wave 0 walks a sub-batch
  static_assert(TILE % SUB == 0 && TILE <= 64, "tile shape");
  __shared__ __attribute__((aligned(16))) uint8_t buf[SUB * kFscSlot];
  __shared__ uint32_t pool[TILE * kPoolRec];
  __shared__ uint32_t s_off[TILE], s_len[TILE];
  __shared__ uint32_t s_n[TILE], s_k[TILE], s_v[TILE], s_st[TILE];
  __shared__ uint32_t s_bn[TILE], s_bk[TILE], s_bv[TILE];  // exclusive output bases
  __shared__ uint64_t s_slow, s_ok;                         // bit per block
  __shared__ uint32_t s_tile;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint32_t ntiles = (p.nblk + TILE - 1) / TILE;
  uint64_t t_prev = p.stamps ? __builtin_amdgcn_s_memtime() : 0;
  if (tid == 0) {
    uint32_t t = blockIdx.x;
    if (!(p.ablate & 8)) {
      t = atomicAdd(p.gcnt, 1u);
      if (t == ntiles - 1) atomicExch(p.gcnt, 0u);  // every ticket is taken
    }
    s_tile = t;
    s_slow = 0;
    s_ok = 0;
  }
  __syncthreads();
  const uint32_t tile = s_tile;
  const uint32_t b0 = tile * TILE;
  const uint32_t nb = min(TILE, p.nblk - b0);
  const uint32_t nsub = (nb + SUB - 1) / SUB;
  if (tid < nb) {
    s_off[tid] = p.blk_off[b0 + tid];
    s_len[tid] = p.blk_len[b0 + tid];
  }
  __syncthreads();
  FSC_STAMP(0)  // ticket + block [off, len)

  // ---- phase 1: stream the sub-batches through LDS, walk each
  uint4 R[SUB], RT;
  auto issue = [&](uint32_t j) {
#pragma unroll
    for (uint32_t i = 0; i < SUB; i++) {
      const uint32_t bi = j * SUB + i;
      R[i] = bi < nb ? block_chunk(p, s_off[bi], s_len[bi], tid) : make_uint4(0, 0, 0, 0);
    }
    const uint32_t ti = j * SUB + (tid >> 1);  // chunks 256, 257 of each block
    RT = (tid < 2 * SUB && ti < nb) ? block_chunk(p, s_off[ti], s_len[ti], 256 + (tid & 1))
                                    : make_uint4(0, 0, 0, 0);
  };
  issue(0);
  uint32_t* const wm = p.wmeta;
  for (uint32_t j = 0; j < nsub; j++) {
    __syncthreads();  // the previous sub-batch's walk is done with buf
    FSC_STAMP(1)      // barrier
#pragma unroll
    for (uint32_t i = 0; i < SUB; i++)
      *reinterpret_cast<uint4*>(buf + i * kFscSlot + 16 * tid) = R[i];
    if (tid < 2 * SUB)
      *reinterpret_cast<uint4*>(buf + (tid >> 1) * kFscSlot + 16 * (256 + (tid & 1))) = RT;
    FSC_STAMP(2)      // load wait + LDS writes
    __syncthreads();
    FSC_STAMP(3)      // barrier
    if (j + 1 < nsub) issue(j + 1);  // in flight while wave 0 walks sub-batch j
    FSC_STAMP(4)      // issue
    if (wave != 0) continue;
    // group g = lane / 8 walks block j * SUB + g; k = lane % 8 is the lane's guess index.
    // Group state (pos, n, S, K, V, the reference entry shape) is identical in its 8 lanes.
    const uint32_t g = lane >> 3, k = lane & 7, gb = lane & ~7u, bi = j * SUB + g;
    const bool has = bi < nb;
    const uint32_t off = has ? s_off[bi] : 0u, len = has ? s_len[bi] : 0u;
    uint32_t n = 0, K = 0, V = 0, S = 0, pos = 0, st = LSMGPU_BLK_OK;
    uint32_t stride = 0, kref = 0xffffffffu, vref = 0xffffffffu;  // no reference yet
    bool any_plen = false, done = !has || (p.ablate & 4);
    if (has && (len > kFscMaxLen || (uint64_t)off + len > p.data_len)) {
      st = LSMGPU_BLK_RANGE;
      done = true;
    }
    uint32_t* const pr = pool + bi * kPoolRec;
    uint32_t* const gr = wm + (uint64_t)(b0 + bi) * p.wcap;
    const LdsSrc src{buf + g * kFscSlot, off & 15u};
    while (!done) {
      // lane k: the entry n + k IF entries n .. n + k - 1 all have the reference shape
      const uint32_t q = pos + k * stride;
      const Hdr h = src.hdr(min(q, len));  // reads stay inside the slot
      const uint32_t end = q + 10 + h.klen + h.vlen;
      const bool eof = q >= len;                                // iterator.go:115-118
      const bool trunc = !eof && len - q < 10;
      const bool term = (h.klen | h.plen) == 0;                 // iterator.go:124-127
      const bool fplen = n + k == 0 && h.plen != 0;             // iterator.go:129-133
      const bool poob = 10 + h.plen > len;                      // base key = entry 0's
      const bool vovf = end > len;                              // iterator.go:101-106
      const bool stop = eof | trunc | term | fplen | poob | vovf;
      const uint32_t code = (eof | (!trunc & term)) ? LSMGPU_BLK_OK
                            : trunc                 ? LSMGPU_BLK_TRUNC_HEADER
                            : fplen                 ? LSMGPU_BLK_FIRST_PLEN
                            : poob                  ? LSMGPU_BLK_PREFIX_OOB
                                                    : LSMGPU_BLK_VALUE_OVERFLOW;
      // e: a real entry of the reference shape, so the next guess (q + stride) is right
      const bool e = !stop && h.plen == 0 && h.klen == kref && h.vlen == vref;
      const uint64_t A = __ballot(e), Vm = __ballot(!stop);
      const uint32_t t = __builtin_ctz(~(uint32_t)((A >> gb) & 0xffu));  // run length, <= 8
      const bool vt = t < 8 && ((Vm >> (gb + t)) & 1);  // entry n + t is real: the run's end
      const uint32_t m = t + (vt ? 1u : 0u);
      if (k < m) {
        const uint32_t rec = q | ((S + k * kref) << 16);  // k < t: shape = reference
        if (n + k < kPoolRec) pr[n + k] = rec;
        else gr[n + k] = rec;
      }
      const uint32_t sl = gb + min(t, 7u);
      const uint32_t hkv = (uint32_t)__shfl((int)(h.klen | (h.vlen << 16)), (int)sl);
      const uint32_t hpc = (uint32_t)__shfl((int)(h.plen | (code << 16)), (int)sl);
      const uint32_t tk = t * kref, tv = t * vref;  // t == 0: 0 whatever the reference
      if (t == 8) {
        pos += 8 * stride;
        n += 8;
        S += tk;
        K += tk;
        V += tv;
      } else if (vt) {  // entry n + t ends the run (another shape): it becomes the reference
        const uint32_t kt = hkv & 0xffffu, vtl = hkv >> 16, pt = hpc & 0xffffu;
        n += t + 1;
        S += tk + kt;
        K += tk + pt + kt;
        V += tv + vtl;
        pos = pos + t * stride + 10 + kt + vtl;
        kref = kt;
        vref = vtl;
        stride = 10 + kt + vtl;
        any_plen = any_plen || pt != 0;
      } else {  // entry n + t stops the iterator (or the block ends there)
        n += t;
        S += tk;
        K += tk;
        V += tv;
        pos = pos + t * stride;
        st = hpc >> 16;
        done = true;
      }
    }
    if (has && k == 0) {
      const uint32_t rec = pos | (S << 16);  // sentinel
      if (n < kPoolRec) pr[n] = rec;
      else gr[n] = rec;
      s_n[bi] = n;
      s_k[bi] = K;
      s_v[bi] = V;
      s_st[bi] = st;
    }
    const uint64_t sm = __ballot(has && k == 0 && any_plen);  // bit 8g per slow block
    if (lane == 0 && sm) {
      uint64_t bits = 0;
      for (uint32_t x = 0; x < SUB; x++) bits |= ((sm >> (8 * x)) & 1ull) << x;
      s_slow |= bits << (j * SUB);
    }
    FSC_STAMP(5)  // walk
    if (p.stamps && tid == 0) atomicAdd(reinterpret_cast<unsigned long long*>(p.stamps + 12), 1ull);
  }
  // records past 63 went to global scratch: complete them before other waves read them
  if (wave == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  FSC_STAMP(6)  // phase-1 tail

  // ---- phase 2: tile scan, look-back, per-block outputs (wave 0: lane = block)
  if (wave == 0) {
    const bool has = lane < nb;
    const uint32_t n = has ? s_n[lane] : 0u, K = has ? s_k[lane] : 0u, V = has ? s_v[lane] : 0u;
    const uint32_t in_ = wave_scan_sat(n, lane), ik = wave_scan_sat(K, lane),
                   iv = wave_scan_sat(V, lane);
    const uint32_t tn = readlane(in_, 63), tk = readlane(ik, 63), tv = readlane(iv, 63);
    uint64_t* Rr = p.lb + (uint64_t)tile * 8;
    Tot ex{0, 0, 0};
    if (tile > 0 && !(p.ablate & 1)) {
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
      ok = (uint64_t)en + n <= p.ent_cap && (uint64_t)en + n <= 0xffffffffull;
      if (p.mode & LSMGPU_MODE_MATERIALIZE) {
        const uint64_t kend = (uint64_t)ek + K, vend = (uint64_t)ev + V;
        ok = ok && (kend <= p.key_cap || !p.key_data) && (vend <= p.val_cap || !p.val_data);
        ok = ok && kend < 0xffffffffull && vend <= 0xffffffffull;
      }
      if (!ok) atomicOr(reinterpret_cast<unsigned long long*>(p.result + 5), 1ull);
    }
    const uint64_t okm = __ballot(ok);
    if (lane == 0) s_ok = okm;
  }
  __syncthreads();
  FSC_STAMP(7)  // scan + look-back + per-block outputs
  if (p.ablate & 2) return;

  // ---- phase 3: copy, one wave per block
  const bool mat = (p.mode & LSMGPU_MODE_MATERIALIZE) != 0;
  const bool view = (p.mode & LSMGPU_MODE_VIEW) != 0 && p.view;
  if (!mat && !view) return;
  const uint64_t okm = s_ok, slowm = s_slow;
  for (uint32_t bi = wave; bi < nb; bi += 4) {
    const uint32_t n = uniform(s_n[bi]);
    if (n == 0 || !((okm >> bi) & 1)) continue;
    const uint64_t en = uniform(s_bn[bi]), ek = uniform(s_bk[bi]), ev = uniform(s_bv[bi]);
    const uint32_t off = uniform(s_off[bi]);
    const uint8_t* blk = p.data + off;
    if ((slowm >> bi) & 1) {
      fsc_copy_block_slow(p, blk, n, en, ek, ev, off, mat, view, lane);
      continue;
    }
    const uint32_t* pr = pool + bi * kPoolRec;
    const uint32_t* gr = wm + (uint64_t)(b0 + bi) * p.wcap;
    const uint32_t pre = pr[min(lane, n)];  // records 0..63 are in the pool
    uint8_t* kbase = (mat && p.key_data) ? p.key_data + ek : nullptr;
    uint8_t* vbase = (mat && p.val_data) ? p.val_data + ev : nullptr;
    fsc_copy_block<8, 5>(p, pr, gr, pre, blk, kbase, vbase, n, en, ek, ev, off, mat, view, lane);
  }
  FSC_STAMP(8)  // copy (wave 0's blocks)
  if (p.stamps && tid == 0) atomicAdd(reinterpret_cast<unsigned long long*>(p.stamps + 13), 1ull);
}

hipError_t launch_decode_fsc(const DecodeParams& p, hipStream_t s) {
  constexpr uint32_t TILE = 32;
  const uint32_t ntiles = (p.nblk + TILE - 1) / TILE;
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
  hipLaunchKernelGGL((fsc_kernel<TILE>), dim3(ntiles), dim3(256), 0, s, q);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && q.stamps) {
    uint64_t h[16] = {0};
    (void)hipMemcpyAsync(h, stamps, sizeof(h), hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    const double it = h[12] ? (double)h[12] : 1.0, tl = h[13] ? (double)h[13] : 1.0;
    fprintf(stderr, "[lsmgpu] fsc stamps per sub-batch (cycles): barrier %.0f ldswait+write %.0f "
            "barrier2 %.0f issue %.0f walk %.0f | per tile: start %.0f p1tail %.0f scan+lookback %.0f "
            "copy %.0f | sub-batches %llu tiles %llu\n", h[1] / it, h[2] / it, h[3] / it, h[4] / it,
            h[5] / it, h[0] / tl, h[6] / tl, h[7] / tl, h[8] / tl, (unsigned long long)h[12],
            (unsigned long long)h[13]);
  }
  return e;
}

}  // namespace lsmgpu
