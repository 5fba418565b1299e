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

// ---- streaming walk (blocks <= 4 KiB): the tile's blocks pass through LDS kSwSub at a time
constexpr uint32_t kSwSub = 8;       // blocks per LDS sub-batch
constexpr uint32_t kSwSlot = 4128;   // a <= 4096-B block at any 16-B shift + the 8-B header
                                     // over-read, as 258 16-B chunks
constexpr uint32_t kSwMaxLen = 4096;
constexpr uint32_t kSwTile = 256;    // blocks per streaming-walk tile (64-block tiles: slower)

__device__ __forceinline__ uint4 sw_chunk(const DecodeParams& p, uint32_t off, uint32_t len,
                                          uint32_t c) {
  // chunk c of block [off, off + len)'s 16-B aligned span; zero past it or past the data
  if (len > kSwMaxLen || (uint64_t)off + len > p.data_len) return make_uint4(0, 0, 0, 0);
  const uint32_t a0 = off & ~15u;
  if (c >= (((off - a0) + len + 15) >> 4)) return make_uint4(0, 0, 0, 0);
  const uint64_t a = (uint64_t)a0 + 16ull * c;
  if (a + 16 <= p.data_len) return *reinterpret_cast<const uint4*>(p.data + a);
  uint4 v = make_uint4(0, 0, 0, 0);  // the line crossing the end of the data buffer
  for (int i = 0; i < 16; i++)
    if (a + i < p.data_len) set_byte(v, i, p.data[a + i]);
  return v;
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

// ---- scan walk (blocks <= 4 KiB): the header chain found by a data-parallel scan, not walked
//
// The serial chain pos -> pos + 10 + klen + vlen (iterator.go:93-135) is replaced by a test every
// byte position can run on its own.  Every header Builder writes has plen == 0 (keyDiff returns
// the whole key) and a back-pointer `prev` = the previous header's block offset
// (builder.go:103-109; the terminator's prev is the last entry), which in a block < 64 KiB has
// two zero high bytes -- except the first header's, 0xffffffff.  So a position q > 0 is a
// CANDIDATE when bytes q, q+1, q+6, q+7 are zero (q = 0 when q, q+1 are), and it is ACCEPTED
// when its successor end(q) = q + 10 + klen + vlen either closes the block (end == len; for
// klen == 0, a terminator, only that) or holds a header whose prev == q.
//
// The test is only a filter; exactness comes from VERIFYING that the accepted positions, in
// order, are the iterator's chain: the first is 0, each non-last one is an entry whose end is
// the next, no terminator before the last, and the last ends at len.  Then the iterator,
// started at 0, visits exactly these positions and stops after the last with status OK (every
// entry has plen == 0, end <= len, and its header fits).  Any other block -- a false positive
// (bytes inside a value that look like a chained header), plen > 0, an error status, no
// terminator -- fails verification and takes the serial walk (walk_meta) from global memory.
// Both produce the same records, so the copy kernel cannot tell them apart.
//
// Cost model (measured with SQ_INSTS_VALU): a wave64 VALU instruction holds a 16-lane SIMD for
// 4 cycles, so a CU retires ~1 wave-instruction per cycle and HBM delivers a 4 KiB block per
// ~420 CU cycles: the scan must stay well under ~400 wave-instructions per block.  Hence the
// byte tests are OR-combined before one zero-byte test per dword, and flags are gathered in a
// permuted bit order (2 instructions per dword); order is restored by the positional pass 2.
constexpr uint32_t kNoPos = 0xffffffffu;

// Candidate flags of a lane's 64-B LDS window, in PERMUTED order: bit 32m + 8j + k is window
// position o = 32m + 4k + j (m < 2, k < 8, j < 4).  20 dwords: the window + 16 B of the next.
__device__ __forceinline__ uint64_t header_candidates(const uint8_t* win) {
  const uint4* w4 = reinterpret_cast<const uint4*>(win);
  uint32_t w[20];
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const uint4 v = w4[i];
    w[4 * i] = v.x;
    w[4 * i + 1] = v.y;
    w[4 * i + 2] = v.z;
    w[4 * i + 3] = v.w;
  }
  uint32_t t[18];  // byte j of t[d]: window bytes 4d + j | 4d + j + 1
#pragma unroll
  for (int d = 0; d < 18; d++) t[d] = w[d] | __builtin_amdgcn_alignbyte(w[d + 1], w[d], 1);
  uint32_t acc[2] = {0, 0};
#pragma unroll
  for (int d = 0; d < 16; d++) {
    // byte j: bytes o, o+1, o+6, o+7 OR-ed (o = 4d + j); bit 7 of y's byte j set iff non-zero
    const uint32_t v = t[d] | __builtin_amdgcn_alignbyte(t[d + 2], t[d + 1], 2);
    const uint32_t y = ((v & 0x7f7f7f7fu) + 0x7f7f7f7fu) | v;
    acc[d >> 3] = (acc[d >> 3] >> 1) | (y & 0x80808080u);  // dword 8m + k -> bits 8j + k
  }
  return ~(((uint64_t)acc[1] << 32) | acc[0]);  // zero flags
}

// klen (low 16) and vlen (high 16) of the header at LDS byte p
__device__ __forceinline__ void scan_kv(const uint8_t* slot, uint32_t p, uint32_t& klen,
                                        uint32_t& vlen) {
  const uint32_t x = lds_u32(slot, p + 2);
  klen = __builtin_amdgcn_perm(0u, x, 0x0c0c0001u);
  vlen = __builtin_amdgcn_perm(0u, x, 0x0c0c0203u);
}

// One block in the wave's LDS slot (byte 0 at slot + sh, len <= 4096; the slot holds 4128 B).
// Writes the same records as walk_meta; the result is valid in lane 0.
__device__ WalkResult scan_block(const uint8_t* slot, uint32_t sh, uint32_t len,
                                 const uint8_t* gblk, uint2* meta, uint32_t lane) {
  const int base = 64 * (int)lane - (int)sh;  // block position of the lane's window byte 0
  // pass 1 (any order): accept candidates; per lane: positional mask, count / key / value sums,
  // the lowest accepted position and the end of the highest, the terminator (if any)
  uint64_t cand = len >= 10 ? header_candidates(slot + 64 * lane) : 0ull;
  uint64_t acc = 0;
  uint32_t c = 0, Ks = 0, Vs = 0, lo_q = kNoPos, hi_q = 0, hi_end = kNoPos, tq = kNoPos;
  auto accept = [&](uint32_t q, uint32_t o) {
    uint32_t klen, vlen;
    scan_kv(slot, sh + q, klen, vlen);
    const uint32_t end = q + 10 + klen + vlen;
    const bool succ = end + 10 <= len;  // a successor header fits: its prev must point back
    const uint32_t prev = bswap32(lds_u32(slot, sh + (succ ? end + 6 : 0u)));  // (clamped read)
    // a terminator (finishBlock) closing the block; the block's last entry (no terminator); an
    // entry whose successor's prev points back
    const bool a = klen == 0 ? end == len : (end == len || (succ && prev == q));
    if (!a) return;
    acc |= 1ull << o;
    lo_q = min(lo_q, q);
    if (hi_end == kNoPos || q > hi_q) {
      hi_q = q;
      hi_end = end;
    }
    if (klen == 0) {
      tq = q;
    } else {
      c++;
      Ks += klen;
      Vs += vlen;
    }
  };
  if (lane == 0 && len >= 10 && (lds_u32(slot, sh) & 0xffffu) == 0) accept(0, sh);  // q = 0
  while (cand) {
    const uint32_t bit = (uint32_t)__builtin_ctzll(cand);
    cand &= cand - 1;
    const uint32_t o = (bit & 32u) + 4 * (bit & 7u) + ((bit >> 3) & 3u);
    const int qi = base + (int)o;
    if (qi <= 0 || (uint32_t)qi + 10 > len) continue;  // outside the block (q = 0: above)
    accept((uint32_t)qi, o);
  }
  // entries (<= 409) and key bytes (<= 4096) share one scan: c | Ks << 16 cannot carry over
  const uint32_t ick = wave_scan_sat(c | (Ks << 16), lane), iv = wave_scan_sat(Vs, lane);
  const uint32_t ic = ick & 0xffffu, ik = ick >> 16;
  const uint32_t n = readlane(ic, 63), K = readlane(ik, 63), V = readlane(iv, 63);
  // pass 2 (positional): the lane's records, and its chain -- each accepted position is the
  // previous one's end, nothing after a terminator
  uint32_t idx = ic - c, kr = ik - Ks, vr = iv - Vs, last_end = kNoPos;
  bool ok = true;
  for (uint64_t a = acc; a;) {
    const uint32_t o = (uint32_t)__builtin_ctzll(a);
    a &= a - 1;
    const uint32_t q = (uint32_t)(base + (int)o);
    uint32_t klen, vlen;
    scan_kv(slot, sh + q, klen, vlen);
    ok = ok && (last_end == kNoPos || last_end == q);
    if (klen == 0) {  // the terminator: the lane's last accepted position
      ok = ok && a == 0;
      break;
    }
    last_end = q + 10 + klen + vlen;
    meta[idx] = make_uint2(q | (vr << 16), kr);
    kr += klen;
    vr += vlen;
    idx++;
  }
  // across lanes: each non-empty lane's last end is the next non-empty lane's first position
  // (len for the last one); the lowest non-empty lane starts at 0
  const bool ne = acc != 0;
  const uint64_t neb = __ballot(ne);
  const uint64_t later = lane == 63 ? 0ull : neb >> (lane + 1);
  const uint32_t nl = later ? lane + 1 + (uint32_t)__builtin_ctzll(later) : lane;
  const uint32_t nextf = (uint32_t)__shfl((int)lo_q, (int)nl);
  const bool bad = ne && (!ok || hi_end != (later ? nextf : len));
  const bool good = neb != 0 && __ballot(bad) == 0 && readlane(lo_q, 0) == 0;
  if (!good) {  // serial walk: every stop rule in the iterator's order (rewrites every record)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // pass 2's stores land first
    WalkResult r{0, 0, 0, LSMGPU_BLK_OK};
    if (lane == 0) r = walk_meta(GlobalSrc{gblk}, nullptr, len, meta);
    return r;
  }
  const uint64_t tb = __ballot(tq != kNoPos);
  const uint32_t stop = tb ? readlane(tq, (uint32_t)__builtin_ctzll(tb)) : len;
  if (lane == 0) meta[n] = make_uint2(stop | (V << 16), K);  // sentinel
  return WalkResult{n, K, V, LSMGPU_BLK_OK};
}

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
// MODE kWalkStream (p.wwalk, blocks <= 4 KiB): the tile's blocks go through LDS kSwSub at a time,
// every thread loading one 16-B chunk of each block of the NEXT sub-batch (coalesced, 1 KiB per
// wave instruction) while wave 0 walks the current one from LDS, one lane per block.  An LDS
// walk costs ~210 cycles per entry in latency whatever the number of lanes walking
// (scripts/walk_probe.hip), so it pays when many blocks walk at once and nothing else holds the
// bytes in LDS -- as here, where the copy is a separate launch.
template <int MODE, uint32_t TB>  // TB = blocks per tile (<= 256 threads: thread t owns block t)
__global__ void __launch_bounds__(256) wsc_walk_kernel(DecodeParams p) {
  static_assert(TB <= 256, "one thread per block of the tile");
  constexpr bool STREAM = MODE == kWalkStream;
  constexpr bool SCAN = MODE == kWalkScan;
  constexpr uint32_t kStageBytes = 256 * kWalkStage * sizeof(uint2);
  // group walk: a 32-record ring per block (its LDS also serves the view epilogue's owner map);
  // scan walk: one block slot per wave
  constexpr uint32_t kLdsBytes = STREAM ? kSwSub * kSwSlot
                                 : SCAN ? 4 * kSwSlot
                                 : MODE == kWalkGroup ? TB * 16 * sizeof(uint2) : kStageBytes;
  static_assert(MODE != kWalkLane || kLdsBytes == kStageBytes,
                "the lane walk stages 16 records per lane");
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
  uint2* const stage = reinterpret_cast<uint2*>(lds);
  __shared__ uint32_t s_tile;
  __shared__ uint32_t s_wave[4][3];
  __shared__ uint32_t s_ex[3];
  __shared__ uint32_t s_first[257];  // p.wfuse: tile-relative first entry of each block
  __shared__ uint32_t s_off[MODE == kWalkGroup || SCAN ? TB : 256];  // each block's input offset
  __shared__ uint32_t s_len[STREAM ? 256 : SCAN ? TB : 1];
  constexpr uint32_t kRes = MODE == kWalkLane ? 1 : MODE == kWalkGroup || SCAN ? TB : 256;
  __shared__ uint32_t s_res[4][kRes];  // stream / group walk: n, K, V, status per block
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint32_t ntiles = (p.nblk + TB - 1) / TB;
  if (tid == 0) {
    const uint32_t t = atomicAdd(p.gcnt, 1u);
    if (t == ntiles - 1) atomicExch(p.gcnt, 0u);  // every ticket is taken
    s_tile = t;
  }
  __syncthreads();
  const uint32_t tile = s_tile;
  // thread t owns block tile * TB + t (threads past TB own none: zero entries)
  const uint32_t b = tid < TB ? tile * TB + tid : 0xffffffffu;
  uint32_t n = 0, K = 0, V = 0, st = LSMGPU_BLK_OK;
  if constexpr (STREAM) {
    const uint32_t nb = min(TB, p.nblk - tile * TB);
    const uint32_t nsub = (nb + kSwSub - 1) / kSwSub;
    if (b < p.nblk) {
      s_off[tid] = p.blk_off[b];
      s_len[tid] = p.blk_len[b];
    }
    __syncthreads();
    uint4 R[kSwSub], RT;
    auto issue = [&](uint32_t j) {
#pragma unroll
      for (uint32_t i = 0; i < kSwSub; i++) {
        const uint32_t bi = j * kSwSub + i;
        R[i] = bi < nb ? sw_chunk(p, s_off[bi], s_len[bi], tid) : make_uint4(0, 0, 0, 0);
      }
      const uint32_t ti = j * kSwSub + (tid >> 1);  // chunks 256, 257 of each block
      RT = (tid < 2 * kSwSub && ti < nb) ? sw_chunk(p, s_off[ti], s_len[ti], 256 + (tid & 1))
                                         : make_uint4(0, 0, 0, 0);
    };
    issue(0);
    for (uint32_t j = 0; j < nsub; j++) {
      __syncthreads();  // the previous sub-batch's walk is done with the buffer
#pragma unroll
      for (uint32_t i = 0; i < kSwSub; i++)
        *reinterpret_cast<uint4*>(lds + i * kSwSlot + 16 * tid) = R[i];
      if (tid < 2 * kSwSub)
        *reinterpret_cast<uint4*>(lds + (tid >> 1) * kSwSlot + 16 * (256 + (tid & 1))) = RT;
      __syncthreads();
      if (j + 1 < nsub) issue(j + 1);  // in flight while wave 0 walks sub-batch j
      const uint32_t bi = j * kSwSub + lane;
      if (wave == 0 && lane < kSwSub && bi < nb) {
        const uint32_t off = s_off[bi], len = s_len[bi];
        uint2* meta = reinterpret_cast<uint2*>(p.wmeta) + (uint64_t)(tile * TB + bi) * p.wcap;
        WalkResult r{0, 0, 0, LSMGPU_BLK_RANGE};
        if ((uint64_t)off + len > p.data_len) {
          meta[0] = make_uint2(0, 0);
        } else if (p.ablate & 4) {  // timing only: no walk
          r = WalkResult{0, 0, 0, LSMGPU_BLK_OK};
          meta[0] = make_uint2(0, 0);
        } else if (len > kSwMaxLen) {  // only if the caller's max_blk_len was wrong: global walk
          r = walk_meta(GlobalSrc{p.data + off}, nullptr, len, meta);
        } else {
          const uint8_t* slot = lds + lane * kSwSlot;
          r = walk_meta(LdsSrc{slot, off & 15u}, slot + (off & 15u), len, meta);
        }
        s_res[0][bi] = r.n;
        s_res[1][bi] = r.K;
        s_res[2][bi] = r.V;
        s_res[3][bi] = r.status;
      }
    }
    // the records are global stores of wave 0: complete before other waves read them
    if (wave == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
          kref = shape & 0xffffu;
          vref = shape >> 16;
          stride = 10 + kref + vref;
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
  } else if constexpr (SCAN) {
    // wave w takes the tile's blocks [w * TB / 4, (w + 1) * TB / 4) one after another: block i's
    // 16-B aligned lines go into the wave's LDS slot (coalesced, 1 KiB per wave instruction),
    // block i + 1's loads are issued into registers, then block i is scanned (scan_block)
    constexpr uint32_t PW = TB / 4;
    static_assert(TB % 4 == 0, "four waves share the tile");
    if (b < p.nblk) {
      s_off[tid] = p.blk_off[b];
      s_len[tid] = p.blk_len[b];
    }
    __syncthreads();
    static_assert(PW <= 64, "a wave's blocks: one [off, len) per lane");
    const uint32_t nb = min(TB, p.nblk - tile * TB);
    const uint32_t i0 = wave * PW, i1 = min(i0 + PW, nb);
    uint8_t* const slot = lds + wave * kSwSlot;
    // lane i holds block i0 + i's [off, len): a block's values are one v_readlane away
    const uint32_t w_off = i0 + lane < i1 ? s_off[i0 + lane] : 0u;
    const uint32_t w_len = i0 + lane < i1 ? s_len[i0 + lane] : 0u;
    // two blocks' loads in flight while a third is scanned (one in flight left the wave
    // waiting on HBM latency after every block)
    uint4 R0[4], R1[4], RT0 = make_uint4(0, 0, 0, 0), RT1 = make_uint4(0, 0, 0, 0);
    auto issue = [&](uint32_t bi, uint4 (&R)[4], uint4& RT) {
      const uint32_t off = readlane(w_off, bi - i0), len = readlane(w_len, bi - i0);
      const uint64_t a0 = off & ~15ull;
      if (len <= kSwMaxLen && a0 + kSwSlot <= p.data_len) {  // uniform: no per-chunk checks
        const uint4* src = reinterpret_cast<const uint4*>(p.data + a0);
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) R[i] = src[lane + 64 * i];
        if (lane < 2) RT = src[256 + lane];
      } else {  // the buffer's last lines (or an oversize block: zeros)
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) R[i] = sw_chunk(p, off, len, lane + 64 * i);
        if (lane < 2) RT = sw_chunk(p, off, len, 256 + lane);
      }
    };
    auto scan_one = [&](uint32_t bi, uint4 (&R)[4], uint4& RT) {
      wave_lds_fence();  // the previous block's reads are done with the slot
#pragma unroll
      for (uint32_t i = 0; i < 4; i++) *reinterpret_cast<uint4*>(slot + 16 * (lane + 64 * i)) = R[i];
      if (lane < 2) *reinterpret_cast<uint4*>(slot + 16 * (256 + lane)) = RT;
      wave_lds_fence();
      if (bi + 2 < i1) issue(bi + 2, R, RT);  // in flight while blocks bi, bi + 1 are scanned
      const uint32_t off = readlane(w_off, bi - i0), len = readlane(w_len, bi - i0);
      uint2* meta = reinterpret_cast<uint2*>(p.wmeta) + (uint64_t)(tile * TB + bi) * p.wcap;
      WalkResult r{0, 0, 0, LSMGPU_BLK_RANGE};
      if ((uint64_t)off + len > p.data_len) {
        if (lane == 0) meta[0] = make_uint2(0, 0);
      } else if (len > kSwMaxLen) {  // only if the caller's max_blk_len was wrong: global walk
        if (lane == 0) r = walk_meta(GlobalSrc{p.data + off}, nullptr, len, meta);
      } else if (p.ablate & 4) {  // timing only: loads, no scan
        r = WalkResult{0, 0, 0, LSMGPU_BLK_OK};
        if (lane == 0) meta[0] = make_uint2(0, 0);
      } else {
        r = scan_block(slot, off & 15u, len, p.data + off, meta, lane);
      }
      if (lane == 0) {
        s_res[0][bi] = r.n;
        s_res[1][bi] = r.K;
        s_res[2][bi] = r.V;
        s_res[3][bi] = r.status;
      }
    };
    if (i0 < i1) issue(i0, R0, RT0);
    if (i0 + 1 < i1) issue(i0 + 1, R1, RT1);
    for (uint32_t bi = i0; bi < i1; bi += 2) {
      scan_one(bi, R0, RT0);
      if (bi + 1 < i1) scan_one(bi + 1, R1, RT1);
    }
    // the records are global stores of every wave: complete before the epilogue reads them
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
    if (tile > 0) {
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
    if (!p.wfuse) {
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
  // (u8 slots for the scan walk, whose LDS is smaller: 256 blocks still fit a byte)
  using Owner = typename std::conditional<SCAN, uint8_t, uint16_t>::type;
  Owner* owner = reinterpret_cast<Owner*>(stage);
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

// K2: one wave per block (p.wsplit waves above 8 KiB).
__global__ void __launch_bounds__(256) wsc_copy_kernel(DecodeParams p) {
  const uint32_t lane = lane_id();
  // p.wsplit waves share a block (large blocks): wave `sub` takes passes sub, sub + wsplit, ...
  const uint32_t wave = threadIdx.x >> 6, split = p.wsplit;
  const uint32_t sub = wave % split;
  const uint32_t b = uniform(blockIdx.x * (4 / split) + wave / split);
  if (b >= p.nblk) return;
  const uint2* meta = reinterpret_cast<const uint2*>(p.wmeta) + (uint64_t)b * p.wcap;
  // the first 64 metadata records, one per lane, requested beside the per-block loads below
  // (one round trip fewer before the piece loads; records past the sentinel are never used)
  const uint2 pre = meta[min(lane, p.wcap - 1)];
  const uint64_t* t = p.wstat + 3ull * b;
  const uint32_t n = uniform((uint32_t)t[0]), K = uniform((uint32_t)t[1]),
                 V = uniform((uint32_t)t[2]);
  const uint32_t st = uniform(p.wstatus[b]);
  const uint64_t* bs = p.wbase + 3ull * b;
  const uint64_t en = uniform64(bs[0]), ek = uniform64(bs[1]), ev = uniform64(bs[2]);
  const uint32_t off = uniform(p.blk_off[b]);
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


// ======================================================================= fused tile decode
// Blocks <= 4 KiB in ONE launch that reads the input once.  A one-wave workgroup takes the
// next tile of T consecutive blocks from an ordered ticket, LDS-DMAs them (coalesced, no
// VGPRs), walks each block serially from LDS with one lane per block (the same chain as
// wsc_walk_kernel, at LDS latency), publishes the tile's {entries, key bytes, value bytes},
// finds its output base by decoupled look-back over the tile records, and copies the entries
// global -> global as wsc_copy_kernel does (the source lines were just fetched: L2 hits).
// The ticket gives predecessor tiles a head start, so the look-back never waits on a tile
// that has not been scheduled.  LDS per tile: T * (4128 B slot + 410 x 8 B entry metadata).
constexpr uint32_t kTileSlot = 4128;  // a <= 4096-B block at any 16-B shift + the tail chunk
constexpr uint32_t kTileCap = 410;    // 409 entries of >= 10 B in 4096 B, + the sentinel

template <int T>
__global__ void __launch_bounds__(64) tile_decode_kernel(DecodeParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t slots[T * kTileSlot];
  __shared__ uint2 meta[T * kTileCap];  // {header pos | value offset << 16, key offset}
  const uint32_t lane = lane_id();
  const uint32_t ntiles = (p.nblk + T - 1) / T;
  uint32_t t = blockIdx.x;
  if (!(p.ablate & 64)) {
    if (lane == 0) t = atomicAdd(p.gcnt, 1u);
    t = readlane(t, 0);
    if (t == ntiles - 1 && lane == 0) atomicExch(p.gcnt, 0u);  // every ticket is taken
  }
  if (t >= ntiles) return;
  const uint64_t tag = p.tag;
  const uint32_t b0 = t * T;
  const uint32_t nb = min((uint32_t)T, p.nblk - b0);

  // stage the tile: block i -> slots + i * kTileSlot (16-B aligned source, shift sh)
  // every block's [off, len) in one round trip, then all DMAs back to back
  uint32_t lo = 0, ll = 0;
  if (lane < nb) {
    lo = p.blk_off[b0 + lane];
    ll = p.blk_len[b0 + lane];
  }
  BlockRef ref[T];
#pragma unroll
  for (int i = 0; i < T; i++) {
    ref[i] = BlockRef{0, 0, 0, false, false};
    if ((uint32_t)i < nb)
      ref[i] = prefetch_block<4096, 5>(p, readlane(lo, i), readlane(ll, i), slots + i * kTileSlot,
                                       lane);
  }
#pragma unroll
  for (int i = 0; i < T; i++)
    if (ref[i].fits && ref[i].tail) land_tail(p, ref[i], slots + i * kTileSlot, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  wave_lds_fence();

  // walk: lane i < nb walks block i (table/iterator.go:93-135)
  uint32_t n = 0, K = 0, V = 0, st = LSMGPU_BLK_OK;
  bool any_plen = false;
  if (lane < nb && !(p.ablate & 4)) {
    uint32_t len = 0, sh = 0;
    bool fits = false;
#pragma unroll
    for (int i = 0; i < T; i++)
      if (lane == (uint32_t)i) {
        len = ref[i].len;
        sh = ref[i].sh;
        fits = ref[i].fits;
      }
    uint2* m = meta + lane * kTileCap;
    if (!fits) {
      st = LSMGPU_BLK_RANGE;  // off + len past the data (len <= 4096 on this path)
    } else {
      // one LDS round trip and one branch per entry: the header is read before the bounds
      // checks (pos <= len keeps the read inside the slot), every stop condition of
      // table/iterator.go:93-135 is evaluated at once and resolved in iterator order
      const LdsSrc src{slots + lane * kTileSlot, sh};
      uint32_t pos = 0;
      for (;;) {
        const Hdr h = src.hdr(pos);
        const uint32_t end = pos + 10 + h.klen + h.vlen;
        const bool eof = pos >= len;                              // iterator.go:115-118
        const bool trunc = len - pos < 10;
        const bool term = (h.klen | h.plen) == 0;                 // iterator.go:124-127
        const bool fplen = n == 0 && h.plen != 0;                 // iterator.go:129-133
        const bool poob = 10 + h.plen > len;                      // base key = entry 0's key
        const bool vovf = end > len;                              // iterator.go:101-106
        if (eof | trunc | term | fplen | poob | vovf) {
          st = (eof | (!trunc & term)) ? LSMGPU_BLK_OK
               : trunc                 ? LSMGPU_BLK_TRUNC_HEADER
               : fplen                 ? LSMGPU_BLK_FIRST_PLEN
               : poob                  ? LSMGPU_BLK_PREFIX_OOB
                                       : LSMGPU_BLK_VALUE_OVERFLOW;
          break;
        }
        m[n] = make_uint2(pos | (V << 16), K);
        any_plen = any_plen || h.plen != 0;
        K += h.plen + h.klen;
        V += h.vlen;
        n++;
        pos = end;
      }
    }
    m[n] = make_uint2(V << 16, K);  // sentinel: the block's key / value totals
  }
  wave_lds_fence();
  const bool has_plen = __ballot(any_plen) != 0;

  // tile totals, per-block exclusive offsets inside the tile, output base by look-back
  const uint32_t in_ = wave_scan_sat(lane < nb ? n : 0u, lane);
  const uint32_t ik = wave_scan_sat(lane < nb ? K : 0u, lane);
  const uint32_t iv = wave_scan_sat(lane < nb ? V : 0u, lane);
  const uint32_t nt = readlane(in_, nb - 1), kt = readlane(ik, nb - 1), vt = readlane(iv, nb - 1);
  // Two-level prefix: every tile publishes its aggregate; the last tile of each group of 64
  // sums the group and looks back over GROUP records (64 groups = 4096 tiles per poll), the
  // other members add their in-group predecessors' aggregates to the previous group's
  // inclusive prefix.  (A flat per-tile look-back advances only ~64 tiles per round trip.)
  store3(p.lb + (uint64_t)t * 8, tag, nt, kt, vt, lane);
  const uint32_t g = t >> 6, g0 = g << 6;
  const uint32_t gsize = min(64u, ntiles - g0);
  const uint32_t before = t - g0;  // in-group predecessors
  Tot in{0, 0, 0};
  if (before && !(p.ablate & 1)) {
    uint32_t a = 0, b = 0, c = 0;
    for (SpinBound bound;;) {
      bool ok = true;
      if (lane < before) ok = read3(p.lb + (uint64_t)(g0 + lane) * 8, tag, a, b, c);
      if (__all(ok)) break;
      if (bound.expired()) {
        flag_timeout(p.result, lane);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    in = Tot{wave_sum_sat(lane < before ? a : 0u), wave_sum_sat(lane < before ? b : 0u),
             wave_sum_sat(lane < before ? c : 0u)};
  }
  Tot gx{0, 0, 0};  // exclusive prefix of group g
  if (p.ablate & 1) {
    // timing only: no prefix
  } else if (t == g0 + gsize - 1) {  // group leader
    const uint32_t ga = sat_add(in.n, nt), gb = sat_add(in.k, kt), gc = sat_add(in.v, vt);
    uint64_t* Gr = p.glb + (uint64_t)g * 8;
    if (g > 0) {
      store3(Gr, tag, ga, gb, gc, lane);
      gx = lookback(p.glb, g, tag, lane, p.result);
    }
    store3(Gr + 4, tag, sat_add(gx.n, ga), sat_add(gx.k, gb), sat_add(gx.v, gc), lane);
  } else if (g > 0) {
    const uint64_t* Gp = p.glb + (uint64_t)(g - 1) * 8 + 4;
    for (SpinBound bound;;) {
      if (read3(Gp, tag, gx.n, gx.k, gx.v)) break;
      if (bound.expired()) {
        flag_timeout(p.result, lane);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  const Tot ex{sat_add(gx.n, in.n), sat_add(gx.k, in.k), sat_add(gx.v, in.v)};
  const uint64_t en = ex.n, ek = ex.k, ev = ex.v;

  if (lane < nb) {
    const uint32_t b = b0 + lane;
    if (p.blk_first) p.blk_first[b] = (uint32_t)(en + in_ - n);
    if (p.blk_status) p.blk_status[b] = (int32_t)st;
    if (st != LSMGPU_BLK_OK) {
      atomicAdd(reinterpret_cast<unsigned long long*>(p.result + 4), 1ull);
      atomicMax(reinterpret_cast<unsigned long long*>(p.result + 3),
                (unsigned long long)(p.nblk - b));
    }
  }
  if (t == ntiles - 1 && lane == 0) {  // totals of the whole batch
    if (p.blk_first) p.blk_first[p.nblk] = (uint32_t)(en + nt);
    p.result[0] = en + nt;
    p.result[1] = ek + kt;
    p.result[2] = ev + vt;
  }
  const bool mat = (p.mode & LSMGPU_MODE_MATERIALIZE) != 0;
  const bool view = (p.mode & LSMGPU_MODE_VIEW) != 0 && p.view;
  bool ok = en + nt <= p.ent_cap && en + nt <= 0xffffffffull;
  if (mat) {
    const uint64_t kend = ek + kt, vend = ev + vt;
    ok = ok && (kend <= p.key_cap || !p.key_data) && (vend <= p.val_cap || !p.val_data);
    ok = ok && kend < 0xffffffffull && vend <= 0xffffffffull;
  }
  if (!ok) {
    if (lane == 0) atomicOr(reinterpret_cast<unsigned long long*>(p.result + 5), 1ull);
    return;
  }
  if (nt == 0 || (p.ablate & 2)) return;

  // per-block constants of the tile (uniform): first entry, key / value offsets, source
  uint32_t fb[T], kb[T], vb[T], bo[T], bsh[T];
#pragma unroll
  for (int i = 0; i < T; i++) {
    fb[i] = (uint32_t)i < nb ? readlane(in_ - n, i) : 0xffffffffu;
    kb[i] = readlane(ik - K, i);
    vb[i] = readlane(iv - V, i);
    bo[i] = ref[i].off;
    bsh[i] = ref[i].sh;
  }
  uint8_t* kbase = p.key_data ? p.key_data + ek : nullptr;
  uint8_t* vbase = p.val_data ? p.val_data + ev : nullptr;
  constexpr uint32_t J = 8, G = 4;
  const uint32_t j = lane & (J - 1);
  for (uint32_t e0 = 0; e0 < nt; e0 += G * (kWave / J)) {
    uint32_t kl[G], ks[G], vl[G], ko[G], vo[G], np[G], kp[G], src[G];
    bool on[G];
#pragma unroll
    for (int i = 0; i < G; i++) {
      const uint32_t e = e0 + i * (kWave / J) + (lane >> 3);
      const uint32_t ec = min(e, nt - 1);
      uint32_t blk = 0;
#pragma unroll
      for (int q = 1; q < T; q++) blk += ec >= fb[q] ? 1u : 0u;
      uint32_t f = fb[0], kx = kb[0], vx = vb[0], o = bo[0], shb = bsh[0];
#pragma unroll
      for (int q = 1; q < T; q++)
        if (blk == (uint32_t)q) {
          f = fb[q];
          kx = kb[q];
          vx = vb[q];
          o = bo[q];
          shb = bsh[q];
        }
      const uint2 m0 = meta[blk * kTileCap + ec - f], m1 = meta[blk * kTileCap + ec - f + 1];
      const uint32_t hp = m0.x & 0xffffu;
      vo[i] = vx + (m0.x >> 16);
      ko[i] = kx + m0.y;
      kl[i] = m1.y - m0.y;  // output key bytes (plen + stored)
      vl[i] = (m1.x >> 16) - (m0.x >> 16);
      src[i] = o + hp + 10;
      // stored key bytes: the output key less its shared prefix (prefix-compressed tiles only)
      ks[i] = has_plen ? kl[i] - LdsSrc{slots + blk * kTileSlot, shb}.hdr(hp).plen : kl[i];
      on[i] = e < nt;
      kp[i] = has_plen ? 0u : pieces16(kl[i]);  // prefix-compressed tiles: bytewise below
      np[i] = kp[i] + pieces16(vl[i]);
      if (on[i] && j == 0) {
        if (mat) {
          if (p.key_end) p.key_end[en + e] = (uint32_t)(ek + ko[i] + kl[i]);
          if (p.val_end) p.val_end[en + e] = (uint32_t)(ev + vo[i] + vl[i]);
        }
        if (view)
          p.view[en + e] = (uint64_t)src[i] | ((uint64_t)ks[i] << 32) | ((uint64_t)vl[i] << 48);
      }
    }
    if (!mat) continue;
#pragma unroll
    for (int i = 0; i < G; i++) {
      if (!on[i]) continue;
      for (uint32_t q = j; q < np[i]; q += J) {
        const bool key = q < kp[i];
        uint8_t* dst = key ? kbase : vbase;
        if (!dst) continue;
        const uint32_t len = key ? kl[i] : vl[i];
        copy_piece16(dst + (key ? ko[i] : vo[i]), p.data + (key ? src[i] : src[i] + ks[i]), len,
                   key ? q : q - kp[i]);
      }
    }
  }
  if (has_plen && kbase && mat) {  // baseKey[:plen] ++ diff (iterator.go:98-100): bytewise
    for (uint32_t e = lane >> 3; e < nt; e += kWave / J) {
      uint32_t blk = 0;
#pragma unroll
      for (int q = 1; q < T; q++) blk += e >= fb[q] ? 1u : 0u;
      uint32_t f = fb[0], kx = kb[0], o = bo[0], shb = bsh[0];
#pragma unroll
      for (int q = 1; q < T; q++)
        if (blk == (uint32_t)q) {
          f = fb[q];
          kx = kb[q];
          o = bo[q];
          shb = bsh[q];
        }
      const uint2 m0 = meta[blk * kTileCap + e - f], m1 = meta[blk * kTileCap + e - f + 1];
      const uint32_t hp = m0.x & 0xffffu;
      const uint32_t plen = LdsSrc{slots + blk * kTileSlot, shb}.hdr(hp).plen;
      const uint32_t kl = m1.y - m0.y;
      const uint8_t* blk_p = p.data + o;
      for (uint32_t i = j; i < kl; i += J)
        kbase[kx + m0.y + i] = i < plen ? blk_p[10 + i] : blk_p[hp + 10 + i - plen];
    }
  }
}

hipError_t launch_decode_tile(const DecodeParams& p, hipStream_t s) {
  static const int T = getenv("LSMGPU_TILE") ? atoi(getenv("LSMGPU_TILE")) : 2;
  const uint32_t nblk = p.nblk;
  if (T == 1) {
    hipLaunchKernelGGL(tile_decode_kernel<1>, dim3(nblk), dim3(64), 0, s, p);
  } else if (T == 4) {
    hipLaunchKernelGGL(tile_decode_kernel<4>, dim3((nblk + 3) / 4), dim3(64), 0, s, p);
  } else {
    hipLaunchKernelGGL(tile_decode_kernel<2>, dim3((nblk + 1) / 2), dim3(64), 0, s, p);
  }
  return hipGetLastError();
}

hipError_t launch_decode_wsc(const DecodeParams& p, hipStream_t s, hipEvent_t mid) {
  const uint32_t nblk = p.nblk;
  if (p.wwalk == kWalkScan)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkScan, 256>), dim3((nblk + 255) / 256), dim3(256), 0, s, p);
  else if (p.wwalk == kWalkStream)
    hipLaunchKernelGGL((wsc_walk_kernel<kWalkStream, kSwTile>), dim3((nblk + kSwTile - 1) / kSwTile),
                       dim3(256), 0, s, p);
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
  if (e != hipSuccess || p.wfuse) return e;  // view-only: the walk wrote everything
  const uint32_t per_wg = 4 / p.wsplit;  // blocks per 4-wave workgroup
  hipLaunchKernelGGL(wsc_copy_kernel, dim3((nblk + per_wg - 1) / per_wg), dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace lsmgpu
