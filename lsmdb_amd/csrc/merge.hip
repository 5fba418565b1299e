// merge.hip -- y.MergeIterator (y/iterator.go:74-202) over K sorted runs on gfx950: the
// merge step of compactBuildTables (levels.go:239-258) between the device decode of the input
// tables and the device encode of the output tables.
//
// MergeIterator always emits the least head under elemHeap.Less (y.CompareKeys, then the lower
// `nice` = run index) and Next() drops every head equal to the last emitted key.  For sorted
// runs (SSTs are) that is: the runs' stable merge under (CompareKeys, run), keeping the first
// entry of each group of equal keys.  Computed without a heap, every entry in parallel:
//   check  (lane = entry)   runs in CompareKeys order? keys > 8 B (CompareKeys asserts it)?
//                           drop[i] = equal to its predecessor in its own run
//   tiles  (one lane)       tile bases; F = the largest run (the "fill" run: in a compaction
//                           the bottom level's tables, most of the entries)
//   split  (lane = tile x run) for the first entry of every 256-entry tile of a run other than
//                           F, its rank in every other run (full binary search)
//   rank   (lane = entry of a run other than F)  merged position = own index in its run + for
//                           every other run the number of entries that precede it: binary search
//                           between the tile's splitters, upper bound for lower-index runs (equal
//                           keys of a lower nice come first), lower bound for higher-index runs.
//                           Dropped if a lower-index run holds an equal key; an equal key of F
//                           that follows it is marked dropped.  Writes dst[pos] = entry,
//                           rec[pos] = {key start, kept ? key len : 0, value start, value len}
//                           and the position's bit in the occupancy bitmap (+ its chunk's count)
//   occ    (one workgroup)  occupied positions before every 1024-position chunk
//   emit   (lane = 4 merged positions, workgroup = a 1024-position chunk)  an occupied position
//                           reads its rec; a free one is F's next entry in order (F's index =
//                           position - occupied positions before it), read from F's own end
//                           offsets; the tile's scan of {kept, key bytes, value bytes} and its
//                           output base by decoupled look-back; end offsets, source index, and
//                           8 lanes per kept entry copy 16-B pieces of key and raw vs-enc bytes
// F's entries are never searched: a compaction with one small overlapping run and one large
// run ranks only the small run's entries.
// Unsorted runs (the heap would interleave them differently) and keys <= 8 B are reported in
// result[3] and produce no output.
#include "decode_common.hpp"
#include "kernels.hpp"

namespace lsmgpu {

namespace {

constexpr uint32_t M_UNSORTED = 1, M_KEY_LEN = 2, M_CAPACITY = 4, M_TIMEOUT = 8;
constexpr uint32_t kMergeTile = 256;  // entries per splitter tile

__device__ __forceinline__ const uint8_t* key_of(const MergeParams& p, uint32_t i, uint32_t& len) {
  const uint32_t s = i ? p.ke[i - 1] : 0u;
  len = p.ke[i] - s;
  return p.kd + s;
}

__device__ __forceinline__ uint32_t run_of(const MergeParams& p, uint32_t i) {
  uint32_t lo = 0, hi = p.nruns - 1;  // largest r with run_first[r] <= i
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (p.run_first[mid] <= i) lo = mid; else hi = mid - 1;
  }
  return lo;
}

}  // namespace

__global__ void merge_check_kernel(MergeParams p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  uint32_t li;
  const uint8_t* ki = key_of(p, i, li);
  uint32_t fl = 0;
  uint8_t dup = 0;
  if (li <= 8) {
    fl = M_KEY_LEN;
  } else {
    const uint32_t r = run_of(p, i);
    if (i > p.run_first[r]) {
      uint32_t lp;
      const uint8_t* kp = key_of(p, i - 1, lp);
      if (lp > 8) {
        const int c = compare_keys(kp, lp, ki, li);
        if (c > 0) fl = M_UNSORTED;
        dup = c == 0;
      }
    }
  }
  p.drop[i] = dup;
  if (fl) atomicOr(p.flags, fl);
}

// Entries of run s that precede key x of run r (key < x, or == x with s < r: lower nice
// first), searched in [lo, hi) of run s.  With want_eq, eq = the key next to that rank equals
// x: for s < r the entry just below it (x is then not the first of its equal-key group), for
// s > r the entry at it (which x precedes and makes a duplicate).  The search compared that
// entry last whenever it moved the matching bound; otherwise one more compare.
__device__ __forceinline__ uint32_t rank_in(const MergeParams& p, uint32_t s, uint32_t r,
                                            const uint8_t* kx, uint32_t lx, uint32_t lo,
                                            uint32_t hi, bool want_eq, bool& eq) {
  const bool before = s < r;
  int clo = 1, chi = 1;
  bool mlo = false, mhi = false;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    uint32_t lm;
    const uint8_t* km = key_of(p, mid, lm);
    const int c = compare_keys(km, lm, kx, lx);
    if (c < 0 || (c == 0 && before)) {
      lo = mid + 1;
      mlo = true;
      clo = c;
    } else {
      hi = mid;
      mhi = true;
      chi = c;
    }
  }
  eq = false;
  if (want_eq) {
    uint32_t lm;
    if (before) {
      if (mlo) eq = clo == 0;
      else if (lo > p.run_first[s]) eq = compare_keys(key_of(p, lo - 1, lm), lm, kx, lx) == 0;
    } else {
      if (mhi) eq = chi == 0;
      else if (lo < p.run_first[s + 1]) eq = compare_keys(key_of(p, lo, lm), lm, kx, lx) == 0;
    }
  }
  return lo;
}

// tile_base[r] = first tile of run r (tiles of kMergeTile entries never span runs); flags[2] =
// the fill run F (the largest, the first of equals)
__global__ void merge_tiles_kernel(MergeParams p) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint32_t t = 0, f = 0, fn = 0;
  for (uint32_t r = 0; r < p.nruns; r++) {
    p.tile_base[r] = t;
    const uint32_t m = p.run_first[r + 1] - p.run_first[r];
    t += (m + kMergeTile - 1) / kMergeTile;
    if (m > fn) {
      fn = m;
      f = r;
    }
  }
  p.tile_base[p.nruns] = t;
  p.flags[2] = f;
}

// Splitters: for the first entry of every tile of a run other than F, its absolute rank
// position in every other run (a full binary search); entries then only search between their
// tile's splitters.
__global__ void merge_split_kernel(MergeParams p) {
  const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t g = x / p.nruns, s = x % p.nruns;
  if (p.flags[0] || g >= p.tile_base[p.nruns]) return;
  uint32_t r = 0;  // run of tile g
  while (p.tile_base[r + 1] <= g) r++;
  if (r == p.flags[2]) return;
  const uint32_t i = p.run_first[r] + (g - p.tile_base[r]) * kMergeTile;
  uint32_t li;
  const uint8_t* ki = key_of(p, i, li);
  bool eq;
  p.spl[(uint64_t)g * p.nruns + s] =
      s == r ? i : rank_in(p, s, r, ki, li, p.run_first[s], p.run_first[s + 1], false, eq);
}

__global__ void merge_rank_kernel(MergeParams p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n || p.flags[0]) return;
  const uint32_t f = p.flags[2];
  if (i >= p.run_first[f] && i < p.run_first[f + 1]) return;  // F fills the free positions
  const uint32_t r = run_of(p, i);
  const uint32_t j = i - p.run_first[r];
  const uint32_t g = p.tile_base[r] + j / kMergeTile;
  const bool last_tile = g + 1 == p.tile_base[r + 1];
  const uint32_t ks = i ? p.ke[i - 1] : 0u, kl = p.ke[i] - ks;
  const uint32_t vs = i ? p.ve[i - 1] : 0u, vl = p.ve[i] - vs;
  const uint8_t* ki = p.kd + ks;
  // dropped: an equal key earlier in its own run (merge_check_kernel) or in a lower-index run
  // (bytes.Equal with the last emitted key, y/iterator.go:172-181: equal keys are adjacent in
  // merged order, the lowest run first)
  bool drop = p.drop[i] != 0;
  uint32_t pos = j;
  for (uint32_t s = 0; s < p.nruns; s++) {
    if (s == r) continue;
    const uint32_t lo = p.spl[(uint64_t)g * p.nruns + s];
    const uint32_t hi = last_tile ? p.run_first[s + 1] : p.spl[(uint64_t)(g + 1) * p.nruns + s];
    bool eq;
    const uint32_t at = rank_in(p, s, r, ki, kl, lo, hi, s < r || s == f, eq);
    pos += at - p.run_first[s];
    if (s < r) drop |= eq;
    else if (s == f && eq) p.drop[at] = 1;  // F's equal key comes after this one: dropped
  }
  p.dst[pos] = i;
  // the emit's per-position record (kl = 0: dropped; kept keys are > 8 B, merge_check_kernel)
  p.rec[pos] = make_uint4(ks, drop ? 0u : kl, vs, vl);
  atomicOr(p.occ + (pos >> 5), 1u << (pos & 31));
  // occupied positions per chunk: one atomic per distinct chunk of the wave (a wave's entries
  // land in one or two chunks; 64 same-address atomics cost 2.5x the whole rank kernel)
  const uint32_t ch = pos / kMergeEmitTile;
  uint64_t todo = __ballot(1);
  while (todo) {
    const uint32_t c0 = (uint32_t)__shfl((int)ch, __builtin_ctzll(todo));
    const uint64_t same = __ballot(ch == c0) & todo;
    if (ch == c0 && lane_id() == (uint32_t)__builtin_ctzll(same)) atomicAdd(p.cpre + c0, (uint32_t)__popcll(same));
    todo &= ~same;
  }
}

// cpre[c]: occupied positions in chunk c (the rank kernel's counts) -> occupied positions
// before chunk c; one workgroup of 1024 threads, each scanning a contiguous range of chunks
__global__ void __launch_bounds__(1024) merge_occ_kernel(MergeParams p) {
  __shared__ uint32_t s_w[16];
  if (p.flags[0]) return;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint32_t nch = (p.n + kMergeEmitTile - 1) / kMergeEmitTile;
  const uint32_t per = (nch + 1023) / 1024, c0 = min(nch, tid * per), c1 = min(nch, c0 + per);
  uint32_t sum = 0;
  for (uint32_t c = c0; c < c1; c++) sum += p.cpre[c];
  const uint32_t inc = wave_scan_sat(sum, lane);  // counts < n < 2^32: never saturates
  if (lane == 63) s_w[wave] = inc;
  __syncthreads();
  uint32_t base = inc - sum;
  for (uint32_t w = 0; w < wave; w++) base += s_w[w];
  for (uint32_t c = c0; c < c1; c++) {
    const uint32_t m = p.cpre[c];
    p.cpre[c] = base;
    base += m;
  }
}

// scan + gather in one pass (lane = 4 consecutive merged positions, a workgroup = one
// 1024-position chunk taken by ticket): occupied positions take the rank kernel's records, free
// ones F's entries in order; the tile scans {kept, key bytes, value bytes}, finds its output
// base by decoupled look-back over the tile records (epoch-tagged granules in p.lb, as in the
// decode walk), writes the end offsets and source index of its kept entries, then 8 lanes per
// kept entry copy the key and raw vs-enc bytes as 16-B pieces.

__device__ __forceinline__ uint4 load16u(const uint8_t* p) {  // any alignment
  uint4 v;
  __builtin_memcpy(&v, p, 16);
  return v;
}
__device__ __forceinline__ void store16u(uint8_t* p, uint4 v) { __builtin_memcpy(p, &v, 16); }

// G entries per 8-lane group per gather trip, every first piece loaded before any is stored
__global__ void __launch_bounds__(256) merge_emit_kernel(MergeParams p) {
  constexpr uint32_t PP = 4, G = 4, kEmitTile = 256 * PP;
  static_assert(kEmitTile == kMergeEmitTile, "emit tile = occupancy chunk");
  // kept entries: {ks, kl, bk, vs}, {vl, bv} (kl = vl = 0: past an output capacity, no copy)
  __shared__ uint4 s_ent[kEmitTile];
  __shared__ uint2 s_env[kEmitTile];
  __shared__ uint32_t s_occ[32][2];  // the chunk's bitmap words, occupied bits before each
  __shared__ uint32_t s_tile;
  __shared__ uint32_t s_wave[4][3];
  __shared__ uint32_t s_ex[3];
  if (p.flags[0]) return;  // input errors (stream-ordered before this launch): no output
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint32_t ntiles = (p.n + kEmitTile - 1) / kEmitTile;
  if (tid == 0) {
    const uint32_t t = atomicAdd(p.gcnt, 1u);
    if (t == ntiles - 1) atomicExch(p.gcnt, 0u);  // every ticket is taken
    s_tile = t;
  }
  __syncthreads();
  const uint32_t tile = s_tile;
  if (wave == 0) {  // the chunk's 32 bitmap words (zeroed past n) and their prefix counts
    const uint32_t w = lane < 32 ? p.occ[tile * 32 + lane] : 0u;
    const uint32_t c = __popc(w), inc = wave_scan_sat(c, lane);
    if (lane < 32) {
      s_occ[lane][0] = w;
      s_occ[lane][1] = inc - c;
    }
  }
  __syncthreads();
  const uint32_t q0 = tile * kEmitTile + PP * tid;
  uint32_t src[PP], kl[PP], vl[PP], ks[PP], vs[PP];
  uint32_t keepm = 0, tn = 0, tk = 0, tv = 0;
  if (q0 < p.n) {
    const uint32_t wi = tid >> 3, sh = (PP * tid) & 31u;
    const uint32_t w = s_occ[wi][0];
    // F's index of the first free position among this thread's: position - occupied before
    uint32_t fj = q0 - (p.cpre[tile] + s_occ[wi][1] + __popc(w & ((1u << sh) - 1u)));
    const uint32_t f0 = p.run_first[p.flags[2]], f1 = p.run_first[p.flags[2] + 1];
#pragma unroll
    for (uint32_t c = 0; c < PP; c++) {
      kl[c] = vl[c] = ks[c] = vs[c] = src[c] = 0;
      if (q0 + c >= p.n) continue;
      bool keep;
      if ((w >> (sh + c)) & 1u) {
        const uint4 rc = p.rec[q0 + c];
        ks[c] = rc.x;
        kl[c] = rc.y;
        vs[c] = rc.z;
        vl[c] = rc.w;
        keep = kl[c] != 0;
        if (p.osrc) src[c] = p.dst[q0 + c];
      } else {
        const uint32_t i = f0 + fj++;
        if (i >= f1) continue;  // never for ranks that form a permutation (sorted runs)
        ks[c] = i ? p.ke[i - 1] : 0u;
        vs[c] = i ? p.ve[i - 1] : 0u;
        kl[c] = p.ke[i] - ks[c];
        vl[c] = p.ve[i] - vs[c];
        keep = p.drop[i] == 0;
        src[c] = i;
      }
      if (keep) {
        keepm |= 1u << c;
        tn++;
        tk += kl[c];
        tv += vl[c];
      }
    }
  }
  // tile scan (u32: kept key / value bytes are bounded by the <= 4 GiB - 1 input streams)
  const uint32_t in_ = wave_scan_sat(tn, lane), ik = wave_scan_sat(tk, lane),
                 iv = wave_scan_sat(tv, lane);
  if (lane == 63) {
    s_wave[wave][0] = in_;
    s_wave[wave][1] = ik;
    s_wave[wave][2] = iv;
  }
  __syncthreads();
  if (wave == 0) {
    uint32_t an = 0, ak = 0, av = 0;
    for (int w = 0; w < 4; w++) {
      an = sat_add(an, s_wave[w][0]);
      ak = sat_add(ak, s_wave[w][1]);
      av = sat_add(av, s_wave[w][2]);
    }
    uint64_t* R = p.lb + (uint64_t)tile * 8;
    Tot ex{0, 0, 0};
    if (tile > 0) {
      store3(R, p.tag, an, ak, av, lane);
      ex = lookback(p.lb, tile, p.tag, lane, p.result);
    }
    store3(R + 4, p.tag, sat_add(ex.n, an), sat_add(ex.k, ak), sat_add(ex.v, av), lane);
    if (lane == 0) {
      s_ex[0] = ex.n;
      s_ex[1] = ex.k;
      s_ex[2] = ex.v;
      if (tile == ntiles - 1) {  // totals (the last tile's inclusive prefix)
        const uint64_t N = sat_add(ex.n, an), K = sat_add(ex.k, ak), V = sat_add(ex.v, av);
        p.result[0] = N;
        p.result[1] = K;
        p.result[2] = V;
        if (N > p.ent_cap || (p.okd && K > p.key_cap) || (p.ovd && V > p.val_cap))
          atomicOr(p.flags + 1, M_CAPACITY);
      }
    }
  }
  __syncthreads();
  uint32_t ln = in_ - tn, bk = ik - tk, bv = iv - tv;  // exclusive inside the wave
  uint32_t wn = 0;                                       // tile-local entry index base
  for (uint32_t w = 0; w < wave; w++) {
    wn += s_wave[w][0];
    bk += s_wave[w][1];
    bv += s_wave[w][2];
  }
  ln += wn;
  bk += s_ex[1];
  bv += s_ex[2];
  const uint32_t n0 = s_ex[0];
  for (uint32_t c = 0; c < PP; c++) {
    if (!((keepm >> c) & 1u)) continue;
    const uint32_t bn = n0 + ln;
    const bool fits = bn < p.ent_cap && !(p.okd && (uint64_t)bk + kl[c] > p.key_cap) &&
                      !(p.ovd && (uint64_t)bv + vl[c] > p.val_cap);
    s_ent[ln] = make_uint4(ks[c], fits ? kl[c] : 0u, bk, vs[c]);
    s_env[ln] = make_uint2(fits ? vl[c] : 0u, bv);
    if (fits) {
      if (p.oke) p.oke[bn] = bk + kl[c];
      if (p.ove) p.ove[bn] = bv + vl[c];
      if (p.osrc) p.osrc[bn] = src[c];
    }
    ln++;
    bk += kl[c];
    bv += vl[c];
  }
  __syncthreads();
  // gather: 8 lanes per kept entry, G entries per lane per trip with every first-round
  // 16-B piece loaded before any is stored (more loads in flight per wave)
  constexpr uint32_t kGatherG = G;
  const uint32_t m = s_wave[0][0] + s_wave[1][0] + s_wave[2][0] + s_wave[3][0];
  const uint32_t sub = tid & 7u;
  for (uint32_t e0 = tid >> 3; e0 < m; e0 += kGatherG * (256 / 8)) {
    uint4 v[kGatherG];
    uint8_t* d[kGatherG];
#pragma unroll
    for (uint32_t g = 0; g < kGatherG; g++) {
      d[g] = nullptr;
      const uint32_t e = e0 + g * (256 / 8);
      if (e >= m) continue;
      const uint4 a = s_ent[e];
      const uint2 b = s_env[e];
      const uint32_t eks = a.x, ekl = a.y, ebk = a.z, evs = a.w, evl = b.x, ebv = b.y;
      const uint32_t kpc = p.okd ? pieces16(ekl) : 0u, np = kpc + (p.ovd ? pieces16(evl) : 0u);
      for (uint32_t c = sub; c < np; c += 8) {
        const bool key = c < kpc;
        uint8_t* dst = key ? p.okd + ebk : p.ovd + ebv;
        const uint8_t* src = key ? p.kd + eks : p.vd + evs;
        const uint32_t len = key ? ekl : evl, q = key ? c : c - kpc;
        if (c == sub && len >= 16) {  // first round: deferred store
          const uint32_t o = min(16 * q, len - 16);
          v[g] = load16u(src + o);
          d[g] = dst + o;
        } else {
          copy_piece16(dst, src, len, q);
        }
      }
    }
#pragma unroll
    for (uint32_t g = 0; g < kGatherG; g++)
      if (d[g]) store16u(d[g], v[g]);
  }
}

__global__ void merge_flags_kernel(MergeParams p) {
  if (threadIdx.x == 0)
    p.result[3] = (uint64_t)(p.flags[0] | p.flags[1]) | (p.result[5] ? M_TIMEOUT : 0u);
}

hipError_t launch_merge(const MergeParams& p, hipStream_t s) {
  hipError_t e;
  if ((e = hipMemsetAsync(p.flags, 0, 8, s)) != hipSuccess) return e;
  if (p.n) {
    const size_t nch = (p.n + kMergeEmitTile - 1) / kMergeEmitTile;
    if ((e = hipMemsetAsync(p.occ, 0, nch * 128, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(p.cpre, 0, nch * 4, s)) != hipSuccess) return e;
    const dim3 g((p.n + 255) / 256);
    hipLaunchKernelGGL(merge_check_kernel, g, dim3(256), 0, s, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(merge_tiles_kernel, dim3(1), dim3(64), 0, s, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const uint64_t tiles = p.n / kMergeTile + p.nruns;  // >= the tile count
    hipLaunchKernelGGL(merge_split_kernel, dim3((uint32_t)((tiles * p.nruns + 255) / 256)),
                       dim3(256), 0, s, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(merge_rank_kernel, g, dim3(256), 0, s, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(merge_occ_kernel, dim3(1), dim3(1024), 0, s, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(merge_emit_kernel, dim3((p.n + kMergeEmitTile - 1) / kMergeEmitTile),
                       dim3(256), 0, s, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  hipLaunchKernelGGL(merge_flags_kernel, dim3(1), dim3(64), 0, s, p);
  return hipGetLastError();
}

}  // namespace lsmgpu
