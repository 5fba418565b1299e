// decode.hip -- gfx950 SST block decode: the device restatement of blockIterator.Next/parseKV
// (table/iterator.go:93-135) driven over every block of a batch (Iterator.seekToFirst/next,
// iterator.go:201-217,301-326).
//
// Structure (one wave64 per block, blocks in ticket order, persistent grid):
//   1. stage   : the block's bytes -> the wave's LDS slot with 16-B coalesced loads
//   2. walk    : the serial header chain (pos += 10 + klen + vlen) in LDS, wave-uniform
//                (SGPR) arithmetic; records {key pos, key out off, value pos, value out off}
//   3. publish : per-block aggregate {entries, key bytes, value bytes} as agent-scope granules
//   4. look-back: decoupled look-back over predecessor blocks -> exclusive output bases
//   5. emit    : per-entry end offsets (coalesced u32), key and value streams written as
//                aligned 16-B chunks gathered from LDS (byte stores only at stream edges)
// Blocks that do not fit the slot (or have > MAXE entries) take a global-memory slow path
// with identical semantics.
#include "codec_common.hpp"
#include "kernels.hpp"

namespace lsmgpu {

struct Hdr {
  uint32_t plen, klen, vlen;
};

// ---- header readers (the 10-B BE header of table/builder.go:23-45; prev is unused here)
struct LdsSrc {
  const uint8_t* slot;  // 16-B aligned LDS slot
  uint32_t sh;          // block byte 0 lives at slot + sh
  __device__ __forceinline__ Hdr hdr(uint32_t pos) const {
    uint32_t x0 = uniform(lds_u32(slot, sh + pos));
    uint32_t x1 = uniform(lds_u32(slot, sh + pos + 4));
    return Hdr{bswap16(x0 & 0xffffu), bswap16(x0 >> 16), bswap16(x1 & 0xffffu)};
  }
};
struct GlobalSrc {
  const uint8_t* blk;  // global pointer to block byte 0
  __device__ __forceinline__ Hdr hdr(uint32_t pos) const {
    const uint8_t* h = blk + pos;
    return Hdr{uniform(((uint32_t)h[0] << 8) | h[1]), uniform(((uint32_t)h[2] << 8) | h[3]),
               uniform(((uint32_t)h[4] << 8) | h[5])};
  }
};

struct WalkResult {
  uint32_t n, K, V, status, base_pos, end_pos;
};

// The blockIterator forward walk.  `meta` (LDS, stride 4 u16) gets {ks, ko, vs, vo} for
// entries < maxe when record is set.  Every value here is wave-uniform.
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
    uint32_t ks = pos;
    pos += h.klen;                                           // iterator.go:101
    if (pos + h.vlen > len) { st = LSMGPU_BLK_VALUE_OVERFLOW; break; }  // iterator.go:103
    uint32_t vs = pos;
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

struct Tot {
  uint64_t n, k, v;
};

constexpr uint32_t kMaxSpins = 1u << 22;  // ~0.5 s of polling: a hard bound, never expected

// Decoupled look-back: exclusive {entries, key bytes, value bytes} of all tiles before t.
__device__ Tot lookback(const uint64_t* lb, uint32_t t, uint64_t tag, uint32_t lane,
                        uint64_t* result) {
  Tot ex{0, 0, 0};
  int64_t j0 = (int64_t)t - 1;
  uint32_t wsize = 8;
  uint32_t spins = 0;
  while (j0 >= 0) {
    int64_t j = j0 - (int64_t)lane;
    bool active = lane < wsize;
    bool inc = false, ready = false;
    uint64_t a = 0, b = 0, c = 0;
    if (active) {
      if (j < 0) {
        inc = ready = true;
      } else {
        const uint64_t* g = lb + (uint64_t)j * 8;
        uint64_t i0 = gload(g + 4), i1 = gload(g + 5), i2 = gload(g + 6);
        if ((i0 >> kTagShift) == tag && (i1 >> kTagShift) == tag && (i2 >> kTagShift) == tag) {
          inc = ready = true;
          a = i0 & kValMask; b = i1 & kValMask; c = i2 & kValMask;
        } else {
          uint64_t a0 = gload(g + 0), a1 = gload(g + 1), a2 = gload(g + 2);
          if ((a0 >> kTagShift) == tag && (a1 >> kTagShift) == tag && (a2 >> kTagShift) == tag) {
            ready = true;
            a = a0 & kValMask; b = a1 & kValMask; c = a2 & kValMask;
          }
        }
      }
    }
    uint64_t im = __ballot(inc);
    uint64_t rm = __ballot(ready);
    uint32_t first = im ? (uint32_t)__builtin_ctzll(im) : wsize;
    uint32_t last = first < wsize ? first : wsize - 1;
    uint64_t need = (last >= 63) ? ~0ull : ((1ull << (last + 1)) - 1);
    if ((rm & need) != need) {
      if (++spins > kMaxSpins) {
        if (lane == 0) atomicOr(reinterpret_cast<unsigned long long*>(result + 5), 2ull);
        return ex;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    bool contrib = active && lane <= last;
    ex.n += wave_sum64(contrib ? a : 0);
    ex.k += wave_sum64(contrib ? b : 0);
    ex.v += wave_sum64(contrib ? c : 0);
    if (first < wsize) break;
    j0 -= (int64_t)wsize;
    wsize = 64;
  }
  ex.n = uniform64(ex.n);
  ex.k = uniform64(ex.k);
  ex.v = uniform64(ex.v);
  return ex;
}

// Writes stream bytes [0, L) of one block to dst (global, any alignment) as aligned 16-B
// chunks gathered from the LDS copy of the block.  Stream byte t belongs to the entry e with
// o(e) <= t < o(e+1), o = ko (keys) or vo (values) of the walk metadata (meta[4n+*] holds the
// totals).  Key bytes: t - ko(e) < plen(e) -> baseKey prefix (block byte base_pos + u),
// otherwise the stored diff (ks(e) + u - plen(e)) -- blockIterator.parseKV, iterator.go:98-100.
template <bool IS_KEY>
__device__ void gather_stream(uint8_t* dst, uint32_t L, const uint8_t* slot, uint32_t sh,
                              const uint16_t* meta, uint32_t n, uint32_t base_pos,
                              uint32_t lane) {
  if (L == 0) return;
  const uint32_t h = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 15u);
  uint8_t* dal = dst - h;
  const uint32_t nchunk = (h + L + 15) >> 4;
  const uint16_t* ocol = meta + (IS_KEY ? 1 : 3);
  for (uint32_t c = lane; c < nchunk; c += kWave) {
    const int32_t t0 = (int32_t)(c * 16) - (int32_t)h;
    const int32_t lo = t0 < 0 ? 0 : t0;
    const int32_t hi = (t0 + 16 > (int32_t)L) ? (int32_t)L : t0 + 16;
    uint32_t e = meta_search(ocol, n, (uint32_t)lo);
    ushort4 me = *reinterpret_cast<const ushort4*>(meta + 4 * e);
    ushort4 mn = *reinterpret_cast<const ushort4*>(meta + 4 * e + 4);
    uint32_t o0 = IS_KEY ? me.y : me.w, o1 = IS_KEY ? mn.y : mn.w;
    uint32_t plen = IS_KEY ? (o1 - o0) - ((uint32_t)me.z - me.x) : 0;
    const bool full = (lo == t0) && (hi == t0 + 16);
    bool fast = false;
    uint32_t src = 0;
    if (full && (uint32_t)(t0 + 16) <= o1) {
      uint32_t u0 = (uint32_t)t0 - o0;
      if (!IS_KEY) {
        fast = true;
        src = me.z + u0;
      } else if (u0 + 16 <= plen) {
        fast = true;
        src = base_pos + u0;
      } else if (u0 >= plen) {
        fast = true;
        src = me.x + (u0 - plen);
      }
    }
    if (fast) {
      *reinterpret_cast<uint4*>(dal + 16 * c) = lds_u128(slot, sh + src);
      continue;
    }
    uint4 v = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const int32_t t = t0 + i;
      if (t < lo || t >= hi) continue;
      while (o1 <= (uint32_t)t) {  // advance to the entry holding t (skips empty entries)
        e++;
        me = mn;
        mn = *reinterpret_cast<const ushort4*>(meta + 4 * e + 4);
        o0 = o1;
        o1 = IS_KEY ? mn.y : mn.w;
        plen = IS_KEY ? (o1 - o0) - ((uint32_t)me.z - me.x) : 0;
      }
      uint32_t u = (uint32_t)t - o0;
      uint32_t s;
      if (!IS_KEY) s = me.z + u;
      else s = (u < plen) ? base_pos + u : me.x + (u - plen);
      uint32_t byte = slot[sh + s];
      if (full) set_byte(v, i, byte);
      else dal[16 * c + i] = (uint8_t)byte;
    }
    if (full) *reinterpret_cast<uint4*>(dal + 16 * c) = v;
  }
}

// Global-memory path with the same semantics: re-walks the block and copies every entry's
// key and value with the wave's lanes (byte granular).  Used for oversize blocks only.
__device__ void emit_slow(const DecodeParams& p, const uint8_t* blk, uint32_t len, uint32_t n,
                          uint64_t ebase, uint64_t kbase, uint64_t vbase, uint64_t off,
                          uint32_t lane) {
  GlobalSrc src{blk};
  uint32_t pos = 0, base_pos = 0;
  uint64_t kb = kbase, vb = vbase;
  for (uint32_t e = 0; e < n; e++) {
    Hdr hd = src.hdr(pos);
    pos += 10;
    if (e == 0) base_pos = pos;
    uint32_t ks = pos, vs = pos + hd.klen;
    if (p.mode & LSMGPU_MODE_MATERIALIZE) {
      uint32_t kl = hd.plen + hd.klen;
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

template <int SLOT, int MAXE, int WPB>
struct DecodeCfg {
  static constexpr int kData = SLOT + 32;
  static constexpr int kMeta = (MAXE + 1) * 8;
  static constexpr int kWaveBytes = (kData + kMeta + 15) & ~15;
  static constexpr int kLds = kWaveBytes * WPB;
};

template <int SLOT, int MAXE, int WPB>
__global__ void __launch_bounds__(WPB * 64) decode_kernel(DecodeParams p) {
  using Cfg = DecodeCfg<SLOT, MAXE, WPB>;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = lane_id();
  const uint32_t wv = threadIdx.x >> 6;
  uint8_t* slot = smem + wv * Cfg::kWaveBytes;
  uint16_t* meta = reinterpret_cast<uint16_t*>(slot + Cfg::kData);
  const uint64_t tag = p.tag;

  for (;;) {
    uint64_t tk = 0;
    if (lane == 0) tk = atomicAdd(p.ticket, 1ull);
    tk = uniform64(tk) - p.ticket_base;
    if (tk >= p.nblk) break;
    const uint32_t t = (uint32_t)tk;

    const uint64_t off = uniform(p.blk_off[t]);
    const uint32_t len = uniform(p.blk_len[t]);
    WalkResult w{0, 0, 0, LSMGPU_BLK_OK, 0, 0};
    bool fast = false;
    uint32_t sh = 0;
    if (off + len > p.data_len) {
      w.status = LSMGPU_BLK_RANGE;
    } else if (len <= (uint32_t)SLOT) {
      sh = stage_to_lds(slot, p.data, off, len, p.data_len, lane);
      wave_lds_fence();
      w = walk_block(LdsSrc{slot, sh}, len, meta, MAXE, true, lane);
      fast = (w.n <= (uint32_t)MAXE) && (w.K <= 0xffffu) && (w.V <= 0xffffu);
    } else {
      w = walk_block(GlobalSrc{p.data + off}, len, meta, 0, false, lane);
    }
    if (fast && lane == 0) {  // sentinel row: totals
      ushort4 m = make_ushort4((uint16_t)w.end_pos, (uint16_t)w.K, 0, (uint16_t)w.V);
      *reinterpret_cast<ushort4*>(meta + 4 * w.n) = m;
    }

    // ---- publish aggregate, look back, publish inclusive
    uint64_t* g = p.lb + (uint64_t)t * 8;
    const uint64_t mine = lane == 0 ? w.n : (lane == 1 ? w.K : w.V);
    if (t > 0 && lane < 3) gstore(g + lane, (tag << kTagShift) | mine);
    Tot ex = lookback(p.lb, t, tag, lane, p.result);
    const uint64_t incl = lane == 0 ? ex.n + w.n : (lane == 1 ? ex.k + w.K : ex.v + w.V);
    if (lane < 3) gstore(g + 4 + lane, (tag << kTagShift) | incl);
    wave_lds_fence();

    // ---- per-block outputs
    if (lane == 0) {
      if (p.blk_first) p.blk_first[t] = (uint32_t)ex.n;
      if (p.blk_status) p.blk_status[t] = (int32_t)w.status;
      if (w.status != LSMGPU_BLK_OK) {
        atomicAdd(reinterpret_cast<unsigned long long*>(p.result + 4), 1ull);
        atomicMax(reinterpret_cast<unsigned long long*>(p.result + 3),
                  (unsigned long long)(p.nblk - t));
      }
      if (t == p.nblk - 1) {
        if (p.blk_first) p.blk_first[p.nblk] = (uint32_t)(ex.n + w.n);
        p.result[0] = ex.n + w.n;
        p.result[1] = ex.k + w.K;
        p.result[2] = ex.v + w.V;
      }
    }
    if (w.n == 0) continue;

    // ---- capacity checks (skip every write of a block that does not fit)
    const bool mat = (p.mode & LSMGPU_MODE_MATERIALIZE) != 0;
    const bool view = (p.mode & LSMGPU_MODE_VIEW) != 0 && p.view;
    bool ok = ex.n + w.n <= p.ent_cap;
    if (mat) {
      ok = ok && (ex.k + w.K <= p.key_cap || !p.key_data) && (ex.v + w.V <= p.val_cap || !p.val_data);
      ok = ok && ex.k + w.K <= 0xffffffffull && ex.v + w.V <= 0xffffffffull;
    }
    if (!ok) {
      if (lane == 0) atomicOr(reinterpret_cast<unsigned long long*>(p.result + 5), 1ull);
      continue;
    }

    if (!fast) {
      emit_slow(p, p.data + off, len, w.n, ex.n, ex.k, ex.v, off, lane);
      continue;
    }
    // per-entry offsets / view records: lane e handles entry e (coalesced u32 / u64 stores)
    for (uint32_t e = lane; e < w.n; e += kWave) {
      ushort4 me = *reinterpret_cast<const ushort4*>(meta + 4 * e);
      ushort4 mn = *reinterpret_cast<const ushort4*>(meta + 4 * e + 4);
      if (mat) {
        if (p.key_end) p.key_end[ex.n + e] = (uint32_t)(ex.k + mn.y);
        if (p.val_end) p.val_end[ex.n + e] = (uint32_t)(ex.v + mn.w);
      }
      if (view) {
        uint32_t klen = (uint32_t)me.z - me.x, vlen = (uint32_t)mn.w - me.w;
        p.view[ex.n + e] = (uint64_t)(uint32_t)(off + me.x) | ((uint64_t)klen << 32) |
                           ((uint64_t)vlen << 48);
      }
    }
    if (mat) {
      if (p.key_data) gather_stream<true>(p.key_data + ex.k, w.K, slot, sh, meta, w.n, w.base_pos, lane);
      if (p.val_data) gather_stream<false>(p.val_data + ex.v, w.V, slot, sh, meta, w.n, 0, lane);
    }
  }
}

template <int SLOT, int MAXE, int WPB>
static hipError_t launch_cfg(const DecodeParams& p, int num_cus, hipStream_t s,
                             uint64_t* waves_launched) {
  using Cfg = DecodeCfg<SLOT, MAXE, WPB>;
  auto k = decode_kernel<SLOT, MAXE, WPB>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, Cfg::kLds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  int per_cu = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, WPB * 64, Cfg::kLds);
  if (e != hipSuccess) return e;
  if (per_cu < 1) per_cu = 1;
  uint64_t want = ((uint64_t)p.nblk + WPB - 1) / WPB;
  uint64_t grid = (uint64_t)per_cu * (uint64_t)num_cus;
  if (grid > want) grid = want;
  if (grid < 1) grid = 1;
  *waves_launched = grid * WPB;
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(WPB * 64), Cfg::kLds, s, p);
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
