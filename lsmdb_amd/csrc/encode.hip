// encode.hip -- gfx950 SST block encode: the device restatement of Builder.Add/addHelper/
// finishBlock/blockIndex (table/builder.go:84-160) for a sorted batch of entries.
//
// Every output position is closed-form, so the encoder needs no scan:
//   entry e of block b starts at  10*e + key_start(e) + vs_start(e) + 13*b
// (each earlier entry contributes its 10-B header, its full key -- keyDiff always returns the
// whole key, builder.go:74-82 -- and its ValueStruct bytes; each earlier block its 13-B
// terminator, builder.go:121-123).  One wave builds one block: it stages the block's key and
// value bytes in LDS with coalesced loads, then writes the block as aligned 16-B chunks
// (headers synthesised in registers), plus its restart (block end offset) in the index.
#include "codec_common.hpp"
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

// Header byte r (0..9) of header{plen=0, klen, vlen, prev} (builder.go:30-35).
__device__ __forceinline__ uint32_t hdr_byte(uint32_t r, uint32_t klen, uint32_t vlen,
                                             uint32_t prev) {
  switch (r) {
    case 0: case 1: return 0;  // plen == 0 always (keyDiff, builder.go:74-82)
    case 2: return (klen >> 8) & 0xff;
    case 3: return klen & 0xff;
    case 4: return (vlen >> 8) & 0xff;
    case 5: return vlen & 0xff;
    default: return (prev >> (8 * (9 - r))) & 0xff;
  }
}

template <int SLOT, int MAXE, int WPB>
struct EncodeCfg {
  static constexpr int kData = SLOT + 64;
  static constexpr int kMeta = (MAXE + 2) * 8;
  static constexpr int kWaveBytes = (kData + kMeta + 15) & ~15;
  static constexpr int kLds = kWaveBytes * WPB;
};

// Slow path: byte-granular writes straight from global memory (blocks too large for LDS).
__device__ void encode_block_slow(const EncodeParams& p, uint32_t b, uint64_t f, uint64_t l,
                                  uint64_t bs, uint32_t lane) {
  uint64_t pos = bs;
  uint32_t prev = 0xffffffffu;
  const uint64_t k0 = key_start(p, f), v0 = vs_start(p, f);
  for (uint64_t e = f; e <= l; e++) {
    uint32_t klen, vlen;
    uint64_t ks = 0, vss = 0;
    if (e < l) {
      ks = key_start(p, e);
      vss = vs_start(p, e);
      klen = (uint32_t)(p.key_end[e] - ks);
      vlen = (uint32_t)(p.vs_end[e] - vss);
    } else {
      klen = 0;
      vlen = 3;
    }
    uint32_t total = 10 + klen + vlen;
    for (uint32_t i = lane; i < total; i += kWave) {
      uint32_t byte;
      if (i < 10) byte = hdr_byte(i, klen, vlen, prev);
      else if (i < 10 + klen) byte = p.keys[ks + (i - 10)];
      else byte = (e < l) ? p.vs[vss + (i - 10 - klen)] : 0;
      p.out[pos + i] = (uint8_t)byte;
    }
    prev = (uint32_t)(pos - bs);
    pos += total;
  }
  (void)k0; (void)v0; (void)b;
}

template <int SLOT, int MAXE, int WPB>
__global__ void __launch_bounds__(WPB * 64) encode_kernel(EncodeParams p) {
  using Cfg = EncodeCfg<SLOT, MAXE, WPB>;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = lane_id();
  const uint32_t wv = threadIdx.x >> 6;
  uint8_t* slot = smem + wv * Cfg::kWaveBytes;
  uint16_t* meta = reinterpret_cast<uint16_t*>(slot + Cfg::kData);
  const uint32_t nwaves = gridDim.x * WPB;

  for (uint32_t b = blockIdx.x * WPB + wv; b < p.nblocks; b += nwaves) {
    uint64_t f, l;
    block_range(p, b, f, l);
    f = uniform64(f);
    l = uniform64(l);
    const uint64_t kf = uniform64(key_start(p, f)), kl = uniform64(key_start(p, l));
    const uint64_t vf = uniform64(vs_start(p, f)), vl = uniform64(vs_start(p, l));
    const uint64_t m = l - f;
    const uint64_t bs = 10 * f + kf + vf + 13ull * b;       // block start
    const uint64_t bsize = 10 * m + (kl - kf) + (vl - vf) + 13;
    const uint64_t be = bs + bsize;                          // block end = restart value

    // entry validation (y.go:93-100 ParseKey needs len(key) > 8; vlen is a uint16)
    uint32_t bad = 0;
    for (uint64_t e = f + lane; e < l; e += kWave) {
      uint64_t klen = p.key_end[e] - key_start(p, e), vlen = p.vs_end[e] - vs_start(p, e);
      if (klen <= 8 || klen > 0xffff) bad |= 1;
      if (vlen > 0xffff) bad |= 2;
    }
    if (bad) atomicOr(p.flags, bad);

    // restart entry of the index (builder.go:146-160), BE32, byte stores (any alignment)
    if (lane < 4) p.out[p.data_len + 4ull * b + lane] = (uint8_t)((uint32_t)be >> (8 * (3 - lane)));
    if (b == p.nblocks - 1 && lane >= 4 && lane < 8)
      p.out[p.data_len + 4ull * p.nblocks + (lane - 4)] =
          (uint8_t)(p.nblocks >> (8 * (7 - lane)));

    const uint64_t nk = kl - kf, nv = vl - vf;
    const bool fast = (m <= (uint64_t)MAXE) && (bsize <= 0xffffull) && (nk + nv + 48 <= (uint64_t)Cfg::kData);
    if (!fast) {
      encode_block_slow(p, b, f, l, bs, lane);
      continue;
    }
    // stage keys at slot[shk..], values at slot[vbase + shv..]
    const uint32_t shk = stage_to_lds(slot, p.keys, kf, (uint32_t)nk, p.key_total, lane);
    const uint32_t vbase = (uint32_t)((shk + nk + 15) & ~15ull);
    const uint32_t shv = stage_to_lds(slot + vbase, p.vs, vf, (uint32_t)nv, p.vs_total, lane);
    const uint32_t vsrc = vbase + shv;
    // meta row i (i <= m): {pos in block, key off in LDS, vs off in LDS, 0}; row m = terminator
    for (uint32_t i = lane; i <= (uint32_t)m; i += kWave) {
      uint64_t e = f + i;
      uint32_t ko = (uint32_t)(key_start(p, e) - kf), vo = (uint32_t)(vs_start(p, e) - vf);
      uint32_t pos = 10 * i + ko + vo;
      *reinterpret_cast<ushort4*>(meta + 4 * i) =
          make_ushort4((uint16_t)pos, (uint16_t)(shk + ko), (uint16_t)(vsrc + vo), 0);
    }
    if (lane == 0)  // row m+1: end sentinel (terminator value bytes are zeros, see below)
      *reinterpret_cast<ushort4*>(meta + 4 * (m + 1)) =
          make_ushort4((uint16_t)bsize, (uint16_t)(shk + nk), (uint16_t)(vsrc + nv), 0);
    wave_lds_fence();

    // gather-write the block [bs, be) in aligned 16-B chunks
    uint8_t* dst = p.out + bs;
    const uint32_t h = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 15u);
    uint8_t* dal = dst - h;
    const uint32_t L = (uint32_t)bsize;
    const uint32_t nchunk = (h + L + 15) >> 4;
    for (uint32_t c = lane; c < nchunk; c += kWave) {
      const int32_t t0 = (int32_t)(c * 16) - (int32_t)h;
      const int32_t lo = t0 < 0 ? 0 : t0;
      const int32_t hi = (t0 + 16 > (int32_t)L) ? (int32_t)L : t0 + 16;
      uint32_t e = meta_search(meta, (uint32_t)m + 1, (uint32_t)lo);
      ushort4 me = *reinterpret_cast<const ushort4*>(meta + 4 * e);
      ushort4 mn = *reinterpret_cast<const ushort4*>(meta + 4 * e + 4);
      const bool full = (lo == t0) && (hi == t0 + 16);
      if (full && e < m) {
        uint32_t klen = (uint32_t)mn.y - me.y;
        uint32_t r0 = (uint32_t)t0 - me.x;
        uint32_t tend = (uint32_t)mn.x;  // next entry start
        if (r0 >= 10 && r0 + 16 <= 10 + klen) {
          *reinterpret_cast<uint4*>(dal + 16 * c) = lds_u128(slot, me.y + r0 - 10);
          continue;
        }
        if (r0 >= 10 + klen && (uint32_t)t0 + 16 <= tend) {
          *reinterpret_cast<uint4*>(dal + 16 * c) = lds_u128(slot, me.z + (r0 - 10 - klen));
          continue;
        }
      }
      uint4 v = make_uint4(0, 0, 0, 0);
      uint32_t prev = 0xffffffffu;
      if (e > 0) prev = meta[4 * (e - 1)];
#pragma unroll
      for (int i = 0; i < 16; i++) {
        const int32_t t = t0 + i;
        if (t < lo || t >= hi) continue;
        while (e < m && (uint32_t)mn.x <= (uint32_t)t) {
          prev = me.x;
          e++;
          me = mn;
          mn = *reinterpret_cast<const ushort4*>(meta + 4 * e + 4);
        }
        uint32_t r = (uint32_t)t - me.x;
        uint32_t klen = (e < m) ? (uint32_t)mn.y - me.y : 0;
        uint32_t vlen = (e < m) ? (uint32_t)mn.z - me.z : 3;
        uint32_t byte;
        if (r < 10) byte = hdr_byte(r, klen, vlen, prev);
        else if (r < 10 + klen) byte = slot[me.y + r - 10];
        else byte = (e < m) ? slot[me.z + (r - 10 - klen)] : 0;
        if (full) set_byte(v, i, byte);
        else dal[16 * c + i] = (uint8_t)byte;
      }
      if (full) *reinterpret_cast<uint4*>(dal + 16 * c) = v;
    }
    wave_lds_fence();
  }
}

template <int SLOT, int MAXE, int WPB>
static hipError_t launch_enc(const EncodeParams& p, int num_cus, hipStream_t s) {
  using Cfg = EncodeCfg<SLOT, MAXE, WPB>;
  auto k = encode_kernel<SLOT, MAXE, WPB>;
  int per_cu = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, WPB * 64, Cfg::kLds);
  if (e != hipSuccess) return e;
  if (per_cu < 1) per_cu = 1;
  uint64_t want = ((uint64_t)p.nblocks + WPB - 1) / WPB;
  uint64_t grid = (uint64_t)per_cu * (uint64_t)num_cus;
  if (grid > want) grid = want;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(WPB * 64), Cfg::kLds, s, p);
  return hipGetLastError();
}

hipError_t launch_encode(const EncodeParams& p, int num_cus, hipStream_t s) {
  // the slot holds one block's key + value bytes
  if (p.vs_total + p.key_total == 0 || true) {
    // choose by the average block payload when no exact bound is known
    uint64_t payload = (p.key_total + p.vs_total) / (p.nblocks ? p.nblocks : 1);
    if (payload + 64 <= 3072) return launch_enc<4096, 128, 4>(p, num_cus, s);
    if (payload + 64 <= 12288) return launch_enc<16384, 512, 2>(p, num_cus, s);
  }
  return launch_enc<32768, 1024, 1>(p, num_cus, s);
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
