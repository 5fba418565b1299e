// copy_real_probe.hip -- the copy kernel's job on C2-shaped blocks with the real shape mix
// (workload.encode_values: 16-B keys; ValueStruct 2 + uvarint + 100 B, 10 % with an ExpiresAt
// varint of 1..10 B, 5 % value pointers of 12 B), one wave per block, one block per wave, 1 GiB:
//   pieces : the wsc_copy_kernel pattern (8 lanes per entry, 5 entry groups per trip, records by
//            lane shuffle; each field as unaligned 16-B pieces, the last overlapping back, 8/4/1-B
//            pieces below 16 B)
//   chunks : each stream (keys, values) of the block as ALIGNED 16-B output chunks, one lane
//            each, over a combined key + value chunk index: an LDS owner table (entry of each
//            chunk's first byte, filled by the entry lanes), a 16-B load from the owner and one
//            more from each following entry the chunk runs into, merged under byte masks; the
//            stream's partial head / tail chunks (shared with the neighbouring blocks) as
//            naturally aligned 8/4/2/1-B stores
// Both outputs are checked against a host copy.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/copy_real_probe scripts/copy_real_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

constexpr uint32_t kCap = 64;        // records per block slot (n <= 63 + the sentinel)
constexpr uint32_t kOwn = 512;       // owner-table bytes per wave (chunks of both streams)

__device__ __forceinline__ uint32_t pieces16(uint32_t len) {
  return len >= 16 ? (len + 15) >> 4 : (len >= 4 ? 2u : len);
}
__device__ __forceinline__ void copy_piece16(uint8_t* dst, const uint8_t* src, uint32_t len, uint32_t q) {
  if (len >= 16) {
    const uint32_t o = min(16 * q, len - 16);
    uint4 v;
    __builtin_memcpy(&v, src + o, 16);
    __builtin_memcpy(dst + o, &v, 16);
  } else if (len >= 8) {
    const uint32_t o = q ? len - 8 : 0;
    uint2 v;
    __builtin_memcpy(&v, src + o, 8);
    __builtin_memcpy(dst + o, &v, 8);
  } else if (len >= 4) {
    const uint32_t o = q ? len - 4 : 0;
    uint32_t v;
    __builtin_memcpy(&v, src + o, 4);
    __builtin_memcpy(dst + o, &v, 4);
  } else {
    dst[q] = src[q];
  }
}

struct Blocks {
  const uint8_t* data;
  const uint32_t* off;   // block start in data
  const uint32_t* n;     // entries
  const uint32_t* rec;   // kCap records per block: pos | value offset << 16, rec[n] the sentinel
  const uint64_t* ek;    // key / value stream base of the block
  const uint64_t* ev;
  const uint32_t* K;     // key / value bytes of the block
  const uint32_t* V;
  uint8_t* kd;
  uint8_t* vd;
  uint32_t nb;
  const uint32_t* en;    // first entry of the block
  uint32_t* key_end;     // per-entry end offsets (EO variants)
  uint32_t* val_end;
};

// EO: the per-entry end offsets first, one lane per entry (entry_outputs); XCD: workgroup w runs
// on XCD w % 8 (round-robin dispatch), so each XCD takes a contiguous eighth of the blocks
template <bool EO, bool XCD>
__global__ void __launch_bounds__(256) pieces(Blocks p) {
  const uint32_t lane = threadIdx.x & 63;
  uint32_t wg = blockIdx.x;
  if (XCD) {
    const uint32_t per = gridDim.x / 8;  // grid a multiple of 8
    wg = (blockIdx.x % 8) * per + blockIdx.x / 8;
  }
  const uint32_t b = wg * 4 + (threadIdx.x >> 6);
  if (b >= p.nb) return;
  const uint32_t n = p.n[b];
  const uint32_t* meta = p.rec + (uint64_t)b * kCap;
  const uint32_t pre = meta[lane];
  if (EO) {
    const uint32_t m1 = (uint32_t)__shfl((int)pre, (int)min(lane + 1, 63u));
    const uint32_t vo1 = m1 >> 16;
    if (lane < n) {
      p.key_end[p.en[b] + lane] = (uint32_t)(p.ek[b] + (m1 & 0xffffu) - 10 * (lane + 1) - vo1);
      p.val_end[p.en[b] + lane] = (uint32_t)(p.ev[b] + vo1);
    }
  }
  const uint8_t* blk = p.data + p.off[b];
  uint8_t* kb = p.kd + p.ek[b];
  uint8_t* vb = p.vd + p.ev[b];
  constexpr uint32_t J = 8, G = 5;
  const uint32_t j = lane & (J - 1);
  for (uint32_t e0 = 0; e0 < n; e0 += G * 8) {
    uint32_t hp[G], kl[G], vl[G], ko[G], vo[G], np[G], kp[G];
    bool on[G];
#pragma unroll
    for (uint32_t i = 0; i < G; i++) {
      const uint32_t e = e0 + i * 8 + lane / J, ec = min(e, n - 1);
      const uint32_t m0 = (uint32_t)__shfl((int)pre, (int)ec), m1 = (uint32_t)__shfl((int)pre, (int)ec + 1);
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
    for (uint32_t i = 0; i < G; i++) {
      if (!on[i]) continue;
      for (uint32_t q = j; q < np[i]; q += J) {
        const bool key = q < kp[i];
        copy_piece16(key ? kb + ko[i] : vb + vo[i], blk + hp[i] + 10 + (key ? 0u : kl[i]),
                     key ? kl[i] : vl[i], key ? q : q - kp[i]);
      }
    }
  }
}

__device__ __forceinline__ uint32_t bytes_from(uint32_t k, uint32_t d) {  // mask: bytes of dword d at >= k
  const int32_t t = (int32_t)k - 4 * (int32_t)d;
  return t <= 0 ? 0xffffffffu : t >= 4 ? 0u : ~((1u << (8 * t)) - 1u);
}
__device__ __forceinline__ uint4 merge_from(uint4 v, uint4 w, uint32_t k) {
  uint4 o;
  o.x = (v.x & ~bytes_from(k, 0)) | (w.x & bytes_from(k, 0));
  o.y = (v.y & ~bytes_from(k, 1)) | (w.y & bytes_from(k, 1));
  o.z = (v.z & ~bytes_from(k, 2)) | (w.z & bytes_from(k, 2));
  o.w = (v.w & ~bytes_from(k, 3)) | (w.w & bytes_from(k, 3));
  return o;
}
// bytes [s, s + len) of v (s + len <= 16) stored at d with naturally aligned 1/2/4/8-B stores
__device__ __forceinline__ void store_part(uint8_t* d, uint4 v, uint32_t s, uint32_t len) {
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
  while (len) {
    const uintptr_t a = (uintptr_t)d;
    uint32_t p = 8;
    while (p > len || (a & (p - 1))) p >>= 1;
    uint64_t x = 0;
    for (uint32_t i = 0; i < p; i++) x |= (uint64_t)((w[(s + i) >> 2] >> (8 * ((s + i) & 3))) & 0xffu) << (8 * i);
    if (p == 8) *reinterpret_cast<uint64_t*>(d) = x;
    else if (p == 4) *reinterpret_cast<uint32_t*>(d) = (uint32_t)x;
    else if (p == 2) *reinterpret_cast<uint16_t*>(d) = (uint16_t)x;
    else *d = (uint8_t)x;
    d += p;
    s += p;
    len -= p;
  }
}

__global__ void __launch_bounds__(256) chunks(Blocks p) {
  __shared__ uint8_t own_all[4][kOwn];
  __shared__ uint32_t so1_all[4][2][kCap], dd_all[4][2][kCap];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, b = blockIdx.x * 4 + wave;
  if (b >= p.nb) return;
  uint8_t* own = own_all[wave];
  const uint32_t n = p.n[b], K = p.K[b], V = p.V[b];
  const uint32_t* meta = p.rec + (uint64_t)b * kCap;
  const uint32_t m0 = meta[lane];
  const uint32_t m1 = (uint32_t)__shfl((int)m0, (int)min(lane + 1, 63u));
  const uint8_t* blk = p.data + p.off[b];
  uint8_t* kb = p.kd + p.ek[b];
  uint8_t* vb = p.vd + p.ev[b];
  const uint32_t ak = (uint32_t)((uintptr_t)kb & 15u), av = (uint32_t)((uintptr_t)vb & 15u);
  const uint32_t CK = (K + ak + 15) >> 4, CV = (V + av + 15) >> 4;
  // entry lane e: its key stream range [ko, ko1) and value range [vo, vo1), and the input
  // address bases (input byte of stream byte x = D + x)
  const uint32_t hp = m0 & 0xffffu, vo = m0 >> 16, hp1 = m1 & 0xffffu, vo1 = m1 >> 16;
  const uint32_t vl = vo1 - vo, kl = hp1 - hp - 10 - vl, ko = hp - 10 * lane - vo, ko1 = ko + kl;
  const bool ent = lane < n;
  if (ent) {
    so1_all[wave][0][lane] = ko1;
    dd_all[wave][0][lane] = hp + 10 - ko;
    so1_all[wave][1][lane] = vo1;
    dd_all[wave][1][lane] = hp1 - vo1;
    // owner marks: chunk c >= 1 starts at stream byte 16 c - a; chunk 0 at byte 0
    const uint32_t k_lo = ko == 0 ? 0u : (ko + ak + 15) >> 4, k_hi = kl ? (ko1 + ak + 15) >> 4 : k_lo;
    const uint32_t v_lo = vo == 0 ? 0u : (vo + av + 15) >> 4, v_hi = vl ? (vo1 + av + 15) >> 4 : v_lo;
    for (uint32_t c = k_lo; c < k_hi; c++) own[c] = (uint8_t)lane;
    for (uint32_t c = v_lo; c < v_hi; c++) own[CK + c] = (uint8_t)lane;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  for (uint32_t c = lane; c < CK + CV; c += 64) {
    const bool key = c < CK;
    const uint32_t cc = key ? c : c - CK, a = key ? ak : av, S = key ? K : V, s = key ? 0u : 1u;
    const uint32_t x0 = cc ? 16 * cc - a : 0u;                 // first stream byte of the chunk
    const uint32_t L = min(cc ? 16u : 16u - a, S - x0);        // its bytes
    uint32_t e = own[c];
    uint4 v;
    __builtin_memcpy(&v, blk + dd_all[wave][s][e] + x0, 16);
    uint32_t k = so1_all[wave][s][e] - x0;
    while (k < L) {  // the chunk runs into entry e + 1
      e++;
      uint4 w;
      __builtin_memcpy(&w, blk + dd_all[wave][s][e] + x0, 16);
      v = merge_from(v, w, k);
      k = so1_all[wave][s][e] - x0;
    }
    uint8_t* d = (key ? kb : vb) + x0;
    if (L == 16) *reinterpret_cast<uint4*>(d) = v;
    else store_part(d, v, 0, L);
  }
}

int main() {
  // C2-shaped blocks: entries of 10 + 16 + vs bytes until the block reaches 4 KiB (Builder's
  // byte target), a 13-B terminator after each block
  srand(7);
  std::vector<uint8_t> data;
  std::vector<uint32_t> off, nn, rec, KK, VV, ens;
  std::vector<uint64_t> ek, ev;
  const uint64_t target = 1ull << 30;
  uint64_t kt = 0, vt = 0;
  while (data.size() < target) {
    const uint32_t o = (uint32_t)data.size();
    uint32_t pos = 0, V = 0, n = 0;
    std::vector<uint8_t> blk;
    std::vector<uint32_t> r;
    while (pos < 4096 - 150 && n < 63) {
      const uint32_t u = rand() % 100;
      const uint32_t vn = u < 10 ? 1 + rand() % 10 : 1;
      const uint32_t vl = 2 + vn + (u >= 10 && u < 15 ? 12 : 100);
      r.push_back(pos | (V << 16));
      for (uint32_t i = 0; i < 10 + 16 + vl; i++) blk.push_back((uint8_t)rand());
      pos += 10 + 16 + vl;
      V += vl;
      n++;
    }
    r.push_back(pos | (V << 16));
    for (int i = 0; i < 13; i++) blk.push_back(0);
    r.resize(kCap, 0);
    data.insert(data.end(), blk.begin(), blk.end());
    off.push_back(o);
    ens.push_back((uint32_t)(kt / 16));
    nn.push_back(n);
    rec.insert(rec.end(), r.begin(), r.end());
    KK.push_back(16 * n);
    VV.push_back(V);
    ek.push_back(kt);
    ev.push_back(vt);
    kt += 16 * n;
    vt += V;
  }
  const uint32_t nb = (uint32_t)off.size();
  // host reference
  std::vector<uint8_t> kref(kt), vref(vt);
  for (uint32_t b = 0; b < nb; b++) {
    const uint32_t* r = &rec[(size_t)b * kCap];
    for (uint32_t e = 0; e < nn[b]; e++) {
      const uint32_t hp = r[e] & 0xffff, vo = r[e] >> 16, hp1 = r[e + 1] & 0xffff, vo1 = r[e + 1] >> 16;
      const uint32_t vl = vo1 - vo, kl = hp1 - hp - 10 - vl;
      memcpy(&kref[ek[b] + 16 * e], &data[off[b] + hp + 10], kl);
      memcpy(&vref[ev[b] + vo], &data[off[b] + hp + 10 + kl], vl);
    }
  }
  uint8_t *d_data, *kd, *vd;
  uint32_t *d_off, *d_n, *d_rec, *d_K, *d_V, *d_en, *d_ke, *d_ve;
  uint64_t *d_ek, *d_ev;
  (void)hipMalloc(&d_data, data.size() + 64);
  (void)hipMalloc(&kd, kt + 64);
  (void)hipMalloc(&vd, vt + 64);
  (void)hipMalloc(&d_off, nb * 4);
  (void)hipMalloc(&d_n, nb * 4);
  (void)hipMalloc(&d_K, nb * 4);
  (void)hipMalloc(&d_V, nb * 4);
  (void)hipMalloc(&d_rec, rec.size() * 4);
  (void)hipMalloc(&d_ek, nb * 8);
  (void)hipMalloc(&d_ev, nb * 8);
  (void)hipMalloc(&d_en, nb * 4);
  (void)hipMalloc(&d_ke, kt / 16 * 4 + 64);
  (void)hipMalloc(&d_ve, kt / 16 * 4 + 64);
  (void)hipMemcpy(d_en, ens.data(), nb * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_data, data.data(), data.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(d_off, off.data(), nb * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_n, nn.data(), nb * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_K, KK.data(), nb * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_V, VV.data(), nb * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_rec, rec.data(), rec.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_ek, ek.data(), nb * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_ev, ev.data(), nb * 8, hipMemcpyHostToDevice);
  Blocks p{d_data, d_off, d_n, d_rec, d_ek, d_ev, d_K, d_V, kd, vd, nb, d_en, d_ke, d_ve};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  printf("%u blocks, %zu B input, %llu key + %llu value bytes\n", nb, data.size(),
         (unsigned long long)kt, (unsigned long long)vt);
  const double bytes = (double)(kt + vt) * 2;
  const char* names[] = {"pieces", "chunks", "pieces_eo", "pieces_eo_xcd", "pieces_xcd"};
  const uint32_t grid = (nb + 31) / 32 * 8;  // a multiple of 8 workgroups
  uint64_t bad_all = 0;
  for (int round = 0; round < 2; round++) {
    for (int v = 0; v < 5; v++) {
      (void)hipMemset(kd, 0, kt);
      (void)hipMemset(vd, 0, vt);
      float best = 1e9, sum = 0;
      for (int r = 0; r < 11; r++) {
        (void)hipEventRecord(e0);
        if (v == 0) hipLaunchKernelGGL((pieces<false, false>), dim3(grid), dim3(256), 0, 0, p);
        else if (v == 1) hipLaunchKernelGGL(chunks, dim3(grid), dim3(256), 0, 0, p);
        else if (v == 2) hipLaunchKernelGGL((pieces<true, false>), dim3(grid), dim3(256), 0, 0, p);
        else if (v == 3) hipLaunchKernelGGL((pieces<true, true>), dim3(grid), dim3(256), 0, 0, p);
        else hipLaunchKernelGGL((pieces<false, true>), dim3(grid), dim3(256), 0, 0, p);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (r) {
          best = ms < best ? ms : best;
          sum += ms;
        }
      }
      std::vector<uint8_t> k2(kt), v2(vt);
      (void)hipMemcpy(k2.data(), kd, kt, hipMemcpyDeviceToHost);
      (void)hipMemcpy(v2.data(), vd, vt, hipMemcpyDeviceToHost);
      uint64_t bad = 0;
      for (uint64_t i = 0; i < kt; i++) bad += k2[i] != kref[i];
      for (uint64_t i = 0; i < vt; i++) bad += v2[i] != vref[i];
      bad_all += bad;
      printf("%-13s best %.4f ms mean %.4f ms  %.0f GB/s  mismatching bytes %llu\n", names[v], best, sum / 10,
             bytes / (best / 1e3) / 1e9, (unsigned long long)bad);
    }
  }
  return bad_all != 0;
}
