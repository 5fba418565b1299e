// align_probe.hip -- does an output-aligned copy of C2-shaped entries beat the copy kernel's
// unaligned 16-B pieces when both read each block's lines once (one wave per block of 32 uniform
// 129-B entries: 10 B header, 16 B key, 103 B value -> a dense key stream and a dense value
// stream; 32 x 103 B = 206 whole 16-B chunks, so each block's value range is 16-B aligned)?
//   pieces : 8 lanes per entry, lane 0 the key, lanes 1-7 the value's 16-B pieces (the last
//            overlapping back): unaligned stores, the wsc_copy_kernel pattern
//   aligned: keys one lane each (aligned 16-B stores); the value range as 206 ALIGNED 16-B
//            chunks, one lane each, bytes from one or two entries (two unaligned loads merged
//            under byte masks)
//   aligned_pf: the same with every load of the block issued before its first store
//   dense  : unaligned 16-B pieces as the pieces variant writes them (each inside its entry, the
//            last overlapping back), but packed one per lane: 64 consecutive value pieces per
//            store instruction (keys one lane each) -- density without alignment
// (merge_store_probe.hip's merged variant fetched every input line twice: keys and values were
// handled in separate passes of its grid-stride loop.)
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/align_probe scripts/align_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

constexpr uint32_t kEnt = 129, kKey = 16, kVal = 103, kPer = 32, kChunks = kPer * kVal / 16;

__device__ __forceinline__ uint4 ld16(const uint8_t* p) {
  uint4 v;
  __builtin_memcpy(&v, p, 16);
  return v;
}
__device__ __forceinline__ void st16(uint8_t* p, uint4 v) { __builtin_memcpy(p, &v, 16); }

__device__ __forceinline__ uint32_t bmask(int32_t x, int d) {  // bytes of dword d below x
  const int32_t k = x - 4 * d;
  return k >= 4 ? 0xffffffffu : k <= 0 ? 0u : (1u << (8 * k)) - 1u;
}

__global__ void __launch_bounds__(256) pieces(const uint8_t* __restrict__ s, uint8_t* __restrict__ kd,
                                              uint8_t* __restrict__ vd, uint32_t nb) {
  const uint32_t lane = threadIdx.x & 63, w0 = (blockIdx.x * 256 + threadIdx.x) >> 6, nw = gridDim.x * 4;
  const uint32_t g = lane >> 3, j = lane & 7;
  for (uint32_t b = w0; b < nb; b += nw) {
    const uint8_t* bs = s + (uint64_t)b * kPer * kEnt;
    for (uint32_t e = g; e < kPer; e += 8) {
      const uint8_t* src = bs + e * kEnt + 10;
      if (j == 0) {
        st16(kd + ((uint64_t)b * kPer + e) * kKey, ld16(src));
      } else {
        const uint32_t o = min(16u * (j - 1), kVal - 16);
        st16(vd + ((uint64_t)b * kPer + e) * kVal + o, ld16(src + kKey + o));
      }
    }
  }
}

template <bool PF>
__global__ void __launch_bounds__(256) aligned(const uint8_t* __restrict__ s, uint8_t* __restrict__ kd,
                                               uint8_t* __restrict__ vd, uint32_t nb) {
  const uint32_t lane = threadIdx.x & 63, w0 = (blockIdx.x * 256 + threadIdx.x) >> 6, nw = gridDim.x * 4;
  for (uint32_t b = w0; b < nb; b += nw) {
    const uint8_t* bs = s + (uint64_t)b * kPer * kEnt;
    uint8_t* vb = vd + (uint64_t)b * kChunks * 16;
    constexpr int kPass = (kChunks + 63) / 64;
    uint4 a[kPass], c2[kPass];
    int32_t x[kPass];
    uint4 key = make_uint4(0, 0, 0, 0);
    if (lane < kPer) key = ld16(bs + lane * kEnt + 10);
    if (!PF && lane < kPer) st16(kd + ((uint64_t)b * kPer + lane) * kKey, key);
#pragma unroll
    for (int p = 0; p < kPass; p++) {
      const uint32_t c = lane + 64 * p;
      x[p] = 16;
      if (c < kChunks) {
        const uint32_t w = 16 * c;
        const uint32_t e = (w * 10181u) >> 20;  // w / 103 for w < 4,096
        const uint32_t o = w - e * kVal;
        x[p] = (int32_t)min(16u, kVal - o);
        const uint8_t* pe = bs + e * kEnt + 10 + kKey;
        a[p] = ld16(pe + o);
        if (x[p] < 16) c2[p] = ld16(pe + kEnt - x[p]);
      }
      if (!PF && c < kChunks) {
        uint4 out = a[p];
        if (x[p] < 16) {
          out.x = (a[p].x & bmask(x[p], 0)) | (c2[p].x & ~bmask(x[p], 0));
          out.y = (a[p].y & bmask(x[p], 1)) | (c2[p].y & ~bmask(x[p], 1));
          out.z = (a[p].z & bmask(x[p], 2)) | (c2[p].z & ~bmask(x[p], 2));
          out.w = (a[p].w & bmask(x[p], 3)) | (c2[p].w & ~bmask(x[p], 3));
        }
        *reinterpret_cast<uint4*>(vb + 16 * c) = out;
      }
    }
    if (PF) {
      if (lane < kPer) st16(kd + ((uint64_t)b * kPer + lane) * kKey, key);
#pragma unroll
      for (int p = 0; p < kPass; p++) {
        const uint32_t c = lane + 64 * p;
        if (c >= kChunks) continue;
        uint4 out = a[p];
        if (x[p] < 16) {
          out.x = (a[p].x & bmask(x[p], 0)) | (c2[p].x & ~bmask(x[p], 0));
          out.y = (a[p].y & bmask(x[p], 1)) | (c2[p].y & ~bmask(x[p], 1));
          out.z = (a[p].z & bmask(x[p], 2)) | (c2[p].z & ~bmask(x[p], 2));
          out.w = (a[p].w & bmask(x[p], 3)) | (c2[p].w & ~bmask(x[p], 3));
        }
        *reinterpret_cast<uint4*>(vb + 16 * c) = out;
      }
    }
  }
}

__global__ void __launch_bounds__(256) dense(const uint8_t* __restrict__ s, uint8_t* __restrict__ kd,
                                             uint8_t* __restrict__ vd, uint32_t nb) {
  const uint32_t lane = threadIdx.x & 63, w0 = (blockIdx.x * 256 + threadIdx.x) >> 6, nw = gridDim.x * 4;
  constexpr uint32_t kPieces = (kVal + 15) / 16;  // 7 per value
  for (uint32_t b = w0; b < nb; b += nw) {
    const uint8_t* bs = s + (uint64_t)b * kPer * kEnt;
    if (lane < kPer)
      st16(kd + ((uint64_t)b * kPer + lane) * kKey, ld16(bs + lane * kEnt + 10));
    for (uint32_t c = lane; c < kPer * kPieces; c += 64) {
      const uint32_t e = c / kPieces, j = c - e * kPieces;
      const uint32_t o = min(16u * j, kVal - 16);
      st16(vd + ((uint64_t)b * kPer + e) * kVal + o, ld16(bs + e * kEnt + 10 + kKey + o));
    }
  }
}

int main() {
  const uint32_t nb = (uint32_t)((1ull << 30) / (kPer * kEnt));
  const uint64_t n = (uint64_t)nb * kPer;
  uint8_t *s, *kd, *vd, *kd2, *vd2;
  (void)hipMalloc(&s, n * kEnt + 64);
  (void)hipMalloc(&kd, n * kKey + 64);
  (void)hipMalloc(&vd, n * kVal + 64);
  (void)hipMalloc(&kd2, n * kKey + 64);
  (void)hipMalloc(&vd2, n * kVal + 64);
  uint8_t* h = (uint8_t*)malloc(n * kEnt);
  for (uint64_t i = 0; i < n * kEnt; i++) h[i] = (uint8_t)(i * 2654435761u >> 13);
  (void)hipMemcpy(s, h, n * kEnt, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const double bytes = 2.0 * n * (kKey + kVal);
  const char* names[] = {"pieces", "aligned", "aligned_pf", "dense"};
  for (int wg : {1024, 2048, 4096, 8192}) {
    for (int v = 0; v < 4; v++) {
      float best = 1e9;
      for (int r = 0; r < 7; r++) {
        (void)hipEventRecord(e0);
        if (v == 0) hipLaunchKernelGGL(pieces, dim3(wg), dim3(256), 0, 0, s, kd, vd, nb);
        else if (v == 1) hipLaunchKernelGGL(aligned<false>, dim3(wg), dim3(256), 0, 0, s, kd2, vd2, nb);
        else if (v == 2) hipLaunchKernelGGL(aligned<true>, dim3(wg), dim3(256), 0, 0, s, kd2, vd2, nb);
        else hipLaunchKernelGGL(dense, dim3(wg), dim3(256), 0, 0, s, kd2, vd2, nb);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (r && ms < best) best = ms;
      }
      printf("%-10s grid %5d: %.4f ms  %.0f GB/s (read + write of keys and values)\n", names[v], wg,
             best, bytes / (best / 1e3) / 1e9);
    }
  }
  uint8_t* a = (uint8_t*)malloc(n * kVal);
  uint8_t* b = (uint8_t*)malloc(n * kVal);
  (void)hipMemcpy(a, vd, n * kVal, hipMemcpyDeviceToHost);
  (void)hipMemcpy(b, vd2, n * kVal, hipMemcpyDeviceToHost);
  uint64_t bad = 0;
  for (uint64_t i = 0; i < n * kVal; i++) bad += a[i] != b[i];
  (void)hipMemcpy(a, kd, n * kKey, hipMemcpyDeviceToHost);
  (void)hipMemcpy(b, kd2, n * kKey, hipMemcpyDeviceToHost);
  for (uint64_t i = 0; i < n * kKey; i++) bad += a[i] != b[i];
  printf("mismatching bytes: %llu\n", (unsigned long long)bad);
  return bad != 0;
}
