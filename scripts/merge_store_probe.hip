// merge_store_probe.hip -- does an aligned-destination copy of C2-shaped entries beat the
// copy kernel's unaligned 16-B pieces?  1 GiB of uniform 129-B entries (10 B header, 16 B key,
// 103 B value) -> a dense key stream (16 B each, aligned) and a dense value stream:
//   pieces : 8 lanes per entry, 16-B pieces, the last overlapping back (unaligned stores) --
//            the wsc_copy_kernel pattern
//   merged : one lane per ALIGNED 16-B output chunk of the value stream; its bytes come from one
//            or two entries: two unaligned loads, the second from (next value - x) so its bytes
//            already sit at their window positions, merged with v_bfi under byte masks
//   merged32: the same with 32-bit index math (entry = chunk * 16 / 103 by a float reciprocal and
//            one correction step; round 3's form divided 64-bit integers per lane)
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/merge_store_probe scripts/merge_store_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr uint32_t kEnt = 129, kKey = 16, kVal = 103;

__device__ __forceinline__ uint4 ld16(const uint8_t* p) {
  uint4 v;
  __builtin_memcpy(&v, p, 16);
  return v;
}

__global__ void __launch_bounds__(256) pieces(const uint8_t* __restrict__ s, uint8_t* __restrict__ kd,
                                              uint8_t* __restrict__ vd, uint64_t n) {
  const uint64_t gl = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t t = gl; t < n * 8; t += stride) {
    const uint64_t e = t >> 3;
    const uint32_t j = t & 7;
    const uint8_t* src = s + e * kEnt + 10;
    if (j == 0) {
      const uint4 v = ld16(src);
      __builtin_memcpy(kd + e * kKey, &v, 16);
    } else {
      const uint32_t o = min(16u * (j - 1), kVal - 16);
      const uint4 v = ld16(src + kKey + o);
      __builtin_memcpy(vd + e * kVal + o, &v, 16);
    }
  }
}

__device__ __forceinline__ uint32_t bmask(int32_t x, int d) {  // bytes of dword d below x
  const int32_t k = x - 4 * d;
  return k >= 4 ? 0xffffffffu : k <= 0 ? 0u : (1u << (8 * k)) - 1u;
}

__global__ void __launch_bounds__(256) merged(const uint8_t* __restrict__ s, uint8_t* __restrict__ kd,
                                              uint8_t* __restrict__ vd, uint64_t n) {
  const uint64_t gl = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  const uint64_t nk = n, nv = n * kVal / 16;  // key chunks, whole value chunks
  for (uint64_t t = gl; t < nk + nv; t += stride) {
    if (t < nk) {
      const uint4 v = ld16(s + t * kEnt + 10);
      *reinterpret_cast<uint4*>(kd + t * kKey) = v;
      continue;
    }
    const uint64_t c = t - nk, w = 16 * c;
    const uint64_t e = w / kVal;
    const uint32_t o = (uint32_t)(w - e * kVal);
    const int32_t x = (int32_t)min(16u, kVal - o);  // bytes from entry e
    const uint4 a = ld16(s + e * kEnt + 10 + kKey + o);
    uint4 out = a;
    if (x < 16 && e + 1 < n) {
      const uint4 b = ld16(s + (e + 1) * kEnt + 10 + kKey - x);
      out.x = (a.x & bmask(x, 0)) | (b.x & ~bmask(x, 0));
      out.y = (a.y & bmask(x, 1)) | (b.y & ~bmask(x, 1));
      out.z = (a.z & bmask(x, 2)) | (b.z & ~bmask(x, 2));
      out.w = (a.w & bmask(x, 3)) | (b.w & ~bmask(x, 3));
    }
    *reinterpret_cast<uint4*>(vd + w) = out;
  }
}

__global__ void __launch_bounds__(256) merged32(const uint8_t* __restrict__ s, uint8_t* __restrict__ kd,
                                                uint8_t* __restrict__ vd, uint32_t n) {
  const uint32_t gl = blockIdx.x * 256 + threadIdx.x;
  const uint32_t stride = gridDim.x * 256;
  const uint32_t nk = n, nv = (uint32_t)((uint64_t)n * kVal / 16);
  for (uint32_t t = gl; t < nk + nv; t += stride) {
    if (t < nk) {
      const uint4 v = ld16(s + (uint64_t)t * kEnt + 10);
      *reinterpret_cast<uint4*>(kd + (uint64_t)t * kKey) = v;
      continue;
    }
    const uint32_t c = t - nk, w = 16 * c;
    uint32_t e = (uint32_t)((float)w * (1.0f / kVal));
    if (e * kVal > w) e--;
    if ((e + 1) * kVal <= w) e++;
    const uint32_t o = w - e * kVal;
    const int32_t x = (int32_t)min(16u, kVal - o);
    const uint8_t* pe = s + (uint64_t)e * kEnt + 10 + kKey;
    const uint4 a = ld16(pe + o);
    uint4 out = a;
    if (x < 16 && e + 1 < n) {
      const uint4 b = ld16(pe + kEnt - x);
      out.x = (a.x & bmask(x, 0)) | (b.x & ~bmask(x, 0));
      out.y = (a.y & bmask(x, 1)) | (b.y & ~bmask(x, 1));
      out.z = (a.z & bmask(x, 2)) | (b.z & ~bmask(x, 2));
      out.w = (a.w & bmask(x, 3)) | (b.w & ~bmask(x, 3));
    }
    *reinterpret_cast<uint4*>(vd + w) = out;
  }
}

int main() {
  const uint64_t n = (1ull << 30) / kEnt;
  uint8_t *s, *kd, *vd, *kd2, *vd2;
  hipMalloc(&s, n * kEnt + 64);
  hipMalloc(&kd, n * kKey + 64);
  hipMalloc(&vd, n * kVal + 64);
  hipMalloc(&kd2, n * kKey + 64);
  hipMalloc(&vd2, n * kVal + 64);
  uint8_t* h = (uint8_t*)malloc(n * kEnt);
  for (uint64_t i = 0; i < n * kEnt; i++) h[i] = (uint8_t)(i * 2654435761u >> 13);
  hipMemcpy(s, h, n * kEnt, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double bytes = 2.0 * n * (kKey + kVal);
  for (int wg : {1024, 2048, 4096, 8192}) {
    for (int v = 0; v < 3; v++) {
      float best = 1e9;
      for (int r = 0; r < 7; r++) {
        hipEventRecord(e0);
        if (v == 0) hipLaunchKernelGGL(pieces, dim3(wg), dim3(256), 0, 0, s, kd, vd, n);
        else if (v == 1) hipLaunchKernelGGL(merged, dim3(wg), dim3(256), 0, 0, s, kd2, vd2, n);
        else hipLaunchKernelGGL(merged32, dim3(wg), dim3(256), 0, 0, s, kd2, vd2, (uint32_t)n);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (r && ms < best) best = ms;
      }
      printf("%-8s grid %5d: %.4f ms  %.0f GB/s (read + write of keys and values)\n",
             v == 2 ? "merged32" : v ? "merged" : "pieces", wg, best, bytes / (best / 1e3) / 1e9);
    }
  }
  // both variants wrote the same streams
  uint8_t* a = (uint8_t*)malloc(n * kVal);
  uint8_t* b = (uint8_t*)malloc(n * kVal);
  hipMemcpy(a, vd, n * kVal / 16 * 16, hipMemcpyDeviceToHost);
  hipMemcpy(b, vd2, n * kVal / 16 * 16, hipMemcpyDeviceToHost);
  uint64_t bad = 0;
  for (uint64_t i = 0; i < n * kVal / 16 * 16; i++) bad += a[i] != b[i];
  hipMemcpy(a, kd, n * kKey, hipMemcpyDeviceToHost);
  hipMemcpy(b, kd2, n * kKey, hipMemcpyDeviceToHost);
  for (uint64_t i = 0; i < n * kKey; i++) bad += a[i] != b[i];
  printf("mismatching bytes: %llu\n", (unsigned long long)bad);
  return bad != 0;
}
