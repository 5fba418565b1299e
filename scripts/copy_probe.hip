// copy_probe.hip -- what a device copy of the decode's size can reach on gfx950, to know how far
// the walk-scan-copy copy kernel (~4.8 TB/s read + write) is from the ceiling.  Variants over a
// 1 GiB source -> 1 GiB destination: 16 B per lane grid-stride, 4 x 16 B per lane unrolled,
// the same with non-temporal stores, plus read-only (xor-reduce) and write-only streams.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/copy_probe scripts/copy_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void __launch_bounds__(256) copy16(const uint4* __restrict__ s, uint4* __restrict__ d,
                                              size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    d[i] = s[i];
}

template <bool NT>
__global__ void __launch_bounds__(256) copy64(const uint4* __restrict__ s, uint4* __restrict__ d,
                                              size_t n) {
  // 4 consecutive 1 KiB wave pieces per wave iteration
  const size_t stride = (size_t)gridDim.x * 1024;
  for (size_t b = blockIdx.x * 1024ull; b < n; b += stride) {
    uint4 v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const size_t i = b + j * 256 + threadIdx.x;
      v[j] = i < n ? s[i] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const size_t i = b + j * 256 + threadIdx.x;
      if (i < n) {
        if (NT) {
          typedef unsigned u4 __attribute__((ext_vector_type(4)));
          u4 w = {v[j].x, v[j].y, v[j].z, v[j].w};
          __builtin_nontemporal_store(w, reinterpret_cast<u4*>(d + i));
        }
        else d[i] = v[j];
      }
    }
  }
}

__global__ void __launch_bounds__(256) read64(const uint4* __restrict__ s, uint32_t* out, size_t n) {
  uint32_t acc = 0;
  const size_t stride = (size_t)gridDim.x * 1024;
  for (size_t b = blockIdx.x * 1024ull; b < n; b += stride) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const size_t i = b + j * 256 + threadIdx.x;
      if (i < n) {
        const uint4 v = s[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
      }
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void __launch_bounds__(256) write64(uint4* __restrict__ d, size_t n) {
  const size_t stride = (size_t)gridDim.x * 1024;
  for (size_t b = blockIdx.x * 1024ull; b < n; b += stride) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const size_t i = b + j * 256 + threadIdx.x;
      if (i < n) d[i] = make_uint4((uint32_t)i, 1, 2, 3);
    }
  }
}

// the walk's access pattern without its dependency: thread t owns 4 KiB block t and reads one
// 8-B word per 128-B line, line by line (every lane of a wave in a different block)
__global__ void __launch_bounds__(256) lines_lane(const uint8_t* __restrict__ s, uint32_t* out,
                                                  size_t nblk) {
  uint32_t acc = 0;
  for (size_t t = blockIdx.x * 256ull + threadIdx.x; t < nblk; t += (size_t)gridDim.x * 256) {
    const uint8_t* b = s + t * 4096;
#pragma unroll 8
    for (int j = 0; j < 32; j++) acc ^= *reinterpret_cast<const uint32_t*>(b + j * 128 + 40);
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// the same lines read coalesced: lane j of a half-wave reads line j of one block
__global__ void __launch_bounds__(256) lines_coal(const uint8_t* __restrict__ s, uint32_t* out,
                                                  size_t nblk) {
  uint32_t acc = 0;
  const uint32_t j = threadIdx.x & 31;
  for (size_t t = blockIdx.x * 8ull + (threadIdx.x >> 5); t < nblk; t += (size_t)gridDim.x * 8)
    acc ^= *reinterpret_cast<const uint32_t*>(s + t * 4096 + j * 128 + 40);
  if (acc == 0x12345678u) out[0] = acc;
}

// 16-B pieces at unaligned source and destination addresses (the copy kernel's pieces are)
__global__ void __launch_bounds__(256) copy16u(const uint8_t* __restrict__ s, uint8_t* __restrict__ d,
                                               size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    uint4 v;
    __builtin_memcpy(&v, s + 16 * i, 16);
    __builtin_memcpy(d + 16 * i, &v, 16);
  }
}

// C2-shaped entries (10-B header, 16-B key, 103-B value = 129 B) copied into a key stream and a
// value stream, 8 lanes per entry.  PIECES: the copy kernel's pieces (16 B, the last overlapping
// back inside the stream, stores unaligned).  ALIGNED: each stream range cut at 16-B output
// boundaries -- whole pieces stored aligned, the partial head / tail as two overlapping 8/4/2-B
// (or 1-B) stores inside the range.
constexpr uint32_t kEnt = 129, kKey = 16, kVal = 103;

__device__ __forceinline__ void small_copy(uint8_t* d, const uint8_t* s, uint32_t n) {
  // n in [1, 15]: two overlapping pieces of the largest power of two <= n
  if (n >= 8) {
    uint2 a, b;
    __builtin_memcpy(&a, s, 8);
    __builtin_memcpy(&b, s + n - 8, 8);
    __builtin_memcpy(d, &a, 8);
    __builtin_memcpy(d + n - 8, &b, 8);
  } else if (n >= 4) {
    uint32_t a, b;
    __builtin_memcpy(&a, s, 4);
    __builtin_memcpy(&b, s + n - 4, 4);
    __builtin_memcpy(d, &a, 4);
    __builtin_memcpy(d + n - 4, &b, 4);
  } else if (n >= 2) {
    uint16_t a, b;
    __builtin_memcpy(&a, s, 2);
    __builtin_memcpy(&b, s + n - 2, 2);
    __builtin_memcpy(d, &a, 2);
    __builtin_memcpy(d + n - 2, &b, 2);
  } else {
    d[0] = s[0];
  }
}

template <bool ALIGNED>
__global__ void __launch_bounds__(256) entry_copy(const uint8_t* __restrict__ s, uint8_t* __restrict__ kd,
                                                  uint8_t* __restrict__ vd, size_t nent) {
  const uint32_t j = threadIdx.x & 7;
  for (size_t e = blockIdx.x * 32ull + (threadIdx.x >> 3); e < nent; e += (size_t)gridDim.x * 32) {
    const uint8_t* src = s + e * kEnt + 10;
    if (j == 0) {  // the key: 16 B, aligned output
      uint4 v;
      __builtin_memcpy(&v, src, 16);
      *reinterpret_cast<uint4*>(kd + e * kKey) = v;
    }
    const uint8_t* vs = src + kKey;
    uint8_t* vo = vd + e * kVal;
    if (!ALIGNED) {
      for (uint32_t q = j; q < 7; q += 8) {  // pieces 0..6, lanes 0..6
        const uint32_t o = min(16 * q, kVal - 16);
        uint4 v;
        __builtin_memcpy(&v, vs + o, 16);
        __builtin_memcpy(vo + o, &v, 16);
      }
    } else {
      const size_t a = e * kVal, b = a + kVal;
      const size_t a1 = (a + 15) & ~15ull, b1 = b & ~15ull;  // whole pieces [a1, b1)
      const uint32_t nfull = (uint32_t)((b1 - a1) >> 4);
      // piece q: 0 = head [a, a1), 1 = tail [b1, b), 2.. = whole piece q - 2
      for (uint32_t q = j; q < nfull + 2; q += 8) {
        if (q == 0) {
          if (a1 > a) small_copy(vo, vs, (uint32_t)(a1 - a));
        } else if (q == 1) {
          if (b > b1) small_copy(vd + b1, vs + (b1 - a), (uint32_t)(b - b1));
        } else {
          const size_t o = a1 + 16ull * (q - 2);
          uint4 v;
          __builtin_memcpy(&v, vs + (o - a), 16);
          *reinterpret_cast<uint4*>(vd + o) = v;
        }
      }
    }
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  const size_t bytes = 1ull << 30, n = bytes / 16;
  uint4 *s, *d;
  uint32_t* o;
  CK(hipMalloc(&s, bytes));
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&o, 64));
  CK(hipMemset(s, 1, bytes));
  CK(hipMemset(d, 0, bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  int cus = 256;
  for (int grid_per_cu : {4, 8, 16, 32}) {
    const int grid = grid_per_cu * cus;
    for (int v = 0; v < 9; v++) {
      float best = 1e9f;
      for (int r = 0; r < 8; r++) {
        CK(hipEventRecord(a, 0));
        if (v == 0) hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, 0, s, d, n);
        if (v == 1) hipLaunchKernelGGL(copy64<false>, dim3(grid), dim3(256), 0, 0, s, d, n);
        if (v == 2) hipLaunchKernelGGL(copy64<true>, dim3(grid), dim3(256), 0, 0, s, d, n);
        if (v == 3) hipLaunchKernelGGL(read64, dim3(grid), dim3(256), 0, 0, s, o, n);
        if (v == 4) hipLaunchKernelGGL(write64, dim3(grid), dim3(256), 0, 0, d, n);
        if (v == 7)
          hipLaunchKernelGGL(copy16u, dim3(grid), dim3(256), 0, 0, (const uint8_t*)s + 5, (uint8_t*)d + 9, n - 1);
        if (v == 8)
          hipLaunchKernelGGL(copy16u, dim3(grid), dim3(256), 0, 0, (const uint8_t*)s + 5, (uint8_t*)d, n - 1);
        if (v == 5)
          hipLaunchKernelGGL(lines_lane, dim3(grid), dim3(256), 0, 0, (const uint8_t*)s, o, bytes / 4096);
        if (v == 6)
          hipLaunchKernelGGL(lines_coal, dim3(grid), dim3(256), 0, 0, (const uint8_t*)s, o, bytes / 4096);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r > 0 && ms < best) best = ms;
      }
      const double moved = (v <= 2 || v >= 7 ? 2.0 : 1.0) * (double)bytes;
      static const char* names[] = {"copy16", "copy64", "copy64-nt", "read", "write",
                                    "lines-lane", "lines-coal", "copy16-u59", "copy16-u50"};
      printf("grid %5d (%2d/CU) %-10s %.4f ms  %.2f TB/s\n", grid, grid_per_cu, names[v], best,
             moved / best / 1e9);
    }
  }
  {  // C2-shaped entry copies: the source is `s`, keys to the front of `d`, values after
    const size_t nent = bytes / kEnt;
    uint8_t* kd = (uint8_t*)d;
    uint8_t* vd = kd + ((nent * kKey + 255) & ~255ull);
    for (int grid_per_cu : {8, 16, 32, 64}) {
      for (int v = 0; v < 2; v++) {
        float best = 1e9f;
        for (int r = 0; r < 8; r++) {
          CK(hipEventRecord(a, 0));
          if (v == 0)
            hipLaunchKernelGGL(entry_copy<false>, dim3(grid_per_cu * cus), dim3(256), 0, 0, (const uint8_t*)s, kd, vd, nent);
          else
            hipLaunchKernelGGL(entry_copy<true>, dim3(grid_per_cu * cus), dim3(256), 0, 0, (const uint8_t*)s, kd, vd, nent);
          CK(hipEventRecord(b, 0));
          CK(hipEventSynchronize(b));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, a, b));
          if (r > 0 && ms < best) best = ms;
        }
        const double moved = (double)nent * (kKey + kVal) * 2.0;
        printf("entries grid %2d/CU %-8s %.4f ms  %.2f TB/s (read + write of keys and values)\n",
               grid_per_cu, v ? "aligned" : "pieces", best, moved / best / 1e9);
      }
    }
  }
  CK(hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0));
  CK(hipEventRecord(a, 0));
  CK(hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0));
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  printf("hipMemcpyDtoD %.4f ms  %.2f TB/s\n", ms, 2.0 * bytes / ms / 1e9);
  return 0;
}
