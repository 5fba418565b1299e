// stage_probe.hip -- what sets the 0.24 ms load floor of the LDS-staged walks?
// 1 GiB of 4,012-B blocks (the C2 block size, consecutive, so every block has its own 16-B
// shift), read with the streaming walk's access pattern, one ingredient added at a time:
//   grid      grid-stride 16-B reads, 4 per lane (the copy probe's `read`, the reference)
//   tile      256 threads per 256-block tile, 8 blocks per sub-batch, thread t reads chunk t
//             (and 256/257) of each block, next sub-batch issued before this one is consumed
//   tile+lds  + the sub-batch's lines written to LDS slots (no barrier)
//   tile+bar  + __syncthreads before and after the LDS writes (the stream walk's loop)
//   tile+off  + block offsets read from LDS (s_off) to form the next sub-batch's addresses
//   wave      one wave per block, 64 blocks per wave in order, 2 blocks in flight (the scan
//             walk's loop), lines to a per-wave LDS slot
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/stage_probe scripts/stage_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                        \
    }                                                                  \
  } while (0)

constexpr uint32_t kBlk = 4012, kSub = 8, kTile = 256, kSlot = 4128;

__device__ __forceinline__ uint4 line(const uint8_t* d, uint64_t len, uint64_t off, uint32_t c) {
  const uint64_t last = (len - 16) & ~15ull;
  uint64_t a = (off & ~15ull) + 16ull * c;
  a = a < last ? a : last;
  return *reinterpret_cast<const uint4*>(d + a);
}
__device__ __forceinline__ uint32_t fold(uint4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

__global__ void __launch_bounds__(256) k_grid(const uint4* __restrict__ s, uint32_t* out, size_t n) {
  uint32_t acc = 0;
  for (size_t b = blockIdx.x * 1024ull; b < n; b += (size_t)gridDim.x * 1024) {
    uint4 v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const size_t i = b + j * 256 + threadIdx.x;
      v[j] = i < n ? s[i] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; j++) acc ^= fold(v[j]);
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// MODE 0 tile, 1 tile+lds, 2 tile+bar, 3 tile+off
template <int MODE>
__global__ void __launch_bounds__(256) k_tile(const uint8_t* __restrict__ d, uint64_t len,
                                              uint32_t nblk, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kSub * kSlot];
  __shared__ uint32_t s_off[kTile];
  const uint32_t tid = threadIdx.x, b0 = blockIdx.x * kTile;
  const uint32_t nb = min(kTile, nblk - b0);
  if (MODE >= 3) {
    s_off[tid] = (b0 + min(tid, nb - 1)) * kBlk;
    __syncthreads();
  }
  auto off_of = [&](uint32_t bi) -> uint64_t {
    return MODE >= 3 ? (uint64_t)s_off[bi] : (uint64_t)(b0 + bi) * kBlk;
  };
  uint4 R[kSub];
  uint32_t acc = 0;
  auto issue = [&](uint32_t j) {
#pragma unroll
    for (uint32_t i = 0; i < kSub; i++) R[i] = line(d, len, off_of(min(j * kSub + i, nb - 1)), tid);
  };
  const uint32_t nsub = (nb + kSub - 1) / kSub;
  issue(0);
  for (uint32_t j = 0; j < nsub; j++) {
    if (MODE >= 2) __syncthreads();
    uint4 C[kSub];
#pragma unroll
    for (uint32_t i = 0; i < kSub; i++) C[i] = R[i];
    if (MODE >= 1) {
#pragma unroll
      for (uint32_t i = 0; i < kSub; i++) *reinterpret_cast<uint4*>(lds + i * kSlot + 16 * tid) = C[i];
    }
    if (MODE >= 2) __syncthreads();
    if (j + 1 < nsub) issue(j + 1);
    if (MODE >= 1) {
      acc ^= *reinterpret_cast<const uint32_t*>(lds + (tid & 7) * kSlot + 4 * (tid >> 3));
    } else {
#pragma unroll
      for (uint32_t i = 0; i < kSub; i++) acc ^= fold(C[i]);
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void __launch_bounds__(256) k_wave(const uint8_t* __restrict__ d, uint64_t len,
                                              uint32_t nblk, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4 * kSlot];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t i0 = blockIdx.x * kTile + wave * 64;
  const uint32_t i1 = min(i0 + 64, nblk);
  uint8_t* slot = lds + wave * kSlot;
  uint4 R0[5], R1[5];
  uint32_t acc = 0;
  auto issue = [&](uint32_t b, uint4 (&R)[5]) {
#pragma unroll
    for (uint32_t q = 0; q < 5; q++) R[q] = line(d, len, (uint64_t)b * kBlk, lane + 64 * q);
  };
  auto take = [&](uint32_t b, uint4 (&R)[5]) {
#pragma unroll
    for (uint32_t q = 0; q < 5; q++)
      if (q < 4 || lane < 2) *reinterpret_cast<uint4*>(slot + 16 * (lane + 64 * q)) = R[q];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (b + 2 < i1) issue(b + 2, R);
    acc ^= *reinterpret_cast<const uint32_t*>(slot + 4 * lane);
  };
  if (i0 >= i1) return;
  issue(i0, R0);
  if (i0 + 1 < i1) issue(i0 + 1, R1);
  for (uint32_t b = i0; b < i1; b += 2) {
    take(b, R0);
    if (b + 1 < i1) take(b + 1, R1);
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const uint32_t nblk = (uint32_t)((1ull << 30) / kBlk);
  const uint64_t len = (uint64_t)nblk * kBlk + 64;
  uint8_t* d;
  uint32_t* out;
  CK(hipMalloc(&d, len));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(d, 1, len));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const uint32_t tiles = (nblk + kTile - 1) / kTile;
  const char* names[] = {"grid", "tile", "tile+lds", "tile+bar", "tile+off", "wave"};
  for (int v = 0; v < 6; v++) {
    float best = 1e9f;
    for (int r = 0; r < 7; r++) {
      CK(hipEventRecord(a, 0));
      if (v == 0) hipLaunchKernelGGL(k_grid, dim3(4 * cus), dim3(256), 0, 0, (const uint4*)d, out, (size_t)(len / 16));
      if (v == 1) hipLaunchKernelGGL(k_tile<0>, dim3(tiles), dim3(256), 0, 0, d, len, nblk, out);
      if (v == 2) hipLaunchKernelGGL(k_tile<1>, dim3(tiles), dim3(256), 0, 0, d, len, nblk, out);
      if (v == 3) hipLaunchKernelGGL(k_tile<2>, dim3(tiles), dim3(256), 0, 0, d, len, nblk, out);
      if (v == 4) hipLaunchKernelGGL(k_tile<3>, dim3(tiles), dim3(256), 0, 0, d, len, nblk, out);
      if (v == 5) hipLaunchKernelGGL(k_wave, dim3(tiles), dim3(256), 0, 0, d, len, nblk, out);
      CK(hipGetLastError());
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      if (r > 0 && ms < best) best = ms;
    }
    printf("%-10s %.4f ms  %.2f TB/s\n", names[v], best, (double)nblk * kBlk / (best / 1e3) / 1e12);
  }
  CK(hipFree(d));
  CK(hipFree(out));
  return 0;
}
