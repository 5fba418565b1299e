// sector_probe.hip -- does the L2 fetch less than a whole 128-B line for the walk's 8-B header
// reads under some cache policy?  1 GiB of 4,096-B "blocks", one lane per block reading 8 B at
// every 129-B stride (C2's entry size) -- either as a dependent chain (the next offset comes from
// the loaded word, as the walk's header chain) or independently -- with the load's cache-policy
// bits: default, nt, sc0 sc1, sc0 sc1 nt.  Timed with HIP events (best of 5); run it under
// rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum for the
// request sizes.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/sector_probe scripts/sector_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr uint32_t kBlk = 4096, kStride = 129, kEnt = 31;

template <int POL>
__device__ __forceinline__ uint2 load8(const uint8_t* p) {
  uint2 r;
  if constexpr (POL == 0) {
    asm volatile("global_load_dwordx2 %0, %1, off\n s_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
  } else if constexpr (POL == 1) {
    asm volatile("global_load_dwordx2 %0, %1, off nt\n s_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
  } else if constexpr (POL == 2) {
    asm volatile("global_load_dwordx2 %0, %1, off sc0 sc1\n s_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
  } else {
    asm volatile("global_load_dwordx2 %0, %1, off sc0 sc1 nt\n s_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
  }
  return r;
}

// dependent chain: the next offset is read from the loaded word (always kStride here, but the
// hardware cannot know it)
template <int POL>
__global__ void __launch_bounds__(256) chain(const uint8_t* __restrict__ d, uint64_t nblk,
                                             uint32_t* __restrict__ out) {
  const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= nblk) return;
  const uint8_t* blk = d + b * kBlk;
  uint32_t pos = 0, acc = 0;
  for (uint32_t i = 0; i < kEnt; i++) {
    const uint2 w = load8<POL>(blk + pos);
    acc += w.y;
    pos += w.x;  // the buffer holds kStride in every word's low half
  }
  out[b] = acc + pos;
}

__global__ void fill(uint32_t* d, uint64_t nwords) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < nwords; i += (uint64_t)gridDim.x * 256)
    d[i] = 0;
}
__global__ void plant(uint8_t* d, uint64_t nblk) {  // kStride as a LE u32 at every chain position
  const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= nblk) return;
  for (uint32_t i = 0; i < kEnt; i++) {
    uint8_t* p = d + b * kBlk + i * kStride;
    p[0] = kStride;
    p[1] = p[2] = p[3] = 0;
  }
}

int main() {
  const uint64_t bytes = 1ull << 30, nblk = bytes / kBlk;
  uint8_t* d;
  uint32_t* out;
  hipMalloc(&d, bytes + 64);
  hipMalloc(&out, nblk * 4);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint32_t*)d, (bytes + 64) / 4);
  hipLaunchKernelGGL(plant, dim3((nblk + 255) / 256), dim3(256), 0, 0, d, nblk);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"default", "nt", "sc0 sc1", "sc0 sc1 nt"};
  for (int pol = 0; pol < 4; pol++) {
    float best = 1e9f;
    for (int r = 0; r < 6; r++) {
      hipEventRecord(e0);
      const dim3 g((nblk + 255) / 256);
      if (pol == 0) hipLaunchKernelGGL(chain<0>, g, dim3(256), 0, 0, d, nblk, out);
      if (pol == 1) hipLaunchKernelGGL(chain<1>, g, dim3(256), 0, 0, d, nblk, out);
      if (pol == 2) hipLaunchKernelGGL(chain<2>, g, dim3(256), 0, 0, d, nblk, out);
      if (pol == 3) hipLaunchKernelGGL(chain<3>, g, dim3(256), 0, 0, d, nblk, out);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (r && ms < best) best = ms;
    }
    printf("chain %-11s %.4f ms  (%.0f GB/s of input)\n", names[pol], best, bytes / (best / 1e3) / 1e9);
  }
  uint32_t h[4];
  hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
  printf("check %u\n", h[0]);
  return 0;
}
