// residency_probe.hip -- how many workgroups of T threads and S bytes of dynamic LDS are
// co-resident per CU on this device (the persistent decode grid must never exceed it).
// Each workgroup arrives on a counter, then polls it (bounded by s_memrealtime) and records
// the largest value it saw: the number of workgroups running at the same time.
// Build: hipcc --offload-arch=gfx950 -O2 -o scripts/residency_probe scripts/residency_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void probe(unsigned* ctr, unsigned* seen) {
  extern __shared__ unsigned char lds[];
  if (threadIdx.x == 0) {
    lds[0] = 1;
    unsigned v = atomicAdd(ctr, 1u) + 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
    unsigned best = v;
    while (__builtin_amdgcn_s_memrealtime() - t0 < 200000ull) {      // 2 ms
      v = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      best = v > best ? v : best;
      __builtin_amdgcn_s_sleep(4);
    }
    atomicMax(seen, best);
    atomicSub(ctr, 1u);  // departure: the counter is the number running right now
  }
}

int main(int argc, char** argv) {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  unsigned *ctr, *seen;
  hipMalloc(&ctr, 4);
  hipMalloc(&seen, 4);
  hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  const int threads[] = {64, 128, 256};
  const int sizes[] = {16384, 32768, 37408, 40960, 49152, 53248, 54112, 54272, 54784,
                       55296, 65536, 81920, 81921, 98304};
  printf("cus %d lds_per_block_max %zu\n", cus, (size_t)prop.sharedMemPerBlock);
  for (int t : threads) {
    for (int s : sizes) {
      int api = 0;
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&api, probe, t, s);
      const unsigned grid = cus * 8;
      hipMemset(ctr, 0, 4);
      hipMemset(seen, 0, 4);
      hipLaunchKernelGGL(probe, dim3(grid), dim3(t), s, 0, ctr, seen);
      hipError_t e = hipDeviceSynchronize();
      unsigned h = 0;
      hipMemcpy(&h, seen, 4, hipMemcpyDeviceToHost);
      printf("threads %4d lds %6d api_per_cu %d resident %5u = %.2f per CU %s\n", t, s, api, h,
             (double)h / cus, e == hipSuccess ? "" : hipGetErrorString(e));
    }
  }
  return 0;
}
