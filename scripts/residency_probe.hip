// residency_probe.hip -- how many workgroups of T threads and S bytes of dynamic LDS are
// co-resident per CU on this device (the persistent decode grid must never exceed it).
// Each workgroup arrives on a counter, then polls it (bounded by s_memrealtime) and records
// the largest value it saw: the number of workgroups running at the same time.
// Build: hipcc --offload-arch=gfx950 -O2 -o scripts/residency_probe scripts/residency_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

// V > 0: the kernel allocates at least V VGPRs (inline-asm clobbers), as a real kernel would
template <int V>
__global__ void probe(unsigned* ctr, unsigned* seen) {
  extern __shared__ unsigned char lds[];
  if constexpr (V >= 80) asm volatile("" ::: "v40", "v50", "v60", "v70", "v79");
  if constexpr (V >= 96) asm volatile("" ::: "v95");
  if constexpr (V >= 128) asm volatile("" ::: "v127");
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

// the lane walk's shape: 576 threads, 76,268 B of STATIC LDS, launch bounds 576
__global__ void __launch_bounds__(576) probe_static(unsigned* ctr, unsigned* seen) {
  __shared__ unsigned char big[76268];
  for (unsigned i = threadIdx.x; i < 76268; i += blockDim.x) big[i] = (unsigned char)i;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned v = atomicAdd(ctr, 1u) + 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned best = v;
    while (__builtin_amdgcn_s_memrealtime() - t0 < 200000ull) {
      v = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      best = v > best ? v : best;
      __builtin_amdgcn_s_sleep(4);
    }
    atomicMax(seen, best + (big[(v * 131u) % 76268u] == 255u ? 1u : 0u) * 0u + (big[77] != 77u));
    atomicSub(ctr, 1u);
  }
}

int main(int argc, char** argv) {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  unsigned *ctr, *seen;
  hipMalloc(&ctr, 4);
  hipMalloc(&seen, 4);
  hipFuncSetAttribute((const void*)probe<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  hipFuncSetAttribute((const void*)probe<80>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  hipFuncSetAttribute((const void*)probe<96>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  hipFuncSetAttribute((const void*)probe<128>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  const int threads[] = {576};
  const int sizes[] = {76156};
  printf("cus %d lds_per_block_max %zu\n", cus, (size_t)prop.sharedMemPerBlock);
  for (int t : threads) {
    for (int s : sizes) for (int vg : {0, 80, 96, 128}) {
      int api = 0;
      auto k = vg == 0 ? probe<0> : vg == 80 ? probe<80> : vg == 96 ? probe<96> : probe<128>;
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&api, k, t, s);
      const unsigned grid = cus * 8;
      hipMemset(ctr, 0, 4);
      hipMemset(seen, 0, 4);
      hipLaunchKernelGGL(k, dim3(grid), dim3(t), s, 0, ctr, seen);
      hipError_t e = hipDeviceSynchronize();
      unsigned h = 0;
      hipMemcpy(&h, seen, 4, hipMemcpyDeviceToHost);
      printf("threads %4d lds %6d vgprs>=%3d api_per_cu %d resident %5u = %.2f per CU %s\n", t, s, vg, api, h,
             (double)h / cus, e == hipSuccess ? "" : hipGetErrorString(e));
    }
  }
  {
    hipMemset(ctr, 0, 4);
    hipMemset(seen, 0, 4);
    hipLaunchKernelGGL(probe_static, dim3(cus * 4), dim3(576), 0, 0, ctr, seen);
    hipError_t e = hipDeviceSynchronize();
    unsigned h = 0;
    hipMemcpy(&h, seen, 4, hipMemcpyDeviceToHost);
    printf("static 576 threads lds 76268 resident %5u = %.2f per CU %s\n", h, (double)h / cus,
           e == hipSuccess ? "" : hipGetErrorString(e));
  }
  return 0;
}
