// lds_probe.hip -- cost of 16-B LDS accesses on gfx950 by address alignment (one wave per CU
// and 8 waves per CU): dependent-chain latency and independent throughput, in s_memtime cycles.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/lds_probe scripts/lds_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kIters = 256;

// mode 0: dependent reads (latency), 1: independent reads, 2: independent writes,
// 3: 5 x ds_read_b32 + alignbyte window (the old unaligned idiom), dependent
__global__ void probe(int mode, int mis, unsigned long long* out, unsigned* sink) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[65536];
  const unsigned lane = threadIdx.x & 63;
  for (unsigned i = threadIdx.x; i < 65536 / 4; i += blockDim.x) reinterpret_cast<unsigned*>(lds)[i] = i * 2654435761u;
  __syncthreads();
  unsigned base = (threadIdx.x >> 6) * 8192 + lane * 112 + mis;  // 112-B lane stride (entry-like)
  unsigned acc = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (mode == 0) {
    unsigned a = base;
    for (int i = 0; i < kIters; i++) {
      uint4 v;
      __builtin_memcpy(&v, lds + (a & 4095) + (threadIdx.x >> 6) * 8192, 16);
      a += (v.x & 1) + 16;  // dependent
      acc ^= v.y;
    }
  } else if (mode == 1) {
    for (int i = 0; i < kIters; i += 4) {
      uint4 v[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        uint4 t;
        __builtin_memcpy(&t, lds + ((base + 16 * (i + j)) & 8191), 16);
        v[j] = t;
      }
#pragma unroll
      for (int j = 0; j < 4; j++) acc ^= v[j].x ^ v[j].w;
    }
  } else if (mode == 2) {
    for (int i = 0; i < kIters; i++) {
      const uint4 v = make_uint4(i, i + 1, i + 2, lane);
      __builtin_memcpy(lds + ((base + 16 * i) & 8191) + (threadIdx.x >> 6) * 8192, &v, 16);
    }
  } else {
    unsigned a = base;
    for (int i = 0; i < kIters; i++) {
      const unsigned p = (a & 4095) + (threadIdx.x >> 6) * 8192;
      const unsigned* w = reinterpret_cast<const unsigned*>(lds + (p & ~3u));
      const unsigned r = p & 3u;
      const unsigned x = __builtin_amdgcn_alignbyte(w[1], w[0], r);
      const unsigned y = __builtin_amdgcn_alignbyte(w[2], w[1], r);
      const unsigned z = __builtin_amdgcn_alignbyte(w[3], w[2], r);
      const unsigned q = __builtin_amdgcn_alignbyte(w[4], w[3], r);
      a += (x & 1) + 16;
      acc ^= y ^ z ^ q;
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) atomicAdd(out, t1 - t0);
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  unsigned long long* out;
  unsigned* sink;
  hipMalloc(&out, 8);
  hipMalloc(&sink, 4);
  const char* names[] = {"dep read b128", "indep read b128", "indep write b128", "dep 5xb32+align"};
  for (int waves : {1, 8}) {
    for (int mode = 0; mode < 4; mode++) {
      for (int mis : {0, 4, 8, 1, 3, 10}) {
        hipMemset(out, 0, 8);
        hipLaunchKernelGGL(probe, dim3(256), dim3(64 * waves), 0, 0, mode, mis, out, sink);
        hipDeviceSynchronize();
        unsigned long long h = 0;
        hipMemcpy(&h, out, 8, hipMemcpyDeviceToHost);
        printf("waves/CU %d %-18s misalign %2d: %7.1f cycles per access per wave\n", waves,
               names[mode], mis, (double)h / (256.0 * waves) / kIters);
      }
    }
  }
  return 0;
}
