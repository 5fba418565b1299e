// walk_probe.hip -- cost per entry of the serial header walk (table/iterator.go:93-135 chain) on
// blocks resident in LDS, one lane per block, in s_memtime cycles: how fast can an LDS walk go on
// gfx950 with no other traffic?  Variants: 0 = the fused kernel's fast loop (record to LDS),
// 1 = no record store, 2 = bare chain (read, 2 perms, add); 3 / 4 / 5 = the same with three
// aligned ds_read_b32 + v_alignbyte instead of one misaligned ds_read_b64.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/walk_probe scripts/walk_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int kBlocks = 16;
constexpr int kSlot = 4128;

template <int V>
__global__ void __launch_bounds__(64) probe(unsigned long long* out, unsigned* sink, int reps) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[kBlocks * kSlot];
  __shared__ unsigned pool[kBlocks * 64];
  const unsigned lane = threadIdx.x;
  // C2-like blocks: 16-B keys, 103-B values (one in 8 entries 111 B), terminator
  if (lane < kBlocks) {
    unsigned char* b = lds + lane * kSlot;
    unsigned pos = 0, prev = 0xffffffffu, i = 0;
    for (;;) {
      const unsigned vl = (i % 8 == 5) ? 111 : 103;
      if (pos + 10 + 16 + vl + 13 > 4096) break;
      b[pos] = 0; b[pos + 1] = 0; b[pos + 2] = 0; b[pos + 3] = 16; b[pos + 4] = vl >> 8; b[pos + 5] = vl & 255;
      b[pos + 6] = prev >> 24; b[pos + 7] = prev >> 16; b[pos + 8] = prev >> 8; b[pos + 9] = prev;
      for (unsigned k = 0; k < 16 + vl; k++) b[pos + 10 + k] = (unsigned char)(k * 7 + i);
      prev = pos;
      pos += 26 + vl;
      i++;
    }
    for (unsigned k = 0; k < 13; k++) b[pos + k] = k == 5 ? 3 : 0;
    for (unsigned k = pos + 13; k < kSlot; k++) b[k] = 0xee;
  }
  __syncthreads();
  const unsigned len = 4096;
  unsigned acc = 0, steps = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; r++) {
    if (lane < kBlocks) {
      const unsigned char* sb = lds + lane * kSlot;
      unsigned pos = 0, n = 0, S = 0;
      for (;;) {
        uint2 hw;
        if (V >= 3) {  // aligned dwords + v_alignbyte
          const unsigned* w = reinterpret_cast<const unsigned*>(sb + (pos & ~3u));
          const unsigned w0 = w[0], w1 = w[1], w2 = w[2];
          hw.x = __builtin_amdgcn_alignbyte(w1, w0, pos & 3u);
          hw.y = __builtin_amdgcn_alignbyte(w2, w1, pos & 3u);
        } else {
          __builtin_memcpy(&hw, sb + pos, 8);
        }
        const unsigned plen = __builtin_amdgcn_perm(0u, hw.x, 0x0c0c0001u);
        const unsigned klen = __builtin_amdgcn_perm(0u, hw.x, 0x0c0c0203u);
        const unsigned vlen = __builtin_amdgcn_perm(0u, hw.y, 0x0c0c0001u);
        const unsigned end = pos + 10 + klen + vlen;
        if (V == 2 || V == 5) {
          if (klen == 0 || end > len) break;
        } else {
          if ((len - pos < 10) | (klen == 0) | (plen != 0) | (end > len) | (n >= 63)) break;
        }
        if (V == 0 || V == 3) pool[lane * 64 + n] = pos | (S << 16);
        S += klen;
        n++;
        pos = end;
      }
      acc += S + pos;
      steps += n;
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    out[blockIdx.x * 2] = t1 - t0;
    out[blockIdx.x * 2 + 1] = steps;
  }
  if (acc == 12345) sink[lane] = acc;
}

template <int V>
static void run(int grid, int reps) {
  unsigned long long* d;
  unsigned* s;
  (void)hipMalloc(&d, 2 * grid * sizeof(unsigned long long));
  (void)hipMalloc(&s, 256);
  hipLaunchKernelGGL(probe<V>, dim3(grid), dim3(64), 0, 0, d, s, reps);
  (void)hipDeviceSynchronize();
  unsigned long long h[2];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("variant %d grid %d: %.1f cycles per entry step (%llu steps of lane 0's walks)\n", V, grid,
         (double)h[0] / (double)(h[1] ? h[1] : 1), h[1]);
  (void)hipFree(d);
  (void)hipFree(s);
}

int main() {
  for (int grid : {1, 256, 768}) {
    run<0>(grid, 200);
    run<1>(grid, 200);
    run<2>(grid, 200);
    run<3>(grid, 200);
    run<4>(grid, 200);
    run<5>(grid, 200);
  }
  return 0;
}
