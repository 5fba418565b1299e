// CPU harness for lsmdb_amd/csrc/copy_pool.hpp (tests/test_copy_pool.py): random sizes and
// offsets, 1..9 threads, pools reused across many copies; every byte checked.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "copy_pool.hpp"

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 200;
  std::mt19937_64 rng(7);
  std::vector<uint8_t> src(24u << 20), dst(24u << 20);
  for (auto& b : src) b = (uint8_t)rng();
  long fails = 0, copies = 0;
  for (unsigned th = 1; th <= 9; th += 2) {
    lsmgpu::CopyPool pool(th);
    for (int r = 0; r < rounds; r++) {
      const size_t n = rng() % 3 == 0 ? rng() % 4096 : rng() % (16u << 20);
      const size_t so = rng() % (src.size() - n), d0 = rng() % (dst.size() - n);
      pool.copy(dst.data() + d0, src.data() + so, n);
      copies++;
      for (size_t i = 0; i < n; i++)
        if (dst[d0 + i] != src[so + i]) {
          fails++;
          break;
        }
    }
  }
  printf("{\"copies\": %ld, \"fails\": %ld}\n", copies, fails);
  return fails ? 1 : 0;
}
