// open_tables.hip -- batched OpenTable index work on gfx950: for many
// SSTs resident in HBM at once, what table/table.go:88-144 does per table on the host.
//
//   tail    (lane = table)  readIndex's tail parse (table.go:177-199): bloom span, restart
//                           count, position of the restart array
//   scan    (rocPRIM)       block bases over tables
//   blocks  (lane = block)  restart -> [off, len) (table.go:202-215, monotone check), the first
//                           header and first key (table.go:219-246: plen == 0 asserted, reads
//                           bounded by the file as t.read is)
//   sorted  (lane = block)  is the block index already in y.CompareKeys order (table.go:267)?
//                           first keys <= 8 B make Go's sort panic (y.go:85)
//   order   (lane = block)  identity for sorted tables; else the rank of each first key
//                           (ties in SST order: Go's sort.Sort is unstable)
//   ends    (lane = table)  status by priority, smallest (forward Rewind: first entry of the
//                           first sorted block) and biggest (reversed Rewind: SeekToLast of the
//                           last sorted block = forward walk, then Prev() through the last
//                           decoded header's prev; iterator.go:86-91,112-155,201-235)
// Block slices in Go are windows of the mmap'd file, so headers/keys past a block but inside
// the file are legal reads; only reads past the file panic.  The oracle restatement is
// sstref_open_table (oracle/sstref.c).
#include <rocprim/device/device_scan.hpp>

#include "codec_common.hpp"
#include "kernels.hpp"

namespace lsmgpu {

namespace {

constexpr uint32_t F_BAD_TAIL = 1, F_FIRST_PLEN = 2, F_READ = 4, F_KEY_LEN = 8, F_UNSORTED = 16;

__device__ __forceinline__ uint32_t ld_be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
__device__ __forceinline__ uint32_t ld_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// table of block i: largest t with blk_base[t] <= i
__device__ __forceinline__ uint32_t table_of(const uint32_t* base, uint32_t ntables, uint32_t i) {
  uint32_t lo = 0, hi = ntables - 1;
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (base[mid] <= i) lo = mid; else hi = mid - 1;
  }
  return lo;
}

}  // namespace

__global__ void open_tail_kernel(OpenParams p) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= p.ntables) return;
  const uint64_t base = p.sst_off[t], len = p.sst_len[t];
  uint32_t nr = 0, bo = 0, bl = 0, rp = 0, fl = 0;
  if (base + len > p.data_len || len > 0xffffffffull || len < 8) {
    fl = F_BAD_TAIL;
  } else {
    const uint8_t* d = p.data + base;
    uint64_t pos = len - 4;
    bl = ld_be32(d + pos);                                  // table.go:181-183
    if (bl > pos || pos - bl < 4) {
      fl = F_BAD_TAIL;
    } else {
      pos -= bl;
      bo = (uint32_t)pos;
      pos -= 4;                                             // table.go:188-190
      nr = ld_be32(d + pos);
      if ((uint64_t)nr * 4 > pos) {
        fl = F_BAD_TAIL;
        nr = 0;
      } else {
        rp = (uint32_t)(pos - 4ull * nr);                   // table.go:192-199
      }
    }
  }
  if (fl) nr = 0;
  p.out.nblk[t] = nr;
  p.out.bloom_off[t] = bo;
  p.out.bloom_len[t] = bl;
  p.rpos[t] = rp;
  p.flags[t] = fl;
}

__global__ void open_blocks_kernel(OpenParams p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.out.blk_cap || i >= p.out.blk_base[p.ntables]) return;
  const uint32_t t = table_of(p.out.blk_base, p.ntables, i);
  const uint32_t j = i - p.out.blk_base[t];
  const uint64_t len = p.sst_len[t];
  const uint8_t* d = p.data + p.sst_off[t];
  const uint32_t rp = p.rpos[t];
  const uint32_t o = ld_be32(d + rp + 4ull * j);
  const uint32_t prev = j ? ld_be32(d + rp + 4ull * (j - 1)) : 0u;
  uint32_t fl = 0;
  if (o < prev || o > rp) fl |= F_BAD_TAIL;                 // lsmgpu_parse_index's checks
  p.out.blk_off[i] = prev;
  p.out.blk_len[i] = o - prev;
  uint32_t ko = 0, kl = 0;
  if ((uint64_t)prev + 10 > len) {
    fl |= F_READ;                                           // "While reading first header"
  } else {
    const uint32_t plen = ld_be16(d + prev), klen = ld_be16(d + prev + 2);
    if (plen != 0) {
      fl |= F_FIRST_PLEN;                                   // table.go:239
    } else if ((uint64_t)prev + 10 + klen > len) {
      fl |= F_READ;                                         // "While reading first key"
    } else {
      ko = prev + 10;
      kl = klen;
    }
  }
  p.out.key_off[i] = ko;
  p.out.key_len[i] = kl;
  if (fl) atomicOr(p.flags + t, fl);
}

__global__ void open_sorted_kernel(OpenParams p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.out.blk_cap || i >= p.out.blk_base[p.ntables]) return;
  const uint32_t t = table_of(p.out.blk_base, p.ntables, i);
  const uint32_t j = i - p.out.blk_base[t];
  if (p.out.nblk[t] < 2) return;                            // sort.Sort compares nothing
  const uint8_t* d = p.data + p.sst_off[t];
  const uint32_t kl = p.out.key_len[i];
  uint32_t fl = 0;
  if (kl <= 8) {
    fl = F_KEY_LEN;                                         // y.go:85 AssertTrue(len > 8)
  } else if (j > 0) {
    const uint32_t pl = p.out.key_len[i - 1];
    if (pl > 8 && compare_keys(d + p.out.key_off[i - 1], pl, d + p.out.key_off[i], kl) > 0)
      fl = F_UNSORTED;
  }
  if (fl) atomicOr(p.flags + t, fl);
}

__global__ void open_order_kernel(OpenParams p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.out.blk_cap || i >= p.out.blk_base[p.ntables]) return;
  const uint32_t t = table_of(p.out.blk_base, p.ntables, i);
  const uint32_t b0 = p.out.blk_base[t], j = i - b0;
  const uint32_t fl = p.flags[t];
  if (!(fl & F_UNSORTED) || (fl & (F_BAD_TAIL | F_FIRST_PLEN | F_READ | F_KEY_LEN)) ||
      (uint64_t)b0 + p.out.nblk[t] > p.out.blk_cap) {
    p.out.order[i] = j;
    return;
  }
  // rank of key j among the table's first keys (ties: SST order)
  const uint8_t* d = p.data + p.sst_off[t];
  const uint32_t n = p.out.nblk[t];
  const uint8_t* kj = d + p.out.key_off[i];
  const uint32_t lj = p.out.key_len[i];
  uint32_t rank = 0;
  for (uint32_t k = 0; k < n; k++) {
    if (k == j) continue;
    const int c = compare_keys(d + p.out.key_off[b0 + k], p.out.key_len[b0 + k], kj, lj);
    rank += (c < 0 || (c == 0 && k < j)) ? 1u : 0u;
  }
  p.out.order[b0 + rank] = j;
}

__global__ void open_ends_kernel(OpenParams p) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= p.ntables) return;
  const uint32_t fl = p.flags[t];
  const uint32_t b0 = p.out.blk_base[t], n = p.out.nblk[t];
  uint32_t sm[3] = {0, 0, 0}, bg[5] = {0, 0, 0, 0, 0};
  int32_t st = LSMGPU_TBL_OK;
  if (fl & F_BAD_TAIL) st = LSMGPU_TBL_BAD_TAIL;
  else if ((uint64_t)b0 + n > p.out.blk_cap) st = LSMGPU_TBL_CAPACITY;
  else if (fl & F_FIRST_PLEN) st = LSMGPU_TBL_FIRST_PLEN;
  else if (fl & F_READ) st = LSMGPU_TBL_READ;
  else if (fl & F_KEY_LEN) st = LSMGPU_TBL_KEY_LEN;
  if (st == LSMGPU_TBL_OK && n > 0) {
    const uint64_t len = p.sst_len[t];
    const uint8_t* d = p.data + p.sst_off[t];
    {  // smallest: block order[0], SeekToFirst -> Init -> Next (iterator.go:81-84,112-135)
      const uint32_t b = b0 + p.out.order[b0];
      const uint32_t off = p.out.blk_off[b], bl = p.out.blk_len[b];
      if (bl >= 10) {
        const uint32_t plen = ld_be16(d + off), klen = ld_be16(d + off + 2),
                       vlen = ld_be16(d + off + 4);
        if (!(klen == 0 && plen == 0) && 10u + klen + vlen <= bl) {
          sm[0] = 1;
          sm[1] = off + 10;
          sm[2] = klen;
        }
      }
    }
    {  // biggest: block order[n-1], SeekToLast: Next until invalid, then Prev()
      const uint32_t b = b0 + p.out.order[b0 + n - 1];
      const uint32_t off = p.out.blk_off[b], bl = p.out.blk_len[b];
      uint32_t pos = 0, last_prev = 0;  // itr.last starts as the zero header
      bool have_base = false, bad = false;
      for (;;) {
        if (pos >= bl) break;                                           // io.EOF
        if ((uint64_t)off + pos + 10 > len) { bad = true; break; }      // Decode past the file
        const uint32_t plen = ld_be16(d + off + pos), klen = ld_be16(d + off + pos + 2),
                       vlen = ld_be16(d + off + pos + 4);
        last_prev = ld_be32(d + off + pos + 6);
        pos += 10;
        if (klen == 0 && plen == 0) break;                              // io.EOF
        if (!have_base) {
          if (plen != 0) { bad = true; break; }                         // AssertTrue panic
          if ((uint64_t)off + pos + klen > len) { bad = true; break; }
          have_base = true;
        }
        if ((uint64_t)off + 10 + plen > len || (uint64_t)off + pos + klen > len) {
          bad = true;
          break;
        }
        pos += klen;
        if (pos + vlen > bl) break;                                     // "Value exceeded"
        pos += vlen;
      }
      if (!bad && last_prev != 0xffffffffu) {                           // Prev()
        const uint32_t q = last_prev;
        if (q >= bl || (uint64_t)off + q + 10 > len) {
          bad = true;
        } else {
          const uint32_t plen = ld_be16(d + off + q), klen = ld_be16(d + off + q + 2),
                         vlen = ld_be16(d + off + q + 4);
          const uint64_t base_cap = have_base ? len - (off + 10) : 0;   // cap(baseKey)
          if (plen > base_cap || (uint64_t)off + q + 10 + klen > len) {
            bad = true;
          } else if ((uint64_t)q + 10 + klen + vlen <= bl) {
            bg[0] = 1;
            bg[1] = off + 10;
            bg[2] = plen;
            bg[3] = off + q + 10;
            bg[4] = klen;
          }
        }
      }
      if (bad) st = LSMGPU_TBL_BIGGEST;
    }
  }
  p.out.status[t] = st;
  for (int k = 0; k < 3; k++) p.out.smallest[3 * t + k] = sm[k];
  for (int k = 0; k < 5; k++) p.out.biggest[5 * t + k] = bg[k];
  if (st != LSMGPU_TBL_OK) atomicAdd(reinterpret_cast<unsigned long long*>(p.result + 1), 1ull);
  if (t == 0) p.result[0] = p.out.blk_base[p.ntables];
}

size_t open_scan_bytes(uint32_t ntables) {
  size_t bytes = 0;
  (void)rocprim::inclusive_scan(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                (size_t)ntables, rocprim::plus<uint32_t>());
  return bytes;
}

hipError_t launch_open_tables(const OpenParams& p, void* scan_tmp, size_t scan_bytes,
                              hipStream_t s) {
  const uint32_t nt = p.ntables;
  const dim3 tg((nt + 63) / 64), bg((uint32_t)((p.out.blk_cap + 255) / 256));
  hipError_t e;
  hipLaunchKernelGGL(open_tail_kernel, tg, dim3(64), 0, s, p);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = hipMemsetAsync(p.out.blk_base, 0, 4, s)) != hipSuccess) return e;
  size_t bytes = scan_bytes;
  e = rocprim::inclusive_scan(scan_tmp, bytes, p.out.nblk, p.out.blk_base + 1, (size_t)nt,
                              rocprim::plus<uint32_t>(), s);
  if (e != hipSuccess) return e;
  if (p.out.blk_cap) {
    hipLaunchKernelGGL(open_blocks_kernel, bg, dim3(256), 0, s, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(open_sorted_kernel, bg, dim3(256), 0, s, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(open_order_kernel, bg, dim3(256), 0, s, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  hipLaunchKernelGGL(open_ends_kernel, tg, dim3(64), 0, s, p);
  return hipGetLastError();
}

}  // namespace lsmgpu
