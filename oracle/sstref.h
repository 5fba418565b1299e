/*
 * sstref.h -- CPU ORACLE for the lsmdb SST block codec.  TEST INFRASTRUCTURE ONLY.
 *
 * This is a plain-C restatement of the reference Go path (impact-eintr/lsmdb @ v0):
 *   table/builder.go   (header codec, Builder.Add/addHelper/finishBlock/blockIndex/Finish)
 *   table/iterator.go  (blockIterator.Next/parseKV -- the decode semantics)
 *   table/table.go     (readIndex tail parse, block boundaries)
 *   y/iterator.go      (ValueStruct EncodedSize/Encode/Decode, uvarint)
 *   y/y.go             (KeyWithTs, ParseKey, CompareKeys)
 * Each function cites the file:line it follows.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / CPU baseline -- never as the product path.
 *
 * Parity pinning: the Go toolchain is absent (no go, no module cache), so the reference
 * cannot be executed here or on the GPU box.  The oracle is pinned by (1) the reference's
 * own known answers in table/table_test.go (counts, value order, Meta, seek tables) and
 * (2) byte-level KATs hand-derived from table/builder.go (tests/golden/kat.json).  The
 * bloom tail (third-party bbloom, not vendored) is restated in bbloom.c: its SipHash core is
 * pinned by the published test vector, the rest is "parity unpinned" (see bbloom.c).
 */
#ifndef SSTREF_H
#define SSTREF_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Per-block decode status (same numbering as include/lsmgpu.h LSMGPU_BLK_*). */
enum {
  SSTREF_BLK_OK = 0,               /* terminator reached, or pos >= len (iterator.go:115,124) */
  SSTREF_BLK_VALUE_OVERFLOW = 1,   /* iterator.go:103-106 "Value exceeded size of block"     */
  SSTREF_BLK_FIRST_PLEN = 2,       /* iterator.go:131 / table.go:239 AssertTrue(plen==0)     */
  SSTREF_BLK_TRUNC_HEADER = 3,     /* < 10 bytes left for a header (Go reads past the block)  */
  SSTREF_BLK_PREFIX_OOB = 4,       /* baseKey[:plen] reaches past the block end               */
  SSTREF_BLK_RANGE = 5             /* block [off,off+len) outside the data buffer             */
};

/* ---- y/iterator.go ValueStruct ---- */
int      sstref_uvarint_size(uint64_t x);                                 /* y/iterator.go:20-29 */
uint16_t sstref_vs_encoded_size(uint64_t expires_at, size_t value_len);   /* y/iterator.go:31-38 */
size_t   sstref_vs_encode(uint8_t meta, uint8_t user_meta, uint64_t expires_at,
                          const uint8_t* value, size_t value_len, uint8_t* out); /* :48-62 */
/* y/iterator.go:40-46 (binary.Uvarint).  Returns the value offset inside b, or -1. */
int      sstref_vs_decode(const uint8_t* b, size_t len, uint8_t* meta, uint8_t* user_meta,
                          uint64_t* expires_at);

/* ---- table/builder.go Builder ---- */
typedef struct sstref_builder sstref_builder;
/* NewTableBuilder (builder.go:61-67).  entries_per_block = resultInterval (builder.go:14,
 * default 100).  block_bytes > 0 enables the opt-in byte-target cut (not in the reference):
 * a new block is started before an entry when the current block is non-empty and
 * (block bytes + entry bytes + 13) > block_bytes. */
sstref_builder* sstref_builder_new(uint32_t entries_per_block, uint32_t block_bytes);
void     sstref_builder_free(sstref_builder*);
/* Builder.Add (builder.go:125-137) with the full-key rule of keyDiff (builder.go:74-82). */
void     sstref_builder_add(sstref_builder*, const uint8_t* key, size_t klen,
                            const uint8_t* vsenc, size_t vlen_full);
int      sstref_builder_reached_capacity(const sstref_builder*, int64_t cap); /* :140-143 */
int      sstref_builder_empty(const sstref_builder*);                         /* :71 */
/* Finish minus the bloom (builder.go:163-198): final terminator + blockIndex.  Returns a
 * pointer to the internal buffer ([data blocks][restarts BE32 x N][N BE32]) and its length.
 * The caller appends bloom JSON + BE32(len(bloom)). */
const uint8_t* sstref_builder_finish(sstref_builder*, size_t* out_len, size_t* data_len,
                                     const uint32_t** restarts, size_t* nrestarts);

/* Batch build: entries i in [0,n) are keys[key_end[i-1]:key_end[i]], vs[vs_end[i-1]:vs_end[i]].
 * Writes [data][index] into out (cap bytes).  Returns total length or 0 on overflow. */
size_t sstref_build(const uint8_t* keys, const uint32_t* key_end, const uint8_t* vs,
                    const uint32_t* vs_end, size_t n, uint32_t entries_per_block,
                    uint32_t block_bytes, uint8_t* out, size_t cap, size_t* data_len,
                    uint32_t* restarts, size_t restarts_cap, size_t* nrestarts);

/* ---- table/table.go readIndex (table.go:177-215) ---- */
/* Returns 0 OK, -1 malformed tail, -2 cap too small. */
int sstref_parse_index(const uint8_t* sst, size_t len, uint32_t* blk_off, uint32_t* blk_len,
                       size_t cap, size_t* nblk, size_t* bloom_off, size_t* bloom_len);

/* ---- table/iterator.go blockIterator forward decode (iterator.go:93-135) ---- */
typedef struct {
  uint64_t n_entries, key_bytes, val_bytes;
  int64_t  first_bad_block;   /* -1 if none */
  uint64_t n_bad_blocks;
  int      overflow;          /* 1 if an output capacity was too small */
} sstref_totals;

/* Decodes nblk blocks of data (block b = data[blk_off[b] : blk_off[b]+blk_len[b]]) and
 * materialises, in iterator order:
 *   key_data/key_end: decoded keys (baseKey[:plen] ++ diff), key_end[i] = running end offset
 *   val_data/val_end: the raw ValueStruct bytes (what blockIterator.Value() returns)
 *   view[i]         : (u64)(hdr_pos+10) | klen<<32 | vlen<<48   (zero-copy entry index)
 *   blk_first[b]    : index of block b's first entry; blk_first[nblk] = total entries
 *   blk_status[b]   : SSTREF_BLK_*
 * Any output pointer may be NULL (not produced).  Returns 0, or 1 on capacity overflow. */
int sstref_decode_blocks(const uint8_t* data, size_t data_len, const uint32_t* blk_off,
                         const uint32_t* blk_len, size_t nblk,
                         uint8_t* key_data, size_t key_cap, uint32_t* key_end,
                         uint8_t* val_data, size_t val_cap, uint32_t* val_end,
                         uint64_t* view, size_t ent_cap,
                         uint32_t* blk_first, int32_t* blk_status, sstref_totals* tot);

/* Multi-threaded CPU baseline: same as above, blocks split in nthreads contiguous ranges,
 * each thread decoding its range into per-thread scratch (outputs discarded except totals).
 * Used only by bench.py's cpu_baseline leg. Returns elapsed seconds for `reps` passes. */
double sstref_decode_bench(const uint8_t* data, size_t data_len, const uint32_t* blk_off,
                           const uint32_t* blk_len, size_t nblk, int nthreads, int reps,
                           uint64_t* checksum);

/* ---- table/table.go OpenTable index work (table.go:88-144 OpenTable, 177-269 readIndex) ----
 * Per-table status; a Go panic / error becomes a code (priority: the first listed wins). */
enum {
  SSTREF_TBL_OK = 0,
  SSTREF_TBL_BAD_TAIL = 1,    /* malformed tail (sstref_parse_index -1)                        */
  SSTREF_TBL_FIRST_PLEN = 2,  /* table.go:239 AssertTruef(h.plen == 0): a panic                */
  SSTREF_TBL_READ = 3,        /* table.go:226-237 t.read past the file: readIndex returns err  */
  SSTREF_TBL_KEY_LEN = 4,     /* sort.Sort -> y.CompareKeys AssertTrue(len > 8): a panic       */
  SSTREF_TBL_CAPACITY = 5,    /* more blocks than the caller's capacity                        */
  SSTREF_TBL_BIGGEST = 6      /* SeekToLast/Prev would panic or read past the block; biggest nil */
};
typedef struct {
  uint32_t nblk;
  uint32_t bloom_off, bloom_len;
  int32_t  status;
  /* smallest = Rewind() of a forward iterator: first entry of block order[0] (iterator.go:201-217) */
  int32_t  has_smallest;
  uint32_t smallest_off, smallest_len;             /* table-relative key span (plen == 0)    */
  /* biggest = Rewind() of a reversed iterator: block order[nblk-1].SeekToLast() ->
   * walk forward until invalid, then Prev() to the last decoded header's `prev`
   * (iterator.go:86-91,137-155); key = baseKey[:plen] ++ diff */
  int32_t  has_biggest;
  uint32_t big_base_off, big_plen, big_diff_off, big_klen;  /* table-relative */
} sstref_table_info;
/* blk_off/blk_len (table-relative, SST order), key_off/key_len (each block's first key, the
 * blockIndex keys), order[i] = SST index of the i-th block of the sorted blockIndex
 * (sort.Sort(byKey), table.go:267; equal keys keep SST order -- Go's sort is unstable).
 * Returns info->status. */
int sstref_open_table(const uint8_t* sst, size_t len, uint32_t* blk_off, uint32_t* blk_len,
                      uint32_t* key_off, uint32_t* key_len, uint32_t* order, size_t cap,
                      sstref_table_info* info);

/* ---- y/iterator.go MergeIterator (y/iterator.go:74-202) ----
 * nruns iterators over entries [run_first[r], run_first[r+1]) of one key stream (key i =
 * kd[ke[i-1]:ke[i]]).  The heap's top is always the least head under elemHeap.Less (CompareKeys,
 * then lower nice = run index); Next() drops every head equal to the last emitted key
 * (storeKey/curKey).  out_src[i] = entry index of the i-th output.  Returns the output count
 * (or (size_t)-1 if cap is too small). */
size_t sstref_merge(const uint8_t* kd, const uint32_t* ke, const uint32_t* run_first,
                    size_t nruns, uint32_t* out_src, size_t cap);

/* ---- bloom tail (bbloom.c: AndreasBriese/bbloom v0.0.0-20190825152654-46b345b51c96 restated;
 *      table/builder.go:164-195, table/table.go:180-186,301) ---- */
uint64_t sstref_siphash24(uint64_t k0, uint64_t k1, const uint8_t* p, size_t n);
void   sstref_bloom_params(double num_entries, double wrongs, uint64_t* size_bits,
                           uint64_t* set_locs, uint32_t* exponent);
void   sstref_bloom_add(uint64_t* bitset, uint64_t size_bits, uint32_t exponent,
                        uint64_t set_locs, const uint8_t* key, size_t n);
int    sstref_bloom_has(const uint64_t* bitset, uint64_t size_bits, uint32_t exponent,
                        uint64_t set_locs, const uint8_t* key, size_t n);
size_t sstref_bloom_json(const uint64_t* bitset, uint64_t size_bits, uint64_t set_locs,
                         uint8_t* out, size_t cap);
int    sstref_bloom_build(const uint8_t* keys, const uint32_t* key_end, size_t n,
                          uint64_t* bitset, uint64_t size_bits, uint32_t exponent,
                          uint64_t set_locs);

/* ---- y/y.go key helpers ---- */
int sstref_compare_keys(const uint8_t* k1, size_t l1, const uint8_t* k2, size_t l2); /* y.go:84-90 */

#ifdef __cplusplus
}
#endif
#endif
