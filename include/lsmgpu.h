/*
 * lsmgpu.h -- C ABI of the MI355X-native (gfx950 / CDNA4) SST block codec for lsmdb.
 *
 * This is the drop-in boundary.  The reference (impact-eintr/lsmdb @ v0, pure Go) has no FFI
 * layer: the path sits behind the Go `table` package.  Each entry point below names the
 * reference interface it replaces (file:line); INTEGRATION.md shows the cgo shim that binds
 * them so table.Builder / table.Table keep their Go API and the on-disk .sst layout.
 *
 * Conventions
 *  - Plain pointers and sizes only; the caller owns every buffer; nothing is retained past
 *    return (cgo pointer rules).  `*_on_device` flags say whether pointers are HIP device
 *    pointers (device-resident path) or host pointers (the library stages through HBM).
 *  - Offsets inside one call are u32, as in the SST format itself (builder.go:53,146-160);
 *    one call handles at most 4 GiB - 1 of block bytes.
 *  - Functions return LSMGPU_OK (0) or a positive LSMGPU_ERR_* code; they never abort.
 *  - One lsmgpu_ctx per OS thread (like a Go Builder/Iterator: single-goroutine objects).
 */
#ifndef LSMGPU_H
#define LSMGPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2 (round 4): size queries (decode with every output pointer NULL, encode with out == NULL),
 * LSMGPU_ERR_CORRUPT, stream probe kinds 4-7 and its argument checks.
 * 3 (round 5): lsmgpu_host_register is refcounted per page segment (overlapping and re-used
 * ranges), LSMGPU_ERR_HOST_PINNED, unregister of an unknown pointer is LSMGPU_ERR_ARG.
 * 4 (round 6): the library never page-locks caller memory: pageable host buffers are staged
 * through page-locked buffers it owns (hipHostMalloc, per ctx), runtime-pinned ones are DMA'd
 * directly; lsmgpu_host_alloc / lsmgpu_host_free hand out such memory; lsmgpu_host_register /
 * unregister keep their argument and error rules but pin nothing. */
#define LSMGPU_ABI_VERSION 4

/* ---- call status ---- */
#define LSMGPU_OK 0
#define LSMGPU_ERR_ARG 1        /* NULL / inconsistent argument                               */
#define LSMGPU_ERR_BAD_TAIL 2   /* malformed SST tail: table.go:177-215 would panic or ErrEOF  */
#define LSMGPU_ERR_CAPACITY 3   /* an output buffer is too small; lsmgpu_decoded.* has the need */
#define LSMGPU_ERR_HIP 4        /* HIP runtime error                                          */
#define LSMGPU_ERR_KEY_LEN 5    /* encode: key length <= 8 (y.go:98 AssertTruef) or > 65535    */
#define LSMGPU_ERR_VALUE_LEN 6  /* encode: vs-enc > 65535 (y/iterator.go:31-38 uint16 trunc.) */
#define LSMGPU_ERR_TOO_LARGE 7  /* more than 4 GiB - 1 bytes in one call                        */
#define LSMGPU_ERR_INTERNAL 8   /* device look-back did not converge (never expected)          */
#define LSMGPU_ERR_NO_DEVICE 9  /* no HIP device / bad device index                            */
#define LSMGPU_ERR_CORRUPT 10   /* compaction input: a block with a non-OK LSMGPU_BLK_* status, or
                                   a table whose keys are not in CompareKeys order              */
#define LSMGPU_ERR_HOST_PINNED 11 /* host_register: the range overlaps memory page-locked outside
                                   this library (hipHostMalloc, the caller's hipHostRegister);
                                   nothing was registered -- such memory needs no registration */

/* ---- per-block decode status (lsmgpu_decoded.blk_status) ---- */
#define LSMGPU_BLK_OK 0             /* terminator, or pos >= len (iterator.go:115-118,124-127) */
#define LSMGPU_BLK_VALUE_OVERFLOW 1 /* "Value exceeded size of block" (iterator.go:103-106)     */
#define LSMGPU_BLK_FIRST_PLEN 2     /* AssertTrue(h.plen == 0) (iterator.go:131, table.go:239)  */
#define LSMGPU_BLK_TRUNC_HEADER 3   /* < 10 B left for a header (Go reads past the block slice)  */
#define LSMGPU_BLK_PREFIX_OOB 4     /* baseKey[:plen] would read past the block                 */
#define LSMGPU_BLK_RANGE 5          /* block [off, off+len) is outside the data buffer          */

/* ---- decode modes (bit mask) ---- */
#define LSMGPU_MODE_MATERIALIZE 1 /* key_data/key_end + val_data/val_end                       */
#define LSMGPU_MODE_VIEW 2        /* view[] zero-copy entry index                              */

typedef struct lsmgpu_ctx lsmgpu_ctx;

/* Context: owns a HIP stream (or borrows one), look-back scratch and staging buffers. */
int lsmgpu_open(int device, lsmgpu_ctx** out);
void lsmgpu_close(lsmgpu_ctx* ctx);
/* Use an external hipStream_t (e.g. the caller's current stream); NULL restores the ctx's own. */
int lsmgpu_set_stream(lsmgpu_ctx* ctx, void* hip_stream);
void* lsmgpu_get_stream(lsmgpu_ctx* ctx);
int lsmgpu_synchronize(lsmgpu_ctx* ctx);
/* Diagnostics (no reference counterpart): with timing on, walk-scan-copy decodes record HIP
 * events on the ctx's stream before the walk, between the walk and the copy, and after the
 * copy; lsmgpu_kernel_times waits for the last decode's events and returns the walk and copy
 * durations (copy 0 for view-only decodes that finish in the walk), or LSMGPU_ERR_ARG when the
 * last decode was not timed or took another decode path. */
int lsmgpu_set_kernel_timing(lsmgpu_ctx* ctx, int on);
int lsmgpu_kernel_times(lsmgpu_ctx* ctx, float* walk_ms, float* copy_ms);
/* Diagnostics (no reference counterpart): the practical HBM ceilings bench.py prices the decode
 * against -- a grid-stride 16-B-per-lane streaming copy or read of `bytes` from d_src (to d_dst;
 * for a read, d_dst is a 4-B sink), wg_per_cu 256-thread workgroups per CU.  kind bit 0: read
 * (else copy); bit 1: non-temporal loads and stores; bit 2: 16 loads in flight per lane (else 4).
 * `bytes` must be a multiple of 16 and both pointers 16-B aligned (else LSMGPU_ERR_ARG).
 * Asynchronous on the ctx stream. */
int lsmgpu_stream_probe_async(lsmgpu_ctx* ctx, int kind, const void* d_src, void* d_dst,
                              uint64_t bytes, uint32_t wg_per_cu);
const char* lsmgpu_strerror(int code);
/* The HIP call behind this thread's last LSMGPU_ERR_HIP ("call -> HIP error string (where)"),
 * "" if none yet.  Valid until this thread's next failing call. */
const char* lsmgpu_last_error(void);
int lsmgpu_abi_version(void);

/* Replaces Table.readIndex's tail parse (table/table.go:177-215): bloom length + bloom span,
 * restart count, restart offsets -> block b = [blk_off[b], blk_off[b]+blk_len[b]).  Host only.
 * *nblk is set even when cap is too small (then LSMGPU_ERR_CAPACITY). */
int lsmgpu_parse_index(const uint8_t* sst, uint64_t len, uint32_t* blk_off, uint32_t* blk_len,
                       uint64_t cap, uint64_t* nblk, uint64_t* bloom_off, uint64_t* bloom_len);

/* Decoded output.  In materialize mode, entry i (in Table.Iterator order) has
 *   key   = key_data[key_end[i-1] : key_end[i]]   (blockIterator.Key(): baseKey[:plen] ++ diff)
 *   value = val_data[val_end[i-1] : val_end[i]]   (blockIterator.Value(): raw ValueStruct bytes)
 * (key_end[-1] = val_end[-1] = 0).  In view mode view[i] = key_pos | klen << 32 | vlen << 48
 * where key_pos is the absolute offset of the entry's stored key bytes in `data` (header at
 * key_pos-10, value at key_pos+klen).  blk_first[b] = first entry of block b (nblk+1 words),
 * blk_status[b] = LSMGPU_BLK_*.  Entries of a block with an error status are the ones the Go
 * blockIterator yields before it turns invalid. */
typedef struct {
  uint8_t* key_data;  uint64_t key_cap;
  uint32_t* key_end;
  uint8_t* val_data;  uint64_t val_cap;
  uint32_t* val_end;
  uint64_t* view;
  uint64_t ent_cap;          /* capacity (entries) of key_end / val_end / view */
  uint32_t* blk_first;       /* nblk + 1 */
  int32_t* blk_status;       /* nblk */
  /* results, written by the synchronous call */
  uint64_t n_entries, key_bytes, val_bytes;
  int64_t first_bad_block;   /* -1 if every block decoded cleanly */
  uint64_t n_bad_blocks;
} lsmgpu_decoded;

/* Replaces the per-entry blockIterator.Next/parseKV loop (table/iterator.go:93-135) driven by
 * Iterator.seekToFirst/next (iterator.go:201-217,301-326) over a batch of blocks, e.g. every
 * block of the tables compactBuildTables (levels.go:239-338) merges.  blk_off/blk_len are host
 * arrays (from lsmgpu_parse_index, offsets relative to `data`).  If data_on_device is 0, `data`
 * and every output pointer are host memory and the library stages through HBM.
 * Size query: with every output pointer of `out` NULL the blocks are walked and n_entries,
 * key_bytes, val_bytes, first_bad_block and n_bad_blocks report exactly what the real call
 * needs (ent_cap >= n_entries, key_cap >= key_bytes, val_cap >= val_bytes); returns LSMGPU_OK.
 * A real call whose buffers are too small returns LSMGPU_ERR_CAPACITY with the same needs. */
int lsmgpu_decode_blocks(lsmgpu_ctx* ctx, const uint8_t* data, uint64_t data_len,
                         int data_on_device, const uint32_t* blk_off, const uint32_t* blk_len,
                         uint64_t nblk, int mode, lsmgpu_decoded* out);

/* Host-memory calls (data_on_device = 0) with blocks sorted by offset are pipelined: chunks of
 * ~32 MiB (LSMGPU_HOST_CHUNK) are copied in, decoded and copied out on three streams at once.
 * Host memory is never page-locked by the library (ABI 4).  Memory the HIP runtime already
 * knows as page-locked -- lsmgpu_host_alloc, hipHostMalloc, torch's pinned allocator -- is DMA'd
 * directly at PCIe rate; any other host memory (a Go heap buffer under LoadToRAM,
 * table.go:117-123,329-338; an mmap'd .sst, y/mmap.go:11-21; pageable output arrays) is staged
 * through page-locked buffers the ctx owns, filled and drained by memcpy on a small per-ctx
 * thread pool (LSMGPU_COPY_THREADS, default half the hardware threads, at most 16).  So a caller that wants
 * one copy of a table end to end reads the file into lsmgpu_host_alloc memory.
 * Every host call has finished all DMA into or out of caller memory when it returns.  A device
 * pointer passed as host `data` (data_on_device = 0) is LSMGPU_ERR_ARG. */
int lsmgpu_host_alloc(lsmgpu_ctx* ctx, uint64_t bytes, void** out);  /* hipHostMalloc, portable */
int lsmgpu_host_free(lsmgpu_ctx* ctx, void* p);  /* p NULL: no-op; ctx may be NULL (any device) */

/* ABI 3 compatibility: records a range the caller will pass (nothing is page-locked).  Returns
 * LSMGPU_ERR_HOST_PINNED (nothing recorded) for memory the runtime already knows as page-locked
 * (it needs no registration); lsmgpu_host_unregister(p) drops the latest record at p and returns
 * LSMGPU_ERR_ARG if there is none.  Thread-safe. */
int lsmgpu_host_register(lsmgpu_ctx* ctx, void* p, uint64_t bytes);
int lsmgpu_host_unregister(lsmgpu_ctx* ctx, void* p);

/* Device-resident asynchronous form (the benchmarked kernel): all pointers are device
 * pointers, max_blk_len bounds blk_len[] (selects the LDS slot), `d_result` (device, 8 u64)
 * receives {n_entries, key_bytes, val_bytes, first_bad_block+1, n_bad_blocks, flags, 0, 0}
 * with flags bit0 = capacity overflow, bit1 = look-back timeout.  Enqueued on the ctx stream. */
int lsmgpu_decode_blocks_async(lsmgpu_ctx* ctx, const uint8_t* d_data, uint64_t data_len,
                               const uint32_t* d_blk_off, const uint32_t* d_blk_len,
                               uint64_t nblk, uint32_t max_blk_len, int mode,
                               const lsmgpu_decoded* out, uint64_t* d_result);

/* Replaces Builder.Add x n + Builder.Finish minus the bloom (table/builder.go:84-198):
 * entry i = (keys[key_end[i-1]:key_end[i]], vs[vs_end[i-1]:vs_end[i]]) where vs is the
 * encoded ValueStruct (y/iterator.go:48-62), entries sorted by the caller as Add requires.
 * Blocks are cut every entries_per_block entries (resultInterval, builder.go:14,126; 100 is the
 * reference) or, if block_bytes > 0, before an entry that would grow a non-empty block past
 * block_bytes (opt-in knob, not in the reference).  Writes [data blocks][restarts BE32 x N]
 * [N BE32] to out; the caller appends bbloom JSON + BE32(len) exactly as builder.go:190-195.
 * restarts (host, optional) receives the block end offsets.
 * Size query: out == NULL fills *out_len / *data_len / *nrestarts from key_end / vs_end alone
 * (keys and vs may be NULL, and ctx may be NULL for host arrays) and returns LSMGPU_OK, or the
 * KEY_LEN / VALUE_LEN / TOO_LARGE error the real call would return. */
int lsmgpu_encode_blocks(lsmgpu_ctx* ctx, const uint8_t* keys, const uint32_t* key_end,
                         const uint8_t* vs, const uint32_t* vs_end, uint64_t n, int on_device,
                         uint32_t entries_per_block, uint32_t block_bytes, uint8_t* out,
                         uint64_t out_cap, uint64_t* out_len, uint64_t* data_len,
                         uint32_t* restarts, uint64_t restarts_cap, uint64_t* nrestarts);

/* Device-resident asynchronous encode with a precomputed block plan: d_blk_first (device,
 * nblocks+1 entry indices) or NULL with entries_per_block > 0.  key_total/vs_total are
 * key_end[n-1]/vs_end[n-1].  d_flags (device u32) gets bit0 = key length error,
 * bit1 = value length error.  Output length = 10n + key_total + vs_total + 13*nblocks
 * + 4*nblocks + 4. */
int lsmgpu_encode_blocks_async(lsmgpu_ctx* ctx, const uint8_t* d_keys, const uint32_t* d_key_end,
                               const uint8_t* d_vs, const uint32_t* d_vs_end, uint64_t n,
                               uint32_t entries_per_block, const uint32_t* d_blk_first,
                               uint64_t nblocks, uint64_t key_total, uint64_t vs_total,
                               uint8_t* d_out, uint64_t out_cap, uint32_t* d_flags);

/* Host block planner for the byte-target policy (same rule as lsmgpu_encode_blocks).
 * Writes blk_first[0..nblocks] (cap entries) and returns the block count in *nblocks. */
int lsmgpu_plan_blocks(const uint32_t* key_end, const uint32_t* vs_end, uint64_t n,
                       uint32_t entries_per_block, uint32_t block_bytes, uint32_t* blk_first,
                       uint64_t cap, uint64_t* nblocks);

/* Replaces ValueStruct.EncodeTo (y/iterator.go:55-62) for a batch of values:
 * vs[i] = [meta[i]][user_meta[i]][uvarint expires_at[i]][values[value_end[i-1]:value_end[i]]].
 * vs_end (n words) receives running end offsets.  on_device selects pointer space. */
int lsmgpu_encode_values(lsmgpu_ctx* ctx, const uint8_t* meta, const uint8_t* user_meta,
                         const uint64_t* expires_at, const uint8_t* values,
                         const uint32_t* value_end, uint64_t n, int on_device, uint8_t* vs,
                         uint64_t vs_cap, uint32_t* vs_end, uint64_t* vs_len);

/* ---- Batched OpenTable index work on the device ----------------------
 * Replaces, for ntables SSTs resident in device memory at once, what OpenTable does per table
 * on the host (table/table.go:88-144): readIndex (table.go:177-269: tail parse, every block's
 * first header + first key with the plen == 0 assertion -- the 64-goroutine fan-out -- and
 * sort.Sort(byKey) of the block index by y.CompareKeys), then smallest = a forward iterator's
 * Rewind (first entry of the first sorted block, iterator.go:201-217) and biggest = a reversed
 * iterator's Rewind (SeekToLast of the last sorted block: forward walk, then Prev() through the
 * last decoded header's `prev`, iterator.go:86-91,137-155,219-235).
 * Table t is data[sst_off[t], sst_off[t] + sst_len[t]); every offset below is relative to it.
 * Keys are views: first key i = table[key_off[i], +key_len[i]); smallest = table[off, +len];
 * biggest = table[base_off, +plen] ++ table[diff_off, +klen] (baseKey[:plen] ++ diff -- Go's
 * block slices are windows of the mmap'd file, so these may extend past the block). */
#define LSMGPU_TBL_OK 0
#define LSMGPU_TBL_BAD_TAIL 1    /* malformed tail / restarts (lsmgpu_parse_index's BAD_TAIL)    */
#define LSMGPU_TBL_FIRST_PLEN 2  /* a block's first header has plen != 0 (table.go:239 panic)    */
#define LSMGPU_TBL_READ 3        /* first header/key past the file (table.go:226-237 read error) */
#define LSMGPU_TBL_KEY_LEN 4     /* a first key of <= 8 B compared by the sort (y.go:85 panic)   */
#define LSMGPU_TBL_CAPACITY 5    /* the batch has more blocks than blk_cap                       */
#define LSMGPU_TBL_BIGGEST 6     /* SeekToLast/Prev would panic (read past the file); no biggest */
typedef struct {
  /* per table [ntables] */
  uint32_t* nblk;         /* restart count N (table.go:188-199)                                  */
  uint32_t* blk_base;     /* [ntables + 1]: table t's blocks are entries [blk_base[t], blk_base[t+1]) */
  uint32_t* bloom_off;    /* bloom JSON span (table.go:181-186)                                  */
  uint32_t* bloom_len;
  int32_t* status;        /* LSMGPU_TBL_*; the outputs below are defined when OK or BIGGEST      */
  uint32_t* smallest;     /* 3 per table: {has, off, len}                                        */
  uint32_t* biggest;      /* 5 per table: {has, base_off, plen, diff_off, klen}                  */
  /* per block [blk_cap], SST order within each table */
  uint32_t* blk_off;      /* Table.blockIndex offsets / lengths (table.go:202-215)               */
  uint32_t* blk_len;
  uint32_t* key_off;      /* the block's first key (blockIndex key, table.go:236-246)            */
  uint32_t* key_len;
  uint32_t* order;        /* sorted blockIndex: order[blk_base[t] + i] = SST index of block i    */
  uint64_t blk_cap;
} lsmgpu_tables;
/* Device pointers only; asynchronous on the context's stream.  d_result (device, 8 u64):
 * [0] total blocks, [1] tables whose status is not LSMGPU_TBL_OK. */
int lsmgpu_open_tables_async(lsmgpu_ctx* ctx, const uint8_t* d_data, uint64_t data_len,
                             const uint64_t* d_sst_off, const uint64_t* d_sst_len,
                             uint32_t ntables, const lsmgpu_tables* out, uint64_t* d_result);

/* ---- K-way merge of sorted runs --------------------------------------
 * y.MergeIterator (y/iterator.go:74-202) as used by compactBuildTables (levels.go:239-258):
 * run r = entries [run_first[r], run_first[r+1]) of one key / value stream in the layout
 * lsmgpu_decode_blocks produces (a decode of all input tables in one batch: run_first =
 * blk_first of each table's first block).  Output = the iterator's sequence: CompareKeys order,
 * equal keys resolved to the lowest run index (`nice`), every later entry equal to the last
 * emitted key dropped (y/iterator.go:159-184).  Values are the raw ValueStruct bytes
 * (Value() + Builder.Add re-encode them identically when the uvarint is canonical).
 * Runs must be in CompareKeys order (SSTs are) and keys longer than 8 B (CompareKeys asserts
 * it): otherwise result[3] has LSMGPU_MERGE_UNSORTED / LSMGPU_MERGE_KEY_LEN and nothing is
 * written.  All pointers are device pointers; asynchronous on the context's stream.
 * d_result (8 u64): [0] entries out, [1] key bytes, [2] value bytes, [3] flags. */
#define LSMGPU_MERGE_UNSORTED 1
#define LSMGPU_MERGE_KEY_LEN 2
#define LSMGPU_MERGE_CAPACITY 4
#define LSMGPU_MERGE_TIMEOUT 8   /* look-back did not converge (never on a healthy device) */
typedef struct {
  const uint8_t* key_data;
  const uint32_t* key_end;   /* running end offsets over all runs (key i = [key_end[i-1], key_end[i])) */
  const uint8_t* val_data;
  const uint32_t* val_end;
  const uint32_t* run_first; /* nruns + 1 entries, device */
  uint32_t nruns;
  uint64_t n;                /* run_first[nruns] */
} lsmgpu_runs;
typedef struct {
  uint8_t* key_data;         /* may be NULL (keys not gathered) */
  uint64_t key_cap;
  uint32_t* key_end;
  uint8_t* val_data;         /* may be NULL */
  uint64_t val_cap;
  uint32_t* val_end;
  uint32_t* src;             /* may be NULL: input entry index of each output entry */
  uint64_t ent_cap;
} lsmgpu_merged;
int lsmgpu_merge_runs_async(lsmgpu_ctx* ctx, const lsmgpu_runs* in, const lsmgpu_merged* out,
                            uint64_t* d_result);

/* ---- Compaction output tables (levels.go:259-271 with Builder.ReachedCapacity) ------------
 * Cut a sorted entry stream (e.g. the merge output) into tables exactly where compactBuildTables
 * starts a new Builder: before each Add, ReachedCapacity(cap) = buf.Len() + 8 + 4*len(restarts)
 * + 8 > cap (table/builder.go:140-143) with entries_per_block entries per block (100 =
 * resultInterval).  Outputs (device): tbl_first[t] = first entry of table t, tbl_blk[t] = first
 * block, tbl_out[t] = byte offset of its image; entry [ntables] closes each array.  Images are
 * "Finish minus bloom" ([blocks][restarts BE32 x N][N BE32], like lsmgpu_encode_blocks), back
 * to back.  d_result (8 u64): [0] tables, [1] blocks, [2] image bytes, [3] 1 if tables_cap
 * was too small. */
int lsmgpu_cut_tables_async(lsmgpu_ctx* ctx, const uint32_t* d_key_end, const uint32_t* d_vs_end,
                            uint64_t n, uint32_t entries_per_block, int64_t cap,
                            uint32_t* d_tbl_first, uint32_t* d_tbl_blk, uint64_t* d_tbl_out,
                            uint32_t tables_cap, uint64_t* d_result);
/* The same cut; flags LSMGPU_CUT_BLOOM also reserves each table's bloom tail (Finish's
 * bbloom JSON + BE32 length, table/builder.go:189-195) after its index, so tbl_out / the image
 * bytes describe complete .sst files once lsmgpu_bloom_tables_async has filled the tails. */
#define LSMGPU_CUT_BLOOM 1u
int lsmgpu_cut_tables_ex_async(lsmgpu_ctx* ctx, const uint32_t* d_key_end, const uint32_t* d_vs_end,
                               uint64_t n, uint32_t entries_per_block, int64_t cap, uint32_t flags,
                               uint32_t* d_tbl_first, uint32_t* d_tbl_blk, uint64_t* d_tbl_out,
                               uint32_t tables_cap, uint64_t* d_result);
/* Encodes every table of a cut (one launch over all their blocks) into d_out (sized for the
 * cut's image bytes).  max_blocks bounds the tables' total block count (grid size), e.g.
 * ceil(n / entries_per_block) + tables_cap.  key_total / vs_total (0 if unknown) pick the lanes
 * per entry.  d_flags as lsmgpu_encode_blocks_async. */
int lsmgpu_encode_tables_async(lsmgpu_ctx* ctx, const uint8_t* d_keys, const uint32_t* d_key_end,
                               const uint8_t* d_vs, const uint32_t* d_vs_end, uint64_t n,
                               uint64_t key_total, uint64_t vs_total,
                               uint32_t entries_per_block, const uint32_t* d_tbl_first,
                               const uint32_t* d_tbl_blk, const uint64_t* d_tbl_out,
                               uint32_t tables_cap, uint64_t max_blocks, uint8_t* d_out,
                               uint32_t* d_flags);
/* Gather form for a merge output without its bytes (lsmgpu_merge_runs_async with key_data =
 * val_data = NULL, src set): entry i of the tables is source entry d_src[i] of the merge's INPUT
 * streams (d_keys / d_key_end, d_vs / d_vs_end), placed by the merged end offsets d_out_key_end /
 * d_out_vs_end (the merge's key_end / val_end, which the cut also read).  The bytes move once,
 * decoded tables -> output images, as compactBuildTables' builder.Add(it.Key(), it.Value())
 * copies them once (levels.go:273).  Images are byte-identical to lsmgpu_encode_tables_async
 * over the gathered streams. */
int lsmgpu_encode_tables_gather_async(lsmgpu_ctx* ctx, const uint8_t* d_keys,
                                      const uint32_t* d_key_end, const uint8_t* d_vs,
                                      const uint32_t* d_vs_end, const uint32_t* d_src,
                                      const uint32_t* d_out_key_end, const uint32_t* d_out_vs_end,
                                      uint64_t n, uint64_t key_total, uint64_t vs_total,
                                      uint32_t entries_per_block, const uint32_t* d_tbl_first,
                                      const uint32_t* d_tbl_blk, const uint64_t* d_tbl_out,
                                      uint32_t tables_cap, uint64_t max_blocks, uint8_t* d_out,
                                      uint32_t* d_flags);

/* ---- Bloom tail (table/builder.go:164-195 Finish, table/table.go:180-186 readIndex, :301
 * DoesNotHave) -------------------------------------------------------------------------------
 * The reference's third-party github.com/AndreasBriese/bbloom v0.0.0-20190825152654-46b345b51c96
 * restated (DESIGN.md "Bloom tail"; parity of the bbloom-specific bytes unpinned).
 * lsmgpu_bloom_params: bbloom.New(float64(key_count), 0.01) -> filter bits (a power of two
 * >= 512), setLocs, and the byte length of its JSONMarshal output (key_count 0: setLocs =
 * 1 << 63, Go's uint64(NaN) on amd64). */
int lsmgpu_bloom_params(uint64_t key_count, uint64_t* bits, uint64_t* set_locs, uint64_t* json_len);
/* Finish's filter: bf.Add(ParseKey(key)) for every key of the batch -- keys WITH their 8-B ts
 * (what Builder.Add takes), key i = d_keys[d_key_end[i-1], d_key_end[i]).  d_bitset: bits / 64
 * u64 words, cleared here.  *d_flags |= 1 if a key is <= 8 B (y.go:98 AssertTruef panic; that
 * key is skipped).  Device pointers, asynchronous on the context's stream. */
int lsmgpu_bloom_build_async(lsmgpu_ctx* ctx, const uint8_t* d_keys, const uint32_t* d_key_end,
                             uint64_t n, uint64_t* d_bitset, uint64_t bits, uint64_t set_locs,
                             uint32_t* d_flags);
/* bf.JSONMarshal(): {"FilterSet":"<base64 std of the filter bytes>","SetLocs":N}, json_len bytes
 * (lsmgpu_bloom_params) into d_out (out_cap >= json_len). */
int lsmgpu_bloom_json_async(lsmgpu_ctx* ctx, const uint64_t* d_bitset, uint64_t bits,
                            uint64_t set_locs, uint8_t* d_out, uint64_t out_cap);
/* Table.DoesNotHave for a batch: d_has[i] = bf.Has(key i) (0 = DoesNotHave); keys as the
 * caller passes them (level_handler.go:221-224 passes ParseKey(key), no ts). */
int lsmgpu_bloom_has_async(lsmgpu_ctx* ctx, const uint64_t* d_bitset, uint64_t bits,
                           uint64_t set_locs, const uint8_t* d_keys, const uint32_t* d_key_end,
                           uint64_t n, uint8_t* d_has);

/* Finish's bloom tail for every table of a LSMGPU_CUT_BLOOM cut (after
 * lsmgpu_encode_tables_async): table t's filter over ParseKey of its keys (entries
 * [tbl_first[t], tbl_first[t+1]) of the stream) and JSON ++ BE32(len) into the last bytes of
 * [tbl_out[t], tbl_out[t+1]) of d_out.  tbl_first / tbl_out are HOST copies of the cut's
 * arrays (ntables + 1 each); d_scratch holds the filters of 32 tables side by side (the sum
 * of bits / 64 words over each group of 32 consecutive tables, lsmgpu_bloom_params).
 * *d_flags |= 1 for a key of <= 8 B.  Asynchronous: one memset + 2 launches per 32 tables. */
int lsmgpu_bloom_tables_async(lsmgpu_ctx* ctx, const uint8_t* d_keys, const uint32_t* d_key_end,
                              const uint32_t* tbl_first, const uint64_t* tbl_out, uint32_t ntables,
                              uint8_t* d_out, uint64_t* d_scratch, uint64_t scratch_words,
                              uint32_t* d_flags);
/* Gather form (see lsmgpu_encode_tables_gather_async): key i of the tables is key d_src[i] of
 * d_keys / d_key_end. */
int lsmgpu_bloom_tables_gather_async(lsmgpu_ctx* ctx, const uint8_t* d_keys,
                                     const uint32_t* d_key_end, const uint32_t* d_src,
                                     const uint32_t* tbl_first, const uint64_t* tbl_out,
                                     uint32_t ntables, uint8_t* d_out, uint64_t* d_scratch,
                                     uint64_t scratch_words, uint32_t* d_flags);

/* ---- Whole compaction data path for tables in host memory -------------
 * Replaces the data path of levelsController.compactBuildTables (levels.go:239-298) in one call:
 * the input .sst images (host memory, e.g. the mmap'd files of cd.top and cd.bot) are decoded
 * in one device batch, merged as y.NewMergeIterator(iters) (y/iterator.go:74-202) where iterator
 * r = tables [run_first[r], run_first[r+1]) chained in order (one table per L0 top iterator,
 * appendIteratorsReversed order; the bottom level's tables as the last run, the
 * ConcatIterator of levels.go:252), cut where `builder.ReachedCapacity(max_table_size)` starts a
 * new Builder (levels.go:265-271, 100 entries per block) and encoded as Finish() would
 * (table/builder.go:163-198).  flags LSMGPU_COMPACT_BLOOM appends the restated bbloom tail to
 * every table (complete .sst files); without it each image is Finish minus the bloom (the caller
 * appends Go bbloom's JSONMarshal + BE32 length, byte-identical to the reference).
 * A block with a value overflow contributes the entries before it, as Go's iterator skips the
 * rest of that block (iterator.go:103-106,318-323); any other bad block (a Go panic) returns
 * LSMGPU_ERR_CORRUPT.  The result stays in the ctx: *out_len bytes of images back to back and
 * *out_tables tables; lsmgpu_compact_result copies them out.  Synchronous. */
#define LSMGPU_COMPACT_BLOOM 1u
int lsmgpu_compact_tables(lsmgpu_ctx* ctx, const uint8_t* const* ssts, const uint64_t* sst_len,
                          uint32_t ntables, const uint32_t* run_first, uint32_t nruns,
                          int64_t max_table_size, uint32_t flags, uint64_t* out_len,
                          uint32_t* out_tables);
/* Copies the last lsmgpu_compact_tables result: out (out_cap >= *out_len) receives the images,
 * tbl_off (tbl_cap >= tables + 1) the offset of each table's image in out plus the end. */
int lsmgpu_compact_result(lsmgpu_ctx* ctx, uint8_t* out, uint64_t out_cap, uint64_t* tbl_off,
                          uint64_t tbl_cap);

#ifdef __cplusplus
}
#endif
#endif /* LSMGPU_H */
