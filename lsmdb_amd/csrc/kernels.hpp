// kernels.hpp -- launch interface between the C ABI (api.hip) and the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lsmgpu.h"

namespace lsmgpu {

// Experiment knobs.  The product library (liblsmgpu.so) compiles only the adopted decode and
// encode paths: every DecodeParams field marked "(diag)" below reads as its default there, and
// the rejected variants are not instantiated.  The diagnostic build (LSMGPU_DIAG, built as
// liblsmgpu_diag.so by `LSMGPU_BUILD_DIAG=1 python -m lsmdb_amd._build`) reads them from the
// LSMGPU_WSC_* / LSMGPU_ENC_* / LSMGPU_ABLATE environment and keeps the per-phase stamps, for
// the A/B records in DESIGN.md.
#ifdef LSMGPU_DIAG
#ifndef LSMGPU_STAMPS
#define LSMGPU_STAMPS 1
#endif
#define LSMGPU_KNOB(v, dflt) (v)
#else
#define LSMGPU_KNOB(v, dflt) (dflt)
#endif
// timing-only ablation bits (diag): 0 in the product library
#define ABLATE(p, m) LSMGPU_KNOB(((p).ablate & (m)), 0u)

// Decode: one-wave workgroups over a persistent, fully resident grid, one SST data block per
// iteration, software-pipelined (walk block k, emit block k-2); output bases from a two-level
// prefix over per-block {entries, key bytes, value bytes}.  DESIGN.md.
struct DecodeParams {
  const uint8_t* data;
  uint64_t data_len;
  const uint32_t* blk_off;
  const uint32_t* blk_len;
  uint32_t nblk;
  int mode;
  uint8_t* key_data;
  uint64_t key_cap;
  uint32_t* key_end;
  uint8_t* val_data;
  uint64_t val_cap;
  uint32_t* val_end;
  uint64_t* view;
  uint64_t ent_cap;
  uint32_t* blk_first;
  int32_t* blk_status;
  uint64_t* lb;             // per-block records: aggregate [0..2], exclusive prefix [4..6]
  uint64_t* glb;            // per-group records (64 blocks): aggregate [0..2], inclusive [4..6]
  uint32_t* gcnt;           // [0]: tile ticket of the walk / fused tile kernels (0 between launches)
  uint64_t* result;         // 8 u64, zeroed before launch
  uint32_t tag;             // 24-bit epoch tag of this launch
  uint32_t ablate;          // timing-only diagnostics (LSMGPU_ABLATE): 1 no prefix, 2 no emit, 4 no walk
                            // (walk-scan-copy: 1 no look-back, 2 no copy, 4 no group walk)
  uint32_t* census;         // residency census mode (launch_decode calibration), else nullptr
  uint64_t* stamps;         // per-phase s_memtime totals (LSMGPU_STAMPS diagnostics), else nullptr
  // walk-scan-copy path (decode_wsc.hip): per-entry metadata (2 words x wcap per block),
  // per-block descriptor for the copy, 32 B: wdesc[2b] = {n, K, V, status | kPlenFlag},
  // wdesc[2b + 1] = {entry base, key base, value base, input offset} (written once, by the walk
  // epilogue; two 16-B loads in the copy instead of five arrays)
  uint32_t* wmeta;
  uint32_t wcap;
  uint4* wdesc;
  uint32_t wsplit;          // walk-scan-copy: waves per block in the copy (1, 2 or 4)
  uint32_t wj;              // walk-scan-copy: lanes per entry forced (8, 16), 0 = per block
  uint32_t wfuse;           // walk-scan-copy, view-only mode: the walk writes the view index
                            // and per-block outputs itself (no copy launch)
  uint32_t wwalk;           // walk-scan-copy walk: kWalkLane / kWalkGroup (+ wlanes)
  uint32_t wlanes;          // kWalkGroup: lanes per block (4, 8 or 16)
  uint32_t zero_result;     // walk-scan-copy with a copy launch: the walk zeroes result[0..7]
  uint32_t wchunk;          // lane walk: records per flushed chunk (16 or 32)
  uint32_t wkeep;           // view-only lane walk: records kept in LDS (kWalkLaneView)
  uint32_t wtile;           // lane walks: blocks (= threads) per workgroup: 256 ((diag) 64, 128, 192)
  uint32_t walign;          // copy: aligned 16-B output chunks for blocks of <= 63 entries
  uint32_t wwide;           // lane walks: 0 (256-block tiles, 4 per CU) or 576 (2 per CU)
  uint32_t wlbfull;         // walk: every thread of a tile sums predecessor aggregates (no windows)
  uint32_t wpad;            // lane walk (256-block tiles): dynamic LDS bytes (residency experiments)
  uint32_t wbidir;          // group walk: 8 lanes forward + 8 backward per block (kWalkGroupBi)
  uint32_t weo;             // lane walk (materialize): the walk writes key_end / val_end / view
  uint32_t weosep;          // copy, 16 lanes per entry: per-entry outputs in a separate pass
  uint32_t wtbe;            // wide lane walks: blocks per tile (<= 576; set whenever wwide is)
  uint32_t wpersist;        // wide lane walk (materialize): two tiles per workgroup, walked back to back
  uint32_t wscopy;          // 64-lane staged group walk: each wave copies its block from LDS
  uint32_t wslot;           // 64-lane staged group walk: 0 = kStageSlot, 1 = kStageSlotSmall
  uint32_t wsub;            // group walk: odd-shaped entries re-guessed inside a round
  uint32_t wview;           // kWalkLaneView: owners by scatter + max-scan (else binary search)
  uint32_t wdpp;            // group walk (<= 16 lanes): round results by DPP (else LDS shuffles)
  // (diag) group walks: the copy runs in the walk's launch -- workgroups drawing a ticket past
  // the tiles copy blocks as soon as their tile's descriptors are published (wncop of them)
  uint32_t wcopyfuse;
  uint32_t wncop;
  uint32_t wdense;          // (diag) copy: dense piece mapping for blocks of > 128-B entries (1)
  uint32_t wpipe;           // copy: pipelined 8-lane groups for blocks of < 64 entries (1), of any (2)
  uint32_t wdpipe;          // (diag) copy: the dense piece mapping pipelined (1)
  uint32_t wdmax;           // (diag) copy: largest average entry for the pipelined dense mapping (any)
  uint32_t wdmin;           // (diag) copy: the dense mapping above this average entry (128)
  uint32_t wpdepth;         // (diag) copy_entries_pipe: entry groups in flight + 1 (3)
  uint32_t wlbidir;         // lane walk: a second lane per block walking backward (blocks > 8 KiB)
  uint32_t wb16;            // (diag) group walk's backward reads: one 16-B load per header

};

// Encode: one wave per output block; every byte position is closed-form
// (pos(e) = 10e + key_start(e) + vs_start(e) + 13*block(e)), so no scan is needed.
struct EncodeParams {
  const uint8_t* keys;
  const uint32_t* key_end;
  const uint8_t* vs;
  const uint32_t* vs_end;
  uint64_t n;
  uint32_t epb;               // entries per block (when blk_first == nullptr)
  const uint32_t* blk_first;  // optional explicit plan (nblocks+1)
  uint32_t nblocks;
  uint64_t key_total, vs_total;
  uint8_t* out;
  uint64_t data_len;          // size of the data region (index starts here)
  uint32_t* flags;
  // multi-table mode (tbl_first != nullptr): table t = entries [tbl_first[t], tbl_first[t+1]),
  // blocks [tbl_blk[t], tbl_blk[t+1]) of epb entries, image at out + tbl_out[t]
  const uint32_t* tbl_first;
  const uint32_t* tbl_blk;
  const uint64_t* tbl_out;
  uint32_t ntables;
  // gather mode (src != nullptr): entry e's bytes are source entry src[e] of keys / vs, whose
  // ends are src_key_end / src_vs_end; key_end / vs_end are the entries' own (merged) ends
  const uint32_t* src;
  const uint32_t* src_key_end;
  const uint32_t* src_vs_end;
  uint32_t hdr16;  // set by launch_encode: header + the key's first 6 bytes as one 16-B store
  const uint8_t* pad;  // 16 readable device bytes: the source of loads no piece uses
  uint32_t dense;  // set by launch_encode: encode_dense_kernel for blocks of large entries
  uint32_t pipe;   // set by launch_encode: encode_pipe_kernel (next pass's first pieces loaded
                   // before this pass's stores)
};

// Builder.ReachedCapacity table cut over a sorted entry stream (encode.hip)
struct CutParams {
  const uint32_t* key_end;
  const uint32_t* vs_end;
  uint64_t n;
  uint32_t epb;
  int64_t cap;
  uint32_t* tbl_first;  // tables_cap + 1
  uint32_t* tbl_blk;    // tables_cap + 1
  uint64_t* tbl_out;    // tables_cap + 1
  uint32_t tables_cap;
  uint64_t* result;     // [0] tables, [1] blocks, [2] image bytes, [3] overflow
  // bloom != 0: each image also reserves Finish's bloom tail (JSON + BE32 length,
  // table/builder.go:189-195), sized by bbloom.New(cnt, 0.01) with host constants
  uint32_t bloom;
  double logw, ln2, ln2sq;  // ln(0.01), 0.69314718056, 0.69314718056^2 (Go's float64 values)
};
hipError_t launch_cut_tables(const CutParams& p, hipStream_t s);

struct ValuesParams {
  const uint8_t* meta;
  const uint8_t* user_meta;
  const uint64_t* expires_at;
  const uint8_t* values;
  const uint32_t* value_end;
  uint64_t n;
  uint8_t* vs;
  uint32_t* vs_end;   // input: already holds the scanned end offsets
};

// Batched table open (open_tables.hip): per-table scratch rpos (restart array position) and
// flags (error / unsorted bits), both ntables u32.
struct OpenParams {
  const uint8_t* data;
  uint64_t data_len;
  const uint64_t* sst_off;
  const uint64_t* sst_len;
  uint32_t ntables;
  lsmgpu_tables out;
  uint32_t* rpos;
  uint32_t* flags;
  uint64_t* result;
};
size_t open_scan_bytes(uint32_t ntables);
hipError_t launch_open_tables(const OpenParams& p, void* scan_tmp, size_t scan_bytes,
                              hipStream_t s);

// K-way merge (merge.hip): MergeIterator over nruns sorted runs of one key/value stream.
struct MergeParams {
  const uint8_t* kd;
  const uint32_t* ke;
  const uint8_t* vd;
  const uint32_t* ve;
  const uint32_t* run_first;  // nruns + 1
  uint32_t nruns;
  uint32_t n;                 // entries (run_first[nruns])
  uint32_t* dst;              // scratch: merged position -> entry
  uint4* rec;                 // scratch: merged position -> {ks, kept ? kl : 0, vs, vl}
  uint32_t* occ;              // scratch: positions taken by runs other than F (bitmap, chunks
                              // of kMergeEmitTile bits)
  uint32_t* cpre;             // scratch: occupied positions before each chunk
  uint8_t* drop;              // scratch: entry -> a duplicate (an equal key comes first)
  uint32_t* gcnt;             // emit tile ticket (0 between launches, reset by the last ticket)
  uint64_t* lb;               // emit tile records (64 B per tile, epoch-tagged)
  uint64_t tag;
  uint32_t* flags;            // scratch: [0] input errors, [1] capacity, [2] fill run F
  uint32_t* tile_base;        // scratch: nruns + 1
  uint32_t* spl;              // scratch: (n / 256 + nruns) x nruns splitter ranks
  uint8_t* okd;
  uint64_t key_cap;
  uint32_t* oke;
  uint8_t* ovd;
  uint64_t val_cap;
  uint32_t* ove;
  uint32_t* osrc;
  uint64_t ent_cap;
  uint64_t* result;
};
constexpr uint32_t kMergeEmitTile = 1024;  // merged positions per emit workgroup (the largest tile)
hipError_t launch_merge(const MergeParams& p, hipStream_t s);

// launchers (return hipError_t)
hipError_t launch_decode(const DecodeParams& p, uint32_t max_blk_len, int num_cus,
                         hipStream_t s, uint64_t* waves_launched);
hipError_t launch_encode(const EncodeParams& p, int num_cus, hipStream_t s);
// walk-scan-copy decode (blocks < 64 KiB): scratch (wmeta, wdesc) sized by
// the caller; p.gcnt[0] = 0 between launches (the walk's tile ticket), p.lb tile records
// mid (optional): an event recorded between the walk and the copy launch (kernel timing)
hipError_t launch_decode_wsc(const DecodeParams& p, hipStream_t s, hipEvent_t mid = nullptr);

// bloom tail (bloom.hip; bbloom restated, table/builder.go:164-195, table/table.go:301)
struct BloomParams {
  const uint8_t* keys;
  const uint32_t* key_end;  // running end offsets: key i = keys[key_end[i-1], key_end[i])
  uint64_t n;
  uint64_t* bitset;         // bits / 64 little-endian words
  uint64_t mask;            // bits - 1
  uint64_t locs;            // setLocs
  uint32_t shift;           // 64 - log2(bits)
  uint32_t* flags;          // build: bit 0 = a key of <= 8 B
  uint8_t* has;             // probe: 1 = Has(key)
  const uint32_t* key_base; // key 0 starts at *key_base (a sub-range of a stream), else 0
};
struct BloomJson {
  const uint64_t* bitset;
  uint64_t nbytes;          // bits / 8
  uint8_t* out;
  uint32_t head_len, tail_len;
  uint8_t text[64];         // head ++ tail (++ BE32 of the JSON length: Finish's bloomLen)
};
// Finish's bloom tails of up to kBloomSegs compaction tables in one build + one JSON launch
constexpr uint32_t kBloomSegs = 32;  // the segment table travels in the kernel arguments
struct BloomSeg {
  uint64_t word_off;   // the table's filter in the scratch (u64 words)
  uint64_t mask;       // bits - 1
  uint64_t json_out;   // byte offset of its JSON in out
  uint64_t group_off;  // first base64 group of this table in the JSON launch
  uint32_t first;      // first key (stream entry index)
  uint32_t shift;      // 64 - log2(bits)
  uint32_t locs;       // setLocs
  uint32_t tail_len;   // tail text bytes incl. the BE32 length
  uint8_t tail[28];    // ","SetLocs":N} ++ BE32(json length)
};
struct BloomTables {
  const uint8_t* keys;
  const uint32_t* key_end;
  const uint32_t* src;  // gather mode: key i is key src[i] of keys / key_end
  uint64_t* scratch;
  uint8_t* out;
  uint32_t* flags;
  uint32_t nseg;
  uint32_t end;        // one past the last key of the last table
  BloomSeg seg[kBloomSegs];
};
static_assert(sizeof(BloomTables) + 8 <= 4096, "kernel arguments are limited to 4 KiB");
hipError_t launch_bloom_tables(const BloomTables& p, uint64_t groups, hipStream_t s);
hipError_t launch_bloom_build(const BloomParams& p, hipStream_t s);
hipError_t launch_bloom_has(const BloomParams& p, hipStream_t s);
hipError_t launch_bloom_json(const BloomJson& p, hipStream_t s);

// walk-scan-copy walk modes (DecodeParams::wwalk)
constexpr int kWalkLane = 0;    // one lane per block, header by header from HBM
constexpr int kWalkGroup = 2;   // wlanes lanes per block, speculative same-shape runs from HBM
constexpr int kWalkGroupBi = 4; // the group walk plus a backward group per block (p.wbidir)
// the 64-lane group walk's LDS slot per block (bytes): 4 slots + rows leave 2 workgroups per CU
constexpr uint32_t kStageSlot = 19456;
constexpr uint32_t kStageSlotSmall = 4352;  // (LSMGPU_WSC_SLOT=small: C2's <= 4.2 KiB blocks)
constexpr int kWalkLaneView = 3;  // view-only lane walk keeping each block's records in LDS
constexpr uint32_t kViewRec = 33;  // records a kWalkLaneView LDS row keeps (more go to wmeta)
// which decode path a batch takes: 0 register-lag (<= 4 KiB), 1 LDS-lag, 2 walk-scan-copy
// (blocks < 64 KiB, batches of >= kWscMinBlocks blocks)
constexpr uint32_t kWscMinBlocks = 1024;
int decode_path(uint32_t max_blk_len, uint32_t nblk);
hipError_t launch_values_sizes(const ValuesParams& p, hipStream_t s);
hipError_t launch_values_write(const ValuesParams& p, hipStream_t s);

// probe.hip: practical streaming ceilings (kind 0 copy, 1 read, 2 copy nt, 3 read nt)
hipError_t launch_stream_probe(int kind, const void* src, void* dst, uint64_t bytes,
                               uint32_t grid, hipStream_t s);

}  // namespace lsmgpu
