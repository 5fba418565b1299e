/*
 * sstref.c -- CPU ORACLE (test infrastructure only) for the lsmdb SST block codec.
 * A line-by-line C restatement of the reference Go path; see sstref.h for scope and pinning.
 * Citations are relative to the reference checkout (impact-eintr/lsmdb @ v0).
 */
#include "sstref.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define MAXU32 0xFFFFFFFFu

static inline void put_be16(uint8_t* b, uint16_t v) { b[0] = (uint8_t)(v >> 8); b[1] = (uint8_t)v; }
static inline void put_be32(uint8_t* b, uint32_t v) {
  b[0] = (uint8_t)(v >> 24); b[1] = (uint8_t)(v >> 16); b[2] = (uint8_t)(v >> 8); b[3] = (uint8_t)v;
}
static inline uint16_t be16(const uint8_t* b) { return (uint16_t)((b[0] << 8) | b[1]); }
static inline uint32_t be32(const uint8_t* b) {
  return ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
}

/* ------------------------------------------------------------------ y/iterator.go */

/* y/iterator.go:20-29 sizeVarint */
int sstref_uvarint_size(uint64_t x) {
  int n = 0;
  for (;;) {
    n++;
    x >>= 7;
    if (x == 0) break;
  }
  return n;
}

/* y/iterator.go:31-38 EncodedSize -- note the silent uint16 truncation. */
uint16_t sstref_vs_encoded_size(uint64_t expires_at, size_t value_len) {
  size_t sz = value_len + 2; /* meta, usermeta */
  if (expires_at == 0) return (uint16_t)(sz + 1);
  return (uint16_t)(sz + (size_t)sstref_uvarint_size(expires_at));
}

/* y/iterator.go:48-62 Encode/EncodeTo: [Meta][UserMeta][uvarint ExpiresAt][Value] */
size_t sstref_vs_encode(uint8_t meta, uint8_t user_meta, uint64_t expires_at,
                        const uint8_t* value, size_t value_len, uint8_t* out) {
  size_t p = 0;
  out[p++] = meta;
  out[p++] = user_meta;
  uint64_t x = expires_at; /* encoding/binary.PutUvarint */
  while (x >= 0x80) {
    out[p++] = (uint8_t)(x | 0x80);
    x >>= 7;
  }
  out[p++] = (uint8_t)x;
  if (value_len) memcpy(out + p, value, value_len);
  return p + value_len;
}

/* y/iterator.go:40-46 Decode (binary.Uvarint semantics: overflow/short -> n<=0). */
int sstref_vs_decode(const uint8_t* b, size_t len, uint8_t* meta, uint8_t* user_meta,
                     uint64_t* expires_at) {
  if (len < 2) return -1;
  *meta = b[0];
  *user_meta = b[1];
  uint64_t x = 0;
  unsigned s = 0;
  for (size_t i = 2; i < len && i < 2 + 10; i++) {
    uint8_t c = b[i];
    if (c < 0x80) {
      if (i - 2 == 9 && c > 1) return -1; /* overflow */
      *expires_at = x | ((uint64_t)c << s);
      return (int)(i + 1);
    }
    x |= (uint64_t)(c & 0x7f) << s;
    s += 7;
  }
  return -1;
}

/* ------------------------------------------------------------------ y/y.go */

static int bytes_compare(const uint8_t* a, size_t la, const uint8_t* b, size_t lb) {
  size_t m = la < lb ? la : lb;
  int c = m ? memcmp(a, b, m) : 0;
  if (c) return c < 0 ? -1 : 1;
  return la < lb ? -1 : (la > lb ? 1 : 0);
}

/* y/y.go:84-90 CompareKeys (the len>8 assertion is the caller's contract). */
int sstref_compare_keys(const uint8_t* k1, size_t l1, const uint8_t* k2, size_t l2) {
  int c = bytes_compare(k1, l1 - 8, k2, l2 - 8);
  if (c) return c;
  return bytes_compare(k1 + l1 - 8, 8, k2 + l2 - 8, 8);
}

/* ------------------------------------------------------------------ table/builder.go */

struct sstref_builder {
  uint32_t counter;     /* builder.go:48 */
  uint8_t* buf;         /* builder.go:49 */
  size_t len, cap;
  size_t base_key_len;  /* builder.go:50 (only its emptiness matters, see keyDiff) */
  uint32_t base_offset; /* builder.go:51 */
  uint32_t* restarts;   /* builder.go:53 */
  size_t nrestarts, rcap;
  uint32_t prev_offset; /* builder.go:55 */
  uint64_t key_count;   /* builder.go:58 */
  uint32_t epb;         /* resultInterval, builder.go:14 */
  uint32_t block_bytes; /* opt-in byte-target cut (0 = off, reference behaviour) */
};

static void buf_write(sstref_builder* b, const void* p, size_t n) {
  if (b->len + n > b->cap) {
    size_t nc = b->cap ? b->cap : (1u << 20); /* newBuffer(1<<20), builder.go:17-21 */
    while (nc < b->len + n) nc *= 2;
    b->buf = (uint8_t*)realloc(b->buf, nc);
    b->cap = nc;
  }
  if (n) memcpy(b->buf + b->len, p, n);
  b->len += n;
}

static void push_restart(sstref_builder* b, uint32_t v) {
  if (b->nrestarts == b->rcap) {
    b->rcap = b->rcap ? 2 * b->rcap : 64;
    b->restarts = (uint32_t*)realloc(b->restarts, b->rcap * sizeof(uint32_t));
  }
  b->restarts[b->nrestarts++] = v;
}

sstref_builder* sstref_builder_new(uint32_t entries_per_block, uint32_t block_bytes) {
  sstref_builder* b = (sstref_builder*)calloc(1, sizeof(*b)); /* builder.go:61-67 */
  b->prev_offset = MAXU32;
  b->epb = entries_per_block;
  b->block_bytes = block_bytes;
  return b;
}

void sstref_builder_free(sstref_builder* b) {
  if (!b) return;
  free(b->buf);
  free(b->restarts);
  free(b);
}

int sstref_builder_empty(const sstref_builder* b) { return b->len == 0; } /* builder.go:71 */

/* builder.go:74-82 keyDiff.  The loop variable `i` shadows the outer `var i int`, so the
 * function ALWAYS returns newKey[0:]: plen is always 0. */
static size_t key_diff_start(const sstref_builder* b, const uint8_t* new_key, size_t nk) {
  size_t i_outer = 0;
  (void)new_key;
  for (size_t i = 0; i < nk && i < b->base_key_len; i++) {
    /* compares against baseKey and breaks -- without effect on i_outer */
  }
  return i_outer;
}

/* builder.go:84-118 addHelper */
static void add_helper(sstref_builder* b, const uint8_t* key, size_t klen, const uint8_t* vs,
                       size_t vlen_full) {
  if (klen > 0) b->key_count++; /* bloom staging, builder.go:86-93 (bloom is out of scope) */
  size_t diff_start;
  if (b->base_key_len == 0) { /* builder.go:96-98 */
    b->base_key_len = klen;
    diff_start = 0;
  } else {
    diff_start = key_diff_start(b, key, klen); /* builder.go:100 */
  }
  size_t dlen = klen - diff_start;
  uint8_t h[10]; /* header{plen,klen,vlen,prev}.Encode, builder.go:30-35,103-113 */
  put_be16(h + 0, (uint16_t)(klen - dlen));
  put_be16(h + 2, (uint16_t)dlen);
  put_be16(h + 4, (uint16_t)vlen_full); /* uint16(v.EncodedSize()) */
  put_be32(h + 6, b->prev_offset);
  b->prev_offset = (uint32_t)b->len - b->base_offset; /* builder.go:109 */
  buf_write(b, h, 10);
  buf_write(b, key + diff_start, dlen);
  buf_write(b, vs, vlen_full); /* v.EncodeTo writes every byte, builder.go:116 */
  b->counter++;
}

/* builder.go:121-123 finishBlock: addHelper([]byte{}, ValueStruct{}) -> vs-enc = 00 00 00 */
static void finish_block(sstref_builder* b) {
  static const uint8_t empty_vs[3] = {0, 0, 0};
  add_helper(b, NULL, 0, empty_vs, 3);
}

/* builder.go:125-137 Add */
void sstref_builder_add(sstref_builder* b, const uint8_t* key, size_t klen, const uint8_t* vsenc,
                        size_t vlen_full) {
  int cut = (b->epb > 0 && b->counter >= b->epb);
  if (!cut && b->block_bytes > 0 && b->counter > 0) {
    size_t cur = b->len - b->base_offset;
    cut = (cur + 10 + klen + vlen_full + 13) > b->block_bytes;
  }
  if (cut) {
    finish_block(b);
    push_restart(b, (uint32_t)b->len);
    b->counter = 0;
    b->base_key_len = 0;
    b->base_offset = (uint32_t)b->len;
    b->prev_offset = MAXU32;
  }
  add_helper(b, key, klen, vsenc, vlen_full);
}

/* builder.go:140-143 ReachedCapacity */
int sstref_builder_reached_capacity(const sstref_builder* b, int64_t cap) {
  int64_t est = (int64_t)b->len + 8 + 4 * (int64_t)b->nrestarts + 8;
  return est > cap;
}

/* builder.go:163-198 Finish (minus bbloom) -> builder.go:146-160 blockIndex */
const uint8_t* sstref_builder_finish(sstref_builder* b, size_t* out_len, size_t* data_len,
                                     const uint32_t** restarts, size_t* nrestarts) {
  finish_block(b);                   /* builder.go:185 */
  push_restart(b, (uint32_t)b->len); /* builder.go:148 */
  if (data_len) *data_len = b->len;
  uint8_t w[4];
  for (size_t i = 0; i < b->nrestarts; i++) {
    put_be32(w, b->restarts[i]);
    buf_write(b, w, 4);
  }
  put_be32(w, (uint32_t)b->nrestarts); /* builder.go:158 */
  buf_write(b, w, 4);
  if (restarts) *restarts = b->restarts;
  if (nrestarts) *nrestarts = b->nrestarts;
  *out_len = b->len;
  return b->buf;
}

size_t sstref_build(const uint8_t* keys, const uint32_t* key_end, const uint8_t* vs,
                    const uint32_t* vs_end, size_t n, uint32_t entries_per_block,
                    uint32_t block_bytes, uint8_t* out, size_t cap, size_t* data_len,
                    uint32_t* restarts, size_t restarts_cap, size_t* nrestarts) {
  sstref_builder* b = sstref_builder_new(entries_per_block, block_bytes);
  uint32_t k0 = 0, v0 = 0;
  for (size_t i = 0; i < n; i++) {
    sstref_builder_add(b, keys + k0, key_end[i] - k0, vs + v0, vs_end[i] - v0);
    k0 = key_end[i];
    v0 = vs_end[i];
  }
  size_t len = 0, dl = 0, nr = 0;
  const uint32_t* rs = NULL;
  const uint8_t* p = sstref_builder_finish(b, &len, &dl, &rs, &nr);
  size_t ret = 0;
  if (len <= cap && (!restarts || nr <= restarts_cap)) {
    memcpy(out, p, len);
    if (restarts) memcpy(restarts, rs, nr * sizeof(uint32_t));
    ret = len;
  }
  if (data_len) *data_len = dl;
  if (nrestarts) *nrestarts = nr;
  sstref_builder_free(b);
  return ret;
}

/* ------------------------------------------------------------------ table/table.go */

/* table.go:177-215 readIndex: [blocks][restarts BE32 x N][N BE32][bloom JSON][BE32 bloomLen] */
int sstref_parse_index(const uint8_t* sst, size_t len, uint32_t* blk_off, uint32_t* blk_len,
                       size_t cap, size_t* nblk, size_t* bloom_off, size_t* bloom_len) {
  if (len < 8) return -1;
  size_t pos = len - 4;
  uint32_t bl = be32(sst + pos); /* table.go:181-183 */
  if ((size_t)bl > pos || pos - bl < 4) return -1;
  pos -= bl;
  if (bloom_off) *bloom_off = pos;
  if (bloom_len) *bloom_len = bl;
  pos -= 4; /* table.go:188-190 */
  uint32_t nr = be32(sst + pos);
  if ((uint64_t)nr * 4 > pos) return -1;
  pos -= (size_t)nr * 4; /* table.go:192-199 */
  *nblk = nr;
  if (nr > cap) return -2;
  uint32_t prev = 0;
  for (uint32_t i = 0; i < nr; i++) { /* table.go:202-215 */
    uint32_t o = be32(sst + pos + 4 * (size_t)i);
    if (o < prev || (size_t)o > pos) return -1;
    blk_off[i] = prev;
    blk_len[i] = o - prev;
    prev = o;
  }
  return 0;
}

/* ------------------------------------------------------------------ table/iterator.go */

typedef struct {
  uint8_t* key_data; size_t key_cap; uint32_t* key_end;
  uint8_t* val_data; size_t val_cap; uint32_t* val_end;
  uint64_t* view; size_t ent_cap;
  uint64_t ne, kb, vb;
  int overflow;
} sink_t;

/* One blockIterator walked forward from SeekToFirst until Valid() is false
 * (iterator.go:81-84 SeekToFirst -> Init -> Next, then Next repeatedly, iterator.go:112-135).
 * `blk` is the block slice; `blk_abs` its offset in the data buffer (for the view index). */
static int decode_block(const uint8_t* blk, uint32_t len, uint32_t blk_abs, sink_t* s) {
  uint32_t pos = 0;             /* iterator.go:15 */
  int have_base = 0;            /* len(itr.baseKey) != 0 */
  uint32_t base_pos = 0;        /* baseKey = data[base_pos : ...] (iterator.go:132) */
  for (;;) {
    if (pos >= len) return SSTREF_BLK_OK; /* iterator.go:115-118 -> io.EOF */
    if (len - pos < 10) return SSTREF_BLK_TRUNC_HEADER; /* Go would read past the block */
    uint16_t plen = be16(blk + pos), klen = be16(blk + pos + 2), vlen = be16(blk + pos + 4);
    pos += 10;                                     /* iterator.go:121 */
    if (klen == 0 && plen == 0) return SSTREF_BLK_OK; /* iterator.go:124-127 terminator */
    if (!have_base) {                              /* iterator.go:129-133 */
      if (plen != 0) return SSTREF_BLK_FIRST_PLEN; /* y.AssertTrue(h.plen == 0) */
      base_pos = pos;
      have_base = 1; /* klen > 0 here, so baseKey is non-empty */
    }
    /* parseKV, iterator.go:93-110.  baseKey[:plen] may extend past len(baseKey) (Go slices
     * up to cap), i.e. it is data[base_pos : base_pos+plen]; past the block -> PREFIX_OOB. */
    if ((uint64_t)base_pos + plen > len) return SSTREF_BLK_PREFIX_OOB;
    uint32_t kpos = pos;
    pos += klen;                                        /* iterator.go:101 */
    if ((uint64_t)pos + vlen > len) return SSTREF_BLK_VALUE_OVERFLOW; /* iterator.go:103-106 */
    uint32_t vpos = pos;
    pos += vlen;                                        /* iterator.go:109 */
    /* emit (key, value) */
    uint64_t i = s->ne;
    uint32_t kfull = (uint32_t)plen + klen;
    if (s->key_data || s->key_end) {
      if (s->kb + kfull > s->key_cap || s->kb + kfull > 0xFFFFFFFFull) s->overflow = 1;
      else if (s->key_data) {
        memcpy(s->key_data + s->kb, blk + base_pos, plen);
        memcpy(s->key_data + s->kb + plen, blk + kpos, klen);
      }
    }
    if (s->val_data || s->val_end) {
      if (s->vb + vlen > s->val_cap || s->vb + vlen > 0xFFFFFFFFull) s->overflow = 1;
      else if (s->val_data) memcpy(s->val_data + s->vb, blk + vpos, vlen);
    }
    s->kb += kfull;
    s->vb += vlen;
    if (i >= s->ent_cap) s->overflow = 1;
    else {
      if (s->key_end) s->key_end[i] = (uint32_t)s->kb;
      if (s->val_end) s->val_end[i] = (uint32_t)s->vb;
      if (s->view)
        s->view[i] = (uint64_t)(uint32_t)(blk_abs + kpos) | ((uint64_t)klen << 32) |
                     ((uint64_t)vlen << 48);
    }
    s->ne++;
  }
}

int sstref_decode_blocks(const uint8_t* data, size_t data_len, const uint32_t* blk_off,
                         const uint32_t* blk_len, size_t nblk,
                         uint8_t* key_data, size_t key_cap, uint32_t* key_end,
                         uint8_t* val_data, size_t val_cap, uint32_t* val_end,
                         uint64_t* view, size_t ent_cap,
                         uint32_t* blk_first, int32_t* blk_status, sstref_totals* tot) {
  sink_t s;
  memset(&s, 0, sizeof(s));
  s.key_data = key_data; s.key_cap = key_cap; s.key_end = key_end;
  s.val_data = val_data; s.val_cap = val_cap; s.val_end = val_end;
  s.view = view; s.ent_cap = ent_cap;
  int64_t first_bad = -1;
  uint64_t nbad = 0;
  for (size_t b = 0; b < nblk; b++) {
    if (blk_first) blk_first[b] = (uint32_t)s.ne;
    int st;
    if ((uint64_t)blk_off[b] + blk_len[b] > data_len) st = SSTREF_BLK_RANGE;
    else st = decode_block(data + blk_off[b], blk_len[b], blk_off[b], &s);
    if (blk_status) blk_status[b] = st;
    if (st != SSTREF_BLK_OK) {
      nbad++;
      if (first_bad < 0) first_bad = (int64_t)b;
    }
  }
  if (blk_first) blk_first[nblk] = (uint32_t)s.ne;
  if (tot) {
    tot->n_entries = s.ne; tot->key_bytes = s.kb; tot->val_bytes = s.vb;
    tot->first_bad_block = first_bad; tot->n_bad_blocks = nbad; tot->overflow = s.overflow;
  }
  return s.overflow;
}

/* ------------------------------------------------------------------ CPU baseline timing */

typedef struct {
  const uint8_t* data; size_t data_len; const uint32_t* off; const uint32_t* len;
  size_t b0, b1; int reps; uint64_t csum; pthread_barrier_t* bar; double secs;
} bench_arg;

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static void* bench_worker(void* p) {
  bench_arg* a = (bench_arg*)p;
  /* per-thread materialise buffers sized by the range's input bytes (plen==0 data) */
  uint64_t in_bytes = 0, max_ent = 0;
  for (size_t b = a->b0; b < a->b1; b++) { in_bytes += a->len[b]; max_ent += a->len[b] / 10 + 1; }
  uint8_t* kd = (uint8_t*)malloc(in_bytes + 16);
  uint8_t* vd = (uint8_t*)malloc(in_bytes + 16);
  uint32_t* ke = (uint32_t*)malloc(max_ent * 4 + 16);
  uint32_t* ve = (uint32_t*)malloc(max_ent * 4 + 16);
  uint32_t* bf = (uint32_t*)malloc((a->b1 - a->b0 + 1) * 4);
  int32_t* bs = (int32_t*)malloc((a->b1 - a->b0 + 1) * 4);
  uint64_t cs = 0;
  for (int r = -1; r < a->reps; r++) { /* r == -1: untimed warm-up (page faults) */
    if (r == 0) { pthread_barrier_wait(a->bar); a->secs = now_s(); }
    sstref_totals t;
    sstref_decode_blocks(a->data, a->data_len, a->off + a->b0, a->len + a->b0, a->b1 - a->b0,
                         kd, in_bytes, ke, vd, in_bytes, ve, NULL, max_ent, bf, bs, &t);
    cs += t.n_entries * 1315423911ull + t.key_bytes + t.val_bytes;
    if (t.n_entries) cs ^= ke[t.n_entries - 1] + ((uint64_t)ve[t.n_entries - 1] << 20);
  }
  a->secs = now_s() - a->secs;
  a->csum = cs;
  free(kd); free(vd); free(ke); free(ve); free(bf); free(bs);
  return NULL;
}

double sstref_decode_bench(const uint8_t* data, size_t data_len, const uint32_t* blk_off,
                           const uint32_t* blk_len, size_t nblk, int nthreads, int reps,
                           uint64_t* checksum) {
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  bench_arg* args = (bench_arg*)calloc((size_t)nthreads, sizeof(bench_arg));
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, NULL, (unsigned)nthreads);
  for (int t = 0; t < nthreads; t++) {
    args[t].data = data; args[t].data_len = data_len; args[t].off = blk_off; args[t].len = blk_len;
    args[t].b0 = nblk * (size_t)t / (size_t)nthreads;
    args[t].b1 = nblk * (size_t)(t + 1) / (size_t)nthreads;
    args[t].reps = reps;
    args[t].bar = &bar;
  }
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, bench_worker, &args[t]);
  uint64_t cs = 0;
  double secs = 0;
  for (int t = 0; t < nthreads; t++) {
    pthread_join(th[t], NULL);
    cs += args[t].csum;
    if (args[t].secs > secs) secs = args[t].secs; /* max over threads */
  }
  pthread_barrier_destroy(&bar);
  if (checksum) *checksum = cs;
  free(th); free(args);
  return secs;
}

/* ------------------------------------------------------------------ table/table.go OpenTable */

static const uint8_t* g_sort_sst;   /* qsort context (single-threaded test oracle) */
static const uint32_t* g_sort_koff;
static const uint32_t* g_sort_klen;
static int cmp_block_keys(const void* a, const void* b) {
  const uint32_t i = *(const uint32_t*)a, j = *(const uint32_t*)b;
  int c = sstref_compare_keys(g_sort_sst + g_sort_koff[i], g_sort_klen[i],
                              g_sort_sst + g_sort_koff[j], g_sort_klen[j]);
  if (c) return c;
  return i < j ? -1 : (i > j ? 1 : 0); /* ties: SST order (documented divergence) */
}

int sstref_open_table(const uint8_t* sst, size_t len, uint32_t* blk_off, uint32_t* blk_len,
                      uint32_t* key_off, uint32_t* key_len, uint32_t* order, size_t cap,
                      sstref_table_info* info) {
  memset(info, 0, sizeof(*info));
  size_t nblk = 0, bo = 0, bl = 0;
  int rc = sstref_parse_index(sst, len, blk_off, blk_len, cap, &nblk, &bo, &bl);
  if (rc == -1) return info->status = SSTREF_TBL_BAD_TAIL;
  info->nblk = (uint32_t)nblk;
  if (rc == -2) return info->status = SSTREF_TBL_CAPACITY;
  info->bloom_off = (uint32_t)bo;
  info->bloom_len = (uint32_t)bl;
  /* readIndex first headers and keys (table.go:219-256): t.read checks the whole file */
  int plen_bad = 0, read_bad = 0;
  for (size_t i = 0; i < nblk; i++) {
    const size_t off = blk_off[i];
    key_off[i] = 0;
    key_len[i] = 0;
    if (off + 10 > len) { read_bad = 1; continue; }           /* "While reading first header" */
    const uint16_t plen = be16(sst + off), klen = be16(sst + off + 2);
    if (plen != 0) { plen_bad = 1; continue; }                /* table.go:239 */
    if (off + 10 + klen > len) { read_bad = 1; continue; }    /* "While reading first key" */
    key_off[i] = (uint32_t)(off + 10);
    key_len[i] = klen;
  }
  if (plen_bad) return info->status = SSTREF_TBL_FIRST_PLEN;
  if (read_bad) return info->status = SSTREF_TBL_READ;
  for (size_t i = 0; i < nblk; i++) order[i] = (uint32_t)i;
  if (nblk >= 2) {                                            /* table.go:267 sort.Sort(byKey) */
    for (size_t i = 0; i < nblk; i++)
      if (key_len[i] <= 8) return info->status = SSTREF_TBL_KEY_LEN; /* y.go:85 */
    g_sort_sst = sst;
    g_sort_koff = key_off;
    g_sort_klen = key_len;
    qsort(order, nblk, sizeof(uint32_t), cmp_block_keys);
  }
  if (nblk == 0) return info->status = SSTREF_TBL_OK;         /* both iterators: io.EOF */
  /* smallest: seekToFirst -> block order[0] SeekToFirst -> Init -> Next (iterator.go:81-84,112-135) */
  {
    const uint32_t b = order[0], off = blk_off[b], bl = blk_len[b];
    if (bl >= 10) {
      const uint16_t plen = be16(sst + off), klen = be16(sst + off + 2), vlen = be16(sst + off + 4);
      if (!(klen == 0 && plen == 0) && 10u + klen + vlen <= bl) {
        info->has_smallest = 1;
        info->smallest_off = off + 10;
        info->smallest_len = klen;
      }
    }
  }
  /* biggest: seekToLast -> block order[n-1].SeekToLast: Next until invalid, then Prev().
   * Go's block slice is a window of the mmap'd file: reads past the block but inside the
   * file (headers, keys, baseKey[:plen]) are legal and read the following bytes; only reads
   * past the file panic (-> SSTREF_TBL_BIGGEST).  Bounds below are therefore `len`. */
  {
    const uint32_t b = order[nblk - 1], off = blk_off[b], bl = blk_len[b];
    uint32_t pos = 0, last_prev = 0;                          /* itr.last: the zero header */
    int have_base = 0, bad = 0;
    for (;;) {                                                /* Next(), iterator.go:112-135 */
      if (pos >= bl) break;                                   /* io.EOF */
      if ((size_t)off + pos + 10 > len) { bad = 1; break; }   /* h.Decode past the file */
      const uint16_t plen = be16(sst + off + pos), klen = be16(sst + off + pos + 2),
                     vlen = be16(sst + off + pos + 4);
      last_prev = be32(sst + off + pos + 6);
      pos += 10;
      if (klen == 0 && plen == 0) break;                      /* io.EOF */
      if (!have_base) {
        if (plen != 0) { bad = 1; break; }                    /* AssertTrue(h.plen == 0) */
        if ((size_t)off + pos + klen > len) { bad = 1; break; }
        have_base = 1;                                        /* baseKey = data[10:10+klen] */
      }
      if ((size_t)off + 10 + plen > len || (size_t)off + pos + klen > len) { bad = 1; break; }
      pos += klen;                                            /* parseKV */
      if (pos + vlen > bl) break;                             /* "Value exceeded": invalid */
      pos += vlen;
    }
    if (!bad && last_prev != MAXU32) {                        /* Prev(), iterator.go:137-155 */
      const uint32_t p = last_prev;
      if (p >= bl || (size_t)off + p + 10 > len) {
        bad = 1;                                              /* AssertTruef(pos < len) / Decode */
      } else {
        const uint16_t plen = be16(sst + off + p), klen = be16(sst + off + p + 2),
                       vlen = be16(sst + off + p + 4);
        const size_t base_cap = have_base ? len - (off + 10) : 0; /* cap(baseKey) */
        if (plen > base_cap || (size_t)off + p + 10 + klen > len) {
          bad = 1;
        } else if ((uint64_t)p + 10 + klen + vlen <= bl) {    /* else parseKV error: invalid */
          info->has_biggest = 1;
          info->big_base_off = off + 10;
          info->big_plen = plen;
          info->big_diff_off = off + p + 10;
          info->big_klen = klen;
        }
      }
    }
    if (bad) return info->status = SSTREF_TBL_BIGGEST;
  }
  return info->status = SSTREF_TBL_OK;
}

/* ------------------------------------------------------------------ y/iterator.go MergeIterator */

static inline const uint8_t* key_at(const uint8_t* kd, const uint32_t* ke, uint32_t i, uint32_t* len) {
  const uint32_t s = i ? ke[i - 1] : 0;
  *len = ke[i] - s;
  return kd + s;
}

size_t sstref_merge(const uint8_t* kd, const uint32_t* ke, const uint32_t* run_first,
                    size_t nruns, uint32_t* out_src, size_t cap) {
  uint32_t* cur = (uint32_t*)malloc((nruns + 1) * sizeof(uint32_t));
  for (size_t r = 0; r < nruns; r++) cur[r] = run_first[r];
  size_t n = 0;
  int have_last = 0;
  uint32_t last = 0;
  for (;;) {
    /* the heap top: least valid head by (CompareKeys, nice)  (elemHeap.Less, y/iterator.go:82-93) */
    long best = -1;
    for (size_t r = 0; r < nruns; r++) {
      if (cur[r] >= run_first[r + 1]) continue; /* !Valid(): popped (y/iterator.go:166-169) */
      if (best < 0) { best = (long)r; continue; }
      uint32_t la, lb;
      const uint8_t* a = key_at(kd, ke, cur[r], &la);
      const uint8_t* b = key_at(kd, ke, cur[best], &lb);
      if (sstref_compare_keys(a, la, b, lb) < 0) best = (long)r; /* ties: lower nice (r) stays */
    }
    if (best < 0) break;
    const uint32_t i = cur[best]++;
    if (have_last) { /* Next(): skip heads equal to curKey (bytes.Equal, y/iterator.go:172-181) */
      uint32_t la, lb;
      const uint8_t* a = key_at(kd, ke, i, &la);
      const uint8_t* b = key_at(kd, ke, last, &lb);
      if (la == lb && memcmp(a, b, la) == 0) continue;
    }
    if (n >= cap) { free(cur); return (size_t)-1; }
    out_src[n++] = i;
    last = i;
    have_last = 1;
  }
  free(cur);
  return n;
}
