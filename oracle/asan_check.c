/* asan_check.c -- test infrastructure: drives the oracle (sstref.c, bbloom.c) under
 * AddressSanitizer + UndefinedBehaviorSanitizer on the host (`make -C oracle build/asan_check`,
 * run by tests/test_oracle_asan.py).  Valid tables built by the oracle Builder are parsed,
 * opened, decoded (round trip checked) and merged; then the same tables with random byte
 * corruption, truncated blocks and broken tails go through the same readers, which must
 * report statuses without touching memory outside their inputs and outputs (the GPU path is
 * checked against these readers, so a read past a buffer here would hide in every parity
 * test).  Exit status 0 = clean; any sanitizer report aborts. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sstref.h"

static uint64_t rng_state;
static uint64_t rnd(void) {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 7;
  rng_state ^= rng_state << 17;
  return rng_state;
}
static uint32_t rnd_in(uint32_t lo, uint32_t hi) { return lo + (uint32_t)(rnd() % (hi - lo + 1)); }

/* n entries: 8-B big-endian counter + filler + 8-B ts (sorted, distinct), random ValueStructs */
typedef struct {
  size_t n;
  uint8_t *keys, *vs;
  uint32_t *key_end, *vs_end;
} cols;

static void make_cols(cols* c, size_t n, uint64_t start, uint64_t stride) {
  c->n = n;
  c->key_end = malloc(n * 4 + 4);
  c->vs_end = malloc(n * 4 + 4);
  c->keys = malloc(n * 48 + 1);
  c->vs = malloc(n * (12 + 10 + 80) + 1);
  size_t kb = 0, vb = 0;
  for (size_t i = 0; i < n; i++) {
    const uint64_t ctr = start + i * stride;
    for (int j = 0; j < 8; j++) c->keys[kb++] = (uint8_t)(ctr >> (56 - 8 * j));
    const uint32_t fill = rnd_in(1, 24);
    for (uint32_t j = 0; j < fill; j++) c->keys[kb++] = (uint8_t)('a' + rnd() % 26);
    const uint64_t ts = rnd() >> 4;
    for (int j = 0; j < 8; j++) c->keys[kb++] = (uint8_t)(ts >> (56 - 8 * j));
    c->key_end[i] = (uint32_t)kb;
    uint8_t val[80];
    const uint32_t vl = rnd_in(0, 80);
    for (uint32_t j = 0; j < vl; j++) val[j] = (uint8_t)rnd();
    const uint64_t exp = (rnd() & 3) ? 0 : (rnd() >> rnd_in(0, 63)) | 1;
    vb += sstref_vs_encode((uint8_t)(rnd() & 3), (uint8_t)rnd(), exp, val, vl, c->vs + vb);
    c->vs_end[i] = (uint32_t)vb;
  }
}

static void free_cols(cols* c) {
  free(c->keys);
  free(c->vs);
  free(c->key_end);
  free(c->vs_end);
}

/* decode every block of data[0:data_len) into buffers of exactly the given capacities */
static int decode_all(const uint8_t* data, size_t data_len, const uint32_t* off,
                      const uint32_t* len, size_t nblk, size_t key_cap, size_t val_cap,
                      size_t ent_cap, sstref_totals* tot, uint8_t** kd_out, uint32_t** ke_out) {
  uint8_t* kd = malloc(key_cap + 1);
  uint8_t* vd = malloc(val_cap + 1);
  uint32_t* ke = malloc(ent_cap * 4 + 4);
  uint32_t* ve = malloc(ent_cap * 4 + 4);
  uint64_t* view = malloc(ent_cap * 8 + 8);
  uint32_t* first = malloc(nblk * 4 + 4);
  int32_t* st = malloc(nblk * 4 + 4);
  const int rc = sstref_decode_blocks(data, data_len, off, len, nblk, kd, key_cap, ke, vd,
                                      val_cap, ve, view, ent_cap, first, st, tot);
  free(vd);
  free(ve);
  free(view);
  free(first);
  free(st);
  if (kd_out) *kd_out = kd; else free(kd);
  if (ke_out) *ke_out = ke; else free(ke);
  return rc;
}

static int check_table(const cols* c, uint32_t epb, uint32_t bb, int corrupt) {
  const size_t cap = 10 * c->n + c->key_end[c->n - 1] + c->vs_end[c->n - 1] + 13 * (c->n + 1) +
                     4 * (c->n + 2) + 64;
  uint8_t* sst = malloc(cap);
  uint32_t* rs = malloc((c->n + 2) * 4);
  size_t data_len = 0, nr = 0;
  const size_t total = sstref_build(c->keys, c->key_end, c->vs, c->vs_end, c->n, epb, bb, sst,
                                    cap, &data_len, rs, c->n + 2, &nr);
  if (!total) return 1;
  /* an empty bloom tail: "{}" + BE32(2) */
  uint8_t* tbl = malloc(total + 6);
  memcpy(tbl, sst, total);
  memcpy(tbl + total, "{}\0\0\0\2", 6);
  const size_t tlen = total + 6;
  if (corrupt) { /* random bytes anywhere, then a random cut of the whole file */
    const uint32_t flips = rnd_in(1, 64);
    for (uint32_t i = 0; i < flips; i++) tbl[rnd() % tlen] = (uint8_t)rnd();
  }
  const size_t use = corrupt && (rnd() & 1) ? (size_t)(rnd() % (tlen + 1)) : tlen;
  uint8_t* exact = malloc(use ? use : 1); /* exactly `use` bytes: ASan sees any over-read */
  memcpy(exact, tbl, use);
  const size_t bcap = nr + 8;
  uint32_t* off = malloc(bcap * 4);
  uint32_t* len = malloc(bcap * 4);
  size_t nblk = 0, bo = 0, bl = 0;
  const int prc = sstref_parse_index(exact, use, off, len, bcap, &nblk, &bo, &bl);
  int bad = 0;
  if (prc == 0) {
    size_t dlen = 0;
    for (size_t b = 0; b < nblk; b++) {
      const size_t e = (size_t)off[b] + len[b];
      if (e <= use && e > dlen) dlen = e;
    }
    /* blocks past the file are reported by status, never read */
    sstref_totals tot;
    uint8_t* kd = NULL;
    uint32_t* ke = NULL;
    const size_t kcap = corrupt ? (size_t)rnd_in(0, c->key_end[c->n - 1] + 64) : c->key_end[c->n - 1];
    const size_t vcap = corrupt ? (size_t)rnd_in(0, c->vs_end[c->n - 1] + 64) : c->vs_end[c->n - 1];
    const size_t ecap = corrupt ? (size_t)rnd_in(0, (uint32_t)c->n + 8) : c->n;
    const int drc = decode_all(exact, dlen, off, len, nblk, kcap, vcap, ecap, &tot, &kd, &ke);
    if (!corrupt) { /* the round trip */
      bad |= drc != 0 || tot.n_entries != c->n || tot.n_bad_blocks != 0;
      bad |= memcmp(kd, c->keys, c->key_end[c->n - 1]) != 0;
      bad |= memcmp(ke, c->key_end, c->n * 4) != 0;
    }
    free(kd);
    free(ke);
  } else if (!corrupt) {
    bad = 1;
  }
  /* OpenTable's index work on the same bytes */
  uint32_t* ko = malloc(bcap * 4);
  uint32_t* kl = malloc(bcap * 4);
  uint32_t* ord = malloc(bcap * 4);
  sstref_table_info info;
  const int orc = sstref_open_table(exact, use, off, len, ko, kl, ord, bcap, &info);
  if (!corrupt) bad |= orc != SSTREF_TBL_OK;
  free(ko);
  free(kl);
  free(ord);
  free(off);
  free(len);
  free(exact);
  free(tbl);
  free(sst);
  free(rs);
  return bad;
}

static int check_merge(void) {
  /* three overlapping sorted runs over one key stream, duplicates across and inside runs */
  cols r[3];
  size_t n = 0;
  for (int k = 0; k < 3; k++) {
    make_cols(&r[k], rnd_in(1, 400), rnd() % 50, (uint64_t)rnd_in(1, 3));
    n += r[k].n;
  }
  uint32_t* ke = malloc(n * 4);
  uint8_t* kd = malloc(n * 48);
  uint32_t rf[4] = {0, 0, 0, 0};
  size_t kb = 0, e = 0;
  for (int k = 0; k < 3; k++) {
    rf[k] = (uint32_t)e;
    for (size_t i = 0; i < r[k].n; i++) {
      const uint32_t s = i ? r[k].key_end[i - 1] : 0, l = r[k].key_end[i] - s;
      memcpy(kd + kb, r[k].keys + s, l);
      /* the same ts for equal counters: equal keys across runs */
      memset(kd + kb + l - 8, (int)(kd[kb + 7] & 1), 8);
      kb += l;
      ke[e++] = (uint32_t)kb;
    }
  }
  rf[3] = (uint32_t)e;
  uint32_t* out = malloc(n * 4 + 4);
  const size_t m = sstref_merge(kd, ke, rf, 3, out, n);
  int bad = m == (size_t)-1 || m > n;
  for (int k = 0; k < 3; k++) free_cols(&r[k]);
  free(ke);
  free(kd);
  free(out);
  return bad;
}

static int check_bloom(const cols* c) {
  uint64_t bits = 0, locs = 0;
  uint32_t exp = 0;
  sstref_bloom_params((double)c->n, 0.01, &bits, &locs, &exp);
  uint64_t* bs = calloc(bits / 64 + 1, 8);
  if (sstref_bloom_build(c->keys, c->key_end, c->n, bs, bits, exp, locs) != 0) return 1;
  int bad = 0;
  for (size_t i = 0; i < c->n; i++) {
    const uint32_t s = i ? c->key_end[i - 1] : 0, l = c->key_end[i] - s;
    bad |= !sstref_bloom_has(bs, bits, exp, locs, c->keys + s, l - 8);  /* keyNoTs */
  }
  const size_t jcap = bits / 8 * 2 + 256;
  uint8_t* js = malloc(jcap);
  bad |= sstref_bloom_json(bs, bits, locs, js, jcap) == 0;
  free(js);
  free(bs);
  return bad;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  rng_state = 0x9e3779b97f4a7c15ull;
  int fails = 0;
  for (int it = 0; it < iters; it++) {
    cols c;
    make_cols(&c, rnd_in(1, 3000), rnd() % 1000, 1);
    const uint32_t epb = rnd_in(1, 200), bb = (rnd() & 1) ? rnd_in(64, 8192) : 0;
    fails += check_table(&c, epb, bb, 0);
    for (int k = 0; k < 4; k++) (void)check_table(&c, epb, bb, 1); /* statuses only */
    fails += check_merge();
    if ((it & 7) == 0) fails += check_bloom(&c);
    free_cols(&c);
  }
  printf("asan_check: %d iterations, %d failures\n", iters, fails);
  return fails != 0;
}
