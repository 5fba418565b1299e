/*
 * bbloom.c -- CPU ORACLE for the SST bloom tail.  TEST INFRASTRUCTURE ONLY (see sstref.h).
 *
 * The reference builds the tail with github.com/AndreasBriese/bbloom
 * v0.0.0-20190825152654-46b345b51c96 (go.mod:6, go.sum:1-2), which is not vendored under
 * /root/reference and cannot be fetched.  This file restates that version's published
 * algorithm, anchored on the reference's call sites:
 *   table/builder.go:86-93    addHelper: keyBuf gets ParseKey(key) (the key minus its 8-B ts)
 *   table/builder.go:164-181  Finish: bbloom.New(float64(keyCount), 0.01), Add(every keyBuf key)
 *   table/builder.go:189-195  bf.JSONMarshal() written after the index, then its BE32 length
 *   table/table.go:180-186    readIndex: bbloom.JSONUnmarshal(tail)
 *   table/table.go:301        DoesNotHave(key) = !bf.Has(key)  (level_handler.go:224 passes keyNoTs)
 * bbloom's algorithm, as restated:
 *   New(n, wrongs < 1): size = -1 * n * ln(wrongs) / 0.69314718056^2 (float64),
 *     locs = ceil(0.69314718056 * size / n); then getSize(uint64(size)): the next power of
 *     two >= max(uint64(size), 512) = 2^exp bits; Bloom{size: 2^exp - 1, setLocs: locs,
 *     shift: 64 - exp}, bitset = 2^exp / 64 uint64 words.
 *   sipHash(key): SipHash-2-4 with k0 = 0xdeadbeaf, k1 = 0xfaebdaed (bbloom's initial state
 *     v0..v3 = 8317987320269560794, 7237128889637516672, 7816392314733513934,
 *     8387220255325274014), hash = v0 ^ v1 ^ v2 ^ v3, h = hash >> shift,
 *     l = hash << shift >> shift.
 *   Add(key): for i < setLocs: set bit (h + i * l) & size -- byte ((idx % 64) >> 3) of word
 *     idx >> 6, mask 1 << (idx % 8): bit idx % 64 of the little-endian word.
 *   Has(key): all setLocs bits set.
 *   JSONMarshal: {"FilterSet":"<base64 std of the bitset's bytes>","SetLocs":<locs>}.
 * Parity status: the SipHash-2-4 core is pinned by the published SipHash test vector (key
 * 00..0f, message 00..0e -> 0xa129ca6149be45e5; tests/test_bloom_oracle.py) and the four
 * initial-state constants are cross-checked (each k0/k1 pair decodes the same way); the
 * bbloom-specific choices (k0/k1, h/l split, bit order, JSON shape) are PARITY UNPINNED:
 * neither Go nor bbloom's source is available, and no reference test checks bloom bytes.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "sstref.h"

#define ROTL(x, b) (uint64_t)(((x) << (b)) | ((x) >> (64 - (b))))
#define SIPROUND                                                     \
  do {                                                               \
    v0 += v1; v1 = ROTL(v1, 13); v1 ^= v0; v0 = ROTL(v0, 32);        \
    v2 += v3; v3 = ROTL(v3, 16); v3 ^= v2;                           \
    v0 += v3; v3 = ROTL(v3, 21); v3 ^= v0;                           \
    v2 += v1; v1 = ROTL(v1, 17); v1 ^= v2; v2 = ROTL(v2, 32);        \
  } while (0)

/* SipHash-2-4 (Aumasson & Bernstein), 64-bit output, little-endian message words */
uint64_t sstref_siphash24(uint64_t k0, uint64_t k1, const uint8_t* p, size_t n) {
  uint64_t v0 = k0 ^ 0x736f6d6570736575ull, v1 = k1 ^ 0x646f72616e646f6dull;
  uint64_t v2 = k0 ^ 0x6c7967656e657261ull, v3 = k1 ^ 0x7465646279746573ull;
  uint64_t t = (uint64_t)n << 56;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t m = 0;
    for (int b = 0; b < 8; b++) m |= (uint64_t)p[i + b] << (8 * b);
    v3 ^= m;
    SIPROUND;
    SIPROUND;
    v0 ^= m;
  }
  for (size_t b = 0; i + b < n; b++) t |= (uint64_t)p[i + b] << (8 * b);
  v3 ^= t;
  SIPROUND;
  SIPROUND;
  v0 ^= t;
  v2 ^= 0xff;
  SIPROUND;
  SIPROUND;
  SIPROUND;
  SIPROUND;
  return v0 ^ v1 ^ v2 ^ v3;
}

/* bbloom.New(num_entries, wrongs) with wrongs < 1 (calcSizeByWrongPositives + getSize) */
void sstref_bloom_params(double num_entries, double wrongs, uint64_t* size_bits,
                         uint64_t* set_locs, uint32_t* exponent) {
  const double ln2 = 0.69314718056;
  const double size = -1 * num_entries * log(wrongs) / (ln2 * ln2);
  const double locs = ceil(ln2 * size / num_entries);
  uint64_t entries = (uint64_t)size;
  /* Go's uint64(NaN) on amd64 (0 entries: 0 / 0) is 1 << 63; C's conversion is undefined */
  *set_locs = isnan(locs) ? (1ull << 63) : (uint64_t)locs;
  if (entries < 512) entries = 512;
  uint64_t sz = 1;
  uint32_t e = 0;
  while (sz < entries) {
    sz <<= 1;
    e++;
  }
  *size_bits = sz;
  *exponent = e;
}

static void bloom_hash(const uint8_t* key, size_t n, uint32_t exponent, uint64_t* l, uint64_t* h) {
  const uint64_t hash = sstref_siphash24(0xdeadbeafull, 0xfaebdaedull, key, n);
  const uint32_t shift = 64 - exponent;
  *h = hash >> shift;
  *l = (hash << shift) >> shift;
}

void sstref_bloom_add(uint64_t* bitset, uint64_t size_bits, uint32_t exponent, uint64_t set_locs,
                      const uint8_t* key, size_t n) {
  uint64_t l, h;
  bloom_hash(key, n, exponent, &l, &h);
  for (uint64_t i = 0; i < set_locs; i++) {
    const uint64_t idx = (h + i * l) & (size_bits - 1);
    bitset[idx >> 6] |= 1ull << (idx & 63);
  }
}

int sstref_bloom_has(const uint64_t* bitset, uint64_t size_bits, uint32_t exponent,
                     uint64_t set_locs, const uint8_t* key, size_t n) {
  uint64_t l, h;
  bloom_hash(key, n, exponent, &l, &h);
  for (uint64_t i = 0; i < set_locs; i++) {
    const uint64_t idx = (h + i * l) & (size_bits - 1);
    if (!((bitset[idx >> 6] >> (idx & 63)) & 1)) return 0;
  }
  return 1;
}

/* JSONMarshal: returns the JSON length; writes it when cap suffices */
size_t sstref_bloom_json(const uint64_t* bitset, uint64_t size_bits, uint64_t set_locs,
                         uint8_t* out, size_t cap) {
  static const char b64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  const size_t nbytes = (size_t)(size_bits / 8);
  char tail[48];
  const int tl = snprintf(tail, sizeof tail, "\",\"SetLocs\":%llu}", (unsigned long long)set_locs);
  static const char head[] = "{\"FilterSet\":\"";
  const size_t hl = sizeof head - 1, bl = 4 * ((nbytes + 2) / 3);
  const size_t total = hl + bl + (size_t)tl;
  if (!out || cap < total) return total;
  memcpy(out, head, hl);
  const uint8_t* s = (const uint8_t*)bitset;  /* the words' bytes, little-endian */
  uint8_t* o = out + hl;
  for (size_t i = 0; i < nbytes; i += 3) {
    const uint32_t a = s[i], b = i + 1 < nbytes ? s[i + 1] : 0, c = i + 2 < nbytes ? s[i + 2] : 0;
    const uint32_t w = (a << 16) | (b << 8) | c;
    *o++ = (uint8_t)b64[(w >> 18) & 63];
    *o++ = (uint8_t)b64[(w >> 12) & 63];
    *o++ = i + 1 < nbytes ? (uint8_t)b64[(w >> 6) & 63] : '=';
    *o++ = i + 2 < nbytes ? (uint8_t)b64[w & 63] : '=';
  }
  memcpy(o, tail, (size_t)tl);
  return total;
}

/* Finish's bloom (builder.go:164-195) over a batch of keys WITH their 8-B ts (the Builder's
 * Add input): every key contributes ParseKey(key) = key[:len - 8].  bitset must hold
 * size_bits / 64 words for sstref_bloom_params(n, 0.01) and is cleared here.  Returns 0, or
 * -1 if a key is <= 8 B (y.go:98 AssertTruef: a panic in Go). */
int sstref_bloom_build(const uint8_t* keys, const uint32_t* key_end, size_t n, uint64_t* bitset,
                       uint64_t size_bits, uint32_t exponent, uint64_t set_locs) {
  memset(bitset, 0, (size_t)(size_bits / 8));
  for (size_t i = 0; i < n; i++) {
    const uint32_t s = i ? key_end[i - 1] : 0, e = key_end[i];
    if (e - s <= 8) return -1;
    sstref_bloom_add(bitset, size_bits, exponent, set_locs, keys + s, e - s - 8);
  }
  return 0;
}
