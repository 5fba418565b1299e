"""The SST bloom tail's host-side pieces: bbloom.New's sizing and JSONUnmarshal's parse.

The reference writes `bbloom.New(float64(keyCount), 0.01).JSONMarshal()` after the index and
reads it back with `bbloom.JSONUnmarshal` (table/builder.go:164,189-195, table/table.go:180-186;
github.com/AndreasBriese/bbloom v0.0.0-20190825152654-46b345b51c96, not vendored).  The filter
itself -- SipHash-2-4 of every ParseKey(key), setLocs bits per key -- is built and probed on the
device (csrc/bloom.hip through Codec.bloom_tail_host / Codec.bloom_has_host); DESIGN.md states
the restated algorithm and its pinning (SipHash core pinned by the published vectors, the
bbloom-specific bytes "parity unpinned").
"""
from __future__ import annotations

import base64
import json
import math

import numpy as np

LN2 = 0.69314718056  # the constant bbloom uses


def bbloom_params(num_entries: float, wrongs: float = 0.01) -> tuple[int, int]:
    """(size in bits, setLocs) of bbloom.New(num_entries, wrongs)."""
    if num_entries > 0:
        size_f = -1 * num_entries * math.log(wrongs) / (LN2 ** 2)
        locs = int(math.ceil(LN2 * size_f / num_entries))
    else:  # 0/0 = NaN in Go; uint64(NaN) is 1<<63 on amd64
        size_f = 0.0
        locs = 1 << 63
    entries = int(size_f)
    if entries < 512:
        entries = 512
    size = 1
    while size < entries:
        size <<= 1
    return size, locs


_M64 = (1 << 64) - 1
K0, K1 = 0xDEADBEAF, 0xFAEBDAED  # bbloom's SipHash key (DESIGN.md "Bloom tail")


def _rotl(x: int, b: int) -> int:
    return ((x << b) | (x >> (64 - b))) & _M64


def siphash24(k0: int, k1: int, data: bytes) -> int:
    """SipHash-2-4, 64-bit output (the hash bbloom.sipHash restates; the device build uses
    the same function, csrc/bloom.hip).  For one-key host probes only."""
    v0, v1 = k0 ^ 0x736F6D6570736575, k1 ^ 0x646F72616E646F6D
    v2, v3 = k0 ^ 0x6C7967656E657261, k1 ^ 0x7465646279746573

    def rnd(v0, v1, v2, v3):
        v0 = (v0 + v1) & _M64; v1 = _rotl(v1, 13) ^ v0; v0 = _rotl(v0, 32)
        v2 = (v2 + v3) & _M64; v3 = _rotl(v3, 16) ^ v2
        v0 = (v0 + v3) & _M64; v3 = _rotl(v3, 21) ^ v0
        v2 = (v2 + v1) & _M64; v1 = _rotl(v1, 17) ^ v2; v2 = _rotl(v2, 32)
        return v0, v1, v2, v3

    n = len(data)
    full = n - n % 8
    for i in range(0, full, 8):
        m = int.from_bytes(data[i: i + 8], "little")
        v3 ^= m
        v0, v1, v2, v3 = rnd(*rnd(v0, v1, v2, v3))
        v0 ^= m
    t = ((n & 0xFF) << 56) | int.from_bytes(data[full:], "little")
    v3 ^= t
    v0, v1, v2, v3 = rnd(*rnd(v0, v1, v2, v3))
    v0 ^= t
    v2 ^= 0xFF
    for _ in range(4):
        v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
    return v0 ^ v1 ^ v2 ^ v3


def has(bitset: np.ndarray, locs: int, key: bytes) -> bool:
    """bf.Has(key) (table.go:301) for ONE key on the host: Get's latency-bound probe needs no
    device round trip.  Batches go to the device (Codec.bloom_has_device)."""
    bits = int(bitset.size) * 64
    shift = 64 - (bits.bit_length() - 1)
    h64 = siphash24(K0, K1, bytes(key))
    h = h64 >> shift
    l = ((h64 << shift) & _M64) >> shift
    mask = bits - 1
    for i in range(min(locs, bits)):  # setLocs > bits only for the empty table's NaN sizing
        idx = (h + i * l) & mask
        if not (int(bitset[idx >> 6]) >> (idx & 63)) & 1:
            return False
    return True


def all_ones_json(key_count: int) -> bytes:
    """A bbloom-shaped tail whose every bit is set: Has() is true for every key, so a Go
    reader's DoesNotHave never skips a table.  The conservative tail for files a Go reader
    opens while the restated bbloom bytes are parity unpinned."""
    bits, locs = bbloom_params(float(key_count))
    fs = base64.b64encode(b"\xff" * (bits // 8)).decode()
    return json.dumps({"FilterSet": fs, "SetLocs": locs}, separators=(",", ":")).encode()


def parse(bloom_json: bytes) -> tuple[np.ndarray, int]:
    """bbloom.JSONUnmarshal (table/table.go:186): (filter as little-endian u64 words, setLocs).
    Raises ValueError on a tail Go could not load either."""
    try:
        doc = json.loads(bloom_json)
        fs = base64.b64decode(doc["FilterSet"], validate=True)
        locs = int(doc["SetLocs"])
    except (ValueError, KeyError, TypeError) as e:
        raise ValueError(f"bloom tail: {e}") from e
    if len(fs) < 8 or len(fs) % 8 or (len(fs) & (len(fs) - 1)):
        raise ValueError("bloom tail: FilterSet is not a power-of-two number of u64 words")
    return np.frombuffer(fs, dtype="<u8").copy(), locs
