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
