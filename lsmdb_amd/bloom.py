"""bbloom-shaped bloom tail for SSTs built by lsmdb_amd.Builder.

The reference writes `bbloom.New(float64(keyCount), 0.01).JSONMarshal()` after the index
(table/builder.go:164,190-195; AndreasBriese/bbloom v0.0.0-20190825152654-46b345b51c96, not
vendored, source absent).  Its hash bits are PARITY UNPINNED here.  To stay loadable and safe
for a Go reader we emit the same JSON shape and filter size with EVERY bit set: Go's
bbloom.JSONUnmarshal accepts it and `Has` is always true, so `Table.DoesNotHave` never
excludes a present key (it only loses the filtering).  An exact bbloom restatement is SURVEY
section 8(f) rank 3.
"""
from __future__ import annotations

import base64
import json
import math

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


def bloom_tail(key_count: int) -> bytes:
    """JSON bytes of an all-ones bbloom filter sized like bbloom.New(key_count, 0.01)."""
    size, locs = bbloom_params(float(key_count))
    filter_set = b"\xff" * (size // 8)
    doc = {"FilterSet": base64.b64encode(filter_set).decode(), "SetLocs": locs}
    return json.dumps(doc, separators=(",", ":")).encode()


def may_contain(bloom_json: bytes, key: bytes) -> bool:
    """Table.DoesNotHave's complement.  Exact for all-ones filters; any other filter is
    answered conservatively (True) because the bbloom hash is not restated (unpinned)."""
    try:
        doc = json.loads(bloom_json)
        fs = base64.b64decode(doc.get("FilterSet", ""))
    except Exception:
        return True
    if fs and all(b == 0xFF for b in fs):
        return True
    return True
