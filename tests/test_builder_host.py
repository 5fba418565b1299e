"""Builder's host-side bookkeeping (Empty / ReachedCapacity after every Add) against the
oracle Builder -- the compaction split rule of levels.go:265-270.  No GPU."""
import ctypes

import numpy as np
import pytest

from lsmdb_amd import table as T
from lsmdb_amd.y import AssertionFailed, ValueStruct, key_with_ts


@pytest.mark.parametrize("epb,bb", [(100, 0), (31, 0), (0, 4096), (100, 4096)])
def test_reached_capacity_tracks_oracle(oracle, epb, bb):
    L = oracle.lib()
    ob = L.sstref_builder_new(epb, bb)
    b = T.Builder(entries_per_block=epb, block_bytes=bb)
    rng = np.random.default_rng(epb + bb)
    assert b.Empty() and L.sstref_builder_empty(ob) == 1
    for i in range(3000):
        k = key_with_ts(b"k%09d" % i, 0)
        v = ValueStruct(meta=0x41, expires_at=int(rng.integers(0, 2 ** 20)) if i % 7 == 0 else 0,
                        value=bytes(rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8)))
        b.Add(k, v)
        enc = np.frombuffer(v.encode(), np.uint8)
        kb = np.frombuffer(k, np.uint8)
        L.sstref_builder_add(ob, kb.ctypes.data, len(k), enc.ctypes.data, enc.size)
        for cap in (1 << 10, 1 << 16, 1 << 20, (1 << 20) + 12345):
            assert b.ReachedCapacity(cap) == bool(L.sstref_builder_reached_capacity(ob, cap))
        assert not b.Empty()
    L.sstref_builder_free(ob)
    _ = ctypes


def test_add_rejects_short_keys():
    b = T.Builder()
    with pytest.raises(AssertionFailed):
        b.Add(b"12345678", ValueStruct())
    with pytest.raises(ValueError):
        b.Add(b"k" * 9, ValueStruct(value=b"x" * 70000))
