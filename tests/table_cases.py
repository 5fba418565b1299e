"""table/table_test.go, re-expressed over the host mirror (lsmdb_amd.table).

Every scenario takes an `env` that builds and opens tables:
  * CpuEnv: the oracle builds the bytes and decodes the blocks (host-logic tests, no GPU);
  * GpuEnv: lsmdb_amd.table.Builder (gfx950 encoder) + OpenTable (gfx950 decoder).
The expected values are the reference's own known answers (table_test.go line numbers cited).
"""
from __future__ import annotations

import os
import struct
import tempfile

from lsmdb_amd import bloom, table as T
from lsmdb_amd.y import MergeIterator, ValueStruct, key_with_ts, parse_key

NS = [101, 199, 200, 250, 9999, 10000]  # table_test.go:63 etc.


def key(prefix: str, i: int) -> str:
    return prefix + "%04d" % i  # table_test.go:15-17


def test_kvs(prefix: str, n: int):
    return [(key(prefix, i), "%d" % i) for i in range(n)]  # table_test.go:19-28


class CpuEnv:
    """Oracle-built tables, oracle-decoded blocks: exercises only the host iterator logic."""

    def __init__(self, oracle):
        self.o = oracle

    def build_bytes(self, kvs) -> bytes:
        kvs = sorted(kvs, key=lambda kv: kv[0])  # table_test.go:44-46
        keys = [key_with_ts(k.encode(), 0) for k, _ in kvs]
        vss = [ValueStruct(meta=ord("A"), value=v.encode()).encode() for _, v in kvs]
        body, _, _ = self.o.build(keys, vss, entries_per_block=100)
        kb, ke = self.o.columns(keys, vss)[:2]
        bs, bits, locs, _ = self.o.bloom_build(kb, ke)
        bd = self.o.bloom_json(bs, bits, locs)
        return body + bd + struct.pack(">I", len(bd))

    def open(self, raw: bytes, mode: int = T.MEMORY_MAP):
        return T.OpenTable(raw, mode, decoder=self.o.decode)


class GpuEnv:
    """lsmdb_amd Builder (GPU encode) + OpenTable (GPU decode), through real .sst files."""

    def __init__(self, codec):
        self.codec = codec
        self.dir = tempfile.mkdtemp(prefix="lsmgpu_")
        self.next_id = 1

    def build_bytes(self, kvs) -> bytes:
        kvs = sorted(kvs, key=lambda kv: kv[0])
        # the device bbloom tail (Builder's default is all-ones): byte-compared with the oracle
        b = T.Builder(bloom=T.BLOOM_BBLOOM, codec=self.codec)
        for k, v in kvs:
            b.Add(key_with_ts(k.encode(), 0), ValueStruct(meta=ord("A"), user_meta=0,
                                                          value=v.encode()))
        return b.Finish()

    def open(self, raw: bytes, mode: int = T.MEMORY_MAP):
        path = T.NewFilename(self.next_id, self.dir)
        self.next_id += 1
        with open(path, "wb") as f:
            f.write(raw)
        return T.OpenTable(path, mode, codec=self.codec)


def build_test_table(env, prefix, n, mode=T.MEMORY_MAP):
    return env.open(env.build_bytes(test_kvs(prefix, n)), mode)


def build_table(env, kvs, mode=T.MEMORY_MAP):
    return env.open(env.build_bytes(kvs), mode)


# ---------------------------------------------------------------- scenarios
def seek_to_first(env, n):  # table_test.go:62-78
    t = build_test_table(env, "key", n)
    it = t.NewIterator(False)
    it.seekToFirst()
    assert it.Valid()
    v = it.Value()
    assert v.value == b"0" and v.meta == ord("A")
    it.Close()
    t.DecrRef()


def seek_to_last(env, n):  # table_test.go:80-101
    t = build_test_table(env, "key", n)
    it = t.NewIterator(False)
    it.seekToLast()
    assert it.Valid()
    v = it.Value()
    assert v.value == b"%d" % (n - 1) and v.meta == ord("A")
    it.prev()
    assert it.Valid()
    v = it.Value()
    assert v.value == b"%d" % (n - 2) and v.meta == ord("A")
    it.Close()
    t.DecrRef()


def seek(env):  # table_test.go:103-136
    t = build_test_table(env, "k", 10000)
    it = t.NewIterator(False)
    data = [("abc", True, "k0000"), ("k0100", True, "k0100"), ("k0100b", True, "k0101"),
            ("k1234", True, "k1234"), ("k1234b", True, "k1235"), ("k9999", True, "k9999"),
            ("z", False, "")]
    for inp, valid, out in data:
        it.seek(key_with_ts(inp.encode(), 0))
        if not valid:
            assert not it.Valid()
            continue
        assert it.Valid()
        assert parse_key(it.Key()) == out.encode()
    it.Close()
    t.DecrRef()


def seek_for_prev(env):  # table_test.go:138-171
    t = build_test_table(env, "k", 10000)
    it = t.NewIterator(False)
    data = [("abc", False, ""), ("k0100", True, "k0100"), ("k0100b", True, "k0100"),
            ("k1234", True, "k1234"), ("k1234b", True, "k1234"), ("k9999", True, "k9999"),
            ("z", True, "k9999")]
    for inp, valid, out in data:
        it.seekForPrev(key_with_ts(inp.encode(), 0))
        if not valid:
            assert not it.Valid()
            continue
        assert it.Valid()
        assert parse_key(it.Key()) == out.encode()
    it.Close()
    t.DecrRef()


def iterate_from_start(env, n):  # table_test.go:173-198
    t = build_test_table(env, "key", n)
    ti = t.NewIterator(False)
    ti.reset()
    ti.seekToFirst()
    assert ti.Valid()
    count = 0
    while ti.Valid():
        v = ti.Value()
        assert v.value == b"%d" % count and v.meta == ord("A")
        count += 1
        ti.next()
    assert count == n
    ti.Close()
    t.DecrRef()


def iterate_from_end(env, n):  # table_test.go:200-224 (FileIO mode)
    t = build_test_table(env, "key", n, T.FILE_IO)
    ti = t.NewIterator(False)
    ti.reset()
    ti.seek(key_with_ts(b"zzzzzz", 0))
    assert not ti.Valid()
    for i in range(n - 1, -1, -1):
        ti.prev()
        assert ti.Valid()
        v = ti.Value()
        assert v.value == b"%d" % i and v.meta == ord("A")
    ti.prev()
    assert not ti.Valid()
    ti.Close()
    t.DecrRef()


def table_seek_iterate(env):  # table_test.go:226-251
    t = build_test_table(env, "key", 10000, T.FILE_IO)
    ti = t.NewIterator(False)
    kid = 1010
    ti.seek(key_with_ts(key("key", kid).encode(), 0))
    while ti.Valid():
        assert parse_key(ti.Key()) == key("key", kid).encode()
        kid += 1
        ti.next()
    assert kid == 10000
    ti.seek(key_with_ts(key("key", 99999).encode(), 0))
    assert not ti.Valid()
    ti.seek(key_with_ts(key("key", -1).encode(), 0))
    assert ti.Valid()
    assert parse_key(ti.Key()) == key("key", 0).encode()
    ti.Close()
    t.DecrRef()


def iterate_back_and_forth(env):  # table_test.go:253-292
    t = build_test_table(env, "key", 10000)
    sk = key_with_ts(key("key", 1010).encode(), 0)
    it = t.NewIterator(False)
    it.seek(sk)
    assert it.Valid()
    assert it.Key() == sk
    it.prev()
    it.prev()
    assert it.Valid()
    assert parse_key(it.Key()) == key("key", 1008).encode()
    it.next()
    it.next()
    assert it.Valid()
    assert parse_key(it.Key()) == key("key", 1010).encode()
    it.seek(key_with_ts(key("key", 2000).encode(), 0))
    assert it.Valid()
    assert parse_key(it.Key()) == key("key", 2000).encode()
    it.prev()
    assert it.Valid()
    assert parse_key(it.Key()) == key("key", 1999).encode()
    it.seekToFirst()
    assert parse_key(it.Key()) == key("key", 0).encode()
    it.Close()
    t.DecrRef()


def uni_iterator(env):  # table_test.go:294-323
    t = build_test_table(env, "key", 10000)
    for rev in (False, True):
        it = t.NewIterator(rev)
        count = 0
        it.Rewind()
        while it.Valid():
            v = it.Value()
            want = count if not rev else 10000 - 1 - count
            assert v.value == b"%d" % want and v.meta == ord("A")
            count += 1
            it.Next()
        assert count == 10000
        it.Close()
    t.DecrRef()


def concat_one_table(env):  # table_test.go:325-346
    t = build_table(env, [("k1", "a1"), ("k2", "a2")])
    it = T.NewConcatIterator([t], False)
    it.Rewind()
    assert it.Valid()
    assert parse_key(it.Key()) == b"k1"
    vs = it.Value()
    assert vs.value == b"a1" and vs.meta == ord("A")
    it.Close()
    t.DecrRef()


def concat_iterator(env):  # table_test.go:348-426
    tbl = build_test_table(env, "keya", 10000)
    tbl2 = build_test_table(env, "keyb", 10000, T.LOAD_TO_RAM)
    tbl3 = build_test_table(env, "keyc", 10000, T.LOAD_TO_RAM)
    it = T.NewConcatIterator([tbl, tbl2, tbl3], False)
    it.Rewind()
    assert it.Valid()
    count = 0
    while it.Valid():
        vs = it.Value()
        assert vs.value == b"%d" % (count % 10000) and vs.meta == ord("A")
        count += 1
        it.Next()
    assert count == 30000
    it.Seek(key_with_ts(b"a", 0))
    assert parse_key(it.Key()) == b"keya0000"
    assert it.Value().value == b"0"
    it.Seek(key_with_ts(b"keyb", 0))
    assert parse_key(it.Key()) == b"keyb0000"
    assert it.Value().value == b"0"
    it.Seek(key_with_ts(b"keyb9999b", 0))
    assert parse_key(it.Key()) == b"keyc0000"
    assert it.Value().value == b"0"
    it.Seek(key_with_ts(b"keyd", 0))
    assert not it.Valid()
    it.Close()

    it = T.NewConcatIterator([tbl, tbl2, tbl3], True)
    it.Rewind()
    assert it.Valid()
    count = 0
    while it.Valid():
        vs = it.Value()
        assert vs.value == b"%d" % (10000 - (count % 10000) - 1) and vs.meta == ord("A")
        count += 1
        it.Next()
    assert count == 30000
    it.Seek(key_with_ts(b"a", 0))
    assert not it.Valid()
    it.Seek(key_with_ts(b"keyb", 0))
    assert parse_key(it.Key()) == b"keya9999"
    assert it.Value().value == b"9999"
    it.Seek(key_with_ts(b"keyb9999b", 0))
    assert parse_key(it.Key()) == b"keyb9999"
    assert it.Value().value == b"9999"
    it.Seek(key_with_ts(b"keyd", 0))
    assert parse_key(it.Key()) == b"keyc9999"
    assert it.Value().value == b"9999"
    it.Close()
    for t in (tbl, tbl2, tbl3):
        t.DecrRef()


def _expect(it, pairs):
    for k, v in pairs:
        assert it.Valid()
        assert parse_key(it.Key()) == k
        vs = it.Value()
        assert vs.value == v and vs.meta == ord("A")
        it.Next()
    assert not it.Valid()


def merging_iterator(env, reversed_):  # table_test.go:428-506
    t1 = build_table(env, [("k1", "a1"), ("k2", "a2")], T.LOAD_TO_RAM)
    t2 = build_table(env, [("k1", "b1"), ("k2", "b2")], T.LOAD_TO_RAM)
    it1 = t1.NewIterator(reversed_)
    it2 = T.NewConcatIterator([t2], reversed_)
    it = MergeIterator([it1, it2], reversed_)
    it.Rewind()
    want = [(b"k1", b"a1"), (b"k2", b"a2")]
    _expect(it, want[::-1] if reversed_ else want)
    it.Close()
    t1.DecrRef()
    t2.DecrRef()


def merging_take(env, which):  # table_test.go:508-586 (one side is an EMPTY table)
    full = [("k1", "a1"), ("k2", "a2")]
    ka, kb = (full, []) if which == 1 else ([], full)
    t1 = build_table(env, ka, T.LOAD_TO_RAM)
    t2 = build_table(env, kb, T.LOAD_TO_RAM)
    it = MergeIterator([T.NewConcatIterator([t1], False), T.NewConcatIterator([t2], False)], False)
    it.Rewind()
    _expect(it, [(b"k1", b"a1"), (b"k2", b"a2")])
    it.Close()
    t1.DecrRef()
    t2.DecrRef()


def file_lifecycle(env):
    """table.go:53-71 DecrRef at ref 0 removes the file (GpuEnv only opens real files)."""
    t = build_test_table(env, "key", 150)
    name = t.Filename()
    it = t.NewIterator(False)
    it.Close()
    t.DecrRef()
    if name:
        assert not os.path.exists(name)
