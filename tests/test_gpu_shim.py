"""The cgo shim's exact call sequences, replayed through ctypes on the GPU:

* decodeTable: parse_index size query -> allocate -> parse_index; newDecodedBatch with upper
  bounds -> decode_blocks (-> the reported needs and a second decode_blocks only on
  LSMGPU_ERR_CAPACITY); the table's bytes pageable (an mmap / Go heap buffer: staged by the
  library) or read into lsmgpu_host_alloc memory (loadToHost: direct DMA).  Checked against the oracle's decode
  of the same blocks (table/iterator.go:93-135).
* finishBlocks: encode_blocks size query (out == NULL) -> allocate out_len -> encode_blocks.
  Checked byte for byte against the oracle Builder (table/builder.go:84-198).
* compactBuildTables: lsmgpu_compact_tables -> lsmgpu_compact_result, checked against the oracle
  MergeIterator order and the oracle Builder driven like the Go loop (levels.go:239-298).
"""
import ctypes
from ctypes import byref, c_uint64

import numpy as np
import pytest

import kat_defs as K
import open_cases as C
from lsmdb_amd import _lib, workload
from lsmdb_amd.codec import _ptr

pytestmark = pytest.mark.gpu

MAT_VIEW = _lib.MODE_MATERIALIZE | _lib.MODE_VIEW


def shim_decode_table(ctx, sst: bytes, pin: bool = False):
    """decodeTable step by step: tail parse, upper-bound buffers (entries <=
    data/10, key and value bytes <= data), one decode; on LSMGPU_ERR_CAPACITY (prefix-compressed
    keys that expand) the reported needs are allocated and the decode repeated.  pin: the
    table's bytes in lsmgpu_host_alloc memory (loadToHost, table.go:117-123,329-338 under
    LoadToRAM), else pageable.  Returns the host SoA, the final call's needs, the block list and
    the number of decode calls made."""
    L = _lib.lib()
    hp = ctypes.c_void_p()
    if pin:  # loadToHost
        assert L.lsmgpu_host_alloc(ctx, len(sst) + 1, byref(hp)) == _lib.OK
        base = np.frombuffer((ctypes.c_uint8 * (len(sst) + 1)).from_address(hp.value), np.uint8)
        base[:len(sst)] = np.frombuffer(sst, np.uint8)
    else:
        base = np.frombuffer(sst + b"\0", np.uint8).copy()
    nblk, bo, bl = c_uint64(0), c_uint64(0), c_uint64(0)
    rc = L.lsmgpu_parse_index(_ptr(base), len(sst), None, None, 0, byref(nblk), byref(bo), byref(bl))
    assert rc in (_lib.OK, _lib.ERR_CAPACITY)
    off = np.zeros(max(nblk.value, 1), np.uint32)
    ln = np.zeros(max(nblk.value, 1), np.uint32)
    assert L.lsmgpu_parse_index(_ptr(base), len(sst), _ptr(off), _ptr(ln), nblk.value, byref(nblk),
                                byref(bo), byref(bl)) == _lib.OK
    n = nblk.value
    data_end = int(off[n - 1]) + int(ln[n - 1]) if n else 0

    def batch(entries, kbytes, vbytes):  # newDecodedBatch
        arrs = dict(kd=np.zeros(max(kbytes, 1), np.uint8), vd=np.zeros(max(vbytes, 1), np.uint8),
                    ke=np.zeros(max(entries, 1), np.uint32), ve=np.zeros(max(entries, 1), np.uint32),
                    vw=np.zeros(max(entries, 1), np.uint64), bf=np.zeros(n + 1, np.uint32),
                    bs=np.zeros(max(n, 1), np.int32))
        d = _lib.LsmgpuDecoded()
        d.key_data, d.key_cap, d.key_end = _ptr(arrs["kd"]), kbytes, _ptr(arrs["ke"])
        d.val_data, d.val_cap, d.val_end = _ptr(arrs["vd"]), vbytes, _ptr(arrs["ve"])
        d.view, d.ent_cap = _ptr(arrs["vw"]), entries
        d.blk_first, d.blk_status = _ptr(arrs["bf"]), _ptr(arrs["bs"])
        return d, arrs

    calls = 1
    d, arrs = batch(data_end // 10 + 1, data_end, data_end)
    rc = L.lsmgpu_decode_blocks(ctx, _ptr(base), data_end, 0, _ptr(off), _ptr(ln), n, MAT_VIEW, byref(d))
    if rc == _lib.ERR_CAPACITY:
        calls += 1
        d, arrs = batch(d.n_entries, d.key_bytes, d.val_bytes)
        rc = L.lsmgpu_decode_blocks(ctx, _ptr(base), data_end, 0, _ptr(off), _ptr(ln), n, MAT_VIEW,
                                    byref(d))
    if pin:  # freeHost (Table.DecrRef)
        del base
        assert L.lsmgpu_host_free(ctx, hp) == _lib.OK
    assert rc == _lib.OK
    m = d.n_entries
    need = (d.n_entries, d.key_bytes, d.val_bytes, d.first_bad_block, d.n_bad_blocks)
    got = dict(n=m, kd=arrs["kd"][: d.key_bytes].tobytes(), vd=arrs["vd"][: d.val_bytes].tobytes(),
               ke=arrs["ke"][:m], ve=arrs["ve"][:m], view=arrs["vw"][:m], bf=arrs["bf"],
               bs=arrs["bs"][:n], fbb=d.first_bad_block, nbad=d.n_bad_blocks, calls=calls)
    return got, need, off[:n], ln[:n]


def _check_against_oracle(oracle, sst, got, need, off, ln):
    o = oracle.decode(sst, off, ln)
    assert need == (o.n_entries, o.key_data.size, o.val_data.size, o.first_bad_block,
                    o.n_bad_blocks)
    assert got["n"] == o.n_entries
    assert got["kd"] == o.key_data.tobytes() and got["vd"] == o.val_data.tobytes()
    assert np.array_equal(got["ke"], o.key_end) and np.array_equal(got["ve"], o.val_end)
    assert np.array_equal(got["view"], o.view)
    assert np.array_equal(got["bf"], o.blk_first) and np.array_equal(got["bs"], o.blk_status)
    assert got["fbb"] == o.first_bad_block and got["nbad"] == o.n_bad_blocks


@pytest.mark.parametrize("cfg,n", [(1, 10000), (2, 40000), (3, 3000), (5, 20000), (1, 0)])
def test_shim_decode_table(codec, oracle, cfg, n):
    if n:
        c = workload.config_columns(cfg, n)
        body, _, _ = oracle.build_cols(c.keys, c.key_end, c.vs, c.vs_end, c.entries_per_block,
                                       c.block_bytes)
    else:
        body, _, _ = oracle.build([], [], 100)
    sst = body + C.TAIL
    for pin in (False, True):
        got, need, off, ln = shim_decode_table(codec._ctx, sst, pin=pin)
        _check_against_oracle(oracle, sst, got, need, off, ln)
        assert got["calls"] == 1  # one copy of the table: no size-query pass


def test_shim_decode_table_pipelined(codec, oracle, monkeypatch):
    """decodeTable on a table larger than several pipeline chunks (LSMGPU_HOST_CHUNK = 1 MiB),
    pinned and not."""
    monkeypatch.setenv("LSMGPU_HOST_CHUNK", str(1 << 20))
    c = workload.config_columns(2, 120000)
    body, _, _ = oracle.build_cols(c.keys, c.key_end, c.vs, c.vs_end, c.entries_per_block,
                                   c.block_bytes)
    sst = body + C.TAIL
    for pin in (False, True):
        got, need, off, ln = shim_decode_table(codec._ctx, sst, pin=pin)
        _check_against_oracle(oracle, sst, got, need, off, ln)
        assert got["calls"] == 1


def test_shim_decode_expanding_and_bad_blocks(codec, oracle):
    """Prefix-compressed keys that expand past the input's size: the first call returns
    LSMGPU_ERR_CAPACITY with the exact needs (and the bad-block counts), the second succeeds."""
    import struct
    big = bytearray()  # 4,000 entries of plen 2,900: ~11.6 MB of keys from a 20 KB block
    prev = 0xFFFFFFFF
    for e in range(4000):
        pos = len(big)
        plen, diff = (0, bytes(range(256)) * 12) if e == 0 else (2900, b"x")
        big += struct.pack(">HHHI", plen, len(diff), 1, prev) + diff + b"v"
        prev = pos
    big += struct.pack(">HHHI", 0, 0, 3, prev) + b"\0\0\0"
    blocks = [K.PLEN_BLOCK] * 40 + [bytes(big)] + [kat[1] for kat in K.DECODE_KATS]
    data = b"".join(blocks)
    ends = np.cumsum([len(b) for b in blocks]).astype(np.uint32)
    sst = C.with_tail(data, ends)
    got, need, off, ln = shim_decode_table(codec._ctx, sst)
    _check_against_oracle(oracle, sst, got, need, off, ln)
    assert need[3] >= 0 and need[4] > 0 and got["calls"] == 2


@pytest.mark.parametrize("cfg,n", [(1, 10000), (2, 20000), (3, 2000), (5, 10000), (1, 0)])
def test_shim_finish_blocks(codec, oracle, cfg, n):
    L = _lib.lib()
    if n:
        c = workload.config_columns(cfg, n)
        kb, ke, vb, ve = c.keys, c.key_end, c.vs, c.vs_end
        epb, bb = c.entries_per_block, c.block_bytes
    else:
        kb, vb = np.zeros(1, np.uint8), np.zeros(1, np.uint8)
        ke = ve = np.zeros(0, np.uint32)
        epb, bb = 100, 0
    out_len, data_len, nr = c_uint64(0), c_uint64(0), c_uint64(0)
    # step 1: the size query (out == NULL)
    assert L.lsmgpu_encode_blocks(codec._ctx, None, _ptr(ke), None, _ptr(ve), ke.size, 0, epb, bb,
                                  None, 0, byref(out_len), byref(data_len), None, 0,
                                  byref(nr)) == _lib.OK
    out = np.zeros(max(out_len.value, 1), np.uint8)
    rs = np.zeros(max(nr.value, 1), np.uint32)
    assert L.lsmgpu_encode_blocks(codec._ctx, _ptr(kb), _ptr(ke), _ptr(vb), _ptr(ve), ke.size, 0,
                                  epb, bb, _ptr(out), out_len.value, byref(out_len),
                                  byref(data_len), _ptr(rs), rs.size, byref(nr)) == _lib.OK
    if n:
        ref, ref_dl, ref_rs = oracle.build_cols(kb, ke, vb, ve, epb, bb)
    else:
        ref, ref_dl, ref_rs = oracle.build([], [], 100)
    assert out[: out_len.value].tobytes() == ref and data_len.value == ref_dl
    assert np.array_equal(rs[: nr.value], ref_rs)


def _tables(oracle, nt, per, seed, space=4):
    """nt overlapping tables of one key space (updates across tables), oracle-built."""
    out = []
    c = workload.config_columns(space, per * 2, seed_offset=0)
    for s in range(nt):
        idx = np.nonzero(np.random.default_rng(seed + s).random(per * 2) < 0.5)[0]
        keys = [bytes(c.keys[(c.key_end[i - 1] if i else 0): c.key_end[i]]) for i in idx]
        vss = [bytes(c.vs[(c.vs_end[i - 1] if i else 0): c.vs_end[i]]) for i in idx]
        vss = [v[:1] + bytes([s]) + v[2:] for v in vss]  # UserMeta = table: which one won a tie
        out.append(oracle.build(keys, vss, entries_per_block=100)[0] + C.TAIL)
    return out


def _oracle_compaction(oracle, ssts, run_first, cap, bloom):
    """MergeIterator over the runs (each run's tables chained, like ConcatIterator), then the Go
    loop `if ReachedCapacity(cap) { break }; Add` per output table (levels.go:259-283)."""
    from test_gpu_compaction import _oracle_tables
    kd, ke, vd, ve, rf = b"", [], b"", [], [0]
    for r in range(len(run_first) - 1):
        for t in range(run_first[r], run_first[r + 1]):
            off, ln, _, _ = oracle.parse_index(ssts[t])
            d = oracle.decode(ssts[t], off, ln)
            ke.extend((d.key_end.astype(np.int64) + len(kd)).tolist())
            ve.extend((d.val_end.astype(np.int64) + len(vd)).tolist())
            kd += d.key_data.tobytes()
            vd += d.val_data.tobytes()
        rf.append(len(ke))
    ke, ve = np.array(ke, np.uint32), np.array(ve, np.uint32)
    src = oracle.merge(kd, ke, np.array(rf, np.uint32))
    ks = [kd[(ke[i - 1] if i else 0): ke[i]] for i in src]
    vs = [vd[(ve[i - 1] if i else 0): ve[i]] for i in src]
    return _oracle_tables(oracle, ks, vs, cap, bloom)


@pytest.mark.parametrize("bloom", [False, True])
@pytest.mark.parametrize("shape", ["l0", "ln"])
def test_shim_compact_tables(codec, oracle, shape, bloom):
    """compactBuildTables' data path in one call: L0 (every top table its own iterator, then
    the bottom tables as one ConcatIterator run) and Ln (one top table + the bottom run)."""
    if shape == "l0":
        tops = _tables(oracle, 3, 8000, 70)
        bots = _bottom_run(oracle, 4, 6000)
        ssts = tops + bots
        run_first = [0, 1, 2, 3, len(ssts)]
    else:
        tops = _tables(oracle, 1, 20000, 90)
        bots = _bottom_run(oracle, 3, 10000)
        ssts = tops + bots
        run_first = [0, 1, len(ssts)]
    cap = 1 << 20
    got = codec.compact_host(ssts, run_first, cap, bloom=bloom)
    want = _oracle_compaction(oracle, ssts, run_first, cap, bloom)
    assert len(got) == len(want) >= 2
    for k, (g, w) in enumerate(zip(got, want)):
        assert g == w, f"table {k}"


def _bottom_run(oracle, nt, per):
    """nt tables with disjoint, increasing key ranges (a level >= 1: ConcatIterator input)."""
    c = workload.config_columns(4, nt * per, seed_offset=1)
    out = []
    for t in range(nt):
        keys = [bytes(c.keys[(c.key_end[i - 1] if i else 0): c.key_end[i]])
                for i in range(t * per, (t + 1) * per)]
        vss = [bytes(c.vs[(c.vs_end[i - 1] if i else 0): c.vs_end[i]])
               for i in range(t * per, (t + 1) * per)]
        out.append(oracle.build(keys, vss, entries_per_block=100)[0] + C.TAIL)
    return out


def _go_compaction(oracle, ssts, run_first, cap):
    """compactBuildTables (levels.go:239-283) run by the host mirror of the reference's own
    iterator state machines (lsmdb_amd/table.py: OpenTable, Iterator, ConcatIterator;
    lsmdb_amd/y.py: MergeIterator) over the ORACLE decode, then the oracle Builder loop.  Every
    run is a ConcatIterator (one table behaves as its Iterator).  Returns None where Go panics
    or log.Fatal()s (AssertTrue, a slice out of range, Decode of a nil value)."""
    from lsmdb_amd import table as T, y
    from test_gpu_compaction import _oracle_tables
    try:
        tables = [T.OpenTable(s, decoder=oracle.decode) for s in ssts]
        iters = [T.ConcatIterator(tables[a:b]) for a, b in zip(run_first[:-1], run_first[1:])]
        it = y.MergeIterator(iters)
        it.Rewind()
        ks, vs = [], []
        while it.Valid():
            k, v = it.Key(), it.Value()  # Value() of a nil block value panics (Decode)
            ks.append(bytes(k))
            vs.append(v.encode())
            it.Next()
    except (AssertionError, IndexError, TypeError, T.TableError):
        return None
    return _oracle_tables(oracle, ks, vs, cap, False)


def _table_of(blocks):
    data = b"".join(blocks)
    return C.with_tail(data, np.cumsum([len(b) for b in blocks]).astype(np.uint32))


def _good_blocks(oracle, lo, hi, step=1):
    """Blocks of one Builder table over workload keys [lo, hi) (100 entries per block)."""
    c = workload.config_columns(4, hi, seed_offset=3)
    keys = [bytes(c.keys[(c.key_end[i - 1] if i else 0): c.key_end[i]]) for i in range(lo, hi, step)]
    vss = [bytes(c.vs[(c.vs_end[i - 1] if i else 0): c.vs_end[i]]) for i in range(lo, hi, step)]
    sst = oracle.build(keys, vss, entries_per_block=100)[0] + C.TAIL
    off, ln, _, _ = oracle.parse_index(sst)
    return [sst[int(o): int(o) + int(n)] for o, n in zip(off, ln)]


def _overflow_first(block: bytes) -> bytes:
    """The block with its first entry's vlen raised past the block end (a value overflow at
    entry 0: Go's blockIterator stops with "Value exceeded size of block")."""
    b = bytearray(block)
    b[4:6] = (0xFFF0).to_bytes(2, "big")
    return bytes(b)


def test_shim_compact_corrupt_first_entries(codec, oracle):
    """Go's iterator reachability on corrupt inputs: a table whose first block
    yields nothing is dropped (seekToFirst invalid); as the first table of a ConcatIterator run
    it drops the whole run; a later block that yields nothing is a Go crash (ERR_CORRUPT).
    Expected values come from the host mirror of the Go iterators over the oracle decode."""
    good = lambda lo, hi: _table_of(_good_blocks(oracle, lo, hi))
    tb = _good_blocks(oracle, 0, 400, 2)          # 2 blocks of 100 entries (even keys)
    bad_first = _table_of([_overflow_first(tb[0]), tb[1]])      # block 0 yields nothing
    bad_later = _table_of([tb[0], _overflow_first(tb[1])])      # block 1 yields nothing
    empty_tbl = oracle.build([], [], 100)[0] + C.TAIL           # one terminator-only block
    no_blocks = b"\0\0\0\0" + C.TAIL                          # restarts count 0: no blocks
    cases = {
        # L0 shape: three top tables, one bottom run of two disjoint tables
        "top_first_overflow": ([bad_first, good(1, 300), good(300, 600), good(600, 900)], [0, 1, 2, 4]),
        "bottom_first_overflow": ([good(1, 300), bad_first, good(600, 900)], [0, 1, 3]),
        "bottom_second_overflow": ([good(1, 300), good(0, 200), bad_first], [0, 1, 3]),
        "bottom_first_empty": ([good(1, 300), empty_tbl, good(600, 900)], [0, 1, 3]),
        "bottom_first_no_blocks": ([good(1, 300), no_blocks, good(600, 900)], [0, 1, 3]),
        "top_empty": ([empty_tbl, good(0, 300)], [0, 1, 2]),
        "later_block_overflow": ([bad_later, good(1, 300)], [0, 1, 2]),
        "later_block_overflow_in_dropped_run": ([good(1, 300), empty_tbl, bad_later], [0, 1, 3]),
    }
    for name, (ssts, rf) in cases.items():
        want = _go_compaction(oracle, ssts, rf, 1 << 20)
        if want is None:
            with pytest.raises(_lib.LsmgpuError) as e:
                codec.compact_host(ssts, rf, 1 << 20)
            assert e.value.code == _lib.ERR_CORRUPT, name
        else:
            got = codec.compact_host(ssts, rf, 1 << 20)
            assert got == want, name
    # the mirror agrees with the analysis for the cases that define the rules
    assert _go_compaction(oracle, *cases["later_block_overflow"], 1 << 20) is None
    assert _go_compaction(oracle, *cases["bottom_first_overflow"], 1 << 20) is not None


def test_shim_compact_empty_and_corrupt(codec, oracle):
    L = _lib.lib()
    empty = oracle.build([], [], 100)[0] + C.TAIL
    assert codec.compact_host([empty, empty], [0, 1, 2], 1 << 20) == []
    # a block whose first header has plen != 0 is a Go log.Fatal: corrupt input
    bad = C.with_tail(K.hdr(3, 10, 5, K.NOPREV) + K.K1 + K.V1, np.array([25], np.uint32))
    with pytest.raises(_lib.LsmgpuError) as e:
        codec.compact_host([bad], [0, 1], 1 << 20)
    assert e.value.code == _lib.ERR_CORRUPT
    # a value overflow: the entries before it survive (Go's iterator skips the block's rest)
    vo = C.with_tail(K.DECODE_KATS[5][1], np.array([len(K.DECODE_KATS[5][1])], np.uint32))
    got = codec.compact_host([vo], [0, 1], 1 << 20)
    want = _oracle_compaction(oracle, [vo], [0, 1], 1 << 20, False)
    assert got == want and len(got) == 1
    _ = (L, ctypes)
