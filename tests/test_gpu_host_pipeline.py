"""lsmgpu_decode_blocks on host memory (data_on_device = 0), the path a cgo caller with an mmap'd
.sst takes (table/table.go:88-144,153-166): blocks sorted by offset are decoded as a pipeline of
chunks (copy-in / decode / copy-out on three streams, api.hip decode_host_pipelined).  Chunk
sizes of 1-3 MiB (LSMGPU_HOST_CHUNK) cut the test inputs into many chunks, so the per-chunk
bases, the block-index and status arrays across chunk borders, the first bad block and the
capacity rules are all exercised; every output is checked against the oracle.  Unsorted block
lists and chunks whose prefix-compressed keys outgrow their device slot take the one-shot path."""
import ctypes
from ctypes import byref

import numpy as np
import pytest

import kat_defs as K
from lsmdb_amd import _lib
from lsmdb_amd.codec import MODE_MATERIALIZE, MODE_VIEW, _ptr
from test_gpu_parity import _assert_same, _cols, _random_cols, _sst_blocks

pytestmark = pytest.mark.gpu


def _mixed(oracle):
    c2 = _cols(2, 50000, seed=61)
    c5 = _cols(5, 8000, seed=62)
    c4 = _cols(4, 20000, seed=63)
    parts = [oracle.build_cols(c2.keys, c2.key_end, c2.vs, c2.vs_end, 0, 4096)[0],
             oracle.build_cols(c5.keys, c5.key_end, c5.vs, c5.vs_end, 0, c5.block_bytes)[0],
             oracle.build_cols(*_random_cols(20000, 64), 0, 4096)[0],
             oracle.build_cols(c4.keys, c4.key_end, c4.vs, c4.vs_end, 100, 0)[0]]
    data, off, ln = _sst_blocks(oracle, parts)
    kd = bytearray(data)
    offs, lens = [int(x) for x in off], [int(x) for x in ln]
    for i, (_n, block, _e, _s) in enumerate(K.DECODE_KATS * 2):  # error statuses, plen > 0
        kd += b"\xab" * (i % 13)
        offs.append(len(kd))
        lens.append(len(block))
        kd += block
    return bytes(kd), np.array(offs, np.uint32), np.array(lens, np.uint32)


@pytest.fixture(scope="module")
def mixed(oracle):
    """The mixed input, its oracle decode, and a page-aligned copy of it registered once for the
    module (lsmgpu_host_register, as the shim pins an mmap): registering one buffer per test
    re-registers whatever pages the allocator hands back, a pattern the shim never has."""
    from lsmdb_amd.codec import Codec
    data, off, ln = _mixed(oracle)
    ref = oracle.decode(data, off, ln)
    page = 4096
    raw = np.zeros(len(data) + 2 * page, np.uint8)
    a = (-raw.ctypes.data) % page
    pinned = raw[a:a + len(data)]
    pinned[:] = np.frombuffer(data, np.uint8)
    reg = Codec(0)
    reg.host_register(pinned)
    yield data, off, ln, ref, pinned
    reg.host_unregister(pinned)
    reg.close()
    del raw


@pytest.mark.parametrize("chunk", ["1048576", "3000000"])
@pytest.mark.parametrize("mode", ["both", "view", "materialize"])
def test_host_pipeline_vs_oracle(codec, mixed, monkeypatch, chunk, mode):
    monkeypatch.setenv("LSMGPU_HOST_CHUNK", chunk)
    data, off, ln, ref, pinned_buf = mixed
    m = {"both": MODE_MATERIALIZE | MODE_VIEW, "view": MODE_VIEW, "materialize": MODE_MATERIALIZE}[mode]
    for pinned in (False, True):
        buf = pinned_buf if pinned else np.frombuffer(data, np.uint8).copy()
        g = codec.decode_host(buf, off, ln, mode=m)
        if m == MODE_VIEW:
            assert g.n_entries == ref.n_entries and np.array_equal(g.view, ref.view)
            assert np.array_equal(g.blk_first, ref.blk_first)
            assert np.array_equal(g.blk_status, ref.blk_status)
            assert g.first_bad_block == ref.first_bad_block and g.n_bad_blocks == ref.n_bad_blocks
        else:
            if m == MODE_MATERIALIZE:
                g.view = None
            _assert_same(g, ref, f"chunk={chunk} pinned={pinned}")


def _decode_raw(codec, data, off, ln, mode, key_cap, val_cap, ent_cap):
    buf = np.frombuffer(data, np.uint8)
    nblk = off.size
    kd, vd = np.zeros(max(key_cap, 1), np.uint8), np.zeros(max(val_cap, 1), np.uint8)
    ke, ve = np.zeros(max(ent_cap, 1), np.uint32), np.zeros(max(ent_cap, 1), np.uint32)
    vw = np.zeros(max(ent_cap, 1), np.uint64)
    bf, bs = np.zeros(nblk + 1, np.uint32), np.zeros(nblk, np.int32)
    d = _lib.LsmgpuDecoded()
    d.key_data, d.key_cap, d.key_end = _ptr(kd), key_cap, _ptr(ke)
    d.val_data, d.val_cap, d.val_end = _ptr(vd), val_cap, _ptr(ve)
    d.view, d.ent_cap, d.blk_first, d.blk_status = _ptr(vw), ent_cap, _ptr(bf), _ptr(bs)
    rc = _lib.lib().lsmgpu_decode_blocks(codec._ctx, _ptr(buf), buf.size, 0, _ptr(off), _ptr(ln),
                                         nblk, mode, byref(d))
    return rc, d, (kd, ke, vd, ve, vw, bf, bs)


def test_host_pipeline_capacity(codec, oracle, monkeypatch):
    """Upper-bound buffers succeed in one call; buffers short by one entry / one byte return
    LSMGPU_ERR_CAPACITY with the exact needs (the shim's retry), blk_first / blk_status filled."""
    monkeypatch.setenv("LSMGPU_HOST_CHUNK", "1048576")
    data, off, ln = _mixed(oracle)
    ref = oracle.decode(data, off, ln)
    both = MODE_MATERIALIZE | MODE_VIEW
    n, kb, vb = ref.n_entries, ref.key_data.size, ref.val_data.size
    rc, d, arrs = _decode_raw(codec, data, off, ln, both, len(data), len(data), len(data) // 10 + 1)
    assert rc == _lib.OK and (d.n_entries, d.key_bytes, d.val_bytes) == (n, kb, vb)
    assert arrs[0][:kb].tobytes() == ref.key_data.tobytes() and np.array_equal(arrs[4][:n], ref.view)
    for caps in ((kb, vb, n - 1), (kb - 1, vb, n), (kb, vb - 1, n)):
        rc, d, arrs = _decode_raw(codec, data, off, ln, both, *caps)
        assert rc == _lib.ERR_CAPACITY, caps
        assert (d.n_entries, d.key_bytes, d.val_bytes) == (n, kb, vb)
        assert (d.first_bad_block, d.n_bad_blocks) == (ref.first_bad_block, ref.n_bad_blocks)
        assert np.array_equal(arrs[5], ref.blk_first) and np.array_equal(arrs[6], ref.blk_status)
    rc, d, _ = _decode_raw(codec, data, off, ln, both, kb, vb, n)  # exactly the needs
    assert rc == _lib.OK


def test_host_pipeline_fallbacks(codec, oracle, monkeypatch):
    """Unsorted block lists and prefix-compressed keys that outgrow a chunk's device slot decode
    in one shot, with the same results."""
    import struct
    monkeypatch.setenv("LSMGPU_HOST_CHUNK", "1048576")
    data, off, ln = _mixed(oracle)
    rev_o, rev_l = np.ascontiguousarray(off[::-1]), np.ascontiguousarray(ln[::-1])
    _assert_same(codec.decode_host(data, rev_o, rev_l), oracle.decode(data, rev_o, rev_l), "reversed")
    # a 60 KiB block of prefix-compressed entries whose keys expand to ~10 MB, among C2 blocks
    rng = np.random.default_rng(5)
    blk = bytearray()
    base = bytes(rng.integers(0, 256, 3000, dtype=np.uint8))
    prev = 0xFFFFFFFF
    for e in range(4000):
        pos = len(blk)
        plen, diff = (0, base) if e == 0 else (2900, b"x")
        blk += struct.pack(">HHHI", plen, len(diff), 1, prev) + diff + b"v"
        prev = pos
    blk += struct.pack(">HHHI", 0, 0, 3, prev) + b"\0\0\0"
    c2 = _cols(2, 40000, seed=65)
    sst = oracle.build_cols(c2.keys, c2.key_end, c2.vs, c2.vs_end, 0, 4096)[0]
    d2, o2, l2 = _sst_blocks(oracle, [sst])
    full = d2 + bytes(blk)
    o3 = np.concatenate([o2, [len(d2)]]).astype(np.uint32)
    l3 = np.concatenate([l2, [len(blk)]]).astype(np.uint32)
    ref = oracle.decode(full, o3, l3)
    assert ref.key_data.size > len(full)
    _assert_same(codec.decode_host(full, o3, l3), ref, "expanding keys")
    _ = ctypes
