"""lsmgpu_decode_blocks on host memory (data_on_device = 0), the path a cgo caller with an mmap'd
.sst takes (table/table.go:88-144,153-166): blocks sorted by offset are decoded as a pipeline of
chunks (copy-in / decode / copy-out on three streams, api.hip decode_host_pipelined).  Chunk
sizes of 1-3 MiB (LSMGPU_HOST_CHUNK) cut the test inputs into many chunks, so the per-chunk
bases, the block-index and status arrays across chunk borders, the first bad block and the
capacity rules are all exercised; every output is checked against the oracle.  Unsorted block
lists and chunks whose prefix-compressed keys outgrow their device slot take the one-shot path.

ABI 4 (host_io.hpp): pageable input and outputs are staged through the ctx's own page-locked
buffers; lsmgpu_host_alloc memory is DMA'd directly.  Both sides are run in every combination.
lsmgpu_host_register pins nothing any more; the register / unregister / re-use cycles that
faulted in round 5 (GPUTEST_r05) stay here as the regression test of that fix."""
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
    data, off, ln = _mixed(oracle)
    return data, off, ln, oracle.decode(data, off, ln)


def _check(g, ref, m, what):
    if m == MODE_VIEW:
        assert g.n_entries == ref.n_entries and np.array_equal(g.view, ref.view), what
        assert np.array_equal(g.blk_first, ref.blk_first), what
        assert np.array_equal(g.blk_status, ref.blk_status), what
        assert g.first_bad_block == ref.first_bad_block and g.n_bad_blocks == ref.n_bad_blocks, what
    else:
        if m == MODE_MATERIALIZE:
            g.view = None
        _assert_same(g, ref, what)


@pytest.mark.parametrize("chunk", ["1048576", "3000000"])
@pytest.mark.parametrize("mode", ["both", "view", "materialize"])
def test_host_pipeline_vs_oracle(codec, mixed, monkeypatch, chunk, mode):
    """Input pageable, registered (register -> decode -> unregister on a fresh buffer: the
    allocator hands back pages of earlier tests' buffers, as compaction's OpenTable / DecrRef
    cycles do, levels.go:281-298, table/table.go:53-71) or in host_alloc memory; outputs pageable
    or in host_alloc memory: the staged and the direct DMA branches of both copy directions."""
    monkeypatch.setenv("LSMGPU_HOST_CHUNK", chunk)
    data, off, ln, ref = mixed
    m = {"both": MODE_MATERIALIZE | MODE_VIEW, "view": MODE_VIEW, "materialize": MODE_MATERIALIZE}[mode]
    for src in ("pageable", "registered", "host_alloc"):
        for pinned_out in (False, True):
            if src == "host_alloc":
                buf = codec.host_alloc(len(data))
                buf[:] = np.frombuffer(data, np.uint8)
            else:
                buf = np.frombuffer(data, np.uint8).copy()
            if src == "registered":
                codec.host_register(buf)
            try:
                g = codec.decode_host(buf, off, ln, mode=m, pinned_out=pinned_out)
            finally:
                if src == "registered":
                    codec.host_unregister(buf)
            _check(g, ref, m, f"chunk={chunk} src={src} pinned_out={pinned_out}")


def test_host_churn_reused_addresses(codec, mixed, monkeypatch):
    """Compaction's OpenTable / DecrRef churn (levels.go:281-298, table/table.go:53-71,117-123):
    40 rounds of allocate -> register -> decode -> unregister -> free, at random sizes and
    misalignments, so buffers come back at addresses earlier rounds used (the round-5 fault,
    GPUTEST_r05); every round checked against the oracle.  Registration pins nothing: registering
    the same range twice is accepted (the runtime does not see it as page-locked)."""
    monkeypatch.setenv("LSMGPU_HOST_CHUNK", "1048576")
    data, off, ln, ref = mixed
    rng = np.random.default_rng(11)
    n = len(data)
    for r in range(40):
        pad = int(rng.integers(0, 8192))
        raw = np.empty(n + pad + int(rng.integers(0, 3 << 20)), np.uint8)
        buf = raw[pad:pad + n]
        buf[:] = np.frombuffer(data, np.uint8)
        codec.host_register(buf)
        assert _lib.lib().lsmgpu_host_register(codec._ctx, _ptr(buf), buf.nbytes) == _lib.OK
        g = codec.decode_host(buf, off, ln, pinned_out=bool(r % 3 == 2))
        codec.host_unregister(buf)
        codec.host_unregister(buf)
        _check(g, ref, 3, f"churn round {r}")
        del raw, buf, g


def test_host_register_shared_pages(codec, mixed, monkeypatch):
    """Two non-page-aligned copies of the input in one allocation, 16 B apart (a page shared by
    both, as Go heap buffers under LoadToRAM share pages, table/table.go:117-123,329-338): both
    registered, both decoded, the first unregistered and the second decoded again, then
    unregistered, then the first decoded unregistered.  (Since ABI 4 registration is bookkeeping
    only -- nothing is page-locked -- so this checks that the registry's ranges, not pages,
    decide what is registered.)"""
    monkeypatch.setenv("LSMGPU_HOST_CHUNK", "1048576")
    data, off, ln, ref = mixed
    n = len(data)
    big = np.zeros(2 * n + 8192, np.uint8)
    a0 = 100 + (-big.ctypes.data) % 4096  # 100 B past a page start
    a = big[a0:a0 + n]
    b = big[a0 + n + 16:a0 + 2 * n + 16]
    a[:] = np.frombuffer(data, np.uint8)
    b[:] = a
    codec.host_register(a)
    codec.host_register(b)
    _check(codec.decode_host(a, off, ln), ref, 3, "a")
    _check(codec.decode_host(b, off, ln), ref, 3, "b")
    codec.host_unregister(a)
    _check(codec.decode_host(b, off, ln), ref, 3, "b after a unpinned")
    codec.host_unregister(b)
    _check(codec.decode_host(a, off, ln), ref, 3, "a unpinned")


def test_host_register_cycles_and_nesting(codec, mixed, monkeypatch):
    """register / unregister / register again at one address (the round-5 fault: GPUTEST_r05,
    illegal address on the first D2H of this test); a sub-range registered inside a registered
    range and decoded at an unaligned pointer; unregistering in either order; an unknown pointer
    is LSMGPU_ERR_ARG."""
    monkeypatch.setenv("LSMGPU_HOST_CHUNK", "1048576")
    data, off, ln, ref = mixed
    buf = np.zeros(len(data) + 4096 + 13, np.uint8)
    sub = buf[13:13 + len(data)]
    sub[:] = np.frombuffer(data, np.uint8)
    for _ in range(3):
        codec.host_register(sub)
        _check(codec.decode_host(sub, off, ln), ref, 3, "cycle")
        codec.host_unregister(sub)
    codec.host_register(buf)
    codec.host_register(sub)  # nested inside a registered range
    _check(codec.decode_host(sub, off, ln), ref, 3, "nested")
    codec.host_unregister(buf)  # the outer range goes first: sub stays registered
    _check(codec.decode_host(sub, off, ln), ref, 3, "nested, outer unpinned")
    codec.host_unregister(sub)
    rc = _lib.lib().lsmgpu_host_unregister(codec._ctx, _ptr(sub))
    assert rc == _lib.ERR_ARG


def test_host_register_readonly_mmap(codec, oracle, tmp_path, monkeypatch):
    """A real .sst file mmap'd read-only (MemoryMap mode, table/table.go:88-144, y/mmap.go:11-21)
    is registered, decoded through the pipeline (staged) and unregistered."""
    import mmap
    monkeypatch.setenv("LSMGPU_HOST_CHUNK", "1048576")
    c2 = _cols(2, 60000, seed=71)
    body, _, _ = oracle.build_cols(c2.keys, c2.key_end, c2.vs, c2.vs_end, 0, 4096)
    sst = body + b"{}" + (2).to_bytes(4, "big")
    path = tmp_path / "000001.sst"
    path.write_bytes(sst)
    off, ln, _, _ = oracle.parse_index(sst)
    ref = oracle.decode(sst, off, ln)
    with open(path, "rb") as f:
        mm = mmap.mmap(f.fileno(), 0, prot=mmap.PROT_READ)
        arr = np.frombuffer(mm, np.uint8)
        codec.host_register(arr)
        try:
            g = codec.decode_host(arr, off, ln)
        finally:
            codec.host_unregister(arr)
        _check(g, ref, 3, "read-only mmap")
        del arr
        mm.close()


def test_host_register_foreign_pinned(codec, mixed, monkeypatch):
    """Memory page-locked outside the library (torch's pinned allocator, hipHostMalloc) is not
    registered: LSMGPU_ERR_HOST_PINNED, and it decodes as it is (direct DMA)."""
    import torch
    monkeypatch.setenv("LSMGPU_HOST_CHUNK", "1048576")
    data, off, ln, ref = mixed
    t = torch.empty(len(data), dtype=torch.uint8, pin_memory=True)
    arr = t.numpy()
    arr[:] = np.frombuffer(data, np.uint8)
    rc = _lib.lib().lsmgpu_host_register(codec._ctx, _ptr(arr), arr.nbytes)
    assert rc == _lib.ERR_HOST_PINNED
    _check(codec.decode_host(arr, off, ln), ref, 3, "foreign pinned")
    assert _lib.lib().lsmgpu_host_unregister(codec._ctx, _ptr(arr)) == _lib.ERR_ARG


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


def test_host_mode_rejects_device_pointer(codec, oracle):
    """data_on_device = 0 with a device pointer is an argument error (LSMGPU_ERR_ARG), not a host
    memcpy from device memory."""
    import torch
    c2 = _cols(2, 5000, seed=81)
    body, _, _ = oracle.build_cols(c2.keys, c2.key_end, c2.vs, c2.vs_end, 0, 4096)
    sst = body + b"{}" + (2).to_bytes(4, "big")
    off, ln, _, _ = oracle.parse_index(sst)
    d_sst = torch.from_numpy(np.frombuffer(sst, np.uint8).copy()).cuda()
    d = _lib.LsmgpuDecoded()
    bf = np.zeros(off.size + 1, np.uint32)
    d.blk_first = _ptr(bf)
    rc = _lib.lib().lsmgpu_decode_blocks(codec._ctx, d_sst.data_ptr(), len(sst), 0, _ptr(off), _ptr(ln),
                                         off.size, MODE_VIEW, byref(d))
    assert rc == _lib.ERR_ARG
