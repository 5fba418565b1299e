"""GPU parity of the fused stream-walk-scan-copy decode (decode_fsc.hip, LSMGPU_DECODE_PATH=fsc):
one launch per batch of <= 4 KiB blocks, ticket-ordered 32-block tiles with a decoupled
look-back, each tile streamed through LDS 8 blocks at a time.  Every output array is checked
bit-exact against the oracle (oracle/sstref.c, the C restatement of table/iterator.go:93-135).
"""
import struct

import numpy as np
import pytest

import kat_defs as K
from lsmdb_amd import workload
from test_gpu_parity import _assert_same, _random_cols, _sst_blocks, test_prefix_compressed_random

pytestmark = pytest.mark.gpu


@pytest.fixture
def fsc(monkeypatch):
    monkeypatch.setenv("LSMGPU_DECODE_PATH", "fsc")


def _kat_batch(reps=3, base=b""):
    kd = bytearray(base)
    offs, lens = [], []
    for i, (_n, block, _e, _s) in enumerate(K.DECODE_KATS * reps):
        kd += b"\xab" * (i % 13)
        offs.append(len(kd))
        lens.append(len(block))
        kd += block
    return bytes(kd), offs, lens


def _c2_sst(oracle, n, seed):
    c = workload.config_columns(2, n, seed)
    sst, _, _ = oracle.build_cols(c.keys, c.key_end, c.vs, c.vs_end, 0, 4096)
    return c, sst


def test_fsc_shapes(codec, oracle, fsc):
    """C2 4 KiB blocks, C3 64 B / 1 KiB entries, short random entries (90-180 per block),
    tiny entries (~170 per block, keys/values < 16 B), the KAT blocks (every error status,
    terminators, plen > 0) at odd alignments, all in one batch and separately."""
    c2 = workload.config_columns(2, 30000, 3)
    c3 = workload.config_columns(3, 3000, 4)
    parts = [oracle.build_cols(c2.keys, c2.key_end, c2.vs, c2.vs_end, 0, 4096)[0],
             oracle.build_cols(c3.keys, c3.key_end, c3.vs, c3.vs_end, 0, 4096)[0],
             oracle.build_cols(*_random_cols(20000, 5), 0, 4096)[0],
             oracle.build_cols(*_random_cols(60000, 11, 9, 10, 3, 4), 0, 4096)[0]]
    data, off, ln = _sst_blocks(oracle, parts)
    assert int(ln.max()) <= 4096
    _assert_same(codec.decode_host(data, off, ln), oracle.decode(data, off, ln), "fsc mixed")
    kd, offs, lens = _kat_batch(3, data)
    o2 = np.concatenate([off, np.array(offs, np.uint32)]).astype(np.uint32)
    l2 = np.concatenate([ln, np.array(lens, np.uint32)]).astype(np.uint32)
    _assert_same(codec.decode_host(kd, o2, l2), oracle.decode(kd, o2, l2), "fsc + kats")
    kd2, offs2, lens2 = _kat_batch(2)
    o3, l3 = np.array(offs2, np.uint32), np.array(lens2, np.uint32)
    _assert_same(codec.decode_host(kd2, o3, l3), oracle.decode(kd2, o3, l3), "fsc kats")
    test_prefix_compressed_random(codec, oracle)


def test_fsc_many_tiles(codec, oracle, fsc):
    """~10,000 blocks = ~320 tiles of 32 (look-back across hundreds of tile records), a
    ragged last tile, non-contiguous block lists (every other block, reversed order)."""
    c, sst = _c2_sst(oracle, 330000, 13)
    sst = sst + b"{}" + (2).to_bytes(4, "big")
    off, ln, _, _ = oracle.parse_index(sst)
    assert len(off) % 32 != 0
    g = codec.decode_host(sst, off, ln)
    _assert_same(g, oracle.decode(sst, off, ln), "many tiles")
    assert g.key_data.tobytes() == c.keys.tobytes()
    assert g.val_data.tobytes() == c.vs.tobytes()
    for sl in (slice(None, None, 2), slice(None, None, -1), slice(7, 7 + 33)):
        o2, l2 = np.ascontiguousarray(off[sl]), np.ascontiguousarray(ln[sl])
        _assert_same(codec.decode_host(sst, o2, l2), oracle.decode(sst, o2, l2), f"slice {sl}")


def _prefix_blocks(rng, nblocks):
    """Prefix-compressed 4 KiB blocks whose OUTPUT keys pass 64 KiB per block (a 3,000-B base
    key, ~70 entries sharing 2,000-3,000 B of it): key offsets must not be held in 16 bits."""
    out = []
    for _ in range(nblocks):
        blk = bytearray()
        base = bytes(rng.integers(0, 256, 3000, dtype=np.uint8))
        prev = 0xFFFFFFFF
        blk += struct.pack(">HHHI", 0, len(base), 1, prev) + base + b"v"
        prev = 0
        while True:
            plen = int(rng.integers(2000, 3001))
            diff = bytes(rng.integers(0, 256, int(rng.integers(0, 3)), dtype=np.uint8))
            val = bytes(rng.integers(0, 256, int(rng.integers(0, 4)), dtype=np.uint8))
            ent = struct.pack(">HHHI", plen, len(diff), len(val), prev) + diff + val
            if len(blk) + len(ent) + 13 > 4096:
                break
            prev = len(blk)
            blk += ent
        blk += struct.pack(">HHHI", 0, 0, 3, prev) + b"\0\0\0"
        out.append(bytes(blk))
    return out


def test_fsc_prefix_large_output(codec, oracle, fsc):
    rng = np.random.default_rng(41)
    blocks = _prefix_blocks(rng, 5)
    _c, sst = _c2_sst(oracle, 20000, 5)
    o2, l2, _, _ = oracle.parse_index(sst + b"{}" + (2).to_bytes(4, "big"))
    data = bytearray()
    offs, lens = [], []
    for i, b in enumerate(blocks):  # prefix blocks between ordinary ones, in one tile and across
        offs.append(len(data))
        lens.append(len(b))
        data += b
    base = len(data)
    data += sst
    off = np.concatenate([np.array(offs, np.uint32), o2 + base]).astype(np.uint32)
    ln = np.concatenate([np.array(lens, np.uint32), l2]).astype(np.uint32)
    order = np.concatenate([np.arange(5, 40), np.arange(0, 5), np.arange(40, len(off))])
    off, ln = off[order].copy(), ln[order].copy()
    data = bytes(data)
    ref = oracle.decode(data, off, ln)
    assert ref.key_data.size > 65536
    _assert_same(codec.decode_host(data, off, ln), ref, "fsc prefix")


@pytest.mark.parametrize("path", ["fsc", "wsc-fused-view", "wsc-copy"])
@pytest.mark.parametrize("mode", ["view", "both", "none"])
def test_modes_device(codec, oracle, monkeypatch, path, mode):
    """Device-resident calls in view-only, materialize+view and mode 0 on the fused path and on
    walk-scan-copy (view epilogue in the walk forced on / off): view records match the oracle;
    mode 0 leaves a passed view buffer untouched (advisor finding, round 1)."""
    import torch
    from lsmdb_amd.codec import MODE_MATERIALIZE, MODE_VIEW
    monkeypatch.setenv("LSMGPU_DECODE_PATH", path[:3])
    if path.startswith("wsc"):
        monkeypatch.setenv("LSMGPU_WSC_VIEWFUSE", "1" if path == "wsc-fused-view" else "0")
    c, sst = _c2_sst(oracle, 60000, 21)
    sst = sst + b"{}" + (2).to_bytes(4, "big")
    off, ln, _, _ = oracle.parse_index(sst)
    o = oracle.decode(sst, off, ln)
    m = {"view": MODE_VIEW, "both": MODE_MATERIALIZE | MODE_VIEW, "none": 0}[mode]
    dev = torch.device("cuda", codec.device)
    d = torch.from_numpy(np.frombuffer(sst, np.uint8).copy()).to(dev)
    d_off = torch.from_numpy(off.view(np.int32)).to(dev)
    d_len = torch.from_numpy(ln.view(np.int32)).to(dev)
    bufs = codec.alloc_decode(len(sst), len(sst), len(off), MODE_MATERIALIZE | MODE_VIEW,
                              ent_cap=int(o.n_entries))
    bufs.view.fill_(-1)
    codec.decode_device_async(d, d_off, d_len, int(ln.max()), m, bufs)
    codec.synchronize()
    res = bufs.result.cpu().numpy()
    assert int(res[0]) == o.n_entries and int(res[5]) == 0
    assert np.array_equal(bufs.blk_first.cpu().numpy().view(np.uint32), o.blk_first)
    view = bufs.view.cpu().numpy().view(np.uint64)
    if m & MODE_VIEW:
        assert np.array_equal(view, o.view)
    else:
        assert (view == np.uint64(0xFFFFFFFFFFFFFFFF)).all()
    if m & MODE_MATERIALIZE:
        assert bufs.key_data[: int(res[1])].cpu().numpy().tobytes() == o.key_data.tobytes()
        assert bufs.val_data[: int(res[2])].cpu().numpy().tobytes() == o.val_data.tobytes()
        assert np.array_equal(bufs.key_end[: o.n_entries].cpu().numpy().view(np.uint32), o.key_end)
        assert np.array_equal(bufs.val_end[: o.n_entries].cpu().numpy().view(np.uint32), o.val_end)


def test_fsc_capacity_and_repeat(codec, oracle, fsc):
    """Output capacity overflow is reported (not written past), and repeated launches on one
    context (epoch-tagged look-back records, ticket reset by the last tile) stay exact."""
    c, sst = _c2_sst(oracle, 40000, 8)
    sst = sst + b"{}" + (2).to_bytes(4, "big")
    off, ln, _, _ = oracle.parse_index(sst)
    o = oracle.decode(sst, off, ln)
    for _ in range(3):
        _assert_same(codec.decode_host(sst, off, ln), o, "repeat")
    import torch
    from lsmdb_amd.codec import MODE_MATERIALIZE
    dev = torch.device("cuda", codec.device)
    d = torch.from_numpy(np.frombuffer(sst, np.uint8).copy()).to(dev)
    d_off = torch.from_numpy(off.view(np.int32)).to(dev)
    d_len = torch.from_numpy(ln.view(np.int32)).to(dev)
    bufs = codec.alloc_decode(len(sst), len(sst), len(off), MODE_MATERIALIZE,
                              ent_cap=int(o.n_entries) - 1)
    codec.decode_device_async(d, d_off, d_len, int(ln.max()), MODE_MATERIALIZE, bufs)
    codec.synchronize()
    assert int(bufs.result.cpu().numpy()[5]) & 1
