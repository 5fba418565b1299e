"""The CPU oracle against hand-derived known answers (tests/kat_defs.py)."""
import numpy as np
import pytest

import kat_defs as K


@pytest.mark.parametrize("name,keys,vss,epb,data,index", K.BUILDER_KATS)
def test_builder_kat(oracle, name, keys, vss, epb, data, index):
    out, data_len, restarts = oracle.build(keys, vss, entries_per_block=epb)
    assert data_len == len(data)
    assert out[:data_len] == data, name
    assert out[data_len:] == index, name
    off, ln, _, _ = oracle.parse_index(out + b'{"x":1}' + len(b'{"x":1}').to_bytes(4, "big"))
    assert int(off[-1] + ln[-1]) == data_len


@pytest.mark.parametrize("meta,um,exp,val,enc,size", K.VS_KATS)
def test_valuestruct_kat(oracle, meta, um, exp, val, enc, size):
    assert oracle.vs_encoded_size(exp, len(val)) == size
    got = oracle.vs_encode(meta, um, exp, val)
    if enc is not None:
        assert got == enc


@pytest.mark.parametrize("name,block,entries,status", K.DECODE_KATS)
def test_decode_kat(oracle, name, block, entries, status):
    pad = b"\xee" * 7  # bytes around the block: the decoder must never read past it
    data = pad + block + pad
    d = oracle.decode(data, np.array([len(pad)], np.uint32), np.array([len(block)], np.uint32))
    assert int(d.blk_status[0]) == status, name
    assert d.n_entries == len(entries)
    for i, (k, v) in enumerate(entries):
        assert d.key(i) == k
        assert d.value(i) == v
    assert int(d.blk_first[1]) == len(entries)


def test_builder_reached_capacity_and_empty(oracle):
    import ctypes
    L = oracle.lib()
    b = L.sstref_builder_new(100, 0)
    assert L.sstref_builder_empty(b) == 1
    k = K.K1
    v = K.V1
    kb = np.frombuffer(k, np.uint8)
    vb = np.frombuffer(v, np.uint8)
    L.sstref_builder_add(b, kb.ctypes.data, len(k), vb.ctypes.data, len(v))
    assert L.sstref_builder_empty(b) == 0
    # buf.Len() = 25: estimate = 25 + 8 + 0 + 8 = 41 (builder.go:140-143)
    assert L.sstref_builder_reached_capacity(b, 40) == 1
    assert L.sstref_builder_reached_capacity(b, 41) == 0
    L.sstref_builder_free(b)
    _ = ctypes
