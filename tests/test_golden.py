"""The committed golden fixtures vs the seeded generator and the C oracle (CPU).

Pins three things at once: the workload generator (input digests), the oracle encoder
(Builder.Add/Finish restatement -> identical SST bytes) and the oracle decoder (blockIterator
restatement -> identical streams / offsets).  The fixtures' block KATs are also checked against
the hand-derived statuses of tests/kat_defs.py, which were written from the Go source, not by
the oracle.
"""
import numpy as np
import pytest

import golden_io as G
import kat_defs as K
import oracle_ffi as ofi
from lsmdb_amd import workload


@pytest.mark.parametrize("name", G.sst_names())
def test_generator_pinned(name):
    c = G.manifest()["sst"][name]
    cols = workload.config_columns(c["config"], c["entries"])
    d = c["input_sha256"]
    assert G.sha(cols.keys) == d["keys"]
    assert G.sha(cols.key_end.astype("<u4")) == d["key_end"]
    assert G.sha(cols.vs) == d["vs"]
    assert G.sha(cols.vs_end.astype("<u4")) == d["vs_end"]


@pytest.mark.parametrize("name", G.sst_names())
def test_oracle_encode_matches_golden(name):
    c, sst, *_ = G.load_sst(name)
    cols = workload.config_columns(c["config"], c["entries"])
    out, data_len, restarts = ofi.build_cols(cols.keys.tobytes(), cols.key_end, cols.vs.tobytes(),
                                             cols.vs_end, c["entries_per_block"], c["block_bytes"])
    assert data_len == c["data_len"] and restarts.size == c["nblocks"]
    assert G.sha(out) == c["sst_sha256"] and out == sst


@pytest.mark.parametrize("name", G.sst_names())
def test_oracle_decode_matches_golden(name):
    c, sst, off, ln, key_end, val_end, blk_first = G.load_sst(name)
    d = ofi.decode(sst[: c["data_len"]], off, ln)
    assert d.n_entries == c["entries"] and d.n_bad_blocks == 0
    assert np.array_equal(d.key_end, key_end) and np.array_equal(d.val_end, val_end)
    assert np.array_equal(d.blk_first, blk_first)
    assert G.sha(d.key_data) == c["key_sha256"] and G.sha(d.val_data) == c["val_sha256"]


def test_golden_blocks_match_hand_kats():
    b, data, off, ln = G.load_blocks()
    assert b["names"] == [k[0] for k in K.DECODE_KATS]
    assert b["blk_status"] == [k[3] for k in K.DECODE_KATS]
    expect = [[k.hex(), v.hex()] for _, _, ents, _ in K.DECODE_KATS for k, v in ents]
    assert b["entries"] == expect
    d = ofi.decode(data, off, ln)
    assert [int(s) for s in d.blk_status] == b["blk_status"]
    assert [int(x) for x in d.blk_first] == b["blk_first"]
    assert d.first_bad_block == b["first_bad_block"] and d.n_bad_blocks == b["n_bad_blocks"]
