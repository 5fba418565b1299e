"""Batched table open on the GPU (lsmgpu_open_tables_async) against the
oracle restatement sstref_open_table: every case of open_cases.py in ONE batch (tables at odd
offsets of one device buffer), statuses, block index, sorted order, smallest / biggest; a batch
of C4-sized tables; the capacity bound."""
import numpy as np
import pytest

import open_cases as C

pytestmark = pytest.mark.gpu


def _check(label, got, ref):
    assert got["status"] == ref["status"], label
    if ref["status"] not in (0, 6):
        return
    assert got["nblk"] == ref["nblk"], label
    assert (got["bloom_off"], got["bloom_len"]) == (ref["bloom_off"], ref["bloom_len"]), label
    for k in ("blk_off", "blk_len", "key_off", "key_len", "order"):
        assert np.array_equal(got[k], ref[k]), (label, k)
    assert got["smallest"] == ref["smallest"], label
    assert got["biggest"] == ref["biggest"], label


def test_open_tables_batch(codec, oracle):
    cases = C.cases(oracle)
    # odd offsets: pad each image (the padding is outside every table)
    ssts = [sst for _, sst in cases]
    got = codec.open_tables_host(ssts)
    for (label, sst), g in zip(cases, got):
        _check(label, g, oracle.open_table(sst))


def test_open_tables_one_by_one(codec, oracle):
    for label, sst in C.cases(oracle):
        _check(label, codec.open_tables_host([sst])[0], oracle.open_table(sst))


def test_open_tables_c4(codec, oracle):
    """C4: SSTs cut by ReachedCapacity(64 MiB) at 100 entries/block (~5,196 blocks each), one
    of them with its blocks shuffled (the device rank sort)."""
    from lsmdb_amd import workload
    ssts = []
    for s in range(3):
        c = workload.config_columns(4, 520000, seed_offset=s)
        sst, _, _ = oracle.build_cols(c.keys, c.key_end, c.vs, c.vs_end, c.entries_per_block,
                                      c.block_bytes)
        ssts.append(sst + C.TAIL)
    nb = len(C.blocks_of(oracle, ssts[0][: -len(C.TAIL)]))
    perm = np.random.default_rng(1).permutation(nb)
    ssts.append(C.reorder(oracle, ssts[0][: -len(C.TAIL)], perm))
    got = codec.open_tables_host(ssts)
    for t, (sst, g) in enumerate(zip(ssts, got)):
        ref = oracle.open_table(sst)
        assert ref["nblk"] > 5000
        _check(f"C4 table {t}", g, ref)


def test_open_tables_capacity(codec, oracle):
    cases = C.cases(oracle)
    ssts = [cases[0][1], cases[1][1]]
    n0 = oracle.open_table(ssts[0])["nblk"]
    got = codec.open_tables_host(ssts, blk_cap=n0 + 1)  # table 1 does not fit
    _check("fits", got[0], oracle.open_table(ssts[0]))
    assert got[1]["status"] == 5
