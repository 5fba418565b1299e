"""Batched table open, CPU side: the oracle restatement
sstref_open_table (oracle/sstref.c) against the host mirror of Table/Iterator
(lsmdb_amd/table.py, run on the oracle decoder) -- two independent restatements of
table.go:88-144,177-269 and iterator.go:86-155,201-235 -- on every well-formed case."""
import numpy as np
import pytest

import open_cases as C


def _host_open(oracle, sst):
    from lsmdb_amd import table as T
    return T.OpenTable(sst, decoder=lambda d, o, n: oracle.decode(bytes(d), o, n))


def test_oracle_matches_host_mirror(oracle):
    checked = 0
    for label, sst in C.cases(oracle):
        ref = oracle.open_table(sst)
        if ref["status"] != 0:
            continue
        t = _host_open(oracle, sst)
        assert t.Smallest() == ref["smallest"], label
        assert t.Biggest() == ref["biggest"], label
        got = [ko.fblk for ko in t.block_index]
        assert got == [int(x) for x in ref["order"]], label
        assert [ko.offset for ko in t.block_index] == [int(ref["blk_off"][i]) for i in ref["order"]], label
        checked += 1
    assert checked >= 10


def test_oracle_statuses(oracle):
    st = {label: oracle.open_table(sst)["status"] for label, sst in C.cases(oracle)}
    assert st["bad tail: bloom length"] == 1
    assert st["bad tail: restarts"] == 1
    assert st["first plen"] == 2
    assert st["first key past the file"] == 3
    assert st["short keys, 3 blocks"] == 4
    assert st["short keys, 1 block"] == 0  # one block: sort.Sort compares nothing
    assert oracle.open_table(C.cases(oracle)[0][1], cap=3)["status"] == 5
