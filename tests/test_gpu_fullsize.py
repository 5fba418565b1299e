"""Parity at BASELINE.json's full sizes:

* C2: a whole 1 GiB shard of 4 KiB blocks, built by the device encoder and decoded through
  lsmgpu_decode_blocks_async (the benchmarked call), must give back the encoder's input columns
  byte for byte (decode(encode(x)) == x), its block plan, and a view index whose records point
  at those same bytes.
* C4: full 64 MiB ReachedCapacity-cut tables -- one alone (group walk: <= 64 blocks per CU) and
  eight in one batch (~43 K blocks, the lane walk at C4 scale: the 8-SST compaction replay's
  decode) -- against the oracle decode (table/iterator.go:93-135), every output array; then
  the replay's merge of three overlapping 64 MiB tables against the oracle MergeIterator.
"""
import numpy as np
import pytest

import open_cases as C
from lsmdb_amd import workload

pytestmark = pytest.mark.gpu


def test_c2_full_gib_round_trip(codec):
    import torch
    import bench
    from lsmdb_amd.codec import MODE_MATERIALIZE, MODE_VIEW
    dev = torch.device("cuda", codec.device)
    torch.cuda.set_device(dev)
    w = bench.build_device_sst(codec, torch, dev, 2, 1 << 30, 0)
    assert w["data_len"] > 1_000_000_000 and w["max_len"] <= 4096
    both = MODE_MATERIALIZE | MODE_VIEW
    bufs = codec.alloc_decode(w["data_len"], w["data_len"], w["nblocks"], both, ent_cap=w["n"])
    codec.decode_device_async(w["d_sst"], w["d_off"], w["d_len"], w["max_len"], both, bufs,
                              data_len=w["data_len"])
    codec.synchronize()
    r = bufs.result.cpu().numpy()
    n, kb, vb = int(r[0]), int(r[1]), int(r[2])
    assert (n, kb, vb) == (w["n"], w["key_total"], w["vs_total"]) and r[4] == 0 and r[5] == 0
    assert torch.equal(bufs.key_data[:kb], w["d_keys"]) and torch.equal(bufs.val_data[:vb], w["d_vs"])
    assert torch.equal(bufs.key_end[:n], w["d_ke"]) and torch.equal(bufs.val_end[:n], w["d_ve"])
    assert torch.equal(bufs.blk_first[: w["nblocks"] + 1], w["d_plan"])
    assert int((bufs.blk_status[: w["nblocks"]] != 0).sum().item()) == 0
    # view records: key at key_pos (klen bytes), value right after it (vlen bytes)
    v = bufs.view[:n]
    kpos = (v & 0xFFFFFFFF)
    klen = (v >> 32) & 0xFFFF
    vlen = (v >> 48) & 0xFFFF
    ke = w["d_ke"].to(torch.int64)
    ve = w["d_ve"].to(torch.int64)
    assert torch.equal(klen, torch.diff(ke, prepend=ke.new_zeros(1)))
    assert torch.equal(vlen, torch.diff(ve, prepend=ve.new_zeros(1)))
    # every key's first and last 8 bytes, read through its view record, are the key's bytes
    sst = w["d_sst"]
    ks = ke - klen
    for off in (0, 8):
        got = torch.stack([sst[kpos + off + j] for j in range(8)], 1)
        want = torch.stack([w["d_keys"][ks + off + j] for j in range(8)], 1)
        assert torch.equal(got, want)
    # and every value's first byte (Meta) sits right after its key
    assert torch.equal(sst[kpos + klen], w["d_vs"][ve - vlen])


def test_c2_full_gib_repeated_view_and_materialize(codec):
    """The live walk's shared prefix machinery under repetition at 2^30 B: 1,041 walk tiles for
    1,024 resident workgroup slots (more workgroups than fit at once), the ticket counter reset
    by the last ticket of each launch, epoch-tagged tile records never cleared between launches
    and the decoupled look-back.  40 decodes back to back alternate view-only (the fused view
    epilogue) and materialize (walk + copy); every one must give the block plan as blk_first,
    no error flag, and the same view records / end offsets as the first.  (Round 4's removed
    one-pass kernel produced a wrong block index once and shared the ticket / tag / look-back
    primitives -- DESIGN section 5.)"""
    import torch
    import bench
    from lsmdb_amd.codec import MODE_MATERIALIZE, MODE_VIEW
    dev = torch.device("cuda", codec.device)
    torch.cuda.set_device(dev)
    w = bench.build_device_sst(codec, torch, dev, 2, 1 << 30, 0)
    assert (w["nblocks"] + 255) // 256 > 4 * 256  # more walk tiles than resident workgroups
    vb = codec.alloc_decode(w["data_len"], 0, w["nblocks"], MODE_VIEW, ent_cap=w["n"])
    mb = codec.alloc_decode(w["data_len"], w["data_len"], w["nblocks"], MODE_MATERIALIZE, ent_cap=w["n"])
    plan = w["d_plan"]
    first_view = None
    for i in range(40):
        view = i % 2 == 0
        b = vb if view else mb
        codec.decode_device_async(w["d_sst"], w["d_off"], w["d_len"], w["max_len"],
                                  MODE_VIEW if view else MODE_MATERIALIZE, b, data_len=w["data_len"])
        codec.synchronize()
        r = b.result.cpu().numpy()
        assert int(r[0]) == w["n"] and r[4] == 0 and r[5] == 0, (i, r)
        assert torch.equal(b.blk_first[: w["nblocks"] + 1], plan), i
        if view:
            if first_view is None:
                first_view = b.view[: w["n"]].clone()
            else:
                assert torch.equal(b.view[: w["n"]], first_view), i
        else:
            assert torch.equal(b.key_end[: w["n"]], w["d_ke"]) and torch.equal(b.val_end[: w["n"]], w["d_ve"]), i
    assert torch.equal(mb.key_data[: w["key_total"]], w["d_keys"])


def _c4_table(oracle, seed: int, select=None) -> bytes:
    """One 64 MiB ReachedCapacity(64 MiB)-cut table, oracle-built (100 entries per block)."""
    import bench
    cols = workload.config_columns(4, 560_000 if select is None else 1_600_000, seed_offset=seed)
    ke, ve = cols.key_end.astype(np.int64), cols.vs_end.astype(np.int64)
    if select is not None:  # a subset of a shared key space: tables that overlap
        idx = np.nonzero(select(cols.n))[0]
        kl = np.diff(ke, prepend=0)[idx]
        vl = np.diff(ve, prepend=0)[idx]
        k2 = cols.keys.reshape(-1, 16)[idx].reshape(-1)
        vs_start = (ve - np.diff(ve, prepend=0))[idx]
        v2 = np.concatenate([cols.vs[s: s + l] for s, l in zip(vs_start, vl)])
        ke, ve = np.cumsum(kl), np.cumsum(vl)
        keys, vs = k2, v2
    else:
        keys, vs = cols.keys, cols.vs
    n = bench.c4_table_entries(ke.astype(np.uint32), ve.astype(np.uint32), 64 << 20)
    body, _, _ = oracle.build_cols(keys[: ke[n - 1]], ke[:n].astype(np.uint32),
                                   vs[: ve[n - 1]], ve[:n].astype(np.uint32), 100, 0)
    assert len(body) > 64_000_000
    return body + C.TAIL


def _blocks(oracle, ssts):
    offs, lens, first, base = [], [], [], 0
    datas = []
    for s in ssts:
        o, l, _, _ = oracle.parse_index(s)
        first.append(sum(x.size for x in offs))
        offs.append(o + base)
        lens.append(l)
        end = int(o[-1]) + int(l[-1])
        datas.append(s[:end])
        base += end
    return (b"".join(datas), np.concatenate(offs).astype(np.uint32),
            np.concatenate(lens).astype(np.uint32), first)


def _same(g, o):
    assert g.n_entries == o.n_entries
    assert g.key_data.tobytes() == o.key_data.tobytes() and g.val_data.tobytes() == o.val_data.tobytes()
    assert np.array_equal(g.key_end, o.key_end) and np.array_equal(g.val_end, o.val_end)
    assert np.array_equal(g.view, o.view) and np.array_equal(g.blk_first, o.blk_first)
    assert np.array_equal(g.blk_status, o.blk_status)


def test_c4_one_table(codec, oracle):
    data, off, ln, _ = _blocks(oracle, [_c4_table(oracle, 0)])
    assert off.size > 5000
    _same(codec.decode_host(data, off, ln), oracle.decode(data, off, ln))


def test_c4_eight_tables_and_merge(codec, oracle):
    rng = np.random.default_rng(11)
    # tables 0-2 share one key space (each takes a third of it + 20 % of the rest: duplicates
    # across tables), tables 3-7 are disjoint key ranges, as the bottom level would be
    sel = [lambda n, t=t: (np.arange(n) % 3 == t) | (rng.random(n) < 0.2) for t in range(3)]
    ssts = [_c4_table(oracle, 0, sel[t]) for t in range(3)] + [_c4_table(oracle, s) for s in range(3, 8)]
    data, off, ln, first = _blocks(oracle, ssts)
    assert off.size > 40_000
    g = codec.decode_host(data, off, ln)
    o = oracle.decode(data, off, ln)
    _same(g, o)
    # the replay's merge of the three overlapping tables (MergeIterator, y/iterator.go:74-202)
    rf = np.array([int(g.blk_first[first[t]]) for t in range(3)] + [int(g.blk_first[first[3]])],
                  np.uint32)
    kd, vd = g.key_data.tobytes(), g.val_data.tobytes()
    ke, ve = g.key_end[: rf[-1]], g.val_end[: rf[-1]]
    mk, mke, mv, mve, msrc, fl = codec.merge_host(kd[: int(ke[-1])], ke, vd[: int(ve[-1])], ve, rf)
    want = oracle.merge(kd[: int(ke[-1])], ke, rf)
    assert fl == 0 and np.array_equal(msrc, want)
    assert msrc.size < rf[-1]  # duplicates were dropped
    ks = np.concatenate([[0], ke.astype(np.int64)])
    lens = (ks[want + 1] - ks[want])
    assert np.array_equal(np.diff(mke.astype(np.int64), prepend=0), lens)
