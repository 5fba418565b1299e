"""bench.py's multi-GPU contract on CPU with gloo, world_size 2 (no GPU): every rank builds and
decodes its OWN shard (no data exchange), shards are disjoint and globally ordered, and the only
collectives -- max wall clock, parity AND, shard-byte sum -- give the whole-job aggregate."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, q):
    sys.path[:0] = [ROOT, HERE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import oracle_ffi as ofi
        from lsmdb_amd import codec as C, workload
        n = 2000
        cols = workload.config_columns(2, n, seed_offset=rank)      # bench.build_device_sst's shard
        plan = C.plan_blocks(cols.key_end, cols.vs_end, cols.entries_per_block, cols.block_bytes)
        sst, data_len, restarts = ofi.build_cols(cols.keys.tobytes(), cols.key_end,
                                                 cols.vs.tobytes(), cols.vs_end,
                                                 cols.entries_per_block, cols.block_bytes)
        assert restarts.size == plan.size - 1
        off = np.concatenate([[0], restarts[:-1]]).astype(np.uint32)
        d = ofi.decode(sst[:data_len], off, (restarts - off).astype(np.uint32))
        ok = d.key_data.tobytes() == cols.keys.tobytes() and d.val_data.tobytes() == cols.vs.tobytes()
        wall = 0.010 * (rank + 1)                                     # rank 1 is the slow one
        w, parity, total = bench.reduce_over_ranks(dist, torch, torch.device("cpu"), wall,
                                                   "ok" if ok else "MISMATCH", data_len)
        first_last = (cols.keys[:16].tobytes(), cols.keys[-16:].tobytes())
        q.put((rank, w, parity, total, data_len, first_last))
    finally:
        dist.destroy_process_group()


def test_two_rank_shards_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    walls = {r[1] for r in res}
    assert walls == {0.020}                        # max over ranks, seen by every rank
    assert all(r[2] == "ok" for r in res)
    total = res[0][4] + res[1][4]
    assert all(r[3] == total for r in res)         # sum of shard bytes
    (_, _, _, _, _, (f0, l0)), (_, _, _, _, _, (f1, l1)) = res
    assert f0 < l0 < f1 < l1                       # disjoint, globally ordered shards
    import bench
    assert bench.aggregate_gibs(total, 20.0 / 1) == pytest.approx(total / 0.020 / (1 << 30))


def test_one_rank_is_identity():
    import bench
    assert bench.reduce_over_ranks(None, torch, None, 1.5, "ok", 123) == (1.5, "ok", 123)
