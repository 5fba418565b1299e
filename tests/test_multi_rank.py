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
        w, parity, total, per = bench.reduce_over_ranks(dist, torch, torch.device("cpu"), wall,
                                                        "ok" if ok else "MISMATCH", data_len)
        assert per == [0.010, 0.020]
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
    assert bench.reduce_over_ranks(None, torch, None, 1.5, "ok", 123) == (1.5, "ok", 123, [1.5])


def test_bench_spawns_ranks_itself():
    """`python bench.py --gpus 2` (the driver's form without torch.distributed.run) starts two
    ranks from a parent that never touches the GPU; with --launcher-selftest the ranks do the
    real rank bookkeeping (gloo group, barriers, MAX / SUM / per-rank gather) around sleep
    steps, so n_gpus and the summed bytes are checked without a GPU."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps",
                          "5", "--launcher-selftest"], env=env, capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1                          # rank 0 prints ONE line
    assert out.stdout.strip() == lines[0]           # and nothing else: gloo's notices go to stderr
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["total_bytes"] == 2 << 30 and len(j["per_rank_ms"]) == 2
    assert j["parity"] == "ok" and j["metric"].startswith("launcher self-test")


def test_spawn_stops_ranks_when_one_fails(tmp_path):
    """A failing rank ends the job with its exit code instead of leaving the others waiting at
    a barrier (bench.spawn_ranks)."""
    import bench
    import time
    t0 = time.time()
    rc = bench.spawn_ranks(2, ["--gpus", "2", "--config", "9"])  # argparse rejects config 9
    assert rc != 0 and time.time() - t0 < 120


def test_c4_table_entries_matches_builder(oracle):
    """bench's C4 cut (one ReachedCapacity(cap) table per GPU) equals the oracle Builder driven
    like compactBuildTables' loop (levels.go:265-271), at small caps and the real 64 MiB."""
    import bench
    from lsmdb_amd import workload
    cols = workload.config_columns(4, 6000)
    L = oracle.lib()
    for cap in (1 << 14, 100_000, 300_000):
        b = L.sstref_builder_new(100, 0)
        i = 0
        while i < cols.n:
            if L.sstref_builder_reached_capacity(b, cap):
                break
            k0 = int(cols.key_end[i - 1]) if i else 0
            v0 = int(cols.vs_end[i - 1]) if i else 0
            k = cols.keys[k0: int(cols.key_end[i])].tobytes()
            v = cols.vs[v0: int(cols.vs_end[i])].tobytes()
            L.sstref_builder_add(b, k, len(k), v, len(v))
            i += 1
        L.sstref_builder_free(b)
        assert bench.c4_table_entries(cols.key_end, cols.vs_end, cap) == i
    big = workload.config_columns(4, 560_000)
    n = bench.c4_table_entries(big.key_end, big.vs_end, 64 << 20)
    # SURVEY 8 quotes 519,540 entries for fixed 129-B entries; the generator mixes in 15-B value
    # pointers and longer ExpiresAt varints, so a 64 MiB table holds a few % more
    assert 500_000 < n < 550_000 and n < big.n
