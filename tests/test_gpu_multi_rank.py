"""bench.py's multi-GPU path with the HIP library in every rank: world
size 2 over gloo, each rank on device rank % device_count (both on device 0 on a one-GPU box),
each rank builds its OWN shard with the gfx950 encoder (bench.build_device_sst, seeded per
rank), decodes it device-resident through the C ABI and checks the decode against the oracle
(the checker); the reduction (max wall, parity AND, byte sum) is bench.reduce_over_ranks.  No
data path collective: shards are independent."""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, q):
    sys.path[:0] = [ROOT, HERE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import oracle_ffi as ofi
        from lsmdb_amd.codec import Codec, MODE_MATERIALIZE
        dev_i = rank % torch.cuda.device_count()
        torch.cuda.set_device(dev_i)
        dev = torch.device("cuda", dev_i)
        with Codec(dev_i) as codec:
            w = bench.build_device_sst(codec, torch, dev, 2, 24 << 20, rank)  # ~6,000 blocks
            bufs = codec.alloc_decode(w["data_len"], w["data_len"], w["nblocks"], MODE_MATERIALIZE,
                                      ent_cap=w["n"])
            codec.decode_device_async(w["d_sst"], w["d_off"], w["d_len"], w["max_len"],
                                      MODE_MATERIALIZE, bufs, data_len=w["data_len"])
            codec.synchronize()
            n, kt, vt = w["n"], w["key_total"], w["vs_total"]
            sst = w["d_sst"][: w["data_len"]].cpu().numpy().tobytes()
            ref = ofi.decode(sst, w["offs"], w["lens"])
            ok = (ref.n_entries == n and
                  bufs.key_data[:kt].cpu().numpy().tobytes() == ref.key_data.tobytes() and
                  bufs.val_data[:vt].cpu().numpy().tobytes() == ref.val_data.tobytes() and
                  np.array_equal(bufs.key_end[:n].cpu().numpy().view(np.uint32), ref.key_end) and
                  np.array_equal(bufs.val_end[:n].cpu().numpy().view(np.uint32), ref.val_end) and
                  np.array_equal(bufs.blk_first.cpu().numpy().view(np.uint32), ref.blk_first))
            first_key = bufs.key_data[:16].cpu().numpy().tobytes()
            wall = 0.010 * (rank + 1)
            wmax, parity, total, per = bench.reduce_over_ranks(dist, torch, torch.device("cpu"), wall,
                                                               "ok" if ok else "MISMATCH", w["data_len"])
            q.put((rank, wmax, parity, total, w["data_len"], first_key, dev_i))
    finally:
        dist.destroy_process_group()


def test_two_rank_hip_decode_gloo():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=110) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert {r[1] for r in res} == {0.020}             # max wall over ranks, seen by every rank
    assert all(r[2] == "ok" for r in res)             # every rank's HIP decode == oracle
    assert all(r[3] == res[0][4] + res[1][4] for r in res)
    assert res[0][5] != res[1][5]                     # each rank decoded its own shard
