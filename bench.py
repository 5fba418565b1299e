#!/usr/bin/env python3
"""bench.py -- device-resident SST block decode throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): per GPU, 1 GiB of SST data blocks cut at
4 KiB (16 B hex keys / 100 B ValueStruct payloads, 10 % ExpiresAt, 5 % value pointers), built
on the device by the gfx950 encoder and resident in HBM before timing.  One step = one
lsmgpu_decode_blocks_async over every block (materialize mode: key + value byte streams and
per-entry end offsets -- what Table.Iterator yields).  Multi-GPU: one process per GPU, each
decodes its own 1 GiB shard (weak scaling, no data-path collective).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--gib G] [--no-cpu]

Prints ONE JSON line (rank 0).  `roofline` is priced from the algorithmic bytes of the
decode kernel and its average duration measured with HIP events on the stream it runs on;
`cpu_baseline` times the C restatement of the reference decode (oracle/) on host cores.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "SST block decode GiB/s (device-resident), 4 KiB blocks, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def build_device_sst(codec, torch, dev, cfg: int, target_bytes: int, shard: int):
    """Synthetic columns (host numpy) -> device -> gfx950 encoder -> device-resident SST data
    blocks + device block offset/length arrays."""
    from lsmdb_amd import codec as C
    from lsmdb_amd import workload
    n = workload.entries_for_bytes(cfg, target_bytes)
    t0 = time.time()
    cols = workload.config_columns(cfg, n, seed_offset=shard)
    plan = C.plan_blocks(cols.key_end, cols.vs_end, cols.entries_per_block, cols.block_bytes)
    nblocks = plan.size - 1
    key_total, vs_total = int(cols.key_end[-1]), int(cols.vs_end[-1])
    data_len = 10 * n + key_total + vs_total + 13 * nblocks
    out_len = data_len + 4 * nblocks + 4
    d_keys = torch.from_numpy(cols.keys).to(dev)
    d_ke = torch.from_numpy(cols.key_end.view(np.int32)).to(dev)
    d_vs = torch.from_numpy(cols.vs).to(dev)
    d_ve = torch.from_numpy(cols.vs_end.view(np.int32)).to(dev)
    d_plan = torch.from_numpy(plan.view(np.int32)).to(dev)
    d_sst = torch.empty(out_len + 64, dtype=torch.uint8, device=dev)
    d_flags = torch.zeros(4, dtype=torch.int32, device=dev)
    codec.encode_device_async(d_keys, d_ke, d_vs, d_ve, n, key_total, vs_total, d_sst, d_flags,
                              entries_per_block=cols.entries_per_block, blk_first=d_plan,
                              nblocks=nblocks)
    codec.synchronize()
    if int(d_flags[0].item()) != 0:
        raise RuntimeError("encoder flagged invalid entries")
    idx = d_sst[data_len: data_len + 4 * nblocks].cpu().numpy()
    ends = idx.view(">u4").astype(np.uint32)
    offs = np.concatenate([[0], ends[:-1]]).astype(np.uint32)
    lens = (ends - offs).astype(np.uint32)
    assert int(ends[-1]) == data_len
    d_off = torch.from_numpy(offs.view(np.int32)).to(dev)
    d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    log(f"shard {shard}: {n} entries, {nblocks} blocks, {data_len} B data "
        f"(max block {int(lens.max())} B) built in {time.time() - t0:.1f}s")
    return dict(n=n, nblocks=nblocks, data_len=data_len, key_total=key_total, vs_total=vs_total,
                d_sst=d_sst, d_off=d_off, d_len=d_len, d_keys=d_keys, d_vs=d_vs, d_ke=d_ke,
                d_ve=d_ve, max_len=int(lens.max()), offs=offs, lens=lens, d_plan=d_plan,
                epb=cols.entries_per_block, out_len=out_len)


def time_encode(codec, torch, w, steps: int) -> dict:
    """The encoder (Builder.Add/finishBlock/blockIndex, table/builder.go:84-198) re-run over the
    same columns into a second buffer: HIP-event time per call, output checked byte-identical
    to the shard the decode benchmark reads.  Algorithmic bytes: keys + vs bytes + 2 x u32 end
    offsets per entry + plan, read; block image + index, written."""
    stream = torch.cuda.current_stream()
    d_out = torch.empty_like(w["d_sst"])
    d_flags = torch.zeros(4, dtype=torch.int32, device=w["d_sst"].device)
    run = lambda: codec.encode_device_async(w["d_keys"], w["d_ke"], w["d_vs"], w["d_ve"], w["n"],
                                            w["key_total"], w["vs_total"], d_out, d_flags,
                                            entries_per_block=w["epb"], blk_first=w["d_plan"],
                                            nblocks=w["nblocks"])
    run()
    ts = []
    for _ in range(steps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        run()
        b.record(stream)
        b.synchronize()
        ts.append(a.elapsed_time(b))
    n_out = w["out_len"]
    same = bool(torch.equal(d_out[:n_out], w["d_sst"][:n_out])) and int(d_flags[0].item()) == 0
    del d_out
    ms = float(np.median(ts))
    rd = w["key_total"] + w["vs_total"] + 8 * w["n"] + 4 * (w["nblocks"] + 1)
    wr = n_out
    gbs = (rd + wr) / (ms / 1e3) / 1e9
    return {"gibs_per_gpu": round(w["data_len"] / (ms / 1e3) / (1 << 30), 2), "kernel_ms": round(ms, 4),
            "achieved_gbs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
            "algorithmic_bytes": rd + wr, "identical_to_decoded_shard": same}


def _lib_sha256():
    import hashlib
    with open(os.path.join(ROOT, "lsmdb_amd", "liblsmgpu.so"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def algorithmic_bytes(w, mode: int) -> tuple[int, int]:
    """(read, write) bytes one decode launch must move."""
    read = w["data_len"] + 8 * w["nblocks"]            # block bytes + (off, len) per block
    write = 8 * w["nblocks"]                           # blk_first + blk_status
    if mode & 1:
        write += w["key_total"] + w["vs_total"] + 8 * w["n"]   # streams + 2 x u32 end offsets
    if mode & 2:
        write += 8 * w["n"]                            # u64 view record per entry
    return read, write


def time_decode(codec, torch, w, bufs, mode: int, steps: int, warmup: int, dist=None):
    stream = torch.cuda.current_stream()
    for _ in range(warmup):
        codec.decode_device_async(w["d_sst"], w["d_off"], w["d_len"], w["max_len"], mode, bufs,
                                  data_len=w["data_len"])
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        ev[i][0].record(stream)
        codec.decode_device_async(w["d_sst"], w["d_off"], w["d_len"], w["max_len"], mode, bufs,
                                  data_len=w["data_len"])
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kms = [a.elapsed_time(b) for a, b in ev]
    return wall, float(np.mean(kms)), float(np.median(kms))


def kernel_split(codec, w, bufs, mode: int, reps: int = 10):
    """Walk and copy durations of the walk-scan-copy decode, from HIP events the library records
    on its stream between its two launches (lsmgpu_kernel_times), outside the timed loop.  The
    copy's bytes: key + vs bytes read and written, u32 key_end + val_end per entry, blk_first +
    blk_status per block.  None when the batch takes another decode path."""
    walk, copy = [], []
    codec.set_kernel_timing(True)
    try:
        for _ in range(reps):
            codec.decode_device_async(w["d_sst"], w["d_off"], w["d_len"], w["max_len"], mode, bufs,
                                      data_len=w["data_len"])
            a, b = codec.kernel_times()
            walk.append(a)
            copy.append(b)
    except Exception:
        return None
    finally:
        codec.set_kernel_timing(False)
    wm, cm = float(np.mean(walk)), float(np.mean(copy))
    copy_bytes = 2 * (w["key_total"] + w["vs_total"]) + 8 * w["n"] + 8 * w["nblocks"]
    return {"walk_ms": round(wm, 4), "copy_ms": round(cm, 4),
            "walk_input_gbs": round(w["data_len"] / (wm / 1e3) / 1e9, 1),
            "copy_gbs": round(copy_bytes / (cm / 1e3) / 1e9, 1) if cm > 0 else None,
            "copy_algorithmic_bytes": copy_bytes,
            "source": "HIP events recorded by the library around its walk and copy launches"}


def device_copy_peak(torch, dev, nbytes: int, reps: int = 10) -> dict:
    """Practical HBM peak: a device-to-device copy of the decode's input size on
    the same stream, read + write bytes / time (median of `reps`)."""
    src = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    stream = torch.cuda.current_stream()
    for _ in range(2):
        dst.copy_(src)
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        dst.copy_(src)
        b.record(stream)
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ms = float(np.median(ts))
    del src, dst
    return {"kind": f"torch copy_ of {nbytes} B on the device (read + write)", "ms": round(ms, 4),
            "gbs": round(2 * nbytes / (ms / 1e3) / 1e9, 1)}


def check_round_trip(torch, w, bufs) -> str:
    """Full-size parity property: decode(encode(x)) == x for every byte and offset."""
    res = bufs.result.cpu().numpy()
    n, kb, vb = int(res[0]), int(res[1]), int(res[2])
    ok = (n == w["n"] and kb == w["key_total"] and vb == w["vs_total"] and res[5] == 0
          and int(res[4]) == 0)
    ok = ok and torch.equal(bufs.key_data[:kb], w["d_keys"]) and torch.equal(bufs.val_data[:vb], w["d_vs"])
    ok = ok and torch.equal(bufs.key_end[:n], w["d_ke"]) and torch.equal(bufs.val_end[:n], w["d_ve"])
    return "ok" if ok else "MISMATCH"


def reduce_over_ranks(dist, torch, dev, wall: float, parity: str,
                      shard_bytes: int) -> tuple[float, str, int]:
    """MAX of the timed wall clock, AND of the parity verdicts and SUM of the shard bytes over
    all ranks (the only collectives; the decode itself exchanges nothing)."""
    if dist is None:
        return wall, parity, shard_bytes
    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    p = torch.tensor([1.0 if parity == "ok" else 0.0], dtype=torch.float64, device=dev)
    dist.all_reduce(p, op=dist.ReduceOp.MIN)
    b = torch.tensor([shard_bytes], dtype=torch.int64, device=dev)
    dist.all_reduce(b, op=dist.ReduceOp.SUM)
    return float(t.item()), ("ok" if p.item() == 1.0 else "MISMATCH"), int(b.item())


def aggregate_gibs(total_bytes: int, ms_per_step: float) -> float:
    """Whole-job input GiB/s: the bytes all ranks decode per step / the slowest rank's step."""
    return total_bytes / (ms_per_step / 1e3) / (1 << 30)


def cpu_baseline(torch, w, seconds: float) -> dict:
    """The oracle (C restatement of blockIterator.Next/parseKV) on a bounded sample of the same
    blocks, multi-threaded over block ranges on the host cores."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi  # test infrastructure: the CPU baseline leg only
    sample = w["data_len"]  # the whole shard: larger than the host L3, no cache-resident inflation
    nb = int(np.searchsorted(w["offs"].astype(np.int64) + w["lens"], sample, side="right"))
    nb = max(nb, 1)
    end = int(w["offs"][nb - 1]) + int(w["lens"][nb - 1])
    host = w["d_sst"][:end].cpu().numpy()
    offs, lens = w["offs"][:nb], w["lens"][:nb]
    threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))
    t1, _ = oracle_ffi.decode_bench(host, offs, lens, threads, 1)
    reps = max(1, int(seconds / max(t1, 1e-3)))
    secs, _ = oracle_ffi.decode_bench(host, offs, lens, threads, reps)
    gibs = end * reps / secs / (1 << 30)
    s1, _ = oracle_ffi.decode_bench(host, offs, lens, 1, 1)
    reps1 = max(1, int(min(5.0, seconds / 2) / max(s1, 1e-3)))
    secs1, _ = oracle_ffi.decode_bench(host, offs, lens, 1, reps1)
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(gibs, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{end} B ({nb} blocks) of the same C2 blocks, x{reps} passes, "
                      f"{secs:.1f}s, materialize outputs; C restatement of "
                      f"table/iterator.go:93-135 (oracle/sstref.c)",
            "single_core_gibs": round(end * reps1 / secs1 / (1 << 30), 3),
            "cpu_model": cpu_model}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--gib", type=float, default=1.0, help="block bytes per GPU (GiB)")
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-view", action="store_true")
    args = ap.parse_args()

    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # rehearsal only (a one-GPU box): BENCH_DEVICE_OVERRIDE puts every rank on one device and
    # BENCH_DIST_BACKEND=gloo replaces RCCL, which refuses two ranks on one GPU
    if os.environ.get("BENCH_DEVICE_OVERRIDE"):
        local = int(os.environ["BENCH_DEVICE_OVERRIDE"])
    if world > 1:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            tdist.init_process_group(backend)
        dist = tdist
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local)

    from lsmdb_amd import workload
    from lsmdb_amd.codec import Codec, MODE_MATERIALIZE, MODE_VIEW
    codec = Codec(local)
    stream = torch.cuda.Stream(device=dev)  # a real (non-null) stream shared with the events
    torch.cuda.set_stream(stream)
    codec.set_stream(stream.cuda_stream)

    w = build_device_sst(codec, torch, dev, args.config, int(args.gib * (1 << 30)), rank)
    mode = MODE_MATERIALIZE
    bufs = codec.alloc_decode(w["data_len"], w["data_len"], w["nblocks"], mode, ent_cap=w["n"])
    wall, kms_mean, kms_med = time_decode(codec, torch, w, bufs, mode, args.steps, args.warmup, dist)
    parity = check_round_trip(torch, w, bufs)
    split = kernel_split(codec, w, bufs, mode)

    view = None
    if not args.no_view:
        vbufs = codec.alloc_decode(w["data_len"], 0, w["nblocks"], MODE_VIEW, ent_cap=w["n"])
        vwall, vk, _ = time_decode(codec, torch, w, vbufs, MODE_VIEW, args.steps, args.warmup, dist)
        vr, vw = algorithmic_bytes(w, MODE_VIEW)
        view = {"gibs_per_gpu": round(w["data_len"] / (vk / 1e3) / (1 << 30), 2),
                "kernel_ms": round(vk, 4), "achieved_gbs": round((vr + vw) / (vk / 1e3) / 1e9, 1),
                "frac": round((vr + vw) / (vk / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
        del vbufs

    practical = device_copy_peak(torch, dev, w["data_len"])
    encode = time_encode(codec, torch, w, min(args.steps, 10))

    wall, parity, total_bytes = reduce_over_ranks(dist, torch, dev, wall, parity, w["data_len"])

    ms_per_step = wall / args.steps * 1e3
    value = aggregate_gibs(total_bytes, ms_per_step)
    rd, wr = algorithmic_bytes(w, mode)
    achieved = (rd + wr) / (kms_mean / 1e3) / 1e9
    traffic = None
    tp = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tp):
        try:
            with open(tp) as f:
                tj = json.load(f)
            if (tj.get("workload_bytes") == w["data_len"] and tj.get("mode") == mode
                    and tj.get("lib_sha256") == _lib_sha256()):
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded; built on device by the gfx950 encoder)",
        "config": {
            "workload": f"C{args.config}: {w['data_len']} B of SST data blocks per GPU, "
                        f"{workload.DESCRIPTIONS[args.config]}, device-resident decode, "
                        f"{'materialize' if mode & 1 else 'view'} mode",
            "blocks_per_gpu": w["nblocks"],
            "entries_per_gpu": w["n"],
            "max_block_bytes": w["max_len"],
            "parallelism": f"{world} shard(s), one SST shard per GPU, no collective",
        },
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "algorithmic_bytes_per_launch": rd + wr, "kernel_ms_mean": round(kms_mean, 4),
                     "kernel_ms_median": round(kms_med, 4),
                     "practical_peak_gbs": practical["gbs"],
                     "frac_of_practical": round(achieved / practical["gbs"], 4),
                     "practical_peak_kind": practical["kind"],
                     "kernels": split},
        "parity": f"round-trip {parity} (decode(encode(x)) == x, all bytes and offsets)",
    }
    if view is not None:
        out["view_mode"] = view
    out["encode"] = encode
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(torch, w, args.cpu_seconds)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    codec.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
