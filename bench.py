#!/usr/bin/env python3
"""bench.py -- device-resident SST block decode throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], SURVEY 8(d) C2, the default): per GPU, 1 GiB of SST data
blocks cut at 4 KiB (16 B hex keys / 100 B ValueStruct payloads, 10 % ExpiresAt, 5 % value
pointers), built on the device by the gfx950 encoder and resident in HBM before timing.  One
step = one lsmgpu_decode_blocks_async over every block (materialize mode: key + value byte
streams and per-entry end offsets -- what Table.Iterator yields).

Other configs (parity-test shapes, also measurable): --config 3 (64 B / 1 KiB entries),
--config 4 (ONE 64 MiB SST per GPU, cut where Builder.ReachedCapacity(64 MiB) stops, 100 entries
per block: the per-GPU unit of the 8-SST compaction replay), --config 5 (Zipf keys, 32 KiB
blocks; the 1/2/4/8 scaling curve is `--gpus N` for N = 1, 2, 4, 8).

Multi-GPU: one process per GPU, each decoding its own shard (no exchange, no
data-path collective; weak scaling).  `python bench.py --gpus N` spawns the N ranks itself from
a parent that never touches the GPU; under `torch.distributed.run` (WORLD_SIZE set) the process
is one rank.  Barrier + synchronize bracket the timed steps; the wall time is the MAX over
ranks and `value` = all ranks' input bytes / that time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C] [--gib G] [--no-cpu]

Prints ONE JSON line (rank 0).  `roofline` is priced from the algorithmic bytes of the decode
and its average duration measured with HIP events on the stream it runs on; practical ceilings
come from the library's own streaming copy / read kernels (lsmgpu_stream_probe_async);
`cpu_baseline` times the C restatement of the reference decode (oracle/) on the host cores.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import tempfile
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "SST block decode GiB/s (device-resident), 4 KiB blocks, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
C4_TABLE_CAP = 64 << 20  # options.go:80 MaxTableSize, the ReachedCapacity cap (levels.go:269)


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


# ------------------------------------------------------------------ launcher (no GPU here)
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv: list[str], timeout_s: float = 1800.0) -> int:
    """Start n copies of this script as ranks 0..n-1 (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_*), one per GPU, and wait for all of them.  The parent never initialises HIP (a
    process that did must not exec or fork GPU children).  If one rank fails the others are
    stopped (they would wait at a barrier forever).  Returns the worst exit code."""
    port = _free_port()
    procs = []
    # rank 0's stdout goes to a file and only its JSON line is forwarded to ours: the process
    # group libraries print connection notices on stdout (gloo does), and the driver reads ONE
    # JSON line.  Every other rank's stdout joins stderr.
    out0 = tempfile.TemporaryFile(mode="w+")
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=out0 if r == 0 else sys.stderr))
    try:
        return _wait_ranks(procs, timeout_s)
    finally:
        out0.seek(0)
        for line in out0:
            if line.lstrip().startswith("{"):
                sys.stdout.write(line)
            else:
                sys.stderr.write(line)
        sys.stdout.flush()
        out0.close()


def _wait_ranks(procs: list, timeout_s: float) -> int:
    t0, rc = time.time(), 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0:
                rc = max(rc, abs(code))
                for q in live:
                    q.terminate()
        if time.time() - t0 > timeout_s:
            for q in live:
                q.kill()
            return 124
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc


# ------------------------------------------------------------------ workloads
def c4_table_entries(key_end: np.ndarray, vs_end: np.ndarray, cap: int, epb: int = 100) -> int:
    """Entries in the first table of the compaction loop (levels.go:265-271): entry i is added
    while ReachedCapacity(cap) is false before it, i.e. buf.Len() + 8 + 4 * len(restarts) + 8
    <= cap (table/builder.go:140-143) with buf.Len() = 10 e + keys + vs + 13 (e - 1) // epb."""
    e = np.arange(1, key_end.size + 1, dtype=np.int64)
    fb = (e - 1) // epb
    est = 10 * e + key_end.astype(np.int64) + vs_end.astype(np.int64) + 13 * fb + 8 + 4 * fb + 8
    over = np.nonzero(est > cap)[0]
    # est[i-1] is the estimate after i entries, i.e. the check before entry i
    return int(over[0]) + 1 if over.size else int(key_end.size)


def build_device_sst(codec, torch, dev, cfg: int, target_bytes: int, shard: int):
    """Synthetic columns (host numpy) -> device -> gfx950 encoder -> device-resident SST data
    blocks + device block offset/length arrays."""
    from lsmdb_amd import codec as C
    from lsmdb_amd import workload
    t0 = time.time()
    if cfg == 4:  # one ReachedCapacity(64 MiB)-cut SST per GPU
        cols = workload.config_columns(4, 560_000, seed_offset=shard)
        n = c4_table_entries(cols.key_end, cols.vs_end, C4_TABLE_CAP)
        kt, vt = int(cols.key_end[n - 1]), int(cols.vs_end[n - 1])
        cols = workload.Columns(cols.keys[:kt], cols.key_end[:n], cols.vs[:vt], cols.vs_end[:n],
                                cols.entries_per_block, cols.block_bytes)
    else:  # at least target_bytes of block data: generated long, trimmed at the exact size
        n = workload.entries_for_bytes(cfg, target_bytes)
        cols = workload.config_columns(cfg, n, seed_offset=shard)
        plan = C.plan_blocks(cols.key_end, cols.vs_end, cols.entries_per_block, cols.block_bytes)
        cols = workload.trim_to_bytes(cols, plan, target_bytes)
        n = cols.n
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


# ------------------------------------------------------------------ measurements
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
    """The timed region: exactly `steps` decodes enqueued back to back between a barrier +
    synchronize on each side (wall clock, max over ranks by the caller).  Per-decode HIP-event
    times come from a second, untimed pass of the same decodes, so the timed region holds no
    event records between the steps (they cost ~7 us per step: C4 0.067 vs 0.060 ms)."""
    stream = torch.cuda.current_stream()

    def one():
        codec.decode_device_async(w["d_sst"], w["d_off"], w["d_len"], w["max_len"], mode, bufs,
                                  data_len=w["data_len"])
    for _ in range(warmup):
        one()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    for i in range(steps):
        ev[i][0].record(stream)
        one()
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    kms = [a.elapsed_time(b) for a, b in ev]
    return wall, float(np.mean(kms)), float(np.median(kms))


def walk_fetch_bytes(torch, w, view, blk_first) -> int:
    """The bytes the walk must fetch from HBM: every 128-B line holding one of the 8-B header
    reads it makes -- each entry's header and each block's stop header (the terminator, or the
    header it stops at), iterator.go:112-135.  Computed from a view decode's records (key
    position, klen, vlen per entry) and the block list, on the device.  For C2's 129-B entries
    this is every line of the input; for C3's 1,101-B entries about 4 lines of a block's 26."""
    n = int(blk_first[-1].item())
    bf = blk_first.to(torch.int64)
    # a wrong decode must raise here, not fault the queue in the gathers below
    if (n != w.get("n", n) or n > view.numel() or int(bf[0].item()) != 0
            or bool((bf[1:] < bf[:-1]).any().item())):
        raise RuntimeError(f"view decode returned an invalid block index (n={n}, expected {w.get('n')})")
    v = view[:n].to(torch.int64)
    kp = v & 0xFFFFFFFF
    kl = (v >> 32) & 0xFFFF
    vl = (v >> 48) & 0xFFFF
    heads = [kp - 10]
    cnt = bf[1:] - bf[:-1]
    off = w["d_off"].to(torch.int64) & 0xFFFFFFFF
    ln = w["d_len"].to(torch.int64) & 0xFFFFFFFF
    last = torch.clamp(bf[1:] - 1, min=0)
    stop = torch.where(cnt > 0, kp[last] + kl[last] + vl[last] if n else off, off)
    heads.append(stop[stop + 10 <= off + ln])  # a header read only where 10 bytes remain
    h = torch.cat(heads)
    lines = torch.unique(torch.cat([h >> 7, (h + 7) >> 7]))
    return int(lines.numel()) * 128


def kernel_split(codec, w, bufs, mode: int, reps: int = 10, fetch: int = 0):
    """Walk and copy durations of the walk-scan-copy decode, from HIP events the library records
    on its stream between its two launches (lsmgpu_kernel_times), outside the timed loop.  The
    copy's bytes: key + vs bytes read and written, u32 key_end + val_end per entry, blk_first +
    blk_status per block.  None only when the batch takes another decode path (the library
    answers LSMGPU_ERR_ARG: the decode recorded no kernel times); other errors propagate."""
    from lsmdb_amd import _lib
    walk, copy = [], []
    codec.set_kernel_timing(True)
    try:
        for _ in range(reps):
            codec.decode_device_async(w["d_sst"], w["d_off"], w["d_len"], w["max_len"], mode, bufs,
                                      data_len=w["data_len"])
            try:
                a, b = codec.kernel_times()
            except _lib.LsmgpuError as e:
                if e.code == _lib.ERR_ARG:
                    return None
                raise
            walk.append(a)
            copy.append(b)
    finally:
        codec.set_kernel_timing(False)
    wm, cm = float(np.mean(walk)), float(np.mean(copy))
    copy_bytes = 2 * (w["key_total"] + w["vs_total"]) + 8 * w["n"] + 8 * w["nblocks"]
    walk_bytes = fetch + 8 * w["nblocks"]  # header lines + (off, len) per block
    return {"walk_ms": round(wm, 4), "copy_ms": round(cm, 4),
            # the input rate (bytes of blocks walked / time): NOT a roofline fraction
            "walk_input_gbs": round(w["data_len"] / (wm / 1e3) / 1e9, 1),
            # roofline: the lines the walk must fetch (walk_fetch_bytes) / time / peak
            "walk_fetch_bytes": walk_bytes,
            "walk_read_frac": round(walk_bytes / (wm / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "copy_gbs": round(copy_bytes / (cm / 1e3) / 1e9, 1) if cm > 0 else None,
            "copy_frac": round(copy_bytes / (cm / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if cm > 0 else None,
            "copy_algorithmic_bytes": copy_bytes,
            "source": "HIP events recorded by the library around its walk and copy launches"}


def practical_peaks(codec, torch, dev, nbytes: int, reps: int = 7) -> dict:
    """Practical HBM ceilings from the library's own 16-B-per-lane streaming
    kernels over nbytes (the decode's input size): the best copy (read + write bytes / time)
    and the best pure read over default / non-temporal policies and 2-16 workgroups per CU
    (median of `reps` each), HIP events on the codec's stream."""
    nbytes = nbytes // 16 * 16
    src = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    src.random_(0, 255)
    dst = torch.empty_like(src)
    stream = torch.cuda.current_stream()
    best = {}
    kinds = ((0, "copy", 2), (2, "copy_nt", 2), (4, "copy_u16", 2), (6, "copy_nt_u16", 2),
             (1, "read", 1), (3, "read_nt", 1), (5, "read_u16", 1), (7, "read_nt_u16", 1))
    for kind, name, mult in kinds:
        for wg in (2, 4, 8, 16):
            codec.stream_probe_async(kind, src, dst, nbytes, wg)
            ts = []
            for _ in range(reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                codec.stream_probe_async(kind, src, dst, nbytes, wg)
                b.record(stream)
                b.synchronize()
                ts.append(a.elapsed_time(b))
            gbs = mult * nbytes / (float(np.median(ts)) / 1e3) / 1e9
            fam = "read" if kind & 1 else "copy"
            if gbs > best.get(fam, (0,))[0]:
                best[fam] = (gbs, f"{name}, {wg} workgroups/CU")
    del src, dst
    return {"copy_gbs": round(best["copy"][0], 1), "copy_kind": best["copy"][1],
            "read_gbs": round(best["read"][0], 1), "read_kind": best["read"][1],
            "bytes": nbytes, "source": "lsmgpu_stream_probe_async (csrc/probe.hip), best of "
                                       "default / nt policies, 4 or 16 16-B loads in flight per "
                                       "lane, 2-16 workgroups per CU"}


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
                      shard_bytes: int) -> tuple[float, str, int, list]:
    """MAX of the timed wall clock, AND of the parity verdicts, SUM of the shard bytes and every
    rank's wall time (the only collectives; the decode itself exchanges nothing)."""
    if dist is None:
        return wall, parity, shard_bytes, [wall]
    world = dist.get_world_size()
    w = torch.tensor([wall], dtype=torch.float64, device=dev)
    walls = [torch.zeros(1, dtype=torch.float64, device=dev) for _ in range(world)]
    dist.all_gather(walls, w)
    p = torch.tensor([1.0 if parity == "ok" else 0.0], dtype=torch.float64, device=dev)
    dist.all_reduce(p, op=dist.ReduceOp.MIN)
    b = torch.tensor([shard_bytes], dtype=torch.int64, device=dev)
    dist.all_reduce(b, op=dist.ReduceOp.SUM)
    per = [float(x.item()) for x in walls]
    return max(per), ("ok" if p.item() == 1.0 else "MISMATCH"), int(b.item()), per


def aggregate_gibs(total_bytes: int, ms_per_step: float) -> float:
    """Whole-job input GiB/s: the bytes all ranks decode per step / the slowest rank's step."""
    return total_bytes / (ms_per_step / 1e3) / (1 << 30)


def host_cores() -> dict:
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU quota if any
    (on the GPU box os.cpu_count() shows the whole machine, not this job's share)."""
    nproc = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        quota = None
    used = min(aff, quota) if quota else aff
    return {"nproc": nproc, "affinity": aff, "cgroup_quota": quota, "used": used}


def cpu_baseline(torch, w, seconds: float) -> dict:
    """The oracle (C restatement of blockIterator.Next/parseKV) on a bounded sample of the same
    blocks, multi-threaded over block ranges on every host core this job may use."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi  # test infrastructure: the CPU baseline leg only
    sample = w["data_len"]  # the whole shard: larger than the host L3, no cache-resident inflation
    nb = int(np.searchsorted(w["offs"].astype(np.int64) + w["lens"], sample, side="right"))
    nb = max(nb, 1)
    end = int(w["offs"][nb - 1]) + int(w["lens"][nb - 1])
    host = w["d_sst"][:end].cpu().numpy()
    offs, lens = w["offs"][:nb], w["lens"][:nb]
    cores = host_cores()
    threads = cores["used"]
    t1, _ = oracle_ffi.decode_bench(host, offs, lens, threads, 1)
    reps = max(1, int(seconds / max(t1, 1e-3)))
    secs, _ = oracle_ffi.decode_bench(host, offs, lens, threads, reps)
    gibs = end * reps / secs / (1 << 30)
    # thread scaling (1, 4, 16 threads and every core this job may use), ~3 s each: says whether
    # the port is bound by cores or by the host's memory bandwidth
    scaling = {}
    for t in sorted({1, 4, 16, threads}):
        if t > threads:
            continue
        st, _ = oracle_ffi.decode_bench(host, offs, lens, t, 1)
        rt = max(1, int(min(3.0, seconds / 4) / max(st, 1e-3)))
        secs_t, _ = oracle_ffi.decode_bench(host, offs, lens, t, rt)
        scaling[str(t)] = round(end * rt / secs_t / (1 << 30), 3)
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
            "sample": f"{end} B ({nb} blocks) of the same blocks, x{reps} passes, "
                      f"{secs:.1f}s, materialize outputs; C restatement of "
                      f"table/iterator.go:93-135 (oracle/sstref.c)",
            "single_core_gibs": scaling["1"], "threads_gibs": scaling,
            "host_cpus": cores, "cpu_model": cpu_model}


def _traffic(w, mode: int):
    """HBM bytes per launch from the committed PMC summary, if it describes this library and
    workload (profiles/pmc_traffic.json, scripts/profile_round.sh)."""
    tp = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(tp):
        return None
    try:
        with open(tp) as f:
            tj = json.load(f)
    except (OSError, ValueError):
        return None
    if (tj.get("workload_bytes") == w["data_len"] and tj.get("mode") == mode
            and tj.get("lib_sha256") == _lib_sha256()):
        return tj.get("hbm_bytes_per_launch")
    return None


# ------------------------------------------------------------------ one rank
def launcher_selftest(args, rank: int, world: int) -> None:
    """--launcher-selftest (CPU, tests only): the rank bookkeeping of a real run -- gloo process
    group, barrier-bracketed timed loop, MAX / SUM over ranks -- with a 1 ms sleep as the step
    and no GPU work.  Its line says so in `metric`; it is never a measurement."""
    import torch
    import torch.distributed as tdist
    tdist.init_process_group("gloo")
    shard = 1 << 30
    tdist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.001)
    tdist.barrier()
    wall = time.perf_counter() - t0
    wall, parity, total, per = reduce_over_ranks(tdist, torch, torch.device("cpu"), wall, "ok", shard)
    if rank == 0:
        ms = wall / args.steps * 1e3
        print(json.dumps({"metric": "launcher self-test (no GPU work: sleep steps)",
                          "value": round(aggregate_gibs(total, ms), 3), "unit": "GiB/s",
                          "n_gpus": world, "steps": args.steps, "total_bytes": total,
                          "per_rank_ms": [round(x / args.steps * 1e3, 4) for x in per],
                          "parity": parity}), flush=True)
    tdist.destroy_process_group()


def run_rank(args) -> None:
    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launcher_selftest:
        return launcher_selftest(args, rank, world)
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
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    coll_dev = dev if (dist is not None and os.environ.get("BENCH_DIST_BACKEND", "nccl") == "nccl") \
        else torch.device("cpu")

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

    # the lines the walk must fetch, from one view decode's records (outside any timed region)
    vbufs = codec.alloc_decode(w["data_len"], 0, w["nblocks"], MODE_VIEW, ent_cap=w["n"])
    codec.decode_device_async(w["d_sst"], w["d_off"], w["d_len"], w["max_len"], MODE_VIEW, vbufs,
                              data_len=w["data_len"])
    torch.cuda.synchronize()
    fetch = walk_fetch_bytes(torch, w, vbufs.view, vbufs.blk_first)
    split = kernel_split(codec, w, bufs, mode, fetch=fetch)

    view = None
    if not args.no_view:
        vwall, vk, _ = time_decode(codec, torch, w, vbufs, MODE_VIEW, args.steps, args.warmup, dist)
        _, vw = algorithmic_bytes(w, MODE_VIEW)
        vread = fetch + 8 * w["nblocks"]  # the header lines + (off, len) per block
        view = {"gibs_per_gpu": round(w["data_len"] / (vk / 1e3) / (1 << 30), 2),
                "kernel_ms": round(vk, 4),
                "achieved_gbs": round((vread + vw) / (vk / 1e3) / 1e9, 1),
                "frac": round((vread + vw) / (vk / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                # the north star's HBM-read roofline: the bytes view mode must fetch (every
                # 128-B line holding a header) / kernel time / 8 TB/s
                "read_frac": round(fetch / (vk / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                "fetch_bytes": fetch,
                "input_gbs": round(w["data_len"] / (vk / 1e3) / 1e9, 1)}
    del vbufs

    practical = None if args.no_peaks else practical_peaks(codec, torch, dev, w["data_len"])
    if view is not None and practical is not None:
        view["read_frac_of_practical"] = round(
            fetch / (view["kernel_ms"] / 1e3) / 1e9 / practical["read_gbs"], 4)
    encode = time_encode(codec, torch, w, min(args.steps, 10))

    wall, parity, total_bytes, per_rank = reduce_over_ranks(dist, torch, coll_dev, wall, parity,
                                                            w["data_len"])

    ms_per_step = wall / args.steps * 1e3
    value = aggregate_gibs(total_bytes, ms_per_step)
    rd, wr = algorithmic_bytes(w, mode)
    achieved = (rd + wr) / (kms_mean / 1e3) / 1e9
    traffic = _traffic(w, mode)
    cfg_name = {2: "configs[1]", 3: "configs[2]", 4: "configs[3] per-GPU unit", 5: "configs[4]"}
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "per_rank_ms": [round(x / args.steps * 1e3, 4) for x in per_rank],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded; built on device by the gfx950 encoder)",
        "config": {
            "workload": f"C{args.config} ({cfg_name.get(args.config, 'config')}): "
                        f"{w['data_len']} B of SST data blocks per GPU, "
                        f"{workload.DESCRIPTIONS[args.config]}, device-resident decode, "
                        f"{'materialize' if mode & 1 else 'view'} mode",
            "blocks_per_gpu": w["nblocks"],
            "entries_per_gpu": w["n"],
            "max_block_bytes": w["max_len"],
            "parallelism": f"{world} shard(s), one SST shard per GPU, no collective",
        },
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_ratio": round(traffic / (rd + wr), 4) if traffic else None,
                     "algorithmic_bytes_per_launch": rd + wr, "kernel_ms_mean": round(kms_mean, 4),
                     "kernel_ms_median": round(kms_med, 4),
                     "practical_copy_gbs": practical["copy_gbs"] if practical else None,
                     "frac_of_practical": round(achieved / practical["copy_gbs"], 4)
                     if practical else None,
                     "practical": practical,
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


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--gib", type=float, default=1.0, help="block bytes per GPU (GiB); C4 ignores it")
    ap.add_argument("--config", type=int, default=2, choices=(2, 3, 4, 5))
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-view", action="store_true")
    ap.add_argument("--no-peaks", action="store_true", help="skip the practical-peak probes "
                    "(profiling passes); frac_of_practical is then null")
    ap.add_argument("--launcher-selftest", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU, started before anything touches the GPU
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    run_rank(args)


if __name__ == "__main__":
    main()
