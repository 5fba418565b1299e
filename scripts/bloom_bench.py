"""Bloom tail timing (csrc/bloom.hip) at one C4 64 MiB table: 519,540 keys -> a 2^23-bit
filter + its 1.4 MB JSON (Builder.Finish, table/builder.go:164-195), and a batch of 1 M
DoesNotHave probes (table.go:301).  HIP events on the codec's stream; the oracle restatement
(oracle/bbloom.c, one core) is timed beside it.  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from lsmdb_amd import workload  # noqa: E402
from lsmdb_amd.codec import Codec  # noqa: E402
import oracle_ffi as oracle  # noqa: E402  (the checker / CPU baseline only)


def main():
    n, nq, reps = 519540, 1 << 20, 20
    if len(sys.argv) > 1 and sys.argv[1] == "distinct":  # 16-B random user keys + 8-B ts
        rng = np.random.default_rng(3)
        kb = rng.integers(0, 256, n * 24, dtype=np.uint8).tobytes()
        ke = (np.arange(1, n + 1, dtype=np.uint64) * 24).astype(np.uint32)
        label = "distinct keys: 519,540 random 16-B user keys + 8-B ts"
    else:  # C4's BenchmarkRead keys: ParseKey keeps "00000000" for every key
        c = workload.config_columns(4, n, 4)
        kb, ke = c.keys.tobytes(), c.key_end
        label = "C4 keys (16-B hex, no ts: one distinct ParseKey)"
    codec = Codec(0)
    dev = torch.device("cuda", 0)
    kd = torch.from_numpy(np.frombuffer(kb + b"\0" * 16, np.uint8).copy()).to(dev)
    ked = torch.from_numpy(ke.view(np.int32).copy()).to(dev)
    s = torch.cuda.ExternalStream(codec.stream_handle())
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(3):
        o = codec.bloom_build_device(kd, ked, n)
    codec.synchronize()
    ev[0].record(s)
    for _ in range(reps):
        o = codec.bloom_build_device(kd, ked, n)
    ev[1].record(s)
    codec.synchronize()
    build_ms = ev[0].elapsed_time(ev[1]) / reps
    bs, bits, locs, ex = oracle.bloom_build(kb, ke)
    ok = np.array_equal(o["bitset"].cpu().numpy().view(np.uint64), bs)
    # probes: the table's keys without ts, then absent keys (half / half)
    rng = np.random.default_rng(9)
    qlen = np.full(nq, 8, np.int64)
    qb = rng.integers(0, 256, int(qlen.sum()), dtype=np.uint8)
    qe = np.cumsum(qlen).astype(np.uint32)
    qd = torch.from_numpy(np.concatenate([qb, np.zeros(16, np.uint8)])).to(dev)
    qed = torch.from_numpy(qe.view(np.int32).copy()).to(dev)
    for _ in range(3):
        has = codec.bloom_has_device(o["bitset"], bits, locs, qd, qed, nq)
    codec.synchronize()
    ev[0].record(s)
    for _ in range(reps):
        has = codec.bloom_has_device(o["bitset"], bits, locs, qd, qed, nq)
    ev[1].record(s)
    codec.synchronize()
    has_ms = ev[0].elapsed_time(ev[1]) / reps
    t0 = time.perf_counter()
    oracle.bloom_build(kb, ke)
    js = oracle.bloom_json(bs, bits, locs)
    cpu_ms = (time.perf_counter() - t0) * 1e3
    print(json.dumps({
        "what": "bloom tail at one C4 64 MiB table (519,540 keys, 2^23-bit filter)", "keys": label,
        "build_json_ms": round(build_ms, 4), "keys_per_s": round(n / build_ms * 1e3),
        "json_bytes": len(js), "bit_exact": bool(ok),
        "probe_ms_1M": round(has_ms, 4), "probes_per_s": round(nq / has_ms * 1e3),
        "cpu_oracle_build_json_ms_1core": round(cpu_ms, 2)}))


if __name__ == "__main__":
    main()
