"""Batched table open (lsmgpu_open_tables_async) timing: N C4 SSTs (ReachedCapacity 64 MiB,
100 entries/block) built on the device by the gfx950 encoder in one buffer, opened in one
call; HIP-event time (median of 20) beside the oracle restatement sstref_open_table run
table by table on the host (the reference does this per table with 64 goroutines + a sort).
Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    from lsmdb_amd import workload
    from lsmdb_amd import codec as C
    ntab = int(os.environ.get("TABLES", "8"))
    codec = C.Codec(0)
    dev = torch.device("cuda", 0)
    tail = np.frombuffer(b"{}" + (2).to_bytes(4, "big"), np.uint8)
    images, offs, lens, pos = [], [], [], 0
    for t in range(ntab):
        cols = workload.config_columns(4, 519540, seed_offset=t)
        plan = C.plan_blocks(cols.key_end, cols.vs_end, cols.entries_per_block, cols.block_bytes)
        nb = plan.size - 1
        kt, vt = int(cols.key_end[-1]), int(cols.vs_end[-1])
        n = cols.key_end.size
        data_len = 10 * n + kt + vt + 13 * nb
        out_len = data_len + 4 * nb + 4
        d_out = torch.empty(out_len + tail.size, dtype=torch.uint8, device=dev)
        flags = torch.zeros(4, dtype=torch.int32, device=dev)
        codec.encode_device_async(torch.from_numpy(cols.keys).to(dev),
                                  torch.from_numpy(cols.key_end.view(np.int32)).to(dev),
                                  torch.from_numpy(cols.vs).to(dev),
                                  torch.from_numpy(cols.vs_end.view(np.int32)).to(dev),
                                  n, kt, vt, d_out, flags, entries_per_block=cols.entries_per_block,
                                  blk_first=torch.from_numpy(plan.view(np.int32)).to(dev),
                                  nblocks=nb)
        codec.synchronize()
        d_out[out_len:] = torch.from_numpy(tail.copy()).to(dev)
        images.append(d_out)
        offs.append(pos)
        lens.append(d_out.numel())
        pos += d_out.numel()
    data = torch.cat(images)
    del images
    d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
    d_len = torch.tensor(lens, dtype=torch.int64, device=dev)
    blk_cap = sum(n // 13 for n in lens)
    torch.cuda.synchronize()
    stream = torch.cuda.Stream(device=dev)  # a real stream shared by the codec and the events
    torch.cuda.set_stream(stream)           # (handle 0 would select the codec's own stream)
    codec.set_stream(stream.cuda_stream)
    o = codec.open_tables_device(data, d_off, d_len, blk_cap)
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        o = codec.open_tables_device(data, d_off, d_len, blk_cap)
        b.record(stream)
        b.synchronize()
        ts.append(a.elapsed_time(b))
    st = o["status"].cpu().numpy()
    nblk = int(o["result"][0].item())
    ms = float(np.median(ts))
    # CPU: the oracle, table by table (single thread), on the same images
    import oracle_ffi
    oracle_ffi.lib()
    host = data.cpu().numpy()
    t0 = time.perf_counter()
    ok = True
    for t in range(ntab):
        ref = oracle_ffi.open_table(host[offs[t]: offs[t] + lens[t]].tobytes(), cap=1 << 16)
        ok = ok and ref["status"] == int(st[t]) and ref["nblk"] == int(o["nblk"][t].item())
    cpu_s = time.perf_counter() - t0
    print(json.dumps({"what": "batched table open (OpenTable index work)", "tables": ntab,
                      "table_bytes": lens[0], "blocks": nblk, "gpu_ms": round(ms, 4),
                      "tables_per_s": round(ntab / (ms / 1e3), 1),
                      "cpu_oracle_ms_total": round(cpu_s * 1e3, 2),
                      "cpu_kind": "oracle sstref_open_table, 1 thread, incl. Python FFI and a "
                                  "copy of each table",
                      "statuses": [int(x) for x in st], "matches_oracle": ok}))
    codec.close()


if __name__ == "__main__":
    main()
