"""Probe (GPU box): the materialize decode of the C2 1 GiB shard cut into K consecutive chunks
decoded back to back on one stream (each chunk = walk + copy launch; bases not chained, so
outputs overlap -- timing only).  With small chunks the copy re-reads lines its walk has just
pulled through the 256 MiB Infinity Cache; the per-chunk walk / copy split shows what that buys
and what the walk loses with fewer lanes in flight.  Prints one JSON line per K.

    python scripts/chunk_probe.py [--ks 1,2,4,8,16] [--reps 5]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ks", default="1,2,4,8,16")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cfg", type=int, default=2)
    args = ap.parse_args()
    import torch
    import bench
    from lsmdb_amd.codec import Codec, MODE_MATERIALIZE
    dev = torch.device("cuda", 0)
    codec = Codec(0)
    w = bench.build_device_sst(codec, torch, dev, args.cfg, 1 << 30, 0)
    nblk, data_len = w["nblocks"], w["data_len"]
    bufs = codec.alloc_decode(data_len, data_len, nblk, MODE_MATERIALIZE, ent_cap=w["n"])
    for k in [int(x) for x in args.ks.split(",")]:
        cuts = [nblk * i // k for i in range(k + 1)]

        def run():
            for i in range(k):
                a, b = cuts[i], cuts[i + 1]
                codec.decode_device_async(w["d_sst"], w["d_off"][a:b], w["d_len"][a:b], w["max_len"],
                                          MODE_MATERIALIZE, bufs, data_len=data_len)
        run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        # per-chunk kernel split (synchronizes after each chunk)
        codec.set_kernel_timing(True)
        walk = copy = 0.0
        for i in range(k):
            a, b = cuts[i], cuts[i + 1]
            codec.decode_device_async(w["d_sst"], w["d_off"][a:b], w["d_len"][a:b], w["max_len"],
                                      MODE_MATERIALIZE, bufs, data_len=data_len)
            x, y = codec.kernel_times()
            walk += x
            copy += y
        codec.set_kernel_timing(False)
        res = bufs.result.cpu().numpy()
        print(json.dumps({"chunks": k, "ms_median": round(float(np.median(ts)), 4),
                          "gibs": round(data_len / (float(np.median(ts)) * 1e-3) / (1 << 30), 1),
                          "walk_ms_sum": round(walk, 4), "copy_ms_sum": round(copy, 4),
                          "last_chunk_flags": int(res[5])}), flush=True)
    codec.close()


if __name__ == "__main__":
    main()
