"""Premise test for overlapping the walk with the copy: two independent C2 1 GiB decodes
(materialize) on two codec contexts, back to back on one stream vs concurrently on two
streams.  Prints ms per decode for both."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from lsmdb_amd.codec import Codec, MODE_MATERIALIZE  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    ca, cb = Codec(0), Codec(0)
    torch.cuda.set_stream(s1)
    ca.set_stream(s1.cuda_stream)
    cb.set_stream(s1.cuda_stream)
    w = bench.build_device_sst(ca, torch, dev, 2, 1 << 30, 0)
    ba = ca.alloc_decode(w["data_len"], w["data_len"], w["nblocks"], MODE_MATERIALIZE, ent_cap=w["n"])
    bb = cb.alloc_decode(w["data_len"], w["data_len"], w["nblocks"], MODE_MATERIALIZE, ent_cap=w["n"])

    def run(c, b):
        c.decode_device_async(w["d_sst"], w["d_off"], w["d_len"], w["max_len"], MODE_MATERIALIZE, b,
                              data_len=w["data_len"])

    reps = 20
    for concurrent in (False, True, False, True):
        cb.set_stream((s2 if concurrent else s1).cuda_stream)
        for _ in range(3):
            run(ca, ba)
            run(cb, bb)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            run(ca, ba)
            run(cb, bb)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / (2 * reps)
        print(f"{'concurrent' if concurrent else 'sequential'}: {ms:.4f} ms per 1 GiB decode",
              flush=True)
    print("parity a", bench.check_round_trip(torch, w, ba), "b", bench.check_round_trip(torch, w, bb))


if __name__ == "__main__":
    main()
