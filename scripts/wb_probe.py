"""Does the previous decode's write-back slow the next walk?  C2 1 GiB materialize decodes,
kernel times from the library's HIP events (lsmgpu_kernel_times): back to back, vs each decode
after a synchronize and a 20 ms idle gap (the caches' dirty lines drained)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from lsmdb_amd.codec import Codec, MODE_MATERIALIZE  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    c = Codec(0)
    c.set_stream(s.cuda_stream)
    w = bench.build_device_sst(c, torch, dev, 2, 1 << 30, 0)
    b = c.alloc_decode(w["data_len"], w["data_len"], w["nblocks"], MODE_MATERIALIZE, ent_cap=w["n"])
    c.set_kernel_timing(True)

    def one():
        c.decode_device_async(w["d_sst"], w["d_off"], w["d_len"], w["max_len"], MODE_MATERIALIZE, b,
                              data_len=w["data_len"])
        return c.kernel_times()

    for _ in range(3):
        one()
    for label in ("back-to-back", "after idle", "back-to-back", "after idle"):
        walk, copy = [], []
        for _ in range(10):
            if label == "after idle":
                torch.cuda.synchronize()
                time.sleep(0.02)
            a, d = one()
            walk.append(a)
            copy.append(d)
        print(f"{label:13s} walk {np.mean(walk):.4f} ms  copy {np.mean(copy):.4f} ms", flush=True)


if __name__ == "__main__":
    main()
