"""Diagnostic (diag build, LSMGPU_WSC_LBIDIR=1 LSMGPU_ABLATE=1024): how many C5 blocks' forward
and backward walks met, and the mean walk-loop steps per wave, against the entries per block."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from lsmdb_amd.codec import Codec, MODE_MATERIALIZE
    dev = torch.device("cuda", 0)
    codec = Codec(0)
    w = bench.build_device_sst(codec, torch, dev, 5, 1 << 30, 0)
    bufs = codec.alloc_decode(w["data_len"], w["data_len"], w["nblocks"], MODE_MATERIALIZE, ent_cap=w["n"])
    codec.decode_device_async(w["d_sst"], w["d_off"], w["d_len"], w["max_len"], MODE_MATERIALIZE, bufs,
                              data_len=w["data_len"])
    codec.synchronize()
    r = bufs.result.cpu().numpy()
    waves = (w["nblocks"] + 31) // 32
    print({"blocks": w["nblocks"], "entries": int(r[0]), "met": int(r[6]),
           "mean_steps_per_wave": float(r[7]) / waves, "entries_per_block": int(r[0]) / w["nblocks"]})
    codec.close()


if __name__ == "__main__":
    main()
