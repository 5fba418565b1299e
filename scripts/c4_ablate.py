"""Walk / copy kernel times under timing-only ablations (LSMGPU_ABLATE: 1 no look-back,
2 no copy / no view records, 4 no walk, 128 / 256 no record flush, with 2 only) and walk knobs -- outputs are NOT checked (ablations
break them).  C4 by default; --config 2 for C2 at 2^30 B.
    python scripts/c4_ablate.py [--config N]   (one process per setting, one line each)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SETTINGS = [("full", {}), ("no_lookback", {"LSMGPU_ABLATE": "1"}), ("no_walk", {"LSMGPU_ABLATE": "4"}),
            ("no_walk_no_lb", {"LSMGPU_ABLATE": "5"}), ("no_copy", {"LSMGPU_ABLATE": "2"}),
            ("g16", {"LSMGPU_WSC_WALK": "group16"}), ("g16_no_walk", {"LSMGPU_WSC_WALK": "group16", "LSMGPU_ABLATE": "4"}),
            ("lane", {"LSMGPU_WSC_WALK": "lane"})]
SETTINGS_C2 = [("full", {}), ("no_lookback", {"LSMGPU_ABLATE": "1"}), ("no_walk", {"LSMGPU_ABLATE": "4"}),
               ("no_out", {"LSMGPU_ABLATE": "2"}), ("no_walk_no_out", {"LSMGPU_ABLATE": "6"}),
               ("no_walk_lb_out", {"LSMGPU_ABLATE": "7"}),
               # record flushes (128: in the walk loop, 256: the last chunk) -- only with 2
               ("no_out_no_flush", {"LSMGPU_ABLATE": "130"}), ("no_out_no_flush_all", {"LSMGPU_ABLATE": "386"})]


def one(cfg):
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    import bench
    from lsmdb_amd.codec import Codec, MODE_MATERIALIZE, MODE_VIEW
    dev = torch.device("cuda", 0)
    codec = Codec(0)
    w = bench.build_device_sst(codec, torch, dev, cfg, 1 << 30, 0)
    out = {}
    for name, mode in (("mat", MODE_MATERIALIZE | MODE_VIEW), ("view", MODE_VIEW)):
        bufs = codec.alloc_decode(w["data_len"], w["data_len"], w["nblocks"], mode, ent_cap=w["n"])
        for _ in range(3):
            codec.decode_device_async(w["d_sst"], w["d_off"], w["d_len"], w["max_len"], mode, bufs,
                                      data_len=w["data_len"])
        torch.cuda.synchronize()
        ks = bench.kernel_split(codec, w, bufs, mode, reps=20)
        out[name] = (ks["walk_ms"], ks["copy_ms"])
    print(json.dumps(out))


if __name__ == "__main__":
    cfg = int(sys.argv[sys.argv.index("--config") + 1]) if "--config" in sys.argv else 4
    if "--one" in sys.argv:
        one(cfg)
        sys.exit(0)
    settings = SETTINGS if cfg == 4 else SETTINGS_C2
    for name, env in settings:
        r = subprocess.run([sys.executable, __file__, "--one", "--config", str(cfg)], env={**os.environ, **env},
                           capture_output=True, text=True, timeout=300)
        line = r.stdout.strip().splitlines()[-1] if r.returncode == 0 else f"rc={r.returncode} {r.stderr[-300:]}"
        print(name, line, flush=True)
