"""Walk residency census from the stamps build's per-tile rows (LSMGPU_STAMPS_FILE): per launch,
how many tiles started at once (start < 20 us after the first), when the rest started, the
walk / look-back / epilogue medians and the span.
Usage: python scripts/tile_census.py gpurun_out/<tag>/tiles_*.txt"""
import sys

import numpy as np

for f in sys.argv[1:]:
    a = np.loadtxt(f, dtype=np.int64, ndmin=2)
    cuts = list(np.nonzero(a[:, 0] == 0)[0]) + [len(a)]
    for i in range(len(cuts) - 1):
        t = a[cuts[i]:cuts[i + 1]] / 100.0  # 100 MHz ticks -> us
        st, we, lb, ep = t[:, 1], t[:, 2], t[:, 3], t[:, 4]
        early = st < 20
        late = st[~early]
        print(f"{f.split('/')[-1]} launch {i}: {len(t)} tiles, {early.sum()} at once, "
              f"{(~early).sum()} later (from {late.min() if late.size else 0:.1f} us) | walk "
              f"{np.median(we - st):.1f} look-back {np.median(lb - we):.1f} epilogue "
              f"{np.median(ep - lb):.2f} | span {ep.max():.1f} us")
