#!/bin/bash
# decode at full size with capped persistent grids: which grids run without spin timeouts
mkdir -p gpurun_out/probe
for g in 256 512 640 768; do
  LSMGPU_GRID=$g timeout -k 10 60 python bench.py --no-cpu --no-view --steps 2 --warmup 1 > gpurun_out/probe/g$g.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/probe/g$g.json')); print('grid $g', d['roofline']['kernel_ms_mean'], d['parity'][:20])"
done
