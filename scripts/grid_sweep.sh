#!/bin/bash
# decode time vs persistent-grid size (workgroups per CU x 256): how latency-bound is it?
set -o pipefail
mkdir -p gpurun_out/probe
for g in ${GRIDS:-1024 1536 2048 2304 2560 2816}; do
  LSMGPU_GRID=$g timeout -k 10 60 python bench.py --no-cpu --no-view --steps 10 --warmup 2 > gpurun_out/probe/g$g.json 2>/dev/null || exit 1
  echo "grid $g $(python scripts/bench_brief.py gpurun_out/probe/g$g.json)"
done
