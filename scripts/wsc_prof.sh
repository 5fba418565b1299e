#!/bin/bash
# per-kernel times of the walk-scan-copy decode (C2 forced onto it, C5 native)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wsc
for c in 2 5; do
  LSMGPU_DECODE_PATH=wsc timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/wsc/c$c -o run --output-format csv -- python3 bench.py --no-cpu --no-view --config $c --steps 5 --warmup 1 > gpurun_out/wsc/c$c.json 2> gpurun_out/wsc/c$c.err || exit 1
  echo "config $c"; cut -d, -f1-4 gpurun_out/wsc/c$c/run_kernel_stats.csv | grep -i "wsc\|scan\|lsmgpu" | cut -c1-160
done
