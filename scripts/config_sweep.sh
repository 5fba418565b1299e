#!/bin/bash
# decode throughput of every BASELINE config shape on one GPU (C2 is bench.py's default)
set -o pipefail
mkdir -p gpurun_out/cfg
for c in ${CONFIGS:-5 4 1 3}; do
  g=1
  [ "$c" = 4 ] && g=0.0625
  [ "$c" = 1 ] && g=0.00125
  LSMGPU_DEBUG=1 timeout -k 10 120 python bench.py --no-cpu --no-view --config $c --gib $g --steps 10 > gpurun_out/cfg/c$c.json 2> gpurun_out/cfg/c$c.err || exit 1
  python scripts/bench_brief.py gpurun_out/cfg/c$c.json
  grep "decode " gpurun_out/cfg/c$c.err | tail -1 || true
done
