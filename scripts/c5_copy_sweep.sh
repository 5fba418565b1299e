#!/bin/bash
# C5 copy A/B: waves per block (LSMGPU_WSC_SPLIT) x lanes per entry (LSMGPU_WSC_J)
set -o pipefail
T=${1:-c5s}
mkdir -p gpurun_out/$T
for S in ${SPLITS:-2 4}; do
  for J in ${JS:-16 8}; do
    LSMGPU_WSC_SPLIT=$S LSMGPU_WSC_J=$J timeout -k 10 150 python bench.py --no-cpu --no-view --config 5 --steps 10 > gpurun_out/$T/s${S}_j$J.json 2> gpurun_out/$T/s${S}_j$J.err || { tail -5 gpurun_out/$T/s${S}_j$J.err; exit 1; }
    echo "split=$S J=$J"; python scripts/bench_brief.py gpurun_out/$T/s${S}_j$J.json | head -1
  done
done
