#!/bin/bash
# XCD-aware copy map A/B (LSMGPU_WSC_XCD): C2 1 GiB materialize, alternating, then C5 / C3.
set -o pipefail
mkdir -p gpurun_out/xcd
for V in 0 1 0 1; do
  LSMGPU_WSC_XCD=$V timeout -k 10 120 python bench.py --no-cpu --no-view --steps 20 > gpurun_out/xcd/c2_$V.json 2> gpurun_out/xcd/c2_$V.err || { tail -5 gpurun_out/xcd/c2_$V.err; exit 1; }
  echo "xcd $V"; python scripts/bench_brief.py gpurun_out/xcd/c2_$V.json | head -1
done
for C in 5 3; do for V in 0 1; do
  LSMGPU_WSC_XCD=$V timeout -k 10 120 python bench.py --no-cpu --no-view --steps 10 --config $C > gpurun_out/xcd/c${C}_$V.json 2> gpurun_out/xcd/c${C}_$V.err || exit 1
  echo "xcd $V"; python scripts/bench_brief.py gpurun_out/xcd/c${C}_$V.json | head -1
done; done
