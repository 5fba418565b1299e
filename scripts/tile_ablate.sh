#!/bin/bash
# fused tile decode timing ablations (LSMGPU_ABLATE bits: 1 no prefix, 2 no copy, 64 blockIdx order)
set -o pipefail
mkdir -p gpurun_out/tile
for A in ${ABLATIONS:-0 64 1 65 2 3 67}; do
  LSMGPU_DECODE_PATH=tile LSMGPU_TILE=${T:-2} LSMGPU_ABLATE=$A timeout -k 10 120 python bench.py --no-cpu --no-view --steps 10 > gpurun_out/tile/ab$A.json 2> gpurun_out/tile/ab$A.err || { tail -20 gpurun_out/tile/ab$A.err; exit 1; }
  echo "ablate=$A"; python scripts/bench_brief.py gpurun_out/tile/ab$A.json
done
