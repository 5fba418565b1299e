#!/bin/bash
# fused tile decode: forced-path parity, then C2 timing for tile sizes T = 1, 2, 4
set -o pipefail
mkdir -p gpurun_out/tile
LSMGPU_DECODE_PATH=tile timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "forced" > gpurun_out/tile/tests.log 2>&1 || { tail -30 gpurun_out/tile/tests.log; exit 1; }
tail -2 gpurun_out/tile/tests.log
for T in ${TILES:-2 1 4}; do
  LSMGPU_DECODE_PATH=tile LSMGPU_TILE=$T timeout -k 10 120 python bench.py --no-cpu --steps 20 > gpurun_out/tile/c2_t$T.json 2> gpurun_out/tile/c2_t$T.err || { tail -20 gpurun_out/tile/c2_t$T.err; exit 1; }
  echo "T=$T"; python scripts/bench_brief.py gpurun_out/tile/c2_t$T.json
done
