#!/bin/bash
# walk-scan-copy: waves-per-block sweep of the copy (LSMGPU_WSC_SPLIT) on C5 / C4 / C2
set -o pipefail
mkdir -p gpurun_out/split
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "split" > gpurun_out/split/tests.log 2>&1 || { tail -30 gpurun_out/split/tests.log; exit 1; }
tail -1 gpurun_out/split/tests.log
for cfg in ${CFGS:-5 4 2}; do
  g=1; [ "$cfg" = 4 ] && g=0.0625
  for S in ${SPLITS:-1 2 4}; do
    LSMGPU_WSC_SPLIT=$S timeout -k 10 120 python bench.py --no-cpu --no-view --config $cfg --gib $g --steps 20 > gpurun_out/split/c${cfg}_$S.json 2> gpurun_out/split/c${cfg}_$S.err || { tail -20 gpurun_out/split/c${cfg}_$S.err; exit 1; }
    echo "split=$S"; python scripts/bench_brief.py gpurun_out/split/c${cfg}_$S.json
  done
done
