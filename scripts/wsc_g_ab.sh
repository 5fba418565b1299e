#!/bin/bash
# walk-scan-copy copy kernel A/B over LSMGPU_WSC_G (entry groups per loop trip)
set -o pipefail
mkdir -p gpurun_out/wscg
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "split or forced or large" > gpurun_out/wscg/tests.log 2>&1 || { tail -30 gpurun_out/wscg/tests.log; exit 1; }
tail -1 gpurun_out/wscg/tests.log
for cfg in 2 5; do for G in 1 2 4; do
  LSMGPU_WSC_G=$G timeout -k 10 120 python bench.py --no-cpu --no-view --steps 20 --config $cfg > gpurun_out/wscg/c${cfg}g$G.json 2> gpurun_out/wscg/c${cfg}g$G.err || { tail -5 gpurun_out/wscg/c${cfg}g$G.err; exit 1; }
  echo "G=$G"; python scripts/bench_brief.py gpurun_out/wscg/c${cfg}g$G.json | head -1
done; done
