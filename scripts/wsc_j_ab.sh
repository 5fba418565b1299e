#!/bin/bash
# walk-scan-copy copy kernel: parity with lanes-per-entry forced to 16 and 8, then C5/C2 A/B
# of the per-block choice (default) against forced 8 / 16
set -o pipefail
mkdir -p gpurun_out/wscj
for J in 16 8; do
LSMGPU_WSC_J=$J timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "split or forced or large or tiles" > gpurun_out/wscj/tests$J.log 2>&1 || { tail -30 gpurun_out/wscj/tests$J.log; exit 1; }
tail -1 gpurun_out/wscj/tests$J.log
done
for cfg in 5 2 4; do for J in auto 8 16; do
  g=1; [ "$cfg" = 4 ] && g=0.0625
  if [ $J = auto ]; then unset LSMGPU_WSC_J; else export LSMGPU_WSC_J=$J; fi
  timeout -k 10 120 python bench.py --no-cpu --no-view --steps 20 --config $cfg --gib $g > gpurun_out/wscj/c${cfg}j$J.json 2> gpurun_out/wscj/c${cfg}j$J.err || { tail -5 gpurun_out/wscj/c${cfg}j$J.err; exit 1; }
  echo "J=$J"; python scripts/bench_brief.py gpurun_out/wscj/c${cfg}j$J.json | head -1
done; done
