#!/bin/bash
# GPU round check: parity tests, bench (no CPU leg), optional PMC instruction pass.
# Usage (on the GPU box): bash scripts/gpu_check.sh <tag> [pmc]
set -o pipefail
T=${1:-chk}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { tail -40 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -3 gpurun_out/$T/gpu_tests.log
timeout -k 10 150 python bench.py --no-cpu > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
cat gpurun_out/$T/bench.json
if [ "$2" = "pmc" ]; then bash scripts/pmc_decode.sh gpurun_out/$T/pmc || exit 1; fi
if [ "$2" = "stamps" ]; then
  LSMGPU_DEBUG=1 LSMGPU_STAMPS=1 timeout -k 10 100 python bench.py --no-cpu --no-view --steps 2 --warmup 1 > gpurun_out/$T/stamps.json 2> gpurun_out/$T/stamps.err || exit 1
  grep "lsmgpu" gpurun_out/$T/stamps.err | tail -4
fi
