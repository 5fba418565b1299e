#!/bin/bash
# walk-scan-copy chunked on ONE stream (copy c right after walk c: Infinity-Cache reuse)
set -o pipefail
mkdir -p gpurun_out/one
LSMGPU_WSC_ONE_STREAM=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "chunked" > gpurun_out/one/tests.log 2>&1 || { tail -30 gpurun_out/one/tests.log; exit 1; }
tail -1 gpurun_out/one/tests.log
for cfg in ${CFGS:-2 5}; do
for C in ${CHUNKS:-1 4 8 16}; do
  LSMGPU_WSC_ONE_STREAM=1 LSMGPU_WSC_CHUNKS=$C timeout -k 10 120 python bench.py --no-cpu --no-view --config $cfg --steps 20 > gpurun_out/one/c${cfg}_$C.json 2> gpurun_out/one/c${cfg}_$C.err || { tail -20 gpurun_out/one/c${cfg}_$C.err; exit 1; }
  echo "chunks=$C"; python scripts/bench_brief.py gpurun_out/one/c${cfg}_$C.json
done
done
