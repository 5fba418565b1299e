#!/bin/bash
# Fused-decode iteration on the GPU box: its parity tests, then the bench with the path forced.
# Usage: bash scripts/fsc_check.sh <tag> [extra env for the bench, e.g. LSMGPU_ABLATE=2]
set -o pipefail
T=${1:-fsc}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_fsc.py "tests/test_gpu_parity.py::test_forced_decode_paths" -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -40 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
for P in fsc wsc; do
  env LSMGPU_DECODE_PATH=$P $2 timeout -k 10 150 python bench.py --no-cpu --steps 20 > gpurun_out/$T/bench_$P.json 2> gpurun_out/$T/bench_$P.err || { tail -20 gpurun_out/$T/bench_$P.err; exit 1; }
  echo "== $P"; python scripts/bench_brief.py gpurun_out/$T/bench_$P.json
  python -c "import json;d=json.loads(open('gpurun_out/$T/bench_$P.json').read().strip().splitlines()[-1]);print('  view',d.get('view_mode'))"
done
