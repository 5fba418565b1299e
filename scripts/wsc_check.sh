#!/bin/bash
# Walk-scan-copy iteration on the GPU box: its parity tests, then the bench with each walk.
# Usage: bash scripts/wsc_check.sh <tag>
set -o pipefail
T=${1:-wscc}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fsc.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -40 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
for W in stream global; do
  LSMGPU_WSC_WALK=$W timeout -k 10 150 python bench.py --no-cpu --steps 20 > gpurun_out/$T/bench_$W.json 2> gpurun_out/$T/bench_$W.err || { tail -20 gpurun_out/$T/bench_$W.err; exit 1; }
  echo "== $W"; python scripts/bench_brief.py gpurun_out/$T/bench_$W.json
  python -c "import json;d=json.loads(open('gpurun_out/$T/bench_$W.json').read().strip().splitlines()[-1]);print('  view',d.get('view_mode'))"
done
