#!/bin/bash
# Scan-walk iteration on the GPU box: its parity tests, then C2 1 GiB bench with each walk.
# Usage: bash scripts/scan_check.sh <tag> [walks...]
set -o pipefail
T=${1:-scan}
shift
WALKS=${*:-scan lane}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "walk_modes or adversarial" > gpurun_out/$T/tests.log 2>&1 || { tail -40 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
for W in $WALKS; do
  LSMGPU_WSC_WALK=$W timeout -k 10 150 python bench.py --no-cpu --steps 20 > gpurun_out/$T/bench_$W.json 2> gpurun_out/$T/bench_$W.err || { tail -20 gpurun_out/$T/bench_$W.err; exit 1; }
  echo "== $W"; python scripts/bench_brief.py gpurun_out/$T/bench_$W.json
  python -c "import json;d=json.loads(open('gpurun_out/$T/bench_$W.json').read().strip().splitlines()[-1]);print('  view',d.get('view_mode'))"
done
