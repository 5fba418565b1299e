#!/bin/bash
# Walk-scan-copy iteration on the GPU box: its parity tests, then the bench with each walk
# (C2 1 GiB; C4 64 MiB and C5 1 GiB with WALK_CONFIGS="4 5").
# Usage: bash scripts/wsc_check.sh <tag> [walks...]
set -o pipefail
T=${1:-wscc}
shift
WALKS=${*:-lane group group4 group16}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fsc.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -40 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
for W in $WALKS; do
  LSMGPU_WSC_WALK=$W timeout -k 10 150 python bench.py --no-cpu --steps 20 > gpurun_out/$T/bench_$W.json 2> gpurun_out/$T/bench_$W.err || { tail -20 gpurun_out/$T/bench_$W.err; exit 1; }
  echo "== $W"; python scripts/bench_brief.py gpurun_out/$T/bench_$W.json
  python -c "import json;d=json.loads(open('gpurun_out/$T/bench_$W.json').read().strip().splitlines()[-1]);print('  view',d.get('view_mode'))"
  for c in ${WALK_CONFIGS:-}; do
    g=1
    [ "$c" = 4 ] && g=0.0625
    LSMGPU_WSC_WALK=$W timeout -k 10 120 python bench.py --no-cpu --no-view --config $c --gib $g --steps 10 > gpurun_out/$T/c${c}_$W.json 2> gpurun_out/$T/c${c}_$W.err || exit 1
    echo "  C$c:"; python scripts/bench_brief.py gpurun_out/$T/c${c}_$W.json
  done
done
