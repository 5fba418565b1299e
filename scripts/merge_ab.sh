#!/bin/bash
# Merge emit tile A/B: merge parity tests, then the compaction replay with each positions-per-
# thread setting.  Usage: bash scripts/merge_ab.sh <tag> [pp...]
set -o pipefail
T=${1:-mab}
shift
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_merge.py tests/test_gpu_compaction.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
for PP in ${*:-4 2 1}; do
  G=4; [ "${PP#g}" != "$PP" ] && { G=8; PP=${PP#g}; }
  LSMGPU_MERGE_G=$G LSMGPU_MERGE_PP=$PP timeout -k 10 200 python scripts/compaction_bench.py > gpurun_out/$T/c_$PP$G.json 2> gpurun_out/$T/c_$PP$G.err || { tail -5 gpurun_out/$T/c_$PP$G.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/$T/c_$PP$G.json').read().strip().splitlines()[-1]);print('pp $PP g $G merge', d['merge_ms'], 'total', d['total_ms'], 'ok', d['merge_matches_oracle'])"
done
