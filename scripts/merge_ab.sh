#!/bin/bash
# Merge A/B: merge parity tests, then the compaction replay.  Usage: bash scripts/merge_ab.sh <tag>
set -o pipefail
T=${1:-mab}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_merge.py tests/test_gpu_compaction.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
timeout -k 10 200 python scripts/compaction_bench.py > gpurun_out/$T/c.json 2> gpurun_out/$T/c.err || { tail -5 gpurun_out/$T/c.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/$T/c.json').read().strip().splitlines()[-1]);print('merge', d['merge_ms'], 'total', d['total_ms'], 'ok', d['merge_matches_oracle'])"
