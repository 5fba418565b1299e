#!/bin/bash
# Round-4 debug: the walk-scan-copy parity subset without -x (which cases fail)
set -o pipefail
O=gpurun_out/${1:-r04dbg}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread \
  -k "walk_modes or many_tiles or forced or adversarial or mixed_copy or view_only" -rf > $O/tests.log 2>&1
rc=$?
grep -E "^FAILED|passed|failed" $O/tests.log | tail -60
exit $rc
