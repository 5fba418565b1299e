#!/bin/bash
# Round-end evidence in one GPU call: the GPU suite, smoke, the bench + rocprofv3 + PMC traffic
# passes (scripts/profile_round.sh) and the other configs (C3/C4/C5) and the E2E host-path line.
# Usage (on the GPU box): bash scripts/round_final.sh <tag>
set -o pipefail
T=${1:-final}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash scripts/profile_round.sh $T || exit 1
bash scripts/r04_ab.sh $T "e c"
