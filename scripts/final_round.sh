#!/bin/bash
# Round end: library A/B vs liblsmgpu_prev.so, the full GPU suite, smoke, and the profile round
set -o pipefail


timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || { tail -30 gpurun_out/final_tests.log; exit 1; }
tail -1 gpurun_out/final_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
bash scripts/profile_round.sh r03r && python -c "import json;j=json.load(open('gpurun_out/prof_r03r/bench.json'));k=j['roofline']['kernels'];print('bench',j['value'],j['ms_per_step'],k['walk_ms'],k['copy_ms'],'view',j['view_mode']['gibs_per_gpu'])"
