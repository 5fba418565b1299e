#!/bin/bash
# One-pass decode (decode_onepass.hip) vs walk-scan-copy, same box: the one-pass parity tests,
# then C2 1 GiB bench lines for each path and a workers-per-CU sweep.
# Usage (on the GPU box): bash scripts/onepass_ab.sh <tag> [config] [wpc list]
set -o pipefail
T=${1:-onepass}
CFG=${2:-2}
WPCS=${3:-"8 12 16 24"}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "one or many_tiles or lane16" > gpurun_out/$T/tests.log 2>&1 || { tail -40 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --config $CFG --no-cpu --no-peaks --steps 20 \
    > gpurun_out/$T/bench_$name.json 2> gpurun_out/$T/bench_$name.err || { tail -20 gpurun_out/$T/bench_$name.err; exit 1; }
  python - gpurun_out/$T/bench_$name.json $name <<'EOF'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = j["roofline"]
print(sys.argv[2], j["value"], "GiB/s", r["kernel_ms_mean"], "ms", "view", j.get("view_mode", {}).get("kernel_ms"),
      "ms", "split", (r.get("kernels") or {}).get("walk_ms"), (r.get("kernels") or {}).get("copy_ms"))
EOF
}
run wsc LSMGPU_DECODE_PATH=wsc
run wsc_ch16 LSMGPU_DECODE_PATH=wsc LSMGPU_WSC_CHUNK=16
for w in $WPCS; do run one_w$w LSMGPU_DECODE_PATH=one LSMGPU_ONEPASS_WPC=$w; done
run one_nopf LSMGPU_DECODE_PATH=one LSMGPU_ONEPASS_PF=0
run one_batch LSMGPU_DECODE_PATH=one LSMGPU_ONEPASS_BATCH=1
run one_tb8 LSMGPU_DECODE_PATH=one LSMGPU_ONEPASS_TB=8
run wsc2 LSMGPU_DECODE_PATH=wsc
