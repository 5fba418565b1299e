#!/bin/bash
# Scan-walk A/B: parity (walk modes, adversarial), then C4 (one 64 MiB table) and C2 (1 GiB).
set -o pipefail
T=gpurun_out/scanab
mkdir -p $T
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "walk_modes or adversarial" -x -q --timeout 120 --timeout-method thread > $T/tests.log 2>&1 || { tail -40 $T/tests.log; exit 1; }
tail -1 $T/tests.log
run() {  # cfg tag env...
  local cfg=$1 tag=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --config $cfg --no-cpu --no-peaks > $T/c${cfg}_$tag.json 2> $T/c${cfg}_$tag.err || { tail -20 $T/c${cfg}_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('$T/c${cfg}_$tag.json'));k=d['roofline']['kernels'];print('C$cfg $tag', d['value'], d['ms_per_step'], k['walk_ms'], k['copy_ms'], 'view', d['view_mode']['kernel_ms'], d['parity'][:14])"
}
run 4 group LSMGPU_WSC_WALK=group
run 4 scan16 LSMGPU_WSC_WALK=scan16


run 2 lane LSMGPU_WSC_WALK=lane
run 2 scan64_0 LSMGPU_WSC_WALK=scan64 LSMGPU_WSC_SCANCOPY=0

run 2 scan16_0 LSMGPU_WSC_WALK=scan16 LSMGPU_WSC_SCANCOPY=0
