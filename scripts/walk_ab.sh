#!/bin/bash
# Walk A/B (LSMGPU_WSC_WALK) on C2 / C4 / C5: walk-mode parity first, then bench lines.
set -o pipefail
T=${1:-walkab}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "walk_modes or walk_adversarial" > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
run() {  # config walk
  LSMGPU_WSC_WALK=$2 timeout -k 10 150 python bench.py --no-cpu --config $1 > gpurun_out/$T/c$1_$2.json 2> gpurun_out/$T/c$1_$2.err || { tail -20 gpurun_out/$T/c$1_$2.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/$T/c$1_$2.json'));k=j['roofline']['kernels'];print('C$1 $2',j['value'],j['ms_per_step'],k['walk_ms'],k['copy_ms'],j['view_mode']['kernel_ms'],j['parity'][:12])"
}
for w in group4 group group16; do run 4 $w || exit 1; done
for w in lane group4 group; do run 2 $w || exit 1; done
for w in lane group; do run 5 $w || exit 1; done
