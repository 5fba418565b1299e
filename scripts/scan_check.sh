#!/bin/bash
set -o pipefail
T=gpurun_out/scan1
mkdir -p $T
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "walk_modes or adversarial" -x -q --timeout 120 --timeout-method thread > $T/tests.log 2>&1 || { tail -40 $T/tests.log; exit 1; }
tail -3 $T/tests.log
for w in group scan scan0; do
  LSMGPU_WSC_WALK=${w%0} LSMGPU_WSC_SCANCOPY=$([ $w = scan0 ] && echo 0 || echo 1) timeout -k 10 200 python bench.py --config 4 --no-cpu --no-view > $T/c4_$w.json 2> $T/c4_$w.err || { tail -20 $T/c4_$w.err; exit 1; }
  python -c "import json;d=json.load(open('$T/c4_$w.json'));print('$w', d['value'], d['ms_per_step'], d['roofline'].get('kernels'))"
done
