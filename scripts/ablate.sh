#!/bin/bash
# timing-only ablations of the decode kernel (outputs are wrong by design):
# 1 = no prefix protocol, 2 = no emit, 4 = no walk (combinations add)
set -o pipefail
mkdir -p gpurun_out/abl
for a in ${ABLATIONS:-0 1 2 3 6 7}; do
  LSMGPU_ABLATE=$a timeout -k 10 60 python bench.py --no-cpu --steps 10 --no-view > gpurun_out/abl/a$a.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/abl/a$a.json')); print('ablate $a', d['roofline']['kernel_ms_mean'], d['parity'][:14])"
done
