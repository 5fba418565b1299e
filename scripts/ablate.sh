#!/bin/bash
# timing-only ablations of the decode kernel (outputs are wrong by design)
set -o pipefail
for a in 0 1 2 3 4 6 7; do
  echo "ABLATE=$a" 
  LSMGPU_ABLATE=$a timeout -k 10 200 python bench.py --no-cpu --steps 10 --no-view 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel_ms_mean'], d['parity'][:14])" || exit 1
done
