#!/bin/bash
# Fused-decode ablations (timing only; LSMGPU_ABLATE bits: 1 no look-back, 2 no copy,
# 4 no walk, 8 no ticket, 16 no record writes).  Usage: bash scripts/fsc_ablate.sh <tag> "<list>"
set -o pipefail
T=${1:-fsca}
mkdir -p gpurun_out/$T
for A in ${2:-0 2 3 6 7 15 31}; do
  LSMGPU_DECODE_PATH=${PATH_OVERRIDE:-fsc} LSMGPU_ABLATE=$A timeout -k 10 120 python bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/$T/b_$A.json 2> gpurun_out/$T/b_$A.err || { tail -5 gpurun_out/$T/b_$A.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/$T/b_$A.json').read().strip().splitlines()[-1]);print('ablate $A', 'mat_ms', d['roofline']['kernel_ms_mean'], 'view_ms', d['view_mode']['kernel_ms'])"
done
