#!/bin/bash
# Walk-scan-copy ablations (timing only; LSMGPU_ABLATE bits: 2 no copy / view emit, 4 no walk
# in the streaming walk).  Usage: bash scripts/wsc_ablate.sh <tag> "<ablate list>" [walk]
set -o pipefail
T=${1:-wsca}
mkdir -p gpurun_out/$T
for A in ${2:-0 2 4 6}; do
  LSMGPU_DECODE_PATH=wsc LSMGPU_WSC_WALK=${3:-stream} LSMGPU_ABLATE=$A timeout -k 10 120 python bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/$T/b_$A.json 2> gpurun_out/$T/b_$A.err || { tail -5 gpurun_out/$T/b_$A.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/$T/b_$A.json').read().strip().splitlines()[-1]);print('ablate $A', 'mat_ms', d['roofline']['kernel_ms_mean'], 'view_ms', d['view_mode']['kernel_ms'])"
done
