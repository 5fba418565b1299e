#!/bin/bash
# Fused-decode phase stamps (LSMGPU_STAMPS, s_memtime cycles; diagnostics only).
set -o pipefail
T=${1:-fscs}
mkdir -p gpurun_out/$T
for A in ${2:-0}; do
  LSMGPU_DECODE_PATH=fsc LSMGPU_STAMPS=1 LSMGPU_ABLATE=$A timeout -k 10 120 python bench.py --no-cpu --steps 2 --warmup 1 > gpurun_out/$T/s_$A.json 2> gpurun_out/$T/s_$A.err || { tail -5 gpurun_out/$T/s_$A.err; exit 1; }
  echo "== ablate $A"; grep "fsc stamps" gpurun_out/$T/s_$A.err | tail -2
done
