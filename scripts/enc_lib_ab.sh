#!/bin/bash
# Encode A/B of two builds on one box: liblsmgpu.so vs liblsmgpu_${VARIANT:-prev}.so, alternating
set -o pipefail
mkdir -p gpurun_out/eab
for k in 1 2 3; do
  for V in cur ${VARIANT:-prev}; do
    if [ $V = cur ]; then unset LSMGPU_LIB_VARIANT; else export LSMGPU_LIB_VARIANT=$V; fi
    timeout -k 10 120 python bench.py --no-cpu --no-view --steps 10 --config ${CFG:-2} > gpurun_out/eab/$V$k.json 2> gpurun_out/eab/$V$k.err || { tail -5 gpurun_out/eab/$V$k.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/eab/$V$k.json')); e=d['encode']; print('$V $k', d['value'], e['gibs_per_gpu'], e['kernel_ms'], e['identical_to_decoded_shard'])"
  done
done
