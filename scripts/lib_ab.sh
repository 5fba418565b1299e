#!/bin/bash
# A/B of two builds of the codec on one box: liblsmgpu.so vs liblsmgpu_$VARIANT.so, alternating
set -o pipefail
mkdir -p gpurun_out/ab
for k in 1 2 3; do
  for V in cur ${VARIANT:-prev}; do
    if [ $V = cur ]; then unset LSMGPU_LIB_VARIANT; else export LSMGPU_LIB_VARIANT=$V; fi
    timeout -k 10 120 python bench.py --no-cpu --no-view --steps 20 --config ${CFG:-2} > gpurun_out/ab/$V$k.json 2> gpurun_out/ab/$V$k.err || { tail -5 gpurun_out/ab/$V$k.err; exit 1; }
    echo "$V $k $(python scripts/bench_brief.py gpurun_out/ab/$V$k.json | head -1)"
  done
done
