#!/bin/bash
# encoder A/B over LSMGPU_ENC_G (entry-group passes per loop trip) / LSMGPU_ENC_J (lanes per entry)
set -o pipefail
mkdir -p gpurun_out/encab
for V in ${VARIANTS:-G1 J4 J16}; do
  case $V in G*) export LSMGPU_ENC_G=${V#G}; unset LSMGPU_ENC_J;; J*) export LSMGPU_ENC_J=${V#J}; unset LSMGPU_ENC_G;; esac
  timeout -k 10 120 python bench.py --no-cpu --no-view --steps 10 --config ${CFG:-2} > gpurun_out/encab/$V.json 2> gpurun_out/encab/$V.err || { tail -5 gpurun_out/encab/$V.err; exit 1; }
  echo "$V"; python scripts/bench_brief.py gpurun_out/encab/$V.json | tail -1
done
