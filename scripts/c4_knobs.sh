#!/bin/bash
# C4 (one 64 MiB table, 12.9 KB blocks) decode under the copy's split / lanes-per-entry knobs.
set -o pipefail
mkdir -p gpurun_out/c4k
for V in ${VARIANTS:-S2 S1 S4 S4J16 S2J16 S2}; do
  S=${V#S}; S=${S%%J*}; J=""; case $V in *J*) J=${V##*J};; esac
  LSMGPU_WSC_SPLIT=$S LSMGPU_WSC_J=$J timeout -k 10 120 python bench.py --no-cpu --no-view --config 4 --gib 0.0625 --steps 20 > gpurun_out/c4k/$V.json 2> gpurun_out/c4k/$V.err || { tail -5 gpurun_out/c4k/$V.err; exit 1; }
  echo "$V"; python scripts/bench_brief.py gpurun_out/c4k/$V.json | head -1
done
