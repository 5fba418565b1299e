#!/bin/bash
# Round-5 walk phase stamps: the diagnostic library (LSMGPU_BUILD_DIAG=1,
# lsmdb_amd/liblsmgpu_diag.so) run through bench.py, every walk launch printing its per-tile
# timeline (start, walk end, look-back end, epilogue end; s_memrealtime at 100 MHz) and appending
# the raw per-tile rows to a file.  C2 2^30 B (materialize and the view-only decode) and C4.
# Usage (on the GPU box): bash scripts/r05_stamps.sh <tag>
set -o pipefail
T=${1:-r05stamps}
O=gpurun_out/$T
mkdir -p $O
for cfg in 2 4; do
  LSMGPU_LIB_VARIANT=diag LSMGPU_STAMPS=1 LSMGPU_STAMPS_FILE=$O/tiles_c$cfg.txt \
    timeout -k 10 200 python bench.py --config $cfg --no-cpu --no-peaks --steps 3 --warmup 1 \
    > $O/bench_c$cfg.json 2> $O/bench_c$cfg.err || { tail -20 $O/bench_c$cfg.err; exit 1; }
  grep "walk stamps" $O/bench_c$cfg.err | tail -12
done
