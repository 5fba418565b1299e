#!/bin/bash
# PMC instruction profile of the decode kernel per timing-only ablation (see scripts/ablate.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for a in ${ABLATIONS:-0 1 2 3 7}; do
  OUT=gpurun_out/pmca/a$a
  mkdir -p $OUT
  LSMGPU_ABLATE=$a timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM -d $OUT -o run --output-format csv -- python3 bench.py --no-cpu --no-view --steps 2 --warmup 1 > $OUT/b.json 2> $OUT/b.err || exit 1
done
