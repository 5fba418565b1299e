#!/bin/bash
# PMC instruction profile of the decode kernel (counters only with --kernel-trace)
set -o pipefail
OUT=${1:-gpurun_out/pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d $OUT -o run --output-format csv -- python3 bench.py --no-cpu --no-view --steps 2 --warmup 1 > $OUT/b.json 2> $OUT/b.err
