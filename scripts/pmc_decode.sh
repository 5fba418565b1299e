#!/bin/bash
# PMC instruction / stall profile of the decode kernel (counters only with --kernel-trace)
set -o pipefail
OUT=${1:-gpurun_out/pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_WAIT_INST_ANY -d $OUT/a -o run --output-format csv -- python3 bench.py --no-cpu --no-view --steps 2 --warmup 1 > $OUT/a.json 2> $OUT/a.err || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $OUT/b -o run --output-format csv -- python3 bench.py --no-cpu --no-view --steps 2 --warmup 1 > $OUT/b.json 2> $OUT/b.err || exit 1
