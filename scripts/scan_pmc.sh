#!/bin/bash
# PMC instruction / stall profile of the scan walk (C2 1 GiB, LSMGPU_WSC_WALK=scan64, copy launch)
set -o pipefail
OUT=gpurun_out/scanpmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export LSMGPU_WSC_WALK=${WALK:-scan64} LSMGPU_WSC_SCANCOPY=0
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_WAIT_INST_ANY -d $OUT/a -o run --output-format csv -- python3 bench.py --no-cpu --no-view --no-peaks --steps 2 --warmup 1 > $OUT/a.json 2> $OUT/a.err || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $OUT/b -o run --output-format csv -- python3 bench.py --no-cpu --no-view --no-peaks --steps 2 --warmup 1 > $OUT/b.json 2> $OUT/b.err || exit 1
PMC_FILTER=walk python3 scripts/pmc_summary.py $OUT/a/run_counter_collection.csv $OUT/b/run_counter_collection.csv
