#!/bin/bash
# VALU / SALU / LDS instruction counts of the scan walk (one pass, C2 1 GiB)
set -o pipefail
OUT=${1:-gpurun_out/scanpmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
LSMGPU_WSC_WALK=scan timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_WAIT_INST_ANY -d $OUT/a -o run --output-format csv -- python3 bench.py --no-cpu --no-view --steps 2 --warmup 1 > $OUT/a.json 2> $OUT/a.err || exit 1
PMC_FILTER=walk python scripts/pmc_summary.py $(find $OUT/a -name "*counter_collection.csv")
