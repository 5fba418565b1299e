#!/bin/bash
# Full bench (with CPU baseline) + rocprofv3 kernel-trace/stats of the same command + HBM
# traffic passes (each --pmc pass its own run; counters per MI355X_MICROARCH.md limits).
# Usage (on the GPU box): bash scripts/profile_round.sh <tag>
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/rocprof -o run --output-format csv -- python3 bench.py --no-cpu --no-view --no-peaks > $OUT/bench_prof.json 2> $OUT/bench_prof.err || exit 1
P="python3 bench.py --no-cpu --no-view --no-peaks --steps 3 --warmup 1"
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d $OUT/pmc_rd -o run --output-format csv -- $P > $OUT/pmc_rd.json 2> $OUT/pmc_rd.err || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $OUT/pmc_wr -o run --output-format csv -- $P > $OUT/pmc_wr.json 2> $OUT/pmc_wr.err || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- $P > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- $P > $OUT/pmc_write.json 2> $OUT/pmc_write.err || exit 1
python scripts/traffic_summary.py $OUT/pmc_rd/run_counter_collection.csv $OUT/pmc_wr/run_counter_collection.csv $OUT/pmc_fetch/run_counter_collection.csv $OUT/pmc_write/run_counter_collection.csv $OUT/pmc_fetch.json $OUT/pmc_traffic.json
