#!/bin/bash
# Full bench (with CPU baseline) + rocprofv3 kernel-trace/stats of the same command.
# Usage (on the GPU box): bash scripts/profile_round.sh <tag>
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/rocprof -o run --output-format csv -- python3 bench.py --no-cpu --no-view > $OUT/bench_prof.json 2> $OUT/bench_prof.err || exit 1
# HBM traffic: separate --pmc passes (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950)
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --no-cpu --no-view --steps 3 --warmup 1 > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --no-cpu --no-view --steps 3 --warmup 1 > $OUT/pmc_write.json 2> $OUT/pmc_write.err || exit 1
python scripts/traffic_summary.py $OUT/pmc_fetch/run_counter_collection.csv $OUT/pmc_write/run_counter_collection.csv $OUT/pmc_fetch.json $OUT/pmc_traffic.json
