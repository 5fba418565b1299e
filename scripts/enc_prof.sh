#!/bin/bash
# encoder: C2 bench line + rocprofv3 kernel stats (encode kernel next to the decode kernels)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/enc
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "encode or golden or slow or table" > gpurun_out/enc/tests.log 2>&1 || { tail -30 gpurun_out/enc/tests.log; exit 1; }
tail -1 gpurun_out/enc/tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/enc/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-view --steps 10 > gpurun_out/enc/c2.json 2> gpurun_out/enc/c2.err || exit 1
python scripts/bench_brief.py gpurun_out/enc/c2.json
cut -d, -f1-4 gpurun_out/enc/prof/run_kernel_stats.csv | grep -i "encode\|wsc" | cut -c1-150
