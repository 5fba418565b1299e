#!/bin/bash
# Round-3 check: new GPU tests, default bench, C4 / C5 bench lines, 2-rank self-spawn rehearsal.
set -o pipefail
T=${1:-r03}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_shim.py tests/test_gpu_bloom.py -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/new_tests.log 2>&1 || { tail -40 gpurun_out/$T/new_tests.log; exit 1; }
tail -3 gpurun_out/$T/new_tests.log
timeout -k 10 300 python bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
cat gpurun_out/$T/bench.json
timeout -k 10 200 python bench.py --config 4 --no-cpu > gpurun_out/$T/bench_c4.json 2> gpurun_out/$T/bench_c4.err || { tail -20 gpurun_out/$T/bench_c4.err; exit 1; }
timeout -k 10 200 python bench.py --config 5 --no-cpu > gpurun_out/$T/bench_c5.json 2> gpurun_out/$T/bench_c5.err || { tail -20 gpurun_out/$T/bench_c5.err; exit 1; }
BENCH_DIST_BACKEND=gloo BENCH_DEVICE_OVERRIDE=0 timeout -k 10 300 python bench.py --gpus 2 --no-cpu --no-view --steps 5 > gpurun_out/$T/bench_n2.json 2> gpurun_out/$T/bench_n2.err || { tail -20 gpurun_out/$T/bench_n2.err; exit 1; }
head -c 600 gpurun_out/$T/bench_n2.json
