#!/bin/bash
# Round-3 end: C3 / C4 / C5 bench lines, the compaction replay, and the 2-rank self-spawn rehearsal
# on one GPU (gloo, both ranks on device 0)
set -o pipefail
T=gpurun_out/r03cfg
mkdir -p $T
for c in 3 4 5; do
  timeout -k 10 200 python bench.py --config $c --no-cpu > $T/bench_c$c.json 2> $T/bench_c$c.err || { tail -20 $T/bench_c$c.err; exit 1; }
  python -c "import json;j=json.load(open('$T/bench_c$c.json'));k=j['roofline']['kernels'];print('C$c',j['value'],j['ms_per_step'],k['walk_ms'],k['copy_ms'],'view',j['view_mode']['kernel_ms'],'enc',j['encode']['kernel_ms'])"
done
timeout -k 10 300 python scripts/compaction_bench.py > $T/compaction.json 2> $T/compaction.err || { tail -20 $T/compaction.err; exit 1; }
tail -c 1500 $T/compaction.json
BENCH_DIST_BACKEND=gloo BENCH_DEVICE_OVERRIDE=0 timeout -k 10 300 python bench.py --gpus 2 --no-cpu --no-view --steps 5 > $T/bench_n2.json 2> $T/bench_n2.err || { tail -20 $T/bench_n2.err; exit 1; }
python -c "import json;j=json.load(open('$T/bench_n2.json'));print('n2', j['n_gpus'], j['value'], j['per_rank_ms'])"
