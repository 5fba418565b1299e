set -o pipefail
O=gpurun_out/r06e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for r in 1 2; do
for f in 1 0; do
LSMGPU_WSC_COPYFUSE=$f timeout -k 10 200 python bench.py --config 4 --no-cpu --no-peaks --no-view --steps 50 > $O/c4_f${f}_r$r.json 2>> $O/bench.err || exit 1
python -c "import json;d=json.loads(open('$O/c4_f${f}_r$r.json').read().strip().splitlines()[-1]);print('fuse=$f', d['ms_per_step'], d['value'], d['roofline']['kernels']['walk_ms'], d['roofline']['kernels']['copy_ms'])"
done
done
