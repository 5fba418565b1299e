# copy_entries_pipe depth A/B (diag, LSMGPU_WSC_PDEPTH 2 / 3 / 4): parity at 3 and 4, then C2
set -o pipefail
O=gpurun_out/${OUT:-r06u}
mkdir -p $O
for d in 3 4; do
LSMGPU_LIB_VARIANT=diag LSMGPU_WSC_PDEPTH=$d timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_golden.py > $O/parity_d$d.log 2>&1 || { tail -30 $O/parity_d$d.log; exit 1; }
tail -1 $O/parity_d$d.log
done
for r in 1 2; do
for d in 2 3 4; do
LSMGPU_LIB_VARIANT=diag LSMGPU_WSC_PDEPTH=$d timeout -k 10 200 python bench.py --config 2 --no-cpu --no-peaks --no-view --steps 50 > $O/c2_d${d}_r$r.json 2>> $O/bench.err || exit 1
python -c "
import json; d=json.load(open('$O/c2_d${d}_r$r.json')); k=d['roofline']['kernels']
print('cfg=2 depth=$d', d['value'], d['ms_per_step'], k['walk_ms'], k['copy_ms'], d['parity'][:13])"
done
done
