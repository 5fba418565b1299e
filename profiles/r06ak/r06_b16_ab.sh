# the group walk's backward header reads as one 16-B load (diag, LSMGPU_WSC_B16): parity, then C4
set -o pipefail
O=gpurun_out/${OUT:-r06ak}
mkdir -p $O
LSMGPU_LIB_VARIANT=diag LSMGPU_WSC_B16=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_golden.py -k "not kernel_times" > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for r in 1 2 3; do
for b in 0 1; do
LSMGPU_LIB_VARIANT=diag LSMGPU_WSC_B16=$b timeout -k 10 200 python bench.py --config 4 --no-cpu --no-peaks --steps 50 > $O/c4_b${b}_r$r.json 2>> $O/bench.err || exit 1
python -c "
import json; d=json.load(open('$O/c4_b${b}_r$r.json')); k=d['roofline']['kernels']; v=d.get('view_mode') or {}
print('cfg=4 b16=$b', d['value'], d['ms_per_step'], k['walk_ms'], k['copy_ms'], 'view', v.get('kernel_ms'), d['parity'][:13])"
done
done
