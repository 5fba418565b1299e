# copy_entries_dense_pipe A/B (diag build, LSMGPU_WSC_DPIPE): parity first, then C5 decode
# alternating on one box
set -o pipefail
O=gpurun_out/${OUT:-r06r}
mkdir -p $O
LSMGPU_LIB_VARIANT=diag LSMGPU_WSC_DPIPE=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py \
  > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
for c in 5; do
for r in 1 2 3; do
for pipe in 0 1; do
LSMGPU_LIB_VARIANT=diag LSMGPU_WSC_DPIPE=$pipe timeout -k 10 200 python bench.py --config $c --no-cpu --no-peaks --no-view --steps 30 > $O/c${c}_p${pipe}_r$r.json 2>> $O/bench.err || exit 1
python -c "
import json; d=json.load(open('$O/c${c}_p${pipe}_r$r.json')); k=d['roofline']['kernels']
print('cfg=$c dpipe=$pipe', d['value'], d['ms_per_step'], k['walk_ms'], k['copy_ms'], d['parity'][:13])"
done
done
done
