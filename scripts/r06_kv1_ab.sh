# the copy pipeline's key and value stores through one resource (diag, LSMGPU_WSC_KV1): parity, C2
# (the knob was removed with the variant after this measurement; the script is the record of profiles/r06am)
set -o pipefail
O=gpurun_out/${OUT:-r06am}
mkdir -p $O
LSMGPU_LIB_VARIANT=diag LSMGPU_WSC_KV1=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py -k "not kernel_times" > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for r in 1 2 3; do
for kv in 0 1; do
LSMGPU_LIB_VARIANT=diag LSMGPU_WSC_KV1=$kv timeout -k 10 200 python bench.py --config 2 --no-cpu --no-peaks --no-view --steps 50 > $O/c2_kv${kv}_r$r.json 2>> $O/bench.err || exit 1
python -c "
import json; d=json.load(open('$O/c2_kv${kv}_r$r.json')); k=d['roofline']['kernels']
print('cfg=2 kv1=$kv', d['value'], d['ms_per_step'], k['walk_ms'], k['copy_ms'], d['parity'][:13])"
done
done
