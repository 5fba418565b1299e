# the pipelined dense mapping for small entries too (diag, LSMGPU_WSC_DMIN=0): C4 and C2
set -o pipefail
O=gpurun_out/${OUT:-r06y}
mkdir -p $O
LSMGPU_LIB_VARIANT=diag LSMGPU_WSC_DMIN=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_golden.py > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for c in 4 2; do
for r in 1 2; do
for dm in 128 0; do
LSMGPU_LIB_VARIANT=diag LSMGPU_WSC_DMIN=$dm timeout -k 10 200 python bench.py --config $c --no-cpu --no-peaks --no-view --steps 30 > $O/c${c}_dm${dm}_r$r.json 2>> $O/bench.err || exit 1
python -c "
import json; d=json.load(open('$O/c${c}_dm${dm}_r$r.json')); k=d['roofline']['kernels']
print('cfg=$c dmin=$dm', d['value'], d['ms_per_step'], k['walk_ms'], k['copy_ms'], d['parity'][:13])"
done
done
done
