# the lane walk with a backward lane per block (diag, LSMGPU_WSC_LBIDIR=1): parity with the lane
# walk forced, then C5 and the compaction replay's decode (48 K blocks of 100 entries)
set -o pipefail
O=gpurun_out/${OUT:-r06ai}
mkdir -p $O
LSMGPU_LIB_VARIANT=diag LSMGPU_WSC_WALK=lane LSMGPU_WSC_LBIDIR=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_golden.py -k "not kernel_times" > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for r in 1 2; do
for bi in 0 1; do
LSMGPU_LIB_VARIANT=diag LSMGPU_WSC_LBIDIR=$bi timeout -k 10 200 python bench.py --config 5 --no-cpu --no-peaks --steps 30 > $O/c5_bi${bi}_r$r.json 2>> $O/bench.err || exit 1
python -c "
import json; d=json.load(open('$O/c5_bi${bi}_r$r.json')); k=d['roofline']['kernels']; v=d.get('view_mode') or {}
print('cfg=5 lbidir=$bi', d['value'], d['ms_per_step'], k['walk_ms'], k['copy_ms'], 'view', v.get('kernel_ms'), d['parity'][:13])"
LSMGPU_LIB_VARIANT=diag LSMGPU_WSC_LBIDIR=$bi timeout -k 10 300 python scripts/compaction_bench.py > $O/cb_bi${bi}_r$r.json 2>> $O/cb.err || exit 1
python -c "
import json; d=json.load(open('$O/cb_bi${bi}_r$r.json')); print('compaction lbidir=$bi decode', d['decode_ms'], 'total', d['total_ms'], d['merge_matches_oracle'])"
done
done
