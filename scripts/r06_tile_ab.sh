# lane-walk tiles of 128 / 64 blocks for batches with fewer 256-block tiles than CUs (C5 2^30 B):
# parity with the lane walk forced at each tile size (diag), then C5 at 256 / 128 / 64
set -o pipefail
O=gpurun_out/${OUT:-r06z}
mkdir -p $O
for t in 64 128; do
LSMGPU_LIB_VARIANT=diag LSMGPU_WSC_WALK=lane LSMGPU_WSC_TILE=$t timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_golden.py -k "not kernel_times" > $O/parity_t$t.log 2>&1 || { tail -30 $O/parity_t$t.log; exit 1; }
tail -1 $O/parity_t$t.log
done
for r in 1 2; do
for t in 256 128 64; do
LSMGPU_LIB_VARIANT=diag LSMGPU_WSC_TILE=$t timeout -k 10 200 python bench.py --config 5 --no-cpu --no-peaks --steps 30 > $O/c5_t${t}_r$r.json 2>> $O/bench.err || exit 1
python -c "
import json; d=json.load(open('$O/c5_t${t}_r$r.json')); k=d['roofline']['kernels']; v=d.get('view_mode') or {}
print('cfg=5 tile=$t', d['value'], d['ms_per_step'], k['walk_ms'], k['copy_ms'], 'view', v.get('kernel_ms'), d['parity'][:13])"
done
done
