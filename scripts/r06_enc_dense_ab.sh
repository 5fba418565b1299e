# encode_dense_kernel A/B (diag, LSMGPU_ENC_DENSE): parity, then C5 / C3 encode times
set -o pipefail
O=gpurun_out/${OUT:-r06ab}
mkdir -p $O
LSMGPU_LIB_VARIANT=diag LSMGPU_ENC_DENSE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "encode" tests/test_gpu_golden.py tests/test_gpu_compaction.py > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for c in 5 3; do
for r in 1 2; do
for dn in 0 1; do
LSMGPU_LIB_VARIANT=diag LSMGPU_ENC_DENSE=$dn timeout -k 10 200 python bench.py --config $c --no-cpu --no-peaks --no-view --steps 10 > $O/c${c}_d${dn}_r$r.json 2>> $O/bench.err || exit 1
python -c "
import json; d=json.load(open('$O/c${c}_d${dn}_r$r.json')); e=d['encode']
print('cfg=$c dense=$dn', e['kernel_ms'], e['frac'], e['identical_to_decoded_shard'], d['parity'][:13])"
done
done
done
