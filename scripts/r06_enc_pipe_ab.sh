# encode_pipe_kernel A/B (diag build, LSMGPU_ENC_PIPE): parity first, then C2 / C3 / C5 encode
# times alternating on one box
set -o pipefail
O=gpurun_out/${OUT:-r06o}
mkdir -p $O
LSMGPU_LIB_VARIANT=diag timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "encode_pipe_kernel or encode_template or encode_kat or encode_decode_vs" \
  > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
for c in 2 5 3; do
for r in 1 2; do
for pipe in 0 1 2; do
LSMGPU_LIB_VARIANT=diag LSMGPU_ENC_PIPE=$pipe timeout -k 10 200 python bench.py --config $c --no-cpu --no-peaks --no-view --steps 10 > $O/c${c}_p${pipe}_r$r.json 2>> $O/bench.err || exit 1
python -c "
import json; d=json.load(open('$O/c${c}_p${pipe}_r$r.json')); e=d['encode']
print('cfg=$c pipe=$pipe', e['kernel_ms'], e['frac'], e['identical_to_decoded_shard'], d['parity'][:13])"
done
done
done
