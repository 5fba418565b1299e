# product library: the GPU suite, then one bench line per config (C2 default, C3, C4, C5)
set -o pipefail
O=gpurun_out/${OUT:-r06t}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1 || { tail -30 $O/gpu_suite.log; exit 1; }
tail -1 $O/gpu_suite.log
for c in 2 3 4 5; do
timeout -k 10 300 python bench.py --config $c --no-cpu --no-peaks --steps 30 > $O/c$c.json 2>> $O/bench.err || exit 1
python -c "
import json; d=json.load(open('$O/c$c.json')); k=d['roofline']['kernels']; e=d['encode']
print('cfg=$c', d['value'], d['ms_per_step'], k['walk_ms'], k['copy_ms'], 'view', d.get('view', {}).get('ms_per_step'), 'enc', e['kernel_ms'], e['frac'], d['parity'][:13])"
done
