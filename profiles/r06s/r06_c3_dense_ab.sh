# C3 (1.1 KB entries): the 16-lane groups vs the pipelined dense mapping (diag, LSMGPU_WSC_DMAX)
set -o pipefail
O=gpurun_out/${OUT:-r06s}
mkdir -p $O
for r in 1 2; do
for dm in 512 4096; do
LSMGPU_LIB_VARIANT=diag LSMGPU_WSC_DMAX=$dm timeout -k 10 200 python bench.py --config 3 --no-cpu --no-peaks --no-view --steps 30 > $O/c3_dm${dm}_r$r.json 2>> $O/bench.err || exit 1
python -c "
import json; d=json.load(open('$O/c3_dm${dm}_r$r.json')); k=d['roofline']['kernels']
print('cfg=3 dmax=$dm', d['value'], d['ms_per_step'], k['walk_ms'], k['copy_ms'], d['parity'][:13])"
done
done
