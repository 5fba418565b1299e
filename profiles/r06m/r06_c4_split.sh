# C4 copy: waves per block (diag build, LSMGPU_WSC_SPLIT), two rounds, same box
set -o pipefail
O=gpurun_out/r06m
mkdir -p $O
for r in 1 2; do
for sp in 2 4 1; do
LSMGPU_LIB_VARIANT=diag LSMGPU_WSC_SPLIT=$sp timeout -k 10 200 python bench.py --config 4 --no-cpu --no-peaks --no-view --steps 50 > $O/c4_s${sp}_r$r.json 2>> $O/bench.err || exit 1
python -c "import json;d=json.loads(open('$O/c4_s${sp}_r$r.json').read().strip().splitlines()[-1]);k=d['roofline']['kernels'];print('split=$sp', d['ms_per_step'], d['roofline']['kernel_ms_mean'], k['walk_ms'], k['copy_ms'], d['parity'][:13])"
done
done
