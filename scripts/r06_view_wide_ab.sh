# view decode (C2) with the 256-block kept tiles (LSMGPU_WSC_WIDE=0, a product test hook) vs the
# default 576-block ones, alternating, two rounds
set -o pipefail
O=gpurun_out/${OUT:-r06aq}
mkdir -p $O
for r in 1 2; do
for w in d 0; do
  if [ "$w" = d ]; then unset LSMGPU_WSC_WIDE; else export LSMGPU_WSC_WIDE=$w; fi
  timeout -k 10 200 python bench.py --config 2 --no-cpu --no-peaks --steps 30 > $O/c2_w${w}_r$r.json 2>> $O/bench.err || exit 1
  python -c "
import json; d=json.loads(open('$O/c2_w${w}_r$r.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels']; v=d.get('view_mode') or {}
print('C2 wide=$w r$r', d['ms_per_step'], k['walk_ms'], k['copy_ms'], 'view', v.get('kernel_ms'), d['parity'][:13])"
done
done
unset LSMGPU_WSC_WIDE
