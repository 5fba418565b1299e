set -o pipefail
mkdir -p gpurun_out/r04g
for g in 0.96 1.0 0.96 1.0; do
  timeout -k 10 200 python bench.py --gib $g --no-cpu --no-peaks --steps 20 > gpurun_out/r04g/b_$g.json 2> gpurun_out/r04g/b_$g.err || exit 1
  python -c "import json,sys; j=json.loads(open('gpurun_out/r04g/b_$g.json').read().strip().splitlines()[-1]); r=j['roofline']; print('$g', j['config']['blocks_per_gpu'], j['value'], r['kernel_ms_mean'], r['kernels']['walk_ms'], r['kernels']['copy_ms'], j['view_mode']['kernel_ms'])"
done
