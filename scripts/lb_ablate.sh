#!/bin/bash
# Walk look-back cost: the timing-only variant library liblsmgpu_lb.so honours LSMGPU_ABLATE=1
# (walk tiles skip the decoupled look-back: every tile's base 0, output wrong by design).
set -o pipefail
mkdir -p gpurun_out/lb
for A in 0 1 0 1; do
  LSMGPU_LIB_VARIANT=lb LSMGPU_ABLATE=$A timeout -k 10 120 python bench.py --no-cpu --steps 20 > gpurun_out/lb/b_$A.json 2> gpurun_out/lb/b_$A.err || { tail -5 gpurun_out/lb/b_$A.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/lb/b_$A.json').read().strip().splitlines()[-1]);r=d['roofline'];print('ablate $A mat', r['kernel_ms_mean'], r['kernels']['walk_ms'], r['kernels']['copy_ms'], 'view', d['view_mode']['kernel_ms'])"
done
