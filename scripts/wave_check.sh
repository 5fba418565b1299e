#!/bin/bash
# Ring walk (LSMGPU_WSC_WALK=wave): parity, then C2 1 GiB A/B against the lane walk, plus the
# loader alone (LSMGPU_ABLATE=4, timing only) and rocprofv3 kernel stats.
set -o pipefail
T=${1:-wave}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "walk_modes or walk_adversarial" > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
for w in lane wave; do
  LSMGPU_WSC_WALK=$w timeout -k 10 150 python bench.py --no-cpu > gpurun_out/$T/b_$w.json 2> gpurun_out/$T/b_$w.err || { tail -20 gpurun_out/$T/b_$w.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/$T/b_$w.json'));k=j['roofline']['kernels'];print('$w',j['value'],j['ms_per_step'],k['walk_ms'],k['copy_ms'],j['view_mode']['kernel_ms'],j['parity'])"
done
LSMGPU_ABLATE=4 LSMGPU_WSC_WALK=wave timeout -k 10 150 python bench.py --no-cpu > gpurun_out/$T/b_wave_ablate4.json 2> gpurun_out/$T/b_wave_ablate4.err
python -c "import json;j=json.load(open('gpurun_out/$T/b_wave_ablate4.json'));k=j['roofline']['kernels'];print('wave loader only',k['walk_ms'],j['view_mode']['kernel_ms'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
LSMGPU_WSC_WALK=wave timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-view > gpurun_out/$T/prof.json 2> gpurun_out/$T/prof.err || exit 1
find gpurun_out/$T/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-4 {} | head -8'
