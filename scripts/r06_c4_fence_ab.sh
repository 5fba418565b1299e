# C4 copy-fusion A/B on the diagnostic build (timing only): fused with the agent release /
# acquire per tile, fused without them (LSMGPU_ABLATE=512, unsafe: measurement only), unfused
set -o pipefail
O=gpurun_out/r06f
mkdir -p $O
export LSMGPU_LIB_VARIANT=diag
for r in 1 2; do
for v in "fence:LSMGPU_WSC_COPYFUSE=1" "nofence:LSMGPU_WSC_COPYFUSE=1 LSMGPU_ABLATE=512" "launch:LSMGPU_WSC_COPYFUSE=0"; do
n=${v%%:*}; e=${v#*:}
env $e timeout -k 10 200 python bench.py --config 4 --no-cpu --no-peaks --no-view --steps 50 > $O/c4_${n}_r$r.json 2>> $O/bench.err || exit 1
python -c "import json;d=json.loads(open('$O/c4_${n}_r$r.json').read().strip().splitlines()[-1]);print('$n', d['ms_per_step'], d['value'], d['roofline']['kernels']['walk_ms'], d['roofline']['kernels']['copy_ms'], d['parity'])"
done
done
