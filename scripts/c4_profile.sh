set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c4p
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c4p/prof -o c4 -- python bench.py --no-cpu --no-view --config 4 --gib 0.0625 --steps 10 > gpurun_out/c4p/c4.json 2> gpurun_out/c4p/c4.err || exit 1
python scripts/bench_brief.py gpurun_out/c4p/c4.json
for p in wsc reg lds; do
  LSMGPU_DECODE_PATH=$p timeout -k 10 120 python bench.py --no-cpu --no-view --config 1 --gib 0.00125 --steps 20 > gpurun_out/c4p/c1_$p.json 2> gpurun_out/c4p/c1_$p.err || exit 1
  echo "C1 $p"; python scripts/bench_brief.py gpurun_out/c4p/c1_$p.json
done
