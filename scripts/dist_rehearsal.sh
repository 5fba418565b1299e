#!/bin/bash
# Rehearse bench.py's multi-GPU contract on a ONE-GPU box: torch.distributed.run with N ranks,
# every rank on device 0 and gloo instead of RCCL (RCCL refuses two ranks on one GPU).  The
# round-end driver runs the real N = 1/2/4/8 on an 8-GPU node with RCCL.
set -o pipefail
N=${N:-2}
mkdir -p gpurun_out/dist
BENCH_DIST_BACKEND=gloo BENCH_DEVICE_OVERRIDE=0 timeout -k 10 300 python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus $N --steps 5 --warmup 1 > gpurun_out/dist/n$N.json 2> gpurun_out/dist/n$N.err || { tail -20 gpurun_out/dist/n$N.err; exit 1; }
cat gpurun_out/dist/n$N.json
