#!/bin/bash
# Round-5 same-box A/B: lane-walk tiles of 576 / 256 blocks (LSMGPU_WSC_WIDE) on C2 at 2^30 B
# (1,041 tiles of 256 for 1,024 resident slots), alternating, two rounds.  (profiles/r05d: 576 vs
# 256 at 2^30 B and at round 3's size; profiles/r05e: 384-block tiles too, since removed.)
# Usage (on the GPU box): bash scripts/r05_wide_ab.sh <tag> [config] [GiB]
set -o pipefail
T=${1:-r05wide}
CFG=${2:-2}
O=gpurun_out/$T
mkdir -p $O
line() {
  python - "$2" "$1" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = j["roofline"]; k = r.get("kernels") or {}; v = j.get("view_mode") or {}
print(sys.argv[2], j["config"]["blocks_per_gpu"], "blocks", j["value"], "GiB/s", r["kernel_ms_mean"],
      "ms | walk", k.get("walk_ms"), "copy", k.get("copy_ms"), "| view", v.get("kernel_ms"),
      v.get("read_frac"), flush=True)
PY
}
run() {  # name gib env...
  local name=$1 gib=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --config $CFG --gib $gib --no-cpu --no-peaks --steps 20 \
    > $O/bench_$name.json 2> $O/bench_$name.err || { tail -20 $O/bench_$name.err; exit 1; }
  line $name $O/bench_$name.json
}
GIB=${3:-1.0}
for r in 1 2; do
  run w576_$r $GIB LSMGPU_WSC_WIDE=1
  run w256_$r $GIB LSMGPU_WSC_WIDE=0
done
