#!/bin/bash
# Round-5 same-box A/B: the copy's aligned 16-B output chunks (LSMGPU_WSC_ALIGN=1, default off) vs
# the unaligned pieces, alternating, two rounds, on the given config.
# Usage (on the GPU box): bash scripts/r05_align_ab.sh <tag> [config] [GiB]
set -o pipefail
T=${1:-r05align}; CFG=${2:-2}; GIB=${3:-1.0}
O=gpurun_out/$T
mkdir -p $O
line() {
  python - "$2" "$1" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = j["roofline"]; k = r.get("kernels") or {}; v = j.get("view_mode") or {}; e = j.get("encode") or {}
print(sys.argv[2], j["config"]["blocks_per_gpu"], "blocks", j["value"], "GiB/s", r["kernel_ms_mean"],
      "ms | walk", k.get("walk_ms"), "copy", k.get("copy_ms"), k.get("copy_frac"), "| view", v.get("kernel_ms"),
      "| encode", e.get("kernel_ms"), j["parity"][:12], flush=True)
PY
}
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --config $CFG --gib $GIB --no-cpu --no-peaks --steps 20 \
    > $O/bench_$name.json 2> $O/bench_$name.err || { tail -20 $O/bench_$name.err; exit 1; }
  line $name $O/bench_$name.json
}
for r in 1 2; do
  run align_$r LSMGPU_WSC_ALIGN=1
  run pieces_$r LSMGPU_WSC_ALIGN=0
done
