#!/bin/bash
# Round-5 same-box A/B of the copy's store patterns (LSMGPU_WSC_ALIGN: 0 the unaligned pieces,
# the default; 1 aligned chunks per entry group; 2 dense aligned chunks), alternating, two rounds.
# Usage (on the GPU box): bash scripts/r05_align_ab.sh <tag> [config] [GiB] [modes, e.g. "0 2"]
set -o pipefail
T=${1:-r05align}; CFG=${2:-2}; GIB=${3:-1.0}; MODES=${4:-"0 2"}
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
  for m in $MODES; do run align${m}_$r LSMGPU_WSC_ALIGN=$m; done
done
