#!/bin/bash
# Round-5 same-box A/B: the round-3 library (8753d61, built as
# lsmdb_amd/liblsmgpu_r03.so) against the current one, each on C2 at round 3's size
# (1,035,769,950 B = 1,004 walk tiles, all resident) and at 2^30 B (1,041 tiles for 1,024
# resident workgroup slots), alternating, two rounds.  Separates shard size from code.
# Usage (on the GPU box): bash scripts/r05_walk_ab.sh <tag> [extra env for the HEAD runs]
set -o pipefail
T=${1:-r05ab}
O=gpurun_out/$T
mkdir -p $O
line() {
  python - "$2" "$1" <<'EOF'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = j["roofline"]; k = r.get("kernels") or {}
print(sys.argv[2], j["config"]["blocks_per_gpu"], "blocks", j["value"], "GiB/s", r["kernel_ms_mean"],
      "ms | walk", k.get("walk_ms"), "copy", k.get("copy_ms"), "| view",
      (j.get("view_mode") or {}).get("kernel_ms"), flush=True)
EOF
}
run() {  # name gib env...
  local name=$1 gib=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --config 2 --gib $gib --no-cpu --no-peaks --steps 20 \
    > $O/bench_$name.json 2> $O/bench_$name.err || { tail -20 $O/bench_$name.err; exit 1; }
  line $name $O/bench_$name.json
}
for r in 1 2; do
  run head_r03size_$r 0.96464 $2
  run r03_r03size_$r 0.96464 LSMGPU_LIB_VARIANT=r03
  run head_2p30_$r 1.0 $2
  run r03_2p30_$r 1.0 LSMGPU_LIB_VARIANT=r03
done
