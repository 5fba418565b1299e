#!/bin/bash
# Round-4 same-box A/B: walk-scan-copy knobs (flush chunk), the E2E host pipeline through the C
# ABI, and the other configs.  (The one-pass decode's phase stamps of profiles/r04c came from
# this script's removed "s" part.)
# Usage (on the GPU box): bash scripts/r04_ab.sh <tag> [parts]   parts: any of t a g s v e c (default all)
set -o pipefail
T=${1:-r04ab}
PARTS=${2:-"t a e c"}
O=gpurun_out/$T
mkdir -p $O
has() { [[ " $PARTS " == *" $1 "* ]]; }
line() {  # name json: one summary line
  python - "$2" "$1" <<'EOF'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = j["roofline"]; k = r.get("kernels") or {}
print(sys.argv[2], j["value"], "GiB/s", r["kernel_ms_mean"], "ms | walk", k.get("walk_ms"), "copy",
      k.get("copy_ms"), "| view", (j.get("view_mode") or {}).get("kernel_ms"), "ms",
      (j.get("view_mode") or {}).get("read_frac"))
EOF
}
run() {  # name config env...
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --config $cfg --no-cpu --no-peaks --steps 20 \
    > $O/bench_$name.json 2> $O/bench_$name.err || { tail -20 $O/bench_$name.err; exit 1; }
  line $name $O/bench_$name.json
}
if has t; then
  timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "walk_modes or many_tiles or forced or adversarial or mixed_copy or view_only" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
if has a; then
  run c2 2
  run c2_t192 2 LSMGPU_WSC_TILE=192
  run c2b 2
  run c2_t192b 2 LSMGPU_WSC_TILE=192
fi
if has g; then  # C4 (5,700 blocks: the group walk) -- one or two walk directions
  run c4 4
  run c4b 4
fi
if has s; then  # C2 through the staged 64-lane walk with 4.25 KiB slots (one read of the input)
  run c2_g64s 2 LSMGPU_WSC_WALK=group64 LSMGPU_WSC_SLOT=small
  run c2_g64snc 2 LSMGPU_WSC_WALK=group64 LSMGPU_WSC_SLOT=small LSMGPU_WSC_STAGECOPY=0
fi
if has v; then  # C2 view epilogue: owners by binary search vs scatter + max-scan
  run c2 2
  run c2_vsearch 2 LSMGPU_WSC_VIEWSCAN=0
  run c2b 2
  run c2_vsearchb 2 LSMGPU_WSC_VIEWSCAN=0
fi
if has e; then
  timeout -k 10 300 python scripts/e2e_abi.py > $O/e2e.json 2> $O/e2e.err || { tail -20 $O/e2e.err; exit 1; }
  cat $O/e2e.json
fi
if has c; then
  for cfg in 3 4 5; do
    run c${cfg} $cfg
  done
fi
