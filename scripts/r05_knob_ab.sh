#!/bin/bash
# Same-box A/B of decode knobs, alternating, two rounds.  Each variant is name=ENV1=v1,ENV2=v2
# ("default" for none).  With STAMPS=1 the stamps library runs instead (per-tile timelines in
# $O/tiles_<name>.txt; times are then not comparable).
# Usage (on the GPU box): bash scripts/r05_knob_ab.sh <tag> <config> <GiB> <variant>...
set -o pipefail
T=$1; CFG=$2; GIB=$3; shift 3
O=gpurun_out/$T
mkdir -p $O
line() {
  python - "$2" "$1" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = j["roofline"]; k = r.get("kernels") or {}; v = j.get("view_mode") or {}
print(sys.argv[2], j["value"], "GiB/s", r["kernel_ms_mean"], "ms | walk", k.get("walk_ms"), "copy",
      k.get("copy_ms"), "| view", v.get("kernel_ms"), j["parity"][:12], flush=True)
PY
}
rounds=2
[ -n "$STAMPS" ] && rounds=1
for r in $(seq $rounds); do
  for v in "$@"; do
    name=${v%%=*}; envs=${v#*=}
    [ "$envs" = "default" ] && envs=""
    extra=()
    if [ -n "$STAMPS" ]; then
      extra=(LSMGPU_LIB_VARIANT=stamps LSMGPU_STAMPS=1 LSMGPU_STAMPS_FILE=$O/tiles_$name.txt)
    fi
    env ${envs//,/ } "${extra[@]}" timeout -k 10 200 python bench.py --config $CFG --gib $GIB --no-cpu \
      --no-peaks --steps ${STEPS:-20} --warmup 2 > $O/bench_${name}_$r.json 2> $O/bench_${name}_$r.err \
      || { tail -20 $O/bench_${name}_$r.err; exit 1; }
    line ${name}_$r $O/bench_${name}_$r.json
  done
done
