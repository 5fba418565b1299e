#!/bin/bash
# Same-box A/B of two in-tree libraries (LSMGPU_LIB_VARIANT: "" = liblsmgpu.so, else
# liblsmgpu_<variant>.so), alternating, two rounds, over the given configs.
# Usage (GPU box): bash scripts/r06_lib_ab.sh <tag> "<configs>" "<variantA> <variantB>" [extra bench args]
set -o pipefail
T=$1; CFGS=${2:-"2 5"}; VARS=${3:-"pre cur"}; shift 3
O=gpurun_out/$T
mkdir -p $O
for r in 1 2; do
for c in $CFGS; do
for v in $VARS; do
  if [ "$v" = "cur" ]; then unset LSMGPU_LIB_VARIANT; else export LSMGPU_LIB_VARIANT=$v; fi
  timeout -k 10 300 python bench.py --config $c --no-cpu --no-peaks ${NOVIEW---no-view} --steps 20 "$@" > $O/c${c}_${v}_r$r.json 2>> $O/bench.err || { echo "bench failed: c$c $v"; exit 1; }
  python -c "import json;d=json.loads(open('$O/c${c}_${v}_r$r.json').read().strip().splitlines()[-1]);k=d['roofline']['kernels'];print('C$c $v r$r', d['ms_per_step'], d['value'], k['walk_ms'], k['copy_ms'], d['encode']['kernel_ms'], (d.get('view_mode') or {}).get('kernel_ms'), d['parity'][:13])"
done
done
done
unset LSMGPU_LIB_VARIANT
