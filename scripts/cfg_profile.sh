#!/bin/bash
# per-kernel times (rocprofv3 kernel stats) of the decode on other BASELINE configs
# Usage: bash scripts/cfg_profile.sh <tag>   (CONFIGS="5 4" by default)
set -o pipefail
T=${1:-cfgp}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$T
for c in ${CONFIGS:-5 4}; do
  g=1
  [ "$c" = 4 ] && g=0.0625
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/c$c -o c$c --output-format csv -- python3 bench.py --no-cpu --no-view --config $c --gib $g --steps 10 > gpurun_out/$T/c$c.json 2> gpurun_out/$T/c$c.err || exit 1
  echo "== C$c"; python scripts/bench_brief.py gpurun_out/$T/c$c.json | head -1
  f=$(find gpurun_out/$T/c$c -name "*kernel_stats.csv" | head -1)
  grep -E "wsc_|decode" $f | cut -d, -f1-4
done
