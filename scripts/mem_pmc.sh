#!/bin/bash
# L1 / TLB / TA / TD stall counters per kernel (walk, copy, and the practical streaming copy and
# read probes as a calibration baseline), one --pmc pass each.
# Usage (on the GPU box): bash scripts/mem_pmc.sh <tag> [config] [gib]
set -o pipefail
T=${1:-mempmc}; C=${2:-2}; G=${3:-1}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$T
mkdir -p $O
P="python3 bench.py --no-cpu --no-view --config $C --gib $G --steps 3 --warmup 1"
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" -d $O/$name -o run --output-format csv -- $P \
    > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
}
pass tcp1 TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum
pass tcp2 TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_PENDING_STALL_CYCLES_sum
pass tcp3 TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_WRITE_TAGCONFLICT_STALL_CYCLES_sum
pass ta2 TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
pass td2 TD_TC_STALL_sum TD_TD_BUSY_sum
pass ta3 TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum
python3 - $O <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
for part in ("tcp1", "tcp2", "tcp3", "ta2", "td2", "ta3"):
    fs = glob.glob(f"{d}/{part}/**/*counter_collection.csv", recursive=True)
    if not fs:
        print(part, "no csv"); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = {}
    for r in csv.DictReader(open(fs[0])):
        k = r["Kernel_Name"]
        if "wsc_" not in k and "stream_" not in k:
            continue
        key = k.split("(")[0][-44:]
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        print(part, k, {c: round(sum(v) / len(v)) for c, v in cs.items()}, flush=True)
PY
