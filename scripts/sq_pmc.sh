#!/bin/bash
# SQ / TA / TD counters per decode kernel (walk, copy), one --pmc pass each (MI355X_MICROARCH.md
# slot limits: 8 SQ, 2 TA, 2 TD per pass), plus the gfx950 counter list.
# Usage (on the GPU box): bash scripts/sq_pmc.sh <tag> [config] [gib] [extra bench args]
set -o pipefail
T=${1:-sqpmc}; C=${2:-2}; G=${3:-1}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$T
mkdir -p $O
P="python3 bench.py --no-cpu --no-view --no-peaks --config $C --gib $G --steps 3 --warmup 1 $4"
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc "$@" -d $O/$name -o run --output-format csv -- $P \
    > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
}
pass sq1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU
pass sq2 SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS
pass ta TA_BUSY_avr TA_TA_BUSY_sum
pass td TD_TD_BUSY_sum TD_BUSY_avr
python3 - $O <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
for part in ("sq1", "sq2", "ta", "td"):
    fs = glob.glob(f"{d}/{part}/**/*counter_collection.csv", recursive=True)
    if not fs:
        print(part, "no csv"); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(fs[0])):
        k = r["Kernel_Name"]
        if "wsc_" not in k:
            continue
        acc[k.split("(")[0][-40:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        print(part, k, {c: v[-1] for c, v in cs.items()}, flush=True)
PY
