#!/bin/bash
# HBM traffic per decode kernel on another config (TCC_EA0 read / write request passes)
# Usage: bash scripts/cfg_pmc.sh <tag> <config> [gib]
set -o pipefail
T=${1:-cfgpmc}; C=${2:-5}; G=${3:-1}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$T
P="python3 bench.py --no-cpu --no-view --config $C --gib $G --steps 3 --warmup 1"
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d gpurun_out/$T/rd -o run --output-format csv -- $P > gpurun_out/$T/rd.json 2> gpurun_out/$T/rd.err || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d gpurun_out/$T/wr -o run --output-format csv -- $P > gpurun_out/$T/wr.json 2> gpurun_out/$T/wr.err || exit 1
python3 - gpurun_out/$T <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
for part in ("rd", "wr"):
    f = glob.glob(f"{d}/{part}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "wsc_" not in k:
            continue
        acc[k.split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        print(part, k, {c: v[-1] for c, v in cs.items()})
PY
