#!/bin/bash
# Per-kernel counter split for one config (the C5 copy, the encode):
# SQ issue / wait counts, L1 -> L2 request counts and latencies, HBM (EA) request counts, one
# --pmc pass each (slot limits of MI355X_MICROARCH.md), for wsc_copy_kernel, wsc_walk_kernel and
# encode_kernel.  Per-launch averages; EA bytes = 64 B x (RDREQ) / 64 B x WRREQ_64B + 32 B x rest
# (see scripts/traffic_summary.py for the corrected HBM figure).
# Usage (on the GPU box): bash scripts/r05_pmc.sh <tag> [config] [gib]
set -o pipefail
T=${1:-r05pmc}; C=${2:-5}; G=${3:-1}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$T/c$C
mkdir -p $O
P="python3 bench.py --no-cpu --no-view --no-peaks --config $C --gib $G --steps 3 --warmup 1"
for pass in "sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES" \
            "tcp TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum" \
            "ea TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" \
            "tatd TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum TD_BUSY_avr"; do
  set -- $pass
  name=$1; shift
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc "$@" -d $O/$name -o run --output-format csv -- $P \
    > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
done
python3 - $O <<'PY'
import csv, glob, os, sys, collections
d = sys.argv[1]
for f in sorted(glob.glob(f"{d}/*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if not any(s in k for s in ("wsc_copy", "wsc_walk", "encode_kernel")):
            continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in sorted(acc.items()):
        print(os.path.relpath(f, d).split("/")[0], k,
              {c: round(sum(v) / len(v)) for c, v in cs.items()}, flush=True)
PY
