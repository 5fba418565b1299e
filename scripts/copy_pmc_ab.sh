#!/bin/bash
# Copy kernel counters across LSMGPU_WSC_ALIGN modes (0 unaligned pieces, 1 aligned chunks per
# entry group, 2 dense chunks, 3 chunks gathered from the block staged in LDS): SQ issue / wait,
# LDS and occupancy counters, L1 -> L2 request counts and latencies, one --pmc pass each.
# Usage (on the GPU box): MODES="3 0" bash scripts/copy_pmc_ab.sh <tag> [config]
set -o pipefail
T=${1:-copypmc}; C=${2:-2}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$T
mkdir -p $O
P="python3 bench.py --no-cpu --no-view --no-peaks --config $C --steps 3 --warmup 1"
for A in ${MODES:-1 0}; do
  for pass in "sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU" \
              "lds SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_LEVEL_WAVES SQ_BUSY_CYCLES SQ_WAVES" \
              "tcp TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum" \
              "ea TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum"; do
    set -- $pass
    name=$1; shift
    LSMGPU_WSC_ALIGN=$A timeout -s KILL 200 rocprofv3 --kernel-trace --pmc "$@" -d $O/${name}_a$A -o run --output-format csv -- $P \
      > $O/${name}_a$A.json 2> $O/${name}_a$A.err || { tail -5 $O/${name}_a$A.err; exit 1; }
  done
done
python3 - $O <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
for f in sorted(glob.glob(f"{d}/*_a*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "wsc_copy" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f.split("/")[-2], {c: round(sum(v) / len(v)) for c, v in acc.items()}, flush=True)
PY
