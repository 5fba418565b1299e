set -o pipefail
mkdir -p gpurun_out/sector
timeout -k 10 60 ./scripts/sector_probe > gpurun_out/sector/times.txt 2>&1 || exit 1
cat gpurun_out/sector/times.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d gpurun_out/sector/pmc -o run --output-format csv -- ./scripts/sector_probe > gpurun_out/sector/pmc.txt 2>&1 || exit 1
python3 - <<'PY'
import csv, collections
agg=collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open('gpurun_out/sector/pmc/run_counter_collection.csv')):
    agg[r['Kernel_Name'][:40]][r['Counter_Name']].append((int(r['Dispatch_Id']), float(r['Counter_Value'])))
for k,v in agg.items():
    if 'chain' not in k: continue
    print(k)
    for c, lst in sorted(v.items()):
        d=collections.defaultdict(float)
        for i,x in lst: d[i]+=x
        vals=[d[i] for i in sorted(d)]
        print('   ', c, [int(x) for x in vals[:2]])
PY
