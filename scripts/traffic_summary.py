"""HBM-side bytes per decode launch from rocprofv3 --pmc passes, summed over every kernel of
the decode pipeline (walk-scan-copy: wsc_walk_kernel + rocPRIM scan of the Tri64 triples +
wsc_copy_kernel; the single-kernel paths: lsmgpu::decode*/tile_decode).

Reads are counted by request size -- TCC_EA0_RDREQ_{32B,64B,128B} x {32, 64, 128} B -- so no
access-width calibration is assumed (MI355X_MICROARCH.md: FETCH_SIZE tallies 128-B requests at
64 B; only wide streaming reads are calibrated).  Writes: TCC_EA0_WRREQ_64B x 64 B + the other
write requests x 32 B.  FETCH_SIZE x 2 and WRITE_SIZE are kept beside them as a cross-check.
Infinity-Cache hits are counted, not excluded (guide): the TCC_EA0 counters are the L2's requests
to the fabric, whichever of the Infinity Cache or HBM serves them -- at 1 GiB of input the walk's
and the copy's reads of the same lines cannot both stay in the 256 MiB cache, and the one-pass
kernel's walk / copy re-reads that miss L2 are counted though the Infinity Cache serves them.

usage: traffic_summary.py <rd.csv> <wr.csv> <fetch.csv> <write.csv> <bench.json> <out.json>
"""
import csv
import hashlib
import json
import os
import sys

PIPELINE = ("lsmgpu::decode", "wsc_walk_kernel", "wsc_walk_persist_kernel", "wsc_copy_kernel", "wsc_carry_kernel", "Tri64",
            "tile_decode_kernel", "fsw_kernel", "fsc_kernel")
# not part of a materialize decode: the view-only walk (kWalkLaneView = 3) that bench.py's
# walk_fetch_bytes runs once to price the walk
EXCLUDE = ("wsc_walk_kernel<3,",)


def in_pipeline(name):
    return any(k in name for k in PIPELINE) and not any(k in name for k in EXCLUDE)


def per_launch(path, counters):
    """{counter: value per decode launch}: per kernel name the median of its last 3 dispatches
    (the timed launches come last), summed over the pipeline's kernels."""
    vals = {}  # counter -> kernel name -> dispatch id -> value
    for r in csv.DictReader(open(path)):
        name, c = r["Kernel_Name"], r["Counter_Name"]
        if c in counters and in_pipeline(name):
            d = vals.setdefault(c, {}).setdefault(name, {})
            d[int(r["Dispatch_Id"])] = d.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    out = {}
    for c in counters:
        tot = 0.0
        for name, disp in vals.get(c, {}).items():
            v = [disp[k] for k in sorted(disp)][-3:]
            tot += sorted(v)[len(v) // 2]
        out[c] = tot
    return out


def kernels(path):
    names = []
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if in_pipeline(n):
            short = n.split("(")[0][:90]
            if short not in names:
                names.append(short)
    return names


def lib_sha256():
    """Hash of the liblsmgpu.so that was profiled: bench.py reports the traffic only for it."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "lsmdb_amd", "liblsmgpu.so"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def main():
    rd_csv, wr_csv, fetch_csv, write_csv, bench_json, out = sys.argv[1:7]
    rd = per_launch(rd_csv, ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum",
                             "TCC_EA0_RDREQ_128B_sum"))
    wr = per_launch(wr_csv, ("TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum"))
    fs = per_launch(fetch_csv, ("FETCH_SIZE",))["FETCH_SIZE"]
    ws = per_launch(write_csv, ("WRITE_SIZE",))["WRITE_SIZE"]
    b = json.loads(open(bench_json).read().strip().splitlines()[-1])
    r32, r64, r128 = rd["TCC_EA0_RDREQ_32B_sum"], rd["TCC_EA0_RDREQ_64B_sum"], rd["TCC_EA0_RDREQ_128B_sum"]
    read_b = 32 * r32 + 64 * r64 + 128 * r128
    w64 = wr["TCC_EA0_WRREQ_64B_sum"]
    write_b = 64 * w64 + 32 * max(0.0, wr["TCC_EA0_WRREQ_sum"] - w64)
    alg = b["roofline"]["algorithmic_bytes_per_launch"]
    doc = {
        "kernels": kernels(rd_csv),
        "mode": 1,
        "workload_bytes": int(b["config"]["workload"].split(":")[1].split("B")[0].strip()),
        "rdreq": rd,
        "wrreq": wr,
        "read_bytes": int(read_b),
        "write_bytes": int(write_b),
        "hbm_bytes_per_launch": int(read_b + write_b),
        "algorithmic_bytes_per_launch": alg,
        "ratio_to_algorithmic": round((read_b + write_b) / alg, 4),
        "cross_check": {"fetch_size_kib": fs, "fetch_x2_bytes": int(fs * 2048),
                        "write_size_kib": ws, "write_bytes": int(ws * 1024)},
        "method": "reads 32/64/128 B x TCC_EA0_RDREQ_{32B,64B,128B}_sum; writes 64 B x WRREQ_64B + "
                  "32 B x other WRREQ; per kernel median of the last 3 dispatches, summed over the "
                  "decode pipeline",
        "lib_sha256": lib_sha256(),
    }
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps(doc))


if __name__ == "__main__":
    main()
