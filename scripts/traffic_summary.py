"""HBM bytes per decode launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

MI355X_MICROARCH.md (HBM): both counters are in KiB; on gfx950 FETCH_SIZE reports exactly half
of the bytes of a wide coalesced streaming read -> x2.  WRITE_SIZE is exact for 16-B stores.
Writes profiles/pmc_traffic.json, which bench.py reports as roofline.traffic when the workload
matches.
"""
import csv
import hashlib
import json
import os
import sys


def kernel_values(path, counter):
    rows = list(csv.DictReader(open(path)))
    return [float(r["Counter_Value"]) for r in rows
            if "lsmgpu::decode" in r["Kernel_Name"] and r["Counter_Name"] == counter]


def kernel_name(path):
    for r in csv.DictReader(open(path)):
        if "lsmgpu::decode" in r["Kernel_Name"]:
            return r["Kernel_Name"].split("(")[0]
    return "?"


def lib_sha256():
    """Hash of the liblsmgpu.so that was profiled: bench.py reports the traffic only for it."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "lsmdb_amd", "liblsmgpu.so"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def main():
    fetch_csv, write_csv, bench_json, out = sys.argv[1:5]
    f = kernel_values(fetch_csv, "FETCH_SIZE")
    w = kernel_values(write_csv, "WRITE_SIZE")
    b = json.loads(open(bench_json).read().strip().splitlines()[-1])
    # the timed launches are the last ones (warmup first); take the median of the last 3
    fk = sorted(f[-3:])[len(f[-3:]) // 2]
    wk = sorted(w[-3:])[len(w[-3:]) // 2]
    fetch_b = fk * 1024 * 2
    write_b = wk * 1024
    doc = {
        "kernel": kernel_name(fetch_csv),
        "mode": 1,
        "workload_bytes": int(b["config"]["workload"].split(":")[1].split("B")[0].strip()),
        "fetch_size_kib_raw": fk,
        "write_size_kib_raw": wk,
        "fetch_bytes_corrected": fetch_b,
        "write_bytes": write_b,
        "hbm_bytes_per_launch": int(fetch_b + write_b),
        "algorithmic_bytes_per_launch": b["roofline"]["algorithmic_bytes_per_launch"],
        "ratio_to_algorithmic": round((fetch_b + write_b) / b["roofline"]["algorithmic_bytes_per_launch"], 4),
        "correction": "FETCH_SIZE x2 (gfx950 wide-stream undercount), KiB -> bytes",
        "lib_sha256": lib_sha256(),
    }
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps(doc))


if __name__ == "__main__":
    main()
