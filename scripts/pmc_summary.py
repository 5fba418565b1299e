"""Per-block instruction counts of the decode kernel from a rocprofv3 --pmc CSV."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
nblk = int(sys.argv[2]) if len(sys.argv) > 2 else 256991
by = collections.defaultdict(dict)
for r in rows:
    if "decode_kernel" in r["Kernel_Name"]:
        by[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
        by[r["Dispatch_Id"]]["_us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
v = list(by.values())[-1]
print("kernel us %.1f  per block: VALU %.0f SALU %.0f LDS %.0f VMEM %.0f" % (
    v["_us"], v["SQ_INSTS_VALU"] / nblk, v["SQ_INSTS_SALU"] / nblk, v["SQ_INSTS_LDS"] / nblk,
    v["SQ_INSTS_VMEM"] / nblk))
