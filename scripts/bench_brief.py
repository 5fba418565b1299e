"""One-line summary of a bench.py JSON line."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(d["config"]["workload"].split(":")[0], "value", d["value"], d["unit"], "kernel_ms",
      r["kernel_ms_mean"], "frac", r["frac"], "blocks", d["config"]["blocks_per_gpu"],
      "max_block", d["config"]["max_block_bytes"], d["parity"][:14])
if "encode" in d:
    e = d["encode"]
    print("  encode", e["gibs_per_gpu"], "GiB/s", "ms", e["kernel_ms"], "frac", e["frac"],
          "identical", e["identical_to_decoded_shard"])
