#!/bin/bash
# stamps (diagnostic build) + PMC instruction mix of the decode kernel
set -o pipefail
mkdir -p gpurun_out/diag
for a in 0 3; do
  LSMGPU_LIB_VARIANT=stamps LSMGPU_ABLATE=$a LSMGPU_STAMPS=1 timeout -k 10 60 python bench.py --no-cpu --no-view --steps 1 --warmup 1 2> gpurun_out/diag/st$a.err > /dev/null || exit 1
  echo "ablate $a: $(grep stamps gpurun_out/diag/st$a.err | tail -1)"
done
[ -n "$PMC" ] && bash scripts/pmc_decode.sh gpurun_out/diag/pmc && python scripts/pmc_summary.py gpurun_out/diag/pmc/a/run_counter_collection.csv gpurun_out/diag/pmc/b/run_counter_collection.csv
