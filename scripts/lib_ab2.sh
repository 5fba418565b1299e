#!/bin/bash
# Library A/B on one box: lsmdb_amd/liblsmgpu.so (new) vs lsmdb_amd/liblsmgpu_prev.so, alternating,
# after the GPU parity suites on the new library.  Usage: bash scripts/lib_ab2.sh <tag> [configs]
set -o pipefail
T=gpurun_out/${1:-libab}
mkdir -p $T
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_table.py tests/test_gpu_shim.py -x -q --timeout 120 --timeout-method thread > $T/tests.log 2>&1 || { tail -30 $T/tests.log; exit 1; }
tail -1 $T/tests.log
cp lsmdb_amd/liblsmgpu.so $T/new.so
run() {  # lib cfg round
  cp $T/$1.so lsmdb_amd/liblsmgpu.so
  timeout -k 10 150 python bench.py --no-cpu --no-peaks --config $2 > $T/c$2_$1_$3.json 2> $T/c$2_$1_$3.err || { tail -20 $T/c$2_$1_$3.err; exit 1; }
  python -c "import json;j=json.load(open('$T/c$2_$1_$3.json'));k=j['roofline']['kernels'];print('C$2 $1',j['value'],j['ms_per_step'],k['walk_ms'],k['copy_ms'],'view',j['view_mode']['kernel_ms'],j['parity'][:14])"
}
cp lsmdb_amd/liblsmgpu_prev.so $T/prev.so
for c in ${2:-2 2 5 3 4}; do for l in new prev; do run $l $c $RANDOM || exit 1; done; done
cp $T/new.so lsmdb_amd/liblsmgpu.so
