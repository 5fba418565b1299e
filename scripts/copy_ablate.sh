set -o pipefail
# NOTE: LSMGPU_ABLATE bits 8 / 16 / 32 (skip key pieces / value pieces / end-offset stores in
# copy_entries) existed only in an experiment build (profiles/r03m/README); the library ignores them.
T=gpurun_out/ablcopy; mkdir -p $T
for a in 0 8 16 32 24 0; do
  LSMGPU_ABLATE=$a timeout -k 10 150 python bench.py --no-cpu --no-peaks --no-view > $T/a$a.json 2> $T/a$a.err || { tail -5 $T/a$a.err; exit 1; }
  python -c "import json;j=json.load(open('$T/a$a.json'));k=j['roofline']['kernels'];print('ablate $a',j['ms_per_step'],k['walk_ms'],k['copy_ms'])"
done
