# 100-entry (C4-shaped) blocks in a large batch: the compaction replay's decode of 1 + 8 tables
# (48 K blocks) with the copy pipeline for blocks of >= 64 entries (diag, LSMGPU_WSC_PIPE=2) or not
set -o pipefail
O=gpurun_out/${OUT:-r06w}
mkdir -p $O
for r in 1 2 3; do
for pipe in 1 2; do
LSMGPU_LIB_VARIANT=diag LSMGPU_WSC_PIPE=$pipe timeout -k 10 300 python scripts/compaction_bench.py > $O/cb_p${pipe}_r$r.json 2>> $O/cb.err || exit 1
python -c "
import json; d=json.load(open('$O/cb_p${pipe}_r$r.json')); print('pipe=$pipe decode', d['decode_ms'], 'total', d['total_ms'], d['merge_matches_oracle'])"
done
done
