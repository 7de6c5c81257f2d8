#!/bin/bash
# Round-3 visit x: C4 item-major tile distribution A/B (contiguous runs vs grid-cyclic), alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for r in 1 2 3; do
  for v in 0 2; do
    CE_AMD_ILEAVE=$v timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/b_NMC_il${v}_$r.json 2> $OUT/b_NMC_il${v}_$r.err || exit $?
  done
  echo "round $r ok" >> $OUT/steps.log
done
