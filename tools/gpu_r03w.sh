#!/bin/bash
# Round-3 visit w: C4 tile distribution A/B on one box, alternating (contiguous
# run per wave / block-interleaved / grid-cyclic), both layouts
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "large or full_size or fuzz" --timeout 240 --timeout-method thread > $OUT/pytest_base.log 2>&1 || exit $?
CE_AMD_ILEAVE=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "large or full_size or fuzz" --timeout 240 --timeout-method thread > $OUT/pytest_cyc.log 2>&1 || exit $?
echo "tests ok" >> $OUT/steps.log
for r in 1 2; do
  for v in 0 2 1; do
    for L in NMC MNC; do
      CE_AMD_ILEAVE=$v timeout -k 10 300 python bench.py --no-cpu-baseline --layout $L > $OUT/b_${L}_il${v}_$r.json 2> $OUT/b_${L}_il${v}_$r.err || exit $?
    done
  done
  echo "round $r ok" >> $OUT/steps.log
done
