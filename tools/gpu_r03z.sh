#!/bin/bash
# Round-3 visit z: C5 wide stream, contiguous item runs vs grid-cyclic items (CE_AMD_ILEAVE=2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
CE_AMD_ILEAVE=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "wide or chunk" --timeout 240 --timeout-method thread > $OUT/pytest_cyc.log 2>&1
rc=$?; echo "cyclic wide tests rc=$rc" >> $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 2; do
    CE_AMD_ILEAVE=$v timeout -k 10 300 python tools/bench_c5.py --items 12000000 --chunk 2000000 > $OUT/c5_il${v}_$r.json 2> $OUT/c5_il${v}_$r.err || exit $?
  done
  echo "round $r ok" >> $OUT/steps.log
done
