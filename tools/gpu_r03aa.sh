#!/bin/bash
# Round-3 visit aa: fused frames, grid-cyclic steps (default) vs a run per wave (CE_AMD_ILEAVE=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x -k "frames" --timeout 300 --timeout-method thread > $OUT/pytest_frames.log 2>&1
rc=$?; echo "frames tests rc=$rc" >> $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 2 0; do
    CE_AMD_ILEAVE=$v timeout -k 10 300 python3 tools/bench_configs.py --only 8 > $OUT/configs8_il${v}_$r.log 2>&1 || exit $?
  done
  echo "round $r ok" >> $OUT/steps.log
done
