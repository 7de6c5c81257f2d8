#!/bin/bash
# Round-3 visit s: f64 small pools with 4 member loads per batch (UNR 4, item slots throttled) A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
D=$ROOT/tools/_diag
CE_AMD_LIB=$D/libce_amd_u4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_selector.py -q -x --timeout 240 --timeout-method thread > $OUT/pytest_u4.log 2>&1
rc=$?; echo "u4 tests rc=$rc" >> $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  TAG=def${r}_ CFGS="c1 c2hc c2mix c3" PMCCFG=none PHASE=small bash tools/gpu_round.sh || exit $?
  TAG=u4${r}_ CFGS="c1 c2hc c2mix c3" PMCCFG=none CE_AMD_LIB=$D/libce_amd_u4.so PHASE=small bash tools/gpu_round.sh || exit $?
done
