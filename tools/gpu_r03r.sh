#!/bin/bash
# Round-3 visit r: per-wave floor (CE_SMALL_FLOOR_WAVE) A/B on the small pools
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
D=$ROOT/tools/_diag
CE_AMD_LIB=$D/libce_amd_fw.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_selector.py -q -x --timeout 240 --timeout-method thread -k "batched or golden or small or mix or tie or fuzz or session" > $OUT/pytest_fw.log 2>&1
rc=$?; echo "fw tests rc=$rc" >> $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  TAG=def${r}_ CFGS="c1 c2hc c2mix c3 c3r" PMCCFG=none PHASE=small bash tools/gpu_round.sh || exit $?
  TAG=fw${r}_ CFGS="c1 c2hc c2mix c3 c3r" PMCCFG=none CE_AMD_LIB=$D/libce_amd_fw.so PHASE=small bash tools/gpu_round.sh || exit $?
done
