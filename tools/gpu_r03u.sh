#!/bin/bash
# Round-3 visit u: GPU suite on the default build; the mix with its hc rows
# prefetched (A/B library) -- its tests, then alternating small-pool traces
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
D=$ROOT/tools/_diag
bash tools/gpu_tests_then.sh || exit $?
CE_AMD_LIB=$D/libce_amd_mx.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_selector.py -q -x --timeout 240 --timeout-method thread -k "mix or golden or session" > $OUT/pytest_mx.log 2>&1
rc=$?; echo "mx tests rc=$rc" >> $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  TAG=def${r}_ CFGS="c1 c2hc c2mix c3 c3r" PMCCFG=none PHASE=small bash tools/gpu_round.sh || exit $?
  TAG=mx${r}_ CFGS="c2mix" PMCCFG=none CE_AMD_LIB=$D/libce_amd_mx.so PHASE=small bash tools/gpu_round.sh || exit $?
done
