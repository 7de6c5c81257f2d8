#!/bin/bash
# Round-3 visit f: GPU tests on the default build (single-block pools: slot
# loads no longer under branches -> the log-table commit waits for the table
# only); small-pool traces per A/B library (throttled slot issue, row-level
# shared-reciprocal division); rowdiv bit-exactness; bench lines per library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
bash tools/gpu_tests_then.sh || exit $?
D=$PWD/tools/_diag
TAG=def_ CFGS="c1 c2hc c2mix c3 c3r" PMCCFG=none PHASE=small bash tools/gpu_round.sh || exit $?
for v in thr1 thr2 rowdiv thr1rd; do
  TAG=${v}_ CFGS="c1 c2hc c2mix c3 c3r" PMCCFG=none CE_AMD_LIB=$D/libce_amd_$v.so PHASE=small bash tools/gpu_round.sh || exit $?
done
CE_AMD_LIB=$D/libce_amd_rowdiv.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_selector.py -q -x --timeout 240 --timeout-method thread > $OUT/pytest_rowdiv.log 2>&1
echo "rowdiv tests rc=$?" >> $OUT/steps.log
b() {
  local n=$1; shift
  timeout -k 10 300 env "$@" > $OUT/bench_$n.json 2> $OUT/bench_$n.err || exit $?
  echo "bench $n ok" >> $OUT/steps.log
}
b nmc python bench.py --no-cpu-baseline
b nmc_rd CE_AMD_LIB=$D/libce_amd_rowdiv.so python bench.py --no-cpu-baseline
b mnc python bench.py --no-cpu-baseline --layout MNC
b mnc_rd CE_AMD_LIB=$D/libce_amd_rowdiv.so python bench.py --no-cpu-baseline --layout MNC
