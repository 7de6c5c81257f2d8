#!/bin/bash
# Round-3 validation visit: GPU tests, both bench layouts, small-pool traces +
# PMC (new kernels and the r02 library), first-call latency.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
bash tools/gpu_tests_then.sh || exit $?
CE_AMD_LIB=$PWD/tools/_diag/libce_amd_fastdiv.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -s -k "row_division or golden or large" --timeout 240 --timeout-method thread > $OUT/pytest_fastdiv.log 2>&1
rc=$?; echo "fastdiv tests rc=$rc" >> $OUT/steps.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_nmc.json 2> $OUT/bench_nmc.err || exit $?
echo "bench nmc ok" >> $OUT/steps.log
timeout -k 10 300 python bench.py --no-cpu-baseline --layout MNC > $OUT/bench_mnc.json 2> $OUT/bench_mnc.err || exit $?
echo "bench mnc ok" >> $OUT/steps.log
PHASE=small bash tools/gpu_round.sh || exit $?
TAG=r02_ CE_AMD_LIB=$PWD/tools/_diag/libce_amd_r02.so PHASE=small bash tools/gpu_round.sh || exit $?
PHASE=firstcall LIBS="tools/_diag/libce_amd_r02.so consensus-entropy_amd/ce_amd/libce_amd.so" bash tools/gpu_round.sh
