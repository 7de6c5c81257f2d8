#!/bin/bash
# Round-3 visit d: GPU tests; small-pool traces (mix UNR fix); interleaved
# tiles A/B on both layouts; the whole GPU suite on the debug build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
bash tools/gpu_tests_then.sh || exit $?
b() {
  local n=$1; shift
  timeout -k 10 300 env "$@" > $OUT/bench_$n.json 2> $OUT/bench_$n.err || exit $?
  echo "bench $n ok" >> $OUT/steps.log
}
b nmc python bench.py --no-cpu-baseline
b nmc_il CE_AMD_ILEAVE=1 python bench.py --no-cpu-baseline
b mnc python bench.py --no-cpu-baseline --layout MNC
b mnc_il CE_AMD_ILEAVE=1 python bench.py --no-cpu-baseline --layout MNC
CFGS="c1 c2hc c2mix c3 c3r" PMCCFG=none PHASE=small bash tools/gpu_round.sh || exit $?
TAG=fd_ CFGS="c1 c3" PMCCFG=none CE_AMD_LIB=$PWD/tools/_diag/libce_amd_fastdiv.so PHASE=small bash tools/gpu_round.sh
PHASE=debug bash tools/gpu_round.sh
