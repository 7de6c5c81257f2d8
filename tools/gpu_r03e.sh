#!/bin/bash
# Round-3 visit e (fresh container): GPU tests, smoke, the driver's bench line,
# layout / interleave A/B lines, small-pool traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
bash tools/gpu_tests_then.sh || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
echo "smoke ok" >> $OUT/steps.log
b() {
  local n=$1; shift
  timeout -k 10 300 env "$@" > $OUT/bench_$n.json 2> $OUT/bench_$n.err || exit $?
  echo "bench $n ok" >> $OUT/steps.log
}
b default python bench.py
b nmc_il CE_AMD_ILEAVE=1 python bench.py --no-cpu-baseline
b mnc python bench.py --no-cpu-baseline --layout MNC
b mnc_il CE_AMD_ILEAVE=1 python bench.py --no-cpu-baseline --layout MNC
CFGS="c1 c2hc c2mix c3 c3r" PMCCFG=none PHASE=small bash tools/gpu_round.sh || exit $?
