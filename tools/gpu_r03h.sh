#!/bin/bash
# Round-3 visit h: GPU tests + smoke on the new defaults (throttled slots,
# row-level division), phase stamps of C3, small-pool traces, bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
bash tools/gpu_tests_then.sh || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
echo "smoke ok" >> $OUT/steps.log
bash tools/gpu_phase.sh || exit $?
TAG=h_ CFGS="c1 c2hc c2mix c3 c3r" PMCCFG=${PMCCFG:-c3} PHASE=small bash tools/gpu_round.sh || exit $?
b() {
  local n=$1; shift
  timeout -k 10 300 env "$@" > $OUT/bench_$n.json 2> $OUT/bench_$n.err || exit $?
  echo "bench $n ok" >> $OUT/steps.log
}
b nmc python bench.py --no-cpu-baseline
b mnc python bench.py --no-cpu-baseline --layout MNC
