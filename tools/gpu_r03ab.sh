#!/bin/bash
# Round-3 final visit: GPU suite, smoke, rocprofv3 of the driver's exact bench
# command + FETCH/WRITE passes, the full 50M-item C5 job, small-pool traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
bash tools/gpu_tests_then.sh || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
echo "smoke ok" >> $OUT/steps.log
PHASE=benchprof bash tools/gpu_round.sh || exit $?
timeout -k 10 300 python tools/bench_c5.py > $OUT/c5_full.json 2> $OUT/c5_full.err || exit $?
echo "c5 full ok" >> $OUT/steps.log
TAG=fin_ CFGS="c1 c2hc c2mix c3 c3r" PMCCFG=none PHASE=small bash tools/gpu_round.sh || exit $?
