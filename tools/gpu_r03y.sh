#!/bin/bash
# Round-3 visit y: GPU suite + smoke + bench lines on the per-layout tile orders
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
bash tools/gpu_tests_then.sh || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
echo "smoke ok" >> $OUT/steps.log
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --layout MNC > $OUT/bench_mnc.json 2> $OUT/bench_mnc.err || exit $?
CE_AMD_ILEAVE=0 timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_il0.json 2> $OUT/bench_il0.err || exit $?
echo "bench ok" >> $OUT/steps.log
