#!/bin/bash
# Round-3 visit v (final evidence on one box): GPU suite, smoke, the driver's
# bench line, the full 50M-item C5 job, every secondary config under rocprofv3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_tests_then.sh || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
echo "smoke ok" >> $OUT/steps.log
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit $?
echo "bench ok" >> $OUT/steps.log
timeout -k 10 300 python tools/bench_c5.py > $OUT/c5_full.json 2> $OUT/c5_full.err || exit $?
echo "c5 full ok" >> $OUT/steps.log
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof/configs -o run --output-format csv -- python3 $ROOT/tools/bench_configs.py --only 0,1,2,5,6,7,8 > $OUT/configs.log 2>&1 || exit $?
echo "configs ok" >> $OUT/steps.log
