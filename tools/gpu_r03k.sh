#!/bin/bash
# Round-3 visit k: the driver's bench command (with the CPU baseline), the
# secondary configs under rocprofv3 (incl. the fused frames -> selection vs
# the two-step path), first-call latency of the in-tree library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit $?
echo "bench default ok" >> $OUT/steps.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof/configs -o run --output-format csv -- python3 $ROOT/tools/bench_configs.py --only 0,1,2,5,8 > $OUT/configs.log 2>&1 || exit $?
echo "configs ok" >> $OUT/steps.log
cd $ROOT
timeout -k 10 300 python3 tools/first_call.py > $OUT/first_call.json 2> $OUT/first_call.err || exit $?
echo "first call ok" >> $OUT/steps.log
