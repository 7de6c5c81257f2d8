#!/bin/bash
# Round-3 visit l: the fused frames -> selection configs under rocprofv3, first call
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof/configs8 -o run --output-format csv -- python3 $ROOT/tools/bench_configs.py --only 8 > $OUT/configs8.log 2>&1 || exit $?
echo "configs8 ok" >> $OUT/steps.log
cd $ROOT
timeout -k 10 300 python3 tools/first_call.py > $OUT/first_call.json 2> $OUT/first_call.err || exit $?
echo "first call ok" >> $OUT/steps.log
