#!/bin/bash
# Generic GPU visit: pytest (-k $K if given), then bench_configs --only $ONLY
# (CE_AMD_SMALL=0 and =1 for A/B), each under its own limit; stops at the
# first failure other than test failures.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
: > $OUT/step.log
st() { echo "$2: $1" >> $OUT/step.log; case $1 in 0|1) ;; *) exit $1 ;; esac; }
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "$K" > $OUT/pytest_k.log 2>&1
  st $? pytest
fi
if [ -n "$ONLY" ]; then
  for ab in ${AB:-1}; do
    CE_AMD_SMALL=$ab timeout -k 10 300 python tools/bench_configs.py --only $ONLY > $OUT/configs_$ab.json 2> $OUT/configs_$ab.err
    st $? "configs small=$ab"
  done
fi
echo done >> $OUT/step.log
