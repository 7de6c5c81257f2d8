#!/bin/bash
# Round-3 visit ae: single-GPU proxies of one rank at 1/2/4/8 GPUs on the final code
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python tools/scale_proxy.py > $OUT/scale_proxy.json 2> $OUT/scale_proxy.err || exit $?
echo "scale proxy ok" >> $OUT/steps.log
