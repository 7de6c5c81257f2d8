#!/bin/bash
# Round-3 visit p: frames kernels (DMA / direct variants by size): tests + timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x -k "frames" --timeout 300 --timeout-method thread > $OUT/pytest_frames.log 2>&1
rc=$?; echo "frames tests rc=$rc" >> $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/bench_configs.py --only 8 > $OUT/configs8.log 2>&1 || exit $?
echo "configs8 ok" >> $OUT/steps.log
