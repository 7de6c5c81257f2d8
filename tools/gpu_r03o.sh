#!/bin/bash
# Round-3 visit o: frames kernel, LDS-DMA tiles vs direct loads for grouped members
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "frames" --timeout 240 --timeout-method thread > $OUT/pytest_frames.log 2>&1
rc=$?; echo "frames tests rc=$rc" >> $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
CE_AMD_FRAMES_DMA=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "frames" --timeout 240 --timeout-method thread > $OUT/pytest_frames_direct.log 2>&1
rc=$?; echo "frames direct tests rc=$rc" >> $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  CE_AMD_FRAMES_DMA=$v timeout -k 10 300 python3 tools/bench_configs.py --only 8 > $OUT/configs8_d$v.log 2>&1 || exit $?
  echo "configs8 dma=$v ok" >> $OUT/steps.log
done
