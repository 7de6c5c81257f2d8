#!/bin/bash
# Round-3 visit j: the LDS-DMA wide stream (k_stream_wide_dma): its parity
# tests first, the GPU suite, then the C5 job A/B (register ring vs LDS-DMA).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "wide or chunk" --timeout 240 --timeout-method thread > $OUT/pytest_wide.log 2>&1
rc=$?; echo "wide tests rc=$rc" >> $OUT/steps.log; [ $rc -le 1 ] || exit $rc
bash tools/gpu_tests_then.sh || exit $?
for r in 1 2; do
  for v in 1 0; do
    CE_AMD_WIDE_DMA=$v timeout -k 10 300 python tools/bench_c5.py --items 12000000 --chunk 2000000 > $OUT/c5_dma${v}_$r.json 2> $OUT/c5_dma${v}_$r.err || exit $?
    echo "c5 dma=$v run $r ok" >> $OUT/steps.log
  done
done
