#!/bin/bash
# Round-3 visit ac: C5 with grid-cyclic items, register ring vs LDS-DMA tiles, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "wide_dma" --timeout 280 --timeout-method thread > $OUT/pytest_wdma.log 2>&1
rc=$?; echo "wide dma tests rc=$rc" >> $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    CE_AMD_WIDE_DMA=$v timeout -k 10 300 python tools/bench_c5.py --items 12000000 --chunk 2000000 > $OUT/c5_dma${v}_$r.json 2> $OUT/c5_dma${v}_$r.err || exit $?
  done
  echo "round $r ok" >> $OUT/steps.log
done
