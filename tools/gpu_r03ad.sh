#!/bin/bash
# Round-3 visit ad: C5 register ring depth 2 (default) vs 3 (A/B library), grid-cyclic items, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
D=$PWD/tools/_diag
CE_AMD_LIB=$D/libce_amd_nb3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "wide_stream_vs or chunked_pool" --timeout 240 --timeout-method thread > $OUT/pytest_nb3.log 2>&1
rc=$?; echo "nb3 tests rc=$rc" >> $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  timeout -k 10 300 python tools/bench_c5.py --items 12000000 --chunk 2000000 > $OUT/c5_nb2_$r.json 2> $OUT/c5_nb2_$r.err || exit $?
  CE_AMD_LIB=$D/libce_amd_nb3.so timeout -k 10 300 python tools/bench_c5.py --items 12000000 --chunk 2000000 > $OUT/c5_nb3_$r.json 2> $OUT/c5_nb3_$r.err || exit $?
  echo "round $r ok" >> $OUT/steps.log
done
