#!/usr/bin/env bash
# Round 5: realign variants round 2 (LDS workgroup sizes, DPP + LDS) and the checker's negative control.
set -u
OUT=gpurun_out/r05b; mkdir -p $OUT
for k in 4 12 1; do
  timeout -k 10 120 ./tools/bin/realign_variants 1024 3 10 $k > $OUT/rv_k$k.txt 2>&1 || exit $?
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_single.py -k "checker" > $OUT/pytest.txt 2>&1
rc=$?
tail -3 $OUT/pytest.txt
exit $rc
