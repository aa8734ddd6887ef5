#!/usr/bin/env bash
# Round 4: realigned fan-in with 1 (product) or 4 (build/ab/libishmem_amd_rb4.so) 1 KiB blocks per
# workgroup: parity of the variant, then tools/misaligned_probe.py at 1 GiB interleaved x3.
set -u
TAG="$1"; OUT=gpurun_out/$TAG; mkdir -p $OUT
ISHMEM_AMD_LIB=$PWD/build/ab/libishmem_amd_rb4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_single.py -m gpu -x -q \
  -k "realigned or misaligned" -p no:cacheprovider > $OUT/pytest_rb4.log 2>&1 || { tail -20 $OUT/pytest_rb4.log; exit 1; }
tail -1 $OUT/pytest_rb4.log
for rep in 1 2 3; do
  for v in base rb4; do
    if [ $v = rb4 ]; then export ISHMEM_AMD_LIB=$PWD/build/ab/libishmem_amd_rb4.so; else unset ISHMEM_AMD_LIB; fi
    MISALIGNED_MIB=1024 timeout -k 10 120 python tools/misaligned_probe.py > $OUT/probe_${v}_r$rep.json 2> $OUT/probe_${v}_r$rep.err || exit $?
    python -c "import json; d=json.load(open('$OUT/probe_${v}_r$rep.json')); print('$v r$rep', ' '.join('%s=%.4f' % (k, v['ms']) for k, v in d.items()))" | tee -a $OUT/ab.txt
  done
done
