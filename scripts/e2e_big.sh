#!/usr/bin/env bash
# One staged call over 4 GiB of pinned host memory (128 / 64 chunks of 32 / 64 MiB) vs 1 GiB calls.
set -u
TAG="$1"; OUT=gpurun_out/$TAG; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 E2E_BIG=4
for rep in 1 2; do
  for v in s4 s2; do
    case $v in
      s4) export ISHMEM_STAGING_SLOTS=4 ISHMEM_STAGING_SIZE=128M ;;
      s2) export ISHMEM_STAGING_SLOTS=2 ISHMEM_STAGING_SIZE=128M ;;
    esac
    timeout -k 10 150 python -u tools/e2e_trace.py > $OUT/big_${v}_r$rep.txt 2>&1 || exit $?
    echo "== $v rep$rep: $(grep -h '{' $OUT/big_${v}_r$rep.txt | tr '\n' ' ')"
  done
done
