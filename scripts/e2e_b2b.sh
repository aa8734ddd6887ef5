#!/usr/bin/env bash
# Back-to-back on-stream host-memory reduces (pinned) vs synced ones, under staging shapes:
# slots 2 / 4 / 8 of a 128 MiB region and 4 slots of 256 MiB (tools/e2e_trace.py phases).
set -u
TAG="$1"; OUT=gpurun_out/$TAG; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2; do
  for v in s4 s2 s8 big4; do
    case $v in
      s4) export ISHMEM_STAGING_SLOTS=4 ISHMEM_STAGING_SIZE=128M ;;
      s2) export ISHMEM_STAGING_SLOTS=2 ISHMEM_STAGING_SIZE=128M ;;
      s8) export ISHMEM_STAGING_SLOTS=8 ISHMEM_STAGING_SIZE=128M ;;
      big4) export ISHMEM_STAGING_SLOTS=4 ISHMEM_STAGING_SIZE=256M ;;
    esac
    timeout -k 10 120 python -u tools/e2e_trace.py > $OUT/b2b_${v}_r$rep.txt 2>&1 || exit $?
    echo "== $v rep$rep: $(grep -h '{' $OUT/b2b_${v}_r$rep.txt | tr '\n' ' ')"
  done
done
