#!/usr/bin/env bash
# Staged pipeline: host-side window (ISHMEM_STAGED_WINDOW chunks ahead, polled; 0 = off) x slot
# size (4 x 32 MiB / 2 x 64 MiB of the 128 MiB staging region): single calls of E2E_BIG GiB, then
# 1 GiB calls warm-up / back to back / synced (tools/e2e_trace.py), interleaved twice.
set -u
TAG="$1"; OUT=gpurun_out/$TAG; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 E2E_BIG=${E2E_BIG:-8} ISHMEM_STAGING_SIZE=128M
for rep in 1 2; do
  for v in s2w0 s4w16 s2w16 s4w0; do
    case $v in
      s4w16) export ISHMEM_STAGING_SLOTS=4 ISHMEM_STAGED_WINDOW=16 ;;
      s2w16) export ISHMEM_STAGING_SLOTS=2 ISHMEM_STAGED_WINDOW=16 ;;
      s4w0) export ISHMEM_STAGING_SLOTS=4 ISHMEM_STAGED_WINDOW=0 ;;
      s2w0) export ISHMEM_STAGING_SLOTS=2 ISHMEM_STAGED_WINDOW=0 ;;
    esac
    timeout -k 10 170 python -u tools/e2e_trace.py > $OUT/win_${v}_r$rep.txt 2>&1 || exit $?
    echo "== $v rep$rep: $(grep -h '{' $OUT/win_${v}_r$rep.txt | tr '\n' ' ')"
  done
done
