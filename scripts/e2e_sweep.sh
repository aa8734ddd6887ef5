#!/usr/bin/env bash
# Host-memory pipeline shape sweep (round 3): staging slots x staging size, 1 PE, 1 GiB.
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for size in ${SIZES:-128M 256M}; do
  for slots in ${SLOTS:-2 4 8}; do
    ISHMEM_STAGING_SIZE=$size ISHMEM_STAGING_SLOTS=$slots timeout -k 10 120 python tools/e2e_sweep.py >> $OUT/e2e_sweep.jsonl 2>> $OUT/e2e_sweep.err || exit $?
  done
done
