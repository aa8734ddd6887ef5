#!/usr/bin/env bash
# Latency cost of the round-4 waiting footprint (kernels.h): 64 KiB .. 16 MiB f32 sum at 2 PEs on
# the one GPU with one-PE-per-GPU launch shapes (--emulate-share1), interleaved A B C A B C:
#   ws16    wait_slots 16 (default: each waiting launch <= 1/16 of the device)
#   ws1     wait_slots 1 (round 3: the whole device per launch)
#   phased  the phased path forced from 0 bytes (never-waiting full-device grids between barriers)
# HBM-bound on one GPU, so an upper bound on what a smaller grid costs; over xGMI the links bound
# both.  (ws1 is not run at 4 PEs: four whole-device waiting grids on one GPU time out — the
# hazard itself, profiles/r04/wait_cost/.)
set -u
TAG="$1"; OUT=gpurun_out/$TAG; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 ISHMEM_BENCH_SAME_DEVICE=1 ISHMEM_TIMEOUT_MS=5000
for rep in 1 2; do
  for v in ws16 ws1 phased; do
    case $v in
      ws16) export ISHMEM_WAIT_SLOTS=16; unset ISHMEM_PHASED_MIN_BYTES ;;
      ws1) export ISHMEM_WAIT_SLOTS=1; unset ISHMEM_PHASED_MIN_BYTES ;;
      phased) export ISHMEM_WAIT_SLOTS=16 ISHMEM_PHASED_MIN_BYTES=0 ;;
    esac
    timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29752 tools/sweep.py --emulate-share1 --max-mib 16 \
      --min-bytes 65536 --factor 2 --iters 50 > $OUT/wait_${v}_p2_r$rep.csv 2> $OUT/wait_${v}_p2_r$rep.err || exit $?
    echo "== $v p2 rep$rep"; grep -E "^[0-9]" $OUT/wait_${v}_p2_r$rep.csv
  done
done
