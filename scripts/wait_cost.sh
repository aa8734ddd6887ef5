#!/usr/bin/env bash
# Latency cost of the round-4 waiting footprint (kernels.h): 64 KiB .. 16 MiB f32 sum at 2 and 4
# PEs on the one GPU with one-PE-per-GPU launch shapes (--emulate-share1), wait_slots 16 (default:
# each waiting launch <= 1/16 of the device) against 1 (round 3: the whole device), interleaved
# A B A B.  HBM-bound on one GPU, so an upper bound on what a smaller grid costs; over xGMI the
# links bound both.
set -u
TAG="$1"; OUT=gpurun_out/$TAG; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 ISHMEM_BENCH_SAME_DEVICE=1
for np_ in 2 4; do
  for rep in 1 2; do
    for ws in 16 1; do
      ISHMEM_WAIT_SLOTS=$ws timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ \
        --master-addr 127.0.0.1 --master-port 2975$np_ tools/sweep.py --emulate-share1 --max-mib 16 \
        --min-bytes 65536 --factor 2 --iters 50 > $OUT/wait_ws${ws}_p${np_}_r$rep.csv 2> $OUT/wait_ws${ws}_p${np_}_r$rep.err || exit $?
      echo "== ws=$ws p$np_ rep$rep"; grep -E "^[0-9]" $OUT/wait_ws${ws}_p${np_}_r$rep.csv
    done
  done
done
