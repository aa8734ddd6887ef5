#!/usr/bin/env bash
# Same-device 2-rank bench legs in isolation: where do small config-5 calls lose time? (dev tool)
set -u
OUT=gpurun_out/${1:-cfg5ab}; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 ISHMEM_BENCH_SAME_DEVICE=1
COMMON="--gpus 2 --steps 5 --warmup 2 --mib 64 --sweep-max-mib 16 --no-tuning --no-probe --no-e2e --no-rccl"
timeout -k 10 200 python bench.py $COMMON --no-tripwire --no-cpu-baseline > $OUT/a_plain.log 2>&1 || exit $?
timeout -k 10 200 python bench.py $COMMON --no-cpu-baseline > $OUT/b_tripwire.log 2>&1 || exit $?
timeout -k 10 200 python bench.py $COMMON --no-tripwire > $OUT/c_cpu.log 2>&1 || exit $?
