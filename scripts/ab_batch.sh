#!/usr/bin/env bash
# Phased reduce-scatter at a run-time team size (3 PEs on the one GPU, 1 GiB each): member loads
# batched by 4 (product) vs one member at a time (build/ab/libishmem_amd_batch1.so), interleaved.
set -u
TAG="$1"; OUT=gpurun_out/$TAG; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 ISHMEM_BENCH_SAME_DEVICE=1
LEGS="--no-cpu-baseline --no-sweep --no-probe --no-tuning --no-tripwire --no-e2e --no-rccl --no-full-check"
for rep in 1 2; do
  for v in product batch1; do
    if [ $v = product ]; then unset ISHMEM_AMD_LIB; else export ISHMEM_AMD_LIB=build/ab/libishmem_amd_batch1.so; fi
    timeout -k 10 240 python bench.py --gpus 3 --steps 20 --warmup 5 $LEGS > $OUT/bench_${v}_p3_r$rep.json 2> $OUT/bench_${v}_p3_r$rep.err || exit $?
    echo "$v p3 r$rep $(python -c "import json; d=json.load(open('$OUT/bench_${v}_p3_r$rep.json')); print(d.get('ms_per_step'), (d.get('phases') or {}).get('ms'), d.get('error'))")"
  done
done
