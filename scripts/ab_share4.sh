#!/usr/bin/env bash
# Phased vs persistent at 4 PEs sharing the one GPU (the kPhasedMaxShare boundary), interleaved.
set -u
TAG="$1"; OUT=gpurun_out/$TAG; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 ISHMEM_BENCH_SAME_DEVICE=1
LEGS="--no-cpu-baseline --no-sweep --no-probe --no-tuning --no-tripwire --no-e2e --no-rccl --no-full-check"
for rep in 1 2; do
  for v in phased persistent; do
    if [ $v = phased ]; then export ISHMEM_PHASED_MIN_BYTES=0; else export ISHMEM_PHASED_MIN_BYTES=-1; fi
    timeout -k 10 240 python bench.py --gpus 4 --steps 20 --warmup 5 $LEGS > $OUT/bench_${v}_p4_r$rep.json 2> $OUT/bench_${v}_p4_r$rep.err || exit $?
    echo "$v p4 r$rep $(python -c "import json; d=json.load(open('$OUT/bench_${v}_p4_r$rep.json')); print(d.get('ms_per_step'), d.get('kernel_ms'), d.get('error'))")"
  done
done
