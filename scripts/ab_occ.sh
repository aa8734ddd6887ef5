#!/usr/bin/env bash
# A/B of the multi-PE kernel's occupancy: the product build (3 workgroups of
# 256 per CU, 8 loads per lane staged) against build/ab/libishmem_amd_occ4.so (4 per CU, 4 loads),
# 1 GiB per PE, PEs sharing the box's one GPU; interleaved A B A B; bench kernel_ms + phase trace.
set -u
TAG="$1"
OUT=gpurun_out/$TAG
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 ISHMEM_BENCH_SAME_DEVICE=1
LEGS="--no-cpu-baseline --no-sweep --no-probe --no-tuning --no-tripwire --no-e2e --no-rccl --no-full-check"
for rep in 1 2; do
  for v in base occ4; do
    if [ $v = occ4 ]; then export ISHMEM_AMD_LIB=build/ab/libishmem_amd_occ4.so; else unset ISHMEM_AMD_LIB; fi
    for np_ in 2 8; do
      timeout -k 10 240 python bench.py --gpus $np_ --steps 20 --warmup 5 $LEGS > $OUT/bench_${v}_p${np_}_r$rep.json 2> $OUT/bench_${v}_p${np_}_r$rep.err || exit $?
      echo "$v p$np_ r$rep $(python -c "import json,sys; d=json.load(open('$OUT/bench_${v}_p${np_}_r$rep.json')); print(d.get('ms_per_step'), d.get('kernel_ms'), d.get('error'))")"
    done
    timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29811 tools/phase_trace.py --sizes 1073741824,1073741824 > $OUT/trace_${v}_r$rep.log 2>&1 || exit $?
  done
done
