#!/usr/bin/env bash
# A/B of library variants on the multi-PE kernel (1 GiB per PE, PEs sharing the box's one GPU):
# interleaved rounds of bench kernel_ms at 2 and 8 PEs plus a 2-PE phase trace per variant.
# Usage: scripts/ab_occ.sh TAG [name=libpath ...]   ("product" = ishmem_amd/libishmem_amd.so)
# Round 3: product (4 workgroups per CU) vs occ3=build/ab/libishmem_amd_occ3.so (round 2's 3).
set -u
TAG="$1"; shift
VARIANTS="${*:-product=product occ3=build/ab/libishmem_amd_occ3.so}"
OUT=gpurun_out/$TAG
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 ISHMEM_BENCH_SAME_DEVICE=1
LEGS="--no-cpu-baseline --no-sweep --no-probe --no-tuning --no-tripwire --no-e2e --no-rccl --no-full-check"
for rep in 1 2; do
  for nv in $VARIANTS; do
    v=${nv%%=*}; lib=${nv#*=}
    if [ "$lib" = product ]; then unset ISHMEM_AMD_LIB; else export ISHMEM_AMD_LIB=$lib; fi
    for np_ in 2 8; do
      timeout -k 10 240 python bench.py --gpus $np_ --steps 20 --warmup 5 $LEGS > $OUT/bench_${v}_p${np_}_r$rep.json 2> $OUT/bench_${v}_p${np_}_r$rep.err || exit $?
      echo "$v p$np_ r$rep $(python -c "import json,sys; d=json.load(open('$OUT/bench_${v}_p${np_}_r$rep.json')); print(d.get('ms_per_step'), d.get('kernel_ms'), d.get('error'))")"
    done
    timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29811 tools/phase_trace.py --sizes 1073741824,1073741824 > $OUT/trace_${v}_r$rep.log 2>&1 || exit $?
  done
done
