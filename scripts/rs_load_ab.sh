#!/usr/bin/env bash
# Round 4: the phased reduce-scatter's own-chunk loads as buffer loads (product) or global nt loads
# (build/ab/libishmem_amd_rsg.so, -DISHMEMI_RS_OWN_GLOBAL), interleaved, 2 and 4 PEs x 1 GiB as
# processes on the one GPU (kernel efficiency where HBM bounds; the node is xGMI-bound).
set -u
TAG="$1"; OUT=gpurun_out/$TAG; mkdir -p $OUT
export ISHMEM_BENCH_SAME_DEVICE=1
LEGS="--no-cpu-baseline --no-sweep --no-probe --no-tuning --no-tripwire --no-e2e --no-rccl --no-full-check"
for rep in 1 2 3; do
  for np_ in 2 4; do
    for v in base rsg; do
      if [ $v = rsg ]; then export ISHMEM_AMD_LIB=$PWD/build/ab/libishmem_amd_rsg.so; else unset ISHMEM_AMD_LIB; fi
      timeout -k 10 240 python bench.py --gpus $np_ --steps 20 --warmup 5 $LEGS > $OUT/b_${v}_p${np_}_r$rep.json 2> $OUT/b_${v}_p${np_}_r$rep.err || exit $?
      python -c "import json; d=json.load(open('$OUT/b_${v}_p${np_}_r$rep.json')); ph=d['phases']['ms']; print('$v p$np_ r$rep step_ms %.4f rs_ms %.4f ag_ms %.4f' % (d['ms_per_step'], ph['reduce_scatter'], ph['all_gather']))" | tee -a $OUT/ab.txt
    done
  done
done
