#!/usr/bin/env bash
# Round 4: fan-in kernel source loads as global nontemporal loads (product) or as buffer loads
# based at the workgroup's first item (build/ab/libishmem_amd_fbl.so, -DISHMEMI_FANIN_BUFFER_LOADS),
# interleaved A B A B A B on the N=1 bench (copy = the 1-PE reduce, and the a + b combine leg).
set -u
TAG="$1"; OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in 1 2 3; do
  for v in base fbl; do
    if [ $v = fbl ]; then export ISHMEM_AMD_LIB=$PWD/build/ab/libishmem_amd_fbl.so; else unset ISHMEM_AMD_LIB; fi
    timeout -k 10 180 python bench.py --steps 30 --warmup 5 --no-e2e --no-cpu-baseline > $OUT/bench_${v}_r$rep.json 2> $OUT/bench_${v}_r$rep.err || exit $?
    python -c "import json; d=json.load(open('$OUT/bench_${v}_r$rep.json')); print('$v r$rep copy_ms %.4f combine_ms %.4f value %.1f' % (d['kernel_ms'], d['combine']['ms'], d['value']))" | tee -a $OUT/ab.txt
  done
done
