#!/usr/bin/env bash
# Round 5: fcollect at 256 KiB - 8 MiB per PE with the granule path off: persistent collect kernel
# below the phased threshold (default) against the barrier-bracketed pull grid at every size
# (ISHMEM_PHASED_MIN_BYTES=0), 2 / 4 PEs with one-PE-per-GPU launch shapes, interleaved x2.
set -u
OUT=gpurun_out/r05zzm; mkdir -p $OUT
for rep in 1 2; do
  for np_ in 2 4; do
    for pm in default 0; do
      if [ $pm = 0 ]; then export ISHMEM_PHASED_MIN_BYTES=0; else unset ISHMEM_PHASED_MIN_BYTES; fi
      ISHMEM_LL_MAX_BYTES=0 ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ \
        --master-addr 127.0.0.1 --master-port 29737 tools/sweep.py --coll fcollect --min-bytes 262144 --max-mib 8 --factor 2 --iters 30 \
        --emulate-share1 > $OUT/p${np_}_pm${pm}_r$rep.csv 2> $OUT/p${np_}_pm${pm}_r$rep.err || exit $?
      echo "p$np_ fcollect phased_min=$pm r$rep: $(grep -v 'Gloo\|peer ranks\|^#\|bytes' $OUT/p${np_}_pm${pm}_r$rep.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
    done
  done
done
