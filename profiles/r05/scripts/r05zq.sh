#!/usr/bin/env bash
# Round 5: phased reduce-scatter with sources 4 B off dest's phase — rs_phase_realign_kernel (DPP +
# LDS realign, default) against rs_phase_kernel with unaligned 16-B source loads
# (set_param phase_unaligned=1), 2 / 4 PEs with one-PE-per-GPU launch shapes, 64 MiB and 1 GiB,
# interleaved x2; --phases prints the grids' times for the 1 GiB call.
set -u
OUT=gpurun_out/r05zq; mkdir -p $OUT
for rep in 1 2; do
  for np_ in 2 4; do
    for un in 0 1; do
      ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ \
        --master-addr 127.0.0.1 --master-port 29707 tools/sweep.py --min-bytes 67108864 --max-mib 1024 --factor 16 --iters 10 \
        --src-offset 4 --phases --emulate-share1 --param phase_unaligned=$un > $OUT/p${np_}_un${un}_r$rep.csv 2> $OUT/p${np_}_un${un}_r$rep.err || exit $?
      echo "p$np_ unaligned$un r$rep: $(grep -v 'Gloo\|peer ranks\|^# coll\|bytes' $OUT/p${np_}_un${un}_r$rep.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
    done
  done
done
