#!/usr/bin/env bash
# Round 6: the phased reduce-scatter with sources 4 B off dest's phase (unaligned 16-B loads), block
# order vs XCD-grouped block order (set_param rs_xcd 0 / 1), 2 / 4 PEs with one-PE-per-GPU launch
# shapes (the whole-array fold off: xgmi_fold_max_bytes 0), 1 GiB, interleaved x2, aligned sources
# as the reference; --phases prints the grids' times.  Then the shifted-source parity tests.
set -u
OUT=gpurun_out/r06c; mkdir -p $OUT
for rep in 1 2; do
  for np_ in 2 4; do
    for cfg in "4 0" "4 1" "0 1"; do
      set -- $cfg; off=$1; x=$2
      ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ \
        --master-addr 127.0.0.1 --master-port 29707 tools/sweep.py --min-bytes 1073741824 --max-mib 1024 --iters 10 \
        --src-offset $off --phases --emulate-share1 --param rs_xcd=$x --param xgmi_fold_max_bytes=0 \
        > $OUT/p${np_}_off${off}_x${x}_r$rep.csv 2> $OUT/p${np_}_off${off}_x${x}_r$rep.err || exit $?
      echo "p$np_ src+$off rs_xcd=$x r$rep: $(grep -v 'Gloo\|peer ranks\|^# coll\|bytes' $OUT/p${np_}_off${off}_x${x}_r$rep.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
    done
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  -k "realigned or offsets or phased_reduce_scatter or whole_array or shifted or emulated" > $OUT/pytest_sel.txt 2>&1
echo "pytest rc=$?" | tee -a $OUT/ab.txt
tail -3 $OUT/pytest_sel.txt
