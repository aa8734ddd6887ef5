#!/usr/bin/env bash
# Round 5: realigned phased fcollect / collect — parity on the collect / broadcast / phased tests,
# then fcollect of 64 MiB + {0, 4, 1} bytes per PE at 2 and 4 PEs, realigned (default) vs narrow
# items (set by COLLECT_REALIGN=0 through ISHMEM... A/B via the probe's env), interleaved.
set -u
OUT=gpurun_out/${TAG:-r05z}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_multi.py -k "collect or broadcast or phased_paths or stream_memop" > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for np_ in ${NPS:-2 4}; do
  for rep in 1 2; do
    for v in 1 0; do
      COLLECT_REALIGN=$v ISHMEM_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node $np_ --master-addr 127.0.0.1 --master-port 2968$np_ tools/collect_probe.py \
        > $OUT/p${np_}_realign${v}_r$rep.csv 2> $OUT/p${np_}_realign${v}_r$rep.err || exit $?
      echo "p$np_ realign=$v r$rep: $(grep -v 'bytes\|Gloo\|peer' $OUT/p${np_}_realign${v}_r$rep.csv | tr '\n' ' ')" | tee -a $OUT/ab.txt
    done
  done
done
