#!/usr/bin/env bash
# Phased reduce-scatter / all-gather (ISHMEM_PHASED_MIN_BYTES) against the persistent kernel:
#   1. a parity subset of the multi-PE GPU tests with the phased path forced for every heap reduce
#      above the LL threshold (and the 2-PE one-shot fold off, so 2-PE calls take it too);
#   2. interleaved bench rounds at 2 and 8 PEs (1 GiB per PE, PEs sharing the box's one GPU);
#   3. a 2-PE and an 8-PE size sweep per variant (crossover).
# Usage: scripts/ab_phased.sh TAG [steps]   steps: tests bench sweep (default: all three)
set -u
TAG="$1"; shift
STEPS="${*:-tests bench sweep}"
OUT=gpurun_out/$TAG
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
LEGS="--no-cpu-baseline --no-sweep --no-probe --no-tuning --no-tripwire --no-e2e --no-rccl --no-full-check"
for s in $STEPS; do
  case $s in
  tests)
    ISHMEM_PHASED_MIN_BYTES=0 ISHMEM_ONESHOT_P2_MAX_BYTES=0 timeout -k 10 900 python -u -m pytest tests/test_gpu_multi.py \
      -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
      -k "phased or golden or inplace or two_pe or eight_pes_compile or config3 or config4 or huge or large_f32 or graph or tripwire or concurrent or teams or stream_staged" \
      > $OUT/pytest_phased.log 2>&1 || { tail -30 $OUT/pytest_phased.log; exit 1; }
    tail -3 $OUT/pytest_phased.log ;;
  bench)
    export ISHMEM_BENCH_SAME_DEVICE=1
    for rep in 1 2; do
      for v in base phased; do
        if [ $v = phased ]; then export ISHMEM_PHASED_MIN_BYTES=0; else export ISHMEM_PHASED_MIN_BYTES=-1; fi
        for np_ in 2 8; do
          timeout -k 10 240 python bench.py --gpus $np_ --steps 20 --warmup 5 $LEGS > $OUT/bench_${v}_p${np_}_r$rep.json 2> $OUT/bench_${v}_p${np_}_r$rep.err || exit $?
          echo "$v p$np_ r$rep $(python -c "import json,sys; d=json.load(open('$OUT/bench_${v}_p${np_}_r$rep.json')); print(d.get('ms_per_step'), d.get('kernel_ms'), d.get('checked'), d.get('error'))")"
        done
      done
    done
    unset ISHMEM_PHASED_MIN_BYTES ISHMEM_BENCH_SAME_DEVICE ;;
  colltests)
    ISHMEM_PHASED_MIN_BYTES=0 timeout -k 10 900 python -u -m pytest tests/test_gpu_multi.py tests/test_examples.py tests/test_gpu_cpp.py \
      -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
      -k "collect or bcast or teams or team or example or patterns or device" \
      > $OUT/pytest_phased_coll.log 2>&1 || { tail -30 $OUT/pytest_phased_coll.log; exit 1; }
    tail -3 $OUT/pytest_phased_coll.log ;;
  collsweep)
    export ISHMEM_BENCH_SAME_DEVICE=1
    for np_ in 2 8; do
      for v in base phased; do
        if [ $v = phased ]; then export ISHMEM_PHASED_MIN_BYTES=0; else export ISHMEM_PHASED_MIN_BYTES=-1; fi
        timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ --master-addr 127.0.0.1 \
          --master-port 2962$np_ tools/sweep.py --coll fcollect --max-mib $((512 / np_)) --min-bytes 1048576 --factor 4 --iters 20 \
          > $OUT/coll_${v}_p$np_.csv 2> $OUT/coll_${v}_p$np_.err || exit $?
        echo "== fcollect $v p$np_"; grep -v Gloo $OUT/coll_${v}_p$np_.csv
      done
    done
    unset ISHMEM_PHASED_MIN_BYTES ISHMEM_BENCH_SAME_DEVICE ;;
  scansweep)
    export ISHMEM_BENCH_SAME_DEVICE=1
    for np_ in 2 8; do
      for v in base phased; do
        if [ $v = phased ]; then export ISHMEM_PHASED_MIN_BYTES=0; else export ISHMEM_PHASED_MIN_BYTES=-1; fi
        timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ --master-addr 127.0.0.1 \
          --master-port 2963$np_ tools/sweep.py --coll inscan --max-mib 256 --min-bytes 1048576 --factor 4 --iters 20 \
          > $OUT/scan_${v}_p$np_.csv 2> $OUT/scan_${v}_p$np_.err || exit $?
        echo "== inscan $v p$np_"; grep -v Gloo $OUT/scan_${v}_p$np_.csv
      done
    done
    unset ISHMEM_PHASED_MIN_BYTES ISHMEM_BENCH_SAME_DEVICE ;;
  sweep)
    export ISHMEM_BENCH_SAME_DEVICE=1
    for np_ in 2 8; do
      for v in base phased; do
        if [ $v = phased ]; then export ISHMEM_PHASED_MIN_BYTES=0; else export ISHMEM_PHASED_MIN_BYTES=-1; fi
        timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ --master-addr 127.0.0.1 \
          --master-port 2961$np_ tools/sweep.py --max-mib 1024 --min-bytes 1048576 --factor 2 --iters 20 \
          > $OUT/sweep_${v}_p$np_.csv 2> $OUT/sweep_${v}_p$np_.err || exit $?
        echo "== sweep $v p$np_"; cat $OUT/sweep_${v}_p$np_.csv
      done
    done
    unset ISHMEM_PHASED_MIN_BYTES ISHMEM_BENCH_SAME_DEVICE ;;
  esac
done
