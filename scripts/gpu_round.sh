#!/usr/bin/env bash
# GPU-box driver for one measurement round.  Each GPU step has its own time limit; a fault,
# abort, segfault or timeout (exit 124/134/137/139) ends the script at once — no retries.
# Usage: scripts/gpu_round.sh TAG [steps...]   steps: smoke single multi bench prof pmc
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r01}"; shift || true
STEPS="${*:-smoke single multi bench prof}"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R"

fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # name seconds cmd...
  local name="$1" secs="$2"; shift 2
  echo "=== $name ($(date +%T))" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL rc=$rc in $name: stopping" | tee -a "$OUT/steps.log"; exit $rc; fi
  return 0
}

rocminfo 2>/dev/null | grep -m3 -E "gfx950|Marketing" > "$OUT/device.txt" || true
nproc > "$OUT/host.txt"; lscpu | grep -m1 "Model name" >> "$OUT/host.txt" || true

for s in $STEPS; do
  case "$s" in
    smoke)  run smoke 180 python -c "import __graft_entry__ as g; g.smoke()" ;;
    init)   # init time by phase at 2 PEs, heap 1 / 4 / 9 GiB then 1 GiB again (the first run is the
            # box's first HIP process: cold), ISHMEM_DEBUG=2 phase lines on stderr
            run init_timing 400 python tools/init_timing.py --npes ${INIT_NPES:-2} --sizes ${INIT_SIZES:-1G,4G,9G,1G} \
                --splits ${INIT_SPLITS:-0} ;;
    gpu)    run pytest_gpu 1500 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider ;;
    sel)    run pytest_sel ${SEL_SECS:-1500} python -u -m pytest tests -m gpu -x -v --timeout ${SEL_TIMEOUT:-900} \
                --timeout-method thread -p no:cacheprovider -k "$SEL" ;;
    soak)   STRESS_ITERS=${ITERS:-300} STRESS_SEED=${SEED:-9001} STRESS_TIMEOUT=${STRESS_TIMEOUT:-780} run soak ${SOAK_SECS:-900} python -u -m pytest tests/test_gpu_multi.py \
                -m gpu -x -v --timeout 800 --timeout-method thread -p no:cacheprovider -k randomised_protocol_stress -s ;;
    single) run pytest_single 900 python -m pytest tests/test_gpu_single.py -m gpu -x -q -p no:cacheprovider ;;
    multi)  run pytest_multi 1200 python -m pytest tests/test_gpu_multi.py -m gpu -x -q -p no:cacheprovider ;;
    bench)  run bench 600 python bench.py --steps 20 --warmup 5 ;;
    local2|local4|local8)  # N-rank rehearsal on the one GPU (self-launched ranks, same device)
            np_=${s#local}
            ISHMEM_BENCH_SAME_DEVICE=1 run bench_$s 900 python bench.py --gpus $np_ --steps 10 --warmup 3 \
                --mib ${MIB:-1024} --sweep-max-mib ${SWEEP_MIB:-4096} ;;
    elocal2|elocal4|elocal8)  # the same rehearsal with every rank on its own emulated GPU (test-hooks
            # library): the cross-device thresholds and `recommended` keys of one PE per GPU
            np_=${s#elocal}
            ISHMEM_BENCH_SAME_DEVICE=1 ISHMEM_BENCH_EMULATE_SHARE1=1 run bench_$s 900 python bench.py --gpus $np_ \
                --steps 10 --warmup 3 --mib ${MIB:-1024} --sweep-max-mib ${SWEEP_MIB:-256} --no-e2e --no-rccl ;;
    sweep1) run sweep1 300 python tools/sweep.py --max-mib 1024 ;;
    bw2)    # tests/cpp/reduce_bw.cpp at 2 PEs (all modes incl. device_multi_wg 1/2/4/8 groups), CSV
            key=bw$RANDOM$RANDOM
            for pe in 0 1; do
              ISHMEM_PE=$pe ISHMEM_NPES=2 ISHMEM_DEVICE=0 ISHMEM_BOOTSTRAP_KEY=$key ISHMEM_SYMMETRIC_SIZE=1G \
                timeout -k 10 600 build/reduce_bw --csv -m ${BW_MAX:-1048576} > "$OUT/reduce_bw_p2_pe$pe.csv" 2>&1 &
            done
            wait; rc=$?
            echo "=== bw2 rc=$rc" | tee -a "$OUT/steps.log"; tail -3 "$OUT/reduce_bw_p2_pe0.csv"
            if fatal $rc; then exit $rc; fi ;;
    sweep2|sweep4|sweep8) np_=${s#sweep}
            ISHMEM_BENCH_SAME_DEVICE=1 run $s 600 python -m torch.distributed.run \
                --nnodes=1 --nproc-per-node $np_ --master-addr 127.0.0.1 --master-port 2951$np_ tools/sweep.py --max-mib 256 ;;
    llcmp)  for np_ in 2 4; do for ll in 0 65536; do
              ISHMEM_BENCH_SAME_DEVICE=1 ISHMEM_MAX_BLOCKS=${MB:-128} ISHMEM_LL_MAX_BYTES=$ll run llcmp_p${np_}_ll${ll} 300 \
                python -m torch.distributed.run --nnodes=1 --nproc-per-node $np_ --master-addr 127.0.0.1 \
                --master-port 2952$np_ tools/sweep.py --max-mib 1 --min-bytes 2048 --factor 2 --iters 50
            done; done ;;
    coll)   for c in fcollect inscan; do
              ISHMEM_BENCH_SAME_DEVICE=1 ISHMEM_MAX_BLOCKS=${MB:-256} run coll_${c}_p2 300 \
                python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
                --master-port 29541 tools/sweep.py --coll $c --max-mib 256 --min-bytes 4096 --factor 4
            done ;;
    graph)  for g in "" "--graph"; do
              ISHMEM_BENCH_SAME_DEVICE=1 ISHMEM_MAX_BLOCKS=${MB:-128} run graph_p2${g:+_graph} 300 \
                python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
                --master-port 29551 tools/sweep.py --max-mib 16 --min-bytes 256 --factor 4 --iters 50 $g
            done ;;
    prof)   cd /tmp && export TMPDIR=/tmp
            run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
                python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline
            cd "$R" ;;
    pmc)    cd /tmp && export TMPDIR=/tmp
            run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
                python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline
            run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
                python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline
            cd "$R" ;;
  esac
done
echo "done" >> "$OUT/steps.log"
