#!/usr/bin/env bash
# PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs) of the same-device multi-PE rehearsal.
# Counters are device-wide: with every PE on the one GPU they sum all PEs' traffic.
# Usage: scripts/pmc_multi.sh TAG NPES MIB
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; NP="$2"; MIB="$3"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 ISHMEM_BENCH_SAME_DEVICE=1 ISHMEM_TIMEOUT_MS=5000
cd /tmp && export TMPDIR=/tmp
ARGS="--gpus $NP --steps 3 --warmup 1 --mib $MIB --no-sweep --no-tuning --no-cpu-baseline --no-e2e --no-tripwire --no-probe --no-full-check"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c -d "$OUT/pmc_$c" -o run --output-format csv -- \
      python3 "$R/bench.py" $ARGS > "$OUT/pmc_$c.log" 2>&1
  rc=$?; echo "pmc $c rc=$rc"; tail -2 "$OUT/pmc_$c.log"
  case $rc in 0) ;; *) exit $rc;; esac
done
