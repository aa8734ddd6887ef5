#!/usr/bin/env bash
# rocprofv3 of the same-device multi-PE rehearsal (kernel trace + stats; optional PMC passes).
# Usage: scripts/prof_multi.sh TAG NPES MIB [pmc]
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; NP="$2"; MIB="$3"; PMC="${4:-}"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 ISHMEM_BENCH_SAME_DEVICE=1
cd /tmp && export TMPDIR=/tmp
ARGS="--gpus $NP --steps 10 --warmup 3 --mib $MIB --no-sweep --no-tuning --no-cpu-baseline --no-e2e --no-tripwire --no-probe --no-full-check"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" $ARGS > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; tail -3 "$OUT/trace.log"
case $rc in 0) ;; *) exit $rc;; esac
if [ -n "$PMC" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c -d "$OUT/pmc_$c" -o run --output-format csv -- \
        python3 "$R/bench.py" $ARGS > "$OUT/pmc_$c.log" 2>&1
    rc=$?; echo "pmc $c rc=$rc"; tail -3 "$OUT/pmc_$c.log"
    case $rc in 0) ;; *) exit $rc;; esac
  done
fi
