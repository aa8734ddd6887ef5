#!/usr/bin/env bash
# rocprofv3 kernel trace of the device-initiated work-group reduce (tests/cpp/reduce_bw.cpp,
# modes device_grp1 / device_subgroup / on_queue / host) with 2 PEs as processes on the one GPU.
# Usage: scripts/prof_device_api.sh TAG [max_nelems]
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-devapi}"; M="${2:-1048576}"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 ISHMEM_NPES=2 ISHMEM_DEVICE=0 ISHMEM_BOOTSTRAP_KEY="devapi$$"
export ISHMEM_MAX_BLOCKS=32 ISHMEM_TIMEOUT_MS=20000 ISHMEM_SYMMETRIC_SIZE=512M
cd /tmp && export TMPDIR=/tmp
pids=()
for pe in 0 1; do
  ISHMEM_PE=$pe timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/pe$pe" -o run --output-format csv -- \
      "$R/build/reduce_bw" --csv -m "$M" > "$OUT/pe$pe.log" 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
echo "rc=$rc"; grep -E "csv,reduce_bw|PASS|FAIL" "$OUT/pe0.log" | tail -60
exit $rc
