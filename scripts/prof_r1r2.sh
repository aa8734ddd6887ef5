#!/usr/bin/env bash
# Kernel traces of the round-1 tree (abtest_r1) and this tree at one size, 2 PEs same device.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$R/gpurun_out/${1:-profr1r2}"; MIN="${2:-4194304}"; MAXMIB="${3:-4}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 ISHMEM_BENCH_SAME_DEVICE=1
cd /tmp && export TMPDIR=/tmp
for tree in abtest_r1 .; do
  name=$( [ "$tree" = "." ] && echo r2 || echo r1 )
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run --output-format csv -- \
      python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29711 \
      "$R/$tree/tools/sweep.py" --max-mib $MAXMIB --min-bytes $MIN --iters 50 > "$OUT/$name.log" 2>&1 || exit $?
done
