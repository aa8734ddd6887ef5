#!/usr/bin/env bash
# 1 GiB per PE, p = 2 and 8 on the one GPU, three trees (round 1, round-2 first version, this
# tree) back to back on the same box (dev tool; the abtest_* worktrees are not in the repository).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$R/gpurun_out/${1:-abbig}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 ISHMEM_BENCH_SAME_DEVICE=1
for np_ in 2 8; do
  for tree in ${TREES:-abtest_r1 abtest_r2a .}; do
    name=$(basename $( [ "$tree" = "." ] && echo r2 || echo $tree ))_p$np_
    mb=$( [ $np_ = 8 ] && echo 96 || echo 1024 )
    (cd "$R/$tree" && ISHMEM_MAX_BLOCKS=$mb timeout -k 10 200 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node $np_ --master-addr 127.0.0.1 --master-port 29721 tools/sweep.py --max-mib ${MIB:-1024} \
        --min-bytes $(( ${MIB:-1024} * 1048576 )) --iters 20 > "$OUT/$name.log" 2>&1) || exit $?
  done
done
