#!/usr/bin/env bash
# A/B: the round-1 tree (abtest_r1, git worktree of aa1a413, built in place) vs this tree, same
# box, same-device 2-PE sweeps (dev tool; abtest_r1 is not part of the repository).
# Usage: scripts/sweep_r1r2.sh TAG "name:tree:env ..."
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$R/gpurun_out/${1:-r1r2}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 ISHMEM_BENCH_SAME_DEVICE=1
for spec in $2; do
  name=${spec%%:*}; rest=${spec#*:}; tree=${rest%%:*}; envs=${rest#*:}
  (cd "$R/$tree" && env ${envs//,/ } timeout -k 10 200 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node ${NP:-2} --master-addr 127.0.0.1 --master-port 29701 tools/sweep.py --max-mib 1024 \
      > "$OUT/$name.log" 2>&1) || exit $?
done
