import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import ishmem_amd as ish
from ishmem_amd import hip
ish.init(0, 1, 0, "blk%d" % os.getpid())
src, dst = ish.ishmem_malloc(1 << 20), ish.ishmem_malloc(1 << 20)
st = hip.stream_create()
def t(name, fn, k=2000):
    for _ in range(50): fn()
    t0 = time.perf_counter()
    for _ in range(k): fn()
    print(f"{name}: {1e6*(time.perf_counter()-t0)/k:.2f} us/call", flush=True)
t("blocking reduce (null stream + sync)", lambda: ish.ishmem_float_sum_reduce(dst, src, 1024))
t("on_stream + stream_synchronize", lambda: (ish.ishmemx_float_sum_reduce_on_stream(dst, src, 1024, 0, st), hip.stream_synchronize(st)))
t("on_stream only (enqueue)", lambda: ish.ishmemx_float_sum_reduce_on_stream(dst, src, 1024, 0, st), k=20000)
hip.stream_synchronize(st)
t("stream_synchronize idle", lambda: hip.stream_synchronize(st))
t("device synchronize idle", lambda: hip.synchronize())
ish.ishmem_finalize()
