/* ishmem_amd — C-ABI of the MI355X-native reduction-collective path.
 *
 * This is the drop-in boundary: plain C types, plain pointers and sizes, no torch/HIP types in
 * the signatures (streams are passed as `void *` = hipStream_t).  The C++ API with the
 * reference's exact names (include/ishmem.h, include/ishmemx.h) is a header-only layer of
 * inline wrappers over these entry points, so a maintainer can bind this library from any
 * language that speaks the C ABI (ctypes / cffi / JNI).
 *
 * Every function returns 0 on success and nonzero on failure (reference convention:
 * src/ishmem/err.h, collectives return int 0/!=0, src/collectives/reduce_impl.h:259-317);
 * pointer-returning functions return NULL on failure.  Nothing throws across this ABI.
 * ishmemi_c_last_error() returns a human-readable reason for the last failure of this thread.
 *
 * Citations are reference paths (oneapi-src/ishmem v1.5.1) of the interface each entry replaces.
 */
#ifndef ISHMEM_AMD_CAPI_H
#define ISHMEM_AMD_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Reduction operators — relative order of AND_REDUCE..PROD_REDUCE in src/ishmem/types.h:66-72. */
typedef enum {
    ISHMEMI_OP_AND = 0,
    ISHMEMI_OP_OR = 1,
    ISHMEMI_OP_XOR = 2,
    ISHMEMI_OP_MAX = 3,
    ISHMEMI_OP_MIN = 4,
    ISHMEMI_OP_SUM = 5,
    ISHMEMI_OP_PROD = 6,
    ISHMEMI_OP_COUNT = 7
} ishmemi_c_op_t;

/* Canonical fixed-width element types (the reference canonicalises every C type to these before
 * combining: src/collectives/reduce_impl.h:22-59, src/ishmem/util.h:452-479). */
typedef enum {
    ISHMEMI_DT_INT8 = 0,
    ISHMEMI_DT_INT16 = 1,
    ISHMEMI_DT_INT32 = 2,
    ISHMEMI_DT_INT64 = 3,
    ISHMEMI_DT_UINT8 = 4,
    ISHMEMI_DT_UINT16 = 5,
    ISHMEMI_DT_UINT32 = 6,
    ISHMEMI_DT_UINT64 = 7,
    ISHMEMI_DT_FLOAT = 8,
    ISHMEMI_DT_DOUBLE = 9,
    ISHMEMI_DT_COUNT = 10
} ishmemi_c_dtype_t;

/* Team handles — src/ishmem.h:61-72 (ISHMEM_TEAM_WORLD 0, ISHMEM_TEAM_SHARED 1) and
 * src/ishmemx.h:11 (ISHMEMX_TEAM_NODE 2).  On one MI355X node all three span every PE. */
#define ISHMEMI_C_TEAM_INVALID (-1)
#define ISHMEMI_C_TEAM_WORLD 0
#define ISHMEMI_C_TEAM_SHARED 1
#define ISHMEMI_C_TEAM_NODE 2

/* API version and vendor string reported by ishmem_info_get_version / _name (src/ishmem.h:17-21,
 * src/ishmem.cpp:495-512): the reference API version this library implements. */
#define ISHMEMI_C_SPEC_MAJOR 1
#define ISHMEMI_C_SPEC_MINOR 5
#define ISHMEMI_C_SPEC_PATCH 1
#define ISHMEMI_C_MAX_NAME_LEN 256
#define ISHMEMI_C_VENDOR_STRING "ishmem_amd (AMD Instinct MI355X, HIP)"

/* Thread levels (src/ishmem.h:23-26). */
#define ISHMEMI_C_THREAD_SINGLE 0
#define ISHMEMI_C_THREAD_FUNNELED 1
#define ISHMEMI_C_THREAD_SERIALIZED 2
#define ISHMEMI_C_THREAD_MULTIPLE 3

/* ---- lifecycle — replaces ishmem_init / ishmem_finalize (src/ishmem.h:40-41,
 *      src/ishmem.cpp:224-407) and ishmemx_init_attr (src/ishmemx.h:21-37) ---------------------
 * ishmemi_c_init(): PE identity from the process's launcher, where the reference takes it from
 *   its MPI / PMI runtime (src/runtime/runtime_mpi.cpp:1256-1282), first match wins:
 *   ISHMEM_PE / ISHMEM_NPES / ISHMEM_DEVICE; torchrun's RANK / WORLD_SIZE / LOCAL_RANK; MPICH
 *   hydra and Intel MPI (`mpiexec -n N ./app`, test/cmake/common.cmake:28-43) PMI_RANK /
 *   PMI_SIZE / MPI_LOCALRANKID; Open MPI OMPI_COMM_WORLD_RANK / _SIZE / _LOCAL_RANK; srun
 *   SLURM_PROCID / SLURM_NTASKS / SLURM_LOCALID.  Device = node-local rank.  Bootstrap key from
 *   ISHMEM_BOOTSTRAP_KEY, else from the launcher (torchrun's MASTER_PORT, the MPI launcher's
 *   per-node daemon, the Slurm job step).  A job spread over several nodes is refused.
 * ishmemi_c_init_pe(): the same with explicit values (device < 0: keep the env rule).
 * ishmemi_c_launch_info(): what ishmemi_c_init would use (no GPU touched): pe, npes, device,
 *   the launcher's name ("ishmem", "torchrun", "pmi", "openmpi", "slurm", "none") and the
 *   bootstrap key; nonzero (and ishmemi_c_last_error) when init would refuse it.
 * The bootstrap (handle exchange + host barrier) is a POSIX shared-memory segment on the node;
 * it replaces the reference's MPI/OpenSHMEM/PMI runtime (src/runtime.h:22-84) for the only job
 * it does on this path: exchanging the heap IPC handles (src/ipc.cpp:123-233). */
int ishmemi_c_init(void);
int ishmemi_c_init_pe(int pe, int npes, int device, const char *bootstrap_key);
int ishmemi_c_launch_info(int *pe, int *npes, int *device, char *launcher, size_t launcher_len, char *key,
                          size_t key_len);
int ishmemi_c_finalize(void);
int ishmemi_c_initialized(void);
int ishmemi_c_my_pe(void);  /* ishmem_my_pe, src/ishmem.h:54 */
int ishmemi_c_n_pes(void);  /* ishmem_n_pes, src/ishmem.h:55 */
int ishmemi_c_device(void); /* HIP device ordinal this PE runs on */
/* ishmem_init_thread / ishmem_query_thread (src/ishmem.h:44-45, src/ishmem.cpp:409-419): the
 * runtime's host calls are serialised by one lock, so ISHMEM_THREAD_MULTIPLE is always provided
 * (collectives of one team must still be called in the same order on every member, as in the
 * reference, src/teams.h:29-38).  init_thread initialises like ishmemi_c_init. */
int ishmemi_c_init_thread(int requested, int *provided);
int ishmemi_c_query_thread(int *provided);

/* ---- symmetric heap in HBM — replaces ishmem_malloc/align/calloc/free (src/ishmem.h:48-51,
 *      src/memory.cpp:200-300) and ishmem_ptr (src/ishmem.h:56) -----------------------------
 * One hipMalloc'd heap per PE (size: ISHMEM_SYMMETRIC_SIZE, src/ishmem/env_defs.h:20), mapped
 * into every peer by HIP IPC.  Allocation is collective and deterministic (same offsets on every
 * PE).  ishmemi_c_ptr returns the address of `dest` on PE `pe` in this process (NULL if `dest`
 * is not in the heap). */
void *ishmemi_c_malloc(size_t size);
void *ishmemi_c_align(size_t alignment, size_t size);
void *ishmemi_c_calloc(size_t count, size_t size);
void ishmemi_c_free(void *ptr);
void *ishmemi_c_ptr(const void *dest, int pe);
int ishmemi_c_heap_info(void **base, size_t *size, size_t *used);

/* ---- teams — src/ishmem.h:74-86 ------------------------------------------------------------ */
int ishmemi_c_team_my_pe(int team);
int ishmemi_c_team_n_pes(int team);
int ishmemi_c_team_translate_pe(int src_team, int src_pe, int dest_team);
int ishmemi_c_team_split_strided(int parent_team, int start, int stride, int size, int *new_team);
int ishmemi_c_team_split_2d(int parent_team, int xrange, int *xaxis_team, int *yaxis_team);
void ishmemi_c_team_destroy(int team);
/* Team configuration (ishmem_team_config_t = {int num_contexts}, src/ishmem.h:63-67, :78;
 * src/teams.cpp:545-570).  Contexts do not exist on this path; the value given at split time is
 * stored and reported.  get_config: config_mask 0 or ISHMEM_TEAM_NUM_CONTEXTS (1); returns 0, or
 * nonzero for an invalid team / mask / a NULL out-pointer with a nonzero mask. */
int ishmemi_c_team_get_config(int team, long config_mask, int *num_contexts);
int ishmemi_c_team_set_config(int team, long config_mask, int num_contexts);

/* ---- synchronisation — ishmem_barrier_all / sync_all / team_sync (src/ishmem.h:1555-1559,
 *      device implementation src/collectives/sync_impl.h:30-69) --------------------------------- */
int ishmemi_c_barrier_all(void);
int ishmemi_c_sync_all(void);
int ishmemi_c_team_sync(int team);
/* The team barrier enqueued on `stream` (ishmemx_team_sync_on_queue / sync_all_on_queue /
 * barrier_all_on_queue, src/ishmemx.h:2228-2235); *ret as for ishmemi_c_reduce_on_stream. */
int ishmemi_c_team_sync_on_stream(int team, int *ret, void *stream);
/* Recovery after a device-side timeout (no reference counterpart: the reference aborts the job,
 * src/proxy.cpp:79-84).  Collective over ALL PEs, called with no collective in flight: the PEs
 * agree on the newest epoch of every team over the bootstrap, so later collectives of a team whose
 * members fell out of step work again; pending device error words are cleared. */
int ishmemi_c_resync(void);

/* ---- THE HOT PATH ----------------------------------------------------------------------------
 * ishmemi_c_reduce: blocking reduction over a team.  Replaces every
 *   int ishmem_<TYPENAME>_<op>_reduce([ishmem_team_t team,] TYPE *dest, const TYPE *source,
 *                                     size_t nreduce)
 * (src/ishmem.h:923-1238, instantiated in src/collectives/reduce.cpp:8-417) whose body is
 * ishmemi_reduce<T,OP>(team, dest, source, nreduce) (src/collectives/reduce_impl.h:259-317).
 * `dest`/`source`: symmetric-heap device memory (device path), or any device / host memory
 * (staged through the heap).  `source == dest` (in place) or disjoint, as the reference requires
 * (docs/source/collectives.rst:1025-1028).  Returns when `dest` holds the result on this PE and
 * `source` may be reused (collectives.rst:1046-1050).
 *
 * ishmemi_c_reduce_on_stream: the HIP-stream analogue of
 *   sycl::event ishmemx_<TYPENAME>_<op>_reduce_on_queue(..., int *ret, sycl::queue &q, deps)
 * (src/ishmemx.h:1172-1803, src/collectives/reduce_impl.h:444-474): enqueues the collective on
 * `stream` (hipStream_t) and returns at once.  *ret (device-visible int, may be NULL) is set to 0
 * in stream order at the start of the call and to nonzero by any of the call's launches that
 * fails, so it reads 0 after the call completes only on success (reduce_impl.h:461-463). */
int ishmemi_c_reduce(int team, int op, int dtype, void *dest, const void *source, size_t nreduce);
int ishmemi_c_reduce_on_stream(int team, int op, int dtype, void *dest, const void *source,
                               size_t nreduce, int *ret, void *stream);
/* The same with the reference's event plumbing: the call runs after every hipEvent_t in
 * deps[0..ndeps) (its `const std::vector<sycl::event> &deps`, reduce_impl.h:445-453), and, when
 * `done` (a hipEvent_t) is not NULL, `done` is recorded on `stream` after the call's last launch
 * (the sycl::event the reference returns, reduce_impl.h:471-472). */
int ishmemi_c_reduce_on_stream_deps(int team, int op, int dtype, void *dest, const void *source,
                                    size_t nreduce, int *ret, void *stream, void *const *deps,
                                    size_t ndeps, void *done);

/* Local combine unit of the path (what one reduce step does per element):
 *   dst[i] = op(srcs[0][i], srcs[1][i], ..., srcs[nsrc-1][i]), folded in source order.
 * Replaces vector_reduce / vector_reduce_work_group (src/collectives/reduce_impl.h:105-183).
 * Device pointers; asynchronous on `stream`. nsrc in 1..16. */
int ishmemi_c_combine(int op, int dtype, void *dst, const void *const *srcs, int nsrc, size_t n,
                      void *stream);
/* Measurement hook (bench.py's xGMI probe, no reference counterpart): dst = sum of the nsrc f32
 * arrays as 16-B items, every source load issued with the cache policy the collectives would use
 * on peer memory: policy 0 = nontemporal (L2-cached, nt), 1 = system-coherent (sc0 sc1, what the
 * reduce / collect / scan kernels issue).  nbytes must be a multiple of 16, pointers 16-B
 * aligned; srcs may be peers' heap addresses (ishmemi_c_ptr).  Asynchronous on `stream`. */
int ishmemi_c_pull_probe(void *dst, const void *const *srcs, int nsrc, size_t nbytes, int policy,
                         void *stream);
/* Test hook (no reference counterpart): enqueues on `stream` a kernel of `grid` workgroups that
 * each hold half a CU (1024 work-items, 80 KiB of LDS) for `usec` microseconds (<= 60 s), so a
 * test can run collectives while another kernel holds most CUs. */
int ishmemi_c_occupy(int grid, unsigned long long usec, void *stream);
/* Test hook (no reference counterpart): dst[i] = a[i] + b[i] over n uint32 with ordinary loads and
 * stores, like a user's producer kernel (its results may still be dirty in this device's L2 when
 * the next kernel starts).  Asynchronous on `stream`; 4-B aligned pointers. */
int ishmemi_c_produce_u32(void *dst, const void *a, const void *b, size_t n, void *stream);

/* ---- the collectives next to the reduce, same machinery -------------
 * fcollect: dest[j*nbytes ..] = member j's source, in team order, on every member
 *   (ishmem_<TN>_fcollect / ishmem_fcollectmem, src/ishmem.h:894-921, collect_impl.h).
 * collect: members may contribute different byte counts; concatenated in team order
 *   (ishmem_<TN>_collect / ishmem_collectmem).  Blocking only.
 * scan: prefix sum over the team in team order, inclusive (ishmem_<TN>_sum_inscan) or exclusive
 *   (ishmem_<TN>_sum_exscan; the first member gets 0), src/collectives/scan_impl.h, proxied by the
 *   reference to MPI_Scan / MPI_Exscan (src/runtime/runtime_mpi.cpp:816-835).
 * For teams of more than one PE, source and dest must be symmetric-heap memory. */
int ishmemi_c_fcollect(int team, void *dest, const void *source, size_t nbytes);
int ishmemi_c_fcollect_on_stream(int team, void *dest, const void *source, size_t nbytes, int *ret,
                                 void *stream);
int ishmemi_c_collect(int team, void *dest, const void *source, size_t nbytes);
/* collect enqueued on `stream` (ishmemx_<TN>_collect_on_queue, src/ishmemx.h): the members'
 * byte counts are exchanged on the device inside the launch, so the call returns at once.  *ret as
 * for ishmemi_c_reduce_on_stream.  dest and (non-empty) source: symmetric-heap memory. */
int ishmemi_c_collect_on_stream(int team, void *dest, const void *source, size_t nbytes, int *ret,
                                void *stream);
int ishmemi_c_scan(int team, int dtype, int inclusive, void *dest, const void *source, size_t nelems);
/* broadcast: dest on every member (the root included) = the root's `nbytes` of source
 * (ishmem_<TN>_broadcast / ishmem_broadcastmem, src/ishmem.h:761-813, broadcast_impl.h's pull
 * variant).  `root` is the root's index in the team.  Sources outside the heap are staged. */
int ishmemi_c_broadcast(int team, void *dest, const void *source, size_t nbytes, int root);
/* broadcast enqueued on `stream` (ishmemx_<TN>_broadcast_on_queue, src/ishmemx.h:846-954): the
 * source must be symmetric-heap memory (the root's is found at the same offset), dest
 * device-writable on every member.  *ret as for ishmemi_c_reduce_on_stream. */
int ishmemi_c_broadcast_on_stream(int team, void *dest, const void *source, size_t nbytes, int root,
                                  int *ret, void *stream);
int ishmemi_c_scan_on_stream(int team, int dtype, int inclusive, void *dest, const void *source,
                             size_t nelems, int *ret, void *stream);
/* The `deps` / returned-event plumbing of every _on_queue form (fcollect, collect, inscan, exscan;
 * the reduce has ishmemi_c_reduce_on_stream_deps): make `stream` wait for deps[0..ndeps)
 * (hipEvent_t), and record `done` (hipEvent_t, may be NULL) on it after the call. */
int ishmemi_c_stream_wait_events(void *stream, void *const *deps, size_t ndeps);
int ishmemi_c_stream_record_event(void *stream, void *done);

/* ---- device-initiated collectives ----------------------------------------------------------
 * The reference's device-callable reductions (ishmemx_<TN>_<op>_reduce_work_group,
 * src/collectives/reduce_impl.h:386-418, :505-518, src/ishmemx.h:1648-1699) read the library
 * state from a SYCL device global.  A HIP user kernel lives in its own code object, so the state
 * is handed to it explicitly: ishmemi_c_device_ctx() returns a DEVICE pointer to this struct,
 * which the user passes to its kernel and on to the header-only device API (ishmemx_device.h).
 * Layout is part of the ABI. */
#define ISHMEMI_C_MAX_PES 16
/* Team slots: the reference's ISHMEM_TEAMS_MAX default and cap (src/ishmem/env_defs.h:34,
 * src/teams.cpp:245-248); ISHMEM_TEAMS_MAX (3..64) lowers the number in use. */
#define ISHMEMI_C_MAX_TEAMS 64
#define ISHMEMI_C_DEV_PHASES 4
typedef struct {
    int32_t pe, npes;
    uint64_t timeout_ticks;                       /* s_memrealtime ticks (100 MHz) */
    char *heap_base;                              /* this PE's symmetric heap */
    uint64_t heap_size;
    char *peer_heap[ISHMEMI_C_MAX_PES];           /* every PE's heap, mapped here */
    uint32_t *my_dflags;                          /* [team][phase][pe] epochs, fine-grained */
    uint32_t *peer_dflags[ISHMEMI_C_MAX_PES];
    uint32_t *epochs;                             /* [team] last device-API epoch (this PE) */
    uint32_t *err;                                /* device-API error word (host-visible) */
    int32_t team_start[ISHMEMI_C_MAX_TEAMS], team_stride[ISHMEMI_C_MAX_TEAMS];
    int32_t team_size[ISHMEMI_C_MAX_TEAMS], team_my_idx[ISHMEMI_C_MAX_TEAMS];
    uint64_t *dev_counts;                         /* symmetric [team][8] u64: device collect counts */
} ishmemi_c_device_ctx_t;
void *ishmemi_c_device_ctx(void);
/* Device-API context slots: every HIP translation unit that includes ishmemx_device.h owns a
 * `__device__ const ishmemi_c_device_ctx_t *` and registers the address of its host shadow here
 * from a static initializer.  init writes the context's device address into every registered slot
 * (hipMemcpyToSymbol) and finalize clears them; a slot registered after init is written at once.
 * Returns 0. */
int ishmemi_c_register_device_ctx_slot(const void *host_shadow);

/* ---- diagnostics / parameters ----------------------------------------------------------------
 * ishmemi_c_set_param names: "max_blocks" (workgroups per collective launch, <= 1024),
 * "ll_max_bytes" (cap on the one-hop granule path, default 524288, <= 1048576; the path also stops
 * at the team's ring capacity, 2 MiB / team size: get_param "ll_capacity_bytes" for TEAM_WORLD),
 * "timeout_ms" (bound on every device-side spin), "stream_order" (1: collectives issued on
 * different streams are ordered by the library in call order, ~2 us per call; 0, the default: the
 * caller orders them, as the reference requires), "oneshot_p2_max_bytes" (co-located two-member
 * teams: one-phase fold up to this size, default 32 MiB; 3-4 members: oneshot_p2 / 4 / (p - 1)),
 * "direct_p2" (1, default: that fold as barrier + one grid + barrier; 0: the persistent kernel's
 * one-shot mode), "phased_min_bytes" (payloads of at least this size take the phased path:
 * barrier, one-shot reduce-scatter, barrier, one-shot all-gather, barrier; -1 disables it),
 * "xgmi_ll_max_bytes" / "xgmi_fold_max_bytes" (teams whose members sit on different GPUs: the
 * granule-path / whole-array fold thresholds, -1 = the link-byte model of ishmemi_c_path_limits;
 * ISHMEM_XGMI_LL_MAX_BYTES / ISHMEM_XGMI_FOLD_MAX_BYTES at init), "xgmi_link_mbps" (the model's
 * link rate per direction, default 76800), "phase_events" (1: the next phased reduces record HIP
 * events between their five launches, read with ishmemi_c_phase_times; a measurement hook),
 * "debug"; A/B switches for measurements, set alike on every PE: "ar_shifted" (1, default: the
 * persistent kernel keeps 16-B items for sources on another 16-B phase than dest, read with
 * unaligned loads; 0: element-granular), "phase_unaligned" (1, default: the phased reduce-scatter
 * reads such sources with unaligned 16-B loads; 0: the realigning kernel), "rs_xcd" (1, default:
 * that reduce-scatter's XCD-grouped block order when the PE has its GPU to itself; 0: block
 * order), "collect_realign" (1, default: collect members off the 16-B grid realigned; 0: narrow
 * items), "block_spin" (blocking calls' wait: 2, default, spin on a stream-written host word; 1 the
 * spin then hipStreamSynchronize; 0 hipStreamSynchronize), "direct_max_pes" (largest team taking
 * the whole-array fold, default 4), "direct_inplace" (1, default: in-place calls with p * B <= 4 MiB
 * fold into the team's private scratch, allocated with the team, and copy back).  The thresholds
 * choose the kernels of a multi-PE call: init agrees on them (the minimum over the PEs; the
 * maximum for "phased_min_bytes") and a later set_param must be made with the same value on every
 * PE.  "max_blocks" may differ between PEs (the kernels grab work, nothing is paired by workgroup
 * index).  ishmemi_c_get_param also reports "staging_bytes", "heap_bytes", "flags_fine_grained",
 * "ll_capacity_bytes" / "ll_limit_bytes" / "fold_limit_bytes" (TEAM_WORLD's granule ring capacity,
 * granule threshold and whole-array fold bound), "team_colocated" (1: every TEAM_WORLD member on
 * one GPU), "teams_max" (ISHMEM_TEAMS_MAX, default 64), "flag_block_bytes" (flag memory this PE
 * holds: the base block plus one block per split team it belongs to; "flag_block_bytes_round5" =
 * round 5's fixed 16-slot block, for comparison; "flag_block_pool_bytes" = the exported team blocks
 * this PE holds in its pool, in use or free for the next split), "init_us_<phase>" (init's phases: hip, heap,
 * flags, bootstrap, ipc_heap, ipc_flags, teams, total; printed under ISHMEM_DEBUG=2), "cu_count"
 * (compute units of this PE's device) and "device_share" (PEs of the job on this PE's device: 1
 * with one PE per GPU). */
const char *ishmemi_c_last_error(void);
int ishmemi_c_set_param(const char *name, long long value);
long long ishmemi_c_get_param(const char *name);
/* Durations (ms) of the last phased reduce's five launches — start barrier, reduce-scatter grid,
 * middle barrier, all-gather grid, end barrier — recorded while set_param("phase_events", 1) is
 * on.  Synchronises on the last event.  Returns 0, or nonzero if no phased reduce was recorded. */
int ishmemi_c_phase_times(float *ms5);
/* Number of collective launches whose device-side barriers timed out since init. */
int ishmemi_c_error_count(void);
/* Bytes of one element of `dtype` (0 if invalid); 1 if (op, dtype) is a valid pair. */
size_t ishmemi_c_dtype_size(int dtype);
int ishmemi_c_op_dtype_valid(int op, int dtype);
/* Partition used by the multi-PE schedule: items of member `c` out of `nitems` (test hook). */
int ishmemi_c_chunk_bounds(uint64_t nitems, int npes, int c, uint64_t *begin, uint64_t *end);
/* Path thresholds of a team of `npes` members (no reference counterpart; no GPU needed): payloads
 * up to *ll_limit bytes take the granule path, disjoint payloads up to *fold_limit the whole-array
 * fold between two barriers (0: never).  colocated != 0: every member on one GPU (round 5's
 * measured crossovers); 0: members on different GPUs (the link-byte model of runtime.cpp
 * path_limits, or ISHMEM_XGMI_LL_MAX_BYTES / ISHMEM_XGMI_FOLD_MAX_BYTES).  Computed with the
 * current parameters (the defaults before init). */
int ishmemi_c_path_limits(int npes, int colocated, long long *ll_limit, long long *fold_limit);
/* Native bootstrap self-test (no GPU needed): allgather of one int per PE + barrier.
 * Fills out[npes]; used by the multi-process CPU tests. */
int ishmemi_c_bootstrap_selftest(int pe, int npes, const char *key, int value, int *out);
const char *ishmemi_c_version(void);

#ifdef __cplusplus
}
#endif

#endif /* ISHMEM_AMD_CAPI_H */
