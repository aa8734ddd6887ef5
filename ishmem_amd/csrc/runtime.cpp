// ishmem_amd — host runtime + C-ABI of the reduction-collective path.
//
// Reference layers replaced here: L1 device/memory substrate (Level-Zero
// accelerator src/accelerator.cpp, symmetric heap src/memory.cpp:35-132, IPC handle exchange
// src/ipc.cpp:123-233, team tables src/teams.cpp:73-161), and L4's host dispatch
// ishmemi_reduce (src/collectives/reduce_impl.h:259-317) plus the on_queue launcher (:444-474).
// The device data plane is in kernels.hip.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>
#include <stdint.h>
#include <errno.h>
#include <sys/prctl.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <limits>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "bootstrap.h"
#include "kernels.h"
#include "types.h"

namespace ishmemi {
namespace {

// Team slots: the reference's table size, ISHMEM_TEAMS_MAX (default 64, src/ishmem/env_defs.h:34),
// capped at 64 by its 64-bit slot mask (src/teams.cpp:245-248) — as here, where the free-slot mask
// agreed at split is a u64.  Slots 0-2 are WORLD, SHARED and NODE.
constexpr int kMaxTeams = ISHMEMI_C_MAX_TEAMS;
constexpr int kPredefTeams = ISHMEMI_C_TEAM_NODE + 1;
constexpr int kTeamsMaxDefault = 64;
static_assert(kMaxTeams == 64, "the split's free-slot mask is a u64");
static_assert(kMaxPes == ISHMEMI_C_MAX_PES, "device ctx layout");
// Device-API flags ([team][phase][pe] u32, 256 B per slot).
constexpr size_t kDevFlagWordsPerTeam = (size_t) ISHMEMI_C_DEV_PHASES * kMaxPes;
constexpr size_t kDevFlagBytes = (size_t) kMaxTeams * kDevFlagWordsPerTeam * 4;
// Base flag block, allocated and IPC-exported at init (round 6): the predefined teams' flag blocks
// (kernels.h kTeamFlagBytes each), the device-API flags of every slot, then the predefined teams'
// small-message rings (kLLTeamBytes each), 256-B aligned.  A team created by a split gets a block
// of its own (kTeamAllocBytes: flag block + ring), taken from the PE's pool and exchanged among its
// members at the split, returned to the pool at destroy (TeamMem, PoolBlock: HIP keeps an
// IPC-exported allocation after hipFree, so blocks are reused and freed only at finalize); a PE
// holds (and peers map) at most as many blocks as teams existed at once.  Round 5 reserved flag block + ring for 16 slots at init: 132 MiB per PE whatever the
// teams (kRound5FlagBytes, for get_param "flag_block_bytes" comparisons).
constexpr size_t kBaseDevOffset = (size_t) kPredefTeams * kTeamFlagBytes;
constexpr size_t kBaseLLOffset = (kBaseDevOffset + kDevFlagBytes + 255) & ~(size_t) 255;
constexpr size_t kBaseAllocBytes = kBaseLLOffset + (size_t) kPredefTeams * kLLTeamBytes;
constexpr size_t kTeamLLOffset = (kTeamFlagBytes + 255) & ~(size_t) 255;
constexpr size_t kTeamAllocBytes = kTeamLLOffset + kLLTeamBytes;
constexpr size_t kRound5FlagBytes = (((size_t) 16 * kTeamFlagBytes + 16 * kDevFlagWordsPerTeam * 4 + 255) & ~(size_t) 255) +
                                    (size_t) 16 * kLLTeamBytes;
// In-place whole-array fold (reduce_heap): while p * B <= this, into a team-private scratch of
// kInplaceFoldBytes / p + 256 bytes, allocated when the team is created.
constexpr uint64_t kInplaceFoldBytes = 4u << 20;
constexpr size_t kHeapAlign = 256;
// Symmetric scratch of the team-management collectives (split's slot mask and handle exchange).
constexpr size_t kTeamScratchBytes = 4096;
constexpr size_t kSplitRecBytes = 128;  // one member's record in the split's handle exchange
// Offset of team_exchange's arrays in the host-mapped error-word allocation (after the words).
constexpr size_t kErrExchOffset = ((kMaxTeams + 1) * sizeof(uint32_t) + 63) & ~(size_t) 63;
// Completion word of the blocking calls' host wait (host_wait), on its own line.
constexpr size_t kErrDoneOffset = (kErrExchOffset + 2 * kMaxPes * sizeof(uint64_t) + 63) & ~(size_t) 63;
constexpr size_t kLargeAllocBytes = (size_t) 1 << 20, kLargeAlign = (size_t) 2 << 20;
// Slots of the host-memory pipeline (reduce_staged): chunk k uses slot k mod slots, a chunk is
// staging / slots bytes; ISHMEM_STAGING_SLOTS, agreed at init (the minimum).  Default 2, i.e.
// 64 MiB chunks of the 128 MiB region (round 4, scripts/e2e_b2b.sh / e2e_window.sh,
// profiles/r04/host_pipeline/queue_depth/): with 32 MiB chunks (4 slots) single calls of 4-8 GiB
// and back-to-back 1 GiB calls fell to 11-38 GiB/s in most runs, with 64 MiB chunks they held
// 42.5-45.5; single synced 1 GiB calls are 42-44 either way (the copy engines do not keep both
// directions streaming on 32 MiB transfers queued deep; a host-side window of chunks in flight,
// tried, made it worse: 19-25 GiB/s).
constexpr int kMaxStagingSlots = 8;
constexpr int kStagingSlotsDefault = 2;
constexpr int kStagedCopyKernelDefault = 0;

thread_local std::string g_last_error;

// IPC export mode.  The MI355X driver on this node exports device memory for IPC as dma-buf only,
// and ROCr picks the export mode from HSA_ENABLE_IPC_MODE_LEGACY when HIP initialises (the first
// HIP call of the process).  A drop-in program launched the reference's way (`mpirun -n N ./app`,
// test/cmake/common.cmake:28-43) sets nothing, so the library sets the variable to 0 when it is
// loaded — for a program linked against it that is before main and before any HIP call — unless
// the user already chose a value.  A process that initialised HIP before loading the library
// (e.g. a Python program that used torch.cuda first) keeps the mode HIP started with; init then
// fails naming the variable (ipc_hint) instead of with a bare "invalid argument".
bool g_ipc_env_set_by_lib = false;

__attribute__((constructor)) void ipc_mode_default()
{
    if (!getenv("HSA_ENABLE_IPC_MODE_LEGACY")) {
        setenv("HSA_ENABLE_IPC_MODE_LEGACY", "0", 0);
        g_ipc_env_set_by_lib = true;
    }
}

std::string ipc_hint()
{
    const char *v = getenv("HSA_ENABLE_IPC_MODE_LEGACY");
    std::string h = std::string(" [HSA_ENABLE_IPC_MODE_LEGACY=") + (v ? v : "(unset)");
    if (v && strcmp(v, "0") == 0)
        h += g_ipc_env_set_by_lib ? ", set by libishmem_amd when it loaded" : "";
    h += ": this node's driver shares device memory between processes as dma-buf only, which needs "
         "HSA_ENABLE_IPC_MODE_LEGACY=0 in the environment before the process's first HIP call; "
         "libishmem_amd sets it when loaded unless the variable is already set, so a process that "
         "set it to 1, or initialised HIP (e.g. torch.cuda) before loading the library, must set it itself]";
    return h;
}

// ISHMEM_DEBUG: the reference's boolean (src/ishmem/env_defs.h:10, parsed by
// src/env_utils.cpp:138-149: "0" / "false" off, any other value on); a decimal value above 1 is
// this library's more verbose level.
int debug_level()
{
    const char *s = getenv("ISHMEM_DEBUG");
    if (!s || !*s) return 0;
    char *end = nullptr;
    const long v = strtol(s, &end, 10);
    if (end != s && *end == '\0') return v > 0 ? (int) std::min<long>(v, 1 << 20) : 0;
    return strcasecmp(s, "false") == 0 ? 0 : 1;
}

int fail(const std::string &msg)
{
    g_last_error = msg;
    if (debug_level() > 0)
        fprintf(stderr, "[ishmem_amd] %s\n", msg.c_str());
    return 1;
}

int hipfail(const char *what, hipError_t e)
{
    return fail(std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) return hipfail(#expr, e_);                                           \
    } while (0)

// Byte counts from the environment: plain bytes or with a K / M / G / T suffix (powers of 1024),
// optionally followed by "iB" or "B" ("16M", "16MiB", "16MB"); surrounding blanks allowed.  Anything
// else (trailing junk, no digits, NaN) is an error that fails init: these values choose kernel
// paths every PE must agree on, so a typo must not parse as something else.  Values past
// LLONG_MAX clamp to it; negative values mean "off" (-1) where the variable allows it.
std::string g_env_error;  // first malformed variable seen by init's parsing

bool parse_bytes(const char *s, long long &out)
{
    while (*s == ' ' || *s == '\t') ++s;
    char *end = nullptr;
    double v = strtod(s, &end);
    if (end == s || v != v) return false;
    double mul = 1.0;
    switch (*end) {
        case 'k': case 'K': mul = 1024.0; ++end; break;
        case 'm': case 'M': mul = 1024.0 * 1024.0; ++end; break;
        case 'g': case 'G': mul = 1024.0 * 1024.0 * 1024.0; ++end; break;
        case 't': case 'T': mul = 1024.0 * 1024.0 * 1024.0 * 1024.0; ++end; break;
        default: break;
    }
    if (mul > 1.0 && (*end == 'i' || *end == 'I')) ++end;
    if (*end == 'b' || *end == 'B') ++end;
    while (*end == ' ' || *end == '\t') ++end;
    if (*end) return false;
    v *= mul;
    if (v < 0) out = -1;
    else if (v >= 9.2233720368547748e18) out = std::numeric_limits<long long>::max();
    else out = (long long) v;
    return true;
}

long long env_bytes(const char *name, long long dflt)
{
    const char *s = getenv(name);
    if (!s || !*s) return dflt;
    long long v = 0;
    if (!parse_bytes(s, v)) {
        if (g_env_error.empty())
            g_env_error = std::string(name) + "='" + s + "' is not a byte count (digits, then K / M / G / T)";
        return dflt;
    }
    return v;
}

// Sizes that must be positive (heap, staging).
size_t env_size(const char *name, size_t dflt)
{
    const long long v = env_bytes(name, (long long) dflt);
    if (v <= 0) {
        if (g_env_error.empty() && getenv(name) && *getenv(name))
            g_env_error = std::string(name) + " must be a positive byte count";
        return dflt;
    }
    return (size_t) v;
}

// Integers from the environment: decimal, surrounding blanks allowed.  A malformed ISHMEM_*
// value fails init with the variable named, like a malformed byte count ("4x", "sixteen" and
// out-of-range values used to parse as a prefix or wrap); other variables (HIP's) fall back to
// the default.
long long env_ll(const char *name, long long dflt)
{
    const char *s = getenv(name);
    if (!s || !*s) return dflt;
    const char *b = s;
    while (*b == ' ' || *b == '\t') ++b;
    char *end = nullptr;
    errno = 0;
    const long long v = strtoll(b, &end, 10);
    const char *e = end;
    while (*e == ' ' || *e == '\t') ++e;
    if (end == b || *e || errno == ERANGE) {
        if (strncmp(name, "ISHMEM_", 7) == 0 && g_env_error.empty())
            g_env_error = std::string(name) + "='" + s + "' is not an integer";
        return dflt;
    }
    return v;
}

// The reference's boolean variables (src/env_utils.cpp:138-149): "0" or "false" (any case) is
// false, any other value true; unset (or empty, here) is the default.
bool env_flag_false(const char *name)
{
    const char *s = getenv(name);
    return s && *s && (strcmp(s, "0") == 0 || strcasecmp(s, "false") == 0);
}
bool env_flag_true(const char *name)
{
    const char *s = getenv(name);
    return s && *s && !env_flag_false(name);
}

// ISHMEM_* variables this library reads (runtime, launcher identity, build, tests) or accepts from
// the reference's list (src/ishmem/env_defs.h; the ones this path has no use for are read and
// ignored, as a drop-in must start under the reference's job scripts).  Any other ISHMEM_* name
// gets the reference's warning at init (src/env_utils.cpp:193-196), not an error.
void warn_unknown_env()
{
    static const char *const known[] = {
        // the reference's (src/ishmem/env_defs.h)
        "DEBUG", "ENABLE_VERBOSE_PRINT", "STACK_PRINT_LIMIT", "ENABLE_GPU_IPC", "ENABLE_GPU_IPC_PIDFD",
        "SYMMETRIC_SIZE", "ENABLE_ACCESSIBLE_HOST_HEAP", "NBI_COUNT", "MWAIT_BURST", "SHMEM_LIB_NAME",
        "MPI_LIB_NAME", "PMI_LIB_NAME", "TEAMS_MAX", "TEAM_SHARED_ONLY_SELF", "RUNTIME", "RUNTIME_USE_OSHMPI", "ROOT",
        // this library's
        "PE", "NPES", "DEVICE", "BOOTSTRAP_KEY", "TIMEOUT_MS", "MAX_BLOCKS", "WAIT_SLOTS", "LL_MAX_BYTES",
        "ONESHOT_P2_MAX_BYTES", "PHASED_MIN_BYTES", "PHASED_PEER_NT", "STAGING_SIZE", "STAGING_SLOTS",
        "STAGED_COPY_KERNEL", "STREAM_ORDER", "FLAGS_KIND", "EP_UNCACHED", "BARRIER_KIND", "XGMI_LL_MAX_BYTES",
        "XGMI_FOLD_MAX_BYTES", "TEST_FLAGS_UNAVAILABLE", "TEST_PCI_BUS",
        // the Python package, build and bench harness
        "AMD_LIB", "OFFLOAD_ARCH", "BENCH_SAME_DEVICE", "BENCH_EMULATE_SHARE1", "BENCH_SETUP_WATCHDOG_S"};
    for (char **e = ::environ; e && *e; ++e) {
        if (strncmp(*e, "ISHMEM_", 7) != 0) continue;
        const char *name = *e + 7, *eq = strchr(name, '=');
        const size_t len = eq ? (size_t) (eq - name) : strlen(name);
        bool ok = false;
        for (const char *k : known) ok = ok || (strlen(k) == len && strncmp(k, name, len) == 0);
        if (!ok) fprintf(stderr, "[ishmem_amd] WARN: Environment variable 'ISHMEM_%.*s' is not a supported variable\n", (int) len, name);
    }
}

// Lowest ISHMEM_WAIT_SLOTS / set_param("wait_slots") accepted: the process's hardware queue count.
long long wait_slots_floor() { return std::max<long long>(1, env_ll("GPU_MAX_HW_QUEUES", 4)); }

struct Team {
    bool valid = false;
    int start = 0, stride = 1, size = 1;  // in world PEs (src/teams.h:56-76)
    int my_idx = -1;                      // my index in the team, -1 if not a member
    int num_contexts = 0;                 // ishmem_team_config_t given at split (reported only)
    // Every member on one device (co-located PEs: tests, rehearsals) or not (one PE per GPU over
    // xGMI): picks the path thresholds (path_limits).  The same on every member (from the
    // device identities allgathered at init).
    bool colocated = true;
};

// Memory of a team slot on this PE (round 6).  Predefined teams point into the base block; a
// split team uses one block of this PE's team-block pool (flag block + ring) and its co-members'
// pool blocks, mapped here; destroy returns the block to the pool.
struct TeamMem {
    uint32_t *flags[kMaxPes] = {};  // the team's flag block on world PE j, mapped here (members only)
    uint64_t *ring[kMaxPes] = {};   // the team's small-message ring on world PE j
    int pool_idx = -1;              // this PE's pool block of a split team
    char *fold_scratch = nullptr;   // in-place whole-array fold (kInplaceFoldBytes / p + 256 B)
    size_t fold_scratch_bytes = 0;
};

// Team blocks are pooled, never freed while the library is initialised: HIP keeps an allocation
// that was exported for IPC allocated after hipFree until the process exits (8.25 MiB blocks,
// 100 rounds: hipFree returned nothing after hipIpcGetMemHandle, every byte without it;
// tools/ipc_leak_probe.py, profiles/r06/teams/), so a split / destroy cycle that allocated, exported
// and freed a block leaked ~10 MiB per team and PE (the churn test caught 1460 MiB over 120
// rounds).  A split takes a free pool block (zeroed) or exports a new one; destroy returns it.
// The pool grows to the most split teams this PE was in at once.  Peers' pool blocks stay mapped
// here once opened (keyed by PE and pool index), so re-splits reuse the mapping instead of
// opening the handle again.
struct PoolBlock {
    uint32_t *ptr = nullptr;
    hipIpcMemHandle_t handle{};
    bool in_use = false;
};

constexpr long long kPhasedOff = std::numeric_limits<long long>::max();
// Round 3 put the threshold at 16 MiB: 2 PEs x 1 GiB 0.84 ms phased against 0.99-1.13 ms
// persistent; 2 PEs x 32 / 64 MiB 36 / 59 us against the two-member one-shot fold's 42 / 78 us;
// 4 PEs x 16 MiB 40 vs 48 us.  Round 4 caps the persistent kernel's grid (it waits for peers, so
// it may hold at most 1 / wait_slots of the device, kernels.h) and lowers the threshold to 4 MiB,
// where the phased path's never-waiting full-device grids overtake the capped grid
// (profiles/r04/wait_cost/: 2 PEs with one-PE-per-GPU shapes, 4 / 8 MiB 16.6-17.3 / 19.2-20.1 us
// phased against 20.5-20.7 / 33.8-34.0 us persistent, 2 MiB 16-17 against 14.1-14.3 us).  Over
// xGMI the same crossover follows from the links: a 64-workgroup grid keeps ~1 MiB of peer loads
// in flight, near the 7 links' bandwidth-delay product, while the three barriers cost a few fabric
// round trips; the N > 1 bench line's xgmi_tuning leg records both paths at 2-64 MiB.
constexpr long long kPhasedDefault = 4ll << 20;
// Round 3 turned it off when more than 4 PEs shared one GPU (co-located rehearsals, where the
// three barrier launches cost ~40-80 us each among eight time-sliced processes).  Round 4 drops
// that rule: co-located runs take the path one PE per GPU takes, so the 8-PE tests at BASELINE's
// sizes exercise rs_phase_kernel<P=8> + ag_phase_kernel.

struct PeRecord {
    int32_t pe, pid, device, flags_kind;
    int32_t flags_kind_requested;  // ISHMEM_FLAGS_KIND (tests): where this PE's ladder started
    char pci_bus[32];  // identifies the physical GPU across processes
    uint64_t heap_size;
    // Path-choosing parameters (LL / two-member one-shot / phased, staging chunks): every PE must
    // take the same path per call, so init agrees on them.  max_blocks travels for diagnostics
    // only: the kernels grab work, so the grid cap is per PE.
    int64_t max_blocks, ll_max_bytes, oneshot_p2, phased_min;
    uint64_t staging_bytes;
    int64_t staging_slots;
    int64_t xgmi_ll_max, xgmi_fold_max;  // path_limits overrides for cross-device teams (-1: model)
    hipIpcMemHandle_t heap_handle;
    hipIpcMemHandle_t flags_handle;
};

struct State {
    std::mutex mu;
    bool initialized = false;
    int pe = 0, npes = 1, device = 0;
    ShmBootstrap boot;

    char *heap = nullptr;
    size_t heap_size = 0;
    std::map<size_t, size_t> free_list;  // offset -> bytes
    std::map<size_t, size_t> used;       // offset -> bytes
    char *peer_heap[kMaxPes] = {};

    uint32_t *flags = nullptr;  // base flag block (predefined teams, device-API flags), see FlagMem
    int flags_kind = 0;         // FlagMem of the base block; split teams' blocks take the same kind
    uint32_t *peer_flags[kMaxPes] = {};  // every PE's base block, mapped here
    int dev_id[kMaxPes] = {};            // world PE j's device, as an index into the job's devices
    TeamMem tmem[kMaxTeams];
    int teams_max = kTeamsMaxDefault;    // ISHMEM_TEAMS_MAX: slots [0, teams_max) are used
    size_t team_block_bytes = 0;         // pool blocks in use by split teams (get_param "flag_block_bytes")
    std::vector<PoolBlock> team_pool;    // this PE's team blocks (PoolBlock)
    std::map<std::pair<int, uint32_t>, void *> peer_pool;  // (world PE, its pool index) -> mapping here
    uint32_t *err_host = nullptr;  // host-mapped error words, one per team (+1: device API)
    uint32_t *err_dev = nullptr;
    // Host-mapped coherent [2][kMaxPes] u64 (same allocation as err_host): team_exchange's arrays.
    uint64_t *exch_host = nullptr, *exch_dev = nullptr;
    // Blocking calls' completion word (host-mapped; host_wait) and its sequence; block_spin:
    // 0 = hipStreamSynchronize, 1 = spin on the word a stream write stores after the call's
    // launches, then hipStreamSynchronize, 2 = the spin alone (set_param "block_spin").
    uint32_t *done_host = nullptr, *done_dev = nullptr;
    uint32_t done_seq = 0;
    int block_spin = 2;
    ishmemi_c_device_ctx_t *dctx = nullptr;  // device copy of the device-API context
    uint32_t *dev_epochs = nullptr;
    uint32_t *kern_ep = nullptr;  // [team][kEpTeamWords] launch words of the host-launched kernels

    char *team_scratch = nullptr;  // small symmetric buffer for team-management collectives
    char *count_slots = nullptr;   // symmetric, one 64-B line per team: collect_on_stream counts
    char *staging = nullptr;  // symmetric staging region for non-heap / host buffers
    size_t staging_bytes = 0;
    hipStream_t copy_in = nullptr, copy_out = nullptr;  // staging pipeline streams
    // Stream of the previous collective: a collective enqueued on another stream first waits
    // for it, so epochs, flag rows and the staging region are used in call order.
    hipStream_t last_stream = nullptr;
    bool last_stream_set = false;
    bool stream_order = false;
    // Two-member teams fold the whole array in one phase up to this many bytes
    // (ISHMEM_ONESHOT_P2_MAX_BYTES; round 5: barrier + fold grid + barrier, 1-16 MiB 9.5-22.6 us
    // against 11.4-29 us; tied at 32 MiB on one GPU, where RS + AG's 2.5B of HBM per PE against
    // 3B then wins — over one xGMI link both move B per direction).
    long long oneshot_p2 = 32ll << 20;
    // Payloads of at least this many bytes (16-B vector body) take the phased reduce-scatter /
    // all-gather (two one-shot grids between one-workgroup barriers, kernels_impl.h) instead of
    // the persistent kernel (ISHMEM_PHASED_MIN_BYTES; kPhasedOff disables it).
    long long phased_min = kPhasedDefault;
    hipEvent_t order_ev = nullptr;
    // Completion of the last use of the staging region (staged pipeline or scan scratch); the
    // next user waits on it, whatever stream it runs on.
    hipEvent_t staging_ev = nullptr;
    bool staging_used = false;
    int staging_slots = kStagingSlotsDefault;
    // Host buffers the GPU can address (pinned / registered): copy chunks in (bit 1) / out (bit 0)
    // of the staging region with the copy KERNEL instead of the DMA engines (ISHMEM_STAGED_COPY_KERNEL,
    // set_param "staged_copy_kernel"; per PE, nothing is paired).
    int staged_copy_kernel = 0;
    bool test_flags_unavailable = false;  // ISHMEM_TEST_FLAGS_UNAVAILABLE (alloc_flags)
    // Measurement only (set_param "phased_peer_nt"): the phased grids load peers' bytes
    // nontemporal instead of sc0 sc1 (kernels.h PhaseArgs::peer_nt).  Must be set alike on every PE.
    int phased_peer_nt = 0;
    // Persistent kernel with sources on another 16-B phase than dest (set_param "ar_shifted",
    // default 1): vector items laid out by dest, the sources read with unaligned 16-B loads;
    // 0 = the element-granular instantiation (A/B only).
    int ar_shifted = 1;
    // The shifted reduce-scatter's block order (PhaseArgs::xcd_group; set_param "rs_xcd", default 1).
    int rs_xcd = 1;
    // Two-member disjoint reduces up to oneshot_p2 bytes: barrier + one whole-array fold grid +
    // barrier (1, default) or the persistent kernel's one-shot mode (0; set_param "direct_p2",
    // alike on every PE).
    int direct_p2 = 1;
    int direct_max_pes = 4;  // the whole-array fold up to this team size (set_param "direct_max_pes", >= 2)
    int direct_inplace = 1;
    // Cross-device teams' thresholds (path_limits): -1 = the link-byte model's; ISHMEM_XGMI_LL_MAX_BYTES /
    // ISHMEM_XGMI_FOLD_MAX_BYTES (agreed at init) or set_param override them, e.g. with the crossovers
    // the N > 1 bench line's `recommended` block measured on the node.
    long long xgmi_ll_max = -1, xgmi_fold_max = -1;
    double xgmi_link_bps = 76.8e9;  // per link and direction (set_param "xgmi_link_mbps")
    hipEvent_t ev_in[kMaxStagingSlots] = {}, ev_red[kMaxStagingSlots] = {}, ev_out[kMaxStagingSlots] = {};

    Team teams[kMaxTeams];
    int max_blocks = kMaxBlocks;
    long long ll_max_bytes = (long long) kLLDefaultBytes;
    long long timeout_ms = 60000;
    int debug = 0;
    int error_count = 0;
    uint64_t *trace = nullptr;  // development phase-timestamp buffer (device memory)
    // Measurement hook (set_param "phase_events"): events around the phased reduce's launches.
    bool phase_events = false, phase_recorded = false;
    hipEvent_t phase_ev[6] = {};
    // Init phase durations (us), printed under ISHMEM_DEBUG=2 and read by get_param("init_us_<phase>").
    double init_us[8] = {};
};

// Init phases timed (State::init_us): names for the debug line and get_param.
const char *const kInitPhase[8] = {"hip", "heap", "flags", "bootstrap", "ipc_heap", "ipc_flags", "teams", "total"};

State &S()
{
    static State s;
    return s;
}

// Device-API context slots (ishmemi_c_register_device_ctx_slot): host shadows of the per-code-object
// `__device__` context pointers of include/ishmemx_device.h.
struct CtxSlots {
    std::mutex mu;
    std::vector<const void *> shadows;
};
CtxSlots &ctx_slots()
{
    static CtxSlots c;
    return c;
}

// Writes `ctx` (device address, or null) into one slot.  A code object whose kernels never use
// the device API may have dropped the variable: that slot is skipped.
void write_ctx_slot(const void *shadow, const void *ctx)
{
    if (hipMemcpyToSymbol(shadow, &ctx, sizeof(ctx), 0, hipMemcpyHostToDevice) != hipSuccess)
        (void) hipGetLastError();
}

void write_ctx_slots(const void *ctx)
{
    CtxSlots &c = ctx_slots();
    std::lock_guard<std::mutex> lk(c.mu);
    for (const void *sh : c.shadows) write_ctx_slot(sh, ctx);
}

bool in_heap(const State &s, const void *p)
{
    return s.heap && (const char *) p >= s.heap && (const char *) p < s.heap + s.heap_size;
}

// Address of heap pointer `p` (own heap) as mapped in this process for world PE `pe`.
char *translate(const State &s, const void *p, int pe)
{
    if (!in_heap(s, p)) return nullptr;
    if (pe == s.pe) return (char *) p;
    if (pe < 0 || pe >= s.npes || !s.peer_heap[pe]) return nullptr;
    return s.peer_heap[pe] + ((const char *) p - s.heap);
}

// A predefined team's flag block / ring inside a base block (own or a peer's, mapped here).
uint32_t *base_team_flags(uint32_t *base, int team)
{
    return base ? base + (size_t) team * (kTeamFlagBytes / 4) : nullptr;
}

uint64_t *base_team_ring(uint32_t *base, int team)
{
    return base ? (uint64_t *) ((char *) base + kBaseLLOffset + (size_t) team * kLLTeamBytes) : nullptr;
}

// The device-API flag rows of every slot, in a base block.
uint32_t *dev_flags(uint32_t *base) { return base ? base + kBaseDevOffset / 4 : nullptr; }

// ---------------- symmetric heap allocator (deterministic first fit, same on every PE) -------
void *heap_alloc(State &s, size_t bytes, size_t align)
{
    if (bytes == 0) bytes = 1;
    align = std::max(align, kHeapAlign);
    // Large arrays start on a 2 MiB boundary: streaming a 1 GiB copy from 256-B-skewed
    // operands measured 80.3 % of HBM peak vs 83.9 % aligned (tools/stream_variants.hip,
    // layouts heap256 / heap0, profiles/r01_extra/stream_variants_layout.txt).
    if (bytes >= kLargeAllocBytes) align = std::max(align, kLargeAlign);
    bytes = (bytes + kHeapAlign - 1) & ~(kHeapAlign - 1);
    for (auto it = s.free_list.begin(); it != s.free_list.end(); ++it) {
        const size_t off = it->first, len = it->second;
        const size_t aligned = (off + align - 1) & ~(align - 1);
        if (aligned + bytes > off + len) continue;
        s.free_list.erase(it);
        if (aligned > off) s.free_list[off] = aligned - off;
        if (aligned + bytes < off + len) s.free_list[aligned + bytes] = off + len - aligned - bytes;
        s.used[aligned] = bytes;
        return s.heap + aligned;
    }
    fail("ishmem_malloc: symmetric heap exhausted (raise ISHMEM_SYMMETRIC_SIZE)");
    return nullptr;
}

void heap_free(State &s, void *p)
{
    if (!p || !in_heap(s, p)) return;
    const size_t off = (char *) p - s.heap;
    auto it = s.used.find(off);
    if (it == s.used.end()) return;
    size_t start = off, len = it->second;
    s.used.erase(it);
    auto next = s.free_list.lower_bound(start);
    if (next != s.free_list.end() && next->first == start + len) {
        len += next->second;
        s.free_list.erase(next);
    }
    auto prev = s.free_list.lower_bound(start);
    if (prev != s.free_list.begin()) {
        --prev;
        if (prev->first + prev->second == start) {
            start = prev->first;
            len += prev->second;
            s.free_list.erase(prev);
        }
    }
    s.free_list[start] = len;
}

// ---------------- launch planning ----------------------------------------------------------
struct Plan {
    bool vec;
    uint64_t head, nitems, tail, items_per_chunk, seg_items;
    int grid;
};

// The partition of the multi-PE schedule: member c owns items [c*ipc, min((c+1)*ipc, n)),
// ipc rounded up to 64 items (1 KiB of 16-B vectors) so chunk edges stay line aligned.
uint64_t items_per_chunk(uint64_t nitems, int npes)
{
    const uint64_t per = (nitems + (uint64_t) npes - 1) / (uint64_t) npes;
    return std::max<uint64_t>(64, (per + 63) & ~uint64_t(63));
}

// Reduce-scatter segment (the unit of work grabbing and of the RS -> AG hand-off): whole tiles,
// at most kMaxBlocks segments per chunk (one "ready" flag slot each).
constexpr uint64_t kTileItems = (uint64_t) kBlock * kUnroll;
uint64_t seg_items(uint64_t chunk_items)
{
    const uint64_t per = (chunk_items + kMaxBlocks - 1) / kMaxBlocks;
    return std::max<uint64_t>(kTileItems, (per + kTileItems - 1) / kTileItems * kTileItems);
}

uint64_t nsegs(uint64_t len, uint64_t seg) { return std::max<uint64_t>(1, (len + seg - 1) / seg); }

Plan make_plan(const void *dst, const void *const *srcs, int nsrc, size_t n, size_t es, int npes,
               int max_blocks, int max_grid)
{
    Plan pl{};
    const uintptr_t d = (uintptr_t) dst;
    bool same_residue = (d % es) == 0;
    for (int i = 0; i < nsrc; ++i) {
        const uintptr_t sp = (uintptr_t) srcs[i];
        same_residue = same_residue && ((sp ^ d) & 15) == 0 && (sp % es) == 0;
    }
    pl.vec = same_residue;
    if (pl.vec) {
        const size_t mis = d & 15;
        pl.head = std::min<uint64_t>(n, mis ? (16 - mis) / es : 0);
        const uint64_t ve = 16 / es;
        pl.nitems = (n - pl.head) / ve;
        pl.tail = n - pl.head - pl.nitems * ve;
    } else {
        pl.head = 0;
        pl.nitems = n;
        pl.tail = 0;
    }
    if (npes > 1) {
        // Workgroups: enough for the larger of the two phases' work lists (RS segments of one
        // chunk; AG items = p-1 peers x segments), capped; the kernel grabs work, so any grid
        // size is correct.
        pl.items_per_chunk = items_per_chunk(pl.nitems, npes);
        pl.seg_items = seg_items(pl.items_per_chunk);
        const uint64_t ns = nsegs(std::min(pl.items_per_chunk, pl.nitems), pl.seg_items);
        const uint64_t g = std::max<uint64_t>(ns, (uint64_t) (npes - 1) * ns);
        pl.grid = (int) std::max<uint64_t>(1, std::min<uint64_t>(g, (uint64_t) max_blocks));
    } else {
        pl.items_per_chunk = pl.nitems;
        const uint64_t g = (pl.nitems + kFaninBlock - 1) / kFaninBlock;
        pl.grid = (int) std::max<uint64_t>(1, std::min<uint64_t>(g, (uint64_t) max_grid));
    }
    return pl;
}

// Fills the kernel arguments common to every collective of `team`.
int team_args(State &s, int team, ReduceArgs &a, std::string &why)
{
    Team &t = s.teams[team];
    memset(&a, 0, sizeof(a));
    a.p = t.size;
    a.me = t.my_idx;
    a.my_flags = s.tmem[team].flags[s.pe];
    a.err = s.err_dev + team;
    a.timeout_ticks = (uint64_t) s.timeout_ms * 100000ull;  // s_memrealtime runs at 100 MHz
    for (int j = 0; j < t.size; ++j) {
        const int gpe = t.start + j * t.stride;
        a.peer_flags[j] = s.tmem[team].flags[gpe];
        if (!a.peer_flags[j]) {
            why = "team member " + std::to_string(gpe) + " has no mapped flag block";
            return 1;
        }
    }
    a.ep_ctr = s.kern_ep + (size_t) kEpTeamWords * team;
    return 0;
}

int check_team_errors(State &s, int team)
{
    const uint32_t e = __atomic_load_n(&s.err_host[team], __ATOMIC_ACQUIRE);
    if (e) {
        __atomic_store_n(&s.err_host[team], 0u, __ATOMIC_RELEASE);
        s.error_count++;
        char mask[16];
        snprintf(mask, sizeof(mask), "0x%x", e);
        return fail(std::string("device barrier timed out (phase mask ") + mask +
                    "): a team member did not arrive within timeout_ms");
    }
    return 0;
}

enum class Kind { Heap, Device, Host };

Kind classify(const State &s, const void *p)
{
    if (in_heap(s, p)) return Kind::Heap;
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) == hipSuccess) {
        if (attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged) return Kind::Device;
        return Kind::Host;
    }
    (void) hipGetLastError();
    return Kind::Host;
}

// Fan-in operands whose addresses differ mod 16 (no common vector body): with 1 or 2 sources and
// every operand element-aligned, the realigned kernel (kernels_impl.h fanin_realign_kernel) runs
// the body at full vector width; otherwise the element-granular path.  Every PE computes the same
// plan for the same addresses, and the fan-in never touches peers, so nothing is paired.
constexpr size_t kRealignMinBytes = 1024;

void plan_fanin(FaninArgs &f, Plan &pl, const void *dst, const void *const *srcs, int nsrc, size_t n, size_t es)
{
    pl = make_plan(dst, srcs, nsrc, n, es, 1, 0, kFaninMaxGrid);
    f.head = pl.head;
    f.nitems = pl.nitems;
    f.tail = pl.tail;
    f.realign = 0;
    const uintptr_t d = (uintptr_t) dst;
    bool ok = !pl.vec && nsrc >= 1 && nsrc <= 2 && n * es >= kRealignMinBytes && d % es == 0;
    for (int j = 0; ok && j < nsrc; ++j) ok = (uintptr_t) srcs[j] % es == 0;
    if (!ok) return;
    const uint64_t h = std::min<uint64_t>(n, ((kRealignPeel - d % kRealignPeel) % kRealignPeel) / es);
    f.head = h;
    f.nitems = (n - h) * es / 16;
    f.tail = n - h - f.nitems * (16 / es);
    for (int j = 0; j < nsrc; ++j) f.shift[j] = (uint32_t) (((uintptr_t) srcs[j] + h * es) % 16);
    f.total = n * es;
    f.realign = 1;
    pl.grid = (int) std::max<uint64_t>(1, std::min<uint64_t>((f.nitems + kRealignBlock - 1) / kRealignBlock,
                                                             (uint64_t) kRealignMaxGrid));
}

int launch_copy(void *dst, const void *src, size_t bytes, hipStream_t st)
{
    if (bytes == 0 || dst == src) return 0;
    FaninArgs f{};
    f.src[0] = (const char *) src;
    f.dst = (char *) dst;
    f.nsrc = 1;
    const void *srcs[1] = {src};
    Plan pl;
    plan_fanin(f, pl, dst, srcs, 1, bytes, 1);
    HIP_TRY(launch_fanin(ISHMEMI_OP_OR, ISHMEMI_DT_UINT8, pl.vec, f, pl.grid, st));
    return 0;
}

// ---------------- path thresholds (round 6: per team, by topology) ---------------------------
// Two thresholds pick a multi-PE reduce's path below the phased one (phased_min):
//   ll    - payloads up to it take the granule path (ll_kernel: one push of {data, epoch} granules
//           into every peer's ring, no barriers; 2 link bytes per payload byte, the granules
//           carry 4 B of payload in 8);
//   fold  - disjoint payloads up to it, on teams of 2 .. direct_max_pes members, take the
//           whole-array fold between two barriers (every member pulls every peer's whole source:
//           B per link) instead of reduce-scatter + all-gather (2B / p per link).
// Co-located teams (every member on one GPU: tests, rehearsals) keep round 5's measured
// crossovers: ll = min(ll_max_bytes, ring capacity), and 768 KiB / p for
// 3-4-member teams, where the fold's flat ~9-10 us beat the granules; fold = oneshot_p2 at 2
// members, oneshot_p2 / 4 / (p - 1) at 3-4 (each member reads (p - 1) B).  Those were measured
// where link bytes are free (all PEs on one HBM), so teams whose members sit on different GPUs
// (one PE per GPU over xGMI) take them from a link-byte model instead:
//   t_ll(B)   = a_ll(p)   + 1 hop  + 2B / L
//   t_fold(B) = a_fold(p) + 2 hops + B / L        (two barriers)
//   t_rsag(B) = a_rsag(p) + 3 hops + 2B / (p L)   (start / segment / done handshakes)
// L = xgmi_link_bps per link and direction (76.8 GB/s: the brief's 153.6 GB/s per link read as
// both directions together), a hop = one fabric round trip (kHopUs, assumed: never measured
// between GPUs here), a_*(p) = the fixed costs measured with one-PE-per-GPU launch shapes on one
// GPU in round 5 (the granule path 4.1-4.6 us at 2 PEs, 5.5-6.3 at 4; the fold 9.5 / 10.0-10.6 /
// 11.3-12.5 us at 2 / 3 / 4; the persistent kernel 9.6-10.2 / 13.8-14.1 / 16-17).
// Each threshold is the crossover of two lines, so it is closed-form.  ISHMEM_XGMI_LL_MAX_BYTES /
// ISHMEM_XGMI_FOLD_MAX_BYTES (or set_param "xgmi_ll_max_bytes" / "xgmi_fold_max_bytes") replace
// the model's values, e.g. with the crossovers the node run's `recommended` block measured.
constexpr double kHopUs = 1.0;
constexpr long long kUnlimited = std::numeric_limits<long long>::max();
struct Line {
    double a_us, b_us_per_byte;
};
Line model_ll(int p, double L) { return {4.5 + 0.5 * (p - 2) + 1 * kHopUs, 2e6 / L}; }
Line model_fold(int p, double L) { return {9.0 + 0.75 * (p - 2) + 2 * kHopUs, 1e6 / L}; }
Line model_rsag(int p, double L) { return {9.5 + 2.5 * (p - 2) + 3 * kHopUs, 2e6 / (p * L)}; }

// Largest payload for which line f is not slower than line g (f steeper or equal), or kUnlimited.
long long crossover(const Line &f, const Line &g)
{
    if (f.a_us > g.a_us) return 0;
    if (f.b_us_per_byte <= g.b_us_per_byte) return kUnlimited;
    return (long long) ((g.a_us - f.a_us) / (f.b_us_per_byte - g.b_us_per_byte));
}

// ll, fold: as above (fold 0 when the team does not take the fold: direct_p2 off, or more than
// direct_max_pes members); oneshot: the same bound ungated, for the persistent kernel's two-member
// one-shot mode (direct_p2 0, or operands without a common 16-B body).
struct PathLimits {
    long long ll, fold, oneshot;
};

PathLimits path_limits(const State &s, int p, bool colocated)
{
    PathLimits r{0, 0, 0};
    if (p < 2) return r;
    const long long cap = std::min<long long>(std::max<long long>(s.ll_max_bytes, 0), (long long) ll_capacity(p));
    const bool fold_team = s.direct_p2 && p <= s.direct_max_pes;
    if (colocated) {
        r.ll = cap;
        if (p >= 3 && fold_team) r.ll = std::min<long long>(r.ll, (768ll << 10) / p);
        r.fold = p == 2 ? s.oneshot_p2 : s.oneshot_p2 / 4 / (p - 1);
    } else {
        const double L = s.xgmi_link_bps;
        long long ll = crossover(model_ll(p, L), model_rsag(p, L));
        if (fold_team) ll = std::min(ll, crossover(model_ll(p, L), model_fold(p, L)));
        if (s.xgmi_ll_max >= 0) ll = s.xgmi_ll_max;
        r.ll = std::min(cap, ll);
        r.fold = s.xgmi_fold_max >= 0 ? s.xgmi_fold_max : crossover(model_fold(p, L), model_rsag(p, L));
    }
    r.oneshot = r.fold;
    if (!fold_team) r.fold = 0;
    return r;
}

PathLimits team_limits(const State &s, const Team &t) { return path_limits(s, t.size, t.colocated); }

// Small payloads (<= the team's ll threshold; device memory anywhere, any element-aligned address
// — the kernel picks 8-, 4- or 1-byte accesses, ll_load / ll_store): one-hop push of {data, epoch}
// granules into the peers' rings, no barriers (ll_kernel).  The choice depends on the byte count
// and the team only, which every member shares.
bool ll_eligible(const State &s, const Team &t, const void *dst, const void *src, size_t bytes)
{
    (void) dst;
    (void) src;
    return t.size > 1 && bytes > 0 && (long long) bytes <= team_limits(s, t).ll;
}

// Collectives of one PE run in the order they were called, whatever streams they were enqueued
// on (the flag protocol pairs the k-th collective of a team on every PE; the staging region is
// shared).  Same stream as last time: nothing to do.
// Cross-stream ordering (ISHMEM_STREAM_ORDER=1 / set_param "stream_order"): every collective
// records one device-scope event after its launches (mark_stream) and a collective enqueued on
// another stream than the previous one first waits on it (order_stream).  The event is the
// library's, so the earlier stream may since have been destroyed.  Off by default: like the
// reference (collectives of a team are not concurrency-safe, src/teams.h:29-38), the caller
// orders collectives it issues on different streams; the per-call event costs ~2 us of device
// time per collective.  The staging region is always protected (staging_ev).
bool capturing(hipStream_t st)
{
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess) {
        (void) hipGetLastError();
        return false;
    }
    return cs != hipStreamCaptureStatusNone;
}

// Blocking calls wait for their stream here.  block_spin (default 2): a stream write of the next
// sequence number into the host-mapped completion word follows the call's launches — stream
// ordered, so it lands after their kernels completed — and the host spins on it (bounded: after
// 20 ms it falls back to hipStreamSynchronize); mode 1 adds hipStreamSynchronize after the spin,
// mode 0 is hipStreamSynchronize alone.  2 PEs, one-PE-per-GPU launch shapes: a blocking 8 B reduce
// 12.7-13.5 us against 17.3-17.9 (mode 1: 23.4-24.1), a blocking fcollect 25.5-28.7 against
// 35.5-36.1 (profiles/r05/blocking/).  Device timeouts still surface through the host-mapped error
// words (check_team_errors); HIP's own asynchronous errors at the next synchronising HIP call.
int host_wait(State &s, hipStream_t st)
{
    if (s.block_spin && s.done_dev && !capturing(st)) {
        const uint32_t seq = ++s.done_seq;
        if (hipStreamWriteValue32(st, s.done_dev, seq, 0) == hipSuccess) {
            const auto t0 = std::chrono::steady_clock::now();
            int spins = 0;
            while (__atomic_load_n(s.done_host, __ATOMIC_ACQUIRE) != seq) {
                __builtin_ia32_pause();
                if (++spins == 4096) {
                    spins = 0;
                    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) break;
                }
            }
            if (s.block_spin == 2 && __atomic_load_n(s.done_host, __ATOMIC_ACQUIRE) == seq) return 0;
        } else {
            (void) hipGetLastError();
        }
    }
    HIP_TRY(hipStreamSynchronize(st));
    return 0;
}

// Team barrier on `st`, stream ordered (everything before it on the stream has completed on this
// PE, and on every member, when the stream passes it): team_sync_kernel, one workgroup polling
// the flag row (kPhaseSync, 0) with a bounded spin (*ret on timeout).  Round 5 also had a barrier
// of stream memory operations (ISHMEM_BARRIER_KIND=stream: hipStreamWriteValue32 into the peers'
// rows, hipStreamWaitValue32 on its own); it lost every measurement (2 PEs 20.7 vs 9.3 us per
// phased call, 8 co-located PEs 651-687 vs 130-175 us, two-stream probe 9.6 vs 5.7 us per
// barrier), had no timeout, and had to fall back to this kernel under stream capture — a path
// choice one PE could make differently from its peers — so round 6 removed it.
int team_barrier(State &s, int team, const ReduceArgs &a, hipStream_t st)
{
    (void) s;
    (void) team;
    HIP_TRY(launch_team_sync(a, st));
    return 0;
}


// Work captured into a hipGraph runs when the graph is launched: ordering it against other
// collectives is the caller's (launch order), so captured calls neither wait nor mark.
int order_stream(State &s, hipStream_t st)
{
    if (!s.stream_order) return 0;
    if (s.last_stream_set && s.last_stream != st && !capturing(st))
        HIP_TRY(hipStreamWaitEvent(st, s.order_ev, 0));
    return 0;
}

int mark_stream(State &s, hipStream_t st)
{
    if (!s.stream_order || capturing(st)) return 0;
    if (!s.order_ev)
        HIP_TRY(hipEventCreateWithFlags(&s.order_ev, hipEventDisableTiming | hipEventDisableSystemFence));
    HIP_TRY(hipEventRecord(s.order_ev, st));
    s.last_stream = st;
    s.last_stream_set = true;
    return 0;
}

int staging_acquire(State &s, hipStream_t st)
{
    if (s.staging_used && !capturing(st)) HIP_TRY(hipStreamWaitEvent(st, s.staging_ev, 0));
    return 0;
}

int staging_release(State &s, hipStream_t st)
{
    if (capturing(st)) return 0;
    if (!s.staging_ev) HIP_TRY(hipEventCreateWithFlags(&s.staging_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(s.staging_ev, st));
    s.staging_used = true;
    return 0;
}

// mode: kernels.h kLLReduce / kLLInscan / kLLExscan / kLLCollect (what the received items become).
int reduce_ll(State &s, int team, int op, int dt, void *dst, const void *src, size_t bytes, int *ret,
              hipStream_t st, int mode = kLLReduce, int root = 0)
{
    if (order_stream(s, st)) return 1;
    Team &t = s.teams[team];
    LLArgs a;
    memset(&a, 0, sizeof(a));
    a.src = (const char *) src;
    a.dst = (char *) dst;
    a.my_ring = s.tmem[team].ring[s.pe];
    for (int j = 0; j < t.size; ++j) {
        const int gpe = t.start + j * t.stride;
        a.peer_ring[j] = s.tmem[team].ring[gpe];
        if (!a.peer_ring[j]) return fail("reduce: PE " + std::to_string(gpe) + " ring not mapped");
    }
    a.err = s.err_dev + team;
    a.ret = ret;
    a.nbytes = bytes;
    a.timeout_ticks = (uint64_t) s.timeout_ms * 100000ull;
    a.ep_ctr = s.kern_ep + (size_t) kEpTeamWords * team;
    a.p = t.size;
    a.me = t.my_idx;
    a.mode = mode;
    a.root = root;
    HIP_TRY(launch_ll(op, dt, a, st));
    return 0;
}

// Device-resident collective on symmetric-heap buffers: one allreduce_kernel launch.
int reduce_heap(State &s, int team, int op, int dt, void *dst, const void *src, size_t n, int *ret,
                hipStream_t st)
{
    if (order_stream(s, st)) return 1;
    Team &t = s.teams[team];
    const size_t es = dtype_size(dt);
    ReduceArgs a;
    std::string why;
    if (team_args(s, team, a, why)) return fail("reduce: " + why);
    for (int j = 0; j < t.size; ++j) {
        const int gpe = t.start + j * t.stride;
        a.src[j] = translate(s, src, gpe);
        a.dstp[j] = translate(s, dst, gpe);
        if (!a.src[j] || !a.dstp[j])
            return fail("reduce: buffer not mapped for PE " + std::to_string(gpe));
    }
    a.dst = (char *) dst;
    a.ret = ret;
    a.trace = s.trace;
    const void *srcs[1] = {src};
    Plan pl = make_plan(dst, srcs, 1, n, es, t.size, s.max_blocks, 0);
    a.head = pl.head;
    a.nitems = pl.nitems;
    a.tail = pl.tail;
    a.items_per_chunk = pl.items_per_chunk;
    a.seg_items = pl.seg_items;
    // Every choice below depends only on symmetric-address properties, the byte count, the team
    // size and parameters agreed at init, so every member makes the same one.
    const uintptr_t d0 = (uintptr_t) dst, s0 = (uintptr_t) src, nb = n * es;
    // Source and dest on different 16-B phases (same on every PE: the offsets are symmetric): the
    // phased / whole-array grids keep dest's 16-B items and read the sources with unaligned loads
    // (PhaseArgs::shift; phase_unaligned 0: the realigning kernel), the persistent kernel likewise
    // below (ar_shifted), instead of an element-granular path.
    const bool realign = !pl.vec && d0 % es == 0 && s0 % es == 0 && nb >= kRealignMinBytes;
    if (realign && (long long) nb < s.phased_min && s.ar_shifted) {
        // Below phased_min: the persistent kernel's vector instantiation with items laid out by
        // dest's phase; every source is read at dest's item offsets with unaligned 16-B loads (the
        // hardware splits a load that crosses a line: tools/realign_variants.hip "unaligned buf",
        // 0.78 of HBM at 1 GiB against 0.84 aligned, profiles/r05/realign/).  The all-gather
        // reads peers' dests, on dest's phase on every PE (symmetric offsets), so it stays aligned.
        const void *dsts[1] = {dst};
        pl = make_plan(dst, dsts, 1, n, es, t.size, s.max_blocks, 0);
        a.head = pl.head;
        a.nitems = pl.nitems;
        a.tail = pl.tail;
        a.items_per_chunk = pl.items_per_chunk;
        a.seg_items = pl.seg_items;
    }
    const bool disjoint = d0 + nb <= s0 || s0 + nb <= d0;
    // Two members, disjoint buffers, up to the team's fold bound, 16-B body (or shifted sources):
    // barrier, ONE one-shot grid in which each member folds the whole array from both sources,
    // barrier (round 5, PhaseArgs::whole) — the phased path's shape without the all-gather and its
    // barrier.  Over one link it moves the same B per direction as reduce-scatter + all-gather.
    // Three or four members (round 5): the same whole-array fold.  On one GPU it beat the
    // persistent / phased paths up to 8 MiB at 3 PEs and 4 MiB at 4 (1 / 2 MiB at 4 PEs: 11.3-12.5 /
    // 11.5-12.6 us against 17.9-18.5 / 25.3-25.4); each member pulls (p - 1) * B over the links
    // where reduce-scatter + all-gather pulls 2(p - 1) / p * B, hence the tighter bound for teams
    // across GPUs (path_limits).
    const PathLimits lim = team_limits(s, t);
    const bool fold_size = lim.fold > 0 && (long long) nb <= lim.fold;
    // In place (source == dest): the same fold into the team's private scratch on this device
    // (dest's 16-B phase; peers never read it, so it is plain device memory, allocated with the
    // team: no allocation on the call path, the same path captured or not), the end barrier (every
    // member has read every source), then a local copy into dest.  The staging region with its
    // events was tried first and lost to the persistent kernel (profiles/r05/direct_p2/r05zzp_*);
    // set_param "direct_inplace" 0 turns this off.
    char *scratch = nullptr;
    // Only while p * B <= 4 MiB: the copy back costs 2B of HBM and a launch, and the fold's gain
    // over the persistent kernel is gone by 2 MiB at 2 PEs and 1 MiB at 4 (2 PEs 1 MiB 12.8-13.4
    // vs 14.9-15.4 us, 4 MiB 20.6-22.4 vs 18.6-19.5; 4 PEs 512 KiB 14.2-14.7 vs 19.7-21.3;
    // profiles/r05/direct_p2/r05zzs_ab_inplace_scratch.txt).
    if (fold_size && d0 == s0 && pl.vec && s.direct_inplace && (uint64_t) t.size * nb <= kInplaceFoldBytes) {
        const TeamMem &m = s.tmem[team];
        if (!m.fold_scratch || m.fold_scratch_bytes < nb + 16)  // sized for p * B <= 4 MiB at creation
            return fail("reduce: the team's in-place fold scratch is missing");
        scratch = m.fold_scratch + (d0 & 15);
    }
    const bool inplace_fold = scratch != nullptr;
    const bool direct = (fold_size && disjoint && (pl.vec || realign)) || inplace_fold;
    if ((pl.vec || realign) && (direct || (long long) nb >= s.phased_min)) {
        // From phased_min bytes: barrier, one-shot reduce-scatter, barrier, one-shot all-gather,
        // barrier (kernels_impl.h, "Phased reduce-scatter + all-gather").  The barriers carry *ret.
        PhaseArgs ph;
        memset(&ph, 0, sizeof(ph));
        for (int j = 0; j < t.size; ++j) {
            ph.src[j] = a.src[j];
            ph.dstp[j] = a.dstp[j];
        }
        ph.dst = a.dst;
        ph.head = pl.head;
        ph.nitems = pl.nitems;
        ph.tail = pl.tail;
        ph.items_per_chunk = pl.items_per_chunk;
        ph.elem = (uint32_t) es;
        ph.p = t.size;
        ph.me = t.my_idx;
        ph.peer_nt = s.phased_peer_nt;
        ph.whole = direct ? 1 : 0;
        // XCD-grouped block order for shifted sources: only when this PE has its GPU to itself.  The
        // order assumes workgroup b runs on XCD b mod 8, which holds for a kernel running alone (1 GiB
        // a + b from sources 4 / 12 B off: 0.75 -> 0.83 of HBM, one process); with co-located PEs'
        // grids dispatched together it does not (2 / 4 PEs x 1 GiB, sources 4 B off: reduce-scatter
        // grid 0.524-0.537 ms either way, profiles/r06/realign/r06c_ab.txt).  Block order only: no
        // member pairs with another's blocks, so PEs may differ.
        ph.xcd_group = s.rs_xcd && device_share() == 1 ? 1 : 0;
        if (inplace_fold) ph.dst = scratch;
        if (realign) {
            const uint64_t h = std::min<uint64_t>(n, ((16 - d0 % 16) % 16) / es);
            ph.head = h;
            ph.nitems = (n - h) * es / 16;
            ph.tail = n - h - ph.nitems * (16 / es);
            ph.items_per_chunk = items_per_chunk(ph.nitems, t.size);
            ph.shift = (uint32_t) ((s0 + h * es) % 16);
            ph.total = nb;
        }
        const bool ev = s.phase_events && !capturing(st);
        auto mark = [&](int k) -> int {
            if (ev) HIP_TRY(hipEventRecord(s.phase_ev[k], st));
            return 0;
        };
        if (mark(0)) return 1;
        if (team_barrier(s, team, a, st)) return 1;
        if (mark(1)) return 1;
        HIP_TRY(launch_rs_phase(op, dt, ph, st));
        if (mark(2)) return 1;
        if (!direct) {
            if (team_barrier(s, team, a, st)) return 1;
            if (mark(3)) return 1;
            HIP_TRY(launch_ag_phase(ph, st));
        } else if (mark(3)) {
            return 1;
        }
        if (mark(4)) return 1;
        if (team_barrier(s, team, a, st)) return 1;
        if (mark(5)) return 1;
        if (inplace_fold && launch_copy(dst, scratch, nb, st)) return 1;
        s.phase_recorded = s.phase_recorded || ev;
        return 0;
    }
    if (t.size == 2 && (long long) nb <= lim.oneshot && disjoint) {
        a.oneshot = 1;
        a.items_per_chunk = pl.nitems;
        a.seg_items = seg_items(pl.nitems);
        pl.grid = (int) std::max<uint64_t>(
            1, std::min<uint64_t>(nsegs(pl.nitems, a.seg_items), (uint64_t) s.max_blocks));
    }
    HIP_TRY(launch_allreduce(op, dt, pl.vec, a, pl.grid, st));
    return 0;
}

// Pageable host memory (plain malloc) as a staged buffer: the DMA engines read and write only
// page-locked memory, so HIP copies pageable bytes synchronously through its own bounce buffers,
// one direction at a time (measured, 1 GiB f32 at 1 PE: 25.8 GiB/s against 40.4 pinned).  For
// the call the buffer is page-locked in place (hipHostRegister: ~2 ms per GiB measured, unlocked
// at the end), so both directions stream asynchronously at once, like pinned buffers.  Small
// buffers, and ranges HIP refuses (e.g. already registered), keep the synchronous copies.
constexpr size_t kPinMinBytes = (size_t) 1 << 20;

bool pageable_host(const void *p)
{
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void) hipGetLastError();
        return true;
    }
    return attr.type == hipMemoryTypeUnregistered || (attr.type == hipMemoryTypeHost && attr.devicePointer == nullptr);
}

struct CallPins {
    void *pinned[2] = {nullptr, nullptr};
    void pin(void *p, size_t bytes)
    {
        if (!p || bytes < kPinMinBytes || !pageable_host(p)) return;
        for (void *q : pinned)
            if (q == p) return;  // in place: one registration
        const hipError_t e = hipHostRegister(p, bytes, hipHostRegisterDefault);
        if (e != hipSuccess) {
            (void) hipGetLastError();
            if (debug_level() > 0)
                fprintf(stderr, "[ishmem_amd] hipHostRegister(%p, %zu): %s (synchronous copies)\n", p, bytes,
                        hipGetErrorString(e));
            return;
        }
        if (debug_level() > 1)
            fprintf(stderr, "[ishmem_amd] page-locked %p, %zu bytes for the call\n", p, bytes);
        (pinned[0] ? pinned[1] : pinned[0]) = p;
    }
    bool any() const { return pinned[0] || pinned[1]; }
    // After the call's last copy has completed (the caller synchronises first).
    void release()
    {
        for (void *&q : pinned)
            if (q) {
                (void) hipHostUnregister(q);
                q = nullptr;
            }
    }
};

// Non-symmetric buffers (host memory, or device memory outside the heap): a 3-stage pipeline
// through two halves of the symmetric staging region.  Chunk k: copy-in on the `in` stream,
// in-place collective on the caller's stream, copy-out on the `out` stream; chunk k+1's copy-in
// and chunk k-1's copy-out overlap chunk k's collective (PCIe is full duplex).  Replaces the
// synchronous 64 KiB bounce loop ishmemi_generic_op_reduce (src/collectives/reduce_impl.h:186-228).
int reduce_staged_pipeline(State &s, int team, int op, int dt, void *dst, const void *src, size_t n,
                           int *ret, hipStream_t st);

// The pipeline, with pageable host buffers page-locked for the call.  A call that pinned a buffer
// completes before it returns (the buffers are unlocked after their last copy), which a pageable
// buffer's synchronous copies would have made it do anyway.
int reduce_staged(State &s, int team, int op, int dt, void *dst, const void *src, size_t n, int *ret,
                  hipStream_t st)
{
    const size_t bytes = n * dtype_size(dt);
    CallPins pins;
    // Not while the stream is being captured into a hipGraph: the synchronize below would
    // invalidate the capture, and the buffers would be unlocked again before any replay.  The
    // captured copies then stay HIP's own pageable copies.
    if (!capturing(st)) {
        pins.pin(const_cast<void *>(src), bytes);
        pins.pin(dst, bytes);
    }
    int rc = reduce_staged_pipeline(s, team, op, dt, dst, src, n, ret, st);
    if (pins.any()) {
        // Every copy of the call has completed (also after a failure part-way) before unlocking.
        bool ok = hipStreamSynchronize(st) == hipSuccess;
        if (s.copy_in) ok = hipStreamSynchronize(s.copy_in) == hipSuccess && ok;
        if (s.copy_out) ok = hipStreamSynchronize(s.copy_out) == hipSuccess && ok;
        if (!ok && !rc) rc = fail("reduce: stream synchronize failed");
        pins.release();
    }
    return rc;
}

// Device address of host memory the GPU can load / store directly (hipHostMalloc'd, or registered
// by the caller or by CallPins), else null.
char *host_device_view(const void *p)
{
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void) hipGetLastError();
        return nullptr;
    }
    return attr.type == hipMemoryTypeHost ? (char *) attr.devicePointer : nullptr;
}

int reduce_staged_pipeline(State &s, int team, int op, int dt, void *dst, const void *src, size_t n,
                           int *ret, hipStream_t st)
{
    const size_t es = dtype_size(dt);
    const char *src_dev = (s.staged_copy_kernel & 2) ? host_device_view(src) : nullptr;
    char *dst_dev = (s.staged_copy_kernel & 1) ? host_device_view(dst) : nullptr;
    const int nslots = s.staging_slots;
    const size_t slot_bytes = (s.staging_bytes / (size_t) nslots) & ~(kHeapAlign - 1);
    const size_t chunk = (slot_bytes / es) & ~size_t(63);
    if (chunk == 0) return fail("reduce: staging region too small");
    if (order_stream(s, st)) return 1;
    if (!s.copy_in) {
        HIP_TRY(hipStreamCreateWithFlags(&s.copy_in, hipStreamNonBlocking));
        HIP_TRY(hipStreamCreateWithFlags(&s.copy_out, hipStreamNonBlocking));
        for (int i = 0; i < kMaxStagingSlots; ++i) {
            HIP_TRY(hipEventCreateWithFlags(&s.ev_in[i], hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&s.ev_red[i], hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&s.ev_out[i], hipEventDisableTiming));
        }
    }
    if (staging_acquire(s, st)) return 1;
    HIP_TRY(hipEventRecord(s.ev_red[0], st));  // copy-ins start after the caller's prior work
    HIP_TRY(hipStreamWaitEvent(s.copy_in, s.ev_red[0], 0));
    bool used[kMaxStagingSlots] = {};
    for (size_t off = 0, k = 0; off < n; off += chunk, ++k) {
        const int sl = (int) (k % (size_t) nslots);
        char *buf = s.staging + (size_t) sl * slot_bytes;
        const size_t m = std::min(chunk, n - off);
        if (used[sl]) HIP_TRY(hipStreamWaitEvent(s.copy_in, s.ev_out[sl], 0));  // slot drained
        if (src_dev) {
            if (launch_copy(buf, src_dev + off * es, m * es, s.copy_in)) return 1;
        } else {
            HIP_TRY(hipMemcpyAsync(buf, (const char *) src + off * es, m * es, hipMemcpyDefault, s.copy_in));
        }
        HIP_TRY(hipEventRecord(s.ev_in[sl], s.copy_in));
        HIP_TRY(hipStreamWaitEvent(st, s.ev_in[sl], 0));
        // One PE: the in-place reduce of the staged chunk is the identity (reduce_impl.h:288-289).
        if (s.teams[team].size > 1) {
            const bool ll = ll_eligible(s, s.teams[team], buf, buf, m * es);
            if (ll ? reduce_ll(s, team, op, dt, buf, buf, m * es, ret, st)
                   : reduce_heap(s, team, op, dt, buf, buf, m, ret, st))
                return 1;
        }
        HIP_TRY(hipEventRecord(s.ev_red[sl], st));
        HIP_TRY(hipStreamWaitEvent(s.copy_out, s.ev_red[sl], 0));
        if (dst_dev) {
            if (launch_copy(dst_dev + off * es, buf, m * es, s.copy_out)) return 1;
        } else {
            HIP_TRY(hipMemcpyAsync((char *) dst + off * es, buf, m * es, hipMemcpyDefault, s.copy_out));
        }
        HIP_TRY(hipEventRecord(s.ev_out[sl], s.copy_out));
        used[sl] = true;
    }
    for (int sl = 0; sl < nslots; ++sl)  // the caller's stream completes only after every copy-out
        if (used[sl]) HIP_TRY(hipStreamWaitEvent(st, s.ev_out[sl], 0));
    return staging_release(s, st);
}

// ---------------- fcollect / collect / scan --------------------------
int team_sync_locked(State &s, int team, hipStream_t st, int *ret);

template <typename A>
int fill_team_sync_args(State &s, int team, A &a, std::string &why)
{
    ReduceArgs r;
    if (team_args(s, team, r, why)) return 1;
    a.my_flags = r.my_flags;
    for (int j = 0; j < r.p; ++j) a.peer_flags[j] = r.peer_flags[j];
    a.err = r.err;
    a.timeout_ticks = r.timeout_ticks;
    a.ep_ctr = r.ep_ctr;
    a.p = r.p;
    a.me = r.me;
    return 0;
}

// nbytes[j] = bytes member j contributes; dest slot of j starts at the sum of the earlier ones.
int collect_launch(State &s, int team, void *dst, const void *src, const uint64_t *nbytes, int *ret,
                   hipStream_t st, const uint64_t *dst_off = nullptr, const char *const *srcs = nullptr)
{
    Team &t = s.teams[team];
    if (order_stream(s, st)) return 1;
    CollectArgs a;
    memset(&a, 0, sizeof(a));
    std::string why;
    if (fill_team_sync_args(s, team, a, why)) return fail("collect: " + why);
    uint64_t off = 0, orv = (uintptr_t) src | (uintptr_t) dst, maxb = 0;
    for (int j = 0; j < t.size; ++j) {
        const int gpe = t.start + j * t.stride;
        a.src[j] = srcs ? srcs[j] : translate(s, src, gpe);
        if (!a.src[j]) return fail("collect: source must be symmetric-heap memory");
        a.dst_off[j] = dst_off ? dst_off[j] : off;
        a.nbytes[j] = nbytes[j];
        orv |= a.dst_off[j] | nbytes[j] | (uintptr_t) a.src[j];
        off += nbytes[j];
        maxb = std::max(maxb, nbytes[j]);
    }
    a.dst = (char *) dst;
    a.ret = ret;
    a.unit = (orv & 15) == 0 ? 16 : (orv & 3) == 0 ? 4 : 1;
    if (t.size > 1 && (long long) off >= s.phased_min) {
        // Large: barrier, one-shot pull grid, barrier (kernels_coll.hip collect_phase_kernel).
        // Decided on the total bytes only, which every member knows, so all take the same path.
        ReduceArgs r;
        if (team_args(s, team, r, why)) return fail("collect: " + why);
        r.ret = ret;
        if (team_barrier(s, team, r, st)) return 1;
        HIP_TRY(launch_collect_phase(a, st));
        if (team_barrier(s, team, r, st)) return 1;
        return 0;
    }
    const uint64_t items = maxb / a.unit, tile = (uint64_t) kBlock * kUnroll;
    const int grid = (int) std::max<uint64_t>(1, std::min<uint64_t>((items + tile - 1) / tile, s.max_blocks));
    HIP_TRY(launch_collect(a, grid, st));
    return 0;
}

// Memory a kernel of this device may write: the heap, device memory, pinned host memory.
bool device_writable(const State &s, const void *p)
{
    if (in_heap(s, p)) return true;
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void) hipGetLastError();
        return false;  // pageable host memory
    }
    return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged ||
           (attr.type == hipMemoryTypeHost && attr.devicePointer != nullptr);
}

// fcollect / collect with a source outside the heap (host or plain device memory, which peers
// cannot map): like the reference's intra-node collect, which copies from any local source
// (src/collectives/collect_impl.h:93-114), the bytes go through the symmetric staging region,
// segment by segment — copy this member's part of segment k in, then the pull collect of segment k
// from every member's staging region.  A member's next copy follows its kernel, which returns only
// after every peer has finished reading its staging region ("done reading").
int collect_staged(State &s, int team, char *dst, const char *src, const uint64_t *nbytes, int *ret,
                   hipStream_t st)
{
    const Team &t = s.teams[team];
    const uint64_t S = (uint64_t) s.staging_bytes & ~(uint64_t) 15;
    uint64_t maxb = 0, off[kMaxPes], acc = 0;
    for (int j = 0; j < t.size; ++j) {
        off[j] = acc;
        acc += nbytes[j];
        maxb = std::max<uint64_t>(maxb, nbytes[j]);
    }
    const uint64_t nseg = std::max<uint64_t>(1, (maxb + S - 1) / S);
    if (staging_acquire(s, st)) return 1;
    for (uint64_t k = 0; k < nseg; ++k) {
        uint64_t segb[kMaxPes], segoff[kMaxPes];
        for (int j = 0; j < t.size; ++j) {
            const uint64_t lo = std::min<uint64_t>(nbytes[j], k * S);
            segb[j] = std::min<uint64_t>(S, nbytes[j] - lo);
            segoff[j] = off[j] + lo;
        }
        const uint64_t mine = segb[t.my_idx];
        if (mine) HIP_TRY(hipMemcpyAsync(s.staging, src + k * S, mine, hipMemcpyDefault, st));
        if (collect_launch(s, team, dst, s.staging, segb, ret, st, segoff)) return 1;
    }
    return staging_release(s, st);
}

// Stream-ordered collect: the members' counts meet on the device (collect_dyn_kernel), so nothing
// here waits for the host to learn them.  Count slots: one 64-B line per team (s.count_slots).
int collect_on_stream_impl(int team, void *dst, const void *src, size_t nbytes, int *ret, hipStream_t st)
{
    State &s = S();
    std::lock_guard<std::mutex> lk(s.mu);
    if (!s.initialized) return fail("collect: not initialized");
    if (team < 0 || team >= kMaxTeams || !s.teams[team].valid || s.teams[team].my_idx < 0)
        return fail("collect: invalid team or caller not a member");
    Team &t = s.teams[team];
    if (ret) HIP_TRY(hipMemsetAsync(ret, 0, sizeof(int), st));
    if (t.size == 1) {
        if (nbytes && dst != src && launch_copy(dst, src, nbytes, st)) return 1;
        return mark_stream(s, st);
    }
    if (!in_heap(s, dst)) return fail("collect: dest must be symmetric-heap memory");
    // Peers' sources are found at the offset of this PE's (symmetric) source, so it must be in
    // the heap even when this PE contributes nothing.
    if (!in_heap(s, src)) return fail("collect: source must be symmetric-heap memory");
    if (order_stream(s, st)) return 1;
    CollectArgs a;
    memset(&a, 0, sizeof(a));
    std::string why;
    if (fill_team_sync_args(s, team, a, why)) return fail("collect: " + why);
    char *slot = s.count_slots + (size_t) team * 64;
    for (int j = 0; j < t.size; ++j) {
        const int gpe = t.start + j * t.stride;
        a.src[j] = translate(s, src, gpe);
        a.count_at[j] = (const uint64_t *) translate(s, slot, gpe);
        if (!a.src[j] || !a.count_at[j]) return fail("collect: buffer not mapped for PE " + std::to_string(gpe));
    }
    a.dst = (char *) dst;
    a.ret = ret;
    a.my_count = nbytes;
    a.my_count_slot = (uint64_t *) slot;
    // Grid from this member's share (the others' are not known here): the kernel strides over
    // whatever every member contributes.
    const uint64_t tile = (uint64_t) kBlock * kUnroll * 16;
    const uint64_t g = ((uint64_t) t.size * nbytes + tile - 1) / tile;
    const int grid = (int) std::max<uint64_t>(8, std::min<uint64_t>(g, (uint64_t) s.max_blocks));
    HIP_TRY(launch_collect_dyn(a, grid, st));
    return mark_stream(s, st);
}

// staged: 1 / 0 = the members agreed (blocking calls exchange it first, see ishmemi_c_fcollect);
// -1 = this PE decides from its own source (stream-ordered calls: every member must then pass
// the same kind of source, as their launches must match).
int fcollect_impl(int team, void *dst, const void *src, size_t nbytes, int *ret, hipStream_t st,
                  bool blocking, int staged = -1)
{
    State &s = S();
    std::lock_guard<std::mutex> lk(s.mu);
    if (!s.initialized) return fail("fcollect: not initialized");
    if (team < 0 || team >= kMaxTeams || !s.teams[team].valid || s.teams[team].my_idx < 0)
        return fail("fcollect: invalid team or caller not a member");
    Team &t = s.teams[team];
    if (ret) HIP_TRY(hipMemsetAsync(ret, 0, sizeof(int), st));  // sticky: launches OR failures in
    if (t.size == 1) {
        if (nbytes && dst != src && launch_copy(dst, src, nbytes, st)) return 1;
    } else {
        if (!device_writable(s, dst)) return fail("fcollect: dest must be heap, device or pinned host memory");
        uint64_t nb[kMaxPes];
        for (int j = 0; j < t.size; ++j) nb[j] = nbytes;
        // A source outside the heap is staged (the staged call is several launches, so the members
        // must agree on it).  Zero bytes: only the team synchronises.
        if (staged < 0) staged = in_heap(s, src) ? 0 : 1;
        if (nbytes == 0) {
            if (team_sync_locked(s, team, st, ret)) return 1;
        } else if (!staged && ll_eligible(s, t, dst, src, nbytes) && 2 * nbytes <= ll_capacity(t.size)) {
            // Small payloads (round 5): the granule exchange, every member's bytes stored at their
            // team-order offset (kLLCollect) — no start / done handshakes.  Up to half the ring's
            // capacity: the pull kernel moves (p-1)·B where the granules move 2(p-1)·B, and at
            // 4 PEs x 256 KiB the two were already within 8 % (profiles/r05/ll_coll/).  The kernel
            // stores dest locally whatever its kind (heap, device, pinned host), so the choice
            // depends on the byte count and the team only: the same on every member (round 6; it
            // also required a non-host dest, which one member could pass alone — ADVICE r05).
            if (reduce_ll(s, team, ISHMEMI_OP_OR, ISHMEMI_DT_UINT8, dst, src, nbytes, ret, st, kLLCollect)) return 1;
        } else if (staged) {
            if (order_stream(s, st) || collect_staged(s, team, (char *) dst, (const char *) src, nb, ret, st)) return 1;
        } else if (collect_launch(s, team, dst, src, nb, ret, st)) {
            return 1;
        }
    }
    if (mark_stream(s, st)) return 1;
    if (blocking) {
        if (host_wait(s, st)) return 1;
        if (check_team_errors(s, team)) return 1;
    }
    return 0;
}

// One u64 per member, in team order, on every member (an 8-byte fcollect through the team
// scratch): blocking calls agree on their path and on local argument failures with it before
// anything that must match across members is launched (a member that failed alone would leave
// its peers waiting for launches that never come).  Called without the state lock.
constexpr uint64_t kAgreeStaged = 1ull << 62, kAgreeFail = 1ull << 63;
bool member_call(const State &s, int team);

// The agreement step of the blocking fcollect / collect / scan / broadcast (staged path, counts,
// argument failures): an allgather of one u64 per member, before anything else is launched.
// One small-message (LL) launch on a host-mapped coherent array: member i's word sits in slot i,
// zeros elsewhere, so a uint64 SUM over the team is the allgather, read by the host once the
// launch completes — no copy in or out.  Round 3 used a synchronous H2D copy, a whole fcollect
// launch (start and done handshakes) and a synchronous D2H copy (the exchange roughly
// doubled a small blocking fcollect / scan; BASELINE.md round 4 has the before / after).
int team_exchange(int team, uint64_t mine, uint64_t *all)
{
    State &s = S();
#ifdef ISHMEMI_EXCHANGE_VIA_FCOLLECT  // round-3 exchange (A/B builds only)
    const int p = s.teams[team].size;
    if (hipMemcpy(s.team_scratch, &mine, 8, hipMemcpyHostToDevice) != hipSuccess)
        return fail("team exchange: copy failed");
    if (fcollect_impl(team, s.team_scratch + 64, s.team_scratch, 8, nullptr, 0, true, 0)) return 1;
    if (hipMemcpy(all, s.team_scratch + 64, 8 * (size_t) p, hipMemcpyDeviceToHost) != hipSuccess)
        return fail("team exchange: copy failed");
    return 0;
#else
    std::lock_guard<std::mutex> lk(s.mu);
    if (!member_call(s, team)) return fail("team exchange: invalid team or caller not a member");
    const Team &t = s.teams[team];
    const int p = t.size;
    volatile uint64_t *src = s.exch_host, *dst = s.exch_host + kMaxPes;
    for (int j = 0; j < p; ++j) {
        src[j] = j == t.my_idx ? mine : 0;
        dst[j] = 0;
    }
    if (p > 1) {
        if (reduce_ll(s, team, ISHMEMI_OP_SUM, ISHMEMI_DT_UINT64, s.exch_dev + kMaxPes, s.exch_dev, 8 * (size_t) p,
                      nullptr, 0))
            return 1;
        if (mark_stream(s, 0)) return 1;
        if (host_wait(s, 0)) return 1;
        if (check_team_errors(s, team)) return 1;
    } else {
        dst[0] = mine;
    }
    for (int j = 0; j < p; ++j) all[j] = dst[j];
    return 0;
#endif
}

bool member_call(const State &s, int team)
{
    return s.initialized && team >= 0 && team < kMaxTeams && s.teams[team].valid && s.teams[team].my_idx >= 0;
}

int scan_impl(int team, int dt, int inclusive, void *dst, const void *src, size_t n, int *ret,
              hipStream_t st, bool blocking)
{
    State &s = S();
    std::lock_guard<std::mutex> lk(s.mu);
    if (!s.initialized) return fail("scan: not initialized");
    if (!op_dtype_valid(ISHMEMI_OP_SUM, dt)) return fail("scan: invalid dtype");
    if (team < 0 || team >= kMaxTeams || !s.teams[team].valid || s.teams[team].my_idx < 0)
        return fail("scan: invalid team or caller not a member");
    Team &t = s.teams[team];
    const size_t es = dtype_size(dt);
    if (ret) HIP_TRY(hipMemsetAsync(ret, 0, sizeof(int), st));  // sticky over the segments
    if (t.size == 1) {  // inclusive: the source; exclusive: the sum of nothing
        if (n && inclusive && dst != src && launch_copy(dst, src, n * es, st)) return 1;
        if (n && !inclusive) HIP_TRY(hipMemsetAsync(dst, 0, n * es, st));
    } else if (n == 0) {
        if (team_sync_locked(s, team, st, ret)) return 1;
    } else {
        if (!in_heap(s, dst) || !in_heap(s, src)) return fail("scan: buffers must be symmetric-heap memory");
        if (((uintptr_t) dst | (uintptr_t) src) % es) return fail("scan: misaligned buffers");
        if (ll_eligible(s, t, dst, src, n * es)) {
            // Small payloads (round 5): the granule exchange, each member folding members 0..me
            // (inclusive) or 0..me-1 (exclusive) — no scratch rows, no handshakes.
            if (reduce_ll(s, team, ISHMEMI_OP_SUM, dt, dst, src, n * es, ret, st, inclusive ? kLLInscan : kLLExscan))
                return 1;
            if (mark_stream(s, st)) return 1;
            if (blocking) {
                if (host_wait(s, st)) return 1;
                if (check_team_errors(s, team)) return 1;
            }
            return 0;
        }
        // Segments whose p scratch rows fit the staging region (member c's rows: [k][chunk c]).
        const uint64_t ipc_max = ((s.staging_bytes / es) / (uint64_t) t.size) & ~uint64_t(63);
        const uint64_t seg = ipc_max * (uint64_t) t.size;
        if (ipc_max == 0) return fail("scan: staging region too small for this team");
        const uintptr_t d0 = (uintptr_t) dst, s0 = (uintptr_t) src, nb = n * es;
        const bool disjoint = d0 + nb <= s0 || s0 + nb <= d0;
        if (disjoint && (t.size == 2 || (long long) nb <= team_limits(s, t).fold)) {
            // Two members, disjoint buffers: barrier, direct one-shot fold, barrier (no scratch;
            // kernels_coll.hip scan_direct_kernel).  Every member sees the same n and the same
            // symmetric offsets, so all take this path together.  At every size past the granule
            // path since round 5 (it was the phased threshold's): 1 / 2 MiB 8.9-9.3 / 9.0 us
            // against the scratch kernel's 17.8-18.1 / 19.7-20.8 (profiles/r05/scan/).  Three and
            // four members under the reduce's whole-array bound (path_limits; 0 with direct_p2
            // off, so an A/B of direct_p2 switches reduces and scans together — ADVICE r05).
            if (order_stream(s, st)) return 1;
            ScanArgs a;
            memset(&a, 0, sizeof(a));
            std::string why;
            if (fill_team_sync_args(s, team, a, why)) return fail("scan: " + why);
            for (int j = 0; j < t.size; ++j) a.src[j] = translate(s, src, t.start + j * t.stride);
            a.dst = (char *) dst;
            a.ret = ret;
            a.nelems = n;
            a.inclusive = inclusive;
            ReduceArgs r;
            if (team_args(s, team, r, why)) return fail("scan: " + why);
            r.ret = ret;
            const bool vec = ((d0 | s0) & 15) == 0;
            if (team_barrier(s, team, r, st)) return 1;
            HIP_TRY(launch_scan_direct(dt, a, vec, st));
            if (team_barrier(s, team, r, st)) return 1;
            if (mark_stream(s, st)) return 1;
            if (blocking) {
                if (host_wait(s, st)) return 1;
                if (check_team_errors(s, team)) return 1;
            }
            return 0;
        }
        if (order_stream(s, st) || staging_acquire(s, st)) return 1;
        for (uint64_t off = 0; off < n; off += seg) {
            const uint64_t m = std::min<uint64_t>(seg, n - off);
            ScanArgs a;
            memset(&a, 0, sizeof(a));
            std::string why;
            if (fill_team_sync_args(s, team, a, why)) return fail("scan: " + why);
            for (int j = 0; j < t.size; ++j) {
                const int gpe = t.start + j * t.stride;
                a.src[j] = translate(s, (const char *) src + off * es, gpe);
                a.scratch[j] = translate(s, s.staging, gpe);
            }
            a.dst = (char *) dst + off * es;
            a.ret = ret;
            a.nelems = m;
            a.items_per_chunk = items_per_chunk(m, t.size);
            a.inclusive = inclusive;
            const bool vec = (((uintptr_t) dst | (uintptr_t) src | (uintptr_t) s.staging) & 15) == 0;
            if ((long long) (m * es) >= s.phased_min) {
                // Large segment: barrier, one-shot fold grid, barrier, one-shot pull grid, barrier
                // (kernels_coll.hip scan_p1_kernel / scan_p2_kernel).  Every member knows m.
                ReduceArgs r;
                if (team_args(s, team, r, why)) return fail("scan: " + why);
                r.ret = ret;
                if (team_barrier(s, team, r, st)) return 1;
                HIP_TRY(launch_scan_phase(dt, a, vec, 1, st));
                if (team_barrier(s, team, r, st)) return 1;
                HIP_TRY(launch_scan_phase(dt, a, vec, 2, st));
                if (team_barrier(s, team, r, st)) return 1;
                continue;
            }
            const uint64_t tile = (uint64_t) kBlock * 2 * (vec ? 16 / es : 1);
            const int grid = (int) std::max<uint64_t>(
                1, std::min<uint64_t>((a.items_per_chunk + tile - 1) / tile, s.max_blocks));
            HIP_TRY(launch_scan(dt, a, vec, grid, st));
        }
        if (staging_release(s, st)) return 1;
    }
    if (mark_stream(s, st)) return 1;
    if (blocking) {
        if (host_wait(s, st)) return 1;
        if (check_team_errors(s, team)) return 1;
    }
    return 0;
}

int team_sync_locked(State &s, int team, hipStream_t st, int *ret)
{
    Team &t = s.teams[team];
    if (t.size <= 1) return 0;
    if (order_stream(s, st)) return 1;
    ReduceArgs a;
    std::string why;
    if (team_args(s, team, a, why)) return fail("team_sync: " + why);
    a.ret = ret;
    if (team_barrier(s, team, a, st)) return 1;
    return 0;
}

int reduce_impl(int team, int op, int dt, void *dst, const void *src, size_t n, int *ret,
                hipStream_t st, bool blocking)
{
    State &s = S();
    std::lock_guard<std::mutex> lk(s.mu);
    if (!s.initialized) return fail("reduce: ishmem not initialized");
    if (!op_dtype_valid(op, dt)) return fail("reduce: invalid (op, dtype) pair");
    if (team < 0 || team >= kMaxTeams || !s.teams[team].valid)
        return fail("reduce: invalid team handle");
    Team &t = s.teams[team];
    if (t.my_idx < 0) return fail("reduce: calling PE is not a member of the team");
    if (n > 0 && (!dst || !src)) return fail("reduce: null buffer");
    const size_t es = dtype_size(dt);
    const size_t bytes = n * es;
    // *ret: zeroed once here; every launch of the call ORs a failure into it (sticky).
    if (ret) HIP_TRY(hipMemsetAsync(ret, 0, sizeof(int), st));

    if (t.size == 1) {
        // One PE: the reduction is a copy (reduce_impl.h:288-289 with no peers to fold).
        if (n > 0 && dst != src) {
            const Kind kd = classify(s, dst), ks = classify(s, src);
            if (kd == Kind::Host || ks == Kind::Host) {
                // Host buffers take the same HBM-staged pipeline as on a multi-PE team, so the
                // path's host-to-host rate is the one reported in DESIGN.md.
                if (reduce_staged(s, team, op, dt, dst, src, n, ret, st)) return 1;
            } else if (launch_copy(dst, src, bytes, st)) {
                return 1;
            }
        }
    } else if (n == 0) {
        // The reference still synchronises the team (reduce_impl.h:244, :254).
        if (team_sync_locked(s, team, st, ret)) return 1;
    } else if (ll_eligible(s, t, dst, src, bytes) && classify(s, dst) != Kind::Host &&
               classify(s, src) != Kind::Host) {
        if (reduce_ll(s, team, op, dt, dst, src, bytes, ret, st)) return 1;
    } else if (in_heap(s, dst) && in_heap(s, src)) {
        if (reduce_heap(s, team, op, dt, dst, src, n, ret, st)) return 1;
    } else {
        if (reduce_staged(s, team, op, dt, dst, src, n, ret, st)) return 1;
    }
    if (mark_stream(s, st)) return 1;
    if (blocking) {
        if (host_wait(s, st)) return 1;
        if (check_team_errors(s, team)) return 1;
    }
    return 0;
}

// Refresh the device copy of the device-API context (after init and after team changes).
int sync_device_ctx(State &s)
{
    ishmemi_c_device_ctx_t c;
    memset(&c, 0, sizeof(c));
    c.pe = s.pe;
    c.npes = s.npes;
    c.timeout_ticks = (uint64_t) s.timeout_ms * 100000ull;
    c.heap_base = s.heap;
    c.heap_size = s.heap_size;
    for (int j = 0; j < s.npes; ++j) {
        c.peer_heap[j] = s.peer_heap[j];
        c.peer_dflags[j] = dev_flags(s.peer_flags[j]);
    }
    c.my_dflags = dev_flags(s.flags);  // device-API rows of every slot live in the base block
    c.epochs = s.dev_epochs;
    c.dev_counts = (uint64_t *) (s.count_slots + (size_t) kMaxTeams * 64);
    c.err = s.err_dev + kMaxTeams;
    for (int t = 0; t < kMaxTeams; ++t) {
        const Team &tm = s.teams[t];
        c.team_start[t] = tm.start;
        c.team_stride[t] = tm.stride;
        c.team_size[t] = tm.valid ? tm.size : 0;
        c.team_my_idx[t] = tm.valid ? tm.my_idx : -1;
    }
    HIP_TRY(hipMemcpy(s.dctx, &c, sizeof(c), hipMemcpyHostToDevice));
    return 0;
}

// Memory of the flag block (start / ready / done rows and the LL rings), which peers store into
// over xGMI while this PE's kernels poll it.  Best first:
//   uncached VRAM      every access goes to HBM, so a peer's store is seen by the next poll;
//   fine-grained VRAM  coherent device memory (hipDeviceMallocFinegrained);
//   coarse-grained     plain hipMalloc: polls are system-scope loads, but a line of local
//                      coarse-grained memory may stay in this device's L2 while a peer on another
//                      device writes HBM behind it — safe only when the PEs share one device.
enum FlagMem { kFlagsUncached = 0, kFlagsFineGrained = 1, kFlagsCoarse = 2, kFlagKinds = 3 };

const char *flag_kind_name(int k)
{
    return k == kFlagsUncached ? "uncached" : k == kFlagsFineGrained ? "fine-grained" : "coarse-grained";
}

// Allocates (zeroed) `bytes` of flag memory of the first kind >= `kind` (exactly `kind` when
// `exact`) that this device can allocate AND, when `exportable`, export over IPC.  Returns nonzero
// if none can; *out / *kind_out receive the block and its kind.
int alloc_flag_mem(State &s, size_t bytes, int kind, bool exact, bool exportable, hipIpcMemHandle_t *h,
                   uint32_t **out, int *kind_out, const char *what)
{
    // Test hook: behave as if uncached / fine-grained VRAM could not be allocated (the refusal of
    // coarse-grained flags across devices is tested with it on a one-GPU box).
    if (s.test_flags_unavailable) kind = std::max<int>(kind, kFlagsCoarse);
    for (int k = kind; k < (exact ? kind + 1 : (int) kFlagKinds); ++k) {
        uint32_t *f = nullptr;
        hipError_t e = k == kFlagsUncached ? hipExtMallocWithFlags((void **) &f, bytes, hipDeviceMallocUncached)
                       : k == kFlagsFineGrained
                           ? hipExtMallocWithFlags((void **) &f, bytes, hipDeviceMallocFinegrained)
                           : hipMalloc((void **) &f, bytes);
        if (e != hipSuccess) {
            (void) hipGetLastError();
            continue;
        }
        if (exportable && hipIpcGetMemHandle(h, f) != hipSuccess) {
            (void) hipGetLastError();
            (void) hipFree(f);
            continue;
        }
        if (hipMemset(f, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
            (void) hipFree(f);
            return fail(std::string(what) + ": flag block memset failed");
        }
        *out = f;
        *kind_out = k;
        return 0;
    }
    return fail(std::string(what) + ": no flag-block memory of kind " + flag_kind_name(kind) + (exact ? "" : " or lesser") +
                " could be allocated" + (exportable ? " and exported" + ipc_hint() : ""));
}

// The base block (init): the first kind >= `kind` this device can allocate and export.
int alloc_flags(State &s, int kind, bool exportable, hipIpcMemHandle_t *h)
{
    return alloc_flag_mem(s, kBaseAllocBytes, kind, false, exportable, h, &s.flags, &s.flags_kind, "init");
}

// In-place fold scratch of a team of `p` members (reduce_heap): allocated with the team.
int alloc_fold_scratch(State &s, int team, int p)
{
    TeamMem &m = s.tmem[team];
    if (p < 2) return 0;
    const size_t bytes = (size_t) (kInplaceFoldBytes / (uint64_t) p) + 256;
    if (hipMalloc((void **) &m.fold_scratch, bytes) != hipSuccess) {
        (void) hipGetLastError();
        m.fold_scratch = nullptr;
        return fail("team: in-place fold scratch of " + std::to_string(bytes) + " bytes not allocated");
    }
    m.fold_scratch_bytes = bytes;
    return 0;
}

// Releases a slot's memory on this PE: the imported blocks of its members, its own block (split
// teams), its fold scratch.  hipFree waits for the device, so no kernel of this PE still uses them;
// a peer's mapping of this PE's block keeps that memory alive until the peer closes it.
void release_team_mem(State &s, int team)
{
    TeamMem &m = s.tmem[team];
    if (m.pool_idx >= 0 || m.fold_scratch) (void) hipDeviceSynchronize();  // this PE's kernels are done with them
    if (m.pool_idx >= 0 && m.pool_idx < (int) s.team_pool.size()) {
        s.team_pool[(size_t) m.pool_idx].in_use = false;  // zeroed again when a split takes it
        s.team_block_bytes -= kTeamAllocBytes;
    }
    if (m.fold_scratch) (void) hipFree(m.fold_scratch);  // plain device memory, never exported
    m = TeamMem{};
}

// At finalize: the peers' pool blocks mapped here, then this PE's own pool.
void release_team_pool(State &s)
{
    for (auto &kv : s.peer_pool) (void) hipIpcCloseMemHandle(kv.second);
    s.peer_pool.clear();
    for (PoolBlock &b : s.team_pool) (void) hipFree(b.ptr);
    s.team_pool.clear();
    s.team_block_bytes = 0;
}

// Device identity of every PE as small integers (PEs on one GPU share one), from the PCI bus ids
// allgathered at init; a team is co-located when all its members share one.
bool team_colocated(const State &s, const Team &t)
{
    for (int j = 1; j < t.size; ++j)
        if (s.dev_id[t.start + j * t.stride] != s.dev_id[t.start]) return false;
    return true;
}

int init_impl(int pe, int npes, int device, const std::string &key)
{
    State &s = S();
    std::lock_guard<std::mutex> lk(s.mu);
    if (s.initialized) return 0;
    if (npes < 1 || npes > kMaxPes || pe < 0 || pe >= npes)
        return fail("init: invalid pe/npes (npes must be 1.." + std::to_string(kMaxPes) + ")");
    s.pe = pe;
    s.npes = npes;
    set_device_share(1);
    // Default: 16, or 4 per hardware queue when the process was given more than 4 (GPU_MAX_HW_QUEUES):
    // the cap must leave room for every kernel the process's queues can run at once (kernels.h).
    // The floor is the queue count itself: below it one process's queues could run more waiting
    // launches than the device holds slots for, the round-3 footprint that hung 4 co-located PEs
    // (profiles/r04/wait_cost/r04b_wait_cost_p4_ws1_killed.txt), so such a value fails init.
    const long long hwq = std::max<long long>(1, env_ll("GPU_MAX_HW_QUEUES", 4));
    const long long ws = env_ll("ISHMEM_WAIT_SLOTS", std::max<long long>(kWaitSlotsDefault, 4 * hwq));
    if (ws < wait_slots_floor() && g_env_error.empty())
        g_env_error = "ISHMEM_WAIT_SLOTS=" + std::to_string(ws) + " is below " + std::to_string(wait_slots_floor()) +
                      " (GPU_MAX_HW_QUEUES): every kernel a process's hardware queues can run at once needs "
                      "its own slot of the device, or collectives of different teams can wait on each other forever";
    set_wait_slots((int) std::min<long long>(1 << 20, std::max<long long>(wait_slots_floor(), ws)));
    // Reference switches this path cannot honour: it is IPC-only (every PE maps every peer's heap)
    // and its heap is device memory (src/ishmem/env_defs.h:16,22; src/teams.cpp:86-89,
    // src/ishmem.cpp:319-330, where they move intra-node traffic off IPC).  Refused, not ignored.
    if (env_flag_false("ISHMEM_ENABLE_GPU_IPC") && g_env_error.empty())
        g_env_error = std::string("ISHMEM_ENABLE_GPU_IPC=") + getenv("ISHMEM_ENABLE_GPU_IPC") +
                      " is not supported: ishmem_amd's collectives are IPC-only (peer loads over xGMI from "
                      "IPC-mapped heaps; there is no proxy path)";
    if (env_flag_true("ISHMEM_ENABLE_ACCESSIBLE_HOST_HEAP") && g_env_error.empty())
        g_env_error = std::string("ISHMEM_ENABLE_ACCESSIBLE_HOST_HEAP=") + getenv("ISHMEM_ENABLE_ACCESSIBLE_HOST_HEAP") +
                      " is not supported: the symmetric heap is device memory shared over IPC (host buffers "
                      "are accepted by every call and staged)";
    s.max_blocks = (int) std::min<long long>(kMaxBlocks, std::max<long long>(1, env_ll("ISHMEM_MAX_BLOCKS", kMaxBlocks)));
    s.timeout_ms = std::max<long long>(1, env_ll("ISHMEM_TIMEOUT_MS", 60000));
    s.ll_max_bytes = std::min<long long>((long long) kLLMaxBytes,
                                         std::max<long long>(0, env_bytes("ISHMEM_LL_MAX_BYTES", (long long) kLLDefaultBytes)));
    s.debug = debug_level();
    s.trace = nullptr;
    s.stream_order = env_ll("ISHMEM_STREAM_ORDER", 0) != 0;
    s.oneshot_p2 = std::max<long long>(0, env_bytes("ISHMEM_ONESHOT_P2_MAX_BYTES", 32ll << 20));
    s.phased_min = env_bytes("ISHMEM_PHASED_MIN_BYTES", kPhasedDefault);
    if (s.phased_min < 0) s.phased_min = kPhasedOff;
    s.staging_bytes = (env_size("ISHMEM_STAGING_SIZE", (size_t) 128 << 20) + kHeapAlign - 1) &
                      ~(size_t) (kHeapAlign - 1);
    s.staging_slots = (int) std::min<long long>(kMaxStagingSlots, std::max<long long>(2, env_ll("ISHMEM_STAGING_SLOTS", kStagingSlotsDefault)));
    s.staged_copy_kernel = (int) (env_ll("ISHMEM_STAGED_COPY_KERNEL", kStagedCopyKernelDefault) & 3);
    const size_t heap_request = env_size("ISHMEM_SYMMETRIC_SIZE", (size_t) 4 << 30);
    // ISHMEM_FLAGS_KIND (tests): start the flag-memory ladder at FlagMem 1 or 2 instead of uncached VRAM.
    const int first_kind = (int) std::min<long long>(kFlagsCoarse, std::max<long long>(0, env_ll("ISHMEM_FLAGS_KIND", 0)));
#ifdef ISHMEMI_TEST_HOOKS
    s.test_flags_unavailable = env_ll("ISHMEM_TEST_FLAGS_UNAVAILABLE", 0) != 0;
#else
    // The test hooks (fake device identity, flag memory "unavailable") exist only in the test
    // build (libishmem_amd_testhooks.so, ishmem_amd/_build.py); the product library refuses them
    // rather than silently running a test against unhooked behaviour.
    for (const char *hook : {"ISHMEM_TEST_FLAGS_UNAVAILABLE", "ISHMEM_TEST_PCI_BUS"})
        if (getenv(hook) && g_env_error.empty())
            g_env_error = std::string(hook) + " is a test hook, honoured only by libishmem_amd_testhooks.so";
#endif
    const bool ep_uncached = env_ll("ISHMEM_EP_UNCACHED", 0) != 0;
    s.phased_peer_nt = env_ll("ISHMEM_PHASED_PEER_NT", 0) != 0;
    // ISHMEM_TEAMS_MAX (src/ishmem/env_defs.h:34, default 64): the team table's size.  Below the 3
    // predefined teams it is raised to 3, as the reference does (src/teams.cpp:118-119); above 64
    // init fails as the reference's does (src/teams.cpp:245-248: its slot mask has 64 bits).
    s.teams_max = kTeamsMaxDefault;
    if (const char *tm = getenv("ISHMEM_TEAMS_MAX"); tm && *tm) {
        const long long v = env_ll("ISHMEM_TEAMS_MAX", kTeamsMaxDefault);
        if (v < 0 && g_env_error.empty())
            g_env_error = std::string("ISHMEM_TEAMS_MAX='") + tm + "' is not a team count";
        else if (v > kMaxTeams && g_env_error.empty())
            g_env_error = "ISHMEM_TEAMS_MAX=" + std::to_string(v) + ": requested " + std::to_string(v) +
                          " teams, but only " + std::to_string(kMaxTeams) + " are supported";
        s.teams_max = (int) std::min<long long>(kMaxTeams, std::max<long long>(kPredefTeams, v));
    }
    // Cross-device teams' thresholds (path_limits): -1 / unset = the link-byte model.
    s.xgmi_ll_max = std::max<long long>(-1, env_bytes("ISHMEM_XGMI_LL_MAX_BYTES", -1));
    s.xgmi_fold_max = std::max<long long>(-1, env_bytes("ISHMEM_XGMI_FOLD_MAX_BYTES", -1));
    s.xgmi_link_bps = 76.8e9;
    // Round 5's stream-memory-op barrier was removed in round 6 (team_barrier): "kernel" is still
    // accepted, "stream" is refused rather than silently ignored.
    if (const char *bk = getenv("ISHMEM_BARRIER_KIND"); bk && *bk && strcasecmp(bk, "kernel") != 0 && g_env_error.empty())
        g_env_error = std::string("ISHMEM_BARRIER_KIND='") + bk +
                      "' is not supported: team barriers are the one-workgroup barrier kernel ('kernel')";
    if (!g_env_error.empty()) {
        const std::string e = g_env_error;
        g_env_error.clear();
        return fail("init: " + e);
    }
    warn_unknown_env();

    using clk = std::chrono::steady_clock;
    const auto t_start = clk::now();
    auto t_mark = t_start;
    // Under ISHMEM_DEBUG=2 every phase prints as it ends, so a stalled init shows where it is.
    auto phase_done = [&](int k) {
        const auto now = clk::now();
        s.init_us[k] = std::chrono::duration<double, std::micro>(now - t_mark).count();
        t_mark = now;
        if (s.debug > 1) {
            fprintf(stderr, "[ishmem_amd] PE %d init: %s done (%.1f ms)\n", pe, kInitPhase[k], s.init_us[k] / 1000.0);
            fflush(stderr);
        }
    };
    for (double &u : s.init_us) u = 0;
    if (s.debug > 1) {
        fprintf(stderr, "[ishmem_amd] PE %d of %d init: start (device %d, heap %zu MiB, key '%s')\n", pe, npes, device,
                heap_request >> 20, key.c_str());
        fflush(stderr);
    }

    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (ndev < 1) return fail("init: no HIP device visible");
    s.device = device >= 0 ? device % ndev : 0;
    HIP_TRY(hipSetDevice(s.device));
    HIP_TRY(hipFree(nullptr));  // the HIP runtime's own initialisation, timed on its own
    phase_done(0);

    // Symmetric heap: ONE hipMalloc (coarse-grained HBM) per PE, src/memory.cpp:35-132.
    s.heap_size = heap_request;
    s.heap_size = (s.heap_size + (2u << 20) - 1) & ~(size_t) ((2u << 20) - 1);
    HIP_TRY(hipMalloc((void **) &s.heap, s.heap_size));
    s.free_list.clear();
    s.used.clear();
    s.free_list[0] = s.heap_size;
    phase_done(1);

    // Barrier flags (written by peers over xGMI): the best memory kind that can also be exported.
    hipIpcMemHandle_t flags_handle{};
    if (alloc_flags(s, first_kind, npes > 1, &flags_handle)) return 1;
    HIP_TRY(hipHostMalloc((void **) &s.err_host, kErrDoneOffset + 64, hipHostMallocMapped | hipHostMallocCoherent));
    memset(s.err_host, 0, kErrDoneOffset + 64);
    HIP_TRY(hipHostGetDevicePointer((void **) &s.err_dev, s.err_host, 0));
    s.exch_host = (uint64_t *) ((char *) s.err_host + kErrExchOffset);
    s.exch_dev = (uint64_t *) ((char *) s.err_dev + kErrExchOffset);
    s.done_host = (uint32_t *) ((char *) s.err_host + kErrDoneOffset);
    s.done_dev = (uint32_t *) ((char *) s.err_dev + kErrDoneOffset);
    s.done_seq = 0;
    HIP_TRY(hipDeviceSynchronize());

    for (int i = 0; i < kMaxPes; ++i) {
        s.peer_heap[i] = nullptr;
        s.peer_flags[i] = nullptr;
    }
    s.peer_heap[pe] = s.heap;
    s.peer_flags[pe] = s.flags;
    for (int i = 0; i < kMaxPes; ++i) s.dev_id[i] = 0;
    phase_done(2);

    if (npes > 1) {
        // Let peers import our dma-buf handles (pidfd_getfd needs ptrace rights under Yama), for
        // the import window only: the guard restores the default when this block is left.
        struct PtracerWindow {
            PtracerWindow() { prctl(PR_SET_PTRACER, PR_SET_PTRACER_ANY, 0, 0, 0); }
            ~PtracerWindow() { prctl(PR_SET_PTRACER, 0, 0, 0, 0); }
        } ptracer_window;
        std::string err;
        if (s.boot.attach(pe, npes, key, (int) std::max<long long>(s.timeout_ms, 10000), err))
            return fail(err);
        PeRecord mine{};
        mine.pe = pe;
        mine.pid = (int32_t) getpid();
        mine.device = s.device;
        mine.flags_kind = s.flags_kind;
        mine.flags_kind_requested = first_kind;
        mine.heap_size = s.heap_size;
        mine.max_blocks = s.max_blocks;
        mine.ll_max_bytes = s.ll_max_bytes;
        mine.oneshot_p2 = s.oneshot_p2;
        mine.phased_min = s.phased_min;
        mine.staging_bytes = s.staging_bytes;
        mine.staging_slots = s.staging_slots;
        mine.xgmi_ll_max = s.xgmi_ll_max;
        mine.xgmi_fold_max = s.xgmi_fold_max;
        if (hipDeviceGetPCIBusId(mine.pci_bus, sizeof(mine.pci_bus), s.device) != hipSuccess) {
            (void) hipGetLastError();
            snprintf(mine.pci_bus, sizeof(mine.pci_bus), "dev%d", s.device);
        }
        // Test hook: a device identity of the test's choosing (PEs sharing the box's one GPU then
        // count as PEs on different devices wherever the runtime decides by device identity).
#ifdef ISHMEMI_TEST_HOOKS
        if (const char *fake = getenv("ISHMEM_TEST_PCI_BUS"))
            snprintf(mine.pci_bus, sizeof(mine.pci_bus), "%s", fake);
#endif
        if (hipError_t e = hipIpcGetMemHandle(&mine.heap_handle, s.heap); e != hipSuccess)
            return fail(std::string("init: hipIpcGetMemHandle of the symmetric heap: ") + hipGetErrorString(e) + ipc_hint());
        mine.flags_handle = flags_handle;
        PeRecord all[kMaxPes];
        if (s.boot.allgather(&mine, all, sizeof(PeRecord), err)) return fail(err);
        phase_done(3);
        // Agree on the parameters that choose a call's kernel (the minimum over the PEs), so a
        // per-process environment difference cannot split LL from RS/AG or one-shot from RS/AG.
        // The grid cap (max_blocks) stays per PE: the kernels grab work, nothing is paired.
        for (int j = 0; j < npes; ++j) {
            s.ll_max_bytes = std::min<long long>(s.ll_max_bytes, all[j].ll_max_bytes);
            s.oneshot_p2 = std::min<long long>(s.oneshot_p2, all[j].oneshot_p2);
            s.phased_min = std::max<long long>(s.phased_min, all[j].phased_min);
            s.staging_bytes = std::min<size_t>(s.staging_bytes, all[j].staging_bytes);
            s.staging_slots = (int) std::min<int64_t>(s.staging_slots, all[j].staging_slots);
            // The cross-device overrides: the smallest value any PE set (-1, the model, only when
            // none did).
            if (all[j].xgmi_ll_max >= 0)
                s.xgmi_ll_max = s.xgmi_ll_max < 0 ? all[j].xgmi_ll_max : std::min<long long>(s.xgmi_ll_max, all[j].xgmi_ll_max);
            if (all[j].xgmi_fold_max >= 0)
                s.xgmi_fold_max = s.xgmi_fold_max < 0 ? all[j].xgmi_fold_max
                                                       : std::min<long long>(s.xgmi_fold_max, all[j].xgmi_fold_max);
        }
        int share = 0;
        for (int j = 0; j < npes; ++j)
            share += strncmp(all[j].pci_bus, mine.pci_bus, sizeof(mine.pci_bus)) == 0;
        // Device ids: the first PE with the same PCI bus id (identical on every PE).
        for (int j = 0; j < npes; ++j) {
            s.dev_id[j] = j;
            for (int k = 0; k < j; ++k)
                if (strncmp(all[j].pci_bus, all[k].pci_bus, sizeof(all[j].pci_bus)) == 0) {
                    s.dev_id[j] = s.dev_id[k];
                    break;
                }
        }
        bool coarse_forced = false;  // a test asked for coarse-grained flags (ISHMEM_FLAGS_KIND=2)
        for (int j = 0; j < npes; ++j) coarse_forced = coarse_forced || all[j].flags_kind_requested == kFlagsCoarse;
        set_device_share(share);
        for (int j = 0; j < npes; ++j) {
            if (j == pe) continue;
            if (all[j].heap_size != s.heap_size)
                return fail("init: ISHMEM_SYMMETRIC_SIZE differs between PEs");
            if (all[j].device != s.device) {
                // The kernels load peers' memory directly over xGMI: without peer access those
                // loads would fault the GPU, so refuse to initialise instead.
                int can = 0;
                if (hipDeviceCanAccessPeer(&can, s.device, all[j].device) != hipSuccess || !can)
                    return fail("init: no peer access from device " + std::to_string(s.device) +
                                " to device " + std::to_string(all[j].device) + " (PE " +
                                std::to_string(j) + ")");
                hipError_t e = hipDeviceEnablePeerAccess(all[j].device, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
                    return hipfail("hipDeviceEnablePeerAccess", e);
                (void) hipGetLastError();
            }
            if (hipError_t e = hipIpcOpenMemHandle((void **) &s.peer_heap[j], all[j].heap_handle,
                                                   hipIpcMemLazyEnablePeerAccess);
                e != hipSuccess)
                return fail("init: hipIpcOpenMemHandle of PE " + std::to_string(j) + "'s heap: " + hipGetErrorString(e) +
                            ipc_hint());
        }
        phase_done(4);
        // Flags (+ LL rings): every PE uses the same memory kind, the least capable one any PE
        // could allocate and export; if some PE cannot import a peer's block of that kind, all
        // step down one kind together and exchange new blocks.
        int kind = 0;
        bool fresh = false;  // identical on every PE: all take the same branches below
        for (int j = 0; j < npes; ++j) kind = std::max(kind, (int) all[j].flags_kind);
        for (int j = 0; j < npes; ++j) fresh = fresh || all[j].flags_kind != kind;
        hipIpcMemHandle_t hs[kMaxPes];
        for (int j = 0; j < npes; ++j) hs[j] = all[j].flags_handle;
        for (;;) {
            if (fresh) {
                // Every PE replaces its block by one of `kind` (or the next kind it can make).
                if (s.boot.barrier(err)) return fail(err);  // no peer still maps our old block
                (void) hipFree(s.flags);
                s.flags = nullptr;
                hipIpcMemHandle_t h{};
                if (alloc_flags(s, kind, true, &h)) return 1;
                s.peer_flags[pe] = s.flags;
                int32_t k = s.flags_kind, ks[kMaxPes];
                if (s.boot.allgather(&k, ks, sizeof(k), err)) return fail(err);
                if (s.boot.allgather(&h, hs, sizeof(h), err)) return fail(err);
                int agreed = kind;
                for (int j = 0; j < npes; ++j) agreed = std::max(agreed, (int) ks[j]);
                fresh = false;
                for (int j = 0; j < npes; ++j) fresh = fresh || ks[j] != agreed;
                kind = agreed;
                if (fresh) continue;  // PEs ended on different kinds: again, at the lesser one
            }
            int32_t opened = 1;
            for (int j = 0; j < npes && opened; ++j) {
                if (j == pe) continue;
                if (hipIpcOpenMemHandle((void **) &s.peer_flags[j], hs[j], hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
                    (void) hipGetLastError();
                    s.peer_flags[j] = nullptr;
                    opened = 0;
                }
            }
            int32_t all_opened[kMaxPes];
            if (s.boot.allgather(&opened, all_opened, sizeof(int32_t), err)) return fail(err);
            bool ok = true;
            for (int j = 0; j < npes; ++j) ok = ok && all_opened[j];
            if (ok) break;
            for (int j = 0; j < npes; ++j) {
                if (j != pe && s.peer_flags[j]) (void) hipIpcCloseMemHandle(s.peer_flags[j]);
                s.peer_flags[j] = nullptr;
            }
            s.peer_flags[pe] = s.flags;
            if (++kind >= kFlagKinds) return fail("init: no flag-block memory kind can be imported by every PE");
            fresh = true;
        }
        if (s.flags_kind == kFlagsCoarse && share < npes && !coarse_forced) {
            // A line of local coarse-grained memory may stay in this device's L2 while a peer on
            // another device stores into HBM behind it: the polls could miss the flags and every
            // collective would end in device timeouts.  Refuse, on every PE alike (the kind,
            // the device identities and the requests were all agreed / allgathered above).
            std::string kinds;
            for (int j = 0; j < npes; ++j)
                kinds += (j ? ", " : "") + std::string("PE ") + std::to_string(j) + " " +
                         flag_kind_name(all[j].flags_kind) + " on " + all[j].pci_bus;
            return fail("init: the PEs span several devices but could only share coarse-grained flag "
                        "memory (uncached / fine-grained VRAM could not be allocated, exported or imported "
                        "by every PE: " + kinds + "); peers' flag stores could stay invisible to this "
                        "device's polls.  ISHMEM_FLAGS_KIND=2 forces it anyway (tests only)");
        }
        if (s.boot.barrier(err)) return fail(err);  // every peer has imported our handles
        phase_done(5);
    }

    // Teams: WORLD, SHARED, NODE all span the node (src/teams.cpp:108-257); their flag blocks and
    // rings live in the base block of every PE.
    for (int i = 0; i < kMaxTeams; ++i) {
        s.teams[i] = Team{};
        s.tmem[i] = TeamMem{};
    }
    s.team_block_bytes = 0;
    for (int i = 0; i < kPredefTeams; ++i) {
        Team &t = s.teams[i];
        t.valid = true;
        t.start = 0;
        t.stride = 1;
        t.size = npes;
        t.my_idx = pe;
        t.colocated = team_colocated(s, t);
        for (int j = 0; j < npes; ++j) {
            s.tmem[i].flags[j] = base_team_flags(s.peer_flags[j], i);
            s.tmem[i].ring[j] = base_team_ring(s.peer_flags[j], i);
        }
        if (alloc_fold_scratch(s, i, npes)) return 1;
    }
    // Symmetric staging region (first allocation on every PE, hence the same offset).
    s.staging = (char *) heap_alloc(s, s.staging_bytes, kHeapAlign);
    if (!s.staging) return 1;
    s.team_scratch = (char *) heap_alloc(s, kTeamScratchBytes, kHeapAlign);
    if (!s.team_scratch) return 1;
    // [0, kMaxTeams) lines: collect_on_stream; [kMaxTeams, 2 kMaxTeams): the device API's collect.
    s.count_slots = (char *) heap_alloc(s, (size_t) 2 * kMaxTeams * 64, kHeapAlign);
    if (!s.count_slots) return 1;
    HIP_TRY(hipMalloc((void **) &s.dctx, sizeof(ishmemi_c_device_ctx_t)));
    // Launch words: local to this device, touched only by device-scope atomics (work grabs,
    // counters) and system-scope loads/stores (the epoch), which do not depend on the memory
    // type; ordinary device memory (ISHMEM_EP_UNCACHED=1: fine-grained uncached, for comparison).
    const size_t ep_bytes = (size_t) kEpTeamWords * kMaxTeams * sizeof(uint32_t);
    if (!ep_uncached ||
        hipExtMallocWithFlags((void **) &s.kern_ep, ep_bytes, hipDeviceMallocUncached) != hipSuccess) {
        (void) hipGetLastError();
        HIP_TRY(hipMalloc((void **) &s.kern_ep, ep_bytes));
    }
    HIP_TRY(hipMemset(s.kern_ep, 0, ep_bytes));
    HIP_TRY(hipMalloc((void **) &s.dev_epochs, kMaxTeams * sizeof(uint32_t)));
    HIP_TRY(hipMemset(s.dev_epochs, 0, kMaxTeams * sizeof(uint32_t)));
    if (sync_device_ctx(s)) return 1;
    HIP_TRY(hipDeviceSynchronize());
    phase_done(6);
    s.init_us[7] = std::chrono::duration<double, std::micro>(clk::now() - t_start).count();
    if (s.debug > 1) {
        std::string line;
        char buf[64];
        for (int k = 0; k < 8; ++k) {
            snprintf(buf, sizeof(buf), " %s %.1f", kInitPhase[k], s.init_us[k] / 1000.0);
            line += buf;
        }
        fprintf(stderr, "[ishmem_amd] PE %d init phases (ms):%s (heap %zu MiB, flag block %zu KiB)\n", pe, line.c_str(),
                s.heap_size >> 20, kBaseAllocBytes >> 10);
    }
    s.initialized = true;
    write_ctx_slots(s.dctx);
    return 0;
}

const char *env_str(const char *name)
{
    const char *s = getenv(name);
    return s && *s ? s : nullptr;
}

// Parent pid of process `pid` (/proc/<pid>/stat field 4), or -1.
long parent_of(long pid)
{
    char path[64];
    snprintf(path, sizeof(path), "/proc/%ld/stat", pid);
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    char buf[512];
    const size_t n = fread(buf, 1, sizeof(buf) - 1, f);
    fclose(f);
    buf[n] = '\0';
    const char *rp = strrchr(buf, ')');  // the command name may hold spaces and parentheses
    long ppid = -1;
    char state;
    if (!rp || sscanf(rp + 1, " %c %ld", &state, &ppid) != 2) return -1;
    return ppid;
}

// Whether process `pid`'s environment defines `var`; -1 if it cannot be read.
int env_of_has(long pid, const char *var)
{
    char path[64];
    snprintf(path, sizeof(path), "/proc/%ld/environ", pid);
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    const size_t vl = strlen(var);
    std::string entry;
    int found = 0;
    for (int c; (c = fgetc(f)) != EOF;) {
        if (c != '\0') {
            entry.push_back((char) c);
            continue;
        }
        if (entry.size() > vl && entry.compare(0, vl, var) == 0 && entry[vl] == '=') found = 1;
        entry.clear();
        if (found) break;
    }
    fclose(f);
    return found;
}

// The launcher's per-node daemon that started every local rank (hydra_pmi_proxy, orted / prted,
// slurmstepd): the nearest ancestor whose environment lacks the launcher's rank variable.  Ranks
// started through a wrapper script (the reference's `mpirun -n N scripts/ishmrun ./app`,
// test/cmake/common.cmake:28-43) still find the same daemon, hence the same bootstrap key.
long launcher_daemon(const char *rank_var)
{
    long p = (long) getppid();
    for (int depth = 0; depth < 64 && p > 1; ++depth) {
        const int has = env_of_has(p, rank_var);
        if (has == 0) return p;
        const long pp = parent_of(p);
        if (has < 0 || pp <= 1) break;
        p = pp;
    }
    return (long) getppid();
}

// PE identity from the process's launcher.  The reference's ishmem_init takes rank and size from
// its runtime (MPI: src/runtime/runtime_mpi.cpp:1256-1282; PMI / OpenSHMEM alike); this library
// has no runtime of its own, so it reads what the launcher exports, first match wins:
//   ISHMEM_PE / ISHMEM_NPES / ISHMEM_DEVICE   explicit (tests, custom launchers)
//   RANK / WORLD_SIZE / LOCAL_RANK            torchrun
//   PMI_RANK / PMI_SIZE / MPI_LOCALRANKID     MPICH hydra, Intel MPI (mpiexec / mpirun)
//   OMPI_COMM_WORLD_RANK / _SIZE / _LOCAL_RANK  Open MPI
//   SLURM_PROCID / SLURM_STEP_NUM_TASKS / SLURM_LOCALID   an srun task step (numeric SLURM_STEP_ID)
// ISHMEM_PE, ISHMEM_NPES, ISHMEM_DEVICE and ISHMEM_BOOTSTRAP_KEY each override the launcher's
// value.  The device is the node-local rank (one PE per GPU; modulo the visible devices).
struct LaunchInfo {
    int pe = 0, npes = 1, local = 0, local_n = 0, nodes = 0;
    std::string launcher = "none", key;
    std::string err;  // first malformed identity variable (strict, like env_ll)
};

// Slurm step ids that are not an srun task step: a program started directly in the batch script,
// an salloc shell or the extern step runs as a 1-PE world, not as PE 0 of the allocation.
bool slurm_task_step(const char *step)
{
    if (!step) return false;
    for (const char *c = step; *c; ++c)
        if (*c < '0' || *c > '9') return false;  // "batch", "interactive", "extern", ...
    return true;
}

LaunchInfo launch_info()
{
    LaunchInfo li;
    // Identity values pick the bootstrap world, so a malformed one fails resolve_launch with its
    // name instead of parsing as a prefix ("2x" -> 2, "abc" -> 0) and hanging in the bootstrap.
    auto num = [&li](const char *name, int dflt) -> int {
        const char *v = env_str(name);
        if (!v) return dflt;
        const char *b = v;
        while (*b == ' ' || *b == '\t') ++b;
        char *end = nullptr;
        errno = 0;
        const long long x = strtoll(b, &end, 10);
        const char *e = end;
        while (*e == ' ' || *e == '\t') ++e;
        if (end == b || *e || errno == ERANGE || x < INT32_MIN || x > INT32_MAX) {
            if (li.err.empty()) li.err = std::string(name) + "='" + v + "' is not an integer";
            return dflt;
        }
        return (int) x;
    };
    if (env_str("ISHMEM_PE")) {
        li.launcher = "ishmem";
        li.pe = num("ISHMEM_PE", 0);
        li.npes = env_str("ISHMEM_NPES") ? num("ISHMEM_NPES", 1) : num("WORLD_SIZE", 1);
        li.local = num("LOCAL_RANK", 0);
    } else if (env_str("RANK")) {
        li.launcher = "torchrun";
        li.pe = num("RANK", 0);
        li.npes = num("WORLD_SIZE", 1);
        li.local = num("LOCAL_RANK", 0);
        li.local_n = num("LOCAL_WORLD_SIZE", 0);
    } else if (env_str("PMI_RANK")) {
        li.launcher = "pmi";
        li.pe = num("PMI_RANK", 0);
        li.npes = num("PMI_SIZE", 1);
        li.local = num("MPI_LOCALRANKID", li.pe);
        li.local_n = num("MPI_LOCALNRANKS", 0);
        li.key = "pmi_d" + std::to_string(launcher_daemon("PMI_RANK"));
    } else if (env_str("OMPI_COMM_WORLD_RANK")) {
        li.launcher = "openmpi";
        li.pe = num("OMPI_COMM_WORLD_RANK", 0);
        li.npes = num("OMPI_COMM_WORLD_SIZE", 1);
        li.local = num("OMPI_COMM_WORLD_LOCAL_RANK", li.pe);
        li.local_n = num("OMPI_COMM_WORLD_LOCAL_SIZE", 0);
        const char *job = env_str("OMPI_MCA_ess_base_jobid") ? env_str("OMPI_MCA_ess_base_jobid") : env_str("PMIX_NAMESPACE");
        li.key = job ? std::string("ompi_") + job : "ompi_d" + std::to_string(launcher_daemon("OMPI_COMM_WORLD_RANK"));
    } else if (env_str("SLURM_PROCID") && env_str("SLURM_STEP_NUM_TASKS") && slurm_task_step(env_str("SLURM_STEP_ID"))) {
        // srun task step only: the step-scoped variables, which srun sets and the batch script's
        // environment lacks (there SLURM_PROCID=0 / SLURM_NTASKS=N describe the allocation, and a
        // program started without srun is one process, i.e. a 1-PE world).
        li.launcher = "slurm";
        li.pe = num("SLURM_PROCID", 0);
        li.npes = num("SLURM_STEP_NUM_TASKS", 1);
        li.local = num("SLURM_LOCALID", li.pe);
        li.nodes = num("SLURM_STEP_NUM_NODES", 0);
        li.key = std::string("slurm_") + (env_str("SLURM_JOB_ID") ? env_str("SLURM_JOB_ID") : "0") + "_" +
                 env_str("SLURM_STEP_ID");
    }
    if (env_str("ISHMEM_NPES")) li.npes = num("ISHMEM_NPES", li.npes);
    if (env_str("ISHMEM_DEVICE")) li.local = num("ISHMEM_DEVICE", li.local);
    if (const char *k = env_str("ISHMEM_BOOTSTRAP_KEY")) {
        li.key = k;
    } else if (li.key.empty()) {
        std::string key = "job";
        const char *port = env_str("MASTER_PORT"), *run = env_str("TORCHELASTIC_RUN_ID");
        if (port) key += std::string("_p") + port;
        if (run) key += std::string("_") + run;
        // No launcher variables: the PEs of one job are siblings (started by one launcher
        // process), so its pid keeps concurrent jobs on a node apart.
        if (!port && !run) key += "_pp" + std::to_string((long) getppid());
        li.key = key;
    }
    return li;
}

std::string default_key() { return launch_info().key; }

// The launcher's identity, checked: this library spans one node (every PE maps every peer's heap),
// so a job the launcher spread over several nodes is refused instead of becoming several
// independent worlds.
int resolve_launch(LaunchInfo &li)
{
    li = launch_info();
    if (!li.err.empty()) return fail("init: " + li.err);
    if (li.npes < 1 || li.pe < 0 || li.pe >= li.npes)
        return fail("init: launcher '" + li.launcher + "' gives PE " + std::to_string(li.pe) + " of " +
                    std::to_string(li.npes));
    if (li.local_n > 0 && li.local_n < li.npes && !env_str("ISHMEM_NPES"))
        return fail("init: the launcher ('" + li.launcher + "') started " + std::to_string(li.npes) +
                    " PEs but only " + std::to_string(li.local_n) +
                    " on this node; ishmem_amd's PEs must share one node (xGMI peer mappings)");
    if (li.nodes > 1 && !env_str("ISHMEM_NPES"))
        return fail("init: the launcher ('" + li.launcher + "') spread the job's " + std::to_string(li.npes) +
                    " PEs over " + std::to_string(li.nodes) +
                    " nodes; ishmem_amd's PEs must share one node (xGMI peer mappings)");
    return 0;
}

}  // namespace
}  // namespace ishmemi

using namespace ishmemi;

extern "C" {

int ishmemi_c_init(void)
{
    LaunchInfo li;
    if (resolve_launch(li)) return 1;
    return init_impl(li.pe, li.npes, li.local, li.key);
}

int ishmemi_c_init_pe(int pe, int npes, int device, const char *key)
{
    if (device < 0) device = launch_info().local;
    return init_impl(pe, npes, device, key && *key ? std::string(key) : default_key());
}

int ishmemi_c_launch_info(int *pe, int *npes, int *device, char *launcher, size_t launcher_len, char *key,
                          size_t key_len)
{
    LaunchInfo li;
    const int rc = resolve_launch(li);
    if (pe) *pe = li.pe;
    if (npes) *npes = li.npes;
    if (device) *device = li.local;
    if (launcher && launcher_len) snprintf(launcher, launcher_len, "%s", li.launcher.c_str());
    if (key && key_len) snprintf(key, key_len, "%s", li.key.c_str());
    return rc;
}

int ishmemi_c_finalize(void)
{
    State &s = S();
    std::lock_guard<std::mutex> lk(s.mu);
    if (!s.initialized) return 0;
    (void) hipDeviceSynchronize();
    write_ctx_slots(nullptr);  // device-API calls after finalize fail instead of using freed state
    if (s.npes > 1) {
        std::string err;
        s.boot.barrier(err);  // no peer may still be reading our heap
        for (int j = 0; j < s.npes; ++j) {
            if (j == s.pe) continue;
            if (s.peer_heap[j]) (void) hipIpcCloseMemHandle(s.peer_heap[j]);
            if (s.peer_flags[j]) (void) hipIpcCloseMemHandle(s.peer_flags[j]);
            s.peer_heap[j] = nullptr;
            s.peer_flags[j] = nullptr;
        }
        // The peers' team-pool blocks too, before the barrier after which every PE frees its own
        // exported memory (freeing an exported block while a peer still maps it is not something
        // to depend on: tools/ipc_leak_probe.py's free-before-close case never completed).
        for (auto &kv : s.peer_pool) (void) hipIpcCloseMemHandle(kv.second);
        s.peer_pool.clear();
        s.boot.barrier(err);
        s.boot.detach();
    }
    if (s.copy_in) {
        (void) hipStreamDestroy(s.copy_in);
        (void) hipStreamDestroy(s.copy_out);
        for (int i = 0; i < kMaxStagingSlots; ++i) {
            (void) hipEventDestroy(s.ev_in[i]);
            (void) hipEventDestroy(s.ev_red[i]);
            (void) hipEventDestroy(s.ev_out[i]);
        }
        s.copy_in = s.copy_out = nullptr;
    }
    if (s.phase_ev[0])
        for (hipEvent_t &e : s.phase_ev) {
            (void) hipEventDestroy(e);
            e = nullptr;
        }
    s.phase_events = s.phase_recorded = false;
    (void) hipFree(s.heap);
    (void) hipFree(s.flags);
    (void) hipHostFree(s.err_host);
    (void) hipFree(s.dctx);
    for (int t = 0; t < kMaxTeams; ++t) {
        release_team_mem(s, t);
        s.teams[t] = Team{};
    }
    release_team_pool(s);
    (void) hipFree(s.dev_epochs);
    (void) hipFree(s.kern_ep);
    s.kern_ep = nullptr;
    if (s.order_ev) (void) hipEventDestroy(s.order_ev);
    if (s.staging_ev) (void) hipEventDestroy(s.staging_ev);
    s.order_ev = s.staging_ev = nullptr;
    s.staging_used = false;
    s.last_stream = nullptr;
    s.last_stream_set = false;
    s.dctx = nullptr;
    s.dev_epochs = nullptr;
    s.heap = nullptr;
    s.flags = nullptr;
    s.err_host = s.err_dev = nullptr;
    s.exch_host = s.exch_dev = nullptr;
    s.done_host = s.done_dev = nullptr;
    s.initialized = false;
    return 0;
}

int ishmemi_c_initialized(void) { return S().initialized ? 1 : 0; }

int ishmemi_c_register_device_ctx_slot(const void *host_shadow)
{
    if (!host_shadow) return 0;
    {
        CtxSlots &c = ctx_slots();
        std::lock_guard<std::mutex> lk(c.mu);
        c.shadows.push_back(host_shadow);
    }
    State &s = S();
    std::lock_guard<std::mutex> lk(s.mu);
    if (s.initialized) write_ctx_slot(host_shadow, s.dctx);  // a code object loaded after init
    return 0;
}

int ishmemi_c_init_thread(int requested, int *provided)
{
    // src/ishmem.cpp:409-419: always ISHMEM_THREAD_MULTIPLE (host calls are serialised here).
    (void) requested;
    const int r = ishmemi_c_init();
    if (provided) *provided = ISHMEMI_C_THREAD_MULTIPLE;
    return r;
}

int ishmemi_c_query_thread(int *provided)
{
    if (provided) *provided = ISHMEMI_C_THREAD_MULTIPLE;
    return S().initialized ? 0 : fail("query_thread: not initialized");
}
int ishmemi_c_my_pe(void) { return S().initialized ? S().pe : -1; }
int ishmemi_c_n_pes(void) { return S().initialized ? S().npes : -1; }
int ishmemi_c_device(void) { return S().initialized ? S().device : -1; }

void *ishmemi_c_align(size_t alignment, size_t size)
{
    State &s = S();
    void *p;
    {
        std::lock_guard<std::mutex> lk(s.mu);
        if (!s.initialized) {
            fail("ishmem_malloc: not initialized");
            return nullptr;
        }
        if (alignment & (alignment - 1)) {
            fail("ishmem_align: alignment must be a power of two");
            return nullptr;
        }
        p = heap_alloc(s, size, alignment ? alignment : kHeapAlign);
    }
    // Collective like the reference (barrier on every alloc, src/memory.cpp:234).
    if (s.npes > 1) {
        std::string err;
        if (s.boot.barrier(err)) fail(err);
    }
    return p;
}

void *ishmemi_c_malloc(size_t size) { return ishmemi_c_align(kHeapAlign, size); }

void *ishmemi_c_calloc(size_t count, size_t size)
{
    void *p = ishmemi_c_align(kHeapAlign, count * size);
    if (p && hipMemset(p, 0, count * size) != hipSuccess) {
        fail("ishmem_calloc: hipMemset failed");
        return nullptr;
    }
    return p;
}

void ishmemi_c_free(void *ptr)
{
    State &s = S();
    if (!s.initialized) return;
    (void) hipDeviceSynchronize();
    if (s.npes > 1) {  // src/memory.cpp:286: peers must be done with the buffer
        std::string err;
        s.boot.barrier(err);
    }
    std::lock_guard<std::mutex> lk(s.mu);
    heap_free(s, ptr);
}

void *ishmemi_c_ptr(const void *dest, int pe)
{
    State &s = S();
    if (!s.initialized) return nullptr;
    return translate(s, dest, pe);
}

int ishmemi_c_heap_info(void **base, size_t *size, size_t *used)
{
    State &s = S();
    std::lock_guard<std::mutex> lk(s.mu);
    if (base) *base = s.heap;
    if (size) *size = s.heap_size;
    if (used) {
        size_t u = 0;
        for (auto &kv : s.used) u += kv.second;
        *used = u;
    }
    return s.initialized ? 0 : 1;
}

int ishmemi_c_team_my_pe(int team)
{
    State &s = S();
    if (!s.initialized || team < 0 || team >= kMaxTeams || !s.teams[team].valid) return -1;
    return s.teams[team].my_idx;
}

int ishmemi_c_team_n_pes(int team)
{
    State &s = S();
    if (!s.initialized || team < 0 || team >= kMaxTeams || !s.teams[team].valid) return -1;
    return s.teams[team].size;
}

int ishmemi_c_team_translate_pe(int src_team, int src_pe, int dest_team)
{
    State &s = S();
    if (!s.initialized) return -1;
    if (src_team < 0 || src_team >= kMaxTeams || dest_team < 0 || dest_team >= kMaxTeams) return -1;
    const Team &a = s.teams[src_team], &b = s.teams[dest_team];
    if (!a.valid || !b.valid || src_pe < 0 || src_pe >= a.size) return -1;
    const int gpe = a.start + src_pe * a.stride;
    if (b.stride == 0) return -1;
    const int d = gpe - b.start;
    if (d % b.stride) return -1;
    const int idx = d / b.stride;
    return (idx >= 0 && idx < b.size) ? idx : -1;
}

int ishmemi_c_team_split_strided(int parent, int start, int stride, int size, int *new_team)
{
    // Collective over the parent team (src/teams.cpp:294-452).
    State &s = S();
    if (new_team) *new_team = ISHMEMI_C_TEAM_INVALID;
    uint64_t free_mask = 0;
    Team t;
    {
        std::lock_guard<std::mutex> lk(s.mu);
        if (!s.initialized) return fail("team_split_strided: not initialized");
        if (parent < 0 || parent >= kMaxTeams || !s.teams[parent].valid)
            return fail("team_split_strided: invalid parent team");
        const Team &pt = s.teams[parent];
        if (pt.my_idx < 0) return fail("team_split_strided: caller not in parent team");
        stride = (stride == 0 || size == 1) ? 1 : stride;  // teams.cpp:304
        const int gstart = pt.start + start * pt.stride;
        const int gstride = pt.stride * stride;
        const int gend = gstart + gstride * (size - 1);
        if (start < 0 || start >= pt.size || size <= 0 || size > pt.size || gstart < 0 ||
            gstart >= s.npes || gend < 0 || gend >= s.npes)  // teams.cpp:309-325
            return fail("team_split_strided: invalid <start, stride, size>");
        t.valid = true;
        t.start = gstart;
        t.stride = gstride;
        t.size = size;
        const int d = s.pe - gstart;
        t.my_idx = (d % gstride == 0 && d / gstride >= 0 && d / gstride < size) ? d / gstride : -1;
        t.colocated = team_colocated(s, t);
        for (int i = kPredefTeams; i < s.teams_max; ++i)
            if (!s.teams[i].valid) free_mask |= 1ull << i;
    }
    const Team pt = s.teams[parent];
    // Agree on a slot free on every parent member: AND-reduce the free masks over the parent
    // team with the library's own reduction (the reference's bit reduction, teams.cpp:327-345).
    if (hipMemcpy(s.team_scratch, &free_mask, 8, hipMemcpyHostToDevice) != hipSuccess)
        return fail("team_split_strided: mask copy failed");
    if (ishmemi_c_reduce(parent, ISHMEMI_OP_AND, ISHMEMI_DT_UINT64, s.team_scratch, s.team_scratch, 1))
        return 1;
    if (hipMemcpy(&free_mask, s.team_scratch, 8, hipMemcpyDeviceToHost) != hipSuccess)
        return fail("team_split_strided: mask copy failed");
    if (!free_mask)  // the same outcome on every parent member (src/teams.cpp:369-371)
        return fail("team_split_strided: no more teams available (max = " + std::to_string(s.teams_max) +
                    "), try increasing ISHMEM_TEAMS_MAX");
    const int slot = __builtin_ctzll(free_mask);
    // The new team's flag block and ring (round 6: per team, not reserved at init).  Every member
    // allocates one of the kind agreed at init and exports it; the parent exchanges the handles
    // (an fcollect of one record per parent member through the symmetric team scratch: members
    // outside the new team send an empty record); each member opens its co-members' blocks.  Both
    // outcomes are agreed over the parent (AND-reduce), so a failure on one member fails the split
    // on all of them, with nothing left allocated.  The dma-buf import needs the exporter's ptrace
    // consent (pidfd_getfd under Yama), given for the exchange only, as at init.
    struct PtracerWindow {
        PtracerWindow() { prctl(PR_SET_PTRACER, PR_SET_PTRACER_ANY, 0, 0, 0); }
        ~PtracerWindow() { prctl(PR_SET_PTRACER, 0, 0, 0, 0); }
    } ptracer_window;
    struct SplitRec {
        uint32_t ok, kind;
        uint64_t bytes;
        uint32_t pool_idx, pad;
        hipIpcMemHandle_t handle;
    };
    static_assert(sizeof(SplitRec) <= kSplitRecBytes && kSplitRecBytes * kMaxPes + 256 <= kTeamScratchBytes,
                  "split exchange layout");
    const bool needs_mem = t.my_idx >= 0 && t.size > 1;
    uint32_t *block = nullptr;
    int pidx = -1;  // this PE's pool block for the new team
    SplitRec mine{};
    std::string why;
    auto agree = [&](bool ok_here) -> int {  // AND over the parent; -1 if the reduce itself failed
        uint64_t v = ok_here ? 1 : 0;
        if (hipMemcpy(s.team_scratch, &v, 8, hipMemcpyHostToDevice) != hipSuccess) return -1;
        if (ishmemi_c_reduce(parent, ISHMEMI_OP_AND, ISHMEMI_DT_UINT64, s.team_scratch, s.team_scratch, 1)) return -1;
        if (hipMemcpy(&v, s.team_scratch, 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
        return v ? 1 : 0;
    };
    bool ok = true;
    if (needs_mem) {
        std::lock_guard<std::mutex> lk(s.mu);
        for (size_t i = 0; i < s.team_pool.size() && pidx < 0; ++i)
            if (!s.team_pool[i].in_use) pidx = (int) i;
        if (pidx >= 0) {
            // A pooled block still holds its last team's epochs: zero it before its handle goes
            // out (the new team's launch words restart at 0, so an old epoch could read as arrived).
            PoolBlock &b = s.team_pool[(size_t) pidx];
            if (hipMemset(b.ptr, 0, kTeamAllocBytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
                (void) hipGetLastError();
                ok = false;
                why = "team block reset failed";
            }
        } else {
            PoolBlock b;
            int kind = -1;
            if (alloc_flag_mem(s, kTeamAllocBytes, s.flags_kind, true, s.npes > 1, &b.handle, &b.ptr, &kind,
                               "team_split_strided")) {
                ok = false;
                why = g_last_error;
            } else {
                s.team_pool.push_back(b);
                pidx = (int) s.team_pool.size() - 1;
            }
        }
        if (ok && alloc_fold_scratch(s, slot, t.size)) {
            ok = false;
            why = g_last_error;
        }
        if (pidx >= 0) {
            PoolBlock &b = s.team_pool[(size_t) pidx];
            b.in_use = true;
            block = b.ptr;
            mine.handle = b.handle;
            mine.pool_idx = (uint32_t) pidx;
        }
        if (ok) {
            mine.ok = 1;
            mine.kind = (uint32_t) s.flags_kind;
            mine.bytes = kTeamAllocBytes;
        }
    }
    auto undo = [&]() {  // back to the state before the split (peers' mappings stay cached)
        std::lock_guard<std::mutex> lk(s.mu);
        TeamMem &m = s.tmem[slot];
        if (pidx >= 0) s.team_pool[(size_t) pidx].in_use = false;
        if (m.fold_scratch) (void) hipFree(m.fold_scratch);
        m = TeamMem{};
        block = nullptr;
    };
    char *rec_src = s.team_scratch + 64, *rec_dst = s.team_scratch + 256;
    if (hipMemcpy(rec_src, &mine, sizeof(mine), hipMemcpyHostToDevice) != hipSuccess ||
        ishmemi_c_fcollect(parent, rec_dst, rec_src, kSplitRecBytes)) {
        undo();  // a local failure of the exchange itself: the peers time out in it and report it
        return fail("team_split_strided: handle exchange failed: " + std::string(g_last_error));
    }
    std::vector<SplitRec> recs((size_t) pt.size);
    {
        std::vector<char> raw((size_t) pt.size * kSplitRecBytes);
        if (hipMemcpy(raw.data(), rec_dst, raw.size(), hipMemcpyDeviceToHost) != hipSuccess) ok = false;
        for (int i = 0; i < pt.size; ++i) memcpy(&recs[(size_t) i], raw.data() + (size_t) i * kSplitRecBytes, sizeof(SplitRec));
    }
    if (needs_mem && ok) {
        std::lock_guard<std::mutex> lk(s.mu);
        TeamMem &m = s.tmem[slot];
        for (int j = 0; j < t.size && ok; ++j) {
            const int gpe = t.start + j * t.stride;
            const SplitRec &r = recs[(size_t) ((gpe - pt.start) / pt.stride)];
            if (!r.ok || r.kind != (uint32_t) s.flags_kind || r.bytes != kTeamAllocBytes) {
                ok = false;
                why = "member " + std::to_string(gpe) + " could not allocate its team block";
                break;
            }
            void *p = block;
            if (gpe != s.pe) {
                const auto key = std::make_pair(gpe, r.pool_idx);
                auto it = s.peer_pool.find(key);
                if (it != s.peer_pool.end()) {
                    p = it->second;  // mapped by an earlier split that used the same peer block
                } else if (hipIpcOpenMemHandle(&p, r.handle, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
                    (void) hipGetLastError();
                    ok = false;
                    why = "hipIpcOpenMemHandle of member " + std::to_string(gpe) + "'s team block failed" + ipc_hint();
                    break;
                } else {
                    s.peer_pool[key] = p;
                }
            }
            m.flags[gpe] = (uint32_t *) p;
            m.ring[gpe] = (uint64_t *) ((char *) p + kTeamLLOffset);
        }
    }
    const int agreed = agree(ok);
    if (agreed != 1) {
        undo();
        return fail("team_split_strided: the new team's flag blocks could not be set up on every member" +
                    (why.empty() ? std::string() : " (" + why + ")"));
    }
    {
        std::lock_guard<std::mutex> lk(s.mu);
        // Only members hold the slot.  A later team that reuses it on a non-member is disjoint
        // from this team (every member of this one has the slot reserved, so the AND-reduced
        // mask of any parent containing one of them excludes it).
        if (t.my_idx >= 0) {
            s.teams[slot] = t;
            s.tmem[slot].pool_idx = pidx;
            if (pidx >= 0) s.team_block_bytes += kTeamAllocBytes;
        }
        // Launch words and device-API rows of the slot: zero them locally, then the parent sync
        // below orders the zeroing before any member's first collective on the new team (the
        // block itself was zeroed before it was exported).
        if (hipMemset(dev_flags(s.flags) + (size_t) slot * kDevFlagWordsPerTeam, 0, kDevFlagWordsPerTeam * 4) != hipSuccess ||
            hipMemset(s.dev_epochs + slot, 0, sizeof(uint32_t)) != hipSuccess ||
            hipMemset(s.kern_ep + (size_t) kEpTeamWords * slot, 0, kEpTeamWords * sizeof(uint32_t)) != hipSuccess)
            return fail("team_split_strided: flag reset failed");
        if (sync_device_ctx(s)) return 1;
        if (hipDeviceSynchronize() != hipSuccess) return fail("team_split_strided: sync failed");
    }
    if (ishmemi_c_team_sync(parent)) return 1;
    if (new_team && t.my_idx >= 0) *new_team = slot;
    return 0;
}

int ishmemi_c_team_split_2d(int parent, int xrange, int *xaxis_team, int *yaxis_team)
{
    // src/teams.cpp:453-518: x-axis teams are contiguous groups of xrange parent PEs, y-axis
    // teams take every xrange-th parent PE; both are split_strided calls over the parent.
    State &s = S();
    if (xaxis_team) *xaxis_team = ISHMEMI_C_TEAM_INVALID;
    if (yaxis_team) *yaxis_team = ISHMEMI_C_TEAM_INVALID;
    if (!s.initialized) return fail("team_split_2d: not initialized");
    if (parent < 0 || parent >= kMaxTeams || !s.teams[parent].valid)
        return fail("team_split_2d: invalid parent team");
    if (xrange < 1) return fail("team_split_2d: xrange must be >= 1");
    const int psize = s.teams[parent].size;
    if (xrange > psize) xrange = psize;
    const int nx = (psize + xrange - 1) / xrange, ny = xrange;
    int start = 0;
    for (int i = 0; i < nx; ++i, start += xrange) {
        const int xsize = (i == nx - 1 && psize % xrange) ? psize % xrange : xrange;
        int t = ISHMEMI_C_TEAM_INVALID;
        if (ishmemi_c_team_split_strided(parent, start, 1, xsize, &t)) return 1;
        if (t != ISHMEMI_C_TEAM_INVALID && xaxis_team) *xaxis_team = t;
    }
    for (int i = 0; i < ny; ++i) {
        const int rem = psize % xrange, yr = psize / xrange;
        const int ysize = (rem && i < rem) ? yr + 1 : yr;
        int t = ISHMEMI_C_TEAM_INVALID;
        if (ishmemi_c_team_split_strided(parent, i, xrange, ysize, &t)) return 1;
        if (t != ISHMEMI_C_TEAM_INVALID && yaxis_team) *yaxis_team = t;
    }
    return 0;
}

int ishmemi_c_team_get_config(int team, long config_mask, int *num_contexts)
{
    // src/teams.cpp:545-570: mask 0 reports nothing; mask ISHMEM_TEAM_NUM_CONTEXTS needs the pointer.
    State &s = S();
    std::lock_guard<std::mutex> lk(s.mu);
    if (!s.initialized) return fail("team_get_config: not initialized");
    if (team < 0 || team >= kMaxTeams || !s.teams[team].valid) return fail("team_get_config: invalid team");
    if (config_mask == 0) return 0;
    if (config_mask != 1) return fail("team_get_config: invalid config mask");
    if (!num_contexts) return fail("team_get_config: NULL config with a nonzero mask");
    *num_contexts = s.teams[team].num_contexts;
    return 0;
}

int ishmemi_c_team_set_config(int team, long config_mask, int num_contexts)
{
    State &s = S();
    std::lock_guard<std::mutex> lk(s.mu);
    if (!s.initialized) return fail("team_set_config: not initialized");
    if (team < 0 || team >= kMaxTeams || !s.teams[team].valid) return fail("team_set_config: invalid team");
    if (config_mask != 0 && config_mask != 1) return fail("team_set_config: invalid config mask");
    if (config_mask) s.teams[team].num_contexts = num_contexts;
    return 0;
}

void ishmemi_c_team_destroy(int team)
{
    State &s = S();
    std::lock_guard<std::mutex> lk(s.mu);
    if (team <= ISHMEMI_C_TEAM_NODE || team >= kMaxTeams) return;
    // Local, as in the reference (src/teams.cpp:259-275): the slot is free again on this PE, and
    // the team's memory goes with it — the co-members' blocks mapped here are closed and this PE's
    // own block freed (after this PE's kernels are done with it; a co-member that still maps it
    // keeps the memory alive until it destroys the team too).
    if (s.initialized) {
        s.teams[team] = Team{};
        release_team_mem(s, team);
        sync_device_ctx(s);
    }
}

int ishmemi_c_team_sync(int team)
{
    State &s = S();
    std::lock_guard<std::mutex> lk(s.mu);
    if (!s.initialized) return fail("team_sync: not initialized");
    if (team < 0 || team >= kMaxTeams || !s.teams[team].valid) return fail("team_sync: invalid team");
    if (s.teams[team].my_idx < 0) return fail("team_sync: caller not in team");
    if (team_sync_locked(s, team, 0, nullptr) || mark_stream(s, 0)) return 1;
    if (host_wait(s, 0)) return 1;
    return check_team_errors(s, team);
}

int ishmemi_c_sync_all(void) { return ishmemi_c_team_sync(ISHMEMI_C_TEAM_WORLD); }

int ishmemi_c_team_sync_on_stream(int team, int *ret, void *stream)
{
    // ishmemx_team_sync_on_queue / sync_all_on_queue / barrier_all_on_queue (src/ishmemx.h:2228-2235):
    // the team barrier kernel enqueued on `stream` (stream order completes everything before it).
    State &s = S();
    std::lock_guard<std::mutex> lk(s.mu);
    if (!member_call(s, team)) return fail("team_sync_on_stream: not initialized, invalid team or caller not a member");
    hipStream_t st = (hipStream_t) stream;
    if (ret) HIP_TRY(hipMemsetAsync(ret, 0, sizeof(int), st));
    if (team_sync_locked(s, team, st, ret)) return 1;
    return mark_stream(s, st);
}

int ishmemi_c_barrier_all(void)
{
    // ishmem_barrier_all = quiet + sync_all: complete all outstanding device work first.
    if (hipDeviceSynchronize() != hipSuccess) return fail("barrier_all: device sync failed");
    return ishmemi_c_team_sync(ISHMEMI_C_TEAM_WORLD);
}

int ishmemi_c_resync(void)
{
    // After a device-side timeout the members of a team disagree on its epoch (a PE that timed
    // out advanced, a PE that never arrived did not), so every later collective of the team would
    // time out too.  The reference aborts the job instead (src/proxy.cpp:79-84).  Here every PE,
    // with no collective of its own in flight, agrees on the wrap-safe maximum of every team's
    // epochs (host and device-API launches) over the bootstrap; every flag row and ring granule
    // then holds an epoch <= the new one, so the next launch starts clean on every member.
    State &s = S();
    std::lock_guard<std::mutex> lk(s.mu);
    if (!s.initialized) return fail("resync: not initialized");
    HIP_TRY(hipDeviceSynchronize());
    struct Epochs {
        uint32_t host[kMaxTeams], dev[kMaxTeams];
    } mine{}, all[kMaxPes];
    static_assert(sizeof(Epochs) <= ShmBootstrap::kSlotBytes, "resync exchange");
    std::vector<uint32_t> words((size_t) kMaxTeams * kEpTeamWords);
    HIP_TRY(hipMemcpy(words.data(), s.kern_ep, words.size() * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(mine.dev, s.dev_epochs, sizeof(mine.dev), hipMemcpyDeviceToHost));
    for (int t = 0; t < kMaxTeams; ++t) mine.host[t] = words[(size_t) t * kEpTeamWords + kEpEpoch];
    if (s.npes > 1) {
        std::string err;
        if (s.boot.allgather(&mine, all, sizeof(Epochs), err)) return fail("resync: " + err);
    } else {
        all[0] = mine;
    }
    auto newest = [](uint32_t a, uint32_t b) { return (int32_t) (b - a) > 0 ? b : a; };
    for (int t = 0; t < kMaxTeams; ++t) {
        uint32_t h = all[0].host[t], d = all[0].dev[t];
        for (int j = 1; j < s.npes; ++j) {
            h = newest(h, all[j].host[t]);
            d = newest(d, all[j].dev[t]);
        }
        uint32_t *w = words.data() + (size_t) t * kEpTeamWords;
        for (int k = 0; k < kEpTeamWords; ++k) w[k] = 0;
        w[kEpEpoch] = h;
        for (int r = 0; r < kEpReplicas; ++r) w[(kEpRepLine + r) * kLineWords] = h;
        mine.dev[t] = d;
    }
    HIP_TRY(hipMemcpy(s.kern_ep, words.data(), words.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(s.dev_epochs, mine.dev, sizeof(mine.dev), hipMemcpyHostToDevice));
    for (int t = 0; t <= kMaxTeams; ++t) __atomic_store_n(&s.err_host[t], 0u, __ATOMIC_RELEASE);
    HIP_TRY(hipDeviceSynchronize());
    if (s.npes > 1) {
        std::string err;
        if (s.boot.barrier(err)) return fail("resync: " + err);
    }
    return 0;
}

int ishmemi_c_reduce(int team, int op, int dtype, void *dest, const void *source, size_t nreduce)
{
    return reduce_impl(team, op, dtype, dest, source, nreduce, nullptr, 0, true);
}

int ishmemi_c_reduce_on_stream(int team, int op, int dtype, void *dest, const void *source,
                               size_t nreduce, int *ret, void *stream)
{
    return reduce_impl(team, op, dtype, dest, source, nreduce, ret, (hipStream_t) stream, false);
}

int ishmemi_c_reduce_on_stream_deps(int team, int op, int dtype, void *dest, const void *source,
                                    size_t nreduce, int *ret, void *stream, void *const *deps,
                                    size_t ndeps, void *done)
{
    // The reference's `deps` (set_cmd_grp_dependencies, reduce_impl.h:452-453) become stream
    // waits ahead of the call's first launch; its returned sycl::event becomes `done`, recorded
    // after the call's last launch.  Stream order already gives what the reference's per-queue
    // "last on_queue event" dependency gives on an out-of-order queue.
    hipStream_t st = (hipStream_t) stream;
    if (ndeps && !deps) return fail("reduce_on_stream: deps is NULL with ndeps > 0");
    for (size_t i = 0; i < ndeps; ++i) {
        if (!deps[i]) return fail("reduce_on_stream: null dependency event");
        HIP_TRY(hipStreamWaitEvent(st, (hipEvent_t) deps[i], 0));
    }
    if (reduce_impl(team, op, dtype, dest, source, nreduce, ret, st, false)) return 1;
    if (done) HIP_TRY(hipEventRecord((hipEvent_t) done, st));
    return 0;
}

int ishmemi_c_stream_wait_events(void *stream, void *const *deps, size_t ndeps)
{
    if (ndeps && !deps) return fail("stream_wait_events: deps is NULL with ndeps > 0");
    for (size_t i = 0; i < ndeps; ++i) {
        if (!deps[i]) return fail("stream_wait_events: null dependency event");
        HIP_TRY(hipStreamWaitEvent((hipStream_t) stream, (hipEvent_t) deps[i], 0));
    }
    return 0;
}

int ishmemi_c_stream_record_event(void *stream, void *done)
{
    if (done) HIP_TRY(hipEventRecord((hipEvent_t) done, (hipStream_t) stream));
    return 0;
}

int ishmemi_c_combine(int op, int dtype, void *dst, const void *const *srcs, int nsrc, size_t n,
                      void *stream)
{
    if (!op_dtype_valid(op, dtype)) return fail("combine: invalid (op, dtype) pair");
    if (nsrc < 1 || nsrc > kMaxFanin) return fail("combine: nsrc must be 1..16");
    if (n == 0) return 0;
    if (!dst || !srcs) return fail("combine: null pointer");
    FaninArgs f{};
    for (int i = 0; i < nsrc; ++i) {
        if (!srcs[i]) return fail("combine: null source");
        f.src[i] = (const char *) srcs[i];
    }
    f.dst = (char *) dst;
    f.nsrc = nsrc;
    Plan pl;
    plan_fanin(f, pl, dst, srcs, nsrc, n, dtype_size(dtype));
    HIP_TRY(launch_fanin(op, dtype, pl.vec, f, pl.grid, (hipStream_t) stream));
    return 0;
}

int ishmemi_c_pull_probe(void *dst, const void *const *srcs, int nsrc, size_t nbytes, int policy,
                         void *stream)
{
    if (nsrc < 1 || nsrc > kMaxFanin) return fail("pull_probe: nsrc must be 1..16");
    if (!dst || !srcs || nbytes % 16 || ((uintptr_t) dst & 15))
        return fail("pull_probe: 16-B aligned pointers and a multiple of 16 bytes required");
    if (nbytes == 0) return 0;
    FaninArgs f{};
    for (int i = 0; i < nsrc; ++i) {
        if (!srcs[i] || ((uintptr_t) srcs[i] & 15)) return fail("pull_probe: misaligned or null source");
        f.src[i] = (const char *) srcs[i];
    }
    f.dst = (char *) dst;
    f.nsrc = nsrc;
    f.nitems = nbytes / 16;
    HIP_TRY(launch_pull_probe(f, policy ? 1 : 0, (hipStream_t) stream));
    return 0;
}

int ishmemi_c_produce_u32(void *dst, const void *a, const void *b, size_t n, void *stream)
{
    if (n && (!dst || !a || !b)) return fail("produce_u32: null pointer");
    if (((uintptr_t) dst | (uintptr_t) a | (uintptr_t) b) & 3) return fail("produce_u32: misaligned pointer");
    HIP_TRY(launch_produce_u32((uint32_t *) dst, (const uint32_t *) a, (const uint32_t *) b, n, (hipStream_t) stream));
    return 0;
}

int ishmemi_c_occupy(int grid, unsigned long long usec, void *stream)
{
    HIP_TRY(launch_occupy(grid, (uint64_t) usec, (hipStream_t) stream));
    return 0;
}

int ishmemi_c_fcollect(int team, void *dest, const void *source, size_t nbytes)
{
    // Members agree on the staged path (any member's source outside the heap: all stage) and on
    // argument failures before anything is launched.
    State &s = S();
    int staged = -1;
    if (member_call(s, team) && s.teams[team].size > 1 && nbytes > 0) {
        const uint64_t mine = (in_heap(s, source) ? 0 : kAgreeStaged) | (device_writable(s, dest) ? 0 : kAgreeFail);
        uint64_t all[kMaxPes], any = 0;
        if (team_exchange(team, mine, all)) return 1;
        for (int j = 0; j < s.teams[team].size; ++j) any |= all[j];
        if (any & kAgreeFail)
            return fail("fcollect: a member's dest is not device-writable (heap, device or pinned host memory)");
        staged = (any & kAgreeStaged) ? 1 : 0;
    }
    return fcollect_impl(team, dest, source, nbytes, nullptr, 0, true, staged);
}

int ishmemi_c_fcollect_on_stream(int team, void *dest, const void *source, size_t nbytes, int *ret,
                                 void *stream)
{
    return fcollect_impl(team, dest, source, nbytes, ret, (hipStream_t) stream, false);
}

int ishmemi_c_collect(int team, void *dest, const void *source, size_t nbytes)
{
    // Every member's byte count first (an fcollect of one u64 through the team scratch), then
    // the all-gather at the resulting offsets (src/collectives/collect_impl.h:36-50).
    State &s = S();
    if (!s.initialized) return fail("collect: not initialized");
    if (team < 0 || team >= kMaxTeams || !s.teams[team].valid || s.teams[team].my_idx < 0)
        return fail("collect: invalid team or caller not a member");
    const int p = s.teams[team].size;
    if (p == 1) return ishmemi_c_fcollect(team, dest, source, nbytes);
    // With the count: kAgreeStaged = that member's source is outside the heap (then every member
    // takes the staged path: peers' sources are only found from a symmetric source address);
    // kAgreeFail = its dest is not device-writable (then every member fails, nothing launched).
    const uint64_t mine = nbytes | (in_heap(s, source) ? 0 : kAgreeStaged) | (device_writable(s, dest) ? 0 : kAgreeFail);
    uint64_t counts[kMaxPes];
    if (team_exchange(team, mine, counts)) return 1;
    bool staged = false, failed = false;
    for (int j = 0; j < p; ++j) {
        staged = staged || (counts[j] & kAgreeStaged);
        failed = failed || (counts[j] & kAgreeFail);
        counts[j] &= ~(kAgreeStaged | kAgreeFail);
    }
    if (failed) return fail("collect: a member's dest is not device-writable (heap, device or pinned host memory)");
    std::lock_guard<std::mutex> lk(s.mu);
    if (staged) {
        if (order_stream(s, 0) || collect_staged(s, team, (char *) dest, (const char *) source, counts, nullptr, 0))
            return 1;
    } else if (collect_launch(s, team, dest, source, counts, nullptr, 0)) {
        return 1;
    }
    if (mark_stream(s, 0)) return 1;
    if (host_wait(s, 0)) return 1;
    return check_team_errors(s, team);
}

int ishmemi_c_collect_on_stream(int team, void *dest, const void *source, size_t nbytes, int *ret,
                                void *stream)
{
    return collect_on_stream_impl(team, dest, source, nbytes, ret, (hipStream_t) stream);
}

int ishmemi_c_scan(int team, int dtype, int inclusive, void *dest, const void *source, size_t nelems)
{
    // Buffers outside the heap (the reference proxies host buffers to MPI_Scan / MPI_Exscan,
    // runtime_mpi.cpp:816-835) go through symmetric temporaries, copied in / out around the device
    // scan.  The members first agree (team_exchange) whether ANY of them needs temporaries; if so
    // every member allocates both, in the same order, from an allocator in the same state (all
    // other allocations are collective), so the source temporaries sit at the same offset on
    // every member, which the scan kernel requires.  Callers serialise collectives per team, as in
    // the reference (src/teams.h:29-38).
    State &s = S();
    const size_t bytes = nelems * dtype_size(dtype);
    if (!member_call(s, team) || nelems == 0 || s.teams[team].size == 1 || !op_dtype_valid(ISHMEMI_OP_SUM, dtype))
        return scan_impl(team, dtype, inclusive, dest, source, nelems, nullptr, 0, true);
    const uint64_t mine = (in_heap(s, source) && in_heap(s, dest)) ? 0 : kAgreeStaged;
    uint64_t all[kMaxPes], any = 0;
    if (team_exchange(team, mine, all)) return 1;
    for (int j = 0; j < s.teams[team].size; ++j) any |= all[j];
    if (!(any & kAgreeStaged)) return scan_impl(team, dtype, inclusive, dest, source, nelems, nullptr, 0, true);
    char *ts, *td;
    {
        std::lock_guard<std::mutex> lk(s.mu);
        ts = (char *) heap_alloc(s, bytes, 256);
        td = (char *) heap_alloc(s, bytes, 256);
    }
    int rc = (!ts || !td) ? 1 : 0;  // the same outcome on every member (same allocator state)
    if (!rc && hipMemcpy(ts, source, bytes, hipMemcpyDefault) != hipSuccess) rc = fail("scan: staging copy-in failed");
    char *d = in_heap(s, dest) ? (char *) dest : td;
    if (!rc) rc = scan_impl(team, dtype, inclusive, d, ts, nelems, nullptr, 0, true);
    if (!rc && d != dest && hipMemcpy(dest, d, bytes, hipMemcpyDefault) != hipSuccess)
        rc = fail("scan: staging copy-out failed");
    std::lock_guard<std::mutex> lk(s.mu);
    if (td) heap_free(s, td);
    if (ts) heap_free(s, ts);
    return rc;
}

int ishmemi_c_broadcast_on_stream(int team, void *dest, const void *source, size_t nbytes, int root,
                                  int *ret, void *stream)
{
    // ishmemx_<TN>_broadcast_on_queue (src/ishmemx.h:846-954): nothing can be exchanged on the host
    // here, so the source is a symmetric address (the root's is found at the same offset of its
    // heap, as the reference requires of symmetric objects) and every member's dest must be
    // device-writable.
    State &s = S();
    std::lock_guard<std::mutex> lk(s.mu);
    if (!member_call(s, team)) return fail("broadcast_on_stream: not initialized, invalid team or caller not a member");
    const Team &t = s.teams[team];
    if (root < 0 || root >= t.size) return fail("broadcast_on_stream: root is not a team index");
    hipStream_t st = (hipStream_t) stream;
    if (ret) HIP_TRY(hipMemsetAsync(ret, 0, sizeof(int), st));
    if (t.size == 1) {
        if (nbytes && dest != source) {
            if (device_writable(s, dest) && classify(s, source) != Kind::Host) {
                if (launch_copy(dest, source, nbytes, st)) return 1;
            } else {
                HIP_TRY(hipMemcpyAsync(dest, source, nbytes, hipMemcpyDefault, st));
            }
        }
        return mark_stream(s, st);
    }
    if (nbytes == 0) return team_sync_locked(s, team, st, ret) || mark_stream(s, st);
    if (!in_heap(s, source)) return fail("broadcast_on_stream: source must be symmetric-heap memory");
    if (!device_writable(s, dest)) return fail("broadcast_on_stream: dest must be heap, device or pinned host memory");
    if (ll_eligible(s, t, dest, source, nbytes) && 2 * nbytes <= ll_capacity(t.size)) {
        // Small payloads (round 5): the root's bytes as granules into every member's ring, the
        // others one token each (kLLBroadcast) — no handshakes.  Dest is stored locally whatever
        // its kind, so every member decides alike from the byte count (round 6: the choice no
        // longer depends on this PE's dest being in the heap — ADVICE r05).
        if (reduce_ll(s, team, ISHMEMI_OP_OR, ISHMEMI_DT_UINT8, dest, source, nbytes, ret, st, kLLBroadcast, root)) return 1;
        return mark_stream(s, st);
    }
    uint64_t counts[kMaxPes] = {}, zero[kMaxPes] = {};
    counts[root] = nbytes;
    const char *srcs[kMaxPes];
    const char *rsrc = translate(s, source, t.start + root * t.stride);
    for (int j = 0; j < t.size; ++j) srcs[j] = rsrc;
    if (collect_launch(s, team, dest, nullptr, counts, ret, st, zero, srcs)) return 1;
    return mark_stream(s, st);
}

int ishmemi_c_broadcast(int team, void *dest, const void *source, size_t nbytes, int root)
{
    // The reference's intra-node pull (broadcast_impl.h: team sync, every member gets the root's
    // source, team sync) on the collect kernel: only the root contributes, every member's dest
    // receives it at offset 0.  The members exchange the root's source offset in the heap (its
    // source is found from it, whatever the others pass), whether it must be staged (outside the
    // heap) and any local argument failure, before anything is launched.
    State &s = S();
    if (!member_call(s, team)) return fail("broadcast: not initialized, invalid team or caller not a member");
    const int p = s.teams[team].size;
    if (root < 0 || root >= p) return fail("broadcast: root is not a team index");
    if (p == 1) {  // the root alone: dest = source, from or to any kind of memory
        if (nbytes && dest != source) HIP_TRY(hipMemcpy(dest, source, nbytes, hipMemcpyDefault));
        return 0;
    }
    const Team &t = s.teams[team];
    const bool me_root = t.my_idx == root;
    uint64_t mine = 0;
    if (me_root) mine = in_heap(s, source) ? (uint64_t) ((const char *) source - s.heap) : kAgreeStaged;
    if (nbytes && !device_writable(s, dest)) mine |= kAgreeFail;
    uint64_t all[kMaxPes], any = 0;
    if (team_exchange(team, mine, all)) return 1;
    for (int j = 0; j < p; ++j) any |= all[j];
    if (any & kAgreeFail) return fail("broadcast: a member's dest is not device-writable (heap, device or pinned host memory)");
    if (nbytes == 0) return ishmemi_c_team_sync(team);
    uint64_t counts[kMaxPes] = {}, zero[kMaxPes] = {};
    counts[root] = nbytes;
    std::lock_guard<std::mutex> lk(s.mu);
    if (!(all[root] & kAgreeStaged) && ll_eligible(s, t, dest, source, nbytes) && 2 * nbytes <= ll_capacity(p)) {
        // Small payloads, the root's source in the heap (agreed above): the granule broadcast
        // (kLLBroadcast); the root reads its own source, the others none, and every member
        // stores its own dest, of any device-writable kind.
        if (reduce_ll(s, team, ISHMEMI_OP_OR, ISHMEMI_DT_UINT8, dest, source, nbytes, nullptr, 0, kLLBroadcast, root))
            return 1;
    } else if (all[root] & kAgreeStaged) {
        if (order_stream(s, 0) || collect_staged(s, team, (char *) dest, (const char *) source, counts, nullptr, 0))
            return 1;
    } else {
        const char *srcs[kMaxPes];
        const int groot = t.start + root * t.stride;
        for (int j = 0; j < p; ++j) srcs[j] = s.peer_heap[groot] + all[root];
        if (collect_launch(s, team, dest, nullptr, counts, nullptr, 0, zero, srcs)) return 1;
    }
    if (mark_stream(s, 0)) return 1;
    if (host_wait(s, 0)) return 1;
    return check_team_errors(s, team);
}

int ishmemi_c_scan_on_stream(int team, int dtype, int inclusive, void *dest, const void *source,
                             size_t nelems, int *ret, void *stream)
{
    return scan_impl(team, dtype, inclusive, dest, source, nelems, ret, (hipStream_t) stream, false);
}

void *ishmemi_c_device_ctx(void)
{
    State &s = S();
    return s.initialized ? (void *) s.dctx : nullptr;
}

const char *ishmemi_c_last_error(void) { return g_last_error.c_str(); }

int ishmemi_c_phase_times(float *ms5)
{
    State &s = S();
    if (!ms5) return fail("phase_times: null output");
    if (!s.phase_recorded || !s.phase_ev[0]) return fail("phase_times: no phased reduce recorded (set_param phase_events 1)");
    HIP_TRY(hipEventSynchronize(s.phase_ev[5]));
    for (int k = 0; k < 5; ++k) HIP_TRY(hipEventElapsedTime(&ms5[k], s.phase_ev[k], s.phase_ev[k + 1]));
    return 0;
}

int ishmemi_c_set_param(const char *name, long long value)
{
    State &s = S();
    std::lock_guard<std::mutex> lk(s.mu);
    const std::string n = name ? name : "";
    if (n == "max_blocks") s.max_blocks = (int) std::min<long long>(kMaxBlocks, std::max<long long>(1, value));
    else if (n == "staged_copy_kernel") s.staged_copy_kernel = (int) (value & 3);
    else if (n == "wait_slots") {
        if (value < wait_slots_floor())
            return fail("set_param: wait_slots " + std::to_string(value) + " is below " +
                        std::to_string(wait_slots_floor()) + " (GPU_MAX_HW_QUEUES), see ISHMEM_WAIT_SLOTS");
        set_wait_slots((int) std::min<long long>(1 << 20, value));
    }
    else if (n == "timeout_ms") s.timeout_ms = std::max<long long>(1, value);
    else if (n == "stream_order") s.stream_order = value != 0;
    else if (n == "oneshot_p2_max_bytes") s.oneshot_p2 = std::max<long long>(0, value);
    else if (n == "phased_min_bytes") s.phased_min = value < 0 ? kPhasedOff : value;
    else if (n == "ll_max_bytes") s.ll_max_bytes = std::min<long long>((long long) kLLMaxBytes, std::max<long long>(0, value));
    else if (n == "debug") s.debug = (int) value;
    else if (n == "phased_peer_nt") s.phased_peer_nt = value != 0;
    else if (n == "xgmi_ll_max_bytes") s.xgmi_ll_max = std::max<long long>(-1, value);      // alike on every PE
    else if (n == "xgmi_fold_max_bytes") s.xgmi_fold_max = std::max<long long>(-1, value);  // alike on every PE
    else if (n == "xgmi_link_mbps") {
        if (value <= 0) return fail("set_param: xgmi_link_mbps must be positive");
        s.xgmi_link_bps = (double) value * 1e6;  // alike on every PE (the model's thresholds follow)
    }
    else if (n == "realign_grid_cap") set_realign_grid_cap((int) std::min<long long>(std::max<long long>(value, 0), 1 << 30));
    else if (n == "collect_realign") set_collect_realign((int) (value != 0));
    else if (n == "ar_shifted") s.ar_shifted = value != 0;  // measurement: set alike on every PE
    else if (n == "rs_xcd") s.rs_xcd = value != 0;          // measurement (local: no pairing)
    else if (n == "direct_p2") s.direct_p2 = value != 0;  // measurement: set alike on every PE
    else if (n == "direct_inplace") s.direct_inplace = value != 0;  // measurement: set alike on every PE
    else if (n == "block_spin") s.block_spin = (int) std::min<long long>(std::max<long long>(value, 0), 2);
    else if (n == "direct_max_pes") s.direct_max_pes = (int) std::min<long long>(std::max<long long>(value, 2), kMaxPes);
    else if (n == "phase_unaligned") set_phase_unaligned((int) (value != 0));
    else if (n == "trace_buffer") s.trace = (uint64_t *) (uintptr_t) value;
    else if (n == "phase_events") {
        if (value && !s.phase_ev[0])
            for (hipEvent_t &e : s.phase_ev) HIP_TRY(hipEventCreate(&e));
        s.phase_events = value != 0;
    }
    else return fail("set_param: unknown parameter " + n);
    return 0;
}

long long ishmemi_c_get_param(const char *name)
{
    State &s = S();
    const std::string n = name ? name : "";
    if (n == "max_blocks") return s.max_blocks;
    if (n == "staged_copy_kernel") return s.staged_copy_kernel;
    if (n == "wait_slots") return wait_slots();
    if (n == "timeout_ms") return s.timeout_ms;
    if (n == "stream_order") return s.stream_order ? 1 : 0;
    if (n == "oneshot_p2_max_bytes") return s.oneshot_p2;
    if (n == "phased_min_bytes") return s.phased_min == kPhasedOff ? -1 : s.phased_min;
    if (n == "ll_max_bytes") return s.ll_max_bytes;
    if (n == "ll_capacity_bytes") return (long long) ll_capacity(s.npes);  // TEAM_WORLD's ring capacity
    // TEAM_WORLD's thresholds (path_limits: by its topology, co-located or across GPUs).
    if (n == "ll_limit_bytes") return team_limits(s, s.teams[0]).ll;
    if (n == "fold_limit_bytes") return team_limits(s, s.teams[0]).fold;
    if (n == "team_colocated") return s.teams[0].colocated ? 1 : 0;
    if (n == "xgmi_ll_max_bytes") return s.xgmi_ll_max;
    if (n == "xgmi_fold_max_bytes") return s.xgmi_fold_max;
    if (n == "xgmi_link_mbps") return (long long) (s.xgmi_link_bps / 1e6);
    if (n == "teams_max") return s.teams_max;
    // Flag memory this PE holds (base block + the split teams' blocks), against round 5's fixed
    // 16-slot block ("flag_block_bytes_round5").
    if (n == "flag_block_bytes") return s.initialized ? (long long) (kBaseAllocBytes + s.team_block_bytes) : 0;
    // Team blocks this PE holds in its pool, in use or free for the next split (PoolBlock).
    if (n == "flag_block_pool_bytes") return (long long) (s.team_pool.size() * kTeamAllocBytes);
    if (n == "flag_block_bytes_round5") return (long long) kRound5FlagBytes;
    for (int k = 0; k < 8; ++k)
        if (n == std::string("init_us_") + kInitPhase[k]) return (long long) s.init_us[k];
    if (n == "debug") return s.debug;
    if (n == "phased_peer_nt") return s.phased_peer_nt;
    if (n == "realign_grid_cap") return realign_grid_cap();
    if (n == "collect_realign") return collect_realign();
    if (n == "ar_shifted") return s.ar_shifted;
    if (n == "rs_xcd") return s.rs_xcd;
    if (n == "direct_p2") return s.direct_p2;
    if (n == "direct_inplace") return s.direct_inplace;
    if (n == "block_spin") return s.block_spin;
    if (n == "direct_max_pes") return s.direct_max_pes;
    if (n == "phase_unaligned") return phase_unaligned();
    if (n == "flags_fine_grained") return s.flags_kind != kFlagsCoarse ? 1 : 0;
    if (n == "flags_kind") return s.flags_kind;
    if (n == "staging_bytes") return (long long) s.staging_bytes;
    if (n == "staging_slots") return s.staging_slots;
    if (n == "heap_bytes") return (long long) s.heap_size;
    if (n == "device_share") return device_share();  // PEs of the job on this PE's device
    if (n == "launch_words") return (long long) (uintptr_t) s.kern_ep;  // debug: device address
    if (n == "cu_count") {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
            (void) hipGetLastError();
            return -1;
        }
        return cus;
    }
    return -1;
}

int ishmemi_c_error_count(void)
{
    // Errors already reported by blocking calls, plus error words the device has set since and no
    // blocking call has collected yet (stream-ordered collectives and the device API).
    State &s = S();
    int pending = 0;
    if (s.err_host)
        for (int t = 0; t <= kMaxTeams; ++t)
            pending += __atomic_load_n(&s.err_host[t], __ATOMIC_ACQUIRE) != 0;
    return s.error_count + pending;
}

size_t ishmemi_c_dtype_size(int dtype)
{
    return (dtype >= 0 && dtype < ISHMEMI_DT_COUNT) ? dtype_size(dtype) : 0;
}

int ishmemi_c_op_dtype_valid(int op, int dtype) { return op_dtype_valid(op, dtype) ? 1 : 0; }

int ishmemi_c_chunk_bounds(uint64_t nitems, int npes, int c, uint64_t *begin, uint64_t *end)
{
    if (npes < 1 || c < 0 || c >= npes || !begin || !end) return 1;
    const uint64_t ipc = npes > 1 ? items_per_chunk(nitems, npes) : nitems;
    *begin = std::min<uint64_t>((uint64_t) c * ipc, nitems);
    *end = std::min<uint64_t>(*begin + ipc, nitems);
    return 0;
}

int ishmemi_c_path_limits(int npes, int colocated, long long *ll_limit, long long *fold_limit)
{
    if (npes < 1 || npes > kMaxPes || !ll_limit || !fold_limit) return fail("path_limits: invalid arguments");
    State &s = S();
    std::lock_guard<std::mutex> lk(s.mu);
    const PathLimits r = path_limits(s, npes, colocated != 0);
    *ll_limit = r.ll;
    *fold_limit = r.fold;
    return 0;
}

int ishmemi_c_bootstrap_selftest(int pe, int npes, const char *key, int value, int *out)
{
    ShmBootstrap b;
    std::string err;
    if (b.attach(pe, npes, key ? key : "selftest", 20000, err)) return fail(err);
    if (b.allgather(&value, out, sizeof(int), err)) return fail(err);
    if (b.barrier(err)) return fail(err);
    return 0;
}

const char *ishmemi_c_version(void) { return "ishmem_amd 0.1.0 (reduction path; ref ishmem 1.5.1)"; }

}  // extern "C"
