// ishmem_amd — kernel launch interface (host side of the HIP kernels in kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "types.h"

namespace ishmemi {

// One node of MI355X has 8 GPUs; 16 leaves room for several PEs per GPU (tests run 2-4 PEs
// on one device).  The reference caps node-local PEs at 64 (src/ishmem/util.h:29).
constexpr int kMaxPes = 16;
// Upper bound of workgroups per collective launch; flag arrays are sized from it.
constexpr int kMaxBlocks = 1024;
// Barrier phases of one collective (start, mid, end) + a standalone team-sync phase.
constexpr int kPhases = 4;
constexpr int kPhaseStart = 0, kPhaseMid = 1, kPhaseEnd = 2, kPhaseSync = 3;
// Per-team flag block: [phase][block][pe] uint32 epochs, then an error word.
constexpr size_t kFlagWordsPerTeam = (size_t) kPhases * kMaxBlocks * kMaxPes;
constexpr size_t kTeamFlagBytes = kFlagWordsPerTeam * 4 + 256;
constexpr int kBlock = 256;  // 4 waves of 64
constexpr int kUnroll = 4;   // items in flight per thread per source (allreduce tiles)
constexpr int kFaninBlock = 64;  // local combine: one wave, one 16-B item per thread, one-shot grid
// AQL grid sizes count work-items in 32 bits: cap the one-shot grid at 2^31 work-items; larger
// arrays (> 32 GiB of 16-B items) take the kernel's grid-stride loop.
constexpr int kFaninMaxGrid = (int) ((1ull << 31) / kFaninBlock);

// Arguments of the multi-PE reduce-scatter + all-gather kernel.  All pointers are already
// translated into this process's address space (own heap or IPC-mapped peer heap).
struct ReduceArgs {
    const char *src[kMaxPes];   // member j's source (element 0), j in team order
    const char *dstp[kMaxPes];  // member j's dest (element 0), for all-gather pulls
    char *dst;                  // own dest (element 0)
    uint32_t *my_flags;         // own team flag block (fine-grained, written by peers)
    uint32_t *peer_flags[kMaxPes];
    uint32_t *err;  // own error word
    int *ret;       // optional user status word (ishmemx_*_on_stream), may be null
    uint64_t head;  // scalar elements before the 16-B aligned body (vector mode)
    uint64_t nitems;  // body items (16-B vectors in vector mode, elements in scalar mode)
    uint64_t tail;    // scalar elements after the body
    uint64_t items_per_chunk;
    uint64_t timeout_ticks;  // s_memrealtime ticks (100 MHz)
    int oneshot;  // 1: every member folds the WHOLE array (no mid barrier, no all-gather)
    uint32_t *ep_ctr;  // team's kernel-epoch counter: [0] last epoch, [1] workgroups done
    int p, me;
};

// Small-message ("LL") path: 8-byte granules {4 data bytes | 32-bit epoch} pushed into every
// peer's fine-grained receive ring; [parity 2][sender kMaxPes][kLLGranules] u64 per team.
constexpr size_t kLLMaxBytes = 65536;                 // LL ring capacity: payload bytes per PE
constexpr size_t kLLDefaultBytes = 65536;             // default LL threshold (ISHMEM_LL_MAX_BYTES)
constexpr size_t kLLGranules = kLLMaxBytes / 4;       // 4 payload bytes per granule
constexpr size_t kLLTeamBytes = (size_t) 2 * kMaxPes * kLLGranules * 8;  // 4 MiB
struct LLArgs {
    const char *src;
    char *dst;
    uint64_t *my_ring;              // this team's ring base on this PE (parity 0, sender 0)
    uint64_t *peer_ring[kMaxPes];   // the same ring base on every member, mapped here
    uint32_t *err;
    int *ret;
    uint64_t nbytes;
    uint64_t timeout_ticks;
    uint32_t *ep_ctr;  // team's kernel-epoch counter: [0] last epoch, [1] workgroups done
    int p, me;
};
hipError_t launch_ll(int op, int dt, const LLArgs &a, hipStream_t s);

// fcollect / collect (all-gather of the members' sources): member j's bytes land at
// dst + dst_off[j].  Same pairwise barriers as the reduce (start, end).
struct CollectArgs {
    const char *src[kMaxPes];  // member j's source, mapped here
    char *dst;
    uint64_t dst_off[kMaxPes];
    uint64_t nbytes[kMaxPes];
    uint32_t *my_flags;
    uint32_t *peer_flags[kMaxPes];
    uint32_t *err;
    int *ret;
    uint64_t timeout_ticks;
    uint32_t *ep_ctr;  // team's kernel-epoch counter: [0] last epoch, [1] workgroups done
    int p, me;
    int unit;  // bytes per item: 16, 4 or 1 (largest dividing every address and length)
};
hipError_t launch_collect(const CollectArgs &a, int grid, hipStream_t s);

// Inclusive / exclusive prefix sum across the team (MPI_Scan / MPI_Exscan semantics).
struct ScanArgs {
    const char *src[kMaxPes];      // member j's source
    const char *scratch[kMaxPes];  // member j's scratch (staging region), mapped here
    char *dst;
    uint32_t *my_flags;
    uint32_t *peer_flags[kMaxPes];
    uint32_t *err;
    int *ret;
    uint64_t nelems, items_per_chunk;
    uint64_t timeout_ticks;
    uint32_t *ep_ctr;  // team's kernel-epoch counter: [0] last epoch, [1] workgroups done
    int p, me;
    int inclusive;
};
hipError_t launch_scan(int dt, const ScanArgs &a, bool vec, int grid, hipStream_t s);

// Arguments of the local k-input fan-in combine: dst = op(src0, src1, ..., src_{k-1}).
constexpr int kMaxFanin = 16;
struct FaninArgs {
    const char *src[kMaxFanin];
    char *dst;
    uint64_t head, nitems, tail;
    int nsrc;
};

// Returns hipSuccess or a launch error.  `vec` selects the 16-B vector body (all operands
// share the same address residue mod 16) or the element-granular path.
hipError_t launch_allreduce(int op, int dt, bool vec, const ReduceArgs &a, int grid,
                            hipStream_t s);
hipError_t launch_fanin(int op, int dt, bool vec, const FaninArgs &a, int grid, hipStream_t s);
hipError_t launch_team_sync(const ReduceArgs &a, hipStream_t s);
// xGMI measurement hook: dst = sum of a.nsrc f32 arrays (a.nitems 16-B items), source loads with
// cache policy 0 = nt, 1 = sc0 sc1.
hipError_t launch_pull_probe(const FaninArgs &a, int policy, hipStream_t s);

}  // namespace ishmemi
