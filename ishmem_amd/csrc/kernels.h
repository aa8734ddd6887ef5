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
// Flag rows of one team, [phase][slot][pe] u32 epochs written by peers into this PE's block:
//   kPhaseStart, slot 0 - member pe's launch has started (its source is final);
//   kPhaseMid, slot s   - member pe's reduced segment s (or, for a scan, all of its chunk) is
//                         stored and readable;
//   kPhaseEnd, slot 0   - member pe has finished every read of this PE's memory;
//   kPhaseSync, slot 0  - standalone team barrier.
// A launch never pairs its workgroups with a peer's: any workgroup may satisfy a start flag,
// segments are grabbed from a per-launch work counter, and only the launch's last workgroup
// waits for the peers' end flags, so progress never depends on which workgroups are resident.
constexpr int kPhases = 4;
constexpr int kPhaseStart = 0, kPhaseMid = 1, kPhaseEnd = 2, kPhaseSync = 3;
// Per-team flag block: [phase][slot][pe] uint32 epochs, then an error word.
constexpr size_t kFlagWordsPerTeam = (size_t) kPhases * kMaxBlocks * kMaxPes;
constexpr size_t kTeamFlagBytes = kFlagWordsPerTeam * 4 + 256;
constexpr int kBlock = 256;  // 4 waves of 64
constexpr int kUnroll = 4;   // items in flight per thread per source (allreduce tiles)
constexpr int kFaninBlock = 64;  // local combine: one wave, one 16-B item per thread, one-shot grid
// AQL grid sizes count work-items in 32 bits: cap the one-shot grid at 2^31 work-items; larger
// arrays (> 32 GiB of 16-B items) take the kernel's grid-stride loop.
constexpr int kFaninMaxGrid = (int) ((1ull << 31) / kFaninBlock);

// Per-team launch words (device memory, kEpTeamWords u32 per team; `ep_ctr` in the argument
// structs points at the team's first word).  Line 0 (16 words) holds the kEp* words below; all
// are zero between launches except kEpEpoch; the launch's last workgroup resets the others.
// Words read or updated by every workgroup of a launch are spread over 64-B lines of their own,
// so hundreds of workgroups never queue on one line (MI355X_MICROARCH.md: a counter with 255
// arrivals costs ~3.3 us; sharded per XCD it is ~8x less contended):
//   lines kEpRepLine .. +63  - replicas of the epoch (workgroup b reads replica b mod 64);
//   lines kEpShardLine .. +7 - the "finished" count sharded by blockIdx mod 8, line
//                              kEpTopLine counts the shards that completed.
constexpr int kEpWords = 16;  // words of line 0
constexpr int kLineWords = 16;
constexpr int kEpReplicas = 64;
constexpr int kEpRepLine = 1, kEpShardLine = kEpRepLine + kEpReplicas, kEpShards = 8;
constexpr int kEpTopLine = kEpShardLine + kEpShards;
//   lines kEpClaimLine ..    - one claim word per reduce-scatter segment (kMaxBlocks), holding
//                              the epoch of the launch that claimed it (never reset).
constexpr int kEpClaimLine = kEpTopLine + 1;
constexpr int kEpTeamWords = kEpClaimLine * kLineWords + kMaxBlocks;
constexpr int kEpEpoch = 0;    // epoch of the team's last launch
constexpr int kEpDone = 1;     // workgroups of this launch that have finished
constexpr int kEpRsHead = 2;   // next reduce-scatter segment (scan: phase-1 piece) to grab
constexpr int kEpAgHead = 3;   // next all-gather item to grab
constexpr int kEpStarted = 4;  // workgroups that have started (the first announces the launch)
constexpr int kEpFail = 5;     // nonzero once any wait of this launch timed out: drain at once
constexpr int kEpP1Done = 6;   // scan: phase-1 pieces completed
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
    uint64_t seg_items;      // items per reduce-scatter segment (a multiple of kBlock*kUnroll)
    uint64_t timeout_ticks;  // s_memrealtime ticks (100 MHz)
    int oneshot;  // 1: every member folds the WHOLE array (no hand-off, no all-gather)
    uint32_t *ep_ctr;  // team's launch words (kEpTeamWords, see kEp*)
    int p, me;
    uint64_t *trace;     // development phase timestamps (set_param "trace_buffer"), normally null
};

// Small-message ("LL") path: 8-byte granules {4 data bytes | 32-bit epoch} pushed into every
// peer's fine-grained receive ring.  One ring of kLLTeamBytes per team, laid out by the team's size
// p as [parity 2][sender p][ll_sender_granules(p)] u64, so a sender's capacity is
// kLLTeamBytes / (4p) payload bytes: 1 MiB at 2 PEs, 512 KiB at 4, 256 KiB at 8, 128 KiB at 16.
// The default threshold is the smaller of that and kLLDefaultBytes (512 KiB): measured against the
// persistent kernel, the granule path wins up to 512 KiB at 2 and 4 PEs and loses at 1 MiB
// (DESIGN.md §3, round 5); its link traffic, 2(p-1)·B per PE, grows with p as the capacity shrinks.
#ifndef ISHMEMI_LL_TEAM_BYTES
#define ISHMEMI_LL_TEAM_BYTES (8u << 20)
#endif
constexpr size_t kLLTeamBytes = ISHMEMI_LL_TEAM_BYTES;
__host__ __device__ constexpr uint64_t ll_sender_granules(int p)
{
    // Whole blocks of 64 items (128 granules: ll_granule below).
    return ((uint64_t) kLLTeamBytes / 8 / (2 * (uint64_t) (p < 1 ? 1 : p))) & ~uint64_t(127);
}
// Granule index of item `item`'s half h (0: low 4 bytes, 1: high) in a sender's slot.  Items are
// grouped by 64 (one wave's lanes): [low halves of items 64b .. 64b+63][their high halves], so each
// of a wave's two granule stores (and polls) covers 512 contiguous bytes, whole 64-B lines of the
// uncached ring, instead of every other 8 B of 1 KiB.  ISHMEMI_LL_PAIRED=1 keeps the round-4
// layout (item i at granules 2i, 2i + 1; A/B builds only).
#ifndef ISHMEMI_LL_PAIRED
#define ISHMEMI_LL_PAIRED 0
#endif
__host__ __device__ constexpr uint64_t ll_granule(uint64_t item, int h)
{
    return ISHMEMI_LL_PAIRED ? 2 * item + (uint64_t) h : (item & ~uint64_t(63)) * 2 + (uint64_t) h * 64 + (item & 63);
}
__host__ __device__ constexpr uint64_t ll_capacity(int p) { return ll_sender_granules(p) * 4; }
// The largest capacity (2 PEs) caps ISHMEM_LL_MAX_BYTES / set_param "ll_max_bytes"; their default
// is kLLDefaultBytes.
constexpr size_t kLLMaxBytes = ll_capacity(2);
constexpr size_t kLLDefaultBytes = 512u << 10;
struct LLArgs {
    const char *src;
    char *dst;
    uint64_t *my_ring;              // this team's ring base on this PE (parity 0, sender 0)
    uint64_t *peer_ring[kMaxPes];   // the same ring base on every member, mapped here
    uint32_t *err;
    int *ret;
    uint64_t nbytes;
    uint64_t timeout_ticks;
    uint32_t *ep_ctr;  // team's launch words (kEpTeamWords, see kEp*)
    int p, me;
    // What the received items become (round 5; every member exchanges with every member in each
    // mode, so no member can run more than one collective ahead of another):
    //   kLLReduce - dest = fold of all p members' items;
    //   kLLInscan / kLLExscan - dest = fold of members 0..me / 0..me-1 (sum; member 0's exclusive
    //               result is 0);
    //   kLLCollect - member j's bytes land at dest + j * nbytes (fcollect);
    //   kLLBroadcast - member `root`'s bytes land at every member's dest; the others push one
    //               token item (no source read) so every member still hears from every member.
    int mode;
    int root;
};
constexpr int kLLReduce = 0, kLLInscan = 1, kLLExscan = 2, kLLCollect = 3, kLLBroadcast = 4;
hipError_t launch_ll(int op, int dt, const LLArgs &a, hipStream_t s);

// fcollect / collect (all-gather of the members' sources): member j's bytes land at
// dst + dst_off[j].  Same start / finish protocol as the reduce.
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
    uint32_t *ep_ctr;  // team's launch words (kEpTeamWords, see kEp*)
    int p, me;
    int unit;  // bytes per item: 16, 4 or 1 (largest dividing every address and length)
    // Stream-ordered collect (counts not known on the host): this member publishes my_count into
    // its symmetric count slot before announcing the launch; every workgroup then reads every
    // member's slot (count_at[j], mapped here) and derives the offsets in team order.
    uint64_t my_count;
    uint64_t *my_count_slot;
    const uint64_t *count_at[kMaxPes];
};
hipError_t launch_collect(const CollectArgs &a, int grid, hipStream_t s);
hipError_t launch_collect_dyn(const CollectArgs &a, int grid, hipStream_t s);
// Phased collect: one-shot pull grid, to be bracketed by launch_team_sync on the same stream.
hipError_t launch_collect_phase(const CollectArgs &a, hipStream_t s);

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
    uint32_t *ep_ctr;  // team's launch words (kEpTeamWords, see kEp*)
    int p, me;
    int inclusive;
};
hipError_t launch_scan(int dt, const ScanArgs &a, bool vec, int grid, hipStream_t s);
// Phased scan: phase 1 (fold chunk me into this PE's scratch rows) or 2 (pull this PE's rows),
// one-shot grids, to be separated by launch_team_sync on the same stream.
hipError_t launch_scan_phase(int dt, const ScanArgs &a, bool vec, int phase, hipStream_t s);
// Direct two-member scan (no scratch): one-shot fold of members 0..me into dest, between team
// barriers launched by the caller.
hipError_t launch_scan_direct(int dt, const ScanArgs &a, bool vec, hipStream_t s);

// Arguments of the local k-input fan-in combine: dst = op(src0, src1, ..., src_{k-1}).
constexpr int kMaxFanin = 16;
// Realigned fan-in (kernels_impl.h fanin_realign_kernel): threads per workgroup, one 16-B dest
// item each; the workgroup's last lane loads one vector of the next workgroup's first line, so
// the extra fetch is one line per 8 KiB (round 4's one-wave workgroups: one per 1 KiB).
#ifndef ISHMEMI_REALIGN_BLOCK
#define ISHMEMI_REALIGN_BLOCK 512
#endif
constexpr int kRealignBlock = ISHMEMI_REALIGN_BLOCK;
constexpr int kRealignWaves = kRealignBlock / 64;
constexpr int kRealignMaxGrid = (int) ((1ull << 31) / kRealignBlock);
// The phased reduce-scatter's realigned kernel (rs_phase_realign_kernel): one-wave workgroups
// measured best there (kernels_impl.h rs_realign_block), unlike the 1-PE fan-in.
#ifndef ISHMEMI_RS_REALIGN_BLOCK
#define ISHMEMI_RS_REALIGN_BLOCK 64
#endif
constexpr int kRsRealignBlock = ISHMEMI_RS_REALIGN_BLOCK;
// Dest alignment the realigned body starts at (the head before it runs element-wise): 256 B, so
// the workgroups' 1 KiB store blocks cover whole lines instead of sharing one with a neighbour.
#ifndef ISHMEMI_REALIGN_PEEL
#define ISHMEMI_REALIGN_PEEL 256
#endif
constexpr uint64_t kRealignPeel = ISHMEMI_REALIGN_PEEL;

struct FaninArgs {
    const char *src[kMaxFanin];
    char *dst;
    uint64_t head, nitems, tail;
    int nsrc;
    // Realigned body (fanin_realign_kernel, 1 or 2 sources whose addresses differ from dst's mod
    // 16): head = elements until dst is 16-B aligned; shift[j] = source j's byte offset from the
    // 16-B grid at that point; total = payload bytes (bounds of the sources' aligned loads).
    int realign;
    uint32_t shift[kMaxFanin];
    uint64_t total;
};

// Phased reduce-scatter / all-gather of large payloads (p > 1, 16-B vector body): two one-shot
// grids that never wait, between one-workgroup team barriers (team_sync_kernel).  Pointers are
// translated into this process's address space, as in ReduceArgs.
struct PhaseArgs {
    const char *src[kMaxPes];   // member j's source (element 0)
    const char *dstp[kMaxPes];  // member j's dest (element 0)
    char *dst;                  // own dest
    uint64_t head, nitems, tail;  // scalar head elements, 16-B body items, scalar tail elements
    uint64_t items_per_chunk;     // the reduce-scatter partition (a multiple of 64 items)
    uint32_t elem;                // element bytes (the all-gather copies head / tail bytes)
    int p, me;
    // Measurement only (set_param "phased_peer_nt", default 0): load peers' bytes with nontemporal
    // loads instead of system-coherent (sc0 sc1) ones, leaning on the kernel-boundary acquire for
    // visibility.  For the N > 1 bench's A/B over xGMI (speed, and the tripwire for coherence).
    int peer_nt;
    // Sources on another 16-B phase than dest (runtime.cpp reduce_heap): the byte shift of every
    // member's source at the first dest vector (head = elements until dest is 16-B aligned), and
    // the payload bytes that bound the realigned loads; 0 = same phase.
    uint32_t shift;
    uint64_t total;
    // 1: every member folds the WHOLE array (two-member direct path, runtime.cpp reduce_heap): the
    // reduce-scatter grid over all items and both edges, no all-gather.
    int whole;
    // Shifted sources (shift != 0) on rs_phase_kernel: 1 = XCD-grouped block order (default since
    // round 6, kernels_impl.h xcd_grouped_block), 0 = block order (set_param "rs_xcd", A/B only).
    int xcd_group;
};
hipError_t launch_rs_phase(int op, int dt, const PhaseArgs &a, hipStream_t s);
hipError_t launch_ag_phase(const PhaseArgs &a, hipStream_t s);

// Returns hipSuccess or a launch error.  `vec` selects the 16-B vector body (all operands
// share the same address residue mod 16) or the element-granular path.
hipError_t launch_allreduce(int op, int dt, bool vec, const ReduceArgs &a, int grid,
                            hipStream_t s);
hipError_t launch_fanin(int op, int dt, bool vec, const FaninArgs &a, int grid, hipStream_t s);
hipError_t launch_team_sync(const ReduceArgs &a, hipStream_t s);
// xGMI measurement hook: dst = sum of a.nsrc f32 arrays (a.nitems 16-B items), source loads with
// cache policy 0 = nt, 1 = sc0 sc1.
hipError_t launch_pull_probe(const FaninArgs &a, int policy, hipStream_t s);
// PEs that share this process's GPU (several PEs per device: tests and rehearsals).  Each
// multi-PE launch then takes at most 1/share of the device's resident workgroups, so every
// co-located PE's launch fits at once and one PE's waiting workgroups can never hold the CUs a
// co-located peer needs to make progress (across GPUs that cannot happen).
void set_device_share(int share);
int device_share();
// Waiting footprint (round 4).  The kernels whose workgroups wait for peers — the persistent
// reduce (start handshake, segment hand-offs), the small-message rings, the persistent collect /
// scan — each take at most 1 / (share x wait_slots) of the device's resident workgroups.  A
// device can then hold wait_slots such launches of every co-located PE at once, so a launch whose
// workgroups wait for a peer can never keep a kernel of another team (on another stream, issued in
// the other order on that peer) from becoming resident: collectives of different teams may be in
// flight together, as in the reference (src/teams.h:29-38).  With one PE per GPU and HIP's 4
// hardware queues per process (GPU_MAX_HW_QUEUES) at most 4 kernels of a process run at once, so
// the default 16 keeps a 4x margin (ISHMEM_WAIT_SLOTS).  The phased grids and the fan-in kernel
// never wait and keep the whole device.
constexpr int kWaitSlotsDefault = 16;
void set_wait_slots(int slots);
int wait_slots();
// Tests only (set_param "realign_grid_cap"): at most this many workgroups for the realigned
// kernels (0 = no cap), so their grid-stride loops — which otherwise run only past 2^31 items —
// are exercised at test sizes.
void set_realign_grid_cap(int cap);
int realign_grid_cap();
// The phased fcollect / collect moves members whose addresses or counts are not 16-B aligned with
// realigned 16-B loads (kernels_coll.hip collect_phase_realign_kernel); 0 (set_param
// "collect_realign", A/B only) keeps the narrow 4- / 1-byte items.
void set_collect_realign(int on);
int collect_realign();
// The phased reduce-scatter with sources on another 16-B phase than dest (set_param
// "phase_unaligned", default 1): rs_phase_kernel with unaligned 16-B source loads (the hardware
// splits a load that crosses a line); 0 = rs_phase_realign_kernel (aligned loads, DPP + LDS
// realign).  2 PEs x 1 GiB on one GPU, source 4 B off: reduce-scatter grid 0.525-0.528 vs
// 0.556-0.563 ms; 4 PEs 0.920-0.922 vs 0.932-0.945 (profiles/r05/phase_unaligned/).
void set_phase_unaligned(int on);
int phase_unaligned();
// Test hook: `grid` workgroups that each hold half a CU (1024 work-items, 80 KiB LDS) for `usec`.
hipError_t launch_occupy(int grid, uint64_t usec, hipStream_t s);
hipError_t launch_produce_u32(uint32_t *dst, const uint32_t *a, const uint32_t *b, uint64_t n, hipStream_t s);

}  // namespace ishmemi
