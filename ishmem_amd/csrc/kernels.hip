// ishmem_amd — launch dispatch of the reduction-collective kernels (see kernels_impl.h for the
// kernels and their design notes; kernels_op.hip instantiates them once per op).
#include "kernels_impl.h"

namespace ishmemi {

namespace {
int g_device_share = 1;
int g_wait_slots = kWaitSlotsDefault;
}
void set_device_share(int share) { g_device_share = share < 1 ? 1 : share; }
int device_share() { return g_device_share; }
void set_wait_slots(int slots) { g_wait_slots = slots < 1 ? 1 : slots; }
int wait_slots() { return g_wait_slots; }
int g_realign_grid_cap = 0;
void set_realign_grid_cap(int cap) { g_realign_grid_cap = cap < 0 ? 0 : cap; }
int realign_grid_cap() { return g_realign_grid_cap; }
int g_collect_realign = 1;
void set_collect_realign(int on) { g_collect_realign = on != 0; }
int collect_realign() { return g_collect_realign; }
int g_phase_unaligned = 1;
void set_phase_unaligned(int on) { g_phase_unaligned = on != 0; }
int phase_unaligned() { return g_phase_unaligned; }

#define ISHMEMI_DECL_OP(N)                                                                         \
    hipError_t launch_allreduce_op##N(int dt, bool vec, const ReduceArgs &a, int grid,             \
                                      hipStream_t s);                                              \
    hipError_t launch_fanin_op##N(int dt, bool vec, const FaninArgs &a, int grid, hipStream_t s); \
    hipError_t launch_ll_op##N(int dt, const LLArgs &a, hipStream_t s);                            \
    hipError_t launch_rs_phase_op##N(int dt, const PhaseArgs &a, hipStream_t s);
ISHMEMI_DECL_OP(0)
ISHMEMI_DECL_OP(1)
ISHMEMI_DECL_OP(2)
ISHMEMI_DECL_OP(3)
ISHMEMI_DECL_OP(4)
ISHMEMI_DECL_OP(5)
ISHMEMI_DECL_OP(6)

hipError_t launch_allreduce(int op, int dt, bool vec, const ReduceArgs &a, int grid, hipStream_t s)
{
    if (!op_dtype_valid(op, dt)) return hipErrorInvalidValue;
    switch (op) {
        case 0: return launch_allreduce_op0(dt, vec, a, grid, s);
        case 1: return launch_allreduce_op1(dt, vec, a, grid, s);
        case 2: return launch_allreduce_op2(dt, vec, a, grid, s);
        case 3: return launch_allreduce_op3(dt, vec, a, grid, s);
        case 4: return launch_allreduce_op4(dt, vec, a, grid, s);
        case 5: return launch_allreduce_op5(dt, vec, a, grid, s);
        case 6: return launch_allreduce_op6(dt, vec, a, grid, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_fanin(int op, int dt, bool vec, const FaninArgs &a, int grid, hipStream_t s)
{
    if (!op_dtype_valid(op, dt)) return hipErrorInvalidValue;
    switch (op) {
        case 0: return launch_fanin_op0(dt, vec, a, grid, s);
        case 1: return launch_fanin_op1(dt, vec, a, grid, s);
        case 2: return launch_fanin_op2(dt, vec, a, grid, s);
        case 3: return launch_fanin_op3(dt, vec, a, grid, s);
        case 4: return launch_fanin_op4(dt, vec, a, grid, s);
        case 5: return launch_fanin_op5(dt, vec, a, grid, s);
        case 6: return launch_fanin_op6(dt, vec, a, grid, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_ll(int op, int dt, const LLArgs &a, hipStream_t s)
{
    if (!op_dtype_valid(op, dt)) return hipErrorInvalidValue;
    switch (op) {
        case 0: return launch_ll_op0(dt, a, s);
        case 1: return launch_ll_op1(dt, a, s);
        case 2: return launch_ll_op2(dt, a, s);
        case 3: return launch_ll_op3(dt, a, s);
        case 4: return launch_ll_op4(dt, a, s);
        case 5: return launch_ll_op5(dt, a, s);
        case 6: return launch_ll_op6(dt, a, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_rs_phase(int op, int dt, const PhaseArgs &a, hipStream_t s)
{
    if (!op_dtype_valid(op, dt)) return hipErrorInvalidValue;
    switch (op) {
        case 0: return launch_rs_phase_op0(dt, a, s);
        case 1: return launch_rs_phase_op1(dt, a, s);
        case 2: return launch_rs_phase_op2(dt, a, s);
        case 3: return launch_rs_phase_op3(dt, a, s);
        case 4: return launch_rs_phase_op4(dt, a, s);
        case 5: return launch_rs_phase_op5(dt, a, s);
        case 6: return launch_rs_phase_op6(dt, a, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_ag_phase(const PhaseArgs &a, hipStream_t s)
{
    // One workgroup per (peer, 64-item block) of a full chunk (ag_phase_kernel's work list).
    const uint64_t blocks = (a.items_per_chunk + kFaninBlock - 1) / kFaninBlock;
    hipLaunchKernelGGL(ag_phase_kernel, dim3(phase_grid(ag_phase_kernel, (uint64_t) (a.p - 1) * blocks * kFaninBlock)),
                       dim3(kFaninBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_team_sync(const ReduceArgs &a, hipStream_t s)
{
    hipLaunchKernelGGL(team_sync_kernel, dim3(1), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

}  // namespace ishmemi
