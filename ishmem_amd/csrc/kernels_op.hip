// ishmem_amd — instantiation unit for ONE reduction op (compiled once per op with
// -DISHMEMI_KOP=<0..6>, see ishmem_amd/_build.py): all element types of that op, both kernels.
#include "kernels_impl.h"

#ifndef ISHMEMI_KOP
#error "compile with -DISHMEMI_KOP=<op>"
#endif
#define ISHMEMI_CAT2(a, b) a##b
#define ISHMEMI_CAT(a, b) ISHMEMI_CAT2(a, b)

namespace ishmemi {

hipError_t ISHMEMI_CAT(launch_allreduce_op, ISHMEMI_KOP)(int dt, bool vec, const ReduceArgs &a,
                                                         int grid, hipStream_t s)
{
    auto l = [&]<typename T, int OP>() { return ar_t<T, OP>(vec, a, grid, s); };
    return dispatch_dt<ISHMEMI_KOP, ReduceArgs>(dt, l);
}

hipError_t ISHMEMI_CAT(launch_fanin_op, ISHMEMI_KOP)(int dt, bool vec, const FaninArgs &a, int grid,
                                                     hipStream_t s)
{
    auto l = [&]<typename T, int OP>() { return fi_t<T, OP>(vec, a, grid, s); };
    return dispatch_dt<ISHMEMI_KOP, FaninArgs>(dt, l);
}

hipError_t ISHMEMI_CAT(launch_rs_phase_op, ISHMEMI_KOP)(int dt, const PhaseArgs &a, hipStream_t s)
{
    auto l = [&]<typename T, int OP>() { return rs_phase_t<T, OP>(a, s); };
    return dispatch_dt<ISHMEMI_KOP, PhaseArgs>(dt, l);
}

hipError_t ISHMEMI_CAT(launch_ll_op, ISHMEMI_KOP)(int dt, const LLArgs &a, hipStream_t s)
{
    auto l = [&]<typename T, int OP>() { return ll_t<T, OP>(a, s); };
    return dispatch_dt<ISHMEMI_KOP, LLArgs>(dt, l);
}

}  // namespace ishmemi
