// ishmem_amd — shared (host + device) type/op helpers.  The enums themselves are the public
// C-ABI ones (include/ishmem_capi.h).
//
// Element types are canonical fixed-width types: the reference canonicalises every C type to a
// fixed-width signed/unsigned integer before combining (vector_reduce_helper,
// src/collectives/reduce_impl.h:22-59).  Signedness only changes MIN/MAX, so the kernels fold
// SUM/PROD/AND/OR/XOR on the unsigned type of the same width (two's-complement wrap, identical
// bits) and keep the signed type for MIN/MAX.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "ishmem_capi.h"

namespace ishmemi {

inline constexpr size_t dtype_size(int dt)
{
    return (dt == ISHMEMI_DT_INT8 || dt == ISHMEMI_DT_UINT8)     ? 1
           : (dt == ISHMEMI_DT_INT16 || dt == ISHMEMI_DT_UINT16) ? 2
           : (dt == ISHMEMI_DT_INT32 || dt == ISHMEMI_DT_UINT32 || dt == ISHMEMI_DT_FLOAT)
               ? 4
               : 8;
}

inline constexpr bool dtype_is_float(int dt)
{
    return dt == ISHMEMI_DT_FLOAT || dt == ISHMEMI_DT_DOUBLE;
}

// Reference validity matrix (docs/source/collectives.rst:910-936, src/collectives/reduce.cpp:95-417):
// bitwise ops only on integer types; fp only max/min/sum/prod.
inline constexpr bool op_dtype_valid(int op, int dt)
{
    if (op < 0 || op >= ISHMEMI_OP_COUNT || dt < 0 || dt >= ISHMEMI_DT_COUNT) return false;
    if (dtype_is_float(dt) && op <= ISHMEMI_OP_XOR) return false;
    return true;
}

}  // namespace ishmemi
