// internal.h — context shared by the translation units of libqknit.so (not part of the ABI).
#ifndef QKNIT_INTERNAL_H
#define QKNIT_INTERNAL_H

#include <hip/hip_runtime.h>

#include <string>

#include "../../include/qknit.h"

struct qk_ctx {
    int device;
    hipStream_t own;     // created with the context
    hipStream_t stream;  // where launches go (own, or an external stream)
    int cus;             // compute units the stream may use (its CU mask): persistent grids are sized to it
    std::string err;     // last error message (qk_last_error)
};

#endif  // QKNIT_INTERNAL_H
