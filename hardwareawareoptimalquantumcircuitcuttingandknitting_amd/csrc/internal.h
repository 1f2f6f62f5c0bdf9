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

// qknit_select.hip: nearest_probability_distribution (quasi_distr.py:28-43) of count (key, value) pairs
// with keys below 2^key_bits — sort by key, stably by value, prefix sums, the closed-form projection
size_t npd_pairs_bytes(int64_t count);
int npd_pairs_bits(qk_ctx* ctx, int64_t count, const int64_t* keys, const double* vals, int key_bits, void* ws,
                   int64_t ws_bytes, int64_t* out_keys, double* out_vals, int64_t* n_out_dev);

#endif  // QKNIT_INTERNAL_H
