// prim.h — device-wide primitives of libqknit.so, hand-written for gfx950 (qknit_prim.hip): counting,
// unordered selection, exclusive prefix sums and a stable LSD radix sort of (key, value) pairs. They
// serve the reference-shaped result (QuasiDistr's ACCURACY truncation, quasi_distr.py:7-10, and
// nearest_probability_distribution, quasi_distr.py:28-43, run.py:71; qknit_post.hip, qknit_select.hip).
// Not part of the C ABI.
#ifndef QKNIT_PRIM_H
#define QKNIT_PRIM_H

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace qkp {

// Sum of one value per thread over a 256-thread workgroup (4 waves), returned to every thread.
// `red` is __shared__ scratch of 4 entries. Wave sums by butterfly shuffles, then the 4 wave sums
// in a fixed order (deterministic).
template <typename T>
__device__ __forceinline__ T block_sum256(T v, T* red) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    const int wave = threadIdx.x >> 6;
    __syncthreads();  // `red` may still be read by a previous call
    if ((threadIdx.x & 63) == 0) red[wave] = v;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
}

// Key orders of radix_sort_pairs: keys compared as unsigned 64-bit integers, or as the fp64 values
// whose bit patterns they are (ascending, -0.0 before +0.0; no NaN).
enum KeyOrder { KEY_U64 = 0, KEY_F64 = 1 };

// Temporary bytes radix_sort_pairs needs for n pairs.
size_t radix_sort_bytes(int64_t n);
// Stable ascending sort of n (key, value) pairs by key bits [begin_bit, end_bit) (of the key's
// order-preserving u64 image). keys_in / vals_in are not modified; keys_out / vals_out receive the
// result (may not alias the inputs). 8-bit digits, one pass per digit: a per-wave digit histogram, an
// exclusive scan of the (digit, wave) counts, a per-wave stable scatter (peer lanes of a digit found
// with 8 ballots; no workgroup barrier in the digit passes).
hipError_t radix_sort_pairs(hipStream_t s, int64_t n, const uint64_t* keys_in, const uint64_t* vals_in,
                            uint64_t* keys_out, uint64_t* vals_out, int begin_bit, int end_bit, KeyOrder order,
                            void* tmp, size_t tmp_bytes);

// Temporary bytes exclusive_sum needs for n doubles.
size_t scan_bytes(int64_t n);
// out[i] = in[0] + ... + in[i - 1] (out[0] = 0), deterministic (fixed association); out may alias in.
hipError_t exclusive_sum(hipStream_t s, int64_t n, const double* in, double* out, void* tmp, size_t tmp_bytes);

// Temporary bytes count_abs_above needs.
size_t count_bytes();
// *count_dev (device int64) = #{i < n : |v[i]| > acc}. Reads v once with 16-B loads on a grid of
// 8 workgroups per CU; per-workgroup partials summed by one workgroup (deterministic, no atomics).
hipError_t count_abs_above(hipStream_t s, int cus, int64_t n, const double* v, double acc, int64_t* count_dev,
                           void* tmp, size_t tmp_bytes);

// Appends (i, v[i]) for every |v[i]| > acc to idx / vals (unordered: one atomic per wave of kept
// lanes) and counts them in *count (device, zeroed by the caller); entries past `capacity` are counted,
// not written.
hipError_t select_abs_above(hipStream_t s, int cus, int64_t n, const double* v, double acc, int64_t* idx,
                            double* vals, unsigned long long* count, int64_t capacity);

}  // namespace qkp

#endif  // QKNIT_PRIM_H
