// qknit_plan.hip — plan-level knit: operand transforms + contraction in one C call (qk_knit).
//
// The reference's VirtualCircuit.knit (virtual_circuit.py:50-68: merge of every fragment's
// per-label distributions, then the per-gate knits last to first) is, on the swept rows q_f of
// each fragment, R[key] = sum_k prod_f X_f[k][x_f] with X_f = W_f^T q_f: W_f the
// fragment's transform ([rows_f][K]: label gathers, knit coefficients, the factored / basis /
// light-cone folds, all precomputed by the host planner) and key = sum_f pdep(x_f, mask_f). A host
// that is not Python hands this the transforms and masks once and the swept rows per run:
//   1. X_f = W_f^T q_f                      (qk_gemm_keyed: contraction over the swept rows)
//   2. fragments ordered as engine.contract_order (the one holding clbit 0 last: the N axis);
//      3+ fragments: the leading ones folded by Khatri-Rao products, their keys added
//   3. out[kA(i) + kB(j)] = sum_k A[k][i] B[k][j]  (qk_gemm_keyed; one fragment: B = ones)
// Keys are pdep tables built on the device (affine strides when a fragment's clbits are
// contiguous). The result equals the Python pipeline's exact contraction (data-rank compression,
// a per-step optimisation with a device-side check, stays in KnitPipeline).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

#include "internal.h"

namespace {

int pfail(qk_ctx* ctx, int code, const std::string& msg) {
    if (ctx) ctx->err = msg;
    return code;
}

__global__ void qk_pdep_keys_kernel(int64_t n, uint64_t mask, int64_t* keys) {
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n; x += (int64_t)gridDim.x * blockDim.x) {
        uint64_t m = mask, k = 0, bit = 1;
        for (; m; m &= m - 1, bit <<= 1)
            if ((uint64_t)x & bit) k |= m & (~m + 1);
        keys[x] = (int64_t)k;
    }
}

// keys[i + j * M] = ka[i] + kb[j] (the Khatri-Rao column order of qk_khatri_rao)
__global__ void qk_add_keys_kernel(int64_t M, int64_t N, const int64_t* ka, const int64_t* kb, int64_t* out) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < M * N; e += (int64_t)gridDim.x * blockDim.x)
        out[e] = ka[e % M] + kb[e / M];
}

__global__ void qk_fill_kernel(int64_t n, double v, double* out) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x)
        out[e] = v;
}

unsigned grid_of(int64_t n) {
    const int64_t g = (n + 255) / 256;
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(g, 65536));
}

int64_t align16(int64_t b) { return (b + 255) & ~int64_t(255); }

struct Layout {
    std::vector<int> order;            // contraction order of the fragments
    std::vector<int64_t> x_off;        // workspace offsets (bytes) of X_f [K][2^m_f]
    std::vector<int64_t> key_off;      // offsets of the key tables (-1: affine)
    int64_t kr_off = -1, kr_size = 0;  // Khatri-Rao products (3+ fragments): two ping-pong buffers
    int64_t krk_off = -1, krk_size = 0;
    int64_t ones_off = -1;             // B = ones (1 fragment)
    int64_t total = 0;
};

bool contiguous_bits(uint64_t m) { return m && (((m >> __builtin_ctzll(m)) + 1) & (m >> __builtin_ctzll(m))) == 0; }

int layout(const qk_knit_plan* p, Layout& L, std::string& why) {
    if (!p || p->n_frag < 1 || p->n_frag > 4 || p->terms < 1 || p->nbits < 1 || p->nbits > 34 || !p->rows ||
        !p->clbit_masks || !p->transforms) {
        why = "qk_knit: need 1..4 fragments, terms >= 1, 1 <= nbits <= 34 and the plan arrays";
        return QK_EARG;
    }
    uint64_t seen = 0;
    for (int f = 0; f < p->n_frag; ++f) {
        const uint64_t m = p->clbit_masks[f];
        if (p->rows[f] < 1 || !p->transforms[f]) {
            why = "qk_knit: every fragment needs swept rows and a transform";
            return QK_EARG;
        }
        if ((m & seen) || (p->nbits < 64 && (m >> p->nbits))) {
            why = "qk_knit: fragment clbit masks must be disjoint and below nbits";
            return QK_EARG;
        }
        if (__builtin_popcountll(m) > 24) {
            why = "qk_knit: at most 24 measured clbits per fragment";
            return QK_EARG;
        }
        seen |= m;
    }
    // engine.contract_order: descending lowest clbit, so the fragment holding the lowest goes last
    L.order.resize(p->n_frag);
    for (int f = 0; f < p->n_frag; ++f) L.order[f] = f;
    auto low = [&](int f) { return p->clbit_masks[f] ? __builtin_ctzll(p->clbit_masks[f]) : 1 << 30; };
    std::stable_sort(L.order.begin(), L.order.end(), [&](int a, int b) { return low(a) > low(b); });
    const int64_t K = p->terms;
    int64_t off = 0;
    L.x_off.assign(p->n_frag, 0);
    L.key_off.assign(p->n_frag, -1);
    for (int f = 0; f < p->n_frag; ++f) {
        const int64_t w = int64_t(1) << __builtin_popcountll(p->clbit_masks[f]);
        L.x_off[f] = off;
        off += align16(K * w * 8);
        if (!contiguous_bits(p->clbit_masks[f]) || p->n_frag > 2) {
            L.key_off[f] = off;
            off += align16(w * 8);
        }
    }
    if (p->n_frag > 2) {
        int64_t M = 1;
        for (int i = 0; i + 1 < p->n_frag; ++i) M *= int64_t(1) << __builtin_popcountll(p->clbit_masks[L.order[i]]);
        L.kr_off = off;
        L.kr_size = align16(K * M * 8);
        off += 2 * L.kr_size;
        L.krk_off = off;
        L.krk_size = align16(M * 8);
        off += 2 * L.krk_size;
    }
    if (p->n_frag == 1) {
        L.ones_off = off;
        off += align16(K * 8);
    }
    L.total = off;
    return QK_OK;
}

}  // namespace

extern "C" {

int qk_knit_workspace_bytes(const qk_knit_plan* plan, int64_t* bytes) {
    if (!bytes) return QK_EARG;
    Layout L;
    std::string why;
    const int rc = layout(plan, L, why);
    if (rc) return rc;
    *bytes = L.total;
    return QK_OK;
}

int qk_knit(qk_ctx* ctx, const qk_knit_plan* plan, const double* const* q, void* workspace, int64_t workspace_bytes,
            double* out) {
    if (!ctx) return QK_EARG;
    Layout L;
    std::string why;
    int rc = layout(plan, L, why);
    if (rc) return pfail(ctx, rc, why);
    if (!q || !out || !workspace || workspace_bytes < L.total)
        return pfail(ctx, QK_EARG, "qk_knit: null rows / output, or workspace below qk_knit_workspace_bytes");
    for (int f = 0; f < plan->n_frag; ++f)
        if (!q[f]) return pfail(ctx, QK_EARG, "qk_knit: null swept rows");
    if (hipSetDevice(ctx->device) != hipSuccess) return pfail(ctx, QK_EHIP, "qk_knit: hipSetDevice");
    char* ws = static_cast<char*>(workspace);
    const int64_t K = plan->terms;
    auto width = [&](int f) { return int64_t(1) << __builtin_popcountll(plan->clbit_masks[f]); };
    auto X = [&](int f) { return reinterpret_cast<double*>(ws + L.x_off[f]); };
    auto keys = [&](int f) { return L.key_off[f] < 0 ? nullptr : reinterpret_cast<int64_t*>(ws + L.key_off[f]); };
    // 1. operands X_f[k][x] = sum_l W_f[l][k] q_f[l][x]
    for (int f = 0; f < plan->n_frag; ++f) {
        const int64_t w = width(f);
        rc = qk_gemm_keyed(ctx, K, w, plan->rows[f], plan->transforms[f], K, q[f], w, nullptr, w, nullptr, 1, X(f), 0);
        if (rc) return rc;
        if (keys(f)) {
            hipLaunchKernelGGL(qk_pdep_keys_kernel, dim3(grid_of(w)), dim3(256), 0, ctx->stream, w,
                               (uint64_t)plan->clbit_masks[f], keys(f));
        }
    }
    auto stride_of = [&](int f) -> int64_t {
        const uint64_t m = plan->clbit_masks[f];
        return m ? int64_t(1) << __builtin_ctzll(m) : 0;
    };
    // 2.-3. contraction
    if (plan->n_frag == 1) {
        const int f = 0;
        double* ones = reinterpret_cast<double*>(ws + L.ones_off);
        hipLaunchKernelGGL(qk_fill_kernel, dim3(grid_of(K)), dim3(256), 0, ctx->stream, K, 1.0, ones);
        rc = qk_gemm_keyed(ctx, width(f), 1, K, X(f), width(f), ones, 1, keys(f), keys(f) ? 0 : stride_of(f), nullptr,
                           0, out, 0);
        if (!rc && hipGetLastError() != hipSuccess) rc = pfail(ctx, QK_EHIP, "qk_knit: launch failed");
        return rc;
    }
    const int fb = L.order.back();
    const double* A = X(L.order[0]);
    const int64_t* kA = keys(L.order[0]);
    int64_t M = width(L.order[0]), sA = kA ? 0 : stride_of(L.order[0]);
    for (int i = 1; i + 1 < plan->n_frag; ++i) {  // Khatri-Rao fold of the leading fragments
        const int f = L.order[i];
        double* kr = reinterpret_cast<double*>(ws + L.kr_off + (i & 1) * L.kr_size);
        int64_t* kk = reinterpret_cast<int64_t*>(ws + L.krk_off + (i & 1) * L.krk_size);
        rc = qk_khatri_rao(ctx, K, M, width(f), A, M, X(f), width(f), kr);
        if (rc) return rc;
        hipLaunchKernelGGL(qk_add_keys_kernel, dim3(grid_of(M * width(f))), dim3(256), 0, ctx->stream, M, width(f), kA,
                           keys(f), kk);
        A = kr;
        kA = kk;
        sA = 0;
        M *= width(f);
    }
    rc = qk_gemm_keyed(ctx, M, width(fb), K, A, M, X(fb), width(fb), kA, sA, keys(fb), keys(fb) ? 0 : stride_of(fb),
                       out, 0);
    if (!rc && hipGetLastError() != hipSuccess) rc = pfail(ctx, QK_EHIP, "qk_knit: launch failed");
    return rc;
}

}  // extern "C"

// ---- qk_knit_lowrank: the benched single-GPU knit (KnitPipeline's device data rank) in one call -----
// Steps, all on ctx->stream with no host synchronisation (DESIGN.md §2 "Data-rank compression"); with at
// most 80 swept rows per side steps 1, 3 and 4 are the q-space chain (qk_qprep_grams, qk_qprep_compress_check
// and two transforms X = Wt^T q predicated on k == 0 for step 6), as the benched pipeline takes them:
//   1. qk_prep_operands   X_A = Wt_A^T q_A, X_B = Wt_B^T q_B, G_A, G_B, U = X_B P^T
//   2. qk_rank_factors    T_A, T_B, r from the Grams (r = 0: no factorisation of rank <= 8)
//   3. qk_compress_operands  A'' = T_A X_A, B'' = T_B X_B  (8 rows)
//   4. qk_probe_errors    accepted rank k = r when every probe error is <= max(rank_tol, rank_tol_rel ||R p||)
//   5. qk_knit_outer_stream_range  the write-bound knit of A'', B'' with K = k (k = 0: nothing)
//   6. qk_gemm_keyed_pred the exact K-term contraction of X_A, X_B, predicated on k == 0
namespace {

constexpr int LR_RMAX = 8;
constexpr int LR_PROBES = 16;

struct LowrankLayout {
    int64_t xa, xb, g, u, prep, ta, tb, r, a2, b2, e2, k, err, probe, ka, kb, total;
    int64_t prep_bytes, probe_bytes;
    bool qspace;  // the q-space chain (qk_qprep_*): at most 80 swept rows per side, widths % 256
};

// as KnitPipeline._qspace_prep / engine.qprep_ok: the chain the benched step takes for these shapes
bool lowrank_qspace(const qk_lowrank_plan* p) {
    const int64_t NA = int64_t(1) << __builtin_popcountll(p->mask_a), NB = int64_t(1) << __builtin_popcountll(p->mask_b);
    const char* env = getenv("QKNIT_QPREP");  // opt-in, as engine.QPREP (the X path measured faster)
    return env && env[0] == '1' && p->rows_a <= 80 && p->rows_b <= 80 && NA % 512 == 0 && NB % 512 == 0;
}

int lowrank_layout(qk_ctx* ctx, const qk_lowrank_plan* p, LowrankLayout& L, std::string& why) {
    if (!p || p->terms < 2 || p->terms > 64 || (p->terms & 1) || p->rows_a < 1 || p->rows_b < 1 || !p->wt_a ||
        !p->wt_b || !p->probes || p->nbits < 2 || p->nbits > 32) {
        why = "qk_knit_lowrank: need even 2 <= terms <= 64, swept rows, transforms, probes, 2 <= nbits <= 32";
        return QK_EARG;
    }
    if (p->rows_a > INT32_MAX || p->rows_b > INT32_MAX) {  // qk_prep_operands takes int row counts
        why = "qk_knit_lowrank: rows_a and rows_b must be at most INT32_MAX";
        return QK_EARG;
    }
    const uint64_t full = (uint64_t(1) << p->nbits) - 1;
    if ((p->mask_a & p->mask_b) || (p->mask_a | p->mask_b) != full || !(p->mask_b & 1)) {
        why = "qk_knit_lowrank: masks must be disjoint, cover all nbits output bits, bit 0 in mask_b";
        return QK_EARG;
    }
    const int64_t NA = int64_t(1) << __builtin_popcountll(p->mask_a), NB = int64_t(1) << __builtin_popcountll(p->mask_b);
    if (NA % 128 || NB % 128) {
        why = "qk_knit_lowrank: each fragment needs >= 7 measured clbits (operand widths multiples of 128)";
        return QK_EARG;
    }
    const int64_t K = p->terms;
    int64_t prep = 0, probe = 0;
    int rc = qk_prep_workspace_bytes(ctx, NA, NB, &prep);
    if (!rc) rc = qk_probe_workspace_bytes(ctx, NA, &probe);
    int64_t qprep = 0;
    if (!rc) rc = qk_qprep_workspace_bytes(ctx, NA, NB, &qprep);
    L.qspace = lowrank_qspace(p);
    if (L.qspace && qprep > prep) prep = qprep;
    if (rc) {
        why = "qk_knit_lowrank: workspace queries failed";
        return rc;
    }
    int64_t off = 0;
    auto take = [&](int64_t bytes) { const int64_t o = off; off += align16(bytes); return o; };
    L.xa = take(K * NA * 8);
    L.xb = take(K * NB * 8);
    L.g = take(2 * K * K * 8);
    L.u = take(K * LR_PROBES * 8);
    L.prep = take(prep);
    L.ta = take(LR_RMAX * K * 8);
    L.tb = take(LR_RMAX * K * 8);
    L.r = take(8);
    L.a2 = take(LR_RMAX * NA * 8);
    L.b2 = take(LR_RMAX * NB * 8);
    L.e2 = take(2 * LR_PROBES * 8);
    L.k = take(8);
    L.err = take(8);
    L.probe = take(probe);
    L.ka = contiguous_bits(p->mask_a) ? -1 : take(NA * 8);
    L.kb = contiguous_bits(p->mask_b) ? -1 : take(NB * 8);
    L.total = off;
    L.prep_bytes = prep;
    L.probe_bytes = probe;
    return QK_OK;
}

__global__ void qk_copy_i32_kernel(const int32_t* src, int32_t* dst) { *dst = *src; }

}  // namespace

extern "C" {

int qk_knit_lowrank_workspace_bytes(qk_ctx* ctx, const qk_lowrank_plan* plan, int64_t* bytes) {
    if (!ctx || !bytes) return QK_EARG;
    LowrankLayout L;
    std::string why;
    const int rc = lowrank_layout(ctx, plan, L, why);
    if (rc) return pfail(ctx, rc, why);
    *bytes = L.total;
    return QK_OK;
}

int qk_knit_lowrank(qk_ctx* ctx, const qk_lowrank_plan* p, const double* q_a, const double* q_b, void* workspace,
                    int64_t workspace_bytes, double* out, int32_t* rank_out) {
    if (!ctx) return QK_EARG;
    LowrankLayout L;
    std::string why;
    int rc = lowrank_layout(ctx, p, L, why);
    if (rc) return pfail(ctx, rc, why);
    if (!q_a || !q_b || !out || !workspace || workspace_bytes < L.total)
        return pfail(ctx, QK_EARG, "qk_knit_lowrank: null rows / output, or workspace below qk_knit_lowrank_workspace_bytes");
    if (hipSetDevice(ctx->device) != hipSuccess) return pfail(ctx, QK_EHIP, "qk_knit_lowrank: hipSetDevice");
    char* ws = static_cast<char*>(workspace);
    auto D = [&](int64_t off) { return reinterpret_cast<double*>(ws + off); };
    const int K = p->terms;
    const int64_t NA = int64_t(1) << __builtin_popcountll(p->mask_a), NB = int64_t(1) << __builtin_popcountll(p->mask_b);
    double *XA = D(L.xa), *XB = D(L.xb), *G = D(L.g), *U = D(L.u);
    int32_t* r = reinterpret_cast<int32_t*>(ws + L.r);
    int32_t* k = reinterpret_cast<int32_t*>(ws + L.k);
    if (L.qspace) {
        // q-space chain (qknit_prep.hip): X is formed only by the predicated transforms of the exact path
        const int RA = (int)p->rows_a, RB = (int)p->rows_b;
        rc = qk_qprep_grams(ctx, K, RA, p->wt_a, q_a, NA, NA, RB, p->wt_b, q_b, NB, NB, p->probes, G, G + K * K, U,
                            D(L.prep), L.prep_bytes);
        if (!rc) rc = qk_rank_factors(ctx, K, G, G + K * K, p->lam_tol, p->s_tol, p->s_abs, LR_RMAX, D(L.ta), D(L.tb), r);
        if (!rc)
            rc = qk_qprep_compress_check(ctx, K, LR_RMAX, RA, p->wt_a, q_a, NA, NA, RB, p->wt_b, q_b, NB, NB, D(L.ta),
                                         D(L.tb), U, p->probes, D(L.a2), D(L.b2), D(L.e2), r, p->rank_tol,
                                         p->rank_tol_rel, k, D(L.err), D(L.prep), L.prep_bytes);
        if (!rc) rc = qk_gemm_keyed_pred(ctx, K, NA, RA, p->wt_a, K, q_a, NA, nullptr, NA, nullptr, 1, XA, 0, k);
        if (!rc) rc = qk_gemm_keyed_pred(ctx, K, NB, RB, p->wt_b, K, q_b, NB, nullptr, NB, nullptr, 1, XB, 0, k);
    } else {
        rc = qk_prep_operands(ctx, K, (int)p->rows_a, p->wt_a, q_a, NA, NA, XA, (int)p->rows_b, p->wt_b, q_b, NB, NB,
                              XB, p->probes, G, G + K * K, U, D(L.prep), L.prep_bytes);
        if (!rc) rc = qk_rank_factors(ctx, K, G, G + K * K, p->lam_tol, p->s_tol, p->s_abs, LR_RMAX, D(L.ta), D(L.tb), r);
        if (!rc) rc = qk_compress_operands(ctx, K, LR_RMAX, D(L.ta), XA, NA, D(L.a2), D(L.tb), XB, NB, D(L.b2));
        if (!rc)
            rc = qk_probe_errors(ctx, K, LR_RMAX, XA, NA, NA, D(L.a2), NA, U, D(L.b2), NB, NB, p->probes, NB, D(L.e2),
                                 r, p->rank_tol, p->rank_tol_rel, k, D(L.err), D(L.probe), L.probe_bytes);
    }
    if (!rc)
        rc = qk_knit_outer_stream_range(ctx, p->nbits, LR_RMAX, D(L.a2), NA, D(L.b2), NB, p->mask_a, p->mask_b, 0,
                                        int64_t(1) << p->nbits, k, out);
    if (rc) return rc;
    int64_t* ka = L.ka >= 0 ? reinterpret_cast<int64_t*>(ws + L.ka) : nullptr;
    int64_t* kb = L.kb >= 0 ? reinterpret_cast<int64_t*>(ws + L.kb) : nullptr;
    if (ka) hipLaunchKernelGGL(qk_pdep_keys_kernel, dim3(grid_of(NA)), dim3(256), 0, ctx->stream, NA, p->mask_a, ka);
    if (kb) hipLaunchKernelGGL(qk_pdep_keys_kernel, dim3(grid_of(NB)), dim3(256), 0, ctx->stream, NB, p->mask_b, kb);
    const int64_t sa = ka ? 0 : int64_t(1) << __builtin_ctzll(p->mask_a);
    const int64_t sb = kb ? 0 : int64_t(1) << __builtin_ctzll(p->mask_b);
    rc = qk_gemm_keyed_pred(ctx, NA, NB, K, XA, NA, XB, NB, ka, sa, kb, sb, out, 0, k);
    if (rc) return rc;
    if (rank_out) hipLaunchKernelGGL(qk_copy_i32_kernel, dim3(1), dim3(1), 0, ctx->stream, k, rank_out);
    if (hipGetLastError() != hipSuccess) return pfail(ctx, QK_EHIP, "qk_knit_lowrank: launch failed");
    return QK_OK;
}

}  // extern "C"
