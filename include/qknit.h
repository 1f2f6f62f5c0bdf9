/*
 * qknit.h — C ABI of the MI355X (gfx950) circuit-knitting engine, libqknit.so.
 *
 * Drop-in boundary for the reference's knitting hot path
 * (thangktran/HardwareAwareOptimalQuantumCircuitCuttingAndKnitting):
 *
 *   qk_sweep         replaces the simulator plug  `virt.get_backend(frag).run(instantiations,
 *                    shots)` + `job.result().get_counts()` + `QuasiDistr.from_counts`
 *                    (third_party/qvm/qvm/run.py:36-58, quasi_distr.py:12-20): exact
 *                    per-instance distributions of every cut instantiation of one fragment,
 *                    batched, one launch per pass.
 *   qk_reduce_labels folds the config-bit branches of each instance label with their signs
 *                    (the `split` + subtract of virtual_gates.py:105-124,179-194,262-286).
 *   qk_gemm_keyed    replaces the merge + per-vgate knit (virtual_circuit.py:50-68,165-171,
 *                    216-228; quasi_distr.py:55-60): a dense fp64 MFMA contraction over the
 *                    instance-label axis with the output scattered to global clbit keys.
 *   qk_khatri_rao    row-wise outer product (3+ fragment knits).
 *   qk_gather_rows   label gather + coefficient scaling of fragment rows.
 *
 * Conventions: every function returns 0 on success and a QK_E* code otherwise (message via
 * qk_last_error). Sizes are int64_t. All data buffers are DEVICE pointers owned by the caller,
 * except qk_program.passes (HOST). Complex values are interleaved (re, im) doubles.
 * One context per (thread, device); a context holds one HIP stream and no other mutable
 * global state, so distinct contexts may be driven concurrently from different threads.
 */
#ifndef QKNIT_H
#define QKNIT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QK_OK 0
#define QK_EARG 1     /* invalid argument / shape */
#define QK_EHIP 2     /* HIP runtime error */
#define QK_ESTATE 3   /* invalid context state */

#define QK_TILE_BITS 12
#define QK_FIBER_BITS 4

/* op kinds (sweep_plan.py K_*). Matrices are interleaved complex unless noted:
 *   U1 2x2 (8)  D1 diag (4)  U2 4x4 (32)  D2 diag4 (8)  SCALE (2 per variant)
 *   U1R real 2x2 (4 reals)   U1X [m00, Im m01, Im m10, m11] for real-diagonal /
 *   imaginary-off-diagonal 2x2 (rx-type, 4 reals)   D1R real diag (2 per variant)
 *   D2R real diag4 (4)   SCALER real scalar (1 per variant).
 * Variant index = bit(e1) + 2*bit(e2) of the thread's fixed state bits (-1: bit taken as 0). */
enum { QK_U1 = 0, QK_D1 = 1, QK_SLOT = 2, QK_U2 = 3, QK_D2 = 4, QK_CX = 5, QK_SWAP = 6, QK_SCALE = 7,
       QK_U1R = 8, QK_U1X = 9, QK_D1R = 10, QK_D2R = 11, QK_SCALER = 12 };

typedef struct qk_op {      /* 32 bytes */
    int32_t kind;
    int32_t a, b;            /* fiber positions (0..3) */
    int32_t e1, e2;          /* external state bits selecting a variant (-1: none) */
    int32_t slot;            /* QK_SLOT: slot index into the job's slot table */
    int32_t mat;             /* offset (doubles) into qk_program.mats */
    int32_t pad;
} qk_op;

typedef struct qk_group {   /* 32 bytes: one fiber (4 tile positions) and its ops */
    int32_t pos[4];
    int32_t op_begin, op_end;
    int32_t pad[2];
} qk_group;

typedef struct qk_pass {    /* 24 bytes */
    uint64_t tile_mask;      /* state bits resident in the tile (SPLIT mode) */
    int32_t group_begin, group_end;
    int32_t flags;           /* 1: INIT (state starts as |0..0>), 2: FINAL (emit probabilities) */
    uint32_t traced_local;   /* FINAL: tile positions that are traced out */
} qk_pass;

typedef struct qk_program {
    int32_t n;               /* fragment qubits */
    int32_t n_eff;           /* padded width (PACKED: >= 4) */
    int32_t m;               /* measured qubits = local qubits 0..m-1 */
    int32_t n_slots;         /* virtual-gate endpoints in this fragment */
    int32_t packed;          /* 1: n_eff <= 12, whole jobs per tile */
    int32_t n_passes;
    const qk_pass* passes;   /* HOST */
    const qk_op* ops;        /* DEVICE */
    const qk_group* groups;  /* DEVICE */
    const double* mats;      /* DEVICE */
} qk_program;

typedef struct qk_ctx qk_ctx;

int qk_ctx_create(int device, qk_ctx** out);
int qk_ctx_destroy(qk_ctx* ctx);
/* Launch on an external hipStream_t (e.g. torch's current stream); NULL selects the null stream.
 * A new context launches on its own non-blocking stream until this is called. */
int qk_ctx_set_stream(qk_ctx* ctx, void* hip_stream);
int qk_ctx_synchronize(qk_ctx* ctx);
const char* qk_last_error(qk_ctx* ctx);

/* A HIP stream restricted to a set of compute units (hipExtStreamCreateWithCUMask): bit i of
 * cu_mask (mask_words 32-bit words) enables logical CU i. Kernels launched through a context bound
 * to such a stream (qk_ctx_set_stream) size their persistent grids to its CU count. The pipelined
 * step runs the write-bound knit on one CU set and the next step's sweep + data-rank
 * preparation on the others. qk_stream_cu_count: the CUs a stream may use (all for NULL). */
int qk_stream_create_cu_masked(int device, const uint32_t* cu_mask, int mask_words, void** stream);
int qk_stream_destroy(void* stream);
int qk_stream_cu_count(int device, void* stream, int* cus);
const char* qk_version(void);

/* Output buffers for the write-bound knit kernels (qknit_mem.hip): at least `bytes` of device memory
 * built from 1-GiB physical allocations (hipMemCreate) mapped read-write (below 1 GiB: one
 * allocation). Replaces the output dict the reference allocates per merge (quasi_distr.py:55-60): the
 * caller owns the buffer; qk_out_free synchronizes the device, unmaps it and releases its memory (its
 * address range is never handed out again). qk_out_mapped_bytes: the mapped size of a qk_out_alloc
 * pointer (QK_EARG otherwise). qk_out_write_rate: GB/s of the knit's store order into [ptr, ptr +
 * bytes) (one timed launch; overwrites the contents; the range must lie in one live qk_out_alloc
 * mapping; the device is drained first and an error left by earlier work is reported as
 * "pre-existing") — the 2^32-entry knit writes at 4.8-5.0 ms into most buffers and at 5.2-5.9 ms into
 * others, fixed per buffer, whatever the store order, so the engine keeps a large
 * output only if it writes fast (engine.out_buffer). qk_out_stats: process counters into out[0, n):
 * reservations made, reservations failed, chunk maps failed, live mappings, live bytes, retired
 * ranges, retired bytes, largest mapping, write-rate calls that found a pre-existing error. */
int qk_out_alloc(qk_ctx* ctx, int64_t bytes, void** ptr);
int qk_out_free(qk_ctx* ctx, void* ptr);
int qk_out_mapped_bytes(const void* ptr, int64_t* bytes);
int qk_out_write_rate(qk_ctx* ctx, void* ptr, int64_t bytes, double* gbs);
int qk_out_stats(int64_t* out, int n);

/* Workspace (bytes) qk_sweep needs for n_jobs jobs of prog (0 in PACKED mode). */
int qk_sweep_workspace_bytes(const qk_program* prog, int64_t n_jobs, int64_t* bytes);

/* Batched exact sweep of one fragment.
 *   job_slots : [n_jobs][n_slots][2][2] complex (8 doubles per slot)
 *   job_sign  : [n_jobs]
 *   pjob      : [n_jobs][2^m] out: sign * P(x), traced over unmeasured qubits */
int qk_sweep(qk_ctx* ctx, const qk_program* prog, int64_t n_jobs, const double* job_slots,
             const double* job_sign, void* workspace, int64_t workspace_bytes, double* pjob);

/* ---- per-program sweep kernels (run-time compiled; qknit_jit.hip, sweep_codegen.py) --------
 * Same contract as qk_sweep for SPLIT programs (n > 12), but the passes run as kernels
 * specialised to one fragment program (tile layout, fibers, ops and matrices as constants). */
typedef struct qk_module qk_module;

/* Compile HIP source with hiprtc for gfx950 and load it; names: its extern "C" kernels. */
int qk_module_compile(qk_ctx* ctx, const char* source, const char* const* names, int n_names,
                      qk_module** out);
int qk_module_destroy(qk_module* module);
/* A module from a code object compiled earlier (qk_module_code of a compiled module, or the same
 * source compiled ahead of time: hipcc --genco --offload-arch=gfx950 -O3 -std=c++17 plus the
 * source's qk-options line), without hiprtc. */
int qk_module_load(qk_ctx* ctx, const void* image, int64_t image_bytes, const char* const* names, int n_names,
                   qk_module** out);
/* The code object a module was loaded from: *bytes = its size; copied to buf when buf is non-NULL
 * (*bytes at least that size on entry). */
int qk_module_code(const qk_module* module, void* buf, int64_t* bytes);

/* qk_sweep with pass i launched as module kernel i (kernel args: job_slots, job_sign, state,
 * pjob, n_jobs), same grid (sparse INIT pass: one tile per job). */
int qk_sweep_compiled(qk_ctx* ctx, const qk_module* module, const qk_program* prog, int64_t n_jobs,
                      const double* job_slots, const double* job_sign, void* workspace,
                      int64_t workspace_bytes, double* pjob);

/* qk_sweep_compiled fused with qk_reduce_labels: the FINAL pass runs per (label, tile) and sums the
 * label's branch jobs [label_offsets[l], label_offsets[l+1]) (DEVICE, n_labels+1) in registers, so
 * q[l][x] = sum_j sign_j P_j(x) is stored once and no per-job rows exist. */
int qk_sweep_compiled_labels(qk_ctx* ctx, const qk_module* module, const qk_program* prog, int64_t n_jobs,
                             const double* job_slots, const double* job_sign, int64_t n_labels,
                             const int64_t* label_offsets, void* workspace, int64_t workspace_bytes, double* q);

/* Up to 4 compiled SPLIT programs of one tile width swept together (module from
 * sweep_codegen.generate_multi): pass round r of every program that has one runs in ONE launch, each
 * program on its own block range, so independent fragments share launches. Per program f (HOST
 * arrays of device pointers): label_offsets[f] non-NULL -> outs[f] = per-label rows as
 * qk_sweep_compiled_labels; NULL -> per-job rows as qk_sweep_compiled.
 * block_maps (HOST array, one entry per pass round, or NULL): a non-NULL block_maps[r] (DEVICE,
 * one uint64 per block of round r) sends block b to program (map[b] >> 56), block
 * (map[b] & (2^56 - 1)) of that program's range, so the caller orders the work (e.g. the FINAL
 * pass's labels by descending branch-job count); entries outside a range are skipped. */
int qk_sweep_compiled_multi(qk_ctx* ctx, const qk_module* module, int n_prog, const qk_program* progs,
                            const int64_t* n_jobs, const double* const* job_slots, const double* const* job_sign,
                            const int64_t* n_labels, const int64_t* const* label_offsets, void* const* workspaces,
                            const int64_t* workspace_bytes, double* const* outs, const uint64_t* const* block_maps);

/* qk_sweep_compiled_multi with shared INIT tiles. The sparse INIT pass of a two-pass program depends
 * on a job only through the slot matrices its ops read (syc 32 5: 750 branch jobs, 50 distinct
 * prefixes). For program f with prefix_of[f] non-NULL (DEVICE, int32 per job), the INIT round runs
 * n_init[f] units whose slot rows are init_slots[f] (DEVICE, n_init x n_slots x 8 doubles) into
 * workspace state slots [0, n_init), and the FINAL pass of job j starts from slot prefix_of[f][j].
 * prefix_of[f] NULL: that program runs as in qk_sweep_compiled_multi. Results are bitwise those of
 * qk_sweep_compiled_multi when every job's INIT slot rows equal its prefix's. */
int qk_sweep_compiled_multi_shared(qk_ctx* ctx, const qk_module* module, int n_prog, const qk_program* progs,
                                   const int64_t* n_jobs, const double* const* job_slots,
                                   const double* const* job_sign, const int64_t* n_labels,
                                   const int64_t* const* label_offsets, void* const* workspaces,
                                   const int64_t* workspace_bytes, double* const* outs,
                                   const uint64_t* const* block_maps, const int64_t* n_init,
                                   const double* const* init_slots, const int32_t* const* prefix_of);

/* q[l][x] = sum_{j in [offsets[l], offsets[l+1])} pjob[j][x]   (offsets: DEVICE, n_labels+1) */
int qk_reduce_labels(qk_ctx* ctx, int64_t n_labels, const int64_t* offsets, int64_t width,
                     const double* pjob, double* q);

/* out[keyA[i] + keyB[j]] (=|+=) sum_k A[k*lda + i] * B[k*ldb + j],  i < M, j < N.
 * A NULL key table means an affine one: keyA[i] = i*strideA, keyB[j] = j*strideB.
 * beta: 0 overwrite, 1 accumulate. */
int qk_gemm_keyed(qk_ctx* ctx, int64_t M, int64_t N, int64_t K, const double* A, int64_t lda,
                  const double* B, int64_t ldb, const int64_t* keyA, int64_t strideA,
                  const int64_t* keyB, int64_t strideB, double* out, int beta);

/* qk_gemm_keyed predicated on a DEVICE flag: nothing is written when *skip > 0 (skip may be NULL).
 * The exact contraction of a step whose data-rank compression may be rejected on the device
 * (KnitPipeline: skip = the accepted rank, 0 when rejected), so no host synchronisation decides. */
int qk_gemm_keyed_pred(qk_ctx* ctx, int64_t M, int64_t N, int64_t K, const double* A, int64_t lda,
                       const double* B, int64_t ldb, const int64_t* keyA, int64_t strideA,
                       const int64_t* keyB, int64_t strideB, double* out, int beta, const int32_t* skip);

/* Small-K keyed outer product, output-write bound (1 <= K <= 8): the same result as
 * qk_gemm_keyed with beta = 0, for a key table whose column pairs are adjacent outputs:
 * keyB[2i + 1] == keyB[2i] + 1 and keyB[2i] even (the N side holds clbit 0; the caller checks,
 * the kernel writes each pair with one 16-B store). N even; B and out 16-B aligned. Used for the
 * data-rank-compressed two-fragment knit (pipeline.KnitPipeline); replaces the same
 * merge + knit as qk_gemm_keyed (virtual_circuit.py:50-68,165-171, quasi_distr.py:55-60). */
int qk_gemm_outer_paired(qk_ctx* ctx, int64_t M, int64_t N, int64_t K, const double* A, int64_t lda,
                         const double* B, int64_t ldb, const int64_t* keyA, int64_t strideA,
                         const int64_t* keyB, double* out);

/* Small-K two-fragment knit as one streaming write over all 2^nbits outputs (nbits <= 32,
 * 1 <= K <= 8): out[o] = sum_k A[k*lda + pext(o, maskA)] * B[k*ldb + pext(o, maskB)], where
 * maskA / maskB are the two fragments' clbit masks (disjoint, covering bits 0..nbits-1, bit 0 in
 * maskB; pext = the outcome index of the fragment's bits). Same result as qk_gemm_outer_paired with
 * deposit key tables; written in output order (contiguous 1-KiB runs per wave store). B and out
 * 16-B aligned, ldb even. Replaces the same merge + knit (virtual_circuit.py:50-68,165-171). */
int qk_knit_outer_stream(qk_ctx* ctx, int nbits, int64_t K, const double* A, int64_t lda, const double* B,
                         int64_t ldb, uint64_t maskA, uint64_t maskB, double* out);

/* qk_knit_outer_stream over the output range [o_begin, o_begin + o_count) only, written to
 * out[o - o_begin] (a rank's contiguous slice of the distribution: multi-GPU slice mode). k_dev
 * (DEVICE int32, or NULL) overrides K at run time (min(K, *k_dev)); *k_dev <= 0 makes the call write
 * nothing (a knit predicated on a device-side check, no host sync). Ranges and k_dev need the blocked
 * kernel: tasks of 2^TB outputs with 9 <= TB <= 16, TB at most the trailing zero bits of o_begin and
 * o_count, and the K x (2^a + 2^b) staged operand values within 24 KiB of LDS (2^16 for syc 32 5 at
 * K <= 8); QK_EARG when no such TB exists. */
int qk_knit_outer_stream_range(qk_ctx* ctx, int nbits, int64_t K, const double* A, int64_t lda, const double* B,
                               int64_t ldb, uint64_t maskA, uint64_t maskB, int64_t o_begin, int64_t o_count,
                               const int32_t* k_dev, double* out);

/* out[k][i + j*M] = A[k*lda + i] * B[k*ldb + j] */
/* The kernel qk_knit_outer_stream_range launches for these arguments (no launch): *kind = 0 the
 * per-output gather kernel (qk_knit_outer_stream_kernel), 1 the blocked kernel with A and B staged in
 * LDS (qk_knit_outer_blocked_kernel<false>), 2 the blocked kernel reading B from global memory
 * (<true>), 3 the rows kernel holding B runs in registers (qk_knit_outer_rows_kernel: B holds the
 * low output bits, syc 32 1); *task_bits = log2 outputs per task / piece (0 for kind 0). */
int qk_knit_outer_stream_kind(int nbits, int64_t K, uint64_t maskA, uint64_t maskB, int64_t o_begin,
                              int64_t o_count, int* kind, int* task_bits);
int qk_khatri_rao(qk_ctx* ctx, int64_t K, int64_t M, int64_t N, const double* A, int64_t lda,
                  const double* B, int64_t ldb, double* out);

/* dst[r][x] = coef[r] * src[idx[r]][x]  (width columns, rows R) */
int qk_gather_rows(qk_ctx* ctx, int64_t R, int64_t width, const int64_t* idx, const double* coef,
                   const double* src, double* dst);

/* ---- plan-level knit (qknit_plan.hip) -------------------------------------------------------
 * The whole knit of virtual_circuit.py:50-68 (merge + per-gate knits, i.e. qd:55-60 and
 * vg:105-124,179-194,262-286 over every global label) from the swept rows of each fragment:
 *   X_f = W_f^T q_f,  out[sum_f pdep(x_f, clbit_mask_f)] = sum_k prod_f X_f[k][x_f]
 * with the transforms W_f ([rows_f][terms], DEVICE, row-major) precomputed by the planner (label
 * gathers + knit coefficients, or the factored / basis / light-cone transforms: engine.knit_operands)
 * and q_f = qk_sweep / qk_sweep_compiled_labels output ([rows_f][2^popcount(mask_f)], DEVICE). Writes
 * every one of the 2^nbits outputs covered by the masks (clbits no fragment measures stay 0: pass a
 * zeroed out). 1..4 fragments; 3+ are Khatri-Rao folded; the contraction is qk_gemm_keyed (fp64 MFMA).
 * Replaces KnitPipeline.knit's exact path for non-Python hosts. */
typedef struct qk_knit_plan {
    int32_t n_frag;                  /* 1..4 */
    int32_t nbits;                   /* output clbits N: out has 2^N entries */
    int64_t terms;                   /* contraction terms K */
    const int64_t* rows;             /* HOST [n_frag]: swept rows per fragment */
    const uint64_t* clbit_masks;     /* HOST [n_frag]: global clbits each fragment measures (disjoint) */
    const double* const* transforms; /* HOST [n_frag] of DEVICE [rows_f][terms] */
} qk_knit_plan;

int qk_knit_workspace_bytes(const qk_knit_plan* plan, int64_t* bytes);
int qk_knit(qk_ctx* ctx, const qk_knit_plan* plan, const double* const* q, void* workspace, int64_t workspace_bytes,
            double* out);

/* ---- plan-level low-rank knit: the benched single-GPU step's knit in one call (qknit_plan.hip) ----
 * KnitPipeline's device data rank for a two-fragment knit, chained on the context's
 * stream with no host synchronisation: qk_prep_operands -> qk_rank_factors -> qk_compress_operands ->
 * qk_probe_errors -> qk_knit_outer_stream_range (write-bound, K = accepted rank) -> qk_gemm_keyed_pred
 * (the exact terms-wide contraction, runs only when the check rejected). Same result as qk_knit on the
 * same transforms within the probe tolerance. q_a / q_b: the swept rows ([rows][2^popcount(mask)]).
 * *rank_out (DEVICE int32, may be NULL): the accepted rank, 0 when the exact contraction ran.
 * Replaces virtual_circuit.py:50-68 (merge + per-gate knits) for hosts that are not Python. */
typedef struct qk_lowrank_plan {
    int32_t nbits;           /* output clbits (2 <= nbits <= 32): out has 2^nbits entries, all written */
    int32_t terms;           /* K: contraction terms (light-cone transforms), even, <= 64 */
    int64_t rows_a, rows_b;  /* swept rows of the two fragments */
    uint64_t mask_a, mask_b; /* clbit masks: disjoint, covering the nbits output bits, bit 0 in mask_b,
                                >= 7 bits each */
    const double* wt_a;      /* DEVICE [rows_a][terms] */
    const double* wt_b;      /* DEVICE [rows_b][terms] */
    const double* probes;    /* DEVICE [16][2^popcount(mask_b)]: fixed Gaussian probe vectors */
    double lam_tol, s_tol, s_abs;  /* qk_rank_factors tolerances (data_rank.py LAM_TOL / S_TOL / S_ABS) */
    double rank_tol;         /* probe acceptance bound, absolute floor (KnitPipeline.rank_tol) ... */
    double rank_tol_rel;     /* ... and relative to max_p ||R p|| (KnitPipeline.rank_tol_rel) */
} qk_lowrank_plan;

int qk_knit_lowrank_workspace_bytes(qk_ctx* ctx, const qk_lowrank_plan* plan, int64_t* bytes);
int qk_knit_lowrank(qk_ctx* ctx, const qk_lowrank_plan* plan, const double* q_a, const double* q_b, void* workspace,
                    int64_t workspace_bytes, double* out, int32_t* rank_out);

/* ---- collectives (qknit_comm.hip: RCCL over xGMI) ----------------------------------------------
 * The reference's Pool(8) sum of partial knits (run.py:64-67) across GPUs, for a host that is not
 * Python: one process per GPU; rank 0 calls qk_comm_unique_id and the host hands the 128 bytes to
 * every rank (MPI, a file, torch.distributed), then each calls qk_comm_init with its context. The
 * collectives run on the context's stream over fp64 element counts (sums). Reduce mode = each rank's
 * partial qk_knit over its label slice + qk_reduce to the root; slice mode's exchanges
 * are qk_alltoall (column blocks), qk_allreduce (Grams, probe errors) and qk_allgather (compressed
 * operands). */
#define QK_COMM_ID_BYTES 128
typedef struct qk_comm qk_comm;
int qk_comm_unique_id(uint8_t* id);
int qk_comm_init(qk_ctx* ctx, const uint8_t* id, int nranks, int rank, qk_comm** out);
int qk_comm_destroy(qk_comm* comm);
int qk_comm_size(qk_comm* comm, int* nranks, int* rank);
int qk_allreduce(qk_ctx* ctx, qk_comm* comm, const double* send, double* recv, int64_t count);
int qk_reduce(qk_ctx* ctx, qk_comm* comm, const double* send, double* recv, int64_t count, int root);
int qk_allgather(qk_ctx* ctx, qk_comm* comm, const double* send, double* recv, int64_t count);
int qk_alltoall(qk_ctx* ctx, qk_comm* comm, const double* send, double* recv, int64_t count);

/* ---- data-rank factors (qknit_rank.hip; data_rank.py is the host form) ----------------------
 * Two-fragment knit R = A^T B (A: [K][M], B: [K][N] operands of virtual_circuit.py:50-68's knit)
 * from its Gram matrices GA = A A^T, GB = B B^T ([K][K], DEVICE): pivoted Cholesky of each Gram
 * (stopped when the residual trace is <= lam_tol * max diagonal, at most 32 steps), core SVD by
 * one-sided Jacobi, rank r = #{s > max(s_tol s_0, s_abs)}; writes TA, TB ([rmax][K], DEVICE, rows >= r
 * zero) with R ~= (TA A)^T (TB B), and *r_out (DEVICE int32) = r, or 0 when there is no usable
 * factorisation (R = 0, no convergence, r > rmax). One workgroup; K <= 64, rmax <= 8. The caller
 * verifies the product before trusting it (KnitPipeline: probes on the real operands). */
int qk_rank_factors(qk_ctx* ctx, int64_t K, const double* GA, const double* GB, double lam_tol, double s_tol,
                    double s_abs, int rmax, double* TA, double* TB, int32_t* r_out);

/* Operand preparation of the data-rank step in one pass over the swept rows (csrc/qknit_prep.hip):
 *   X_A = Wt_A^T q_A ([K][NA]), X_B = Wt_B^T q_B ([K][NB]) (Wt: [R][K], q: [R][ldq] row-major),
 *   GA = X_A X_A^T, GB = X_B X_B^T ([K][K]), U = X_B P^T ([K][16], P = probes [16][NB]).
 * K <= 64; NA, NB positive multiples of 128. work: qk_prep_workspace_bytes (per-workgroup partial
 * sums, reduced in a fixed order: results are deterministic). All pointers DEVICE. */
int qk_prep_workspace_bytes(qk_ctx* ctx, int64_t NA, int64_t NB, int64_t* bytes);
int qk_prep_operands(qk_ctx* ctx, int K, int RA, const double* WtA, const double* qA, int64_t ldqA, int64_t NA,
                     double* XA, int RB, const double* WtB, const double* qB, int64_t ldqB, int64_t NB, double* XB,
                     const double* probes, double* GA, double* GB, double* U, double* work, int64_t work_bytes);

/* The same preparation without materialising X_s (round 5, "q-space"; swept rows R_s <= 80 per side):
 * qk_qprep_grams forms G_A, G_B [K][K] and U [K][16] from Gq_s = q_s q_s^T and Pq = q_B P^T (one MFMA
 * pass over q, a fixed-order reduction, G_s = Wt_s^T Gq_s Wt_s); qk_qprep_compress_check forms
 * A2 = (TA Wt_A^T) q_A, B2 = (TB Wt_B^T) q_B ([rmax][N], rmax <= 8) and the acceptance check of
 * qk_probe_errors over every column of A from the materialised A2 / B2 (e2: 32 doubles or NULL; with
 * k_out the accepted rank as qk_probe_errors). NA, NB multiples of 512 for the check, 128 for the
 * Grams. work: qk_qprep_workspace_bytes (covers both calls). All pointers DEVICE. */
int qk_qprep_workspace_bytes(qk_ctx* ctx, int64_t NA, int64_t NB, int64_t* bytes);
int qk_qprep_grams(qk_ctx* ctx, int K, int RA, const double* WtA, const double* qA, int64_t ldqA, int64_t NA, int RB,
                   const double* WtB, const double* qB, int64_t ldqB, int64_t NB, const double* probes, double* GA,
                   double* GB, double* U, double* work, int64_t work_bytes);
int qk_qprep_compress_check(qk_ctx* ctx, int K, int rmax, int RA, const double* WtA, const double* qA, int64_t ldqA,
                            int64_t NA, int RB, const double* WtB, const double* qB, int64_t ldqB, int64_t NB,
                            const double* TA, const double* TB, const double* U, const double* probes, double* A2,
                            double* B2, double* e2, const int32_t* r_dev, double tol, double rel_tol, int32_t* k_out,
                            double* err_out, double* work, int64_t work_bytes);

/* A2 = TA X_A ([rmax][NA]), B2 = TB X_B ([rmax][NB]) for [rmax][K] factors (rmax <= 8), one launch. */
int qk_compress_operands(qk_ctx* ctx, int K, int rmax, const double* TA, const double* XA, int64_t NA, double* A2,
                         const double* TB, const double* XB, int64_t NB, double* B2);
/* The same with leading dimensions: rows of X_A, A2, X_B, B2 ldxa / lda2 / ldxb / ldb2 apart (a replicated
 * multi-GPU rank compresses only the A columns its output slice reads, into those columns of a full-width
 * A2; the pointers are offset to the first column). */
int qk_compress_operands_ld(qk_ctx* ctx, int K, int rmax, const double* TA, const double* XA, int64_t NA, int64_t ldxa,
                            double* A2, int64_t lda2, const double* TB, const double* XB, int64_t NB, int64_t ldxb,
                            double* B2, int64_t ldb2);

/* qk_compress_operands_ld with the probe check's V pass fused in: also vpart[b][j][p] = sum over the b-th
 * 512-column block of B of B2[j][c] probes[p][c] (j < 8, rows >= rmax zero; ceil(NB / 512) blocks of 128
 * doubles), which qk_probe_errors_vpart takes instead of reading B2 and the probes again. Even widths and
 * leading dimensions, 16-B aligned operands. */
int qk_compress_probe_v(qk_ctx* ctx, int K, int rmax, const double* TA, const double* XA, int64_t NA, int64_t ldxa,
                        double* A2, int64_t lda2, const double* TB, const double* XB, int64_t NB, int64_t ldxb,
                        double* B2, int64_t ldb2, const double* probes, int64_t ldp, double* vpart,
                        int64_t vpart_doubles);

/* qk_probe_errors_tally from qk_compress_probe_v's gv V partials (no B2 / probes pass of its own). */
int qk_probe_errors_vpart(qk_ctx* ctx, int K, int rmax, const double* XA, int64_t ldx, int64_t NA, const double* A2,
                          int64_t lda2, const double* U, const double* vpart, int64_t gv, double* e2,
                          const int32_t* r_dev, double tol, double rel_tol, int32_t* k_out, double* err_out,
                          double* work, int64_t work_bytes, int64_t* tally);

/* Acceptance check of a compressed knit on the real operands (the probe products of the torch form,
 * not materialised): e2[p] = ||(X_A^T X_B - A2^T B2) P_p||^2 and e2[16 + p] = ||X_A^T X_B P_p||^2
 * (the reference product, ~||R||_F^2), summed over the NA columns of X_A given (X_A: [K][ldx], A2:
 * [rmax][lda2] the same columns; U = X_B P^T [K][16] over ALL columns of X_B; B2: [rmax][ldb2] and P:
 * [16][ldp] over all NB columns); e2 holds 32 doubles. With k_out: *err_out = sqrt(max_p e2[p]) and
 * *k_out = (*r_dev > 0 && err <= max(tol, rel_tol sqrt(max_p e2[16 + p]))) ? *r_dev : 0 (the accepted
 * rank; 0 = exact contraction). qk_probe_accept does that last step on e2 rows summed elsewhere
 * (multi-GPU: all-reduced partial e2 of each rank's columns; n rows of 32). e2 / r_dev / k_out /
 * err_out: DEVICE. */
int qk_probe_workspace_bytes(qk_ctx* ctx, int64_t NA, int64_t* bytes);
int qk_probe_errors(qk_ctx* ctx, int K, int rmax, const double* XA, int64_t ldx, int64_t NA, const double* A2,
                    int64_t lda2, const double* U, const double* B2, int64_t ldb2, int64_t NB, const double* probes,
                    int64_t ldp, double* e2, const int32_t* r_dev, double tol, double rel_tol, int32_t* k_out,
                    double* err_out, double* work, int64_t work_bytes);
/* qk_probe_errors with the step's data-rank statistics updated in the same launch (qk_rank_tally's
 * contract on tally, DEVICE int64[4]; needs k_out): one dependent launch fewer per step. */
int qk_probe_errors_tally(qk_ctx* ctx, int K, int rmax, const double* XA, int64_t ldx, int64_t NA, const double* A2,
                          int64_t lda2, const double* U, const double* B2, int64_t ldb2, int64_t NB,
                          const double* probes, int64_t ldp, double* e2, const int32_t* r_dev, double tol,
                          double rel_tol, int32_t* k_out, double* err_out, double* work, int64_t work_bytes,
                          int64_t* tally);
int qk_probe_accept(qk_ctx* ctx, const double* e2, int n, const int32_t* r_dev, double tol, double rel_tol,
                    int32_t* k_out, double* err_out);
/* Device-side statistics of a step's data rank (r: factorisation rank, k: accepted rank, both DEVICE
 * int32): acc[0] += (r == 0), acc[1] += (r > 0 && k == 0), acc[2] = k, acc[3] += 1 (acc: DEVICE int64[4]),
 * so steps in a loop never read their verdicts back; the host reads acc when it needs the counts. */
int qk_rank_tally(qk_ctx* ctx, const int32_t* r_dev, const int32_t* k_dev, int64_t* acc);

/* ---- post-processing (reference-shaped results; quasi_distr.py:3-43, run.py:71) ---------- */

/* Workspace for qk_threshold_count / qk_npd over n dense values with `count` kept entries. */
int qk_npd_workspace_bytes(int64_t n, int64_t count, int64_t* bytes);

/* *count_dev (device int64) = #{i : |vals[i]| > acc}  (QuasiDistr truncation, quasi_distr.py:7-10) */
int qk_threshold_count(qk_ctx* ctx, int64_t n, const double* vals, double acc, void* ws, int64_t ws_bytes,
                       int64_t* count_dev);

/* Truncate at acc, then nearest_probability_distribution (quasi_distr.py:28-43): writes the kept
 * (key, value) pairs ascending by value into out_keys/out_vals (capacity count) and their number
 * into *n_out_dev (device int64). count must be qk_threshold_count's result. */
int qk_npd(qk_ctx* ctx, int64_t n, const double* vals, double acc, int64_t count, void* ws, int64_t ws_bytes,
           int64_t* out_keys, double* out_vals, int64_t* n_out_dev);

/* The entries |vals[i]| > acc of a dense vector as (i + key_base, vals[i]) pairs, unordered, into keys /
 * out_vals (DEVICE, capacity entries); *count_dev (DEVICE int64, set here) = their number, which may
 * exceed capacity (then call again with more room). The multi-GPU dict result's exact fallback: a
 * rank's dense output slice starting at output key_base (pipeline.KnitPipeline.knit_dict). */
int qk_select_above(qk_ctx* ctx, int64_t n, const double* vals, double acc, int64_t key_base, int64_t capacity,
                    int64_t* keys, double* out_vals, int64_t* count_dev);

/* ---- shot sampling (qknit_sample.hip; run.py:42 `backend.run(instantiations, shots)` +
 * quasi_distr.py:12-20 `from_counts`) ----------------------------------------------------------
 * An instance s owns the pjob rows [seg_off[s], seg_off[s+1]) (its branch jobs, width values each);
 * its outcome distribution over (row, x) is |pjob|. Reference label l samples instance
 * label_seg[l] `shots` times and owns the count rows [label_row_off[l], label_row_off[l+1]). */

/* cdf[i] = inclusive prefix sum of |pjob| within each instance (same layout as pjob). */
int qk_sample_cdf(qk_ctx* ctx, int64_t n_seg, const int64_t* seg_off, int64_t width, const double* pjob,
                  double* cdf);

/* counts[label_row_off[l]*width + i] += #{draws s < shots : i = first index with cdf > u * total},
 * u = u(seed, label_base + l, s) a counter-based SplitMix64 stream: results do not depend on
 * scheduling or on how labels are split over calls. counts must be zeroed by the caller. */
int qk_sample_counts(qk_ctx* ctx, int64_t n_labels, int64_t label_base, const int64_t* label_seg,
                     const int64_t* seg_off, const int64_t* label_row_off, int64_t width, const double* cdf,
                     int64_t shots, uint64_t seed, unsigned int* counts);

/* q[l][x] = sum_r row_sign[r] * f_r(x) over the label's count rows, f = counts / shots, keeping only
 * f > acc (from_counts truncation at ACCURACY): the config-bit sign fold of the knit. */
int qk_fold_counts(qk_ctx* ctx, int64_t n_labels, const int64_t* label_row_off, int64_t width,
                   const double* row_sign, const unsigned int* counts, int64_t shots, double acc, double* q);

/* ---- thresholded knit (qknit_select.hip): the dict result without the dense 2^N vector --------
 * Every output v = sum_{k<K} A[k*lda + i] B[k*ldb + j] (i < 2^popcount(maskA), j < 2^popcount(maskB),
 * key = pdep(i, maskA) | pdep(j, maskB)) with |v| > acc is appended to keys / vals (DEVICE, capacity
 * entries); *count_dev (DEVICE int64) = the number of such outputs, which may exceed capacity (then
 * only capacity entries were written: call again with more room). This is the knit of
 * virtual_circuit.py:50-68 fused with QuasiDistr's ACCURACY truncation (quasi_distr.py:7-10): values
 * are formed exactly as the dense qk_knit_outer_stream_range writes them (bit-identical), in
 * unspecified order. Tiles whose per-column-block bound sum_k max|A[k]| max|B[k]| cannot exceed acc
 * are skipped without forming their outputs. k_dev (DEVICE int32 or NULL) overrides K at run time;
 * *k_dev <= 0 writes nothing (count 0): the caller falls back to the exact dense contraction.
 * K <= 8; masks disjoint, inside the nbits output bits. work: qk_knit_select_workspace_bytes. */
int qk_knit_select_workspace_bytes(int nbits, uint64_t maskA, uint64_t maskB, int64_t* bytes);
int qk_knit_select(qk_ctx* ctx, int nbits, int64_t K, const double* A, int64_t lda, const double* B, int64_t ldb,
                   uint64_t maskA, uint64_t maskB, double acc, const int32_t* k_dev, void* work, int64_t work_bytes,
                   int64_t capacity, int64_t* keys, double* vals, int64_t* count_dev);

/* nearest_probability_distribution (quasi_distr.py:28-43) on count (key, value) pairs (DEVICE, e.g.
 * qk_knit_select's output, already truncated): writes the kept pairs ascending by value (ties by key)
 * into out_keys / out_vals (capacity count) and their number into *n_out_dev (DEVICE int64). */
int qk_npd_pairs_workspace_bytes(int64_t count, int64_t* bytes);
int qk_npd_pairs(qk_ctx* ctx, int64_t count, const int64_t* keys, const double* vals, void* ws, int64_t ws_bytes,
                 int64_t* out_keys, double* out_vals, int64_t* n_out_dev);

/* acc3[0] = sum sqrt(max(p,0) max(q,0)), acc3[1] = sum max(p,0), acc3[2] = sum max(q,0) (device).
 * Hellinger fidelity = (acc3[0] / sqrt(acc3[1] acc3[2]))^2 (Utilities.py:222-224). */
/* Reference truncation semantics (qknit_trunc.hip): dense quasi-distributions whose entries with
 * |v| <= acc are zero after every operation, as the reference's QuasiDistr drops them from its dict on
 * every construction (quasi_distr.py:7-10). One rounding per reference operation.
 *   qk_qd_from_rows  out[dst[r] * width + x] = trunc(rows[r * width + x])       (from_counts, :12-20)
 *   qk_qd_merge      out = 0, then out[ka[i] ^ kb[j]] = trunc(a[i] * b[j]) for every nonzero product
 *                    (ka / kb NULL: identity keys): the dict merge of :55-60, whose entries are the
 *                    kept products; two nonzero products must not share a key
 *   qk_qd_axpby      out[i] = trunc(alpha * a[i] + beta * b[i]) as fma(alpha, a, beta * b): +, - with
 *                    (1, +-1), scalar * with (s, 0) (:62-86 and the per-gate knits,
 *                    virtual_gates.py:105-124,179-194,262-286) */
int qk_qd_from_rows(qk_ctx* ctx, int64_t n_rows, int64_t width, const double* rows, const int64_t* dst, double acc,
                    double* out);
int qk_qd_merge(qk_ctx* ctx, int64_t na, const double* a, const int64_t* ka, int64_t nb, const double* b,
                const int64_t* kb, double acc, int64_t n_out, double* out);
int qk_qd_axpby(qk_ctx* ctx, int64_t n, double alpha, const double* a, double beta, const double* b, double acc,
                double* out);

int qk_hellinger(qk_ctx* ctx, int64_t n, const double* p, const double* q, double* acc3);

#ifdef __cplusplus
}
#endif
#endif /* QKNIT_H */
