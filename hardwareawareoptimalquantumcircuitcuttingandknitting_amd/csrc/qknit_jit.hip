// qknit_jit.hip — per-program sweep kernels compiled at run time (hiprtc, gfx950).
//
// The interpreter kernel (qk_sweep_pass_kernel) reads every op descriptor and matrix at run
// time and dispatches on it; on syc 32 5 it spends most of its issue slots on that and on
// index arithmetic (PMC: 12% of VALU instructions are f64 FMAs, 49% of wave time waiting).
// sweep_codegen.py instead emits one kernel per pass with the tile layout, fiber positions,
// op sequence and gate matrices as constants (the same ops, from sweep_ops.h); this file
// compiles such source with hiprtc, loads the code object, and launches its passes with
// qk_sweep's grid and argument contract.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "internal.h"

// tile widths of the per-program kernels: 2^(bits - 4) threads of 16 amplitudes, 2^bits x 16 B of LDS
#define QK_JIT_TILE_MIN 10
#define QK_JIT_TILE_MAX 13

struct qk_module {
    hipModule_t mod = nullptr;
    std::vector<hipFunction_t> fns;
    std::vector<char> code;  // the code object it was loaded from (qk_module_code)
};

namespace {

int jfail(qk_ctx* ctx, int code, const std::string& msg) {
    if (ctx) ctx->err = msg;
    return code;
}

}  // namespace

extern "C" {

int qk_module_compile(qk_ctx* ctx, const char* source, const char* const* names, int n_names,
                      qk_module** out) {
    if (!ctx || !source || !names || n_names < 1 || !out) return QK_EARG;
    *out = nullptr;
    if (hipSetDevice(ctx->device) != hipSuccess) return jfail(ctx, QK_EHIP, "qk_module_compile: hipSetDevice");
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, source, "qk_sweep_jit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
        return jfail(ctx, QK_EHIP, "qk_module_compile: hiprtcCreateProgram failed");
    for (int i = 0; i < n_names; ++i) hiprtcAddNameExpression(prog, names[i]);
    // extra compiler options from a first source line "// qk-options: -fa -fb" (sweep_codegen asks
    // for -fno-signed-zeros -ffinite-math-only so known-zero amplitudes fold away)
    std::vector<std::string> extra;
    const std::string tag = "// qk-options:";
    const std::string src(source);
    if (src.compare(0, tag.size(), tag) == 0) {
        const std::string line = src.substr(tag.size(), src.find('\n') - tag.size());
        size_t i = 0;
        while (i < line.size()) {
            while (i < line.size() && line[i] == ' ') ++i;
            size_t j = i;
            while (j < line.size() && line[j] != ' ') ++j;
            if (j > i) extra.push_back(line.substr(i, j - i));
            i = j;
        }
    }
    std::vector<const char*> opts = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
    for (const std::string& o : extra) opts.push_back(o.c_str());
    const hiprtcResult rc = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
    if (rc != HIPRTC_SUCCESS) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string log(n, '\0');
        if (n) hiprtcGetProgramLog(prog, &log[0]);
        hiprtcDestroyProgram(&prog);
        return jfail(ctx, QK_EARG, "qk_module_compile: " + std::string(hiprtcGetErrorString(rc)) + "\n" + log);
    }
    size_t code_size = 0;
    hiprtcGetCodeSize(prog, &code_size);
    std::vector<char> code(code_size);
    hiprtcGetCode(prog, code.data());
    hiprtcDestroyProgram(&prog);
    return qk_module_load(ctx, code.data(), (int64_t)code.size(), names, n_names, out);
}

int qk_module_load(qk_ctx* ctx, const void* image, int64_t image_bytes, const char* const* names, int n_names,
                   qk_module** out) {
    if (!ctx || !image || image_bytes <= 0 || !names || n_names < 1 || !out) return QK_EARG;
    *out = nullptr;
    if (hipSetDevice(ctx->device) != hipSuccess) return jfail(ctx, QK_EHIP, "qk_module_load: hipSetDevice");
    qk_module* m = new qk_module();
    m->code.assign((const char*)image, (const char*)image + image_bytes);
    if (hipModuleLoadData(&m->mod, m->code.data()) != hipSuccess) {
        delete m;
        return jfail(ctx, QK_EHIP, "qk_module_load: hipModuleLoadData failed");
    }
    for (int i = 0; i < n_names; ++i) {
        hipFunction_t f;
        if (hipModuleGetFunction(&f, m->mod, names[i]) != hipSuccess) {
            hipModuleUnload(m->mod);
            delete m;
            return jfail(ctx, QK_EARG, std::string("qk_module_load: no kernel ") + names[i]);
        }
        m->fns.push_back(f);
    }
    *out = m;
    return QK_OK;
}

int qk_module_code(const qk_module* m, void* buf, int64_t* bytes) {
    if (!m || !bytes) return QK_EARG;
    if (buf) {
        if (*bytes < (int64_t)m->code.size()) return QK_EARG;
        memcpy(buf, m->code.data(), m->code.size());
    }
    *bytes = (int64_t)m->code.size();
    return QK_OK;
}

int qk_module_destroy(qk_module* m) {
    if (!m) return QK_EARG;
    if (m->mod) (void)hipModuleUnload(m->mod);
    delete m;
    return QK_OK;
}

}  // extern "C"

namespace {

// Passes of a compiled program; with label_off the FINAL pass runs one workgroup per (label, tile)
// and sums the label's branch jobs (signed) before its single store.
int sweep_compiled(qk_ctx* ctx, const qk_module* module, const qk_program* p, int64_t n_jobs,
                   const double* job_slots, const double* job_sign, void* workspace, int64_t workspace_bytes,
                   double* pjob, int64_t n_labels, const int64_t* label_off) {
    if (!ctx) return QK_EARG;
    if (!module || !p || !p->passes || p->n_passes < 1) return jfail(ctx, QK_EARG, "qk_sweep_compiled: empty program");
    if ((int)module->fns.size() != p->n_passes)
        return jfail(ctx, QK_EARG, "qk_sweep_compiled: module does not hold one kernel per pass");
    if (n_jobs <= 0) return QK_OK;
    if (p->packed || p->n <= QK_TILE_BITS || p->n > 40)
        return jfail(ctx, QK_EARG, "qk_sweep_compiled: SPLIT programs only");
    if (!job_sign || !pjob || (p->n_slots > 0 && !job_slots))
        return jfail(ctx, QK_EARG, "qk_sweep_compiled: null buffer");
    const int64_t need = n_jobs * ((int64_t)1 << p->n) * (int64_t)(2 * sizeof(double));
    if (!workspace || workspace_bytes < need) return jfail(ctx, QK_EARG, "qk_sweep_compiled: workspace too small");
    if (hipSetDevice(ctx->device) != hipSuccess) return jfail(ctx, QK_EHIP, "qk_sweep_compiled: hipSetDevice");
    for (int ip = 0; ip < p->n_passes; ++ip) {
        const bool sparse_init = ip == 0 && p->n_passes > 1;  // qk_sweep: INIT tile of each job only
        const bool fin = ip == p->n_passes - 1;
        const int64_t units = (fin && label_off) ? n_labels : n_jobs;
        // tile width of this program (10 to 13 state bits): 2^(bits - 4) threads of 16 amplitudes
        const int tb = __builtin_popcountll(p->passes[ip].tile_mask);
        if (tb < QK_JIT_TILE_MIN || tb > QK_JIT_TILE_MAX || tb >= p->n)
            return jfail(ctx, QK_EARG, "qk_sweep_compiled: tiles must hold 10 to 13 state bits");
        const int64_t blocks = sparse_init ? n_jobs : (units << (p->n - tb));
        if (blocks > 0x7fffffff) return jfail(ctx, QK_EARG, "qk_sweep_compiled: too many tiles");
        struct {
            const double* slots;
            const double* sign;
            void* state;
            double* pjob;
            int64_t n_jobs;
            const int64_t* label_off;
        } args{job_slots, job_sign, workspace, pjob, n_jobs, fin ? label_off : nullptr};
        size_t size = sizeof(args);
        void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size,
                       HIP_LAUNCH_PARAM_END};
        const hipError_t e = hipModuleLaunchKernel(module->fns[ip], (unsigned)blocks, 1, 1, 1u << (tb - 4), 1, 1, 0,
                                                   ctx->stream, nullptr, cfg);
        if (e != hipSuccess) return jfail(ctx, QK_EHIP, std::string("qk_sweep_compiled: ") + hipGetErrorString(e));
    }
    return QK_OK;
}

}  // namespace

extern "C" {

int qk_sweep_compiled(qk_ctx* ctx, const qk_module* module, const qk_program* p, int64_t n_jobs,
                      const double* job_slots, const double* job_sign, void* workspace,
                      int64_t workspace_bytes, double* pjob) {
    return sweep_compiled(ctx, module, p, n_jobs, job_slots, job_sign, workspace, workspace_bytes, pjob, 0,
                          nullptr);
}

// Kernel argument of a multi-fragment pass launch (sweep_codegen.generate_multi declares the same).
#define QK_MULTI_MAX 4
struct qk_multi_args {
    const double* slots[QK_MULTI_MAX];
    const double* sign[QK_MULTI_MAX];
    void* state[QK_MULTI_MAX];
    double* out[QK_MULTI_MAX];
    const int64_t* label_off[QK_MULTI_MAX];
    int64_t n_jobs[QK_MULTI_MAX];
    int64_t begin[QK_MULTI_MAX];
    int64_t end[QK_MULTI_MAX];
    const uint64_t* map;  // block -> (program << 56 | block within its range), or NULL: ranges in order
    const double* islots[QK_MULTI_MAX];  // INIT round with shared prefixes: slot rows of the prefixes
    const int* pfx[QK_MULTI_MAX];        // FINAL round of a shared two-pass program: job -> prefix slot
};

}  // extern "C"

namespace {

int sweep_compiled_multi(qk_ctx* ctx, const qk_module* module, int n_prog, const qk_program* progs,
                         const int64_t* n_jobs, const double* const* job_slots, const double* const* job_sign,
                         const int64_t* n_labels, const int64_t* const* label_offsets, void* const* workspaces,
                         const int64_t* workspace_bytes, double* const* outs, const uint64_t* const* block_maps,
                         const int64_t* n_init, const double* const* init_slots, const int32_t* const* prefix_of) {
    if (!ctx) return QK_EARG;
    if (!module || !progs || n_prog < 1 || n_prog > QK_MULTI_MAX || !n_jobs || !job_slots || !job_sign ||
        !n_labels || !label_offsets || !workspaces || !workspace_bytes || !outs)
        return jfail(ctx, QK_EARG, "qk_sweep_compiled_multi: bad arguments");
    int rounds = 0, tb = 0;
    for (int f = 0; f < n_prog; ++f) {
        const qk_program& p = progs[f];
        if (p.packed || !p.passes || p.n_passes < 1 || p.n > 40)
            return jfail(ctx, QK_EARG, "qk_sweep_compiled_multi: SPLIT programs only");
        const int t = __builtin_popcountll(p.passes[0].tile_mask);
        if ((f && t != tb) || t < QK_JIT_TILE_MIN || t > QK_JIT_TILE_MAX || t >= p.n)
            return jfail(ctx, QK_EARG, "qk_sweep_compiled_multi: programs need one tile width of 10 to 13 bits");
        tb = t;
        if (n_jobs[f] < 1 || !job_sign[f] || !outs[f] || (p.n_slots > 0 && !job_slots[f]))
            return jfail(ctx, QK_EARG, "qk_sweep_compiled_multi: empty program or null buffer");
        if (label_offsets[f] && n_labels[f] < 1)
            return jfail(ctx, QK_EARG, "qk_sweep_compiled_multi: label offsets need n_labels >= 1");
        const int64_t need = n_jobs[f] * ((int64_t)1 << p.n) * (int64_t)(2 * sizeof(double));
        if (!workspaces[f] || workspace_bytes[f] < need)
            return jfail(ctx, QK_EARG, "qk_sweep_compiled_multi: workspace too small");
        if (prefix_of && prefix_of[f]) {
            // shared INIT prefixes: two-pass programs only (a middle pass would write per-job state
            // over the prefix slots); the prefixes' slot rows and count come with the map
            if (p.n_passes != 2 || !n_init || n_init[f] < 1 || n_init[f] > n_jobs[f] ||
                !init_slots || (p.n_slots > 0 && !init_slots[f]))
                return jfail(ctx, QK_EARG, "qk_sweep_compiled_multi_shared: bad shared-prefix arguments");
        }
        if (p.n_passes > rounds) rounds = p.n_passes;
    }
    if ((int)module->fns.size() != rounds)
        return jfail(ctx, QK_EARG, "qk_sweep_compiled_multi: module does not hold one kernel per pass round");
    if (hipSetDevice(ctx->device) != hipSuccess) return jfail(ctx, QK_EHIP, "qk_sweep_compiled_multi: hipSetDevice");
    for (int r = 0; r < rounds; ++r) {
        qk_multi_args a{};
        int64_t total = 0;
        // one tile width per round (a FINAL pass may be narrower than the INIT pass:
        // sweep_plan.narrow_final_tile); the round's kernel has 2^(tb - 4) threads
        tb = 0;
        for (int f = 0; f < n_prog; ++f) {
            const qk_program& p = progs[f];
            a.begin[f] = a.end[f] = total;
            if (p.n_passes <= r) continue;
            const int t = __builtin_popcountll(p.passes[r].tile_mask);
            if ((tb && t != tb) || t < QK_JIT_TILE_MIN || t > QK_JIT_TILE_MAX || t >= p.n)
                return jfail(ctx, QK_EARG, "qk_sweep_compiled_multi: programs need one tile width of 10 to 13 "
                                           "bits per pass round");
            tb = t;
            const bool sparse_init = r == 0 && p.n_passes > 1;
            const bool fin = r == p.n_passes - 1;
            const bool shared = prefix_of && prefix_of[f];
            const int64_t units = (fin && label_offsets[f]) ? n_labels[f] : n_jobs[f];
            total += sparse_init ? (shared ? n_init[f] : n_jobs[f]) : (units << (p.n - tb));
            a.end[f] = total;
            a.slots[f] = job_slots[f];
            a.islots[f] = (shared && sparse_init) ? init_slots[f] : nullptr;
            a.pfx[f] = (shared && fin) ? prefix_of[f] : nullptr;
            a.sign[f] = job_sign[f];
            a.state[f] = workspaces[f];
            a.out[f] = outs[f];
            a.label_off[f] = fin ? label_offsets[f] : nullptr;
            a.n_jobs[f] = n_jobs[f];
        }
        if (total > 0x7fffffff) return jfail(ctx, QK_EARG, "qk_sweep_compiled_multi: too many tiles");
        a.map = block_maps ? block_maps[r] : nullptr;
        size_t size = sizeof(a);
        void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size, HIP_LAUNCH_PARAM_END};
        const hipError_t e = hipModuleLaunchKernel(module->fns[r], (unsigned)total, 1, 1, 1u << (tb - 4), 1, 1, 0,
                                                   ctx->stream, nullptr, cfg);
        if (e != hipSuccess)
            return jfail(ctx, QK_EHIP, std::string("qk_sweep_compiled_multi: ") + hipGetErrorString(e));
    }
    return QK_OK;
}

}  // namespace

extern "C" {

int qk_sweep_compiled_multi(qk_ctx* ctx, const qk_module* module, int n_prog, const qk_program* progs,
                            const int64_t* n_jobs, const double* const* job_slots, const double* const* job_sign,
                            const int64_t* n_labels, const int64_t* const* label_offsets, void* const* workspaces,
                            const int64_t* workspace_bytes, double* const* outs,
                            const uint64_t* const* block_maps) {
    return sweep_compiled_multi(ctx, module, n_prog, progs, n_jobs, job_slots, job_sign, n_labels, label_offsets,
                                workspaces, workspace_bytes, outs, block_maps, nullptr, nullptr, nullptr);
}

int qk_sweep_compiled_multi_shared(qk_ctx* ctx, const qk_module* module, int n_prog, const qk_program* progs,
                                   const int64_t* n_jobs, const double* const* job_slots,
                                   const double* const* job_sign, const int64_t* n_labels,
                                   const int64_t* const* label_offsets, void* const* workspaces,
                                   const int64_t* workspace_bytes, double* const* outs,
                                   const uint64_t* const* block_maps, const int64_t* n_init,
                                   const double* const* init_slots, const int32_t* const* prefix_of) {
    if (!prefix_of || !n_init || !init_slots)
        return jfail(ctx, QK_EARG, "qk_sweep_compiled_multi_shared: null shared-prefix arrays");
    return sweep_compiled_multi(ctx, module, n_prog, progs, n_jobs, job_slots, job_sign, n_labels, label_offsets,
                                workspaces, workspace_bytes, outs, block_maps, n_init, init_slots, prefix_of);
}

int qk_sweep_compiled_labels(qk_ctx* ctx, const qk_module* module, const qk_program* p, int64_t n_jobs,
                             const double* job_slots, const double* job_sign, int64_t n_labels,
                             const int64_t* label_offsets, void* workspace, int64_t workspace_bytes, double* q) {
    if (!ctx) return QK_EARG;
    if (n_labels < 1 || !label_offsets)
        return jfail(ctx, QK_EARG, "qk_sweep_compiled_labels: need n_labels >= 1 and label offsets");
    if ((n_labels << (p ? (p->n > QK_TILE_BITS ? p->n - QK_TILE_BITS : 0) : 0)) > 0x7fffffff)
        return jfail(ctx, QK_EARG, "qk_sweep_compiled_labels: too many tiles");
    return sweep_compiled(ctx, module, p, n_jobs, job_slots, job_sign, workspace, workspace_bytes, q, n_labels,
                          label_offsets);
}

}  // extern "C"
