// qknit_comm.hip — collectives of the multi-GPU knit for a non-Python host (RCCL over xGMI).
//
// The reference sums its per-chunk knits in a process Pool(8) on one host (run.py:64-67,
// virtual_circuit.py:50-68); across GPUs the same reduction is an RCCL collective. KnitPipeline
// drives RCCL through torch.distributed; these entry points give a C / FFI host the same
// collectives on a qk_ctx's stream, so it can run the reduce mode (label-sliced partial knits + one
// qk_reduce) or assemble the slice mode's exchanges (qk_alltoall of column blocks, qk_allreduce of
// the Grams, qk_allgather of the compressed operands) itself:
//   qk_comm_unique_id   rank 0 creates the RCCL id; the host distributes its 128 bytes to every rank
//   qk_comm_init        one communicator per (process, GPU): ncclCommInitRank
//   qk_allreduce / qk_reduce / qk_allgather / qk_alltoall   fp64 sum collectives on ctx->stream
// One process per GPU, as RCCL requires; counts are fp64 elements.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>

#include "internal.h"

struct qk_comm {
    ncclComm_t comm;
    int nranks, rank, device;
};

namespace {

int cfail(qk_ctx* ctx, const std::string& msg, int code = QK_EARG) {
    if (ctx) ctx->err = msg;
    return code;
}

int nccl_status(qk_ctx* ctx, ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return QK_OK;
    return cfail(ctx, std::string(what) + ": " + ncclGetErrorString(r), QK_EHIP);
}

int check_comm(qk_ctx* ctx, qk_comm* comm, const char* what) {
    if (!comm) return cfail(ctx, std::string(what) + ": null communicator");
    if (comm->device != ctx->device) return cfail(ctx, std::string(what) + ": communicator of another device");
    return QK_OK;
}

}  // namespace

extern "C" {

int qk_comm_unique_id(uint8_t* id) {
    if (!id) return QK_EARG;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return QK_EHIP;
    std::memcpy(id, u.internal, QK_COMM_ID_BYTES);
    return QK_OK;
}

int qk_comm_init(qk_ctx* ctx, const uint8_t* id, int nranks, int rank, qk_comm** out) {
    if (!ctx) return QK_EARG;
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks)
        return cfail(ctx, "qk_comm_init: need the unique id, 0 <= rank < nranks and an output pointer");
    if (hipSetDevice(ctx->device) != hipSuccess) return cfail(ctx, "qk_comm_init: hipSetDevice", QK_EHIP);
    ncclUniqueId u;
    std::memcpy(u.internal, id, QK_COMM_ID_BYTES);
    qk_comm* c = new qk_comm{nullptr, nranks, rank, ctx->device};
    const int rc = nccl_status(ctx, ncclCommInitRank(&c->comm, nranks, u, rank), "qk_comm_init");
    if (rc) {
        delete c;
        return rc;
    }
    *out = c;
    return QK_OK;
}

int qk_comm_destroy(qk_comm* comm) {
    if (!comm) return QK_OK;
    const ncclResult_t r = ncclCommDestroy(comm->comm);
    delete comm;
    return r == ncclSuccess ? QK_OK : QK_EHIP;
}

int qk_allreduce(qk_ctx* ctx, qk_comm* comm, const double* send, double* recv, int64_t count) {
    if (!ctx) return QK_EARG;
    if (int rc = check_comm(ctx, comm, "qk_allreduce")) return rc;
    if (count < 0 || (count && (!send || !recv))) return cfail(ctx, "qk_allreduce: bad buffers / count");
    return nccl_status(ctx, ncclAllReduce(send, recv, (size_t)count, ncclFloat64, ncclSum, comm->comm, ctx->stream),
                       "qk_allreduce");
}

int qk_reduce(qk_ctx* ctx, qk_comm* comm, const double* send, double* recv, int64_t count, int root) {
    if (!ctx) return QK_EARG;
    if (int rc = check_comm(ctx, comm, "qk_reduce")) return rc;
    if (count < 0 || root < 0 || root >= comm->nranks || (count && !send) || (count && comm->rank == root && !recv))
        return cfail(ctx, "qk_reduce: bad buffers / count / root");
    return nccl_status(ctx, ncclReduce(send, recv, (size_t)count, ncclFloat64, ncclSum, root, comm->comm, ctx->stream),
                       "qk_reduce");
}

int qk_allgather(qk_ctx* ctx, qk_comm* comm, const double* send, double* recv, int64_t count) {
    if (!ctx) return QK_EARG;
    if (int rc = check_comm(ctx, comm, "qk_allgather")) return rc;
    if (count < 0 || (count && (!send || !recv))) return cfail(ctx, "qk_allgather: bad buffers / count");
    return nccl_status(ctx, ncclAllGather(send, recv, (size_t)count, ncclFloat64, comm->comm, ctx->stream),
                       "qk_allgather");
}

int qk_alltoall(qk_ctx* ctx, qk_comm* comm, const double* send, double* recv, int64_t count) {
    if (!ctx) return QK_EARG;
    if (int rc = check_comm(ctx, comm, "qk_alltoall")) return rc;
    if (count < 0 || (count && (!send || !recv))) return cfail(ctx, "qk_alltoall: bad buffers / count");
    return nccl_status(ctx, ncclAllToAll(send, recv, (size_t)count, ncclFloat64, comm->comm, ctx->stream),
                       "qk_alltoall");
}

int qk_comm_size(qk_comm* comm, int* nranks, int* rank) {
    if (!comm || !nranks || !rank) return QK_EARG;
    *nranks = comm->nranks;
    *rank = comm->rank;
    return QK_OK;
}

}  // extern "C"
