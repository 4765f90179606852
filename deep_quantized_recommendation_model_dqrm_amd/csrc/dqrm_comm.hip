// dqrm_comm.hip — the N > 1 exchange's collectives, issued by libdqrm itself on a RCCL
// communicator it owns (host code; no kernels here).
//
// Reference: sgd_quantized_gradients_parallel_comm.py quantize_emb_grad :850-890 issues two
// blocking collectives per table (all_reduce of the scale :865, sparse all_reduce of the
// quantized gradient :878), 52 per step, each a Python -> c10d -> Gloo round trip. Here the
// step is two ncclAllGather calls for all tables (per-slot maxima, then the fixed-capacity
// INT8 payloads), enqueued on the compute stream between the step's kernels by
// the same C call that launches them: one host call for the gradient half of the step
// (dqrm_exchange_grad) and one for the update (dqrm_exchange_apply).
//
// RCCL is taken from the process (PyTorch links librccl.so.1; dlopen with RTLD_NOLOAD finds
// that instance), else loaded from the ROCm install. Only a handful of entry points are used,
// resolved by name, so libdqrm has no link-time RCCL dependency and loads on hosts without it
// (the CPU test suite).
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <mutex>

#include "../../include/dqrm.h"

extern "C" int dqrm_internal_set_error(int code, const char* msg);  // dqrm_kernels.hip (hidden)

namespace {

// the subset of rccl.h used here (ABI-stable since NCCL 2.x)
typedef struct { char internal[128]; } RcclId;
typedef void* RcclComm;
typedef int RcclResult;                 // ncclSuccess = 0
constexpr int kRcclUint8 = 1;           // ncclUint8

struct Rccl {
    void* handle = nullptr;
    RcclResult (*get_unique_id)(RcclId*) = nullptr;
    RcclResult (*comm_init_rank)(RcclComm*, int, RcclId, int) = nullptr;
    RcclResult (*comm_destroy)(RcclComm) = nullptr;
    RcclResult (*all_gather)(const void*, void*, size_t, int, RcclComm, hipStream_t) = nullptr;
    const char* (*error_string)(RcclResult) = nullptr;
    bool ok = false;
};

Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // PyTorch's, when loaded
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        r.handle = h;
        r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
        r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
        r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
        r.all_gather = reinterpret_cast<decltype(r.all_gather)>(dlsym(h, "ncclAllGather"));
        r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
        r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_gather && r.error_string;
    });
    return r;
}

int fail(int code, const char* what, const char* detail) {
    char buf[384];
    snprintf(buf, sizeof(buf), "%s: %s", what, detail);
    return dqrm_internal_set_error(code, buf);
}

int rccl_fail(const char* what, RcclResult e) {
    return fail(DQRM_E_HIP, what, rccl().error_string ? rccl().error_string(e) : "RCCL error");
}

}  // namespace

struct dqrm_comm {
    RcclComm comm;              // RCCL (dqrm_comm_init), or null for a caller-served transport
    int nranks;
    int rank;
    dqrm_allgather_fn fn;       // caller-served all-gather (dqrm_comm_init_external), else null
    void* user;
};

extern "C" {

int dqrm_comm_unique_id(void* id128) {
    if (!id128) return fail(DQRM_E_INVALID, "dqrm_comm_unique_id", "null id");
    Rccl& r = rccl();
    if (!r.ok) return fail(DQRM_E_HIP, "dqrm_comm_unique_id", "RCCL (librccl.so.1) not available");
    RcclId id;
    const RcclResult e = r.get_unique_id(&id);
    if (e) return rccl_fail("ncclGetUniqueId", e);
    memcpy(id128, &id, sizeof(id));
    return DQRM_OK;
}

int dqrm_comm_init(dqrm_comm** comm, int nranks, int rank, const void* id128) {
    if (!comm || !id128 || nranks <= 0 || rank < 0 || rank >= nranks)
        return fail(DQRM_E_INVALID, "dqrm_comm_init", "bad arguments");
    Rccl& r = rccl();
    if (!r.ok) return fail(DQRM_E_HIP, "dqrm_comm_init", "RCCL (librccl.so.1) not available");
    RcclId id;
    memcpy(&id, id128, sizeof(id));
    RcclComm c = nullptr;
    const RcclResult e = r.comm_init_rank(&c, nranks, id, rank);
    if (e) return rccl_fail("ncclCommInitRank", e);
    *comm = new dqrm_comm{c, nranks, rank, nullptr, nullptr};
    return DQRM_OK;
}

int dqrm_comm_init_external(dqrm_comm** comm, int nranks, int rank, dqrm_allgather_fn fn, void* user) {
    if (!comm || !fn || nranks <= 0 || rank < 0 || rank >= nranks)
        return fail(DQRM_E_INVALID, "dqrm_comm_init_external", "bad arguments");
    *comm = new dqrm_comm{nullptr, nranks, rank, fn, user};
    return DQRM_OK;
}

int dqrm_comm_destroy(dqrm_comm* comm) {
    if (!comm) return DQRM_OK;
    const RcclResult e = comm->comm ? rccl().comm_destroy(comm->comm) : 0;
    delete comm;
    return e ? rccl_fail("ncclCommDestroy", e) : DQRM_OK;
}

int dqrm_comm_allgather(dqrm_comm* comm, const void* send, void* recv, size_t bytes, void* stream) {
    if (!comm || !send || !recv) return fail(DQRM_E_INVALID, "dqrm_comm_allgather", "null argument");
    if (comm->fn) {  // the caller's transport, called on this thread in stream order
        const int rc = comm->fn(send, recv, bytes, stream, comm->user);
        return rc ? fail(DQRM_E_HIP, "dqrm_comm_allgather", "the caller's all-gather failed") : DQRM_OK;
    }
    const RcclResult e = rccl().all_gather(send, recv, bytes, kRcclUint8, comm->comm, (hipStream_t)stream);
    return e ? rccl_fail("ncclAllGather", e) : DQRM_OK;
}

int dqrm_comm_size(const dqrm_comm* comm) { return comm ? comm->nranks : DQRM_E_INVALID; }

static int check_exchange(const dqrm_exchange* x, const char* who) {
    if (!x || !x->set) return fail(DQRM_E_INVALID, who, "null exchange / table set");
    if (x->comm ? x->num_ranks != x->comm->nranks : x->num_ranks != 1)
        return fail(DQRM_E_INVALID, who, "num_ranks does not match the communicator (1 without one)");
    if (x->comm && (!x->absmax_all || !x->gathered))
        return fail(DQRM_E_INVALID, who, "gather buffers (absmax_all, gathered) required with a communicator");
    if (!x->payload || !x->s_avg || !x->cap_base || x->cap_total < 0 || x->payload_bytes == 0)
        return fail(DQRM_E_INVALID, who, "null payload / s_avg / cap_base");
    if (x->grad_bits != 32 && (x->grad_bits < 2 || x->grad_bits > 16))
        return fail(DQRM_E_INVALID, who, "grad_bits must be 2..16 or 32");
    if (x->payload_bytes != dqrm_payload_bytes(x->set->num_tables, x->cap_total, x->set->dim, x->grad_bits))
        return fail(DQRM_E_INVALID, who, "payload_bytes does not match dqrm_payload_bytes(T, cap_total, D, grad_bits)");
    return DQRM_OK;
}

int dqrm_exchange_grad(const dqrm_exchange* x, const dqrm_batch* batch, const float* dy, int64_t dy_stride_t,
                       int64_t dy_stride_b, int ste, void* stream) {
    int rc = check_exchange(x, "dqrm_exchange_grad");
    if (rc) return rc;
    if (!x->ws_cap_base || !x->ws_rows || !x->ws_vals || !x->ws_ucount || !x->ws_absmax)
        return fail(DQRM_E_INVALID, "dqrm_exchange_grad", "null coalesce workspace");
    const int T = x->set->num_tables, S = DQRM_TABLE_SPLIT;
    if ((rc = dqrm_emb_bwd_coalesce(x->set, batch, dy, dy_stride_t, dy_stride_b, ste, x->ws_cap_base, x->ws_rows,
                                    x->ws_vals, x->ws_ucount, x->ws_absmax, x->workspace, x->workspace_bytes,
                                    stream)))
        return rc;
    const float* am = x->ws_absmax;
    if (x->comm && x->grad_bits != 32) {  // 1. the ranks' per-slot max|grad|
        if ((rc = dqrm_comm_allgather(x->comm, x->ws_absmax, x->absmax_all, (size_t)T * S * sizeof(float), stream)))
            return rc;
        am = x->absmax_all;
    }
    if ((rc = dqrm_grad_quant_pack_strided(T, x->set->dim, x->ws_cap_base, x->ws_cap_total, x->ws_rows, x->ws_vals,
                                           x->ws_ucount, am, (int64_t)T * S, x->num_ranks, x->grad_bits,
                                           x->cap_base, x->cap_total, x->s_avg, x->payload, stream)))
        return rc;
    if (x->comm)  // 2. the fixed-capacity payloads
        return dqrm_comm_allgather(x->comm, x->payload, x->gathered, x->payload_bytes, stream);
    return DQRM_OK;
}

int dqrm_exchange_apply(const dqrm_exchange* x, float lr, int mode, int repack_bits, void* stream) {
    const int rc = check_exchange(x, "dqrm_exchange_apply");
    if (rc) return rc;
    const void* g = x->comm ? x->gathered : x->payload;
    return dqrm_apply_sparse_update_fwd(x->set, x->cap_base, x->cap_total, g, x->payload_bytes, x->payload_bytes,
                                        x->num_ranks, x->grad_bits, x->s_avg, lr, mode, repack_bits, x->apply_ws,
                                        x->apply_ws_bytes, nullptr, 0, 0u, nullptr, 0, 0, stream);
}

int dqrm_exchange_apply_fwd(const dqrm_exchange* x, float lr, int mode, int repack_bits, const dqrm_batch* next,
                            int fwd_bits, uint32_t fwd_flags, float* out, int64_t out_stride_t, int64_t out_stride_b,
                            void* stream) {
    const int rc = check_exchange(x, "dqrm_exchange_apply_fwd");
    if (rc) return rc;
    const void* g = x->comm ? x->gathered : x->payload;
    return dqrm_apply_sparse_update_fwd(x->set, x->cap_base, x->cap_total, g, x->payload_bytes, x->payload_bytes,
                                        x->num_ranks, x->grad_bits, x->s_avg, lr, mode, repack_bits, x->apply_ws,
                                        x->apply_ws_bytes, next, fwd_bits, fwd_flags, out, out_stride_t, out_stride_b,
                                        stream);
}

}  // extern "C"
