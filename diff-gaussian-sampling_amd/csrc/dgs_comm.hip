// dgs_comm.hip -- the collective of the dense sharded path for callers of the C ABI that do not
// use torch.distributed (dgs_allreduce_grads on an RCCL communicator; 8e: one
// all-reduce of the packed per-Gaussian gradients over xGMI).
//
// RCCL is loaded on first use (dlopen "librccl.so.1"): the library is ~0.5 GB and most callers
// never need it, so libdgs.so carries no load-time dependency on it.  The communicator is an
// ncclComm_t made by dgs_comm_init (or by the caller's own RCCL: then pass the SAME library's
// communicator; torch's bundled RCCL is a separate copy whose communicators are not
// interchangeable with this one).
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <mutex>
#include <string>

#include <rccl/rccl.h>

#include "dgs.h"
#include "dgs_internal.h"

namespace {

struct Rccl {
    void *h = nullptr;
    ncclResult_t (*uid)(ncclUniqueId *) = nullptr;
    ncclResult_t (*init)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*allreduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    const char *(*errstr)(ncclResult_t) = nullptr;
    std::string why;
};

const Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            r.h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (r.h) break;
        }
        if (!r.h) {
            const char *e = dlerror();
            r.why = std::string("RCCL not found: ") + (e ? e : "dlopen failed");
            return;
        }
        r.uid = reinterpret_cast<decltype(r.uid)>(dlsym(r.h, "ncclGetUniqueId"));
        r.init = reinterpret_cast<decltype(r.init)>(dlsym(r.h, "ncclCommInitRank"));
        r.destroy = reinterpret_cast<decltype(r.destroy)>(dlsym(r.h, "ncclCommDestroy"));
        r.allreduce = reinterpret_cast<decltype(r.allreduce)>(dlsym(r.h, "ncclAllReduce"));
        r.errstr = reinterpret_cast<decltype(r.errstr)>(dlsym(r.h, "ncclGetErrorString"));
        if (!r.uid || !r.init || !r.destroy || !r.allreduce || !r.errstr) r.why = "RCCL symbols missing";
    });
    return r;
}

int rccl_fail(const Rccl &r, ncclResult_t e, const char *what) {
    return dgs::fail(DGS_ERR_HIP, std::string(what) + ": " + (r.errstr ? r.errstr(e) : "RCCL error"));
}

}  // namespace

extern "C" size_t dgs_comm_id_bytes(void) { return sizeof(ncclUniqueId); }

extern "C" int dgs_comm_unique_id(void *id_out) {
    const Rccl &r = rccl();
    if (!r.why.empty()) return dgs::fail(DGS_ERR_HIP, r.why);
    if (!id_out) return dgs::fail(DGS_ERR_ARG, "dgs_comm_unique_id: id_out required");
    const ncclResult_t e = r.uid(static_cast<ncclUniqueId *>(id_out));
    return e == ncclSuccess ? DGS_OK : rccl_fail(r, e, "ncclGetUniqueId");
}

extern "C" int dgs_comm_init(void **comm_out, int nranks, const void *id, int rank) {
    const Rccl &r = rccl();
    if (!r.why.empty()) return dgs::fail(DGS_ERR_HIP, r.why);
    if (!comm_out || !id || nranks < 1 || rank < 0 || rank >= nranks)
        return dgs::fail(DGS_ERR_ARG, "dgs_comm_init: bad arguments");
    ncclComm_t c = nullptr;
    const ncclResult_t e = r.init(&c, nranks, *static_cast<const ncclUniqueId *>(id), rank);
    if (e != ncclSuccess) return rccl_fail(r, e, "ncclCommInitRank");
    *comm_out = c;
    return DGS_OK;
}

extern "C" int dgs_comm_destroy(void *comm) {
    const Rccl &r = rccl();
    if (!r.why.empty()) return dgs::fail(DGS_ERR_HIP, r.why);
    if (!comm) return DGS_OK;
    const ncclResult_t e = r.destroy(static_cast<ncclComm_t>(comm));
    return e == ncclSuccess ? DGS_OK : rccl_fail(r, e, "ncclCommDestroy");
}

extern "C" int dgs_allreduce_grads(float *grads, size_t count, void *comm, size_t chunk_elems, dgs_stream_t stream) {
    const Rccl &r = rccl();
    if (!r.why.empty()) return dgs::fail(DGS_ERR_HIP, r.why);
    if (!comm || (count && !grads)) return dgs::fail(DGS_ERR_ARG, "dgs_allreduce_grads: bad arguments");
    const size_t step = chunk_elems ? chunk_elems : count;
    for (size_t o = 0; o < count; o += step) {  // (chunks back to back: RCCL pipelines them)
        const size_t n = count - o < step ? count - o : step;
        const ncclResult_t e = r.allreduce(grads + o, grads + o, n, ncclFloat32, ncclSum,
                                           static_cast<ncclComm_t>(comm), reinterpret_cast<hipStream_t>(stream));
        if (e != ncclSuccess) return rccl_fail(r, e, "ncclAllReduce");
    }
    return DGS_OK;
}
