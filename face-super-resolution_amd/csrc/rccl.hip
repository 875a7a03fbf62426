// Direct RCCL for the data-parallel gradient exchange (fen_rccl_*, include/fen.h).
//
// The reference all-reduces its gradients through DDP (trainer.py:126-134, scripts/train.py:
// 325-330).  Here each backward bucket (a contiguous slice of the flat fp32 gradient arena,
// src/training/dp.py) is summed by ONE ncclAllReduce issued on the caller's stream: no c10d
// Work object, no HIP events, no watchdog thread, so a collective issued from any host thread
// (autograd's device thread runs the module path's post-accumulate hooks) records into a
// hipGraph capture like any kernel.  torch.distributed is used for the rendezvous only (the
// unique id's broadcast).
//
// RCCL is resolved at run time (dlopen): the instance torch already loaded (its bundled
// librccl.so) when present, else the system's librccl.so.1 -- one RCCL per process either way
// for the common case, and no link-time dependency of libfen_hip.so on either.
#include <dlfcn.h>
#include <link.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <mutex>
#include <stdio.h>
#include <string.h>

#include "fen.h"

namespace {

struct Rccl {
    void* h = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*async_error)(ncclComm_t, ncclResult_t*) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    const char* path = "none";
};

Rccl g_rccl;
std::once_flag g_once;
thread_local char g_err[256] = "none";

void set_err(const char* what, const char* detail) {
    snprintf(g_err, sizeof(g_err), "%s: %s", what, detail ? detail : "?");
}

void resolve() {
    static const char* const names[] = {"librccl.so", "librccl.so.1", "/opt/rocm/lib/librccl.so.1"};
    void* h = nullptr;
    const char* path = nullptr;
    for (const char* n : names) {   // an instance already in the process first (torch's)
        h = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
        if (h) { path = n; break; }
    }
    for (int i = 0; !h && i < 3; ++i) {
        h = dlopen(names[i], RTLD_NOW | RTLD_LOCAL);
        if (h) path = names[i];
    }
    if (!h) return;
    Rccl r;
    r.h = h;
    r.path = path;
    struct link_map* lm = nullptr;     // report the file actually mapped
    if (dlinfo(h, RTLD_DI_LINKMAP, &lm) == 0 && lm && lm->l_name && lm->l_name[0]) r.path = lm->l_name;
    r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
    r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
    r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
    r.async_error = (decltype(r.async_error))dlsym(h, "ncclCommGetAsyncError");
    r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
    if (r.get_unique_id && r.comm_init_rank && r.all_reduce && r.comm_destroy && r.async_error && r.error_string)
        g_rccl = r;
}

const Rccl* rccl() {
    std::call_once(g_once, resolve);
    if (!g_rccl.h) {
        set_err("dlopen", "no librccl.so / librccl.so.1 in the process or on the loader path");
        return nullptr;
    }
    return &g_rccl;
}

int rc(const Rccl* r, ncclResult_t e, const char* what) {
    if (e == ncclSuccess) return FEN_OK;
    set_err(what, r->error_string(e));
    return FEN_ERCCL;
}

}  // namespace

extern "C" int fen_rccl_unique_id(void* id) {
    if (!id) return FEN_EINVAL;
    const Rccl* r = rccl();
    if (!r) return FEN_ERCCL;
    ncclUniqueId u;
    int s = rc(r, r->get_unique_id(&u), "ncclGetUniqueId");
    if (s == FEN_OK) memcpy(id, &u, sizeof(u));
    return s;
}

extern "C" int fen_rccl_init(void** comm, const void* id, int nranks, int rank, int device) {
    if (!comm || !id || nranks < 1 || rank < 0 || rank >= nranks || device < 0) return FEN_EINVAL;
    const Rccl* r = rccl();
    if (!r) return FEN_ERCCL;
    hipError_t he = hipSetDevice(device);
    if (he != hipSuccess) {
        set_err("hipSetDevice", hipGetErrorString(he));
        return FEN_ERCCL;
    }
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclComm_t c = nullptr;
    int s = rc(r, r->comm_init_rank(&c, nranks, u, rank), "ncclCommInitRank");
    *comm = s == FEN_OK ? (void*)c : nullptr;
    return s;
}

extern "C" int fen_rccl_allreduce_bucket(void* comm, float* buf, size_t count, void* stream) {
    if (!comm || (!buf && count)) return FEN_EINVAL;
    if (!count) return FEN_OK;
    const Rccl* r = rccl();
    if (!r) return FEN_ERCCL;
    return rc(r, r->all_reduce(buf, buf, count, ncclFloat32, ncclSum, (ncclComm_t)comm, (hipStream_t)stream),
              "ncclAllReduce");
}

extern "C" int fen_rccl_check(void* comm) {
    if (!comm) return FEN_EINVAL;
    const Rccl* r = rccl();
    if (!r) return FEN_ERCCL;
    ncclResult_t a = ncclSuccess;
    int s = rc(r, r->async_error((ncclComm_t)comm, &a), "ncclCommGetAsyncError");
    return s == FEN_OK ? rc(r, a, "asynchronous RCCL error") : s;
}

extern "C" int fen_rccl_destroy(void* comm) {
    if (!comm) return FEN_OK;
    const Rccl* r = rccl();
    if (!r) return FEN_ERCCL;
    return rc(r, r->comm_destroy((ncclComm_t)comm), "ncclCommDestroy");
}

extern "C" const char* fen_last_rccl_error(void) { return g_err; }

extern "C" const char* fen_rccl_library(void) {
    const Rccl* r = rccl();
    return r ? r->path : "none";
}
