// comm.cpp -- the one collective of the multi-GPU path: an RCCL communicator over
// the node's ranks (one process per GPU, xGMI between them) and the all-gather of the per-frame
// detection records, enqueued on a caller's HIP stream so it runs beside the next step's kernels.
// The reference has no multi-device code; nothing here restates it.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>

#include "../../../include/zaru_hip.h"

namespace zr_internal {
int set_error(int code, const std::string &msg);
}

struct zr_comm {
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0, device = 0;
};

namespace {

// A failure of earlier HIP work on this thread (a kernel launch the runtime has not yet checked)
// must not vanish inside a communicator call: every entry point first takes the thread's pending
// HIP error and, if there is one, returns it as ZR_ERR_DEVICE without calling RCCL.
int pending_hip_error(const char *where) {
    const hipError_t e = hipGetLastError();
    if (e == hipSuccess) return ZR_OK;
    return zr_internal::set_error(ZR_ERR_DEVICE, std::string(where) + ": pending HIP error from earlier work: " +
                                                     hipGetErrorString(e));
}

// RCCL's own HIP calls (capture queries on the caller's stream among them) may leave the thread's
// last-error slot set although the call succeeded; the runtime's next hipGetLastError() check after
// a kernel launch would then report RCCL's stale status as its own failure.  So after an RCCL call
// (and only then: anything pending before it was already taken by pending_hip_error) the slot is
// cleared.
void clear_rccl_status() { (void)hipGetLastError(); }

int nccl_err(const char *what, ncclResult_t r) {
    return zr_internal::set_error(ZR_ERR_DEVICE, std::string(what) + ": " + ncclGetErrorString(r));
}

template <class F>
int guarded(F &&body) noexcept {
    try {
        return body();
    } catch (const std::bad_alloc &) {
        return zr_internal::set_error(ZR_ERR_DEVICE, "out of host memory");
    } catch (...) {
        return zr_internal::set_error(ZR_ERR_INTERNAL, "internal error in the communicator");
    }
}

}  // namespace

extern "C" {

int zr_comm_unique_id(uint8_t id[128]) {
    return guarded([&]() -> int {
        static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
        if (!id) return zr_internal::set_error(ZR_ERR_INVALID_ARGUMENT, "null id");
        if (int e = pending_hip_error("zr_comm_unique_id")) return e;
        ncclUniqueId u;
        const ncclResult_t r = ncclGetUniqueId(&u);
        clear_rccl_status();
        if (r) return nccl_err("ncclGetUniqueId", r);
        std::memcpy(id, &u, sizeof u);
        return ZR_OK;
    });
}

int zr_comm_create(const uint8_t id[128], int nranks, int rank, int device, zr_comm **out) {
    return guarded([&]() -> int {
        if (!id || !out || nranks <= 0 || rank < 0 || rank >= nranks)
            return zr_internal::set_error(ZR_ERR_INVALID_ARGUMENT, "bad communicator arguments");
        *out = nullptr;
        if (int e = pending_hip_error("zr_comm_create")) return e;
        if (hipSetDevice(device) != hipSuccess) {
            (void)hipGetLastError();
            return zr_internal::set_error(ZR_ERR_DEVICE, "no HIP device " + std::to_string(device));
        }
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof u);
        auto *c = new zr_comm;
        c->nranks = nranks;
        c->rank = rank;
        c->device = device;
        const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
        clear_rccl_status();
        if (r) {
            delete c;
            return nccl_err("ncclCommInitRank", r);
        }
        *out = c;
        return ZR_OK;
    });
}

void zr_comm_destroy(zr_comm *c) {
    if (!c) return;
    if (c->comm) {
        // teardown: RCCL's status is cleared; an error of earlier work is reported by the caller's
        // own synchronisation, which sees the failed stream, not by this slot
        (void)ncclCommDestroy(c->comm);
        clear_rccl_status();
    }
    delete c;
}

int zr_comm_size(const zr_comm *c, int *nranks) {
    if (!c || !nranks) return zr_internal::set_error(ZR_ERR_INVALID_ARGUMENT, "null communicator or output");
    *nranks = c->nranks;
    return ZR_OK;
}

int zr_comm_all_gather_async(zr_comm *c, const void *d_send, void *d_recv, size_t bytes, void *hip_stream) {
    return guarded([&]() -> int {
        if (!c || !c->comm || !d_send || !d_recv)
            return zr_internal::set_error(ZR_ERR_INVALID_ARGUMENT, "null communicator or buffer");
        // the gather runs on a stream of the caller's pipeline; the legacy NULL stream (which
        // waits for, and blocks, every blocking stream of the device, and which RCCL's stream
        // bookkeeping treats as a special case) is refused
        if (!hip_stream)
            return zr_internal::set_error(ZR_ERR_INVALID_ARGUMENT, "the all-gather needs a HIP stream (not the NULL stream)");
        if (int e = pending_hip_error("zr_comm_all_gather_async")) return e;
        if (bytes == 0) return ZR_OK;
        // bytes as ncclChar elements: the records are opaque 32-bit words (f32 and u32 bits)
        const ncclResult_t r = ncclAllGather(d_send, d_recv, bytes, ncclChar, c->comm, (hipStream_t)hip_stream);
        clear_rccl_status();
        if (r) return nccl_err("ncclAllGather", r);
        return ZR_OK;
    });
}

}  // extern "C"
