// libmpbp -- ghost-row exchange of the row-partitioned apply over RCCL point-to-point (xGMI).
//
// Rank k owns grid rows [r0, r0 + L) of every field; its vectors hold the owned rows field-major and
// then the ghosts: h rows above of every field, then h rows below of every field (distributed.py's
// "ext" layout), so each direction's ghosts are one contiguous block.  A halo exchange is one RCCL group
// of four neighbour operations -- no collective over all ranks, no Python in the loop:
//   send own rows [r0, r0+h) of every field      -> up   (= rank k-1, periodic): its rows below
//   send own rows [r0+L-h, r0+L) of every field  -> down (= rank k+1, periodic): its rows above
//   recv the rows below <- down,  recv the rows above <- up
// A one-field vector sends its rows in place; a four-field one first gathers them (mpbp_gather, one
// kernel, launched before the group opens) into [top rows of every field | bottom rows of every field].  Per peer pair the operations
// are matched in issue order, so every rank issues them in the same order (send up, send down, recv
// down, recv up), which also covers world = 2 (up == down) and world = 1 (the wrap onto itself).
//
// mpbp_halo_exchange has the mpbp_halo_fn signature: mpbp_schur_apply calls it with phase BEGIN before
// a sweep's interior launch and END before its boundary launch.  Two schedules (mpbp_halo_set_mode):
//   IN_ORDER (default): the group is issued at END on the apply stream itself, after the interior.
//   OVERLAP: the group runs on the halo's own highest-priority stream, forked at BEGIN and joined at
//     END by events, so the transfer can overlap the interior rows.
// Measured on one MI355X (self-exchange, 1024^2): OVERLAP gains nothing -- the group's kernel waits for
// CUs behind the interior sweep, and each event packet adds ~15 us of queue latency -- so IN_ORDER.
//
// RCCL is resolved at run time (dlopen of the library the caller names -- the one torch loaded, so the
// process holds one RCCL), which keeps libmpbp free of a link-time RCCL dependency.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>

#include "mpbp.h"

namespace {

struct Rccl {
    void* lib = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};

char g_halo_err[512] = "";

int halo_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(g_halo_err, sizeof(g_halo_err), fmt, ap);
    va_end(ap);
    return code;
}

int load_rccl(const char* path, Rccl* r) {
    r->lib = dlopen(path && *path ? path : "librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!r->lib) return halo_error(MPBP_ERR_ARG, "dlopen RCCL: %s", dlerror());
#define MPBP_SYM(field, name)                                                                  \
    do {                                                                                       \
        *reinterpret_cast<void**>(&r->field) = dlsym(r->lib, name);                           \
        if (!r->field) return halo_error(MPBP_ERR_ARG, "RCCL symbol %s missing", name);        \
    } while (0)
    MPBP_SYM(get_unique_id, "ncclGetUniqueId");
    MPBP_SYM(comm_init_rank, "ncclCommInitRank");
    MPBP_SYM(comm_destroy, "ncclCommDestroy");
    MPBP_SYM(comm_abort, "ncclCommAbort");
    MPBP_SYM(send, "ncclSend");
    MPBP_SYM(recv, "ncclRecv");
    MPBP_SYM(group_start, "ncclGroupStart");
    MPBP_SYM(group_end, "ncclGroupEnd");
    MPBP_SYM(error_string, "ncclGetErrorString");
#undef MPBP_SYM
    return MPBP_OK;
}

}  // namespace

struct mpbp_halo {
    Rccl rccl;
    ncclComm_t comm = nullptr;
    int world = 0, rank = 0, up = 0, down = 0;
    int n = 0, r0 = 0, rows = 0;
    int h[2] = {0, 0};     // ghost depth of velocity (4 fields) and pressure (1 field) vectors
    int nf[2] = {4, 1};
    hipStream_t stream = nullptr;
    hipEvent_t ready[2] = {nullptr, nullptr}, done[2] = {nullptr, nullptr};
    int32_t* pack_idx[2] = {nullptr, nullptr};   // device: owned indices of [top rows | bottom rows] (nf > 1)
    double* pack_buf[2] = {nullptr, nullptr};    // device: 2 nf h n staged values
    int mode = MPBP_HALO_IN_ORDER;
    int status = MPBP_OK;  // first error seen by mpbp_halo_exchange (its signature returns nothing)
    bool captured = false; // an exchange was recorded into a hipGraph (stream capture) with this communicator
    char err[512] = "";
};

namespace {

void fail(mpbp_halo* H, int code, const char* what, const char* detail) {
    if (H->status == MPBP_OK) {
        H->status = code;
        std::snprintf(H->err, sizeof(H->err), "halo exchange: %s: %s", what, detail);
    }
}

}  // namespace

extern "C" {

int mpbp_rccl_unique_id(const char* rccl_path, uint8_t* id_out) {
    if (!id_out) return halo_error(MPBP_ERR_ARG, "rccl_unique_id: null output");
    Rccl r;
    int rc = load_rccl(rccl_path, &r);
    if (rc) return rc;
    ncclUniqueId id;
    const ncclResult_t e = r.get_unique_id(&id);
    if (e != ncclSuccess) return halo_error(MPBP_ERR_HIP, "ncclGetUniqueId: %s", r.error_string(e));
    std::memcpy(id_out, &id, sizeof(id));
    return MPBP_OK;
}

int mpbp_halo_create(const char* rccl_path, const uint8_t* id, int32_t world, int32_t rank, int32_t n,
                     int32_t r0, int32_t rows, int32_t h_u, int32_t h_p, mpbp_halo** out) {
    if (!id || !out || world < 1 || rank < 0 || rank >= world || n < 1 || rows < 1 || r0 < 0 || r0 + rows > n ||
        h_u < 1 || h_p < 1 || h_u > rows || h_p > rows)
        return halo_error(MPBP_ERR_ARG, "halo_create: bad partition (world %d rank %d n %d r0 %d rows %d h %d/%d)",
                          world, rank, n, r0, rows, h_u, h_p);
    mpbp_halo* H = new (std::nothrow) mpbp_halo();
    if (!H) return halo_error(MPBP_ERR_ARG, "halo_create: out of host memory");
    int rc = load_rccl(rccl_path, &H->rccl);
    if (rc) {
        delete H;
        return rc;
    }
    H->world = world;
    H->rank = rank;
    H->up = (rank + world - 1) % world;
    H->down = (rank + 1) % world;
    H->n = n;
    H->r0 = r0;
    H->rows = rows;
    H->h[0] = h_u;
    H->h[1] = h_p;
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    const ncclResult_t e = H->rccl.comm_init_rank(&H->comm, world, uid, rank);
    if (e != ncclSuccess) {
        halo_error(MPBP_ERR_HIP, "ncclCommInitRank: %s", H->rccl.error_string(e));
        delete H;
        return MPBP_ERR_HIP;
    }
    // The group's kernel is launched next to the interior sweep, which fills every CU: on a
    // highest-priority stream it is dispatched first instead of waiting for the sweep to drain.
    int least = 0, greatest = 0;
    bool ok = hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess &&
              hipStreamCreateWithPriority(&H->stream, hipStreamNonBlocking, greatest) == hipSuccess;
    for (int k = 0; k < 2 && ok; ++k)
        ok = hipEventCreateWithFlags(&H->ready[k], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&H->done[k], hipEventDisableTiming) == hipSuccess;
    for (int k = 0; k < 2 && ok; ++k) {
        if (H->nf[k] == 1) continue;
        const int nf = H->nf[k], h = H->h[k];
        const size_t cnt = (size_t)2 * nf * h * n;
        int32_t* idx = static_cast<int32_t*>(std::malloc(cnt * sizeof(int32_t)));
        ok = idx != nullptr;
        for (int f = 0; ok && f < nf; ++f)
            for (int j = 0; j < h * n; ++j) {
                idx[(size_t)f * h * n + j] = f * rows * n + j;                                  // top rows
                idx[(size_t)(nf + f) * h * n + j] = f * rows * n + (rows - h) * n + j;          // bottom rows
            }
        ok = ok && hipMalloc(&H->pack_idx[k], cnt * sizeof(int32_t)) == hipSuccess &&
             hipMalloc(&H->pack_buf[k], cnt * sizeof(double)) == hipSuccess &&
             hipMemcpy(H->pack_idx[k], idx, cnt * sizeof(int32_t), hipMemcpyHostToDevice) == hipSuccess;
        std::free(idx);
    }
    if (!ok) {
        mpbp_halo_destroy(H);
        return halo_error(MPBP_ERR_HIP, "halo_create: stream / event / buffer creation failed");
    }
    *out = H;
    return MPBP_OK;
}

void mpbp_halo_destroy(mpbp_halo* H) {
    if (!H) return;
    if (H->stream) (void)hipStreamSynchronize(H->stream);
    for (int k = 0; k < 2; ++k) {
        if (H->ready[k]) (void)hipEventDestroy(H->ready[k]);
        if (H->done[k]) (void)hipEventDestroy(H->done[k]);
    }
    if (H->stream) (void)hipStreamDestroy(H->stream);
    for (int k = 0; k < 2; ++k) {
        if (H->pack_idx[k]) (void)hipFree(H->pack_idx[k]);
        if (H->pack_buf[k]) (void)hipFree(H->pack_buf[k]);
    }
    // A communicator whose operations were captured into a hipGraph is not destroyed: with RCCL 2.26.6,
    // ncclCommDestroy never returns once a graph holding this communicator's point-to-point kernels has
    // been instantiated and destroyed (measured: tools/capture_probe.py).  It is
    // released with the process instead (MPBP_HALO_CAPTURED_DESTROY=abort tries ncclCommAbort,
    // =destroy the plain destroy).
    if (H->comm) {
        const char* pol = std::getenv("MPBP_HALO_CAPTURED_DESTROY");
        if (!H->captured || (pol && std::strcmp(pol, "destroy") == 0)) H->rccl.comm_destroy(H->comm);
        else if (pol && std::strcmp(pol, "abort") == 0) H->rccl.comm_abort(H->comm);
    }
    // the RCCL library stays loaded: torch (or another communicator) may still use it
    delete H;
}

namespace {

// One exchange of vector kind k on stream `on`: a multi-field vector's boundary rows are first gathered
// into pack_buf by one kernel launched BEFORE the RCCL group opens (a kernel launch never sits between
// ncclGroupStart and ncclGroupEnd, which graph capture of the group requires to be plain RCCL calls); then
// one group: own top rows -> up, own bottom rows -> down, rows below <- down, rows above <- up.
struct HaloBufs {
    const double* top;
    const double* bot;
    double* above;
    double* below;
    size_t cnt;   // values per direction
};

int halo_pack(mpbp_halo* H, int k, double* x_ext, hipStream_t on, HaloBufs* b) {
    const int nf = H->nf[k], h = H->h[k], n = H->n, L = H->rows;
    b->cnt = (size_t)nf * h * n;
    b->top = x_ext;                               // nf == 1: the rows in place
    b->bot = x_ext + (size_t)(L - h) * n;
    if (nf > 1) {
        const int rc = mpbp_gather((int32_t)(2 * b->cnt), H->pack_idx[k], x_ext, H->pack_buf[k], (void*)on);
        if (rc != MPBP_OK) return rc;
        b->top = H->pack_buf[k];
        b->bot = H->pack_buf[k] + b->cnt;
    }
    b->above = x_ext + (size_t)nf * L * n;
    b->below = b->above + b->cnt;
    return MPBP_OK;
}

// The sends / receives of one vector (inside an open group).
ncclResult_t halo_ops(mpbp_halo* H, const HaloBufs& b, hipStream_t on) {
    const Rccl& R = H->rccl;
    ncclResult_t e = R.send(b.top, b.cnt, ncclFloat64, H->up, H->comm, on);
    if (e == ncclSuccess) e = R.send(b.bot, b.cnt, ncclFloat64, H->down, H->comm, on);
    if (e == ncclSuccess) e = R.recv(b.below, b.cnt, ncclFloat64, H->down, H->comm, on);
    if (e == ncclSuccess) e = R.recv(b.above, b.cnt, ncclFloat64, H->up, H->comm, on);
    return e;
}

void note_capture(mpbp_halo* H, hipStream_t on) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(on, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) H->captured = true;
}

ncclResult_t halo_group(mpbp_halo* H, int k, double* x_ext, hipStream_t on) {
    note_capture(H, on);
    HaloBufs b;
    if (halo_pack(H, k, x_ext, on, &b) != MPBP_OK) return ncclUnhandledCudaError;
    const ncclResult_t e = H->rccl.group_start();
    const ncclResult_t e2 = e == ncclSuccess ? halo_ops(H, b, on) : e;
    const ncclResult_t eg = H->rccl.group_end();
    return e2 == ncclSuccess ? eg : e2;
}

}  // namespace

void mpbp_halo_exchange(void* ctx, int32_t vec_kind, double* x_ext, int32_t phase, void* stream) {
    mpbp_halo* H = static_cast<mpbp_halo*>(ctx);
    if (!H || H->status != MPBP_OK) return;
    if (vec_kind != MPBP_VEC_VELOCITY && vec_kind != MPBP_VEC_PRESSURE) {
        fail(H, MPBP_ERR_ARG, "vector kind", "unknown");
        return;
    }
    const int k = vec_kind == MPBP_VEC_VELOCITY ? 0 : 1;
    const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (H->mode == MPBP_HALO_IN_ORDER) {
        // the group goes on the apply stream between the interior and the boundary launches: no event
        // packets (each costs ~15 us of queue latency here), and its host-side enqueue overlaps the interior
        if (phase == MPBP_HALO_END) {
            const ncclResult_t e = halo_group(H, k, x_ext, st);
            if (e != ncclSuccess) fail(H, MPBP_ERR_HIP, "RCCL group", H->rccl.error_string(e));
        }
        return;
    }
    if (phase == MPBP_HALO_END) {
        if (hipStreamWaitEvent(st, H->done[k], 0) != hipSuccess) fail(H, MPBP_ERR_HIP, "join", "hipStreamWaitEvent");
        return;
    }
    if (hipEventRecord(H->ready[k], st) != hipSuccess || hipStreamWaitEvent(H->stream, H->ready[k], 0) != hipSuccess) {
        fail(H, MPBP_ERR_HIP, "fork", "hipEventRecord / hipStreamWaitEvent");
        return;
    }
    const ncclResult_t e = halo_group(H, k, x_ext, H->stream);
    if (e != ncclSuccess) {
        fail(H, MPBP_ERR_HIP, "RCCL group", H->rccl.error_string(e));
        return;
    }
    if (hipEventRecord(H->done[k], H->stream) != hipSuccess) fail(H, MPBP_ERR_HIP, "fork", "hipEventRecord");
}

void mpbp_halo_exchange_pair(void* ctx, double* xu_ext, double* xp_ext, void* stream) {
    mpbp_halo* H = static_cast<mpbp_halo*>(ctx);
    if (!H || H->status != MPBP_OK) return;
    const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    // both vectors' operations in one group; the velocity rows are gathered before the group opens
    note_capture(H, st);
    HaloBufs bu, bp;
    if (halo_pack(H, 0, xu_ext, st, &bu) != MPBP_OK || halo_pack(H, 1, xp_ext, st, &bp) != MPBP_OK) {
        fail(H, MPBP_ERR_HIP, "pack", "mpbp_gather");
        return;
    }
    const ncclResult_t e0 = H->rccl.group_start();
    ncclResult_t e = e0 == ncclSuccess ? halo_ops(H, bu, st) : e0;
    if (e == ncclSuccess) e = halo_ops(H, bp, st);
    const ncclResult_t eg = H->rccl.group_end();
    if (e == ncclSuccess) e = eg;
    if (e != ncclSuccess) fail(H, MPBP_ERR_HIP, "RCCL pair group", H->rccl.error_string(e));
}

int mpbp_halo_set_mode(mpbp_halo* H, int32_t mode) {
    if (!H || (mode != MPBP_HALO_OVERLAP && mode != MPBP_HALO_IN_ORDER))
        return halo_error(MPBP_ERR_ARG, "halo_set_mode: mode must be MPBP_HALO_OVERLAP or MPBP_HALO_IN_ORDER");
    H->mode = mode;
    return MPBP_OK;
}

int mpbp_halo_status(const mpbp_halo* H) { return H ? H->status : MPBP_ERR_ARG; }

const char* mpbp_halo_last_error(const mpbp_halo* H) { return (H && H->status != MPBP_OK) ? H->err : g_halo_err; }

}  // extern "C"
