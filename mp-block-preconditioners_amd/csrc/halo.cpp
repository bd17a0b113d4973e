// libmpbp -- ghost-row exchange of the row-partitioned apply over RCCL point-to-point (xGMI).
//
// Rank k owns grid rows [r0, r0 + L) of every field; its vectors hold the owned rows field-major and
// then the ghosts: h rows above of every field, then h rows below of every field (distributed.py's
// "ext" layout), so each direction's ghosts are one contiguous block.  A halo exchange is one RCCL group
// of four neighbour operations -- no collective over all ranks, no Python in the loop:
//   send own rows [r0, r0+h) of every field      -> up   (= rank k-1, periodic): its rows below
//   send own rows [r0+L-h, r0+L) of every field  -> down (= rank k+1, periodic): its rows above
//   recv the rows below <- down,  recv the rows above <- up
// A one-field vector sends its rows in place; a multi-field one first gathers them (mpbp_gather, one
// kernel, launched before the group opens) into [top rows of every field | bottom rows of every field].  Per
// peer pair the operations are matched in issue order, so every rank issues them in the same order (send
// up, send down, recv down, recv up), which also covers world = 2 (up == down) and world = 1 (the wrap
// onto itself).
//
// Vector kinds.  A halo object serves any number of vector layouts ("kinds": fields, grid size, owned rows,
// ghost depth): kinds 0 and 1 are the Schur apply's velocity (4 fields) and pressure (1 field) vectors, made
// by mpbp_halo_create; mpbp_halo_add_kind adds more (the system vector of the partitioned operator A, the
// multigrid levels).  Gather kinds (mpbp_halo_add_gather) all-gather a partitioned vector into the whole
// field-major vector on every rank (the multigrid levels run replicated below the partitioned ones).
//
// mpbp_halo_exchange has the mpbp_halo_fn signature: mpbp_schur_apply calls it with phase BEGIN before
// a sweep's interior launch and END before its boundary launch.  Two schedules per kind:
//   IN_ORDER (default): the group is issued at END on the caller's stream itself, after the interior.
//   OVERLAP: the group runs on the halo's own highest-priority stream, forked at BEGIN and joined at
//     END by events, so the transfer can overlap the interior rows.
// Measured on one MI355X (self-exchange, 1024^2 apply): OVERLAP gains nothing there -- the group's kernel
// waits for CUs behind the interior sweep, and each event packet adds ~15 us of queue latency.
//
// RCCL is resolved at run time (dlopen of the library the caller names -- the one torch loaded, so the
// process holds one RCCL), which keeps libmpbp free of a link-time RCCL dependency.
//
// Communicators: mpbp_halo_create opens one; mpbp_halo_create_shared gives another halo object (its own vector kinds,
// buffers and stream) the same communicator, reference-counted.  The Python layer shares one communicator between the
// partitioned PRECONDITIONERS of a process group (all their exchanges in order on the caller's stream, the same program
// order on every rank) and gives the partitioned operator A u (DistributedMatrix) a communicator of its own: its
// exchanges run eagerly on this object's side stream (OVERLAP) while a preconditioner's may be graph-replayed, and eager
// side-stream and graph-replayed operations are never mixed on one communicator.  A
// communicator whose point-to-point kernels were captured into a hipGraph is not destroyed when its last halo object
// goes (see mpbp_halo_destroy): with RCCL 2.26.6 ncclCommDestroy then never returns.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

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
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
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
    MPBP_SYM(all_gather, "ncclAllGather");
    MPBP_SYM(group_start, "ncclGroupStart");
    MPBP_SYM(group_end, "ncclGroupEnd");
    MPBP_SYM(error_string, "ncclGetErrorString");
#undef MPBP_SYM
    return MPBP_OK;
}

// One vector layout: nf fields of an n-column grid, owned rows [r0, r0 + rows), h ghost rows each side.
struct Kind {
    int nf = 1, n = 0, r0 = 0, rows = 0, h = 0;
    int mode = MPBP_HALO_IN_ORDER;
    int32_t* pack_idx = nullptr;   // device: owned indices of [top rows | bottom rows] (nf > 1)
    double* pack_buf = nullptr;    // device: 2 nf h n staged values
    hipEvent_t ready = nullptr, done = nullptr;
};

// All-gather of a partitioned nf-field vector of an n x n grid (rank k owns rows [r0s[k], r0s[k] + rows[k]) of
// every field) into the whole field-major vector: the owned rows padded to the largest rank's (send), one
// ncclAllGather into stage, one gather kernel into place (full[i] = stage[idx[i]]).
struct GatherKind {
    int nf = 1, n = 0, lmax = 0, rows = 0;
    int32_t* send_idx = nullptr;   // device: owned -> padded send slots (nullptr: owned rows already padded)
    double* send = nullptr;        // device: nf * lmax * n
    double* stage = nullptr;       // device: world * nf * lmax * n
    int32_t* full_idx = nullptr;   // device: nf * n * n
};

// A communicator shared by the halo objects of one process group (refs: the objects holding it).
struct SharedComm {
    ncclComm_t comm = nullptr;
    int refs = 0;
    bool captured = false;   // an exchange was recorded into a hipGraph (stream capture) on this communicator
};

}  // namespace

struct mpbp_halo {
    Rccl rccl;
    SharedComm* shared = nullptr;
    ncclComm_t comm = nullptr;   // == shared->comm
    int world = 0, rank = 0, up = 0, down = 0;
    std::vector<Kind> kinds;
    std::vector<GatherKind> gathers;
    hipStream_t stream = nullptr;
    int default_mode = MPBP_HALO_IN_ORDER;
    int status = MPBP_OK;  // first error seen by mpbp_halo_exchange (its signature returns nothing)
    char err[512] = "";
};

namespace {

void fail(mpbp_halo* H, int code, const char* what, const char* detail) {
    if (H->status == MPBP_OK) {
        H->status = code;
        std::snprintf(H->err, sizeof(H->err), "halo exchange: %s: %s", what, detail);
    }
}

int upload_idx(const std::vector<int32_t>& v, int32_t** out) {
    if (v.empty()) return MPBP_OK;
    if (hipMalloc(out, v.size() * sizeof(int32_t)) != hipSuccess ||
        hipMemcpy(*out, v.data(), v.size() * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess)
        return halo_error(MPBP_ERR_HIP, "halo: index upload failed");
    return MPBP_OK;
}

int halo_init_local(mpbp_halo* H, int n, int r0, int rows, int h_u, int h_p);

int make_kind(mpbp_halo* H, int nf, int n, int r0, int rows, int h, int mode) {
    if (nf < 1 || n < 1 || rows < 1 || r0 < 0 || h < 1 || h > rows || (int64_t)2 * nf * h * n > INT32_MAX ||
        (mode != MPBP_HALO_IN_ORDER && mode != MPBP_HALO_OVERLAP))
        return halo_error(MPBP_ERR_ARG, "halo kind: bad layout (fields %d n %d r0 %d rows %d h %d mode %d)", nf, n, r0,
                          rows, h, mode);
    Kind k;
    k.nf = nf;
    k.n = n;
    k.r0 = r0;
    k.rows = rows;
    k.h = h;
    k.mode = mode;
    if (hipEventCreateWithFlags(&k.ready, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&k.done, hipEventDisableTiming) != hipSuccess)
        return halo_error(MPBP_ERR_HIP, "halo kind: event creation failed");
    if (nf > 1) {
        const size_t cnt = (size_t)2 * nf * h * n;
        std::vector<int32_t> idx(cnt);
        for (int f = 0; f < nf; ++f)
            for (int j = 0; j < h * n; ++j) {
                idx[(size_t)f * h * n + j] = f * rows * n + j;                                  // top rows
                idx[(size_t)(nf + f) * h * n + j] = f * rows * n + (rows - h) * n + j;          // bottom rows
            }
        int rc = upload_idx(idx, &k.pack_idx);
        if (rc == MPBP_OK && hipMalloc(&k.pack_buf, cnt * sizeof(double)) != hipSuccess)
            rc = halo_error(MPBP_ERR_HIP, "halo kind: buffer allocation failed");
        if (rc) {
            (void)hipEventDestroy(k.ready);
            (void)hipEventDestroy(k.done);
            if (k.pack_idx) (void)hipFree(k.pack_idx);
            return rc;
        }
    }
    H->kinds.push_back(k);
    return (int)H->kinds.size() - 1;
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
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    H->shared = new (std::nothrow) SharedComm();
    if (!H->shared) {
        delete H;
        return halo_error(MPBP_ERR_ARG, "halo_create: out of host memory");
    }
    const ncclResult_t e = H->rccl.comm_init_rank(&H->shared->comm, world, uid, rank);
    if (e != ncclSuccess) {
        halo_error(MPBP_ERR_HIP, "ncclCommInitRank: %s", H->rccl.error_string(e));
        delete H->shared;
        delete H;
        return MPBP_ERR_HIP;
    }
    H->shared->refs = 1;
    H->comm = H->shared->comm;
    const int rc2 = halo_init_local(H, n, r0, rows, h_u, h_p);
    if (rc2) return rc2;
    *out = H;
    return MPBP_OK;
}

int mpbp_halo_create_shared(const mpbp_halo* base, int32_t n, int32_t r0, int32_t rows, int32_t h_u, int32_t h_p,
                            mpbp_halo** out) {
    if (!base || !base->shared || !out || n < 1 || rows < 1 || r0 < 0 || r0 + rows > n || h_u < 1 || h_p < 1 ||
        h_u > rows || h_p > rows)
        return halo_error(MPBP_ERR_ARG, "halo_create_shared: bad arguments (n %d r0 %d rows %d h %d/%d)", n, r0, rows,
                          h_u, h_p);
    mpbp_halo* H = new (std::nothrow) mpbp_halo();
    if (!H) return halo_error(MPBP_ERR_ARG, "halo_create_shared: out of host memory");
    H->rccl = base->rccl;
    H->world = base->world;
    H->rank = base->rank;
    H->up = base->up;
    H->down = base->down;
    H->shared = base->shared;
    H->comm = base->shared->comm;
    ++H->shared->refs;
    const int rc = halo_init_local(H, n, r0, rows, h_u, h_p);
    if (rc) return rc;
    *out = H;
    return MPBP_OK;
}

const void* mpbp_halo_comm(const mpbp_halo* H) { return H && H->shared ? (const void*)H->shared->comm : nullptr; }

int mpbp_halo_comm_refs(const mpbp_halo* H) { return H && H->shared ? H->shared->refs : 0; }

}  // extern "C"

namespace {
// The object's own stream and the Schur apply's two vector kinds; on failure the object is destroyed.
int halo_init_local(mpbp_halo* H, int n, int r0, int rows, int h_u, int h_p) {
    // The group's kernel is launched next to the interior sweep, which fills every CU: on a
    // highest-priority stream it is dispatched first instead of waiting for the sweep to drain.
    int least = 0, greatest = 0;
    bool ok = hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess &&
              hipStreamCreateWithPriority(&H->stream, hipStreamNonBlocking, greatest) == hipSuccess;
    // kinds 0 (MPBP_VEC_VELOCITY) and 1 (MPBP_VEC_PRESSURE) of the Schur apply
    ok = ok && make_kind(H, 4, n, r0, rows, h_u, MPBP_HALO_IN_ORDER) == MPBP_VEC_VELOCITY &&
         make_kind(H, 1, n, r0, rows, h_p, MPBP_HALO_IN_ORDER) == MPBP_VEC_PRESSURE;
    if (!ok) {
        mpbp_halo_destroy(H);
        return halo_error(MPBP_ERR_HIP, "halo_create: stream / event / buffer creation failed");
    }
    return MPBP_OK;
}
}  // namespace

extern "C" {

int mpbp_halo_add_kind(mpbp_halo* H, int32_t nfields, int32_t n, int32_t r0, int32_t rows, int32_t h, int32_t mode) {
    if (!H) return halo_error(MPBP_ERR_ARG, "halo_add_kind: null halo");
    if (r0 + rows > n) return halo_error(MPBP_ERR_ARG, "halo_add_kind: rows [%d, %d) outside the grid %d", r0, r0 + rows, n);
    return make_kind(H, nfields, n, r0, rows, h, mode);
}

int mpbp_halo_add_gather(mpbp_halo* H, int32_t nfields, int32_t n, const int32_t* r0s, const int32_t* rows_s) {
    if (!H || !r0s || !rows_s || nfields < 1 || n < 1 || (int64_t)nfields * n * n > INT32_MAX)
        return halo_error(MPBP_ERR_ARG, "halo_add_gather: bad args");
    GatherKind g;
    g.nf = nfields;
    g.n = n;
    int covered = 0;
    for (int k = 0; k < H->world; ++k) {
        if (rows_s[k] < 0 || r0s[k] < 0 || r0s[k] + rows_s[k] > n)
            return halo_error(MPBP_ERR_ARG, "halo_add_gather: rank %d rows [%d, %d) outside %d", k, r0s[k],
                              r0s[k] + rows_s[k], n);
        g.lmax = rows_s[k] > g.lmax ? rows_s[k] : g.lmax;
        covered += rows_s[k];
    }
    if (covered != n || g.lmax < 1) return halo_error(MPBP_ERR_ARG, "halo_add_gather: ranks cover %d of %d rows", covered, n);
    g.rows = rows_s[H->rank];
    const size_t per = (size_t)g.nf * g.lmax * n;
    std::vector<int32_t> full((size_t)nfields * n * n, -1);
    for (int k = 0; k < H->world; ++k)
        for (int f = 0; f < nfields; ++f)
            for (int64_t j = 0; j < (int64_t)rows_s[k] * n; ++j)
                full[(size_t)f * n * n + (size_t)r0s[k] * n + j] = (int32_t)(k * per + (size_t)f * g.lmax * n + j);
    for (int32_t v : full)
        if (v < 0) return halo_error(MPBP_ERR_ARG, "halo_add_gather: ranks' rows overlap or leave gaps");
    int rc = upload_idx(full, &g.full_idx);
    if (!rc && g.rows != g.lmax) {   // pad the owned rows of every field to lmax
        std::vector<int32_t> snd(per, 0);
        for (int f = 0; f < nfields; ++f)
            for (int64_t j = 0; j < (int64_t)g.rows * n; ++j) snd[(size_t)f * g.lmax * n + j] = (int32_t)(f * g.rows * n + j);
        rc = upload_idx(snd, &g.send_idx);
        if (!rc && hipMalloc(&g.send, per * sizeof(double)) != hipSuccess) rc = halo_error(MPBP_ERR_HIP, "halo_add_gather: alloc");
    }
    if (!rc && hipMalloc(&g.stage, per * H->world * sizeof(double)) != hipSuccess)
        rc = halo_error(MPBP_ERR_HIP, "halo_add_gather: alloc");
    if (rc) {
        if (g.full_idx) (void)hipFree(g.full_idx);
        if (g.send_idx) (void)hipFree(g.send_idx);
        if (g.send) (void)hipFree(g.send);
        return rc;
    }
    H->gathers.push_back(g);
    return (int)H->gathers.size() - 1;
}

void mpbp_halo_destroy(mpbp_halo* H) {
    if (!H) return;
    if (H->stream) (void)hipStreamSynchronize(H->stream);
    for (Kind& k : H->kinds) {
        if (k.ready) (void)hipEventDestroy(k.ready);
        if (k.done) (void)hipEventDestroy(k.done);
        if (k.pack_idx) (void)hipFree(k.pack_idx);
        if (k.pack_buf) (void)hipFree(k.pack_buf);
    }
    for (GatherKind& g : H->gathers) {
        if (g.full_idx) (void)hipFree(g.full_idx);
        if (g.send_idx) (void)hipFree(g.send_idx);
        if (g.send) (void)hipFree(g.send);
        if (g.stage) (void)hipFree(g.stage);
    }
    if (H->stream) (void)hipStreamDestroy(H->stream);
    // A communicator whose operations were captured into a hipGraph is not destroyed: with RCCL 2.26.6,
    // ncclCommDestroy never returns once a graph holding this communicator's point-to-point kernels has
    // been instantiated and destroyed (measured: tools/capture_probe.py).  It is
    // released with the process instead (MPBP_HALO_CAPTURED_DESTROY=abort tries ncclCommAbort,
    // =destroy the plain destroy).
    if (H->shared && --H->shared->refs == 0) {   // the last object of the process group
        SharedComm* sc = H->shared;
        if (sc->comm) {
            const char* pol = std::getenv("MPBP_HALO_CAPTURED_DESTROY");
            if (!sc->captured || (pol && std::strcmp(pol, "destroy") == 0)) H->rccl.comm_destroy(sc->comm);
            else if (pol && std::strcmp(pol, "abort") == 0) H->rccl.comm_abort(sc->comm);
        }
        delete sc;
    }
    // the RCCL library stays loaded: torch (or another communicator) may still use it
    delete H;
}

}  // extern "C"

namespace {

// One exchange of vector kind K on stream `on`: a multi-field vector's boundary rows are first gathered
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

int halo_pack(const Kind& K, double* x_ext, hipStream_t on, HaloBufs* b) {
    const int nf = K.nf, h = K.h, n = K.n, L = K.rows;
    b->cnt = (size_t)nf * h * n;
    b->top = x_ext;                               // nf == 1: the rows in place
    b->bot = x_ext + (size_t)(L - h) * n;
    if (nf > 1) {
        const int rc = mpbp_gather((int32_t)(2 * b->cnt), K.pack_idx, x_ext, K.pack_buf, (void*)on);
        if (rc != MPBP_OK) return rc;
        b->top = K.pack_buf;
        b->bot = K.pack_buf + b->cnt;
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
    if (hipStreamIsCapturing(on, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) H->shared->captured = true;
}

ncclResult_t halo_group(mpbp_halo* H, const Kind& K, double* x_ext, hipStream_t on) {
    note_capture(H, on);
    HaloBufs b;
    if (halo_pack(K, x_ext, on, &b) != MPBP_OK) return ncclUnhandledCudaError;
    const ncclResult_t e = H->rccl.group_start();
    const ncclResult_t e2 = e == ncclSuccess ? halo_ops(H, b, on) : e;
    const ncclResult_t eg = H->rccl.group_end();
    return e2 == ncclSuccess ? eg : e2;
}

}  // namespace

extern "C" {

void mpbp_halo_exchange(void* ctx, int32_t vec_kind, double* x_ext, int32_t phase, void* stream) {
    mpbp_halo* H = static_cast<mpbp_halo*>(ctx);
    if (!H || H->status != MPBP_OK) return;
    if (vec_kind < 0 || vec_kind >= (int32_t)H->kinds.size()) {
        fail(H, MPBP_ERR_ARG, "vector kind", "unknown");
        return;
    }
    Kind& K = H->kinds[vec_kind];
    const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (K.mode == MPBP_HALO_IN_ORDER) {
        // the group goes on the caller's stream between the interior and the boundary launches: no event
        // packets (each costs ~15 us of queue latency here), and its host-side enqueue overlaps the interior
        if (phase == MPBP_HALO_END) {
            const ncclResult_t e = halo_group(H, K, x_ext, st);
            if (e != ncclSuccess) fail(H, MPBP_ERR_HIP, "RCCL group", H->rccl.error_string(e));
        }
        return;
    }
    if (phase == MPBP_HALO_END) {
        if (hipStreamWaitEvent(st, K.done, 0) != hipSuccess) fail(H, MPBP_ERR_HIP, "join", "hipStreamWaitEvent");
        return;
    }
    if (hipEventRecord(K.ready, st) != hipSuccess || hipStreamWaitEvent(H->stream, K.ready, 0) != hipSuccess) {
        fail(H, MPBP_ERR_HIP, "fork", "hipEventRecord / hipStreamWaitEvent");
        return;
    }
    const ncclResult_t e = halo_group(H, K, x_ext, H->stream);
    if (e != ncclSuccess) {
        fail(H, MPBP_ERR_HIP, "RCCL group", H->rccl.error_string(e));
        return;
    }
    if (hipEventRecord(K.done, H->stream) != hipSuccess) fail(H, MPBP_ERR_HIP, "fork", "hipEventRecord");
}

void mpbp_halo_exchange_pair(void* ctx, double* xu_ext, double* xp_ext, void* stream) {
    mpbp_halo* H = static_cast<mpbp_halo*>(ctx);
    if (!H || H->status != MPBP_OK) return;
    const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    // both vectors' operations in one group; the velocity rows are gathered before the group opens
    note_capture(H, st);
    HaloBufs bu, bp;
    if (halo_pack(H->kinds[MPBP_VEC_VELOCITY], xu_ext, st, &bu) != MPBP_OK ||
        halo_pack(H->kinds[MPBP_VEC_PRESSURE], xp_ext, st, &bp) != MPBP_OK) {
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

void mpbp_halo_allgather(void* ctx, int32_t gather_kind, const double* x_owned, double* x_full, void* stream) {
    mpbp_halo* H = static_cast<mpbp_halo*>(ctx);
    if (!H || H->status != MPBP_OK) return;
    if (gather_kind < 0 || gather_kind >= (int32_t)H->gathers.size()) {
        fail(H, MPBP_ERR_ARG, "gather kind", "unknown");
        return;
    }
    const GatherKind& g = H->gathers[gather_kind];
    const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    note_capture(H, st);
    const size_t per = (size_t)g.nf * g.lmax * g.n;
    const double* snd = x_owned;
    if (g.send_idx) {
        if (mpbp_gather((int32_t)per, g.send_idx, x_owned, g.send, (void*)st) != MPBP_OK) {
            fail(H, MPBP_ERR_HIP, "gather pack", "mpbp_gather");
            return;
        }
        snd = g.send;
    }
    const ncclResult_t e = H->rccl.all_gather(snd, g.stage, per, ncclFloat64, H->comm, st);
    if (e != ncclSuccess) {
        fail(H, MPBP_ERR_HIP, "ncclAllGather", H->rccl.error_string(e));
        return;
    }
    if (mpbp_gather((int32_t)((size_t)g.nf * g.n * g.n), g.full_idx, g.stage, x_full, (void*)st) != MPBP_OK)
        fail(H, MPBP_ERR_HIP, "gather unpack", "mpbp_gather");
}

int mpbp_halo_set_mode(mpbp_halo* H, int32_t mode) {
    if (!H || (mode != MPBP_HALO_OVERLAP && mode != MPBP_HALO_IN_ORDER))
        return halo_error(MPBP_ERR_ARG, "halo_set_mode: mode must be MPBP_HALO_OVERLAP or MPBP_HALO_IN_ORDER");
    H->default_mode = mode;
    for (Kind& k : H->kinds) k.mode = mode;
    return MPBP_OK;
}

int mpbp_halo_status(const mpbp_halo* H) { return H ? H->status : MPBP_ERR_ARG; }

const char* mpbp_halo_last_error(const mpbp_halo* H) { return (H && H->status != MPBP_OK) ? H->err : g_halo_err; }

}  // extern "C"
