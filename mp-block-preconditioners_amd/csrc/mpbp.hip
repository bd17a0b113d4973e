// libmpbp -- MI355X (gfx950) HIP kernels + C ABI for the multiphase-Stokes
// block-preconditioner apply.  Header: include/mpbp.h.  Design: DESIGN.md.
//
// Built with -ffp-contract=off: every kernel performs the IEEE operations of the
// sequential checker oracle/csr_oracle.c in the same order (row sums left to
// right from 0.0, no fused multiply-add), so results are bit-identical to it.
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <type_traits>
#include <vector>

#include "mpbp.h"

namespace {

thread_local char g_err[1024] = "";
// Kernel choices (mpbp_kernel_opts, include/mpbp.h): the process defaults (mpbp_set_*), and the choices of the plan
// being applied -- mpbp_schur_apply / mpbp_mg_solve install their plan's copy for the duration of the call (OptsScope),
// so two preconditioners with different choices coexist and a captured graph holds its own plan's choices.
// Measured defaults: march_rows 0 = the count that fills one round of workgroups (256^2 1 row -> 13.5k applies/s vs
// 7.6k at 4; 1024^2 4; 2048^2 16 -> 753 vs 727).
mpbp_kernel_opts g_defaults = {
    /*march_rows*/ 0, /*init_diag*/ 1, /*f_pair*/ 1, /*f_direct*/ 0, /*gtg_fused*/ 1, /*gtg_tpb*/ 512, /*gtg_drhs*/ 1,
    /*q13_sym*/ 1, /*f_tile*/ 1, /*f_solve*/ 1, /*mg_galerkin_mf*/ 2, /*mg_galerkin_mf_p*/ 1, /*pg_direct*/ 1,
    /*mg_group_rows*/ 65536, /*mg_svl*/ 1, /*mg_mf_transfer*/ 1, /*csr_table*/ 1, /*mg_fuse_l0*/ 1,
    /*mg_coarse_tree*/ 0, /*f_solve_tile*/ 1, /*q13_mf*/ 0, /*mg_fuse_small*/ 1, /*gtg_solve_tile*/ 1, {0}};
thread_local const mpbp_kernel_opts* t_opts = nullptr;
inline const mpbp_kernel_opts& KO() { return t_opts ? *t_opts : g_defaults; }
struct OptsScope {   // installs a plan's kernel choices (when it has its own) for one entry-point call
    const mpbp_kernel_opts* prev;
    explicit OptsScope(const mpbp_kernel_opts* o) : prev(t_opts) {
        if (o) t_opts = o;
    }
    ~OptsScope() { t_opts = prev; }
};
inline int pg_rows() { return KO().march_rows; }
// a plan's kernel choices must be values the setters accept
int set_error(int code, const char* fmt, ...);
inline int check_opts(const mpbp_kernel_opts* o, const char* who) {
    if (!o) return MPBP_OK;
    const bool ok = o->march_rows >= 0 && o->march_rows <= 4096 && (o->gtg_tpb == 256 || o->gtg_tpb == 512) &&
                    o->f_solve_tile >= 0 && o->f_solve_tile <= 1 &&
                    o->mg_galerkin_mf >= 0 && o->mg_galerkin_mf <= 2 && o->mg_group_rows >= 0 &&
                    (o->init_diag | o->f_pair | o->f_direct | o->gtg_fused | o->gtg_drhs | o->q13_sym | o->f_tile |
                     o->f_solve | o->mg_galerkin_mf_p | o->pg_direct | o->mg_svl | o->mg_mf_transfer | o->csr_table |
                     o->mg_fuse_l0 | o->mg_coarse_tree | o->q13_mf | o->mg_fuse_small | o->gtg_solve_tile) >= 0 &&
                    (o->init_diag | o->f_pair | o->f_direct | o->gtg_fused | o->gtg_drhs | o->q13_sym | o->f_tile |
                     o->f_solve | o->mg_galerkin_mf_p | o->pg_direct | o->mg_svl | o->mg_mf_transfer | o->csr_table |
                     o->mg_fuse_l0 | o->mg_coarse_tree | o->q13_mf | o->mg_fuse_small | o->gtg_solve_tile) <= 1;
    return ok ? MPBP_OK : set_error(MPBP_ERR_ARG, "%s: kernel options out of range", who);
}   // rows per workgroup of the D / G / Gt_G marching kernels: as F

int set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

#define MPBP_HIP(call)                                                                      \
    do {                                                                                    \
        hipError_t e_ = (call);                                                             \
        if (e_ != hipSuccess)                                                               \
            return set_error(MPBP_ERR_HIP, "%s: %s", #call, hipGetErrorString(e_));         \
    } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int kBlock = 256;                    // 4 wave64 per workgroup, one row per thread

inline int grid_for(int64_t n, int block = kBlock) { return (int)((n + block - 1) / block); }

// Cache policy of the once-touched streams.  The SELL and CSR kernels read their matrix (touched once per SpMV)
// and write their result with nontemporal hints (+2-4 % on the 1024^2 A SpMV); the stencil kernels keep
// default-policy loads and stores (their x / b / d vectors are re-read by the next sweep from the cache;
// nontemporal costs them 3-7 %).
constexpr bool kSellNT = true, kCsrNT = true;
template <class T>
__device__ inline T ld_stream(const T* p) { return *p; }
template <bool NT = false, class T>
__device__ inline void st_stream(T* p, T v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ inline double2 ld_matrix(const double2* p) {
    if constexpr (NT) {
        const f64x2 v = __builtin_nontemporal_load(reinterpret_cast<const f64x2*>(p));
        return make_double2(v.x, v.y);
    } else {
        return *p;
    }
}
template <bool NT>
__device__ inline int2 ld_matrix(const int2* p) {
    if constexpr (NT) {
        const i32x2 v = __builtin_nontemporal_load(reinterpret_cast<const i32x2*>(p));
        return make_int2(v.x, v.y);
    } else {
        return *p;
    }
}

// ================================================================== theta ====
// thn(y, x) = 0.25 sin(2 pi x) sin(2 pi y) + 0.5 -- preconditioner.py:9-11
__device__ inline double thn_fn(double y, double x) {
    const double two_pi = 2.0 * 3.141592653589793;
    return 0.25 * sin(two_pi * x) * sin(two_pi * y) + 0.5;
}

__global__ void k_theta(int n, double* cell, double* uface, double* vface) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)n * n) return;
    const int r = (int)(i / n), c = (int)(i % n);
    const double dx = 1.0 / n, dy = 1.0 / n;
    cell[i] = thn_fn(-(r + 0.5) * dy, (c + 0.5) * dx);   // get_thn_vals cell centres
    uface[i] = thn_fn(-(r + 0.5) * dy, c * dx);          // w_thn, u rows (preconditioner.py:325)
    vface[i] = thn_fn((double)(-r) * dy, (c + 0.5) * dx);  // w_thn, v rows (preconditioner.py:326)
}

// =============================================================== stencils ====
// The reference assigns into dense matrices; a later write to the same (row, col)
// replaces the earlier one (n <= 2 only).  RowBuf restates that: last write wins.
struct RowBuf {
    int m;
    int32_t col[16];
    double val[16];
};

__device__ inline void put(RowBuf& w, int32_t col, double v) {
    for (int k = 0; k < w.m; ++k)
        if (w.col[k] == col) { w.val[k] = v; return; }
    w.col[w.m] = col;
    w.val[w.m] = v;
    ++w.m;
}

__device__ inline void sort_row(RowBuf& w) {
    for (int i = 1; i < w.m; ++i) {
        const int32_t cj = w.col[i];
        const double cv = w.val[i];
        int t = i - 1;
        while (t >= 0 && w.col[t] > cj) { w.col[t + 1] = w.col[t]; w.val[t + 1] = w.val[t]; --t; }
        w.col[t + 1] = cj;
        w.val[t + 1] = cv;
    }
}

// Periodic cell-centred volume fraction of one phase (ths = 1 - thn, preconditioner.py:74-81).
struct Phase {
    int n;
    const double* cell;
    int s;
    // Periodic index for a in [-1, n]: every stencil offset is +-1 (no integer division).
    __device__ int wrap(int a) const { return a < 0 ? a + n : (a >= n ? a - n : a); }
    __device__ int32_t idx(int r, int c) const { return wrap(r) * n + wrap(c); }
    __device__ double T(int r, int c) const { const double v = cell[idx(r, c)]; return s ? 1.0 - v : v; }
};

// L rows of one phase (2N x 2N) and the XI diagonal entry of that row.
// u rows: preconditioner.py:100-179 ; v rows: preconditioner.py:240-295 ; XI: :124-125.
__device__ void phase_L_row(const Phase& g, double xi, int32_t i, RowBuf& w, double& xi_ii) {
    const int n = g.n;
    const int32_t N = n * n;
    const double dx = 1.0 / n, dy = 1.0 / n;
    w.m = 0;
    if (i < N) {
        const int r = i / n, c = i % n;
        const double tij = g.T(r, c - 1), tip1j = g.T(r, c);
        const double tijp1 = g.T(r - 1, c - 1), tip1jp1 = g.T(r - 1, c);
        const double tijm1 = g.T(r + 1, c - 1), tip1jm1 = g.T(r + 1, c);
        const double iph_jph = 0.25 * (tij + tijp1 + tip1jp1 + tip1j);
        const double iph_jmh = 0.25 * (tij + tip1j + tijm1 + tip1jm1);
        const double iph_j = 0.5 * (tij + tip1j);
        xi_ii = xi * iph_j * (1.0 - iph_j);
        put(w, i, 1.0 / (dx * dx) * (-tip1j - tij) + 1.0 / (dy * dy) * (-iph_jph - iph_jmh));
        put(w, N + g.idx(r, c), 1.0 / (dx * dy) * (-tip1j + iph_jph));
        put(w, g.idx(r, c - 1), 1.0 / (dx * dx) * (tij));
        put(w, g.idx(r, c + 1), tip1j / (dx * dx));
        put(w, g.idx(r - 1, c), 1.0 / (dy * dy) * (iph_jph));
        put(w, g.idx(r + 1, c), 1.0 / (dy * dy) * (iph_jmh));
        put(w, N + g.idx(r, c - 1), 1.0 / (dy * dx) * (tij - iph_jph));
        put(w, N + g.idx(r + 1, c - 1), 1.0 / (dy * dx) * (iph_jmh - tij));
        put(w, N + g.idx(r + 1, c), 1.0 / (dx * dy) * (tip1j - iph_jmh));
    } else {
        const int32_t k = i - N;
        const int r = k / n, c = k % n;
        const double ip1_jph = 0.5 * (g.T(r, c) + g.T(r - 1, c));   // set in the u loop (:125)
        xi_ii = xi * ip1_jph * (1.0 - ip1_jph);
        const double tij = g.T(r, c), tip1j = g.T(r, c + 1);
        const double tijp1 = g.T(r - 1, c), tip1jp1 = g.T(r - 1, c + 1);
        const double tim1j = g.T(r, c - 1), tim1jp1 = g.T(r - 1, c - 1);
        const double imh_jph = 0.25 * (tim1j + tim1jp1 + tij + tijp1);
        const double iph_jph = 0.25 * (tij + tip1j + tijp1 + tip1jp1);
        put(w, i, -1.0 / (dy * dy) * (tijp1 + tij) - 1.0 / (dx * dx) * (iph_jph + imh_jph));
        put(w, N + g.idx(r, c - 1), 1.0 / (dx * dx) * imh_jph);
        put(w, N + g.idx(r, c + 1), 1.0 / (dx * dx) * iph_jph);
        put(w, N + g.idx(r - 1, c), 1.0 / (dy * dy) * tijp1);
        put(w, N + g.idx(r + 1, c), 1.0 / (dy * dy) * tij);
        put(w, k, 1.0 / (dx * dy) * (imh_jph - tij));
        put(w, g.idx(r, c + 1), 1.0 / (dy * dx) * (tij - iph_jph));
        put(w, g.idx(r - 1, c), 1.0 / (dy * dx) * (tijp1 - imh_jph));
        put(w, g.idx(r - 1, c + 1), 1.0 / (dy * dx) * (iph_jph - tijp1));
    }
    sort_row(w);
}

// G rows of one phase (2N x N), preconditioner.py:203-219.
__device__ void phase_G_row(const Phase& g, int32_t i, RowBuf& w) {
    const int n = g.n;
    const int32_t N = n * n;
    const double dx = 1.0 / n, dy = 1.0 / n;
    w.m = 0;
    if (i < N) {
        const int r = i / n, c = i % n;
        const double imh_j = 0.5 * (g.T(r, c) + g.T(r, c - 1));
        put(w, i, (1.0 / dx) * imh_j);
        put(w, g.idx(r, c - 1), -(1.0 / dx) * imh_j);
    } else {
        const int32_t k = i - N;
        const int r = k / n, c = k % n;
        const double i_jph = 0.5 * (g.T(r, c) + g.T(r - 1, c));
        put(w, k, -(1.0 / dy) * i_jph);
        put(w, g.idx(r - 1, c), (1.0 / dy) * i_jph);
    }
    sort_row(w);
}

// D rows of one phase (N x 2N), preconditioner.py:221-238.
__device__ void phase_D_row(const Phase& g, int32_t k, RowBuf& w) {
    const int n = g.n;
    const int32_t N = n * n;
    const double dx = 1.0 / n, dy = 1.0 / n;
    const int r = k / n, c = k % n;
    const double tij = g.T(r, c);
    const double iph_j = 0.5 * (tij + g.T(r, c + 1));
    const double imh_j = 0.5 * (tij + g.T(r, c - 1));
    const double i_jph = 0.5 * (tij + g.T(r - 1, c));
    const double i_jmh = 0.5 * (tij + g.T(r + 1, c));
    w.m = 0;
    put(w, g.idx(r, c + 1), 1.0 / dx * iph_j);
    put(w, k, -1.0 / dx * imh_j);
    put(w, N + k, 1.0 / dy * i_jph);
    put(w, N + g.idx(r + 1, c), -1.0 / dy * i_jmh);
    sort_row(w);
}

struct StokesDev {
    int n;
    double xi, eta_n, eta_s, c, d_u, d_p, d_div;
    const double* cell;
    const double* uface;
    const double* vface;
};

__device__ inline void append(RowBuf& o, int32_t col, double v) {
    o.col[o.m] = col;
    o.val[o.m] = v;
    ++o.m;
}

// F row R of [u_n, v_n, u_s, v_s]: F = XI + d_u blockdiag(eta_n L_n, eta_s L_s)
// (preconditioner.py:310, 315-337).  Columns come out sorted.
__device__ void F_row(const StokesDev& P, int32_t R, RowBuf& o) {
    const int32_t N = P.n * P.n;
    const int p = R >= 2 * N;
    const int32_t i = R - p * 2 * N;
    const Phase g{P.n, P.cell, p};
    RowBuf L;
    double xi_ii;
    phase_L_row(g, P.xi, i, L, xi_ii);
    // Face tables are absent when only the pattern is counted.
    const double th = !P.uface ? 0.0 : (i < N) ? P.uface[i] : P.vface[i - N];
    const double w = p ? P.c * (1.0 - th) : P.c * th;          // w_ths = c*ths, w_thn = c*thn
    const double eta = p ? P.eta_s : P.eta_n;
    const int32_t off = p * 2 * N, other = (1 - p) * 2 * N;
    o.m = 0;
    if (p == 1) append(o, other + i, P.d_u * xi_ii);              // d_u * XI_s (cross block)
    for (int k = 0; k < L.m; ++k) {
        double v = P.d_u * (eta * L.val[k]);
        if (L.col[k] == i) v = (w - P.d_u * xi_ii) + v;           // (w - d_u XI) + d_u eta L
        append(o, off + L.col[k], v);
    }
    if (p == 0) append(o, other + i, P.d_u * xi_ii);              // d_u * XI_n (cross block)
}

__device__ void build_row(const StokesDev& P, int op, int32_t R, RowBuf& o) {
    const int32_t N = P.n * P.n;
    RowBuf t;
    double xi_ii;
    o.m = 0;
    switch (op) {
    case MPBP_OP_A:
        if (R < 4 * N) {
            F_row(P, R, o);
            const int p = R >= 2 * N;
            phase_G_row(Phase{P.n, P.cell, p}, R - p * 2 * N, t);
            for (int k = 0; k < t.m; ++k) append(o, 4 * N + t.col[k], P.d_p * t.val[k]);
        } else {
            const int32_t q = R - 4 * N;
            phase_D_row(Phase{P.n, P.cell, 0}, q, t);
            for (int k = 0; k < t.m; ++k) append(o, t.col[k], P.d_div * t.val[k]);
            phase_D_row(Phase{P.n, P.cell, 1}, q, t);
            for (int k = 0; k < t.m; ++k) append(o, 2 * N + t.col[k], P.d_div * t.val[k]);
        }
        break;
    case MPBP_OP_F:
        F_row(P, R, o);
        break;
    case MPBP_OP_D:
        phase_D_row(Phase{P.n, P.cell, 0}, R, t);
        for (int k = 0; k < t.m; ++k) append(o, t.col[k], t.val[k]);
        phase_D_row(Phase{P.n, P.cell, 1}, R, t);
        for (int k = 0; k < t.m; ++k) append(o, 2 * N + t.col[k], t.val[k]);
        break;
    case MPBP_OP_G: {
        const int p = R >= 2 * N;
        phase_G_row(Phase{P.n, P.cell, p}, R - p * 2 * N, t);
        for (int k = 0; k < t.m; ++k) append(o, t.col[k], P.d_p * t.val[k]);
        break;
    }
    case MPBP_OP_L_N:
    case MPBP_OP_L_S:
        phase_L_row(Phase{P.n, P.cell, op == MPBP_OP_L_S}, P.xi, R, o, xi_ii);
        break;
    case MPBP_OP_D_N:
    case MPBP_OP_D_S:
        phase_D_row(Phase{P.n, P.cell, op == MPBP_OP_D_S}, R, o);
        break;
    case MPBP_OP_G_N:
    case MPBP_OP_G_S:
        phase_G_row(Phase{P.n, P.cell, op == MPBP_OP_G_S}, R, o);
        break;
    case MPBP_OP_XI_N:
    case MPBP_OP_XI_S:
        phase_L_row(Phase{P.n, P.cell, op == MPBP_OP_XI_S}, P.xi, R, t, xi_ii);
        append(o, R, xi_ii);
        break;
    default:
        break;
    }
}

// rows (optional): the operator rows to assemble, in order (a rank's owned + ghost rows); the output CSR's row i is
// operator row rows[i] with its global columns.  NULL: every row.
__global__ void k_stokes_count(StokesDev P, int op, int64_t nrows, int32_t* row_nnz, const int32_t* rows = nullptr) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nrows) return;
    RowBuf o;
    build_row(P, op, rows ? rows[i] : (int32_t)i, o);
    row_nnz[i] = o.m;
}

__global__ void k_stokes_fill(StokesDev P, int op, int64_t nrows, const int32_t* rp, int32_t* ci,
                              double* va, const int32_t* rows = nullptr) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nrows) return;
    RowBuf o;
    build_row(P, op, rows ? rows[i] : (int32_t)i, o);
    const int32_t base = rp[i];
    for (int k = 0; k < o.m; ++k) {
        ci[base + k] = o.col[k];
        va[base + k] = o.val[k];
    }
}

// One 1024-thread workgroup scans the whole array in 1024-element chunks (setup only).
// Exclusive scan of row counts into row_ptr (int64 running sums, so an int32 overflow is detected).
// Three passes over tiles of kScanTile counts: tile sums; one workgroup scans the tile sums (and writes
// row_ptr[n] = total); every tile then scans its counts from LDS and adds its offset.
constexpr int kScanTile = 4096;   // 256 threads x 16 counts

// Inclusive scan of one value per thread over a 256-thread workgroup; *sum = the workgroup's total.
__device__ inline long long block_scan256(long long x, long long* wsum, long long* sum) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int d = 1; d < 64; d <<= 1) {
        const long long y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    long long off = 0;
    for (int w = 0; w < wid; ++w) off += wsum[w];
    *sum = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
    return x + off;
}

// Tile t's counts into LDS (coalesced; zeros past n).
__device__ inline void scan_load_tile(const int32_t* in, int64_t n, int32_t* tile) {
    const int64_t base = (int64_t)blockIdx.x * kScanTile;
    for (int i = threadIdx.x; i < kScanTile; i += 256) tile[i] = base + i < n ? in[base + i] : 0;
    __syncthreads();
}

__global__ void __launch_bounds__(256) k_scan_tiles(const int32_t* in, int64_t n, long long* tile_sum) {
    __shared__ int32_t tile[kScanTile];
    __shared__ long long wsum[4];
    scan_load_tile(in, n, tile);
    long long s = 0;
    for (int i = 0; i < 16; ++i) s += tile[threadIdx.x * 16 + i];
    long long tot;
    block_scan256(s, wsum, &tot);
    if (threadIdx.x == 0) tile_sum[blockIdx.x] = tot;
}

// In place: tile_sum[t] -> exclusive prefix of the tile sums; out[n] = total = *total.
__global__ void __launch_bounds__(256) k_scan_offsets(long long* tile_sum, int64_t ntiles, int32_t* out, int64_t n,
                                                      long long* total) {
    __shared__ long long wsum[4];
    long long carry = 0;
    for (int64_t base = 0; base < ntiles; base += 256) {
        const int64_t i = base + threadIdx.x;
        const long long v = i < ntiles ? tile_sum[i] : 0;
        long long sum;
        const long long inc = block_scan256(v, wsum, &sum);
        if (i < ntiles) tile_sum[i] = carry + inc - v;
        carry += sum;
    }
    if (threadIdx.x == 0) {
        out[n] = (int32_t)carry;
        *total = carry;
    }
}

__global__ void __launch_bounds__(256) k_scan_apply(const int32_t* in, int64_t n, const long long* tile_off,
                                                    int32_t* out) {
    __shared__ int32_t tile[kScanTile];
    __shared__ long long wsum[4];
    scan_load_tile(in, n, tile);
    int32_t c[16];
    long long s = 0;
    for (int i = 0; i < 16; ++i) {
        c[i] = tile[threadIdx.x * 16 + i];
        s += c[i];
    }
    long long tot;
    long long run = tile_off[blockIdx.x] + block_scan256(s, wsum, &tot) - s;
    for (int i = 0; i < 16; ++i) {   // exclusive values back into the tile (this thread's own slots)
        tile[threadIdx.x * 16 + i] = (int32_t)run;
        run += c[i];
    }
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * kScanTile;
    for (int i = threadIdx.x; i < kScanTile; i += 256)
        if (base + i < n) out[base + i] = tile[i];
}

// ================================================================ SpGEMM ====
struct Csr {
    const int32_t* rp;
    const int32_t* ci;
    const double* va;
    int32_t ncols = 0;   // set by to_csr (the uniform CSR path's x buffer descriptor); 0 = unknown
};

constexpr int kSpgemmMaxW = 64;

// Row r of A*B: first-touch order over (A row order, B row order), then sorted by column.
// Same operation order as oracle/csr_oracle.c:row_product.
__device__ int spgemm_row(const Csr A, const Csr B, int32_t r, int32_t* cols, double* vals) {
    int m = 0;
    for (int32_t ka = A.rp[r]; ka < A.rp[r + 1]; ++ka) {
        const double a = A.va[ka];
        const int32_t k = A.ci[ka];
        for (int32_t kb = B.rp[k]; kb < B.rp[k + 1]; ++kb) {
            const int32_t j = B.ci[kb];
            const double v = a * B.va[kb];
            int t = 0;
            while (t < m && cols[t] != j) ++t;
            if (t < m) {
                vals[t] += v;
            } else {
                if (m == kSpgemmMaxW) return -1;
                cols[m] = j;
                vals[m] = v;
                ++m;
            }
        }
    }
    for (int i = 1; i < m; ++i) {
        const int32_t cj = cols[i];
        const double cv = vals[i];
        int t = i - 1;
        while (t >= 0 && cols[t] > cj) { cols[t + 1] = cols[t]; vals[t + 1] = vals[t]; --t; }
        cols[t + 1] = cj;
        vals[t + 1] = cv;
    }
    return m;
}

__global__ void k_spgemm_count(Csr A, Csr B, int32_t nrows, int32_t* row_nnz, int* overflow) {
    const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrows) return;
    int32_t cols[kSpgemmMaxW];
    double vals[kSpgemmMaxW];
    const int m = spgemm_row(A, B, r, cols, vals);
    if (m < 0) { atomicAdd(overflow, 1); row_nnz[r] = 0; }
    else row_nnz[r] = m;
}

__global__ void k_spgemm_fill(Csr A, Csr B, int32_t nrows, double alpha, const int32_t* crp,
                              int32_t* cci, double* cva) {
    const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrows) return;
    int32_t cols[kSpgemmMaxW];
    double vals[kSpgemmMaxW];
    const int m = spgemm_row(A, B, r, cols, vals);
    const int32_t base = crp[r];
    for (int k = 0; k < m; ++k) {
        cci[base + k] = cols[k];
        cva[base + k] = alpha * vals[k];
    }
}

// ============================================================ helpers ====
__global__ void k_csr_diag(Csr A, int32_t nrows, int32_t col_offset, double* diag, int* missing) {
    const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrows) return;
    double d = 0.0;
    bool found = false;
    for (int32_t k = A.rp[r]; k < A.rp[r + 1]; ++k)
        if (A.ci[k] == r + col_offset) { d = A.va[k]; found = true; }
    diag[r] = d;
    if (!found) atomicAdd(missing, 1);
}

__global__ void k_gershgorin(Csr A, int32_t nrows, const double* diag, unsigned long long* out) {
    const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    double q = 0.0;
    if (r < nrows) {
        double s = 0.0;
        for (int32_t k = A.rp[r]; k < A.rp[r + 1]; ++k) s += fabs(A.va[k]);
        q = s / fabs(diag[r]);
    }
    // non-negative doubles order like their bit patterns
    for (int d = 32; d > 0; d >>= 1) {
        const double o = __shfl_xor(q, d, 64);
        q = o > q ? o : q;
    }
    if ((threadIdx.x & 63) == 0) atomicMax(out, (unsigned long long)__double_as_longlong(q));
}

__global__ void k_extract_count(Csr A, const int32_t* rows, int32_t nloc, int32_t* row_nnz) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nloc) return;
    const int32_t r = rows[i];
    row_nnz[i] = A.rp[r + 1] - A.rp[r];
}

__global__ void k_extract_fill(Csr A, const int32_t* rows, int32_t nloc, const int32_t* colmap,
                               const int32_t* lrp, int32_t* lci, double* lva, int* bad) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nloc) return;
    const int32_t r = rows[i];
    int32_t o = lrp[i];
    for (int32_t k = A.rp[r]; k < A.rp[r + 1]; ++k, ++o) {   // keep the global row's order
        const int32_t lc = colmap[A.ci[k]];
        if (lc < 0) atomicAdd(bad, 1);
        lci[o] = lc < 0 ? 0 : lc;
        lva[o] = A.va[k];
    }
}

__global__ void k_gather(int32_t count, const int32_t* idx, const double* src, double* dst) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) dst[i] = src[idx[i]];
}

__global__ void k_scatter(int32_t count, const int32_t* idx, const double* src, double* dst) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) dst[idx[i]] = src[i];
}

// ============================================================ multigrid transfers ====
// Geometric coarsening of a periodic n x n MAC grid by 2 in each direction, field by field.  Along an axis a
// field is cell-centred (MPBP_MG_CELL: fine 2i and 2i+1 lie around coarse i, linear weights 3/4, 1/4) or
// node-centred (MPBP_MG_NODE: fine 2i sits on coarse i, fine 2i+1 halfway to coarse i+1).  P (fine <- coarse)
// is the tensor product of the two 1D lists; R = P^T exactly.  Every weight is a dyadic rational, so the
// values are exact and the columns of each row come out sorted (periodic wrap included).
struct MgFields {
    int32_t nfields;
    int32_t ky[8], kx[8];
};

template <int CAP>
__device__ inline void sort_pairs(int m, int* idx, double* w) {
#pragma unroll
    for (int a = 1; a < CAP; ++a)
#pragma unroll
        for (int b = CAP - 1; b >= a; --b)
            if (b < m && idx[b - 1] > idx[b]) {
                const int ti = idx[b - 1];
                idx[b - 1] = idx[b];
                idx[b] = ti;
                const double tw = w[b - 1];
                w[b - 1] = w[b];
                w[b] = tw;
            }
}

// P's 1D list for fine index f (coarse size nc): <= 2 entries.
__device__ inline int mg_p1d(int kind, int nc, int f, int* idx, double* w) {
    const int i = f >> 1;
    if (kind == MPBP_MG_NODE && !(f & 1)) {
        idx[0] = i;
        w[0] = 1.0;
        return 1;
    }
    const int j = (kind == MPBP_MG_CELL && !(f & 1)) ? (i + nc - 1) % nc : (i + 1) % nc;
    idx[0] = i;
    w[0] = kind == MPBP_MG_CELL ? 0.75 : 0.5;
    idx[1] = j;
    w[1] = kind == MPBP_MG_CELL ? 0.25 : 0.5;
    sort_pairs<2>(2, idx, w);
    return 2;
}

// R's 1D list for coarse index i (fine size nf) = column i of P: <= 4 entries.
__device__ inline int mg_r1d(int kind, int nf, int i, int* idx, double* w) {
    const int f = 2 * i;
    int m;
    if (kind == MPBP_MG_CELL) {
        idx[0] = (f + nf - 1) % nf; w[0] = 0.25;
        idx[1] = f;                 w[1] = 0.75;
        idx[2] = f + 1;             w[2] = 0.75;
        idx[3] = (f + 2) % nf;      w[3] = 0.25;
        m = 4;
    } else {
        idx[0] = (f + nf - 1) % nf; w[0] = 0.5;
        idx[1] = f;                 w[1] = 1.0;
        idx[2] = f + 1;             w[2] = 0.5;
        m = 3;
    }
    sort_pairs<4>(m, idx, w);
    return m;
}

// Unsigned division by a run-time invariant d (>= 1) with one high multiply (Granlund-Montgomery, round-up variant):
// q = (umulhi(x, m) + x) >> s for every 32-bit x.
struct DivU {
    uint32_t m, s;
};
inline DivU divu(uint32_t d) {
    uint32_t s = 0;
    while ((uint64_t(1) << s) < d) ++s;
    const uint64_t m = ((uint64_t(1) << 32) * ((uint64_t(1) << s) - d)) / d + 1;
    return DivU{(uint32_t)m, s};
}
__device__ inline uint32_t divu(uint32_t x, DivU d) {
    return (uint32_t)(((uint64_t)__umulhi(x, d.m) + x) >> d.s);
}

// P's 1D list for fine index f (coarse size nc), in increasing index order (= mg_p1d's sorted list)
__device__ inline int mg_p1d_fast(int kind, int nc, int f, int* idx, double* w) {
    const int i = f >> 1;
    if (kind == MPBP_MG_NODE && !(f & 1)) {
        idx[0] = i;
        w[0] = 1.0;
        return 1;
    }
    const double wi = kind == MPBP_MG_CELL ? 0.75 : 0.5, wj = kind == MPBP_MG_CELL ? 0.25 : 0.5;
    const bool down = kind == MPBP_MG_CELL && !(f & 1);             // the other coarse point is i - 1, else i + 1
    const int j = down ? (i == 0 ? nc - 1 : i - 1) : (i + 1 == nc ? 0 : i + 1);
    const bool jfirst = j < i;
    idx[0] = jfirst ? j : i;  w[0] = jfirst ? wj : wi;
    idx[1] = jfirst ? i : j;  w[1] = jfirst ? wi : wj;
    return 2;
}
// R's 1D list for coarse index i (fine size nf), in increasing index order (= mg_r1d's sorted list)
__device__ inline int mg_r1d_fast(int kind, int nf, int i, int* idx, double* w) {
    const int f = 2 * i;
    if (kind == MPBP_MG_CELL) {   // f-1, f, f+1, f+2 with 1/4, 3/4, 3/4, 1/4; the wrapped one moves to its end
        if (f == 0) {
            idx[0] = 0; w[0] = 0.75; idx[1] = 1; w[1] = 0.75; idx[2] = 2 % nf; w[2] = 0.25; idx[3] = nf - 1; w[3] = 0.25;
        } else if (f + 2 == nf) {
            idx[0] = 0; w[0] = 0.25; idx[1] = f - 1; w[1] = 0.25; idx[2] = f; w[2] = 0.75; idx[3] = f + 1; w[3] = 0.75;
        } else {
            idx[0] = f - 1; w[0] = 0.25; idx[1] = f; w[1] = 0.75; idx[2] = f + 1; w[2] = 0.75; idx[3] = f + 2; w[3] = 0.25;
        }
        return 4;
    }
    if (f == 0) {                 // f-1, f, f+1 with 1/2, 1, 1/2
        idx[0] = 0; w[0] = 1.0; idx[1] = 1; w[1] = 0.5; idx[2] = nf - 1; w[2] = 0.5;
    } else {
        idx[0] = f - 1; w[0] = 0.5; idx[1] = f; w[1] = 1.0; idx[2] = f + 1; w[2] = 0.5;
    }
    return 3;
}

// y = op(T x) for T = P or R of the n x n grid (n = fine size), matrix-free: each row rebuilds its tensor-product
// weights and columns exactly as k_mg_transfer stores them (same order, same products), so the sums are the CSR
// SpMV's bit for bit; no matrix stream, and the x gathers issue without waiting for column loads.  The row's field
// and grid position come from two multiply-shift divisions and the 1D lists from selects (no integer division, no
// sorting network: 28 -> ~8 us for the 1024^2 prolongation).
struct MgDiv {
    DivU per, nr;   // rows per field, grid size of the rows' level
};
// Row `row` of T = P (rows = fine unknowns) or R (rows = coarse unknowns) of the n x n fine grid: its field, the 1D
// lists of both directions and the columns' field offset (nk = the columns' grid size).  The one place the matrix-free
// transfers build a row, so every kernel that folds a transfer in takes the same lists in the same order.
struct MgRow {
    int my, mx, nk, off;
    int yi[4], xi[4];
    double yw[4], xw[4];
};
__device__ inline void mg_row(const MgFields& F, const MgDiv& dv, int32_t n, int32_t which, int32_t row, MgRow& T) {
    const int nc = n / 2;
    const int nr = which == MPBP_MG_P ? n : nc;
    T.nk = which == MPBP_MG_P ? nc : n;
    const uint32_t per = (uint32_t)nr * (uint32_t)nr;
    const int fld = (int)divu((uint32_t)row, dv.per);
    const uint32_t cell = (uint32_t)row - (uint32_t)fld * per;
    const int r = (int)divu(cell, dv.nr), c = (int)(cell - (uint32_t)r * (uint32_t)nr);
    T.my = which == MPBP_MG_P ? mg_p1d_fast(F.ky[fld], nc, r, T.yi, T.yw) : mg_r1d_fast(F.ky[fld], n, r, T.yi, T.yw);
    T.mx = which == MPBP_MG_P ? mg_p1d_fast(F.kx[fld], nc, c, T.xi, T.xw) : mg_r1d_fast(F.kx[fld], n, c, T.xi, T.xw);
    T.off = fld * T.nk * T.nk;
}
template <class Epi>
__global__ void __launch_bounds__(kBlock) k_mg_transfer_spmv(MgFields F, MgDiv dv, int32_t n, int32_t which,
                                                             int32_t nrows, const double* __restrict__ x, Epi epi) {
    const int32_t row = (int32_t)(blockIdx.x * kBlock + threadIdx.x);
    if (row >= nrows) return;
    const typename Epi::P pe = epi.pre(row);
    MgRow T;
    mg_row(F, dv, n, which, row, T);
    double acc = 0.0;
#pragma unroll
    for (int a = 0; a < 4; ++a)   // (constant trip counts keep the lists in registers)
#pragma unroll
        for (int b = 0; b < 4; ++b)
            if (a < T.my && b < T.mx) acc += (T.yw[a] * T.xw[b]) * x[T.off + T.yi[a] * T.nk + T.xi[b]];
    epi(row, acc, pe);
}

// which: MPBP_MG_P (rows = fine unknowns) or MPBP_MG_R (rows = coarse unknowns); n = fine grid size.
// rl (optional): the global rows to build, output row i = rl[i] (a rank's band of a row-partitioned hierarchy)
__global__ void k_mg_transfer(MgFields F, int32_t n, int32_t which, int64_t nrows, const int32_t* rp,
                              int32_t* row_nnz, int32_t* ci, double* va, const int32_t* rl = nullptr) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nrows) return;
    const int64_t row = rl ? (int64_t)rl[i] : i;
    const int nc = n / 2;
    const int nr = which == MPBP_MG_P ? n : nc;       // grid size of the rows' level
    const int nk = which == MPBP_MG_P ? nc : n;       // ... and of the columns' level
    const int64_t per = (int64_t)nr * nr;
    const int fld = (int)(row / per);
    const int64_t cell = row - fld * per;
    const int r = (int)(cell / nr), c = (int)(cell % nr);
    int yi[4], xi[4];
    double yw[4], xw[4];
    const int my = which == MPBP_MG_P ? mg_p1d(F.ky[fld], nc, r, yi, yw) : mg_r1d(F.ky[fld], n, r, yi, yw);
    const int mx = which == MPBP_MG_P ? mg_p1d(F.kx[fld], nc, c, xi, xw) : mg_r1d(F.kx[fld], n, c, xi, xw);
    if (row_nnz) {
        row_nnz[i] = my * mx;
        return;
    }
    const int64_t off = (int64_t)fld * nk * nk;
    int32_t k = rp[i];
    for (int a = 0; a < my; ++a)
        for (int b = 0; b < mx; ++b) {
            ci[k] = (int32_t)(off + (int64_t)yi[a] * nk + xi[b]);
            va[k] = yw[a] * xw[b];
            ++k;
        }
}

// ================================================================== SpMV ====
// Row blocks are dealt round-robin over the 8 XCDs; give every XCD a contiguous run of
// blocks instead, so the +-n stencil neighbours of a block's rows sit in the same L2.
// Placement changes speed only, never results.
__device__ inline int xcd_swizzle(int b, int nb) {
    const int full = nb & ~7;
    if (b >= full) return b;
    const int per = full >> 3;
    return (b & 7) * per + (b >> 3);
}

// Epilogues.  pre(r) issues the row's operand loads at kernel start (they overlap the matrix
// stream); operator() finishes the row once its sum is known.
struct EpiStore {
    double* y;
    struct P {};
    __device__ P pre(int32_t) const { return {}; }
    __device__ P pre_lite(int32_t) const { return {}; }
    template <bool NT = false>
    __device__ void apply(int32_t r, double acc, const P&) const { st_stream<NT>(y + r, acc); }
    __device__ void operator()(int32_t r, double acc, const P& p) const { apply<false>(r, acc, p); }
};
struct EpiAdd {   // rhs = D Finv_v + v_p   (solve.py:259)
    const double* z;
    double* y;
    struct P { double z; };
    __device__ P pre(int32_t r) const { return {ld_stream(z + r)}; }
    __device__ P pre_lite(int32_t r) const { return {ld_stream(z + r)}; }
    template <bool NT = false>
    __device__ void apply(int32_t r, double acc, const P& p) const { st_stream<NT>(y + r, acc + p.z); }
    __device__ void operator()(int32_t r, double acc, const P& p) const { apply<false>(r, acc, p); }
};
// The pressure solves' right-hand sides, written with the first Gt_G sweep's staged iterate beside them:
// y = rhs and x0 = c2 (rhs / diag) -- the value that sweep would otherwise recompute at each staged point (XInit),
// so the sweep stages x0 from memory (same bits).  EpiAddX0: rhs = D Finv_v + v_p (solve.py:259); EpiStoreX0:
// x_b = Gt_F_G x_a (solve.py:267).
struct EpiAddX0 {
    const double* z;
    double* y;
    const double* diag;
    double c2;
    double* x0;
    struct P { double z, pdiag; };
    __device__ P pre(int32_t r) const { return {ld_stream(z + r), diag[r]}; }
    __device__ P pre_lite(int32_t r) const { return pre(r); }
    template <bool NT = false>
    __device__ void apply(int32_t r, double acc, const P& p) const {
        const double v = acc + p.z;
        st_stream<NT>(y + r, v);
        st_stream<NT>(x0 + r, c2 * (v / p.pdiag));
    }
    __device__ void operator()(int32_t r, double acc, const P& p) const { apply<false>(r, acc, p); }
};
struct EpiStoreX0 {
    double* y;
    const double* diag;
    double c2;
    double* x0;
    struct P { double pdiag; };
    __device__ P pre(int32_t r) const { return {diag[r]}; }
    __device__ P pre_lite(int32_t r) const { return pre(r); }
    template <bool NT = false>
    __device__ void apply(int32_t r, double acc, const P& p) const {
        st_stream<NT>(y + r, acc);
        st_stream<NT>(x0 + r, c2 * (acc / p.pdiag));
    }
    __device__ void operator()(int32_t r, double acc, const P& p) const { apply<false>(r, acc, p); }
};
struct EpiResid {
    const double* z;
    double* y;
    struct P { double z; };
    __device__ P pre(int32_t r) const { return {ld_stream(z + r)}; }
    __device__ P pre_lite(int32_t r) const { return {ld_stream(z + r)}; }
    template <bool NT = false>
    __device__ void apply(int32_t r, double acc, const P& p) const { st_stream<NT>(y + r, p.z - acc); }
    __device__ void operator()(int32_t r, double acc, const P& p) const { apply<false>(r, acc, p); }
};
// The solver epilogues carry two run-time switches -- `sub` (the solve's last sweep returns sub - x) and
// `store_d` (the direction is stored except on a solve's last sweep).  The marching kernels get them as
// template flags instead (FIXED = true; launch_march picks the instance): no load or store then sits under
// a branch (the compiler's wait counts stay exact) and the unused operand costs no registers.
// RCP (tolerance-mode F policy only, FStencilFast): the diagonal handed over by set_diag is its reciprocal, so the
// update multiplies instead of dividing.
template <bool FIXED = false, bool SUB = true, bool RCP = false>
struct EpiJacobiT {   // x = (b - R x)/D in residual form (solve.py:158)
    const double* xin;
    const double* b;
    const double* diag;
    const double* sub;
    double* xout;
    struct P { double x, b, dg, s; };
    __device__ bool has_sub() const { return FIXED ? SUB : sub != nullptr; }
    __device__ P pre(int32_t r) const { return {xin[r], ld_stream(b + r), diag ? diag[r] : 0.0, sub ? ld_stream(sub + r) : 0.0}; }
    // x_in and diag supplied by the caller (set_x / set_diag)
    __device__ P pre_lite(int32_t r) const { return {0.0, ld_stream(b + r), 0.0, has_sub() ? ld_stream(sub + r) : 0.0}; }
    template <bool NT = false>
    __device__ void apply(int32_t r, double acc, const P& p) const {
        const double x = p.x + (RCP ? (p.b - acc) * p.dg : (p.b - acc) / p.dg);
        st_stream<NT>(xout + r, has_sub() ? p.s - x : x);
    }
    __device__ void operator()(int32_t r, double acc, const P& p) const { apply<false>(r, acc, p); }
};
// BX (FIXED instances of the marching kernels only): b is not loaded -- the kernel recomputes it per row and hands
// it over with set_b (the second F solve's right-hand side W = G x_p, solve.py:273-274, never stored).
template <bool FIXED = false, bool SUB = true, bool SD = true, bool BX = false, bool RCP = false>
struct EpiChebT {
    const double* xin;
    const double* b;
    const double* diag;
    double* d;
    double c1, c2;
    const double* sub;
    double* xout;
    int store_d = 1;   // 0: the inner solve's last sweep (its direction is never read again)
    struct P { double x, b, dg, d, s; };
    __device__ bool has_sub() const { return FIXED ? SUB : sub != nullptr; }
    __device__ bool stores_d() const { return FIXED ? SD : store_d != 0; }
    __device__ P pre(int32_t r) const { return {xin[r], ld_stream(b + r), diag ? diag[r] : 0.0, ld_stream(d + r), sub ? ld_stream(sub + r) : 0.0}; }
    // BX: `sub` is loaded in the epilogue itself instead of ahead of the row -- the fused
    // second solve's last sweep otherwise spills (128 VGPRs + 24 B scratch): 40.9 -> 38.9 us per launch
    // (2541-2565 -> 2573-2640 applies/s, A/B on one box)
    static constexpr bool kSubLate = BX, kBX = BX;
    __device__ P pre_lite(int32_t r) const { return {0.0, BX ? 0.0 : ld_stream(b + r), 0.0, ld_stream(d + r), (has_sub() && !kSubLate) ? ld_stream(sub + r) : 0.0}; }
    template <bool NT = false>
    __device__ void apply(int32_t r, double acc, const P& p) const {
        const double z = RCP ? (p.b - acc) * p.dg : (p.b - acc) / p.dg;
        const double dn = c1 * p.d + c2 * z;
        if (stores_d()) st_stream<NT>(d + r, dn);
        const double x = p.x + dn;
        const double sv = kSubLate && has_sub() ? ld_stream(sub + r) : p.s;
        st_stream<NT>(xout + r, has_sub() ? sv - x : x);
    }
    __device__ void operator()(int32_t r, double acc, const P& p) const { apply<false>(r, acc, p); }
};
// EpiCheb for the first sweep after x0 = d0 = c2[0] b / diag: the previous direction is the staged x0
// itself (x and diag supplied by the stencil via set_x / set_diag), so d is written but not read.
template <bool FIXED = false, bool SUB = true, bool SD = true, bool BX = false, bool RCP = false>
struct EpiChebFirstT {
    const double* b;
    double* d;
    double c1, c2;
    const double* sub;
    double* xout;
    int store_d = 1;
    struct P { double x, b, dg, s; };
    __device__ bool has_sub() const { return FIXED ? SUB : sub != nullptr; }
    __device__ bool stores_d() const { return FIXED ? SD : store_d != 0; }
    __device__ P pre(int32_t r) const { return {0.0, ld_stream(b + r), 0.0, sub ? ld_stream(sub + r) : 0.0}; }
    __device__ P pre_lite(int32_t r) const { return {0.0, BX ? 0.0 : ld_stream(b + r), 0.0, has_sub() ? ld_stream(sub + r) : 0.0}; }
    template <bool NT = false>
    __device__ void apply(int32_t r, double acc, const P& p) const {
        const double z = RCP ? (p.b - acc) * p.dg : (p.b - acc) / p.dg;
        const double dn = c1 * p.x + c2 * z;
        if (stores_d()) st_stream<NT>(d + r, dn);
        const double x = p.x + dn;
        st_stream<NT>(xout + r, has_sub() ? p.s - x : x);
    }
    __device__ void operator()(int32_t r, double acc, const P& p) const { apply<false>(r, acc, p); }
};
using EpiJacobi = EpiJacobiT<>;
using EpiCheb = EpiChebT<>;
using EpiChebFirst = EpiChebFirstT<>;

// Run fn with the epilogue's run-time switches turned into template flags (other epilogues unchanged).  RCP: the
// stencil hands over the reciprocal diagonal (FStencilFast), the solver epilogues multiply by it.
template <bool RCP = false, class Epi, class Fn>
__host__ inline int with_fixed_epi(const Epi& e, Fn&& fn) { return fn(e); }
template <bool RCP = false, class Fn>
__host__ inline int with_fixed_epi(const EpiJacobi& e, Fn&& fn) {
    return e.sub ? fn(EpiJacobiT<true, true, RCP>{e.xin, e.b, e.diag, e.sub, e.xout})
                 : fn(EpiJacobiT<true, false, RCP>{e.xin, e.b, e.diag, e.sub, e.xout});
}
template <bool RCP = false, class Fn>
__host__ inline int with_fixed_epi(const EpiCheb& e, Fn&& fn) {
#define MPBP_CHEB(SUB, SD) fn(EpiChebT<true, SUB, SD, false, RCP>{e.xin, e.b, e.diag, e.d, e.c1, e.c2, e.sub, e.xout, e.store_d})
    return e.sub ? (e.store_d ? MPBP_CHEB(true, true) : MPBP_CHEB(true, false))
                 : (e.store_d ? MPBP_CHEB(false, true) : MPBP_CHEB(false, false));
#undef MPBP_CHEB
}
template <bool RCP = false, class Fn>
__host__ inline int with_fixed_epi(const EpiChebFirst& e, Fn&& fn) {
#define MPBP_CHEBF(SUB, SD) fn(EpiChebFirstT<true, SUB, SD, false, RCP>{e.b, e.d, e.c1, e.c2, e.sub, e.xout, e.store_d})
    return e.sub ? (e.store_d ? MPBP_CHEBF(true, true) : MPBP_CHEBF(true, false))
                 : (e.store_d ? MPBP_CHEBF(false, true) : MPBP_CHEBF(false, false));
#undef MPBP_CHEBF
}

// The same, with b supplied by the kernel (BX): the F sweeps of the second F solve with W = G x_p recomputed.
template <bool RCP = false, class Epi, class Fn>
__host__ inline int with_fixed_epi_bx(const Epi& e, Fn&& fn) { return set_error(MPBP_ERR_ARG, "no BX epilogue"); }
template <bool RCP = false, class Fn>
__host__ inline int with_fixed_epi_bx(const EpiCheb& e, Fn&& fn) {
#define MPBP_CHEB(SUB, SD) fn(EpiChebT<true, SUB, SD, true, RCP>{e.xin, e.b, e.diag, e.d, e.c1, e.c2, e.sub, e.xout, e.store_d})
    return e.sub ? (e.store_d ? MPBP_CHEB(true, true) : MPBP_CHEB(true, false))
                 : (e.store_d ? MPBP_CHEB(false, true) : MPBP_CHEB(false, false));
#undef MPBP_CHEB
}
template <bool RCP = false, class Fn>
__host__ inline int with_fixed_epi_bx(const EpiChebFirst& e, Fn&& fn) {
#define MPBP_CHEBF(SUB, SD) fn(EpiChebFirstT<true, SUB, SD, true, RCP>{e.b, e.d, e.c1, e.c2, e.sub, e.xout, e.store_d})
    return e.sub ? (e.store_d ? MPBP_CHEBF(true, true) : MPBP_CHEBF(true, false))
                 : (e.store_d ? MPBP_CHEBF(false, true) : MPBP_CHEBF(false, false));
#undef MPBP_CHEBF
}

// Epilogues a tolerance-mode policy may feed: those that ignore the diagonal, and the RCP solver epilogues.
template <class E> struct RcpOk : std::false_type {};
template <> struct RcpOk<EpiStore> : std::true_type {};
template <> struct RcpOk<EpiAdd> : std::true_type {};
template <> struct RcpOk<EpiResid> : std::true_type {};
template <bool S> struct RcpOk<EpiJacobiT<true, S, true>> : std::true_type {};
template <bool S, bool D, bool B> struct RcpOk<EpiChebT<true, S, D, B, true>> : std::true_type {};
template <bool S, bool D, bool B> struct RcpOk<EpiChebFirstT<true, S, D, B, true>> : std::true_type {};

// XI entry xi * a * (1 - a) as the assembly evaluates it (left to right).
__device__ inline double xi_of(double xi, double a) { return xi * a * (1.0 - a); }

template <class PT>
__device__ inline void set_b(PT& p, double b) { p.b = b; }
template <class PT>
__device__ inline void set_diag(PT& p, double d) { p.dg = d; }
template <class PT>
__device__ inline void set_x(PT& p, double x) { p.x = x; }
template <>
__device__ inline void set_x<EpiStore::P>(EpiStore::P&, double) {}
template <>
__device__ inline void set_x<EpiAdd::P>(EpiAdd::P&, double) {}
template <>
__device__ inline void set_x<EpiResid::P>(EpiResid::P&, double) {}
template <>
__device__ inline void set_diag<EpiStore::P>(EpiStore::P&, double) {}
template <>
__device__ inline void set_diag<EpiAdd::P>(EpiAdd::P&, double) {}
template <>
__device__ inline void set_diag<EpiResid::P>(EpiResid::P&, double) {}
template <>
__device__ inline void set_x<EpiAddX0::P>(EpiAddX0::P&, double) {}
template <>
__device__ inline void set_diag<EpiAddX0::P>(EpiAddX0::P&, double) {}

// CSR SpMV over the same row blocks, one wavefront per 64-row quarter of a block and no block-wide
// barrier.  Each wave streams its rows' [row_ptr[ra], row_ptr[rb]) entries in chunks of kWaveCap with
// 16-byte loads (1 KiB of values per wave-instruction) and transposes the chunk through its own LDS
// (values and columns as pairs, 9 KiB); each lane then walks the part of its own row that lies in the
// chunk, gathers x for it and adds the products left to right, chunk after chunk -- the oracle's
// sequential order, so bit-exact.  Gathering per row (lane = row, as in SELL) makes one
// wave-instruction's x addresses the same stencil neighbour of 64 consecutive rows instead of all
// neighbours of ~10 rows: fewer cache lines per instruction (153 vs 172 us for the 1024^2 A).  A 1024^2
// A row block (12 entries per velocity row) is one chunk per wave.
// Measured dead end: no staging at all, each lane loading its own row (16-byte loads 96 B apart across
// the wave) -- 567 us, the texture addresser then touches ~48 cache lines per wave-instruction.
constexpr int kWaveCap = 768;                 // entries per wave chunk (64 rows x 12 entries)
constexpr int kWavePairs = kWaveCap / 128;     // 16-byte loads per lane per chunk
constexpr int kRowBatch = 8;                   // pairs of a row gathered at once (16 entries)

// A wave-uniform int32 element through a scalar (constant address space) load.
typedef __attribute__((address_space(4))) const int32_t cint32;
__device__ inline int32_t ld_uniform_i32(const int32_t* p, int32_t i) {
    return ((cint32*)p)[__builtin_amdgcn_readfirstlane(i)];
}

// Lanes of one wave exchange data through LDS: order the LDS writes before the reads (compiler
// and wave scope; a wave's LDS operations complete in order).
__device__ inline void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// A wave whose 64 rows all hold LEN entries (stencil operators: A's velocity rows 12, pressure rows 8,
// F's rows 10) from an even start: its entries are exactly one chunk, lane l's row is pairs
// [l*LEN/2, (l+1)*LEN/2) of it, so the loads, LDS transposition, gathers and sums unroll with no
// per-entry bounds tests.  Same additions in the same order as the general loop (bit-exact).
// XB: x gathered with buffer loads (one descriptor for x, a 32-bit byte offset per entry: no 64-bit
// address arithmetic per gather); needs ncols * 8 < 2^31.
// Returns false (nothing stored) when some row of the wave does not hold LEN entries.  The
// matrix loads are issued before that check -- they depend on the wave's first entry s alone (and stay inside
// [s, s + 64 LEN) = the wave's entries), so their HBM latency overlaps the per-row row_ptr loads' instead of
// following it.
// TRUST: the wave table says the wave is uniform (no row check).
// GL (table-trusted waves whose entry offset is a multiple of 4): the chunk is copied into LDS by LDS-DMA
// (global_load_lds_dwordx4, nontemporal) instead of through VGPRs -- the same lane-linear image, no staging registers
// or LDS stores: 137.0-137.3 vs 138.8-141.8 us for the 1024^2 A on one box (tools/spmv_lab.py, r05h).
__device__ inline void glds16(const void* g, void* lds) {
    __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds, 16, 0, 2);
}
template <int LEN, bool XB, class Epi, bool TRUST = false, bool GL = false>
__device__ inline bool csr_wave_uniform(const Csr& A, const double* __restrict__ x, int32_t s, int lane,
                                        double2* vs, int2* cs, int32_t ks, int32_t ke, int32_t r, const Epi& epi,
                                        const typename Epi::P& pe) {
    constexpr int P = LEN / 2;   // pairs per row == 16-byte loads per lane
    if constexpr (GL) {
        static_assert(TRUST, "LDS-DMA staging only for table-trusted waves");
        // values: P instructions of 64 x 16 B; columns: LEN / 4 whole instructions and, for LEN = 10, half of one
#pragma unroll
        for (int j = 0; j < P; ++j) glds16(A.va + s + 2 * (lane + 64 * j), vs + 64 * j);
#pragma unroll
        for (int j = 0; j < LEN / 4; ++j) glds16(A.ci + s + 4 * (lane + 64 * j), cs + 128 * j);
        if constexpr (LEN % 4 != 0) {
            if (lane < 32) glds16(A.ci + s + 4 * (lane + 64 * (LEN / 4)), cs + 128 * (LEN / 4));
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        double2 v[P];
        int2 cc[P];
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int32_t k = s + 2 * (lane + 64 * j);
            v[j] = ld_matrix<kCsrNT>(reinterpret_cast<const double2*>(A.va + k));
            cc[j] = ld_matrix<kCsrNT>(reinterpret_cast<const int2*>(A.ci + k));
        }
        // (a compiler memory barrier: the loads above may not sink below the check, which would serialise them
        // behind the row_ptr loads again; it emits no instruction and no wait)
        asm volatile("" ::: "memory");
        if (!TRUST && !__all(ke - ks == LEN)) return false;
#pragma unroll
        for (int j = 0; j < P; ++j) {
            vs[lane + 64 * j] = v[j];
            cs[lane + 64 * j] = cc[j];
        }
    }
    wave_lds_sync();
    const int p0 = lane * P;
    int2 c[P];
#pragma unroll
    for (int i = 0; i < P; ++i) c[i] = cs[p0 + i];
    double x0[P], x1[P];
    if constexpr (XB) {
        const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(x), (short)0, A.ncols * 8, 0x00020000);
#pragma unroll
        for (int i = 0; i < P; ++i) {
            x0[i] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, c[i].x * 8, 0, 0));
            x1[i] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, c[i].y * 8, 0, 0));
        }
    } else {
#pragma unroll
        for (int i = 0; i < P; ++i) {
            x0[i] = x[c[i].x];
            x1[i] = x[c[i].y];
        }
    }
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < P; ++i) {
        const double2 q = vs[p0 + i];
        acc += q.x * x0[i];
        acc += q.y * x1[i];
    }
    epi.template apply<kCsrNT>(r, acc, pe);   // every lane holds a row here
    return true;
}

// The wave table (mpbp_rowblocks.table; mpbp_set_csr_table(0) ignores it): a wave flagged uniform starts its matrix loads
// right after one scalar load of its block's 32-byte table entry -- no dependent row-range load, no row_ptr reads.
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(4))) const i32x4 ci32x4;
template <class Epi>
__global__ void __launch_bounds__(kBlock) k_csr_wave(Csr A, const double* __restrict__ x,
                                                     const int2* __restrict__ blocks, int nblocks,
                                                     const int32_t* __restrict__ table, Epi epi) {
    __shared__ double2 vstage[kBlock / 64][kWaveCap / 2];
    __shared__ int2 cstage[kBlock / 64][kWaveCap / 2];
    const int b = xcd_swizzle(blockIdx.x, nblocks);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (table && A.ncols > 0 && A.ncols < (1 << 28)) {
        const i32x4 t0 = ((ci32x4*)table)[2 * b], t1 = ((ci32x4*)table)[2 * b + 1];
        const int32_t ra = t0.x + 64 * w;
        if (ra >= t0.y) return;
        const int len = (t1.w >> (8 * w)) & 255;
        if (len) {
            const int32_t s = w == 0 ? t0.z : w == 1 ? t0.w : w == 2 ? t1.x : t1.y;
            const int32_t r = ra + lane;
            const typename Epi::P pe = epi.pre(r);
            constexpr bool XB = true;
            if ((s & 3) == 0) {   // 16-byte aligned column chunk: LDS-DMA staging
                if (len == 12) csr_wave_uniform<12, XB, Epi, true, true>(A, x, s, lane, vstage[w], cstage[w], 0, 0, r, epi, pe);
                else if (len == 10) csr_wave_uniform<10, XB, Epi, true, true>(A, x, s, lane, vstage[w], cstage[w], 0, 0, r, epi, pe);
                else csr_wave_uniform<8, XB, Epi, true, true>(A, x, s, lane, vstage[w], cstage[w], 0, 0, r, epi, pe);
                return;
            }
            if (len == 12) csr_wave_uniform<12, XB, Epi, true>(A, x, s, lane, vstage[w], cstage[w], 0, 0, r, epi, pe);
            else if (len == 10) csr_wave_uniform<10, XB, Epi, true>(A, x, s, lane, vstage[w], cstage[w], 0, 0, r, epi, pe);
            else csr_wave_uniform<8, XB, Epi, true>(A, x, s, lane, vstage[w], cstage[w], 0, 0, r, epi, pe);
            return;
        }
    }
    const int2 blk = blocks[b];
    const int32_t ra = __builtin_amdgcn_readfirstlane(blk.x + 64 * w);
    if (ra >= blk.y) return;   // waves are independent: no workgroup barrier below
    const int32_t rb = min(ra + 64, blk.y);
    const int32_t r = ra + lane;
    const bool live = r < rb;
    // the wave's entry range through scalar loads (their own counter: the matrix loads of the uniform path wait for
    // them alone), the rows' bounds through unconditional vector loads (lanes past the block re-read row ra)
    const int32_t s = ld_uniform_i32(A.rp, ra), e = ld_uniform_i32(A.rp, rb);
    const int32_t rr = live ? r : ra;
    const int32_t ks = A.rp[rr], ke0 = A.rp[rr + 1];
    const int32_t ke = live ? ke0 : ks;   // (an empty row for lanes past the block)
    typename Epi::P pe{};
    if (live) pe = epi.pre(r);
    double acc = 0.0;
    double2* vs = vstage[w];
    const double* vs1 = reinterpret_cast<const double*>(vs);
    {
        const int32_t len = (e - s) >> 6;   // wave-uniform
        if (rb - ra == 64 && ((e - s) & 63) == 0 && (s & 1) == 0 && (len == 8 || len == 10 || len == 12)) {
            constexpr bool XB = true;
            bool done;
            if (XB && A.ncols > 0 && A.ncols < (1 << 28))
                done = len == 12 ? csr_wave_uniform<12, XB>(A, x, s, lane, vs, cstage[w], ks, ke, r, epi, pe)
                                 : (len == 10 ? csr_wave_uniform<10, XB>(A, x, s, lane, vs, cstage[w], ks, ke, r, epi, pe)
                                              : csr_wave_uniform<8, XB>(A, x, s, lane, vs, cstage[w], ks, ke, r, epi, pe));
            else
                done = len == 12 ? csr_wave_uniform<12, false>(A, x, s, lane, vs, cstage[w], ks, ke, r, epi, pe)
                                 : (len == 10 ? csr_wave_uniform<10, false>(A, x, s, lane, vs, cstage[w], ks, ke, r, epi, pe)
                                              : csr_wave_uniform<8, false>(A, x, s, lane, vs, cstage[w], ks, ke, r, epi, pe));
            if (done) return;
        }
    }
    for (int32_t cb = s & ~1; cb < e; cb += kWaveCap) {
        double2 v[kWavePairs];
        int2 cc[kWavePairs];
#pragma unroll
        for (int j = 0; j < kWavePairs; ++j) {
            const int32_t k = cb + 2 * (lane + 64 * j);
            if (k + 1 < e) {
                v[j] = ld_matrix<kCsrNT>(reinterpret_cast<const double2*>(A.va + k));
                cc[j] = ld_matrix<kCsrNT>(reinterpret_cast<const int2*>(A.ci + k));
            } else if (k < e) {
                v[j] = make_double2(A.va[k], 0.0);
                cc[j] = make_int2(A.ci[k], 0);
            } else {
                v[j] = make_double2(0.0, 0.0);
                cc[j] = make_int2(0, 0);
            }
        }
        int32_t t = max(ks, cb) - cb;                       // this lane's row within the chunk
        const int32_t tend = min(ke, cb + kWaveCap) - cb;
        if (cb != (s & ~1)) wave_lds_sync();   // the previous chunk's reads are done
        int2* cs = cstage[w];
        const int32_t* cs1 = reinterpret_cast<const int32_t*>(cs);
#pragma unroll
        for (int j = 0; j < kWavePairs; ++j) {
            vs[lane + 64 * j] = v[j];
            cs[lane + 64 * j] = cc[j];
        }
        wave_lds_sync();
        if ((t & 1) && t < tend) {   // odd start: one entry, then whole pairs
            acc += vs1[t] * x[cs1[t]];
            ++t;
        }
        for (; t < tend; t += 2 * kRowBatch) {
            const int32_t p0 = t >> 1;
            int2 c[kRowBatch];
            double x0[kRowBatch], x1[kRowBatch];
#pragma unroll
            for (int i = 0; i < kRowBatch; ++i) c[i] = (t + 2 * i < tend) ? cs[p0 + i] : make_int2(0, 0);
#pragma unroll
            for (int i = 0; i < kRowBatch; ++i) {
                x0[i] = (t + 2 * i < tend) ? x[c[i].x] : 0.0;
                x1[i] = (t + 2 * i + 1 < tend) ? x[c[i].y] : 0.0;
            }
#pragma unroll
            for (int i = 0; i < kRowBatch; ++i) {
                if (t + 2 * i < tend) {
                    const double2 q = vs[p0 + i];
                    acc += q.x * x0[i];
                    if (t + 2 * i + 1 < tend) acc += q.y * x1[i];
                }
            }
        }
    }
    if (live) epi.template apply<kCsrNT>(r, acc, pe);
}

// ---------------------------------------------------- HBM calibration (measurement only) ----
// The bench's same-run reference rates for the CSR SpMV roofline (mpbp_hbm_stream): mode 0 reads `bytes` once in order
// (16 B per lane, nontemporal, 16 KiB per workgroup); mode 1 the SpMV's own stream shape without its x gathers -- per
// 64-lane wave 9 KiB read in order and 64 doubles written (nontemporal), as a wave of 64 twelve-entry rows moves.
__global__ void __launch_bounds__(kBlock) k_hbm_read(const f64x2* __restrict__ p, int64_t n16, double* sink) {
    const int64_t base = (int64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 1024 + threadIdx.x;
    f64x2 acc = {0.0, 0.0};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int64_t i = base + 256 * j;
        if (i < n16) acc += __builtin_nontemporal_load(p + i);
    }
    if (acc.x == 1234.5678 && acc.y == -8765.4321) sink[threadIdx.x] = acc.x;   // keeps the loads; never taken on data
}
__global__ void __launch_bounds__(kBlock) k_hbm_readwrite(const f64x2* __restrict__ p, int64_t nwaves, double* y) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t wv = (int64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 4 + w;
    if (wv >= nwaves) return;
    const f64x2* q = p + wv * 576;
    f64x2 acc = {0.0, 0.0};
#pragma unroll
    for (int j = 0; j < 9; ++j) acc += __builtin_nontemporal_load(q + lane + 64 * j);
    __builtin_nontemporal_store(acc.x + acc.y, y + wv * 64 + lane);
}

// ---------------------------------------------------- CSR, segmented reduction ----
// The same product under north_star's value bar instead of the oracle's order: identical row_ptr / col_idx
// handling, row sums within 1e-12 (relative infinity norm) of the sequential ones (np.matmul's BLAS sums are
// not sequential either, apply.py:72).  A uniform wave (64 rows of LEN = 2P entries from an even start, as in
// k_csr_wave) needs no LDS transposition: each row's P entry pairs sit in P consecutive lanes of a G-lane group
// (G = 4 for P = 4, else 8; lanes P..G-1 of a group repeat the group's last pair and add 0), a wave-instruction
// covers 64/G whole rows (contiguous 16-byte loads), every lane multiplies its own pair (x gathered by its own
// columns), and the group sums its pairs by DPP cross-lane adds (half-row mirror, then the two quad swaps; every
// lane of the group ends with the same bits, commutativity).  The row sums then go through 512 B of LDS so the
// epilogue runs one row per lane.  LDS 2 KiB per workgroup instead of 36 KiB: occupancy is set by registers.
// Non-uniform waves take a plain lane-per-row loop (correct, not fast: tree order is for stencil operators).
template <int CTRL>
__device__ inline double dpp_f64(double v) {
    const int2 h = __builtin_bit_cast(int2, v);
    const int lo = __builtin_amdgcn_update_dpp(0, h.x, CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, h.y, CTRL, 0xf, 0xf, false);
    return __builtin_bit_cast(double, make_int2(lo, hi));
}
constexpr int kDppQuadSwap2 = 0x4e;      // quad_perm [2,3,0,1]
constexpr int kDppQuadSwap1 = 0xb1;      // quad_perm [1,0,3,2]
constexpr int kDppHalfMirror = 0x141;    // row_half_mirror: lane k <- lane 7-k within 8

template <int LEN, class Epi>
__device__ inline bool csr_seg_uniform(const Csr& A, const double* __restrict__ x, int32_t s, int lane,
                                       double* ys, int32_t ks, int32_t ke, int32_t r, const Epi& epi,
                                       const typename Epi::P& pe) {
    constexpr int P = LEN / 2;               // entry pairs per row
    constexpr int G = P <= 4 ? 4 : 8;        // lanes per row group
    constexpr int RPI = 64 / G;              // rows per wave-instruction
    constexpr int NI = 64 / RPI;             // wave-instructions for the wave's 64 rows
    const int k = lane % G, rg = lane / G;
    const int kc = k < P ? k : P - 1;        // idle lanes re-read the group's last pair (same cache line)
    double2 v[NI];
    int2 c[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) {
        const int32_t q = s + 2 * ((j * RPI + rg) * P + kc);
        v[j] = ld_matrix<kCsrNT>(reinterpret_cast<const double2*>(A.va + q));
        c[j] = ld_matrix<kCsrNT>(reinterpret_cast<const int2*>(A.ci + q));
    }
    asm volatile("" ::: "memory");           // keep the matrix loads ahead of the row check (as csr_wave_uniform)
    if (!__all(ke - ks == LEN)) return false;
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(x), (short)0, A.ncols * 8, 0x00020000);
    double t[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) {
        const double x0 = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, c[j].x * 8, 0, 0));
        const double x1 = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, c[j].y * 8, 0, 0));
        // (a bit mask, not a branch: the gathers of idle lanes stay unconditional, so they issue back to back)
        const uint64_t keep = k < P ? ~0ull : 0ull;
        t[j] = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, __builtin_fma(v[j].y, x1, v[j].x * x0)) & keep);
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
        if constexpr (G == 8) t[j] += dpp_f64<kDppHalfMirror>(t[j]);
        t[j] += dpp_f64<kDppQuadSwap2>(t[j]);
        t[j] += dpp_f64<kDppQuadSwap1>(t[j]);
        if (k == 0) ys[j * RPI + rg] = t[j];
    }
    wave_lds_sync();
    epi.template apply<kCsrNT>(r, ys[lane], pe);
    return true;
}

template <class Epi>
__global__ void __launch_bounds__(kBlock) k_csr_seg(Csr A, const double* __restrict__ x,
                                                    const int2* __restrict__ blocks, int nblocks, Epi epi) {
    __shared__ double ystage[kBlock / 64][64];
    const int b = xcd_swizzle(blockIdx.x, nblocks);
    const int2 blk = blocks[b];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int32_t ra = __builtin_amdgcn_readfirstlane(blk.x + 64 * w);
    if (ra >= blk.y) return;
    const int32_t rb = min(ra + 64, blk.y);
    const int32_t r = ra + lane;
    const bool live = r < rb;
    const int32_t s = ld_uniform_i32(A.rp, ra), e = ld_uniform_i32(A.rp, rb);
    const int32_t rr = live ? r : ra;
    const int32_t ks = A.rp[rr], ke0 = A.rp[rr + 1];
    const int32_t ke = live ? ke0 : ks;
    typename Epi::P pe{};
    if (live) pe = epi.pre(r);
    const int32_t len = (e - s) >> 6;
    if (rb - ra == 64 && ((e - s) & 63) == 0 && (s & 1) == 0 && A.ncols > 0 && A.ncols < (1 << 28)) {
        // every lane is live here: the raw row end ke0, so no select on it waits for the row_ptr loads before
        // the matrix loads issue
        bool done = false;
        if (len == 12) done = csr_seg_uniform<12>(A, x, s, lane, ystage[w], ks, ke0, r, epi, pe);
        else if (len == 10) done = csr_seg_uniform<10>(A, x, s, lane, ystage[w], ks, ke0, r, epi, pe);
        else if (len == 8) done = csr_seg_uniform<8>(A, x, s, lane, ystage[w], ks, ke0, r, epi, pe);
        if (done) return;
    }
    double acc = 0.0;
    for (int32_t kk = ks; kk < ke; ++kk) acc += A.va[kk] * x[A.ci[kk]];
    if (live) epi.template apply<kCsrNT>(r, acc, pe);
}

// ---------------------------------------------- CSR, G lanes per row (small levels) ----
// The multigrid's small levels (<= 64^2 cells per field: 1-16 K rows of 20-46 entries) are latency-bound, not
// bandwidth-bound: one lane per row walks its row in batches, each batch a matrix load -> x gather chain, so a
// 4 K-row sweep took ~9 us for 2 MB.  Here G lanes share a row: each loads J of its entries (entries k, k + G, ...;
// all loads of the row in flight at once), gathers x and forms the products v * x in parallel, writes them to
// LDS, and the group's first lane adds them left to right from 0.0 -- the CSR row's sequential sum, bit for bit
// (same products, same order, no FMA).  One latency chain per row instead of one per batch, and G times the lanes
// for the few rows.  Rows longer than G * J entries take several chunks (correct for any CSR).  A DZ epilogue
// reads the Chebyshev direction as +0.0 without loading it (the smoother's restart after a coarse correction,
// same IEEE operations as a zeroed vector: no memset launch).
constexpr int kGrpJ = 8;   // entries per lane per chunk
template <class Epi>
struct EpiZeroD : Epi {   // Epi = EpiCheb: d read as +0.0 (never loaded)
    using P = typename Epi::P;
    __device__ P pre(int32_t r) const {
        return {this->xin[r], ld_stream(this->b + r), this->diag ? this->diag[r] : 0.0, 0.0,
                this->sub ? ld_stream(this->sub + r) : 0.0};
    }
    // the stencil kernels' form (x and the diagonal from the stencil itself)
    __device__ P pre_lite(int32_t r) const {
        return {0.0, Epi::kBX ? 0.0 : ld_stream(this->b + r), 0.0, 0.0,
                (this->has_sub() && !Epi::kSubLate) ? ld_stream(this->sub + r) : 0.0};
    }
};
// The first Chebyshev sweep from x = 0 with the init pass folded in (XS = XInit gathers x0 = c2_0 (b / diag) at every
// column, the same expression k_cheb_init stores): the epilogue's x and direction are the row's own x0.
struct EpiChebFirstGrp : EpiChebFirst {
    const double* diag;
    double c2_0;
    __device__ P pre(int32_t r) const {
        P p = EpiChebFirst::pre(r);
        p.dg = diag[r];
        p.x = c2_0 * (p.b / p.dg);
        return p;
    }
};
template <int G, class XS, class Epi>
__global__ void __launch_bounds__(kBlock) k_csr_grp(Csr A, int32_t nrows, XS xs, Epi epi) {
    constexpr int RPB = kBlock / G, CAP = G * kGrpJ;
    __shared__ double prod[RPB * CAP];
    const int g = threadIdx.x / G, k = threadIdx.x % G;
    const int32_t r = xcd_swizzle(blockIdx.x, gridDim.x) * RPB + g;
    const bool live = r < nrows;
    const int32_t rr = live ? r : nrows - 1;
    const int32_t ks = A.rp[rr], ke = live ? A.rp[rr + 1] : ks;
    typename Epi::P pe{};
    if (live && k == 0) pe = epi.pre(r);
    double* pr = prod + g * CAP;
    double acc = 0.0;
    for (int32_t cb = ks; cb < ke; cb += CAP) {
        double v[kGrpJ];
        int32_t c[kGrpJ];
#pragma unroll
        for (int j = 0; j < kGrpJ; ++j) {
            const int32_t e = cb + k + G * j;
            const bool in = e < ke;
            v[j] = in ? A.va[e] : 0.0;
            c[j] = in ? A.ci[e] : 0;
        }
        double p[kGrpJ];
#pragma unroll
        for (int j = 0; j < kGrpJ; ++j) p[j] = v[j] * xs(c[j]);
        if (cb != ks) wave_lds_sync();   // the previous chunk's sums have read their slots
#pragma unroll
        for (int j = 0; j < kGrpJ; ++j) pr[k + G * j] = p[j];
        wave_lds_sync();                 // a group never spans two waves (G divides 64)
        if (k == 0) {
            const int32_t cnt = min(ke - cb, (int32_t)CAP);
            for (int32_t i = 0; i < cnt; ++i) acc += pr[i];
        }
    }
    if (live && k == 0) epi(r, acc, pe);
}

// ------------------------------------------------------------ stencil-values layout ----
// The multigrid's large Galerkin levels (F level 1 at 1024^2: 1 M rows x 40 entries) stream 12 B per entry on SELL;
// their rows all hold the same (field, dr, dc) offsets (translation-invariant operator on a periodic grid), so the
// column indices are rebuilt as row + delta[f][s] and only the values are streamed, slot-major (coalesced per slot
// across consecutive rows, nontemporal).  One thread per interior row (threads enumerate the interior cells of
// every field densely, so no wave mixes the two paths): K products in slot order = the CSR row's column order;
// the x gathers need no column load, so they issue beside the value loads.  Then one thread per edge row (within
// `reach` of the periodic edge, where the wrapped columns sort differently): the CSR row, left to right.  Both the
// CSR SpMV's additions exactly (bit-identical), at 8 B instead of 12 B per entry for all but the edge rows.
struct Svl {
    int nf, m, R, K;
    const int32_t* delta;
    const double* vals;
    const int32_t* edge;
    int n_edge;
};
constexpr int kSvB = 8;  // slots per batch (values + gathers in flight together)

constexpr int kSvMaxDelta = 256;     // nf * K
constexpr int kSvEdgeG = 8;          // lanes per edge row (k_csr_grp's scheme: one latency chain per row)
template <class XS, class Epi>
__global__ void __launch_bounds__(kBlock) k_svl(Svl V, Csr A, int32_t nrows, XS xs, Epi epi) {
    __shared__ int32_t sdelta[kSvMaxDelta];
    __shared__ double prod[kBlock * kGrpJ];
    for (int i = threadIdx.x; i < V.nf * V.K; i += kBlock) sdelta[i] = V.delta[i];
    __syncthreads();
    // interior: one thread per pair of horizontally adjacent cells (reach is even, so W = m - 2 reach is even and a
    // pair starts on an even row id): 16-byte value loads, two rows' products, two ordered sums
    const int W = V.m - 2 * V.R;
    const int W2 = W >> 1;
    const int32_t per = W2 * W;                        // pairs per field
    const int32_t ni = V.nf * per;
    // the edge rows' latency-bound CSR chains in the first-dispatched workgroups (round-robin over the XCDs), the
    // interior pairs behind them (XCD-contiguous runs): otherwise the edge chains start last, behind the stream
    // (multigrid apply 1.767 -> 1.731 ms, A/B on one box)
    const int32_t nb_edge = (V.n_edge * kSvEdgeG + kBlock - 1) / kBlock;
    const bool eb = (int32_t)blockIdx.x < nb_edge;
    const int32_t t0 = (int32_t)blockIdx.x * kBlock + (int32_t)threadIdx.x;
    const int32_t t = eb ? ni : (int32_t)xcd_swizzle(blockIdx.x - nb_edge, gridDim.x - nb_edge) * kBlock + (int32_t)threadIdx.x;
    const bool edge_ok = eb && t0 < V.n_edge * kSvEdgeG;
    if (t < ni) {
        const uint32_t f = (uint32_t)t / (uint32_t)per;
        const uint32_t i = (uint32_t)t - f * (uint32_t)per;
        const uint32_t q = i / (uint32_t)W2;
        const int r = V.R + (int)q, c = V.R + 2 * (int)(i - q * (uint32_t)W2);
        const int32_t row = ((int32_t)f * V.m + r) * V.m + c;
        const typename Epi::P pe0 = epi.pre(row), pe1 = epi.pre(row + 1);
        const int32_t* dl = sdelta + f * V.K;
        const double* vp = V.vals + row;
        double a0 = 0.0, a1 = 0.0;
        for (int s0 = 0; s0 < V.K; s0 += kSvB) {
            f64x2 v[kSvB];
            double x0[kSvB], x1[kSvB];
#pragma unroll
            for (int j = 0; j < kSvB; ++j) {
                const int sj = min(s0 + j, V.K - 1);   // (a tail batch re-reads the last slot and discards it)
                v[j] = __builtin_nontemporal_load(reinterpret_cast<const f64x2*>(vp + (int64_t)sj * nrows));
                const int32_t col = row + dl[sj];
                x0[j] = xs(col);
                x1[j] = xs(col + 1);
            }
#pragma unroll
            for (int j = 0; j < kSvB; ++j)
                if (s0 + j < V.K) {
                    a0 += v[j].x * x0[j];
                    a1 += v[j].y * x1[j];
                }
        }
        epi(row, a0, pe0);
        epi(row + 1, a1, pe1);
    } else if (edge_ok) {
        const int64_t u = t0;
        // edge row: kSvEdgeG lanes load its CSR entries at once and form the products, the first lane sums them in
        // order (k_csr_grp)
        constexpr int G = kSvEdgeG, CAP = G * kGrpJ;
        const int32_t row = V.edge[u / G];
        const int k = (int)(u % G);
        double* pr = prod + (threadIdx.x / G) * CAP;
        typename Epi::P pe{};
        if (k == 0) pe = epi.pre(row);
        const int32_t ks = A.rp[row], ke = A.rp[row + 1];
        double acc = 0.0;
        for (int32_t cb = ks; cb < ke; cb += CAP) {
            double p[kGrpJ];
#pragma unroll
            for (int j = 0; j < kGrpJ; ++j) {
                const int32_t e = cb + k + G * j;
                const bool in = e < ke;
                p[j] = (in ? A.va[e] : 0.0) * xs(in ? A.ci[e] : row);
            }
            if (cb != ks) wave_lds_sync();
#pragma unroll
            for (int j = 0; j < kGrpJ; ++j) pr[k + G * j] = p[j];
            wave_lds_sync();
            if (k == 0) {
                const int32_t cnt = min(ke - cb, (int32_t)CAP);
                for (int32_t i = 0; i < cnt; ++i) acc += pr[i];
            }
        }
        if (k == 0) epi(row, acc, pe);
    }
}

// ------------------------------------------------------------------ SELL-64 ----
// Sliced ELLPACK with one wavefront per slice: a slice is <= 64 consecutive rows, its entries
// stored column-major in pairs -- pair-row j of the slice holds entries (2j, 2j+1) of every row,
// one double2 / int2 per lane -- so each wave-instruction reads 1 KiB of values and 512 B of
// column indices contiguously, and each lane owns one row: no LDS, no barrier, no reduction
// across lanes.  Entries keep their CSR order, so row sums stay bit-exact with the oracle.
// slices[s] = {row0, rows, width, first pair-row}; row_len[r] = CSR length of row r (< 256).
struct Sell {
    const int4* slices;
    const uint8_t* rlen;
    const double2* val;
    const int2* col;
};

constexpr int kSellPairs = 8;   // rows of up to 16 entries take the fully unrolled path

template <class Epi>
__global__ void __launch_bounds__(kBlock) k_sell_rows(Sell S, const double* __restrict__ x, int nslices,
                                                      Epi epi) {
    const int b = xcd_swizzle(blockIdx.x, gridDim.x);
    const int sidx = b * (kBlock / 64) + (int)(threadIdx.x >> 6);
    if (sidx >= nslices) return;
    const int lane = threadIdx.x & 63;
    const int4 sl = S.slices[sidx];
    const int32_t r = sl.x + lane;
    const bool live = lane < sl.y;
    const int len = live ? (int)S.rlen[r] : 0;
    typename Epi::P pe{};
    if (live) pe = epi.pre(r);
    const int np = (sl.z + 1) >> 1;
    const double2* vp = S.val + (size_t)sl.w * 64 + lane;
    const int2* cp = S.col + (size_t)sl.w * 64 + lane;
    double acc = 0.0;
    // pair-rows [j0, j0 + kSellPairs): every load of the batch first (slice padding is zero, so loads past a
    // row's end are harmless), then the x gathers, then the products added in CSR order.  Rows of up to 16
    // entries take one batch; longer ones (multigrid coarse operators: 20-50 entries) loop over batches.
    auto batch = [&](int j0) {
        double2 v[kSellPairs];
        int2 c[kSellPairs];
#pragma unroll
        for (int j = 0; j < kSellPairs; ++j) {
            if (j0 + j < np) {   // wave-uniform
                v[j] = ld_matrix<kSellNT>(vp + (size_t)(j0 + j) * 64);
                c[j] = ld_matrix<kSellNT>(cp + (size_t)(j0 + j) * 64);
            } else {
                v[j] = make_double2(0.0, 0.0);
                c[j] = make_int2(0, 0);
            }
        }
        double x0[kSellPairs], x1[kSellPairs];
#pragma unroll
        for (int j = 0; j < kSellPairs; ++j) {
            x0[j] = (2 * (j0 + j) < len) ? x[c[j].x] : 0.0;
            x1[j] = (2 * (j0 + j) + 1 < len) ? x[c[j].y] : 0.0;
        }
#pragma unroll
        for (int j = 0; j < kSellPairs; ++j) {
            if (2 * (j0 + j) < len) acc += v[j].x * x0[j];
            if (2 * (j0 + j) + 1 < len) acc += v[j].y * x1[j];
        }
    };
    if (np <= kSellPairs) {
        batch(0);
    } else {
        for (int j0 = 0; j0 < np; j0 += kSellPairs) batch(j0);
    }
    if (live) epi.template apply<kSellNT>(r, acc, pe);
}

// ------------------------------------------------------------- F stencil ----
// Matrix-free rows of F = XI + d_u blockdiag(eta_n L_n, eta_s L_s): the ten entries of a row are
// recomputed from the thn tables (L1/L2-resident) with exactly the assembly's arithmetic
// (phase_L_row / F_row above) and their products summed in the assembled row's column order -- the same
// IEEE operations as a sweep over the assembled F, without streaming its 12 bytes x 10 entries per row
// from HBM.  Needs n >= 3 (no coinciding periodic neighbours).
//
// Column order on the periodic edge.  A stencil's products are listed in the interior's sorted-column order;
// on the grid's edge a wrapped neighbour moves (row -1 -> n-1 sorts last, row n -> 0 first, and likewise for
// columns).  Instead of sorting, the edge form adds every product at each position it can occupy, with the
// positions it does not occupy on this lane contributing -0.0 -- the exact identity of IEEE addition in
// round-to-nearest (x + -0.0 == x for every x, signed zeros included) -- so the sum performs exactly the
// sorted row's additions, with no sorting network and the same code on every lane.
struct Wrap {
    bool r0, rl, c0, cl;   // the cell's grid row is 0 / n-1, its column 0 / n-1
};
__device__ inline double opt(bool c, double p) { return c ? p : -0.0; }
// Five-point products p = {N, W, C, E, S} (interior column order), added to acc in the row's column order.
template <bool EDGE>
__device__ inline double add5(double acc, const double* p, const Wrap& w) {
    if constexpr (!EDGE) {
#pragma unroll
        for (int t = 0; t < 5; ++t) acc += p[t];
        return acc;
    }
    acc += opt(w.rl, p[4]);    // S wrapped to row 0: first
    acc += opt(!w.r0, p[0]);   // N
    acc += opt(w.cl, p[3]);    // E wrapped to column 0: before W
    acc += opt(!w.c0, p[1]);   // W
    acc += p[2];               // C
    acc += opt(!w.cl, p[3]);   // E
    acc += opt(w.c0, p[1]);    // W wrapped to column n-1: after E
    acc += opt(!w.rl, p[4]);   // S
    acc += opt(w.r0, p[0]);    // N wrapped to row n-1: last
    return acc;
}
// 2 x 2 block products p = {a_lo, a_hi, b_lo, b_hi} (rows a above b, columns lo left of hi): the lower row
// comes first when it wraps (bwrap), the high column first when the pair wraps (cwrap).
template <bool EDGE>
__device__ inline double add4(double acc, const double* p, bool bwrap, bool cwrap) {
    if constexpr (!EDGE) {
#pragma unroll
        for (int t = 0; t < 4; ++t) acc += p[t];
        return acc;
    }
    acc += opt(bwrap && cwrap, p[3]);
    acc += opt(bwrap, p[2]);
    acc += opt(bwrap && !cwrap, p[3]);
    acc += opt(cwrap, p[1]);
    acc += p[0];
    acc += opt(!cwrap, p[1]);
    acc += opt(!bwrap && cwrap, p[3]);
    acc += opt(!bwrap, p[2]);
    acc += opt(!bwrap && !cwrap, p[3]);
    return acc;
}

// Offset of local grid row lr (-h <= lr < L + h) of field f in an nf-field vector of the row-partition
// layout: the owned rows field-major, then h ghost rows above of every field (increasing row order), then
// h ghost rows below of every field.
__device__ inline int32_t ext_row(int nf, int f, int lr, int L, int h, int n) {
    if (lr >= 0 && lr < L) return (f * L + lr) * n;
    return nf * L * n + (lr < 0 ? f * h + h + lr : nf * h + f * h + lr - L) * n;
}

struct FStencilDev {
    static constexpr bool kFast = false;   // FStencilFast: tolerance-mode rows (rows4 / rdiag4, reciprocal diagonals)
    int n;
    double xi, eta_n, eta_s, c, d_u;
    const double* cell;
    const double* uface;
    const double* vface;
    // grid constants, evaluated once on the host exactly as the assembly evaluates them on the device
    double dxdx;   // dx * dx
    double idx2;   // 1.0 / (dx * dx)   (== 1.0 / (dy * dy), 1.0 / (dx * dy): dx == dy)
    double midy2;  // -1.0 / (dy * dy)
    // row partition: this rank owns grid rows [r0, r0 + L) of each of the 4 velocity fields; the ghosts
    // follow the 4*L*n owned entries: h rows above of every field, then h rows below of every field.
    // One GPU: r0 = 0, L = n, h = 0.
    int r0, L, h, which;
    int pow2;      // n is a power of two: dx * dx is a power of two and v / (dx * dx) == v * idx2 exactly
    int ext = 0;   // which = 3: ghost rows computed on each side
    int oh = 0;    // ghost depth of the output's layout (== h)
    double ce0 = 0.0, ce1 = 0.0;   // pow2: eta_n * idx2, eta_s * idx2 (exact: idx2 is a power of two)

    __device__ int wrap(int a) const { return a < 0 ? a + n : (a >= n ? a - n : a); }
    // index in x of (field f, grid row gr, column 0) for gr in [r0 - h, r0 + L + h)
    __device__ int32_t xrow(int f, int gr) const {
        if (h == 0) return (f * n + wrap(gr)) * n;
        return ext_row(4, f, gr - r0, L, h, n);
    }
    // k_march policy: the 4 velocity fields staged, the cell's 4 rows out; per cell, the u- and v-face
    // thn values are requested with the epilogue operands (before the barrier), not inside the rows
    static constexpr int NF = 4, NOUT = 4;
    struct Cell { double face[2]; };
    __device__ Cell cell_pre(int gr, int gc) const { return {{uface[gr * n + gc], vface[gr * n + gc]}}; }
    __device__ int32_t out_row(int f, int lr, int gc) const {
        return (lr >= 0 && lr < L ? (f * L + lr) * n : ext_row(4, f, lr, L, oh, n)) + gc;
    }
    template <bool EDGE, class TA, class XA>
    __device__ double row(int f, int gr, int gc, const TA& ta, const XA& xa, double* fd, const Cell& cl) const;
    // k_march_init: the face thn a staged point's diagonal needs, and that diagonal
    struct Stage { double face[2]; };
    __device__ Stage stage_pre(int gr, int gcw) const {
        const int32_t k = wrap(gr) * n + gcw;
        return {{uface[k], vface[k]}};
    }
    template <class TA>
    __device__ double stage_diag(int f, int gr, int gc, const TA& ta, const Stage& s) const;
};

// The diagonal of an F row (phase_L_row's diagonal + XI + the c-weighted identity, F_row), with the
// intermediate thn averages the row's off-diagonal entries reuse.  One definition serves the row itself
// (f_row) and the first inner sweep's staged x0 = c2 b / diag (k_march_init), so both see the same bits.
// M: f_row's compile-time parameter identities.
template <int M>
struct FDiagCommon {
    __device__ static double dmul(const FStencilDev& P, double y) { return (M & 1) ? -y : P.d_u * y; }
    __device__ static double emul(const FStencilDev& P, int p, double y) {
        const bool eta1 = p ? (M & 4) != 0 : (M & 2) != 0;
        return eta1 ? y : (p ? P.eta_s : P.eta_n) * y;
    }
};
template <int M>
struct FDiagU : FDiagCommon<M> {   // u row at (gr, gc): preconditioner.py:100-179
    double iph_jph, iph_jmh, xi_ii, fd;
    template <class TA>
    __device__ FDiagU(const FStencilDev& P, int p, const TA& ta, int gr, int gc, double th) {
        const double tij = ta.T(p, gr, gc - 1), tip1j = ta.T(p, gr, gc);
        const double tijp1 = ta.T(p, gr - 1, gc - 1), tip1jp1 = ta.T(p, gr - 1, gc);
        const double tijm1 = ta.T(p, gr + 1, gc - 1), tip1jm1 = ta.T(p, gr + 1, gc);
        iph_jph = 0.25 * (tij + tijp1 + tip1jp1 + tip1j);
        iph_jmh = 0.25 * (tij + tip1j + tijm1 + tip1jm1);
        const double iph_j = 0.5 * (tij + tip1j);
        xi_ii = xi_of(P.xi, iph_j);
        const double wt = p ? P.c * (1.0 - th) : P.c * th;
        const double Ldiag = P.idx2 * (-tip1j - tij) + P.idx2 * (-iph_jph - iph_jmh);
        fd = (wt - this->dmul(P, xi_ii)) + this->dmul(P, this->emul(P, p, Ldiag));
    }
};
template <int M>
struct FDiagV : FDiagCommon<M> {   // v row at (gr, gc): preconditioner.py:182-295
    double tij, tijp1, imh_jph, iph_jph, xi_ii, fd;
    template <class TA>
    __device__ FDiagV(const FStencilDev& P, int p, const TA& ta, int gr, int gc, double th) {
        tij = ta.T(p, gr, gc);
        const double tip1j = ta.T(p, gr, gc + 1);
        tijp1 = ta.T(p, gr - 1, gc);
        const double tip1jp1 = ta.T(p, gr - 1, gc + 1);
        const double tim1j = ta.T(p, gr, gc - 1), tim1jp1 = ta.T(p, gr - 1, gc - 1);
        const double ip1_jph = 0.5 * (tij + tijp1);
        xi_ii = xi_of(P.xi, ip1_jph);
        const double wt = p ? P.c * (1.0 - th) : P.c * th;
        imh_jph = 0.25 * (tim1j + tim1jp1 + tij + tijp1);
        iph_jph = 0.25 * (tij + tip1j + tijp1 + tip1jp1);
        const double Ldiag = P.midy2 * (tijp1 + tij) - P.idx2 * (iph_jph + imh_jph);
        fd = (wt - this->dmul(P, xi_ii)) + this->dmul(P, this->emul(P, p, Ldiag));
    }
};

template <int M, class TA>
__device__ inline double f_stage_diag(const FStencilDev& P, int f, int gr, int gc, const TA& ta,
                                      const FStencilDev::Stage& s) {
    const int p = f >> 1;
    return (f & 1) == 0 ? FDiagU<M>(P, p, ta, gr, gc, s.face[0]).fd : FDiagV<M>(P, p, ta, gr, gc, s.face[1]).fd;
}
template <class TA>
__device__ inline double FStencilDev::stage_diag(int f, int gr, int gc, const TA& ta, const Stage& s) const {
    return f_stage_diag<0>(*this, f, gr, gc, ta, s);
}

// The ten entries of one F row, built in the assembled row's column order for interior points and
// sorted (with fixed networks) where periodic wrap-around reorders them.  TA::T(s, gr, gc) is thn of
// phase s at a cell, XA::X(f, gr, gc) the x entry of field f at a grid point (gr in [-1, n], gc in
// [-1, n]; the accessors wrap).  Same operations as phase_L_row / F_row, same summation order.
// M (exact parameter identities, compile time): bit 0 d_u == -1 (d_u * y is an exact negation, folded into
// the products as a sign), bit 1 eta_n == 1, bit 2 eta_s == 1 (eta * y == y exactly), bit 3 idx2 a power of
// two: eta * (idx2 * y) == y * (eta * idx2) for every y (idx2 * y and eta * idx2 are exact scalings, so both
// sides are the one rounding of the same real), one multiply per off-diagonal entry instead of two.  Every
// entry keeps the assembly's rounding; only multiplications whose result is exactly known are skipped.
template <bool EDGE, class TA, class XA, bool VIRT = false, int M = 0>
__device__ inline double f_row(const FStencilDev& P, int f, int gr, int gc, const TA& ta, const XA& xa,
                               double* fdiag, const double* face = nullptr) {
    const int n = P.n;
    const int p = f >> 1;
    const double idx2 = P.idx2;
    const double eta = p ? P.eta_s : P.eta_n;
    const bool eta1 = p ? (M & 4) != 0 : (M & 2) != 0;
    auto dmul = [&](double y) -> double { return (M & 1) ? -y : P.d_u * y; };   // d_u * y
    auto emul = [&](double y) -> double { return eta1 ? y : eta * y; };          // eta * y
    auto sc = [&](double y) -> double {                                          // eta * (idx2 * y)
        if constexpr ((M & 8) != 0) return eta1 ? idx2 * y : y * (p ? P.ce1 : P.ce0);
        else return emul(idx2 * y);
    };
    const int fu = 2 * p, fv = 2 * p + 1;
    const int32_t kc = VIRT ? P.wrap(gr) * n + P.wrap(gc) : gr * n + gc;   // VIRT: (gr, gc) may lie one cell outside
    auto T = [&](int r, int c) -> double { return ta.T(p, r, c); };
    const Wrap w{gr == 0, gr == n - 1, gc == 0, gc == n - 1};   // read by the EDGE form only
    double acc = 0.0;
    const double xcross = xa.X(f ^ 2, gr, gc);
    if ((f & 1) == 0) {   // u row: preconditioner.py:100-179
        const double tij = T(gr, gc - 1), tip1j = T(gr, gc);
        const double th = face ? face[0] : P.uface[kc];   // face: thn at the u / v face, loaded ahead
        const FDiagU<M> dd(P, p, ta, gr, gc, th);
        const double iph_jph = dd.iph_jph, iph_jmh = dd.iph_jmh, xi_ii = dd.xi_ii;
        const double fd = dd.fd;
        *fdiag = fd;
        // same field: N, W, C, E, S; the other component (v of this phase): (gr, gc-1), (gr, gc), (gr+1, gc-1),
        // (gr+1, gc)
        const double lo[5] = {dmul(sc(iph_jph)) * xa.X(fu, gr - 1, gc),
                              dmul(sc(tij)) * xa.X(fu, gr, gc - 1),
                              fd * xa.X(fu, gr, gc),
                              dmul((M & 8) ? sc(tip1j) : emul(P.pow2 ? tip1j * idx2 : tip1j / P.dxdx)) * xa.X(fu, gr, gc + 1),
                              dmul(sc(iph_jmh)) * xa.X(fu, gr + 1, gc)};
        const double hi[4] = {dmul(sc(tij - iph_jph)) * xa.X(fv, gr, gc - 1),
                              dmul(sc(-tip1j + iph_jph)) * xa.X(fv, gr, gc),
                              dmul(sc(iph_jmh - tij)) * xa.X(fv, gr + 1, gc - 1),
                              dmul(sc(tip1j - iph_jmh)) * xa.X(fv, gr + 1, gc)};
        const double vcross = dmul(xi_ii);
        if (p == 1) acc += vcross * xcross;
        acc = add5<EDGE>(acc, lo, w);
        acc = add4<EDGE>(acc, hi, w.rl, w.c0);
        if (p == 0) acc += vcross * xcross;
    } else {              // v row: preconditioner.py:182-295
        const double th = face ? face[1] : P.vface[kc];
        const FDiagV<M> dd(P, p, ta, gr, gc, th);
        const double tij = dd.tij, tijp1 = dd.tijp1;
        const double imh_jph = dd.imh_jph, iph_jph = dd.iph_jph, xi_ii = dd.xi_ii;
        const double fd = dd.fd;
        *fdiag = fd;
        // the other component (u of this phase): (gr-1, gc), (gr-1, gc+1), (gr, gc), (gr, gc+1); same field: N, W,
        // C, E, S
        const double lo[4] = {dmul(sc(tijp1 - imh_jph)) * xa.X(fu, gr - 1, gc),
                              dmul(sc(iph_jph - tijp1)) * xa.X(fu, gr - 1, gc + 1),
                              dmul(sc(imh_jph - tij)) * xa.X(fu, gr, gc),
                              dmul(sc(tij - iph_jph)) * xa.X(fu, gr, gc + 1)};
        const double hi[5] = {dmul(sc(tijp1)) * xa.X(fv, gr - 1, gc),
                              dmul(sc(imh_jph)) * xa.X(fv, gr, gc - 1),
                              fd * xa.X(fv, gr, gc),
                              dmul(sc(iph_jph)) * xa.X(fv, gr, gc + 1),
                              dmul(sc(tij)) * xa.X(fv, gr + 1, gc)};
        const double vcross = dmul(xi_ii);
        if (p == 1) acc += vcross * xcross;
        acc = add4<EDGE>(acc, lo, w.r0, w.cl);
        acc = add5<EDGE>(acc, hi, w);
        if (p == 0) acc += vcross * xcross;
    }
    return acc;
}

// ---- tolerance-mode F (plan numerics "fast"): north_star's 1e-12 bar instead of the assembly's bits ----
// The same operator with its four rows per cell regrouped around the phase-n thn at the cell centres and at the grid
// nodes (corner K(r, c): the average of the four cells around the node between rows r-1, r and columns c-1, c;
// phase s uses 1 - t), FMA-contracted.  With a = d_u eta idx2 and -d_u xi h (1 - h) the XI coupling (h: the face
// average), a u row (left / right cells A1 = T(r, c-1), A2 = T(r, c), nodes KN = K(r, c), KS = K(r+1, c)) is
//   F u = wt u_C - d_u xi_h (u_C - u_o) + a [KN (u_N - u_C + v2 - v1) + A1 (u_W - u_C + v1 - v3)
//                                           + A2 (u_E - u_C + v4 - v2) + KS (u_S - u_C + v3 - v4)]
// (v1..v4 = v(r, c-1), v(r, c), v(r+1, c-1), v(r+1, c)), diag = wt - d_u xi_h - a (A1 + A2 + KN + KS) -- the
// entries of preconditioner.py:100-179 collected per coefficient; a v row (:182-295) likewise with B1 = T(r-1, c),
// B2 = T(r, c), KW = K(r, c), KE = K(r, c+1) and u1..u4 = u(r-1, c), u(r-1, c+1), u(r, c), u(r, c+1).  Per row
// about 40 fp64 VALU operations (corners once per cell, a reciprocal diagonal by v_rcp_f64 and two Newton steps)
// instead of ~170 for the bit-exact rows; every value stays within a few ulp of the assembled row (numpy check:
// 3e-16 of max |F x|).  No periodic sorting: the sum has no order to reproduce.
__device__ inline double rcp_nr(double y) {
    double r = __builtin_amdgcn_rcp(y);
    double e = __builtin_fma(-y, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-y, r, 1.0);
    return __builtin_fma(r, e, r);
}
struct FStencilFast : FStencilDev {
    static constexpr bool kFast = true;
    struct Nb { double nw, nn, ne, w, c, e, sw, s; };   // phase-n thn around (r, c) (the 3 x 3 block minus (r+1, c+1))
    template <class TA>
    __device__ static Nb nb(const TA& ta, int gr, int gc) {
        return {ta.T(0, gr - 1, gc - 1), ta.T(0, gr - 1, gc), ta.T(0, gr - 1, gc + 1), ta.T(0, gr, gc - 1),
                ta.T(0, gr, gc), ta.T(0, gr, gc + 1), ta.T(0, gr + 1, gc - 1), ta.T(0, gr + 1, gc)};
    }
    // per-cell coefficients, phase n: A1 = w, A2 = B2 = c, B1 = nn; nodes kc = K(r, c), ks = K(r+1, c), ke = K(r, c+1)
    struct Co { double w, c, nn, kc, ks, ke, xu, xv; };
    __device__ Co coeffs(const Nb& t) const {
        const double wc = t.w + t.c;
        Co k;
        k.w = t.w; k.c = t.c; k.nn = t.nn;
        k.kc = 0.25 * ((t.nw + t.nn) + wc);
        k.ks = 0.25 * (wc + (t.sw + t.s));
        k.ke = 0.25 * ((t.nn + t.ne) + (t.c + t.e));
        const double hu = 0.5 * wc, hv = 0.5 * (t.nn + t.c);
        const double mx = -d_u * xi;             // -d_u xi h (1 - h): the same for both phases (h_s = 1 - h_n)
        k.xu = mx * (hu * (1.0 - hu));
        k.xv = mx * (hv * (1.0 - hv));
        return k;
    }
    __device__ double aco(int p) const { return d_u * (p ? eta_s : eta_n) * idx2; }
    // a cell's level-invariant row terms beside Co: the identity weights c thn_p at its u / v face, per phase
    struct W4 { double wu[2], wv[2]; };
    __device__ W4 weights(const Cell& cl) const {
        return {{c * cl.face[0], c * (1.0 - cl.face[0])}, {c * cl.face[1], c * (1.0 - cl.face[1])}};
    }
    // the four rows (u_n, v_n, u_s, v_s) of cell (gr, gc) from its coefficients k and weights w.  The XI coupling
    // xu (u_C - u_o) of the s phase is the n phase's negated (u_s - u_n = -(u_n - u_s) and xu (-y) = -(xu y) exactly in
    // round-to-nearest): one difference and one product serve both phases.
    template <class XA>
    __device__ void rows4_co(int gr, int gc, const Co& k, const W4& w, const XA& xa, double* acc) const {
        const double xdu = k.xu * (xa.X(0, gr, gc) - xa.X(2, gr, gc));
        const double xdv = k.xv * (xa.X(1, gr, gc) - xa.X(3, gr, gc));
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int fu = 2 * p, fv = 2 * p + 1;
            auto ph = [&](double t) { return p ? 1.0 - t : t; };
            const double a = aco(p);
            const double A1 = ph(k.w), A2 = ph(k.c), B1 = ph(k.nn), KC = ph(k.kc), KS = ph(k.ks), KE = ph(k.ke);
            const double uC = xa.X(fu, gr, gc), uN = xa.X(fu, gr - 1, gc), uS = xa.X(fu, gr + 1, gc);
            const double uW = xa.X(fu, gr, gc - 1), uE = xa.X(fu, gr, gc + 1), uNE = xa.X(fu, gr - 1, gc + 1);
            const double vC = xa.X(fv, gr, gc), vN = xa.X(fv, gr - 1, gc), vS = xa.X(fv, gr + 1, gc);
            const double vW = xa.X(fv, gr, gc - 1), vE = xa.X(fv, gr, gc + 1), vSW = xa.X(fv, gr + 1, gc - 1);
            // the node (r, c) and centre (r, c) terms are shared by the u and v rows: the v row's are -tn (the same
            // differences negated: exact) and tc (the same sum, operands swapped: exact)
            const double tn = (uN - uC) + (vC - vW), tc = (uE - uC) + (vS - vC);
            // u row: v1 = vW, v2 = vC, v3 = vSW, v4 = vS
            double br = KC * tn;
            br = __builtin_fma(A1, (uW - uC) + (vW - vSW), br);
            br = __builtin_fma(A2, tc, br);
            br = __builtin_fma(KS, (uS - uC) + (vSW - vS), br);
            acc[fu] = __builtin_fma(a, br, __builtin_fma(w.wu[p], uC, p ? -xdu : xdu));
            // v row: u1 = uN, u2 = uNE, u3 = uC, u4 = uE
            double bv = B1 * ((vN - vC) + (uN - uNE));
            bv = __builtin_fma(KC, -tn, bv);
            bv = __builtin_fma(KE, (vE - vC) + (uNE - uE), bv);
            bv = __builtin_fma(A2, tc, bv);
            acc[fv] = __builtin_fma(a, bv, __builtin_fma(w.wv[p], vC, p ? -xdv : xdv));
        }
    }
    // the four rows (u_n, v_n, u_s, v_s) of cell (gr, gc) and their reciprocal diagonals
    // RD = false: the diagonals are the caller's (k_ftile level B reuses level A's, computed by the same operations)
    template <bool RD = true, class TA, class XA>
    __device__ void rows4(int gr, int gc, const TA& ta, const XA& xa, const Cell& cl, double* acc, double* rd) const {
        const Co k = coeffs(nb(ta, gr, gc));
        const W4 w = weights(cl);
        rows4_co(gr, gc, k, w, xa, acc);
        if constexpr (RD) rdiag4_co(k, w, rd);
    }
    // the reciprocal diagonals from a cell's coefficients and weights (rdiag4's arithmetic)
    __device__ void rdiag4_co(const Co& k, const W4& w, double* rd) const {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            auto ph = [&](double t) { return p ? 1.0 - t : t; };
            const double a = aco(p);
            const double A1 = ph(k.w), A2 = ph(k.c), B1 = ph(k.nn), KC = ph(k.kc), KS = ph(k.ks), KE = ph(k.ke);
            rd[2 * p] = rcp_nr(__builtin_fma(-a, (A1 + A2) + (KC + KS), w.wu[p] + k.xu));
            rd[2 * p + 1] = rcp_nr(__builtin_fma(-a, (B1 + A2) + (KC + KE), w.wv[p] + k.xv));
        }
    }
    // the reciprocal diagonals of the four rows at a staged point (k_march_init: x0 = c2 b / diag)
    template <class TA>
    __device__ void rdiag4(int gr, int gc, const TA& ta, const Stage& sg, double* rd) const {
        const Co k = coeffs(nb(ta, gr, gc));
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            auto ph = [&](double t) { return p ? 1.0 - t : t; };
            const double a = aco(p);
            const double A1 = ph(k.w), A2 = ph(k.c), B1 = ph(k.nn), KC = ph(k.kc), KS = ph(k.ks), KE = ph(k.ke);
            rd[2 * p] = rcp_nr(__builtin_fma(-a, (A1 + A2) + (KC + KS), c * ph(sg.face[0]) + k.xu));
            rd[2 * p + 1] = rcp_nr(__builtin_fma(-a, (B1 + A2) + (KC + KE), c * ph(sg.face[1]) + k.xv));
        }
    }
};

// Tolerance-mode F inner solve from x = 0 on a row partition's owned rows (the per-operator exchange schedule: the
// multigrid level-0 smoothing and the Chebyshev / Jacobi F solves there): x0 = d0 = (c2 b) (1 / diag) with the
// reciprocal diagonals of FStencilFast::rdiag4 over the global thn table -- the operations of the one-GPU fast first
// sweep (k_ftile / k_fsolve level 0, k_march_init), so the partitioned fast solve starts from the same bits (the stored
// diagonal's c2 (b / diag) does not).  One thread per owned cell, its four rows.
struct TGlob {   // thn at wrapped grid coordinates, straight from the global table
    const double* t;
    int n;
    __device__ double T(int sph, int r, int c) const {
        r = r < 0 ? r + n : (r >= n ? r - n : r);
        c = c < 0 ? c + n : (c >= n ? c - n : c);
        const double v = t[r * n + c];
        return sph ? 1.0 - v : v;
    }
};
template <bool CHEB>
__global__ void __launch_bounds__(256) k_f_fast_init(FStencilFast P, const double* __restrict__ b, double c2,
                                                     double* __restrict__ d, const double* __restrict__ sub,
                                                     double* __restrict__ xo) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)P.L * P.n) return;
    const int lr = (int)(i / P.n), gc = (int)(i - (int64_t)lr * P.n);
    const int gr = P.r0 + lr;
    const int32_t k = gr * P.n + gc;
    const FStencilDev::Stage sg{{P.uface[k], P.vface[k]}};
    double rd[4];
    P.rdiag4(gr, gc, TGlob{P.cell, P.n}, sg, rd);
#pragma unroll
    for (int f = 0; f < 4; ++f) {
        const int64_t o = ((int64_t)f * P.L + lr) * P.n + gc;
        const double x0 = c2 * b[o] * rd[f];
        if constexpr (CHEB) d[o] = x0;
        xo[o] = sub ? sub[o] - x0 : x0;
    }
}

// ---- marching kernels: a workgroup owns a 256-column strip of `rows` consecutive grid rows and walks
// down it with a 3-row LDS ring per staged field (+ thn).  Each step stages ONE new grid row (its loads
// are issued before the current row is computed, so their latency hides under the arithmetic) instead
// of three, and the epilogue operands of the row are requested before the barrier.  The kernel is
// generic over the stencil S (F, D, G, Gt_G below):
//   S::NF staged input fields, S::NOUT output rows per cell, S::xrow(f, gr) the input layout,
//   S::out_row(o, lr, gc) the output layout, S::row<EDGE>(o, ...) output row o's sum and diagonal
//   (EDGE: the cell is on the grid's border, where periodic wrap reorders the row's columns);
// and over the source XS of the staged input: the vector itself, or (first inner sweep) the inner
// solver's x0 = c2 * (b / diag) recomputed from b and diag, so that sweep needs no init pass.
constexpr int kMB = 256;   // columns (threads) per marching workgroup
constexpr int kMTileW = kMB + 2;       // + one halo column each side
struct XRing {
    const double* x;   // [NF][3][kMTileW]
    int s[3];          // ring slot of rows gr-1, gr, gr+1
    int gr, c0;
    __device__ double X(int f, int r, int c) const { return x[(f * 3 + s[r - gr + 1]) * kMTileW + (c - c0 + 1)]; }
};
template <int W, int OFF>
struct TRingT {
    const double* t;   // [slots][W]: tile column 0 is grid column c0 - OFF
    int s[3];
    int gr, c0;
    __device__ double T(int sph, int r, int c) const {
        const double v = t[s[r - gr + 1] * W + (c - c0 + OFF)];
        return sph ? 1.0 - v : v;
    }
};
using TRing = TRingT<kMTileW, 1>;

// Staged sources: load(i) issues the loads of element i (raw registers, nothing consumes them yet), value(raw)
// turns them into the staged value at LDS-store time -- so a tile row's loads stay in flight through the
// previous row's compute even when the staged value needs arithmetic (XInit's division).
struct XPlain {        // staged value = x[i]
    const double* __restrict__ x;
    typedef double Raw;
    __device__ Raw load(int32_t i) const { return x[i]; }
    __device__ double value(const Raw& r) const { return r; }
    __device__ double operator()(int32_t i) const { return x[i]; }
};
struct XInitRaw {
    double b, d;
};
struct XInit {         // staged value = the first inner iterate: c2 * (b[i] / diag[i]) (c2 = 1: Jacobi)
    const double* __restrict__ b;
    const double* __restrict__ dg;
    double c2;
    typedef XInitRaw Raw;
    __device__ Raw load(int32_t i) const { return {b[i], dg[i]}; }
    __device__ double value(const Raw& r) const { return c2 * (r.b / r.d); }
    __device__ double operator()(int32_t i) const { return c2 * (b[i] / dg[i]); }
};

// Right-hand-side sources of the marching F sweeps.  BNone: the epilogue loads b.  GxB: b is the velocity row of
// W = G x_p (solve.py:273), recomputed per row from x_p and the staged cell thn with GStencilDev::row's arithmetic
// (d_p, 1/dx, -1/dx and the wrapped neighbour's position exactly as there), so the second F solve of the apply
// (solve.py:274) reads one pressure field (8 B per cell, cached neighbours) instead of W's four (32 B per cell),
// and W is never written.  One GPU (whole-grid layouts).
struct BNone {
    static constexpr bool on = false, part = false;
    struct Q {};
    __device__ Q load(int, int, int) const { return {}; }
    template <class TA>
    __device__ double b(int, int, int, int, const TA&, const Q&) const { return 0.0; }
};
// PART: x_p in a row partition's ghost layout (L owned rows, h ghost rows each side); else the whole grid.
template <bool PART>
struct GxBT {
    static constexpr bool on = true, part = PART;
    const double* __restrict__ xp;
    double d_p, inv, minv;
    int n;
    int L = 0, h = 0;
    struct Q { double c, w, nn; };   // x_p at the cell and at its west and north neighbours (periodic)
    __device__ int32_t row(int lr, int gr) const { return PART ? ext_row(1, 0, lr, L, h, n) : gr * n; }
    // lr: the cell's local row in the partition layout, (gr, gc): its wrapped global grid coordinates
    __device__ Q load(int lr, int gr, int gc) const {
        const int gw = gc == 0 ? n - 1 : gc - 1, gn = gr == 0 ? n - 1 : gr - 1;
        const int32_t rc = row(lr, gr), rn = row(lr - 1, gn);
        return {xp[rc + gc], xp[rc + gw], xp[rn + gc]};
    }
    // velocity row o (u_n, v_n, u_s, v_s) at the cell: TA::T(p, r, c) in the accessor's coordinates (gr, c), the
    // cell's wrapped column gc decides the periodic order as GStencilDev::row does
    template <class TA>
    __device__ double b(int o, int gr, int c, int gc, const TA& ta, const Q& q) const {
        return b_at(o, gr, c, gc == 0, gr == 0, ta, q);
    }
    // the same with ta at coordinates (r, c) of the accessor's own and the cell's periodic position given as flags:
    // wrapw, its grid column is 0 (its west neighbour wraps); wrapn, its grid row is 0
    template <class TA>
    __device__ double b_at(int o, int r, int c, bool wrapw, bool wrapn, const TA& ta, const Q& q) const {
        const int p = o >> 1;
        const double t0 = ta.T(p, r, c);
        double acc = 0.0;
        if ((o & 1) == 0) {   // u row: entries p(gr, gc-1), p(gr, gc); the wrapped one sorts last
            const double gu = 0.5 * (t0 + ta.T(p, r, c - 1));
            const double uC = (d_p * (inv * gu)) * q.c, uW = (d_p * (minv * gu)) * q.w;
            acc += wrapw ? uC : uW;
            acc += wrapw ? uW : uC;
        } else {              // v row: entries p(gr-1, gc), p(gr, gc)
            const double gv = 0.5 * (t0 + ta.T(p, r - 1, c));
            const double vC = (d_p * (minv * gv)) * q.c, vN = (d_p * (inv * gv)) * q.nn;
            acc += wrapn ? vC : vN;
            acc += wrapn ? vN : vC;
        }
        return acc;
    }
};
using GxB = GxBT<false>;
using GxBPart = GxBT<true>;

// Row of tile values held between its loads and its LDS store: every lane's main column (xa, ta; tile columns
// c0-1 .. c0+254) and (lanes 0, 1) the halo columns c0+255, c0+256 (h0, t0).  (Holding the halo columns in SGPRs
// through scalar loads measured slower)
template <int NF, class Raw>
struct TileRow {
    Raw xa[NF], h0[NF];
    double ta, t0;
};

// Columns of the strip's right-hand halo (tile columns kMB, kMB + 1) and whether they exist.
struct HaloCols {
    int g0, g1;     // wrapped grid columns
    bool ok0, ok1;  // inside the grid or its periodic right neighbour (column n -> 0)
    int gl;         // this lane's halo column (lanes 0, 1: g0, g1; others re-read their main column, cached)
};

template <class S, class XS>
__device__ inline void load_tile_row(const S& P, const XS& xs, int gr, int gcA, bool okA, const HaloCols& hc,
                                     TileRow<S::NF, typename XS::Raw>& tr) {
    // Every load unconditional (lanes without a column of their own read a clamped one): no branch around a
    // load, so the compiler's wait counts stay exact and the row's loads remain in flight through the next
    // compute.  The selects happen at the LDS store (store_tile_row).
    const int ca = okA ? gcA : 0;
#pragma unroll
    for (int f = 0; f < S::NF; ++f) {
        const int32_t base = P.xrow(f, gr);
        tr.xa[f] = xs.load(base + ca);
        tr.h0[f] = xs.load(base + hc.gl);
    }
    const int32_t tb = P.wrap(gr) * P.n;
    tr.ta = P.cell[tb + ca];
    tr.t0 = P.cell[tb + hc.gl];
}

template <class XS, int NF>
__device__ inline void store_tile_row(const XS& xs, double* sx, double* st, int slot, int tid, bool okA,
                                      const HaloCols& hc, const TileRow<NF, typename XS::Raw>& tr) {
#pragma unroll
    for (int f = 0; f < NF; ++f) sx[(f * 3 + slot) * kMTileW + tid] = okA ? xs.value(tr.xa[f]) : 0.0;
    st[slot * kMTileW + tid] = okA ? tr.ta : 0.0;
    if (tid < 2) {   // lanes 0 and 1 store the halo columns
        const bool ok = tid == 0 ? hc.ok0 : hc.ok1;
#pragma unroll
        for (int f = 0; f < NF; ++f) sx[(f * 3 + slot) * kMTileW + kMB + tid] = ok ? xs.value(tr.h0[f]) : 0.0;
        st[slot * kMTileW + kMB + tid] = ok ? tr.t0 : 0.0;
    }
}

// Grid rows [la, lb) of workgroup chunk `chunk` of `nchunks`: which = 0 all owned rows, 1 rows 1 .. L-2 (no
// ghost read), 2 rows 0 and L-1 (one chunk each), 3 the owned rows and `ext` ghost rows each side.  The
// rows are split evenly (chunk sizes differ by at most one), so a launch can be sized to one round of
// workgroups (launch_march).
__device__ inline bool march_rows(int which, int L, int ext, int chunk, int nchunks, int* la, int* lb) {
    if (which == 2) {
        *la = chunk == 0 ? 0 : L - 1;
        *lb = *la + 1;
        return chunk < (L >= 2 ? 2 : 1);
    }
    const int lo = which == 1 ? 1 : which == 3 ? -ext : 0;
    const int hi = which == 1 ? L - 1 : which == 3 ? L + ext : L;
    const int rows = hi - lo;
    *la = lo + (int)((int64_t)chunk * rows / nchunks);
    *lb = lo + (int)((int64_t)(chunk + 1) * rows / nchunks);
    return *la < *lb;
}

template <class S, class XS, class Epi, class BS = BNone>
// (4 waves per SIMD asked for explicitly: the F Chebyshev instance would otherwise take 130 VGPRs -> 3)
__global__ void __launch_bounds__(kMB) __attribute__((amdgpu_waves_per_eu(4, 8)))
k_march(S P, XS xs, int nchunks, Epi epi, BS bs = BS{}) {
    constexpr int NF = S::NF, NO = S::NOUT;
    static_assert(!S::kFast || RcpOk<Epi>::value, "a tolerance-mode policy hands over reciprocal diagonals");
    __shared__ double sx[NF * 3 * kMTileW];
    __shared__ double st[3 * kMTileW];
    const int n = P.n;
    const int strips = (n + kMB - 1) / kMB;
    const int b = xcd_swizzle(blockIdx.x, gridDim.x);
    const int strip = b % strips, chunk = b / strips;
    int la, lb;
    if (!march_rows(P.which, P.L, P.ext, chunk, nchunks, &la, &lb)) return;
    const int c0 = strip * kMB, tid = threadIdx.x;
    const int colA = c0 - 1 + tid;
    const bool okA = colA <= n;
    const int gcA = P.wrap(colA);
    // the right-hand halo columns c0+255, c0+256 (the grid's last column's periodic neighbour is column 0)
    HaloCols hc;
    {
        const int b0 = c0 + kMB - 1, b1 = c0 + kMB;
        hc.ok0 = b0 <= n;
        hc.ok1 = b1 <= n;
        hc.g0 = b0 < n ? b0 : 0;
        hc.g1 = b1 < n ? b1 : 0;
        hc.gl = tid == 0 ? hc.g0 : tid == 1 ? hc.g1 : (okA ? gcA : 0);
    }
    const int gc = c0 + tid;
    const bool live = gc < n;
    // prologue: rows la-1 -> slot 0, la -> slot 1; row la+1 in registers -- all three requested at once
    typedef TileRow<NF, typename XS::Raw> TR;
    TR tr, tp0, tp1;
    load_tile_row(P, xs, P.r0 + la - 1, gcA, okA, hc, tp0);
    load_tile_row(P, xs, P.r0 + la, gcA, okA, hc, tp1);
    load_tile_row(P, xs, P.r0 + la + 1, gcA, okA, hc, tr);
    store_tile_row(xs, sx, st, 0, tid, okA, hc, tp0);
    store_tile_row(xs, sx, st, 1, tid, okA, hc, tp1);
    // One step: row lr+1 into the ring, the next row's loads issued (LOAD: every step but the last, which is
    // peeled off so that no load sits under a branch), row lr computed from LDS.
    auto step = [&](int lr, auto load_next) {
        const int k = lr - la;
        const int sm = k % 3, s0 = (k + 1) % 3, sp = (k + 2) % 3;
        store_tile_row(xs, sx, st, sp, tid, okA, hc, tr);   // row lr+1
        // operands of this row's epilogues and cells, requested unconditionally (lanes past the grid edge
        // read row 0 and discard it) so the wait counts stay exact and later loads stay in flight
        const int gcl = live ? gc : 0;
        typename Epi::P pe[NO];
#pragma unroll
        for (int o = 0; o < NO; ++o) pe[o] = epi.pre_lite(P.out_row(o, lr, gcl));
        const typename S::Cell cl = P.cell_pre(P.wrap(P.r0 + lr), gcl);   // ghost rows wrap periodically
        const typename BS::Q bq = bs.load(lr, P.wrap(P.r0 + lr), gcl);
        __syncthreads();
        if constexpr (decltype(load_next)::value) load_tile_row(P, xs, P.r0 + lr + 2, gcA, okA, hc, tr);
        if (live) {
            const int gr = P.wrap(P.r0 + lr);
            const XRing xa{sx, {sm, s0, sp}, gr, c0};
            const TRing ta{st, {sm, s0, sp}, gr, c0};
            if constexpr (S::kFast) {   // tolerance mode: the cell's rows at once, reciprocal diagonals
                double acc[NO], rd[NO];
                P.rows4(gr, gc, ta, xa, cl, acc, rd);
#pragma unroll
                for (int o = 0; o < NO; ++o) {
                    set_diag(pe[o], rd[o]);
                    set_x(pe[o], xa.X(o, gr, gc));
                    if constexpr (BS::on) set_b(pe[o], bs.b(o, gr, gc, gc, ta, bq));
                    epi(P.out_row(o, lr, gc), acc[o], pe[o]);
                }
            } else {
            // the wrap-aware (sorting) form is exact for interior cells too: take it for the whole wave when
            // any of its cells is on the periodic edge, so a wave never runs both forms
            const bool edge = __builtin_amdgcn_readfirstlane(__any(gr == 0 || gr == n - 1 || gc == 0 || gc == n - 1)) != 0;
#pragma unroll
            for (int o = 0; o < NO; ++o) {
                double dg;
                const double acc = edge ? P.template row<true>(o, gr, gc, ta, xa, &dg, cl)
                                        : P.template row<false>(o, gr, gc, ta, xa, &dg, cl);
                set_diag(pe[o], dg);
                set_x(pe[o], xa.X(S::NF == 1 ? 0 : o, gr, gc));
                if constexpr (BS::on) set_b(pe[o], bs.b(o, gr, gc, gc, ta, bq));
                epi(P.out_row(o, lr, gc), acc, pe[o]);
            }
            }
        }
        __syncthreads();                                     // slot sm is rewritten next step
    };
    for (int lr = la; lr < lb - 1; ++lr) step(lr, std::true_type{});
    step(lb - 1, std::false_type{});
}

// ---- direct kernel for the pressure-side stencils (D, G, Gt_G) ----
// One thread per cell, no LDS and no barrier: the stencil reads its neighbours straight from global memory (the
// 8 MB pressure vectors and the thn table stay L2-resident), so a launch is n^2 / 256 independent workgroups at
// full occupancy instead of one round of marching workgroups.  Same accessors' values, same row arithmetic.
// Measured at 1024^2 (trace means, r02o vs r02l): D 17.7 -> 13.2 us, Gt_G sweeps 13.2 / 12.1 -> 11.9 / 11.3 us, the
// Gt_G first sweep (5 divisions per cell for the staged x0) 15.6 either way.
// (lr: the thread's local row in the partition layout, gr: the same row's wrapped global index -- the row the
// stencil's accessors are called around; a neighbour row r maps to local row lr + (r - gr))
template <class S, class XS>
struct XDirect {
    const S& P;
    const XS& xs;
    int lr, gr;
    __device__ double X(int f, int r, int c) const { return xs(P.xrow(f, P.r0 + lr + (r - gr)) + P.wrap(c)); }
};
struct TDirect {
    const double* __restrict__ cell;
    int n;
    __device__ double T(int sph, int r, int c) const {
        const int rr = r < 0 ? r + n : (r >= n ? r - n : r), cc = c < 0 ? c + n : (c >= n ? c - n : c);
        const double v = cell[rr * n + cc];
        return sph ? 1.0 - v : v;
    }
};
// Rows [la, la + rows) of the partition (which = 2: rows 0 and L - 1), one thread per (row, column).
template <class S, class XS, class Epi, class BS = BNone>
__global__ void __launch_bounds__(256) k_direct(S P, XS xs, Epi epi, int la, int rows, BS bs = BS{}) {
    constexpr int NO = S::NOUT;
    static_assert(!S::kFast || RcpOk<Epi>::value, "a tolerance-mode policy hands over reciprocal diagonals");
    const int n = P.n;
    const int64_t t = (int64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 256 + threadIdx.x;
    const bool live = t < (int64_t)rows * n;
    const int tt = live ? (int)t : 0;
    const int li = tt / n, gc = tt - li * n;
    const int lr = P.which == 2 ? (li == 0 ? 0 : P.L - 1) : la + li;
    const int gr = P.wrap(P.r0 + lr);
    typename Epi::P pe[NO];
#pragma unroll
    for (int o = 0; o < NO; ++o) pe[o] = epi.pre_lite(P.out_row(o, lr, gc));
    const typename S::Cell cl = P.cell_pre(gr, gc);
    const XDirect<S, XS> xa{P, xs, lr, gr};
    const TDirect ta{P.cell, n};
    const typename BS::Q bq = bs.load(lr, gr, gc);
    if constexpr (S::kFast) {   // tolerance-mode F: the cell's four rows at once, reciprocal diagonals
        if (!live) return;
        double acc[NO], rd[NO];
        P.rows4(gr, gc, ta, xa, cl, acc, rd);
#pragma unroll
        for (int o = 0; o < NO; ++o) {
            set_diag(pe[o], rd[o]);
            set_x(pe[o], xa.X(o, gr, gc));
            if constexpr (BS::on) set_b(pe[o], bs.b(o, gr, gc, gc, ta, bq));
            epi(P.out_row(o, lr, gc), acc[o], pe[o]);
        }
        return;
    }
    const bool edge = __builtin_amdgcn_readfirstlane(__any(gr == 0 || gr == n - 1 || gc == 0 || gc == n - 1)) != 0;
    if (!live) return;
#pragma unroll
    for (int o = 0; o < NO; ++o) {
        double dg;
        const double acc = edge ? P.template row<true>(o, gr, gc, ta, xa, &dg, cl)
                                : P.template row<false>(o, gr, gc, ta, xa, &dg, cl);
        set_diag(pe[o], dg);
        set_x(pe[o], xa.X(S::NF == 1 ? 0 : o, gr, gc));
        epi(P.out_row(o, lr, gc), acc, pe[o]);
    }
}

// ---- first inner sweep with the init pass folded in, diagonal recomputed (k_march_init) ----
// The sweep stages x0 = c2 * (b / diag) (c2 = 1: Jacobi) wherever k_march would stage x, with diag -- the
// operator's own diagonal at the staged point -- rebuilt from the thn tile by the stencil (S::stage_diag, the
// same expression its rows use), so the sweep streams b alone: no diag vector, and one value in flight per
// staged point.  Rebuilding the staged row's diagonal needs thn one row below it, so the thn ring runs a row
// ahead of the x ring: 5 slots over columns c0-2 .. c0+257 (one more each side than the x tile, for the v
// rows' and the halo columns' neighbours).  Invariant at the start of step k: thn rows k-1 .. k+2 and x0 rows
// k-1, k in LDS, b row k+1 (+ its S::Stage operands) in registers.
constexpr int kTW = kMTileW + 2;
template <int NF, class Stage, class BS = BNone>
struct InitRow {
    double xa[NF], h0[NF];   // b at the lane's main column and (lanes 0, 1) its halo column
    Stage sa, sh;            // the stencil's per-point operands for the diagonal (F: the u/v face thn)
};
template <int NF, class Stage, bool PT>
struct InitRow<NF, Stage, GxBT<PT>> {
    typename GxBT<PT>::Q qa, qh;   // b recomputed from x_p (GxB): its operands at the main and the halo column
    Stage sa, sh;
};
struct ThnRow {
    double ta, te;           // thn at the lane's main column; lanes 0..3 an extra column (c0+255, c0+256, c0-2, c0+257)
};
__device__ inline int thn_extra_col(int tid, int c0) {
    return tid == 0 ? c0 + kMB - 1 : tid == 1 ? c0 + kMB : tid == 2 ? c0 - 2 : c0 + kMB + 1;
}
__device__ inline int thn_extra_slot(int tid) { return tid == 0 ? kMB + 1 : tid == 1 ? kMB + 2 : tid == 2 ? 0 : kMB + 3; }

template <class S>
__device__ inline void load_thn_row(const S& P, int gr, int colA, int tid, int c0, ThnRow& t) {
    const int n = P.n;
    const int32_t tb = P.wrap(gr) * n;
    const int ce = thn_extra_col(tid, c0);
    t.ta = P.cell[tb + (colA <= n + 1 ? P.wrap(colA) : 0)];
    t.te = P.cell[tb + (ce <= n + 1 ? P.wrap(ce) : 0)];
}
__device__ inline void store_thn_row(double* st, int slot, int tid, const ThnRow& t) {
    st[slot * kTW + tid + 1] = t.ta;
    if (tid < 4) st[slot * kTW + thn_extra_slot(tid)] = t.te;
}
template <class S, class BS>
__device__ inline void load_init_row(const S& P, const double* __restrict__ b, int gr, int gcA, bool okA,
                                     const HaloCols& hc, InitRow<S::NF, typename S::Stage, BS>& tr, const BS& bs) {
    const int ca = okA ? gcA : 0;
    if constexpr (BS::on) {   // (gr: the unwrapped global row; its local row is gr - r0)
        tr.qa = bs.load(gr - P.r0, P.wrap(gr), ca);
        tr.qh = bs.load(gr - P.r0, P.wrap(gr), hc.gl);
    } else {
#pragma unroll
        for (int f = 0; f < S::NF; ++f) {
            const int32_t base = P.xrow(f, gr);
            tr.xa[f] = b[base + ca];
            tr.h0[f] = b[base + hc.gl];
        }
    }
    tr.sa = P.stage_pre(gr, ca);
    tr.sh = P.stage_pre(gr, hc.gl);
}
// x0 of staged grid row gr (ring slot `slot`) from b and the diagonal rebuilt over thn rows gr-1 .. gr+1.
template <class S, class BS>
__device__ inline void store_init_row(const S& P, double c2, double* sx, const double* st, int slot, const int ts[3],
                                      int gr, int c0, int tid, int colA, bool okA, const HaloCols& hc,
                                      const InitRow<S::NF, typename S::Stage, BS>& tr, const BS& bs) {
    const TRingT<kTW, 2> ta{st, {ts[0], ts[1], ts[2]}, gr, c0};
    if constexpr (S::kFast) {   // tolerance mode: x0 = c2 b (1 / diag), the four reciprocal diagonals at once
        double rd[4];
        P.rdiag4(gr, colA, ta, tr.sa, rd);
#pragma unroll
        for (int f = 0; f < S::NF; ++f) {
            double bf;
            if constexpr (BS::on) bf = bs.b(f, gr, colA, P.wrap(colA), ta, tr.qa);
            else bf = tr.xa[f];
            sx[(f * 3 + slot) * kMTileW + tid] = okA ? c2 * bf * rd[f] : 0.0;
        }
        if (tid < 2) {
            const bool ok = tid == 0 ? hc.ok0 : hc.ok1;
            const int col = c0 + kMB - 1 + tid;
            P.rdiag4(gr, col, ta, tr.sh, rd);
#pragma unroll
            for (int f = 0; f < S::NF; ++f) {
                double bf;
                if constexpr (BS::on) bf = bs.b(f, gr, col, P.wrap(col), ta, tr.qh);
                else bf = tr.h0[f];
                sx[(f * 3 + slot) * kMTileW + kMB + tid] = ok ? c2 * bf * rd[f] : 0.0;
            }
        }
        return;
    }
#pragma unroll
    for (int f = 0; f < S::NF; ++f) {
        const double dg = P.stage_diag(f, gr, colA, ta, tr.sa);
        double bf;
        if constexpr (BS::on) bf = bs.b(f, gr, colA, P.wrap(colA), ta, tr.qa);
        else bf = tr.xa[f];
        sx[(f * 3 + slot) * kMTileW + tid] = okA ? c2 * (bf / dg) : 0.0;
    }
    if (tid < 2) {   // lanes 0 and 1: the halo columns c0+255, c0+256
        const bool ok = tid == 0 ? hc.ok0 : hc.ok1;
        const int col = c0 + kMB - 1 + tid;
#pragma unroll
        for (int f = 0; f < S::NF; ++f) {
            const double dg = P.stage_diag(f, gr, col, ta, tr.sh);
            double bf;
            if constexpr (BS::on) bf = bs.b(f, gr, col, P.wrap(col), ta, tr.qh);
            else bf = tr.h0[f];
            sx[(f * 3 + slot) * kMTileW + kMB + tid] = ok ? c2 * (bf / dg) : 0.0;
        }
    }
}

template <class S, class Epi, class BS = BNone>
__global__ void __launch_bounds__(kMB) __attribute__((amdgpu_waves_per_eu(4, 8)))
k_march_init(S P, const double* __restrict__ b, double c2, int nchunks, Epi epi, BS bs = BS{}) {
    constexpr int NF = S::NF, NO = S::NOUT;
    static_assert(!S::kFast || RcpOk<Epi>::value, "a tolerance-mode policy hands over reciprocal diagonals");
    __shared__ double sx[NF * 3 * kMTileW];
    __shared__ double st[5 * kTW];
    const int n = P.n;
    const int strips = (n + kMB - 1) / kMB;
    const int bk = xcd_swizzle(blockIdx.x, gridDim.x);
    const int strip = bk % strips, chunk = bk / strips;
    int la, lb;
    if (!march_rows(P.which, P.L, P.ext, chunk, nchunks, &la, &lb)) return;
    const int c0 = strip * kMB, tid = threadIdx.x;
    const int colA = c0 - 1 + tid;
    const bool okA = colA <= n;
    const int gcA = P.wrap(colA <= n + 1 ? colA : 0);
    HaloCols hc;
    {
        const int b0 = c0 + kMB - 1, b1 = c0 + kMB;
        hc.ok0 = b0 <= n;
        hc.ok1 = b1 <= n;
        hc.g0 = b0 < n ? b0 : 0;
        hc.g1 = b1 < n ? b1 : 0;
        hc.gl = tid == 0 ? hc.g0 : tid == 1 ? hc.g1 : (okA ? gcA : 0);
    }
    const int gc = c0 + tid;
    const bool live = gc < n;
    auto tslot = [&](int lr) { return (lr - la + 2) % 5; };   // thn ring slot of local row lr (lr >= la - 2)
    auto xslot = [&](int lr) { return (lr - la + 1) % 3; };   // x ring slot (lr >= la - 1)
    auto grow = [&](int lr) { return P.wrap(P.r0 + lr); };    // grid row (ghost rows wrap periodically)
    typedef InitRow<NF, typename S::Stage, BS> IR;
    // prologue: thn rows la-2 .. la+2, x0 rows la-1 and la; b row la+1 into registers
    {
        ThnRow t[5];
        IR r0, r1;
#pragma unroll
        for (int i = 0; i < 5; ++i) load_thn_row(P, P.r0 + la - 2 + i, colA, tid, c0, t[i]);
        load_init_row(P, b, P.r0 + la - 1, gcA, okA, hc, r0, bs);
        load_init_row(P, b, P.r0 + la, gcA, okA, hc, r1, bs);
#pragma unroll
        for (int i = 0; i < 5; ++i) store_thn_row(st, i, tid, t[i]);
        __syncthreads();
        const int s0[3] = {tslot(la - 2), tslot(la - 1), tslot(la)};
        store_init_row(P, c2, sx, st, xslot(la - 1), s0, grow(la - 1), c0, tid, colA, okA, hc, r0, bs);
        const int s1[3] = {tslot(la - 1), tslot(la), tslot(la + 1)};
        store_init_row(P, c2, sx, st, xslot(la), s1, grow(la), c0, tid, colA, okA, hc, r1, bs);
    }
    IR tr;
    ThnRow tn;
    load_init_row(P, b, P.r0 + la + 1, gcA, okA, hc, tr, bs);
    auto step = [&](int lr, auto load_next) {
        {   // x0 of row lr+1 (thn rows lr .. lr+2)
            const int ts[3] = {tslot(lr), tslot(lr + 1), tslot(lr + 2)};
            store_init_row(P, c2, sx, st, xslot(lr + 1), ts, grow(lr + 1), c0, tid, colA, okA, hc, tr, bs);
        }
        const int gcl = live ? gc : 0;
        typename Epi::P pe[NO];
#pragma unroll
        for (int o = 0; o < NO; ++o) pe[o] = epi.pre_lite(P.out_row(o, lr, gcl));
        const typename S::Cell cl = P.cell_pre(grow(lr), gcl);
        const typename BS::Q bq = bs.load(lr, grow(lr), gcl);
        __syncthreads();
        if constexpr (decltype(load_next)::value) {   // thn row lr+3 first: it is stored at the end of this step
            load_thn_row(P, P.r0 + lr + 3, colA, tid, c0, tn);
            load_init_row(P, b, P.r0 + lr + 2, gcA, okA, hc, tr, bs);
        }
        if constexpr (S::kFast) if (live) {
            const int gr = grow(lr);
            const XRing xa{sx, {xslot(lr - 1), xslot(lr), xslot(lr + 1)}, gr, c0};
            const TRingT<kTW, 2> ta{st, {tslot(lr - 1), tslot(lr), tslot(lr + 1)}, gr, c0};
            double acc[NO], rd[NO];
            P.rows4(gr, gc, ta, xa, cl, acc, rd);
#pragma unroll
            for (int o = 0; o < NO; ++o) {
                set_diag(pe[o], rd[o]);
                set_x(pe[o], xa.X(o, gr, gc));
                if constexpr (BS::on) set_b(pe[o], bs.b(o, gr, gc, gc, ta, bq));
                epi(P.out_row(o, lr, gc), acc[o], pe[o]);
            }
        }
        if constexpr (!S::kFast) if (live) {
            const int gr = grow(lr);
            const XRing xa{sx, {xslot(lr - 1), xslot(lr), xslot(lr + 1)}, gr, c0};
            const TRingT<kTW, 2> ta{st, {tslot(lr - 1), tslot(lr), tslot(lr + 1)}, gr, c0};
            const bool edge = __builtin_amdgcn_readfirstlane(__any(gr == 0 || gr == n - 1 || gc == 0 || gc == n - 1)) != 0;
#pragma unroll
            for (int o = 0; o < NO; ++o) {
                double dg;
                const double acc = edge ? P.template row<true>(o, gr, gc, ta, xa, &dg, cl)
                                        : P.template row<false>(o, gr, gc, ta, xa, &dg, cl);
                set_diag(pe[o], dg);
                set_x(pe[o], xa.X(S::NF == 1 ? 0 : o, gr, gc));
                if constexpr (BS::on) set_b(pe[o], bs.b(o, gr, gc, gc, ta, bq));
                epi(P.out_row(o, lr, gc), acc, pe[o]);
            }
        }
        if constexpr (decltype(load_next)::value) store_thn_row(st, tslot(lr + 3), tid, tn);   // slot of row lr-2
        __syncthreads();
    };
    for (int lr = la; lr < lb - 1; ++lr) step(lr, std::true_type{});
    step(lb - 1, std::false_type{});
}

// ---- two fused Chebyshev sweeps over F, tolerance mode (k_march2) ----
// Sweeps s and s+1 of an F Chebyshev solve in one pass down the strip.  Level A stages x_{s-1} (x_in) in a 3-row
// LDS ring and computes x_s, d_s of grid row t; x_s goes to a second ring, d_s (and b, the faces) stay in the lane's
// registers -- level B, one row behind, computes x_{s+1} of row t-1 on the same column from that ring.  Per F row the
// pair reads x_in, d_in, b (or x_p, GxB), thn and writes x_out (+ d_out unless the pair ends the solve): 38 B instead of
// 84 B for two k_march sweeps; x_s and d_s never leave the CU.  Level A also computes x_s on the columns either side
// of the strip (c0 - 1, c0 + 256: one extra pass of lanes 0, 1) for level B's stencil.  Each level performs exactly
// the IEEE operations of one tolerance-mode k_march sweep (FStencilFast::rows4, the RCP Chebyshev update), so the pair
// is bit-identical to two k_march sweeps.  Rows: level A [la-1, lb], level B [la, lb) -- under a row partition the
// input needs one more ghost row each side than the output (the CA schedule's depths provide it).
constexpr int kRA = kMB + 4;   // ring A (x_in) and the thn ring: columns c0-2 .. c0+257
template <int W, int OFF>
struct XRingW {
    const double* x;   // [4][3][W]: tile column 0 is grid column c0 - OFF
    int s[3];
    int gr, c0;
    __device__ double X(int f, int r, int c) const { return x[(f * 3 + s[r - gr + 1]) * W + (c - c0 + OFF)]; }
};
struct Fused2 {
    const double* x_in;
    const double* d_in;
    const double* b;      // BNone: the right-hand side; GxB: unused (recomputed from x_p)
    const double* sub;    // SUB: the solve's last sweep returns sub - x
    double* x_out;
    double* d_out;        // SD: level B's direction is stored
    double c1a, c2a, c1b, c2b;
};
struct Stage2 {
    double x[4], xh[4];   // x_in at the lane's column c0-2+tid and (lanes 0..3) c0+254+tid
    double t, th;         // thn at the same columns
};
template <class BS>
struct OpsA {             // level A's operands at one column of row t
    double d[4], face[2];
    typename BS::Q q;
    double b[4];
};

template <bool SUB, bool SD, class BS>
__global__ void __launch_bounds__(kMB) __attribute__((amdgpu_waves_per_eu(2, 8)))
k_march2(FStencilFast P, Fused2 a, int nchunks, BS bs) {
    __shared__ double ra[4 * 3 * kRA];
    __shared__ double rb[4 * 3 * kMTileW];
    __shared__ double st[5 * kRA];
    const int n = P.n;
    const int strips = (n + kMB - 1) / kMB;
    const int bk = xcd_swizzle(blockIdx.x, gridDim.x);
    const int strip = bk % strips, chunk = bk / strips;
    int la, lb;
    if (!march_rows(P.which, P.L, P.ext, chunk, nchunks, &la, &lb)) return;
    const int c0 = strip * kMB, tid = threadIdx.x;
    const int cm = c0 - 2 + tid, ch = c0 + kMB - 2 + tid;   // staged columns (ch: lanes 0..3)
    const bool okm = cm <= n + 1, okh = tid < 4 && ch <= n + 1;
    const int gm = okm ? P.wrap(cm) : 0, gh = okh ? P.wrap(ch) : gm;
    const int gc = c0 + tid;                                  // levels A and B: the lane's column
    const bool liveA = gc <= n, liveB = gc < n;
    const int gcl = liveB ? gc : 0;                           // operand column (column n: level A's halo, wraps to 0)
    const int gca = liveA ? P.wrap(gc) : 0;
    // lanes 0, 1: level A's halo columns c0-1, c0+256 (extra pass)
    const int cx = tid == 0 ? c0 - 1 : c0 + kMB;
    const bool liveX = tid < 2 && cx <= n;
    const int gcx = liveX ? P.wrap(cx) : gca;
    auto xslot = [&](int r) { return (r - la + 2) % 3; };   // ring A (rows >= la-2)
    auto tslot = [&](int r) { return (r - la + 2) % 5; };   // thn ring
    auto bslot = [&](int r) { return (r - la + 1) % 3; };   // ring B (rows >= la-1)
    auto grow = [&](int lr) { return P.wrap(P.r0 + lr); };
    // a row of the output layout: one GPU wraps level A's rows -1 and n periodically; a partition's ghost rows are in
    // the ext layout
    auto orow = [&](int lr) { return P.h == 0 ? P.wrap(lr) : lr; };
    auto load_stage = [&](int lr, Stage2& g) {
        const int gr = P.r0 + lr;
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            const int32_t base = P.xrow(f, gr);
            g.x[f] = a.x_in[base + gm];
            g.xh[f] = a.x_in[base + gh];
        }
        const int32_t tb = P.wrap(gr) * n;
        g.t = P.cell[tb + gm];
        g.th = P.cell[tb + gh];
    };
    auto store_stage = [&](int lr, const Stage2& g) {
        const int xs = xslot(lr), ts = tslot(lr);
#pragma unroll
        for (int f = 0; f < 4; ++f) ra[(f * 3 + xs) * kRA + tid] = okm ? g.x[f] : 0.0;
        st[ts * kRA + tid] = okm ? g.t : 0.0;
        if (tid < 4) {
#pragma unroll
            for (int f = 0; f < 4; ++f) ra[(f * 3 + xs) * kRA + kMB + tid] = okh ? g.xh[f] : 0.0;
            st[ts * kRA + kMB + tid] = okh ? g.th : 0.0;
        }
    };
    // level A's operands at (local row lr, wrapped column g): d_in, the faces, b (or G x_p's operands)
    auto load_ops = [&](int lr, int g, OpsA<BS>& o) {
#pragma unroll
        for (int f = 0; f < 4; ++f) o.d[f] = a.d_in[P.out_row(f, orow(lr), g)];
        const int32_t k = grow(lr) * n + g;
        o.face[0] = P.uface[k];
        o.face[1] = P.vface[k];
        if constexpr (BS::on) o.q = bs.load(lr, grow(lr), g);
        else {
#pragma unroll
            for (int f = 0; f < 4; ++f) o.b[f] = a.b[P.out_row(f, orow(lr), g)];
        }
    };
    // level A at row lr, column c (virtual: -1 and n wrap): x_s into ring B, d_s and b returned
    auto level_a = [&](int lr, int c, const OpsA<BS>& o, double* dA, double* bA) {
        const int gr = grow(lr);
        const XRingW<kRA, 2> xa{ra, {xslot(lr - 1), xslot(lr), xslot(lr + 1)}, gr, c0};
        const TRingT<kRA, 2> ta{st, {tslot(lr - 1), tslot(lr), tslot(lr + 1)}, gr, c0};
        const FStencilDev::Cell cl{{o.face[0], o.face[1]}};
        double acc[4], rd[4];
        P.rows4(gr, c, ta, xa, cl, acc, rd);
        const int bsl = bslot(lr);
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            double bf;
            if constexpr (BS::on) bf = bs.b(f, gr, c, P.wrap(c), ta, o.q);
            else bf = o.b[f];
            const double z = (bf - acc[f]) * rd[f];
            const double dn = a.c1a * o.d[f] + a.c2a * z;
            rb[(f * 3 + bsl) * kMTileW + (c - c0 + 1)] = xa.X(f, gr, c) + dn;
            dA[f] = dn;
            bA[f] = bf;
        }
    };
    // prologue: x_in and thn rows la-2, la-1 in the rings, row la in registers
    Stage2 g;
    {
        Stage2 g0, g1;
        load_stage(la - 2, g0);
        load_stage(la - 1, g1);
        load_stage(la, g);
        store_stage(la - 2, g0);
        store_stage(la - 1, g1);
    }
    double dP[4] = {0.0, 0.0, 0.0, 0.0}, bP[4] = {0.0, 0.0, 0.0, 0.0}, fP[2] = {0.0, 0.0};   // level A of row t-1
    auto step = [&](int t, auto load_next) {
        store_stage(t + 1, g);
        OpsA<BS> oa, ox;
        load_ops(t, gca, oa);
        load_ops(t, gcx, ox);
        double sv[4] = {0.0, 0.0, 0.0, 0.0};
        const bool doB = t - 1 >= la;
        if constexpr (SUB) {
#pragma unroll
            for (int f = 0; f < 4; ++f) sv[f] = a.sub[P.out_row(f, orow(t - 1), gcl)];
        }
        __syncthreads();
        if constexpr (decltype(load_next)::value) load_stage(t + 2, g);
        double dA[4] = {0.0, 0.0, 0.0, 0.0}, bA[4] = {0.0, 0.0, 0.0, 0.0};
        if (liveA) level_a(t, gc, oa, dA, bA);
        if (liveX) {
            double dx[4], bx[4];
            level_a(t, cx, ox, dx, bx);
        }
        __syncthreads();
        if (doB && liveB) {   // level B: row t-1 from ring B
            const int lr = t - 1, gr = grow(lr);
            const XRingW<kMTileW, 1> xa{rb, {bslot(lr - 1), bslot(lr), bslot(lr + 1)}, gr, c0};
            const TRingT<kRA, 2> ta{st, {tslot(lr - 1), tslot(lr), tslot(lr + 1)}, gr, c0};
            const FStencilDev::Cell cl{{fP[0], fP[1]}};
            double acc[4], rd[4];
            P.rows4(gr, gc, ta, xa, cl, acc, rd);
#pragma unroll
            for (int f = 0; f < 4; ++f) {
                const double z = (bP[f] - acc[f]) * rd[f];
                const double dn = a.c1b * dP[f] + a.c2b * z;
                const int32_t o = P.out_row(f, orow(lr), gc);
                if constexpr (SD) a.d_out[o] = dn;
                const double x = xa.X(f, gr, gc) + dn;
                a.x_out[o] = SUB ? sv[f] - x : x;
            }
        }
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            dP[f] = dA[f];
            bP[f] = bA[f];
        }
        fP[0] = oa.face[0];
        fP[1] = oa.face[1];
    };
    for (int t = la - 1; t < lb; ++t) step(t, std::true_type{});
    step(lb, std::false_type{});
}

// Workgroups of one marching-kernel instance the device holds at once (occupancy x CUs), queried once.
template <auto K>
int64_t march_capacity() {
    static int64_t cap = -1;
    if (cap < 0) {
        int dev = 0, cus = 0, per_cu = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, K, kMB, 0) != hipSuccess)
            cus = per_cu = 0;
        cap = (int64_t)cus * per_cu;
    }
    return cap;
}

// Launch k_march over the partition rows P.which selects, rows_per_block rows per workgroup -- except that
// a launch up to 25 % over one round of workgroups is rebalanced into exactly one round (chunks of
// rows_per_block or rows_per_block + 1 rows): a second round of a few workgroups would cost almost a whole
// sweep's latency (ghost-row launches of the CA schedule, multi-GPU row partitions).
// Chunks (workgroup row ranges) of a marching launch over the rows P.which selects; 0: nothing to do.
template <class S>
int64_t march_chunks(const S& P, int rows_per_block, int64_t capacity) {
    const int64_t grows = P.which == 0 ? P.L : P.which == 1 ? (P.L > 2 ? P.L - 2 : 0)
                          : P.which == 3 ? P.L + 2 * P.ext : (P.L >= 2 ? 2 : 1);
    if (grows == 0) return 0;
    const int64_t strips = (P.n + kMB - 1) / kMB;
    if (rows_per_block <= 0) {   // auto: the rows per workgroup that fill one round (1024^2: 4; 2048^2: 16; 512^2: 1)
        const int64_t fill = capacity > 0 ? grows * strips / capacity : 4;
        rows_per_block = (int)(fill < 1 ? 1 : fill > 16 ? 16 : fill);
    }
    int64_t chunks = P.which == 2 ? grows : (grows + rows_per_block - 1) / rows_per_block;
    if (P.which != 2) {
        const int64_t one_round = capacity / strips;
        if (one_round > 0 && chunks > one_round && chunks * 4 <= one_round * 5) chunks = one_round;
    }
    return chunks;
}

template <class S, class XS, class Epi, class BS = BNone>
int launch_march_fixed(const S& P, const XS& xs, Epi epi, int rows_per_block, hipStream_t st, const BS& bs = BS{}) {
    // D, G, Gt_G on one GPU, and (KO().f_direct) the tolerance-mode F rows: the direct kernel
    if constexpr ((!std::is_base_of_v<FStencilDev, S> && !BS::on) || S::kFast) {
        if (S::kFast ? KO().f_direct != 0 : KO().pg_direct != 0) {
            // rows as march_rows: 0 all owned, 1 rows 1 .. L-2, 2 rows 0 and L-1, 3 owned + ext ghost rows each side
            const int la = P.which == 1 ? 1 : P.which == 3 ? -P.ext : 0;
            const int lb = P.which == 1 ? P.L - 1 : P.which == 3 ? P.L + P.ext : P.L;
            const int rows = P.which == 2 ? (P.L >= 2 ? 2 : 1) : lb - la;
            if (rows <= 0) return MPBP_OK;
            const int64_t cells = (int64_t)rows * P.n;
            k_direct<S, XS, Epi, BS><<<(unsigned)((cells + 255) / 256), 256, 0, st>>>(P, xs, epi, la, rows, bs);
            MPBP_HIP(hipGetLastError());
            return MPBP_OK;
        }
    }
    const int64_t chunks = march_chunks(P, rows_per_block, march_capacity<k_march<S, XS, Epi, BS>>());
    if (chunks == 0) return MPBP_OK;
    const int64_t strips = (P.n + kMB - 1) / kMB;
    k_march<S, XS, Epi, BS><<<(unsigned)(chunks * strips), kMB, 0, st>>>(P, xs, (int)chunks, epi, bs);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

// ---- two F sweeps per launch on a 2D tile, tolerance mode (k_ftile) ----
// A workgroup owns a 64 x 8 tile of cells (two per lane: rows t>>6 and 4 + t>>6 of the tile, column t & 63).  It first
// stages, with coalesced loads, thn and (!INIT) x_in over the tile plus a two-cell halo (68 x 12 cells, 32.6 KB of LDS):
// every stencil operand after that is an LDS read at a constant offset from the cell's slot, with no periodic wrap and
// no 64-bit address arithmetic per neighbour.  Level A runs on the tile plus a one-cell halo (66 x 10 cells): INIT, the
// pointwise first iterate x0 = d0 = c2_0 b / diag (diag rebuilt from thn, FStencilFast::rdiag4); otherwise sweep s from
// x_in and d_in.  Level A's x replaces x_in in the same LDS slots (after a barrier: its stencil reads x_in around the
// cell), its d and the reciprocal diagonals of the lane's two tile cells stay in registers; level B (sweep 1, or s + 1)
// computes the tile from LDS, reusing those diagonals, and writes x_out (and d_out when SD).  Every workgroup is
// independent.  Each level performs the IEEE operations of the marching kernels' tolerance-mode rows and updates, so
// k_ftile is bit-identical to k_march_init + (k_march or) k_march2.  One GPU, whole grid.
// The LDS-tiled stencil kernels read each operand with its own ds_read_b64 (2 LDS cycles per wave on gfx950) instead
// of letting the compiler pair neighbouring slots into ds_read2_b64 (8 cycles: half the bytes per clock).
#ifndef MPBP_LDS_SINGLE
#define MPBP_LDS_SINGLE 1
#endif
#if MPBP_LDS_SINGLE && defined(__HIP_DEVICE_COMPILE__)   // (a device-code attribute: the host pass has no such feature)
#define MPBP_LDS_READS __attribute__((target("no-load-store-opt")))
#else
#define MPBP_LDS_READS
#endif
constexpr int kFTW = 64, kFTH = 8, kFSW = kFTW + 4, kFSH = kFTH + 4, kFSN = kFSW * kFSH;
template <int W, int H>
struct XTileT {  // 4 fields over a W x H block of LDS ([4][H][W]), slot (0, 0) = virtual grid cell (rb, cb)
    const double* x;
    int rb, cb;
    __device__ double X(int f, int r, int c) const { return x[(f * H + (r - rb)) * W + (c - cb)]; }
};
constexpr int kFAW = kFTW + 2, kFAH = kFTH + 2, kFAN = kFAW * kFAH;   // level A's cells: the tile + 1 halo
template <int W>
struct TTileT {  // staged thn at virtual grid coordinates, W columns per staged row
    const double* t;
    int rb, cb;
    __device__ double T(int sph, int r, int c) const {
        const double v = t[(r - rb) * W + (c - cb)];
        return sph ? 1.0 - v : v;
    }
};
template <int W>
struct TTileWT {  // staged thn at wrapped grid coordinates (GxBT::b: its wrap tests need the wrapped row / column)
    const double* t;
    int rb, cb, n;
    __device__ double T(int sph, int r, int c) const {
        int lr = r - rb, lc = c - cb;
        lr = lr < 0 ? lr + n : (lr >= n ? lr - n : lr);
        lc = lc < 0 ? lc + n : (lc >= n ? lc - n : lc);
        const double v = t[lr * W + lc];
        return sph ? 1.0 - v : v;
    }
};
struct FTile {
    const double* x_in;   // !INIT: x_{s-1}
    const double* d_in;   // !INIT: d_{s-1}
    const double* b;      // BNone: the right-hand side
    const double* sub;    // SUB: level B returns sub - x
    double* x_out;
    double* d_out;        // SD
    double c1a, c2a, c1b, c2b;   // INIT: c2a = c2_0 (c1a unused)
    int dzero = 0;        // !INIT: d_{s-1} is +0.0 (a restart: multigrid post-smoothing), d_in is not read
    const double* xc = nullptr;   // !INIT: x_in + P_0 xc (the coarse correction of a multigrid level 0, the F
                                  // hierarchy's MAC kinds) is the iterate -- the prolongation launch folded in
};

// multigrid level 1's tile and windows (k_gal1; the level-0 fused kernels stage the same windows)
constexpr int kG1W = 32, kG1H = 4;                          // coarse tile
constexpr int kG1FW = 2 * kG1W + 2, kG1FH = 2 * kG1H + 2;   // t1: fine [2 c0 - 1, 2 c0 + 2 W + 1)
constexpr int kG1PW = kG1FW + 2, kG1PH = kG1FH + 2;         // t0 and thn: one more fine cell each side
constexpr int kG1CW = kG1W + 4;                             // coarse x: [c0 - 2, c0 + W + 2)
template <int KY, int KX, int S = kG1CW>
__device__ inline double g1_p(const double* xf, int gr, int gc, int nc, int rb, int cb);
template <int KY, int KX, int S = kG1CW>
__device__ inline double g1_p_in(const double* xf, int r, int c);
template <int KY, int KX, int W, int OFF>
__device__ inline double g1_rw_in(const double* tf, int lr, int lc);
__device__ inline bool g1_inner(int cr0, int cc0, int th, int tw, int nc);
template <bool INIT, bool SUB, bool SD, class BS, bool PRO = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 8))) MPBP_LDS_READS k_ftile(FStencilFast P, FTile a, BS bs) {
    __shared__ double xs[INIT ? 1 : 4 * kFSN];   // !INIT: x_in over the tile + 2 halo
    __shared__ double ts[kFSN];                   // thn over the tile + 2 halo
    __shared__ double xl[4 * kFAN];               // level A's x over the tile + 1 halo (PRO: first the coarse window)
    const int n = P.n;
    const int tx = (n + kFTW - 1) / kFTW;
    const int bk = xcd_swizzle(blockIdx.x, gridDim.x);
    const int r0 = (bk / tx) * kFTH, c0 = (bk % tx) * kFTW;
    const int rb = r0 - 2, cb = c0 - 2;
    const int tid = threadIdx.x;
    const int nn = n * n;
    // PRO: the coarse correction over [r0 / 2 - 2, r0 / 2 + 6) x [c0 / 2 - 2, c0 / 2 + 34) of 4 fields (k_gal1's window)
    constexpr int CW = kFTW / 2 + 4, CH = kFTH / 2 + 4, CN = CW * CH;
    static_assert(!PRO || 4 * CN <= 4 * kFAN, "the coarse window fits the level-A buffer");
    static_assert(CW == kG1CW && kFSW == kG1PW && kFSH == kG1PH, "g1_p_in's window geometry");
    const int nc = n >> 1, ncc = nc * nc, cr0 = r0 >> 1, cc0 = c0 >> 1;
    // stage thn (and x_in) over rows r0-2 .. r0+9, columns c0-2 .. c0+65: every load issued before the first LDS store
    {
        constexpr int IT = (kFSN + 255) / 256, NF = INIT ? 1 : 5, IC = PRO ? (4 * CN + 255) / 256 : 1;
        double v[IT][NF], vc[IC];
        if constexpr (PRO) {
            auto wrapc = [&](int q) { return q < 0 ? q + nc : (q >= nc ? q - nc : q); };
#pragma unroll
            for (int it = 0; it < IC; ++it) {
                const int i = tid + it * 256;
                if (i < 4 * CN) {
                    const int f = i / CN, j = i - f * CN, r = j / CW, c = j - r * CW;
                    vc[it] = a.xc[f * ncc + wrapc(cr0 - 2 + r) * nc + wrapc(cc0 - 2 + c)];
                }
            }
        }
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = tid + it * 256;
            if (i < kFSN) {
                const int sr = i / kFSW, sc = i - sr * kFSW;
                const int32_t k = P.wrap(rb + sr) * n + P.wrap(cb + sc);
                v[it][0] = P.cell[k];
                if constexpr (!INIT) {
#pragma unroll
                    for (int f = 0; f < 4; ++f) v[it][1 + f] = a.x_in[f * nn + k];
                }
            }
        }
        if constexpr (PRO) {
#pragma unroll
            for (int it = 0; it < IC; ++it)
                if (tid + it * 256 < 4 * CN) xl[tid + it * 256] = vc[it];
            __syncthreads();
        }
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = tid + it * 256;
            if (i < kFSN) {
                ts[i] = v[it][0];
                if constexpr (!INIT) {
                    if constexpr (PRO) {   // x_in + P_0 xc: k_mg_transfer_spmv's prolongation and EpiAdd's sum
                        const int sr = i / kFSW, sc = i - sr * kFSW;
                        const int gr = P.wrap(rb + sr), gc = P.wrap(cb + sc);
                        const bool inner = g1_inner(cr0, cc0, kFTH / 2, kFTW / 2, nc);   // (window coordinates)
#pragma unroll
                        for (int f = 0; f < 4; ++f) {
                            const double pc =
                                inner ? ((f & 1) ? g1_p_in<MPBP_MG_NODE, MPBP_MG_CELL>(xl + f * CN, sr, sc)
                                                 : g1_p_in<MPBP_MG_CELL, MPBP_MG_NODE>(xl + f * CN, sr, sc))
                                      : ((f & 1) ? g1_p<MPBP_MG_NODE, MPBP_MG_CELL>(xl + f * CN, gr, gc, nc, cr0 - 2, cc0 - 2)
                                                 : g1_p<MPBP_MG_CELL, MPBP_MG_NODE>(xl + f * CN, gr, gc, nc, cr0 - 2, cc0 - 2));
                            xs[f * kFSN + i] = pc + v[it][1 + f];
                        }
                    } else {
#pragma unroll
                        for (int f = 0; f < 4; ++f) xs[f * kFSN + i] = v[it][1 + f];
                    }
                }
            }
        }
    }
    __syncthreads();
    const TTileT<kFSW> tt{ts, rb, cb};
    const TTileWT<kFSW> tw{ts, rb, cb, n};
    const XTileT<kFSW, kFSH> xa{xs, rb, cb};
    const XTileT<kFAW, kFAH> xb{xl, rb + 1, cb + 1};
    // level A at virtual cell (vr, vc): its x (xn), d (dA) and the reciprocal diagonals (rd)
    auto level_a = [&](int vr, int vc, double* dA, double* rd) {
        const int si = (vr - rb - 1) * kFAW + (vc - cb - 1);
        const int gr = P.wrap(vr), gc = P.wrap(vc);
        const int32_t k = gr * n + gc;
        double bv[4];
        typename BS::Q q{};
        if constexpr (BS::on) q = bs.load(gr, gr, gc);
        else {
#pragma unroll
            for (int f = 0; f < 4; ++f) bv[f] = a.b[f * nn + k];
        }
        const FStencilDev::Stage sg{{P.uface[k], P.vface[k]}};
        if constexpr (INIT) {
            P.rdiag4(vr, vc, tt, sg, rd);
#pragma unroll
            for (int f = 0; f < 4; ++f) {
                const double bf = BS::on ? bs.b(f, gr, gc, gc, tw, q) : bv[f];
                const double x0 = a.c2a * bf * rd[f];
                xl[f * kFAN + si] = x0;
                dA[f] = x0;
            }
        } else {
            double acc[4];
            P.rows4(vr, vc, tt, xa, FStencilDev::Cell{{sg.face[0], sg.face[1]}}, acc, rd);
#pragma unroll
            for (int f = 0; f < 4; ++f) {
                const double bf = BS::on ? bs.b(f, gr, gc, gc, tw, q) : bv[f];
                const double z = (bf - acc[f]) * rd[f];
                const double dprev = a.dzero ? 0.0 : a.d_in[f * nn + k];
                const double dn = a.c1a * dprev + a.c2a * z;
                xl[f * kFAN + si] = xa.X(f, vr, vc) + dn;
                dA[f] = dn;
            }
        }
    };
    const int lc = tid & 63, lr = tid >> 6;
    double dA0[4], dA1[4], rd0[4], rd1[4];
    level_a(r0 + lr, c0 + lc, dA0, rd0);
    level_a(r0 + 4 + lr, c0 + lc, dA1, rd1);
    // the halo ring: rows -1 and kFTH (66 cells each), columns -1 and kFTW of rows 0 .. kFTH-1: 148 cells
    constexpr int kRing = 2 * (kFTW + 2) + 2 * kFTH;
    if (tid < kRing) {
        int hr, hc;
        if (tid < 2 * (kFTW + 2)) {
            const int j = tid < kFTW + 2 ? tid : tid - (kFTW + 2);
            hr = tid < kFTW + 2 ? r0 - 1 : r0 + kFTH;
            hc = c0 - 1 + j;
        } else {
            const int j = tid - 2 * (kFTW + 2);
            hr = r0 + (j >> 1);
            hc = (j & 1) ? c0 + kFTW : c0 - 1;
        }
        double dh[4], rh[4];
        level_a(hr, hc, dh, rh);
    }
    __syncthreads();
    // level B on the tile's own cells
    auto level_b = [&](int vr, int vc, const double* dA, const double* rdA) {
        if (vr >= n || vc >= n) return;   // a tile past the grid's last row / column
        const int32_t k = vr * n + vc;
        const FStencilDev::Cell cl{{P.uface[k], P.vface[k]}};
        double acc[4], rdx[4];
        P.template rows4<false>(vr, vc, tt, xb, cl, acc, rdx);
        typename BS::Q q{};
        if constexpr (BS::on) q = bs.load(vr, vr, vc);
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            const double bf = BS::on ? bs.b(f, vr, vc, vc, tw, q) : a.b[f * nn + k];
            const double z = (bf - acc[f]) * rdA[f];
            const double dn = a.c1b * dA[f] + a.c2b * z;
            const int32_t o = f * nn + k;
            if constexpr (SD) a.d_out[o] = dn;
            const double x = xb.X(f, vr, vc) + dn;
            a.x_out[o] = SUB ? a.sub[o] - x : x;
        }
    };
    level_b(r0 + lr, c0 + lc, dA0, rd0);
    level_b(r0 + 4 + lr, c0 + lc, dA1, rd1);
}

template <bool INIT, bool SUB, bool SD, class BS>
int launch_ftile_t(const FStencilFast& P, const FTile& a, hipStream_t st, const BS& bs) {
    const int64_t tiles = (int64_t)((P.n + kFTW - 1) / kFTW) * ((P.n + kFTH - 1) / kFTH);
    if constexpr (!INIT && !BS::on) {
        if (a.xc) {
            k_ftile<INIT, SUB, SD, BS, true><<<(unsigned)tiles, 256, 0, st>>>(P, a, bs);
            MPBP_HIP(hipGetLastError());
            return MPBP_OK;
        }
    }
    k_ftile<INIT, SUB, SD, BS><<<(unsigned)tiles, 256, 0, st>>>(P, a, bs);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}
// INIT: level A = x0, level B = sweep 1 (the solve's first two updates); else sweeps s, s + 1.  One GPU, whole grid.
// Grids whose cells a tile and its staged halo wrap onto at most once each way.
inline bool ftile_ok(int n) { return n >= kFTW + kFTH + 4; }
template <bool INIT, class BS = BNone>
int launch_ftile(const FStencilDev& Pd, const FTile& a, hipStream_t st, const BS& bs = BS{}) {
    const FStencilFast P{Pd};
    if (P.h != 0 || P.which != 0 || !ftile_ok(P.n)) return set_error(MPBP_ERR_ARG, "ftile: one GPU, whole grid, n >= 76");
    if (!a.x_out || (!INIT && (!a.x_in || (!a.d_in && !a.dzero) || a.x_in == a.x_out)) || (!BS::on && !a.b) ||
        (a.d_out && (a.d_out == a.d_in || a.d_out == a.x_in)) || (a.xc && (INIT || BS::on || (P.n & 1))))
        return set_error(MPBP_ERR_ARG, "ftile: bad vectors");
    const bool sub = a.sub != nullptr, sd = a.d_out != nullptr;
    return sub ? (sd ? launch_ftile_t<INIT, true, true>(P, a, st, bs) : launch_ftile_t<INIT, true, false>(P, a, st, bs))
               : (sd ? launch_ftile_t<INIT, false, true>(P, a, st, bs) : launch_ftile_t<INIT, false, false>(P, a, st, bs));
}

// ---- a whole tolerance-mode F Chebyshev solve in one launch (k_fsolve) ----
// x = F^-1 b by K = H + 1 Chebyshev-Jacobi updates from x0 = 0 (the first is the pointwise x0 = d0 = c2_0 b / diag),
// on the 64 x 8 tiles of k_ftile: thn is staged over the tile plus H + 1 halo cells, level 0 builds x0 over the tile
// plus H, and level l = 1 .. H recomputes the tile plus H - l from level l - 1 (LDS ping-pong), the last writing x.
// Every cell a workgroup computes has one owning lane for all its levels: the lane's two tile cells (as k_ftile) and
// cell t of each halo ring r = 1 .. H (140 + 8 r cells, lane t < that), so its d, b, faces and reciprocal diagonals
// stay in that lane's registers from level 0 on.  Each level performs the IEEE operations of the marching kernels'
// tolerance-mode rows and updates: bit-identical to k_ftile<INIT> + k_ftile pair (H = 3) or + k_ftile sweep.  HBM:
// b (or x_p), thn, faces in, x out once -- against x, d, b re-read per launch by the two-launch solve.
template <int H>
struct FsTile {
    static constexpr int RW = kFTW + 2 * H, RH = kFTH + 2 * H, N = RW * RH;   // x levels: the tile + H
    static constexpr int TW = RW + 2, TH = RH + 2, TN = TW * TH;             // thn: the tile + H + 1
};
struct FSolve {
    const double* b;      // BNone: the right-hand side
    const double* sub;    // the result is sub - x when set
    double* x_out;
    double c2_0;
    double c1[4], c2[4];  // updates 1 .. H
};
// ring r's cell j: rows r0 - r and r0 + TH - 1 + r (all 64 + 2r columns), then columns c0 - r and c0 + TW - 1 + r of
// the rows between
__device__ inline void fs_ring_cell(int r, int j, int r0, int c0, int& vr, int& vc) {
    const int w = kFTW + 2 * r;
    if (j < 2 * w) {
        vr = j < w ? r0 - r : r0 + kFTH - 1 + r;
        vc = c0 - r + (j < w ? j : j - w);
    } else {
        const int k = j - 2 * w;
        vr = r0 - r + 1 + (k >> 1);
        vc = (k & 1) ? c0 + kFTW - 1 + r : c0 - r;
    }
}

// PART (row partition, the CA schedule): the tiles cover the owned rows and P.ext ghost rows each side; b and x are
// in the partition's ghost layout (P.xrow, P.out_row), the thn tables global.  Rows past b's ghost depth (padding of
// the last tile row and its halo, which no output reads) load a clamped row.
template <int H, bool SUB, bool PART, class BS>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 8))) MPBP_LDS_READS
k_fsolve(FStencilFast P, FSolve a, BS bs) {
    using T = FsTile<H>;
    constexpr int NT = 2;       // tile cells per lane
    constexpr int NSL = H + 2;  // owned cells per lane: the tile's two (rows lr, lr + 4), then ring r at slot 1 + r
    constexpr int NS = H + 1;   // ... with updates after x0 (ring H only needs x0)
    constexpr int PW = T::RW + 1, PN = PW * (T::RH + 1);   // BS: x_p over the tile + H, + its west / north neighbours
    __shared__ double ts[T::TN];
    __shared__ double xa[4 * T::N], xb[4 * T::N];
    __shared__ double ps[BS::on ? PN : 1];
    const int n = P.n, nn = n * n;
    const int tx = (n + kFTW - 1) / kFTW;
    const int bk = xcd_swizzle(blockIdx.x, gridDim.x);
    const int lo = PART ? P.r0 - P.ext : 0, hi = PART ? P.r0 + P.L + P.ext : n;   // output rows [lo, hi)
    const int r0 = lo + (bk / tx) * kFTH, c0 = (bk % tx) * kFTW;
    const int rbt = r0 - H - 1, cbt = c0 - H - 1, rb = r0 - H, cb = c0 - H;
    const int tid = threadIdx.x;
    // a row of the input layouts: the virtual row itself (one GPU: wrapped) or, clamped to the ghost depth, local
    auto in_row = [&](int vr, int h) {
        if constexpr (PART) {
            const int lr = vr - P.r0;
            return lr < -h ? -h : (lr >= P.L + h ? P.L + h - 1 : lr);
        } else {
            return P.wrap(vr);
        }
    };
    {
        constexpr int IT = (T::TN + 255) / 256;
        double v[IT];
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = tid + it * 256;
            if (i < T::TN) {
                const int sr = i / T::TW, sc = i - sr * T::TW;
                v[it] = P.cell[P.wrap(rbt + sr) * n + P.wrap(cbt + sc)];
            }
        }
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = tid + it * 256;
            if (i < T::TN) ts[i] = v[it];
        }
    }
    if constexpr (BS::on) {
        constexpr int IT = (PN + 255) / 256;
        double v[IT];
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = tid + it * 256;
            if (i < PN) {
                const int sr = i / PW, sc = i - sr * PW;
                const int pr = in_row(rb - 1 + sr, PART ? bs.h : 0);
                v[it] = bs.xp[(PART ? ext_row(1, 0, pr, P.L, bs.h, n) : pr * n) + P.wrap(cb - 1 + sc)];
            }
        }
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = tid + it * 256;
            if (i < PN) ps[i] = v[it];
        }
    }
    const int lr = tid >> 6, lc = tid & 63;
    // the owned cells and their rings (0: a tile cell; ring r lives through level H - r)
    int cr[NSL], cc[NSL], rr[NSL];
    bool own[NSL];
#pragma unroll
    for (int m = 0; m < NT; ++m) {
        cr[m] = r0 + lr + 4 * m; cc[m] = c0 + lc; own[m] = true; rr[m] = 0;
    }
#pragma unroll
    for (int r = 1; r <= H; ++r) {
        own[1 + r] = tid < 140 + 8 * r;
        rr[1 + r] = r;
        fs_ring_cell(r, own[1 + r] ? tid : 0, r0, c0, cr[1 + r], cc[1 + r]);
    }
    // every owned cell's faces and b (BNone) are loaded here, behind the staging loads and ahead of the barrier: one
    // global-memory latency for the whole level 0 instead of one per cell
    double fl[NSL][2], bl[BS::on ? 1 : NSL][4];
#pragma unroll
    for (int sl = 0; sl < NSL; ++sl) {
        if (!own[sl]) continue;
        const int gr = P.wrap(cr[sl]), gc = P.wrap(cc[sl]);
        const int32_t k = gr * n + gc;
        fl[sl][0] = P.uface[k];
        fl[sl][1] = P.vface[k];
        if constexpr (!BS::on) {
            const int br = in_row(cr[sl], P.h);
#pragma unroll
            for (int f = 0; f < 4; ++f) bl[sl][f] = a.b[(PART ? ext_row(4, f, br, P.L, P.h, n) : (f * n + br) * n) + gc];
        }
    }
    __syncthreads();
    const TTileT<T::TW> tt{ts, rbt, cbt};
    double d[NS][4], rd[NS][4], bv[NS][4], fc[NS][2];
    // level 0: x0 = d0 = c2_0 b / diag over the tile + H
#pragma unroll
    for (int sl = 0; sl < NSL; ++sl) {
        if (!own[sl]) continue;
        const int vr = cr[sl], vc = cc[sl];
        const int gr = P.wrap(vr), gc = P.wrap(vc);
        const FStencilDev::Stage sg{{fl[sl][0], fl[sl][1]}};
        double b4[4], r4[4];
        P.rdiag4(vr, vc, tt, sg, r4);
        if constexpr (BS::on) {   // b = G x_p, x_p and thn from LDS at virtual coordinates
            const int pi = (vr - rb + 1) * PW + (vc - cb + 1);
            const typename BS::Q q{ps[pi], ps[pi - 1], ps[pi - PW]};
#pragma unroll
            for (int f = 0; f < 4; ++f) b4[f] = bs.b_at(f, vr, vc, gc == 0, gr == 0, tt, q);
        } else {
#pragma unroll
            for (int f = 0; f < 4; ++f) b4[f] = bl[sl][f];
        }
        const int si = (vr - rb) * T::RW + (vc - cb);
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            const double x0 = a.c2_0 * b4[f] * r4[f];
            xa[f * T::N + si] = x0;
            if (sl < NS) {
                d[sl][f] = x0;
                rd[sl][f] = r4[f];
                bv[sl][f] = b4[f];
            }
        }
        if (sl < NS) {
            fc[sl][0] = sg.face[0];
            fc[sl][1] = sg.face[1];
        }
    }
    // levels 1 .. H
    double* cur = xa;
    double* nxt = xb;
    double sv[NT][4];   // SUB: the tile cells' sub entries, loaded at the start of level H (its stencil work hides them)
#pragma unroll
    for (int l = 1; l <= H; ++l) {
        __syncthreads();
        const XTileT<T::RW, T::RH> xt{cur, rb, cb};
        const double c1 = a.c1[l - 1], c2 = a.c2[l - 1];
        if constexpr (SUB) {
            if (l == H) {
#pragma unroll
                for (int m = 0; m < NT; ++m) {
                    const int vr = cr[m], vc = cc[m];
                    if (vr >= hi || vc >= n) continue;
#pragma unroll
                    for (int f = 0; f < 4; ++f)
                        sv[m][f] = a.sub[PART ? P.out_row(f, vr - P.r0, vc) : f * nn + vr * n + vc];
                }
            }
        }
#pragma unroll
        for (int sl = 0; sl < NS; ++sl) {
            if (sl >= NT && (!own[sl] || rr[sl] > H - l)) continue;   // ring r lives through level H - r
            const int vr = cr[sl], vc = cc[sl];
            if (l == H && (vr >= hi || vc >= n)) continue;            // a tile past the last row / column
            double acc[4], rdx[4];
            P.template rows4<false>(vr, vc, tt, xt, FStencilDev::Cell{{fc[sl][0], fc[sl][1]}}, acc, rdx);
            const int si = (vr - rb) * T::RW + (vc - cb);
#pragma unroll
            for (int f = 0; f < 4; ++f) {
                const double z = (bv[sl][f] - acc[f]) * rd[sl][f];
                const double dn = c1 * d[sl][f] + c2 * z;
                const double x = cur[f * T::N + si] + dn;
                if (l < H) {
                    nxt[f * T::N + si] = x;
                    d[sl][f] = dn;
                } else {
                    const int32_t o = PART ? P.out_row(f, vr - P.r0, vc) : f * nn + vr * n + vc;
                    if constexpr (SUB) a.x_out[o] = sv[sl < NT ? sl : 0][f] - x;   // (level H: tile cells only)
                    else a.x_out[o] = x;
                }
            }
        }
        double* t = cur;
        cur = nxt;
        nxt = t;
    }
}

// Grids a tile's staged thn (tile + H + 1 each side) wraps onto at most once.
template <int H>
inline bool fsolve_ok_n(int n) { return n >= FsTile<H>::TW && n >= FsTile<H>::TH; }
template <int H, bool PART, class BS>
int launch_fsolve_t(const FStencilFast& P, const FSolve& a, hipStream_t st, const BS& bs) {
    const int rows = PART ? P.L + 2 * P.ext : P.n;
    const int64_t tiles = (int64_t)((P.n + kFTW - 1) / kFTW) * ((rows + kFTH - 1) / kFTH);
    if (a.sub) k_fsolve<H, true, PART, BS><<<(unsigned)tiles, 256, 0, st>>>(P, a, bs);
    else k_fsolve<H, false, PART, BS><<<(unsigned)tiles, 256, 0, st>>>(P, a, bs);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}
// ---- k_fsolve on narrower tiles with the halo rings spread evenly over the waves (kernel option f_solve_tile) ----
// The same whole-solve launch as k_fsolve, the same operations per cell and level (bit-identical), on a TW x TH tile
// (32 x 16: 10 % fewer cell-levels than 64 x 8 -- 2 680 instead of 2 968 per 512 outputs at H = 3 -- because the
// halo rings are shorter).  A level's time is set by the wave with the most owned cells it updates, so ring r's cells
// are dealt out in four equal contiguous runs, one per wave: rings 1 .. H - 1 share one slot (lanes 0 .. 51 of every
// wave at 32 x 16, H = 3), ring H (x0 only) a second.  Per wave and level: x0 on 4 cells (k_fsolve 64 x 8: 5), then
// 3, 3, 2 stencil cells (4, 3, 2), and three cells' state in registers instead of four.  The level-invariant part of
// the rows is computed once: the node averages K(r, c) into an LDS table (FStencilFast::coeffs' kc / ks / ke are
// K(r, c), K(r + 1, c), K(r, c + 1), the same sums in the same order), and each owned cell keeps its XI couplings and
// identity weights in registers (in place of its two face values), so a level reads 6 coefficients instead of 8
// thn values and skips ~27 of the row's ~115 fp64 operations.  (An in-place variant -- one x image, a second barrier
// per level, 34 KB of LDS for three workgroups per CU -- spilled ~700 B per lane at the 168-VGPR cap and ran 4.5x
// slower: removed.)
template <int TW, int TH, int H>
struct FsGeom {
    static constexpr int RW = TW + 2 * H, RH = TH + 2 * H, N = RW * RH;   // x levels: the tile + H
    static constexpr int TSW = RW + 2, TSH = RH + 2, TSN = TSW * TSH;     // thn: the tile + H + 1
    static constexpr int NT = TW * TH / 256;                             // tile cells per lane
    static constexpr int ring(int r) { return 2 * TW + 2 * TH + 8 * r - 4; }
    static constexpr int q(int r) { return ring(r) / 4; }               // ring r's cells per wave
    static constexpr int qa() {                                          // slot A: rings 1 .. H - 1, per wave
        int s = 0;
        for (int r = 1; r < H; ++r) s += q(r);
        return s;
    }
};
template <int TW, int TH>
__device__ inline void fs_ring_cell_t(int r, int j, int r0, int c0, int& vr, int& vc) {
    const int w = TW + 2 * r;
    if (j < 2 * w) {
        vr = j < w ? r0 - r : r0 + TH - 1 + r;
        vc = c0 - r + (j < w ? j : j - w);
    } else {
        const int k = j - 2 * w;
        vr = r0 - r + 1 + (k >> 1);
        vc = (k & 1) ? c0 + TW - 1 + r : c0 - r;
    }
}
template <int TW, int TH, int H, bool SUB, bool PART, class BS>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 8))) MPBP_LDS_READS
k_fsolve_w(FStencilFast P, FSolve a, BS bs) {
    using T = FsGeom<TW, TH, H>;
    static_assert(TW * TH == 256 * T::NT && TW % 32 == 0, "whole rows of 32 lanes, NT cells per lane");
    static_assert((2 * TW + 2 * TH - 4) % 4 == 0, "every ring splits into four equal runs");
    static_assert(T::qa() <= 64 && T::q(H) <= 64, "one ring slot for rings 1 .. H - 1 and one for ring H");
    constexpr int NT = T::NT;
    constexpr int NSL = NT + 2;   // owned cells per lane: NT tile cells, slot A (rings 1 .. H - 1), slot B (ring H)
    constexpr int NS = NT + 1;    // ... with updates after x0 (ring H only needs x0)
    constexpr int PW = T::RW + 1, PN = PW * (T::RH + 1);   // BS: x_p over the tile + H, + its west / north neighbours
    constexpr int KW = T::RW + 1, KN = KW * (T::RH + 1);   // node averages K(r, c) of the tile + H, + 1 row / column
    __shared__ double ts[T::TSN];
    __shared__ double kt[KN];
    __shared__ double xa[4 * T::N], xb[4 * T::N];
    __shared__ double ps[BS::on ? PN : 1];
    const int n = P.n, nn = n * n;
    const int tx = (n + TW - 1) / TW;
    const int bk = xcd_swizzle(blockIdx.x, gridDim.x);
    const int lo = PART ? P.r0 - P.ext : 0, hi = PART ? P.r0 + P.L + P.ext : n;   // output rows [lo, hi)
    const int r0 = lo + (bk / tx) * TH, c0 = (bk % tx) * TW;
    const int rbt = r0 - H - 1, cbt = c0 - H - 1, rb = r0 - H, cb = c0 - H;
    const int tid = threadIdx.x;
    auto in_row = [&](int vr, int h) {
        if constexpr (PART) {
            const int lr = vr - P.r0;
            return lr < -h ? -h : (lr >= P.L + h ? P.L + h - 1 : lr);
        } else {
            return P.wrap(vr);
        }
    };
    {
        constexpr int IT = (T::TSN + 255) / 256;
        double v[IT];
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = tid + it * 256;
            if (i < T::TSN) {
                const int sr = i / T::TSW, sc = i - sr * T::TSW;
                v[it] = P.cell[P.wrap(rbt + sr) * n + P.wrap(cbt + sc)];
            }
        }
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = tid + it * 256;
            if (i < T::TSN) ts[i] = v[it];
        }
    }
    if constexpr (BS::on) {
        constexpr int IT = (PN + 255) / 256;
        double v[IT];
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = tid + it * 256;
            if (i < PN) {
                const int sr = i / PW, sc = i - sr * PW;
                const int pr = in_row(rb - 1 + sr, PART ? bs.h : 0);
                v[it] = bs.xp[(PART ? ext_row(1, 0, pr, P.L, bs.h, n) : pr * n) + P.wrap(cb - 1 + sc)];
            }
        }
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = tid + it * 256;
            if (i < PN) ps[i] = v[it];
        }
    }
    const int lane = tid & 63, wv = tid >> 6;
    int cr[NSL], cc[NSL], rr[NSL];
    bool own[NSL];
#pragma unroll
    for (int m = 0; m < NT; ++m) {   // tile cell m: row (tid / TW) + m (256 / TW), column tid % TW
        cr[m] = r0 + tid / TW + m * (256 / TW); cc[m] = c0 + tid % TW; own[m] = true; rr[m] = 0;
    }
    {   // slot A: rings 1 .. H - 1 in consecutive lane ranges; slot B: ring H
        int r = 0, j = 0, base = 0;
#pragma unroll
        for (int q = 1; q < H; ++q) {
            if (r == 0 && lane < base + T::q(q)) {
                r = q;
                j = wv * T::q(q) + lane - base;
            }
            base += T::q(q);
        }
        own[NT] = r != 0;
        rr[NT] = r;
        fs_ring_cell_t<TW, TH>(r ? r : 1, j, r0, c0, cr[NT], cc[NT]);
        own[NT + 1] = lane < T::q(H);
        rr[NT + 1] = H;
        fs_ring_cell_t<TW, TH>(H, own[NT + 1] ? wv * T::q(H) + lane : 0, r0, c0, cr[NT + 1], cc[NT + 1]);
    }
    double fl[NSL][2], bl[BS::on ? 1 : NSL][4];
#pragma unroll
    for (int sl = 0; sl < NSL; ++sl) {
        if (!own[sl]) continue;
        const int gr = P.wrap(cr[sl]), gc = P.wrap(cc[sl]);
        const int32_t k = gr * n + gc;
        fl[sl][0] = P.uface[k];
        fl[sl][1] = P.vface[k];
        if constexpr (!BS::on) {
            const int br = in_row(cr[sl], P.h);
#pragma unroll
            for (int f = 0; f < 4; ++f) bl[sl][f] = a.b[(PART ? ext_row(4, f, br, P.L, P.h, n) : (f * n + br) * n) + gc];
        }
    }
    __syncthreads();
    const TTileT<T::TSW> tt{ts, rbt, cbt};
    // the node averages every level reads (FStencilFast::coeffs' kc of cell (r, c), ks of (r - 1, c), ke of (r, c - 1):
    // the same sum in the same order), computed once; first read after level 1's barrier
    {
        constexpr int IK = (KN + 255) / 256;
#pragma unroll
        for (int it = 0; it < IK; ++it) {
            const int i = tid + it * 256;
            if (i < KN) {
                const int r = rb + i / KW, c = cb + i % KW;
                kt[i] = 0.25 * ((tt.T(0, r - 1, c - 1) + tt.T(0, r - 1, c)) + (tt.T(0, r, c - 1) + tt.T(0, r, c)));
            }
        }
    }
    // per owned cell: d, its reciprocal diagonals, b, and the level-invariant row terms (XI couplings xu / xv, weights)
    double d[NS][4], rd[NS][4], bv[NS][4], kx[NS][2];
    typename FStencilFast::W4 wt[NS];
    // level 0: x0 = d0 = c2_0 b / diag over the tile + H
#pragma unroll
    for (int sl = 0; sl < NSL; ++sl) {
        if (!own[sl]) continue;
        const int vr = cr[sl], vc = cc[sl];
        const int gr = P.wrap(vr), gc = P.wrap(vc);
        const FStencilDev::Cell cl{{fl[sl][0], fl[sl][1]}};
        const typename FStencilFast::Co k = P.coeffs(P.nb(tt, vr, vc));
        const typename FStencilFast::W4 w = P.weights(cl);
        double b4[4], r4[4];
        P.rdiag4_co(k, w, r4);
        if constexpr (BS::on) {
            const int pi = (vr - rb + 1) * PW + (vc - cb + 1);
            const typename BS::Q q{ps[pi], ps[pi - 1], ps[pi - PW]};
#pragma unroll
            for (int f = 0; f < 4; ++f) b4[f] = bs.b_at(f, vr, vc, gc == 0, gr == 0, tt, q);
        } else {
#pragma unroll
            for (int f = 0; f < 4; ++f) b4[f] = bl[sl][f];
        }
        const int si = (vr - rb) * T::RW + (vc - cb);
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            const double x0 = a.c2_0 * b4[f] * r4[f];
            xa[f * T::N + si] = x0;
            if (sl < NS) {
                d[sl][f] = x0;
                rd[sl][f] = r4[f];
                bv[sl][f] = b4[f];
            }
        }
        if (sl < NS) {
            kx[sl][0] = k.xu;
            kx[sl][1] = k.xv;
            wt[sl] = w;
        }
    }
    double* cur = xa;
    double* nxt = xb;
    double sv[NT][4];
#pragma unroll
    for (int l = 1; l <= H; ++l) {
        __syncthreads();
        const XTileT<T::RW, T::RH> xt{cur, rb, cb};
        const double c1 = a.c1[l - 1], c2 = a.c2[l - 1];
        if constexpr (SUB) {
            if (l == H) {
#pragma unroll
                for (int m = 0; m < NT; ++m) {
                    const int vr = cr[m], vc = cc[m];
                    if (vr >= hi || vc >= n) continue;
#pragma unroll
                    for (int f = 0; f < 4; ++f)
                        sv[m][f] = a.sub[PART ? P.out_row(f, vr - P.r0, vc) : f * nn + vr * n + vc];
                }
            }
        }
#pragma unroll
        for (int sl = 0; sl < NS; ++sl) {
            if (sl >= NT && (!own[sl] || rr[sl] > H - l)) continue;   // ring r lives through level H - r
            const int vr = cr[sl], vc = cc[sl];
            if (l == H && (vr >= hi || vc >= n)) continue;            // a tile past the last row / column
            typename FStencilFast::Co k;
            k.w = tt.T(0, vr, vc - 1);
            k.c = tt.T(0, vr, vc);
            k.nn = tt.T(0, vr - 1, vc);
            const int ki = (vr - rb) * KW + (vc - cb);
            k.kc = kt[ki];
            k.ks = kt[ki + KW];
            k.ke = kt[ki + 1];
            k.xu = kx[sl][0];
            k.xv = kx[sl][1];
            double acc[4];
            P.rows4_co(vr, vc, k, wt[sl], xt, acc);
            const int si = (vr - rb) * T::RW + (vc - cb);
#pragma unroll
            for (int f = 0; f < 4; ++f) {
                const double z = (bv[sl][f] - acc[f]) * rd[sl][f];
                const double dn = c1 * d[sl][f] + c2 * z;
                if (l < H) {
                    nxt[f * T::N + si] = cur[f * T::N + si] + dn;
                    d[sl][f] = dn;
                } else {
                    const double x = cur[f * T::N + si] + dn;
                    const int32_t o = PART ? P.out_row(f, vr - P.r0, vc) : f * nn + vr * n + vc;
                    if constexpr (SUB) a.x_out[o] = sv[sl < NT ? sl : 0][f] - x;
                    else a.x_out[o] = x;
                }
            }
        }
        double* t = cur;
        cur = nxt;
        nxt = t;
    }
}
// Grids the narrow tile's staged thn (tile + H + 1 each side) wraps onto at most once.
template <int TW, int TH, int H>
inline bool fsolve_w_ok_n(int n) { return n >= FsGeom<TW, TH, H>::TSW && n >= FsGeom<TW, TH, H>::TSH; }
template <int H, bool PART, class BS>
int launch_fsolve_w(const FStencilFast& P, const FSolve& a, hipStream_t st, const BS& bs) {
    constexpr int TW = 32, TH = 16;
    const int rows = PART ? P.L + 2 * P.ext : P.n;
    const int64_t tiles = (int64_t)((P.n + TW - 1) / TW) * ((rows + TH - 1) / TH);
    if (a.sub) k_fsolve_w<TW, TH, H, true, PART, BS><<<(unsigned)tiles, 256, 0, st>>>(P, a, bs);
    else k_fsolve_w<TW, TH, H, false, PART, BS><<<(unsigned)tiles, 256, 0, st>>>(P, a, bs);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

// K = 3 or 4 Chebyshev updates (x0 and H = K - 1 stencil sweeps); columns wrap at most once per tile.
inline bool fsolve_ok(int K, int n) { return (K == 3 && fsolve_ok_n<2>(n)) || (K == 4 && fsolve_ok_n<3>(n)); }
// One GPU, whole grid (P.h == 0), or a row partition's owned rows + P.ext ghost rows (P.which == 3), b's ghost depth
// P.h >= P.ext + H (+ 1 for x_p's with GxBPart).
template <class BS = BNone>
int launch_fsolve(const FStencilDev& Pd, int K, const double* c1, const double* c2, const double* b, const double* sub,
                  double* x_out, hipStream_t st, const BS& bs = BS{}) {
    const FStencilFast P{Pd};
    const bool part = P.h != 0;
    int xp_h = 0;   // x_p's ghost depth (GxBPart)
    if constexpr (BS::on) {
        if (BS::part != part) return set_error(MPBP_ERR_ARG, "fsolve: G x_p's layout does not match F's");
        if constexpr (BS::part) xp_h = bs.h;
    }
    if (!fsolve_ok(K, P.n) || (!part && P.which != 0) ||
        (part && (P.which != 3 || P.h < P.ext + K - 1 || P.oh < P.ext || (BS::on && xp_h < P.ext + K))))
        return set_error(MPBP_ERR_ARG, "fsolve: one GPU whole grid, or owned + ext rows with b ext + K - 1 deep");
    if (!x_out || (!BS::on && !b) || x_out == b) return set_error(MPBP_ERR_ARG, "fsolve: bad vectors");
    FSolve a{b, sub, x_out, c2[0], {}, {}};
    for (int l = 1; l < K; ++l) {
        a.c1[l - 1] = c1[l];
        a.c2[l - 1] = c2[l];
    }
    constexpr bool bpart = BS::on && BS::part;   // GxBPart launches only the partitioned kernel, GxB the other
    if (KO().f_solve_tile) {   // 32 x 16 tiles, rings spread over the waves, level-invariant terms cached
        if (!(K == 3 ? fsolve_w_ok_n<32, 16, 2>(P.n) : fsolve_w_ok_n<32, 16, 3>(P.n)))
            return set_error(MPBP_ERR_ARG, "fsolve: grid smaller than the 32 x 16 tile's staging");
        if constexpr (BS::on) {
            return K == 3 ? launch_fsolve_w<2, bpart>(P, a, st, bs) : launch_fsolve_w<3, bpart>(P, a, st, bs);
        } else {
            if (part) return K == 3 ? launch_fsolve_w<2, true>(P, a, st, bs) : launch_fsolve_w<3, true>(P, a, st, bs);
            return K == 3 ? launch_fsolve_w<2, false>(P, a, st, bs) : launch_fsolve_w<3, false>(P, a, st, bs);
        }
    }
    if constexpr (BS::on) {
        return K == 3 ? launch_fsolve_t<2, bpart>(P, a, st, bs) : launch_fsolve_t<3, bpart>(P, a, st, bs);
    } else {
        if (part) return K == 3 ? launch_fsolve_t<2, true>(P, a, st, bs) : launch_fsolve_t<3, true>(P, a, st, bs);
        return K == 3 ? launch_fsolve_t<2, false>(P, a, st, bs) : launch_fsolve_t<3, false>(P, a, st, bs);
    }
}

// Sweeps s, s+1 of an F Chebyshev solve fused (k_march2, tolerance mode) over the rows P.which selects (0: the whole
// grid, 3: owned + ext ghost rows; level A then covers ext + 1).  d_in may be d_out only when the pair does not store
// its direction (SD false): level A reads d_in on its neighbours' rows and columns.
template <bool SUB, bool SD, class BS>
int launch_march2_t(const FStencilFast& P, const Fused2& a, hipStream_t st, const BS& bs) {
    const int64_t chunks = march_chunks(P, KO().march_rows, march_capacity<k_march2<SUB, SD, BS>>());
    if (chunks == 0) return MPBP_OK;
    const int64_t strips = (P.n + kMB - 1) / kMB;
    k_march2<SUB, SD, BS><<<(unsigned)(chunks * strips), kMB, 0, st>>>(P, a, (int)chunks, bs);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}
template <class BS = BNone>
int launch_march2(const FStencilDev& Pd, const Fused2& a, hipStream_t st, const BS& bs = BS{}) {
    const FStencilFast P{Pd};
    if (P.which == 1 || P.which == 2) return set_error(MPBP_ERR_ARG, "march2: interior / boundary row splits unsupported");
    if (!a.x_in || !a.d_in || !a.x_out || a.x_in == a.x_out || (!BS::on && !a.b) || (a.d_out && a.d_out == a.d_in))
        return set_error(MPBP_ERR_ARG, "march2: bad vectors");
    const bool sub = a.sub != nullptr, sd = a.d_out != nullptr;
    return sub ? (sd ? launch_march2_t<true, true>(P, a, st, bs) : launch_march2_t<true, false>(P, a, st, bs))
               : (sd ? launch_march2_t<false, true>(P, a, st, bs) : launch_march2_t<false, false>(P, a, st, bs));
}

// The first inner sweep with x0 = c2 b / diag staged and diag rebuilt from thn (k_march_init).  BS = GxB: b is
// W = G x_p recomputed per point (the second F solve of the apply).
template <class S, class Epi, class BS = BNone>
int launch_march_init(const S& P, const double* b, double c2, Epi epi, int rows_per_block, hipStream_t st,
                      const BS& bs = BS{}) {
    auto go = [&](const auto& e) {
        using E = std::decay_t<decltype(e)>;
        const int64_t chunks = march_chunks(P, rows_per_block, march_capacity<k_march_init<S, E, BS>>());
        if (chunks == 0) return (int)MPBP_OK;
        const int64_t strips = (P.n + kMB - 1) / kMB;
        k_march_init<S, E, BS><<<(unsigned)(chunks * strips), kMB, 0, st>>>(P, b, c2, (int)chunks, e, bs);
        MPBP_HIP(hipGetLastError());
        return (int)MPBP_OK;
    };
    if constexpr (BS::on) return with_fixed_epi_bx<S::kFast>(epi, go);
    else return with_fixed_epi<S::kFast>(epi, go);
}

template <class S, class XS, class Epi, class BS = BNone>
int launch_march(const S& P, const XS& xs, Epi epi, int rows_per_block, hipStream_t st, const BS& bs = BS{}) {
    auto go = [&](const auto& e) { return launch_march_fixed(P, xs, e, rows_per_block, st, bs); };
    if constexpr (BS::on) return with_fixed_epi_bx<S::kFast>(epi, go);
    else return with_fixed_epi<S::kFast>(epi, go);
}

// F row of field f at a cell (k_march policy).
template <bool EDGE, class TA, class XA>
__device__ inline double FStencilDev::row(int f, int gr, int gc, const TA& ta, const XA& xa, double* fd,
                                          const Cell& cl) const {
    return f_row<EDGE>(*this, f, gr, gc, ta, xa, fd, cl.face);
}

// The F policy with the parameter identities of f_row's M compiled in (the reference's own parameters,
// d_u = -1 and eta_s = 1, solve.py:292-297 / apply.py:33-35): fewer fp64 multiplies per row, same bits.
template <int M>
struct FStencilDevM : FStencilDev {
    template <bool EDGE, class TA, class XA>
    __device__ double row(int f, int gr, int gc, const TA& ta, const XA& xa, double* fd, const Cell& cl) const {
        return f_row<EDGE, TA, XA, false, M>(*this, f, gr, gc, ta, xa, fd, cl.face);
    }
    template <class TA>
    __device__ double stage_diag(int f, int gr, int gc, const TA& ta, const Stage& s) const {
        return f_stage_diag<M>(*this, f, gr, gc, ta, s);
    }
};

// Calls fn with the F policy the plan's numerics select: the tolerance-mode rows (fast) or the bit-exact rows
// specialised for P's parameter identities.
template <class Fn>
int with_f_identities(const FStencilDev& P, Fn&& fn);
template <class Fn>
int with_f_policy(const FStencilDev& P, bool fast, Fn&& fn) {
    if (fast) return fn(FStencilFast{P});
    return with_f_identities(P, fn);
}

// Calls fn with the F policy specialised for P's parameters (M = 0: none apply).
template <class Fn>
int with_f_identities(const FStencilDev& P, Fn&& fn) {
    if (P.d_u == -1.0 && P.eta_s == 1.0) {
        if (P.eta_n != 1.0 && P.pow2 && P.ce0 != 0.0 && __builtin_isfinite(P.ce0)) return fn(FStencilDevM<13>{P});
        return P.eta_n == 1.0 ? fn(FStencilDevM<7>{P}) : fn(FStencilDevM<5>{P});
    }
    return fn(P);
}

// ------------------------------------------------------- matrix-free D, G, Gt_G ----
// The pressure-side operators rebuilt per row from the cell thn table: D (pressure rows, reading the 4
// velocity fields), G (velocity rows, reading pressure) and Gt_G = -(D G) (pressure rows), with the
// arithmetic of phase_D_row / phase_G_row (x d_p) / k_spgemm_fill (products accumulated in D's column
// order, then scaled by alpha = -1) and summed in CSR column order -- the assembled operators' results
// bit for bit.  Needs n >= 3 (distinct periodic neighbours).
struct PGDev {
    static constexpr bool kFast = false;
    int n;
    const double* cell;
    double d_p, inv, minv;   // d_p, 1.0 / dx, -1.0 / dx  (dx == dy; evaluated as the assembly does)
    // partition of the INPUT vector's grid rows, as FStencilDev (one GPU: r0 = 0, L = n, h = 0)
    int r0, L, h, which;
    int ext = 0;   // which = 3: ghost rows computed on each side
    int oh = 0;    // ghost depth of the output's layout (D: pressure, G: velocity, Gt_G: == h)
    int unit = 0;  // d_p == 1 and minv == -inv: Gt_G's eight products per phase are +-X^2 (GtGStencilDev::entries)
    __device__ int wrap(int a) const { return a < 0 ? a + n : (a >= n ? a - n : a); }
    template <int NFI>
    __device__ int32_t xrow_of(int f, int gr) const {
        if (h == 0) return (f * n + wrap(gr)) * n;
        return ext_row(NFI, f, gr - r0, L, h, n);
    }
    template <int NFO>
    __device__ int32_t out_of(int f, int lr, int gc) const {
        return (lr >= 0 && lr < L ? (f * L + lr) * n : ext_row(NFO, f, lr, L, oh, n)) + gc;
    }
};

// y = D x: pressure row (gr, gc) = sum over phases of the 4 velocity entries in column order.
struct DStencilDev : PGDev {
    struct Cell {};
    __device__ Cell cell_pre(int, int) const { return {}; }
    static constexpr int NF = 4, NOUT = 1;
    __device__ int32_t xrow(int f, int gr) const { return xrow_of<4>(f, gr); }
    __device__ int32_t out_row(int, int lr, int gc) const { return out_of<1>(0, lr, gc); }
    template <bool EDGE, class TA, class XA>
    __device__ double row(int, int gr, int gc, const TA& ta, const XA& xa, double* dg, const Cell&) const {
        const bool lastc = EDGE && gc == n - 1, lastr = EDGE && gr == n - 1;   // wrapped neighbour sorts first
        double acc = 0.0;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const double t0 = ta.T(p, gr, gc), tE = ta.T(p, gr, gc + 1), tW = ta.T(p, gr, gc - 1);
            const double tN = ta.T(p, gr - 1, gc), tS = ta.T(p, gr + 1, gc);
            const double uE = (inv * (0.5 * (t0 + tE))) * xa.X(2 * p, gr, gc + 1);
            const double uC = (minv * (0.5 * (t0 + tW))) * xa.X(2 * p, gr, gc);
            const double vC = (inv * (0.5 * (t0 + tN))) * xa.X(2 * p + 1, gr, gc);
            const double vS = (minv * (0.5 * (t0 + tS))) * xa.X(2 * p + 1, gr + 1, gc);
            acc += lastc ? uE : uC;
            acc += lastc ? uC : uE;
            acc += lastr ? vS : vC;
            acc += lastr ? vC : vS;
        }
        *dg = 0.0;
        return acc;
    }
};

// y = G x: velocity row o (u_n, v_n, u_s, v_s) at (gr, gc), two pressure entries in column order.
struct GStencilDev : PGDev {
    struct Cell {};
    __device__ Cell cell_pre(int, int) const { return {}; }
    static constexpr int NF = 1, NOUT = 4;
    __device__ int32_t xrow(int f, int gr) const { return xrow_of<1>(f, gr); }
    __device__ int32_t out_row(int f, int lr, int gc) const { return out_of<4>(f, lr, gc); }
    template <bool EDGE, class TA, class XA>
    __device__ double row(int o, int gr, int gc, const TA& ta, const XA& xa, double* dg, const Cell&) const {
        const int p = o >> 1;
        const double t0 = ta.T(p, gr, gc), xC = xa.X(0, gr, gc);
        double acc = 0.0;
        *dg = 0.0;
        if ((o & 1) == 0) {   // u row: entries p(gr, gc-1), p(gr, gc); the wrapped one sorts last
            const double gu = 0.5 * (t0 + ta.T(p, gr, gc - 1));
            const double uC = (d_p * (inv * gu)) * xC, uW = (d_p * (minv * gu)) * xa.X(0, gr, gc - 1);
            const bool wrapw = EDGE && gc == 0;
            acc += wrapw ? uC : uW;
            acc += wrapw ? uW : uC;
        } else {              // v row: entries p(gr-1, gc), p(gr, gc)
            const double gv = 0.5 * (t0 + ta.T(p, gr - 1, gc));
            const double vC = (d_p * (minv * gv)) * xC, vN = (d_p * (inv * gv)) * xa.X(0, gr - 1, gc);
            const bool wrapn = EDGE && gr == 0;
            acc += wrapn ? vC : vN;
            acc += wrapn ? vN : vC;
        }
        return acc;
    }
};

// Gt_G = -(D G): row (gr, gc) has the five entries N, W, C, E, S (grid neighbours).  Each off-diagonal
// gets one product per phase; the diagonal gets four per phase, accumulated in D's column order.
struct GtGStencilDev : PGDev {
    struct Cell {};
    __device__ Cell cell_pre(int, int) const { return {}; }
    static constexpr int NF = 1, NOUT = 1;
    __device__ int32_t xrow(int f, int gr) const { return xrow_of<1>(f, gr); }
    __device__ int32_t out_row(int, int lr, int gc) const { return out_of<1>(0, lr, gc); }
    // e = {N, W, C, E, S}.  (vr, vc): the cell in the accessor's coordinates (it may lie up to a few cells
    // outside the grid in the fused solve); (gr, gc): the same cell wrapped onto the grid.
    template <class TA>
    __device__ void entries(int vr, int vc, int gr, int gc, const TA& ta, double* e) const {
        const bool lastc = gc == n - 1, lastr = gr == n - 1;
        double cN = 0.0, cW = 0.0, cC = 0.0, cE = 0.0, cS = 0.0;
        if (unit) {
            // d_p == 1 and minv == -inv: with X = inv * (0.5 * (t0 + t_nb)) per face, every D entry is +-X and
            // every G factor d_p * (+-inv * g) is +-X too (g is the same half sum), so the eight products below
            // are +-X^2 -- the same roundings (RN(-a b) = -RN(a b)), same bits, 12 multiplies per phase, not 28
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                const double t0 = ta.T(p, vr, vc), tE = ta.T(p, vr, vc + 1), tW = ta.T(p, vr, vc - 1);
                const double tN = ta.T(p, vr - 1, vc), tS = ta.T(p, vr + 1, vc);
                const double XW = inv * (0.5 * (t0 + tW)), XE = inv * (0.5 * (t0 + tE));
                const double XN = inv * (0.5 * (t0 + tN)), XS = inv * (0.5 * (t0 + tS));
                const double qW = XW * XW, qE = XE * XE, qN = XN * XN, qS = XS * XS;
                // uC_C = -qW, uC_W = qW, uE_E = qE, uE_C = -qE, vC_C = -qN, vC_N = qN, vS_S = qS, vS_C = -qS
                const double u1 = lastc ? -qE : -qW, u2 = lastc ? -qW : -qE;
                const double v1 = lastr ? -qS : -qN, v2 = lastr ? -qN : -qS;
                if (p == 0) {
                    cC = u1; cW = qW; cE = qE; cN = qN; cS = qS;
                } else {
                    cC += u1; cW += qW; cE += qE; cN += qN; cS += qS;
                }
                cC += u2;
                cC += v1;
                cC += v2;
            }
            e[0] = -1.0 * cN; e[1] = -1.0 * cW; e[2] = -1.0 * cC; e[3] = -1.0 * cE; e[4] = -1.0 * cS;
            return;
        }
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const double t0 = ta.T(p, vr, vc), tE = ta.T(p, vr, vc + 1), tW = ta.T(p, vr, vc - 1);
            const double tN = ta.T(p, vr - 1, vc), tS = ta.T(p, vr + 1, vc);
            // D row entries (phase_D_row)
            const double DuE = inv * (0.5 * (t0 + tE)), DuC = minv * (0.5 * (t0 + tW));
            const double DvC = inv * (0.5 * (t0 + tN)), DvS = minv * (0.5 * (t0 + tS));
            // G rows of the velocity unknowns u(gr,gc), u(gr,gc+1), v(gr,gc), v(gr+1,gc) (phase_G_row x d_p)
            const double gC = 0.5 * (t0 + tW), gE = 0.5 * (tE + t0);
            const double gN = 0.5 * (t0 + tN), gS = 0.5 * (tS + t0);
            const double uC_C = DuC * (d_p * (inv * gC)), uC_W = DuC * (d_p * (minv * gC));
            const double uE_E = DuE * (d_p * (inv * gE)), uE_C = DuE * (d_p * (minv * gE));
            const double vC_C = DvC * (d_p * (minv * gN)), vC_N = DvC * (d_p * (inv * gN));
            const double vS_S = DvS * (d_p * (minv * gS)), vS_C = DvS * (d_p * (inv * gS));
            const double u1 = lastc ? uE_C : uC_C, u2 = lastc ? uC_C : uE_C;
            const double v1 = lastr ? vS_C : vC_C, v2 = lastr ? vC_C : vS_C;
            if (p == 0) {   // first touch stores the product itself (k_spgemm_fill)
                cC = u1; cW = uC_W; cE = uE_E; cN = vC_N; cS = vS_S;
            } else {
                cC += u1; cW += uC_W; cE += uE_E; cN += vC_N; cS += vS_S;
            }
            cC += u2;
            cC += v1;
            cC += v2;
        }
        e[0] = -1.0 * cN; e[1] = -1.0 * cW; e[2] = -1.0 * cC; e[3] = -1.0 * cE; e[4] = -1.0 * cS;
    }
    // Gt_G x at a cell: the five entries summed in CSR column order (EDGE: sorted by wrapped column)
    template <bool EDGE, class TA, class XA>
    __device__ double apply_v(int vr, int vc, int gr, int gc, const TA& ta, const XA& xa, double* dg) const {
        double e[5];
        entries(vr, vc, gr, gc, ta, e);
        *dg = e[2];
        const double p[5] = {e[0] * xa.X(0, vr - 1, vc), e[1] * xa.X(0, vr, vc - 1), e[2] * xa.X(0, vr, vc),
                             e[3] * xa.X(0, vr, vc + 1), e[4] * xa.X(0, vr + 1, vc)};
        return add5<EDGE>(0.0, p, Wrap{gr == 0, gr == n - 1, gc == 0, gc == n - 1});
    }
    template <bool EDGE, class TA, class XA>
    __device__ double row(int, int gr, int gc, const TA& ta, const XA& xa, double* dg, const Cell&) const {
        return apply_v<EDGE>(gr, gc, gr, gc, ta, xa, dg);
    }
};

// ---- one Gt_G Chebyshev solve in one launch (k_gtg_solve) ----
// The pressure solves x = Gt_G^-1 b of the apply (solve.py:265, 271) as K Chebyshev-Jacobi sweeps from x0 = 0, fused:
// a workgroup owns a TW x TH tile of cells and stages b and thn over the tile plus a halo of H = K - 1 cells, and
// x0 = d0 = c2_0 (b / diag) there from the stored diagonal (level 0).  Level l = 1 .. H recomputes the tile with halo
// H - l from level l - 1 (LDS ping-pong), the last writing the tile.  As in k_fsolve every cell has one owning lane for
// all its levels (the lane's two tile cells, and cell t of each halo ring r = 1 .. H - 1), which builds the cell's five
// entries once (GtGStencilDev::entries, from the staged thn) and keeps them, b and d in registers: a level reads only
// the five x values of the stencil from LDS.  Each row is GtGStencilDev::apply_v's IEEE operations (the entries', the
// products', add5's column order) and each update the Chebyshev epilogue's (EpiChebFirst at level 1, EpiCheb after):
// bit-identical to the K - 1 sweeps of the per-sweep path, for one launch and one pass over b instead of K - 1 passes
// over x, d, b.
constexpr int kGTW = kFTW, kGTH = kFTH;   // the 64 x 8 tile and ring numbering of k_fsolve (fs_ring_cell)
struct ChebK {
    double c1[8], c2[8];   // sweep s's coefficients (c2[0]: the initial iterate's)
};
template <int H, int GW = kGTW, int GH = kGTH>
struct GtgTile {   // a GW x GH tile of cells with H halo levels
    static constexpr int RW = GW + 2 * H, RH = GH + 2 * H, N = RW * RH;
    static constexpr int ring(int r) { return 2 * GW + 2 * GH - 4 + 8 * r; }   // cells of halo ring r
    static constexpr int rings(int h) { return h < 1 ? 0 : ring(h) + rings(h - 1); }
};
template <int H>
struct TTile {   // thn of the staged tile; (r, c) in the tile's virtual grid coordinates
    const double* t;
    int rb, cb;
    __device__ double T(int sph, int r, int c) const {
        const double v = t[(r - rb) * GtgTile<H>::RW + (c - cb)];
        return sph ? 1.0 - v : v;
    }
};

// PART: the tiles cover a row partition's owned rows and P.ext ghost rows each side (the CA schedule); b and diag in
// its ghost layout (depth P.h >= P.ext + H; deeper rows, read only for cells no output depends on, clamped), out in
// the output layout (depth P.oh).
// TPB = 512: one tile cell and at most one ring cell per lane (rings 1 .. H - 1 numbered across the workgroup), so a
// level's critical path is half as long and the smaller register state lets more waves share the CU.
// DB (one GPU): the right-hand side is rhs = D Y + v_p (solve.py:259), built at every staged cell with
// DStencilDev::row's operations and EpiAdd's sum from thn staged one cell wider and Y (the four velocity fields) from
// memory: the D launch, and rhs's write and re-read, disappear.
struct GtgD {
    const double* Y;    // Finv_v: u_n, v_n, u_s, v_s
    const double* vp;   // v's pressure part
};
template <int H, bool PART, int TPB, bool DB, int GW = kGTW, int GH = kGTH>
__global__ void __launch_bounds__(TPB) MPBP_LDS_READS k_gtg_solve(GtGStencilDev P, const double* __restrict__ b,
                                                   const double* __restrict__ diag, ChebK ck, double* __restrict__ out,
                                                   GtgD dv) {
    using G = GtgTile<H, GW, GH>;
    constexpr int SW = DB ? G::RW + 2 : G::RW, TN = DB ? SW * (G::RH + 2) : G::N;   // staged thn
    constexpr int NM = GW * GH / TPB;                // tile cells per lane
    constexpr int NR = TPB == 256 ? H - 1 : 1;       // ring slots per lane (rings 1 .. H - 1)
    constexpr int NS = NM + NR;
    static_assert(NM * TPB == GW * GH && TPB % GW == 0, "whole tile rows per lane group");
    static_assert(TPB == 512 || G::ring(H - 1) <= 256, "256 lanes own one cell of each ring");
    static_assert(TPB == 256 || G::rings(H - 1) <= 512, "512 lanes own at most one ring cell each");
    __shared__ double ts[TN], bs[G::N], xa[G::N], xb[G::N];
    const int n = P.n;
    const int tx = (n + GW - 1) / GW;
    const int bk = xcd_swizzle(blockIdx.x, gridDim.x);
    const int lo = PART ? P.r0 - P.ext : 0, hi = PART ? P.r0 + P.L + P.ext : n;   // output rows [lo, hi)
    const int r0 = lo + (bk / tx) * GH, c0 = (bk % tx) * GW;
    const int rb = r0 - H, cb = c0 - H;   // virtual coordinates of staged cell 0
    const int tid = threadIdx.x;
    // level 0 over the whole staged region: thn, b, x0 = c2_0 (b / diag); every load issued before the first LDS store
    if constexpr (DB) {
        const int nn = n * n;
        {   // thn one cell wider than the staged region
            constexpr int IT = (TN + TPB - 1) / TPB;
            double tv[IT];
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const int i = tid + it * TPB;
                if (i < TN) {
                    const int rr = i / SW, cc = i - rr * SW;
                    tv[it] = P.cell[P.wrap(rb - 1 + rr) * n + P.wrap(cb - 1 + cc)];
                }
            }
#pragma unroll
            for (int it = 0; it < IT; ++it)
                if (tid + it * TPB < TN) ts[tid + it * TPB] = tv[it];
        }
        // every staged cell's Y, v_p and diagonal loaded ahead of the barrier: one memory latency, not one per cell
        constexpr int IY = (G::N + TPB - 1) / TPB;
        double yl[IY][8], vpl[IY], dgl[IY];
#pragma unroll
        for (int it = 0; it < IY; ++it) {
            const int i = tid + it * TPB;
            if (i >= G::N) break;
            const int rr = i / G::RW, cc = i - rr * G::RW;
            const int gr = P.wrap(rb + rr), gc = P.wrap(cb + cc);
            const int ge = gc == n - 1 ? 0 : gc + 1, gs = gr == n - 1 ? 0 : gr + 1;
            const int32_t k = gr * n + gc;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                yl[it][4 * q + 0] = dv.Y[2 * q * nn + gr * n + ge];         // u at the east face
                yl[it][4 * q + 1] = dv.Y[2 * q * nn + k];                   // u at the cell's west face
                yl[it][4 * q + 2] = dv.Y[(2 * q + 1) * nn + k];             // v at its north face
                yl[it][4 * q + 3] = dv.Y[(2 * q + 1) * nn + gs * n + gc];   // v at the south face
            }
            vpl[it] = dv.vp[k];
            dgl[it] = diag[k];
        }
        __syncthreads();
        const TTileT<SW> tD{ts, rb - 1, cb - 1};
#pragma unroll
        for (int it = 0; it < IY; ++it) {
            const int i = tid + it * TPB;
            if (i >= G::N) break;
            const int rr = i / G::RW, cc = i - rr * G::RW;
            const int vr = rb + rr, vc = cb + cc, gr = P.wrap(vr), gc = P.wrap(vc);
            const double* yv = yl[it];
            const double vpk = vpl[it], dgk = dgl[it];
            const bool lastc = gc == n - 1, lastr = gr == n - 1;   // the wrapped neighbour sorts first (DStencilDev)
            double acc = 0.0;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const double t0 = tD.T(q, vr, vc), tE = tD.T(q, vr, vc + 1), tWv = tD.T(q, vr, vc - 1);
                const double tN = tD.T(q, vr - 1, vc), tS = tD.T(q, vr + 1, vc);
                const double uE = (P.inv * (0.5 * (t0 + tE))) * yv[4 * q + 0];
                const double uC = (P.minv * (0.5 * (t0 + tWv))) * yv[4 * q + 1];
                const double vC = (P.inv * (0.5 * (t0 + tN))) * yv[4 * q + 2];
                const double vS = (P.minv * (0.5 * (t0 + tS))) * yv[4 * q + 3];
                acc += lastc ? uE : uC;
                acc += lastc ? uC : uE;
                acc += lastr ? vS : vC;
                acc += lastr ? vC : vS;
            }
            const double bvv = acc + vpk;   // EpiAdd
            bs[i] = bvv;
            xa[i] = ck.c2[0] * (bvv / dgk);
        }
    } else {
        constexpr int IT = (G::N + TPB - 1) / TPB;
        double bv[IT], tv[IT], dv_[IT];
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = tid + it * TPB;
            if (i < G::N) {
                const int rr = i / G::RW, cc = i - rr * G::RW;
                const int gr = P.wrap(rb + rr), gc = P.wrap(cb + cc);
                int32_t kb = gr * n + gc;
                if constexpr (PART) {
                    int lr = rb + rr - P.r0;
                    lr = lr < -P.h ? -P.h : (lr >= P.L + P.h ? P.L + P.h - 1 : lr);
                    kb = ext_row(1, 0, lr, P.L, P.h, n) + gc;
                }
                bv[it] = b[kb];
                tv[it] = P.cell[gr * n + gc];
                dv_[it] = diag[kb];
            }
        }
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = tid + it * TPB;
            if (i < G::N) {
                ts[i] = tv[it];
                bs[i] = bv[it];
                xa[i] = ck.c2[0] * (bv[it] / dv_[it]);
            }
        }
    }
    __syncthreads();
    // the owned cells (slot 0, 1: the tile's; slot 1 + r: ring r), their entries, b and d0 = x0
    const TTileT<SW> ta{ts, DB ? rb - 1 : rb, DB ? cb - 1 : cb};
    const int lr = tid / GW, lc = tid % GW;
    int cr[NS], cc[NS], si[NS], rr[NS];
    bool own[NS], edge[NS];
    double e[NS][5], bo[NS], d[NS];
#pragma unroll
    for (int m = 0; m < NM; ++m) {
        cr[m] = r0 + lr + (TPB / GW) * m; cc[m] = c0 + lc; own[m] = true; rr[m] = 0;
    }
    if constexpr (TPB == 256) {
#pragma unroll
        for (int r = 1; r < H; ++r) {
            own[NM + r - 1] = tid < G::ring(r);
            rr[NM + r - 1] = r;
            fs_ring_cell_t<GW, GH>(r, own[NM + r - 1] ? tid : 0, r0, c0, cr[NM + r - 1], cc[NM + r - 1]);
        }
    } else if constexpr (NR > 0) {
        int r = 0, j = tid;   // rings 1 .. H - 1 numbered ring 1 first: lane t owns cell t of that sequence
#pragma unroll
        for (int q = 1; q < H; ++q)
            if (r == 0) {
                if (j < G::ring(q)) r = q;
                else j -= G::ring(q);
            }
        own[NM] = r != 0;
        rr[NM] = r;
        fs_ring_cell_t<GW, GH>(r ? r : 1, r ? j : 0, r0, c0, cr[NM], cc[NM]);
    }
#pragma unroll
    for (int sl = 0; sl < NS; ++sl) {
        const int vr = cr[sl], vc = cc[sl], gr = P.wrap(vr), gc = P.wrap(vc);
        si[sl] = (vr - rb) * G::RW + (vc - cb);
        edge[sl] = __builtin_amdgcn_readfirstlane(__any(own[sl] && (gr == 0 || gr == n - 1 || gc == 0 ||
                                                                    gc == n - 1))) != 0;
        if (own[sl]) {
            P.entries(vr, vc, gr, gc, ta, e[sl]);
            bo[sl] = bs[si[sl]];
            d[sl] = xa[si[sl]];
        }
    }
    double* cur = xa;
    double* nxt = xb;
#pragma unroll
    for (int l = 1; l <= H; ++l) {
        if (l > 1) __syncthreads();
        const double c1 = ck.c1[l], c2 = ck.c2[l];
#pragma unroll
        for (int sl = 0; sl < NS; ++sl) {
            if (TPB == 256 && sl >= NM && sl - NM + 1 > H - l) continue;   // (compile time) ring sl - NM + 1 is done
            if (sl >= NM && (!own[sl] || rr[sl] > H - l)) continue;        // ring rr lives through level H - rr
            const int vr = cr[sl], vc = cc[sl];
            if (l == H && (vr >= hi || vc >= n)) continue;            // a tile past the last row / column
            const int i = si[sl];
            const double p[5] = {e[sl][0] * cur[i - G::RW], e[sl][1] * cur[i - 1], e[sl][2] * cur[i],
                                 e[sl][3] * cur[i + 1], e[sl][4] * cur[i + G::RW]};
            const int gr = P.wrap(vr), gc = P.wrap(vc);
            const Wrap wr{gr == 0, gr == n - 1, gc == 0, gc == n - 1};
            const double acc = edge[sl] ? add5<true>(0.0, p, wr) : add5<false>(0.0, p, wr);
            const double z = (bo[sl] - acc) / e[sl][2];
            const double dn = c1 * d[sl] + c2 * z;
            const double x = cur[i] + dn;
            if (l < H) {
                nxt[i] = x;
                d[sl] = dn;
            } else {
                out[PART ? P.out_row(0, vr - P.r0, vc) : vr * n + vc] = x;
            }
        }
        double* t = cur;
        cur = nxt;
        nxt = t;
    }
}


// ---- multigrid level 0 of the pressure hierarchy (matrix-free Gt_G): descent and ascent in one launch each ----
// k_gpre: x0 = c2_0 (b / diag) over the tile + 3, the Chebyshev sweep x1 over the tile + 2 (written on the tile), the
// residual r = b - Gt_G x1 over the tile + 1 (in LDS) and R_0 r on the tile's 32 x 4 coarse cells (cell-centred both
// ways).  k_gpost: x = x_in + P_0 x_c staged over the tile + 2, two Chebyshev sweeps from d = +0.0 (the restart of the
// post-smoothing), the last writing the tile (sub - x when sub is set).  k_gtg_solve's 512-lane layout (one tile cell
// and at most one ring cell per lane, the cell's five entries built once from thn), its rows and updates, the
// transfers' k_mg_transfer_spmv lists and orders, EpiResid's and EpiAdd's sums: bit-identical to the launches they
// replace (the first / plain / zero-direction sweeps, the residual, the restriction, the prolongation).
template <int KY, int KX, int W>
__device__ inline double g1_rw(const double* tf, int cr, int cc, int n, int rb, int cb);
template <bool PRE, bool SUB>
__global__ void __launch_bounds__(512) MPBP_LDS_READS
k_gtg_level0(GtGStencilDev P, const double* __restrict__ b, const double* __restrict__ diag, const double* __restrict__ xin,
             const double* __restrict__ xc, const double* __restrict__ sub, ChebK ck, double* __restrict__ x_out,
             double* __restrict__ bc) {
    constexpr int H = PRE ? 3 : 2;   // staged halo: the tile + H
    using G = GtgTile<H>;
    constexpr int CW = kGTW / 2 + 4, CH = kGTH / 2 + 4, CN = CW * CH;   // k_gpost's coarse window (k_gal1's geometry)
    static_assert(CW == kG1CW, "g1_p_in's window stride");
    __shared__ double ts[G::N], bs[G::N], xa[G::N], xb[G::N];
    __shared__ double cs[PRE ? 1 : CN];
    const int n = P.n, nc = n >> 1;
    const int tx = (n + kGTW - 1) / kGTW;
    const int bk = xcd_swizzle(blockIdx.x, gridDim.x);
    const int r0 = (bk / tx) * kGTH, c0 = (bk % tx) * kGTW;
    const int rb = r0 - H, cb = c0 - H;
    const int cr0 = r0 >> 1, cc0 = c0 >> 1;
    const int tid = threadIdx.x;
    auto wrapc = [&](int q) { return q < 0 ? q + nc : (q >= nc ? q - nc : q); };
    {
        constexpr int IT = (G::N + 511) / 512, IC = PRE ? 1 : (CN + 511) / 512;
        double bv[IT], tv[IT], wv[IT], cv[IC];
        if constexpr (!PRE) {
#pragma unroll
            for (int it = 0; it < IC; ++it) {
                const int i = tid + it * 512;
                if (i < CN) {
                    const int r = i / CW, c = i - r * CW;
                    cv[it] = xc[wrapc(cr0 - 2 + r) * nc + wrapc(cc0 - 2 + c)];
                }
            }
        }
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = tid + it * 512;
            if (i < G::N) {
                const int rr = i / G::RW, cc = i - rr * G::RW;
                const int32_t k = P.wrap(rb + rr) * n + P.wrap(cb + cc);
                bv[it] = b[k];
                tv[it] = P.cell[k];
                wv[it] = PRE ? diag[k] : xin[k];
            }
        }
        if constexpr (!PRE) {
#pragma unroll
            for (int it = 0; it < IC; ++it)
                if (tid + it * 512 < CN) cs[tid + it * 512] = cv[it];
            __syncthreads();
        }
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = tid + it * 512;
            if (i < G::N) {
                ts[i] = tv[it];
                bs[i] = bv[it];
                if constexpr (PRE) {
                    xa[i] = ck.c2[0] * (bv[it] / wv[it]);   // x0 (k_cheb_init's expression, XInit's)
                } else {                                     // x_in + P_0 x_c (the prolongation's sum)
                    const int rr = i / G::RW, cc = i - rr * G::RW;
                    const double pc = g1_inner(cr0, cc0, kGTH / 2, kGTW / 2, nc)
                                          ? g1_p_in<MPBP_MG_CELL, MPBP_MG_CELL>(cs, rr, cc)
                                          : g1_p<MPBP_MG_CELL, MPBP_MG_CELL>(cs, P.wrap(rb + rr), P.wrap(cb + cc), nc,
                                                                             cr0 - 2, cc0 - 2);
                    xa[i] = pc + wv[it];
                }
            }
        }
    }
    __syncthreads();
    const TTileT<G::RW> ta{ts, rb, cb};
    const int lr = tid >> 6, lc = tid & 63;
    // slot 0: the tile cell; slot 1: ring cell t of rings 1 .. H - 1 numbered ring 1 first
    int cr[2], cc[2], si[2], rr[2];
    bool own[2], edge[2];
    double e[2][5], bo[2], d[2];
    cr[0] = r0 + lr; cc[0] = c0 + lc; own[0] = true; rr[0] = 0;
    {
        int r = 0, j = tid;
#pragma unroll
        for (int q = 1; q < H; ++q)
            if (r == 0) {
                if (j < 140 + 8 * q) r = q;
                else j -= 140 + 8 * q;
            }
        own[1] = r != 0;
        rr[1] = r;
        fs_ring_cell(r ? r : 1, r ? j : 0, r0, c0, cr[1], cc[1]);
    }
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
        const int vr = cr[sl], vc = cc[sl], gr = P.wrap(vr), gc = P.wrap(vc);
        si[sl] = (vr - rb) * G::RW + (vc - cb);
        edge[sl] = __builtin_amdgcn_readfirstlane(__any(own[sl] && (gr == 0 || gr == n - 1 || gc == 0 ||
                                                                    gc == n - 1))) != 0;
        if (own[sl]) {
            P.entries(vr, vc, gr, gc, ta, e[sl]);
            bo[sl] = bs[si[sl]];
            d[sl] = PRE ? xa[si[sl]] : 0.0;   // PRE: d0 = x0; post: the restart's +0.0
        }
    }
    double* cur = xa;
    double* nxt = xb;
    constexpr int L = PRE ? 2 : 2;   // PRE: the sweep, then the residual; post: two sweeps
#pragma unroll
    for (int l = 1; l <= L; ++l) {
        if (l > 1) __syncthreads();
        const double c1 = ck.c1[l], c2 = ck.c2[l];
#pragma unroll
        for (int sl = 0; sl < 2; ++sl) {
            // PRE: ring rr lives through level 3 - rr (the residual at level 2 covers the tile + 1); post: 2 - rr
            if (sl == 1 && (!own[1] || rr[1] > (PRE ? 3 : 2) - l)) continue;
            const int vr = cr[sl], vc = cc[sl];
            const int i = si[sl];
            const double p[5] = {e[sl][0] * cur[i - G::RW], e[sl][1] * cur[i - 1], e[sl][2] * cur[i],
                                 e[sl][3] * cur[i + 1], e[sl][4] * cur[i + G::RW]};
            const int gr = P.wrap(vr), gc = P.wrap(vc);
            const Wrap wr{gr == 0, gr == n - 1, gc == 0, gc == n - 1};
            const double acc = edge[sl] ? add5<true>(0.0, p, wr) : add5<false>(0.0, p, wr);
            if (PRE && l == 2) {   // the residual (EpiResid)
                nxt[i] = bo[sl] - acc;
                continue;
            }
            const double z = (bo[sl] - acc) / e[sl][2];
            const double dn = c1 * d[sl] + c2 * z;
            const double x = cur[i] + dn;
            nxt[i] = x;
            d[sl] = dn;
            const bool out = PRE ? (l == 1) : (l == L);
            if (sl == 0 && out && vr < n && vc < n) {
                const int32_t o = vr * n + vc;
                x_out[o] = (SUB && !PRE) ? sub[o] - x : x;
            }
        }
        double* t = cur;
        cur = nxt;
        nxt = t;
    }
    if constexpr (PRE) {   // R_0 r on the tile's coarse cells (cur holds r over the tile + 1)
        __syncthreads();
        constexpr int CTW = kGTW / 2, CTH = kGTH / 2;   // the tile's coarse cells
        if (tid < CTW * CTH) {
            const int crr = cr0 + tid / CTW, ccc = cc0 + tid % CTW;
            if (crr < nc && ccc < nc)
                bc[crr * nc + ccc] = g1_inner(cr0, cc0, CTH, CTW, nc)
                                         ? g1_rw_in<MPBP_MG_CELL, MPBP_MG_CELL, G::RW, 2>(cur, crr - cr0, ccc - cc0)
                                         : g1_rw<MPBP_MG_CELL, MPBP_MG_CELL, G::RW>(cur, crr, ccc, n, rb, cb);
        }
    }
}

// ---- multigrid level 1 of a tolerance-mode F hierarchy in one launch (k_gal1) ----
// A_1 x = R_0 (F (P_0 x)) (MgGal) with the two fine-size intermediates kept in LDS: a workgroup owns a 16 x 8 tile of
// coarse cells (a 32 x 16 fine block; kGF* below), stages the coarse x of its four fields over the tile + 2 and thn
// over the fine block + 2, builds t0 = P_0 x on the fine block + 2 (36 x 20), t1 = F t0 on the fine block + 1 (34 x 18,
// the tolerance-mode rows), and R_0 t1 on its coarse rows, handing each to the level's epilogue.  Each value is built
// by the operations of the three launches it replaces (k_mg_transfer_spmv's 1D lists and product order,
// FStencilFast::rows4), so the result is bit-identical; HBM: x, thn and the epilogue operands once, no fine vector
// written or read.  (The 32 x 4 tile of kG1* above -- the level-0 fused kernels' coarse windows -- took 42 KB of LDS,
// three workgroups per CU: 33.1 vs 28.5 us per launch, profiles/r06s_ab_gal1_tile.txt.)
// a grid index to its slot in a staged window starting at virtual index `base` (the window is < the grid)
__device__ inline int g1_slot(int i, int base, int m) { int l = i - base; return l < 0 ? l + m : (l >= m ? l - m : l); }
// P_0's row at fine (gr, gc) of a field with compile-time kinds: k_mg_transfer_spmv's list order and products
// (S: the coarse window's row stride)
template <int KY, int KX, int S>
__device__ inline double g1_p(const double* xf, int gr, int gc, int nc, int rb, int cb) {
    int yi[2], xi[2];
    double yw[2], xw[2];
    const int my = mg_p1d_fast(KY, nc, gr, yi, yw), mx = mg_p1d_fast(KX, nc, gc, xi, xw);
    double acc = 0.0;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        if (a >= my) break;
        const double* xr = xf + g1_slot(yi[a], rb, nc) * S;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            if (b >= mx) break;
            acc += (yw[a] * xw[b]) * xr[g1_slot(xi[b], cb, nc)];
        }
    }
    return acc;
}
// R_0's row at coarse (cr, cc): 4 (cell) x 3 or 4 entries, compile-time counts (S: the fine window's row stride)
template <int KY, int KX, int S = kG1FW>
__device__ inline double g1_r(const double* tf, int cr, int cc, int n, int rb, int cb) {
    constexpr int MY = KY == MPBP_MG_CELL ? 4 : 3, MX = KX == MPBP_MG_CELL ? 4 : 3;
    int yi[4], xi[4];
    double yw[4], xw[4];
    mg_r1d_fast(KY, n, cr, yi, yw);
    mg_r1d_fast(KX, n, cc, xi, xw);
    double acc = 0.0;
#pragma unroll
    for (int a = 0; a < MY; ++a) {
        const double* tr1 = tf + g1_slot(yi[a], rb, n) * S;
#pragma unroll
        for (int b = 0; b < MX; ++b) acc += (yw[a] * xw[b]) * tr1[g1_slot(xi[b], cb, n)];
    }
    return acc;
}
// Interior tiles (no staged window wraps and no 1D list takes its periodic special case): P_0's and R_0's rows in
// window coordinates straight from the fine / coarse parity -- the same entries, weights, order and products as
// mg_p1d_fast / mg_r1d_fast give there, without their wrap tests, sorted-order selects and runtime weights.  A node
// kind's one-entry row (even fine index) takes a second entry of weight 0: its products are +-0 added to a sum that
// started from +0.0 (never -0.0), so the sum's bits are unchanged for finite x.  With t1 in t0's LDS (occupancy 2 -> 3
// workgroups per CU): k_gal1 45 -> 33 us, multigrid apply 1.610 -> 1.510 ms (A/B on one box, profiles/r05zd_ab.txt).
template <int K>
__device__ inline void g1_p1d_in(int r, int& lo, double& w0, double& w1) {
    const bool odd = r & 1;
    if constexpr (K == MPBP_MG_CELL) {   // even: c_{i-1} (1/4), c_i (3/4); odd: c_i (3/4), c_{i+1} (1/4)
        lo = (r >> 1) + (odd ? 1 : 0);
        w0 = odd ? 0.75 : 0.25;
        w1 = odd ? 0.25 : 0.75;
    } else {                             // even: c_i (1); odd: c_i, c_{i+1} (1/2 each)
        lo = (r >> 1) + 1;
        w0 = odd ? 0.5 : 1.0;
        w1 = odd ? 0.5 : 0.0;
    }
}
// P_0's row at window fine (r, c) of the block + 2 (the coarse window starts two coarse cells before the tile)
template <int KY, int KX, int S>
__device__ inline double g1_p_in(const double* xf, int r, int c) {
    int ry, cx;
    double y0, y1, x0, x1;
    g1_p1d_in<KY>(r, ry, y0, y1);
    g1_p1d_in<KX>(c, cx, x0, x1);
    const double* q = xf + ry * S + cx;
    double acc = 0.0;
    acc += (y0 * x0) * q[0];
    acc += (y0 * x1) * q[1];
    acc += (y1 * x0) * q[S];
    acc += (y1 * x1) * q[S + 1];
    return acc;
}
// R_0's row at tile coarse (lr, lc) over a fine window of row stride W whose slot OFF holds fine index 2 c0 - 1 (the
// tile's first coarse cell's first restriction entry): 2 lr + OFF + 0 .. 3 (cell) / 0 .. 2 (node)
template <int KY, int KX, int W, int OFF>
__device__ inline double g1_rw_in(const double* tf, int lr, int lc) {
    constexpr int MY = KY == MPBP_MG_CELL ? 4 : 3, MX = KX == MPBP_MG_CELL ? 4 : 3;
    constexpr double WC[4] = {0.25, 0.75, 0.75, 0.25}, WN[3] = {0.5, 1.0, 0.5};
    const double* q = tf + (2 * lr + OFF) * W + 2 * lc + OFF;
    double acc = 0.0;
#pragma unroll
    for (int a = 0; a < MY; ++a)
#pragma unroll
        for (int b = 0; b < MX; ++b)
            acc += ((KY == MPBP_MG_CELL ? WC[a] : WN[a]) * (KX == MPBP_MG_CELL ? WC[b] : WN[b])) * q[a * W + b];
    return acc;
}
// ... over t1's window (fine block + 1)
template <int KY, int KX, int S = kG1FW>
__device__ inline double g1_r_in(const double* tf, int lr, int lc) { return g1_rw_in<KY, KX, S, 0>(tf, lr, lc); }
// a tile whose transfers' windows neither wrap nor reach a 1D list's periodic special case (coarse tile of TH x TW
// cells at (cr0, cc0), windows two coarse cells beyond it)
__device__ inline bool g1_inner(int cr0, int cc0, int th, int tw, int nc) {
    return cr0 >= 2 && cr0 + th + 2 <= nc && cc0 >= 2 && cc0 + tw + 2 <= nc;
}
// Level 1 under a row partition (PART): this rank owns coarse rows [r0, r0 + L) of every field and its level-1 vectors
// hold them followed by h ghost rows above and below (ext_row's layout).  The tiles cover the owned rows only; every
// value is computed in global coordinates exactly as on one GPU (the same windows, lists and rows), so the rank's rows
// are the one-GPU launch's bits.
struct G1Part {
    int r0 = 0, L = 0, h = 0;
};
// level-1 x index of (field f, coarse row gr -- unwrapped, within two rows of the tile --, wrapped column c); window
// rows past the ghosts (a partial last tile's) are clamped: they feed only outputs the tile does not own
template <bool PART>
__device__ inline int32_t g1_xidx(const G1Part& q, int nf, int f, int gr, int c, int nc) {
    if constexpr (!PART) {
        (void)q; (void)nf;
        return (f * nc + (gr < 0 ? gr + nc : (gr >= nc ? gr - nc : gr))) * nc + c;
    } else {
        const int lr = min(max(gr - q.r0, -q.h), q.L + q.h - 1);
        return ext_row(nf, f, lr, q.L, q.h, nc) + c;
    }
}
// the level-1 row of an owned output (f, cr, cc)
template <bool PART>
__device__ inline int32_t g1_orow(const G1Part& q, int f, int cr, int cc, int nc) {
    return PART ? (f * q.L + cr - q.r0) * nc + cc : (f * nc + cr) * nc + cc;
}
// PRO (the post-smoothing's first sweep after level 2's correction): the staged x is x + P_1 x_c, level 2's window
// [cr0 / 2 - 2, cr0 / 2 + kGFQH - 2) x [cc0 / 2 - 2, cc0 / 2 + kGFQW - 2) staged first (k_ftile<PRO>'s scheme one level
// down: the same P rows in window coordinates, k_mg_transfer_spmv's lists and EpiAdd's sum), and the epilogue's iterate
// is the row's own staged value -- the prolongation launch folded in, bit-identical.
// k_gal1's own tile: 16 x 8 coarse cells (a 32 x 16 fine block) -- its windows and t0 take 36.5 KB of LDS, so four
// workgroups share a CU (the 32 x 4 tile's 42 KB held three), and F's rows on the block + 1 are 612 instead of 660
constexpr int kGFW = 16, kGFH = 8;
constexpr int kGFCW = kGFW + 4, kGFCH = kGFH + 4;               // coarse x: [c0 - 2, c0 + W + 2)
constexpr int kGFFW = 2 * kGFW + 2, kGFFH = 2 * kGFH + 2;       // t1: fine block + 1
constexpr int kGFPW = kGFFW + 2, kGFPH = kGFFH + 2;             // t0 and thn: fine block + 2
constexpr int kGFQW = kGFW / 2 + 4, kGFQH = kGFH / 2 + 4;       // PRO: level 2's window (row stride kGFQW)
constexpr int kG1QW = kG1W / 2 + 4;                             // (k_gal1p's level-2 window columns)
template <bool INNER, class Epi, bool MAC, class XS, bool PART, bool PRO>
__device__ __forceinline__ void gal1_run(const FStencilFast& P, const MgFields& tr, const XS& xin, const Epi& epi,
                                         double* xs, double* ts, double* t0, double* t1, int cr0, int cc0,
                                         const G1Part& q, const double* xc, double* xq);
// MAC: the F hierarchy's kinds (u: rows cell-, columns node-centred; v: the reverse) at compile time
// XS: the coarse x as staged -- XPlain (x itself) or XInit (x0 = c2_0 (b / diag): a pre-smoothing's first sweep with the
// init pass folded in, as the grouped small levels do; the epilogue then EpiChebFirstGrp)
template <class Epi, bool MAC = false, class XS = XPlain, bool PART = false, bool PRO = false>
__global__ void __launch_bounds__(256) MPBP_LDS_READS k_gal1(FStencilFast P, MgFields tr, XS xin, Epi epi, G1Part q,
                                                              const double* __restrict__ xc = nullptr) {
    constexpr int CN = kGFCW * kGFCH, PN = kGFPW * kGFPH, FN = kGFFW * kGFFH;
    static_assert(!PRO || (MAC && !PART), "the folded prolongation: MAC kinds, whole level");
    __shared__ double xs[4 * CN];
    __shared__ double ts[PN];
    __shared__ double t0[4 * PN];
    __shared__ double xq[PRO ? 4 * kGFQW * kGFQH : 1];
    double* t1 = t0;
    static_assert(FN <= PN, "t1 fits t0");
    const int nc = P.n >> 1;
    const int tx = (nc + kGFW - 1) / kGFW;
    const int bk = xcd_swizzle(blockIdx.x, gridDim.x);
    const int cr0 = (PART ? q.r0 : 0) + (bk / tx) * kGFH, cc0 = (bk % tx) * kGFW;     // the coarse tile
    if constexpr (MAC) {
        if (g1_inner(cr0, cc0, kGFH, kGFW, nc)) {
            gal1_run<true, Epi, MAC, XS, PART, PRO>(P, tr, xin, epi, xs, ts, t0, t1, cr0, cc0, q, xc, xq);
            return;
        }
    }
    gal1_run<false, Epi, MAC, XS, PART, PRO>(P, tr, xin, epi, xs, ts, t0, t1, cr0, cc0, q, xc, xq);
}
template <bool INNER, class Epi, bool MAC, class XS, bool PART, bool PRO>
__device__ __forceinline__ void gal1_run(const FStencilFast& P, const MgFields& tr, const XS& xin, const Epi& epi,
                                         double* xs, double* ts, double* t0, double* t1, int cr0, int cc0,
                                         const G1Part& q, const double* xc, double* xq) {
    constexpr int CN = kGFCW * kGFCH, PN = kGFPW * kGFPH, FN = kGFFW * kGFFH;
    const int n = P.n, nc = n >> 1;
    const int fr0 = 2 * cr0, fc0 = 2 * cc0;                      // its fine block
    const int tid = threadIdx.x;
    auto wrapc = [&](int a) { return a < 0 ? a + nc : (a >= nc ? a - nc : a); };
    // a grid index to its slot in a staged window starting at virtual index `base` (the window is < the grid)
    auto slot = [](int i, int base, int m) { int l = i - base; return l < 0 ? l + m : (l >= m ? l - m : l); };
    {   // stage the coarse x (4 fields) and thn, every load before the first LDS store
        constexpr int IX = (4 * CN + 255) / 256, IT = (PN + 255) / 256;
        typename XS::Raw vx[IX];
        double vt[IT];
#pragma unroll
        for (int it = 0; it < IX; ++it) {
            const int i = tid + it * 256;
            if (i < 4 * CN) {
                const int f = i / CN, j = i - f * CN, r = j / kGFCW, c = j - r * kGFCW;
                vx[it] = xin.load(g1_xidx<PART>(q, 4, f, cr0 - 2 + r, wrapc(cc0 - 2 + c), nc));
            }
        }
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = tid + it * 256;
            if (i < PN) {
                const int r = i / kGFPW, c = i - r * kGFPW;
                vt[it] = P.cell[P.wrap(fr0 - 2 + r) * n + P.wrap(fc0 - 2 + c)];
            }
        }
        const int n2 = nc >> 1;
        if constexpr (PRO) {   // level 2's window first: the staged x needs it
            auto wrap2 = [&](int a) { return a < 0 ? a + n2 : (a >= n2 ? a - n2 : a); };
            constexpr int QF = kGFQW * kGFQH, IQ = (4 * QF + 255) / 256;
            double vq[IQ];
#pragma unroll
            for (int it = 0; it < IQ; ++it) {
                const int i = tid + it * 256;
                if (i < 4 * QF) {
                    const int f = i / QF, j = i - f * QF, r = j / kGFQW, c = j - r * kGFQW;
                    vq[it] = xc[(f * n2 + wrap2((cr0 >> 1) - 2 + r)) * n2 + wrap2((cc0 >> 1) - 2 + c)];
                }
            }
#pragma unroll
            for (int it = 0; it < IQ; ++it) {
                const int i = tid + it * 256;
                if (i < 4 * QF) {
                    const int f = i / QF, j = i - f * QF, r = j / kGFQW, c = j - r * kGFQW;
                    xq[(f * kGFQH + r) * kGFQW + c] = vq[it];
                }
            }
            __syncthreads();
        }
        const bool inner2 = PRO && g1_inner(cr0 >> 1, cc0 >> 1, kGFH / 2, kGFW / 2, n2);
#pragma unroll
        for (int it = 0; it < IX; ++it) {
            const int i = tid + it * 256;
            if (i >= 4 * CN) continue;
            double v = xin.value(vx[it]);
            if constexpr (PRO) {   // x + P_1 x_c (EpiAdd: the row sum, then + x)
                const int f = i / CN, j = i - f * CN, r = j / kGFCW, c = j - r * kGFCW;
                const double* xf = xq + f * kGFQH * kGFQW;
                const int gr = wrapc(cr0 - 2 + r), gc = wrapc(cc0 - 2 + c), rb = (cr0 >> 1) - 2, cb = (cc0 >> 1) - 2;
                const double pc = inner2 ? ((f & 1) ? g1_p_in<MPBP_MG_NODE, MPBP_MG_CELL, kGFQW>(xf, r, c)
                                                    : g1_p_in<MPBP_MG_CELL, MPBP_MG_NODE, kGFQW>(xf, r, c))
                                         : ((f & 1) ? g1_p<MPBP_MG_NODE, MPBP_MG_CELL, kGFQW>(xf, gr, gc, n2, rb, cb)
                                                    : g1_p<MPBP_MG_CELL, MPBP_MG_NODE, kGFQW>(xf, gr, gc, n2, rb, cb));
                v = pc + v;
            }
            xs[i] = v;
        }
#pragma unroll
        for (int it = 0; it < IT; ++it)
            if (tid + it * 256 < PN) ts[tid + it * 256] = vt[it];
    }
    // the faces of this lane's t1 cells, loaded ahead (their latency behind the P_0 stage, not in the F stage)
    constexpr int IF = (FN + 255) / 256;
    double fu[IF], fv[IF];
#pragma unroll
    for (int it = 0; it < IF; ++it) {
        const int i = tid + it * 256;
        if (i < FN) {
            const int r = i / kGFFW, c = i - r * kGFFW;
            const int32_t k = P.wrap(fr0 - 1 + r) * n + P.wrap(fc0 - 1 + c);
            fu[it] = P.uface[k];
            fv[it] = P.vface[k];
        }
    }
    __syncthreads();
    // t0 = P_0 x on the fine block + 2
    for (int i = tid; i < PN; i += 256) {
        const int r = i / kGFPW, c = i - r * kGFPW;
        const int gr = P.wrap(fr0 - 2 + r), gc = P.wrap(fc0 - 2 + c);
        if constexpr (MAC && INNER) {
#pragma unroll
            for (int f = 0; f < 4; ++f)
                t0[f * PN + i] = (f & 1) ? g1_p_in<MPBP_MG_NODE, MPBP_MG_CELL, kGFCW>(xs + f * CN, r, c)
                                         : g1_p_in<MPBP_MG_CELL, MPBP_MG_NODE, kGFCW>(xs + f * CN, r, c);
            continue;
        }
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            if constexpr (MAC) {
                t0[f * PN + i] = (f & 1)
                    ? g1_p<MPBP_MG_NODE, MPBP_MG_CELL, kGFCW>(xs + f * CN, gr, gc, nc, cr0 - 2, cc0 - 2)
                    : g1_p<MPBP_MG_CELL, MPBP_MG_NODE, kGFCW>(xs + f * CN, gr, gc, nc, cr0 - 2, cc0 - 2);
                continue;
            }
            int yi[4], xi[4];
            double yw[4], xw[4];
            const int my = mg_p1d_fast(tr.ky[f], nc, gr, yi, yw), mx = mg_p1d_fast(tr.kx[f], nc, gc, xi, xw);
            double acc = 0.0;
            for (int a = 0; a < my; ++a) {
                const double* xr = xs + f * CN + slot(yi[a], cr0 - 2, nc) * kGFCW;
                for (int b = 0; b < mx; ++b) acc += (yw[a] * xw[b]) * xr[slot(xi[b], cc0 - 2, nc)];
            }
            t0[f * PN + i] = acc;
        }
    }
    __syncthreads();
    // t1 = F t0 on the fine block + 1
    {
        const TTileT<kGFPW> tt{ts, fr0 - 2, fc0 - 2};
        const XTileT<kGFPW, kGFPH> xt{t0, fr0 - 2, fc0 - 2};
        // t1 takes t0's LDS (63 -> 42 KB per workgroup: 3 resident per CU instead of 2): rows kept in registers until
        // every lane has read its t0 neighbours
        double tv[IF][4];
#pragma unroll
        for (int it = 0; it < IF; ++it) {
            const int i = tid + it * 256;
            if (i >= FN) break;
            const int r = i / kGFFW, c = i - r * kGFFW;
            double rd[4];
            P.template rows4<false>(fr0 - 1 + r, fc0 - 1 + c, tt, xt, FStencilDev::Cell{{fu[it], fv[it]}}, tv[it], rd);
        }
        __syncthreads();
#pragma unroll
        for (int it = 0; it < IF; ++it) {
            const int i = tid + it * 256;
            if (i >= FN) break;
#pragma unroll
            for (int f = 0; f < 4; ++f) t1[f * FN + i] = tv[it][f];
        }
    }
    __syncthreads();
    // R_0 t1 on the tile's coarse rows (4 fields x 128 cells), each to the epilogue
    if constexpr (MAC) {   // lane t: cell t & 127 of fields (t >> 7) and (t >> 7) + 2 -- one kind pair per wave
        const int cell = tid & (kGFW * kGFH - 1), fp = tid >> 7;
        const int cr = cr0 + cell / kGFW, cc = cc0 + cell % kGFW;
        if (cr < (PART ? q.r0 + q.L : nc) && cc < nc) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int f = fp + 2 * h;
                const int32_t row = g1_orow<PART>(q, f, cr, cc, nc);
                typename Epi::P pe;
                if constexpr (PRO) {   // the iterate is the staged x + P_1 x_c at the row
                    pe = epi.pre_lite(row);
                    set_x(pe, xs[f * CN + (cr - cr0 + 2) * kGFCW + (cc - cc0 + 2)]);
                    set_diag(pe, epi.diag[row]);
                } else {
                    pe = epi.pre(row);
                }
                double acc;
                if constexpr (INNER)
                    acc = fp ? g1_r_in<MPBP_MG_NODE, MPBP_MG_CELL, kGFFW>(t1 + f * FN, cr - cr0, cc - cc0)
                             : g1_r_in<MPBP_MG_CELL, MPBP_MG_NODE, kGFFW>(t1 + f * FN, cr - cr0, cc - cc0);
                else
                    acc = fp ? g1_r<MPBP_MG_NODE, MPBP_MG_CELL, kGFFW>(t1 + f * FN, cr, cc, n, fr0 - 1, fc0 - 1)
                             : g1_r<MPBP_MG_CELL, MPBP_MG_NODE, kGFFW>(t1 + f * FN, cr, cc, n, fr0 - 1, fc0 - 1);
                epi(row, acc, pe);
            }
        }
        return;
    }
    for (int j = tid; j < 4 * kGFW * kGFH; j += 256) {
        const int f = j / (kGFW * kGFH), cell = j - f * (kGFW * kGFH);
        const int cr = cr0 + cell / kGFW, cc = cc0 + cell % kGFW;
        if (cr >= (PART ? q.r0 + q.L : nc) || cc >= nc) continue;
        const int32_t row = g1_orow<PART>(q, f, cr, cc, nc);
        const typename Epi::P pe = epi.pre(row);
        int yi[4], xi[4];
        double yw[4], xw[4];
        const int my = mg_r1d_fast(tr.ky[f], n, cr, yi, yw), mx = mg_r1d_fast(tr.kx[f], n, cc, xi, xw);
        double acc = 0.0;
        for (int a = 0; a < my; ++a) {
            const double* tr1 = t1 + f * FN + slot(yi[a], fr0 - 1, n) * kGFFW;
            for (int b = 0; b < mx; ++b) acc += (yw[a] * xw[b]) * tr1[slot(xi[b], fc0 - 1, n)];
        }
        epi(row, acc, pe);
    }
}

// ---- multigrid level 0 of a tolerance-mode F hierarchy: pre-smoothing, residual and restriction in one launch ----
// k_fpre (the V-cycle's descent at level 0, V(2, .) from x = 0): on k_fsolve's 64 x 8 tiles with H = 3 levels -- x0 =
// c2_0 b / diag over the tile + 3, the Chebyshev sweep x1 over the tile + 2 (written out on the tile: the iterate the
// post-smoothing continues from), the residual r = b - F x1 over the tile + 1 (in LDS), then R_0 r on the tile's 32 x 4
// coarse cells into the coarse right-hand side.  Each value is built by the operations of the launches it replaces
// (k_ftile<INIT>'s x0 and sweep, the residual sweep's tolerance-mode rows and EpiResid, k_mg_transfer_spmv's restriction
// lists and product order): bit-identical to them.  HBM: b, thn and faces in, x1 and the coarse rhs out -- the residual
// is never written.
template <int KY, int KX, int W>
__device__ inline double g1_rw(const double* tf, int cr, int cc, int n, int rb, int cb) {
    constexpr int MY = KY == MPBP_MG_CELL ? 4 : 3, MX = KX == MPBP_MG_CELL ? 4 : 3;
    int yi[4], xi[4];
    double yw[4], xw[4];
    mg_r1d_fast(KY, n, cr, yi, yw);
    mg_r1d_fast(KX, n, cc, xi, xw);
    double acc = 0.0;
#pragma unroll
    for (int a = 0; a < MY; ++a) {
        const double* tr1 = tf + g1_slot(yi[a], rb, n) * W;
#pragma unroll
        for (int b = 0; b < MX; ++b) acc += (yw[a] * xw[b]) * tr1[g1_slot(xi[b], cb, n)];
    }
    return acc;
}
struct FPre {
    const double* b;   // the level's right-hand side
    double* x_out;     // x1 (the pre-smoothed iterate)
    double* bc;        // the coarse right-hand side R_0 (b - F x1)
    double c2_0, c1, c2;
};
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 8))) MPBP_LDS_READS
k_fpre(FStencilFast P, FPre a) {
    constexpr int H = 3;
    using T = FsTile<H>;
    // slots: the two tile cells (0, 1), rings 1 .. 3 (2 .. 4); ring 1 lives through the residual level, ring 2
    // through the sweep, ring 3 is x0 only -- state (d, 1 / diag) for slots 0 .. 3
    constexpr int NT = 2, NSL = H + 2, NS = H + 1;
    __shared__ double ts[T::TN];
    __shared__ double xa[4 * T::N], xb[4 * T::N];
    const int n = P.n, nn = n * n, nc = n >> 1, ncc = nc * nc;
    const int tx = (n + kFTW - 1) / kFTW;
    const int bk = xcd_swizzle(blockIdx.x, gridDim.x);
    const int r0 = (bk / tx) * kFTH, c0 = (bk % tx) * kFTW;
    const int rbt = r0 - H - 1, cbt = c0 - H - 1, rb = r0 - H, cb = c0 - H;
    const int tid = threadIdx.x;
    {
        constexpr int IT = (T::TN + 255) / 256;
        double v[IT];
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = tid + it * 256;
            if (i < T::TN) {
                const int sr = i / T::TW, sc = i - sr * T::TW;
                v[it] = P.cell[P.wrap(rbt + sr) * n + P.wrap(cbt + sc)];
            }
        }
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = tid + it * 256;
            if (i < T::TN) ts[i] = v[it];
        }
    }
    const int lr = tid >> 6, lc = tid & 63;
    int cr[NSL], cc[NSL], rr[NSL];
    bool own[NSL];
#pragma unroll
    for (int m = 0; m < NT; ++m) {
        cr[m] = r0 + lr + 4 * m; cc[m] = c0 + lc; own[m] = true; rr[m] = 0;
    }
#pragma unroll
    for (int r = 1; r <= H; ++r) {
        own[1 + r] = tid < 140 + 8 * r;
        rr[1 + r] = r;
        fs_ring_cell(r, own[1 + r] ? tid : 0, r0, c0, cr[1 + r], cc[1 + r]);
    }
    double fl[NSL][2], bl[NSL][4];
#pragma unroll
    for (int sl = 0; sl < NSL; ++sl) {
        if (!own[sl]) continue;
        const int gr = P.wrap(cr[sl]), gc = P.wrap(cc[sl]);
        const int32_t k = gr * n + gc;
        fl[sl][0] = P.uface[k];
        fl[sl][1] = P.vface[k];
#pragma unroll
        for (int f = 0; f < 4; ++f) bl[sl][f] = a.b[(f * n + gr) * n + gc];
    }
    __syncthreads();
    const TTileT<T::TW> tt{ts, rbt, cbt};
    double d[NS][4], rd[NS][4];
    // level 0: x0 = d0 = c2_0 b / diag over the tile + 3
#pragma unroll
    for (int sl = 0; sl < NSL; ++sl) {
        if (!own[sl]) continue;
        const int vr = cr[sl], vc = cc[sl];
        const FStencilDev::Stage sg{{fl[sl][0], fl[sl][1]}};
        double r4[4];
        P.rdiag4(vr, vc, tt, sg, r4);
        const int si = (vr - rb) * T::RW + (vc - cb);
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            const double x0 = a.c2_0 * bl[sl][f] * r4[f];
            xa[f * T::N + si] = x0;
            if (sl < NS) {
                d[sl][f] = x0;
                rd[sl][f] = r4[f];
            }
        }
    }
    __syncthreads();
    // level 1: the sweep over the tile + 2 (x1 into xb; the tile's cells also to memory)
    {
        const XTileT<T::RW, T::RH> xt{xa, rb, cb};
#pragma unroll
        for (int sl = 0; sl < NS; ++sl) {
            if (sl >= NT && (!own[sl] || rr[sl] > 2)) continue;
            const int vr = cr[sl], vc = cc[sl];
            double acc[4], rdx[4];
            P.template rows4<false>(vr, vc, tt, xt, FStencilDev::Cell{{fl[sl][0], fl[sl][1]}}, acc, rdx);
            const int si = (vr - rb) * T::RW + (vc - cb);
#pragma unroll
            for (int f = 0; f < 4; ++f) {
                const double z = (bl[sl][f] - acc[f]) * rd[sl][f];
                const double dn = a.c1 * d[sl][f] + a.c2 * z;
                const double x = xa[f * T::N + si] + dn;
                xb[f * T::N + si] = x;
                if (sl < NT && vr < n && vc < n) a.x_out[f * nn + vr * n + vc] = x;
            }
        }
    }
    __syncthreads();
    // level 2: r = b - F x1 over the tile + 1 (into xa)
    {
        const XTileT<T::RW, T::RH> xt{xb, rb, cb};
#pragma unroll
        for (int sl = 0; sl < NS; ++sl) {
            if (sl >= NT && (!own[sl] || rr[sl] > 1)) continue;
            const int vr = cr[sl], vc = cc[sl];
            double acc[4], rdx[4];
            P.template rows4<false>(vr, vc, tt, xt, FStencilDev::Cell{{fl[sl][0], fl[sl][1]}}, acc, rdx);
            const int si = (vr - rb) * T::RW + (vc - cb);
#pragma unroll
            for (int f = 0; f < 4; ++f) xa[f * T::N + si] = bl[sl][f] - acc[f];
        }
    }
    __syncthreads();
    // R_0 r on the tile's coarse rows (4 fields x 128 cells; the F hierarchy's MAC kinds): lane t, cell t & 127 of
    // fields (t >> 7) and (t >> 7) + 2
    const int cell = tid & (kG1W * kG1H - 1), fp = tid >> 7;
    const int crr = (r0 >> 1) + cell / kG1W, ccc = (c0 >> 1) + cell % kG1W;
    if (crr < nc && ccc < nc) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int f = fp + 2 * h;
            const bool inner = g1_inner(r0 >> 1, c0 >> 1, kFTH / 2, kFTW / 2, nc);   // (window coordinates, slot 2 =
                                                                                     // fine 2 c0 - 1: rb = r0 - 3)
            const int lr = crr - (r0 >> 1), lc = ccc - (c0 >> 1);
            const double acc =
                inner ? (fp ? g1_rw_in<MPBP_MG_NODE, MPBP_MG_CELL, T::RW, 2>(xa + f * T::N, lr, lc)
                            : g1_rw_in<MPBP_MG_CELL, MPBP_MG_NODE, T::RW, 2>(xa + f * T::N, lr, lc))
                      : (fp ? g1_rw<MPBP_MG_NODE, MPBP_MG_CELL, T::RW>(xa + f * T::N, crr, ccc, n, rb, cb)
                            : g1_rw<MPBP_MG_CELL, MPBP_MG_NODE, T::RW>(xa + f * T::N, crr, ccc, n, rb, cb));
            a.bc[f * ncc + crr * nc + ccc] = acc;
        }
    }
}

// The pressure hierarchy's level 1 the same way (tolerance mode): A_1 x = R_0 (Gt_G (P_0 x)) on a 32 x 8 coarse tile
// (a 64 x 16 fine block), one field, cell-centred both ways; Gt_G's rows by GtGStencilDev::entries and add5 (the
// matrix-free level-0 sweep's operations), the transfers' by k_mg_transfer_spmv's: bit-identical to the three launches.
constexpr int kG1PH2 = 8;                                     // coarse tile rows (pressure)
constexpr int kGPFH = 2 * kG1PH2 + 2, kGPPH = kGPFH + 2;       // fine t1 / t0 rows
// PRO: as k_gal1's (x + P_1 x_c staged, level 2's window of the 16 x 4 level-2 cells under the tile first)
constexpr int kG1PQH = kG1PH2 / 2 + 4;   // level-2 window rows (columns kG1QW, row stride kG1CW)
template <class Epi, class XS = XPlain, bool PART = false, bool PRO = false>
__global__ void __launch_bounds__(256) MPBP_LDS_READS k_gal1p(GtGStencilDev P, XS xin, Epi epi, G1Part q,
                                                               const double* __restrict__ xc = nullptr) {
    constexpr int CH = kG1PH2 + 4, CN = kG1CW * CH, PN = kG1PW * kGPPH, FN = kG1FW * kGPFH;
    __shared__ double xs[CN];
    __shared__ double ts[PN];
    __shared__ double t0[PN];
    __shared__ double xq[PRO ? kG1CW * kG1PQH : 1];
    static_assert(!PRO || !PART, "the folded prolongation: whole level");
    double* t1 = t0;   // (k_gal1's aliasing: 34.7 -> 25 KB per workgroup)
    static_assert(FN <= PN, "t1 fits t0");
    const int n = P.n, nc = n >> 1;
    const int tx = (nc + kG1W - 1) / kG1W;
    const int bk = xcd_swizzle(blockIdx.x, gridDim.x);
    const int cr0 = (PART ? q.r0 : 0) + (bk / tx) * kG1PH2, cc0 = (bk % tx) * kG1W;
    const int fr0 = 2 * cr0, fc0 = 2 * cc0;
    const int tid = threadIdx.x;
    auto wrapc = [&](int a) { return a < 0 ? a + nc : (a >= nc ? a - nc : a); };
    {
        constexpr int IX = (CN + 255) / 256, IT = (PN + 255) / 256;
        typename XS::Raw vx[IX];
        double vt[IT];
#pragma unroll
        for (int it = 0; it < IX; ++it) {
            const int i = tid + it * 256;
            if (i < CN) {
                const int r = i / kG1CW, c = i - r * kG1CW;
                vx[it] = xin.load(g1_xidx<PART>(q, 1, 0, cr0 - 2 + r, wrapc(cc0 - 2 + c), nc));
            }
        }
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = tid + it * 256;
            if (i < PN) {
                const int r = i / kG1PW, c = i - r * kG1PW;
                vt[it] = P.cell[P.wrap(fr0 - 2 + r) * n + P.wrap(fc0 - 2 + c)];
            }
        }
        const int n2 = nc >> 1;
        if constexpr (PRO) {   // level 2's window first
            auto wrap2 = [&](int a) { return a < 0 ? a + n2 : (a >= n2 ? a - n2 : a); };
            constexpr int QN = kG1QW * kG1PQH, IQ = (QN + 255) / 256;
            double vq[IQ];
#pragma unroll
            for (int it = 0; it < IQ; ++it) {
                const int i = tid + it * 256;
                if (i < QN) {
                    const int r = i / kG1QW, c = i - r * kG1QW;
                    vq[it] = xc[wrap2((cr0 >> 1) - 2 + r) * n2 + wrap2((cc0 >> 1) - 2 + c)];
                }
            }
#pragma unroll
            for (int it = 0; it < IQ; ++it) {
                const int i = tid + it * 256;
                if (i < QN) {
                    const int r = i / kG1QW, c = i - r * kG1QW;
                    xq[r * kG1CW + c] = vq[it];
                }
            }
            __syncthreads();
        }
        const bool inner2 = PRO && g1_inner(cr0 >> 1, cc0 >> 1, kG1PH2 / 2, kG1W / 2, n2);
#pragma unroll
        for (int it = 0; it < IX; ++it) {
            const int i = tid + it * 256;
            if (i >= CN) continue;
            double v = xin.value(vx[it]);
            if constexpr (PRO) {   // x + P_1 x_c (EpiAdd: the row sum, then + x)
                const int r = i / kG1CW, c = i - r * kG1CW;
                const double pc =
                    inner2 ? g1_p_in<MPBP_MG_CELL, MPBP_MG_CELL>(xq, r, c)
                           : g1_p<MPBP_MG_CELL, MPBP_MG_CELL>(xq, wrapc(cr0 - 2 + r), wrapc(cc0 - 2 + c), n2,
                                                              (cr0 >> 1) - 2, (cc0 >> 1) - 2);
                v = pc + v;
            }
            xs[i] = v;
        }
#pragma unroll
        for (int it = 0; it < IT; ++it)
            if (tid + it * 256 < PN) ts[tid + it * 256] = vt[it];
    }
    __syncthreads();
    const bool inner = g1_inner(cr0, cc0, kG1PH2, kG1W, nc);   // (k_gal1's g1_*_in)
    for (int i = tid; i < PN; i += 256) {   // t0 = P_0 x on the fine block + 2
        const int r = i / kG1PW, c = i - r * kG1PW;
        t0[i] = inner ? g1_p_in<MPBP_MG_CELL, MPBP_MG_CELL>(xs, r, c)
                      : g1_p<MPBP_MG_CELL, MPBP_MG_CELL>(xs, P.wrap(fr0 - 2 + r), P.wrap(fc0 - 2 + c), nc, cr0 - 2, cc0 - 2);
    }
    __syncthreads();
    {   // t1 = Gt_G t0 on the fine block + 1
        const TTileT<kG1PW> ta{ts, fr0 - 2, fc0 - 2};
        constexpr int IT1 = (FN + 255) / 256;
        double tv[IT1];
#pragma unroll
        for (int it = 0; it < IT1; ++it) {
            const int i0 = it * 256;
            const int i = i0 + tid;
            const bool live = i < FN;
            const int ii = live ? i : 0;
            const int r = ii / kG1FW, c = ii - r * kG1FW;
            const int vr = fr0 - 1 + r, vc = fc0 - 1 + c, gr = P.wrap(vr), gc = P.wrap(vc);
            const bool edge = __builtin_amdgcn_readfirstlane(__any(live && (gr == 0 || gr == n - 1 || gc == 0 ||
                                                                            gc == n - 1))) != 0;
            if (!live) continue;
            double e[5];
            P.entries(vr, vc, gr, gc, ta, e);
            const int si = (r + 1) * kG1PW + (c + 1);
            const double pr[5] = {e[0] * t0[si - kG1PW], e[1] * t0[si - 1], e[2] * t0[si], e[3] * t0[si + 1],
                                  e[4] * t0[si + kG1PW]};
            const Wrap wr{gr == 0, gr == n - 1, gc == 0, gc == n - 1};
            tv[it] = edge ? add5<true>(0.0, pr, wr) : add5<false>(0.0, pr, wr);
        }
        __syncthreads();
#pragma unroll
        for (int it = 0; it < IT1; ++it)
            if (it * 256 + tid < FN) t1[it * 256 + tid] = tv[it];
    }
    __syncthreads();
    {   // R_0 t1 on the tile's 256 coarse rows, each to the epilogue
        const int cr = cr0 + tid / kG1W, cc = cc0 + tid % kG1W;
        if (cr < (PART ? q.r0 + q.L : nc) && cc < nc) {
            const int32_t row = g1_orow<PART>(q, 0, cr, cc, nc);
            typename Epi::P pe;
            if constexpr (PRO) {   // the iterate is the staged x + P_1 x_c at the row
                pe = epi.pre_lite(row);
                set_x(pe, xs[(cr - cr0 + 2) * kG1CW + (cc - cc0 + 2)]);
                set_diag(pe, epi.diag[row]);
            } else {
                pe = epi.pre(row);
            }
            epi(row, inner ? g1_r_in<MPBP_MG_CELL, MPBP_MG_CELL>(t1, cr - cr0, cc - cc0)
                           : g1_r<MPBP_MG_CELL, MPBP_MG_CELL>(t1, cr, cc, n, fr0 - 1, fc0 - 1), pe);
        }
    }
}

// One thread per (slice, lane): copy the CSR row into its column-major slots.
__global__ void k_sell_fill(Csr A, const int4* slices, int nslices, uint8_t* rlen, double* val, int32_t* col) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int sidx = (int)(t >> 6), lane = (int)(t & 63);
    if (sidx >= nslices) return;
    const int4 sl = slices[sidx];
    if (lane >= sl.y) return;
    const int32_t r = sl.x + lane;
    const int32_t k0 = A.rp[r], len = A.rp[r + 1] - k0;
    rlen[r] = (uint8_t)len;
    for (int k = 0; k < len; ++k) {
        const size_t slot = ((size_t)sl.w + (k >> 1)) * 64 + lane;
        val[2 * slot + (k & 1)] = A.va[k0 + k];
        col[2 * slot + (k & 1)] = A.ci[k0 + k];
    }
}

__global__ void k_jacobi_init(int32_t n, const double* b, const double* diag, const double* sub,
                              double* xout) {
    const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const double x = b[r] / diag[r];
    xout[r] = sub ? sub[r] - x : x;
}

__global__ void k_cheb_init(int32_t n, const double* b, const double* diag, double c2, double* d,
                            const double* sub, double* xout) {
    const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const double z = b[r] / diag[r];
    const double dn = c2 * z;
    d[r] = dn;
    xout[r] = sub ? sub[r] - dn : dn;
}

inline Csr to_csr(const mpbp_csr* A) { return Csr{A->row_ptr, A->col_idx, A->val, A->ncols}; }

template <class Epi>
int launch_rows(const mpbp_csr* A, const mpbp_rowblocks* blk, const double* x, Epi epi, hipStream_t st) {
    if (!blk || blk->count <= 0) return MPBP_OK;
    k_csr_wave<Epi><<<blk->count, kBlock, 0, st>>>(to_csr(A), x, reinterpret_cast<const int2*>(blk->pairs),
                                                    blk->count, KO().csr_table ? blk->table : nullptr, epi);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}
// Small-level CSR products through k_csr_grp: lanes per row from the mean row length (2: <= 16 entries, 4: <= 32,
// 8: longer), so one chunk holds a multigrid coarse row (transfers 1-16 entries, Galerkin levels 20-46).
template <class Epi, class XS = XPlain>
int launch_grp(const mpbp_csr* A, const XS& xs, Epi epi, hipStream_t st) {
    if (A->nrows <= 0) return MPBP_OK;
    const int64_t avg = A->nnz / A->nrows;
    auto go = [&](auto gc) {
        constexpr int G = decltype(gc)::value;
        constexpr int rpb = kBlock / G;
        k_csr_grp<G, XS, Epi><<<(unsigned)((A->nrows + rpb - 1) / rpb), kBlock, 0, st>>>(to_csr(A), A->nrows, xs, epi);
        MPBP_HIP(hipGetLastError());
        return (int)MPBP_OK;
    };
    return avg <= 16 ? go(std::integral_constant<int, 2>{})
                     : avg <= 32 ? go(std::integral_constant<int, 4>{}) : go(std::integral_constant<int, 8>{});
}
inline bool use_grp(const mpbp_csr& A) { return KO().mg_group_rows > 0 && A.nrows > 0 && A.nrows <= KO().mg_group_rows && A.nnz > 0; }
int grp_spmv(const mpbp_csr* A, int32_t mode, const double* x, const double* z, double* y, hipStream_t st) {
    const XPlain xs{x};
    switch (mode) {
    case MPBP_SPMV_STORE: return launch_grp(A, xs, EpiStore{y}, st);
    case MPBP_SPMV_ADD: return launch_grp(A, xs, EpiAdd{z, y}, st);
    case MPBP_SPMV_RESID: return launch_grp(A, xs, EpiResid{z, y}, st);
    default: return set_error(MPBP_ERR_ARG, "grp_spmv: unknown mode %d", mode);
    }
}
int grp_cheb(const mpbp_csr* A, const double* xin, const double* b, const double* dg, double c1, double c2, double* d,
             const double* sub, double* xo, hipStream_t st, int store_d, bool dzero) {
    const EpiCheb e{xin, b, dg, d, c1, c2, sub, xo, store_d};
    const XPlain xs{xin};
    return dzero ? launch_grp(A, xs, EpiZeroD<EpiCheb>{e}, st) : launch_grp(A, xs, e, st);
}
// First sweep from x = 0: x0 = d0 = c2_0 b / diag folded in (no k_cheb_init launch, same bits).
int grp_cheb_first(const mpbp_csr* A, const double* b, const double* dg, double c2_0, double c1, double c2, double* d,
                   const double* sub, double* xo, hipStream_t st, int store_d) {
    EpiChebFirstGrp e;
    static_cast<EpiChebFirst&>(e) = EpiChebFirst{b, d, c1, c2, sub, xo, store_d};
    e.diag = dg;
    e.c2_0 = c2_0;
    return launch_grp(A, XInit{b, dg, c2_0}, e, st);
}

// ---- small multigrid levels with their transfers folded in (kernel option mg_fuse_small) ----
// b_c = R (b - A x) in one launch, one wave per coarse row I: four lanes per fine row of R's row (<= 4 x 4 of them)
// gather that row's CSR entries at once and the slot's first lane adds the products left to right from 0.0 (k_csr_grp's
// sum) and forms b_j - sum (EpiResid); the wave's first lane then adds R's products (yw xw) r_j in list order
// (k_mg_transfer_spmv's restriction).  The residual and restriction launches' operations, bit for bit, without r's
// store and reload.  A fine row shared by neighbouring coarse rows is recomputed by each (up to 4x), so it pays only
// where the two launches are latency-bound: coarse levels of <= kRrMaxCoarse rows (1024^2, mg:1, profiles/
// r06l_mg_apply_kernel_trace.md: 7.3 vs 5.0 + 4.9 us into 1024 coarse rows, 6.6 vs ~9.8 into 256; into 4096, 10.4 vs
// 5.1 + 4.9; into 16384, 32 vs 11 + 5).  Folding the prolongation into the first post-smoothing sweep's gathers
// (x + P x_c per gathered column: five loads instead of one) measured slower than its two launches at every level
// (10-31 vs 9-17 us) and is not kept.
constexpr int32_t kRrMaxCoarse = 1024;
constexpr int kRrL = 4, kRrJ = 12, kRrCap = kRrL * kRrJ;   // lanes per fine row, entries per lane and chunk
__device__ inline int sel4(const int* v, int i) { return i == 0 ? v[0] : i == 1 ? v[1] : i == 2 ? v[2] : v[3]; }
__global__ void __launch_bounds__(kBlock) k_grp_rr(Csr A, MgFields F, MgDiv dv, int32_t n, int32_t ncr,
                                                  const double* __restrict__ x, const double* __restrict__ b,
                                                  double* __restrict__ bc) {
    constexpr int WPB = kBlock / 64;
    __shared__ double prod[WPB * 16 * kRrCap];
    __shared__ double rs[WPB * 16];
    const int w = threadIdx.x / 64, lane = threadIdx.x % 64, s = lane / kRrL, k = lane % kRrL;
    const int32_t I = blockIdx.x * WPB + w;   // wave-uniform: a wave past the last coarse row leaves whole
    if (I >= ncr) return;
    MgRow R;
    mg_row(F, dv, n, MPBP_MG_R, I, R);
    const bool live = s < R.my * R.mx;
    const int a = live ? (s >= R.mx) + (s >= 2 * R.mx) + (s >= 3 * R.mx) : 0, c = s - a * R.mx;
    const int32_t j = live ? R.off + sel4(R.yi, a) * n + sel4(R.xi, c) : 0;
    const int32_t ks = A.rp[j], ke = live ? A.rp[j + 1] : ks;
    const double bj = (live && k == 0) ? b[j] : 0.0;
    double* pr = prod + (w * 16 + s) * kRrCap;
    double acc = 0.0;
    for (int32_t cb = ks; cb < ke; cb += kRrCap) {
        double v[kRrJ];
        int32_t ci[kRrJ];
#pragma unroll
        for (int u = 0; u < kRrJ; ++u) {
            const int32_t e = cb + k + kRrL * u;
            const bool in = e < ke;
            v[u] = in ? A.va[e] : 0.0;
            ci[u] = in ? A.ci[e] : 0;
        }
        double p[kRrJ];
#pragma unroll
        for (int u = 0; u < kRrJ; ++u) p[u] = v[u] * x[ci[u]];
        if (cb != ks) wave_lds_sync();   // the previous chunk's sums have read their slots
#pragma unroll
        for (int u = 0; u < kRrJ; ++u) pr[k + kRrL * u] = p[u];
        wave_lds_sync();
        if (k == 0) {
            const int32_t cnt = min(ke - cb, (int32_t)kRrCap);
            for (int32_t e = 0; e < cnt; ++e) acc += pr[e];
        }
    }
    if (live && k == 0) rs[w * 16 + s] = bj - acc;
    wave_lds_sync();
    if (lane == 0) {
        double r = 0.0;
#pragma unroll
        for (int ya = 0; ya < 4; ++ya)
#pragma unroll
            for (int xb = 0; xb < 4; ++xb)
                if (ya < R.my && xb < R.mx) r += (R.yw[ya] * R.xw[xb]) * rs[w * 16 + ya * R.mx + xb];
        bc[I] = r;
    }
}

// Products through the stencil-values layout (k_svl).
inline Svl to_svl(const mpbp_svl* V) {
    return Svl{V->nfields, V->m, V->reach, V->slots, V->delta, V->vals, V->edge_rows, V->n_edge};
}
int check_svl(const mpbp_svl* V, const mpbp_csr* A) {
    if (!V || !A || V->slots < 1 || V->nfields < 1 || V->nfields * V->slots > kSvMaxDelta || V->reach < 0 ||
        V->m < 2 * V->reach + 2 || (V->m & 1) || (V->reach & 1) || (int64_t)V->nfields * V->m * V->m != A->nrows ||
        (int64_t)V->slots * A->nrows > INT32_MAX || !V->delta || !V->vals ||
        V->n_edge < 0 || (V->n_edge && !V->edge_rows))
        return set_error(MPBP_ERR_ARG, "svl: layout does not match the operator");
    return MPBP_OK;
}
template <class Epi, class XS = XPlain>
int launch_svl(const mpbp_svl* V, const mpbp_csr* A, const XS& xs, Epi epi, hipStream_t st) {
    const int64_t w = V->m - 2 * V->reach;
    const int64_t per = (w / 2) * w;
    const int64_t threads = (((int64_t)V->n_edge * kSvEdgeG + kBlock - 1) / kBlock) * kBlock + V->nfields * per;
    if (threads <= 0) return MPBP_OK;
    k_svl<XS, Epi><<<(unsigned)((threads + kBlock - 1) / kBlock), kBlock, 0, st>>>(to_svl(V), to_csr(A), A->nrows, xs,
                                                                                    epi);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}
int svl_spmv(const mpbp_svl* V, const mpbp_csr* A, int32_t mode, const double* x, const double* z, double* y,
             hipStream_t st) {
    const XPlain xs{x};
    switch (mode) {
    case MPBP_SPMV_STORE: return launch_svl(V, A, xs, EpiStore{y}, st);
    case MPBP_SPMV_ADD: return launch_svl(V, A, xs, EpiAdd{z, y}, st);
    case MPBP_SPMV_RESID: return launch_svl(V, A, xs, EpiResid{z, y}, st);
    default: return set_error(MPBP_ERR_ARG, "svl_spmv: unknown mode %d", mode);
    }
}
int svl_cheb(const mpbp_svl* V, const mpbp_csr* A, const double* xin, const double* b, const double* dg, double c1,
             double c2, double* d, const double* sub, double* xo, hipStream_t st, int store_d, bool dzero) {
    const EpiCheb e{xin, b, dg, d, c1, c2, sub, xo, store_d};
    const XPlain xs{xin};
    return dzero ? launch_svl(V, A, xs, EpiZeroD<EpiCheb>{e}, st) : launch_svl(V, A, xs, e, st);
}
template <class Epi>
int launch_rows_seg(const mpbp_csr* A, const mpbp_rowblocks* blk, const double* x, Epi epi, hipStream_t st) {
    if (!blk || blk->count <= 0) return MPBP_OK;
    k_csr_seg<Epi><<<blk->count, kBlock, 0, st>>>(to_csr(A), x, reinterpret_cast<const int2*>(blk->pairs),
                                                   blk->count, epi);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

template <class Epi>
int launch_sell(const mpbp_sell* S, const double* x, Epi epi, hipStream_t st) {
    if (!S || S->nslices <= 0) return MPBP_OK;
    const int slices_per_block = kBlock / 64;
    const int grid = (S->nslices + slices_per_block - 1) / slices_per_block;
    k_sell_rows<Epi><<<grid, kBlock, 0, st>>>(
        Sell{reinterpret_cast<const int4*>(S->slices), S->row_len, reinterpret_cast<const double2*>(S->val),
             reinterpret_cast<const int2*>(S->col)},
        x, S->nslices, epi);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int check_csr(const mpbp_csr* A) {
    if (!A || !A->row_ptr || A->nrows < 0) return set_error(MPBP_ERR_ARG, "invalid csr");
    if (A->nnz > 0 && (!A->col_idx || !A->val)) return set_error(MPBP_ERR_ARG, "csr without entries");
    return MPBP_OK;
}

// Chebyshev-Jacobi coefficients (Saad, Iterative Methods, Alg. 12.1 with diag(A)^-1 preconditioning).
void cheb_coeffs(double lmin, double lmax, int sweeps, double* c1, double* c2) {
    const double theta = (lmax + lmin) / 2.0;
    const double delta = (lmax - lmin) / 2.0;
    const double sigma = theta / delta;
    double rho = 1.0 / sigma;
    c1[0] = 0.0;
    c2[0] = 1.0 / theta;
    for (int s = 1; s < sweeps; ++s) {
        const double rho_new = 1.0 / (2.0 * sigma - rho);
        c1[s] = rho_new * rho;
        c2[s] = 2.0 * rho_new / delta;
        rho = rho_new;
    }
}

}  // namespace

// ================================================================ C ABI ====
extern "C" {

const char* mpbp_version(void) { return "libmpbp 0.1 (gfx950)"; }

void mpbp_kernel_opts_default(mpbp_kernel_opts* out) {
    if (out) *out = KO();
}

int mpbp_kernel_opts_set_thread(const mpbp_kernel_opts* o, const mpbp_kernel_opts** prev) {
    if (int rc = check_opts(o, "kernel_opts_set_thread")) return rc;
    if (prev) *prev = t_opts;
    t_opts = o;
    return MPBP_OK;
}

int mpbp_set_march_rows(int32_t rows) {
    if (rows < 0 || rows > 4096) return set_error(MPBP_ERR_ARG, "march rows must be 0 (auto) or in [1, 4096]");
    g_defaults.march_rows = rows;
    return MPBP_OK;
}
int mpbp_set_csr_table(int32_t on) {
    g_defaults.csr_table = on ? 1 : 0;
    return MPBP_OK;
}
int mpbp_set_mg_mf_transfer(int32_t on) {
    g_defaults.mg_mf_transfer = on ? 1 : 0;
    return MPBP_OK;
}
int mpbp_set_mg_svl(int32_t on) {
    g_defaults.mg_svl = on ? 1 : 0;
    return MPBP_OK;
}
int mpbp_set_mg_group_rows(int32_t rows) {
    if (rows < 0) return set_error(MPBP_ERR_ARG, "mg group rows must be >= 0");
    g_defaults.mg_group_rows = rows;
    return MPBP_OK;
}
int mpbp_set_pg_direct(int32_t on) {
    g_defaults.pg_direct = on ? 1 : 0;
    return MPBP_OK;
}

int mpbp_set_mg_galerkin_mf(int32_t on) {
    if (on < 0 || on > 2) return set_error(MPBP_ERR_ARG, "mg_galerkin_mf must be 0, 1 or 2");
    g_defaults.mg_galerkin_mf = on;
    return MPBP_OK;
}
int mpbp_set_mg_galerkin_mf_p(int32_t on) {
    if (on != 0 && on != 1) return set_error(MPBP_ERR_ARG, "mg_galerkin_mf_p must be 0 or 1");
    g_defaults.mg_galerkin_mf_p = on;
    return MPBP_OK;
}
int mpbp_set_f_direct(int32_t on) {
    if (on != 0 && on != 1) return set_error(MPBP_ERR_ARG, "f_direct must be 0 or 1");
    g_defaults.f_direct = on;
    return MPBP_OK;
}
int mpbp_set_gtg_fused(int32_t on) {
    if (on != 0 && on != 1 && on != 256 && on != 512) return set_error(MPBP_ERR_ARG, "gtg_fused must be 0, 1, 256 or 512");
    g_defaults.gtg_fused = on != 0;
    if (on == 256 || on == 512) g_defaults.gtg_tpb = on;
    return MPBP_OK;
}
int mpbp_set_q13_sym(int32_t on) {
    if (on != 0 && on != 1) return set_error(MPBP_ERR_ARG, "q13_sym must be 0 or 1");
    g_defaults.q13_sym = on;
    return MPBP_OK;
}
int mpbp_set_gtg_drhs(int32_t on) {
    if (on != 0 && on != 1) return set_error(MPBP_ERR_ARG, "gtg_drhs must be 0 or 1");
    g_defaults.gtg_drhs = on;
    return MPBP_OK;
}
int mpbp_set_f_tile(int32_t on) {
    if (on != 0 && on != 1) return set_error(MPBP_ERR_ARG, "f_tile must be 0 or 1");
    g_defaults.f_tile = on;
    return MPBP_OK;
}
int mpbp_set_f_solve(int32_t on) {
    if (on != 0 && on != 1) return set_error(MPBP_ERR_ARG, "f_solve must be 0 or 1");
    g_defaults.f_solve = on;
    return MPBP_OK;
}
int mpbp_set_f_pair(int32_t on) {
    if (on != 0 && on != 1) return set_error(MPBP_ERR_ARG, "f_pair must be 0 or 1");
    g_defaults.f_pair = on;
    return MPBP_OK;
}
int mpbp_set_init_diag(int32_t mode) {
    if (mode != 0 && mode != 1) return set_error(MPBP_ERR_ARG, "init diag mode must be 0 or 1");
    g_defaults.init_diag = mode;
    return MPBP_OK;
}
const char* mpbp_last_error(void) { return g_err; }

int mpbp_stokes_theta(int32_t n, double* cell, double* uface, double* vface, void* stream) {
    if (n < 1 || !cell || !uface || !vface) return set_error(MPBP_ERR_ARG, "mpbp_stokes_theta: bad args");
    k_theta<<<grid_for((int64_t)n * n), kBlock, 0, as_stream(stream)>>>(n, cell, uface, vface);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int64_t mpbp_stokes_rows(int32_t n, int32_t op) {
    const int64_t N = (int64_t)n * n;
    switch (op) {
    case MPBP_OP_A: return 5 * N;
    case MPBP_OP_F: case MPBP_OP_G: return 4 * N;
    case MPBP_OP_D: case MPBP_OP_D_N: case MPBP_OP_D_S: return N;
    case MPBP_OP_L_N: case MPBP_OP_L_S: case MPBP_OP_G_N: case MPBP_OP_G_S:
    case MPBP_OP_XI_N: case MPBP_OP_XI_S: return 2 * N;
    default: return set_error(MPBP_ERR_ARG, "unknown operator %d", op);
    }
}

int64_t mpbp_stokes_cols(int32_t n, int32_t op) {
    const int64_t N = (int64_t)n * n;
    switch (op) {
    case MPBP_OP_A: return 5 * N;
    case MPBP_OP_F: case MPBP_OP_D: return 4 * N;
    case MPBP_OP_G: case MPBP_OP_G_N: case MPBP_OP_G_S: return N;
    case MPBP_OP_L_N: case MPBP_OP_L_S: case MPBP_OP_D_N: case MPBP_OP_D_S:
    case MPBP_OP_XI_N: case MPBP_OP_XI_S: return 2 * N;
    default: return set_error(MPBP_ERR_ARG, "unknown operator %d", op);
    }
}

static int make_stokes(const mpbp_stokes_params* prm, const double* cell, const double* uface,
                       const double* vface, StokesDev* P) {
    if (!prm || prm->n < 1 || !cell) return set_error(MPBP_ERR_ARG, "stokes: bad params");
    if ((int64_t)prm->n * prm->n * 5 > INT32_MAX) return set_error(MPBP_ERR_OVERFLOW, "stokes: n too large");
    *P = StokesDev{prm->n, prm->xi, prm->eta_n, prm->eta_s, prm->c, prm->d_u, prm->d_p, prm->d_div,
                   cell, uface, vface};
    return MPBP_OK;
}

int mpbp_stokes_count(const mpbp_stokes_params* prm, int32_t op, const double* cell,
                      int32_t* row_nnz, void* stream) {
    StokesDev P;
    int rc = make_stokes(prm, cell, nullptr, nullptr, &P);
    if (rc) return rc;
    const int64_t rows = mpbp_stokes_rows(prm->n, op);
    if (rows < 0) return (int)rows;
    k_stokes_count<<<grid_for(rows), kBlock, 0, as_stream(stream)>>>(P, op, rows, row_nnz);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int mpbp_stokes_fill(const mpbp_stokes_params* prm, int32_t op, const double* cell,
                     const double* uface, const double* vface, const int32_t* row_ptr,
                     int32_t* col_idx, double* val, void* stream) {
    StokesDev P;
    int rc = make_stokes(prm, cell, uface, vface, &P);
    if (rc) return rc;
    if ((op == MPBP_OP_A || op == MPBP_OP_F) && (!uface || !vface))
        return set_error(MPBP_ERR_ARG, "stokes fill: A/F need face tables");
    const int64_t rows = mpbp_stokes_rows(prm->n, op);
    if (rows < 0) return (int)rows;
    k_stokes_fill<<<grid_for(rows), kBlock, 0, as_stream(stream)>>>(P, op, rows, row_ptr, col_idx, val);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int mpbp_stokes_count_rows(const mpbp_stokes_params* prm, int32_t op, const double* cell, const int32_t* rows,
                           int32_t nrows, int32_t* row_nnz, void* stream) {
    StokesDev P;
    int rc = make_stokes(prm, cell, nullptr, nullptr, &P);
    if (rc) return rc;
    if (mpbp_stokes_rows(prm->n, op) < 0) return set_error(MPBP_ERR_ARG, "stokes count rows: unknown operator %d", op);
    if (nrows < 0 || (nrows > 0 && (!rows || !row_nnz))) return set_error(MPBP_ERR_ARG, "stokes count rows: bad args");
    if (nrows == 0) return MPBP_OK;
    k_stokes_count<<<grid_for(nrows), kBlock, 0, as_stream(stream)>>>(P, op, nrows, row_nnz, rows);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int mpbp_stokes_fill_rows(const mpbp_stokes_params* prm, int32_t op, const double* cell, const double* uface,
                          const double* vface, const int32_t* rows, int32_t nrows, const int32_t* row_ptr,
                          int32_t* col_idx, double* val, void* stream) {
    StokesDev P;
    int rc = make_stokes(prm, cell, uface, vface, &P);
    if (rc) return rc;
    if ((op == MPBP_OP_A || op == MPBP_OP_F) && (!uface || !vface))
        return set_error(MPBP_ERR_ARG, "stokes fill rows: A/F need face tables");
    if (mpbp_stokes_rows(prm->n, op) < 0) return set_error(MPBP_ERR_ARG, "stokes fill rows: unknown operator %d", op);
    if (nrows < 0 || (nrows > 0 && (!rows || !row_ptr))) return set_error(MPBP_ERR_ARG, "stokes fill rows: bad args");
    if (nrows == 0) return MPBP_OK;
    k_stokes_fill<<<grid_for(nrows), kBlock, 0, as_stream(stream)>>>(P, op, nrows, row_ptr, col_idx, val, rows);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int mpbp_exclusive_scan(const int32_t* row_nnz, int32_t* row_ptr, int64_t n, int64_t* total,
                        void* stream) {
    if (n < 0 || !row_ptr || (n > 0 && !row_nnz)) return set_error(MPBP_ERR_ARG, "scan: bad args");
    const int64_t ntiles = (n + kScanTile - 1) / kScanTile;
    long long* d_total = nullptr;   // [total, tile sums...]
    MPBP_HIP(hipMalloc(&d_total, sizeof(long long) * (size_t)(1 + ntiles)));
    hipStream_t st = as_stream(stream);
    if (ntiles > 0) k_scan_tiles<<<(unsigned)ntiles, 256, 0, st>>>(row_nnz, n, d_total + 1);
    k_scan_offsets<<<1, 256, 0, st>>>(d_total + 1, ntiles, row_ptr, n, d_total);
    if (ntiles > 0) k_scan_apply<<<(unsigned)ntiles, 256, 0, st>>>(row_nnz, n, d_total + 1, row_ptr);
    hipError_t e = hipGetLastError();
    long long h = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&h, d_total, sizeof(h), hipMemcpyDeviceToHost, as_stream(stream));
    if (e == hipSuccess) e = hipStreamSynchronize(as_stream(stream));
    (void)hipFree(d_total);
    if (e != hipSuccess) return set_error(MPBP_ERR_HIP, "scan: %s", hipGetErrorString(e));
    if (h > INT32_MAX) return set_error(MPBP_ERR_OVERFLOW, "scan: %lld entries exceed int32 row_ptr", h);
    if (total) *total = h;
    return MPBP_OK;
}

int mpbp_spgemm_count(const mpbp_csr* A, const mpbp_csr* B, int32_t* row_nnz, void* stream) {
    int rc = check_csr(A);
    if (!rc) rc = check_csr(B);
    if (rc) return rc;
    if (A->ncols != B->nrows) return set_error(MPBP_ERR_ARG, "spgemm: shape mismatch");
    int* d_over = nullptr;
    MPBP_HIP(hipMalloc(&d_over, sizeof(int)));
    hipError_t e = hipMemsetAsync(d_over, 0, sizeof(int), as_stream(stream));
    if (e == hipSuccess) {
        k_spgemm_count<<<grid_for(A->nrows), kBlock, 0, as_stream(stream)>>>(to_csr(A), to_csr(B), A->nrows,
                                                                          row_nnz, d_over);
        e = hipGetLastError();
    }
    int h = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&h, d_over, sizeof(int), hipMemcpyDeviceToHost, as_stream(stream));
    if (e == hipSuccess) e = hipStreamSynchronize(as_stream(stream));
    (void)hipFree(d_over);
    if (e != hipSuccess) return set_error(MPBP_ERR_HIP, "spgemm_count: %s", hipGetErrorString(e));
    if (h) return set_error(MPBP_ERR_OVERFLOW, "spgemm: %d rows wider than %d", h, kSpgemmMaxW);
    return MPBP_OK;
}

int mpbp_spgemm_fill(const mpbp_csr* A, const mpbp_csr* B, double alpha, const int32_t* row_ptr,
                     int32_t* col_idx, double* val, void* stream) {
    int rc = check_csr(A);
    if (!rc) rc = check_csr(B);
    if (rc) return rc;
    k_spgemm_fill<<<grid_for(A->nrows), kBlock, 0, as_stream(stream)>>>(to_csr(A), to_csr(B), A->nrows, alpha,
                                                                     row_ptr, col_idx, val);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int64_t mpbp_plan_row_blocks(const int32_t* row_ptr, int32_t row_begin, int32_t row_end,
                             int32_t* pairs, int64_t capacity) {
    if (!row_ptr || row_begin < 0 || row_end < row_begin) return set_error(MPBP_ERR_ARG, "plan: bad args");
    int64_t nb = 0;
    int32_t r = row_begin;
    while (r < row_end) {
        const int32_t s = r;
        int32_t e = r;
        while (e < row_end && e - s < kBlock && row_ptr[e + 1] - row_ptr[s] <= MPBP_BLOCK_NNZ) ++e;
        if (e == s) e = s + 1;   // one row longer than the LDS stage
        if (pairs && nb < capacity) {
            pairs[2 * nb] = s;
            pairs[2 * nb + 1] = e;
        }
        ++nb;
        r = e;
    }
    return nb;
}

int mpbp_csr_diag(const mpbp_csr* A, int32_t col_offset, double* diag, int32_t* missing, void* stream) {
    int rc = check_csr(A);
    if (rc) return rc;
    int* d_miss = nullptr;
    MPBP_HIP(hipMalloc(&d_miss, sizeof(int)));
    hipError_t e = hipMemsetAsync(d_miss, 0, sizeof(int), as_stream(stream));
    if (e == hipSuccess) {
        k_csr_diag<<<grid_for(A->nrows), kBlock, 0, as_stream(stream)>>>(to_csr(A), A->nrows, col_offset,
                                                                      diag, d_miss);
        e = hipGetLastError();
    }
    int h = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&h, d_miss, sizeof(int), hipMemcpyDeviceToHost, as_stream(stream));
    if (e == hipSuccess) e = hipStreamSynchronize(as_stream(stream));
    (void)hipFree(d_miss);
    if (e != hipSuccess) return set_error(MPBP_ERR_HIP, "csr_diag: %s", hipGetErrorString(e));
    if (missing) *missing = h;
    return MPBP_OK;
}

int mpbp_gershgorin(const mpbp_csr* A, const double* diag, double* lmax, void* stream) {
    int rc = check_csr(A);
    if (rc) return rc;
    unsigned long long* d_out = nullptr;
    MPBP_HIP(hipMalloc(&d_out, sizeof(unsigned long long)));
    hipError_t e = hipMemsetAsync(d_out, 0, sizeof(unsigned long long), as_stream(stream));
    if (e == hipSuccess) {
        k_gershgorin<<<grid_for(A->nrows), kBlock, 0, as_stream(stream)>>>(to_csr(A), A->nrows, diag, d_out);
        e = hipGetLastError();
    }
    unsigned long long h = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&h, d_out, sizeof(h), hipMemcpyDeviceToHost, as_stream(stream));
    if (e == hipSuccess) e = hipStreamSynchronize(as_stream(stream));
    (void)hipFree(d_out);
    if (e != hipSuccess) return set_error(MPBP_ERR_HIP, "gershgorin: %s", hipGetErrorString(e));
    double v;
    memcpy(&v, &h, sizeof(v));
    if (lmax) *lmax = v;
    return MPBP_OK;
}

int mpbp_csr_extract_count(const mpbp_csr* A, const int32_t* rows, int32_t nrows_local,
                           int32_t* row_nnz, void* stream) {
    int rc = check_csr(A);
    if (rc) return rc;
    if (nrows_local < 0 || (nrows_local && (!rows || !row_nnz))) return set_error(MPBP_ERR_ARG, "extract: bad args");
    if (nrows_local == 0) return MPBP_OK;
    k_extract_count<<<grid_for(nrows_local), kBlock, 0, as_stream(stream)>>>(to_csr(A), rows, nrows_local, row_nnz);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int mpbp_csr_extract_fill(const mpbp_csr* A, const int32_t* rows, int32_t nrows_local,
                          const int32_t* colmap, const int32_t* row_ptr_local, int32_t* col_local,
                          double* val_local, void* stream) {
    int rc = check_csr(A);
    if (rc) return rc;
    if (nrows_local == 0) return MPBP_OK;
    int* d_bad = nullptr;
    MPBP_HIP(hipMalloc(&d_bad, sizeof(int)));
    hipError_t e = hipMemsetAsync(d_bad, 0, sizeof(int), as_stream(stream));
    if (e == hipSuccess) {
        k_extract_fill<<<grid_for(nrows_local), kBlock, 0, as_stream(stream)>>>(
            to_csr(A), rows, nrows_local, colmap, row_ptr_local, col_local, val_local, d_bad);
        e = hipGetLastError();
    }
    int h = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&h, d_bad, sizeof(int), hipMemcpyDeviceToHost, as_stream(stream));
    if (e == hipSuccess) e = hipStreamSynchronize(as_stream(stream));
    (void)hipFree(d_bad);
    if (e != hipSuccess) return set_error(MPBP_ERR_HIP, "extract_fill: %s", hipGetErrorString(e));
    if (h) return set_error(MPBP_ERR_PATTERN, "extract: %d entries reference columns outside the halo", h);
    return MPBP_OK;
}

int mpbp_spmv(const mpbp_csr* A, const mpbp_rowblocks* blocks, int32_t mode, const double* x,
              const double* z, double* y, void* stream) {
    int rc = check_csr(A);
    if (rc) return rc;
    if (!x || !y || (mode != MPBP_SPMV_STORE && !z)) return set_error(MPBP_ERR_ARG, "spmv: bad vectors");
    const hipStream_t st = as_stream(stream);
    switch (mode) {
    case MPBP_SPMV_STORE: return launch_rows(A, blocks, x, EpiStore{y}, st);
    case MPBP_SPMV_ADD: return launch_rows(A, blocks, x, EpiAdd{z, y}, st);
    case MPBP_SPMV_RESID: return launch_rows(A, blocks, x, EpiResid{z, y}, st);
    default: return set_error(MPBP_ERR_ARG, "spmv: unknown mode %d", mode);
    }
}

int mpbp_hbm_stream(const void* src, int64_t bytes, int32_t mode, double* dst, void* stream) {
    if (!src || !dst || bytes < 16 || (mode != 0 && mode != 1)) return set_error(MPBP_ERR_ARG, "hbm_stream: bad args");
    const hipStream_t st = as_stream(stream);
    if (mode == 0) {
        const int64_t n16 = bytes / 16;
        k_hbm_read<<<(unsigned)((n16 + 1023) / 1024), kBlock, 0, st>>>(reinterpret_cast<const f64x2*>(src), n16, dst);
    } else {
        const int64_t nwaves = bytes / (576 * 16);
        if (nwaves < 1) return set_error(MPBP_ERR_ARG, "hbm_stream: mode 1 needs >= 9 KiB");
        k_hbm_readwrite<<<(unsigned)((nwaves + 3) / 4), kBlock, 0, st>>>(reinterpret_cast<const f64x2*>(src), nwaves,
                                                                         dst);
    }
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int mpbp_spmv_seg(const mpbp_csr* A, const mpbp_rowblocks* blocks, int32_t mode, const double* x,
                  const double* z, double* y, void* stream) {
    int rc = check_csr(A);
    if (rc) return rc;
    if (!x || !y || (mode != MPBP_SPMV_STORE && !z)) return set_error(MPBP_ERR_ARG, "spmv_seg: bad vectors");
    const hipStream_t st = as_stream(stream);
    switch (mode) {
    case MPBP_SPMV_STORE: return launch_rows_seg(A, blocks, x, EpiStore{y}, st);
    case MPBP_SPMV_ADD: return launch_rows_seg(A, blocks, x, EpiAdd{z, y}, st);
    case MPBP_SPMV_RESID: return launch_rows_seg(A, blocks, x, EpiResid{z, y}, st);
    default: return set_error(MPBP_ERR_ARG, "spmv_seg: unknown mode %d", mode);
    }
}

int mpbp_jacobi_init(int32_t nrows, const double* b, const double* diag, const double* sub,
                     double* x_out, void* stream) {
    if (nrows < 0 || (nrows && (!b || !diag || !x_out))) return set_error(MPBP_ERR_ARG, "jacobi_init: bad args");
    if (!nrows) return MPBP_OK;
    k_jacobi_init<<<grid_for(nrows), kBlock, 0, as_stream(stream)>>>(nrows, b, diag, sub, x_out);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int mpbp_jacobi_step(const mpbp_csr* A, const mpbp_rowblocks* blocks, const double* x_in,
                     const double* b, const double* diag, const double* sub, double* x_out,
                     void* stream) {
    int rc = check_csr(A);
    if (rc) return rc;
    if (!x_in || !b || !diag || !x_out || x_in == x_out) return set_error(MPBP_ERR_ARG, "jacobi_step: bad vectors");
    return launch_rows(A, blocks, x_in, EpiJacobi{x_in, b, diag, sub, x_out}, as_stream(stream));
}

int mpbp_cheb_init(int32_t nrows, const double* b, const double* diag, double c2, double* d,
                   const double* sub, double* x_out, void* stream) {
    if (nrows < 0 || (nrows && (!b || !diag || !d || !x_out))) return set_error(MPBP_ERR_ARG, "cheb_init: bad args");
    if (!nrows) return MPBP_OK;
    k_cheb_init<<<grid_for(nrows), kBlock, 0, as_stream(stream)>>>(nrows, b, diag, c2, d, sub, x_out);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

static int cheb_step_impl(const mpbp_csr* A, const mpbp_rowblocks* blocks, const double* x_in,
                          const double* b, const double* diag, double c1, double c2, double* d,
                          const double* sub, double* x_out, void* stream, int store_d) {
    int rc = check_csr(A);
    if (rc) return rc;
    if (!x_in || !b || !diag || !d || !x_out || x_in == x_out) return set_error(MPBP_ERR_ARG, "cheb_step: bad vectors");
    return launch_rows(A, blocks, x_in, EpiCheb{x_in, b, diag, d, c1, c2, sub, x_out, store_d}, as_stream(stream));
}

int mpbp_cheb_step(const mpbp_csr* A, const mpbp_rowblocks* blocks, const double* x_in,
                   const double* b, const double* diag, double c1, double c2, double* d,
                   const double* sub, double* x_out, void* stream) {
    return cheb_step_impl(A, blocks, x_in, b, diag, c1, c2, d, sub, x_out, stream, 1);
}

int mpbp_cheb_coeffs(double lmin, double lmax, int32_t sweeps, double* c1, double* c2) {
    if (sweeps < 1 || !c1 || !c2 || !(lmax > lmin) || !(lmin >= 0.0))
        return set_error(MPBP_ERR_ARG, "cheb_coeffs: need sweeps >= 1 and lmax > lmin >= 0");
    cheb_coeffs(lmin, lmax, sweeps, c1, c2);
    return MPBP_OK;
}

int mpbp_gather(int32_t count, const int32_t* idx, const double* src, double* dst, void* stream) {
    if (count <= 0) return MPBP_OK;
    k_gather<<<grid_for(count), kBlock, 0, as_stream(stream)>>>(count, idx, src, dst);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int mpbp_scatter(int32_t count, const int32_t* idx, const double* src, double* dst, void* stream) {
    if (count <= 0) return MPBP_OK;
    k_scatter<<<grid_for(count), kBlock, 0, as_stream(stream)>>>(count, idx, src, dst);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int mpbp_event_create(void** ev) {
    hipEvent_t e;
    MPBP_HIP(hipEventCreate(&e));
    *ev = (void*)e;
    return MPBP_OK;
}

int mpbp_event_create_scoped(void** ev, int32_t device_scope) {
    hipEvent_t e;
    MPBP_HIP(hipEventCreateWithFlags(&e, device_scope ? hipEventReleaseToDevice : hipEventDefault));
    *ev = (void*)e;
    return MPBP_OK;
}

int mpbp_event_record(void* ev, void* stream) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    MPBP_HIP(hipStreamIsCapturing(as_stream(stream), &cs));
    if (cs == hipStreamCaptureStatusNone) MPBP_HIP(hipEventRecord((hipEvent_t)ev, as_stream(stream)));
    return MPBP_OK;
}

int mpbp_event_destroy(void* ev) {
    MPBP_HIP(hipEventDestroy((hipEvent_t)ev));
    return MPBP_OK;
}

int mpbp_event_elapsed_ms(void* start, void* stop, float* ms) {
    MPBP_HIP(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
    return MPBP_OK;
}

}  // extern "C"

// ================================================= Krylov orthogonalisation ====
// FGMRES's classical Gram-Schmidt passes over the Krylov basis V (k vectors of n doubles, row stride ld):
// h = V w (mpbp_gs_dot) and w_out = w - V^T h (mpbp_gs_update).  rocBLAS's gemv over a k x 5 M row-major basis
// streams at ~2 TB/s; these stream V once per pass at HBM speed.  Deterministic: the dot products are per-chunk
// partial sums (each workgroup's in a fixed tree order) added chunk after chunk by one thread per vector.
namespace {
constexpr int kGsVec = 8;      // basis vectors per dot-product workgroup
constexpr int kGsPer = 16;     // elements per thread per chunk
constexpr int kGsBatch = 4;    // elements whose loads are issued together
constexpr int kGsChunk = kBlock * kGsPer;
__global__ void __launch_bounds__(kBlock) k_gs_dot(const double* __restrict__ V, int64_t ld, int k,
                                                   const double* __restrict__ w, int64_t n, double* part) {
    const int64_t c = blockIdx.x;
    const int i0 = blockIdx.y * kGsVec;
    const int nv = min(kGsVec, k - i0);
    double acc[kGsVec];
#pragma unroll
    for (int v = 0; v < kGsVec; ++v) acc[v] = 0.0;
    for (int u = 0; u < kGsPer; u += kGsBatch) {
        double wv[kGsBatch], vv[kGsVec][kGsBatch];
#pragma unroll
        for (int q = 0; q < kGsBatch; ++q) {   // every load of the batch in flight at once
            const int64_t e = c * kGsChunk + (int64_t)(u + q) * kBlock + threadIdx.x;
            const bool ok = e < n;
            const int64_t ee = ok ? e : 0;
            wv[q] = ok ? w[ee] : 0.0;
#pragma unroll
            for (int v = 0; v < kGsVec; ++v) vv[v][q] = v < nv ? V[(int64_t)(i0 + v) * ld + ee] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < kGsBatch; ++q)
#pragma unroll
            for (int v = 0; v < kGsVec; ++v) acc[v] += vv[v][q] * wv[q];
    }
    __shared__ double red[kGsVec][kBlock / 64];
    const int lane = threadIdx.x & 63, wv_ = threadIdx.x >> 6;
#pragma unroll
    for (int v = 0; v < kGsVec; ++v) {
        double a = acc[v];
        for (int off = 32; off > 0; off >>= 1) a += __shfl_down(a, off, 64);
        if (lane == 0) red[v][wv_] = a;
    }
    __syncthreads();
    if (threadIdx.x < nv) {
        double a = 0.0;
        for (int q = 0; q < kBlock / 64; ++q) a += red[threadIdx.x][q];
        part[c * k + i0 + threadIdx.x] = a;
    }
}
// h[i] = the chunk partials of vector i, one workgroup per vector: strided per-thread sums, then a fixed tree.
__global__ void __launch_bounds__(kBlock) k_gs_sum(const double* part, int64_t nchunks, int k, double* h) {
    const int i = blockIdx.x;
    double a = 0.0;
    for (int64_t c = threadIdx.x; c < nchunks; c += kBlock) a += part[c * k + i];
    for (int off = 32; off > 0; off >>= 1) a += __shfl_down(a, off, 64);
    __shared__ double red[kBlock / 64];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int q = 0; q < kBlock / 64; ++q) t += red[q];
        h[i] = t;
    }
}
// (w and wo may alias: each thread reads w[e] before it writes wo[e], so neither is declared __restrict__)
__global__ void __launch_bounds__(kBlock) k_gs_update(const double* __restrict__ V, int64_t ld, int k,
                                                      const double* __restrict__ h, const double* w,
                                                      int64_t n, double* wo) {
    __shared__ double hs[256];
    for (int i = threadIdx.x; i < k; i += kBlock) hs[i] = h[i];
    __syncthreads();
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= n) return;
    double a = 0.0;
    int i = 0;
    for (; i + 8 <= k; i += 8) {   // 8 basis rows' loads in flight, then added in order
        double v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = V[(int64_t)(i + q) * ld + e];
#pragma unroll
        for (int q = 0; q < 8; ++q) a += v[q] * hs[i + q];
    }
    for (; i < k; ++i) a += V[(int64_t)i * ld + e] * hs[i];
    wo[e] = w[e] - a;
}
// ---- reproducible dot products: binned summation (Demmel & Nguyen's pre-rounding, 3 folds) ----
// Every term t = v w (|t| <= 2^E, E from the caller's bounds; N terms in the whole distributed vector) is split as
// t = q0 + q1 + q2 + (dropped): q_f = fl(sigma_f + r) - sigma_f with sigma_f = 1.5 * 2^(E + (f+1) L - 53 f), L >= log2 N + 1,
// r the remainder of the previous folds.  Each q_f is a multiple of ulp(sigma_f) and N of them sum to less than
// 2^53 such ulps, so every partial sum of a fold is EXACT: the fold sums -- and h = (S0 + S1) + S2 -- depend only on
// the set of terms, never on the order, the chunking, the launch configuration or the split of the vector over
// ranks (the sums of the ranks' fold sums are exact too).  FGMRES therefore computes the same bits on one GPU and
// on a row partition.  Accuracy: |h - sum t| <= N 2^(E + 3L - 159) + one rounding (about 2^-51 of the bound for
// N = 2^24), against the N eps sum|t| of a plain sum.  A fold whose sigma would be subnormal is skipped (q = 0).
constexpr int kRdVec = 4;      // basis vectors per workgroup
constexpr int kRdFolds = 3;
__device__ inline void rd_sigmas(double bound, int64_t ntot, double* sig) {
    int E = 0;
    (void)frexp(bound, &E);    // bound < 2^E
    const int L = 65 - __clzll((unsigned long long)(ntot > 0 ? ntot : 1));
    const bool finite = bound == bound && bound <= 1.7976931348623157e308;
#pragma unroll
    for (int f = 0; f < kRdFolds; ++f) {
        const int ex = E + (f + 1) * L - 53 * f;
        sig[f] = (!finite || (bound > 0.0 && E + L > 1023)) ? __longlong_as_double(0x7ff8000000000000LL)   // NaN / range
                 : !(bound > 0.0) ? 0.0                              // all terms 0: nothing to fold
                 : ex >= -1022 ? ldexp(1.5, ex) : 0.0;               // subnormal fold: skipped
    }
}
__device__ inline void rd_fold(double t, const double* sig, double* acc) {
    double r = t;
#pragma unroll
    for (int f = 0; f < kRdFolds; ++f) {
        const double q = (sig[f] + r) - sig[f];
        const double qq = sig[f] != 0.0 ? q : 0.0;
        acc[f] += qq;
        r -= qq;
    }
}
__global__ void __launch_bounds__(kBlock) k_rdot(const double* __restrict__ V, int64_t ld, int k,
                                                 const double* __restrict__ w, int64_t n, int64_t ntot,
                                                 const double* __restrict__ bound_v, const double* __restrict__ bound_w,
                                                 double* part) {
    const int64_t c = blockIdx.x;
    const int i0 = blockIdx.y * kRdVec;
    const int nv = min(kRdVec, k - i0);
    double sig[kRdVec][kRdFolds], acc[kRdVec][kRdFolds];
    const double bw = bound_w[0];
#pragma unroll
    for (int v = 0; v < kRdVec; ++v) {
        rd_sigmas(v < nv ? bound_v[i0 + v] * bw : 0.0, ntot, sig[v]);
#pragma unroll
        for (int f = 0; f < kRdFolds; ++f) acc[v][f] = 0.0;
    }
    for (int u = 0; u < kGsPer; u += kGsBatch) {
        double wv[kGsBatch], vv[kRdVec][kGsBatch];
#pragma unroll
        for (int q = 0; q < kGsBatch; ++q) {   // every load of the batch in flight at once
            const int64_t e = c * kGsChunk + (int64_t)(u + q) * kBlock + threadIdx.x;
            const bool ok = e < n;
            const int64_t ee = ok ? e : 0;
            wv[q] = ok ? w[ee] : 0.0;
#pragma unroll
            for (int v = 0; v < kRdVec; ++v) vv[v][q] = v < nv ? V[(int64_t)(i0 + v) * ld + ee] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < kGsBatch; ++q)
#pragma unroll
            for (int v = 0; v < kRdVec; ++v) rd_fold(vv[v][q] * wv[q], sig[v], acc[v]);
    }
    // block reduction: exact additions, so the tree shape does not matter
    __shared__ double red[kRdVec * kRdFolds][kBlock / 64];
    const int lane = threadIdx.x & 63, wv_ = threadIdx.x >> 6;
#pragma unroll
    for (int v = 0; v < kRdVec; ++v)
#pragma unroll
        for (int f = 0; f < kRdFolds; ++f) {
            double a = acc[v][f];
            for (int off = 32; off > 0; off >>= 1) a += __shfl_down(a, off, 64);
            if (lane == 0) red[v * kRdFolds + f][wv_] = a;
        }
    __syncthreads();
    if (threadIdx.x < nv * kRdFolds) {
        double a = 0.0;
        for (int q = 0; q < kBlock / 64; ++q) a += red[threadIdx.x][q];
        part[c * (3 * (int64_t)k) + 3 * i0 + threadIdx.x] = a;
    }
}
// ---- DCGS2 (Gram-Schmidt with delayed re-orthogonalisation: Swirydowicz et al. 2020, Bielich et al. 2022) ----
// FGMRES iteration j holds q_0 .. q_{j-1} (orthonormal) and u_j (= V[j], projected once, not normalised); one pass over
// the basis forms the block product [V[0..j]] . [u_j, w] (w = A M u_j) -- the fold sums of both columns (k_rdot2) --
// and one more pass (k_dcgs2_update) re-orthogonalises and normalises u_j into q_j and projects w once into u_{j+1}:
// two passes over the basis per iteration instead of CGS2's four.  Scalars (k_dcgs2_coeffs, one thread, fixed order):
//   s = V[0..j-1] . u_j, alpha = u_j . u_j, z = V[0..j-1] . w, beta = u_j . w,
//   r = sqrt(alpha - s.s), q_j = (u_j - V s) / r, c = (beta - s.z) / r = q_j . w, u_{j+1} = w - V z - q_j c
// (j = 0: q_0 = u_0 is the normalised residual, r = 1).  Arnoldi: A Z[j] = w = V z + q_j c + u_{j+1}, and
// u_{j+1} = V' s' + r' q_{j+1} one iteration later, so column j of H is z + s', c + s'_j, r' (one iteration lagged).
// Bounds for the binned sums: |q_i| <= 1 (unit vectors), |u_{j+1}| <= (max|w| + sum |z_i| + |c|) (1 + 2^-40).
__global__ void __launch_bounds__(kBlock) k_rdot2(const double* __restrict__ V, int64_t ld, int k,
                                                  const double* __restrict__ u, const double* __restrict__ w, int64_t n,
                                                  int64_t ntot, const double* __restrict__ bound_v,
                                                  const double* __restrict__ bound_u, const double* __restrict__ bound_w,
                                                  double* part) {
    const int64_t c = blockIdx.x;
    const double bu = bound_u[0], bw = bound_w[0];
    __shared__ double red[kRdVec * 2 * kRdFolds][kBlock / 64];
    const int lane = threadIdx.x & 63, wv_ = threadIdx.x >> 6;
    for (int i0 = 0; i0 < k; i0 += kRdVec) {   // the chunk's u and w re-read per group from L2; V streamed once
        const int nv = min(kRdVec, k - i0);
        double sig[kRdVec][2][kRdFolds], acc[kRdVec][2][kRdFolds];
#pragma unroll
        for (int v = 0; v < kRdVec; ++v) {
            const double b = v < nv ? bound_v[i0 + v] : 0.0;
            rd_sigmas(b * bu, ntot, sig[v][0]);
            rd_sigmas(b * bw, ntot, sig[v][1]);
#pragma unroll
            for (int f = 0; f < kRdFolds; ++f) acc[v][0][f] = acc[v][1][f] = 0.0;
        }
        for (int uu = 0; uu < kGsPer; uu += kGsBatch) {
            double uv[kGsBatch], wv[kGsBatch], vv[kRdVec][kGsBatch];
#pragma unroll
            for (int q = 0; q < kGsBatch; ++q) {
                const int64_t e = c * kGsChunk + (int64_t)(uu + q) * kBlock + threadIdx.x;
                const bool ok = e < n;
                const int64_t ee = ok ? e : 0;
                uv[q] = ok ? u[ee] : 0.0;
                wv[q] = ok ? w[ee] : 0.0;
#pragma unroll
                for (int v = 0; v < kRdVec; ++v) vv[v][q] = (v < nv && ok) ? V[(int64_t)(i0 + v) * ld + ee] : 0.0;
            }
#pragma unroll
            for (int q = 0; q < kGsBatch; ++q)
#pragma unroll
                for (int v = 0; v < kRdVec; ++v) {
                    rd_fold(vv[v][q] * uv[q], sig[v][0], acc[v][0]);
                    rd_fold(vv[v][q] * wv[q], sig[v][1], acc[v][1]);
                }
        }
#pragma unroll
        for (int v = 0; v < kRdVec; ++v)
#pragma unroll
            for (int r = 0; r < 2; ++r)
#pragma unroll
                for (int f = 0; f < kRdFolds; ++f) {
                    double a = acc[v][r][f];
                    for (int off = 32; off > 0; off >>= 1) a += __shfl_down(a, off, 64);
                    if (lane == 0) red[(v * 2 + r) * kRdFolds + f][wv_] = a;
                }
        __syncthreads();
        if (threadIdx.x < nv * 2 * kRdFolds) {
            const int t = threadIdx.x, v = t / (2 * kRdFolds), r = (t / kRdFolds) & 1, f = t % kRdFolds;
            double a = 0.0;
            for (int q = 0; q < kBlock / 64; ++q) a += red[t][q];
            part[c * (6 * (int64_t)k) + r * 3 * (int64_t)k + 3 * (i0 + v) + f] = a;
        }
        __syncthreads();
    }
}
// hu[0..j], hw[0..j] from the fold sums (acc: 3 (j+1) for u, then 3 (j+1) for w); P = {r, 1 / r, c, bound of u_{j+1}}.
__global__ void k_dcgs2_coeffs(int j, const double* __restrict__ acc, const double* __restrict__ bound_w,
                               double* __restrict__ hu, double* __restrict__ hw, double* __restrict__ P) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const int k = j + 1;
    double ss = 0.0, sz = 0.0, b = bound_w[0];
    for (int i = 0; i < k; ++i) {
        hu[i] = (acc[3 * i] + acc[3 * i + 1]) + acc[3 * i + 2];
        hw[i] = (acc[3 * k + 3 * i] + acc[3 * k + 3 * i + 1]) + acc[3 * k + 3 * i + 2];
    }
    for (int i = 0; i < j; ++i) {
        ss = ss + hu[i] * hu[i];
        sz = sz + hu[i] * hw[i];
        b = b + fabs(hw[i]);
    }
    double r = 1.0, rinv = 1.0;
    if (j > 0) {
        const double d = hu[j] - ss;
        r = d > 0.0 ? sqrt(d) : 0.0;
        rinv = r > 0.0 ? 1.0 / r : 0.0;
    }
    const double cc = (hw[j] - sz) * rinv;
    b = ((b + fabs(cc)) * rinv) * (1.0 + 0x1p-40);   // u_{j+1} is stored scaled by 1 / r (k_dcgs2_update)
    P[0] = r;
    P[1] = rinv;
    P[2] = cc;
    P[3] = b;
}
// V[j] <- q_j = (V[j] - V[0..j-1]^T s) / r; V[j + 1] <- u_{j+1} = ((w - V[0..j-1]^T z) - q_j c) / r (both sums in basis
// order from 0.0, k_gs_update's operations; upd_w = 0: q_j only).  w = A M u_j was formed from the raw u_j (norm ~ r):
// scaling u_{j+1} by 1 / r keeps the raw vectors at the size of A M q_j instead of growing by ||A M|| per iteration
// (the Arnoldi column then belongs to Z[j] / r, fgmres's bookkeeping).
__global__ void __launch_bounds__(kBlock) k_dcgs2_update(double* __restrict__ V, int64_t ld, int j,
                                                         const double* __restrict__ hu, const double* __restrict__ hw,
                                                         const double* __restrict__ P, const double* __restrict__ w,
                                                         int64_t n, int upd_w) {
    __shared__ double ss[256], zs[256];
    for (int i = threadIdx.x; i < j; i += kBlock) {
        ss[i] = hu[i];
        zs[i] = hw[i];
    }
    __syncthreads();
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= n) return;
    double su = 0.0, sw = 0.0;
    int i = 0;
    for (; i + 8 <= j; i += 8) {
        double v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = V[(int64_t)(i + q) * ld + e];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            su += v[q] * ss[i + q];
            sw += v[q] * zs[i + q];
        }
    }
    for (; i < j; ++i) {
        const double v = V[(int64_t)i * ld + e];
        su += v * ss[i];
        sw += v * zs[i];
    }
    const double qv = (V[(int64_t)j * ld + e] - su) * P[1];
    V[(int64_t)j * ld + e] = qv;
    if (upd_w) V[(int64_t)(j + 1) * ld + e] = ((w[e] - sw) - qv * P[2]) * P[1];
}

// CGS2's first update and second projection in one kernel: wo = w - V^T h (k_gs_update's operations, same bits) and
// the exact fold sums of V[i] . wo (k_rdot's pre-rounding).  The extractors cannot wait for max|wo|, so they come from
// the a-priori bound B = (max|w| + sum_i bound_v[i] |h[i]|) (1 + 2^-40) >= max|wo| -- the same in every workgroup and
// on every rank (its inputs are global), so the fold sums stay exact and reproducible; the looser bound costs accuracy
// only below 2^-58 of it.  A workgroup updates its chunk (16 elements per thread, kept in LDS), then forms the
// products vector group by vector group as k_rdot does, re-reading the chunk's basis entries it has just streamed
// (from the L2 / MALL while they last) instead of a second full pass -- and wo is never re-read.
__global__ void __launch_bounds__(kBlock) k_gs_update_rdot(const double* __restrict__ V, int64_t ld, int k,
                                                           const double* __restrict__ h, const double* w, int64_t n,
                                                           int64_t ntot, const double* __restrict__ bound_v,
                                                           const double* __restrict__ bound_w, double* wo,
                                                           double* __restrict__ part) {
    __shared__ double hs[256];
    __shared__ double sg[256 * kRdFolds];
    __shared__ double red[kBlock / 64][kRdVec * kRdFolds];
    __shared__ double bnd;
    const int tid = threadIdx.x, lane = tid & 63, wq = tid >> 6;
    for (int i = tid; i < k; i += kBlock) hs[i] = h[i];
    __syncthreads();
    if (tid == 0) {
        double b = bound_w[0];
        for (int i = 0; i < k; ++i) b += bound_v[i] * fabs(hs[i]);
        bnd = b * (1.0 + 0x1p-40);
    }
    __syncthreads();
    for (int i = tid; i < k; i += kBlock) rd_sigmas(bound_v[i] * bnd, ntot, sg + kRdFolds * i);
    const int64_t c = blockIdx.x;
    __shared__ double w1[kGsChunk];   // the updated chunk, [u][thread]
    for (int u = 0; u < kGsPer; ++u) {   // the update, element by element (k_gs_update's order of operations)
        const int64_t e = c * kGsChunk + (int64_t)u * kBlock + tid;
        const bool ok = e < n;
        const int64_t ee = ok ? e : 0;
        double a = 0.0;
        int i = 0;
        for (; i + 8 <= k; i += 8) {
            double v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = V[(int64_t)(i + q) * ld + ee];
#pragma unroll
            for (int q = 0; q < 8; ++q) a += v[q] * hs[i + q];
        }
        for (; i < k; ++i) a += V[(int64_t)i * ld + ee] * hs[i];
        const double r = ok ? w[ee] - a : 0.0;
        w1[u * kBlock + tid] = r;
        if (ok) wo[ee] = r;
    }
    __syncthreads();   // (sg; each thread reads back only its own w1 entries)
    for (int i0 = 0; i0 < k; i0 += kRdVec) {   // the products, kRdVec basis vectors at a time (k_rdot's folds)
        const int nv = min(kRdVec, k - i0);
        double acc[kRdVec][kRdFolds], sig[kRdVec][kRdFolds];
#pragma unroll
        for (int v = 0; v < kRdVec; ++v)
#pragma unroll
            for (int f = 0; f < kRdFolds; ++f) {
                acc[v][f] = 0.0;
                sig[v][f] = v < nv ? sg[kRdFolds * (i0 + v) + f] : 0.0;
            }
        for (int u = 0; u < kGsPer; u += kGsBatch) {
            double vv[kRdVec][kGsBatch];
#pragma unroll
            for (int q = 0; q < kGsBatch; ++q) {
                const int64_t e = c * kGsChunk + (int64_t)(u + q) * kBlock + tid;
                const int64_t ee = e < n ? e : 0;
#pragma unroll
                for (int v = 0; v < kRdVec; ++v) vv[v][q] = v < nv ? V[(int64_t)(i0 + v) * ld + ee] : 0.0;
            }
#pragma unroll
            for (int q = 0; q < kGsBatch; ++q)
#pragma unroll
                for (int v = 0; v < kRdVec; ++v) rd_fold(vv[v][q] * w1[(u + q) * kBlock + tid], sig[v], acc[v]);
        }
#pragma unroll
        for (int v = 0; v < kRdVec; ++v)
#pragma unroll
            for (int f = 0; f < kRdFolds; ++f) {
                double x = acc[v][f];
                for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
                if (lane == 0) red[wq][kRdFolds * v + f] = x;
            }
        __syncthreads();
        if (tid < kRdFolds * nv) {   // the group's partials over the 4 waves (exact)
            double t = 0.0;
#pragma unroll
            for (int q = 0; q < kBlock / 64; ++q) t += red[q][tid];
            part[c * (kRdFolds * (int64_t)k) + kRdFolds * i0 + tid] = t;
        }
        __syncthreads();
    }
}
// acc[j] = sum over chunks of part[c][j] (exact), one workgroup per fold sum
__global__ void __launch_bounds__(kBlock) k_rdot_sum(const double* part, int64_t nchunks, int k3, double* acc) {
    const int j = blockIdx.x;
    double a = 0.0;
    for (int64_t c = threadIdx.x; c < nchunks; c += kBlock) a += part[c * k3 + j];
    for (int off = 32; off > 0; off >>= 1) a += __shfl_down(a, off, 64);
    __shared__ double red[kBlock / 64];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int q = 0; q < kBlock / 64; ++q) t += red[q];
        acc[j] = t;
    }
}
__global__ void k_rdot_finish(int k, const double* acc, double* h) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < k) h[i] = (acc[3 * i] + acc[3 * i + 1]) + acc[3 * i + 2];
}
// amax = max |x| (non-negative doubles order like their bit patterns; NaN's pattern exceeds every finite one)
// Eight loads in flight per thread, the maximum taken on the bit patterns, one atomic per workgroup (one per wave
// made every wave of a 5 M-entry vector queue on the same address: 65 us per call in the FGMRES loop).
__global__ void __launch_bounds__(kBlock) k_absmax(const double* __restrict__ x, int64_t n, unsigned long long* out) {
    __shared__ unsigned long long red[kBlock / 64];
    unsigned long long b = 0;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    for (; e + 7 * stride < n; e += 8 * stride) {
        double a[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) a[u] = x[e + u * stride];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const unsigned long long v = (unsigned long long)__double_as_longlong(fabs(a[u]));
            b = v > b ? v : b;
        }
    }
    for (; e < n; e += stride) {
        const unsigned long long v = (unsigned long long)__double_as_longlong(fabs(x[e]));
        b = v > b ? v : b;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(b, off, 64);
        b = o > b ? o : b;
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int w = 1; w < kBlock / 64; ++w) b = red[w] > b ? red[w] : b;
        atomicMax(out, b);
    }
}
}  // namespace

extern "C" {

int mpbp_gs_dot(const double* V, int64_t ld, int32_t k, const double* w, int64_t n, double* part, double* h,
                void* stream) {
    if (!V || !w || !h || !part || k < 1 || k > 256 || n < 1 || ld < n)
        return set_error(MPBP_ERR_ARG, "gs_dot: bad args (1 <= k <= 256, ld >= n)");
    const int64_t nchunks = (n + kGsChunk - 1) / kGsChunk;
    const dim3 grid((unsigned)nchunks, (unsigned)((k + kGsVec - 1) / kGsVec));
    k_gs_dot<<<grid, kBlock, 0, as_stream(stream)>>>(V, ld, k, w, n, part);
    MPBP_HIP(hipGetLastError());
    k_gs_sum<<<k, kBlock, 0, as_stream(stream)>>>(part, nchunks, k, h);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int64_t mpbp_gs_part_size(int64_t n, int32_t k) { return ((n + kGsChunk - 1) / kGsChunk) * (int64_t)k; }

int64_t mpbp_rdot_part_size(int64_t n, int32_t k) { return ((n + kGsChunk - 1) / kGsChunk) * 3 * (int64_t)k; }

int mpbp_rdot(const double* V, int64_t ld, int32_t k, const double* w, int64_t n, int64_t n_total,
              const double* bound_v, const double* bound_w, double* part, double* acc, void* stream) {
    if (!V || !w || !bound_v || !bound_w || !part || !acc || k < 1 || k > 256 || n < 0 || ld < n || n_total < n)
        return set_error(MPBP_ERR_ARG, "rdot: bad args (1 <= k <= 256, ld >= n, n_total >= n)");
    const hipStream_t st = as_stream(stream);
    if (n == 0) {
        MPBP_HIP(hipMemsetAsync(acc, 0, sizeof(double) * 3 * (size_t)k, st));
        return MPBP_OK;
    }
    const int64_t nchunks = (n + kGsChunk - 1) / kGsChunk;
    const dim3 grid((unsigned)nchunks, (unsigned)((k + kRdVec - 1) / kRdVec));
    k_rdot<<<grid, kBlock, 0, st>>>(V, ld, k, w, n, n_total, bound_v, bound_w, part);
    MPBP_HIP(hipGetLastError());
    k_rdot_sum<<<3 * k, kBlock, 0, st>>>(part, nchunks, 3 * k, acc);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int mpbp_rdot2(const double* V, int64_t ld, int32_t k, const double* u, const double* w, int64_t n, int64_t n_total,
               const double* bound_v, const double* bound_u, const double* bound_w, double* part, double* acc,
               void* stream) {
    if (!V || !u || !w || !bound_v || !bound_u || !bound_w || !part || !acc || k < 1 || k > 256 || n < 0 || ld < n ||
        n_total < n)
        return set_error(MPBP_ERR_ARG, "rdot2: bad args (1 <= k <= 256, ld >= n, n_total >= n)");
    const hipStream_t st = as_stream(stream);
    if (n == 0) {
        MPBP_HIP(hipMemsetAsync(acc, 0, sizeof(double) * 6 * (size_t)k, st));
        return MPBP_OK;
    }
    const int64_t nchunks = (n + kGsChunk - 1) / kGsChunk;
    k_rdot2<<<(unsigned)nchunks, kBlock, 0, st>>>(V, ld, k, u, w, n, n_total, bound_v, bound_u, bound_w, part);
    MPBP_HIP(hipGetLastError());
    k_rdot_sum<<<6 * k, kBlock, 0, st>>>(part, nchunks, 6 * k, acc);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int mpbp_dcgs2_update(double* V, int64_t ld, int32_t j, const double* acc, const double* bound_w, const double* w,
                      int64_t n, int32_t upd_w, double* hu, double* hw, double* P, void* stream) {
    if (!V || !acc || !bound_w || !hu || !hw || !P || (upd_w && !w) || j < 0 || j > 255 || n < 1 || ld < n)
        return set_error(MPBP_ERR_ARG, "dcgs2_update: bad args (0 <= j <= 255, ld >= n)");
    const hipStream_t st = as_stream(stream);
    k_dcgs2_coeffs<<<1, 64, 0, st>>>(j, acc, bound_w, hu, hw, P);
    MPBP_HIP(hipGetLastError());
    k_dcgs2_update<<<grid_for(n), kBlock, 0, st>>>(V, ld, j, hu, hw, P, w, n, upd_w);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int mpbp_gs_update_rdot(const double* V, int64_t ld, int32_t k, const double* h, const double* w, int64_t n,
                        int64_t n_total, const double* bound_v, const double* bound_w, double* w_out, double* part,
                        double* acc, void* stream) {
    if (!V || !w || !h || !w_out || !bound_v || !bound_w || !part || !acc || k < 1 || k > 256 || n < 1 || ld < n ||
        n_total < n)
        return set_error(MPBP_ERR_ARG, "gs_update_rdot: bad args (1 <= k <= 256, ld >= n >= 1, n_total >= n)");
    const hipStream_t st = as_stream(stream);
    const int64_t nchunks = (n + kGsChunk - 1) / kGsChunk;
    k_gs_update_rdot<<<(unsigned)nchunks, kBlock, 0, st>>>(V, ld, k, h, w, n, n_total, bound_v, bound_w, w_out, part);
    MPBP_HIP(hipGetLastError());
    k_rdot_sum<<<3 * k, kBlock, 0, st>>>(part, nchunks, 3 * k, acc);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int mpbp_rdot_finish(int32_t k, const double* acc, double* h, void* stream) {
    if (!acc || !h || k < 1) return set_error(MPBP_ERR_ARG, "rdot_finish: bad args");
    k_rdot_finish<<<grid_for(k), kBlock, 0, as_stream(stream)>>>(k, acc, h);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int mpbp_absmax(const double* x, int64_t n, double* amax, void* stream) {
    if (!amax || n < 0 || (n > 0 && !x)) return set_error(MPBP_ERR_ARG, "absmax: bad args");
    const hipStream_t st = as_stream(stream);
    MPBP_HIP(hipMemsetAsync(amax, 0, sizeof(double), st));
    if (n == 0) return MPBP_OK;
    const int64_t blocks = (n + kBlock * 16 - 1) / (kBlock * 16);
    k_absmax<<<(unsigned)(blocks < 1024 ? blocks : 1024), kBlock, 0, st>>>(x, n, reinterpret_cast<unsigned long long*>(amax));
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int mpbp_gs_update(const double* V, int64_t ld, int32_t k, const double* h, const double* w, int64_t n, double* w_out,
                   void* stream) {
    if (!V || !w || !h || !w_out || k < 1 || k > 256 || n < 1 || ld < n)
        return set_error(MPBP_ERR_ARG, "gs_update: bad args (1 <= k <= 256, ld >= n)");
    k_gs_update<<<grid_for(n), kBlock, 0, as_stream(stream)>>>(V, ld, k, h, w, n, w_out);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

}  // extern "C"

// ============================================================== SELL ABI ====
extern "C" {

int64_t mpbp_sell_plan(const int32_t* row_ptr, const int32_t* ranges, int32_t nranges, int32_t* slices,
                       int64_t capacity, int64_t* pair_rows) {
    if (!row_ptr || nranges < 0 || (nranges && !ranges)) return set_error(MPBP_ERR_ARG, "sell_plan: bad args");
    int64_t ns = 0, pr = 0;
    for (int32_t q = 0; q < nranges; ++q) {
        const int32_t a = ranges[2 * q], b = ranges[2 * q + 1];
        if (a < 0 || b < a) return set_error(MPBP_ERR_ARG, "sell_plan: bad range");
        for (int32_t r0 = a; r0 < b; r0 += 64) {
            const int32_t rows = (b - r0) < 64 ? (b - r0) : 64;
            int32_t w = 0;
            for (int32_t r = r0; r < r0 + rows; ++r) {
                const int32_t len = row_ptr[r + 1] - row_ptr[r];
                if (len > 255) return set_error(MPBP_ERR_OVERFLOW, "sell_plan: row %d has %d > 255 entries", r, len);
                w = len > w ? len : w;
            }
            if (slices && ns < capacity) {
                slices[4 * ns] = r0;
                slices[4 * ns + 1] = rows;
                slices[4 * ns + 2] = w;
                slices[4 * ns + 3] = (int32_t)pr;
            }
            pr += (w + 1) / 2;
            if (pr > INT32_MAX) return set_error(MPBP_ERR_OVERFLOW, "sell_plan: too many pair rows");
            ++ns;
        }
    }
    if (pair_rows) *pair_rows = pr;
    return ns;
}

int mpbp_sell_fill(const mpbp_csr* A, const int32_t* slices, int32_t nslices, uint8_t* row_len, double* val,
                   int32_t* col, void* stream) {
    int rc = check_csr(A);
    if (rc) return rc;
    if (nslices <= 0) return MPBP_OK;
    if (!slices || !row_len || !val || !col) return set_error(MPBP_ERR_ARG, "sell_fill: bad args");
    k_sell_fill<<<grid_for((int64_t)nslices * 64), kBlock, 0, as_stream(stream)>>>(
        to_csr(A), reinterpret_cast<const int4*>(slices), nslices, row_len, val, col);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

static int check_sell(const mpbp_sell* S) {
    if (!S || S->nslices < 0 || (S->nslices && (!S->slices || !S->row_len || !S->val || !S->col)))
        return set_error(MPBP_ERR_ARG, "invalid sell matrix");
    return MPBP_OK;
}

int mpbp_sell_spmv(const mpbp_sell* S, int32_t mode, const double* x, const double* z, double* y, void* stream) {
    int rc = check_sell(S);
    if (rc) return rc;
    if (!x || !y || (mode != MPBP_SPMV_STORE && !z)) return set_error(MPBP_ERR_ARG, "sell_spmv: bad vectors");
    const hipStream_t st = as_stream(stream);
    switch (mode) {
    case MPBP_SPMV_STORE: return launch_sell(S, x, EpiStore{y}, st);
    case MPBP_SPMV_ADD: return launch_sell(S, x, EpiAdd{z, y}, st);
    case MPBP_SPMV_RESID: return launch_sell(S, x, EpiResid{z, y}, st);
    default: return set_error(MPBP_ERR_ARG, "sell_spmv: unknown mode %d", mode);
    }
}

int mpbp_sell_jacobi_step(const mpbp_sell* S, const double* x_in, const double* b, const double* diag,
                          const double* sub, double* x_out, void* stream) {
    int rc = check_sell(S);
    if (rc) return rc;
    if (!x_in || !b || !diag || !x_out || x_in == x_out) return set_error(MPBP_ERR_ARG, "sell_jacobi_step: bad vectors");
    return launch_sell(S, x_in, EpiJacobi{x_in, b, diag, sub, x_out}, as_stream(stream));
}

static int sell_cheb_impl(const mpbp_sell* S, const double* x_in, const double* b, const double* diag, double c1,
                          double c2, double* d, const double* sub, double* x_out, void* stream, int store_d) {
    int rc = check_sell(S);
    if (rc) return rc;
    if (!x_in || !b || !diag || !d || !x_out || x_in == x_out) return set_error(MPBP_ERR_ARG, "sell_cheb_step: bad vectors");
    return launch_sell(S, x_in, EpiCheb{x_in, b, diag, d, c1, c2, sub, x_out, store_d}, as_stream(stream));
}

int mpbp_sell_cheb_step(const mpbp_sell* S, const double* x_in, const double* b, const double* diag, double c1,
                        double c2, double* d, const double* sub, double* x_out, void* stream) {
    return sell_cheb_impl(S, x_in, b, diag, c1, c2, d, sub, x_out, stream, 1);
}

static int make_fstencil(const mpbp_stokes_params* prm, const double* cell, const double* uface,
                         const double* vface, const mpbp_row_part* part, FStencilDev* P) {
    if (!prm || prm->n < 3 || !cell || !uface || !vface)
        return set_error(MPBP_ERR_ARG, "f_stencil: needs n >= 3 and the three thn tables");
    if ((int64_t)prm->n * prm->n * 5 > INT32_MAX) return set_error(MPBP_ERR_OVERFLOW, "f_stencil: n too large");
    const double dx = 1.0 / prm->n;
    int r0 = 0, L = prm->n, h = 0, which = 0, ext = 0, oh = 0;
    if (part && part->halo > 0) {
        r0 = part->r0; L = part->rows; h = part->halo; which = part->which;
        ext = which == 3 ? part->ext : 0;
        oh = part->oh > 0 ? part->oh : h;
        if (L < 1 || r0 < 0 || r0 + L > prm->n || which < 0 || which > 3 || ext < 0 || ext + 1 > h || ext > oh ||
            h > L || oh > L)
            return set_error(MPBP_ERR_ARG, "f_stencil: bad row partition");
    }
    *P = FStencilDev{prm->n, prm->xi, prm->eta_n, prm->eta_s, prm->c, prm->d_u, cell, uface, vface,
                     dx * dx, 1.0 / (dx * dx), -1.0 / (dx * dx), r0, L, h, which,
                     (prm->n & (prm->n - 1)) == 0 ? 1 : 0, ext, oh};
    if (P->pow2) {   // idx2 = n^2 exactly: eta * idx2 is an exact scaling (f_row's M bit 3)
        P->ce0 = prm->eta_n * P->idx2;
        P->ce1 = prm->eta_s * P->idx2;
    }
    return MPBP_OK;
}

}  // extern "C"

namespace {
template <class Epi>
int launch_fstencil(const FStencilDev& P, const double* x, Epi epi, hipStream_t st, bool fast = false) {
    return with_f_policy(P, fast, [&](const auto& Q) { return launch_march(Q, XPlain{x}, epi, KO().march_rows, st); });
}

}  // namespace

extern "C" {

int mpbp_f_stencil_spmv(const mpbp_stokes_params* prm, const double* cell, const double* uface,
                        const double* vface, const mpbp_row_part* part, int32_t mode, const double* x,
                        const double* z, double* y, void* stream) {
    FStencilDev P;
    int rc = make_fstencil(prm, cell, uface, vface, part, &P);
    if (rc) return rc;
    const bool fast = (mode & MPBP_SPMV_FAST) != 0;
    mode &= ~MPBP_SPMV_FAST;
    if (!x || !y || (mode != MPBP_SPMV_STORE && !z)) return set_error(MPBP_ERR_ARG, "f_stencil_spmv: bad vectors");
    const hipStream_t st = as_stream(stream);
    switch (mode) {
    case MPBP_SPMV_STORE: return launch_fstencil(P, x, EpiStore{y}, st, fast);
    case MPBP_SPMV_ADD: return launch_fstencil(P, x, EpiAdd{z, y}, st, fast);
    case MPBP_SPMV_RESID: return launch_fstencil(P, x, EpiResid{z, y}, st, fast);
    default: return set_error(MPBP_ERR_ARG, "f_stencil_spmv: unknown mode %d", mode);
    }
}

static int f_stencil_jacobi_impl(const mpbp_stokes_params* prm, const double* cell, const double* uface,
                                 const double* vface, const mpbp_row_part* part, const double* x_in,
                                 const double* b, const double* sub, double* x_out, void* stream, bool fast) {
    FStencilDev P;
    int rc = make_fstencil(prm, cell, uface, vface, part, &P);
    if (rc) return rc;
    if (!x_in || !b || !x_out || x_in == x_out) return set_error(MPBP_ERR_ARG, "f_stencil_jacobi_step: bad vectors");
    return launch_fstencil(P, x_in, EpiJacobi{x_in, b, nullptr, sub, x_out}, as_stream(stream), fast);
}

int mpbp_f_stencil_jacobi_step(const mpbp_stokes_params* prm, const double* cell, const double* uface,
                               const double* vface, const mpbp_row_part* part, const double* x_in,
                               const double* b, const double* sub, double* x_out, void* stream) {
    return f_stencil_jacobi_impl(prm, cell, uface, vface, part, x_in, b, sub, x_out, stream, false);
}

static int f_stencil_cheb_impl(const mpbp_stokes_params* prm, const double* cell, const double* uface,
                               const double* vface, const mpbp_row_part* part, const double* x_in,
                               const double* b, double c1, double c2, double* d, const double* sub,
                               double* x_out, void* stream, int store_d, bool fast = false) {
    FStencilDev P;
    int rc = make_fstencil(prm, cell, uface, vface, part, &P);
    if (rc) return rc;
    if (!x_in || !b || !d || !x_out || x_in == x_out) return set_error(MPBP_ERR_ARG, "f_stencil_cheb_step: bad vectors");
    return launch_fstencil(P, x_in, EpiCheb{x_in, b, nullptr, d, c1, c2, sub, x_out, store_d}, as_stream(stream),
                           fast);
}

int mpbp_f_stencil_cheb_step(const mpbp_stokes_params* prm, const double* cell, const double* uface,
                             const double* vface, const mpbp_row_part* part, const double* x_in,
                             const double* b, double c1, double c2, double* d, const double* sub,
                             double* x_out, void* stream) {
    return f_stencil_cheb_impl(prm, cell, uface, vface, part, x_in, b, c1, c2, d, sub, x_out, stream, 1);
}

static int make_pgstencil(const mpbp_stokes_params* prm, const double* cell, const mpbp_row_part* part, PGDev* P) {
    if (!prm || prm->n < 3 || !cell) return set_error(MPBP_ERR_ARG, "pg_stencil: needs n >= 3 and the cell thn table");
    if ((int64_t)prm->n * prm->n * 5 > INT32_MAX) return set_error(MPBP_ERR_OVERFLOW, "pg_stencil: n too large");
    const double dx = 1.0 / prm->n;   // as phase_D_row / phase_G_row evaluate 1.0 / dx, -1.0 / dx
    int r0 = 0, L = prm->n, h = 0, which = 0, ext = 0, oh = 0;
    if (part && part->halo > 0) {
        r0 = part->r0; L = part->rows; h = part->halo; which = part->which;
        ext = which == 3 ? part->ext : 0;
        oh = part->oh > 0 ? part->oh : h;
        if (L < 1 || r0 < 0 || r0 + L > prm->n || which < 0 || which > 3 || ext < 0 || ext + 1 > h || ext > oh ||
            h > L || oh > L)
            return set_error(MPBP_ERR_ARG, "pg_stencil: bad row partition");
    }
    *P = PGDev{prm->n, cell, prm->d_p, 1.0 / dx, -1.0 / dx, r0, L, h, which, ext, oh};
    P->unit = P->d_p == 1.0 && P->minv == -P->inv;
    return MPBP_OK;
}

}  // extern "C"

namespace {
template <class S>
int pg_spmv(const S& P, int32_t mode, const double* x, const double* z, double* y, hipStream_t st) {
    switch (mode) {
    case MPBP_SPMV_STORE: return launch_march(P, XPlain{x}, EpiStore{y}, pg_rows(), st);
    case MPBP_SPMV_ADD: return launch_march(P, XPlain{x}, EpiAdd{z, y}, pg_rows(), st);
    case MPBP_SPMV_RESID: return launch_march(P, XPlain{x}, EpiResid{z, y}, pg_rows(), st);
    default: return set_error(MPBP_ERR_ARG, "pg_stencil_spmv: unknown mode %d", mode);
    }
}
}  // namespace

extern "C" {

int mpbp_pg_stencil_spmv(const mpbp_stokes_params* prm, const double* cell, const mpbp_row_part* part, int32_t op,
                         int32_t mode, const double* x, const double* z, double* y, void* stream) {
    PGDev P;
    int rc = make_pgstencil(prm, cell, part, &P);
    if (rc) return rc;
    if (!x || !y || x == y || (mode != MPBP_SPMV_STORE && !z)) return set_error(MPBP_ERR_ARG, "pg_stencil_spmv: bad vectors");
    const hipStream_t st = as_stream(stream);
    switch (op) {
    case MPBP_PG_D: return pg_spmv(DStencilDev{P}, mode, x, z, y, st);
    case MPBP_PG_G: return pg_spmv(GStencilDev{P}, mode, x, z, y, st);
    case MPBP_PG_GTG: return pg_spmv(GtGStencilDev{P}, mode, x, z, y, st);
    default: return set_error(MPBP_ERR_ARG, "pg_stencil_spmv: unknown operator %d", op);
    }
}

int mpbp_gtg_stencil_jacobi_step(const mpbp_stokes_params* prm, const double* cell, const mpbp_row_part* part,
                                 const double* x_in, const double* b, const double* sub, double* x_out,
                                 void* stream) {
    PGDev P;
    int rc = make_pgstencil(prm, cell, part, &P);
    if (rc) return rc;
    if (!x_in || !b || !x_out || x_in == x_out) return set_error(MPBP_ERR_ARG, "gtg_stencil_jacobi_step: bad vectors");
    return launch_march(GtGStencilDev{P}, XPlain{x_in}, EpiJacobi{x_in, b, nullptr, sub, x_out}, pg_rows(),
                        as_stream(stream));
}

// dzero: d is +0.0 (a restart: multigrid post-smoothing), read as such instead of loaded -- no memset launch
static int gtg_stencil_cheb_impl(const mpbp_stokes_params* prm, const double* cell, const mpbp_row_part* part,
                                 const double* x_in, const double* b, double c1, double c2, double* d,
                                 const double* sub, double* x_out, void* stream, int store_d, bool dzero = false) {
    PGDev P;
    int rc = make_pgstencil(prm, cell, part, &P);
    if (rc) return rc;
    if (!x_in || !b || !d || !x_out || x_in == x_out) return set_error(MPBP_ERR_ARG, "gtg_stencil_cheb_step: bad vectors");
    const EpiCheb e{x_in, b, nullptr, d, c1, c2, sub, x_out, store_d};
    if (dzero) return launch_march(GtGStencilDev{P}, XPlain{x_in}, EpiZeroD<EpiCheb>{e}, pg_rows(), as_stream(stream));
    return launch_march(GtGStencilDev{P}, XPlain{x_in}, e, pg_rows(), as_stream(stream));
}

int mpbp_gtg_stencil_cheb_step(const mpbp_stokes_params* prm, const double* cell, const mpbp_row_part* part,
                               const double* x_in, const double* b, double c1, double c2, double* d,
                               const double* sub, double* x_out, void* stream) {
    return gtg_stencil_cheb_impl(prm, cell, part, x_in, b, c1, c2, d, sub, x_out, stream, 1);
}

}  // extern "C"

// ================================================ Gt_F_G, 13-point diamond ====
// Gt_F_G = ((-D) F) G couples every pressure cell with the 13 cells of the diamond |dr| + |dc| <= 2 (n >= 5;
// every structural product kept, so every row has exactly these 13 entries).  The diamond layout stores the
// values alone, slot-major (vals[s * N + cell], slots in (dr, dc) lexicographic order = the CSR row's column
// order for a cell whose diamond does not wrap), and rebuilds the columns from the grid: 104 B per row
// instead of SELL's 156 B of values + column indices.  A cell within two rows / columns of the periodic edge
// has its columns in wrapped order; its wave sorts the 13 products by wrapped column (a transposition
// network in registers) and sums them in that order -- the CSR SpMV's additions exactly, bit for bit.
// Rebuilding the values themselves from thn (as the D / G / Gt_G sweeps do) would cost ~1000 fp64
// operations per row (8 F rows of 10 entries, 80 + 96 products, first-touch accumulation): on this chip that
// is slower than streaming the 104 B.
namespace {
constexpr int kQSlots = 13;
__device__ __host__ constexpr int q13_dr(int s) { return s < 1 ? -2 : s < 4 ? -1 : s < 9 ? 0 : s < 12 ? 1 : 2; }
__device__ __host__ constexpr int q13_dc(int s) {
    return s < 1 ? 0 : s < 4 ? s - 2 : s < 9 ? s - 6 : s < 12 ? s - 10 : 0;
}
// slot of offset (dr, dc), or -1 outside the diamond
__device__ inline int q13_slot(int dr, int dc) {
    const int a = (dr < 0 ? -dr : dr) + (dc < 0 ? -dc : dc);
    if (a > 2) return -1;
    return dr == -2 ? 0 : dr == -1 ? 2 + dc : dr == 0 ? 6 + dc : dr == 1 ? 10 + dc : 12;
}
__device__ inline int q13_off(int d, int n) {   // periodic offset folded into [-2, 2], or 99
    if (d > 2) d -= n;
    if (d < -2) d += n;
    return (d >= -2 && d <= 2) ? d : 99;
}

// row0 (a row partition's block, mpbp_q13_build_rows): Q's row r is grid row (row0 + r / n) mod n, column r % n;
// vals holds Q->nrows cells per slot
__global__ void k_q13_fill(Csr Q, int32_t N, int32_t n, double* vals, int* bad, int32_t row0 = 0) {
    const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= N) return;
    int gr = row0 + r / n;
    gr = ((gr % n) + n) % n;
    const int gc = r - (r / n) * n;
    unsigned seen = 0;
    bool ok = Q.rp[r + 1] - Q.rp[r] == kQSlots;
    for (int32_t k = Q.rp[r]; ok && k < Q.rp[r + 1]; ++k) {
        const int32_t j = Q.ci[k];
        const int s = q13_slot(q13_off(j / n - gr, n), q13_off(j - (j / n) * n - gc, n));
        if (s < 0 || ((seen >> s) & 1u)) {
            ok = false;
            break;
        }
        seen |= 1u << s;
        vals[(int64_t)s * N + r] = Q.va[k];
    }
    if (!ok) atomicAdd(bad, 1);
}

// SYM (tolerance mode): Gt_F_G = G^T F G is symmetric, so its values are read from the upper half of the diamond
// alone -- slots 6 .. 12 ((0, 0) .. (2, 0)) at the cell, and slot 12 - s at the cell's neighbour (dr_s, dc_s) for the
// lower slots s = 0 .. 5, Q(c, c + o) = Q(c + o, c) -- 56 instead of 104 B of values per row (the mirrored reads are the
// neighbouring rows' own, cached).  The stored product is symmetric to rounding (|Q - Q^T| ~ 1.5e-16 |Q|): within the
// tolerance mode's bar, not bit-exact.
template <class Epi, bool SYM = false>
__global__ void __launch_bounds__(kBlock) k_q13(int32_t n, const double* __restrict__ vals,
                                                const double* __restrict__ x, Epi epi) {
    const int32_t N = n * n;
    const int32_t cell = xcd_swizzle(blockIdx.x, gridDim.x) * kBlock + threadIdx.x;
    if (cell >= N) return;
    const typename Epi::P pe = epi.pre(cell);
    const int gr = cell / n, gc = cell - (cell / n) * n;
    double v[kQSlots];
    const bool wraps = gr < 2 || gr >= n - 2 || gc < 2 || gc >= n - 2;
    if constexpr (SYM) {
#pragma unroll
        for (int s = 6; s < kQSlots; ++s) v[s] = vals[(int64_t)s * N + cell];
#pragma unroll
        for (int s = 0; s < 6; ++s) {
            int rr = gr + q13_dr(s), cc = gc + q13_dc(s);
            rr = rr < 0 ? rr + n : rr >= n ? rr - n : rr;
            cc = cc < 0 ? cc + n : cc >= n ? cc - n : cc;
            v[s] = vals[(int64_t)(12 - s) * N + rr * n + cc];
        }
    } else {
#pragma unroll
        for (int s = 0; s < kQSlots; ++s) v[s] = __builtin_nontemporal_load(vals + (int64_t)s * N + cell);
    }
    double acc = 0.0;
    if (!__any(wraps)) {
#pragma unroll
        for (int s = 0; s < kQSlots; ++s) acc += v[s] * x[cell + q13_dr(s) * n + q13_dc(s)];
    } else {   // (wrapped column, product) pairs sorted by column, then summed in that order
        int32_t key[kQSlots];
        double pr[kQSlots];
#pragma unroll
        for (int s = 0; s < kQSlots; ++s) {
            int rr = gr + q13_dr(s), cc = gc + q13_dc(s);
            rr = rr < 0 ? rr + n : rr >= n ? rr - n : rr;
            cc = cc < 0 ? cc + n : cc >= n ? cc - n : cc;
            key[s] = rr * n + cc;
            pr[s] = v[s] * x[key[s]];
        }
#pragma unroll
        for (int round = 0; round < kQSlots; ++round) {
#pragma unroll
            for (int i = round & 1; i + 1 < kQSlots; i += 2) {
                const bool sw = key[i] > key[i + 1];
                const int32_t ka = key[i], kb = key[i + 1];
                const double pa = pr[i], pb = pr[i + 1];
                key[i] = sw ? kb : ka;
                key[i + 1] = sw ? ka : kb;
                pr[i] = sw ? pb : pa;
                pr[i + 1] = sw ? pa : pb;
            }
        }
#pragma unroll
        for (int s = 0; s < kQSlots; ++s) acc += pr[s];
    }
    epi(cell, acc, pe);
}

// The symmetric-half read on a row partition (the owned grid rows [r0, r0 + L) of every rank): vals holds the diamond
// of grid rows r0 - 2 .. r0 + L - 1 (L + 2 rows: the lower slots of the first owned rows come from the two rows above),
// x the owned rows with h >= 2 ghost rows each side (ext_row layout).  Every value, product and the order of the sum
// (slot order, or for cells whose diamond wraps the periodic edge the wrapped global column order) are k_q13<SYM>'s:
// the rank's rows of the one-GPU result bit for bit.
template <class Epi>
__global__ void __launch_bounds__(kBlock) k_q13p(int32_t n, int32_t r0, int32_t L, int32_t h,
                                                 const double* __restrict__ vals, const double* __restrict__ x, Epi epi) {
    const int32_t M = (L + 2) * n;   // cells per slot of the row block
    const int32_t cell = xcd_swizzle(blockIdx.x, gridDim.x) * kBlock + threadIdx.x;
    if (cell >= L * n) return;
    const typename Epi::P pe = epi.pre(cell);
    const int lr = cell / n, gc = cell - (cell / n) * n, gr = r0 + lr;
    const int32_t bc = (lr + 2) * n + gc;   // the cell in the row block
    auto wrapc = [&](int c) { return c < 0 ? c + n : c >= n ? c - n : c; };
    double v[kQSlots];
#pragma unroll
    for (int s = 6; s < kQSlots; ++s) v[s] = vals[(int64_t)s * M + bc];
#pragma unroll
    for (int s = 0; s < 6; ++s) v[s] = vals[(int64_t)(12 - s) * M + (lr + 2 + q13_dr(s)) * n + wrapc(gc + q13_dc(s))];
    double pr[kQSlots];
    int32_t key[kQSlots];
#pragma unroll
    for (int s = 0; s < kQSlots; ++s) {
        const int cc = wrapc(gc + q13_dc(s));
        int rr = gr + q13_dr(s);
        rr = rr < 0 ? rr + n : rr >= n ? rr - n : rr;
        key[s] = rr * n + cc;
        pr[s] = v[s] * x[ext_row(1, 0, lr + q13_dr(s), L, h, n) + cc];
    }
    double acc = 0.0;
    const bool wraps = gr < 2 || gr >= n - 2 || gc < 2 || gc >= n - 2;
    if (!__any(wraps)) {
#pragma unroll
        for (int s = 0; s < kQSlots; ++s) acc += pr[s];
    } else {
#pragma unroll
        for (int round = 0; round < kQSlots; ++round) {
#pragma unroll
            for (int i = round & 1; i + 1 < kQSlots; i += 2) {
                const bool sw = key[i] > key[i + 1];
                const int32_t ka = key[i], kb = key[i + 1];
                const double pa = pr[i], pb = pr[i + 1];
                key[i] = sw ? kb : ka;
                key[i + 1] = sw ? ka : kb;
                pr[i] = sw ? pb : pa;
                pr[i + 1] = sw ? pa : pb;
            }
        }
#pragma unroll
        for (int s = 0; s < kQSlots; ++s) acc += pr[s];
    }
    epi(cell, acc, pe);
}

// max |Q(c, c + o) - Q(c + o, c)| over the diamond (slot s at c against slot 12 - s at c + o) and max |Q|: whether the
// symmetric-half read (k_q13<SYM>) may stand in for the stored product.  Non-negative doubles order like their bits.
__global__ void __launch_bounds__(kBlock) k_q13_asym(int32_t n, const double* __restrict__ vals,
                                                     unsigned long long* out) {
    const int32_t N = n * n;
    const int32_t cell = blockIdx.x * kBlock + threadIdx.x;
    double asym = 0.0, amax = 0.0;
    if (cell < N) {
        const int gr = cell / n, gc = cell - (cell / n) * n;
#pragma unroll
        for (int s = 0; s < kQSlots; ++s) amax = fmax(amax, fabs(vals[(int64_t)s * N + cell]));
#pragma unroll
        for (int s = 0; s < 6; ++s) {
            int rr = gr + q13_dr(s), cc = gc + q13_dc(s);
            rr = rr < 0 ? rr + n : rr >= n ? rr - n : rr;
            cc = cc < 0 ? cc + n : cc >= n ? cc - n : cc;
            asym = fmax(asym, fabs(vals[(int64_t)s * N + cell] - vals[(int64_t)(12 - s) * N + rr * n + cc]));
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        asym = fmax(asym, __shfl_xor(asym, o));
        amax = fmax(amax, __shfl_xor(amax, o));
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(out, (unsigned long long)__double_as_longlong(asym));
        atomicMax(out + 1, (unsigned long long)__double_as_longlong(amax));
    }
}

template <class Epi>
int launch_q13(int32_t n, const double* vals, const double* x, Epi epi, hipStream_t st, bool sym = false) {
    if (sym) k_q13<Epi, true><<<grid_for((int64_t)n * n), kBlock, 0, st>>>(n, vals, x, epi);
    else k_q13<Epi, false><<<grid_for((int64_t)n * n), kBlock, 0, st>>>(n, vals, x, epi);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

// ---- x_b = Gt_F_G x_a matrix-free, tolerance mode (k_qmf, kernel option q13_mf) ----
// solve.py:247-249 forms Gt_F_G = ((-D) F) G once and the apply multiplies it (k_q13: 7 or 13 stored diamond values
// per row, 75-126 MB per apply at 1024^2).  Here the product is applied as its three factors on a 32 x 16 tile of
// pressure cells: y = G x_a on the tile + 1 (its four velocity rows, GxBT::b_at's entries: d_p (+-inv g) with g the
// face's thn average), z = F y on the tile's cells plus their east / south faces (the tolerance-mode rows,
// FStencilFast::rows4_co), then x_b = -(D z) (DStencilDev's entries: +-inv times the face average).  x_a and thn are
// staged over the tile + 2, y and z live in LDS (z over y), only the faces of the z cells and x_b touch memory
// besides: HBM 8 B x_a + 24 B thn / faces + 8 B x_b per cell = 42 MB at 1024^2, against k_q13<SYM>'s 76 MB.  The same
// operator as the stored product; its sums in another order (a few ulp per entry, within north_star's 1e-12 on the
// apply: tests/test_gpu_fast.py, test_gpu_q13.py).  One GPU, whole grid, fast numerics, matrix-free F / D / G.
constexpr int kQmW = 32, kQmH = 16;
constexpr int kQxW = kQmW + 4, kQxH = kQmH + 4, kQxN = kQxW * kQxH;   // x_a, thn: the tile + 2
constexpr int kQyW = kQmW + 3, kQyH = kQmH + 3, kQyN = kQyW * kQyH;   // y = G x_a: rows / columns -1 .. +TW+1
constexpr int kQzW = kQmW + 1, kQzH = kQmH + 1, kQzN = kQzW * kQzH;   // z = F y: the tile's cells + east / south
template <class Epi>
__global__ void __launch_bounds__(256) MPBP_LDS_READS k_qmf(FStencilFast P, PGDev G, const double* __restrict__ xa,
                                                            Epi epi) {
    __shared__ double ts[kQxN], xs[kQxN];
    __shared__ double ys[4 * kQyN];   // y; then z (4 * kQzN <= 4 * kQyN)
    const int n = P.n;
    const int tx = (n + kQmW - 1) / kQmW;
    const int bk = xcd_swizzle(blockIdx.x, gridDim.x);
    const int r0 = (bk / tx) * kQmH, c0 = (bk % tx) * kQmW;
    const int tid = threadIdx.x;
    constexpr int IX = (kQxN + 255) / 256, IZ = (kQzN + 255) / 256;
    {   // x_a and thn over the tile + 2; the faces of this lane's z cells -- every load before the first LDS store
        double vt[IX], vx[IX];
#pragma unroll
        for (int it = 0; it < IX; ++it) {
            const int i = tid + it * 256;
            if (i < kQxN) {
                const int sr = i / kQxW, sc = i - sr * kQxW;
                const int32_t k = P.wrap(r0 - 2 + sr) * n + P.wrap(c0 - 2 + sc);
                vt[it] = P.cell[k];
                vx[it] = xa[k];
            }
        }
#pragma unroll
        for (int it = 0; it < IX; ++it) {
            const int i = tid + it * 256;
            if (i < kQxN) {
                ts[i] = vt[it];
                xs[i] = vx[it];
            }
        }
    }
    double fu[IZ], fv[IZ];
#pragma unroll
    for (int it = 0; it < IZ; ++it) {
        const int i = tid + it * 256;
        if (i < kQzN) {
            const int zr = i / kQzW, zc = i - zr * kQzW;
            const int32_t k = P.wrap(r0 + zr) * n + P.wrap(c0 + zc);
            fu[it] = P.uface[k];
            fv[it] = P.vface[k];
        }
    }
    __syncthreads();
    const TTileT<kQxW> tt{ts, r0 - 2, c0 - 2};
    const XTileT<kQxW, 1> xt{xs, r0 - 2, c0 - 2};
    // y = G x_a: velocity rows (u_n, v_n, u_s, v_s) at (r, c) -- u on the cell's west face, v on its north face
    for (int i = tid; i < kQyN; i += 256) {
        const int vr = r0 - 1 + i / kQyW, vc = c0 - 1 + i % kQyW;
        const double xc = xt.X(0, vr, vc), xw = xt.X(0, vr, vc - 1), xn = xt.X(0, vr - 1, vc);
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const double t0 = tt.T(p, vr, vc);
            const double gu = 0.5 * (t0 + tt.T(p, vr, vc - 1)), gv = 0.5 * (t0 + tt.T(p, vr - 1, vc));
            ys[(2 * p) * kQyN + i] = (G.d_p * (G.minv * gu)) * xw + (G.d_p * (G.inv * gu)) * xc;
            ys[(2 * p + 1) * kQyN + i] = (G.d_p * (G.inv * gv)) * xn + (G.d_p * (G.minv * gv)) * xc;
        }
    }
    __syncthreads();
    // z = F y on the tile's cells and their east / south neighbours (held in registers, then over y)
    double zv[IZ][4];
    {
        const XTileT<kQyW, kQyH> yt{ys, r0 - 1, c0 - 1};
#pragma unroll
        for (int it = 0; it < IZ; ++it) {
            const int i = tid + it * 256;
            if (i >= kQzN) break;
            const int vr = r0 + i / kQzW, vc = c0 + i % kQzW;
            const typename FStencilFast::Co k = P.coeffs(P.nb(tt, vr, vc));
            P.rows4_co(vr, vc, k, P.weights(FStencilDev::Cell{{fu[it], fv[it]}}), yt, zv[it]);
        }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < IZ; ++it) {
        const int i = tid + it * 256;
        if (i >= kQzN) break;
#pragma unroll
        for (int f = 0; f < 4; ++f) ys[f * kQzN + i] = zv[it][f];
    }
    __syncthreads();
    // x_b = -(D z) on the tile (the pressure row: u at the west / east faces, v at the north / south faces, per phase)
    const XTileT<kQzW, kQzH> zt{ys, r0, c0};
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        const int vr = r0 + tid / kQmW + 8 * m, vc = c0 + tid % kQmW;
        if (vr >= n || vc >= n) continue;
        const int32_t row = vr * n + vc;
        const typename Epi::P pe = epi.pre(row);
        double acc = 0.0;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const double t0 = tt.T(q, vr, vc);
            const double uC = (G.minv * (0.5 * (t0 + tt.T(q, vr, vc - 1)))) * zt.X(2 * q, vr, vc);
            const double uE = (G.inv * (0.5 * (t0 + tt.T(q, vr, vc + 1)))) * zt.X(2 * q, vr, vc + 1);
            const double vC = (G.inv * (0.5 * (t0 + tt.T(q, vr - 1, vc)))) * zt.X(2 * q + 1, vr, vc);
            const double vS = (G.minv * (0.5 * (t0 + tt.T(q, vr + 1, vc)))) * zt.X(2 * q + 1, vr + 1, vc);
            acc += uC;
            acc += uE;
            acc += vC;
            acc += vS;
        }
        epi(row, -acc, pe);
    }
}
// whole grid, one GPU: the staged window (tile + 2) wraps at most once
inline bool qmf_ok_n(int n) { return n >= kQxW && n >= kQxH; }
// The plan's Gt_F_G product by k_qmf: kernel option q13_mf, tolerance mode, one GPU, matrix-free F (fast rows) and D / G.
bool qmf_ok(const mpbp_schur_plan* p) {
    return KO().q13_mf && p->f_numerics == MPBP_NUMERICS_FAST && p->f_stencil && p->pg_stencil && !p->halo &&
           p->f_cell && p->f_uface && p->f_vface && qmf_ok_n(p->f_prm.n);
}
template <class Epi>
int launch_qmf(const mpbp_schur_plan* p, const double* xa, Epi epi, hipStream_t st) {
    FStencilDev Pd;
    int rc = make_fstencil(&p->f_prm, p->f_cell, p->f_uface, p->f_vface, nullptr, &Pd);
    if (rc) return rc;
    PGDev G;
    rc = make_pgstencil(&p->f_prm, p->f_cell, nullptr, &G);
    if (rc) return rc;
    const FStencilFast P{Pd};
    if (!qmf_ok_n(P.n) || !xa || xa == epi.y) return set_error(MPBP_ERR_ARG, "qmf: whole grid n >= 36, vectors");
    const int64_t tiles = (int64_t)((P.n + kQmW - 1) / kQmW) * ((P.n + kQmH - 1) / kQmH);
    k_qmf<Epi><<<(unsigned)tiles, 256, 0, st>>>(P, G, xa, epi);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}
}  // namespace

extern "C" {
int mpbp_svl_spmv(const mpbp_svl* V, const mpbp_csr* A, int32_t mode, const double* x, const double* z, double* y,
                  void* stream) {
    int rc = check_csr(A);
    if (!rc) rc = check_svl(V, A);
    if (rc) return rc;
    if (!x || !y || (mode != MPBP_SPMV_STORE && !z)) return set_error(MPBP_ERR_ARG, "svl_spmv: bad vectors");
    return svl_spmv(V, A, mode, x, z, y, as_stream(stream));
}

int mpbp_svl_cheb_step(const mpbp_svl* V, const mpbp_csr* A, const double* x_in, const double* b, const double* diag,
                       double c1, double c2, double* d, const double* sub, double* x_out, void* stream) {
    int rc = check_csr(A);
    if (!rc) rc = check_svl(V, A);
    if (rc) return rc;
    if (!x_in || !b || !diag || !d || !x_out || x_in == x_out) return set_error(MPBP_ERR_ARG, "svl_cheb_step: bad vectors");
    return svl_cheb(V, A, x_in, b, diag, c1, c2, d, sub, x_out, as_stream(stream), 1, false);
}

int mpbp_q13_build(const mpbp_csr* Q, int32_t n, double* vals, void* stream) {
    int rc = check_csr(Q);
    if (rc) return rc;
    if (n < 5 || (int64_t)n * n > INT32_MAX / kQSlots || Q->nrows != n * n || Q->ncols != n * n || !vals)
        return set_error(MPBP_ERR_ARG, "q13_build: needs an n^2 x n^2 operator, n >= 5");
    const hipStream_t st = as_stream(stream);
    int* bad = nullptr;
    MPBP_HIP(hipMallocAsync((void**)&bad, sizeof(int), st));
    MPBP_HIP(hipMemsetAsync(bad, 0, sizeof(int), st));
    k_q13_fill<<<grid_for((int64_t)n * n), kBlock, 0, st>>>(to_csr(Q), n * n, n, vals, bad);
    MPBP_HIP(hipGetLastError());
    int nbad = 0;
    MPBP_HIP(hipMemcpyAsync(&nbad, bad, sizeof(int), hipMemcpyDeviceToHost, st));
    MPBP_HIP(hipFreeAsync(bad, st));
    MPBP_HIP(hipStreamSynchronize(st));
    if (nbad) return set_error(MPBP_ERR_ARG, "q13_build: %d rows are not the 13-point diamond", nbad);
    return MPBP_OK;
}

int mpbp_q13_build_rows(const mpbp_csr* Q, int32_t n, int32_t row0, double* vals, void* stream) {
    int rc = check_csr(Q);
    if (rc) return rc;
    if (n < 5 || Q->nrows < n || Q->nrows % n || Q->nrows > (n + 2) * n || (int64_t)Q->nrows > INT32_MAX / kQSlots ||
        Q->ncols != n * n || !vals)
        return set_error(MPBP_ERR_ARG, "q13_build_rows: needs whole grid rows of an n^2-column operator, n >= 5");
    const hipStream_t st = as_stream(stream);
    int* bad = nullptr;
    MPBP_HIP(hipMallocAsync((void**)&bad, sizeof(int), st));
    MPBP_HIP(hipMemsetAsync(bad, 0, sizeof(int), st));
    k_q13_fill<<<grid_for((int64_t)Q->nrows), kBlock, 0, st>>>(to_csr(Q), Q->nrows, n, vals, bad, row0);
    MPBP_HIP(hipGetLastError());
    int nbad = 0;
    MPBP_HIP(hipMemcpyAsync(&nbad, bad, sizeof(int), hipMemcpyDeviceToHost, st));
    MPBP_HIP(hipFreeAsync(bad, st));
    MPBP_HIP(hipStreamSynchronize(st));
    if (nbad) return set_error(MPBP_ERR_ARG, "q13_build_rows: %d rows are not the 13-point diamond", nbad);
    return MPBP_OK;
}

int mpbp_q13_asymmetry(int32_t n, const double* vals, double* out, void* stream) {
    if (n < 5 || (int64_t)n * n > INT32_MAX / kQSlots || !vals || !out) return set_error(MPBP_ERR_ARG, "q13_asymmetry: bad args");
    const hipStream_t st = as_stream(stream);
    unsigned long long* dev = nullptr;
    MPBP_HIP(hipMallocAsync((void**)&dev, 2 * sizeof(unsigned long long), st));
    MPBP_HIP(hipMemsetAsync(dev, 0, 2 * sizeof(unsigned long long), st));
    k_q13_asym<<<grid_for((int64_t)n * n), kBlock, 0, st>>>(n, vals, dev);
    MPBP_HIP(hipGetLastError());
    unsigned long long h[2] = {0, 0};
    MPBP_HIP(hipMemcpyAsync(h, dev, sizeof(h), hipMemcpyDeviceToHost, st));
    MPBP_HIP(hipFreeAsync(dev, st));
    MPBP_HIP(hipStreamSynchronize(st));
    memcpy(out, h, sizeof(h));
    return MPBP_OK;
}

int mpbp_q13_spmv(int32_t n, const double* vals, int32_t mode, const double* x, const double* z, double* y,
                  void* stream) {
    if (n < 5 || (int64_t)n * n > INT32_MAX / kQSlots || !vals || !x || !y || (mode != MPBP_SPMV_STORE && !z))
        return set_error(MPBP_ERR_ARG, "q13_spmv: bad args");
    const hipStream_t st = as_stream(stream);
    switch (mode) {
    case MPBP_SPMV_STORE: return launch_q13(n, vals, x, EpiStore{y}, st);
    case MPBP_SPMV_ADD: return launch_q13(n, vals, x, EpiAdd{z, y}, st);
    case MPBP_SPMV_RESID: return launch_q13(n, vals, x, EpiResid{z, y}, st);
    default: return set_error(MPBP_ERR_ARG, "q13_spmv: unknown mode %d", mode);
    }
}
}  // extern "C"

// ======================================================= Schur apply ====
namespace {

struct Ctx {
    const mpbp_schur_plan* p;
    hipStream_t st;
};

// Profiling events are recorded only on eager (uncaptured) launches: a capturing stream skips them.
hipError_t record_event(hipEvent_t ev, hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    hipError_t e = hipStreamIsCapturing(st, &cs);
    if (e != hipSuccess) return e;
    return cs == hipStreamCaptureStatusNone ? hipEventRecord(ev, st) : hipSuccess;
}

// One operator of the apply, restricted to interior or boundary rows, in CSR or SELL form.
enum StencilOp { SOP_NONE = 0, SOP_F, SOP_D, SOP_G, SOP_GTG };

struct OpRef {
    const mpbp_csr* csr;
    const mpbp_rowblocks* blk;
    const mpbp_sell* sell;
    const mpbp_schur_plan* stencil;   // rows recomputed from the plan's thn tables (sop says which operator)
    bool empty;
    int32_t which;                    // stencil rows: 0 all, 1 interior, 2 boundary, 3 owned + ext ghost rows
    int32_t sop;
    int32_t ext = 0;                  // which = 3
    int32_t grp = 0;                  // CSR rows through k_csr_grp (multigrid small levels)
    const mpbp_svl* svl = nullptr;    // stencil-values layout of csr (multigrid large levels)
    const struct MgGal* gal = nullptr;   // level 1 of an F hierarchy applied as R0 (F (P0 x)) (tolerance mode)
};

// Level 1 of the F hierarchy without its Galerkin matrix (tolerance mode): A_1 x = R_0 (F (P_0 x)) -- the same operator
// as the stored product (mg_oracle's R A P) in exact arithmetic -- from the matrix-free transfers and the tolerance-mode
// F sweep of level 0, through two fine-size temporaries (level 0's residual and direction buffers, dead while level 1
// runs).  Per application: x_c and the thn read, two fine vectors written and read once, the level-1 epilogue operands;
// ~115 MB at 1024^2 instead of streaming the 40-entry coarse rows' values (386 MB).
struct MgGal {
    const mpbp_mg* m;
    OpRef fine;     // level 0's whole-grid F stencil
    double* t0;     // fine-size temporaries
    double* t1;
};

// F and D read velocity vectors (f_part), G and Gt_G pressure vectors (p_part); D writes a pressure vector
// and G a velocity one (output ghost depth oh).
inline mpbp_row_part stencil_part(const OpRef& o) {
    const mpbp_schur_plan* p = o.stencil;
    mpbp_row_part q = (o.sop == SOP_F || o.sop == SOP_D) ? p->f_part : p->p_part;
    q.which = q.halo > 0 ? o.which : 0;
    q.ext = q.which == 3 ? o.ext : 0;
    q.oh = o.sop == SOP_D ? p->p_part.halo : o.sop == SOP_G ? p->f_part.halo : 0;
    return q;
}

template <class Epi>
int mg_transfer_mf(const mpbp_mg* m, int l, int32_t which, int32_t nrows, const double* x, Epi epi, hipStream_t st);
int op_spmv(const OpRef& o, int32_t mode, const double* x, const double* z, double* y, hipStream_t st);
// t1 = F (P_0 x): the first two stages of a matrix-free Galerkin level-1 product
int gal_fp(const MgGal& g, const double* x, hipStream_t st) {
    const int rc = mg_transfer_mf(g.m, 0, MPBP_MG_P, g.m->levels[0].P.nrows, x, EpiStore{g.t0}, st);
    return rc ? rc : op_spmv(g.fine, MPBP_SPMV_STORE, g.t0, nullptr, g.t1, st);
}
template <class Epi>
int gal_r(const MgGal& g, Epi epi, hipStream_t st) {
    return mg_transfer_mf(g.m, 0, MPBP_MG_R, g.m->levels[0].R.nrows, g.t1, epi, st);
}

// The whole level-1 product as one k_gal1 launch (KO().mg_galerkin_mf == 2): four fields, a grid the staged windows wrap once.
// gal_fused_ok: whether gal_fused takes the one-launch form for this level (else the caller runs the three launches)
// Under a row partition (g.m->part_levels > 0) level 1 is either the whole replicated level (part_levels == 1: the
// one-GPU launch on every rank) or row-partitioned (> 1: the PART launch over the owned coarse rows, its x read with
// >= 2 ghost rows each side -- the windows' reach).
bool gal_part(const MgGal& g, G1Part* q) {
    *q = G1Part{};
    if (g.m->part_levels <= 1) return true;
    const mpbp_mg_level& L1 = g.m->levels[1];
    const int nc = g.fine.stencil->f_prm.n / 2, nf = g.fine.sop == SOP_GTG ? 1 : 4;
    if (L1.nrows == nf * nc * nc && L1.part_r0 == 0) return true;   // one rank: its owned rows are the whole level
    if (nc <= 0 || L1.nrows % (nf * nc) || L1.part_h < 2 || L1.part_r0 < 0) return false;
    q->r0 = L1.part_r0;
    q->L = L1.nrows / (nf * nc);
    q->h = L1.part_h;
    return q->L >= q->h && q->r0 + q->L <= nc;
}
bool gal_fused_ok(const MgGal& g) {
    const mpbp_schur_plan* p = g.fine.stencil;
    if (KO().mg_galerkin_mf != 2 || p->f_prm.n < 2 * kG1CW || (p->f_prm.n & 1)) return false;
    G1Part q;
    if (!gal_part(g, &q)) return false;
    if (g.fine.sop == SOP_GTG) return g.m->tr_nfields == 1 && g.m->tr_ky[0] == MPBP_MG_CELL && g.m->tr_kx[0] == MPBP_MG_CELL;
    return g.m->tr_nfields == 4;
}
template <class Epi, class XS = XPlain>
int gal_fused(const MgGal& g, XS x, Epi epi, hipStream_t st, bool* done) {
    *done = false;
    const mpbp_schur_plan* p = g.fine.stencil;
    if (!gal_fused_ok(g)) return MPBP_OK;
    G1Part q;
    gal_part(g, &q);
    const bool part = q.L > 0;
    if (g.fine.sop == SOP_GTG) {   // the pressure hierarchy: one field, cell-centred (mg.FIELDS_PRESSURE)
        PGDev Pg;
        const int rc = make_pgstencil(&p->f_prm, p->f_cell, nullptr, &Pg);
        if (rc) return rc;
        const int nc = p->f_prm.n / 2;
        const int64_t tiles = (int64_t)((nc + kG1W - 1) / kG1W) * (((part ? q.L : nc) + kG1PH2 - 1) / kG1PH2);
        if (part) k_gal1p<Epi, XS, true><<<(unsigned)tiles, 256, 0, st>>>(GtGStencilDev{Pg}, x, epi, q);
        else k_gal1p<Epi, XS><<<(unsigned)tiles, 256, 0, st>>>(GtGStencilDev{Pg}, x, epi, q);
        MPBP_HIP(hipGetLastError());
        *done = true;
        return MPBP_OK;
    }
    FStencilDev Pd;
    const int rc = make_fstencil(&p->f_prm, p->f_cell, p->f_uface, p->f_vface, nullptr, &Pd);
    if (rc) return rc;
    MgFields F{};
    F.nfields = 4;
    for (int f = 0; f < 4; ++f) {
        F.ky[f] = g.m->tr_ky[f];
        F.kx[f] = g.m->tr_kx[f];
    }
    const int nc = p->f_prm.n / 2;
    const int64_t tiles = (int64_t)((nc + kGFW - 1) / kGFW) * (((part ? q.L : nc) + kGFH - 1) / kGFH);
    bool mac = true;   // the F hierarchy's MAC kinds (mg.FIELDS_VELOCITY)
    for (int f = 0; f < 4; ++f)
        mac = mac && F.ky[f] == ((f & 1) ? MPBP_MG_NODE : MPBP_MG_CELL) && F.kx[f] == ((f & 1) ? MPBP_MG_CELL : MPBP_MG_NODE);
    if (part && !mac) return set_error(MPBP_ERR_ARG, "mg: a row-partitioned matrix-free level 1 needs the MAC kinds");
    if (part) k_gal1<Epi, true, XS, true><<<(unsigned)tiles, 256, 0, st>>>(FStencilFast{Pd}, F, x, epi, q);
    else if (mac) k_gal1<Epi, true, XS><<<(unsigned)tiles, 256, 0, st>>>(FStencilFast{Pd}, F, x, epi, q);
    else k_gal1<Epi, false, XS><<<(unsigned)tiles, 256, 0, st>>>(FStencilFast{Pd}, F, x, epi, q);
    MPBP_HIP(hipGetLastError());
    *done = true;
    return MPBP_OK;
}

MgFields mg_fields(const mpbp_mg* m);
// The post-smoothing's first sweep on a matrix-free level 1 with level 2's correction folded in (k_gal1<PRO>,
// k_gal1p<PRO>): x = x_in + P_1 x_c staged, then the sweep from d = 0 -- the prolongation launch and that sweep's
// operations.  One GPU (or a replicated level 1), the F hierarchy's MAC kinds, the one-launch form.
bool gal_pro_ok(const MgGal& g) {
    G1Part q;
    if (!gal_fused_ok(g) || !gal_part(g, &q) || q.L || g.m->nlevels < 3 || !KO().mg_fuse_l0) return false;
    const int nf = g.fine.sop == SOP_GTG ? 1 : 4;   // (gal_fused_ok: the pressure hierarchy's one cell-centred field)
    if (nf == 4)
        for (int f = 0; f < 4; ++f)
            if (g.m->tr_ky[f] != ((f & 1) ? MPBP_MG_NODE : MPBP_MG_CELL) ||
                g.m->tr_kx[f] != ((f & 1) ? MPBP_MG_CELL : MPBP_MG_NODE))
                return false;
    const int n = g.fine.stencil->f_prm.n, n2 = n / 4;
    return n % 4 == 0 && n2 >= kG1QW && g.m->levels[2].nrows == nf * n2 * n2;
}
int gal_pro(const MgGal& g, const double* x, const double* xc, const EpiZeroD<EpiCheb>& epi, hipStream_t st) {
    const mpbp_schur_plan* p = g.fine.stencil;
    const int nc = p->f_prm.n / 2;
    if (g.fine.sop == SOP_GTG) {
        PGDev Pg;
        const int rc = make_pgstencil(&p->f_prm, p->f_cell, nullptr, &Pg);
        if (rc) return rc;
        const int64_t tiles = (int64_t)((nc + kG1W - 1) / kG1W) * ((nc + kG1PH2 - 1) / kG1PH2);
        k_gal1p<EpiZeroD<EpiCheb>, XPlain, false, true><<<(unsigned)tiles, 256, 0, st>>>(GtGStencilDev{Pg}, XPlain{x},
                                                                                         epi, G1Part{}, xc);
        MPBP_HIP(hipGetLastError());
        return MPBP_OK;
    }
    FStencilDev Pd;
    const int rc = make_fstencil(&p->f_prm, p->f_cell, p->f_uface, p->f_vface, nullptr, &Pd);
    if (rc) return rc;
    const int64_t tiles = (int64_t)((nc + kGFW - 1) / kGFW) * ((nc + kGFH - 1) / kGFH);
    k_gal1<EpiZeroD<EpiCheb>, true, XPlain, false, true><<<(unsigned)tiles, 256, 0, st>>>(
        FStencilFast{Pd}, mg_fields(g.m), XPlain{x}, epi, G1Part{}, xc);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int op_spmv(const OpRef& o, int32_t mode, const double* x, const double* z, double* y, hipStream_t st) {
    if (o.empty) return MPBP_OK;
    if (o.gal) {
        bool done = false;
        int rf = MPBP_OK;
        switch (mode) {
        case MPBP_SPMV_STORE: rf = gal_fused(*o.gal, XPlain{x}, EpiStore{y}, st, &done); break;
        case MPBP_SPMV_ADD: rf = gal_fused(*o.gal, XPlain{x}, EpiAdd{z, y}, st, &done); break;
        case MPBP_SPMV_RESID: rf = gal_fused(*o.gal, XPlain{x}, EpiResid{z, y}, st, &done); break;
        default: break;
        }
        if (rf || done) return rf;
        const int rc = gal_fp(*o.gal, x, st);
        if (rc) return rc;
        switch (mode) {
        case MPBP_SPMV_STORE: return gal_r(*o.gal, EpiStore{y}, st);
        case MPBP_SPMV_ADD: return gal_r(*o.gal, EpiAdd{z, y}, st);
        case MPBP_SPMV_RESID: return gal_r(*o.gal, EpiResid{z, y}, st);
        default: return set_error(MPBP_ERR_ARG, "galerkin spmv: unknown mode %d", mode);
        }
    }
    if (o.stencil) {
        const mpbp_schur_plan* p = o.stencil;
        const mpbp_row_part q = stencil_part(o);
        if (o.sop == SOP_F)
            return mpbp_f_stencil_spmv(&p->f_prm, p->f_cell, p->f_uface, p->f_vface, &q,
                                       mode | (p->f_numerics == MPBP_NUMERICS_FAST ? MPBP_SPMV_FAST : 0), x, z, y,
                                       (void*)st);
        const int32_t op = o.sop == SOP_D ? MPBP_PG_D : o.sop == SOP_G ? MPBP_PG_G : MPBP_PG_GTG;
        return mpbp_pg_stencil_spmv(&p->f_prm, p->f_cell, &q, op, mode, x, z, y, (void*)st);
    }
    if (o.grp) return grp_spmv(o.csr, mode, x, z, y, st);
    if (o.svl) return svl_spmv(o.svl, o.csr, mode, x, z, y, st);
    return o.sell ? mpbp_sell_spmv(o.sell, mode, x, z, y, (void*)st)
                  : mpbp_spmv(o.csr, o.blk, mode, x, z, y, (void*)st);
}
int op_jacobi(const OpRef& o, const double* xin, const double* b, const double* dg, const double* sub, double* xo,
              hipStream_t st) {
    if (o.empty) return MPBP_OK;
    if (o.stencil) {
        const mpbp_schur_plan* p = o.stencil;
        const mpbp_row_part q = stencil_part(o);
        if (o.sop == SOP_F)
            return f_stencil_jacobi_impl(&p->f_prm, p->f_cell, p->f_uface, p->f_vface, &q, xin, b, sub, xo, (void*)st,
                                         p->f_numerics == MPBP_NUMERICS_FAST);
        return mpbp_gtg_stencil_jacobi_step(&p->f_prm, p->f_cell, &q, xin, b, sub, xo, (void*)st);
    }
    return o.sell ? mpbp_sell_jacobi_step(o.sell, xin, b, dg, sub, xo, (void*)st)
                  : mpbp_jacobi_step(o.csr, o.blk, xin, b, dg, sub, xo, (void*)st);
}
int op_cheb(const OpRef& o, const double* xin, const double* b, const double* dg, double c1, double c2, double* d,
            const double* sub, double* xo, hipStream_t st, int store_d, bool dzero = false) {
    if (o.empty) return MPBP_OK;
    if (o.gal) {
        // (dzero: a restart's first sweep reads d as +0.0 -- no memset of the direction)
        auto run = [&](const auto& epi) {
            bool done = false;
            const int rf = gal_fused(*o.gal, XPlain{xin}, epi, st, &done);
            if (rf || done) return rf;
            const int rc = gal_fp(*o.gal, xin, st);
            return rc ? rc : gal_r(*o.gal, epi, st);
        };
        const EpiCheb e{xin, b, dg, d, c1, c2, sub, xo, store_d};
        return dzero ? run(EpiZeroD<EpiCheb>{e}) : run(e);
    }
    if (o.grp) return grp_cheb(o.csr, xin, b, dg, c1, c2, d, sub, xo, st, store_d, dzero);
    if (o.svl) return svl_cheb(o.svl, o.csr, xin, b, dg, c1, c2, d, sub, xo, st, store_d, dzero);
    if (dzero && !(o.stencil && o.sop == SOP_GTG))
        return set_error(MPBP_ERR_ARG, "cheb: a zero direction needs the grouped / stencil-values / Gt_G stencil path");
    if (o.stencil) {
        const mpbp_schur_plan* p = o.stencil;
        const mpbp_row_part q = stencil_part(o);
        if (o.sop == SOP_F)
            return f_stencil_cheb_impl(&p->f_prm, p->f_cell, p->f_uface, p->f_vface, &q, xin, b, c1, c2, d, sub,
                                       xo, (void*)st, store_d, p->f_numerics == MPBP_NUMERICS_FAST);
        return gtg_stencil_cheb_impl(&p->f_prm, p->f_cell, &q, xin, b, c1, c2, d, sub, xo, (void*)st, store_d, dzero);
    }
    return o.sell ? sell_cheb_impl(o.sell, xin, b, dg, c1, c2, d, sub, xo, (void*)st, store_d)
                  : cheb_step_impl(o.csr, o.blk, xin, b, dg, c1, c2, d, sub, xo, (void*)st, store_d);
}

struct OpPair {
    OpRef in, bd;
};

// x0 (= d0 for Chebyshev) of an inner solve from x = 0 over `nrows` owned rows: the tolerance-mode F operator on a row
// partition's owned rows takes the fast reciprocal diagonals (k_f_fast_init, the one-GPU fast first sweep's bits);
// every other operator the stored diagonal (k_cheb_init / k_jacobi_init: c2 (b / diag)).
int op_init(const OpRef& o, int32_t nrows, bool cheb, const double* b, const double* diag, double c2, double* d,
            const double* sub, double* xo, hipStream_t st) {
    const mpbp_schur_plan* p = o.stencil;
    if (p && o.sop == SOP_F && p->f_numerics == MPBP_NUMERICS_FAST && o.which != 3) {
        mpbp_row_part q = stencil_part(o);   // (the interior / boundary split of the sweeps: the init covers every owned row)
        q.which = 0;
        q.ext = 0;
        FStencilDev Pd;
        const int rc = make_fstencil(&p->f_prm, p->f_cell, p->f_uface, p->f_vface, &q, &Pd);
        if (rc) return rc;
        const FStencilFast P{Pd};
        if ((int64_t)4 * P.L * P.n != nrows) return set_error(MPBP_ERR_ARG, "f fast init: %d rows, not the owned ones", nrows);
        const int grid = grid_for((int64_t)P.L * P.n);
        if (cheb) k_f_fast_init<true><<<grid, 256, 0, st>>>(P, b, c2, d, sub, xo);
        else k_f_fast_init<false><<<grid, 256, 0, st>>>(P, b, 1.0, nullptr, sub, xo);
        MPBP_HIP(hipGetLastError());
        return MPBP_OK;
    }
    return cheb ? mpbp_cheb_init(nrows, b, diag, c2, d, sub, xo, (void*)st)
                : mpbp_jacobi_init(nrows, b, diag, sub, xo, (void*)st);
}

// The first sweep of an inner solve can fold in the init pass (x0 = d0 = c2[0] b / diag, recomputed
// from b and diag wherever the sweep stages x) when the operator is a whole-grid marching stencil.
bool can_fuse_init(const OpPair& op) {
    const OpRef& o = op.in;
    return o.stencil && !o.stencil->halo && !o.empty && op.bd.empty && o.which == 0 &&
           (o.sop == SOP_GTG || o.sop == SOP_F);
}

int op_first_sweep(const OpRef& o, bool cheb, const double* b, const double* diag, double c2_0, double c1, double c2,
                   double* d, const double* sub, double* xo, hipStream_t st, int store_d) {
    const mpbp_schur_plan* p = o.stencil;
    const XInit xs{b, diag, cheb ? c2_0 : 1.0};
    const mpbp_row_part q = stencil_part(o);   // one GPU: no partition; CA schedule: owned + ext ghost rows
    if (o.sop == SOP_F) {
        FStencilDev P;
        const int rc = make_fstencil(&p->f_prm, p->f_cell, p->f_uface, p->f_vface, &q, &P);
        if (rc) return rc;
        const bool fast = p->f_numerics == MPBP_NUMERICS_FAST;
        if (fast && cheb && KO().f_tile && q.halo == 0 && o.which == 0 && ftile_ok(P.n))   // x0, sweep 1 on 2D tiles
            return launch_ftile<true>(P, FTile{nullptr, nullptr, b, sub, xo, store_d ? d : nullptr, 0.0, c2_0, c1, c2},
                                      st);
        if (KO().init_diag == 0)
            return with_f_policy(P, fast, [&](const auto& Q) {
                return cheb ? launch_march(Q, xs, EpiChebFirst{b, d, c1, c2, sub, xo, store_d}, KO().march_rows, st)
                            : launch_march(Q, xs, EpiJacobi{nullptr, b, nullptr, sub, xo}, KO().march_rows, st);
            });
        return with_f_policy(P, fast, [&](const auto& Q) {
            return cheb ? launch_march_init(Q, b, xs.c2, EpiChebFirst{b, d, c1, c2, sub, xo, store_d}, KO().march_rows, st)
                        : launch_march_init(Q, b, xs.c2, EpiJacobi{nullptr, b, nullptr, sub, xo}, KO().march_rows, st);
        });
    }
    PGDev P;
    const int rc = make_pgstencil(&p->f_prm, p->f_cell, &q, &P);
    if (rc) return rc;
    // Gt_G: the staged diagonal is streamed (8 B per row; rebuilding it from thn measured slower, 21.6 vs 16.1 us
    // at 1024^2: the sweep is latency-bound and the rebuild lengthens its staging)
    const GtGStencilDev S{P};
    return cheb ? launch_march(S, xs, EpiChebFirst{b, d, c1, c2, sub, xo, store_d}, pg_rows(), st)
                : launch_march(S, xs, EpiJacobi{nullptr, b, nullptr, sub, xo}, pg_rows(), st);
}

OpPair make_op(const mpbp_schur_plan* p, const mpbp_csr& A, const mpbp_rowblocks& bi, const mpbp_rowblocks& bb,
               const mpbp_sell& si, const mpbp_sell& sb) {
    if (p->use_sell)
        return OpPair{OpRef{&A, nullptr, &si, nullptr, false, 0, SOP_NONE},
                      OpRef{&A, nullptr, &sb, nullptr, false, 0, SOP_NONE}};
    return OpPair{OpRef{&A, &bi, nullptr, nullptr, false, 0, SOP_NONE}, OpRef{&A, &bb, nullptr, nullptr, false, 0, SOP_NONE}};
}

// Stencil operator: interior + boundary rows under a row partition, else all rows in one launch.
OpPair make_stencil_op(const mpbp_schur_plan* p, int32_t sop, bool partitioned) {
    if (partitioned)
        return OpPair{OpRef{nullptr, nullptr, nullptr, p, false, 1, sop}, OpRef{nullptr, nullptr, nullptr, p, false, 2, sop}};
    return OpPair{OpRef{nullptr, nullptr, nullptr, p, false, 0, sop}, OpRef{nullptr, nullptr, nullptr, nullptr, true, 0, SOP_NONE}};
}

// Launch one sweep over interior rows, then (after the halo is complete) boundary rows.
template <class Fn>
int two_phase(const Ctx& c, int32_t kind, const double* x_ext, const OpPair& op, Fn&& launch) {
    const mpbp_schur_plan* p = c.p;
    if (p->halo && p->halo_first) {   // exchange first, then every row (stencils: one whole-partition launch)
        p->halo(p->halo_ctx, kind, const_cast<double*>(x_ext), MPBP_HALO_BEGIN, (void*)c.st);
        p->halo(p->halo_ctx, kind, const_cast<double*>(x_ext), MPBP_HALO_END, (void*)c.st);
        const int rc = launch(op.in);
        return rc ? rc : launch(op.bd);
    }
    if (p->halo) p->halo(p->halo_ctx, kind, const_cast<double*>(x_ext), MPBP_HALO_BEGIN, (void*)c.st);
    int rc = launch(op.in);
    if (rc) return rc;
    if (p->halo) p->halo(p->halo_ctx, kind, const_cast<double*>(x_ext), MPBP_HALO_END, (void*)c.st);
    return launch(op.bd);
}

// Tolerance mode on a row partition: Gt_F_G x_a from the diamond's upper half over the rank's row block (k_q13p; the
// plan's q13 then holds grid rows p_part.r0 - 2 .. r0 + rows - 1, mpbp_q13_build_rows), x_a's ghost rows complete.
bool q13p_ok(const mpbp_schur_plan* p) {
    return p->q13 && p->halo && KO().q13_sym && p->f_numerics == MPBP_NUMERICS_FAST && p->q13_n >= 5 &&
           p->p_part.halo >= 2 && p->p_part.rows >= 1 && p->np == p->p_part.rows * p->q13_n;
}
template <class Epi>
int launch_q13p(const mpbp_schur_plan* p, const double* x_ext, Epi epi, hipStream_t st) {
    const int32_t n = p->q13_n, L = p->p_part.rows;
    k_q13p<Epi><<<grid_for((int64_t)L * n), kBlock, 0, st>>>(n, p->p_part.r0, L, p->p_part.halo, p->q13, x_ext, epi);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

// ---- geometric multigrid inner solve (MPBP_INNER_MG) ----
// The reference's own pointer for these inverses: "In IBAMR, we'd use Multigrid PC with Jacobi smoother"
// (solve.py:266, 274).  V-cycles over the levels of an mpbp_mg hierarchy (Galerkin coarse operators
// R A P, mpbp_mg_transfer_*): Chebyshev-Jacobi pre- and post-smoothing on each level, the coarsest level solved
// by its dense (pseudo-)inverse.  Every step is an existing apply-path kernel (SpMV epilogues, Chebyshev
// steps), so the cycle is graph-capturable and its operation order is the oracle's (oracle/mg_oracle.py).
// Level 0 can be any operator of the plan (matrix-free stencil, SELL or CSR: the same bits).
struct MgFine {
    OpPair op;               // level 0's operator (interior + boundary rows under a row partition)
    const double* diag;
    double *x, *t, *r, *d;   // two iterate buffers, residual, Chebyshev direction
    mpbp_halo_fn halo;       // level 0's ghost-row exchange (NULL: one GPU)
    void* hctx;
    int32_t kind;
};

int pair_spmv(const OpPair& o, int32_t mode, const double* x, const double* z, double* y, hipStream_t st) {
    const int rc = op_spmv(o.in, mode, x, z, y, st);
    return rc ? rc : op_spmv(o.bd, mode, x, z, y, st);
}
int pair_cheb(const OpPair& o, const double* xin, const double* b, const double* dg, double c1, double c2, double* d,
              const double* sub, double* xo, hipStream_t st, int store_d, bool dzero = false) {
    const int rc = op_cheb(o.in, xin, b, dg, c1, c2, d, sub, xo, st, store_d, dzero);
    return rc ? rc : op_cheb(o.bd, xin, b, dg, c1, c2, d, sub, xo, st, store_d, dzero);
}

OpRef mg_csr_op(const mpbp_csr& A, const mpbp_rowblocks& blk) {
    return OpRef{&A, &blk, nullptr, nullptr, false, 0, SOP_NONE};
}
// A level's operator: its SELL-64 copy when it has one (same bits), else the CSR form.
OpPair mg_level_op(const mpbp_mg_level& L) {
    const OpRef none{nullptr, nullptr, nullptr, nullptr, true, 0, SOP_NONE};
    if (use_grp(L.A)) return OpPair{OpRef{&L.A, &L.A_blocks, nullptr, nullptr, false, 0, SOP_NONE, 0, 1}, none};
    if (L.A_svl && KO().mg_svl)
        return OpPair{OpRef{&L.A, &L.A_blocks, nullptr, nullptr, false, 0, SOP_NONE, 0, 0, L.A_svl}, none};
    return OpPair{L.A_sell.nslices > 0 ? OpRef{&L.A, nullptr, &L.A_sell, nullptr, false, 0, SOP_NONE}
                                       : mg_csr_op(L.A, L.A_blocks), none};
}
// Ghost rows of a level-l vector (row-partitioned levels l < part_levels; level 0 through the caller's halo).
void mg_exchange(const mpbp_mg* m, int l, const MgFine& f, double* x, hipStream_t st) {
    if (l == 0) {
        if (f.halo) {
            f.halo(f.hctx, f.kind, x, MPBP_HALO_BEGIN, (void*)st);
            f.halo(f.hctx, f.kind, x, MPBP_HALO_END, (void*)st);
        }
        return;
    }
    if (l < m->part_levels && m->halo) {
        m->halo(m->halo_ctx, m->levels[l].halo_kind, x, MPBP_HALO_BEGIN, (void*)st);
        m->halo(m->halo_ctx, m->levels[l].halo_kind, x, MPBP_HALO_END, (void*)st);
    }
}
MgFields mg_fields(const mpbp_mg* m) {
    MgFields F{};
    F.nfields = m->tr_nfields;
    for (int f = 0; f < m->tr_nfields; ++f) {
        F.ky[f] = m->tr_ky[f];
        F.kx[f] = m->tr_kx[f];
    }
    return F;
}
inline MgDiv mg_div(int32_t nr) { return MgDiv{divu((uint32_t)nr * (uint32_t)nr), divu((uint32_t)nr)}; }
// Level l's restriction (which = MPBP_MG_R) or prolongation (MPBP_MG_P) matrix-free when the hierarchy names its
// field kinds and the level is whole-grid (not row-partitioned); 1: launched, 0: not applicable.
template <class Epi>
int mg_transfer_mf(const mpbp_mg* m, int l, int32_t which, int32_t nrows, const double* x, Epi epi, hipStream_t st) {
    const int32_t n = m->tr_n0 >> l, nr = which == MPBP_MG_P ? n : n / 2;
    k_mg_transfer_spmv<Epi><<<grid_for(nrows), kBlock, 0, st>>>(mg_fields(m), mg_div(nr), n, which, nrows, x, epi);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}
inline bool use_mf_transfer(const mpbp_mg* m, int l) {
    return KO().mg_mf_transfer && m->tr_nfields > 0 && m->tr_nfields <= 8 && l >= m->part_levels && (m->tr_n0 >> l) >= 4 &&
           ((m->tr_n0 >> l) << l) == m->tr_n0;
}
// Kernel option mg_fuse_small (k_grp_rr): level l >= 1 of a hierarchy held whole on this GPU (one GPU, or a level every
// rank replicates), its operator on k_csr_grp rows, its transfers matrix-free with the level sizes the transfers imply,
// the coarse level at most kRrMaxCoarse rows.
bool mg_small_ok(const mpbp_mg* m, int l, const OpPair& o) {
    if (!KO().mg_fuse_small || l < 1 || l < m->part_levels || l + 1 >= m->nlevels || !o.in.grp || !o.in.csr ||
        o.in.gal || !o.bd.empty || !use_mf_transfer(m, l))
        return false;
    const int64_t n = m->tr_n0 >> l, rows = (int64_t)m->tr_nfields * n * n;
    const mpbp_csr& A = *o.in.csr;
    return A.nrows == rows && A.ncols == rows && m->levels[l].nrows == rows && m->levels[l + 1].nrows == rows / 4 &&
           rows / 4 <= kRrMaxCoarse;
}
int launch_grp_rr(const mpbp_mg* m, int l, const mpbp_csr* A, const double* x, const double* b, double* bc,
                  hipStream_t st) {
    const int32_t n = m->tr_n0 >> l, ncr = m->tr_nfields * (n / 2) * (n / 2);
    constexpr int WPB = kBlock / 64;
    k_grp_rr<<<(unsigned)((ncr + WPB - 1) / WPB), kBlock, 0, st>>>(to_csr(A), mg_fields(m), mg_div(n / 2), n, ncr, x, b,
                                                                 bc);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}
int mg_transfer(const mpbp_csr& M, const mpbp_rowblocks& blk, const mpbp_sell& S, int32_t mode, const double* x,
                const double* z, double* y, hipStream_t st) {
    if (use_grp(M)) return grp_spmv(&M, mode, x, z, y, st);
    return S.nslices > 0 ? mpbp_sell_spmv(&S, mode, x, z, y, (void*)st) : mpbp_spmv(&M, &blk, mode, x, z, y, (void*)st);
}

// y = M b for the coarsest level's dense (pseudo-)inverse, column-major (Mt[j * m + i] = M[i][j]).  A workgroup
// owns kDR rows: its 1024 threads request a kDK-column slab of them at once (16 loads each, all in flight), form
// the slab's products with b in LDS, then one lane per row adds them over the columns in order from 0.0 -- the CSR
// row's order with every entry stored (bit-identical to the CSR form of the same inverse).
constexpr int kDR = 16, kDK = 1024, kDT = 1024;
__global__ void __launch_bounds__(kDT) k_dense_cm(int32_t m, const double* __restrict__ Mt,
                                                  const double* __restrict__ b, double* __restrict__ y) {
    __shared__ double tile[kDK * kDR];   // [column][row]
    __shared__ double bs[kDK];
    const int32_t r0 = blockIdx.x * kDR;
    const int t = threadIdx.x;
    double acc = 0.0;
    for (int32_t j0 = 0; j0 < m; j0 += kDK) {
        const int kc = min(kDK, m - j0);
        constexpr int U = kDK * kDR / kDT;
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = t + kDT * u, c = e / kDR, row = r0 + e % kDR;
            v[u] = (c < kc && row < m) ? Mt[(size_t)(j0 + c) * m + row] : 0.0;
        }
        const double bv = t < kc ? b[j0 + t] : 0.0;
        bs[t] = bv;
        __syncthreads();
        // the slab's products M[row][col] * b[col] formed by all 1024 threads at once, so the summing lanes' loop is
        // LDS reads and dependent adds only (22 -> ~6 us for the 1024-row coarsest F level)
#pragma unroll
        for (int u = 0; u < U; ++u) tile[t + kDT * u] = v[u] * bs[(t + kDT * u) / kDR];
        __syncthreads();
        if (t < kDR) {   // 32 LDS reads in flight ahead of each run of dependent adds (same order)
            int c = 0;
            for (; c + 32 <= kc; c += 32) {
                double q[32];
#pragma unroll
                for (int u = 0; u < 32; ++u) q[u] = tile[(c + u) * kDR + t];
#pragma unroll
                for (int u = 0; u < 32; ++u) acc += q[u];
            }
            for (; c < kc; ++c) acc += tile[c * kDR + t];
        }
        __syncthreads();
    }
    if (t < kDR && r0 + t < m) y[r0 + t] = acc;
}

// The same product in tolerance mode (kernel option mg_coarse_tree): a workgroup owns kDR rows and every thread sums the
// products of its 16 columns of one row in registers as it loads them (no LDS round trip per product); the row's 64
// partial sums are then added pairwise in LDS.  One memory round trip and a 6-deep tree instead of the ordered row sum's
// m dependent additions (~1e-16 relative from the exact mode's k_dense_cm, which keeps the CSR row's bits).
__global__ void __launch_bounds__(kDT) k_dense_tree(int32_t m, const double* __restrict__ Mt,
                                                   const double* __restrict__ b, double* __restrict__ y) {
    constexpr int CPT = kDK * kDR / kDT;   // 16 columns per thread and slab
    constexpr int NP = kDT / kDR;          // 64 partial sums per row
    __shared__ double part[kDR * NP];
    const int32_t r0 = blockIdx.x * kDR;
    const int t = threadIdx.x, row = r0 + t % kDR, k = t / kDR;   // thread t: row t % 16, columns k + 64 u
    double acc = 0.0;
    for (int32_t j0 = 0; j0 < m; j0 += kDK) {
        double v[CPT], bv[CPT];
#pragma unroll
        for (int u = 0; u < CPT; ++u) {
            const int32_t c = j0 + k + NP * u;
            const bool in = c < m && row < m;
            v[u] = in ? Mt[(size_t)c * m + row] : 0.0;   // (lanes of a wave: 16 rows x 4 columns, 128-byte runs)
            bv[u] = c < m ? b[c] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < CPT; ++u) acc += v[u] * bv[u];
    }
    part[(t % kDR) * NP + k] = acc;
    __syncthreads();
#pragma unroll
    for (int w = NP / 2; w >= 1; w >>= 1) {   // rows' partials pairwise: t < 16 w lanes, row t % 16
        if (t < kDR * w) part[(t % kDR) * NP + t / kDR] += part[(t % kDR) * NP + t / kDR + w];
        __syncthreads();
    }
    if (t < kDR && r0 + t < m) y[r0 + t] = part[t * NP];
}

// K Chebyshev-Jacobi sweeps on [lmin, lmax].  zero: from x = 0 (the first sweep is the init pass: d = x =
// c2[0] b / diag), else from the iterate in *cur (d starts at 0).  The last sweep writes `dst` (or the free
// ping-pong buffer when dst is NULL), as sub - x when sub is set; *cur points at the result on return.  xch(x)
// refreshes x's ghost rows before every sweep that reads them (a no-op on one GPU).
// The last two sweeps of a tolerance-mode F Chebyshev solve may run as one fused launch (k_march2 / k_ftile).
bool f_pair_ok(const mpbp_schur_plan* p) { return p->f_numerics == MPBP_NUMERICS_FAST && KO().f_pair && p->f_stencil; }

template <class Xch>
int mg_smooth(const OpPair& op, int32_t nrows, const double* diag, double lmin, double lmax, int K, bool zero,
              const double* b, double** cur, double* alt, double* d, double* dst, const double* sub, hipStream_t st,
              Xch&& xch, int s0 = 0) {
    double c1[64] = {}, c2[64] = {};
    if (K < 1 || K > 64) return set_error(MPBP_ERR_ARG, "mg: smoothing sweeps must be in [1, 64]");
    cheb_coeffs(lmin, lmax, K, c1, c2);
    const OpRef& o = op.in;
    double* x = *cur;
    double* other = alt;
    int s = s0;   // s0 > 0: sweeps 0 .. s0 - 1 already ran from *cur's predecessor (d holds their direction)
    if (s0 && (zero || s0 >= K)) return set_error(MPBP_ERR_ARG, "mg: a smoothing resumed at sweep %d of %d", s0, K);
    if (zero && K >= 2 && op.bd.empty && o.stencil && !o.stencil->halo && o.which == 0 &&
        (o.sop == SOP_F || o.sop == SOP_GTG)) {
        // whole-grid stencil level (level 0 of the Schur apply's hierarchies): the first sweep stages
        // x0 = d0 = c2[0] b / diag itself (op_first_sweep, as the Chebyshev inner solve): no init launch, same bits
        double* out1 = K == 2 ? (dst ? dst : other) : other;
        const int rc = op_first_sweep(o, true, b, diag, c2[0], c1[1], c2[1], d, K == 2 ? sub : nullptr, out1, st,
                                      K == 2 ? 0 : 1);
        if (rc) return rc;
        other = x;
        x = out1;
        s = 2;
    } else if (zero && K >= 2 && op.bd.empty && o.grp && o.csr->ncols == nrows) {
        // grouped small level: the first sweep gathers x0 = c2[0] b / diag itself (no init launch, same bits; on the
        // large stencil-values levels the division per gathered entry costs more than the init launch: 110 vs 97 us).
        // Not on a row-partitioned level: its columns reach ghost rows, whose x0 only the exchange after an init
        // pass provides (b and diag hold the owned rows alone)
        double* out1 = K == 2 ? (dst ? dst : other) : other;
        const int rc = grp_cheb_first(o.csr, b, diag, c2[0], c1[1], c2[1], d, K == 2 ? sub : nullptr, out1, st,
                                      K == 2 ? 0 : 1);
        if (rc) return rc;
        other = x;
        x = out1;
        s = 2;
    } else if (zero && K >= 2 && op.bd.empty && o.gal && KO().mg_fuse_l0 && gal_fused_ok(*o.gal) &&
               o.gal->m->part_levels <= 1) {
        // matrix-free level 1 (k_gal1 / k_gal1p): the first sweep stages x0 = c2[0] b / diag itself (XInit) and its
        // epilogue takes the row's own x0 as iterate and direction -- no init launch, k_cheb_init's bits.  Not on a
        // row-partitioned level 1 (b and diag hold the owned rows; the ghosts' x0 comes from the init and exchange)
        double* out1 = K == 2 ? (dst ? dst : other) : other;
        EpiChebFirstGrp e;
        static_cast<EpiChebFirst&>(e) = EpiChebFirst{b, d, c1[1], c2[1], K == 2 ? sub : nullptr, out1, K == 2 ? 0 : 1};
        e.diag = diag;
        e.c2_0 = c2[0];
        bool done = false;
        const int rc = gal_fused(*o.gal, XInit{b, diag, c2[0]}, e, st, &done);
        if (rc) return rc;
        if (!done) return set_error(MPBP_ERR_ARG, "mg: the fused level-1 first sweep did not launch");
        other = x;
        x = out1;
        s = 2;
    } else if (zero) {
        double* out0 = K == 1 ? (dst ? dst : other) : x;
        int rc = op_init(o, nrows, true, b, diag, c2[0], d, K == 1 ? sub : nullptr, out0, st);
        if (rc) return rc;
        if (K == 1) {
            *cur = out0;
            return MPBP_OK;
        }
        s = 1;
    }
    // tolerance-mode F level 0 on one GPU: the last two sweeps as one tiled launch (k_ftile); a restart of two sweeps
    // reads d as +0.0 there, so it needs no memset either
    const bool tpair = K - s >= 2 && o.stencil && o.sop == SOP_F && op.bd.empty && !o.stencil->halo && o.which == 0 &&
                       f_pair_ok(o.stencil) && KO().f_tile && ftile_ok(o.stencil->f_prm.n);
    // restart from the iterate in *cur: d = 0 -- read as +0.0 by the grouped kernel's first sweep, else zeroed
    bool dzero = !zero && !s0 && (((op.in.grp || op.in.svl || op.in.gal || (o.stencil && o.sop == SOP_GTG)) && op.bd.empty) ||
                           (tpair && s == K - 2));
    if (!zero && !dzero && !s0) MPBP_HIP(hipMemsetAsync(d, 0, sizeof(double) * (size_t)nrows, st));
    for (; s < K; ++s) {
        if (tpair && s == K - 2) {
            double* out = dst ? dst : other;
            FStencilDev P;
            const mpbp_schur_plan* p = o.stencil;
            int rc = make_fstencil(&p->f_prm, p->f_cell, p->f_uface, p->f_vface, nullptr, &P);
            if (rc) return rc;
            FTile a{x, d, b, sub, out, nullptr, c1[s], c2[s], c1[s + 1], c2[s + 1]};
            a.dzero = dzero ? 1 : 0;
            rc = launch_ftile<false>(P, a, st);
            if (rc) return rc;
            other = x;
            x = out;
            break;
        }
        const bool last = s == K - 1;
        double* nxt = (last && dst) ? dst : other;
        xch(x);
        const int rc = pair_cheb(op, x, b, diag, c1[s], c2[s], d, last ? sub : nullptr, nxt, st, last ? 0 : 1, dzero);
        dzero = false;
        if (rc) return rc;
        other = x;
        x = nxt;
    }
    *cur = x;
    return MPBP_OK;
}

// Level 1 as R_0 (F (P_0 x)): tolerance-mode F (or Gt_G) stencil level 0, level 1 smoothed.  mg_galerkin_mf 1: the three
// launches (one GPU, matrix-free level-0 transfers); 2 (default): the one-launch form where the grid allows it
// (gal_fused_ok: even n >= 72), else the stored Galerkin level -- on one GPU and under a row partition alike (level 0's
// interior / boundary rows and its halo; level 1 replicated whole or its owned rows), so both run the same level 1.
bool mg_gal_ok(const mpbp_mg* m, const MgFine& f) {
    const OpRef& o = f.op.in;
    if (!KO().mg_galerkin_mf || !o.stencil || !(o.sop == SOP_F || (o.sop == SOP_GTG && KO().mg_galerkin_mf_p)) ||
        o.stencil->f_numerics != MPBP_NUMERICS_FAST || m->nlevels <= 2 || !f.r || !f.d)
        return false;
    const MgGal g{m, o, f.r, f.d};
    if (m->part_levels == 0)
        return o.which == 0 && f.op.bd.empty && !f.halo && !o.stencil->halo && use_mf_transfer(m, 0) &&
               (KO().mg_galerkin_mf == 1 || gal_fused_ok(g));
    return f.halo && o.stencil->halo && m->tr_nfields > 0 && m->tr_n0 == o.stencil->f_prm.n && gal_fused_ok(g);
}

// Level 0's descent as ONE k_fpre launch (pre-smoothing V(2, .) from x = 0, residual, restriction): tolerance-mode
// matrix-free F on one GPU, the whole grid, the F hierarchy's MAC transfers matrix-free, a grid the tile's staging
// wraps onto at most once (kernel option mg_fuse_l0).
bool fpre_ok(const mpbp_mg* m, const MgFine& f) {
    const OpRef& o = f.op.in;
    if (!KO().mg_fuse_l0 || !o.stencil || o.sop != SOP_F || o.which != 0 || !f.op.bd.empty || f.halo || o.stencil->halo)
        return false;
    const mpbp_schur_plan* p = o.stencil;
    if (p->f_numerics != MPBP_NUMERICS_FAST || !p->f_stencil || m->part_levels > 0 || !use_mf_transfer(m, 0) ||
        m->tr_nfields != 4)
        return false;
    for (int fl = 0; fl < 4; ++fl)
        if (m->tr_ky[fl] != ((fl & 1) ? MPBP_MG_NODE : MPBP_MG_CELL) || m->tr_kx[fl] != ((fl & 1) ? MPBP_MG_CELL : MPBP_MG_NODE))
            return false;
    const int n = p->f_prm.n;
    return (n & 1) == 0 && m->tr_n0 == n && fsolve_ok_n<3>(n);
}
int launch_fpre(const mpbp_schur_plan* p, const double* b, double lmin, double lmax, double* x_out, double* bc,
                hipStream_t st) {
    FStencilDev Pd;
    const int rc = make_fstencil(&p->f_prm, p->f_cell, p->f_uface, p->f_vface, nullptr, &Pd);
    if (rc) return rc;
    const FStencilFast P{Pd};
    if (P.h != 0 || P.which != 0 || !fsolve_ok_n<3>(P.n) || (P.n & 1) || !b || !x_out || !bc)
        return set_error(MPBP_ERR_ARG, "fpre: one GPU, whole even grid n >= 72");
    double c1[2] = {}, c2[2] = {};
    cheb_coeffs(lmin, lmax, 2, c1, c2);
    const int64_t tiles = (int64_t)((P.n + kFTW - 1) / kFTW) * ((P.n + kFTH - 1) / kFTH);
    k_fpre<<<(unsigned)tiles, 256, 0, st>>>(P, FPre{b, x_out, bc, c2[0], c1[1], c2[1]});
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

// The pressure hierarchy's level 0 the same way (k_gtg_level0): matrix-free Gt_G on one GPU, the whole grid, its
// cell-centred transfers matrix-free, a grid the staging wraps onto at most once (kernel option mg_fuse_l0).
bool gpre_ok(const mpbp_mg* m, const MgFine& f) {
    const OpRef& o = f.op.in;
    if (!KO().mg_fuse_l0 || !o.stencil || o.sop != SOP_GTG || o.which != 0 || !f.op.bd.empty || f.halo || o.stencil->halo)
        return false;
    const mpbp_schur_plan* p = o.stencil;
    if (!p->pg_stencil || m->part_levels > 0 || !use_mf_transfer(m, 0) || m->tr_nfields != 1 ||
        m->tr_ky[0] != MPBP_MG_CELL || m->tr_kx[0] != MPBP_MG_CELL)
        return false;
    const int n = p->f_prm.n;
    return (n & 1) == 0 && m->tr_n0 == n && n >= kGTW + kGTH + 6;
}
// pre: x0, sweep 1 (x_out), r = b - A x1, b_c = R_0 r; post: x = x_in + P_0 x_c, two sweeps from d = 0 (x_out, or
// sub - x when sub is set)
int launch_gtg_level0(bool pre, const mpbp_schur_plan* p, const double* b, const double* diag, const double* xin,
                      const double* xc, const double* sub, double lmin, double lmax, double* x_out, double* bc,
                      hipStream_t st) {
    PGDev Pg;
    const int rc = make_pgstencil(&p->f_prm, p->f_cell, nullptr, &Pg);
    if (rc) return rc;
    const GtGStencilDev S{Pg};
    if (S.n < kGTW + kGTH + 6 || (S.n & 1) || !b || !x_out || (pre && (!diag || !bc)) || (!pre && (!xin || !xc)))
        return set_error(MPBP_ERR_ARG, "gtg_level0: one GPU, whole even grid n >= 78, vectors");
    double c1[2] = {}, c2[2] = {};
    cheb_coeffs(lmin, lmax, 2, c1, c2);
    ChebK ck{};
    if (pre) {
        ck.c2[0] = c2[0];
        ck.c1[1] = c1[1];
        ck.c2[1] = c2[1];
    } else {   // the post-smoothing's sweeps s = 0, 1 as levels 1, 2
        ck.c1[1] = c1[0];
        ck.c2[1] = c2[0];
        ck.c1[2] = c1[1];
        ck.c2[2] = c2[1];
    }
    const int64_t tiles = (int64_t)((S.n + kGTW - 1) / kGTW) * ((S.n + kGTH - 1) / kGTH);
    if (pre) k_gtg_level0<true, false><<<(unsigned)tiles, 512, 0, st>>>(S, b, diag, nullptr, nullptr, nullptr, ck, x_out, bc);
    else if (sub) k_gtg_level0<false, true><<<(unsigned)tiles, 512, 0, st>>>(S, b, nullptr, xin, xc, sub, ck, x_out, nullptr);
    else k_gtg_level0<false, false><<<(unsigned)tiles, 512, 0, st>>>(S, b, nullptr, xin, xc, nullptr, ck, x_out, nullptr);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

// One V-cycle on level l for A_l x = b.  Level 0 uses `fine` (operator and buffers); coarser levels their
// mpbp_mg_level.  *res receives the result's buffer (dst when given).  Row partition (m->part_levels > 0): levels
// l < part_levels hold owned rows (vectors read by an operator carry ghost rows, refreshed by mg_exchange); the
// restriction into level part_levels writes the rank's rows of that level into its r buffer, which is all-gathered
// into its (whole-grid) b, and every coarser level runs replicated on each rank -- the same operators and
// operands as on one GPU, so the same bits.
int mg_vcycle(const mpbp_mg* m, int l, const MgFine& fine, const double* b, bool zero, double* xin, double* dst,
              const double* sub, double** res, hipStream_t st) {
    const mpbp_mg_level& L = m->levels[l];
    const bool top = l == 0;
    OpPair o = top ? fine.op : mg_level_op(L);
    MgGal gal{m, fine.op.in, fine.r, fine.d};   // (fine.r, fine.d: dead while level 1 runs)
    if (l == 1 && mg_gal_ok(m, fine)) {
        o.in = OpRef{nullptr, nullptr, nullptr, nullptr, false, 0, SOP_NONE};
        o.in.gal = &gal;
        o.bd = OpRef{nullptr, nullptr, nullptr, nullptr, true, 0, SOP_NONE};
    }
    const double* diag = top ? fine.diag : L.diag;
    double* bx = top ? fine.x : L.x;
    double* bt = top ? fine.t : L.t;
    double* alt = xin == bx ? bt : bx;
    double* r = top ? fine.r : L.r;
    double* d = top ? fine.d : L.d;
    double* cur = xin;
    auto xch = [&](double* v) { mg_exchange(m, l, fine, v, st); };
    const mpbp_mg_level& C = m->levels[l + 1];
    const bool gather = m->part_levels > 0 && l + 1 == m->part_levels;
    const bool small = mg_small_ok(m, l, o);   // (never a gathering level: l >= part_levels)
    int rc = MPBP_OK;
    if (top && zero && L.pre == 2 && fpre_ok(m, fine)) {
        // x0, sweep 1, r = b - A x and b_c = R r in one launch; x1 where the smoothing would leave it (the free buffer)
        cur = alt;
        rc = launch_fpre(o.in.stencil, b, L.lmin, L.lmax, cur, C.b, st);
        if (rc) return rc;
        alt = cur == bx ? bt : bx;
    } else if (top && zero && L.pre == 2 && gpre_ok(m, fine)) {   // the same for the pressure hierarchy
        cur = alt;
        rc = launch_gtg_level0(true, o.in.stencil, b, diag, nullptr, nullptr, nullptr, L.lmin, L.lmax, cur, C.b, st);
        if (rc) return rc;
        alt = cur == bx ? bt : bx;
    } else {
        rc = mg_smooth(o, L.nrows, diag, L.lmin, L.lmax, L.pre, zero, b, &cur, alt, d, nullptr, nullptr, st, xch);
        if (rc) return rc;
        alt = cur == bx ? bt : bx;
        if (small) {   // r = b - A x and b_c = R r in one launch (k_grp_rr)
            rc = launch_grp_rr(m, l, o.in.csr, cur, b, C.b, st);
        } else {       // r = b - A x ; b_c = R r
            xch(cur);
            rc = pair_spmv(o, MPBP_SPMV_RESID, cur, b, r, st);
            if (rc) return rc;
            if (l < m->part_levels) xch(r);
            rc = use_mf_transfer(m, l) ? mg_transfer_mf(m, l, MPBP_MG_R, L.R.nrows, r, EpiStore{gather ? C.r : C.b}, st)
                                       : mg_transfer(L.R, L.R_blocks, L.R_sell, MPBP_SPMV_STORE, r, nullptr,
                                                     gather ? C.r : C.b, st);
        }
        if (rc) return rc;
    }
    if (gather) {
        if (!m->gather) return set_error(MPBP_ERR_ARG, "mg: a partitioned hierarchy needs its gather callback");
        m->gather(m->halo_ctx, m->gather_kind, C.r, C.b, (void*)st);
    }
    double* xc = C.x;
    if (l + 1 == m->nlevels - 1) {
        if (m->coarse_dense) {
            // tolerance-mode hierarchies (the fine operator a fast-numerics stencil plan): the tree-summed product
            const bool tree = KO().mg_coarse_tree && fine.op.in.stencil &&
                              fine.op.in.stencil->f_numerics == MPBP_NUMERICS_FAST;
            if (tree) k_dense_tree<<<grid_for(C.nrows, kDR), kDT, 0, st>>>(C.nrows, m->coarse_dense, C.b, xc);
            else k_dense_cm<<<grid_for(C.nrows, kDR), kDT, 0, st>>>(C.nrows, m->coarse_dense, C.b, xc);
            MPBP_HIP(hipGetLastError());
        } else {
            rc = mpbp_spmv(&m->coarse_inv, &m->coarse_inv_blocks, MPBP_SPMV_STORE, C.b, nullptr, xc, (void*)st);
        }
    } else {
        rc = mg_vcycle(m, l + 1, fine, C.b, true, C.x, nullptr, nullptr, &xc, st);
    }
    if (rc) return rc;
    // x += P x_c (row-wise in place), then post-smoothing from x
    mg_exchange(m, l + 1, fine, xc, st);
    if (top && L.post == 2 && gpre_ok(m, fine)) {   // x + P_0 x_c and the two post-smoothing sweeps in one launch
        double* out = dst ? dst : alt;
        rc = launch_gtg_level0(false, o.in.stencil, b, nullptr, cur, xc, sub, L.lmin, L.lmax, out, nullptr, st);
        if (rc) return rc;
        *res = out;
        return MPBP_OK;
    }
    if (top && L.post == 2 && fpre_ok(m, fine) && f_pair_ok(o.in.stencil) && KO().f_tile && ftile_ok(o.in.stencil->f_prm.n)) {
        // the prolongation folded into the post-smoothing pair's staging (k_ftile<PRO>: x + P_0 x_c per staged cell,
        // the prolongation launch's operations), the restart's direction read as +0.0 -- mg_smooth's tile pair
        double c1[2] = {}, c2[2] = {};
        cheb_coeffs(L.lmin, L.lmax, 2, c1, c2);
        double* out = dst ? dst : alt;
        const mpbp_schur_plan* p = o.in.stencil;
        FStencilDev P;
        rc = make_fstencil(&p->f_prm, p->f_cell, p->f_uface, p->f_vface, nullptr, &P);
        if (rc) return rc;
        FTile a{cur, d, b, sub, out, nullptr, c1[0], c2[0], c1[1], c2[1]};
        a.dzero = 1;
        a.xc = xc;
        rc = launch_ftile<false>(P, a, st);
        if (rc) return rc;
        *res = out;
        return MPBP_OK;
    }
    if (o.in.gal && L.post >= 1 && L.post <= 64 && gal_pro_ok(*o.in.gal)) {
        // level 1 (matrix-free F): x + P_1 x_c staged by the first post-smoothing sweep (k_gal1<PRO>), the remaining
        // sweeps as mg_smooth's
        double c1[64] = {}, c2[64] = {};
        cheb_coeffs(L.lmin, L.lmax, L.post, c1, c2);
        const bool last = L.post == 1;
        double* x1 = last && dst ? dst : alt;
        const EpiCheb e{cur, b, diag, d, c1[0], c2[0], last ? sub : nullptr, x1, last ? 0 : 1};
        rc = gal_pro(*o.in.gal, cur, xc, EpiZeroD<EpiCheb>{e}, st);
        if (rc) return rc;
        if (!last) rc = mg_smooth(o, L.nrows, diag, L.lmin, L.lmax, L.post, false, b, &x1, cur, d, dst, sub, st, xch, 1);
        if (rc) return rc;
        *res = x1;
        return MPBP_OK;
    }
    rc = use_mf_transfer(m, l) ? mg_transfer_mf(m, l, MPBP_MG_P, L.P.nrows, xc, EpiAdd{cur, cur}, st)
                               : mg_transfer(L.P, L.P_blocks, L.P_sell, MPBP_SPMV_ADD, xc, cur, cur, st);
    if (rc) return rc;
    rc = mg_smooth(o, L.nrows, diag, L.lmin, L.lmax, L.post, false, b, &cur, alt, d, dst, sub, st, xch);
    if (rc) return rc;
    *res = cur;
    return MPBP_OK;
}

// x_out = mg^-1 b by mg->cycles V-cycles from x = 0 (sub - that when sub != NULL).
int mg_solve(const mpbp_mg* m, const MgFine& fine, const double* b, double* x_out, const double* sub, hipStream_t st) {
    if (!m || m->nlevels < 2 || !m->levels || m->cycles < 1 || !m->coarse_inv.row_ptr)
        return set_error(MPBP_ERR_ARG, "mg: hierarchy needs >= 2 levels, >= 1 cycle and the coarse inverse");
    if (x_out == fine.x || x_out == fine.t || x_out == fine.r || x_out == fine.d || b == x_out)
        return set_error(MPBP_ERR_ARG, "mg: x_out must not alias the level-0 work buffers or b");
    double* cur = fine.x;
    for (int k = 0; k < m->cycles; ++k) {
        const bool last = k == m->cycles - 1;
        double* res = nullptr;
        const int rc = mg_vcycle(m, 0, fine, b, k == 0, cur, last ? x_out : nullptr, last ? sub : nullptr, &res, st);
        if (rc) return rc;
        cur = res;
    }
    return MPBP_OK;
}

// rhs = D Finv_v + v_p with the first Gt_G sweep's x0 = c2 (rhs / diag_P) written beside it (one GPU, matrix-free D).
int d_rhs_x0(const mpbp_schur_plan* p, const double* Y, const double* v_p, double* rhs, double c2, double* x0,
             hipStream_t st) {
    PGDev P;
    const int rc = make_pgstencil(&p->f_prm, p->f_cell, nullptr, &P);
    if (rc) return rc;
    return launch_march(DStencilDev{P}, XPlain{Y}, EpiAddX0{v_p, rhs, p->diag_P, c2, x0}, pg_rows(), st);
}

// x = Gt_G^-1 b by the plan's Chebyshev inner solve in one k_gtg_solve launch (one GPU, matrix-free Gt_G, 2..6 sweeps).
template <int H, int GW, int GH>
int launch_gtg_solve_g(const GtGStencilDev& S, const double* b, const double* diag, const ChebK& ck, double* out,
                       hipStream_t st, GtgD dv) {
    const bool part = S.h != 0;
    // every staged cell of a tile (tile + H + 1 each side) must wrap onto the grid at most once (the staging's periodic
    // fold subtracts n once): refuse smaller grids here, whatever the caller checked (gtg_fused_ok) -- one bound for
    // both tiles (the 64 x 8 tile's, the larger), so the tile option never changes which grids the fused solve takes
    constexpr int kMin = kGTW + kGTH + 2 * H;
    static_assert(GW + GH + 2 * H <= kMin, "the documented bound covers this tile");
    if (S.n < kMin)
        return set_error(MPBP_ERR_ARG, "gtg_solve: a %d-sweep fused solve needs n >= %d (n = %d)", H + 1, kMin, S.n);
    const int rows = part ? S.L + 2 * S.ext : S.n;
    const int64_t tiles = (int64_t)((S.n + GW - 1) / GW) * ((rows + GH - 1) / GH);
    const bool db = dv.Y != nullptr;
    if (db && part) return set_error(MPBP_ERR_ARG, "gtg_solve: the fused D right-hand side is one-GPU only");
    // 512 lanes own rings 1 .. H - 1 one cell each (GtgTile::rings(H - 1) <= 512 cells)
    if constexpr (GtgTile<H, GW, GH>::rings(H - 1) <= 512) {
        if (KO().gtg_tpb == 512) {
            if (db) k_gtg_solve<H, false, 512, true, GW, GH><<<(unsigned)tiles, 512, 0, st>>>(S, b, diag, ck, out, dv);
            else if (part)
                k_gtg_solve<H, true, 512, false, GW, GH><<<(unsigned)tiles, 512, 0, st>>>(S, b, diag, ck, out, dv);
            else k_gtg_solve<H, false, 512, false, GW, GH><<<(unsigned)tiles, 512, 0, st>>>(S, b, diag, ck, out, dv);
            MPBP_HIP(hipGetLastError());
            return MPBP_OK;
        }
    }
    {
        if (db) k_gtg_solve<H, false, 256, true, GW, GH><<<(unsigned)tiles, 256, 0, st>>>(S, b, diag, ck, out, dv);
        else if (part) k_gtg_solve<H, true, 256, false, GW, GH><<<(unsigned)tiles, 256, 0, st>>>(S, b, diag, ck, out, dv);
        else k_gtg_solve<H, false, 256, false, GW, GH><<<(unsigned)tiles, 256, 0, st>>>(S, b, diag, ck, out, dv);
    }
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}
// kernel option gtg_solve_tile: 32 x 16 tiles (1) -- shorter halo rings, fewer staged and halo cells per output, as
// k_fsolve_w -- or the 64 x 8 tile (0); every cell's operations are the same, so are the bits
template <int H>
int launch_gtg_solve_t(const GtGStencilDev& S, const double* b, const double* diag, const ChebK& ck, double* out,
                       hipStream_t st, GtgD dv = GtgD{}) {
    return KO().gtg_solve_tile ? launch_gtg_solve_g<H, 32, 16>(S, b, diag, ck, out, st, dv)
                               : launch_gtg_solve_g<H, kGTW, kGTH>(S, b, diag, ck, out, st, dv);
}
// The tile's staged cells must wrap onto the grid at most once each way (P.wrap), so n >= a tile plus its halos.
// part: under a row partition (the CA schedule's solves), else one GPU.
bool gtg_fused_ok(const mpbp_schur_plan* p, bool part = false) {
    const mpbp_inner_solver& in = p->inner_P;
    return KO().gtg_fused && p->pg_stencil && (p->halo != nullptr) == part && in.kind == MPBP_INNER_CHEBYSHEV &&
           in.sweeps >= 2 && in.sweeps <= 6 && in.lmax > in.lmin && in.lmin >= 0.0 &&
           p->f_prm.n >= kGTW + kGTH + 2 * (in.sweeps - 1);
}
// part: the CA schedule's owned + ext ghost rows (b and diag in the pressure ghost layout), else one GPU.
// dv.Y set (one GPU): b is not read; rhs = D dv.Y + dv.vp is built inside (k_gtg_solve<DB>).
int gtg_solve_fused(const mpbp_schur_plan* p, const double* b, double* out, hipStream_t st,
                    const mpbp_row_part* part = nullptr, const double* diag = nullptr, GtgD dv = GtgD{}) {
    PGDev P;
    const int rc = make_pgstencil(&p->f_prm, p->f_cell, part, &P);
    if (rc) return rc;
    const int K = p->inner_P.sweeps;
    if (part && (P.which != 3 || P.h < P.ext + K - 1 || P.oh < P.ext || !diag))
        return set_error(MPBP_ERR_ARG, "gtg_solve_fused: owned + ext rows need b ext + K - 1 deep and the ext diagonal");
    if (!part) diag = p->diag_P;
    ChebK ck{};
    double c1[64] = {}, c2[64] = {};
    cheb_coeffs(p->inner_P.lmin, p->inner_P.lmax, K, c1, c2);
    for (int s = 0; s < K; ++s) {
        ck.c1[s] = c1[s];
        ck.c2[s] = c2[s];
    }
    const GtGStencilDev S{P};
    switch (K - 1) {
    case 1: return launch_gtg_solve_t<1>(S, b, diag, ck, out, st, dv);
    case 2: return launch_gtg_solve_t<2>(S, b, diag, ck, out, st, dv);
    case 3: return launch_gtg_solve_t<3>(S, b, diag, ck, out, st, dv);
    case 4: return launch_gtg_solve_t<4>(S, b, diag, ck, out, st, dv);
    case 5: return launch_gtg_solve_t<5>(S, b, diag, ck, out, st, dv);
    default: return set_error(MPBP_ERR_ARG, "gtg_solve_fused: 2..6 sweeps");
    }
}

}  // namespace

extern "C" int mpbp_gtg_stencil_cheb_solve(const mpbp_stokes_params* prm, const double* cell, const double* b,
                                           const double* diag, double lmin, double lmax, int32_t sweeps,
                                           double* x_out, void* stream) {
    if (!prm || !cell || !b || !diag || !x_out || b == x_out || sweeps < 2 || sweeps > 6 || !(lmax > lmin) ||
        !(lmin >= 0.0))
        return set_error(MPBP_ERR_ARG, "gtg_stencil_cheb_solve: bad args (2..6 sweeps, 0 <= lmin < lmax)");
    PGDev P;
    const int rc = make_pgstencil(prm, cell, nullptr, &P);
    if (rc) return rc;
    ChebK ck{};
    double c1[64] = {}, c2[64] = {};
    cheb_coeffs(lmin, lmax, sweeps, c1, c2);
    for (int s = 0; s < sweeps; ++s) {
        ck.c1[s] = c1[s];
        ck.c2[s] = c2[s];
    }
    const GtGStencilDev S{P};
    const hipStream_t st = as_stream(stream);
    switch (sweeps - 1) {
    case 1: return launch_gtg_solve_t<1>(S, b, diag, ck, x_out, st);
    case 2: return launch_gtg_solve_t<2>(S, b, diag, ck, x_out, st);
    case 3: return launch_gtg_solve_t<3>(S, b, diag, ck, x_out, st);
    case 4: return launch_gtg_solve_t<4>(S, b, diag, ck, x_out, st);
    default: return launch_gtg_solve_t<5>(S, b, diag, ck, x_out, st);
    }
}

namespace {
// The first sweep of a Gt_G Chebyshev solve staging a precomputed x0 = d0 (one GPU, matrix-free Gt_G).
int gtg_first_sweep_x0(const mpbp_schur_plan* p, const double* x0, const double* b, double c1, double c2, double* d,
                       const double* sub, double* xo, int store_d, hipStream_t st) {
    PGDev P;
    const int rc = make_pgstencil(&p->f_prm, p->f_cell, nullptr, &P);
    if (rc) return rc;
    return launch_march(GtGStencilDev{P}, XPlain{x0}, EpiChebFirst{b, d, c1, c2, sub, xo, store_d}, pg_rows(), st);
}

// The last two sweeps of a tolerance-mode F Chebyshev solve fused (k_march2): one GPU whole grid, or (ext >= 0) the CA
// schedule's owned + ext ghost rows.
template <class BS = BNone>
int f_pair(const mpbp_schur_plan* p, int ext, const double* x_in, const double* b, double* dir, double c1a, double c2a,
           double c1b, double c2b, const double* sub, double* x_out, hipStream_t st, const BS& bs = BS{}) {
    FStencilDev P;
    int rc;
    if (ext >= 0) {
        OpRef o{nullptr, nullptr, nullptr, p, false, 3, SOP_F};
        o.ext = ext;
        const mpbp_row_part q = stencil_part(o);
        rc = make_fstencil(&p->f_prm, p->f_cell, p->f_uface, p->f_vface, &q, &P);
    } else {
        rc = make_fstencil(&p->f_prm, p->f_cell, p->f_uface, p->f_vface, nullptr, &P);
    }
    if (rc) return rc;
    if (ext < 0 && KO().f_tile && ftile_ok(P.n))   // one GPU: the pair on 2D tiles
        return launch_ftile<false>(P, FTile{x_in, dir, b, sub, x_out, nullptr, c1a, c2a, c1b, c2b}, st, bs);
    return launch_march2(P, Fused2{x_in, dir, b, sub, x_out, nullptr, c1a, c2a, c1b, c2b}, st, bs);
}

// x = M^-1 b by `inner` sweeps from x0 = 0 (solve.py:251/254 F_inv / Gt_G_factorization roles).
// The final iterate goes to dst (sub - iterate when sub != NULL); ping/pong hold the others.  x0_pre (Gt_G,
// Chebyshev, fusable first sweep): the first iterate c2[0] b / diag already computed by b's producer.
// fn() bracketed by the plan's profiling events (mpbp_schur_plan.prof_events) when asked and not capturing.
template <class Fn>
int profiled(const mpbp_schur_plan* p, bool profile, hipStream_t st, Fn&& fn) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    const bool rec = profile && p->prof_events && p->prof_count && *p->prof_count < p->prof_capacity &&
                     hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone;
    if (rec) MPBP_HIP(record_event((hipEvent_t)p->prof_events[2 * *p->prof_count], st));
    const int rc = fn();
    if (rc) return rc;
    if (rec) {
        MPBP_HIP(record_event((hipEvent_t)p->prof_events[2 * *p->prof_count + 1], st));
        ++*p->prof_count;
    }
    return MPBP_OK;
}

int inner_solve(const Ctx& c, int32_t kind, const OpPair& op, const double* diag, const mpbp_inner_solver& in,
                int32_t nrows, const double* b, double* dst, const double* sub, double* ping, double* pong,
                double* dir, bool profile, const double* x0_pre = nullptr) {
    if (in.kind == MPBP_INNER_MG) {   // one GPU: V-cycles whose level 0 is this operator
        const mpbp_mg* m = kind == MPBP_VEC_VELOCITY ? c.p->mg_F : c.p->mg_P;
        if (!m)
            return set_error(MPBP_ERR_ARG, "schur_apply: a multigrid inner solve needs plan.mg_%s",
                             kind == MPBP_VEC_VELOCITY ? "F" : "P");
        if ((c.p->halo != nullptr) != (m->part_levels > 0))
            return set_error(MPBP_ERR_ARG, "schur_apply: a %s apply needs a %s multigrid hierarchy",
                             c.p->halo ? "row-partitioned" : "one-GPU", c.p->halo ? "row-partitioned" : "whole-grid");
        if (m->levels[0].nrows != nrows) return set_error(MPBP_ERR_ARG, "schur_apply: mg level 0 size mismatch");
        const MgFine f{op, diag, ping, pong, m->levels[0].r, dir, c.p->halo, c.p->halo_ctx, kind};
        return mg_solve(m, f, b, dst, sub, c.st);
    }
    const int K = in.sweeps;
    double c1[64] = {}, c2[64] = {};   // zeros for Jacobi (never read uninitialised)
    if (K < 1 || K > 64) return set_error(MPBP_ERR_ARG, "inner sweeps must be in [1, 64]");
    const bool cheb = in.kind == MPBP_INNER_CHEBYSHEV;
    if (cheb) {
        if (!(in.lmax > in.lmin) || !(in.lmin >= 0.0)) return set_error(MPBP_ERR_ARG, "bad Chebyshev interval");
        cheb_coeffs(in.lmin, in.lmax, K, c1, c2);
    } else if (in.kind != MPBP_INNER_JACOBI) {
        return set_error(MPBP_ERR_ARG, "unknown inner solver %d", in.kind);
    }
    // tolerance-mode F on one GPU: the whole solve as one launch
    if (cheb && f_pair_ok(c.p) && KO().f_solve && op.in.stencil && op.in.sop == SOP_F && op.bd.empty && op.in.which == 0 &&
        !c.p->halo && fsolve_ok(K, c.p->f_prm.n)) {
        FStencilDev P;
        int rc = make_fstencil(&c.p->f_prm, c.p->f_cell, c.p->f_uface, c.p->f_vface, nullptr, &P);
        if (rc) return rc;
        return profiled(c.p, profile, c.st, [&] { return launch_fsolve(P, K, c1, c2, b, sub, dst, c.st); });
    }
    double* cur = (K == 1) ? dst : ping;
    int s = 1, rc = MPBP_OK;
    if (K >= 2 && can_fuse_init(op)) {   // sweep 1 recomputes x0 = d0 from b and diag: no init pass
        double* nxt = K == 2 ? dst : pong;
        rc = (x0_pre && cheb && op.in.sop == SOP_GTG)
                 ? gtg_first_sweep_x0(c.p, x0_pre, b, c1[1], c2[1], dir, K == 2 ? sub : nullptr, nxt, K == 2 ? 0 : 1,
                                      c.st)
                 : op_first_sweep(op.in, cheb, b, diag, c2[0], c1[1], c2[1], dir, K == 2 ? sub : nullptr, nxt, c.st,
                                  K == 2 ? 0 : 1);
        if (rc) return rc;
        cur = nxt;
        s = 2;
    } else {
        const double* s0 = (K == 1) ? sub : nullptr;
        rc = op_init(op.in, nrows, cheb, b, diag, c2[0], dir, s0, cur, c.st);
        if (rc) return rc;
    }
    // tolerance-mode F on one GPU: the last two sweeps as one fused launch
    const bool pair_ok = cheb && f_pair_ok(c.p) && op.in.stencil && op.in.sop == SOP_F && op.bd.empty &&
                         op.in.which == 0 && !c.p->halo;
    while (s < K) {
        const bool pair = pair_ok && s == K - 2;
        const bool last = s == K - 1 || pair;
        double* nxt = last ? dst : (cur == ping ? pong : ping);
        const double* sb = last ? sub : nullptr;
        const mpbp_schur_plan* p = c.p;
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        const bool rec = profile && p->prof_events && p->prof_count && *p->prof_count < p->prof_capacity &&
                         hipStreamIsCapturing(c.st, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone;
        if (rec) MPBP_HIP(record_event((hipEvent_t)p->prof_events[2 * *p->prof_count], c.st));
        if (pair)
            rc = f_pair(p, -1, cur, b, dir, c1[s], c2[s], c1[s + 1], c2[s + 1], sb, nxt, c.st);
        else
            rc = two_phase(c, kind, cur, op, [&](const OpRef& o) {
                return cheb ? op_cheb(o, cur, b, diag, c1[s], c2[s], dir, sb, nxt, c.st, last ? 0 : 1)
                            : op_jacobi(o, cur, b, diag, sb, nxt, c.st);
            });
        if (rc) return rc;
        if (rec) {
            MPBP_HIP(record_event((hipEvent_t)p->prof_events[2 * *p->prof_count + 1], c.st));
            ++*p->prof_count;
        }
        cur = nxt;
        s += pair ? 2 : 1;
    }
    return MPBP_OK;
}

// u = Finv_v - F^-1 (G x_p) (solve.py:273-276) with the second F solve's right-hand side W = G x_p recomputed
// inside each of its sweeps from x_p (GxB) instead of a G launch writing W: one GPU, matrix-free F and G,
// Chebyshev with K >= 2 sweeps.  Each row performs the IEEE operations of G's row followed by inner_solve's
// sweep (bit-identical), and the solve reads one pressure field instead of W's four velocity fields.
int f_solve_gx(const Ctx& c, const double* xp, const mpbp_inner_solver& in, double* dst, const double* sub,
               double* ping, double* pong, double* dir, bool profile) {
    const mpbp_schur_plan* p = c.p;
    const int K = in.sweeps;
    if (in.kind != MPBP_INNER_CHEBYSHEV || K < 2 || K > 64 || !(in.lmax > in.lmin) || !(in.lmin >= 0.0))
        return set_error(MPBP_ERR_ARG, "schur_apply (fused G): needs a Chebyshev F solve of 2..64 sweeps");
    double c1[64] = {}, c2[64] = {};
    cheb_coeffs(in.lmin, in.lmax, K, c1, c2);
    FStencilDev P;
    int rc = make_fstencil(&p->f_prm, p->f_cell, p->f_uface, p->f_vface, nullptr, &P);
    if (rc) return rc;
    PGDev G;
    rc = make_pgstencil(&p->f_prm, p->f_cell, nullptr, &G);
    if (rc) return rc;
    const GxB bs{xp, G.d_p, G.inv, G.minv, G.n};
    if (f_pair_ok(p) && KO().f_solve && fsolve_ok(K, P.n))   // the whole solve as one launch
        return profiled(p, profile, c.st, [&] { return launch_fsolve(P, K, c1, c2, nullptr, sub, dst, c.st, bs); });
    double* cur = K == 2 ? dst : pong;
    if (p->f_numerics == MPBP_NUMERICS_FAST && KO().f_tile && ftile_ok(P.n))   // x0 and sweep 1 on 2D tiles
        rc = launch_ftile<true>(P, FTile{nullptr, nullptr, nullptr, K == 2 ? sub : nullptr, cur, K == 2 ? nullptr : dir,
                                         0.0, c2[0], c1[1], c2[1]}, c.st, bs);
    else
    rc = with_f_policy(P, p->f_numerics == MPBP_NUMERICS_FAST, [&](const auto& Q) {
        return launch_march_init(Q, nullptr, c2[0], EpiChebFirst{nullptr, dir, c1[1], c2[1], K == 2 ? sub : nullptr, cur,
                                                                 K == 2 ? 0 : 1}, KO().march_rows, c.st, bs);
    });
    if (rc) return rc;
    for (int s = 2; s < K;) {
        const bool pair = f_pair_ok(p) && s == K - 2;
        const bool last = s == K - 1 || pair;
        double* nxt = last ? dst : (cur == ping ? pong : ping);
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        const bool rec = profile && p->prof_events && p->prof_count && *p->prof_count < p->prof_capacity &&
                         hipStreamIsCapturing(c.st, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone;
        if (rec) MPBP_HIP(record_event((hipEvent_t)p->prof_events[2 * *p->prof_count], c.st));
        if (pair)
            rc = f_pair(p, -1, cur, nullptr, dir, c1[s], c2[s], c1[s + 1], c2[s + 1], sub, nxt, c.st, bs);
        else
            rc = with_f_policy(P, p->f_numerics == MPBP_NUMERICS_FAST, [&](const auto& Q) {
                return launch_march(Q, XPlain{cur}, EpiCheb{cur, nullptr, nullptr, dir, c1[s], c2[s], last ? sub : nullptr,
                                                            nxt, last ? 0 : 1}, KO().march_rows, c.st, bs);
            });
        if (rc) return rc;
        if (rec) {
            MPBP_HIP(record_event((hipEvent_t)p->prof_events[2 * *p->prof_count + 1], c.st));
            ++*p->prof_count;
        }
        cur = nxt;
        s += pair ? 2 : 1;
    }
    return MPBP_OK;
}

// ---- communication-avoiding schedule (row partition) ----
// A stencil operator over the owned rows and `ext` ghost rows each side.
OpRef ext_op(const mpbp_schur_plan* p, int32_t sop, int ext) {
    OpRef o{nullptr, nullptr, nullptr, p, false, 3, sop};
    o.ext = ext;
    return o;
}

// Inner solve whose result is needed on the owned rows and d_out ghost rows each side: no exchange --
// sweep s (of S = K - 1) runs on d_out + S - s ghost rows, the fused first sweep stages x0 from b and the
// ghost-row diagonal d_out + S rows deep.  Same IEEE operations per row as the one-GPU solve.
int ca_inner_solve(const Ctx& c, int32_t sop, const double* b, const double* diag_ext, const mpbp_inner_solver& in,
                   int32_t n_init, double* dst, const double* sub, double* ping, double* pong, double* dir, int d_out,
                   bool profile) {
    const mpbp_schur_plan* p = c.p;
    const int K = in.sweeps;
    double c1[64] = {}, c2[64] = {};   // zeros for Jacobi (never read uninitialised)
    if (K < 1 || K > 64) return set_error(MPBP_ERR_ARG, "inner sweeps must be in [1, 64]");
    const bool cheb = in.kind == MPBP_INNER_CHEBYSHEV;
    if (cheb) {
        if (!(in.lmax > in.lmin) || !(in.lmin >= 0.0)) return set_error(MPBP_ERR_ARG, "bad Chebyshev interval");
        cheb_coeffs(in.lmin, in.lmax, K, c1, c2);
    } else if (in.kind != MPBP_INNER_JACOBI) {
        return set_error(MPBP_ERR_ARG, "unknown inner solver %d", in.kind);
    }
    if (K == 1) {   // x = x0 elementwise on every row the caller needs (n_init: owned, or the whole ext vector)
        if (n_init <= 0) return MPBP_OK;
        if (cheb) k_cheb_init<<<grid_for(n_init), kBlock, 0, c.st>>>(n_init, b, diag_ext, c2[0], dir, sub, dst);
        else k_jacobi_init<<<grid_for(n_init), kBlock, 0, c.st>>>(n_init, b, diag_ext, sub, dst);
        MPBP_HIP(hipGetLastError());
        return MPBP_OK;
    }
    // Gt_G: the whole Chebyshev solve as one tiled launch over the owned + d_out ghost rows (bit-identical)
    if (cheb && sop == SOP_GTG && !sub && gtg_fused_ok(p, true)) {
        const mpbp_row_part q = stencil_part(ext_op(p, SOP_GTG, d_out));
        if (q.halo >= d_out + K - 1) return gtg_solve_fused(p, b, dst, c.st, &q, diag_ext);
    }
    // tolerance-mode F: the whole solve as one tiled launch over the owned + d_out ghost rows
    if (cheb && sop == SOP_F && f_pair_ok(p) && KO().f_solve && fsolve_ok(K, p->f_prm.n)) {
        const mpbp_row_part q = stencil_part(ext_op(p, SOP_F, d_out));
        FStencilDev P;
        int rc = make_fstencil(&p->f_prm, p->f_cell, p->f_uface, p->f_vface, &q, &P);
        if (rc) return rc;
        if (P.h >= d_out + K - 1)
            return profiled(p, profile, c.st, [&] { return launch_fsolve(P, K, c1, c2, b, sub, dst, c.st); });
    }
    double* cur = K == 2 ? dst : pong;
    int rc = op_first_sweep(ext_op(p, sop, d_out + K - 2), cheb, b, diag_ext, c2[0], c1[1], c2[1], dir,
                            K == 2 ? sub : nullptr, cur, c.st, K == 2 ? 0 : 1);
    if (rc) return rc;
    for (int s = 2; s < K;) {
        const bool pair = cheb && sop == SOP_F && f_pair_ok(p) && s == K - 2;
        const bool last = s == K - 1 || pair;
        double* nxt = last ? dst : (cur == ping ? pong : ping);
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        const bool rec = profile && p->prof_events && p->prof_count && *p->prof_count < p->prof_capacity &&
                         hipStreamIsCapturing(c.st, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone;
        if (rec) MPBP_HIP(record_event((hipEvent_t)p->prof_events[2 * *p->prof_count], c.st));
        const OpRef o = ext_op(p, sop, d_out + K - 1 - s);
        if (pair)   // level B on d_out ghost rows (the last sweep's), level A one deeper (sweep K-2's)
            rc = f_pair(p, d_out, cur, b, dir, c1[s], c2[s], c1[s + 1], c2[s + 1], sub, nxt, c.st);
        else
            rc = cheb ? op_cheb(o, cur, b, nullptr, c1[s], c2[s], dir, last ? sub : nullptr, nxt, c.st, last ? 0 : 1)
                      : op_jacobi(o, cur, b, nullptr, last ? sub : nullptr, nxt, c.st);
        if (rc) return rc;
        if (rec) {
            MPBP_HIP(record_event((hipEvent_t)p->prof_events[2 * *p->prof_count + 1], c.st));
            ++*p->prof_count;
        }
        cur = nxt;
        s += pair ? 2 : 1;
    }
    return MPBP_OK;
}

// The CA schedule's second F solve (owned rows) with W = G x_p recomputed inside its sweeps (GxB over x_p's ghost
// layout, which holds S_F + 1 ghost rows each side -- the G launch's d_W = S_F plus its one-row reach): no G launch
// and no W buffer; the same IEEE operations per row as ca_inner_solve after the G launch.
int ca_f_solve_gx(const Ctx& c, const double* xp, const mpbp_inner_solver& in, double* dst, const double* sub,
                  double* ping, double* pong, double* dir, bool profile) {
    const mpbp_schur_plan* p = c.p;
    const int K = in.sweeps;
    if (in.kind != MPBP_INNER_CHEBYSHEV || K < 2 || K > 64 || !(in.lmax > in.lmin) || !(in.lmin >= 0.0))
        return set_error(MPBP_ERR_ARG, "schur_apply (CA, fused G): needs a Chebyshev F solve of 2..64 sweeps");
    double c1[64] = {}, c2[64] = {};
    cheb_coeffs(in.lmin, in.lmax, K, c1, c2);
    PGDev G;
    int rc = make_pgstencil(&p->f_prm, p->f_cell, &p->p_part, &G);
    if (rc) return rc;
    const GxBPart bs{xp, G.d_p, G.inv, G.minv, G.n, G.L, G.h};
    auto fpol = [&](int ext, FStencilDev* P) {
        const mpbp_row_part q = stencil_part(ext_op(p, SOP_F, ext));
        return make_fstencil(&p->f_prm, p->f_cell, p->f_uface, p->f_vface, &q, P);
    };
    FStencilDev P;
    if (f_pair_ok(p) && KO().f_solve && fsolve_ok(K, p->f_prm.n) && bs.h >= K) {   // the whole solve as one launch
        if ((rc = fpol(0, &P))) return rc;
        if (P.h >= K - 1)
            return profiled(p, profile, c.st, [&] { return launch_fsolve(P, K, c1, c2, nullptr, sub, dst, c.st, bs); });
    }
    if ((rc = fpol(K - 2, &P))) return rc;
    double* cur = K == 2 ? dst : pong;
    rc = with_f_policy(P, p->f_numerics == MPBP_NUMERICS_FAST, [&](const auto& Q) {
        return launch_march_init(Q, nullptr, c2[0], EpiChebFirst{nullptr, dir, c1[1], c2[1], K == 2 ? sub : nullptr, cur,
                                                                 K == 2 ? 0 : 1}, KO().march_rows, c.st, bs);
    });
    if (rc) return rc;
    for (int s = 2; s < K;) {
        const bool pair = f_pair_ok(p) && s == K - 2;
        const bool last = s == K - 1 || pair;
        double* nxt = last ? dst : (cur == ping ? pong : ping);
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        const bool rec = profile && p->prof_events && p->prof_count && *p->prof_count < p->prof_capacity &&
                         hipStreamIsCapturing(c.st, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone;
        if (rec) MPBP_HIP(record_event((hipEvent_t)p->prof_events[2 * *p->prof_count], c.st));
        if (pair) {
            rc = f_pair(p, 0, cur, nullptr, dir, c1[s], c2[s], c1[s + 1], c2[s + 1], sub, nxt, c.st, bs);
        } else {
            if ((rc = fpol(K - 1 - s, &P))) return rc;
            rc = with_f_policy(P, p->f_numerics == MPBP_NUMERICS_FAST, [&](const auto& Q) {
                return launch_march(Q, XPlain{cur}, EpiCheb{cur, nullptr, nullptr, dir, c1[s], c2[s], last ? sub : nullptr,
                                                            nxt, last ? 0 : 1}, KO().march_rows, c.st, bs);
            });
        }
        if (rc) return rc;
        if (rec) {
            MPBP_HIP(record_event((hipEvent_t)p->prof_events[2 * *p->prof_count + 1], c.st));
            ++*p->prof_count;
        }
        cur = nxt;
        s += pair ? 2 : 1;
    }
    return MPBP_OK;
}

// The exchange of one vector, complete before the next launch.
void ca_exchange(const Ctx& c, int32_t kind, double* x_ext) {
    c.p->halo(c.p->halo_ctx, kind, x_ext, MPBP_HALO_BEGIN, (void*)c.st);
    c.p->halo(c.p->halo_ctx, kind, x_ext, MPBP_HALO_END, (void*)c.st);
}

// solve.py:257-277 with 2 halo exchanges: v (velocity and pressure parts) before the first F solve, x_b
// before the second Gt_G solve; every other operator runs on the ghost rows its successors read.
int schur_apply_ca(const Ctx& c, const double* v, double* out) {
    const mpbp_schur_plan* p = c.p;
    const int SF = p->inner_F.sweeps - 1, SP = p->inner_P.sweeps - 1, q = p->ca_reach_q;
    const int d_xa = q, d_rhs = d_xa + SP, d_Y = d_rhs + 1, d_W = SF, d_xp = d_W + 1, d_xb = d_xp + SP;
    if (SF < 0 || SP < 0 || q < 1 || p->f_part.halo < d_Y + SF || p->p_part.halo < d_rhs || p->p_part.halo < d_xb ||
        p->p_part.halo < q || !p->wu_ext || !p->diag_F_ext || !p->diag_P_ext)
        return set_error(MPBP_ERR_ARG, "schur_apply (CA): halo depths %d/%d below the schedule's %d/%d, or ext "
                         "buffers missing", p->f_part.halo, p->p_part.halo, d_Y + SF, d_rhs > d_xb ? d_rhs : d_xb);
    double *Y = p->wu[0], *U0 = p->wu[1], *U1 = p->wu[2], *Ud = p->wu[3], *Vu = p->wu_ext;
    double *Prhs = p->wp[0], *Pxa = p->wp[1], *Pxb = p->wp[2], *Pxp = p->wp[3];
    double *P0 = p->wp[4], *P1 = p->wp[5], *Pd = p->wp[6];
    double* Vp = Pxb;   // v's pressure part lives in x_b's buffer until Gt_F_G overwrites it
    int rc;
    // v with its halo: velocity d_Y + S_F rows deep, pressure d_rhs rows deep (one exchange each)
    MPBP_HIP(hipMemcpyAsync(Vu, v, sizeof(double) * (size_t)p->nu, hipMemcpyDeviceToDevice, c.st));
    MPBP_HIP(hipMemcpyAsync(Vp, v + p->nu, sizeof(double) * (size_t)p->np, hipMemcpyDeviceToDevice, c.st));
    if (p->halo_pair) {
        p->halo_pair(p->halo_ctx, Vu, Vp, (void*)c.st);
    } else {
        ca_exchange(c, MPBP_VEC_VELOCITY, Vu);
        ca_exchange(c, MPBP_VEC_PRESSURE, Vp);
    }
    // 1. Finv_v on owned + d_Y ghost rows                                    solve.py:258
    rc = ca_inner_solve(c, SOP_F, Vu, p->diag_F_ext, p->inner_F, p->nu_ext, Y, nullptr, U0, U1, Ud, d_Y, true);
    if (rc) return rc;
    // 2. rhs = D Finv_v + v_p on owned + d_rhs ghost rows                      solve.py:259
    rc = op_spmv(ext_op(p, SOP_D, d_rhs), MPBP_SPMV_ADD, Y, Vp, Prhs, c.st);
    if (rc) return rc;
    // 3. x_a = Gt_G^-1 rhs on owned + q ghost rows                            solve.py:265
    rc = ca_inner_solve(c, SOP_GTG, Prhs, p->diag_P_ext, p->inner_P, p->np_ext, Pxa, nullptr, P0, P1, Pd, d_xa, false);
    if (rc) return rc;
    // 4. x_b = Gt_F_G x_a on the owned rows (its columns reach q ghost rows)  solve.py:267
    //    (tolerance mode: the diamond's upper half over the rank's row block, as k_q13<SYM> on one GPU)
    if (q13p_ok(p)) {
        rc = launch_q13p(p, Pxa, EpiStore{Pxb}, c.st);
    } else {
        const OpPair Q = make_op(p, p->GtFG, p->Q_int, p->Q_bnd, p->Qs_int, p->Qs_bnd);
        rc = op_spmv(Q.in, MPBP_SPMV_STORE, Pxa, nullptr, Pxb, c.st);
        if (!rc) rc = op_spmv(Q.bd, MPBP_SPMV_STORE, Pxa, nullptr, Pxb, c.st);
    }
    if (rc) return rc;
    ca_exchange(c, MPBP_VEC_PRESSURE, Pxb);
    // 5. x_p = Gt_G^-1 x_b on owned + d_xp ghost rows                         solve.py:271
    rc = ca_inner_solve(c, SOP_GTG, Pxb, p->diag_P_ext, p->inner_P, p->np_ext, Pxp, nullptr, P0, P1, Pd, d_xp, false);
    if (rc) return rc;
    MPBP_HIP(hipMemcpyAsync(out + p->nu, Pxp, sizeof(double) * (size_t)p->np, hipMemcpyDeviceToDevice, c.st));
    // 6.+7. fused: the second F solve recomputes G x_p in its sweeps (Chebyshev F)   solve.py:273-276
    if (p->fuse_g && p->inner_F.kind == MPBP_INNER_CHEBYSHEV && p->inner_F.sweeps >= 2)
        return ca_f_solve_gx(c, Pxp, p->inner_F, out, Y, U0, U1, Ud, true);
    // 6. G x_p on owned + d_W ghost rows (into v's velocity buffer)          solve.py:273
    rc = op_spmv(ext_op(p, SOP_G, d_W), MPBP_SPMV_STORE, Pxp, nullptr, Vu, c.st);
    if (rc) return rc;
    // 7. u = Finv_v - F^-1 (G x_p) on the owned rows                          solve.py:274-276
    return ca_inner_solve(c, SOP_F, Vu, p->diag_F_ext, p->inner_F, p->nu, out, Y, U0, U1, Ud, 0, true);
}

}  // namespace

// Multigrid level 1 of the plan's F (kind MPBP_VEC_VELOCITY) or Gt_G (MPBP_VEC_PRESSURE) hierarchy applied matrix-free
// as ONE fused launch (k_gal1 / k_gal1p: R_0 (A_0 (P_0 x))), y = op(A_1 x) with the modes of mpbp_spmv -- the kernel the
// tolerance-mode multigrid apply runs for its level-1 sweeps and residuals, exposed for timing (bench.py mg_apply).
extern "C" int mpbp_mg_level1_apply(const mpbp_schur_plan* p, int32_t kind, int32_t mode, const double* x,
                                    const double* z, double* y, void* stream) {
    if (!p || !x || !y || (mode != MPBP_SPMV_STORE && !z)) return set_error(MPBP_ERR_ARG, "mg_level1_apply: bad args");
    if (int rc = check_opts(p->opts, "mg_level1_apply")) return rc;
    const OptsScope scope(p->opts);
    const mpbp_mg* m = kind == MPBP_VEC_VELOCITY ? p->mg_F : kind == MPBP_VEC_PRESSURE ? p->mg_P : nullptr;
    if (!m || p->halo || p->f_numerics != MPBP_NUMERICS_FAST || KO().mg_galerkin_mf != 2)
        return set_error(MPBP_ERR_ARG, "mg_level1_apply: a one-GPU fast plan with that multigrid hierarchy, "
                                       "kernel option mg_galerkin_mf = 2");
    const int sop = kind == MPBP_VEC_VELOCITY ? SOP_F : SOP_GTG;
    if ((sop == SOP_F && !p->f_stencil) || (sop == SOP_GTG && (!p->pg_stencil || !KO().mg_galerkin_mf_p)))
        return set_error(MPBP_ERR_ARG, "mg_level1_apply: the level-0 operator is not matrix-free");
    const OpPair fine = make_stencil_op(p, sop, false);
    const MgGal g{m, fine.in, nullptr, nullptr};
    const hipStream_t st = as_stream(stream);
    bool done = false;
    int rc = MPBP_OK;
    switch (mode) {
    case MPBP_SPMV_STORE: rc = gal_fused(g, XPlain{x}, EpiStore{y}, st, &done); break;
    case MPBP_SPMV_ADD: rc = gal_fused(g, XPlain{x}, EpiAdd{z, y}, st, &done); break;
    case MPBP_SPMV_RESID: rc = gal_fused(g, XPlain{x}, EpiResid{z, y}, st, &done); break;
    default: return set_error(MPBP_ERR_ARG, "mg_level1_apply: unknown mode %d", mode);
    }
    if (rc) return rc;
    return done ? MPBP_OK : set_error(MPBP_ERR_ARG, "mg_level1_apply: the grid / transfer kinds do not take the fused kernel");
}

extern "C" int mpbp_schur_apply(const mpbp_schur_plan* p, const double* v, double* out, void* stream) {
    if (!p || !v || !out) return set_error(MPBP_ERR_ARG, "schur_apply: bad args");
    for (int i = 0; i < 4; ++i)
        if (!p->wu[i]) return set_error(MPBP_ERR_ARG, "schur_apply: missing velocity workspace");
    for (int i = 0; i < 7; ++i)
        if (!p->wp[i]) return set_error(MPBP_ERR_ARG, "schur_apply: missing pressure workspace");
    if (!p->wu_owned || !p->diag_F || !p->diag_P) return set_error(MPBP_ERR_ARG, "schur_apply: missing operands");
    if (int rc = check_opts(p->opts, "schur_apply")) return rc;
    const OptsScope scope(p->opts);
    const Ctx c{p, as_stream(stream)};
    // the CA schedule needs every operator but Gt_F_G matrix-free on the marching kernel; otherwise the
    // per-sweep exchanges below (its deeper halos serve them as well)
    if (p->ca && p->halo && p->f_stencil && p->pg_stencil) return schur_apply_ca(c, v, out);
    if (p->f_stencil && p->halo && p->f_part.halo < 1)
        return set_error(MPBP_ERR_ARG, "schur_apply: a partitioned F stencil needs f_part");
    if (p->pg_stencil && p->halo && (p->p_part.halo < 1 || p->f_part.halo < 1))
        return set_error(MPBP_ERR_ARG, "schur_apply: partitioned D / G / Gt_G stencils need f_part and p_part");
    if ((p->f_stencil || p->pg_stencil) && !p->f_cell)
        return set_error(MPBP_ERR_ARG, "schur_apply: stencil operators need the thn tables");
    const bool part = p->halo != nullptr && !p->halo_first;   // stencils split interior / boundary rows
    const OpPair F = p->f_stencil ? make_stencil_op(p, SOP_F, part)
                                  : make_op(p, p->F, p->F_int, p->F_bnd, p->Fs_int, p->Fs_bnd);
    const OpPair D = p->pg_stencil ? make_stencil_op(p, SOP_D, part)
                                   : make_op(p, p->D, p->D_int, p->D_bnd, p->Ds_int, p->Ds_bnd);
    const OpPair G = p->pg_stencil ? make_stencil_op(p, SOP_G, part)
                                   : make_op(p, p->G, p->G_int, p->G_bnd, p->Gs_int, p->Gs_bnd);
    const OpPair P = p->pg_stencil ? make_stencil_op(p, SOP_GTG, part)
                                   : make_op(p, p->GtG, p->P_int, p->P_bnd, p->Ps_int, p->Ps_bnd);
    const OpPair Q = make_op(p, p->GtFG, p->Q_int, p->Q_bnd, p->Qs_int, p->Qs_bnd);
    const double* v_u = v;
    const double* v_p = v + p->nu;
    double* out_u = out;
    double* out_p = out + p->nu;
    double *Y = p->wu[0], *U0 = p->wu[1], *U1 = p->wu[2], *Ud = p->wu[3], *W = p->wu_owned;
    double *Prhs = p->wp[0], *Pxa = p->wp[1], *Pxb = p->wp[2], *Pxp = p->wp[3];
    double *P0 = p->wp[4], *P1 = p->wp[5], *Pd = p->wp[6];
    int rc;
    // one GPU, matrix-free D and Gt_G, Chebyshev Gt_G solves: b's producers (D, Gt_F_G) also write the first Gt_G
    // sweep's x0 = c2[0] b / diag into P0 (the solve's ping buffer, first overwritten by its second sweep)
    // ... unless each Gt_G solve runs as one fused launch (k_gtg_solve), which builds x0 itself
    const bool gfuse = gtg_fused_ok(p);
    const bool px0 = !gfuse && p->pg_stencil && !p->halo && p->inner_P.kind == MPBP_INNER_CHEBYSHEV &&
                     p->inner_P.sweeps >= 2 && p->inner_P.lmax > p->inner_P.lmin && p->inner_P.lmin >= 0.0 &&
                     p->inner_P.sweeps <= 64;
    double pc1[64] = {}, pc2[64] = {};
    if (px0) cheb_coeffs(p->inner_P.lmin, p->inner_P.lmax, p->inner_P.sweeps, pc1, pc2);
    // 1. Finv_v = F_inv @ v[:F.shape[1]]                                   solve.py:258
    rc = inner_solve(c, MPBP_VEC_VELOCITY, F, p->diag_F, p->inner_F, p->nu, v_u, Y, nullptr, U0, U1, Ud, true);
    if (rc) return rc;
    // 2.+3. fused: the first Gt_G solve builds rhs = D Finv_v + v_p itself          solve.py:259, 265
    if (gfuse && KO().gtg_drhs && p->pg_stencil && !px0) {
        rc = gtg_solve_fused(p, nullptr, Pxa, c.st, nullptr, nullptr, GtgD{Y, v_p});
        if (rc) return rc;
    } else {
    // 2. rhs_interim = D @ Finv_v + v[F.shape[1]:]                            solve.py:259
    if (px0)
        rc = d_rhs_x0(p, Y, v_p, Prhs, pc2[0], P0, c.st);
    else
        rc = two_phase(c, MPBP_VEC_VELOCITY, Y, D,
                       [&](const OpRef& o) { return op_spmv(o, MPBP_SPMV_ADD, Y, v_p, Prhs, c.st); });
    if (rc) return rc;
    // 3. x_a = Gt_G_factorization @ rhs_interim                             solve.py:265
    rc = gfuse ? gtg_solve_fused(p, Prhs, Pxa, c.st)
               : inner_solve(c, MPBP_VEC_PRESSURE, P, p->diag_P, p->inner_P, p->np, Prhs, Pxa, nullptr, P0, P1, Pd, false,
                             px0 ? P0 : nullptr);
    if (rc) return rc;
    }
    // 4. x_b = Gt_F_G @ x_a                                                solve.py:267
    //    (one GPU: the diamond layout when the plan has it)
    const bool qmf = qmf_ok(p);   // tolerance mode: the product as its factors, matrix-free (k_qmf)
    const bool qx0 = px0 && (p->q13 || qmf);
    if (qx0 && qmf)
        rc = launch_qmf(p, Pxa, EpiStoreX0{Pxb, p->diag_P, pc2[0], P0}, c.st);
    else if (qx0)
        rc = launch_q13(p->q13_n, p->q13, Pxa, EpiStoreX0{Pxb, p->diag_P, pc2[0], P0}, c.st,
                        KO().q13_sym && p->f_numerics == MPBP_NUMERICS_FAST);
    else if (qmf)
        rc = launch_qmf(p, Pxa, EpiStore{Pxb}, c.st);
    else if (p->q13 && !p->halo)   // tolerance mode: the symmetric product's upper half (k_q13<SYM>)
        rc = launch_q13(p->q13_n, p->q13, Pxa, EpiStore{Pxb}, c.st, KO().q13_sym && p->f_numerics == MPBP_NUMERICS_FAST);
    else if (q13p_ok(p)) {         // ... and on a row partition: x_a's ghost rows first, then the rank's rows
        ca_exchange(c, MPBP_VEC_PRESSURE, Pxa);
        rc = launch_q13p(p, Pxa, EpiStore{Pxb}, c.st);
    } else
        rc = two_phase(c, MPBP_VEC_PRESSURE, Pxa, Q,
                       [&](const OpRef& o) { return op_spmv(o, MPBP_SPMV_STORE, Pxa, nullptr, Pxb, c.st); });
    if (rc) return rc;
    // 5. x_p = Gt_G_factorization @ x_b                                    solve.py:271
    //    (one GPU: straight into the output, which G then reads; a partition needs x_p's ghost rows)
    if (!p->halo) Pxp = out_p;
    rc = gfuse ? gtg_solve_fused(p, Pxb, Pxp, c.st)
               : inner_solve(c, MPBP_VEC_PRESSURE, P, p->diag_P, p->inner_P, p->np, Pxb, Pxp, nullptr, P0, P1, Pd, false,
                             qx0 ? P0 : nullptr);
    if (rc) return rc;
    if (Pxp != out_p)
        MPBP_HIP(hipMemcpyAsync(out_p, Pxp, sizeof(double) * (size_t)p->np, hipMemcpyDeviceToDevice, c.st));
    // 6.+7. fused: the second F solve recomputes G x_p in its sweeps (one GPU, matrix-free F and G, Chebyshev F)
    if (p->fuse_g && !p->halo && p->f_stencil && p->pg_stencil && p->inner_F.kind == MPBP_INNER_CHEBYSHEV &&
        p->inner_F.sweeps >= 2)
        return f_solve_gx(c, Pxp, p->inner_F, out_u, Y, U0, U1, Ud, true);
    // 6. G_xp = G @ x_p                                                     solve.py:273
    rc = two_phase(c, MPBP_VEC_PRESSURE, Pxp, G,
                   [&](const OpRef& o) { return op_spmv(o, MPBP_SPMV_STORE, Pxp, nullptr, W, c.st); });
    if (rc) return rc;
    // 7. u = Finv_v - F_inv @ G_xp                                          solve.py:274-276
    return inner_solve(c, MPBP_VEC_VELOCITY, F, p->diag_F, p->inner_F, p->nu, W, out_u, Y, U0, U1, Ud, true);
}

// ======================================================= multigrid (C ABI) ====
extern "C" {

static int mg_fields(int32_t n, int32_t nfields, const int32_t* kinds, MgFields* F) {
    if (n < 4 || (n & 1) || nfields < 1 || nfields > 8 || !kinds)
        return set_error(MPBP_ERR_ARG, "mg_transfer: need even n >= 4 and 1..8 fields");
    F->nfields = nfields;
    for (int f = 0; f < nfields; ++f) {
        F->ky[f] = kinds[2 * f];
        F->kx[f] = kinds[2 * f + 1];
        if ((F->ky[f] != MPBP_MG_CELL && F->ky[f] != MPBP_MG_NODE) || (F->kx[f] != MPBP_MG_CELL && F->kx[f] != MPBP_MG_NODE))
            return set_error(MPBP_ERR_ARG, "mg_transfer: field kinds must be MPBP_MG_CELL or MPBP_MG_NODE");
    }
    if ((int64_t)nfields * n * n > INT32_MAX) return set_error(MPBP_ERR_ARG, "mg_transfer: too many rows");
    return MPBP_OK;
}

static int64_t mg_rows(int32_t n, int32_t nfields, int32_t which) {
    const int64_t m = which == MPBP_MG_P ? n : n / 2;
    return (int64_t)nfields * m * m;
}

int mpbp_mg_transfer_count(int32_t n, int32_t nfields, const int32_t* kinds, int32_t which, int32_t* row_nnz,
                           void* stream) {
    MgFields F;
    const int rc = mg_fields(n, nfields, kinds, &F);
    if (rc) return rc;
    if (!row_nnz || (which != MPBP_MG_P && which != MPBP_MG_R)) return set_error(MPBP_ERR_ARG, "mg_transfer: bad args");
    const int64_t rows = mg_rows(n, nfields, which);
    k_mg_transfer<<<grid_for(rows), kBlock, 0, as_stream(stream)>>>(F, n, which, rows, nullptr, row_nnz, nullptr, nullptr);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int mpbp_mg_transfer_fill(int32_t n, int32_t nfields, const int32_t* kinds, int32_t which, const int32_t* row_ptr,
                          int32_t* col_idx, double* val, void* stream) {
    MgFields F;
    const int rc = mg_fields(n, nfields, kinds, &F);
    if (rc) return rc;
    if (!row_ptr || !col_idx || !val || (which != MPBP_MG_P && which != MPBP_MG_R))
        return set_error(MPBP_ERR_ARG, "mg_transfer: bad args");
    const int64_t rows = mg_rows(n, nfields, which);
    k_mg_transfer<<<grid_for(rows), kBlock, 0, as_stream(stream)>>>(F, n, which, rows, row_ptr, nullptr, col_idx, val);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int mpbp_mg_transfer_rows_count(int32_t n, int32_t nfields, const int32_t* kinds, int32_t which, const int32_t* rows,
                                int32_t nrows, int32_t* row_nnz, void* stream) {
    MgFields F;
    const int rc = mg_fields(n, nfields, kinds, &F);
    if (rc) return rc;
    if (nrows < 0 || (nrows && (!rows || !row_nnz)) || (which != MPBP_MG_P && which != MPBP_MG_R))
        return set_error(MPBP_ERR_ARG, "mg_transfer_rows: bad args");
    if (nrows == 0) return MPBP_OK;
    k_mg_transfer<<<grid_for(nrows), kBlock, 0, as_stream(stream)>>>(F, n, which, nrows, nullptr, row_nnz, nullptr,
                                                                     nullptr, rows);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int mpbp_mg_transfer_rows_fill(int32_t n, int32_t nfields, const int32_t* kinds, int32_t which, const int32_t* rows,
                               int32_t nrows, const int32_t* row_ptr, int32_t* col_idx, double* val, void* stream) {
    MgFields F;
    const int rc = mg_fields(n, nfields, kinds, &F);
    if (rc) return rc;
    if (nrows < 0 || (nrows && (!rows || !row_ptr || !col_idx || !val)) || (which != MPBP_MG_P && which != MPBP_MG_R))
        return set_error(MPBP_ERR_ARG, "mg_transfer_rows: bad args");
    if (nrows == 0) return MPBP_OK;
    k_mg_transfer<<<grid_for(nrows), kBlock, 0, as_stream(stream)>>>(F, n, which, nrows, row_ptr, nullptr, col_idx, val,
                                                                     rows);
    MPBP_HIP(hipGetLastError());
    return MPBP_OK;
}

int mpbp_mg_solve(const mpbp_mg* mg, const double* b, const double* sub, double* x_out, void* stream) {
    if (!mg || !b || !x_out || mg->nlevels < 2 || !mg->levels) return set_error(MPBP_ERR_ARG, "mg_solve: bad args");
    if (int rc = check_opts(mg->opts, "mg_solve")) return rc;
    const OptsScope scope(mg->opts);
    const mpbp_mg_level& L = mg->levels[0];
    if (check_csr(&L.A)) return MPBP_ERR_ARG;
    if (mg->part_levels < 0 || mg->part_levels >= mg->nlevels || (mg->part_levels > 0 && (!mg->halo || !mg->gather)))
        return set_error(MPBP_ERR_ARG, "mg_solve: part_levels must be in [0, nlevels) with halo and gather callbacks");
    for (int l = 0; l < mg->nlevels; ++l) {
        const mpbp_mg_level& Q = mg->levels[l];
        if (!Q.x || !Q.t || !Q.r || !Q.d || !Q.b || !Q.diag)
            return set_error(MPBP_ERR_ARG, "mg_solve: level %d is missing work vectors", l);
        // (row-partitioned levels: the transfers' columns index the ghost layout, so only the row counts are checked)
        const bool part = l < mg->part_levels;
        if (l + 1 < mg->nlevels && (Q.P.nrows != Q.nrows ||
                                    (!part && (Q.R.nrows != mg->levels[l + 1].nrows || Q.P.ncols != mg->levels[l + 1].nrows ||
                                               Q.R.ncols != Q.nrows))))
            return set_error(MPBP_ERR_ARG, "mg_solve: transfer shapes of level %d do not match", l);
    }
    const MgFine f{mg_level_op(L), L.diag, L.x, L.t, L.r, L.d, mg->part_levels > 0 ? mg->halo : nullptr, mg->halo_ctx,
                   L.halo_kind};
    return mg_solve(mg, f, b, x_out, sub, as_stream(stream));
}

}  // extern "C"
