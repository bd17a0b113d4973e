/* libmpbp -- MI355X (gfx950) multiphase-Stokes block-preconditioner apply, C ABI.
 *
 * Plain pointers and sizes only.  Every pointer named "device" lives in HBM
 * (hipMalloc / torch allocations); every `stream` is a hipStream_t passed as
 * void*.  All functions return MPBP_OK (0) or a negative error code, with a
 * message in mpbp_last_error().  No function allocates or synchronises unless
 * its comment says "setup" -- the apply path is graph-capturable.
 *
 * Reference interfaces replaced (abarret/mp-block-preconditioners @ 2025-02-23):
 *   mpbp_stokes_*         MultiphaseBlockPreconditioner.get_block_matrices   preconditioner.py:86-297
 *                         MultiphaseBlockPreconditioner.get_big_A_matrix     preconditioner.py:299-341
 *                         (thn / ths volume fractions                        preconditioner.py:9-15)
 *   mpbp_spgemm_*         Gt_G = np.matmul(mD, G), Gt_F_G = (mD F) G          solve.py:246-249
 *   mpbp_spmv             b_approx = np.matmul(A, u_vec)                      apply.py:72
 *                         A @ xk in the FGMRES residual callback              solve.py:166
 *   mpbp_jacobi_*         Jacobi(A, b, N, x)                                  solve.py:149-159
 *   mpbp_cheb_*           inner Chebyshev sweeps (BASELINE.json configs[3])
 *   mpbp_f_stencil_*      the F products / sweeps above with F's rows recomputed from thn
 *   mpbp_pg_stencil_spmv  D @ Finv_v (solve.py:259), G @ x_p (solve.py:273), Gt_G products
 *   mpbp_gtg_stencil_*    sweeps over Gt_G = np.matmul(mD, G) (solve.py:246, 265, 271)
 *   mpbp_schur_apply      approx_schur_op(v) -- the LinearOperator matvec    solve.py:257-277
 */
#ifndef MPBP_H
#define MPBP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPBP_OK 0
#define MPBP_ERR_ARG (-1)
#define MPBP_ERR_HIP (-2)
#define MPBP_ERR_OVERFLOW (-3)
#define MPBP_ERR_PATTERN (-4)

/* operator ids for mpbp_stokes_{rows,cols,count,fill} */
#define MPBP_OP_A 0    /* [[F, G], [d_div D, 0]], 5N x 5N                 preconditioner.py:339-341 */
#define MPBP_OP_F 1    /* XI + d_u blockdiag(eta_n L_n, eta_s L_s), 4N x 4N preconditioner.py:331-337 */
#define MPBP_OP_D 2    /* hstack(D_n, D_s) (unscaled), N x 4N             preconditioner.py:311 */
#define MPBP_OP_G 3    /* vstack(d_p G_n, d_p G_s), 4N x N                preconditioner.py:313 */
#define MPBP_OP_L_N 4  /* per-phase blocks of get_block_matrices(is_ths)  preconditioner.py:86-297 */
#define MPBP_OP_L_S 5
#define MPBP_OP_D_N 6
#define MPBP_OP_D_S 7
#define MPBP_OP_G_N 8
#define MPBP_OP_G_S 9
#define MPBP_OP_XI_N 10
#define MPBP_OP_XI_S 11

/* spmv epilogues */
#define MPBP_SPMV_STORE 0  /* y = A x          */
#define MPBP_SPMV_ADD 1    /* y = A x + z      */
#define MPBP_SPMV_RESID 2  /* y = z - A x      */
/* OR'ed into mpbp_f_stencil_spmv's mode: the tolerance-mode F rows (MPBP_NUMERICS_FAST below) */
#define MPBP_SPMV_FAST 0x100

/* Numerics of the matrix-free F sweeps (mpbp_schur_plan.f_numerics).  EXACT: every row performs the assembly's IEEE
 * operations in CSR order (bit-identical to the sequential oracle).  FAST: the same operator with its rows regrouped
 * per coefficient and FMA-contracted, reciprocal diagonals (v_rcp_f64 + 2 Newton steps) -- north_star's bar, within
 * 1e-12 relative inf-norm of the oracle apply; ~4x fewer fp64 VALU operations per row. */
#define MPBP_NUMERICS_EXACT 0
#define MPBP_NUMERICS_FAST 1

/* inner solvers of the approximate Schur preconditioner */
#define MPBP_INNER_JACOBI 0
#define MPBP_INNER_CHEBYSHEV 1
#define MPBP_INNER_MG 2         /* geometric multigrid V-cycles (plan.mg_F / plan.mg_P); sweeps = cycles */

/* multigrid transfers: per field and axis, cell- or node-centred; which operator */
#define MPBP_MG_CELL 0
#define MPBP_MG_NODE 1
#define MPBP_MG_P 0   /* prolongation, fine x coarse */
#define MPBP_MG_R 1   /* restriction = P^T, coarse x fine */

/* halo callback phases / vector kinds (multi-GPU row partition) */
#define MPBP_HALO_BEGIN 0
#define MPBP_HALO_END 1
#define MPBP_VEC_VELOCITY 0
#define MPBP_VEC_PRESSURE 1

typedef struct mpbp_csr {
    int32_t nrows;
    int32_t ncols;
    int64_t nnz;
    const int32_t* row_ptr; /* device, nrows + 1 */
    const int32_t* col_idx; /* device, nnz */
    const double* val;      /* device, nnz */
} mpbp_csr;

/* Row blocks: `count` (start, end) row pairs, device int32[2*count]; each block has at most 256
 * rows and at most MPBP_BLOCK_NNZ nonzeros (or is a single longer row).  Built on the host by
 * mpbp_plan_row_blocks from a host copy of row_ptr. */
typedef struct mpbp_rowblocks {
    const int32_t* pairs;
    int32_t count;
    int32_t reserved;
    /* optional wave table (NULL: the kernels read row_ptr): per block 8 int32 {start row, end row, row_ptr[min(start +
     * 64 w, end)] for w = 0..4, uniform flags} -- byte w of the flags is LEN when the block's wave w covers 64 rows of
     * LEN in {8, 10, 12} entries each from an even entry offset, else 0.  The CSR SpMV's waves then start their matrix
     * loads from one scalar load of the table, with no row_ptr reads on uniform waves.  Built on the host from the same
     * row_ptr as `pairs` (csr.RowBlockList); a plan belongs to its matrix's structure. */
    const int32_t* table;
} mpbp_rowblocks;

#define MPBP_BLOCK_ROWS 256
#define MPBP_BLOCK_NNZ 4095

/* SELL-64: sliced ELLPACK, one wavefront (64 rows) per slice, entries column-major in pairs.
 * slices: device int32[4*nslices] = {row0, rows (<= 64), width, first pair-row}; row_len: device
 * uint8[nrows]; val / col: device arrays of 128 doubles / int32 per pair-row (zero padding). */
typedef struct mpbp_sell {
    int32_t nrows;
    int32_t ncols;
    int32_t nslices;
    int32_t reserved;
    const int32_t* slices;
    const uint8_t* row_len;
    const double* val;
    const int32_t* col;
} mpbp_sell;

/* Stencil-values layout of a translation-invariant operator on `nfields` stacked m x m periodic fields (the
 * multigrid's Galerkin levels: every row of field f holds the same `slots` (field, dr, dc) offsets): the values
 * alone, slot-major (vals[s * nrows + row], slot order = an interior row's CSR column order), the columns rebuilt as
 * row + delta[f * slots + s].  Interior rows (reach <= r, c < m - reach; m and reach even: the kernel takes
 * interior cells in horizontal pairs with 16-byte value loads) sum in slot order; the rows within `reach`
 * of the periodic edge (edge_rows, whose wrapped columns sort differently) are summed from the CSR form.  Same
 * products in the same order as the CSR SpMV: bit-identical.  Built by the Python layer (mg.stencil_values). */
typedef struct mpbp_svl {
    int32_t nfields, m, reach, slots;
    const int32_t* delta;            /* device, nfields * slots */
    const double* vals;              /* device, slots * nrows */
    const int32_t* edge_rows;        /* device, n_edge row ids */
    int32_t n_edge;
    int32_t reserved;
} mpbp_svl;

/* Grid-row partition of the 4 velocity fields (multi-GPU F stencil): the rank owns grid rows
 * [r0, r0 + rows) of every field, followed in its vectors by the ghost rows: `halo` rows above of
 * every field (field-major), then `halo` rows below of every field.  which: 0 all owned rows, 1 rows off the first/last owned grid row, 2 those
 * rows.  NULL (or halo = 0) = one GPU, whole grid. */
typedef struct mpbp_row_part {
    int32_t r0;
    int32_t rows;
    int32_t halo;
    int32_t which;  /* 3: rows [-ext, rows + ext) -- the owned rows and `ext` ghost rows each side */
    int32_t ext;    /* which = 3 only: ghost rows computed redundantly on each side (<= the halo depths) */
    int32_t oh;     /* ghost depth of the OUTPUT vector's layout when it differs from `halo` (D: pressure
                       out of velocity, G: velocity out of pressure); 0 = same as halo */
} mpbp_row_part;

typedef struct mpbp_stokes_params {
    int32_t n;     /* grid is n x n, N = n*n cells, dx = dy = 1/n */
    double xi;     /* drag coefficient */
    double eta_n;  /* network viscosity */
    double eta_s;  /* solvent viscosity */
    double c;      /* c (w_thn = c * thn) */
    double d_u;    /* d_u (viscous / drag scaling) */
    double d_p;    /* d_p (gradient scaling) */
    double d_div;  /* d_div (divergence scaling) */
} mpbp_stokes_params;

typedef struct mpbp_inner_solver {
    int32_t kind;   /* MPBP_INNER_JACOBI or MPBP_INNER_CHEBYSHEV */
    int32_t sweeps; /* >= 1 updates of x from x0 = 0 (sweeps - 1 SpMVs) */
    double lmin;    /* Chebyshev interval of diag(A)^-1 A; ignored by Jacobi */
    double lmax;
} mpbp_inner_solver;

/* One level of a geometric multigrid hierarchy (Galerkin: A_{l+1} = R_l A_l P_l).  The coarsest level's A is
 * solved by mpbp_mg.coarse_inv; R / P are unused there. */
typedef struct mpbp_mg_level {
    int32_t nrows;
    int32_t pre, post;               /* Chebyshev-Jacobi smoothing sweeps (>= 1) */
    int32_t part_r0;                 /* row partition: the first grid row this rank owns of every field of the level */
    double lmin, lmax;               /* smoothing interval of diag(A)^-1 A */
    mpbp_csr A;
    mpbp_rowblocks A_blocks;
    const double* diag;              /* device, nrows */
    mpbp_csr R;                      /* to level + 1 */
    mpbp_rowblocks R_blocks;
    mpbp_csr P;                      /* from level + 1 */
    mpbp_rowblocks P_blocks;
    double *x, *t, *r, *d, *b;       /* device work vectors, nrows each */
    /* optional SELL-64 copies (nslices > 0: used instead of the CSR form, same bits): the Galerkin coarse
     * operators' long uniform rows (20-50 entries) stream better one row per lane */
    mpbp_sell A_sell;
    mpbp_sell R_sell;
    mpbp_sell P_sell;
    /* row partition (mpbp_mg.part_levels > l): the halo kind of this level's vectors; nrows counts the owned rows,
     * x / t / r hold owned + ghost rows (the ext layout), R's columns index that layout and P's the next level's
     * (or, at the last partitioned level, the whole next level) */
    int32_t halo_kind;
    int32_t part_h;                  /* row partition: ghost rows each side of this level's x / t / r (0: whole level) */
    /* optional stencil-values copy of A (NULL: none; used for levels above the grouped kernel's row limit) */
    const mpbp_svl* A_svl;
} mpbp_mg_level;

typedef void (*mpbp_halo_fn)(void* ctx, int32_t vec_kind, double* x_ext, int32_t phase, void* stream);
/* A velocity and a pressure vector's halos in one exchange, complete on `stream` when it returns. */
typedef void (*mpbp_halo_pair_fn)(void* ctx, double* xu_ext, double* xp_ext, void* stream);
/* All-gather of a row-partitioned vector into the whole field-major vector on every rank (on `stream`). */
typedef void (*mpbp_gather_fn)(void* ctx, int32_t gather_kind, const double* x_owned, double* x_full, void* stream);

struct mpbp_kernel_opts;   /* kernel choices: see "kernel choices" below */

typedef struct mpbp_mg {
    int32_t nlevels;                 /* >= 2 */
    int32_t cycles;                  /* V-cycles per solve, from x = 0 */
    const mpbp_mg_level* levels;     /* host array */
    mpbp_csr coarse_inv;             /* (pseudo-)inverse of the coarsest A, every entry stored */
    mpbp_rowblocks coarse_inv_blocks;
    const double* coarse_dense;      /* optional: the same inverse column-major (m x m, m = coarsest nrows), applied
                                      * by a dense kernel (one row per lane, the CSR row's order); NULL: CSR */
    /* Row partition over ranks (multi-GPU; 0 / NULL on one GPU).  Levels [0, part_levels) are row-partitioned (each
     * rank its grid rows, ghost rows refreshed through `halo` before every operator that reads them; level 0 inside
     * mpbp_schur_apply through the plan's halo); the restriction into level part_levels leaves the rank's rows of
     * that level in its r buffer, `gather` (gather_kind) assembles the whole level in its b, and the coarser levels
     * run replicated on every rank.  1 <= part_levels <= nlevels - 1.  Same bits as the one-GPU hierarchy. */
    int32_t part_levels;
    int32_t gather_kind;
    mpbp_halo_fn halo;
    void* halo_ctx;                  /* passed to halo and gather */
    mpbp_gather_fn gather;
    /* optional (tr_nfields > 0): the transfers' field kinds (MPBP_MG_CELL / NODE along y and x per field, as
     * mpbp_mg_transfer_fill) and level 0's grid size: the whole-grid levels' restriction and prolongation are then
     * applied matrix-free, their weights and columns recomputed per row in the CSR form's order (same bits) */
    int32_t tr_nfields;
    int32_t tr_n0;
    int32_t tr_ky[8];
    int32_t tr_kx[8];
    const struct mpbp_kernel_opts* opts; /* optional: kernel choices of a standalone mpbp_mg_solve (NULL: defaults) */
} mpbp_mg;

/* The apply's operands.  On one GPU every matrix's columns index the full vector and the
 * *_bnd row blocks are empty.  Under a row partition the columns index the "ext" layout of the
 * input vector kind (owned rows first, then ghost rows) and the halo callback fills the ghosts:
 * BEGIN before the interior blocks are launched, END before the boundary blocks. */
typedef struct mpbp_schur_plan {
    int32_t nu, np;                  /* owned velocity rows (4N) and pressure rows (N) */
    int32_t nu_ext, np_ext;          /* owned + ghost */
    mpbp_csr F, D, G, GtG, GtFG;
    mpbp_rowblocks F_int, F_bnd, D_int, D_bnd, G_int, G_bnd, P_int, P_bnd, Q_int, Q_bnd; /* P: GtG, Q: GtFG */
    const double* diag_F;            /* device, nu */
    const double* diag_P;            /* device, np (diagonal of GtG) */
    mpbp_inner_solver inner_F, inner_P;
    double* wu[4];                   /* device velocity work vectors, nu_ext each (Y, U0, U1, dir) */
    double* wu_owned;                /* device, nu (W = G x_p) */
    double* wp[7];                   /* device pressure work vectors, np_ext each */
    mpbp_halo_fn halo;               /* NULL on one GPU */
    void* halo_ctx;
    void** prof_events;              /* optional: hipEvent_t pairs around every inner-F SpMV sweep */
    int32_t prof_capacity;           /* number of event pairs available */
    int32_t* prof_count;             /* host int: pairs recorded so far (caller resets) */
    int32_t use_sell;                /* 1: run the SELL-64 copies below instead of CSR row blocks */
    mpbp_sell Fs_int, Fs_bnd, Ds_int, Ds_bnd, Gs_int, Gs_bnd, Ps_int, Ps_bnd, Qs_int, Qs_bnd;
    int32_t f_stencil;               /* 1: F sweeps recompute F's rows from thn (one GPU, n >= 3) */
    mpbp_stokes_params f_prm;        /* the parameters F was assembled with */
    const double* f_cell;            /* device thn tables (n*n each) */
    const double* f_uface;
    const double* f_vface;
    mpbp_row_part f_part;            /* velocity partition (F, D stencils); halo = 0 on one GPU */
    int32_t pg_stencil;              /* 1: D, G and Gt_G recomputed from the cell thn table (n >= 3);
                                        f_prm / f_cell are set whenever f_stencil or pg_stencil is */
    mpbp_row_part p_part;            /* pressure partition (G, Gt_G stencils); halo = 0 on one GPU */
    int32_t halo_first;              /* 1: each exchange completes (BEGIN, END) before the sweep, whose
                                        stencil rows then run as one launch; 0: interior rows launch
                                        between BEGIN and END, boundary rows after */
    /* Communication-avoiding schedule (row partition, every operator but Gt_F_G matrix-free): v's halo
     * and x_b's halo are exchanged once each, deep enough that every other operator runs on its owned
     * rows plus the ghost rows its successors still need (computed redundantly): 2 exchanges per apply
     * instead of one per sweep.  Depths (S_F, S_P = inner sweeps - 1, q = ca_reach_q):
     *   f_part.halo >= q + S_P + 1 + S_F,  p_part.halo >= max(q + S_P, S_F + 1 + S_P). */
    int32_t ca;                      /* 1: use it (ignored on one GPU) */
    int32_t ca_reach_q;              /* grid-row reach of Gt_F_G's columns (its input's ghost depth) */
    double* wu_ext;                  /* device, nu_ext: v's velocity part with its halo, later G x_p */
    const double* diag_F_ext;        /* device, nu_ext: diag(F) on owned + ghost rows */
    const double* diag_P_ext;        /* device, np_ext: diag(Gt_G) on owned + ghost rows */
    mpbp_halo_pair_fn halo_pair;     /* optional (CA schedule): both halves of v in one exchange
                                        (mpbp_halo_exchange_pair); NULL: two halo calls */
    const double* q13;               /* optional: Gt_F_G in the 13-point diamond layout (mpbp_q13_build), used
                                        instead of GtFG / Qs_* when set.  Row partition (tolerance mode, q13_sym):
                                        the diamond of grid rows p_part.r0 - 2 .. r0 + rows - 1 (mpbp_q13_build_rows),
                                        read as its symmetric upper half -- the one-GPU k_q13<SYM> bits per row */
    int32_t q13_n;                   /* its grid size n */
    const mpbp_mg* mg_F;             /* inner_F.kind == MPBP_INNER_MG: F's hierarchy (level 0 = F; row-partitioned
                                        with part_levels >= 1 when halo is set) */
    const mpbp_mg* mg_P;             /* inner_P.kind == MPBP_INNER_MG: Gt_G's hierarchy */
    int32_t fuse_g;                  /* 1 (one GPU, f_stencil and pg_stencil, Chebyshev F solve of >= 2 sweeps): the
                                        second F solve recomputes its right-hand side G x_p inside each sweep (no G
                                        launch, W never stored; bit-identical) */
    int32_t f_numerics;              /* MPBP_NUMERICS_EXACT (0, default) or MPBP_NUMERICS_FAST: the matrix-free F
                                        sweeps' rows (inner solves, multigrid level 0 smoothing and residuals) */
    const struct mpbp_kernel_opts* opts; /* optional: this plan's kernel choices (NULL: the process defaults); they
                                        also govern the plan's multigrid hierarchies inside the apply */
} mpbp_schur_plan;

const char* mpbp_version(void);
const char* mpbp_last_error(void);

/* ---- assembly (setup) ---------------------------------------------------------------------- */
/* thn at cell centres / u faces / v faces, preconditioner.py:9-11 (device arrays of n*n). */
int mpbp_stokes_theta(int32_t n, double* cell, double* uface, double* vface, void* stream);
int64_t mpbp_stokes_rows(int32_t n, int32_t op);
int64_t mpbp_stokes_cols(int32_t n, int32_t op);
/* row_nnz[r] for every row of `op` (device int32[rows]). */
int mpbp_stokes_count(const mpbp_stokes_params* prm, int32_t op, const double* cell,
                      int32_t* row_nnz, void* stream);
/* Fill col_idx / val given row_ptr (device).  Columns sorted within each row. */
int mpbp_stokes_fill(const mpbp_stokes_params* prm, int32_t op, const double* cell,
                     const double* uface, const double* vface, const int32_t* row_ptr,
                     int32_t* col_idx, double* val, void* stream);
/* row_ptr[0] = 0, row_ptr[i+1] = row_ptr[i] + row_nnz[i] (device); *total (host) = row_ptr[n].
 * Setup: synchronises the stream. */
/* The same for a subset of the operator's rows (a rank's owned + ghost rows, preconditioner.py:299-341 row by row):
 * row i of the output is operator row rows[i] (0 <= rows[i] < mpbp_stokes_rows), with its global columns -- the
 * global assembly's rows bit for bit, without assembling the others.  row_ptr is indexed by i (nrows + 1 entries). */
int mpbp_stokes_count_rows(const mpbp_stokes_params* prm, int32_t op, const double* cell, const int32_t* rows,
                           int32_t nrows, int32_t* row_nnz, void* stream);
int mpbp_stokes_fill_rows(const mpbp_stokes_params* prm, int32_t op, const double* cell, const double* uface,
                          const double* vface, const int32_t* rows, int32_t nrows, const int32_t* row_ptr,
                          int32_t* col_idx, double* val, void* stream);
int mpbp_exclusive_scan(const int32_t* row_nnz, int32_t* row_ptr, int64_t n, int64_t* total,
                        void* stream);

/* ---- sparse products (setup) ----------------------------------------------------------------- */
/* C = alpha * A B with every structural product kept; row_nnz device int32[A.nrows].
 * Setup: synchronises the stream (returns MPBP_ERR_OVERFLOW for a row wider than 64). */
int mpbp_spgemm_count(const mpbp_csr* A, const mpbp_csr* B, int32_t* row_nnz, void* stream);
int mpbp_spgemm_fill(const mpbp_csr* A, const mpbp_csr* B, double alpha, const int32_t* row_ptr,
                     int32_t* col_idx, double* val, void* stream);

/* ---- Gt_F_G in the 13-point diamond layout ---------------------------------------------------- */
/* Gt_F_G = ((-D) F) G (solve.py:246-249) couples each pressure cell with the 13 cells |dr| + |dc| <= 2 (n >= 5).
 * mpbp_q13_build copies the CSR values into vals[13 * n^2] (slot-major, slots in (dr, dc) lexicographic order);
 * MPBP_ERR_ARG if a row is not exactly that diamond.  Setup: synchronises the stream.
 * mpbp_q13_spmv: y = Q x (modes as mpbp_spmv), the CSR SpMV's result bit for bit; replaces np.matmul(Gt_F_G, x_a)
 * (solve.py:267) -- the columns are implicit in the grid, so the layout streams 104 B per row instead of 156. */
int mpbp_q13_build(const mpbp_csr* Q, int32_t n, double* vals, void* stream);
/* y = op(A x) through the stencil-values layout V of A (edge rows from A's CSR arrays); modes as mpbp_spmv.  The
 * CSR SpMV's result bit for bit. */
int mpbp_svl_spmv(const mpbp_svl* V, const mpbp_csr* A, int32_t mode, const double* x, const double* z, double* y,
                  void* stream);
/* One Chebyshev-Jacobi sweep (as mpbp_cheb_step) through the stencil-values layout: the multigrid's large-level
 * smoothing sweep, bit-identical to the CSR form. */
int mpbp_svl_cheb_step(const mpbp_svl* V, const mpbp_csr* A, const double* x_in, const double* b, const double* diag,
                       double c1, double c2, double* d, const double* sub, double* x_out, void* stream);
/* out[0] = max |Q(c, c + o) - Q(c + o, c)| over the diamond, out[1] = max |Q| (host doubles; synchronises the stream):
 * whether tolerance mode may read the symmetric half (mpbp_kernel_opts.q13_sym) for this product.  Setup. */
int mpbp_q13_asymmetry(int32_t n, const double* vals, double* out, void* stream);
/* mpbp_q13_build for a block of whole grid rows of Gt_F_G (a row partition's rows r0 - 2 .. r0 + L - 1, with global
 * columns): Q's row i is grid row (row0 + i / n) mod n; vals[13 * Q->nrows], slot-major.  Setup: synchronises. */
int mpbp_q13_build_rows(const mpbp_csr* Q, int32_t n, int32_t row0, double* vals, void* stream);
int mpbp_q13_spmv(int32_t n, const double* vals, int32_t mode, const double* x, const double* z, double* y,
                  void* stream);

/* ---- planning / helpers (setup) ------------------------------------------------------------ */
/* Host-side greedy row blocking of rows [row_begin, row_end) of a HOST row_ptr; writes at most
 * `capacity` pairs to `pairs` (host) and returns the number of blocks needed. */
int64_t mpbp_plan_row_blocks(const int32_t* row_ptr, int32_t row_begin, int32_t row_end,
                             int32_t* pairs, int64_t capacity);
/* diag[r] = A[r, r + col_offset]; *missing (host) = rows without that entry.  Setup (syncs). */
int mpbp_csr_diag(const mpbp_csr* A, int32_t col_offset, double* diag, int32_t* missing, void* stream);
/* *lmax (host) = max_r sum_k |A[r,k]| / |diag[r]| (Gershgorin bound of diag^-1 A). Setup (syncs). */
int mpbp_gershgorin(const mpbp_csr* A, const double* diag, double* lmax, void* stream);
/* Row extraction for a row partition: local row i = global row rows[i]; columns mapped through
 * colmap (global col -> local ext col, -1 = not available).  count writes row_nnz (device);
 * fill returns MPBP_ERR_PATTERN when a needed column is unmapped.  Setup (fill syncs). */
int mpbp_csr_extract_count(const mpbp_csr* A, const int32_t* rows, int32_t nrows_local,
                           int32_t* row_nnz, void* stream);
int mpbp_csr_extract_fill(const mpbp_csr* A, const int32_t* rows, int32_t nrows_local,
                          const int32_t* colmap, const int32_t* row_ptr_local, int32_t* col_local,
                          double* val_local, void* stream);

/* ---- apply path (graph-capturable, no sync) ------------------------------------------------ */
/* y = op(A x) over the rows of `blocks` (mode MPBP_SPMV_*; z unused for STORE). */
int mpbp_spmv(const mpbp_csr* A, const mpbp_rowblocks* blocks, int32_t mode, const double* x,
              const double* z, double* y, void* stream);
/* The same product at north_star's value bar: identical row_ptr / col_idx handling, each row's sum formed by a
 * wavefront segmented reduction (pairs per lane, DPP cross-lane adds, fused multiply-adds) -- within 1e-12
 * relative infinity norm of mpbp_spmv's sequential sums, not bit-identical; deterministic run to run.  Fast for
 * stencil rows (64-row waves of 8, 10 or 12 entries from an even start); other waves take a plain loop.
 * Replaces np.matmul(A, u_vec) (apply.py:72), whose BLAS sums are not sequential either. */
/* HBM calibration for the bench's roofline lines (measurement only, no result): mode 0 reads `bytes` of src once in
 * order; mode 1 reads floor(bytes / 9 KiB) 9-KiB chunks in order and writes 64 doubles of dst per chunk -- the CSR
 * SpMV's stream shape (a wave of 64 twelve-entry rows) without its x gathers.  dst: mode 0 a 256-double sink (never
 * written on real data), mode 1 bytes / 144 doubles. */
int mpbp_hbm_stream(const void* src, int64_t bytes, int32_t mode, double* dst, void* stream);
int mpbp_spmv_seg(const mpbp_csr* A, const mpbp_rowblocks* blocks, int32_t mode, const double* x,
                  const double* z, double* y, void* stream);
/* x_out = b / diag (first Jacobi sweep from 0); x_out = sub - that when sub != NULL. */
int mpbp_jacobi_init(int32_t nrows, const double* b, const double* diag, const double* sub,
                     double* x_out, void* stream);
/* x_out = x_in + (b - A x_in) / diag  (optionally sub - that). */
int mpbp_jacobi_step(const mpbp_csr* A, const mpbp_rowblocks* blocks, const double* x_in,
                     const double* b, const double* diag, const double* sub, double* x_out,
                     void* stream);
/* d = c2 * (b / diag); x_out = d (optionally sub - d). */
int mpbp_cheb_init(int32_t nrows, const double* b, const double* diag, double c2, double* d,
                   const double* sub, double* x_out, void* stream);
/* z = (b - A x_in)/diag; d = c1 d + c2 z; x_out = x_in + d (optionally sub - that). */
int mpbp_cheb_step(const mpbp_csr* A, const mpbp_rowblocks* blocks, const double* x_in,
                   const double* b, const double* diag, double c1, double c2, double* d,
                   const double* sub, double* x_out, void* stream);
/* Chebyshev coefficients used by mpbp_schur_apply for sweep s (0-based): c1[s], c2[s]. Host. */
int mpbp_cheb_coeffs(double lmin, double lmax, int32_t sweeps, double* c1, double* c2);
/* out = M^-1 v with M the block upper-triangular approximate-commutator preconditioner
 * (solve.py:257-277): v, out are device vectors of nu + np owned entries. */
/* Multigrid level 1 of the plan's F (kind MPBP_VEC_VELOCITY) or Gt_G (MPBP_VEC_PRESSURE) hierarchy, y = op(A_1 x) (modes
 * as mpbp_spmv), as the ONE fused matrix-free launch the tolerance-mode multigrid apply runs (k_gal1 / k_gal1p:
 * R_0 (A_0 (P_0 x))).  One GPU, plan f_numerics FAST, kernel option mg_galerkin_mf = 2 (else MPBP_ERR_ARG).  For timing. */
int mpbp_mg_level1_apply(const mpbp_schur_plan* p, int32_t kind, int32_t mode, const double* x, const double* z,
                         double* y, void* stream);
int mpbp_schur_apply(const mpbp_schur_plan* plan, const double* v, double* out, void* stream);

/* ---- SELL-64 (the apply's HBM layout; built once from CSR) --------------------------------- */
/* Host: slices of <= 64 rows over each row range [ranges[2q], ranges[2q+1]) of a HOST row_ptr.
 * Writes at most `capacity` slices; returns the slice count, *pair_rows = storage in pair-rows. */
int64_t mpbp_sell_plan(const int32_t* row_ptr, const int32_t* ranges, int32_t nranges, int32_t* slices,
                       int64_t capacity, int64_t* pair_rows);
/* Copy CSR entries into SELL storage (val / col zero-filled by the caller). */
int mpbp_sell_fill(const mpbp_csr* A, const int32_t* slices, int32_t nslices, uint8_t* row_len,
                   double* val, int32_t* col, void* stream);
/* The CSR apply-path kernels on SELL storage; same arithmetic, same order, same results. */
int mpbp_sell_spmv(const mpbp_sell* S, int32_t mode, const double* x, const double* z, double* y,
                   void* stream);
int mpbp_sell_jacobi_step(const mpbp_sell* S, const double* x_in, const double* b, const double* diag,
                          const double* sub, double* x_out, void* stream);
int mpbp_sell_cheb_step(const mpbp_sell* S, const double* x_in, const double* b, const double* diag,
                        double c1, double c2, double* d, const double* sub, double* x_out, void* stream);

/* ---- matrix-free F (the reference's F, recomputed per row from the thn tables) -------------- */
/* Same results as the assembled-F kernels bit for bit (same formulas, same summation order). */
int mpbp_f_stencil_spmv(const mpbp_stokes_params* prm, const double* cell, const double* uface,
                        const double* vface, const mpbp_row_part* part, int32_t mode, const double* x,
                        const double* z, double* y, void* stream);
int mpbp_f_stencil_jacobi_step(const mpbp_stokes_params* prm, const double* cell, const double* uface,
                               const double* vface, const mpbp_row_part* part, const double* x_in,
                               const double* b, const double* sub, double* x_out, void* stream);
int mpbp_f_stencil_cheb_step(const mpbp_stokes_params* prm, const double* cell, const double* uface,
                             const double* vface, const mpbp_row_part* part, const double* x_in,
                             const double* b, double c1, double c2, double* d, const double* sub,
                             double* x_out, void* stream);

/* ---- matrix-free pressure side: D, G and Gt_G = -(D G) recomputed from the cell thn table ------- */
/* Same results as the assembled D (MPBP_OP_D), G (MPBP_OP_G, d_p from prm) and Gt_G (mpbp_spgemm of D
 * and G, alpha = -1) bit for bit.  part: the INPUT vector's partition (velocity for D, pressure for
 * G and Gt_G); NULL or halo = 0 = one GPU.  solve.py:246 (Gt_G), :259 (D), :273 (G). */
#define MPBP_PG_D 0     /* y = D x    : N pressure rows from the 4 velocity fields */
#define MPBP_PG_G 1     /* y = G x    : 4N velocity rows from pressure */
#define MPBP_PG_GTG 2   /* y = Gt_G x : N pressure rows from pressure */
int mpbp_pg_stencil_spmv(const mpbp_stokes_params* prm, const double* cell, const mpbp_row_part* part, int32_t op,
                         int32_t mode, const double* x, const double* z, double* y, void* stream);
int mpbp_gtg_stencil_jacobi_step(const mpbp_stokes_params* prm, const double* cell, const mpbp_row_part* part,
                                 const double* x_in, const double* b, const double* sub, double* x_out,
                                 void* stream);
int mpbp_gtg_stencil_cheb_step(const mpbp_stokes_params* prm, const double* cell, const mpbp_row_part* part,
                               const double* x_in, const double* b, double c1, double c2, double* d,
                               const double* sub, double* x_out, void* stream);
/* A whole Chebyshev-Jacobi solve of Gt_G x = b from x = 0 (sweeps = 2..6 updates on [lmin, lmax], diag = Gt_G's
 * diagonal) as ONE tiled launch (k_gtg_solve: b read once, the iterates in LDS) -- the apply's fused pressure solve,
 * solve.py:265 / 271; bit-identical to mpbp_gtg_stencil_cheb_step sweeps from x0 = c2 b / diag.  One GPU; the grid must
 * hold a tile and its halos (n >= 72 + 2 (sweeps - 1)), else MPBP_ERR_ARG and nothing is launched. */
int mpbp_gtg_stencil_cheb_solve(const mpbp_stokes_params* prm, const double* cell, const double* b, const double* diag,
                                double lmin, double lmax, int32_t sweeps, double* x_out, void* stream);

/* ---- kernel choices ------------------------------------------------------------------------------ */
/* Which kernel form runs each step.  Every choice gives the same results as every other (bit-identical), except
 * q13_sym (tolerance mode only, within its 1e-12 bar).  A plan (mpbp_schur_plan.opts, mpbp_mg.opts) carries its own
 * copy, so preconditioners with different choices coexist in one process and a captured graph holds the choices its
 * plan had; opts == NULL, and the plan-less entry points (mpbp_spmv, mpbp_f_stencil_*, ...), use the process
 * defaults, which the mpbp_set_* calls below change (mpbp_kernel_opts_default snapshots them for a new plan). */
typedef struct mpbp_kernel_opts {
    int32_t march_rows;        /* grid rows per workgroup of the marching stencil kernels (matrix-free F, D, G, Gt_G);
                                  0 (default): per launch, the count that fills one round of workgroups */
    int32_t init_diag;         /* first F sweep stages x0 = c2 b / diag: 1 (default) rebuilds diag from thn, 0 streams it */
    int32_t f_pair;            /* tolerance mode: an F solve's last two sweeps as one k_march2 launch (1, default) */
    int32_t f_direct;          /* tolerance-mode F sweeps on the direct kernel, one thread per cell (0, default) */
    int32_t gtg_fused;         /* one-GPU Chebyshev Gt_G solves of 2..6 sweeps as ONE k_gtg_solve launch (1, default) */
    int32_t gtg_tpb;           /* k_gtg_solve workgroup lanes: 512 (default) or 256 */
    int32_t gtg_drhs;          /* the first fused Gt_G solve builds rhs = D Finv_v + v_p itself (1, default) */
    int32_t q13_sym;           /* tolerance mode, one GPU: Gt_F_G x from the diamond's upper half (1, default; cleared
                                  per plan when mpbp_q13_asymmetry finds the product not symmetric) */
    int32_t f_tile;            /* one-GPU tolerance-mode F: x0 + sweep 1 and the last pair on 2D tiles (1, default) */
    int32_t f_solve;           /* one-GPU tolerance-mode F solves of 3 or 4 updates as ONE k_fsolve launch (1, default) */
    int32_t mg_galerkin_mf;    /* tolerance-mode F hierarchies: level 1 as R_0 (F (P_0 x)): 2 (default) one k_gal1 launch,
                                  1 three launches, 0 its stored Galerkin matrix */
    int32_t mg_galerkin_mf_p;  /* the pressure hierarchy's level 1 as R_0 (Gt_G (P_0 x)) (1, default) */
    int32_t pg_direct;         /* matrix-free D, G, Gt_G sweeps one thread per cell (1, default) or marching (0) */
    int32_t mg_group_rows;     /* multigrid levels / transfers with <= this many rows on the grouped CSR kernel (65536) */
    int32_t mg_svl;            /* multigrid levels with a stencil-values copy use it (1, default) */
    int32_t mg_mf_transfer;    /* whole-grid multigrid transfers matrix-free when the kinds are known (1, default) */
    int32_t csr_table;         /* CSR SpMV waves start from the row blocks' wave table when present (1, default) */
    int32_t mg_fuse_l0;        /* tolerance-mode F hierarchies, one GPU: level 0's pre-smoothing, residual and restriction
                                  as ONE k_fpre launch, and the prolongation inside the post-smoothing pair; the matrix-free
                                  level 1's prolongation inside its first post-smoothing sweep (k_gal1 / k_gal1p <PRO>) (1, default) */
    int32_t mg_coarse_tree;    /* tolerance-mode hierarchies: the coarsest level's dense inverse applied with its row sums
                                  split over the workgroup and combined by a tree (1; default 0: another order of the
                                  ill-conditioned coarsest F inverse's sums moves the apply by ~5e-13) */
    int32_t f_solve_tile;      /* tolerance-mode whole F solves (k_fsolve): 0 the 64 x 8 tile, halo rings owned by the
                                  first lanes; 1 (default) a 32 x 16 tile, each ring dealt out evenly over the four waves, the
                                  rows' level-invariant terms computed once (k_fsolve_w).  Both compute the same bits */
    int32_t q13_mf;            /* tolerance mode, one GPU, matrix-free F / D / G: x_b = Gt_F_G x_a applied as its factors
                                  -(D (F (G x_a))) on 32 x 16 tiles (k_qmf; 42 instead of 76 MB per apply at 1024^2),
                                  not the stored product (1); 0: the stored product (k_q13) */
    int32_t mg_fuse_small;     /* whole-grid multigrid levels l >= 1 on k_csr_grp rows (<= mg_group_rows) with matrix-free
                                  transfers and a coarse level of <= 1024 rows: residual + restriction as ONE launch
                                  (k_grp_rr; 1, default; the same bits as 0) */
    int32_t gtg_solve_tile;    /* fused Gt_G solves (k_gtg_solve): 1 (default) 32 x 16 tiles, 0 the 64 x 8 tile; the same bits */
    int32_t reserved[1];
} mpbp_kernel_opts;
/* *out = the calling thread's current choices: its mpbp_kernel_opts_set_thread scope, else the process defaults. */
void mpbp_kernel_opts_default(mpbp_kernel_opts* out);
/* Kernel choices for the plan-less entry points called from THIS thread (a plan's own opts still win inside its apply);
 * NULL returns the thread to the process defaults.  *prev (optional) receives the previous thread choice, to restore
 * it.  The struct must stay valid while installed. */
int mpbp_kernel_opts_set_thread(const mpbp_kernel_opts* o, const mpbp_kernel_opts** prev);
/* Process defaults (see mpbp_kernel_opts for each field's meaning; results are bit-identical for every value, q13_sym
 * aside).  Plans built before a call keep their own copies. */
int mpbp_set_march_rows(int32_t rows);
int mpbp_set_init_diag(int32_t mode);
int mpbp_set_f_pair(int32_t on);
int mpbp_set_f_direct(int32_t on);
int mpbp_set_gtg_drhs(int32_t on);
int mpbp_set_q13_sym(int32_t on);
int mpbp_set_gtg_fused(int32_t on);   /* also 256 / 512: on, with that many lanes per workgroup */
int mpbp_set_f_tile(int32_t on);
int mpbp_set_f_solve(int32_t on);
int mpbp_set_mg_galerkin_mf(int32_t on);
int mpbp_set_mg_galerkin_mf_p(int32_t on);
int mpbp_set_pg_direct(int32_t on);
int mpbp_set_mg_group_rows(int32_t rows);
int mpbp_set_mg_svl(int32_t on);
int mpbp_set_mg_mf_transfer(int32_t on);
int mpbp_set_csr_table(int32_t on);

/* ---- geometric multigrid inner solves (the reference's pointer: solve.py:266, 274) ------------------ */
/* P (which = MPBP_MG_P, fine x coarse) or R = P^T (MPBP_MG_R) of an n x n periodic grid (n even, >= 4) coarsened by 2,
 * for nfields stacked fields; kinds (host) = {ky, kx} per field (MPBP_MG_CELL / MPBP_MG_NODE along rows / columns).
 * Columns sorted, values exact dyadic rationals.  count writes row_nnz (device); fill needs row_ptr.  Setup. */
int mpbp_mg_transfer_count(int32_t n, int32_t nfields, const int32_t* kinds, int32_t which, int32_t* row_nnz,
                           void* stream);
int mpbp_mg_transfer_fill(int32_t n, int32_t nfields, const int32_t* kinds, int32_t which, const int32_t* row_ptr,
                          int32_t* col_idx, double* val, void* stream);
/* The same transfer's rows `rows` (device, global row ids; any order) only, output row i = row rows[i], global columns:
 * a rank's band of a row-partitioned hierarchy without the whole-grid transfer.  Setup. */
int mpbp_mg_transfer_rows_count(int32_t n, int32_t nfields, const int32_t* kinds, int32_t which, const int32_t* rows,
                                int32_t nrows, int32_t* row_nnz, void* stream);
int mpbp_mg_transfer_rows_fill(int32_t n, int32_t nfields, const int32_t* kinds, int32_t which, const int32_t* rows,
                               int32_t nrows, const int32_t* row_ptr, int32_t* col_idx, double* val, void* stream);
/* x_out = mg->cycles V-cycles for levels[0].A x = b from x = 0 (sub - x when sub != NULL).  Graph-capturable.
 * Row-partitioned hierarchies (part_levels > 0): b, sub, x_out hold the rank's owned rows of level 0. */
int mpbp_mg_solve(const mpbp_mg* mg, const double* b, const double* sub, double* x_out, void* stream);

/* ---- ghost rows over RCCL point-to-point (multi-GPU row partition) ------------------------------ */
/* One RCCL group of neighbour sends / receives: the owned boundary rows (packed into one buffer per
 * direction when a vector has several fields) straight into the ghost rows of the ext layout
 * (csrc/halo.cpp).  RCCL is dlopen'ed from rccl_path (NULL: "librccl.so").
 * Setup: mpbp_rccl_unique_id on one rank (128 bytes), shared by the caller, then mpbp_halo_create on
 * every rank (collective).  mpbp_halo_exchange is an mpbp_halo_fn: plan.halo = mpbp_halo_exchange,
 * plan.halo_ctx = the handle; it cannot return an error, so callers check mpbp_halo_status after an
 * apply.  world = 1 exchanges with itself (the periodic wrap) -- the single-GPU test of this path. */
typedef struct mpbp_halo mpbp_halo;
int mpbp_rccl_unique_id(const char* rccl_path, uint8_t* id_out);
int mpbp_halo_create(const char* rccl_path, const uint8_t* id, int32_t world, int32_t rank, int32_t n,
                     int32_t r0, int32_t rows, int32_t h_u, int32_t h_p, mpbp_halo** out);
/* Another halo object (its own kinds 0 / 1 for the given layout, buffers and stream) on base's communicator: one RCCL
 * communicator per process group, reference-counted (released with its last object, unless captured -- see
 * mpbp_halo_destroy).  Local: no collective.  Replaces a second mpbp_halo_create on the same group. */
int mpbp_halo_create_shared(const mpbp_halo* base, int32_t n, int32_t r0, int32_t rows, int32_t h_u, int32_t h_p,
                            mpbp_halo** out);
/* The object's communicator (an opaque identity, for checks) and how many halo objects hold it. */
const void* mpbp_halo_comm(const mpbp_halo* halo);
int mpbp_halo_comm_refs(const mpbp_halo* halo);
void mpbp_halo_destroy(mpbp_halo* halo);
void mpbp_halo_exchange(void* halo, int32_t vec_kind, double* x_ext, int32_t phase, void* stream);
int mpbp_halo_status(const mpbp_halo* halo);
#define MPBP_HALO_IN_ORDER 0   /* group issued on the apply stream between interior and boundary (default) */
#define MPBP_HALO_OVERLAP 1    /* group on a side stream, forked / joined by events around the interior */
/* mpbp_halo_pair_fn over RCCL: one group with both vectors' neighbour sends / receives (IN_ORDER on
 * `stream`; the velocity rows gathered first). */
void mpbp_halo_exchange_pair(void* ctx, double* xu_ext, double* xp_ext, void* stream);
/* Mode of every kind defined so far (kinds added later take their own mode). */
int mpbp_halo_set_mode(mpbp_halo* halo, int32_t mode);
const char* mpbp_halo_last_error(const mpbp_halo* halo);
/* Another vector layout on the same communicator: nfields fields of an n x n grid, owned rows [r0, r0 + rows),
 * h ghost rows each side; returns its kind id for mpbp_halo_exchange (kinds 0 / 1 are the Schur apply's velocity /
 * pressure vectors).  Used for the system vector of the partitioned operator A (apply.py:72, the FGMRES A @ x)
 * and for the multigrid levels.  Setup. */
int mpbp_halo_add_kind(mpbp_halo* halo, int32_t nfields, int32_t n, int32_t r0, int32_t rows, int32_t h, int32_t mode);
/* An all-gather layout: rank k owns rows [r0s[k], r0s[k] + rows_s[k]) of each of nfields fields of an n x n grid
 * (host arrays of world entries, covering the grid); returns its id for mpbp_halo_allgather.  Setup. */
int mpbp_halo_add_gather(mpbp_halo* halo, int32_t nfields, int32_t n, const int32_t* r0s, const int32_t* rows_s);
/* mpbp_gather_fn over RCCL: pad the owned rows, one ncclAllGather, one gather kernel into x_full (on `stream`). */
void mpbp_halo_allgather(void* ctx, int32_t gather_kind, const double* x_owned, double* x_full, void* stream);

/* gather: dst[i] = src[idx[i]] ; scatter: dst[idx[i]] = src[i]   (halo pack / unpack) */
int mpbp_gather(int32_t count, const int32_t* idx, const double* src, double* dst, void* stream);
int mpbp_scatter(int32_t count, const int32_t* idx, const double* src, double* dst, void* stream);

/* hipEvent helpers for callers without a HIP binding (bench profiling). */
int mpbp_event_create(void** ev);
/* device_scope = 1: the event's release is device scope (hipEventReleaseToDevice) -- recording it does not write
 * the L2 back to memory, so a kernel timed between two such events runs as it does inside the captured apply (a
 * system-scope release after every sweep drains the dirty L2 the next sweep would have read); 0: hipEventDefault. */
int mpbp_event_create_scoped(void** ev, int32_t device_scope);
/* hipEventRecord on `stream` (NULL: the default stream); skipped while the stream is capturing. */
int mpbp_event_record(void* ev, void* stream);
int mpbp_event_destroy(void* ev);
int mpbp_event_elapsed_ms(void* start, void* stop, float* ms);

/* ---- FGMRES orthogonalisation (the outer Krylov loop of solve.py:285, pyamg.krylov.fgmres) ---------------- */
/* h[0:k] = V w with V the k Krylov basis vectors of n doubles at row stride ld (device; 1 <= k <= 256).
 * part: device scratch of mpbp_gs_part_size(n, k) doubles.  Deterministic (fixed reduction order). */
int mpbp_gs_dot(const double* V, int64_t ld, int32_t k, const double* w, int64_t n, double* part, double* h,
                void* stream);
int64_t mpbp_gs_part_size(int64_t n, int32_t k);
/* w_out = w - V^T h (w_out may alias w: element-wise, each element read before it is written). */
int mpbp_gs_update(const double* V, int64_t ld, int32_t k, const double* h, const double* w, int64_t n, double* w_out,
                   void* stream);
/* Reproducible dot products (binned summation, 3 folds; the FGMRES of a row partition computes the same bits as on
 * one GPU): acc[3i .. 3i+2] = the exact fold sums of V[i] . w over this rank's n entries (i < k).  bound_v (device,
 * k) and bound_w (device, 1) bound |V[i][e]| and |w[e]| over EVERY rank's entries (a max-reduction of local
 * maxima, mpbp_absmax); n_total is the length of the whole distributed vector.  The fold sums of different ranks
 * add exactly (a sum-reduction in any order), and mpbp_rdot_finish gives h[i] = (S0 + S1) + S2 -- the same bits
 * for every row partition, chunking and launch order.  Error <= about 2^-51 of bound_v[i] bound_w.  part: device
 * scratch of mpbp_rdot_part_size(n, k) doubles. */
int mpbp_rdot(const double* V, int64_t ld, int32_t k, const double* w, int64_t n, int64_t n_total,
              const double* bound_v, const double* bound_w, double* part, double* acc, void* stream);
int64_t mpbp_rdot_part_size(int64_t n, int32_t k);
/* CGS2's first update and second projection in one pass over V (FGMRES, solve.py): w_out = w - V^T h (mpbp_gs_update's
 * bits; w_out may be w) and acc[3i + f] = the exact fold sums of V[i] . w_out (mpbp_rdot's, finished by
 * mpbp_rdot_finish), with the fold extractors from the a-priori bound (bound_w[0] + sum_i bound_v[i] |h[i]|)(1 + 2^-40)
 * on |w_out| (bound_w[0] = max |w| over all ranks) -- identical on every rank, so the sums stay reproducible.
 * 1 <= k <= 256; part: mpbp_rdot_part_size(n, k) doubles.  Replaces the reference's pyamg fgmres orthogonalisation
 * step (solve.py:285; pyamg is absent, see oracle/krylov_oracle.py). */
/* DCGS2 (FGMRES with delayed re-orthogonalisation, two basis passes per iteration).  mpbp_rdot2: the exact fold sums of
 * V[i] . u (acc[3i .. 3i+2]) and V[i] . w (acc[3k + 3i ..]) for i < k in ONE pass over V (k <= 256; part:
 * mpbp_rdot_part_size(n, 2k) doubles); bounds as mpbp_rdot (bound_u, bound_w: max |u|, max |w| bounds).
 * mpbp_dcgs2_update, iteration j (V[0..j-1] orthonormal, V[j] = u_j projected once, acc = mpbp_rdot2 of V[0..j] with
 * u = V[j] and w): hu[0..j], hw[0..j] the finished products, P = {r, 1/r, c, bound}: r = sqrt(hu[j] - s.s) (j = 0: 1),
 * c = (hw[j] - s.z) / r; then V[j] <- (V[j] - V[0..j-1]^T s) / r and, upd_w != 0, V[j+1] <- (w - V[0..j-1]^T z) - V[j] c
 * (s = hu[0..j-1], z = hw[0..j-1]); P[3] = (bound_w + sum |z_i| + |c|)(1 + 2^-40) bounds |V[j+1]|.  r = 0 marks a
 * breakdown (V[j] then 0).  All scalars in a fixed order on the device: rank-independent given reduced fold sums. */
int mpbp_rdot2(const double* V, int64_t ld, int32_t k, const double* u, const double* w, int64_t n, int64_t n_total,
               const double* bound_v, const double* bound_u, const double* bound_w, double* part, double* acc,
               void* stream);
int mpbp_dcgs2_update(double* V, int64_t ld, int32_t j, const double* acc, const double* bound_w, const double* w,
                      int64_t n, int32_t upd_w, double* hu, double* hw, double* P, void* stream);
int mpbp_gs_update_rdot(const double* V, int64_t ld, int32_t k, const double* h, const double* w, int64_t n,
                        int64_t n_total, const double* bound_v, const double* bound_w, double* w_out, double* part,
                        double* acc, void* stream);
int mpbp_rdot_finish(int32_t k, const double* acc, double* h, void* stream);
/* amax[0] = max_e |x[e]| (device scalar, overwritten; NaN if x holds one). */
int mpbp_absmax(const double* x, int64_t n, double* amax, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MPBP_H */
