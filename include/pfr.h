/*
 * pfr.h -- C ABI of the MI355X plate frequency-response solver (libpfr.so).
 *
 * Drop-in boundary for the reference's native solver path:
 *   pybind11 class InnerState (source/jax_plate_lib/src/main.cpp:6-19) bound by
 *   SolverState (source/jax_plate/Sparse.py:19-44) and called through the JAX
 *   primitives' CPU lowering (Sparse.py:150-160, 187-197).
 *
 * Plain C: opaque handles, integer status codes (no exceptions cross the ABI),
 * plain pointers and sizes.  Complex numbers are interleaved (re, im) doubles
 * (numpy complex128 / torch.complex128 memory layout).  Every *_dev pointer is
 * a device (HBM) pointer; `stream` is a hipStream_t (NULL = default stream).
 * Host pointers are only read during the call.
 */
#ifndef PFR_H
#define PFR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PFR_API __attribute__((visibility("default")))

/* status codes */
#define PFR_OK 0
#define PFR_ERR_ARG 1        /* invalid argument (cf. Sparse.py:120-140 checks) */
#define PFR_ERR_SYMBOLIC 2   /* symbolic analysis failed (cf. umfpack_interface.h:10-18) */
#define PFR_ERR_HIP 3        /* HIP runtime error */
#define PFR_ERR_NOMEM 4      /* device allocation failed */
#define PFR_ERR_STATE 5      /* call out of order (e.g. operator not set) */

/* per-frequency status flags (bitwise OR into an int32 array) */
#define PFR_FLAG_BAD_PIVOT 1 /* zero / non-finite static pivot */
#define PFR_FLAG_BACKWARD_ERROR 2     /* forward solution: componentwise backward error above the tolerance */
#define PFR_FLAG_BACKWARD_ERROR_ADJ 4 /* adjoint solution: componentwise backward error above the tolerance */

/* pfr_set_check modes (bitwise OR) */
#define PFR_CHECK_FORWARD 1   /* backward error of the forward solution (A x = b) */
#define PFR_CHECK_ADJOINT 2   /* backward error of the adjoint solution (A^T l = g; loss sweeps, transposed solves) */
#define PFR_CHECK_REFINE 4    /* one step of iterative refinement of the forward (and, in loss sweeps, the
                               * adjoint) solution on the same factors, x += A^{-1} (b - A x), before the
                               * checks (UMFPACK refines by default, up to 2 steps) */
#define PFR_CHECK_CORRECT 8   /* functional correction (pfr_sweep): fr += Re(mu^T (b - A x)) with mu the adjoint
                               * of fr (A^T mu = d fr / d x) -- fr to second order in the solve's error, the
                               * accuracy the reference's refined UMFPACK solves give; the loss, its
                               * cotangent and the gradient are formed from the corrected fr; in loss sweeps
                               * the cotangent also carries the solve-error scale fr / (mu^T A x) (complex; the
                               * static-pivot solves' error next to a resonance is a complex multiple of the
                               * solution itself, which this divides out of the gradient contraction; env
                               * PFR_SCALE_CORR=0 turns it off) */

#define PFR_CHECK_REFINE_ADJ 16 /* selective adjoint refinement (loss sweeps with PFR_CHECK_CORRECT, symmetric
                               * mode): after the forward residual walk, the 64-frequency groups holding a frequency
                               * whose functional correction exceeds the tolerance (pfr_set_refine_tol; the
                               * first-order fr error estimate, large next to a resonance) get one refinement step
                               * of the fr adjoint, mu += A^-T (d fr / d x - A^T mu), and their gradient contraction
                               * and correction are redone with it (opt-in: with the solve-error scale of
                               * PFR_CHECK_CORRECT the gradient is already within the oracle's accuracy) */

/* loss types (Problem.py:948-975) */
#define PFR_LOSS_NONE -1
#define PFR_LOSS_MSE 0
#define PFR_LOSS_RMSE 1
#define PFR_LOSS_MSE_AFC 2
#define PFR_LOSS_MSE_LOG_AFC 3
#define PFR_LOSS_COTANGENT 4  /* ref holds dL/dfr (real part), loss not computed */

typedef struct pfr_symbolic pfr_symbolic;
typedef struct pfr_solver pfr_solver;

typedef struct pfr_symbolic_options {
  int32_t leaf_size;   /* nested-dissection leaf size (default 10000): parts at or below it are
                        * ordered by multiple minimum degree */
  int32_t ordering;    /* 0 nested dissection + multiple-minimum-degree leaves (default), 1 natural,
                        * 2 nested dissection + exact minimum-degree leaves (the round 1-3 ordering) */
  int32_t relax_small, relax_mid, relax_big; /* supernode amalgamation (4, 8, 24) */
  double zrelax_mid, zrelax_big;             /* (0.5, 0.1) */
  /* 1: symmetric-structure analysis (default 0).  The caller guarantees that the matrices
   * factorised with it are complex symmetric (A = A^T, non-conjugate) once the Dirichlet
   * rows -- rows holding only their diagonal entry (tgv = -1 rows, pyFFInterface.py:176) --
   * and their columns are removed.  Those nodes are decoupled (their column entries move
   * to the right-hand side / the adjoint's Dirichlet rows), the rest is factorised as
   * A = L U with U = diag(U) L^T implicit: only L is formed and read. */
  int32_t symmetric;
  /* Nodes to be eliminated last, together (default none): ordered after every other node, they
   * form the root front.  The engine passes the loss functional's support, so that the adjoint's
   * bottom-up solve stays inside the root and both top-down solves run as one pass. */
  int32_t n_last;
  const int32_t* last;
  int32_t max_ns;      /* fundamental supernodes split into pieces of at most max_ns pivots (default 256;
                        * 0 = no split) */
  int32_t md_delta;    /* multiple minimum degree: each stage eliminates an independent set of the
                        * nodes of external degree <= minimum + md_delta (default 4) */
} pfr_symbolic_options;

typedef struct pfr_symbolic_stats {
  int32_t n;
  int64_t nnz;
  int32_t n_fronts;
  int32_t n_levels;
  int32_t max_front;
  int64_t total_rows;      /* sum of front sizes */
  int64_t factor_entries;  /* sum of squared front sizes (dense front storage per frequency) */
  int64_t nnz_lu;          /* entries of L + U (per frequency) */
  double factor_flops;     /* real flops of one numeric factorisation */
  int32_t symmetric;       /* analysis built with options.symmetric = 1 */
  int32_t n_dirichlet;     /* symmetric mode: decoupled Dirichlet nodes */
  int64_t n_coupling;      /* symmetric mode: entries (i, d), i not Dirichlet, d Dirichlet */
} pfr_symbolic_stats;

/* export ids for pfr_symbolic_export (int32 arrays unless noted) */
#define PFR_EXPORT_PERM 0        /* n: new -> old */
#define PFR_EXPORT_IPERM 1       /* n: old -> new */
#define PFR_EXPORT_FRONTS 2      /* n_fronts x 8 int64: ns, f, row0, col0, parent, level, off, wv */
#define PFR_EXPORT_IDX 3         /* total_rows */
#define PFR_EXPORT_RELPOS 4      /* total_rows */
#define PFR_EXPORT_ASM_PTR 5     /* total_rows + 1 */
#define PFR_EXPORT_ASM_COL 6     /* nnz */
#define PFR_EXPORT_ASM_NZ 7      /* nnz */
#define PFR_EXPORT_EA_PTR 8      /* total_rows + 1 */
#define PFR_EXPORT_EA_SRC 9      /* ea_ptr[total_rows] */
#define PFR_EXPORT_LEVEL_PTR 10  /* n_levels + 1 */
#define PFR_EXPORT_LEVEL_FRONTS 11 /* n_fronts */
#define PFR_EXPORT_DIRICHLET 12  /* n_dirichlet x 2: permuted node, CSC index of its diagonal entry */
#define PFR_EXPORT_COUPLING 13   /* n_coupling x 3: permuted row i, Dirichlet slot, CSC index; by row */

PFR_API const char* pfr_version(void);
/* Message of the last failed call on this thread ("" if none). */
PFR_API const char* pfr_last_error(void);
PFR_API void pfr_symbolic_options_default(pfr_symbolic_options* opt);

/* ---------------------------------------------------------------- symbolic (host only, no GPU)
 * Replaces InnerState::add_mat -> umfpack_zi_symbolic (InnerState.h:120-162) and
 * create_symbolic (Sparse.py:92-116).  Pattern = n x n CSC (colptr n+1, rowind nnz),
 * the union pattern of Problem.py:317-332.  opt may be NULL (defaults). */
PFR_API int pfr_symbolic_create(int32_t n, int64_t nnz, const int32_t* colptr, const int32_t* rowind,
                                const pfr_symbolic_options* opt, pfr_symbolic** out);
PFR_API int pfr_symbolic_stats_get(const pfr_symbolic* sym, pfr_symbolic_stats* out);
PFR_API int pfr_symbolic_export(const pfr_symbolic* sym, int32_t what, void* dst, int64_t capacity_bytes);
PFR_API void pfr_symbolic_destroy(pfr_symbolic* sym);

/* ---------------------------------------------------------------- device solver
 * Uploads the symbolic maps and allocates frequency-minor workspaces for up to
 * max_batch frequencies per chunk.  Keeps a copy of colptr/rowind for matvec. */
PFR_API int pfr_solver_create(const pfr_symbolic* sym, const int32_t* colptr, const int32_t* rowind,
                              int32_t device, int32_t max_batch, pfr_solver** out);
PFR_API void pfr_solver_destroy(pfr_solver* s);
/* device bytes pfr_solver_create would allocate for max_batch */
PFR_API int64_t pfr_solver_workspace_bytes(const pfr_symbolic* sym, int32_t max_batch);
PFR_API int32_t pfr_solver_max_batch(const pfr_solver* s);

/* ---------------------------------------------------------------- InnerState-compatible entry points
 * pfr_solve: x[q] = A_q^{-1} b[q]  (transpose != 0: A_q^{-T} b[q], NON-conjugate, = UMFPACK_Aat,
 * InnerState.h:183-185).  A_q values on the CSC pattern: data_dev + q * data_stride (complex, nnz);
 * data_stride = 0 broadcasts one matrix (modes 0/2 of InnerState::solve, InnerState.h:192-233);
 * b_stride likewise (0 = broadcast b, mode 1).  Batch-major (batch, n) complex output.
 * Replaces InnerState::solve (InnerState.h:164-308).  flags_dev: int32 per batch item (may be NULL).
 * Needs a solver on a general analysis (options.symmetric = 0): explicit matrices carry no symmetry
 * guarantee (PFR_ERR_STATE otherwise). */
PFR_API int pfr_solve(pfr_solver* s, int32_t batch, const double* data_dev, int64_t data_stride,
                      const double* b_dev, int64_t b_stride, double* x_dev, int32_t transpose,
                      int32_t* flags_dev, void* stream);

/* Several right-hand sides per matrix on the same factors: the reference's batching mode 4
 * (data (B, nnz), b (J, B, N), Sparse.py:245-282, used by jax.hessian), which refactorises for every
 * right-hand side (InnerState.h:289-305).  b of rhs r, item q at b_dev + 2 * (r * b_rhs_stride +
 * q * b_stride) doubles (b_stride 0 = broadcast); x of rhs r at x_dev + 2 * r * x_rhs_stride
 * (items contiguous, stride n; x_rhs_stride >= batch * n when nrhs > 1). */
PFR_API int pfr_solve_multi(pfr_solver* s, int32_t batch, int32_t nrhs, const double* data_dev,
                            int64_t data_stride, const double* b_dev, int64_t b_stride, int64_t b_rhs_stride,
                            double* x_dev, int64_t x_rhs_stride, int32_t transpose, int32_t* flags_dev,
                            void* stream);
/* pfr_matvec: y[q] = A_q x[q] (or A_q^T x[q]); replaces InnerState::matvec (InnerState.h:310-470). */
PFR_API int pfr_matvec(pfr_solver* s, int32_t batch, const double* data_dev, int64_t data_stride,
                       const double* x_dev, int64_t x_stride, double* y_dev, int32_t transpose, void* stream);

/* ---------------------------------------------------------------- fused operator-form sweep
 * The hot path of Problem.getFRFunction / getLossFunction (Problem.py:432-477, 948-975) fused
 * with the reverse pass JAX derives from Sparse.py:162-222:
 *   A(omega) = K - omega^2 M,  b(omega) = rhs * (beta - omega^2 mass_sum),
 *   fr = sqrt(ts^2|aU.x|^2 + ts^2|aV.x|^2 + |aW.x|^2),
 *   loss = scale * sum_q term(fr_q, ref_q),
 *   w_k = sum_q ( -lam_q^T S_k x_q + e_k lam_q^T rhs ),   A^T lam_q = d loss / d x_q.
 * The (F, nnz) matrix batch is never materialised. */

/* K_out_dev = sum_k coef_k * S_k  (S registered by pfr_set_stiffness), complex nnz.  n_stiff is 18
 * (A, B, D coefficient matrices of Problem.py:440-445) or 12 (A and D only: the B coefficients vanish
 * for mid-plane symmetric laminates, so their matrices and gradient partials are left out).
 * pfr_set_stiffness registers stiff_dev: pfr_combine, the Hessian sweep and the gradient contraction of
 * every loss sweep (fused into the forward residual walk by default) read it at every call, so the
 * buffer must stay alive and unchanged while the solver uses it (an entry-ordered copy is also taken
 * for the k_contract_eg path; after changing the values, call pfr_set_stiffness again). */
PFR_API int pfr_set_stiffness(pfr_solver* s, int32_t n_stiff, const double* stiff_dev /* (nnz, n_stiff) */,
                              const double* rhs_weights /* host, n_stiff: e_k */);
PFR_API int pfr_combine(pfr_solver* s, const double* coef /* host complex n_stiff */, double* K_out_dev,
                        void* stream);
PFR_API int pfr_set_operator(pfr_solver* s, const double* K_dev /* complex nnz */, const double* M_dev /* real nnz */);
PFR_API int pfr_set_rhs(pfr_solver* s, const double* rhs_host /* real n, caller numbering */, double beta_re,
                        double beta_im, double mass_sum);
PFR_API int pfr_set_functional(pfr_solver* s, int32_t n_support, const int32_t* index_host /* caller numbering */,
                               const double* a_host /* 3 x n_support: aU, aV, aW */, double ts);
/* nfreq frequencies [Hz] (device).  loss_type PFR_LOSS_NONE: forward only (fr_dev).  Otherwise ref_dev
 * (complex nfreq) and the reverse pass: loss_dev[0] += sum of terms * scale ... (raw sum, unscaled),
 * w_dev (complex n_stiff) += gradient partials.  fr_dev / loss_dev / w_dev / flags_dev may be NULL. */
PFR_API int pfr_sweep(pfr_solver* s, int32_t nfreq, const double* freqs_dev, int32_t loss_type,
                      const double* ref_dev, double scale, double* fr_dev, double* loss_dev, double* w_dev,
                      int32_t* flags_dev, void* stream);
/* pfr_sweep with fresh outputs: loss_dev[0], w_dev (n_stiff complex) and flags_dev[0 .. nfreq) zeroed and the
 * pfr_set_check backward-error buffer set to NaN by the sweep's first kernel, then filled as pfr_sweep accumulates
 * them -- the loss step's initialisation without separate fills before the sweep (Problem._Engine.loss_step). */
PFR_API int pfr_sweep_fresh(pfr_solver* s, int32_t nfreq, const double* freqs_dev, int32_t loss_type,
                            const double* ref_dev, double scale, double* fr_dev, double* loss_dev, double* w_dev,
                            int32_t* flags_dev, void* stream);
/* Sweeps of this solver replayed from its captured hipGraph so far.  A pfr_sweep called again with the same
 * arguments, stream and solver state (no setter called in between; pfr_set_check's mode, tolerance and berr
 * pointer are part of the arguments) is captured into a hipGraph on that second call and replayed with one
 * hipGraphLaunch afterwards -- the same kernels with the same arguments; only with PFR_GRAPH=1 (off by default).  The
 * reference's analogue is none: its sweep is a host loop of UMFPACK calls (InnerState.h:276-288). */
PFR_API int64_t pfr_sweep_graph_launches(const pfr_solver* s);
/* Stream ordering for a host that drives several solver lanes: work enqueued on `waiter` after this call starts
 * only after the work enqueued on `signaller` before it (one event of the calling thread and device, recorded on
 * signaller, waited for on waiter; both HIP stream handles of the current device).  The loss step orders each lane's
 * stream after the caller's and the caller's after every lane with it (Problem._Engine._run) -- one C call where
 * torch's Stream.wait_stream makes and destroys an event.  No reference analogue (its sweep is a host loop,
 * InnerState.h:276-288). */
PFR_API int pfr_stream_order(void* waiter, void* signaller);

/* Exact second derivatives with the factors of the sweep reused (replaces the reference's
 * forward-over-reverse Hessian, `jax.jacobian(grad)` in Optimizers.py:125-136, whose mode-4
 * batched solves refactorise per direction, InnerState.h:289-305).  Per frequency: one
 * factorisation, then x, the adjoint l, and per tangent direction i (n_dir of them, complex
 * coefficient directions dcoef[i] = d c / d theta_i, host memory, n_dir x n_stiff complex):
 *   A dx_i = db_i - dA_i x,   A^T dl_i = dG_i(dx_i) - dA_i^T l     (dA_i = sum_k dcoef_ik S_k)
 * Accumulates loss_dev[0] (may be NULL) and w_dev (n_stiff complex) as pfr_sweep, and
 *   h_dev[i * n_stiff + k] += sum_f [ -dl_i^T S_k x + e_k dl_i^T b0 - l^T S_k dx_i ]
 * so that d2L / dtheta_i dtheta_j = Re sum_k ( h_ik dc_kj + w_k d2c_k / dtheta_i dtheta_j ).
 * loss_type must be one of MSE, RMSE, MSE_AFC, MSE_LOG_AFC. */
PFR_API int pfr_hessian_sweep(pfr_solver* s, int32_t nfreq, const double* freqs_dev, int32_t loss_type,
                              const double* ref_dev, double scale, int32_t n_dir, const double* dcoef,
                              double* loss_dev, double* w_dev, double* h_dev, int32_t* flags_dev, void* stream);

/* Backward-error checks of the solves and the accuracy options (the failure detection a static pivot
 * order needs; the reference turns UMFPACK's status into an exception, umfpack_interface.h:10-18, and
 * its solves refine by default).  After each solve the componentwise (Oettli-Prager) backward error
 *   berr = max_i |b - A x|_i / (|A| |x| + |b|)_i        (|z| = |re| + |im|)
 * of the ORIGINAL system is computed on the device per frequency / batch item -- UMFPACK's sparse
 * backward error, invariant under row / column scaling -- and the item's flag
 * PFR_FLAG_BACKWARD_ERROR (forward) / PFR_FLAG_BACKWARD_ERROR_ADJ (adjoint) is set when berr > tol
 * (or not finite).  mode: PFR_CHECK_* bits (0 = off, the default).  berr_dev (device, may be NULL):
 * every later pfr_sweep / pfr_solve call writes berr_dev[2 q] (forward) and berr_dev[2 q + 1]
 * (adjoint) for its items q = 0 .. nfreq - 1 (slots of a solve that is not checked are left
 * alone), so it must hold 2 nfreq doubles of every such call.  With PFR_CHECK_REFINE a loss sweep
 * runs its forward solve, refinement and adjoint in sequence (not the paired top-down pass).
 * PFR_CHECK_CORRECT: every pfr_sweep (forward-only sweeps too) also solves for the adjoint of fr --
 * in symmetric mode inside the paired top-down pass -- and the forward residual walk (the forward
 * check) accumulates the correction; in a loss sweep that adjoint is the loss adjoint up to one
 * scalar per frequency, so the correction costs only the residual walk.  pfr_hessian_sweep applies
 * the correction to its loss and gradient (they equal pfr_sweep's), not the checks; its second-order
 * seeds (the directional derivatives of the loss cotangent) are formed from the uncorrected fr, so its
 * Hessian is that of the uncorrected functional (the two differ by the solve's first-order error). */
PFR_API int pfr_set_check(pfr_solver* s, int32_t mode, double tol, double* berr_dev);
/* PFR_CHECK_REFINE_ADJ threshold: refine the groups where |Re(mu^T r)| > tol |fr| (default 2e-8) */
PFR_API int pfr_set_refine_tol(pfr_solver* s, double tol);

/* Diagnostic: the last chunk's solution vectors of pfr_sweep for chunk lane q (which 0: the forward solution x,
 * 1: the adjoint (mu, the adjoint of fr, under PFR_CHECK_CORRECT; lambda otherwise)), caller numbering, n complex
 * into out_host.  Synchronises the device. */
PFR_API int pfr_debug_solution(pfr_solver* s, int32_t which, int32_t q, double* out_host);

/* Per-phase device times [ms] of the last pfr_sweep/pfr_solve call on this solver, measured with HIP
 * events on the call's stream (0 = factor, 1 = forward solves, 2 = functional, 3 = adjoint solves,
 * 4 = contraction).  Timing is enabled by pfr_set_timing(s, 1). */
PFR_API int pfr_set_timing(pfr_solver* s, int32_t enable);
PFR_API int pfr_last_timings(const pfr_solver* s, double* ms_out /* 5 */);

/* With pfr_set_timing(s, 3) the factorisation additionally brackets every launch with HIP events:
 * summed device times [ms] of the last call per kernel class (0 = A11 assembly, 1 = A11 LU,
 * 2 = L21/U12 rows/columns, 3 = Schur complement A22 of the large update blocks (16 x 16 LDS
 * blocks, symmetric mode), 4 = Schur complement A22 of the other fronts (4 x 4 tiles)) and their launch
 * counts (NULL allowed). */
PFR_API int pfr_last_kernel_timings(const pfr_solver* s, double* ms_out /* 5 */, int64_t* launches_out /* 5 */);

/* Algorithmic HBM bytes per frequency of one factorisation, per kernel class as above: complex
 * entries each class must store plus the entries it must read once (children's update-matrix
 * entries it gathers, factor blocks it consumes); index data, shared by all frequencies, excluded. */
PFR_API int pfr_solver_alg_bytes(const pfr_solver* s, int64_t* bytes_out /* 5 */);

/* Algorithmic HBM bytes per frequency of the triangular solves of one loss pfr_sweep under the
 * solver's current check mode: factor entries each pass must read (16 B each) plus rhs in / solution
 * out.  Symmetric mode without refinement, functional from the bottom-up passes (PFR_FN_DOT, default):
 * [0] the one bottom-up chain over the fronts the rhs or the loss support reach, [1] the paired top-down
 * pass over every front.  With PFR_FN_DOT=0 (the paired passes): [0] forward bottom-up over the fronts
 * the rhs reaches + forward top-down over the fronts the loss support reaches, [1] adjoint bottom-up
 * over that reach + the single top-down pass that reads every U value once for the adjoint and the
 * rest of the forward solution.  Otherwise [0] / [1] forward / adjoint pair (reached bottom-up + full
 * top-down; with PFR_CHECK_REFINE plus the full correction solve). */
PFR_API int pfr_solver_solve_bytes(const pfr_solver* s, int64_t* bytes_out /* 2 */);

#ifdef __cplusplus
}
#endif

#endif /* PFR_H */
