// Host launchers of the HIP kernels (defined in kernels.hip).
#pragma once

#include "device_types.hpp"

namespace pfr {

struct RhsDesc {
  const double* rhsP = nullptr;   // RHS 0: permuted Dirichlet vector (device)
  double beta_re = 0, beta_im = 0, mass_sum = 0;
  const double* freqs = nullptr;  // chunk frequencies (device, padded)
  const double2* B = nullptr;     // RHS 1: explicit batch (device, batch-major, caller numbering)
  int64_t b_stride = 0;
  const double2* G = nullptr;     // RHS 2: permuted frequency-minor vector (device)
  int nvalid = 1;                 // RHS 1: valid batch items of the chunk
  const int* cslot = nullptr;     // RHS 3: coupled-row slot per permuted row (symmetric mode)
  const double2* Bc = nullptr;    // RHS 3: Dirichlet corrections (slot-major)
};

// Dirichlet decoupling lists of a symmetric-mode solver (device pointers) + operator
struct DirDesc {
  const int2* dir = nullptr;
  const int* crow = nullptr;
  const int* cptr = nullptr;
  const int2* ce = nullptr;
  const int* dptr = nullptr;
  const int2* de = nullptr;
  const double2* K = nullptr;
  const double* M = nullptr;
  const double* freqs = nullptr;
};

// the first launch configuration refused since the last call (a kernel's dynamic LDS size), NULL: none; the
// refused launch was skipped
const char* launch_refused();

void launch_combine(const double* stiff, int n_stiff, int64_t nnz, const CoefPack& coef, double2* K, hipStream_t st);
void launch_assemble(int mode, const int4* recs, int nrec, const int* xptr, const int2* xl, int ngroups, double2* F,
                     int64_t Fc, const double* freqs, const double2* K, const double* M, const double2* data,
                     int64_t ds, int nvalid, hipStream_t st);
// G: lane groups per wave of the symmetric kernel (FAC_G, 4 or 8)
void launch_factor(bool sym, const DevPattern& P, const int* lvl, int nfronts, int W, int ngroups, double2* F, int64_t Fc,
                   int* flags, hipStream_t st, int G = FAC_G);
// symmetric A11 LU with the pivot block in LDS (one front x one frequency per workgroup); maxns = the level's
// largest pivot block (sizes the dynamic LDS: (maxns (maxns + 1) / 2 + 4 maxns) x 16 B)
void launch_factor_lds(const DevPattern& P, const int* lvl, int nfronts, int maxns, double2* F, int64_t Fc, int* flags,
                       hipStream_t st);
// L21 rows (and U12 columns in general mode) of a level's items; pipelined: the software-pipelined prefix
// (symmetric, operator-form launches with few waves)
// the bottom level fused (k_front0, Plan::fused0): fl = level-0 fronts, the first nsmall with <= 2 pivots
void launch_front0(const DevPattern& P, const int* fl, int nfronts, int nsmall, const int* fptr, const int* fnz,
                   int ngroups, double2* F, int64_t Fc, const double* freqs, const double2* K, const double* M,
                   int* flags, hipStream_t st);
void launch_offdiag(int mode, const DevPattern& P, const int4* items, int nitems, const int2* orec, const int* oxp,
                    const int2* ox, int ngroups, double2* F, int64_t Fc, const double* freqs, const double2* K,
                    const double* M, const double2* data, int64_t ds, int nvalid, int maxns, hipStream_t st,
                    bool pipelined = false);
// Schur complement A22 -= L21 U12 for a level's tile list (TM x TN = 4 x 4 tiles)
void launch_schur(bool sym, const DevPattern& P, const int4* tiles, int ntiles, const int* g1, const int* gxp,
                  const int2* gx, int ngroups, double2* F, int64_t Fc, hipStream_t st);
// symmetric mode, large update blocks: 16 x 16 blocks, operands staged in LDS per workgroup
void launch_schur_blk(const DevPattern& P, const int4* blocks, int nblocks, const int* bg1, const int* bgxp,
                      const int2* bgx, int ngroups, double2* F, int64_t Fc, hipStream_t st);
// which: 0 = L (bottom-up), 1 = U (top-down), 2 = U^T (bottom-up), 3 = L^T (top-down)
// split > 1 (L and U solves): the update part of every front (L: the update rows; U: the pivot rows'
// products with the update-row solution) runs first / last over `split` workgroups of SPLIT_W waves per
// (front, frequency group) -- the top levels' few fronts otherwise pull their L21 blocks through one CU each
// glist (may be NULL): the groups to solve, REFINE_CAP of them (-1: none), indexed by grid row (pass
// ngroups = REFINE_CAP); the selective adjoint refinement's solves
void launch_solve(int which, int rhs_mode, bool sym, const DevPattern& P, const int* lvl, int nfronts, int W, int ngroups,
                  const double2* F, int64_t Fc, double2* WV, const RhsDesc& rd, const double2* Yin, double2* Out,
                  const int* reach, hipStream_t st, int split = 1, const int* glist = nullptr);
// nslices (<= 4) bottom-up L solves as one chain of launches (blockIdx.z = slice; slice z: the fronts
// lvl[z][0 .. nf[z]), its work vectors WV[z], rhs rd[z] (rhs_mode 0 or 3 for every slice), solution Y[z])
void launch_lsolve_multi(int rhs_mode, const DevPattern& P, int nslices, const int* const* lvl, const int* nf, int W,
                         int ngroups, const double2* F, int64_t Fc, double2* const* WV, const RhsDesc* rd,
                         double2* const* Y, const int* const* reach, hipStream_t st, int split, bool nar = false,
                         int maxns = 0, int maxf = 0,    // nar (split > 1): pivot blocks in LDS, update rows
                                                         // column-split (k_lsolve_level_z<., true>, k_lsolve_rows_zc)
                         bool rl = true);                // nar + rl: pivot blocks right-looking (k_lsolve_rl_z)
// functional from the bottom-up passes: partial dot products (FN_PARTS x 3 x Fc), the functional / loss
// / cotangent from them (fcoef: 3 x Fc, G at the support rows), and L^-1 g = sum_k c_k L^-1 a_k in Yk[0]
void launch_fn_dot(const int2* rows, int nrows, const double2* F, const double2* Yb, const double2* const* Yk, int64_t Fc,
                   double2* parts, hipStream_t st);
void launch_functional_fn(const FunctionalArgs& A, const double2* parts, int64_t Fc, int nvalid, int64_t q0,
                          double* fr_out, double* loss_terms, double2* G, double2* fcoef, hipStream_t st);
void launch_fn_combine(const int* rows, int nrows, const double2* fcoef, double2* const* Yk, int64_t Fc, hipStream_t st);
// two top-down U solves in one pass (vector 0 skipped on the fronts flagged in skip0), symmetric
// mode; small: the low-register variant for levels of small fronts
void launch_usolve2(const DevPattern& P, const int* lvl, int nfronts, int W, bool small, int ngroups,
                    const double2* F, int64_t Fc, const double2* Y0, double2* X0, const int* reach0, const int* skip0,
                    const double2* Y1, double2* X1, const int* reach1, hipStream_t st, int split = 1,
                    int tiny = 0,     // tiny 4 / 8: the level's pivot blocks all <= tiny (k_usolve2_tiny)
                    bool nar = false, int maxns = 0,    // nar (split > 1): the update part column-split (k_usolve2_updc)
                    bool rl = true);                    // nar + rl: pivot blocks right-looking, prefetched (k_usolve2_rl)
// Hessian sweep: tangent right-hand sides (rows of the permuted matrix, or of its
// transpose with accumulate = 1) and the directional derivative of the loss cotangent
void launch_tangent_spmv(const int* ptr, const int* idx, const int* nzs, int nrows, const double2* Kd,
                         const double2* X, int64_t Fc, const double* rhsP, double2 beta, double2* Y, int accumulate,
                         hipStream_t st);
void launch_functional_tangent(const FunctionalArgs& A, const double2* X, const double2* DX, int64_t Fc, int nvalid,
                               int64_t q0, double2* G, hipStream_t st);
void launch_functional(const FunctionalArgs& A, const double2* X, int64_t Fc, int nvalid, int64_t q0, double* fr_out,
                       double* loss_terms, double2* G, hipStream_t st);
// gradient contraction with the frequency sum first (one partial per workgroup: contract_eg_parts of them)
// msc (may be NULL): per-frequency factor of Lam (functional correction: the loss cotangent scale)
void launch_contract_eg(const int4* ent, int nent, const double* se, int n_stiff, const double2* Lam, const double2* X,
                        int64_t Fc, int nvalid, double2* partial, hipStream_t st, const double2* msc = nullptr);
// entry-ordered copy of the stiffness matrices (se)
void launch_gather_entries(const int4* ent, int nent, const double* stiff, int ns, double* se, hipStream_t st);
void launch_rhs_dot(const int* sup, const double* val, int n_sup, const double2* Lam, int64_t Fc, double2* t_out,
                    hipStream_t st, const double2* msc = nullptr);
// w_out[k] += -sum(partial[., k]) + e_k sum_q t_q ;  loss_out += sum_q loss_terms (q < nvalid)
void launch_reduce(const double2* partial, int nparts, int n_stiff, const double2* t_q, const CoefPack& e,
                   const double* loss_terms, int nvalid, int64_t Fc, double2* w_out, double* loss_out,
                   hipStream_t st);
// symmetric mode: forward right-hand-side corrections (src 0: operator rhs -> Bc; src 2: G in
// place) and the adjoint's Dirichlet rows (X in place)
void launch_dirichlet_rhs(int src, const DirDesc& d, int n_crow, const RhsDesc& rd, double2* G, double2* Bc,
                          int64_t Fc, hipStream_t st);
void launch_dirichlet_post(const DirDesc& d, int n_dir, double2* X, int64_t Fc, hipStream_t st, const int* glist = nullptr);
// Backward-error check: the original system's rows (forward) or columns (adjoint) in the permuted
// numbering, A = K - omega^2 M (mode 0) or the explicit batch (mode 1); rhs 0 operator, 1 explicit
// B, 2 vector G.  The per-frequency componentwise backward error accumulates in acc (max, zero on
// entry); acc == NULL: only the residual is written to R.
struct ResidDesc {
  const int* ptr = nullptr;
  const int* idx = nullptr;
  const int* nzs = nullptr;
  int n = 0;
  const double2* K = nullptr;
  const double* M = nullptr;
  const double* freqs = nullptr;
  const double2* data = nullptr;
  int64_t data_stride = 0;
  int nvalid = 1;
  const double* rhsP = nullptr;
  double beta_re = 0, beta_im = 0, mass_sum = 0;
  const double2* B = nullptr;
  int64_t b_stride = 0;
  const int* perm = nullptr;
  const double2* G = nullptr;
  const int* walk = nullptr;   // the n rows (permuted numbering) in walk order
  // the gradient contraction fused into the forward walk (mode 0, rhs 0, Mu != NULL): stiffness values
  // nz-major (n_stiff 12 or 18 per nz) and the per (workgroup, k, frequency) output
  const double* se = nullptr;
  int n_stiff = 0;
  double2* kpart = nullptr;
  const int* glist = nullptr;  // the groups to walk (REFINE_CAP, -1: none; NULL: every group)
  int unroll = 4;              // entries per gather batch of the adjoint check walk (4 or 8; the same bits)
};
// Mu != NULL (mode 0, rhs 0): also the functional-correction dot products sum_p Mu_p r_p, one partial
// per workgroup and frequency in cpart (residual_parts(n) x Fc), summed by launch_correct_finish
// partial[t * n_stiff + k] = sum_{q in tile t} msc[q] sum_b kpart[b][k][q] (msc NULL: 1; tiles of 64
// frequencies): the fused walk's contraction as Fc / 64 parts
void launch_reduce_q(const double2* kpart, int nparts, int n_stiff, const double2* msc, int nvalid, int64_t Fc,
                     double2* partial, hipStream_t st);
void launch_residual(int mode, int rhs, const ResidDesc& d, const double2* X, int64_t Fc, double2* R, double* acc,
                     hipStream_t st, const double2* Mu = nullptr, double2* cpart = nullptr);
// corrected fr (fr_out, global index; may be NULL), loss terms and cotangent scales of a chunk
// gind != NULL: per 64-frequency group its largest |correction| / |fr| (launch_select_groups picks from them)
// tq != NULL: t_q = mu^T rhsP in, m_q t_q out, and the solve-error scale in m_q (k_correct_finish)
void launch_correct_finish(const FunctionalArgs& A, const double* fr0, const double2* cpart, int nparts, int64_t Fc,
                           int nvalid, int64_t q0, double* fr_out, double* loss_terms, double2* mscale,
                           hipStream_t st, double* gind = nullptr, double2* tq = nullptr,
                           const RhsScale& bsc = RhsScale());
// glist[0 .. REFINE_CAP): the groups with the largest indicators above tol, largest first, -1 past them
void launch_select_groups(const double* gind, int ngroups, double tol, int* glist, hipStream_t st);
// flags |= flag where acc[q] > tol (or not finite); acc cleared
void launch_berr_finish(double* acc, int64_t Fc, int nvalid, double tol, int flag, int* flags, double* berr_out,
                        int64_t q0, int which, hipStream_t st);
void launch_axpy_vec(double2* X, const double2* D, int64_t count, hipStream_t st, const int* glist = nullptr,
                     int64_t Fc = 64);
void launch_scale_vec(double2* X, const double2* m, int n, int64_t Fc, hipStream_t st);
void launch_unpermute(const int* perm, int n, const double2* X, int64_t Fc, int nvalid, double2* out, hipStream_t st);
void launch_matvec(const int* colptr, const int* rowind, int n, const double2* data, int64_t ds, const double2* x,
                   int64_t xs, double2* y, int transpose, int batch, hipStream_t st);

}  // namespace pfr
