// C ABI of libpfr.so (see include/pfr.h).  Host orchestration of the HIP kernels:
// level-scheduled launches over frequency chunks, workspaces, timing.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <functional>
#include <cstring>
#include <string>
#include <vector>

#include "launch.hpp"

using pfr::DevPattern;
using pfr::Front;
using pfr::Symbolic;

struct pfr_symbolic {
  Symbolic S;
};

namespace {
thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

// after a group of launches: a refused launch configuration (pfr::launch_refused) or a launch error
#define LAUNCH_TRY()                                                                      \
  do {                                                                                    \
    if (const char* _k = pfr::launch_refused())                                           \
      return fail(PFR_ERR_HIP, std::string("hipFuncSetAttribute refused the dynamic LDS size of ") + _k); \
    HIP_TRY(hipGetLastError());                                                           \
  } while (0)

#define HIP_TRY(expr)                                                                     \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess)                                                                 \
      return fail(_e == hipErrorOutOfMemory ? PFR_ERR_NOMEM : PFR_ERR_HIP,                \
                  std::string(#expr) + ": " + hipGetErrorString(_e));                     \
  } while (0)

template <class T>
int upload(T** dst, const std::vector<T>& src) {
  *dst = nullptr;
  if (src.empty()) return PFR_OK;
  HIP_TRY(hipMalloc(dst, src.size() * sizeof(T)));
  HIP_TRY(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
  return PFR_OK;
}

int64_t round64(int64_t x) { return (x + 63) / 64 * 64; }

}  // namespace

struct pfr_solver {
  int device = 0;
  int n = 0;
  int64_t nnz = 0;
  int64_t Fc = 0;  // frequencies per chunk (multiple of 64)
  std::vector<int32_t> level_ptr, level_maxf, level_maxns, level_W, perm, iperm;
  std::vector<int32_t> tile_ptr, blk_ptr, asm_ptr, item_ptr;   // per level: first Schur tile / block, A11 record, L21 item
  DevPattern P{};
  // owned device arrays
  std::vector<void*> owned;
  int32_t* d_level_fronts = nullptr;
  int4* d_tiles = nullptr;              // Schur tiles (front, i0, j0, 0), grouped by level
  int4* d_items = nullptr;              // off-diagonal panel items (front, first row/col, kind, record offset)
  int2* d_orec = nullptr;               // per item x lane group x pivot: (nz, first child source) of the entry
  bool fused0 = false;                  // level 0 through k_front0 (Plan::fused0)
  int n_f0 = 0, f0_small = 0;
  int32_t *d_f0_front = nullptr, *d_f0_ptr = nullptr, *d_f0_nz = nullptr;
  int32_t* d_oxp = nullptr;             // per item: range of further child sources in d_ox
  int2* d_ox = nullptr;                 // (pivot * OFF_G OFF_RPL + row slot, element id)
  int32_t* d_g1 = nullptr;              // per super-tile, lane group, position: first child source (or -1)
  int32_t* d_gxp = nullptr;             // per super-tile: range of further sources in d_gx
  int2* d_gx = nullptr;                 // (lane group * 16 + position, element id) of the rare extra sources
  // symmetric mode, fronts with large update blocks: 16 x 16 Schur blocks (k_schur_sym_blk)
  int4* d_blocks = nullptr;             // (front, i0, j0, 0), grouped by level
  int32_t* d_bg1 = nullptr;             // per block, wave, position: first child source (or -1)
  int32_t* d_bgxp = nullptr;            // per block: range of further sources in d_bgx
  int2* d_bgx = nullptr;                // (wave * 16 + position, element id)
  int4* d_asm = nullptr;                // panel-entry assembly records (dst, nz, first child source, 0), by level
  int32_t* d_asm_xp = nullptr;          // per 8-record chunk: range of further child sources in d_asm_x
  int2* d_asm_x = nullptr;              // (record within chunk, child element id)
  int32_t* d_colptr = nullptr;
  int32_t* d_rowind = nullptr;
  // symmetric mode (options.symmetric): U never formed; Dirichlet nodes decoupled
  bool sym = false;
  int n_dir = 0, n_crow = 0;
  int2* d_dir = nullptr;                // per Dirichlet node: (permuted node, diagonal entry)
  int32_t* d_crow = nullptr;            // coupled rows (permuted)
  int32_t* d_cptr_dir = nullptr;        // their entry ranges in d_ce
  int2* d_ce = nullptr;                 // (Dirichlet slot, entry) by coupled row
  int32_t* d_dptr = nullptr;            // per Dirichlet node: entry range in d_de
  int2* d_de = nullptr;                 // (permuted row, entry) by Dirichlet node
  int32_t* d_cslot = nullptr;           // per permuted row: coupled-row slot or -1
  double2* Bc = nullptr;                // forward right-hand-side corrections (n_crow x Fc)
  // right-hand-side reach (0 = forward operator rhs, 1 = loss adjoint on the functional support):
  // the fronts holding a support row and their elimination-tree ancestors -- the only fronts
  // whose bottom-up solve can be non-zero (per-front flags + the fronts level by level)
  std::vector<int32_t> front_of_col, front_parent, level_fronts_host, front_ns, front_f;
  std::vector<char> reach_host[2];
  // functional from the bottom-up passes (symmetric loss / correction sweeps, PFR_FN_DOT, default on):
  // slices 1-3 of the forward bottom-up chain solve L w_k = a_k over the support's reach; F_k = w_k^T
  // diag(U)^-1 y; the adjoint's bottom-up result = sum_k c_k w_k -- no top-down pass over the support's
  // fronts and no separate adjoint bottom-up pass
  int fn_dot = 1;
  bool fn_ready = false;                // row lists below match the current reaches
  std::vector<int32_t> front_off, front_col0;
  std::vector<double> a_perm;           // 3 x n: a_k at the permuted support rows
  double* d_aP = nullptr;               // device copy of a_perm
  int32_t* d_noslot = nullptr;          // n x -1 (no coupling slot: slices 1-3)
  int2* d_fn_rows = nullptr;            // (row, factor element of U(row, row)): pivot rows in both reaches
  int n_fn_rows = 0;
  int32_t* d_sup_rows = nullptr;        // pivot rows of the support-reach fronts
  int n_sup_rows = 0;
  double2* WVk = nullptr;               // 3 x total_rows x Fc (slices 1-3 work vectors)
  double2* YVk = nullptr;               // 2 x n x Fc (slices 2, 3 solutions; slice 1's is Y2)
  double2* fn_parts = nullptr;          // FN_PARTS x 3 x Fc
  double2* fcoef = nullptr;             // 3 x Fc
  // the gradient contraction fused into the forward residual walk (PFR_CONTRACT_WALK, default on; needs
  // the functional correction's walk): per (workgroup, k, frequency) sums, reduced with m_q by k_reduce_q
  int contract_walk = 1;
  double2* kpart = nullptr;
  int32_t* d_reach[2] = {nullptr, nullptr};
  int32_t* d_reach_fronts[2] = {nullptr, nullptr};
  std::vector<int32_t> reach_ptr[2];
  double2 *F = nullptr, *WV = nullptr, *X = nullptr, *Y = nullptr, *XA = nullptr, *G = nullptr, *Y2 = nullptr;
  double2* XR = nullptr;                // refinement correction of the adjoint (PFR_CHECK_REFINE)
  // Hessian sweep: permuted matrix by rows and by columns ((ptr, index, nz) each),
  // tangent solution / adjoint vectors, combined tangent operators (lazily allocated)
  int32_t *d_rptr = nullptr, *d_ridx = nullptr, *d_rnz = nullptr;
  int32_t* d_walk = nullptr;            // rows (permuted numbering) in original order: the residual
                                        // walks' order (mesh-local gathers, whatever the ordering)
  int32_t *d_cptr = nullptr, *d_cidx = nullptr, *d_cnz = nullptr;
  double2 *DX = nullptr, *DL = nullptr, *Kdir = nullptr;
  // gradient contraction entries (k_contract_eg): per permuted row a pseudo-entry (-1, -1, -1, i), then
  // (column, nz of (i, j) or -1, nz of (j, i) or -1, i) over the union of the row's and the column's patterns
  int4* d_uent = nullptr;
  int n_uent = 0;
  double* d_se = nullptr;               // entry-ordered S_k(i, j) (pfr_set_stiffness)
  int n_kdir = 0;
  double2 *partial = nullptr, *tq = nullptr;
  double *freqs = nullptr, *loss_terms = nullptr;
  // functional correction (PFR_CHECK_CORRECT): fr of the solve, per-frequency cotangent scale, and
  // the residual walk's per-workgroup dot-product partials (residual_parts(n) x Fc)
  double* fr0 = nullptr;
  double2 *mscale = nullptr, *cpart = nullptr;     // mscale complex: the solve-error scale (k_correct_finish)
  int scale_corr = 1;                   // PFR_SCALE_CORR: the solve-error scale of the loss sweeps' cotangent
  int us2_tiny = 8;                     // PFR_US2_TINY (0 / 4 / 8): levels whose pivot blocks are <= this, one wave per front
  int off_pu_waves = 0;                 // PFR_OFF_PU_WAVES: L21 launches with fewer waves run the pipelined prefix
  int32_t* flags = nullptr;
  // operator / rhs / functional / stiffness state
  const double2* K = nullptr;
  const double* M = nullptr;
  double* rhsP = nullptr;
  int32_t* rhs_sup = nullptr;
  double* rhs_val = nullptr;
  int n_rhs_sup = 0;
  std::vector<double> rhs_host;         // last Dirichlet vector uploaded (original order)
  double beta_re = 0, beta_im = 0, mass_sum = 0;
  bool has_rhs = false;
  pfr::FunctionalArgs fn{};
  bool has_fn = false;
  const double* stiff = nullptr;
  int n_stiff = 0;
  pfr::CoefPack e{};
  // timing: bit 0 = phases, bit 1 = factorisation kernel classes (5 events per level).
  // Events of every chunk of the last call are kept and read only when the caller
  // asks (pfr_last_timings): no host synchronisation inside a call, so solvers on
  // different streams overlap.
  struct ChunkEvents {
    hipEvent_t ev[6]{};
    std::vector<hipEvent_t> kev;        // factorisation kernel classes: NKC + 1 events per level
    bool used[5]{};
    bool f0 = false;                    // level 0 ran fused (k_front0): its launches are all class 0
  };
  int timing = 0;
  std::vector<ChunkEvents> tev;
  int n_tev = 0;                        // chunks recorded by the last call
  // algorithmic HBM bytes per frequency of each factorisation kernel class, per level (16 B per complex entry
  // loaded or stored; index data is shared by all frequencies and not counted)
  std::vector<std::array<int64_t, pfr::NKC>> lev_bytes;
  pfr::Workspace ws;                    // element counts of the chunk buffers (plan.cpp; what is allocated)
  // launch-shape tuning knobs, read from the environment when the solver is created (so that a
  // process can build solvers with different settings, e.g. tests forcing each kernel variant):
  // PFR_SOLVE_WMAX (waves per solve workgroup, at most), PFR_FAC_WMAX (waves per A11 LU
  // workgroup, at most), PFR_US2_SMALL (largest front of a level the paired top-down solve treats
  // with its low-register small-front variant)
  int solve_wmax = 8, fac_wmax = 16, us2_small = 110;
  int fac_lds = -1;                     // PFR_FAC_LDS: which levels factor A11 in LDS (k_factor_sym_lds): n > 0
                                        // those whose largest pivot block has at least n pivots, 0 none, -1 auto
                                        // (default since round 3: 512-frequency sweeps +2.6 %, 4,096 unchanged)
  int fac_lds_wg = 160;                 // PFR_FAC_LDS_WG: auto mode threshold (workgroups of k_factor_sym)
  int res_unroll = 8;                   // PFR_RES_UNROLL: entries per gather batch of the adjoint check walk (4 / 8)
  int fac_g_wg = 0;                     // PFR_FAC_G_WG: k_factor_sym launches below this many workgroups take G = 4 / 8
  int fac_gbig = 4, fac_g_ns = 64;      // PFR_FAC_GBIG / PFR_FAC_G_NS: k_factor_sym's lane groups per wave on the
                                        // levels whose largest pivot block exceeds PFR_FAC_G_NS pivots
  int us2_nar = 256;                    // PFR_US2_NAR: solve launches (paired top-down, bottom-up chain) with fewer
                                        // (front, group) workgroups than this take the narrow-level forms -- pivot
                                        // blocks in LDS, left-looking, the update parts with their columns split
                                        // over the waves (k_usolve2_updc + k_usolve2_rl, k_lsolve_level_z<., true>
                                        // + k_lsolve_rows_zc); 0: never.  Measured best at 256 for both passes
                                        // (1,024 / 4,096: no gain at 512 frequencies, slower at 4,096)
  int us2_rl = 1;                       // PFR_US2_RL: k_usolve2_rl for the narrow levels' paired pivot blocks
  int ls_rl = 1;                        // PFR_LS_RL: k_lsolve_rl_z for the bottom-up chain's narrow pivot blocks
  int split_target = 256;               // PFR_SOLVE_SPLIT: solve launches with fewer (front, group) workgroups
                                        // than this (one per CU) split their update parts up to about this
                                        // many workgroups (0: off)
  // backward-error checks (pfr_set_check): PFR_CHECK_* bits, tolerance, optional per-item output;
  // per-frequency maxima scratch, forward and adjoint (kept zero between checks)
  int check_mode = 0;
  double check_tol = 1e-10;
  double refine_tol = 2e-8;             // PFR_CHECK_REFINE_ADJ group threshold (pfr_set_refine_tol)
  double* gind = nullptr;               // per 64-frequency group: largest |correction| / |fr| of the chunk
  int32_t* glist = nullptr;             // the groups whose adjoint is refined (REFINE_CAP, -1: none)
  double2* Gx = nullptr;                // the fr seed of the forward solution (support rows; zero elsewhere)
  double* berr_out = nullptr;
  double* d_berr_acc = nullptr;
  // sweep graphs (PFR_GRAPH=1): a pfr_sweep called again with the same arguments and solver state (gen:
  // bumped by every setter that changes what a sweep enqueues) is captured once into a hipGraph and from then on
  // replayed with one hipGraphLaunch instead of ~160-290 kernel launches; any other sweep runs the launches
  // directly.  graph_off: a capture failed on this solver, no further attempts.
  int graph_mode = 0;
  bool graph_off = false;
  uint64_t gen = 0;
  std::array<uint64_t, 14> gkey{};
  bool gkey_valid = false;
  hipGraph_t graph = nullptr;
  hipGraphExec_t gexec = nullptr;
  int64_t graph_launches = 0;           // sweeps replayed from the graph (pfr_sweep_graph_launches)

  void drop_graph() {
    if (gexec) (void)hipGraphExecDestroy(gexec);
    if (graph) (void)hipGraphDestroy(graph);
    gexec = nullptr;
    graph = nullptr;
  }
  ~pfr_solver() {
    drop_graph();
    for (void* p : owned) (void)hipFree(p);
    for (auto& c : tev) {
      for (auto& x : c.ev)
        if (x) (void)hipEventDestroy(x);
      for (auto& x : c.kev)
        if (x) (void)hipEventDestroy(x);
    }
  }
  template <class T>
  int alloc(T** p, int64_t count) {
    *p = nullptr;
    if (count <= 0) return PFR_OK;
    HIP_TRY(hipMalloc(p, count * sizeof(T)));
    owned.push_back(*p);
    return PFR_OK;
  }
  template <class T>
  int up(T** p, const std::vector<T>& v) {
    int rc = upload(p, v);
    if (rc == PFR_OK && *p) owned.push_back(*p);
    return rc;
  }
  // a plan record array (pfr::I2 / I4) as its HIP vector type (same layout), never empty on the device
  template <class D, class H>
  int up_rec(D** p, const std::vector<H>& v, H pad) {
    static_assert(sizeof(D) == sizeof(H), "record layout");
    std::vector<H> w(v);
    if (w.empty()) w.push_back(pad);
    *p = nullptr;
    HIP_TRY(hipMalloc(p, w.size() * sizeof(H)));
    owned.push_back(*p);
    HIP_TRY(hipMemcpy(*p, w.data(), w.size() * sizeof(H), hipMemcpyHostToDevice));
    return PFR_OK;
  }
};

namespace {

int64_t workspace_bytes(const Symbolic& S, int64_t Fc) {
  int n_crow = 0;                     // coupled rows (Dirichlet decoupling): count as in build_plan
  for (size_t c = 0; c < S.cpl_p.size(); ++c) n_crow += c == 0 || S.cpl_p[c] != S.cpl_p[c - 1];
  return pfr::workspace(S, Fc, S.symmetric ? n_crow : 0).bytes;
}

// start the timing record of a new chunk (events created once per chunk slot)
int begin_chunk(pfr_solver* s) {
  if (!s->timing) return PFR_OK;
  if ((int)s->tev.size() <= s->n_tev) {
    s->tev.emplace_back();
    for (auto& e : s->tev.back().ev) HIP_TRY(hipEventCreate(&e));
  }
  auto& c = s->tev[s->n_tev];
  const size_t nk = (pfr::NKC + 1) * (s->level_ptr.size() - 1);
  while ((s->timing & 2) && c.kev.size() < nk) {
    hipEvent_t e;
    HIP_TRY(hipEventCreate(&e));
    c.kev.push_back(e);
  }
  return PFR_OK;
}

void record(pfr_solver* s, int i, hipStream_t st) {
  if (s->timing) (void)hipEventRecord(s->tev[s->n_tev].ev[i], st);
}

int finish_timing(pfr_solver* s, const bool* used) {
  if (!s->timing) return PFR_OK;
  for (int i = 0; i < 5; ++i) s->tev[s->n_tev].used[i] = used[i];
  ++s->n_tev;
  return PFR_OK;
}

void reset_timing(pfr_solver* s) { s->n_tev = 0; }

// Waves per workgroup of a solve launch over nf fronts of level l: the level's size-based count,
// raised (up to 8) when the launch has too few workgroups to fill the chip -- the sparse passes
// and the top levels, which are latency-bound: every wave more takes rows off each wave's chain.
int solve_W(const pfr_solver* s, int l, int nf) { return pfr::solve_waves(s->level_W[l], nf, s->Fc, s->solve_wmax); }

// Workgroups per (front, frequency group) for the update part of a solve launch over nf fronts: 1 when the
// launch already has split_target workgroups, else enough to reach it (at most 16).
int solve_split(const pfr_solver* s, int nf) { return pfr::solve_split(nf, s->Fc, s->split_target); }

// A11 of level l factored in LDS (k_factor_sym_lds): PFR_FAC_LDS = n > 0: levels whose largest pivot block has
// >= n pivots; -1: levels on which the global-memory kernel would get fewer than PFR_FAC_LDS_WG workgroups (the
// top of the tree in small chunks: 512 frequencies levels 10-16, 2,048 level 16 -- faster per level there, slower
// elsewhere; the default since the MMD ordering: 512-frequency sweeps 31.8k -> 32.6k freq-solves/s, 4,096
// unchanged)
bool level_lds(const pfr_solver* s, int l) {
  const int64_t wgs = (int64_t)(s->level_ptr[l + 1] - s->level_ptr[l]) * (s->Fc / 64) * pfr::FAC_G;
  return s->sym && s->level_maxns[l] <= 64 &&
         (s->fac_lds > 0 ? s->level_maxns[l] >= s->fac_lds
                         : s->fac_lds < 0 && s->level_maxns[l] >= 16 && wgs < s->fac_lds_wg);
}

int factor_all(pfr_solver* s, int mode, const double2* data, int64_t ds, int nvalid, hipStream_t st) {
  const int L = (int)s->level_ptr.size() - 1;
  const int ngroups = (int)(s->Fc / 64);
  const bool kt = (s->timing & 2) && s->n_tev < (int)s->tev.size() && !s->tev[s->n_tev].kev.empty();
  hipEvent_t* kev = kt ? s->tev[s->n_tev].kev.data() : nullptr;
  auto mark = [&](int l, int c) {
    if (kt) (void)hipEventRecord(kev[(pfr::NKC + 1) * l + c], st);
  };
  if (kt) s->tev[s->n_tev].f0 = false;
  for (int l = 0; l < L; ++l) {
    int nf = s->level_ptr[l + 1] - s->level_ptr[l];
    mark(l, 0);
    if (l == 0 && s->fused0 && mode == 0) {
      if (kt) s->tev[s->n_tev].f0 = true;
      // the bottom level's leaf fronts in one pass (k_front0): A11, L21 and update block per frequency in registers
      pfr::launch_front0(s->P, s->d_f0_front, s->n_f0, s->f0_small, s->d_f0_ptr, s->d_f0_nz, ngroups, s->F, s->Fc,
                         s->freqs, s->K, s->M, s->flags, st);
      for (int c = 1; c <= 5; ++c) mark(l, c);
      continue;
    }
    // panel: enough workgroups (front x 16 frequencies) to fill the chip -> one wave
    // each (no idle waves at the block barriers); few large fronts -> more waves
    // (symmetric kernel: up to 16 waves -- the top levels' few fronts are latency-bound, every
    // wave more takes rows off each wave's serial chain)
    const int fac_wmax = s->fac_wmax;
    // lane groups per wave of the symmetric A11 kernel: FAC_G; fac_gbig on the levels with a pivot block of more
    // than fac_g_ns pivots, whose long chains gain from more row slots per wave (the deep tree's level 25 with its
    // 76-pivot separator at 2,048 frequencies: 0.61 -> 0.41 ms with 4; the levels of 2-3 fronts of <= 35 pivots
    // below it were slower with 4, gpurun_out/fg2_t2048_*); raised to 4 / 8 while the launch has fewer than
    // fac_g_wg workgroups (default off)
    int G = (s->sym && s->level_maxns[l] > s->fac_g_ns) ? s->fac_gbig : pfr::FAC_G;
    while (s->sym && G < 8 && (int64_t)nf * ngroups * G < s->fac_g_wg) G *= 2;
    const int64_t wgs = (int64_t)nf * ngroups * G;
    const int64_t wfill = (4096 + wgs - 1) / wgs;
    const int Wp = (int)std::max<int64_t>(
        1, s->sym ? std::min<int64_t>(fac_wmax, wfill) : std::min<int64_t>(s->level_W[l], wfill));
    pfr::launch_assemble(mode, s->d_asm + s->asm_ptr[l], s->asm_ptr[l + 1] - s->asm_ptr[l],
                         s->d_asm_xp + s->asm_ptr[l] / 8, s->d_asm_x, ngroups, s->F, s->Fc, s->freqs, s->K, s->M,
                         data, ds, nvalid, st);
    mark(l, 1);
    if (level_lds(s, l))
      pfr::launch_factor_lds(s->P, s->d_level_fronts + s->level_ptr[l], nf, s->level_maxns[l], s->F, s->Fc, s->flags, st);
    else
      pfr::launch_factor(s->sym, s->P, s->d_level_fronts + s->level_ptr[l], nf, Wp, ngroups, s->F, s->Fc, s->flags, st,
                         G);
    mark(l, 2);
    // the software-pipelined L21 prefix on the launches with few waves (symmetric analyses, operator form)
    const int64_t owaves = (int64_t)(s->item_ptr[l + 1] - s->item_ptr[l]) * ngroups;
    pfr::launch_offdiag(mode, s->P, s->d_items + s->item_ptr[l], s->item_ptr[l + 1] - s->item_ptr[l], s->d_orec,
                        s->d_oxp + s->item_ptr[l], s->d_ox, ngroups, s->F, s->Fc, s->freqs, s->K, s->M, data, ds,
                        nvalid, s->level_maxns[l], st, s->sym && owaves < s->off_pu_waves);
    mark(l, 3);
    pfr::launch_schur_blk(s->P, s->d_blocks + s->blk_ptr[l], s->blk_ptr[l + 1] - s->blk_ptr[l],
                          s->d_bg1 + (int64_t)s->blk_ptr[l] * 16 * 16, s->d_bgxp + s->blk_ptr[l], s->d_bgx, ngroups, s->F,
                          s->Fc, st);
    mark(l, 4);
    pfr::launch_schur(s->sym, s->P, s->d_tiles + s->tile_ptr[l], s->tile_ptr[l + 1] - s->tile_ptr[l],
                      s->d_g1 + (int64_t)s->tile_ptr[l] * pfr::SCHUR_TM * pfr::SCHUR_TN * pfr::SCHUR_SR * pfr::SCHUR_SC,
                      s->d_gxp + s->tile_ptr[l], s->d_gx, ngroups, s->F, s->Fc, st);
    mark(l, 5);
  }
  LAUNCH_TRY();
  return PFR_OK;
}

// which: 0 L, 1 U, 2 U^T, 3 L^T ; bottom-up for 0/2, top-down for 1/3
// subset (0 forward rhs, 1 loss adjoint, -1 none): bottom-up passes visit only the reached
// fronts; top-down passes treat the pivot values of unreached fronts as zero
int solve_all(pfr_solver* s, int which, int rhs_mode, const pfr::RhsDesc& rd, const double2* Yin, double2* Out,
              hipStream_t st, int subset = -1, const int* glist = nullptr) {
  const int L = (int)s->level_ptr.size() - 1;
  const int ngroups = glist ? pfr::REFINE_CAP : (int)(s->Fc / 64);
  const bool up = (which == 0 || which == 2);
  const int* reach = subset >= 0 ? s->d_reach[subset] : nullptr;
  for (int t = 0; t < L; ++t) {
    int l = up ? t : L - 1 - t;
    const int32_t* lvl = s->d_level_fronts + s->level_ptr[l];
    int nf = s->level_ptr[l + 1] - s->level_ptr[l];
    if (up && subset >= 0) {
      lvl = s->d_reach_fronts[subset] + s->reach_ptr[subset][l];
      nf = s->reach_ptr[subset][l + 1] - s->reach_ptr[subset][l];
    }
    // the update parts split over several workgroups: L solves, and U solves in symmetric mode
    const int split = (which == 0 || (which == 1 && s->sym)) ? solve_split(s, nf) : 1;
    pfr::launch_solve(which, rhs_mode, s->sym, s->P, lvl, nf, solve_W(s, l, nf), ngroups, s->F, s->Fc, s->WV, rd, Yin, Out,
                      reach, st, split, glist);
  }
  LAUNCH_TRY();
  return PFR_OK;
}

pfr::DirDesc dir_desc(const pfr_solver* s) {
  pfr::DirDesc d;
  d.dir = s->d_dir;
  d.crow = s->d_crow;
  d.cptr = s->d_cptr_dir;
  d.ce = s->d_ce;
  d.dptr = s->d_dptr;
  d.de = s->d_de;
  d.K = s->K;
  d.M = s->M;
  d.freqs = s->freqs;
  return d;
}

// A x = b on the chunk's factors, x -> Out (permuted).  rhs_mode 0: operator right-hand side
// (rd.rhsP ...); 2: vector rd.G (overwritten in symmetric mode).  Symmetric mode: Dirichlet
// columns moved to the right-hand side first, then L and U = diag(U) L^T.
int forward_solve(pfr_solver* s, int rhs_mode, pfr::RhsDesc rd, double2* Out, hipStream_t st, int subset = -1) {
  int rc;
  if (s->sym) {
    const pfr::DirDesc dd = dir_desc(s);
    if (rhs_mode == 0) {
      pfr::launch_dirichlet_rhs(0, dd, s->n_crow, rd, nullptr, s->Bc, s->Fc, st);
      rd.cslot = s->d_cslot;
      rd.Bc = s->Bc;
      if (s->n_crow > 0) rhs_mode = 3;
    } else {
      pfr::launch_dirichlet_rhs(2, dd, s->n_crow, rd, const_cast<double2*>(rd.G), nullptr, s->Fc, st);
    }
  }
  if ((rc = solve_all(s, 0, rhs_mode, rd, nullptr, s->Y, st, subset))) return rc;
  return solve_all(s, 1, 0, rd, s->Y, Out, st, subset);
}

// A^T l = g (g = rg.G, permuted), l -> Out.  Symmetric mode: the decoupled matrix is symmetric,
// so L and U = diag(U) L^T again, then the Dirichlet rows of l are corrected.
int adjoint_solve(pfr_solver* s, const pfr::RhsDesc& rg, double2* Out, hipStream_t st, int subset = -1,
                  const int* glist = nullptr) {
  int rc;
  if (s->sym) {
    if ((rc = solve_all(s, 0, 2, rg, nullptr, s->Y, st, subset, glist)) ||
        (rc = solve_all(s, 1, 0, rg, s->Y, Out, st, subset, glist)))
      return rc;
    pfr::launch_dirichlet_post(dir_desc(s), s->n_dir, Out, s->Fc, st, glist);
    return PFR_OK;
  }
  if ((rc = solve_all(s, 2, 2, rg, nullptr, s->Y, st, subset))) return rc;
  return solve_all(s, 3, 0, rg, s->Y, Out, st, subset);
}

// Row lists and buffers of the functional-from-bottom-up path (allocated on first use, lists rebuilt
// whenever a reach changed)
int fn_setup(pfr_solver* s) {
  int rc;
  const int64_t n = s->n;
  if (!s->WVk) {
    if ((rc = s->alloc(&s->WVk, s->ws.WVk)) || (rc = s->alloc(&s->YVk, s->ws.YVk)) ||
        (rc = s->alloc(&s->fn_parts, s->ws.fn_parts)) || (rc = s->alloc(&s->fcoef, s->ws.fcoef)) ||
        (rc = s->up(&s->d_noslot, std::vector<int32_t>(n, -1))) || (rc = s->alloc(&s->d_aP, 3 * n)) ||
        (rc = s->alloc(&s->d_fn_rows, n)) || (rc = s->alloc(&s->d_sup_rows, n)))
      return rc;
    HIP_TRY(hipMemcpy(s->d_aP, s->a_perm.data(), s->a_perm.size() * 8, hipMemcpyHostToDevice));
  }
  if (s->fn_ready) return PFR_OK;
  std::vector<int2> both;
  std::vector<int32_t> sup;
  for (size_t t = 0; t < s->front_ns.size(); ++t) {
    if (!s->reach_host[1][t]) continue;
    for (int a = 0; a < s->front_ns[t]; ++a) {
      const int32_t row = s->front_col0[t] + a;
      sup.push_back(row);
      if (s->reach_host[0][t])
        both.push_back(make_int2(row, s->front_off[t] + a * s->front_f[t] + a));
    }
  }
  s->n_fn_rows = (int)both.size();
  s->n_sup_rows = (int)sup.size();
  // at most n rows each (pivot rows are distinct): into the buffers allocated for n
  if (!both.empty()) HIP_TRY(hipMemcpy(s->d_fn_rows, both.data(), both.size() * sizeof(int2), hipMemcpyHostToDevice));
  if (!sup.empty()) HIP_TRY(hipMemcpy(s->d_sup_rows, sup.data(), sup.size() * 4, hipMemcpyHostToDevice));
  s->fn_ready = true;
  return PFR_OK;
}

// forward bottom-up over the rhs reach (slice 0) and L w_k = a_k over the support reach (slices 1-3),
// one launch chain
int fn_bottom_up(pfr_solver* s, int rhs_mode, const pfr::RhsDesc& rf, hipStream_t st) {
  const int L = (int)s->level_ptr.size() - 1;
  const int ngroups = (int)(s->Fc / 64);
  int64_t total_rows = 0;
  for (size_t t = 0; t < s->front_f.size(); ++t) total_rows += s->front_f[t];
  pfr::RhsDesc rd[4] = {rf, rf, rf, rf};
  double2* WV[4] = {s->WV, s->WVk, s->WVk + total_rows * s->Fc, s->WVk + 2 * total_rows * s->Fc};
  double2* Y[4] = {s->Y, s->Y2, s->YVk, s->YVk + (int64_t)s->n * s->Fc};
  const int* reach[4] = {s->d_reach[0], s->d_reach[1], s->d_reach[1], s->d_reach[1]};
  for (int k = 1; k < 4; ++k) {
    rd[k].rhsP = s->d_aP + (int64_t)(k - 1) * s->n;
    rd[k].mass_sum = 0.0;
    rd[k].beta_re = 1.0;
    rd[k].beta_im = 0.0;
    rd[k].cslot = s->d_noslot;
  }
  for (int l = 0; l < L; ++l) {
    const int* lvl[4];
    int nf[4];
    lvl[0] = s->d_reach_fronts[0] + s->reach_ptr[0][l];
    nf[0] = s->reach_ptr[0][l + 1] - s->reach_ptr[0][l];
    for (int k = 1; k < 4; ++k) {
      lvl[k] = s->d_reach_fronts[1] + s->reach_ptr[1][l];
      nf[k] = s->reach_ptr[1][l + 1] - s->reach_ptr[1][l];
    }
    const int nmax = std::max(nf[0], nf[1]);
    if (nmax == 0) continue;
    const int nsum = nf[0] + 3 * nf[1];
    const bool nar = (int64_t)nsum * ngroups < s->us2_nar && pfr::ls_nar_fits(s->level_maxns[l]);
    pfr::launch_lsolve_multi(rhs_mode, s->P, 4, lvl, nf, solve_W(s, l, nmax), ngroups, s->F, s->Fc, WV, rd, Y, reach,
                             st, solve_split(s, nsum), nar, s->level_maxns[l], s->level_maxf[l], s->ls_rl != 0);
  }
  LAUNCH_TRY();
  return PFR_OK;
}

// Symmetric mode, loss + gradient: the forward top-down pass first over the fronts the loss
// support reaches only (they hold every support row), then -- once the loss cotangent is known
// and its bottom-up pass (same fronts) done -- ONE top-down pass computes the adjoint on every
// front and the forward solution on the rest, each factor value loaded once for both.
int sym_top_down_support(pfr_solver* s, const pfr::RhsDesc& rd, hipStream_t st) {
  const int L = (int)s->level_ptr.size() - 1;
  const int ngroups = (int)(s->Fc / 64);
  for (int l = L - 1; l >= 0; --l) {
    const int nf = s->reach_ptr[1][l + 1] - s->reach_ptr[1][l];
    pfr::launch_solve(1, 0, true, s->P, s->d_reach_fronts[1] + s->reach_ptr[1][l], nf, solve_W(s, l, nf), ngroups, s->F,
                      s->Fc, s->WV, rd, s->Y, s->X, s->d_reach[0], st, solve_split(s, nf));
  }
  LAUNCH_TRY();
  return PFR_OK;
}

int sym_top_down_pair(pfr_solver* s, hipStream_t st, bool fwd_all = false) {
  const int L = (int)s->level_ptr.size() - 1;
  const int ngroups = (int)(s->Fc / 64);
  for (int l = L - 1; l >= 0; --l) {
    const int nf = s->level_ptr[l + 1] - s->level_ptr[l];
    const bool small = s->level_maxf[l] <= s->us2_small;
    const int tiny = s->us2_tiny > 0 && s->level_maxns[l] <= s->us2_tiny ? (s->level_maxns[l] <= 4 ? 4 : 8) : 0;
    const bool nar = (int64_t)nf * ngroups < s->us2_nar;
    pfr::launch_usolve2(s->P, s->d_level_fronts + s->level_ptr[l], nf, solve_W(s, l, nf), small, ngroups, s->F, s->Fc,
                        s->Y, s->X, s->d_reach[0], fwd_all ? nullptr : s->d_reach[1], s->Y2, s->XA, s->d_reach[1], st,
                        nar ? std::max(2, solve_split(s, nf)) : solve_split(s, nf), nar ? 0 : tiny, nar,
                        s->level_maxns[l], s->us2_rl != 0);
  }
  LAUNCH_TRY();
  return PFR_OK;
}

// Mark the fronts holding the given permuted rows and all their ancestors; upload the flags and
// the marked fronts level by level (level_fronts order kept).
int set_reach(pfr_solver* s, int which, const std::vector<int32_t>& prows) {
  std::vector<int32_t> mark, list;
  pfr::reach_lists(s->front_of_col, s->front_parent, s->level_ptr, s->level_fronts_host, prows, mark, list,
                   s->reach_ptr[which]);
  s->reach_host[which].assign(mark.begin(), mark.end());
  s->fn_ready = false;
  HIP_TRY(hipMemcpy(s->d_reach[which], mark.data(), mark.size() * 4, hipMemcpyHostToDevice));
  if (!list.empty()) HIP_TRY(hipMemcpy(s->d_reach_fronts[which], list.data(), list.size() * 4, hipMemcpyHostToDevice));
  return PFR_OK;
}

// Backward error of the solution X (permuted, frequency-minor) of the original system (which = 0:
// A x = b over the rows, 1: A^T l = g over the columns); mode 0 operator form, 1 explicit batch
// (data, ds, nvalid); rhs as pfr::ResidDesc (0 operator, 1 explicit B, 2 vector G).  Sets the
// chunk's flags and the caller's berr slots (q0 < 0: no berr output).  R != NULL: only the residual
// b - A x is written there (the refinement step), nothing is checked.
void check_solution(pfr_solver* s, int which, int mode, int rhs, const pfr::RhsDesc& rd, const double2* data,
                    int64_t ds, int nvalid, const double2* X, double2* R, int64_t q0, hipStream_t st,
                    const double2* Mu = nullptr, bool check = true, bool contract = false, const int* glist = nullptr) {
  pfr::ResidDesc d;
  d.ptr = which == 0 ? s->d_rptr : s->d_cptr;
  d.idx = which == 0 ? s->d_ridx : s->d_cidx;
  d.nzs = which == 0 ? s->d_rnz : s->d_cnz;
  d.n = s->n;
  d.K = s->K;
  d.M = s->M;
  d.freqs = s->freqs;
  d.data = data;
  d.data_stride = ds;
  d.nvalid = nvalid;
  d.rhsP = rd.rhsP;
  d.beta_re = rd.beta_re;
  d.beta_im = rd.beta_im;
  d.mass_sum = rd.mass_sum;
  d.B = rd.B;
  d.b_stride = rd.b_stride;
  d.perm = s->P.perm;
  d.G = rd.G;
  d.walk = s->d_walk;
  d.glist = glist;
  d.unroll = s->res_unroll;
  if (contract) {
    d.se = s->stiff;
    d.n_stiff = s->n_stiff;
    d.kpart = s->kpart;
  }
  if (R) {   // refinement residual only: no maxima, no flags
    pfr::launch_residual(mode, rhs, d, X, s->Fc, R, nullptr, st);
    return;
  }
  // Mu: the forward walk also accumulates the functional correction's dot products (s->cpart);
  // check = false: only those (no backward error)
  pfr::launch_residual(mode, rhs, d, X, s->Fc, nullptr, check ? s->d_berr_acc : nullptr, st, Mu, Mu ? s->cpart : nullptr);
  if (!check) return;
  pfr::launch_berr_finish(s->d_berr_acc, s->Fc, nvalid, s->check_tol,
                          which == 0 ? PFR_FLAG_BACKWARD_ERROR : PFR_FLAG_BACKWARD_ERROR_ADJ, s->flags,
                          q0 >= 0 ? s->berr_out : nullptr, q0, which, st);
}

// s_{q,k} partials of sum_nz S_k(nz) lam[row] x[col] over the union pattern's distinct entries
// (k_contract_eg, the loss sweep's contraction; no checks)
void contract_rows(pfr_solver* s, const double2* lam, const double2* x, int nv, hipStream_t st) {
  pfr::launch_contract_eg(s->d_uent, s->n_uent, s->d_se, s->n_stiff, lam, x, s->Fc, nv, s->partial, st);
}

}  // namespace

namespace pfr {
void launch_flags_merge(const int* chunk, int nvalid, int* out, hipStream_t st);
// a chunk's frequencies (padded with the last) and its flags cleared, one kernel
void launch_chunk_start(double* freqs, const double* src, int nvalid, int64_t Fc, int* flags, hipStream_t st,
                        double* loss = nullptr, double* w = nullptr, int nw = 0, int* out_flags = nullptr,
                        double* berr = nullptr, int nfreq = 0);
// p[0 .. n) = 0 (complex entries)
void launch_zero(double2* p, int64_t n, hipStream_t st);
}

extern "C" {

const char* pfr_version(void) { return "pfr 0.1.0 (gfx950, frequency-minor multifrontal)"; }
const char* pfr_last_error(void) { return g_last_error.c_str(); }

void pfr_symbolic_options_default(pfr_symbolic_options* o) {
  pfr::SymbolicOptions d;
  o->leaf_size = d.leaf_size;
  o->ordering = d.ordering;
  o->relax_small = d.relax_small;
  o->relax_mid = d.relax_mid;
  o->relax_big = d.relax_big;
  o->zrelax_mid = d.zrelax_mid;
  o->zrelax_big = d.zrelax_big;
  o->symmetric = d.symmetric;
  o->n_last = 0;
  o->last = nullptr;
  o->max_ns = d.max_ns;
  o->md_delta = d.md_delta;
}

int pfr_symbolic_create(int32_t n, int64_t nnz, const int32_t* colptr, const int32_t* rowind,
                        const pfr_symbolic_options* opt, pfr_symbolic** out) {
  if (!out || !colptr || (nnz > 0 && !rowind) || n <= 0 || nnz < 0) return fail(PFR_ERR_ARG, "bad arguments");
  if (nnz > INT32_MAX) return fail(PFR_ERR_ARG, "nnz exceeds int32 (cf. Problem.py:311 TODO)");
  pfr::SymbolicOptions o;
  if (opt) {
    o.leaf_size = opt->leaf_size;
    o.ordering = opt->ordering;
    o.relax_small = opt->relax_small;
    o.relax_mid = opt->relax_mid;
    o.relax_big = opt->relax_big;
    o.zrelax_mid = opt->zrelax_mid;
    o.zrelax_big = opt->zrelax_big;
    o.symmetric = opt->symmetric;
    o.max_ns = opt->max_ns;
    o.md_delta = opt->md_delta;
    if (opt->n_last > 0) {
      if (!opt->last) return fail(PFR_ERR_ARG, "n_last > 0 without last nodes");
      o.last.assign(opt->last, opt->last + opt->n_last);
    }
  }
  auto* sym = new pfr_symbolic();
  if (pfr::analyse(n, nnz, colptr, rowind, o, sym->S) != 0) {
    std::string msg = "symbolic analysis failed: " + sym->S.error;
    delete sym;
    return fail(PFR_ERR_SYMBOLIC, msg);
  }
  *out = sym;
  return PFR_OK;
}

int pfr_symbolic_stats_get(const pfr_symbolic* sym, pfr_symbolic_stats* o) {
  if (!sym || !o) return fail(PFR_ERR_ARG, "null argument");
  const Symbolic& S = sym->S;
  o->n = S.n;
  o->nnz = S.nnz;
  o->n_fronts = (int32_t)S.fronts.size();
  o->n_levels = (int32_t)S.level_ptr.size() - 1;
  o->max_front = S.max_front;
  o->total_rows = S.total_rows;
  o->factor_entries = S.factor_entries;
  o->nnz_lu = S.nnz_lu;
  o->factor_flops = S.factor_flops;
  o->symmetric = S.symmetric;
  o->n_dirichlet = (int32_t)S.dir_p.size();
  o->n_coupling = (int64_t)S.cpl_p.size();
  return PFR_OK;
}

int pfr_symbolic_export(const pfr_symbolic* sym, int32_t what, void* dst, int64_t cap) {
  if (!sym || !dst) return fail(PFR_ERR_ARG, "null argument");
  const Symbolic& S = sym->S;
  const void* src = nullptr;
  int64_t bytes = 0;
  std::vector<int64_t> fr;
  std::vector<int32_t> tmp;
  auto pick = [&](const std::vector<int32_t>& v) {
    src = v.data();
    bytes = (int64_t)v.size() * 4;
  };
  switch (what) {
    case PFR_EXPORT_PERM: pick(S.perm); break;
    case PFR_EXPORT_IPERM: pick(S.iperm); break;
    case PFR_EXPORT_FRONTS:
      for (const Front& f : S.fronts) {
        int64_t v[8] = {f.ns, f.f, f.row0, f.col0, f.parent, f.level, f.off, f.wv};
        fr.insert(fr.end(), v, v + 8);
      }
      src = fr.data();
      bytes = (int64_t)fr.size() * 8;
      break;
    case PFR_EXPORT_IDX: pick(S.idx); break;
    case PFR_EXPORT_RELPOS: pick(S.relpos); break;
    case PFR_EXPORT_ASM_PTR: pick(S.asm_ptr); break;
    case PFR_EXPORT_ASM_COL: pick(S.asm_col); break;
    case PFR_EXPORT_ASM_NZ: pick(S.asm_nz); break;
    case PFR_EXPORT_EA_PTR: pick(S.ea_ptr); break;
    case PFR_EXPORT_EA_SRC: pick(S.ea_src); break;
    case PFR_EXPORT_LEVEL_PTR: pick(S.level_ptr); break;
    case PFR_EXPORT_LEVEL_FRONTS: pick(S.level_fronts); break;
    case PFR_EXPORT_DIRICHLET:
      for (size_t d = 0; d < S.dir_p.size(); ++d) tmp.insert(tmp.end(), {S.dir_p[d], S.dir_nz[d]});
      pick(tmp);
      break;
    case PFR_EXPORT_COUPLING:
      for (size_t c = 0; c < S.cpl_p.size(); ++c) tmp.insert(tmp.end(), {S.cpl_p[c], S.cpl_dir[c], S.cpl_nz[c]});
      pick(tmp);
      break;
    default: return fail(PFR_ERR_ARG, "unknown export id");
  }
  if (bytes > cap) return fail(PFR_ERR_ARG, "destination too small");
  if (bytes) std::memcpy(dst, src, bytes);
  return PFR_OK;
}

void pfr_symbolic_destroy(pfr_symbolic* sym) { delete sym; }

int64_t pfr_solver_workspace_bytes(const pfr_symbolic* sym, int32_t max_batch) {
  if (!sym || max_batch <= 0) return -1;
  return workspace_bytes(sym->S, round64(max_batch));
}

int pfr_solver_create(const pfr_symbolic* sym, const int32_t* colptr, const int32_t* rowind, int32_t device,
                      int32_t max_batch, pfr_solver** out) {
  if (!sym || !out || max_batch <= 0 || !colptr || !rowind) return fail(PFR_ERR_ARG, "bad arguments");
  HIP_TRY(hipSetDevice(device));
  const Symbolic& S = sym->S;
  auto* s = new pfr_solver();
  auto bail = [&](int rc) {
    delete s;
    return rc;
  };
  s->device = device;
  auto knob = [](const char* name, int def, int lo, int hi) {
    const char* e = getenv(name);
    return e ? std::max(lo, std::min(hi, atoi(e))) : def;
  };
  // launch-shape and path knobs (the measured-slower variants of rounds 1-4 are in git history, DESIGN.md
  // section 8): waves per solve / A11 LU workgroup, the small-front paired top-down variant's front limit,
  // the solve update-part split target, the A11 LU in LDS, the functional from the bottom-up passes, the
  // contraction in the forward walk, the cotangent's solve-error scale, the one-wave top-down pass, the
  // Schur block-kernel threshold and the pipelined L21 prefix
  s->solve_wmax = knob("PFR_SOLVE_WMAX", 8, 1, 8);
  s->fac_wmax = knob("PFR_FAC_WMAX", 16, 1, 16);
  s->fac_g_wg = knob("PFR_FAC_G_WG", 0, 0, 1 << 20);
  s->res_unroll = knob("PFR_RES_UNROLL", 8, 4, 8) == 8 ? 8 : 4;
  s->fac_gbig = knob("PFR_FAC_GBIG", 4, 2, 8);
  if (s->fac_gbig != 2 && s->fac_gbig != 8) s->fac_gbig = 4;
  s->fac_g_ns = knob("PFR_FAC_G_NS", 64, 0, 1 << 20);
  s->us2_small = knob("PFR_US2_SMALL", 110, 0, pfr::MAX_FRONT);
  s->split_target = knob("PFR_SOLVE_SPLIT", 256, 0, 1 << 20);
  s->us2_nar = knob("PFR_US2_NAR", 256, 0, 1 << 30);
  s->fac_lds = knob("PFR_FAC_LDS", -1, -1, 64);
  s->fn_dot = knob("PFR_FN_DOT", 1, 0, 1);
  s->contract_walk = knob("PFR_CONTRACT_WALK", 1, 0, 1);
  s->scale_corr = knob("PFR_SCALE_CORR", 1, 0, 1);
  // 8: the bottom two levels at 2,048 frequencies 685 / 612 -> 509 / 489 us (profiles/r04/experiments/us2_tiny_*)
  s->us2_tiny = knob("PFR_US2_TINY", 8, 0, 8);
  // the narrow levels' paired top-down pivot blocks right-looking with prefetched factor entries (k_usolve2_rl)
  s->us2_rl = knob("PFR_US2_RL", 1, 0, 1);
  const int blk_min = knob("PFR_SCHUR_BLK_MIN", 24, 0, pfr::MAX_FRONT);   // update blocks of >= this many rows: block kernel
  pfr::PlanOptions po;
  po.blk_min = blk_min;
  s->n = S.n;
  s->nnz = S.nnz;
  s->Fc = round64(max_batch);
  // the same for the bottom-up chain's pivot blocks (k_lsolve_rl_z), on chunks of up to 1,024 frequencies: 512-
  // frequency sweeps forward solves 1.65 -> 1.33 ms per step, 41.6k against 38.9-39.7k freq-solves/s; on 2,048-
  // frequency chunks 0.37 -> 0.50 ms per sweep (four slices x 128 groups of 16 frequencies each stage the frontal
  // index chains: profiles/EXPERIMENTS.md, round 6)
  s->ls_rl = knob("PFR_LS_RL", s->Fc <= 1024 ? 1 : 0, 0, 1);
  // the pipelined L21 prefix on launches of fewer than 8,000 waves in chunks of <= 1,024 frequencies (the narrow
  // levels of C4's per-rank sweeps: 512 frequencies 35.3-35.7k -> 36.2-36.6k freq-solves/s; 2,048-frequency
  // chunks unchanged, profiles/r04/offdiag_layout/pu3_*)
  s->off_pu_waves = knob("PFR_OFF_PU_WAVES", s->Fc <= 1024 ? 8000 : 0, 0, 1 << 30);
  s->level_ptr = S.level_ptr;
  s->level_maxf = S.level_maxf;
  s->perm = S.perm;
  s->iperm = S.iperm;
  for (int m : S.level_maxf) s->level_W.push_back(pfr::waves_for(m));
  // the launch plan (host, plan.cpp): every record array the kernels gather through, level by level
  pfr::Plan pl;
  std::string perr;
  if (pfr::build_plan(S, po, pl, perr)) return bail(fail(PFR_ERR_ARG, perr));
  s->sym = pl.sym;
  s->level_maxns = pl.level_maxns;
  s->tile_ptr = pl.tile_ptr;
  s->blk_ptr = pl.blk_ptr;
  s->asm_ptr = pl.asm_ptr;
  s->item_ptr = pl.item_ptr;
  s->lev_bytes = pl.lev_bytes;
  // PFR_FRONT0=0: level 0 through the four class kernels instead of the fused k_front0 (tests/test_gpu_bitwise.py
  // checks the two give the same factors bit for bit)
  s->fused0 = pl.fused0 && knob("PFR_FRONT0", 1, 0, 1);
  // PFR_GRAPH=1: repeated sweeps captured into and replayed from a hipGraph (off by default: bitwise the same
  // results and the host's enqueue of a 512-frequency sweep 427 -> 75 us, but 512 frequencies within the spread
  // and 4,096 frequencies 1 % slower on the device, 67.0-67.6k -> 66.5-66.8k, gpurun_out/r6r_e4096)
  s->graph_mode = knob("PFR_GRAPH", 0, 0, 1);
  s->n_f0 = (int)pl.f0_front.size();
  s->f0_small = pl.f0_small;
  Front* d_fronts = nullptr;
  int rc = PFR_OK;
  std::vector<Front> fv(S.fronts);
  if ((rc = s->up(&d_fronts, fv))) return bail(rc);
  int32_t *idx, *relpos, *rowf, *ap, *ac, *an, *ep, *es, *pm, *pr, *pc;
  if ((rc = s->up(&idx, S.idx)) || (rc = s->up(&relpos, S.relpos)) || (rc = s->up(&rowf, S.row_front)) ||
      (rc = s->up(&ap, S.asm_ptr)) || (rc = s->up(&ac, S.asm_col)) || (rc = s->up(&an, S.asm_nz)) ||
      (rc = s->up(&ep, S.ea_ptr)) || (rc = s->up(&es, S.ea_src)) || (rc = s->up(&pm, S.perm)) ||
      (rc = s->up(&pr, S.prow)) || (rc = s->up(&pc, S.pcol)) || (rc = s->up(&s->d_level_fronts, S.level_fronts)))
    return bail(rc);
  const pfr::I2 z2{0, 0}, n2{-1, -1};
  const pfr::I4 z4{0, 0, 0, 0}, n4{-1, -1, -1, -1};
  if ((rc = s->up_rec(&s->d_tiles, pl.tiles, z4)) || (rc = s->up(&s->d_g1, pl.g1)) || (rc = s->up(&s->d_gxp, pl.gxp)) ||
      (rc = s->up_rec(&s->d_gx, pl.gx, z2)) || (rc = s->up_rec(&s->d_blocks, pl.blocks, z4)) ||
      (rc = s->up_rec(&s->d_bg1, pl.bg1, -1)) || (rc = s->up(&s->d_bgxp, pl.bgxp)) || (rc = s->up_rec(&s->d_bgx, pl.bgx, z2)) ||
      (rc = s->up_rec(&s->d_asm, pl.asm_rec, n4)) || (rc = s->up(&s->d_asm_xp, pl.asm_xp)) ||
      (rc = s->up_rec(&s->d_asm_x, pl.asm_x, z2)) || (rc = s->up_rec(&s->d_items, pl.items, z4)) ||
      (rc = s->up_rec(&s->d_orec, pl.orec, n2)) || (rc = s->up(&s->d_oxp, pl.oxp)) || (rc = s->up_rec(&s->d_ox, pl.ox, z2)))
    return bail(rc);
  if (s->fused0 && ((rc = s->up(&s->d_f0_front, pl.f0_front)) || (rc = s->up(&s->d_f0_ptr, pl.f0_ptr)) ||
                    (rc = s->up(&s->d_f0_nz, pl.f0_nz))))
    return bail(rc);
  std::vector<int32_t> cp(colptr, colptr + S.n + 1), ri(rowind, rowind + S.nnz);
  if ((rc = s->up(&s->d_colptr, cp)) || (rc = s->up(&s->d_rowind, ri))) return bail(rc);
  if (s->sym && !S.dir_p.empty()) {
    s->n_dir = pl.n_dir;
    s->n_crow = pl.n_crow;
    if ((rc = s->up_rec(&s->d_dir, pl.dir, z2)) || (rc = s->up_rec(&s->d_crow, pl.crow, 0)) ||
        (rc = s->up(&s->d_cptr_dir, pl.cptr_dir)) || (rc = s->up_rec(&s->d_ce, pl.ce, z2)) ||
        (rc = s->up(&s->d_dptr, pl.dptr)) || (rc = s->up_rec(&s->d_de, pl.de, z2)) || (rc = s->up(&s->d_cslot, pl.cslot)) ||
        (rc = s->alloc(&s->Bc, pfr::workspace(S, s->Fc, s->n_crow).Bc)))
      return bail(rc);
  }
  if ((rc = s->up(&s->d_rptr, pl.rptr)) || (rc = s->up(&s->d_ridx, pl.ridx)) || (rc = s->up(&s->d_rnz, pl.rnz)) ||
      (rc = s->up(&s->d_cptr, pl.cptr)) || (rc = s->up(&s->d_cidx, pl.cidx)) || (rc = s->up(&s->d_cnz, pl.cnz)) ||
      (rc = s->up(&s->d_walk, S.iperm)) || (rc = s->up_rec(&s->d_uent, pl.uent, n4)))
    return bail(rc);
  s->n_uent = pl.n_uent;
  s->P = DevPattern{d_fronts, idx, relpos, rowf, ap, ac, an, ep, es, pm, pr, pc, S.n};
  {
    const int nf = (int)S.fronts.size();
    s->front_of_col.assign(S.n, -1);
    s->front_parent.resize(nf);
    for (int t = 0; t < nf; ++t) {
      const Front& F = S.fronts[t];
      s->front_parent[t] = F.parent;
      s->front_ns.push_back(F.ns);
      s->front_f.push_back(F.f);
      s->front_off.push_back((int32_t)F.off);
      s->front_col0.push_back(F.col0);
      for (int a = 0; a < F.ns; ++a) s->front_of_col[F.col0 + a] = t;
    }
    s->level_fronts_host = S.level_fronts;
    for (int w = 0; w < 2; ++w) {
      if ((rc = s->alloc(&s->d_reach[w], nf)) || (rc = s->alloc(&s->d_reach_fronts[w], nf))) return bail(rc);
      if ((rc = set_reach(s, w, {}))) return bail(rc);
    }
  }
  const int64_t Fc = s->Fc;
  s->ws = pfr::workspace(S, Fc, s->n_crow);
  if ((rc = s->alloc(&s->F, s->ws.F)) || (rc = s->alloc(&s->WV, s->ws.WV)) ||
      (rc = s->alloc(&s->X, (int64_t)S.n * Fc)) || (rc = s->alloc(&s->Y, (int64_t)S.n * Fc)) ||
      (rc = s->alloc(&s->XA, (int64_t)S.n * Fc)) || (rc = s->alloc(&s->G, (int64_t)S.n * Fc)) ||
      (rc = s->alloc(&s->Y2, (int64_t)S.n * Fc)) || (rc = s->alloc(&s->XR, (int64_t)S.n * Fc)) ||
      (rc = s->alloc(&s->freqs, Fc)) || (rc = s->alloc(&s->loss_terms, Fc)) || (rc = s->alloc(&s->flags, Fc)) ||
      (rc = s->alloc(&s->tq, Fc)) || (rc = s->alloc(&s->d_berr_acc, 2 * Fc)) || (rc = s->alloc(&s->fr0, Fc)) ||
      (rc = s->alloc(&s->mscale, Fc)) || (rc = s->alloc(&s->cpart, s->ws.cpart)) ||
      (rc = s->alloc(&s->gind, Fc / 64)) || (rc = s->alloc(&s->glist, pfr::REFINE_CAP)))
    return bail(rc);
  HIP_TRY(hipMemset(s->d_berr_acc, 0, 2 * Fc * sizeof(double)));
  *out = s;
  return PFR_OK;
}

void pfr_solver_destroy(pfr_solver* s) {
  if (!s) return;
  (void)hipSetDevice(s->device);
  (void)hipDeviceSynchronize();
  delete s;
}

int32_t pfr_solver_max_batch(const pfr_solver* s) { return s ? (int32_t)s->Fc : 0; }

int pfr_set_timing(pfr_solver* s, int32_t enable) {
  if (!s) return fail(PFR_ERR_ARG, "null solver");
  ++s->gen;
  s->timing = enable == 0 ? 0 : (enable | 1);
  return PFR_OK;
}

int pfr_debug_solution(pfr_solver* s, int32_t which, int32_t q, double* out) {
  if (!s || !out || which < 0 || which > 1 || q < 0 || q >= s->Fc) return fail(PFR_ERR_ARG, "bad debug arguments");
  HIP_TRY(hipSetDevice(s->device));
  HIP_TRY(hipDeviceSynchronize());
  std::vector<double2> col((size_t)s->n);
  const double2* src = which == 0 ? s->X : s->XA;
  HIP_TRY(hipMemcpy2D(col.data(), sizeof(double2), src + q, (size_t)s->Fc * sizeof(double2), sizeof(double2), s->n,
                      hipMemcpyDeviceToHost));
  for (int p = 0; p < s->n; ++p) {       // permuted row p holds caller row perm[p]
    out[2 * (int64_t)s->perm[p]] = col[p].x;
    out[2 * (int64_t)s->perm[p] + 1] = col[p].y;
  }
  return PFR_OK;
}

int pfr_set_refine_tol(pfr_solver* s, double tol) {
  if (!s || !(tol >= 0.0)) return fail(PFR_ERR_ARG, "bad refine tolerance");
  ++s->gen;
  s->refine_tol = tol;
  return PFR_OK;
}

int pfr_set_check(pfr_solver* s, int32_t mode, double tol, double* berr_dev) {
  if (!s || mode < 0 || mode > 31 || !(tol >= 0.0)) return fail(PFR_ERR_ARG, "bad check arguments");
  s->check_mode = mode;
  s->check_tol = tol;
  s->berr_out = berr_dev;
  return PFR_OK;
}

int pfr_last_timings(const pfr_solver* s, double* ms) {
  if (!s || !ms) return fail(PFR_ERR_ARG, "null argument");
  for (int i = 0; i < 5; ++i) ms[i] = 0.0;
  if (s->n_tev > 0) HIP_TRY(hipEventSynchronize(s->tev[s->n_tev - 1].ev[5]));
  for (int c = 0; c < s->n_tev; ++c)
    for (int i = 0; i < 5; ++i)
      if (s->tev[c].used[i]) {
        float m = 0;
        HIP_TRY(hipEventElapsedTime(&m, s->tev[c].ev[i], s->tev[c].ev[i + 1]));
        ms[i] += m;
      }
  return PFR_OK;
}

int pfr_last_kernel_timings(const pfr_solver* s, double* ms, int64_t* launches) {
  if (!s || !ms) return fail(PFR_ERR_ARG, "null argument");
  for (int i = 0; i < pfr::NKC; ++i) {
    ms[i] = 0.0;
    if (launches) launches[i] = 0;
  }
  if (!(s->timing & 2) || s->n_tev == 0) return PFR_OK;
  HIP_TRY(hipEventSynchronize(s->tev[s->n_tev - 1].ev[5]));
  const int L = (int)s->level_ptr.size() - 1;
  for (int c = 0; c < s->n_tev; ++c) {
    if (!s->tev[c].used[0]) continue;
    for (int l = 0; l < L; ++l) {
      int work[pfr::NKC] = {s->asm_ptr[l + 1] - s->asm_ptr[l], s->level_ptr[l + 1] - s->level_ptr[l],
                            s->item_ptr[l + 1] - s->item_ptr[l], s->blk_ptr[l + 1] - s->blk_ptr[l],
                            s->tile_ptr[l + 1] - s->tile_ptr[l]};
      if (l == 0 && s->tev[c].f0) {   // the fused bottom level: one or two k_front0 launches, all in class 0
        work[0] = (s->f0_small > 0) + (s->n_f0 > s->f0_small);
        for (int k = 1; k < pfr::NKC; ++k) work[k] = 0;
      }
      for (int k = 0; k < pfr::NKC; ++k) {
        float m = 0;
        HIP_TRY(hipEventElapsedTime(&m, s->tev[c].kev[(pfr::NKC + 1) * l + k], s->tev[c].kev[(pfr::NKC + 1) * l + k + 1]));
        ms[k] += m;
        if (launches) launches[k] += l == 0 && s->tev[c].f0 ? work[k] : work[k] > 0;   // empty classes launch nothing
      }
    }
  }
  return PFR_OK;
}

int pfr_solver_alg_bytes(const pfr_solver* s, int64_t* bytes) {
  if (!s || !bytes) return fail(PFR_ERR_ARG, "null argument");
  for (int i = 0; i < pfr::NKC; ++i) bytes[i] = 0;
  for (int l = 0; l + 1 < (int)s->level_ptr.size(); ++l)
    for (int i = 0; i < pfr::NKC; ++i) bytes[i] += s->lev_bytes[l][i];
  return PFR_OK;
}

int pfr_solver_solve_bytes(const pfr_solver* s, int64_t* bytes) {
  if (!s || !bytes) return fail(PFR_ERR_ARG, "null argument");
  // factor entries each pass reads once: lower[w] = L11 + L21 of the fronts reach w holds (the
  // bottom-up pass of rhs w), upper_r[w] = U11 + U12 of those fronts, upper / lower_all = every front
  int64_t lower[2] = {0, 0}, upper_r[2] = {0, 0}, upper = 0, lower_all = 0, lower_union = 0, sup_rows = 0;
  for (size_t t = 0; t < s->front_ns.size(); ++t) {
    const int64_t ns = s->front_ns[t], r = s->front_f[t] - ns;
    const int64_t u = ns * (ns + 1) / 2 + r * ns;             // U11 + U12 (symmetric: diag(U) L^T)
    const int64_t l = ns * (ns - 1) / 2 + r * ns;             // L11 (unit diagonal) + L21
    upper += u;
    lower_all += l;
    if (s->reach_host[0][t] || s->reach_host[1][t]) lower_union += l;
    if (s->reach_host[1][t]) sup_rows += ns;
    for (int w = 0; w < 2; ++w)
      if (s->reach_host[w][t]) {
        lower[w] += l;
        upper_r[w] += u;
      }
  }
  const int64_t vec = 2 * 16 * (int64_t)s->n;                 // rhs in, solution out
  const bool refine = (s->check_mode & PFR_CHECK_REFINE) != 0;
  if (s->sym && !refine && s->fn_dot) {
    // loss sweep, functional from the bottom-up passes: ONE bottom-up chain over the rhs reach and the
    // support reach together (the support's three vectors share each L value of their fronts) + the
    // paired top-down pass over every front (each U value once for the adjoint and the forward solution)
    bytes[0] = 16 * lower_union + vec + 3 * 32 * sup_rows;
    bytes[1] = 16 * upper + 2 * vec;
  } else if (s->sym && !refine) {
    // loss sweep, paired: forward bottom-up over its reach + forward top-down over the fronts the loss
    // support reaches; adjoint bottom-up over that reach + ONE top-down pass over every front that
    // forms the adjoint and the rest of the forward solution together (each U value loaded once)
    bytes[0] = 16 * (lower[0] + upper_r[1]) + vec;
    bytes[1] = 16 * (lower[1] + upper) + 2 * vec;
  } else {
    // forward and adjoint solved one after the other; a refinement step adds a full pair each
    const int64_t ref = refine ? 16 * (lower_all + upper) + vec : 0;
    bytes[0] = 16 * (lower[0] + upper) + vec + ref;
    bytes[1] = 16 * (lower[1] + upper) + vec + ref;
  }
  return PFR_OK;
}

int pfr_set_stiffness(pfr_solver* s, int32_t n_stiff, const double* stiff_dev, const double* w) {
  if (!s || (n_stiff != 12 && n_stiff != 18) || !stiff_dev || !w)
    return fail(PFR_ERR_ARG, "bad stiffness arguments (n_stiff must be 12 or 18)");
  ++s->gen;
  s->stiff = stiff_dev;
  s->n_stiff = n_stiff;
  std::memset(&s->e, 0, sizeof(s->e));
  for (int k = 0; k < n_stiff; ++k) s->e.re[k] = w[k];
  HIP_TRY(hipSetDevice(s->device));
  if (!s->partial) {
    // written by k_contract_eg (contract_eg_parts(n_uent) parts) and by k_reduce_q (one part per 64-frequency
    // tile of the chunk: Fc / 64), 18 partials each
    const int64_t parts = std::max<int64_t>(pfr::contract_eg_parts(s->n_uent), s->Fc / 64);
    int rc = s->alloc(&s->partial, parts * 18);
    if (rc) return rc;
  }
  if (!s->d_se) {
    int rc = s->alloc(&s->d_se, (int64_t)18 * (s->n_uent + 4));
    if (rc) return rc;
  }
  // the entry-ordered copy of S the gradient contraction reads (taken now: a later change of the
  // registered buffer needs another pfr_set_stiffness, include/pfr.h)
  pfr::launch_gather_entries(s->d_uent, s->n_uent + 4, stiff_dev, n_stiff, s->d_se, nullptr);
  HIP_TRY(hipStreamSynchronize(nullptr));
  return PFR_OK;
}

int pfr_combine(pfr_solver* s, const double* coef, double* K_out, void* stream) {
  if (!s || !coef || !K_out) return fail(PFR_ERR_ARG, "null argument");
  if (!s->stiff) return fail(PFR_ERR_STATE, "pfr_set_stiffness not called");
  HIP_TRY(hipSetDevice(s->device));
  pfr::CoefPack c{};
  for (int k = 0; k < s->n_stiff; ++k) {
    c.re[k] = coef[2 * k];
    c.im[k] = coef[2 * k + 1];
  }
  pfr::launch_combine(s->stiff, s->n_stiff, s->nnz, c, reinterpret_cast<double2*>(K_out), (hipStream_t)stream);
  LAUNCH_TRY();
  return PFR_OK;
}

int pfr_set_operator(pfr_solver* s, const double* K_dev, const double* M_dev) {
  if (!s || !K_dev || !M_dev) return fail(PFR_ERR_ARG, "null argument");
  ++s->gen;
  s->K = reinterpret_cast<const double2*>(K_dev);
  s->M = M_dev;
  return PFR_OK;
}

int pfr_set_rhs(pfr_solver* s, const double* rhs, double beta_re, double beta_im, double mass_sum) {
  if (!s || !rhs) return fail(PFR_ERR_ARG, "null argument");
  ++s->gen;
  s->beta_re = beta_re;
  s->beta_im = beta_im;
  s->mass_sum = mass_sum;
  // the Dirichlet vector rarely changes (only the scale does, per theta): upload it
  // only when it differs from the last one (no device allocation per call)
  if (s->has_rhs && std::equal(s->rhs_host.begin(), s->rhs_host.end(), rhs)) return PFR_OK;
  HIP_TRY(hipSetDevice(s->device));
  std::vector<double> rp(s->n);
  std::vector<int32_t> sup;
  std::vector<double> val;
  for (int p = 0; p < s->n; ++p) {
    rp[p] = rhs[s->perm[p]];
    if (rp[p] != 0.0) {
      sup.push_back(p);
      val.push_back(rp[p]);
    }
  }
  int rc;
  if (!s->rhsP) {
    if ((rc = s->alloc(&s->rhsP, s->n)) || (rc = s->alloc(&s->rhs_sup, s->n)) || (rc = s->alloc(&s->rhs_val, s->n)))
      return rc;
  }
  HIP_TRY(hipMemcpy(s->rhsP, rp.data(), s->n * 8, hipMemcpyHostToDevice));
  if (!sup.empty()) {
    HIP_TRY(hipMemcpy(s->rhs_sup, sup.data(), sup.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(s->rhs_val, val.data(), val.size() * 8, hipMemcpyHostToDevice));
  }
  s->n_rhs_sup = (int)sup.size();
  {
    // forward reach: rhs support (+ rows coupled to Dirichlet columns in symmetric mode)
    std::vector<int32_t> rows(sup);
    std::vector<int32_t> crow(std::max(1, s->n_crow));
    if (s->sym && s->n_crow > 0) {
      HIP_TRY(hipMemcpy(crow.data(), s->d_crow, s->n_crow * 4, hipMemcpyDeviceToHost));
      rows.insert(rows.end(), crow.begin(), crow.begin() + s->n_crow);
    }
    if ((rc = set_reach(s, 0, rows))) return rc;
  }
  s->rhs_host.assign(rhs, rhs + s->n);
  s->has_rhs = true;
  return PFR_OK;
}

int pfr_set_functional(pfr_solver* s, int32_t n_support, const int32_t* index, const double* a, double ts) {
  if (!s || n_support <= 0 || !index || !a) return fail(PFR_ERR_ARG, "bad functional arguments");
  ++s->gen;
  HIP_TRY(hipSetDevice(s->device));
  std::vector<int32_t> pidx(n_support);
  for (int i = 0; i < n_support; ++i) {
    if (index[i] < 0 || index[i] >= s->n) return fail(PFR_ERR_ARG, "functional index out of range");
    pidx[i] = s->iperm[index[i]];
  }
  std::vector<double> av(a, a + 3 * (int64_t)n_support);
  int32_t* d_idx;
  double* d_a;
  int rc;
  if ((rc = s->up(&d_idx, pidx)) || (rc = s->up(&d_a, av))) return rc;
  if ((rc = set_reach(s, 1, pidx))) return rc;        // loss adjoint reach: functional support
  s->a_perm.assign(3 * (size_t)s->n, 0.0);
  for (int k = 0; k < 3; ++k)
    for (int i = 0; i < n_support; ++i) s->a_perm[(size_t)k * s->n + pidx[i]] += av[(size_t)k * n_support + i];
  if (s->d_aP) HIP_TRY(hipMemcpy(s->d_aP, s->a_perm.data(), s->a_perm.size() * 8, hipMemcpyHostToDevice));
  s->fn.n_support = n_support;
  s->fn.pidx = d_idx;
  s->fn.a = d_a;
  s->fn.ts = ts;
  s->has_fn = true;
  return PFR_OK;
}

}  // extern "C"

namespace {
// The launches of one sweep (pfr_sweep after its argument checks), direct or under stream capture.
int sweep_launches(pfr_solver* s, int32_t nfreq, const double* freqs_dev, int32_t loss_type, const double* ref_dev,
                   double scale, double* fr_dev, double* loss_dev, double* w_dev, int32_t* flags_dev, hipStream_t st,
                   bool fresh) {
  const bool reverse = loss_type != PFR_LOSS_NONE;
  reset_timing(s);
  const int64_t Fc = s->Fc;
  const bool refine = (s->check_mode & PFR_CHECK_REFINE) != 0;
  // functional correction: the adjoint of fr is solved in every sweep (in a loss sweep it IS the loss
  // adjoint up to one scalar per frequency) and the forward residual walk adds Re(mu^T r) to fr
  const bool correct = (s->check_mode & PFR_CHECK_CORRECT) != 0;
  const bool adj = reverse || correct;                 // an adjoint solve runs
  const bool paired = s->sym && adj && !refine;        // one top-down pass for both solutions
  const bool fwd_late = paired || correct;             // forward residual walk after the adjoint
  const bool fn_fast = paired && s->fn_dot;            // functional from the bottom-up passes
  if (fn_fast)
    if (int rc0 = fn_setup(s)) return rc0;
  bool used[5] = {true, true, true, adj, adj};
  for (int64_t q0 = 0; q0 < nfreq; q0 += Fc) {
    const int nv = (int)std::min<int64_t>(Fc, nfreq - q0);
    if (fresh && q0 == 0)      // the caller's outputs initialised here (pfr_sweep_fresh)
      pfr::launch_chunk_start(s->freqs, freqs_dev + q0, nv, Fc, s->flags, st, loss_dev, w_dev,
                              reverse && w_dev ? 2 * s->n_stiff : 0, flags_dev, s->berr_out, nfreq);
    else
      pfr::launch_chunk_start(s->freqs, freqs_dev + q0, nv, Fc, s->flags, st);
    if (int rc0 = begin_chunk(s)) return rc0;
    record(s, 0, st);
    pfr::RhsDesc rd;
    rd.rhsP = s->rhsP;
    rd.beta_re = s->beta_re;
    rd.beta_im = s->beta_im;
    rd.mass_sum = s->mass_sum;
    rd.freqs = s->freqs;
    pfr::RhsDesc rf = rd;
    int rc;
    if (paired) {
      pfr::launch_dirichlet_rhs(0, dir_desc(s), s->n_crow, rd, nullptr, s->Bc, s->Fc, st);
      rf.cslot = s->d_cslot;
      rf.Bc = s->Bc;
      if ((rc = factor_all(s, 0, nullptr, 0, nv, st))) return rc;
      record(s, 1, st);   // the forward bottom-up pass belongs to the solve phases (sptrsv_roofline)
      if (fn_fast) {
        if ((rc = fn_bottom_up(s, s->n_crow > 0 ? 3 : 0, rf, st))) return rc;
      } else if ((rc = solve_all(s, 0, s->n_crow > 0 ? 3 : 0, rf, nullptr, s->Y, st, 0))) {
        return rc;
      }
    } else {
      rc = factor_all(s, 0, nullptr, 0, nv, st);
      if (rc) return rc;
      record(s, 1, st);
    }
    // symmetric mode with an adjoint: forward top-down only over the loss support's fronts, then one
    // combined top-down pass (sym_top_down_pair); otherwise the full forward solve first
    if (paired) {
      if (!fn_fast && (rc = sym_top_down_support(s, rf, st))) return rc;
    } else {
      if ((rc = forward_solve(s, 0, rd, s->X, st, 0))) return rc;
      if (refine) {
        // one refinement step on the same factors: r = b - A x (into G), A d = r (into XA), x += d
        check_solution(s, 0, 0, 0, rd, nullptr, 0, nv, s->X, s->G, q0, st);
        pfr::RhsDesc rr;
        rr.G = s->G;
        if ((rc = forward_solve(s, 2, rr, s->XA, st))) return rc;
        pfr::launch_axpy_vec(s->X, s->XA, (int64_t)s->n * Fc, st);
      }
      if (!fwd_late && (s->check_mode & PFR_CHECK_FORWARD))
        check_solution(s, 0, 0, 0, rd, nullptr, 0, nv, s->X, nullptr, q0, st);
    }
    record(s, 2, st);
    pfr::FunctionalArgs fa = s->fn;
    fa.loss_type = reverse ? loss_type : -1;
    fa.ref = reinterpret_cast<const double2*>(ref_dev);
    fa.scale = scale;
    if (adj) pfr::launch_zero(s->G, (int64_t)s->n * Fc, st);
    if (fn_fast) {
      const double2* Yk[3] = {s->Y2, s->YVk, s->YVk + (int64_t)s->n * Fc};
      pfr::launch_fn_dot(s->d_fn_rows, s->n_fn_rows, s->F, s->Y, Yk, Fc, s->fn_parts, st);
      pfr::FunctionalArgs fs = fa;
      if (correct) fs.fr0 = s->fr0;
      pfr::launch_functional_fn(fs, s->fn_parts, Fc, nv, q0, correct ? nullptr : fr_dev, correct ? nullptr : s->loss_terms,
                                s->G, s->fcoef, st);
    } else if (correct) {
      pfr::FunctionalArgs fs = fa;
      fs.fr0 = s->fr0;          // seed: fr of this solve kept, G = d fr / d x
      pfr::launch_functional(fs, s->X, Fc, nv, q0, nullptr, nullptr, s->G, st);
    } else {
      pfr::launch_functional(fa, s->X, Fc, nv, q0, fr_dev, s->loss_terms, s->G, st);
    }
    record(s, 3, st);
    if (adj) {
      pfr::RhsDesc rg;
      rg.G = s->G;
      if (fn_fast) {
        double2* Yk[3] = {s->Y2, s->YVk, s->YVk + (int64_t)s->n * Fc};
        pfr::launch_fn_combine(s->d_sup_rows, s->n_sup_rows, s->fcoef, Yk, Fc, st);
        if ((rc = sym_top_down_pair(s, st, true))) return rc;
        pfr::launch_dirichlet_post(dir_desc(s), s->n_dir, s->XA, s->Fc, st);
        if (correct) {
          // the correction fr(x) + Re(mu^T r) needs fr OF the solution x whose residual r is walked (the
          // dot product's fr has its own rounding error, which the correction does not see): fr0 from x
          pfr::FunctionalArgs fs = fa;
          fs.fr0 = s->fr0;
          pfr::launch_functional(fs, s->X, Fc, nv, q0, nullptr, nullptr, nullptr, st);
        }
      } else if (paired) {
        if ((rc = solve_all(s, 0, 2, rg, nullptr, s->Y2, st, 1)) || (rc = sym_top_down_pair(s, st))) return rc;
        pfr::launch_dirichlet_post(dir_desc(s), s->n_dir, s->XA, s->Fc, st);
      } else {
        if ((rc = adjoint_solve(s, rg, s->XA, st, 1))) return rc;
        if (refine) {
          // l += A^{-T} (g - A^T l): residual into Y2, correction into XR
          check_solution(s, 1, 0, 2, rg, nullptr, 0, nv, s->XA, s->Y2, q0, st);
          pfr::RhsDesc rr;
          rr.G = s->Y2;
          if ((rc = adjoint_solve(s, rr, s->XR, st))) return rc;
          pfr::launch_axpy_vec(s->XA, s->XR, (int64_t)s->n * Fc, st);
        }
      }
      record(s, 4, st);
      bool want_f = fwd_late && (s->check_mode & PFR_CHECK_FORWARD);
      bool want_a = (s->check_mode & PFR_CHECK_ADJOINT) != 0;
      // the gradient contraction rides on the forward residual walk (loss sweeps with the correction)
      const bool cwalk = reverse && correct && s->contract_walk &&
                         (s->n_stiff == 12 || s->n_stiff == 18);
      if (cwalk && !s->kpart) {
        if ((rc = s->alloc(&s->kpart, s->ws.kpart))) return rc;
      }
      // selective adjoint refinement (PFR_CHECK_REFINE_ADJ): the groups next to a resonance, where the unrefined
      // solves' first-order error dominates the gradient, get one refinement step of mu
      const bool refine_adj = reverse && correct && cwalk && fn_fast && (s->check_mode & PFR_CHECK_REFINE_ADJ);
      // the solve-error scale of the cotangent (k_correct_finish): t_q = mu^T rhsP in, m_q t_q out
      const bool scorr = reverse && correct && s->scale_corr;
      pfr::RhsScale bsc;
      bsc.freqs = s->freqs;
      bsc.mass_sum = s->mass_sum;
      bsc.beta_re = s->beta_re;
      bsc.beta_im = s->beta_im;
      if (correct) {
        // the forward residual walk: backward error (when checked) + the correction's dot products,
        // then the corrected fr, its loss terms and the per-frequency cotangent scales
        check_solution(s, 0, 0, 0, rd, nullptr, 0, nv, s->X, nullptr, q0, st, s->XA, want_f, cwalk);
        want_f = false;
        if (scorr) pfr::launch_rhs_dot(s->rhs_sup, s->rhs_val, s->n_rhs_sup, s->XA, Fc, s->tq, st);
        pfr::launch_correct_finish(fa, s->fr0, s->cpart, pfr::residual_parts(s->n), Fc, nv, q0, fr_dev, s->loss_terms,
                                   s->mscale, st, refine_adj ? s->gind : nullptr, scorr ? s->tq : nullptr, bsc);
      }
      if (refine_adj) {
        // the listed groups (largest first-order fr error estimates above the tolerance, at most REFINE_CAP):
        // mu += A^-T (G - A^T mu) with the fr seed G = d fr / d x of THIS x (k_functional seed mode; the adjoint
        // was solved for the seed of the bottom-up dot products, whose rounding differs), then their correction
        // dot products and gradient contraction again with the refined mu, and their fr / m_q
        pfr::launch_select_groups(s->gind, (int)(Fc / 64), s->refine_tol, s->glist, st);
        if (!s->Gx) {
          if ((rc = s->alloc(&s->Gx, s->ws.nvec))) return rc;
          HIP_TRY(hipMemsetAsync(s->Gx, 0, (size_t)s->n * Fc * 16, st));   // only the support rows are ever written
        }
        pfr::FunctionalArgs fs = fa;
        fs.fr0 = s->fr0;
        pfr::launch_functional(fs, s->X, Fc, nv, q0, nullptr, nullptr, s->Gx, st);
        pfr::RhsDesc rgx;
        rgx.G = s->Gx;
        check_solution(s, 1, 0, 2, rgx, nullptr, 0, nv, s->XA, s->XR, q0, st, nullptr, false, false, s->glist);
        pfr::RhsDesc rr;
        rr.G = s->XR;
        if ((rc = adjoint_solve(s, rr, s->Y2, st, -1, s->glist))) return rc;
        pfr::launch_axpy_vec(s->XA, s->Y2, (int64_t)s->n * Fc, st, s->glist, Fc);
        check_solution(s, 0, 0, 0, rd, nullptr, 0, nv, s->X, nullptr, q0, st, s->XA, false, true, s->glist);
        if (scorr) pfr::launch_rhs_dot(s->rhs_sup, s->rhs_val, s->n_rhs_sup, s->XA, Fc, s->tq, st);
        pfr::launch_correct_finish(fa, s->fr0, s->cpart, pfr::residual_parts(s->n), Fc, nv, q0, fr_dev, s->loss_terms,
                                   s->mscale, st, nullptr, scorr ? s->tq : nullptr, bsc);
      }
      const double2* msc = correct ? s->mscale : nullptr;
      if (cwalk)
        pfr::launch_reduce_q(s->kpart, pfr::residual_parts(s->n), s->n_stiff, msc, nv, Fc, s->partial, st);
      else if (reverse)
        pfr::launch_contract_eg(s->d_uent, s->n_uent, s->d_se, s->n_stiff, s->XA, s->X, Fc, nv, s->partial, st, msc);
      // the checks as row / column walks of the original pattern (k_residual)
      if (want_f) check_solution(s, 0, 0, 0, rd, nullptr, 0, nv, s->X, nullptr, q0, st);
      if (want_a) check_solution(s, 1, 0, 2, rg, nullptr, 0, nv, s->XA, nullptr, q0, st);
      if (reverse) {
        if (!scorr) pfr::launch_rhs_dot(s->rhs_sup, s->rhs_val, s->n_rhs_sup, s->XA, Fc, s->tq, st, msc);
        pfr::launch_reduce(s->partial, cwalk ? (int)(Fc / 64) : pfr::contract_eg_parts(s->n_uent), s->n_stiff, s->tq, s->e,
                           s->loss_terms, nv, Fc, reinterpret_cast<double2*>(w_dev), loss_dev, st);
      }
    } else {
      record(s, 4, st);
    }
    record(s, 5, st);
    if (flags_dev) pfr::launch_flags_merge(s->flags, nv, flags_dev + q0, st);
    LAUNCH_TRY();
    if ((rc = finish_timing(s, used))) return rc;
  }
  return PFR_OK;
}

template <class T>
uint64_t key_bits(T v) {
  uint64_t b = 0;
  static_assert(sizeof(T) <= sizeof(b), "key word");
  std::memcpy(&b, &v, sizeof(T));
  return b;
}
}  // namespace

extern "C" {

namespace {
int sweep_impl(pfr_solver* s, int32_t nfreq, const double* freqs_dev, int32_t loss_type, const double* ref_dev,
               double scale, double* fr_dev, double* loss_dev, double* w_dev, int32_t* flags_dev, void* stream,
               bool fresh) {
  if (!s || nfreq <= 0 || !freqs_dev) return fail(PFR_ERR_ARG, "bad sweep arguments");
  if (!s->K || !s->M) return fail(PFR_ERR_STATE, "operator not set (pfr_set_operator)");
  if (!s->has_rhs) return fail(PFR_ERR_STATE, "rhs not set (pfr_set_rhs)");
  if (!s->has_fn) return fail(PFR_ERR_STATE, "functional not set (pfr_set_functional)");
  const bool reverse = loss_type != PFR_LOSS_NONE;
  if (reverse && (loss_type < 0 || loss_type > PFR_LOSS_COTANGENT || !ref_dev))
    return fail(PFR_ERR_ARG, "bad loss type / missing ref");
  if (reverse && (!s->stiff || !w_dev)) return fail(PFR_ERR_STATE, "reverse pass needs pfr_set_stiffness and w_dev");
  HIP_TRY(hipSetDevice(s->device));
  hipStream_t st = (hipStream_t)stream;
  auto direct = [&] { return sweep_launches(s, nfreq, freqs_dev, loss_type, ref_dev, scale, fr_dev, loss_dev, w_dev,
                                            flags_dev, st, fresh); };
  // per-launch timing events are host work between the launches: never under a graph
  if (!s->graph_mode || s->graph_off || s->timing) return direct();
  const std::array<uint64_t, 14> key = {s->gen * 2 + (fresh ? 1 : 0), key_bits(s->check_mode), key_bits(s->check_tol),
                                        key_bits(s->berr_out),
                                        key_bits(nfreq), key_bits(freqs_dev), key_bits(loss_type), key_bits(ref_dev),
                                        key_bits(scale), key_bits(fr_dev), key_bits(loss_dev), key_bits(w_dev),
                                        key_bits(flags_dev), key_bits(st)};
  if (!s->gkey_valid || key != s->gkey) {
    // a new sweep configuration: run it directly (its first run also makes the lazy allocations and uploads,
    // which a capture must not contain); the same configuration again is captured
    s->drop_graph();
    s->gkey = key;
    s->gkey_valid = true;
    return direct();
  }
  if (!s->gexec) {
    hipGraph_t g = nullptr;
    HIP_TRY(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    const int rc = direct();
    const hipError_t e = hipStreamEndCapture(st, &g);
    hipGraphExec_t x = nullptr;
    if (rc == PFR_OK && e == hipSuccess && g && hipGraphInstantiate(&x, g, nullptr, nullptr, 0) == hipSuccess) {
      s->graph = g;
      s->gexec = x;
    } else {
      // nothing of the captured work ran: no graphs on this solver from now on, and this sweep directly
      if (g) (void)hipGraphDestroy(g);
      (void)hipGetLastError();
      s->graph_off = true;
      return direct();
    }
  }
  HIP_TRY(hipGraphLaunch(s->gexec, st));
  ++s->graph_launches;
  return PFR_OK;
}
}  // namespace

int pfr_sweep(pfr_solver* s, int32_t nfreq, const double* freqs_dev, int32_t loss_type, const double* ref_dev,
              double scale, double* fr_dev, double* loss_dev, double* w_dev, int32_t* flags_dev, void* stream) {
  return sweep_impl(s, nfreq, freqs_dev, loss_type, ref_dev, scale, fr_dev, loss_dev, w_dev, flags_dev, stream, false);
}

int pfr_sweep_fresh(pfr_solver* s, int32_t nfreq, const double* freqs_dev, int32_t loss_type, const double* ref_dev,
                    double scale, double* fr_dev, double* loss_dev, double* w_dev, int32_t* flags_dev, void* stream) {
  return sweep_impl(s, nfreq, freqs_dev, loss_type, ref_dev, scale, fr_dev, loss_dev, w_dev, flags_dev, stream, true);
}

int64_t pfr_sweep_graph_launches(const pfr_solver* s) { return s ? s->graph_launches : 0; }

int pfr_stream_order(void* waiter, void* signaller) {
  // one event per (thread, device), recorded again for every ordering: a wait takes the event's state at the time
  // of the hipStreamWaitEvent call, so a later record does not move an earlier wait
  thread_local std::vector<hipEvent_t> evs;
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  if ((int)evs.size() <= dev) evs.resize(dev + 1, nullptr);
  if (!evs[dev]) HIP_TRY(hipEventCreateWithFlags(&evs[dev], hipEventDisableTiming));
  HIP_TRY(hipEventRecord(evs[dev], (hipStream_t)signaller));
  HIP_TRY(hipStreamWaitEvent((hipStream_t)waiter, evs[dev], 0));
  return PFR_OK;
}

int pfr_hessian_sweep(pfr_solver* s, int32_t nfreq, const double* freqs_dev, int32_t loss_type, const double* ref_dev,
                      double scale, int32_t n_dir, const double* dcoef, double* loss_dev, double* w_dev,
                      double* h_dev, int32_t* flags_dev, void* stream) {
  if (!s || nfreq <= 0 || !freqs_dev || !ref_dev || !w_dev || !h_dev || n_dir <= 0 || !dcoef)
    return fail(PFR_ERR_ARG, "bad hessian sweep arguments");
  ++s->gen;
  if (loss_type < PFR_LOSS_MSE || loss_type > PFR_LOSS_MSE_LOG_AFC)
    return fail(PFR_ERR_ARG, "hessian sweep needs a loss type (MSE, RMSE, MSE_AFC, MSE_LOG_AFC)");
  if (!s->K || !s->M) return fail(PFR_ERR_STATE, "operator not set (pfr_set_operator)");
  if (!s->has_rhs) return fail(PFR_ERR_STATE, "rhs not set (pfr_set_rhs)");
  if (!s->has_fn) return fail(PFR_ERR_STATE, "functional not set (pfr_set_functional)");
  if (!s->stiff) return fail(PFR_ERR_STATE, "pfr_set_stiffness not called");
  HIP_TRY(hipSetDevice(s->device));
  hipStream_t st = (hipStream_t)stream;
  reset_timing(s);
  const int64_t Fc = s->Fc, n = s->n;
  int rc;
  if (!s->DX && ((rc = s->alloc(&s->DX, n * Fc)) || (rc = s->alloc(&s->DL, n * Fc)))) return rc;
  if (s->n_kdir < n_dir) {
    if ((rc = s->alloc(&s->Kdir, (int64_t)n_dir * s->nnz))) return rc;   // previous block stays owned
    s->n_kdir = n_dir;
  }
  // tangent operators dA_i = sum_k dc_ik S_k and right-hand-side weights beta_i = sum_k dc_ik e_k
  std::vector<double2> beta(n_dir);
  pfr::CoefPack zero{};
  for (int i = 0; i < n_dir; ++i) {
    pfr::CoefPack c{};
    double br = 0, bi = 0;
    for (int k = 0; k < s->n_stiff; ++k) {
      c.re[k] = dcoef[2 * (i * s->n_stiff + k)];
      c.im[k] = dcoef[2 * (i * s->n_stiff + k) + 1];
      br += c.re[k] * s->e.re[k];
      bi += c.im[k] * s->e.re[k];
    }
    beta[i] = make_double2(br, bi);
    pfr::launch_combine(s->stiff, s->n_stiff, s->nnz, c, s->Kdir + (int64_t)i * s->nnz, st);
  }
  double2* H = reinterpret_cast<double2*>(h_dev);
  for (int64_t q0 = 0; q0 < nfreq; q0 += Fc) {
    const int nv = (int)std::min<int64_t>(Fc, nfreq - q0);
    pfr::launch_chunk_start(s->freqs, freqs_dev + q0, nv, Fc, s->flags, st);
    if ((rc = factor_all(s, 0, nullptr, 0, nv, st))) return rc;
    // forward solve, loss, adjoint, gradient partials (as pfr_sweep)
    pfr::RhsDesc rd;
    rd.rhsP = s->rhsP;
    rd.beta_re = s->beta_re;
    rd.beta_im = s->beta_im;
    rd.mass_sum = s->mass_sum;
    rd.freqs = s->freqs;
    if ((rc = forward_solve(s, 0, rd, s->X, st, 0))) return rc;
    pfr::FunctionalArgs fa = s->fn;
    fa.loss_type = loss_type;
    fa.ref = reinterpret_cast<const double2*>(ref_dev);
    fa.scale = scale;
    HIP_TRY(hipMemsetAsync(s->G, 0, (size_t)n * Fc * 16, st));
    pfr::RhsDesc rg;
    rg.G = s->G;
    rg.rhsP = s->rhsP;
    rg.freqs = s->freqs;
    if (s->check_mode & PFR_CHECK_CORRECT) {
      // as pfr_sweep: the adjoint of fr, the corrected fr's loss terms and cotangent scales, then
      // lambda = m_q mu in place -- loss and gradient equal the corrected loss sweep's
      pfr::FunctionalArgs fs = fa;
      fs.fr0 = s->fr0;
      pfr::launch_functional(fs, s->X, Fc, nv, q0, nullptr, nullptr, s->G, st);
      if ((rc = adjoint_solve(s, rg, s->XA, st, 1))) return rc;
      check_solution(s, 0, 0, 0, rd, nullptr, 0, nv, s->X, nullptr, q0, st, s->XA, false);
      // the loss sweep's cotangent, solve-error scale included (k_correct_finish): its gradient is the loss sweep's
      pfr::RhsScale bsc;
      bsc.freqs = s->freqs;
      bsc.mass_sum = s->mass_sum;
      bsc.beta_re = s->beta_re;
      bsc.beta_im = s->beta_im;
      if (s->scale_corr) pfr::launch_rhs_dot(s->rhs_sup, s->rhs_val, s->n_rhs_sup, s->XA, Fc, s->tq, st);
      pfr::launch_correct_finish(fa, s->fr0, s->cpart, pfr::residual_parts(s->n), Fc, nv, q0, nullptr, s->loss_terms,
                                 s->mscale, st, nullptr, s->scale_corr ? s->tq : nullptr, bsc);
      pfr::launch_scale_vec(s->XA, s->mscale, s->n, Fc, st);
      // the second-order seeds G (k_functional_tangent) are formed from fa, not the seed mode
    } else {
      pfr::launch_functional(fa, s->X, Fc, nv, q0, nullptr, s->loss_terms, s->G, st);
      if ((rc = adjoint_solve(s, rg, s->XA, st, 1))) return rc;
    }
    contract_rows(s, s->XA, s->X, nv, st);
    pfr::launch_rhs_dot(s->rhs_sup, s->rhs_val, s->n_rhs_sup, s->XA, Fc, s->tq, st);
    pfr::launch_reduce(s->partial, pfr::contract_eg_parts(s->n_uent), s->n_stiff, s->tq, s->e, s->loss_terms, nv, Fc,
                       reinterpret_cast<double2*>(w_dev), loss_dev, st);
    // second order, per direction i (same factors):
    //   A dx_i = db_i - dA_i x ;  A^T dl_i = dG_i(dx_i) - dA_i^T l
    //   h_ki += sum_q [ -dl_i^T S_k x + e_k dl_i^T b0 - l^T S_k dx_i ]
    for (int i = 0; i < n_dir; ++i) {
      const double2* Kd = s->Kdir + (int64_t)i * s->nnz;
      pfr::launch_tangent_spmv(s->d_rptr, s->d_ridx, s->d_rnz, (int)n, Kd, s->X, Fc, s->rhsP, beta[i], s->G, 0, st);
      if ((rc = forward_solve(s, 2, rg, s->DX, st))) return rc;
      HIP_TRY(hipMemsetAsync(s->G, 0, (size_t)n * Fc * 16, st));
      pfr::launch_functional_tangent(fa, s->X, s->DX, Fc, nv, q0, s->G, st);
      pfr::launch_tangent_spmv(s->d_cptr, s->d_cidx, s->d_cnz, (int)n, Kd, s->XA, Fc, nullptr, make_double2(0, 0),
                               s->G, 1, st);
      if ((rc = adjoint_solve(s, rg, s->DL, st))) return rc;
      contract_rows(s, s->DL, s->X, nv, st);
      pfr::launch_rhs_dot(s->rhs_sup, s->rhs_val, s->n_rhs_sup, s->DL, Fc, s->tq, st);
      pfr::launch_reduce(s->partial, pfr::contract_eg_parts(s->n_uent), s->n_stiff, s->tq, s->e, s->loss_terms, nv, Fc,
                         H + (int64_t)i * s->n_stiff, nullptr, st);
      contract_rows(s, s->XA, s->DX, nv, st);
      pfr::launch_reduce(s->partial, pfr::contract_eg_parts(s->n_uent), s->n_stiff, s->tq, zero, s->loss_terms, nv, Fc,
                         H + (int64_t)i * s->n_stiff, nullptr, st);
    }
    if (flags_dev) pfr::launch_flags_merge(s->flags, nv, flags_dev + q0, st);
    LAUNCH_TRY();
  }
  return PFR_OK;
}

int pfr_solve_multi(pfr_solver* s, int32_t batch, int32_t nrhs, const double* data_dev, int64_t data_stride,
                    const double* b_dev, int64_t b_stride, int64_t b_rhs_stride, double* x_dev, int64_t x_rhs_stride,
                    int32_t transpose, int32_t* flags_dev, void* stream) {
  if (!s || batch <= 0 || nrhs <= 0 || !data_dev || !b_dev || !x_dev || data_stride < 0 || b_stride < 0 ||
      b_rhs_stride < 0 || x_rhs_stride < 0)
    return fail(PFR_ERR_ARG, "bad solve arguments");
  ++s->gen;
  if (data_stride != 0 && data_stride < s->nnz) return fail(PFR_ERR_ARG, "data_stride < nnz");
  if (b_stride != 0 && b_stride < s->n) return fail(PFR_ERR_ARG, "b_stride < n");
  if (nrhs > 1 && x_rhs_stride < (int64_t)batch * s->n) return fail(PFR_ERR_ARG, "x_rhs_stride < batch * n");
  if (s->sym)
    return fail(PFR_ERR_STATE, "explicit-matrix solves need a solver on a general analysis (symmetric = 0)");
  HIP_TRY(hipSetDevice(s->device));
  hipStream_t st = (hipStream_t)stream;
  reset_timing(s);
  const int64_t Fc = s->Fc;
  const double2* data = reinterpret_cast<const double2*>(data_dev);
  const double2* B = reinterpret_cast<const double2*>(b_dev);
  double2* Xo = reinterpret_cast<double2*>(x_dev);
  bool used[5] = {true, !transpose, false, (bool)transpose, false};
  for (int64_t q0 = 0; q0 < batch; q0 += Fc) {
    const int nv = (int)std::min<int64_t>(Fc, batch - q0);
    HIP_TRY(hipMemsetAsync(s->flags, 0, Fc * sizeof(int32_t), st));
    if (int rc0 = begin_chunk(s)) return rc0;
    record(s, 0, st);
    // padded lanes repeat the last valid item (stride 0 broadcast handled by the kernel's clamp)
    int rc = factor_all(s, 1, data + q0 * data_stride, data_stride, nv, st);
    if (rc) return rc;
    record(s, 1, st);
    // every right-hand side of the chunk on the same factors (reference mode 4
    // refactorises per right-hand side, InnerState.h:289-305)
    for (int32_t r = 0; r < nrhs; ++r) {
      pfr::RhsDesc rd;
      rd.B = B + r * b_rhs_stride + q0 * b_stride;
      rd.b_stride = b_stride;
      rd.nvalid = nv;
      if (!transpose) {
        if ((rc = solve_all(s, 0, 1, rd, nullptr, s->Y, st))) return rc;
        if ((rc = solve_all(s, 1, 1, rd, s->Y, s->X, st))) return rc;
      }
      if (r == 0) {
        record(s, 2, st);
        record(s, 3, st);
      }
      if (transpose) {
        if ((rc = solve_all(s, 2, 1, rd, nullptr, s->Y, st))) return rc;
        if ((rc = solve_all(s, 3, 1, rd, s->Y, s->X, st))) return rc;
      }
      const int which = transpose ? 1 : 0;
      const double2* dq = data + q0 * data_stride;
      if (s->check_mode & PFR_CHECK_REFINE) {
        // x += A^{-1} (b - A x) (or the transposed system) on the same factors
        check_solution(s, which, 1, 1, rd, dq, data_stride, nv, s->X, s->G, r == 0 ? q0 : -1, st);
        pfr::RhsDesc rr;
        rr.G = s->G;
        if ((rc = solve_all(s, transpose ? 2 : 0, 2, rr, nullptr, s->Y, st))) return rc;
        if ((rc = solve_all(s, transpose ? 3 : 1, 0, rr, s->Y, s->XA, st))) return rc;
        pfr::launch_axpy_vec(s->X, s->XA, (int64_t)s->n * Fc, st);
      }
      if (s->check_mode & (transpose ? PFR_CHECK_ADJOINT : PFR_CHECK_FORWARD))
        check_solution(s, which, 1, 1, rd, dq, data_stride, nv, s->X, nullptr, r == 0 ? q0 : -1, st);
      pfr::launch_unpermute(s->P.perm, s->n, s->X, Fc, nv, Xo + r * x_rhs_stride + q0 * s->n, st);
    }
    record(s, 4, st);
    record(s, 5, st);
    if (flags_dev) pfr::launch_flags_merge(s->flags, nv, flags_dev + q0, st);
    LAUNCH_TRY();
    if ((rc = finish_timing(s, used))) return rc;
  }
  return PFR_OK;
}

int pfr_solve(pfr_solver* s, int32_t batch, const double* data_dev, int64_t data_stride, const double* b_dev,
              int64_t b_stride, double* x_dev, int32_t transpose, int32_t* flags_dev, void* stream) {
  return pfr_solve_multi(s, batch, 1, data_dev, data_stride, b_dev, b_stride, 0, x_dev, 0, transpose, flags_dev,
                         stream);
}

int pfr_matvec(pfr_solver* s, int32_t batch, const double* data_dev, int64_t data_stride, const double* x_dev,
               int64_t x_stride, double* y_dev, int32_t transpose, void* stream) {
  if (!s || batch <= 0 || !data_dev || !x_dev || !y_dev) return fail(PFR_ERR_ARG, "bad matvec arguments");
  ++s->gen;
  HIP_TRY(hipSetDevice(s->device));
  hipStream_t st = (hipStream_t)stream;
  if (!transpose) HIP_TRY(hipMemsetAsync(y_dev, 0, (size_t)batch * s->n * 16, st));
  pfr::launch_matvec(s->d_colptr, s->d_rowind, s->n, reinterpret_cast<const double2*>(data_dev), data_stride,
                     reinterpret_cast<const double2*>(x_dev), x_stride, reinterpret_cast<double2*>(y_dev),
                     transpose, batch, st);
  LAUNCH_TRY();
  return PFR_OK;
}

}  // extern "C"
