// Host-side launch plans of the numeric factorisation and solves: everything libpfr derives from the symbolic
// analysis before any device work -- level tables, gather records of every kernel class, Dirichlet lists,
// compressed rows / columns, the contraction's entry list, reach lists -- and the element counts of every
// device buffer a solver allocates.  HIP-free (plain C++17): pfr_solver_create (api.cpp) uploads a Plan,
// and the sanitizer driver (asan_driver.cpp, tests/test_asan_host.py) builds plans for every engine shape
// under -fsanitize=address,undefined and checks each index a launch will use against the buffer it addresses
// (check_plan).  The launch-geometry functions below are the ones the launchers use (kernels.hip), so the
// checks and the launches cannot drift apart.
#pragma once

#include <algorithm>
#include <array>
#include <cstdint>
#include <string>
#include <vector>

#include "symbolic.hpp"

namespace pfr {

// layouts of HIP's int2 / int4 (device records are uploaded byte for byte)
struct I2 {
  int32_t x, y;
};
struct I4 {
  int32_t x, y, z, w;
};

// ---- kernel shape constants (device_types.hpp / kernels.hip use these)
// Schur super-tile: a wavefront = SCHUR_QG frequencies x (SCHUR_SR x SCHUR_SC) lane groups, each lane group one
// SCHUR_TM x SCHUR_TN register tile.  Lane = frequency, one 4 x 4 tile per wave (measured 10 % faster than 16
// frequencies x a 2 x 2 arrangement of 4 x 4 tiles).
constexpr int SCHUR_SR = 1, SCHUR_SC = 1, SCHUR_QG = 64 / (SCHUR_SR * SCHUR_SC);
constexpr int SCHUR_TM = 4, SCHUR_TN = 4;
static_assert(SCHUR_SR * SCHUR_SC * SCHUR_QG == 64, "one wavefront per super-tile");
constexpr int SCHUR_TILE = SCHUR_TM * SCHUR_TN * SCHUR_SR * SCHUR_SC;   // first-source ids per tile
constexpr int SCHUR_BLK = 16;                 // k_schur_sym_blk block edge (16 waves x 4 x 4 tiles)
constexpr int SCHUR_BLK_IDS = 16 * SCHUR_BLK; // first-source ids per block (wave x position)
// Off-diagonal panel kernel: a wave = OFF_G lane groups of 64 / OFF_G frequencies, OFF_RPL rows (columns) per
// lane.  Lane = frequency, two rows per lane (measured best of 1 / 2 lane groups and 1 / 2 / 4 rows per lane).
constexpr int OFF_G = 1;
constexpr int OFF_RPL = 2;
constexpr int FAC_G = 2;                      // A11 LU: lane groups per wave (64 / FAC_G frequencies each)
constexpr int MAX_FRONT = 1024;               // largest front the solve kernels stage index lists for in LDS
constexpr int NKC = 5;                        // factorisation kernel classes: assembly, A11 LU, L21 rows, Schur
                                              // blocks, Schur tiles
constexpr int FN_PARTS_HOST = 16;             // k_fn_dot partials per frequency group (kernels.hip: FN_PARTS)
constexpr int REFINE_CAP = 4;                 // groups of the selective adjoint refinement per chunk
constexpr int SPLIT_W = 4;                    // waves per workgroup of the split solve update parts
constexpr int CEG_EW = 8;                     // entries per wave of k_contract_eg
constexpr int64_t LDS_BYTES = 160 * 1024;

// ---- launch geometry shared by the launchers and the checks
inline int residual_parts(int n) { return (int)std::min<int64_t>((n + 3) / 4, 256); }   // k_residual grid.x
inline int contract_eg_parts(int nent) { return ((nent + CEG_EW - 1) / CEG_EW + 3) / 4; }   // k_contract_eg grid
// dynamic LDS of k_factor_sym_lds for a level whose largest pivot block is maxns (triangle + 8 W columns)
inline int64_t fac_lds_bytes(int maxns) { return ((int64_t)maxns * (maxns + 1) / 2 + (int64_t)maxns * 8) * 16; }
// k_lsolve_level_z's NAR form: the level's largest pivot block's values in dynamic LDS (ns x 64 x 16 B), beside
// the frontal gather's static index staging (~36 KiB)
constexpr int64_t LS_NAR_DYN_MAX = 112 * 1024;
inline bool ls_nar_fits(int maxns) { return (int64_t)maxns * 64 * 16 <= LS_NAR_DYN_MAX; }
// waves per workgroup for a level whose largest front is maxf
inline int waves_for(int maxf) { return std::max(1, std::min(8, (maxf + 23) / 24)); }
// Workgroups per (front, frequency group) for the update part of a solve launch over nf fronts: 1 when the
// launch already has `target` workgroups, else enough to reach it (at most 16)
inline int solve_split(int64_t nf, int64_t Fc, int target) {
  const int64_t wgs = nf * (Fc / 64);
  if (target <= 0 || wgs <= 0 || wgs >= target) return 1;
  return (int)std::min<int64_t>(16, (target + wgs - 1) / wgs);
}
// Waves per workgroup of a solve launch over nf fronts of a level with size-based count level_w, raised (up to
// wmax) when the launch has too few workgroups to fill the chip
inline int solve_waves(int level_w, int64_t nf, int64_t Fc, int wmax) {
  const int64_t wgs = std::max<int64_t>(1, nf * (Fc / 64));
  const int64_t fill = (4096 + wgs - 1) / wgs;
  return (int)std::max<int64_t>(level_w, std::min<int64_t>(wmax, fill));
}

// The bottom level fused (k_front0): symmetric analyses whose level-0 fronts (leaves) all have at most F0_NS pivots
// and F0_RM update rows -- per (front, frequency) A11, L21 and the update block formed in registers, one pass
constexpr int F0_NS = 4, F0_RM = 10;

struct PlanOptions {
  int blk_min = 24;      // PFR_SCHUR_BLK_MIN: update blocks of at least this many rows through the block kernel
};

struct Plan {
  int L = 0;                             // levels
  bool sym = false;
  std::vector<int32_t> level_maxns;      // largest pivot block per level
  std::vector<char> blk_front;           // front's Schur complement by the block kernel
  // Schur tiles (front, i0, j0, -) by level, per tile SCHUR_TILE first child sources, overflow ranges
  std::vector<I4> tiles;
  std::vector<int32_t> g1, gxp, tile_ptr;
  std::vector<I2> gx;                    // (lane group * TM TN + position, element id)
  // Schur blocks (front, i0, j0, -) by level, per block SCHUR_BLK_IDS first child sources, overflow ranges
  std::vector<I4> blocks;
  std::vector<int32_t> bg1, bgxp, blk_ptr;
  std::vector<I2> bgx;                   // (wave * 16 + position, element id)
  // A11 assembly records (dst, nz, first child source, -) in chunks of 8, levels padded to 8
  std::vector<I4> asm_rec;
  std::vector<int32_t> asm_xp, asm_ptr;  // per chunk: overflow range; per level: first record
  std::vector<I2> asm_x;                 // (record within the chunk, element id)
  // L21 (U12) items (front, first row, kind, record offset) by level; per item x row slot x pivot (nz, source)
  std::vector<I4> items;
  std::vector<I2> orec;
  std::vector<int32_t> oxp, item_ptr;
  bool fused0 = false;                   // level 0 through k_front0 (operator-form sweeps)
  int f0_small = 0;                      // the first f0_small listed fronts have <= 2 pivots
  std::vector<int32_t> f0_front, f0_ptr; // level-0 fronts (<= 2 pivots first); their first record
  std::vector<int32_t> f0_nz;            // per front: A11 lower (a >= b) then the L21 rows: original nz or -1
  std::vector<I2> ox;                    // (pivot * OFF_G OFF_RPL + row slot, element id)
  // algorithmic bytes per frequency, level and kernel class (operator-form sweeps)
  std::vector<std::array<int64_t, NKC>> lev_bytes;
  // symmetric mode: Dirichlet decoupling lists
  int n_dir = 0, n_crow = 0;
  std::vector<I2> dir, ce, de;           // (permuted node, diagonal nz); (Dirichlet slot, nz); (permuted row, nz)
  std::vector<int32_t> crow, cptr_dir, dptr, cslot;
  // permuted matrix compressed by rows and by columns (ptr, index, nz)
  std::vector<int32_t> rptr, ridx, rnz, cptr, cidx, cnz;
  // contraction entries: per permuted row a pseudo-entry (-1, -1, -1, i), then (column, nz of (i, j) or -1, nz of
  // (j, i) or -1, i); padded by 4 entries
  std::vector<I4> uent;
  int n_uent = 0;
};

// Element counts of the device buffers a solver with chunk Fc allocates (api.cpp allocates exactly these)
struct Workspace {
  int64_t F = 0, WV = 0, nvec = 0;       // factor entries x Fc, total rows x Fc, one n x Fc vector
  int64_t n_nvec = 0;                    // n-vectors: X, Y, XA, G, Y2, XR, Gx
  int64_t cpart = 0, kpart = 0, partial = 0, berr_acc = 0, gind = 0;
  int64_t WVk = 0, YVk = 0, fn_parts = 0, fcoef = 0, Bc = 0;
  int64_t bytes = 0;                     // all of it (pfr_solver_workspace_bytes)
};
Workspace workspace(const Symbolic& S, int64_t Fc, int n_crow);

// Builds the plan; returns 0, or non-zero with err set (a front too large for the kernels, int32 overflow)
int build_plan(const Symbolic& S, const PlanOptions& o, Plan& P, std::string& err);

// The fronts holding the given permuted rows and all their ancestors: per-front flags and the marked fronts
// level by level (level order kept; ptr per level).  front_of_col: the front of each pivot column (permuted).
void reach_lists(const std::vector<int32_t>& front_of_col, const std::vector<int32_t>& front_parent,
                 const std::vector<int32_t>& level_ptr, const std::vector<int32_t>& level_fronts,
                 const std::vector<int32_t>& prows, std::vector<int32_t>& mark, std::vector<int32_t>& list,
                 std::vector<int32_t>& ptr);

// Every index each launch of a solver with chunk Fc takes from the plan, against the buffer it addresses
// (element ids < factor entries, nz < nnz, record offsets and overflow ranges inside their arrays, LDS sizes,
// the per-workgroup partial buffers against the grids that write them, the split solve parts covering every
// row once).  Returns "" or the first violation.
std::string check_plan(const Symbolic& S, const Plan& P, int64_t Fc, int split_target);

}  // namespace pfr
