// Types shared by the host launchers and the HIP kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/pfr.h"
#include "symbolic.hpp"

namespace pfr {

// Device copy of the symbolic maps (all pointers are device pointers).
struct DevPattern {
  const Front* fronts;
  const int32_t* idx;
  const int32_t* relpos;
  const int32_t* row_front;
  const int32_t* asm_ptr;
  const int32_t* asm_col;
  const int32_t* asm_nz;
  const int32_t* ea_ptr;
  const int32_t* ea_src;
  const int32_t* perm;
  const int32_t* prow;
  const int32_t* pcol;
  int32_t n;
};

// Schur super-tile: a wavefront = SCHUR_QG frequencies x (SCHUR_SR x SCHUR_SC) lane groups,
// each lane group one SCHUR_TM x SCHUR_TN register tile -> (SCHUR_TM SCHUR_SR) x
// (SCHUR_TN SCHUR_SC) entries per wave.
#ifndef PFR_SCHUR_SR
#define PFR_SCHUR_SR 1
#endif
#ifndef PFR_SCHUR_TM
#define PFR_SCHUR_TM 4
#endif
constexpr int SCHUR_SR = PFR_SCHUR_SR, SCHUR_SC = PFR_SCHUR_SR, SCHUR_QG = 64 / (SCHUR_SR * SCHUR_SC);
#ifndef PFR_SCHUR_TN
#define PFR_SCHUR_TN PFR_SCHUR_TM
#endif
constexpr int SCHUR_TM = PFR_SCHUR_TM, SCHUR_TN = PFR_SCHUR_TN;
static_assert(SCHUR_SR * SCHUR_SC * SCHUR_QG == 64, "one wavefront per super-tile");

// Off-diagonal panel kernel: a wave = OFF_G lane groups of 64 / OFF_G frequencies, OFF_RPL rows
// (columns) per lane: OFF_G OFF_RPL rows per wave.
#ifndef PFR_OFF_G
#define PFR_OFF_G 1
#endif
#ifndef PFR_OFF_RPL
#define PFR_OFF_RPL 2
#endif
constexpr int OFF_G = PFR_OFF_G;
// A11 factorisation kernel: lane groups per wave (64 / FAC_G frequencies each, one front row each)
#ifndef PFR_FAC_G
#define PFR_FAC_G 2
#endif
constexpr int FAC_G = PFR_FAC_G;
constexpr int OFF_RPL = PFR_OFF_RPL;

// Largest front the solve kernels stage index lists for in LDS (checked at solver creation)
constexpr int MAX_FRONT = 1024;
constexpr int SCHUR_BLK = 16;   // k_schur_sym_blk block edge (16 waves x 4 x 4 tiles)

constexpr int COEF_MAX = 32;
struct CoefPack {
  double re[COEF_MAX];
  double im[COEF_MAX];
};

// The A11 assembly fused into the symmetric A11 LU (k_factor_sym prologue, PFR_FUSE_ASM): the
// assembly records of the level (dst, nz, first child source, -) with each front's first record at
// rec0[front] (its ns (ns + 1) / 2 records, lower triangle row by row), the overflow lists of further
// child sources per 8-record chunk (xptr / xl, global chunk numbering), and the operator K - omega^2 M.
// recs == NULL: A11 was assembled by k_assemble_level.
struct AsmArgs {
  const int4* recs = nullptr;
  const int32_t* rec0 = nullptr;
  const int32_t* xptr = nullptr;
  const int2* xl = nullptr;
  const double* freqs = nullptr;
  const double2* K = nullptr;
  const double* M = nullptr;
};

// b = rhsP * (beta_re - omega^2 mass_sum + i beta_im) per frequency (the rhs of a sweep's solves)
struct RhsScale {
  const double* freqs = nullptr;   // chunk-local frequencies [Hz]
  double mass_sum = 0, beta_re = 0, beta_im = 0;
};

struct FunctionalArgs {
  int32_t n_support;
  const int32_t* pidx;    // permuted DOF index of each support entry (device)
  const double* a;        // [aU | aV | aW], 3 * n_support (device)
  double ts;              // transverse sensitivity
  int32_t loss_type;      // PFR_LOSS_* or -1 (forward only)
  const double2* ref;     // reference FR (complex) or cotangent (re), indexed by global frequency
  double scale;           // 1 / F_total (mean over the whole sweep)
  double* fr0;            // != NULL: seed mode of k_functional (functional correction): fr of the solve -> fr0,
                          // G = d fr / d x (no loss terms); k_correct_finish forms the corrected fr and the loss
};

}  // namespace pfr
