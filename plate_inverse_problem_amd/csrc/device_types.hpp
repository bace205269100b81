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
// (SCHUR_TN SCHUR_SC) entries per wave.  Lane = frequency, one 4 x 4 tile per wave (measured 10 %
// faster than 16 frequencies x a 2 x 2 arrangement of 4 x 4 tiles).
constexpr int SCHUR_SR = 1, SCHUR_SC = 1, SCHUR_QG = 64 / (SCHUR_SR * SCHUR_SC);
constexpr int SCHUR_TM = 4, SCHUR_TN = 4;
static_assert(SCHUR_SR * SCHUR_SC * SCHUR_QG == 64, "one wavefront per super-tile");

// Off-diagonal panel kernel: a wave = OFF_G lane groups of 64 / OFF_G frequencies, OFF_RPL rows
// (columns) per lane: OFF_G OFF_RPL rows per wave.  Lane = frequency, two rows per lane (measured best of
// 1 / 2 lane groups and 1 / 2 / 4 rows per lane; the other shapes are in git history).
constexpr int OFF_G = 1;
constexpr int OFF_RPL = 2;
// A11 factorisation kernel: lane groups per wave (64 / FAC_G frequencies each, one front row each)
constexpr int FAC_G = 2;

// Largest front the solve kernels stage index lists for in LDS (checked at solver creation)
constexpr int MAX_FRONT = 1024;
constexpr int SCHUR_BLK = 16;   // k_schur_sym_blk block edge (16 waves x 4 x 4 tiles)

constexpr int COEF_MAX = 32;
struct CoefPack {
  double re[COEF_MAX];
  double im[COEF_MAX];
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
