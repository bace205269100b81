// Types shared by the host launchers and the HIP kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/pfr.h"
#include "plan.hpp"
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
