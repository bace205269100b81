// Batched multifrontal LU, forward/adjoint triangular solves, FR functional and
// adjoint gradient contraction for CDNA4 (gfx950).
//
// Layout: FREQUENCY-MINOR.  Every scalar of the factorisation (a front entry, a
// work-vector entry, a solution entry) is stored as `Fc` consecutive complex
// doubles, one per frequency of the chunk.  A wavefront = 64 consecutive
// frequencies of the same entry: every index is wave-uniform (scalar loads),
// every value load/store is one 1 KiB contiguous wave-instruction, no lane ever
// diverges (all frequencies share the pattern and the static pivot order).
// Workgroup = (front, 64 frequencies); its W waves split the rows of the front.
//
// Reference hot loop replaced: InnerState::solve mode 3, one UMFPACK numeric
// factorisation + solve per frequency inside `omp parallel for`
// (source/jax_plate_lib/include/InnerState.h:276-288), plus the XLA-fused
// assembly and functional of source/jax_plate/Problem.py:437-477 and the
// spsolve/matvec transpose rules of source/jax_plate/Sparse.py:162-222.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include <algorithm>
#include <atomic>

#include "launch.hpp"

namespace pfr {

using cplx = double2;

__device__ __forceinline__ cplx cadd(cplx a, cplx b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ cplx cmul(cplx a, cplx b) {
  return make_double2(fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x));
}
// c - a*b
__device__ __forceinline__ cplx cfms(cplx c, cplx a, cplx b) {
  return make_double2(fma(-a.x, b.x, fma(a.y, b.y, c.x)), fma(-a.x, b.y, fma(-a.y, b.x, c.y)));
}
__device__ __forceinline__ cplx cscale(cplx a, double m) { return make_double2(a.x * m, a.y * m); }
__device__ __forceinline__ cplx crecip(cplx b) {
  double d = fma(b.x, b.x, b.y * b.y);
  double inv = 1.0 / d;
  return make_double2(b.x * inv, -b.y * inv);
}
__device__ __forceinline__ void pivot_check(cplx p, int* flags, int64_t q) {
  double m = fabs(p.x) + fabs(p.y);
  if (!(m > 0.0) || !isfinite(m)) atomicOr(flags + q, PFR_FLAG_BAD_PIVOT);
}

constexpr int KB = 4;    // factorisation pivot block
constexpr int KBS = 8;   // triangular-solve block (its lower triangle: 28 loads, all in flight)

// ------------------------------------------------------------------ helpers
// XCD-aware workgroup order: the dispatcher deals workgroups round-robin over
// the 8 XCDs (each with its own L2), so workgroup `orig` is renumbered such that
// every XCD receives one contiguous range of logical ids (bijective for any
// count; MI355X_MICROARCH.md, workgroup dispatch / T1 swizzle).  Speed only.
__device__ __forceinline__ int64_t xcd_swizzle(int64_t orig, int64_t nwg) {
  const int64_t q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

struct Ctx {
  int lane, w, W;
  int64_t q;
};
// With a group list (the selective adjoint refinement: a few 64-frequency groups of the chunk, the launch's grid
// rows indexing the list) the workgroup's frequencies are the listed group's; false: no group (list entry -1).
__device__ __forceinline__ bool pick_group(Ctx& c, const int* __restrict__ glist) {
  if (!glist) return true;
  const int g = glist[c.q >> 6];
  if (g < 0) return false;
  c.q = (int64_t)g * 64 + c.lane;
  return true;
}
// ctx() for the level-solve kernels with the XCD-aware workgroup order: the workgroups of one
// 64-frequency group run on one XCD, so the solution rows that many fronts of a level gather
// (their common ancestors' pivots) are fetched into one L2, not eight.  bx: the front slot.
__device__ __forceinline__ Ctx ctx_xcd(int& bx) {
  const int64_t lid = xcd_swizzle(blockIdx.x + (int64_t)gridDim.x * blockIdx.y, (int64_t)gridDim.x * gridDim.y);
  bx = (int)(lid % gridDim.x);
  Ctx c;
  c.lane = threadIdx.x & 63;
  c.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  c.W = blockDim.x >> 6;
  c.q = (lid / gridDim.x) * 64 + c.lane;
  return c;
}
__device__ __forceinline__ Ctx ctx() {
  Ctx c;
  c.lane = threadIdx.x & 63;
  c.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  c.W = blockDim.x >> 6;
  c.q = (int64_t)blockIdx.y * 64 + c.lane;
  return c;
}

// ------------------------------------------------------------------ K1: combine
// K[nz] = sum_k coef_k * stiff[nz * n_stiff + k]   (Problem.py:440-445, theta part)
__global__ void k_combine(const double* __restrict__ stiff, int n_stiff, int64_t nnz, CoefPack coef,
                          cplx* __restrict__ K) {
  int64_t nz = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (nz >= nnz) return;
  const double* s = stiff + nz * n_stiff;
  double re = 0, im = 0;
  for (int k = 0; k < n_stiff; ++k) {
    re = fma(coef.re[k], s[k], re);
    im = fma(coef.im[k], s[k], im);
  }
  K[nz] = make_double2(re, im);
}

// ------------------------------------------------------------------ K2a: assemble + panel
// MODE 0: A_q = K - omega_q^2 M assembled on the fly (operator form).
// MODE 1: A_q = data[q * data_stride + nz] (explicit batch, InnerState::solve data).
// The front (f x f, row-major, frequency-minor) is assembled, then the first ns
// pivots are eliminated with static diagonal pivots, restricted right-looking:
// every block of KB pivots updates the pivot rows (all columns) and the panel
// columns of the update rows; the Schur block A22 (update rows x update
// columns) is left for k_schur_level (a register-tiled GEMM over all pivots).
constexpr int JB = 4;     // columns per batched read-modify-write step

// Assembly of a level's panel regions as a gather: a wavefront = 64 frequencies
// x 8 consecutive records (dst, nz, src, -); every record is one store of
// original entry (K - omega^2 M, or the explicit batch) + the first child
// update-matrix entry landing there; the rare further child entries of the
// chunk come from the overflow list.  All loads of a chunk are in flight
// together; each panel entry is written exactly once.
template <int MODE>
__global__ __launch_bounds__(256) void k_assemble_level(const int4* __restrict__ recs, int nrec,
                                                         const int* __restrict__ xptr, const int2* __restrict__ xl,
                                                         cplx* __restrict__ F, int64_t Fc,
                                                         const double* __restrict__ freqs,
                                                         const cplx* __restrict__ K, const double* __restrict__ M,
                                                         const cplx* __restrict__ data, int64_t data_stride,
                                                         int nvalid) {
  const int lane = threadIdx.x & 63;
  const int chunk = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  if (chunk * 8 >= nrec) return;
  const int64_t q = (int64_t)blockIdx.y * 64 + lane;
  double om2 = 0.0;
  if (MODE == 0) {
    const double om = 6.283185307179586 * freqs[q];
    om2 = om * om;
  }
  const cplx* __restrict__ dq = data + min(q, (int64_t)nvalid - 1) * data_stride;
  int4 r[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = recs[chunk * 8 + k];
  cplx v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    cplx o = make_double2(0.0, 0.0), c = make_double2(0.0, 0.0);
    if (r[k].y >= 0) {
      if (MODE == 0) {
        const cplx kk = K[r[k].y];
        o = make_double2(fma(-om2, M[r[k].y], kk.x), kk.y);
      } else {
        o = dq[r[k].y];
      }
    }
    if (r[k].z >= 0) c = F[(int64_t)r[k].z * Fc + q];
    v[k] = cadd(o, c);
  }
  const int x1 = xptr[chunk + 1];
  for (int x = xptr[chunk]; x < x1; ++x) {
    const int2 g = xl[x];
    const cplx c = F[(int64_t)g.y * Fc + q];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (g.x == k) v[k] = cadd(v[k], c);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k)
    if (r[k].x >= 0) F[(int64_t)r[k].x * Fc + q] = v[k];
}

// One row of a rank-kb update, A(i, j) -= sum_t l_t U(k0 + t, j) for j in [j0, jend).
// Reads through `rd`, writes through `wr` (both the front base): every element
// is read once and then written once, never re-read, so the two access paths
// are declared non-aliasing -- this lets the compiler issue the next batch's
// loads before the current batch's stores (otherwise each batch pays a full
// store + load round trip).
__device__ __forceinline__ void row_update(const cplx* __restrict__ rd, cplx* __restrict__ wr, int64_t row_i,
                                           int64_t row_k0, int f, int64_t Fc, int j0, int jend, int kb,
                                           const cplx (&l)[KB]) {
#pragma unroll 2
  for (int jb = j0; jb < jend; jb += JB) {
    cplx u[KB][JB], v[JB];
#pragma unroll
    for (int jj = 0; jj < JB; ++jj) {
      const int j = min(jb + jj, jend - 1);
      v[jj] = rd[(row_i + j) * Fc];
#pragma unroll
      for (int t = 0; t < KB; ++t) u[t][jj] = rd[(row_k0 + (int64_t)min(t, kb - 1) * f + j) * Fc];
    }
    // l[t] = 0 for t >= kb (callers), so the clamped rows add nothing; no load sits under a
    // runtime test (that compiles to a branch + vmcnt(0) per load)
#pragma unroll
    for (int jj = 0; jj < JB; ++jj)
#pragma unroll
      for (int t = 0; t < KB; ++t) v[jj] = cfms(v[jj], l[t], u[t][jj]);
#pragma unroll
    for (int jj = 0; jj < JB; ++jj)
      if (jb + jj < jend) wr[(row_i + jb + jj) * Fc] = v[jj];
  }
}

// Pivot rows of a block, columns j = j0, j0 + stride, ...: x = L11^{-1} x in
// place (unit lower, strictly-lower part of L11 in registers).  Same
// read/write split as row_update: each element is read once, written once.
__device__ __forceinline__ void col_solve(const cplx* __restrict__ rd, cplx* __restrict__ wr, int64_t row_k0, int f,
                                          int64_t Fc, int j0, int jend, int stride, int kb,
                                          const cplx (&L)[KB][KB]) {
#pragma unroll 2
  for (int j = j0; j < jend; j += stride) {
    cplx x[KB];
#pragma unroll
    for (int i = 0; i < KB; ++i)
      if (i < kb) x[i] = rd[(row_k0 + (int64_t)i * f + j) * Fc];
#pragma unroll
    for (int i = 1; i < KB; ++i)
      if (i < kb) {
#pragma unroll
        for (int t = 0; t < KB; ++t)
          if (t < i) x[i] = cfms(x[i], L[i][t], x[t]);
      }
#pragma unroll
    for (int i = 1; i < KB; ++i)
      if (i < kb) wr[(row_k0 + (int64_t)i * f + j) * Fc] = x[i];
  }
}

// Panel kernel lane map: a wavefront covers 64 / FAC_G frequencies x FAC_G front rows
// (lane = (64 / FAC_G) * sub + frequency; FAC_G = 2 measured best of 1, 2, 4), so every
// wave-instruction advances FAC_G rows (or columns) at once and the pivot-row values it
// reads are shared by the row groups; workgroup = (front, 64 / FAC_G frequencies), W waves.
// DIAG = true: only the diagonal block A11 = L11 U11 (rows and columns < ns);
// L21 and U12 are then formed row / column-wise by k_offdiag_level.
template <bool DIAG>
__global__ __launch_bounds__(512) void k_factor_level(DevPattern P, const int* __restrict__ lvl,
                                                       cplx* __restrict__ F, int64_t Fc,
                                                       int* __restrict__ flags) {
  Ctx c;
  c.lane = threadIdx.x & 63;
  c.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  c.W = blockDim.x >> 6;
  constexpr int QG = 64 / FAC_G;     // frequencies per lane group
  c.q = (int64_t)blockIdx.y * QG + c.lane % QG;
  const int sub = c.lane / QG;
  const Front fr = P.fronts[lvl[blockIdx.x]];
  const int f = fr.f, ns = fr.ns;
  const int lim = DIAG ? ns : f;     // rows / pivot-row columns handled here
  cplx* __restrict__ base = F + fr.off * Fc + c.q;
#define E(a, b) base[((int64_t)(a) * f + (b)) * Fc]
  // 2. blocked restricted right-looking elimination of the ns pivots
  for (int k0 = 0; k0 < ns; k0 += KB) {
    const int kb = min(KB, ns - k0);
    const int k1 = k0 + kb;
    if (c.w == 0) {
      // diagonal block: one load burst, LU in registers, one store burst
      cplx D[KB][KB];
#pragma unroll
      for (int i = 0; i < KB; ++i)
#pragma unroll
        for (int j = 0; j < KB; ++j) {
          const int a = k0 + min(i, kb - 1), b = k0 + min(j, kb - 1);
          D[i][j] = E(a, b);
        }
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        if (k < kb) {
          pivot_check(D[k][k], flags, c.q);
          const cplx inv = crecip(D[k][k]);
#pragma unroll
          for (int i = k + 1; i < KB; ++i) {
            D[i][k] = cmul(D[i][k], inv);
#pragma unroll
            for (int j = k + 1; j < KB; ++j) D[i][j] = cfms(D[i][j], D[i][k], D[k][j]);
          }
        }
      }
      if (sub == 0) {
#pragma unroll
        for (int i = 0; i < KB; ++i)
#pragma unroll
          for (int j = 0; j < KB; ++j)
            if (i < kb && j < kb) E(k0 + i, k0 + j) = D[i][j];
      }
    }
    __syncthreads();
    // pivot rows of the block, columns >= k1:  L11^{-1} A12 (columns over waves)
    {
      cplx L[KB][KB];
#pragma unroll
      for (int i = 0; i < KB; ++i)
#pragma unroll
        for (int j = 0; j < KB; ++j)
          if (j < i && i < kb) L[i][j] = E(k0 + i, k0 + j);
      col_solve(base, base, (int64_t)k0 * f, f, Fc, k1 + FAC_G * c.w + sub, lim, FAC_G * c.W, kb, L);
    }
    __syncthreads();
    // rows >= k1: l = A(i, block) U11^{-1}; then update
    //   pivot rows (i < ns): columns [k1, f)      update rows (i >= ns): columns [k1, ns)
    {
      cplx U[KB][KB];
      cplx Dinv[KB];
#pragma unroll
      for (int i = 0; i < KB; ++i)
#pragma unroll
        for (int j = 0; j < KB; ++j)
          if (i < j && j < kb) U[i][j] = E(k0 + i, k0 + j);
#pragma unroll
      for (int i = 0; i < KB; ++i)
        if (i < kb) Dinv[i] = crecip(E(k0 + i, k0 + i));
      for (int i = k1 + FAC_G * c.w + sub; i < lim; i += FAC_G * c.W) {
        cplx l[KB];
#pragma unroll
        for (int t = 0; t < KB; ++t) l[t] = cscale(E(i, k0 + min(t, kb - 1)), t < kb ? 1.0 : 0.0);
#pragma unroll
        for (int t = 0; t < KB; ++t)
          if (t < kb) {
#pragma unroll
            for (int s = 0; s < KB; ++s)
              if (s < t) l[t] = cfms(l[t], l[s], U[s][t]);
            l[t] = cmul(l[t], Dinv[t]);
            E(i, k0 + t) = l[t];
          }
        const int jend = i < ns ? lim : ns;
        row_update(base, base, (int64_t)i * f, (int64_t)k0 * f, f, Fc, k1, jend, kb, l);
      }
    }
    __syncthreads();
  }
#undef E
}

// global -> LDS copy of one 1 KiB row (lane l's 16 B to lds_row + 16 l), issued as inline asm so
// that the compiler's wait insertion does not see it: with the builtin it waits vmcnt(0) before
// every LDS read of the staging array (the copies in flight might alias), which serialises the
// pipeline.  Every wait on these copies is therefore explicit (PFR_WAIT_VM).
__device__ __forceinline__ void glds16(const cplx* g, cplx* lds_row) {
  const uint32_t dst = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds_row);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(dst)
               : "memory");
}

// Workgroup barrier for the LDS-staged kernels: LDS reads retired (lgkmcnt(0)), then s_barrier,
// as one asm statement with a memory clobber so that the compiler moves no LDS access across it
// (the builtin s_barrier is no compiler fence: reads of a buffer were sunk below the barrier after
// which other waves overwrite it).  Global->LDS copies in flight are NOT waited for here.
#define PFR_BARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")

// s_waitcnt vmcnt(n) alone (expcnt / lgkmcnt left at their no-wait maxima; gfx9 encoding)
#define PFR_WAIT_VM(n) __builtin_amdgcn_s_waitcnt(((n) & 15) | (((n) >> 4) << 14) | (7 << 4) | (15 << 8))

// Symmetric mode: A11 is symmetric, so only its lower triangle is kept up to date (trailing
// updates over j <= i: half the LU's work and traffic) and U11 = diag(U11) L11^T is written from
// each L row as it is formed (no pivot-row solves).  Pivots in super-blocks of 8 = two 4-pivot
// blocks A, B with lookahead: A's diagonal block and L rows, B's columns updated by A alone, B's
// diagonal block and L rows, then ONE rank-8 update of the trailing lower triangle -- which is
// read and written once per 8 pivots instead of once per 4 (the dominant traffic of this kernel).
// Lane map as k_factor_level; up to 16 waves per front.
template <int R, int JBU>
__device__ __forceinline__ void row_updateR(const cplx* __restrict__ rd, cplx* __restrict__ wr, int64_t row_i,
                                            int64_t row_k0, int f, int64_t Fc, int j0, int jend, int kr,
                                            const cplx (&l)[R]) {
#pragma unroll 2
  for (int jb = j0; jb < jend; jb += JBU) {
    cplx u[R][JBU], v[JBU];
#pragma unroll
    for (int jj = 0; jj < JBU; ++jj) {
      const int j = min(jb + jj, jend - 1);
      v[jj] = rd[(row_i + j) * Fc];
#pragma unroll
      for (int t = 0; t < R; ++t) u[t][jj] = rd[(row_k0 + (int64_t)min(t, kr - 1) * f + j) * Fc];
    }
#pragma unroll
    for (int jj = 0; jj < JBU; ++jj)
#pragma unroll
      for (int t = 0; t < R; ++t) v[jj] = cfms(v[jj], l[t], u[t][jj]);   // l[t] = 0 for t >= kr
#pragma unroll
    for (int jj = 0; jj < JBU; ++jj)
      if (jb + jj < jend) wr[(row_i + jb + jj) * Fc] = v[jj];
  }
}

constexpr int FAC_JBU = 2;   // trailing-update columns per read-modify-write step
constexpr int FAC_SB = 2;    // 4-pivot blocks per super-block (rank of the trailing update / 4)

// One front's A11 LU for the 64 / G frequencies of c.q's lane group: c.w / c.W the wave's index and count
// among the waves working on these frequencies (every wave of the workgroup reaches the same barriers)
template <int G>
__device__ __forceinline__ void factor_sym_front(const DevPattern& P, int front, cplx* __restrict__ F, int64_t Fc,
                                                 int* __restrict__ flags, const Ctx& c, int sub) {
  const Front fr = P.fronts[front];
  const int f = fr.f, ns = fr.ns;
  cplx* __restrict__ base = F + fr.off * Fc + c.q;
  const int r0 = G * c.w + sub, rs = G * c.W;   // this lane's first row offset, row stride
#define E(a, b) base[((int64_t)(a) * f + (b)) * Fc]
  // 4-pivot diagonal block at k0 (kb pivots): one load burst from the lower triangle, LU in
  // registers (U = diag(U) L^T up to rounding), one store burst
  auto diag = [&](int k0, int kb) {
    if (c.w != 0) return;
    cplx D[KB][KB];
#pragma unroll
    for (int i = 0; i < KB; ++i)
#pragma unroll
      for (int j = 0; j < KB; ++j) {
        const int a = k0 + min(i, kb - 1), b = k0 + min(j, kb - 1);
        D[i][j] = E(max(a, b), min(a, b));
      }
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      if (k < kb) {
        pivot_check(D[k][k], flags, c.q);
        const cplx inv = crecip(D[k][k]);
#pragma unroll
        for (int i = k + 1; i < KB; ++i) {
          D[i][k] = cmul(D[i][k], inv);
#pragma unroll
          for (int j = k + 1; j < KB; ++j) D[i][j] = cfms(D[i][j], D[i][k], D[k][j]);
        }
      }
    }
    if (sub == 0) {
#pragma unroll
      for (int i = 0; i < KB; ++i)
#pragma unroll
        for (int j = 0; j < KB; ++j)
          if (i < kb && j < kb) E(k0 + i, k0 + j) = D[i][j];
    }
  };
  // rows i >= i0 of the block's columns: L(i, blk) = A(i, blk) U_blk^{-1}, U(blk, i) = diag L(i, blk)^T
  auto rows = [&](int k0, int kb, int i0) {
    cplx U[KB][KB];
    cplx Dg[KB], Dinv[KB];
#pragma unroll
    for (int i = 0; i < KB; ++i)
#pragma unroll
      for (int j = 0; j < KB; ++j)
        if (i < j) U[i][j] = E(k0 + min(i, kb - 1), k0 + min(j, kb - 1));
#pragma unroll
    for (int i = 0; i < KB; ++i) {
      Dg[i] = E(k0 + min(i, kb - 1), k0 + min(i, kb - 1));
      Dinv[i] = crecip(Dg[i]);
    }
    for (int i = i0 + r0; i < ns; i += rs) {
      cplx l[KB];
#pragma unroll
      for (int t = 0; t < KB; ++t) l[t] = E(i, k0 + min(t, kb - 1));
#pragma unroll
      for (int t = 0; t < KB; ++t)
        if (t < kb) {
#pragma unroll
          for (int s = 0; s < KB; ++s)
            if (s < t) l[t] = cfms(l[t], l[s], U[s][t]);
          l[t] = cmul(l[t], Dinv[t]);
          E(i, k0 + t) = l[t];
          E(k0 + t, i) = cmul(Dg[t], l[t]);
        }
    }
  };
  constexpr int SB = FAC_SB, R = SB * KB;
  for (int k0 = 0; k0 < ns; k0 += R) {
    const int kr = min(R, ns - k0);
#pragma unroll 1
    for (int b = 0; b < SB; ++b) {
      const int kb0 = k0 + KB * b, kbs = min(KB, kr - KB * b);
      if (kbs <= 0) break;
      if (b > 0) {
        // this block's columns (lower part) updated by the super-block's earlier blocks: rank 4b
        for (int i = kb0 + r0; i < ns; i += rs) {
          cplx l[R];
#pragma unroll
          for (int t = 0; t < R; ++t) l[t] = cscale(E(i, k0 + min(t, KB * b - 1)), t < KB * b ? 1.0 : 0.0);
          row_updateR<R, 1>(base, base, (int64_t)i * f, (int64_t)k0 * f, f, Fc, kb0, min(kb0 + kbs, i + 1),
                            KB * b, l);
        }
        __syncthreads();
      }
      diag(kb0, kbs);
      __syncthreads();
      rows(kb0, kbs, kb0 + kbs);
      __syncthreads();
    }
    const int k1 = k0 + kr;
    if (k1 < ns) {
      // trailing lower triangle: A(i, j) -= L(i, k0:k1) U(k0:k1, j), k1 <= j <= i, rank kr
      for (int i = k1 + r0; i < ns; i += rs) {
        cplx l[R];
#pragma unroll
        for (int t = 0; t < R; ++t) l[t] = cscale(E(i, k0 + min(t, kr - 1)), t < kr ? 1.0 : 0.0);
        row_updateR<R, FAC_JBU>(base, base, (int64_t)i * f, (int64_t)k0 * f, f, Fc, k1, i + 1, kr, l);
      }
      __syncthreads();
    }
  }
#undef E
}

// G lane groups per wave (64 / G frequencies x G front rows): FAC_G, or 4 / 8 on the levels whose launch would
// otherwise have few workgroups (a single 76-pivot separator at 2,048 frequencies: 64) -- more workgroups of
// fewer frequencies, each wave-instruction advancing G rows, so each workgroup's pivot chain passes over fewer
// row strides
template <int G>
__global__ __launch_bounds__(1024) void k_factor_sym(DevPattern P, const int* __restrict__ lvl, cplx* __restrict__ F,
                                               int64_t Fc, int* __restrict__ flags) {
  Ctx c;
  c.lane = threadIdx.x & 63;
  c.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  c.W = blockDim.x >> 6;
  constexpr int QG = 64 / G;     // frequencies per lane group
  c.q = (int64_t)blockIdx.y * QG + c.lane % QG;
  factor_sym_front<G>(P, lvl[blockIdx.x], F, Fc, flags, c, c.lane / QG);
}

// Symmetric A11 LU with the pivot block resident in LDS, for the levels where the frequency-minor kernel gets few
// workgroups (the top of the elimination tree: few fronts, long pivot chains).  The lower triangle of A11 (packed,
// idx(i, j) = i (i + 1) / 2 + j) is read once into LDS, factored there and written once: L11 below the diagonal,
// U11 = diag(U) L11^T above it, U(k, k) on it -- the same entries k_factor_sym writes.
__device__ __forceinline__ int tri_row(int e) {
  int i = (int)((sqrtf(8.0f * e + 1.0f) - 1.0f) * 0.5f);
  if ((i + 1) * (i + 2) / 2 <= e) ++i;
  else if (i * (i + 1) / 2 > e) --i;
  return i;
}

__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
__device__ __forceinline__ cplx readlane_c(cplx v, int l) { return make_double2(readlane_d(v.x, l), readlane_d(v.y, l)); }

// Workgroup = one front x one frequency, 4 waves; the packed lower triangle in LDS.  Per block of FAC_LB pivots:
// wave 0 (lane = row, rows < 64) eliminates the block's pivots and forms the panel rows wave-synchronously -- each
// lane holds its row's FAC_LB block entries in registers, the pivot and the pivot rows' entries broadcast by
// v_readlane -- writing L(i, p) to the triangle and W(i, t) = U(p, p) L(i, p) to a column-major scratch; then all
// threads update the trailing lower triangle, A(i, j) -= sum_t L(i, k0 + t) W(j, t).  Two barriers per 8 pivots.
constexpr int FAC_LB = 8;
__global__ __launch_bounds__(256) void k_factor_sym_lds(DevPattern P, const int* __restrict__ lvl,
                                                        cplx* __restrict__ F, int64_t Fc, int* __restrict__ flags,
                                                        int maxns) {
  extern __shared__ cplx sA[];
  cplx* __restrict__ sW = sA + (int64_t)maxns * (maxns + 1) / 2;   // W(i, t) at sW[t * maxns + i]
  const int64_t lid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int slot = (int)(lid / Fc);
  const int64_t q = lid % Fc;
  const Front fr = P.fronts[lvl[slot]];
  const int f = fr.f, ns = fr.ns;
  const int tid = threadIdx.x, S = blockDim.x, lane = tid & 63;
  cplx* __restrict__ base = F + fr.off * Fc + q;
  const int nlow = ns * (ns + 1) / 2;
#define E(a, b) base[((int64_t)(a) * f + (b)) * Fc]
#define A(i, j) sA[((i) * ((i) + 1)) / 2 + (j)]
  // UB loads in flight per thread before their LDS stores
  constexpr int UB = 8;
  for (int e0 = tid; e0 < nlow; e0 += UB * S) {
    cplx v[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int e = min(e0 + u * S, nlow - 1);
      const int i = tri_row(e), j = e - i * (i + 1) / 2;
      v[u] = E(i, j);
    }
#pragma unroll
    for (int u = 0; u < UB; ++u)
      if (e0 + u * S < nlow) sA[e0 + u * S] = v[u];
  }
  __syncthreads();
  for (int k0 = 0; k0 < ns; k0 += FAC_LB) {
    const int kb = min(FAC_LB, ns - k0), k1 = k0 + kb;
    if (tid < 64) {
      // the block's pivots and the panel rows, lane = row (rows outside [k0, ns) hold clamped copies, never stored)
      const int row = lane, ri = min(max(row, k0), ns - 1);
      cplx a[FAC_LB];
#pragma unroll
      for (int t = 0; t < FAC_LB; ++t) a[t] = A(ri, min(k0 + t, ri));
#pragma unroll
      for (int t = 0; t < FAC_LB; ++t)
        if (t < kb) {
          const int p = k0 + t;
          const cplx d = readlane_c(a[t], p);
          if (lane == 0) pivot_check(d, flags, q);
          const cplx rd = crecip(d);
          cplx b[FAC_LB];      // W(k0 + u, t): the pivot column's unscaled entries of the block rows below p
#pragma unroll
          for (int u = t + 1; u < FAC_LB; ++u) b[u] = readlane_c(a[t], min(k0 + u, 63));
          const cplx wt = a[t], lt = cmul(wt, rd);
#pragma unroll
          for (int u = t + 1; u < FAC_LB; ++u) a[u] = cfms(a[u], lt, b[u]);
          if (row > p && row < ns) {
            A(row, p) = lt;
            sW[t * maxns + row] = wt;
          } else if (row == p) {
            A(p, p) = d;
          }
        }
    }
    __syncthreads();
    // trailing lower triangle (a short block is the last one: kb = FAC_LB whenever k1 < ns)
    const int m = ns - k1, nt = m * (m + 1) / 2;
    for (int e = tid; e < nt; e += S) {
      const int ii = tri_row(e), I = k1 + ii, J = k1 + e - ii * (ii + 1) / 2;
      cplx v = A(I, J);
#pragma unroll
      for (int t = 0; t < FAC_LB; ++t) v = cfms(v, A(I, k0 + t), sW[t * maxns + J]);
      A(I, J) = v;
    }
    __syncthreads();
  }
  // write back: L below the diagonal, U(k, k) on it, U(j, i) = U(j, j) L(i, j) above it
  for (int e = tid; e < nlow; e += S) {
    const int i = tri_row(e), j = e - i * (i + 1) / 2;
    const cplx v = sA[e];
    E(i, j) = v;
    if (j < i) E(j, i) = cmul(A(j, j), v);
  }
#undef A
#undef E
}

// Off-diagonal panel blocks once A11 = L11 U11 is factored, every row of L21 and
// every column of U12 independently (read once, written once):
//   kind 0, row i >= ns:     L(i, :ns) = A(i, :ns) U11^{-1}
//   kind 1, column j >= ns:  U(:ns, j) = L11^{-1} A(:ns, j)
// left-looking in chunks of OB columns (rows) held in registers; the L11 / U11
// entries each step reads are the same for the four lane groups of a wave.
// Item = (front, first row / column, kind): one wave = 16 frequencies x 4
// consecutive rows (columns).
constexpr int OB = 8;   // columns per left-looking chunk of k_offdiag_level (the tail cases cover 1-7)

// Where the off-diagonal entries come from (the panel entries of L21 / U12 are
// assembled here, at their first load, instead of being stored by the assembly
// kernel and read back): record (nz, first child element) per entry, further
// child elements in the item's overflow list.
struct OffSrc {
  const int2* rec[OFF_RPL];   // this lane's records per row slot, indexed by pivot
  const int2* ox;             // overflow (pivot * OFF_G OFF_RPL + slot, element id)
  int ox0, ox1, slot0;        // slot of row 0 of this lane: h * 4 + lane group
  double om2;                 // MODE 0: omega^2 of this lane's frequency
  const cplx* K;
  const double* M;
  const cplx* dq;             // MODE 1: this lane's explicit matrix values
};

template <int MODE>
__device__ __forceinline__ cplx off_source(const OffSrc& S, const cplx* __restrict__ F, int64_t Fc, int64_t q,
                                           int h, int c) {
  const int2 g = S.rec[h][c];
  cplx o;
  if (MODE == 0) {
    const cplx k = S.K[max(g.x, 0)];
    o = make_double2(fma(-S.om2, S.M[max(g.x, 0)], k.x), k.y);
  } else {
    o = S.dq[max(g.x, 0)];
  }
  const cplx ch = F[(int64_t)max(g.y, 0) * Fc + q];
  // masks as multipliers: with a select the load is sunk under a branch and waited for at once
  return cadd(cscale(o, g.x >= 0 ? 1.0 : 0.0), cscale(ch, g.y >= 0 ? 1.0 : 0.0));
}

// One chunk of NB consecutive columns (kind 0) / rows (kind 1) c0 .. c0+NB-1 of
// this lane's OFF_RPL rows (columns); the shared L11 / U11 values each step loads
// serve all of them.
template <int MODE, int NB, bool PRE = true, int PU = 2>
__device__ __forceinline__ void offdiag_chunk(cplx* __restrict__ base, const int64_t (&so)[OFF_RPL], int64_t sc,
                                              int64_t sa, int64_t sb, bool unit, const bool (&valid)[OFF_RPL],
                                              int c0, const OffSrc& S, const cplx* __restrict__ F, int64_t Fc,
                                              int64_t q) {
  cplx x[OFF_RPL][NB];
#pragma unroll
  for (int h = 0; h < OFF_RPL; ++h)
#pragma unroll
    for (int j = 0; j < NB; ++j) x[h][j] = off_source<MODE>(S, F, Fc, q, h, c0 + j);
  for (int e = S.ox0; e < S.ox1; ++e) {       // rare: several children cover one entry
    const int2 g = S.ox[e];
    const int c = g.x / (OFF_G * OFF_RPL) - c0, slot = g.x % (OFF_G * OFF_RPL);
    if (c >= 0 && c < NB) {
      const cplx v = F[(int64_t)g.y * Fc + q];
#pragma unroll
      for (int h = 0; h < OFF_RPL; ++h)
        if (slot == S.slot0 + OFF_G * h) {
#pragma unroll
          for (int j = 0; j < NB; ++j)
            if (j == c) x[h][j] = cadd(x[h][j], v);
        }
    }
  }
  // x -= own(0:c0) * shared(0:c0, c0:c0+NB)   (PRE = false: c0 = 0, no prefix); PU = 3: software-pipelined
  int t0 = 0;
  if (PU == 3 && PRE && c0 > 0) {
    // software-pipelined prefix: the next D pivots' loads are in flight while a pivot's products run, so the
    // products wait only for the oldest loads (the compiler's s_waitcnt counts the younger ones) instead of the
    // plain loop's drain at every pivot; same products, same order.  c0 is a multiple of OB, so the rounds of D
    // pivots are whole: no conditional load (a load under a branch makes the compiler drain every load at the
    // join).  Running element pointers, advanced once per pivot: no 64-bit index product per load (round 6: 94
    // instead of 180 instructions per pivot).  D = 4 measured slower (255 VGPRs; profiles/EXPERIMENTS.md).
    constexpr int D = 2;
    static_assert(OB % D == 0, "whole rounds");
    cplx lb[D][OFF_RPL], ub[D][NB];
    const cplx* lq[OFF_RPL];
#pragma unroll
    for (int h = 0; h < OFF_RPL; ++h) lq[h] = base + so[h] * Fc;
    const cplx* uq = base + (int64_t)c0 * sb * Fc;
    const int64_t lstep = sc * Fc, ustep = sa * Fc, ucol = sb * Fc;
    auto ld = [&](cplx (&l)[OFF_RPL], cplx (&u)[NB]) {
#pragma unroll
      for (int h = 0; h < OFF_RPL; ++h) {
        l[h] = *lq[h];
        lq[h] += lstep;
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) u[j] = uq[j * ucol];
      uq += ustep;
    };
    auto fm = [&](const cplx (&l)[OFF_RPL], const cplx (&u)[NB]) {
#pragma unroll
      for (int h = 0; h < OFF_RPL; ++h)
#pragma unroll
        for (int j = 0; j < NB; ++j) x[h][j] = cfms(x[h][j], l[h], u[j]);
    };
#pragma unroll
    for (int d = 0; d < D; ++d) ld(lb[d], ub[d]);
    for (int t = 0; t + 2 * D <= c0; t += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        fm(lb[d], ub[d]);
        ld(lb[d], ub[d]);
        // keep this pivot's loads here, in issue order: sunk below the later products (the scheduler's choice)
        // they reach the next round's first wait as the youngest, and every load drains there
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int d = 0; d < D; ++d) fm(lb[d], ub[d]);
    t0 = c0;
  }
#pragma unroll 2
  for (int t = t0; t < (PRE ? c0 : 0); ++t) {
    cplx l[OFF_RPL], u[NB];
#pragma unroll
    for (int h = 0; h < OFF_RPL; ++h) l[h] = base[(so[h] + (int64_t)t * sc) * Fc];
#pragma unroll
    for (int j = 0; j < NB; ++j) u[j] = base[((int64_t)t * sa + (int64_t)(c0 + j) * sb) * Fc];
#pragma unroll
    for (int h = 0; h < OFF_RPL; ++h)
#pragma unroll
      for (int j = 0; j < NB; ++j) x[h][j] = cfms(x[h][j], l[h], u[j]);
  }
  // triangular block shared(c0:c0+NB, c0:c0+NB), column by column
#pragma unroll
  for (int j = 0; j < NB; ++j) {
#pragma unroll
    for (int a = 0; a < NB; ++a)
      if (a < j) {
        const cplx t = base[((int64_t)(c0 + a) * sa + (int64_t)(c0 + j) * sb) * Fc];
#pragma unroll
        for (int h = 0; h < OFF_RPL; ++h) x[h][j] = cfms(x[h][j], x[h][a], t);
      }
    if (!unit) {
      const cplx d = crecip(base[((int64_t)(c0 + j) * (sa + sb)) * Fc]);
#pragma unroll
      for (int h = 0; h < OFF_RPL; ++h) x[h][j] = cmul(x[h][j], d);
    }
  }
#pragma unroll
  for (int h = 0; h < OFF_RPL; ++h)
    if (valid[h]) {
#pragma unroll
      for (int j = 0; j < NB; ++j) base[(so[h] + (int64_t)(c0 + j) * sc) * Fc] = x[h][j];
    }
}

// Item = (front, first row / column, kind, record offset): one wave = 64 / OFF_G
// frequencies x OFF_G lane groups x OFF_RPL rows (columns) per lane = OFF_G OFF_RPL
// consecutive rows (columns); row i0 + OFF_G h + lane group.  Default: lane = frequency
// (OFF_G = 1), 2 rows per lane: every load a 1 KiB run, each U11 value serving two rows
// (measured 26 % faster than 16 frequencies x 4 rows).
// SMALL: every front of the launch has ns <= OB (one chunk, no prefix loop): the register budget of
// the prefix loop is not needed (96 VGPRs: 5 waves/SIMD against 4) -- the bottom levels'
// rows are short and their waves bound by the latency of their item -> front -> record -> source
// load chain, which more resident waves overlap.
// One item (OFF_G OFF_RPL rows / columns of a front) of the panel for the frequency group `by`: the wave's
// own work, no barrier
template <int MODE, bool SMALL, int PU = 2>
__device__ __forceinline__ void offdiag_item(const DevPattern& P, const int4* __restrict__ items, int wid,
                                             const int2* __restrict__ orec, const int* __restrict__ oxp,
                                             const int2* __restrict__ ox, cplx* __restrict__ F, int64_t Fc,
                                             const double* __restrict__ freqs, const cplx* __restrict__ K,
                                             const double* __restrict__ M, const cplx* __restrict__ data,
                                             int64_t data_stride, int nvalid, int by) {
  const int lane = threadIdx.x & 63;
  constexpr int QG = 64 / OFF_G;                  // frequencies per lane group
  const int sub = lane / QG;
  const int64_t q = (int64_t)by * QG + lane % QG;
  const int4 it = items[wid];
  const Front fr = P.fronts[it.x];
  const int f = fr.f, ns = fr.ns;
  cplx* __restrict__ base = F + fr.off * Fc + q;
  // kind 0: own(c) = E(r, c), shared(a, b) = U(a, b) = E(a, b)
  // kind 1: own(c) = E(c, r), shared(a, b) = L(b, a) = E(b, a)   (transposed roles)
  const int64_t sc = it.z == 0 ? 1 : f;
  const int64_t sa = it.z == 0 ? f : 1, sb = it.z == 0 ? 1 : f;  // shared (a, b) at a * sa + b * sb
  const bool unit = it.z != 0;                                   // L11 has a unit diagonal
  OffSrc S;
  int64_t so[OFF_RPL];
  bool valid[OFF_RPL];
#pragma unroll
  for (int h = 0; h < OFF_RPL; ++h) {
    const int idx = it.y + OFF_G * h + sub;
    valid[h] = idx < f;
    const int r = min(idx, f - 1);
    so[h] = it.z == 0 ? (int64_t)r * f : r;                      // own element c at so + c * sc
    S.rec[h] = orec + it.w + (int64_t)(OFF_G * h + sub) * ns;
  }
  S.ox = ox;
  S.ox0 = oxp[wid];
  S.ox1 = oxp[wid + 1];
  S.slot0 = sub;
  S.om2 = 0.0;
  if (MODE == 0) {
    const double om = 6.283185307179586 * freqs[q];
    S.om2 = om * om;
  }
  S.K = K;
  S.M = M;
  S.dq = data + min(q, (int64_t)nvalid - 1) * data_stride;
  if (SMALL) {
    switch (ns) {
#define SMALLC(n) \
  case n: offdiag_chunk<MODE, n, false>(base, so, sc, sa, sb, unit, valid, 0, S, F, Fc, q); break;
      SMALLC(1) SMALLC(2) SMALLC(3) SMALLC(4) SMALLC(5) SMALLC(6) SMALLC(7) SMALLC(8)
#undef SMALLC
      default: break;
    }
    return;
  }
  int c0 = 0;
  for (; c0 + OB <= ns; c0 += OB) offdiag_chunk<MODE, OB, true, PU>(base, so, sc, sa, sb, unit, valid, c0, S, F, Fc, q);
  switch (ns - c0) {     // wave-uniform tail width
#define TAIL(n) \
  case n: offdiag_chunk<MODE, n, true, PU>(base, so, sc, sa, sb, unit, valid, c0, S, F, Fc, q); break;
    TAIL(1) TAIL(2) TAIL(3) TAIL(4) TAIL(5) TAIL(6) TAIL(7)
#undef TAIL
    default: break;
  }
}

// XCD-aware order: a frequency group's items on one XCD, sharing its L2
template <int MODE, bool SMALL, int PU = 2>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SMALL ? 5 : 1))) void k_offdiag_level(
    DevPattern P, const int4* __restrict__ items, int nitems, const int2* __restrict__ orec, const int* __restrict__ oxp,
    const int2* __restrict__ ox, cplx* __restrict__ F, int64_t Fc, const double* __restrict__ freqs,
    const cplx* __restrict__ K, const double* __restrict__ M, const cplx* __restrict__ data, int64_t data_stride,
    int nvalid) {
  const int64_t lid = xcd_swizzle(blockIdx.x + (int64_t)gridDim.x * blockIdx.y, (int64_t)gridDim.x * gridDim.y);
  const int bx = (int)(lid % gridDim.x), by = (int)(lid / gridDim.x);
  const int wid = __builtin_amdgcn_readfirstlane(bx * (blockDim.x >> 6) + (threadIdx.x >> 6));
  if (wid < nitems)
    offdiag_item<MODE, SMALL, PU>(P, items, wid, orec, oxp, ox, F, Fc, freqs, K, M, data, data_stride, nvalid, by);
}

// ------------------------------------------------------------------ K0: the bottom level fused
// Level 0's ~3,000 leaf fronts (1-4 pivots, at most F0_RM update rows, no children) in ONE pass instead of the
// four class launches: one wave per (front, 64 frequencies), four fronts per workgroup, everything in registers --
// the panel's original entries (K - omega^2 M), the A11 LU (k_factor_sym's 4-pivot diagonal block), the L21 rows
// (k_offdiag_level's column order) and the lower update block (k_schur_sym_level's pivot order), each stored once
// and nothing read back.  Same operations in the same order as the four kernels: bit-for-bit the same factors.
template <int NS>
__global__ __launch_bounds__(256) void k_front0(DevPattern P, const int* __restrict__ fl, int nfronts,
                                                const int* __restrict__ fptr, const int* __restrict__ fnz,
                                                cplx* __restrict__ F, int64_t Fc, const double* __restrict__ freqs,
                                                const cplx* __restrict__ K, const double* __restrict__ M,
                                                int* __restrict__ flags) {
  static_assert(NS <= F0_NS && NS <= KB, "one diagonal block");
  int bx;
  const Ctx c = ctx_xcd(bx);
  const int slot = bx * 4 + c.w;
  if (slot >= nfronts) return;
  const Front fr = P.fronts[fl[slot]];
  const int f = fr.f, ns = fr.ns, r = f - ns;
  const int* __restrict__ rec = fnz + fptr[slot];
  const int nrec = ns * (ns + 1) / 2 + r * ns;
  const double om = 6.283185307179586 * freqs[c.q];
  const double om2 = om * om;
  // every load unconditional from a clamped record, masked arithmetically
  auto val = [&](int e) {
    const int nz = rec[min(e, nrec - 1)];
    const cplx k = K[max(nz, 0)];
    const double m = M[max(nz, 0)];
    return cscale(make_double2(fma(-om2, m, k.x), k.y), nz >= 0 ? 1.0 : 0.0);
  };
  cplx* __restrict__ base = F + fr.off * Fc + c.q;
#define E(a, b) base[((int64_t)(a) * f + (b)) * Fc]
  cplx D[NS][NS];
#pragma unroll
  for (int i = 0; i < NS; ++i)
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const int a = max(min(i, ns - 1), min(j, ns - 1)), b = min(min(i, ns - 1), min(j, ns - 1));
      D[i][j] = val(a * (a + 1) / 2 + b);
    }
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    if (k < ns) {
      pivot_check(D[k][k], flags, c.q);
      const cplx inv = crecip(D[k][k]);
#pragma unroll
      for (int i = k + 1; i < NS; ++i) {
        D[i][k] = cmul(D[i][k], inv);
#pragma unroll
        for (int j = k + 1; j < NS; ++j) D[i][j] = cfms(D[i][j], D[i][k], D[k][j]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NS; ++i)
#pragma unroll
    for (int j = 0; j < NS; ++j)
      if (i < ns && j < ns) E(i, j) = D[i][j];
  // L21 rows: L(i, t) = (A(i, t) - sum_{s < t} L(i, s) U(s, t)) / U(t, t); columns past ns zero
  const int e0 = ns * (ns + 1) / 2;
  cplx L[F0_RM][NS];
#pragma unroll
  for (int i = 0; i < F0_RM; ++i) {
#pragma unroll
    for (int t = 0; t < NS; ++t) L[i][t] = val(e0 + min(i, max(r - 1, 0)) * ns + min(t, ns - 1));
#pragma unroll
    for (int t = 0; t < NS; ++t) {
#pragma unroll
      for (int s = 0; s < t; ++s) L[i][t] = cfms(L[i][t], L[i][s], D[s][t]);
      // columns past ns: the clamped copies' "pivot" can be 0 (a multiplicative mask would keep the NaN)
      const cplx lt = cmul(L[i][t], crecip(t < ns ? D[t][t] : make_double2(1.0, 0.0)));
      L[i][t] = t < ns ? lt : make_double2(0.0, 0.0);
    }
#pragma unroll
    for (int t = 0; t < NS; ++t)
      if (i < r && t < ns) E(ns + i, t) = L[i][t];
  }
  // the update block, lower: A22(i, j) = - sum_t (L(i, t) U(t, t)) L(j, t)
#pragma unroll
  for (int i = 0; i < F0_RM; ++i) {
    cplx lu[NS];
#pragma unroll
    for (int t = 0; t < NS; ++t) lu[t] = cmul(L[i][t], t < ns ? D[t][t] : make_double2(0.0, 0.0));
#pragma unroll
    for (int j = 0; j <= i; ++j) {
      cplx acc = make_double2(0.0, 0.0);
#pragma unroll
      for (int t = 0; t < NS; ++t) acc = cfms(acc, lu[t], L[j][t]);
      if (i < r) E(ns + i, ns + j) = acc;
    }
  }
#undef E
}

// ------------------------------------------------------------------ K2b: Schur complement
// A22 -= L21 U12 over all ns pivots of the front: one wavefront per TM x TN tile
// of A22 (64 lanes = 64 frequencies), accumulators in registers, no stores in
// the K loop so every load of a k-step is independent.
constexpr int TM = SCHUR_TM, TN = SCHUR_TN;

// Lane map: a wavefront = SCHUR_QG frequencies x SCHUR_SR x SCHUR_SC sub-tiles of
// SCHUR_TM x SCHUR_TN.  Default (device_types.hpp): lane = frequency, one 4 x 4 tile per
// wave, every operand load one 1 KiB run of 64 frequencies -- measured 10 % faster than 16
// frequencies x a 2 x 2 arrangement of 4 x 4 tiles (four 256 B runs per load, each loaded
// value shared by two sub-tiles).
// SYM (symmetric mode): only the lower triangle of A22 is formed; U12 = diag(U11) L21^T is
// not stored, its entries are made from the L21 rows at load.
// PF: the next pivot step's loads are issued before the current step's arithmetic.
template <bool SYM, bool PF, int KU>
__device__ __forceinline__ void schur_tile(const DevPattern& P, const int4* __restrict__ tiles, int ntiles,
                                           const int* __restrict__ g1, const int* __restrict__ gxp,
                                           const int2* __restrict__ gx, cplx* __restrict__ F, int64_t Fc) {
  const int lane = threadIdx.x & 63;
  // all super-tiles of one (front, 16 frequencies) on one XCD: the L21 rows and
  // U12 columns they share are fetched into that XCD's L2 once
  const int64_t lid = xcd_swizzle(blockIdx.x + (int64_t)gridDim.x * blockIdx.y, (int64_t)gridDim.x * gridDim.y);
  const int bx = (int)(lid % gridDim.x), by = (int)(lid / gridDim.x);
  const int tid = __builtin_amdgcn_readfirstlane(bx * (blockDim.x >> 6) + (threadIdx.x >> 6));
  if (tid >= ntiles) return;
  const int sub = lane / SCHUR_QG;
  const int64_t q = (int64_t)by * SCHUR_QG + lane % SCHUR_QG;
  int4 t = tiles[tid];
  t.y += TM * (sub / SCHUR_SC);
  t.z += TN * (sub % SCHUR_SC);
  const Front fr = P.fronts[t.x];
  const int f = fr.f, ns = fr.ns;
  cplx* __restrict__ base = F + fr.off * Fc + q;
  int ri[TM], cj[TN];
#pragma unroll
  for (int m = 0; m < TM; ++m) ri[m] = min(ns + t.y + m, f - 1);
#pragma unroll
  for (int n = 0; n < TN; ++n) cj[n] = min(ns + t.z + n, f - 1);
  // children's update-matrix entries landing in this tile (extend-add as a
  // gather): 16 source ids per lane group in 4 vector loads, then all 16 value
  // loads in flight at once (a missing source reads entry 0 and is dropped)
  cplx acc[TM][TN];
  {
    const int4* __restrict__ g4 =
        reinterpret_cast<const int4*>(g1 + ((int64_t)tid * (SCHUR_SR * SCHUR_SC) + sub) * (TM * TN));
    int src[TM * TN];
#pragma unroll
    for (int u = 0; u < TM * TN / 4; ++u) {
      const int4 v = g4[u];
      src[4 * u] = v.x;
      src[4 * u + 1] = v.y;
      src[4 * u + 2] = v.z;
      src[4 * u + 3] = v.w;
    }
#pragma unroll
    for (int m = 0; m < TM; ++m)
#pragma unroll
      for (int n = 0; n < TN; ++n) {
        const int e = src[m * TN + n];
        const cplx v = F[(int64_t)max(e, 0) * Fc + q];
        acc[m][n] = e >= 0 ? v : make_double2(0.0, 0.0);
      }
    // rare further sources (two or more children covering one position)
    const int x1 = gxp[tid + 1];
    for (int x = gxp[tid]; x < x1; ++x) {
      const int2 g = gx[x];
      if (g.x / (TM * TN) == sub) {
        const cplx v = F[(int64_t)g.y * Fc + q];
#pragma unroll
        for (int m = 0; m < TM; ++m)
#pragma unroll
          for (int n = 0; n < TN; ++n)
            if (g.x % (TM * TN) == m * TN + n) acc[m][n] = cadd(acc[m][n], v);
      }
    }
  }
  // row pointers: L21 row r, pivot k at pa[k * Fc]; U12 column c at pb[k * f * Fc] (general) or
  // L21 row c at pb[k * Fc] times the pivot U(k, k) (symmetric).  All loads of a pivot step are
  // issued before the arithmetic that uses them.
  const cplx* pa[TM];
  const cplx* pb[TN];
#pragma unroll
  for (int m = 0; m < TM; ++m) pa[m] = base + (int64_t)ri[m] * f * Fc;
#pragma unroll
  for (int n = 0; n < TN; ++n) pb[n] = base + (SYM ? (int64_t)cj[n] * f * Fc : (int64_t)cj[n] * Fc);
  const int64_t sb = SYM ? Fc : (int64_t)f * Fc, sd = (int64_t)(f + 1) * Fc;
  // KU pivot steps per iteration; with PF the next KU steps' loads are issued before this
  // iteration's arithmetic.  Steps past ns load the last pivot and contribute zero.
  cplx a[KU][TM], b[KU][TN], d[KU];
  auto load = [&](int k0, cplx (&aa)[KU][TM], cplx (&bb)[KU][TN], cplx (&dd)[KU]) {
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int k = min(k0 + u, ns - 1);
#pragma unroll
      for (int m = 0; m < TM; ++m) aa[u][m] = pa[m][k * Fc];
#pragma unroll
      for (int n = 0; n < TN; ++n) bb[u][n] = pb[n][k * sb];
      if (SYM) dd[u] = base[k * sd];
    }
  };
  if (PF && ns > 0) load(0, a, b, d);
  for (int k0 = 0; k0 < ns; k0 += KU) {
    cplx ca[KU][TM], cb[KU][TN], cd[KU];
    if (PF) {
#pragma unroll
      for (int u = 0; u < KU; ++u) {
#pragma unroll
        for (int m = 0; m < TM; ++m) ca[u][m] = a[u][m];
#pragma unroll
        for (int n = 0; n < TN; ++n) cb[u][n] = b[u][n];
        cd[u] = d[u];
      }
      if (k0 + KU < ns) load(k0 + KU, a, b, d);
    } else {
      load(k0, ca, cb, cd);
    }
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      if (SYM) {
        const cplx du = k0 + u < ns ? cd[u] : make_double2(0.0, 0.0);
#pragma unroll
        for (int m = 0; m < TM; ++m) ca[u][m] = cmul(ca[u][m], du);
      } else if (k0 + u >= ns) {
#pragma unroll
        for (int m = 0; m < TM; ++m) ca[u][m] = make_double2(0.0, 0.0);
      }
#pragma unroll
      for (int m = 0; m < TM; ++m)
#pragma unroll
        for (int n = 0; n < TN; ++n) acc[m][n] = cfms(acc[m][n], ca[u][m], cb[u][n]);
    }
  }
#pragma unroll
  for (int m = 0; m < TM; ++m)
#pragma unroll
    for (int n = 0; n < TN; ++n)
      if (ns + t.y + m < f && ns + t.z + n < f && (!SYM || t.y + m >= t.z + n))
        base[((int64_t)(ns + t.y + m) * f + ns + t.z + n) * Fc] = acc[m][n];
}

__global__ __launch_bounds__(256) void k_schur_level(DevPattern P, const int4* __restrict__ tiles, int ntiles,
                                                      const int* __restrict__ g1, const int* __restrict__ gxp,
                                                      const int2* __restrict__ gx, cplx* __restrict__ F, int64_t Fc) {
  schur_tile<false, false, 1>(P, tiles, ntiles, g1, gxp, gx, F, Fc);
}

// symmetric mode: explicit register budget (3 waves per SIMD) so that every load of a pivot
// step is in flight at once (the default budget serialises them; 1 step at 3 waves/SIMD measured 4 %
// faster than 2 steps at 2 waves/SIMD)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void k_schur_sym_level(
    DevPattern P, const int4* __restrict__ tiles, int ntiles, const int* __restrict__ g1,
    const int* __restrict__ gxp, const int2* __restrict__ gx, cplx* __restrict__ F, int64_t Fc) {
  schur_tile<true, true, 1>(P, tiles, ntiles, g1, gxp, gx, F, Fc);
}

// Symmetric mode, large update blocks (r >= PFR_SCHUR_BLK_MIN rows): a workgroup = 16 waves
// forms one 16 x 16 block of A22's lower triangle for 64 frequencies (lane = frequency), wave w
// the 4 x 4 tile (w / 4, w % 4).  Per stage of BKC pivots the block's 16 row operands L21(i, k),
// 16 column operands L21(j, k) and the pivots U(k, k) are copied once into LDS by global->LDS
// loads (no staging registers), double-buffered: stage s + 1 is in flight while stage s is
// multiplied.  Per pivot step that is 33 1-KiB loads for the block instead of 16 x 9 for 16
// independent 4 x 4 tiles -- the tile kernel is bound by its L2 operand traffic, not by HBM.
// BC = 16: 16 x 16 blocks, 16 waves; BC = 8: 16 x 8 blocks, 8 waves (half the LDS and waves per
// workgroup, so two blocks share a CU and one's barriers and prologue overlap the other's work).

// NB LDS buffers of KC pivots each.  NB = 2: plain double buffering, one __syncthreads per
// stage (it drains the next stage's copies).  NB >= 3: the copies of NB - 1 stages ahead stay in
// flight across a raw s_barrier, each stage retired by a counted vmcnt.
// block `bid` for the frequency group `by` (the workgroup's BC waves; barriers inside)
template <int NB, int KC, int BC>
__device__ __forceinline__ void schur_blk_body(const DevPattern& P, int bid, int by, const int4* __restrict__ blocks,
                                               const int* __restrict__ bg1, const int* __restrict__ bgxp,
                                               const int2* __restrict__ bgx, cplx* __restrict__ F, int64_t Fc) {
  constexpr int BR = SCHUR_BLK, NW = BC, TCW = BC / 4;   // block rows, waves, tile columns
  constexpr int BROWS = BR + BC + 1;      // LDS rows per pivot: row operands, column operands, U(k, k)
  __shared__ cplx sop[NB][KC][BROWS][64];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t q = (int64_t)by * 64 + lane;
  const int4 bk = blocks[bid];
  const Front fr = P.fronts[bk.x];
  const int f = fr.f, ns = fr.ns, r = f - ns;
  cplx* __restrict__ base = F + fr.off * Fc + q;
  const int ti = 4 * (w / TCW), tj = 4 * (w % TCW);
  // the tile holds a lower-triangle entry inside the update block
  const bool active = bk.y + ti < r && bk.y + ti + 3 >= bk.z + tj;
  cplx acc[4][4];
  if (active) {
    const int4* __restrict__ g4 = reinterpret_cast<const int4*>(bg1 + ((int64_t)bid * NW + w) * 16);
    int src[16];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int4 v = g4[u];
      src[4 * u] = v.x;
      src[4 * u + 1] = v.y;
      src[4 * u + 2] = v.z;
      src[4 * u + 3] = v.w;
    }
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int e = src[m * 4 + n];
        const cplx v = F[(int64_t)max(e, 0) * Fc + q];
        acc[m][n] = e >= 0 ? v : make_double2(0.0, 0.0);
      }
    const int x1 = bgxp[bid + 1];
    for (int x = bgxp[bid]; x < x1; ++x) {
      const int2 g = bgx[x];
      if (g.x / 16 == w) {
        const cplx v = F[(int64_t)g.y * Fc + q];
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int n = 0; n < 4; ++n)
            if (g.x % 16 == m * 4 + n) acc[m][n] = cadd(acc[m][n], v);
      }
    }
  }
  // stage copy: row slot rho of pivot u: rho < 16 -> L21 row i0 + rho, rho < 32 -> L21 row
  // j0 + rho - 16, rho = 32 -> U(k, k); wave w copies row operands w + NW h (h < BR / NW), column
  // operand w and, if w == u, U(k, k).  Rows past the block and pivots past ns read clamped (valid)
  // addresses.  Every address is scalar (saddr form: wave-uniform row pointer + lane * 16) and the
  // pivot offsets advance by one scalar add per stage: the scalar unit issues for all 16 waves of the
  // CU, and the per-copy 64-bit index products, generic->LDS casts and M0 saves it had to issue
  // before set the pivot rate (measured: as many scalar as vector instructions per pivot).
  const uint32_t voff = (uint32_t)lane * 16u;
  const int64_t rowb = Fc * 16;                                  // bytes between consecutive entries
  const char* sb = reinterpret_cast<const char*>(F + fr.off * Fc + (int64_t)by * 64);   // uniform
  const char* ra[BR / NW];
#pragma unroll
  for (int h = 0; h < BR / NW; ++h) ra[h] = sb + (int64_t)(ns + min(bk.y + w + NW * h, r - 1)) * f * rowb;
  const char* rb = sb + (int64_t)(ns + min(bk.z + w, r - 1)) * f * rowb;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)&sop[0][0][0][0]);
  constexpr uint32_t kRowB = 64 * sizeof(cplx), kPivB = BROWS * kRowB, kBufB = KC * kPivB;
  // pivot of the next stage to issue, and its byte offsets (row entry k, diagonal entry (k, k))
  int kn = 0;
  int64_t offk = 0, offd = 0;
  const int64_t diagb = (int64_t)(f + 1) * rowb;
  auto stage = [&](int buf) {
#pragma unroll
    for (int u = 0; u < KC; ++u) {
      const uint32_t d = lds0 + (uint32_t)buf * kBufB + (uint32_t)u * kPivB;
      uint32_t keep;
      if (w == u)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(voff), "s"(sb + offd), "s"(d + (uint32_t)(BR + BC) * kRowB)
                     : "memory");
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\t"
          "s_mov_b32 m0, %5\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %3\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(voff), "s"(ra[0] + offk), "s"(rb + offk), "s"(d + (uint32_t)w * kRowB),
            "s"(d + (uint32_t)(BR + w) * kRowB)
          : "memory");
#pragma unroll
      for (int h = 1; h < BR / NW; ++h)   // BC = 8: a second row operand per wave
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(voff), "s"(ra[h] + offk), "s"(d + (uint32_t)(w + NW * h) * kRowB)
                     : "memory");
      if (kn < ns - 1) {        // advance; past the last pivot the copies repeat it (never read)
        ++kn;
        offk += rowb;
        offd += diagb;
      }
    }
  };
  auto compute = [&](int buf, int k0) {
    if (!active) return;
#pragma unroll
    for (int u = 0; u < KC; ++u) {
      if (k0 + u < ns) {
        const cplx d = sop[buf][u][BR + BC][lane];
        cplx a[4], b[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) a[m] = cmul(sop[buf][u][ti + m][lane], d);
#pragma unroll
        for (int n = 0; n < 4; ++n) b[n] = sop[buf][u][BR + tj + n][lane];
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int n = 0; n < 4; ++n) acc[m][n] = cfms(acc[m][n], a[m], b[n]);
      }
    }
  };
  const int nst = (ns + KC - 1) / KC;
  // prologue: stages 0 .. NB - 2 in flight (stages past nst copy clamped rows, never read).  The
  // children's entries gathered above are older than these copies, so the first counted wait
  // retires them together with stage 0: one memory round trip for both.
#pragma unroll
  for (int p = 0; p < NB - 1; ++p) stage(p);
  // the gathered values are needed from here on: tie them down once (otherwise the compiler waits
  // for them -- vmcnt(0), copies in flight included -- inside the loop, every step)
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) asm volatile("" : "+v"(acc[m][n].x), "+v"(acc[m][n].y));
  for (int st = 0; st < nst; ++st) {
    // retire stage st: NB - 2 later stages may stay in flight (2 KC copies per wave and stage;
    // waves 0 .. KC-1 issue their pivot copy first and one more per stage, so they wait for a
    // copy or two more than needed)
    PFR_WAIT_VM((NB - 2) * (BR / NW + 1) * KC);
    PFR_BARRIER();   // stage st visible to all; everyone done with stage st - 1
    stage((st + NB - 1) % NB);
    compute(st % NB, st * KC);
  }
  PFR_WAIT_VM(0);
  if (active) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int i = bk.y + ti + m, j = bk.z + tj + n;
        if (i < r && j <= i) base[((int64_t)(ns + i) * f + ns + j) * Fc] = acc[m][n];
      }
  }
}

template <int NB, int KC, int BC>
__global__ __launch_bounds__(64 * BC) void k_schur_sym_blk(DevPattern P, const int4* __restrict__ blocks, int nblocks,
                                                         const int* __restrict__ bg1, const int* __restrict__ bgxp,
                                                         const int2* __restrict__ bgx, cplx* __restrict__ F,
                                                         int64_t Fc) {
  const int64_t lid = xcd_swizzle(blockIdx.x + (int64_t)gridDim.x * blockIdx.y, (int64_t)gridDim.x * gridDim.y);
  const int bid = (int)(lid % gridDim.x), by = (int)(lid / gridDim.x);
  if (bid >= nblocks) return;                // whole workgroup: uniform
  schur_blk_body<NB, KC, BC>(P, bid, by, blocks, bg1, bgxp, bgx, F, Fc);
}

// ------------------------------------------------------------------ right-hand sides
// RHS 0: b_p = rhsP[p] * (beta0 - omega^2 * mass_sum)   (Problem.py:447-449)
// RHS 1: b_p = B[q * b_stride + perm[p]]                 (explicit batch)
// RHS 2: b_p = G[p * Fc + q]                             (permuted device vector)
// RHS 3: RHS 0 + Bc[cslot[p] * Fc + q]                   (symmetric mode: Dirichlet columns moved
//        to the right-hand side, b_i - sum_d A_id b_d / A_dd, k_dirichlet_rhs)
struct RhsArgs {
  const double* rhsP;     // RHS 0: permuted Dirichlet vector
  double beta_re, beta_im, mass_sum;
  const double* freqs;
  const cplx* B;          // RHS 1
  int64_t b_stride;
  const cplx* G;          // RHS 2
  int nvalid;             // RHS 1: padded lanes repeat the last valid item
  const int* cslot;       // RHS 3: coupled-row slot of each permuted row (or -1)
  const cplx* Bc;         // RHS 3: Dirichlet corrections, slot-major (slot * Fc + q)
};

constexpr int MAX_SLICES = 4;
struct LSlices {          // k_lsolve_level_z / k_lsolve_rows_z: one bottom-up solve per slice
  const int* lvl[MAX_SLICES];     // the level's fronts of the slice
  int nf[MAX_SLICES];
  cplx* WV[MAX_SLICES];           // frontal work vectors (total_rows x Fc each)
  cplx* Y[MAX_SLICES];            // solution (permuted, n x Fc)
  const int* reach[MAX_SLICES];
  RhsArgs R[MAX_SLICES];
};

template <int RHS>
__device__ __forceinline__ cplx rhs_value(const DevPattern& P, const RhsArgs& R, int p, int64_t q, int64_t Fc) {
  if (RHS == 0 || RHS == 3) {
    const double v = R.rhsP[p];
    cplx b = make_double2(0.0, 0.0);
    if (v != 0.0) {
      const double om = 6.283185307179586 * R.freqs[q];
      b = make_double2(v * fma(-om * om, R.mass_sum, R.beta_re), v * R.beta_im);
    }
    if (RHS == 3) {
      const int c = R.cslot[p];
      if (c >= 0) b = cadd(b, R.Bc[(int64_t)c * Fc + q]);
    }
    return b;
  } else if (RHS == 1) {
    return R.B[min(q, (int64_t)R.nvalid - 1) * R.b_stride + P.perm[p]];
  } else {
    return R.G[(int64_t)p * Fc + q];
  }
}

// Gather the frontal vector: pivot rows from the rhs, plus children's update vectors.
// reach (per front, may be NULL): fronts whose update vector can be non-zero for this right-hand
// side (the RHS support and its elimination-tree ancestors); others' stale vectors are skipped.
// The index chains (row -> child entries -> child front -> reach; row -> permuted index -> rhs
// scalars) are resolved first by all threads at once into LDS, so the row loop issues only the
// value loads (each row's chain walked by one wave cost several dependent memory round trips).
constexpr int GATHER_CAP = 4096;    // child entries per front staged in LDS (more: direct path)

template <int RHS>
__device__ __forceinline__ cplx rhs_staged(const RhsArgs& R, int p, double rv, int cs, double om2, int64_t q,
                                           int64_t Fc) {
  if (RHS == 0 || RHS == 3) {
    cplx b = make_double2(0.0, 0.0);
    if (rv != 0.0) b = make_double2(rv * fma(-om2, R.mass_sum, R.beta_re), rv * R.beta_im);
    if (RHS == 3 && cs >= 0) b = cadd(b, R.Bc[(int64_t)cs * Fc + q]);
    return b;
  } else if (RHS == 1) {
    return R.B[min(q, (int64_t)R.nvalid - 1) * R.b_stride + p];    // p = perm[idx] here
  } else {
    return R.G[(int64_t)p * Fc + q];
  }
}

template <int RHS>
__device__ __forceinline__ void gather_frontal(const DevPattern& P, const Front& fr, const RhsArgs& R,
                                               cplx* __restrict__ WV, int64_t Fc, const Ctx& c,
                                               const int* __restrict__ reach, cplx* __restrict__ sv = nullptr) {
  __shared__ int s_ptr[MAX_FRONT + 1];
  __shared__ int s_src[GATHER_CAP];
  __shared__ int s_p[MAX_FRONT];
  __shared__ double s_rv[MAX_FRONT];
  __shared__ int s_cs[MAX_FRONT];
  const int f = fr.f, ns = fr.ns;
  const int E0 = P.ea_ptr[fr.row0], nE = P.ea_ptr[fr.row0 + f] - E0;
  if (nE > GATHER_CAP) {
    for (int a = c.w; a < f; a += c.W) {
      const int r = fr.row0 + a;
      cplx v = make_double2(0.0, 0.0);
      if (a < fr.ns) v = rhs_value<RHS>(P, R, P.idx[r], c.q, Fc);
      const int x1 = P.ea_ptr[r + 1];
      for (int e = P.ea_ptr[r]; e < x1; ++e) {
        const int src = P.ea_src[e];
        if (!reach || reach[P.row_front[src]]) v = cadd(v, WV[(int64_t)src * Fc + c.q]);
      }
      WV[(int64_t)r * Fc + c.q] = v;
      if (sv && a < fr.ns) sv[a * 64 + c.lane] = v;
    }
    return;
  }
  for (int t = threadIdx.x; t <= f; t += blockDim.x) s_ptr[t] = P.ea_ptr[fr.row0 + t] - E0;
  for (int t = threadIdx.x; t < nE; t += blockDim.x) {
    const int src = P.ea_src[E0 + t];
    s_src[t] = (!reach || reach[P.row_front[src]]) ? src : -1;
  }
  for (int t = threadIdx.x; t < ns; t += blockDim.x) {
    const int p = P.idx[fr.row0 + t];
    s_p[t] = RHS == 1 ? P.perm[p] : p;
    if (RHS == 0 || RHS == 3) s_rv[t] = R.rhsP[p];
    if (RHS == 3) s_cs[t] = R.cslot[p];
  }
  double om2 = 0.0;
  if (RHS == 0 || RHS == 3) {
    const double om = 6.283185307179586 * R.freqs[c.q];
    om2 = om * om;
  }
  __syncthreads();
  for (int a = c.w; a < f; a += c.W) {
    cplx v = make_double2(0.0, 0.0);
    if (a < ns)
      v = rhs_staged<RHS>(R, __builtin_amdgcn_readfirstlane(s_p[a]), s_rv[a], __builtin_amdgcn_readfirstlane(s_cs[a]),
                          om2, c.q, Fc);
    const int x0 = __builtin_amdgcn_readfirstlane(s_ptr[a]), x1 = __builtin_amdgcn_readfirstlane(s_ptr[a + 1]);
    for (int e = x0; e < x1; ++e) {
      const int src = __builtin_amdgcn_readfirstlane(s_src[e]);
      if (src >= 0) v = cadd(v, WV[(int64_t)src * Fc + c.q]);
    }
    WV[(int64_t)(fr.row0 + a) * Fc + c.q] = v;
    if (sv && a < ns) sv[a * 64 + c.lane] = v;
  }
}

// ------------------------------------------------------------------ K3a: L y = b (bottom-up)
// Workgroup = (front, 64 frequencies), W waves.  Pivot rows: blocks of KBS pivots, the
// diagonal block solved by wave 0 in registers (its loads independent of the chain), the
// later pivot rows updated by all waves.  Update rows: V(i) -= L21(i, :) y in ONE
// read-modify-write per row, SRB rows per wave, y in chunks of SKC.
constexpr int SRB = 4, SKC = 8;

// Pivot blocks of the solves: every load unconditional (indices clamped into the block) and the
// entries past the block masked arithmetically.  A load under a runtime condition -- even a
// wave-uniform one like `t < kb` -- becomes a branch around that load followed by vmcnt(0), so a
// 16-pivot block cost ~130 dependent memory round trips (~85 us) instead of a few.


// acc_v -= sum_{j0 <= j < j1} E(i, j) x_v(j): one factor row (erow = &E(i, 0), column stride Fc) against NV vectors
// resident in LDS (sx[v] + 64 j); the next 8 columns' loads are issued before the current 8 columns' products
// (the narrow-level solves: their loop otherwise waits on every batch)
template <int NV>
__device__ __forceinline__ void dot_row_lds(cplx (&acc)[NV], const cplx* __restrict__ erow, int64_t Fc,
                                            const cplx* const (&sx)[NV], int j0, int j1) {
  constexpr int U = 8;
  if (j0 >= j1) return;
  cplx ea[U], eb[U];
  auto ld = [&](cplx (&e)[U], int j) {
#pragma unroll
    for (int u = 0; u < U; ++u) e[u] = erow[(int64_t)min(j + u, j1 - 1) * Fc];
  };
  auto fm = [&](const cplx (&e)[U], int j) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int jj = min(j + u, j1 - 1);
      const cplx eu = cscale(e[u], j + u < j1 ? 1.0 : 0.0);
#pragma unroll
      for (int v = 0; v < NV; ++v) acc[v] = cfms(acc[v], eu, sx[v][jj * 64]);
    }
  };
  ld(ea, j0);
  int j = j0;
  for (; j + U < j1; j += 2 * U) {
    ld(eb, j + U);
    fm(ea, j);
    if (j + 2 * U < j1) ld(ea, j + 2 * U);
    fm(eb, j + U);
  }
  if (j < j1) fm(ea, j);
}

// V(i) -= L21(i, :) y for the update rows i = i_begin, i_begin + i_step, ... (SRB rows per step; y = the
// pivot part of the frontal vector, already solved)
__device__ __forceinline__ void lsolve_rows(const Front& fr, const cplx* __restrict__ base, cplx* __restrict__ wv,
                                            int64_t Fc, int i_begin, int i_step) {
  const int f = fr.f, ns = fr.ns;
#define E(a, b) base[((int64_t)(a) * f + (b)) * Fc]
#define V(a) wv[(int64_t)(a) * Fc]
  for (int i0 = i_begin; i0 < f; i0 += i_step) {
    int ri[SRB];
    cplx acc[SRB];
#pragma unroll
    for (int r = 0; r < SRB; ++r) {
      ri[r] = min(i0 + r, f - 1);
      acc[r] = V(ri[r]);
    }
    for (int k0 = 0; k0 < ns; k0 += SKC) {
      cplx y[SKC];
#pragma unroll
      for (int u = 0; u < SKC; ++u) y[u] = k0 + u < ns ? V(k0 + u) : make_double2(0.0, 0.0);
#pragma unroll
      for (int r = 0; r < SRB; ++r)
#pragma unroll
        for (int u = 0; u < SKC; ++u) acc[r] = cfms(acc[r], E(ri[r], min(k0 + u, ns - 1)), y[u]);
    }
#pragma unroll
    for (int r = 0; r < SRB; ++r)
      if (i0 + r < f) V(i0 + r) = acc[r];
  }
#undef E
#undef V
}

// NAR (the levels with few (front, group) workgroups, update rows split off): the pivot values resident in LDS
// (sv, ns x 64) and each KBS block walked LEFT-looking -- the block's rows form their sums over the solved columns
// (wave t row k0 + t: loads independent of the chain, solved values from LDS), then wave 0 solves the block's
// triangle; the right-looking form below waits on a global round trip per row batch and per block (the top
// levels of the bottom-up chain, ~35-100 us each at 2,048 frequencies).  Rounding differs from the default order.
template <int RHS, bool NAR = false>
__device__ __forceinline__ void lsolve_front(const DevPattern& P, const Front& fr, const cplx* __restrict__ F, int64_t Fc,
                                             cplx* __restrict__ WV, const RhsArgs& R, cplx* __restrict__ Y,
                                             const int* __restrict__ reach, int rows_split, const Ctx& c,
                                             cplx* __restrict__ sv = nullptr) {
  const int f = fr.f, ns = fr.ns;
  const cplx* __restrict__ base = F + fr.off * Fc + c.q;
  cplx* __restrict__ wv = WV + (int64_t)fr.row0 * Fc + c.q;
#define E(a, b) base[((int64_t)(a) * f + (b)) * Fc]
#define V(a) wv[(int64_t)(a) * Fc]
  gather_frontal<RHS>(P, fr, R, WV, Fc, c, reach, NAR ? sv : nullptr);
  __syncthreads();
  if (NAR) {
#define SV(a) sv[(a) * 64 + c.lane]
    for (int k0 = 0; k0 < ns; k0 += KBS) {
      const int kb = min(KBS, ns - k0);
      for (int t = c.w; t < kb; t += c.W) {
        const int i = k0 + t;
        cplx acc[1] = {make_double2(0.0, 0.0)};
        const cplx* const sx[1] = {sv + c.lane};
        dot_row_lds<1>(acc, base + (int64_t)i * f * Fc, Fc, sx, 0, k0);
        SV(i) = cadd(SV(i), acc[0]);
      }
      __syncthreads();
      if (c.w == 0) {
        cplx v[KBS];
#pragma unroll
        for (int t = 0; t < KBS; ++t) v[t] = SV(k0 + min(t, kb - 1));
#pragma unroll
        for (int i = 1; i < KBS; ++i) {
          const int ri = k0 + min(i, kb - 1);
#pragma unroll
          for (int k = 0; k < i; ++k) v[i] = cfms(v[i], E(ri, k0 + min(k, kb - 1)), v[k]);
        }
#pragma unroll
        for (int t = 0; t < KBS; ++t)
          if (t < kb) SV(k0 + t) = v[t];
      }
      __syncthreads();
    }
    for (int a = c.w; a < ns; a += c.W) {
      const cplx y = SV(a);
      V(a) = y;
      Y[(int64_t)(fr.col0 + a) * Fc + c.q] = y;
    }
#undef SV
    if (!rows_split) {
      __syncthreads();
      lsolve_rows(fr, base, wv, Fc, ns + SRB * c.w, SRB * c.W);
    }
    return;
  }
  for (int k0 = 0; k0 < ns; k0 += KBS) {
    const int kb = min(KBS, ns - k0), k1 = k0 + kb;
    if (c.w == 0) {
      // row-oriented forward substitution; rows past the block compute garbage that no row of
      // the block reads
      cplx v[KBS];
#pragma unroll
      for (int t = 0; t < KBS; ++t) v[t] = V(k0 + min(t, kb - 1));
#pragma unroll
      for (int i = 1; i < KBS; ++i) {
        const int ri = k0 + min(i, kb - 1);
#pragma unroll
        for (int k = 0; k < i; ++k) v[i] = cfms(v[i], E(ri, k0 + min(k, kb - 1)), v[k]);
      }
#pragma unroll
      for (int t = 0; t < KBS; ++t)
        if (t < kb) V(k0 + t) = v[t];
    }
    __syncthreads();
    if (k1 < ns) {
      cplx z[KBS];
#pragma unroll
      for (int t = 0; t < KBS; ++t) z[t] = V(k0 + min(t, kb - 1));
      __builtin_amdgcn_sched_group_barrier(0x020, KBS, 0);   // the KBS loads in flight together
#pragma unroll
      for (int t = 0; t < KBS; ++t) z[t] = cscale(z[t], t < kb ? 1.0 : 0.0);
      for (int i = k1 + c.w; i < ns; i += c.W) {
        cplx v = V(i);
#pragma unroll
        for (int t = 0; t < KBS; ++t) v = cfms(v, E(i, k0 + min(t, kb - 1)), z[t]);
        V(i) = v;
      }
      __syncthreads();
    }
  }
  if (!rows_split) lsolve_rows(fr, base, wv, Fc, ns + SRB * c.w, SRB * c.W);
  for (int a = c.w; a < ns; a += c.W) Y[(int64_t)(fr.col0 + a) * Fc + c.q] = V(a);
#undef E
#undef V
}

template <int RHS>
__global__ __launch_bounds__(512) void k_lsolve_level(DevPattern P, const int* __restrict__ lvl, const cplx* __restrict__ F, int64_t Fc,
                               cplx* __restrict__ WV, RhsArgs R, cplx* __restrict__ Y, const int* __restrict__ reach,
                               int rows_split, const int* __restrict__ glist) {
  int bx;
  Ctx c = ctx_xcd(bx);
  if (!pick_group(c, glist)) return;
  lsolve_front<RHS>(P, P.fronts[lvl[bx]], F, Fc, WV, R, Y, reach, rows_split, c);
}

// Several bottom-up L solves in ONE chain of launches (blockIdx.z = slice): in a loss sweep the forward
// right-hand side over its reach and the three functional vectors aU, aV, aW over theirs (real
// coefficients: the slices' RhsArgs carry rhsP = a_k, mass_sum = 0, beta = 1, no coupling slots), so
// that fr comes from  a_k^T x = (L^-1 a_k)^T diag(U)^-1 (L^-1 b)  without a top-down pass over the
// support's fronts, and the adjoint's bottom-up result is a combination of the slices' (k_fn_combine).
// Workgroups past a slice's front count return at once (the grid is sized for the largest slice).
template <int RHS, bool NAR = false>
__global__ __launch_bounds__(512) void k_lsolve_level_z(DevPattern P, LSlices S, const cplx* __restrict__ F, int64_t Fc,
                                                        int rows_split) {
  extern __shared__ cplx s_piv[];   // NAR: the pivot values (ns x 64)
  int bx;
  const Ctx c = ctx_xcd(bx);
  const int z = blockIdx.z;
  if (bx >= S.nf[z]) return;
  lsolve_front<RHS, NAR>(P, P.fronts[S.lvl[z][bx]], F, Fc, S.WV[z], S.R[z], S.Y[z], S.reach[z], rows_split, c, s_piv);
}

// Update rows of the L solve at the top levels, split over S workgroups per (front, frequency group)
// (launch_solve with split > 1, after k_lsolve_level<..., rows_split = 1> formed the pivot values): at
// small frequency counts one workgroup per front reads the whole L21 block through one CU, bound by
// that CU's memory return rate, while most CUs idle.
__global__ __launch_bounds__(256) void k_lsolve_rows(DevPattern P, const int* __restrict__ lvl, const cplx* __restrict__ F,
                                                     int64_t Fc, cplx* __restrict__ WV, int S, const int* __restrict__ glist) {
  int bx;
  Ctx c = ctx_xcd(bx);
  if (!pick_group(c, glist)) return;
  const int slot = bx / S, split = bx % S;
  const Front fr = P.fronts[lvl[slot]];
  lsolve_rows(fr, F + fr.off * Fc + c.q, WV + (int64_t)fr.row0 * Fc + c.q, Fc, fr.ns + SRB * (split * c.W + c.w),
              SRB * c.W * S);
}

__global__ __launch_bounds__(256) void k_lsolve_rows_z(DevPattern P, LSlices S, const cplx* __restrict__ F, int64_t Fc,
                                                       int split) {
  int bx;
  const Ctx c = ctx_xcd(bx);
  const int z = blockIdx.z;
  const int slot = bx / split, part = bx % split;
  if (slot >= S.nf[z]) return;
  const Front fr = P.fronts[S.lvl[z][slot]];
  lsolve_rows(fr, F + fr.off * Fc + c.q, S.WV[z] + (int64_t)fr.row0 * Fc + c.q, Fc, fr.ns + SRB * (part * c.W + c.w),
              SRB * c.W * split);
}

// The bottom-up update rows on the split levels with the pivot COLUMNS split over the waves (the NAR path): a
// workgroup = LRC_SR update rows of one front x one frequency group x one slice, its LRC_W waves each summing every
// LRC_W-th chunk of LRC_SK pivot columns, the partial sums added in wave order through LDS (k_lsolve_rows_z: each
// wave's rows walk all ns columns, a dependent load round per 8 columns).
constexpr int LRC_SR = 4, LRC_SK = 8, LRC_W = 4;
__global__ __launch_bounds__(64 * LRC_W) void k_lsolve_rows_zc(DevPattern P, LSlices S, const cplx* __restrict__ F,
                                                              int64_t Fc, int RB) {
  int bx;
  const Ctx c = ctx_xcd(bx);
  const int z = blockIdx.z;
  const int slot = bx / RB, rb = bx % RB;
  if (slot >= S.nf[z]) return;
  const Front fr = P.fronts[S.lvl[z][slot]];
  const int f = fr.f, ns = fr.ns;
  const int i0 = ns + rb * LRC_SR;
  if (i0 >= f) return;                          // the whole workgroup (the level's largest front sizes RB)
  const cplx* __restrict__ base = F + fr.off * Fc + c.q;
  cplx* __restrict__ wv = S.WV[z] + (int64_t)fr.row0 * Fc + c.q;
#define E(a, b) base[((int64_t)(a) * f + (b)) * Fc]
#define V(a) wv[(int64_t)(a) * Fc]
  __shared__ cplx part[LRC_W][LRC_SR][64];
  int ri[LRC_SR];
  cplx acc[LRC_SR];
#pragma unroll
  for (int r = 0; r < LRC_SR; ++r) {
    ri[r] = min(i0 + r, f - 1);
    acc[r] = make_double2(0.0, 0.0);
  }
  for (int k0 = LRC_SK * c.w; k0 < ns; k0 += LRC_SK * LRC_W) {
    cplx y[LRC_SK], e[LRC_SR][LRC_SK];
#pragma unroll
    for (int u = 0; u < LRC_SK; ++u) y[u] = V(min(k0 + u, ns - 1));
#pragma unroll
    for (int r = 0; r < LRC_SR; ++r)
#pragma unroll
      for (int u = 0; u < LRC_SK; ++u) e[r][u] = E(ri[r], min(k0 + u, ns - 1));
#pragma unroll
    for (int u = 0; u < LRC_SK; ++u) y[u] = cscale(y[u], k0 + u < ns ? 1.0 : 0.0);
#pragma unroll
    for (int r = 0; r < LRC_SR; ++r)
#pragma unroll
      for (int u = 0; u < LRC_SK; ++u) acc[r] = cfms(acc[r], e[r][u], y[u]);
  }
#pragma unroll
  for (int r = 0; r < LRC_SR; ++r) part[c.w][r][c.lane] = acc[r];
  __syncthreads();
  if (c.w == 0) {
#pragma unroll
    for (int r = 0; r < LRC_SR; ++r)
      if (i0 + r < f) {
        cplx t = V(i0 + r);
        for (int w = 0; w < LRC_W; ++w) t = cadd(t, part[w][r][c.lane]);
        V(i0 + r) = t;
      }
  }
#undef E
#undef V
}

// v - sum_{b in [ns, f)} e[b * es] * X[ix[b]]: the update-row solution values are
// gathered 8 at a time (one scalar index load, then 16 independent vector loads)
__device__ __forceinline__ cplx offdiag_dot(cplx v, const cplx* __restrict__ e, int64_t es,
                                            const cplx* __restrict__ X, const int* __restrict__ ix, int ns, int f,
                                            int64_t Fc, int64_t q) {
  int b = ns;
  for (; b + 8 <= f; b += 8) {
    int iv[8];
    cplx ev[8], xv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) iv[u] = ix[b + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      ev[u] = e[(int64_t)(b + u) * es];
      xv[u] = X[(int64_t)iv[u] * Fc + q];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) v = cfms(v, ev[u], xv[u]);
  }
  for (; b < f; ++b) v = cfms(v, e[(int64_t)b * es], X[(int64_t)ix[b] * Fc + q]);
  return v;
}

// ------------------------------------------------------------------ K3b: U x = y (top-down)
// Pivot rows first take the update-row solution: v_a = y_a - U12(a, :) x_upd, SRB pivot rows
// per wave sharing each gathered x value (SYM: U12(a, b) = U(a, a) L21(b, a), read from L21);
// then U11 backward in KBS blocks, the diagonal block by wave 0 in registers.
// Pivot rows' update part of the U solve: V(a) = y_a + U(a, a) L21(:, a)^T x_upd (SYM) for the pivot
// rows a = a_begin, a_begin + a_step, ... (SRB per step)
template <bool SYM>
__device__ __forceinline__ void usolve_upd(const Front& fr, const int* ix, const cplx* __restrict__ base,
                                           cplx* __restrict__ wv, const cplx* __restrict__ Y, const cplx* __restrict__ X,
                                           int64_t Fc, int64_t q, bool live, int a_begin, int a_step) {
  const int f = fr.f, ns = fr.ns;
  const Ctx c{0, 0, 0, q};
#define E(a, b) base[((int64_t)(a) * f + (b)) * Fc]
#define V(a) wv[(int64_t)(a) * Fc]
  for (int a0 = a_begin; a0 < ns; a0 += a_step) {
    int ra[SRB];
    cplx acc[SRB];
#pragma unroll
    for (int r = 0; r < SRB; ++r) {
      ra[r] = min(a0 + r, ns - 1);
      acc[r] = make_double2(0.0, 0.0);
    }
    // U12(a, b) of pivot row a at pu[a][b * su] (SYM: column a of L21); update-row solution
    // values gathered through wave-uniform (scalar) indices; every load of a chunk issued first
    const cplx* pu[SRB];
#pragma unroll
    for (int r = 0; r < SRB; ++r) pu[r] = base + (SYM ? (int64_t)ra[r] : (int64_t)ra[r] * f) * Fc;
    const int64_t su = SYM ? (int64_t)f * Fc : Fc;
    const cplx* __restrict__ xq = X + c.q;
    for (int b0 = ns; b0 < f; b0 += SKC) {
      int iv[SKC];
      cplx xv[SKC], ev[SRB][SKC];
#pragma unroll
      for (int u = 0; u < SKC; ++u) iv[u] = __builtin_amdgcn_readfirstlane(ix[min(b0 + u, f - 1)]);
#pragma unroll
      for (int u = 0; u < SKC; ++u) xv[u] = xq[(int64_t)iv[u] * Fc];
#pragma unroll
      for (int r = 0; r < SRB; ++r)
#pragma unroll
        for (int u = 0; u < SKC; ++u) ev[r][u] = pu[r][min(b0 + u, f - 1) * su];
      __builtin_amdgcn_sched_group_barrier(0x020, SKC * (SRB + 1), 0);   // all vector loads first
      __builtin_amdgcn_sched_group_barrier(0x002, 4 * SKC * SRB + 8, 0);
#pragma unroll
      for (int u = 0; u < SKC; ++u)
        if (b0 + u >= f) xv[u] = make_double2(0.0, 0.0);
#pragma unroll
      for (int r = 0; r < SRB; ++r)
#pragma unroll
        for (int u = 0; u < SKC; ++u) acc[r] = cfms(acc[r], ev[r][u], xv[u]);
    }
#pragma unroll
    for (int r = 0; r < SRB; ++r)
      if (a0 + r < ns) {
        const cplx y = live ? Y[(int64_t)(fr.col0 + a0 + r) * Fc + c.q] : make_double2(0.0, 0.0);
        V(a0 + r) = SYM ? cadd(y, cmul(E(ra[r], ra[r]), acc[r])) : cadd(y, acc[r]);
      }
  }
#undef E
#undef V
}

template <bool SYM>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void k_usolve_level(DevPattern P, const int* __restrict__ lvl, const cplx* __restrict__ F, int64_t Fc,
                               cplx* __restrict__ WV, const cplx* __restrict__ Y, cplx* __restrict__ X,
                               const int* __restrict__ reach, int upd_done, const int* __restrict__ glist) {
  int bx;
  Ctx c = ctx_xcd(bx);
  if (!pick_group(c, glist)) return;
  const bool live = !reach || reach[lvl[bx]];   // unreached front: y = 0
  const Front fr = P.fronts[lvl[bx]];
  const int f = fr.f, ns = fr.ns;
  const cplx* __restrict__ base = F + fr.off * Fc + c.q;
  cplx* __restrict__ wv = WV + (int64_t)fr.row0 * Fc + c.q;
  // the front's row indices, staged in LDS once: the solution gathers of every pivot row read
  // them there instead of through dependent global loads
  __shared__ int six[MAX_FRONT];
  if (!upd_done) {
    for (int a = threadIdx.x; a < f; a += blockDim.x) six[a] = P.idx[fr.row0 + a];
    __syncthreads();
    usolve_upd<SYM>(fr, six, base, wv, Y, X, Fc, c.q, live, SRB * c.w, SRB * c.W);
  }
  __syncthreads();
#define E(a, b) base[((int64_t)(a) * f + (b)) * Fc]
#define V(a) wv[(int64_t)(a) * Fc]
  for (int k1 = ns; k1 > 0; k1 -= KBS) {
    const int k0 = max(0, k1 - KBS), kb = k1 - k0;
    if (c.w == 0) {
      // row-oriented backward substitution; rows past the block are forced to zero
      cplx v[KBS];
#pragma unroll
      for (int t = 0; t < KBS; ++t) v[t] = V(k0 + min(t, kb - 1));
#pragma unroll
      for (int i = KBS - 1; i >= 0; --i) {
        const int ri = k0 + min(i, kb - 1);
#pragma unroll
        for (int k = i + 1; k < KBS; ++k) v[i] = cfms(v[i], E(ri, k0 + min(k, kb - 1)), v[k]);
        v[i] = cscale(cmul(v[i], crecip(E(ri, ri))), i < kb ? 1.0 : 0.0);
      }
#pragma unroll
      for (int t = 0; t < KBS; ++t)
        if (t < kb) {
          V(k0 + t) = v[t];
          X[(int64_t)(fr.col0 + k0 + t) * Fc + c.q] = v[t];
        }
    }
    __syncthreads();
    if (k0 > 0) {
      cplx x[KBS];
#pragma unroll
      for (int t = 0; t < KBS; ++t) x[t] = V(k0 + min(t, kb - 1));
      __builtin_amdgcn_sched_group_barrier(0x020, KBS, 0);   // the KBS loads in flight together
#pragma unroll
      for (int t = 0; t < KBS; ++t) x[t] = cscale(x[t], t < kb ? 1.0 : 0.0);
      for (int i = c.w; i < k0; i += c.W) {
        cplx v = V(i);
#pragma unroll
        for (int t = 0; t < KBS; ++t) v = cfms(v, E(i, k0 + min(t, kb - 1)), x[t]);
        V(i) = v;
      }
      __syncthreads();
    }
  }
#undef E
#undef V
}

// the pivot rows' update part of k_usolve_level split over S workgroups per (front, frequency group)
template <bool SYM>
__global__ __launch_bounds__(256) void k_usolve_upd(DevPattern P, const int* __restrict__ lvl, const cplx* __restrict__ F,
                                                    int64_t Fc, cplx* __restrict__ WV, const cplx* __restrict__ Y,
                                                    const cplx* __restrict__ X, const int* __restrict__ reach, int S,
                                                    const int* __restrict__ glist) {
  int bx;
  Ctx c = ctx_xcd(bx);
  if (!pick_group(c, glist)) return;
  const int slot = bx / S, split = bx % S;
  const bool live = !reach || reach[lvl[slot]];
  const Front fr = P.fronts[lvl[slot]];
  __shared__ int six[MAX_FRONT];
  for (int a = threadIdx.x; a < fr.f; a += blockDim.x) six[a] = P.idx[fr.row0 + a];
  __syncthreads();
  usolve_upd<SYM>(fr, six, F + fr.off * Fc + c.q, WV + (int64_t)fr.row0 * Fc + c.q, Y, X, Fc, c.q, live,
                  SRB * (split * c.W + c.w), SRB * c.W * S);
}

// ------------------------------------------------------------------ K3b': two top-down solves in one pass
// U x = y for two right-hand sides on the same factors (symmetric mode: the forward solution x
// and the adjoint lambda), each L21 / U11 value loaded once for both.  Vector v is computed on
// the fronts where act = !skip[front] (the forward pass is skipped on the fronts it was already
// solved on, those the loss support reaches); its y is zero on fronts outside reach.  X itself
// is the scratch of a front's pivot values.
struct UPair {
  const cplx* Y;
  cplx* X;
  const int* reach;   // y non-zero only on these fronts (NULL = all)
  const int* skip;    // fronts this vector is not computed on (NULL = none)
};

// SR pivot rows per wave sharing each gathered solution value, SK values per chunk, WPE waves per
// SIMD: (4, 8, 2) for the levels of large fronts; (2, 4, 4) for levels of small fronts, where the
// many tiny workgroups are latency-bound and occupancy, not per-wave reuse, hides it.
// the pivot rows' update part of the paired pass: XV(v, a) = y_a + U(a, a) L21(:, a)^T x_upd for
// a = a_begin, a_begin + a_step, ... (SR per step)
template <bool SYM, int SR, int SK>
__device__ __forceinline__ void usolve2_upd(const Front& fr, const int* six, const cplx* __restrict__ base,
                                            int64_t Fc, int64_t q, const bool (&act)[2], const bool (&live)[2],
                                            const cplx* const (&Ys)[2], cplx* const (&Xs)[2], int a_begin, int a_step) {
  const int f = fr.f, ns = fr.ns;
  const Ctx c{0, 0, 0, q};
#define E(a, b) base[((int64_t)(a) * f + (b)) * Fc]
#define XV(v, a) Xs[v][(int64_t)(fr.col0 + (a)) * Fc + c.q]
  for (int a0 = a_begin; a0 < ns; a0 += a_step) {
    int ra[SR];
    cplx acc[2][SR];
#pragma unroll
    for (int r = 0; r < SR; ++r) {
      ra[r] = min(a0 + r, ns - 1);
      acc[0][r] = acc[1][r] = make_double2(0.0, 0.0);
    }
    const cplx* pu[SR];
#pragma unroll
    for (int r = 0; r < SR; ++r) pu[r] = base + (SYM ? (int64_t)ra[r] : (int64_t)ra[r] * f) * Fc;
    const int64_t su = SYM ? (int64_t)f * Fc : Fc;
    for (int b0 = ns; b0 < f; b0 += SK) {
      int iv[SK];
      cplx xv[2][SK], ev[SR][SK];
#pragma unroll
      for (int u = 0; u < SK; ++u) iv[u] = __builtin_amdgcn_readfirstlane(six[min(b0 + u, f - 1)]);
#pragma unroll
      for (int v = 0; v < 2; ++v)
#pragma unroll
        for (int u = 0; u < SK; ++u) xv[v][u] = Xs[v][(int64_t)iv[u] * Fc + c.q];   // inactive: unused
#pragma unroll
      for (int r = 0; r < SR; ++r)
#pragma unroll
        for (int u = 0; u < SK; ++u) ev[r][u] = pu[r][min(b0 + u, f - 1) * su];
      __builtin_amdgcn_sched_group_barrier(0x020, SK * (SR + 2), 0);   // all vector loads first
      __builtin_amdgcn_sched_group_barrier(0x002, 8 * SK * SR + 16, 0);
#pragma unroll
      for (int v = 0; v < 2; ++v)
#pragma unroll
        for (int u = 0; u < SK; ++u)
          if (b0 + u >= f) xv[v][u] = make_double2(0.0, 0.0);
#pragma unroll
      for (int v = 0; v < 2; ++v)
#pragma unroll
        for (int r = 0; r < SR; ++r)
#pragma unroll
          for (int u = 0; u < SK; ++u) acc[v][r] = cfms(acc[v][r], ev[r][u], xv[v][u]);
    }
#pragma unroll
    for (int r = 0; r < SR; ++r)
      if (a0 + r < ns) {
        const cplx urr = SYM ? E(ra[r], ra[r]) : make_double2(1.0, 0.0);
#pragma unroll
        for (int v = 0; v < 2; ++v)
          if (act[v]) {
            const cplx y = live[v] ? Ys[v][(int64_t)(fr.col0 + a0 + r) * Fc + c.q] : make_double2(0.0, 0.0);
            XV(v, a0 + r) = SYM ? cadd(y, cmul(urr, acc[v][r])) : cadd(y, acc[v][r]);
          }
      }
  }
#undef E
#undef XV
}

// U11 backward for the pivot values XV(v, 0 .. ns) the update part left there: KBS blocks, the diagonal
// block by wave 0 in registers, the rows above updated by all waves
__device__ __forceinline__ void usolve2_tri(const Front& fr, const cplx* __restrict__ base, int64_t Fc, const Ctx& c,
                                            const bool (&act)[2], cplx* const (&Xs)[2]) {
  const int f = fr.f, ns = fr.ns;
#define E(a, b) base[((int64_t)(a) * f + (b)) * Fc]
#define XV(v, a) Xs[v][(int64_t)(fr.col0 + (a)) * Fc + c.q]
  for (int k1 = ns; k1 > 0; k1 -= KBS) {
    const int k0 = max(0, k1 - KBS), kb = k1 - k0;
    if (c.w == 0) {
#pragma unroll
      for (int v = 0; v < 2; ++v)
        if (act[v]) {
          cplx x[KBS];
#pragma unroll
          for (int t = 0; t < KBS; ++t) x[t] = XV(v, k0 + min(t, kb - 1));
#pragma unroll
          for (int i = KBS - 1; i >= 0; --i) {
            const int ri = k0 + min(i, kb - 1);
#pragma unroll
            for (int k = i + 1; k < KBS; ++k) x[i] = cfms(x[i], E(ri, k0 + min(k, kb - 1)), x[k]);
            x[i] = cscale(cmul(x[i], crecip(E(ri, ri))), i < kb ? 1.0 : 0.0);
          }
#pragma unroll
          for (int t = 0; t < KBS; ++t)
            if (t < kb) XV(v, k0 + t) = x[t];
        }
    }
    __syncthreads();
    if (k0 > 0) {
#pragma unroll
      for (int v = 0; v < 2; ++v)
        if (act[v]) {
          cplx x[KBS];
#pragma unroll
          for (int t = 0; t < KBS; ++t) x[t] = XV(v, k0 + min(t, kb - 1));
          __builtin_amdgcn_sched_group_barrier(0x020, KBS, 0);   // the KBS loads in flight together
#pragma unroll
          for (int t = 0; t < KBS; ++t) x[t] = cscale(x[t], t < kb ? 1.0 : 0.0);
          for (int i = c.w; i < k0; i += c.W) {
            cplx y = XV(v, i);
#pragma unroll
            for (int t = 0; t < KBS; ++t) y = cfms(y, E(i, k0 + min(t, kb - 1)), x[t]);
            XV(v, i) = y;
          }
        }
      __syncthreads();
    }
  }
#undef E
#undef XV
}


template <bool SYM, int SR, int SK, int WPE>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(WPE))) void k_usolve2_level(
    DevPattern P, const int* __restrict__ lvl, const cplx* __restrict__ F, int64_t Fc, UPair A, UPair B, int upd_done) {
  int bx;
  const Ctx c = ctx_xcd(bx);
  const int ft = lvl[bx];
  const bool act[2] = {!A.skip || !A.skip[ft], !B.skip || !B.skip[ft]};
  const bool live[2] = {!A.reach || A.reach[ft], !B.reach || B.reach[ft]};
  const cplx* const Ys[2] = {A.Y, B.Y};
  cplx* const Xs[2] = {A.X, B.X};
  const Front fr = P.fronts[ft];
  const int f = fr.f;
  const cplx* __restrict__ base = F + fr.off * Fc + c.q;
  __shared__ int six[MAX_FRONT];
  if (!upd_done) {
    for (int a = threadIdx.x; a < f; a += blockDim.x) six[a] = P.idx[fr.row0 + a];
    __syncthreads();
    usolve2_upd<SYM, SR, SK>(fr, six, base, Fc, c.q, act, live, Ys, Xs, SR * c.w, SR * c.W);
  }
  __syncthreads();
  usolve2_tri(fr, base, Fc, c, act, Xs);
}

// Pivot-block triangular solves of the narrow levels, RIGHT-looking by single pivots with the factor entries
// prefetched: a workgroup = one front x 16 frequencies, W waves, lane = (one of 16 frequencies, one of 4 row slots);
// the lane of slot s = 4 w + (lane >> 4) owns rows i = s + 4 W r (r < RPL) and keeps their running sums acc[v][r] in
// registers.  Per pivot p (UP: ns - 1 .. 0, U11 backward, x_p = acc_p / U(p, p), then acc_i -= U(i, p) x_p on the
// rows i < p; !UP: 0 .. ns - 1, unit L11 forward, y_p = acc_p, then acc_i -= L(i, p) y_p on the rows p < i < ns) the
// owner forms x_p, stores it and broadcasts it through LDS: one barrier per pivot.  Every lane's column entries
// E(i, p) of the next PF pivots are already in registers (a ring loaded PF pivots ahead, independent of the chain),
// so the chain carries no global-memory latency -- the left-looking form of round 5 (the pivot values in LDS, per
// 8-pivot block the rows' sums over the solved columns, then wave 0's triangle) waited on about two global round
// trips per block: the paired pass's 28 narrow levels 1.06 -> 0.67 ms per 2,048-frequency chunk.  The 16-frequency workgroups also give the narrow levels 4x the workgroups.
// dst[v] (and dst2 for vector 0 when not NULL): the solution's pivot rows (already offset by the first pivot row and the lane's
// frequency).
constexpr int RL_Q = 16, RL_WMAX = 8, RL_RING = 16;   // ring entries per lane: PF = RL_RING / RPL pivots ahead
// rows per lane slot for a level whose largest pivot block is maxns (1, 2 or 4: maxns <= 128), and the waves
inline int rl_rpl(int maxns) { return maxns <= 4 * RL_WMAX ? 1 : maxns <= 8 * RL_WMAX ? 2 : 4; }
inline int rl_waves(int maxns) { return std::min(RL_WMAX, (maxns + 4 * rl_rpl(maxns) - 1) / (4 * rl_rpl(maxns))); }
template <bool UP, int NV, int RPL, int PF>
__device__ __forceinline__ void tri_rl16(const cplx* __restrict__ base, int f, int ns, int64_t Fc, int w, int W,
                                         int lane, const bool (&act)[NV], cplx (&acc)[NV][RPL],
                                         cplx* const (&dst)[NV], cplx (*sx)[NV][RL_Q],
                                         cplx* __restrict__ dst2 = nullptr) {
  const int slot = 4 * w + (lane >> 4), nsl = 4 * W, ql = lane & (RL_Q - 1);
  int ir[RPL], ic[RPL];
#pragma unroll
  for (int r = 0; r < RPL; ++r) {
    ir[r] = slot + nsl * r;
    ic[r] = min(ir[r], ns - 1);
  }
  cplx dinv[RPL];
#pragma unroll
  for (int r = 0; r < RPL; ++r) dinv[r] = UP ? crecip(base[((int64_t)ic[r] * f + ic[r]) * Fc]) : make_double2(1.0, 0.0);
  cplx pre[PF][RPL];
  // the ring's next column pointer per row (the pivot of step t + PF, clamped into the block), advanced by one
  // column per step; the owner slot p % nsl likewise (no per-step index arithmetic: every wave of every
  // workgroup runs each step's instructions, so they set the step time)
  // A row uses the column entry of pivot p only on one side of the diagonal (UP: rows i < p; !UP: rows i > p); on the
  // other side its ring loads its own diagonal entry instead (one address, cached), so the ring reads the factor
  // triangle once rather than whole columns: column max(p, i) (UP) / min(p, i) (!UP) of row i.
  const int64_t dcol = UP ? -Fc : Fc;
  const cplx* lp[RPL];
  auto col = [&](int t) { const int tc = min(t, ns - 1); return UP ? ns - 1 - tc : tc; };
  auto cc = [&](int t, int i) { return UP ? max(col(t), i) : min(col(t), i); };
#pragma unroll
  for (int r = 0; r < RPL; ++r) lp[r] = base + (int64_t)ic[r] * f * Fc;
#pragma unroll
  for (int u = 0; u < PF; ++u)
#pragma unroll
    for (int r = 0; r < RPL; ++r) pre[u][r] = lp[r][(int64_t)cc(u, ic[r]) * Fc];
#pragma unroll
  for (int r = 0; r < RPL; ++r) lp[r] += (int64_t)cc(PF, ic[r]) * Fc;
  int os = col(0) % nsl;
  // one pivot step t with the column entries e; the owner's solved value through LDS (buffer t & 1)
  auto step = [&](int t, const cplx (&e)[RPL]) {
    const int p = UP ? ns - 1 - t : t, par = t & 1;
    // the owner lane (row ir[r] == p) turns acc into x_p and broadcasts it; every row's candidate is formed and the
    // owner's picked by lane predicates (an index by p / nsl makes the compiler address acc in scratch memory)
    if (slot == os) {
#pragma unroll
      for (int v = 0; v < NV; ++v)
        if (act[v]) {
          cplx xs = make_double2(0.0, 0.0);
#pragma unroll
          for (int r = 0; r < RPL; ++r) {
            const bool own = ir[r] == p;
            const cplx x = UP ? cmul(acc[v][r], dinv[r]) : acc[v][r];
            acc[v][r].x = own ? x.x : acc[v][r].x;
            acc[v][r].y = own ? x.y : acc[v][r].y;
            xs.x = own ? x.x : xs.x;
            xs.y = own ? x.y : xs.y;
          }
          sx[par][v][ql] = xs;
        }
    }
    os = UP ? (os == 0 ? nsl - 1 : os - 1) : (os == nsl - 1 ? 0 : os + 1);
    PFR_BARRIER();
#pragma unroll
    for (int v = 0; v < NV; ++v)
      if (act[v]) {
        const cplx x = sx[par][v][ql];
#pragma unroll
        for (int r = 0; r < RPL; ++r)
          if (UP ? ir[r] < p : (ir[r] > p && ir[r] < ns)) acc[v][r] = cfms(acc[v][r], e[r], x);
      }
  };
  // whole rounds of PF steps (the ring slot u refilled PF steps ahead: straight-line code, so that the waits on
  // the ring are counted, not drained), then the tail from the ring without refills
  int t0 = 0;
  for (; t0 + PF <= ns; t0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      cplx e[RPL];
      const int tn = t0 + u + PF + 1, pn = UP ? ns - 1 - tn : tn;   // the pointers move to step tn's column
#pragma unroll
      for (int r = 0; r < RPL; ++r) {
        e[r] = pre[u][r];
        pre[u][r] = *lp[r];
        if (tn < ns && (UP ? pn >= ic[r] : pn <= ic[r])) lp[r] += dcol;
      }
      step(t0 + u, e);
    }
  }
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (t0 + u < ns) step(t0 + u, pre[u]);
  // every lane's solved rows out
#pragma unroll
  for (int v = 0; v < NV; ++v)
    if (act[v])
#pragma unroll
      for (int r = 0; r < RPL; ++r)
        if (ir[r] < ns) {
          dst[v][(int64_t)ir[r] * Fc] = acc[v][r];
          if (dst2 && v == 0) dst2[(int64_t)ir[r] * Fc] = acc[v][r];
        }
}

// The paired top-down pass's pivot blocks on the narrow levels (after k_usolve2_updc left y_a + U12(a, :) x_upd in
// X): tri_rl16 over both vectors.  Grid (fronts, Fc / 16), 64 W threads with 4 W RPL >= the level's largest ns.
template <int RPL>
__global__ __launch_bounds__(64 * RL_WMAX) void k_usolve2_rl(DevPattern P, const int* __restrict__ lvl,
                                                    const cplx* __restrict__ F, int64_t Fc, UPair A, UPair B) {
  __shared__ cplx sx[2][2][RL_Q];
  const int64_t lid = xcd_swizzle(blockIdx.x + (int64_t)gridDim.x * blockIdx.y, (int64_t)gridDim.x * gridDim.y);
  const int bx = (int)(lid % gridDim.x);
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), W = blockDim.x >> 6;
  const int64_t q = (lid / gridDim.x) * RL_Q + (lane & (RL_Q - 1));
  const int ft = lvl[bx];
  const bool act[2] = {!A.skip || !A.skip[ft], !B.skip || !B.skip[ft]};
  const Front fr = P.fronts[ft];
  const int ns = fr.ns;
  cplx* const dst[2] = {A.X + (int64_t)fr.col0 * Fc + q, B.X + (int64_t)fr.col0 * Fc + q};
  cplx acc[2][RPL];
  const int slot = 4 * w + (lane >> 4);
#pragma unroll
  for (int r = 0; r < RPL; ++r) {
    const int i = min(slot + 4 * W * r, ns - 1);
#pragma unroll
    for (int v = 0; v < 2; ++v) acc[v][r] = act[v] ? dst[v][(int64_t)i * Fc] : make_double2(0.0, 0.0);
  }
  tri_rl16<true, 2, RPL, RL_RING / RPL>(F + fr.off * Fc + q, fr.f, ns, Fc, w, W, lane, act, acc, dst, sx);
}

// The bottom-up chain's pivot blocks on the narrow levels (k_lsolve_level_z<., true>'s role, the update rows left to
// k_lsolve_rows_zc): per (front, 16 frequencies, slice) the frontal vector gathered -- pivot rows into the owning
// lanes' registers, update rows into WV -- then tri_rl16's unit forward substitution, y to Y and to WV's pivot rows.
// Grid (largest slice's fronts, Fc / 16, slices), 64 W threads with 4 W RPL >= the level's largest ns.
template <int RHS, int RPL>
__global__ __launch_bounds__(64 * RL_WMAX) void k_lsolve_rl_z(DevPattern P, LSlices S, const cplx* __restrict__ F, int64_t Fc) {
  __shared__ cplx sx[2][1][RL_Q];
  __shared__ int s_ptr[MAX_FRONT + 1];
  __shared__ int s_src[GATHER_CAP];
  __shared__ int s_p[MAX_FRONT];
  __shared__ double s_rv[MAX_FRONT];
  __shared__ int s_cs[MAX_FRONT];
  const int64_t lid = xcd_swizzle(blockIdx.x + (int64_t)gridDim.x * blockIdx.y, (int64_t)gridDim.x * gridDim.y);
  const int bx = (int)(lid % gridDim.x), z = blockIdx.z;
  if (bx >= S.nf[z]) return;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), W = blockDim.x >> 6;
  const int64_t q = (lid / gridDim.x) * RL_Q + (lane & (RL_Q - 1));
  const Front fr = P.fronts[S.lvl[z][bx]];
  const int f = fr.f, ns = fr.ns, slot = 4 * w + (lane >> 4), nsl = 4 * W;
  const RhsArgs& R = S.R[z];
  const int* __restrict__ reach = S.reach[z];
  cplx* __restrict__ WV = S.WV[z];
  // the frontal gather (gather_frontal's chains resolved into LDS by all threads; rows per lane slot, so the row
  // indices are not wave-uniform here)
  const int E0 = P.ea_ptr[fr.row0], nE = P.ea_ptr[fr.row0 + f] - E0;
  const bool staged = nE <= GATHER_CAP;
  if (staged) {
    for (int t = threadIdx.x; t <= f; t += blockDim.x) s_ptr[t] = P.ea_ptr[fr.row0 + t] - E0;
    for (int t = threadIdx.x; t < nE; t += blockDim.x) {
      const int src = P.ea_src[E0 + t];
      s_src[t] = (!reach || reach[P.row_front[src]]) ? src : -1;
    }
  }
  for (int t = threadIdx.x; t < ns; t += blockDim.x) {
    const int p = P.idx[fr.row0 + t];
    s_p[t] = p;
    s_rv[t] = R.rhsP[p];
    s_cs[t] = RHS == 3 ? R.cslot[p] : -1;
  }
  const double om = 6.283185307179586 * R.freqs[q], om2 = om * om;
  __syncthreads();
  auto gather = [&](int a) {
    cplx v = make_double2(0.0, 0.0);
    if (a < ns) v = rhs_staged<RHS>(R, s_p[a], s_rv[a], s_cs[a], om2, q, Fc);
    if (staged) {
      for (int e = s_ptr[a]; e < s_ptr[a + 1]; ++e) {
        const int src = s_src[e];
        if (src >= 0) v = cadd(v, WV[(int64_t)src * Fc + q]);
      }
    } else {
      for (int e = P.ea_ptr[fr.row0 + a]; e < P.ea_ptr[fr.row0 + a + 1]; ++e) {
        const int src = P.ea_src[e];
        if (!reach || reach[P.row_front[src]]) v = cadd(v, WV[(int64_t)src * Fc + q]);
      }
    }
    return v;
  };
  // pivot rows through LDS to their owners (gathered by row slot like the update rows, which go to WV)
  __shared__ cplx s_b[4 * RL_WMAX * RPL][RL_Q];
  for (int a = slot; a < f; a += nsl) {
    const cplx v = gather(a);
    if (a < ns) s_b[a][lane & (RL_Q - 1)] = v;
    else WV[(int64_t)(fr.row0 + a) * Fc + q] = v;
  }
  __syncthreads();
  cplx acc[1][RPL];
#pragma unroll
  for (int r = 0; r < RPL; ++r) acc[0][r] = s_b[min(slot + nsl * r, ns - 1)][lane & (RL_Q - 1)];
  const bool act[1] = {true};
  cplx* const dst[1] = {S.Y[z] + (int64_t)fr.col0 * Fc + q};
  tri_rl16<false, 1, RPL, RL_RING / RPL>(F + fr.off * Fc + q, f, ns, Fc, w, W, lane, act, acc, dst, sx,
                                         WV + (int64_t)fr.row0 * Fc + q);
}

// The paired top-down pass on levels of tiny fronts (every pivot block <= NSM): ONE WAVE per (front, frequency
// group), four fronts per workgroup, no LDS and no barrier -- the pivot rows' update sums and the U11 backward
// solve in registers.  k_usolve2_level gives each of the bottom levels' ~3,000 fronts x 32 groups a workgroup
// whose waves meet at two barriers and pass the pivot values through global memory; here a front is one
// wave's independent task (more of them resident per CU, each a shorter dependent chain).  Operations per
// value and their order are k_usolve2_level's (update columns ascending, then the pivot block bottom-up), so
// the results are identical bit for bit.
template <int NSM>   // NSM <= KBS: the level kernel's pivot block is one KBS block, solved in the order below
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NSM <= 4 ? 6 : 3))) void k_usolve2_tiny(
    DevPattern P, const int* __restrict__ lvl, int nfronts, const cplx* __restrict__ F, int64_t Fc, UPair A, UPair B) {
  static_assert(NSM <= KBS, "one pivot block of the level kernel's triangular solve");
  int bx;
  const Ctx c = ctx_xcd(bx);
  const int slot = bx * 4 + c.w;
  if (slot >= nfronts) return;
  const int ft = lvl[slot];
  const bool act[2] = {!A.skip || !A.skip[ft], !B.skip || !B.skip[ft]};
  const bool live[2] = {!A.reach || A.reach[ft], !B.reach || B.reach[ft]};
  const cplx* const Ys[2] = {A.Y, B.Y};
  cplx* const Xs[2] = {A.X, B.X};
  const Front fr = P.fronts[ft];
  const int f = fr.f, ns = fr.ns;
  const cplx* __restrict__ base = F + fr.off * Fc + c.q;
  const int* __restrict__ ix = P.idx + fr.row0;
#define E(a, b) base[((int64_t)(a) * f + (b)) * Fc]
  cplx acc[2][NSM];
#pragma unroll
  for (int a = 0; a < NSM; ++a) acc[0][a] = acc[1][a] = make_double2(0.0, 0.0);
  for (int b = ns; b < f; ++b) {
    const int iv = __builtin_amdgcn_readfirstlane(ix[b]);
    const cplx x0 = Xs[0][(int64_t)iv * Fc + c.q], x1 = Xs[1][(int64_t)iv * Fc + c.q];
    cplx e[NSM];
#pragma unroll
    for (int a = 0; a < NSM; ++a) e[a] = E(b, min(a, ns - 1));
#pragma unroll
    for (int a = 0; a < NSM; ++a) {
      acc[0][a] = cfms(acc[0][a], e[a], x0);
      acc[1][a] = cfms(acc[1][a], e[a], x1);
    }
  }
  // z_a = y_a + U(a, a) acc_a, then U11 z = ... bottom-up (k_usolve2_level's pivot block, ns <= KBS)
  cplx z[2][NSM];
#pragma unroll
  for (int a = 0; a < NSM; ++a) {
    const int ra = min(a, ns - 1);
    const cplx urr = E(ra, ra);
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const cplx y = live[v] ? Ys[v][(int64_t)(fr.col0 + ra) * Fc + c.q] : make_double2(0.0, 0.0);
      z[v][a] = cadd(y, cmul(urr, acc[v][a]));
    }
  }
#pragma unroll
  for (int i = NSM - 1; i >= 0; --i)
    if (i < ns) {
#pragma unroll
      for (int k = i + 1; k < NSM; ++k)
        if (k < ns) {
          const cplx u = E(i, k);
#pragma unroll
          for (int v = 0; v < 2; ++v) z[v][i] = cfms(z[v][i], u, z[v][k]);
        }
      const cplx d = crecip(E(i, i));
#pragma unroll
      for (int v = 0; v < 2; ++v) z[v][i] = cmul(z[v][i], d);
    }
#pragma unroll
  for (int v = 0; v < 2; ++v)
    if (act[v]) {
#pragma unroll
      for (int a = 0; a < NSM; ++a)
        if (a < ns) Xs[v][(int64_t)(fr.col0 + a) * Fc + c.q] = z[v][a];
    }
#undef E
}

// The pivot rows' update part on the split levels with the update COLUMNS split over the waves (the NAR path):
// a workgroup = UPC_SR pivot rows of one front x one frequency group, its UPC_W waves each summing every
// UPC_W-th chunk of UPC_SK update columns for those rows (each chunk's gathers and L21 loads independent of the
// others), the partial sums added in wave order through LDS.  k_usolve2_upd gives each wave a row pair and the
// whole column range: r / 4 dependent load rounds per wave (16-18 on the narrow levels of C3, 22-64 us per level).
constexpr int UPC_SR = 2, UPC_SK = 8, UPC_W = 8;
__global__ __launch_bounds__(64 * UPC_W) void k_usolve2_updc(DevPattern P, const int* __restrict__ lvl,
                                                            const cplx* __restrict__ F, int64_t Fc, UPair A, UPair B,
                                                            int RB) {
  int bx;
  const Ctx c = ctx_xcd(bx);
  const int slot = bx / RB, rb = bx % RB;
  const int ft = lvl[slot];
  const Front fr = P.fronts[ft];
  const int f = fr.f, ns = fr.ns;
  const int a0 = rb * UPC_SR;
  if (a0 >= ns) return;                         // the whole workgroup (the level's largest pivot block sizes RB)
  const bool act[2] = {!A.skip || !A.skip[ft], !B.skip || !B.skip[ft]};
  const bool live[2] = {!A.reach || A.reach[ft], !B.reach || B.reach[ft]};
  const cplx* const Ys[2] = {A.Y, B.Y};
  cplx* const Xs[2] = {A.X, B.X};
  const cplx* __restrict__ base = F + fr.off * Fc + c.q;
  __shared__ int six[MAX_FRONT];
  __shared__ cplx part[UPC_W][2][UPC_SR][64];
  for (int a = threadIdx.x; a < f; a += blockDim.x) six[a] = P.idx[fr.row0 + a];
  __syncthreads();
  int ra[UPC_SR];
  const cplx* pu[UPC_SR];
#pragma unroll
  for (int r = 0; r < UPC_SR; ++r) {
    ra[r] = min(a0 + r, ns - 1);
    pu[r] = base + (int64_t)ra[r] * Fc;         // column ra of L21: E(b, ra) at pu + b f Fc
  }
  const int64_t su = (int64_t)f * Fc;
  cplx acc[2][UPC_SR];
#pragma unroll
  for (int v = 0; v < 2; ++v)
#pragma unroll
    for (int r = 0; r < UPC_SR; ++r) acc[v][r] = make_double2(0.0, 0.0);
  for (int b0 = ns + UPC_SK * c.w; b0 < f; b0 += UPC_SK * UPC_W) {
    int iv[UPC_SK];
    cplx xv[2][UPC_SK], ev[UPC_SR][UPC_SK];
#pragma unroll
    for (int u = 0; u < UPC_SK; ++u) iv[u] = __builtin_amdgcn_readfirstlane(six[min(b0 + u, f - 1)]);
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
      for (int u = 0; u < UPC_SK; ++u) xv[v][u] = Xs[v][(int64_t)iv[u] * Fc + c.q];   // inactive: unused
#pragma unroll
    for (int r = 0; r < UPC_SR; ++r)
#pragma unroll
      for (int u = 0; u < UPC_SK; ++u) ev[r][u] = pu[r][min(b0 + u, f - 1) * su];
#pragma unroll
    for (int u = 0; u < UPC_SK; ++u) {
      const double m = b0 + u < f ? 1.0 : 0.0;
#pragma unroll
      for (int v = 0; v < 2; ++v) xv[v][u] = cscale(xv[v][u], m);
    }
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
      for (int r = 0; r < UPC_SR; ++r)
#pragma unroll
        for (int u = 0; u < UPC_SK; ++u) acc[v][r] = cfms(acc[v][r], ev[r][u], xv[v][u]);
  }
#pragma unroll
  for (int v = 0; v < 2; ++v)
#pragma unroll
    for (int r = 0; r < UPC_SR; ++r) part[c.w][v][r][c.lane] = acc[v][r];
  __syncthreads();
  if (c.w == 0) {
#pragma unroll
    for (int r = 0; r < UPC_SR; ++r)
      if (a0 + r < ns) {
        const cplx urr = base[((int64_t)ra[r] * f + ra[r]) * Fc];
#pragma unroll
        for (int v = 0; v < 2; ++v)
          if (act[v]) {
            cplx t = part[0][v][r][c.lane];
            for (int w = 1; w < UPC_W; ++w) t = cadd(t, part[w][v][r][c.lane]);
            const cplx y = live[v] ? Ys[v][(int64_t)(fr.col0 + a0 + r) * Fc + c.q] : make_double2(0.0, 0.0);
            Xs[v][(int64_t)(fr.col0 + a0 + r) * Fc + c.q] = cadd(y, cmul(urr, t));
          }
      }
  }
}

// the pivot rows' update part of k_usolve2_level split over S workgroups per (front, frequency group)
template <bool SYM, int SR, int SK>
__global__ __launch_bounds__(256) void k_usolve2_upd(DevPattern P, const int* __restrict__ lvl, const cplx* __restrict__ F,
                                                     int64_t Fc, UPair A, UPair B, int S) {
  int bx;
  const Ctx c = ctx_xcd(bx);
  const int slot = bx / S, split = bx % S;
  const int ft = lvl[slot];
  const bool act[2] = {!A.skip || !A.skip[ft], !B.skip || !B.skip[ft]};
  const bool live[2] = {!A.reach || A.reach[ft], !B.reach || B.reach[ft]};
  const cplx* const Ys[2] = {A.Y, B.Y};
  cplx* const Xs[2] = {A.X, B.X};
  const Front fr = P.fronts[ft];
  __shared__ int six[MAX_FRONT];
  for (int a = threadIdx.x; a < fr.f; a += blockDim.x) six[a] = P.idx[fr.row0 + a];
  __syncthreads();
  usolve2_upd<SYM, SR, SK>(fr, six, F + fr.off * Fc + c.q, Fc, c.q, act, live, Ys, Xs, SR * (split * c.W + c.w),
                           SR * c.W * S);
}

// ------------------------------------------------------------------ K3c: U^T y = g (bottom-up)
template <int RHS>
__global__ __launch_bounds__(512) void k_utsolve_level(DevPattern P, const int* __restrict__ lvl, const cplx* __restrict__ F, int64_t Fc,
                                cplx* __restrict__ WV, RhsArgs R, cplx* __restrict__ Y, const int* __restrict__ reach) {
  int bx;
  const Ctx c = ctx_xcd(bx);
  const Front fr = P.fronts[lvl[bx]];
  const int f = fr.f, ns = fr.ns;
  const cplx* __restrict__ base = F + fr.off * Fc + c.q;
  cplx* __restrict__ wv = WV + (int64_t)fr.row0 * Fc + c.q;
#define E(a, b) base[((int64_t)(a) * f + (b)) * Fc]
#define V(a) wv[(int64_t)(a) * Fc]
  gather_frontal<RHS>(P, fr, R, WV, Fc, c, reach);
  __syncthreads();
  for (int k0 = 0; k0 < ns; k0 += KBS) {
    const int kb = min(KBS, ns - k0), k1 = k0 + kb;
    if (c.w == 0)
      for (int k = k0; k < k1; ++k) {
        const cplx y = cmul(V(k), crecip(E(k, k)));
        V(k) = y;
        for (int i = k + 1; i < k1; ++i) V(i) = cfms(V(i), E(k, i), y);
      }
    __syncthreads();
    cplx y[KBS];
#pragma unroll
    for (int t = 0; t < KBS; ++t)
      if (t < kb) y[t] = V(k0 + t);
    for (int i = k1 + c.w; i < f; i += c.W) {
      cplx v = V(i);
#pragma unroll
      for (int t = 0; t < KBS; ++t)
        if (t < kb) v = cfms(v, E(k0 + t, i), y[t]);
      V(i) = v;
    }
    __syncthreads();
  }
  for (int a = c.w; a < ns; a += c.W) Y[(int64_t)(fr.col0 + a) * Fc + c.q] = V(a);
#undef E
#undef V
}

// ------------------------------------------------------------------ K3d: L^T x = y (top-down)
__global__ __launch_bounds__(512) void k_ltsolve_level(DevPattern P, const int* __restrict__ lvl, const cplx* __restrict__ F, int64_t Fc,
                                cplx* __restrict__ WV, const cplx* __restrict__ Y, cplx* __restrict__ X,
                               const int* __restrict__ reach) {
  int bx;
  const Ctx c = ctx_xcd(bx);
  const bool live = !reach || reach[lvl[bx]];   // unreached front: y = 0
  const Front fr = P.fronts[lvl[bx]];
  const int f = fr.f, ns = fr.ns;
  const cplx* __restrict__ base = F + fr.off * Fc + c.q;
  cplx* __restrict__ wv = WV + (int64_t)fr.row0 * Fc + c.q;
  const int* __restrict__ ix = P.idx + fr.row0;
#define E(a, b) base[((int64_t)(a) * f + (b)) * Fc]
#define V(a) wv[(int64_t)(a) * Fc]
  for (int a = c.w; a < ns; a += c.W) {
    cplx v = live ? Y[(int64_t)(fr.col0 + a) * Fc + c.q] : make_double2(0.0, 0.0);
    v = offdiag_dot(v, &E(0, a), (int64_t)f * Fc, X, ix, ns, f, Fc, c.q);
    V(a) = v;
  }
  __syncthreads();
  for (int k1 = ns; k1 > 0; k1 -= KBS) {
    const int k0 = max(0, k1 - KBS), kb = k1 - k0;
    if (c.w == 0)
      for (int k = k1 - 1; k >= k0; --k) {
        const cplx x = V(k);
        X[(int64_t)(fr.col0 + k) * Fc + c.q] = x;
        for (int i = k0; i < k; ++i) V(i) = cfms(V(i), E(k, i), x);
      }
    __syncthreads();
    cplx x[KBS];
#pragma unroll
    for (int t = 0; t < KBS; ++t)
      if (t < kb) x[t] = V(k0 + t);
    for (int i = c.w; i < k0; i += c.W) {
      cplx v = V(i);
#pragma unroll
      for (int t = 0; t < KBS; ++t)
        if (t < kb) v = cfms(v, E(k0 + t, i), x[t]);
      V(i) = v;
    }
    __syncthreads();
  }
#undef E
#undef V
}

// ------------------------------------------------------------------ Dirichlet decoupling (symmetric mode)
// A Dirichlet row d holds only A_dd; its column entries A_id (i not Dirichlet) are left out
// of the factorisation, which then sees the decoupled matrix diag(A_DD) + A_rr (A_rr complex
// symmetric).  Exactly equivalent rewrites of the original systems:
//   forward  A x = b:       b_i -= sum_d A_id b_d / A_dd        (before the solve)
//   adjoint  A^T l = g:     l_d -= sum_i A_id l_i / A_dd        (after the solve)
// A = K - omega^2 M (operator form).  One wave per coupled row / Dirichlet node (64 frequencies).
struct DirArgs {
  const int2* dir;        // per Dirichlet node: (permuted node, diagonal entry)
  const int* crow;        // coupled rows (permuted)
  const int* cptr;        // entry range of each coupled row in ce
  const int2* ce;         // (Dirichlet slot, entry)
  const int* dptr;        // entry range of each Dirichlet node in de
  const int2* de;         // (permuted row, entry)
  const cplx* K;
  const double* M;
  const double* freqs;
};

__device__ __forceinline__ cplx op_entry(const DirArgs& D, int nz, double om2) {
  const cplx k = D.K[nz];
  return make_double2(fma(-om2, D.M[nz], k.x), k.y);
}

__device__ __forceinline__ cplx cdiv(cplx a, cplx b) { return cmul(a, crecip(b)); }

// SRC 0: b from the operator right-hand side (RHS 0), corrections into Bc (slot-major);
// SRC 2: b = G (permuted, frequency-minor), corrected in place
template <int SRC>
__global__ __launch_bounds__(64) void k_dirichlet_rhs(DirArgs D, RhsArgs R, cplx* __restrict__ G,
                                                      cplx* __restrict__ Bc, int64_t Fc) {
  const int slot = blockIdx.x;
  const int64_t q = (int64_t)blockIdx.y * 64 + threadIdx.x;
  const double om = 6.283185307179586 * D.freqs[q];
  const double om2 = om * om;
  cplx v = make_double2(0.0, 0.0);
  const int e1 = D.cptr[slot + 1];
  for (int e = D.cptr[slot]; e < e1; ++e) {
    const int2 c = D.ce[e];
    const int2 d = D.dir[c.x];
    cplx bd;
    if (SRC == 0) {
      const double r = R.rhsP[d.x];
      bd = make_double2(r * fma(-om2, R.mass_sum, R.beta_re), r * R.beta_im);
    } else {
      bd = G[(int64_t)d.x * Fc + q];
    }
    v = cfms(v, op_entry(D, c.y, om2), cdiv(bd, op_entry(D, d.y, om2)));
  }
  if (SRC == 0) {
    Bc[(int64_t)slot * Fc + q] = v;
  } else {
    cplx* g = G + (int64_t)D.crow[slot] * Fc + q;
    *g = cadd(*g, v);
  }
}

__global__ __launch_bounds__(64) void k_dirichlet_post(DirArgs D, cplx* __restrict__ X, int64_t Fc,
                                                        const int* __restrict__ glist) {
  const int gy = glist ? glist[blockIdx.y] : (int)blockIdx.y;
  if (gy < 0) return;
  const int slot = blockIdx.x;
  const int64_t q = (int64_t)gy * 64 + threadIdx.x;
  const double om = 6.283185307179586 * D.freqs[q];
  const double om2 = om * om;
  const int2 d = D.dir[slot];
  cplx s = make_double2(0.0, 0.0);
  const int e1 = D.dptr[slot + 1];
  for (int e = D.dptr[slot]; e < e1; ++e) {
    const int2 c = D.de[e];
    s = cfms(s, op_entry(D, c.y, om2), X[(int64_t)c.x * Fc + q]);   // -sum A_id l_i
  }
  cplx* x = X + (int64_t)d.x * Fc + q;
  *x = cadd(*x, cdiv(s, op_entry(D, d.y, om2)));
}

// ------------------------------------------------------------------ Hessian: tangent operators
// Y[p] = rhsP[p] * beta - sum_e Kd[nz_e] X[idx_e]        (accumulate = 0; forward tangent
//        right-hand side  db - dA x, rows of the permuted matrix)
// Y[p] = Y[p]           - sum_e Kd[nz_e] X[idx_e]        (accumulate = 1; with the column
//        structure: dG - dA^T lambda)
// One wavefront per row (64 frequencies); the row's index pairs are wave-uniform.
__global__ __launch_bounds__(256) void k_tangent_spmv(const int* __restrict__ ptr, const int* __restrict__ idx,
                                                       const int* __restrict__ nzs, int nrows,
                                                       const cplx* __restrict__ Kd, const cplx* __restrict__ X,
                                                       int64_t Fc, const double* __restrict__ rhsP, cplx beta,
                                                       cplx* __restrict__ Y, int accumulate) {
  const int p = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  if (p >= nrows) return;
  const int64_t q = (int64_t)blockIdx.y * 64 + (threadIdx.x & 63);
  cplx acc;
  if (accumulate) {
    acc = Y[(int64_t)p * Fc + q];
  } else {
    const double r = rhsP ? rhsP[p] : 0.0;
    acc = make_double2(r * beta.x, r * beta.y);
  }
  const int e1 = ptr[p + 1];
  int e = ptr[p];
  for (; e + 4 <= e1; e += 4) {
    cplx k[4], x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      k[u] = Kd[nzs[e + u]];
      x[u] = X[(int64_t)idx[e + u] * Fc + q];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc = cfms(acc, k[u], x[u]);
  }
  for (; e < e1; ++e) acc = cfms(acc, Kd[nzs[e]], X[(int64_t)idx[e] * Fc + q]);
  Y[(int64_t)p * Fc + q] = acc;
}

// ------------------------------------------------------------------ backward error (per frequency)
// Componentwise (Oettli-Prager) backward error of a computed solution,
//   berr = max_p |b - A x|_p / (|A| |x| + |b|)_p      (|z| = |re z| + |im z|, LAPACK's CABS1),
// per frequency -- the sparse backward error UMFPACK's refinement monitors (its omega1; the
// reference's solves run it by default, Control = NULL at InnerState.h:246-247), invariant under
// row and column scaling, so it stays meaningful for these badly scaled systems (membrane, bending
// and unit Dirichlet rows; a normwise measure is dominated by the membrane rows).  A is the
// ORIGINAL system on the permuted pattern: its rows (forward, A x = b) or its columns (adjoint,
// A^T l = g), A = K - omega^2 M (MODE 0) or the explicit batch (MODE 1).  A wave takes rows
// p = wave id, wave id + waves, ... for 64 frequencies and keeps a per-lane maximum, merged once
// per wave into acc[q] by atomicMax on its bit pattern (non-negative doubles order like their
// 64-bit patterns).  RHS: 0 = operator rhs (rhsP (beta - omega^2 mass_sum)), 1 = explicit batch B
// (caller numbering, through perm), 2 = vector G (permuted).  R (may be NULL) receives r.
struct ResidArgs {
  const int* ptr;
  const int* idx;
  const int* nzs;
  int n;
  const cplx* K;
  const double* M;
  const double* freqs;
  const cplx* data;
  int64_t data_stride;
  int nvalid;
  const double* rhsP;
  double beta_re, beta_im, mass_sum;
  const cplx* B;
  int64_t b_stride;
  const int* perm;
  const cplx* G;
  const int* walk;   // rows in walk order (original numbering: mesh-local gathers of X)
  const double* se;  // NSK > 0: stiffness values, nz-major (se[nz * NSK + k])
  cplx* kpart;       // NSK > 0: per (workgroup, k, frequency) sums of S_k(nz) mu_row x_col
  const int* glist;  // the groups to walk, indexed by grid row (-1: none; NULL: grid row = group)
};

__device__ __forceinline__ double cabs1(cplx z) { return fabs(z.x) + fabs(z.y); }

// Compensated residual (the functional correction's walk): r = b - sum A x accumulated as an unevaluated sum
// rh + rl (Ogita-Rump-Oishi Dot2: every product split exactly by an fma, every addition by TwoSum), i.e. as if
// in twice the working precision and rounded once.  Next to a resonance the static-pivot solves are backward
// stable to ~1e-15, so b - A x is as small as the rounding of the plain fp64 accumulation itself and the
// correction mu^T r read mostly that rounding; with the compensated sum it reads the solve's error, and the
// corrected fr no longer depends on the rounding order of the factorisation.  Contraction off: an fma fused
// into TwoSum would break its exactness.
__device__ __forceinline__ void dd_sub_prod(double& h, double& l, double a, double b) {
#pragma clang fp contract(off)
  const double p = a * b;
  const double pe = fma(a, b, -p);        // a b - p exactly
  const double s = h - p;
  const double bb = s - h;
  const double se = (h - (s - bb)) + (-p - bb);
  h = s;
  l -= pe;
  l += se;
}
__device__ __forceinline__ void cfms_dd(cplx& rh, cplx& rl, cplx a, cplx x) {
  dd_sub_prod(rh.x, rl.x, a.x, x.x);
  dd_sub_prod(rh.x, rl.x, -a.y, x.y);
  dd_sub_prod(rh.y, rl.y, a.x, x.y);
  dd_sub_prod(rh.y, rl.y, a.y, x.x);
}

template <int MODE>
__device__ __forceinline__ cplx resid_entry(const ResidArgs& A, const cplx* __restrict__ dq, int nz, double om2) {
  if (MODE == 0) {
    const cplx k = A.K[nz];
    return make_double2(fma(-om2, A.M[nz], k.x), k.y);
  }
  return dq[nz];
}

constexpr int RES_WPE = 4;   // the fused walk at 114 VGPRs with the compensated residual (round 3: 5 waves/SIMD, 96 VGPRs, 9.5 -> 8.0 ms)
// NSK > 0 (with DOT, the loss sweep's forward walk under the functional correction): the gradient
// contraction rides on the walk -- every entry (p, j, nz) it visits has x_j gathered and mu_p loaded
// already, so s_k(q) += S_k(nz) mu_p x_j per lane (frequency), per workgroup; the loss cotangent scale
// m_q is only known after this walk (k_correct_finish), so the partials stay per frequency and
// k_reduce_q applies m_q.  Replaces k_contract_eg's separate entry walk.
// CMP: the residual accumulated compensated (Dot2) -- the correction walk (DOT) and the refinement's residual (R):
// both read the solve's own error, which a plain fp64 sum of the row's terms rounds away
// RU: entries per batch of the row loop (all their gathers issued before the batch's products; the products in entry
// order whatever RU, so every RU gives the same bits)
template <int MODE, int RHS, bool DOT = false, int NSK = 0, bool CMP = DOT, int RU = 4>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NSK > 0 ? RES_WPE : 1))) void k_residual(ResidArgs A, const cplx* __restrict__ X, int64_t Fc,
                                                  cplx* __restrict__ R, double* __restrict__ acc,
                                                  const cplx* __restrict__ Mu, cplx* __restrict__ cpart) {
  // XCD-aware order: the workgroups of one 64-frequency group run together on one XCD, so the
  // solution rows their window of rows gathers (~2 MB) stay in that XCD's L2 instead of every
  // XCD's L2 holding windows of eight groups
  const int64_t lid = xcd_swizzle(blockIdx.x + (int64_t)gridDim.x * blockIdx.y, (int64_t)gridDim.x * gridDim.y);
  const int bx = (int)(lid % gridDim.x), by = A.glist ? A.glist[lid / gridDim.x] : (int)(lid / gridDim.x);
  if (by < 0) return;                       // no listed group (the selective adjoint refinement)
  const int64_t q = (int64_t)by * 64 + (threadIdx.x & 63);
  const int wave0 = __builtin_amdgcn_readfirstlane(bx * (blockDim.x >> 6) + (threadIdx.x >> 6));
  const int nwaves = gridDim.x * (blockDim.x >> 6);
  double om2 = 0.0;
  if (MODE == 0 || RHS == 0) {
    const double om = 6.283185307179586 * A.freqs[q];
    om2 = om * om;
  }
  const int64_t item = min(q, (int64_t)A.nvalid - 1);
  const cplx* __restrict__ dq = A.data + item * A.data_stride;
  double berr = 0.0;
  bool bad = false;         // NaN / Inf residual or a non-zero residual over a zero denominator
  cplx dot = make_double2(0, 0);   // sum_p Mu_p r_p (functional correction, Mu != NULL)
  cplx ks[NSK > 0 ? NSK : 1];
#pragma unroll
  for (int k = 0; k < (NSK > 0 ? NSK : 1); ++k) ks[k] = make_double2(0, 0);
  for (int t = wave0; t < A.n; t += nwaves) {
    const int p = A.walk[t];
    cplx mup = make_double2(0, 0);
    if (NSK > 0) mup = Mu[(int64_t)p * Fc + q];
    cplx b;
    if (RHS == 0) {
      const double v = A.rhsP[p];
      b = make_double2(v * fma(-om2, A.mass_sum, A.beta_re), v * A.beta_im);
    } else if (RHS == 1) {
      b = A.B[item * A.b_stride + A.perm[p]];
    } else {
      b = A.G[(int64_t)p * Fc + q];
    }
    cplx r = b, rl = make_double2(0.0, 0.0);    // CMP: r + rl compensated
    double den = cabs1(b);
    const int e1 = A.ptr[p + 1];
    int e = A.ptr[p];
    for (; e + RU <= e1; e += RU) {
      cplx a[RU], x[RU];
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        a[u] = resid_entry<MODE>(A, dq, A.nzs[e + u], om2);
        x[u] = X[(int64_t)A.idx[e + u] * Fc + q];
      }
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        if (CMP)
          cfms_dd(r, rl, a[u], x[u]);
        else
          r = cfms(r, a[u], x[u]);
        den = fma(cabs1(a[u]), cabs1(x[u]), den);
      }
      if (NSK > 0) {
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          const cplx mx = cmul(mup, x[u]);
          const double* sk = A.se + (int64_t)A.nzs[e + u] * NSK;
#pragma unroll
          for (int k = 0; k < NSK; ++k) {
            ks[k].x = fma(sk[k], mx.x, ks[k].x);
            ks[k].y = fma(sk[k], mx.y, ks[k].y);
          }
        }
      }
    }
    for (; e < e1; ++e) {
      const cplx a = resid_entry<MODE>(A, dq, A.nzs[e], om2);
      const cplx x = X[(int64_t)A.idx[e] * Fc + q];
      if (CMP)
        cfms_dd(r, rl, a, x);
      else
        r = cfms(r, a, x);
      den = fma(cabs1(a), cabs1(x), den);
      if (NSK > 0) {
        const cplx mx = cmul(mup, x);
        const double* sk = A.se + (int64_t)A.nzs[e] * NSK;
#pragma unroll
        for (int k = 0; k < NSK; ++k) {
          ks[k].x = fma(sk[k], mx.x, ks[k].x);
          ks[k].y = fma(sk[k], mx.y, ks[k].y);
        }
      }
    }
    if (CMP) r = cadd(r, rl);
    if (R) R[(int64_t)p * Fc + q] = r;
    if (DOT) {
      const cplx m = NSK > 0 ? mup : Mu[(int64_t)p * Fc + q];
      dot = cadd(dot, cmul(m, r));
    }
    const double cr = cabs1(r);
    bad = bad || !isfinite(cr) || !isfinite(den) || (den == 0.0 && cr > 0.0);
    if (den > 0.0) berr = fmax(berr, cr / den);
  }
  if (DOT) {
    // deterministic per-workgroup partial of the correction dot product: the waves' sums in LDS,
    // added in wave order, one partial per (workgroup, frequency) (k_correct_finish sums them in order)
    __shared__ cplx sdot[4][64];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    sdot[w][lane] = dot;
    __syncthreads();
    if (w == 0) {
      cplx t = sdot[0][lane];
      for (int k = 1; k < (int)(blockDim.x >> 6); ++k) t = cadd(t, sdot[k][lane]);
      cpart[(int64_t)bx * Fc + q] = t;
    }
  }
  if (NSK > 0) {
    // the waves' contraction sums in LDS, added in wave order: one partial per (workgroup, k, frequency)
    __shared__ cplx sks[4][64];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < NSK; ++k) {
      __syncthreads();
      sks[w][lane] = ks[k];
      __syncthreads();
      if (w == 0)
        A.kpart[((int64_t)bx * NSK + k) * Fc + q] =
            cadd(cadd(sks[0][lane], sks[1][lane]), cadd(sks[2][lane], sks[3][lane]));
    }
  }
  if (!acc) return;          // residual only (refinement step / correction without a check)
  if (bad) berr = __longlong_as_double(0x7ff0000000000000LL);     // +inf
  atomicMax(reinterpret_cast<unsigned long long*>(acc + q), (unsigned long long)__double_as_longlong(berr));
}

// Per-frequency loss term and its derivative d term / d fr (Problem.py:948-975); PFR_LOSS_COTANGENT:
// no term, derivative = ref.re (dL/dfr supplied by the caller).
__device__ __forceinline__ void loss_term(int loss_type, double fr, cplx r, double& term, double& dl) {
  const double rabs = sqrt(r.x * r.x + r.y * r.y);
  term = 0.0;
  dl = 0.0;
  switch (loss_type) {
    case PFR_LOSS_MSE: {
      const double dre = fr - r.x;
      term = dre * dre + r.y * r.y;
      dl = 2.0 * dre;
    } break;
    case PFR_LOSS_RMSE: {
      const double dre = fr - r.x, r2 = rabs * rabs;
      term = (dre * dre + r.y * r.y) / r2;
      dl = 2.0 * dre / r2;
    } break;
    case PFR_LOSS_MSE_AFC: {
      const double d = fr - rabs;
      term = d * d;
      dl = 2.0 * d;
    } break;
    case PFR_LOSS_MSE_LOG_AFC: {
      const double d = log(fr) - log(rabs);
      term = d * d;
      dl = 2.0 * d / fr;
    } break;
    case PFR_LOSS_COTANGENT:
      dl = r.x;
      break;
    default:
      break;
  }
}

// Functional correction (adjoint-weighted residual): with mu the adjoint of fr (A^T mu = d fr / d x,
// k_functional's seed mode) and r = b - A x the forward residual, fr(x*) = fr(x) + Re(mu^T r) up to
// second order in the solve's error -- the accuracy UMFPACK's default refinement (IRSTEP = 2) buys the
// reference's fr, for one dot product per row folded into the residual walk.  Per frequency: the
// corrected fr (fr_out, global index), the loss term of it and the cotangent scale
// m_q = scale * d term / d fr (lambda = m_q mu: the gradient contraction and k_rhs_dot take it).
// gind != NULL: also each 64-frequency group's largest first-order fr error estimate |Re(mu^T r)| / fr (the
// correction itself; large next to a resonance), from which k_select_groups picks the groups to refine.
//
// tq != NULL (the solve-error scale, on in loss sweeps): tq holds t_q = mu^T rhsP on entry and m_q t_q on exit,
// and m_q is complex, dl * scale * fr / (mu^T A x).  Next to a resonance the static-pivot solves' error is
// almost all along the resonant mode, i.e. along the solution itself: x = (1 + dx) x*, mu = (1 + dm) mu*
// with complex scalars dx, dm of up to ~cond * eps.  The gradient contraction mu^T S_k x then carries
// (1 + dx)(1 + dm), whose imaginary part the real gradient does not forgive (the partials cancel by 1e7-1e9
// over the sweep); fr = mu*^T A x* = mu*^T b, so mu^T A x = (1 + dx)(1 + dm) fr to first order, and
// mu^T A x = mu^T b - mu^T r is two dot products the sweep has already formed (k_rhs_dot, the correction's
// walk): dividing by it removes both factors with no further solve ("Gradient at full size")
__global__ __launch_bounds__(256) void k_correct_finish(FunctionalArgs A, const double* __restrict__ fr0,
                                                        const cplx* __restrict__ cpart, int nparts, int64_t Fc,
                                                        int nvalid, int64_t q_global0, double* __restrict__ fr_out,
                                                        double* __restrict__ loss_terms, cplx* __restrict__ mscale,
                                                        double* __restrict__ gind, cplx* __restrict__ tq, RhsScale bsc) {
  // 4 waves per 64 frequencies: wave w sums the partials b = w, w + 4, ... (8 loads in flight), then
  // wave 0 adds the four in order -- a fixed summation order (deterministic)
  __shared__ cplx sd[4][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 64 + lane;
  cplx d = make_double2(0, 0);
#pragma unroll 8
  for (int b = w; b < nparts; b += 4) d = cadd(d, cpart[(int64_t)b * Fc + q]);
  sd[w][lane] = d;
  __syncthreads();
  if (w != 0) return;
  d = cadd(cadd(sd[0][lane], sd[1][lane]), cadd(sd[2][lane], sd[3][lane]));
  const bool valid = q < nvalid;
  const double fr = fr0[q] + d.x;
  if (gind) {
    double v = valid ? fabs(d.x) / fabs(fr) : 0.0;
    if (!(v <= 1e300)) v = 1e300;                                  // NaN / Inf: refine first
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off));
    if (lane == 0) gind[blockIdx.x] = v;
  }
  if (valid && fr_out) fr_out[q_global0 + q] = fr;
  if (A.loss_type < 0) return;
  double term = 0.0, dl = 0.0;
  if (valid) loss_term(A.loss_type, fr, A.ref[q_global0 + q], term, dl);
  loss_terms[q] = term;
  cplx m = make_double2(valid ? dl * A.scale : 0.0, 0.0);
  if (tq) {
    const cplx t0 = tq[q];
    if (valid) {
      const double om = 6.283185307179586 * bsc.freqs[q];
      const cplx bs = make_double2(fma(-om * om, bsc.mass_sum, bsc.beta_re), bsc.beta_im);
      const cplx bt = cmul(bs, t0);
      const cplx den = make_double2(bt.x - d.x, bt.y - d.y);        // mu^T A x
      const double dd = den.x * den.x + den.y * den.y;
      if (dd > 0.0 && isfinite(dd)) {
        const double f = m.x * fr / dd;                             // m fr / den = m fr conj(den) / |den|^2
        m = make_double2(f * den.x, -f * den.y);
      }
    }
    tq[q] = cmul(m, t0);
  }
  mscale[q] = m;
}

// flag the frequencies whose backward error exceeds tol; optional per-frequency output (global
// index q0 + q, slot `which` of 2); the maxima are cleared for the next check.
__global__ void k_berr_finish(double* __restrict__ acc, int64_t Fc, int nvalid, double tol, int flag,
                              int* __restrict__ flags, double* __restrict__ berr_out, int64_t q0, int which) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Fc) return;
  const double berr = acc[q];
  if (q < nvalid && !(berr <= tol)) atomicOr(flags + q, flag);
  if (berr_out && q < nvalid) berr_out[2 * (q0 + q) + which] = berr;
  acc[q] = 0.0;
}

// X[p, q] *= m[q] over a permuted frequency-minor vector (lambda = m_q mu, functional correction)
__global__ void k_scale_vec(cplx* __restrict__ X, const cplx* __restrict__ m, int n, int64_t Fc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < (int64_t)n * Fc) X[i] = cmul(X[i], m[i % Fc]);
}

// X += D over a permuted frequency-minor vector (iterative refinement)
// glist != NULL: count = rows x REFINE_CAP x 64, element (row, list slot, lane) of the listed group
__global__ void k_axpy_vec(cplx* __restrict__ X, const cplx* __restrict__ D, int64_t count, const int* __restrict__ glist,
                           int64_t Fc) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  if (glist) {
    const int64_t row = i / (REFINE_CAP * 64), r = i % (REFINE_CAP * 64);
    const int g = glist[r >> 6];
    if (g < 0) return;
    i = row * Fc + (int64_t)g * 64 + (r & 63);
  }
  X[i] = cadd(X[i], D[i]);
}

// The (at most REFINE_CAP) groups with the largest indicators above tol, largest first; -1 past them.  One wave.
__global__ __launch_bounds__(64) void k_select_groups(const double* __restrict__ gind, int ngroups, double tol,
                                                      int* __restrict__ glist) {
  const int t = threadIdx.x;
  double v = t < ngroups ? gind[t] : -1.0;
  for (int k = 0; k < REFINE_CAP; ++k) {
    double m = v;
    int who = t;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double mo = __shfl_xor(m, off);
      const int wo = __shfl_xor(who, off);
      if (mo > m || (mo == m && wo < who)) {
        m = mo;
        who = wo;
      }
    }
    if (t == 0) glist[k] = m > tol ? who : -1;
    if (t == who) v = -1.0;
  }
}

// Directional derivative of the loss cotangent G (k_functional) along dx:
//   G = s h,  s = scale l'(fr) / fr,  h = ts^2 conj(U) aU + ts^2 conj(V) aV + conj(W) aW
//   dG = ds h + s dh,  ds = scale (l''(fr) / fr - l'(fr) / fr^2) dfr,
//   dfr = Re(ts^2 conj(U) dU + ts^2 conj(V) dV + conj(W) dW) / fr
// (second derivatives of the losses of Problem.py:948-975).  Writes the support entries of G.
__global__ void k_functional_tangent(FunctionalArgs A, const cplx* __restrict__ X, const cplx* __restrict__ DX,
                                     int64_t Fc, int nvalid, int64_t q_global0, cplx* __restrict__ G) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Fc) return;
  cplx U = make_double2(0, 0), V = U, W = U, dU = U, dV = U, dW = U;
  for (int s = 0; s < A.n_support; ++s) {
    const int64_t o = (int64_t)A.pidx[s] * Fc + q;
    const cplx x = X[o], d = DX[o];
    const double au = A.a[s], av = A.a[A.n_support + s], aw = A.a[2 * A.n_support + s];
    U.x = fma(au, x.x, U.x); U.y = fma(au, x.y, U.y);
    V.x = fma(av, x.x, V.x); V.y = fma(av, x.y, V.y);
    W.x = fma(aw, x.x, W.x); W.y = fma(aw, x.y, W.y);
    dU.x = fma(au, d.x, dU.x); dU.y = fma(au, d.y, dU.y);
    dV.x = fma(av, d.x, dV.x); dV.y = fma(av, d.y, dV.y);
    dW.x = fma(aw, d.x, dW.x); dW.y = fma(aw, d.y, dW.y);
  }
  const double ts2 = A.ts * A.ts;
  const double fr = sqrt(ts2 * (U.x * U.x + U.y * U.y) + ts2 * (V.x * V.x + V.y * V.y) + W.x * W.x + W.y * W.y);
  double s = 0.0, ds = 0.0;
  if (q < nvalid && fr > 0.0) {
    const double dfr =
        (ts2 * (U.x * dU.x + U.y * dU.y) + ts2 * (V.x * dV.x + V.y * dV.y) + W.x * dW.x + W.y * dW.y) / fr;
    const cplx r = A.ref[q_global0 + q];
    const double rabs = sqrt(r.x * r.x + r.y * r.y);
    double d1 = 0.0, d2 = 0.0;   // l'(fr), l''(fr)
    switch (A.loss_type) {
      case PFR_LOSS_MSE: d1 = 2.0 * (fr - r.x); d2 = 2.0; break;
      case PFR_LOSS_RMSE: d1 = 2.0 * (fr - r.x) / (rabs * rabs); d2 = 2.0 / (rabs * rabs); break;
      case PFR_LOSS_MSE_AFC: d1 = 2.0 * (fr - rabs); d2 = 2.0; break;
      case PFR_LOSS_MSE_LOG_AFC: {
        const double d = log(fr) - log(rabs);
        d1 = 2.0 * d / fr;
        d2 = 2.0 * (1.0 - d) / (fr * fr);
      } break;
      default: break;
    }
    s = A.scale * d1 / fr;
    ds = A.scale * (d2 / fr - d1 / (fr * fr)) * dfr;
  }
  // dG = ds h + s dh, h and dh share the support
  const cplx hU = make_double2(ts2 * U.x, -ts2 * U.y), hV = make_double2(ts2 * V.x, -ts2 * V.y),
             hW = make_double2(W.x, -W.y);
  const cplx kU = make_double2(ts2 * dU.x, -ts2 * dU.y), kV = make_double2(ts2 * dV.x, -ts2 * dV.y),
             kW = make_double2(dW.x, -dW.y);
  const cplx cU = make_double2(ds * hU.x + s * kU.x, ds * hU.y + s * kU.y);
  const cplx cV = make_double2(ds * hV.x + s * kV.x, ds * hV.y + s * kV.y);
  const cplx cW = make_double2(ds * hW.x + s * kW.x, ds * hW.y + s * kW.y);
  for (int t = 0; t < A.n_support; ++t) {
    const double au = A.a[t], av = A.a[A.n_support + t], aw = A.a[2 * A.n_support + t];
    G[(int64_t)A.pidx[t] * Fc + q] =
        make_double2(au * cU.x + av * cV.x + aw * cW.x, au * cU.y + av * cV.y + aw * cW.y);
  }
}

// ------------------------------------------------------------------ K4: functional + loss cotangent
// U = aU.x, V = aV.x, W = aW.x; fr = sqrt(ts^2|U|^2 + ts^2|V|^2 + |W|^2)  (Problem.py:454-477)
// loss terms of Problem.py:948-975; g = dl/fr * (ts^2 conj(U) aU + ts^2 conj(V) aV + conj(W) aW)
__global__ void k_functional(FunctionalArgs A, const cplx* __restrict__ X, int64_t Fc, int nvalid, int64_t q_global0,
                             double* __restrict__ fr_out, double* __restrict__ loss_terms, cplx* __restrict__ G) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Fc) return;
  cplx U = make_double2(0, 0), Vv = make_double2(0, 0), W = make_double2(0, 0);
#pragma unroll 8
  for (int s = 0; s < A.n_support; ++s) {
    const cplx x = X[(int64_t)A.pidx[s] * Fc + q];
    const double au = A.a[s], av = A.a[A.n_support + s], aw = A.a[2 * A.n_support + s];
    U.x = fma(au, x.x, U.x); U.y = fma(au, x.y, U.y);
    Vv.x = fma(av, x.x, Vv.x); Vv.y = fma(av, x.y, Vv.y);
    W.x = fma(aw, x.x, W.x); W.y = fma(aw, x.y, W.y);
  }
  const double ts2 = A.ts * A.ts;
  const double u2 = U.x * U.x + U.y * U.y, v2 = Vv.x * Vv.x + Vv.y * Vv.y, w2 = W.x * W.x + W.y * W.y;
  const double fr = sqrt(ts2 * u2 + ts2 * v2 + w2);
  const bool valid = q < nvalid;
  double s = 0.0;
  if (A.fr0) {
    // seed mode (functional correction): fr of this solve kept for k_correct_finish, G = d fr / d x
    A.fr0[q] = valid ? fr : 0.0;
    s = valid && fr > 0.0 ? 1.0 / fr : 0.0;
  } else {
    if (valid && fr_out) fr_out[q_global0 + q] = fr;
    if (A.loss_type < 0) return;
    double term = 0.0, dl = 0.0;
    if (valid) loss_term(A.loss_type, fr, A.ref[q_global0 + q], term, dl);
    loss_terms[q] = term;
    s = valid && fr > 0.0 ? dl * A.scale / fr : 0.0;
  }
  if (!G) return;             // fr0 only (the functional-from-bottom-up path: fr of the final x)
  const cplx cU = make_double2(s * ts2 * U.x, -s * ts2 * U.y);
  const cplx cV = make_double2(s * ts2 * Vv.x, -s * ts2 * Vv.y);
  const cplx cW = make_double2(s * W.x, -s * W.y);
  for (int t = 0; t < A.n_support; ++t) {
    const double au = A.a[t], av = A.a[A.n_support + t], aw = A.a[2 * A.n_support + t];
    cplx g;
    g.x = au * cU.x + av * cV.x + aw * cW.x;
    g.y = au * cU.y + av * cV.y + aw * cW.y;
    G[(int64_t)A.pidx[t] * Fc + q] = g;
  }
}

// ------------------------------------------------------------------ K4': functional from the bottom-up passes
// F_k = a_k^T x = sum_i (L^-1 a_k)_i (L^-1 b)_i / U(i, i) over the pivot rows i reached by both the rhs
// and the support (rows: (permuted row, factor element of U(i, i))).  Per frequency group FN_PARTS
// workgroups, each one partial per frequency (deterministic; k_functional_fn sums them in order).
constexpr int FN_PARTS = FN_PARTS_HOST;
__global__ __launch_bounds__(256) void k_fn_dot(const int2* __restrict__ rows, int nrows, const cplx* __restrict__ F,
                                                const cplx* __restrict__ Yb, const cplx* __restrict__ Y0,
                                                const cplx* __restrict__ Y1, const cplx* __restrict__ Y2, int64_t Fc,
                                                cplx* __restrict__ parts) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t q = (int64_t)blockIdx.y * 64 + lane;
  const int part = blockIdx.x;
  cplx s0 = make_double2(0, 0), s1 = s0, s2 = s0;
  for (int t = part * 4 + w; t < nrows; t += FN_PARTS * 4) {
    const int2 r = rows[t];
    const int64_t o = (int64_t)r.x * Fc + q;
    const cplx yb = cmul(Yb[o], crecip(F[(int64_t)r.y * Fc + q]));
    s0 = cadd(s0, cmul(Y0[o], yb));
    s1 = cadd(s1, cmul(Y1[o], yb));
    s2 = cadd(s2, cmul(Y2[o], yb));
  }
  __shared__ cplx sh[3][4][64];
  sh[0][w][lane] = s0;
  sh[1][w][lane] = s1;
  sh[2][w][lane] = s2;
  __syncthreads();
  if (w < 3) {
    const cplx v = cadd(cadd(sh[w][0][lane], sh[w][1][lane]), cadd(sh[w][2][lane], sh[w][3][lane]));
    parts[((int64_t)part * 3 + w) * Fc + q] = v;
  }
}

// k_functional with U, V, W from k_fn_dot's partials; also the cotangent coefficients (c_U, c_V, c_W)
// per frequency (fcoef, 3 x Fc) for k_fn_combine.  G (zeroed) gets the adjoint rhs at the support rows.
__global__ void k_functional_fn(FunctionalArgs A, const cplx* __restrict__ parts, int64_t Fc, int nvalid,
                                int64_t q_global0, double* __restrict__ fr_out, double* __restrict__ loss_terms,
                                cplx* __restrict__ G, cplx* __restrict__ fcoef) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Fc) return;
  cplx U = make_double2(0, 0), Vv = U, W = U;
  for (int p = 0; p < FN_PARTS; ++p) {
    U = cadd(U, parts[((int64_t)p * 3 + 0) * Fc + q]);
    Vv = cadd(Vv, parts[((int64_t)p * 3 + 1) * Fc + q]);
    W = cadd(W, parts[((int64_t)p * 3 + 2) * Fc + q]);
  }
  const double ts2 = A.ts * A.ts;
  const double fr = sqrt(ts2 * (U.x * U.x + U.y * U.y) + ts2 * (Vv.x * Vv.x + Vv.y * Vv.y) + W.x * W.x + W.y * W.y);
  const bool valid = q < nvalid;
  double s = 0.0;
  if (A.fr0) {
    A.fr0[q] = valid ? fr : 0.0;
    s = valid && fr > 0.0 ? 1.0 / fr : 0.0;
  } else {
    if (valid && fr_out) fr_out[q_global0 + q] = fr;
    if (A.loss_type >= 0) {
      double term = 0.0, dl = 0.0;
      if (valid) loss_term(A.loss_type, fr, A.ref[q_global0 + q], term, dl);
      loss_terms[q] = term;
      s = valid && fr > 0.0 ? dl * A.scale / fr : 0.0;
    }
  }
  const cplx cU = make_double2(s * ts2 * U.x, -s * ts2 * U.y);
  const cplx cV = make_double2(s * ts2 * Vv.x, -s * ts2 * Vv.y);
  const cplx cW = make_double2(s * W.x, -s * W.y);
  fcoef[q] = cU;
  fcoef[Fc + q] = cV;
  fcoef[2 * Fc + q] = cW;
  for (int t = 0; t < A.n_support; ++t) {
    const double au = A.a[t], av = A.a[A.n_support + t], aw = A.a[2 * A.n_support + t];
    G[(int64_t)A.pidx[t] * Fc + q] =
        make_double2(au * cU.x + av * cV.x + aw * cW.x, au * cU.y + av * cV.y + aw * cW.y);
  }
}

// The adjoint's bottom-up result over the support's fronts: L^-1 g = sum_k c_k (L^-1 a_k), in place in Y0
// (rows: the pivot rows of the support-reach fronts, permuted)
__global__ __launch_bounds__(256) void k_fn_combine(const int* __restrict__ rows, int nrows, const cplx* __restrict__ fcoef,
                                                    cplx* __restrict__ Y0, const cplx* __restrict__ Y1,
                                                    const cplx* __restrict__ Y2, int64_t Fc) {
  const int lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.y * 64 + lane;
  const cplx c0 = fcoef[q], c1 = fcoef[Fc + q], c2 = fcoef[2 * Fc + q];
  for (int t = blockIdx.x * 4 + (threadIdx.x >> 6); t < nrows; t += gridDim.x * 4) {
    const int64_t o = (int64_t)rows[t] * Fc + q;
    Y0[o] = cadd(cadd(cmul(c0, Y0[o]), cmul(c1, Y1[o])), cmul(c2, Y2[o]));
  }
}

// ------------------------------------------------------------------ K5: gradient contraction + checks
// s_{q,k} = sum_nz stiff[nz][k] * Lam[prow] * X[pcol]   (Sparse.py:173-176 matrix cotangent,
// contracted with the stiffness matrices as JAX's einsum transpose does), fused with the checks.
// Entries of the union pattern, rows ascending: each permuted row i starts with a pseudo-entry (-1, -1, -1, i),
// followed by (column j, nz of A(i, j) or -1, nz of A(j, i) or -1, i) over the union of row i's and column i's
// patterns.  se[NS e + k] = S_k(i, j) (zeros where the entry is absent), copied once per stiffness upload.
__global__ void k_gather_entries(const int4* __restrict__ ent, int nent, const double* __restrict__ stiff, int ns,
                                 double* __restrict__ se) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nent) return;
  const int4 en = ent[e];
  const bool ij = en.x >= 0 && en.y >= 0;
  for (int k = 0; k < ns; ++k) se[(int64_t)e * ns + k] = ij ? stiff[(int64_t)en.y * ns + k] : 0.0;
}

// Gradient contraction, entry-major: w_k = sum_e S_k(e) P_e with P_e = sum_q lambda_i(q) x_j(q) -- the
// frequency sum is taken first.  A wave owns EW consecutive entries and walks every 64-frequency group
// of the chunk, accumulating P_e per lane (contiguous 1 KiB runs of x_j and lambda_i per group); then one
// cross-lane sum per entry and S_k(e) P_e with the S row read once per entry (not once per entry and
// frequency group: with the sum over frequencies inside, the 12-18 scalar stiffness loads per entry and
// the per-lane accumulators of all stiffness matrices drop out of the frequency loop).
// Pseudo entries (row starts) and absent entries carry S = 0.  One partial per wave (k_reduce).
// MS: lambda = m_q Lam per frequency (functional correction: Lam is the adjoint of fr, m_q the loss
// cotangent scale k_correct_finish formed); m_q = 0 on the padded frequencies.
template <int NS, int EW, bool MS>
__global__ __launch_bounds__(256) void k_contract_eg(const int4* __restrict__ ent, int nent,
                                                     const double* __restrict__ se, const cplx* __restrict__ Lam,
                                                     const cplx* __restrict__ X, int64_t Fc, int nvalid,
                                                     const cplx* __restrict__ msc, cplx* __restrict__ partial) {
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  const int e0 = min(wv * EW, nent - 1);     // waves past the end: clamped entries, masked below
  int64_t oi[EW], oj[EW];
#pragma unroll
  for (int u = 0; u < EW; ++u) {
    const int4 en = ent[min(e0 + u, nent - 1)];
    oi[u] = (int64_t)max(en.w, 0) * Fc + lane;
    oj[u] = (int64_t)max(en.x, 0) * Fc + lane;
  }
  cplx P[EW];
#pragma unroll
  for (int u = 0; u < EW; ++u) P[u] = make_double2(0, 0);
  for (int64_t g = 0; g < Fc; g += 64) {
    cplx li[EW], xj[EW];
#pragma unroll
    for (int u = 0; u < EW; ++u) {
      li[u] = Lam[oi[u] + g];
      xj[u] = X[oj[u] + g];
    }
    const cplx m = MS ? msc[g + lane] : make_double2(g + lane < nvalid ? 1.0 : 0.0, 0.0);
#pragma unroll
    for (int u = 0; u < EW; ++u) P[u] = cadd(P[u], cmul(cmul(li[u], xj[u]), m));
  }
  cplx part[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) part[k] = make_double2(0, 0);
#pragma unroll
  for (int u = 0; u < EW; ++u) {
    double re = P[u].x, im = P[u].y;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      re += __shfl_xor(re, o);
      im += __shfl_xor(im, o);
    }
    const double in = wv * EW + u < nent ? 1.0 : 0.0;
    const double* sk = se + (int64_t)min(e0 + u, nent - 1) * NS;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      part[k].x = fma(sk[k] * in, re, part[k].x);
      part[k].y = fma(sk[k] * in, im, part[k].y);
    }
  }
  // the workgroup's 4 wave partials summed in wave order (one partial per workgroup: k_reduce's loop
  // is 4x shorter; deterministic)
  __shared__ cplx sp[4][NS];
  const int w = threadIdx.x >> 6;
  if (lane < NS) {
    cplx v = part[0];
#pragma unroll
    for (int k = 1; k < NS; ++k) v = lane == k ? part[k] : v;
    sp[w][lane] = v;
  }
  __syncthreads();
  if (w == 0 && lane < NS)
    partial[(int64_t)blockIdx.x * NS + lane] = cadd(cadd(sp[0][lane], sp[1][lane]), cadd(sp[2][lane], sp[3][lane]));
}

// t_q = sum_p Lam[p] * rhsP[p] over the Dirichlet support (d b / d beta)
__global__ void k_rhs_dot(const int* __restrict__ sup, const double* __restrict__ val, int n_sup,
                          const cplx* __restrict__ Lam, int64_t Fc, const cplx* __restrict__ msc,
                          cplx* __restrict__ t_out) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Fc) return;
  cplx t = make_double2(0, 0);
  for (int s = 0; s < n_sup; ++s) {
    const cplx l = Lam[(int64_t)sup[s] * Fc + q];
    t.x = fma(val[s], l.x, t.x);
    t.y = fma(val[s], l.y, t.y);
  }
  t_out[q] = msc ? cmul(t, msc[q]) : t;
}

// Deterministic reduction over (blocks, valid frequencies):
//   w[k] += sum_q ( -sum_blk partial[blk][k][q] + e_k * t_q ),  loss += sum_q loss_terms[q]
// partial[t * n_stiff + k] = sum_{q in tile t} m_q sum_b kpart[b][k][q] (fixed order; tile = 64 frequencies):
// the fused walk's contraction in k_contract_eg's partial layout (one part per tile), so that k_reduce
// completes it unchanged.  Block = (k, tile), 4 waves splitting the workgroup partials b.
__global__ __launch_bounds__(256) void k_reduce_q(const cplx* __restrict__ kpart, int nparts, int n_stiff,
                                                  const cplx* __restrict__ msc, int nvalid, int64_t Fc,
                                                  cplx* __restrict__ partial) {
  __shared__ double sre[4][64], sim[4][64];
  const int k = blockIdx.x, tile = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t q = (int64_t)tile * 64 + lane;
  double pr = 0, pi = 0;
#pragma unroll 8
  for (int b = w; b < nparts; b += 4) {
    const cplx v = kpart[((int64_t)b * n_stiff + k) * Fc + q];
    pr += v.x;
    pi += v.y;
  }
  sre[w][lane] = pr;
  sim[w][lane] = pi;
  __syncthreads();
  if (w == 0) {
    const cplx m = q < nvalid ? (msc ? msc[q] : make_double2(1.0, 0.0)) : make_double2(0.0, 0.0);
    const double sr = (sre[0][lane] + sre[1][lane]) + (sre[2][lane] + sre[3][lane]);
    const double si = (sim[0][lane] + sim[1][lane]) + (sim[2][lane] + sim[3][lane]);
    double re = m.x * sr - m.y * si;
    double im = m.x * si + m.y * sr;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      re += __shfl_xor(re, o);
      im += __shfl_xor(im, o);
    }
    if (lane == 0) partial[(int64_t)tile * n_stiff + k] = make_double2(re, im);
  }
}

__global__ void k_reduce(const cplx* __restrict__ partial, int nparts, int n_stiff, const cplx* __restrict__ t_q,
                         CoefPack e, const double* __restrict__ loss_terms, int nvalid, int64_t Fc,
                         cplx* __restrict__ w_out, double* __restrict__ loss_out) {
  __shared__ double sre[1024], sim[1024];
  const int k = blockIdx.x;   // 0..n_stiff-1: stiffness; n_stiff: loss
  double re = 0, im = 0;
  if (k < n_stiff) {
#pragma unroll 4
    for (int b = threadIdx.x; b < nparts; b += blockDim.x) {
      const cplx v = partial[(int64_t)b * n_stiff + k];
      re -= v.x;
      im -= v.y;
    }
    for (int q = threadIdx.x; q < nvalid; q += blockDim.x) {
      const cplx t = t_q[q];
      re += e.re[k] * t.x;
      im += e.re[k] * t.y;
    }
  } else {
    for (int q = threadIdx.x; q < nvalid; q += blockDim.x) re += loss_terms[q];
  }
  sre[threadIdx.x] = re;
  sim[threadIdx.x] = im;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      sre[threadIdx.x] += sre[threadIdx.x + s];
      sim[threadIdx.x] += sim[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (k < n_stiff) {
      w_out[k].x += sre[0];
      w_out[k].y += sim[0];
    } else if (loss_out) {
      loss_out[0] += sre[0];
    }
  }
}

// ------------------------------------------------------------------ misc
// x_out[q * n + perm[p]] = X[p * Fc + q]  (back to the caller's numbering, batch-major)
__global__ void k_unpermute(const int* __restrict__ perm, int n, const cplx* __restrict__ X, int64_t Fc, int nvalid,
                            cplx* __restrict__ out) {
  const int p = blockIdx.x;
  const int q = blockIdx.y * blockDim.x + threadIdx.x;
  if (q >= nvalid || p >= n) return;
  out[(int64_t)q * n + perm[p]] = X[(int64_t)p * Fc + q];
}

// y = A x (or A^T x) for a batch of matrices on the CSC pattern (InnerState::matvec,
// InnerState.h:310-470; csc_matvec.h:31-66).  One thread per (column, batch item).
__global__ void k_matvec(const int* __restrict__ colptr, const int* __restrict__ rowind, int n,
                         const cplx* __restrict__ data, int64_t data_stride, const cplx* __restrict__ x,
                         int64_t x_stride, cplx* __restrict__ y, int transpose, int batch) {
  const int q = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n || q >= batch) return;
  const cplx* d = data + q * data_stride;
  const cplx* xv = x + q * x_stride;
  cplx* yv = y + (int64_t)q * n;
  if (transpose) {
    cplx acc = make_double2(0, 0);
    for (int e = colptr[j]; e < colptr[j + 1]; ++e) acc = cadd(acc, cmul(d[e], xv[rowind[e]]));
    yv[j] = acc;
  } else {
    const cplx xj = xv[j];
    for (int e = colptr[j]; e < colptr[j + 1]; ++e) {
      const cplx v = cmul(d[e], xj);
      atomicAdd(&yv[rowind[e]].x, v.x);
      atomicAdd(&yv[rowind[e]].y, v.y);
    }
  }
}

// ================================================================== launchers
#define LAUNCH(kern, grid, block, st, ...) hipLaunchKernelGGL(kern, grid, block, 0, st, __VA_ARGS__)
#define LAUNCH_DYN(kern, grid, block, lds, st, ...) hipLaunchKernelGGL(kern, grid, block, lds, st, __VA_ARGS__)

// The first launch configuration the runtime refused since the last launch_refused() call (a kernel whose dynamic
// LDS could not be raised above the default): the launch is skipped and the C ABI call that issued it fails with
// this name (api.cpp LAUNCH_TRY), instead of a later generic launch error.
static std::atomic<const char*> g_refused{nullptr};
const char* launch_refused() { return g_refused.exchange(nullptr); }
static bool dyn_lds(const void* fn, int bytes, const char* name) {
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess) return true;
  const char* none = nullptr;
  g_refused.compare_exchange_strong(none, name);
  return false;
}

void launch_combine(const double* stiff, int n_stiff, int64_t nnz, const CoefPack& coef, double2* K, hipStream_t st) {
  LAUNCH(k_combine, dim3((unsigned)((nnz + 255) / 256)), dim3(256), st, stiff, n_stiff, nnz, coef, K);
}

void launch_schur(bool sym, const DevPattern& P, const int4* tiles, int ntiles, const int* g1, const int* gxp,
                  const int2* gx, int ngroups, double2* F, int64_t Fc, hipStream_t st) {
  if (ntiles <= 0) return;
  dim3 g((ntiles + 3) / 4, ngroups * (64 / SCHUR_QG)), b(256);
  if (sym) LAUNCH(k_schur_sym_level, g, b, st, P, tiles, ntiles, g1, gxp, gx, F, Fc);
  else LAUNCH(k_schur_level, g, b, st, P, tiles, ntiles, g1, gxp, gx, F, Fc);
}

// 4 LDS buffers of one pivot each, 16 x 16 blocks (measured best of 2-4 buffers, 1-2 pivots per stage, 16 x 8 blocks)
void launch_schur_blk(const DevPattern& P, const int4* blocks, int nblocks, const int* bg1, const int* bgxp,
                      const int2* bgx, int ngroups, double2* F, int64_t Fc, hipStream_t st) {
  if (nblocks <= 0) return;
  LAUNCH((k_schur_sym_blk<4, 1, 16>), dim3(nblocks, ngroups), dim3(64 * 16), st, P, blocks, nblocks, bg1, bgxp, bgx, F, Fc);
}

void launch_assemble(int mode, const int4* recs, int nrec, const int* xptr, const int2* xl, int ngroups, double2* F,
                     int64_t Fc, const double* freqs, const double2* K, const double* M, const double2* data,
                     int64_t ds, int nvalid, hipStream_t st) {
  if (nrec <= 0) return;
  dim3 g((nrec / 8 + 3) / 4, ngroups), b(256);
  if (mode == 0) LAUNCH(k_assemble_level<0>, g, b, st, recs, nrec, xptr, xl, F, Fc, freqs, K, M, data, ds, nvalid);
  else LAUNCH(k_assemble_level<1>, g, b, st, recs, nrec, xptr, xl, F, Fc, freqs, K, M, data, ds, nvalid);
}

void launch_factor_lds(const DevPattern& P, const int* lvl, int nfronts, int maxns, double2* F, int64_t Fc, int* flags,
                       hipStream_t st) {
  const size_t lds = (size_t)fac_lds_bytes(maxns);
  static_assert(FAC_LB == 8, "fac_lds_bytes: 8 W columns per row");
  // dynamic LDS beyond the default 64 KiB (up to 64 pivots: 37 KiB; headroom)
  static const bool attr = dyn_lds(reinterpret_cast<const void*>(&k_factor_sym_lds), 160 * 1024, "k_factor_sym_lds");
  if (!attr) {
    const char* none = nullptr;
    g_refused.compare_exchange_strong(none, "k_factor_sym_lds");
    return;
  }
  LAUNCH_DYN(k_factor_sym_lds, dim3((unsigned)(nfronts * Fc)), dim3(256), lds, st, P, lvl, F, Fc, flags, maxns);
}

void launch_factor(bool sym, const DevPattern& P, const int* lvl, int nfronts, int W, int ngroups, double2* F,
                   int64_t Fc, int* flags, hipStream_t st, int G) {
  if (sym && G == 8) LAUNCH(k_factor_sym<8>, dim3(nfronts, ngroups * 8), dim3(64 * W), st, P, lvl, F, Fc, flags);
  else if (sym && G == 4) LAUNCH(k_factor_sym<4>, dim3(nfronts, ngroups * 4), dim3(64 * W), st, P, lvl, F, Fc, flags);
  else if (sym) LAUNCH(k_factor_sym<FAC_G>, dim3(nfronts, ngroups * FAC_G), dim3(64 * W), st, P, lvl, F, Fc, flags);
  else LAUNCH(k_factor_level<true>, dim3(nfronts, ngroups * FAC_G), dim3(64 * W), st, P, lvl, F, Fc, flags);
}

void launch_front0(const DevPattern& P, const int* fl, int nfronts, int nsmall, const int* fptr, const int* fnz,
                   int ngroups, double2* F, int64_t Fc, const double* freqs, const double2* K, const double* M,
                   int* flags, hipStream_t st) {
  if (nsmall > 0)
    LAUNCH((k_front0<2>), dim3((nsmall + 3) / 4, ngroups), dim3(256), st, P, fl, nsmall, fptr, fnz, F, Fc, freqs, K,
           M, flags);
  if (nfronts > nsmall)
    LAUNCH((k_front0<F0_NS>), dim3((nfronts - nsmall + 3) / 4, ngroups), dim3(256), st, P, fl + nsmall,
           nfronts - nsmall, fptr + nsmall, fnz, F, Fc, freqs, K, M, flags);
}

void launch_offdiag(int mode, const DevPattern& P, const int4* items, int nitems, const int2* orec, const int* oxp,
                    const int2* ox, int ngroups, double2* F, int64_t Fc, const double* freqs, const double2* K,
                    const double* M, const double2* data, int64_t ds, int nvalid, int maxns, hipStream_t st, bool pipelined) {
  if (nitems <= 0) return;
  const bool small = maxns <= 8;
  dim3 g((nitems + 3) / 4, ngroups * OFF_G), b(256);
  static_assert(OB >= 8, "the SMALL variant covers pivot blocks of up to 8");
#define OL(MD, SM, PU) LAUNCH((k_offdiag_level<MD, SM, PU>), g, b, st, P, items, nitems, orec, oxp, ox, F, Fc, freqs, K, M, data, ds, nvalid)
  // pipelined: the prefix loop with the next pivot's loads issued before the current pivot's products (the
  // narrow levels, where few waves are resident)
  if (mode == 0 && small) OL(0, true, 2);
  else if (mode == 0 && pipelined) OL(0, false, 3);
  else if (mode == 0) OL(0, false, 2);
  else if (small) OL(1, true, 2);
  else OL(1, false, 2);
#undef OL
}

static RhsArgs make_rhs(const RhsDesc& d) {
  RhsArgs r;
  r.rhsP = d.rhsP; r.beta_re = d.beta_re; r.beta_im = d.beta_im; r.mass_sum = d.mass_sum;
  r.freqs = d.freqs; r.B = d.B; r.b_stride = d.b_stride; r.G = d.G; r.nvalid = d.nvalid;
  r.cslot = d.cslot; r.Bc = d.Bc;
  return r;
}

void launch_solve(int which, int rhs_mode, bool sym, const DevPattern& P, const int* lvl, int nfronts, int W, int ngroups,
                  const double2* F, int64_t Fc, double2* WV, const RhsDesc& rd, const double2* Yin, double2* Out,
                  const int* reach, hipStream_t st, int split, const int* glist) {
  if (nfronts <= 0) return;
  dim3 g(nfronts, ngroups), b(64 * W);
  const dim3 gs(nfronts * split, ngroups), bs(64 * SPLIT_W);
  const int rs = split > 1;
  RhsArgs R = make_rhs(rd);
  switch (which) {
    case 0:  // L solve (split > 1: the update rows by k_lsolve_rows over `split` workgroups per front)
      if (rhs_mode == 0) LAUNCH(k_lsolve_level<0>, g, b, st, P, lvl, F, Fc, WV, R, Out, reach, rs, glist);
      else if (rhs_mode == 1) LAUNCH(k_lsolve_level<1>, g, b, st, P, lvl, F, Fc, WV, R, Out, reach, rs, glist);
      else if (rhs_mode == 2) LAUNCH(k_lsolve_level<2>, g, b, st, P, lvl, F, Fc, WV, R, Out, reach, rs, glist);
      else LAUNCH(k_lsolve_level<3>, g, b, st, P, lvl, F, Fc, WV, R, Out, reach, rs, glist);
      if (rs) LAUNCH(k_lsolve_rows, gs, bs, st, P, lvl, F, Fc, WV, split, glist);
      break;
    case 1:  // U solve (split > 1: the pivot rows' update part first, by k_usolve_upd)
      if (rs && sym) LAUNCH(k_usolve_upd<true>, gs, bs, st, P, lvl, F, Fc, WV, Yin, Out, reach, split, glist);
      else if (rs) LAUNCH(k_usolve_upd<false>, gs, bs, st, P, lvl, F, Fc, WV, Yin, Out, reach, split, glist);
      if (sym) LAUNCH(k_usolve_level<true>, g, b, st, P, lvl, F, Fc, WV, Yin, Out, reach, rs, glist);
      else LAUNCH(k_usolve_level<false>, g, b, st, P, lvl, F, Fc, WV, Yin, Out, reach, rs, glist);
      break;
    case 2:  // U^T solve
      if (rhs_mode == 0) LAUNCH(k_utsolve_level<0>, g, b, st, P, lvl, F, Fc, WV, R, Out, reach);
      else if (rhs_mode == 1) LAUNCH(k_utsolve_level<1>, g, b, st, P, lvl, F, Fc, WV, R, Out, reach);
      else LAUNCH(k_utsolve_level<2>, g, b, st, P, lvl, F, Fc, WV, R, Out, reach);
      break;
    default:  // L^T solve
      LAUNCH(k_ltsolve_level, g, b, st, P, lvl, F, Fc, WV, Yin, Out, reach);
      break;
  }
}

void launch_lsolve_multi(int rhs_mode, const DevPattern& P, int nslices, const int* const* lvl, const int* nf, int W,
                         int ngroups, const double2* F, int64_t Fc, double2* const* WV, const RhsDesc* rd,
                         double2* const* Y, const int* const* reach, hipStream_t st, int split, bool nar,
                         int maxns, int maxf, bool rl) {
  LSlices S{};
  int nmax = 0;
  for (int z = 0; z < nslices; ++z) {
    S.lvl[z] = lvl[z];
    S.nf[z] = nf[z];
    S.WV[z] = WV[z];
    S.Y[z] = Y[z];
    S.reach[z] = reach[z];
    S.R[z] = make_rhs(rd[z]);
    nmax = std::max(nmax, nf[z]);
  }
  if (nmax <= 0) return;
  const dim3 g(nmax, ngroups, nslices), b(64 * W);
  const int rs = split > 1;
  if (rl && maxns > 16 * RL_WMAX) rl = false;   // k_lsolve_rl_z: at most 4 rows per lane slot
  if (rs && nar && rl) {
    const int rpl = rl_rpl(maxns);
    const dim3 gq(nmax, (unsigned)(Fc / RL_Q), nslices), bq(64 * rl_waves(maxns));
#define LRL(RH, RP) LAUNCH((k_lsolve_rl_z<RH, RP>), gq, bq, st, P, S, F, Fc)
    if (rhs_mode == 0) {
      if (rpl == 1) LRL(0, 1); else if (rpl == 2) LRL(0, 2); else LRL(0, 4);
    } else {
      if (rpl == 1) LRL(3, 1); else if (rpl == 2) LRL(3, 2); else LRL(3, 4);
    }
#undef LRL
  } else if (rs && nar) {
    static const bool attr =
        dyn_lds(reinterpret_cast<const void*>(&k_lsolve_level_z<0, true>), (int)LS_NAR_DYN_MAX, "k_lsolve_level_z<0,NAR>") &&
        dyn_lds(reinterpret_cast<const void*>(&k_lsolve_level_z<3, true>), (int)LS_NAR_DYN_MAX, "k_lsolve_level_z<3,NAR>");
    if (!attr) {
      const char* none = nullptr;
      g_refused.compare_exchange_strong(none, "k_lsolve_level_z<NAR>");
      return;
    }
    const size_t lds = (size_t)maxns * 64 * 16;
    if (rhs_mode == 0) LAUNCH_DYN((k_lsolve_level_z<0, true>), g, b, lds, st, P, S, F, Fc, rs);
    else LAUNCH_DYN((k_lsolve_level_z<3, true>), g, b, lds, st, P, S, F, Fc, rs);
  } else if (rhs_mode == 0) LAUNCH(k_lsolve_level_z<0>, g, b, st, P, S, F, Fc, rs);
  else LAUNCH(k_lsolve_level_z<3>, g, b, st, P, S, F, Fc, rs);
  if (rs && nar) {
    const int RB = (std::max(1, maxf - 1) + LRC_SR - 1) / LRC_SR;
    LAUNCH(k_lsolve_rows_zc, dim3(nmax * RB, ngroups, nslices), dim3(64 * LRC_W), st, P, S, F, Fc, RB);
  } else if (rs) {
    LAUNCH(k_lsolve_rows_z, dim3(nmax * split, ngroups, nslices), dim3(64 * SPLIT_W), st, P, S, F, Fc, split);
  }
}

void launch_fn_dot(const int2* rows, int nrows, const double2* F, const double2* Yb, const double2* const* Yk, int64_t Fc,
                   double2* parts, hipStream_t st) {
  LAUNCH(k_fn_dot, dim3(FN_PARTS, (unsigned)(Fc / 64)), dim3(256), st, rows, nrows, F, Yb, Yk[0], Yk[1], Yk[2], Fc, parts);
}

void launch_functional_fn(const FunctionalArgs& A, const double2* parts, int64_t Fc, int nvalid, int64_t q0,
                          double* fr_out, double* loss_terms, double2* G, double2* fcoef, hipStream_t st) {
  LAUNCH(k_functional_fn, dim3((unsigned)((Fc + 63) / 64)), dim3(64), st, A, parts, Fc, nvalid, q0, fr_out, loss_terms,
         G, fcoef);
}

void launch_fn_combine(const int* rows, int nrows, const double2* fcoef, double2* const* Yk, int64_t Fc, hipStream_t st) {
  if (nrows <= 0) return;
  const unsigned nb = (unsigned)std::min(64, (nrows + 3) / 4);
  LAUNCH(k_fn_combine, dim3(nb, (unsigned)(Fc / 64)), dim3(256), st, rows, nrows, fcoef, Yk[0], Yk[1], Yk[2], Fc);
}

void launch_usolve2(const DevPattern& P, const int* lvl, int nfronts, int W, bool small, int ngroups,
                    const double2* F, int64_t Fc, const double2* Y0, double2* X0, const int* reach0, const int* skip0,
                    const double2* Y1, double2* X1, const int* reach1, hipStream_t st, int split, int tiny,
                    bool nar, int maxns, bool rl) {
  if (nfronts <= 0) return;
  if (rl && maxns > 16 * RL_WMAX) rl = false;   // k_usolve2_rl: at most 4 rows per lane slot
  // nar && !rl: the column-split update part (k_usolve2_updc), then k_usolve2_level's pivot block
  UPair a{Y0, X0, reach0, skip0}, b{Y1, X1, reach1, nullptr};
  if (tiny > 0 && split <= 1) {
    // every pivot block of the level <= tiny (4 or 8): one wave per (front, group)
    dim3 gt((unsigned)((nfronts + 3) / 4), ngroups), bt(256);
    if (tiny <= 4) LAUNCH((k_usolve2_tiny<4>), gt, bt, st, P, lvl, nfronts, F, Fc, a, b);
    else LAUNCH((k_usolve2_tiny<8>), gt, bt, st, P, lvl, nfronts, F, Fc, a, b);
    return;
  }
  dim3 g(nfronts, ngroups), bl(64 * W);
  const int rs = split > 1;
  // split > 1: the pivot rows' update part over `split` workgroups per front first (the small-front
  // register shape: many short waves)
  if (rs && nar) {
    const int RB = (maxns + UPC_SR - 1) / UPC_SR;
    LAUNCH(k_usolve2_updc, dim3(nfronts * RB, ngroups), dim3(64 * UPC_W), st, P, lvl, F, Fc, a, b, RB);
  } else if (rs) {
    LAUNCH((k_usolve2_upd<true, 2, 4>), dim3(nfronts * split, ngroups), dim3(64 * SPLIT_W), st, P, lvl, F, Fc, a, b, split);
  }
  // symmetric mode only (the paired top-down pass serves the symmetric loss + gradient sweep).  Small-front levels:
  // 8 pivot rows per pass share each gathered update-row value, 2 values per chunk, 3 waves/SIMD (18 % less traffic
  // than 2 rows x 4 values at 4 waves/SIMD, the same time: profiles/r04/solve_traffic/)
  if (rs && nar && rl) {
    const int rpl = rl_rpl(maxns);
    const dim3 gq(nfronts, (unsigned)(Fc / RL_Q)), bq(64 * rl_waves(maxns));
    if (rpl == 1) LAUNCH((k_usolve2_rl<1>), gq, bq, st, P, lvl, F, Fc, a, b);
    else if (rpl == 2) LAUNCH((k_usolve2_rl<2>), gq, bq, st, P, lvl, F, Fc, a, b);
    else LAUNCH((k_usolve2_rl<4>), gq, bq, st, P, lvl, F, Fc, a, b);
  } else if (small) LAUNCH((k_usolve2_level<true, 8, 2, 3>), g, bl, st, P, lvl, F, Fc, a, b, rs);
  else LAUNCH((k_usolve2_level<true, 4, 8, 2>), g, bl, st, P, lvl, F, Fc, a, b, rs);
}

void launch_tangent_spmv(const int* ptr, const int* idx, const int* nzs, int nrows, const double2* Kd,
                         const double2* X, int64_t Fc, const double* rhsP, double2 beta, double2* Y, int accumulate,
                         hipStream_t st) {
  LAUNCH(k_tangent_spmv, dim3((nrows + 3) / 4, (unsigned)(Fc / 64)), dim3(256), st, ptr, idx, nzs, nrows, Kd, X, Fc,
         rhsP, beta, Y, accumulate);
}


void launch_residual(int mode, int rhs, const ResidDesc& d, const double2* X, int64_t Fc, double2* R, double* acc,
                     hipStream_t st, const double2* Mu, double2* cpart) {
  ResidArgs a;
  a.ptr = d.ptr; a.idx = d.idx; a.nzs = d.nzs; a.n = d.n;
  a.K = d.K; a.M = d.M; a.freqs = d.freqs; a.data = d.data; a.data_stride = d.data_stride; a.nvalid = d.nvalid;
  a.rhsP = d.rhsP; a.beta_re = d.beta_re; a.beta_im = d.beta_im; a.mass_sum = d.mass_sum;
  a.B = d.B; a.b_stride = d.b_stride; a.perm = d.perm; a.G = d.G; a.walk = d.walk;
  a.se = d.se; a.kpart = d.kpart; a.glist = d.glist;
  const dim3 g((unsigned)residual_parts(d.n), (unsigned)(d.glist ? REFINE_CAP : Fc / 64)), b(256);
  // unroll 8 on the forward walk with the contraction: 1.87 -> 1.94 ms per 2,048-frequency chunk (not taken)
  if (mode == 0 && rhs == 0 && Mu && d.kpart && d.n_stiff == 12)
    LAUNCH((k_residual<0, 0, true, 12>), g, b, st, a, X, Fc, R, acc, Mu, cpart);
  else if (mode == 0 && rhs == 0 && Mu && d.kpart && d.n_stiff == 18)
    LAUNCH((k_residual<0, 0, true, 18>), g, b, st, a, X, Fc, R, acc, Mu, cpart);
  else if (mode == 0 && rhs == 0 && Mu) LAUNCH((k_residual<0, 0, true>), g, b, st, a, X, Fc, R, acc, Mu, cpart);
  else if (R) {   // the refinement's residual: compensated
    if (mode == 0 && rhs == 0) LAUNCH((k_residual<0, 0, false, 0, true>), g, b, st, a, X, Fc, R, acc, Mu, cpart);
    else if (mode == 0) LAUNCH((k_residual<0, 2, false, 0, true>), g, b, st, a, X, Fc, R, acc, Mu, cpart);
    else if (rhs == 1) LAUNCH((k_residual<1, 1, false, 0, true>), g, b, st, a, X, Fc, R, acc, Mu, cpart);
    else LAUNCH((k_residual<1, 2, false, 0, true>), g, b, st, a, X, Fc, R, acc, Mu, cpart);
  } else if (mode == 0 && rhs == 0) LAUNCH((k_residual<0, 0>), g, b, st, a, X, Fc, R, acc, Mu, cpart);
  // the adjoint's check walk with 8 entries per gather batch: 757 -> 638 us per 2,048-frequency chunk
  // (gpurun_out/ru2_*)
  else if (mode == 0 && d.unroll == 8) LAUNCH((k_residual<0, 2, false, 0, false, 8>), g, b, st, a, X, Fc, R, acc, Mu, cpart);
  else if (mode == 0) LAUNCH((k_residual<0, 2>), g, b, st, a, X, Fc, R, acc, Mu, cpart);
  else if (rhs == 1) LAUNCH((k_residual<1, 1>), g, b, st, a, X, Fc, R, acc, Mu, cpart);
  else LAUNCH((k_residual<1, 2>), g, b, st, a, X, Fc, R, acc, Mu, cpart);
}

void launch_correct_finish(const FunctionalArgs& A, const double* fr0, const double2* cpart, int nparts, int64_t Fc,
                           int nvalid, int64_t q0, double* fr_out, double* loss_terms, double2* mscale,
                           hipStream_t st, double* gind, double2* tq, const RhsScale& bsc) {
  LAUNCH(k_correct_finish, dim3((unsigned)(Fc / 64)), dim3(256), st, A, fr0, cpart, nparts, Fc, nvalid, q0,
         fr_out, loss_terms, mscale, gind, tq, bsc);
}

void launch_berr_finish(double* acc, int64_t Fc, int nvalid, double tol, int flag, int* flags, double* berr_out,
                        int64_t q0, int which, hipStream_t st) {
  LAUNCH(k_berr_finish, dim3((unsigned)((Fc + 63) / 64)), dim3(64), st, acc, Fc, nvalid, tol, flag, flags, berr_out,
         q0, which);
}

void launch_scale_vec(double2* X, const double2* m, int n, int64_t Fc, hipStream_t st) {
  const int64_t count = (int64_t)n * Fc;
  LAUNCH(k_scale_vec, dim3((unsigned)((count + 255) / 256)), dim3(256), st, X, m, n, Fc);
}

void launch_axpy_vec(double2* X, const double2* D, int64_t count, hipStream_t st, const int* glist, int64_t Fc) {
  if (glist) count = count / Fc * REFINE_CAP * 64;   // rows x the listed groups
  LAUNCH(k_axpy_vec, dim3((unsigned)((count + 255) / 256)), dim3(256), st, X, D, count, glist, Fc);
}

void launch_select_groups(const double* gind, int ngroups, double tol, int* glist, hipStream_t st) {
  LAUNCH(k_select_groups, dim3(1), dim3(64), st, gind, ngroups, tol, glist);
}

void launch_functional_tangent(const FunctionalArgs& A, const double2* X, const double2* DX, int64_t Fc, int nvalid,
                               int64_t q0, double2* G, hipStream_t st) {
  LAUNCH(k_functional_tangent, dim3((unsigned)((Fc + 63) / 64)), dim3(64), st, A, X, DX, Fc, nvalid, q0, G);
}

void launch_functional(const FunctionalArgs& A, const double2* X, int64_t Fc, int nvalid, int64_t q0, double* fr_out,
                       double* loss_terms, double2* G, hipStream_t st) {
  LAUNCH(k_functional, dim3((unsigned)((Fc + 63) / 64)), dim3(64), st, A, X, Fc, nvalid, q0, fr_out, loss_terms, G);
}

void launch_gather_entries(const int4* ent, int nent, const double* stiff, int ns, double* se, hipStream_t st) {
  if (nent <= 0) return;
  LAUNCH(k_gather_entries, dim3((nent + 255) / 256), dim3(256), st, ent, nent, stiff, ns, se);
}


void launch_contract_eg(const int4* ent, int nent, const double* se, int n_stiff, const double2* Lam, const double2* X,
                        int64_t Fc, int nvalid, double2* partial, hipStream_t st, const double2* msc) {
  const dim3 g(contract_eg_parts(nent)), b(256);
  if (n_stiff == 12 && msc) LAUNCH((k_contract_eg<12, CEG_EW, true>), g, b, st, ent, nent, se, Lam, X, Fc, nvalid, msc, partial);
  else if (n_stiff == 12) LAUNCH((k_contract_eg<12, CEG_EW, false>), g, b, st, ent, nent, se, Lam, X, Fc, nvalid, msc, partial);
  else if (msc) LAUNCH((k_contract_eg<18, CEG_EW, true>), g, b, st, ent, nent, se, Lam, X, Fc, nvalid, msc, partial);
  else LAUNCH((k_contract_eg<18, CEG_EW, false>), g, b, st, ent, nent, se, Lam, X, Fc, nvalid, msc, partial);
}

void launch_rhs_dot(const int* sup, const double* val, int n_sup, const double2* Lam, int64_t Fc, double2* t_out,
                    hipStream_t st, const double2* msc) {
  LAUNCH(k_rhs_dot, dim3((unsigned)((Fc + 63) / 64)), dim3(64), st, sup, val, n_sup, Lam, Fc, msc, t_out);
}

void launch_reduce_q(const double2* kpart, int nparts, int n_stiff, const double2* msc, int nvalid, int64_t Fc,
                     double2* partial, hipStream_t st) {
  LAUNCH(k_reduce_q, dim3(n_stiff, (unsigned)(Fc / 64)), dim3(256), st, kpart, nparts, n_stiff, msc, nvalid, Fc, partial);
}

void launch_reduce(const double2* partial, int nparts, int n_stiff, const double2* t_q, const CoefPack& e,
                   const double* loss_terms, int nvalid, int64_t Fc, double2* w_out, double* loss_out,
                   hipStream_t st) {
  LAUNCH(k_reduce, dim3(n_stiff + 1), dim3(1024), st, partial, nparts, n_stiff, t_q, e, loss_terms, nvalid, Fc, w_out,
         loss_out);
}

void launch_unpermute(const int* perm, int n, const double2* X, int64_t Fc, int nvalid, double2* out, hipStream_t st) {
  LAUNCH(k_unpermute, dim3(n, (nvalid + 63) / 64), dim3(64), st, perm, n, X, Fc, nvalid, out);
}

void launch_matvec(const int* colptr, const int* rowind, int n, const double2* data, int64_t ds, const double2* x,
                   int64_t xs, double2* y, int transpose, int batch, hipStream_t st) {
  LAUNCH(k_matvec, dim3((n + 255) / 256, batch), dim3(256), st, colptr, rowind, n, data, ds, x, xs, y, transpose,
         batch);
}

static DirArgs make_dir(const DirDesc& d) {
  DirArgs a;
  a.dir = d.dir; a.crow = d.crow; a.cptr = d.cptr; a.ce = d.ce; a.dptr = d.dptr; a.de = d.de;
  a.K = d.K; a.M = d.M; a.freqs = d.freqs;
  return a;
}

void launch_dirichlet_rhs(int src, const DirDesc& d, int n_crow, const RhsDesc& rd, double2* G, double2* Bc,
                          int64_t Fc, hipStream_t st) {
  if (n_crow <= 0) return;
  dim3 g(n_crow, (unsigned)(Fc / 64)), b(64);
  if (src == 0) LAUNCH(k_dirichlet_rhs<0>, g, b, st, make_dir(d), make_rhs(rd), G, Bc, Fc);
  else LAUNCH(k_dirichlet_rhs<2>, g, b, st, make_dir(d), make_rhs(rd), G, Bc, Fc);
}

void launch_dirichlet_post(const DirDesc& d, int n_dir, double2* X, int64_t Fc, hipStream_t st, const int* glist) {
  if (n_dir <= 0) return;
  LAUNCH(k_dirichlet_post, dim3(n_dir, (unsigned)(glist ? REFINE_CAP : Fc / 64)), dim3(64), st, make_dir(d), X, Fc, glist);
}

// fill padded frequency slots with the last valid frequency (keeps padded lanes well-posed)
// A chunk's start in one kernel (no memcpy / memset nodes in a captured sweep): its frequencies from the caller's
// array, padded to Fc with the last one, and its flags cleared.  Fresh outputs (pfr_sweep_fresh, first chunk): the
// caller's loss, gradient partials and flags zeroed and the backward errors set to NaN here, instead of by separate
// fills before the sweep.
struct FreshOut {
  double* loss = nullptr;
  double* w = nullptr;
  int nw = 0;               // doubles of w
  int* flags = nullptr;
  double* berr = nullptr;   // 2 per frequency
  int nfreq = 0;
};
__global__ void k_chunk_start(double* __restrict__ freqs, const double* __restrict__ src, int nvalid, int64_t Fc,
                              int* __restrict__ flags, FreshOut o) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q < Fc) {
    freqs[q] = src[q < nvalid ? q : nvalid - 1];
    flags[q] = 0;
  }
  if (o.nfreq > 0) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = q; i < o.nfreq; i += stride) {
      if (o.flags) o.flags[i] = 0;
      if (o.berr) {
        o.berr[2 * i] = __longlong_as_double(0x7ff8000000000000LL);
        o.berr[2 * i + 1] = __longlong_as_double(0x7ff8000000000000LL);
      }
    }
    if (o.loss && q == 0) o.loss[0] = 0.0;
    if (o.w && q < o.nw) o.w[q] = 0.0;
  }
}
void launch_chunk_start(double* freqs, const double* src, int nvalid, int64_t Fc, int* flags, hipStream_t st,
                        double* loss, double* w, int nw, int* out_flags, double* berr, int nfreq) {
  FreshOut o;
  o.loss = loss;
  o.w = w;
  o.nw = nw;
  o.flags = out_flags;
  o.berr = berr;
  o.nfreq = nfreq;
  LAUNCH(k_chunk_start, dim3((unsigned)((Fc + 255) / 256)), dim3(256), st, freqs, src, nvalid, Fc, flags, o);
}
__global__ void k_zero(double2* __restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = make_double2(0.0, 0.0);
}
void launch_zero(double2* p, int64_t n, hipStream_t st) {
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8192);
  LAUNCH(k_zero, dim3((unsigned)blocks), dim3(256), st, p, n);
}
__global__ void k_flags_merge(const int* chunk, int nvalid, int* out) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q < nvalid) out[q] |= chunk[q];
}
void launch_flags_merge(const int* chunk, int nvalid, int* out, hipStream_t st) {
  LAUNCH(k_flags_merge, dim3((nvalid + 63) / 64), dim3(64), st, chunk, nvalid, out);
}

}  // namespace pfr
