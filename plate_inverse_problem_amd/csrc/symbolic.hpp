// Host-side symbolic analysis for the batched multifrontal LU.
//
// Replaces the UMFPACK symbolic phase the reference runs once per pattern
// (InnerState::add_mat -> umfpack_zi_symbolic, source/jax_plate_lib/include/
// InnerState.h:120-162, umfpack_interface.h:20-64).  Everything here is plain
// C++17: fill-reducing nested-dissection ordering, elimination tree,
// supernodes (relaxed), and the maps the HIP kernels need (front index lists,
// original-entry assembly lists, child->parent extend-add lists, level
// schedule).  The numeric phase uses a STATIC diagonal pivot order shared by
// every frequency (see DESIGN.md "Pivoting").
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace pfr {

struct SymbolicOptions {
  int leaf_size = 10000;     // nested-dissection parts at or below this size are ordered by minimum degree
  int relax_small = 4;       // always amalgamate supernodes with <= this many pivots
  int relax_mid = 8;         // ... with <= this many pivots when zero fraction < zrelax_mid
  int relax_big = 24;        // ... with <= this many pivots when zero fraction < zrelax_big
  double zrelax_mid = 0.5;
  double zrelax_big = 0.1;
  int ordering = 0;          // 0 = nested dissection + multiple minimum degree leaves, 1 = natural
                             // (tests), 2 = nested dissection + exact minimum degree leaves (round 1-3)
  int md_delta = 4;          // multiple minimum degree: eliminate nodes of degree <= min + md_delta
  int symmetric = 0;         // 1 = symmetric-structure analysis with decoupled Dirichlet nodes
  std::vector<int> last;     // nodes eliminated last, together (they form the root front)
  int max_ns = 256;          // > 0: fundamental supernodes are split into pieces of at most this many pivots
};

struct Front {
  int32_t ns;        // pivots
  int32_t f;         // front size = ns + r
  int32_t row0;      // first global front-row id (offset into idx/relpos/asm_ptr/ea_ptr)
  int32_t col0;      // first pivot column (permuted numbering)
  int32_t parent;    // parent front or -1
  int32_t level;     // 0 = leaves
  int64_t off;       // offset (entries) of the dense f x f front in factor storage
  int64_t wv;        // offset (entries) of the f-long work vector
};

struct Symbolic {
  int32_t n = 0;
  int64_t nnz = 0;
  std::vector<int32_t> perm;    // new -> old
  std::vector<int32_t> iperm;   // old -> new
  std::vector<Front> fronts;
  // per front row (size total_rows = sum f)
  std::vector<int32_t> idx;     // permuted global index of the row/column
  std::vector<int32_t> relpos;  // for non-pivot rows: position in the parent front; -1 otherwise
  std::vector<int32_t> row_front; // front owning each front row
  std::vector<int32_t> asm_ptr; // original entries of each front row: [asm_ptr[r], asm_ptr[r+1])
  std::vector<int32_t> asm_col; //   local column of the entry
  std::vector<int32_t> asm_nz;  //   index of the entry in the CSC value array
  std::vector<int32_t> ea_ptr;  // extend-add sources of each front row
  std::vector<int32_t> ea_src;  //   global front-row id (of a child's update row) added into this row
  std::vector<int32_t> level_ptr;    // fronts of level l: level_fronts[level_ptr[l] .. level_ptr[l+1])
  std::vector<int32_t> level_fronts;
  std::vector<int32_t> level_maxf;   // largest front of each level
  // CSC coordinates in permuted numbering (for the gradient contraction)
  std::vector<int32_t> prow, pcol;
  int64_t total_rows = 0;       // sum f
  int64_t factor_entries = 0;   // sum f^2
  int64_t nnz_lu = 0;           // sum (2 ns f - ns^2)
  double factor_flops = 0.0;    // real flops of the numeric factorisation (complex MAC = 8)
  int32_t max_front = 0;
  // symmetric mode (options.symmetric): Dirichlet nodes d (rows holding only their diagonal)
  // are decoupled 1 x 1 fronts; the entries (i, d) of their columns are not assembled into
  // any front but listed here (forward right-hand-side and adjoint corrections)
  int symmetric = 0;
  std::vector<int32_t> dir_p, dir_nz;            // per Dirichlet node: permuted index, diagonal entry
  std::vector<int32_t> cpl_p, cpl_dir, cpl_nz;   // coupling entries sorted by permuted row: row, dir slot, entry
  std::string error;
};

// Build the symbolic analysis of an n x n CSC pattern.  Returns 0 on success.
int analyse(int32_t n, int64_t nnz, const int32_t* colptr, const int32_t* rowind,
            const SymbolicOptions& opt, Symbolic& out);

}  // namespace pfr
