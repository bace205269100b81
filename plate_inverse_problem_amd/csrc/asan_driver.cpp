// Host-only driver of the symbolic analysis and the launch plans for sanitizer builds (`make asan-host`: g++
// with -fsanitize=address,undefined; no HIP).  The C ABI's pfr_symbolic_create runs exactly this pfr::analyse
// and pfr_solver_create this pfr::build_plan (api.cpp); tests/test_asan_host.py feeds it the plate patterns with
// every ordering option the engine uses, compares the statistics with libpfr's, and has every plan checked
// (pfr::check_plan) for every engine shape: chunks of 64 .. 4,096 frequencies (one or two lanes split a sweep
// into such chunks), Schur block thresholds and solve split targets.
//
// Input file (little-endian): int32 n, int64 nnz, int32 colptr[n + 1], int32 rowind[nnz],
// int32 n_last, int32 last[n_last].  Each further argument is one option set
// "leaf,ordering,symmetric,max_ns,md_delta,use_last"; per set one output line:
// "n_fronts n_levels max_front total_rows nnz_lu factor_flops perm_hash n_dirichlet n_coupling", then one line
// "plan ok <plans checked>" or "plan error <shape>: <violation>".
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "plan.hpp"
#include "symbolic.hpp"

namespace {
template <class T>
bool rd(FILE* f, T* p, size_t n) {
  return fread(p, sizeof(T), n, f) == n;
}
}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s pattern.bin leaf,ordering,symmetric,max_ns,md_delta,use_last ...\n", argv[0]);
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  int32_t n = 0, n_last = 0;
  int64_t nnz = 0;
  if (!rd(f, &n, 1) || !rd(f, &nnz, 1) || n <= 0 || nnz < 0) return 2;
  std::vector<int32_t> colptr(n + 1), rowind(nnz);
  if (!rd(f, colptr.data(), colptr.size()) || (nnz && !rd(f, rowind.data(), rowind.size())) || !rd(f, &n_last, 1))
    return 2;
  std::vector<int32_t> last(n_last);
  if (n_last && !rd(f, last.data(), last.size())) return 2;
  fclose(f);
  for (int a = 2; a < argc; ++a) {
    int leaf, ordering, symmetric, max_ns, md_delta, use_last;
    if (sscanf(argv[a], "%d,%d,%d,%d,%d,%d", &leaf, &ordering, &symmetric, &max_ns, &md_delta, &use_last) != 6)
      return 2;
    pfr::SymbolicOptions o;
    o.leaf_size = leaf;
    o.ordering = ordering;
    o.symmetric = symmetric;
    o.max_ns = max_ns;
    o.md_delta = md_delta;
    if (use_last) o.last.assign(last.begin(), last.end());
    pfr::Symbolic S;
    if (pfr::analyse(n, nnz, colptr.data(), rowind.data(), o, S) != 0) {
      printf("error %s\n", S.error.c_str());
      continue;
    }
    uint64_t h = 1469598103934665603ull;   // FNV-1a over the permutation
    for (int32_t v : S.perm) h = (h ^ (uint32_t)v) * 1099511628211ull;
    printf("%d %d %d %lld %lld %.17g %llu %d %d\n", (int)S.fronts.size(), (int)S.level_ptr.size() - 1, S.max_front,
           (long long)S.total_rows, (long long)S.nnz_lu, S.factor_flops, (unsigned long long)h, (int)S.dir_p.size(),
           (int)S.cpl_p.size());
    // launch plans of every engine shape
    int checked = 0;
    std::string err;
    const int blk_mins[] = {24, 0, 4};
    const int splits[] = {256, 0, 1000000};
    const int64_t chunks[] = {64, 512, 1024, 2048, 4096};
    for (int bm : blk_mins) {
      pfr::PlanOptions po;
      po.blk_min = bm;
      pfr::Plan P;
      if (pfr::build_plan(S, po, P, err)) {
        printf("plan error blk_min=%d: %s\n", bm, err.c_str());
        goto next;
      }
      for (int64_t Fc : chunks)
        for (int sp : splits) {
          const std::string e = pfr::check_plan(S, P, Fc, sp);
          if (!e.empty()) {
            printf("plan error blk_min=%d Fc=%lld split=%d: %s\n", bm, (long long)Fc, sp, e.c_str());
            goto next;
          }
          ++checked;
        }
    }
    {
      // reach lists of the loss support (the last nodes, when given) and of every 97th row
      std::vector<int32_t> foc(S.n, -1), par, rows, mark, list, ptr;
      for (size_t t = 0; t < S.fronts.size(); ++t) {
        par.push_back(S.fronts[t].parent);
        for (int a = 0; a < S.fronts[t].ns; ++a) foc[S.fronts[t].col0 + a] = (int32_t)t;
      }
      for (int32_t v : last) rows.push_back(S.iperm[v]);
      for (int i = 0; i < S.n; i += 97) rows.push_back(i);
      pfr::reach_lists(foc, par, S.level_ptr, S.level_fronts, rows, mark, list, ptr);
      if ((int)ptr.size() != (int)S.level_ptr.size() || ptr.back() != (int32_t)list.size()) {
        printf("plan error reach lists\n");
        goto next;
      }
    }
    printf("plan ok %d\n", checked);
  next:;
  }
  return 0;
}
