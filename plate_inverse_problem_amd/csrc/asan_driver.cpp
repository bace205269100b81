// Host-only driver of the symbolic analysis for sanitizer builds (`make asan-host`: g++ with
// -fsanitize=address,undefined; no HIP).  The C ABI's pfr_symbolic_create runs exactly this
// pfr::analyse (api.cpp); tests/test_asan_host.py feeds it the plate patterns with every ordering
// option the engine uses and compares its statistics with libpfr's.
//
// Input file (little-endian): int32 n, int64 nnz, int32 colptr[n + 1], int32 rowind[nnz],
// int32 n_last, int32 last[n_last].  Each further argument is one option set
// "leaf,ordering,symmetric,max_ns,md_delta,use_last"; per set one output line:
// "n_fronts n_levels max_front total_rows nnz_lu factor_flops perm_hash n_dirichlet n_coupling".
#include <cstdio>
#include <cstdlib>
#include <vector>

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
  }
  return 0;
}
