// Host-side launch plans (plan.hpp): built by pfr_solver_create (api.cpp) and, under AddressSanitizer /
// UndefinedBehaviorSanitizer, by the host driver (asan_driver.cpp).  HIP-free.
#include "plan.hpp"

#include <algorithm>
#include <climits>
#include <cstdio>
#include <utility>

namespace pfr {

Workspace workspace(const Symbolic& S, int64_t Fc, int n_crow) {
  Workspace w;
  const int64_t n = S.n;
  w.F = S.factor_entries * Fc;
  w.WV = S.total_rows * Fc;
  w.nvec = n * Fc;
  w.n_nvec = 7;                                             // X, Y, XA, G, Y2, XR, Gx (the refinement's seed)
  w.cpart = (int64_t)residual_parts(S.n) * Fc;             // k_residual: one partial per (workgroup, frequency)
  w.kpart = (int64_t)residual_parts(S.n) * 18 * Fc;        // ... and per stiffness matrix (contraction in the walk)
  w.berr_acc = 2 * Fc;
  w.gind = Fc / 64;
  w.Bc = (int64_t)std::max(1, n_crow) * Fc;
  if (S.symmetric) {                                        // functional from the bottom-up passes
    w.WVk = 3 * S.total_rows * Fc;
    w.YVk = 2 * n * Fc;
    w.fn_parts = 3 * (int64_t)FN_PARTS_HOST * Fc;
    w.fcoef = 3 * Fc;
  }
  int64_t b = 16 * (w.F + w.WV + w.n_nvec * w.nvec + w.cpart + w.kpart + w.WVk + w.YVk + w.fn_parts + w.fcoef + w.Bc);
  b += Fc * (8 + 8 + 4 + 16) + Fc * (8 + 16) + 8 * (w.berr_acc + w.gind);   // freqs, loss, flags, tq; fr0, mscale
  w.bytes = b;
  return w;
}

namespace {

// children's update-matrix entries per A22 position of front t: the first densely (r x r, -1 none), the rare
// further ones (two or more children covering a position) sorted aside as (i r + j, element id)
void a22_sources(const Symbolic& S, const std::vector<std::vector<int>>& kids, int t, bool sym,
                 std::vector<int32_t>& first, std::vector<std::pair<int32_t, int32_t>>& more) {
  const Front& F = S.fronts[t];
  const int r = F.f - F.ns;
  first.assign((size_t)r * r, -1);
  more.clear();
  for (int c : kids[t]) {
    const Front& C = S.fronts[c];
    const int32_t* rp = S.relpos.data() + C.row0;
    for (int a = C.ns; a < C.f; ++a) {
      const int i = rp[a] - F.ns;
      if (i < 0) continue;
      for (int b = C.ns; b < C.f; ++b) {
        const int j = rp[b] - F.ns;
        if (j < 0 || (sym && j > i)) continue;   // symmetric: lower triangle only
        const int32_t id = (int32_t)(C.off + (int64_t)a * C.f + b);
        int32_t& f1 = first[(size_t)i * r + j];
        if (f1 < 0)
          f1 = id;
        else
          more.emplace_back(i * r + j, id);
      }
    }
  }
  std::sort(more.begin(), more.end());
}

template <class F>
void each_more(const std::vector<std::pair<int32_t, int32_t>>& more, int32_t key, F&& fn) {
  auto lo = std::lower_bound(more.begin(), more.end(), std::make_pair(key, INT32_MIN));
  for (; lo != more.end() && lo->first == key; ++lo) fn(lo->second);
}

}  // namespace

int build_plan(const Symbolic& S, const PlanOptions& o, Plan& P, std::string& err) {
  P = Plan();
  if (S.max_front > MAX_FRONT) {
    err = "front larger than MAX_FRONT (plan.hpp)";
    return 1;
  }
  if (S.factor_entries > INT32_MAX) {
    err = "front storage exceeds int32 element ids";
    return 1;
  }
  const bool sym = S.symmetric != 0;
  const int L = (int)S.level_ptr.size() - 1;
  const int nfr = (int)S.fronts.size();
  P.L = L;
  P.sym = sym;
  P.level_maxns.assign(L, 0);
  for (const Front& F : S.fronts) P.level_maxns[F.level] = std::max(P.level_maxns[F.level], F.ns);
  std::vector<std::vector<int>> kids(nfr);
  for (int t = 0; t < nfr; ++t)
    if (S.fronts[t].parent >= 0) kids[S.fronts[t].parent].push_back(t);

  // ---- Schur complement: 16 x 16 blocks (symmetric mode, update blocks of >= blk_min rows) or 4 x 4 tiles, level
  // by level, with the children's update-matrix entries landing in each (the extend-add as a gather)
  P.blk_front.assign(nfr, 0);
  P.gxp.assign(1, 0);
  P.bgxp.assign(1, 0);
  P.tile_ptr.assign(1, 0);
  P.blk_ptr.assign(1, 0);
  std::vector<int32_t> first;
  std::vector<std::pair<int32_t, int32_t>> more;
  for (int l = 0; l < L; ++l) {
    for (int e = S.level_ptr[l]; e < S.level_ptr[l + 1]; ++e) {
      const int t = S.level_fronts[e];
      const Front& F = S.fronts[t];
      const int r = F.f - F.ns;
      a22_sources(S, kids, t, sym, first, more);
      if (sym && o.blk_min > 0 && r >= o.blk_min) {
        // blocks touching the lower triangle; wave w owns the 4 x 4 tile (w / 4, w % 4)
        constexpr int B = SCHUR_BLK, BC = SCHUR_BLK, tcw = BC / 4;
        for (int i0 = 0; i0 < r; i0 += B)
          for (int j0 = 0; j0 < i0 + B; j0 += BC) {
            P.blocks.push_back({t, i0, j0, 0});
            for (int w = 0; w < BC; ++w)
              for (int pos = 0; pos < 16; ++pos) {
                const int i = i0 + 4 * (w / tcw) + pos / 4, j = j0 + 4 * (w % tcw) + pos % 4;
                if (i >= r || j > i) {
                  P.bg1.push_back(-1);
                  continue;
                }
                P.bg1.push_back(first[(size_t)i * r + j]);
                each_more(more, i * r + j, [&](int32_t id) { P.bgx.push_back({w * 16 + pos, id}); });
              }
            P.bgxp.push_back((int32_t)P.bgx.size());
          }
        P.blk_front[t] = 1;
        continue;
      }
      // super-tiles (symmetric: those touching the lower triangle); lane group `sub` owns the TM x TN tile at
      // (TM (sub / SC), TN (sub % SC)); per super-tile the dense first-source ids, then one overflow range
      constexpr int TM = SCHUR_TM, TN = SCHUR_TN, SR = SCHUR_SR, SC = SCHUR_SC, STR = TM * SR, STC = TN * SC;
      for (int i0 = 0; i0 < r; i0 += STR)
        for (int j0 = 0; j0 < r && (!sym || j0 <= i0 + STR - 1); j0 += STC) {
          P.tiles.push_back({t, i0, j0, 0});
          for (int sub = 0; sub < SR * SC; ++sub)
            for (int pos = 0; pos < TM * TN; ++pos) {
              const int i = i0 + TM * (sub / SC) + pos / TN, j = j0 + TN * (sub % SC) + pos % TN;
              if (i >= r || j >= r || (sym && j > i)) {
                P.g1.push_back(-1);
                continue;
              }
              P.g1.push_back(first[(size_t)i * r + j]);
              each_more(more, i * r + j, [&](int32_t id) { P.gx.push_back({sub * TM * TN + pos, id}); });
            }
          P.gxp.push_back((int32_t)P.gx.size());
        }
    }
    P.tile_ptr.push_back((int32_t)P.tiles.size());
    P.blk_ptr.push_back((int32_t)P.blocks.size());
  }

  // ---- panel-region sources of every front, as a gather: per entry the original matrix entry (or -1) and the
  // first child update-matrix entry landing there (or -1), rare further child entries in overflow lists
  //  * A11: assembly records (dst, nz, src, -) in chunks of 8 (k_assemble_level), levels padded to 8 records;
  //  * L21 rows / U12 columns: gathered by k_offdiag_level itself at their first load (records (nz, src) per
  //    item x row slot x pivot, item.w = offset), so those entries are never stored before their final value
  P.asm_xp.assign(1, 0);
  P.oxp.assign(1, 0);
  P.asm_ptr.assign(1, 0);
  P.item_ptr.assign(1, 0);
  std::vector<int32_t> nzm, s1m;
  std::vector<std::pair<int32_t, int32_t>> morem;   // (a * f + b, id)
  bool ok0 = sym;
  std::vector<std::pair<int32_t, std::vector<int32_t>>> f0;   // level-0 fronts: (front, records)
  for (int l = 0; l < L; ++l) {
    for (int e = S.level_ptr[l]; e < S.level_ptr[l + 1]; ++e) {
      const int t = S.level_fronts[e];
      const Front& F = S.fronts[t];
      const int f = F.f, ns = F.ns;
      nzm.assign((size_t)f * f, -1);
      s1m.assign((size_t)f * f, -1);
      morem.clear();
      for (int a = 0; a < f; ++a) {
        const int r = F.row0 + a;
        const int width = a < ns ? f : ns;
        for (int x = S.asm_ptr[r]; x < S.asm_ptr[r + 1]; ++x)
          if (S.asm_col[x] < width) nzm[(size_t)a * f + S.asm_col[x]] = S.asm_nz[x];
        for (int x = S.ea_ptr[r]; x < S.ea_ptr[r + 1]; ++x) {
          const int src = S.ea_src[x];
          const Front& C = S.fronts[S.row_front[src]];
          const int32_t* rp = S.relpos.data() + C.row0;
          for (int b = C.ns; b < C.f; ++b) {
            const int pb = rp[b];
            if (pb >= width) continue;
            // symmetric: the child's update matrix holds its lower triangle only
            const int ca = src - C.row0;
            const int32_t id = (int32_t)(C.off + (sym && ca < b ? (int64_t)b * C.f + ca : (int64_t)ca * C.f + b));
            int32_t& s1 = s1m[(size_t)a * f + pb];
            if (s1 < 0)
              s1 = id;
            else
              morem.emplace_back(a * f + pb, id);
          }
        }
      }
      std::sort(morem.begin(), morem.end());
      if (l == 0 && ok0) {
        ok0 = ns <= F0_NS && f - ns <= F0_RM && morem.empty();
        std::vector<int32_t> rec;
        for (int a = 0; a < f && ok0; ++a)
          for (int b = 0; b < std::min(a + 1, ns); ++b) {
            ok0 = ok0 && s1m[(size_t)a * f + b] < 0;   // leaves: no child entries
            rec.push_back(nzm[(size_t)a * f + b]);
          }
        if (ok0) f0.emplace_back(t, std::move(rec));
      }
      for (int a = 0; a < ns; ++a)
        for (int b = 0; b < (sym ? a + 1 : ns); ++b) {   // symmetric: A11's lower triangle only
          const int k = (int)(P.asm_rec.size() % 8);
          P.asm_rec.push_back({(int32_t)(F.off + (int64_t)a * f + b), nzm[(size_t)a * f + b], s1m[(size_t)a * f + b], 0});
          each_more(morem, a * f + b, [&](int32_t id) { P.asm_x.push_back({k, id}); });
          if (P.asm_rec.size() % 8 == 0) P.asm_xp.push_back((int32_t)P.asm_x.size());
        }
      for (int kind = 0; kind < (sym ? 1 : 2); ++kind)   // symmetric: U12 = diag(U11) L21^T implicit
        for (int i0 = ns; i0 < f; i0 += OFF_G * OFF_RPL) {
          P.items.push_back({t, i0, kind, (int32_t)P.orec.size()});
          for (int slot = 0; slot < OFF_G * OFF_RPL; ++slot)   // row i0 + slot = i0 + OFF_G h + lane group
            for (int c = 0; c < ns; ++c) {
              const int idx = i0 + slot;
              if (idx >= f) {
                P.orec.push_back({-1, -1});
                continue;
              }
              const int a = kind == 0 ? idx : c, b = kind == 0 ? c : idx;
              P.orec.push_back({nzm[(size_t)a * f + b], s1m[(size_t)a * f + b]});
              each_more(morem, a * f + b, [&](int32_t id) { P.ox.push_back({c * OFF_G * OFF_RPL + slot, id}); });
            }
          P.oxp.push_back((int32_t)P.ox.size());
        }
    }
    while (P.asm_rec.size() % 8) {        // pad: no-op records (dst = -1)
      P.asm_rec.push_back({-1, -1, -1, 0});
      if (P.asm_rec.size() % 8 == 0) P.asm_xp.push_back((int32_t)P.asm_x.size());
    }
    P.asm_ptr.push_back((int32_t)P.asm_rec.size());
    P.item_ptr.push_back((int32_t)P.items.size());
  }

  // ---- the fused bottom level
  P.fused0 = ok0 && !f0.empty() && L > 0;
  if (P.fused0) {
    std::stable_partition(f0.begin(), f0.end(), [&](const auto& x) { return S.fronts[x.first].ns <= 2; });
    P.f0_ptr.assign(1, 0);
    for (const auto& x : f0) {
      P.f0_front.push_back(x.first);
      P.f0_nz.insert(P.f0_nz.end(), x.second.begin(), x.second.end());
      P.f0_ptr.push_back((int32_t)P.f0_nz.size());
      P.f0_small += S.fronts[x.first].ns <= 2;
    }
  }

  // ---- algorithmic bytes per frequency and level of classes 0-4 (16 B per complex entry loaded or stored)
  P.lev_bytes.assign(L, std::array<int64_t, NKC>{});
  for (int t = 0; t < nfr; ++t) {
    const Front& F = S.fronts[t];
    const int64_t r = F.f - F.ns, ns = F.ns;
    const int64_t a11 = sym ? ns * (ns + 1) / 2 : ns * ns;
    auto& b = P.lev_bytes[F.level];
    b[0] += 16 * a11;                                                // A11 (symmetric: lower) stores
    b[1] += 16 * (a11 + ns * ns);                                    // A11 read + L11 / U11 write
    b[2] += 16 * ((sym ? 1 : 2) * r * ns + ns * ns);                 // L21 / U12 stores + L11 / U11 read
    b[3 + (P.blk_front[t] ? 0 : 1)] += 16 * ((sym ? r * (r + 1) / 2 : r * r) + (sym ? 1 : 2) * r * ns);   // A22 + L21
  }
  for (int l = 0; l < L; ++l) {                                      // + the children's entries each class gathers
    auto& b = P.lev_bytes[l];
    int64_t g = 0;
    for (int r = P.asm_ptr[l]; r < P.asm_ptr[l + 1]; ++r) g += P.asm_rec[r].z >= 0;
    b[0] += 16 * (g + P.asm_xp[P.asm_ptr[l + 1] / 8] - P.asm_xp[P.asm_ptr[l] / 8]);
    g = 0;
    const int64_t o0 = P.item_ptr[l] < (int)P.items.size() ? P.items[P.item_ptr[l]].w : (int64_t)P.orec.size();
    const int64_t o1 = P.item_ptr[l + 1] < (int)P.items.size() ? P.items[P.item_ptr[l + 1]].w : (int64_t)P.orec.size();
    for (int64_t x = o0; x < o1; ++x) g += P.orec[x].y >= 0;
    b[2] += 16 * (g + P.oxp[P.item_ptr[l + 1]] - P.oxp[P.item_ptr[l]]);
    g = 0;
    for (size_t x = (size_t)P.blk_ptr[l] * SCHUR_BLK_IDS; x < (size_t)P.blk_ptr[l + 1] * SCHUR_BLK_IDS; ++x) g += P.bg1[x] >= 0;
    b[3] += 16 * (g + P.bgxp[P.blk_ptr[l + 1]] - P.bgxp[P.blk_ptr[l]]);
    g = 0;
    for (size_t x = (size_t)P.tile_ptr[l] * SCHUR_TILE; x < (size_t)P.tile_ptr[l + 1] * SCHUR_TILE; ++x) g += P.g1[x] >= 0;
    b[4] += 16 * (g + P.gxp[P.tile_ptr[l + 1]] - P.gxp[P.tile_ptr[l]]);
  }
  if (P.fused0) {   // level 0 in one pass (class 0): A11 block, L21 rows and update block stored once, nothing read back
    auto& b = P.lev_bytes[0];
    b = {};
    for (const int32_t t : P.f0_front) {
      const int64_t ns = S.fronts[t].ns, r = S.fronts[t].f - ns;
      b[0] += 16 * (ns * ns + r * ns + r * (r + 1) / 2);
    }
  }

  // ---- symmetric mode: Dirichlet decoupling lists -- coupled rows (with their entries), per Dirichlet node the
  // entries of its column (adjoint correction), the coupled-row slot of every permuted row
  P.cslot.assign(S.n, -1);
  P.cptr_dir.assign(1, 0);
  P.dptr.assign(1, 0);
  if (sym && !S.dir_p.empty()) {
    for (size_t d = 0; d < S.dir_p.size(); ++d) P.dir.push_back({S.dir_p[d], S.dir_nz[d]});
    for (size_t c = 0; c < S.cpl_p.size(); ++c) {
      if (P.crow.empty() || P.crow.back() != S.cpl_p[c]) {
        if (!P.crow.empty()) P.cptr_dir.push_back((int32_t)P.ce.size());
        P.cslot[S.cpl_p[c]] = (int32_t)P.crow.size();
        P.crow.push_back(S.cpl_p[c]);
      }
      P.ce.push_back({S.cpl_dir[c], S.cpl_nz[c]});
    }
    P.cptr_dir.push_back((int32_t)P.ce.size());
    for (size_t d = 0; d < S.dir_p.size(); ++d) {
      for (size_t c = 0; c < S.cpl_p.size(); ++c)
        if (S.cpl_dir[c] == (int32_t)d) P.de.push_back({S.cpl_p[c], S.cpl_nz[c]});
      P.dptr.push_back((int32_t)P.de.size());
    }
    P.n_dir = (int)S.dir_p.size();
    P.n_crow = (int)(P.cptr_dir.size() - 1);
  }

  // ---- permuted matrix compressed by rows and by columns (residual walks, Hessian tangent operators)
  auto compress = [&](const std::vector<int32_t>& key, const std::vector<int32_t>& other, std::vector<int32_t>& ptr,
                      std::vector<int32_t>& idx, std::vector<int32_t>& nz) {
    ptr.assign(S.n + 1, 0);
    idx.assign(S.nnz, 0);
    nz.assign(S.nnz, 0);
    for (int64_t e = 0; e < S.nnz; ++e) ++ptr[key[e] + 1];
    for (int i = 0; i < S.n; ++i) ptr[i + 1] += ptr[i];
    std::vector<int32_t> fill(ptr.begin(), ptr.end() - 1);
    for (int64_t e = 0; e < S.nnz; ++e) {
      const int32_t at = fill[key[e]]++;
      idx[at] = other[e];
      nz[at] = (int32_t)e;
    }
  };
  compress(S.prow, S.pcol, P.rptr, P.ridx, P.rnz);
  compress(S.pcol, S.prow, P.cptr, P.cidx, P.cnz);

  // ---- union row structure of the gradient contraction (k_contract_eg): rows in original order (mesh-local:
  // neighbouring walks gather the same solution rows whatever the ordering), entries of a row by permuted column
  {
    std::vector<int64_t> key(S.nnz);
    std::vector<int32_t> ord(S.nnz);
    for (int64_t e = 0; e < S.nnz; ++e) {
      key[e] = (int64_t)S.prow[e] * S.n + S.pcol[e];
      ord[e] = (int32_t)e;
    }
    std::sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) { return key[a] < key[b]; });
    auto find = [&](int64_t k) -> int32_t {
      auto it = std::lower_bound(ord.begin(), ord.end(), k, [&](int32_t a, int64_t v) { return key[a] < v; });
      return (it != ord.end() && key[*it] == k) ? *it : -1;
    };
    std::vector<std::vector<I4>> rows(S.n);
    for (int32_t e : ord) {   // row-major, columns ascending
      const int32_t i = S.prow[e], j = S.pcol[e];
      rows[i].push_back({j, e, find((int64_t)j * S.n + i), 0});
    }
    for (int32_t e : ord) {   // (i, j) whose mirror (j, i) is not in the pattern: column-only entry of row j
      const int32_t i = S.prow[e], j = S.pcol[e];
      if (find((int64_t)j * S.n + i) < 0) rows[j].push_back({i, -1, e, 0});
    }
    for (int t = 0; t < S.n; ++t) {
      const int i = S.iperm[t];
      std::sort(rows[i].begin(), rows[i].end(), [](const I4& a, const I4& b) { return a.x < b.x; });
      P.uent.push_back({-1, -1, -1, i});
      for (const I4& v : rows[i]) P.uent.push_back({v.x, v.y, v.z, i});
    }
    P.n_uent = (int)P.uent.size();
    for (int pad = 0; pad < 4; ++pad) P.uent.push_back({-1, -1, -1, -1});   // a step reads 4 entries at once
  }
  return 0;
}

void reach_lists(const std::vector<int32_t>& front_of_col, const std::vector<int32_t>& front_parent,
                 const std::vector<int32_t>& level_ptr, const std::vector<int32_t>& level_fronts,
                 const std::vector<int32_t>& prows, std::vector<int32_t>& mark, std::vector<int32_t>& list,
                 std::vector<int32_t>& ptr) {
  mark.assign(front_parent.size(), 0);
  for (int32_t p : prows)
    for (int t = front_of_col[p]; t >= 0 && !mark[t]; t = front_parent[t]) mark[t] = 1;
  const int L = (int)level_ptr.size() - 1;
  list.clear();
  ptr.assign(1, 0);
  for (int l = 0; l < L; ++l) {
    for (int e = level_ptr[l]; e < level_ptr[l + 1]; ++e)
      if (mark[level_fronts[e]]) list.push_back(level_fronts[e]);
    ptr.push_back((int32_t)list.size());
  }
}

std::string check_plan(const Symbolic& S, const Plan& P, int64_t Fc, int split_target) {
  char buf[256];
  auto bad = [&](const char* what, int64_t at, int64_t v, int64_t lim) {
    snprintf(buf, sizeof buf, "%s: entry %lld = %lld outside [0, %lld)", what, (long long)at, (long long)v, (long long)lim);
    return std::string(buf);
  };
  const int64_t FE = S.factor_entries, NNZ = S.nnz;
  const int nfr = (int)S.fronts.size(), L = P.L;
  auto id_ok = [&](int64_t v) { return v >= -1 && v < FE; };   // element id or -1
  auto nz_ok = [&](int64_t v) { return v >= -1 && v < NNZ; };
  if (Fc <= 0 || Fc % 64) return "chunk not a multiple of 64";
  // fronts: storage, work vectors, pivot columns, index staging
  for (int t = 0; t < nfr; ++t) {
    const Front& F = S.fronts[t];
    if (F.off < 0 || F.off + (int64_t)F.f * F.f > FE) return bad("front storage", t, F.off, FE);
    if (F.row0 < 0 || F.row0 + (int64_t)F.f > S.total_rows) return bad("front rows", t, F.row0, S.total_rows);
    if (F.col0 < 0 || F.col0 + F.ns > S.n) return bad("front pivots", t, F.col0, S.n);
    if (F.f > MAX_FRONT || F.ns < 1 || F.ns > F.f) return bad("front size", t, F.f, MAX_FRONT + 1);
    if (F.parent >= nfr || F.level < 0 || F.level >= L) return bad("front parent / level", t, F.parent, nfr);
  }
  for (int64_t r = 0; r < S.total_rows; ++r)
    if (S.idx[r] < 0 || S.idx[r] >= S.n) return bad("front row index", r, S.idx[r], S.n);
  // A11 assembly: records in chunks of 8 per launch (grid covers asm_ptr[l + 1] - asm_ptr[l] records)
  if (P.asm_rec.size() % 8 || P.asm_xp.size() != P.asm_rec.size() / 8 + 1) return "assembly chunks";
  for (size_t x = 0; x < P.asm_rec.size(); ++x) {
    const I4& a = P.asm_rec[x];
    if (!id_ok(a.x) || !nz_ok(a.y) || !id_ok(a.z)) return bad("assembly record", x, a.x, FE);
  }
  for (size_t c = 0; c + 1 < P.asm_xp.size(); ++c)
    if (P.asm_xp[c] > P.asm_xp[c + 1] || P.asm_xp[c + 1] > (int64_t)P.asm_x.size()) return bad("assembly overflow", c, P.asm_xp[c], P.asm_x.size());
  for (size_t x = 0; x < P.asm_x.size(); ++x)
    if (P.asm_x[x].x < 0 || P.asm_x[x].x >= 8 || P.asm_x[x].y < 0 || P.asm_x[x].y >= FE) return bad("assembly extra", x, P.asm_x[x].y, FE);
  for (int l = 0; l <= L; ++l)
    if (P.asm_ptr[l] % 8) return bad("assembly level padding", l, P.asm_ptr[l], 8);
  // L21 items: each item's OFF_G OFF_RPL rows x ns records inside orec, rows inside the front
  if (P.oxp.size() != P.items.size() + 1) return "item overflow ranges";
  for (size_t i = 0; i < P.items.size(); ++i) {
    const I4& it = P.items[i];
    if (it.x < 0 || it.x >= nfr) return bad("item front", i, it.x, nfr);
    const Front& F = S.fronts[it.x];
    if (it.y < F.ns || it.y >= F.f) return bad("item row", i, it.y, F.f);
    if (it.w < 0 || it.w + (int64_t)OFF_G * OFF_RPL * F.ns > (int64_t)P.orec.size()) return bad("item records", i, it.w, P.orec.size());
    if (P.oxp[i] > P.oxp[i + 1] || P.oxp[i + 1] > (int64_t)P.ox.size()) return bad("item overflow", i, P.oxp[i], P.ox.size());
    for (int x = P.oxp[i]; x < P.oxp[i + 1]; ++x)
      if (P.ox[x].x < 0 || P.ox[x].x >= OFF_G * OFF_RPL * F.ns || P.ox[x].y < 0 || P.ox[x].y >= FE)
        return bad("item extra", x, P.ox[x].y, FE);
  }
  for (size_t x = 0; x < P.orec.size(); ++x)
    if (!nz_ok(P.orec[x].x) || !id_ok(P.orec[x].y)) return bad("item record", x, P.orec[x].y, FE);
  // Schur tiles / blocks: origins inside the update block, first-source ids and overflow ranges
  if (P.g1.size() != P.tiles.size() * SCHUR_TILE || P.gxp.size() != P.tiles.size() + 1) return "tile sources";
  if (P.bg1.size() != P.blocks.size() * SCHUR_BLK_IDS || P.bgxp.size() != P.blocks.size() + 1) return "block sources";
  for (size_t i = 0; i < P.tiles.size(); ++i) {
    const I4& tt = P.tiles[i];
    if (tt.x < 0 || tt.x >= nfr) return bad("tile front", i, tt.x, nfr);
    const int r = S.fronts[tt.x].f - S.fronts[tt.x].ns;
    if (tt.y < 0 || tt.y >= r || tt.z < 0 || tt.z >= r) return bad("tile origin", i, tt.y, r);
    if (P.gxp[i] > P.gxp[i + 1] || P.gxp[i + 1] > (int64_t)P.gx.size()) return bad("tile overflow", i, P.gxp[i], P.gx.size());
  }
  for (size_t i = 0; i < P.blocks.size(); ++i) {
    const I4& bk = P.blocks[i];
    if (bk.x < 0 || bk.x >= nfr) return bad("block front", i, bk.x, nfr);
    const int r = S.fronts[bk.x].f - S.fronts[bk.x].ns;
    if (bk.y < 0 || bk.y >= r || bk.z < 0 || bk.z > bk.y + SCHUR_BLK) return bad("block origin", i, bk.y, r);
    if (P.bgxp[i] > P.bgxp[i + 1] || P.bgxp[i + 1] > (int64_t)P.bgx.size()) return bad("block overflow", i, P.bgxp[i], P.bgx.size());
  }
  for (size_t x = 0; x < P.g1.size(); ++x)
    if (!id_ok(P.g1[x])) return bad("tile source", x, P.g1[x], FE);
  for (size_t x = 0; x < P.bg1.size(); ++x)
    if (!id_ok(P.bg1[x])) return bad("block source", x, P.bg1[x], FE);
  for (size_t x = 0; x < P.gx.size(); ++x)
    if (P.gx[x].x < 0 || P.gx[x].x >= SCHUR_TILE || P.gx[x].y < 0 || P.gx[x].y >= FE) return bad("tile extra", x, P.gx[x].y, FE);
  for (size_t x = 0; x < P.bgx.size(); ++x)
    if (P.bgx[x].x < 0 || P.bgx[x].x >= SCHUR_BLK_IDS || P.bgx[x].y < 0 || P.bgx[x].y >= FE) return bad("block extra", x, P.bgx[x].y, FE);
  // the fused bottom level: every level-0 front listed once, <= 2-pivot fronts first, records of its panel
  if (P.fused0) {
    const int n0 = (int)P.f0_front.size();
    if ((int)P.f0_ptr.size() != n0 + 1 || P.f0_ptr[0] != 0 || P.f0_ptr[n0] != (int)P.f0_nz.size() ||
        n0 != S.level_ptr[1] - S.level_ptr[0] || P.f0_small < 0 || P.f0_small > n0)
      return "fused level 0 lists";
    for (int i = 0; i < n0; ++i) {
      const int t = P.f0_front[i];
      if (t < 0 || t >= (int)S.fronts.size()) return bad("fused level 0 front", i, t, (int64_t)S.fronts.size());
      const Front& F = S.fronts[t];
      const int r = F.f - F.ns;
      if (F.level != 0 || F.ns > F0_NS || r > F0_RM || (F.ns <= 2) != (i < P.f0_small) ||
          P.f0_ptr[i + 1] - P.f0_ptr[i] != F.ns * (F.ns + 1) / 2 + r * F.ns)
        return bad("fused level 0 front", i, F.ns, r);
    }
    for (size_t x = 0; x < P.f0_nz.size(); ++x)
      if (P.f0_nz[x] < -1 || P.f0_nz[x] >= S.nnz) return bad("fused level 0 nz", x, P.f0_nz[x], S.nnz);
  }
  // per-level ranges monotone and complete
  if ((int)P.tile_ptr.size() != L + 1 || (int)P.blk_ptr.size() != L + 1 || (int)P.item_ptr.size() != L + 1 ||
      (int)P.asm_ptr.size() != L + 1)
    return "level ranges";
  for (int l = 0; l < L; ++l)
    if (P.tile_ptr[l] > P.tile_ptr[l + 1] || P.blk_ptr[l] > P.blk_ptr[l + 1] || P.item_ptr[l] > P.item_ptr[l + 1] ||
        P.asm_ptr[l] > P.asm_ptr[l + 1])
      return bad("level range order", l, P.tile_ptr[l], P.tile_ptr[l + 1]);
  // A11 in LDS (k_factor_sym_lds) on the levels whose pivot blocks reach at most 64
  for (int l = 0; l < L; ++l)
    if (P.level_maxns[l] <= 64 && fac_lds_bytes(P.level_maxns[l]) > LDS_BYTES) return bad("A11 LDS", l, P.level_maxns[l], 64);
  // Dirichlet lists
  const Workspace W = workspace(S, Fc, P.n_crow);
  for (size_t d = 0; d < P.dir.size(); ++d)
    if (P.dir[d].x < 0 || P.dir[d].x >= S.n || !nz_ok(P.dir[d].y)) return bad("Dirichlet node", d, P.dir[d].x, S.n);
  for (size_t c = 0; c < P.crow.size(); ++c)
    if (P.crow[c] < 0 || P.crow[c] >= S.n) return bad("coupled row", c, P.crow[c], S.n);
  for (size_t x = 0; x < P.ce.size(); ++x)
    if (P.ce[x].x < 0 || P.ce[x].x >= P.n_dir || !nz_ok(P.ce[x].y)) return bad("coupling entry", x, P.ce[x].x, P.n_dir);
  for (size_t x = 0; x < P.de.size(); ++x)
    if (P.de[x].x < 0 || P.de[x].x >= S.n || !nz_ok(P.de[x].y)) return bad("Dirichlet column entry", x, P.de[x].x, S.n);
  for (int p = 0; p < S.n; ++p)   // k_dirichlet_rhs writes Bc[cslot * Fc + q]
    if (P.cslot[p] >= P.n_crow || (int64_t)(P.cslot[p] + 1) * Fc > W.Bc) return bad("coupled-row slot", p, P.cslot[p], P.n_crow);
  // compressed rows / columns
  for (int64_t e = 0; e < S.nnz; ++e)
    if (P.ridx[e] < 0 || P.ridx[e] >= S.n || P.cidx[e] < 0 || P.cidx[e] >= S.n || P.rnz[e] >= NNZ || P.cnz[e] >= NNZ)
      return bad("compressed index", e, P.ridx[e], S.n);
  // contraction entries: rows / columns inside n, nz inside nnz, 4 padding entries for the 4-entry steps
  if ((int64_t)P.uent.size() != P.n_uent + 4) return "contraction padding";
  for (int e = 0; e < P.n_uent; ++e) {
    const I4& u = P.uent[e];
    if (u.w < 0 || u.w >= S.n || u.x < -1 || u.x >= S.n || !nz_ok(u.y) || !nz_ok(u.z)) return bad("contraction entry", e, u.x, S.n);
  }
  // per-workgroup partial buffers against the grids that write them
  if ((int64_t)residual_parts(S.n) * Fc > W.cpart) return "k_residual partials";                  // cpart[bx Fc + q]
  if ((int64_t)residual_parts(S.n) * 18 * Fc > W.kpart) return "k_residual contraction partials"; // kpart[(bx 18 + k) Fc + q]
  {
    const int64_t partial = (int64_t)std::max<int64_t>(contract_eg_parts(P.n_uent), Fc / 64) * 18;   // api.cpp's size
    if ((int64_t)contract_eg_parts(P.n_uent) * 18 > partial || (Fc / 64) * 18 > partial) return "gradient partials";
  }
  // split solve update parts: the rows every (part, wave) walks cover the update rows (L solve) / pivot rows (U
  // solve) exactly once for every split the launches use
  for (int l = 0; l < L; ++l) {
    const int64_t nf = S.level_ptr[l + 1] - S.level_ptr[l];
    const int split = solve_split(nf, Fc, split_target);
    if (split < 1 || split > 16) return bad("solve split", l, split, 17);
    constexpr int SRB = 4, SR = 2;   // rows per step: k_lsolve_rows (SRB), k_usolve2_upd (SR)
    for (int e = S.level_ptr[l]; e < S.level_ptr[l + 1]; ++e) {
      const Front& F = S.fronts[S.level_fronts[e]];
      std::vector<int> seen(F.f, 0);
      for (int part = 0; part < split; ++part)
        for (int w = 0; w < SPLIT_W; ++w) {
          for (int i0 = F.ns + SRB * (part * SPLIT_W + w); i0 < F.f; i0 += SRB * SPLIT_W * split)
            for (int r = 0; r < SRB && i0 + r < F.f; ++r) ++seen[i0 + r];
          for (int a0 = SR * (part * SPLIT_W + w); a0 < F.ns; a0 += SR * SPLIT_W * split)
            for (int r = 0; r < SR && a0 + r < F.ns; ++r) ++seen[a0 + r];
        }
      for (int a = 0; a < F.f; ++a)
        if (seen[a] != 1) return bad("split coverage", a, seen[a], 2);
    }
  }
  return "";
}

}  // namespace pfr
