// mof_amg_host.cpp -- one-time host build of the aggregation multigrid hierarchy.
//
// Preconditioner for the inner PCG (MOF_PRECOND_AMG): unsmoothed-aggregation
// AMG on the 2x2-block operator A = a1 + lambda a2. Everything that depends
// only on the mesh is built here once; the per-timestep coarse operators are
// Galerkin products computed on the GPU (mof_amg.hip).
//
//  * aggregation: greedy, deterministic (root + its free neighbours, then the
//    leftovers join their most frequent neighbouring aggregate);
//  * near-null space: at the fine level the three ambient directions seen in
//    each vertex's tangent frame, B_i = [e_i^0; e_i^1] (2 x 3) -- rigid
//    in-plane translations of the surface; per aggregate a QR of the stacked
//    B gives the tentative prolongator Q (orthonormal columns) and R, the
//    coarse near-null space (3 x 3 per aggregate);
//  * columns that vanish in the QR (flat aggregates) are dropped and their
//    coarse dof is marked dead (identity on the coarse diagonal);
//  * every level's block pattern is stored SELL-64 like the fine level, and
//    each coarse block keeps the list of fine blocks whose Galerkin terms
//    Q_i^T A_ij Q_j fold into it (deterministic gather, no atomics).
#include <algorithm>
#include <cmath>

#include "mof_amg.h"

namespace mof {
namespace {

// greedy aggregation of a graph given as sorted adjacency with self loops
int32_t aggregate(const std::vector<int32_t> &vptr, const std::vector<int32_t> &vcol, int32_t n,
                  std::vector<int32_t> &agg) {
    agg.assign(n, -1);
    int32_t na = 0;
    for (int32_t i = 0; i < n; ++i) {
        bool free_nb = true;
        for (int32_t q = vptr[i]; q < vptr[i + 1] && free_nb; ++q) free_nb = agg[vcol[q]] < 0;
        if (!free_nb) continue;
        for (int32_t q = vptr[i]; q < vptr[i + 1]; ++q) agg[vcol[q]] = na;
        ++na;
    }
    std::vector<int32_t> cnt;
    for (int32_t i = 0; i < n; ++i) {
        if (agg[i] >= 0) continue;
        // most frequent aggregate among the neighbours (smallest id on ties)
        int32_t best = -1, best_c = 0;
        for (int32_t q = vptr[i]; q < vptr[i + 1]; ++q) {
            const int32_t a = agg[vcol[q]];
            if (a < 0) continue;
            int32_t c = 0;
            for (int32_t r = vptr[i]; r < vptr[i + 1]; ++r) c += agg[vcol[r]] == a;
            if (c > best_c || (c == best_c && a < best)) {
                best = a;
                best_c = c;
            }
        }
        agg[i] = best >= 0 ? best : na++;
    }
    return na;
}

// QR of a (m x 3) row-major matrix by modified Gram-Schmidt with one
// re-orthogonalisation; columns whose remaining norm is below tol * max
// column norm are dropped (zero column in Q, zero row in R).
void qr3(const std::vector<double> &Bm, int32_t m, std::vector<double> &Q, double R[9],
         bool dead[3]) {
    Q = Bm;
    for (int k = 0; k < 9; ++k) R[k] = 0.0;
    double cmax = 0.0;
    for (int c = 0; c < 3; ++c) {
        double s = 0.0;
        for (int32_t r = 0; r < m; ++r) s += Bm[3 * r + c] * Bm[3 * r + c];
        cmax = std::max(cmax, std::sqrt(s));
    }
    for (int c = 0; c < 3; ++c) {
        for (int pass = 0; pass < 2; ++pass)
            for (int p = 0; p < c; ++p) {
                if (dead[p]) continue;
                double d = 0.0;
                for (int32_t r = 0; r < m; ++r) d += Q[3 * r + p] * Q[3 * r + c];
                R[3 * p + c] += d;
                for (int32_t r = 0; r < m; ++r) Q[3 * r + c] -= d * Q[3 * r + p];
            }
        double s = 0.0;
        for (int32_t r = 0; r < m; ++r) s += Q[3 * r + c] * Q[3 * r + c];
        s = std::sqrt(s);
        dead[c] = !(s > 1e-6 * cmax) || m < c + 1;
        if (dead[c]) {
            for (int32_t r = 0; r < m; ++r) Q[3 * r + c] = 0.0;
            for (int p = 0; p < 3; ++p) R[3 * p + c] = 0.0;
            R[3 * c + c] = 0.0;
            continue;
        }
        R[3 * c + c] = s;
        for (int32_t r = 0; r < m; ++r) Q[3 * r + c] /= s;
    }
}

void sell_layout(AmgLevel &L) {
    const int32_t n = L.n;
    const int32_t ns = (n + kSlice - 1) / kSlice;
    L.sell_off.assign(ns + 1, 0);
    for (int32_t s = 0; s < ns; ++s) {
        int32_t w = 0;
        for (int32_t i = s * kSlice; i < std::min(n, (s + 1) * kSlice); ++i)
            w = std::max(w, L.vptr[i + 1] - L.vptr[i]);
        L.sell_off[s + 1] = L.sell_off[s] + w * kSlice;
    }
    L.sell_col.assign(L.sell_off[ns], 0);
    L.sell_blk.assign(L.sell_off[ns], -1);
    L.diag_pos.assign(n, 0);
    L.sell_row.assign(L.sell_off[ns], 0);
    for (int32_t s = 0; s < ns; ++s) {
        const int32_t w = (L.sell_off[s + 1] - L.sell_off[s]) / kSlice;
        for (int32_t l = 0; l < kSlice; ++l) {
            const int32_t i = s * kSlice + l;
            int32_t td = 0;  // diagonal first in every row (sell_slot)
            if (i < n)
                while (td < L.vptr[i + 1] - L.vptr[i] - 1 && L.vcol[L.vptr[i] + td] != i) ++td;
            for (int32_t t = 0; t < w; ++t) {
                const int64_t pos = L.sell_off[s] + (int64_t)t * kSlice + l;
                int32_t c = std::min(i, n - 1);
                if (i < n) {
                    const int32_t deg = L.vptr[i + 1] - L.vptr[i];
                    if (t < deg) {
                        const int32_t tb = sell_block(t, td);
                        c = L.vcol[L.vptr[i] + tb];
                        L.sell_blk[pos] = L.vptr[i] + tb;
                        if (c == i) L.diag_pos[i] = (int32_t)pos;
                    } else {
                        c = i;
                    }
                }
                L.sell_col[pos] = c;
                L.sell_row[pos] = i;
            }
        }
    }
}

}  // namespace

void build_amg(const Pattern &fine, const double *e_internal, const AmgParams &prm,
               AmgHierarchy &H) {
    H.levels.clear();
    // level 0: the fine pattern (SELL already built by build_pattern)
    {
        AmgLevel L0;
        L0.n = fine.N;
        L0.bs = 2;
        L0.vptr = fine.vptr;
        L0.vcol = fine.vcol;
        L0.sell_off = fine.sell_off;
        L0.sell_col = fine.sell_col;
        L0.sell_blk = fine.sell_blk;
        L0.diag_pos = fine.diag_pos;
        H.levels.push_back(std::move(L0));
    }
    // near-null space of level 0: B_i = e_i (2 x 3), double
    std::vector<double> B(6 * (size_t)fine.N);
    for (size_t q = 0; q < B.size(); ++q) B[q] = e_internal[q];
    while ((int32_t)H.levels.size() < prm.max_levels) {
        AmgLevel &F = H.levels.back();
        if (F.n * 3 <= prm.max_coarse_dofs) break;
        const int32_t bs = F.bs;
        std::vector<int32_t> agg;
        const int32_t nc = aggregate(F.vptr, F.vcol, F.n, agg);
        if (nc >= F.n) break;  // no coarsening possible
        F.agg = agg;
        // members CSR
        F.mptr.assign(nc + 1, 0);
        for (int32_t i = 0; i < F.n; ++i) F.mptr[agg[i] + 1]++;
        for (int32_t I = 0; I < nc; ++I) F.mptr[I + 1] += F.mptr[I];
        F.mlist.assign(F.n, 0);
        {
            std::vector<int32_t> fill(F.mptr.begin(), F.mptr.end() - 1);
            for (int32_t i = 0; i < F.n; ++i) F.mlist[fill[agg[i]]++] = i;
        }
        F.apos.assign(F.n, 0);
        for (int32_t q = 0; q < F.n; ++q) F.apos[F.mlist[q]] = q;
        // tentative prolongator per aggregate
        F.Q.assign((size_t)F.n * bs * 3, 0.f);
        std::vector<double> Bc(9 * (size_t)nc, 0.0);
        std::vector<uint8_t> dead(3 * (size_t)nc, 0);
        std::vector<double> Bm, Qm;
        for (int32_t I = 0; I < nc; ++I) {
            const int32_t m = F.mptr[I + 1] - F.mptr[I];
            Bm.assign(3 * (size_t)m * bs, 0.0);
            for (int32_t a = 0; a < m; ++a) {
                const int32_t i = F.mlist[F.mptr[I] + a];
                for (int r = 0; r < bs; ++r)
                    for (int c = 0; c < 3; ++c) Bm[3 * ((size_t)a * bs + r) + c] = B[(size_t)i * bs * 3 + 3 * r + c];
            }
            double R[9];
            bool dd[3] = {false, false, false};
            qr3(Bm, m * bs, Qm, R, dd);
            for (int32_t a = 0; a < m; ++a) {
                const int32_t i = F.mlist[F.mptr[I] + a];
                for (int r = 0; r < bs; ++r)
                    for (int c = 0; c < 3; ++c)
                        F.Q[(size_t)i * bs * 3 + 3 * r + c] = (float)Qm[3 * ((size_t)a * bs + r) + c];
            }
            for (int k = 0; k < 9; ++k) Bc[9 * (size_t)I + k] = R[k];
            for (int c = 0; c < 3; ++c) dead[3 * (size_t)I + c] = dd[c];
        }
        // member-order copy (restriction reads members contiguously)
        F.Qm.assign(F.Q.size(), 0.f);
        for (int32_t q = 0; q < F.n; ++q)
            std::copy_n(F.Q.begin() + (size_t)F.mlist[q] * bs * 3, bs * 3, F.Qm.begin() + (size_t)q * bs * 3);
        // coarse pattern: (agg(i), agg(j)) of every fine block, sorted
        AmgLevel C;
        C.n = nc;
        C.bs = 3;
        C.dead = dead;
        {
            std::vector<std::vector<int32_t>> rows(nc);
            for (int32_t i = 0; i < F.n; ++i)
                for (int32_t q = F.vptr[i]; q < F.vptr[i + 1]; ++q) rows[agg[i]].push_back(agg[F.vcol[q]]);
            C.vptr.assign(nc + 1, 0);
            for (int32_t I = 0; I < nc; ++I) {
                auto &r = rows[I];
                std::sort(r.begin(), r.end());
                r.erase(std::unique(r.begin(), r.end()), r.end());
                C.vcol.insert(C.vcol.end(), r.begin(), r.end());
                C.vptr[I + 1] = (int32_t)C.vcol.size();
            }
        }
        sell_layout(C);
        // Galerkin gather lists: coarse block -> fine blocks (in fine block order)
        const int32_t cnb = (int32_t)C.vcol.size();
        std::vector<int32_t> cblk_of_fine(F.vcol.size());
        std::vector<int32_t> cnt(cnb + 1, 0);
        for (int32_t i = 0; i < F.n; ++i)
            for (int32_t q = F.vptr[i]; q < F.vptr[i + 1]; ++q) {
                const int32_t I = agg[i], J = agg[F.vcol[q]];
                const int32_t p = (int32_t)(std::lower_bound(C.vcol.begin() + C.vptr[I],
                                                             C.vcol.begin() + C.vptr[I + 1], J) -
                                            C.vcol.begin());
                cblk_of_fine[q] = p;
                cnt[p + 1]++;
            }
        for (int32_t p = 0; p < cnb; ++p) cnt[p + 1] += cnt[p];
        // gather ranges indexed by coarse SELL position
        std::vector<int32_t> fine_pos(F.vcol.size());
        for (int64_t pos = 0; pos < (int64_t)F.sell_blk.size(); ++pos)
            if (F.sell_blk[pos] >= 0) fine_pos[F.sell_blk[pos]] = (int32_t)pos;
        F.gptr.assign(C.sell_blk.size() + 1, 0);
        std::vector<int32_t> by_block(cnt.back() * 3);
        {
            std::vector<int32_t> fill(cnt.begin(), cnt.end() - 1);
            for (int32_t i = 0; i < F.n; ++i)
                for (int32_t q = F.vptr[i]; q < F.vptr[i + 1]; ++q) {
                    const int32_t p = cblk_of_fine[q];
                    const int32_t k = fill[p]++;
                    const bool ghost = H.levels.size() == 1 && prm.nown >= 0 &&
                                       (i >= prm.nown || F.vcol[q] >= prm.nown);
                    by_block[3 * k + 0] = ghost ? (F.vcol[q] == i ? -1 : -2) : fine_pos[q];
                    by_block[3 * k + 1] = i;
                    by_block[3 * k + 2] = F.vcol[q];
                }
        }
        F.gent.clear();
        F.gent.reserve(by_block.size());
        for (int64_t pos = 0; pos < (int64_t)C.sell_blk.size(); ++pos) {
            const int32_t p = C.sell_blk[pos];
            if (p >= 0)
                F.gent.insert(F.gent.end(), by_block.begin() + 3 * cnt[p], by_block.begin() + 3 * cnt[p + 1]);
            F.gptr[pos + 1] = (int32_t)(F.gent.size() / 3);
        }
        B.swap(Bc);
        H.levels.push_back(std::move(C));
    }
    AmgLevel &Lc = H.levels.back();
    H.coarse_dofs = Lc.n * Lc.bs;
}

}  // namespace mof
