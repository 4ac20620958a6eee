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
// order (optional): the nodes in visit order (the aggregates then do not
// depend on the node numbering, only on this order)
int32_t aggregate(const std::vector<int32_t> &vptr, const std::vector<int32_t> &vcol, int32_t n,
                  std::vector<int32_t> &agg, const int32_t *order = nullptr) {
    agg.assign(n, -1);
    int32_t na = 0;
    for (int32_t oi = 0; oi < n; ++oi) {
        const int32_t i = order ? order[oi] : oi;
        bool free_nb = true;
        for (int32_t q = vptr[i]; q < vptr[i + 1] && free_nb; ++q) free_nb = agg[vcol[q]] < 0;
        if (!free_nb) continue;
        for (int32_t q = vptr[i]; q < vptr[i + 1]; ++q) agg[vcol[q]] = na;
        ++na;
    }
    std::vector<int32_t> cnt;
    for (int32_t oi = 0; oi < n; ++oi) {
        const int32_t i = order ? order[oi] : oi;
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

// P = (I - w D^-1 a2) Q at level 0 (bs = 2): row i gets its own tentative
// block and -w D_i^-1 a2_ij Q_j for every neighbour j (itself included), in
// the row's block order, merged per aggregate; rows sorted by aggregate.
void smooth_prolongator(const Pattern &fine, const AmgParams &prm, const std::vector<int32_t> &agg,
                        const std::vector<float> &Q, std::vector<int32_t> &pptr, std::vector<int32_t> &pcol,
                        std::vector<float> &P) {
    const int32_t n = fine.N;
    std::vector<double> ab(4 * fine.vcol.size(), 0.0);  // a2 per adjacency block
    for (size_t pos = 0; pos < fine.sell_blk.size(); ++pos)
        if (fine.sell_blk[pos] >= 0)
            for (int k = 0; k < 4; ++k) ab[4 * (size_t)fine.sell_blk[pos] + k] = prm.a2[4 * pos + k];
    const double w = prm.smooth_omega;
    pptr.assign(n + 1, 0);
    pcol.clear();
    P.clear();
    std::vector<int32_t> rk;
    std::vector<double> rv;
    for (int32_t i = 0; i < n; ++i) {
        rk.clear();
        rv.clear();
        auto add = [&](int32_t K, const double (&t)[6]) {
            size_t e = 0;
            while (e < rk.size() && rk[e] != K) ++e;
            if (e == rk.size()) {
                rk.push_back(K);
                rv.insert(rv.end(), 6, 0.0);
            }
            for (int c = 0; c < 6; ++c) rv[6 * e + c] += t[c];
        };
        double own[6];
        for (int c = 0; c < 6; ++c) own[c] = Q[6 * (size_t)i + c];
        add(agg[i], own);
        int32_t qd = -1;
        for (int32_t q = fine.vptr[i]; q < fine.vptr[i + 1]; ++q)
            if (fine.vcol[q] == i) qd = q;
        const double *d = qd >= 0 ? &ab[4 * (size_t)qd] : nullptr;
        const double det = d ? d[0] * d[3] - d[1] * d[2] : 0.0;
        if (d && det != 0.0 && std::isfinite(det)) {
            const double di[4] = {d[3] / det, -d[1] / det, -d[2] / det, d[0] / det};
            for (int32_t q = fine.vptr[i]; q < fine.vptr[i + 1]; ++q) {
                const int32_t j = fine.vcol[q];
                const double *a = &ab[4 * (size_t)q];
                const double m[4] = {di[0] * a[0] + di[1] * a[2], di[0] * a[1] + di[1] * a[3],
                                     di[2] * a[0] + di[3] * a[2], di[2] * a[1] + di[3] * a[3]};
                double t[6];
                for (int r = 0; r < 2; ++r)
                    for (int c = 0; c < 3; ++c)
                        t[3 * r + c] = -w * (m[2 * r] * Q[6 * (size_t)j + c] + m[2 * r + 1] * Q[6 * (size_t)j + 3 + c]);
                add(agg[j], t);
            }
        }
        std::vector<size_t> ord(rk.size());
        for (size_t e = 0; e < ord.size(); ++e) ord[e] = e;
        std::sort(ord.begin(), ord.end(), [&](size_t x, size_t y) { return rk[x] < rk[y]; });
        for (size_t e : ord) {
            pcol.push_back(rk[e]);
            for (int c = 0; c < 6; ++c) P.push_back((float)rv[6 * e + c]);
        }
        pptr[i + 1] = (int32_t)pcol.size();
    }
}

// P = (I - w D^-1 a) Q at a coarse level (bs = 3; a: 9 doubles per adjacency
// block of F, row-major): as smooth_prolongator, with a dof of F that has no
// prolongator column (dead) given a unit diagonal in D.
void smooth_prolongator3(const AmgLevel &F, const std::vector<double> &a, double w, const std::vector<int32_t> &agg,
                         const std::vector<float> &Q, std::vector<int32_t> &pptr, std::vector<int32_t> &pcol,
                         std::vector<float> &P) {
    const int32_t n = F.n;
    pptr.assign(n + 1, 0);
    pcol.clear();
    P.clear();
    std::vector<int32_t> rk;
    std::vector<double> rv;
    for (int32_t i = 0; i < n; ++i) {
        rk.clear();
        rv.clear();
        auto add = [&](int32_t K, const double (&t)[9]) {
            size_t e = 0;
            while (e < rk.size() && rk[e] != K) ++e;
            if (e == rk.size()) {
                rk.push_back(K);
                rv.insert(rv.end(), 9, 0.0);
            }
            for (int c = 0; c < 9; ++c) rv[9 * e + c] += t[c];
        };
        double own[9];
        for (int c = 0; c < 9; ++c) own[c] = Q[9 * (size_t)i + c];
        add(agg[i], own);
        int32_t qd = -1;
        for (int32_t q = F.vptr[i]; q < F.vptr[i + 1]; ++q)
            if (F.vcol[q] == i) qd = q;
        double d[9];
        bool ok = qd >= 0;
        if (ok) {
            for (int k = 0; k < 9; ++k) d[k] = a[9 * (size_t)qd + k];
            for (int c = 0; c < 3; ++c)
                if (!F.dead.empty() && F.dead[3 * (size_t)i + c]) d[4 * c] += 1.0;
        }
        double di[9];
        if (ok) {  // 3x3 inverse by cofactors
            const double c00 = d[4] * d[8] - d[5] * d[7], c01 = d[5] * d[6] - d[3] * d[8], c02 = d[3] * d[7] - d[4] * d[6];
            const double det = d[0] * c00 + d[1] * c01 + d[2] * c02;
            ok = det != 0.0 && std::isfinite(det);
            if (ok) {
                const double id = 1.0 / det;
                di[0] = c00 * id;
                di[1] = (d[2] * d[7] - d[1] * d[8]) * id;
                di[2] = (d[1] * d[5] - d[2] * d[4]) * id;
                di[3] = c01 * id;
                di[4] = (d[0] * d[8] - d[2] * d[6]) * id;
                di[5] = (d[2] * d[3] - d[0] * d[5]) * id;
                di[6] = c02 * id;
                di[7] = (d[1] * d[6] - d[0] * d[7]) * id;
                di[8] = (d[0] * d[4] - d[1] * d[3]) * id;
            }
        }
        if (ok) {
            for (int32_t q = F.vptr[i]; q < F.vptr[i + 1]; ++q) {
                const int32_t j = F.vcol[q];
                const double *aq = &a[9 * (size_t)q];
                double m[9];  // D^-1 a_ij
                for (int r = 0; r < 3; ++r)
                    for (int c = 0; c < 3; ++c)
                        m[3 * r + c] = di[3 * r] * aq[c] + di[3 * r + 1] * aq[3 + c] + di[3 * r + 2] * aq[6 + c];
                double t[9];
                for (int r = 0; r < 3; ++r)
                    for (int c = 0; c < 3; ++c)
                        t[3 * r + c] = -w * (m[3 * r] * Q[9 * (size_t)j + c] + m[3 * r + 1] * Q[9 * (size_t)j + 3 + c] +
                                             m[3 * r + 2] * Q[9 * (size_t)j + 6 + c]);
                add(agg[j], t);
            }
        }
        std::vector<size_t> ord(rk.size());
        for (size_t e = 0; e < ord.size(); ++e) ord[e] = e;
        std::sort(ord.begin(), ord.end(), [&](size_t x, size_t y) { return rk[x] < rk[y]; });
        for (size_t e : ord) {
            pcol.push_back(rk[e]);
            for (int c = 0; c < 9; ++c) P.push_back((float)rv[9 * e + c]);
        }
        pptr[i + 1] = (int32_t)pcol.size();
    }
}

// The Galerkin image C = P^T a P of a fine operator given per adjacency block
// (bs x bs doubles, fine vptr / vcol order) on the coarse pattern
// (C.vptr / vcol), 9 doubles per coarse adjacency block, fp64.
std::vector<double> galerkin_image(const AmgLevel &F, int bs, const std::vector<double> &a, const AmgLevel &C) {
    std::vector<double> out(9 * C.vcol.size(), 0.0);
    for (int32_t i = 0; i < F.n; ++i)
        for (int32_t q = F.vptr[i]; q < F.vptr[i + 1]; ++q) {
            const int32_t j = F.vcol[q];
            const double *aq = &a[(size_t)bs * bs * q];
            for (int32_t ka = F.pptr[i]; ka < F.pptr[i + 1]; ++ka) {
                const int32_t I = F.pcol[ka];
                const float *pi = &F.Q[(size_t)bs * 3 * ka];
                for (int32_t kb = F.pptr[j]; kb < F.pptr[j + 1]; ++kb) {
                    const float *pj = &F.Q[(size_t)bs * 3 * kb];
                    const int32_t p = (int32_t)(std::lower_bound(C.vcol.begin() + C.vptr[I], C.vcol.begin() + C.vptr[I + 1],
                                                                 F.pcol[kb]) -
                                                C.vcol.begin());
                    double T[4][3];  // a_ij P_j (bs x 3)
                    for (int r = 0; r < bs; ++r)
                        for (int c = 0; c < 3; ++c) {
                            double s = 0.0;
                            for (int k = 0; k < bs; ++k) s += aq[bs * r + k] * (double)pj[3 * k + c];
                            T[r][c] = s;
                        }
                    for (int r = 0; r < 3; ++r)
                        for (int c = 0; c < 3; ++c) {
                            double s = 0.0;
                            for (int k = 0; k < bs; ++k) s += (double)pi[3 * k + r] * T[k][c];
                            out[9 * (size_t)p + 3 * r + c] += s;
                        }
                }
            }
        }
    return out;
}

}  // namespace

bool amg_auto_smooth(const Pattern &fine) {
    // vertex valence = adjacency row length minus the diagonal
    const int32_t n = fine.N;
    if (n <= 0) return false;
    double s = 0.0, s2 = 0.0;
    for (int32_t i = 0; i < n; ++i) {
        const double v = fine.vptr[i + 1] - fine.vptr[i] - 1;
        s += v;
        s2 += v * v;
    }
    const double mean = s / n, var = std::max(0.0, s2 / n - mean * mean);
    return std::sqrt(var) > 0.5;
}

// sigma_3 / sigma_1 of a 3-column block from its QR factor R (3x3, upper
// triangular, row-major): the eigenvalues of R^T R by cyclic Jacobi
static double sv_ratio(const double R[9]) {
    double a[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0.0;
            for (int k = 0; k < 3; ++k) s += R[3 * k + i] * R[3 * k + j];
            a[i][j] = s;
        }
    for (int sweep = 0; sweep < 12; ++sweep) {
        double off = std::fabs(a[0][1]) + std::fabs(a[0][2]) + std::fabs(a[1][2]);
        if (off <= 1e-300) break;
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                if (std::fabs(a[p][q]) <= 1e-300) continue;
                const double th = 0.5 * (a[q][q] - a[p][p]) / a[p][q];
                const double t = (th >= 0 ? 1.0 : -1.0) / (std::fabs(th) + std::sqrt(th * th + 1.0));
                const double c = 1.0 / std::sqrt(t * t + 1.0), sn = t * c;
                for (int k = 0; k < 3; ++k) {  // columns p, q
                    const double kp = a[k][p], kq = a[k][q];
                    a[k][p] = c * kp - sn * kq;
                    a[k][q] = sn * kp + c * kq;
                }
                for (int k = 0; k < 3; ++k) {  // rows p, q
                    const double pk = a[p][k], qk = a[q][k];
                    a[p][k] = c * pk - sn * qk;
                    a[q][k] = sn * pk + c * qk;
                }
            }
    }
    const double l0 = std::max(0.0, a[0][0]), l1 = std::max(0.0, a[1][1]), l2 = std::max(0.0, a[2][2]);
    const double mx = std::max({l0, l1, l2}), mn = std::min({l0, l1, l2});
    return mx > 0.0 ? std::sqrt(mn / mx) : 0.0;
}

void build_amg(const Pattern &fine, const double *e_internal, const AmgParams &prm,
               AmgHierarchy &H) {
    H.levels.clear();
    H.curl.clear();
    H.max_curl = 0.0;
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
        const int32_t nc = aggregate(F.vptr, F.vcol, F.n, agg, H.levels.size() == 1 ? prm.order : nullptr);
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
        std::vector<double> Bm, Qm, ratio(nc);
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
            ratio[I] = sv_ratio(R);
        }
        std::nth_element(ratio.begin(), ratio.begin() + nc / 2, ratio.end());
        H.curl.push_back(ratio[nc / 2]);
        if (nc >= 64) H.max_curl = std::max(H.max_curl, ratio[nc / 2]);
        // member-order copy (restriction reads members contiguously)
        F.Qm.assign(F.Q.size(), 0.f);
        for (int32_t q = 0; q < F.n; ++q)
            std::copy_n(F.Q.begin() + (size_t)F.mlist[q] * bs * 3, bs * 3, F.Qm.begin() + (size_t)q * bs * 3);
        // prolongator rows: the tentative Q (one block per node), or smoothed
        const bool smooth = H.levels.size() == 1 && prm.nown < 0 && prm.a2 &&
                            (prm.smooth > 0 || (prm.smooth < 0 && amg_auto_smooth(fine)));
        // coarse levels: level 1 (smooth1 = 1), or every level above the fused
        // tiny ones (smooth1 = 2), each from its own image of a2
        const bool smooth1 = (H.levels.size() == 2 || (H.levels.size() > 2 && prm.smooth1 > 1)) && prm.smooth1 > 0 &&
                             !F.a2img.empty() && F.n > kSubNodes;
        if (smooth || smooth1) {
            std::vector<float> P;
            if (smooth)
                smooth_prolongator(fine, prm, agg, F.Q, F.pptr, F.pcol, P);
            else
                smooth_prolongator3(F, F.a2img, prm.smooth_omega, agg, F.Q, F.pptr, F.pcol, P);
            F.Q.swap(P);  // P blocks, indexed by the gather lists and the prolongation
            F.smoothed = true;
            for (int32_t i = 0; i < F.n; ++i) F.apos[i] = i;  // restriction gathers by node
        } else {
            F.pptr.resize(F.n + 1);
            for (int32_t i = 0; i <= F.n; ++i) F.pptr[i] = i;
            F.pcol = agg;
        }
        // restriction lists: coarse node -> {fine node, P block}, fine node order
        F.rptr.assign(nc + 1, 0);
        for (int32_t k = 0; k < F.pptr[F.n]; ++k) F.rptr[F.pcol[k] + 1]++;
        for (int32_t I = 0; I < nc; ++I) F.rptr[I + 1] += F.rptr[I];
        F.rent.assign(2 * (size_t)F.pptr[F.n], 0);
        {
            std::vector<int32_t> fill(F.rptr.begin(), F.rptr.end() - 1);
            for (int32_t i = 0; i < F.n; ++i)
                for (int32_t k = F.pptr[i]; k < F.pptr[i + 1]; ++k) {
                    const int32_t e = fill[F.pcol[k]]++;
                    F.rent[2 * (size_t)e] = i;
                    F.rent[2 * (size_t)e + 1] = k;
                }
        }
        // coarse pattern: (K, L) for every fine block (i, j), K of a P block of
        // row i and L of one of row j
        AmgLevel C;
        C.n = nc;
        C.bs = 3;
        C.dead = dead;
        {
            std::vector<std::vector<int32_t>> rows(nc);
            for (int32_t i = 0; i < F.n; ++i)
                for (int32_t q = F.vptr[i]; q < F.vptr[i + 1]; ++q) {
                    const int32_t j = F.vcol[q];
                    for (int32_t ka = F.pptr[i]; ka < F.pptr[i + 1]; ++ka)
                        for (int32_t kb = F.pptr[j]; kb < F.pptr[j + 1]; ++kb) rows[F.pcol[ka]].push_back(F.pcol[kb]);
                }
            C.vptr.assign(nc + 1, 0);
            for (int32_t I = 0; I < nc; ++I) {
                auto &r = rows[I];
                std::sort(r.begin(), r.end());
                r.erase(std::unique(r.begin(), r.end()), r.end());
                C.vcol.insert(C.vcol.end(), r.begin(), r.end());
                C.vptr[I + 1] = (int32_t)C.vcol.size();
                std::vector<int32_t>().swap(r);
            }
        }
        sell_layout(C);
        // level 1's image of the mesh's a2 (its smoothing, smooth1)
        if (H.levels.size() == 1 && prm.nown < 0 && prm.a2 && prm.smooth1 > 0 && C.n > kSubNodes) {
            std::vector<double> ab(4 * fine.vcol.size(), 0.0);  // a2 per adjacency block
            for (size_t pos = 0; pos < fine.sell_blk.size(); ++pos)
                if (fine.sell_blk[pos] >= 0)
                    for (int k = 0; k < 4; ++k) ab[4 * (size_t)fine.sell_blk[pos] + k] = prm.a2[4 * pos + k];
            C.a2img = galerkin_image(F, 2, ab, C);
        } else if (H.levels.size() >= 2 && prm.smooth1 > 1 && !F.a2img.empty() && C.n > kSubNodes) {
            C.a2img = galerkin_image(F, 3, F.a2img, C);
        }
        // Galerkin gather lists: coarse block -> terms P_iK^T A_ij P_jL, in fine
        // block order (then P block order)
        const int32_t cnb = (int32_t)C.vcol.size();
        std::vector<int32_t> term_cb;
        std::vector<int32_t> cnt(cnb + 1, 0);
        for (int32_t i = 0; i < F.n; ++i)
            for (int32_t q = F.vptr[i]; q < F.vptr[i + 1]; ++q) {
                const int32_t j = F.vcol[q];
                for (int32_t ka = F.pptr[i]; ka < F.pptr[i + 1]; ++ka) {
                    const int32_t I = F.pcol[ka];
                    for (int32_t kb = F.pptr[j]; kb < F.pptr[j + 1]; ++kb) {
                        const int32_t p = (int32_t)(std::lower_bound(C.vcol.begin() + C.vptr[I],
                                                                     C.vcol.begin() + C.vptr[I + 1], F.pcol[kb]) -
                                                    C.vcol.begin());
                        term_cb.push_back(p);
                        cnt[p + 1]++;
                    }
                }
            }
        for (int32_t p = 0; p < cnb; ++p) cnt[p + 1] += cnt[p];
        // gather ranges indexed by coarse SELL position
        std::vector<int32_t> fine_pos(F.vcol.size());
        for (int64_t pos = 0; pos < (int64_t)F.sell_blk.size(); ++pos)
            if (F.sell_blk[pos] >= 0) fine_pos[F.sell_blk[pos]] = (int32_t)pos;
        F.gptr.assign(C.sell_blk.size() + 1, 0);
        std::vector<int32_t> by_block((size_t)cnt.back() * 3);
        {
            std::vector<int32_t> fill(cnt.begin(), cnt.end() - 1);
            size_t t = 0;
            for (int32_t i = 0; i < F.n; ++i)
                for (int32_t q = F.vptr[i]; q < F.vptr[i + 1]; ++q) {
                    const int32_t j = F.vcol[q];
                    // a decomposed part's ghost couplings (tentative P only)
                    const bool ghost = H.levels.size() == 1 && prm.nown >= 0 && (i >= prm.nown || j >= prm.nown);
                    for (int32_t ka = F.pptr[i]; ka < F.pptr[i + 1]; ++ka)
                        for (int32_t kb = F.pptr[j]; kb < F.pptr[j + 1]; ++kb) {
                            const size_t k = (size_t)fill[term_cb[t++]]++;
                            by_block[3 * k + 0] = ghost ? (j == i ? -1 : -2)
                                                  : H.levels.size() == 1 && prm.mirror ? prm.mirror[fine_pos[q]]
                                                                                       : fine_pos[q];
                            by_block[3 * k + 1] = ka;
                            by_block[3 * k + 2] = kb;
                        }
                }
        }
        // the coarse operator is symmetric: only its diagonal and upper blocks
        // get terms; each lower block is its upper twin transposed (C.low /
        // C.twin, written by st_pair) -- half the product's terms, and the twins
        // equal to the bit (round 6)
        std::vector<int32_t> cpos(C.vcol.size(), -1);  // adjacency index -> SELL position
        for (int64_t pos = 0; pos < (int64_t)C.sell_blk.size(); ++pos)
            if (C.sell_blk[pos] >= 0) cpos[C.sell_blk[pos]] = (int32_t)pos;
        C.low.clear();
        C.twin.clear();
        F.gent.clear();
        F.gent.reserve(by_block.size() / 2 + 3 * (size_t)C.n);
        for (int64_t pos = 0; pos < (int64_t)C.sell_blk.size(); ++pos) {
            const int32_t p = C.sell_blk[pos];
            if (p >= 0) {
                const int32_t I = C.sell_row[pos], J = C.sell_col[pos];
                if (J < I) {
                    const int32_t q = (int32_t)(std::lower_bound(C.vcol.begin() + C.vptr[J],
                                                                 C.vcol.begin() + C.vptr[J + 1], I) -
                                                C.vcol.begin());
                    C.low.push_back((int32_t)pos);
                    C.twin.push_back(cpos[q]);
                } else {
                    F.gent.insert(F.gent.end(), by_block.begin() + 3 * (size_t)cnt[p],
                                  by_block.begin() + 3 * (size_t)cnt[p + 1]);
                }
            }
            F.gptr[pos + 1] = (int32_t)(F.gent.size() / 3);
        }
        B.swap(Bc);
        H.levels.push_back(std::move(C));
    }
    AmgLevel &Lc = H.levels.back();
    H.coarse_dofs = Lc.n * Lc.bs;
}

}  // namespace mof
