// mof_dd_plan.cpp -- host side of the domain-decomposed solve (SURVEY.md §8(e),
// config C5): vertex partition by recursive coordinate bisection and the halo
// plan of every part.
//
// A part owns a set of vertices and both unknowns of each (rows i and i+N of
// the reference's planar system, compute_optical_flow.py:83-84). Its local
// mesh is every triangle with at least one owned corner, kept in the caller's
// triangle order, so the assembled rows of its owned vertices are the
// reference's rows bit for bit (every triangle that touches an owned vertex is
// local). The other corners of those triangles are its ghosts: read-only
// copies of the neighbours' unknowns, refreshed by the halo exchange before
// every operator application.
//
// Local row order: owned vertices first (by global RCM position: the band of
// the global ordering survives inside the part), then ghosts grouped by owner
// part (ascending) and by RCM position inside a group. The send list of q to
// p enumerates p's ghosts owned by q in exactly that order, so a received
// segment lands contiguously in p's ghost rows.
#include <algorithm>
#include <numeric>

#include "mof_dd.h"

namespace mof {

namespace {

// split `ids` (by axis of largest extent, median at the size ratio) until
// each piece is one part; parts [p0, p0 + np)
void rcb(const double *xyz, std::vector<int32_t> &ids, size_t lo, size_t hi, int32_t p0, int32_t np,
         int32_t *part) {
    if (np == 1) {
        for (size_t k = lo; k < hi; ++k) part[ids[k]] = p0;
        return;
    }
    double mn[3] = {1e300, 1e300, 1e300}, mx[3] = {-1e300, -1e300, -1e300};
    for (size_t k = lo; k < hi; ++k)
        for (int d = 0; d < 3; ++d) {
            mn[d] = std::min(mn[d], xyz[3 * (size_t)ids[k] + d]);
            mx[d] = std::max(mx[d], xyz[3 * (size_t)ids[k] + d]);
        }
    int ax = 0;
    for (int d = 1; d < 3; ++d)
        if (mx[d] - mn[d] > mx[ax] - mn[ax]) ax = d;
    const int32_t nl = np / 2;
    // sizes proportional to the part counts: every part gets floor or ceil(n/np)
    const size_t n = hi - lo;
    const size_t cut = lo + (size_t)((n * (size_t)nl) / (size_t)np);
    auto less = [&](int32_t a, int32_t b) {
        const double xa = xyz[3 * (size_t)a + ax], xb = xyz[3 * (size_t)b + ax];
        return xa != xb ? xa < xb : a < b;  // total order: deterministic
    };
    std::nth_element(ids.begin() + lo, ids.begin() + cut, ids.begin() + hi, less);
    rcb(xyz, ids, lo, cut, p0, nl, part);
    rcb(xyz, ids, cut, hi, p0 + nl, np - nl, part);
}

}  // namespace

void partition_rcb(const double *xyz, int32_t N, int32_t P, int32_t *part) {
    MOF_REQUIRE(N > 0 && P >= 1 && P <= N, "need 1 <= nparts <= N");
    std::vector<int32_t> ids(N);
    std::iota(ids.begin(), ids.end(), 0);
    rcb(xyz, ids, 0, (size_t)N, 0, P, part);
}

void build_dd_plan(const int32_t *tri, int32_t N, int32_t M, int32_t P, const int32_t *part,
                   const int32_t *rank_key, DdPlan &plan) {
    MOF_REQUIRE(P >= 1 && N > 0 && M > 0, "bad plan arguments");
    plan.P = P;
    plan.N = N;
    plan.M = M;
    plan.part.assign(part, part + N);
    for (int32_t i = 0; i < N; ++i) MOF_REQUIRE(part[i] >= 0 && part[i] < P, "part id out of range");
    plan.parts.assign(P, DdPart{});
    plan.g2l.assign(N, -1);
    auto key = [&](int32_t v) { return rank_key ? rank_key[v] : v; };
    // owned rows
    for (int32_t v = 0; v < N; ++v) plan.parts[part[v]].l2g.push_back(v);
    for (int32_t p = 0; p < P; ++p) {
        DdPart &D = plan.parts[p];
        MOF_REQUIRE(!D.l2g.empty(), "a part owns no vertex");
        std::sort(D.l2g.begin(), D.l2g.end(), [&](int32_t a, int32_t b) { return key(a) < key(b); });
        D.n_own = (int32_t)D.l2g.size();
        for (int32_t r = 0; r < D.n_own; ++r) plan.g2l[D.l2g[r]] = r;
    }
    // local triangles (caller order) and ghost candidates
    std::vector<std::vector<int32_t>> ghosts(P);
    for (int32_t T = 0; T < M; ++T) {
        const int32_t *t = tri + 3 * (size_t)T;
        int32_t ps[3] = {part[t[0]], part[t[1]], part[t[2]]};
        for (int c = 0; c < 3; ++c) {
            bool dup = false;
            for (int q = 0; q < c; ++q) dup |= ps[q] == ps[c];
            if (dup) continue;
            DdPart &D = plan.parts[ps[c]];
            D.tris.push_back(T);
            for (int k = 0; k < 3; ++k)
                if (part[t[k]] != ps[c]) ghosts[ps[c]].push_back(t[k]);
        }
    }
    for (int32_t p = 0; p < P; ++p) {
        DdPart &D = plan.parts[p];
        std::vector<int32_t> &g = ghosts[p];
        std::sort(g.begin(), g.end());
        g.erase(std::unique(g.begin(), g.end()), g.end());
        std::sort(g.begin(), g.end(), [&](int32_t a, int32_t b) {
            return part[a] != part[b] ? part[a] < part[b] : key(a) < key(b);
        });
        D.n_ghost = (int32_t)g.size();
        D.recv_off.assign(1, 0);
        D.ghost_src.resize(g.size());
        for (size_t k = 0; k < g.size(); ++k) {
            const int32_t q = part[g[k]];
            if (D.nbr.empty() || D.nbr.back() != q) {
                if (!D.nbr.empty()) D.recv_off.push_back((int32_t)k);
                D.nbr.push_back(q);
            }
            D.l2g.push_back(g[k]);
            D.ghost_src[k] = plan.g2l[g[k]];
        }
        if (!D.nbr.empty()) D.recv_off.push_back((int32_t)g.size());
    }
    // send lists: q sends to p the rows p's ghost range for q names
    for (int32_t p = 0; p < P; ++p) plan.parts[p].send_off.assign(1, 0);
    for (int32_t q = 0; q < P; ++q) {
        DdPart &S = plan.parts[q];
        for (int32_t p : S.nbr) {  // neighbour relation is symmetric (shared triangle)
            const DdPart &R = plan.parts[p];
            const auto it = std::lower_bound(R.nbr.begin(), R.nbr.end(), q);
            MOF_REQUIRE(it != R.nbr.end() && *it == q, "asymmetric halo (internal error)");
            const size_t k = (size_t)(it - R.nbr.begin());
            for (int32_t r = R.recv_off[k]; r < R.recv_off[k + 1]; ++r)
                S.send_idx.push_back(plan.g2l[R.l2g[R.n_own + r]]);
            S.send_off.push_back((int32_t)S.send_idx.size());
        }
    }
}

}  // namespace mof
