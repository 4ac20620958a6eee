// mof_pattern.cpp -- one-time host build of the block sparsity pattern.
//
// The reference discovers the pattern implicitly: it scatters every
// per-triangle term into a scipy lil_matrix (compute_optical_flow.py:78-93,
// 127-141). Here the pattern is built once per mesh so that every
// per-timestep assembly is a deterministic gather (no atomics):
//  * vptr/vcol   vertex adjacency (self included, sorted): the 2x2 blocks;
//  * cptr/clist  for each block (i, j) the (triangle, local i, local j)
//                terms that land on it, in triangle order -- the order in
//                which the reference's lil "+=" folds them;
//  * sell_off/sell_col  SELL-64 layout of the blocks for the SpMV;
//  * tsell_off/tinc      SELL-64 vertex -> incident-triangle lists, for the
//                        per-triangle (matrix-free) application of a1.
#include <algorithm>
#include <chrono>

#include "mof_internal.h"

namespace mof {

void build_pattern(const int32_t *tri, int32_t N, int32_t M, Pattern &pat, const int32_t *torder) {
    MOF_REQUIRE(N > 0 && M > 0, "mesh needs N > 0 vertices and M > 0 triangles");
    MOF_REQUIRE((int64_t)M * 9 < (int64_t)INT32_MAX, "too many triangles for int32 term codes");
    for (int64_t q = 0; q < 3 * (int64_t)M; ++q)
        MOF_REQUIRE(tri[q] >= 0 && tri[q] < N, "triangle vertex index out of range");
    pat.N = N;
    pat.M = M;

    // incidence counts -> candidate neighbour lists (3 per incident corner)
    std::vector<int64_t> inc(N + 1, 0);
    for (int64_t q = 0; q < 3 * (int64_t)M; ++q) inc[tri[q] + 1]++;
    for (int32_t i = 0; i < N; ++i) inc[i + 1] += inc[i];
    std::vector<int32_t> cand(3 * inc[N] + N);
    std::vector<int64_t> cfill(N);
    std::vector<int64_t> cbase(N + 1);
    for (int32_t i = 0; i <= N; ++i) cbase[i] = 3 * inc[i] + i;
    for (int32_t i = 0; i < N; ++i) {
        cfill[i] = cbase[i];
        cand[cfill[i]++] = i;  // every vertex keeps its diagonal block
    }
    for (int32_t T = 0; T < M; ++T) {
        const int32_t *v = tri + 3 * (int64_t)T;
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
                if (a == b) continue;
                cand[cfill[v[a]]++] = v[b];
            }
    }
    pat.vptr.assign(N + 1, 0);
    pat.vcol.clear();
    pat.vcol.reserve(7 * (size_t)N);
    for (int32_t i = 0; i < N; ++i) {
        auto b = cand.begin() + cbase[i], e = cand.begin() + cfill[i];
        std::sort(b, e);
        e = std::unique(b, e);
        pat.vcol.insert(pat.vcol.end(), b, e);
        pat.vptr[i + 1] = (int32_t)pat.vcol.size();
    }
    const int32_t nb = (int32_t)pat.vcol.size();

    // contribution lists: term (T, a, b) -> block (v_a, v_b); T ascending
    auto block_of = [&](int32_t i, int32_t j) -> int32_t {
        auto b = pat.vcol.begin() + pat.vptr[i], e = pat.vcol.begin() + pat.vptr[i + 1];
        return (int32_t)(std::lower_bound(b, e, j) - pat.vcol.begin());
    };
    pat.cptr.assign(nb + 1, 0);
    std::vector<int32_t> term_block(9 * (size_t)M);
    for (int32_t q = 0; q < M; ++q) {
        const int32_t T = torder ? torder[q] : q;  // caller's triangle order
        const int32_t *v = tri + 3 * (int64_t)T;
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
                int32_t p = block_of(v[a], v[b]);
                term_block[9 * (size_t)T + 3 * a + b] = p;
                pat.cptr[p + 1]++;
            }
    }
    for (int32_t p = 0; p < nb; ++p) pat.cptr[p + 1] += pat.cptr[p];
    pat.clist.assign(pat.cptr[nb], 0);
    std::vector<int32_t> fill(pat.cptr.begin(), pat.cptr.end() - 1);
    for (int32_t q = 0; q < M; ++q) {
        const int32_t T = torder ? torder[q] : q;  // caller's triangle order
        for (int c = 0; c < 9; ++c) {
            int32_t p = term_block[9 * (size_t)T + c];
            pat.clist[fill[p]++] = 9 * T + c;
        }
    }

    // SELL-64
    pat.nslices = (N + kSlice - 1) / kSlice;
    pat.sell_off.assign(pat.nslices + 1, 0);
    for (int32_t s = 0; s < pat.nslices; ++s) {
        int32_t w = 0;
        for (int32_t i = s * kSlice; i < std::min(N, (s + 1) * kSlice); ++i)
            w = std::max(w, pat.vptr[i + 1] - pat.vptr[i]);
        pat.sell_off[s + 1] = pat.sell_off[s] + w * kSlice;
    }
    pat.sell_col.assign(pat.sell_off[pat.nslices], 0);
    pat.sell_blk.assign(pat.sell_off[pat.nslices], -1);
    pat.blk_row.assign(nb, 0);
    for (int32_t i = 0; i < N; ++i)
        for (int32_t q = pat.vptr[i]; q < pat.vptr[i + 1]; ++q) pat.blk_row[q] = i;
    for (int32_t s = 0; s < pat.nslices; ++s) {
        int32_t w = (pat.sell_off[s + 1] - pat.sell_off[s]) / kSlice;
        for (int32_t l = 0; l < kSlice; ++l) {
            int32_t i = s * kSlice + l;
            int32_t td = 0;  // the diagonal's index in the row (vcol order)
            if (i < N)
                td = (int32_t)(std::lower_bound(pat.vcol.begin() + pat.vptr[i], pat.vcol.begin() + pat.vptr[i + 1], i) -
                               (pat.vcol.begin() + pat.vptr[i]));
            for (int32_t t = 0; t < w; ++t) {  // slot t: diagonal first (sell_slot)
                int32_t c = 0;
                const int64_t pos = pat.sell_off[s] + (int64_t)t * kSlice + l;
                if (i < N) {
                    int32_t deg = pat.vptr[i + 1] - pat.vptr[i];
                    const int32_t tb = sell_block(t, td);
                    c = t < deg ? pat.vcol[pat.vptr[i] + tb] : i;
                    if (t < deg) pat.sell_blk[pos] = pat.vptr[i] + tb;
                }
                pat.sell_col[pos] = c;
            }
        }
    }
    pat.diag_pos.assign(N, 0);
    for (int32_t i = 0; i < N; ++i) pat.diag_pos[i] = pat.sell_off[i / kSlice] + (i % kSlice);  // slot 0

    // vertex -> incident (triangle, corner) in triangle order, SELL-64
    std::vector<int32_t> tdeg(N, 0);
    for (int64_t q = 0; q < 3 * (int64_t)M; ++q) tdeg[tri[q]]++;
    pat.tsell_off.assign(pat.nslices + 1, 0);
    for (int32_t s = 0; s < pat.nslices; ++s) {
        int32_t w = 0;
        for (int32_t i = s * kSlice; i < std::min(N, (s + 1) * kSlice); ++i) w = std::max(w, tdeg[i]);
        pat.tsell_off[s + 1] = pat.tsell_off[s] + w * kSlice;
    }
    const int64_t tnb = pat.tsell_off[pat.nslices];
    pat.tinc.assign(4 * (size_t)tnb, 0);
    for (int32_t s = 0; s < pat.nslices; ++s) {
        const int32_t w = (pat.tsell_off[s + 1] - pat.tsell_off[s]) / kSlice;
        for (int32_t l = 0; l < kSlice; ++l) {
            const int32_t i = std::min(s * kSlice + l, N - 1);
            for (int32_t t = 0; t < w; ++t) {  // padding: zero triangle slot M
                int32_t *q = &pat.tinc[4 * ((int64_t)pat.tsell_off[s] + (int64_t)t * kSlice + l)];
                q[0] = M; q[1] = 0; q[2] = i; q[3] = i;
            }
        }
    }
    std::vector<int32_t> tfill(N, 0);
    pat.tslot.assign((size_t)tnb, 0);
    // SELL slot of block (i, j) in row i (diagonal first, sell_slot)
    auto slot_of = [&](int32_t i, int32_t j) {
        const auto b = pat.vcol.begin() + pat.vptr[i], e = pat.vcol.begin() + pat.vptr[i + 1];
        const int32_t t = (int32_t)(std::lower_bound(b, e, j) - b), td = (int32_t)(std::lower_bound(b, e, i) - b);
        return sell_slot(t, td);
    };
    for (int32_t q = 0; q < M; ++q) {
        const int32_t T = torder ? torder[q] : q;  // caller's triangle order
        const int32_t *v = tri + 3 * (int64_t)T;
        for (int a = 0; a < 3; ++a) {
            const int32_t i = v[a];
            const int32_t t = tfill[i]++;
            const int64_t e = (int64_t)pat.tsell_off[i / kSlice] + (int64_t)t * kSlice + (i % kSlice);
            int32_t *ent = &pat.tinc[4 * e];
            ent[0] = T; ent[1] = a; ent[2] = v[(a + 1) % 3]; ent[3] = v[(a + 2) % 3];
            pat.tslot[e] = slot_of(i, ent[2]) | (slot_of(i, ent[3]) << 8);
        }
    }
    pat.max_w = 0;
    for (int32_t s = 0; s < pat.nslices; ++s) pat.max_w = std::max(pat.max_w, (pat.sell_off[s + 1] - pat.sell_off[s]) / kSlice);
}

// Mirror table of the SELL-64 layout (per position, shared by all systems):
// the fp32 / bf16 operators are symmetric (A(j,i) = A(i,j)^T up to the
// rounding of the fold), so row i reads a block (i, j) of the lower triangle
// (j < i) as the transpose of block (j, i), which row j reads anyway: only
// the diagonal and upper blocks ever leave HBM. Entry: the position to read
// (| kMirT if transposed), or -1 for padding (read as the row's diagonal,
// masked: padding lines never leave HBM either). Rows >= nown (ghost rows of
// a part) and blocks coupling to them read their own position.
// The mirrored reads of a wave are coalesced only as far as neighbouring rows
// have their neighbours in the same slots (regular meshes): `sym` = 1 uses
// them, 0 keeps every block at its own position (identity table), -1 decides
// per mesh from the 128-B lines a wave instruction touches (fp32 blocks):
// symmetric reads when own + mirrored lines stay within 2x the lines of the
// plain layout. Round 4, forced either way on one box (profiles/r04_ab/sym/):
// C3 1.08x; the S1-like patch 1.43x: +9 % (906 -> 988 timesteps/s, same
// iterations); S1s 1.53x: +0.8 %; R3 in plain RCM order 2.81x: -6 %
// (648 -> 610), window-sorted R3 3.37x: -11 % (round 3). The bound was 1.25x.
std::vector<int32_t> sell_mirror(const Pattern &pat, int32_t nown, int sym, bool *used) {
    const int64_t snb = pat.sell_off[pat.nslices];
    MOF_REQUIRE(snb < kMirT, "SELL layout too large for the mirror table");
    std::vector<int32_t> mir((size_t)snb, -1);
    auto slot_of = [&](int32_t i, int32_t j) {
        const auto b = pat.vcol.begin() + pat.vptr[i], e = pat.vcol.begin() + pat.vptr[i + 1];
        const int32_t t = (int32_t)(std::lower_bound(b, e, j) - b), td = (int32_t)(std::lower_bound(b, e, i) - b);
        return sell_slot(t, td);
    };
    for (int32_t s = 0; s < pat.nslices; ++s) {
        const int32_t w = (pat.sell_off[s + 1] - pat.sell_off[s]) / kSlice;
        for (int32_t l = 0; l < kSlice; ++l) {
            const int32_t i = s * kSlice + l;
            if (i >= pat.N) break;
            for (int32_t t = 0; t < w; ++t) {
                const int64_t pos = pat.sell_off[s] + (int64_t)t * kSlice + l;
                if (pat.sell_blk[pos] < 0) continue;  // padding
                const int32_t j = pat.sell_col[pos];
                if (sym != 0 && j < i && i < nown)
                    mir[pos] = (int32_t)(pat.sell_off[j / kSlice] + (int64_t)slot_of(j, i) * kSlice + j % kSlice) | kMirT;
                else
                    mir[pos] = (int32_t)pos;
            }
        }
    }
    if (sym < 0) {  // lines (128 B = 8 fp32 blocks) per wave instruction, summed
        int64_t plain = 0, mirrored = 0;
        std::vector<int64_t> ln;
        for (int32_t s = 0; s < pat.nslices; ++s) {
            const int32_t w = (pat.sell_off[s + 1] - pat.sell_off[s]) / kSlice;
            for (int32_t t = 0; t < w; ++t) {
                const int64_t base = pat.sell_off[s] + (int64_t)t * kSlice;
                ln.clear();
                int64_t last = -1;
                for (int32_t l = 0; l < kSlice; ++l) {
                    const int32_t v = mir[base + l];
                    if (v < 0) continue;
                    if (((base + l) >> 3) != last) ++plain, last = (base + l) >> 3;
                    ln.push_back((int64_t)(v & kMirPos) >> 3);
                }
                std::sort(ln.begin(), ln.end());
                mirrored += std::unique(ln.begin(), ln.end()) - ln.begin();
            }
        }
        sym = mirrored <= 2 * plain ? 1 : 0;
        if (!sym)
            for (int64_t q = 0; q < snb; ++q)
                if (mir[q] >= 0) mir[q] = (int32_t)q;
    }
    if (used) *used = sym != 0;
    return mir;
}

// Reverse Cuthill-McKee order of the vertex graph in `pat` (adjacency
// only). Returns perm with perm[old] = new. BFS from a pseudo-peripheral
// vertex of every connected component, neighbours in increasing degree,
// then reversed: rows that share columns end up close together, which keeps
// the SpMV's z gathers inside the L2 of the XCD that owns the row chunk.
std::vector<int32_t> rcm_order(const Pattern &pat) {
    const int32_t N = pat.N;
    std::vector<int32_t> deg(N), order, perm(N, -1);
    order.reserve(N);
    for (int32_t i = 0; i < N; ++i) deg[i] = pat.vptr[i + 1] - pat.vptr[i];
    std::vector<int32_t> level(N, -1), queue;
    queue.reserve(N);
    // farthest vertex of a BFS from s (ties: smallest degree); marks nothing
    auto far = [&](int32_t s) {
        std::vector<int32_t> seen_list{s};
        level[s] = 0;
        size_t h = 0;
        int32_t last = s;
        while (h < seen_list.size()) {
            const int32_t v = seen_list[h++];
            if (level[v] > level[last] || (level[v] == level[last] && deg[v] < deg[last])) last = v;
            for (int32_t q = pat.vptr[v]; q < pat.vptr[v + 1]; ++q) {
                const int32_t w = pat.vcol[q];
                if (level[w] < 0) {
                    level[w] = level[v] + 1;
                    seen_list.push_back(w);
                }
            }
        }
        for (int32_t v : seen_list) level[v] = -1;
        return last;
    };
    std::vector<char> done(N, 0);
    std::vector<int32_t> nb;
    for (int32_t s0 = 0; s0 < N; ++s0) {
        if (done[s0]) continue;
        int32_t s = far(far(s0));
        size_t h = order.size();
        order.push_back(s);
        done[s] = 1;
        while (h < order.size()) {
            const int32_t v = order[h++];
            nb.clear();
            for (int32_t q = pat.vptr[v]; q < pat.vptr[v + 1]; ++q)
                if (!done[pat.vcol[q]]) nb.push_back(pat.vcol[q]);
            std::sort(nb.begin(), nb.end(), [&](int32_t a, int32_t b) {
                return deg[a] != deg[b] ? deg[a] < deg[b] : a < b;
            });
            for (int32_t w : nb) {
                done[w] = 1;
                order.push_back(w);
            }
        }
    }
    std::reverse(order.begin(), order.end());
    for (int32_t k = 0; k < N; ++k) perm[order[k]] = k;
    return perm;
}

}  // namespace mof
