// Micro-benchmark for DESIGN.md §9 item 6: the inner PCG's SpMV + vector
// update (k_pcg_spmv's FIRST = false path: q = A z + beta q, p = z + beta p,
// x += alpha p_old) with the operator in four forms, on one mesh, B systems:
//   mat   : materialised fp32 2x2 blocks per system, SELL-64, every slot
//   matm  : the same, lower blocks read as the transposed upper ones
//           through a mirror table (the product's symmetric reads)
//   tri_g : lambda a2 from one shared copy (SELL-64) + a1 per incident
//           triangle from g_T (3 floats per triangle per system, sqrt(A_T/12)
//           folded in) and the shared tangent bases E_v
//   tri_u : the same with u_{T,v} = E_v^T g_T stored (6 floats per triangle)
//   tri_g2: tri_g for two systems per thread (shared loads once for both)
// Not product code: test infrastructure for a design decision. Input: a
// binary mesh file written by tools/spmv_tri_proto.py (RCM vertex order,
// triangles by smallest vertex). Prints one JSON line per form.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

constexpr int kWG = 256, kSl = 64, kU = 8;
constexpr int32_t kMirT = 1 << 30, kMirPos = kMirT - 1;

struct Vec {
    const float2 *z;
    float2 *p, *q, *x;
    float al, be;
};

// workgroup -> (row block, system): XCD x = w % 8 runs row blocks x, x+8, ...,
// all B systems of one row block back to back, so a row block's shared data
// stays in that XCD's L2 while its systems pass
__device__ __forceinline__ bool task(int32_t nblk, int32_t B, int32_t &rb, int32_t &b) {
    const int32_t w = blockIdx.x, xcd = w & 7, k = w >> 3;
    rb = (k / B) * 8 + xcd;
    b = k % B;
    return rb < nblk;
}

__device__ __forceinline__ void epilogue(const Vec &v, int64_t vi, float y0, float y1) {
    const float2 zi = v.z[vi], p0 = v.p[vi], q0 = v.q[vi];
    float2 xi = v.x[vi];
    xi.x += v.al * p0.x;
    xi.y += v.al * p0.y;
    v.q[vi] = make_float2(y0 + v.be * q0.x, y1 + v.be * q0.y);
    v.p[vi] = make_float2(zi.x + v.be * p0.x, zi.y + v.be * p0.y);
    v.x[vi] = xi;
}

template <bool MIR>
__global__ __launch_bounds__(kWG) void k_mat(int32_t N, int32_t nblk, int32_t B, const int32_t *__restrict__ off,
                                            const int32_t *__restrict__ col, const int32_t *__restrict__ mir,
                                            const float4 *__restrict__ A, int64_t nb, Vec v) {
    int32_t rb, b;
    if (!task(nblk, B, rb, b)) return;
    const int32_t i = rb * kWG + threadIdx.x;
    if (i >= N) return;
    const int32_t s = i >> 6, l = i & 63, o = off[s], w = (off[s + 1] - o) >> 6;
    const float4 *Ab = A + (int64_t)b * nb;
    const float2 *zb = v.z + (int64_t)b * N;
    float a0 = 0.f, a1 = 0.f;
    for (int32_t t0 = 0; t0 < w; t0 += kU) {
        int32_t j[kU], m[kU];
        float4 k[kU];
        float2 xj[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int32_t t = min(t0 + u, w - 1);
            j[u] = col[o + t * kSl + l];
            if (MIR) m[u] = mir[o + t * kSl + l];
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int32_t t = min(t0 + u, w - 1);
            k[u] = MIR ? Ab[m[u] < 0 ? o + l : (m[u] & kMirPos)] : Ab[o + t * kSl + l];
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) xj[u] = zb[j[u]];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            bool on = t0 + u < w;
            float b1 = k[u].y, b2 = k[u].z;
            if (MIR) {
                on = on && m[u] >= 0;
                if (m[u] & kMirT) {
                    b1 = k[u].z;
                    b2 = k[u].y;
                }
            }
            a0 += on ? k[u].x * xj[u].x + b1 * xj[u].y : 0.f;
            a1 += on ? b2 * xj[u].x + k[u].w * xj[u].y : 0.f;
        }
    }
    epilogue(v, (int64_t)b * N + i, a0, a1);
}

// STORE_U: per-system u (6 floats per triangle) instead of g (3) and E
template <bool STORE_U>
__global__ __launch_bounds__(kWG) void k_tri(int32_t N, int32_t M, int32_t nblk, int32_t B,
                                            const int32_t *__restrict__ off, const int32_t *__restrict__ col,
                                            const float4 *__restrict__ a2, const int32_t *__restrict__ toff,
                                            const int4 *__restrict__ tinc, const float *__restrict__ E,
                                            const float *__restrict__ G, Vec v) {
    int32_t rb, b;
    if (!task(nblk, B, rb, b)) return;
    const int32_t i = rb * kWG + threadIdx.x;
    if (i >= N) return;
    const int32_t s = i >> 6, l = i & 63;
    const float2 *zb = v.z + (int64_t)b * N;
    float a0 = 0.f, a1 = 0.f;
    {
        const int32_t o = off[s], w = (off[s + 1] - o) >> 6;
        for (int32_t t0 = 0; t0 < w; t0 += kU) {
            int32_t j[kU];
            float4 k[kU];
            float2 xj[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) j[u] = col[o + min(t0 + u, w - 1) * kSl + l];
#pragma unroll
            for (int u = 0; u < kU; ++u) k[u] = a2[o + min(t0 + u, w - 1) * kSl + l];
#pragma unroll
            for (int u = 0; u < kU; ++u) xj[u] = zb[j[u]];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const bool on = t0 + u < w;
                a0 += on ? k[u].x * xj[u].x + k[u].y * xj[u].y : 0.f;
                a1 += on ? k[u].z * xj[u].x + k[u].w * xj[u].y : 0.f;
            }
        }
    }
    const float2 zi = zb[i];
    float ei[6];
    if (!STORE_U)
#pragma unroll
        for (int d = 0; d < 6; ++d) ei[d] = E[6 * (int64_t)i + d];
    const float *Gb = G + (int64_t)b * (M + 1) * (STORE_U ? 6 : 3);
    const int32_t o = toff[s], w = (toff[s + 1] - o) >> 6;
    constexpr int U = 4;
    for (int32_t t0 = 0; t0 < w; t0 += U) {
        int4 q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) q[u] = tinc[o + min(t0 + u, w - 1) * kSl + l];
        float2 ui[U], uj[U], uk[U], xj[U], xk[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            xj[u] = zb[q[u].z];
            xk[u] = zb[q[u].w];
            if (STORE_U) {
                const float2 *uT = reinterpret_cast<const float2 *>(Gb + 6 * (int64_t)q[u].x);
                const float2 P0 = uT[0], P1 = uT[1], P2 = uT[2];
                const int c = q[u].y;
                ui[u] = c == 0 ? P0 : (c == 1 ? P1 : P2);
                uj[u] = c == 0 ? P1 : (c == 1 ? P2 : P0);
                uk[u] = c == 0 ? P2 : (c == 1 ? P0 : P1);
            } else {
                const float *gT = Gb + 3 * (int64_t)q[u].x;
                const float g0 = gT[0], g1 = gT[1], g2 = gT[2];
                const float *ej = E + 6 * (int64_t)q[u].z, *ek = E + 6 * (int64_t)q[u].w;
                ui[u] = make_float2(ei[0] * g0 + ei[1] * g1 + ei[2] * g2, ei[3] * g0 + ei[4] * g1 + ei[5] * g2);
                uj[u] = make_float2(ej[0] * g0 + ej[1] * g1 + ej[2] * g2, ej[3] * g0 + ej[4] * g1 + ej[5] * g2);
                uk[u] = make_float2(ek[0] * g0 + ek[1] * g1 + ek[2] * g2, ek[3] * g0 + ek[4] * g1 + ek[5] * g2);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float si = ui[u].x * zi.x + ui[u].y * zi.y;
            const float sj = uj[u].x * xj[u].x + uj[u].y * xj[u].y;
            const float sk = uk[u].x * xk[u].x + uk[u].y * xk[u].y;
            const float cc = t0 + u < w ? (si + si) + sj + sk : 0.f;
            a0 += ui[u].x * cc;
            a1 += ui[u].y * cc;
        }
    }
    epilogue(v, (int64_t)b * N + i, a0, a1);
}

// tri_g2: the g form for two systems per thread, every shared load (SELL
// columns, a2 blocks, incidence entries, E) issued once for both
__global__ __launch_bounds__(kWG) void k_tri2(int32_t N, int32_t M, int32_t nblk, int32_t B,
                                             const int32_t *__restrict__ off, const int32_t *__restrict__ col,
                                             const float4 *__restrict__ a2, const int32_t *__restrict__ toff,
                                             const int4 *__restrict__ tinc, const float *__restrict__ E,
                                             const float *__restrict__ G, Vec v) {
    int32_t rb, bp;
    if (!task(nblk, B / 2, rb, bp)) return;
    const int32_t i = rb * kWG + threadIdx.x;
    if (i >= N) return;
    const int32_t s = i >> 6, l = i & 63;
    const float2 *zb[2] = {v.z + (int64_t)(2 * bp) * N, v.z + (int64_t)(2 * bp + 1) * N};
    const float *Gb[2] = {G + (int64_t)(2 * bp) * (M + 1) * 3, G + (int64_t)(2 * bp + 1) * (M + 1) * 3};
    float a0[2] = {0.f, 0.f}, a1[2] = {0.f, 0.f};
    {
        const int32_t o = off[s], w = (off[s + 1] - o) >> 6;
        constexpr int U = 4;
        for (int32_t t0 = 0; t0 < w; t0 += U) {
            int32_t j[U];
            float4 k[U];
            float2 xj[2][U];
#pragma unroll
            for (int u = 0; u < U; ++u) j[u] = col[o + min(t0 + u, w - 1) * kSl + l];
#pragma unroll
            for (int u = 0; u < U; ++u) k[u] = a2[o + min(t0 + u, w - 1) * kSl + l];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int t = 0; t < 2; ++t) xj[t][u] = zb[t][j[u]];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const bool on = t0 + u < w;
                    a0[t] += on ? k[u].x * xj[t][u].x + k[u].y * xj[t][u].y : 0.f;
                    a1[t] += on ? k[u].z * xj[t][u].x + k[u].w * xj[t][u].y : 0.f;
                }
        }
    }
    float2 zi[2] = {zb[0][i], zb[1][i]};
    float ei[6];
#pragma unroll
    for (int d = 0; d < 6; ++d) ei[d] = E[6 * (int64_t)i + d];
    const int32_t o = toff[s], w = (toff[s + 1] - o) >> 6;
    constexpr int U = 2;
    for (int32_t t0 = 0; t0 < w; t0 += U) {
        int4 q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) q[u] = tinc[o + min(t0 + u, w - 1) * kSl + l];
        float ej[U][6], ek[U][6], g[2][U][3];
        float2 xj[2][U], xk[2][U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int d = 0; d < 6; ++d) {
                ej[u][d] = E[6 * (int64_t)q[u].z + d];
                ek[u][d] = E[6 * (int64_t)q[u].w + d];
            }
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                xj[t][u] = zb[t][q[u].z];
                xk[t][u] = zb[t][q[u].w];
#pragma unroll
                for (int d = 0; d < 3; ++d) g[t][u][d] = Gb[t][3 * (int64_t)q[u].x + d];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const float *gg = g[t][u];
                const float2 ui = make_float2(ei[0] * gg[0] + ei[1] * gg[1] + ei[2] * gg[2],
                                              ei[3] * gg[0] + ei[4] * gg[1] + ei[5] * gg[2]);
                const float2 uj = make_float2(ej[u][0] * gg[0] + ej[u][1] * gg[1] + ej[u][2] * gg[2],
                                              ej[u][3] * gg[0] + ej[u][4] * gg[1] + ej[u][5] * gg[2]);
                const float2 uk = make_float2(ek[u][0] * gg[0] + ek[u][1] * gg[1] + ek[u][2] * gg[2],
                                              ek[u][3] * gg[0] + ek[u][4] * gg[1] + ek[u][5] * gg[2]);
                const float si = ui.x * zi[t].x + ui.y * zi[t].y;
                const float sj = uj.x * xj[t][u].x + uj.y * xj[t][u].y;
                const float sk = uk.x * xk[t][u].x + uk.y * xk[t][u].y;
                const float cc = t0 + u < w ? (si + si) + sj + sk : 0.f;
                a0[t] += ui.x * cc;
                a1[t] += ui.y * cc;
            }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) epilogue(v, (int64_t)(2 * bp + t) * N + i, a0[t], a1[t]);
}

template <typename T>
static T *dev(const std::vector<T> &h) {
    T *d;
    CK(hipMalloc(&d, h.size() * sizeof(T)));
    CK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return d;
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s mesh.bin [B] [reps]\n", argv[0]);
        return 2;
    }
    const int32_t B = argc > 2 ? (atoi(argv[2]) + 1) / 2 * 2 : 256, reps = argc > 3 ? atoi(argv[3]) : 20;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    int32_t N, M;
    if (fread(&N, 4, 1, f) != 1 || fread(&M, 4, 1, f) != 1) return 2;
    std::vector<int32_t> tri(3 * (size_t)M);
    std::vector<float> E(6 * (size_t)N), w12(M);
    if (fread(tri.data(), 4, tri.size(), f) != tri.size() || fread(E.data(), 4, E.size(), f) != E.size() ||
        fread(w12.data(), 4, w12.size(), f) != w12.size())
        return 2;
    fclose(f);
    // rows: diagonal, then neighbours ascending
    std::vector<std::vector<int32_t>> nb(N);
    std::vector<std::vector<int4>> inc(N);
    for (int32_t T = 0; T < M; ++T)
        for (int c = 0; c < 3; ++c) {
            const int32_t a = tri[3 * T + c], j = tri[3 * T + (c + 1) % 3], k = tri[3 * T + (c + 2) % 3];
            nb[a].push_back(j);
            nb[a].push_back(k);
            inc[a].push_back(make_int4(T, c, j, k));
        }
    for (int32_t i = 0; i < N; ++i) {
        auto &r = nb[i];
        std::sort(r.begin(), r.end());
        r.erase(std::unique(r.begin(), r.end()), r.end());
        r.insert(r.begin(), i);
    }
    const int32_t ns = (N + kSl - 1) / kSl, nblk = (N + kWG - 1) / kWG;
    std::vector<int32_t> off(ns + 1, 0), toff(ns + 1, 0);
    for (int32_t s = 0; s < ns; ++s) {
        int32_t w = 0, wt = 0;
        for (int32_t l = 0; l < kSl && s * kSl + l < N; ++l) {
            w = std::max<int32_t>(w, nb[s * kSl + l].size());
            wt = std::max<int32_t>(wt, inc[s * kSl + l].size());
        }
        off[s + 1] = off[s] + w * kSl;
        toff[s + 1] = toff[s] + wt * kSl;
    }
    const int64_t nbk = off[ns];
    auto pos = [&](int32_t i, int32_t j) -> int64_t {
        const auto &r = nb[i];
        int32_t t = j == i ? 0 : (int32_t)(std::lower_bound(r.begin() + 1, r.end(), j) - r.begin());
        return off[i / kSl] + (int64_t)t * kSl + i % kSl;
    };
    std::vector<int32_t> col(nbk), mir(nbk, -1);
    std::vector<int4> tinc(toff[ns]);
    for (int32_t i = 0; i < N; ++i) {
        const int32_t s = i / kSl, l = i % kSl;
        const int32_t w = (off[s + 1] - off[s]) / kSl, wt = (toff[s + 1] - toff[s]) / kSl;
        for (int32_t t = 0; t < w; ++t) {
            const int64_t p = off[s] + (int64_t)t * kSl + l;
            if (t < (int32_t)nb[i].size()) {
                const int32_t j = nb[i][t];
                col[p] = j;
                mir[p] = j < i ? (int32_t)pos(j, i) | kMirT : (int32_t)p;
            } else {
                col[p] = i;
            }
        }
        for (int32_t t = 0; t < wt; ++t)
            tinc[toff[s] + (int64_t)t * kSl + l] = t < (int32_t)inc[i].size() ? inc[i][t] : make_int4(M, 0, i, i);
    }
    // a2: lambda * L_ij E_i^T E_j (graph Laplacian weights); g: random per
    // triangle with sqrt(w12) folded in (one system's values, copied to all)
    const float lam = 0.1f;
    std::vector<float4> a2(nbk, make_float4(0, 0, 0, 0)), A1(nbk);
    auto ete = [&](int32_t i, int32_t j, float c) {
        const float *a = &E[6 * (size_t)i], *b = &E[6 * (size_t)j];
        auto d = [](const float *x, const float *y) { return x[0] * y[0] + x[1] * y[1] + x[2] * y[2]; };
        return make_float4(c * d(a, b), c * d(a, b + 3), c * d(a + 3, b), c * d(a + 3, b + 3));
    };
    for (int32_t i = 0; i < N; ++i)
        for (size_t t = 0; t < nb[i].size(); ++t) {
            const int32_t j = nb[i][t];
            a2[pos(i, j)] = ete(i, j, j == i ? lam * (float)(nb[i].size() - 1) : -lam);
        }
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> U(-1.f, 1.f);
    std::vector<float> g(3 * (size_t)(M + 1), 0.f), u(6 * (size_t)(M + 1), 0.f);
    for (int32_t T = 0; T < M; ++T)
        for (int d = 0; d < 3; ++d) g[3 * (size_t)T + d] = U(rng) * std::sqrt(w12[T]);
    for (int32_t T = 0; T < M; ++T)
        for (int c = 0; c < 3; ++c) {
            const float *e = &E[6 * (size_t)tri[3 * T + c]], *gg = &g[3 * (size_t)T];
            u[6 * (size_t)T + 2 * c] = e[0] * gg[0] + e[1] * gg[1] + e[2] * gg[2];
            u[6 * (size_t)T + 2 * c + 1] = e[3] * gg[0] + e[4] * gg[1] + e[5] * gg[2];
        }
    std::vector<float4> A(a2);
    for (int32_t T = 0; T < M; ++T)
        for (int a = 0; a < 3; ++a)
            for (int c = 0; c < 3; ++c) {
                const int32_t i = tri[3 * T + a], j = tri[3 * T + c];
                const float *ua = &u[6 * (size_t)T + 2 * a], *uc = &u[6 * (size_t)T + 2 * c];
                const float m = a == c ? 2.f : 1.f;
                float4 &k = A[pos(i, j)];
                k.x += m * ua[0] * uc[0];
                k.y += m * ua[0] * uc[1];
                k.z += m * ua[1] * uc[0];
                k.w += m * ua[1] * uc[1];
            }
    // device data, B systems
    std::vector<float4> AB((size_t)B * nbk);
    std::vector<float> gB((size_t)B * g.size()), uB((size_t)B * u.size());
    for (int32_t b = 0; b < B; ++b) {
        std::copy(A.begin(), A.end(), AB.begin() + (size_t)b * nbk);
        std::copy(g.begin(), g.end(), gB.begin() + (size_t)b * g.size());
        std::copy(u.begin(), u.end(), uB.begin() + (size_t)b * u.size());
    }
    std::vector<float2> z((size_t)B * N);
    for (auto &e : z) e = make_float2(U(rng), U(rng));
    int32_t *d_off = dev(off), *d_col = dev(col), *d_mir = dev(mir), *d_toff = dev(toff);
    int4 *d_tinc = dev(tinc);
    float4 *d_A = dev(AB), *d_a2 = dev(a2);
    float *d_E = dev(E), *d_g = dev(gB), *d_u = dev(uB);
    std::vector<float4>().swap(AB);
    float2 *d_z = dev(z), *d_p, *d_q, *d_x;
    const size_t vb = (size_t)B * N * sizeof(float2);
    CK(hipMalloc(&d_p, vb));
    CK(hipMalloc(&d_q, vb));
    CK(hipMalloc(&d_x, vb));
    const int32_t grid = ((nblk + 7) / 8) * 8 * B;
    auto launch = [&](int form, float al, float be) {
        Vec v{d_z, d_p, d_q, d_x, al, be};
        if (form == 0) k_mat<false><<<grid, kWG>>>(N, nblk, B, d_off, d_col, d_mir, d_A, nbk, v);
        if (form == 1) k_mat<true><<<grid, kWG>>>(N, nblk, B, d_off, d_col, d_mir, d_A, nbk, v);
        if (form == 2) k_tri<false><<<grid, kWG>>>(N, M, nblk, B, d_off, d_col, d_a2, d_toff, d_tinc, d_E, d_g, v);
        if (form == 3) k_tri<true><<<grid, kWG>>>(N, M, nblk, B, d_off, d_col, d_a2, d_toff, d_tinc, d_E, d_u, v);
        if (form == 4)
            k_tri2<<<((nblk + 7) / 8) * 8 * (B / 2), kWG>>>(N, M, nblk, B, d_off, d_col, d_a2, d_toff, d_tinc, d_E,
                                                           d_g, v);
        CK(hipGetLastError());
    };
    const char *names[5] = {"mat", "matm", "tri_g", "tri_u", "tri_g2"};
    std::vector<float2> ref, got((size_t)B * N);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int form = 0; form < 5; ++form) {
        // parity: alpha = beta = 0 leaves q = A z
        CK(hipMemset(d_p, 0, vb));
        CK(hipMemset(d_q, 0, vb));
        CK(hipMemset(d_x, 0, vb));
        launch(form, 0.f, 0.f);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got.data(), d_q, vb, hipMemcpyDeviceToHost));
        if (form == 0) ref = got;
        double err = 0, mx = 0;
        for (size_t k = 0; k < got.size(); ++k) {
            err = std::max(err, (double)std::fabs(got[k].x - ref[k].x));
            err = std::max(err, (double)std::fabs(got[k].y - ref[k].y));
            mx = std::max(mx, (double)std::fabs(ref[k].x));
        }
        for (int r = 0; r < 3; ++r) launch(form, 0.5f, 0.3f);
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch(form, 0.5f, 0.3f);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1e3 * ms / reps;
        printf("{\"form\": \"%s\", \"N\": %d, \"M\": %d, \"B\": %d, \"us_per_launch\": %.1f, \"us_per_system\": %.3f, "
               "\"B_per_vertex_at_8TBs\": %.1f, \"max_abs_diff_vs_mat\": %.3g, \"max_abs\": %.3g}\n",
               names[form], N, M, B, us, us / B, us / B * 1e-6 * 8e12 / N, err, mx);
        fflush(stdout);
    }
    return 0;
}
