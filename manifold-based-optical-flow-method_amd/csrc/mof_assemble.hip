// mof_assemble.hip -- geometry and per-timestep FEM assembly kernels (gfx950).
//
// Compiled with -ffp-contract=off: every product and sum below is rounded
// exactly where the reference's numpy code rounds it, and the only fused
// multiply-adds are the explicit fma() calls that restate np.dot of two
// float64 3-vectors on the reference's BLAS (fma(x2,y2, fma(x1,y1, x0*y0)),
// DESIGN.md §Bit-exact assembly). The assembled A and f therefore match the
// reference's bit for bit (tests/test_gpu_parity.py).
//
// All per-timestep accumulation is a gather in triangle order over the
// pre-built contribution lists (mof_pattern.cpp): deterministic, no atomics.
#include "mof_amg.h"
#include "mof_internal.h"
#include "mof_rowkern.h"

namespace mof {
namespace {

__device__ __forceinline__ double dot64(const double *x, const double *y) {
    return fma(x[2], y[2], fma(x[1], y[1], x[0] * y[0]));
}

// np.dot of two float32 3-vectors on scipy-openblas: float products summed
// in double, rounded to float once.
__device__ __forceinline__ float dot32(const float *x, const float *y) {
    double acc = 0.0;
    acc += (double)(x[0] * y[0]);
    acc += (double)(x[1] * y[1]);
    acc += (double)(x[2] * y[2]);
    return (float)acc;
}

// compute_orthonormal_basis (compute_optical_flow.py:210-235), one vertex per
// thread. numpy types the basis float64 even for float32 normals.
__global__ __launch_bounds__(kWG) void k_basis(const double *__restrict__ nrm, int32_t N,
                                               double *__restrict__ e) {
    const int32_t i = blockIdx.x * kWG + threadIdx.x;
    if (i >= N) return;
    const double n[3] = {nrm[3 * (int64_t)i], nrm[3 * (int64_t)i + 1], nrm[3 * (int64_t)i + 2]};
    double a[3], c[3];
    if (n[0] != 0.0 || n[1] != 0.0) {
        a[0] = -n[1]; a[1] = n[0]; a[2] = 0.0;
    } else {
        a[0] = 0.0; a[1] = -n[2]; a[2] = n[1];
    }
    c[0] = n[1] * a[2] - n[2] * a[1];
    c[1] = n[2] * a[0] - n[0] * a[2];
    c[2] = n[0] * a[1] - n[1] * a[0];
    const double na = sqrt(dot64(a, a)), nc = sqrt(dot64(c, c));
    double *o = e + 6 * (int64_t)i;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        o[d] = a[d] / na;
        o[3 + d] = c[d] / nc;
    }
}

// compute_gradient_w(p_i, p_j, p_k) (:238-255): the altitude vector from i
// scaled by 1/|h|^2.
__device__ void grad_w64(const double *pi, const double *pj, const double *pk, double *g) {
    double jk[3], ji[3], ih[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        jk[d] = pk[d] - pj[d];
        ji[d] = pi[d] - pj[d];
    }
    const double s = dot64(ji, jk), q = dot64(jk, jk);
#pragma unroll
    for (int d = 0; d < 3; ++d) ih[d] = (pj[d] - pi[d]) + (s * jk[d]) / q;
    const double h = dot64(ih, ih);
#pragma unroll
    for (int d = 0; d < 3; ++d) g[d] = ih[d] / h;
}

__device__ void grad_w32(const double *pid, const double *pjd, const double *pkd, double *g) {
    float pi[3], pj[3], pk[3], jk[3], ji[3], ih[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        pi[d] = (float)pid[d];
        pj[d] = (float)pjd[d];
        pk[d] = (float)pkd[d];
    }
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        jk[d] = pk[d] - pj[d];
        ji[d] = pi[d] - pj[d];
    }
    const float s = dot32(ji, jk), q = dot32(jk, jk);
#pragma unroll
    for (int d = 0; d < 3; ++d) ih[d] = (pj[d] - pi[d]) + (s * jk[d]) / q;
    const float h = dot32(ih, ih);
#pragma unroll
    for (int d = 0; d < 3; ++d) g[d] = (double)(ih[d] / h);
}

// grad_w (M,3,3) and integral_wi_wj (M,2) (:60-75), one triangle per thread.
template <bool F32>
__global__ __launch_bounds__(kWG) void k_gradw(const double *__restrict__ xyz,
                                               const int32_t *__restrict__ tri,
                                               const double *__restrict__ area, int32_t M,
                                               double *__restrict__ gw, double *__restrict__ iw) {
    const int32_t T = blockIdx.x * kWG + threadIdx.x;
    if (T >= M) return;
    const int32_t *v = tri + 3 * (int64_t)T;
    double P[3][3];
#pragma unroll
    for (int l = 0; l < 3; ++l)
#pragma unroll
        for (int d = 0; d < 3; ++d) P[l][d] = xyz[3 * (int64_t)v[l] + d];
    double *g = gw + 9 * (int64_t)T;
    if (F32) {
        grad_w32(P[0], P[1], P[2], g);
        grad_w32(P[1], P[0], P[2], g + 3);
        grad_w32(P[2], P[0], P[1], g + 6);
    } else {
        grad_w64(P[0], P[1], P[2], g);
        grad_w64(P[1], P[0], P[2], g + 3);
        grad_w64(P[2], P[0], P[1], g + 6);
    }
    const double A = area[T];
    iw[2 * (int64_t)T] = A / 6;
    iw[2 * (int64_t)T + 1] = A / 12;
}

__device__ __forceinline__ int64_t sell_pos(const int32_t *sell_off, int32_t i, int32_t t) {
    return (int64_t)sell_off[i >> 6] + (int64_t)t * kSlice + (i & 63);
}

// a2 (:78-93, compute_a2 :258-270), one vertex row per thread: block (i, j)
// entry (alpha, beta) = fold over the triangles holding edge (i, j) of
// (e_i^alpha . e_j^beta)(grad w_a . grad w_b) A_T, in triangle order.
__global__ __launch_bounds__(kWG) void k_a2(int32_t N, const int32_t *__restrict__ vptr,
                                            const int32_t *__restrict__ vcol,
                                            const int32_t *__restrict__ cptr,
                                            const int32_t *__restrict__ clist,
                                            const int32_t *__restrict__ sell_off,
                                            const double *__restrict__ e,
                                            const double *__restrict__ gw,
                                            const double *__restrict__ area,
                                            double *__restrict__ a2) {
    const int32_t i = blockIdx.x * kWG + threadIdx.x;
    if (i >= N) return;
    const double *ei = e + 6 * (int64_t)i;
    int32_t td = 0;
    while (vcol[vptr[i] + td] != i) ++td;
    for (int32_t p = vptr[i], t = 0; p < vptr[i + 1]; ++p, ++t) {
        const int32_t j = vcol[p];
        const double *ej = e + 6 * (int64_t)j;
        double ee[4];
#pragma unroll
        for (int al = 0; al < 2; ++al)
#pragma unroll
            for (int be = 0; be < 2; ++be) ee[2 * al + be] = dot64(ei + 3 * al, ej + 3 * be);
        double acc[4] = {0.0, 0.0, 0.0, 0.0};
        for (int32_t c = cptr[p]; c < cptr[p + 1]; ++c) {
            const int32_t code = clist[c];
            const int32_t T = code / 9, a = (code % 9) / 3, b = code % 3;
            const double *g = gw + 9 * (int64_t)T;
            const double gg = dot64(g + 3 * a, g + 3 * b);
            const double A = area[T];
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[q] += ee[q] * gg * A;
        }
        double *o = a2 + 4 * sell_pos(sell_off, i, sell_slot(t, td));
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = acc[q];
    }
}

// Per-triangle half of worker (:113-126, compute_f :288-311) for B systems:
// grad_M I and, for each corner a and alpha, u = grad_M I . e_a^alpha and the
// f term (u (2 dI_a + sum of the other distinct corners' dI) A_T) / 12.
// Triangle slot M of u / fc stays zero (padding of the incidence lists).
__global__ __launch_bounds__(kWG) void k_tri_step(int32_t M, int32_t B, const int32_t *__restrict__ tri,
                                                  const int32_t *__restrict__ icorner,
                                                  const double *__restrict__ gw,
                                                  const double *__restrict__ e,
                                                  const double *__restrict__ area,
                                                  const double *__restrict__ I0,
                                                  const double *__restrict__ I1, int64_t ldI,
                                                  const double *__restrict__ dt,
                                                  double *__restrict__ u, double *__restrict__ fc,
                                                  float *__restrict__ u32) {
    // one triangle per thread for all B systems: the geometry is read once
    const int32_t T = blockIdx.x * kWG + threadIdx.x;
    if (T >= M) return;
    const int32_t v[3] = {tri[3 * (int64_t)T], tri[3 * (int64_t)T + 1], tri[3 * (int64_t)T + 2]};
    double g[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) g[q] = gw[9 * (int64_t)T + q];
    // I rows are indexed by icorner: the caller's vertex ids, or the internal
    // ids when the rows were permuted to the internal order (k_gather_I)
    const int32_t vo[3] = {icorner[3 * (int64_t)T], icorner[3 * (int64_t)T + 1],
                           icorner[3 * (int64_t)T + 2]};
    const double A = area[T];
    double ev[3][6];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int q = 0; q < 6; ++q) ev[a][q] = e[6 * (int64_t)v[a] + q];
    for (int32_t b = 0; b < B; ++b) {
        const double *i0 = I0 + b * ldI;
        const double *i1 = I1 + b * ldI;
        const double a0 = i0[vo[0]], a1 = i0[vo[1]], a2 = i0[vo[2]];
        double gI[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) gI[d] = (a0 * g[d] + a1 * g[3 + d]) + a2 * g[6 + d];
        const double h = dt[b];
        const double pd[3] = {(i1[vo[0]] - a0) / h, (i1[vo[1]] - a1) / h, (i1[vo[2]] - a2) / h};
        const int64_t base = 6 * ((int64_t)b * (M + 1) + T);
        double uo[6], fo[6];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            // set(T) - {i}: distinct corners other than vertex v[a], in corner order
            double po = 0.0;
            int cnt = 0;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                bool dup = false;
#pragma unroll
                for (int q = 0; q < c; ++q) dup |= (v[q] == v[c]);
                if (dup || v[c] == v[a]) continue;
                po = cnt ? po + pd[c] : pd[c];
                ++cnt;
            }
#pragma unroll
            for (int al = 0; al < 2; ++al) {
                const double uu = dot64(gI, &ev[a][3 * al]);
                uo[2 * a + al] = uu;
                fo[2 * a + al] = uu * (2 * pd[a] + po) * A / 12;
            }
        }
#pragma unroll
        for (int q = 0; q < 6; q += 2) {
            if (u) *reinterpret_cast<double2 *>(u + base + q) = make_double2(uo[q], uo[q + 1]);
            *reinterpret_cast<double2 *>(fc + base + q) = make_double2(fo[q], fo[q + 1]);
            if (u32) *reinterpret_cast<float2 *>(u32 + base + q) = make_float2((float)uo[q], (float)uo[q + 1]);
        }
    }
}

// Solve-path A_b = a1_b + lambda a2 of B systems (fp64 PCG), one SELL
// position per thread (coalesced stores): the a1 block is folded in fp64 over
// its terms in triangle order exactly as the export path does (the mixed
// path uses k_assemble_mixed below). The thread
// holding a diagonal block also folds f_i (bit-identical to the reference's
// f) and writes the 2x2 block-Jacobi inverse of vertex i. Terms are fetched
// four at a time (indices, then u pairs) so the fold is not one memory round
// trip per term. SELL padding is never written and stays zero.
template <typename V>
__global__ __launch_bounds__(kWG) void k_assemble_blocks(
    int64_t sell_nb, int32_t N, int32_t M, int32_t B, const int32_t *__restrict__ sell_blk,
    const int32_t *__restrict__ blk_row, const int32_t *__restrict__ vcol,
    const int32_t *__restrict__ cptr, const int32_t *__restrict__ clist,
    const double *__restrict__ iw, const double *__restrict__ a2s, const double *__restrict__ u,
    const double *__restrict__ fc, int block_jacobi, V *__restrict__ A,
    double *__restrict__ dinv64, float *__restrict__ dinv32, double *__restrict__ rhs) {
    // XCD-aware tiles: the B systems of a 256-slot tile run back to back on
    // one XCD and share the tile's structure, lambda a2 and iw in its L2
    int32_t tile, b;
    if (!xcd_map((int32_t)((sell_nb + kWG - 1) / kWG), B, tile, b, kGrpAsm)) return;
    const int64_t pos = (int64_t)tile * kWG + threadIdx.x;
    if (pos >= sell_nb) return;
    const int32_t p = sell_blk[pos];
    if (p < 0) return;
    const int32_t i = blk_row[p];
    const bool diag = (vcol[p] == i);
    const double *ub = u + 6 * (int64_t)b * (M + 1);
    const double *fb = fc + 6 * (int64_t)b * (M + 1);
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    double f0 = 0.0, f1 = 0.0;
    const int32_t c0 = cptr[p], c1 = cptr[p + 1];
    constexpr int U = 4;
    for (int32_t c = c0; c < c1; c += U) {
        int32_t T[U], a[U], bb[U];
#pragma unroll
        for (int q = 0; q < U; ++q) {
            const int32_t code = clist[min(c + q, c1 - 1)];
            T[q] = code / 9;
            a[q] = (code % 9) / 3;
            bb[q] = code % 3;
        }
        double2 ua[U], uv[U];
        double integ[U];
#pragma unroll
        for (int q = 0; q < U; ++q) {
            ua[q] = *reinterpret_cast<const double2 *>(ub + 6 * (int64_t)T[q] + 2 * a[q]);
            uv[q] = *reinterpret_cast<const double2 *>(ub + 6 * (int64_t)T[q] + 2 * bb[q]);
            integ[q] = iw[2 * (int64_t)T[q] + (diag ? 0 : 1)];
        }
#pragma unroll
        for (int q = 0; q < U; ++q) {
            if (c + q >= c1) break;
            acc[0] += ua[q].x * uv[q].x * integ[q];
            acc[1] += ua[q].x * uv[q].y * integ[q];
            acc[2] += ua[q].y * uv[q].x * integ[q];
            acc[3] += ua[q].y * uv[q].y * integ[q];
            if (diag && a[q] == bb[q]) {
                const double2 fv = *reinterpret_cast<const double2 *>(fb + 6 * (int64_t)T[q] + 2 * a[q]);
                f0 += fv.x;
                f1 += fv.y;
            }
        }
    }
    const double2 s01 = *reinterpret_cast<const double2 *>(a2s + 4 * pos);
    const double2 s23 = *reinterpret_cast<const double2 *>(a2s + 4 * pos + 2);
    const double Av[4] = {acc[0] + s01.x, acc[1] + s01.y, acc[2] + s23.x, acc[3] + s23.y};
    V *o = A + 4 * ((int64_t)b * sell_nb + pos);
    if constexpr (sizeof(V) == 4) {
        *reinterpret_cast<float4 *>(o) =
            make_float4((float)Av[0], (float)Av[1], (float)Av[2], (float)Av[3]);
    } else {
        *reinterpret_cast<double2 *>(o) = make_double2(Av[0], Av[1]);
        *reinterpret_cast<double2 *>(o + 2) = make_double2(Av[2], Av[3]);
    }
    if (!diag) return;
    double inv[4];
    if (block_jacobi) {
        const double det = Av[0] * Av[3] - Av[1] * Av[2];
        inv[0] = Av[3] / det; inv[1] = -Av[1] / det; inv[2] = -Av[2] / det; inv[3] = Av[0] / det;
    } else {
        inv[0] = 1.0 / Av[0]; inv[1] = 0.0; inv[2] = 0.0; inv[3] = 1.0 / Av[3];
    }
    const int64_t vi = (int64_t)b * N + i;
    *reinterpret_cast<double2 *>(dinv64 + 4 * vi) = make_double2(inv[0], inv[1]);
    *reinterpret_cast<double2 *>(dinv64 + 4 * vi + 2) = make_double2(inv[2], inv[3]);
    *reinterpret_cast<float4 *>(dinv32 + 4 * vi) =
        make_float4((float)inv[0], (float)inv[1], (float)inv[2], (float)inv[3]);
    *reinterpret_cast<double2 *>(rhs + 2 * vi) = make_double2(f0, f1);
}

// lambda * a2 for the solve operator (fp64 copy bit-identical to the
// reference's lambda_ * a2, :144) and its fp32 rounding.
// Mixed-precision solve path: A32 = a1 + lambda a2 folded in fp32 from the
// fp32 copy of u (half the gathered bytes of the fp64 fold; the inner PCG
// runs on fp32 A anyway and the fp64 refinement uses the exact operator).
// The diagonal slot also folds f in fp64 from the f terms (bit-identical to
// the reference's f: its own-corner terms in triangle order; folding them in
// the main loop measured 0.5 % slower) and writes the 2x2 block-Jacobi
// inverse. With the multigrid preconditioner (Ah != null)
// the bf16 copies of A and D^-1 the level-0 smoother sweeps read are written
// here too (D^-1 then only in bf16: the PCG applies the V-cycle, not D^-1).
__global__ __launch_bounds__(kWG) void k_assemble_mixed(
    int64_t sell_nb, int32_t N, int32_t M, int32_t B, const int32_t *__restrict__ sell_blk,
    const int32_t *__restrict__ blk_row, const int32_t *__restrict__ vcol,
    const int32_t *__restrict__ cptr, const int32_t *__restrict__ clist,
    const float *__restrict__ w12, const float *__restrict__ a2s, const float *__restrict__ u,
    const double *__restrict__ fc, int block_jacobi, float *__restrict__ A,
    float *__restrict__ dinv32, double *__restrict__ rhs, uint2 *__restrict__ Ah, int32_t nown) {
    int32_t tile, b;
    if (!xcd_map((int32_t)((sell_nb + kWG - 1) / kWG), B, tile, b, kGrpAsm)) return;
    const int64_t pos = (int64_t)tile * kWG + threadIdx.x;
    if (pos >= sell_nb) return;
    const int32_t p = sell_blk[pos];
    if (p < 0) return;
    const int32_t i = blk_row[p];
    const bool diag = (vcol[p] == i);
    const float *ub = u + 6 * (int64_t)b * (M + 1);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    const int32_t c0 = cptr[p], c1 = cptr[p + 1];
    constexpr int U = 4;  // 6 / 8: 7492 / 8475 vs 7065 us per 256-system launch
    for (int32_t c = c0; c < c1; c += U) {
        int32_t T[U], a[U], bb[U];
#pragma unroll
        for (int q = 0; q < U; ++q) {
            const int32_t code = clist[min(c + q, c1 - 1)];
            T[q] = code / 9;
            a[q] = (code % 9) / 3;
            bb[q] = code % 3;
        }
        float2 ua[U], uv[U];
        float wq[U];
#pragma unroll
        for (int q = 0; q < U; ++q) {
            ua[q] = *reinterpret_cast<const float2 *>(ub + 6 * (int64_t)T[q] + 2 * a[q]);
            uv[q] = *reinterpret_cast<const float2 *>(ub + 6 * (int64_t)T[q] + 2 * bb[q]);
            wq[q] = w12[T[q]];
        }
#pragma unroll
        for (int q = 0; q < U; ++q) {
            const bool on = c + q < c1;
            const float integ = on ? (diag ? 2.f * wq[q] : wq[q]) : 0.f;
            acc[0] += ua[q].x * uv[q].x * integ;
            acc[1] += ua[q].x * uv[q].y * integ;
            acc[2] += ua[q].y * uv[q].x * integ;
            acc[3] += ua[q].y * uv[q].y * integ;
        }
    }
    const float4 s4 = reinterpret_cast<const float4 *>(a2s)[pos];
    const float Av[4] = {acc[0] + s4.x, acc[1] + s4.y, acc[2] + s4.z, acc[3] + s4.w};
    const int64_t q = (int64_t)b * sell_nb + pos;
    reinterpret_cast<float4 *>(A)[q] = make_float4(Av[0], Av[1], Av[2], Av[3]);
    if (Ah) {
        // a decomposed part's ghost rows: identity rows, no coupling (the
        // smoother and coarse levels see the owned rows' Dirichlet problem)
        const bool g = i >= nown || vcol[p] >= nown;
        if (g)
            h0_st(Ah, q, diag ? 1.f : 0.f, 0.f, 0.f, diag ? 1.f : 0.f);
        else
            h0_st(Ah, q, Av[0], Av[1], Av[2], Av[3]);
    }
    if (!diag) return;
    // f_i in fp64, in the reference's triangle order
    const double *fb = fc + 6 * (int64_t)b * (M + 1);
    double f0 = 0.0, f1 = 0.0;
    // the codes and f terms of a chunk are all fetched before the in-order
    // fold (masked slots add nothing: the running sum is never -0.0)
    constexpr int UF = 8;
    for (int32_t c = c0; c < c1; c += UF) {
        int32_t code[UF];
#pragma unroll
        for (int q = 0; q < UF; ++q) code[q] = clist[min(c + q, c1 - 1)];
        double2 fv[UF];
#pragma unroll
        for (int q = 0; q < UF; ++q)
            fv[q] = *reinterpret_cast<const double2 *>(fb + 6 * (int64_t)(code[q] / 9) + 2 * ((code[q] % 9) / 3));
#pragma unroll
        for (int q = 0; q < UF; ++q) {
            const bool on = c + q < c1 && (code[q] % 9) / 3 == code[q] % 3;
            if (on) {
                f0 += fv[q].x;
                f1 += fv[q].y;
            }
        }
    }
    double inv[4];
    const double d0 = Av[0], d1 = Av[1], d2 = Av[2], d3 = Av[3];
    if (block_jacobi) {
        const double det = d0 * d3 - d1 * d2;
        inv[0] = d3 / det; inv[1] = -d1 / det; inv[2] = -d2 / det; inv[3] = d0 / det;
    } else {
        inv[0] = 1.0 / d0; inv[1] = 0.0; inv[2] = 0.0; inv[3] = 1.0 / d3;
    }
    const int64_t vi = (int64_t)b * N + i;
    // multigrid (Ah): the smoother's D comes from the bf16 diagonal blocks
    if (!Ah)
        reinterpret_cast<float4 *>(dinv32)[vi] =
            make_float4((float)inv[0], (float)inv[1], (float)inv[2], (float)inv[3]);
    *reinterpret_cast<double2 *>(rhs + 2 * vi) = make_double2(f0, f1);
}

// Row i's stores of one system: A blocks (+ lambda a2), the bf16 copies,
// the diagonal block's inverse and f_i.
template <int WMAX>
__device__ __forceinline__ void rows_store(const float (&acc)[WMAX][4], double f0, double f1, int32_t i, int32_t b,
                                           int32_t N, int32_t deg, int64_t o, int64_t sell_nb,
                                           const int32_t *__restrict__ sell_col, const float *__restrict__ a2s,
                                           int block_jacobi, float *__restrict__ A, float *__restrict__ dinv32,
                                           double *__restrict__ rhs, uint2 *__restrict__ Ah, int32_t nown,
                                           const int32_t *__restrict__ mir) {
#pragma unroll
    for (int z = 0; z < WMAX; ++z) {
        if (z >= deg) continue;
        const int64_t pos = o + (int64_t)z * kSlice;
        // symmetric layout: lower blocks are read as transposed upper
        // ones and never leave the registers
        if (mir && (mir[pos] & kMirT)) continue;
        const int64_t qq = (int64_t)b * sell_nb + pos;
        const float4 s4 = reinterpret_cast<const float4 *>(a2s)[pos];
        const float Av[4] = {acc[z][0] + s4.x, acc[z][1] + s4.y, acc[z][2] + s4.z, acc[z][3] + s4.w};
        reinterpret_cast<float4 *>(A)[qq] = make_float4(Av[0], Av[1], Av[2], Av[3]);
        if (Ah) {
            const bool g = i >= nown || sell_col[pos] >= nown;
            if (g)
                h0_st(Ah, qq, z == 0 ? 1.f : 0.f, 0.f, 0.f, z == 0 ? 1.f : 0.f);
            else
                h0_st(Ah, qq, Av[0], Av[1], Av[2], Av[3]);
        }
        if (z != 0) continue;
        double inv[4];
        const double d0 = Av[0], d1 = Av[1], d2 = Av[2], d3 = Av[3];
        if (block_jacobi) {
            const double det = d0 * d3 - d1 * d2;
            inv[0] = d3 / det; inv[1] = -d1 / det; inv[2] = -d2 / det; inv[3] = d0 / det;
        } else {
            inv[0] = 1.0 / d0; inv[1] = 0.0; inv[2] = 0.0; inv[3] = 1.0 / d3;
        }
        const int64_t vi = (int64_t)b * N + i;
        if (!Ah)  // multigrid: the smoother's D comes from the bf16 diagonal blocks
            reinterpret_cast<float4 *>(dinv32)[vi] =
                make_float4((float)inv[0], (float)inv[1], (float)inv[2], (float)inv[3]);
        *reinterpret_cast<double2 *>(rhs + 2 * vi) = make_double2(f0, f1);
    }
}

// Mixed-precision assembly by vertex rows (the PCG row layout and XCD-aware
// (row block, system) order). Thread i walks the incident triangles of
// vertex i in the caller's triangle order (tinc, SELL-64) and, per
// triangle, forms grad_M I, u = grad_M I . e_i and
// row i's f term in k_tri_step's exact arithmetic (the I0 values in the
// triangle's own corner order, np.dot's fma chain, the f term's operation
// order), then adds the
// triangle's three a1 terms of row i -- (i,i), (i,v_{a+1}), (i,v_{a+2}) --
// to register accumulators of the row's SELL slots (tslot; WMAX >= the
// widest row: fma by 0/1 slot masks, no dynamic register indexing). f folds
// in fp64 in the reference's triangle order, bit for bit; A32 is an fp32
// fold (the inner operator). Measured and not kept (round 2): a separate
// per-triangle pass storing u32 / f terms for the rows to gather back (72 B
// stored and 120 B gathered per triangle and system: 4.13 + 8.22 vs 10.19 ms
// per 512-system launch at C3), 2 / 4 systems per thread sharing each
// triangle's geometry (VGPRs 124 -> 290, 10.0 / 10.4 / 14.6 ms at 1 / 2 / 4),
// a mul-add fold (11.9 ms), LDS slot accumulators (21.0 ms).
struct TriGeo {
    const double *gw, *e, *area, *J0, *J1, *dt;  // J0 / J1: the batch's I rows (internal order, stride N)
};
// Round 4: the a1 fold in ambient 3-D. a1's block (i, j) is
// sum_T w_ij (E_i gI_T)(E_j gI_T)^T = E_i G_ij E_j^T with the symmetric 3x3
// G_ij = sum_T w_ij gI_T gI_T^T (compute_a1 :273-285), so a row folds one
// outer product per incident triangle into its slots' G (6 floats each) and
// projects each stored slot once at the end -- no tangent frames of the two
// other corners gathered per incidence and no u_j, u_k dots (A32 is an fp32
// fold of the same operator, rounded differently; f keeps its bits). C3,
// B = 512, rocprof on one box (profiles/r04_ab/call1b/): 9047-9163 -> 8630 us
// per launch against the round-3 per-incidence 2x2 fold.
// g3_store: the slots' blocks E_i G E_j^T + lambda a2, then rows_store's stores.
template <int WMAX>
__device__ __forceinline__ void g3_project(const float (&G)[WMAX][6], const double (&ei)[6], int32_t deg, int64_t o,
                                           const int32_t *__restrict__ sell_col, const double *__restrict__ e,
                                           const int32_t *__restrict__ mir, float (&acc)[WMAX][4]) {
    float eif[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) eif[k] = (float)ei[k];
#pragma unroll
    for (int z = 0; z < WMAX; ++z) {
        acc[z][0] = acc[z][1] = acc[z][2] = acc[z][3] = 0.f;
        if (z >= deg) continue;
        const int64_t pos = o + (int64_t)z * kSlice;
        if (mir && (mir[pos] & kMirT)) continue;  // lower blocks are never stored
        const int32_t j = sell_col[pos];
        float ej[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) ej[k] = (float)e[6 * (int64_t)j + k];
        // G = [xx xy xz; xy yy yz; xz yz zz]; H = G E_j^T (3 x 2)
        const float *g = G[z];
        float H[3][2];
#pragma unroll
        for (int be = 0; be < 2; ++be) {
            const float *v = ej + 3 * be;
            H[0][be] = g[0] * v[0] + g[1] * v[1] + g[2] * v[2];
            H[1][be] = g[1] * v[0] + g[3] * v[1] + g[4] * v[2];
            H[2][be] = g[2] * v[0] + g[4] * v[1] + g[5] * v[2];
        }
#pragma unroll
        for (int al = 0; al < 2; ++al)
#pragma unroll
            for (int be = 0; be < 2; ++be)
                acc[z][2 * al + be] = eif[3 * al] * H[0][be] + eif[3 * al + 1] * H[1][be] + eif[3 * al + 2] * H[2][be];
    }
}
// WMAX = 8 at 4 waves per SIMD (128 VGPRs, no scratch; 130 and 3 waves
// left to the compiler): 16.87 -> 16.48 ms per 1024-system launch (round 4,
// profiles/r04_ab/asm_w4/); WMAX = 16 spills at 4 and keeps its own choice.
// Measured and not kept: the next incidence's tinc / tslot loaded one
// iteration ahead (127 VGPRs, 2 spilled): 18.6-19.6 vs 16.5 ms
// (profiles/r04_ab/asm_pre/)
template <int WMAX>
__global__ __launch_bounds__(kWG) __attribute__((amdgpu_waves_per_eu(WMAX <= 8 ? 4 : 1))) void k_assemble_rows_rc(
    int32_t N, int32_t M, int32_t nblk, int32_t B, int64_t sell_nb, const int32_t *__restrict__ sell_off,
    const int32_t *__restrict__ sell_col, const int32_t *__restrict__ vptr, const int32_t *__restrict__ tsell_off,
    const int4 *__restrict__ tinc, const int32_t *__restrict__ tslot, const float *__restrict__ w12,
    const float *__restrict__ a2s, int block_jacobi, float *__restrict__ A, float *__restrict__ dinv32,
    double *__restrict__ rhs, uint2 *__restrict__ Ah, int32_t nown, const int32_t *__restrict__ mir, TriGeo geo) {
    int32_t rb, b;
    if (!xcd_map(nblk, B, rb, b, kGrpAsm)) return;
    const double *I0b = geo.J0 + (int64_t)b * N, *I1b = geo.J1 + (int64_t)b * N;
    const double hb = geo.dt[b];
#pragma unroll 1
    for (int r = 0; r < kRows; ++r) {
        const int32_t i = rb * kRowsPerWG + r * kWG + threadIdx.x;
        if (i >= N) break;
        const int32_t s = i >> 6, l = i & 63;
        float acc[WMAX][4];
        float G[WMAX][6];  // the slots' 3x3 a1 sums (symmetric: xx xy xz yy yz zz)
        double ei[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) ei[k] = geo.e[6 * (int64_t)i + k];
#pragma unroll
        for (int z = 0; z < WMAX; ++z)
#pragma unroll
            for (int x = 0; x < 6; ++x) G[z][x] = 0.f;
        double f0 = 0.0, f1 = 0.0;
        const double Ii0 = I0b[i], pdi = (I1b[i] - Ii0) / hb;
        const int32_t to = tsell_off[s], tw = (tsell_off[s + 1] - to) >> 6;
        for (int32_t t = 0; t < tw; ++t) {
            const int64_t e = (int64_t)to + (int64_t)t * kSlice + l;
            const int4 q = tinc[e];
            const int32_t sl = tslot[e];
            const bool real = q.x < M;  // padding (T = M): weight 0, no f term
            const int64_t T = min(q.x, M - 1);
            const int32_t c = q.y, vj = q.z, vk = q.w;
            double g[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) g[k] = geo.gw[9 * T + k];
            const double At = geo.area[T];
            const float wv = w12[q.x];
            const int32_t sj = sl & 0xff, sk = sl >> 8;
            // set(T) - {i} in corner order: at most 2 distinct other corners
            const bool hj = vj != i, hk = vk != i && vk != vj;
            const double aj = I0b[vj], ak = I0b[vk];
            const double pdj = (I1b[vj] - aj) / hb, pdk = (I1b[vk] - ak) / hb;
            // the triangle's I0 in its own corner order (corner c is i)
            const double c0 = c == 0 ? Ii0 : (c == 1 ? ak : aj);
            const double c1 = c == 0 ? aj : (c == 1 ? Ii0 : ak);
            const double c2 = c == 0 ? ak : (c == 1 ? aj : Ii0);
            double gI[3];
#pragma unroll
            for (int d = 0; d < 3; ++d) gI[d] = (c0 * g[d] + c1 * g[3 + d]) + c2 * g[6 + d];
            const double ui0 = dot64(gI, ei), ui1 = dot64(gI, ei + 3);
            const double po = hj ? (hk ? pdj + pdk : pdj) : (hk ? pdk : 0.0);
            if (real) {  // f in the reference's triangle order
                f0 += ui0 * (2 * pdi + po) * At / 12;
                f1 += ui1 * (2 * pdi + po) * At / 12;
            }
            // the a1 terms (compute_a1's (u_i^a u_j^b) w) as one outer product
            // of grad_M I per incidence, weighted per slot: A/6 = 2 A/12 on the
            // diagonal block (a degenerate triangle's second corner at i
            // included), A/12 on the blocks of the other two corners
            const float wd = wv + wv, wj = sj == 0 ? wd : wv, wk = sk == 0 ? wd : wv;
            const float gx = (float)gI[0], gy = (float)gI[1], gz = (float)gI[2];
            const float op[6] = {gx * gx, gx * gy, gx * gz, gy * gy, gy * gz, gz * gz};
#pragma unroll
            for (int z = 0; z < WMAX; ++z) {
                const float cz = (z == 0 ? wd : 0.f) + (z == sj ? wj : 0.f) + (z == sk ? wk : 0.f);
#pragma unroll
                for (int x = 0; x < 6; ++x) G[z][x] = __builtin_fmaf(cz, op[x], G[z][x]);
            }
        }
        g3_project<WMAX>(G, ei, vptr[i + 1] - vptr[i], sell_off[s] + l, sell_col, geo.e, mir, acc);
        rows_store<WMAX>(acc, f0, f1, i, b, N, vptr[i + 1] - vptr[i], sell_off[s] + l, sell_nb, sell_col, a2s,
                         block_jacobi, A, dinv32, rhs, Ah, nown, mir);
    }
}

__global__ __launch_bounds__(kWG) void k_scale_a2(int64_t n, double lambda,
                                                  const double *__restrict__ a2,
                                                  double *__restrict__ s64,
                                                  float *__restrict__ s32) {
    const int64_t q = (int64_t)blockIdx.x * kWG + threadIdx.x;
    if (q >= n) return;
    const double v = lambda * a2[q];
    s64[q] = v;
    s32[q] = (float)v;
}

// A_T / 12 per triangle (= integral_wi_wj[T][1]), slot M = 0.
__global__ __launch_bounds__(kWG) void k_w12(int32_t M, const double *__restrict__ iw,
                                             double *__restrict__ w64, float *__restrict__ w32) {
    const int32_t T = blockIdx.x * kWG + threadIdx.x;
    if (T > M) return;
    const double v = T < M ? iw[2 * (int64_t)T + 1] : 0.0;
    w64[T] = v;
    w32[T] = (float)v;
}

// Export path (mof_assemble): the reference's A = a1 + lambda*a2 of one
// timestep, one SELL position per thread, bit for bit (:127-146): block
// (i, j) of a1 = fold over its terms of (u_a^alpha u_b^beta) integral in
// triangle order; the diagonal-block thread also folds f_i.
__global__ __launch_bounds__(kWG) void k_assemble_export(
    int64_t sell_nb, int32_t N, int32_t M, const int32_t *__restrict__ sell_blk,
    const int32_t *__restrict__ blk_row, const int32_t *__restrict__ vcol,
    const int32_t *__restrict__ cptr, const int32_t *__restrict__ clist,
    const double *__restrict__ iw, const double *__restrict__ a2, const double *__restrict__ u,
    const double *__restrict__ fc, double lambda, double *__restrict__ A64,
    double *__restrict__ f) {
    const int64_t pos = (int64_t)blockIdx.x * kWG + threadIdx.x;
    if (pos >= sell_nb) return;
    const int32_t p = sell_blk[pos];
    if (p < 0) return;  // SELL padding stays zero
    const int32_t i = blk_row[p], j = vcol[p];
    const bool diag = (j == i);
    double f0 = 0.0, f1 = 0.0;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int32_t c = cptr[p]; c < cptr[p + 1]; ++c) {
        const int32_t code = clist[c];
        const int32_t T = code / 9, a = (code % 9) / 3, bb = code % 3;
        const double2 ua = *reinterpret_cast<const double2 *>(u + 6 * (int64_t)T + 2 * a);
        const double2 uv = *reinterpret_cast<const double2 *>(u + 6 * (int64_t)T + 2 * bb);
        const double integ = iw[2 * (int64_t)T + (diag ? 0 : 1)];
        acc[0] += ua.x * uv.x * integ;
        acc[1] += ua.x * uv.y * integ;
        acc[2] += ua.y * uv.x * integ;
        acc[3] += ua.y * uv.y * integ;
        if (diag && a == bb) {
            const double2 fv = *reinterpret_cast<const double2 *>(fc + 6 * (int64_t)T + 2 * a);
            f0 += fv.x;
            f1 += fv.y;
        }
    }
    const double2 s01 = *reinterpret_cast<const double2 *>(a2 + 4 * pos);
    const double2 s23 = *reinterpret_cast<const double2 *>(a2 + 4 * pos + 2);
    double *o64 = A64 + 4 * pos;
    *reinterpret_cast<double2 *>(o64) = make_double2(acc[0] + lambda * s01.x, acc[1] + lambda * s01.y);
    *reinterpret_cast<double2 *>(o64 + 2) = make_double2(acc[2] + lambda * s23.x, acc[3] + lambda * s23.y);
    if (diag) {
        f[i] = f0;
        f[N + i] = f1;
    }
}

// x64 (interleaved, internal order) -> V (B, 2N) planar in the caller's
// vertex order (one caller vertex per thread: gathered reads, coalesced
// writes); failed systems are NaN-filled.
__global__ __launch_bounds__(kWG) void k_to_planar(int32_t N, const double *__restrict__ x,
                                                   const int32_t *__restrict__ perm,
                                                   const int32_t *__restrict__ sysi,
                                                   double *__restrict__ V) {
    const int32_t o = blockIdx.x * kWG + threadIdx.x;
    const int32_t b = blockIdx.y;
    if (o >= N) return;
    const bool failed = sysi[b * kSysStride + SI_FAILED] != 0;
    const double2 v = *reinterpret_cast<const double2 *>(x + 2 * ((int64_t)b * N + perm[o]));
    const double nan = __builtin_nan("");
    V[(int64_t)b * 2 * N + o] = failed ? nan : v.x;
    V[(int64_t)b * 2 * N + N + o] = failed ? nan : v.y;
}

// S3's epilogue (find_singularity_point.py:28-69, S3…py:130-132): the 3-D
// tangent vector V^0 e^0 + V^1 e^1 of every vertex and its length, with
// numpy's roundings (products, then sums; |v| = sqrt((x^2 + y^2) + z^2)).
constexpr int kVVFields = 4;  // fields per thread: e_i loaded once for all of them

__global__ __launch_bounds__(kWG) void k_velocity_vectors(int32_t N, int32_t K, const double *__restrict__ e,
                                                          const double *__restrict__ V,
                                                          double *__restrict__ Vc,
                                                          double *__restrict__ speed) {
    // vertex i of fields kVVFields*blockIdx.y + f; the (N,3) output of the
    // workgroup's 256 vertices is staged in LDS and stored as 16-B chunks
    __shared__ double st[3 * kWG];
    const int32_t i0 = blockIdx.x * kWG;
    const int32_t i = i0 + threadIdx.x;
    double ei[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    if (i < N) {
#pragma unroll
        for (int d = 0; d < 6; ++d) ei[d] = e[6 * (int64_t)i + d];
    }
    const int32_t nv = min(kWG, N - i0);
    for (int f = 0; f < kVVFields; ++f) {
        const int64_t k = (int64_t)blockIdx.y * kVVFields + f;
        if (k >= K) break;
        double c[3] = {0.0, 0.0, 0.0};
        if (i < N) {
            const double v0 = V[2 * k * N + i], v1 = V[2 * k * N + N + i];
#pragma unroll
            for (int d = 0; d < 3; ++d) c[d] = v0 * ei[d] + v1 * ei[3 + d];
            if (speed) speed[k * N + i] = sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
        }
        if (!Vc) continue;
        __syncthreads();  // st reuse across fields
#pragma unroll
        for (int d = 0; d < 3; ++d) st[3 * threadIdx.x + d] = c[d];
        __syncthreads();
        double *out = Vc + 3 * (k * N + i0);
        if (((3 * (k * N + i0)) & 1) == 0) {  // 16-B aligned
            for (int32_t q = threadIdx.x; 2 * q + 1 < 3 * nv; q += kWG)
                reinterpret_cast<double2 *>(out)[q] = make_double2(st[2 * q], st[2 * q + 1]);
            if (((3 * nv) & 1) && threadIdx.x == 0) out[3 * nv - 1] = st[3 * nv - 1];
        } else {
            for (int32_t q = threadIdx.x; q < 3 * nv; q += kWG) out[q] = st[q];
        }
    }
}

// Recovery solve after a multigrid solve failed: the 2x2 block-Jacobi
// inverses of the fp32 A (that assembly kept D^-1 only in bf16).
__global__ __launch_bounds__(kWG) void k_dinv_from_A32(int32_t N, int64_t sell_nb, const int32_t *__restrict__ diag_pos,
                                                       const float *__restrict__ A, float *__restrict__ dinv32) {
    const int32_t i = blockIdx.x * kWG + threadIdx.x;
    const int32_t b = blockIdx.y;
    if (i >= N) return;
    const float4 d = reinterpret_cast<const float4 *>(A)[(int64_t)b * sell_nb + diag_pos[i]];
    const double d0 = d.x, d1 = d.y, d2 = d.z, d3 = d.w;
    const double det = d0 * d3 - d1 * d2;
    reinterpret_cast<float4 *>(dinv32)[(int64_t)b * N + i] =
        make_float4((float)(d3 / det), (float)(-d1 / det), (float)(-d2 / det), (float)(d0 / det));
}

inline dim3 grid1(int64_t n) { return dim3((unsigned)((n + kWG - 1) / kWG)); }

// Host-side guard before any launch: every device array a kernel indexes is
// allocated with the size the pattern implies (a missing upload would
// otherwise surface as a GPU memory fault).
void check_mesh_arrays(const mof_mesh *m) {
    const Pattern &P = m->pat;
    const size_t N = m->N, M = m->M;
    auto ok = [](const auto &d, size_t n) { return d.p != nullptr && d.n >= n; };
    MOF_REQUIRE(ok(m->tri, 3 * M) && ok(m->tri_orig, 3 * M) && ok(m->perm_d, N) && ok(m->area, M),
                "mesh arrays not uploaded");
    MOF_REQUIRE(ok(m->vptr, N + 1) && ok(m->vcol, P.vcol.size()) && ok(m->cptr, P.cptr.size()) &&
                    ok(m->clist, P.clist.size()) && ok(m->sell_off, P.sell_off.size()) &&
                    ok(m->sell_col, (size_t)P.sell_nb()) && ok(m->sell_blk, (size_t)P.sell_nb()) &&
                    ok(m->blk_row, P.blk_row.size()) && ok(m->diag_pos, N) &&
                    ok(m->tsell_off, P.tsell_off.size()) && ok(m->tinc, 4 * (size_t)P.tsell_nb()) &&
                    ok(m->tslot, (size_t)P.tsell_nb()),
                "pattern arrays not uploaded");
    MOF_REQUIRE(ok(m->e, 6 * N) && ok(m->gw, 9 * M) && ok(m->iw, 2 * M) &&
                    ok(m->a2, 4 * (size_t)P.sell_nb()) && ok(m->w12_64, M + 1) && ok(m->w12_32, M + 1),
                "geometry arrays not allocated");
}

}  // namespace

void launch_geometry(mof_mesh *m, const double *d_xyz, const double *d_nrm, bool f32_points) {
    check_mesh_arrays(m);
    MOF_REQUIRE(d_xyz && d_nrm, "NULL coordinates");
    hipStream_t s = m->stream;
    k_basis<<<grid1(m->N), kWG, 0, s>>>(d_nrm, m->N, m->e.p);
    if (f32_points)
        k_gradw<true><<<grid1(m->M), kWG, 0, s>>>(d_xyz, m->tri.p, m->area.p, m->M, m->gw.p, m->iw.p);
    else
        k_gradw<false><<<grid1(m->M), kWG, 0, s>>>(d_xyz, m->tri.p, m->area.p, m->M, m->gw.p, m->iw.p);
    k_w12<<<grid1(m->M + 1), kWG, 0, s>>>(m->M, m->iw.p, m->w12_64.p, m->w12_32.p);
    MOF_HIP(hipGetLastError());
}

void launch_a2(mof_mesh *m) {
    k_a2<<<grid1(m->N), kWG, 0, m->stream>>>(m->N, m->vptr.p, m->vcol.p, m->cptr.p, m->clist.p,
                                             m->sell_off.p, m->e.p, m->gw.p, m->area.p, m->a2.p);
    MOF_HIP(hipGetLastError());
}

void prepare_operator(mof_mesh *m, double lambda, hipStream_t s) {
    if (m->a2s_valid && m->a2s_lambda == lambda) return;
    const int64_t n = 4 * m->pat.sell_nb();
    k_scale_a2<<<grid1(n), kWG, 0, s>>>(n, lambda, m->a2.p, m->a2s64.p, m->a2s32.p);
    MOF_HIP(hipGetLastError());
    m->a2s_lambda = lambda;
    m->a2s_valid = true;
}

// The batch's I rows in the internal vertex order, so that k_tri_step's
// gathers of the three corners of consecutive triangles hit the same cache
// lines (in the caller's order they scatter over the row: 3835 -> 3013 us per
// 256-system k_tri_step on C3, 5151 -> 2979 us with a random vertex order).
// One XCD per row (workgroup w runs on XCD w mod 8): the row's gathers stay
// in that XCD's L2. Row r < R0 comes from I0 + r ldI, the others from I1.
__global__ __launch_bounds__(kWG) void k_gather_I(int32_t N, int32_t R, int32_t R0, const double *__restrict__ I0,
                                                  const double *__restrict__ I1, int64_t ldI,
                                                  const int32_t *__restrict__ icol, double *__restrict__ out) {
    const int32_t w = blockIdx.x, q = w >> 3;
    const int32_t nbi = (N + kWG - 1) / kWG;
    const int32_t r = (w & 7) + 8 * (q / nbi);
    const int32_t i = (q % nbi) * kWG + threadIdx.x;
    if (r >= R || i >= N) return;
    const double *src = r < R0 ? I0 + r * ldI : I1 + (int64_t)(r - R0) * ldI;
    out[(int64_t)r * N + i] = src[icol[i]];
}

// The per-triangle term arrays ([cap][M+1][6]: u64, the fp32 u32, the f
// terms fc; triangle slot M stays zero, the incidence lists' padding) only
// the per-triangle paths use -- the fp64 solve, the mixed path on meshes too
// wide for the row assembly, the fp64 recovery and mof_assemble -- so they
// are allocated on first use at the workspace capacity (20 GB at C3, B = 512,
// that the row-assembly path never touches).
static void ensure_tri_terms(mof_mesh *m, bool u64, bool u32, hipStream_t s) {
    Workspace &w = m->ws;
    const size_t n = 6 * ((size_t)m->M + 1) * std::max(w.cap, 1);
    auto need = [&](auto &arr) {
        if (arr.n < n) {
            arr.alloc(n);
            arr.zero(s);
        }
    };
    need(w.fc);
    if (u64) need(w.u64);
    if (u32) need(w.u32);
}

// After a mixed solve's fp64 recovery: the fp64 A and the per-triangle term
// arrays it allocated at the workspace capacity (≈8 GB each at C3, B = 512)
// go back, so the row-assembly path keeps its headroom (the residual re-forms
// u when u64 is absent).
void release_f64_terms(mof_mesh *m) {
    Workspace &w = m->ws;
    w.A64.release();
    w.u64.release();
    w.u32.release();
    w.fc.release();
    w.u64_stale = false;
}

void launch_assemble(mof_mesh *m, int32_t B, const double *I0, const double *I1, int64_t ldI,
                     bool block_jacobi, uint32_t precision, hipStream_t s, bool amg) {
    Workspace &w = m->ws;
    check_mesh_arrays(m);
    const size_t nbs = (size_t)m->pat.sell_nb();
    MOF_REQUIRE(B >= 1 && B <= w.cap && I0 && I1 && w.dt.n >= (size_t)B && m->a2s_valid,
                "assembly workspace / operator not prepared");
    MOF_REQUIRE(precision == MOF_PREC_MIXED ? w.A32.n >= 4 * nbs * B : w.A64.n >= 4 * nbs * B,
                "assembly target A not allocated");
    MOF_REQUIRE(ldI >= 1 && m->icol.n >= (size_t)m->N && w.Iint.n >= 2 * (size_t)m->N * B,
                "I permutation buffers not prepared");
    {
        // consecutive timesteps of one array share B-1 rows: B+1 rows then
        const bool shared = I1 == I0 + ldI;
        const int32_t R = shared ? B + 1 : 2 * B, R0 = shared ? R : B;
        const int32_t nbi = (m->N + kWG - 1) / kWG;
        k_gather_I<<<dim3((unsigned)(8 * ((R + 7) / 8) * nbi)), kWG, 0, s>>>(m->N, R, R0, I0, I1, ldI, m->icol.p,
                                                                            w.Iint.p);
    }
    const double *J0 = w.Iint.p, *J1 = w.Iint.p + (I1 == I0 + ldI ? (int64_t)m->N : (int64_t)m->N * B);
    dim3 gt((unsigned)((m->M + kWG - 1) / kWG));
    // row assembly (forming the triangle terms itself) when the widest row
    // fits the register accumulators; otherwise k_tri_step + the per-block
    // kernels (and the fp64 path)
    const int32_t W = m->pat.max_w;
    const bool rows = precision == MOF_PREC_MIXED && W <= 16;
    const bool skip_u64 = precision == MOF_PREC_MIXED;  // the residual re-forms u from the I rows
    if (!rows) ensure_tri_terms(m, !skip_u64, precision == MOF_PREC_MIXED, s);
    if (!rows)
        k_tri_step<<<gt, kWG, 0, s>>>(m->M, B, m->tri.p, m->tri.p, m->gw.p, m->e.p, m->area.p, J0, J1, m->N, w.dt.p,
                                      skip_u64 ? nullptr : w.u64.p, w.fc.p,
                                      precision == MOF_PREC_MIXED ? w.u32.p : nullptr);
    w.u64_stale = skip_u64;  // u64 (and with the row assembly fc) re-formed by the fp64 recovery if needed
    w.J0 = J0;
    w.J1 = J1;
    w.JB = B;
    const TriGeo geo{m->gw.p, m->e.p, m->area.p, J0, J1, w.dt.p};
    const int64_t snb = m->pat.sell_nb();
    const dim3 gb(xcd_grid((int32_t)((snb + kWG - 1) / kWG), B, kGrpAsm));
    const int bj = block_jacobi ? 1 : 0;
    // multigrid: the level-0 smoother's bf16 operator comes from here
    AmgBf16 bf{nullptr};
    if (amg && precision == MOF_PREC_MIXED) bf = amg_bf16_targets(m, B);
    const int32_t nblk_rows = (int32_t)((m->N + kRowsPerWG - 1) / kRowsPerWG);
    const int32_t *mirw = m->sym_reads ? m->sell_mir.p : nullptr;
#define MOF_ASM_RC_LAUNCH(WM)                                                                                     \
    k_assemble_rows_rc<WM><<<xcd_grid(nblk_rows, B, kGrpAsm), kWG, 0, s>>>(                                        \
        m->N, m->M, nblk_rows, B, snb, m->sell_off.p, m->sell_col.p, m->vptr.p, m->tsell_off.p,                    \
        reinterpret_cast<const int4 *>(m->tinc.p), m->tslot.p, m->w12_32.p, m->a2s32.p, bj, w.A32.p, w.dinv32.p,   \
        w.rhs.p, bf.A0h, m->n_own, mirw, geo)
    if (rows && W <= 8)
        MOF_ASM_RC_LAUNCH(8);
    else if (rows)
        MOF_ASM_RC_LAUNCH(16);
#undef MOF_ASM_RC_LAUNCH
    else if (precision == MOF_PREC_MIXED)
        k_assemble_mixed<<<gb, kWG, 0, s>>>(snb, m->N, m->M, B, m->sell_blk.p, m->blk_row.p, m->vcol.p,
                                            m->cptr.p, m->clist.p, m->w12_32.p, m->a2s32.p, w.u32.p,
                                            w.fc.p, bj, w.A32.p, w.dinv32.p, w.rhs.p, bf.A0h, m->n_own);
    else
        k_assemble_blocks<double><<<gb, kWG, 0, s>>>(snb, m->N, m->M, B, m->sell_blk.p, m->blk_row.p,
                                                     m->vcol.p, m->cptr.p, m->clist.p, m->iw.p,
                                                     m->a2s64.p, w.u64.p, w.fc.p, bj, w.A64.p,
                                                     w.dinv64.p, w.dinv32.p, w.rhs.p);
    MOF_HIP(hipGetLastError());
}

void launch_recovery_operator(mof_mesh *m, int32_t B, uint32_t precision, hipStream_t s) {
    Workspace &w = m->ws;
    check_mesh_arrays(m);
    const int64_t snb = m->pat.sell_nb();
    MOF_REQUIRE(B >= 1 && B <= w.cap && m->a2s_valid, "recovery: workspace / operator not prepared");
    if (precision == MOF_PREC_MIXED) {
        MOF_REQUIRE(w.A32.n >= 4 * (size_t)snb * B && w.dinv32.n >= 4 * (size_t)m->N * B,
                    "recovery: fp32 A not assembled");
        k_dinv_from_A32<<<dim3((unsigned)((m->N + kWG - 1) / kWG), (unsigned)B), kWG, 0, s>>>(
            m->N, snb, m->diag_pos.p, w.A32.p, w.dinv32.p);
    } else {
        MOF_REQUIRE(w.A64.n >= 4 * (size_t)snb * B, "recovery: fp64 A not allocated");
        ensure_tri_terms(m, true, false, s);
        if (w.u64_stale) {  // the batch's u64 was never stored: form it from the same I rows
            MOF_REQUIRE(w.J0 && w.J1 && w.JB >= B, "recovery: the batch's I rows are gone");
            k_tri_step<<<dim3((unsigned)((m->M + kWG - 1) / kWG)), kWG, 0, s>>>(
                m->M, B, m->tri.p, m->tri.p, m->gw.p, m->e.p, m->area.p, w.J0, w.J1, m->N, w.dt.p, w.u64.p, w.fc.p,
                nullptr);
            w.u64_stale = false;
        }
        const dim3 gb(xcd_grid((int32_t)((snb + kWG - 1) / kWG), B, kGrpAsm));
        k_assemble_blocks<double><<<gb, kWG, 0, s>>>(snb, m->N, m->M, B, m->sell_blk.p, m->blk_row.p, m->vcol.p,
                                                     m->cptr.p, m->clist.p, m->iw.p, m->a2s64.p, w.u64.p, w.fc.p,
                                                     1, w.A64.p, w.dinv64.p, w.dinv32.p, w.rhs.p);
    }
    MOF_HIP(hipGetLastError());
}

void launch_assemble_export(mof_mesh *m, const double *I0, const double *I1, double lambda,
                            hipStream_t s) {
    Workspace &w = m->ws;
    ensure_tri_terms(m, true, false, s);
    dim3 gt((unsigned)((m->M + kWG - 1) / kWG), 1u);
    k_tri_step<<<gt, kWG, 0, s>>>(m->M, 1, m->tri.p, m->tri_orig.p, m->gw.p, m->e.p, m->area.p, I0, I1, 0, w.dt.p,
                                  w.u64.p, w.fc.p, nullptr);
    const int64_t snb = m->pat.sell_nb();
    k_assemble_export<<<grid1(snb), kWG, 0, s>>>(snb, m->N, m->M, m->sell_blk.p, m->blk_row.p,
                                                 m->vcol.p, m->cptr.p, m->clist.p, m->iw.p, m->a2.p,
                                                 w.u64.p, w.fc.p, lambda, m->Aexp.p, m->fexp.p);
    MOF_HIP(hipGetLastError());
}

void launch_velocity_vectors(int32_t N, int32_t K, const double *e, const double *V, double *Vc,
                             double *speed, hipStream_t s) {
    const int64_t total = (int64_t)N * K;
    if (total == 0) return;
    const int64_t step = 65535LL * kVVFields;  // grid.y limit
    for (int64_t k0 = 0; k0 < K; k0 += step) {
        const int32_t kn = (int32_t)std::min<int64_t>(step, K - k0);
        k_velocity_vectors<<<dim3((unsigned)((N + kWG - 1) / kWG), (unsigned)((kn + kVVFields - 1) / kVVFields)),
                             kWG, 0, s>>>(N, kn, e, V + 2 * k0 * N, Vc ? Vc + 3 * k0 * N : nullptr,
                                          speed ? speed + k0 * N : nullptr);
    }
    MOF_HIP(hipGetLastError());
}

void launch_to_planar(mof_mesh *m, int32_t B, double *V, hipStream_t s) {
    dim3 g((unsigned)((m->N + kWG - 1) / kWG), (unsigned)B);
    k_to_planar<<<g, kWG, 0, s>>>(m->N, m->ws.x64.p, m->perm_d.p, m->ws.sysi.p, V);
    MOF_HIP(hipGetLastError());
}

}  // namespace mof
