// mof_amg.hip -- aggregation multigrid V-cycle on gfx950 (inner-PCG preconditioner).
//
// Per batch of B systems (timesteps) the mesh-only hierarchy of
// mof_amg_host.cpp gets its per-timestep values:
//   k_galerkin0_ns /   A_{l+1} = Q^T A_l Q, one coarse block of 4 systems per
//   k_galerkin3_ns     thread, folded over the pre-built gather lists (no
//                      atomics), plus the 3x3 block-Jacobi inverse of each
//                      coarse node;
//   k_coarse_inverse   the coarsest operator (<= 128 dofs) inverted by the
//                      symmetric sweep operator in registers (fp64, one
//                      workgroup per system).
// Each PCG iteration applies one symmetric V(1,1)-cycle to the residual r
// (damped block Jacobi: w = 0.85 on level 0, w1 = 1.05 on the coarse levels):
//   level 0 pre-smooth x0 = w D^-1 r is fused into k_pcg_update / k_pcg_init;
//   per level l:  k_res0 / k_res3  r_l = b_l - A_l x_l, written in member
//                                  order of the next level's aggregates
//                 k_restrict       b_{l+1} = Q^T r_l (contiguous members),
//                                  x_{l+1} = w1 D^-1 b_{l+1} (next pre-smooth)
//   levels with <= kSubNodes nodes and the coarsest solve y = A_c^-1 b run in
//   one launch (k_subcycle, one workgroup per system);
//   per level l:  k_prolong0 / k_prolong  x_l += Q y_{l+1}
//                 k_post0 / k_post3  y_l = x_l + w D^-1 (b_l - A_l x_l); at
//                                  level 0 y = z and the partial r.z of the PCG
// Every launch covers all B systems and skips retired systems. Level 0 sweeps
// a bf16 copy of the inner solver's SELL A (its diagonal blocks give the
// smoother's D), written by the assembly, in the PCG row-kernel layout (XCD-aware,
// batched loads); coarse levels keep fp32 3x3 blocks (12 floats, rows padded
// to 4) for the Galerkin products and int8 copies (9 codes + a bf16 scale,
// 12 B per block, st_a9) for the sweeps, vectors
// as float4. All sums run in a fixed order: the cycle is
// deterministic and independent of B.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "mof_amg.h"
#include "mof_rowkern.h"

namespace mof {
namespace {

constexpr int kB3 = 12;  // floats per coarse 3x3 block / per coarse D^-1

__device__ __forceinline__ bool retired(const int32_t *sysi, int32_t b) {
    return !sysi[b * kSysStride + SI_ACTIVE] || sysi[b * kSysStride + SI_CONV] >= 0;
}

// per-node vector: BS = 2 -> float2 (stride 2), BS = 3 -> float4 (stride 4)
template <int BS>
__device__ __forceinline__ void ldv(const float *v, int64_t node, float (&x)[BS]) {
    if constexpr (BS == 2) {
        const float2 t = reinterpret_cast<const float2 *>(v)[node];
        x[0] = t.x; x[1] = t.y;
    } else {
        const float4 t = reinterpret_cast<const float4 *>(v)[node];
        x[0] = t.x; x[1] = t.y; x[2] = t.z;
    }
}
// the restricted residual of level BSF: level 0 keeps it as a bf16 pair
// (4 B per vertex, written once by k_res0 and read once by the restriction)
template <int BSF>
__device__ __forceinline__ void ldr(const float *r, int64_t b, int64_t n, int64_t q, float (&x)[BSF]) {
    if constexpr (BSF == 2) {
        const uint32_t h = reinterpret_cast<const uint32_t *>(r)[b * n + q];
        x[0] = bf16_lo(h);
        x[1] = bf16_hi(h);
    } else {
        ldv<BSF>(r + b * n * 4, q, x);
    }
}
template <int BS>
__device__ __forceinline__ void stv(float *v, int64_t node, const float (&x)[BS]) {
    if constexpr (BS == 2)
        reinterpret_cast<float2 *>(v)[node] = make_float2(x[0], x[1]);
    else
        reinterpret_cast<float4 *>(v)[node] = make_float4(x[0], x[1], x[2], 0.f);
}
// BS x BS block: BS = 2 -> 4 floats, BS = 3 -> 12 floats (rows padded to 4)
template <int BS>
__device__ __forceinline__ void ldm(const float *A, int64_t idx, float (&a)[BS][BS]) {
    if constexpr (BS == 2) {
        const float4 t = reinterpret_cast<const float4 *>(A)[idx];
        a[0][0] = t.x; a[0][1] = t.y; a[1][0] = t.z; a[1][1] = t.w;
    } else {
        const float4 *p = reinterpret_cast<const float4 *>(A) + 3 * idx;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const float4 t = p[r];
            a[r][0] = t.x; a[r][1] = t.y; a[r][2] = t.z;
        }
    }
}
template <int BS>
constexpr int vstride() { return BS == 2 ? 2 : 4; }
template <int BS>
constexpr int bstride() { return BS == 2 ? 4 : kB3; }

template <int BS>
__device__ __forceinline__ void matvec(const float (&a)[BS][BS], const float (&x)[BS], float (&y)[BS]) {
#pragma unroll
    for (int r = 0; r < BS; ++r) {
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < BS; ++c) s += a[r][c] * x[c];
        y[r] = s;
    }
}

// 3x3 inverse by cofactors (fp64 inside)
__device__ void inv3(const float (&a)[3][3], float (&o)[3][3]) {
    const double a00 = a[0][0], a01 = a[0][1], a02 = a[0][2], a10 = a[1][0], a11 = a[1][1],
                 a12 = a[1][2], a20 = a[2][0], a21 = a[2][1], a22 = a[2][2];
    const double c00 = a11 * a22 - a12 * a21, c01 = a12 * a20 - a10 * a22, c02 = a10 * a21 - a11 * a20;
    const double det = a00 * c00 + a01 * c01 + a02 * c02;
    const double id = det != 0.0 ? 1.0 / det : 0.0;
    o[0][0] = (float)(c00 * id);
    o[0][1] = (float)((a02 * a21 - a01 * a22) * id);
    o[0][2] = (float)((a01 * a12 - a02 * a11) * id);
    o[1][0] = (float)(c01 * id);
    o[1][1] = (float)((a00 * a22 - a02 * a20) * id);
    o[1][2] = (float)((a02 * a10 - a00 * a12) * id);
    o[2][0] = (float)(c02 * id);
    o[2][1] = (float)((a01 * a20 - a00 * a21) * id);
    o[2][2] = (float)((a00 * a11 - a01 * a10) * id);
}

__device__ __forceinline__ void st3(float *A, int64_t idx, const float (&a)[3][3]) {
    float4 *p = reinterpret_cast<float4 *>(A) + 3 * idx;
#pragma unroll
    for (int r = 0; r < 3; ++r) p[r] = make_float4(a[r][0], a[r][1], a[r][2], 0.f);
}

__device__ __forceinline__ void st_h9(uint4 *H, uint16_t *H22, int64_t q, const float (&c)[3][3]) {
    H[q] = make_uint4(bf16_bits(c[0][0]) | (bf16_bits(c[0][1]) << 16), bf16_bits(c[0][2]) | (bf16_bits(c[1][0]) << 16),
                      bf16_bits(c[1][1]) | (bf16_bits(c[1][2]) << 16), bf16_bits(c[2][0]) | (bf16_bits(c[2][1]) << 16));
    H22[q] = (uint16_t)bf16_bits(c[2][2]);
}

// The coarse levels' sweep copy of A (levels >= 1 except the coarsest):
// 12 B per 3x3 block, the 9 entries as offset-binary int8 (q + 128) with one
// bf16 scale per block (s = max |a| / 127): H viewed as uint2[] (entries
// 0..7), H22 as uint32_t[] (entry 8 | scale << 16). A block and its
// transposed twin have the same entries, so the same scale and the same
// codes: the preconditioner stays symmetric (round 2: 18 B bf16 entries
// before, level-1 k_res3 / k_post3 442 / 430 -> 360 / 337 us, C3 +1.6 %).
// uint32 words of Ah and uint16 words of Ah22 per block
constexpr size_t kAhWords = 2, kAh22Words = 2;

__device__ __forceinline__ void st_a9(uint4 *H, uint16_t *H22, int64_t q, const float (&c)[3][3]) {
    {
        float m = 0.f;
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int k = 0; k < 3; ++k) m = fmaxf(m, fabsf(c[r][k]));
        const uint32_t sb = bf16_bits(m / 127.f);
        const float sc = bf16_lo(sb);
        uint32_t u[9];
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const float v = sc > 0.f ? rintf(c[r][k] / sc) : 0.f;
                u[3 * r + k] = (uint32_t)(fminf(fmaxf(v, -127.f), 127.f) + 128.f);
            }
        reinterpret_cast<uint2 *>(H)[q] =
            make_uint2(u[0] | (u[1] << 8) | (u[2] << 16) | (u[3] << 24), u[4] | (u[5] << 8) | (u[6] << 16) | (u[7] << 24));
        reinterpret_cast<uint32_t *>(H22)[q] = u[8] | (sb << 16);
    }
}
// A product's block C at position pos of system b and, for an upper block
// (tw >= 0: its lower twin's position, AmgLevel::twin), C^T at the twin: the
// products cover the diagonal and upper blocks only (round 6), and the
// coarse operator is symmetric to the bit
__device__ __forceinline__ void st_pair(float *__restrict__ Ac, uint4 *__restrict__ Ah, uint16_t *__restrict__ Ah22,
                                        int64_t b, int64_t c_sell_nb, int64_t pos, int32_t tw,
                                        const float (&C)[3][3]) {
    st3(Ac, b * c_sell_nb + pos, C);
    if (Ah) st_a9(Ah, Ah22, b * c_sell_nb + pos, C);
    if (tw >= 0) {
        float T[3][3];
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) T[r][c] = C[c][r];
        st3(Ac, b * c_sell_nb + tw, T);
        if (Ah) st_a9(Ah, Ah22, b * c_sell_nb + tw, T);
    }
}

// ---- per-timestep setup --------------------------------------------------

// A32 -> the level-0 sweep copy (h0_st)
__global__ __launch_bounds__(kWG) void k_to_h0(int64_t n, const float4 *__restrict__ A, uint2 *__restrict__ H) {
    const int64_t q = (int64_t)blockIdx.x * kWG + threadIdx.x;
    if (q >= n) return;
    const float4 v = A[q];
    h0_st(H, q, v.x, v.y, v.z, v.w);
}

// Level 0's Galerkin product with kNS systems per thread: the gather entry
// (fine position, P blocks of i and j) and both P blocks are loaded once and
// applied to the fine blocks of every system (level 0 has 7.5x the entries
// with a smoothed prolongator). Fine blocks from the smoother's bf16 copy
// (Afh) or the fp32 A (Af), folded per system in list order.
// Systems per thread: C3 (512 systems) 6.08 ms per launch at 4, 8.06 at 8,
// 14.7 at 16 (the per-system fine-block gathers, not the shared gather
// lists, bound it; more systems per thread only lower the occupancy); one
// system per thread (k_galerkin<2>): 9.02 ms.
// The system quads of a coarse tile run back to back on an XCD in groups of
// kGrpGal (8 quads = 32 systems); 2 quads per group (fewer systems' fine
// blocks in flight per tile) measured slower: C3 3424-3428 vs 3443-3446
// timesteps/s (round 3, profiles/r03_ab/gal2_*).
constexpr int kGalNS = 4;
__global__ __launch_bounds__(kWG) void k_galerkin0_ns(
    int64_t c_sell_nb, int32_t nC, int32_t B, const int32_t *__restrict__ c_sell_row,
    const int32_t *__restrict__ c_diag, const uint8_t *__restrict__ c_dead, const int32_t *__restrict__ c_twin,
    const int32_t *__restrict__ gptr, const int32_t *__restrict__ gent, const float *__restrict__ Q,
    const float *__restrict__ Af, int64_t f_sell_nb, float *__restrict__ Ac, uint4 *__restrict__ Dh,
    uint16_t *__restrict__ Dh22, uint4 *__restrict__ Ah, uint16_t *__restrict__ Ah22,
    const uint2 *__restrict__ Afh) {
    // no fp contraction: every system slot of the unrolled loops rounds alike
    // (a system's bits must not depend on its slot, i.e. on the batch split)
#pragma clang fp contract(off)
    int32_t tile, bq;
    const int32_t nq = (B + kGalNS - 1) / kGalNS;
    if (!xcd_map((int32_t)((c_sell_nb + kWG - 1) / kWG), nq, tile, bq, kGrpGal)) return;
    const int64_t pos = (int64_t)tile * kWG + threadIdx.x;
    if (pos >= c_sell_nb) return;
    const int32_t I = c_sell_row[pos];
    if (I >= nC) return;
    const int32_t b0 = bq * kGalNS;
    float Cm[kGalNS][3][3] = {};
    const int32_t g0 = gptr[pos], g1 = gptr[pos + 1];
    if (g0 == g1 && pos != c_diag[I]) return;  // a lower block (its upper twin writes it, st_pair) or padding
    // one gather entry per load batch (92 VGPRs, 5 waves per SIMD) instead
    // of 2 (140, 3 waves): 6.37 -> 5.92 ms per launch (round 3)
    constexpr int U = 1;
    for (int32_t t0 = g0; t0 < g1; t0 += U) {
        int32_t fp[U], ii[U], jj[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t g = min(t0 + u, g1 - 1);
            fp[u] = gent[3 * g];
            ii[u] = gent[3 * g + 1];
            jj[u] = gent[3 * g + 2];
        }
        float qi[U][6], qj[U][6], a[U][kGalNS][4];
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                qi[u][k] = Q[(int64_t)ii[u] * 6 + k];
                qj[u][k] = Q[(int64_t)jj[u] * 6 + k];
            }
            const int32_t fq = fp[u] < 0 ? 0 : fp[u] & kMirPos;
            const bool tr = fp[u] >= 0 && (fp[u] & kMirT);  // transposed upper block
#pragma unroll
            for (int t = 0; t < kGalNS; ++t) {
                const int64_t bb = min(b0 + t, B - 1);
                if (Afh) {
                    h0_dec(h0_ld(Afh, bb * f_sell_nb + fq), a[u][t][0], a[u][t][1], a[u][t][2], a[u][t][3]);
                } else {
                    const float4 v = reinterpret_cast<const float4 *>(Af)[bb * f_sell_nb + fq];
                    a[u][t][0] = v.x; a[u][t][1] = v.y; a[u][t][2] = v.z; a[u][t][3] = v.w;
                }
                if (tr) {
                    const float t01 = a[u][t][1];
                    a[u][t][1] = a[u][t][2];
                    a[u][t][2] = t01;
                }
                if (fp[u] < 0) {  // a decomposed part's ghost block: identity / zero
                    const float d = fp[u] == -1 ? 1.f : 0.f;
                    a[u][t][0] = d; a[u][t][1] = 0.f; a[u][t][2] = 0.f; a[u][t][3] = d;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float on = t0 + u < g1 ? 1.f : 0.f;
#pragma unroll
            for (int t = 0; t < kGalNS; ++t) {
                float T[2][3];  // A Q_j
#pragma unroll
                for (int r = 0; r < 2; ++r)
#pragma unroll
                    for (int c = 0; c < 3; ++c)
                        T[r][c] = on * (a[u][t][2 * r] * qj[u][c] + a[u][t][2 * r + 1] * qj[u][3 + c]);
#pragma unroll
                for (int r = 0; r < 3; ++r)
#pragma unroll
                    for (int c = 0; c < 3; ++c) Cm[t][r][c] += qi[u][r] * T[0][c] + qi[u][3 + r] * T[1][c];
            }
        }
    }
#pragma unroll
    for (int t = 0; t < kGalNS; ++t) {
        const int32_t b = b0 + t;
        if (b >= B) continue;
        if (pos == c_diag[I]) {
#pragma unroll
            for (int d = 0; d < 3; ++d)
                if (c_dead[3 * (int64_t)I + d]) Cm[t][d][d] += 1.f;
            float D[3][3];
            inv3(Cm[t], D);
            st_h9(Dh, Dh22, (int64_t)b * nC + I, D);
        }
        st_pair(Ac, Ah, Ah22, b, c_sell_nb, pos, c_twin[pos], Cm[t]);
    }
}

// Level 0's Galerkin product by gather entry (tentative prolongator): a
// workgroup takes a range of coarse positions with at most kWG gather
// entries in total (ggrp, built on the host), one entry per thread for
// kGalNS systems -- the entry and its two Q rows loaded once, every fine block
// of the systems gathered at once -- stages each term Q_i^T A_ij Q_j in LDS,
// then one thread per (coarse position, system) sums its terms in list order.
// The same terms in the same order as k_galerkin0_ns (bit-identical), with
// two dependent loads per thread instead of two per entry of a position.
// Systems per workgroup (C3, 512 systems, one box, round 3: 4 -> 5288 us per
// launch, 4 with the first task's position data loaded beside the entry
// 4978, 2 4670-4735, 1 5613, 8 6271; the old per-position kernel 5952, its
// reads 32.5 -> 4.35 GB per launch). Spreading the sums over the 9 block
// entries (every thread busy, a second barrier) took 9376 us.
constexpr int kGalENS = 2;
__global__ __launch_bounds__(kWG) void k_galerkin0_ent(
    int32_t ngrp, const int32_t *__restrict__ ggrp, int32_t nC, int32_t B, const int32_t *__restrict__ c_sell_row,
    const int32_t *__restrict__ c_diag, const uint8_t *__restrict__ c_dead, const int32_t *__restrict__ c_twin, const int32_t *__restrict__ gptr,
    const int32_t *__restrict__ gent, const float *__restrict__ Q, const uint2 *__restrict__ Afh,
    int64_t f_sell_nb, int64_t c_sell_nb, float *__restrict__ Ac, uint4 *__restrict__ Dh,
    uint16_t *__restrict__ Dh22, uint4 *__restrict__ Ah, uint16_t *__restrict__ Ah22) {
    // no fp contraction: every system slot rounds alike, and as k_galerkin0_ns
#pragma clang fp contract(off)
    __shared__ float con[kGalENS][9][kWG];
    int32_t g, bq;
    const int32_t nq = (B + kGalENS - 1) / kGalENS;
    if (!xcd_map(ngrp, nq, g, bq, kGrpGal)) return;
    const int32_t b0 = bq * kGalENS;
    const int32_t p0 = ggrp[2 * g], p1 = ggrp[2 * g + 1];
    const int32_t e0 = gptr[p0], e1 = gptr[p1];
    const int32_t e = e0 + (int32_t)threadIdx.x;
    const int32_t np = p1 - p0;
    // the first task's position data, loaded beside the entry's (the tasks
    // run after the barrier; most groups have one task per thread or fewer)
    int32_t tI = nC, tq0 = 0, tq1 = 0, tdg = -1;
    if ((int32_t)threadIdx.x < np * kGalENS) {
        const int32_t pos = p0 + (int32_t)threadIdx.x / kGalENS;
        tI = c_sell_row[pos];
        tq0 = gptr[pos];
        tq1 = gptr[pos + 1];
        if (tI < nC) tdg = c_diag[tI];
    }
    if (e < e1) {
        const int32_t fp = gent[3 * (int64_t)e], ii = gent[3 * (int64_t)e + 1], jj = gent[3 * (int64_t)e + 2];
        float qi[6], qj[6], a[kGalENS][4];
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            qi[k] = Q[(int64_t)ii * 6 + k];
            qj[k] = Q[(int64_t)jj * 6 + k];
        }
        const int32_t fq = fp < 0 ? 0 : fp & kMirPos;
        const bool tr = fp >= 0 && (fp & kMirT);  // transposed upper block
#pragma unroll
        for (int t = 0; t < kGalENS; ++t) {
            const int64_t bb = min(b0 + t, B - 1);
            h0_dec(h0_ld(Afh, bb * f_sell_nb + fq), a[t][0], a[t][1], a[t][2], a[t][3]);
            if (tr) {
                const float t01 = a[t][1];
                a[t][1] = a[t][2];
                a[t][2] = t01;
            }
            if (fp < 0) {  // a decomposed part's ghost block: identity / zero
                const float d = fp == -1 ? 1.f : 0.f;
                a[t][0] = d; a[t][1] = 0.f; a[t][2] = 0.f; a[t][3] = d;
            }
        }
#pragma unroll
        for (int t = 0; t < kGalENS; ++t) {
            float T[2][3];  // A Q_j
#pragma unroll
            for (int r = 0; r < 2; ++r)
#pragma unroll
                for (int c = 0; c < 3; ++c) T[r][c] = 1.f * (a[t][2 * r] * qj[c] + a[t][2 * r + 1] * qj[3 + c]);
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int c = 0; c < 3; ++c) con[t][3 * r + c][threadIdx.x] = qi[r] * T[0][c] + qi[3 + r] * T[1][c];
        }
    }
    __syncthreads();
    for (int32_t task = threadIdx.x; task < np * kGalENS; task += kWG) {
        const int32_t pos = p0 + task / kGalENS, t = task % kGalENS, b = b0 + t;
        const bool first = task == (int32_t)threadIdx.x;
        const int32_t I = first ? tI : c_sell_row[pos];
        if (I >= nC || b >= B) continue;
        float Cm[3][3] = {};
        const int32_t q0 = first ? tq0 : gptr[pos], q1 = first ? tq1 : gptr[pos + 1];
        const bool diag = pos == (first ? tdg : c_diag[I]);
        if (q0 == q1 && !diag) continue;  // a lower block (its upper twin writes it, st_pair) or padding
        for (int32_t q = q0; q < q1; ++q)
#pragma unroll
            for (int k = 0; k < 9; ++k) Cm[k / 3][k % 3] += con[t][k][q - e0];
        if (diag) {
#pragma unroll
            for (int d = 0; d < 3; ++d)
                if (c_dead[3 * (int64_t)I + d]) Cm[d][d] += 1.f;
            float D[3][3];
            inv3(Cm, D);
            st_h9(Dh, Dh22, (int64_t)b * nC + I, D);
        }
        st_pair(Ac, Ah, Ah22, b, c_sell_nb, pos, c_twin[pos], Cm);
    }
}

// Level 0 with the smoothed prolongator, by system slab: the gather lists
// are wave-uniform and the 64 lanes of a wave are 64 systems of one coarse
// position. The per-position kernel above (one position of 4 systems per
// thread) gathers a 16-byte fine block per system from 4 lines 20 MB apart,
// 64 positions' scattered blocks per load: S1 122 ms per 1536-system batch,
// L2-line bound. Here a slab of kSlab systems' fp32 level-0 blocks is first
// transposed to [fine position][system] (k_a_slab), so one fine block of
// the whole wave is one 1 KB read, and the entry and its two P blocks are
// scalar loads shared by the 64 systems. Every system runs the same
// instructions in its own lane: the bits do not depend on the batch split.
// S1, per 1536-system batch: level 0 122.5 -> 12.3 (k_a_slab) + 40.6 ms,
// S1 1014 -> 1064 timesteps/s; with level 1 -> 2 from the slab copy level 0
// writes beside its A (k_galerkin_sys<3>, instead of the chunked / by-entry
// products, 55 ms): level 0 46.5 + level 1 29.6 ms, R3 906 -> 918
// (profiles/r05_ab/gal_slab/).
constexpr int kSlab = 64;
constexpr int kSlabPos = 64;  // fine positions per k_a_slab workgroup
// T = float4: the fp32 A; T = uint2 (round 6, regular closed meshes -- F3):
// the level-0 sweep copy's bf16 blocks, as the tentative product by entry
// reads them, half the bytes for the transpose and for the product's ~7
// reads of each block: F3 +4 %; on the open patch S1 the bf16 coarse
// operator cost 14 of 3,072 solves a recovery (profiles/r06/slab_bf16/)
template <typename T>
__global__ __launch_bounds__(kWG) void k_a_slab(int64_t f_sell_nb, int32_t b0, int32_t nb,
                                                const T *__restrict__ Af, T *__restrict__ AI) {
    __shared__ T t[kSlabPos][kSlab + 1];
    const int64_t q0 = (int64_t)blockIdx.x * kSlabPos;
    const int32_t lane = (int32_t)threadIdx.x & 63, w = (int32_t)threadIdx.x >> 6;
    // read: a wave takes one system's 64 consecutive blocks
    for (int32_t s = w; s < kSlab; s += kWG / 64) {
        const int64_t q = q0 + lane;
        T v = {};
        if (s < nb && q < f_sell_nb) v = Af[(int64_t)(b0 + s) * f_sell_nb + q];
        t[lane][s] = v;
    }
    __syncthreads();
    // write: a wave takes one fine position's 64 systems
    for (int32_t k = w; k < kSlabPos; k += kWG / 64) {
        const int64_t q = q0 + k;
        if (q < f_sell_nb) AI[q * kSlab + lane] = t[k][lane];
    }
}

constexpr int kGalSysPos = kWG / 64;  // coarse positions per workgroup, one per wave
// Level l's Galerkin product over one system slab: BSF = 2 reads the level-0
// slab (k_a_slab, float4 blocks or, H, bf16 as uint2; mirror entries), BSF = 3 the slab a level
// l >= 1 product wrote beside its level's A (CS: [sell_nb][kSlab][3] float4,
// the stored rows). Gather entries per load batch: 4 at level 0, 2 on the
// coarse levels (their P blocks are 18 scalar registers each).
template <int BSF, bool H = false>
__global__ __launch_bounds__(kWG) void k_galerkin_sys(
    int64_t c_sell_nb, int32_t nC, int32_t B, int32_t b0, const int32_t *__restrict__ c_sell_row,
    const int32_t *__restrict__ c_diag, const uint8_t *__restrict__ c_dead, const int32_t *__restrict__ c_twin, const int32_t *__restrict__ gptr,
    const int32_t *__restrict__ gent, const float *__restrict__ Q, const float4 *__restrict__ FS,
    float *__restrict__ Ac, uint4 *__restrict__ Dh, uint16_t *__restrict__ Dh22, uint4 *__restrict__ Ah,
    uint16_t *__restrict__ Ah22, float4 *__restrict__ CS) {
    constexpr int U = BSF == 2 ? 4 : 2;
    constexpr int QS = 3 * BSF;  // floats per P block
    int32_t tile, bq;
    if (!xcd_map((int32_t)((c_sell_nb + kGalSysPos - 1) / kGalSysPos), 1, tile, bq, 1)) return;
    const int64_t pos = (int64_t)tile * kGalSysPos + __builtin_amdgcn_readfirstlane((int32_t)threadIdx.x >> 6);
    if (pos >= c_sell_nb) return;
    const int32_t I = c_sell_row[pos];
    if (I >= nC) return;
    const int32_t lane = (int32_t)threadIdx.x & 63;
    float Cm[3][3] = {};
    const int32_t g0 = gptr[pos], g1 = gptr[pos + 1];
    if (g0 == g1 && pos != c_diag[I]) return;  // a lower block (its upper twin writes it, st_pair) or padding
    // U entries per load batch (the entries' scalar loads, then their fine
    // blocks, in flight together); a batch's tail entries past g1 are
    // clamped to the last one and skipped (wave-uniform)
    for (int32_t t0 = g0; t0 < g1; t0 += U) {
        int32_t fp[U];
        float qi[U][QS], qj[U][QS], a[U][BSF][BSF];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t g = min(t0 + u, g1 - 1);
            fp[u] = gent[3 * g];
            const int32_t ii = gent[3 * g + 1], jj = gent[3 * g + 2];
#pragma unroll
            for (int k = 0; k < QS; ++k) {
                qi[u][k] = Q[(int64_t)ii * QS + k];
                qj[u][k] = Q[(int64_t)jj * QS + k];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (fp[u] < 0) {  // a decomposed part's ghost block: identity / zero
#pragma unroll
                for (int r = 0; r < BSF; ++r)
#pragma unroll
                    for (int c = 0; c < BSF; ++c) a[u][r][c] = (fp[u] == -1 && r == c) ? 1.f : 0.f;
            } else if constexpr (BSF == 2) {
                const bool tr = fp[u] & kMirT;  // transposed upper block
                if constexpr (H) {
                    const uint2 h = reinterpret_cast<const uint2 *>(FS)[(int64_t)(fp[u] & kMirPos) * kSlab + lane];
                    h0_dec(tr ? h0_tr(h) : h, a[u][0][0], a[u][0][1], a[u][1][0], a[u][1][1]);
                } else {
                    const float4 v = FS[(int64_t)(fp[u] & kMirPos) * kSlab + lane];
                    a[u][0][0] = v.x; a[u][0][1] = tr ? v.z : v.y; a[u][1][0] = tr ? v.y : v.z; a[u][1][1] = v.w;
                }
            } else {
                const float4 *p = FS + ((int64_t)fp[u] * kSlab + lane) * 3;
#pragma unroll
                for (int r = 0; r < 3; ++r) {
                    const float4 v = p[r];
                    a[u][r][0] = v.x; a[u][r][1] = v.y; a[u][r][2] = v.z;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (t0 + u >= g1) break;
            // P blocks are BSF x 3, row-major: q[k * 3 + c]
            float T[BSF][3];  // A Q_j
#pragma unroll
            for (int r = 0; r < BSF; ++r)
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    float sum = 0.f;
#pragma unroll
                    for (int k = 0; k < BSF; ++k) sum += a[u][r][k] * qj[u][k * 3 + c];
                    T[r][c] = sum;
                }
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    float sum = 0.f;
#pragma unroll
                    for (int k = 0; k < BSF; ++k) sum += qi[u][k * 3 + r] * T[k][c];
                    Cm[r][c] += sum;
                }
        }
    }
    const int32_t b = b0 + lane;
    if (b >= B) return;
    if (pos == c_diag[I]) {
#pragma unroll
        for (int d = 0; d < 3; ++d)
            if (c_dead[3 * (int64_t)I + d]) Cm[d][d] += 1.f;
        float D[3][3];
        inv3(Cm, D);
        st_h9(Dh, Dh22, (int64_t)b * nC + I, D);
    }
    st_pair(Ac, Ah, Ah22, b, c_sell_nb, pos, c_twin[pos], Cm);
    if (CS) {
        float4 *p = CS + (pos * kSlab + lane) * 3;
#pragma unroll
        for (int r = 0; r < 3; ++r) p[r] = make_float4(Cm[r][0], Cm[r][1], Cm[r][2], 0.f);
        if (c_twin[pos] >= 0) {
            float4 *q = CS + ((int64_t)c_twin[pos] * kSlab + lane) * 3;
#pragma unroll
            for (int r = 0; r < 3; ++r) q[r] = make_float4(Cm[0][r], Cm[1][r], Cm[2][r], 0.f);
        }
    }
}

// Levels >= 1: the Galerkin product with NS systems per thread sharing each
// gather entry and its two Q blocks (k_galerkin0_ns's scheme for the fp32
// 3x3 blocks), folded per system in list order. Level 1 at C3 (512 systems):
// 1217 us per launch with one system per thread (round 2's k_galerkin<3>,
// 4 entries per load batch), 935 with 2, 851 with 4 (132 VGPRs, 3 waves);
// C3 +0.5 %, R3 (denser level 1) within noise (round 3).
constexpr int kGal3NS = 4;
template <int NS>
__global__ __launch_bounds__(kWG) void k_galerkin3_ns(
    int64_t c_sell_nb, int32_t nC, int32_t B, const int32_t *__restrict__ c_sell_row,
    const int32_t *__restrict__ c_diag, const uint8_t *__restrict__ c_dead, const int32_t *__restrict__ c_twin,
    const int32_t *__restrict__ gptr, const int32_t *__restrict__ gent, const float *__restrict__ Q,
    const float *__restrict__ Af, int64_t f_sell_nb, float *__restrict__ Ac, uint4 *__restrict__ Dh,
    uint16_t *__restrict__ Dh22, uint4 *__restrict__ Ah, uint16_t *__restrict__ Ah22) {
#pragma clang fp contract(off)
    int32_t tile, bq;
    if (!xcd_map((int32_t)((c_sell_nb + kWG - 1) / kWG), (B + NS - 1) / NS, tile, bq, kGrpGal)) return;
    const int64_t pos = (int64_t)tile * kWG + threadIdx.x;
    if (pos >= c_sell_nb) return;
    const int32_t I = c_sell_row[pos];
    if (I >= nC) return;
    const int32_t b0 = bq * NS;
    float Cm[NS][3][3] = {};
    const int32_t g0 = gptr[pos], g1 = gptr[pos + 1];
    if (g0 == g1 && pos != c_diag[I]) return;  // a lower block (its upper twin writes it, st_pair) or padding
    for (int32_t g = g0; g < g1; ++g) {
        const int32_t fp = gent[3 * g], ii = gent[3 * g + 1], jj = gent[3 * g + 2];
        float qi[3][3], qj[3][3];
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                qi[k][c] = Q[((int64_t)ii * 3 + k) * 3 + c];
                qj[k][c] = Q[((int64_t)jj * 3 + k) * 3 + c];
            }
        float a[NS][3][3];
#pragma unroll
        for (int t = 0; t < NS; ++t) {
            ldm<3>(Af + (int64_t)min(b0 + t, B - 1) * f_sell_nb * kB3, max(fp, 0), a[t]);
            if (fp < 0) {
#pragma unroll
                for (int r = 0; r < 3; ++r)
#pragma unroll
                    for (int k = 0; k < 3; ++k) a[t][r][k] = (fp == -1 && r == k) ? 1.f : 0.f;
            }
        }
#pragma unroll
        for (int t = 0; t < NS; ++t) {
            float T[3][3];  // A Q_j
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    float sum = 0.f;
#pragma unroll
                    for (int k = 0; k < 3; ++k) sum += a[t][r][k] * qj[k][c];
                    T[r][c] = sum;
                }
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    float sum = 0.f;
#pragma unroll
                    for (int k = 0; k < 3; ++k) sum += qi[k][r] * T[k][c];
                    Cm[t][r][c] += sum;
                }
        }
    }
#pragma unroll
    for (int t = 0; t < NS; ++t) {
        const int32_t b = b0 + t;
        if (b >= B) continue;
        if (pos == c_diag[I]) {
#pragma unroll
            for (int d = 0; d < 3; ++d)
                if (c_dead[3 * (int64_t)I + d]) Cm[t][d][d] += 1.f;
            float D[3][3];
            inv3(Cm[t], D);
            st_h9(Dh, Dh22, (int64_t)b * nC + I, D);
        }
        st_pair(Ac, Ah, Ah22, b, c_sell_nb, pos, c_twin[pos], Cm[t]);
    }
}

// Levels >= 1 by gather entry (k_galerkin0_ent's scheme for the fp32 3x3
// blocks): one entry of kGalENS systems per thread, its terms staged in LDS,
// one thread per (coarse position, system) summing them in list order -- the
// same bits as k_galerkin3_ns.
__global__ __launch_bounds__(kWG) void k_galerkin3_ent(
    int32_t ngrp, const int32_t *__restrict__ ggrp, int32_t nC, int32_t B, const int32_t *__restrict__ c_sell_row,
    const int32_t *__restrict__ c_diag, const uint8_t *__restrict__ c_dead, const int32_t *__restrict__ c_twin, const int32_t *__restrict__ gptr,
    const int32_t *__restrict__ gent, const float *__restrict__ Q, const float *__restrict__ Af, int64_t f_sell_nb,
    int64_t c_sell_nb, float *__restrict__ Ac, uint4 *__restrict__ Dh, uint16_t *__restrict__ Dh22,
    uint4 *__restrict__ Ah, uint16_t *__restrict__ Ah22) {
#pragma clang fp contract(off)
    __shared__ float con[kGalENS][9][kWG];
    int32_t g, bq;
    const int32_t nq = (B + kGalENS - 1) / kGalENS;
    if (!xcd_map(ngrp, nq, g, bq, kGrpGal)) return;
    const int32_t b0 = bq * kGalENS;
    const int32_t p0 = ggrp[2 * g], p1 = ggrp[2 * g + 1];
    const int32_t e0 = gptr[p0], e1 = gptr[p1];
    const int32_t e = e0 + (int32_t)threadIdx.x;
    const int32_t np = p1 - p0;
    int32_t tI = nC, tq0 = 0, tq1 = 0, tdg = -1;
    if ((int32_t)threadIdx.x < np * kGalENS) {
        const int32_t pos = p0 + (int32_t)threadIdx.x / kGalENS;
        tI = c_sell_row[pos];
        tq0 = gptr[pos];
        tq1 = gptr[pos + 1];
        if (tI < nC) tdg = c_diag[tI];
    }
    if (e < e1) {
        const int32_t fp = gent[3 * (int64_t)e], ii = gent[3 * (int64_t)e + 1], jj = gent[3 * (int64_t)e + 2];
        float qi[3][3], qj[3][3];
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                qi[k][c] = Q[((int64_t)ii * 3 + k) * 3 + c];
                qj[k][c] = Q[((int64_t)jj * 3 + k) * 3 + c];
            }
        float a[kGalENS][3][3];
#pragma unroll
        for (int t = 0; t < kGalENS; ++t) {
            ldm<3>(Af + (int64_t)min(b0 + t, B - 1) * f_sell_nb * kB3, max(fp, 0), a[t]);
            if (fp < 0) {
#pragma unroll
                for (int r = 0; r < 3; ++r)
#pragma unroll
                    for (int k = 0; k < 3; ++k) a[t][r][k] = (fp == -1 && r == k) ? 1.f : 0.f;
            }
        }
#pragma unroll
        for (int t = 0; t < kGalENS; ++t) {
            float T[3][3];  // A Q_j
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    float sum = 0.f;
#pragma unroll
                    for (int k = 0; k < 3; ++k) sum += a[t][r][k] * qj[k][c];
                    T[r][c] = sum;
                }
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    float sum = 0.f;
#pragma unroll
                    for (int k = 0; k < 3; ++k) sum += qi[k][r] * T[k][c];
                    con[t][3 * r + c][threadIdx.x] = sum;
                }
        }
    }
    __syncthreads();
    for (int32_t task = threadIdx.x; task < np * kGalENS; task += kWG) {
        const int32_t pos = p0 + task / kGalENS, t = task % kGalENS, b = b0 + t;
        const bool first = task == (int32_t)threadIdx.x;
        const int32_t I = first ? tI : c_sell_row[pos];
        if (I >= nC || b >= B) continue;
        float Cm[3][3] = {};
        const int32_t q0 = first ? tq0 : gptr[pos], q1 = first ? tq1 : gptr[pos + 1];
        const bool diag = pos == (first ? tdg : c_diag[I]);
        if (q0 == q1 && !diag) continue;  // a lower block (its upper twin writes it, st_pair) or padding
        for (int32_t q = q0; q < q1; ++q)
#pragma unroll
            for (int k = 0; k < 9; ++k) Cm[k / 3][k % 3] += con[t][k][q - e0];
        if (diag) {
#pragma unroll
            for (int d = 0; d < 3; ++d)
                if (c_dead[3 * (int64_t)I + d]) Cm[d][d] += 1.f;
            float D[3][3];
            inv3(Cm, D);
            st_h9(Dh, Dh22, (int64_t)b * nC + I, D);
        }
        st_pair(Ac, Ah, Ah22, b, c_sell_nb, pos, c_twin[pos], Cm);
    }
}

// Levels >= 1, the coarse positions with more than kGalBig gather entries
// (a smoothed level's: S1 level 1 mean 105, p90 247, max 789 entries; 85 %
// of its terms sit in positions past 128, where one thread per position
// leaves a SELL wave 0.24 busy): one workgroup per (position, NSB systems)
// walks the list in chunks of kWG entries -- every thread one entry's term
// for the NSB systems, staged in LDS -- and 9 NSB threads, one per (system,
// block entry), fold each chunk in list order. Each block entry is a sum of
// its own terms, so the bits are k_galerkin3_ns's. S1 (1536 systems), level
// 1 -> 2: 42.8 ms per launch per position -> 20.9 by chunk (and 4.6 ms for
// the positions below the bound by entry); 4 systems per workgroup 23.1, 8
// 25.8, bound 64 entries 24.9 + 3.3 (profiles/r05_ab/gal_slab/).
constexpr int kGalBig = 128;
template <int NSB>
__global__ __launch_bounds__(kWG) void k_galerkin3_big(
    int32_t nbig, const int32_t *__restrict__ gbig, int32_t nC, int32_t B, const int32_t *__restrict__ c_sell_row,
    const int32_t *__restrict__ c_diag, const uint8_t *__restrict__ c_dead, const int32_t *__restrict__ c_twin, const int32_t *__restrict__ gptr,
    const int32_t *__restrict__ gent, const float *__restrict__ Q, const float *__restrict__ Af, int64_t f_sell_nb,
    int64_t c_sell_nb, float *__restrict__ Ac, uint4 *__restrict__ Dh, uint16_t *__restrict__ Dh22,
    uint4 *__restrict__ Ah, uint16_t *__restrict__ Ah22) {
#pragma clang fp contract(off)
    // rows padded by one word: the 9 NSB summing lanes read one column at
    // a time, kWG + 1 words apart -- distinct banks
    __shared__ float con[NSB][9][kWG + 1];
    __shared__ float fin[NSB][9];
    int32_t g, bq;
    if (!xcd_map(nbig, (B + NSB - 1) / NSB, g, bq, kGrpGal)) return;
    const int32_t b0 = bq * NSB;
    const int32_t pos = gbig[g];
    const int32_t e0 = gptr[pos], e1 = gptr[pos + 1];
    const int32_t sk = (int32_t)threadIdx.x;  // summing lane: system sk / 9, block entry sk % 9
    float acc = 0.f;
    for (int32_t c0 = e0; c0 < e1; c0 += kWG) {
        const int32_t e = c0 + (int32_t)threadIdx.x;
        if (e < e1) {
            const int32_t fp = gent[3 * (int64_t)e], ii = gent[3 * (int64_t)e + 1], jj = gent[3 * (int64_t)e + 2];
            float qi[3][3], qj[3][3];
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    qi[k][c] = Q[((int64_t)ii * 3 + k) * 3 + c];
                    qj[k][c] = Q[((int64_t)jj * 3 + k) * 3 + c];
                }
            float a[NSB][3][3];
#pragma unroll
            for (int t = 0; t < NSB; ++t) {
                ldm<3>(Af + (int64_t)min(b0 + t, B - 1) * f_sell_nb * kB3, max(fp, 0), a[t]);
                if (fp < 0) {
#pragma unroll
                    for (int r = 0; r < 3; ++r)
#pragma unroll
                        for (int k = 0; k < 3; ++k) a[t][r][k] = (fp == -1 && r == k) ? 1.f : 0.f;
                }
            }
#pragma unroll
            for (int t = 0; t < NSB; ++t) {
                float T[3][3];  // A Q_j
#pragma unroll
                for (int r = 0; r < 3; ++r)
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        float sum = 0.f;
#pragma unroll
                        for (int k = 0; k < 3; ++k) sum += a[t][r][k] * qj[k][c];
                        T[r][c] = sum;
                    }
#pragma unroll
                for (int r = 0; r < 3; ++r)
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        float sum = 0.f;
#pragma unroll
                        for (int k = 0; k < 3; ++k) sum += qi[k][r] * T[k][c];
                        con[t][3 * r + c][threadIdx.x] = sum;
                    }
            }
        }
        __syncthreads();
        if (sk < 9 * NSB) {
            const float *row = con[sk / 9][sk % 9];
            const int32_t m = min(kWG, e1 - c0);
            int32_t q = 0;
            for (; q + 8 <= m; q += 8) {
                float v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = row[q + u];
#pragma unroll
                for (int u = 0; u < 8; ++u) acc += v[u];
            }
            for (; q < m; ++q) acc += row[q];
        }
        __syncthreads();
    }
    if (sk < 9 * NSB) fin[sk / 9][sk % 9] = acc;
    __syncthreads();
    if ((int32_t)threadIdx.x >= NSB) return;
    const int32_t t = (int32_t)threadIdx.x, b = b0 + t;
    if (b >= B) return;
    const int32_t I = c_sell_row[pos];
    float Cm[3][3];
#pragma unroll
    for (int k = 0; k < 9; ++k) Cm[k / 3][k % 3] = fin[t][k];
    if (pos == c_diag[I]) {
#pragma unroll
        for (int d = 0; d < 3; ++d)
            if (c_dead[3 * (int64_t)I + d]) Cm[d][d] += 1.f;
        float D[3][3];
        inv3(Cm, D);
        st_h9(Dh, Dh22, (int64_t)b * nC + I, D);
    }
    st_pair(Ac, Ah, Ah22, b, c_sell_nb, pos, c_twin[pos], Cm);
}
constexpr int kGalBigNS = 2;

constexpr int kMaxCoarse = 128;
constexpr int kInvWG = 1024;
constexpr int kSweepRows = kMaxCoarse * kMaxCoarse / kInvWG;  // 16 matrix rows per thread

// Inverse of the coarsest operator (nc = 3 n <= 128 dofs) of system b by the
// symmetric sweep operator: sweeping pivot k maps
//   a_kk -> -1/a_kk, a_ik -> a_ik/a_kk, a_kj -> a_kj/a_kk,
//   a_ij -> a_ij - a_ik a_kj / a_kk,
// and after all pivots the matrix holds -A^-1. Symmetry gives column k =
// row k, so a step broadcasts one row through LDS. Thread t owns column
// t % 128 of rows (t / 128) * 16 + [0, 16) in fp64 registers.
__global__ __launch_bounds__(kInvWG) void k_coarse_inverse(int32_t n, const int32_t *__restrict__ sell_off,
                                                        const int32_t *__restrict__ sell_col,
                                                        const float *__restrict__ Ac, int64_t sell_nb,
                                                        float *__restrict__ cinv) {
    __shared__ float M[kMaxCoarse][kMaxCoarse + 1];
    __shared__ double rowk[kMaxCoarse];
    const int32_t b = blockIdx.x;
    const int32_t nc = 3 * n;
    for (int32_t q = threadIdx.x; q < kMaxCoarse * kMaxCoarse; q += kInvWG)
        M[q / kMaxCoarse][q % kMaxCoarse] = 0.f;
    __syncthreads();
    const float *A = Ac + (int64_t)b * sell_nb * kB3;
    // one thread per node row: no two threads write the same row
    for (int32_t I = threadIdx.x; I < n; I += kInvWG) {
        const int32_t s = I >> 6, l = I & 63;
        const int32_t o = sell_off[s], w = (sell_off[s + 1] - o) >> 6;
        for (int32_t t = 0; t < w; ++t) {
            const int64_t pos = (int64_t)o + t * kSlice + l;
            const int32_t J = sell_col[pos];
            float a[3][3];
            ldm<3>(A, pos, a);
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) M[3 * I + r][3 * J + c] += a[r][c];
        }
    }
    __syncthreads();
    const int32_t c = threadIdx.x & (kMaxCoarse - 1);
    const int32_t h = threadIdx.x / kMaxCoarse;
    double a[kSweepRows];
#pragma unroll
    for (int mm = 0; mm < kSweepRows; ++mm) a[mm] = (double)M[h * kSweepRows + mm][c];
    if (threadIdx.x < kMaxCoarse) rowk[threadIdx.x] = 0.0;
    __syncthreads();
    for (int32_t k = 0; k < nc; ++k) {
        if (h == k / kSweepRows && c < nc) {
            const int32_t mk = k % kSweepRows;
            double v = 0.0;
#pragma unroll
            for (int mm = 0; mm < kSweepRows; ++mm) v = (mm == mk) ? a[mm] : v;
            rowk[c] = v;
        }
        __syncthreads();
        double piv = rowk[k];
        piv = piv != 0.0 ? piv : 1.0;
        const double ip = 1.0 / piv;
        const double akc = rowk[c] * ip;
        const bool ck = c == k;
        const double rowfix = ck ? -ip : akc;  // the new row k
        // branch-free (every LDS read unconditional, so they pipeline):
        // column k scales by 1/piv, row k is replaced, the rest updates
        const double f = ck ? 0.0 : akc, sc = ck ? ip : 1.0;
#pragma unroll
        for (int mm = 0; mm < kSweepRows; ++mm) {
            const int32_t r = h * kSweepRows + mm;
            const double v = fma(-rowk[r], f, a[mm]) * sc;
            a[mm] = (r == k) ? rowfix : v;
        }
        __syncthreads();
    }
    float *out = cinv + (int64_t)b * nc * nc;
    if (c < nc) {
#pragma unroll
        for (int mm = 0; mm < kSweepRows; ++mm) {
            const int32_t r = h * kSweepRows + mm;
            if (r < nc) out[(int64_t)r * nc + c] = (float)(-a[mm]);
        }
    }
}

// ---- V-cycle ---------------------------------------------------------------

// Device view of one level (pointers to system 0; system b adds its stride).
struct Lvl {
    int32_t n;
    int64_t sell_nb;
    const int32_t *sell_off, *sell_col;  // level >= 1
    const float *A;                      // level >= 1: [B][sell_nb][12]
    const uint4 *Dh;                     // level >= 1: 3x3 D^-1, bf16 entries 0..7 [B][n]
    const uint16_t *Dh22;                // and entry (2,2)
    const uint4 *Ah;                     // bf16 A for the sweeps: [B][sell_nb] entries 0..7, or null
    const uint16_t *Ah22;                // [B][sell_nb] entry (2,2)
    float *b, *x, *r, *y;                // [B][n][4] (level 0: x [B][n][2], r bf16 [B][n][2])
    const int32_t *agg, *mptr, *apos;    // transition to level + 1
    const int32_t *mlist;                // aggregate members (level 0: r1 gathered in member order)
    const float *Q, *Qm;                 // tentative rows (node order / member order), or P blocks
    const int32_t *pptr, *pcol;          // smoothed P: row blocks of each fine node
    const int32_t *rptr, *rent;          // smoothed P: {fine node, P block} per coarse node
    const int32_t *rperm;                // smoothed P: each restriction group's entries by fine node
    SysMap sm;                           // the systems the cycle's launches cover (amg_vcycle)
};

// 3x3 bf16 block stored as 8 entries in 16 B + entry (2,2) in 2 B
__device__ __forceinline__ void ld_h9(const uint4 *H, const uint16_t *H22, int64_t q, float (&a)[3][3]) {
    const uint4 h = H[q];
    a[0][0] = bf16_lo(h.x);
    a[0][1] = bf16_hi(h.x);
    a[0][2] = bf16_lo(h.y);
    a[1][0] = bf16_hi(h.y);
    a[1][1] = bf16_lo(h.z);
    a[1][2] = bf16_hi(h.z);
    a[2][0] = bf16_lo(h.w);
    a[2][1] = bf16_hi(h.w);
    a[2][2] = bf16_lo((uint32_t)H22[q]);
}
// block q of a coarse level's sweep copy (st_a9)
__device__ __forceinline__ void ld_a9(const uint4 *H, const uint16_t *H22, int64_t q, float (&a)[3][3]) {
    {
        const uint2 h = reinterpret_cast<const uint2 *>(H)[q];
        const uint32_t t = reinterpret_cast<const uint32_t *>(H22)[q];
        const float sc = bf16_hi(t);
        const uint32_t w[3] = {h.x, h.y, t};
#pragma unroll
        for (int e = 0; e < 9; ++e)
            a[e / 3][e % 3] = (float)((int32_t)((w[e >> 2] >> (8 * (e & 3))) & 0xffu) - 128) * sc;
    }
}
// the smoother's 3x3 D^-1 of node i of system b
__device__ __forceinline__ void ld_dh(const Lvl &L, int32_t b, int32_t i, float (&d)[3][3]) {
    ld_h9(L.Dh, L.Dh22, (int64_t)b * L.n + i, d);
}

// (A x)_i of a coarse level, slots U at a time with all loads of a chunk
// issued first (as spmv_row).
__device__ __forceinline__ void spmv_row3(const Lvl &L, int32_t b, int32_t i, const float *__restrict__ xb,
                                          float (&acc)[3]) {
    constexpr int U = 4;
    const float *Ab = L.A + (int64_t)b * L.sell_nb * kB3;
    const int64_t hb = (int64_t)b * L.sell_nb;  // system b's first block of the sweep copy (ld_a9 index)
    const bool half = L.Ah != nullptr;
    const int32_t s = i >> 6, l = i & 63;
    const int32_t o = L.sell_off[s], w = (L.sell_off[s + 1] - o) >> 6;
    acc[0] = acc[1] = acc[2] = 0.f;
    for (int32_t t0 = 0; t0 < w; t0 += U) {
        int32_t j[U];
        float a[U][3][3], xj[U][3];
#pragma unroll
        for (int u = 0; u < U; ++u) j[u] = L.sell_col[(int64_t)o + min(t0 + u, w - 1) * kSlice + l];
        if (half) {
#pragma unroll
            for (int u = 0; u < U; ++u) ld_a9(L.Ah, L.Ah22, hb + o + min(t0 + u, w - 1) * kSlice + l, a[u]);
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) ldm<3>(Ab, (int64_t)o + min(t0 + u, w - 1) * kSlice + l, a[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) ldv<3>(xb, j[u], xj[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool on = t0 + u < w;
            float ax[3];
            matvec<3>(a[u], xj[u], ax);
#pragma unroll
            for (int c = 0; c < 3; ++c) acc[c] += on ? ax[c] : 0.f;
        }
    }
}

// coarse level: r = b - A x at the member position of node i
__device__ __forceinline__ void res3_node(const Lvl &L, int32_t b, int32_t i) {
    const int64_t vo = (int64_t)b * L.n * 4;
    float ax[3], bi[3];
    spmv_row3(L, b, i, L.x + vo, ax);
    ldv<3>(L.b + vo, i, bi);
    const float ri[3] = {bi[0] - ax[0], bi[1] - ax[1], bi[2] - ax[2]};
    stv<3>(L.r + vo, L.apos[i], ri);
}

// Level 0's restricted residual r1 stays in aggregate member order (k_res0
// scatters into it): node order made k_res0's stores coalesced (1053 -> 961
// us) but the restriction's member gathers scattered (233 -> 361 us), a net
// loss (round 2, C3, B = 512).
template <int BSF>
__device__ __forceinline__ int32_t r_at(const Lvl &, int32_t q) {
    return q;
}

// b_C[I] = sum over the members of aggregate I of Q^T r (member order,
// contiguous, U at a time); with smooth also x_C[I] = w D_C^-1 b_C[I].
template <int BSF>
__device__ __forceinline__ void restrict_node(const Lvl &F, const Lvl &C, int32_t b, int32_t I, bool smooth,
                                              float omega) {
    constexpr int U = 4;
    float acc[3] = {0.f, 0.f, 0.f};
    const int32_t q0 = F.mptr[I], q1 = F.mptr[I + 1];
    for (int32_t t0 = q0; t0 < q1; t0 += U) {
        float ri[U][BSF], qm[U][BSF * 3];
#pragma unroll
        for (int u = 0; u < U; ++u) ldr<BSF>(F.r, b, F.n, r_at<BSF>(F, min(t0 + u, q1 - 1)), ri[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float *p = F.Qm + (int64_t)min(t0 + u, q1 - 1) * BSF * 3;
#pragma unroll
            for (int k = 0; k < BSF * 3; ++k) qm[u][k] = p[k];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float on = t0 + u < q1 ? 1.f : 0.f;
#pragma unroll
            for (int k = 0; k < BSF; ++k)
#pragma unroll
                for (int c = 0; c < 3; ++c) acc[c] += qm[u][3 * k + c] * (on * ri[u][k]);
        }
    }
    const int64_t vo = (int64_t)b * C.n * 4;
    stv<3>(C.b + vo, I, acc);
    if (smooth) {
        float d[3][3], x[3];
        ld_dh(C, b, I, d);
        matvec<3>(d, acc, x);
#pragma unroll
        for (int c = 0; c < 3; ++c) x[c] *= omega;
        stv<3>(C.x + vo, I, x);
    }
}

// x_i += Q_i y_C[agg(i)]; level 0's corrected iterate in the x0 format in
// place (XM = 1) or as float2 in F.y (XM = 2), see AmgDevice::xm
template <int BSF, int XM = 2>
__device__ __forceinline__ void prolong_node(const Lvl &F, const Lvl &C, int32_t b, int32_t i) {
    float y[3], xi[BSF];
    ldv<3>(C.y + (int64_t)b * C.n * 4, F.agg[i], y);
    float *xb = F.x + (int64_t)b * F.n * vstride<BSF>();
    if constexpr (BSF == 2) {
        const float2 t = ld_x0(F.x, (int64_t)b * F.n + i);
        xi[0] = t.x;
        xi[1] = t.y;
    } else {
        ldv<BSF>(xb, i, xi);
    }
    const float *qi = F.Q + (int64_t)i * BSF * 3;
#pragma unroll
    for (int k = 0; k < BSF; ++k) xi[k] += qi[3 * k] * y[0] + qi[3 * k + 1] * y[1] + qi[3 * k + 2] * y[2];
    if constexpr (BSF == 2 && XM == 2)  // full-precision x for the post-smoothing
        reinterpret_cast<float2 *>(F.y)[(int64_t)b * F.n + i] = make_float2(xi[0], xi[1]);
    else if constexpr (BSF == 2)
        st_x0(F.x, (int64_t)b * F.n + i, xi[0], xi[1]);
    else
        stv<BSF>(xb, i, xi);
}

// coarse level: y = x + w D^-1 (b - A x)
__device__ __forceinline__ void post3_node(const Lvl &L, int32_t b, int32_t i, float omega) {
    const int64_t vo = (int64_t)b * L.n * 4;
    float ax[3], res[3], xi[3], d[3][3], dr[3];
    spmv_row3(L, b, i, L.x + vo, ax);
    ldv<3>(L.b + vo, i, res);
    ldv<3>(L.x + vo, i, xi);
    ld_dh(L, b, i, d);
#pragma unroll
    for (int c = 0; c < 3; ++c) res[c] -= ax[c];
    matvec<3>(d, res, dr);
#pragma unroll
    for (int c = 0; c < 3; ++c) xi[c] += omega * dr[c];
    stv<3>(L.y + vo, i, xi);
}

__global__ __launch_bounds__(kWG) void k_res3(Lvl L, const int32_t *__restrict__ sysi) {
    const int32_t i = blockIdx.x * kWG + threadIdx.x, b = sm_b(L.sm, blockIdx.y);
    if (i >= L.n || retired(sysi, b)) return;
    res3_node(L, b, i);
}

// Restriction by aggregate groups: a workgroup takes whole aggregates with
// at most kRG members in total (group boundaries built on the host), reads
// its members' r and Q rows coalesced (one member per thread), stages the
// per-member contributions Q_q^T r_q in LDS, and one thread per aggregate
// sums them in member order (deterministic). An aggregate with more than
// kRG members forms its own group and is summed straight from memory.
constexpr int kRG = 1024;

// NS systems per workgroup share each member's Q row load; the contributions
// of all NS systems are staged in LDS (level 0: NS = kRestrS = 2, C3 232 ->
// 194 us per 512-system launch; NS = 4: 235 us, its 48-KB LDS stage lowers
// the occupancy).
constexpr int kRestrS = 2;
template <int BSF, int NS = 1>
__global__ __launch_bounds__(kWG) void k_restrict(Lvl F, Lvl C, const int32_t *__restrict__ grp, int32_t ngrp,
                                                  int32_t B, int32_t smooth, float omega,
                                                  const int32_t *__restrict__ sysi) {
    // no fp contraction: every system slot of the unrolled loops rounds alike
#pragma clang fp contract(off)
    __shared__ float con[NS][3][kRG];
    int32_t g, bq;
    if (!xcd_map(ngrp, (F.sm.n + NS - 1) / NS, g, bq, kGrpRestr)) return;
    const int32_t b0 = bq * NS;
    bool any = false;
#pragma unroll
    for (int t = 0; t < NS; ++t) any |= b0 + t < F.sm.n && !retired(sysi, sm_b(F.sm, b0 + t));
    if (!any) return;
    const int32_t I0 = grp[g], I1 = grp[g + 1];
    const int32_t q0 = F.mptr[I0], q1 = F.mptr[I1];
    if (q1 - q0 > kRG) {  // one oversized aggregate
        if (threadIdx.x == 0)
            for (int t = 0; t < NS; ++t)
                if (b0 + t < F.sm.n && !retired(sysi, sm_b(F.sm, b0 + t)))
                    restrict_node<BSF>(F, C, sm_b(F.sm, b0 + t), I0, smooth != 0, omega);
        return;
    }
    for (int32_t q = q0 + threadIdx.x; q < q1; q += kWG) {
        float ri[NS][BSF];
#pragma unroll
        for (int t = 0; t < NS; ++t) ldr<BSF>(F.r, sm_b(F.sm, b0 + t), F.n, r_at<BSF>(F, q), ri[t]);
        const float *qm = F.Qm + (int64_t)q * BSF * 3;
        float qv[BSF * 3];
#pragma unroll
        for (int k = 0; k < BSF * 3; ++k) qv[k] = qm[k];
#pragma unroll
        for (int t = 0; t < NS; ++t) {
            float c3[3] = {0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < BSF; ++k)
#pragma unroll
                for (int c = 0; c < 3; ++c) c3[c] += qv[3 * k + c] * ri[t][k];
#pragma unroll
            for (int c = 0; c < 3; ++c) con[t][c][q - q0] = c3[c];
        }
    }
    __syncthreads();
    for (int32_t I = I0 + threadIdx.x; I < I1; I += kWG) {
        float acc[NS][3] = {};
        for (int32_t q = F.mptr[I]; q < F.mptr[I + 1]; ++q)
#pragma unroll
            for (int t = 0; t < NS; ++t)
#pragma unroll
                for (int c = 0; c < 3; ++c) acc[t][c] += con[t][c][q - q0];
#pragma unroll
        for (int t = 0; t < NS; ++t) {
            if (b0 + t >= F.sm.n) continue;
            const int32_t b = sm_b(F.sm, b0 + t);
            if (retired(sysi, b)) continue;
            const int64_t vo = (int64_t)b * C.n * 4;
            stv<3>(C.b + vo, I, acc[t]);
            if (smooth) {
                float d[3][3], x[3];
                ld_dh(C, b, I, d);
                matvec<3>(d, acc[t], x);
#pragma unroll
                for (int c = 0; c < 3; ++c) x[c] *= omega;
                stv<3>(C.x + vo, I, x);
            }
        }
    }
}

// Level 0 with a smoothed prolongator: b_C[I] = sum over I's restriction
// list (fine node order) of P^T r (r in node order). As k_restrict: a
// workgroup takes whole coarse nodes with at most kRGS list entries in
// total and kNSR systems; one thread per entry loads the entry and its P
// block once and forms P_e^T r_i of every system into LDS, then one thread
// per (coarse node, system) sums the node's entries in list order; with
// smooth also x_C[I] = w D_C^-1 b_C[I].
// Round 4 (S1, B = 1024, rocprof, profiles/r04_ab/sa_xfer/; V bit-identical,
// tools/vhash.py): the sums by coarse node alone left most of the
// workgroup idle behind a few long serial loops -- by (node, system)
// 1615 -> 1434 us per launch, and 8 instead of 4 systems per workgroup
// 1344 us (48-KB LDS stage); the prolongation with 8 systems per thread
// 1263 -> 1112 us: S1 990 -> 1018 timesteps/s; 16 per thread (72 VGPRs, no
// scratch) 1089 -> 975 us, while 16 systems per restriction workgroup over
// 256-entry groups stay at 1347 us (profiles/r04_ab/sa_xfer/call38/); two
// list entries per thread and pass with their loads in flight together
// 1347 -> 1300 us (call42/).
// Round 5: the entry pass in fine-node order within each group (rperm;
// the per-node sums keep list order, same bits): S1 (1536 systems) 1653 ->
// 1445 us per launch, the level-1 restriction 533 -> 439 us, S1 +0.9 %
// (profiles/r05_ab/restr_sort/).
// (The tentative k_restrict by (aggregate, system): 397 -> 448 us at C3,
// and with two members per thread and pass: 360 vs 360 us (call43/); neither
// kept.)
constexpr int kNSR = 8;    // systems per workgroup in the smoothed-P restriction
constexpr int kNSP = 16;   // systems per thread in the smoothed-P prolongation
constexpr int kRGS = 512;  // list entries per restriction group (smoothed P)
// BSF = 3: level 1's smoothed prolongator (AmgParams::smooth1), r as float4
// in node order; round 5 (F3): 938 us per 1024-system launch with one
// (coarse node, system) per thread walking its list
template <int BSF = 2>
__global__ __launch_bounds__(kWG) void k_restrict0_sa(Lvl F, Lvl C, const int32_t *__restrict__ grp, int32_t ngrp,
                                                      int32_t B, int32_t smooth, float omega,
                                                      const int32_t *__restrict__ sysi) {
    // no fp contraction: every system slot of the unrolled loops rounds alike
    // (a system's bits must not depend on its slot, i.e. on the batch split)
#pragma clang fp contract(off)
    __shared__ float con[kNSR][3][kRGS];
    int32_t g, bq;
    const int32_t nq = (F.sm.n + kNSR - 1) / kNSR;
    if (!xcd_map(ngrp, nq, g, bq, kGrpRestr)) return;
    const int32_t b0 = bq * kNSR;
    bool any = false;
#pragma unroll
    for (int t = 0; t < kNSR; ++t) any |= b0 + t < F.sm.n && !retired(sysi, sm_b(F.sm, b0 + t));
    if (!any) return;
    const int32_t I0 = grp[g], I1 = grp[g + 1];
    const int32_t e0 = F.rptr[I0], e1 = F.rptr[I1];
    const bool big = e1 - e0 > kRGS;  // one coarse node with an oversized list: summed from memory
    auto contrib = [&](int32_t e, float (&c3)[kNSR][3]) {
        const int32_t i = F.rent[2 * (int64_t)e];
        const float *p = F.Q + (int64_t)F.rent[2 * (int64_t)e + 1] * (BSF * 3);
        float pm[BSF * 3];
#pragma unroll
        for (int k = 0; k < BSF * 3; ++k) pm[k] = p[k];
        float ri[kNSR][BSF];
#pragma unroll
        for (int t = 0; t < kNSR; ++t) ldr<BSF>(F.r, sm_b(F.sm, b0 + t), F.n, i, ri[t]);
#pragma unroll
        for (int t = 0; t < kNSR; ++t)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                float v = pm[c] * ri[t][0] + pm[3 + c] * ri[t][1];
                if constexpr (BSF == 3) v += pm[6 + c] * ri[t][2];
                c3[t][c] = v;
            }
    };
    // two entries per thread and pass, both entries' loads in flight together;
    // the entries visited in fine-node order (rperm: adjacent lanes gather
    // adjacent r), each staged at its list slot
    for (int32_t q = e0 + threadIdx.x; q < e1 && !big; q += 2 * kWG) {
        const bool two = q + kWG < e1;
        const int32_t ea = F.rperm ? F.rperm[q] : q;
        const int32_t eb = two ? (F.rperm ? F.rperm[q + kWG] : q + kWG) : ea;
        float c3[2][kNSR][3];
        contrib(ea, c3[0]);
        contrib(eb, c3[1]);
#pragma unroll
        for (int t = 0; t < kNSR; ++t)
#pragma unroll
            for (int c = 0; c < 3; ++c) con[t][c][ea - e0] = c3[0][t][c];
        if (two)
#pragma unroll
            for (int t = 0; t < kNSR; ++t)
#pragma unroll
                for (int c = 0; c < 3; ++c) con[t][c][eb - e0] = c3[1][t][c];
    }
    __syncthreads();
    // one thread per (coarse node, system), nodes adjacent across threads:
    // kNSR times the threads of one per node, each summing its node's
    // entries in list order (the same per-system sums, bit for bit)
    const int32_t nI = I1 - I0;
    for (int32_t q = threadIdx.x; q < nI * kNSR; q += kWG) {
        const int32_t t = q / nI, I = I0 + q - t * nI;
        if (b0 + t >= F.sm.n) continue;
        const int32_t b = sm_b(F.sm, b0 + t);
        if (retired(sysi, b)) continue;
        float acc[3] = {};
        for (int32_t e = F.rptr[I]; e < F.rptr[I + 1]; ++e) {
            float c3[3];
            if (big) {
                float all[kNSR][3];
                contrib(e, all);
#pragma unroll
                for (int c = 0; c < 3; ++c) c3[c] = all[t][c];
            } else {
#pragma unroll
                for (int c = 0; c < 3; ++c) c3[c] = con[t][c][e - e0];
            }
#pragma unroll
            for (int c = 0; c < 3; ++c) acc[c] += c3[c];
        }
        const int64_t vo = (int64_t)b * C.n * 4;
        stv<3>(C.b + vo, I, acc);
        if (smooth) {
            float d[3][3], x[3];
            ld_dh(C, b, I, d);
            matvec<3>(d, acc, x);
#pragma unroll
            for (int c = 0; c < 3; ++c) x[c] *= omega;
            stv<3>(C.x + vo, I, x);
        }
    }
}

// Level 0 with a smoothed prolongator: x_i = x0_i + sum_k P_ik y_C[pcol k],
// kNSP systems per thread (the row's P blocks and columns loaded once)
template <int XM>
__global__ __launch_bounds__(kWG) void k_prolong0_sa(Lvl F, Lvl C, int32_t nblk, int32_t B,
                                                     const int32_t *__restrict__ sysi) {
    // no fp contraction: every system slot of the unrolled loops rounds alike
    // (a system's bits must not depend on its slot, i.e. on the batch split)
#pragma clang fp contract(off)
    int32_t rb, bq;
    const int32_t nq = (F.sm.n + kNSP - 1) / kNSP;
    if (!xcd_map(nblk, nq, rb, bq, kGrpProl)) return;
    const int32_t b0 = bq * kNSP;
    const int32_t i = rb * kWG + threadIdx.x;
    if (i >= F.n) return;
    float x[kNSP][2];
#pragma unroll
    for (int t = 0; t < kNSP; ++t) {
        const float2 v = ld_x0(F.x, (int64_t)sm_b(F.sm, b0 + t) * F.n + i);
        x[t][0] = v.x;
        x[t][1] = v.y;
    }
    const int32_t k0 = F.pptr[i], k1 = F.pptr[i + 1];
    for (int32_t k = k0; k < k1; ++k) {
        const int32_t K = F.pcol[k];
        const float *q = F.Q + (int64_t)k * 6;
        float qm[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) qm[c] = q[c];
        float y[kNSP][3];
#pragma unroll
        for (int t = 0; t < kNSP; ++t) ldv<3>(C.y + (int64_t)sm_b(F.sm, b0 + t) * C.n * 4, K, y[t]);
#pragma unroll
        for (int t = 0; t < kNSP; ++t) {
            x[t][0] += qm[0] * y[t][0] + qm[1] * y[t][1] + qm[2] * y[t][2];
            x[t][1] += qm[3] * y[t][0] + qm[4] * y[t][1] + qm[5] * y[t][2];
        }
    }
#pragma unroll
    for (int t = 0; t < kNSP; ++t) {
        if (b0 + t >= F.sm.n) continue;
        const int32_t b = sm_b(F.sm, b0 + t);
        if (retired(sysi, b)) continue;
        if constexpr (XM == 2)  // full-precision x for the post-smoothing
            reinterpret_cast<float2 *>(F.y)[(int64_t)b * F.n + i] = make_float2(x[t][0], x[t][1]);
        else
            st_x0(F.x, (int64_t)b * F.n + i, x[t][0], x[t][1]);
    }
}

// x_i += sum over the fine node's P blocks of P_ik y_C[pcol k] (level 1,
// smoothed prolongator), in place; kNS3 systems per thread share the row's P
// blocks and columns (round 5, F3: 559 us per 1024-system launch with one
// system per thread)
constexpr int kNS3 = 8;
__global__ __launch_bounds__(kWG) void k_prolong3_sa(Lvl F, Lvl C, int32_t nblk, int32_t B,
                                                     const int32_t *__restrict__ sysi) {
#pragma clang fp contract(off)
    int32_t rb, bq;
    if (!xcd_map(nblk, (F.sm.n + kNS3 - 1) / kNS3, rb, bq, kGrpProl)) return;
    const int32_t i = rb * kWG + threadIdx.x;
    if (i >= F.n) return;
    const int32_t b0 = bq * kNS3;
    float x[kNS3][3];
#pragma unroll
    for (int t = 0; t < kNS3; ++t) ldv<3>(F.x + (int64_t)sm_b(F.sm, b0 + t) * F.n * 4, i, x[t]);
    for (int32_t k = F.pptr[i]; k < F.pptr[i + 1]; ++k) {
        const float *p = F.Q + (int64_t)k * 9;
        float pm[9];
#pragma unroll
        for (int c = 0; c < 9; ++c) pm[c] = p[c];
        const int32_t K = F.pcol[k];
        float y[kNS3][3];
#pragma unroll
        for (int t = 0; t < kNS3; ++t) ldv<3>(C.y + (int64_t)sm_b(F.sm, b0 + t) * C.n * 4, K, y[t]);
#pragma unroll
        for (int t = 0; t < kNS3; ++t)
#pragma unroll
            for (int r = 0; r < 3; ++r) x[t][r] += pm[3 * r] * y[t][0] + pm[3 * r + 1] * y[t][1] + pm[3 * r + 2] * y[t][2];
    }
#pragma unroll
    for (int t = 0; t < kNS3; ++t) {
        if (b0 + t >= F.sm.n) continue;
        const int32_t b = sm_b(F.sm, b0 + t);
        if (retired(sysi, b)) continue;
        stv<3>(F.x + (int64_t)b * F.n * 4, i, x[t]);
    }
}

template <int BSF>
__global__ __launch_bounds__(kWG) void k_prolong(Lvl F, Lvl C, const int32_t *__restrict__ sysi) {
    const int32_t i = blockIdx.x * kWG + threadIdx.x, b = sm_b(F.sm, blockIdx.y);
    if (i >= F.n || retired(sysi, b)) return;
    prolong_node<BSF>(F, C, b, i);
}

// Level 0 with the XCD-aware (node block, system) order: the B systems of a
// node block run back to back on one XCD and share its Q rows in L2 instead
// of re-reading Q per system (183 vs 261 us per 256-system launch with the
// system-major grid; the coarse levels' kernels measured slower this way).
// kProlR nodes x kProlS systems per thread, every load of the batch issued
// before the first store: one node of one system per thread left each wave a
// dependent agg -> y gather and little else (latency-bound), and the
// systems of a thread share the node's agg and Q row loads. C3, 512
// systems: 314 us (1 x 1), 270 (4 nodes), 231 (2 x 2), 202 (1 x 4), 210 (1 x 8)
constexpr int kProlR = 1, kProlS = 4;
template <int XM>
__global__ __launch_bounds__(kWG) void k_prolong0(Lvl F, Lvl C, int32_t nblk, int32_t B,
                                                  const int32_t *__restrict__ sysi) {
    // no fp contraction: every system slot of the unrolled loops rounds alike
#pragma clang fp contract(off)
    int32_t rb, bq;
    if (!xcd_map(nblk, (F.sm.n + kProlS - 1) / kProlS, rb, bq, kGrpProl)) return;
    const int32_t n = F.n;
    int32_t ii[kProlR], ag[kProlR];
    float q[kProlR][6];
#pragma unroll
    for (int r = 0; r < kProlR; ++r) {
        ii[r] = (rb * kProlR + r) * kWG + threadIdx.x;
        const int32_t i = min(ii[r], n - 1);
        ag[r] = F.agg[i];
#pragma unroll
        for (int k = 0; k < 6; ++k) q[r][k] = F.Q[(int64_t)i * 6 + k];
    }
    float2 x0[kProlS][kProlR];
    float y[kProlS][kProlR][3];
#pragma unroll
    for (int t = 0; t < kProlS; ++t) {
        const int32_t b = sm_b(F.sm, bq * kProlS + t);
        const float *yb = C.y + (int64_t)b * C.n * 4;
#pragma unroll
        for (int r = 0; r < kProlR; ++r) {
            x0[t][r] = ld_x0(F.x, (int64_t)b * n + min(ii[r], n - 1));
            ldv<3>(yb, ag[r], y[t][r]);
        }
    }
#pragma unroll
    for (int t = 0; t < kProlS; ++t) {
        if (bq * kProlS + t >= F.sm.n) continue;
        const int32_t b = sm_b(F.sm, bq * kProlS + t);
        if (retired(sysi, b)) continue;
        const int64_t vb = (int64_t)b * n;
#pragma unroll
        for (int r = 0; r < kProlR; ++r) {
            if (ii[r] >= n) break;
            float xi[2] = {x0[t][r].x, x0[t][r].y};
#pragma unroll
            for (int k = 0; k < 2; ++k)
                xi[k] += q[r][3 * k] * y[t][r][0] + q[r][3 * k + 1] * y[t][r][1] + q[r][3 * k + 2] * y[t][r][2];
            if constexpr (XM == 2)  // full-precision x for the post-smoothing
                reinterpret_cast<float2 *>(F.y)[vb + ii[r]] = make_float2(xi[0], xi[1]);
            else
                st_x0(F.x, vb + ii[r], xi[0], xi[1]);
        }
    }
}

__global__ __launch_bounds__(kWG) void k_post3(Lvl L, float omega, const int32_t *__restrict__ sysi) {
    const int32_t i = blockIdx.x * kWG + threadIdx.x, b = sm_b(L.sm, blockIdx.y);
    if (i >= L.n || retired(sysi, b)) return;
    post3_node(L, b, i, omega);
}

// The cycle below level S (all levels with <= kSubNodes nodes) in one launch:
// one workgroup per system walks the tiny levels with barriers in between,
// replacing ~4 launches per level.
// 512 threads: a 400-node level (the 3,249-vertex S1s's level 1) takes one
// row per thread in its sweeps instead of two
constexpr int kSubWG = 512;
// kSubNodes: mof_amg.h
constexpr int kMaxLevels = 12;

struct SubArgs {
    int32_t first, last;  // levels first..last (last = coarsest), first >= 1
    Lvl lv[kMaxLevels];
    const float *cinv;
    float omega;
    const int32_t *sysi;
};

__global__ __launch_bounds__(kSubWG) void k_subcycle(SubArgs a) {
    const int32_t b = sm_b(a.lv[0].sm, blockIdx.x);
    if (retired(a.sysi, b)) return;
    const int32_t tid = threadIdx.x;
    // down: level first already holds b and the pre-smoothed x
    for (int32_t l = a.first; l < a.last; ++l) {
        const Lvl &F = a.lv[l], &C = a.lv[l + 1];
        for (int32_t i = tid; i < F.n; i += kSubWG) res3_node(F, b, i);
        __syncthreads();
        for (int32_t I = tid; I < C.n; I += kSubWG) restrict_node<3>(F, C, b, I, l + 1 < a.last, a.omega);
        __syncthreads();
    }
    // coarsest: y = A_c^-1 b (the inverse is symmetric: read by columns);
    // b staged in LDS, the k range split over the kH groups of kMaxCoarse
    // threads, 16 independent loads in flight per thread, the groups'
    // partial sums added in group order
    {
        constexpr int kH = kSubWG / kMaxCoarse;
        __shared__ float bl[kMaxCoarse];
        __shared__ float part[kH][kMaxCoarse];
        const Lvl &C = a.lv[a.last];
        const int32_t nc = 3 * C.n;
        const float *Mi = a.cinv + (int64_t)b * nc * nc;
        const float *bb = C.b + (int64_t)b * C.n * 4;
        for (int32_t q = tid; q < nc; q += kSubWG) bl[q] = bb[4 * (q / 3) + q % 3];
        __syncthreads();
        const int32_t d = tid % kMaxCoarse, hf = tid / kMaxCoarse;
        const int32_t chunk = (nc + kH - 1) / kH;
        const int32_t k0 = min(nc, hf * chunk), k1 = min(nc, k0 + chunk);
        float sum = 0.f;
        if (d < nc) {
            constexpr int U = 16;
            for (int32_t k = k0; k < k1; k += U) {
                float mv[U];
#pragma unroll
                for (int u = 0; u < U; ++u) mv[u] = Mi[(int64_t)min(k + u, k1 - 1) * nc + d];
#pragma unroll
                for (int u = 0; u < U; ++u) sum += (k + u < k1) ? mv[u] * bl[min(k + u, k1 - 1)] : 0.f;
            }
        }
        part[hf][d] = sum;
        __syncthreads();
        if (!hf && d < nc) {
            float t = part[0][d];
#pragma unroll
            for (int h = 1; h < kH; ++h) t += part[h][d];
            C.y[(int64_t)b * C.n * 4 + 4 * (d / 3) + d % 3] = t;
        }
        __syncthreads();
    }
    // up
    for (int32_t l = a.last - 1; l >= a.first; --l) {
        const Lvl &F = a.lv[l], &C = a.lv[l + 1];
        for (int32_t i = tid; i < F.n; i += kSubWG) prolong_node<3>(F, C, b, i);
        __syncthreads();
        for (int32_t i = tid; i < F.n; i += kSubWG) post3_node(F, b, i, a.omega);
        __syncthreads();
    }
}

// Level 0: r1 = r - A x0 (x0 = w D^-1 r from the PCG update), stored at the
// member position of each vertex; PCG row layout. NS systems per thread sharing the row's column / mirror loads:
// grid over (row block, system group of NS) in the XCD order (round 2: 916
// -> 829 us per 512-system launch at NS = 2; 4 lowered the occupancy).
constexpr int kRes0NS = 2, kRes0U = kSweepU;
template <int NS>
__global__ __launch_bounds__(kWG) MOF_ROW_OCC void k_res0_ns(int32_t N, int32_t nblk, int32_t B, SysMap sm, MatH mat,
                                                 const float *__restrict__ rv, const float *__restrict__ xv,
                                                 const int32_t *__restrict__ apos,
                                                 const int32_t *__restrict__ sysi, float *__restrict__ r1) {
#pragma clang fp contract(off)
    int32_t rb, bq;
    if (!xcd_map(nblk, (sm.n + NS - 1) / NS, rb, bq, kGrpSmooth > NS ? kGrpSmooth / NS : 1)) return;
    int32_t bs[NS];
    bool act[NS];
    bool any = false;
#pragma unroll
    for (int t = 0; t < NS; ++t) {
        const int32_t l = bq * NS + t;
        bs[t] = sm_b(sm, l);
        act[t] = l < sm.n && !retired(sysi, bs[t]);
        any |= act[t];
    }
    if (!any) return;
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
        const int32_t i = rb * kRowsPerWG + r * kWG + threadIdx.x;
        if (i >= N) break;
        float y[NS][2];
        auto xl = [&](int t, int32_t j) { return ld_x0(xv, (int64_t)bs[t] * N + j); };
        if (mat.sell_mir)
            spmv_row_hx_ns<true, NS, kRes0U>(mat, bs, i, xl, y);
        else
            spmv_row_hx_ns<false, NS, kRes0U>(mat, bs, i, xl, y);
#pragma unroll
        for (int t = 0; t < NS; ++t) {
            if (!act[t]) continue;
            const int64_t vb = (int64_t)bs[t] * N;
            const float2 ri = reinterpret_cast<const float2 *>(rv)[vb + i];
            reinterpret_cast<uint32_t *>(r1)[vb + (apos ? apos[i] : i)] =
                bf16_bits(ri.x - y[t][0]) | (bf16_bits(ri.y - y[t][1]) << 16);
        }
    }
}

// Level 0's post-smoothing z = x + w D^-1 (r - A x) and the PCG's partial
// r.z, NS systems per thread sharing the row's column / mirror loads, 4 slots
// per load batch to keep the waves (round 2: 918 -> 864 us per 512-system
// launch; 8 slots per batch 1030 us). D^-1 from the row's own diagonal block.
constexpr int kPost0NS = 2, kPost0U = 4;
template <int XM, bool ZH, int NS>
__global__ __launch_bounds__(kWG) MOF_ROW_OCC void k_post0_ns(int32_t N, int32_t nblk, int32_t B, SysMap sm, MatH mat,
                                                  const float *__restrict__ rv,
                                                  const float *__restrict__ xv, float omega,
                                                  const int32_t *__restrict__ sysi,
                                                  float *__restrict__ zv, double *__restrict__ part,
                                                  RedArgs rd) {
#pragma clang fp contract(off)
    __shared__ double lds[8 * NS];
    int32_t rb, bq;
    if (!xcd_map(nblk, (sm.n + NS - 1) / NS, rb, bq, kGrpSmooth > NS ? kGrpSmooth / NS : 1)) return;
    int32_t bs[NS];
    bool act[NS];
    bool any = false;
#pragma unroll
    for (int t = 0; t < NS; ++t) {
        const int32_t l = bq * NS + t;
        bs[t] = sm_b(sm, l);
        act[t] = l < sm.n && !retired(sysi, bs[t]);
        any |= act[t];
    }
    if (!any) return;
    double rz[NS];
#pragma unroll
    for (int t = 0; t < NS; ++t) rz[t] = 0.0;
#pragma unroll
    for (int g = 0; g < kRows; ++g) {
        const int32_t i = rb * kRowsPerWG + g * kWG + threadIdx.x;
        if (i >= N) break;
        float y[NS][2];
        uint2 dg[NS];  // the rows' diagonal blocks (slot 0), kept from the SpMV
        auto xl = [&](int t, int32_t j) {
            const int64_t vj = (int64_t)bs[t] * N + j;
            if constexpr (XM == 2)
                return reinterpret_cast<const float2 *>(xv)[vj];
            else
                return ld_x0(xv, vj);
        };
        if (mat.sell_mir)
            spmv_row_hx_ns<true, NS, kPost0U>(mat, bs, i, xl, y, dg);
        else
            spmv_row_hx_ns<false, NS, kPost0U>(mat, bs, i, xl, y, dg);
#pragma unroll
        for (int t = 0; t < NS; ++t) {
            const int64_t vb = (int64_t)bs[t] * N;
            const float2 xi = xl(t, i);
            const float2 ri = reinterpret_cast<const float2 *>(rv)[vb + i];
            const float2 ds = bf16_diag_solve(dg[t], ri.x - y[t][0], ri.y - y[t][1]);
            float z0 = xi.x + omega * ds.x;
            float z1 = xi.y + omega * ds.y;
            if constexpr (ZH) {
                const uint32_t h = bf16_bits(z0) | (bf16_bits(z1) << 16);
                if (act[t]) reinterpret_cast<uint32_t *>(zv)[vb + i] = h;
                z0 = bf16_lo(h);
                z1 = bf16_hi(h);
            } else {
                if (act[t]) reinterpret_cast<float2 *>(zv)[vb + i] = make_float2(z0, z1);
            }
            if (i < rd.nown) rz[t] += (double)ri.x * z0 + (double)ri.y * z1;
        }
    }
    block_sum<NS>(rz, lds);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int t = 0; t < NS; ++t)
            if (act[t]) part[2 * (((int64_t)rd.part * B + bs[t]) * rd.nmax + rb)] = rz[t];
    }
}

// Open surfaces: `sweeps` extra block-Jacobi sweeps (damping omega, b = r)
// on the boundary rows and their neighbour ring only, after the fused
// pre-smoothing and before the post-smoothing (the cycle stays symmetric).
// At a Neumann boundary vertex the diagonal block lacks the missing
// triangles, so one damped sweep leaves those rows least smoothed.
// The ring is its own small SELL-64 matrix (per mesh, host-built: ring
// position p's slot t at bsw_roff[p/64] + 64 t + p%64, the same slots in the
// same order as the row's level-0 SELL slots, padding included): per slot
// the operand's source, a ring position (>= 0), an outside column (-1 - k:
// bsw_ocol[k]) or none (kBswOff), and per batch the slot's bf16 block
// gathered (transposed where the symmetric reads would) from the level-0
// sweep copy by k_bsw_extract. One workgroup per system: the ring's iterates
// (two buffers: a Jacobi sweep reads only the previous one) and the outside
// operands, which do not change, live in LDS; the blocks stream coalesced.
// The same products summed in the same order as spmv_row_hx_ns: the same
// bits as the level-0 kernels' arithmetic. Round 6: the first version read
// the ring rows' slots in place (three dependent trips per slot, one
// scattered line per block): 705 us per 2-sweep launch on S1, 1536 systems.
// F32X: x as fp32 pairs (the corrected iterate with xm = 2), else the bf16
// x0 format.
constexpr int kBswWG = 1024;
constexpr int32_t kBswOff = INT32_MIN;
constexpr int64_t kBswLdsMax = 160 * 1024;  // a workgroup may take the CU's whole LDS (gfx950)
struct BswArgs {
    int32_t N, nbr, nout, nslot;
    const int32_t *rows, *roff, *wrow, *xsrc, *ocol;
    const uint2 *A;  // [cap][nslot] blocks
};
template <bool F32X>
__device__ __forceinline__ float2 bsw_ldx(const float *xv, int64_t vj) {
    if constexpr (F32X)
        return reinterpret_cast<const float2 *>(xv)[vj];
    else
        return ld_x0(xv, vj);
}
// per batch: the ring slots' blocks of every system from the level-0 copy
__global__ __launch_bounds__(kWG) void k_bsw_extract(int32_t nslot, int32_t B, const int32_t *__restrict__ bsrc,
                                                     const uint2 *__restrict__ A0h, int64_t sell_nb,
                                                     uint2 *__restrict__ out) {
    const int64_t q = (int64_t)blockIdx.x * kWG + threadIdx.x;
    if (q >= (int64_t)nslot * B) return;
    const int32_t b = (int32_t)(q / nslot), t = (int32_t)(q - (int64_t)b * nslot);
    const int32_t src = bsrc[t];
    uint2 h = make_uint2(0u, 0u);
    if (src >= 0) {
        h = h0_ld(A0h, (int64_t)b * sell_nb + (src & kMirPos));
        if (src & kMirT) h = h0_tr(h);
    }
    out[q] = h;
}
template <bool F32X>
__global__ __launch_bounds__(kBswWG) void k_bsweep(BswArgs a, SysMap sm, const float *__restrict__ rv,
                                                   float *__restrict__ xv, float omega, int32_t sweeps,
                                                   const int32_t *__restrict__ sysi) {
#pragma clang fp contract(off)
    extern __shared__ float2 bsw_lds[];  // [2][nbr] iterates, [nout] outside operands
    if ((int32_t)blockIdx.x >= sm.n) return;
    const int32_t b = sm_b(sm, blockIdx.x);
    if (retired(sysi, b)) return;
    const int64_t vb = (int64_t)b * a.N;
    float2 *xs[2] = {bsw_lds, bsw_lds + a.nbr};
    float2 *xo = bsw_lds + 2 * a.nbr;
    for (int32_t p = threadIdx.x; p < a.nbr; p += kBswWG) xs[0][p] = bsw_ldx<F32X>(xv, vb + a.rows[p]);
    for (int32_t k = threadIdx.x; k < a.nout; k += kBswWG) xo[k] = bsw_ldx<F32X>(xv, vb + a.ocol[k]);
    __syncthreads();
    const uint2 *Ab = a.A + (int64_t)b * a.nslot;
    constexpr int U = kPost0U;
    int cur = 0;
    for (int32_t k = 0; k < sweeps; ++k) {
        for (int32_t p = threadIdx.x; p < a.nbr; p += kBswWG) {
            const int32_t base = a.roff[p >> 6] + (p & 63), w = a.wrow[p];
            const float2 ri = reinterpret_cast<const float2 *>(rv)[vb + a.rows[p]];
            float acc0 = 0.f, acc1 = 0.f;
            uint2 dg = make_uint2(0u, 0u);
            for (int32_t t0 = 0; t0 < w; t0 += U) {
                int32_t src[U];
                uint2 blk[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int32_t q = base + min(t0 + u, w - 1) * kSlice;
                    src[u] = a.xsrc[q];
                    blk[u] = Ab[q];
                }
                if (t0 == 0) dg = blk[0];  // slot 0: the diagonal block
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const bool on = t0 + u < w && src[u] != kBswOff;
                    float2 xj = make_float2(0.f, 0.f);
                    if (on) xj = src[u] >= 0 ? xs[cur][src[u]] : xo[-1 - src[u]];
                    float e00, e01, e10, e11;
                    h0_dec(blk[u], e00, e01, e10, e11);
                    acc0 += on ? e00 * xj.x + e01 * xj.y : 0.f;
                    acc1 += on ? e10 * xj.x + e11 * xj.y : 0.f;
                }
            }
            const float2 ds = bf16_diag_solve(dg, ri.x - acc0, ri.y - acc1);
            const float2 xi = xs[cur][p];
            xs[cur ^ 1][p] = make_float2(xi.x + omega * ds.x, xi.y + omega * ds.y);
        }
        __syncthreads();
        cur ^= 1;
    }
    for (int32_t p = threadIdx.x; p < a.nbr; p += kBswWG) {
        const float2 v = xs[cur][p];
        if constexpr (F32X)
            reinterpret_cast<float2 *>(xv)[vb + a.rows[p]] = v;
        else
            st_x0(xv, vb + a.rows[p], v.x, v.y);
    }
}
BswArgs bsw_args(const AmgDevice &G) {
    BswArgs a;
    a.N = G.bsw_N;
    a.nbr = G.bsw_n;
    a.nout = G.bsw_nout;
    a.nslot = G.bsw_nslot;
    a.rows = G.bsw_rows.p;
    a.roff = G.bsw_roff.p;
    a.wrow = G.bsw_wrow.p;
    a.xsrc = G.bsw_xsrc.p;
    a.ocol = G.bsw_ocol.p;
    a.A = reinterpret_cast<const uint2 *>(G.bsw_A.p);
    return a;
}
template <bool F32X>
void launch_bsweep(const AmgDevice &G, SysMap sm, const float *rv, float *xv, float omega, const int32_t *sysi,
                   hipStream_t s) {
    const size_t lds = sizeof(float2) * (2 * (size_t)G.bsw_n + G.bsw_nout);
    k_bsweep<F32X><<<dim3((unsigned)sm.n), kBswWG, lds, s>>>(bsw_args(G), sm, rv, xv, omega, G.bsw_sweeps, sysi);
}

template <int XM, bool ZH, typename... Args>
void launch_post0(int32_t nblk, int32_t B, hipStream_t s, Args... args) {
    const dim3 g(xcd_grid(nblk, (B + kPost0NS - 1) / kPost0NS, kGrpSmooth > kPost0NS ? kGrpSmooth / kPost0NS : 1));
    k_post0_ns<XM, ZH, kPost0NS><<<g, kWG, 0, s>>>(args...);
}

inline dim3 grid2(int64_t n, int32_t B) { return dim3((unsigned)((n + kWG - 1) / kWG), (unsigned)B); }

MatH level0_mat(mof_mesh *m) {
    MatH mt;
    mt.sell_nb = m->pat.sell_nb();
    mt.sell_off = m->sell_off.p;
    mt.sell_col = m->sell_col.p;
    mt.sell_mir = m->sym_reads ? m->sell_mir.p : nullptr;
    mt.vptr = m->sym_reads ? nullptr : m->vptr.p;
    mt.A = reinterpret_cast<const uint2 *>(m->amg->A0h.p);
    return mt;
}

}  // namespace

// ---- host side ---------------------------------------------------------------

bool amg_build(mof_mesh *m) {
    AmgParams prm;
    // an open surface (boundary edges: 3 M != 2 E) damps the fine smoother
    // more: at a Neumann boundary vertex the diagonal block lacks the missing
    // triangles while its couplings stay, and 0.85 leaves the block-Jacobi
    // sweep non-contractive there -- round 4, the S1-like patches: every
    // multigrid solve broke down at 0.85 (3,249 and 160,801 vertices), none at
    // 0.7 (S1s 22.5 PCG its/timestep); on the closed meshes 0.7 costs C3
    // 17.0 -> 18.5 its (-7 %) and C2 21.6 -> 23.0, R3 51.4 -> 50.6
    // (profiles/r04_ab/call4/). A decomposed part keeps 0.85 (its ghost rows
    // are decoupled, not a Neumann boundary).
    const bool open_surface = [&] {
        const int64_t E = ((int64_t)m->pat.nblocks() - m->N) / 2;
        return m->n_own == m->N && 3 * (int64_t)m->M != 2 * E;
    }();
    // and takes the smoothed prolongator (the translations an open patch
    // nearly leaves free converge slowly on the tentative one: S1, 160,801
    // vertices, 86 -> 51.5 PCG its/timestep; the 3,249-vertex S1s is
    // irregular enough to have it already)
    if (open_surface) {
        prm.omega = 0.7f;
        prm.smooth = 1;
    }
    // MOF_AMG_OMEGA = w0[,w1]: the fine [and coarse] smoother damping
    float omega1_set = 0.f;
    if (const char *v = knob(Knob::AmgOmega)) {
        char *end = nullptr;
        prm.omega = std::strtof(v, &end);
        if (end && *end == ',') omega1_set = prm.omega1 = std::strtof(end + 1, nullptr);
    }
    if (knob(Knob::AmgSmooth)) prm.smooth = knob_int(Knob::AmgSmooth, 0) != 0;  // 1 / 0 force, unset auto
    // level 1's smoothed prolongator: auto (below: where level 0 is smoothed,
    // and folded closed surfaces)
    prm.smooth1 = -1;
    if (m->n_own < m->N) prm.nown = m->n_own;
    if (m->amg && m->amg->built) return m->amg->lv.size() >= 2;
    if (!m->amg) m->amg = new AmgDevice();
    AmgDevice &G = *m->amg;
    hipStream_t s = m->stream;
    // the host hierarchy of this mesh and parameter set: built once per mesh
    // and shared by its handles on other devices (MeshShared); the inputs
    // (pattern, e, a2) are the same on every device, bit for bit
    MeshShared *sh = m->shared.get();
    char key[160];
    std::snprintf(key, sizeof(key), "%a/%a/%d/%d/%a/%d/%d", (double)prm.omega, (double)prm.omega1, prm.smooth,
                  prm.nown, (double)prm.smooth_omega, (int)m->sym_reads, prm.smooth1);
    std::unique_lock<std::mutex> build_lock;
    std::shared_ptr<const AmgHierarchy> Hp;
    if (sh) {
        build_lock = std::unique_lock<std::mutex>(sh->amg_build_mu);
        std::lock_guard<std::mutex> lk(sh->mu);
        for (const auto &kv : sh->amg)
            if (kv.first == key) Hp = kv.second;
    }
    if (!Hp) {
        std::vector<double> e(6 * (size_t)m->N);
        MOF_HIP(hipMemcpyAsync(e.data(), m->e.p, e.size() * sizeof(double), hipMemcpyDeviceToHost, s));
        MOF_HIP(hipStreamSynchronize(s));
        // the mesh's a2 (unscaled, fine SELL layout) for the smoothed prolongator
        std::vector<double> a2;
        if (prm.nown < 0 && ((prm.smooth != 0 && (prm.smooth > 0 || amg_auto_smooth(m->pat))) || prm.smooth1 != 0)) {
            a2.resize(4 * (size_t)m->pat.sell_nb());
            MOF_HIP(hipMemcpyAsync(a2.data(), m->a2.p, a2.size() * sizeof(double), hipMemcpyDeviceToHost, s));
            MOF_HIP(hipStreamSynchronize(s));
            prm.a2 = a2.data();
        }
        if (!m->agg_order.empty()) prm.order = m->agg_order.data();
        std::vector<int32_t> mir;
        if (m->sym_reads) {
            mir = sell_mirror(m->pat, m->n_own, 1, nullptr);
            prm.mirror = mir.data();
        }
        auto built = std::make_shared<AmgHierarchy>();
        AmgParams p1 = prm;
        // level 1 smoothed at once where level 0 is (irregular or open
        // surfaces): round 5, same box (profiles/r05_ab/sa1/): R3 742 ->
        // 842 timesteps/s (53.6 -> 41.8 PCG its), S1 905 (with the level-1
        // W-cycle, since removed) -> 995 (44.8 its)
        const bool l0_smooth = prm.nown < 0 && prm.a2 && prm.smooth != 0 && (prm.smooth > 0 || amg_auto_smooth(m->pat));
        p1.smooth1 = prm.smooth1 > 0 ? prm.smooth1 : (prm.smooth1 < 0 && l0_smooth ? 1 : 0);
        // open surfaces: every explicit coarse level smoothed (with the
        // boundary sweeps below; round 6, same box, profiles/r06/bsw/): S1
        // 1,188 -> 1,377 timesteps/s, 42.9 -> 35.5 PCG its (alone, without the
        // sweeps: 1,121 at 46.1 its -- the CPU prototype agrees, 36 -> 36
        // its to 1e-8 alone, 30 with them, tools/amg_proto.py); S1m / S1s
        // have no explicit level past 1 (the same hierarchy)
        if (open_surface && p1.smooth1 == 1) p1.smooth1 = 2;
        build_amg(m->pat, e.data(), p1, *built);
        // auto: a closed surface whose coarse aggregates turn strongly (the
        // median sigma_3 / sigma_1 of their near-null blocks >= kFoldCurl at
        // some level: folds at the coarse levels' scale) is rebuilt with
        // level 1's prolongator smoothed, and level 0's too where the finest
        // aggregates stay flat (curl[0] < kFlatCurl: a folded surface, not a
        // rough one -- the 640k jittered sphere C5 turns 0.34 at level 0 and
        // loses 9 % with level 0 smoothed, 945 -> 859 timesteps/s at 15.2 ->
        // 13.0 its, profiles/r06/sweep/C5.json; F3 turns 0.07 there;
        // MOF_AMG_SMOOTH = 0 keeps level 0 tentative). Round 5, same box
        // (profiles/r05_ab/sa1/): level 1 alone, F3 (curl 0.46-0.51) 2003 ->
        // 2292 timesteps/s, 31.0 -> 26.2 PCG its; C3 (curl <= 0.25) gains no
        // iteration (17.0) and loses 12 % to the level-1 product. Round 6,
        // same box (profiles/r06/f3_fold/): level 0 as well, with the
        // regular mesh's storage formats kept (below), F3 2548 / 2584 ->
        // 2794 / 2797 timesteps/s, 26.2 -> 17.5 its (level 0 smoothed with
        // the irregular meshes' fp32 iterates: 19.0 its, 2546)
        if (prm.smooth1 < 0 && p1.smooth1 == 0 && prm.nown < 0 && prm.a2 && !built->levels.empty() &&
            !built->levels[0].smoothed && built->max_curl >= kFoldCurl) {
            const double curl = built->max_curl;
            p1.smooth1 = 1;
            if (prm.smooth != 0 && !built->curl.empty() && built->curl[0] < kFlatCurl) p1.smooth = 1;
            auto again = std::make_shared<AmgHierarchy>();
            build_amg(m->pat, e.data(), p1, *again);
            again->max_curl = curl;
            again->folded = true;
            built = again;
        }
        Hp = built;
        if (sh) {
            std::lock_guard<std::mutex> lk(sh->mu);
            sh->amg.emplace_back(key, Hp);
        }
    }
    if (build_lock.owns_lock()) build_lock.unlock();
    const AmgHierarchy &H = *Hp;
    G.omega = prm.omega;
    G.omega1 = prm.omega1;
    // level 0's corrected iterate x0 + Q y: bf16 in place on meshes with the
    // tentative prolongator (C3 +3.8 %, C2 mixed +3.3 %, same iterations),
    // fp32 with the smoothed one (R3: bf16 costs 54.5 vs 50 its, -5 %)
    G.xm = 2;
    G.lv.clear();
    G.built = true;
    // a mesh that does not coarsen (<= 42 vertices) keeps block Jacobi
    if (H.levels.size() < 2) return false;
    // The bf16 iterates (x here, z in the PCG) and omega1 = 1.1 were tuned on
    // the regular meshes; an irregular mesh keeps fp32 and 1.05 whichever
    // prolongator it runs (round 3: R3 forced onto the tentative P took
    // 146.5 PCG its/timestep with the regular meshes' choices)
    // (round 4: and closed -- an open patch's near-null modes suffer from
    // the bf16 iterates as from the stronger coarse damping). The choice
    // follows the mesh, not the prolongator: a regular closed mesh keeps
    // them with a smoothed level 0 too (round 6: F3 folded 17.5 its, +9 %;
    // C3 forced smoothed, round 5: 3653-3730 vs 3253-3268 timesteps/s
    // without them)
    G.regular = !amg_auto_smooth(m->pat) && !open_surface;
    G.xm = G.regular ? 1 : 2;
    // coarse-level damping: 1.1 on regular meshes (round 2, C3 17.2 -> 17.0
    // its, +1.8 %; C2 mixed +2 %), 1.05 otherwise (R3 as measured; 1.2
    // diverges there with the tentative P)
    if (omega1_set <= 0.f) G.omega1 = G.regular ? 1.1f : 1.05f;
    // (a W-cycle at level 1 -- the levels below visited twice -- was
    // measured in rounds 5-6 and removed: slower than level 1's smoothed
    // prolongator on every mesh (S1 905 vs 995, F3 1934 vs 2292, C3 3370 vs
    // 3652 timesteps/s, profiles/r05_ab/wcycle/), and together with it it
    // broke 15 of 3072 S1 solves down: the cycle below level 1 over-corrects
    // there (lambda(B2 A2) up to 2.2 with the coarse damping 1.05,
    // tools/wcycle_study.py), which a V-cycle tolerates and the second
    // coarse correction of a W-cycle does not)
    MOF_REQUIRE(H.coarse_dofs <= kMaxCoarse, "coarsest multigrid level too large");
    MOF_REQUIRE(H.levels.size() <= (size_t)kMaxLevels, "too many multigrid levels");
    G.lv.resize(H.levels.size());
    auto put_i = [&](DevArray<int32_t> &d, const std::vector<int32_t> &h) {
        d.alloc(h.size());
        if (!h.empty()) d.upload(h.data(), h.size(), s);
    };
    auto put_f = [&](DevArray<float> &d, const std::vector<float> &h) {
        d.alloc(h.size());
        if (!h.empty()) d.upload(h.data(), h.size(), s);
    };
    // open surfaces: the boundary rows (fewer incident triangles than
    // neighbours: the diagonal block's contribution list has one entry per
    // incident triangle) and one ring of their neighbours, for k_bsweep: 2
    // sweeps per side on every open surface whose ring fits the sweep
    // kernel's LDS (a larger ring keeps no boundary sweeps, said under
    // MOF_VERBOSE); MOF_AMG_BSW = sweeps per side (0 off). Round 5 (one
    // workgroup reading the ring rows in place, 705 us per launch on S1) ran
    // them only where the ring is >= 1/20 of the rows (S1s, 14 %: 28.6 ->
    // 19.8 PCG its/timestep); round 6, the ring as its own SELL matrix (180
    // us), same box (profiles/r06/bsw/): S1s 27,458 -> 29,287 timesteps/s
    // (same bits), S1m (ring 4 %) 4,646 -> 6,012 at 43.9 -> 30.9 its, S1
    // (2 %, with its coarse levels smoothed, above) 1,148 -> 1,377.
    G.bsw_n = 0;
    G.bsw_sweeps = 0;
    int32_t bsw = -1;
    if (knob(Knob::AmgBsw)) bsw = std::max(0, std::min(8, knob_int(Knob::AmgBsw, 0)));
    if (open_surface && bsw != 0) {
        const Pattern &P = m->pat;
        std::vector<uint8_t> mark(m->N, 0);
        for (int32_t i = 0; i < m->N; ++i) {
            const int32_t a = P.vptr[i], e2 = P.vptr[i + 1];
            const int32_t d = (int32_t)(std::lower_bound(P.vcol.begin() + a, P.vcol.begin() + e2, i) - P.vcol.begin());
            if (P.cptr[d + 1] - P.cptr[d] < e2 - a - 1) mark[i] = 1;
        }
        std::vector<uint8_t> ring(mark);
        for (int32_t i = 0; i < m->N; ++i)
            if (mark[i])
                for (int32_t q = P.vptr[i]; q < P.vptr[i + 1]; ++q) ring[P.vcol[q]] = 1;
        std::vector<int32_t> rows, pos(m->N, -1);
        for (int32_t i = 0; i < m->N; ++i)
            if (ring[i]) {
                pos[i] = (int32_t)rows.size();
                rows.push_back(i);
            }
        if (!rows.empty()) {
            // the ring's SELL-64 matrix: ring position p's slots are row
            // rows[p]'s level-0 slots (spmv_row_hx_ns's order and masks)
            const int32_t nbr = (int32_t)rows.size(), nrs = (nbr + kSlice - 1) / kSlice;
            std::vector<int32_t> mir;
            if (m->sym_reads) mir = sell_mirror(P, m->n_own, 1, nullptr);
            std::vector<int32_t> wrow(nbr), roff(nrs + 1, 0), ocol, opos(m->N, -1);
            for (int32_t p = 0; p < nbr; ++p) {
                const int32_t s0 = rows[p] / kSlice;
                wrow[p] = (int32_t)((P.sell_off[s0 + 1] - P.sell_off[s0]) / kSlice);
            }
            for (int32_t r = 0; r < nrs; ++r) {
                int32_t wmax = 0;
                for (int32_t p = r * kSlice; p < std::min(nbr, (r + 1) * kSlice); ++p) wmax = std::max(wmax, wrow[p]);
                roff[r + 1] = roff[r] + wmax * kSlice;
            }
            const int32_t nslot = roff[nrs];
            std::vector<int32_t> xsrc(nslot, kBswOff), bsrc(nslot, -1);
            for (int32_t p = 0; p < nbr; ++p) {
                const int32_t i = rows[p], s0 = i / kSlice, l = i % kSlice;
                const int64_t o = P.sell_off[s0];
                const int32_t w = wrow[p];
                const int32_t wl = m->sym_reads ? w : std::min(w, P.vptr[i + 1] - P.vptr[i]);
                for (int32_t t = 0; t < w; ++t) {
                    const int64_t pp = o + (int64_t)std::min(t, wl - 1) * kSlice + l;
                    const int32_t j = P.sell_col[pp];
                    int32_t src = (int32_t)pp;
                    bool on = t < wl;
                    if (m->sym_reads) {
                        const int32_t mr = mir[pp];
                        on = on && mr >= 0;
                        src = mr < 0 ? (int32_t)(o + l) : mr;  // position | kMirT (transposed)
                    }
                    if (!on) continue;
                    const int64_t q = roff[p / kSlice] + (int64_t)t * kSlice + p % kSlice;
                    bsrc[q] = src;
                    if (pos[j] >= 0) {
                        xsrc[q] = pos[j];
                    } else {
                        if (opos[j] < 0) {
                            opos[j] = (int32_t)ocol.size();
                            ocol.push_back(j);
                        }
                        xsrc[q] = -1 - opos[j];
                    }
                }
            }
            const int64_t lds = (int64_t)sizeof(float2) * (2 * (int64_t)nbr + (int64_t)ocol.size());
            if (lds > kBswLdsMax) {
                if (knob(Knob::Verbose))
                    std::fprintf(stderr, "mof amg: boundary ring of %d rows needs %lld B of LDS: no boundary sweeps\n",
                                 nbr, (long long)lds);
            } else {
                put_i(G.bsw_rows, rows);
                put_i(G.bsw_roff, roff);
                put_i(G.bsw_wrow, wrow);
                put_i(G.bsw_xsrc, xsrc);
                put_i(G.bsw_bsrc, bsrc);
                put_i(G.bsw_ocol, ocol);
                G.bsw_N = m->N;
                G.bsw_n = nbr;
                G.bsw_nout = (int32_t)ocol.size();
                G.bsw_nslot = nslot;
                G.bsw_sweeps = bsw > 0 ? bsw : 2;
                if (knob(Knob::Verbose))
                    std::fprintf(stderr, "mof amg: boundary sweeps x%d on a ring of %d rows (%d outside, %lld B of LDS)\n",
                                 G.bsw_sweeps, nbr, G.bsw_nout, (long long)lds);
                if (lds > 64 * 1024) {
                    MOF_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_bsweep<true>),
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                    MOF_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_bsweep<false>),
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                }
            }
        }
    }
    for (size_t l = 0; l < H.levels.size(); ++l) {
        const AmgLevel &L = H.levels[l];
        AmgDevLevel &D = G.lv[l];
        D.n = L.n;
        D.bs = L.bs;
        D.sell_nb = L.sell_nb();
        if (l > 0) {
            {  // each upper block's lower twin (st_pair), -1 elsewhere
                std::vector<int32_t> tw((size_t)L.sell_nb(), -1);
                for (size_t k = 0; k < L.low.size(); ++k) tw[L.twin[k]] = L.low[k];
                put_i(D.twin, tw);
            }
            put_i(D.sell_off, L.sell_off);
            put_i(D.sell_col, L.sell_col);
            put_i(D.sell_row, L.sell_row);
            put_i(D.diag_pos, L.diag_pos);
            D.dead.alloc(L.dead.size());
            D.dead.upload(L.dead.data(), L.dead.size(), s);
        }
        if (l + 1 < H.levels.size()) {
            put_i(D.agg, L.agg);
            put_i(D.mptr, L.mptr);
            put_i(D.mlist, L.mlist);
            put_i(D.apos, L.apos);
            put_i(D.gptr, L.gptr);
            put_i(D.gent, L.gent);
            put_f(D.Q, L.Q);
            put_f(D.Qm, L.Qm);
            D.smoothed = L.smoothed;
            if (L.smoothed) {
                put_i(D.pptr, L.pptr);
                put_i(D.pcol, L.pcol);
                put_i(D.rptr, L.rptr);
                put_i(D.rent, L.rent);
            }
            // restriction groups: whole aggregates, <= kRG members (smoothed P:
            // restriction list entries) each
            std::vector<int32_t> grp{0};
            const std::vector<int32_t> &gp = L.smoothed ? L.rptr : L.mptr;
            const int32_t na = (int32_t)gp.size() - 1;
            for (int32_t I = 0; I < na; ++I) {
                const int32_t g0 = grp.back();
                if (I > g0 && gp[I + 1] - gp[g0] > (L.smoothed ? kRGS : kRG)) grp.push_back(I);
            }
            grp.push_back(na);
            D.ngrp = (int32_t)grp.size() - 1;
            put_i(D.rgrp, grp);
            // smoothed P: each group's list entries by fine node (stable), for
            // k_restrict0_sa's gathers (same bits as list order)
            if (L.smoothed) {
                std::vector<int32_t> perm(L.rent.size() / 2);
                for (int32_t g = 0; g + 1 < (int32_t)grp.size(); ++g) {
                    const int32_t e0 = L.rptr[grp[g]], e1 = L.rptr[grp[g + 1]];
                    for (int32_t e = e0; e < e1; ++e) perm[e] = e;
                    std::stable_sort(perm.begin() + e0, perm.begin() + e1,
                                     [&](int32_t x, int32_t y) { return L.rent[2 * x] < L.rent[2 * y]; });
                }
                put_i(D.rperm, perm);
            }
            // tentative P (every level but a smoothed level 0): coarse position
            // ranges of <= kWG gather entries and positions for the products by
            // entry, k_galerkin0_ent / k_galerkin3_ent (unless a level-0
            // position has more). Levels >= 1: positions past kGalBig entries
            // go to k_galerkin3_big.
            if (!L.smoothed || l >= 1) {
                const int32_t big = l == 0 ? 0 : std::min<int32_t>(kWG, kGalBig);
                const std::vector<int32_t> &gq = L.gptr;
                const int32_t npos = (int32_t)gq.size() - 1;
                bool ok = true;
                for (int32_t p = 0; p < npos && ok; ++p) ok = big > 0 || gq[p + 1] - gq[p] <= kWG;
                if (ok) {
                    // [p0, p1) pairs of consecutive positions within the bound;
                    // a big position closes the open range
                    std::vector<int32_t> gg, gbig;
                    int32_t p0 = -1;
                    for (int32_t p = 0; p < npos; ++p) {
                        const bool isbig = big > 0 && gq[p + 1] - gq[p] > big;
                        if (p0 >= 0 && (isbig || gq[p + 1] - gq[p0] > kWG || p - p0 >= kWG)) {
                            gg.push_back(p0);
                            gg.push_back(p);
                            p0 = -1;
                        }
                        if (isbig)
                            gbig.push_back(p);
                        else if (p0 < 0)
                            p0 = p;
                    }
                    if (p0 >= 0) {
                        gg.push_back(p0);
                        gg.push_back(npos);
                    }
                    D.nggrp = (int32_t)gg.size() / 2;
                    put_i(D.ggrp, gg);
                    D.nbig = (int32_t)gbig.size();
                    put_i(D.gbig, gbig);
                }
            }
        }
    }
    G.nc = H.coarse_dofs;
    G.cap = 0;
    if (knob(Knob::Verbose)) {
        for (size_t l = 0; l < H.levels.size(); ++l)
            std::fprintf(stderr, "mof amg level %zu: n=%d bs=%d blocks=%zu sell=%lld%s curl %.3f%s\n", l,
                         H.levels[l].n, H.levels[l].bs, H.levels[l].vcol.size(), (long long)H.levels[l].sell_nb(),
                         H.levels[l].smoothed ? " (smoothed P)" : "", l < H.curl.size() ? H.curl[l] : 0.0,
                         l == 0 && H.folded ? " (folded)" : "");
    }
    MOF_HIP(hipStreamSynchronize(s));
    return true;
}

void amg_ensure(mof_mesh *m, int32_t B) {
    AmgDevice &G = *m->amg;
    if (G.cap >= B) return;
    hipStream_t s = m->stream;
    for (size_t l = 0; l < G.lv.size(); ++l) {
        AmgDevLevel &D = G.lv[l];
        const size_t n = D.n;
        if (l == 0) {
            D.x.alloc(2 * n * B);
            if (G.xm == 2) D.y.alloc(2 * n * B);
            D.r.alloc(n * B);  // bf16 pairs (ldr<2>)
            G.A0h.alloc((size_t)(2 * m->pat.sell_nb() * B));  // 8 B per block
            G.A0h.zero(s);  // SELL padding: never written by the assembly, read as 0
            // the smoothed level-0 Galerkin product by system slab (k_a_slab,
            // k_galerkin_sys)
            if (D.smoothed && G.aslab.n == 0) G.aslab.alloc((size_t)4 * kSlab * m->pat.sell_nb());
        } else {
            D.A.alloc((size_t)kB3 * D.sell_nb * B);
            D.A.zero(s);
            // (a level 1 of the fused tiny levels keeps its product by entry:
            // S1s, 400 nodes, 25050 -> 26450 timesteps/s without the chain)
            if (l == 1 && G.aslab.n > 0 && G.lv.size() >= 3 && D.n > kSubNodes && D.slab.n == 0)
                D.slab.alloc((size_t)kB3 * kSlab * D.sell_nb);
            if (l + 1 < G.lv.size()) {  // sweep copy, st_a9 (the coarsest stays fp32)
                D.Ah.alloc(kAhWords * D.sell_nb * B);
                D.Ah.zero(s);
                D.Ah22.alloc(kAh22Words * D.sell_nb * B);
                D.Ah22.zero(s);
            }
            D.Dh.alloc((size_t)4 * n * B);
            D.Dh22.alloc((size_t)n * B);
            D.b.alloc(4 * n * B);
            D.x.alloc(4 * n * B);
            D.r.alloc(4 * n * B);
            D.y.alloc(4 * n * B);
        }
    }
    G.cinv.alloc((size_t)G.nc * G.nc * B);
    if (G.bsw_n > 0) G.bsw_A.alloc((size_t)2 * G.bsw_nslot * B);  // the ring slots' blocks (uint2)
    G.cap = B;
    MOF_HIP(hipStreamSynchronize(s));
}

AmgBf16 amg_bf16_targets(mof_mesh *m, int32_t B) {
    AmgDevice &G = *m->amg;
    MOF_REQUIRE(G.cap >= B, "multigrid storage not sized for the batch");
    G.bf16_fresh = true;
    return AmgBf16{reinterpret_cast<uint2 *>(G.A0h.p)};
}

AmgFine amg_fine(mof_mesh *m) {
    AmgDevice &G = *m->amg;
    AmgFine f;
    f.A0h = G.A0h.p;
    f.sell_nb = m->pat.sell_nb();
    f.sell_off = m->sell_off.p;
    f.x0 = G.lv[0].x.p;
    f.omega = G.omega;
    f.smoothed = G.lv[0].smoothed;
    f.regular = G.regular;
    return f;
}

static uint4 *ah(AmgDevLevel &C) { return C.Ah.n > 1 ? reinterpret_cast<uint4 *>(C.Ah.p) : nullptr; }
static uint16_t *ah22(AmgDevLevel &C) { return C.Ah22.n > 1 ? C.Ah22.p : nullptr; }
static uint4 *dh(AmgDevLevel &C) { return reinterpret_cast<uint4 *>(C.Dh.p); }

void amg_setup_batch(mof_mesh *m, int32_t B, hipStream_t s) {
    AmgDevice &G = *m->amg;
    Workspace &w = m->ws;
    const size_t L = G.lv.size();
    if (!G.bf16_fresh) {
        const int64_t nb0 = m->pat.sell_nb() * B;
        k_to_h0<<<dim3((unsigned)((nb0 + kWG - 1) / kWG)), kWG, 0, s>>>(
            nb0, reinterpret_cast<const float4 *>(w.A32.p), reinterpret_cast<uint2 *>(G.A0h.p));
    }
    G.bf16_fresh = false;
    if (G.bsw_n > 0) {
        const int64_t n = (int64_t)G.bsw_nslot * B;
        k_bsw_extract<<<dim3((unsigned)((n + kWG - 1) / kWG)), kWG, 0, s>>>(
            G.bsw_nslot, B, G.bsw_bsrc.p, reinterpret_cast<const uint2 *>(G.A0h.p), m->pat.sell_nb(),
            reinterpret_cast<uint2 *>(G.bsw_A.p));
    }
    // a dispatch's grid is at most 2^32 - 1 work-items: a by-entry product
    // whose (group, system pair) grid would pass it (a batch of 1024 over
    // more than ~32k entry groups) takes the per-position kernel -- the same
    // terms in the same order, bit-identical (round 4: an unsliced by-entry
    // launch past the bound skipped workgroups)
    auto fits = [&](int32_t nblk, int32_t ns) {
        const int64_t nq = (B + ns - 1) / ns, G = sys_group((int32_t)nq, kGrpGal);
        return 8 * G * ((nq + G - 1) / G) * ((nblk + 7) / 8) * kWG < ((int64_t)1 << 32);
    };
    auto ent_fits = [&](const AmgDevLevel &F) {
        return (F.nggrp > 0 || F.nbig > 0) && fits(F.nggrp, kGalENS) && fits(F.nbig, kGalBigNS);
    };
    // a smoothed level 0: its product, and level 1's when level 1 kept a
    // slab copy, by system slab (k_a_slab -> k_galerkin_sys<2> -> <3>)
    size_t l_first = 0;
    if (G.lv[0].smoothed && G.aslab.n > 0) {
        AmgDevLevel &F = G.lv[0], &C = G.lv[1];
        const bool l1 = L >= 3 && C.slab.n > 0;
        const int64_t fnb = m->pat.sell_nb();
        auto sys_grid = [](int64_t nb) { return dim3(xcd_grid((int32_t)((nb + kGalSysPos - 1) / kGalSysPos), 1, 1)); };
        for (int32_t b0 = 0; b0 < B; b0 += kSlab) {
            const dim3 gs((unsigned)((fnb + kSlabPos - 1) / kSlabPos));
            if (G.regular)
                k_a_slab<uint2><<<gs, kWG, 0, s>>>(fnb, b0, std::min(kSlab, B - b0),
                                                   reinterpret_cast<const uint2 *>(G.A0h.p),
                                                   reinterpret_cast<uint2 *>(G.aslab.p));
            else
                k_a_slab<float4><<<gs, kWG, 0, s>>>(fnb, b0, std::min(kSlab, B - b0),
                                                    reinterpret_cast<const float4 *>(w.A32.p),
                                                    reinterpret_cast<float4 *>(G.aslab.p));
            auto *cs = l1 ? reinterpret_cast<float4 *>(C.slab.p) : nullptr;
            if (G.regular)
                k_galerkin_sys<2, true><<<sys_grid(C.sell_nb), kWG, 0, s>>>(
                    C.sell_nb, C.n, B, b0, C.sell_row.p, C.diag_pos.p, C.dead.p, C.twin.p, F.gptr.p, F.gent.p, F.Q.p,
                    reinterpret_cast<const float4 *>(G.aslab.p), C.A.p, dh(C), C.Dh22.p, ah(C), ah22(C), cs);
            else
                k_galerkin_sys<2><<<sys_grid(C.sell_nb), kWG, 0, s>>>(
                    C.sell_nb, C.n, B, b0, C.sell_row.p, C.diag_pos.p, C.dead.p, C.twin.p, F.gptr.p, F.gent.p, F.Q.p,
                    reinterpret_cast<const float4 *>(G.aslab.p), C.A.p, dh(C), C.Dh22.p, ah(C), ah22(C), cs);
            if (l1) {
                AmgDevLevel &C2 = G.lv[2];
                k_galerkin_sys<3><<<sys_grid(C2.sell_nb), kWG, 0, s>>>(
                    C2.sell_nb, C2.n, B, b0, C2.sell_row.p, C2.diag_pos.p, C2.dead.p, C2.twin.p, C.gptr.p, C.gent.p, C.Q.p,
                    reinterpret_cast<const float4 *>(C.slab.p), C2.A.p, dh(C2), C2.Dh22.p, ah(C2), ah22(C2), nullptr);
            }
        }
        l_first = l1 ? 2 : 1;
    }
    for (size_t l = l_first; l + 1 < L; ++l) {
        AmgDevLevel &F = G.lv[l], &C = G.lv[l + 1];
        const bool ent = ent_fits(F);
        if (l == 0 && ent)
            k_galerkin0_ent<<<dim3(xcd_grid(F.nggrp, (B + kGalENS - 1) / kGalENS, kGrpGal)), kWG, 0, s>>>(
                F.nggrp, F.ggrp.p, C.n, B, C.sell_row.p, C.diag_pos.p, C.dead.p, C.twin.p, F.gptr.p, F.gent.p, F.Q.p,
                reinterpret_cast<const uint2 *>(G.A0h.p), m->pat.sell_nb(), C.sell_nb, C.A.p, dh(C), C.Dh22.p, ah(C),
                ah22(C));
        else if (l == 0)
            k_galerkin0_ns<<<dim3(xcd_grid((int32_t)((C.sell_nb + kWG - 1) / kWG), (B + kGalNS - 1) / kGalNS,
                                           kGrpGal)),
                             kWG, 0, s>>>(C.sell_nb, C.n, B, C.sell_row.p, C.diag_pos.p, C.dead.p, C.twin.p, F.gptr.p, F.gent.p,
                                          F.Q.p, w.A32.p, m->pat.sell_nb(), C.A.p, dh(C), C.Dh22.p, ah(C), ah22(C),
                                          F.smoothed ? nullptr : reinterpret_cast<const uint2 *>(G.A0h.p));
        else if (ent) {
            if (F.nggrp > 0)
                k_galerkin3_ent<<<dim3(xcd_grid(F.nggrp, (B + kGalENS - 1) / kGalENS, kGrpGal)), kWG, 0, s>>>(
                    F.nggrp, F.ggrp.p, C.n, B, C.sell_row.p, C.diag_pos.p, C.dead.p, C.twin.p, F.gptr.p, F.gent.p, F.Q.p, F.A.p,
                    F.sell_nb, C.sell_nb, C.A.p, dh(C), C.Dh22.p, ah(C), ah22(C));
            if (F.nbig > 0)
                k_galerkin3_big<kGalBigNS>
                    <<<dim3(xcd_grid(F.nbig, (B + kGalBigNS - 1) / kGalBigNS, kGrpGal)), kWG, 0, s>>>(
                        F.nbig, F.gbig.p, C.n, B, C.sell_row.p, C.diag_pos.p, C.dead.p, C.twin.p, F.gptr.p, F.gent.p, F.Q.p,
                        F.A.p, F.sell_nb, C.sell_nb, C.A.p, dh(C), C.Dh22.p, ah(C), ah22(C));
        } else
            k_galerkin3_ns<kGal3NS>
                <<<dim3(xcd_grid((int32_t)((C.sell_nb + kWG - 1) / kWG), (B + kGal3NS - 1) / kGal3NS, kGrpGal)), kWG,
                   0, s>>>(C.sell_nb, C.n, B, C.sell_row.p, C.diag_pos.p, C.dead.p, C.twin.p, F.gptr.p, F.gent.p, F.Q.p, F.A.p,
                           F.sell_nb, C.A.p, dh(C), C.Dh22.p, ah(C), ah22(C));
    }
    AmgDevLevel &Lc = G.lv[L - 1];
    k_coarse_inverse<<<dim3((unsigned)B), kInvWG, 0, s>>>(Lc.n, Lc.sell_off.p, Lc.sell_col.p, Lc.A.p,
                                                       Lc.sell_nb, G.cinv.p);
    MOF_HIP(hipGetLastError());
}

Lvl level_view(const AmgDevLevel &D) {
    Lvl v;
    v.n = D.n;
    v.sell_nb = D.sell_nb;
    v.sell_off = D.sell_off.p;
    v.sell_col = D.sell_col.p;
    v.A = D.A.p;
    v.Dh = reinterpret_cast<const uint4 *>(D.Dh.p);
    v.Dh22 = D.Dh22.p;
    v.Ah = D.Ah.n > 1 ? reinterpret_cast<const uint4 *>(D.Ah.p) : nullptr;
    v.Ah22 = D.Ah22.n > 1 ? D.Ah22.p : nullptr;
    v.b = D.b.p;
    v.x = D.x.p;
    v.r = D.r.p;
    v.y = D.y.p;
    v.agg = D.agg.p;
    v.mptr = D.mptr.p;
    v.mlist = D.mlist.p;
    v.apos = D.apos.p;
    v.Q = D.Q.p;
    v.Qm = D.Qm.p;
    v.pptr = D.pptr.p;
    v.pcol = D.pcol.p;
    v.rptr = D.rptr.p;
    v.rent = D.rent.p;
    v.rperm = D.rperm.n > 0 ? D.rperm.p : nullptr;
    return v;
}

void amg_vcycle(mof_mesh *m, int32_t B, const float *r0, float *z0, double *part_slot, int32_t nblk,
                const RedArgs &rd, hipStream_t s, bool zh, const int32_t *smap, int32_t nl) {
    AmgDevice &G = *m->amg;
    Workspace &w = m->ws;
    const int32_t L = (int32_t)G.lv.size();
    const int32_t *sysi = w.sysi.p;
    const float om = G.omega;
    const float om1 = G.omega1;  // levels >= 1
    const MatH mat0 = level0_mat(m);
    Lvl v[kMaxLevels];
    // the launches cover nL systems: smap's (the PCG's tail iterations) or all B
    const int32_t nL = smap ? nl : B;
    const SysMap sm{smap, nL};
    for (int32_t l = 0; l < L; ++l) {
        v[l] = level_view(G.lv[l]);
        v[l].sm = sm;
    }
    // levels S.. run fused in k_subcycle
    int32_t S = 1;
    while (S < L - 1 && G.lv[S].n > kSubNodes) ++S;
    // the cycle below level 0 from level 1's restricted b and pre-smoothed
    // x: down (residual, restriction + next pre-smooth), the fused tiny
    // levels, up (prolongation, post-smoothing into y)
    auto coarse = [&](Lvl (&u)[kMaxLevels]) {
        for (int32_t l = 1; l < S; ++l) {
            const int32_t smooth = l + 1 < L - 1;
            k_res3<<<grid2(u[l].n, nL), kWG, 0, s>>>(u[l], sysi);
            if (G.lv[l].smoothed)
                k_restrict0_sa<3><<<dim3(xcd_grid(G.lv[l].ngrp, (nL + kNSR - 1) / kNSR, kGrpRestr)), kWG, 0, s>>>(
                    u[l], u[l + 1], G.lv[l].rgrp.p, G.lv[l].ngrp, B, smooth, om1, sysi);
            else
                k_restrict<3><<<dim3(xcd_grid(G.lv[l].ngrp, nL, kGrpRestr)), kWG, 0, s>>>(
                    u[l], u[l + 1], G.lv[l].rgrp.p, G.lv[l].ngrp, B, smooth, om1, sysi);
        }
        SubArgs sa;
        sa.first = S;
        sa.last = L - 1;
        for (int32_t l = 0; l < L; ++l) sa.lv[l] = u[l];
        sa.cinv = G.cinv.p;
        sa.omega = om1;
        sa.sysi = sysi;
        k_subcycle<<<dim3((unsigned)nL), kSubWG, 0, s>>>(sa);
        for (int32_t l = S - 1; l >= 1; --l) {
            if (G.lv[l].smoothed) {
                const int32_t nb = (u[l].n + kWG - 1) / kWG;
                k_prolong3_sa<<<dim3(xcd_grid(nb, (nL + kNS3 - 1) / kNS3, kGrpProl)), kWG, 0, s>>>(u[l], u[l + 1], nb,
                                                                                                   B, sysi);
            }
            else
                k_prolong<3><<<grid2(u[l].n, nL), kWG, 0, s>>>(u[l], u[l + 1], sysi);
            k_post3<<<grid2(u[l].n, nL), kWG, 0, s>>>(u[l], om1, sysi);
        }
    };
    // down at level 0: residual of the pre-smoothed x, restriction (+ level
    // 1's pre-smooth)
    for (int32_t l = 0; l < 1; ++l) {
        const int32_t smooth = l + 1 < L - 1;
        if (l == 0) {
            if (G.bsw_n > 0) launch_bsweep<false>(G, sm, r0, v[0].x, om, sysi, s);
            k_res0_ns<kRes0NS><<<dim3(xcd_grid(nblk, (nL + kRes0NS - 1) / kRes0NS,
                                               kGrpSmooth > kRes0NS ? kGrpSmooth / kRes0NS : 1)),
                                 kWG, 0, s>>>(v[0].n, nblk, B, sm, mat0, r0, v[0].x,
                                              G.lv[0].smoothed ? nullptr : v[0].apos, sysi, v[0].r);
            if (G.lv[0].smoothed) {
                k_restrict0_sa<2><<<dim3(xcd_grid(G.lv[0].ngrp, (nL + kNSR - 1) / kNSR, kGrpRestr)), kWG, 0, s>>>(
                    v[0], v[1], G.lv[0].rgrp.p, G.lv[0].ngrp, B, smooth, om1, sysi);
            } else {
                k_restrict<2, kRestrS><<<dim3(xcd_grid(G.lv[0].ngrp, (nL + kRestrS - 1) / kRestrS, kGrpRestr)), kWG, 0, s>>>(
                    v[0], v[1], G.lv[0].rgrp.p, G.lv[0].ngrp, B, smooth, om1, sysi);
            }
        }
    }
    if (S == 1) {  // level 1 is already one of the fused tiny levels
        SubArgs sa;
        sa.first = 1;
        sa.last = L - 1;
        for (int32_t l = 0; l < L; ++l) sa.lv[l] = v[l];
        sa.cinv = G.cinv.p;
        sa.omega = om1;
        sa.sysi = sysi;
        k_subcycle<<<dim3((unsigned)nL), kSubWG, 0, s>>>(sa);
    } else {
        coarse(v);
    }
    // up at level 0: coarse correction, post-smooth
    for (int32_t l = 0; l >= 0; --l) {
        if (l == 0) {
            const int32_t nb0 = (v[0].n + kWG - 1) / kWG;
            const int32_t nb0p = (v[0].n + kWG * kProlR - 1) / (kWG * kProlR);
            const dim3 gsa(xcd_grid(nb0, (nL + kNSP - 1) / kNSP, kGrpProl)), gp(xcd_grid(nb0p, (nL + kProlS - 1) / kProlS, kGrpProl));
            if (G.xm == 2) {
                if (G.lv[0].smoothed)
                    k_prolong0_sa<2><<<gsa, kWG, 0, s>>>(v[0], v[1], nb0, B, sysi);
                else
                    k_prolong0<2><<<gp, kWG, 0, s>>>(v[0], v[1], nb0p, B, sysi);
                if (G.bsw_n > 0) launch_bsweep<true>(G, sm, r0, v[0].y, om, sysi, s);
                if (zh)
                    launch_post0<2, true>(nblk, nL, s, v[0].n, nblk, B, sm, mat0, r0, v[0].y, om, sysi, z0, part_slot, rd);
                else
                    launch_post0<2, false>(nblk, nL, s, v[0].n, nblk, B, sm, mat0, r0, v[0].y, om, sysi, z0, part_slot, rd);
            } else {
                if (G.lv[0].smoothed)
                    k_prolong0_sa<1><<<gsa, kWG, 0, s>>>(v[0], v[1], nb0, B, sysi);
                else
                    k_prolong0<1><<<gp, kWG, 0, s>>>(v[0], v[1], nb0p, B, sysi);
                if (G.bsw_n > 0) launch_bsweep<false>(G, sm, r0, v[0].x, om, sysi, s);
                if (zh)
                    launch_post0<1, true>(nblk, nL, s, v[0].n, nblk, B, sm, mat0, r0, v[0].x, om, sysi, z0, part_slot, rd);
                else
                    launch_post0<1, false>(nblk, nL, s, v[0].n, nblk, B, sm, mat0, r0, v[0].x, om, sysi, z0, part_slot, rd);
            }
        }
    }
    MOF_HIP(hipGetLastError());
}

void amg_destroy(AmgDevice *g) { delete g; }

float amg_set_omega(mof_mesh *m, float omega) {
    if (!m->amg) return 0.f;
    const float old = m->amg->omega;
    m->amg->omega = omega;
    return old;
}

int32_t amg_levels(const mof_mesh *m) { return m->amg && m->amg->built ? (int32_t)m->amg->lv.size() : 0; }

}  // namespace mof
