// mof_amg.hip -- aggregation multigrid V-cycle on gfx950 (inner-PCG preconditioner).
//
// Per batch of B systems (timesteps) the mesh-only hierarchy of
// mof_amg_host.cpp gets its per-timestep values:
//   k_galerkin<BSF>    A_{l+1} = Q^T A_l Q, one coarse block per thread, folded
//                      over the pre-built gather lists (no atomics), plus the
//                      3x3 block-Jacobi inverse of each coarse node;
//   k_coarse_inverse   the coarsest operator (<= 128 dofs) inverted by the
//                      symmetric sweep operator in registers (fp64, one
//                      workgroup per system).
// Each PCG iteration applies one symmetric V(1,1)-cycle to the residual r:
//   level 0 pre-smooth x0 = w D^-1 r is fused into k_pcg_update / k_pcg_init;
//   per level l:  k_res0 / k_res3  r_l = b_l - A_l x_l, written in member
//                                  order of the next level's aggregates
//                 k_restrict       b_{l+1} = Q^T r_l (contiguous members),
//                                  x_{l+1} = w D^-1 b_{l+1} (next pre-smooth)
//   coarsest:     k_coarse_solve   y = A_c^-1 b
//   per level l:  k_prolong        x_l += Q y_{l+1}
//                 k_post3 / k_post0  y_l = x_l + w D^-1 (b_l - A_l x_l); at
//                                  level 0 y = z and the partial r.z of the PCG
// Every launch covers all B systems and skips retired systems. Level 0 reuses
// the inner solver's fp32 SELL A, 2x2 D^-1 and row-kernel layout (XCD-aware,
// batched loads); coarse levels store 3x3 blocks as 12 floats (rows padded to
// 4) and vectors as float4. All sums run in a fixed order: the cycle is
// deterministic and independent of B.
#include <algorithm>

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

// ---- per-timestep setup --------------------------------------------------

// Block (I, J) at coarse SELL position pos of A_{l+1} = Q^T A_l Q for system
// b, summed over its gather list in list order; the diagonal block also gets
// 1 on dead dofs and stores its 3x3 inverse for the smoother.
template <int BSF>
__global__ __launch_bounds__(kWG) void k_galerkin(
    int64_t c_sell_nb, int32_t nC, const int32_t *__restrict__ c_sell_row,
    const int32_t *__restrict__ c_diag, const uint8_t *__restrict__ c_dead,
    const int32_t *__restrict__ gptr, const int32_t *__restrict__ gent, const float *__restrict__ Q,
    const float *__restrict__ Af, int64_t f_sell_nb, float *__restrict__ Ac, float *__restrict__ Dc) {
    const int64_t pos = (int64_t)blockIdx.x * kWG + threadIdx.x;
    const int32_t b = blockIdx.y;
    if (pos >= c_sell_nb) return;
    const int32_t I = c_sell_row[pos];
    if (I >= nC) return;  // rows past n in the last slice
    const float *A = Af + (int64_t)b * f_sell_nb * bstride<BSF>();
    float C[3][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
    const int32_t g0 = gptr[pos], g1 = gptr[pos + 1];
    for (int32_t g = g0; g < g1; ++g) {
        const int32_t fp = gent[3 * (int64_t)g], i = gent[3 * (int64_t)g + 1],
                      j = gent[3 * (int64_t)g + 2];
        float a[BSF][BSF], qi[BSF][3], qj[BSF][3];
        ldm<BSF>(A, fp, a);
#pragma unroll
        for (int k = 0; k < BSF; ++k)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                qi[k][c] = Q[((int64_t)i * BSF + k) * 3 + c];
                qj[k][c] = Q[((int64_t)j * BSF + k) * 3 + c];
            }
        float T[BSF][3];  // A Q_j
#pragma unroll
        for (int r = 0; r < BSF; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                float sum = 0.f;
#pragma unroll
                for (int k = 0; k < BSF; ++k) sum += a[r][k] * qj[k][c];
                T[r][c] = sum;
            }
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                float sum = 0.f;
#pragma unroll
                for (int k = 0; k < BSF; ++k) sum += qi[k][r] * T[k][c];
                C[r][c] += sum;
            }
    }
    if (pos == c_diag[I]) {
#pragma unroll
        for (int d = 0; d < 3; ++d)
            if (c_dead[3 * (int64_t)I + d]) C[d][d] += 1.f;
        float D[3][3];
        inv3(C, D);
        st3(Dc, (int64_t)b * nC + I, D);
    }
    st3(Ac, (int64_t)b * c_sell_nb + pos, C);
}

constexpr int kMaxCoarse = 128;
constexpr int kSweepRows = kMaxCoarse * kMaxCoarse / kWG;  // 64 matrix rows per thread

// Inverse of the coarsest operator (nc = 3 n <= 128 dofs) of system b by the
// symmetric sweep operator: sweeping pivot k maps
//   a_kk -> -1/a_kk, a_ik -> a_ik/a_kk, a_kj -> a_kj/a_kk,
//   a_ij -> a_ij - a_ik a_kj / a_kk,
// and after all pivots the matrix holds -A^-1. Symmetry gives column k =
// row k, so a step broadcasts one row through LDS. Thread t owns column
// t % 128 of rows (t / 128) * 64 + [0, 64) in fp64 registers.
__global__ __launch_bounds__(kWG) void k_coarse_inverse(int32_t n, const int32_t *__restrict__ sell_off,
                                                        const int32_t *__restrict__ sell_col,
                                                        const float *__restrict__ Ac, int64_t sell_nb,
                                                        float *__restrict__ cinv) {
    __shared__ float M[kMaxCoarse][kMaxCoarse + 1];
    __shared__ double rowk[kMaxCoarse];
    const int32_t b = blockIdx.x;
    const int32_t nc = 3 * n;
    for (int32_t q = threadIdx.x; q < kMaxCoarse * kMaxCoarse; q += kWG)
        M[q / kMaxCoarse][q % kMaxCoarse] = 0.f;
    __syncthreads();
    const float *A = Ac + (int64_t)b * sell_nb * kB3;
    // one thread per node row: no two threads write the same row
    for (int32_t I = threadIdx.x; I < n; I += kWG) {
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
#pragma unroll
        for (int mm = 0; mm < kSweepRows; ++mm) {
            const int32_t r = h * kSweepRows + mm;
            const double ark = rowk[r];
            if (r == k)
                a[mm] = (c == k) ? -ip : a[mm] * ip;
            else if (c == k)
                a[mm] = a[mm] * ip;
            else
                a[mm] -= ark * akc;
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

// Level 0: r1 = r - A x0 (x0 = w D^-1 r from the PCG update), stored at the
// member position of each vertex. PCG row layout, XCD-aware grid.
__global__ __launch_bounds__(kWG) void k_res0(int32_t N, int32_t nblk, int32_t B, MatArgs<float> mat,
                                              const float *__restrict__ rv, const float *__restrict__ xv,
                                              const int32_t *__restrict__ apos,
                                              const int32_t *__restrict__ sysi, float *__restrict__ r1) {
    int32_t rb, b;
    if (!xcd_map(nblk, B, rb, b) || retired(sysi, b)) return;
    const int64_t vb = (int64_t)b * N;
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
        const int32_t i = rb * kRowsPerWG + r * kWG + threadIdx.x;
        if (i >= N) break;
        float y0, y1;
        spmv_row<float>(mat, b, i, xv + 2 * vb, y0, y1);
        const float2 ri = reinterpret_cast<const float2 *>(rv)[vb + i];
        reinterpret_cast<float2 *>(r1)[vb + apos[i]] = make_float2(ri.x - y0, ri.y - y1);
    }
}

// Coarse level: r = b - A x, stored at the member position of each node.
__global__ __launch_bounds__(kWG) void k_res3(int32_t n, const int32_t *__restrict__ sell_off,
                                              const int32_t *__restrict__ sell_col,
                                              const float *__restrict__ A, int64_t sell_nb,
                                              const float *__restrict__ bv, const float *__restrict__ xv,
                                              const int32_t *__restrict__ apos,
                                              const int32_t *__restrict__ sysi, float *__restrict__ rv) {
    const int32_t i = blockIdx.x * kWG + threadIdx.x;
    const int32_t b = blockIdx.y;
    if (i >= n || retired(sysi, b)) return;
    const float *Ab = A + (int64_t)b * sell_nb * kB3;
    const float *xb = xv + (int64_t)b * n * 4;
    float acc[3];
    ldv<3>(bv + (int64_t)b * n * 4, i, acc);
    const int32_t s = i >> 6, l = i & 63;
    const int32_t o = sell_off[s], w = (sell_off[s + 1] - o) >> 6;
    for (int32_t t = 0; t < w; ++t) {
        const int64_t pos = (int64_t)o + t * kSlice + l;
        float a[3][3], xj[3], ax[3];
        ldm<3>(Ab, pos, a);
        ldv<3>(xb, sell_col[pos], xj);
        matvec<3>(a, xj, ax);
#pragma unroll
        for (int c = 0; c < 3; ++c) acc[c] -= ax[c];
    }
    stv<3>(rv + (int64_t)b * n * 4, apos[i], acc);
}

// b_{l+1}[I] = sum over the members of aggregate I of Q^T r (member order,
// contiguous); with D (not the coarsest level) also x_{l+1} = w D^-1 b_{l+1}.
template <int BSF>
__global__ __launch_bounds__(kWG) void k_restrict(int32_t nF, int32_t nC, const int32_t *__restrict__ mptr,
                                                  const float *__restrict__ Qm,
                                                  const float *__restrict__ rv,
                                                  const float *__restrict__ Dc, float omega,
                                                  const int32_t *__restrict__ sysi,
                                                  float *__restrict__ bc, float *__restrict__ xc) {
    const int32_t I = blockIdx.x * kWG + threadIdx.x;
    const int32_t b = blockIdx.y;
    if (I >= nC || retired(sysi, b)) return;
    const float *rb = rv + (int64_t)b * nF * vstride<BSF>();
    float acc[3] = {0.f, 0.f, 0.f};
    const int32_t q0 = mptr[I], q1 = mptr[I + 1];
    for (int32_t q = q0; q < q1; ++q) {
        float ri[BSF];
        ldv<BSF>(rb, q, ri);
        const float *qi = Qm + (int64_t)q * BSF * 3;
#pragma unroll
        for (int k = 0; k < BSF; ++k)
#pragma unroll
            for (int c = 0; c < 3; ++c) acc[c] += qi[3 * k + c] * ri[k];
    }
    stv<3>(bc + (int64_t)b * nC * 4, I, acc);
    if (Dc) {
        float d[3][3], x[3];
        ldm<3>(Dc + (int64_t)b * nC * kB3, I, d);
        matvec<3>(d, acc, x);
#pragma unroll
        for (int c = 0; c < 3; ++c) x[c] *= omega;
        stv<3>(xc + (int64_t)b * nC * 4, I, x);
    }
}

// y = A_c^-1 b on the coarsest level (one workgroup per system)
__global__ __launch_bounds__(kWG) void k_coarse_solve(int32_t n, const float *__restrict__ cinv,
                                                      const float *__restrict__ bv,
                                                      const int32_t *__restrict__ sysi,
                                                      float *__restrict__ yv) {
    __shared__ float bl[kMaxCoarse];
    const int32_t b = blockIdx.x;
    if (retired(sysi, b)) return;
    const int32_t nc = 3 * n;
    for (int32_t q = threadIdx.x; q < nc; q += kWG) bl[q] = bv[(int64_t)b * n * 4 + 4 * (q / 3) + q % 3];
    __syncthreads();
    const float *Mi = cinv + (int64_t)b * nc * nc;
    for (int32_t d = threadIdx.x; d < nc; d += kWG) {
        float s = 0.f;
        for (int32_t k = 0; k < nc; ++k) s += Mi[(int64_t)k * nc + d] * bl[k];  // symmetric
        yv[(int64_t)b * n * 4 + 4 * (d / 3) + d % 3] = s;
    }
}

// x_i += Q_i y_{l+1}[agg(i)]
template <int BSF>
__global__ __launch_bounds__(kWG) void k_prolong(int32_t nF, int32_t nC, const int32_t *__restrict__ agg,
                                                 const float *__restrict__ Q,
                                                 const float *__restrict__ yc,
                                                 const int32_t *__restrict__ sysi,
                                                 float *__restrict__ xv) {
    const int32_t i = blockIdx.x * kWG + threadIdx.x;
    const int32_t b = blockIdx.y;
    if (i >= nF || retired(sysi, b)) return;
    float y[3], xi[BSF];
    ldv<3>(yc + (int64_t)b * nC * 4, agg[i], y);
    float *xb = xv + (int64_t)b * nF * vstride<BSF>();
    ldv<BSF>(xb, i, xi);
    const float *qi = Q + (int64_t)i * BSF * 3;
#pragma unroll
    for (int k = 0; k < BSF; ++k) xi[k] += qi[3 * k] * y[0] + qi[3 * k + 1] * y[1] + qi[3 * k + 2] * y[2];
    stv<BSF>(xb, i, xi);
}

// y = x + w D^-1 (b - A x) on a coarse level (one node per thread)
__global__ __launch_bounds__(kWG) void k_post3(int32_t n, const int32_t *__restrict__ sell_off,
                                               const int32_t *__restrict__ sell_col,
                                               const float *__restrict__ A, int64_t sell_nb,
                                               const float *__restrict__ Dinv,
                                               const float *__restrict__ bv,
                                               const float *__restrict__ xv, float omega,
                                               const int32_t *__restrict__ sysi,
                                               float *__restrict__ yv) {
    const int32_t i = blockIdx.x * kWG + threadIdx.x;
    const int32_t b = blockIdx.y;
    if (i >= n || retired(sysi, b)) return;
    const float *Ab = A + (int64_t)b * sell_nb * kB3;
    const float *xb = xv + (int64_t)b * n * 4;
    float res[3], xi[3];
    ldv<3>(bv + (int64_t)b * n * 4, i, res);
    ldv<3>(xb, i, xi);
    const int32_t s = i >> 6, l = i & 63;
    const int32_t o = sell_off[s], w = (sell_off[s + 1] - o) >> 6;
    for (int32_t t = 0; t < w; ++t) {
        const int64_t pos = (int64_t)o + t * kSlice + l;
        float a[3][3], xj[3], ax[3];
        ldm<3>(Ab, pos, a);
        ldv<3>(xb, sell_col[pos], xj);
        matvec<3>(a, xj, ax);
#pragma unroll
        for (int c = 0; c < 3; ++c) res[c] -= ax[c];
    }
    float d[3][3], dr[3];
    ldm<3>(Dinv + (int64_t)b * n * kB3, i, d);
    matvec<3>(d, res, dr);
#pragma unroll
    for (int c = 0; c < 3; ++c) xi[c] += omega * dr[c];
    stv<3>(yv + (int64_t)b * n * 4, i, xi);
}

// Level 0: z = x + w D^-1 (r - A x) and the PCG's partial r.z (component 0
// of the row block's record). PCG row layout, XCD-aware grid.
__global__ __launch_bounds__(kWG) void k_post0(int32_t N, int32_t nblk, int32_t B, MatArgs<float> mat,
                                               const float *__restrict__ Dinv,
                                               const float *__restrict__ rv,
                                               const float *__restrict__ xv, float omega,
                                               const int32_t *__restrict__ sysi,
                                               float *__restrict__ zv, double *__restrict__ part) {
    __shared__ double lds[8];
    int32_t rb, b;
    if (!xcd_map(nblk, B, rb, b) || retired(sysi, b)) return;
    const int64_t vb = (int64_t)b * N;
    double rz = 0.0;
#pragma unroll
    for (int g = 0; g < kRows; ++g) {
        const int32_t i = rb * kRowsPerWG + g * kWG + threadIdx.x;
        if (i >= N) break;
        float y0, y1;
        spmv_row<float>(mat, b, i, xv + 2 * vb, y0, y1);
        const float2 ri = reinterpret_cast<const float2 *>(rv)[vb + i];
        const float2 xi = reinterpret_cast<const float2 *>(xv)[vb + i];
        float d[4];
        ld_blk(Dinv, vb + i, d);
        const float s0 = ri.x - y0, s1 = ri.y - y1;
        const float z0 = xi.x + omega * (d[0] * s0 + d[1] * s1);
        const float z1 = xi.y + omega * (d[2] * s0 + d[3] * s1);
        reinterpret_cast<float2 *>(zv)[vb + i] = make_float2(z0, z1);
        rz += (double)ri.x * z0 + (double)ri.y * z1;
    }
    double v[1] = {rz};
    block_sum<1>(v, lds);
    if (threadIdx.x == 0) part[2 * ((int64_t)b * nblk + rb)] = v[0];
}

inline dim3 grid2(int64_t n, int32_t B) { return dim3((unsigned)((n + kWG - 1) / kWG), (unsigned)B); }

MatArgs<float> level0_mat(mof_mesh *m) {
    MatArgs<float> mt;
    mt.sell_nb = m->pat.sell_nb();
    mt.sell_off = m->sell_off.p;
    mt.sell_col = m->sell_col.p;
    mt.A = m->ws.A32.p;
    return mt;
}

}  // namespace

// ---- host side ---------------------------------------------------------------

bool amg_build(mof_mesh *m) {
    const AmgParams prm;
    if (m->amg && m->amg->built) return m->amg->lv.size() >= 2;
    if (!m->amg) m->amg = new AmgDevice();
    AmgDevice &G = *m->amg;
    hipStream_t s = m->stream;
    std::vector<double> e(6 * (size_t)m->N);
    MOF_HIP(hipMemcpyAsync(e.data(), m->e.p, e.size() * sizeof(double), hipMemcpyDeviceToHost, s));
    MOF_HIP(hipStreamSynchronize(s));
    AmgHierarchy H;
    build_amg(m->pat, e.data(), prm, H);
    G.omega = prm.omega;
    G.lv.clear();
    G.built = true;
    // a mesh that does not coarsen (<= 42 vertices) keeps block Jacobi
    if (H.levels.size() < 2) return false;
    MOF_REQUIRE(H.coarse_dofs <= kMaxCoarse, "coarsest multigrid level too large");
    G.lv.resize(H.levels.size());
    auto put_i = [&](DevArray<int32_t> &d, const std::vector<int32_t> &h) {
        d.alloc(h.size());
        if (!h.empty()) d.upload(h.data(), h.size(), s);
    };
    auto put_f = [&](DevArray<float> &d, const std::vector<float> &h) {
        d.alloc(h.size());
        if (!h.empty()) d.upload(h.data(), h.size(), s);
    };
    for (size_t l = 0; l < H.levels.size(); ++l) {
        const AmgLevel &L = H.levels[l];
        AmgDevLevel &D = G.lv[l];
        D.n = L.n;
        D.bs = L.bs;
        D.sell_nb = L.sell_nb();
        if (l > 0) {
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
            put_i(D.apos, L.apos);
            put_i(D.gptr, L.gptr);
            put_i(D.gent, L.gent);
            put_f(D.Q, L.Q);
            put_f(D.Qm, L.Qm);
        }
    }
    G.nc = H.coarse_dofs;
    G.cap = 0;
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
            D.r.alloc(2 * n * B);
        } else {
            D.A.alloc((size_t)kB3 * D.sell_nb * B);
            D.A.zero(s);
            D.Dinv.alloc((size_t)kB3 * n * B);
            D.b.alloc(4 * n * B);
            D.x.alloc(4 * n * B);
            D.r.alloc(4 * n * B);
            D.y.alloc(4 * n * B);
        }
    }
    G.cinv.alloc((size_t)G.nc * G.nc * B);
    G.cap = B;
    MOF_HIP(hipStreamSynchronize(s));
}

float *amg_level0_x(mof_mesh *m) { return m->amg->lv[0].x.p; }
float amg_omega(const mof_mesh *m) { return m->amg->omega; }

void amg_setup_batch(mof_mesh *m, int32_t B, hipStream_t s) {
    AmgDevice &G = *m->amg;
    Workspace &w = m->ws;
    const size_t L = G.lv.size();
    for (size_t l = 0; l + 1 < L; ++l) {
        AmgDevLevel &F = G.lv[l], &C = G.lv[l + 1];
        if (l == 0)
            k_galerkin<2><<<grid2(C.sell_nb, B), kWG, 0, s>>>(C.sell_nb, C.n, C.sell_row.p, C.diag_pos.p,
                                                              C.dead.p, F.gptr.p, F.gent.p, F.Q.p, w.A32.p,
                                                              m->pat.sell_nb(), C.A.p, C.Dinv.p);
        else
            k_galerkin<3><<<grid2(C.sell_nb, B), kWG, 0, s>>>(C.sell_nb, C.n, C.sell_row.p, C.diag_pos.p,
                                                              C.dead.p, F.gptr.p, F.gent.p, F.Q.p, F.A.p,
                                                              F.sell_nb, C.A.p, C.Dinv.p);
    }
    AmgDevLevel &Lc = G.lv[L - 1];
    k_coarse_inverse<<<dim3((unsigned)B), kWG, 0, s>>>(Lc.n, Lc.sell_off.p, Lc.sell_col.p, Lc.A.p,
                                                       Lc.sell_nb, G.cinv.p);
    MOF_HIP(hipGetLastError());
}

void amg_vcycle(mof_mesh *m, int32_t B, const float *r0, float *z0, double *part_slot, int32_t nblk,
                hipStream_t s) {
    AmgDevice &G = *m->amg;
    Workspace &w = m->ws;
    const size_t L = G.lv.size();
    const int32_t *sysi = w.sysi.p;
    const float om = G.omega;
    const MatArgs<float> mat0 = level0_mat(m);
    const dim3 gx(xcd_grid(nblk, B));
    // down: residual of the pre-smoothed x, restriction (+ next pre-smooth)
    for (size_t l = 0; l + 1 < L; ++l) {
        AmgDevLevel &F = G.lv[l], &C = G.lv[l + 1];
        const bool coarsest = l + 2 == L;
        const float *Dn = coarsest ? nullptr : C.Dinv.p;
        if (l == 0) {
            k_res0<<<gx, kWG, 0, s>>>(F.n, nblk, B, mat0, r0, F.x.p, F.apos.p, sysi, F.r.p);
            k_restrict<2><<<grid2(C.n, B), kWG, 0, s>>>(F.n, C.n, F.mptr.p, F.Qm.p, F.r.p, Dn, om, sysi,
                                                        C.b.p, C.x.p);
        } else {
            k_res3<<<grid2(F.n, B), kWG, 0, s>>>(F.n, F.sell_off.p, F.sell_col.p, F.A.p, F.sell_nb, F.b.p,
                                                 F.x.p, F.apos.p, sysi, F.r.p);
            k_restrict<3><<<grid2(C.n, B), kWG, 0, s>>>(F.n, C.n, F.mptr.p, F.Qm.p, F.r.p, Dn, om, sysi,
                                                        C.b.p, C.x.p);
        }
    }
    AmgDevLevel &Lc = G.lv[L - 1];
    k_coarse_solve<<<dim3((unsigned)B), kWG, 0, s>>>(Lc.n, G.cinv.p, Lc.b.p, sysi, Lc.y.p);
    // up: coarse correction, post-smooth
    for (size_t l = L - 1; l-- > 0;) {
        AmgDevLevel &F = G.lv[l], &C = G.lv[l + 1];
        if (l == 0) {
            k_prolong<2><<<grid2(F.n, B), kWG, 0, s>>>(F.n, C.n, F.agg.p, F.Q.p, C.y.p, sysi, F.x.p);
            k_post0<<<gx, kWG, 0, s>>>(F.n, nblk, B, mat0, w.dinv32.p, r0, F.x.p, om, sysi, z0, part_slot);
        } else {
            k_prolong<3><<<grid2(F.n, B), kWG, 0, s>>>(F.n, C.n, F.agg.p, F.Q.p, C.y.p, sysi, F.x.p);
            k_post3<<<grid2(F.n, B), kWG, 0, s>>>(F.n, F.sell_off.p, F.sell_col.p, F.A.p, F.sell_nb,
                                                   F.Dinv.p, F.b.p, F.x.p, om, sysi, F.y.p);
        }
    }
    MOF_HIP(hipGetLastError());
}

void amg_destroy(AmgDevice *g) { delete g; }

int32_t amg_levels(const mof_mesh *m) { return m->amg && m->amg->built ? (int32_t)m->amg->lv.size() : 0; }

}  // namespace mof
