// mof_sing.hip -- SURVEY.md §8(f)4: critical points of K velocity fields.
//
// Restates find_singularity_points(coordinates, triangles, V_now, eps)
// (find_singularity_point.py:140-189) for K timesteps in three launches:
//   k_sing_vmax    v_length_max = max_i sqrt(v0**2 + v1**2 + v2**2)   (:164-165)
//                  (a max is order-free: atomicMax on the bits of a
//                  non-negative double, exact)
//   k_sing_vertex  |V_i / vmax| <= eps, np.linalg.norm = sqrt(ddot)   (:72-90,168-170)
//   k_sing_tri     triangles without a zero vertex: n = (B-A)x(C-A)/|.|,
//                  V_proj = V/vmax - (V/vmax . n) n, and the 3x2 least
//                  squares M [lam mu]^T = -VC_proj of
//                  has_zero_velocity_interior (:93-137); inside when
//                  lam + mu <= 1, lam >= 0, mu >= 0.
// vmax and the vertex test are bit-identical to numpy (same operations, the
// FMA pattern of OpenBLAS's ddot, -ffp-contract=off). np.linalg.lstsq is
// LAPACK dgelsd (SVD); here the 3x2 system is solved by Householder QR and a
// 2x2 SVD of R with dgelsd's rank cutoff (rcond = eps * 3): lam, mu agree to
// rounding, so a triangle can differ only when lam, mu or 1-lam-mu is within
// rounding of 0 (tests exclude that band). With float32 coordinates (pyvista
// points) the normal is formed in float32 as numpy does.
#include <cmath>
#include <cstdint>

#include "mof_internal.h"

namespace mof {
namespace {

__device__ __forceinline__ double ddot3(const double *x, const double *y) {
    return fma(x[2], y[2], fma(x[1], y[1], x[0] * y[0]));
}
__device__ __forceinline__ float sdot3(const float *x, const float *y) {
    return (float)(((double)(x[0] * y[0]) + (double)(x[1] * y[1])) + (double)(x[2] * y[2]));
}

__global__ void k_sing_vmax(int32_t N, const double *__restrict__ V, unsigned long long *__restrict__ vmax) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const int32_t k = blockIdx.y;
    double l = 0.0;
    if (i < N) {
        const double *v = V + 3 * ((int64_t)k * N + i);
        l = sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]);
    }
    // NaN wins (np.max propagates it); all lengths are >= 0 or NaN
    unsigned long long bits = (unsigned long long)__double_as_longlong(fabs(l));
    if (l != l) bits = 0x7ff8000000000000ull;
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long other = __shfl_down(bits, o, 64);
        bits = other > bits ? other : bits;
    }
    if ((threadIdx.x & 63) == 0 && bits) atomicMax(vmax + k, bits);
}

__global__ void k_sing_vertex(int32_t N, const double *__restrict__ V, const double *__restrict__ vmax,
                              double eps, uint8_t *__restrict__ vflag) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const int32_t k = blockIdx.y;
    if (i >= N) return;
    const double *v = V + 3 * ((int64_t)k * N + i);
    const double m = vmax[k];
    const double x[3] = {v[0] / m, v[1] / m, v[2] / m};
    vflag[(int64_t)k * N + i] = sqrt(ddot3(x, x)) <= eps ? 1 : 0;
}

// x = argmin |M x - b| for M = [c0 c1] (3x2) with dgelsd's minimum-norm
// truncation (singular values <= 3 eps sigma_max treated as zero).
__device__ void lstsq32(const double c0[3], const double c1[3], const double b[3], double &x0, double &x1) {
    // Householder QR of M: R = [[r11, r12], [0, r22]], c = Q^T b (first 2)
    double v[3], a0[3], a1[3], bb[3];
    for (int i = 0; i < 3; ++i) {
        a0[i] = c0[i];
        a1[i] = c1[i];
        bb[i] = b[i];
    }
    auto reflect = [](const double *vv, double vtv, double *y, int from) {
        if (vtv == 0.0) return;
        double s = 0.0;
        for (int i = from; i < 3; ++i) s += vv[i] * y[i];
        s = 2.0 * s / vtv;
        for (int i = from; i < 3; ++i) y[i] -= s * vv[i];
    };
    double nrm = sqrt(a0[0] * a0[0] + a0[1] * a0[1] + a0[2] * a0[2]);
    const double r11 = a0[0] > 0 ? -nrm : nrm;
    v[0] = a0[0] - r11;
    v[1] = a0[1];
    v[2] = a0[2];
    double vtv = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    reflect(v, vtv, a1, 0);
    reflect(v, vtv, bb, 0);
    const double r12 = a1[0];
    nrm = sqrt(a1[1] * a1[1] + a1[2] * a1[2]);
    const double r22 = a1[1] > 0 ? -nrm : nrm;
    v[0] = 0.0;
    v[1] = a1[1] - r22;
    v[2] = a1[2];
    vtv = v[1] * v[1] + v[2] * v[2];
    reflect(v, vtv, bb, 1);
    const double c[2] = {bb[0], bb[1]};
    // SVD of R: eigenvectors of R^T R by one Jacobi rotation
    const double g11 = r11 * r11, g12 = r11 * r12, g22 = r12 * r12 + r22 * r22;
    const double th = 0.5 * atan2(2.0 * g12, g11 - g22);
    const double cs = cos(th), sn = sin(th);
    const double V1[2] = {cs, sn}, V2[2] = {-sn, cs};
    double u1[2] = {r11 * V1[0] + r12 * V1[1], r22 * V1[1]};
    double u2[2] = {r11 * V2[0] + r12 * V2[1], r22 * V2[1]};
    double s1 = sqrt(u1[0] * u1[0] + u1[1] * u1[1]), s2 = sqrt(u2[0] * u2[0] + u2[1] * u2[1]);
    const double smax = fmax(s1, s2);
    const double cut = 3.0 * 2.220446049250313e-16 * smax;
    x0 = x1 = 0.0;
    if (s1 > cut && s1 > 0.0) {
        const double w = (u1[0] * c[0] + u1[1] * c[1]) / (s1 * s1);
        x0 += w * V1[0];
        x1 += w * V1[1];
    }
    if (s2 > cut && s2 > 0.0) {
        const double w = (u2[0] * c[0] + u2[1] * c[1]) / (s2 * s2);
        x0 += w * V2[0];
        x1 += w * V2[1];
    }
}

// Compact output (CMP): flagged vertices / triangles are appended as
// (field, index[, lam, mu]) records at an atomic cursor (order fixed later on
// the host by sorting); the dense flags are then not written for triangles.
struct SingList {
    unsigned long long *cnt;  // [0] vertex records, [1] triangle records
    int64_t cap;
    int2 *vrec;               // (field, vertex)
    int2 *trec;               // (field, triangle)
    double2 *tlm;             // (lam, mu) of each triangle record
};

__global__ void k_sing_vlist(int32_t N, const uint8_t *__restrict__ vflag, SingList L) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const int32_t k = blockIdx.y;
    if (i >= N || !vflag[(int64_t)k * N + i]) return;
    const unsigned long long q = atomicAdd(L.cnt, 1ull);
    if ((int64_t)q < L.cap) L.vrec[q] = make_int2(k, i);
}

template <bool F32, bool CMP>
__global__ void k_sing_tri(int32_t N, int32_t M, const void *__restrict__ coords, const int32_t *__restrict__ tri,
                           const double *__restrict__ V, const double *__restrict__ vmax,
                           const uint8_t *__restrict__ vflag, uint8_t *__restrict__ tflag,
                           double *__restrict__ lam_mu, SingList L) {
    const int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const int32_t k = blockIdx.y;
    if (t >= M) return;
    const int32_t a = tri[3 * (int64_t)t], b = tri[3 * (int64_t)t + 1], c = tri[3 * (int64_t)t + 2];
    const int64_t vk = (int64_t)k * N;
    const int64_t o = (int64_t)k * M + t;
    if (!CMP) {
        tflag[o] = 0;
        lam_mu[2 * o] = 0.0;
        lam_mu[2 * o + 1] = 0.0;
    }
    if (vflag[vk + a] | vflag[vk + b] | vflag[vk + c]) return;  // :173-174
    double n[3];
    if constexpr (F32) {
        const float *P = static_cast<const float *>(coords);
        float ab[3], ac[3], nf[3];
        for (int d = 0; d < 3; ++d) {
            ab[d] = P[3 * (int64_t)b + d] - P[3 * (int64_t)a + d];
            ac[d] = P[3 * (int64_t)c + d] - P[3 * (int64_t)a + d];
        }
        nf[0] = ab[1] * ac[2] - ab[2] * ac[1];
        nf[1] = ab[2] * ac[0] - ab[0] * ac[2];
        nf[2] = ab[0] * ac[1] - ab[1] * ac[0];
        const float ln = sqrtf(sdot3(nf, nf));
        for (int d = 0; d < 3; ++d) n[d] = (double)(nf[d] / ln);
    } else {
        const double *P = static_cast<const double *>(coords);
        double ab[3], ac[3];
        for (int d = 0; d < 3; ++d) {
            ab[d] = P[3 * (int64_t)b + d] - P[3 * (int64_t)a + d];
            ac[d] = P[3 * (int64_t)c + d] - P[3 * (int64_t)a + d];
        }
        n[0] = ab[1] * ac[2] - ab[2] * ac[1];
        n[1] = ab[2] * ac[0] - ab[0] * ac[2];
        n[2] = ab[0] * ac[1] - ab[1] * ac[0];
        const double ln = sqrt(ddot3(n, n));
        for (int d = 0; d < 3; ++d) n[d] = n[d] / ln;
    }
    const double m = vmax[k];
    double pr[3][3];
    const int32_t vid[3] = {a, b, c};
    for (int q = 0; q < 3; ++q) {
        const double *v = V + 3 * (vk + vid[q]);
        const double x[3] = {v[0] / m, v[1] / m, v[2] / m};
        const double dn = ddot3(x, n);
        for (int d = 0; d < 3; ++d) pr[q][d] = x[d] - dn * n[d];
    }
    double c0[3], c1[3], rhs[3];
    for (int d = 0; d < 3; ++d) {
        c0[d] = pr[0][d] - pr[2][d];
        c1[d] = pr[1][d] - pr[2][d];
        rhs[d] = -pr[2][d];
    }
    double lam, mu;
    lstsq32(c0, c1, rhs, lam, mu);
    if (lam + mu <= 1 && lam >= 0 && mu >= 0) {
        if (CMP) {
            const unsigned long long q = atomicAdd(L.cnt + 1, 1ull);
            if ((int64_t)q < L.cap) {
                L.trec[q] = make_int2(k, t);
                L.tlm[q] = make_double2(lam, mu);
            }
        } else {
            tflag[o] = 1;
            lam_mu[2 * o] = lam;
            lam_mu[2 * o + 1] = mu;
        }
    }
}

}  // namespace

void launch_singularities(int32_t N, int32_t M, int32_t K, const void *coords, bool f32, const int32_t *tri,
                          const double *V, double eps, double *vmax, uint8_t *vflag, uint8_t *tflag,
                          double *lam_mu, hipStream_t s) {
    MOF_HIP(hipMemsetAsync(vmax, 0, sizeof(double) * K, s));
    const dim3 gv((unsigned)((N + kWG - 1) / kWG), (unsigned)K), gt((unsigned)((M + kWG - 1) / kWG), (unsigned)K);
    k_sing_vmax<<<gv, kWG, 0, s>>>(N, V, reinterpret_cast<unsigned long long *>(vmax));
    k_sing_vertex<<<gv, kWG, 0, s>>>(N, V, vmax, eps, vflag);
    if (M > 0) {
        const SingList none{nullptr, 0, nullptr, nullptr, nullptr};
        if (f32)
            k_sing_tri<true, false><<<gt, kWG, 0, s>>>(N, M, coords, tri, V, vmax, vflag, tflag, lam_mu, none);
        else
            k_sing_tri<false, false><<<gt, kWG, 0, s>>>(N, M, coords, tri, V, vmax, vflag, tflag, lam_mu, none);
    }
    MOF_HIP(hipGetLastError());
}

void launch_singularities_compact(int32_t N, int32_t M, int32_t K, const void *coords, bool f32,
                                  const int32_t *tri, const double *V, double eps, double *vmax, uint8_t *vflag,
                                  unsigned long long *cnt, int64_t cap, int2 *vrec, int2 *trec, double2 *tlm,
                                  hipStream_t s) {
    MOF_HIP(hipMemsetAsync(vmax, 0, sizeof(double) * K, s));
    MOF_HIP(hipMemsetAsync(cnt, 0, sizeof(unsigned long long) * 2, s));
    const dim3 gv((unsigned)((N + kWG - 1) / kWG), (unsigned)K), gt((unsigned)((M + kWG - 1) / kWG), (unsigned)K);
    const SingList L{cnt, cap, vrec, trec, tlm};
    k_sing_vmax<<<gv, kWG, 0, s>>>(N, V, reinterpret_cast<unsigned long long *>(vmax));
    k_sing_vertex<<<gv, kWG, 0, s>>>(N, V, vmax, eps, vflag);
    k_sing_vlist<<<gv, kWG, 0, s>>>(N, vflag, L);
    if (M > 0) {
        if (f32)
            k_sing_tri<true, true><<<gt, kWG, 0, s>>>(N, M, coords, tri, V, vmax, vflag, nullptr, nullptr, L);
        else
            k_sing_tri<false, true><<<gt, kWG, 0, s>>>(N, M, coords, tri, V, vmax, vflag, nullptr, nullptr, L);
    }
    MOF_HIP(hipGetLastError());
}

}  // namespace mof
