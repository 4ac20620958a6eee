// mof_rowkern.h -- device helpers shared by the row kernels of the PCG
// (mof_pcg.hip) and of the multigrid cycle (mof_amg.hip): block loads,
// deterministic reductions, the SELL-64 block SpMV row and the XCD-aware
// (row block, system) mapping.
#pragma once

#include "mof_internal.h"

namespace mof {
namespace {

template <typename V>
struct VT;
template <>
struct VT<float> {
    using V2 = float2;
};
template <>
struct VT<double> {
    using V2 = double2;
};

// Row kernels: a workgroup covers kRows groups of 256 consecutive vertex rows
// (thread t takes rows base + 256 r + t, so every group stays 4 whole SELL
// slices and every access stays coalesced); nblk = ceil(N / (256 kRows))
// partial records per system, reduced once per system into the PCG scalars
// (k_red_rzrr / k_red_pq). kRows = 1: a workgroup lives one 256-row group
// long, so the workgroups of neighbouring row blocks run side by side and the
// symmetric layout's transposed reads find their lines in L2 (C3 SpMV fetch
// 11.9 -> 8.9 GB per launch); 4 was the shape while every workgroup
// re-reduced the previous launch's partials itself.
constexpr int kRows = 1;
constexpr int kRowsPerWG = kWG * kRows;

__device__ __forceinline__ void ld_blk(const float *A, int64_t pos, float (&a)[4]) {
    const float4 v = reinterpret_cast<const float4 *>(A)[pos];
    a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w;
}
__device__ __forceinline__ void ld_blk(const double *A, int64_t pos, double (&a)[4]) {
    const double2 v0 = reinterpret_cast<const double2 *>(A)[2 * pos];
    const double2 v1 = reinterpret_cast<const double2 *>(A)[2 * pos + 1];
    a[0] = v0.x; a[1] = v0.y; a[2] = v1.x; a[3] = v1.y;
}

// bf16 copies of the level-0 operator for the multigrid smoother sweeps (the
// preconditioner only needs an SPD approximation of A; rounding the blocks
// (i,j) and (j,i)^T alike keeps it symmetric) -- half the bytes of A32.
__device__ __forceinline__ uint32_t bf16_bits(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;  // round to nearest even
}
__device__ __forceinline__ float bf16_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }
__device__ __forceinline__ uint2 bf16x4(float a, float b, float c, float d) {
    return make_uint2(bf16_bits(a) | (bf16_bits(b) << 16), bf16_bits(c) | (bf16_bits(d) << 16));
}

// The level-0 sweep copy of A (k_res0, k_post0, the smoother's D from the
// diagonal block, the level-0 Galerkin product): 4 bf16 entries (8 B) per
// 2x2 block, handled as a raw uint2. Measured and not kept (round 2,
// profiles/r02_ab/l0_i8_*): 6 B per block as 4 int8 codes and a bf16 scale in
// 64-position records -- the sweeps moved fewer bytes but issued more (two
// loads and a record address per slot, the decode): k_post0 934 -> 1206 us,
// k_res0 959 -> 1045 us, the assembly 9.9 -> 11.0 ms; C3 -5.7 %.
__device__ __forceinline__ uint2 h0_ld(const uint2 *H, int64_t q) { return H[q]; }
__device__ __forceinline__ void h0_st(uint2 *H, int64_t q, float a, float b, float c, float d) {
    H[q] = bf16x4(a, b, c, d);
}
// the transposed block (swap the off-diagonal entries)
__device__ __forceinline__ uint2 h0_tr(uint2 h) {
    return make_uint2((h.x & 0xFFFFu) | (h.y << 16), (h.x >> 16) | (h.y & 0xFFFF0000u));
}
// entries a00, a01, a10, a11
__device__ __forceinline__ void h0_dec(uint2 h, float &a00, float &a01, float &a10, float &a11) {
    a00 = bf16_lo(h.x); a01 = bf16_hi(h.x); a10 = bf16_lo(h.y); a11 = bf16_hi(h.y);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    return v;  // valid in lane 0
}

// Deterministic workgroup sum of NV values over NT threads (lds: NT / 64 * NV
// doubles), waves summed in order; every thread gets the result. Waves that
// contribute 0 leave the bits of the 256-thread sum unchanged.
template <int NV, int NT = kWG>
__device__ __forceinline__ void block_sum(double (&v)[NV], double *lds) {
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = wave_sum(v[k]);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) lds[w * NV + k] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        double s = ((lds[k] + lds[NV + k]) + lds[2 * NV + k]) + lds[3 * NV + k];
#pragma unroll
        for (int q = 4; q < NT / 64; ++q) s += lds[q * NV + k];
        v[k] = s;
    }
    __syncthreads();
}

// block_sum over each group of kWG threads of an NQ * kWG workgroup (the
// fused solve runs NQ row blocks side by side): lds holds NQ * 4 * NV
// doubles; the same order as block_sum<NV, kWG>, so the same bits.
template <int NV, int NQ>
__device__ __forceinline__ void block_sum_q(double (&v)[NV], double *lds) {
    if constexpr (NQ == 1) {
        block_sum<NV, kWG>(v, lds);
    } else {
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] = wave_sum(v[k]);
        const int w = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) {
#pragma unroll
            for (int k = 0; k < NV; ++k) lds[w * NV + k] = v[k];
        }
        __syncthreads();
        const double *L = lds + (w & ~3) * NV;
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] = ((L[k] + L[NV + k]) + L[2 * NV + k]) + L[3 * NV + k];
        __syncthreads();
    }
}
// the thread's index within its group of kWG (row kernels: its row)
__device__ __forceinline__ int32_t row_tid() { return (int32_t)(threadIdx.x & (kWG - 1)); }

// Maxima of non-negative values (the refinement's error control): the
// order-free counterparts of wave_sum / block_sum_q.
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_down(v, o, 64));
    return v;  // valid in lane 0
}
// over each group of kWG threads of an NQ * kWG workgroup (lds: NQ * 4 * NV
// doubles); every thread of the group gets its group's maxima
template <int NV, int NQ>
__device__ __forceinline__ void block_max_q(double (&v)[NV], double *lds) {
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = wave_max(v[k]);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) lds[w * NV + k] = v[k];
    }
    __syncthreads();
    const double *L = lds + (w & ~3) * NV;
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = fmax(fmax(L[k], L[NV + k]), fmax(L[2 * NV + k], L[3 * NV + k]));
    __syncthreads();
}
// over the whole NT-thread workgroup (lds: NT / 64 * NV doubles)
template <int NV, int NT>
__device__ __forceinline__ void block_max(double (&v)[NV], double *lds) {
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = wave_max(v[k]);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) lds[w * NV + k] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        double s = lds[k];
#pragma unroll
        for (int q = 1; q < NT / 64; ++q) s = fmax(s, lds[q * NV + k]);
        v[k] = s;
    }
    __syncthreads();
}

// Sum n partials of NV values each (record stride NV) in a fixed order: the
// first kWG threads load, so any workgroup size NT gets the same bits.
template <int NV, int NT = kWG>
__device__ __forceinline__ void reduce_partials(const double *part, int n, double (&out)[NV],
                                                double *lds) {
#pragma unroll
    for (int k = 0; k < NV; ++k) out[k] = 0.0;
    int q = threadIdx.x < kWG ? (int)threadIdx.x : n;
    for (; q + 3 * kWG < n; q += 4 * kWG) {  // four independent loads in flight
        double v[4][NV];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int k = 0; k < NV; ++k) v[u][k] = part[(int64_t)(q + u * kWG) * NV + k];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int k = 0; k < NV; ++k) out[k] += v[u][k];
    }
    for (; q < n; q += kWG) {
#pragma unroll
        for (int k = 0; k < NV; ++k) out[k] += part[(int64_t)q * NV + k];
    }
    block_sum<NV, NT>(out, lds);
}

// Materialised A of B systems (inner PCG operator).
template <typename V>
struct MatArgs {
    int64_t sell_nb;
    const int32_t *sell_off, *sell_col;
    const int32_t *sell_mir;  // mirror table (symmetric reads), or null
    const int32_t *vptr;      // plain reads: the adjacency row pointers (row i holds
                              // vptr[i+1] - vptr[i] blocks), or null (slice width)
    const V *A;  // [B][sell_nb][4]
};

// The slots row i reads in a plain-read pass: its own block count, not the
// slice width. A lane past its row's blocks re-loads its last block (already
// in the wave's cache lines) and is masked, so the padding of a slice whose
// rows are sorted by degree (irregular meshes, mesh_prepare_host) -- whole
// 128-B lines of tail lanes -- is never fetched (R3: 1.32 M SELL slots for
// 1.15 M blocks). Bit-identical: a padding slot only ever added 0.
__device__ __forceinline__ int32_t row_width(const int32_t *vptr, int32_t i, int32_t w) {
    return vptr ? min(w, vptr[i + 1] - vptr[i]) : w;
}

// Symmetric reads: the fp32 and bf16 operators read a lower
// block (i, j), j < i, as the transpose of block (j, i) through the mirror
// table (sell_mirror), so only the diagonal and upper blocks move from HBM;
// row j of the same or a recent row block has just read them, and the
// mirrored reads of 64 neighbouring rows fall on about as few cache lines as
// their own reads would. Padding slots read the row's diagonal, masked.
__device__ __forceinline__ int64_t mir_pos(int32_t m, int64_t diag) { return m < 0 ? diag : (int64_t)(m & kMirPos); }

template <typename V>
__device__ __forceinline__ typename VT<V>::V2 ld2(const V *p) {
    return *reinterpret_cast<const typename VT<V>::V2 *>(p);
}

// y_i = sum_t A_blk(i,t) x_col(i,t) over the SELL-64 row of vertex i.
// Slots are processed U at a time with every load of a chunk issued before
// the first use (column indices, then block values, then the x gathers), so
// a row costs two memory round trips instead of two per slot. Slots past
// the slice width re-load the last valid slot and are masked out, keeping
// every load unconditional.
// The fine-level operator passes run at >= 5 waves per SIMD (82-88 VGPRs,
// no scratch; 92-105 at 4 waves: k_post0 -5.6 %, C3 +1.7 %), 8 slots per
// load batch (4: SpMV +3 %).
#define MOF_ROW_OCC __attribute__((amdgpu_waves_per_eu(5, 8)))
constexpr int kSpmvU = 8, kSweepU = 8;

// ZH: the operand is a bf16 pair per row (uint32 each; x points at the
// system's first one) instead of V2
template <bool sym, typename V, bool ZH = false>
__device__ __forceinline__ void spmv_row_t(const MatArgs<V> &mt, int32_t b, int32_t i,
                                           const V *__restrict__ x, V &y0, V &y1) {
    // no fp contraction: the symmetric and the plain instance must round
    // alike (the fp64 A is bit-symmetric, so both give the same bits), which
    // contraction left to the code generator would not guarantee
#pragma clang fp contract(off)
    using V2 = typename VT<V>::V2;
    constexpr int U = kSpmvU;  // fp64: 525 vs 536 us per C2 launch with 4
    const V *A = mt.A + 4 * (int64_t)b * mt.sell_nb;
    const int32_t s = i >> 6, l = i & 63;
    const int32_t o = mt.sell_off[s];
    const int32_t w = (mt.sell_off[s + 1] - o) >> 6;
    const int32_t wl = sym ? w : row_width(mt.vptr, i, w);  // this row's slots
    V a0 = 0, a1 = 0;
    for (int32_t t0 = 0; t0 < w; t0 += U) {
        int32_t j[U], mr[U];
        V blk[U][4];
        V2 xj[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int32_t t = min(t0 + u, wl - 1);
            j[u] = mt.sell_col[(int64_t)o + t * kSlice + l];
            if constexpr (sym) mr[u] = mt.sell_mir[(int64_t)o + t * kSlice + l];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int32_t t = min(t0 + u, wl - 1);
            if constexpr (sym)
                ld_blk(A, mir_pos(mr[u], (int64_t)o + l), blk[u]);
            else
                ld_blk(A, (int64_t)o + t * kSlice + l, blk[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if constexpr (ZH) {
                const uint32_t h = reinterpret_cast<const uint32_t *>(x)[j[u]];
                xj[u] = V2{bf16_lo(h), bf16_hi(h)};
            } else {
                xj[u] = ld2(x + 2 * (int64_t)j[u]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if constexpr (sym) {
                const bool on = t0 + u < w && mr[u] >= 0;
                const bool tr = (mr[u] & kMirT) != 0;
                const V b1 = tr ? blk[u][2] : blk[u][1], b2 = tr ? blk[u][1] : blk[u][2];
                a0 += on ? blk[u][0] * xj[u].x + b1 * xj[u].y : (V)0;
                a1 += on ? b2 * xj[u].x + blk[u][3] * xj[u].y : (V)0;
            } else {
                const bool on = t0 + u < wl;
                a0 += on ? blk[u][0] * xj[u].x + blk[u][1] * xj[u].y : (V)0;
                a1 += on ? blk[u][2] * xj[u].x + blk[u][3] * xj[u].y : (V)0;
            }
        }
    }
    y0 = a0;
    y1 = a1;
}
// sell_mir == nullptr (a mesh without symmetric reads, and fp64): every block
// at its own position, no table reads
template <typename V, bool ZH = false>
__device__ __forceinline__ void spmv_row(const MatArgs<V> &mt, int32_t b, int32_t i,
                                         const V *__restrict__ x, V &y0, V &y1) {
    // fp64 too: the fp64 A is bit-symmetric (the reference's mirrored
    // assignment, §2.2), so the transposed reads give the same bits
    if (mt.sell_mir)
        spmv_row_t<true, V, ZH>(mt, b, i, x, y0, y1);
    else
        spmv_row_t<false, V, ZH>(mt, b, i, x, y0, y1);
}

// XCD-aware workgroup -> (row block, system): workgroups w and w+8 share an
// XCD (round-robin dispatch; speed only, never correctness). XCD x takes row
// blocks [x*chunk, (x+1)*chunk) of every system and walks them in groups of G
// systems: row block by row block with the G systems of a row block back to
// back, then the next group. The workgroups in flight on an XCD share the row
// block's column indices (and any other per-row data common to all systems)
// in that XCD's L2, and with a small G the neighbour rows a system gathers
// from the next row block are still in L2 when that row block comes up.
// G per kernel family (C3, B=256, rocprof: SpMV -7 %, smoother sweeps -3 %,
// level-0 Galerkin -13 %, residual -8 % against G = B; G = 0 means all B).
// Round 3 (same box, profiles/r03_ab/grp/): the row assembly 32 -> 8
// (10.2 -> 8.8 ms per 512-system batch), the residual 32 -> 8 system pairs
// (5.73 -> 5.55 ms per launch); the Galerkin products at 1 instead of 8:
// -0.7 % timesteps/s.
// Round 6, rocprof on one box (profiles/r06/xfer_grp/): the transfers from
// G = B to 8 -- F3's smoothed restriction 1740 -> 1526 us, level 1's 645 ->
// 402, the smoothed prolongation 1155 -> 1086; C3's tentative prolongation
// 638 -> 609 (4 / 16 / 32 no better).
constexpr int32_t kGrpSpmv = 8, kGrpSmooth = 8, kGrpRes = 8, kGrpGal = 8, kGrpAsm = 8, kGrpProl = 8,
                  kGrpRestr = 8;
__host__ __device__ __forceinline__ int32_t sys_group(int32_t B, int32_t G) { return G > 0 && G < B ? G : B; }

__host__ __device__ __forceinline__ bool xcd_map_w(int32_t w, int32_t nblk, int32_t B, int32_t &rb, int32_t &sys,
                                                   int32_t grp_sz) {
    const int32_t q = w >> 3;
    const int32_t chunk = (nblk + 7) >> 3;
    const int32_t G = sys_group(B, grp_sz);
    const int32_t grp = q / (chunk * G), rem = q - grp * chunk * G;
    sys = grp * G + rem % G;
    rb = (w & 7) * chunk + rem / G;
    return rb < nblk && sys < B;
}
__device__ __forceinline__ bool xcd_map(int32_t nblk, int32_t B, int32_t &rb, int32_t &sys, int32_t grp_sz) {
    return xcd_map_w((int32_t)blockIdx.x, nblk, B, rb, sys, grp_sz);
}

// A dispatch's grid is at most 2^32 - 1 work-items (kWG per workgroup): a
// launch past it would run only part of its workgroups, so it fails loudly
// here instead (round 4: an unsliced by-entry Galerkin launch at S1's size).
inline unsigned xcd_grid(int32_t nblk, int32_t B, int32_t grp_sz) {
    const int64_t G = sys_group(B, grp_sz);
    const int64_t n = 8 * G * ((B + G - 1) / G) * ((nblk + 7) / 8);
    MOF_REQUIRE(n * kWG < ((int64_t)1 << 32), "launch grid past 2^32 work-items (batch too large for this mesh)");
    return (unsigned)n;
}
// The largest batch whose xcd_grid over `nblk` blocks per system (system
// groups of grp_sz) stays within 2^32 - 1 work-items.
inline int32_t xcd_batch_cap(int64_t nblk, int32_t grp_sz) {
    const int64_t lim = (((int64_t)1 << 32) - 1) / kWG;  // workgroups
    const int64_t per = 8 * ((nblk + 7) / 8);          // workgroups per system (padded to the 8 XCDs)
    int64_t B = std::min<int64_t>(lim / per, 1 << 30);
    auto n = [&](int64_t b) {
        const int64_t G = b > grp_sz && grp_sz > 0 ? grp_sz : b;
        return 8 * G * ((b + G - 1) / G) * ((nblk + 7) / 8);
    };
    while (B > 1 && n(B) > lim) --B;
    return (int32_t)std::max<int64_t>(1, B);
}


// A launch over n logical systems: logical l is system map[l] (map null: l
// itself). A batch's tail iterations launch only the systems still running
// (pcg: at most a quarter of the batch left), so the grid is not mostly
// early-exiting workgroups; a system's arithmetic is the same whichever slot
// of a launch it runs in (no fp contraction in the multi-system kernels).
struct SysMap {
    const int32_t *map;
    int32_t n;
};
inline SysMap sys_all(int32_t B) { return SysMap{nullptr, B}; }
__device__ __forceinline__ int32_t sm_b(const SysMap &s, int32_t l) {
    l = min(l, s.n - 1);
    return s.map ? s.map[l] : l;
}

struct MatH {
    int64_t sell_nb;
    const int32_t *sell_off, *sell_col;
    const int32_t *sell_mir;  // mirror table (symmetric reads), or null
    const int32_t *vptr;      // plain reads: row block counts (row_width), or null
    const uint2 *A;  // the level-0 sweep copy (h0_ld), [B][sell_nb] blocks
};

// spmv_row_hx_t for NS systems of one row per thread: the column and mirror
// loads (shared by all systems) are issued once for the NS systems. No fp
// contraction, so every system slot rounds alike (a system's bits must not
// depend on its slot, i.e. on the batch split). xload(t, j): system t's
// operand of column j.
template <bool sym, int NS, int U = kSweepU, typename XL>
__device__ __forceinline__ void spmv_row_hx_ns(const MatH &mt, const int32_t (&bs)[NS], int32_t i, XL &&xload,
                                               float (&y)[NS][2], uint2 *diag = nullptr) {
#pragma clang fp contract(off)
    const int32_t s = i >> 6, l = i & 63;
    const int32_t o = mt.sell_off[s];
    const int32_t w = (mt.sell_off[s + 1] - o) >> 6;
    const int32_t wl = sym ? w : row_width(mt.vptr, i, w);  // this row's slots
    float acc[NS][2];
#pragma unroll
    for (int t = 0; t < NS; ++t) acc[t][0] = acc[t][1] = 0.f;
    for (int32_t t0 = 0; t0 < w; t0 += U) {
        int32_t j[U], mr[U];
        int64_t pos[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            pos[u] = (int64_t)o + min(t0 + u, wl - 1) * kSlice + l;
            j[u] = mt.sell_col[pos[u]];
            if constexpr (sym) mr[u] = mt.sell_mir[pos[u]];
        }
        if constexpr (sym) {
#pragma unroll
            for (int u = 0; u < U; ++u) pos[u] = mir_pos(mr[u], (int64_t)o + l);
        }
        uint2 blk[NS][U];
        float2 xj[NS][U];
#pragma unroll
        for (int t = 0; t < NS; ++t)
#pragma unroll
            for (int u = 0; u < U; ++u) blk[t][u] = h0_ld(mt.A, (int64_t)bs[t] * mt.sell_nb + pos[u]);
        if (diag && t0 == 0) {  // slot 0: the diagonal block, never mirrored
#pragma unroll
            for (int t = 0; t < NS; ++t) diag[t] = blk[t][0];
        }
#pragma unroll
        for (int t = 0; t < NS; ++t)
#pragma unroll
            for (int u = 0; u < U; ++u) xj[t][u] = xload(t, j[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            bool on = t0 + u < wl;
            bool tr = false;
            if constexpr (sym) {
                on = on && mr[u] >= 0;
                tr = (mr[u] & kMirT) != 0;
            }
#pragma unroll
            for (int t = 0; t < NS; ++t) {
                const uint2 h = tr ? h0_tr(blk[t][u]) : blk[t][u];
                float e00, e01, e10, e11;
                h0_dec(h, e00, e01, e10, e11);
                acc[t][0] += on ? e00 * xj[t][u].x + e01 * xj[t][u].y : 0.f;
                acc[t][1] += on ? e10 * xj[t][u].x + e11 * xj[t][u].y : 0.f;
            }
        }
    }
#pragma unroll
    for (int t = 0; t < NS; ++t) {
        y[t][0] = acc[t][0];
        y[t][1] = acc[t][1];
    }
}

// The V-cycle's level-0 iterate: the pre-smoothed x0 = w D^-1 r (written by
// the PCG update, gathered by k_res0, read by the prolongation) as a bf16
// pair (4 B), and the corrected x = x0 + Q y (written by the prolongation,
// gathered by k_post0) chosen per mesh (AmgDevice::xm): in the x0 format in
// place, or float2 in level 0's y buffer. Round-1 comparison (PCG
// its/timestep and timesteps/s, C3 / R3 / C2 mixed): both float2 18 / 101.9 /
// 22.8 at 2357 / 374 / 9474; both bf16 18 / 115.8 / 22.8 at 2472 / 345 /
// 9943; bf16 x0, float2 x 18 / 103 / 22.8 at 2428 / 376 / 9676 (same box).
__device__ __forceinline__ float2 ld_x0(const float *x, int64_t vi) {
    const uint32_t h = reinterpret_cast<const uint32_t *>(x)[vi];
    return make_float2(bf16_lo(h), bf16_hi(h));
}
__device__ __forceinline__ void st_x0(float *x, int64_t vi, float a, float b) {
    reinterpret_cast<uint32_t *>(x)[vi] = bf16_bits(a) | (bf16_bits(b) << 16);
}

// 2x2 block stored as 4 bf16: y = D v
__device__ __forceinline__ float2 bf16_mat2(uint2 d, float v0, float v1) {
    return make_float2(bf16_lo(d.x) * v0 + bf16_hi(d.x) * v1, bf16_lo(d.y) * v0 + bf16_hi(d.y) * v1);
}

// The level-0 smoother's D^-1 v from the diagonal block of the bf16 operator
// itself (slot 0 of the row: diagonal first), solved in fp32: no separate
// D^-1 array to stream (the pre- and post-smoothing use the same D, so the
// cycle stays symmetric; round 2: k_post0 1328 -> 1266 us).
__device__ __forceinline__ float2 bf16_diag_solve(uint2 a, float v0, float v1) {
    float a00, a01, a10, a11;
    h0_dec(a, a00, a01, a10, a11);
    const float id = 1.f / (a00 * a11 - a01 * a10);
    return make_float2((a11 * v0 - a01 * v1) * id, (a00 * v1 - a10 * v0) * id);
}
// slot 0 (the diagonal block) of row i of system b in a SELL-64 bf16 operator
__device__ __forceinline__ uint2 bf16_diag_block(const uint2 *A, int64_t sell_nb, const int32_t *sell_off,
                                                 int32_t b, int32_t i) {
    return h0_ld(A, (int64_t)b * sell_nb + sell_off[i >> 6] + (i & 63));
}

}  // namespace
}  // namespace mof
