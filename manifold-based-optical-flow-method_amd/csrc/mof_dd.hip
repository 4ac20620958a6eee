// mof_dd.hip -- domain-decomposed solve of one timestep over P vertex parts
// (mof_dd.h): halo kernels, the two transports
// (in-process on one device, RCCL with one process per GPU) and the mof_dd_*
// entry points of include/mof.h.
//
// Halo (in-process): one gather launch covers the ghost rows of every part,
//   z_p[b][n_own_p + g] = z_q[b][ghost_src]   (one entry per ghost row).
// Halo (RCCL): pack the rows each neighbour reads into [B][rows][2] segments,
//   ncclSend/ncclRecv with all neighbours inside one group, unpack into the
//   ghost rows (they are grouped by owner, so a received segment is one
//   contiguous ghost range per system).
// Partial sums: every PCG kernel writes its part's records of the shared
//   [P][B][nmax] array; with RCCL each rank then all-gathers them in place.
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <type_traits>

#include <rccl/rccl.h>

#include "mof_dd.h"
#include "mof_internal.h"
#include "mof_rowkern.h"

int mof_io_guard(const std::function<void()> &f);  // mof_abi.cpp

namespace mof {

// ---- RCCL, opened at run time (only the RCCL transport needs it) ----------
// The entry points this file calls, with rccl.h's types.
struct RcclApi {
    void *h = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
};

namespace {

RcclApi *rccl_open() {
    static RcclApi api;
    static bool tried = false;
    static std::mutex mu;  // handles may be created from several host threads
    std::lock_guard<std::mutex> lock(mu);
    if (api.h) return &api;
    MOF_REQUIRE(!tried, "librccl could not be loaded");
    tried = true;
    const char *env = knob(Knob::RcclLib);
    const char *names[] = {env, "librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"};
    for (const char *n : names) {
        if (!n) continue;
        api.h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
        if (api.h) break;
    }
    if (!api.h) throw Error{MOF_E_HIP, std::string("cannot load librccl: ") + dlerror()};
    auto sym = [&](const char *s) {
        void *f = dlsym(api.h, s);
        if (!f) throw Error{MOF_E_HIP, std::string("librccl lacks ") + s};
        return f;
    };
    auto load = [&](auto &fn, const char *name) { fn = reinterpret_cast<std::decay_t<decltype(fn)>>(sym(name)); };
    load(api.get_unique_id, "ncclGetUniqueId");
    load(api.comm_init_rank, "ncclCommInitRank");
    load(api.comm_destroy, "ncclCommDestroy");
    load(api.all_gather, "ncclAllGather");
    load(api.send, "ncclSend");
    load(api.recv, "ncclRecv");
    load(api.group_start, "ncclGroupStart");
    load(api.group_end, "ncclGroupEnd");
    load(api.error_string, "ncclGetErrorString");
    return &api;
}

void nccl_check(RcclApi *a, ncclResult_t rc, const char *what) {
    if (rc != ncclSuccess) throw Error{MOF_E_HIP, std::string(what) + " failed: " + a->error_string(rc)};
}

// ---- kernels ----------------------------------------------------------------

// z_dst[b][dst row] = z_src[b][src row] for every ghost row of every part
template <typename V>
__global__ __launch_bounds__(kWG) void k_halo_pull(int64_t n, int32_t B, const int4 *__restrict__ ent,
                                                   void *const *__restrict__ base,
                                                   const int32_t *__restrict__ nloc) {
    const int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x;
    if (e >= n) return;
    using V2 = typename std::conditional<sizeof(V) == 4, float2, double2>::type;
    const int4 q = ent[e];
    V2 *dst = reinterpret_cast<V2 *>(base[q.x]);
    const V2 *src = reinterpret_cast<const V2 *>(base[q.z]);
    const int64_t ld = nloc[q.x], ls = nloc[q.z];
    for (int32_t b = 0; b < B; ++b) dst[b * ld + q.y] = src[b * ls + q.w];
}

// sendbuf segment k (rows [off_k, off_k + cnt_k) of the send list) as
// [B][cnt_k][2] at element offset 2 B off_k; ent = {row, off_k, cnt_k, -}
template <typename V>
__global__ __launch_bounds__(kWG) void k_halo_pack(int64_t n, int32_t B, int32_t nloc,
                                                   const int4 *__restrict__ ent, const V *__restrict__ x,
                                                   V *__restrict__ buf) {
    const int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x;
    if (e >= n) return;
    const int4 q = ent[e];
    for (int32_t b = 0; b < B; ++b) {
        const int64_t o = 2 * ((int64_t)B * q.y + (int64_t)b * q.z + (e - q.y));
        buf[o] = x[2 * ((int64_t)b * nloc + q.x)];
        buf[o + 1] = x[2 * ((int64_t)b * nloc + q.x) + 1];
    }
}

// ghost row g (= entry e) of the local part from the receive buffer; ent =
// {n_own + g, off_k, cnt_k, -}
template <typename V>
__global__ __launch_bounds__(kWG) void k_halo_unpack(int64_t n, int32_t B, int32_t nloc,
                                                     const int4 *__restrict__ ent, const V *__restrict__ buf,
                                                     V *__restrict__ x) {
    const int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x;
    if (e >= n) return;
    const int4 q = ent[e];
    for (int32_t b = 0; b < B; ++b) {
        const int64_t o = 2 * ((int64_t)B * q.y + (int64_t)b * q.z + (e - q.y));
        x[2 * ((int64_t)b * nloc + q.x)] = buf[o];
        x[2 * ((int64_t)b * nloc + q.x) + 1] = buf[o + 1];
    }
}

// planar V rows of one part's owned vertices (caller order; failed systems
// NaN-filled): V[b][g] = x[b][i].0, V[b][N + g] = x[b][i].1
__global__ __launch_bounds__(kWG) void k_dd_scatter(int32_t n_own, int32_t nloc, int32_t N,
                                                    const int32_t *__restrict__ l2g,
                                                    const double *__restrict__ x,
                                                    const int32_t *__restrict__ sysi,
                                                    double *__restrict__ V) {
    const int32_t i = blockIdx.x * kWG + threadIdx.x;
    const int32_t b = blockIdx.y;
    if (i >= n_own) return;
    const bool failed = sysi[b * kSysStride + SI_FAILED] != 0;
    const double2 v = *reinterpret_cast<const double2 *>(x + 2 * ((int64_t)b * nloc + i));
    const int32_t g = l2g[i];
    const double nan = __builtin_nan("");
    V[(int64_t)b * 2 * N + g] = failed ? nan : v.x;
    V[(int64_t)b * 2 * N + N + g] = failed ? nan : v.y;
}

// RCCL: owned x64 rows -> this rank's [B][nmax_own][2] record of vgather
__global__ __launch_bounds__(kWG) void k_dd_own_pack(int32_t n_own, int32_t nloc, int32_t nmax_own,
                                                     const double *__restrict__ x,
                                                     const int32_t *__restrict__ sysi,
                                                     double *__restrict__ out) {
    const int32_t i = blockIdx.x * kWG + threadIdx.x;
    const int32_t b = blockIdx.y;
    if (i >= n_own) return;
    const bool failed = sysi[b * kSysStride + SI_FAILED] != 0;
    double2 v = *reinterpret_cast<const double2 *>(x + 2 * ((int64_t)b * nloc + i));
    if (failed) v = make_double2(__builtin_nan(""), __builtin_nan(""));
    *reinterpret_cast<double2 *>(out + 2 * ((int64_t)b * nmax_own + i)) = v;
}

// RCCL: all parts' gathered owned rows -> planar V
__global__ __launch_bounds__(kWG) void k_dd_own_scatter(int32_t P, int32_t B, int32_t nmax_own, int32_t N,
                                                        const int32_t *__restrict__ l2g,
                                                        const double *__restrict__ in,
                                                        double *__restrict__ V) {
    const int32_t i = blockIdx.x * kWG + threadIdx.x;
    const int32_t b = blockIdx.y;
    if (i >= nmax_own) return;
    for (int32_t q = 0; q < P; ++q) {
        const int32_t g = l2g[(int64_t)q * nmax_own + i];
        if (g < 0) continue;
        const double2 v = *reinterpret_cast<const double2 *>(in + 2 * (((int64_t)q * B + b) * nmax_own + i));
        V[(int64_t)b * 2 * N + g] = v.x;
        V[(int64_t)b * 2 * N + N + g] = v.y;
    }
}

inline unsigned blocks(int64_t n) { return (unsigned)((n + kWG - 1) / kWG); }

}  // namespace

// ---- transport hooks ---------------------------------------------------------

namespace {

void host_check(int rc, const char *what) {
    if (rc != 0) throw Error{MOF_E_HIP, std::string("host transport: ") + what + " failed (" + std::to_string(rc) + ")"};
}

// host-staged all-gather of `per` elements of esz bytes at base + per*rank
// into base[0 .. P*per) of every rank
void host_allgather(mof_dd *d, void *base, size_t per, size_t esz, hipStream_t s) {
    const size_t bytes = per * esz, all = bytes * (size_t)d->P;
    if (d->hrecv.size() < all) d->hrecv.resize(all);
    char *h = d->hrecv.data();
    MOF_HIP(hipMemcpyAsync(h + bytes * d->rank, static_cast<char *>(base) + bytes * d->rank, bytes,
                           hipMemcpyDeviceToHost, s));
    MOF_HIP(hipStreamSynchronize(s));
    host_check(d->host.allgather(d->host.ctx, h + bytes * d->rank, h, (int64_t)bytes), "allgather");
    MOF_HIP(hipMemcpyAsync(base, h, all, hipMemcpyHostToDevice, s));
    MOF_HIP(hipStreamSynchronize(s));
}

}  // namespace

void dd_sync_partials(mof_dd *d, double *base, size_t per_part, hipStream_t s) {
    if (d->rank < 0 || d->P == 1) return;  // in-process: one shared array
    if (d->hosted) {
        host_allgather(d, base, per_part, sizeof(double), s);
        return;
    }
    nccl_check(d->nccl,
               d->nccl->all_gather(base + per_part * (size_t)d->rank, base, per_part, ncclFloat64, static_cast<ncclComm_t>(d->comm), s),
               "ncclAllGather(partials)");
}

// The minimum of one value over the ranks (every rank gets the same): an
// all-gather of one double per rank into `agree`.
double dd_all_min(mof_dd *d, double mine, hipStream_t s) {
    if (d->rank < 0 || d->P == 1) return mine;
    MOF_HIP(hipMemcpyAsync(d->agree.p + d->rank, &mine, sizeof(double), hipMemcpyHostToDevice, s));
    if (d->hosted)
        host_allgather(d, d->agree.p, 1, sizeof(double), s);
    else
        nccl_check(d->nccl,
                   d->nccl->all_gather(d->agree.p + d->rank, d->agree.p, 1, ncclFloat64,
                                       static_cast<ncclComm_t>(d->comm), s),
                   "ncclAllGather(status)");
    std::vector<double> all(d->P);
    MOF_HIP(hipMemcpyAsync(all.data(), d->agree.p, sizeof(double) * d->P, hipMemcpyDeviceToHost, s));
    MOF_HIP(hipStreamSynchronize(s));
    double v = mine;
    for (double x : all) v = std::min(v, x);
    return v;
}

bool dd_all_ok(mof_dd *d, bool ok, hipStream_t s) { return dd_all_min(d, ok ? 1.0 : 0.0, s) == 1.0; }

// The pack -> exchange -> unpack path: the RCCL transport, or in-process
// parts with MOF_DD_STAGED (the same kernels and segment offsets, the
// exchange done by device copies).
static bool staged(const mof_dd *d) { return d->rank >= 0 || (d->flags & MOF_DD_STAGED); }

void dd_halo(mof_dd *d, int32_t B, bool f32, int which, hipStream_t s) {
    if (d->P == 1) return;
    if (!staged(d)) {
        const int64_t n = d->n_halo;
        if (n == 0) return;
        void *const *tab = d->vbase.p + (which ? d->P : 0);
        if (f32)
            k_halo_pull<float><<<blocks(n), kWG, 0, s>>>(n, B, d->halo.p, tab, d->nloc.p);
        else
            k_halo_pull<double><<<blocks(n), kWG, 0, s>>>(n, B, d->halo.p, tab, d->nloc.p);
        MOF_HIP(hipGetLastError());
        return;
    }
    const size_t esz = f32 ? 4 : 8;
    const size_t L = d->parts.size();
    char *sbuf = reinterpret_cast<char *>(d->sendbuf.p), *rbuf = reinterpret_cast<char *>(d->recvbuf.p);
    // byte address of element e of local part l's send / receive region
    auto sptr = [&](size_t l, int64_t e) { return sbuf + (2 * (size_t)d->cap * d->send_base[l] + e) * esz; };
    auto rptr = [&](size_t l, int64_t e) { return rbuf + (2 * (size_t)d->cap * d->recv_base[l] + e) * esz; };
    auto vec = [&](size_t l) {
        return which ? (void *)d->parts[l]->ws.x64.p : (void *)d->parts[l]->ws.vz.p;
    };
    for (size_t l = 0; l < L; ++l) {
        const DdPart &D = d->plan.parts[d->part_ids[l]];
        const int64_t ns = (int64_t)D.send_idx.size();
        if (ns == 0) continue;
        const int4 *ent = d->send_ent.p + d->send_base[l];
        if (f32)
            k_halo_pack<float><<<blocks(ns), kWG, 0, s>>>(ns, B, D.n_loc(), ent, static_cast<const float *>(vec(l)),
                                                          reinterpret_cast<float *>(sptr(l, 0)));
        else
            k_halo_pack<double><<<blocks(ns), kWG, 0, s>>>(ns, B, D.n_loc(), ent,
                                                           static_cast<const double *>(vec(l)),
                                                           reinterpret_cast<double *>(sptr(l, 0)));
    }
    MOF_HIP(hipGetLastError());
    if (d->rank >= 0 && d->hosted) {
        // the rank's packed segments to the host, one exchange call with all
        // neighbours, the received segments back to the device
        const DdPart &D = d->plan.parts[d->rank];
        const size_t sb = 2 * (size_t)B * D.send_idx.size() * esz, rb = 2 * (size_t)B * D.n_ghost * esz;
        if (d->hsend.size() < sb) d->hsend.resize(sb);
        if (d->hrecv.size() < rb) d->hrecv.resize(rb);
        if (sb) MOF_HIP(hipMemcpyAsync(d->hsend.data(), sptr(0, 0), sb, hipMemcpyDeviceToHost, s));
        MOF_HIP(hipStreamSynchronize(s));
        const size_t nn = D.nbr.size();
        std::vector<const void *> sp(nn);
        std::vector<void *> rp(nn);
        std::vector<int64_t> sc(nn), rc(nn);
        for (size_t k = 0; k < nn; ++k) {
            sp[k] = d->hsend.data() + 2 * (size_t)B * D.send_off[k] * esz;
            sc[k] = (int64_t)(2 * (size_t)B * (D.send_off[k + 1] - D.send_off[k]) * esz);
            rp[k] = d->hrecv.data() + 2 * (size_t)B * D.recv_off[k] * esz;
            rc[k] = (int64_t)(2 * (size_t)B * (D.recv_off[k + 1] - D.recv_off[k]) * esz);
        }
        host_check(d->host.exchange(d->host.ctx, (int32_t)nn, D.nbr.data(), sp.data(), sc.data(), rp.data(), rc.data()),
                   "exchange");
        if (rb) MOF_HIP(hipMemcpyAsync(rptr(0, 0), d->hrecv.data(), rb, hipMemcpyHostToDevice, s));
        MOF_HIP(hipStreamSynchronize(s));
    } else if (d->rank >= 0) {
        const DdPart &D = d->plan.parts[d->rank];
        const ncclDataType_t dt = f32 ? ncclFloat32 : ncclFloat64;
        RcclApi *a = d->nccl;
        ncclComm_t comm = static_cast<ncclComm_t>(d->comm);
        nccl_check(a, a->group_start(), "ncclGroupStart");
        for (size_t k = 0; k < D.nbr.size(); ++k) {
            const size_t sc = 2 * (size_t)B * (D.send_off[k + 1] - D.send_off[k]);
            const size_t rc = 2 * (size_t)B * (D.recv_off[k + 1] - D.recv_off[k]);
            if (sc) nccl_check(a, a->send(sptr(0, 2 * (int64_t)B * D.send_off[k]), sc, dt, D.nbr[k], comm, s), "ncclSend");
            if (rc) nccl_check(a, a->recv(rptr(0, 2 * (int64_t)B * D.recv_off[k]), rc, dt, D.nbr[k], comm, s), "ncclRecv");
        }
        nccl_check(a, a->group_end(), "ncclGroupEnd");
    } else {
        // in-process: part q's segment for p -> p's receive segment for q
        for (size_t p = 0; p < L; ++p) {
            const DdPart &D = d->plan.parts[p];
            for (size_t k = 0; k < D.nbr.size(); ++k) {
                const int32_t q = D.nbr[k];
                const DdPart &Q = d->plan.parts[q];
                const size_t kk = (size_t)(std::lower_bound(Q.nbr.begin(), Q.nbr.end(), (int32_t)p) - Q.nbr.begin());
                const size_t cnt = (size_t)(D.recv_off[k + 1] - D.recv_off[k]);
                MOF_REQUIRE(kk < Q.nbr.size() && (size_t)(Q.send_off[kk + 1] - Q.send_off[kk]) == cnt,
                            "halo segments disagree (internal error)");
                MOF_HIP(hipMemcpyAsync(rptr(p, 2 * (int64_t)B * D.recv_off[k]), sptr(q, 2 * (int64_t)B * Q.send_off[kk]),
                                       2 * (size_t)B * cnt * esz, hipMemcpyDeviceToDevice, s));
            }
        }
    }
    for (size_t l = 0; l < L; ++l) {
        const DdPart &D = d->plan.parts[d->part_ids[l]];
        const int64_t ng = D.n_ghost;
        if (ng == 0) continue;
        const int4 *ent = d->recv_ent.p + d->recv_base[l];
        if (f32)
            k_halo_unpack<float><<<blocks(ng), kWG, 0, s>>>(ng, B, D.n_loc(), ent,
                                                            reinterpret_cast<const float *>(rptr(l, 0)),
                                                            static_cast<float *>(vec(l)));
        else
            k_halo_unpack<double><<<blocks(ng), kWG, 0, s>>>(ng, B, D.n_loc(), ent,
                                                             reinterpret_cast<const double *>(rptr(l, 0)),
                                                             static_cast<double *>(vec(l)));
    }
    MOF_HIP(hipGetLastError());
}

void dd_gather_v(mof_dd *d, int32_t B, double *V, hipStream_t s) {
    if (!staged(d)) {
        for (size_t l = 0; l < d->parts.size(); ++l) {
            const DdPart &D = d->plan.parts[d->part_ids[l]];
            mof_mesh *m = d->parts[l];
            k_dd_scatter<<<dim3(blocks(D.n_own), (unsigned)B), kWG, 0, s>>>(
                D.n_own, D.n_loc(), d->N, d->own_l2g.p + d->own_off[l], m->ws.x64.p, m->ws.sysi.p, V);
        }
        MOF_HIP(hipGetLastError());
        return;
    }
    // every part's owned rows into its [B][nmax_own][2] record, all-gathered
    // (RCCL), then one scatter of all records into the planar V
    const size_t per = 2 * (size_t)B * d->nmax_own;
    for (size_t l = 0; l < d->parts.size(); ++l) {
        const int32_t p = d->part_ids[l];
        const DdPart &D = d->plan.parts[p];
        mof_mesh *m = d->parts[l];
        k_dd_own_pack<<<dim3(blocks(D.n_own), (unsigned)B), kWG, 0, s>>>(D.n_own, D.n_loc(), d->nmax_own, m->ws.x64.p,
                                                                         m->ws.sysi.p, d->vgather.p + per * p);
    }
    MOF_HIP(hipGetLastError());
    if (d->rank >= 0 && d->P > 1 && d->hosted)
        host_allgather(d, d->vgather.p, per, sizeof(double), s);
    else if (d->rank >= 0 && d->P > 1)
        nccl_check(d->nccl, d->nccl->all_gather(d->vgather.p + per * d->rank, d->vgather.p, per, ncclFloat64,
                                                static_cast<ncclComm_t>(d->comm), s),
                   "ncclAllGather(V)");
    k_dd_own_scatter<<<dim3(blocks(d->nmax_own), (unsigned)B), kWG, 0, s>>>(d->P, B, d->nmax_own, d->N,
                                                                            d->all_l2g.p, d->vgather.p, V);
    MOF_HIP(hipGetLastError());
}

void dd_ensure(mof_dd *d, int32_t B, uint32_t precision) {
    for (mof_mesh *m : d->parts) ensure_workspace(m, B, precision);
    if (!staged(d)) {
        // halo pointer tables (the workspaces may have been reallocated)
        std::vector<void *> tab(2 * (size_t)d->P);
        for (int32_t p = 0; p < d->P; ++p) {
            tab[p] = d->parts[p]->ws.vz.p;
            tab[d->P + p] = d->parts[p]->ws.x64.p;
        }
        MOF_HIP(hipMemcpy(d->vbase.p, tab.data(), sizeof(void *) * tab.size(), hipMemcpyHostToDevice));
    }
    if (d->cap >= B) return;
    d->cap = B;
    int32_t nmax = 0;
    for (const DdPart &D : d->plan.parts)
        nmax = std::max(nmax, (int32_t)((D.n_loc() + kRowsPerWG - 1) / kRowsPerWG));
    d->nmax = nmax;
    const size_t rec = (size_t)d->P * B * nmax;
    d->part_pq.alloc(2 * rec);  // by iteration parity
    d->part_rzrr.alloc(4 * rec);
    d->part_rr0.alloc(2 * rec);
    int32_t nvmax = 0;  // k_outer_update's blocks of the largest part
    for (const DdPart &D : d->plan.parts) nvmax = std::max(nvmax, (int32_t)((D.n_loc() + kWG - 1) / kWG));
    d->nvmax = nvmax;
    d->part_dx.alloc(2 * (size_t)d->P * B * nvmax);
    if (staged(d)) {
        d->sendbuf.alloc(2 * (size_t)B * std::max<int64_t>(1, d->send_base.back()));
        d->recvbuf.alloc(2 * (size_t)B * std::max<int64_t>(1, d->recv_base.back()));
        d->vgather.alloc(2 * (size_t)d->P * B * d->nmax_own);
    }
}

}  // namespace mof

namespace {

double dd_now_ms() {
    using namespace std::chrono;
    return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

struct DevGuard {
    int prev = 0;
    explicit DevGuard(int dev) {
        (void)hipGetDevice(&prev);
        MOF_HIP(hipSetDevice(dev));
    }
    ~DevGuard() { (void)hipSetDevice(prev); }
};

// host halo/plan tables and the part meshes of one mof_dd
void dd_setup(mof_dd *d, const double *xyz, const double *nrm, const int32_t *tri, const double *area,
              const int32_t *part_in) {
    using namespace mof;
    const double t0 = dd_now_ms();
    const int32_t N = d->N, M = d->M, P = d->P;
    std::vector<int32_t> part(N);
    if (part_in)
        std::copy(part_in, part_in + N, part.begin());
    else
        partition_rcb(xyz, N, P, part.data());
    // global RCM position orders the rows inside each part
    Pattern adj;
    build_pattern(tri, N, M, adj);
    const std::vector<int32_t> key = rcm_order(adj);
    build_dd_plan(tri, N, M, P, part.data(), key.data(), d->plan);
    MOF_HIP(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
    if (d->rank < 0)
        for (int32_t p = 0; p < P; ++p) d->part_ids.push_back(p);
    else
        d->part_ids.push_back(d->rank);
    std::vector<int32_t> own;
    for (int32_t p : d->part_ids) {
        const DdPart &D = d->plan.parts[p];
        const int32_t nl = D.n_loc(), ml = (int32_t)D.tris.size();
        std::vector<double> lx(3 * (size_t)nl), ln(3 * (size_t)nl), la(ml);
        std::vector<int32_t> lt(3 * (size_t)ml), gt(3 * (size_t)ml), loc(N, -1), ident(nl);
        for (int32_t r = 0; r < nl; ++r) {
            loc[D.l2g[r]] = r;
            ident[r] = r;
            for (int c = 0; c < 3; ++c) {
                lx[3 * (size_t)r + c] = xyz[3 * (size_t)D.l2g[r] + c];
                ln[3 * (size_t)r + c] = nrm[3 * (size_t)D.l2g[r] + c];
            }
        }
        for (int32_t t = 0; t < ml; ++t) {
            const int32_t T = D.tris[t];
            la[t] = area[T];
            for (int c = 0; c < 3; ++c) {
                gt[3 * (size_t)t + c] = tri[3 * (size_t)T + c];
                lt[3 * (size_t)t + c] = loc[tri[3 * (size_t)T + c]];
            }
        }
        auto *m = new mof_mesh();
        d->parts.push_back(m);
        // local order fixed (owned first); triangles keep the caller's order for
        // the folds; I is gathered by the caller's (global) vertex ids
        mesh_build(m, lx.data(), ln.data(), lt.data(), la.data(), nl, ml, d->device, d->flags, ident.data(),
                   gt.data());
        mesh_set_own(m, D.n_own);  // ghost rows: decoupled in the part's multigrid cycle
        d->own_off.push_back((int64_t)own.size());
        own.insert(own.end(), D.l2g.begin(), D.l2g.begin() + D.n_own);
    }
    d->own_l2g.alloc(own.size());
    d->own_l2g.upload(own.data(), own.size(), d->stream);
    if (d->rank < 0) {
        std::vector<int4> ent;
        for (int32_t p = 0; p < P; ++p) {
            const DdPart &D = d->plan.parts[p];
            for (int32_t g = 0; g < D.n_ghost; ++g)
                ent.push_back(make_int4(p, D.n_own + g, d->plan.part[D.l2g[D.n_own + g]], D.ghost_src[g]));
        }
        d->n_halo = (int64_t)ent.size();
        d->halo.alloc(std::max<size_t>(1, ent.size()));
        if (!ent.empty()) d->halo.upload(ent.data(), ent.size(), d->stream);
        std::vector<int32_t> nl(P);
        for (int32_t p = 0; p < P; ++p) nl[p] = d->plan.parts[p].n_loc();
        d->nloc.alloc(P);
        d->nloc.upload(nl.data(), P, d->stream);
        d->vbase.alloc(2 * (size_t)P);
    }
    if (d->rank >= 0 || (d->flags & MOF_DD_STAGED)) {
        // pack / unpack entries of every local part, concatenated
        std::vector<int4> se, re;
        d->send_base.assign(1, 0);
        d->recv_base.assign(1, 0);
        for (int32_t p : d->part_ids) {
            const DdPart &D = d->plan.parts[p];
            for (size_t k = 0; k < D.nbr.size(); ++k) {
                for (int32_t e = D.send_off[k]; e < D.send_off[k + 1]; ++e)
                    se.push_back(make_int4(D.send_idx[e], D.send_off[k], D.send_off[k + 1] - D.send_off[k], 0));
                for (int32_t g = D.recv_off[k]; g < D.recv_off[k + 1]; ++g)
                    re.push_back(make_int4(D.n_own + g, D.recv_off[k], D.recv_off[k + 1] - D.recv_off[k], 0));
            }
            d->send_base.push_back((int64_t)se.size());
            d->recv_base.push_back((int64_t)re.size());
        }
        d->send_ent.alloc(std::max<size_t>(1, se.size()));
        if (!se.empty()) d->send_ent.upload(se.data(), se.size(), d->stream);
        d->recv_ent.alloc(std::max<size_t>(1, re.size()));
        if (!re.empty()) d->recv_ent.upload(re.data(), re.size(), d->stream);
        int32_t nmo = 0;
        for (const DdPart &Q : d->plan.parts) nmo = std::max(nmo, Q.n_own);
        d->nmax_own = nmo;
        std::vector<int32_t> all((size_t)P * nmo, -1);
        for (int32_t q = 0; q < P; ++q)
            for (int32_t i = 0; i < d->plan.parts[q].n_own; ++i) all[(size_t)q * nmo + i] = d->plan.parts[q].l2g[i];
        d->all_l2g.alloc(all.size());
        d->all_l2g.upload(all.data(), all.size(), d->stream);
        d->agree.alloc((size_t)P);
    }
    MOF_HIP(hipStreamSynchronize(d->stream));
    d->ms_setup = dd_now_ms() - t0;
}

void dd_free(mof_dd *d) {
    if (!d) return;
    {
        DevGuard g(d->device);
        if (d->stream) (void)hipStreamSynchronize(d->stream);
        for (mof_mesh *m : d->parts) mof_mesh_destroy(m);
        d->parts.clear();
        if (d->comm && d->nccl) (void)d->nccl->comm_destroy(static_cast<ncclComm_t>(d->comm));
        d->comm = nullptr;
        if (d->stream) (void)hipStreamDestroy(d->stream);
        d->stream = nullptr;
        delete d;
    }
}

void check_mesh_args(const double *xyz, const double *nrm, const int32_t *tri, const double *area, int32_t N,
                     int32_t M, int32_t nparts, const int32_t *part) {
    MOF_REQUIRE(xyz && nrm && tri && area, "NULL input array");
    MOF_REQUIRE(N > 0 && M > 0, "mesh needs N > 0 vertices and M > 0 triangles");
    MOF_REQUIRE(nparts >= 1 && nparts <= N, "need 1 <= nparts <= N");
    for (int64_t q = 0; q < 3 * (int64_t)M; ++q)
        MOF_REQUIRE(tri[q] >= 0 && tri[q] < N, "triangle vertex index out of range");
    if (part)
        for (int32_t i = 0; i < N; ++i) MOF_REQUIRE(part[i] >= 0 && part[i] < nparts, "part id out of range");
}

}  // namespace

extern "C" {

int mof_partition_rcb(const double *xyz, int32_t N, int32_t nparts, int32_t *part) {
    return mof_io_guard([&] {
        MOF_REQUIRE(xyz && part, "NULL argument");
        mof::partition_rcb(xyz, N, nparts, part);
    });
}

int mof_dd_plan_info(const int32_t *tri, int32_t N, int32_t M, int32_t nparts, const int32_t *part,
                     int32_t *n_own, int32_t *n_ghost, int32_t *n_nbr, int32_t *n_tri, int64_t *n_send) {
    return mof_io_guard([&] {
        MOF_REQUIRE(tri && part && n_own && n_ghost && n_nbr && n_tri && n_send, "NULL argument");
        MOF_REQUIRE(N > 0 && M > 0 && nparts >= 1, "bad sizes");
        for (int64_t q = 0; q < 3 * (int64_t)M; ++q)
            MOF_REQUIRE(tri[q] >= 0 && tri[q] < N, "triangle vertex index out of range");
        mof::DdPlan plan;
        mof::build_dd_plan(tri, N, M, nparts, part, nullptr, plan);
        for (int32_t p = 0; p < nparts; ++p) {
            const mof::DdPart &D = plan.parts[p];
            n_own[p] = D.n_own;
            n_ghost[p] = D.n_ghost;
            n_nbr[p] = (int32_t)D.nbr.size();
            n_tri[p] = (int32_t)D.tris.size();
            n_send[p] = (int64_t)D.send_idx.size();
        }
    });
}

int mof_dd_create(const double *xyz, const double *nrm, const int32_t *tri, const double *area, int32_t N,
                  int32_t M, int32_t nparts, const int32_t *part, int32_t device, uint32_t flags, mof_dd **out) {
    return mof_io_guard([&] {
        MOF_REQUIRE(out, "out is NULL");
        *out = nullptr;
        check_mesh_args(xyz, nrm, tri, area, N, M, nparts, part);
        int ndev = 0;
        MOF_HIP(hipGetDeviceCount(&ndev));
        MOF_REQUIRE(device >= 0 && device < ndev, "device ordinal out of range");
        DevGuard g(device);
        auto *d = new mof_dd();
        d->N = N;
        d->M = M;
        d->P = nparts;
        d->device = device;
        d->flags = flags;
        try {
            dd_setup(d, xyz, nrm, tri, area, part);
        } catch (...) {
            dd_free(d);
            throw;
        }
        *out = d;
    });
}

int mof_dd_unique_id(uint8_t *id) {
    return mof_io_guard([&] {
        MOF_REQUIRE(id, "NULL argument");
        mof::RcclApi *a = mof::rccl_open();
        ncclUniqueId u;
        mof::nccl_check(a, a->get_unique_id(&u), "ncclGetUniqueId");
        std::memcpy(id, u.internal, MOF_DD_ID_BYTES);
    });
}

int mof_dd_create_rank(const double *xyz, const double *nrm, const int32_t *tri, const double *area, int32_t N,
                       int32_t M, int32_t nranks, const int32_t *part, int32_t rank, const uint8_t *id,
                       int32_t device, uint32_t flags, mof_dd **out) {
    return mof_io_guard([&] {
        MOF_REQUIRE(out && id, "NULL argument");
        *out = nullptr;
        check_mesh_args(xyz, nrm, tri, area, N, M, nranks, part);
        MOF_REQUIRE(rank >= 0 && rank < nranks, "rank out of range");
        int ndev = 0;
        MOF_HIP(hipGetDeviceCount(&ndev));
        MOF_REQUIRE(device >= 0 && device < ndev, "device ordinal out of range");
        DevGuard g(device);
        auto *d = new mof_dd();
        d->N = N;
        d->M = M;
        d->P = nranks;
        d->device = device;
        d->flags = flags;
        d->rank = rank;
        try {
            d->nccl = mof::rccl_open();
            ncclUniqueId u;
            std::memcpy(u.internal, id, sizeof(u.internal));
            ncclComm_t comm = nullptr;
            mof::nccl_check(d->nccl, d->nccl->comm_init_rank(&comm, nranks, u, rank), "ncclCommInitRank");
            d->comm = comm;
            dd_setup(d, xyz, nrm, tri, area, part);
        } catch (...) {
            dd_free(d);
            throw;
        }
        *out = d;
    });
}

int mof_dd_create_rank_host(const double *xyz, const double *nrm, const int32_t *tri, const double *area,
                            int32_t N, int32_t M, int32_t nranks, const int32_t *part, int32_t rank,
                            const mof_dd_transport *transport, int32_t device, uint32_t flags, mof_dd **out) {
    return mof_io_guard([&] {
        MOF_REQUIRE(out && transport && transport->allgather && transport->exchange, "NULL argument");
        *out = nullptr;
        check_mesh_args(xyz, nrm, tri, area, N, M, nranks, part);
        MOF_REQUIRE(rank >= 0 && rank < nranks, "rank out of range");
        int ndev = 0;
        MOF_HIP(hipGetDeviceCount(&ndev));
        MOF_REQUIRE(device >= 0 && device < ndev, "device ordinal out of range");
        DevGuard g(device);
        auto *d = new mof_dd();
        d->N = N;
        d->M = M;
        d->P = nranks;
        d->device = device;
        d->flags = flags;
        d->rank = rank;
        d->hosted = true;
        d->host = *transport;
        try {
            dd_setup(d, xyz, nrm, tri, area, part);
        } catch (...) {
            dd_free(d);
            throw;
        }
        *out = d;
    });
}

int mof_dd_destroy(mof_dd *d) {
    return mof_io_guard([&] { dd_free(d); });
}

int mof_dd_test_fail_recovery_alloc(mof_dd *d, int32_t rank) {
    return mof_io_guard([&] {
        MOF_REQUIRE(d, "NULL argument");
        d->test_oom_rank = rank;
    });
}

int mof_dd_get_info(const mof_dd *d, mof_dd_info *info) {
    return mof_io_guard([&] {
        MOF_REQUIRE(d && info, "NULL argument");
        std::memset(info, 0, sizeof(*info));
        info->nparts = d->P;
        info->local_parts = (int32_t)d->parts.size();
        info->rank = d->rank;
        for (const mof::DdPart &D : d->plan.parts) {
            info->ghost_rows += D.n_ghost;
            info->send_rows += (int64_t)D.send_idx.size();
            info->max_neighbours = std::max(info->max_neighbours, (int32_t)D.nbr.size());
            info->max_owned = std::max(info->max_owned, D.n_own);
        }
        info->ms_setup = d->ms_setup;
    });
}

int mof_dd_solve_range(mof_dd *d, const double *I, const double *I2, const double *t_k, int32_t T, int32_t k0,
                       int32_t k1, double lambda, const mof_opts *opts, double *V_out, mof_stats *stats) {
    return mof_io_guard([&] {
        using namespace mof;
        MOF_REQUIRE(d && I && t_k && V_out, "NULL argument");
        MOF_REQUIRE(T >= 1 && k0 >= 0 && k0 <= k1 && k1 <= T - 1, "need 0 <= k0 <= k1 <= T-1");
        mof_opts o{};
        if (opts) {
            MOF_REQUIRE(opts->struct_size == 0 || opts->struct_size >= sizeof(mof_opts),
                        "mof_opts.struct_size too small");
            o = *opts;
        }
        MOF_REQUIRE(o.precision == MOF_PREC_F64 || o.precision == MOF_PREC_MIXED, "unknown precision");
        SolveParams sp;
        sp.precision = o.precision;
        sp.amg = (o.flags & MOF_PRECOND_AMG) != 0;
        MOF_REQUIRE(!sp.amg || o.precision == MOF_PREC_MIXED, "MOF_PRECOND_AMG needs MOF_PREC_MIXED");
        sp.block_jacobi = sp.amg || !(o.flags & MOF_NO_BLOCK_JACOBI);
        sp.time_spmv = false;
        // the single-domain defaults (mof_solve_range): a multigrid inner
        // solve takes tens of iterations, so 1000 and a stagnation window
        // mark a bad preconditioner, and the system goes to the recovery
        sp.max_iter = o.max_iter > 0 ? o.max_iter : (sp.amg ? 1000 : 10000);
        sp.max_outer = o.max_outer > 0 ? o.max_outer : 10;
        sp.rtol = o.rtol > 0 ? o.rtol : 1e-8;
        sp.inner_rtol = o.inner_rtol > 0 ? o.inner_rtol : 1e-4;
        // error control: etol 0 -> 1e-7 of max|V|, < 0 -> off
        sp.etol = o.etol > 0 ? o.etol : (o.etol < 0 ? 0.0 : 1e-7);
        sp.stall = sp.amg ? kPcgStall : 0;
        sp.fail_at_max_iter = sp.amg;
        const bool recovery = !(o.flags & MOF_NO_RECOVERY);
        const bool dev_io = (o.flags & MOF_IO_DEVICE) != 0;
        if (!I2) I2 = I;
        DevGuard g(d->device);
        hipStream_t s = o.stream ? (hipStream_t)o.stream : d->stream;
        const int32_t K = k1 - k0;
        const int64_t N = d->N;
        mof_stats st{};
        if (K > 0) {
            int32_t Bmax = o.batch;
            if (Bmax <= 0) {
                size_t free_b = 0, total_b = 0;
                MOF_HIP(hipMemGetInfo(&free_b, &total_b));
                const double per_sys = 620.0 * (double)N * (d->rank < 0 ? 1.0 : 1.0 / d->P) + 1.0;
                Bmax = (int32_t)std::max(1.0, std::min(64.0, 0.25 * (double)free_b / per_sys));
            }
            // every launch grid within 2^32 work-items (xcd_grid), checked for
            // the largest of this rank's parts and agreed over the ranks, so
            // that no rank refuses a launch the others go on past
            int32_t cap = 1 << 30;
            for (mof_mesh *m : d->parts) cap = std::min(cap, grid_batch_cap(m));
            cap = (int32_t)dd_all_min(d, (double)cap, d->stream);
            const int32_t B = std::min(K, std::min(Bmax, cap));
            dd_ensure(d, B, sp.precision);
            DevArray<double> Ibuf, Vbuf;
            if (!dev_io) {
                Ibuf.alloc(2 * (size_t)N * B);
                Vbuf.alloc(2 * (size_t)N * B);
            }
            for (mof_mesh *m : d->parts) prepare_operator(m, lambda, s);
            // subdomain multigrid (every part, or none): built before the first
            // assembly, which writes the level-0 smoother copies
            bool amg = sp.amg;
            for (mof_mesh *m : d->parts) amg = amg && amg_build(m);
            if (amg)
                for (mof_mesh *m : d->parts) amg_ensure(m, B);
            hipEvent_t ev[3];
            for (auto &e : ev) MOF_HIP(hipEventCreate(&e));
            std::vector<double> dts(B);
            std::vector<uint8_t> only(B);
            try {
                for (int32_t k = k0; k < k1; k += B) {
                    const int32_t nb = std::min(B, k1 - k);
                    for (int32_t b = 0; b < nb; ++b) dts[b] = t_k[k + b + 1] - t_k[k + b];
                    for (mof_mesh *m : d->parts)
                        MOF_HIP(hipMemcpyAsync(m->ws.dt.p, dts.data(), sizeof(double) * nb, hipMemcpyHostToDevice, s));
                    const double *I0p, *I1p;
                    if (dev_io) {
                        I0p = I + (int64_t)k * N;
                        I1p = I2 + (int64_t)(k + 1) * N;
                    } else {
                        MOF_HIP(hipMemcpyAsync(Ibuf.p, I + (int64_t)k * N, sizeof(double) * N * nb,
                                               hipMemcpyHostToDevice, s));
                        MOF_HIP(hipMemcpyAsync(Ibuf.p + N * B, I2 + (int64_t)(k + 1) * N, sizeof(double) * N * nb,
                                               hipMemcpyHostToDevice, s));
                        I0p = Ibuf.p;
                        I1p = Ibuf.p + N * B;
                    }
                    MOF_HIP(hipEventRecord(ev[0], s));
                    for (mof_mesh *m : d->parts)
                        launch_assemble(m, nb, I0p, I1p, N, sp.block_jacobi, sp.precision, s, amg);
                    MOF_HIP(hipEventRecord(ev[1], s));
                    int32_t outer = 0;
                    st.iterations += solve_batch_dd(d, nb, sp, s, &outer, &st.max_iterations);
                    st.outer_steps = outer;
                    // failed systems re-solved alone, as in mof_solve_range
                    // (every part / rank sees the same flags)
                    if (recovery)
                        recover_systems(
                            nb, sp, o.max_iter, d->parts[0]->h_sysi, only, st,
                            [&](uint32_t prec) {
                                // a workspace allocation can fail on one rank
                                // only: every rank learns of it before the
                                // pass's collectives, and all skip the pass
                                // (its systems stay failed, NaN-filled)
                                bool ok = true;
                                Error err{MOF_E_HIP, ""};
                                try {
                                    dd_ensure(d, nb, prec);
                                } catch (const Error &e) {
                                    if (e.code != MOF_E_HIP) throw;
                                    (void)hipGetLastError();
                                    ok = false;
                                    err = e;
                                }
                                if (d->rank >= 0 && d->test_oom_rank == d->rank && prec == MOF_PREC_F64) {
                                    ok = false;  // test hook (mof_dd_test_fail_recovery_alloc): this rank's fp64 workspace "fails"
                                    err = Error{MOF_E_HIP, "injected allocation failure"};
                                }
                                if (!dd_all_ok(d, ok, s))
                                    throw ok ? Error{MOF_E_HIP, "workspace allocation failed on another rank"} : err;
                                for (mof_mesh *m : d->parts) launch_recovery_operator(m, nb, prec, s);
                            },
                            [&](const SolveParams &rp, const uint8_t *on) {
                                int32_t outer_r = 0;
                                return solve_batch_dd(d, nb, rp, s, &outer_r, &st.max_iterations, on);
                            },
                            [&] {
                                for (mof_mesh *m : d->parts) release_f64_terms(m);
                            });
                    double *Vdst = dev_io ? V_out + (int64_t)(k - k0) * 2 * N : Vbuf.p;
                    dd_gather_v(d, nb, Vdst, s);
                    MOF_HIP(hipEventRecord(ev[2], s));
                    if (!dev_io)
                        MOF_HIP(hipMemcpyAsync(V_out + (int64_t)(k - k0) * 2 * N, Vbuf.p, sizeof(double) * 2 * N * nb,
                                               hipMemcpyDeviceToHost, s));
                    MOF_HIP(hipStreamSynchronize(s));
                    float a = 0.f, b2 = 0.f;
                    (void)hipEventElapsedTime(&a, ev[0], ev[1]);
                    (void)hipEventElapsedTime(&b2, ev[1], ev[2]);
                    st.ms_assembly += a;
                    st.ms_solve += b2;
                    const mof_mesh *m0 = d->parts[0];
                    for (int32_t b = 0; b < nb; ++b) {
                        if (m0->h_sysi[b * kSysStride + SI_FAILED]) st.failed++;
                        st.max_rel_residual = std::max(st.max_rel_residual, m0->h_sysd[b * kSysStride + SD_REL]);
                        const double xm = m0->h_sysd[b * kSysStride + SD_XMAX];
                        if (xm > 0.0) st.max_err_est = std::max(st.max_err_est, m0->h_sysd[b * kSysStride + SD_EST] / xm);
                    }
                    st.batches++;
                }
            } catch (...) {
                for (auto &e : ev) (void)hipEventDestroy(e);
                throw;
            }
            for (auto &e : ev) (void)hipEventDestroy(e);
        }
        st.systems = K;
        if (stats) *stats = st;
        if (st.failed)
            throw Error{MOF_E_NOCONV, std::to_string(st.failed) + " system(s) did not converge; their V is NaN-filled"};
    });
}

}  // extern "C"
