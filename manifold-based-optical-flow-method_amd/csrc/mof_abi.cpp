// mof_abi.cpp -- extern "C" entry points of libmofhip.so (include/mof.h).
//
// Host orchestration only: argument checks, device uploads, batching of
// timesteps, and result copies. All arithmetic runs in the HIP kernels of
// mof_assemble.hip / mof_pcg.hip / mof_amg.hip / mof_sing.hip (the CSV and
// PLY entry points are host code: mof_io.cpp, mof_ply.cpp).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <future>
#include <memory>
#include <mutex>
#include <new>

#include "mof_amg.h"
#include "mof_dd.h"
#include "mof_hostio.h"
#include "mof_internal.h"

namespace {

thread_local std::string g_err;

template <class F>
int guarded(F &&f) {
    try {
        f();
        return MOF_OK;
    } catch (const mof::Error &e) {
        g_err = e.msg;
        return e.code;
    } catch (const std::bad_alloc &) {
        g_err = "host allocation failed";
        return MOF_E_HIP;
    } catch (const std::exception &e) {
        g_err = e.what();
        return MOF_E_ARG;
    }
}

struct DeviceGuard {
    int prev = 0;
    explicit DeviceGuard(int d) {
        (void)hipGetDevice(&prev);
        MOF_HIP(hipSetDevice(d));
    }
    ~DeviceGuard() { (void)hipSetDevice(prev); }
};

struct Events {
    hipEvent_t e[3] = {nullptr, nullptr, nullptr};
    Events() {
        for (auto &x : e) MOF_HIP(hipEventCreate(&x));
    }
    ~Events() {
        for (auto &x : e)
            if (x) (void)hipEventDestroy(x);
    }
    float ms(int a, int b) const {
        float v = 0.f;
        (void)hipEventElapsedTime(&v, e[a], e[b]);
        return v;
    }
};

double now_ms() {
    using namespace std::chrono;
    return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

// SELL block layout (internal order) -> canonical scalar CSR (2N x 2N) in
// the caller's vertex order.
void sell_to_csr(const mof_mesh *m, const std::vector<double> &blk, int32_t drop_zeros,
                 int32_t *indptr, int32_t *indices, double *data, int64_t *nnz_out) {
    const mof::Pattern &P = m->pat;
    const int32_t N = m->N;
    int64_t nnz = 0;
    indptr[0] = 0;
    std::vector<std::pair<int32_t, int64_t>> row;  // (caller column vertex, SELL pos)
    for (int32_t r = 0; r < 2 * N; ++r) {
        const int32_t io = r % N, al = r / N;
        const int32_t i = m->perm[io];
        row.clear();
        const int32_t td = (int32_t)(std::lower_bound(P.vcol.begin() + P.vptr[i], P.vcol.begin() + P.vptr[i + 1], i) -
                                     (P.vcol.begin() + P.vptr[i]));
        for (int32_t p = P.vptr[i], t = 0; p < P.vptr[i + 1]; ++p, ++t)
            row.emplace_back(m->inv[P.vcol[p]],
                             (int64_t)P.sell_off[i >> 6] + (int64_t)mof::sell_slot(t, td) * mof::kSlice + (i & 63));
        std::sort(row.begin(), row.end());
        for (int half = 0; half < 2; ++half) {  // columns j, then j + N
            for (const auto &cp : row) {
                const double v = blk[4 * cp.second + 2 * al + half];
                if (drop_zeros && v == 0.0) continue;
                indices[nnz] = cp.first + half * N;
                data[nnz] = v;
                ++nnz;
            }
        }
        indptr[r + 1] = (int32_t)nnz;
    }
    *nnz_out = nnz;
}

// Pinned ring, copy stream and the two device slots of a host-pointer solve
// (mof_hostio.h); kept on the handle across calls.
// The ring's chunk follows the job: a quarter of the larger per-batch
// transfer in whole MiB, at most stage_cap() (32): pinning the 4 x 32 MiB
// ring took tens of ms -- longer than a 3k-vertex, 97-timestep job's whole
// solve. A later, larger job replaces the stage. direct: only the device
// slots (the batches' copies run on the compute stream, solve_batches).
// MOF_STAGE_MB (MiB, default 32): the ring's largest chunk
size_t stage_cap() { return (size_t)std::max(1, mof::knob_int(mof::Knob::StageMB, 32)) << 20; }

void host_io_prepare(mof_mesh *m, int64_t in_elems, int64_t out_elems, bool direct) {
    const size_t mib = (size_t)1 << 20, cap = stage_cap();
    const size_t larger = (size_t)std::max(in_elems, out_elems) * sizeof(double);
    const size_t want = std::min(cap, (larger / 4 + mib - 1) / mib * mib);
    if (!direct && m->stage && m->stage->chunk() < want) {
        delete m->stage;  // synchronises its copy stream
        m->stage = nullptr;
    }
    if (!direct && !m->stage) {
        // copy threads: one per MiB of a chunk, at most stage_threads()
        m->stage = new mof::HostStage(want, std::max<int32_t>(1, std::min<int32_t>(mof::stage_threads(), (int32_t)(want / mib))));
        for (auto &e : m->hev) {
            if (!e) MOF_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            MOF_HIP(hipEventRecord(e, m->stage->stream()));  // every wait has a recorded event
        }
    }
    for (int sl = 0; sl < 2; ++sl) {
        if ((int64_t)m->hin[sl].n < in_elems) m->hin[sl].alloc(in_elems);
        if ((int64_t)m->hout[sl].n < out_elems) m->hout[sl].alloc(out_elems);
    }
}

// The batches of mof_solve_range's range [k0, k1) (batch j = timesteps
// k0 + j B ...), each assembled, solved, recovered and written as planar V
// on stream s. Host pointers: the handle's double-buffered copy pipeline
// (mof_hostio.h). Measured and not kept (round 4,
// profiles/r04_ab/call1*/c3_l2_*, c3_b256_l2): two batches in flight on one
// GPU (the batches alternating between the handle and a same-device twin on
// their own streams and host threads) -- 3533 vs 3602 timesteps/s at B = 512
// and 3419 vs 3463 at B = 256: the latency-bound setup kernels beside the
// other batch's bandwidth-bound sweeps slow both.
void solve_batches(mof_mesh *m, const double *I, const double *I2, const double *t_k, int32_t k0, int32_t k1,
                   int32_t B, double lambda, const mof::SolveParams &sp_in, const mof_opts &o, bool recovery,
                   bool dev_io, hipStream_t s, double *V_out, mof_stats &st, mof::SpmvTiming &timing) {
    mof::SolveParams sp = sp_in;
    const int32_t K = k1 - k0;
    // MOF_VERBOSE: helper-thread and wait times, and the call's setup steps,
    // on stderr
    const bool hostio_verbose = mof::knob(mof::Knob::Verbose) != nullptr;
    double tp[5];
    tp[0] = now_ms();
    mof::ensure_workspace(m, B, sp.precision);
    mof::Workspace &w = m->ws;
    const int64_t N = m->N;
    Events ev;
    mof::prepare_operator(m, lambda, s);
    tp[1] = now_ms();
    // multigrid hierarchy before the first assembly (which writes the
    // level-0 smoother's bf16 copies)
    const bool amg = sp.amg && sp.precision == MOF_PREC_MIXED && mof::amg_build(m);
    tp[2] = now_ms();
    if (amg) mof::amg_ensure(m, B);
    // large irregular or open meshes (the smoothed-prolongator hierarchies):
    // the first refinement step's inner solve to 1e-5 instead of 1e-4
    // (unless the caller set one) -- it leaves the second step with the outer
    // target in reach, so a third step (and its fp64 residual) is rarely
    // needed: S1 857 -> 889, R3 702 -> 717 timesteps/s; on the regular meshes
    // the deeper first step only adds iterations (C3 17.0 -> 18.0 its, -5 %;
    // profiles/r04_ab/call10/), and on a small one (S1s, 3,249 vertices,
    // 30137 -> 28329) a third step costs less than the extra iterations
    if (amg && o.inner_rtol <= 0 && !mof::amg_fine(m).regular && m->N >= 16384) sp.inner_rtol = 1e-5;
    tp[3] = now_ms();
    // host pointers: one upload of the nb+1 rows when I2 is I (S3
    // passes I_k twice), else nb rows of each
    const bool shared_I = (I2 == I);
    const int64_t in_rows = shared_I ? B + 1 : 2 * (int64_t)B;
    // host transfers of at most 16 MiB per batch (half the ring's chunk cap
    // when MOF_STAGE_MB sets it lower): straight pageable copies on the
    // compute stream (the runtime stages them), no copy stream, helper thread
    // or pinned ring -- creating those cost a small job 4-12 ms, more than its
    // solve (S1s: 3.8 ms)
    const bool direct = !dev_io && (size_t)std::max(in_rows, 2 * (int64_t)B) * N * sizeof(double) <=
                                       std::min<size_t>((size_t)16 << 20, stage_cap() / 2);
    if (!dev_io) host_io_prepare(m, in_rows * N, 2 * N * B, direct);
    tp[4] = now_ms();
    if (hostio_verbose)
        fprintf(stderr, "[mof setup] workspace + operator %.2f ms, hierarchy %.2f ms, its storage %.2f ms, host staging %.2f ms\n",
                tp[1] - tp[0], tp[2] - tp[1], tp[3] - tp[2], tp[4] - tp[3]);
    // batch starts: B timesteps each; a host-pointer job of more than two
    // batches starts and ends with a quarter batch, so the pipeline's fill
    // (the first batch's I rows) and drain (the last batch's V) are short
    // -- V does not depend on the split (round 6: C3's host-to-host rate
    // over 4 batches, profiles/r06/taper/)
    std::vector<int32_t> kst{k0};
    if (!dev_io && !direct && K > 2 * B) {
        const int32_t sm = std::max(1, B / 4);
        int32_t k = k0 + sm;
        kst.push_back(k);
        while (k1 - k > B + sm) kst.push_back(k += B);
        if (k1 - k > sm) kst.push_back(k1 - sm);
    } else {
        for (int32_t k = k0 + B; k < k1; k += B) kst.push_back(k);
    }
    kst.push_back(k1);
    const int32_t nbat = (int32_t)kst.size() - 1;
    auto bk = [&](int32_t q) { return kst[q]; };
    auto bn = [&](int32_t q) { return kst[q + 1] - kst[q]; };
    // helper-thread steps of the host pipeline (copy stream): batch q's I rows
    // into slot q&1 once batch q-2's assembly has read it, and batch q's V
    // out of slot q&1 into V_out
    double t_in = 0.0, t_out = 0.0, t_wait = 0.0;
    const double t_call = now_ms();
    mof::g_fetch_ms = 0.0;
    mof::g_fetch_n = 0;
    auto stage_in = [&](int32_t q) {
        const double t0 = now_ms();
        struct Acc {
            double &t, t0;
            ~Acc() { t += now_ms() - t0; }
        } acc{t_in, t0};
        MOF_HIP(hipSetDevice(m->device));
        const int32_t sl = q & 1, kj = bk(q), nb = bn(q);
        hipStream_t cs = m->stage->stream();
        MOF_HIP(hipStreamWaitEvent(cs, m->hev[2 + sl], 0));
        if (shared_I) {
            m->stage->h2d(m->hin[sl].p, I + (int64_t)kj * N, sizeof(double) * N * (nb + 1));
        } else {
            m->stage->h2d(m->hin[sl].p, I + (int64_t)kj * N, sizeof(double) * N * nb);
            m->stage->h2d(m->hin[sl].p + N * B, I2 + (int64_t)(kj + 1) * N, sizeof(double) * N * nb);
        }
        MOF_HIP(hipEventRecord(m->hev[sl], cs));
    };
    auto drain_out = [&](int32_t q) {
        struct Acc {
            double &t, t0;
            ~Acc() { t += now_ms() - t0; }
        } acc{t_out, now_ms()};
        MOF_HIP(hipSetDevice(m->device));
        const int32_t sl = q & 1;
        m->stage->d2h(V_out + (int64_t)(bk(q) - k0) * 2 * N, m->hout[sl].p, sizeof(double) * 2 * N * bn(q),
                      m->hev[4 + sl]);
    };
    std::vector<double> dts(B);
    std::vector<uint8_t> only(B);
    // declared after everything its tasks reference: its destructor
    // waits for a task still running when an error unwinds
    std::future<void> io;
    if (!dev_io && !direct) io = std::async(std::launch::async, [&] { stage_in(0); });
    for (int32_t q = 0; q < nbat; ++q) {
        const int32_t k = bk(q), nb = bn(q), sl = q & 1;
        for (int32_t b = 0; b < nb; ++b) dts[b] = t_k[k + b + 1] - t_k[k + b];
        MOF_HIP(hipMemcpyAsync(w.dt.p, dts.data(), sizeof(double) * nb, hipMemcpyHostToDevice, s));
        const double *I0p, *I1p;
        if (dev_io) {
            I0p = I + (int64_t)k * N;
            I1p = I2 + (int64_t)(k + 1) * N;
        } else if (direct) {
            double *hin = m->hin[0].p;
            if (shared_I) {
                MOF_HIP(hipMemcpyAsync(hin, I + (int64_t)k * N, sizeof(double) * N * (nb + 1), hipMemcpyHostToDevice, s));
            } else {
                MOF_HIP(hipMemcpyAsync(hin, I + (int64_t)k * N, sizeof(double) * N * nb, hipMemcpyHostToDevice, s));
                MOF_HIP(hipMemcpyAsync(hin + N * B, I2 + (int64_t)(k + 1) * N, sizeof(double) * N * nb,
                                       hipMemcpyHostToDevice, s));
            }
            I0p = hin;
            I1p = shared_I ? I0p + N : I0p + N * B;
        } else {
            const double tw = now_ms();
            io.get();  // batch q staged, batch q-1 drained
            t_wait += now_ms() - tw;
            if (q + 1 < nbat || q > 0)
                io = std::async(std::launch::async, [&, q] {
                    if (q + 1 < nbat) stage_in(q + 1);
                    if (q > 0) drain_out(q - 1);
                });
            MOF_HIP(hipStreamWaitEvent(s, m->hev[sl], 0));
            I0p = m->hin[sl].p;
            I1p = shared_I ? I0p + N : I0p + N * B;
        }
        MOF_HIP(hipEventRecord(ev.e[0], s));
        mof::launch_assemble(m, nb, I0p, I1p, N, sp.block_jacobi, sp.precision, s, amg);
        if (!dev_io && !direct) MOF_HIP(hipEventRecord(m->hev[2 + sl], s));
        MOF_HIP(hipEventRecord(ev.e[1], s));
        int32_t outer = 0;
        st.iterations += mof::solve_batch(m, nb, sp, s, &outer, &st.max_iterations, &timing);
        st.outer_steps = outer;
        if (recovery)
            mof::recover_systems(
                nb, sp, o.max_iter, m->h_sysi, only, st,
                [&](uint32_t prec) {
                    mof::ensure_workspace(m, nb, prec);
                    mof::launch_recovery_operator(m, nb, prec, s);
                },
                [&](const mof::SolveParams &rp, const uint8_t *on) {
                    int32_t outer_r = 0;
                    return mof::solve_batch(m, nb, rp, s, &outer_r, &st.max_iterations, nullptr, on);
                },
                [&] { mof::release_f64_terms(m); });
        double *Vdst = dev_io ? V_out + (int64_t)(k - k0) * 2 * N : m->hout[direct ? 0 : sl].p;
        mof::launch_to_planar(m, nb, Vdst, s);
        if (direct)
            MOF_HIP(hipMemcpyAsync(V_out + (int64_t)(k - k0) * 2 * N, Vdst, sizeof(double) * 2 * N * nb,
                                   hipMemcpyDeviceToHost, s));
        else if (!dev_io)
            MOF_HIP(hipEventRecord(m->hev[4 + sl], s));
        MOF_HIP(hipEventRecord(ev.e[2], s));
        MOF_HIP(hipEventSynchronize(ev.e[2]));
        st.ms_assembly += ev.ms(0, 1);
        st.ms_solve += ev.ms(1, 2);
        for (int32_t b = 0; b < nb; ++b) {
            if (m->h_sysi[b * mof::kSysStride + mof::SI_FAILED]) st.failed++;
            st.max_rel_residual = std::max(st.max_rel_residual, m->h_sysd[b * mof::kSysStride + mof::SD_REL]);
            const double xm = m->h_sysd[b * mof::kSysStride + mof::SD_XMAX];
            if (xm > 0.0) st.max_err_est = std::max(st.max_err_est, m->h_sysd[b * mof::kSysStride + mof::SD_EST] / xm);
        }
        st.batches++;
    }
    if ((dev_io || direct) && hostio_verbose)
        fprintf(stderr, "[mof hostio] %s K=%d B=%d: call %.1f ms, %lld flag fetches %.1f ms\n",
                dev_io ? "device" : "direct", K, B, now_ms() - t_call, (long long)mof::g_fetch_n, mof::g_fetch_ms);
    if (!dev_io && !direct) {
        if (io.valid()) io.get();
        drain_out(nbat - 1);
        if (hostio_verbose)
            fprintf(stderr,
                    "[mof hostio] K=%d B=%d: stage_in %.1f ms, drain %.1f ms, main waited %.1f ms, "
                    "call %.1f ms, %lld flag fetches %.1f ms\n",
                    K, B, t_in, t_out, t_wait, now_ms() - t_call, (long long)mof::g_fetch_n, mof::g_fetch_ms);
    }
}

}  // namespace

namespace mof {

// the fine-level smoother damping of the recovery's multigrid pass
constexpr float kRecoverOmega = 0.6f;

// Systems of the batch whose solve failed are re-solved alone: with the
// multigrid at a smaller fine-level damping (after a multigrid solve), 2x2
// block-Jacobi PCG in the same precision after a multigrid solve, then in
// fp64 (no stagnation test, the full iteration budget); only what all of
// them fail stays failed (NaN-filled by k_to_planar). An fp64 solve gets
// one fp64 block-Jacobi pass when its first solve ran without block Jacobi
// or with a smaller budget (else the same solve would only repeat). An fp64
// pass whose A64 workspace cannot be allocated leaves its systems failed
// (NaN-filled, reported) instead of failing the whole call; after a mixed
// solve the A64 it allocated is released again. Shared by the single-domain
// and the decomposed paths: `ensure` sizes the workspace of a pass, `solve`
// runs it on the `only` systems, `sysi` is the host flag mirror.
void recover_systems(int32_t nb, const SolveParams &sp, int32_t user_max_iter, const int32_t *sysi,
                     std::vector<uint8_t> &only, mof_stats &st, const std::function<void(uint32_t)> &ensure,
                     const std::function<int64_t(const SolveParams &, const uint8_t *)> &solve,
                     const std::function<void()> &release_f64) {
    auto failed = [&](int32_t b) { return sysi[b * kSysStride + SI_FAILED] != 0; };
    const int32_t budget = std::max(user_max_iter, 10000);  // the full budget, never less than the caller's
    // passes: {precision, multigrid}; after a multigrid solve first the same
    // multigrid with a more strongly damped fine smoother (kRecoverOmega): a
    // V-cycle whose damped block Jacobi is not contractive on a system (an
    // indefinite preconditioner: breakdown after a few iterations -- round 4,
    // the S1-like patch under an atan2 pinwheel signal, every system at
    // omega 0.85, none at 0.7) converges in tens of iterations there, where
    // block Jacobi takes hundreds
    struct Pass {
        uint32_t prec;
        bool amg;
    };
    std::vector<Pass> passes;
    if (sp.precision == MOF_PREC_MIXED && sp.amg) {
        passes.push_back({MOF_PREC_MIXED, true});
        passes.push_back({MOF_PREC_MIXED, false});
    }
    if (sp.precision == MOF_PREC_MIXED || !sp.block_jacobi || sp.max_iter < budget)
        passes.push_back({MOF_PREC_F64, false});
    std::vector<uint8_t> first(nb, 0);
    int32_t nfirst = 0;
    for (int32_t b = 0; b < nb; ++b) nfirst += (first[b] = failed(b));
    if (!nfirst) return;
    // MOF_VERBOSE: why and when the first solve's failed systems failed
    if (knob(Knob::Verbose)) {
        int32_t why[8] = {0}, itmin = 1 << 30, itmax = 0;
        for (int32_t b = 0; b < nb; ++b)
            if (first[b]) {
                why[std::min(7, std::max(0, sysi[b * kSysStride + SI_FAIL_WHY]))]++;
                itmin = std::min(itmin, sysi[b * kSysStride + SI_FAIL_IT]);
                itmax = std::max(itmax, sysi[b * kSysStride + SI_FAIL_IT]);
            }
        std::fprintf(stderr,
                     "[mof recover] %d of %d failed: breakdown %d diverged %d stalled %d max_iter %d residual %d; "
                     "at inner iteration %d..%d\n",
                     nfirst, nb, why[FW_BREAKDOWN], why[FW_DIVERGED], why[FW_STALLED], why[FW_MAXITER],
                     why[FW_RESIDUAL], itmin, itmax);
    }
    bool used_f64 = false;
    for (const Pass &ps : passes) {
        const uint32_t prec = ps.prec;
        int32_t n = 0;
        for (int32_t b = 0; b < nb; ++b) n += (only[b] = failed(b));
        if (!n) break;
        SolveParams rp = sp;
        rp.precision = prec;
        rp.amg = ps.amg;
        rp.block_jacobi = true;
        rp.time_spmv = false;
        if (ps.amg) {  // the first solve's limits (stagnation, max_iter) stand
            rp.amg_omega = kRecoverOmega;
        } else {
            rp.stall = 0;
            rp.fail_at_max_iter = false;
            rp.max_iter = budget;
        }
        if (prec == MOF_PREC_F64 && sp.precision == MOF_PREC_MIXED) {
            try {
                ensure(prec);
            } catch (const Error &e) {
                if (e.code != MOF_E_HIP) throw;
                (void)hipGetLastError();  // an allocation failure: the systems stay failed
                release_f64();
                break;
            }
            used_f64 = true;
        } else {
            ensure(prec);
        }
        st.iterations += solve(rp, only.data());
        for (int32_t b = 0; b < nb; ++b)
            if (only[b] && !failed(b) && prec == MOF_PREC_F64) st.recovered_f64++;
    }
    if (used_f64) release_f64();
    for (int32_t b = 0; b < nb; ++b)
        if (first[b] && !failed(b)) st.recovered++;
}

}  // namespace mof

// error handling for the host-only entry points of mof_io.cpp
int mof_io_guard(const std::function<void()> &f) { return guarded(f); }

namespace mof {

void mesh_set_own(mof_mesh *m, int32_t nown) {
    MOF_HIP(hipSetDevice(m->device));
    m->n_own = nown;
    // MOF_SYM_READS: 1 / 0 force the symmetric / plain reads, unset: per mesh
    const int sym = knob(Knob::SymReads) ? (knob_int(Knob::SymReads, 0) != 0) : -1;
    // one host mirror table per (mesh, nown, mode), shared by the clones
    std::shared_ptr<const MirrorTable> mt;
    {
        MeshShared *sh = m->shared.get();
        std::unique_lock<std::mutex> lk;
        if (sh) lk = std::unique_lock<std::mutex>(sh->mu);
        if (sh && sh->mirror && sh->mirror->nown == nown && sh->mirror->sym == sym) {
            mt = sh->mirror;
        } else {
            auto t = std::make_shared<MirrorTable>();
            t->nown = nown;
            t->sym = sym;
            t->table = sell_mirror(m->pat, nown, sym, &t->used);
            if (sh) sh->mirror = t;
            mt = t;
        }
    }
    m->sym_reads = mt->used;
    const std::vector<int32_t> &mir = mt->table;
    m->sell_mir.alloc(mir.size());
    m->sell_mir.upload(mir.data(), mir.size(), m->stream);
    int64_t own = 0;  // positions read at their own place: diagonal + upper blocks
    for (int32_t v : mir) own += v >= 0 && !(v & kMirT);
    m->blocks_read = own;
    MOF_HIP(hipStreamSynchronize(m->stream));
}

// Host half of a mesh build: internal vertex / triangle order, the
// relabelled inputs and the block pattern. Kept in MeshShared so further
// handles of the same mesh on other devices (mof_mesh_clone) only upload.
constexpr int32_t kRowsPerWindow = 256;  // = kRowsPerWG of the row kernels (mof_rowkern.h)

void mesh_prepare_host(mof_mesh *m, const double *xyz, const double *nrm, const int32_t *tri,
                       const double *area, int32_t N, int32_t M, uint32_t flags, const int32_t *perm_in,
                       const int32_t *tri_ids) {
    m->N = N;
    m->n_own = N;
    m->M = M;
    m->flags = flags;
    double t0 = now_ms();
    MOF_REQUIRE(N > 0 && M > 0, "mesh needs N > 0 vertices and M > 0 triangles");
    for (int64_t q = 0; q < 3 * (int64_t)M; ++q)
        MOF_REQUIRE(tri[q] >= 0 && tri[q] < N, "triangle vertex index out of range");
    // internal vertex order (RCM) and triangle order (by smallest
    // internal vertex id), and the relabelled inputs
    m->perm.resize(N);
    m->tperm.resize(M);
    for (int32_t i = 0; i < N; ++i) m->perm[i] = i;
    for (int32_t T = 0; T < M; ++T) m->tperm[T] = T;
    if (perm_in || !(flags & MOF_NO_REORDER)) {
        if (perm_in) {
            m->perm.assign(perm_in, perm_in + N);
        } else {
            mof::Pattern adj;
            mof::build_pattern(tri, N, M, adj);
            m->perm = mof::rcm_order(adj);
            // irregular valence (the smoothed-aggregation criterion): sort the
            // vertices by degree within each 256-row window (one row kernel
            // workgroup) of the RCM order, so a 64-row SELL slice holds rows
            // of like width -- R3: 1.72 M -> 1.32 M SELL slots for 1.15 M
            // blocks -- while every gather stays within the window's lines.
            // Wider windows pad less (512 / 1024 / 2048 rows: ≈1.24 / 1.20 /
            // 1.18 M slots) but scatter the gathers: R3 687 / 676 / 670 vs
            // 696 timesteps/s (round 3, profiles/r03_ab/r3win*).
            const bool wsort = mof::amg_auto_smooth(adj);
            if (wsort) {
                std::vector<int32_t> byrcm(N);  // byrcm[rcm position] = caller vertex
                for (int32_t i = 0; i < N; ++i) byrcm[m->perm[i]] = i;
                std::vector<int32_t> newpos(N);  // rcm position -> internal id
                std::vector<int32_t> win;
                for (int32_t w0 = 0; w0 < N; w0 += kRowsPerWindow) {
                    const int32_t w1 = std::min(N, w0 + kRowsPerWindow);
                    win.resize(w1 - w0);
                    for (int32_t q = w0; q < w1; ++q) win[q - w0] = q;
                    auto deg = [&](int32_t q) { return adj.vptr[byrcm[q] + 1] - adj.vptr[byrcm[q]]; };
                    std::stable_sort(win.begin(), win.end(), [&](int32_t a, int32_t b) { return deg(a) > deg(b); });
                    for (int32_t q = w0; q < w1; ++q) newpos[win[q - w0]] = q;
                }
                m->agg_order.resize(N);
                for (int32_t q = 0; q < N; ++q) m->agg_order[q] = newpos[q];
                for (int32_t i = 0; i < N; ++i) m->perm[i] = newpos[m->perm[i]];
            }
        }
        std::vector<int32_t> key(M);
        for (int32_t T = 0; T < M; ++T)
            key[T] = std::min({m->perm[tri[3 * (size_t)T]], m->perm[tri[3 * (size_t)T + 1]],
                               m->perm[tri[3 * (size_t)T + 2]]});
        std::stable_sort(m->tperm.begin(), m->tperm.end(),
                         [&](int32_t a, int32_t b) { return key[a] < key[b]; });
    }
    m->inv.resize(N);
    for (int32_t i = 0; i < N; ++i) m->inv[m->perm[i]] = i;
    m->tinv.resize(M);
    for (int32_t T = 0; T < M; ++T) m->tinv[m->tperm[T]] = T;
    auto sh = std::make_shared<MeshShared>();
    sh->tri_new.resize(3 * (size_t)M);
    sh->tri_old.resize(3 * (size_t)M);
    sh->area_new.resize(M);
    for (int32_t T = 0; T < M; ++T) {
        const int32_t To = m->tperm[T];
        for (int c = 0; c < 3; ++c) {
            sh->tri_old[3 * (size_t)T + c] = (tri_ids ? tri_ids : tri)[3 * (size_t)To + c];
            sh->tri_new[3 * (size_t)T + c] = m->perm[tri[3 * (size_t)To + c]];
        }
        sh->area_new[T] = area[To];
    }
    sh->xyz_new.resize(3 * (size_t)N);
    sh->nrm_new.resize(3 * (size_t)N);
    for (int32_t i = 0; i < N; ++i)
        for (int d = 0; d < 3; ++d) {
            sh->xyz_new[3 * (size_t)m->perm[i] + d] = xyz[3 * (size_t)i + d];
            sh->nrm_new[3 * (size_t)m->perm[i] + d] = nrm[3 * (size_t)i + d];
        }
    // vertices in no triangle are never gathered: column 0
    sh->icol.assign(N, 0);
    for (size_t q = 0; q < 3 * (size_t)M; ++q) sh->icol[sh->tri_new[q]] = sh->tri_old[q];
    mof::build_pattern(sh->tri_new.data(), N, M, m->pat, m->tinv.data());
    m->shared = std::move(sh);
    m->ms_pattern = now_ms() - t0;
}

// Device half: uploads, the per-mesh kernels (bases, hat gradients, a2) on
// m->device. Identical results on every device (same inputs, same kernels).
void mesh_upload(mof_mesh *m) {
    const MeshShared &H = *m->shared;
    const int32_t N = m->N, M = m->M;
    MOF_HIP(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));
    hipStream_t s = m->stream;
    const mof::Pattern &P = m->pat;
    m->tri.alloc(3 * (size_t)M);
    m->tri.upload(H.tri_new.data(), 3 * (size_t)M, s);
    m->tri_orig.alloc(3 * (size_t)M);
    m->tri_orig.upload(H.tri_old.data(), 3 * (size_t)M, s);
    m->perm_d.alloc(N);
    m->perm_d.upload(m->perm.data(), N, s);
    m->icol.alloc(N);
    m->icol.upload(H.icol.data(), N, s);
    m->area.alloc(M);
    m->area.upload(H.area_new.data(), M, s);
    auto put = [&](mof::DevArray<int32_t> &d, const std::vector<int32_t> &h) {
        d.alloc(h.size());
        d.upload(h.data(), h.size(), s);
    };
    put(m->vptr, P.vptr);
    put(m->vcol, P.vcol);
    put(m->cptr, P.cptr);
    put(m->clist, P.clist);
    put(m->sell_off, P.sell_off);
    put(m->sell_col, P.sell_col);
    put(m->sell_blk, P.sell_blk);
    put(m->blk_row, P.blk_row);
    put(m->diag_pos, P.diag_pos);
    put(m->tsell_off, P.tsell_off);
    put(m->tinc, P.tinc);
    put(m->tslot, P.tslot);
    mesh_set_own(m, N);
    mof::DevArray<double> dxyz, dnrm;
    dxyz.alloc(3 * (size_t)N);
    dxyz.upload(H.xyz_new.data(), 3 * (size_t)N, s);
    dnrm.alloc(3 * (size_t)N);
    dnrm.upload(H.nrm_new.data(), 3 * (size_t)N, s);
    m->e.alloc(6 * (size_t)N);
    m->gw.alloc(9 * (size_t)M);
    m->iw.alloc(2 * (size_t)M);
    m->a2.alloc(4 * (size_t)P.sell_nb());
    m->a2.zero(s);
    m->a2s64.alloc(4 * (size_t)P.sell_nb());
    m->a2s32.alloc(4 * (size_t)P.sell_nb());
    m->w12_64.alloc((size_t)M + 1);
    m->w12_32.alloc((size_t)M + 1);
    m->Aexp.alloc(4 * (size_t)P.sell_nb());
    m->Aexp.zero(s);
    m->fexp.alloc(2 * (size_t)N);
    Events ev;
    MOF_HIP(hipEventRecord(ev.e[0], s));
    mof::launch_geometry(m, dxyz.p, dnrm.p, (m->flags & MOF_GEOM_F32_POINTS) != 0);
    mof::launch_a2(m);
    MOF_HIP(hipEventRecord(ev.e[1], s));
    MOF_HIP(hipStreamSynchronize(s));
    m->ms_geometry = ev.ms(0, 1);
}

void mesh_build(mof_mesh *m, const double *xyz, const double *nrm, const int32_t *tri,
                const double *area, int32_t N, int32_t M, int32_t device, uint32_t flags,
                const int32_t *perm_in, const int32_t *tri_ids) {
    m->device = device;
    mesh_prepare_host(m, xyz, nrm, tri, area, N, M, flags, perm_in, tri_ids);
    mesh_upload(m);
}

}  // namespace mof

extern "C" {

const char *mof_version(void) { return "mofhip 0.6.3 (gfx950, abi 4)"; }

int mof_abi_version(void) { return MOF_ABI_VERSION; }

const char *mof_last_error(void) { return g_err.c_str(); }

int mof_device_count(int32_t *count) {
    return guarded([&] {
        MOF_REQUIRE(count, "count is NULL");
        int n = 0;
        hipError_t e = hipGetDeviceCount(&n);
        *count = (e == hipSuccess) ? n : 0;
    });
}

int mof_mesh_create(const double *xyz, const double *nrm, const int32_t *tri, const double *area,
                    int32_t N, int32_t M, int32_t device, uint32_t flags, mof_mesh **out) {
    return guarded([&] {
        MOF_REQUIRE(out, "out is NULL");
        *out = nullptr;
        MOF_REQUIRE(xyz && nrm && tri && area, "NULL input array");
        int ndev = 0;
        MOF_HIP(hipGetDeviceCount(&ndev));
        MOF_REQUIRE(device >= 0 && device < ndev, "device ordinal out of range");
        DeviceGuard dg(device);
        auto *m = new mof_mesh();
        try {
            mof::mesh_build(m, xyz, nrm, tri, area, N, M, device, flags, nullptr, nullptr);
        } catch (...) {
            mof_mesh_destroy(m);
            throw;
        }
        *out = m;
    });
}

int mof_mesh_clone(const mof_mesh *src, int32_t device, mof_mesh **out) {
    return guarded([&] {
        MOF_REQUIRE(out, "out is NULL");
        *out = nullptr;
        MOF_REQUIRE(src && src->shared, "source mesh is NULL or not a mof_mesh_create handle");
        mof::mesh_join_prep(const_cast<mof_mesh *>(src));
        int ndev = 0;
        MOF_HIP(hipGetDeviceCount(&ndev));
        MOF_REQUIRE(device >= 0 && device < ndev, "device ordinal out of range");
        DeviceGuard dg(device);
        auto *m = new mof_mesh();
        try {
            // host state of the source (pattern, orders): copied, not rebuilt
            m->N = src->N;
            m->M = src->M;
            m->n_own = src->N;
            m->flags = src->flags;
            m->device = device;
            m->pat = src->pat;
            m->perm = src->perm;
            m->inv = src->inv;
            m->tperm = src->tperm;
            m->tinv = src->tinv;
            m->agg_order = src->agg_order;
            m->shared = src->shared;
            m->ms_pattern = 0.0;
            mof::mesh_upload(m);
        } catch (...) {
            mof_mesh_destroy(m);
            throw;
        }
        *out = m;
    });
}

int mof_mesh_destroy(mof_mesh *m) {
    if (!m) return MOF_OK;
    return guarded([&] {
        mof::mesh_join_prep(m);  // its error, if any, dies with the handle
        {
            DeviceGuard dg(m->device);
            if (m->stream) (void)hipStreamSynchronize(m->stream);
            if (m->h_sysi) (void)hipHostFree(m->h_sysi);
            if (m->h_sysd) (void)hipHostFree(m->h_sysd);
            for (auto e : m->spmv_events) (void)hipEventDestroy(e);
            delete m->stage;
            m->stage = nullptr;
            for (auto &e : m->hev)
                if (e) (void)hipEventDestroy(e);
            mof::amg_destroy(m->amg);
            m->amg = nullptr;
            if (m->stream) (void)hipStreamDestroy(m->stream);
            m->stream = nullptr;
            delete m;  // DevArray destructors free on the current (guarded) device
        }
    });
}

// The multigrid hierarchy (host build and upload) of the options' solves on a
// host thread of the handle: a per-mesh setup, started by the drop-in's
// compute_geometrical_quantities (the reference builds a2 there,
// compute_optical_flow.py:27-97) so that the first compute_velocity_field
// call finds it built -- round 4: 5-8 ms of that call's 12-16 ms on the
// reference's 3,249-vertex surfaces. Nothing else on the handle is touched
// by the thread but its multigrid state and stream (uploads); the calls that
// use them join it first.
int mof_mesh_prepare(mof_mesh *m, const mof_opts *opts) {
    return guarded([&] {
        MOF_REQUIRE(m, "mesh is NULL");
        mof_opts o{};
        if (opts) {
            MOF_REQUIRE(opts->struct_size == 0 || opts->struct_size >= sizeof(mof_opts),
                        "mof_opts.struct_size too small");
            o = *opts;
        }
        mof::mesh_join_prep(m);
        std::lock_guard<std::mutex> lk(m->prep_mu);
        m->prep_err = nullptr;  // a new setup supersedes the last one's error
        if (!(o.flags & MOF_PRECOND_AMG) || o.precision != MOF_PREC_MIXED || m->n_own != m->N) return;
        m->prep = std::async(std::launch::async, [m] {
            DeviceGuard dg(m->device);
            (void)mof::amg_build(m);
        });
    });
}

int mof_mesh_sync(mof_mesh *m) {
    return guarded([&] {
        MOF_REQUIRE(m, "mesh is NULL");
        mof::mesh_join_prep(m, true);
    });
}

int mof_mesh_get_info(const mof_mesh *m, mof_mesh_info *info) {
    return guarded([&] {
        MOF_REQUIRE(m && info, "NULL argument");
        info->N = m->N;
        info->M = m->M;
        info->device = m->device;
        info->nblocks = m->pat.nblocks();
        info->nnz_struct = 4 * (int64_t)m->pat.nblocks();
        info->sell_blocks = m->pat.sell_nb();
        info->ms_geometry = m->ms_geometry;
        info->ms_pattern = m->ms_pattern;
        info->blocks_read = m->blocks_read;
        info->max_batch = mof::grid_batch_cap(m);
        info->pad_ = 0;
    });
}

int mof_geometry_export(mof_mesh *m, double *e, double *grad_w, double *iw) {
    return guarded([&] {
        MOF_REQUIRE(m, "mesh is NULL");
        DeviceGuard dg(m->device);
        hipStream_t s = m->stream;
        std::vector<double> e_int, gw_int, iw_int;
        if (e) {
            e_int.resize(m->e.n);
            MOF_HIP(hipMemcpyAsync(e_int.data(), m->e.p, m->e.bytes(), hipMemcpyDeviceToHost, s));
        }
        if (grad_w) {
            gw_int.resize(m->gw.n);
            MOF_HIP(hipMemcpyAsync(gw_int.data(), m->gw.p, m->gw.bytes(), hipMemcpyDeviceToHost, s));
        }
        if (iw) {
            iw_int.resize(m->iw.n);
            MOF_HIP(hipMemcpyAsync(iw_int.data(), m->iw.p, m->iw.bytes(), hipMemcpyDeviceToHost, s));
        }
        MOF_HIP(hipStreamSynchronize(s));
        // back to the caller's vertex and triangle order
        if (e)
            for (int32_t i = 0; i < m->N; ++i)
                std::memcpy(e + 6 * (size_t)i, e_int.data() + 6 * (size_t)m->perm[i], 6 * sizeof(double));
        if (grad_w)
            for (int32_t T = 0; T < m->M; ++T)
                std::memcpy(grad_w + 9 * (size_t)T, gw_int.data() + 9 * (size_t)m->tinv[T], 9 * sizeof(double));
        if (iw)
            for (int32_t T = 0; T < m->M; ++T)
                std::memcpy(iw + 2 * (size_t)T, iw_int.data() + 2 * (size_t)m->tinv[T], 2 * sizeof(double));
    });
}

int mof_csr_export(mof_mesh *m, int32_t which, int32_t drop_zeros, int32_t *indptr,
                   int32_t *indices, double *data, int64_t *nnz) {
    return guarded([&] {
        MOF_REQUIRE(m && indptr && indices && data && nnz, "NULL argument");
        MOF_REQUIRE(which == MOF_CSR_A2 || which == MOF_CSR_A_LAST, "unknown matrix id");
        DeviceGuard dg(m->device);
        const int64_t snb = m->pat.sell_nb();
        std::vector<double> blk(4 * (size_t)snb);
        const double *src = m->a2.p;
        if (which == MOF_CSR_A_LAST) {
            if (!m->have_last_A) throw mof::Error{MOF_E_STATE, "no assembled system: call mof_assemble first"};
            src = m->Aexp.p;
        }
        MOF_HIP(hipMemcpyAsync(blk.data(), src, sizeof(double) * blk.size(), hipMemcpyDeviceToHost,
                               m->stream));
        MOF_HIP(hipStreamSynchronize(m->stream));
        sell_to_csr(m, blk, drop_zeros, indptr, indices, data, nnz);
    });
}

int mof_assemble(mof_mesh *m, const double *I0, const double *I1, double dt, double lambda,
                 double *f) {
    return guarded([&] {
        MOF_REQUIRE(m && I0 && I1, "NULL argument");
        mof::mesh_join_prep(m);
        DeviceGuard dg(m->device);
        hipStream_t s = m->stream;
        mof::ensure_workspace(m, 1, MOF_PREC_MIXED);
        mof::Workspace &w = m->ws;
        const int64_t N = m->N;
        MOF_HIP(hipMemcpyAsync(w.Ibuf.p, I0, sizeof(double) * N, hipMemcpyHostToDevice, s));
        MOF_HIP(hipMemcpyAsync(w.Ibuf.p + N, I1, sizeof(double) * N, hipMemcpyHostToDevice, s));
        MOF_HIP(hipMemcpyAsync(w.dt.p, &dt, sizeof(double), hipMemcpyHostToDevice, s));
        mof::launch_assemble_export(m, w.Ibuf.p, w.Ibuf.p + N, lambda, s);
        m->have_last_A = true;
        std::vector<double> fi(2 * N);
        if (f)
            MOF_HIP(hipMemcpyAsync(fi.data(), m->fexp.p, sizeof(double) * 2 * N, hipMemcpyDeviceToHost, s));
        MOF_HIP(hipStreamSynchronize(s));
        if (f)
            for (int64_t i = 0; i < N; ++i) {
                f[i] = fi[m->perm[i]];
                f[N + i] = fi[N + m->perm[i]];
            }
    });
}

int mof_solve_range(mof_mesh *m, const double *I, const double *I2, const double *t_k, int32_t T,
                    int32_t k0, int32_t k1, double lambda, const mof_opts *opts, double *V_out,
                    mof_stats *stats) {
    int nonconv = 0;
    int rc = guarded([&] {
        MOF_REQUIRE(m && I && t_k && V_out, "NULL argument");
        MOF_REQUIRE(T >= 1 && k0 >= 0 && k0 <= k1 && k1 <= T - 1, "need 0 <= k0 <= k1 <= T-1");
        mof::mesh_join_prep(m);  // its error: below, for the multigrid solve
        mof_opts o{};
        if (opts) {
            MOF_REQUIRE(opts->struct_size == 0 || opts->struct_size >= sizeof(mof_opts),
                        "mof_opts.struct_size too small");
            o = *opts;
        }
        MOF_REQUIRE(o.precision == MOF_PREC_F64 || o.precision == MOF_PREC_MIXED, "unknown precision");
        mof::SolveParams sp;
        sp.precision = o.precision;
        sp.amg = (o.flags & MOF_PRECOND_AMG) != 0;
        MOF_REQUIRE(!sp.amg || o.precision == MOF_PREC_MIXED, "MOF_PRECOND_AMG needs MOF_PREC_MIXED");
        if (sp.amg) mof::mesh_join_prep(m, true);  // the multigrid setup's error, if any
        // the multigrid smoother is the 2x2 block Jacobi
        sp.block_jacobi = sp.amg || !(o.flags & MOF_NO_BLOCK_JACOBI);
        sp.time_spmv = (o.flags & MOF_TIME_SPMV) != 0;
        sp.max_iter = o.max_iter > 0 ? o.max_iter : (sp.amg ? 1000 : 10000);
        sp.max_outer = o.max_outer > 0 ? o.max_outer : 10;
        sp.rtol = o.rtol > 0 ? o.rtol : 1e-8;
        sp.inner_rtol = o.inner_rtol > 0 ? o.inner_rtol : 1e-4;
        // error control: etol 0 -> 1e-7 of max|V|, < 0 -> off
        sp.etol = o.etol > 0 ? o.etol : (o.etol < 0 ? 0.0 : 1e-7);
        // a multigrid-preconditioned inner solve takes tens of iterations:
        // one that stops improving, or hits max_iter, has a bad preconditioner
        sp.stall = sp.amg ? mof::kPcgStall : 0;
        sp.fail_at_max_iter = sp.amg;
        sp.fused = (o.flags & MOF_SOLVE_EAGER) ? 0 : ((o.flags & MOF_SOLVE_FUSED) ? 1 : -1);
        const bool recovery = !(o.flags & MOF_NO_RECOVERY);
        const bool dev_io = (o.flags & MOF_IO_DEVICE) != 0;
        if (!I2) I2 = I;
        DeviceGuard dg(m->device);
        const int32_t K = k1 - k0;
        mof_stats st{};
        mof::SpmvTiming timing;
        if (K > 0) {
            int32_t Bmax = o.batch;
            if (Bmax <= 0) {
                // auto: 1024 timesteps per launch sequence (C3: +4.6 % for 512
                // over 256 (round 2), +1-4 % for 1024 over 512 by box (round
                // 4, profiles/r04_ab/batch/)), fewer when half the free device
                // memory cannot hold their workspace (~720 B per vertex and
                // system with the multigrid levels; C3 at 1024: 121 GB)
                size_t free_b = 0, total_b = 0;
                MOF_HIP(hipMemGetInfo(&free_b, &total_b));
                const double per_sys = 720.0 * (double)m->N + 1.0;
                // a mixed solve's fp64 recovery pass allocates A64, u64 and
                // fc at the batch size on top (~330 B per vertex and
                // system): the workspace keeps half the free memory and,
                // with the recovery's arrays, 85 % of it
                const double per_rec = per_sys + 8.0 * (4.0 * (double)m->pat.sell_nb() + 6.0 * (m->M + 1.0));
                Bmax = (int32_t)std::max(1.0, std::min({1024.0, 0.5 * (double)free_b / per_sys,
                                                        0.85 * (double)free_b / per_rec}));
            }
            // every launch grid within 2^32 work-items (an explicit batch
            // too: V does not depend on the batch size)
            const int32_t B = std::min(K, std::min(Bmax, mof::grid_batch_cap(m)));
            hipStream_t s = o.stream ? (hipStream_t)o.stream : m->stream;
            solve_batches(m, I, I2, t_k, k0, k1, B, lambda, sp, o, recovery, dev_io, s, V_out, st, timing);
        }
        st.systems = K;
        st.spmv_launches = timing.launches;
        st.ms_spmv = timing.ms;
        st.spmv_bytes = timing.bytes;
        st.spmv_systems = timing.systems;
        st.spmv_full_launches = timing.full_launches;
        st.ms_spmv_full = timing.ms_full;
        st.fused_launches = timing.fused_launches;
        st.ms_fused = timing.ms_fused;
        if (stats) *stats = st;
        if (st.failed) {
            nonconv = 1;
            g_err = std::to_string(st.failed) + " system(s) did not converge; their V is NaN-filled";
        }
    });
    if (rc == MOF_OK && nonconv) return MOF_E_NOCONV;
    return rc;
}

int mof_velocity_vectors(int32_t device, const double *e, const double *V, int32_t N, int32_t K,
                         double *V_coord, double *speed, uint32_t flags, void *stream) {
    return guarded([&] {
        MOF_REQUIRE(e && V && N > 0 && K >= 0, "bad arguments");
        int ndev = 0;
        MOF_HIP(hipGetDeviceCount(&ndev));
        MOF_REQUIRE(device >= 0 && device < ndev, "device ordinal out of range");
        DeviceGuard dg(device);
        if (K == 0 || (!V_coord && !speed)) return;
        hipStream_t s = (hipStream_t)stream;
        if (flags & MOF_IO_DEVICE) {
            mof::launch_velocity_vectors(N, K, e, V, V_coord, speed, s);
            MOF_HIP(hipStreamSynchronize(s));
            return;
        }
        const size_t nk = (size_t)N * K;
        mof::DevArray<double> de, dV, dc, dsp;
        de.alloc(6 * (size_t)N);
        de.upload(e, 6 * (size_t)N, s);
        dV.alloc(2 * nk);
        dV.upload(V, 2 * nk, s);
        if (V_coord) dc.alloc(3 * nk);
        if (speed) dsp.alloc(nk);
        mof::launch_velocity_vectors(N, K, de.p, dV.p, V_coord ? dc.p : nullptr,
                                     speed ? dsp.p : nullptr, s);
        if (V_coord)
            MOF_HIP(hipMemcpyAsync(V_coord, dc.p, 3 * nk * sizeof(double), hipMemcpyDeviceToHost, s));
        if (speed) MOF_HIP(hipMemcpyAsync(speed, dsp.p, nk * sizeof(double), hipMemcpyDeviceToHost, s));
        MOF_HIP(hipStreamSynchronize(s));
    });
}

int mof_singularities(int32_t device, const void *coords, const int32_t *triangles, int32_t N, int32_t M,
                      const double *V_coord, int32_t K, double eps, uint32_t flags, void *stream,
                      double *vmax, uint8_t *vertex_flag, uint8_t *triangle_flag, double *lam_mu) {
    return guarded([&] {
        MOF_REQUIRE(coords && V_coord && vmax && vertex_flag && N > 0 && M >= 0 && K >= 0,
                    "bad arguments");
        MOF_REQUIRE(M == 0 || (triangles && triangle_flag && lam_mu), "NULL triangle argument");
        int ndev = 0;
        MOF_HIP(hipGetDeviceCount(&ndev));
        MOF_REQUIRE(device >= 0 && device < ndev, "device ordinal out of range");
        DeviceGuard dg(device);
        if (K == 0) return;
        hipStream_t s = (hipStream_t)stream;
        const bool f32 = (flags & MOF_COORDS_F32) != 0;
        const size_t cb = 3 * (size_t)N * (f32 ? sizeof(float) : sizeof(double));
        if (!(flags & MOF_IO_DEVICE)) {
            // triangle indices checked on the host before any gather
            for (int64_t q = 0; q < 3 * (int64_t)M; ++q)
                MOF_REQUIRE(triangles[q] >= 0 && triangles[q] < N, "triangle index out of range");
        }
        if (flags & MOF_IO_DEVICE) {
            mof::launch_singularities(N, M, K, coords, f32, triangles, V_coord, eps, vmax, vertex_flag,
                                      triangle_flag, lam_mu, s);
            MOF_HIP(hipStreamSynchronize(s));
            return;
        }
        const size_t nk = (size_t)N * K, mk = (size_t)M * K;
        mof::DevArray<uint8_t> dc, dvf, dtf;
        mof::DevArray<int32_t> dt;
        mof::DevArray<double> dV, dmax, dlm;
        dc.alloc(cb);
        MOF_HIP(hipMemcpyAsync(dc.p, coords, cb, hipMemcpyHostToDevice, s));
        dt.alloc(3 * (size_t)M);
        if (M) dt.upload(triangles, 3 * (size_t)M, s);
        dV.alloc(3 * nk);
        dV.upload(V_coord, 3 * nk, s);
        dmax.alloc(K);
        dvf.alloc(nk);
        dtf.alloc(mk);
        dlm.alloc(2 * mk);
        mof::launch_singularities(N, M, K, dc.p, f32, dt.p, dV.p, eps, dmax.p, dvf.p, dtf.p, dlm.p, s);
        MOF_HIP(hipMemcpyAsync(vmax, dmax.p, K * sizeof(double), hipMemcpyDeviceToHost, s));
        MOF_HIP(hipMemcpyAsync(vertex_flag, dvf.p, nk, hipMemcpyDeviceToHost, s));
        if (M) {
            MOF_HIP(hipMemcpyAsync(triangle_flag, dtf.p, mk, hipMemcpyDeviceToHost, s));
            MOF_HIP(hipMemcpyAsync(lam_mu, dlm.p, 2 * mk * sizeof(double), hipMemcpyDeviceToHost, s));
        }
        MOF_HIP(hipStreamSynchronize(s));
    });
}

int mof_singularities_compact(int32_t device, const void *coords, const int32_t *triangles, int32_t N,
                              int32_t M, const double *V_coord, int32_t K, double eps, uint32_t flags, void *stream,
                              int64_t cap, int64_t *totals, double *vmax, int64_t *n_vert, int32_t *vert_idx,
                              int64_t *n_tri, int32_t *tri_idx, double *lam_mu) {
    return guarded([&] {
        MOF_REQUIRE(coords && V_coord && totals && vmax && n_vert && n_tri && N > 0 && M >= 0 && K >= 0 &&
                        cap >= 0,
                    "bad arguments");
        MOF_REQUIRE(M == 0 || triangles, "NULL triangles");
        MOF_REQUIRE(cap == 0 || (vert_idx && tri_idx && lam_mu), "NULL output list");
        int ndev = 0;
        MOF_HIP(hipGetDeviceCount(&ndev));
        MOF_REQUIRE(device >= 0 && device < ndev, "device ordinal out of range");
        DeviceGuard dg(device);
        totals[0] = totals[1] = 0;
        for (int32_t k = 0; k < K; ++k) n_vert[k] = n_tri[k] = 0;
        if (K == 0) return;
        const bool dev_io = (flags & MOF_IO_DEVICE) != 0;
        if (!dev_io)
            for (int64_t q = 0; q < 3 * (int64_t)M; ++q)
                MOF_REQUIRE(triangles[q] >= 0 && triangles[q] < N, "triangle index out of range");
        hipStream_t s = (hipStream_t)stream;
        const bool f32 = (flags & MOF_COORDS_F32) != 0;
        const size_t cb = 3 * (size_t)N * (f32 ? sizeof(float) : sizeof(double));
        const size_t nk = (size_t)N * K;
        mof::DevArray<uint8_t> dc, dvf;
        mof::DevArray<int32_t> dt;
        mof::DevArray<double> dV, dmax;
        mof::DevArray<unsigned long long> dcnt;
        mof::DevArray<int2> dvr, dtr;
        mof::DevArray<double2> dlm;
        const void *pc = coords;
        const int32_t *pt = triangles;
        const double *pV = V_coord;
        if (!dev_io) {
            dc.alloc(cb);
            MOF_HIP(hipMemcpyAsync(dc.p, coords, cb, hipMemcpyHostToDevice, s));
            dt.alloc(3 * (size_t)M);
            if (M) dt.upload(triangles, 3 * (size_t)M, s);
            dV.alloc(3 * nk);
            dV.upload(V_coord, 3 * nk, s);
            pc = dc.p;
            pt = dt.p;
            pV = dV.p;
        }
        dmax.alloc(K);
        dvf.alloc(nk);
        dcnt.alloc(2);
        dvr.alloc(std::max<int64_t>(1, cap));
        dtr.alloc(std::max<int64_t>(1, cap));
        dlm.alloc(std::max<int64_t>(1, cap));
        mof::launch_singularities_compact(N, M, K, pc, f32, pt, pV, eps, dmax.p, dvf.p, dcnt.p, cap, dvr.p, dtr.p,
                                          dlm.p, s);
        unsigned long long cnt[2] = {0, 0};
        MOF_HIP(hipMemcpyAsync(cnt, dcnt.p, sizeof(cnt), hipMemcpyDeviceToHost, s));
        MOF_HIP(hipMemcpyAsync(vmax, dmax.p, K * sizeof(double), hipMemcpyDeviceToHost, s));
        MOF_HIP(hipStreamSynchronize(s));
        totals[0] = (int64_t)cnt[0];
        totals[1] = (int64_t)cnt[1];
        MOF_REQUIRE(totals[0] <= cap && totals[1] <= cap,
                    "record capacity too small (totals holds the vertex / triangle record counts needed)");
        std::vector<int2> vr(cnt[0]), tr(cnt[1]);
        std::vector<double2> lm(cnt[1]);
        if (cnt[0]) MOF_HIP(hipMemcpyAsync(vr.data(), dvr.p, cnt[0] * sizeof(int2), hipMemcpyDeviceToHost, s));
        if (cnt[1]) {
            MOF_HIP(hipMemcpyAsync(tr.data(), dtr.p, cnt[1] * sizeof(int2), hipMemcpyDeviceToHost, s));
            MOF_HIP(hipMemcpyAsync(lm.data(), dlm.p, cnt[1] * sizeof(double2), hipMemcpyDeviceToHost, s));
        }
        MOF_HIP(hipStreamSynchronize(s));
        // records arrive in atomic order: field-major, ascending index
        auto key = [](const int2 &r) { return ((int64_t)r.x << 32) | (uint32_t)r.y; };
        std::sort(vr.begin(), vr.end(), [&](const int2 &a, const int2 &b) { return key(a) < key(b); });
        for (size_t q = 0; q < vr.size(); ++q) {
            vert_idx[q] = vr[q].y;
            n_vert[vr[q].x]++;
        }
        std::vector<size_t> ord(tr.size());
        for (size_t q = 0; q < ord.size(); ++q) ord[q] = q;
        std::sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return key(tr[a]) < key(tr[b]); });
        for (size_t q = 0; q < ord.size(); ++q) {
            tri_idx[q] = tr[ord[q]].y;
            lam_mu[2 * q] = lm[ord[q]].x;
            lam_mu[2 * q + 1] = lm[ord[q]].y;
            n_tri[tr[ord[q]].x]++;
        }
    });
}

int mof_amg_probe(const int32_t *tri, const double *e, int32_t N, int32_t M, int32_t *n_levels,
                  int32_t *level_nodes, double *qtq_err, double *max_curl) {
    return guarded([&] {
        MOF_REQUIRE(tri && e && n_levels && level_nodes && N > 0 && M > 0, "bad arguments");
        for (int64_t q = 0; q < 3 * (int64_t)M; ++q)
            MOF_REQUIRE(tri[q] >= 0 && tri[q] < N, "triangle vertex index out of range");
        mof::Pattern pat;
        mof::build_pattern(tri, N, M, pat);
        mof::AmgHierarchy H;
        mof::build_amg(pat, e, mof::AmgParams{}, H);
        *n_levels = (int32_t)std::min<size_t>(16, H.levels.size());
        if (max_curl) *max_curl = H.max_curl;
        for (int32_t l = 0; l < *n_levels; ++l) level_nodes[l] = H.levels[l].n;
        if (qtq_err) {
            double err = 0.0;
            const mof::AmgLevel &F = H.levels[0];
            for (size_t I = 0; I + 1 < F.mptr.size(); ++I)
                for (int a = 0; a < 3; ++a)
                    for (int c = 0; c < 3; ++c) {
                        double sum = 0.0;
                        for (int32_t q = F.mptr[I]; q < F.mptr[I + 1]; ++q) {
                            const int32_t i = F.mlist[q];
                            for (int r = 0; r < 2; ++r)
                                sum += (double)F.Q[(size_t)i * 6 + 3 * r + a] * F.Q[(size_t)i * 6 + 3 * r + c];
                        }
                        const bool dead_col = H.levels.size() > 1 && H.levels[1].dead[3 * I + a];
                        const double want = (a == c && !dead_col) ? 1.0 : 0.0;
                        err = std::max(err, std::fabs(sum - want));
                    }
            *qtq_err = err;
        }
    });
}

int mof_xcd_map_check(int32_t nblk, int32_t batch, int32_t group) {
    return guarded([&] {
        MOF_REQUIRE(nblk > 0 && batch > 0 && group >= 0, "bad arguments");
        MOF_REQUIRE(mof::xcd_map_covers(nblk, batch, group), "XCD order does not cover every (row block, system) once");
    });
}

int mof_xcd_batch_cap(int64_t nblk, int32_t group, int32_t *batch) {
    return guarded([&] {
        MOF_REQUIRE(nblk > 0 && group >= 0 && batch, "bad arguments");
        *batch = mof::xcd_batch_cap_host(nblk, group);
    });
}

int mof_bench_spmv(mof_mesh *m, uint32_t precision, int32_t batch, int32_t reps,
                   double *ms_per_launch, double *bytes_per_launch) {
    return guarded([&] {
        MOF_REQUIRE(m && ms_per_launch && bytes_per_launch, "NULL argument");
        MOF_REQUIRE(reps > 0, "reps must be positive");
        mof::mesh_join_prep(m);
        DeviceGuard dg(m->device);
        *ms_per_launch = mof::bench_spmv(m, precision, batch, reps, m->stream, bytes_per_launch);
    });
}

}  // extern "C"
