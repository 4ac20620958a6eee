// mof_internal.h -- shared declarations of libmofhip (MI355X / gfx950).
//
// Device data layout:
//  * vertex 2x2 blocks: block p = (i, j) of vertex row i holds
//      {A(i,j), A(i,j+N), A(i+N,j), A(i+N,j+N)}  (planar unknowns of the
//      reference, compute_optical_flow.py:83-84);
//  * the smoothness matrix a2 is stored SELL-64: row i = slice i/64, lane
//    i%64; its t-th block lives at sell_off[i/64] + 64*t + i%64, so one
//    wave-instruction reads 64 consecutive blocks;
//  * A_b = a1_b + lambda a2 of every system is materialised in the same SELL
//    layout in the inner solver's precision; the fp64 residual applies a1
//    per triangle from u_T = (grad_M I . e_a^alpha), 6 values per triangle,
//    through a SELL-64 vertex -> incident-triangle list (tinc);
//  * solver vectors are interleaved per vertex: v[2*i + alpha].
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <functional>
#include <future>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/mof.h"
#include "mof_knobs.h"

namespace mof {

constexpr int kWG = 256;     // threads per workgroup (4 waves)
constexpr int kSlice = 64;   // SELL slice height = wavefront size

struct Error {
    int code;
    std::string msg;
};

#define MOF_HIP(call)                                                              \
    do {                                                                           \
        hipError_t e_ = (call);                                                    \
        if (e_ != hipSuccess)                                                      \
            throw ::mof::Error{MOF_E_HIP, std::string(#call) + " failed: " +       \
                                              hipGetErrorString(e_)};              \
    } while (0)

#define MOF_REQUIRE(cond, msg)                                                     \
    do {                                                                           \
        if (!(cond)) throw ::mof::Error{MOF_E_ARG, (msg)};                         \
    } while (0)

template <typename T>
struct DevArray {
    T *p = nullptr;
    size_t n = 0;
    DevArray() = default;
    DevArray(const DevArray &) = delete;
    DevArray &operator=(const DevArray &) = delete;
    ~DevArray() { release(); }
    void alloc(size_t count) {
        release();
        if (count == 0) count = 1;
        MOF_HIP(hipMalloc(&p, count * sizeof(T)));
        n = count;
    }
    void zero(hipStream_t s) { MOF_HIP(hipMemsetAsync(p, 0, n * sizeof(T), s)); }
    void upload(const T *h, size_t count, hipStream_t s) {
        MOF_HIP(hipMemcpyAsync(p, h, count * sizeof(T), hipMemcpyHostToDevice, s));
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    size_t bytes() const { return n * sizeof(T); }
};

// SELL slot of block t (vcol order) of a row whose diagonal block is its
// td-th: the diagonal goes first, so each wave of a per-position kernel (one
// slot of 64 rows) holds only diagonal or only off-diagonal blocks -- the
// diagonal ones fold every incident triangle (plus f and D^-1 in the
// assembly), the others two. Also for the coarse multigrid levels.
__host__ __device__ inline int32_t sell_slot(int32_t t, int32_t td) { return t == td ? 0 : (t < td ? t + 1 : t); }
__host__ __device__ inline int32_t sell_block(int32_t slot, int32_t td) {
    return slot == 0 ? td : (slot <= td ? slot - 1 : slot);
}

// Symmetric reads of the operators through the mirror table (mof_rowkern.h
// spmv_row), chosen per mesh (sell_mirror): the assembly then stores no lower
// blocks and the level-0 Galerkin lists read them as transposed upper ones.
// sell_mirror entries: position | kMirT = read the block transposed
constexpr int32_t kMirT = 1 << 30;
constexpr int32_t kMirPos = kMirT - 1;

// Host-side sparsity structures, built once per mesh (mof_pattern.cpp).
struct Pattern {
    int32_t N = 0, M = 0;
    std::vector<int32_t> vptr, vcol;   // vertex adjacency, self included, sorted
    std::vector<int32_t> cptr, clist;  // per block: contributions T*9 + a*3 + b, T ascending
    int32_t nslices = 0;
    std::vector<int32_t> sell_off;     // (nslices+1), in blocks (multiples of 64)
    std::vector<int32_t> sell_col;     // (sell_nb) column vertex, padding -> row itself
    std::vector<int32_t> sell_blk;     // (sell_nb) block index at a SELL position, -1 = padding
    std::vector<int32_t> blk_row;      // (nblocks) row vertex of each block
    std::vector<int32_t> diag_pos;     // (N) SELL position of the diagonal block of row i
    // vertex -> incident triangles, SELL-64, triangle order; 4 ints per entry:
    // {T, corner of i in T, vertex of corner a+1, vertex of corner a+2};
    // padding entries point at the all-zero triangle slot T = M.
    std::vector<int32_t> tsell_off;    // (nslices+1), in entries
    std::vector<int32_t> tinc;         // (4 * tsell_nb)
    // per incidence entry: SELL slots (in row i) of the blocks (i, v_{a+1})
    // and (i, v_{a+2}), packed s1 | s2 << 8 (row-wise assembly)
    std::vector<int32_t> tslot;        // (tsell_nb)
    int32_t max_w = 0;                 // widest SELL row (blocks)
    int64_t sell_nb() const { return sell_off.empty() ? 0 : sell_off.back(); }
    int64_t tsell_nb() const { return tsell_off.empty() ? 0 : tsell_off.back(); }
    int32_t nblocks() const { return (int32_t)vcol.size(); }
};

// torder (optional): torder[q] = index in `tri` of the caller's triangle q;
// contribution lists then follow the caller's triangle order (the order the
// reference's lil folds), whatever the storage order of `tri`.
void build_pattern(const int32_t *tri, int32_t N, int32_t M, Pattern &pat,
                   const int32_t *torder = nullptr);
std::vector<int32_t> rcm_order(const Pattern &pat);
std::vector<int32_t> sell_mirror(const Pattern &pat, int32_t nown, int sym, bool *used);

// Per-batch device workspace (capacity B systems).
struct Workspace {
    int32_t cap = 0;        // systems
    int32_t nblk = 0;       // workgroups per system for row kernels
    DevArray<double> u64, fc;          // [B][M+1][6] per-triangle u = grad_M I . e, f terms
    DevArray<float> u32;               // [B][M+1][6] fp32 u (mixed-precision assembly)
    DevArray<float> A32;               // [B][sell_nb][4] A_b in fp32 (MOF_PREC_MIXED)
    DevArray<double> A64;              // [B][sell_nb][4] A_b in fp64 (MOF_PREC_F64), lazily
    DevArray<double> dinv64;           // [B][N][4] 2x2 block-Jacobi inverses
    DevArray<float> dinv32;
    DevArray<double> rhs;              // [B][N][2] f (interleaved)
    DevArray<double> x64, r64;         // [B][N][2] outer solution / residual
    DevArray<double> vx, vr, vz, vp, vq;  // [B][N][2] inner PCG vectors (fp64 sized)
    DevArray<double> part_pq;          // [B][nblk]
    DevArray<double> part_rzrr;        // [2][B][nblk][2]
    DevArray<double> part_rr0;         // [B][nblk][2]
    DevArray<double> part_dx;          // [B][nvb][2]: max|d|, max|x64| per k_outer_update block
    DevArray<double> sc;               // pre-reduced PCG scalars: r.z, |r|^2 [2][B][2], p.q [2][B]
    DevArray<double> sysd;             // [B][8] per-system scalars
    DevArray<int32_t> sysi;            // [B][8] per-system flags
    DevArray<int32_t> smap;            // [B] the systems a PCG tail chunk's launches cover (SysMap)
    DevArray<double> dt;               // [B]
    DevArray<double> Ibuf;             // [B][N] I0 rows + [B][N] I1 rows (host-staged)
    DevArray<double> Iint;             // the batch's I rows in internal vertex order ([B+1] or [2B] rows)
    DevArray<double> Vbuf;             // [B][2N] planar output staging
    // the mixed path leaves u64 unwritten (the fp64 residual re-forms u from
    // the batch's I rows); the fp64 recovery re-runs k_tri_step from the rows
    // below when it needs u64
    bool u64_stale = false;
    const double *J0 = nullptr, *J1 = nullptr;  // the batch's I0 / I1 rows (in Iint), row stride N
    int32_t JB = 0;                              // their systems
};


// per-system scalar slots (Workspace::sysd / sysi)
//  SD_RR0 / SD_BEST: |r|^2 at the start of the inner solve / smallest so far
//  SI_BEST_IT: iteration of SD_BEST (stagnation detector)
//  SI_FAIL_IT / SI_FAIL_WHY: inner iteration and reason (FailWhy) of a failure
//  SI_ITSUM / SI_ITMAX / SD_OUTER: the fused solve's (k_solve_fused) inner
//  iterations summed over its refinement steps, the largest inner solve, and
//  the refinement steps taken (the eager path counts these on the host)
//  SD_EST / SD_XMAX: the error estimate after the last refinement step,
//  max|d| |r_{k+1}| / |r_k| (k_outer_check), and max|x64| (error control)
//  SI_MET: the last outer check found rel <= rtol (the system only stayed
//  active for the error estimate): a later inner solve that fails leaves
//  x64 at that iterate, and the system retires instead of failing
enum SysD { SD_TOL2 = 0, SD_RR = 1, SD_FF = 2, SD_REL = 3, SD_RR0 = 4, SD_BEST = 5, SD_OUTER = 6, SD_EST = 7,
            SD_XMAX = 8 };
enum SysI { SI_CONV = 0, SI_ACTIVE = 1, SI_FAILED = 2, SI_ITSUM = 3, SI_BEST_IT = 4, SI_FAIL_IT = 5, SI_FAIL_WHY = 6,
            SI_ITMAX = 7, SI_MET = 8 };
enum FailWhy { FW_BREAKDOWN = 1, FW_DIVERGED = 2, FW_STALLED = 3, FW_MAXITER = 4, FW_RESIDUAL = 5 };
constexpr int kSysStride = 12;

struct AmgDevice;     // mof_amg.h
struct AmgHierarchy;  // mof_amg.h
class HostStage;      // mof_hostio.h

// Host state of one mesh shared by its handles on several devices
// (mof_mesh_create builds it once, mof_mesh_clone reuses it): the inputs in
// the internal vertex / triangle order, the symmetric-read mirror table, and
// the multigrid hierarchies built so far (per parameter set), so N device
// handles cost one host pattern + hierarchy build, not N.
struct MirrorTable {
    int32_t nown = 0;
    int sym = -1;
    bool used = false;
    std::vector<int32_t> table;
};
struct MeshShared {
    std::vector<int32_t> tri_new, tri_old, icol;
    std::vector<double> area_new, xyz_new, nrm_new;
    std::mutex mu;  // guards mirror and amg
    std::shared_ptr<const MirrorTable> mirror;
    std::vector<std::pair<std::string, std::shared_ptr<const AmgHierarchy>>> amg;
    std::mutex amg_build_mu;  // one hierarchy build at a time per mesh
};

// Cross-part reduction layout of the PCG kernels: partial record of
// (part, system b, workgroup w) at ((part * B + b) * nmax + w) * NV; rows
// >= nown (a decomposed part's ghosts) are computed but never summed.
struct RedArgs {
    int32_t P = 1, part = 0, nmax = 0, nown = 0;
};

}  // namespace mof

// The opaque handle of the C ABI.
struct mof_mesh {
    int32_t N = 0, M = 0, device = 0;
    // mof_mesh_prepare's per-mesh solver setup running on a host thread;
    // every call that may use what it builds waits for it first
    // (mof::mesh_join_prep). prep_mu guards prep and prep_err: a handle may
    // be cloned from several host threads while it is solved on; the
    // setup's error is kept for the calls that need the hierarchy
    std::mutex prep_mu;
    std::future<void> prep;
    std::exception_ptr prep_err;
    // rows [n_own, N) are a decomposed part's ghosts (mof_dd.h): the
    // multigrid preconditioner decouples them (identity rows); N otherwise
    int32_t n_own = 0;
    uint32_t flags = 0;
    hipStream_t stream = nullptr;
    mof::Pattern pat;
    // Internal vertex order: RCM unless MOF_NO_REORDER. perm[old] = new,
    // inv[new] = old; the API always speaks the caller's (old) order.
    std::vector<int32_t> perm, inv;
    // internal triangle order: tperm[internal] = caller's triangle index
    std::vector<int32_t> tperm, tinv;
    // irregular meshes: the internal ids in RCM order (the vertices are
    // degree-sorted within 256-row windows of it); the multigrid aggregation
    // visits them in this order. Empty: the internal order is the RCM order.
    std::vector<int32_t> agg_order;
    mof::DevArray<int32_t> perm_d;    // (N) old -> new, for the planar V gather
    mof::DevArray<int32_t> tri_orig;  // (M,3) caller's vertex ids, for gathers of I
    mof::DevArray<int32_t> icol;      // (N) internal vertex -> its column of the caller's I
    // device mesh data (internal order)
    mof::DevArray<int32_t> tri, vptr, vcol, cptr, clist, sell_off, sell_col, sell_blk, blk_row,
        diag_pos, tsell_off, tinc, tslot;
    mof::DevArray<int32_t> sell_mir;  // sell_mirror(pat, n_own): (re)uploaded by mesh_set_own
    int64_t blocks_read = 0;          // blocks an fp32 / bf16 operator pass reads per system
    bool sym_reads = false;           // the mirror table transposes lower blocks
    mof::DevArray<double> e, gw, iw, area, a2;  // a2: [sell_nb][4] (unscaled, bit-exact)
    // operator copies: lambda*a2 (cached per lambda) and A_T/12 with a zero slot M
    mof::DevArray<double> a2s64, w12_64;
    mof::DevArray<float> a2s32, w12_32;
    double a2s_lambda = 0.0;
    bool a2s_valid = false;
    // mof_assemble / mof_csr_export(MOF_CSR_A_LAST): one assembled A (SELL) and f
    mof::DevArray<double> Aexp, fexp;
    mof::Workspace ws;
    bool have_last_A = false;
    double ms_geometry = 0.0, ms_pattern = 0.0;
    // pinned host mirror of per-system flags
    int32_t *h_sysi = nullptr;
    double *h_sysd = nullptr;
    int32_t h_cap = 0;
    // HIP event pairs bracketing timed SpMV launches (MOF_TIME_SPMV)
    std::vector<hipEvent_t> spmv_events;
    // PCG iterations the previous batch needed, per (precision, outer step)
    std::vector<int32_t> iter_hint;
    // aggregation multigrid hierarchy (MOF_PRECOND_AMG), built on first use
    mof::AmgDevice *amg = nullptr;
    // host-pointer solves: pinned staging ring + copy stream, and two device
    // slots each for a batch's I rows and its planar V (double buffering);
    // events: [0..1] I rows uploaded, [2..3] I rows consumed by the assembly,
    // [4..5] V written
    mof::HostStage *stage = nullptr;
    mof::DevArray<double> hin[2], hout[2];
    // host state shared with the clones of this mesh on other devices
    std::shared_ptr<mof::MeshShared> shared;
    hipEvent_t hev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
};

namespace mof {

// kernels launched from the host side (mof_assemble.hip / mof_pcg.hip)
void launch_geometry(mof_mesh *m, const double *d_xyz, const double *d_nrm, bool f32_points);
void launch_a2(mof_mesh *m);
// lambda * a2 operator copies (cached per lambda)
void prepare_operator(mof_mesh *m, double lambda, hipStream_t s);
// per-timestep terms of B systems: u, f, D^-1. I0 / I1 rows are device
// pointers (row b at +b*ldI).
// amg: the multigrid preconditioner's hierarchy is built and sized for B
// (amg_build + amg_ensure): also write the level-0 bf16 smoother copies.
void launch_assemble(mof_mesh *m, int32_t B, const double *I0, const double *I1, int64_t ldI,
                     bool block_jacobi, uint32_t precision, hipStream_t s, bool amg = false);
// bit-exact A (SELL, fp64) and f of one timestep into m->Aexp / m->fexp
void launch_assemble_export(mof_mesh *m, const double *I0, const double *I1, double lambda,
                            hipStream_t s);
void launch_to_planar(mof_mesh *m, int32_t B, double *V, hipStream_t s);  // V in caller order
// find_singularity_points for K fields (mof_sing.hip); device pointers
void launch_singularities(int32_t N, int32_t M, int32_t K, const void *coords, bool f32, const int32_t *tri,
                          const double *V, double eps, double *vmax, uint8_t *vflag, uint8_t *tflag,
                          double *lam_mu, hipStream_t s);
// the same with the flagged vertices / triangles appended as records (SingList)
void launch_singularities_compact(int32_t N, int32_t M, int32_t K, const void *coords, bool f32,
                                  const int32_t *tri, const double *V, double eps, double *vmax, uint8_t *vflag,
                                  unsigned long long *cnt, int64_t cap, int2 *vrec, int2 *trec, double2 *tlm,
                                  hipStream_t s);
void launch_velocity_vectors(int32_t N, int32_t K, const double *e, const double *V, double *Vc,
                             double *speed, hipStream_t s);

// Timed SpMV launches: each is charged with the systems it actually
// processed (a system that converged, or failed, earlier in a chunk of
// launches returns at once and moves no block bytes).
// host time spent in the flag fetches of the solver (diagnostics)
extern thread_local double g_fetch_ms;
extern thread_local int64_t g_fetch_n;

struct SpmvTiming {
    int64_t launches = 0;
    int64_t systems = 0;         // systems processed, summed over the launches
    int64_t full_launches = 0;   // launches in which every system of the solve worked
    double ms = 0.0, bytes = 0.0;
    double ms_full = 0.0;        // their summed time
    int64_t fused_launches = 0;  // fused solves (k_solve_fused), one per batch ...
    double ms_fused = 0.0;       // ... and their summed time
};

// Algorithmic bytes of one k_pcg_spmv launch over `active` systems
// (Roofline).
double spmv_launch_bytes(const mof_mesh *m, uint32_t precision, int32_t active);

// a multigrid-preconditioned inner solve takes tens of iterations: one whose
// |r|^2 sets no new minimum for this many fails (its system goes to the
// recovery solves)
constexpr int32_t kPcgStall = 64;

struct SolveParams {
    uint32_t precision;
    bool block_jacobi;
    bool time_spmv;
    bool amg;  // mixed precision only: multigrid V-cycle preconditioner
    int32_t max_iter, max_outer;
    double rtol, inner_rtol;
    // error control: a system retires when its residual meets rtol AND its
    // estimated error max|d_k| |r_{k+1}| / |r_k| (times the safety factor
    // kErrSafety) is at most etol max|x64|; 0: the residual alone
    double etol = 0.0;
    // stagnation window: an inner solve whose |r|^2 sets no new minimum for
    // this many iterations fails (0: off; kPcgStall with the multigrid)
    int32_t stall = 0;
    // an inner solve that ends at max_iter unconverged fails the system
    // (instead of handing the partial correction to the next refinement step)
    bool fail_at_max_iter = false;
    // refinement steps after the first: per-system inner tolerance from the
    // outer residual still missing (k_pcg_tol)
    bool adaptive_inner = true;
    // the whole fp64 solve of a batch in one launch, one workgroup per system
    // (k_solve_fused): 0 never, 1 when the batch is eligible, -1 auto (small
    // meshes: row blocks <= kFusedMaxBlk)
    int32_t fused = -1;
    // > 0: the multigrid's fine-level smoother damping for this solve instead
    // of the hierarchy's (the recovery's damped multigrid pass)
    float amg_omega = 0.f;
};
// Wait for a pending mof_mesh_prepare on the handle (thread-safe). Its error
// stays on the handle; take_error rethrows (and clears) it -- the calls that
// need the multigrid hierarchy (the multigrid solve, mof_mesh_sync).
void mesh_join_prep(mof_mesh *m, bool take_error = false);
// The largest batch whose launch grids all stay within 2^32 - 1 work-items
// (xcd_grid refuses a larger one): the block-level assembly pass over the
// SELL slots of every system is the widest grid of a solve.
int32_t grid_batch_cap(const mof_mesh *m);
// Solve the B assembled systems in the workspace; fills sysd/sysi.
// Returns total inner iterations; sets *outer to the refinement steps used.
// only (B flags, optional): re-solve just these systems; the others keep
// their x64 and flags from the previous solve of the batch.
int64_t solve_batch(mof_mesh *m, int32_t B, const SolveParams &sp, hipStream_t s, int32_t *outer,
                    int32_t *max_iters, SpmvTiming *timing, const uint8_t *only = nullptr);
// Re-solve the failed systems of a solved batch (block Jacobi in the same
// precision after a multigrid solve, then fp64); mof_abi.cpp.
void recover_systems(int32_t nb, const SolveParams &sp, int32_t user_max_iter, const int32_t *sysi,
                     std::vector<uint8_t> &only, mof_stats &st, const std::function<void(uint32_t)> &ensure,
                     const std::function<int64_t(const SolveParams &, const uint8_t *)> &solve,
                     const std::function<void()> &release_f64);
// Operators a recovery solve needs that the first solve's assembly did not
// write: with MOF_PREC_MIXED the fp32 2x2 block-Jacobi inverses from the fp32
// A (the multigrid assembly keeps D^-1 in bf16 only); with MOF_PREC_F64 the
// fp64 A and D^-1 (from the u / f terms the assembly left in the workspace).
void launch_recovery_operator(mof_mesh *m, int32_t B, uint32_t precision, hipStream_t s);
// the fp64 A and per-triangle term arrays of a recovery pass, released (mof_assemble.hip)
void release_f64_terms(mof_mesh *m);
void ensure_workspace(mof_mesh *m, int32_t B, uint32_t precision);
// aggregation multigrid preconditioner (mof_amg.hip)
bool amg_build(mof_mesh *m);  // hierarchy from the mesh (once); false: mesh too small
void amg_ensure(mof_mesh *m, int32_t B);            // per-system storage
void amg_setup_batch(mof_mesh *m, int32_t B, hipStream_t s);  // Galerkin + coarse inverse
// z = V-cycle(r) on the fp32 inner vectors; writes partial r.z (component 0)
// into the part_rzrr slot `part_slot`
// zh: write z as a bf16 pair per vertex (uint32) instead of float2
// smap / nl: the launches cover the nl systems smap lists (the PCG's tail
// iterations), or all B when smap is null
void amg_vcycle(mof_mesh *m, int32_t B, const float *r, float *z, double *part_slot, int32_t nblk,
                const RedArgs &rd, hipStream_t s, bool zh, const int32_t *smap = nullptr, int32_t nl = 0);
// level-0 smoother data the PCG update / init write the pre-smoothing with
struct AmgFine {
    const void *A0h;  // bf16 level-0 operator [B][sell_nb] (its diagonal blocks give the smoother's D)
    int64_t sell_nb;
    const int32_t *sell_off;
    float *x0;        // smoother x
    float omega;
    bool smoothed;    // level 0 has the smoothed prolongator (irregular mesh)
    bool regular;     // tentative prolongator on a regular mesh (bf16 z is tuned for it)
};
AmgFine amg_fine(mof_mesh *m);
// bf16 level-0 A of the next batch, written by the assembly (marks it
// fresh, so amg_setup_batch does not convert A32 again)
struct AmgBf16 {
    uint2 *A0h;
};
AmgBf16 amg_bf16_targets(mof_mesh *m, int32_t B);
void amg_destroy(AmgDevice *g);

int32_t amg_levels(const mof_mesh *m);
// set the fine-level smoother damping of m's multigrid cycle; returns the
// previous value (0 and no change when m has no hierarchy)
float amg_set_omega(mof_mesh *m, float omega);

// every (row block, system) pair of the XCD order (mof_rowkern.h) visited once
bool xcd_map_covers(int32_t nblk, int32_t B, int32_t grp);
// xcd_batch_cap on the host (tests, via mof_xcd_batch_cap)
int32_t xcd_batch_cap_host(int64_t nblk, int32_t grp);
double bench_spmv(mof_mesh *m, uint32_t precision, int32_t B, int32_t reps, hipStream_t s,
                  double *bytes);

}  // namespace mof
