// mof_dd.h -- domain-decomposed solve: one
// timestep's system split over P vertex parts, each part a mof_mesh built on
// its local mesh (owned vertices + one ring of ghosts), PCG iterations in
// lockstep with a halo exchange of the SpMV operand and cross-part reductions
// of the CG scalars.
//
// Two transports behind one solver loop (mof_pcg.hip, solve_batch_dd):
//  * in-process: all P parts in one process on one device (one stream); the
//    halo is one gather kernel over the ghost rows of every part and the
//    per-part partial sums live in one shared array (no copies);
//  * RCCL: one process per GPU, one part per rank; the halo is pack ->
//    ncclSend/ncclRecv with every neighbour (grouped) -> unpack, the partial
//    sums are ncclAllGather'ed in place. librccl is opened at run time.
// Either way every part reduces the same [P][B][nmax] partial records in the
// same order, so all parts take identical CG decisions, bit for bit.
#pragma once

#include <cstdint>
#include <vector>

#include "mof_internal.h"

namespace mof {

struct DdPart {
    int32_t n_own = 0, n_ghost = 0;
    std::vector<int32_t> l2g;        // (n_own + n_ghost) local row -> caller vertex
    std::vector<int32_t> tris;       // caller triangle ids with >= 1 owned corner, ascending
    std::vector<int32_t> nbr;        // neighbour parts, ascending
    std::vector<int32_t> recv_off;   // (|nbr|+1) ghost range received from each neighbour
    std::vector<int32_t> send_off;   // (|nbr|+1) ranges of send_idx per neighbour
    std::vector<int32_t> send_idx;   // owned local rows sent, in the receiver's ghost order
    std::vector<int32_t> ghost_src;  // (n_ghost) the owner's local row of each ghost
    int32_t n_loc() const { return n_own + n_ghost; }
};

struct DdPlan {
    int32_t P = 0, N = 0, M = 0;
    std::vector<int32_t> part;  // (N) owner part of every vertex
    std::vector<int32_t> g2l;   // (N) local row of every vertex in its owner part
    std::vector<DdPart> parts;
};

// Recursive coordinate bisection: P parts of floor/ceil(N/P) vertices.
void partition_rcb(const double *xyz, int32_t N, int32_t P, int32_t *part);
// Halo plan for a vertex partition; rank_key (optional, (N)) orders the rows
// inside a part (the global RCM position).
void build_dd_plan(const int32_t *tri, int32_t N, int32_t M, int32_t P, const int32_t *part,
                   const int32_t *rank_key, DdPlan &plan);

// mof_mesh construction shared with mof_mesh_create: perm (optional) fixes the
// internal vertex order (perm[caller] = internal; triangles are then sorted
// by their smallest internal vertex); tri_ids (optional, (M,3)) are the vertex
// ids the I gathers use (a part's global ids, so it reads the caller's I rows).
void mesh_build(mof_mesh *m, const double *xyz, const double *nrm, const int32_t *tri,
                const double *area, int32_t N, int32_t M, int32_t device, uint32_t flags,
                const int32_t *perm, const int32_t *tri_ids);

// rows >= nown are a part's ghost rows; re-uploads the SELL mirror table
void mesh_set_own(mof_mesh *m, int32_t nown);

struct RcclApi;  // mof_dd.hip

}  // namespace mof

// Opaque handle of mof_dd_* (include/mof.h).
struct mof_dd {
    int32_t N = 0, M = 0, P = 0, device = 0;
    uint32_t flags = 0;
    int32_t rank = -1;  // RCCL transport: this process's part; -1: in-process (all parts)
    mof::DdPlan plan;
    std::vector<mof_mesh *> parts;   // local parts: P (in-process) or 1 (RCCL)
    std::vector<int32_t> part_ids;   // global part id of each local part
    hipStream_t stream = nullptr;
    int32_t cap = 0, nmax = 0;       // systems / workgroups per part the partials hold
    mof::DevArray<double> part_pq, part_rzrr, part_rr0;  // [2][P][B][nmax] (x NV)
    int32_t test_oom_rank = -1;          // mof_dd_test_fail_recovery_alloc (tests only)
    int32_t nvmax = 0;                   // k_outer_update blocks of the largest part
    mof::DevArray<double> part_dx;       // [P][B][nvmax][2]: max|d|, max|x64| (error control)
    // in-process halo: one entry per ghost row of every part
    // {dst part, dst row, src part, src row}
    mof::DevArray<int4> halo;
    int64_t n_halo = 0;
    mof::DevArray<void *> vbase;     // (2P) per-part bases: z (inner PCG) then x64
    mof::DevArray<int32_t> nloc;     // (P) local rows per part
    mof::DevArray<int32_t> own_l2g;  // owned caller vertices of the local parts, concatenated
    std::vector<int64_t> own_off;    // offset of each local part in own_l2g
    // RCCL transport (rank >= 0)
    mof::RcclApi *nccl = nullptr;
    void *comm = nullptr;
    // host-staged transport (rank >= 0, mof_dd_create_rank_host): the caller's
    // callbacks over host staging buffers
    bool hosted = false;
    mof_dd_transport host{};
    std::vector<char> hsend, hrecv;
    // pack -> exchange -> unpack (RCCL, or in-process with MOF_DD_STAGED):
    // entries {row, segment offset, segment rows, -} of the local parts,
    // concatenated; part l's entries start at send_base[l] / recv_base[l] and
    // its buffer region at 2 * cap * send_base[l] elements
    mof::DevArray<int4> send_ent, recv_ent;
    std::vector<int64_t> send_base, recv_base;
    mof::DevArray<double> sendbuf, recvbuf;  // [B][rows][2] per neighbour segment (fp64 sized)
    mof::DevArray<double> vgather;      // [P][B][nmax_own][2] owned V of every part
    int32_t nmax_own = 0;
    mof::DevArray<int32_t> all_l2g;     // [P][nmax_own] owned caller vertices (-1: none)
    mof::DevArray<double> agree;        // (P) one status word per rank (dd_all_ok), allocated at setup
    double ms_setup = 0.0;
};

namespace mof {

void dd_ensure(mof_dd *d, int32_t B, uint32_t precision);
// One batch of B assembled systems: mixed (fp32 inner + fp64 refinement) or
// fp64 block-Jacobi PCG over all parts; returns summed inner iterations.
// only (B flags, optional): re-solve just these systems from x = 0; the
// others keep their solution and flags (the recovery passes).
int64_t solve_batch_dd(mof_dd *d, int32_t B, const SolveParams &sp, hipStream_t s, int32_t *outer,
                       int32_t *max_iters, const uint8_t *only = nullptr);
// transport hooks (mof_dd.hip)
void dd_sync_partials(mof_dd *d, double *base, size_t per_part, hipStream_t s);
// refresh the ghost rows of every local part's z (which = 0; fp32 when f32) or
// x64 (which = 1)
void dd_halo(mof_dd *d, int32_t B, bool f32, int which, hipStream_t s);
// planar V (B, 2N) in the caller's order from the owned rows of all parts
void dd_gather_v(mof_dd *d, int32_t B, double *V, hipStream_t s);
// true on every rank iff `ok` on every rank (one all-gather of a status
// word; in-process: `ok`). Used where one rank can fail alone (a workspace
// allocation) before collectives every rank must enter.
bool dd_all_ok(mof_dd *d, bool ok, hipStream_t s);
double dd_all_min(mof_dd *d, double mine, hipStream_t s);

}  // namespace mof
