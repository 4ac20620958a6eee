// mof_amg.h -- aggregation multigrid preconditioner (host hierarchy + device levels).
#pragma once

#include <deque>

#include "mof_internal.h"

namespace mof {

struct AmgParams {
    int32_t max_levels = 10;
    int32_t max_coarse_dofs = 128;  // coarsest level: dense inverse in LDS (fp64), one workgroup per system
    float omega = 0.85f;            // damped block-Jacobi smoother, fine level (1.0 diverges on irregular meshes)
    // coarse levels' 3x3 block-Jacobi smoother: C3 / C2 / C5 / R3 PCG its per
    // timestep 19 / 23.4 / 16.5 / 110 at 0.85, 18 / 22.8 / 16 / 102 at 1.0,
    // 17.2 / 21.8 / - / 102.3 at 1.05, 17 / 21.5 / 15.2 / 104.6 at 1.1;
    // 1.2 diverges on R3
    float omega1 = 1.05f;
    // level-0 rows >= nown are a decomposed part's ghosts: the Galerkin lists
    // use an identity block on their diagonal and zero for every coupling
    // that touches them (the Dirichlet problem of the owned rows); -1: none
    int32_t nown = -1;
    // smoothed aggregation at level 0: P = (I - w D^-1 a2) P_tent with the
    // mesh's a2 (per mesh: D^-1 (lambda a2) does not depend on lambda, and
    // the per-timestep a1 is left out). 1 on, 0 off, -1 auto: on for
    // irregular meshes (vertex valence standard deviation > 0.5: the random
    // hull R3 1.33, icospheres <= 0.14). CPU prototype (tools/amg_proto.py,
    // PCG its to 1e-4): R3 40 -> 18, C3 8 -> 6 for 7.5x the level-0 Galerkin
    // terms and a level-1 operator with 2x the blocks per row.
    int32_t smooth = -1;
    float smooth_omega = 0.66f;
    // smoothed aggregation at level 1 (the transition 1 -> 2), with the
    // Galerkin image P0^T a2 P0 of the mesh's a2 (per mesh, fp64 on the
    // host): P1 = (I - w D1^-1 a2_1) P1_tent. 1 on, 0 off (amg_build's
    // auto choice: folded closed surfaces); applied when level 1 has more
    // than kSubNodes nodes (the fused tiny levels keep the tentative
    // transfers). CPU prototype (tools/amg_proto.py sa1a2=0.66 sa1only=1,
    // PCG its to 1e-4): the two-grid bound with an exact level-1 solve is 8
    // its on F3 and 7 on C3, the V-cycle 18 / 8 -- the recursion below level
    // 1 was F3's weakness; with P1 smoothed 12 / 7 (C3 with the GPU's
    // storage formats: 8 / 8).
    int32_t smooth1 = 0;
    const double *a2 = nullptr;  // [sell_nb][4] level-0 a2 in the fine SELL layout (smoothing)
    // the fine level's mirror table when its operators are read symmetrically
    // (sell_mirror): level-0 gather entries of lower blocks then point at the
    // transposed upper block (| kMirT), which is all the assembly writes
    const int32_t *mirror = nullptr;
    // level-0 aggregation visit order (internal node ids), or null: node
    // order. A mesh renumbered within windows (mesh_prepare_host) passes its
    // RCM order, so the aggregates are the RCM-ordered mesh's.
    const int32_t *order = nullptr;
};

// One level of the hierarchy. Level 0 is the fine mesh (bs = 2); coarser
// levels have 3 dofs per node. The transition fields (agg ... gent) describe
// the restriction to the next level and are empty on the coarsest level.
// levels of at most this many nodes run fused in one launch per cycle
// (k_subcycle) with the tentative transfers
constexpr int32_t kSubNodes = 512;

struct AmgLevel {
    int32_t n = 0, bs = 0;
    std::vector<int32_t> vptr, vcol;               // block adjacency (self included, sorted)
    std::vector<int32_t> sell_off, sell_col, sell_blk, diag_pos;  // SELL-64 block layout
    std::vector<int32_t> sell_row;                 // row of each SELL position
    std::vector<uint8_t> dead;                     // (n*3) dofs without a prolongator column
    // transition to level + 1
    std::vector<int32_t> agg;                      // (n) aggregate of each node
    std::vector<int32_t> mptr, mlist;              // aggregate members, CSR
    std::vector<int32_t> apos;                     // (n) position of node i in mlist
    std::vector<float> Q;                          // (n, bs, 3) tentative prolongator rows
    std::vector<float> Qm;                         // the same rows in member (mlist) order
    std::vector<int32_t> gptr;                     // (next sell_nb + 1) Galerkin gather ranges
    std::vector<int32_t> gent;                     // triples {fine SELL pos (| kMirT: transposed), P block of i, P block of j}
    // as the target of a product (level >= 1): the lower blocks' SELL
    // positions and their upper twins' (the products cover the diagonal and
    // upper blocks and write each lower twin as the transpose, st_pair)
    std::vector<int32_t> low, twin;
    // smoothed prolongator (level 0 with AmgParams::smooth): P rows as blocks
    // (bs x 3 floats each, in Q) with CSR pptr / pcol over the fine nodes, and
    // the restriction lists per coarse node: pairs {fine node, P block}. The
    // tentative prolongator is the special case pptr = 0..n, pcol = agg.
    bool smoothed = false;
    std::vector<int32_t> pptr, pcol, rptr, rent;
    // level 1 (host build only): the Galerkin image of the mesh's a2, 9
    // doubles per adjacency block (vptr / vcol order), for its smoothing
    std::vector<double> a2img;
    int64_t sell_nb() const { return sell_off.empty() ? 0 : sell_off.back(); }
};

struct AmgHierarchy {
    std::vector<AmgLevel> levels;
    int32_t coarse_dofs = 0;
    // per transition l -> l+1: the median over the aggregates of
    // sigma_3 / sigma_1 of the stacked near-null block (how much the tangent
    // planes turn inside an aggregate; 0 on a flat one), and the largest of
    // these over transitions with >= 64 aggregates (amg_build's level-1
    // smoothing choice, kFoldCurl)
    std::vector<double> curl;
    double max_curl = 0.0;
    bool folded = false;  // amg_build's auto choice rebuilt it with level 1 smoothed
};

// the fold criterion on AmgHierarchy::max_curl (amg_build): F3 0.46-0.51, the
// jittered spheres 0.13 (C2) / 0.25 (C3) / 0.41 (C5: the 0.5 % jitter is
// rough against a 640k mesh's edges), R3 0.09, S1 0.03
constexpr double kFoldCurl = 0.35;
// ... and level 0's too when the finest aggregates' median turn is below
// this (folded, not rough: F3 0.07, C3 0.20, C5 0.34)
constexpr double kFlatCurl = 0.15;

void build_amg(const Pattern &fine, const double *e_internal, const AmgParams &prm,
               AmgHierarchy &H);
// deterministic per-mesh choice of AmgParams::smooth = -1
bool amg_auto_smooth(const Pattern &fine);

// Device copy of a level. Level 0 borrows the mesh's SELL arrays and the
// inner solver's A32 / dinv32 / r / z; it owns only its smoother scratch.
struct AmgDevLevel {
    int32_t n = 0, bs = 0;
    int64_t sell_nb = 0;
    DevArray<int32_t> sell_off, sell_col, sell_row, diag_pos;  // level >= 1
    DevArray<uint8_t> dead;                          // level >= 1
    DevArray<int32_t> agg, mptr, mlist, apos, gptr, gent;  // transition to level + 1
    DevArray<int32_t> rgrp;                         // restriction groups (aggregate ranges)
    DevArray<int32_t> ggrp;                         // Galerkin groups for the products by entry: coarse
                                                    // position ranges [p0, p1) of <= kWG gather entries
    DevArray<int32_t> gbig;                         // levels >= 1: positions past kGalBig entries, one
                                                    // workgroup each (k_galerkin3_big)
    int32_t nbig = 0;
    bool smoothed = false;                          // level 0: smoothed prolongator
    DevArray<int32_t> pptr, pcol, rptr, rent;
    DevArray<int32_t> rperm;                        // smoothed P: restriction group entries by fine node
    DevArray<int32_t> twin;                         // level >= 1: each upper block's lower twin position, or -1
    int32_t ngrp = 0, nggrp = 0;
    DevArray<float> Q, Qm;
    // per system, capacity AmgDevice::cap
    DevArray<float> A;           // [B][sell_nb][12] (level >= 1)
    DevArray<uint32_t> Dh;       // [B][n][4] 3x3 D^-1 bf16 entries 0..7 (level >= 1)
    DevArray<uint16_t> Dh22;     // [B][n] entry (2,2)
    DevArray<uint32_t> Ah;       // sweep copy (not the coarsest), st_a9: [B][sell_nb][2] int8 codes 0..7
    DevArray<uint16_t> Ah22;     // [B][sell_nb][2] code 8 | bf16 scale (MOF_COARSE_I8=0: [4] / [1] bf16)
    DevArray<float> slab;        // level 1 of a smoothed level 0: one system slab's A as
                                 // [sell_nb][64][12] (k_galerkin_sys<2> -> <3>)
    DevArray<float> b, x, r, y;  // [B][n][4] (level >= 1); level 0: x [B][n][2], r bf16 pairs [B][n]
                                 // r is stored in member order of the next level
};

struct AmgDevice {
    bool built = false;
    int32_t cap = 0;
    int32_t nc = 0;  // coarsest dofs (dense)
    float omega = 0.85f, omega1 = 1.05f;
    int32_t xm = 2;  // level 0's corrected iterate: 1 in the x0 format in place, 2 fp32 in lv[0].y
    bool regular = false;  // tentative prolongator on a regular mesh: the bf16 iterates and omega1 1.1
    // (one block-Jacobi sweep per side on the coarse levels; 2 measured in
    // round 5, profiles/r05_ab/nu1/: fewer its, fewer timesteps/s but on F3)
    // open surfaces: extra level-0 sweeps on the boundary rows and their
    // neighbour ring (k_bsweep); bsw_n rows (0: none), bsw_pos[N] = the row's
    // index in bsw_rows or -1
    // (k_bsweep: the ring as its own SELL-64 matrix, mof_amg.hip)
    int32_t bsw_n = 0, bsw_sweeps = 0, bsw_N = 0, bsw_nout = 0, bsw_nslot = 0;
    DevArray<int32_t> bsw_rows, bsw_roff, bsw_wrow, bsw_xsrc, bsw_bsrc, bsw_ocol;
    DevArray<uint32_t> bsw_A;  // [cap][bsw_nslot] bf16 blocks (uint2), per batch
    std::deque<AmgDevLevel> lv;  // deque: DevArray is not movable
    DevArray<float> cinv;  // [B][nc][nc] coarsest inverse
    DevArray<uint32_t> A0h;  // [B][sell_nb][2] level-0 A in bf16 (smoother sweeps)
    // smoothed level 0: one slab of 64 systems' level-0 blocks as
    // [sell_nb][64] float4 (fp32 A), or uint2 (the bf16 sweep copy's, on
    // regular meshes) (k_a_slab -> k_galerkin_sys<2>), reused slab by slab
    DevArray<float> aslab;
    bool bf16_fresh = false;  // A0h written by the batch's assembly
};

}  // namespace mof
