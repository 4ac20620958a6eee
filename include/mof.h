/*
 * mof.h -- C ABI of libmofhip.so, the MI355X-native manifold optical-flow
 * solver (per-timestep FEM assembly + preconditioned CG on gfx950).
 *
 * Drop-in boundary for utils/compute_optical_flow.py of
 * SEU-dynamical-models/Manifold-based-optical-flow-method (reference @
 * 2025-10-31). Each entry point names the reference interface it replaces.
 *
 * Conventions
 *  - Every function returns int status: MOF_OK (0) or a negative MOF_E_*;
 *    mof_last_error() then describes the failure (thread-local string).
 *  - The caller owns every host buffer; the library owns the device buffers
 *    behind a mof_mesh handle.
 *  - One handle lives on one device. Calls on one handle are serialised by the
 *    caller; different handles may be driven from different host threads
 *    concurrently (ctypes releases the GIL).
 *  - Unknown ordering is the reference's planar one: x[i + N*alpha],
 *    alpha in {0,1} (compute_optical_flow.py:83-84,133-134).
 *  - Arrays are C-contiguous row-major: xyz/nrm (N,3), tri (M,3), I (T,N),
 *    e (N,2,3), grad_w (M,3,3), integral_wi_wj (M,2), V (K,2N).
 */
#ifndef MOF_H_
#define MOF_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version: bumped whenever a public struct or signature changes (2:
 * mof_stats grew recovered / recovered_f64 and the SpMV accounting fields,
 * mof_mesh_info blocks_read; mof_mesh_clone; 4: mof_opts.etol, mof_stats
 * max_err_est -- the refinement's error control; mof_mesh_info max_batch). A binding checks
 * mof_abi_version() == MOF_ABI_VERSION of the header it was built against:
 * the library writes whole structs, so a stale header would be overrun. */
#define MOF_ABI_VERSION 4

/* status codes */
#define MOF_OK 0
#define MOF_E_ARG (-1)        /* invalid argument / shape */
#define MOF_E_HIP (-2)        /* HIP runtime error (no device, OOM, fault) */
#define MOF_E_NOCONV (-3)     /* a system did not converge; its V is NaN-filled */
#define MOF_E_STATE (-4)      /* call out of order (e.g. export before assemble) */

/* mof_mesh_create flags */
#define MOF_GEOM_F32_POINTS 1u /* xyz holds float32 values: grad_w in float32
                                  arithmetic, as numpy does for pyvista's
                                  float32 points (S3…py:79, :238-255) */
#define MOF_NO_REORDER 2u      /* keep the caller's vertex order on the device
                                  (default: reverse Cuthill-McKee; results and
                                  every export are in the caller's order either
                                  way, bit for bit) */

/* mof_opts.precision */
#define MOF_PREC_F64 0         /* fp64 values + vectors, Jacobi-PCG */
#define MOF_PREC_MIXED 1       /* fp32 inner PCG, fp64 residual refinement */

/* mof_opts.flags */
#define MOF_IO_DEVICE 1u       /* I, I2 and V_out are device pointers on the
                                  handle's device (inputs resident in HBM) */
#define MOF_NO_BLOCK_JACOBI 2u /* scalar Jacobi instead of 2x2 block Jacobi */
#define MOF_TIME_SPMV 4u       /* bracket every PCG SpMV launch with HIP events
                                  (fills mof_stats.ms_spmv / spmv_bytes) */
#define MOF_PRECOND_AMG 8u     /* MOF_PREC_MIXED: aggregation-multigrid V(1,1)
                                  preconditioner for the inner PCG (built
                                  once per mesh; meshes of <= 64 vertices
                                  keep block Jacobi). Smoother damping:
                                  0.85 on the fine level, 1.05 on the coarse
                                  levels; the environment variable
                                  MOF_AMG_OMEGA=w0[,w1], read when the
                                  hierarchy is built, overrides them */
#define MOF_NO_RECOVERY 16u    /* systems whose solve fails (breakdown,
                                  divergence, stagnation, max_iter) are
                                  NaN-filled at once. Default: they are
                                  re-solved, alone, with the multigrid at a
                                  fine-level damping of 0.6 and with
                                  block-Jacobi PCG in the same precision
                                  (after a multigrid solve) and then in fp64 (an fp64 solve:
                                  once more in fp64 with block Jacobi when
                                  it ran without it or with max_iter below
                                  10^4), each with max(max_iter, 10^4)
                                  iterations and no stagnation test, and
                                  only a system all of these fail is
                                  NaN-filled -- spsolve is direct and always
                                  answers an SPD system
                                  (compute_optical_flow.py:147). The same in
                                  mof_dd_solve_range. A recovery pass whose
                                  fp64 workspace cannot be allocated leaves
                                  its systems NaN-filled (MOF_E_NOCONV)
                                  rather than failing the call */
#define MOF_SOLVE_FUSED 128u   /* MOF_PREC_F64: solve each batch in one launch,
                                  one workgroup per system (the eager
                                  kernels' bodies run row block by row block;
                                  bit-identical V, flags and iteration
                                  counts). Default: on for meshes of at most
                                  16 row blocks of 256 vertices, where the eager
                                  launches are latency-bound */
#define MOF_SOLVE_EAGER 256u   /* never the fused solve */

/* mof_csr_export which */
#define MOF_CSR_A2 0           /* smoothness matrix a2 (2N x 2N) */
#define MOF_CSR_A_LAST 1       /* A = a1 + lambda*a2 of the last mof_assemble */

typedef struct mof_mesh mof_mesh;

typedef struct mof_opts {
    uint32_t struct_size;  /* sizeof(mof_opts) */
    uint32_t precision;    /* MOF_PREC_* */
    uint32_t flags;        /* MOF_IO_DEVICE | MOF_NO_BLOCK_JACOBI | MOF_TIME_SPMV | MOF_PRECOND_AMG */
    int32_t batch;         /* timesteps solved together per launch (0: auto =
                              1024, fewer if device memory is short); a
                              host-pointer job of more than two batches runs
                              its first and last at a quarter of it (short
                              copy-pipeline fill and drain; V is the same for
                              any split) */
    int32_t max_iter;      /* PCG iterations per inner solve (0: 10000; 1000
                              with MOF_PRECOND_AMG, whose inner solves take
                              tens: more means a bad preconditioner, and
                              the system goes to the recovery solves) */
    int32_t max_outer;     /* refinement steps, MOF_PREC_MIXED (0: 10) */
    double rtol;           /* stop at ||f - A V||_2 <= rtol ||f||_2 (0: 1e-8) */
    double inner_rtol;     /* MOF_PREC_MIXED inner PCG tolerance (0: 1e-4) */
    void *stream;          /* hipStream_t to run on, NULL: the handle's own */
    double etol;           /* error control (ABI 4): a system also needs its
                              estimated error 2 max|d_k| |r_{k+1}| / |r_k|
                              (d_k the last refinement correction) to be at
                              most etol max|V| (0: 1e-7; < 0: residual only) */
} mof_opts;

typedef struct mof_stats {
    int64_t systems;          /* timesteps solved */
    int64_t iterations;       /* PCG iterations summed over systems */
    int32_t max_iterations;   /* largest per-system PCG iteration count */
    int32_t failed;           /* systems that did not converge (NaN-filled) */
    int32_t outer_steps;      /* refinement steps of the last batch */
    int32_t batches;          /* batches launched */
    double max_rel_residual;  /* max over systems of ||f - A V|| / ||f|| */
    double ms_assembly;       /* device time, HIP events on the solve stream */
    double ms_solve;
    int64_t spmv_launches;    /* MOF_TIME_SPMV: PCG SpMV launches timed */
    double ms_spmv;           /* MOF_TIME_SPMV: summed SpMV launch time */
    double spmv_bytes;        /* MOF_TIME_SPMV: summed algorithmic bytes of
                                 those launches (the batched CSR
                                 SpMV, B nnz s_v + 4 nnz + 4 (R+1) + B R (s_x+s_y)),
                                 each charged with the systems it processed
                                  */
    int64_t spmv_systems;     /* MOF_TIME_SPMV: systems processed, summed over
                                 the timed launches (a system that converged
                                 earlier in a chunk exits at once) */
    int64_t spmv_full_launches; /* MOF_TIME_SPMV: launches in which every
                                   system of the inner solve worked ... */
    double ms_spmv_full;      /* ... and their summed time */
    int32_t recovered;        /* systems the first solve failed and a recovery
                                 solve (block Jacobi, then fp64) solved */
    int32_t recovered_f64;    /* of those, solved by the fp64 recovery */
    int64_t fused_launches;   /* MOF_TIME_SPMV: fused solves (one per batch) ... */
    double ms_fused;          /* ... and their summed kernel time */
    double max_err_est;       /* max over systems of the error estimate
                                 max|d_k| |r_{k+1}| / |r_k| over max|V| (ABI 4) */
} mof_stats;

typedef struct mof_mesh_info {
    int32_t N, M;              /* vertices, triangles */
    int32_t device;
    int32_t nblocks;           /* vertex 2x2 blocks (= N + 2E on a closed mesh) */
    int64_t nnz_struct;        /* 4 * nblocks: structural nnz of a2 / A */
    int64_t sell_blocks;       /* blocks incl. SELL-64 padding */
    double ms_geometry;        /* one-time device geometry + a2 build */
    double ms_pattern;         /* one-time host pattern build */
    int64_t blocks_read;       /* distinct blocks one fp32 / bf16 operator pass
                                  reads per system: the diagonal and upper
                                  blocks (lower ones are read as transposes),
                                  = nblocks in a build without symmetric reads */
    int32_t max_batch;         /* the largest batch whose launch grids stay
                                  within 2^32 - 1 work-items; mof_solve_range
                                  never exceeds it (ABI 4) */
    int32_t pad_;
} mof_mesh_info;

/* Library / device queries. */
const char *mof_version(void);
int mof_abi_version(void);  /* MOF_ABI_VERSION the library was built with */
const char *mof_last_error(void);
int mof_device_count(int32_t *count);

/* Replaces compute_geometrical_quantities(coordinates, normals, triangles,
 * areas) (compute_optical_flow.py:27-97): builds on `device` the tangent
 * bases e, the hat-function gradients grad_w, integral_wi_wj, the block
 * sparsity pattern and the smoothness matrix a2. xyz/nrm (N,3), tri (M,3)
 * zero-based, area (M,). */
int mof_mesh_create(const double *xyz, const double *nrm, const int32_t *tri,
                    const double *area, int32_t N, int32_t M, int32_t device,
                    uint32_t flags, mof_mesh **out);
/* Another handle of the same mesh on `device` (one handle per GPU of a
 * timestep-sharded compute_velocity_field, :157-177): the source's host
 * state -- internal vertex order, block pattern, mirror table and every
 * multigrid hierarchy built so far (or later, by either handle) -- is shared,
 * not rebuilt; only the uploads and the per-mesh kernels run on `device`.
 * Results are bit-identical to a mof_mesh_create handle. Handles may be
 * cloned concurrently from different host threads. */
int mof_mesh_clone(const mof_mesh *src, int32_t device, mof_mesh **out);
int mof_mesh_destroy(mof_mesh *mesh);
/* Start the per-mesh setup that solves with `opts` need -- the multigrid
 * hierarchy of MOF_PRECOND_AMG + MOF_PREC_MIXED: host build and upload -- on
 * a host thread of the handle, and return at once (a no-op for other
 * options). The solves, mof_assemble, mof_mesh_clone and mof_mesh_destroy
 * wait for it; an error it met is returned by the next of them. The drop-in
 * starts it in compute_geometrical_quantities, a per-mesh call like the
 * reference's a2 build (compute_optical_flow.py:27-97). */
int mof_mesh_prepare(mof_mesh *mesh, const mof_opts *opts);
/* Wait for the handle's pending mof_mesh_prepare; its status. */
int mof_mesh_sync(mof_mesh *mesh);
int mof_mesh_get_info(const mof_mesh *mesh, mof_mesh_info *info);

/* Host copies of the geometric quantities compute_geometrical_quantities
 * returns (:97): e (N,2,3), grad_w (M,3,3), integral_wi_wj (M,2). Any pointer
 * may be NULL. */
int mof_geometry_export(mof_mesh *mesh, double *e, double *grad_w, double *iw);

/* CSR (2N x 2N, canonical: sorted columns) of a2 (MOF_CSR_A2, the lil matrix
 * of :49,83-93) or of the last assembled A (MOF_CSR_A_LAST, :144-146).
 * indptr has 2N+1 entries; indices/data need nnz_struct entries. With
 * drop_zeros != 0 exact zeros are removed, as lil and csr+csr do in the
 * reference. *nnz receives the entry count written. */
int mof_csr_export(mof_mesh *mesh, int32_t which, int32_t drop_zeros,
                   int32_t *indptr, int32_t *indices, double *data, int64_t *nnz);

/* The assembly half of worker(k, ...) (:100-146) for one timestep: builds
 * A = a1 + lambda*a2 and f from I0 = I_k[k], I1 = I_k_2[k+1] (host, N each)
 * and dt = t_k[k+1] - t_k[k]. f (2N,) host, may be NULL; A is kept for
 * mof_csr_export(MOF_CSR_A_LAST). */
int mof_assemble(mof_mesh *mesh, const double *I0, const double *I1, double dt,
                 double lambda, double *f);

/* Replaces compute_velocity_field(processes_num, time_steps, a2, grad_w, e,
 * integral_wi_wj, triangles, t_k, areas, lambda_, I_k, I_k_2) (:152-194)
 * for k in [k0, k1), and worker(k, ...) (:100-149) for k1 = k0 + 1:
 * V_out[k - k0] (2N,) solves (a1_k + lambda a2) V = f_k with I0 = I[k],
 * I1 = I2[k+1] (I2 == NULL: I2 = I), dt = t_k[k+1] - t_k[k].
 * I, I2: (T, N) f64; t_k: (T,) host f64; V_out: (k1-k0, 2N) f64.
 * Host or device pointers per opts->flags. opts may be NULL (defaults).
 * Systems that do not converge are NaN-filled and MOF_E_NOCONV is returned
 * after every other system has been solved (spsolve's MatrixRankWarning +
 * NaN result, scipy linsolve.py:287-289). stats may be NULL. */
int mof_solve_range(mof_mesh *mesh, const double *I, const double *I2,
                    const double *t_k, int32_t T, int32_t k0, int32_t k1,
                    double lambda, const mof_opts *opts, double *V_out,
                    mof_stats *stats);

/* Replaces S3's epilogue: find_singularity_point.process_V_k(V_k, e)
 * (find_singularity_point.py:28-69: V_coord[k][i] = V[k][i] e_i^0 +
 * V[k][i+N] e_i^1) and the speed V_c = sqrt(sum(V_coord**2, axis=2))
 * (S3…py:130-132), bit-identical to numpy. e (N,2,3), V (K,2N) planar,
 * V_coord (K,N,3), speed (K,N); either output may be NULL. Host pointers, or
 * device pointers with MOF_IO_DEVICE in flags (stream: hipStream_t or NULL).
 * Needs no mesh handle. */
int mof_velocity_vectors(int32_t device, const double *e, const double *V, int32_t N,
                         int32_t K, double *V_coord, double *speed, uint32_t flags,
                         void *stream);

/* find_singularity_points(coordinates, triangles, V_now,
 * eps) (find_singularity_point.py:140-189) for K velocity fields V_coord
 * (K,N,3) at once. coords (N,3) f64, or f32 with MOF_COORDS_F32 (pyvista
 * points; the triangle normal is then formed in float32 as numpy does);
 * triangles (M,3) int32. Outputs: vmax (K) = v_length_max (bit-identical),
 * vertex_flag (K,N) = |V_i/vmax| <= eps (bit-identical), triangle_flag (K,M)
 * = zero inside the triangle (has_zero_velocity_interior, skipped when a
 * corner is flagged) with its barycentric (lam, mu) in lam_mu (K,M,2) (the
 * reference's np.linalg.lstsq is restated by QR + 2x2 SVD: equal to
 * rounding). Host pointers, or device pointers with MOF_IO_DEVICE. */
#define MOF_COORDS_F32 32u      /* mof_singularities: coords are float32 */
int mof_singularities(int32_t device, const void *coords, const int32_t *triangles, int32_t N,
                      int32_t M, const double *V_coord, int32_t K, double eps, uint32_t flags,
                      void *stream, double *vmax, uint8_t *vertex_flag, uint8_t *triangle_flag,
                      double *lam_mu);

/* mof_singularities with the reference's list-shaped result
 * (find_singularity_point.py:156-189 returns the zero vertices and the
 * triangles holding a zero, not dense flags): per field k, n_vert[k] zero
 * vertices and n_tri[k] zero triangles; vert_idx / tri_idx / lam_mu (2 per
 * triangle) hold them field-major, ascending index within a field (compacted
 * on the device, so only the lists cross PCIe). cap = capacity of each list
 * (entries over all fields); totals[0..1] receives the vertex / triangle
 * counts, and MOF_E_ARG is returned when either exceeds cap. Host outputs;
 * coords / triangles / V_coord host, or device with MOF_IO_DEVICE. */
int mof_singularities_compact(int32_t device, const void *coords, const int32_t *triangles, int32_t N,
                              int32_t M, const double *V_coord, int32_t K, double eps, uint32_t flags,
                              void *stream, int64_t cap, int64_t *totals, double *vmax, int64_t *n_vert,
                              int32_t *vert_idx, int64_t *n_tri, int32_t *tri_idx, double *lam_mu);

/* ---- the S3 CSV files (host threads, no device) ------
 * mof_csv_write replaces the write of reshape_and_save_data
 * (compute_optical_flow.py:314-320, pd.DataFrame(data).to_csv(path)):
 * data (rows, cols) row-major f64, byte-identical to pandas' output (header
 * ",0,1,...", index column, Python float repr, NaN as an empty field).
 * mof_csv_shape / mof_csv_read replace load_potentials
 * (compute_optical_flow.py:203-207, pd.read_csv(path, header='infer',
 * index_col=0).values): the header line and index column are dropped, empty
 * fields and pandas' NA strings read as NaN, numbers are parsed exactly as
 * pandas' default float parser does (bit-identical values).
 * threads 0 = $MOF_IO_THREADS, else $OMP_NUM_THREADS, else all host cores
 * (at most 64). */
int mof_csv_write(const char *path, const double *data, int64_t rows, int64_t cols,
                  int32_t threads);
int mof_csv_shape(const char *path, int64_t *rows, int64_t *cols);
#define MOF_CSV_ROUND_TRIP 1u /* mof_csv_read: correctly rounded parse (pandas
                                  float_precision='round_trip') instead of
                                  pandas' default parser */
int mof_csv_read(const char *path, double *out, int64_t rows, int64_t cols, uint32_t flags,
                 int32_t threads);

/* ---- the S3 surface without pyvista (host) -----------
 * Replace pv.read(surface_path) and the attributes S3 takes from it
 * (S3…py:75-84): points (N,3) float32, triangles (M,3) int64 (faces
 * reshaped), point normals (N,3) float32 (vtkPolyDataNormals restated, or
 * the file's nx/ny/nz when present), cell areas (M,) float64
 * (compute_cell_sizes()['Area']). PLY: ascii and binary, triangle faces.
 * VTK is absent here: these restate its algorithms, parity unpinned. */
int mof_ply_info(const char *path, int64_t *n_vertices, int64_t *n_faces, uint32_t *has_normals);
int mof_ply_read(const char *path, float *points, int64_t *triangles, float *normals);
int mof_point_normals(const float *points, const int64_t *triangles, int64_t N, int64_t M,
                      float *normals);
int mof_cell_areas(const float *points, const int64_t *triangles, int64_t N, int64_t M,
                   double *areas);

/* Diagnostic (host only, no device): the multigrid hierarchy the solver would
 * build for this mesh in the caller's vertex order -- vertex adjacency, greedy
 * aggregation, tentative prolongators from e (N,2,3) -- for tests of the host
 * setup without a GPU. level_nodes[0..*n_levels) receives the node count of
 * each level (at most 16 levels); qtq_err the largest |Q^T Q - I| entry over
 * the level-0 aggregates (orthonormal prolongator columns); max_curl (ABI 4,
 * optional) the largest per-level median sigma_3 / sigma_1 of the aggregates'
 * near-null blocks -- the multigrid's criterion for smoothing level 1's
 * prolongator on a closed surface (>= 0.35: folds). */
int mof_amg_probe(const int32_t *tri, const double *e, int32_t N, int32_t M, int32_t *n_levels,
                  int32_t *level_nodes, double *qtq_err, double *max_curl);

/* Diagnostic (host only): checks that the XCD-aware workgroup order of the
 * row kernels -- nblk row blocks x batch systems, walked in groups of
 * `group` systems (0: all) -- visits every (row block, system) pair exactly
 * once. MOF_OK, or an error with mof_last_error() set. */
int mof_xcd_map_check(int32_t nblk, int32_t batch, int32_t group);
/* Diagnostic (host only): the largest batch whose XCD-ordered grid over nblk
 * blocks per system (groups of `group`) stays within 2^32 - 1 work-items --
 * the bound mof_solve_range's batch never passes (mof_mesh_info.max_batch). */
int mof_xcd_batch_cap(int64_t nblk, int32_t group, int32_t *batch);

/* ---- one timestep's system decomposed over P
 * vertex parts (stretch; timestep shards stay the throughput path) --------
 * A part owns vertices (both unknowns of each); its local mesh is every
 * triangle with an owned corner, in the caller's triangle order, so its rows
 * of A and f are the reference's (compute_optical_flow.py:100-146) bit for
 * bit. The PCG iterations run in lockstep: the SpMV operand's ghost rows are
 * exchanged before every product, the CG scalars are reduced over all parts
 * in one fixed order (every part takes the same decisions; V is deterministic
 * for a given partition and within the solve tolerance of mof_solve_range).
 * Preconditioner: 2x2 block Jacobi, or with MOF_PRECOND_AMG (mixed precision)
 * block Jacobi over the parts with each part's multigrid V-cycle on its owned
 * rows (ghost rows decoupled: the owned rows' Dirichlet problem). */
typedef struct mof_dd mof_dd;

typedef struct mof_dd_info {
    int32_t nparts;         /* P */
    int32_t local_parts;    /* parts this handle drives (P in-process, 1 per rank) */
    int32_t rank;           /* RCCL rank, -1 in-process */
    int32_t max_neighbours; /* most neighbour parts of any part */
    int32_t max_owned;      /* largest part (vertices) */
    int32_t pad_;
    int64_t ghost_rows;     /* ghost vertices summed over parts (halo volume) */
    int64_t send_rows;      /* rows sent per exchange, summed over parts */
    double ms_setup;        /* partition, plans and part meshes */
} mof_dd_info;

#define MOF_DD_ID_BYTES 128

/* Recursive coordinate bisection of the vertices into nparts parts of
 * floor/ceil(N/nparts) vertices (host): part (N). */
int mof_partition_rcb(const double *xyz, int32_t N, int32_t nparts, int32_t *part);

/* Host-only diagnostic of the halo plan of a partition: per part (nparts
 * entries each) owned vertices, ghost vertices, neighbour parts, local
 * triangles and rows sent per exchange. */
int mof_dd_plan_info(const int32_t *tri, int32_t N, int32_t M, int32_t nparts, const int32_t *part,
                     int32_t *n_own, int32_t *n_ghost, int32_t *n_nbr, int32_t *n_tri,
                     int64_t *n_send);

/* All nparts parts in this process on one device (in-process transport: halo
 * by one gather kernel, shared partial sums). part (N) NULL: RCB. Arguments as
 * mof_mesh_create (flags: MOF_GEOM_F32_POINTS, MOF_DD_STAGED). */
#define MOF_DD_STAGED 64u     /* mof_dd_create: exchange halos and gather V
                                  through the pack / copy / unpack kernels and
                                  segment layout of the RCCL transport (device
                                  copies instead of ncclSend/Recv): exercises
                                  that path on one GPU */
int mof_dd_create(const double *xyz, const double *nrm, const int32_t *tri, const double *area,
                  int32_t N, int32_t M, int32_t nparts, const int32_t *part, int32_t device,
                  uint32_t flags, mof_dd **out);

/* RCCL transport, one process (rank) per GPU and one part per rank: rank 0
 * makes the id, the caller broadcasts it (e.g. torch.distributed), every rank
 * calls mof_dd_create_rank with the same mesh and partition. Halo by
 * ncclSend/ncclRecv with the neighbour ranks, partial sums by ncclAllGather
 * (librccl is loaded at run time; $MOF_RCCL_LIB overrides its path). */
int mof_dd_unique_id(uint8_t *id /* MOF_DD_ID_BYTES */);
int mof_dd_create_rank(const double *xyz, const double *nrm, const int32_t *tri, const double *area,
                       int32_t N, int32_t M, int32_t nranks, const int32_t *part, int32_t rank,
                       const uint8_t *id, int32_t device, uint32_t flags, mof_dd **out);

/* Host-staged transport (no RCCL): the same one-part-per-rank plans, pack /
 * unpack kernels, segment order and all-gathers as the RCCL transport, with
 * every exchange staged through host memory and carried by the caller's
 * callbacks (e.g. torch.distributed over gloo). For hosts without RCCL
 * between the ranks' devices, and to run the per-rank path of a P-part
 * decomposition on one GPU (RCCL refuses two ranks on one device). Each
 * callback returns 0 on success and is called by every rank in the same
 * order. */
typedef struct mof_dd_transport {
    void *ctx;
    /* every rank passes `bytes` at send; recv (nranks * bytes) receives all
       contributions in rank order (send may alias its own slot of recv) */
    int (*allgather)(void *ctx, const void *send, void *recv, int64_t bytes);
    /* with each of the n peer ranks: send[k] (sbytes[k]) to peers[k] and
       receive rbytes[k] from it into recv[k] */
    int (*exchange)(void *ctx, int32_t n, const int32_t *peers, const void *const *send, const int64_t *sbytes,
                    void *const *recv, const int64_t *rbytes);
} mof_dd_transport;
int mof_dd_create_rank_host(const double *xyz, const double *nrm, const int32_t *tri, const double *area,
                            int32_t N, int32_t M, int32_t nranks, const int32_t *part, int32_t rank,
                            const mof_dd_transport *transport, int32_t device, uint32_t flags, mof_dd **out);
int mof_dd_destroy(mof_dd *dd);
int mof_dd_get_info(const mof_dd *dd, mof_dd_info *info);
/* Test hook (never read from the environment): the fp64 recovery pass's
 * workspace allocation reports a failure on rank `rank` of this handle's
 * solves (-1: off) -- exercises the ranks' agreement on a failed recovery. */
int mof_dd_test_fail_recovery_alloc(mof_dd *dd, int32_t rank);

/* mof_solve_range on the decomposed system (same arguments and results; with
 * RCCL every rank passes the same k-range and receives the whole V). */
int mof_dd_solve_range(mof_dd *dd, const double *I, const double *I2, const double *t_k,
                       int32_t T, int32_t k0, int32_t k1, double lambda, const mof_opts *opts,
                       double *V_out, mof_stats *stats);

/* Measurement helper for bench.py: launches the PCG SpMV kernel `reps` times
 * back to back on `batch` systems of the last solve's working set, timed with
 * HIP events on the handle's stream. Returns the mean launch time and the
 * algorithmic bytes one launch moves. */
int mof_bench_spmv(mof_mesh *mesh, uint32_t precision, int32_t batch, int32_t reps,
                   double *ms_per_launch, double *bytes_per_launch);

#ifdef __cplusplus
}
#endif
#endif /* MOF_H_ */
