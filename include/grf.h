/*
 * grf.h -- C ABI of the MI355X (gfx950) Graph Random Features engine.
 *
 * Every compute entry point is asynchronous on the HIP stream it is given,
 * takes DEVICE pointers (allocated by the caller, e.g. torch tensors on
 * cuda:N), plain integer sizes and no C++ / torch types.  Return value:
 * GRF_OK (0) or a negative grf_status; the message of the last failure on
 * the calling thread is in grf_last_error().  No exception crosses the ABI.
 * Buffers whose size depends on the data are bounded by documented caps
 * (`*_cap` arguments) so that no entry point needs a host round trip.
 *
 * The reference has no FFI: its boundary is a set of Python functions
 * (SURVEY.md §8b).  Each entry point below replaces the reference routine
 * cited next to it (paths relative to the reference checkout).
 */
#ifndef GRF_H
#define GRF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *grf_stream_t; /* hipStream_t; NULL = default stream */

enum grf_status {
    GRF_OK = 0,
    GRF_EINVAL = -1,      /* bad argument (reference: ValueError / AssertionError) */
    GRF_EHIP = -2,        /* HIP runtime / launch failure                           */
    GRF_ECAPACITY = -3,   /* an output cap was too small                            */
    GRF_EUNSUPPORTED = -4 /* size outside what this build handles                   */
};

/* Record unit of the banded transpose (bytes per descriptor unit) */
enum grf_rec_unit {
    GRF_REC_LINE = 128,  /* every bucket starts on a 128-byte line: dense buckets (C4)      */
    GRF_REC_PACKED = 12, /* buckets packed pair after pair: sparse buckets (C5, N = 1M)     */
    GRF_REC_SLOT = 32    /* one 32-byte slot per bucket: {u32 pairs, u32 first overflow pair,
                            the first two pairs inline}, the rest packed after all the slots:
                            the Gram reads a small bucket with its header in ONE line
                            (grf_transpose_banded_self and the 8-wave Gram tiles only)           */
};

/* Laplacian semantics */
enum grf_laplacian_mode {
    GRF_LAP_SCIPY = 0,         /* utils_sparse/graph_utils.py:5-30  (D^-1/2 (D-A) D^-1/2, scipy order) */
    GRF_LAP_NUMPY = 1,         /* graph_kernels/utils.py:21-26      (I - D^-1/2 W D^-1/2, dinv=0 at deg<=0) */
    GRF_LAP_NUMPY_SAFE = 2,    /* preprocessing/laplacian_np.py:13-20 (safe degrees)                   */
    GRF_LAP_COMBINATORIAL = 3, /* preprocessing/laplacian_np.py:32-34 (D - W)                          */
    GRF_LAP_NONE = 4           /* walk the matrix as given (RandomWalk(Graph(adj)))                    */
};

enum grf_rng {
    GRF_RNG_PCG64 = 0, /* numpy PCG64 stream replay, one sequential stream per chunk (reference-exact) */
    GRF_RNG_PHILOX = 1 /* Philox4x32-10 keyed (seed), counter (step pair, walk, source, block)     */
};

enum grf_load_rule {
    GRF_LOAD_CUMULATIVE = 0,    /* load *= deg*w/(1-p)   sparse_sampler.py:54, sampler.py:58 */
    GRF_LOAD_NONCUMULATIVE = 1, /* load  = deg*w/(1-p)   sampler.py:183                      */
    GRF_LOAD_ABLATION = 2       /* load  = w             sampler.py:180-181                  */
};

enum grf_norm {
    GRF_NORM_DIV = 0,      /* value / m       (sampler.py:201)                          */
    GRF_NORM_MUL_RECIP = 1 /* value * (1/m)   (sparse_sampler.py:130 via scipy _mul_scalar) */
};

/* The ABI revision of this header: grf_version() returns it, and a binding must refuse a library whose
 * revision differs (argument lists, or -- ABI 7 -- the GRF_RNG_PHILOX stream, change between revisions;
 * ABI 8 added grf_phi_row_shifts_padded and grf_gram_sparse_cols_padded). */
#define GRF_ABI_VERSION 8

const char *grf_last_error(void);
int32_t grf_version(void);
/* number of HIP devices visible (0 if none); never fails */
int32_t grf_device_count(void);
/* select the device for subsequent calls on this host thread */
int32_t grf_set_device(int32_t device);

/* ------------------------------------------------------------------ Laplacian
 * Replaces efficient_graph_gp_sparse/utils_sparse/graph_utils.py:5-30
 * (get_normalized_laplacian, sparse) for mode GRF_LAP_SCIPY.
 * In : A (n x n CSR, canonical: sorted, no duplicates): a_ptr[n+1] (int64),
 *      a_idx[nnz] (int32), a_val[nnz] (float64).
 * Out: l_ptr[n+1], l_idx[l_cap], l_val[l_cap] with l_cap >= nnz(A) + n;
 *      deg[n], dinv[n] (float64, scratch + diagnostics).  Columns ascending. */
int32_t grf_laplacian_csr(int64_t n, const int64_t *a_ptr, const int32_t *a_idx, const double *a_val, int32_t mode,
                          int64_t *l_ptr, int32_t *l_idx, double *l_val, int64_t l_cap, double *deg, double *dinv,
                          void *workspace, size_t workspace_bytes, grf_stream_t stream);

size_t grf_laplacian_csr_workspace_bytes(int64_t n);

/* Replaces efficient_graph_gp/graph_kernels/utils.py:6-28 and
 * efficient_graph_gp/preprocessing/laplacian_np.py:3-35 followed by the
 * neighbour scan np.flatnonzero(L[row]) of random_walk_samplers/sampler.py:22-28.
 * In : W dense row-major n x n float64.  mode: NUMPY / NUMPY_SAFE / COMBINATORIAL / NONE.
 * Out: the walk matrix as CSR of its nonzeros (ascending columns), l_cap >= nnz. */
int32_t grf_laplacian_dense(int64_t n, const double *W, int32_t mode, int64_t *l_ptr, int32_t *l_idx, double *l_val,
                            int64_t l_cap, double *deg, void *workspace, size_t workspace_bytes, grf_stream_t stream);

size_t grf_laplacian_dense_workspace_bytes(int64_t n);

/* --------------------------------------------------------------------- walks
 * Replaces the walk loops of
 *   efficient_graph_gp_sparse/random_walk_samplers_sparse/sparse_sampler.py:26-56 and
 *   efficient_graph_gp/random_walk_samplers/sampler.py:30-61,148-186.
 * Walks on the CSR (g_ptr, g_idx, g_val).  Records visit slots
 *   slot_node[(s - src_begin) * L * m + l * m + w] (int32, -1 = no visit),
 *   slot_load[same]                                   (float64)
 * for sources s in [src_begin, src_end).
 * RNG GRF_RNG_PHILOX: key = seed (64 bit).  Any [src_begin, src_end).  Block (l / 2, w, s, 0) of
 *   Philox4x32-10 serves steps l = 2j, 2j + 1 of walk (s, w): the even step halts iff x0 < ceil(p 2^32)
 *   and takes neighbour Lemire(x1, deg), the odd step uses x2 and x3; a Lemire rejection of step l
 *   continues on blocks (l, w, s, 1), (l, w, s, 2), ...; the L-th recorded visit draws nothing.
 * RNG GRF_RNG_PCG64 : chunks = np.array_split(arange(n), n_chunks); chunk c is one
 *   numpy default_rng(seed + c) stream; [src_begin, src_end) must be a union of
 *   whole chunks (use grf_chunk_bounds). */
typedef struct grf_walk_params {
    int64_t walks_per_node; /* m                     */
    double p_halt;          /* p                     */
    int32_t max_walk_length;/* L                     */
    int32_t load_rule;      /* enum grf_load_rule    */
    int32_t rng;            /* enum grf_rng          */
    int32_t reserved;
    int64_t n_chunks;       /* PCG64 only            */
    uint64_t seed;          /* PCG64: chunk c seeded with seed + c; Philox: key */
} grf_walk_params;

int32_t grf_walk(int64_t n, const int64_t *g_ptr, const int32_t *g_idx, const double *g_val,
                 const grf_walk_params *params, int64_t src_begin, int64_t src_end, int32_t *slot_node,
                 double *slot_load, grf_stream_t stream);
/* grf_walk with the augmented walk matrix (grf_walk_aug of the same walk matrix; NULL: grf_walk):
 * each step is one dependent memory round trip instead of two; the same draws, bit-identical slots in
 * both RNG modes (the PCG64 replay's one lane per chunk is latency-bound on exactly that chain). */
int32_t grf_walk_ex(int64_t n, const int64_t *g_ptr, const int32_t *g_idx, const double *g_val, const void *g_aug,
                    const grf_walk_params *params, int64_t src_begin, int64_t src_end, int32_t *slot_node,
                    double *slot_load, grf_stream_t stream);

/* host helper: first source of chunk c (np.array_split boundaries) */
int64_t grf_chunk_bounds(int64_t n, int64_t n_chunks, int64_t c);

/* ------------------------------------------------------- per-step occupancy
 * Replaces the accumulate/normalise part of sparse_sampler.py:36-47,107-130 and
 * sampler.py:137-146,188-203: for every (source, step) the distinct visited nodes
 * (ascending) with value = (sum of loads in walk order) normalised by `norm`.
 * Out (padded rows, row capacity m): step_cnt[ns*L], step_idx[ns*L*m],
 * step_val[ns*L*m] at row (s_local * L + l).  Explicit zeros are kept. */
int32_t grf_steps(int64_t n_src, int64_t m, int32_t L, int32_t norm, const int32_t *slot_node,
                  const double *slot_load, int32_t *step_cnt, int32_t *step_idx, double *step_val,
                  grf_stream_t stream);

/* Dense (N, N, L) feature tensor of RandomWalk.get_random_walk_matrices
 * (sampler.py:188-203): out[(s * n_cols + j) * L + l] = step value; out must be
 * zero-filled by the caller. */
int32_t grf_steps_densify(int64_t n_src, int64_t m, int32_t L, int64_t n_cols, const int32_t *step_cnt,
                          const int32_t *step_idx, const double *step_val, double *out, grf_stream_t stream);

/* ------------------------------------------------------------------------ Phi
 * Replaces efficient_graph_gp_sparse/graph_kernels_sparse/fast_grf_kernel_general.py:47-52
 * (Phi = sum_l f_l M_l, exact zeros dropped; steps l < min(n_f, L)).
 * From padded step rows (grf_steps output).  Out: padded Phi rows with capacity
 * phi_cap >= min(m * L, n): phi_cnt[ns], phi_idx[ns*phi_cap], phi_val[ns*phi_cap]
 * (float64), and optionally phi_val32 (float32 copy, may be NULL). */
int32_t grf_phi(int64_t n_src, int64_t m, int32_t L, const int32_t *step_cnt, const int32_t *step_idx,
                const double *step_val, const double *f, int32_t n_f, int64_t phi_cap, int32_t *phi_cnt,
                int32_t *phi_idx, double *phi_val, float *phi_val32, grf_stream_t stream);

/* Fused slots -> Phi (no step rows), same result bit-for-bit as grf_steps + grf_phi.
 * Requires m * L <= 4096.  norm as in grf_steps. */
/* Philox walks of the sources [src_begin, src_end) straight to Phi rows in one kernel (the
 * visit slots never touch HBM): bit-identical to grf_walk (params->rng = GRF_RNG_PHILOX)
 * followed by grf_phi_fused.  Requires m * L <= 4096.
 * Optional (t_count != NULL): also count the banded transpose's buckets of the rows written,
 * t_count[((row - count_row0) / band_width) * n + col] += 1 -- pass the transpose workspace (zeroed)
 * and then grf_transpose_banded_plan(..., counted = 1, ...); phi_cap must not truncate rows.
 * count_row0 (<= src_begin) is the first row of the transposed matrix: 0 for all of Phi, src_begin
 * for a transpose of these rows alone (the column-block multi-GPU Gram). 
 * phi_val (float64) may be NULL when phi_val32 is given: only the float32 copy is written. 
 * Optional (g_aug != NULL, from grf_walk_aug on the same walk matrix, nnz < 2^32): each step of a
 * walk is one dependent memory round trip instead of two -- same draws, same Phi bits. */
int32_t grf_walk_phi(int64_t n, const int64_t *g_ptr, const int32_t *g_idx, const double *g_val, const void *g_aug,
                     const grf_walk_params *params, int64_t src_begin, int64_t src_end, int32_t norm, const double *f,
                     int32_t n_f, int64_t phi_cap, int32_t *phi_cnt, int32_t *phi_idx, double *phi_val,
                     float *phi_val32, int32_t *t_count, int64_t band_width, int64_t count_row0,
                     grf_stream_t stream);
/* The augmented walk matrix of grf_walk_phi (opaque to the caller): a 32-byte header, then one
 * record per entry e of the CSR walk matrix (g_ptr, g_idx, g_val) holding the target v, the row
 * start and row length of v and the weight g_val[e] -- 16 bytes ({v, row start, length} packed
 * into 64 bits, float64 weight) when the node ids, row starts and lengths fit 64 bits together,
 * else 32 bytes; one record per walk step either way.  grf_walk_aug_bytes(nnz) bytes (enough for
 * both), 32-byte aligned. */
int32_t grf_walk_aug(int64_t n, const int64_t *g_ptr, const int32_t *g_idx, const double *g_val, void *g_aug,
                     grf_stream_t stream);
size_t grf_walk_aug_bytes(int64_t nnz);
int32_t grf_phi_fused(int64_t n_src, int64_t m, int32_t L, int32_t norm, const int32_t *slot_node,
                      const double *slot_load, const double *f, int32_t n_f, int64_t phi_cap, int32_t *phi_cnt,
                      int32_t *phi_idx, double *phi_val, float *phi_val32, grf_stream_t stream);

/* --------------------------------------------------------- sparse utilities */
/* exclusive scan of int32 counts -> int64 row pointers out[n+1] */
int32_t grf_scan_counts(int64_t n, const int32_t *cnt, int64_t *out_ptr, void *workspace, size_t workspace_bytes,
                        grf_stream_t stream);
size_t grf_scan_workspace_bytes(int64_t n);
/* padded rows (row r at r*cap, cnt[r] entries) -> compact CSR using out_ptr from grf_scan_counts.
 * Any of the value arrays may be NULL. */
int32_t grf_compact_rows(int64_t n_rows, int64_t cap, const int32_t *cnt, const int64_t *out_ptr,
                         const int32_t *in_idx, const double *in_val, const float *in_val32, int32_t *out_idx,
                         double *out_val, float *out_val32, grf_stream_t stream);
/* grf_compact_rows (float values required) that also writes the rows' Gram shift statistics into
 * `stats` (grf_phi_row_shifts_workspace_bytes(n_rows) bytes) for grf_phi_row_shifts_stats. */
int32_t grf_compact_rows_stats(int64_t n_rows, int64_t cap, const int32_t *cnt, const int64_t *out_ptr,
                               const int32_t *in_idx, const double *in_val, const float *in_val32, int32_t *out_idx,
                               double *out_val, float *out_val32, void *stats, size_t stats_bytes,
                               grf_stream_t stream);

/* dst[dst_off[r] + i] = src[r * stride + i] for i < seg_len[r], r < n_seg (4-byte elements; lengths
 * and offsets are device arrays): the compaction of a fixed-stride all-gather of n_seg ranks'
 * CSR segments (the multi-GPU Phi gather, grf_amd/dist.py) without reading any size back. */
int32_t grf_concat_segments(int32_t n_seg, int64_t stride, const void *src, const int64_t *seg_len,
                            const int64_t *dst_off, void *dst, grf_stream_t stream);

/* Banded transpose for the Gram kernel: entries (j, k, v) of Phi (CSR rows j)
 * bucketed by (band = j / band_width, k):  bucket id b = band * n_cols + k.
 * A bucket is a run of 12-byte record PAIRS {u16 8 (j0 - band start), u16 8 (j1 - band start)
 * (low / high half of one word), f32 v0, f32 v1}, starting on a unit boundary (rec_unit =
 * GRF_REC_LINE: a 128-byte line; GRF_REC_PACKED: right after the previous bucket); an odd
 * bucket ends with the pad record (0, +0.0).  Two calls (and the Gram) take the same rec_unit:
 *   plan: t_desc[2 * (n_bands * n_cols + 1)] = per bucket {first unit, pairs}; the last
 *         entry holds the total unit count (lo, hi words).  counted = 1: the bucket counts
 *         are already in the workspace (from grf_walk_phi over all rows), skip counting.
 *   fill: t_rec (>= total units * rec_unit bytes, 128-byte aligned), t_maxabs[1] = max |Phi| and
 *         t_rowshift[n_rows]: the Gram kernel's per-row fixed-point scale 2^shift (every term
 *         < 2^51, the row's sum of |terms| < 2^62).
 * workspace >= grf_transpose_workspace_bytes(n_bands * n_cols), shared by both calls.
 * band_width <= 8192. */
int32_t grf_transpose_banded_plan(int64_t n_rows, int64_t n_cols, int64_t band_width, int32_t rec_unit,
                                  const int64_t *ptr, const int32_t *idx, uint32_t *t_desc, int32_t counted,
                                  void *workspace, size_t workspace_bytes, grf_stream_t stream);
int32_t grf_transpose_banded_fill(int64_t n_rows, int64_t n_cols, int64_t band_width, int32_t rec_unit,
                                  const int64_t *ptr, const int32_t *idx, const float *val, const uint32_t *t_desc,
                                  void *t_rec, int64_t t_rec_bytes, float *t_maxabs, int32_t *t_rowshift,
                                  void *workspace, size_t workspace_bytes, grf_stream_t stream);
size_t grf_transpose_workspace_bytes(int64_t n_buckets);
/* The same fill in two coalesced passes (entries binned by (band, 128-column region) into
 * `staging`, then each region's records built in LDS and written whole); band_width must be
 * a multiple of 64, nnz = ptr[n_rows].  Record order inside a bucket is unspecified in both
 * fills (the Gram's fixed-point sum does not depend on it). */
int32_t grf_transpose_banded_fill_staged(int64_t n_rows, int64_t n_cols, int64_t band_width, int32_t rec_unit,
                                         const int64_t *ptr, const int32_t *idx, const float *val,
                                         const uint32_t *t_desc, void *t_rec, int64_t t_rec_bytes, float *t_maxabs,
                                         int32_t *t_rowshift, void *workspace, size_t workspace_bytes, int64_t nnz,
                                         void *staging, size_t staging_bytes, grf_stream_t stream);
size_t grf_transpose_staging_bytes(int64_t n_rows, int64_t n_cols, int64_t band_width, int64_t nnz);

/* The staged transpose without a plan: no bucket counts from the walk (grf_walk_phi's t_count may
 * then be NULL) and no scan over every bucket.  Each (band, region) of the binning gets a slab of
 * record units bounded by its entry and bucket counts (one scan over the regions); its placing
 * workgroup counts its buckets in LDS, lays them out in the slab and writes their descriptors
 * t_desc (same meaning as the plan's: {first unit, pairs}; t_desc[nbk] = the slabs' total, an
 * upper bound of the units written).  Buckets stay in (band, column) order; unused slab tails are
 * never read.  t_rec >= grf_transpose_self_units_bound(...) * rec_unit bytes; workspace >=
 * grf_transpose_self_workspace_bytes; staging as for grf_transpose_banded_fill_staged.
 * t_split (NULL: none; else 16 bytes per bucket, 16-byte aligned, band_width <= 8192): every
 * bucket's entries are laid out by sub-band (the 8 row ranges of band_width / 8 rows, in order)
 * and t_split[b] holds 8 uint16 entry offsets, the entries of bucket b before each sub-band
 * (all 0 for a region too large for the LDS image: order unspecified there).  The symmetric
 * Gram entry points take it to start a diagonal tile's buckets at its row's sub-band. */
int32_t grf_transpose_banded_self(int64_t n_rows, int64_t n_cols, int64_t band_width, int32_t rec_unit,
                                  const int64_t *ptr, const int32_t *idx, const float *val, uint32_t *t_desc,
                                  void *t_split, void *t_rec, int64_t t_rec_bytes, float *t_maxabs, int32_t *t_rowshift,
                                  void *workspace, size_t workspace_bytes, int64_t nnz, void *staging,
                                  size_t staging_bytes, grf_stream_t stream);
size_t grf_transpose_self_workspace_bytes(int64_t n_rows, int64_t n_cols, int64_t band_width);
int64_t grf_transpose_self_units_bound(int64_t n_rows, int64_t n_cols, int64_t band_width, int32_t rec_unit,
                                       int64_t nnz);

/* ---------------------------------------------------------------------- Gram
 * Replaces `Phi @ Phi.T` of fast_grf_kernel_general.py:55 (sparse) and :39 (dense).
 * Sparse path: K[r, :] for rows r in [row_begin, row_end) of Phi (compact CSR,
 * float32 values) against the banded transpose of the FULL Phi (band_width equal
 * to the transpose's, multiple of 64, <= 8192; t_desc / t_rec / t_rowshift from the transpose).
 * K is float32, row-major with leading dimension ldk (>= n_total); K row
 * (r - row_begin) is written.  Each K entry is the fp32 rounding of the exact
 * int64 fixed-point sum of the exact products Phi[r,k]*Phi[j,k] (per-row
 * power-of-two scale), so K does not depend on summation order: it is
 * bit-reproducible run to run, across row splits and GPU counts. */
int32_t grf_gram_sparse(int64_t n_total, int64_t row_begin, int64_t row_end, const int64_t *ptr, const int32_t *idx,
                        const float *val, int64_t band_width, int32_t rec_unit, const uint32_t *t_desc,
                        const void *t_rec, const int32_t *t_rowshift, float *K, int64_t ldk, void *workspace,
                        size_t workspace_bytes, grf_stream_t stream);
/* device workspace of one grf_gram_sparse / grf_gram_sparse_sym call (reserved for a tile
 * work counter; this build does not touch it and accepts NULL) */
size_t grf_gram_workspace_bytes(void);

/* Whole K = Phi Phi^T on one device using its symmetry: the Gram kernel computes the tiles
 * K[i, band >= band(i)] (about half the work) and a mirror pass copies K[j, i] = K[i, j]
 * for band(j) > band(i).  Same arguments and per-entry values as grf_gram_sparse with
 * row_begin = 0, row_end = n_total, except that the mirrored entries carry the
 * fixed-point rounding of row i (K is exactly symmetric).  band_width multiple of 64.
 * t_split: the transpose's sub-band split (grf_transpose_banded_self) or NULL; with it a tile on
 * its row's own band fetches only the buckets' sub-bands from the row's on (the entries below the
 * diagonal it skips are the mirror's to write). */
int32_t grf_gram_sparse_sym(int64_t n_total, const int64_t *ptr, const int32_t *idx, const float *val,
                            int64_t band_width, int32_t rec_unit, const uint32_t *t_desc, const void *t_rec,
                            const void *t_split, const int32_t *t_rowshift, float *K, int64_t ldk, void *workspace, size_t workspace_bytes,
                            grf_stream_t stream);

/* The Gram half of grf_gram_sparse_sym alone: the tiles K[i, band >= band(i)] (the lower parts
 * of the diagonal band tiles are written too and are overwritten by the mirror), restricted to
 * the parts [part_begin, part_end) of the band-major tile sequence cut into n_parts equal parts
 * (0, 1, 1 = all).  All parts followed by grf_gram_mirror on one stream is grf_gram_sparse_sym;
 * split so that other work can be scheduled against the Gram's tail and the HBM-bound mirror. */
int32_t grf_gram_sparse_upper(int64_t n_total, const int64_t *ptr, const int32_t *idx, const float *val,
                              int64_t band_width, int32_t rec_unit, const uint32_t *t_desc, const void *t_rec,
                              const void *t_split, const int32_t *t_rowshift, float *K, int64_t ldk, int32_t part_begin,
                              int32_t part_end, int32_t n_parts, void *workspace, size_t workspace_bytes,
                              grf_stream_t stream);

/* grf_gram_sparse_upper whose tile write-out ADDS the rounded fixed-point sums to K instead of
 * storing them: K's entries on and above the diagonal must hold the dense part first (the hub
 * columns' MFMA Gram, grf_gram_dense_upper).  With the hub columns' buckets emptied from the
 * transpose (grf_transpose_drop_columns) and their entries in the dense panel (grf_hub_panel),
 * dense upper + this + grf_gram_mirror is K = Phi Phi^T within the fp32 K tolerance (the hub part is
 * an fp32 MFMA sum instead of the exact fixed-point one).  Same arguments as grf_gram_sparse_upper. */
int32_t grf_gram_sparse_upper_add(int64_t n_total, const int64_t *ptr, const int32_t *idx, const float *val,
                                  int64_t band_width, int32_t rec_unit, const uint32_t *t_desc, const void *t_rec,
                                  const void *t_split, const int32_t *t_rowshift, float *K, int64_t ldk, int32_t part_begin,
                                  int32_t part_end, int32_t n_parts, void *workspace, size_t workspace_bytes,
                                  grf_stream_t stream);

/* Wave shares by record pairs (skewed graphs, where a row's long buckets cluster in its column
 * order).  grf_gram_row_cuts: col_w[k] = the record pairs of column k over all n_bands bands of
 * the transpose (t_desc, after any hub drop), then for every row of Phi (ptr, idx) 8 cuts
 * row_cuts[8 row + s] = the first nonzero (offset in the row) whose prefix of column weights
 * reaches s / 8 of the row's total (s = 0: 0).  col_w: n_cols int32 scratch; row_cuts: 8 n_rows int32.
 * grf_gram_sparse_upper_ex: grf_gram_sparse_upper (add_k = 0) or _add (add_k = 1) whose tiles give
 * each wave the nonzeros between its cuts instead of equal counts; row_cuts NULL = the plain call.
 * K is bit-identical either way (integer sums).  Line / packed buckets only (not GRF_REC_SLOT).
 * Replaces nothing in the reference: scheduling only (the reference's Phi @ Phi.T,
 * efficient_graph_gp_sparse/graph_kernels_sparse/fast_grf_kernel_general.py:55). */
int32_t grf_gram_row_cuts(int64_t n_rows, const int64_t *ptr, const int32_t *idx, int64_t n_bands, int64_t n_cols,
                          const uint32_t *t_desc, int32_t *col_w, int32_t *row_cuts, grf_stream_t stream);
int32_t grf_gram_sparse_upper_ex(int64_t n_total, const int64_t *ptr, const int32_t *idx, const float *val,
                                 int64_t band_width, int32_t rec_unit, const uint32_t *t_desc, const void *t_rec,
                                 const void *t_split, const int32_t *t_rowshift, const int32_t *row_cuts, float *K,
                                 int64_t ldk, int32_t part_begin, int32_t part_end, int32_t n_parts, int32_t add_k,
                                 grf_stream_t stream);

/* Hub-column split (hub-heavy graphs: Enron, Facebook, power-law).  grf_hub_panel writes the entries
 * Phi[r, k] of the columns with hub_pos[k] >= 0 into the dense fp32 panel P[r, hub_pos[k]] (row-major,
 * n_rows x ldp, zeroed by the caller; int32 hub_pos[n_cols], -1 elsewhere).  grf_transpose_drop_columns
 * empties the buckets of the n_drop columns cols[] in all n_bands bands of a banded transpose
 * (t_desc as returned by grf_transpose_banded_*, n_cols = the transposed matrix's columns). */
int32_t grf_hub_panel(int64_t n_rows, const int64_t *ptr, const int32_t *idx, const float *val,
                      const int32_t *hub_pos, float *P, int64_t ldp, grf_stream_t stream);
int32_t grf_transpose_drop_columns(int64_t n_bands, int64_t n_cols, uint32_t *t_desc, const int32_t *cols,
                                   int32_t n_drop, grf_stream_t stream);

/* Column block of K against another row set: K[r - row_begin, 0 : t_rows] = sum_k Phi[r, k] Phi_B[:, k]
 * for the rows r in [row_begin, row_end) of Phi (CSR ptr/idx/val, n_cols columns), where Phi_B
 * (t_rows rows, the same n_cols columns) is given by its banded transpose (grf_transpose_banded_*
 * of Phi_B) and row_shift holds the fixed-point shifts of Phi's rows (grf_phi_row_shifts over all
 * of Phi).  With Phi_B = Phi[b:e] the block is K[:, b:e], entry for entry the row mode's K[r, b + j]
 * (bit-identical to grf_gram_sparse): the multi-GPU path in which each rank transposes only its
 * own rows.  band_width: a multiple of 64 in [64, 8192]; ldk >= t_rows.
 * sym_row0 >= 0 declares Phi_B = Phi[sym_row0, sym_row0 + t_rows) (inside [row_begin, row_end)):
 * the square K[B, B] is then computed on and above its diagonal only and mirrored (its entries
 * below the diagonal carry the upper entry's bits, as in grf_gram_sparse_sym); sym_row0 < 0: none. */
int32_t grf_gram_sparse_cols(int64_t n_cols, int64_t row_begin, int64_t row_end, const int64_t *ptr,
                             const int32_t *idx, const float *val, const int32_t *row_shift, int64_t t_rows,
                             int64_t sym_row0, int64_t band_width, int32_t rec_unit, const uint32_t *t_desc,
                             const void *t_rec, const void *t_split, float *K, int64_t ldk, void *workspace,
                             size_t workspace_bytes, grf_stream_t stream);
/* The Gram fixed-point row shifts of a CSR (n_rows rows; float values) and its max |value|
 * (*maxabs, device): the same rule and the same per-row summation order as the banded transpose's
 * t_rowshift / t_maxabs, so grf_gram_sparse_cols reproduces grf_gram_sparse's bits. */
size_t grf_phi_row_shifts_workspace_bytes(int64_t n_rows);
int32_t grf_phi_row_shifts(int64_t n_rows, const int64_t *ptr, const float *val, float *maxabs, int32_t *row_shift,
                           void *workspace, size_t workspace_bytes, grf_stream_t stream);
/* The same shifts from statistics grf_compact_rows_stats left in `stats` while compacting the rows
 * (one pass over the values fewer; identical bits). */
int32_t grf_phi_row_shifts_stats(int64_t n_rows, const void *stats, float *maxabs, int32_t *row_shift,
                                 grf_stream_t stream);
/* The same shifts of padded rows (ABI 8): row r's cnt[r] entries at val[r * cap ...) (grf_walk_phi's output, not
 * compacted); workspace as grf_phi_row_shifts'. */
int32_t grf_phi_row_shifts_padded(int64_t n_rows, int64_t cap, const int32_t *cnt, const float *val, float *maxabs,
                                  int32_t *row_shift, void *workspace, size_t workspace_bytes, grf_stream_t stream);
/* grf_gram_sparse_cols from Phi as padded rows (ABI 8): row r's cnt[r] entries at idx / val [r * cap, ...) for
 * every row r < row_end (grf_walk_phi's output over sources [0, row_end), not compacted), Phi_B's transpose in
 * GRF_REC_SLOT buckets, no symmetric square; the pipelined column-block kernel (bit-identical to the CSR path
 * on the compacted rows). */
int32_t grf_gram_sparse_cols_padded(int64_t n_cols, int64_t row_begin, int64_t row_end, int64_t cap,
                                    const int32_t *cnt, const int32_t *idx, const float *val, const int32_t *row_shift,
                                    int64_t t_rows, int64_t band_width, const uint32_t *t_desc, const void *t_rec,
                                    float *K, int64_t ldk, grf_stream_t stream);

/* Partial Gram over a slice of the inner dimension: K[r, :] = sum over k in [k_begin, k_end)
 * of Phi[r, k] Phi[:, k] (same fixed-point rule as grf_gram_sparse).  The partial Grams of
 * disjoint slices sum to K -- the "partial K + all-reduce" multi-GPU option. */
int32_t grf_gram_sparse_kslice(int64_t n_total, int64_t row_begin, int64_t row_end, int64_t k_begin, int64_t k_end,
                               const int64_t *ptr, const int32_t *idx, const float *val, int64_t band_width,
                               int32_t rec_unit, const uint32_t *t_desc, const void *t_rec,
                               const int32_t *t_rowshift, float *K, int64_t ldk, void *workspace,
                               size_t workspace_bytes, grf_stream_t stream);

/* The mirror pass of grf_gram_sparse_sym alone: K[j, i] = K[i, j] for every j > i.
 * max_workgroups <= 0: one workgroup per 64 x 64 block (fastest alone); > 0: at most that many
 * workgroups striding over the blocks, which leaves CU slots to work on another stream (1024 =
 * 4 per CU was best beside the next step's walks: tools/gpu_mirror_ab.sh). */
int32_t grf_gram_mirror(int64_t n, float *K, int64_t ldk, int64_t max_workgroups, grf_stream_t stream);

/* Dense path: K = A A^T for A float32 row-major [n x lda] (columns >= k_dim are zero padding;
 * lda % 16 == 0, A 16-byte aligned).  K float32 [n x ldk] (ldk % 4 == 0, K 16-byte aligned), exactly
 * symmetric: the 128 x 128 tiles on and above the diagonal on the fp32 MFMA
 * (v_mfma_f32_16x16x4f32 / 32x32x2f32), each written to both triangles.
 * Replaces efficient_graph_gp/graph_kernels/fast_grf_kernel_general.py:39 (Phi @ Phi.T). */
int32_t grf_gram_dense(int64_t n, int64_t k_dim, const float *A, int64_t lda, float *K, int64_t ldk,
                       grf_stream_t stream);
/* grf_gram_dense's tiles on and above the diagonal only, nothing mirrored: every K[i, j >= i] is
 * written, entries below the diagonal only where a diagonal tile covers them.  The hub part of the
 * hub-column split (grf_gram_sparse_upper_add adds the sparse part on top). */
int32_t grf_gram_dense_upper(int64_t n, int64_t k_dim, const float *A, int64_t lda, float *K, int64_t ldk,
                             grf_stream_t stream);
/* As grf_gram_dense, with a device workspace for split-K: when the tiles alone would leave CUs idle
 * (every tile for small n, the last tiles of a large n), a tile is cut into k-slices whose partial
 * tiles are summed in slice order (deterministic) by the last of them to finish.  workspace:
 * grf_gram_dense_workspace_bytes(n, k_dim) bytes, 256-byte aligned, ZERO on first use (its first
 * 4 KiB hold the tiles' tickets, which every call leaves zero; the layout does not depend on n or
 * k_dim, so one workspace serves calls of any size in stream order); NULL or a smaller workspace
 * runs unsplit. */
size_t grf_gram_dense_workspace_bytes(int64_t n, int64_t k_dim);
int32_t grf_gram_dense_ws(int64_t n, int64_t k_dim, const float *A, int64_t lda, float *K, int64_t ldk,
                          void *workspace, size_t workspace_bytes, grf_stream_t stream);
/* The same K on the bf16 matrix cores (ABI 6): A is split exactly into three bf16 planes (a = a0 + a1 +
 * a2), K = sum over the six plane products a_p b_q with p + q <= 2 on v_mfma_f32_32x32x16_bf16 (16x the
 * fp32 MFMA's rate), a0 b0 and the five corrections accumulated apart in fp32.  The dropped products
 * |a1 b2| + |a2 b1| + |a2 b2| are at most (2u^3 + u^4) |a b| = (2^-23 + 2^-32) |a b| per term (bf16 unit
 * roundoff u = 2^-8), so the error bound is the fp32 path's plus (2^-23 + 2^-32) sum_k |A_ik A_jk| for
 * normal planes (an entry within 2^16 of the bf16 subnormal range can also lose its plane 2)
 * (measured against fp64: tests/test_gpu_parity.py test_gram_dense_split_*).  Symmetry and determinism as
 * grf_gram_dense_ws; from 64 tile rows on (n > 8064) 256 x 128 items of 8 waves on stream-K (bits then differ
 * from the 128-tile decomposition's within the bound above; GRF_DENSE_WIDE=0 / 1 forces it off / on).  Finite inputs below 2^128 (1 - 2^-9)
 * in magnitude only: an entry whose sum involves an infinite or NaN value of A (or one that rounds to an
 * infinite bf16) is NaN, where grf_gram_dense_ws follows IEEE (+-inf where no 0 * inf occurs).  workspace (required):
 * grf_gram_dense_split_workspace_bytes(n, k_dim) bytes, 256-byte aligned, ZERO on first use (the ticket
 * block of grf_gram_dense_ws at the same place, then the partial tiles of either decomposition). */
size_t grf_gram_dense_split_workspace_bytes(int64_t n, int64_t k_dim);
int32_t grf_gram_dense_split(int64_t n, int64_t k_dim, const float *A, int64_t lda, float *K, int64_t ldk,
                             void *workspace, size_t workspace_bytes, grf_stream_t stream);
/* grf_gram_dense_upper on the split products (ABI 6): the hub-column split's panel. */
int32_t grf_gram_dense_split_upper(int64_t n, int64_t k_dim, const float *A, int64_t lda, float *K, int64_t ldk,
                                   grf_stream_t stream);
/* The split's three bf16 planes written once (ABI 7): P row r holds, per k-tile t of 16, 96 bytes at
 * r ldp + 96 t -- plane 0 of k = 16 t .. 16 t + 15 (bf16, k order), plane 1, plane 2 -- the planes
 * grf_gram_dense_split forms in registers for every staged k-tile.  ldp >= grf_planes_row_bytes(k_dim)
 * (= 96 ceil(k_dim / 16)), a multiple of 16.  grf_split_planes reads A (zero-padded to 16 ceil(k_dim / 16)
 * columns, as grf_gram_dense_split requires); grf_densify_padded_planes writes them straight from the walk's
 * padded rows (grf_densify_padded's arguments, n_cols = k_dim).  grf_gram_dense_planes: K = A A^T from them with
 * nothing but fragment reads and MFMAs in the k-loop, on grf_gram_dense_split's decomposition for the size (the
 * 256 x 128 wide workgroups from 64 tile rows on, GRF_DENSE_WIDE as there; else the 128-tiles with their k-slices)
 * and bit-identical to it wherever both take the same work items (the same planes, the same products in the same
 * order); workspace as grf_gram_dense_split's (grf_gram_dense_split_workspace_bytes, ZERO on first use). */
int64_t grf_planes_row_bytes(int64_t k_dim);
int32_t grf_split_planes(int64_t n, int64_t k_dim, const float *A, int64_t lda, void *P, int64_t ldp,
                         grf_stream_t stream);
int32_t grf_densify_padded_planes(int64_t n_rows, int64_t cap, int64_t n_cols, const int32_t *cnt, const int32_t *idx,
                                  const float *val, void *P, int64_t ldp, grf_stream_t stream);
int32_t grf_gram_dense_planes(int64_t n, int64_t k_dim, const void *P, int64_t ldp, float *K, int64_t ldk,
                              void *workspace, size_t workspace_bytes, grf_stream_t stream);

/* CSR (float32) -> dense float32 [n_rows x lda], zero filled. */
int32_t grf_densify(int64_t n_rows, const int64_t *ptr, const int32_t *idx, const float *val, float *out,
                    int64_t lda, grf_stream_t stream);
/* The same from padded rows (grf_walk_phi's output: row r's cnt[r] entries at idx / val [r * cap, ...),
 * columns < n_cols), with no compaction: every row written whole once (zeros included) through LDS.
 * lda % 4 == 0, lda >= n_cols, lda * 4 <= 160 KiB (one CU's LDS), out 16-byte aligned.  ABI v5.
 * Replaces the dense path's Phi = F f (efficient_graph_gp/graph_kernels/fast_grf_kernel_general.py:38)
 * handed to the Gram as a dense matrix. */
int32_t grf_densify_padded(int64_t n_rows, int64_t cap, int64_t n_cols, const int32_t *cnt, const int32_t *idx,
                           const float *val, float *out, int64_t lda, grf_stream_t stream);

/* -------------------------------------- GPflow surface: a dense (N, N, L) step tensor F
 * Replaces efficient_graph_gp/gpflow_kernels/general_kernel_fast_grf.py:74-77 and
 * diffusion_kernel_fast_grf.py:52-60 (Phi = F f by tf.linalg.matmul, K = Phi Phi^T) and the
 * modulator gradient TensorFlow takes through them.  F float64 [n][n][L] contiguous (the
 * RandomWalk.get_random_walk_matrices tensor, random_walk_samplers/sampler.py:188-203).
 * grf_dense_steps_phi: Phi[i, j] = sum_l F[i, j, l] f[l] (fp64, l ascending) -> phi64 [n x n]
 * (optional, NULL to skip) and the zero-padded fp32 image phi32 [n x lda32] (lda32 >= n) that
 * grf_gram_dense / grf_gram_dense_ws read as A.
 * grf_dense_steps_grad: grad[l] = sum_ij F[i, j, l] ((G + G^T) Phi)[i, j] for the upstream gradient
 * G [n x ldg] of L w.r.t. K = Phi Phi^T (fp64 MFMA GEMM with the reduction fused into its
 * epilogue; partials summed in a fixed order: deterministic).  workspace:
 * grf_dense_steps_grad_workspace_bytes(n, L) bytes. */
int32_t grf_dense_steps_phi(int64_t n, int32_t L, const double *F, const double *f, double *phi64, float *phi32,
                            int64_t lda32, grf_stream_t stream);
size_t grf_dense_steps_grad_workspace_bytes(int64_t n, int32_t L);
int32_t grf_dense_steps_grad(int64_t n, int32_t L, const double *F, const double *phi64, const double *G,
                             int64_t ldg, double *grad, void *workspace, size_t workspace_bytes,
                             grf_stream_t stream);

/* ------------------------------------------- K.v and the pathwise-conditioning CG
 * The step after the path: SparseGraphGP.predict
 * (efficient_graph_gp_sparse/models/sparse_grf_model.py:21-45) and the linear_cg it
 * calls (line 43; linear_operator 0.5 via gpytorch==1.11).  K = Phi Phi^T is never
 * formed: K_rows,cols V = Phi[rows] (Phi[cols]^T V).  Dense blocks are float32
 * row-major [rows x ld] with the S right-hand sides / samples as columns.
 * `row_map` (int32, optional) selects rows of Phi; NULL = rows 0..n-1. */

/* (Phi[row_map])^T as CSR: t_ptr[n_cols + 1] (int64), t_idx / t_val [nnz]; t_idx are positions in
 * row_map; every column lists them in ascending order (a stable radix sort by column of the entries
 * laid out in row order).  nnz: the entries of the selected rows, or any upper bound of them (then
 * t_ptr[n_cols] holds the real count and the tail of t_idx / t_val is unused): a caller sizing from
 * bounds reads nothing back to the host. */
int32_t grf_csr_transpose(int64_t n_sel, const int64_t *ptr, const int32_t *idx, const float *val,
                          const int32_t *row_map, int64_t n_cols, int64_t nnz, int64_t *t_ptr, int32_t *t_idx,
                          float *t_val, void *workspace, size_t workspace_bytes, grf_stream_t stream);
size_t grf_csr_transpose_workspace_bytes(int64_t n_sel, int64_t n_cols, int64_t nnz);

/* Y[r, :] = sum_e val[e] X[idx[e], :] over row row_map[r] (fp32, fixed summation order):
 * phi_test @ v, eps1 @ phi_train.T (sparse_grf_model.py:39-40, 45). */
int32_t grf_spmm_csr(int64_t n_out, const int64_t *ptr, const int32_t *idx, const float *val, const int32_t *row_map,
                     const float *X, int64_t ldx, int32_t n_rhs, float *Y, int64_t ldy, grf_stream_t stream);
/* the same with fp64 dense blocks and accumulation (A's fp32 values widened) */
int32_t grf_spmm_csr_f64(int64_t n_out, const int64_t *ptr, const int32_t *idx, const float *val,
                         const int32_t *row_map, const double *X, int64_t ldx, int32_t n_rhs, double *Y, int64_t ldy,
                         grf_stream_t stream);

/* linear_cg(A._matmul, rhs, tolerance) with A = Phi_t Phi_t^T + noise I, Phi_t = Phi[row_map]
 * (n_sys rows; t_* its transpose from grf_csr_transpose): sparse_grf_model.py:34, 43.
 * rhs / x: [n_sys x ld] fp32, n_rhs in [1, 256] columns solved together.  Same rule as
 * linear_cg: per-column normalisation, eps = stop_updating_after = 1e-10, stop after
 * iteration k >= min(10, max_iter - 1) once the mean residual norm < tolerance.
 * *iters_out (host pointer, may be NULL) receives the iterations run and resid_out (host,
 * n_rhs doubles, may be NULL) the final residual norms of the normalised systems (the
 * quantities the stopping rule averages); the call returns when they are (it polls a
 * device flag, so it synchronises the stream).
 * grf_cg_gram_solve keeps the reference's fp32 vectors and scalars; the _f64 variant
 * runs the same recurrence in fp64 (Phi's fp32 values widened).  linear_cg's
 * trajectory is sensitive to rounding once CG loses orthogonality (K + s2 I with
 * condition ~1e4 reaches the cg_tolerance after 24 iterations in fp64, 36 in fp32; in
 * fp64 a 1e-15 relative change of the rhs already moves the 11-iteration result by ~1e-3),
 * so the fp64 solve is the one that tracks the algorithm itself. */
int32_t grf_cg_gram_solve(int64_t n_sys, const int64_t *ptr, const int32_t *idx, const float *val,
                          const int32_t *row_map, int64_t n_cols, const int64_t *t_ptr, const int32_t *t_idx,
                          const float *t_val, double noise, const float *rhs, int64_t ld_rhs, int32_t n_rhs,
                          double tolerance, int32_t max_iter, float *x, int64_t ldx, void *workspace,
                          size_t workspace_bytes, int32_t *iters_out, double *resid_out, grf_stream_t stream);
int32_t grf_cg_gram_solve_f64(int64_t n_sys, const int64_t *ptr, const int32_t *idx, const float *val,
                              const int32_t *row_map, int64_t n_cols, const int64_t *t_ptr, const int32_t *t_idx,
                              const float *t_val, double noise, const double *rhs, int64_t ld_rhs, int32_t n_rhs,
                              double tolerance, int32_t max_iter, double *x, int64_t ldx, void *workspace,
                              size_t workspace_bytes, int32_t *iters_out, double *resid_out, grf_stream_t stream);
/* (covers both precisions) */
size_t grf_cg_workspace_bytes(int64_t n_sys, int64_t n_cols, int32_t n_rhs);

/* ------------------------------------------- the GPyTorch surface's feature algebra
 * Device-resident step matrices (one CSR per step: int64 row pointers, sorted int32 columns,
 * float32 values -- the preprocessor's torch CSR values) for
 * efficient_graph_gp_sparse/gptorch_kernels_sparse/sparse_grf_kernel.py:24-61 and
 * sparse_diffusion_kernel.py:74-96; K[x1, x2] = Phi[x1] Phi[x2]^T runs on the Gram kernels above
 * (grf_gram_sparse_cols), the modulator gradient on grf_csr_transpose + grf_spmm_csr + these. */

/* Phi = sum_l f_l M_l over L <= 64 step matrices (step_* are HOST arrays of L device pointers):
 * `phi = sum(mod_vec * mat for ...)` (sparse_grf_kernel.py:54-60).  Per entry the terms of the
 * steps holding it are summed in step order in fp64 (0.0 + first term, left to right), exact
 * zeros dropped.  Two passes: _count writes the row lengths (int32 [n_rows]; scan them with
 * grf_scan_counts), _fill writes the rows at phi_ptr (phi_val and/or phi_val32 may be NULL). */
int32_t grf_phi_steps_csr_count(int64_t n_rows, int32_t L, const int64_t *const *step_ptr,
                                const int32_t *const *step_idx, const float *const *step_val, const double *f,
                                int32_t n_f, int32_t *phi_cnt, grf_stream_t stream);
int32_t grf_phi_steps_csr_fill(int64_t n_rows, int32_t L, const int64_t *const *step_ptr,
                               const int32_t *const *step_idx, const float *const *step_val, const double *f,
                               int32_t n_f, const int64_t *phi_ptr, int32_t *phi_idx, double *phi_val,
                               float *phi_val32, grf_stream_t stream);

/* phi[x_idx] (sparse_grf_kernel.py:33-41): len[r] = nnz of row row_map[r] (NULL map: row r);
 * then, with out_ptr = grf_scan_counts(len), the rows copied contiguously. */
int32_t grf_csr_row_lengths(int64_t n_sel, const int64_t *ptr, const int32_t *row_map, int32_t *len,
                            grf_stream_t stream);
int32_t grf_csr_gather_rows(int64_t n_sel, const int64_t *ptr, const int32_t *idx, const float *val,
                            const int32_t *row_map, const int64_t *out_ptr, int32_t *out_idx, float *out_val,
                            grf_stream_t stream);

/* out[r] = A[rows_a[r]] . B[rows_b[r]] (sorted CSR rows, fp64 sum of the exact products,
 * deterministic order; NULL row maps = identity): `(phi_x1 * phi_x2).sum(dim=-1)` (:43-45), and
 * with A = M_l the diagonal's modulator gradient. */
int32_t grf_csr_rowdot(int64_t n_pairs, const int64_t *a_ptr, const int32_t *a_idx, const float *a_val,
                       const int32_t *rows_a, const int64_t *b_ptr, const int32_t *b_idx, const float *b_val,
                       const int32_t *rows_b, double *out, grf_stream_t stream);

/* out[r] = sum_e val[e] Z[idx[e] * ldz + r] over the entries e of row row_map[r]: one step matrix's
 * rows contracted with the columns of a dense Z (n_cols x ldz, fp32, ldz >= n_sel).  With
 * Z = Phi[x2]^T G^T this is the modulator gradient of K[x1, x2] = Phi[x1] Phi[x2]^T:
 * dL/df_l = sum_r (M_l[x1] Z)[r, r] + (the same with x1, x2 and G^T swapped). */
int32_t grf_csr_rows_dot_cols(int64_t n_sel, const int64_t *ptr, const int32_t *idx, const float *val,
                              const int32_t *row_map, const float *Z, int64_t ldz, double *out, grf_stream_t stream);

/* K (dense fp32 on the device, n_rows x n_cols, row pitch ldk) -> the scipy CSR the reference's sparse
 * entry point returns (graph_kernels_sparse/fast_grf_kernel_general.py:55: `Phi @ Phi.T`, float64
 * values, sorted columns, exact zeros absent).  _count: cnt[r] = nonzeros of row r; with
 * out_ptr = grf_scan_counts(cnt), _fill writes the int32 columns and the float64-widened values. */
int32_t grf_dense_to_csr_count(int64_t n_rows, int64_t n_cols, const float *K, int64_t ldk, int32_t *cnt,
                               grf_stream_t stream);
int32_t grf_dense_to_csr_fill(int64_t n_rows, int64_t n_cols, const float *K, int64_t ldk, const int64_t *out_ptr,
                              int32_t *out_idx, double *out_val, grf_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* GRF_H */
