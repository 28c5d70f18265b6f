/*
 * maxk_hip.h -- C ABI of the MI355X-native MaxK-GNN aggregation hot path
 * (libmaxk_hip.so, built from spgemm-prunning_amd/csrc for gfx950).
 *
 * Plain pointers and sizes only.  Every device pointer is caller-owned device
 * memory; every launch goes on the caller's stream (a hipStream_t passed as
 * void*; NULL = the default stream).  Launch functions never allocate, copy to
 * the host or synchronise, so they can be captured into a hipGraph; the setup
 * helpers marked "synchronous" do.
 *
 * Return value: MAXK_OK (0) or a negative MAXK_ERR_*; maxk_last_error() then
 * holds a message for the calling thread.
 *
 * Layouts (all row-major, C-contiguous):
 *   CSR     row_ptr int32 [num_rows+1], col_idx int32 [num_e] (< num_cols),
 *           edge_val f32 [num_e]
 *   CBSR    cbsr_val f32 [num_cols, k], cbsr_idx u8 [num_cols, k] (< dim_origin)
 *   dense   f32 [rows, dim_origin]
 *   warp4   int32 [W, 4] = (row, loc, len, 0)
 * Limits: 1 <= k <= dim_origin <= 256 (the selector is uint8).
 */
#ifndef MAXK_HIP_H_
#define MAXK_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MAXK_OK 0
#define MAXK_ERR_INVALID (-1)  /* bad argument (shape, null pointer, k/D range, workspace) */
#define MAXK_ERR_HIP (-2)      /* a HIP runtime call or launch failed */
#define MAXK_ERR_NODEVICE (-3) /* no HIP device visible */
#define MAXK_ERR_LIBRARY (-4)  /* rocSPARSE failure (baseline only) */

/* ABI version (major*100 + minor). */
int maxk_version(void);

/* Message for the last failing call on this thread ("" if none). */
const char *maxk_last_error(void);

/* Number of visible HIP devices (0 without a GPU; never fails). */
int maxk_device_count(void);

/* First 16 hex digits of the SHA-256 of the sources this library was built from
 * (spgemm-prunning_amd/Makefile: the .hip, .cpp and .h files of csrc and this header, in
 * C-locale path order), so a test can tell a stale binary from one built from the tree. */
const char *maxk_source_digest(void);

/* The extra compiler flags (EXTRA_HIPFLAGS: MAXK_* tuning / ablation macros) this library was
 * built with; "" for the product build.  The digest above covers them too. */
const char *maxk_build_config(void);

/* ---------------------------------------------------------------------------
 * Forward row-wise-product SpGEMM:  out = diag(1/row_div) . A . scatter(cbsr)
 *   out[r, cbsr_idx[c,l]] += edge_val[e] * cbsr_val[c,l]   (e in row r, c = col_idx[e])
 * Every output row is written (rows without edges get zeros): no zero-init of
 * `out` is needed.  row_div may be NULL (no normalisation).  Duplicate
 * selectors within a CBSR row accumulate; selectors >= dim_origin are ignored.
 * Replaces: spmm_kernel_opt2_sparse_v3 (kernels/spmm_maxk.cu:17-106),
 *           its launcher spmm_kernel_opt2_sparse_v3_wrapper
 *           (cuda_kernel_wrappers.cu:38-56) and the /in_degrees of
 *           maxk_spgemm_function.py:85-86.
 * chunk_edges: tokens (rows + edges) per wavefront work item (0 = auto: about 8 items per
 *              resident wave slot in [256, 2048], or on a smaller graph all items resident
 *              in one round, down to 64).
 * workspace: >= maxk_spgemm_forward_workspace_size(...) bytes, 256-B aligned
 *            (packed CBSR records + split-row slabs).
 * ------------------------------------------------------------------------- */
size_t maxk_spgemm_forward_workspace_size(int64_t num_rows, int64_t num_cols, int64_t num_e,
                                          int32_t dim_origin, int32_t dim_k, int32_t chunk_edges);
int maxk_spgemm_forward(const int32_t *row_ptr, const int32_t *col_idx, const float *edge_val,
                        const float *cbsr_val, const uint8_t *cbsr_idx, const float *row_div,
                        float *out, int64_t num_rows, int64_t num_cols, int64_t num_e,
                        int32_t dim_origin, int32_t dim_k, int32_t chunk_edges,
                        void *workspace, size_t workspace_bytes, void *stream);
/* The same forward, also writing each edge's selectors: edge_sel[e, l] = cbsr_idx[col_idx[e], l]
 * (u8 [num_e, k]), the stream maxk_sspmm_backward_csc_sel reads.  The forward gathers every
 * edge's CBSR record anyway, so the stream costs one coalesced write of num_e * k bytes
 * (tables past 2^24 columns or 4 GiB of records: a separate gather, maxk_edge_selectors). */
int maxk_spgemm_forward_sel(const int32_t *row_ptr, const int32_t *col_idx, const float *edge_val,
                            const float *cbsr_val, const uint8_t *cbsr_idx, const float *row_div,
                            float *out, int64_t num_rows, int64_t num_cols, int64_t num_e,
                            int32_t dim_origin, int32_t dim_k, int32_t chunk_edges,
                            void *workspace, size_t workspace_bytes, void *stream,
                            uint8_t *edge_sel);
/* The same product added onto out (out += ...; out must hold valid values): a row range's
 * result summed over several column ranges of A, e.g. the sharded forward's pipelined halves
 * (maxk_dist.py), without a separate pass over out.  Same arguments and workspace. */
int maxk_spgemm_forward_accumulate(const int32_t *row_ptr, const int32_t *col_idx,
                                   const float *edge_val, const float *cbsr_val,
                                   const uint8_t *cbsr_idx, const float *row_div, float *out,
                                   int64_t num_rows, int64_t num_cols, int64_t num_e,
                                   int32_t dim_origin, int32_t dim_k, int32_t chunk_edges,
                                   void *workspace, size_t workspace_bytes, void *stream);
/* Both: the product added onto out and the edge-selector stream written (the sharded forward's
 * later pipelined parts, whose backward reads their own part's stream). */
int maxk_spgemm_forward_accumulate_sel(const int32_t *row_ptr, const int32_t *col_idx,
                                       const float *edge_val, const float *cbsr_val,
                                       const uint8_t *cbsr_idx, const float *row_div, float *out,
                                       int64_t num_rows, int64_t num_cols, int64_t num_e,
                                       int32_t dim_origin, int32_t dim_k, int32_t chunk_edges,
                                       void *workspace, size_t workspace_bytes, void *stream,
                                       uint8_t *edge_sel);
/* Transport records (the sharded forward, r05): [k f32 | k u8] per vertex at a stride of 5k bytes,
 * the bytes a vertex-range shard all-gathers anyway, built by each owner for its own rows
 * (maxk_cbsr_records) so the receivers walk the gathered buffer (maxk_spgemm_forward_records)
 * with no record pack over every gathered vertex.  Selectors stay the caller's bytes; a repeated
 * selector's first occurrence carries the sum of its values in l order and the later ones, like
 * selectors >= dim_origin, a skip marker (a NaN payload; a kept NaN value is stored as the
 * canonical quiet NaN) -- the same sums as maxk_spgemm_forward.  maxk_records_ok says whether
 * the records forward applies: the streaming walker of a sparse graph (average degree < 128) or
 * the deep-batch walker of a dense one, dim_k % 4 == 0 in [24, 32], num_cols * 5 * dim_k < 2^32 (where the 5k-byte stride costs no
 * extra line per gather against the packed record).  rec 4-B aligned; workspace as
 * maxk_spgemm_forward_workspace_size; accumulate adds onto out.  Replaces the same reference
 * kernel as maxk_spgemm_forward (spmm_maxk.cu:17-113). */
int maxk_records_ok(int64_t num_rows, int64_t num_cols, int64_t num_e, int32_t dim_origin,
                    int32_t dim_k);
int maxk_cbsr_records(const float *cbsr_val, const uint8_t *cbsr_idx, uint8_t *rec,
                      int64_t num_rows, int32_t dim_origin, int32_t dim_k, void *stream);
int maxk_spgemm_forward_records(const int32_t *row_ptr, const int32_t *col_idx,
                                const float *edge_val, const uint8_t *rec, const float *row_div,
                                float *out, int64_t num_rows, int64_t num_cols, int64_t num_e,
                                int32_t dim_origin, int32_t dim_k, int32_t chunk_edges,
                                void *workspace, size_t workspace_bytes, void *stream,
                                int32_t accumulate);

/* ---------------------------------------------------------------------------
 * Backward outer-product sampled SpMM (SSpMM):
 *   grad_cbsr[c,l] = sum_{e=(r->c)} edge_val[e] * grad_out[r, cbsr_idx[c,l]] / row_div[r]
 *                  = (A^T diag(1/row_div) G)[c, cbsr_idx[c,l]]     (from the CSR of A)
 * grad_cbsr [num_cols, k] is fully overwritten.  row_div may be NULL.
 * Replaces: spmm_kernel_opt2_sparse_backward_v3 (kernels/spmm_maxk_backward.cu:15-115),
 *           spmm_kernel_opt2_sparse_backward_v3_wrapper (cuda_kernel_wrappers.cu:58-76)
 *           and the /out_degrees of maxk_spgemm_function.py:154-155.
 * ------------------------------------------------------------------------- */
size_t maxk_sspmm_backward_workspace_size(int64_t num_rows, int64_t num_cols, int64_t num_e,
                                          int32_t dim_origin, int32_t dim_k, int32_t chunk_edges);
int maxk_sspmm_backward(const int32_t *row_ptr, const int32_t *col_idx, const float *edge_val,
                        const float *grad_out, const float *row_div, const uint8_t *cbsr_idx,
                        float *grad_cbsr, int64_t num_rows, int64_t num_cols, int64_t num_e,
                        int32_t dim_origin, int32_t dim_k, int32_t chunk_edges,
                        void *workspace, size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * Same backward, two-phase and atomic-free (bitwise deterministic): phase 1
 * stores each edge's k-float contribution in CSR edge order, phase 2 gathers
 * and sums the contributions of every destination through the CSC permutation.  Needs the transpose plan of the graph
 * (maxk_transpose_plan) and a workspace of
 * maxk_sspmm_backward_csc_workspace_size(...) bytes (about num_e*k*4).
 * ------------------------------------------------------------------------- */
size_t maxk_sspmm_backward_csc_workspace_size(int64_t num_rows, int64_t num_cols, int64_t num_e,
                                              int32_t dim_origin, int32_t dim_k,
                                              int32_t chunk_edges);
int maxk_sspmm_backward_csc(const int32_t *row_ptr, const int32_t *col_idx, const float *edge_val,
                            const float *grad_out, const float *row_div, const uint8_t *cbsr_idx,
                            const int32_t *col_ptr, const int32_t *csc_eid, float *grad_cbsr,
                            int64_t num_rows, int64_t num_cols, int64_t num_e, int32_t dim_origin,
                            int32_t dim_k, int32_t chunk_edges, void *workspace,
                            size_t workspace_bytes, void *stream);

/* The same csc backward with the selectors given per edge: edge_sel[num_e, k] (u8, 4-B
 * aligned, dim_k % 4 == 0) with edge_sel[e, l] = cbsr_idx[col_idx[e], l].  Phase 1 then reads
 * them in CSR order beside the weights instead of gathering a random cbsr_idx row (a whole
 * 128-B line) per edge -- the step that bounds phase 1 on large sparse graphs.  A forward that
 * gathered each edge's CBSR record anyway writes the stream for free
 * (maxk_spgemm_forward_sel); maxk_edge_selectors builds it by a gather otherwise. */
int maxk_sspmm_backward_csc_sel(const int32_t *row_ptr, const int32_t *col_idx,
                                const float *edge_val, const float *grad_out, const float *row_div,
                                const uint8_t *edge_sel, const int32_t *col_ptr,
                                const int32_t *csc_eid, float *grad_cbsr, int64_t num_rows,
                                int64_t num_cols, int64_t num_e, int32_t dim_origin, int32_t dim_k,
                                int32_t chunk_edges, void *workspace, size_t workspace_bytes,
                                void *stream);
/* edge_sel[e, l] = cbsr_idx[col_idx[e], l]: any dim_k in [1, 256] and any alignment (16-B words
 * when dim_k % 16 == 0 and both arrays are 16-B aligned, 4-B words for % 4 / 4-B aligned, else
 * bytes) -- also the fallback of maxk_spgemm_forward_sel past 2^24 columns or 4 GiB of records,
 * so a stream that works on a small graph works on a large one. */
int maxk_edge_selectors(const int32_t *col_idx, const uint8_t *cbsr_idx, int64_t num_e,
                        int32_t dim_k, uint8_t *edge_sel, void *stream);
/* Workgroups (256 threads) maxk_edge_selectors launches for n_words words: capped at 64 per
 * CU and walked grid-stride, so num_e * k one-byte words past 2^32 still launch. */
int64_t maxk_edge_selectors_blocks(int64_t n_words);

/* Transpose plan of a CSR graph (once per graph): col_ptr[num_cols+1] of the
 * CSC and csc_eid[num_e] = the CSR edge id held by CSC slot t (stable in CSR order).
 * Replaces the CSC side files of generate_meta_csc.py:14-93 /
 * load_warp4_metadata_csc (binding_v2.py:320-351). */
size_t maxk_transpose_plan_workspace_size(int64_t num_cols, int64_t num_e);
int maxk_transpose_plan(const int32_t *col_idx, int64_t num_cols, int64_t num_e,
                        int32_t *col_ptr, int32_t *csc_eid, void *workspace,
                        size_t workspace_bytes, void *stream);

/* Destination buckets (the pull's tiles, the bsort plan, the hybrid plan): buckets of
 * 2^bucket_shift consecutive columns, nb = maxk_bucket_count(num_cols, shift) of them;
 * maxk_bucket_shift(k) is the largest shift the fp64 LDS accumulator of the bucketed phase 2
 * allows for k (-1 for k <= 0).  (r06: the "bucket" backward mode and its plan entry points,
 * which no BASELINE configuration reached, left the library; bsort keeps the bucketed
 * phase 2.) */
int maxk_bucket_shift(int32_t dim_k);
int64_t maxk_bucket_count(int64_t num_cols, int32_t bucket_shift);

/* ---------------------------------------------------------------------------
 * Same backward, two-phase with window-sorted contribution rows ("bsort", dim_k % 4 == 0),
 * for large sparse graphs at small k, where every contribution row phase 2 reads would
 * otherwise cost a whole random 128-B line (ogbn-products k = 8: 32-B rows).  The CSR edges
 * are cut into windows of W = maxk_bsort_window(dim_k) consecutive edges; phase 1 builds a
 * window's rows in LDS (one workgroup per window) and writes them to the window's range of T
 * ordered by destination bucket, so the bucketed phase 2 (one workgroup per part of a
 * bucket's entry list, fp64 LDS sums) reads a bucket's rows of one window as one run.  edge_sel (optional, u8
 * [num_e, k], 4-B aligned; as maxk_sspmm_backward_csc_sel) replaces the cbsr_idx row
 * gathers; cbsr_idx may be NULL when it is given, col_idx when edge_sel is given.
 * Plan (once per graph and k): maxk_bsort_plan with the shift maxk_bucket_shift(k) --
 * bucket_ptr[nb + 1] the start of each bucket's entries, bucket_dst[num_e] (u16) each entry's
 * column minus its bucket's first column, bucket_pos[num_e] the T row of each bucket entry, win_src[num_e] (u16) the edge (relative to its window) whose row T row p holds,
 * edge_row[num_e] the source row of every CSR edge.
 * Meant for dim_k <= MAXK_BSORT_KMAX (8; the auto rule's limit): W * 4 * dim_k bytes fill the LDS
 * stage, so larger k leaves fewer rows per window and bucket (k = 16 on ogbn-products: one
 * row per run, 5.88 ms against 5.07 for csc) down to W = 160 at dim_k = 256, where the mode is
 * correct (tested) but only slower than csc.
 * Replaces the same reference kernels as maxk_sspmm_backward.
 * ------------------------------------------------------------------------- */
int32_t maxk_bsort_window(int32_t dim_k); /* -1 unless dim_k % 4 == 0 in [4, 256] */
size_t maxk_bsort_plan_workspace_size(int64_t num_cols, int64_t num_e);
int maxk_bsort_plan(const int32_t *row_ptr, const int32_t *col_idx, int64_t num_rows,
                    int64_t num_cols, int64_t num_e, int32_t dim_k, int32_t bucket_shift,
                    int32_t *bucket_ptr, int32_t *bucket_pos, uint16_t *bucket_dst,
                    uint16_t *win_src, int32_t *edge_row, void *workspace,
                    size_t workspace_bytes, void *stream);
size_t maxk_sspmm_backward_bsort_workspace_size(int64_t num_rows, int64_t num_cols,
                                                int64_t num_e, int32_t dim_origin,
                                                int32_t dim_k);
int maxk_sspmm_backward_bsort(const int32_t *row_ptr, const int32_t *col_idx,
                              const float *edge_val, const float *grad_out, const float *row_div,
                              const uint8_t *cbsr_idx, const uint8_t *edge_sel,
                              const int32_t *bucket_ptr, const int32_t *bucket_pos,
                              const uint16_t *bucket_dst, const uint16_t *win_src,
                              const int32_t *edge_row, int32_t bucket_shift, float *grad_cbsr,
                              int64_t num_rows,
                              int64_t num_cols, int64_t num_e, int32_t dim_origin, int32_t dim_k,
                              void *workspace, size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * Backward, pull form (no contribution rows): the same result as maxk_sspmm_backward,
 * summed per tile (row slice x destination bucket of 2^shift columns) from G / row_div
 * gathered directly, fp64 LDS accumulation, then the slices of a bucket added in slice
 * order.  The fp64 tile sums make two runs agree except in rare rounding ties (bitwise
 * repeatability: maxk_sspmm_backward_csc).  For dim_k % 4 == 0 each destination's selectors
 * are first re-ordered by column (quantile slots, sspmm_bwd.hip pull_sel_kernel) so one
 * gather instruction touches fewer lines of a row; the sums return to CBSR order at the
 * end.  With dim_k % 4 == 0 a tile's destination slots may be split by sorted rank into
 * parts of kp = dim_k / H slots, one workgroup each, so a bucket holds H times the
 * destinations (kp >= 8 below dim_k = 32, >= 16 from 32; maxk_pull_shift(dim_k) gives the
 * matching shift).  A selector >= dim_origin contributes 0.  Needs dim_k % 4 == 0 or
 * dim_k <= 64, dim_origin % 4 == 0, bucket_shift in [4, min(15, max(maxk_bucket_shift(dim_k),
 * maxk_pull_shift(dim_k)))] (above maxk_bucket_shift(dim_k) only with dim_k % 4 == 0), the pull
 * plan of the graph built with the same shift, slices and edge_val (maxk_pull_plan), and a
 * workspace of maxk_sspmm_backward_pull_workspace_size(...) bytes (G / row_div, slices x
 * num_cols x k floats of tile partials, and 2 x num_cols x k bytes of slot-ordered
 * selectors).  Replaces the same reference kernels as maxk_sspmm_backward
 * (kernels/spmm_maxk_backward.cu:15-121).
 * ------------------------------------------------------------------------- */
size_t maxk_sspmm_backward_pull_workspace_size(int64_t num_rows, int64_t num_cols,
                                               int32_t dim_origin, int32_t dim_k, int32_t slices);
int maxk_sspmm_backward_pull(const float *grad_out, const float *row_div,
                             const uint8_t *cbsr_idx, const int32_t *tile_ptr,
                             const uint32_t *ent, int32_t bucket_shift, int32_t slices,
                             float *grad_cbsr, int64_t num_rows, int64_t num_cols, int64_t num_e,
                             int32_t dim_origin, int32_t dim_k, void *workspace,
                             size_t workspace_bytes, void *stream);

/* The pull over a listed subset of a plan's tiles (dim_k % 4 == 0), for graphs where only
 * some tiles are dense enough to pull (a community-ordered graph: the tiles near the
 * diagonal) and the rest of the edges go through the two-phase backward (the "hybrid" mode
 * of the Python binding).  tile_list[n_tiles]: tile ids t = s*nb + j, increasing;
 * tile_ent[n_tiles + 1]: their entry ranges in ent; bucket_ptr[nb + 1] / bucket_tiles[n_tiles]:
 * per bucket, the positions in tile_list of its tiles in slice order.  accumulate bit 0 adds
 * the result onto grad_cbsr (which then holds the other edges' sum), else stores it;
 * MAXK_PULL_NO_REDUCE stops once the tile partials are in the workspace and
 * MAXK_PULL_REDUCE_ONLY, with otherwise the same arguments and workspace, runs only the
 * reduce onto grad_cbsr, so the tile kernels can run on another stream beside the two-phase
 * form of the other edges, joined before the reduce.  The
 * workspace holds n_tiles tile partials: maxk_sspmm_backward_pull_tiles_workspace_size.
 * Replaces the same reference kernels as maxk_sspmm_backward (spmm_maxk_backward.cu:15-121). */
#define MAXK_PULL_NO_REDUCE 2
#define MAXK_PULL_REDUCE_ONLY 4
size_t maxk_sspmm_backward_pull_tiles_workspace_size(int64_t num_rows, int64_t num_cols,
                                                     int32_t dim_origin, int32_t dim_k,
                                                     int32_t n_tiles);
int maxk_sspmm_backward_pull_tiles(const float *grad_out, const float *row_div,
                                   const uint8_t *cbsr_idx, const int32_t *tile_list,
                                   const int32_t *tile_ent, int32_t n_tiles,
                                   const int32_t *bucket_ptr, const int32_t *bucket_tiles,
                                   const uint32_t *ent, int32_t bucket_shift, int32_t slices,
                                   int32_t accumulate, float *grad_cbsr, int64_t num_rows,
                                   int64_t num_cols, int64_t num_e, int32_t dim_origin,
                                   int32_t dim_k, void *workspace, size_t workspace_bytes,
                                   void *stream);

/* Pull plan of a CSR graph and its edge values (once per graph, shift and slices):
 * tile_ptr[slices*nb + 1] over tiles t = s*nb + j (rows cut into `slices` slices of
 * ceil(num_rows/slices) <= 65536 rows, nb = maxk_bucket_count(num_cols, shift)); per tile,
 * in CSR order, ent[2*num_e] = one uint32 pair per edge: {row - first row of its slice |
 * (column - first column of its bucket) << 16, bits of edge_val}; bucket_shift in [4, 15]
 * (the backward's 16-B selector copies need 16 | 2^shift * k).  maxk_pull_shift(k) is the
 * bucket shift to use (at least 4); maxk_pull_slices(num_rows, num_cols, dim_origin, dim_k) the
 * default
 * slice count (about 3.5 MiB of G rows per slice and rank part of k -- at most 3 parts' worth
 * -- at least num_rows/65536, 1..256; when that makes at most 5 rounds of workgroups, one per
 * CU of the current device, over num_cols' buckets, the count in [ceil(S/2), S] with the
 * fewest rounds; num_cols <= 0 means num_rows). */
int maxk_pull_shift(int32_t dim_k);
int maxk_pull_slices(int64_t num_rows, int64_t num_cols, int32_t dim_origin, int32_t dim_k);
size_t maxk_pull_plan_workspace_size(int64_t num_rows, int64_t num_cols, int64_t num_e,
                                     int32_t bucket_shift, int32_t slices);
int maxk_pull_plan(const int32_t *row_ptr, const int32_t *col_idx, const float *edge_val,
                   int64_t num_rows, int64_t num_cols, int64_t num_e, int32_t bucket_shift,
                   int32_t slices, int32_t *tile_ptr, uint32_t *ent, void *workspace,
                   size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * Dense route (r05): wide top-k, dim_k >= dim_origin / 2 at dim_origin % 4 == 0,
 * dim_origin <= 128 (MAXK_DENSE_DMAX), dim_k % 4 == 0.  A CBSR row then carries as many bytes as
 * the dense row, so both directions aggregate dense rows.  Replaces the same reference kernels
 * as maxk_spgemm_forward / maxk_sspmm_backward (spmm_maxk.cu:17-106,
 * spmm_maxk_backward.cu:15-121) for those widths; results within fp32 rounding of them.
 *
 * maxk_dense_route: 1 when (dim_origin, dim_k) takes the route.  maxk_spgemm_forward takes it
 *   by itself there (16-B aligned cbsr_val and out, 4-B aligned cbsr_idx; not the _sel forms):
 *   the CBSR scattered into a dense [num_cols, dim_origin] table in the workspace, then one
 *   dense row walk (maxk_spgemm_forward_workspace_size covers it).
 * maxk_dense_plan: the graph's transpose with source rows -- for every CSC slot t of
 *   maxk_transpose_plan (col_ptr, csc_eid), t_src[t] = the CSR row holding edge csc_eid[t] and
 *   t_w[t] = edge_val[csc_eid[t]] (int32 / float [num_e]).  Once per graph and weights.
 * maxk_sspmm_backward_dense: grad_cbsr[c, l] = (A^T diag(1/row_div) G)[c, cbsr_idx[c, l]] from
 *   the transpose plan, walked destination by destination: at dim_k >= dim_origin / 2 over dense
 *   G rows, each finished row stored as its k selected columns; below that (dim_k <= 64) one
 *   selected column per lane, G[src, sel[c, l]] gathered per edge (selectors >= dim_origin read
 *   0).  Any dim_k % 4 == 0 <= dim_origin; the route's rule (maxk_dense_route) is where "auto"
 *   takes it.  Bitwise repeatable.  16-B aligned grad_out and grad_cbsr, 4-B aligned cbsr_idx.
 * ------------------------------------------------------------------------- */
int maxk_dense_route(int32_t dim_origin, int32_t dim_k);
int maxk_dense_plan(const int32_t *row_ptr, const float *edge_val, const int32_t *csc_eid,
                    int64_t num_rows, int64_t num_e, int32_t *t_src, float *t_w, void *stream);
size_t maxk_sspmm_backward_dense_workspace_size(int64_t num_rows, int64_t num_cols,
                                                int64_t num_e, int32_t dim_origin, int32_t dim_k,
                                                int32_t chunk_edges);
int maxk_sspmm_backward_dense(const int32_t *col_ptr, const int32_t *t_src, const float *t_w,
                              const float *grad_out, const float *row_div,
                              const uint8_t *cbsr_idx, float *grad_cbsr, int64_t num_rows,
                              int64_t num_cols, int64_t num_e, int32_t dim_origin, int32_t dim_k,
                              int32_t chunk_edges, void *workspace, size_t workspace_bytes,
                              void *stream);

/* ---------------------------------------------------------------------------
 * Hybrid backward and the "auto" backward rule through the C ABI (the Python binding's
 * hybrid_plan / pull_locality / _bwd_mode / _scaled_entries, maxk_cuda_kernels/__init__.py,
 * rest on these).  Replaces the same reference kernels as maxk_sspmm_backward
 * (spmm_maxk_backward.cu:15-121, launched by cuda_kernel_wrappers.cu:58-76).
 *
 * maxk_backward_mode_auto: the backward a graph should use (pure host arithmetic):
 *   MAXK_BWD_DENSE where maxk_dense_route(dim_origin, dim_k), or (its selected-column form)
 *   for a G of at most 64 MiB on a graph below the pull's density test at dim_origin <= 64,
 *   dim_origin / 4 <= dim_k < dim_origin / 2, both % 4 == 0; else MAXK_BWD_PULL where
 *   dim_k % 4 == 0 or dim_k <= 64, dim_origin % 4 == 0 and the graph has at
 *   least ~1/2 edge per (source row, bucket of 2^maxk_bucket_shift(dim_k) columns) or a G of at
 *   most 64 MiB (and at most 256 x 65536 rows); else MAXK_BWD_HYBRID
 *   when pull_locality (maxk_pull_locality at maxk_pull_shift(dim_k); < 0 = unknown) reaches
 *   MAXK_HYBRID_LOCALITY and dim_k % 4 == 0; else MAXK_BWD_BSORT at dim_k % 4 == 0,
 *   dim_k <= MAXK_BSORT_KMAX when a window of maxk_bsort_window(dim_k) edges holds at least 2
 *   rows per destination bucket on average (W * 2^maxk_bucket_shift(dim_k) >= 2 * num_cols;
 *   ogbn-products k = 8: 4.3); else MAXK_BWD_CSC.  Only csc and dense are bitwise
 *   repeatable.
 * maxk_pull_locality (synchronous): num_e / occupied (source row, bucket of 2^bucket_shift
 *   columns) pairs, columns sorted within rows; workspace >= 8 bytes.
 * maxk_hybrid_plan (synchronous): from the graph's pull plan (maxk_pull_plan with bucket_shift,
 *   slices), the tiles holding at least density x (rows of their slice) entries --
 *   tile_list[S*nb] (increasing tile ids), tile_ent[S*nb+1] (their runs in ent_pull[2*num_e]),
 *   bucket_ptr[nb+1] / bucket_tiles[S*nb] (per bucket, positions in tile_list in slice order)
 *   -- and every other edge as a CSR off_row_ptr[num_rows+1] / off_col[num_e] / off_val[num_e]
 *   (CSR order kept).  counts[3] = {tiles pulled, entries pulled, edges off}.  Buffers are
 *   sized for the worst case; the counts say how much of each holds the plan.
 * maxk_pull_entries_scale: ent_out = ent with each weight divided by its source row's
 *   row_div, for n_runs tile runs (tile_ids[i], or i when NULL; entries tile_ent[i] ..
 *   tile_ent[i+1]) -- once per (plan, divisor), so the pull gathers G instead of G / row_div.
 * maxk_sspmm_backward_hybrid: the csc backward over the off-tile CSR (its transpose plan:
 *   maxk_transpose_plan of off_col) and the listed-tile pull over the rest, accumulated into
 *   grad_cbsr.  With side_stream (and two caller-created events ev_fork / ev_join, as void*)
 *   the tile kernels run beside the csc and are joined before the final reduce; NULL runs
 *   everything on `stream`.  flags: MAXK_HYBRID_PRESCALED when ent_pull carries row_div.
 * ------------------------------------------------------------------------- */
#define MAXK_BWD_PULL 0
#define MAXK_BWD_CSC 1
/* 2 was MAXK_BWD_BUCKET (removed in r06); the code stays unused */
#define MAXK_BWD_HYBRID 3
#define MAXK_BWD_ATOMIC 4
#define MAXK_BWD_BSORT 5
#define MAXK_BWD_DENSE 6
#define MAXK_BSORT_KMAX 8
#define MAXK_HYBRID_LOCALITY 1.5
#define MAXK_HYBRID_DENSITY 0.5f
#define MAXK_HYBRID_PRESCALED 1
int maxk_backward_mode_auto(int64_t num_rows, int64_t num_cols, int64_t num_e, int32_t dim_origin,
                            int32_t dim_k, double pull_locality);
int maxk_pull_locality(const int32_t *row_ptr, const int32_t *col_idx, int64_t num_rows,
                       int64_t num_e, int32_t bucket_shift, double *locality, void *workspace,
                       size_t workspace_bytes, void *stream);
size_t maxk_hybrid_plan_workspace_size(int64_t num_rows, int64_t num_cols, int64_t num_e,
                                       int32_t bucket_shift, int32_t slices);
int maxk_hybrid_plan(const int32_t *row_ptr, const int32_t *col_idx, const float *edge_val,
                     const int32_t *tile_ptr, const uint32_t *ent, int64_t num_rows,
                     int64_t num_cols, int64_t num_e, int32_t bucket_shift, int32_t slices,
                     float density, int32_t *tile_list, int32_t *tile_ent, int32_t *bucket_ptr,
                     int32_t *bucket_tiles, uint32_t *ent_pull, int32_t *off_row_ptr,
                     int32_t *off_col, float *off_val, int64_t *counts, void *workspace,
                     size_t workspace_bytes, void *stream);
int maxk_pull_entries_scale(const uint32_t *ent, const int32_t *tile_ids, const int32_t *tile_ent,
                            int64_t n_runs, int64_t num_rows, int64_t num_cols,
                            int32_t bucket_shift, int32_t slices, const float *row_div,
                            uint32_t *ent_out, void *stream);
size_t maxk_sspmm_backward_hybrid_workspace_size(int64_t num_rows, int64_t num_cols,
                                                 int64_t n_off_e, int32_t dim_origin,
                                                 int32_t dim_k, int64_t n_tiles);
int maxk_sspmm_backward_hybrid(
    const float *grad_out, const float *row_div, const uint8_t *cbsr_idx,
    const int32_t *tile_list, const int32_t *tile_ent, int32_t n_tiles, const int32_t *bucket_ptr,
    const int32_t *bucket_tiles, const uint32_t *ent_pull, int64_t n_pull_e, int32_t bucket_shift,
    int32_t slices, const int32_t *off_row_ptr, const int32_t *off_col, const float *off_val,
    int64_t n_off_e, const int32_t *off_col_ptr, const int32_t *off_csc_eid, int32_t flags,
    float *grad_cbsr, int64_t num_rows, int64_t num_cols, int32_t dim_origin, int32_t dim_k,
    void *workspace, size_t workspace_bytes, void *stream, void *side_stream, void *ev_fork,
    void *ev_join);

/* ---------------------------------------------------------------------------
 * CBSR encode (MaxK top-k): per row the k largest of dim_origin values, in
 * torch.topk(largest=True, sorted=True) order (value descending; NaN largest;
 * equal values by ascending column).  x has leading dimension ld_x (elements).
 * Replaces: torch.topk + .to(uint8) in maxk_spgemm_function.py:51-57 and the
 *           uint8 kernel topk (kernels/maxk_kernel.cu:23-96) behind
 *           cuda_topk_maxk / cuda_topk_maxk_float (cuda_kernel_bindings.cpp:164-238).
 * maxk_topk_cbsr_u8: the same on uint8 input (values copied as uint8).
 * idx32 (optional, may be NULL): the same indices widened to int32.
 * ------------------------------------------------------------------------- */
int maxk_topk_cbsr(const float *x, int64_t ld_x, float *cbsr_val, uint8_t *cbsr_idx,
                   int32_t *idx32, int64_t num_rows, int32_t dim_origin, int32_t dim_k,
                   void *stream);
int maxk_topk_cbsr_u8(const uint8_t *x, int64_t ld_x, uint8_t *cbsr_val, uint8_t *cbsr_idx,
                      int32_t *idx32, int64_t num_rows, int32_t dim_origin, int32_t dim_k,
                      void *stream);
/* The reference uint8 top-k's intended per-row convention (kernels/maxk_kernel.cu:23-94,
 * behind cuda_topk_maxk / cuda_topk_maxk_float, cuda_kernel_bindings.cpp:164-238), for callers
 * that depend on its layout: rows of dim_origin == 256 bytes; each row's threshold from 8
 * bisection steps on [0, 255] over its own bytes; the bytes strictly above it in ascending
 * column order, 32 columns per step, at most dim_k, a pick in column 32s + 31 overwritten by the
 * next step's first pick (the reference counts a step's picks without its lane 31); slots never
 * filled are 0.  val / idx uint8 [num_rows, dim_k].  NOT the CUDA kernel's as-built output: that
 * kernel thresholds every row on its block's first row, per lane (:42, :44-48), racily, and
 * leaves unfilled slots uninitialised; parity with it is unpinned (oracle/oracle.py
 * topk_u8_reference_as_built models it).  Not torch.topk: maxk_topk_cbsr_u8 is the exact one. */
int maxk_topk_u8_reference(const uint8_t *x, uint8_t *val, uint8_t *idx, int64_t num_rows,
                           int32_t dim_origin, int32_t dim_k, void *stream);
/* Rows (over every top-k launch on the current device since the last reset) whose threshold
 * search took other than dim_k winners -- a kernel bug, never expected.  The kernels count such
 * rows, and such a row never writes past its own k winner slots (r02's fault: a dead row's
 * extra winners overwrote another wave's); its own output row is then undefined.  Read (and,
 * with reset != 0, zeroed) in order on `stream`, which it synchronises (not the device, so a
 * hipGraph capture on another stream is left alone).  The Python binding zeroes it before
 * and reads it after every top-k under MAXK_VALIDATE=1, so a count is the launch's own. */
int maxk_topk_error_rows(int64_t *rows, int32_t reset, void *stream);

/* dense[r,:] = 0; dense[r, cbsr_idx[r,l]] = cbsr_val[r,l]  (all of dense written).
 * Replaces: zeros(V,D).scatter_(1, sel, grad_sparse), maxk_spgemm_function.py:152,175. */
int maxk_cbsr_scatter_dense(const float *cbsr_val, const uint8_t *cbsr_idx, float *dense,
                            int64_t num_rows, int32_t dim_origin, int32_t dim_k, void *stream);

/* Fused MaxK activation, forward: maxk_topk_cbsr plus the masked dense output
 * dense[r, j] = x[r, j] if j is among row r's k winners, else 0 (row stride dim_origin),
 * written by the same kernel from the row it already holds.
 * Replaces: MaxK.forward, topk + zeros_like + scatter_ (model_integrated_v3.py:28-38),
 *           i.e. the top-k pass plus two dense V x D passes. */
int maxk_topk_cbsr_dense(const float *x, int64_t ld_x, float *cbsr_val, uint8_t *cbsr_idx,
                         float *dense, int64_t num_rows, int32_t dim_origin, int32_t dim_k,
                         void *stream);

/* Fused MaxK activation, backward, in one pass over the rows:
 *   grad_x[r, :] = 0;  grad_x[r, j] = grad_val[r, l] + grad_dense[r, j]  for j = cbsr_idx[r, l].
 * grad_val [V,k] and grad_dense [V,D] are each optional (NULL = zero); grad_x may alias
 * grad_dense.  Selectors of a row are distinct (top-k output); with duplicates one of them wins.
 * Replaces: OPTMaxK.backward's mask multiply (model_integrated_v3.py:39-43) together with
 *           zeros(V,D).scatter_(1, sel, grad_sparse) (maxk_spgemm_function.py:152,175). */
int maxk_topk_backward(const float *grad_val, const float *grad_dense, const uint8_t *cbsr_idx,
                       float *grad_x, int64_t num_rows, int32_t dim_origin, int32_t dim_k,
                       void *stream);

/* ---------------------------------------------------------------------------
 * warp4 schedule (drop-in for kernels/generate_meta.py:30-48 / generate_meta_csc.py:14-93
 * and the .warp4 files read by load_warp4_metadata, cuda_kernel_bindings.cpp:287-317).
 * maxk_warp4_count: synchronous; number of entries W = sum over rows of ceil(deg/warp_max_nz).
 * maxk_warp4_build: fills warp4[W*4] on the stream; needs
 *   maxk_warp4_build_workspace_size(num_rows) bytes of workspace.
 * maxk_warp4_to_row_ptr: recovers the CSR row_ptr[num_rows+1] a warp4 array
 *   describes (rows absent from it are empty); lets the reference's
 *   spmm_maxk_forward(warp4, ...) signature drive the CSR kernels.
 * ------------------------------------------------------------------------- */
int maxk_warp4_count(const int32_t *row_ptr, int64_t num_rows, int32_t warp_max_nz,
                     int64_t *num_entries, void *stream);
size_t maxk_warp4_build_workspace_size(int64_t num_rows);
int maxk_warp4_build(const int32_t *row_ptr, int64_t num_rows, int32_t warp_max_nz,
                     int32_t *warp4, int64_t num_entries, void *workspace,
                     size_t workspace_bytes, void *stream);
int maxk_warp4_to_row_ptr(const int32_t *warp4, int64_t num_entries, int64_t num_rows,
                          int32_t *row_ptr, void *stream);

/* ---------------------------------------------------------------------------
 * Dense SpMM baseline Y = A . X on rocSPARSE (the speed-up denominator; the
 * MI355X equivalent of spmm_cusparse, kernels/spmm_cusparse.cu:6-62, and of
 * the cusparse_spmm binding, cuda_kernel_bindings.cpp:253-284).
 * A plan owns the rocSPARSE handle, descriptors and buffer (synchronous to
 * create); maxk_dense_spmm_run only launches (alpha=1, beta=0).
 * ------------------------------------------------------------------------- */
typedef struct maxk_dense_spmm_plan maxk_dense_spmm_plan;
int maxk_dense_spmm_plan_create(maxk_dense_spmm_plan **plan, const int32_t *row_ptr,
                                const int32_t *col_idx, const float *edge_val, const float *x,
                                float *y, int64_t num_rows, int64_t num_cols, int64_t num_e,
                                int32_t dim, int32_t alg, void *stream);
int maxk_dense_spmm_run(maxk_dense_spmm_plan *plan, void *stream);
/* Point the plan at new X / Y buffers of the same shape (one plan per graph serves every
 * call, as cusparseSpMM's descriptors do in the reference's callers). */
int maxk_dense_spmm_bind(maxk_dense_spmm_plan *plan, const float *x, float *y);
int maxk_dense_spmm_plan_destroy(maxk_dense_spmm_plan *plan);

#ifdef __cplusplus
}
#endif

#endif /* MAXK_HIP_H_ */
