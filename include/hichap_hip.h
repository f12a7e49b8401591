/*
 * hichap_hip.h — C-ABI of libhichap_hip.so, the MI355X (gfx950) hot path of
 * HiCHap's bias correction and structure analysis.
 *
 * Plain C types only (no torch / HIP types in signatures: streams are passed
 * as `void*` = hipStream_t, device buffers as plain pointers).  Every entry
 * point returns HH_OK (0) or a negative HH_ERR_* code; on error the message is
 * available from hh_last_error() (thread-local) and output buffers are left
 * untouched.  No C++ exception crosses this boundary.
 *
 * What each entry point replaces in the reference (/root/reference):
 *   ICE                 `cooler balance --ignore-diags 1 [--cis-only] --force`
 *                       subprocess strings, HiCHap/matrixBuilding.py:708, :713,
 *                       :1537, :1542, :1761, :1766 (algorithm: cooler.balance,
 *                       third-party, see oracle/ice_ref.py)
 *   hh_twostep          TwoStepCorrection, matrixBuilding.py:984-1023
 *   hh_genomewide_*     GenomeWideMatrixCorrection, matrixBuilding.py:857-901
 *   hh_compartment_*    StructureFind.Distance_Decay / Get_PCA / Select_PC_new,
 *                       StructureFind.py:201-423
 *   hh_di_scan          StructureFind.Get_Gap / Get_DI, StructureFind.py:721-839
 *   hh_viterbi_gmm      StructureFind.viterbipath (ghmm model.viterbi),
 *                       StructureFind.py:1113-1123 (host code)
 *   hh_hiccups_*        StructureFind.pcaller neighbourhood sums (HICCUPS loops),
 *                       StructureFind.py:1631-1830
 *   hh_binner_*         the per-line pair binning loops of TraditionalMatrixBuilding
 *                       (matrixBuilding.py:566-596), TraditionalMatrixInAllelic
 *                       (:817-854) and HaplotypeMatrixBuilding's unimputed
 *                       M_M / P_P / M_P / P_M passes (:1126-1240)
 */
#ifndef HICHAP_HIP_H
#define HICHAP_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HH_OK 0
#define HH_ERR_ARG -1   /* invalid argument / unsupported input            */
#define HH_ERR_HIP -2   /* HIP runtime error                               */
#define HH_ERR_OOM -3   /* device or host allocation failed                */
#define HH_ERR_STATE -4 /* call not valid in the object's current state    */

/* ------------------------------------------------------------ runtime */
const char* hh_last_error(void);
int hh_version(void);                 /* (major<<16)|(minor<<8)|patch */
int hh_device_count(int32_t* n);
int hh_set_device(int32_t device);
int hh_synchronize(void* stream);
/* device-to-device copy of `bytes` on `stream` (asynchronous) */
int hh_device_copy(void* dst, const void* src, int64_t bytes, void* stream);
/* Performance knobs: "band_w" (-1 auto, 0 no dense band, > 0 forced
 * multiple of 16; for matrices built afterwards), "band4" 0/1 (the 4-bit
 * band; later builds), "band4_density_pct" / "band8_big_pct" (its width
 * thresholds, defaults 25 / 5; later builds), "flat_max" (0..255: longest
 * row, in 16-B payload words, of a tile swept by the flat kernel; 0 = none;
 * later builds), "band_concurrent" 0/1 (dense-band sweep on a side stream),
 * "sweep_nb" in {1,2,4,8} (row batches in flight per
 * wave), "unit_entries" (work-unit size used by later matrix builds),
 * "sweep_ablate" 0/1/2 (timing ablations only: 1 skips the LDS gathers,
 * 2 skips the b staging; results are wrong while set), "sweep_trace" n
 * (diagnostic: record start / end wall clock and CU of each block of the
 * single-launch sweep when its grid has <= n blocks; 0 frees the buffer),
 * "fuse_stats" -1/0/1/2 (ICE statistics: -1 auto, 0 never fused into k_marg,
 * 1 fused + last-block tails (auto up to 128 stats tiles), 2 tile sums in
 * k_marg + block-wide group reductions (auto above)), "band_lpt" 0/1 (band chunks dispatched
 * heaviest first), "unit_lpt" 0/1/2 and "unit_lpt_lists" 1..3 (work-unit
 * launch lists by cost; later builds), "flat_defer" 0/1 (flat sweep merges a
 * tile's compact sums after the next tile's barrier), "syrk_split" -1 / 0 /
 * n (K splits of the compartment correlation GEMM: auto, never, forced).
 * fuse_stats / syrk_split change reduction orders (last bits); the ablations
 * give wrong results; the others leave every bit unchanged. */
int hh_tune(const char* key, int64_t value);
/* The last traced single-launch sweep: *n blocks; out (cap >= 3 n words) gets
 * (start, end, cu) per block in grid order (tiled units | band blocks | flat
 * units), wall-clock ticks (100 MHz).  Diagnostic, synchronising. */
int hh_sweep_trace(uint64_t* out, int64_t cap, int64_t* n);
/* Kernel timing (measurement only): while enabled, the dense-path launches
 * (k_rowstats, k_symvc1..3, k_syrk, k_cor_mul, k_select_stats, k_di,
 * k_gap_scan) are bracketed by HIP events on their stream; query returns the
 * summed duration and launch count for one kernel name (synchronising). */
int hh_ktime_enable(int32_t on);
int hh_ktime_query(const char* name, double* total_ms, int64_t* calls);
int hh_ktime_reset(void);

/* ---------------------------------------------------- contact matrix
 * A contact matrix resident in HBM in the "tiled pixel" layout:
 * the symmetric matrix (both triangles of cooler's upper-triangle pixel table)
 * for the rows [row_lo, row_hi) a rank owns, cut into 512-row blocks x
 * 8192-column tiles; each tile stores its rows' entries as uint16
 * (swizzled LDS byte offset << 3 | count, counts 1..7) and uint32 (count << 16 |
 * offset, counts 8..65535)
 * segments, rows padded to 16 B, counts > 65535 in a small per-row wide
 * list, plus a per-row diagonal.  Pixels near the diagonal (|col - row| <= W8,
 * count <= 255) live in a dense uint8 band with implicit columns, and those
 * with W8 < |col - row| <= W4 and count <= 15 in a dense 4-bit band, instead
 * of the tiles (W8, W4 chosen from the data's diagonal occupancy and counts).  Static filters
 * (ignore_diags, cis_only zero_trans, zero counts) are applied at build time.
 * Shards are whole 512-row blocks (row_lo % 512 == 0).
 */
typedef struct hh_matrix hh_matrix;

typedef struct {
    int64_t n_bins;        /* bins of the whole matrix                       */
    int64_t row_lo, row_hi;/* rows held by this object                      */
    int64_t nnz_upper;     /* kept pixels with bin2 - bin1 >= ignore_diags   */
    int64_t n_entries;     /* symmetric off-diagonal entries stored          */
    int64_t n_slots;       /* stored uint32 slots (entries + row padding)    */
    int64_t n_tiles;       /* nonempty (row-block, column-tile) pairs        */
    int64_t n_units;       /* sweep work units                               */
    int64_t n_wide;        /* entries with count >= 2^19 (wide list)         */
    int64_t device_bytes;  /* HBM held by the matrix                         */
    int64_t n_slots_narrow;/* stored uint16 slots (entries + row padding)    */
    int64_t payload_bytes; /* entry bytes streamed per sweep (both widths and
                              the dense band)                                */
    int32_t n_chroms;
    int32_t ignore_diags;
    int32_t cis_only;
    int32_t device;
    int32_t band_w;        /* uint8 diagonal band half-width W8 (0 = none)   */
    int32_t n_units_flat;  /* work units swept by the flat (short-row) kernel */
    int64_t n_band;        /* nonzero entries held by the band               */
    int64_t payload_bytes_flat; /* part of payload_bytes in flat-kernel tiles */
    int32_t band_w4;       /* nibble band outer width (== band_w: none)      */
    int32_t upper;         /* 1: upper-triangle tiles         */
} hh_matrix_info;

/* Build from cooler's pixel table (host arrays; any order: a sorted
 * upper-triangle table is uploaded and built on the device, anything else is
 * built on the host; duplicate (bin1, bin2) pixels fail with HH_ERR_ARG).  Counts must be non-negative integers < 2^32
 * (cooler `count`, int32 in HiCHap's traditional coolers, matrixBuilding.py:196).
 * chrom_offsets[n_chroms+1] = cooler `indexes/chrom_offset`. Rows outside
 * [row_lo, row_hi) are not stored (a shard for multi-GPU genome-wide ICE). */
int hh_matrix_from_pixels(const int64_t* bin1, const int64_t* bin2, const double* count,
                          int64_t nnz, int64_t n_bins, const int64_t* chrom_offsets,
                          int32_t n_chroms, int32_t ignore_diags, int32_t cis_only,
                          int64_t row_lo, int64_t row_hi, void* stream, hh_matrix** out);
/* The same from a DEVICE pixel table in cooler's own order — sorted by
 * (bin1, bin2), bin1 <= bin2, unique — with int32 ids and counts (cooler's
 * `count` dtype for HiCHap's traditional coolers; what hh_binner_pixels_device
 * hands out).  Built entirely on the device (filters, symmetric rows by a
 * radix sort of the lower half, tile counts, payload); the layout equals
 * hh_matrix_from_pixels'.  A table out of order, with a duplicate pixel, a
 * negative count or an id out of range fails with HH_ERR_ARG naming the first
 * offending pixel.  hh_matrix_from_pixels itself takes this path whenever its
 * host table is sorted upper-triangle (uploading it once), and builds on the
 * host otherwise (hh_tune "host_build" 1 forces the host builder). */
int hh_matrix_from_pixels_device(const int32_t* bin1, const int32_t* bin2, const int32_t* count, int64_t nnz,
                                 int64_t n_bins, const int64_t* chrom_offsets, int32_t n_chroms, int32_t ignore_diags,
                                 int32_t cis_only, int64_t row_lo, int64_t row_hi, void* stream, hh_matrix** out);
int hh_matrix_free(hh_matrix* m);
int hh_matrix_get_info(const hh_matrix* m, hh_matrix_info* info);
/* Diagnostic read rates of a matrix's own buffers (no sweep work): out[2i] =
 * ms per pass, out[2i+1] = bytes, for i = 0 wide / 1 narrow tile entries,
 * 2 uint8 / 3 nibble band (linear reads), 4-6 the flat tiles' payload in the
 * flat sweep's order, streamed only; 7-8 the same with coalesced run loads;
 * 9 the narrow entries linearly in lane-major runs.  nout >= 20. */
int hh_matrix_stream_probe(const hh_matrix* m, int32_t reps, double* out, int32_t nout);
/* Copy the stored upper-triangle pixels (bin1 <= bin2, bin1 in the local rows
 * for which bin1 is the row) back to the host; *nnz_inout = capacity on entry,
 * count on exit.  For checking only. */
int hh_matrix_export_upper(const hh_matrix* m, int64_t* bin1, int64_t* bin2, double* count,
                           int64_t* nnz_inout);

/* Synthetic whole-genome contact matrices generated directly in HBM
 * (SURVEY.md §8(d) model; counter-based hashing keyed on the unordered bin
 * pair, so every shard of every rank sees the same matrix). */
typedef struct {
    int32_t n_chroms;
    const int32_t* chrom_nbins; /* host array [n_chroms]                     */
    double A;                   /* cis amplitude                              */
    double decay;               /* power-law exponent (1.08)                  */
    double comp_strength;       /* 0.3                                        */
    double vis_sigma;           /* log-normal visibility sigma (0.3)          */
    double gap_frac;            /* fraction of empty bins (0.02)              */
    double trans_density;       /* uniform trans pixel density                */
    int32_t comp_block;         /* compartment block length in bins           */
    int32_t ignore_diags;
    int32_t cis_only;
    int32_t pad_;
    uint64_t seed;
} hh_synth_params;

/* Counting pass over ALL rows: per-row stored slots (work) and upper-triangle
 * pixel counts (host arrays of n_bins).  Used to partition rows across ranks. */
int hh_synth_count(const hh_synth_params* p, int32_t* row_work, int64_t* row_nnz_upper,
                   void* stream);
/* Dense cis block of chromosome `chrom` of the same synthetic genome as
 * float64 counts into device memory out[N_c * N_c] (bench inputs for the
 * per-chromosome compartment config C5; ignore_diags applies). */
int hh_synth_dense(const hh_synth_params* p, int32_t chrom, double* out, void* stream);
/* The model's pixel table in HBM (bench inputs of the table-driven paths):
 * cooler's upper-triangle table sorted by (bin1, bin2), or with ordered = 1
 * every nonzero cell (i, j) sorted by (i, j) with independent draws for (i, j)
 * and (j, i) (an asymmetric matrix like HiCHap's imputed haplotype matrices).
 * int32 ids and counts, owned by the hh_pixels handle. */
typedef struct hh_pixels hh_pixels;
int hh_synth_pixels(const hh_synth_params* p, int32_t ordered, void* stream, hh_pixels** out);
int hh_pixels_get(const hh_pixels* P, const int32_t** bin1, const int32_t** bin2, const int32_t** count, int64_t* nnz);
int hh_pixels_free(hh_pixels* P);
/* Build rows [row_lo, row_hi) (row_lo % 512 == 0). */
int hh_synth_build(const hh_synth_params* p, int64_t row_lo, int64_t row_hi, void* stream,
                   hh_matrix** out);

/* ---------------------------------------------------------------- ICE
 * cooler's balance_cooler semantics (oracle/ice_ref.py). */
typedef struct {
    int32_t mad_max;           /* 5                                         */
    int32_t min_nnz;           /* 10                                        */
    double min_count;          /* 0                                         */
    double tol;                /* 1e-5                                      */
    int32_t max_iters;         /* 200                                       */
    int32_t rescale_marginals; /* 1                                         */
    int32_t check_every;       /* host polls convergence every k sweeps (0=8)*/
    int32_t pad_;
} hh_ice_opts;

/* One-call balance on one GPU (the matrix must hold every row).
 * weights[n_bins] (host) receive cooler's bins/weight (NaN = masked).
 * Per group (1 group genome-wide, n_chroms groups when cis_only):
 * scale[], var[], iters[], converged[] (host arrays).
 * sweep_seconds (may be NULL) = wall time of the iteration loop only. */
int hh_ice_balance(hh_matrix* m, const hh_ice_opts* o, double* weights, double* scale,
                   double* var, int32_t* iters, int32_t* converged, double* sweep_seconds,
                   void* stream);

/* Fine-grained device API used by the multi-GPU driver (one process per GPU;
 * the marginal vector is exchanged with an all-gather over RCCL by the
 * caller).  All calls are asynchronous on `stream` unless noted. */
typedef struct hh_ice hh_ice;
int hh_ice_create(hh_matrix* m, const hh_ice_opts* o, hh_ice** out);
int hh_ice_free(hh_ice* s);
int hh_ice_n_groups(const hh_ice* s, int32_t* n);
/* mode: 0 = binarized (nnz), 1 = raw counts, 2 = count*b_i*b_j.
 * Writes the marginal of the local rows to marg_local[row_hi - row_lo]
 * (device).  When the matrix holds every row, marg_local may be NULL and the
 * result lands in the internal full marginal directly. */
int hh_ice_marg_local(hh_ice* s, int32_t mode, double* marg_local, void* stream);
/* Scatter an all-gathered, per-rank padded marginal (world x maxlen, device)
 * into the internal full marginal; rank_rows[world+1] host row offsets. */
int hh_ice_set_marg(hh_ice* s, const double* gathered, int32_t world, int64_t maxlen,
                    const int64_t* rank_rows, void* stream);
/* Filters (after set_marg of the matching mode).  mad uses host medians:
 * synchronous. */
int hh_ice_filter_nnz(hh_ice* s, void* stream);
int hh_ice_filter_count_mad(hh_ice* s, void* stream);
/* One ICE update after set_marg(mode 2): variance, bias update, convergence. */
int hh_ice_update(hh_ice* s, void* stream);
/* Number of still-active groups (synchronous). */
int hh_ice_active_groups(hh_ice* s, int32_t* n_active, void* stream);
int hh_ice_iterations_done(const hh_ice* s, int32_t* iters);
/* Full sweeps on one GPU without host polling (bench / single-GPU): runs
 * `n` iterations of marg(mode 2) + update back to back. */
int hh_ice_run(hh_ice* s, int32_t n, void* stream);
/* Final weights + stats (synchronous), as hh_ice_balance. */
int hh_ice_finalize(hh_ice* s, double* weights, double* scale, double* var, int32_t* iters,
                    int32_t* converged, void* stream);
/* Kernel timing of the last hh_ice_run (HIP events on the run's stream):
 * total ms of the sweep kernel, launches. */
int hh_ice_last_sweep_timing(const hh_ice* s, double* sweep_ms_total, int32_t* sweep_launches,
                             double* iter_ms_total);
/* Payload bytes one sweep of this state reads: tile entries + both segments'
 * row pointers + the band bytes its band kernels stream (the upper halves
 * only, plus a shard's halo rows, with the upper-band sweep).
 * A measurement helper (bench.py's roofline), no computation. */
int hh_ice_swept_bytes(const hh_ice* s, int64_t* bytes);
/* The current bias vector b (all n_bins entries, every rank holds the whole
 * vector; 0 = masked) to host memory (synchronous; checking only: the
 * marginal of the next sweep is marg_i = b_i sum_j A_ij b_j). */
int hh_ice_get_bias(const hh_ice* s, double* bias, void* stream);

/* ------------------------------------------------ sharded ICE in C
 * Genome-wide ICE over world processes (one GPU each), each holding the
 * matrix rows rank_rows[rank] .. rank_rows[rank + 1] (whole 512-row blocks):
 * per iteration one all-gather of the local marginals, then the identical
 * update everywhere, iterations enqueued from C++ (no caller code in the
 * loop).  The exchange is a callback: `allgather(send, count, recv, user,
 * stream)` must gather `count` doubles from every rank (device buffers,
 * rank order) into recv[world * count] on `stream` and return 0.  The
 * library's RCCL transport: hh_comm_unique_id on one rank (128 bytes, shared
 * by the caller's own means), hh_comm_init on every rank, then pass
 * hh_comm_allgather with user = the hh_comm. */
typedef int (*hh_allgather_fn)(const double* send, int64_t count, double* recv, void* user, void* stream);
typedef struct hh_comm hh_comm;
int hh_comm_unique_id(uint8_t* id128);
int hh_comm_init(const uint8_t* id128, int32_t world, int32_t rank, hh_comm** out);
int hh_comm_free(hh_comm* c);
int hh_comm_allgather(const double* send, int64_t count, double* recv, void* comm, void* stream);
/* Upper-triangle tiles store an entry of a strictly upper
 * tile once, and its column side belongs to the rank owning that column: a
 * shard's marginals need a second exchange per sweep, an int64 reduce-scatter
 * of the ranks' padded row blocks (integer sums: exact, the same bits on any
 * number of ranks).  `reduce(send, count, recv, user, stream)`: send = world x
 * count int64 (rank-major blocks), recv = count: the sum over the ranks of this
 * rank's block; 0 = ok.  hh_comm_reduce_scatter is RCCL's (user = the
 * hh_comm).  hh_ice_*_sharded register the exchange themselves (RCCL's when
 * their all-gather is hh_comm_allgather, else a reduction through the
 * all-gather callback: world x its bytes); a caller that drives
 * hh_ice_marg_local on a shard registers it once after hh_ice_create
 * (rank -1: inferred from the matrix's row range; reduce NULL keeps one
 * registered before for the same world). */
typedef int (*hh_reduce_fn)(const int64_t* send, int64_t count, int64_t* recv, void* user, void* stream);
int hh_comm_reduce_scatter(const int64_t* send, int64_t count, int64_t* recv, void* comm, void* stream);
int hh_ice_set_column_exchange(hh_ice* s, int32_t world, int32_t rank, const int64_t* rank_rows, hh_reduce_fn reduce,
                               void* reduce_user, hh_allgather_fn allgather, void* allgather_user);
/* The whole balance (filters, iterations to convergence, finalize) on this
 * rank's shard `m`; outputs as hh_ice_balance (weights for every bin, identical
 * on every rank). */
int hh_ice_balance_sharded(hh_matrix* m, const hh_ice_opts* o, int32_t world, int32_t rank, const int64_t* rank_rows,
                           hh_allgather_fn allgather, void* user, double* weights, double* scale, double* var,
                           int32_t* iters, int32_t* converged, double* sweep_seconds, void* stream);
/* `cooler balance --cis-only` (matrixBuilding.py:713, :1542, :1766) over world
 * processes with no collective in the iterations:
 * every rank holds whole chromosomes (dealt by LPT on their pixels) as a
 * compact cis-only matrix `m` -- its chromosomes' bins renumbered
 * consecutively -- whose per-chromosome ICE groups converge independently.
 * The one exchange is `allgather` of max_local_bins doubles per rank (the
 * per-chromosome-normalised raw marginals, zero padded) for cooler's
 * genome-wide MAD cutoff.  Outputs cover this rank's bins and chromosomes. */
int hh_ice_balance_cis_local(hh_matrix* m, const hh_ice_opts* o, int32_t world, int64_t max_local_bins,
                             hh_allgather_fn allgather, void* user, double* weights, double* scale, double* var,
                             int32_t* iters, int32_t* converged, double* sweep_seconds, void* stream);
/* Pieces of it on an hh_ice (bench / fixed iteration counts): the two
 * filters, and n iterations without convergence polling. */
int hh_ice_filters_sharded(hh_ice* s, int32_t world, const int64_t* rank_rows, hh_allgather_fn allgather, void* user,
                           void* stream);
int hh_ice_run_sharded(hh_ice* s, int32_t world, const int64_t* rank_rows, hh_allgather_fn allgather, void* user,
                       int32_t n, void* stream);

/* ------------------------------------------ dense two-step correction
 * Dense row-major N x N matrices; dtype 0 = int64, 1 = float64.  Host
 * pointers (copied in/out) or, with on_device = 1, device pointers. */
/* Per row i over columns [lo[i], hi[i]) (lo = hi = NULL: whole rows): sum
 * (exact for int64) and number of zero entries.  Replaces the row loops of
 * Coverage_M / Gap_defined / Gap_definedLowRes and the alpha row sums,
 * matrixBuilding.py:742-753, :878-881, :904-929, :994-995. */
int hh_dense_rowstats(const void* X, int32_t dtype, int64_t N, const int64_t* lo, const int64_t* hi,
                      double* rowsum, int64_t* zeros, int32_t on_device, void* stream);
/* out = (raw_sum / N^2) / mean(C) * C with C = Correct_VC(Y, exponent),
 * Y = Trans2symmetry(X / alpha[:, None], gap) (gap = NULL: the sum form,
 * Trans2symmetryLowRes).  raw_sum = sum(X) (MM.mean() * N^2).
 * TwoStepCorrection :1007-1021, GenomeWideMatrixCorrection :894-899. */
int hh_dense_symvc(const void* X, int32_t dtype, int64_t N, const double* alpha, const uint8_t* gap,
                   double exponent, double raw_sum, double* out, int32_t on_device, void* stream);
/* TwoStepCorrection(TM, MM, PM) (matrixBuilding.py:984-1023) in one call:
 * int64 N x N inputs, float64 N x N outputs (Nor_MM, Nor_PM), gap masks
 * (gap_m[i] = 1 for i in Gap_M).  The gap / alpha glue runs on the host with
 * np.percentile ('linear') semantics; each matrix crosses PCIe once. */
/* Dense N x N int64 (device `out`, zeroed first) from cells (row, col, count)
 * whose ids are shifted by `offset`: out[r][c] = count, and out[c][r] too for
 * an upper-triangle table (symmetric = 1).  The reference's dense matrices
 * from its per-line loops (matrixBuilding.py:554, :567-570, :1290-1301), built
 * on the device from the binner's tables so only the cells cross PCIe.
 * Cells must be unique; out-of-range ids (or bin1 > bin2 when symmetric)
 * are an error.  on_device = 1: row / col / count are device pointers. */
int hh_dense_from_cells(const int64_t* row, const int64_t* col, const int64_t* count, int64_t nnz, int64_t N,
                        int64_t offset, int32_t symmetric, int32_t on_device, int64_t* out, void* stream);
/* Upper-triangle nonzeros of a dense fp64 N x N device matrix in cooler
 * order, the np.triu(M).nonzero() table NPZ2Cooler writes for the corrected
 * matrices (matrixBuilding.py:1613, :1628-1633): hh_dense_upper_count, then
 * hh_dense_upper_write into caller-sized device buffers. */
int hh_dense_upper_count(const double* X, int64_t N, int64_t* nnz, void* stream);
int hh_dense_upper_write(const double* X, int64_t N, int32_t* bin1, int32_t* bin2, double* value, void* stream);
int hh_twostep(const int64_t* TM, const int64_t* MM, const int64_t* PM, int64_t N, double* nor_mm, double* nor_pm,
               uint8_t* gap_m, uint8_t* gap_p, int32_t on_device, void* stream);
/* IntraChromMatrixCorrection (matrixBuilding.py:1026-1041): hh_twostep over
 * n chromosomes in one call, device pointers only (TM[c], MM[c], PM[c] int64
 * N[c] x N[c]; nor_mm[c], nor_pm[c] fp64 outputs).  The row statistics and
 * the gap / alpha glue of every chromosome run as shared launches; then
 * n_streams = 0: every pass of every chromosome's two symmetrisation chains
 * in one shared launch per pass; 1..16: each chain's launches on the
 * least-loaded of that many streams, largest chromosomes first.  One
 * synchronisation at the end; per chromosome bitwise hh_twostep's results.
 * gap_m / gap_p (host) receive every chromosome's flags concatenated in
 * argument order. */
int hh_twostep_batch(int32_t n, const int64_t* const* TM, const int64_t* const* MM, const int64_t* const* PM,
                     const int64_t* N, double* const* nor_mm, double* const* nor_pm, uint8_t* gap_m,
                     uint8_t* gap_p, int32_t n_streams, void* stream);

/* ------------------------------------ sparse genome-wide correction
 * GenomeWideMatrixCorrection (matrixBuilding.py:857-901) on pixel tables
 * instead of dense 2n x 2n matrices.  T: the traditional whole-genome table
 * (cooler order: bin1 <= bin2, sorted, unique) on n bins, chrom_offsets[n_chroms
 * + 1] its chromosome layout; H: every nonzero cell (row, col, count) of the
 * imputed haplotype matrix, sorted by (row, col), unique, on 2n bins laid out
 * as the M copies of the chromosomes then the P copies (Get_Chro_Bins_Haplotypes
 * :429-454).  hh_gw_create validates both and computes the alpha step's exact
 * integer statistics; the caller computes alpha (NumPy percentile semantics,
 * :878-893) and hh_gw_correct does S = H / Alpha[:, None], the sum
 * symmetrisation (:770-777), Correct_VC(., exponent) and the mean rescale
 * (:894-899), leaving the upper triangle of the result (cooler order, what
 * NPZ2Cooler stores) on the device.  Counts are integers < 2^32. */
typedef struct hh_gw hh_gw;
int hh_gw_create(const int64_t* t_bin1, const int64_t* t_bin2, const double* t_count, int64_t t_nnz,
                 const int64_t* h_row, const int64_t* h_col, const double* h_count, int64_t h_nnz, int64_t n,
                 const int64_t* chrom_offsets, int32_t n_chroms, void* stream, hh_gw** out);
/* the same from device int32 tables (the binner's outputs) */
int hh_gw_create_device(const int32_t* t_bin1, const int32_t* t_bin2, const int32_t* t_count, int64_t t_nnz,
                        const int32_t* h_row, const int32_t* h_col, const int32_t* h_count, int64_t h_nnz, int64_t n,
                        const int64_t* chrom_offsets, int32_t n_chroms, void* stream, hh_gw** out);
int hh_gw_free(hh_gw* g);
/* host arrays: t_rowsum[n], t_nnz_row[n] = sum / nonzero count of T's row
 * within its chromosome block (the diagonal once); h_blocksum[2n] = sum of H's
 * row within its same-chromosome same-haplotype block (M_M / P_P); *h_total =
 * sum(H).  Any pointer may be NULL. */
int hh_gw_stats(const hh_gw* g, int64_t* t_rowsum, int64_t* t_nnz_row, int64_t* h_blocksum, int64_t* h_total);
/* The alpha step (:878-893) per chromosome on those statistics, computed by
 * hh_gw_create on a host thread while the column lists build: alpha[n] in
 * bin order, chrom_ok[n_chroms] (layout order) 0 where the caller must use
 * NumPy's own path (no non-gap bin, or a max that is not positive finite).
 * Replaces matrixBuilding.py:878-886's Python loop. */
int hh_gw_alpha(const hh_gw* g, double* alpha, int32_t* chrom_ok);
/* alpha[2n] (host): the concatenated, duplicated SNP-density factors;
 * exponent: 2/3.  *out_nnz = upper-triangle pixels of the result. */
int hh_gw_correct(hh_gw* g, const double* alpha, double exponent, int64_t* out_nnz, void* stream);
/* hh_gw_correct in two calls, the output owned by the caller: the count
 * (marginals, VC factors, merge count pass, the mean rescale factor; state
 * kept in the handle), then the write of the upper table into device
 * buffers of out_nnz elements. */
int hh_gw_correct_count(hh_gw* g, const double* alpha, double exponent, int64_t* out_nnz, void* stream);
int hh_gw_correct_write(hh_gw* g, int32_t* bin1, int32_t* bin2, double* value, void* stream);
/* the result to host arrays of out_nnz (any may be NULL), or its device
 * pointers (valid until hh_gw_free or the next hh_gw_correct) */
int hh_gw_result(const hh_gw* g, int64_t* bin1, int64_t* bin2, double* value, void* stream);
int hh_gw_result_device(const hh_gw* g, const int32_t** bin1, const int32_t** bin2, const double** value);

/* ---------------------------------------------------- compartment (one chrom)
 * StructureFind.Distance_Decay / Get_PCA / Select_PC_new, StructureFind.py:201-423.
 * M: dense N x N float64 raw contacts (cooler matrix(balance=False).fetch). */
typedef struct hh_comp hh_comp;
int hh_comp_create(const double* M, int64_t N, int32_t on_device, void* stream, hh_comp** out);
int hh_comp_free(hh_comp* c);
/* nnz_col[j] = number of nonzero entries of column j (gap columns, :216-220). */
int hh_comp_colnnz(hh_comp* c, int64_t* nnz_col, void* stream);
/* sums[d] = sum of nonzero M[i][j] with |i-j| = d whose column j is not a gap
 * (gapcol[j] = 1) — the bincount of Distance_Decay before the bin_num division. */
int hh_comp_diag_sums(hh_comp* c, const uint8_t* gapcol, double* sums, void* stream);
/* Get_PCA(SA=True): the Sliding_Approach O/E (StructureFind.py:274-299,
 * step = 600000 // Res // 2 >= 1) materialised on the device (N x N): box
 * sum of M over the (2 step + 1)^2 window / the 3-2-1 weighted expected sum
 * inside [step, N - step - 1]^2, M / decline[|i-j|] on the border.  Later
 * hh_comp_correlation / hh_comp_select_stats use it in place of the plain
 * O/E; decline = NULL switches back. */
int hh_comp_sliding_oe(hh_comp* c, const double* decline, int32_t step, void* stream);
int hh_comp_get_sliding_oe(hh_comp* c, double* oe, void* stream);
/* O/E = M / decline[|i-j|] on nonzeros (or the Sliding_Approach O/E), columns
 * ng[0..n); Pearson correlation of those columns (np.corrcoef(rowvar=False),
 * NaN -> 0) kept on the device. */
int hh_comp_correlation(hh_comp* c, const double* decline, const int64_t* ng, int64_t n, void* stream);
int hh_comp_get_cor(hh_comp* c, double* cor, void* stream);
/* Replace the device correlation (n x n from the last hh_comp_correlation). */
int hh_comp_set_cor(hh_comp* c, const double* cor, void* stream);
/* Top-k right singular vectors of the column-centred correlation (sklearn
 * PCA(k).fit(Cor).components_, sign: max-|.| entry positive), k x n row-major.
 * Default method (hh_tune "pca_method" 1): explicit-restart block Krylov on
 * Cor (16 columns, hh_tune "pca_p" products per cycle) with a Rayleigh-Ritz
 * step for the centred matrix; stops when the top-k Ritz vectors'
 * a-posteriori angle bound max ||A x - theta x|| / gap is < tol, or has
 * stopped shrinking below 1e3 tol (the rounding floor; a degenerate gap never
 * gets there), after at most 2 * max_iters Cor products.  Method 0
 * (and the fallback when the basis would not fit, n < 16 (pca_p + 1)): block
 * subspace iteration, max_iters iterations.  *iters = Cor products (Krylov)
 * or iterations (subspace).  Not converging is not an error: query
 * hh_comp_pca_status.  The Krylov products read only the upper triangle of
 * Cor (hh_tune "cor_sym", default 1; 0: the full matrix), so a Cor set with
 * hh_comp_set_cor is taken as symmetric; hh_tune "ortho_tpb" / "ortho_min_tpb"
 * set the orthogonalisation's rows per block (/ 64). */
int hh_comp_pca(hh_comp* c, int32_t k, double tol, int32_t max_iters, double* components, double* eigvals,
                int32_t* iters, void* stream);
/* Outcome of the last hh_comp_pca: converged (1/0), Cor products, Krylov
 * cycles (subspace: iterations), method (1 Krylov, 0 subspace). */
int hh_comp_pca_status(const hh_comp* c, int32_t* converged, int32_t* products, int32_t* cycles, int32_t* method);
/* Host helper (no GPU): top-k eigenpairs, descending, of a symmetric m x m
 * matrix (Householder tridiagonalisation, implicit QL eigenvalues, inverse
 * iteration) — the Rayleigh-Ritz solver of the Krylov PCA; evecs m x k
 * row-major. */
int hh_sym_topk(const double* H, int32_t m, int32_t k, double* evals, double* evecs);
/* Per PC q < k (<= 3), 8 sums: [0,1] Cor same-sign pairs in (-1, 1-eps) sum,count;
 * [2,3] Cor (pc_i > 0, pc_j < 0) pairs in (-1, 1) sum,count; [4,5] nonzero O/E
 * over (+,+) sum,count; [6,7] over (-,-) — Select_PC_new's means_minus / select_ab. */
int hh_comp_select_stats(hh_comp* c, const double* pcs, int32_t k, double eps, double* stats, void* stream);

/* ------------------------------------------------------- TAD scan (DI)
 * Both scans read column j only within B rows of the diagonal, so the matrix
 * is passed as a diagonal-major band: band[(B + k) * N + j] = M[j + k][j],
 * k in [-B, B] (0 outside the matrix); M balanced with NaN -> 0 for traditional data.
 * hh_gap_scan = StructureFind.Get_Gap (:721-751): gap[j] = 1 when column j
 * has fewer than 2*lb*0.8 nonzeros in M[j-lb:j+lb, j] or is within lb of an
 * edge (lb <= B).  hh_di_scan = Get_DI (:804-839): di[j] from the up / down
 * windows of window_bins[j] <= B bins (0 at gap[j] and edges); test 0 =
 * t-test, 1 = chi-square. */
int hh_gap_scan(const double* band, int64_t N, int32_t B, int32_t lb, uint8_t* gap, int32_t on_device,
                void* stream);
int hh_di_scan(const double* band, int64_t N, int32_t B, const uint8_t* gap, const int32_t* window_bins,
               int32_t test, double* di, int32_t on_device, void* stream);
/* The same scans fed from cooler's pixel table instead of a dense matrix:
 * StructureFind.Data_preprocess (:853-854) loads each chromosome as
 * cooler.matrix(balance=True).fetch(chrom) + np.nan_to_num (allelic data:
 * balance=False, :858-865) and scans it.  hh_band_from_pixels builds that
 * matrix's band on the device, band[(B + k) * N + j] = M[j + k][j] for the
 * chromosome's bins [lo, lo + N), from the unique upper-triangle pixels
 * (bin1 <= bin2, global bin ids): value count * weight[bin1] * weight[bin2]
 * with NaN -> 0, or the raw count when weight is NULL (n_weight >= lo + N).
 * on_device: bin1/bin2/count/weight/band are device pointers; otherwise host
 * pointers (the band is returned to the host).  hh_tad_scan_pixels = band of
 * width B = max(lb, max window_bins) + hh_gap_scan + the first / last bin
 * joining the gap (Data_preprocess :876-884) + hh_di_scan in one call, the
 * pixel table crossing PCIe once (not at all with on_device); gap, di and
 * window_bins are host arrays of N. */
int hh_band_from_pixels(const int64_t* bin1, const int64_t* bin2, const double* count, int64_t nnz,
                        const double* weight, int64_t n_weight, int64_t lo, int64_t N, int32_t B, double* band,
                        int32_t on_device, void* stream);
int hh_tad_scan_pixels(const int64_t* bin1, const int64_t* bin2, const double* count, int64_t nnz,
                       const double* weight, int64_t n_weight, int64_t lo, int64_t N, int32_t lb,
                       const int32_t* window_bins, int32_t test, uint8_t* gap, double* di, int32_t on_device,
                       void* stream);

/* ------------------------------------------------- TAD HMM (host code)
 * Viterbi path of a continuous HMM with Gaussian-mixture emissions, ghmm's
 * `model.viterbi(EmissionSequence)` as StructureFind.viterbipath calls it
 * (:1113-1123): S states, M components per state; A (S x S, row-major) and pi
 * are probabilities, mean / var / weight are S x M (var = variance, ghmm's
 * GaussianMixtureDistribution parameters).  Log space, a_ij = 0 -> -inf, ties
 * to the lowest state.  path[t] = state of obs[t]; *logp = log joint
 * probability of the path.  Runs on the host (no GPU needed). */
int hh_viterbi_gmm(const double* obs, int64_t n, int32_t S, int32_t M, const double* A, const double* pi,
                   const double* mean, const double* var, const double* weight, int32_t* path, double* logp);

/* ---------------------------------------------------------- pair binning
 * Pair text (HiCHap *_Valid.bed: chrom/pos in fields 1, 6, 8, 13; allelic
 * beds: fields 0-3 and a trailing mark) -> cooler pixel tables per target
 * matrix: upper triangle (bin1 <= bin2), sorted by (bin1, bin2), count = number
 * of pairs of the unordered bin pair — what the reference's dense
 * `M[b1][b2] += 1; M[b2][b1] += 1` (once when b1 == b2) + np.triu + nonzero
 * produce (matrixBuilding.py:457-525, :566-596).
 * Lines follow Python's `line.strip().split()`; chromosome fields are
 * `lstrip('chr')`-ed and looked up in the name table.  A line the reference
 * would raise on (missing field, non-integer position, a name that passes the
 * `chroms` filter but is not in genomeSize, a bin outside the matrix) fails the
 * feed with HH_ERR_ARG naming the first such line (negative positions too:
 * the reference's NumPy indexing would wrap them). */
typedef struct hh_binner hh_binner;
typedef struct {
    int32_t col_chrom1, col_pos1, col_chrom2, col_pos2; /* 0-based fields      */
    char mark[16];     /* non-empty: skip lines whose LAST field differs (`if
                          line[-1] != 'Both': continue`, :1133)              */
    int32_t hap1, hap2;/* haplotype half of chrom1 / chrom2 (0 = M or the
                          traditional genome, 1 = P)                         */
    int32_t mode;      /* 0 binning; 1 imputation (HaplotypeMatrixBuilding
                          :1251-1494): lines whose last field == mark are
                          skipped, last field == mark2 selects the R1 branch  */
    char mark2[16];
} hh_pairs_format;
/* names: n_names NUL-terminated names back to back (after lstrip('chr'));
 * name_ids[k] = chromosome index (Sort_Chromosomes order) or -2 for a name
 * the `chroms` filter accepts but genomeSize lacks.  unknown_policy for names
 * not in the table: 0 skip the line, 1 raise if the name is all digits
 * ('#' in chroms), 2 raise (empty chroms list). */
int hh_binner_create(int32_t n_chroms, const char* names, const int32_t* name_ids, int32_t n_names,
                     int32_t unknown_policy, hh_binner** out);
int hh_binner_free(hh_binner* b);
/* One output matrix at resolution `res`: chrom_start[2 * n_chroms] = first
 * global bin of chromosome c in haplotype h (index h * n_chroms + c; the
 * traditional layout uses h = 0 only), chrom_nbins[c] = l // res + 1.
 * local = 1: intra-chromosome matrices only (localRes; trans pairs dropped,
 * per-chromosome bounds), bins still global (split per chromosome by the
 * caller). */
int hh_binner_add_target(hh_binner* b, int32_t res, int32_t local, const int64_t* chrom_start,
                         const int32_t* chrom_nbins, int64_t n_bins, int32_t* index_out);
/* An imputation target (ordered cells: the imputed matrices are asymmetric).
 * Whole (local = 0): `unimputed` = the unimputed whole matrix (host, n_bins x
 * n_bins int64, haplotype layout), L = Imputation_region // res, the
 * Imputation_min / _ratio tests.  Feeds in mode 1: first the M_M text
 * (hap 0), then — after hh_binner_set_stale — the P_P text (hap 1). */
int hh_binner_add_impute_target(hh_binner* b, int32_t res, int32_t local, const int64_t* chrom_start,
                                const int32_t* chrom_nbins, int64_t n_bins, const int64_t* unimputed, int32_t L,
                                int64_t imin, double ratio, int32_t* index_out);
/* The M pass's last line (byte offset in the concatenated feeds) that reached
 * the neighbourhood step, and at which target (-1 / -1: none): the caller
 * rebuilds the reference's stale M_M_sub from it and sets the P pass's sum
 * per whole target (ok = 0: the reference raises there). */
int hh_binner_last_reached(const hh_binner* b, int64_t* byte_offset, int32_t* target);
int hh_binner_set_stale(hh_binner* b, int32_t target, int64_t pp_sum, int32_t ok);
/* Parse + bin host text (staged through pinned chunks of chunk_bytes, cut at
 * line ends; 0 = 256 MB) or device-resident text.  Synchronous. */
int hh_binner_feed(hh_binner* b, const char* text, int64_t nbytes, const hh_pairs_format* f, int64_t chunk_bytes,
                   void* stream);
int hh_binner_feed_device(hh_binner* b, const char* text, int64_t nbytes, const hh_pairs_format* f, void* stream);
/* stats4: lines read, lines binned, skipped by the chromosome filter,
 * skipped by the mark filter. */
int hh_binner_stats(const hh_binner* b, int64_t* stats4);
/* Sort + run-length encode every target (synchronous); then nnz per target. */
int hh_binner_finish(hh_binner* b, void* stream);
int hh_binner_target_nnz(const hh_binner* b, int32_t target, int64_t* nnz, int64_t* n_pairs);
int hh_binner_download(const hh_binner* b, int32_t target, int32_t* bin1, int32_t* bin2, int32_t* count);
/* Device pointers of a finished target (valid until hh_binner_free). */
int hh_binner_pixels_device(const hh_binner* b, int32_t target, const int32_t** bin1, const int32_t** bin2,
                            const int32_t** count);
/* Synthetic pair text generated in device memory (bench input): format 0 =
 * 15-column *_Valid.bed lines, 1 = allelic "chrom pos chrom pos mark".  out =
 * NULL: size query into *nbytes. */
int hh_synth_pairs_text(int32_t n_chroms, const char* names, const int64_t* lengths, int64_t n_lines,
                        double cis_frac, double max_dist, int32_t format, uint64_t seed, int64_t line0, char* out,
                        int64_t capacity, int64_t* nbytes, void* stream);

/* ------------------------------------------------ HICCUPS loop calling
 * The neighbourhood sums of StructureFind.pcaller (StructureFind.py:1631-1830)
 * for one chromosome.  Bands are row-major N x num (num = maxapart / res +
 * maxww + 1; band[r][d] = M[r][r + d], 0 past the matrix): Hb raw counts with
 * the main diagonal zeroed, Cb balanced counts on diagonals ww..num-1 (0
 * elsewhere); Eall[d] = expected on diagonal d (0 for d < ww). */
typedef struct hh_hiccups hh_hiccups;
int hh_hiccups_create(const double* Hb, const double* Cb, const double* Eall, int64_t N, int32_t num, int32_t pw,
                      int32_t on_device, void* stream, hh_hiccups** out);
int hh_hiccups_free(hh_hiccups* h);
/* Candidate pixels (row <= col, col - row < num); resets every pixel to pending. */
int hh_hiccups_set_pixels(hh_hiccups* h, const int32_t* row, const int32_t* col, int64_t n, void* stream);
/* Every pixel back to pending (same pixels; repeated runs). */
int hh_hiccups_reset(hh_hiccups* h, void* stream);
/* One window width w (>= pw): every pending pixel whose lower-left raw reads
 * reach 16 gets its donut / lower-left balanced and expected sums and is
 * assigned; *newly_valid = how many (the caller applies the reference's
 * stop rule: fewer than 10 % of the pending pixels). */
int hh_hiccups_width(hh_hiccups* h, int32_t w, int64_t* newly_valid, void* stream);
/* Per pixel: donut / lower-left sums of the balanced (sK, sY) and expected
 * (eK, eY) bands at its width; width[i] = that w (0 = never assigned). */
int hh_hiccups_results(hh_hiccups* h, double* sK, double* sY, double* eK, double* eY, uint8_t* width, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HICHAP_HIP_H */
