// Internal layout of the HBM-resident contact matrix ("tiled pixel" layout,
// DESIGN.md §3) and of its build plan.  Not part of the C-ABI.
//
// The symmetric matrix (both triangles of cooler's pixel table) is cut into
// row-blocks of kR = 512 rows (global alignment: block = row / 256) and column
// tiles of kW = 8192 columns.  A nonempty (row-block, tile) pair is a *tile*:
// its entries are stored row by row (each row's list column-sorted and padded
// to 16 B), with kR + 1 row pointers.  Entries come in two widths, each a
// row-structured segment of the tile with its own row pointers:
//   narrow  uint16 = swz(c) << 3 | count, counts 1..7
//           (~3/4 of a whole-genome matrix's pixels: far-cis and trans);
//   wide    uint32 = count << 16 | swz(c) << 3, counts 8..65535,
// with c = col - tile_start and swz the LDS bank rotation of the staged bias
// slice, so swz(c) << 3 is the entry's byte offset in LDS: decoding is two
// mask/shift ops.  Counts > 65535 go to a small per-row "wide list" instead.  The sweep kernel stages the tile's 8192 bias
// values in LDS once and gathers from LDS, so the per-entry gathers never
// touch the texture path.
//
// Work is cut into *units*: a run of consecutive tiles of one row-block (all
// of its rows), or a row range of one large tile, each ~kUnitEntries entries.
// A unit writes one partial per row; k_marg adds a row's unit partials in
// unit order, so sums are bitwise deterministic and independent of sharding
// (shards are whole row-blocks).
#pragma once

#include "hh_common.hpp"

namespace hh {

constexpr int kR = 512;                 // rows per row-block
#ifndef HH_KWBITS
#define HH_KWBITS 13
#endif
// 8192-column tiles.  The upper-triangle tiles need the
// 4096-column build (-DHH_KWBITS=12, libhichap_hip_up.so): their blocks
// stage the bias slice AND an int64 column accumulator in LDS
constexpr int kWBits = HH_KWBITS;
constexpr bool kUpperBuild = HH_KWBITS <= 12;  // upper-triangle tiles available
constexpr int kW = 1 << kWBits;         // columns per tile
constexpr uint32_t kColMask = kW - 1;
constexpr uint32_t kCntMax = 65535u;    // largest count stored in a tile (wide entry)
extern int64_t g_unit_lpt;                               // launch lists largest cost class first (hh_tune)
extern int64_t g_unit_lpt_lists;                         // which launch lists unit_lpt orders (bit 0 tiled, bit 1 flat)
extern int64_t g_tile_cost;                              // per-tile cost in the unit split (hh_tune)
extern int64_t g_unit_entries;                           // ~512 KiB of payload per unit (hh_tune)
constexpr int64_t kMaxBins = (int64_t)1 << 30;

constexpr uint32_t kNarrowMax = 7;                        // counts stored as uint16

// Dense diagonal band: the pixels with 1 <= |col - row| <= W
// and count <= 255 are stored as uint8 counts with implicit columns (slots
// below); W is a multiple of 16 chosen from
// the data (the diagonals whose occupancy is >= kBandDensity), 0 = no band.
// Everything else (farther, trans, larger counts) stays in the tiles.
// band work blocks: 64 or 256 rows (ice.hip sweep_band)
constexpr int kBandChunk = 2048;    // band slots per work block
constexpr int kBandMaxW = 16384;
constexpr uint32_t kBandMaxCnt = 255u;
constexpr double kBandDensity = 0.5;
extern int64_t g_band_w;            // hh_tune("band_w"): -1 auto, 0 off, > 0 forced (multiple of 16)
// Nibble band: beyond the uint8 band, the diagonals
// W8 < |d| <= W4 whose counts are <= 15 are stored as 4-bit counts with
// implicit columns, in two segments per row (negative, positive diagonals),
// each K = W4 - W8 slots (a multiple of 32) + 32 slots of zero padding.
// W8 shrinks to where counts > 15 become rare (< g_band8_big of a diagonal's
// pixels), W4 reaches the occupancy break-even of 4-bit slots vs
// 2-byte tile entries (g_band4_density).  Larger counts there stay in the tiles.
constexpr uint32_t kBand4MaxCnt = 15u;
extern double g_band4_density;      // hh_tune("band4_density_pct"), default 25 %
extern double g_band8_big;          // hh_tune("band8_big_pct"), default 5 %
extern int64_t g_band4;             // hh_tune("band4"): 1 nibble band on (default), 0 off
// Upper-triangle tiles (build time, hh_tune "upper_tiles"): a tile entry
// (r, c) is stored only when c's column tile is not left of r's, J(c) >=
// J(r) (J = x >> kWBits); entries of strictly upper tiles then feed their row
// and their column
extern int64_t g_upper_tiles;
struct BandWidths {
    int32_t w8 = 0, w4 = 0;         // uint8 band |d| <= w8; nibble band w8 < |d| <= w4 (w4 == w8: none)
};
// occ[d] = occupancy of diagonal d, big[d] = share of its pixels with count > 15
BandWidths choose_band_widths(const std::vector<double>& occ, const std::vector<double>& big, int ignore_diags);
__host__ __device__ __forceinline__ int64_t band4_seg(int64_t w8, int64_t w4) { return w4 > w8 ? (w4 - w8) / 2 + 16 : 0; }
__host__ __device__ __forceinline__ int64_t band4_stride(int64_t w8, int64_t w4) { return 2 * band4_seg(w8, w4); }
// nibble index of diagonal d (w8 < |d| <= w4) within a row's band4 bytes:
// segment 0 (d < 0) slot d + w4, segment 1 (d > 0) slot d - w8 - 1
__host__ __device__ __forceinline__ int64_t band4_nibble(int64_t d, int64_t w8, int64_t w4) {
    return d < 0 ? d + w4 : 2 * band4_seg(w8, w4) + (d - w8 - 1);
}
__host__ __device__ __forceinline__ bool in_band4(int64_t d, uint32_t v, int64_t w8, int64_t w4) {
    const int64_t a = d < 0 ? -d : d;
    return v > 0 && v <= kBand4MaxCnt && a > w8 && a <= w4;
}
// row r's band slots: s = d + W for diagonals d in [-W, W] (slot W, the main
// diagonal, stays 0), then zero padding: a row is band_stride(W) = 2W + 16
// bytes (a multiple of 16; the padding lets the sweep read 16-slot groups
// shifted by the row's alignment without a bounds case)
__host__ __device__ __forceinline__ int64_t band_slot(int64_t d, int64_t W) { return d + W; }
__host__ __device__ __forceinline__ int64_t band_diag(int64_t s, int64_t W) { return s - W; }
__host__ __device__ __forceinline__ int64_t band_stride(int64_t W) { return W > 0 ? 2 * W + 16 : 0; }
// W from the occupancy of diagonals 1..kBandMaxW (occ[d] / (n - d)): the
// longest prefix of diagonals from ignore_diags on whose occupancy stays >=
// kBandDensity, rounded down to a multiple of 16 (or the forced value).
int32_t choose_band_w(const std::vector<double>& occupancy, int ignore_diags);
inline int64_t pad4(int64_t x) { return (x + 3) & ~(int64_t)3; }

// LDS image of a tile's bias values, XOR-rotated so that a wave reading
// columns c, c+4, c+8, ... (one uint4 per lane on a dense row) hits 32
// distinct 8-byte bank slots: element e = 32h + l is kept at 32h + ((l + h) mod 32).
__host__ __device__ __forceinline__ uint32_t swz(uint32_t e) { return (e & ~31u) | ((e + (e >> 5)) & 31u); }
__host__ __device__ __forceinline__ uint32_t unswz(uint32_t s) { return (s & ~31u) | (((s & 31u) - (s >> 5)) & 31u); }
// entry encodings (c = column offset in the tile)
__host__ __device__ __forceinline__ uint16_t enc_narrow(uint32_t c, uint32_t count) {
    return (uint16_t)((swz(c) << 3) | count);
}
__host__ __device__ __forceinline__ uint32_t enc_wide(uint32_t c, uint32_t count) { return (count << 16) | (swz(c) << 3); }
__host__ __device__ __forceinline__ uint32_t dec_col(uint32_t byteoff) { return unswz((byteoff & 0xFFFFu) >> 3); }
inline int64_t pad8(int64_t x) { return (x + 7) & ~(int64_t)7; }
constexpr int kBands = 5;        // lane-group widths 64, 32, 16, 8, 4
constexpr int kBandSlots = 8;    // kBands + 1 bounds, then the flat flag and row count
// Flat tiles: when no row of either segment of a tile is
// longer than g_flat_max uint4, the tile goes to k_sweep_flat, which streams
// each segment as one flat uint4 array (lane-major runs, rows found by search
// over the compacted row starts, segmented reduction across lanes) instead of
// lane groups per row; its perms then list the nonempty rows in row order.
// Units hold only flat or only non-flat tiles.
constexpr int kFlatWaves = 8;    // waves of a flat-kernel block (= kSweepThreads / 64)
constexpr int kFlatMeta = 2 * 2 * (kFlatWaves + 1);
// per flat tile, one record staged into LDS in one copy: uint16 starts (in
// uint4) of the nonempty rows of both segments, kR + 1 each (padded with the
// segment's uint4 count), then uint16 row ids, kR each; 16-B padded
constexpr int kFrecHalf = 2 * (kR + 1) + 2 * kR;
constexpr int kFrecU4 = (kFrecHalf * 2 + 15) / 16;
constexpr int kFlatFlag = 6;     // band slot: 1 = flat segment
constexpr int kFlatRows = 7;     // band slot: number of nonempty rows
extern int64_t g_flat_max;       // hh_tune("flat_max"), build time
// Column-grouped flat sweep (hh_tune "flat_cols", build time):
// every flat tile is its own work unit (one partial per row per flat tile),
// and the flat tiles of one column tile J are swept together in groups of up
// to g_flat_group by one block that stages b[J] once, each wave walking whole
// tiles on its own (no block barrier per tile).
extern int64_t g_flat_cols;
bool flat_cols_on(int32_t nJ);  // the column-grouped flat sweep for a matrix of nJ column tiles
bool upper_tiles_on(int32_t nJ);  // upper-triangle tiles for a matrix of nJ column tiles (g_upper_tiles)
extern int64_t g_flat_group;   // tiles per column group (0 = auto, 11 .. 44)
// minimum row length (uint4 per row) of band g
__host__ __device__ constexpr uint32_t band_min(int g) { return g == 0 ? 48u : g == 1 ? 24u : g == 2 ? 12u : g == 3 ? 6u : 1u; }

// One flat unit's descriptor in column-group order (k_sweep_flatw): every
// field the sweep needs to start the tile, in one 48-byte record, so grabbing
// the next tile is one (scalar) load instead of a chain of dependent lookups
// (unit -> tile -> split / entries / record).
struct FlatDesc {
    long long entn, ent;     // first narrow / wide entry of the tile
    int32_t frec, slot;      // flat record index, first unit partial
    uint32_t qbn, qbw;       // narrow / wide uint4 counts
    uint16_t nr, nfn, nfw;   // rows of the row-block, nonempty narrow / wide rows
    uint16_t glo, ghi;       // ICE groups of the unit's rows
    uint16_t upper;          // 1: strictly upper tile (its entries also feed their columns)
    uint32_t rb;             // local row-block (global first row = row_lo + kR rb)
};
static_assert(sizeof(FlatDesc) == 48, "FlatDesc layout");

// Host plan + arrays of the tiled layout.
struct TilePlan {
    int64_t nloc = 0;      // local rows
    int64_t nrb = 0;       // local row-blocks
    int32_t nJ = 0;        // column tiles over the whole matrix
    std::vector<int32_t> tile_J;      // per tile
    std::vector<int64_t> tile_ent;    // per tile: first wide entry (multiple of 4)
    HVec<uint32_t> tile_rp;    // per tile: kR + 1 wide row offsets (relative)
    std::vector<int64_t> tile_entn;   // per tile: first narrow entry (multiple of 8)
    HVec<uint32_t> tile_rpn;   // per tile: kR + 1 narrow row offsets (relative)
    // per tile and segment (narrow, wide): rows ordered by decreasing length
    // (uint4 count, counting sort on min(len, 255), stable) and the bands of
    // that order swept with lane groups of 64/32/16/8/4 (kBands + 1 bounds)
    HVec<uint16_t> tile_perm;  // per tile: 2 x kR
    HVec<uint16_t> tile_band;  // per tile: 2 x kBandSlots
    // per flat tile and segment: the 8 waves' split of the nonempty rows,
    // kFlatWaves + 1 pairs (first uint4, first compact row index); the last
    // pair is (segment uint4 count, number of nonempty rows)
    HVec<uint32_t> tile_fw;    // per tile: kFlatMeta words
    std::vector<int32_t> tile_frec;   // per tile: index of its flat record, -1
    HVec<uint16_t> frec;       // flat records, kFrecU4 * 8 halves each
    std::vector<int32_t> tile_rb;     // per tile: local row-block
    std::vector<int32_t> blk_tile_ptr;  // nrb + 1
    std::vector<int32_t> tile_of;     // nrb * nJ -> tile index or -1
    // units
    std::vector<int32_t> u_tlo, u_thi, u_rb, u_rlo, u_rhi, u_slot;
    std::vector<uint16_t> u_glo, u_ghi;
    std::vector<int32_t> blk_unit_ptr;  // nrb + 1
    std::vector<int32_t> u_order;       // launch lists: tiled-kernel units, then flat-kernel units
    std::vector<uint8_t> u_whole;       // 1: the unit covers whole row-blocks (sorted-band sweep)
    std::vector<uint8_t> tile_flat;     // per tile: 1 = flat (every nonempty segment flat)
    std::vector<uint8_t> u_flat;        // per unit: 1 = swept by the flat kernel
    std::vector<int32_t> fg_ptr, fg_unit;  // flat groups (g_flat_cols): units of group g = fg_unit[fg_ptr[g] ..)
    std::vector<FlatDesc> fg_desc;         // per fg_unit entry
    // upper-triangle tiles (g_upper_tiles): the column side of a strictly
    // upper tile (J > J(its rows)) goes to an int64 slot of kW columns -- one
    // per tile of a tiled / flat unit (u_cslot[u] + tile offset), one per
    // flat column group (fg_cslot) -- and k_colsum adds, per column tile J,
    // the slots jslot[jslot_ptr[J] ..) in a fixed order (integers: exact)
    int upper = 0;
    int64_t row_lo = 0;
    std::vector<int32_t> u_cslot, fg_cslot, jslot_ptr, jslot;
    int64_t n_cslots = 0;
    int64_t n_units_flat = 0;
    int64_t payload_bytes_flat = 0;     // payload of the flat units' tiles
    int64_t n_entries_padded = 0;     // wide slots
    int64_t n_narrow_padded = 0;      // narrow slots
    int64_t n_part = 0;
};

// Build the plan from per-(local row, tile) wide and narrow entry counts
// (row-major, nloc x nJ, unpadded; cntn may be null).  row_group: ICE group
// per local row.  Units are sized in 4-byte payload words.
TilePlan plan_tiles(const uint16_t* cntw, const uint16_t* cntn, int64_t nloc, int32_t nJ,
                    const std::vector<uint16_t>& row_group, int64_t row_lo, bool upper);
// a tile of (local) row-block rb and column tile J holds the column side
__host__ __device__ __forceinline__ bool tile_is_upper(int upper, long long row_lo, int rb, int J) {
    return upper && J > (int)((row_lo + (long long)rb * kR) >> kWBits);
}

struct TileDev {
    const uint32_t* pay;
    const uint16_t* payn;
    const int32_t* tile_J;
    const long long* tile_ent;
    const uint32_t* tile_rp;
    const long long* tile_entn;
    const uint32_t* tile_rpn;
    const int32_t* u_tlo;
    const int32_t* u_thi;
    const int32_t* u_rb;
    const int32_t* u_rlo;
    const int32_t* u_rhi;
    const int32_t* u_slot;
    const uint16_t* u_glo;
    const uint16_t* u_ghi;
    const int32_t* blk_unit_ptr;
    const int32_t* u_order;
    const uint16_t* tile_perm;
    const uint16_t* tile_band;
    const uint32_t* tile_fw;
    const int32_t* tile_frec;
    const uint4* frec;
    const uint8_t* u_whole;
    const int32_t* fg_ptr;
    const int32_t* fg_unit;
    const FlatDesc* fg_desc;
    int flat_defer;  // flat kernel: merge a tile's compact sums after the next tile's barrier (hh_tune "flat_defer")
    int upper;                      // the layout has upper-triangle tiles
    long long row_lo;               // first row of the matrix (global)
    const int32_t* u_cslot;         // per unit: its tiles' column slots (upper)
    const int32_t* fg_cslot;        // per flat group: its column slot (upper)
    unsigned long long* colpart;    // n_cslots x kW column partials (int64 fixed point)
    const double* fix;              // {2^e, 2^-e}: this sweep's fixed-point scale of b
    const unsigned long long* bfix; // B = round(b 2^e) of every bin (k_fixscale)
};

extern int g_flat_defer;

}  // namespace hh

struct hh_matrix {
    int device = 0;
    int64_t n_bins = 0, row_lo = 0, row_hi = 0;
    int32_t n_chroms = 0, ignore_diags = 1, cis_only = 0;
    std::vector<int64_t> chrom_offsets;
    int64_t nnz_upper = 0;
    int64_t n_entries = 0;        // stored off-diagonal entries (both triangles)
    int64_t n_tiles = 0, n_units = 0, n_part = 0, n_wide = 0, nJ = 0, nrb = 0;
    int64_t n_units_flat = 0;     // units swept by k_sweep_flat (the last entries of u_order)
    int64_t payload_bytes_flat = 0;
    int64_t n_slots = 0;          // padded wide (uint32) entries in tiles
    int64_t n_slots_narrow = 0;   // padded narrow (uint16) entries in tiles
    int32_t band_w = 0;           // uint8 band half-width W8 (0 = no band)
    int32_t band_w4 = 0;          // nibble band outer width W4 (== band_w: none)
    int64_t n_band = 0;           // nonzero entries held by the bands
    hh::DBuf<uint8_t> band;       // local rows x band_stride(W8)
    hh::DBuf<uint8_t> band4;      // local rows x band4_stride(W8, W4)
    hh::DBuf<uint32_t> pay;
    hh::DBuf<uint16_t> payn;
    hh::DBuf<int32_t> tile_J, tile_rb;
    hh::DBuf<long long> tile_ent, tile_entn;
    hh::DBuf<uint32_t> tile_rp, tile_rpn;
    hh::DBuf<int32_t> u_tlo, u_thi, u_rb, u_rlo, u_rhi, u_slot, blk_unit_ptr, blk_tile_ptr, u_order;
    hh::DBuf<uint16_t> u_glo, u_ghi, tile_perm, tile_band;
    hh::DBuf<uint32_t> tile_fw;
    hh::DBuf<int32_t> tile_frec;
    hh::DBuf<uint16_t> frec;
    hh::DBuf<uint8_t> u_whole;
    hh::DBuf<int32_t> fg_ptr, fg_unit;  // column groups of the flat units (g_flat_cols)
    hh::DBuf<hh::FlatDesc> fg_desc;
    int64_t n_fgroups = 0;
    int32_t upper = 0;             // upper-triangle tiles (g_upper_tiles at build time)
    int32_t flat_perm = 0;         // column-grouped flat tiles' narrow segments interleaved (finalize_flat_layout)
    int64_t n_cslots = 0;
    hh::DBuf<int32_t> u_cslot, fg_cslot, jslot_ptr, jslot;
    hh::DBuf<long long> wide_ptr;  // local rows + 1
    hh::DBuf<int32_t> wide_col;
    hh::DBuf<double> wide_cnt;
    hh::DBuf<double> diag;        // local rows: diagonal count (0 when ignored)
    hh::DBuf<double> row_nnz2;    // local rows: cooler nnz marginal (binarised)
    hh::DBuf<double> row_sum2;    // local rows: cooler raw marginal
    hh::DBuf<uint16_t> row_group; // local rows: ICE group id
    int64_t nloc() const { return row_hi - row_lo; }
    size_t device_bytes() const {
        return pay.bytes() + payn.bytes() + tile_entn.bytes() + tile_rpn.bytes() + tile_J.bytes() +
               tile_rb.bytes() + tile_ent.bytes() + tile_rp.bytes() +
               u_tlo.bytes() * 7 + blk_unit_ptr.bytes() + tile_perm.bytes() + tile_band.bytes() + u_whole.bytes() + tile_fw.bytes() + tile_frec.bytes() + frec.bytes() + blk_tile_ptr.bytes() + u_glo.bytes() * 2 +
               fg_ptr.bytes() + fg_unit.bytes() + fg_desc.bytes() + u_cslot.bytes() + fg_cslot.bytes() +
               jslot_ptr.bytes() + jslot.bytes() +
               wide_ptr.bytes() + wide_col.bytes() + wide_cnt.bytes() + diag.bytes() + row_nnz2.bytes() +
               row_sum2.bytes() + row_group.bytes() + band.bytes() + band4.bytes();
    }
    hh::TileDev dev(unsigned long long* colpart = nullptr, const double* fix = nullptr,
                    const unsigned long long* bfix = nullptr) const {
        return hh::TileDev{pay.p, payn.p, tile_J.p, tile_ent.p, tile_rp.p, tile_entn.p, tile_rpn.p, u_tlo.p,
                           u_thi.p, u_rb.p, u_rlo.p, u_rhi.p, u_slot.p, u_glo.p, u_ghi.p, blk_unit_ptr.p,
                           u_order.p, tile_perm.p, tile_band.p, tile_fw.p, tile_frec.p,
                           reinterpret_cast<const uint4*>(frec.p), u_whole.p, fg_ptr.p, fg_unit.p, fg_desc.p,
                           hh::g_flat_defer, upper && colpart ? 1 : 0, (long long)row_lo, u_cslot.p, fg_cslot.p,
                           colpart, fix, bfix};
    }
};

namespace hh {
// Group id of a bin: chromosome index when cis_only, else 0.
inline std::vector<uint16_t> bin_groups(const hh_matrix& m) {
    std::vector<uint16_t> g(m.n_bins, 0);
    if (m.cis_only)
        for (int c = 0; c < m.n_chroms; ++c)
            for (int64_t b = m.chrom_offsets[c]; b < m.chrom_offsets[c + 1]; ++b) g[b] = (uint16_t)c;
    return g;
}
// Upload the plan arrays (not the payload) into m.
void upload_plan(const TilePlan& P, hh_matrix& m, hipStream_t s);

// Interleaved flat segments (round 6).  The flat walk gives lane l of a wave
// the run of kFlatIlvU consecutive uint4 [q0 + U l, q0 + U l + U) of a step;
// loaded as such (lane-major) every load instruction touches 64 lines 128 B
// apart, and the flat tiles stream at 3.5 TB/s however many loads are in
// flight (hh_matrix_stream_probe: 6.0 TB/s for the same tiles with coalesced
// instructions).  So the column-grouped flat tiles' narrow segments are stored
// per step chunk of m <= 64 U uint4 (chunks aligned to the segment start) in
// element-major order: element k of every lane's run first (lanes 0 ..
// cnt_k - 1, cnt_k = ceil((m - k) / U)), then element k + 1: instruction k
// of a step reads cnt_k consecutive uint4 into exactly the registers the
// lane-major load filled -- the walk and its sums are unchanged, bitwise.
constexpr int kFlatIlvU = 8;
__host__ __device__ inline uint32_t flat_ilv_cnt(uint32_t m, int k) {
    return m > (uint32_t)k ? (m - (uint32_t)k + kFlatIlvU - 1) / kFlatIlvU : 0u;
}
// chunk-relative stored position of chunk-relative logical uint4 i (chunk of m)
__host__ __device__ inline uint32_t flat_ilv_pos(uint32_t m, uint32_t i) {
    const int k = (int)(i % kFlatIlvU);
    uint32_t b = 0;
    for (int j = 0; j < k; ++j) b += flat_ilv_cnt(m, j);
    return b + i / kFlatIlvU;
}
// After a builder wrote the payload: interleave the column-grouped flat
// tiles' narrow segments (m.flat_perm = 1); no-op without column groups.
void finalize_flat_layout(hh_matrix& m, hipStream_t s);
// A copy of m's narrow payload in the plain (lane-major) order (export).
void narrow_payload_plain(const hh_matrix& m, DBuf<uint16_t>& out, hipStream_t s);
// Device helpers shared with the pair binner (pairs.hip): stable LSD radix
// sort of n 64-bit keys on their low `bits` bits (synchronous), exclusive
// scan of n int64 values (*total_dev = the sum, may be null; asynchronous).
// stable LSD radix sort of the key bits [lo_bit, lo_bit + bits) (keys whose
// lower bits are already in order -- an index -- need only the upper ones)
void dev_sort_u64(DBuf<unsigned long long>& keys, int64_t n, int bits, hipStream_t s, int lo_bit = 0);
int64_t dev_sort_cells_by_col(const int32_t* r, const int32_t* c, const uint32_t* v, int64_t nnz, int fmt, int ib,
                              int cbits, DBuf<unsigned long long>& keys, hipStream_t s);
void dev_excl_scan_i64(const long long* in, long long* out, long long n, unsigned long long* total_dev, hipStream_t s);
// Device build from a host pixel table (build.hip); false = not a sorted
// upper-triangle table (nothing built).  g_host_build forces the host builder.
bool build_from_host_pixels_on_device(const int64_t* bin1, const int64_t* bin2, const double* count, int64_t nnz,
                                      int64_t n_bins, const int64_t* chrom_offsets, int32_t n_chroms,
                                      int32_t ignore_diags, int32_t cis_only, int64_t row_lo, int64_t row_hi,
                                      hipStream_t s, hh_matrix** out);
extern int64_t g_host_build;
extern int64_t g_build_debug;  // hh_tune("build_debug"): device-build phase times on stderr
}  // namespace hh
