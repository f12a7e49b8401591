// Internal layout of the HBM-resident contact matrix ("tiled pixel" layout,
// DESIGN.md §3) and of its build plan.  Not part of the C-ABI.
//
// The symmetric matrix (both triangles of cooler's pixel table) is cut into
// row-blocks of kR = 256 rows (global alignment: block = row / 256) and column
// tiles of kW = 8192 columns.  A nonempty (row-block, tile) pair is a *tile*:
// its entries are stored row by row (each row's list column-sorted and padded
// to a multiple of 4 entries = 16 B), with kR + 1 row pointers.  An entry is
// a uint32 = count << 13 | (col - tile_start); counts >= 2^19 go to a small
// per-row "wide" list instead.  The sweep kernel stages the tile's 8192 bias
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

constexpr int kR = 256;                 // rows per row-block
constexpr int kWBits = 13;
constexpr int kW = 1 << kWBits;         // columns per tile
constexpr uint32_t kColMask = kW - 1;
constexpr uint32_t kCntMax = (1u << (32 - kWBits)) - 1u;  // 2^19 - 1
extern int64_t g_unit_entries;                           // ~512 KiB of payload per unit (hh_tune)
constexpr int64_t kMaxBins = (int64_t)1 << 30;

inline int64_t pad4(int64_t x) { return (x + 3) & ~(int64_t)3; }

// Host plan + arrays of the tiled layout.
struct TilePlan {
    int64_t nloc = 0;      // local rows
    int64_t nrb = 0;       // local row-blocks
    int32_t nJ = 0;        // column tiles over the whole matrix
    std::vector<int32_t> tile_J;      // per tile
    std::vector<int64_t> tile_ent;    // per tile: first entry (multiple of 4)
    std::vector<uint32_t> tile_rp;    // per tile: kR + 1 row offsets (relative)
    std::vector<int32_t> tile_rb;     // per tile: local row-block
    std::vector<int32_t> blk_tile_ptr;  // nrb + 1
    std::vector<int32_t> tile_of;     // nrb * nJ -> tile index or -1
    // units
    std::vector<int32_t> u_tlo, u_thi, u_rb, u_rlo, u_rhi, u_slot;
    std::vector<uint16_t> u_glo, u_ghi;
    std::vector<int32_t> blk_unit_ptr;  // nrb + 1
    int64_t n_entries_padded = 0;
    int64_t n_part = 0;
};

// Build the plan from per-(local row, tile) entry counts (row-major,
// nloc x nJ, unpadded).  row_group: ICE group per local row.
TilePlan plan_tiles(const uint16_t* cnt, int64_t nloc, int32_t nJ, const std::vector<uint16_t>& row_group);

struct TileDev {
    const uint32_t* pay;
    const int32_t* tile_J;
    const long long* tile_ent;
    const uint32_t* tile_rp;
    const int32_t* u_tlo;
    const int32_t* u_thi;
    const int32_t* u_rb;
    const int32_t* u_rlo;
    const int32_t* u_rhi;
    const int32_t* u_slot;
    const uint16_t* u_glo;
    const uint16_t* u_ghi;
    const int32_t* blk_unit_ptr;
};

}  // namespace hh

struct hh_matrix {
    int device = 0;
    int64_t n_bins = 0, row_lo = 0, row_hi = 0;
    int32_t n_chroms = 0, ignore_diags = 1, cis_only = 0;
    std::vector<int64_t> chrom_offsets;
    int64_t nnz_upper = 0;
    int64_t n_entries = 0;        // stored off-diagonal entries (both triangles)
    int64_t n_tiles = 0, n_units = 0, n_part = 0, n_wide = 0, nJ = 0, nrb = 0;
    int64_t n_slots = 0;          // padded entries in tiles
    hh::DBuf<uint32_t> pay;
    hh::DBuf<int32_t> tile_J, tile_rb;
    hh::DBuf<long long> tile_ent;
    hh::DBuf<uint32_t> tile_rp;
    hh::DBuf<int32_t> u_tlo, u_thi, u_rb, u_rlo, u_rhi, u_slot, blk_unit_ptr, blk_tile_ptr;
    hh::DBuf<uint16_t> u_glo, u_ghi;
    hh::DBuf<long long> wide_ptr;  // local rows + 1
    hh::DBuf<int32_t> wide_col;
    hh::DBuf<double> wide_cnt;
    hh::DBuf<double> diag;        // local rows: diagonal count (0 when ignored)
    hh::DBuf<double> row_nnz2;    // local rows: cooler nnz marginal (binarised)
    hh::DBuf<double> row_sum2;    // local rows: cooler raw marginal
    hh::DBuf<uint16_t> row_group; // local rows: ICE group id
    int64_t nloc() const { return row_hi - row_lo; }
    size_t device_bytes() const {
        return pay.bytes() + tile_J.bytes() + tile_rb.bytes() + tile_ent.bytes() + tile_rp.bytes() +
               u_tlo.bytes() * 6 + blk_unit_ptr.bytes() + blk_tile_ptr.bytes() + u_glo.bytes() * 2 +
               wide_ptr.bytes() + wide_col.bytes() + wide_cnt.bytes() + diag.bytes() + row_nnz2.bytes() +
               row_sum2.bytes() + row_group.bytes();
    }
    hh::TileDev dev() const {
        return hh::TileDev{pay.p, tile_J.p, tile_ent.p, tile_rp.p, u_tlo.p, u_thi.p, u_rb.p, u_rlo.p,
                           u_rhi.p, u_slot.p, u_glo.p, u_ghi.p, blk_unit_ptr.p};
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
}  // namespace hh
