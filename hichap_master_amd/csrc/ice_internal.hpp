// Internal layout of the HBM-resident contact matrix ("pixel-chunk" layout,
// DESIGN.md §3) and of the ICE state.  Not part of the C-ABI.
#pragma once

#include "hh_common.hpp"

namespace hh {

// Entries per chunk and chunks per segment (the unit of work of one wave in
// the sweep kernel).  A chunk is 256 uint32 = 1 KiB = one uint4 per lane.
// Entry = (count << k) | (col - base) with a per-chunk split k = bits needed
// for the chunk's column span; a chunk closes when full or when
// bits(span) + bits(max count) would exceed 32 (so any count < 2^32 fits).
constexpr int kChunk = 256;
constexpr int kSegChunks = 8;
// Chunk header: base column (27 bits, n_bins < 2^27) | k << 27.
constexpr int kHdrShift = 27;
constexpr uint32_t kHdrBaseMask = (1u << kHdrShift) - 1u;
constexpr int64_t kMaxBins = (int64_t)1 << kHdrShift;

__host__ __device__ __forceinline__ int nbits(uint32_t x) { return x ? 32 - __builtin_clz(x) : 0; }
__host__ __device__ __forceinline__ uint32_t make_hdr(int64_t base, int k) {
    return (uint32_t)base | ((uint32_t)k << kHdrShift);
}
// Slot-major chunk: entry q sits in lane q % 64, component q / 64, so one
// wave-wide component load reads 64 consecutive entries (coalesced gathers of
// b for the near-diagonal band).
__host__ __device__ __forceinline__ int slot_of(int q) { return ((q & 63) << 2) | (q >> 6); }

// The chunks of the stored rows.
struct ChunkLayer {
    DBuf<uint32_t> pay;        // n_chunks * 256 packed entries
    DBuf<uint32_t> hdr;        // n_chunks: make_hdr(first column, k)
    DBuf<int32_t> seg_begin;   // n_segs + 1 (chunk index)
    DBuf<int32_t> row_seg;     // n_local_rows + 1 (segment index)
    DBuf<uint16_t> seg_group;  // n_segs: ICE group of the segment's row
    int64_t n_chunks = 0;
    int64_t n_segs = 0;
    int64_t n_entries = 0;
    size_t bytes() const {
        return pay.bytes() + hdr.bytes() + seg_begin.bytes() + row_seg.bytes() +
               seg_group.bytes();
    }
};

// Host-side chunk layer under construction.
struct HostLayer {
    std::vector<uint32_t> pay;
    std::vector<uint32_t> hdr;
    std::vector<int32_t> seg_begin;
    std::vector<int32_t> row_seg;
    std::vector<uint16_t> seg_group;
    int64_t n_entries = 0;
};

}  // namespace hh

struct hh_matrix {
    int device = 0;
    int64_t n_bins = 0, row_lo = 0, row_hi = 0;
    int32_t n_chroms = 0, ignore_diags = 1, cis_only = 0;
    std::vector<int64_t> chrom_offsets;
    int64_t nnz_upper = 0;
    hh::ChunkLayer main;
    hh::DBuf<double> diag;      // local rows: diagonal count (0 when ignored)
    hh::DBuf<double> row_nnz2;  // local rows: cooler nnz marginal (binarised)
    hh::DBuf<double> row_sum2;  // local rows: cooler raw marginal
    hh::DBuf<uint16_t> row_group;  // local rows: ICE group id
    int64_t nloc() const { return row_hi - row_lo; }
    size_t device_bytes() const {
        return main.bytes() + diag.bytes() + row_nnz2.bytes() + row_sum2.bytes() +
               row_group.bytes();
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
// Upload a host layer; segments are cut from per-row chunk counts.
void upload_layer(const HostLayer& h, ChunkLayer& d, hipStream_t s);
// Build segment tables from per-local-row chunk counts.
void make_segments(const std::vector<int64_t>& row_chunks, const std::vector<uint16_t>& row_group,
                   HostLayer& h);
}  // namespace hh
