// Contact-matrix construction in HBM: cooler pixel table -> pixel-chunk
// layout (host build + upload), and the on-device synthetic genome generator.
//
// Layout: the symmetric matrix stored row by row; each row's
// off-diagonal entries, sorted by column, are cut into chunks of 256 packed
// uint32 entries (count << k | col - base) with an int32 base column and a
// column-offset width k per chunk (ice_internal.hpp).  Chunks of a row are
// grouped into segments of <= 8 chunks (one wave of the sweep kernel each).
#include <algorithm>
#include <cmath>
#include <numeric>

#include "ice_internal.hpp"

namespace hh {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

void make_segments(const std::vector<int64_t>& row_chunks, const std::vector<uint16_t>& row_group,
                   HostLayer& h) {
    const size_t nloc = row_chunks.size();
    h.row_seg.assign(nloc + 1, 0);
    h.seg_begin.clear();
    h.seg_group.clear();
    int64_t chunk = 0;
    for (size_t r = 0; r < nloc; ++r) {
        h.row_seg[r] = (int32_t)h.seg_begin.size();
        for (int64_t k = 0; k < row_chunks[r]; k += kSegChunks) {
            h.seg_begin.push_back((int32_t)(chunk + k));
            h.seg_group.push_back(row_group[r]);
        }
        chunk += row_chunks[r];
    }
    h.row_seg[nloc] = (int32_t)h.seg_begin.size();
    h.seg_begin.push_back((int32_t)chunk);
    if (chunk > INT32_MAX - 1) HH_THROW(HH_ERR_ARG, "too many chunks for one shard (> 2^31); use more ranks");
}

void upload_layer(const HostLayer& h, ChunkLayer& d, hipStream_t s) {
    d.n_chunks = (int64_t)h.hdr.size();
    d.n_segs = (int64_t)h.seg_group.size();
    d.n_entries = h.n_entries;
    d.pay = to_device(h.pay, s);
    d.hdr = to_device(h.hdr, s);
    d.seg_begin = to_device(h.seg_begin, s);
    d.row_seg = to_device(h.row_seg, s);
    d.seg_group = to_device(h.seg_group, s);
}

// Append one row (sorted columns) to a host layer; returns the chunks added.
static int64_t chunk_row(const int32_t* cols, const uint32_t* vals, int64_t n, HostLayer& h) {
    int64_t added = 0;
    int64_t k = 0;
    while (k < n) {
        const int32_t b = cols[k];
        const int64_t start = k;
        uint32_t maxc = 0;
        while (k < n && k - start < kChunk) {
            const uint32_t mc = std::max(maxc, vals[k]);
            if (nbits((uint32_t)(cols[k] - b)) + nbits(mc) > 32) break;
            maxc = mc;
            ++k;
        }
        const int kb = nbits((uint32_t)(cols[k - 1] - b));
        const size_t off = h.pay.size();
        h.pay.resize(off + kChunk, 0u);
        for (int64_t q = start; q < k; ++q)
            h.pay[off + slot_of((int)(q - start))] = (uint32_t)((uint64_t)vals[q] << kb) | (uint32_t)(cols[q] - b);
        h.hdr.push_back(make_hdr(b, kb));
        h.n_entries += k - start;
        ++added;
    }
    return added;
}

}  // namespace hh

using namespace hh;

extern "C" {

const char* hh_last_error(void) { return g_last_error.c_str(); }
int hh_version(void) { return (0 << 16) | (1 << 8) | 0; }

int hh_device_count(int32_t* n) {
    return guard([&] {
        int c = 0;
        HIP_CHECK(hipGetDeviceCount(&c));
        *n = c;
    });
}

int hh_set_device(int32_t device) {
    return guard([&] { HIP_CHECK(hipSetDevice(device)); });
}

int hh_synchronize(void* stream) {
    return guard([&] { HIP_CHECK(hipStreamSynchronize(as_stream(stream))); });
}

int hh_matrix_from_pixels(const int64_t* bin1, const int64_t* bin2, const double* count, int64_t nnz,
                          int64_t n_bins, const int64_t* chrom_offsets, int32_t n_chroms,
                          int32_t ignore_diags, int32_t cis_only, int64_t row_lo, int64_t row_hi,
                          void* stream, hh_matrix** out) {
    return guard([&] {
        HH_REQUIRE(out && n_bins > 0 && nnz >= 0 && n_chroms > 0 && chrom_offsets, "bad arguments");
        HH_REQUIRE(nnz == 0 || (bin1 && bin2 && count), "null pixel arrays");
        HH_REQUIRE(n_bins < kMaxBins, "n_bins must be < 2^27");
        HH_REQUIRE(0 <= row_lo && row_lo <= row_hi && row_hi <= n_bins, "bad row range");
        HH_REQUIRE(chrom_offsets[0] == 0 && chrom_offsets[n_chroms] == n_bins, "chrom_offsets must span [0, n_bins]");
        HH_REQUIRE(n_chroms < 65535, "too many chromosomes");
        HH_REQUIRE(ignore_diags >= 0, "ignore_diags must be >= 0");
        hipStream_t s = as_stream(stream);
        auto m = std::make_unique<hh_matrix>();
        HIP_CHECK(hipGetDevice(&m->device));
        m->n_bins = n_bins;
        m->row_lo = row_lo;
        m->row_hi = row_hi;
        m->n_chroms = n_chroms;
        m->ignore_diags = ignore_diags;
        m->cis_only = cis_only ? 1 : 0;
        m->chrom_offsets.assign(chrom_offsets, chrom_offsets + n_chroms + 1);
        std::vector<int32_t> chrom_of(n_bins);
        for (int c = 0; c < n_chroms; ++c) {
            HH_REQUIRE(chrom_offsets[c] <= chrom_offsets[c + 1], "chrom_offsets not monotone");
            for (int64_t b = chrom_offsets[c]; b < chrom_offsets[c + 1]; ++b) chrom_of[b] = c;
        }
        const int64_t nloc = row_hi - row_lo;
        std::vector<double> diag(nloc, 0.0), rnnz(nloc, 0.0), rsum(nloc, 0.0);
        std::vector<int64_t> deg(nloc + 1, 0);
        // pass 1: validate, filter, count row degrees
        auto keep = [&](int64_t i, int64_t& a, int64_t& b, uint32_t& c) -> bool {
            a = bin1[i];
            b = bin2[i];
            const double v = count[i];
            if (a > b) std::swap(a, b);
            if (a < 0 || b >= n_bins) HH_THROW(HH_ERR_ARG, "bin id out of range at pixel " + std::to_string(i));
            if (!(v >= 0.0) || v != std::floor(v) || v >= 4294967296.0)
                HH_THROW(HH_ERR_ARG, "counts must be non-negative integers < 2^32 (pixel " + std::to_string(i) + ")");
            if (v == 0.0) return false;
            if (cis_only && chrom_of[a] != chrom_of[b]) return false;
            if (b - a < ignore_diags) return false;
            c = (uint32_t)v;
            return true;
        };
        int64_t nnz_upper = 0;
        for (int64_t i = 0; i < nnz; ++i) {
            int64_t a, b;
            uint32_t c;
            if (!keep(i, a, b, c)) continue;
            const bool ina = a >= row_lo && a < row_hi, inb = b >= row_lo && b < row_hi;
            if (a == b) {
                if (ina) {
                    diag[a - row_lo] += c;
                    rnnz[a - row_lo] += 2.0;
                    rsum[a - row_lo] += 2.0 * c;
                    ++nnz_upper;
                }
                continue;
            }
            if (ina) { ++deg[a - row_lo + 1]; ++nnz_upper; rnnz[a - row_lo] += 1.0; rsum[a - row_lo] += c; }
            if (inb) { ++deg[b - row_lo + 1]; rnnz[b - row_lo] += 1.0; rsum[b - row_lo] += c; }
        }
        for (int64_t r = 0; r < nloc; ++r) deg[r + 1] += deg[r];
        std::vector<int32_t> cols(deg[nloc]);
        std::vector<uint32_t> vals(deg[nloc]);
        std::vector<int64_t> pos(deg.begin(), deg.end() - 1);
        for (int64_t i = 0; i < nnz; ++i) {
            int64_t a, b;
            uint32_t c;
            if (!keep(i, a, b, c) || a == b) continue;
            if (a >= row_lo && a < row_hi) { cols[pos[a - row_lo]] = (int32_t)b; vals[pos[a - row_lo]++] = c; }
            if (b >= row_lo && b < row_hi) { cols[pos[b - row_lo]] = (int32_t)a; vals[pos[b - row_lo]++] = c; }
        }
        // rows must be column-sorted for chunking; sort rows that are not
        std::vector<std::pair<int32_t, uint32_t>> tmp;
        for (int64_t r = 0; r < nloc; ++r) {
            const int64_t lo = deg[r], hi = deg[r + 1];
            if (std::is_sorted(cols.begin() + lo, cols.begin() + hi)) continue;
            tmp.clear();
            for (int64_t k = lo; k < hi; ++k) tmp.emplace_back(cols[k], vals[k]);
            std::stable_sort(tmp.begin(), tmp.end(), [](auto& x, auto& y) { return x.first < y.first; });
            for (int64_t k = lo; k < hi; ++k) { cols[k] = tmp[k - lo].first; vals[k] = tmp[k - lo].second; }
        }
        // chunk layer
        std::vector<uint16_t> bg = bin_groups(*m);
        std::vector<uint16_t> rgroup(bg.begin() + row_lo, bg.begin() + row_hi);
        HostLayer hm;
        std::vector<int64_t> rc(nloc, 0);
        hm.pay.reserve((size_t)(deg[nloc] + nloc * 64));
        for (int64_t r = 0; r < nloc; ++r)
            rc[r] = chunk_row(cols.data() + deg[r], vals.data() + deg[r], deg[r + 1] - deg[r], hm);
        make_segments(rc, rgroup, hm);
        upload_layer(hm, m->main, s);
        m->diag = to_device(diag, s);
        m->row_nnz2 = to_device(rnnz, s);
        m->row_sum2 = to_device(rsum, s);
        m->row_group = to_device(rgroup, s);
        m->nnz_upper = nnz_upper;
        HIP_CHECK(hipStreamSynchronize(s));  // host vectors die here
        *out = m.release();
    });
}

int hh_matrix_free(hh_matrix* m) {
    return guard([&] { delete m; });
}

int hh_matrix_get_info(const hh_matrix* m, hh_matrix_info* info) {
    return guard([&] {
        HH_REQUIRE(m && info, "null");
        info->n_bins = m->n_bins;
        info->row_lo = m->row_lo;
        info->row_hi = m->row_hi;
        info->nnz_upper = m->nnz_upper;
        info->n_entries = m->main.n_entries;
        info->n_slots = m->main.n_chunks * kChunk;
        info->n_chunks = m->main.n_chunks;
        info->n_segments = m->main.n_segs;
        info->n_ovf_chunks = 0;
        info->device_bytes = (int64_t)m->device_bytes();
        info->n_chroms = m->n_chroms;
        info->ignore_diags = m->ignore_diags;
        info->cis_only = m->cis_only;
        info->device = m->device;
    });
}

int hh_matrix_export_upper(const hh_matrix* m, int64_t* bin1, int64_t* bin2, double* count,
                           int64_t* nnz_inout) {
    return guard([&] {
        HH_REQUIRE(m && nnz_inout, "null");
        HIP_CHECK(hipSetDevice(m->device));
        const int64_t nloc = m->nloc();
        const ChunkLayer& L = m->main;
        std::vector<uint32_t> pay(L.pay.n);
        std::vector<uint32_t> hdr(L.hdr.n);
        std::vector<int32_t> row_seg(L.row_seg.n), seg_begin(L.seg_begin.n);
        std::vector<double> diag(nloc);
        HIP_CHECK(hipDeviceSynchronize());
        L.pay.download(pay.data(), pay.size(), 0);
        L.hdr.download(hdr.data(), hdr.size(), 0);
        L.row_seg.download(row_seg.data(), row_seg.size(), 0);
        L.seg_begin.download(seg_begin.data(), seg_begin.size(), 0);
        m->diag.download(diag.data(), nloc, 0);
        HIP_CHECK(hipDeviceSynchronize());
        int64_t cnt = 0;
        const int64_t cap = *nnz_inout;
        auto emit = [&](int64_t i, int64_t j, double v) {
            if (v == 0.0) return;
            if (cnt < cap && bin1) { bin1[cnt] = i; bin2[cnt] = j; count[cnt] = v; }
            ++cnt;
        };
        for (int64_t r = 0; r < nloc; ++r) {
            const int64_t gr = m->row_lo + r;
            emit(gr, gr, diag[r]);
            const int64_t c0 = seg_begin[row_seg[r]], c1 = seg_begin[row_seg[r + 1]];
            for (int64_t c = c0; c < c1; ++c) {
                const int kb = (int)(hdr[c] >> kHdrShift);
                const int64_t base = hdr[c] & kHdrBaseMask;
                const uint32_t mask = kb ? (0xFFFFFFFFu >> (32 - kb)) : 0u;
                for (int k = 0; k < kChunk; ++k) {
                    const uint32_t e = pay[(size_t)c * kChunk + slot_of(k)];
                    const int64_t col = base + (int64_t)(e & mask);
                    const double v = kb == 32 ? 0.0 : (double)(e >> kb);
                    if (col > gr) emit(gr, col, v);
                }
            }
        }
        *nnz_inout = cnt;
    });
}

}  // extern "C"
