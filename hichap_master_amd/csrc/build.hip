// Device build of the tiled pixel layout (ice_internal.hpp)
// straight from cooler's pixel table — the input of every `cooler balance`
// HiCHap runs (matrixBuilding.py:699-714: pixels/bin1_id, bin2_id, count,
// sorted by (bin1, bin2), bin1 <= bin2, unique).  Replaces the host builder
// (matrix.hip) for sorted tables; the table is read once from HBM and the
// symmetric row structure is made on the device:
//
//   k_px_check   validate (range, upper triangle, strict (bin1, bin2) order =
//                sorted + unique, integral counts), apply cooler's static
//                filters (zero counts, --ignore-diags, --cis-only zero_trans)
//                into a uint32 count array (0 = dropped), and histogram the
//                near-diagonal occupancy the band widths are chosen from (over
//                the WHOLE table, so every shard picks the same bands)
//   k_px_rowptr  row starts of the upper half (the table is sorted by bin1)
//   k_px_lowkeys the lower half, (bin2 - row_lo) << ib | pixel index for the
//                local rows, radix-sorted (pairs.hip) into per-row lists
//                sorted by column
//   k_px_rows<0> one wave per local row walks lower then upper entries (one
//                column-sorted sequence): per (row, tile) narrow / wide
//                counts, band entries, wide-list sizes, cooler's static
//                marginals; the host plans tiles and units (plan_tiles, as
//                for the synthetic generator)
//   k_px_rows<1> the same walk writes payload, bands and the wide list
//
// Every write position is a function of the row's sorted entries only, so
// the layout (and the ICE sums over it) is identical to the host builder's.
#include <algorithm>
#include <cmath>
#include <numeric>

#include <chrono>
#include <cstdio>

#include "ice_internal.hpp"

namespace hh {

struct PxErr {
    unsigned long long first;  // smallest offending pixel index (ULLONG_MAX: none)
    int code;                  // of that pixel: 1 range, 2 bin1 > bin2, 3 unsorted, 4 duplicate, 5 count
};

constexpr int kOccCopies = 64;

template <class Id, class Cnt>
__global__ __launch_bounds__(256) void k_px_check(const Id* __restrict__ b1, const Id* __restrict__ b2,
                                                  const Cnt* __restrict__ cnt, long long nnz, long long n_bins,
                                                  const int32_t* __restrict__ chrom_of, int ignore_diags,
                                                  int cis_only, int32_t* __restrict__ A, int32_t* __restrict__ B,
                                                  uint32_t* __restrict__ kc, unsigned* __restrict__ occ,
                                                  unsigned* __restrict__ big, int occ_max,
                                                  unsigned long long* __restrict__ errs) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nnz) return;
    const long long a = (long long)b1[i], b = (long long)b2[i];
    const double v = (double)cnt[i];
    int code = 0;
    if (a < 0 || b >= n_bins || b < 0 || a >= n_bins) code = 1;
    else if (a > b) code = 2;
    else if (i > 0) {
        const long long pa = (long long)b1[i - 1], pb = (long long)b2[i - 1];
        if (pa > a || (pa == a && pb > b)) code = 3;
        else if (pa == a && pb == b) code = 4;
    }
    if (!code && (!(v >= 0.0) || v != floor(v) || v >= 4294967296.0)) code = 5;
    if (code) {
        // errs[code - 1] = smallest offending index of that kind
        atomicMin(errs + code - 1, (unsigned long long)i);
        kc[i] = 0u;
        A[i] = 0;
        B[i] = 0;
        return;
    }
    uint32_t c = (uint32_t)v;
    if (cis_only && chrom_of[a] != chrom_of[b]) c = 0u;
    if (b - a < ignore_diags) c = 0u;
    kc[i] = c;
    A[i] = (int32_t)a;
    B[i] = (int32_t)b;
    const long long d = b - a;
    if (c && d >= 1 && d <= occ_max) {
        // one of kOccCopies histogram copies per block: every row hits the
        // same near-diagonal counters, so one copy serialised ~n_bins atomics
        // per address (k_occ_reduce sums the copies)
        const long long o = (long long)(blockIdx.x % kOccCopies) * (occ_max + 1) + d;
        atomicAdd(occ + o, 1u);
        if (c > kBand4MaxCnt) atomicAdd(big + o, 1u);
    }
}

__global__ void k_occ_reduce(const unsigned* __restrict__ occ, const unsigned* __restrict__ big, int len,
                             unsigned* __restrict__ occ_out, unsigned* __restrict__ big_out) {
    const int d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= len) return;
    unsigned a = 0, b = 0;
    for (int k = 0; k < kOccCopies; ++k) {
        a += occ[(long long)k * len + d];
        b += big[(long long)k * len + d];
    }
    occ_out[d] = a;
    big_out[d] = b;
}

// ptr[r] = first i with A[i] >= r, r in [0, n_bins]  (A sorted, nnz >= 1)
__global__ void k_px_rowptr(const int32_t* __restrict__ A, long long nnz, long long n_bins,
                            long long* __restrict__ ptr) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > nnz) return;
    const long long lo = i == 0 ? -1 : (long long)A[i - 1];
    const long long hi = i == nnz ? n_bins : (long long)A[i];
    for (long long r = lo + 1; r <= hi; ++r) ptr[r] = i;
}

// same from the high bits of sorted lower keys: ptr[w] = first k with row >= w
__global__ void k_px_keyptr(const unsigned long long* __restrict__ keys, long long n, int ib, long long nloc,
                            long long* __restrict__ ptr) {
    const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (k > n) return;
    const long long lo = k == 0 ? -1 : (long long)(keys[k - 1] >> ib);
    const long long hi = k == n ? nloc : (long long)(keys[k] >> ib);
    for (long long r = lo + 1; r <= hi; ++r) ptr[r] = k;
}

// lower-half keys of the local rows (order fixed later by the sort)
// One block per kLowChunk pixels.  PASS 0: the block's number of lower-half
// keys -> cnt[block]; PASS 1: the keys at base[block] (exclusive scan of the
// counts) in pixel order.  The key array is then in index order, so the sort
// only has to order the row bits (stable LSD: ties keep index order) -- 3
// radix passes instead of 6-7 -- and no same-address atomics are involved.
constexpr int kLowItems = 16;
constexpr int kLowChunk = 256 * kLowItems;
template <int PASS>
__global__ __launch_bounds__(256) void k_px_lowkeys(const int32_t* __restrict__ A, const int32_t* __restrict__ B,
                                                    const uint32_t* __restrict__ kc, long long nnz, long long row_lo,
                                                    long long row_hi, int ib, unsigned long long* __restrict__ keys,
                                                    long long* __restrict__ cnt_or_base) {
    __shared__ unsigned wcnt[kLowItems][4];
    const long long c0 = (long long)blockIdx.x * kLowChunk;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned long long mk[kLowItems];
#pragma unroll
    for (int k = 0; k < kLowItems; ++k) {
        const long long i = c0 + (long long)k * 256 + threadIdx.x;
        bool take = false;
        if (i < nnz) {
            const long long b = B[i];
            take = kc[i] != 0u && A[i] < b && b >= row_lo && b < row_hi;
        }
        mk[k] = __ballot(take);
        if (lane == 0) wcnt[k][wave] = (unsigned)__popcll(mk[k]);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned tot = 0;
        for (int k = 0; k < kLowItems; ++k)
            for (int w = 0; w < 4; ++w) {
                const unsigned c = wcnt[k][w];
                wcnt[k][w] = tot;  // exclusive offset within the block
                tot += c;
            }
        if (PASS == 0) cnt_or_base[blockIdx.x] = tot;
    }
    if (PASS == 0) return;
    __syncthreads();
    const unsigned long long base = (unsigned long long)cnt_or_base[blockIdx.x];
#pragma unroll
    for (int k = 0; k < kLowItems; ++k) {
        if (!((mk[k] >> lane) & 1ull)) continue;
        const long long i = c0 + (long long)k * 256 + threadIdx.x;
        const long long b = B[i];
        keys[base + wcnt[k][wave] + __popcll(mk[k] & ((1ull << lane) - 1ull))] =
            ((unsigned long long)(b - row_lo) << ib) | (unsigned long long)i;
    }
}

// Sorted lower-half keys -> packed (column | count << 32), in place, once:
// the two row passes then read the lower half contiguously instead of each
// gathering A[i] and kc[i] at random (C3: 8e8 x 2 random 4-byte reads per pass).
__global__ void k_px_lowgather(unsigned long long* __restrict__ keys, long long n, unsigned long long imask,
                               const int32_t* __restrict__ A, const uint32_t* __restrict__ kc) {
    const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const long long i = (long long)(keys[q] & imask);
    keys[q] = (unsigned long long)(uint32_t)A[i] | ((unsigned long long)kc[i] << 32);
}

struct PxRows {
    const int32_t* A;
    const int32_t* B;
    const uint32_t* kc;
    const long long* up_ptr;            // n_bins + 1 (global rows)
    const unsigned long long* lkeys;    // lower half, row-sorted, packed (column | count << 32)
    const long long* lo_ptr;            // nloc + 1
    long long row_lo, nloc;
    int nJ, band_w, band_w4;
    int upper;  // g_upper_tiles: tile entries only where J(col) >= J(row)
    // PASS 0
    uint16_t* cnt;
    uint16_t* cntn;
    int32_t* row_band;
    long long* row_wide;
    long long* row_upper;
    long long* row_ent;
    double* diag;
    double* row_nnz2;
    double* row_sum2;
    // PASS 1
    const int32_t* tile_of;
    const long long* tile_ent;
    const uint32_t* tile_rp;
    const long long* tile_entn;
    const uint32_t* tile_rpn;
    uint32_t* pay;
    uint16_t* payn;
    uint8_t* band;
    uint32_t* band4;
    const long long* wide_ptr;
    int32_t* wide_col;
    double* wide_cnt;
};

template <int PASS>
__global__ __launch_bounds__(256) void k_px_rows(PxRows p) {
    const long long w = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (w >= p.nloc) return;
    const int lane = threadIdx.x & 63;
    const long long r = p.row_lo + w;
    const long long rb = w / kR;
    const int k = (int)(w % kR);
    const unsigned long long lt = (1ull << lane) - 1ull;
    int curJ = -1;
    long long tw = 0, tn = 0, pos = 0, posn = 0;
    long long nb_lane = 0, sum_lane = 0, ent_wave = 0, wide_wave = 0, upper_wave = 0;
    long long wpos = PASS == 1 ? p.wide_ptr[w] : 0;
    double dg = 0.0;
    auto flush = [&]() {
        if (curJ < 0) return;
        if (PASS == 0) {
            if (lane == 0) {
                p.cnt[w * p.nJ + curJ] = (uint16_t)tw;
                p.cntn[w * p.nJ + curJ] = (uint16_t)tn;
            }
        } else {
            const long long pw = (tw + 3) & ~3LL, pn = (tn + 7) & ~7LL;
            for (long long q = tw + lane; q < pw; q += 64) p.pay[pos - tw + q] = 0u;
            for (long long q = tn + lane; q < pn; q += 64) p.payn[posn - tn + q] = 0u;
        }
    };
    // one chunk of (up to) 64 column-sorted entries, one per lane
    auto chunk = [&](long long col, uint32_t v, bool valid) {
        if (valid && col == r) {  // the diagonal pixel (kept only when ignore_diags == 0)
            dg = (double)v;
            valid = false;
        }
        if (valid) sum_lane += v;
        const long long dj = col - r;
        const bool inband = valid && p.band_w > 0 && v <= kBandMaxCnt && dj >= -p.band_w && dj <= p.band_w;
        const bool innib = valid && !inband && in_band4(dj, v, p.band_w, p.band_w4);
        if (inband || innib) {
            if (PASS == 1) {
                if (inband) {
                    p.band[w * band_stride(p.band_w) + band_slot(dj, p.band_w)] = (uint8_t)v;
                } else {
                    const long long nib = w * 2 * band4_stride(p.band_w, p.band_w4) + band4_nibble(dj, p.band_w, p.band_w4);
                    atomicOr(p.band4 + (nib >> 3), v << (4 * (nib & 7)));
                }
            }
            nb_lane += 1;
            valid = false;
        }
        const bool wide = valid && v > kCntMax;
        const unsigned long long mwl = __ballot(wide);
        if (mwl) {
            if (PASS == 1 && wide) {
                const long long q = wpos + __popcll(mwl & lt);
                p.wide_col[q] = (int32_t)col;
                p.wide_cnt[q] = (double)v;
            }
            wpos += __popcll(mwl);
            wide_wave += __popcll(mwl);
            valid = valid && !wide;
        }
        const int J = (int)(col >> kWBits);
        unsigned long long mask = __ballot(valid);
        ent_wave += __popcll(mask) + __popcll(mwl);
        if (p.upper) {  // a lower-tile entry is stored as its mirror (the column side of row col)
            valid = valid && J >= (int)(r >> kWBits);
            mask = __ballot(valid);
        }
        while (mask) {
            const int first = __ffsll((long long)mask) - 1;
            const int Jr = __shfl(J, first, 64);
            const unsigned long long run = __ballot(valid && J == Jr);
            if (Jr != curJ) {
                flush();
                curJ = Jr;
                tw = tn = 0;
                if (PASS == 1) {
                    const int t = p.tile_of[rb * p.nJ + Jr];
                    pos = p.tile_ent[t] + p.tile_rp[(size_t)t * (kR + 1) + k];
                    posn = p.tile_entn[t] + p.tile_rpn[(size_t)t * (kR + 1) + k];
                }
            }
            const bool mine = (run >> lane) & 1ull;
            const bool narrow = mine && v <= kNarrowMax;
            const unsigned long long mn = __ballot(narrow), mw = run & ~mn;
            if (PASS == 1 && mine) {
                if (narrow) p.payn[posn + __popcll(mn & lt)] = enc_narrow((uint32_t)col & kColMask, v);
                else p.pay[pos + __popcll(mw & lt)] = enc_wide((uint32_t)col & kColMask, v);
            }
            const int nn = __popcll(mn), nw = __popcll(mw);
            tn += nn;
            tw += nw;
            posn += nn;
            pos += nw;
            mask &= ~run;
        }
    };
    // lower half: columns < r, the sorted keys replaced by their packed
    // (column, count) (k_px_lowgather): contiguous, no per-pass gathers
    const long long l0 = p.lo_ptr[w], l1 = p.lo_ptr[w + 1];
    for (long long q0 = l0; q0 < l1; q0 += 64) {
        const long long q = q0 + lane;
        const bool valid = q < l1;
        const unsigned long long x = valid ? p.lkeys[q] : 0ull;
        chunk((long long)(uint32_t)x, (uint32_t)(x >> 32), valid);
    }
    // upper half: columns >= r, the row's run of the table
    const long long u0 = p.up_ptr[r], u1 = p.up_ptr[r + 1];
    for (long long q0 = u0; q0 < u1; q0 += 64) {
        const long long q = q0 + lane;
        long long col = 0;
        uint32_t v = 0;
        bool valid = q < u1;
        if (valid) {
            col = p.B[q];
            v = p.kc[q];
            valid = v != 0u;
        }
        upper_wave += __popcll(__ballot(valid));
        chunk(col, v, valid);
    }
    flush();
    const long long nband = wave_sum_ll(nb_lane);
    const long long s = wave_sum_ll(sum_lane);
    dg = wave_sum(dg);  // one lane at most holds the diagonal
    if (PASS == 0 && lane == 0) {
        p.row_band[w] = (int32_t)nband;
        p.row_wide[w] = wide_wave;
        p.row_upper[w] = upper_wave;
        p.row_ent[w] = ent_wave + nband;
        p.diag[w] = dg;
        // cooler's static marginals: bincount(bin1) + bincount(bin2) of the
        // binarised / raw filtered pixels (the diagonal counts twice)
        p.row_nnz2[w] = (double)(ent_wave + nband) + (dg != 0.0 ? 2.0 : 0.0);
        p.row_sum2[w] = (double)s + 2.0 * dg;
    }
}

}  // namespace hh

using namespace hh;

namespace {

template <class Id, class Cnt>
void build_from_device_pixels(const Id* b1, const Id* b2, const Cnt* cnt, int64_t nnz, int64_t n_bins,
                              const int64_t* chrom_offsets, int32_t n_chroms, int32_t ignore_diags, int32_t cis_only,
                              int64_t row_lo, int64_t row_hi, hipStream_t s, hh_matrix** out,
                              bool* unsorted = nullptr) {
    HH_REQUIRE(out && n_bins > 0 && nnz >= 0 && n_chroms > 0 && chrom_offsets, "bad arguments");
    HH_REQUIRE(nnz == 0 || (b1 && b2 && cnt), "null pixel arrays");
    HH_REQUIRE(n_bins < kMaxBins, "n_bins must be < 2^30");
    HH_REQUIRE(0 <= row_lo && row_lo <= row_hi && row_hi <= n_bins, "bad row range");
    HH_REQUIRE((row_lo % kR == 0 || row_lo == n_bins) && (row_hi % kR == 0 || row_hi == n_bins), "shard rows must be aligned to 512-row blocks");
    HH_REQUIRE(chrom_offsets[0] == 0 && chrom_offsets[n_chroms] == n_bins, "chrom_offsets must span [0, n_bins]");
    HH_REQUIRE(n_chroms < 65535, "too many chromosomes");
    HH_REQUIRE(ignore_diags >= 0, "ignore_diags must be >= 0");
    // hh_tune("build_debug", 1): phase times on stderr (synchronises per phase)
    auto t_last = std::chrono::steady_clock::now();
    auto phase = [&](const char* what) {
        if (!g_build_debug) return;
        HIP_CHECK(hipStreamSynchronize(s));
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[build] %-24s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t - t_last).count());
        t_last = t;
    };
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
    const int nJ = (int)((n_bins + kW - 1) / kW);
    const int occ_max = kBandMaxW + 1;
    // ---- validate + filter + occupancy
    DBuf<int32_t> dch = to_device(chrom_of, s);
    DBuf<int32_t> dA(std::max<int64_t>(nnz, 1)), dB(std::max<int64_t>(nnz, 1));
    DBuf<uint32_t> dkc(std::max<int64_t>(nnz, 1));
    DBuf<unsigned> docc(occ_max + 1), dbig(occ_max + 1);
    DBuf<unsigned> docc_c((size_t)kOccCopies * (occ_max + 1)), dbig_c((size_t)kOccCopies * (occ_max + 1));
    DBuf<unsigned long long> derr(5);
    docc_c.zero(s);
    dbig_c.zero(s);
    HIP_CHECK(hipMemsetAsync(derr.p, 0xff, 5 * sizeof(unsigned long long), s));
    if (nnz > 0)
        hipLaunchKernelGGL((k_px_check<Id, Cnt>), dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s, b1, b2, cnt,
                           (long long)nnz, (long long)n_bins, dch.p, ignore_diags, cis_only, dA.p, dB.p, dkc.p, docc_c.p,
                           dbig_c.p, occ_max, derr.p);
    hipLaunchKernelGGL(k_occ_reduce, dim3((unsigned)((occ_max + 1 + 255) / 256)), dim3(256), 0, s, docc_c.p, dbig_c.p,
                       occ_max + 1, docc.p, dbig.p);
    HIP_CHECK(hipGetLastError());
    std::vector<unsigned long long> herr(5);
    derr.download(herr.data(), 5, s);
    std::vector<unsigned> hocc(occ_max + 1), hbig(occ_max + 1);
    docc.download(hocc.data(), hocc.size(), s);
    dbig.download(hbig.data(), hbig.size(), s);
    phase("check");
    HIP_CHECK(hipStreamSynchronize(s));
    {
        static const char* what[5] = {"bin id out of range", "bin1 > bin2 (not an upper-triangle pixel table)",
                                      "pixels not sorted by (bin1, bin2)",
                                      "duplicate pixel (cooler's pixel table has unique (bin1, bin2))",
                                      "counts must be non-negative integers < 2^32"};
        if (unsorted && (herr[1] != ~0ull || herr[2] != ~0ull)) {
            *unsorted = true;  // the caller builds it on the host instead
            return;
        }
        int code = -1;
        unsigned long long at = ~0ull;
        for (int q = 0; q < 5; ++q)
            if (herr[q] < at) { at = herr[q]; code = q; }
        if (code >= 0)
            HH_THROW(HH_ERR_ARG, std::string(what[code]) + " at pixel " + std::to_string(at));
    }
    int32_t W = 0, W4 = 0;
    {
        std::vector<double> occ(kBandMaxW + 2, 0.0), big(kBandMaxW + 2, 0.0);
        for (int64_t d = 1; d < (int64_t)occ.size(); ++d) {
            big[d] = hocc[d] > 0 ? (double)hbig[d] / (double)hocc[d] : 0.0;
            occ[d] = d < n_bins ? (double)hocc[d] / (double)(n_bins - d) : 0.0;
        }
        const BandWidths bw = choose_band_widths(occ, big, ignore_diags);
        W = bw.w8;
        W4 = bw.w4;
    }
    phase("bands chosen");
    // ---- row structure: upper rows from the sorted table, lower rows sorted
    DBuf<long long> up_ptr(n_bins + 1);
    if (nnz > 0)
        hipLaunchKernelGGL(k_px_rowptr, dim3((unsigned)((nnz + 1 + 255) / 256)), dim3(256), 0, s, dA.p, (long long)nnz,
                           (long long)n_bins, up_ptr.p);
    else
        HIP_CHECK(hipMemsetAsync(up_ptr.p, 0, (n_bins + 1) * sizeof(long long), s));
    int ib = 1;
    while (ib < 63 && ((int64_t)1 << ib) < std::max<int64_t>(nnz, 2)) ++ib;
    int rbits = 1;
    while (rbits < 40 && ((int64_t)1 << rbits) < std::max<int64_t>(nloc, 2)) ++rbits;
    HH_REQUIRE(ib + rbits <= 64, "pixel table too large for the 64-bit lower-half keys");
    DBuf<unsigned long long> keys(std::max<int64_t>(nnz, 1));
    unsigned long long hn = 0;
    if (nnz > 0) {
        const long long nblk = (nnz + kLowChunk - 1) / kLowChunk;
        DBuf<long long> bcnt(nblk + 1), bbase(nblk + 1);
        DBuf<unsigned long long> ntot(1);
        HIP_CHECK(hipMemsetAsync(bcnt.p + nblk, 0, sizeof(long long), s));
        hipLaunchKernelGGL(k_px_lowkeys<0>, dim3((unsigned)nblk), dim3(256), 0, s, dA.p, dB.p, dkc.p, (long long)nnz,
                           (long long)row_lo, (long long)row_hi, ib, keys.p, bcnt.p);
        dev_excl_scan_i64(bcnt.p, bbase.p, nblk + 1, ntot.p, s);
        hipLaunchKernelGGL(k_px_lowkeys<1>, dim3((unsigned)nblk), dim3(256), 0, s, dA.p, dB.p, dkc.p, (long long)nnz,
                           (long long)row_lo, (long long)row_hi, ib, keys.p, bbase.p);
        HIP_CHECK(hipGetLastError());
        ntot.download(&hn, 1, s);
        HIP_CHECK(hipStreamSynchronize(s));
    }
    phase("lower keys");
    dev_sort_u64(keys, (int64_t)hn, rbits, s, ib);  // keys in index order: only the row bits
    phase("radix sort");
    DBuf<long long> lo_ptr(nloc + 1);
    hipLaunchKernelGGL(k_px_keyptr, dim3((unsigned)((hn + 1 + 255) / 256)), dim3(256), 0, s, keys.p, (long long)hn, ib,
                       (long long)nloc, lo_ptr.p);
    if (hn)
        hipLaunchKernelGGL(k_px_lowgather, dim3((unsigned)((hn + 255) / 256)), dim3(256), 0, s, keys.p, (long long)hn,
                           ib >= 64 ? ~0ull : ((1ull << ib) - 1ull), dA.p, dkc.p);
    HIP_CHECK(hipGetLastError());
    phase("lower gather");
    // ---- PASS 0: per-(row, tile) counts and row statistics
    m->diag.alloc(nloc);
    m->row_nnz2.alloc(nloc);
    m->row_sum2.alloc(nloc);
    DBuf<uint16_t> cnt_w((size_t)nloc * nJ), cnt_n((size_t)nloc * nJ);
    cnt_w.zero(s);
    cnt_n.zero(s);
    DBuf<int32_t> rband(std::max<int64_t>(nloc, 1));
    DBuf<long long> rwide(nloc + 1), rupper(std::max<int64_t>(nloc, 1)), rent(std::max<int64_t>(nloc, 1));
    PxRows P{};
    P.A = dA.p;
    P.B = dB.p;
    P.kc = dkc.p;
    P.up_ptr = up_ptr.p;
    P.lkeys = keys.p;
    P.lo_ptr = lo_ptr.p;
    P.row_lo = row_lo;
    P.nloc = nloc;
    P.nJ = nJ;
    P.band_w = W;
    P.band_w4 = W4;
    P.upper = upper_tiles_on(nJ) ? 1 : 0;
    P.cnt = cnt_w.p;
    P.cntn = cnt_n.p;
    P.row_band = rband.p;
    P.row_wide = rwide.p;
    P.row_upper = rupper.p;
    P.row_ent = rent.p;
    P.diag = m->diag.p;
    P.row_nnz2 = m->row_nnz2.p;
    P.row_sum2 = m->row_sum2.p;
    const dim3 rgrid((unsigned)((nloc * 64 + 255) / 256));
    if (nloc) hipLaunchKernelGGL((k_px_rows<0>), rgrid, dim3(256), 0, s, P);
    HIP_CHECK(hipGetLastError());
    phase("pass 0");
    std::vector<uint16_t> hc((size_t)nloc * nJ), hnarrow((size_t)nloc * nJ);
    std::vector<int32_t> hb(nloc);
    std::vector<long long> hw(nloc), hu(nloc), he(nloc);
    {
        PinnedDown dl;  // pageable downloads here cost 6-8 ms (profiles/r4e2e)
        dl.add(cnt_w.p, hc.data(), hc.size());
        dl.add(cnt_n.p, hnarrow.data(), hnarrow.size());
        dl.add(rband.p, hb.data(), (size_t)nloc);
        dl.add(rwide.p, hw.data(), (size_t)nloc);
        dl.add(rupper.p, hu.data(), (size_t)nloc);
        dl.add(rent.p, he.data(), (size_t)nloc);
        dl.run(s);
    }
    cnt_w.release();
    cnt_n.release();
    phase("download counts");
    std::vector<uint16_t> bg = bin_groups(*m);
    std::vector<uint16_t> rgroup(bg.begin() + row_lo, bg.begin() + row_hi);
    TilePlan TP = plan_tiles(hc.data(), hnarrow.data(), nloc, nJ, rgroup, row_lo, P.upper != 0);
    phase("plan_tiles (host)");
    upload_plan(TP, *m, s);
    phase("upload plan");
    m->row_group = to_device(rgroup, s);
    DBuf<int32_t> tof = to_device(TP.tile_of, s);
    m->pay.alloc(TP.n_entries_padded);
    m->payn.alloc(TP.n_narrow_padded);
    m->band_w = W;
    m->band_w4 = W4;
    m->band.alloc((size_t)nloc * band_stride(W));
    m->band.zero(s);
    m->band4.alloc((size_t)nloc * band4_stride(W, W4));
    m->band4.zero(s);
    std::vector<long long> wptr(nloc + 1, 0);
    for (int64_t r = 0; r < nloc; ++r) wptr[r + 1] = wptr[r] + hw[r];
    m->wide_ptr = to_device(wptr, s);
    m->wide_col.alloc(std::max<long long>(wptr[nloc], 1));
    m->wide_cnt.alloc(std::max<long long>(wptr[nloc], 1));
    m->n_wide = wptr[nloc];
    phase("alloc + zero");
    // ---- PASS 1: write
    P.tile_of = tof.p;
    P.tile_ent = m->tile_ent.p;
    P.tile_rp = m->tile_rp.p;
    P.tile_entn = m->tile_entn.p;
    P.tile_rpn = m->tile_rpn.p;
    P.pay = m->pay.p;
    P.payn = m->payn.p;
    P.band = m->band.p;
    P.band4 = reinterpret_cast<uint32_t*>(m->band4.p);
    P.wide_ptr = m->wide_ptr.p;
    P.wide_col = m->wide_col.p;
    P.wide_cnt = m->wide_cnt.p;
    if (nloc) hipLaunchKernelGGL((k_px_rows<1>), rgrid, dim3(256), 0, s, P);
    HIP_CHECK(hipGetLastError());
    finalize_flat_layout(*m, s);
    HIP_CHECK(hipStreamSynchronize(s));  // scratch buffers return to the pool
    phase("pass 1");
    int64_t nb = 0, ent = 0, up = 0;
    for (int64_t r = 0; r < nloc; ++r) {
        nb += hb[r];
        ent += he[r];
        up += hu[r];
    }
    m->n_band = nb;
    m->n_entries = ent;
    m->nnz_upper = up;
    *out = m.release();
}

}  // namespace

extern "C" {

int hh_matrix_from_pixels_device(const int32_t* bin1, const int32_t* bin2, const int32_t* count, int64_t nnz,
                                 int64_t n_bins, const int64_t* chrom_offsets, int32_t n_chroms, int32_t ignore_diags,
                                 int32_t cis_only, int64_t row_lo, int64_t row_hi, void* stream, hh_matrix** out) {
    return guard([&] {
        build_from_device_pixels<int32_t, int32_t>(bin1, bin2, count, nnz, n_bins, chrom_offsets, n_chroms,
                                                   ignore_diags, cis_only, row_lo, row_hi, as_stream(stream), out);
    });
}

}  // extern "C"

namespace hh {
// The host entry point's device path (matrix.hip): the host table (int64 ids,
// float64 counts) crosses PCIe once and is built like a device table.
// Returns false (nothing built) when the table is not sorted upper-triangle
// (cooler's own tables always are): the host builder handles any order.
bool build_from_host_pixels_on_device(const int64_t* bin1, const int64_t* bin2, const double* count, int64_t nnz,
                                      int64_t n_bins, const int64_t* chrom_offsets, int32_t n_chroms,
                                      int32_t ignore_diags, int32_t cis_only, int64_t row_lo, int64_t row_hi,
                                      hipStream_t s, hh_matrix** out) {
    DBuf<long long> d1(std::max<int64_t>(nnz, 1)), d2(std::max<int64_t>(nnz, 1));
    DBuf<double> dc(std::max<int64_t>(nnz, 1));
    d1.upload(reinterpret_cast<const long long*>(bin1), nnz, s);
    d2.upload(reinterpret_cast<const long long*>(bin2), nnz, s);
    dc.upload(count, nnz, s);
    bool unsorted = false;
    build_from_device_pixels<long long, double>(d1.p, d2.p, dc.p, nnz, n_bins, chrom_offsets, n_chroms, ignore_diags,
                                                cis_only, row_lo, row_hi, s, out, &unsorted);
    return !unsorted;
}
}  // namespace hh
