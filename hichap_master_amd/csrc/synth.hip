// On-device synthetic whole-genome contact matrix generator (bench inputs for
// configs too large for a host COO, e.g. C4: 6.07e5 diploid bins, ~5e9
// pixels = 60 GB of cooler triplets).
//
// Model: cis lambda(i,j) = A (|i-j|+1)^-decay
// (1 + c s_i s_j) v_i v_j, counts ~ Poisson(lambda) (inversion below 16,
// normal approximation above; clamped to 65535 so every entry fits a
// tile slot); trans pixels uniform with density p * v_i v_j, count 1 or 2.
// Every draw is a pure function of (seed, min(i,j), max(i,j)), so row i's
// lower half equals column i's upper half and every shard of every rank sees
// the same matrix.
//
// One wave per row scans its candidate columns 64 at a time (column tiles are
// 8192 = 128 x 64 wide, so a 64-column group never straddles a tile).
// Pass 0 counts entries per (row, tile) and the row marginals; the host plans
// tiles/units (plan_tiles, shared with the pixel-table builder); pass 1
// compacts each row's nonzeros into its tile slots with ballots.
#include <cmath>
#include <numeric>

#include "ice_internal.hpp"

namespace hh {

struct SynthDev {
    long long n;
    int n_chroms;
    int nJ;
    const int* chrom_lo;   // n_chroms + 1
    const float* vis;      // n (0 = gap bin)
    const signed char* sgn;
    const short* chrom;    // n
    float A, decay, comp, trans;
    int ignore_diags, cis_only;
    unsigned long long seed;
    int band_w;            // uint8 band half-width W8 (0 = none)
    int band_w4;           // nibble band outer width W4 (== band_w: none)
    int ordered;           // 1: independent draws for (i, j) and (j, i) (asymmetric cells)
    int upper;             // g_upper_tiles: tile entries only where J(col) >= J(row)
};

__global__ void k_synth_bins(SynthDev p, float vis_sigma, float gap_frac, int comp_block,
                             float* vis, signed char* sgn) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= p.n) return;
    const int c = p.chrom[i];
    const long long local = i - p.chrom_lo[c];
    const uint64_t h = mix64(p.seed ^ mix64(0xB1A5ull + (uint64_t)i));
    const float u1 = fmaxf(u01(h), 1e-7f), u2 = u01(mix64(h));
    const float z = sqrtf(-2.f * logf(u1)) * cosf(6.2831853f * u2);
    const bool gap = u01(mix64(h ^ 0x5151ull)) < gap_frac;
    vis[i] = gap ? 0.f : expf(vis_sigma * z);
    const uint64_t hb = mix64(p.seed ^ mix64(0xC0FFEEull + ((uint64_t)c << 32) + (uint64_t)(local / comp_block)));
    sgn[i] = (hb & 1) ? 1 : -1;
}

__device__ __forceinline__ uint32_t poisson(float lam, uint64_t h) {
    if (!(lam > 0.f)) return 0u;
    if (lam < 16.f) {
        const float u = u01(h);
        float pk = __expf(-lam), F = pk;
        uint32_t k = 0;
        while (u > F && k < 96u) {
            ++k;
            pk *= lam / (float)k;
            F += pk;
        }
        return k;
    }
    const float u1 = fmaxf(u01(h), 1e-7f), u2 = u01(mix64(h));
    const float z = sqrtf(-2.f * __logf(u1)) * __cosf(6.2831853f * u2);
    const float k = floorf(lam + sqrtf(lam) * z + 0.5f);
    return k <= 0.f ? 0u : (k >= (float)kCntMax ? kCntMax : (uint32_t)k);
}

__device__ __forceinline__ uint32_t synth_count(const SynthDev& p, long long i, long long j) {
    const long long lo = i < j ? i : j, hi = i < j ? j : i;
    // visibilities in (lo, hi) order: float products do not commute bit for
    // bit once chained, and (i, j) order made lam differ in the last place
    // between the two triangles -- the Poisson draw then flipped by 1 for a
    // few pixels, an asymmetric "symmetric" matrix (round 3 fix)
    const float vi = p.vis[lo], vj = p.vis[hi];
    if (vi == 0.f || vj == 0.f) return 0u;
    const long long d = hi - lo;
    if (d < p.ignore_diags) return 0u;
    const uint64_t h = p.ordered ? mix64(p.seed ^ mix64((uint64_t)i * 0x100000001B3ull + (uint64_t)j + 0x0DDull))
                                 : mix64(p.seed ^ mix64((uint64_t)lo * 0x100000001B3ull + (uint64_t)hi));
    if (p.chrom[i] == p.chrom[j]) {
        const float lam = p.A * exp2f(-p.decay * __log2f((float)d + 1.f)) *
                          (1.f + p.comp * (float)(p.sgn[lo] * p.sgn[hi])) * vi * vj;
        return poisson(lam, h);
    }
    if (p.cis_only) return 0u;
    if (u01(h) >= p.trans * vi * vj) return 0u;
    return (mix64(h) & 3u) == 0u ? 2u : 1u;
}

// PASS 0: cnt[w * nJ + J] / cntn[...] = wide / narrow entries of row w in
//         tile J; per-row stats.
// PASS 1: write entries at tile_ent[t] + tile_rp[t][k] (wide) and
//         tile_entn[t] + tile_rpn[t][k] (narrow), t = tile_of[rb][J].
struct SynthOut {
    uint16_t* cnt;
    uint16_t* cntn;
    int32_t* row_work;
    long long* row_upper;
    double* diag;
    double* row_nnz2;
    double* row_sum2;
    const int32_t* tile_of;
    const long long* tile_ent;
    const uint32_t* tile_rp;
    const long long* tile_entn;
    const uint32_t* tile_rpn;
    uint32_t* pay;
    uint16_t* payn;
    uint8_t* band;         // PASS 1: local rows x band_stride(W8)
    uint32_t* band4;       // PASS 1: local rows x band4_stride(W8, W4) bytes (zeroed; nibbles OR-ed in)
    int32_t* row_band;     // PASS 0: band entries per row
};

template <int PASS>
__global__ __launch_bounds__(256) void k_synth_rows(SynthDev p, long long row_lo, long long nrows, SynthOut o) {
    const long long w = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (w >= nrows) return;
    const int lane = threadIdx.x & 63;
    const long long r = row_lo + w;
    const int c = p.chrom[r];
    const long long jlo = p.cis_only ? p.chrom_lo[c] : 0;
    const long long jhi = p.cis_only ? p.chrom_lo[c + 1] : p.n;
    const long long rb = w / kR;
    const int k = (int)(w % kR);
    const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    long long upper = 0, nnz = 0, work = 0, sum_lane = 0, nb_lane = 0, nbu_lane = 0, nd_lane = 0;
    const int Jr = (int)(r >> kWBits);
    int curJ = -1;
    long long tw = 0, tn = 0;      // wide / narrow entries of the current tile
    long long pos = 0, posn = 0;   // PASS 1: next write positions
    auto flush = [&]() {
        if (curJ < 0) return;
        if (PASS == 0) {
            if (lane == 0 && o.cnt) {
                o.cnt[w * p.nJ + curJ] = (uint16_t)tw;
                o.cntn[w * p.nJ + curJ] = (uint16_t)tn;
            }
        } else {
            const long long pw = (tw + 3) & ~3LL, pn = (tn + 7) & ~7LL;
            for (long long q = tw + lane; q < pw; q += 64) o.pay[pos - tw + q] = 0u;
            for (long long q = tn + lane; q < pn; q += 64) o.payn[posn - tn + q] = 0u;
        }
        work += ((tw + 3) & ~3LL) + ((tn + 7) & ~7LL) / 2;  // 4-byte words
    };
    for (long long j0 = jlo & ~63LL; j0 < jhi; j0 += 64) {
        const long long j = j0 + lane;
        const int J = (int)(j0 >> kWBits);
        uint32_t kc = 0;
        if (j >= jlo && j < jhi && j != r) kc = synth_count(p, r, j);
        // dense band: |j - r| <= W and count <= 255 (implicit column)
        const long long dj = j - r;
        const bool inband = kc > 0 && p.band_w > 0 && kc <= kBandMaxCnt && dj >= -p.band_w && dj <= p.band_w;
        const bool innib = !inband && in_band4(dj, kc, p.band_w, p.band_w4);
        if (inband || innib) {  // per-lane counters (the tile counters below are wave-uniform)
            if (PASS == 1) {
                if (inband) {
                    o.band[w * band_stride(p.band_w) + band_slot(dj, p.band_w)] = (uint8_t)kc;
                } else {  // adjacent lanes share bytes: OR the nibble into the zeroed word
                    const long long nib = w * 2 * band4_stride(p.band_w, p.band_w4) + band4_nibble(dj, p.band_w, p.band_w4);
                    atomicOr(o.band4 + (nib >> 3), kc << (4 * (nib & 7)));
                }
            }
            nb_lane += 1;
            nbu_lane += dj > 0 ? 1 : 0;
            sum_lane += kc;
            kc = 0;
        }
        if (p.upper && kc > 0 && J < Jr) {  // lower tile: stored as its mirror (the column side of row j)
            nd_lane += 1;
            sum_lane += kc;
            kc = 0;
        }
        const unsigned long long mask = __ballot(kc > 0);
        if (mask == 0ull) continue;
        if (J != curJ) {
            flush();
            curJ = J;
            tw = tn = 0;
            if (PASS == 1) {
                const int t = o.tile_of[rb * p.nJ + J];
                pos = o.tile_ent[t] + o.tile_rp[(size_t)t * (kR + 1) + k];
                posn = o.tile_entn[t] + o.tile_rpn[(size_t)t * (kR + 1) + k];
            }
        }
        const bool narrow = kc > 0 && kc <= kNarrowMax;
        const unsigned long long mn = __ballot(narrow), mw = mask & ~mn;
        if (PASS == 1) {
            if (narrow) o.payn[posn + __popcll(mn & lt_mask)] = enc_narrow((uint32_t)j & kColMask, kc);
            else if (kc > 0) o.pay[pos + __popcll(mw & lt_mask)] = enc_wide((uint32_t)j & kColMask, kc);
        }
        const int nn = __popcll(mn), nw = __popcll(mw);
        tn += nn;
        tw += nw;
        posn += nn;
        pos += nw;
        nnz += nn + nw;
        upper += __popcll(__ballot(kc > 0 && j > r));
        sum_lane += kc;
    }
    flush();
    const long long s = wave_sum_ll(sum_lane);
    // band entries were counted per lane; tile entries per wave (ballots)
    const long long nband = wave_sum_ll(nb_lane);
    nnz += nband + wave_sum_ll(nd_lane);
    upper += wave_sum_ll(nbu_lane);
    work += ((long long)p.band_w + band4_stride(p.band_w, p.band_w4) / 2) / 2;  // band bytes per row, in 4-byte words
    const uint32_t dg = p.ignore_diags == 0 ? synth_count(p, r, r) : 0u;
    if (lane == 0) {
        if (o.row_band) o.row_band[w] = (int32_t)nband;
        if (o.row_work) o.row_work[w] = (int32_t)work;
        if (o.row_upper) o.row_upper[w] = upper + (dg ? 1 : 0);
        if (o.diag) {
            o.diag[w] = (double)dg;
            o.row_nnz2[w] = (double)nnz + (dg ? 2.0 : 0.0);
            o.row_sum2[w] = (double)s + 2.0 * (double)dg;
        }
    }
}

}  // namespace hh

using namespace hh;

struct hh_pixels {
    int device = 0;
    int64_t nnz = 0;
    DBuf<int32_t> b1, b2, cnt;
};

namespace {
struct SynthHost {
    DBuf<int> chrom_lo;
    DBuf<short> chrom;
    DBuf<float> vis;
    DBuf<signed char> sgn;
    SynthDev dev{};
    std::vector<int64_t> offsets;
};

BandWidths synth_band_w(const hh_synth_params* p, const std::vector<int64_t>& offsets);

void synth_setup(const hh_synth_params* p, SynthHost& h, hipStream_t s) {
    HH_REQUIRE(p && p->chrom_nbins && p->n_chroms > 0 && p->n_chroms < 32767, "bad synth params");
    HH_REQUIRE(p->comp_block > 0 && p->ignore_diags >= 0, "bad synth params");
    h.offsets.assign(1, 0);
    for (int c = 0; c < p->n_chroms; ++c) {
        HH_REQUIRE(p->chrom_nbins[c] > 0, "chromosome with no bins");
        h.offsets.push_back(h.offsets.back() + p->chrom_nbins[c]);
    }
    const int64_t n = h.offsets.back();
    HH_REQUIRE(n < kMaxBins, "too many bins");
    std::vector<int> lo(h.offsets.begin(), h.offsets.end());
    std::vector<short> ch(n);
    for (int c = 0; c < p->n_chroms; ++c)
        for (int64_t b = h.offsets[c]; b < h.offsets[c + 1]; ++b) ch[b] = (short)c;
    h.chrom_lo = to_device(lo, s);
    h.chrom = to_device(ch, s);
    h.vis.alloc(n);
    h.sgn.alloc(n);
    SynthDev& d = h.dev;
    d.n = n;
    d.n_chroms = p->n_chroms;
    d.nJ = (int)((n + kW - 1) / kW);
    d.chrom_lo = h.chrom_lo.p;
    d.vis = h.vis.p;
    d.sgn = h.sgn.p;
    d.chrom = h.chrom.p;
    d.A = (float)p->A;
    d.decay = (float)p->decay;
    d.comp = (float)p->comp_strength;
    d.trans = (float)p->trans_density;
    d.ignore_diags = p->ignore_diags;
    d.cis_only = p->cis_only ? 1 : 0;
    d.seed = p->seed;
    d.upper = upper_tiles_on(d.nJ) ? 1 : 0;
    {
        const BandWidths bw = synth_band_w(p, h.offsets);
        d.band_w = bw.w8;
        d.band_w4 = bw.w4;
    }
    hipLaunchKernelGGL(k_synth_bins, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d,
                       (float)p->vis_sigma, (float)p->gap_frac, p->comp_block, h.vis.p, h.sgn.p);
    HIP_CHECK(hipGetLastError());
}

inline dim3 row_grid(int64_t nrows) { return dim3((unsigned)((nrows * 64 + 255) / 256)); }

// Dense-band width of the synthetic model: expected occupancy of diagonal d =
// P(count > 0) averaged over visibility / compartment draws (the generator's
// distributions, a fixed host sample) x the share of rows whose partner bin
// is cis and not a gap.  Only performance depends on it.
BandWidths synth_band_w(const hh_synth_params* p, const std::vector<int64_t>& offsets) {
    const int S = 2048;
    std::vector<double> x(S);
    uint64_t st = 0x9E3779B97F4A7C15ull ^ p->seed;
    auto uni = [&]() { st = mix64(st); return ((double)(st >> 11) + 0.5) * (1.0 / 9007199254740992.0); };
    for (int k = 0; k < S; ++k) {
        const double z1 = std::sqrt(-2.0 * std::log(uni())) * std::cos(6.283185307179586 * uni());
        const double z2 = std::sqrt(-2.0 * std::log(uni())) * std::cos(6.283185307179586 * uni());
        x[k] = std::exp(p->vis_sigma * z1) * std::exp(p->vis_sigma * z2);
    }
    const int64_t n = offsets.back();
    std::vector<double> occ(kBandMaxW + 2, 0.0), big(kBandMaxW + 2, 0.0);
    // P(X > 15) / P(X > 0) for X ~ Poisson(lam)
    auto tail15 = [](double lam) {
        if (lam > 60.0) return 1.0;
        double term = std::exp(-lam), cdf = term;
        for (int k = 1; k <= 15; ++k) {
            term *= lam / k;
            cdf += term;
        }
        const double nz = 1.0 - std::exp(-lam);
        return nz > 0 ? std::max(0.0, 1.0 - cdf) / nz : 0.0;
    };
    for (int64_t d = 1; d < (int64_t)occ.size() && d < n; ++d) {
        double cis = 0.0;
        for (size_t c = 0; c + 1 < offsets.size(); ++c) cis += (double)std::max<int64_t>(0, offsets[c + 1] - offsets[c] - d);
        cis /= (double)(n - d);
        const double same = std::max(0.0, 1.0 - (double)d / (double)p->comp_block);
        const double lam0 = p->A * std::pow((double)d + 1.0, -p->decay);
        double e = 0.0, bg = 0.0;
        for (int k = 0; k < S; k += (d < 64 ? 1 : 8)) {
            const double lp = lam0 * (1.0 + p->comp_strength) * x[k], lm = lam0 * (1.0 - p->comp_strength) * x[k];
            const double pp = same + 0.5 * (1.0 - same);
            const double op = 1.0 - std::exp(-lp), om = 1.0 - std::exp(-lm);
            e += pp * op + (1.0 - pp) * om;
            bg += pp * op * tail15(lp) + (1.0 - pp) * om * tail15(lm);
        }
        big[d] = e > 0 ? bg / e : 0.0;
        occ[d] = e / (d < 64 ? S : (S + 7) / 8) * cis * (1.0 - p->gap_frac) * (1.0 - p->gap_frac);
    }
    return choose_band_widths(occ, big, p->ignore_diags);
}
}  // namespace

namespace hh {
// Dense cis block of one chromosome: out[i][j] = count(lo + i, lo + j).
__global__ __launch_bounds__(256) void k_synth_dense(SynthDev p, long long lo, long long nc, double* __restrict__ out) {
    const long long j = (long long)blockIdx.x * 64 + (threadIdx.x & 63);
    const long long i0 = (long long)blockIdx.y * 16 + (threadIdx.x >> 6) * 4;
    if (j >= nc) return;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const long long i = i0 + u;
        if (i < nc) out[i * nc + j] = (double)synth_count(p, lo + i, lo + j);
    }
}
// Pixel table of the same model, one wave per row: PASS 0 counts the row's
// cells (upper triangle j >= i, or every j when p.ordered), PASS 1 writes
// them at the row's offset in (row, col) order.
template <int PASS>
__global__ __launch_bounds__(256) void k_synth_cells(SynthDev p, long long* __restrict__ row_cnt,
                                                     const long long* __restrict__ row_off,
                                                     int32_t* __restrict__ b1, int32_t* __restrict__ b2,
                                                     int32_t* __restrict__ cnt) {
    const long long r = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (r >= p.n) return;
    const int lane = threadIdx.x & 63;
    const unsigned long long lt = (1ull << lane) - 1ull;
    const int c = p.chrom[r];
    const long long jlo0 = p.cis_only ? p.chrom_lo[c] : 0, jhi = p.cis_only ? p.chrom_lo[c + 1] : p.n;
    const long long jlo = p.ordered ? jlo0 : (r > jlo0 ? r : jlo0);
    long long pos = PASS == 1 ? row_off[r] : 0, tot = 0;
    for (long long j0 = jlo & ~63LL; j0 < jhi; j0 += 64) {
        const long long j = j0 + lane;
        uint32_t kc = 0;
        if (j >= jlo && j < jhi) kc = (j == r) ? (p.ignore_diags == 0 ? synth_count(p, r, j) : 0u) : synth_count(p, r, j);
        const unsigned long long m = __ballot(kc > 0);
        if (!m) continue;
        if (PASS == 1 && kc) {
            const long long q = pos + __popcll(m & lt);
            b1[q] = (int32_t)r;
            b2[q] = (int32_t)j;
            cnt[q] = (int32_t)kc;
        }
        pos += __popcll(m);
        tot += __popcll(m);
    }
    if (PASS == 0 && lane == 0) row_cnt[r] = tot;
}

}  // namespace hh

extern "C" {

int hh_synth_count(const hh_synth_params* p, int32_t* row_work, int64_t* row_nnz_upper, void* stream) {
    return guard([&] {
        HH_REQUIRE(row_work && row_nnz_upper, "null outputs");
        hipStream_t s = as_stream(stream);
        SynthHost h;
        synth_setup(p, h, s);
        const int64_t n = h.dev.n;
        DBuf<int32_t> rw(n);
        DBuf<long long> ru(n);
        SynthOut o{};
        o.row_work = rw.p;
        o.row_upper = ru.p;
        hipLaunchKernelGGL((k_synth_rows<0>), row_grid(n), dim3(256), 0, s, h.dev, 0LL, (long long)n, o);
        HIP_CHECK(hipGetLastError());
        rw.download(row_work, n, s);
        HIP_CHECK(hipMemcpyAsync(row_nnz_upper, ru.p, n * sizeof(int64_t), hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
    });
}

int hh_synth_build(const hh_synth_params* p, int64_t row_lo, int64_t row_hi, void* stream, hh_matrix** out) {
    return guard([&] {
        HH_REQUIRE(out, "null");
        hipStream_t s = as_stream(stream);
        SynthHost h;
        synth_setup(p, h, s);
        const int64_t n = h.dev.n;
        HH_REQUIRE(0 <= row_lo && row_lo <= row_hi && row_hi <= n, "bad row range");
        HH_REQUIRE((row_lo % kR == 0 || row_lo == n) && (row_hi % kR == 0 || row_hi == n), "shard rows must be aligned to 512-row blocks");
        const int64_t nloc = row_hi - row_lo;
        const int nJ = h.dev.nJ;
        auto m = std::make_unique<hh_matrix>();
        HIP_CHECK(hipGetDevice(&m->device));
        m->n_bins = n;
        m->row_lo = row_lo;
        m->row_hi = row_hi;
        m->n_chroms = p->n_chroms;
        m->ignore_diags = p->ignore_diags;
        m->cis_only = p->cis_only ? 1 : 0;
        m->chrom_offsets = h.offsets;
        m->diag.alloc(nloc);
        m->row_nnz2.alloc(nloc);
        m->row_sum2.alloc(nloc);
        DBuf<uint16_t> cnt((size_t)nloc * nJ), cntn((size_t)nloc * nJ);
        cnt.zero(s);
        cntn.zero(s);
        DBuf<long long> rup(nloc);
        DBuf<int32_t> rband(std::max<int64_t>(nloc, 1));
        {
            SynthOut o{};
            o.cnt = cnt.p;
            o.cntn = cntn.p;
            o.row_upper = rup.p;
            o.row_band = rband.p;
            o.diag = m->diag.p;
            o.row_nnz2 = m->row_nnz2.p;
            o.row_sum2 = m->row_sum2.p;
            if (nloc)
                hipLaunchKernelGGL((k_synth_rows<0>), row_grid(nloc), dim3(256), 0, s, h.dev, (long long)row_lo,
                                   (long long)nloc, o);
        }
        HIP_CHECK(hipGetLastError());
        std::vector<uint16_t> hc((size_t)nloc * nJ), hn((size_t)nloc * nJ);
        cnt.download(hc.data(), hc.size(), s);
        cntn.download(hn.data(), hn.size(), s);
        std::vector<long long> up(nloc);
        rup.download(up.data(), nloc, s);
        std::vector<int32_t> hb(nloc);
        rband.download(hb.data(), nloc, s);
        HIP_CHECK(hipStreamSynchronize(s));
        cnt.release();
        cntn.release();
        std::vector<uint16_t> bg = bin_groups(*m);
        std::vector<uint16_t> rgroup(bg.begin() + row_lo, bg.begin() + row_hi);
        TilePlan P = plan_tiles(hc.data(), hn.data(), nloc, nJ, rgroup, row_lo, h.dev.upper != 0);
        upload_plan(P, *m, s);
        m->row_group = to_device(rgroup, s);
        DBuf<int32_t> tof = to_device(P.tile_of, s);
        m->pay.alloc(P.n_entries_padded);
        m->payn.alloc(P.n_narrow_padded);
        m->band_w = h.dev.band_w;
        m->band_w4 = h.dev.band_w4;
        m->band.alloc((size_t)nloc * band_stride(m->band_w));
        m->band.zero(s);
        m->band4.alloc((size_t)nloc * band4_stride(m->band_w, m->band_w4));
        m->band4.zero(s);
        {
            SynthOut o{};
            o.band = m->band.p;
            o.band4 = reinterpret_cast<uint32_t*>(m->band4.p);
            o.tile_of = tof.p;
            o.tile_ent = m->tile_ent.p;
            o.tile_rp = m->tile_rp.p;
            o.tile_entn = m->tile_entn.p;
            o.tile_rpn = m->tile_rpn.p;
            o.pay = m->pay.p;
            o.payn = m->payn.p;
            if (nloc)
                hipLaunchKernelGGL((k_synth_rows<1>), row_grid(nloc), dim3(256), 0, s, h.dev, (long long)row_lo,
                                   (long long)nloc, o);
        }
        HIP_CHECK(hipGetLastError());
        finalize_flat_layout(*m, s);
        std::vector<long long> wz(nloc + 1, 0);  // no wide entries (counts clamped)
        m->wide_ptr = to_device(wz, s);
        HIP_CHECK(hipStreamSynchronize(s));
        m->nnz_upper = std::accumulate(up.begin(), up.end(), 0LL);
        int64_t ent = 0;
        for (size_t i = 0; i < hc.size(); ++i) ent += (int64_t)hc[i] + hn[i];
        int64_t nb = 0;
        for (int64_t r = 0; r < nloc; ++r) nb += hb[r];
        m->n_band = nb;
        m->n_entries = ent + nb;
        *out = m.release();
    });
}

int hh_synth_pixels(const hh_synth_params* p, int32_t ordered, void* stream, hh_pixels** out) {
    return guard([&] {
        HH_REQUIRE(out, "null");
        hipStream_t s = as_stream(stream);
        SynthHost h;
        synth_setup(p, h, s);
        h.dev.ordered = ordered ? 1 : 0;
        const int64_t n = h.dev.n;
        auto P = std::make_unique<hh_pixels>();
        HIP_CHECK(hipGetDevice(&P->device));
        DBuf<long long> rc(n + 1), off(n + 1);
        hipLaunchKernelGGL((k_synth_cells<0>), row_grid(n), dim3(256), 0, s, h.dev, rc.p, (const long long*)nullptr,
                           (int32_t*)nullptr, (int32_t*)nullptr, (int32_t*)nullptr);
        HIP_CHECK(hipMemsetAsync(rc.p + n, 0, sizeof(long long), s));
        dev_excl_scan_i64(rc.p, off.p, n + 1, nullptr, s);
        long long tot = 0;
        HIP_CHECK(hipMemcpyAsync(&tot, off.p + n, sizeof(long long), hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        P->nnz = tot;
        P->b1.alloc(std::max<long long>(tot, 1));
        P->b2.alloc(std::max<long long>(tot, 1));
        P->cnt.alloc(std::max<long long>(tot, 1));
        hipLaunchKernelGGL((k_synth_cells<1>), row_grid(n), dim3(256), 0, s, h.dev, (long long*)nullptr, off.p,
                           P->b1.p, P->b2.p, P->cnt.p);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipStreamSynchronize(s));
        *out = P.release();
    });
}

int hh_pixels_get(const hh_pixels* P, const int32_t** bin1, const int32_t** bin2, const int32_t** count, int64_t* nnz) {
    return guard([&] {
        HH_REQUIRE(P, "null");
        if (bin1) *bin1 = P->b1.p;
        if (bin2) *bin2 = P->b2.p;
        if (count) *count = P->cnt.p;
        if (nnz) *nnz = P->nnz;
    });
}

int hh_pixels_free(hh_pixels* P) {
    return guard([&] {
        if (P) device_quiesce(P->device);
        delete P;
    });
}

int hh_synth_dense(const hh_synth_params* p, int32_t chrom, double* out, void* stream) {
    return guard([&] {
        HH_REQUIRE(p && out && 0 <= chrom && chrom < p->n_chroms, "bad arguments");
        hipStream_t s = as_stream(stream);
        SynthHost h;
        synth_setup(p, h, s);
        const long long lo = h.offsets[chrom], nc = h.offsets[chrom + 1] - lo;
        if (nc > 0)
            hipLaunchKernelGGL(k_synth_dense, dim3((unsigned)((nc + 63) / 64), (unsigned)((nc + 15) / 16)), dim3(256), 0,
                               s, h.dev, lo, nc, out);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipStreamSynchronize(s));
    });
}

}  // extern "C"
