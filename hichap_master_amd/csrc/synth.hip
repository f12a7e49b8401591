// On-device synthetic whole-genome contact matrix generator (bench inputs for
// configs too large for a host COO, e.g. C4: 6.07e5 diploid bins, ~5e9
// pixels = 60 GB of cooler triplets).
//
// Model: cis lambda(i,j) = A (|i-j|+1)^-decay
// (1 + c s_i s_j) v_i v_j, counts ~ Poisson(lambda) (inversion below 16,
// normal approximation above; clamped to 2^20); trans pixels uniform with
// density p * v_i v_j, count 1 or 2.  Every draw is a pure function of
// (seed, min(i,j), max(i,j)), so row i's lower half equals column i's upper
// half and every shard of every rank sees the same matrix.
//
// One wave per row scans its candidate columns 64 at a time and compacts the
// nonzeros into 256-entry chunks with ballots (the same greedy chunking rule
// as the host builder in matrix.hip).  Pass 0 counts chunks per row, pass 1
// records each chunk's base column and column-offset width k, pass 2 writes
// the packed entries.
#include <cmath>
#include <numeric>

#include "ice_internal.hpp"

namespace hh {

constexpr uint32_t kSynthCountMax = 1u << 20;

struct SynthDev {
    long long n;
    int n_chroms;
    const int* chrom_lo;   // n_chroms + 1
    const float* vis;      // n (0 = gap bin)
    const signed char* sgn;
    const short* chrom;    // n
    float A, decay, comp, trans;
    int ignore_diags, cis_only;
    unsigned long long seed;
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
    return k <= 0.f ? 0u : (k >= (float)kSynthCountMax ? kSynthCountMax : (uint32_t)k);
}

__device__ __forceinline__ uint32_t synth_count(const SynthDev& p, long long i, long long j) {
    const float vi = p.vis[i], vj = p.vis[j];
    if (vi == 0.f || vj == 0.f) return 0u;
    const long long lo = i < j ? i : j, hi = i < j ? j : i;
    const long long d = hi - lo;
    if (d < p.ignore_diags) return 0u;
    const uint64_t h = mix64(p.seed ^ mix64((uint64_t)lo * 0x100000001B3ull + (uint64_t)hi));
    if (p.chrom[i] == p.chrom[j]) {
        const float lam = p.A * exp2f(-p.decay * __log2f((float)d + 1.f)) *
                          (1.f + p.comp * (float)(p.sgn[i] * p.sgn[j])) * vi * vj;
        return poisson(lam, h);
    }
    if (p.cis_only) return 0u;
    if (u01(h) >= p.trans * vi * vj) return 0u;
    return (mix64(h) & 3u) == 0u ? 2u : 1u;
}

// One wave per row.  PASS 0: chunks and upper pixels per row.  PASS 1: base
// column and width k of each chunk (chunk index from row_chunk_start).
// PASS 2: packed entries (k read back) and the per-row marginals.
template <int PASS>
__global__ __launch_bounds__(256) void k_synth_rows(SynthDev p, long long row_lo, long long nrows,
                                                    int32_t* row_chunks, long long* row_upper,
                                                    const long long* row_chunk_start, uint32_t* pay,
                                                    uint32_t* hdr, double* diag,
                                                    double* row_nnz2, double* row_sum2) {
    const long long w = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (w >= nrows) return;
    const int lane = threadIdx.x & 63;
    const long long r = row_lo + w;
    const int c = p.chrom[r];
    const long long jlo = p.cis_only ? p.chrom_lo[c] : 0;
    const long long jhi = p.cis_only ? p.chrom_lo[c + 1] : p.n;
    long long chunk = PASS > 0 ? row_chunk_start[w] : 0;
    long long nchunks = 0, upper = 0, nnz = 0;
    long long sum_lane = 0;
    int fill = 0, kb = 0;
    long long cbase = 0, clast = 0;
    uint32_t cmax = 0;
    const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    auto close_chunk = [&]() {
        if (PASS == 1 && lane == 0) {
            hdr[chunk] = make_hdr(cbase, nbits((uint32_t)(clast - cbase)));
        }
        if (PASS == 2)
            for (int q = fill + lane; q < kChunk; q += 64) pay[(size_t)chunk * kChunk + slot_of(q)] = 0u;
        ++chunk;
        ++nchunks;
        fill = 0;
        cmax = 0;
    };
    for (long long j0 = jlo; j0 < jhi; j0 += 64) {
        const long long j = j0 + lane;
        uint32_t k = 0;
        if (j < jhi && j != r) k = synth_count(p, r, j);
        unsigned long long mask = __ballot(k > 0);
        if (mask == 0ull) continue;
        nnz += __popcll(mask);
        upper += __popcll(__ballot(k > 0 && j > r));
        sum_lane += k;
        while (mask) {
            if (fill == 0) {
                cbase = j0 + __builtin_ctzll(mask);
                if (PASS == 2) kb = (int)(hdr[chunk] >> kHdrShift);
            }
            const bool in = (mask >> lane) & 1ull;
            const int rank = __popcll(mask & lt_mask);
            // inclusive prefix max of the counts of the remaining lanes
            uint32_t pm = in ? k : 0u;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t t = __shfl_up(pm, o, 64);
                if (lane >= o) pm = pm > t ? pm : t;
            }
            const uint32_t mx = pm > cmax ? pm : cmax;
            const bool fit = in && rank < kChunk - fill &&
                             nbits((uint32_t)(j - cbase)) + nbits(mx) <= 32;
            const unsigned long long fm = __ballot(fit);
            if (fm) {
                const int top = 63 - __builtin_clzll(fm);
                if (PASS == 2 && fit)
                    pay[(size_t)chunk * kChunk + slot_of(fill + rank)] =
                        (uint32_t)((unsigned long long)k << kb) | (uint32_t)(j - cbase);
                cmax = __shfl(mx, top, 64);
                clast = j0 + top;
            }
            fill += __popcll(fm);
            mask &= ~fm;
            if (mask != 0ull || fill == kChunk) close_chunk();
        }
    }
    if (fill > 0) close_chunk();
    const long long s = wave_sum_ll(sum_lane);
    const uint32_t dg = p.ignore_diags == 0 ? synth_count(p, r, r) : 0u;
    if (lane == 0) {
        if (row_chunks) row_chunks[w] = (int32_t)nchunks;
        if (row_upper) row_upper[w] = upper + (dg ? 1 : 0);
        if (PASS == 2) {
            diag[w] = (double)dg;
            row_nnz2[w] = (double)nnz + (dg ? 2.0 : 0.0);
            row_sum2[w] = (double)s + 2.0 * (double)dg;
        }
    }
}

}  // namespace hh

using namespace hh;

namespace {
struct SynthHost {
    DBuf<int> chrom_lo;
    DBuf<short> chrom;
    DBuf<float> vis;
    DBuf<signed char> sgn;
    SynthDev dev{};
    std::vector<int64_t> offsets;
};

void synth_setup(const hh_synth_params* p, SynthHost& h, hipStream_t s) {
    HH_REQUIRE(p && p->chrom_nbins && p->n_chroms > 0 && p->n_chroms < 32767, "bad synth params");
    HH_REQUIRE(p->comp_block > 0 && p->ignore_diags >= 0, "bad synth params");
    h.offsets.assign(1, 0);
    for (int c = 0; c < p->n_chroms; ++c) {
        HH_REQUIRE(p->chrom_nbins[c] > 0, "chromosome with no bins");
        h.offsets.push_back(h.offsets.back() + p->chrom_nbins[c]);
    }
    const int64_t n = h.offsets.back();
    HH_REQUIRE(n < kMaxBins, "too many bins (n_bins must be < 2^27)");
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
    hipLaunchKernelGGL(k_synth_bins, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d,
                       (float)p->vis_sigma, (float)p->gap_frac, p->comp_block, h.vis.p, h.sgn.p);
    HIP_CHECK(hipGetLastError());
}
}  // namespace

extern "C" {

int hh_synth_count(const hh_synth_params* p, int32_t* row_chunks, int64_t* row_nnz_upper, void* stream) {
    return guard([&] {
        HH_REQUIRE(row_chunks && row_nnz_upper, "null outputs");
        hipStream_t s = as_stream(stream);
        SynthHost h;
        synth_setup(p, h, s);
        const int64_t n = h.dev.n;
        DBuf<int32_t> rc(n);
        DBuf<long long> ru(n);
        hipLaunchKernelGGL((k_synth_rows<0>), dim3((unsigned)((n * 64 + 255) / 256)), dim3(256), 0, s, h.dev,
                           0LL, (long long)n, rc.p, ru.p, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr);
        HIP_CHECK(hipGetLastError());
        rc.download(row_chunks, n, s);
        HIP_CHECK(hipMemcpyAsync(row_nnz_upper, ru.p, n * sizeof(int64_t), hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
    });
}

int hh_synth_build(const hh_synth_params* p, const int32_t* row_chunks, int64_t row_lo, int64_t row_hi,
                   void* stream, hh_matrix** out) {
    return guard([&] {
        HH_REQUIRE(row_chunks && out, "null");
        hipStream_t s = as_stream(stream);
        SynthHost h;
        synth_setup(p, h, s);
        const int64_t n = h.dev.n;
        HH_REQUIRE(0 <= row_lo && row_lo <= row_hi && row_hi <= n, "bad row range");
        const int64_t nloc = row_hi - row_lo;
        auto m = std::make_unique<hh_matrix>();
        HIP_CHECK(hipGetDevice(&m->device));
        m->n_bins = n;
        m->row_lo = row_lo;
        m->row_hi = row_hi;
        m->n_chroms = p->n_chroms;
        m->ignore_diags = p->ignore_diags;
        m->cis_only = p->cis_only ? 1 : 0;
        m->chrom_offsets = h.offsets;
        std::vector<int64_t> rcl(nloc), start(nloc);
        int64_t tot = 0;
        for (int64_t r = 0; r < nloc; ++r) {
            rcl[r] = row_chunks[row_lo + r];
            start[r] = tot;
            tot += rcl[r];
        }
        std::vector<uint16_t> bg = bin_groups(*m);
        std::vector<uint16_t> rgroup(bg.begin() + row_lo, bg.begin() + row_hi);
        HostLayer hl;
        make_segments(rcl, rgroup, hl);
        ChunkLayer& L = m->main;
        L.n_chunks = tot;
        L.n_segs = (int64_t)hl.seg_group.size();
        L.pay.alloc((size_t)tot * kChunk);
        L.hdr.alloc(tot);
        L.seg_begin = to_device(hl.seg_begin, s);
        L.row_seg = to_device(hl.row_seg, s);
        L.seg_group = to_device(hl.seg_group, s);
        m->row_group = to_device(rgroup, s);
        m->diag.alloc(nloc);
        m->row_nnz2.alloc(nloc);
        m->row_sum2.alloc(nloc);
        DBuf<long long> dstart(nloc), rup(nloc);
        std::vector<long long> st(start.begin(), start.end());
        dstart.upload(st.data(), nloc, s);
        if (nloc) {
            const dim3 g((unsigned)((nloc * 64 + 255) / 256));
            hipLaunchKernelGGL((k_synth_rows<1>), g, dim3(256), 0, s, h.dev, (long long)row_lo, (long long)nloc,
                               nullptr, nullptr, dstart.p, nullptr, L.hdr.p, nullptr, nullptr, nullptr);
            hipLaunchKernelGGL((k_synth_rows<2>), g, dim3(256), 0, s, h.dev, (long long)row_lo, (long long)nloc,
                               nullptr, rup.p, dstart.p, L.pay.p, L.hdr.p, m->diag.p, m->row_nnz2.p,
                               m->row_sum2.p);
        }
        HIP_CHECK(hipGetLastError());
        std::vector<long long> up(nloc);
        rup.download(up.data(), nloc, s);
        HIP_CHECK(hipStreamSynchronize(s));
        m->nnz_upper = std::accumulate(up.begin(), up.end(), 0LL);
        std::vector<double> nz(nloc);
        m->row_nnz2.download(nz.data(), nloc, s);
        HIP_CHECK(hipStreamSynchronize(s));
        double ent = 0;
        for (int64_t r = 0; r < nloc; ++r) ent += nz[r];
        L.n_entries = (int64_t)ent;  // includes 2x diag indicator; diag is 0 when ignored
        *out = m.release();
    });
}

}  // extern "C"
