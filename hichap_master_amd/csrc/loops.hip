// loops.hip — HICCUPS neighbourhood sums (StructureFind.pcaller,
// HiCHap/StructureFind.py:1631-1830) on the GPU.
//
// The reference builds, for every window width w in [ww, maxww], one shifted
// copy of the band per window offset (up to 41 x 41 scipy sparse matrices per
// width) and adds them into the donut / lower-left sums.  Here each band
// (raw counts without the main diagonal, balanced counts and expected, both
// on diagonals ww..num-1) becomes per-row prefix sums over the diagonal
// index, P[r][k] = sum_{d < k} B[r][d]; a rectangle of the window is then two
// prefix lookups per row, and one thread evaluates a pixel's whole
// neighbourhood (donut = window - row 0 - column 0 - peak square + its row-0
// and column-0 parts; lower-left = rows 1..w x columns -w..-1 minus the part
// inside the peak square) from 6 lookups per row and band.
//
// k_band_prefix   one wave per row, wave scan over num diagonals    HBM
// k_hiccups_width one thread per still-pending pixel: lower-left raw
//                 reads; at >= 16 the four balanced / expected sums,
//                 state -> assigned                                  L2 (gathers)
#include "hh_common.hpp"

namespace hh {

constexpr int kLoopThreads = 256;

__device__ __forceinline__ double wave_incl_scan_f64(double v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// P[r][0] = 0, P[r][k] = sum_{d < k} B[r][d] for k <= num (B row-major N x num;
// B == nullptr: the expected band, Eall[d] where r + d < N).
__global__ __launch_bounds__(kLoopThreads) void k_band_prefix(const double* __restrict__ B,
                                                              const double* __restrict__ Eall, long long N, int num,
                                                              double* __restrict__ P) {
    const long long r = (long long)blockIdx.x * (kLoopThreads / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= N) return;
    double* out = P + r * (num + 1);
    if (lane == 0) out[0] = 0.0;
    double carry = 0.0;
    for (int d0 = 0; d0 < num; d0 += 64) {
        const int d = d0 + lane;
        double v = 0.0;
        if (d < num) v = B ? B[r * num + d] : (r + d < N ? Eall[d] : 0.0);
        const double s = wave_incl_scan_f64(v) + carry;
        if (d < num) out[d + 1] = s;
        carry = __shfl(s, 63, 64);
    }
}

struct HicDev {
    const double* PH;  // raw (diag 0 removed)
    const double* PC;  // balanced
    const double* PE;  // expected
    long long N;
    int num;
    int pw;
};

// Prefix value of row R at diagonal bound k (clamped); rows outside -> 0.
__device__ __forceinline__ double pref(const double* P, long long R, int num, long long k) {
    k = k < 0 ? 0 : (k > num ? num : k);
    return P[R * (num + 1) + k];
}

__global__ __launch_bounds__(kLoopThreads) void k_hiccups_width(HicDev H, const int32_t* __restrict__ row,
                                                                const int32_t* __restrict__ col, long long n, int w,
                                                                uint8_t* __restrict__ state, double* __restrict__ sK,
                                                                double* __restrict__ sY, double* __restrict__ eK,
                                                                double* __restrict__ eY,
                                                                unsigned long long* __restrict__ newly) {
    const long long i = (long long)blockIdx.x * kLoopThreads + threadIdx.x;
    bool hit = false;
    if (i < n && state[i] == 0) {
        const long long r = row[i], c = col[i];
        const int pw = H.pw, num = H.num;
        // lower-left raw reads: rows r+1..r+w, columns [c-w, c-1] minus
        // rows r+1..r+pw, columns [c-pw, c-1]
        double reads = 0.0;
        for (int a = 1; a <= w; ++a) {
            const long long R = r + a;
            if (R >= H.N) break;
            const long long k0 = c - R - w, k1 = c - R - pw, k2 = c - R;
            const double p2 = pref(H.PH, R, num, k2);
            reads += p2 - pref(H.PH, R, num, k0);
            if (a <= pw) reads -= p2 - pref(H.PH, R, num, k1);
        }
        if (reads >= 16.0) {
            hit = true;
            double kc = 0.0, ke = 0.0, yc = 0.0, ye = 0.0;
            for (int a = -w; a <= w; ++a) {
                const long long R = r + a;
                if (R < 0 || R >= H.N || a == 0) continue;
                const long long k0 = c - R - w, k1 = c - R - pw, k2 = c - R, k3 = k2 + 1, k4 = c - R + pw + 1,
                                k5 = c - R + w + 1;
                const double c0 = pref(H.PC, R, num, k0), c1 = pref(H.PC, R, num, k1), c2 = pref(H.PC, R, num, k2),
                             c3 = pref(H.PC, R, num, k3), c4 = pref(H.PC, R, num, k4), c5 = pref(H.PC, R, num, k5);
                const double e0 = pref(H.PE, R, num, k0), e1 = pref(H.PE, R, num, k1), e2 = pref(H.PE, R, num, k2),
                             e3 = pref(H.PE, R, num, k3), e4 = pref(H.PE, R, num, k4), e5 = pref(H.PE, R, num, k5);
                const bool inner = a >= -pw && a <= pw;
                // donut row: window minus column 0, or minus the peak square's row part
                kc += (c5 - c0) - (inner ? (c4 - c1) : (c3 - c2));
                ke += (e5 - e0) - (inner ? (e4 - e1) : (e3 - e2));
                if (a >= 1) {
                    yc += (c2 - c0) - (a <= pw ? (c2 - c1) : 0.0);
                    ye += (e2 - e0) - (a <= pw ? (e2 - e1) : 0.0);
                }
            }
            sK[i] = kc;
            eK[i] = ke;
            sY[i] = yc;
            eY[i] = ye;
            state[i] = (uint8_t)w;
        }
    }
    const unsigned long long m = __ballot(hit);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(newly, (unsigned long long)__popcll(m));
}

}  // namespace hh

using namespace hh;

struct hh_hiccups {
    int device = 0;
    long long N = 0;
    int num = 0, pw = 0;
    DBuf<double> PH, PC, PE;
    DBuf<int32_t> row, col;
    DBuf<uint8_t> state;
    DBuf<double> sK, sY, eK, eY;
    DBuf<unsigned long long> newly;
    long long n = 0;
};

extern "C" {

int hh_hiccups_create(const double* Hb, const double* Cb, const double* Eall, int64_t N, int32_t num, int32_t pw,
                      int32_t on_device, void* stream, hh_hiccups** out) {
    return guard([&] {
        HH_REQUIRE(Hb && Cb && Eall && out && N > 0 && num > 0 && pw >= 0, "bad arguments");
        hipStream_t s = as_stream(stream);
        auto S = std::make_unique<hh_hiccups>();
        HIP_CHECK(hipGetDevice(&S->device));
        S->N = N;
        S->num = num;
        S->pw = pw;
        const size_t nb = (size_t)N * num;
        DBuf<double> hb, cb, ea;
        const double *dh = Hb, *dc = Cb, *de = Eall;
        if (!on_device) {
            hb.alloc(nb);
            hb.upload(Hb, nb, s);
            cb.alloc(nb);
            cb.upload(Cb, nb, s);
            ea.alloc(num);
            ea.upload(Eall, num, s);
            dh = hb.p;
            dc = cb.p;
            de = ea.p;
        }
        const size_t np1 = (size_t)N * (num + 1);
        S->PH.alloc(np1);
        S->PC.alloc(np1);
        S->PE.alloc(np1);
        const dim3 g((unsigned)((N + 3) / 4));
        hipLaunchKernelGGL(k_band_prefix, g, dim3(kLoopThreads), 0, s, dh, de, (long long)N, (int)num, S->PH.p);
        hipLaunchKernelGGL(k_band_prefix, g, dim3(kLoopThreads), 0, s, dc, de, (long long)N, (int)num, S->PC.p);
        hipLaunchKernelGGL(k_band_prefix, g, dim3(kLoopThreads), 0, s, (const double*)nullptr, de, (long long)N,
                           (int)num, S->PE.p);
        HIP_CHECK(hipGetLastError());
        S->newly.alloc(1);
        HIP_CHECK(hipStreamSynchronize(s));
        *out = S.release();
    });
}

int hh_hiccups_free(hh_hiccups* h) {
    return guard([&] {
        if (h) device_quiesce(h->device);
        delete h;
    });
}

int hh_hiccups_set_pixels(hh_hiccups* h, const int32_t* row, const int32_t* col, int64_t n, void* stream) {
    return guard([&] {
        HH_REQUIRE(h && n >= 0 && (n == 0 || (row && col)), "bad arguments");
        hipStream_t s = as_stream(stream);
        std::vector<int32_t> r(row, row + n), c(col, col + n);
        for (int64_t k = 0; k < n; ++k)
            HH_REQUIRE(r[k] >= 0 && r[k] < h->N && c[k] >= r[k] && c[k] < h->N && c[k] - r[k] < h->num,
                       "pixel outside the band");
        h->n = n;
        const size_t m = (size_t)std::max<int64_t>(n, 1);
        h->row.alloc(m);
        h->col.alloc(m);
        h->row.upload(r.data(), n, s);
        h->col.upload(c.data(), n, s);
        h->state.alloc(m);
        h->state.zero(s);
        for (DBuf<double>* b : {&h->sK, &h->sY, &h->eK, &h->eY}) {
            b->alloc(m);
            b->zero(s);
        }
        HIP_CHECK(hipStreamSynchronize(s));
    });
}

int hh_hiccups_reset(hh_hiccups* h, void* stream) {
    return guard([&] {
        HH_REQUIRE(h, "null");
        hipStream_t s = as_stream(stream);
        h->state.zero(s);
        for (DBuf<double>* b : {&h->sK, &h->sY, &h->eK, &h->eY}) b->zero(s);
        HIP_CHECK(hipStreamSynchronize(s));
    });
}

int hh_hiccups_width(hh_hiccups* h, int32_t w, int64_t* newly_valid, void* stream) {
    return guard([&] {
        HH_REQUIRE(h && newly_valid && w >= 1 && w <= 255, "bad arguments");
        HH_REQUIRE(w >= h->pw, "window narrower than the peak");
        hipStream_t s = as_stream(stream);
        h->newly.zero(s);
        if (h->n) {
            HH_KTIME("k_hiccups_width", s);
            HicDev D{h->PH.p, h->PC.p, h->PE.p, h->N, h->num, h->pw};
            hipLaunchKernelGGL(k_hiccups_width, dim3((unsigned)((h->n + kLoopThreads - 1) / kLoopThreads)),
                               dim3(kLoopThreads), 0, s, D, h->row.p, h->col.p, (long long)h->n, (int)w, h->state.p,
                               h->sK.p, h->sY.p, h->eK.p, h->eY.p, h->newly.p);
        }
        HIP_CHECK(hipGetLastError());
        unsigned long long v = 0;
        HIP_CHECK(hipMemcpyAsync(&v, h->newly.p, sizeof(v), hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        *newly_valid = (int64_t)v;
    });
}

int hh_hiccups_results(hh_hiccups* h, double* sK, double* sY, double* eK, double* eY, uint8_t* width, void* stream) {
    return guard([&] {
        HH_REQUIRE(h, "null");
        hipStream_t s = as_stream(stream);
        if (sK) h->sK.download(sK, h->n, s);
        if (sY) h->sY.download(sY, h->n, s);
        if (eK) h->eK.download(eK, h->n, s);
        if (eY) h->eY.download(eY, h->n, s);
        if (width) h->state.download(width, h->n, s);
        HIP_CHECK(hipStreamSynchronize(s));
    });
}

}  // extern "C"
