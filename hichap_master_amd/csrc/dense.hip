// Dense per-chromosome kernels of HiCHap's two-step / genome-wide correction
// (matrixBuilding.py:742-1023):
//
//   K4 k_rowstats      per row i, over columns [lo_i, hi_i): sum (exact for
//                      int64 input) and number of zeros (Coverage_M :904,
//                      Gap_defined :915, alpha row sums :994-995 / :878-881)
//   K5 symvc           S = X / alpha[:,None]; Y = Trans2symmetry(S, gap)
//                      (:945-979; gap == NULL -> the "no gap" sum form, also
//                      Trans2symmetryLowRes :770); s = rowsum(Y)^(2/3) with
//                      0 -> 1 (Correct_VC :780-790, Y symmetric so row and
//                      column sums agree); C = Y / (s_j s_i);
//                      out = (mean(X) / mean(C)) * C (:1017-1021, :896-899)
//      three passes over symmetric 64x64 tile pairs (each element read once
//      per pass): rowsum(Y) -> sum(C) -> write out.  Partial sums go to slabs
//      reduced in a fixed order (bitwise deterministic, no float atomics).
#include <cmath>
#include <type_traits>

#include "hh_common.hpp"

namespace hh {

constexpr int kT = 64;  // dense tile edge

template <class T>
__global__ __launch_bounds__(256) void k_rowstats(const T* __restrict__ X, long long N,
                                                  const long long* __restrict__ lo,
                                                  const long long* __restrict__ hi, double* __restrict__ sum,
                                                  long long* __restrict__ zeros) {
    __shared__ double shd[16];
    __shared__ long long shz[16];
    const long long i = blockIdx.x;
    const long long a = lo ? lo[i] : 0, b = hi ? hi[i] : N;
    const T* row = X + i * N;
    long long zc = 0;
    double sd = 0.0;
    long long si = 0;
    for (long long j = a + threadIdx.x; j < b; j += 256) {
        const T v = row[j];
        zc += v == T(0);
        if constexpr (std::is_integral_v<T>) si += (long long)v;  // integer: exact
        else sd += (double)v;
    }
    // reduce
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    zc = wave_sum_ll(zc);
    si = wave_sum_ll(si);
    sd = wave_sum(sd);
    if (lane == 0) { shz[wid] = zc; shd[wid] = sd; shz[8 + wid] = si; }
    __syncthreads();
    if (threadIdx.x == 0) {
        long long z = 0, s = 0;
        double d = 0.0;
        for (int k = 0; k < 4; ++k) { z += shz[k]; s += shz[8 + k]; d += shd[k]; }
        zeros[i] = z;
        sum[i] = std::is_integral_v<T> ? (double)s : d;
    }
}

// Pair (I, J), I <= J, of an nT x nT tile grid -> linear index.
__device__ __forceinline__ long long pair_index(long long I, long long J, long long nT) {
    return I * nT - I * (I - 1) / 2 + (J - I);
}

struct SymArgs {
    long long N, nT;
    const double* alpha;
    const uint8_t* gap;   // nullptr: sum form (no gap)
    const double* s;      // pass 2/3: rowsum(Y)^(exponent), 0 -> 1
    double scale;         // pass 3: mean(X) / mean(C)
};

// Loads S tile (I,J) and the transposed S tile (J,I) into LDS as tile[r][c]
// (row r of I, column c of J) and tileT[r][c] = S[J0+c][I0+r].
template <class T>
__device__ __forceinline__ void load_pair(const T* __restrict__ X, const SymArgs& a, long long I0, long long J0,
                                          double (*st)[kT + 1], double (*stT)[kT + 1]) {
    for (int e = threadIdx.x; e < kT * kT; e += 256) {
        const int r = e / kT, c = e % kT;
        const long long gi = I0 + r, gj = J0 + c;
        double v = 0.0, w = 0.0;
        if (gi < a.N && gj < a.N) v = (double)X[gi * a.N + gj] / a.alpha[gi];
        // transposed: read row J0+r, column I0+c  -> S[J0+r][I0+c], store at stT[c][r]
        const long long ti = J0 + r, tj = I0 + c;
        if (ti < a.N && tj < a.N) w = (double)X[ti * a.N + tj] / a.alpha[ti];
        st[r][c] = v;
        stT[c][r] = w;
    }
}

__device__ __forceinline__ double sym_value(const SymArgs& a, long long gi, long long gj, double sij, double sji) {
    if (gi == gj) return sij;
    if (!a.gap) return sij + sji;
    if (a.gap[gi] && a.gap[gj]) return sij > sji ? sij : sji;  // np.maximum-like on non-NaN
    return (sij + sji) / 2.0;
}

// PASS 1: partial row sums of Y.  part[pair][0..63] rows of I, [64..127] rows of J.
// PASS 2: partial sum of C over tile (I,J) (+ mirrored (J,I) when I != J).
// PASS 3: write out = scale * C for tiles (I,J) and (J,I).
template <class T, int PASS>
__global__ __launch_bounds__(256) void k_symvc(const T* __restrict__ X, SymArgs a, double* __restrict__ part,
                                               double* __restrict__ out) {
    __shared__ double st[kT][kT + 1];
    __shared__ double stT[kT][kT + 1];
    __shared__ double red[kT * 2];
    __shared__ double sh[16];
    // decode pair index -> (I, J)
    const long long p = blockIdx.x;
    long long I = 0, rem = p;
    while (rem >= a.nT - I) { rem -= a.nT - I; ++I; }
    const long long J = I + rem;
    const long long I0 = I * kT, J0 = J * kT;
    load_pair(X, a, I0, J0, st, stT);
    __syncthreads();
    if (PASS == 1) {
        // thread t < 64: row sum of tile row t (over J); t in [64,128): column sum (rows of J)
        const int t = threadIdx.x;
        if (t < 2 * kT) {
            double acc = 0.0;
            if (t < kT) {
                const long long gi = I0 + t;
                for (int c = 0; c < kT; ++c) {
                    const long long gj = J0 + c;
                    if (gi < a.N && gj < a.N) acc += sym_value(a, gi, gj, st[t][c], stT[t][c]);
                }
            } else {
                const int c = t - kT;
                const long long gj = J0 + c;
                for (int r = 0; r < kT; ++r) {
                    const long long gi = I0 + r;
                    if (gi < a.N && gj < a.N) acc += sym_value(a, gi, gj, st[r][c], stT[r][c]);
                }
            }
            part[p * (2 * kT) + t] = acc;
        }
    } else if (PASS == 2) {
        double acc = 0.0;
        for (int e = threadIdx.x; e < kT * kT; e += 256) {
            const int r = e / kT, c = e % kT;
            const long long gi = I0 + r, gj = J0 + c;
            if (gi < a.N && gj < a.N) {
                const double y = sym_value(a, gi, gj, st[r][c], stT[r][c]);
                const double v = y / (a.s[gj] * a.s[gi]);
                acc += (I == J) ? v : 2.0 * v;
            }
        }
        acc = block_sum(acc, sh);
        if (threadIdx.x == 0) part[p] = acc;
    } else {
        // out[gi][gj] and out[gj][gi]
        for (int e = threadIdx.x; e < kT * kT; e += 256) {
            const int r = e / kT, c = e % kT;
            const long long gi = I0 + r, gj = J0 + c;
            if (gi < a.N && gj < a.N) {
                const double y = sym_value(a, gi, gj, st[r][c], stT[r][c]);
                out[gi * a.N + gj] = a.scale * (y / (a.s[gj] * a.s[gi]));
            }
        }
        if (I != J) {
            for (int e = threadIdx.x; e < kT * kT; e += 256) {
                const int r = e / kT, c = e % kT;  // element (J0 + r, I0 + c)
                const long long gi = J0 + r, gj = I0 + c;
                if (gi < a.N && gj < a.N) {
                    // Y[gi][gj] = Y[gj][gi] (symmetric): from tile (I,J) at [c][r]
                    const double y = sym_value(a, gj, gi, st[c][r], stT[c][r]);
                    out[gi * a.N + gj] = a.scale * (y / (a.s[gj] * a.s[gi]));
                }
            }
        }
    }
    (void)red;
}

// rowsum(Y)_i from the pass-1 slab in a fixed order (J = 0 .. nT-1), then
// s_i = rowsum^exponent, 0 -> 1.
__global__ void k_symvc_rows(const double* __restrict__ part, long long N, long long nT, double exponent,
                             double* __restrict__ s) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const long long I = i / kT;
    const int r = (int)(i % kT);
    double acc = 0.0;
    for (long long J = 0; J < nT; ++J) {
        if (J >= I) acc += part[pair_index(I, J, nT) * (2 * kT) + r];
        else acc += part[pair_index(J, I, nT) * (2 * kT) + kT + r];
    }
    double v = pow(acc, exponent);
    if (v == 0.0) v = 1.0;
    s[i] = v;
}

// Fixed-order sum of a slab (one block).
__global__ __launch_bounds__(256) void k_slab_sum(const double* __restrict__ part, long long n, double* out) {
    __shared__ double sh[16];
    double acc = 0.0;
    for (long long k = threadIdx.x; k < n; k += 256) acc += part[k];
    acc = block_sum(acc, sh);
    if (threadIdx.x == 0) *out = acc;
}

template <class T>
static void symvc_run(const T* dX, long long N, const double* dalpha, const uint8_t* dgap, double exponent,
                      double raw_sum, double* dout, hipStream_t s) {
    const long long nT = (N + kT - 1) / kT;
    const long long npairs = nT * (nT + 1) / 2;
    DBuf<double> part((size_t)npairs * 2 * kT);
    DBuf<double> sv(N);
    DBuf<double> tot(1);
    SymArgs a{N, nT, dalpha, dgap, nullptr, 1.0};
    HH_REQUIRE(npairs < (1LL << 31), "matrix too large");
    hipLaunchKernelGGL((k_symvc<T, 1>), dim3((unsigned)npairs), dim3(256), 0, s, dX, a, part.p, nullptr);
    hipLaunchKernelGGL(k_symvc_rows, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, part.p, N, nT, exponent,
                       sv.p);
    a.s = sv.p;
    hipLaunchKernelGGL((k_symvc<T, 2>), dim3((unsigned)npairs), dim3(256), 0, s, dX, a, part.p, nullptr);
    hipLaunchKernelGGL(k_slab_sum, dim3(1), dim3(256), 0, s, part.p, npairs, tot.p);
    double sumC = 0.0;
    HIP_CHECK(hipMemcpyAsync(&sumC, tot.p, sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    const double nn = (double)N * (double)N;
    a.scale = (raw_sum / nn) / (sumC / nn);
    hipLaunchKernelGGL((k_symvc<T, 3>), dim3((unsigned)npairs), dim3(256), 0, s, dX, a, part.p, dout);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace hh

using namespace hh;

extern "C" {

int hh_dense_rowstats(const void* X, int32_t dtype, int64_t N, const int64_t* lo, const int64_t* hi,
                      double* rowsum, int64_t* zeros, int32_t on_device, void* stream) {
    return guard([&] {
        HH_REQUIRE(X && rowsum && zeros && N > 0, "bad arguments");
        HH_REQUIRE(dtype == 0 || dtype == 1, "dtype must be 0 (int64) or 1 (float64)");
        hipStream_t s = as_stream(stream);
        DBuf<char> dX;
        const void* px = X;
        if (!on_device) {
            dX.alloc((size_t)N * N * 8);
            HIP_CHECK(hipMemcpyAsync(dX.p, X, (size_t)N * N * 8, hipMemcpyHostToDevice, s));
            px = dX.p;
        }
        DBuf<long long> dlo, dhi;
        if (lo) { dlo.alloc(N); dhi.alloc(N); dlo.upload((const long long*)lo, N, s); dhi.upload((const long long*)hi, N, s); }
        DBuf<double> dsum(N);
        DBuf<long long> dz(N);
        if (dtype == 0)
            hipLaunchKernelGGL((k_rowstats<long long>), dim3((unsigned)N), dim3(256), 0, s, (const long long*)px, (long long)N,
                               dlo.p, dhi.p, dsum.p, dz.p);
        else
            hipLaunchKernelGGL((k_rowstats<double>), dim3((unsigned)N), dim3(256), 0, s, (const double*)px, (long long)N,
                               dlo.p, dhi.p, dsum.p, dz.p);
        HIP_CHECK(hipGetLastError());
        dsum.download(rowsum, N, s);
        dz.download((long long*)zeros, N, s);
        HIP_CHECK(hipStreamSynchronize(s));
    });
}

int hh_dense_symvc(const void* X, int32_t dtype, int64_t N, const double* alpha, const uint8_t* gap,
                   double exponent, double raw_sum, double* out, int32_t on_device, void* stream) {
    return guard([&] {
        HH_REQUIRE(X && alpha && out && N > 0, "bad arguments");
        HH_REQUIRE(dtype == 0 || dtype == 1, "dtype must be 0 (int64) or 1 (float64)");
        hipStream_t s = as_stream(stream);
        const size_t bytes = (size_t)N * N * 8;
        DBuf<char> dX, dO;
        DBuf<double> dA;
        DBuf<uint8_t> dG;
        const void* px = X;
        double* po = out;
        const double* pa = alpha;
        const uint8_t* pg = gap;
        if (!on_device) {
            dX.alloc(bytes);
            HIP_CHECK(hipMemcpyAsync(dX.p, X, bytes, hipMemcpyHostToDevice, s));
            px = dX.p;
            dO.alloc(bytes);
            po = (double*)dO.p;
            dA.alloc(N);
            dA.upload(alpha, N, s);
            pa = dA.p;
            if (gap) {
                dG.alloc(N);
                dG.upload(gap, N, s);
                pg = dG.p;
            }
        }
        if (dtype == 0) symvc_run((const long long*)px, N, pa, pg, exponent, raw_sum, po, s);
        else symvc_run((const double*)px, N, pa, pg, exponent, raw_sum, po, s);
        if (!on_device) {
            HIP_CHECK(hipMemcpyAsync(out, po, bytes, hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
        }
    });
}

}  // extern "C"
