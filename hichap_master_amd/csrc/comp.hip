// Compartment numerics of StructureFind (StructureFind.py:201-460) for one
// chromosome's dense N x N raw contact matrix M (float64):
//
//   K6 k_colnnz / k_diag_part + k_diag_reduce
//        column nonzero counts (gap columns, :216-220) and per-distance sums
//        of nonzero entries whose column is not a gap (:222-249)
//   K7 k_oe_colsum + k_oe_center   O/E = M / decline[|i-j|] on nonzeros
//        (:323-329), columns NG only, centred by their means (np.cov)
//      k_syrk   Cov = Zc^T Zc / (N - 1) on fp64 MFMA (v_mfma_f64_16x16x4)
//      k_corr_norm   Cor = clip(Cov / sd_i / sd_j, -1, 1), NaN -> 0 (corrcoef)
//   K8 top-k right singular vectors of the column-centred Cor (sklearn
//        PCA(3).fit(Cor).components_, :338-340) by block subspace iteration
//        with Rayleigh-Ritz: A V = Xc^T (Xc V), Xc = Cor - 1 mu^T, applied as
//        two skinny products with Cor on fp64 MFMA (k_cor_mul_part, split-K,
//        + k_cor_mul_sum with the rank-1 centring fused); Gram products
//        k_gram_part/k_gram_sum; b x b algebra (Jacobi, Cholesky) on the host.
//      k_select_stats  masked sums over Cor and O/E[NG, NG] that
//        Select_PC_new's means_minus / select_ab need (:374-423).
// All reductions are fixed-order (deterministic).
#include <algorithm>
#include <cmath>
#include <limits>
#include <numeric>

#include "hh_common.hpp"

namespace hh {

constexpr int kCT = 64;        // tile edge for M / Cor passes
constexpr int kSB = 16;        // subspace block size

typedef double d4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ K6
__global__ __launch_bounds__(256) void k_colnnz(const double* __restrict__ M, long long N, int rows_per_block,
                                                unsigned long long* __restrict__ nnz) {
    const long long j = (long long)blockIdx.x * 256 + threadIdx.x;
    if (j >= N) return;
    const long long r0 = (long long)blockIdx.y * rows_per_block;
    const long long r1 = std::min<long long>(N, r0 + rows_per_block);
    unsigned long long c = 0;
    for (long long i = r0; i < r1; ++i) c += M[i * N + j] != 0.0;
    atomicAdd(&nnz[j], c);  // integer: order-independent
}

// per tile (I, J) of the full grid: partial sums over local diagonals
// delta = c - r in [-63, 63] of entries whose column is not a gap.
__global__ __launch_bounds__(256) void k_diag_part(const double* __restrict__ M, long long N, long long nT,
                                                   const uint8_t* __restrict__ gapcol, double* __restrict__ part) {
    __shared__ double tile[kCT][kCT + 1];
    const long long I = blockIdx.x / nT, J = blockIdx.x % nT;
    const long long I0 = I * kCT, J0 = J * kCT;
    for (int e = threadIdx.x; e < kCT * kCT; e += 256) {
        const int r = e / kCT, c = e % kCT;
        const long long gi = I0 + r, gj = J0 + c;
        double v = 0.0;
        if (gi < N && gj < N && !gapcol[gj]) v = M[gi * N + gj];
        tile[r][c] = v;
    }
    __syncthreads();
    if (threadIdx.x < 2 * kCT - 1) {
        const int delta = (int)threadIdx.x - (kCT - 1);
        double acc = 0.0;
        for (int r = 0; r < kCT; ++r) {
            const int c = r + delta;
            if (c >= 0 && c < kCT) acc += tile[r][c];
        }
        part[(size_t)blockIdx.x * (2 * kCT - 1) + threadIdx.x] = acc;
    }
}

// decline_raw[d] = sum over |i - j| = d: fixed order over (k = J - I, I).
__global__ void k_diag_reduce(const double* __restrict__ part, long long N, long long nT, double* __restrict__ out) {
    const long long d = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= N) return;
    double acc = 0.0;
    // global offset g = j - i = 64 k + delta, delta in [-63, 63]; want g = +d and g = -d (d > 0)
    for (int sgn = 1; sgn >= -1; sgn -= 2) {
        if (sgn == -1 && d == 0) break;
        const long long g = sgn * d;
        const long long klo = (g - (kCT - 1) + (64LL * 4096) ) / kCT - 4096;  // ceil((g-63)/64)
        for (long long k = klo; k <= klo + 2; ++k) {
            const long long delta = g - k * kCT;
            if (delta < -(kCT - 1) || delta > kCT - 1) continue;
            for (long long I = 0; I < nT; ++I) {
                const long long J = I + k;
                if (J < 0 || J >= nT) continue;
                acc += part[(size_t)(I * nT + J) * (2 * kCT - 1) + (delta + kCT - 1)];
            }
        }
    }
    out[d] = acc;
}

// ------------------------------------------------------------------ K7
__device__ __forceinline__ double oe_value(const double* __restrict__ M, const double* __restrict__ dec,
                                           long long N, long long i, long long j) {
    const double m = M[i * N + j];
    if (m == 0.0) return 0.0;
    const long long d = i > j ? i - j : j - i;
    return m / dec[d];
}

// partial column sums of O/E over row chunks: part[chunk][c]
__global__ __launch_bounds__(256) void k_oe_colsum(const double* __restrict__ M, const double* __restrict__ dec,
                                                   const long long* __restrict__ ng, long long N, long long n,
                                                   int rows_per_chunk, double* __restrict__ part) {
    const long long c = (long long)blockIdx.x * 256 + threadIdx.x;
    if (c >= n) return;
    const long long j = ng[c];
    const long long r0 = (long long)blockIdx.y * rows_per_chunk;
    const long long r1 = std::min<long long>(N, r0 + rows_per_chunk);
    double acc = 0.0;
    for (long long i = r0; i < r1; ++i) acc += oe_value(M, dec, N, i, j);
    part[(size_t)blockIdx.y * n + c] = acc;
}

__global__ void k_oe_mean(const double* __restrict__ part, long long n, int chunks, long long N,
                          double* __restrict__ mu) {
    const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    double acc = 0.0;
    for (int k = 0; k < chunks; ++k) acc += part[(size_t)k * n + c];
    mu[c] = acc / (double)N;
}

// Zc[i][c] = OE(i, ng[c]) - mu[c]; rows >= N and columns >= n are zero padding.
__global__ __launch_bounds__(256) void k_oe_center(const double* __restrict__ M, const double* __restrict__ dec,
                                                   const long long* __restrict__ ng, const double* __restrict__ mu,
                                                   long long N, long long n, long long Npad, long long ld,
                                                   double* __restrict__ Z) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
    if (t >= Npad * ld) return;
    const long long i = t / ld, c = t % ld;
    double v = 0.0;
    if (i < N && c < n) v = oe_value(M, dec, N, i, ng[c]) - mu[c];
    Z[t] = v;
}

// Cov tile (bi, bj), bi <= bj, 128 x 128: 4 waves x (4 x 4) MFMA 16x16x4 f64
// tiles (64 x 64 per wave: 16 flops per byte staged, twice the 64 x 64
// tile's, which was bound by the L2 -> CU stream at 0.59 of the fp64 matrix
// peak).  K steps of 16 rows; the next step's global loads are issued before
// the current step's MFMAs (register double buffer), one LDS buffer.  LDS rows
// padded to 144 doubles (= 16 mod 32) so the two 16-lane row groups of a
// 32-lane LDS pass land on disjoint banks.
constexpr int kSyT = 128;
constexpr int kLdS = kSyT + 16;
__global__ __launch_bounds__(256, 2) void k_syrk(const double* __restrict__ Z, long long ld, long long Kpad,
                                              long long nt, double scale, double* __restrict__ C, long long ldc) {
    __shared__ __attribute__((aligned(16))) double As[16][kLdS];
    __shared__ __attribute__((aligned(16))) double Bs[16][kLdS];
    long long bi = 0, rem = blockIdx.x;
    while (rem >= nt - bi) { rem -= nt - bi; ++bi; }
    const long long bj = bi + rem;
    const long long i0 = bi * kSyT, j0 = bj * kSyT;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wr = (w >> 1) * 64, wc = (w & 1) * 64;
    const bool diag = bi == bj;
    d4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
    // 16 rows x 128 cols per operand: thread -> rows lr, lr + 8; 4 doubles at lc
    const int lr = threadIdx.x / 32, lc = (threadIdx.x % 32) * 4;
    d4 va[2], vb[2];
    auto load = [&](long long k0) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            va[h] = *reinterpret_cast<const d4*>(Z + (k0 + lr + 8 * h) * ld + i0 + lc);
            vb[h] = diag ? va[h] : *reinterpret_cast<const d4*>(Z + (k0 + lr + 8 * h) * ld + j0 + lc);
        }
    };
    load(0);
    for (long long k0 = 0; k0 < Kpad; k0 += 16) {
        __syncthreads();  // previous step's LDS reads are done
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            *reinterpret_cast<d4*>(&As[lr + 8 * h][lc]) = va[h];
            *reinterpret_cast<d4*>(&Bs[lr + 8 * h][lc]) = vb[h];
        }
        __syncthreads();
        if (k0 + 16 < Kpad) load(k0 + 16);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int kk = s * 4 + (lane >> 4);
            double a[4], b[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                a[t] = As[kk][wr + t * 16 + (lane & 15)];
                b[t] = Bs[kk][wc + t * 16 + (lane & 15)];
            }
#pragma unroll
            for (int ta = 0; ta < 4; ++ta)
#pragma unroll
                for (int tb = 0; tb < 4; ++tb)
                    acc[ta][tb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ta], b[tb], acc[ta][tb], 0, 0, 0);
        }
    }
    // C/D layout of v_mfma_f64_16x16x4_f64: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
    for (int ta = 0; ta < 4; ++ta)
#pragma unroll
        for (int tb = 0; tb < 4; ++tb)
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) {
                const long long gi = i0 + wr + ta * 16 + (lane >> 4) + 4 * reg;
                const long long gj = j0 + wc + tb * 16 + (lane & 15);
                const double v = acc[ta][tb][reg] * scale;
                C[gi * ldc + gj] = v;
                if (!diag) C[gj * ldc + gi] = v;
            }
}

// numpy corrcoef: c /= sd[:, None]; c /= sd[None, :]; clip(-1, 1); then the
// reference's NaN -> 0 (an inf cannot survive the clip).  Out of place.
__global__ void k_corr_norm_oop(const double* __restrict__ Cov, long long n, long long ldc,
                                double* __restrict__ Cor) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ldc * ldc) return;  // the padding rows too: the split-K products read them (x 0)
    const long long i = t / ldc, j = t % ldc;
    double v = 0.0;
    if (i < n && j < n) {
        const double si = sqrt(Cov[i * ldc + i]), sj = sqrt(Cov[j * ldc + j]);
        v = (Cov[i * ldc + j] / si) / sj;
        if (v != v) v = 0.0;
        else v = v < -1.0 ? -1.0 : (v > 1.0 ? 1.0 : v);
    }
    Cor[t] = v;
}

// ------------------------------------------------------------------ K8
// Y = Cor V (n x B, V row-major) on fp64 MFMA, split over K.  Cor is
// symmetric, so the product is taken as Cor^T V: a lane's A operand is a
// 32-B d4 of a Cor row (16 lanes cover 512 contiguous bytes), giving 4
// MFMAs whose A-row r stands for output row i0 + 4 r + t.  A block = 64
// output rows x 16 K-rows per step (wave w takes K-rows 4w..4w+3); the four
// waves are reduced in LDS in wave order and each K split writes its own
// partial, summed in split order by k_cor_mul_sum (deterministic).
// Cor is ld x ld with zero padding, so only V needs a bound check.
__global__ __launch_bounds__(256) void k_cor_mul_part(const double* __restrict__ Cor, long long ldc, long long n,
                                                      const double* __restrict__ V, int ksteps,
                                                      double* __restrict__ part) {
    __shared__ double red[3][16 * 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long long i0 = (long long)blockIdx.x * 64;
    const long long kbeg = (long long)blockIdx.y * ksteps * 16;
    const int kr = 4 * w + (lane >> 4);
    const int nsteps = (int)std::min<long long>(ksteps, (ldc - kbeg) / 16);
    d4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
    const double* cp = Cor + (kbeg + kr) * ldc + i0 + 4 * (lane & 15);
    long long k = kbeg + kr;
    int st = 0;
    constexpr int U = 8;  // K-steps of loads in flight per wave
    for (; st + U <= nsteps; st += U) {
        d4 av[U];
        double bv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            av[u] = __builtin_nontemporal_load(reinterpret_cast<const d4*>(cp + u * 16 * ldc));
            const long long kk = k + 16 * u;
            const double x = V[(kk < n ? kk : n - 1) * kSB + (lane & 15)];  // clamped: no branch
            bv[u] = kk < n ? x : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int t = 0; t < 4; ++t)
                acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u][t], bv[u], acc[t], 0, 0, 0);
        cp += U * 16 * ldc;
        k += U * 16;
    }
    for (; st < nsteps; ++st) {
        const d4 av = __builtin_nontemporal_load(reinterpret_cast<const d4*>(cp));
        const double x = V[(k < n ? k : n - 1) * kSB + (lane & 15)];
        const double bv = k < n ? x : 0.0;
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[t], bv, acc[t], 0, 0, 0);
        cp += 16 * ldc;
        k += 16;
    }
    if (w > 0)
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) red[w - 1][(t * 4 + reg) * 64 + lane] = acc[t][reg];
    __syncthreads();
    if (w == 0) {
        double* out = part + ((long long)blockIdx.y * ldc + i0) * kSB;
        // D layout: col = lane & 15, row = (lane >> 4) + 4 * reg  ->  output row 4 * row + t
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) {
                const int q = (t * 4 + reg) * 64 + lane;
                const double v = ((acc[t][reg] + red[0][q]) + red[1][q]) + red[2][q];
                out[(4 * ((lane >> 4) + 4 * reg) + t) * kSB + (lane & 15)] = v;
            }
    }
}

// Y[i][b] = sum_s part[s][i][b] - x_i d_b   (x nullptr -> 1; d nullptr -> none)
__global__ void k_cor_mul_sum(const double* __restrict__ part, int ks, long long ldc, long long n,
                              const double* __restrict__ x, const double* __restrict__ d, double* __restrict__ Y) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * kSB) return;
    double acc = 0.0;
    for (int s = 0; s < ks; ++s) acc += part[(long long)s * ldc * kSB + t];
    if (d) acc -= (x ? x[t / kSB] : 1.0) * d[t % kSB];
    Y[t] = acc;
}

// Gram-type reduction: G[a][b] = sum_i X[i][a] * Y[i][b] (n x B each).
// Block partials over 256-row slabs staged through LDS (coalesced), then a
// wave per entry sums the partials (fixed shuffle tree: deterministic).
constexpr int kGramRows = 64;
__global__ __launch_bounds__(256) void k_gram_part(const double* __restrict__ X, const double* __restrict__ Y,
                                                   long long n, double* __restrict__ part) {
    __shared__ double xs[64][kSB + 1], ys[64][kSB + 1];
    const int a = threadIdx.x / kSB, b = threadIdx.x % kSB;
    const long long r0 = (long long)blockIdx.x * kGramRows;
    double acc = 0.0;
    for (int c = 0; c < kGramRows; c += 64) {
        __syncthreads();
        for (int e = threadIdx.x; e < 64 * kSB; e += 256) {
            const long long i = r0 + c + e / kSB;
            xs[e / kSB][e % kSB] = i < n ? X[i * kSB + e % kSB] : 0.0;
            ys[e / kSB][e % kSB] = i < n ? Y[i * kSB + e % kSB] : 0.0;
        }
        __syncthreads();
#pragma unroll 8
        for (int r = 0; r < 64; ++r) acc = fma(xs[r][a], ys[r][b], acc);
    }
    part[(size_t)blockIdx.x * kSB * kSB + threadIdx.x] = acc;
}

__global__ __launch_bounds__(64) void k_gram_sum(const double* __restrict__ part, int nblk, double* __restrict__ G) {
    const int e = blockIdx.x, l = threadIdx.x;
    double acc = 0.0;
    for (int k = l; k < nblk; k += 64) acc += part[(size_t)k * kSB * kSB + e];
    acc = wave_sum(acc);
    if (l == 0) G[e] = acc;
}

// Y = X * R (n x B times B x B) ; optionally out = X - 1 t^T or X - mu u^T
__global__ void k_rot(const double* __restrict__ X, const double* __restrict__ R, long long n,
                      double* __restrict__ Y) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * kSB) return;
    const long long i = t / kSB;
    const int b = (int)(t % kSB);
    double acc = 0.0;
    for (int a = 0; a < kSB; ++a) acc = fma(X[i * kSB + a], R[a * kSB + b], acc);
    Y[t] = acc;
}

// ------------------------------------------------------------------ select
// Per PC k (<= 3): Cor sums {same, ab} with the means_minus masks and O/E
// nonzero sums {aa, bb} for select_ab.  stats[blk][k][8].
__global__ __launch_bounds__(256) void k_select_stats(const double* __restrict__ Cor, long long ldc, long long n,
                                                      const double* __restrict__ M, long long N,
                                                      const double* __restrict__ dec,
                                                      const long long* __restrict__ ng,
                                                      const int8_t* __restrict__ cls, int K, double eps,
                                                      double* __restrict__ part) {
    __shared__ double sh[16];
    const long long i = blockIdx.x;  // one row of Cor / O/E[NG, NG]
    double v[3][8];
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int q = 0; q < 8; ++q) v[k][q] = 0.0;
    const long long gi = ng[i];
    for (long long j = threadIdx.x; j < n; j += 256) {
        const double c = Cor[i * ldc + j];
        const double oe = oe_value(M, dec, N, gi, ng[j]);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (k >= K) break;
            const int ci = cls[(size_t)k * n + i], cj = cls[(size_t)k * n + j];
            if (ci != 0 && ci == cj) {
                if (c > -1.0 && c < 1.0 - eps) { v[k][0] += c; v[k][1] += 1.0; }
                if (oe != 0.0) {
                    if (ci > 0) { v[k][4] += oe; v[k][5] += 1.0; }
                    else { v[k][6] += oe; v[k][7] += 1.0; }
                }
            } else if (ci > 0 && cj < 0) {
                if (c > -1.0 && c < 1.0) { v[k][2] += c; v[k][3] += 1.0; }
            }
        }
    }
    for (int k = 0; k < K; ++k)
        for (int q = 0; q < 8; ++q) {
            const double s = block_sum(v[k][q], sh);
            if (threadIdx.x == 0) part[((size_t)i * 3 + k) * 8 + q] = s;
        }
}

// ------------------------------------------------------------- host algebra
// Cyclic Jacobi eigen-decomposition of a small symmetric matrix (row-major).
static void jacobi_eig(int n, std::vector<double> A, std::vector<double>& evals, std::vector<double>& evecs) {
    evecs.assign(n * n, 0.0);
    for (int i = 0; i < n; ++i) evecs[i * n + i] = 1.0;
    for (int sweep = 0; sweep < 100; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < n; ++p)
            for (int q = p + 1; q < n; ++q) off += A[p * n + q] * A[p * n + q];
        if (off < 1e-300) break;
        for (int p = 0; p < n; ++p)
            for (int q = p + 1; q < n; ++q) {
                const double apq = A[p * n + q];
                if (std::fabs(apq) < 1e-300) continue;
                const double app = A[p * n + p], aqq = A[q * n + q];
                const double theta = (aqq - app) / (2.0 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
                const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < n; ++k) {
                    const double akp = A[k * n + p], akq = A[k * n + q];
                    A[k * n + p] = c * akp - s * akq;
                    A[k * n + q] = s * akp + c * akq;
                }
                for (int k = 0; k < n; ++k) {
                    const double apk = A[p * n + k], aqk = A[q * n + k];
                    A[p * n + k] = c * apk - s * aqk;
                    A[q * n + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < n; ++k) {
                    const double vkp = evecs[k * n + p], vkq = evecs[k * n + q];
                    evecs[k * n + p] = c * vkp - s * vkq;
                    evecs[k * n + q] = s * vkp + c * vkq;
                }
            }
    }
    evals.resize(n);
    for (int i = 0; i < n; ++i) evals[i] = A[i * n + i];
}

// R^{-1} of the Cholesky factor of a small SPD matrix (G = R^T R), upper R.
static bool chol_inv_upper(int n, const std::vector<double>& G, std::vector<double>& Rinv) {
    std::vector<double> R(n * n, 0.0);
    for (int j = 0; j < n; ++j) {
        double d = G[j * n + j];
        for (int k = 0; k < j; ++k) d -= R[k * n + j] * R[k * n + j];
        if (!(d > 0)) return false;
        R[j * n + j] = std::sqrt(d);
        for (int i = j + 1; i < n; ++i) {
            double s = G[j * n + i];
            for (int k = 0; k < j; ++k) s -= R[k * n + j] * R[k * n + i];
            R[j * n + i] = s / R[j * n + j];
        }
    }
    Rinv.assign(n * n, 0.0);
    for (int j = 0; j < n; ++j) {
        Rinv[j * n + j] = 1.0 / R[j * n + j];
        for (int i = j - 1; i >= 0; --i) {
            double s = 0.0;
            for (int k = i + 1; k <= j; ++k) s += R[i * n + k] * Rinv[k * n + j];
            Rinv[i * n + j] = -s / R[i * n + i];
        }
    }
    return true;
}

}  // namespace hh

using namespace hh;

struct hh_comp {
    int device = 0;
    long long N = 0;
    DBuf<double> M;              // N x N (owned unless on_device)
    const double* Mp = nullptr;
    DBuf<double> dec;            // N
    DBuf<long long> ng;          // n
    long long n = 0, ld = 0;     // Cor leading dimension (n padded to 128)
    DBuf<double> cor;            // ld x ld
    int iters = 0;
};

namespace hh {

// Small-matrix workspace of the subspace iteration (no allocation in the loop).
// G = R^T R (R upper) -> Rinv = R^{-1}, on the device (one wave, LDS;
// cheaper than a host round trip).  Not positive definite -> *fail = 1 and
// Rinv = I (keeps the iterate finite until the host sees the flag).
__global__ __launch_bounds__(64) void k_chol_inv(const double* __restrict__ G, double* __restrict__ Rinv,
                                                 int* __restrict__ fail) {
    __shared__ double R[kSB][kSB + 1];
    __shared__ int bad;
    const int t = threadIdx.x;
    if (t == 0) bad = 0;
    if (t < kSB)
        for (int i = 0; i < kSB; ++i) R[i][t] = 0.0;
    __syncthreads();
    for (int j = 0; j < kSB; ++j) {
        if (t == j) {
            double d = G[j * kSB + j];
            for (int k = 0; k < j; ++k) d -= R[k][j] * R[k][j];
            if (d > 0) R[j][j] = sqrt(d);
            else { R[j][j] = 1.0; bad = 1; }
        }
        __syncthreads();
        if (t > j && t < kSB) {
            double x = G[j * kSB + t];
            for (int k = 0; k < j; ++k) x -= R[k][j] * R[k][t];
            R[j][t] = x / R[j][j];
        }
        __syncthreads();
    }
    if (t >= kSB) return;
    if (bad) {
        if (t == 0) *fail = 1;
        for (int i = 0; i < kSB; ++i) Rinv[i * kSB + t] = i == t ? 1.0 : 0.0;
        return;
    }
    // column t of R^{-1} by back substitution
    double col[kSB];
#pragma unroll
    for (int i = 0; i < kSB; ++i) col[i] = 0.0;
#pragma unroll
    for (int i = kSB - 1; i >= 0; --i) {
        if (i > t) continue;
        if (i == t) { col[i] = 1.0 / R[i][i]; continue; }
        double x = 0.0;
#pragma unroll
        for (int k = 0; k < kSB; ++k)
            if (k > i && k <= t) x += R[i][k] * col[k];
        col[i] = -x / R[i][i];
    }
#pragma unroll
    for (int i = 0; i < kSB; ++i) Rinv[i * kSB + t] = col[i];
}

struct PcaWork {
    long long n = 0, ldc = 0;
    int nblk = 0, ks = 1, ksteps = 1;
    DBuf<double> part, G, R, mpart;
    std::vector<double> hG;
    PcaWork(long long n_, long long ldc_) : n(n_), ldc(ldc_) {
        nblk = (int)std::max<long long>(1, (n + kGramRows - 1) / kGramRows);
        part.alloc((size_t)nblk * kSB * kSB);
        G.alloc(kSB * kSB);
        R.alloc(kSB * kSB);
        hG.resize(kSB * kSB);
        // split K so that the product's blocks (24 KB LDS, 4 waves) are all
        // resident at once (~6 per CU): no tail round
        const long long rb = ldc / 64, steps = ldc / 16;
        const long long want = std::max<long long>(1, std::min<long long>(32, 1280 / rb));
        ksteps = (int)((steps + want - 1) / want);
        ks = (int)((steps + ksteps - 1) / ksteps);
        mpart.alloc((size_t)ks * ldc * kSB);
    }
    // G = X^T Y on the device (B x B), fixed-order reduction
    void gram_dev(const double* X, const double* Y, hipStream_t s) {
        hipLaunchKernelGGL(k_gram_part, dim3(nblk), dim3(256), 0, s, X, Y, n, part.p);
        hipLaunchKernelGGL(k_gram_sum, dim3(kSB * kSB), dim3(64), 0, s, part.p, nblk, G.p);
    }
    // ... and hG = G on the host
    void gram(const double* X, const double* Y, hipStream_t s) {
        gram_dev(X, Y, s);
        G.download(hG.data(), hG.size(), s);
        HIP_CHECK(hipStreamSynchronize(s));
    }
    // Y = Cor V - x d^T, d = row 0 of the last gram_dev (d_use) or none
    void cor_mul(const double* Cor, const double* V, const double* x, bool d_use, double* Y, hipStream_t s) {
        {
            HH_KTIME("k_cor_mul", s);
            hipLaunchKernelGGL(k_cor_mul_part, dim3((unsigned)(ldc / 64), (unsigned)ks), dim3(256), 0, s, Cor, ldc, n, V,
                               ksteps, mpart.p);
        }
        hipLaunchKernelGGL(k_cor_mul_sum, dim3((unsigned)((n * kSB + 255) / 256)), dim3(256), 0, s, mpart.p, ks, ldc, n,
                           x, d_use ? (const double*)G.p : nullptr, Y);
    }
    void put_small(const std::vector<double>& m, hipStream_t s) { R.upload(m.data(), m.size(), s); }
};

// V <- V R^{-1} `passes` times (CholQR / CholQR2) without leaving the device; rank loss is
// reported through *fail (checked at the next host synchronisation).
static void orthonormalize_dev(PcaWork& w, DBuf<double>& V, DBuf<double>& tmp, long long n, int* fail,
                               hipStream_t s, int passes = 2) {
    for (int pass = 0; pass < passes; ++pass) {
        w.gram_dev(V.p, V.p, s);
        hipLaunchKernelGGL(k_chol_inv, dim3(1), dim3(64), 0, s, w.G.p, w.R.p, fail);
        hipLaunchKernelGGL(k_rot, dim3((unsigned)((n * kSB + 255) / 256)), dim3(256), 0, s, V.p, w.R.p, n, tmp.p);
        std::swap(V.p, tmp.p);
    }
}

// V <- V R^{-1} twice (CholQR2); returns false if V lost rank.
static bool orthonormalize(PcaWork& w, DBuf<double>& V, DBuf<double>& tmp, long long n, hipStream_t s) {
    for (int pass = 0; pass < 2; ++pass) {
        std::vector<double> Rinv;
        w.gram(V.p, V.p, s);
        if (!chol_inv_upper(kSB, w.hG, Rinv)) return false;
        w.put_small(Rinv, s);
        hipLaunchKernelGGL(k_rot, dim3((unsigned)((n * kSB + 255) / 256)), dim3(256), 0, s, V.p, w.R.p, n, tmp.p);
        std::swap(V.p, tmp.p);
    }
    return true;
}

}  // namespace hh

extern "C" {

int hh_comp_create(const double* M, int64_t N, int32_t on_device, void* stream, hh_comp** out) {
    return guard([&] {
        HH_REQUIRE(M && N > 0 && out, "bad arguments");
        auto c = std::make_unique<hh_comp>();
        HIP_CHECK(hipGetDevice(&c->device));
        c->N = N;
        if (on_device) {
            c->Mp = M;
        } else {
            c->M.alloc((size_t)N * N);
            c->M.upload(M, (size_t)N * N, as_stream(stream));
            c->Mp = c->M.p;
        }
        HIP_CHECK(hipStreamSynchronize(as_stream(stream)));
        *out = c.release();
    });
}

int hh_comp_free(hh_comp* c) {
    return guard([&] {
        if (c) device_quiesce(c->device);
        delete c;
    });
}

int hh_comp_colnnz(hh_comp* c, int64_t* nnz_col, void* stream) {
    return guard([&] {
        HH_REQUIRE(c && nnz_col, "null");
        hipStream_t s = as_stream(stream);
        const long long N = c->N;
        DBuf<unsigned long long> d(N);
        d.zero(s);
        const int rpb = 256;
        hipLaunchKernelGGL(k_colnnz, dim3((unsigned)((N + 255) / 256), (unsigned)((N + rpb - 1) / rpb)), dim3(256),
                           0, s, c->Mp, N, rpb, d.p);
        HIP_CHECK(hipGetLastError());
        d.download(reinterpret_cast<unsigned long long*>(nnz_col), N, s);
        HIP_CHECK(hipStreamSynchronize(s));
    });
}

int hh_comp_diag_sums(hh_comp* c, const uint8_t* gapcol, double* sums, void* stream) {
    return guard([&] {
        HH_REQUIRE(c && gapcol && sums, "null");
        hipStream_t s = as_stream(stream);
        const long long N = c->N, nT = (N + kCT - 1) / kCT;
        DBuf<uint8_t> g(N);
        g.upload(gapcol, N, s);
        DBuf<double> part((size_t)nT * nT * (2 * kCT - 1)), out(N);
        hipLaunchKernelGGL(k_diag_part, dim3((unsigned)(nT * nT)), dim3(256), 0, s, c->Mp, N, nT, g.p, part.p);
        hipLaunchKernelGGL(k_diag_reduce, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, part.p, N, nT, out.p);
        HIP_CHECK(hipGetLastError());
        out.download(sums, N, s);
        HIP_CHECK(hipStreamSynchronize(s));
    });
}

int hh_comp_correlation(hh_comp* c, const double* decline, const int64_t* ng, int64_t n, void* stream) {
    return guard([&] {
        HH_REQUIRE(c && decline && ng && n > 0 && n <= c->N, "bad arguments");
        hipStream_t s = as_stream(stream);
        const long long N = c->N;
        c->n = n;
        c->ld = (n + kSyT - 1) / kSyT * kSyT;  // whole k_syrk tiles (a multiple of 64 for the other kernels)
        c->dec.alloc(N);
        c->dec.upload(decline, N, s);
        c->ng.alloc(n);
        c->ng.upload(reinterpret_cast<const long long*>(ng), n, s);
        // column means of O/E
        const int rpc = 256;
        const int chunks = (int)((N + rpc - 1) / rpc);
        DBuf<double> part((size_t)chunks * n), mu(n);
        hipLaunchKernelGGL(k_oe_colsum, dim3((unsigned)((n + 255) / 256), (unsigned)chunks), dim3(256), 0, s, c->Mp,
                           c->dec.p, c->ng.p, N, (long long)n, rpc, part.p);
        hipLaunchKernelGGL(k_oe_mean, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, part.p, (long long)n, chunks,
                           N, mu.p);
        // centred O/E, padded
        const long long Npad = (N + 15) / 16 * 16;
        DBuf<double> Z((size_t)Npad * c->ld);
        hipLaunchKernelGGL(k_oe_center, dim3((unsigned)((Npad * c->ld + 255) / 256)), dim3(256), 0, s, c->Mp, c->dec.p,
                           c->ng.p, mu.p, N, (long long)n, Npad, c->ld, Z.p);
        // Cov = Z^T Z * (1 / (N - 1))  (np.cov: c *= true_divide(1, fact))
        DBuf<double> cov((size_t)c->ld * c->ld);
        const long long nt = c->ld / kSyT;
        {
            HH_KTIME("k_syrk", s);
            hipLaunchKernelGGL(k_syrk, dim3((unsigned)(nt * (nt + 1) / 2)), dim3(256), 0, s, Z.p, c->ld, Npad, nt,
                               1.0 / (double)(N - 1), cov.p, c->ld);
        }
        Z.release();
        c->cor.alloc((size_t)c->ld * c->ld);
        hipLaunchKernelGGL(k_corr_norm_oop, dim3((unsigned)((c->ld * c->ld + 255) / 256)), dim3(256), 0, s, cov.p,
                           (long long)n, c->ld, c->cor.p);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipStreamSynchronize(s));
    });
}

int hh_comp_set_cor(hh_comp* c, const double* cor, void* stream) {
    return guard([&] {
        HH_REQUIRE(c && cor && c->cor.p, "call hh_comp_correlation first (sets n)");
        hipStream_t s = as_stream(stream);
        HIP_CHECK(hipMemcpy2DAsync(c->cor.p, c->ld * sizeof(double), cor, c->n * sizeof(double),
                                   c->n * sizeof(double), c->n, hipMemcpyHostToDevice, s));
        HIP_CHECK(hipStreamSynchronize(s));
    });
}

int hh_comp_get_cor(hh_comp* c, double* cor, void* stream) {
    return guard([&] {
        HH_REQUIRE(c && cor && c->cor.p, "no correlation computed");
        hipStream_t s = as_stream(stream);
        HIP_CHECK(hipMemcpy2DAsync(cor, c->n * sizeof(double), c->cor.p, c->ld * sizeof(double),
                                   c->n * sizeof(double), c->n, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
    });
}

int hh_comp_pca(hh_comp* c, int32_t k, double tol, int32_t max_iters, double* components, double* eigvals,
                int32_t* iters_out, void* stream) {
    return guard([&] {
        HH_REQUIRE(c && components && c->cor.p && k >= 1 && k <= 8, "bad arguments");
        hipStream_t s = as_stream(stream);
        const long long n = c->n;
        HH_REQUIRE(n >= kSB, "matrix smaller than the subspace block (16)");
        PcaWork wk(n, c->ld);
        // mu and 1 as the first column of n x B blocks, so mu^T X and 1^T X are
        // row 0 of a Gram product; mu = column means of Cor = (Cor 1) / n.
        DBuf<double> mu(n), mupad, onepad, nmu;
        {
            std::vector<double> op((size_t)n * kSB, 0.0), muh(n), mp((size_t)n * kSB, 0.0);
            for (long long i = 0; i < n; ++i) op[i * kSB] = 1.0;
            onepad = to_device(op, s);
            DBuf<double> rs((size_t)n * kSB);
            wk.cor_mul(c->cor.p, onepad.p, nullptr, false, rs.p, s);
            std::vector<double> h((size_t)n * kSB);
            rs.download(h.data(), h.size(), s);
            HIP_CHECK(hipStreamSynchronize(s));
            std::vector<double> nm(n);
            for (long long i = 0; i < n; ++i) {
                muh[i] = h[i * kSB] / (double)n;
                mp[i * kSB] = muh[i];
                nm[i] = (double)n * muh[i];
            }
            mu = to_device(muh, s);
            mupad = to_device(mp, s);
            nmu = to_device(nm, s);
        }
        // deterministic start block
        std::vector<double> v0((size_t)n * kSB);
        for (long long i = 0; i < n; ++i)
            for (int b = 0; b < kSB; ++b) v0[i * kSB + b] = (double)u01(mix64(0x5eedULL + i * kSB + b)) - 0.5;
        DBuf<double> V = to_device(v0, s), W((size_t)n * kSB), W1((size_t)n * kSB), tmp((size_t)n * kSB);
        HH_REQUIRE(orthonormalize(wk, V, tmp, n, s), "start block rank deficient");
        const unsigned ge = (unsigned)((n * kSB + 255) / 256);
        std::vector<double> prev((size_t)n * k, 0.0), cur((size_t)n * k);
        std::vector<double> evals, evecs, Vh((size_t)n * kSB);
        DBuf<int> fail(1);
        fail.zero(s);
        // Subspace iteration V <- orth(A V) on the device; every kCheck
        // iterations a Rayleigh-Ritz step on the host extracts the Ritz
        // vectors and tests convergence (the only host round trips).
        constexpr int kCheck = 4;
        int it = 0;
        bool done = false;
        for (it = 1; it <= max_iters && !done; ++it) {
            // A V = Xc^T Xc V with Xc = Cor - 1 mu^T, Cor symmetric and
            // Cor 1 = n mu:  A = Cor^2 - n mu mu^T, so
            // W1 = Cor V;  W = Cor W1 - (n mu)(mu^T V)  (one Gram row, fused)
            wk.gram_dev(mupad.p, V.p, s);
            wk.cor_mul(c->cor.p, V.p, nullptr, false, W1.p, s);
            wk.cor_mul(c->cor.p, W1.p, nmu.p, true, W.p, s);
            if (it % kCheck != 0 && it != max_iters) {
                // between checks one CholQR pass suffices (cond(A V) ~ l1/l16)
                std::swap(V.p, W.p);
                orthonormalize_dev(wk, V, tmp, n, fail.p, s, 1);
                continue;
            }
            // Rayleigh-Ritz: H = V^T W (V orthonormal), eig -> Y (descending)
            wk.gram(V.p, W.p, s);
            int hfail = 0;
            fail.download(&hfail, 1, s);
            HIP_CHECK(hipStreamSynchronize(s));
            HH_REQUIRE(!hfail, "subspace lost rank");
            std::vector<double> H(kSB * kSB);
            for (int a = 0; a < kSB; ++a)
                for (int b = 0; b < kSB; ++b) H[a * kSB + b] = 0.5 * (wk.hG[a * kSB + b] + wk.hG[b * kSB + a]);
            jacobi_eig(kSB, H, evals, evecs);
            std::vector<int> ord(kSB);
            std::iota(ord.begin(), ord.end(), 0);
            std::sort(ord.begin(), ord.end(), [&](int x, int y) { return evals[x] > evals[y]; });
            std::vector<double> Y(kSB * kSB);
            for (int a = 0; a < kSB; ++a)
                for (int b = 0; b < kSB; ++b) Y[a * kSB + b] = evecs[a * kSB + ord[b]];
            wk.put_small(Y, s);
            // Ritz vectors of this iteration: V Y
            hipLaunchKernelGGL(k_rot, dim3(ge), dim3(256), 0, s, V.p, wk.R.p, n, tmp.p);
            tmp.download(Vh.data(), Vh.size(), s);
            HIP_CHECK(hipStreamSynchronize(s));
            // convergence: largest entry change of the (unit, sign-aligned)
            // top-k Ritz vectors between two checks
            double worst = 0.0;
            for (int q = 0; q < k; ++q) {
                double dot = 0.0, nn = 0.0;
                for (long long i = 0; i < n; ++i) {
                    cur[q * n + i] = Vh[i * kSB + q];
                    dot += cur[q * n + i] * prev[q * n + i];
                    nn += cur[q * n + i] * cur[q * n + i];
                }
                const double sg = dot < 0 ? -1.0 : 1.0, inv = 1.0 / std::sqrt(nn);
                for (long long i = 0; i < n; ++i) {
                    cur[q * n + i] *= inv;
                    worst = std::max(worst, std::fabs(cur[q * n + i] - sg * prev[q * n + i]));
                }
            }
            if (eigvals)
                for (int q = 0; q < k; ++q) eigvals[q] = evals[ord[q]];
            if (it > kCheck && worst < tol) done = true;
            prev = cur;
            if (!done) {
                // next block: orth(W Y)
                hipLaunchKernelGGL(k_rot, dim3(ge), dim3(256), 0, s, W.p, wk.R.p, n, V.p);
                orthonormalize_dev(wk, V, tmp, n, fail.p, s);
            }
        }
        c->iters = it - 1;
        if (iters_out) *iters_out = c->iters;
        // unit norm + sklearn svd_flip(u_based_decision=False): max-|.| entry positive
        for (int q = 0; q < k; ++q) {
            double nn = 0.0;
            long long am = 0;
            for (long long i = 0; i < n; ++i) {
                nn += cur[q * n + i] * cur[q * n + i];
                if (std::fabs(cur[q * n + i]) > std::fabs(cur[q * n + am])) am = i;
            }
            const double sc = (cur[q * n + am] < 0 ? -1.0 : 1.0) / std::sqrt(nn);
            for (long long i = 0; i < n; ++i) components[q * n + i] = cur[q * n + i] * sc;
        }
    });
}

int hh_comp_select_stats(hh_comp* c, const double* pcs, int32_t k, double eps, double* stats, void* stream) {
    return guard([&] {
        HH_REQUIRE(c && pcs && stats && c->cor.p && k >= 1 && k <= 3, "bad arguments");
        hipStream_t s = as_stream(stream);
        const long long n = c->n;
        std::vector<int8_t> cls((size_t)k * n);
        for (long long q = 0; q < (long long)k * n; ++q) cls[q] = pcs[q] > 0 ? 1 : (pcs[q] < 0 ? -1 : 0);
        DBuf<int8_t> dcls = to_device(cls, s);
        DBuf<double> part((size_t)n * 3 * 8);
        {
            HH_KTIME("k_select_stats", s);
            hipLaunchKernelGGL(k_select_stats, dim3((unsigned)n), dim3(256), 0, s, c->cor.p, c->ld, n, c->Mp, c->N,
                               c->dec.p, c->ng.p, dcls.p, (int)k, eps, part.p);
        }
        HIP_CHECK(hipGetLastError());
        std::vector<double> h((size_t)n * 3 * 8);
        part.download(h.data(), h.size(), s);
        HIP_CHECK(hipStreamSynchronize(s));
        for (int q = 0; q < k * 8; ++q) stats[q] = 0.0;
        for (long long i = 0; i < n; ++i)
            for (int q = 0; q < k; ++q)
                for (int t = 0; t < 8; ++t) stats[q * 8 + t] += h[(i * 3 + q) * 8 + t];
    });
}

}  // extern "C"

// ================================================================== DI (K9)
// StructureFind.Get_Gap (:721-751) and Get_DI (:804-839), one thread per
// column.  Both only read column j within +-B rows of the diagonal, so the
// matrix crosses PCIe as a band, stored diagonal-major:
// band[(B + k) * N + j] = M[j + k][j], k in [-B, B] (N x (2B+1) doubles:
// 24 MB instead of 5 GB for chr1 at 10 kb); a wave's loads of one diagonal
// are contiguous.
namespace hh {
__global__ void k_gap_scan(const double* __restrict__ band, long long N, int B, int lb, uint8_t* __restrict__ gap) {
    const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= N) return;
    const double* col = band + (long long)B * N + j;  // col[k * N] = M[j + k][j]
    bool g = true;  // within lb of an edge: gap
    if (lb <= j && j <= N - 1 - lb) {
        int nz = 0;
        for (int k = -lb; k < lb; ++k) nz += col[k * N] != 0.0;  // rows j-lb .. j+lb-1
        g = (double)nz < 2.0 * lb * 0.8;
    }
    gap[j] = g ? 1 : 0;
}

// 8 lanes per column (lane q takes window offsets k = 1 + q + 8i); the
// partial sums are combined by a fixed xor tree (deterministic).
constexpr int kDiLanes = 8;
__device__ __forceinline__ double di_lane_sum(double x) {
    x += __shfl_xor(x, 1, 64);
    x += __shfl_xor(x, 2, 64);
    x += __shfl_xor(x, 4, 64);
    return x;
}
__global__ __launch_bounds__(256) void k_di(const double* __restrict__ band, long long N, int B,
                                            const uint8_t* __restrict__ gap, const int* __restrict__ win, int test,
                                            double* __restrict__ di) {
    const long long j = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / kDiLanes;
    const int q = threadIdx.x % kDiLanes;
    const bool inb = j < N;
    const long long jj = inb ? j : N - 1;  // whole lane groups stay in the shuffles
    const double* col = band + (long long)B * N + jj;
    const int w = win[jj];
    const bool live = inb && !gap[jj] && !(jj < w || jj > N - w - 1) && w >= 1;
    double su = 0.0, sd = 0.0;
    if (live)
        for (int k = 1 + q; k <= w; k += kDiLanes) { su += col[-k * N]; sd += col[k * N]; }
    su = di_lane_sum(su);
    sd = di_lane_sum(sd);
    double v = 0.0;
    if (test == 0) {
        const double um = su / w, dm = sd / w;
        const double den = (double)w * (double)(w - 1);
        double qu = 0.0, qd = 0.0;
        if (live)
            for (int k = 1 + q; k <= w; k += kDiLanes) {
                const double a = col[-k * N] - um, b = col[k * N] - dm;
                qu += a * a / den;
                qd += b * b / den;
            }
        qu = di_lane_sum(qu);
        qd = di_lane_sum(qd);
        const double dsum = sqrt(qu + qd);
        if (live && dsum != 0.0) v = (dm - um) / dsum;
    } else if (live) {
        const double e = (su + sd) / 2.0;
        if (su != sd && e != 0.0)
            v = (sd - su) / fabs(sd - su) * ((su - e) * (su - e) / e + (sd - e) * (sd - e) / e);
    }
    if (inb && q == 0) di[j] = v;
}
}  // namespace hh

namespace {
const double* stage_band(const double* band, int64_t N, int32_t B, int32_t on_device, hh::DBuf<double>& buf,
                         hipStream_t s) {
    if (on_device) return band;
    const size_t cnt = (size_t)N * (2 * B + 1);
    buf.alloc(cnt);
    buf.upload(band, cnt, s);
    return buf.p;
}
}  // namespace

extern "C" int hh_gap_scan(const double* band, int64_t N, int32_t B, int32_t lb, uint8_t* gap, int32_t on_device,
                           void* stream) {
    return guard([&] {
        HH_REQUIRE(band && gap && N > 0 && lb >= 0 && B >= lb, "bad arguments (need 0 <= lb <= B)");
        hipStream_t s = as_stream(stream);
        DBuf<double> dB;
        const double* pb = stage_band(band, N, B, on_device, dB, s);
        DBuf<uint8_t> dg(N);
        {
            HH_KTIME("k_gap_scan", s);
            hipLaunchKernelGGL(k_gap_scan, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, pb, (long long)N, B, lb,
                               dg.p);
        }
        HIP_CHECK(hipGetLastError());
        dg.download(gap, N, s);
        HIP_CHECK(hipStreamSynchronize(s));
    });
}

extern "C" int hh_di_scan(const double* band, int64_t N, int32_t B, const uint8_t* gap, const int32_t* window_bins,
                          int32_t test, double* di, int32_t on_device, void* stream) {
    return guard([&] {
        HH_REQUIRE(band && window_bins && gap && di && N > 0 && B >= 0, "bad arguments");
        HH_REQUIRE(test == 0 || test == 1, "test must be 0 (ttest) or 1 (chitest)");
        for (int64_t j = 0; j < N; ++j) HH_REQUIRE(window_bins[j] <= B, "window larger than the band");
        hipStream_t s = as_stream(stream);
        DBuf<double> dB;
        const double* pb = stage_band(band, N, B, on_device, dB, s);
        DBuf<int> dw(N);
        dw.upload(window_bins, N, s);
        DBuf<uint8_t> dg(N);
        dg.upload(gap, N, s);
        DBuf<double> dd(N);
        {
            HH_KTIME("k_di", s);
            hipLaunchKernelGGL(k_di, dim3((unsigned)((N * kDiLanes + 255) / 256)), dim3(256), 0, s, pb, (long long)N, B,
                               dg.p, dw.p, test, dd.p);
        }
        HIP_CHECK(hipGetLastError());
        dd.download(di, N, s);
        HIP_CHECK(hipStreamSynchronize(s));
    });
}

// ============================================ balanced band from pixels (K10)
// cooler's `matrix(balance=True).fetch(chrom)` followed by np.nan_to_num
// (StructureFind.Data_preprocess :853-854; allelic data: balance=False,
// :858-865), restricted to the band the gap / DI scans read: one thread per
// pixel of the (upper-triangle, unique) pixel table; a pixel of the
// chromosome [lo, lo + N) within B of the diagonal writes M[i][j] and M[j][i]
// with value count * w[bin1] * w[bin2] (cooler's product order; NaN -> 0).
// Every band cell has at most one writer: no atomics, deterministic.
namespace hh {
__global__ void k_band_from_pixels(const int64_t* __restrict__ b1, const int64_t* __restrict__ b2,
                                   const double* __restrict__ cnt, long long nnz, const double* __restrict__ w,
                                   long long lo, long long N, int B, double* __restrict__ band) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nnz) return;
    const long long p = b1[t], q = b2[t];
    const long long i = (p < q ? p : q) - lo, j = (p < q ? q : p) - lo;
    if (i < 0 || j >= N) return;
    const long long d = j - i;
    if (d > B) return;
    double v = cnt[t];
    if (w) {
        v = v * w[p] * w[q];
        if (v != v) v = 0.0;
    }
    band[(long long)(B - d) * N + j] = v;            // M[i][j]: column j, k = -d
    if (d) band[(long long)(B + d) * N + i] = v;     // M[j][i]: column i, k = +d
}
}  // namespace hh

namespace {
// stage the pixel table (and weights) on the device unless already there,
// then build the zeroed (2B+1) x N band at `band` (device)
void band_from_pixels_dev(const int64_t* bin1, const int64_t* bin2, const double* count, int64_t nnz,
                          const double* weight, int64_t n_weight, int64_t lo, int64_t N, int32_t B, int32_t on_device,
                          double* band, hipStream_t s) {
    DBuf<int64_t> d1, d2;
    DBuf<double> dc, dw;
    const int64_t *p1 = bin1, *p2 = bin2;
    const double *pc = count, *pw = weight;
    if (!on_device && nnz > 0) {
        d1.alloc(nnz); d1.upload(bin1, nnz, s); p1 = d1.p;
        d2.alloc(nnz); d2.upload(bin2, nnz, s); p2 = d2.p;
        dc.alloc(nnz); dc.upload(count, nnz, s); pc = dc.p;
        if (weight) { dw.alloc(n_weight); dw.upload(weight, n_weight, s); pw = dw.p; }
    }
    HIP_CHECK(hipMemsetAsync(band, 0, sizeof(double) * (size_t)N * (2 * B + 1), s));
    if (nnz > 0) {
        HH_KTIME("k_band_from_pixels", s);
        hipLaunchKernelGGL(hh::k_band_from_pixels, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s, p1, p2, pc,
                           (long long)nnz, pw, (long long)lo, (long long)N, B, band);
    }
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(s));  // staged inputs are freed on return
}

void check_pixels_args(const int64_t* bin1, const int64_t* bin2, const double* count, int64_t nnz,
                       const double* weight, int64_t n_weight, int64_t lo, int64_t N, int32_t B, int32_t on_device) {
    HH_REQUIRE(nnz >= 0 && N > 0 && B >= 0 && lo >= 0, "bad arguments");
    HH_REQUIRE(nnz == 0 || (bin1 && bin2 && count), "null pixel arrays");
    HH_REQUIRE(!weight || lo + N <= n_weight, "weights do not cover the chromosome");
    HH_REQUIRE((double)N * (2.0 * B + 1.0) < 4e9, "band too large");
    (void)on_device;
}
}  // namespace

extern "C" int hh_band_from_pixels(const int64_t* bin1, const int64_t* bin2, const double* count, int64_t nnz,
                                   const double* weight, int64_t n_weight, int64_t lo, int64_t N, int32_t B,
                                   double* band, int32_t on_device, void* stream) {
    return guard([&] {
        check_pixels_args(bin1, bin2, count, nnz, weight, n_weight, lo, N, B, on_device);
        HH_REQUIRE(band, "null band");
        hipStream_t s = as_stream(stream);
        if (on_device) {
            band_from_pixels_dev(bin1, bin2, count, nnz, weight, n_weight, lo, N, B, 1, band, s);
            return;
        }
        DBuf<double> db((size_t)N * (2 * B + 1));
        band_from_pixels_dev(bin1, bin2, count, nnz, weight, n_weight, lo, N, B, 0, db.p, s);
        db.download(band, db.n, s);
        HIP_CHECK(hipStreamSynchronize(s));
    });
}

extern "C" int hh_tad_scan_pixels(const int64_t* bin1, const int64_t* bin2, const double* count, int64_t nnz,
                                  const double* weight, int64_t n_weight, int64_t lo, int64_t N, int32_t lb,
                                  const int32_t* window_bins, int32_t test, uint8_t* gap, double* di,
                                  int32_t on_device, void* stream) {
    return guard([&] {
        HH_REQUIRE(window_bins && gap && di && lb >= 0, "bad arguments");
        HH_REQUIRE(test == 0 || test == 1, "test must be 0 (ttest) or 1 (chitest)");
        int32_t B = lb;
        for (int64_t j = 0; j < N; ++j) B = std::max(B, window_bins[j]);
        check_pixels_args(bin1, bin2, count, nnz, weight, n_weight, lo, N, B, on_device);
        hipStream_t s = as_stream(stream);
        DBuf<double> db((size_t)N * (2 * B + 1));
        band_from_pixels_dev(bin1, bin2, count, nnz, weight, n_weight, lo, N, B, on_device, db.p, s);
        DBuf<uint8_t> dg(N);
        {
            HH_KTIME("k_gap_scan", s);
            hipLaunchKernelGGL(hh::k_gap_scan, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, db.p, (long long)N,
                               B, lb, dg.p);
        }
        HIP_CHECK(hipGetLastError());
        // Data_preprocess (:876-884): the first and last bins join the gap
        HIP_CHECK(hipMemsetAsync(dg.p, 1, 1, s));
        HIP_CHECK(hipMemsetAsync(dg.p + N - 1, 1, 1, s));
        DBuf<int> dw(N);
        dw.upload(window_bins, N, s);
        DBuf<double> dd(N);
        {
            HH_KTIME("k_di", s);
            hipLaunchKernelGGL(hh::k_di, dim3((unsigned)((N * hh::kDiLanes + 255) / 256)), dim3(256), 0, s, db.p,
                               (long long)N, B, dg.p, dw.p, test, dd.p);
        }
        HIP_CHECK(hipGetLastError());
        dg.download(gap, N, s);
        dd.download(di, N, s);
        HIP_CHECK(hipStreamSynchronize(s));
    });
}
