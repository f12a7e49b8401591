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
#include <chrono>
#include <cstdlib>
#include <cstring>
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
            // I over the tiles with 0 <= I + k < nT, in order; eight loads in flight
            const long long I1 = k < 0 ? nT : nT - k;
            const size_t step = (size_t)(nT + 1) * (2 * kCT - 1);
            const double* p = part + (size_t)(k < 0 ? -k * nT : k) * (2 * kCT - 1) + (delta + kCT - 1);
            long long I = k < 0 ? -k : 0;
            for (; I + 8 <= I1; I += 8, p += 8 * step) {
                double v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = p[u * step];
#pragma unroll
                for (int u = 0; u < 8; ++u) acc += v[u];
            }
            for (; I < I1; ++I, p += step) acc += *p;
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

// Sliding_Approach O/E (StructureFind.py:274-299), two passes over M:
// Hs[i][j] = sum_{|dj| <= step} M[i][j + dj] for the interior columns, then
// OE[i][j] = sum_{|di| <= step} Hs[i + di][j] / E(|i - j|) inside the
// [step, N - step - 1]^2 square, with the reference's 3-2-1 weighted expected
// sum E = 3 d[i-j] + 2 d[i-j-1] + 2 d[i-j+1] + d[i-j-2] + d[i-j+2] (|.|,
// left to right); M / d[|i - j|] on the border.  The box sum's order differs
// from NumPy's slice sum by rounding only.
__global__ __launch_bounds__(256) void k_sa_hsum(const double* __restrict__ M, long long N, int step,
                                                 double* __restrict__ Hs) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
    if (t >= N * N) return;
    const long long i = t / N, j = t % N;
    if (j < step || j > N - step - 1) return;
    const double* row = M + i * N + j;
    double acc = 0.0;
    for (int dj = -step; dj <= step; ++dj) acc += row[dj];
    Hs[t] = acc;
}

__global__ __launch_bounds__(256) void k_sa_oe(const double* __restrict__ M, const double* __restrict__ Hs,
                                               const double* __restrict__ dec, long long N, int step,
                                               double* __restrict__ OE) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
    if (t >= N * N) return;
    const long long i = t / N, j = t % N;
    const long long dd = i - j;
    auto d = [&](long long x) { return dec[x < 0 ? -x : x]; };
    if (i < step || j < step || i > N - step - 1 || j > N - step - 1) {
        OE[t] = M[t] / d(dd);
        return;
    }
    double o = 0.0;
    for (int di = -step; di <= step; ++di) o += Hs[t + (long long)di * N];
    const double e = 3.0 * d(dd) + 2.0 * d(dd - 1) + 2.0 * d(dd + 1) + d(dd - 2) + d(dd + 2);
    OE[t] = o / e;
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
    long long i = r0;
    for (; i + 8 <= r1; i += 8) {  // eight rows' loads in flight, summed in row order
        double m[8], d[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            m[u] = M[(i + u) * N + j];
            d[u] = dec[i + u > j ? i + u - j : j - i - u];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += m[u] == 0.0 ? 0.0 : m[u] / d[u];
    }
    for (; i < r1; ++i) acc += oe_value(M, dec, N, i, j);
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
    // rows on grid y (no 64-bit division per element), columns on x
    const long long c = (long long)blockIdx.x * 256 + threadIdx.x;
    if (c >= ld) return;
    const bool col = c < n;
    const long long j = col ? ng[c] : 0;
    const double m = col ? mu[c] : 0.0;
    for (long long i = blockIdx.y; i < Npad; i += gridDim.y) {
        double v = 0.0;
        if (i < N && col) v = oe_value(M, dec, N, i, j) - m;
        Z[i * ld + c] = v;
    }
}

// Cov tile (bi, bj), bi <= bj, 128 x 128: 4 waves x (4 x 4) MFMA 16x16x4 f64
// tiles (64 x 64 per wave: 16 flops per byte staged, twice the 64 x 64
// tile's, which was bound by the L2 -> CU stream at 0.59 of the fp64 matrix
// peak).  K steps of 16 rows; the next step's global loads are issued before
// the current step's MFMAs (register double buffer), one LDS buffer (two LDS
// buffers with one barrier per step measured 46.4 vs 49.5 TF/s).  LDS rows
// padded to 144 doubles (= 16 mod 32) so the two 16-lane row groups of a
// 32-lane LDS pass land on disjoint banks.
// Split K (SPLIT): block x = split * ntile + tile takes K rows [split * kc,
// (split + 1) * kc) and writes its raw partial tile; k_syrk_reduce sums the
// splits in order.  The host splits when a chromosome's triangle of tiles
// would leave most of the chip idle for its last round (chr21: 105 tiles on
// 512 block slots).
constexpr int kSyT = 128;
constexpr int kLdS = kSyT + 16;
constexpr int kSyTile = kSyT * kSyT;
__device__ __forceinline__ void syrk_tile_ij(long long t, long long nt, long long& bi, long long& bj) {
    long long b = 0, rem = t;
    while (rem >= nt - b) { rem -= nt - b; ++b; }
    bi = b;
    bj = b + rem;
}

// (round 6: loading whole 256-byte row pieces per instruction -- thread t the
// doubles Z[row][t % 32 + 32 u] -- instead of a d4 per lane measured slower:
// k_syrk 78.4 -> 100.3 ms per C5 pass, profiles/r6h/; not kept)
template <bool SPLIT>
__global__ __launch_bounds__(256, 2) void k_syrk(const double* __restrict__ Z, long long ld, long long Kpad,
                                              long long nt, long long kc, double scale, double* __restrict__ C,
                                              long long ldc, double* __restrict__ P) {
    __shared__ __attribute__((aligned(16))) double As[16][kLdS];
    __shared__ __attribute__((aligned(16))) double Bs[16][kLdS];
    const long long ntile = nt * (nt + 1) / 2;
    const long long tile = SPLIT ? blockIdx.x % ntile : blockIdx.x;
    const long long split = SPLIT ? blockIdx.x / ntile : 0;
    long long bi, bj;
    syrk_tile_ij(tile, nt, bi, bj);
    const long long i0 = bi * kSyT, j0 = bj * kSyT;
    const long long kb = split * kc, ke = min(kb + kc, Kpad);
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
            const double* za = Z + (k0 + lr + 8 * h) * ld + i0 + lc;
            const double* zb = Z + (k0 + lr + 8 * h) * ld + j0 + lc;
            va[h] = *reinterpret_cast<const d4*>(za);
            vb[h] = diag ? va[h] : *reinterpret_cast<const d4*>(zb);
        }
    };
    if (kb < ke) load(kb);
    for (long long k0 = kb; k0 < ke; k0 += 16) {
        __syncthreads();  // previous step's LDS reads are done
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            *reinterpret_cast<d4*>(&As[lr + 8 * h][lc]) = va[h];
            *reinterpret_cast<d4*>(&Bs[lr + 8 * h][lc]) = vb[h];
        }
        __syncthreads();
        if (k0 + 16 < ke) load(k0 + 16);
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
                const int li = wr + ta * 16 + (lane >> 4) + 4 * reg;
                const int lj = wc + tb * 16 + (lane & 15);
                if (SPLIT) {
                    P[(size_t)blockIdx.x * kSyTile + li * kSyT + lj] = acc[ta][tb][reg];
                } else {
                    const double v = acc[ta][tb][reg] * scale;
                    C[(i0 + li) * ldc + j0 + lj] = v;
                    if (!diag) C[(j0 + lj) * ldc + i0 + li] = v;
                }
            }
}

// Split-K partial tiles -> Cov (both triangles): splits summed in order, then
// scaled (deterministic).  One thread per element of the tile triangle.
__global__ __launch_bounds__(256) void k_syrk_reduce(const double* __restrict__ P, int nsplit, long long nt,
                                                     double scale, double* __restrict__ C, long long ldc) {
    const long long ntile = nt * (nt + 1) / 2;
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ntile * kSyTile) return;
    const long long tile = e / kSyTile;
    const int li = (int)(e % kSyTile) / kSyT, lj = (int)(e % kSyT);
    double v = 0.0;
    for (int k = 0; k < nsplit; ++k) v += P[((size_t)k * ntile + tile) * kSyTile + (e % kSyTile)];
    v *= scale;
    long long bi, bj;
    syrk_tile_ij(tile, nt, bi, bj);
    C[(bi * kSyT + li) * ldc + bj * kSyT + lj] = v;
    if (bi != bj) C[(bj * kSyT + lj) * ldc + bi * kSyT + li] = v;
}

// numpy corrcoef: c /= sd[:, None]; c /= sd[None, :]; clip(-1, 1); then the
// reference's NaN -> 0 (an inf cannot survive the clip).  Out of place.
// sd[i] = sqrt(Cov[i][i]) once (each element used to gather its column's
// diagonal entry: one cache line per lane), then rows of 4-column groups.
__global__ void k_cor_sd(const double* __restrict__ Cov, long long n, long long ldc, double* __restrict__ sd) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) sd[i] = sqrt(Cov[i * ldc + i]);
}

__global__ __launch_bounds__(256) void k_corr_norm_oop(const double* __restrict__ Cov, const double* __restrict__ sd,
                                                       long long n, long long ldc, double* __restrict__ Cor) {
    const long long j0 = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
    if (j0 >= ldc) return;  // ldc is a multiple of 128
    for (long long i = blockIdx.y; i < ldc; i += gridDim.y) {  // the padding rows too: the products read them (x 0)
        const size_t o = (size_t)i * ldc + j0;
        d4 v = d4{0.0, 0.0, 0.0, 0.0};
        if (i < n) {
            const d4 c = *reinterpret_cast<const d4*>(Cov + o);
            const double si = sd[i];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const long long j = j0 + u;
                if (j >= n) continue;
                double x = (c[u] / si) / sd[j];
                if (x != x) x = 0.0;
                else x = x < -1.0 ? -1.0 : (x > 1.0 ? 1.0 : x);
                v[u] = x;
            }
        }
        *reinterpret_cast<d4*>(Cor + o) = v;
    }
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

// Y = Cor V from the upper triangle only (half the bytes of k_cor_mul_part).
// Cor in 64 x 64 tiles (a, b); a block owns a 256 x 256 rectangle (p, q),
// p <= q, and wave w its 64-row tile a = 4p + w.  For tile (a, b):
//   column product  Y[b cols] += Cor[a, b]^T V[a rows]   (a <= b)
//   row product     Y[a rows] += Cor[a, b] V[b cols]     (a <  b)
// so row i gets sum_{c in tiles <= tile(i)} Cor[c][i] V[c] from the column
// products and sum_{c in tiles > tile(i)} Cor[i][c] V[c] from the row
// products (Cor is symmetric up to the rounding of corrcoef's two divisions).
// Column product: the lane's d4 of a Cor row is the MFMA A operand (as in
// k_cor_mul_part, reduction over rows); row product: the wave's 16 x 64
// chunk goes through LDS so that a lane's A operand runs along a row
// (reduction over columns).  Column partials of the 4 waves are summed in
// wave order -> part_c[p][col]; row partials accumulate over the
// rectangle's column tiles in registers -> part_r[q][row].
// k_cor_sym_sum adds, for row i in range P, part_c[0..P] then part_r[P..].
// Deterministic (fixed order everywhere).
constexpr int kCsR = 256;  // rectangle edge (4 tiles)
constexpr int kCsW = 66;   // LDS row stride (doubles) of the transpose buffer

__global__ __launch_bounds__(256, 2) void k_cor_sym(const double* __restrict__ Cor, long long ldc, long long n,
                                                   const double* __restrict__ V, long long nr,
                                                   double* __restrict__ part_c, double* __restrict__ part_r) {
    // per-wave transpose buffer; at the end of a column tile the same space
    // holds the wave's column partial (64 x 16 doubles)
    __shared__ double Wt[4][16 * kCsW];
    __shared__ double Vc[64 * kSB];  // V rows of the current column tile (row-product B operands)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lr = lane >> 4, lc = lane & 15;
    long long p, q;
    syrk_tile_ij(blockIdx.x, nr, p, q);
    const long long R0 = p * kCsR + 64 * w;  // this wave's rows
    const bool rows_ok = R0 < ldc;
    const bool diag = p == q;
    // column-product B operands (fixed rows): bv[g][j] = V[R0 + 16 g + 4 j + lr][lc]
    double bv[4][4];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const long long r = R0 + 16 * g + 4 * j + lr;
            const double x = V[(r < n ? r : n - 1) * kSB + lc];
            bv[g][j] = r < n ? x : 0.0;
        }
    d4 dr[4];  // row-product accumulators: rows R0 + 16 g + lr + 4 reg, column lc
#pragma unroll
    for (int g = 0; g < 4; ++g) dr[g] = d4{0.0, 0.0, 0.0, 0.0};
    double* wt = Wt[w];
    for (int ct = 0; ct < 4; ++ct) {
        const long long C0 = q * kCsR + 64 * ct;
        if (C0 >= ldc) break;  // uniform over the block
        // tile (a, b) = (4p + w, 4q + ct): diagonal rectangle -> skip below, column product only on the diagonal
        const bool col_on = rows_ok && (!diag || ct >= w);
        const bool row_on = rows_ok && (!diag || ct > w);
        for (int e = threadIdx.x; e < 64 * kSB; e += 256) {
            const long long c = C0 + e / kSB;
            Vc[e] = c < n ? V[c * kSB + e % kSB] : 0.0;
        }
        __syncthreads();
        d4 acc[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
        if (col_on) {
            const double* cp = Cor + (R0 + lr) * ldc + C0 + 4 * lc;
            d4 av[4], an[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) av[j] = __builtin_nontemporal_load(reinterpret_cast<const d4*>(cp + 4 * j * ldc));
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                if (g < 3)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        an[j] = __builtin_nontemporal_load(
                            reinterpret_cast<const d4*>(cp + (16 * (g + 1) + 4 * j) * ldc));
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int t = 0; t < 4; ++t)
                        acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[j][t], bv[g][j], acc[t], 0, 0, 0);
                if (row_on) {
                    // the wave's 16 x 64 chunk -> LDS (row 4 j + lr), then A' = Wt[m = lc][4 cs + lr]
                    __builtin_amdgcn_wave_barrier();
#pragma unroll
                    for (int j = 0; j < 4; ++j)
#pragma unroll
                        for (int t = 0; t < 4; ++t) wt[(4 * j + lr) * kCsW + 4 * lc + t] = av[j][t];
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                    for (int cs = 0; cs < 16; ++cs)
                        dr[g] = __builtin_amdgcn_mfma_f64_16x16x4f64(wt[lc * kCsW + 4 * cs + lr],
                                                                      Vc[(4 * cs + lr) * kSB + lc], dr[g], 0, 0, 0);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                }
                if (g < 3)
#pragma unroll
                    for (int j = 0; j < 4; ++j) av[j] = an[j];
            }
        }
        // column partial of this column tile: the 4 waves in order
        // (D layout: column lc, row lr + 4 reg -> Cor column C0 + 4 (lr + 4 reg) + t)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) wt[(4 * (lr + 4 * reg) + t) * kSB + lc] = acc[t][reg];
        __syncthreads();
        double* out = part_c + ((size_t)p * ldc + C0) * kSB;
        for (int e = threadIdx.x; e < 64 * kSB; e += 256) out[e] = ((Wt[0][e] + Wt[1][e]) + Wt[2][e]) + Wt[3][e];
        __syncthreads();
    }
    if (!rows_ok) return;
    double* outr = part_r + ((size_t)q * ldc + R0) * kSB;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) outr[(16 * g + lr + 4 * reg) * kSB + lc] = dr[g][reg];
}

// k_cor_sym with the rectangle's V rows staged once (all four column tiles,
// one barrier) and each wave's first Cor loads of the next column tile issued
// during the last row group of the current one: the per-column-tile global
// latency of the V staging and of the first loads is no longer exposed.  The
// same MFMA sequence and partial sums per tile: bitwise k_cor_sym's result
// (hh_tune "cor_sym" 2, the default; 1 = k_cor_sym).
// COAL (round 6, hh_tune "cor_sym" 3): lane (lr, lc) loads the doubles
// Cor[row][C0 + lc + 16 t] (t = 0..3) instead of the d4 Cor[row][C0 + 4 lc ..
// 4 lc + 3]: every load instruction then reads 4 rows x 128 contiguous bytes
// (whole lines) instead of 16-byte pieces 32 bytes apart (the lane-major shape
// that held the flat ICE tiles at 3.5 TB/s).  The k-rows of
// each MFMA are the same; only which lane holds which output column changes
// (acc[t] row i = column C0 + i + 16 t instead of C0 + 4 i + t), so every
// output element is summed over the same terms in the same order: bitwise
// k_cor_sym_pf's result.
template <bool COAL>
__global__ __launch_bounds__(256, 2) void k_cor_sym_pf(const double* __restrict__ Cor, long long ldc, long long n,
                                                      const double* __restrict__ V, long long nr,
                                                      double* __restrict__ part_c, double* __restrict__ part_r) {
    __shared__ double Wt[4][16 * kCsW];
    __shared__ double Vc[4][64 * kSB];  // V rows of the rectangle's column tiles
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lr = lane >> 4, lc = lane & 15;
    long long p, q;
    syrk_tile_ij(blockIdx.x, nr, p, q);
    const long long R0 = p * kCsR + 64 * w;
    const bool rows_ok = R0 < ldc;
    const bool diag = p == q;
    const int nct = (int)std::min<long long>(4, (ldc - q * kCsR + 63) / 64);  // column tiles inside the matrix
    for (int e = threadIdx.x; e < 4 * 64 * kSB; e += 256) {
        const long long c = q * kCsR + e / kSB;  // e / kSB = 64 ct + row within the tile
        Vc[e / (64 * kSB)][e % (64 * kSB)] = c < n ? V[c * kSB + e % kSB] : 0.0;
    }
    double bv[4][4];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const long long r = R0 + 16 * g + 4 * j + lr;
            const double x = V[(r < n ? r : n - 1) * kSB + lc];
            bv[g][j] = r < n ? x : 0.0;
        }
    d4 dr[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) dr[g] = d4{0.0, 0.0, 0.0, 0.0};
    double* wt = Wt[w];
    auto col_on = [&](int ct) { return rows_ok && ct < nct && (!diag || ct >= w); };
    const double* cbase = Cor + (R0 + lr) * ldc + q * kCsR + (COAL ? lc : 4 * lc);
    auto load = [&](int ct, int g, d4 (&dst)[4]) __attribute__((always_inline)) {
        const double* cp = cbase + 64 * ct + 16 * g * ldc;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if constexpr (COAL) {
#pragma unroll
                for (int t = 0; t < 4; ++t) dst[j][t] = __builtin_nontemporal_load(cp + 4 * j * ldc + 16 * t);
            } else {
                dst[j] = __builtin_nontemporal_load(reinterpret_cast<const d4*>(cp + 4 * j * ldc));
            }
        }
    };
    d4 av[4], an[4];
    if (col_on(0)) load(0, 0, av);
    __syncthreads();  // Vc staged
    for (int ct = 0; ct < nct; ++ct) {
        const long long C0 = q * kCsR + 64 * ct;
        const bool con = col_on(ct);
        const bool row_on = con && (!diag || ct > w);
        const bool next_on = col_on(ct + 1);
        const double* vct = Vc[ct];
        d4 acc[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
        if (con) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                if (g < 3) load(ct, g + 1, an);
                else if (next_on) load(ct + 1, 0, an);
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int t = 0; t < 4; ++t)
                        acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[j][t], bv[g][j], acc[t], 0, 0, 0);
                if (row_on) {
                    __builtin_amdgcn_wave_barrier();
#pragma unroll
                    for (int j = 0; j < 4; ++j)
#pragma unroll
                        for (int t = 0; t < 4; ++t)
                            wt[(4 * j + lr) * kCsW + (COAL ? lc + 16 * t : 4 * lc + t)] = av[j][t];
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                    for (int cs = 0; cs < 16; ++cs)
                        dr[g] = __builtin_amdgcn_mfma_f64_16x16x4f64(wt[lc * kCsW + 4 * cs + lr],
                                                                      vct[(4 * cs + lr) * kSB + lc], dr[g], 0, 0, 0);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                }
                if (g < 3 || next_on)
#pragma unroll
                    for (int j = 0; j < 4; ++j) av[j] = an[j];
            }
        } else if (next_on) {
            load(ct + 1, 0, av);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int reg = 0; reg < 4; ++reg)
                wt[(COAL ? (lr + 4 * reg) + 16 * t : 4 * (lr + 4 * reg) + t) * kSB + lc] = acc[t][reg];
        __syncthreads();
        double* out = part_c + ((size_t)p * ldc + C0) * kSB;
        for (int e = threadIdx.x; e < 64 * kSB; e += 256) out[e] = ((Wt[0][e] + Wt[1][e]) + Wt[2][e]) + Wt[3][e];
        __syncthreads();
    }
    if (!rows_ok) return;
    double* outr = part_r + ((size_t)q * ldc + R0) * kSB;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) outr[(16 * g + lr + 4 * reg) * kSB + lc] = dr[g][reg];
}

// Y[i][b] = sum_{p <= P} part_c[p][i][b] + sum_{q >= P} part_r[q][i][b], P = i / 256
__global__ void k_cor_sym_sum(const double* __restrict__ part_c, const double* __restrict__ part_r, long long ldc,
                              long long n, long long nr, double* __restrict__ Y) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * kSB) return;
    const long long P = (t / kSB) / kCsR;
    const size_t stride = (size_t)ldc * kSB;
    double acc = 0.0;
    const double* pc = part_c + t;
    long long s = 0;
    for (; s + 4 <= P + 1; s += 4) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = pc[(s + u) * stride];
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += v[u];
    }
    for (; s <= P; ++s) acc += pc[s * stride];
    const double* pr = part_r + t;
    s = P;
    for (; s + 4 <= nr; s += 4) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = pr[(s + u) * stride];
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += v[u];
    }
    for (; s < nr; ++s) acc += pr[s * stride];
    Y[t] = acc;
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
    __shared__ double sh[4][24];
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
    // block_sum's tree (xor butterfly per wave, then the waves in order from
    // 0.0) for all 24 sums with one barrier instead of two per sum
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const double s = wave_sum(v[k][q]);
            if (lane == 0) sh[wid][k * 8 + q] = s;
        }
    __syncthreads();
    if (threadIdx.x < K * 8) {
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < 4; ++w) t += sh[w][threadIdx.x];
        part[(size_t)i * 24 + threadIdx.x] = t;
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
    DBuf<double> sa;             // N x N Sliding_Approach O/E (hh_comp_sliding_oe), used when sa_on
    int sa_on = 0;
    // last hh_comp_pca: converged flag, Cor products, Krylov cycles, method
    // (0 subspace, 1 Krylov, 2 Krylov redone on the multi-launch path after a
    // k_ortho barrier timeout)
    int pca_converged = 0, pca_products = 0, pca_cycles = 0, pca_method = 0;
    int ortho_fallbacks = 0;
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
    DBuf<double> sym_c, sym_r;  // k_cor_sym partials (allocated at the first symmetric product)
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
        if (!x && !d_use && g_cor_sym) {  // plain product: upper triangle only (k_cor_sym)
            const long long nr = (ldc + kCsR - 1) / kCsR;
            if (!sym_c.p) {
                sym_c.alloc((size_t)nr * ldc * kSB);
                sym_r.alloc((size_t)nr * ldc * kSB);
            }
            HH_KTIME("k_cor_mul", s);
            // (occupancy 2: 190 VGPRs; forcing 3 spills and measured 98.9 vs 105.9 chromosomes/s)
            hipLaunchKernelGGL(g_cor_sym == 3   ? k_cor_sym_pf<true>
                               : g_cor_sym == 2 ? k_cor_sym_pf<false>
                                                : k_cor_sym,
                               dim3((unsigned)(nr * (nr + 1) / 2)), dim3(256),
                               0, s, Cor, ldc, n, V, nr, sym_c.p, sym_r.p);
            hipLaunchKernelGGL(k_cor_sym_sum, dim3((unsigned)((n * kSB + 255) / 256)), dim3(256), 0, s, sym_c.p,
                               sym_r.p, ldc, n, nr, Y);
            return;
        }
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

// ------------------------------------------------------- Krylov PCA (K8)
// Explicit-restart block Krylov on Cor with a Rayleigh-Ritz step for
// A = Xc^T Xc (Xc = Cor - 1 mu^T, the matrix sklearn's PCA factors):
//   cycle: Q_0 = [1/sqrt(n) | top-15 Ritz vectors], Q_{j+1} from Cor Q_j
//   (j < P) by two-pass block Gram-Schmidt with shifted Cholesky-QR3 inside
//   the block (stable down to rank deficiency, unlike CholQR2), so that
//   Cor Q = Q_+ T exactly (T from the Gram-Schmidt coefficients and R
//   factors).  Because 1/sqrt(n) is column 0 of Q_0, Xc Q = (I - q0 q0^T)
//   Cor Q = Q_+ S with S = T minus its row 0: A's projection is S^T S (no
//   squared cancellation), eigen-decomposed on the host.  The Krylov space of
//   Cor of degree 2k contains A's of degree k, so a cycle of P products does
//   the work of P / 2 subspace iterations with optimal polynomial weights:
//   ~45 Cor products per chromosome instead of ~200.

// G = X_k^T Y for nb blocks X_k (n x 16 each, contiguous): part[k][blk][a][b]
__global__ __launch_bounds__(256) void k_gram_mp(const double* __restrict__ X, int nb, const double* __restrict__ Y,
                                                 long long n, int nblk, double* __restrict__ part) {
    __shared__ double xs[64][kSB + 1], ys[64][kSB + 1];
    const int a = threadIdx.x / kSB, b = threadIdx.x % kSB;
    const int xb = blockIdx.y;
    const double* Xk = X + (size_t)xb * n * kSB;
    const long long r0 = (long long)blockIdx.x * kGramRows;
    for (int e = threadIdx.x; e < 64 * kSB; e += 256) {
        const long long i = r0 + e / kSB;
        xs[e / kSB][e % kSB] = i < n ? Xk[i * kSB + e % kSB] : 0.0;
        ys[e / kSB][e % kSB] = i < n ? Y[i * kSB + e % kSB] : 0.0;
    }
    __syncthreads();
    double acc = 0.0;
#pragma unroll 8
    for (int r = 0; r < 64; ++r) acc = fma(xs[r][a], ys[r][b], acc);
    part[((size_t)xb * nblk + blockIdx.x) * kSB * kSB + threadIdx.x] = acc;
}

// G[k][e] = sum over row blocks of part[k][.][e]; fixed tree
__global__ __launch_bounds__(64) void k_gram_ms(const double* __restrict__ part, int nblk, double* __restrict__ G) {
    const int e = blockIdx.x % (kSB * kSB), k = blockIdx.x / (kSB * kSB), l = threadIdx.x;
    const double* p = part + (size_t)k * nblk * kSB * kSB;
    double acc = 0.0;
    for (int r = l; r < nblk; r += 64) acc += p[(size_t)r * kSB * kSB + e];
    acc = wave_sum(acc);
    if (l == 0) G[(size_t)k * kSB * kSB + e] = acc;
}

// out = base - sum_k X_k C_k (base != null) or sum_k X_k C_k (base == null);
// C = nb stacked 16 x 16 blocks (row k*16 + a)
__global__ void k_comb_mp(const double* __restrict__ base, const double* __restrict__ X, int nb,
                          const double* __restrict__ Cm, long long n, double* __restrict__ out) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * kSB) return;
    const long long i = t / kSB;
    const int b = (int)(t % kSB);
    double acc = 0.0;
    for (int k = 0; k < nb; ++k) {
        const double* xr = X + ((size_t)k * n + i) * kSB;
        const double* c = Cm + (size_t)k * kSB * kSB + b;
#pragma unroll
        for (int a = 0; a < kSB; ++a) acc = fma(xr[a], c[a * kSB], acc);
    }
    out[t] = base ? base[t] - acc : acc;
}

// out = (in - sum_k Q_k Cm_k) Rinv for 64 rows per block (Cm == null: no
// subtraction; Rinv == null: identity), plus per-block Gram partials of the
// output: gpart[blk] = out_blk^T out_blk and, when qpart != null,
// qpart[k][blk] = Q_k,blk^T out_blk (k < nb) — the next step's reductions
// without another pass over the rows.  256 threads = 16 rows x 16 columns per
// sub-step; LDS: the 64-row tile, Cm, Rinv.
constexpr int kApplyRows = 64;
// CHOL: Rinv is not an input but the inverse Cholesky factor of the Gram
// matrix whose nin per-block partials are in gin (+ shift_scale * trace on
// the diagonal): every block reduces the partials in the same fixed order and
// factors the 16 x 16 matrix itself, so a separate one-block reduce + Cholesky
// launch and its serialisation disappear from each CholeskyQR pass (block 0 writes
// R and the breakdown flag for the host).  gin must not be gpart.
// shift_scale > 0: shifted CholeskyQR (Fukaya et al.), shift = 11 (m n +
// n (n + 1)) u ||X||^2 with the trace bounding ||X||^2.  Not positive
// definite -> *fail = 1, R = R^{-1} = I.
template <bool CHOL>
__global__ __launch_bounds__(256) void k_apply_t(const double* __restrict__ in, const double* __restrict__ Q, int nb,
                                                 const double* __restrict__ Cm, const double* __restrict__ Rinv,
                                                 long long n, double* __restrict__ out, double* __restrict__ gpart,
                                                 double* __restrict__ qpart, int nblk, const double* __restrict__ gin,
                                                 int nin, double shift_scale, double* __restrict__ Rout,
                                                 int* __restrict__ fail) {
    __shared__ double ts[kApplyRows][kSB + 1], os_[kApplyRows][kSB + 1];
    __shared__ double cm[8 * kSB * kSB], ri[kSB * kSB];
    const int t = threadIdx.x, rr = t / kSB, b = t % kSB;
    const long long r0 = (long long)blockIdx.x * kApplyRows;
    constexpr int PER = kApplyRows * kSB / 256;  // row values staged per thread
    double pre[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {  // issued first: they fly during the reduction / factorisation
        const int e = t + 256 * q;
        const long long i = r0 + e / kSB;
        pre[q] = i < n ? in[i * kSB + e % kSB] : 0.0;
    }
    if (Cm)
        for (int e = t; e < nb * kSB * kSB; e += 256) cm[e] = Cm[e];
    if (CHOL) {
        // ts doubles as scratch for the 16 x 16 Gram matrix before the rows
        // are staged; R goes to ri.
        // 32 loads in flight per thread: the grid is < 1 block per CU here,
        // so registers are free and the dependent round trips are the cost
        double acc = 0.0;
        int r = 0;
        for (; r + 32 <= nin; r += 32) {
            double v[32];
#pragma unroll
            for (int u = 0; u < 32; ++u) v[u] = gin[(size_t)(r + u) * kSB * kSB + t];
#pragma unroll
            for (int u = 0; u < 32; ++u) acc += v[u];
        }
        for (; r < nin; ++r) acc += gin[(size_t)r * kSB * kSB + t];
        ts[rr][b] = acc;
        __syncthreads();
        double tr = 0.0;
#pragma unroll
        for (int i = 0; i < kSB; ++i) tr += ts[i][i];
        const double shift = shift_scale > 0 ? shift_scale * tr : 0.0;
        // right-looking Cholesky inside each wave, registers + shuffles (no
        // block barriers): lane l holds column c = l % 16 of rows
        // (l / 16) + 4 q, q = 0..3; every wave computes the same R, wave 0
        // publishes it
        const int lane = t & 63, c = lane & 15, a0 = lane >> 4;
        double g[4], rrow[kSB];
#pragma unroll
        for (int q = 0; q < 4; ++q) g[q] = ts[a0 + 4 * q][c] + (a0 + 4 * q == c ? shift : 0.0);
        bool okall = true;
#pragma unroll
        for (int j = 0; j < kSB; ++j) {
            const double d = __shfl(g[j >> 2], (j & 3) * 16 + j, 64);
            const bool okd = d > 0;
            okall = okall && okd;
            const double rjj = okd ? sqrt(d) : 1.0;
            const double gjc = __shfl(g[j >> 2], (j & 3) * 16 + c, 64);
            const double rjc = c == j ? rjj : (c > j ? gjc / rjj : 0.0);
            rrow[j] = rjc;  // R[j][c]
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int a = a0 + 4 * q;
                const double rja = __shfl(rjc, a, 64);  // R[j][a]
                if (a > j && c > j) g[q] -= rja * rjc;
            }
        }
        if (t < kSB) {  // wave 0, lanes 0..15: column c = t
#pragma unroll
            for (int j = 0; j < kSB; ++j) {
                const double rv = okall ? rrow[j] : (j == c ? 1.0 : 0.0);
                ri[j * kSB + c] = rv;  // R (upper), row-major
                if (blockIdx.x == 0) Rout[j * kSB + c] = rv;
            }
            if (t == 0 && blockIdx.x == 0 && !okall) *fail = 1;
        }
        __syncthreads();  // R published; scratch reads done before the rows are staged
    } else if (Rinv) {
        ri[t] = Rinv[t];
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int e = t + 256 * q;
        ts[e / kSB][e % kSB] = pre[q];
    }
    __syncthreads();
    if (Cm) {
        double acc[kApplyRows / 16];
#pragma unroll
        for (int q = 0; q < kApplyRows / 16; ++q) acc[q] = ts[rr + 16 * q][b];
        for (int k = 0; k < nb; ++k) {
            const double* Qk = Q + (size_t)k * n * kSB;
#pragma unroll
            for (int q = 0; q < kApplyRows / 16; ++q) {
                const long long i = r0 + rr + 16 * q;
                if (i >= n) continue;
                const double* qr = Qk + i * kSB;
                double s = 0.0;
#pragma unroll
                for (int a = 0; a < kSB; ++a) s = fma(qr[a], cm[(k * kSB + a) * kSB + b], s);
                acc[q] -= s;
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kApplyRows / 16; ++q) ts[rr + 16 * q][b] = acc[q];
        __syncthreads();
    }
    if (CHOL) {
        // out_row = row R^{-1}: forward substitution x R = row, one thread
        // per row (no R^{-1}, none of its 16 barrier steps)
        if (t < kApplyRows) {
            const long long i = r0 + t;
            double x[kSB];
#pragma unroll
            for (int c = 0; c < kSB; ++c) {
                double v = ts[t][c];
#pragma unroll
                for (int a = 0; a < c; ++a) v -= x[a] * ri[a * kSB + c];
                x[c] = v / ri[c * kSB + c];
            }
#pragma unroll
            for (int c = 0; c < kSB; ++c) {
                const double v = i < n ? x[c] : 0.0;
                os_[t][c] = v;
                if (i < n) out[i * kSB + c] = v;
            }
        }
    } else {
#pragma unroll
        for (int q = 0; q < kApplyRows / 16; ++q) {
            const int r = rr + 16 * q;
            double v = ts[r][b];
            if (Rinv) {
                v = 0.0;
#pragma unroll
                for (int a = 0; a < kSB; ++a) v = fma(ts[r][a], ri[a * kSB + b], v);
            }
            const long long i = r0 + r;
            if (i >= n) v = 0.0;
            os_[r][b] = v;
            if (i < n) out[i * kSB + b] = v;
        }
    }
    __syncthreads();
    if (gpart) {
        const int a = t / kSB;
        double acc = 0.0;
#pragma unroll 8
        for (int r = 0; r < kApplyRows; ++r) acc = fma(os_[r][a], os_[r][b], acc);
        gpart[(size_t)blockIdx.x * kSB * kSB + t] = acc;
    }
    if (qpart) {
        const int a = t / kSB;
        const long long rmax = n - r0;  // rows of this block inside the matrix
        for (int k = 0; k < nb; ++k) {
            const double* Qk = Q + ((size_t)k * n + r0) * kSB + a;
            double acc = 0.0;
#pragma unroll 16
            for (int r = 0; r < kApplyRows; ++r) {
                const double q = r < rmax ? Qk[(size_t)r * kSB] : 0.0;
                acc = fma(q, os_[r][b], acc);
            }
            qpart[((size_t)k * nblk + blockIdx.x) * kSB * kSB + t] = acc;
        }
    }
}

// start block [1/sqrt(n) | X[:, 0..14]]
__global__ void k_start_block(const double* __restrict__ X, long long n, double* __restrict__ out) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * kSB) return;
    const long long i = t / kSB;
    const int b = (int)(t % kSB);
    out[t] = b == 0 ? 1.0 / sqrt((double)n) : X[i * kSB + b - 1];
}

// ------------------------------------ one-launch block orthogonalisation
// The whole Gram-Schmidt + shifted CholeskyQR3 chain of one Krylov product
// (or of a restart) in ONE launch instead of ~11: the chain is a sequence of
// row-local steps separated by 16 x 16 (or nb x 16 x 16) reductions over all
// rows, so a block owns 64 * TPB rows for the whole launch (kept in LDS) and
// the reductions are grid-wide: per-block partials, a grid barrier, then a
// fixed-order sum over the blocks (every block for a 16 x 16 Gram, a
// reduce-scatter + second barrier for the nb x 16 x 16 projections).
// Deterministic.  The per-block products run on v_mfma_f64_16x16x4f64:
//   Gram / projection: A = X^T or Q^T (lane l: row 4c + l / 16, column l % 16),
//   B = X (same lane map), D = 16 x 16 partial; X -= Q C: A = Q (16 rows),
//   B = C.  D layout (f64): column = lane & 15, row = (lane >> 4) + 4 reg.
// The grid is <= kOrthoMaxBlocks blocks of 256 threads (the chip holds
// several such grids at once, one per stream), and every barrier wait is
// bounded: a grid that cannot become co-resident sets *abort and runs to
// its end (the host raises) instead of hanging.
constexpr int kOrthoMaxBlocks = 64;
constexpr int kOrthoMaxE = 8 * kSB * kSB;  // nb <= P <= 8 coefficient blocks
constexpr double kOrthoFastRatio = 1e3;    // scholqr3's two-pass branch (see there)
// a low-synch pass's Pythagorean Gram G_W - c^T c is used only when its
// smallest pivot^2 is above this fraction of W's largest squared column norm
// (its rounding, ~eps |W|^2, then perturbs the factor by < ~1e-6)
constexpr double kOrthoPythFloor = 1e-10;
enum { kOrthoFull = 0, kOrthoLast = 1, kOrthoStart = 2, kOrthoRitz = 3, kOrthoFullLS = 4 };

struct OrthoArgs {
    const double* xin = nullptr;  // Full / Last: W = Cor Q_j; Start: the start block's rows
    const double* Y = nullptr;    // Ritz: nb stacked 16 x 16 coefficient blocks
    double* xout = nullptr;       // Ritz: X = Q Y out (the host's Ritz vectors)
    const double* Q = nullptr;    // basis blocks (n x 16 each)
    int nb = 0;
    double* qnext = nullptr;       // Full: Q_{j+1}; Start / Ritz: Q_0
    double *c1 = nullptr, *c2 = nullptr, *R = nullptr, *G = nullptr;  // small outputs (block 0)
    int* fail = nullptr;           // one flag per Cholesky (written 0 / 1)
    double *rpart = nullptr, *rout = nullptr, *gpart = nullptr;
    unsigned long long* ctr = nullptr;  // two barrier-arrival counters: this launch uses ctr[par] (from 0)
    int par = 0;                         // and zeroes ctr[1 - par] for the next one
    int* abort = nullptr;
    long long n = 0;
    int nblk = 0;
    double shift_scale = 0.0;
    long long* tstamp = nullptr;  // pca_debug >= 2: block 0's clock at the start, around each barrier, at the end
    int pre = 1;                  // FullLS basis-row prefetch: 0 off, 1 mul_q's, 2 also pass B's proj_part
};

// HH_ORTHO_PRE (environment, read once): OrthoArgs::pre for the experiments.
// Measured (profiles/r5s, serial k_ortho per C5 pass): 0 84.2 ms, 1 81.2 ms,
// 2 81.6 ms -- the prefetched rows make mul_q ~3x faster but queue ahead of
// the reduction's loads, so the reduction gets slower by most of it
static int ortho_pre_level() {
    static const int v = [] {
        const char* e = std::getenv("HH_ORTHO_PRE");
        return e ? std::atoi(e) : 1;
    }();
    return v;
}

// grid barrier (all blocks co-resident); bounded wait.  `between` runs after
// this block's arrival and before its wait (loads issued there do not hold
// up the arrival's release fence)
template <typename F>
__device__ __forceinline__ void ortho_grid_sync(unsigned long long* ctr, unsigned long long target, int* abort,
                                                F&& between) {
    __syncthreads();
    if (threadIdx.x == 0) {
        // release only: this block's partials reach memory.  No acquire
        // fence afterwards -- it would invalidate the XCD's L2 and every Q
        // row read of the next phase would go to HBM; the cross-block data
        // are read with agent-scope atomic loads (ld_agent) instead
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        atomicAdd(ctr, 1ull);
    }
    between();
    if (threadIdx.x == 0) {
        unsigned spins = 0;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if ((++spins & 255u) == 0u &&
                (spins >= (1u << 22) || __hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
                atomicExch(abort, 1);
                break;
            }
        }
    }
    __syncthreads();
}

// a coherent (L2-bypassing) load of another block's partial
__device__ __forceinline__ double ld_agent(const double* p) {
    return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
    const unsigned long long u = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, lane);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), lane);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

template <int TPB>
struct OrthoLds {
    double x[TPB * 64][kSB + 1];  // the block's rows
    double cm[kOrthoMaxE];        // reduced coefficients
    double gs[kSB * kSB];         // reduced Gram
    double ri[kSB * kSB];         // Cholesky factor R (upper, row-major)
    double rd[kSB];               // 1 / R[c][c]
    int ok;                       // the last Cholesky succeeded
    double ws[4][kOrthoMaxE];     // per-wave MFMA partials (Gram: the first 256 of each)
};

template <int MODE, int TPB>
__global__ __launch_bounds__(256) void k_ortho(OrthoArgs Ain) {
    // the arguments as locals (the lambdas below captured the by-value
    // struct by reference, which kept a copy of it in scratch)
    const auto A_G = Ain.G;
    const auto A_Q = Ain.Q;
    const auto A_R = Ain.R;
    const auto A_Y = Ain.Y;
    const auto A_abort = Ain.abort;
    const auto A_c1 = Ain.c1;
    const auto A_c2 = Ain.c2;
    const auto A_ctr = Ain.ctr;
    const auto A_fail = Ain.fail;
    const auto A_gpart = Ain.gpart;
    const auto A_n = Ain.n;
    const auto A_nb = Ain.nb;
    const auto A_nblk = Ain.nblk;
    const auto A_par = Ain.par;
    const auto A_qnext = Ain.qnext;
    const auto A_rout = Ain.rout;
    const auto A_rpart = Ain.rpart;
    const auto A_shift_scale = Ain.shift_scale;
    const auto A_tstamp = Ain.tstamp;
    const auto A_xin = Ain.xin;
    const auto A_xout = Ain.xout;
    const int A_pre = Ain.pre;

    constexpr int B = kSB, BB = kSB * kSB, RPB = 64 * TPB;
    __shared__ OrthoLds<TPB> L;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, lr = lane >> 4, lc = lane & 15;
    const int nblk = A_nblk, g = blockIdx.x;
    const long long n = A_n, r0 = (long long)g * RPB;
    unsigned bar = 0;
    auto stamp = [&](int k) __attribute__((always_inline)) {
        if (A_tstamp && g == 0 && t == 0) A_tstamp[k] = (long long)wall_clock64();
    };
    stamp(0);
    if (g == 0 && t == 0) A_ctr[1 - A_par] = 0ull;  // the previous launch's counter (it has completed)
    auto gsync_then = [&](auto&& between) __attribute__((always_inline)) {
        ++bar;
        stamp(2 * bar - 1);
        ortho_grid_sync(A_ctr + A_par, (unsigned long long)bar * (unsigned long long)nblk, A_abort, between);
        stamp(2 * bar);
    };
    auto gsync = [&]() __attribute__((always_inline)) { gsync_then([] {}); };
    // ---- block-local pieces
    auto gram_part = [&](double* dst) __attribute__((always_inline)) {  // dst[g][256] = X^T X over the block's rows
        d4 acc = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int m = 0; m < TPB; ++m)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const double v = L.x[(w + 4 * m) * 16 + 4 * c + lr][lc];
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(v, v, acc, 0, 0, 0);
            }
#pragma unroll
        for (int r = 0; r < 4; ++r) L.ws[w][(lr + 4 * r) * B + lc] = acc[r];
        __syncthreads();
        dst[(size_t)g * BB + t] = ((L.ws[0][t] + L.ws[1][t]) + L.ws[2][t]) + L.ws[3][t];
        __syncthreads();
    };
    // rpart[g][k][256] = Q_k^T X over the block's rows: each wave its row
    // groups, four k at a time with all their loads in flight (one round
    // trip per four k), the waves' partials summed in wave order
    auto proj_part = [&]() __attribute__((always_inline)) {
        const int nb = A_nb;
        for (int kc = 0; kc < nb; kc += 4) {
            d4 acc[4];
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) acc[kk] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int m = 0; m < TPB; ++m) {
                double q[4][4];
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const long long i = r0 + (w + 4 * m) * 16 + 4 * c + lr;
                        q[kk][c] = (kc + kk < nb && i < n) ? A_Q[((size_t)(kc + kk) * n + i) * B + lc] : 0.0;
                    }
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                    for (int c = 0; c < 4; ++c)
                        acc[kk] = __builtin_amdgcn_mfma_f64_16x16x4f64(q[kk][c], L.x[(w + 4 * m) * 16 + 4 * c + lr][lc],
                                                                       acc[kk], 0, 0, 0);
            }
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
                if (kc + kk < nb)
#pragma unroll
                    for (int r = 0; r < 4; ++r) L.ws[w][(kc + kk) * BB + (lr + 4 * r) * B + lc] = acc[kk][r];
        }
        __syncthreads();
        for (int e = t; e < nb * BB; e += 256)
            A_rpart[(size_t)g * kOrthoMaxE + e] = ((L.ws[0][e] + L.ws[1][e]) + L.ws[2][e]) + L.ws[3][e];
        __syncthreads();
    };
    // X (+|-)= sum_k Q_k cm_k over the block's rows (ADD: X = sum, X zero
    // before); four k at a time with all their loads in flight
    auto mul_q = [&](bool add) __attribute__((always_inline)) {
        const int nb = A_nb;
        d4 acc[TPB];
#pragma unroll
        for (int m = 0; m < TPB; ++m) acc[m] = d4{0.0, 0.0, 0.0, 0.0};
        for (int kc = 0; kc < nb; kc += 4) {
            double q[TPB][4][4];
#pragma unroll
            for (int m = 0; m < TPB; ++m) {
                const long long i = r0 + (w + 4 * m) * 16 + lc;
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj)
                        q[m][kk][jj] =
                            (kc + kk < nb && i < n) ? A_Q[((size_t)(kc + kk) * n + i) * B + 4 * jj + lr] : 0.0;
            }
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                double bcol[4];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj)
                    bcol[jj] = kc + kk < nb ? L.cm[(kc + kk) * BB + (4 * jj + lr) * B + lc] : 0.0;
#pragma unroll
                for (int m = 0; m < TPB; ++m)
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj)
                        acc[m] = __builtin_amdgcn_mfma_f64_16x16x4f64(q[m][kk][jj], bcol[jj], acc[m], 0, 0, 0);
            }
        }
#pragma unroll
        for (int m = 0; m < TPB; ++m) {
            const int rb = (w + 4 * m) * 16;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                double& x = L.x[rb + lr + 4 * r][lc];
                x = add ? acc[m][r] : x - acc[m][r];
            }
        }
        __syncthreads();
    };
    // FullLS at TPB <= 2: the block's basis rows for the next proj_part /
    // mul_q are loaded ahead of the step before them (the row loads, a grid
    // reduction, the Cholesky), so their round trip overlaps it.  The same
    // MFMAs on the same operands in the same order as proj_part / mul_q
    // (bitwise the same results); nb <= 8 blocks in one register set.
    constexpr bool kPre = MODE == kOrthoFullLS && TPB <= 2;
    constexpr int kPT = kPre ? TPB : 1, kPK = kPre ? 8 : 4;
    double qb[kPK][kPT][4];
    auto pre_proj = [&]() __attribute__((always_inline)) {  // proj_part's operand layout
        const int nb = A_nb;
#pragma unroll
        for (int k = 0; k < kPK; ++k)
#pragma unroll
            for (int m = 0; m < kPT; ++m)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const long long i = r0 + (w + 4 * m) * 16 + 4 * c + lr;
                    qb[k][m][c] = (k < nb && i < n) ? A_Q[((size_t)k * n + i) * B + lc] : 0.0;
                }
    };
    auto pre_mul = [&]() __attribute__((always_inline)) {  // mul_q's operand layout
        const int nb = A_nb;
#pragma unroll
        for (int k = 0; k < kPK; ++k)
#pragma unroll
            for (int m = 0; m < kPT; ++m) {
                const long long i = r0 + (w + 4 * m) * 16 + lc;
#pragma unroll
                for (int jj = 0; jj < 4; ++jj)
                    qb[k][m][jj] = (k < nb && i < n) ? A_Q[((size_t)k * n + i) * B + 4 * jj + lr] : 0.0;
            }
    };
    auto proj_part_pre = [&]() __attribute__((always_inline)) {
        const int nb = A_nb;
#pragma unroll
        for (int kc = 0; kc < kPK; kc += 4) {
            if (kc < nb) {
                d4 acc[4];
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) acc[kk] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int m = 0; m < kPT; ++m)
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                        for (int c = 0; c < 4; ++c)
                            acc[kk] = __builtin_amdgcn_mfma_f64_16x16x4f64(
                                qb[kc + kk][m][c], L.x[(w + 4 * m) * 16 + 4 * c + lr][lc], acc[kk], 0, 0, 0);
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
                    if (kc + kk < nb)
#pragma unroll
                        for (int r = 0; r < 4; ++r) L.ws[w][(kc + kk) * BB + (lr + 4 * r) * B + lc] = acc[kk][r];
            }
        }
        __syncthreads();
        for (int e = t; e < nb * BB; e += 256)
            A_rpart[(size_t)g * kOrthoMaxE + e] = ((L.ws[0][e] + L.ws[1][e]) + L.ws[2][e]) + L.ws[3][e];
        __syncthreads();
    };
    auto mul_q_pre = [&](bool add) __attribute__((always_inline)) {
        const int nb = A_nb;
        d4 acc[kPT];
#pragma unroll
        for (int m = 0; m < kPT; ++m) acc[m] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kc = 0; kc < kPK; kc += 4) {
            if (kc < nb) {
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    double bcol[4];
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj)
                        bcol[jj] = kc + kk < nb ? L.cm[(kc + kk) * BB + (4 * jj + lr) * B + lc] : 0.0;
#pragma unroll
                    for (int m = 0; m < kPT; ++m)
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj)
                            acc[m] = __builtin_amdgcn_mfma_f64_16x16x4f64(qb[kc + kk][m][jj], bcol[jj], acc[m], 0, 0, 0);
                }
            }
        }
#pragma unroll
        for (int m = 0; m < kPT; ++m) {
            const int rb = (w + 4 * m) * 16;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                double& x = L.x[rb + lr + 4 * r][lc];
                x = add ? acc[m][r] : x - acc[m][r];
            }
        }
        __syncthreads();
    };
    // L.gs = sum over blocks of gp (fixed block order), every block; all
    // nblk loads in flight at once
    auto reduce_gram = [&](const double* gp) __attribute__((always_inline)) {
        double v[kOrthoMaxBlocks];
#pragma unroll
        for (int b = 0; b < kOrthoMaxBlocks; ++b) v[b] = b < nblk ? ld_agent(gp + (size_t)b * BB + t) : 0.0;
        double acc = 0.0;
#pragma unroll
        for (int b = 0; b < kOrthoMaxBlocks; ++b) acc += v[b];  // trailing + 0.0: exact
        L.gs[t] = acc;
        __syncthreads();
    };
    // nb x 256 projection sums: barrier, reduce-scatter over the blocks,
    // barrier, every block reads all of them into L.cm (block 0 also to `out`)
    auto reduce_proj_then = [&](double* out, int extra, auto&& between) __attribute__((always_inline)) {
        gsync_then(between);  // every block's partials are in
        const int E = (A_nb + extra) * BB, chunk = (E + nblk - 1) / nblk;
        const int e1 = min(E, (g + 1) * chunk);
        for (int e = g * chunk + t; e < e1; e += 256) {
            double v[kOrthoMaxBlocks];
#pragma unroll
            for (int b = 0; b < kOrthoMaxBlocks; ++b)
                v[b] = b < nblk ? ld_agent(A_rpart + (size_t)b * kOrthoMaxE + e) : 0.0;
            double acc = 0.0;
#pragma unroll
            for (int b = 0; b < kOrthoMaxBlocks; ++b) acc += v[b];
            A_rout[e] = acc;
        }
        gsync();
        // every coefficient loaded before the first is stored (clamped
        // addresses, no select): a loop of load -> use compiled to one
        // round trip per 256 coefficients, up to 8 in a row (ISA-checked)
        constexpr int kIt = kOrthoMaxE / 256;
        double cv[kIt];
#pragma unroll
        for (int q = 0; q < kIt; ++q) cv[q] = ld_agent(A_rout + min(t + 256 * q, E - 1));
#pragma unroll
        for (int q = 0; q < kIt; ++q) {
            const int e = t + 256 * q;
            if (e < E) {
                L.cm[e] = cv[q];
                if (g == 0 && e < A_nb * BB) out[e] = cv[q];
            }
        }
        for (int e = t + 256 * kIt; e < E; e += 256) {  // (E <= kOrthoMaxE: not reached)
            const double v = ld_agent(A_rout + e);
            L.cm[e] = v;
            if (g == 0 && e < A_nb * BB) out[e] = v;
        }
        __syncthreads();
    };
    auto reduce_proj = [&](double* out, int extra = 0) __attribute__((always_inline)) {
        reduce_proj_then(out, extra, [] {});
    };
    // low-synch passes (one reduction per pass): the block's Gram X^T X as
    // coefficient block nb of its projection partials, reduced in the same
    // reduce-scatter; then the Gram of X - Qa c by Pythagoras,
    // G - c^T c (Qa orthonormal), into L.gs
    auto gram_into_proj = [&]() __attribute__((always_inline)) {
        d4 acc = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int m = 0; m < TPB; ++m)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const double v = L.x[(w + 4 * m) * 16 + 4 * c + lr][lc];
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(v, v, acc, 0, 0, 0);
            }
#pragma unroll
        for (int r = 0; r < 4; ++r) L.ws[w][(lr + 4 * r) * B + lc] = acc[r];
        __syncthreads();
        A_rpart[(size_t)g * kOrthoMaxE + (size_t)A_nb * BB + t] =
            ((L.ws[0][t] + L.ws[1][t]) + L.ws[2][t]) + L.ws[3][t];
        __syncthreads();
    };
    auto pythagoras = [&]() __attribute__((always_inline)) {
        const int i = t / B, j = t % B;
        double acc = 0.0;
        for (int k = 0; k < A_nb; ++k) {
            const double* ck = L.cm + k * BB;
#pragma unroll
            for (int m = 0; m < B; ++m) acc = fma(ck[m * B + i], ck[m * B + j], acc);
        }
        L.gs[t] = L.cm[A_nb * BB + t] - acc;
        __syncthreads();
    };
    // R = chol(L.gs + shift) in every wave (registers + shuffles), wave 0
    // publishes it; not positive definite -> R = I and the flag
    // R = chol(L.gs + shift) in wave 0: lane c holds column c and the pivot
    // row / diagonal come from their lanes by v_readlane (the loop indices are
    // compile-time: no LDS round trip per step, as the shuffles were); not
    // positive definite -> R = I and the flag
    auto chol = [&](bool shifted, double* Rout, int* flag) __attribute__((always_inline)) {
        if (w == 0) {
            double tr = 0.0;
#pragma unroll
            for (int i = 0; i < B; ++i) tr += L.gs[i * B + i];
            const double shift = shifted ? A_shift_scale * tr : 0.0;
            const int c = lc;
            double gcol[B], rcol[B];
#pragma unroll
            for (int a = 0; a < B; ++a) gcol[a] = L.gs[a * B + c] + (a == c ? shift : 0.0);
            bool okall = true;
#pragma unroll
            for (int j = 0; j < B; ++j) {
                const double d = readlane_d(gcol[j], j);
                const bool okd = d > 0;
                okall = okall && okd;
                // 1 / sqrt(d) from v_rsq_f64 + one Newton step (the serial
                // chain was 16 x (sqrt + divide) = 5 us of the pass)
                const double dd = okd ? d : 1.0;
                double y = __builtin_amdgcn_rsq(dd);
                y = y * fma(-0.5 * dd * y, y, 1.5);
                const double rjj = dd * y;
                const double rjc = c == j ? rjj : (c > j ? gcol[j] * y : 0.0);
                rcol[j] = rjc;
                // the trailing update without a lane predicate: lanes c < j
                // have rjc = 0, and lane j's column is not read again (its
                // pivot and rcol are final), so only lanes c > j matter and
                // they take the same fma as before (no selects per element)
#pragma unroll
                for (int a = j + 1; a < B; ++a) {
                    const double rja = readlane_d(rjc, a);
                    gcol[a] -= rja * rjc;
                }
            }
            if (lane < B) {
#pragma unroll
                for (int j = 0; j < B; ++j) {
                    const double rv = okall ? rcol[j] : (j == c ? 1.0 : 0.0);
                    L.ri[j * B + c] = rv;
                    if (g == 0) Rout[j * B + c] = rv;
                }
                L.rd[c] = 1.0 / (okall ? rcol[c] : 1.0);
                if (lane == 0) L.ok = okall ? 1 : 0;
                if (lane == 0 && g == 0) *flag = okall ? 0 : 1;
            }
        }
        __syncthreads();
    };
    auto apply_rinv = [&]() __attribute__((always_inline)) {  // row <- row R^{-1} (forward substitution, a thread per row)
        for (int r = t; r < RPB; r += 256) {
            double x[B];
#pragma unroll
            for (int c = 0; c < B; ++c) {
                double v = L.x[r][c];
#pragma unroll
                for (int a = 0; a < c; ++a) v -= x[a] * L.ri[a * B + c];
                x[c] = v * L.rd[c];
            }
#pragma unroll
            for (int c = 0; c < B; ++c) L.x[r][c] = x[c];
        }
        __syncthreads();
    };
    // one CholeskyQR pass on the rows (Gram -> barrier -> R -> X R^{-1});
    // the Gram buffers alternate so a block's next partial never overwrites
    // one another block may still be reading
    unsigned gsel = 0;
    auto cholqr = [&](bool shifted, double* Rout, int* flag) __attribute__((always_inline)) {
        double* gp = A_gpart + (size_t)(gsel & 1u) * nblk * BB;
        const bool st = gsel == 1;  // pca_debug 2: the second pass in detail
        ++gsel;
        if (st) stamp(40);
        gram_part(gp);
        if (st) stamp(41);
        gsync();
        if (st) stamp(42);
        reduce_gram(gp);
        if (st) stamp(43);
        chol(shifted, Rout, flag);
        if (st) stamp(44);
        apply_rinv();
        if (st) stamp(45);
    };
    // shifted CholeskyQR3 -> R3[0..2]: when the first (shifted) factor is
    // well conditioned (diagonal ratio < kOrthoFastRatio: the block had no
    // rounding-level direction), one plain pass finishes it (CholQR2's
    // regime) and the third factor is the identity; otherwise shifted,
    // shifted, plain.  Every block takes the same branch (same R).
    auto scholqr3 = [&](double* R3, int* fl) __attribute__((always_inline)) {
        cholqr(true, R3, fl);
        double mx = 0.0, mn = 1e300;
#pragma unroll
        for (int i = 0; i < B; ++i) {
            const double v = fabs(L.ri[i * B + i]);
            mx = fmax(mx, v);
            mn = fmin(mn, v);
        }
        if (L.ok && mn > 0.0 && mx < kOrthoFastRatio * mn) {
            cholqr(false, R3 + BB, fl + 1);
            if (g == 0) {
                R3[2 * BB + t] = (t / B == t % B) ? 1.0 : 0.0;
                if (t == 0) fl[2] = 0;
            }
        } else {
            cholqr(true, R3 + BB, fl + 1);
            cholqr(false, R3 + 2 * BB, fl + 2);
        }
    };
    // (scholqr3 always computes the Gram of the rows in LDS: the robust
    // fallback of a low-synch pass is the round-3 chain on X - Qa c)
    auto scholqr3_direct = [&](double* R3, int* fl) __attribute__((always_inline)) { scholqr3(R3, fl); };
    auto store_rows = [&](double* dst) __attribute__((always_inline)) {
        for (int e = t; e < RPB * B; e += 256) {
            const long long i = r0 + e / B;
            if (i < n) dst[i * B + e % B] = L.x[e / B][e % B];
        }
    };
    // ---- the block's rows in
    if constexpr (kPre)
        if (A_pre >= 1) pre_proj();  // (pass A's basis rows first: in flight with W's)
    if (MODE != kOrthoRitz) {  // W (Full / Last) or the start block
        // all the block's row loads in flight at once (clamped rows, zeroed
        // by a 0 / 1 factor: `i < n ? load : 0` compiled to one round trip
        // per 256 elements, 8 in a row; ISA-checked)
        constexpr int kIt = RPB * B / 256;
        double xv[kIt];
#pragma unroll
        for (int q = 0; q < kIt; ++q) {
            const int e = t + 256 * q;
            const long long i = r0 + e / B;
            xv[q] = A_xin[(i < n ? i : n - 1) * B + e % B];
        }
#pragma unroll
        for (int q = 0; q < kIt; ++q) {
            const int e = t + 256 * q;
            L.x[e / B][e % B] = xv[q] * (r0 + e / B < n ? 1.0 : 0.0);
        }
    } else {  // Ritz vectors X = Q Y out, then the start block [1 / sqrt(n) | X[:, 0..14]]
        for (int e = t; e < A_nb * BB; e += 256) L.cm[e] = A_Y[e];
        __syncthreads();
        mul_q(true);
        store_rows(A_xout);
        __syncthreads();
        const double c0 = 1.0 / sqrt((double)n);
        for (int r = t; r < RPB; r += 256) {
            const bool in = r0 + r < n;
            for (int c = B - 1; c > 0; --c) L.x[r][c] = L.x[r][c - 1];
            L.x[r][0] = in ? c0 : 0.0;
        }
    }
    __syncthreads();
    if (MODE == kOrthoFullLS) {
        // Low-synch CGS2 (two reductions per product instead of ~8): each pass
        // reduces the projections Qa^T X and the Gram X^T X together, forms
        // the Gram of X - Qa c by Pythagoras and factors it.  Pass A's Gram
        // loses digits when W lies nearly in span(Qa), so its (shifted)
        // factor is taken only when well conditioned and not cancelled
        // (every block decides from the same reduced numbers); else the
        // residual's Gram is computed directly and shifted CholeskyQR3 runs,
        // as in the round-3 path.  Pass B's Gram (Q1 against Qa) has no
        // cancellation: Q1 is orthonormal to the working accuracy of pass A.
        auto lowsync_pass = [&](double* cout, double* R3, int* fl, bool shifted, int so) -> bool {
            stamp(so);
            const bool pre = kPre && A_pre >= 1;
            if (pre && (so == 20 || A_pre >= 2)) proj_part_pre();
            else proj_part();
            stamp(so + 1);
            gram_into_proj();
            if (pre) reduce_proj_then(cout, 1, pre_mul);  // mul_q's rows in flight across the barrier
            else reduce_proj(cout, 1);
            stamp(so + 2);
            double gwmax = 0.0;
#pragma unroll
            for (int i = 0; i < B; ++i) gwmax = fmax(gwmax, L.cm[A_nb * BB + i * B + i]);
            pythagoras();
            stamp(so + 3);
            if (pre) {
                mul_q_pre(false);
                if (so == 20 && A_pre >= 2) pre_proj();  // pass B's basis rows, in flight across the Cholesky
            } else {
                mul_q(false);
            }
            stamp(so + 4);
            chol(shifted, R3, fl);
            stamp(so + 5);
            double mx = 0.0, mn = 1e300;
#pragma unroll
            for (int i = 0; i < B; ++i) {
                const double v = fabs(L.ri[i * B + i]);
                mx = fmax(mx, v);
                mn = fmin(mn, v);
            }
            if (!(L.ok && mn > 0.0 && mx < kOrthoFastRatio * mn && mn * mn > kOrthoPythFloor * gwmax)) {
                if (g == 0 && t == 0) *fl = 0;  // the robust path below sets the flags
                return false;
            }
            apply_rinv();
            stamp(so + 6);
            if (g == 0) {
                R3[BB + t] = (t / B == t % B) ? 1.0 : 0.0;
                R3[2 * BB + t] = (t / B == t % B) ? 1.0 : 0.0;
                if (t < 2) fl[1 + t] = 0;
            }
            return true;
        };
        if (!lowsync_pass(A_c1, A_R, A_fail, true, 20)) scholqr3_direct(A_R, A_fail);
        if (!lowsync_pass(A_c2, A_R + 3 * BB, A_fail + 3, false, 28)) scholqr3_direct(A_R + 3 * BB, A_fail + 3);
        store_rows(A_qnext);
    } else if (MODE == kOrthoFull) {
        // pass A: X = W - Qa c1, shifted CholQR3 -> Q1 (factors R0..R2)
        proj_part();
        reduce_proj(A_c1);
        mul_q(false);
        scholqr3(A_R, A_fail);
        // pass B: X = Q1 - Qa c2, shifted CholQR3 -> Q_{j+1} (R3..R5)
        proj_part();
        reduce_proj(A_c2);
        mul_q(false);
        scholqr3(A_R + 3 * BB, A_fail + 3);
        store_rows(A_qnext);
    } else if (MODE == kOrthoLast) {
        // CGS2 coefficients of the last product and the Gram of its residual
        proj_part();
        reduce_proj(A_c1);
        mul_q(false);
        proj_part();
        reduce_proj(A_c2);
        mul_q(false);
        gram_part(A_gpart);
        gsync();
        if (g == 0) {
            reduce_gram(A_gpart);
            A_G[t] = L.gs[t];
        }
    } else {
        scholqr3(A_R, A_fail);
        store_rows(A_qnext);
    }
    stamp(39);
    if (A_tstamp && g == 0 && t == 0) A_tstamp[38] = bar;
}

// ---------------------------------------------- small symmetric eigen (host)
// Householder tridiagonalisation T = Q^T A Q (Golub & Van Loan 8.3.1; A full
// m x m row-major, destroyed), Q kept as reflectors (v_k, beta_k).
struct Tridiag {
    int m = 0;
    std::vector<double> d, e, V, beta;  // e[i] = T[i+1][i]
};
static void tridiagonalize(int m, std::vector<double>& A, Tridiag& T) {
    // only the lower triangle is read and updated (half the traffic of the
    // full-matrix form; the m = 128 matrix does not fit L1): p = A22 v as
    // one pass over the rows, each row giving a dot (j < i) and an axpy into
    // p (j < i), four partial sums so the loops vectorise
    T.m = m;
    T.V.assign((size_t)m * m, 0.0);
    T.beta.assign(m, 0.0);
    std::vector<double> p(m), w(m);
    for (int k = 0; k + 2 < m; ++k) {
        double sig = 0.0;
        for (int i = k + 2; i < m; ++i) sig += A[(size_t)i * m + k] * A[(size_t)i * m + k];
        if (sig == 0.0) continue;
        const double x0 = A[(size_t)(k + 1) * m + k];
        const double mu = std::sqrt(x0 * x0 + sig);
        const double v0 = x0 <= 0 ? x0 - mu : -sig / (x0 + mu);
        const double beta = 2.0 * v0 * v0 / (sig + v0 * v0);
        double* v = &T.V[(size_t)k * m];
        v[k + 1] = 1.0;
        for (int i = k + 2; i < m; ++i) v[i] = A[(size_t)i * m + k] / v0;
        T.beta[k] = beta;
        // A22 <- P A22 P, P = I - beta v v^T:  p = beta A22 v,
        // w = p - (beta / 2)(p^T v) v,  A22 -= v w^T + w v^T
        const double* __restrict__ vr = v;
        double* __restrict__ pr = p.data();
        for (int i = k + 1; i < m; ++i) pr[i] = 0.0;
        for (int i = k + 1; i < m; ++i) {
            const double* __restrict__ ai = &A[(size_t)i * m];
            const double vi = vr[i];
            // the four partial sums and the axpy as one 4-wide vector each
            // (lane q: elements j + q, the same IEEE operations in the same
            // order as four scalar accumulators; the compiler's vectorisers
            // left this loop scalar.  Two rows interleaved, for two dot
            // chains in flight, measured slower)
            typedef double hd4 __attribute__((ext_vector_type(4)));
            hd4 sv = {0.0, 0.0, 0.0, 0.0};
            const hd4 viv = {vi, vi, vi, vi};
            int j = k + 1;
            for (; j + 4 <= i; j += 4) {
                hd4 a, x, q;
                __builtin_memcpy(&a, ai + j, sizeof(a));
                __builtin_memcpy(&x, vr + j, sizeof(x));
                __builtin_memcpy(&q, pr + j, sizeof(q));
                sv += a * x;
                q += a * viv;
                __builtin_memcpy(pr + j, &q, sizeof(q));
            }
            double s0 = sv.x, s1 = sv.y, s2 = sv.z, s3 = sv.w;
            for (; j < i; ++j) {
                s0 += ai[j] * vr[j];
                pr[j] += ai[j] * vi;
            }
            pr[i] += ((s0 + s1) + (s2 + s3)) + ai[i] * vi;
        }
        double pv = 0.0;
        for (int i = k + 1; i < m; ++i) {
            pr[i] *= beta;
            pv += pr[i] * vr[i];
        }
        for (int i = k + 1; i < m; ++i) w[i] = pr[i] - 0.5 * beta * pv * vr[i];
        const double* __restrict__ wr = w.data();
        for (int i = k + 1; i < m; ++i) {
            double* __restrict__ ai = &A[(size_t)i * m];
            const double vi = vr[i], wi = wr[i];
            for (int j = k + 1; j <= i; ++j) ai[j] -= vi * wr[j] + wi * vr[j];
        }
        A[(size_t)(k + 1) * m + k] = mu;
        for (int i = k + 2; i < m; ++i) A[(size_t)i * m + k] = 0.0;
    }
    T.d.resize(m);
    T.e.assign(m, 0.0);
    for (int i = 0; i < m; ++i) T.d[i] = A[(size_t)i * m + i];
    for (int i = 0; i + 1 < m; ++i) T.e[i] = A[(size_t)(i + 1) * m + i];
}

// sqrt(a^2 + b^2) without std::hypot's cost (a libm call per QL rotation was
// half the host eigen time); scaled form only when a square could overflow
static inline double fast_hypot(double a, double b) {
    a = std::fabs(a);
    b = std::fabs(b);
    if (a < 1e150 && b < 1e150) return std::sqrt(a * a + b * b);
    return std::hypot(a, b);
}

// eigenvalues of the symmetric tridiagonal (d, e) by implicit-shift QL
static std::vector<double> tridiag_eigvals(std::vector<double> d, std::vector<double> e) {
    const int m = (int)d.size();
    for (int l = 0; l < m; ++l) {
        for (int iter = 0; iter < 60; ++iter) {
            int mm = l;
            for (; mm < m - 1; ++mm) {
                const double dd = std::fabs(d[mm]) + std::fabs(d[mm + 1]);
                if (std::fabs(e[mm]) <= std::numeric_limits<double>::epsilon() * dd) break;
            }
            if (mm == l) break;
            double g = (d[l + 1] - d[l]) / (2.0 * e[l]);
            double r = fast_hypot(g, 1.0);
            g = d[mm] - d[l] + e[l] / (g + (g >= 0 ? r : -r));
            double s = 1.0, c = 1.0, p = 0.0;
            int i = mm - 1;
            bool underflow = false;
            for (; i >= l; --i) {
                const double f = s * e[i], b = c * e[i];
                r = fast_hypot(f, g);
                e[i + 1] = r;
                if (r == 0.0) {
                    d[i + 1] -= p;
                    e[mm] = 0.0;
                    underflow = true;
                    break;
                }
                s = f / r;
                c = g / r;
                g = d[i + 1] - p;
                r = (d[i] - g) * s + 2.0 * c * b;
                p = s * r;
                d[i + 1] = g + p;
                g = c * r - b;
            }
            if (underflow) continue;
            d[l] -= p;
            e[l] = g;
            e[mm] = 0.0;
        }
    }
    return d;
}

// eigenvectors of the tridiagonal for the k eigenvalues lam[q]: inverse
// iteration with a Gaussian elimination with partial pivoting (two
// superdiagonals), the k shifts side by side (X[i * k + q]: lane q is one
// independent solve; the pivot choice is a per-lane select, so each lane runs
// exactly the operations of a solve on its own)
static void tridiag_invit(const Tridiag& T, const double* lam, int k, double tnorm, std::vector<double>& X) {
    const int m = T.m;
    const double pert = std::max(tnorm, 1e-300) * 1e-14;
    const size_t mk = (size_t)m * k;
    // rows: (sub a_i, diag b_i, sup c_i) of T - sh I
    std::vector<double> l(mk, 0.0), u0(mk), u1(mk, 0.0), u2(mk, 0.0), sh(k), cd(k), cs(k), cs2(k, 0.0);
    std::vector<unsigned char> piv(mk, 0);
    for (int q = 0; q < k; ++q) {
        sh[q] = lam[q] + pert;
        cd[q] = T.d[0] - sh[q];
        cs[q] = m > 1 ? T.e[0] : 0.0;
    }
    // LU with partial pivoting; the current row i holds (cd = diag, cs = sup,
    // cs2 = sup2)
    for (int i = 0; i + 1 < m; ++i) {
        const double na = T.e[i], nc = i + 2 < m ? T.e[i + 1] : 0.0;
        double* __restrict__ li = &l[(size_t)i * k];
        double* __restrict__ a0 = &u0[(size_t)i * k];
        double* __restrict__ a1 = &u1[(size_t)i * k];
        double* __restrict__ a2 = &u2[(size_t)i * k];
        unsigned char* __restrict__ pv = &piv[(size_t)i * k];
        for (int q = 0; q < k; ++q) {
            const double nb = T.d[i + 1] - sh[q];
            const bool sw = std::fabs(na) > std::fabs(cd[q]);  // swap rows i and i+1
            const double cdk = cd[q] == 0.0 ? pert : cd[q];     // (kept row: a zero pivot perturbed)
            const double f = sw ? cd[q] / na : na / cdk;
            pv[q] = sw ? 1 : 0;
            a0[q] = sw ? na : cdk;
            a1[q] = sw ? nb : cs[q];
            a2[q] = sw ? nc : cs2[q];
            li[q] = f;
            const double ncd = sw ? cs[q] - f * nb : nb - f * cs[q];
            const double ncs = sw ? cs2[q] - f * nc : nc - f * cs2[q];
            cd[q] = ncd;
            cs[q] = ncs;
            cs2[q] = 0.0;
        }
    }
    for (int q = 0; q < k; ++q) u0[(size_t)(m - 1) * k + q] = cd[q] == 0.0 ? pert : cd[q];
    X.assign(mk, 0.0);
    for (int i = 0; i < m; ++i)
        for (int q = 0; q < k; ++q)
            X[(size_t)i * k + q] = 1.0 + 0.1 * ((double)u01(mix64(0x7e57ULL * (q + 1) + (uint64_t)i)) - 0.5);
    std::vector<double> nn(k);
    for (int it = 0; it < 3; ++it) {
        // forward: apply the row operations
        for (int i = 0; i + 1 < m; ++i) {
            double* __restrict__ x0 = &X[(size_t)i * k];
            double* __restrict__ x1 = x0 + k;
            const double* __restrict__ li = &l[(size_t)i * k];
            const unsigned char* __restrict__ pv = &piv[(size_t)i * k];
            for (int q = 0; q < k; ++q) {
                const double a = pv[q] ? x1[q] : x0[q], b = pv[q] ? x0[q] : x1[q];
                x0[q] = a;
                x1[q] = b - li[q] * a;
            }
        }
        // back substitution with U
        for (int i = m - 1; i >= 0; --i) {
            double* __restrict__ xi = &X[(size_t)i * k];
            const double* __restrict__ a0 = &u0[(size_t)i * k];
            const double* __restrict__ a1 = &u1[(size_t)i * k];
            const double* __restrict__ a2 = &u2[(size_t)i * k];
            if (i + 2 < m) {
                const double* __restrict__ x1 = xi + k;
                const double* __restrict__ x2 = xi + 2 * k;
                for (int q = 0; q < k; ++q) xi[q] = ((xi[q] - a1[q] * x1[q]) - a2[q] * x2[q]) / a0[q];
            } else if (i + 1 < m) {
                const double* __restrict__ x1 = xi + k;
                for (int q = 0; q < k; ++q) xi[q] = (xi[q] - a1[q] * x1[q]) / a0[q];
            } else {
                for (int q = 0; q < k; ++q) xi[q] = xi[q] / a0[q];
            }
        }
        for (int q = 0; q < k; ++q) nn[q] = 0.0;
        for (int i = 0; i < m; ++i)
            for (int q = 0; q < k; ++q) nn[q] += X[(size_t)i * k + q] * X[(size_t)i * k + q];
        for (int q = 0; q < k; ++q) nn[q] = 1.0 / std::sqrt(nn[q]);
        for (int i = 0; i < m; ++i)
            for (int q = 0; q < k; ++q) X[(size_t)i * k + q] *= nn[q];
    }
}

// top-k eigenpairs (descending) of the symmetric m x m matrix H
static void sym_topk(int m, std::vector<double> H, int k, std::vector<double>& evals, std::vector<double>& evecs) {
    Tridiag T;
    tridiagonalize(m, H, T);
    std::vector<double> ev = tridiag_eigvals(T.d, T.e);
    std::sort(ev.begin(), ev.end(), std::greater<double>());
    double tnorm = 0.0;
    for (int i = 0; i < m; ++i)
        tnorm = std::max(tnorm, std::fabs(T.d[i]) + (i ? std::fabs(T.e[i - 1]) : 0.0) + std::fabs(T.e[i]));
    evals.assign(ev.begin(), ev.begin() + k);
    // column q of an m x k row-major matrix: the k inverse iterations side
    // by side, Gram-Schmidt per vector, the reflectors applied to all k
    tridiag_invit(T, ev.data(), k, tnorm, evecs);
    std::vector<double> yq(m), yr(m);
    for (int q = 0; q < k; ++q) {
        for (int i = 0; i < m; ++i) yq[i] = evecs[(size_t)i * k + q];
        // two Gram-Schmidt passes against the previous vectors (clusters)
        for (int pass = 0; pass < 2; ++pass)
            for (int r = 0; r < q; ++r) {
                double dot = 0.0;
                for (int i = 0; i < m; ++i) dot += yq[i] * evecs[(size_t)i * k + r];
                for (int i = 0; i < m; ++i) yq[i] -= dot * evecs[(size_t)i * k + r];
            }
        double nn = 0.0;
        for (double v : yq) nn += v * v;
        nn = 1.0 / std::sqrt(nn);
        for (int i = 0; i < m; ++i) evecs[(size_t)i * k + q] = yq[i] * nn;
    }
    // back-transform: x = P_0 P_1 ... P_{m-3} y, every column at once (per
    // column the same dot and update order as one vector at a time)
    std::vector<double> dot(k);
    for (int kk = m - 3; kk >= 0; --kk) {
        if (T.beta[kk] == 0.0) continue;
        const double* __restrict__ v = &T.V[(size_t)kk * m];
        double* __restrict__ dq = dot.data();
        double* __restrict__ Yb = evecs.data();
        for (int q = 0; q < k; ++q) dq[q] = 0.0;
        for (int i = kk + 1; i < m; ++i) {
            const double vi = v[i];
            const double* __restrict__ yi = Yb + (size_t)i * k;
            for (int q = 0; q < k; ++q) dq[q] += vi * yi[q];
        }
        for (int q = 0; q < k; ++q) dq[q] *= T.beta[kk];
        for (int i = kk + 1; i < m; ++i) {
            const double vi = v[i];
            double* __restrict__ yi = Yb + (size_t)i * k;
            for (int q = 0; q < k; ++q) yi[q] -= dq[q] * vi;
        }
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

// PCA statistics of the last hh_comp_pca (hh_comp_pca_status)
struct PcaStatus {
    int converged = 0, products = 0, cycles = 0, method = 0;
    double residual[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // ||A x - theta x|| of the last checked Ritz vectors
    double bound = 0.0;                              // max_q ||r_q|| / gap_q (angle bound)
};

// k_ortho's grid barriers need every block of the grid resident at once.  A
// k_ortho block takes a CU's LDS (one block per CU), and up to
// GPU_MAX_HW_QUEUES kernels dispatch at the same time (one per hardware
// queue; the C5 line runs 12 streams): the grid is capped at
// CUs x blocks-per-CU / hardware queues, so every k_ortho grid that can be
// dispatching at once fits the chip together (other kernels' blocks finish
// and free their CUs; k_ortho grids never wait on each other).
struct OrthoAbort : Error {
    OrthoAbort() : Error(HH_ERR_HIP, "k_ortho: grid barrier timed out (blocks not co-resident)") {}
};
static int ortho_grid_cap(int tpb) {
    static std::mutex mu;
    static std::map<std::pair<int, int>, int> cache;  // (device, tpb) -> blocks
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    auto knob = [](int c) { return g_ortho_grid_cap > 0 ? std::max(1, std::min(c, g_ortho_grid_cap)) : c; };
    auto it = cache.find({dev, tpb});
    if (it != cache.end()) return knob(it->second);
    int cus = 0, occ = 0;
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    // the smallest co-residency over every k_ortho instance the solver
    // launches at this tpb (the modes differ in code and registers)
    auto occ_of = [](auto mode_c, auto tpb_c) {
        int o = 0;
        HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &o, (const void*)k_ortho<decltype(mode_c)::value, decltype(tpb_c)::value>, 256, 0));
        return o;
    };
    auto occ_all = [&](auto tpb_c) {
        return std::min({occ_of(std::integral_constant<int, kOrthoFull>{}, tpb_c),
                         occ_of(std::integral_constant<int, kOrthoFullLS>{}, tpb_c),
                         occ_of(std::integral_constant<int, kOrthoLast>{}, tpb_c),
                         occ_of(std::integral_constant<int, kOrthoStart>{}, tpb_c),
                         occ_of(std::integral_constant<int, kOrthoRitz>{}, tpb_c)});
    };
    occ = tpb == 1   ? occ_all(std::integral_constant<int, 1>{})
          : tpb == 2 ? occ_all(std::integral_constant<int, 2>{})
          : tpb == 4 ? occ_all(std::integral_constant<int, 4>{})
                     : occ_all(std::integral_constant<int, 8>{});
    int hwq = 4;  // HIP's default number of hardware queues per process
    if (const char* e = std::getenv("GPU_MAX_HW_QUEUES"))
        if (std::atoi(e) > 0) hwq = std::atoi(e);
    const int cap = std::max(1, std::min(std::max(1, occ) * std::max(1, cus) / hwq, kOrthoMaxBlocks));
    cache[{dev, tpb}] = cap;
    return knob(cap);
}

// Block Krylov PCA (see the K8 comment above).  Returns false when the
// method cannot run (basis larger than the matrix, start block rank
// deficient); the caller then falls back to subspace iteration.
static bool pca_krylov(PcaWork& wk, const double* cor, long long n, int k, double tol, int max_products, int P,
                       double* components, double* eigvals, PcaStatus& st, hipStream_t s, bool allow_coop = true) {
    constexpr int B = kSB, BB = kSB * kSB;
    if (P < 2 || (long long)(P + 1) * B > n) return false;
    const int nblk = (int)((n + kGramRows - 1) / kGramRows);
    const unsigned ge = (unsigned)((n * B + 255) / 256);
    const double eps = std::numeric_limits<double>::epsilon();
    const double shift_scale = 11.0 * ((double)n * B + (double)B * (B + 1)) * eps;
    DBuf<double> Q((size_t)P * n * B), W((size_t)n * B), T1((size_t)n * B), T2((size_t)n * B), X((size_t)n * B);
    const int nap = (int)((n + kApplyRows - 1) / kApplyRows);  // k_apply blocks
    DBuf<double> part((size_t)P * nblk * BB), gpart((size_t)nap * BB), gpart2((size_t)nap * BB),
        qpart((size_t)P * nap * BB);
    double* gcur = gpart.p;  // Gram partials of the last apply that made them
    double* galt = gpart2.p;
    // small outputs of one cycle, per block j: c1 [P], c2 [P], R x 6, G
    const int slot = (2 * P + 7) * BB;
    // + the restart block's R factors, then the Cholesky flags (ints: per
    // block j slots j * 8 + 0..5; restart P * 8 + 0..2; abort P * 8 + 7):
    // one download per cycle
    const int nfl = P * 8 + 8;
    DBuf<double> smalls((size_t)P * slot + 3 * BB + (nfl + 1) / 2);
    double* restartR = smalls.p + (size_t)P * slot;
    struct {
        int* p;
    } fail{reinterpret_cast<int*>(smalls.p + (size_t)P * slot + 3 * BB)};
    DBuf<double> Ydev((size_t)P * B * B);
    std::vector<double> hs((size_t)P * slot + 3 * BB + (nfl + 1) / 2);
    std::vector<int> hf(nfl);
    // host transfers through the thread's pinned staging buffers (slot 0
    // down, slot 1 up): pageable copies stalled the genome-wide correction
    // by ~20 ms each when issued to an idle GPU (profiles/r4gw)
    PinnedStage& pin = pinned_stage();
    auto download_smalls = [&]() {  // hs, hf <- the device (one copy), synchronised
        double* h = (double*)pin.get(0, hs.size() * sizeof(double));
        smalls.download(h, hs.size(), s);
        HIP_CHECK(hipStreamSynchronize(s));
        std::memcpy(hs.data(), h, hs.size() * sizeof(double));
        std::memcpy(hf.data(), hs.data() + (size_t)P * slot + 3 * BB, sizeof(int) * nfl);
    };
    auto gram = [&](const double* Xs, int nb, const double* Y, double* out) {
        hipLaunchKernelGGL(k_gram_mp, dim3((unsigned)nblk, (unsigned)nb), dim3(256), 0, s, Xs, nb, Y, n, nblk, part.p);
        hipLaunchKernelGGL(k_gram_ms, dim3((unsigned)(nb * BB)), dim3(64), 0, s, part.p, nblk, out);
    };
    auto apply = [&](const double* in, int nb, const double* Cm, const double* Ri, double* out, bool g, bool qg) {
        hipLaunchKernelGGL(k_apply_t<false>, dim3((unsigned)nap), dim3(256), 0, s, in, Q.p, nb, Cm, Ri, n, out,
                           g ? gcur : nullptr, qg ? qpart.p : nullptr, nap, nullptr, 0, 0.0, nullptr, nullptr);
    };
    // out = in R^{-1}, R = chol(the Gram of `in` from gcur (+ shift)), in one
    // launch; new Gram partials (g) go to the other buffer
    auto apply_chol = [&](const double* in, int nbq, double* out, bool g, bool qg, bool shifted, double* Rout,
                          int* fl) {
        hipLaunchKernelGGL(k_apply_t<true>, dim3((unsigned)nap), dim3(256), 0, s, in, Q.p, nbq, nullptr, nullptr, n,
                           out, g ? galt : nullptr, qg ? qpart.p : nullptr, nap, gcur, nap,
                           shifted ? shift_scale : 0.0, Rout, fl);
        if (g) std::swap(gcur, galt);
    };
    // shifted CholeskyQR3 of the block whose Gram partials are in gpart (its
    // rows in `in`): out = in R^{-1}, R factors to R3[0..2]; qg: the final
    // pass also leaves Q_k^T out partials in qpart (the next reduction)
    auto scholqr3 = [&](const double* in, double* out, double* R3, int* fl, int nbq) {
        const double* cur = in;
        // passes 0 and 1 shifted: a direction the Gram-Schmidt step left at
        // rounding level (a deflated Krylov direction) comes out of the two
        // shifted passes with kappa ~ 1e3-1e5 instead of 1e8, so the plain
        // third pass cannot break down (its noise direction is a valid new
        // basis vector; the outer second Gram-Schmidt pass re-orthogonalises it)
        for (int pass = 0; pass < 3; ++pass) {
            double* dst = pass == 2 ? out : (cur == T1.p ? T2.p : T1.p);
            apply_chol(cur, nbq, dst, pass < 2, pass == 2 && nbq > 0, pass < 2, R3 + pass * BB, fl + pass);
            cur = dst;
        }
    };
    auto qreduce = [&](int nb, double* out) {  // c = sum of the qpart partials
        hipLaunchKernelGGL(k_gram_ms, dim3((unsigned)(nb * BB)), dim3(64), 0, s, qpart.p, nap, out);
    };
    // one-launch orthogonalisation (k_ortho): a block owns 64 * tpb rows
    // (the fewest rows per block that fit the grid: more CUs pull the basis
    // rows; 128 instead of 256 rows took the serial k_ortho 163 -> 144 ms)
    int tpb = 8;
    if (g_ortho_tpb > 0 && nap <= g_ortho_tpb * ortho_grid_cap(g_ortho_tpb)) tpb = g_ortho_tpb;
    else
        for (int t : {g_ortho_min_tpb, 2, 4})
            if (t >= g_ortho_min_tpb && nap <= t * ortho_grid_cap(t)) { tpb = t; break; }
    const int oblk = (nap + tpb - 1) / tpb;
    const bool coop = allow_coop && g_pca_coop && oblk <= ortho_grid_cap(tpb);
    DBuf<double> orp(coop ? (size_t)oblk * kOrthoMaxE : 1), oro(kOrthoMaxE), ogp(coop ? (size_t)2 * oblk * BB : 1);
    DBuf<unsigned long long> octr(2);
    octr.zero(s);
    int opar = 0;
    int* abort_flag = fail.p + P * 8 + 7;
    DBuf<long long> tst(g_pca_debug >= 2 ? 48 : 1);
    auto ortho = [&](int mode, OrthoArgs a, int nbar) {
        a.Q = Q.p;
        a.rpart = orp.p;
        a.rout = oro.p;
        a.gpart = ogp.p;
        a.ctr = octr.p;
        a.par = opar;
        a.abort = abort_flag;
        a.n = n;
        a.nblk = oblk;
        a.shift_scale = shift_scale;
        a.tstamp = g_pca_debug >= 2 ? tst.p : nullptr;
        a.pre = ortho_pre_level();
        HH_REQUIRE(a.nb >= 0 && a.nb <= 8 && oblk >= 1 && oblk <= kOrthoMaxBlocks, "k_ortho shape");
        const dim3 grid((unsigned)oblk), blk(256);
        HH_KTIME("k_ortho", s);  // bench.py's C5 line: the dominant kernel by time
#define HH_ORTHO(M)                                                  \
    do {                                                             \
        if (tpb == 1) hipLaunchKernelGGL((k_ortho<M, 1>), grid, blk, 0, s, a); \
        else if (tpb == 2) hipLaunchKernelGGL((k_ortho<M, 2>), grid, blk, 0, s, a); \
        else if (tpb == 4) hipLaunchKernelGGL((k_ortho<M, 4>), grid, blk, 0, s, a); \
        else hipLaunchKernelGGL((k_ortho<M, 8>), grid, blk, 0, s, a);          \
    } while (0)
        switch (mode) {
            case kOrthoFull:
                // low-synch CGS2 (two reductions per product; hh_tune "ortho_lowsync" 0: round 3's ~8)
                if (g_ortho_lowsync) HH_ORTHO(kOrthoFullLS);
                else HH_ORTHO(kOrthoFull);
                break;
            case kOrthoLast: HH_ORTHO(kOrthoLast); break;
            case kOrthoStart: HH_ORTHO(kOrthoStart); break;
            default: HH_ORTHO(kOrthoRitz); break;
        }
#undef HH_ORTHO
        HIP_CHECK(hipGetLastError());
        opar ^= 1;
        if (a.tstamp) {
            long long h[48];
            tst.download(h, 48, s);
            HIP_CHECK(hipStreamSynchronize(s));
            fprintf(stderr, "[ortho] mode=%d nb=%d nblk=%d tpb=%d us:", mode, a.nb, oblk, tpb);
            const int nb_ = (int)h[38];
            h[2 * nb_ + 1] = h[39];
            for (int q = 1; q <= 2 * nb_ + 1; ++q) fprintf(stderr, " %.1f", (h[q] - h[q - 1]) / 100.0);
            fprintf(stderr, " | barriers %d total %.1f | pass: gram %.1f sync %.1f reduce %.1f chol %.1f apply %.1f\n",
                    nb_, (h[39] - h[0]) / 100.0, (h[41] - h[40]) / 100.0, (h[42] - h[41]) / 100.0,
                    (h[43] - h[42]) / 100.0, (h[44] - h[43]) / 100.0, (h[45] - h[44]) / 100.0);
            if (mode == kOrthoFull && g_ortho_lowsync)
                for (int so : {20, 28})
                    fprintf(stderr, "[ortho-ls] nb=%d pass=%d us: proj %.2f gram+reduce %.2f pyth %.2f mulq %.2f chol %.2f apply %.2f\n",
                            a.nb, so == 28, (h[so + 1] - h[so]) / 100.0, (h[so + 2] - h[so + 1]) / 100.0,
                            (h[so + 3] - h[so + 2]) / 100.0, (h[so + 4] - h[so + 3]) / 100.0,
                            (h[so + 5] - h[so + 4]) / 100.0, (h[so + 6] - h[so + 5]) / 100.0);
        }
    };
    auto check_abort = [&](const std::vector<int>& flags) {
        // the caller redoes the whole solve on the multi-launch path
        if (coop && (flags[P * 8 + 7] || g_ortho_abort_test)) throw OrthoAbort();
    };
    HIP_CHECK(hipMemsetAsync(fail.p, 0, sizeof(int) * nfl, s));
    // hh_tune("ortho_abort_test", 2): the abort flag raised before the first
    // k_ortho launch, so every block leaves its grid barriers early and the
    // workspace is left partly written -- the fallback must recover from that
    if (coop && g_ortho_abort_test == 2) HIP_CHECK(hipMemsetAsync(abort_flag, 1, 1, s));
    // start block: [1 / sqrt(n) | deterministic pseudo-random columns]; the
    // host source of the upload lives until the first cycle's synchronise
    std::vector<double> v0((size_t)n * B);
    {
        for (long long i = 0; i < n; ++i)
            for (int b = 0; b < B; ++b)
                v0[i * B + b] = b == 0 ? 1.0 / std::sqrt((double)n) : (double)u01(mix64(0x5eedULL + i * B + b)) - 0.5;
        double* h = (double*)pin.get(1, v0.size() * sizeof(double));
        std::memcpy(h, v0.data(), v0.size() * sizeof(double));
        X.upload(h, v0.size(), s);
        if (coop) {
            OrthoArgs a;
            a.xin = X.p;
            a.qnext = Q.p;
            a.R = restartR;
            a.fail = fail.p + P * 8;
            ortho(kOrthoStart, a, 3);
        } else {
            apply(X.p, 0, nullptr, nullptr, W.p, true, false);
            scholqr3(W.p, Q.p, restartR, fail.p + P * 8, 0);
        }
    }
    std::vector<double> cur((size_t)n * k), Xh((size_t)n * B);
    // Ritz coefficients: their upload's host source lives until the next
    // cycle's synchronise
    std::vector<double> ev, Y;
    double last_bound = 1e300;
    int products = 0, cycles = 0;
    bool done = false;
    while (!done && products + P <= max_products) {
        int pe = P;  // blocks of this cycle's basis
        if (!coop) HIP_CHECK(hipMemsetAsync(fail.p, 0, sizeof(int) * P * 8, s));  // k_ortho writes every flag
        for (int j = 0; j < P; ++j) {
            double* sl = smalls.p + (size_t)j * slot;
            double *c1 = sl, *c2 = sl + (size_t)P * BB, *R = sl + (size_t)2 * P * BB, *G = sl + (size_t)(2 * P + 6) * BB;
            double* Qj = Q.p + (size_t)j * n * B;
            ++products;
            const int nb = j + 1;
            if (coop) {
                // W = Cor Q_j (split-K MFMA + its fixed-order sum: a block
                // of k_ortho summing the splits itself was slower -- 32 CUs
                // pulling 8 MB have too few bytes in flight)
                wk.cor_mul(cor, Qj, nullptr, false, W.p, s);
                OrthoArgs a;
                a.xin = W.p;
                a.nb = nb;
                a.c1 = c1;
                a.c2 = c2;
                if (j < P - 1) {
                    a.qnext = Q.p + (size_t)(j + 1) * n * B;
                    a.R = R;
                    a.fail = fail.p + j * 8;
                    ortho(kOrthoFull, a, 10);
                } else {
                    a.G = G;
                    ortho(kOrthoLast, a, 5);
                }
                continue;
            }
            wk.cor_mul(cor, Qj, nullptr, false, W.p, s);
            if (j < P - 1) {
                // pass A: W1 = W - Qa c1 = Q1 RA;  pass B: W2 = Q1 - Qa c2 = Q_{j+1} RB
                gram(Q.p, nb, W.p, c1);
                apply(W.p, nb, c1, nullptr, X.p, true, false);
                scholqr3(X.p, W.p, R, fail.p + j * 8, nb);      // Q1 -> W, Qa^T Q1 partials
                qreduce(nb, c2);
                apply(W.p, nb, c2, nullptr, X.p, true, false);
                scholqr3(X.p, Q.p + (size_t)(j + 1) * n * B, R + 3 * BB, fail.p + j * 8 + 3, 0);
            } else {
                // last product: CGS2 coefficients + Gram of the residual
                gram(Q.p, nb, W.p, c1);
                apply(W.p, nb, c1, nullptr, X.p, false, true);
                qreduce(nb, c2);
                apply(X.p, nb, c2, nullptr, W.p, true, false);
                hipLaunchKernelGGL(k_gram_ms, dim3((unsigned)BB), dim3(64), 0, s, gcur, nap, G);
            }
        }
        const auto c0 = std::chrono::steady_clock::now();
        download_smalls();
        const auto c1 = std::chrono::steady_clock::now();
        const double t_w = std::chrono::duration<double, std::milli>(c1 - c0).count();
        check_abort(hf);
        if (hf[P * 8] || hf[P * 8 + 1] || hf[P * 8 + 2]) return false;  // start block rank deficient
        for (int j = 0; j + 1 < P; ++j) {
            bool bad = false;
            for (int q = 0; q < 6; ++q) bad |= hf[j * 8 + q] != 0;
            if (bad) { pe = j + 1; break; }
        }
        if (pe < 2) return false;  // deflated at the first expansion
        // T (m + B) x m, column block j = [c_j (rows 0 .. (j+1)B); R_j (next B rows)]
        const int m = pe * B;
        // St = S^T (m x (m + B)): row a = coordinates of column a of Xc Q
        const int ldS = m + B;
        std::vector<double> St((size_t)m * ldS, 0.0);
        std::vector<int> slen(m, 0);  // nonzero rows of column a
        auto mm16 = [&](const double* A, const double* Bm, double* C) {  // C = A Bm (16 x 16)
            for (int a = 0; a < B; ++a)
                for (int b = 0; b < B; ++b) {
                    double acc = 0.0;
                    for (int q = 0; q < B; ++q) acc += A[a * B + q] * Bm[q * B + b];
                    C[a * B + b] = acc;
                }
        };
        std::vector<double> RA(BB), RB(BB), tmp(BB), tmp2(BB);
        std::vector<double> extraG;  // Gram of the residual block (last block)
        int last = -1;
        for (int j = 0; j < pe; ++j) {
            const double* sl = hs.data() + (size_t)j * slot;
            const double *c1 = sl, *c2 = sl + (size_t)P * BB, *R = sl + (size_t)2 * P * BB,
                         *G = sl + (size_t)(2 * P + 6) * BB;
            const int nb = j + 1;
            const bool is_last = (j == P - 1);
            if (!is_last && j == pe - 1) {
                // deflated next block: cycle ends here, ignore this product
                break;
            }
            if (!is_last) {
                mm16(R + BB, R, tmp.data());        // R2 R1
                mm16(R + 2 * BB, tmp.data(), RA.data());  // R3 R2 R1
                mm16(R + 4 * BB, R + 3 * BB, tmp.data());
                mm16(R + 5 * BB, tmp.data(), RB.data());
                // coef = c1 + c2 RA ; R_j = RB RA
                for (int r = 0; r < nb * B; ++r)
                    for (int b = 0; b < B; ++b) {
                        double acc = c1[r * B + b];
                        for (int q = 0; q < B; ++q) acc += c2[r * B + q] * RA[q * B + b];
                        St[(size_t)(j * B + b) * ldS + r] = acc;
                    }
                mm16(RB.data(), RA.data(), tmp2.data());
                for (int a = 0; a < B; ++a)
                    for (int b = 0; b < B; ++b) St[(size_t)(j * B + b) * ldS + (j + 1) * B + a] = tmp2[a * B + b];
                for (int b = 0; b < B; ++b) slen[j * B + b] = (j + 2) * B;
                last = j;
            } else {
                for (int r = 0; r < nb * B; ++r)
                    for (int b = 0; b < B; ++b) St[(size_t)(j * B + b) * ldS + r] = c1[r * B + b] + c2[r * B + b];
                for (int b = 0; b < B; ++b) slen[j * B + b] = (j + 1) * B;
                extraG.assign(G, G + BB);
                last = j;
            }
        }
        const int mb = (last + 1) * B;  // basis columns used by Rayleigh-Ritz
        // Xc Q = Q_+ S with row 0 (the 1/sqrt(n) coordinate) removed
        for (int c = 0; c < m; ++c) St[(size_t)c * ldS] = 0.0;
        std::vector<double> H((size_t)mb * mb, 0.0);
        // four columns b at a time: four independent dot chains in flight,
        // each summed over r in order as one column alone
        for (int a = 0; a < mb; ++a) {
            const double* __restrict__ sa = &St[(size_t)a * ldS];
            int b = a;
            for (; b + 4 <= mb; b += 4) {
                const double* __restrict__ s0 = &St[(size_t)b * ldS];
                const double* __restrict__ s1 = s0 + ldS;
                const double* __restrict__ s2 = s1 + ldS;
                const double* __restrict__ s3 = s2 + ldS;
                const int L0 = std::min(slen[a], slen[b]), L1 = std::min(slen[a], slen[b + 1]),
                          L2 = std::min(slen[a], slen[b + 2]), L3 = std::min(slen[a], slen[b + 3]);
                const int Lc = std::min(std::min(L0, L1), std::min(L2, L3));
                double c0 = 0.0, c1 = 0.0, c2 = 0.0, c3 = 0.0;
                int r = 0;
                for (; r < Lc; ++r) {
                    const double x = sa[r];
                    c0 += x * s0[r];
                    c1 += x * s1[r];
                    c2 += x * s2[r];
                    c3 += x * s3[r];
                }
                for (int q = r; q < L0; ++q) c0 += sa[q] * s0[q];
                for (int q = r; q < L1; ++q) c1 += sa[q] * s1[q];
                for (int q = r; q < L2; ++q) c2 += sa[q] * s2[q];
                for (int q = r; q < L3; ++q) c3 += sa[q] * s3[q];
                H[(size_t)a * mb + b] = H[(size_t)b * mb + a] = c0;
                H[(size_t)a * mb + b + 1] = H[(size_t)(b + 1) * mb + a] = c1;
                H[(size_t)a * mb + b + 2] = H[(size_t)(b + 2) * mb + a] = c2;
                H[(size_t)a * mb + b + 3] = H[(size_t)(b + 3) * mb + a] = c3;
            }
            for (; b < mb; ++b) {
                const double* sb = &St[(size_t)b * ldS];
                const int L = std::min(slen[a], slen[b]);
                double acc = 0.0;
                for (int r = 0; r < L; ++r) acc += sa[r] * sb[r];
                H[(size_t)a * mb + b] = H[(size_t)b * mb + a] = acc;
            }
        }
        if (!extraG.empty()) {
            const int o = last * B;
            for (int a = 0; a < B; ++a)
                for (int b = 0; b < B; ++b) H[(size_t)(o + a) * mb + o + b] += 0.5 * (extraG[a * B + b] + extraG[b * B + a]);
        }
        const auto c2 = std::chrono::steady_clock::now();
        sym_topk(mb, H, B, ev, Y);
        const auto c3 = std::chrono::steady_clock::now();
        const double t_h = std::chrono::duration<double, std::milli>(c2 - c1).count();
        const double t_e = std::chrono::duration<double, std::milli>(c3 - c2).count();
        // Ritz vectors X = Qa Y (top B), uploaded as nb stacked 16 x 16 blocks
        {
            // (slot 1's previous upload completed: download_smalls synchronised since)
            double* h = (double*)pin.get(1, (size_t)mb * B * sizeof(double));
            std::memcpy(h, Y.data(), (size_t)mb * B * sizeof(double));
            Ydev.upload(h, (size_t)mb * B, s);
        }
        ++cycles;
        if (eigvals)
            for (int q = 0; q < k; ++q) eigvals[q] = ev[q];
        // Convergence from residuals of the PREVIOUS cycle's Ritz vectors:
        // they are columns 1..k of this cycle's start block, x_q = Q_0 (R e_{q+1})
        // (R = the restart's CholQR factors), and A x_q lies in span(Q_0, Q_1, Q_2)
        // (A = Cor P Cor), so r_q = A x_q - theta x_q = Q (H e - theta e) exactly:
        // ||r_q|| with no cancellation, and sin(x_q, v_q) <= ||r_q|| / gap_q.
        // Done when that bound is < tol for every q < k, or when it has
        // stopped shrinking (< 2x per cycle) below 1e3 tol: the rounding floor
        // of the products (a degenerate gap never gets there: not converged).
        if (cycles > 1 && last >= 2) {
            const double* Rr = hs.data() + (size_t)P * slot;
            std::vector<double> tmpR(BB), Rt(BB);
            mm16(Rr + BB, Rr, tmpR.data());
            mm16(Rr + 2 * BB, tmpR.data(), Rt.data());
            double bound = 0.0;
            for (int q = 0; q < k; ++q) {
                std::vector<double> e(mb, 0.0), He(mb, 0.0);
                for (int a = 0; a < B; ++a) e[a] = Rt[a * B + q + 1];
                for (int a = 0; a < mb; ++a) {
                    double acc = 0.0;
                    for (int c = 0; c < B; ++c) acc += H[(size_t)a * mb + c] * e[c];
                    He[a] = acc;
                }
                double ee = 0.0, eHe = 0.0;
                for (int a = 0; a < mb; ++a) { ee += e[a] * e[a]; eHe += e[a] * He[a]; }
                const double theta = eHe / ee;
                double rr = 0.0;
                for (int a = 0; a < mb; ++a) rr += (He[a] - theta * e[a]) * (He[a] - theta * e[a]);
                const double res = std::sqrt(rr / ee);
                double gap = std::fabs(ev[q] - ev[q + 1]);
                if (q > 0) gap = std::min(gap, std::fabs(ev[q - 1] - ev[q]));
                bound = std::max(bound, gap > 0 ? res / gap : 1e300);
                st.residual[q] = res;
            }
            st.bound = bound;
            if (g_pca_debug)
                fprintf(stderr, "[pca] n=%lld cycle=%d products=%d pe=%d bound=%.3e res=%.3e %.3e %.3e ev=%.6g %.6g %.6g %.6g"
                        " host_ms H=%.3f eig=%.3f gpu_wait_ms=%.3f\n",
                        n, cycles, products, pe, bound, st.residual[0], st.residual[1], st.residual[2], ev[0], ev[1],
                        ev[2], ev[3], t_h, t_e, t_w);
            // this cycle's vectors are better than the checked ones by about
            // the last contraction factor: stop when the predicted bound is met
            const double predicted = last_bound < 1e300 ? bound * std::min(1.0, bound / last_bound) : bound;
            if (predicted < tol || (bound < 1e3 * tol && bound > 0.5 * last_bound)) {
                done = true;
                st.converged = 1;
            }
            last_bound = bound;
        }
        // Ritz vectors out (and, not done, the next cycle's start block Q_0
        // from them: one k_ortho launch)
        if (coop && !done) {
            OrthoArgs a;
            a.Y = Ydev.p;
            a.nb = last + 1;
            a.xout = X.p;
            a.qnext = Q.p;
            a.R = restartR;
            a.fail = fail.p + P * 8;
            ortho(kOrthoRitz, a, 3);
        } else {
            hipLaunchKernelGGL(k_comb_mp, dim3(ge), dim3(256), 0, s, nullptr, Q.p, last + 1, Ydev.p, n, X.p);
        }
        // (the Ritz vectors stay on the device until the loop ends: no
        // download and no synchronise per cycle)
        if (!done && !coop) {
            hipLaunchKernelGGL(k_start_block, dim3(ge), dim3(256), 0, s, X.p, n, T2.p);
            HIP_CHECK(hipMemsetAsync(fail.p + P * 8, 0, sizeof(int) * 8, s));
            apply(T2.p, 0, nullptr, nullptr, W.p, true, false);
            scholqr3(W.p, Q.p, restartR, fail.p + P * 8, 0);
        }
    }
    // a budget-exhausted run leaves a restart block enqueued: drain the
    // stream before this function's buffers go back to the pool
    download_smalls();
    check_abort(hf);
    if (cycles > 0) {  // the last cycle's Ritz vectors
        double* h = (double*)pin.get(0, Xh.size() * sizeof(double));
        X.download(h, Xh.size(), s);
        HIP_CHECK(hipStreamSynchronize(s));
        std::memcpy(Xh.data(), h, Xh.size() * sizeof(double));
        for (int q = 0; q < k; ++q) {
            double nn = 0.0;
            for (long long i = 0; i < n; ++i) nn += Xh[i * B + q] * Xh[i * B + q];
            const double inv = 1.0 / std::sqrt(nn);
            for (long long i = 0; i < n; ++i) cur[q * n + i] = Xh[i * B + q] * inv;
        }
    }
    if (!done) st.converged = 0;
    st.products = products;
    st.cycles = cycles;
    st.method = 1;
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

int hh_comp_sliding_oe(hh_comp* c, const double* decline, int32_t step, void* stream) {
    return guard([&] {
        HH_REQUIRE(c, "null");
        if (!decline) {  // back to the plain O/E
            c->sa_on = 0;
            c->sa.release();
            return;
        }
        const long long N = c->N;
        // step 0 reads d[N] / d[N + 1] in the reference (IndexError there)
        HH_REQUIRE(step >= 1, "Sliding_Approach needs step = window // Res // 2 >= 1");
        hipStream_t s = as_stream(stream);
        DBuf<double> dec(N), Hs((size_t)N * N);
        dec.upload(decline, N, s);
        c->sa.alloc((size_t)N * N);
        const unsigned g = (unsigned)((N * N + 255) / 256);
        hipLaunchKernelGGL(k_sa_hsum, dim3(g), dim3(256), 0, s, c->Mp, N, (int)step, Hs.p);
        hipLaunchKernelGGL(k_sa_oe, dim3(g), dim3(256), 0, s, c->Mp, Hs.p, dec.p, N, (int)step, c->sa.p);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipStreamSynchronize(s));
        c->sa_on = 1;
    });
}

int hh_comp_get_sliding_oe(hh_comp* c, double* oe, void* stream) {
    return guard([&] {
        HH_REQUIRE(c && oe && c->sa_on, "no Sliding_Approach O/E computed");
        hipStream_t s = as_stream(stream);
        c->sa.download(oe, (size_t)c->N * c->N, s);
        HIP_CHECK(hipStreamSynchronize(s));
    });
}

// K splits for the Cov triangle, by a cost model in units of one round of
// full-K tiles on the 2-blocks-per-CU slots: ceil(tiles s / slots) / s for the
// split launch plus the reduction pass, which streams (s + 2) partial-tile
// sizes per tile (128 KB each at ~4 TB/s, against a round of ~0.23 us x K on
// fp64 MFMA): ~0.14 (s + 2) tiles / K.  Splits <= 8, >= 256 K rows each.  The
// triangle's last round is what it buys back: chr21 at 25 kb has 105 tiles
// for 512 slots (s = 4), chr1 2701 (5.3 rounds -> s = 2, 5.5 + 0.15).
static int syrk_splits(long long ntile, long long Kpad) {
    if (g_syrk_split > 0) return (int)std::min<long long>(g_syrk_split, std::max<long long>(1, Kpad / 16));
    if (g_syrk_split == 0) return 1;
    int dev = 0, n_cu = 256;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    const long long slots = 2LL * n_cu;
    int best = 1;
    double best_t = (double)((ntile + slots - 1) / slots);
    for (int k = 2; k <= 8 && Kpad / k >= 256; ++k) {
        const double t = (double)((ntile * k + slots - 1) / slots) / k + 0.14 * (k + 2) * ntile / (double)Kpad;
        if (t < 0.97 * best_t) {
            best_t = t;
            best = k;
        }
    }
    return best;
}

int hh_comp_correlation(hh_comp* c, const double* decline, const int64_t* ng, int64_t n, void* stream) {
    return guard([&] {
        HH_REQUIRE(c && decline && ng && n > 0 && n <= c->N, "bad arguments");
        hipStream_t s = as_stream(stream);
        const long long N = c->N;
        c->n = n;
        c->ld = (n + kSyT - 1) / kSyT * kSyT;  // whole k_syrk tiles (a multiple of 64 for the other kernels)
        c->dec.alloc(N);
        if (c->sa_on) {  // the O/E is already materialised: oe_value(sa, 1) = sa
            std::vector<double> ones(N, 1.0);
            c->dec.upload(ones.data(), N, s);
            HIP_CHECK(hipStreamSynchronize(s));
        } else {
            c->dec.upload(decline, N, s);
        }
        const double* Msrc = c->sa_on ? c->sa.p : c->Mp;
        c->ng.alloc(n);
        c->ng.upload(reinterpret_cast<const long long*>(ng), n, s);
        // column means of O/E
        const int rpc = 256;
        const int chunks = (int)((N + rpc - 1) / rpc);
        DBuf<double> part((size_t)chunks * n), mu(n);
        hipLaunchKernelGGL(k_oe_colsum, dim3((unsigned)((n + 255) / 256), (unsigned)chunks), dim3(256), 0, s, Msrc,
                           c->dec.p, c->ng.p, N, (long long)n, rpc, part.p);
        hipLaunchKernelGGL(k_oe_mean, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, part.p, (long long)n, chunks,
                           N, mu.p);
        // centred O/E, padded
        const long long Npad = (N + 15) / 16 * 16;
        DBuf<double> Z((size_t)Npad * c->ld);
        hipLaunchKernelGGL(k_oe_center, dim3((unsigned)((c->ld + 255) / 256), (unsigned)std::min<long long>(Npad, 65535)),
                           dim3(256), 0, s, Msrc, c->dec.p,
                           c->ng.p, mu.p, N, (long long)n, Npad, c->ld, Z.p);
        // Cov = Z^T Z * (1 / (N - 1))  (np.cov: c *= true_divide(1, fact))
        DBuf<double> cov((size_t)c->ld * c->ld);
        const long long nt = c->ld / kSyT, ntile = nt * (nt + 1) / 2;
        const int ns = syrk_splits(ntile, Npad);
        const long long kc = (Npad / 16 + ns - 1) / ns * 16;
        const double scale = 1.0 / (double)(N - 1);
        // (P and Z stay allocated until the stream is synchronised below: a
        // pooled block released earlier could be handed to another thread's
        // stream while these kernels still use it)
        DBuf<double> P(ns > 1 ? (size_t)ns * ntile * kSyTile : 0);
        {
            HH_KTIME("k_syrk", s);  // (split K: the reduction is inside the timed span)
            if (ns == 1) {
                hipLaunchKernelGGL(k_syrk<false>, dim3((unsigned)ntile),
                                   dim3(256), 0, s, Z.p, c->ld, Npad, nt, Npad, scale, cov.p, c->ld, nullptr);
            } else {
                hipLaunchKernelGGL(k_syrk<true>, dim3((unsigned)(ns * ntile)),
                                   dim3(256), 0, s, Z.p, c->ld, Npad, nt, kc, scale, nullptr, c->ld, P.p);
                hipLaunchKernelGGL(k_syrk_reduce, dim3((unsigned)((ntile * kSyTile + 255) / 256)), dim3(256), 0, s,
                                   P.p, ns, nt, scale, cov.p, c->ld);
            }
        }
        c->cor.alloc((size_t)c->ld * c->ld);
        DBuf<double> sd(n);
        hipLaunchKernelGGL(k_cor_sd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, cov.p, (long long)n, c->ld,
                           sd.p);
        hipLaunchKernelGGL(k_corr_norm_oop, dim3((unsigned)((c->ld / 4 + 255) / 256), (unsigned)std::min<long long>(c->ld, 65535)),
                           dim3(256), 0, s, cov.p, sd.p, (long long)n, c->ld, c->cor.p);
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
        if (g_pca_method == 1) {
            PcaStatus st;
            bool ok = false, fell_back = false;
            try {
                ok = pca_krylov(wk, c->cor.p, n, k, tol, 2 * max_iters, g_pca_p, components, eigvals, st, s);
            } catch (const OrthoAbort&) {
                // k_ortho's grid could not become co-resident (its bounded
                // barrier wait gave up): the same solve on the multi-launch
                // orthogonalisation, no grid barriers
                c->ortho_fallbacks += 1;
                fell_back = true;
                st = PcaStatus{};
                ok = pca_krylov(wk, c->cor.p, n, k, tol, 2 * max_iters, g_pca_p, components, eigvals, st, s, false);
            }
            if (ok) {
                c->iters = st.products;
                c->pca_converged = st.converged;
                c->pca_products = st.products;
                c->pca_cycles = st.cycles;
                c->pca_method = fell_back ? 2 : 1;
                if (iters_out) *iters_out = st.products;
                return;
            }
        }
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
        c->pca_converged = done ? 1 : 0;
        c->pca_products = 2 * c->iters + 1;
        c->pca_cycles = c->iters;
        c->pca_method = 0;
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

int hh_sym_topk(const double* H, int32_t m, int32_t k, double* evals, double* evecs) {
    return guard([&] {
        HH_REQUIRE(H && evals && evecs && m >= 1 && k >= 1 && k <= m, "bad arguments");
        std::vector<double> A(H, H + (size_t)m * m), ev, Y;
        if (m == 1) {
            evals[0] = A[0];
            evecs[0] = 1.0;
            return;
        }
        sym_topk(m, A, k, ev, Y);
        std::copy(ev.begin(), ev.end(), evals);
        std::copy(Y.begin(), Y.end(), evecs);
    });
}

int hh_comp_pca_status(const hh_comp* c, int32_t* converged, int32_t* products, int32_t* cycles, int32_t* method) {
    return guard([&] {
        HH_REQUIRE(c, "null");
        if (converged) *converged = c->pca_converged;
        if (products) *products = c->pca_products;
        if (cycles) *cycles = c->pca_cycles;
        if (method) *method = c->pca_method;
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
            const double* Msrc = c->sa_on ? c->sa.p : c->Mp;
            hipLaunchKernelGGL(k_select_stats, dim3((unsigned)n), dim3(256), 0, s, c->cor.p, c->ld, n, Msrc, c->N,
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
