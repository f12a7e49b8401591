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
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <type_traits>
#include <vector>

#include "ice_internal.hpp"  // hh_common.hpp + dev_excl_scan_i64

namespace hh {

constexpr int kT = 64;  // dense tile edge

// lane `l`'s double (wave-uniform l)
__device__ __forceinline__ double readlane_dbl(double v, int l) {
    const unsigned long long u = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l), hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// x16 (integer T only, may be null): the row copied as uint16, a count >=
// 0xFFFF stored as 0xFFFF (the passes that read the copy take such entries
// from X itself); *ovf set when a value does not fit 32 bits (the later
// passes then read X throughout)
template <class T>
__device__ __forceinline__ void rowstats_row(const T* __restrict__ X, long long N, long long i,
                                             const long long* __restrict__ lo, const long long* __restrict__ hi,
                                             double* __restrict__ sum, long long* __restrict__ zeros,
                                             uint16_t* __restrict__ x16 = nullptr, int* __restrict__ ovf = nullptr) {
    __shared__ double shd[16];
    __shared__ long long shz[16];
    const long long a = lo ? lo[i] : 0, b = hi ? hi[i] : N;
    const T* row = X + i * N;
    long long zc = 0;
    double sd = 0.0;
    long long si = 0;
    bool bad = false;
    auto take = [&](T v, long long j) __attribute__((always_inline)) {
        zc += v == T(0);
        if constexpr (std::is_integral_v<T>) {
            si += (long long)v;  // integer: exact
            if (x16) {
                bad |= (unsigned long long)v > 0xFFFFFFFFull;  // (negative: huge as unsigned)
                x16[i * N + j] = (uint16_t)((unsigned long long)v < 0xFFFFull ? v : 0xFFFF);
            }
        } else {
            sd += (double)v;
        }
    };
    // four loads in flight per thread (each thread still takes its elements
    // in ascending j: the same double sum)
    long long j = a + threadIdx.x;
    for (; j + 3 * 256 < b; j += 4 * 256) {
        const T v0 = row[j], v1 = row[j + 256], v2 = row[j + 512], v3 = row[j + 768];
        take(v0, j);
        take(v1, j + 256);
        take(v2, j + 512);
        take(v3, j + 768);
    }
    for (; j < b; j += 256) take(row[j], j);
    if (x16 && __ballot(bad) != 0ull && (threadIdx.x & 63) == 0) atomicOr(ovf, 1);
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

template <class T>
__global__ __launch_bounds__(256) void k_rowstats(const T* __restrict__ X, long long N,
                                                  const long long* __restrict__ lo,
                                                  const long long* __restrict__ hi, double* __restrict__ sum,
                                                  long long* __restrict__ zeros) {
    rowstats_row<T>(X, N, blockIdx.x, lo, hi, sum, zeros);
}

// The row statistics of many int64 matrices in one launch (hh_twostep_batch):
// matrix m's rows are blocks [row0[m], row0[m + 1])
struct RsDesc {
    const long long* X;
    long long N;
    double* sum;
    long long* zeros;
    uint16_t* x16;  // null: no copy
    int* ovf;
};
__global__ __launch_bounds__(256) void k_rowstats_b(const RsDesc* __restrict__ d, const long long* __restrict__ row0,
                                                    int nd) {
    const long long b = blockIdx.x;
    int lo = 0, hi = nd - 1;  // the last m with row0[m] <= b
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (row0[mid] <= b) lo = mid; else hi = mid - 1;
    }
    const RsDesc m = d[lo];
    rowstats_row<long long>(m.X, m.N, b - row0[lo], nullptr, nullptr, m.sum, m.zeros, m.x16, m.ovf);
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
    const double* scale_p = nullptr;  // pass 3: the same from device memory (no host round trip)
    const long long* ng_p = nullptr;  // streaming passes: the gap count on the device (gap form iff > 0)
};

// Per-tile vectors staged once in LDS: alpha, gap flag and s for the 64
// rows of I and of J (sentinel values past N).
struct TileVecs {
    double aI[kT], aJ[kT], sI[kT], sJ[kT];
    uint8_t gI[kT], gJ[kT];
};

// Loads S tile (I,J) as st[r][c] = S[I0+r][J0+c] and the transposed tile as
// stT[r][c] = S[J0+c][I0+r]; a wave reads one 512-B row per instruction.
template <class T>
__device__ __forceinline__ void load_pair(const T* __restrict__ X, long long N, long long I0, long long J0,
                                          const TileVecs& tv, double (*st)[kT + 1], double (*stT)[kT + 1]) {
    const int c = threadIdx.x & (kT - 1), r0 = threadIdx.x >> 6;
    // all 32 loads issued before the first use (memory-level parallelism:
    // only 2 blocks fit a CU with 66 KB of LDS each)
    T v[kT / 4], w[kT / 4];
#pragma unroll
    for (int k = 0; k < kT / 4; ++k) {
        const int r = r0 + 4 * k;
        const long long gi = I0 + r, gj = J0 + c, ti = J0 + r, tj = I0 + c;
        // unconditional loads from clamped addresses (a guarded load becomes
        // a branch with its own vmcnt(0) wait)
        const bool okv = gi < N && gj < N, okw = ti < N && tj < N;
        const T xv = X[okv ? gi * N + gj : 0], xw = X[okw ? ti * N + tj : 0];
        v[k] = okv ? xv : T(0);
        w[k] = okw ? xw : T(0);
    }
#pragma unroll
    for (int k = 0; k < kT / 4; ++k) {
        const int r = r0 + 4 * k;
        st[r][c] = (double)v[k] / tv.aI[r];  // S = X / alpha[:, None] (true division)
        stT[c][r] = (double)w[k] / tv.aJ[r];
    }
}

// Trans2symmetry element (i != j); d: on the diagonal
__device__ __forceinline__ double sym_value(bool d, bool has_gap, bool gi, bool gj, double sij, double sji) {
    if (d) return sij;
    if (!has_gap) return sij + sji;
    if (gi && gj) return sij > sji ? sij : sji;  // np.maximum-like on non-NaN
    return (sij + sji) / 2.0;
}

// PASS 1: partial row sums of Y.  part[pair][0..63] rows of I, [64..127] rows of J.
// PASS 2: partial sum of C over tile (I,J) (+ mirrored (J,I) when I != J).
// PASS 3: write out = scale * C for tiles (I,J) and (J,I).
// Thread t: row r = t >> 2 and columns c = q + 4k (q = t & 3) for the
// per-row work of passes 1-2; passes 1's column sums use the same split
// transposed; pass 3 writes whole rows per wave.
template <class T, int PASS>
__global__ __launch_bounds__(256) void k_symvc(const T* __restrict__ X, SymArgs a, double* __restrict__ part,
                                               double* __restrict__ out) {
    __shared__ double st[kT][kT + 1];
    __shared__ double stT[kT][kT + 1];
    __shared__ TileVecs tv;
    __shared__ double sh[16];
    const long long p = blockIdx.x;
    long long I = 0, rem = p;
    while (rem >= a.nT - I) { rem -= a.nT - I; ++I; }
    const long long J = I + rem;
    const long long I0 = I * kT, J0 = J * kT, N = a.N;
    const bool has_gap = a.gap != nullptr && (a.ng_p == nullptr || *a.ng_p > 0);
    if (threadIdx.x < kT) {
        const int r = threadIdx.x;
        const long long gi = I0 + r, gj = J0 + r;
        tv.aI[r] = gi < N ? a.alpha[gi] : 1.0;
        tv.aJ[r] = gj < N ? a.alpha[gj] : 1.0;
        tv.gI[r] = (has_gap && gi < N) ? a.gap[gi] : 0;
        tv.gJ[r] = (has_gap && gj < N) ? a.gap[gj] : 0;
        if (PASS > 1) {
            tv.sI[r] = gi < N ? a.s[gi] : 1.0;
            tv.sJ[r] = gj < N ? a.s[gj] : 1.0;
        }
    }
    __syncthreads();
    load_pair(X, N, I0, J0, tv, st, stT);
    __syncthreads();
    const bool diag_tile = I == J;
    const int lim_r = (int)std::min<long long>(kT, N - I0), lim_c = (int)std::min<long long>(kT, N - J0);
    if (PASS == 1) {
        const int r = threadIdx.x >> 2, q = threadIdx.x & 3;
        // row sum of I-row r over J columns
        double acc = 0.0;
        if (r < lim_r)
#pragma unroll 4
            for (int k = 0; k < kT / 4; ++k) {
                const int c = q + 4 * k;
                if (c < lim_c) acc += sym_value(diag_tile && r == c, has_gap, tv.gI[r], tv.gJ[c], st[r][c], stT[r][c]);
            }
        acc += __shfl_xor(acc, 1, 64);
        acc += __shfl_xor(acc, 2, 64);
        // column sum of J-column r (= row J0+r of Y) over I rows
        double acc2 = 0.0;
        if (r < lim_c)
#pragma unroll 4
            for (int k = 0; k < kT / 4; ++k) {
                const int i = q + 4 * k;
                if (i < lim_r)
                    acc2 += sym_value(diag_tile && i == r, has_gap, tv.gI[i], tv.gJ[r], st[i][r], stT[i][r]);
            }
        acc2 += __shfl_xor(acc2, 1, 64);
        acc2 += __shfl_xor(acc2, 2, 64);
        if (q == 0) {
            part[p * (2 * kT) + r] = acc;
            part[p * (2 * kT) + kT + r] = acc2;
        }
    } else if (PASS == 2) {
        const int r = threadIdx.x >> 2, q = threadIdx.x & 3;
        double acc = 0.0;
        if (r < lim_r) {
            const double si = tv.sI[r];
#pragma unroll 4
            for (int k = 0; k < kT / 4; ++k) {
                const int c = q + 4 * k;
                if (c < lim_c) {
                    const double y = sym_value(diag_tile && r == c, has_gap, tv.gI[r], tv.gJ[c], st[r][c], stT[r][c]);
                    acc += y / (tv.sJ[c] * si);
                }
            }
        }
        if (!diag_tile) acc *= 2.0;
        acc = block_sum(acc, sh);
        if (threadIdx.x == 0) part[p] = acc;
    } else {
        const double scale = a.scale_p ? *a.scale_p : a.scale;
        const int c = threadIdx.x & (kT - 1);
        for (int r = threadIdx.x >> 6; r < lim_r; r += 4) {
            if (c < lim_c) {
                const double y = sym_value(diag_tile && r == c, has_gap, tv.gI[r], tv.gJ[c], st[r][c], stT[r][c]);
                __builtin_nontemporal_store(scale * (y / (tv.sJ[c] * tv.sI[r])), &out[(I0 + r) * N + J0 + c]);
            }
        }
        if (!diag_tile) {
            // element (J0 + r, I0 + c) = Y[I0 + c][J0 + r] (Y symmetric)
            for (int r = threadIdx.x >> 6; r < lim_c; r += 4) {
                if (c < lim_r) {
                    const double y = sym_value(false, has_gap, tv.gI[c], tv.gJ[r], st[c][r], stT[c][r]);
                    __builtin_nontemporal_store(scale * (y / (tv.sI[c] * tv.sJ[r])), &out[(J0 + r) * N + I0 + c]);
                }
            }
        }
    }
}

// PASS 3 with one LDS tile (round 4, default; hh_tune "symvc_out"): both
// tiles' X values are loaded into registers (lane = column, coalesced), the
// (J, I) tile goes through LDS transposed for the (I, J) outputs.  Y and C are
// symmetric, so each (J, I) output is the (I, J) output at the transposed
// position -- the same operands and IEEE operations (round 5: computed once,
// sent through the same LDS space transposed, instead of recomputing the two
// true divisions of S and the third of C per element): bitwise k_symvc<T, 3>.
// its LDS, declared by the kernel: one copy whichever element types the
// kernel instantiates the body with (two instantiations each declaring its
// own had k_sv_out_b at 70 KB per block, 2 blocks per CU; with one copy and
// 4 waves per SIMD the 40 kb genome's output pass takes 1.79 -> 1.62 ms).
// Measured and not kept (round 6): the pass by row bands -- each output
// row's 2 KB written by one wave, every element computed at its own
// position -- 1.69 ms: twice the divisions, and the 512-byte row pieces of
// the tile pairs were not what bound it (profiles/r6q/)
struct SvOutLds {
    double u[kT][kT + 1];  // the (J, I) tile transposed (as T), then the (I, J) outputs transposed
    TileVecs tv;
};
template <class T>
__device__ __forceinline__ T (&sv_tt(SvOutLds& S))[kT][kT + 1] {
    static_assert(sizeof(T) <= sizeof(double), "element wider than the LDS cell");
    return *reinterpret_cast<T(*)[kT][kT + 1]>(&S.u);
}

template <class T, class L = T>  // L: the element type read (see ts_gemv_body)
__device__ __forceinline__ void symvc_out_body(SvOutLds& S, const L* __restrict__ X, const SymArgs& a,
                                               double* __restrict__ out, long long p, int cnt = 1,
                                               const long long* __restrict__ Xe = nullptr) {
    // `cnt` consecutive pairs p, p + 1, ...: the next pair's matrix loads are
    // issued before this pair's transposed outputs are written (two pairs per
    // block: 1.88 -> 1.86 ms per genome; plain stores instead of the
    // nontemporal ones: 2.22 ms)
    T (&tt)[kT][kT + 1] = sv_tt<T>(S);  // the (J, I) tile, transposed
    double (&dt)[kT][kT + 1] = S.u;     // then the (I, J) outputs, transposed
    TileVecs& tv = S.tv;
    const long long N = a.N;
    const bool has_gap = a.gap != nullptr && (a.ng_p == nullptr || *a.ng_p > 0);
    const int c = threadIdx.x & (kT - 1);
    const int r0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar row bases
    const double scale = *a.scale_p;
    long long I0 = 0, J0 = 0;
    auto decode = [&](long long q) __attribute__((always_inline)) {
        long long I = 0, rem = q;
        while (rem >= a.nT - I) { rem -= a.nT - I; ++I; }
        I0 = I * kT;
        J0 = (I + rem) * kT;
    };
    // Clamped addresses and no select on any loaded value (a select lets the
    // compiler sink each load into a branch with its own vmcnt(0) wait); a
    // value read from a clamped address is never used: the outputs are
    // guarded by lim_r / lim_c, and a valid output's operands are in range.
    T v[kT / 4], w[kT / 4];
    auto load = [&]() __attribute__((always_inline)) {
        const long long cj = J0 + c < N ? J0 + c : N - 1, ci = I0 + c < N ? I0 + c : N - 1;
#pragma unroll
        for (int k = 0; k < kT / 4; ++k) {
            const int r = r0 + 4 * k;
            const long long gi = I0 + r, ti = J0 + r;
            v[k] = (T)X[(gi < N ? gi : N - 1) * N + cj];
            w[k] = (T)X[(ti < N ? ti : N - 1) * N + ci];
        }
    };
    // escaped counts (rare): from the int64 matrix -- at the pair's first use
    // of v / w, so a prefetched pair's loads stay in flight until then
    auto patch = [&]() __attribute__((always_inline)) {
        if constexpr (!std::is_same_v<L, T>) {
            const long long cj = J0 + c < N ? J0 + c : N - 1, ci = I0 + c < N ? I0 + c : N - 1;
            bool esc = false;
#pragma unroll
            for (int k = 0; k < kT / 4; ++k) esc |= (v[k] == (T)0xFFFF) | (w[k] == (T)0xFFFF);
            if (__ballot(esc) != 0ull) {
#pragma unroll
                for (int k = 0; k < kT / 4; ++k) {
                    const int r = r0 + 4 * k;
                    const long long gi = I0 + r, ti = J0 + r;
                    if (v[k] == (T)0xFFFF) v[k] = (T)Xe[(gi < N ? gi : N - 1) * N + cj];
                    if (w[k] == (T)0xFFFF) w[k] = (T)Xe[(ti < N ? ti : N - 1) * N + ci];
                }
            }
        }
    };
    decode(p);
    load();
    for (int it = 0; it < cnt; ++it) {
        if (it) __syncthreads();  // the previous pair's LDS reads are done
        patch();
        const long long cI0 = I0, cJ0 = J0;
        const bool diag_tile = cI0 == cJ0;
        if (threadIdx.x < kT) {
            const int r = threadIdx.x;
            const long long gi = cI0 + r < N ? cI0 + r : N - 1, gj = cJ0 + r < N ? cJ0 + r : N - 1;
            tv.aI[r] = a.alpha[gi];
            tv.aJ[r] = a.alpha[gj];
            tv.sI[r] = a.s[gi];
            tv.sJ[r] = a.s[gj];
            if (has_gap) {
                tv.gI[r] = a.gap[gi];
                tv.gJ[r] = a.gap[gj];
            } else {
                tv.gI[r] = tv.gJ[r] = 0;
            }
        }
        const int lim_r = (int)std::min<long long>(kT, N - cI0), lim_c = (int)std::min<long long>(kT, N - cJ0);
        // (I, J) outputs: S_ij = v / aI[r], S_ji = X[J0 + c][I0 + r] / aJ[c] = tt[r][c] / aJ[c]
#pragma unroll
        for (int k = 0; k < kT / 4; ++k) tt[c][r0 + 4 * k] = w[k];
        __syncthreads();
        double o[kT / 4];
#pragma unroll
        for (int k = 0; k < kT / 4; ++k) {
            const int r = r0 + 4 * k;
            const double sij = (double)v[k] / tv.aI[r], sji = (double)tt[r][c] / tv.aJ[c];
            const double y = sym_value(diag_tile && r == c, has_gap, tv.gI[r], tv.gJ[c], sij, sji);
            o[k] = scale * (y / (tv.sJ[c] * tv.sI[r]));
            if (r < lim_r && c < lim_c) __builtin_nontemporal_store(o[k], &out[(cI0 + r) * N + cJ0 + c]);
        }
        if (it + 1 < cnt) {  // the next pair's loads, in flight across this pair's transposed writes
            decode(p + it + 1);
            load();
        }
        if (diag_tile) continue;
        __syncthreads();  // every tt read done: the space takes the outputs
        // (J, I) outputs: element (J0 + r, I0 + c) = C[I0 + c][J0 + r] (symmetric)
#pragma unroll
        for (int k = 0; k < kT / 4; ++k) dt[c][r0 + 4 * k] = o[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kT / 4; ++k) {
            const int r = r0 + 4 * k;
            if (r < lim_c && c < lim_r) __builtin_nontemporal_store(dt[r][c], &out[(cJ0 + r) * N + cI0 + c]);
        }
    }
}

template <class T>
__global__ __launch_bounds__(256) void k_symvc_out(const T* __restrict__ X, SymArgs a, double* __restrict__ out) {
    __shared__ SvOutLds S;
    symvc_out_body<T>(S, X, a, out, blockIdx.x);
}

// rowsum(Y)_i from the pass-1 slab in a fixed order (J = 0 .. nT-1), then
// s_i = rowsum^exponent, 0 -> 1.
__global__ void k_symvc_rows(const double* __restrict__ part, long long N, long long nT, double exponent,
                             double* __restrict__ s) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const long long I = i / kT;
    const int r = (int)(i % kT);
    // loads 8 tiles at a time (independent), added in J order: the same sum
    auto at = [&](long long J) {
        return J >= I ? part[pair_index(I, J, nT) * (2 * kT) + r] : part[pair_index(J, I, nT) * (2 * kT) + kT + r];
    };
    double acc = 0.0;
    long long J = 0;
    for (; J + 8 <= nT; J += 8) {
        double x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = at(J + u);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += x[u];
    }
    for (; J < nT; ++J) acc += at(J);
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

// the mean rescale (raw_sum / N^2) / (sum C / N^2) on the device, the same
// IEEE operations as on the host
__global__ void k_symvc_scale(const double* __restrict__ tot, double raw_sum, const double* __restrict__ raw_p,
                              double nn, double* __restrict__ scale) {
    if (threadIdx.x == 0) *scale = ((raw_p ? *raw_p : raw_sum) / nn) / (*tot / nn);
}

// ---- passes 1-2 as row streams (round 4, default; hh_tune "symvc_stream") --
// The tile-pair passes read S_ij and S_ji together through two LDS tiles
// (~113 us each at N = 6 232: 2.8 TB/s, 2 blocks per CU).  Passes 1 and 2
// only need sums, and Y's sums follow from plain row / column sums of S:
//   R_i = sum_j S_ij = (sum_j X_ij) / alpha_i,   Ccol_i = sum_j S_ji
//   gap form (Trans2symmetry :957-979):
//     rowsum(Y)_i = (R_i + Ccol_i) / 2 + [i in G] sum_{j in G, j != i} |S_ij - S_ji| / 2
//     (max(a, b) = (a + b) / 2 + |a - b| / 2 on the both-gap pairs)
//   sum form (no gap, :947-955): rowsum(Y)_i = R_i + Ccol_i - S_ii
//   Q = sum_ij S_ij / (s_i s_j) = sum_i (sum_j X_ij / s_j) / (alpha_i s_i)
//   gap form: sum(C) = Q + sum_{i != j in G} |S_ij - S_ji| / (2 s_i s_j)
//   sum form: sum(C) = 2 Q - sum_i S_ii / s_i^2
// so each pass is one coalesced row-major stream over X (k_ts_gemv) plus a
// gap-pair correction over |G|^2 elements (k_ts_gap).  Every partial is
// summed in a fixed order (deterministic); the sums differ from the
// tile-pair passes only by rounding (the int64 row sums are exact).
// rows per block: hh_tune "symvc_rows" (g_symvc_rows; every wave of the block
// takes every row of it)
constexpr int kGW = 512;      // columns per wave (8 per lane, 512 B per load instruction)
constexpr int kGB = 4 * kGW;  // columns per block: its 4 waves read 16 KB of a row together

// Wave w of block (rc, cb) owns the 512-column span q = 4 cb + w and the
// block's rows r0 .. r0 + gr - 1 (reading a row's 2 048 block columns
// together keeps the HBM pages open; 64x64 tiles read 512 B per row and ran
// at ~2.7 TB/s).
// MODE 1: part_c[rc][j] = sum over the block's rows i of X_ij * (1 / alpha_i);
//         part_r[q][i] = sum over the span's columns of X_ij (int64 exact for
//         integer X, stored in the double slot's bits); the both-gap entries
//         X_ij (i, j gaps) copied to the compact g x g matrix Xc.
// MODE 2: part_r[q][i] = sum over the span's columns of X_ij * rs_j.
// L: the element type read (uint16_t: the batch's copy, 0xFFFF entries taken
// from the int64 matrix Xe); T: the value type the pass computes with.
template <class T, int MODE, bool ROWS = true, class L = T, int KB = 4>
__device__ __forceinline__ void ts_gemv_body(const L* __restrict__ X, long long N, const double* __restrict__ alpha,
                                             const double* __restrict__ rs, int gr, double* __restrict__ part_c,
                                             double* __restrict__ part_r, const int* __restrict__ gpos,
                                             T* __restrict__ Xc, const long long* __restrict__ ng_p, long long bx,
                                             long long by, const long long* __restrict__ Xe = nullptr) {
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long long rc = bx, q = by * 4 + w;
    const long long r0 = rc * gr, c0 = q * kGW;
    if (c0 >= N) return;  // wave-uniform; no block barrier below
    double accc[8], bcol[8];
    bool okc[8];
    int gcol[8];        // MODE 1 with gaps: the column's compact index, -1 if not a gap
    unsigned coff[8];   // clamped column offsets (elements) from the span's first column
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const long long c = c0 + lane + 64 * k;
        okc[k] = c < N;
        coff[k] = (unsigned)((okc[k] ? c : N - 1) - c0);
        accc[k] = 0.0;
        bcol[k] = (MODE == 2 && okc[k]) ? rs[c] : 0.0;
        gcol[k] = (MODE == 1 && gpos && okc[k]) ? gpos[c] : -1;
    }
    const long long rend = std::min<long long>(r0 + gr, N);
    const long long ng = (MODE == 1 && gpos) ? *ng_p : 0;  // Xc's row stride
    // MODE 1: the block's rows' 1 / alpha and gap positions, one lane per row
    // (gr <= 64), taken by v_readlane in the row loop instead of a dependent
    // load per row
    const bool lane_rows = MODE == 1 && gr <= 64;
    double ra_l = 0.0;
    int gp_l = -1;
    if (lane_rows && r0 + lane < rend) {
        ra_l = 1.0 / alpha[r0 + lane];
        if (gpos) gp_l = gpos[r0 + lane];
    }
    constexpr int kB = KB;  // rows per batch: 8 KB loads in flight per lane
#pragma unroll 1
    for (long long i0 = r0; i0 < rend; i0 += kB) {
        T x[kB][8];
#pragma unroll
        for (int b = 0; b < kB; ++b) {
            const bool okr = i0 + b < rend;
            // unconditional loads from clamped addresses (row clamped to the
            // last one, columns to N - 1); the clamped values are weighted by
            // zero or masked where they are summed -- a select on the loaded
            // value lets the compiler sink each load into its own branch
            // with a vmcnt(0) wait (measured: 32 serialised loads)
            const L* row = X + (okr ? i0 + b : rend - 1) * N + c0;
#pragma unroll
            for (int k = 0; k < 8; ++k) x[b][k] = (T)row[coff[k]];
        }
        if constexpr (!std::is_same_v<L, T>) {  // escaped counts (rare): from the int64 matrix
            bool esc = false;
#pragma unroll
            for (int b = 0; b < kB; ++b)
#pragma unroll
                for (int k = 0; k < 8; ++k) esc |= x[b][k] == (T)0xFFFF;
            if (__ballot(esc) != 0ull) {
#pragma unroll
                for (int b = 0; b < kB; ++b) {
                    const long long* rowe = Xe + (i0 + b < rend ? i0 + b : rend - 1) * N + c0;
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        if (x[b][k] == (T)0xFFFF) x[b][k] = (T)rowe[coff[k]];
                }
            }
        }
#pragma unroll
        for (int b = 0; b < kB; ++b) {
            const long long i = i0 + b;
            const bool okr = i < rend;
            if (MODE == 1) {
                // S_ij = X_ij / alpha_i as X_ij * (1 / alpha_i): within an ulp of the
                // true quotient, and a division per element doubles the registers
                double ra;
                if (lane_rows) {
                    const int li = (int)(i - r0) & 63;  // (i >= rend: the value is not used)
                    ra = okr ? readlane_dbl(ra_l, li) : 0.0;
                } else {
                    ra = okr ? 1.0 / alpha[i] : 0.0;
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) accc[k] += (double)x[b][k] * ra;
                if (gpos && okr) {
                    const int gi = lane_rows ? __builtin_amdgcn_readlane(gp_l, (int)(i - r0)) : gpos[i];
                    if (gi >= 0) {
#pragma unroll
                        for (int k = 0; k < 8; ++k)
                            if (gcol[k] >= 0) Xc[(long long)gi * ng + gcol[k]] = x[b][k];
                    }
                }
                if constexpr (!ROWS) {
                    // the row sums come from k_rowstats (hh_twostep)
                } else if constexpr (std::is_integral_v<T>) {
                    long long t = 0;
#pragma unroll
                    for (int k = 0; k < 8; ++k) t += okc[k] ? (long long)x[b][k] : 0LL;
                    t = wave_sum_ll(t);
                    if (lane == 0 && okr) reinterpret_cast<long long*>(part_r)[q * N + i] = t;
                } else {
                    double t = 0.0;
#pragma unroll
                    for (int k = 0; k < 8; ++k) t += okc[k] ? (double)x[b][k] : 0.0;
                    t = wave_sum(t);
                    if (lane == 0 && okr) part_r[q * N + i] = t;
                }
            } else {
                double t = 0.0;
#pragma unroll
                for (int k = 0; k < 8; ++k) t += (double)x[b][k] * bcol[k];
                t = wave_sum(t);
                if (lane == 0 && okr) part_r[q * N + i] = t;
            }
        }
    }
    if (MODE == 1) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (okc[k]) part_c[rc * N + c0 + lane + 64 * k] = accc[k];
    }
}

template <class T, int MODE, bool ROWS = true>
__global__ __launch_bounds__(256) void k_ts_gemv(const T* __restrict__ X, long long N,
                                                 const double* __restrict__ alpha, const double* __restrict__ rs,
                                                 int gr, double* __restrict__ part_c, double* __restrict__ part_r,
                                                 const int* __restrict__ gpos, T* __restrict__ Xc,
                                                 const long long* __restrict__ ng_p) {
    ts_gemv_body<T, MODE, ROWS>(X, N, alpha, rs, gr, part_c, part_r, gpos, Xc, ng_p, blockIdx.x, blockIdx.y);
}

// The both-gap pairs' correction on the compact g x g matrix Xc (gap rows
// and columns in index order): block (A, B) of 64 x 64 tiles gives, for each
// compact row a of A,
//   MODE 1: gpart[B][a] = sum_{b in B, b != a} |S_ab - S_ba| / 2
//   MODE 2: gpart[B][a] = sum_{b in B, b != a} (|S_ab - S_ba| / 2) / (s_b s_a)
// with S_ab = Xc[a][b] / alpha_{G[a]}; (B, A) is read coalesced and
// transposed through LDS.
// (its LDS declared by the kernel: one copy for both element types of the
// batch kernel, which had 58 KB per block with a copy per instantiation)
struct GapLds {
    double tt[kT][kT + 1];  // as T
    double aA[kT], aB[kT], sA[kT], sB[kT];
    double red[4][kT];
};
template <class T, int MODE>
__device__ __forceinline__ void ts_gap_body(GapLds& S, const T* __restrict__ Xc, const long long* __restrict__ ng_p,
                                            const int* __restrict__ glist, const double* __restrict__ alpha,
                                            const double* __restrict__ sv, double* __restrict__ gpart, long long bx,
                                            long long gdx) {
    static_assert(sizeof(T) <= sizeof(double), "element wider than the LDS cell");
    T (&tt)[kT][kT + 1] = *reinterpret_cast<T(*)[kT][kT + 1]>(&S.tt);
    double *aA = S.aA, *aB = S.aB, *sA = S.sA, *sB = S.sB;
    double (&red)[4][kT] = S.red;
    const long long ng = *ng_p, nbt = (ng + kT - 1) / kT;
    const int c = threadIdx.x & (kT - 1), r0 = threadIdx.x >> 6;
    // grid-stride over the nbt x nbt tiles (the gap count is known on the device only)
    for (long long t = bx; t < nbt * nbt; t += gdx) {
        const long long Ab = t / nbt, Bb = t % nbt;
        const long long A0 = Ab * kT, B0 = Bb * kT;
        // clamped addresses, no select on loaded values (see k_symvc_out); a
        // value from a clamped address is never used
        const long long ca = A0 + c < ng ? A0 + c : ng - 1, cbb = B0 + c < ng ? B0 + c : ng - 1;
        T xd[kT / 4];
#pragma unroll
        for (int k = 0; k < kT / 4; ++k) {
            const int r = r0 + 4 * k;
            const long long ra = A0 + r < ng ? A0 + r : ng - 1, rb = B0 + r < ng ? B0 + r : ng - 1;
            tt[c][r] = Xc[rb * ng + ca];  // tt[c][r] = Xc[B0 + r][A0 + c]
            xd[k] = Xc[ra * ng + cbb];    // Xc[A0 + r][B0 + c]
        }
        if (threadIdx.x < kT) {
            const int r = threadIdx.x;
            const int ga = glist[A0 + r < ng ? A0 + r : ng - 1], gb = glist[B0 + r < ng ? B0 + r : ng - 1];
            aA[r] = alpha[ga];
            aB[r] = alpha[gb];
            sA[r] = MODE == 2 ? sv[ga] : 1.0;
            sB[r] = MODE == 2 ? sv[gb] : 1.0;
        }
        __syncthreads();
        // thread: row a = A0 + r (r = r0 + 4 k), column b = B0 + c; reduce over c
#pragma unroll
        for (int k = 0; k < kT / 4; ++k) {
            const int r = r0 + 4 * k;
            const long long a = A0 + r, b = B0 + c;
            double d = 0.0;
            if (a < ng && b < ng && a != b) {
                const double sab = (double)xd[k] / aA[r], sba = (double)tt[r][c] / aB[c];
                d = fabs(sab - sba) / 2.0;
                if (MODE == 2) d = d / (sB[c] * sA[r]);
            }
            d = wave_sum(d);
            if (c == 0) red[r0][k] = d;
        }
        __syncthreads();
        if (threadIdx.x < kT) {
            const int r = threadIdx.x;  // r = r0' + 4 k'
            if (A0 + r < ng) gpart[Bb * ng + A0 + r] = red[r & 3][r >> 2];
        }
        __syncthreads();
    }
}

template <class T, int MODE>
__global__ __launch_bounds__(256) void k_ts_gap(const T* __restrict__ Xc, const long long* __restrict__ ng_p,
                                                const int* __restrict__ glist, const double* __restrict__ alpha,
                                                const double* __restrict__ sv, double* __restrict__ gpart) {
    __shared__ GapLds S;
    ts_gap_body<T, MODE>(S, Xc, ng_p, glist, alpha, sv, gpart, blockIdx.x, gridDim.x);
}

// Ccol_j = sum over the row chunks of part_c[rc][j] (fixed order: wave w
// sums a contiguous range of chunks, the 16 wave sums added in order).
__device__ __forceinline__ void ts_colsum_body(const double* __restrict__ part_c, long long N, long long nrc,
                                               double* __restrict__ ccol, long long bx) {
    __shared__ double red[16][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long long j = bx * 64 + lane;
    const long long per = (nrc + 15) / 16, lo = std::min<long long>(nrc, w * per),
                    hi = std::min<long long>(nrc, lo + per);
    double acc = 0.0;
    if (j < N) {
        long long rc = lo;
        for (; rc + 8 <= hi; rc += 8) {
            double x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) x[u] = part_c[(rc + u) * N + j];
#pragma unroll
            for (int u = 0; u < 8; ++u) acc += x[u];
        }
        for (; rc < hi; ++rc) acc += part_c[rc * N + j];
    }
    red[w][lane] = acc;
    __syncthreads();
    if (threadIdx.x < 64 && j < N) {
        double t = 0.0;
        for (int k = 0; k < 16; ++k) t += red[k][threadIdx.x];
        ccol[j] = t;
    }
}

__global__ __launch_bounds__(1024) void k_ts_colsum(const double* __restrict__ part_c, long long N, long long nrc,
                                                    double* __restrict__ ccol) {
    ts_colsum_body(part_c, N, nrc, ccol, blockIdx.x);
}

// rowsum(Y) from the MODE-1 partials (fixed order), s = rowsum^exponent
// (0 -> 1) and 1 / s.
template <class T>
__device__ __forceinline__ void ts_rows_body(const T* __restrict__ X, long long N, long long ncb,
                                             const double* __restrict__ ccol, const double* __restrict__ part_r,
                                             const double* __restrict__ alpha, const int* __restrict__ gpos,
                                             const double* __restrict__ gpart, const long long* __restrict__ ng_p,
                                             double exponent, const double* __restrict__ rowsum_in,
                                             double* __restrict__ sv, double* __restrict__ rsv, long long bx) {
    const long long i = bx * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const long long ng = ng_p ? *ng_p : 0;  // gap form iff ng > 0 (Trans2symmetry :948)
    const double c = ccol[i];
    double rsum;
    if (rowsum_in) {
        rsum = rowsum_in[i];  // k_rowstats' exact integer row sum (the same double)
    } else if constexpr (std::is_integral_v<T>) {
        long long t = 0;
        for (long long cb = 0; cb < ncb; ++cb) t += reinterpret_cast<const long long*>(part_r)[cb * N + i];
        rsum = (double)t;
    } else {
        double t = 0.0;
        for (long long cb = 0; cb < ncb; ++cb) t += part_r[cb * N + i];
        rsum = t;
    }
    const double ai = alpha[i];
    const double r = rsum / ai;
    double y;
    if (ng > 0) {
        y = (r + c) / 2.0;
        if (gpos[i] >= 0) {  // the both-gap pairs' max - mean, in tile order
            const long long a = gpos[i], nbt = (ng + kT - 1) / kT;
            double gc = 0.0;
            for (long long B = 0; B < nbt; ++B) gc += gpart[B * ng + a];
            y += gc;
        }
    } else {
        y = (r + c) - (double)X[i * N + i] / ai;
    }
    double v = pow(y, exponent);
    if (v == 0.0) v = 1.0;
    sv[i] = v;
    rsv[i] = 1.0 / v;
}

template <class T>
__global__ void k_ts_rows(const T* __restrict__ X, long long N, long long ncb,
                          const double* __restrict__ ccol, const double* __restrict__ part_r,
                          const double* __restrict__ alpha, const int* __restrict__ gpos,
                          const double* __restrict__ gpart, const long long* __restrict__ ng_p, double exponent,
                          const double* __restrict__ rowsum_in, double* __restrict__ sv, double* __restrict__ rsv) {
    ts_rows_body<T>(X, N, ncb, ccol, part_r, alpha, gpos, gpart, ng_p, exponent, rowsum_in, sv, rsv, blockIdx.x);
}

// Per-block partials of sum(C) from the MODE-2 row partials.
template <class T>
__device__ __forceinline__ void ts_q_body(const T* __restrict__ X, long long N, long long ncb,
                                          const double* __restrict__ part_r, const double* __restrict__ alpha,
                                          const double* __restrict__ sv, const double* __restrict__ gpart2,
                                          const long long* __restrict__ ng_p, double* __restrict__ part, long long bx) {
    __shared__ double sh[16];
    const long long i = bx * 256 + threadIdx.x;
    const long long ng = ng_p ? *ng_p : 0;
    double term = 0.0;
    if (i < N) {
        double u = 0.0;
        for (long long cb = 0; cb < ncb; ++cb) u += part_r[cb * N + i];
        const double ai = alpha[i], si = sv[i];
        const double q = u / (ai * si);
        if (ng > 0) {
            term = q;
            if (i < ng) {  // compact gap row i's both-gap share of sum(C)
                const long long nbt = (ng + kT - 1) / kT;
                double g2 = 0.0;
                for (long long B = 0; B < nbt; ++B) g2 += gpart2[B * ng + i];
                term += g2;
            }
        } else {
            const double sii = (double)X[i * N + i] / ai;
            term = 2.0 * q - sii / (si * si);
        }
    }
    term = block_sum(term, sh);
    if (threadIdx.x == 0) part[bx] = term;
}

template <class T>
__global__ __launch_bounds__(256) void k_ts_q(const T* __restrict__ X, long long N, long long ncb,
                                              const double* __restrict__ part_r, const double* __restrict__ alpha,
                                              const double* __restrict__ sv, const double* __restrict__ gpart2,
                                              const long long* __restrict__ ng_p, double* __restrict__ part) {
    ts_q_body<T>(X, N, ncb, part_r, alpha, sv, gpart2, ng_p, part, blockIdx.x);
}

// Workspace of one Trans2symmetry + Correct_VC + rescale chain (alive until
// the stream has run it).
struct SymvcWs {
    DBuf<double> part, sv, tot;
    DBuf<double> part_c, part_r, rsv, ccol, gpart1, gpart2;  // streaming passes
    DBuf<int> glist, gpos;
    DBuf<long long> ngd;
    DBuf<char> xc;  // the compact both-gap matrix
    std::vector<int> hgl, hgp;  // host sources of glist / gpos (alive until the copies ran)
    long long hng = 0;
};

// The gap rows (index order), each row's position among them (-1: not a
// gap) and their count, on the device, for the streaming passes' both-gap
// correction; ng_max bounds the count (sizes the compact matrix).
struct GapIdx {
    const int* gpos = nullptr;
    const int* glist = nullptr;
    const long long* ng_p = nullptr;
    long long ng_max = 0;
};

static void gap_index_host(const uint8_t* hgap, long long N, std::vector<int>& gl, std::vector<int>& gp) {
    gl.clear();
    gp.assign(N, -1);
    for (long long i = 0; i < N; ++i)
        if (hgap[i]) { gp[i] = (int)gl.size(); gl.push_back((int)i); }
}

// Enqueues the chain without a host round trip (the rescale factor is
// formed and read on the device); `ws` must outlive the kernels.  The
// streaming passes take the gap form iff the device gap count is > 0; the
// tile-pair passes (symvc_stream 0) iff dgap != nullptr.  raw_p: the mean
// rescale's raw total on the device (else raw_sum).
template <class T>
static void symvc_enqueue(const T* dX, long long N, const double* dalpha, const uint8_t* dgap, GapIdx gi,
                          double exponent, double raw_sum, const double* raw_p, double* dout, hipStream_t s,
                          SymvcWs& ws, const double* rowsum_in = nullptr) {
    const long long nT = (N + kT - 1) / kT;
    const long long npairs = nT * (nT + 1) / 2;
    HH_REQUIRE(npairs < (1LL << 31), "matrix too large");
    ws.sv.alloc(N);
    ws.tot.alloc(2);
    SymArgs a{N, nT, dalpha, dgap, nullptr, 1.0};
    if (g_symvc_stream) {
        const int gr = g_symvc_rows;
        const long long nrc = (N + gr - 1) / gr, ncb = (N + kGW - 1) / kGW;
        HH_REQUIRE(ncb < 65536 && nrc < (1LL << 31), "matrix too large");
        const long long nb = (N + 255) / 256;
        ws.part_c.alloc((size_t)(nrc * N));
        ws.part_r.alloc((size_t)(ncb * N));
        ws.rsv.alloc(N);
        ws.ccol.alloc(N);
        ws.part.alloc((size_t)nb);
        const long long ngm = (dgap && gi.ng_p) ? gi.ng_max : 0;
        const long long nbtm = (ngm + kT - 1) / kT;
        if (ngm) {
            ws.xc.alloc((size_t)(ngm * ngm) * sizeof(T));
            ws.gpart1.alloc((size_t)(nbtm * ngm));
            ws.gpart2.alloc((size_t)(nbtm * ngm));
        }
        T* xc = ngm ? (T*)ws.xc.p : nullptr;
        const int* gpos = ngm ? gi.gpos : nullptr;
        const long long* ng_p = ngm ? gi.ng_p : nullptr;
        const unsigned ggrid = (unsigned)std::min<long long>(std::max<long long>(nbtm * nbtm, 1), 2048);
        const unsigned gcb = (unsigned)((N + kGB - 1) / kGB);
        {
            HH_KTIME("k_ts_gemv1", s);
            auto kern = rowsum_in ? k_ts_gemv<T, 1, false> : k_ts_gemv<T, 1, true>;
            hipLaunchKernelGGL(kern, dim3((unsigned)nrc, gcb), dim3(256), 0, s, dX, N, dalpha,
                               (const double*)nullptr, gr, ws.part_c.p, ws.part_r.p, gpos, xc, ng_p);
        }
        if (ngm)
            hipLaunchKernelGGL((k_ts_gap<T, 1>), dim3(ggrid), dim3(256), 0, s, (const T*)xc, ng_p, gi.glist, dalpha,
                               (const double*)nullptr, ws.gpart1.p);
        hipLaunchKernelGGL(k_ts_colsum, dim3((unsigned)((N + 63) / 64)), dim3(1024), 0, s, ws.part_c.p, N, nrc,
                           ws.ccol.p);
        hipLaunchKernelGGL((k_ts_rows<T>), dim3((unsigned)nb), dim3(256), 0, s, dX, N, ncb, ws.ccol.p, ws.part_r.p,
                           dalpha, gpos, ws.gpart1.p, ng_p, exponent, rowsum_in, ws.sv.p, ws.rsv.p);
        if (ngm)
            hipLaunchKernelGGL((k_ts_gap<T, 2>), dim3(ggrid), dim3(256), 0, s, (const T*)xc, ng_p, gi.glist, dalpha,
                               ws.sv.p, ws.gpart2.p);
        {
            HH_KTIME("k_ts_gemv2", s);
            hipLaunchKernelGGL((k_ts_gemv<T, 2>), dim3((unsigned)nrc, gcb), dim3(256), 0, s, dX, N, dalpha, ws.rsv.p,
                               gr, ws.part_c.p, ws.part_r.p, (const int*)nullptr, (T*)nullptr,
                               (const long long*)nullptr);
        }
        hipLaunchKernelGGL((k_ts_q<T>), dim3((unsigned)nb), dim3(256), 0, s, dX, N, ncb, ws.part_r.p, dalpha, ws.sv.p,
                           ws.gpart2.p, ng_p, ws.part.p);
        hipLaunchKernelGGL(k_slab_sum, dim3(1), dim3(256), 0, s, ws.part.p, nb, ws.tot.p);
        hipLaunchKernelGGL(k_symvc_scale, dim3(1), dim3(64), 0, s, ws.tot.p, raw_sum, raw_p, (double)N * (double)N,
                           ws.tot.p + 1);
        a.s = ws.sv.p;
        a.scale_p = ws.tot.p + 1;
        // pass 3's form: the device gap count (no gap array: the sum form)
        if (!ng_p) a.gap = nullptr;
        a.ng_p = ng_p;
        {
            HH_KTIME("k_symvc3", s);
            if (g_symvc_out)
                hipLaunchKernelGGL((k_symvc_out<T>), dim3((unsigned)npairs), dim3(256), 0, s, dX, a, dout);
            else
                hipLaunchKernelGGL((k_symvc<T, 3>), dim3((unsigned)npairs), dim3(256), 0, s, dX, a, ws.part.p, dout);
        }
        HIP_CHECK(hipGetLastError());
        return;
    }
    ws.part.alloc((size_t)npairs * 2 * kT);
    {
        HH_KTIME("k_symvc1", s);
        hipLaunchKernelGGL((k_symvc<T, 1>), dim3((unsigned)npairs), dim3(256), 0, s, dX, a, ws.part.p, nullptr);
    }
    hipLaunchKernelGGL(k_symvc_rows, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, ws.part.p, N, nT, exponent,
                       ws.sv.p);
    a.s = ws.sv.p;
    {
        HH_KTIME("k_symvc2", s);
        hipLaunchKernelGGL((k_symvc<T, 2>), dim3((unsigned)npairs), dim3(256), 0, s, dX, a, ws.part.p, nullptr);
    }
    hipLaunchKernelGGL(k_slab_sum, dim3(1), dim3(256), 0, s, ws.part.p, npairs, ws.tot.p);
    hipLaunchKernelGGL(k_symvc_scale, dim3(1), dim3(64), 0, s, ws.tot.p, raw_sum, (const double*)nullptr,
                       (double)N * (double)N, ws.tot.p + 1);
    a.scale_p = ws.tot.p + 1;
    {
        HH_KTIME("k_symvc3", s);
        hipLaunchKernelGGL((k_symvc<T, 3>), dim3((unsigned)npairs), dim3(256), 0, s, dX, a, ws.part.p, dout);
    }
    HIP_CHECK(hipGetLastError());
}

template <class T>
static void symvc_run(const T* dX, long long N, const double* dalpha, const uint8_t* dgap, const uint8_t* hgap,
                      double exponent, double raw_sum, double* dout, hipStream_t s) {
    SymvcWs ws;
    GapIdx gi;
    if (dgap && hgap) {
        gap_index_host(hgap, N, ws.hgl, ws.hgp);
        ws.hng = (long long)ws.hgl.size();
        if (ws.hng) {
            ws.gpos = to_device(ws.hgp, s);
            ws.glist = to_device(ws.hgl, s);
            ws.ngd.alloc(1);
            ws.ngd.upload(&ws.hng, 1, s);
            gi = GapIdx{ws.gpos.p, ws.glist.p, ws.ngd.p, ws.hng};
        } else {
            dgap = nullptr;  // no gap rows: the sum form (Trans2symmetry :948)
        }
    }
    symvc_enqueue(dX, N, dalpha, dgap, gi, exponent, raw_sum, (const double*)nullptr, dout, s, ws);
    HIP_CHECK(hipStreamSynchronize(s));
}


// ---- TwoStepCorrection's glue on the device (round 4; hh_tune "twostep_devglue") ----
// Gap_defined, the SNP alpha and the raw totals from the row statistics
// without a host round trip: the same doubles as the host glue (cov = 1 -
// z / N, np.percentile's 'linear' order statistics found exactly by an
// 8-bit radix select on the bit patterns of the non-negative values, the
// same lerp), and the gap rows compacted in index order for the streaming
// passes.
struct SelLds {
    unsigned hist[256];
    unsigned long long prefix, minb;
    long long k;
    unsigned cnt;
    int flag;
};

// k-th smallest (0-based) of the non-negative doubles x_i (i < n) with
// take(i, x_i); every thread of the block calls it and gets the value.
template <class Get>
__device__ double block_kth(long long n, long long k, Get get, SelLds& L) {
    __syncthreads();
    if (threadIdx.x == 0) { L.prefix = 0; L.k = k; }
    __syncthreads();
    for (int shift = 56; shift >= 0; shift -= 8) {
        for (int t = threadIdx.x; t < 256; t += blockDim.x) L.hist[t] = 0;
        const unsigned long long pre = L.prefix;
        const unsigned long long hm = shift == 56 ? 0ull : (~0ull << (shift + 8));
        __syncthreads();
        for (long long i = threadIdx.x; i < n; i += blockDim.x) {
            double x;
            if (!get(i, x)) continue;
            const unsigned long long b = (unsigned long long)__double_as_longlong(x);
            if ((b & hm) == (pre & hm)) atomicAdd(&L.hist[(b >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            long long acc = 0;
            const long long kk = L.k;
            int d = 0;
            for (; d < 255; ++d) {
                if (acc + (long long)L.hist[d] > kk) break;
                acc += L.hist[d];
            }
            L.k = kk - acc;
            L.prefix = pre | ((unsigned long long)d << shift);
        }
        __syncthreads();
    }
    return __longlong_as_double((long long)L.prefix);
}

// The same k-th smallest with the candidates' bit patterns held in
// registers (kSelPer per thread; ~0 marks "not taken": a non-negative
// double's top bit is 0, so it never matches a prefix), the digits the
// candidates all share skipped (their min / max decide where the first
// differing byte is), and the 256 bins scanned by one wave.
constexpr int kSelPer = 16;  // N <= kSelPer * blockDim.x
__device__ unsigned long long block_kth_regs(const unsigned long long (&b)[kSelPer], long long k,
                                             unsigned long long lo, unsigned long long hi, SelLds& L) {
    if (lo == hi) return lo;
    const int hb = 63 - __clzll(lo ^ hi);
    const int shift0 = (hb / 8) * 8;
    __syncthreads();
    if (threadIdx.x == 0) { L.prefix = shift0 == 56 ? 0ull : (lo & (~0ull << (shift0 + 8))); L.k = k; }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    for (int shift = shift0; shift >= 0; shift -= 8) {
        for (int t = threadIdx.x; t < 256; t += blockDim.x) L.hist[t] = 0;
        const unsigned long long pre = L.prefix;
        const unsigned long long hm = shift == 56 ? 0ull : (~0ull << (shift + 8));
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kSelPer; ++u)
            if (b[u] != ~0ull && (b[u] & hm) == (pre & hm)) atomicAdd(&L.hist[(b[u] >> shift) & 255u], 1u);
        __syncthreads();
        if (threadIdx.x < 64) {
            const long long kk = L.k;
            unsigned h[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) h[q] = L.hist[4 * lane + q];
            long long own = (long long)h[0] + h[1] + h[2] + h[3], incl = own;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const long long y = __shfl_up(incl, o, 64);
                if (lane >= o) incl += y;
            }
            const long long excl = incl - own;
            if (excl <= kk && kk < incl) {
                long long acc = excl;
                int q = 0;
                for (; q < 3; ++q) {
                    if (acc + (long long)h[q] > kk) break;
                    acc += h[q];
                }
                L.k = kk - acc;
                L.prefix = pre | ((unsigned long long)(4 * lane + q) << shift);
            }
        }
        __syncthreads();
    }
    return L.prefix;
}

// Block min / max of the taken bit patterns (every thread gets them).
__device__ void block_minmax_bits(const unsigned long long (&b)[kSelPer], unsigned long long& lo,
                                  unsigned long long& hi, SelLds& L) {
    lo = ~0ull;
    hi = 0;
#pragma unroll
    for (int u = 0; u < kSelPer; ++u)
        if (b[u] != ~0ull) { lo = b[u] < lo ? b[u] : lo; hi = b[u] > hi ? b[u] : hi; }
    __syncthreads();
    if (threadIdx.x == 0) { L.minb = ~0ull; L.prefix = 0; }
    __syncthreads();
    atomicMin(&L.minb, lo);
    atomicMax(&L.prefix, hi);
    __syncthreads();
    lo = L.minb;
    hi = L.prefix;
    __syncthreads();
}

// np.percentile(x[take], pct), 'linear' (the host np_percentile's steps);
// nt = the number taken (> 0).  Register path when n fits kSelPer per thread.
template <class Get>
__device__ double block_percentile(long long n, long long nt, double pct, Get get, SelLds& L) {
    const double q = pct / 100.0;
    const double vi = (double)(nt - 1) * q;
    long long prev = (long long)floor(vi), next = prev + 1;
    if (vi >= (double)(nt - 1)) prev = next = nt - 1;
    if (vi < 0) prev = next = 0;
    const double gamma = vi - (vi >= (double)(nt - 1) ? -1.0 : (double)prev);
    double a, b;
    if (n <= (long long)kSelPer * blockDim.x) {
        unsigned long long v[kSelPer];
#pragma unroll
        for (int u = 0; u < kSelPer; ++u) {
            const long long i = threadIdx.x + (long long)u * blockDim.x;
            double x = 0.0;
            v[u] = (i < n && get(i, x)) ? (unsigned long long)__double_as_longlong(x) : ~0ull;
        }
        unsigned long long lo, hi;
        block_minmax_bits(v, lo, hi, L);
        const unsigned long long ab = block_kth_regs(v, prev, lo, hi, L);
        a = __longlong_as_double((long long)ab);
        b = a;
        if (next != prev) {
            unsigned c = 0;
            unsigned long long mn = ~0ull;
#pragma unroll
            for (int u = 0; u < kSelPer; ++u)
                if (v[u] != ~0ull) {
                    if (v[u] <= ab) ++c;
                    else mn = v[u] < mn ? v[u] : mn;
                }
            __syncthreads();
            if (threadIdx.x == 0) { L.cnt = 0; L.minb = ~0ull; }
            __syncthreads();
            atomicAdd(&L.cnt, c);
            atomicMin(&L.minb, mn);
            __syncthreads();
            b = (long long)L.cnt > next ? a : __longlong_as_double((long long)L.minb);
            __syncthreads();
        }
    } else {
        a = block_kth(n, prev, get, L);
        b = a;
        if (next != prev) {
            // the next order statistic: a again if more than `next` values are <= a, else the smallest value > a
            const unsigned long long ab = (unsigned long long)__double_as_longlong(a);
            if (threadIdx.x == 0) { L.cnt = 0; L.minb = ~0ull; }
            __syncthreads();
            for (long long i = threadIdx.x; i < n; i += blockDim.x) {
                double x;
                if (!get(i, x)) continue;
                const unsigned long long xb = (unsigned long long)__double_as_longlong(x);
                if (xb <= ab) atomicAdd(&L.cnt, 1u);
                else atomicMin(&L.minb, xb);
            }
            __syncthreads();
            b = (long long)L.cnt > next ? a : __longlong_as_double((long long)L.minb);
            __syncthreads();
        }
    }
    const double d = b - a;
    return gamma >= 0.5 ? b - d * (1.0 - gamma) : a + d * gamma;
}

// Gap_defined (:915-929) for MM (block 0) and PM (block 1) from their zero
// counts, and the gap rows compacted (gpos: position or -1, glist, ng).
// err bit 0: every coverage is zero (np.percentile of an empty array).
__device__ __forceinline__ void ts_gapdef_body(const long long* __restrict__ zeros, long long N,
                                               uint8_t* __restrict__ gap, int* __restrict__ gpos,
                                               int* __restrict__ glist, long long* __restrict__ ng,
                                               int* __restrict__ err, int m) {
    __shared__ SelLds L;
    __shared__ int wtot[16];
    const long long* z = zeros + (1 + m) * N;
    uint8_t* g = gap + m * N;
    int* gp = gpos + m * N;
    int* gl = glist + m * N;
    auto cov_of = [&](long long i) { return 1.0 - ((double)z[i] / (double)N); };
    auto get = [&](long long i, double& x) {
        x = cov_of(i);
        return x != 0.0;
    };
    if (threadIdx.x == 0) L.cnt = 0;
    __syncthreads();
    unsigned c = 0;
    for (long long i = threadIdx.x; i < N; i += blockDim.x) c += cov_of(i) != 0.0;
    atomicAdd(&L.cnt, c);
    __syncthreads();
    const long long nnz = L.cnt;
    double th = 0.0;
    if (nnz == 0) {
        if (threadIdx.x == 0) atomicOr(err, 1);
    } else {
        th = block_percentile(N, nnz, 25.0, get, L);
        if (th > 0.2) th = 0.2;
    }
    // flags and the ordered compaction
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    long long base = 0;
    for (long long i0 = 0; i0 < N; i0 += blockDim.x) {
        const long long i = i0 + threadIdx.x;
        const bool f = i < N && cov_of(i) < th;
        if (i < N) g[i] = f;
        const unsigned long long bm = __ballot(f);
        if (lane == 0) wtot[w] = __popcll(bm);
        __syncthreads();
        long long before = 0, tot = 0;
        for (int k = 0; k < nw; ++k) {
            if (k < w) before += wtot[k];
            tot += wtot[k];
        }
        if (i < N) {
            const long long pos = base + before + __popcll(bm & ((1ull << lane) - 1ull));
            gp[i] = f ? (int)pos : -1;
            if (f) gl[pos] = (int)i;
        }
        base += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) ng[m] = base;
}

__global__ __launch_bounds__(1024) void k_ts_gapdef(const long long* __restrict__ zeros, long long N,
                                                    uint8_t* __restrict__ gap, int* __restrict__ gpos,
                                                    int* __restrict__ glist, long long* __restrict__ ng,
                                                    int* __restrict__ err) {
    ts_gapdef_body(zeros, N, gap, gpos, glist, ng, err, blockIdx.x);
}

// alpha (:989-1005) over the union of MM's and PM's non-gap bins, and the
// exact raw totals of MM and PM.  err bit 1: every bin is a gap.
__device__ __forceinline__ void ts_alpha_body(const double* __restrict__ sum, const uint8_t* __restrict__ gap,
                                              long long N, double* __restrict__ alpha, double* __restrict__ raw,
                                              int* __restrict__ err) {
    __shared__ SelLds L;
    __shared__ double wmx[16];
    __shared__ long long wr[2][16];
    const double *sT = sum, *sM = sum + N, *sP = sum + 2 * N;
    const uint8_t *gm = gap, *gp = gap + N;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    double mx = -HUGE_VAL;
    long long t0 = 0, t1 = 0;
    unsigned nu = 0;
    for (long long i = threadIdx.x; i < N; i += blockDim.x) {
        const double a = (sM[i] + sP[i]) / (sT[i] + 1.0);
        alpha[i] = a;
        if (!gm[i] || !gp[i]) { mx = fmax(mx, a); ++nu; }
        t0 += (long long)sM[i];
        t1 += (long long)sP[i];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
    t0 = wave_sum_ll(t0);
    t1 = wave_sum_ll(t1);
    if (threadIdx.x == 0) L.cnt = 0;
    __syncthreads();
    atomicAdd(&L.cnt, nu);
    if (lane == 0) { wmx[w] = mx; wr[0][w] = t0; wr[1][w] = t1; }
    __syncthreads();
    mx = -HUGE_VAL;
    long long r0 = 0, r1 = 0;
    for (int k = 0; k < nw; ++k) { mx = fmax(mx, wmx[k]); r0 += wr[0][k]; r1 += wr[1][k]; }
    const long long nng = L.cnt;
    if (threadIdx.x == 0) {
        raw[0] = (double)r0;
        raw[1] = (double)r1;
        if (nng == 0) atomicOr(err, 2);
    }
    if (nng == 0) return;  // block-uniform
    for (long long i = threadIdx.x; i < N; i += blockDim.x) {
        double a = alpha[i] / mx;
        if (a == 0.0) a = 1.0;
        alpha[i] = a;
    }
    __syncthreads();
    auto get = [&](long long i, double& x) {
        x = alpha[i];
        return !gm[i] || !gp[i];
    };
    const double th = block_percentile(N, nng, 20.0, get, L);
    __syncthreads();
    for (long long i = threadIdx.x; i < N; i += blockDim.x)
        if (alpha[i] < th) alpha[i] = th;
}

__global__ __launch_bounds__(1024) void k_ts_alpha(const double* __restrict__ sum, const uint8_t* __restrict__ gap,
                                                   long long N, double* __restrict__ alpha, double* __restrict__ raw,
                                                   int* __restrict__ err) {
    ts_alpha_body(sum, gap, N, alpha, raw, err);
}

// the glue of many chromosomes in one launch each (hh_twostep_batch)
struct TsDesc {
    long long N;
    const long long* zeros;  // 3N: T, M, P
    const double* sum;       // 3N
    uint8_t* gap;            // 2N
    int* gpos;               // 2N
    int* glist;              // 2N
    long long* ng;           // 2
    double* alpha;           // N
    double* raw;             // 2
    int* err;
};
__global__ __launch_bounds__(1024) void k_ts_gapdef_b(const TsDesc* __restrict__ D) {
    const TsDesc d = D[blockIdx.x >> 1];
    ts_gapdef_body(d.zeros, d.N, d.gap, d.gpos, d.glist, d.ng, d.err, blockIdx.x & 1);
}
__global__ __launch_bounds__(1024) void k_ts_alpha_b(const TsDesc* __restrict__ D) {
    const TsDesc d = D[blockIdx.x];
    ts_alpha_body(d.sum, d.gap, d.N, d.alpha, d.raw, d.err);
}

// One symmetrisation chain (Trans2symmetry + Correct_VC + rescale of one
// haplotype matrix, the streaming passes of symvc_enqueue) as data: every
// chain's pass k runs in ONE launch, blocks [off[k][c], off[k][c + 1]) for
// chain c (hh_twostep_batch).  The same bodies with the same arguments as
// the per-chain launches: bitwise the same results.
struct SvDesc {
    const long long* X;
    const uint16_t* x16;  // the uint16 copy with escapes (k_rowstats_b), read unless *ovf
    const int* ovf;
    long long N, nrc, gcb, ncb, nb, ggrid, npairs, nT;
    int gr;
    const double* alpha;
    const uint8_t* gap;
    const int* gpos;
    const int* glist;
    const long long* ng_p;
    long long* xc;
    double *part_c, *part_r, *ccol, *sv, *rsv, *gpart1, *gpart2, *part, *tot;
    const double* rowsum_in;
    const double* raw_p;
    double* out;
};
enum { kSvGemv = 0, kSvGap, kSvColsum, kSvRows, kSvQ, kSvOut, kSvPhases };
constexpr int kSvOutPairs = 2;  // tile pairs per k_sv_out_b block

// pinned staging of hh_twostep_batch's pass descriptors (the thread's; idle
// again after each call's final synchronisation)
static void* ts_desc_stage(size_t bytes) {
    static thread_local void* p = nullptr;
    static thread_local size_t cap = 0;
    if (bytes > cap) {
        if (p) HIP_CHECK(hipHostFree(p));
        p = nullptr;
        cap = 0;
        const size_t want = std::max<size_t>(bytes, 1 << 20);
        HIP_CHECK(hipHostMalloc(&p, want, hipHostMallocDefault));
        cap = want;
    }
    return p;
}

__device__ __forceinline__ int sv_find(const long long* __restrict__ off, int nd, long long b) {
    int lo = 0, hi = nd - 1;  // the last chain with off[c] <= b
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (off[mid] <= b) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// the chain's matrix as its uint16 k_rowstats_b copy (0xFFFF entries from the
// int64 matrix) unless a value did not fit 32 bits; the same integers either
// way: bitwise the same doubles
__device__ __forceinline__ bool sv_narrow(const SvDesc& d) { return d.x16 && *d.ovf == 0; }

template <int MODE>
__global__ __launch_bounds__(256) void k_sv_gemv_b(const SvDesc* __restrict__ D, const long long* __restrict__ off,
                                                   int nd) {
    const int c = sv_find(off, nd, blockIdx.x);
    const SvDesc& d = D[c];
    const long long l = (long long)blockIdx.x - off[c];
    if (sv_narrow(d)) {
        if (MODE == 1)
            ts_gemv_body<uint32_t, 1, false, uint16_t>(d.x16, d.N, d.alpha, nullptr, d.gr, d.part_c, d.part_r, d.gpos,
                                                       (uint32_t*)d.xc, d.ng_p, l % d.nrc, l / d.nrc, d.X);
        else
            ts_gemv_body<uint32_t, 2, true, uint16_t>(d.x16, d.N, d.alpha, d.rsv, d.gr, d.part_c, d.part_r, nullptr,
                                                      nullptr, nullptr, l % d.nrc, l / d.nrc, d.X);
    } else {
        // (the rare wide chains: 2 rows per batch, so that their registers do
        // not set the kernel's -- the same rows in the same order)
        if (MODE == 1)
            ts_gemv_body<long long, 1, false, long long, 2>(d.X, d.N, d.alpha, nullptr, d.gr, d.part_c, d.part_r,
                                                            d.gpos, d.xc, d.ng_p, l % d.nrc, l / d.nrc);
        else
            ts_gemv_body<long long, 2, true, long long, 2>(d.X, d.N, d.alpha, d.rsv, d.gr, d.part_c, d.part_r,
                                                           nullptr, nullptr, nullptr, l % d.nrc, l / d.nrc);
    }
}
template <int MODE>
__global__ __launch_bounds__(256, 4) void k_sv_gap_b(const SvDesc* __restrict__ D, const long long* __restrict__ off,
                                                  int nd) {
    __shared__ GapLds S;
    const int c = sv_find(off, nd, blockIdx.x);
    const SvDesc& d = D[c];
    if (sv_narrow(d))
        ts_gap_body<uint32_t, MODE>(S, (const uint32_t*)d.xc, d.ng_p, d.glist, d.alpha, MODE == 2 ? d.sv : nullptr,
                                    MODE == 2 ? d.gpart2 : d.gpart1, (long long)blockIdx.x - off[c], d.ggrid);
    else
        ts_gap_body<long long, MODE>(S, d.xc, d.ng_p, d.glist, d.alpha, MODE == 2 ? d.sv : nullptr,
                                     MODE == 2 ? d.gpart2 : d.gpart1, (long long)blockIdx.x - off[c], d.ggrid);
}
__global__ __launch_bounds__(1024) void k_sv_colsum_b(const SvDesc* __restrict__ D, const long long* __restrict__ off,
                                                      int nd) {
    const int c = sv_find(off, nd, blockIdx.x);
    const SvDesc& d = D[c];
    ts_colsum_body(d.part_c, d.N, d.nrc, d.ccol, (long long)blockIdx.x - off[c]);
}
// (rows / q read only the diagonal of X: from the int64 matrix, the same
// integers as the copy)
__global__ __launch_bounds__(256) void k_sv_rows_b(const SvDesc* __restrict__ D, const long long* __restrict__ off,
                                                   int nd, double exponent) {
    const int c = sv_find(off, nd, blockIdx.x);
    const SvDesc& d = D[c];
    ts_rows_body<long long>(d.X, d.N, d.ncb, d.ccol, d.part_r, d.alpha, d.gpos, d.gpart1, d.ng_p, exponent,
                            d.rowsum_in, d.sv, d.rsv, (long long)blockIdx.x - off[c]);
}
__global__ __launch_bounds__(256) void k_sv_q_b(const SvDesc* __restrict__ D, const long long* __restrict__ off,
                                                int nd) {
    const int c = sv_find(off, nd, blockIdx.x);
    const SvDesc& d = D[c];
    ts_q_body<long long>(d.X, d.N, d.ncb, d.part_r, d.alpha, d.sv, d.gpart2, d.ng_p, d.part,
                         (long long)blockIdx.x - off[c]);
}
// k_slab_sum + k_symvc_scale of every chain (one block each; the same
// fixed-order sum and the same IEEE operations)
__global__ __launch_bounds__(256) void k_sv_fin_b(const SvDesc* __restrict__ D) {
    __shared__ double sh[16];
    const SvDesc& d = D[blockIdx.x];
    double acc = 0.0;
    for (long long k = threadIdx.x; k < d.nb; k += 256) acc += d.part[k];
    acc = block_sum(acc, sh);
    if (threadIdx.x == 0) {
        d.tot[0] = acc;
        const double nn = (double)d.N * (double)d.N;
        d.tot[1] = (*d.raw_p / nn) / (acc / nn);
    }
}
__global__ __launch_bounds__(256, 4) void k_sv_out_b(const SvDesc* __restrict__ D, const long long* __restrict__ off,
                                                  int nd) {
    __shared__ SvOutLds S;
    const int c = sv_find(off, nd, blockIdx.x);
    const SvDesc& d = D[c];
    SymArgs a{d.N, d.nT, d.alpha, d.gap, d.sv, 1.0};
    a.scale_p = d.tot + 1;
    a.ng_p = d.ng_p;
    // two consecutive tile pairs per block (kSvOutPairs)
    const long long p = kSvOutPairs * ((long long)blockIdx.x - off[c]);
    const int cnt = (int)std::min<long long>(kSvOutPairs, d.npairs - p);
    if (sv_narrow(d)) symvc_out_body<uint32_t, uint16_t>(S, d.x16, a, d.out, p, cnt, d.X);
    else symvc_out_body<long long>(S, d.X, a, d.out, p, cnt);
}


// Gap_defined (:915-929) from zero counts: cov = 1 - zeros / N.  cov is a
// non-increasing function of the integer zero count, so the percentile's two
// order statistics come from a count per zero count (O(N), no sort): the
// k-th smallest nonzero cov is cov(the k-th largest zero count among them),
// the same doubles as sorting the cov values.
static std::vector<uint8_t> gap_defined(const long long* zeros, long long N) {
    std::vector<double> cov(N);
    std::vector<long long> cnt(N + 1, 0);
    long long nnz = 0;
    for (long long i = 0; i < N; ++i) {
        cov[i] = 1.0 - ((double)zeros[i] / (double)N);
        HH_REQUIRE(zeros[i] >= 0 && zeros[i] <= N, "zero count out of range");
        if (cov[i] != 0.0) { ++cnt[zeros[i]]; ++nnz; }
    }
    HH_REQUIRE(nnz > 0, "percentile of an empty array");
    auto kth = [&](long long k) {  // k-th smallest (0-based) nonzero cov
        long long acc = 0;
        for (long long z = N; z >= 0; --z) {
            acc += cnt[z];
            if (acc > k) return 1.0 - ((double)z / (double)N);
        }
        return 1.0;
    };
    const double q = 25.0 / 100.0;
    const double vi = (double)(nnz - 1) * q;
    long long prev = (long long)std::floor(vi), next = prev + 1;
    if (vi >= (double)(nnz - 1)) prev = next = nnz - 1;
    const double gamma = vi - (vi >= (double)(nnz - 1) ? -1.0 : (double)prev);
    const double a = kth(prev), b = next == prev ? a : kth(next);
    const double d = b - a;
    double th = gamma >= 0.5 ? b - d * (1.0 - gamma) : a + d * gamma;  // np_percentile's lerp
    if (th > 0.2) th = 0.2;
    std::vector<uint8_t> g(N);
    for (long long i = 0; i < N; ++i) g[i] = cov[i] < th;
    return g;
}

// Dense N x N int64 from cells (row, col, count) with ids shifted by
// `offset` (pairs.dense_from_pixels / the reference's per-line dense `+=`
// result, matrixBuilding.py:554, :567-570, :1290-1301): out[r][c] += v, and
// out[c][r] += v (once on the diagonal) for an upper-triangle (symmetric)
// table.  Repeated cells add up, as the reference's `Matrix[bin1][bin2] += 1`
// does: int64 atomics, exact and independent of the order they land in
// (cooler's tables and the binner's run-length output are unique anyway).
__global__ void k_dense_scatter(const long long* __restrict__ r, const long long* __restrict__ c,
                                const long long* __restrict__ v, long long nnz, long long N, long long offset,
                                int sym, long long* __restrict__ out, unsigned long long* __restrict__ bad) {
    const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nnz) return;
    const long long a = r[k] - offset, b = c[k] - offset;
    if (a < 0 || b < 0 || a >= N || b >= N || (sym && a > b)) {
        atomicMin(bad, (unsigned long long)k);
        return;
    }
    const unsigned long long x = (unsigned long long)v[k];  // two's complement: the same add for int64
    atomicAdd((unsigned long long*)&out[a * N + b], x);
    if (sym && a != b) atomicAdd((unsigned long long*)&out[b * N + a], x);
}

// Upper-triangle nonzeros of a dense fp64 N x N matrix in row-major (cooler)
// order -- the np.triu(...).nonzero() table NPZ2Cooler writes for the
// corrected matrices (matrixBuilding.py:1613, :1628-1633).  PASS 0: per-row
// counts (one block per row); PASS 1: write at the scanned row offsets, the
// block's 256-wide chunks in order (ballot compaction keeps column order).
template <int PASS>
__global__ __launch_bounds__(256) void k_upper_nz(const double* __restrict__ X, long long N,
                                                  long long* __restrict__ cnt_or_off, int32_t* __restrict__ ob1,
                                                  int32_t* __restrict__ ob2, double* __restrict__ ov) {
    __shared__ long long wtot[4];
    __shared__ long long base_sh;
    const long long i = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const double* row = X + i * N;
    long long base = PASS ? cnt_or_off[i] : 0;
    for (long long j0 = i; j0 < N; j0 += 256) {
        const long long j = j0 + threadIdx.x;
        const double x = j < N ? row[j] : 0.0;
        const unsigned long long m = __ballot(x != 0.0);
        if (lane == 0) wtot[wave] = __popcll(m);
        __syncthreads();
        long long before = 0, tot = 0;
        for (int w = 0; w < 4; ++w) {
            if (w < wave) before += wtot[w];
            tot += wtot[w];
        }
        if (PASS == 1 && x != 0.0) {
            const long long pos = base + before + __popcll(m & ((1ull << lane) - 1ull));
            ob1[pos] = (int32_t)i;
            ob2[pos] = (int32_t)j;
            ov[pos] = x;
        }
        base += tot;
        __syncthreads();
    }
    if (PASS == 0 && threadIdx.x == 0) cnt_or_off[i] = base;
    (void)base_sh;
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
        {
            HH_KTIME("k_rowstats", s);
            if (dtype == 0)
                hipLaunchKernelGGL((k_rowstats<long long>), dim3((unsigned)N), dim3(256), 0, s, (const long long*)px,
                                   (long long)N, dlo.p, dhi.p, dsum.p, dz.p);
            else
                hipLaunchKernelGGL((k_rowstats<double>), dim3((unsigned)N), dim3(256), 0, s, (const double*)px,
                                   (long long)N, dlo.p, dhi.p, dsum.p, dz.p);
        }
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
        // the gap flags on the host too (the streaming passes list the gap rows there)
        std::vector<uint8_t> hg;
        if (gap) {
            hg.resize(N);
            if (on_device) {
                HIP_CHECK(hipMemcpyAsync(hg.data(), gap, N, hipMemcpyDeviceToHost, s));
                HIP_CHECK(hipStreamSynchronize(s));
            } else {
                std::copy(gap, gap + N, hg.begin());
            }
        }
        const uint8_t* hgp = gap ? hg.data() : nullptr;
        if (dtype == 0) symvc_run((const long long*)px, N, pa, pg, hgp, exponent, raw_sum, po, s);
        else symvc_run((const double*)px, N, pa, pg, hgp, exponent, raw_sum, po, s);
        if (!on_device) {
            HIP_CHECK(hipMemcpyAsync(out, po, bytes, hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
        }
    });
}

// TwoStepCorrection (matrixBuilding.py:984-1023) in one call: each matrix
// crosses PCIe once; gap / alpha glue on the host with NumPy semantics.
int hh_twostep(const int64_t* TM, const int64_t* MM, const int64_t* PM, int64_t N, double* nor_mm, double* nor_pm,
               uint8_t* gap_m, uint8_t* gap_p, int32_t on_device, void* stream) {
    return guard([&] {
        HH_REQUIRE(TM && MM && PM && nor_mm && nor_pm && gap_m && gap_p && N > 0, "bad arguments");
        if (on_device && g_symvc_stream && g_twostep_devglue && g_symvc_out) {
            // device matrices at the default chain: the shared-launch batch of
            // one chromosome (its uint16 copies read a quarter of the int64
            // bytes; bitwise this chain, test_twostep_gpu.py)
            const int64_t* t[1] = {TM};
            const int64_t* m[1] = {MM};
            const int64_t* q[1] = {PM};
            double* om[1] = {nor_mm};
            double* op[1] = {nor_pm};
            const int rc = hh_twostep_batch(1, t, m, q, &N, om, op, gap_m, gap_p, 0, stream);
            if (rc) HH_THROW(rc, std::string(hh_last_error()));
            return;
        }
        hipStream_t s = as_stream(stream);
        const size_t cnt = (size_t)N * N;
        const long long* src[3] = {(const long long*)TM, (const long long*)MM, (const long long*)PM};
        DBuf<long long> buf[3];
        const long long* d[3];
        for (int k = 0; k < 3; ++k) {
            if (on_device) {
                d[k] = src[k];
            } else {
                buf[k].alloc(cnt);
                buf[k].upload(src[k], cnt, s);
                d[k] = buf[k].p;
            }
        }
        // row sums (exact) and zero counts
        DBuf<double> dsum((size_t)3 * N);
        DBuf<long long> dz((size_t)3 * N);
        for (int k = 0; k < 3; ++k) {
            HH_KTIME("k_rowstats", s);
            hipLaunchKernelGGL((k_rowstats<long long>), dim3((unsigned)N), dim3(256), 0, s, d[k], (long long)N,
                               (const long long*)nullptr, (const long long*)nullptr, dsum.p + k * N, dz.p + k * N);
        }
        HIP_CHECK(hipGetLastError());
        PinnedStage& st = pinned_stage();
        if (g_symvc_stream && g_twostep_devglue) {
            // the glue on the device: no host round trip between the row
            // statistics and the corrections (one synchronisation at the end)
            DBuf<uint8_t> dgf((size_t)2 * N);
            DBuf<int> dgpos((size_t)2 * N), dglist((size_t)2 * N);
            DBuf<long long> dng(2);
            DBuf<double> dA(N), draw(2);
            DBuf<int> derr(1);
            HIP_CHECK(hipMemsetAsync(derr.p, 0, sizeof(int), s));
            hipLaunchKernelGGL(k_ts_gapdef, dim3(2), dim3(1024), 0, s, (const long long*)dz.p, (long long)N, dgf.p,
                               dgpos.p, dglist.p, dng.p, derr.p);
            hipLaunchKernelGGL(k_ts_alpha, dim3(1), dim3(1024), 0, s, (const double*)dsum.p, (const uint8_t*)dgf.p,
                               (long long)N, dA.p, draw.p, derr.p);
            HIP_CHECK(hipGetLastError());
            SymvcWs wm, wp;
            const GapIdx gim{dgpos.p, dglist.p, dng.p, N}, gip{dgpos.p + N, dglist.p + N, dng.p + 1, N};
            double* out_m = on_device ? nor_mm : (double*)buf[0].p;
            symvc_enqueue(d[1], N, dA.p, dgf.p, gim, 2.0 / 3.0, 0.0, draw.p, out_m, s, wm, dsum.p + N);
            if (!on_device) HIP_CHECK(hipMemcpyAsync(nor_mm, out_m, cnt * 8, hipMemcpyDeviceToHost, s));
            double* out_p = on_device ? nor_pm : (double*)buf[1].p;
            symvc_enqueue(d[2], N, dA.p, dgf.p + N, gip, 2.0 / 3.0, 0.0, draw.p + 1, out_p, s, wp, dsum.p + 2 * N);
            if (!on_device) HIP_CHECK(hipMemcpyAsync(nor_pm, out_p, cnt * 8, hipMemcpyDeviceToHost, s));
            char* dl = (char*)st.get(0, (size_t)2 * N + 16);
            dgf.download((uint8_t*)dl, (size_t)2 * N, s);
            derr.download((int*)(dl + (((size_t)2 * N + 7) & ~(size_t)7)), 1, s);
            HIP_CHECK(hipStreamSynchronize(s));
            const int e = *(int*)(dl + (((size_t)2 * N + 7) & ~(size_t)7));
            HH_REQUIRE(!(e & 1), "percentile of an empty array");
            HH_REQUIRE(!(e & 2), "every bin is a gap");
            std::memcpy(gap_m, dl, (size_t)N);
            std::memcpy(gap_p, dl + N, (size_t)N);
            return;
        }
        // row statistics down and the per-call vectors up through pinned
        // staging (DMA; pageable copies cost a staging pass each), the
        // vectors in one packed upload
        const size_t dl_bytes = (size_t)3 * N * (sizeof(double) + sizeof(long long));
        char* dl = (char*)st.get(0, dl_bytes);
        double* sum = (double*)dl;
        long long* zeros = (long long*)(dl + (size_t)3 * N * sizeof(double));
        dsum.download(sum, (size_t)3 * N, s);
        dz.download(zeros, (size_t)3 * N, s);
        HIP_CHECK(hipStreamSynchronize(s));
        const std::vector<uint8_t> gm = gap_defined(zeros + N, N), gp = gap_defined(zeros + 2 * N, N);
        // alpha over the union of non-gap bins (:994-1005)
        std::vector<double> alpha(N), ng;
        ng.reserve(N);
        for (long long i = 0; i < N; ++i) alpha[i] = (sum[N + i] + sum[2 * N + i]) / (sum[i] + 1.0);
        double mx = -std::numeric_limits<double>::infinity();
        for (long long i = 0; i < N; ++i)
            if (!gm[i] || !gp[i]) mx = std::max(mx, alpha[i]);
        HH_REQUIRE(mx > -std::numeric_limits<double>::infinity(), "every bin is a gap");
        for (long long i = 0; i < N; ++i) {
            alpha[i] /= mx;
            if (alpha[i] == 0.0) alpha[i] = 1.0;
        }
        for (long long i = 0; i < N; ++i)
            if (!gm[i] || !gp[i]) ng.push_back(alpha[i]);
        const double th = np_percentile(ng, 20.0);
        for (long long i = 0; i < N; ++i)
            if (alpha[i] < th) alpha[i] = th;
        std::vector<int> glm, gpm, glp, gpp;
        gap_index_host(gm.data(), N, glm, gpm);
        gap_index_host(gp.data(), N, glp, gpp);
        const bool any_m = !glm.empty(), any_p = !glp.empty();
        // exact integer totals (MM.mean() * N^2)
        double raw[2];
        for (int k = 0; k < 2; ++k) {
            long long t = 0;  // row sums are exact integers
            for (long long i = 0; i < N; ++i) t += (long long)sum[(k + 1) * N + i];
            raw[k] = (double)t;
        }
        // packed upload: ng_m, ng_p | alpha | gpos_m | glist_m | gpos_p | glist_p | gap_m | gap_p (16-B aligned)
        auto al = [](size_t b) { return (b + 15) & ~(size_t)15; };
        const size_t o_a = 16, o_gpm = o_a + al((size_t)N * 8), o_glm = o_gpm + al((size_t)N * 4),
                     o_gpp = o_glm + al(glm.size() * 4 + 4), o_glp = o_gpp + al((size_t)N * 4),
                     o_gm = o_glp + al(glp.size() * 4 + 4), o_gp = o_gm + al((size_t)N), up_bytes = o_gp + al((size_t)N);
        char* up = (char*)st.get(1, up_bytes);
        ((long long*)up)[0] = (long long)glm.size();
        ((long long*)up)[1] = (long long)glp.size();
        std::memcpy(up + o_a, alpha.data(), (size_t)N * 8);
        std::memcpy(up + o_gpm, gpm.data(), (size_t)N * 4);
        if (any_m) std::memcpy(up + o_glm, glm.data(), glm.size() * 4);
        std::memcpy(up + o_gpp, gpp.data(), (size_t)N * 4);
        if (any_p) std::memcpy(up + o_glp, glp.data(), glp.size() * 4);
        std::memcpy(up + o_gm, gm.data(), (size_t)N);
        std::memcpy(up + o_gp, gp.data(), (size_t)N);
        DBuf<char> dup(up_bytes);
        dup.upload(up, up_bytes, s);
        const double* dA = (const double*)(dup.p + o_a);
        const uint8_t *dgm = (const uint8_t*)(dup.p + o_gm), *dgp = (const uint8_t*)(dup.p + o_gp);
        const long long* dngs = (const long long*)dup.p;
        GapIdx gim{(const int*)(dup.p + o_gpm), (const int*)(dup.p + o_glm), dngs, (long long)glm.size()};
        GapIdx gip{(const int*)(dup.p + o_gpp), (const int*)(dup.p + o_glp), dngs + 1, (long long)glp.size()};
        // outputs: on the host path TM's buffer holds Nor_MM, then MM's holds
        // Nor_PM; both chains enqueued back to back, one synchronisation
        SymvcWs wm, wp;
        double* out_m = on_device ? nor_mm : (double*)buf[0].p;
        symvc_enqueue(d[1], N, dA, any_m ? dgm : nullptr, gim, 2.0 / 3.0, raw[0], (const double*)nullptr, out_m, s, wm,
                      dsum.p + N);
        if (!on_device) HIP_CHECK(hipMemcpyAsync(nor_mm, out_m, cnt * 8, hipMemcpyDeviceToHost, s));
        double* out_p = on_device ? nor_pm : (double*)buf[1].p;
        // (MM's buffer, read by the first chain, is written by the second: stream order)
        symvc_enqueue(d[2], N, dA, any_p ? dgp : nullptr, gip, 2.0 / 3.0, raw[1], (const double*)nullptr, out_p, s, wp,
                      dsum.p + 2 * N);
        if (!on_device) HIP_CHECK(hipMemcpyAsync(nor_pm, out_p, cnt * 8, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        std::copy(gm.begin(), gm.end(), gap_m);
        std::copy(gp.begin(), gp.end(), gap_p);
    });
}

// IntraChromMatrixCorrection (matrixBuilding.py:1026-1041) over a whole
// localRes set: every chromosome's chain (row statistics, the device glue, the
// two symmetrisation chains) enqueued at once, chromosomes largest first dealt
// to the least-loaded of n_streams streams (by N^2), one synchronisation at
// the end.  The small chromosomes' latency-bound launches run beside the big
// ones' streaming passes instead of after them.  Per chromosome the same
// kernels in the same order as hh_twostep: bitwise the same results.
extern "C++" {
namespace {
struct TsWork {
    DBuf<uint16_t> x16[2];  // MM / PM as uint16 with escapes (shared-launch mode)
    DBuf<double> dsum, dA, draw;
    DBuf<long long> dz, dng;
    DBuf<uint8_t> dgf;
    DBuf<int> dgpos, dglist;
    SymvcWs wm, wp;
};
// the side streams, per device (a stream belongs to the device current at
// its creation)
std::vector<hipStream_t>& ts_streams(int k) {
    static std::mutex mu;
    static std::map<int, std::vector<hipStream_t>> by_dev;
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    std::vector<hipStream_t>& v = by_dev[dev];
    while ((int)v.size() < k) {
        hipStream_t s;
        HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        v.push_back(s);
    }
    return v;
}
}  // namespace
}  // extern "C++"

// Waits for s0 and the side streams when a batch is left by an exception
// after its first launch: the buffers it hands back to the pool may still be
// in use by enqueued kernels (the pool's reuse rule: every entry point
// synchronises before returning).  Declared after the batch's buffers, so it
// runs before they are released.
struct TsSyncOnThrow {
    hipStream_t s0;
    std::vector<hipStream_t>* side;
    int nside;
    ~TsSyncOnThrow() {
        if (!std::uncaught_exceptions()) return;
        (void)hipStreamSynchronize(s0);
        for (int k = 0; side && k < nside; ++k) (void)hipStreamSynchronize((*side)[k]);
    }
};

// device bytes hh_twostep_batch allocates for one chromosome of N bins (its
// TsWork and two chains' SymvcWs), an upper bound
static size_t twostep_ws_bytes(int64_t N, bool narrow) {
    const double n = (double)N, gr = (double)g_symvc_rows;
    const double nbtm = std::ceil(n / kT), nrc = std::ceil(n / gr), ncb = std::ceil(n / kGW);
    double b = n * (3 * 8 + 3 * 8 + 2 + 2 * 4 + 2 * 4 + 8) + 64 + (narrow ? 2 * n * n * 2 : 0);
    b += 2 * (n * 8 * 3 + 16 + nrc * n * 8 + ncb * n * 8 + std::ceil(n / 256) * 8 + n * n * 8 + 2 * nbtm * n * 8);
    return (size_t)b + 64 * 512;  // + the pool's 512-byte rounding of ~60 buffers
}

static void twostep_batch_impl(int32_t n, const int64_t* const* TM, const int64_t* const* MM,
                               const int64_t* const* PM, const int64_t* N, double* const* nor_mm,
                               double* const* nor_pm, uint8_t* gap_m, uint8_t* gap_p, int32_t n_streams,
                               hipStream_t s0, int c_base);

int hh_twostep_batch(int32_t n, const int64_t* const* TM, const int64_t* const* MM, const int64_t* const* PM,
                     const int64_t* N, double* const* nor_mm, double* const* nor_pm, uint8_t* gap_m,
                     uint8_t* gap_p, int32_t n_streams, void* stream) {
    return guard([&] {
        HH_REQUIRE(n >= 0 && (n == 0 || (TM && MM && PM && N && nor_mm && nor_pm && gap_m && gap_p)), "bad arguments");
        HH_REQUIRE(n_streams >= 0 && n_streams <= 16, "n_streams in [0, 16]");
        HH_REQUIRE(g_symvc_stream && g_twostep_devglue, "hh_twostep_batch needs the streaming device-glue chain");
        if (n == 0) return;
        std::vector<int64_t> goff((size_t)n + 1, 0);
        for (int c = 0; c < n; ++c) {
            HH_REQUIRE(TM[c] && MM[c] && PM[c] && nor_mm[c] && nor_pm[c] && N[c] > 0, "bad chromosome arguments");
            goff[c + 1] = goff[c] + N[c];
        }
        hipStream_t s0 = as_stream(stream);
        // the workspace grows with the sum over chromosomes (a genome-wide
        // localRes set at 10 kb: ~100 GB beside its 190 GB of inputs and
        // outputs), so the chromosomes go in consecutive groups whose
        // workspace fits the budget: the free device memory plus what the
        // pool holds, less a margin (hh_tune twostep_budget_mb overrides).
        // A chromosome's results do not depend on its group (per-chain
        // descriptors, partials at fixed places): bitwise the same.
        const bool narrow = n_streams == 0;
        size_t budget = (size_t)g_twostep_budget;
        if (!budget) {
            size_t fr = 0, tot = 0;
            HIP_CHECK(hipMemGetInfo(&fr, &tot));
            size_t cached = 0;
            {
                std::lock_guard<std::mutex> lk(g_pool_mu);
                cached = g_pool_cached;
            }
            const size_t avail = fr + cached, margin = std::max<size_t>(size_t(2) << 30, tot / 32);
            budget = avail > margin ? avail - margin : 0;
        }
        for (int a = 0; a < n;) {
            int b = a + 1;
            size_t used = twostep_ws_bytes(N[a], narrow);
            while (b < n && used + twostep_ws_bytes(N[b], narrow) <= budget) used += twostep_ws_bytes(N[b++], narrow);
            twostep_batch_impl(b - a, TM + a, MM + a, PM + a, N + a, nor_mm + a, nor_pm + a, gap_m + goff[a],
                               gap_p + goff[a], n_streams, s0, a);
            a = b;
        }
    });
}

static void twostep_batch_impl(int32_t n, const int64_t* const* TM, const int64_t* const* MM,
                               const int64_t* const* PM, const int64_t* N, double* const* nor_mm,
                               double* const* nor_pm, uint8_t* gap_m, uint8_t* gap_p, int32_t n_streams,
                               hipStream_t s0, int c_base) {
    {
        std::vector<int64_t> goff((size_t)n + 1, 0);
        for (int c = 0; c < n; ++c) goff[c + 1] = goff[c] + N[c];
        std::vector<int> order(n);
        for (int c = 0; c < n; ++c) order[c] = c;
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return N[a] > N[b]; });
        const int K = std::max(1, std::min(n_streams, n));
        std::vector<hipStream_t>& ss = ts_streams(K);
        std::vector<double> load(K, 0.0);
        std::vector<int> sid(n);
        for (int c : order) {  // LPT on N^2 (the streaming passes' bytes)
            const int k = (int)(std::min_element(load.begin(), load.end()) - load.begin());
            sid[c] = k;
            load[k] += (double)N[c] * (double)N[c];
        }
        // every buffer before the first launch (the pool hands out nothing
        // a launched chain still uses), the error flags zeroed on s0
        std::vector<TsWork> w((size_t)n);
        DBuf<int> derr((size_t)n), dovf((size_t)2 * n);
        HIP_CHECK(hipMemsetAsync(derr.p, 0, sizeof(int) * n, s0));
        HIP_CHECK(hipMemsetAsync(dovf.p, 0, sizeof(int) * 2 * n, s0));
        // the shared passes read 32-bit copies of MM / PM (hg19 40 kb genome
        // 7.6 -> 7.0 ms; every pass on the copy beat the write pass on the
        // int64 matrix, 7.4 ms: profiles/r5l2/)
        const bool narrow = n_streams == 0;
        for (int c = 0; c < n; ++c) {
            const size_t Nc = (size_t)N[c];
            w[c].dsum.alloc(3 * Nc);
            w[c].dz.alloc(3 * Nc);
            w[c].dgf.alloc(2 * Nc);
            w[c].dgpos.alloc(2 * Nc);
            w[c].dglist.alloc(2 * Nc);
            w[c].dng.alloc(2);
            w[c].dA.alloc(Nc);
            w[c].draw.alloc(2);
            if (narrow)
                for (int h = 0; h < 2; ++h) w[c].x16[h].alloc(Nc * Nc);
        }
        // shared launches for the row statistics (every matrix's rows) and
        // the glue (every chromosome's gap flags, alpha, raw totals), then
        // each chromosome's two symmetrisation chains on the streams
        std::vector<RsDesc> rs((size_t)3 * n);
        std::vector<long long> row0((size_t)3 * n + 1, 0);
        std::vector<TsDesc> td((size_t)n);
        for (int c = 0; c < n; ++c) {
            TsWork& x = w[c];
            const long long* d[3] = {(const long long*)TM[c], (const long long*)MM[c], (const long long*)PM[c]};
            for (int k = 0; k < 3; ++k) {
                rs[3 * c + k] = RsDesc{d[k], N[c], x.dsum.p + k * N[c], x.dz.p + k * N[c],
                                       narrow && k ? x.x16[k - 1].p : nullptr, narrow && k ? dovf.p + 2 * c + k - 1 : nullptr};
                row0[3 * c + k + 1] = row0[3 * c + k] + N[c];
            }
            td[c] = TsDesc{N[c], x.dz.p, x.dsum.p, x.dgf.p, x.dgpos.p, x.dglist.p, x.dng.p, x.dA.p, x.draw.p,
                           derr.p + c};
        }
        HH_REQUIRE(row0.back() < (1LL << 31), "too many rows for one launch");
        const size_t b_rs = rs.size() * sizeof(RsDesc), b_r0 = row0.size() * 8, b_td = td.size() * sizeof(TsDesc);
        const size_t o_r0 = (b_rs + 15) & ~(size_t)15, o_td = o_r0 + ((b_r0 + 15) & ~(size_t)15);
        DBuf<char> ddesc(o_td + b_td);
        {
            char* up = (char*)pinned_stage().get(1, o_td + b_td);
            std::memcpy(up, rs.data(), b_rs);
            std::memcpy(up + o_r0, row0.data(), b_r0);
            std::memcpy(up + o_td, td.data(), b_td);
            ddesc.upload(up, o_td + b_td, s0);
        }
        // shared-launch mode: every chain's workspace, descriptors and checks
        // before the first launch (an allocation failure or a
        // failed check after it left kernels writing pool memory)
        const int nd = 2 * n;
        std::vector<SvDesc> sd;
        std::vector<long long> off;
        DBuf<char> dsv;
        size_t o_off = 0;
        TsSyncOnThrow sync_guard{s0, &ss, K};
        if (n_streams == 0) {
            // chain 2c = MM of chromosome c, 2c + 1 = PM, largest chromosomes first
            sd.resize((size_t)nd);
            off.assign((size_t)kSvPhases * (nd + 1), 0);
            const int gr = g_symvc_rows;
            int j = 0;
            for (int c : order) {
                TsWork& x = w[c];
                const long long Nc = N[c];
                for (int h = 0; h < 2; ++h, ++j) {
                    SymvcWs& ws = h ? x.wp : x.wm;
                    SvDesc d{};
                    d.X = (const long long*)(h ? PM[c] : MM[c]);
                    d.x16 = x.x16[h].p;
                    d.ovf = dovf.p + 2 * c + h;
                    d.N = Nc;
                    d.gr = gr;
                    d.nrc = (Nc + gr - 1) / gr;
                    d.gcb = (Nc + kGB - 1) / kGB;
                    d.ncb = (Nc + kGW - 1) / kGW;
                    d.nb = (Nc + 255) / 256;
                    d.nT = (Nc + kT - 1) / kT;
                    d.npairs = d.nT * (d.nT + 1) / 2;
                    const long long nbtm = (Nc + kT - 1) / kT;  // the gap count's bound: N (device count)
                    // (the gap passes grid-stride over the device gap count's
                    // tiles: 64 blocks per chain, not one per possible tile)
                    // (64 per chain for a genome -- more measured slower --, up to
                    // 1 024 for one chromosome, as its own launch would take)
                    const long long gcap = std::max<long long>(64, 2048 / nd);
                    d.ggrid = std::min<long long>(std::max<long long>(nbtm * nbtm, 1), gcap);
                    HH_REQUIRE(d.gcb < 65536 && d.npairs < (1LL << 31), "matrix too large");
                    ws.sv.alloc(Nc);
                    ws.tot.alloc(2);
                    ws.part_c.alloc((size_t)(d.nrc * Nc));
                    ws.part_r.alloc((size_t)(d.ncb * Nc));
                    ws.rsv.alloc(Nc);
                    ws.ccol.alloc(Nc);
                    ws.part.alloc((size_t)d.nb);
                    ws.xc.alloc((size_t)(Nc * Nc) * sizeof(long long));
                    ws.gpart1.alloc((size_t)(nbtm * Nc));
                    ws.gpart2.alloc((size_t)(nbtm * Nc));
                    d.alpha = x.dA.p;
                    d.gap = x.dgf.p + h * Nc;
                    d.gpos = x.dgpos.p + h * Nc;
                    d.glist = x.dglist.p + h * Nc;
                    d.ng_p = x.dng.p + h;
                    d.xc = (long long*)ws.xc.p;
                    d.part_c = ws.part_c.p, d.part_r = ws.part_r.p, d.ccol = ws.ccol.p, d.sv = ws.sv.p;
                    d.rsv = ws.rsv.p, d.gpart1 = ws.gpart1.p, d.gpart2 = ws.gpart2.p, d.part = ws.part.p;
                    d.tot = ws.tot.p;
                    d.rowsum_in = x.dsum.p + (1 + h) * Nc;
                    d.raw_p = x.draw.p + h;
                    d.out = h ? nor_pm[c] : nor_mm[c];
                    sd[j] = d;
                    const long long nblk[kSvPhases] = {d.nrc * d.gcb, d.ggrid,  (Nc + 63) / 64,
                                                       d.nb,         d.nb,
                                                       (d.npairs + kSvOutPairs - 1) / kSvOutPairs};
                    for (int k = 0; k < kSvPhases; ++k) off[(size_t)k * (nd + 1) + j + 1] = off[(size_t)k * (nd + 1) + j] + nblk[k];
                }
            }
            for (int k = 0; k < kSvPhases; ++k)
                HH_REQUIRE(off[(size_t)k * (nd + 1) + nd] < (1LL << 31), "too many blocks for one launch");
            const size_t b_sd = sd.size() * sizeof(SvDesc);
            o_off = (b_sd + 15) & ~(size_t)15;
            dsv.alloc(o_off + off.size() * 8);
            {
                // a staging buffer of its own (slot 0 takes the downloads
                // below): no host wait for the row statistics before the
                // passes are enqueued
                char* up = (char*)ts_desc_stage(o_off + off.size() * 8);
                std::memcpy(up, sd.data(), b_sd);
                std::memcpy(up + o_off, off.data(), off.size() * 8);
                dsv.upload(up, o_off + off.size() * 8, s0);
            }
        }
        hipLaunchKernelGGL(k_rowstats_b, dim3((unsigned)row0.back()), dim3(256), 0, s0, (const RsDesc*)ddesc.p,
                           (const long long*)(ddesc.p + o_r0), 3 * n);
        hipLaunchKernelGGL(k_ts_gapdef_b, dim3((unsigned)(2 * n)), dim3(1024), 0, s0,
                           (const TsDesc*)(ddesc.p + o_td));
        hipLaunchKernelGGL(k_ts_alpha_b, dim3((unsigned)n), dim3(1024), 0, s0, (const TsDesc*)(ddesc.p + o_td));
        HIP_CHECK(hipGetLastError());
        if (n_streams == 0) {
            const SvDesc* D = (const SvDesc*)dsv.p;
            auto O = [&](int k) { return (const long long*)(dsv.p + o_off) + (size_t)k * (nd + 1); };
            auto grid = [&](int k) { return dim3((unsigned)off[(size_t)k * (nd + 1) + nd]); };
            const double ex = 2.0 / 3.0;
            hipLaunchKernelGGL(k_sv_gemv_b<1>, grid(kSvGemv), dim3(256), 0, s0, D, O(kSvGemv), nd);
            hipLaunchKernelGGL(k_sv_gap_b<1>, grid(kSvGap), dim3(256), 0, s0, D, O(kSvGap), nd);
            hipLaunchKernelGGL(k_sv_colsum_b, grid(kSvColsum), dim3(1024), 0, s0, D, O(kSvColsum), nd);
            hipLaunchKernelGGL(k_sv_rows_b, grid(kSvRows), dim3(256), 0, s0, D, O(kSvRows), nd, ex);
            hipLaunchKernelGGL(k_sv_gap_b<2>, grid(kSvGap), dim3(256), 0, s0, D, O(kSvGap), nd);
            hipLaunchKernelGGL(k_sv_gemv_b<2>, grid(kSvGemv), dim3(256), 0, s0, D, O(kSvGemv), nd);
            hipLaunchKernelGGL(k_sv_q_b, grid(kSvQ), dim3(256), 0, s0, D, O(kSvQ), nd);
            hipLaunchKernelGGL(k_sv_fin_b, dim3((unsigned)nd), dim3(256), 0, s0, D);
            hipLaunchKernelGGL(k_sv_out_b, grid(kSvOut), dim3(256), 0, s0, D, O(kSvOut), nd);
            HIP_CHECK(hipGetLastError());
            const size_t gbytes = (size_t)2 * goff[n], ebytes = (size_t)n * sizeof(int);
            char* dl = (char*)pinned_stage().get(0, ((gbytes + 15) & ~(size_t)15) + ebytes);
            int* herr = (int*)(dl + ((gbytes + 15) & ~(size_t)15));
            for (int c = 0; c < n; ++c)
                HIP_CHECK(hipMemcpyAsync(dl + 2 * goff[c], w[c].dgf.p, (size_t)2 * N[c], hipMemcpyDeviceToHost, s0));
            derr.download(herr, (size_t)n, s0);
            HIP_CHECK(hipStreamSynchronize(s0));
            for (int c = 0; c < n; ++c) {
                HH_REQUIRE(!(herr[c] & 1), "percentile of an empty array (chromosome " + std::to_string(c_base + c) + ")");
                HH_REQUIRE(!(herr[c] & 2), "every bin is a gap (chromosome " + std::to_string(c_base + c) + ")");
                std::memcpy(gap_m + goff[c], dl + 2 * goff[c], (size_t)N[c]);
                std::memcpy(gap_p + goff[c], dl + 2 * goff[c] + N[c], (size_t)N[c]);
            }
            return;
        }
        hipEvent_t fork;
        HIP_CHECK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
        HIP_CHECK(hipEventRecord(fork, s0));
        for (int k = 0; k < K; ++k) HIP_CHECK(hipStreamWaitEvent(ss[k], fork, 0));
        const size_t gbytes = (size_t)2 * goff[n], ebytes = (size_t)n * sizeof(int);
        char* dl = (char*)pinned_stage().get(0, ((gbytes + 15) & ~(size_t)15) + ebytes);
        int* herr = (int*)(dl + ((gbytes + 15) & ~(size_t)15));
        for (int c : order) {
            hipStream_t s = ss[sid[c]];
            TsWork& x = w[c];
            const long long Nc = N[c];
            const long long* d[3] = {(const long long*)TM[c], (const long long*)MM[c], (const long long*)PM[c]};
            const GapIdx gim{x.dgpos.p, x.dglist.p, x.dng.p, Nc}, gip{x.dgpos.p + Nc, x.dglist.p + Nc, x.dng.p + 1, Nc};
            symvc_enqueue(d[1], Nc, x.dA.p, x.dgf.p, gim, 2.0 / 3.0, 0.0, x.draw.p, nor_mm[c], s, x.wm,
                          x.dsum.p + Nc);
            symvc_enqueue(d[2], Nc, x.dA.p, x.dgf.p + Nc, gip, 2.0 / 3.0, 0.0, x.draw.p + 1, nor_pm[c], s, x.wp,
                          x.dsum.p + 2 * Nc);
            HIP_CHECK(hipMemcpyAsync(dl + 2 * goff[c], x.dgf.p, (size_t)2 * Nc, hipMemcpyDeviceToHost, s));
        }
        for (int k = 0; k < K; ++k) {
            hipEvent_t j;
            HIP_CHECK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
            HIP_CHECK(hipEventRecord(j, ss[k]));
            HIP_CHECK(hipStreamWaitEvent(s0, j, 0));
            HIP_CHECK(hipEventDestroy(j));
        }
        HIP_CHECK(hipEventDestroy(fork));
        derr.download(herr, (size_t)n, s0);
        HIP_CHECK(hipStreamSynchronize(s0));
        for (int c = 0; c < n; ++c) {
            HH_REQUIRE(!(herr[c] & 1), "percentile of an empty array (chromosome " + std::to_string(c_base + c) + ")");
            HH_REQUIRE(!(herr[c] & 2), "every bin is a gap (chromosome " + std::to_string(c_base + c) + ")");
            std::memcpy(gap_m + goff[c], dl + 2 * goff[c], (size_t)N[c]);
            std::memcpy(gap_p + goff[c], dl + 2 * goff[c] + N[c], (size_t)N[c]);
        }
    }
}

int hh_dense_from_cells(const int64_t* row, const int64_t* col, const int64_t* count, int64_t nnz, int64_t N,
                        int64_t offset, int32_t symmetric, int32_t on_device, int64_t* out, void* stream) {
    return guard([&] {
        HH_REQUIRE(out && N > 0 && nnz >= 0 && (nnz == 0 || (row && col && count)), "bad arguments");
        hipStream_t s = as_stream(stream);
        DBuf<long long> buf[3];
        const long long* d[3] = {(const long long*)row, (const long long*)col, (const long long*)count};
        if (!on_device)
            for (int k = 0; k < 3; ++k) {
                buf[k].alloc(std::max<int64_t>(nnz, 1));
                buf[k].upload(d[k], nnz, s);
                d[k] = buf[k].p;
            }
        HIP_CHECK(hipMemsetAsync(out, 0, (size_t)N * N * sizeof(long long), s));
        DBuf<unsigned long long> bad(1);
        HIP_CHECK(hipMemsetAsync(bad.p, 0xff, sizeof(unsigned long long), s));
        if (nnz)
            hipLaunchKernelGGL(k_dense_scatter, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s, d[0], d[1], d[2],
                               (long long)nnz, (long long)N, (long long)offset, symmetric, (long long*)out, bad.p);
        HIP_CHECK(hipGetLastError());
        unsigned long long hb = 0;
        bad.download(&hb, 1, s);
        HIP_CHECK(hipStreamSynchronize(s));
        if (hb != ~0ull)
            HH_THROW(HH_ERR_ARG, std::string(symmetric ? "pixel " : "cell ") + std::to_string(hb) +
                                     " outside the matrix" + (symmetric ? " or below the diagonal" : ""));
    });
}

// two calls: the count (caller sizes device buffers), then the write (which
// recounts: one more read of X, ~80 us at N = 6 232, against a host round trip)
static void upper_offsets(const double* X, int64_t N, DBuf<long long>& off, unsigned long long* m, hipStream_t s) {
    DBuf<long long> cnt(N + 1);
    off.alloc(N + 1);
    HIP_CHECK(hipMemsetAsync(cnt.p + N, 0, sizeof(long long), s));
    hipLaunchKernelGGL(k_upper_nz<0>, dim3((unsigned)N), dim3(256), 0, s, X, (long long)N, cnt.p, (int32_t*)nullptr,
                       (int32_t*)nullptr, (double*)nullptr);
    DBuf<unsigned long long> tot(1);
    dev_excl_scan_i64(cnt.p, off.p, N + 1, tot.p, s);
    tot.download(m, 1, s);
    HIP_CHECK(hipStreamSynchronize(s));
}

int hh_dense_upper_count(const double* X, int64_t N, int64_t* nnz, void* stream) {
    return guard([&] {
        HH_REQUIRE(X && N > 0 && nnz, "bad arguments");
        DBuf<long long> off;
        unsigned long long m = 0;
        upper_offsets(X, N, off, &m, as_stream(stream));
        *nnz = (int64_t)m;
    });
}

int hh_dense_upper_write(const double* X, int64_t N, int32_t* bin1, int32_t* bin2, double* value, void* stream) {
    return guard([&] {
        HH_REQUIRE(X && N > 0 && bin1 && bin2 && value, "bad arguments");
        hipStream_t s = as_stream(stream);
        DBuf<long long> off;
        unsigned long long m = 0;
        upper_offsets(X, N, off, &m, s);
        hipLaunchKernelGGL(k_upper_nz<1>, dim3((unsigned)N), dim3(256), 0, s, X, (long long)N, off.p, bin1, bin2,
                           value);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipStreamSynchronize(s));
    });
}

}  // extern "C"
