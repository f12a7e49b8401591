// Sparse GenomeWideMatrixCorrection (matrixBuilding.py:857-901) for whole-
// genome diploid matrices too large for the reference's dense 2n x 2n NumPy
// arrays (10 kb diploid: 607 282^2 fp64 = 2.9 TB).  Inputs are the pixel
// tables HiCHap's matrix construction produces: the traditional whole-genome
// table T (cooler order: bin1 <= bin2, sorted, unique; n bins) and the
// imputed haplotype matrix H as ordered cells (row, col, count) sorted by
// (row, col) — H is asymmetric (R1/R2 imputation, :1290-1301) — on the
// 2n-bin layout M chromosomes then P chromosomes (:429-454).
//
//   hh_gw_create   validate, H row pointers, a radix sort of H's off-diagonal
//                  cells by column (column lists), and the exact integer row
//                  statistics the alpha step needs: T row sums / nonzeros
//                  within each chromosome's block (Tra_M, Gap_definedLowRes),
//                  H row sums within the same-chromosome same-haplotype block
//                  (M_M / P_P), sum(H)
//   (host glue)    alpha per chromosome with NumPy's percentile semantics
//                  (hichap_master_amd.matrixBuilding, as for the dense path)
//   hh_gw_correct  S = H / Alpha[:, None]; Y = Trans2symmetryLowRes(S) (Y_ij =
//                  S_ij + S_ji off the diagonal, :770-777) as an upper-triangle
//                  table: every (r, c >= r) of H's row plus every lower cell
//                  (i > r, r) without a partner, merged in column order by
//                  binary searches; Correct_VC(Y, 2/3) (:780-790) with the
//                  symmetric marginal rowsum(Y)_r = rowsum(S)_r +
//                  off-diagonal colsum(S)_r; mean rescale (:897-899).
// Every sum is a fixed-order reduction (integer ones exact): deterministic.
#include <algorithm>
#include <cmath>
#include <limits>
#include <memory>
#include <numeric>
#include <thread>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "ice_internal.hpp"

namespace hh {

template <class Id, class Cnt, bool COPY>
__global__ __launch_bounds__(256) void k_gw_check(const Id* __restrict__ r_in, const Id* __restrict__ c_in,
                                                  const Cnt* __restrict__ v_in, long long nnz, long long nb,
                                                  int upper, int32_t* __restrict__ R, int32_t* __restrict__ Cc,
                                                  uint32_t* __restrict__ V, unsigned long long* __restrict__ errs,
                                                  unsigned* __restrict__ vmax) {
    // grid-stride, one max atomic per block (one per wave was 23M same-address
    // atomics on a 1.5e9-cell table: 266 ms)
    unsigned mx = 0u;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nnz;
         i += (long long)gridDim.x * blockDim.x) {
        const long long a = (long long)r_in[i], b = (long long)c_in[i];
        const double v = (double)v_in[i];
        int code = 0;
        if (a < 0 || b < 0 || a >= nb || b >= nb) code = 1;
        else if (upper && a > b) code = 2;
        else if (i > 0) {
            const long long pa = (long long)r_in[i - 1], pb = (long long)c_in[i - 1];
            if (pa > a || (pa == a && pb > b)) code = 3;
            else if (pa == a && pb == b) code = 4;
        }
        if (!code && (!(v >= 0.0) || v != floor(v) || v >= 4294967296.0)) code = 5;
        if (code) {
            atomicMin(errs + code - 1, (unsigned long long)i);
            if (COPY) {
                R[i] = Cc[i] = 0;
                V[i] = 0u;
            }
        } else {
            mx = max(mx, (unsigned)v);
            if (COPY) {
                R[i] = (int32_t)a;
                Cc[i] = (int32_t)b;
                V[i] = (uint32_t)v;
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, (unsigned)__shfl_xor((int)mx, o, 64));
    __shared__ unsigned wm[4];
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        mx = max(max(wm[0], wm[1]), max(wm[2], wm[3]));
        if (mx) atomicMax(vmax, mx);
    }
}

// ptr[r] = first i with A[i] >= r, r in [0, nr] (A sorted)
__global__ void k_px_rowptr_gw(const int32_t* __restrict__ A, long long nnz, long long nr, long long* __restrict__ ptr) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > nnz) return;
    const long long lo = i == 0 ? -1 : (long long)A[i - 1];
    const long long hi = i == nnz ? nr : (long long)A[i];
    for (long long r = lo + 1; r <= hi; ++r) ptr[r] = i;
}

// the same from the high bits of sorted keys (n >= 1): kKpItems keys per
// thread loaded together (clamped), the previous key by a shuffle (a wave's
// first lane: a scalar load)
constexpr int kKpItems = 8;
__global__ __launch_bounds__(256) void k_px_keyptr_gw(const unsigned long long* __restrict__ keys, long long n, int ib,
                                                      long long nr, long long* __restrict__ ptr) {
    const long long base = (long long)blockIdx.x * (256 * kKpItems);
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    long long cur[kKpItems], prv[kKpItems];
#pragma unroll
    for (int q = 0; q < kKpItems; ++q) {
        const long long k = base + q * 256 + threadIdx.x;
        cur[q] = (long long)(keys[std::min(k, n - 1)] >> ib);
        prv[q] = (long long)(keys[std::min(std::max(base + q * 256 + wv * 64 - 1, 0LL), n - 1)] >> ib);
    }
#pragma unroll
    for (int q = 0; q < kKpItems; ++q) {
        const long long k = base + q * 256 + threadIdx.x;
        const long long up = __shfl_up(cur[q], 1, 64);
        if (k > n) continue;
        const long long lo = k == 0 ? -1 : (lane ? up : prv[q]);
        const long long hi = k == n ? nr : cur[q];
        for (long long r = lo + 1; r <= hi; ++r) ptr[r] = k;
    }
}

// Wave-segmented integer sums: lanes hold (key, val) with keys non-decreasing
// across the wave (a sorted table's rows); each key's segment sum goes out
// in one atomic from its last lane (was one same-address atomic per lane:
// 64-way serialised on a sorted table).  Integer sums: order-free, exact.
__device__ __forceinline__ void seg_add_u64(long long key, unsigned long long val, unsigned long long* __restrict__ out) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long vu = __shfl_up(val, o, 64);
        const long long ku = __shfl_up(key, o, 64);
        if (lane >= o && ku == key) val += vu;
    }
    const long long kd = __shfl_down(key, 1, 64);
    if ((lane == 63 || kd != key) && val) atomicAdd(out + key, val);
}

// Grid-stride kernels with a fixed grid: a block's scalar total is reduced
// once and added with one atomic per block.
constexpr int kGwStatBlocks = 2048;

// T row statistics within each chromosome block (both ends of an upper pixel,
// the diagonal once): exact integer sums / counts.  The table is sorted by
// bin1: the bin1 end is a segmented sum, the bin2 end an atomic per pixel
// (distinct columns within a wave).
// PACK: the bin2 end as ONE atomic per pixel, (count << 24) + 1 into rpk
// (the host splits it: sum in the high 40 bits, nonzeros in the low 24), and
// the table's count total in *total so the host can verify that no sum
// reached 2^40 (else it reruns unpacked).  Needs n_bins < 2^24.
// "same chromosome (block)" as a range test on the row's bounds [lo, hi):
// the row's bounds are one broadcast load per wave (rows change rarely along
// the sorted table) instead of a gather of the column's chromosome id
__device__ __forceinline__ bool in_block(int2 bd, int32_t y) { return y >= bd.x && y < bd.y; }

template <bool PACK>
__global__ __launch_bounds__(256) void k_gw_tstats(const int32_t* __restrict__ a, const int32_t* __restrict__ b,
                                                   const uint32_t* __restrict__ v, long long nnz,
                                                   const int2* __restrict__ cbd,
                                                   unsigned long long* __restrict__ rsum,
                                                   unsigned long long* __restrict__ rnz,
                                                   unsigned long long* __restrict__ rpk,
                                                   unsigned long long* __restrict__ total) {
    __shared__ unsigned long long wsum[4];
    const long long stride = (long long)gridDim.x * blockDim.x;
    const long long start = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long end = (nnz + 63) / 64 * 64;  // whole waves iterate together
    unsigned long long t = 0;
    for (long long i = start; i < end; i += stride) {
        long long x = 0x7fffffffLL;
        unsigned long long c = 0, one = 0;
        if (i < nnz) {
            x = a[i];
            const int32_t y = b[i];
            const uint32_t cc = v[i];
            if (PACK) t += cc;
            if (cc != 0u && in_block(cbd[x], y)) {
                c = cc;
                one = 1;
                if (x != y) {
                    if (PACK) {
                        atomicAdd(rpk + y, ((unsigned long long)cc << 24) | 1ull);
                    } else {
                        atomicAdd(rsum + y, (unsigned long long)cc);
                        atomicAdd(rnz + y, 1ull);
                    }
                }
            }
        }
        seg_add_u64(x, c, rsum);
        seg_add_u64(x, one, rnz);
    }
    if (PACK) {
        t = (unsigned long long)wave_sum_ll((long long)t);
        if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = t;
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned long long bt = wsum[0] + wsum[1] + wsum[2] + wsum[3];
            if (bt) atomicAdd(total, bt);
        }
    }
}

// The packed form (PACK above) with the bin2 end privatised in LDS: a block
// takes a contiguous run of the table (rows x0 .. x1, sorted) and adds the
// column end of every pixel with bin2 < x0 + kTsWin to an LDS window (the
// near-diagonal bulk of a cis table: contact counts decay with distance),
// the rest to global memory; the window goes out as one atomic per nonzero
// column at the end.  The row end goes into the same packed counters
// (segmented, one atomic per row run).  1.5e9 same-address-free but
// one-per-pixel global atomics were the whole 17.7 ms of k_gw_tstats at
// 10 kb whole genome.  Integer sums: exact, order-free.
//
// Round 4: a block walks its run in chunks of 256 x IT pixels, each thread's
// IT pixels loaded together from clamped addresses (the per-pixel
// `if (i < p1)` loads were one memory round trip each, 1.1 TB/s); a chunk
// whose first and last pixel share a row (the common case: ~5 000 pixels
// per row at 10 kb) sums its row end in registers, one wave reduction and
// one atomic per wave, instead of a segmented scan per pixel.
constexpr int kTsWin = 8192;
// entries per thread per chunk (a template parameter: T 16, H 8 measured)
constexpr int kStItemsT = 8, kStItemsH = 8;

// CHECK: the statistics kernels also validate their table (k_gw_check's
// rules and codes: range, upper triangle, (row, col) order, duplicates,
// negative counts; first offending entry per code), so an int32 device table
// is read once instead of twice.  Every address they form is clamped to the
// table's ids, so invalid input yields garbage statistics but no stray
// access, and gw_create throws before using them.  The previous entry of a
// wave's first lane is a scalar load (wave-uniform address).
__device__ __forceinline__ int gw_code(int32_t x, int32_t y, uint32_t cnt, int32_t px, int32_t py, bool has_prev,
                                       long long nb, bool upper) {
    if (x < 0 || y < 0 || x >= nb || y >= nb) return 1;
    if (upper && x > y) return 2;
    if (has_prev) {
        if (px > x || (px == x && py > y)) return 3;
        if (px == x && py == y) return 4;
    }
    return (int32_t)cnt < 0 ? 5 : 0;
}

struct StCheck {
    unsigned long long* errs;  // 5 codes: first offending entry (atomicMin)
    unsigned* vmax;            // largest count (H only), or nullptr
    long long* hptr;           // H row pointers (nb + 1), or nullptr
};

// Loads one chunk: each thread's kStItems entries (clamped to `last`) and,
// with CHECK, validates the ones inside the run.  Returns the thread's
// largest count seen (CHECK).
template <int IT, bool CHECK>
__device__ __forceinline__ unsigned st_load(const int32_t* __restrict__ a, const int32_t* __restrict__ b,
                                            const uint32_t* __restrict__ v, long long c0, long long last, long long nb,
                                            bool upper, int32_t* xs, int32_t* ys, uint32_t* cs, StCheck ck,
                                            int32_t* pxs) {
    int32_t pys[IT];
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const long long i = std::min(c0 + k * 256 + threadIdx.x, last);
        xs[k] = a[i];
        ys[k] = b[i];
        cs[k] = v[i];
        if (CHECK) {
            const long long j = std::min(std::max(c0 + k * 256 + wv * 64 - 1, 0LL), last);
            pxs[k] = a[j];
            pys[k] = b[j];
        }
    }
    unsigned mx = 0u;
    if (CHECK) {
        const int lane = threadIdx.x & 63;
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const long long i = c0 + k * 256 + threadIdx.x;
            const int32_t upx = __shfl_up(xs[k], 1, 64), upy = __shfl_up(ys[k], 1, 64);
            const int32_t px = lane ? upx : pxs[k], py = lane ? upy : pys[k];
            const int code = i <= last ? gw_code(xs[k], ys[k], cs[k], px, py, i > 0, nb, upper) : 0;
            if (code) atomicMin(ck.errs + code - 1, (unsigned long long)i);
            else if (i <= last) mx = max(mx, cs[k]);
        }
    }
#pragma unroll
    for (int k = 0; k < IT; ++k)  // past the run: count 0 (clamped duplicates of the last entry)
        cs[k] &= 0u - (uint32_t)(c0 + k * 256 + threadIdx.x <= last);
    return mx;
}

__device__ __forceinline__ int32_t clamp_id(int32_t x, long long nb) {
    return (int32_t)std::min<long long>(std::max<int32_t>(x, 0), nb - 1);
}
__device__ __forceinline__ bool ok_id(int32_t x, long long nb) { return x >= 0 && x < nb; }

template <int IT, bool CHECK>
__global__ __launch_bounds__(256) void k_gw_tstats_win(const int32_t* __restrict__ a, const int32_t* __restrict__ b,
                                                       const uint32_t* __restrict__ v, long long nnz, long long per,
                                                       long long n, const int2* __restrict__ cbd,
                                                       unsigned long long* __restrict__ rpk,
                                                       unsigned long long* __restrict__ total, StCheck ck,
                                                       int wsz) {
    extern __shared__ unsigned long long win[];  // wsz entries (kTsWin unless HH_GW_TSWIN)
    __shared__ unsigned long long wsum[4];
    const long long p0 = (long long)blockIdx.x * per;
    if (p0 >= nnz) return;  // block-uniform
    const long long p1 = std::min(nnz, p0 + per);
    const long long x0 = a[p0];
    for (int c = threadIdx.x; c < wsz; c += 256) win[c] = 0ull;
    __syncthreads();
    unsigned long long t = 0;
    for (long long c0 = p0; c0 < p1; c0 += (256 * IT)) {
        const long long last = std::min(c0 + (256 * IT), p1) - 1;
        const int32_t xf = a[c0], xl = a[last];
        int32_t xs[IT], ys[IT];
        uint32_t cs[IT];
        int32_t pxs[IT];
        st_load<IT, CHECK>(a, b, v, c0, last, n, true, xs, ys, cs, ck, pxs);
        if (xf == xl) {
            const bool okx = ok_id(xf, n);
            const int2 bd = cbd[clamp_id(xf, n)];
            unsigned long long racc = 0;
#pragma unroll
            for (int k = 0; k < IT; ++k) {
                const uint32_t cc = cs[k];
                const int32_t y = ys[k];
                t += cc;
                if (cc != 0u && in_block(bd, y)) {
                    const unsigned long long pk = ((unsigned long long)cc << 24) | 1ull;
                    racc += pk;
                    if (xf != y) {
                        const long long d = (long long)y - x0;
                        if (d >= 0 && d < wsz) atomicAdd(&win[d], pk);
                        else atomicAdd(rpk + y, pk);
                    }
                }
            }
            racc = (unsigned long long)wave_sum_ll((long long)racc);
            if ((threadIdx.x & 63) == 0 && racc && okx) atomicAdd(rpk + xf, racc);
        } else {
            int2 bds[IT];
#pragma unroll
            for (int k = 0; k < IT; ++k) bds[k] = cbd[clamp_id(xs[k], n)];
#pragma unroll
            for (int k = 0; k < IT; ++k) {
                const uint32_t cc = cs[k];
                const int32_t x = xs[k], y = ys[k];
                t += cc;
                unsigned long long pk = 0;
                if (cc != 0u && ok_id(x, n) && in_block(bds[k], y)) {
                    pk = ((unsigned long long)cc << 24) | 1ull;
                    if (x != y) {
                        const long long d = (long long)y - x0;
                        if (d >= 0 && d < wsz) atomicAdd(&win[d], pk);
                        else atomicAdd(rpk + y, pk);
                    }
                }
                seg_add_u64(x, pk, rpk);  // rows non-decreasing across the wave (clamped lanes: pk 0)
            }
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < wsz; c += 256) {
        const unsigned long long w = win[c];
        if (w && x0 + c < n) atomicAdd(rpk + x0 + c, w);
    }
    t = (unsigned long long)wave_sum_ll((long long)t);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long bt = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        if (bt) atomicAdd(total, bt);
    }
}

// H row sums within the same-chromosome same-haplotype block (H sorted by
// row: segmented), and sum(H).  A block walks a contiguous run in chunks as
// k_gw_tstats_win does (batched clamped loads; a one-row chunk sums in
// registers).  CHECK: validates H too and records its largest count.
template <int IT, bool CHECK>
__global__ __launch_bounds__(256) void k_gw_hstats(const int32_t* __restrict__ r, const int32_t* __restrict__ c,
                                                   const uint32_t* __restrict__ v, long long nnz, long long per,
                                                   long long nb, const int2* __restrict__ bbd,
                                                   unsigned long long* __restrict__ bsum,
                                                   unsigned long long* __restrict__ total, StCheck ck) {
    __shared__ unsigned long long wsum[4];
    __shared__ unsigned wmx[4];
    const long long p0 = (long long)blockIdx.x * per;
    if (p0 >= nnz) return;  // block-uniform
    const long long p1 = std::min(nnz, p0 + per);
    unsigned long long t = 0;
    unsigned mx = 0u;
    for (long long c0 = p0; c0 < p1; c0 += (256 * IT)) {
        const long long last = std::min(c0 + (256 * IT), p1) - 1;
        const int32_t xf = r[c0], xl = r[last];
        int32_t xs[IT], ys[IT];
        uint32_t cs[IT];
        int32_t pxs[IT];
        mx = max(mx, st_load<IT, CHECK>(r, c, v, c0, last, nb, false, xs, ys, cs, ck, pxs));
        if (CHECK) {  // H row pointers (k_px_rowptr_gw's rule): ptr[q] = first entry with row >= q
            const int lane = threadIdx.x & 63;
#pragma unroll
            for (int k = 0; k < IT; ++k) {
                const long long i = c0 + k * 256 + threadIdx.x;
                const int32_t up = __shfl_up(xs[k], 1, 64);
                const long long prev = i == 0 ? -1 : (long long)(lane ? up : pxs[k]);
                const long long cur = xs[k];
                if (i <= last && prev < cur && cur < nb) {
                    for (long long q = std::max(prev + 1, 0LL); q <= cur; ++q) ck.hptr[q] = i;
                }
                if (i == nnz - 1 && cur >= 0 && cur < nb)
                    for (long long q = cur + 1; q <= nb; ++q) ck.hptr[q] = nnz;
            }
        }
        if (xf == xl) {
            const int2 bd = bbd[clamp_id(xf, nb)];
            unsigned long long racc = 0;
#pragma unroll
            for (int k = 0; k < IT; ++k) {
                t += cs[k];
                racc += in_block(bd, ys[k]) ? (unsigned long long)cs[k] : 0ull;
            }
            racc = (unsigned long long)wave_sum_ll((long long)racc);
            if ((threadIdx.x & 63) == 0 && racc && ok_id(xf, nb)) atomicAdd(bsum + xf, racc);
        } else {
            int2 bds[IT];
#pragma unroll
            for (int k = 0; k < IT; ++k) bds[k] = bbd[clamp_id(xs[k], nb)];
#pragma unroll
            for (int k = 0; k < IT; ++k) {
                t += cs[k];
                seg_add_u64(xs[k], ok_id(xs[k], nb) && in_block(bds[k], ys[k]) ? (unsigned long long)cs[k] : 0ull,
                            bsum);
            }
        }
    }
    t = (unsigned long long)wave_sum_ll((long long)t);
    if (CHECK) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mx = max(mx, (unsigned)__shfl_xor((int)mx, o, 64));
    }
    if ((threadIdx.x & 63) == 0) {
        wsum[threadIdx.x >> 6] = t;
        wmx[threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long bt = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        if (bt) atomicAdd(total, bt);
        if (CHECK && ck.vmax) {
            const unsigned m = max(max(wmx[0], wmx[1]), max(wmx[2], wmx[3]));
            if (m) atomicMax(ck.vmax, m);
        }
    }
}

// Column lists: H's off-diagonal cells keyed by column and sorted stably by
// the column bits (dev_sort_cells_by_col, pairs.hip; keys formed in its first
// radix pass).  FMT 1 (ids < 2^20, counts < 2^24): the key IS the packed
// cell, col << 44 | row << 24 | count (no index, no gather afterwards).
// FMT 0: col << ib | index, then k_gw_pack.
// column-list entry -> (row, count): FMT 0 row | count << 32 (after
// k_gw_pack), FMT 1 the packed sort key col << 44 | row << 24 | count
template <int FMT>
__device__ __forceinline__ int32_t lrv_row(unsigned long long x) {
    return FMT ? (int32_t)((x >> 24) & 0xFFFFFull) : (int32_t)(uint32_t)x;
}
template <int FMT>
__device__ __forceinline__ double lrv_val(unsigned long long x) {
    return FMT ? (double)(uint32_t)(x & 0xFFFFFFull) : (double)(uint32_t)(x >> 32);
}

__device__ __forceinline__ long long lower_bound_i32(const int32_t* a, long long lo, long long hi, int32_t x) {
    while (lo < hi) {
        const long long mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
// first position in [lo, hi) of the column list whose cell row >= x
template <int FMT>
__device__ __forceinline__ long long lower_bound_keyrow(const unsigned long long* lrv, long long lo, long long hi,
                                                        int32_t x) {
    while (lo < hi) {
        const long long mid = (lo + hi) >> 1;
        if (lrv_row<FMT>(lrv[mid]) < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// The column-sorted keys replaced, in place and once, by their cells' (row,
// count) packed as row | count << 32 (the column is the list segment,
// cptr): the kernels below used to gather R[k] and V[k] at random through
// the keys, each of them again.
__global__ void k_gw_pack(unsigned long long* __restrict__ keys, long long n, unsigned long long imask,
                          const int32_t* __restrict__ R, const uint32_t* __restrict__ V) {
    const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const long long k = (long long)(keys[q] & imask);
    keys[q] = (unsigned long long)(uint32_t)R[k] | ((unsigned long long)V[k] << 32);
}

struct GwDev {
    const int32_t* R;
    const int32_t* C;
    const uint32_t* V;
    const long long* hptr;      // N2 + 1 row pointers of H
    const unsigned long long* lrv;   // off-diagonal cells sorted by (col, row): (row, count) packed
    const long long* cptr;      // N2 + 1 column-list pointers
    long long N2;
    const double* alpha;        // N2
    long long* ustart;          // per row: first cell with col >= row
    long long* lstart;          // per column r: first list entry with row > r
};

// per row r (one wave): rowsum(S)_r and the off-diagonal column sum of S in
// column r, in list order (fixed xor-tree per chunk): the symmetric marginal
// of Y; u/l starts for the merge.  Round 4: kMargWin windows of 64 per step,
// their loads issued together from clamped addresses (out-of-row lanes
// weighted 0: the same per-window sums in the same order), and the starts
// counted on the way (cells left of the diagonal, list rows <= r) instead of
// two serial binary searches by lane 0 (~25 dependent loads per row).
constexpr int kMargWin = 4;
template <int FMT>
__global__ __launch_bounds__(256) void k_gw_marg(GwDev g, double exponent, double* __restrict__ s_out) {
    const long long r = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (r >= g.N2) return;
    const int lane = threadIdx.x & 63;
    const long long h0 = g.hptr[r], h1 = g.hptr[r + 1];
    double acc = 0.0;
    const double ar = g.alpha[r];
    long long nlo = 0;
    for (long long q0 = h0; q0 < h1; q0 += 64 * kMargWin) {
        uint32_t vv[kMargWin];
        int32_t cc[kMargWin];
#pragma unroll
        for (int u = 0; u < kMargWin; ++u) {
            const long long q = std::min(q0 + u * 64 + lane, h1 - 1);
            vv[u] = g.V[q];
            cc[u] = g.C[q];
        }
#pragma unroll
        for (int u = 0; u < kMargWin; ++u) {
            const bool in = q0 + u * 64 + lane < h1;
            acc += wave_sum((double)vv[u] / ar * (in ? 1.0 : 0.0));
            nlo += __popcll(__ballot(in & (cc[u] < (int32_t)r)));
        }
    }
    const long long c0 = g.cptr[r], c1 = g.cptr[r + 1];
    double acc2 = 0.0;
    long long nle = 0;
    for (long long q0 = c0; q0 < c1; q0 += 64 * kMargWin) {
        unsigned long long e[kMargWin];
        double al[kMargWin];
#pragma unroll
        for (int u = 0; u < kMargWin; ++u) e[u] = g.lrv[std::min(q0 + u * 64 + lane, c1 - 1)];
#pragma unroll
        for (int u = 0; u < kMargWin; ++u) al[u] = g.alpha[lrv_row<FMT>(e[u])];
#pragma unroll
        for (int u = 0; u < kMargWin; ++u) {
            const bool in = q0 + u * 64 + lane < c1;
            acc2 += wave_sum(lrv_val<FMT>(e[u]) / al[u] * (in ? 1.0 : 0.0));
            nle += __popcll(__ballot(in & (lrv_row<FMT>(e[u]) <= (int32_t)r)));
        }
    }
    if (lane == 0) {
        const double m = acc + acc2;
        double sv = pow(m, exponent);
        if (sv == 0.0) sv = 1.0;
        s_out[r] = sv;
        g.ustart[r] = h0 + nlo;  // first cell with col >= r (the row is sorted)
        g.lstart[r] = c0 + nle;  // first list entry with row > r
    }
}

// Row r of the corrected upper table, by a wave-level merge of two sorted
// lists: A = H's cells (r, c >= r) (columns ascending) and B = the cells
// (i, r), i > r, of column r's list (rows ascending; their transposes land
// in row r).  The output row is the union by column: Y = S_rc + S_cr where
// both exist (Trans2symmetryLowRes, :770-777), else the one present; C =
// Y / (s_c s_r) (Correct_VC, :780-790).  Per window of 64 elements of each
// list, lane l finds by merge path how many of the first l + 1 merged
// elements come from A (ties: A first, so a B element directly follows its
// A partner); 63 merged elements are consumed per window (64 when element
// 62 and its partner 63 form a pair), a B element tied to the preceding A
// element is absorbed.  PASS 0: per row the union's length and its share of
// sum(C) over the full symmetric matrix (row order, fixed tree); PASS 1:
// write (r, c, rf C) at the row's offset.  O(|A| + |B|) with coalesced
// loads (was a binary search per element in three kernels plus two flag /
// prefix arrays over every column-list entry).
constexpr int kMergeInf = 0x7fffffff;
template <int FMT, int PASS>
__global__ __launch_bounds__(256) void k_gw_merge(GwDev g, const double* __restrict__ s, double rf,
                                                  long long* __restrict__ len_or_off, double* __restrict__ rowc,
                                                  int32_t* __restrict__ ob1, int32_t* __restrict__ ob2,
                                                  double* __restrict__ ov) {
    const long long r = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (r >= g.N2) return;
    const int lane = threadIdx.x & 63;
    long long ia = g.ustart[r];
    const long long a1 = g.hptr[r + 1];
    long long ib = g.lstart[r];
    const long long b1 = g.cptr[r + 1];
    const double ar = g.alpha[r], sr = s[r];
    long long pos = PASS ? len_or_off[r] : 0;
    double csum = 0.0;
    __shared__ int slot_k[4][64];
    __shared__ double slot_v[4][64];
    const int wv = threadIdx.x >> 6;
    // Software-pipelined windows: the raw cells of the current window (cur)
    // and of the 64 after it (nxt) are in registers; a window's consumption
    // (<= 64 of each list) shifts cur / nxt by shuffles, and the loads of the
    // following 64 are issued at the end of the window, one window ahead of
    // use.  Loads from clamped addresses (the row's last cell; its values on
    // padding lanes are never used: their keys are +inf).  Measured
    // (rocprof SQ counters): the one-window-at-a-time loop spent ~77 % of its
    // wave cycles parked on s_waitcnt (three dependent round trips per window:
    // cells, alpha, s); now two.
    const long long aq = std::max(a1 - 1, 0LL), bq = std::max(b1 - 1, 0LL);
    int32_t ca = 0, na = 0;
    uint32_t cva = 0u, nva = 0u;
    unsigned long long ce = 0ull, ne = 0ull;
    if (ia < a1 || ib < b1) {  // (an empty row of an empty table has no cell to clamp to)
        ca = g.C[std::min(ia + lane, aq)];
        cva = g.V[std::min(ia + lane, aq)];
        ce = g.lrv[std::min(ib + lane, bq)];
        na = g.C[std::min(ia + 64 + lane, aq)];
        nva = g.V[std::min(ia + 64 + lane, aq)];
        ne = g.lrv[std::min(ib + 64 + lane, bq)];
    }
    while (ia < a1 || ib < b1) {
        // windows (padded with +inf keys)
        const bool ina = ia + lane < a1, inb = ib + lane < b1;
        const int ka = ina ? ca : kMergeInf;
        const int32_t kb_raw = lrv_row<FMT>(ce);
        const int kb = inb ? kb_raw : kMergeInf;
        const double alb = g.alpha[inb ? kb_raw : 0];
        const double va = (double)cva / ar;
        const double vb = lrv_val<FMT>(ce) / alb;
        // merged position of every element (ties: A first, so a B element
        // directly follows its A partner): A[l] at l + #(B < A[l]), B[l] at
        // l + #(A <= B[l]), each count a branch-free 64-entry binary search
        // over the other (sorted, +inf padded) window; the elements land in
        // the wave's LDS slots and lane l reads merged element l.  (Round 3's
        // per-lane merge-path search over both windows was ~170 of the
        // window's ~350 instructions: the kernel was VALU-bound.)
        int pa = 0, pb = 0;
#pragma unroll
        for (int st = 32; st >= 1; st >>= 1) {
            const int qb = __shfl(kb, pa + st - 1, 64);
            const int qa = __shfl(ka, pb + st - 1, 64);
            pa += qb < ka ? st : 0;
            pb += qa <= kb ? st : 0;
        }
        const int kb63 = __shfl(kb, 63, 64), ka63 = __shfl(ka, 63, 64);
        pa += (pa == 63 && kb63 < ka) ? 1 : 0;
        pb += (pb == 63 && ka63 <= kb) ? 1 : 0;
        const int posA = lane + pa, posB = lane + pb;
        if (posA < 64) {
            slot_k[wv][posA] = ka;
            slot_v[wv][posA] = va;
        }
        if (posB < 64) {
            slot_k[wv][posB] = kb | (int)0x80000000;  // high bit: from B (keys < 2^31)
            slot_v[wv][posB] = vb;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int kraw = slot_k[wv][lane];
        const bool fromA = kraw >= 0;
        const int key = kraw & 0x7fffffff;
        const double val = slot_v[wv][lane];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // the slots are rewritten next window
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // the next merged element (tie partner?)
        const int key_n = __shfl_down(key, 1, 64);
        const bool fromA_n = __shfl_down(fromA ? 1 : 0, 1, 64) != 0;
        const double val_n = __shfl_down(val, 1, 64);
        const bool pair_next = lane < 63 && fromA && !fromA_n && key_n == key && key != kMergeInf;
        const int pn_up = __shfl_up(pair_next ? 1 : 0, 1, 64);
        const bool pair_prev = pn_up != 0 && lane > 0;
        // consume 63 elements, or 64 when 62-63 is a pair
        const int M = __shfl(pair_next ? 1 : 0, 62, 64) ? 64 : 63;
        const bool live = lane < M && key != kMergeInf;
        const bool emit = live && !pair_prev;
        const double y = val + (pair_next ? val_n : 0.0);
        const double cv = emit ? y / (s[emit ? key : 0] * sr) : 0.0;
        const unsigned long long em = __ballot(emit);
        if (PASS == 0) {
            csum += (key == r ? 1.0 : 2.0) * cv;
        } else if (emit) {
            const long long q = pos + __popcll(em & ((1ull << lane) - 1ull));
            ob1[q] = (int32_t)r;
            ob2[q] = key;
            ov[q] = rf * cv;
        }
        pos += __popcll(em);
        const int xa = __popcll(__ballot(posA < M));  // A elements among the M consumed
        const int xb = M - xa;
        ia += xa;
        ib += xb;
        // shift: the new window = cur[xa ..] ++ nxt[.. xa); nxt from memory
        {
            const int sa = (lane + xa) & 63, sb = (lane + xb) & 63;
            const bool fa = lane + xa < 64, fb = lane + xb < 64;
            const int32_t a_c = __shfl(ca, sa, 64), a_n = __shfl(na, sa, 64);
            const uint32_t v_c = (uint32_t)__shfl((int)cva, sa, 64), v_n = (uint32_t)__shfl((int)nva, sa, 64);
            const unsigned long long e_c = __shfl(ce, sb, 64), e_n = __shfl(ne, sb, 64);
            ca = fa ? a_c : a_n;
            cva = fa ? v_c : v_n;
            ce = fb ? e_c : e_n;
        }
        na = g.C[std::min(ia + 64 + lane, aq)];
        nva = g.V[std::min(ia + 64 + lane, aq)];
        ne = g.lrv[std::min(ib + 64 + lane, bq)];
    }
    if (PASS == 0) {
        csum = wave_sum(csum);
        if (lane == 0) {
            len_or_off[r] = pos;
            rowc[r] = csum;
        }
    }
}

// sum of per-row values in blocks of `per` rows (fixed tree per block)
__global__ __launch_bounds__(256) void k_gw_rowsum_blocks(const double* __restrict__ v, long long n, long long per,
                                                          double* __restrict__ part) {
    __shared__ double sh[16];
    const long long lo = (long long)blockIdx.x * per, hi = std::min<long long>(n, lo + per);
    double acc = 0.0;
    for (long long q = lo + threadIdx.x; q < hi; q += 256) acc += v[q];
    acc = block_sum(acc, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

}  // namespace hh

using namespace hh;

namespace { struct GwScratch; }
struct hh_gw {
    int device = 0;
    std::shared_ptr<GwScratch> scratch;  // between hh_gw_correct_count and _write
    int64_t n = 0, N2 = 0, t_nnz = 0, h_nnz = 0, n_keys = 0;
    DBuf<int32_t> tA, tB, R, C;  // converted copies (host / int64 tables); device int32 tables are used in place
    DBuf<uint32_t> tV, V;
    const int32_t *tAp = nullptr, *tBp = nullptr, *Rp = nullptr, *Cp = nullptr;
    const uint32_t *tVp = nullptr, *Vp = nullptr;
    int fmt = 0;  // column-list entry format (RsCells, pairs.hip)
    DBuf<long long> hptr, cptr;
    DBuf<unsigned long long> keys;  // column-sorted cells, (row, count) packed after hh_gw_create
    int ib = 1;
    std::vector<unsigned long long> t_rowsum, t_nnz_row, h_blocksum;
    unsigned long long h_total = 0;
    // the SNP alpha per chromosome (bin order), computed on the host while
    // the GPU builds the column lists (hh_gw_alpha); ok 0: NumPy's own path
    std::vector<double> alpha;
    std::vector<int32_t> alpha_ok;
    // result (upper-triangle table of Nor)
    DBuf<int32_t> ob1, ob2;
    DBuf<double> ov;
    int64_t out_nnz = -1;
};

namespace {

const char* kErrWhat[5] = {"bin id out of range", "bin1 > bin2 in the traditional table (not upper triangle)",
                           "cells not sorted by (row, col)", "duplicate cell", "counts must be non-negative integers < 2^32"};

// HH_GW_TIMING: host timestamps at gw_create's synchronisation points (stderr)
struct GwClock {
    bool on = std::getenv("HH_GW_TIMING") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void lap(const char* what) {
        if (!on) return;
        const auto u = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[gw_create] %s: %.2f ms\n", what, std::chrono::duration<double, std::milli>(u - t).count());
        t = u;
    }
};

// the first offending entry over the five codes (k_gw_check / gw_code)
void throw_first_error(const unsigned long long* he, const char* what) {
    int code = -1;
    unsigned long long at = ~0ull;
    for (int q = 0; q < 5; ++q)
        if (he[q] < at) { at = he[q]; code = q; }
    if (code >= 0) HH_THROW(HH_ERR_ARG, std::string(what) + ": " + kErrWhat[code] + " at entry " + std::to_string(at));
}

// Validate a table (range, order, uniqueness, counts); COPY: convert it into
// int32 / uint32 device arrays (host or int64 tables), else it is used in
// place (int32 device tables).  Returns the largest count.
template <class Id, class Cnt, bool COPY>
unsigned gw_check(const Id* r, const Id* c, const Cnt* v, int64_t nnz, int64_t nb, int upper, DBuf<int32_t>& R,
                  DBuf<int32_t>& Cc, DBuf<uint32_t>& V, const char* what, hipStream_t s) {
    if (COPY) {
        R.alloc(std::max<int64_t>(nnz, 1));
        Cc.alloc(std::max<int64_t>(nnz, 1));
        V.alloc(std::max<int64_t>(nnz, 1));
    }
    GwClock ck;
    DBuf<unsigned long long> err(5);
    DBuf<unsigned> vmax(1);
    ck.lap("check: alloc");
    vmax.zero(s);
    HIP_CHECK(hipMemsetAsync(err.p, 0xff, 5 * sizeof(unsigned long long), s));
    if (nnz > 0)
        hipLaunchKernelGGL((k_gw_check<Id, Cnt, COPY>), dim3((unsigned)std::max<long long>(1, std::min<long long>((nnz + 255) / 256, 16384))), dim3(256), 0, s, r, c, v,
                           (long long)nnz, (long long)nb, upper, R.p, Cc.p, V.p, err.p, vmax.p);
    HIP_CHECK(hipGetLastError());
    ck.lap("check: launch");
    // into pinned memory: a pageable download here measured ~18 ms of host
    // wait beyond the kernel (HH_GW_TIMING)
    unsigned long long he[5];
    unsigned mx = 0;
    char* pin = (char*)pinned_stage().get(0, 64);
    err.download((unsigned long long*)pin, 5, s);
    vmax.download((unsigned*)(pin + 48), 1, s);
    ck.lap("check: downloads enqueued");
    HIP_CHECK(hipStreamSynchronize(s));
    std::memcpy(he, pin, sizeof(he));
    std::memcpy(&mx, pin + 48, sizeof(mx));
    ck.lap("check: sync");
    throw_first_error(he, what);
    return mx;
}

// GenomeWideMatrixCorrection's alpha step (:878-893) per chromosome, the
// reference's NumPy expressions on the exact integer statistics, as
// matrixBuilding.GenomeWideMatrixCorrectionSparse's glue computes them:
// cov = 1 - zeros / L (Coverage_M :904), gap = cov < 0.1
// (Gap_definedLowRes :742-753), alpha = (M + P) / (T + 1) / max over the
// non-gap bins, 0 -> 1, floored at np.percentile(non-gap, 20).  A chromosome
// whose max is not a positive finite number (NumPy's NaN / inf paths) or
// that has no non-gap bin (np.max of an empty array raises) is left to the
// NumPy path (ok 0).
// G.alpha / G.alpha_ok are sized (n, 0 everywhere) by the caller on its own
// thread before this runs, so a throw here leaves every chromosome to NumPy.
static void gw_alpha_host(hh_gw& G, const std::vector<int64_t>& off) {
    const int64_t n = G.n;
    const int nc = (int)off.size() - 1;
    std::vector<double> ng;
    std::vector<uint8_t> gap;
    for (int c = 0; c < nc; ++c) {
        const int64_t s = off[c], e = off[c + 1], L = e - s;
        if (L <= 0) continue;
        double mx = -std::numeric_limits<double>::infinity();
        bool any = false;
        gap.assign(L, 0);
        for (int64_t i = s; i < e; ++i) {
            const int64_t zeros = L - (int64_t)G.t_nnz_row[i];
            const double cov = 1.0 - ((double)zeros / (double)L);
            gap[i - s] = cov < 0.1;
            const int64_t hp = (int64_t)G.h_blocksum[i] + (int64_t)G.h_blocksum[n + i];
            const double a = (double)hp / (double)((int64_t)G.t_rowsum[i] + 1);
            G.alpha[i] = a;
            if (!gap[i - s]) {
                mx = std::max(mx, a);
                any = true;
            }
        }
        if (!any || !(mx > 0.0) || !std::isfinite(mx)) continue;
        ng.clear();
        for (int64_t i = s; i < e; ++i) {
            double a = G.alpha[i] / mx;
            if (a == 0.0) a = 1.0;
            G.alpha[i] = a;
            if (!gap[i - s]) ng.push_back(a);
        }
        const double th = np_percentile(ng, 20.0);
        for (int64_t i = s; i < e; ++i)
            if (G.alpha[i] < th) G.alpha[i] = th;
        G.alpha_ok[c] = 1;
    }
}

// joins the alpha thread on every path out of gw_create
struct ThreadJoin {
    std::thread t;
    ~ThreadJoin() {
        if (t.joinable()) t.join();
    }
};

// Argument checks of hh_gw_create*, before anything touches the device.  The
// column sort (dev_sort_cells_by_col, pairs.hip) keeps its radix offsets in
// 32 bits, so the haplotype cells are capped below 2^32 - 1.
static void gw_check_args(int64_t t_nnz, int64_t h_nnz, int64_t n, const int64_t* chrom_offsets, int32_t n_chroms) {
    HH_REQUIRE(n > 0 && n_chroms > 0 && chrom_offsets && t_nnz >= 0 && h_nnz >= 0, "bad arguments");
    HH_REQUIRE(chrom_offsets[0] == 0 && chrom_offsets[n_chroms] == n, "chrom_offsets must span [0, n]");
    HH_REQUIRE(2 * n < kMaxBins, "too many bins");
    HH_REQUIRE(h_nnz < (int64_t)0xFFFFFFFFLL, "too many haplotype cells: the column sort holds < 2^32 - 1");
}

template <class Id, class Cnt>
void gw_create(hh_gw& G, const Id* t1, const Id* t2, const Cnt* tv, int64_t t_nnz, const Id* hr, const Id* hc,
               const Cnt* hv, int64_t h_nnz, int64_t n, const int64_t* chrom_offsets, int32_t n_chroms,
               hipStream_t s) {
    gw_check_args(t_nnz, h_nnz, n, chrom_offsets, n_chroms);
    GwClock clk;
    if (clk.on) {
        HIP_CHECK(hipStreamSynchronize(s));
        clk.lap("stream idle at entry");
        HIP_CHECK(hipDeviceSynchronize());
        clk.lap("device idle at entry");
    }
    G.n = n;
    G.N2 = 2 * n;
    G.t_nnz = t_nnz;
    G.h_nnz = h_nnz;
    // per bin: its chromosome's [lo, hi) in T, its same-haplotype block's in H
    std::vector<int2> chrom_bd(n), block_bd(2 * n);
    for (int c = 0; c < n_chroms; ++c) {
        HH_REQUIRE(chrom_offsets[c] <= chrom_offsets[c + 1], "chrom_offsets not monotone");
        const int32_t lo = (int32_t)chrom_offsets[c], hi = (int32_t)chrom_offsets[c + 1];
        for (int64_t b = chrom_offsets[c]; b < chrom_offsets[c + 1]; ++b) {
            chrom_bd[b] = make_int2(lo, hi);
            block_bd[b] = make_int2(lo, hi);                                    // M copy of chromosome c
            block_bd[n + b] = make_int2((int32_t)(n + lo), (int32_t)(n + hi));  // P copy
        }
    }
    constexpr bool COPY = !(std::is_same<Id, int32_t>::value && std::is_same<Cnt, int32_t>::value);
    clk.lap("setup");
    unsigned hmax = 0;
    const bool tpack = n < (1LL << 24);
    // int32 device tables: validated by the statistics kernels themselves
    // (one read of each table instead of two); the others are converted and
    // validated first
    const bool fused = !COPY && tpack;
    if (!fused) {
        HH_KTIME("gw_check", s);
        gw_check<Id, Cnt, COPY>(t1, t2, tv, t_nnz, n, 1, G.tA, G.tB, G.tV, "traditional table", s);
        hmax = gw_check<Id, Cnt, COPY>(hr, hc, hv, h_nnz, 2 * n, 0, G.R, G.C, G.V, "haplotype cells", s);
    }
    if (COPY) {
        G.tAp = G.tA.p, G.tBp = G.tB.p, G.tVp = G.tV.p, G.Rp = G.R.p, G.Cp = G.C.p, G.Vp = G.V.p;
    } else {  // validated int32 device tables, read in place (counts >= 0: as uint32)
        G.tAp = reinterpret_cast<const int32_t*>(t1), G.tBp = reinterpret_cast<const int32_t*>(t2);
        G.tVp = reinterpret_cast<const uint32_t*>(tv);
        G.Rp = reinterpret_cast<const int32_t*>(hr), G.Cp = reinterpret_cast<const int32_t*>(hc);
        G.Vp = reinterpret_cast<const uint32_t*>(hv);
    }
    clk.lap("checks");
    // host <-> device transfers of gw_create / gw_prepare go through the
    // per-thread pinned staging buffers: pageable copies measured 20+ ms
    // each here (the 4.9 MB alpha upload: 24 ms for ~0.1 ms of DMA)
    DBuf<int2> dch(n), dblk(2 * n);
    {
        const size_t b1 = (size_t)n * sizeof(int2), b2 = (size_t)2 * n * sizeof(int2);
        char* up = (char*)pinned_stage().get(1, b1 + b2);
        std::memcpy(up, chrom_bd.data(), b1);
        std::memcpy(up + b1, block_bd.data(), b2);
        dch.upload((const int2*)up, n, s);
        dblk.upload((const int2*)(up + b1), 2 * n, s);
    }
    DBuf<unsigned long long> trs(n), tnz(n), hbs(2 * n), htot(1);
    trs.zero(s);
    tnz.zero(s);
    hbs.zero(s);
    htot.zero(s);
    auto sgrid = [](int64_t nnz) { return dim3((unsigned)std::min<int64_t>(kGwStatBlocks, (nnz + 255) / 256)); };
    DBuf<unsigned long long> tpk(tpack ? n : 1), ttot(1);
    if (tpack) tpk.zero(s);
    ttot.zero(s);
    DBuf<unsigned long long> errs(10);
    DBuf<unsigned> vmx(1);
    HIP_CHECK(hipMemsetAsync(errs.p, 0xff, 10 * sizeof(unsigned long long), s));
    vmx.zero(s);
    G.hptr.alloc(2 * n + 1);
    // HH_GW_ST_ITEMS="T,H": entries per thread of the statistics kernels (8 / 16; A/B runs)
    int st_items_t = kStItemsT, st_items_h = kStItemsH;
    if (const char* e = std::getenv("HH_GW_ST_ITEMS")) std::sscanf(e, "%d,%d", &st_items_t, &st_items_h);
    // HH_GW_TSWIN: LDS column window of the T statistics (entries, <= 8192)
    int wsz = kTsWin;
    if (const char* e = std::getenv("HH_GW_TSWIN")) wsz = std::max(256, std::min(kTsWin, std::atoi(e)));
    const StCheck ckT{errs.p, nullptr, nullptr}, ckH{errs.p + 5, vmx.p, G.hptr.p};
    HH_KTIME("gw_stats_to_end", s);  // (from the statistics to the end of create)
    if (t_nnz > 0) {
        if (tpack) {
            const long long nb = std::min<long long>(8192, (t_nnz + 65535) / 65536);
            const long long per = ((t_nnz + nb - 1) / nb + 255) / 256 * 256;
            auto launch_t = [&](auto it) {
                constexpr int IT = decltype(it)::value;
                if (fused)
                    hipLaunchKernelGGL((k_gw_tstats_win<IT, true>), dim3((unsigned)((t_nnz + per - 1) / per)), dim3(256),
                                       (size_t)wsz * 8, s, G.tAp, G.tBp, G.tVp, (long long)t_nnz, per, (long long)n,
                                       dch.p, tpk.p, ttot.p, ckT, wsz);
                else
                    hipLaunchKernelGGL((k_gw_tstats_win<IT, false>), dim3((unsigned)((t_nnz + per - 1) / per)),
                                       dim3(256), (size_t)wsz * 8, s, G.tAp, G.tBp, G.tVp, (long long)t_nnz, per,
                                       (long long)n, dch.p, tpk.p, ttot.p, ckT, wsz);
            };
            if (st_items_t == 8) launch_t(std::integral_constant<int, 8>{});
            else launch_t(std::integral_constant<int, kStItemsT>{});
        }
        else
            hipLaunchKernelGGL(k_gw_tstats<false>, sgrid(t_nnz), dim3(256), 0, s, G.tAp, G.tBp, G.tVp,
                               (long long)t_nnz, dch.p, trs.p, tnz.p, nullptr, nullptr);
    }
    if (h_nnz > 0) {
        const long long nb = std::min<long long>(8192, (h_nnz + 65535) / 65536);
        const long long per = ((h_nnz + nb - 1) / nb + 255) / 256 * 256;
        auto launch_h = [&](auto it) {
            constexpr int IT = decltype(it)::value;
            if (fused)
                hipLaunchKernelGGL((k_gw_hstats<IT, true>), dim3((unsigned)((h_nnz + per - 1) / per)), dim3(256), 0, s,
                                   G.Rp, G.Cp, G.Vp, (long long)h_nnz, per, (long long)(2 * n), dblk.p, hbs.p, htot.p,
                                   ckH);
            else
                hipLaunchKernelGGL((k_gw_hstats<IT, false>), dim3((unsigned)((h_nnz + per - 1) / per)), dim3(256), 0,
                                   s, G.Rp, G.Cp, G.Vp, (long long)h_nnz, per, (long long)(2 * n), dblk.p, hbs.p,
                                   htot.p, ckH);
        };
        if (st_items_h == 16) launch_h(std::integral_constant<int, 16>{});
        else launch_h(std::integral_constant<int, kStItemsH>{});
    }
    HIP_CHECK(hipGetLastError());
    G.t_rowsum.resize(n);
    G.t_nnz_row.resize(n);
    G.h_blocksum.resize(2 * n);
    {
        // pinned layout: t_rowsum n | t_nnz n | h_blocksum 2n | h_total | t_total | packed n | errs 10 | vmax
        unsigned long long* pin = (unsigned long long*)pinned_stage().get(0, ((size_t)5 * n + 13) * 8);
        unsigned long long* p_err = pin + 5 * n + 2;
        unsigned long long *p_trs = pin, *p_tnz = pin + n, *p_hbs = pin + 2 * n, *p_htot = pin + 4 * n,
                           *p_ttot = pin + 4 * n + 1, *p_pk = pin + 4 * n + 2;
        const bool packed = tpack && t_nnz > 0;
        trs.download(p_trs, n, s);
        tnz.download(p_tnz, n, s);
        hbs.download(p_hbs, 2 * n, s);
        htot.download(p_htot, 1, s);
        if (packed) {
            ttot.download(p_ttot, 1, s);
            tpk.download(p_pk, n, s);
        }
        if (fused) {
            errs.download(p_err, 10, s);
            vmx.download((unsigned*)(p_err + 10), 1, s);
        }
        HIP_CHECK(hipStreamSynchronize(s));
        if (fused) {
            throw_first_error(p_err, "traditional table");
            throw_first_error(p_err + 5, "haplotype cells");
            hmax = *(const unsigned*)(p_err + 10);
        }
        std::copy(p_trs, p_trs + n, G.t_rowsum.begin());
        std::copy(p_tnz, p_tnz + n, G.t_nnz_row.begin());
        std::copy(p_hbs, p_hbs + 2 * n, G.h_blocksum.begin());
        G.h_total = *p_htot;
        if (packed) {
            if (*p_ttot < (1ull << 39)) {  // no row + column sum (<= 2 tt) can have carried into bit 64
                for (int64_t y = 0; y < n; ++y) {
                    G.t_rowsum[y] += p_pk[y] >> 24;
                    G.t_nnz_row[y] += p_pk[y] & 0xffffffull;
                }
            } else {  // counts too large for the packed field: the two-atomic pass
                trs.zero(s);
                tnz.zero(s);
                hipLaunchKernelGGL(k_gw_tstats<false>, sgrid(t_nnz), dim3(256), 0, s, G.tAp, G.tBp, G.tVp,
                                   (long long)t_nnz, dch.p, trs.p, tnz.p, nullptr, nullptr);
                HIP_CHECK(hipGetLastError());
                trs.download(p_trs, n, s);
                tnz.download(p_tnz, n, s);
                HIP_CHECK(hipStreamSynchronize(s));
                std::copy(p_trs, p_trs + n, G.t_rowsum.begin());
                std::copy(p_tnz, p_tnz + n, G.t_nnz_row.begin());
            }
        }
    }
    // the alpha glue on a host thread while the GPU builds the column lists
    // (row pointers, column keys, the radix sort: ~45 ms at 10 kb diploid)
    clk.lap("statistics");
    std::vector<int64_t> offv(chrom_offsets, chrom_offsets + n_chroms + 1);
    G.alpha.assign(n, 0.0);  // sized here: a failure on the thread leaves ok = 0 for every chromosome
    G.alpha_ok.assign(n_chroms, 0);
    ThreadJoin alpha_thread;
    alpha_thread.t = std::thread([&G, offv]() {
        try {
            gw_alpha_host(G, offv);
        } catch (...) {
            std::fill(G.alpha_ok.begin(), G.alpha_ok.end(), 0);
        }
    });
    // H row pointers (unless the fused statistics wrote them) and column lists
    if (h_nnz == 0)
        HIP_CHECK(hipMemsetAsync(G.hptr.p, 0, (2 * n + 1) * sizeof(long long), s));
    else if (!fused)
        hipLaunchKernelGGL(k_px_rowptr_gw, dim3((unsigned)((h_nnz + 1 + 255) / 256)), dim3(256), 0, s, G.Rp,
                           (long long)h_nnz, (long long)(2 * n), G.hptr.p);
    int cbits = 1;
    while (cbits < 40 && ((int64_t)1 << cbits) < 2 * n) ++cbits;
    // packed keys (col | row | count) when ids fit 20 bits and counts 24
    G.fmt = (2 * n <= (1LL << 20) && hmax < (1u << 24)) ? 1 : 0;
    if (G.fmt) {
        G.ib = 44;
    } else {
        G.ib = 1;
        while (G.ib < 63 && ((int64_t)1 << G.ib) < std::max<int64_t>(h_nnz, 2)) ++G.ib;
    }
    HH_REQUIRE(G.ib + cbits <= 64, "haplotype matrix too large for 64-bit column keys");
    G.keys.alloc(std::max<int64_t>(h_nnz, 1));
    {
        HH_KTIME("gw_sort", s);
        // the column keys are formed inside the first radix pass (in cell
        // order, so only the column bits are sorted); were a count pass, a
        // key write pass and a full first pass over the written keys
        G.n_keys = dev_sort_cells_by_col(G.Rp, G.Cp, G.Vp, h_nnz, G.fmt, G.ib, cbits, G.keys, s);
    }
    const unsigned long long hn = (unsigned long long)G.n_keys;
    clk.lap("column keys + sort");
    G.cptr.alloc(2 * n + 1);
    if (hn == 0)
        HIP_CHECK(hipMemsetAsync(G.cptr.p, 0, (2 * n + 1) * sizeof(long long), s));
    else
        hipLaunchKernelGGL(k_px_keyptr_gw, dim3((unsigned)((hn + 1 + 256 * kKpItems - 1) / (256 * kKpItems))),
                           dim3(256), 0, s, G.keys.p, (long long)hn, G.ib, (long long)(2 * n), G.cptr.p);
    if (hn && !G.fmt)
        hipLaunchKernelGGL(k_gw_pack, dim3((unsigned)((hn + 255) / 256)), dim3(256), 0, s, G.keys.p, (long long)hn,
                           G.ib >= 64 ? ~0ull : ((1ull << G.ib) - 1ull), G.Rp, G.Vp);
    HIP_CHECK(hipGetLastError());
    clk.lap("sort");
    HIP_CHECK(hipStreamSynchronize(s));
    clk.lap("key pointers");
    alpha_thread.t.join();
    clk.lap("alpha join");
}

}  // namespace

extern "C" {

int hh_gw_create(const int64_t* t_bin1, const int64_t* t_bin2, const double* t_count, int64_t t_nnz,
                 const int64_t* h_row, const int64_t* h_col, const double* h_count, int64_t h_nnz, int64_t n,
                 const int64_t* chrom_offsets, int32_t n_chroms, void* stream, hh_gw** out) {
    return guard([&] {
        HH_REQUIRE(out, "null");
        HH_REQUIRE((t_nnz == 0 || (t_bin1 && t_bin2 && t_count)) && (h_nnz == 0 || (h_row && h_col && h_count)),
                   "null arrays");
        gw_check_args(t_nnz, h_nnz, n, chrom_offsets, n_chroms);
        hipStream_t s = as_stream(stream);
        auto G = std::make_unique<hh_gw>();
        HIP_CHECK(hipGetDevice(&G->device));
        DBuf<long long> a(std::max<int64_t>(t_nnz, 1)), b(std::max<int64_t>(t_nnz, 1)), r(std::max<int64_t>(h_nnz, 1)),
            c(std::max<int64_t>(h_nnz, 1));
        DBuf<double> tv(std::max<int64_t>(t_nnz, 1)), hv(std::max<int64_t>(h_nnz, 1));
        a.upload(reinterpret_cast<const long long*>(t_bin1), t_nnz, s);
        b.upload(reinterpret_cast<const long long*>(t_bin2), t_nnz, s);
        tv.upload(t_count, t_nnz, s);
        r.upload(reinterpret_cast<const long long*>(h_row), h_nnz, s);
        c.upload(reinterpret_cast<const long long*>(h_col), h_nnz, s);
        hv.upload(h_count, h_nnz, s);
        gw_create<long long, double>(*G, a.p, b.p, tv.p, t_nnz, r.p, c.p, hv.p, h_nnz, n, chrom_offsets, n_chroms, s);
        *out = G.release();
    });
}

int hh_gw_create_device(const int32_t* t_bin1, const int32_t* t_bin2, const int32_t* t_count, int64_t t_nnz,
                        const int32_t* h_row, const int32_t* h_col, const int32_t* h_count, int64_t h_nnz, int64_t n,
                        const int64_t* chrom_offsets, int32_t n_chroms, void* stream, hh_gw** out) {
    return guard([&] {
        HH_REQUIRE(out, "null");
        gw_check_args(t_nnz, h_nnz, n, chrom_offsets, n_chroms);
        auto G = std::make_unique<hh_gw>();
        HIP_CHECK(hipGetDevice(&G->device));
        gw_create<int32_t, int32_t>(*G, t_bin1, t_bin2, t_count, t_nnz, h_row, h_col, h_count, h_nnz, n,
                                    chrom_offsets, n_chroms, as_stream(stream));
        *out = G.release();
    });
}

int hh_gw_free(hh_gw* g) {
    return guard([&] {
        if (g) device_quiesce(g->device);
        delete g;
    });
}

int hh_gw_alpha(const hh_gw* g, double* alpha, int32_t* chrom_ok) {
    return guard([&] {
        HH_REQUIRE(g && alpha && chrom_ok, "null");
        HH_REQUIRE((int64_t)g->alpha.size() == g->n, "alpha not computed");
        std::copy(g->alpha.begin(), g->alpha.end(), alpha);
        std::copy(g->alpha_ok.begin(), g->alpha_ok.end(), chrom_ok);
    });
}

int hh_gw_stats(const hh_gw* g, int64_t* t_rowsum, int64_t* t_nnz_row, int64_t* h_blocksum, int64_t* h_total) {
    return guard([&] {
        HH_REQUIRE(g, "null");
        if (t_rowsum) for (int64_t i = 0; i < g->n; ++i) t_rowsum[i] = (int64_t)g->t_rowsum[i];
        if (t_nnz_row) for (int64_t i = 0; i < g->n; ++i) t_nnz_row[i] = (int64_t)g->t_nnz_row[i];
        if (h_blocksum) for (int64_t i = 0; i < g->N2; ++i) h_blocksum[i] = (int64_t)g->h_blocksum[i];
        if (h_total) *h_total = (int64_t)g->h_total;
    });
}

}  // extern "C"

namespace {

// marginals, VC factors, merge count pass and sum(C): everything up to the
// write; returns the output size, leaves s / offsets / rf in the scratch
struct GwScratch {
    DBuf<double> dal, sv, rowc;
    DBuf<long long> ustart, lstart, len, roff;
    double rf = 0.0;
    long long total = 0;
};

template <int FMT>
void gw_prepare(hh_gw* g, const double* alpha, double exponent, GwScratch& W, hipStream_t s) {
    const int64_t N2 = g->N2;
    GwClock ck;
    W.dal.alloc(N2);
    W.sv.alloc(N2);
    W.rowc.alloc(N2);
    ck.lap("prepare: allocs");
    {
        double* up = (double*)pinned_stage().get(1, (size_t)N2 * sizeof(double));
        std::memcpy(up, alpha, (size_t)N2 * sizeof(double));
        W.dal.upload(up, N2, s);
    }
    ck.lap("prepare: alpha upload");
    W.ustart.alloc(N2);
    W.lstart.alloc(N2);
    W.len.alloc(N2 + 1);
    W.roff.alloc(N2 + 1);
    GwDev d{g->Rp, g->Cp, g->Vp, g->hptr.p, g->keys.p, g->cptr.p, (long long)N2, W.dal.p, W.ustart.p, W.lstart.p};
    const unsigned wg = (unsigned)((N2 * 64 + 255) / 256);
    {
        HH_KTIME("gw_marg", s);
        hipLaunchKernelGGL(k_gw_marg<FMT>, dim3(wg), dim3(256), 0, s, d, exponent, W.sv.p);
    }
    {
        HH_KTIME("gw_merge0", s);
        hipLaunchKernelGGL((k_gw_merge<FMT, 0>), dim3(wg), dim3(256), 0, s, d, W.sv.p, 0.0, W.len.p, W.rowc.p,
                           (int32_t*)nullptr, (int32_t*)nullptr, (double*)nullptr);
    }
    HIP_CHECK(hipMemsetAsync(W.len.p + N2, 0, sizeof(long long), s));
    DBuf<unsigned long long> tot(1);
    dev_excl_scan_i64(W.len.p, W.roff.p, N2 + 1, tot.p, s);
    // sum(C) over the full matrix: row shares in row order, fixed tree
    const long long per = 1 << 14;
    const long long nbk = std::max<long long>(1, (N2 + per - 1) / per);
    DBuf<double> part(nbk);
    hipLaunchKernelGGL(k_gw_rowsum_blocks, dim3((unsigned)nbk), dim3(256), 0, s, W.rowc.p, (long long)N2, per, part.p);
    HIP_CHECK(hipGetLastError());
    std::vector<double> hp(nbk);
    unsigned long long m = 0;
    ck.lap("prepare: kernels enqueued");
    char* pin = (char*)pinned_stage().get(0, (size_t)nbk * sizeof(double) + 16);
    part.download((double*)(pin + 16), nbk, s);
    tot.download((unsigned long long*)pin, 1, s);
    ck.lap("prepare: downloads enqueued");
    HIP_CHECK(hipStreamSynchronize(s));
    std::memcpy(hp.data(), pin + 16, (size_t)nbk * sizeof(double));
    std::memcpy(&m, pin, sizeof(m));
    ck.lap("prepare: sync");
    double csum = 0.0;
    for (double x : hp) csum += x;
    const double NN = (double)N2 * (double)N2;
    W.rf = ((double)g->h_total / NN) / (csum / NN);  // R_F = H.mean() / C.mean() (:897-899)
    W.total = (long long)m;
}

template <int FMT>
void gw_write(hh_gw* g, GwScratch& W, int32_t* b1, int32_t* b2, double* v, hipStream_t s) {
    const int64_t N2 = g->N2;
    GwDev d{g->Rp, g->Cp, g->Vp, g->hptr.p, g->keys.p, g->cptr.p, (long long)N2, W.dal.p, W.ustart.p, W.lstart.p};
    const unsigned wg = (unsigned)((N2 * 64 + 255) / 256);
    if (W.total > 0)
        hipLaunchKernelGGL((k_gw_merge<FMT, 1>), dim3(wg), dim3(256), 0, s, d, W.sv.p, W.rf, W.roff.p,
                           (double*)nullptr, b1, b2, v);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace

extern "C" {

int hh_gw_correct(hh_gw* g, const double* alpha, double exponent, int64_t* out_nnz, void* stream) {
    return guard([&] {
        HH_REQUIRE(g && alpha && out_nnz, "null");
        hipStream_t s = as_stream(stream);
        GwScratch W;
        if (g->fmt) gw_prepare<1>(g, alpha, exponent, W, s);
        else gw_prepare<0>(g, alpha, exponent, W, s);
        g->ob1.alloc(std::max<long long>(W.total, 1));
        g->ob2.alloc(std::max<long long>(W.total, 1));
        g->ov.alloc(std::max<long long>(W.total, 1));
        if (g->fmt) gw_write<1>(g, W, g->ob1.p, g->ob2.p, g->ov.p, s);
        else gw_write<0>(g, W, g->ob1.p, g->ob2.p, g->ov.p, s);
        g->out_nnz = W.total;
        *out_nnz = W.total;
    });
}

// The same in two calls so the caller can own the output: the count (and
// everything before the write, kept in the handle), then the write into
// caller-sized device buffers (no copy of a 20 GB result at 10 kb diploid).
int hh_gw_correct_count(hh_gw* g, const double* alpha, double exponent, int64_t* out_nnz, void* stream) {
    return guard([&] {
        HH_REQUIRE(g && alpha && out_nnz, "null");
        hipStream_t s = as_stream(stream);
        g->scratch = std::make_shared<GwScratch>();
        if (g->fmt) gw_prepare<1>(g, alpha, exponent, *g->scratch, s);
        else gw_prepare<0>(g, alpha, exponent, *g->scratch, s);
        *out_nnz = g->scratch->total;
    });
}

int hh_gw_correct_write(hh_gw* g, int32_t* bin1, int32_t* bin2, double* value, void* stream) {
    return guard([&] {
        HH_REQUIRE(g && g->scratch, "call hh_gw_correct_count first");
        HH_REQUIRE(g->scratch->total == 0 || (bin1 && bin2 && value), "null output buffers");
        hipStream_t s = as_stream(stream);
        if (g->fmt) gw_write<1>(g, *g->scratch, bin1, bin2, value, s);
        else gw_write<0>(g, *g->scratch, bin1, bin2, value, s);
        g->scratch.reset();
    });
}

int hh_gw_result(const hh_gw* g, int64_t* bin1, int64_t* bin2, double* value, void* stream) {
    return guard([&] {
        HH_REQUIRE(g && g->out_nnz >= 0, "call hh_gw_correct first");
        hipStream_t s = as_stream(stream);
        const int64_t m = g->out_nnz;
        std::vector<int32_t> a(m), b(m);
        g->ob1.download(a.data(), m, s);
        g->ob2.download(b.data(), m, s);
        if (value) g->ov.download(value, m, s);
        HIP_CHECK(hipStreamSynchronize(s));
        if (bin1) for (int64_t i = 0; i < m; ++i) bin1[i] = a[i];
        if (bin2) for (int64_t i = 0; i < m; ++i) bin2[i] = b[i];
    });
}

int hh_gw_result_device(const hh_gw* g, const int32_t** bin1, const int32_t** bin2, const double** value) {
    return guard([&] {
        HH_REQUIRE(g && g->out_nnz >= 0, "call hh_gw_correct first");
        if (bin1) *bin1 = g->ob1.p;
        if (bin2) *bin2 = g->ob2.p;
        if (value) *value = g->ov.p;
    });
}

}  // extern "C"
