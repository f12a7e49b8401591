// ICE balancing on the pixel-chunk layout (cooler balance_cooler semantics,
// oracle/ice_ref.py; HiCHap call sites matrixBuilding.py:708/713/1537/1542/
// 1761/1766).
//
// One iteration:
//   K1 k_sweep   one wave per segment (<= 8 chunks of one row): streams the
//                packed (count, col) entries, gathers b[col], accumulates
//                sum(count * b[col]) in fp64 -> part[seg]          [HBM bound]
//   K2 k_marg    per local row: marg = b_r * (sum_seg part + 2 * diag * b_r)
//                (cooler's bincount(bin1) + bincount(bin2))
//   K3 stats     per stats tile (a 512-row block cut at group boundaries).
//                Few tiles (<= 128, single chromosomes): nonzero count and sum
//                fused into k_marg when one GPU holds every row (else
//                k_stats1 on the gathered vector), the last block to finish
//                reduces them per group; k_update: b /= marg/mean (marg==0
//                -> 1) and the tile's squared deviations, its last block
//                records var/mean/iters and the next active flag (2 launches
//                after the sweep).  Many tiles: k_stats1, k_stats2,
//                k_update_big, every block re-reducing its group's tile sums
//                (no device-scope fences / one-wave tails over ~1 200 tiles).
// All reductions use fixed trees -> bitwise deterministic, and independent of
// how rows are sharded across GPUs.
#include <algorithm>
#include <chrono>
#include <functional>
#include <cmath>
#include <limits>

#include "ice_internal.hpp"

namespace hh {
constexpr int kThreads = 256;

// ---------------------------------------------------------------- K1
// One workgroup per unit (a run of tiles of one row-block, or a row range of
// one large tile).  Per tile: the 8192 bias values of the tile's columns are
// staged in LDS (coalesced 16-B loads, L2/MALL resident), then every entry
// gathers its b from LDS.  Rows are interleaved over the 8 waves; a row's
// entries in the tile are read as uint4 (4 entries per lane) by a lane group
// of G = 4..64 lanes (G from the tile's mean row length), reduced with
// xor-shuffles inside the group and added to the row's LDS accumulator,
// which only that wave touches -> fixed summation order (deterministic).
constexpr int kSweepThreads = 512;
constexpr int kSweepWaves = kSweepThreads / 64;
constexpr int kFlatU = 8;  // uint4 per lane per step in flat narrow segments
static_assert(kFlatU == kFlatIlvU, "k_sweep_flatw walks the interleaved layout's runs");

// Entry decode: the byte offset of the staged bias value is a field of the
// entry (ice_internal.hpp), so an entry costs mask, shift, cvt, LDS read and
// FMA.  All LDS reads of a uint4 are issued before the FMAs, into two
// accumulators (even / odd entries; fixed order -> deterministic).
__device__ __forceinline__ double lds_b(const double* bl, uint32_t byteoff) {
    return *reinterpret_cast<const double*>(reinterpret_cast<const char*>(bl) + byteoff);
}

__device__ __forceinline__ void tile_dot(const uint4 v, const double* __restrict__ bl, double& a0, double& a1) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    double x[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = lds_b(bl, w[i] & 0xFFFFu);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4; i += 2) {
        a0 = fma((double)(w[i] >> 16), x[i], a0);
        a1 = fma((double)(w[i + 1] >> 16), x[i + 1], a1);
    }
}

// 8 narrow entries (uint16 = byteoff | count) per uint4
__device__ __forceinline__ void tile_dot16(const uint4 v, const double* __restrict__ bl, double& a0, double& a1) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    double x[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        x[2 * i] = lds_b(bl, w[i] & 0xFFF8u);
        x[2 * i + 1] = lds_b(bl, (w[i] >> 16) & 0xFFF8u);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        a0 = fma((double)(w[i] & 7u), x[2 * i], a0);
        a1 = fma((double)((w[i] >> 16) & 7u), x[2 * i + 1], a1);
    }
}

// 16-B payload load as one global_load_dwordx4 (a HIP uint4 copy under a
// select is split into dword loads).  Unconditional: callers clamp the index
// to a valid slot and zero the value of finished rows.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld16(const uint4* p) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// Column side of a strictly upper tile: every stored count
// also feeds its column, count * B[row] added to the block's int64 LDS column
// accumulator -- at the entry's own byte offset, since the accumulator uses
// the bias slice's rotated image.  B = round(b * 2^e) with one power-of-two
// scale per sweep (k_fixscale), so the integer sums are exact whatever order
// the waves add in: deterministic, and the same on any number of GPUs.
typedef unsigned long long u64;
__device__ __forceinline__ u64 fixb(double b, double scale) { return (u64)__double2ll_rn(b * scale); }
__device__ __forceinline__ void lds_add_u64(u64* cacc, uint32_t byteoff, u64 v) {
    __hip_atomic_fetch_add(reinterpret_cast<u64*>(reinterpret_cast<char*>(cacc) + byteoff), v, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
}
// (branch-free: a padding entry adds 0 at offset 0; B < 2^62 / count total,
// so count * B is the 64-bit product of a small count and B)
__device__ __forceinline__ u64 cmul(uint32_t c, u64 B) {
    return (u64)c * (uint32_t)B + ((u64)(c * (uint32_t)(B >> 32)) << 32);
}
template <int EPV>
__device__ __forceinline__ void col_add(const uint4 v, u64 B, u64* __restrict__ cacc) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if constexpr (EPV == 8) {  // narrow: byteoff | count (0..7), two per word
            lds_add_u64(cacc, w[i] & 0xFFF8u, cmul(w[i] & 7u, B));
            lds_add_u64(cacc, (w[i] >> 16) & 0xFFF8u, cmul((w[i] >> 16) & 7u, B));
        } else {  // wide: count << 16 | byteoff
            lds_add_u64(cacc, w[i] & 0xFFFFu, cmul(w[i] >> 16, B));
        }
    }
}

// Rows of one segment of a tile (EPV entries per uint4: 8 narrow uint16, 4
// wide uint32).  Lane groups of G lanes take one row each, NB rows per group
// at a time (their loads issued together).  acc[v] (v = row
// index within the unit, + nr for the wide segment) is owned by one lane
// group per tile -> fixed summation order.
// COL: the tile is strictly upper (column side into cacc, B from bblk = b of
// the row-block's first row, scaled by `scale`)
struct ColArgs {
    const u64* bblk;  // B = round(b 2^e) of the tile's row-block (k_fixscale), row 0 first
    u64* cacc;
};

template <int G, int NB, int ABL, int EPV, bool COL = false>
__device__ __forceinline__ void tile_rows(const uint4* __restrict__ pay4, const uint32_t* __restrict__ rp,
                                          const double* __restrict__ bl, double* __restrict__ acc, int ra,
                                          int rb, int wave, int lane, ColArgs ca = ColArgs{}) {
    constexpr int RP = 64 / G;              // rows per wave step
    constexpr int S = kSweepWaves * RP;     // row distance between a wave's batches
    constexpr int SH = EPV == 8 ? 3 : 2;
    const int gi = lane / G, li = lane % G;
    const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
    for (int r0 = ra + wave * RP; r0 < rb; r0 += NB * S) {
        uint32_t q[NB], qe[NB];
        double a[NB], a1[NB];
        u64 B[NB];
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            const int r = r0 + k * S + gi;
            q[k] = qe[k] = 0;
            B[k] = 0;
            if (r < rb) {
                q[k] = (rp[r] >> SH) + li;
                qe[k] = rp[r + 1] >> SH;
                if (COL) B[k] = ca.bblk[r];
            }
            a[k] = 0.0;
            a1[k] = 0.0;
        }
        bool more = false;
#pragma unroll
        for (int k = 0; k < NB; ++k) more |= q[k] < qe[k];
        while (more) {
            uint4 v[NB];
#pragma unroll
            for (int k = 0; k < NB; ++k) {
                const bool on = q[k] < qe[k];
                const uint4 x = ld16(pay4 + (on ? q[k] : 0u));
                v[k] = on ? x : zero;
            }
            __builtin_amdgcn_sched_barrier(0);  // all NB loads in flight before the first use
            more = false;
#pragma unroll
            for (int k = 0; k < NB; ++k) {
                if (ABL == 1) {  // timing ablation: no LDS gathers
                    a[k] += (double)(v[k].x + v[k].y + v[k].z + v[k].w);
                } else if (EPV == 8) {
                    tile_dot16(v[k], bl, a[k], a1[k]);
                } else {
                    tile_dot(v[k], bl, a[k], a1[k]);
                }
                if (COL) col_add<EPV>(v[k], B[k], ca.cacc);
                q[k] += G;
                more |= q[k] < qe[k];
            }
        }
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            double x = a[k] + a1[k];
#pragma unroll
            for (int o = G >> 1; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
            const int r = r0 + k * S + gi;
            if (li == 0 && r < rb) acc[r - ra] += x;
        }
    }
}

// Sorted-band variant for units that cover whole row-blocks: the rows of a
// band of the tile's length order (perm[lo..hi), all within a 2x length
// range) go to lane groups of width G, so the rows a wave carries at once
// have similar lengths and few lanes idle.
template <int G, int NB, int ABL, int EPV, bool COL = false>
__device__ __forceinline__ void band_rows(const uint4* __restrict__ pay4, const uint32_t* __restrict__ rp,
                                          const uint16_t* __restrict__ perm, int lo, int hi,
                                          const double* __restrict__ bl, double* __restrict__ acc, int wave,
                                          int lane, ColArgs ca = ColArgs{}) {
    constexpr int RP = 64 / G;
    constexpr int S = kSweepWaves * RP;
    constexpr int SH = EPV == 8 ? 3 : 2;
    const int gi = lane / G, li = lane % G;
    const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
    for (int v0 = lo + wave * RP; v0 < hi; v0 += NB * S) {
        uint32_t q[NB], qe[NB];
        int row[NB];
        double a[NB], a1[NB];
        u64 B[NB];
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            const int v = v0 + k * S + gi;
            q[k] = qe[k] = 0;
            row[k] = -1;
            B[k] = 0;
            if (v < hi) {
                const int r = perm[v];
                row[k] = r;
                q[k] = (rp[r] >> SH) + li;
                qe[k] = rp[r + 1] >> SH;
                if (COL) B[k] = ca.bblk[r];
            }
            a[k] = 0.0;
            a1[k] = 0.0;
        }
        bool more = false;
#pragma unroll
        for (int k = 0; k < NB; ++k) more |= q[k] < qe[k];
        while (more) {
            uint4 v[NB];
#pragma unroll
            for (int k = 0; k < NB; ++k) {
                const bool on = q[k] < qe[k];
                const uint4 x = ld16(pay4 + (on ? q[k] : 0u));
                v[k] = on ? x : zero;
            }
            __builtin_amdgcn_sched_barrier(0);  // all NB loads in flight before the first use
            more = false;
#pragma unroll
            for (int k = 0; k < NB; ++k) {
                if (ABL == 1) {
                    a[k] += (double)(v[k].x + v[k].y + v[k].z + v[k].w);
                } else if (EPV == 8) {
                    tile_dot16(v[k], bl, a[k], a1[k]);
                } else {
                    tile_dot(v[k], bl, a[k], a1[k]);
                }
                if (COL) col_add<EPV>(v[k], B[k], ca.cacc);
                q[k] += G;
                more |= q[k] < qe[k];
            }
        }
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            double x = a[k] + a1[k];
#pragma unroll
            for (int o = G >> 1; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
            if (li == 0 && row[k] >= 0) acc[row[k]] += x;
        }
    }
}

// Flat (merge-path) sweep of a whole tile segment whose rows are all short
// (plan_tiles marks it).  The segment's payload is one
// contiguous uint4 array; fbe[0..nfr] are the entry offsets of its nonempty
// rows (row ids fr[i], in row order; fbe[nfr] = end).  Each wave takes the
// rows starting in its eighth of the array; per step every lane streams U
// consecutive uint4 (64 * U fully used uint4 per wave in flight, no idle
// lanes, no per-row setup chain), finds the row of its first uint4 by a
// short search over fbe, and walks its run closing rows at their starts:
//   * a row that starts and ends inside the run is added to acc by the lane;
//   * the part of a row before the run's first start ("head") flows left
//     through a segmented suffix scan over lanes to the lane where the row
//     started ("tail"), which adds tail + heads; lane 0 adds a head whose row
//     started in an earlier step.
// A row's acc is touched only by its wave, in program order; every sum is a
// fixed tree of the tile content -> deterministic.
template <int EPV>
__device__ __forceinline__ double flat_dot(const uint4 v, const double* __restrict__ bl) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    if constexpr (EPV == 8) {
        double g[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            g[2 * i] = lds_b(bl, w[i] & 0xFFF8u);
            g[2 * i + 1] = lds_b(bl, (w[i] >> 16) & 0xFFF8u);
        }
        __builtin_amdgcn_sched_barrier(0);
        double a = 0.0, c = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            a = fma((double)(w[i] & 7u), g[2 * i], a);
            c = fma((double)((w[i] >> 16) & 7u), g[2 * i + 1], c);
        }
        return a + c;
    } else {
        double g[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) g[i] = lds_b(bl, w[i] & 0xFFFFu);
        __builtin_amdgcn_sched_barrier(0);
        double a = 0.0, c = 0.0;
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
            a = fma((double)(w[i] >> 16), g[i], a);
            c = fma((double)(w[i + 1] >> 16), g[i + 1], c);
        }
        return a + c;
    }
}

// U consecutive uint4 of the lane's run starting at s (zeros past qb).
template <int U>
__device__ __forceinline__ void flat_load(const uint4* __restrict__ pay4, uint32_t s, uint32_t qa, uint32_t qb,
                                          uint4 (&v)[U]) {
    const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const bool on = s + k < qb;
        const uint4 x = ld16(pay4 + (on ? s + k : qa));
        v[k] = on ? x : zero;
    }
}

// The same run [q0 + U lane, + U) of a step chunk of an interleaved segment
// (finalize_flat_layout: element k of the chunk's runs stored contiguously,
// cnt_k lanes): U coalesced loads, the registers flat_load would fill.
template <int U>
__device__ __forceinline__ void flat_load_ilv(const uint4* __restrict__ pay4, uint32_t q0, uint32_t qb, int lane,
                                              uint4 (&v)[U]) {
    static_assert(U == kFlatIlvU, "interleaved segments are laid out for kFlatIlvU uint4 per lane");
    const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
    const uint32_t m = qb - q0 < 64u * U ? qb - q0 : 64u * U;
    uint32_t base = q0;
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const uint32_t cnt = flat_ilv_cnt(m, k);
        const bool on = (uint32_t)lane < cnt;
        // off lanes re-read the chunk's first uint4 (in the segment: m >= 1).
        // Not base: with m < U the elements k >= m have no lane (cnt 0) and
        // base is then q0 + m, one past the segment -- past the end of the
        // payload buffer for its last tile
        const uint4 x = ld16(pay4 + (on ? base + (uint32_t)lane : q0));
        v[k] = on ? x : zero;
        base += cnt;
    }
}
// a run of a plain (lane-major) or interleaved segment
template <int U, bool ILV>
__device__ __forceinline__ void flat_run(const uint4* __restrict__ pay4, uint32_t q0, uint32_t qa, uint32_t qb,
                                         int lane, uint4 (&v)[U]) {
    if constexpr (ILV) flat_load_ilv<U>(pay4, q0, qb, lane, v);
    else flat_load<U>(pay4, q0 + (uint32_t)lane * U, qa, qb, v);
}

// One step of a wave over uint4 [q0, q0 + 64 U) of its range [.., qb): v
// holds the lane's run [s, s + U), s = q0 + lane U.  ic = the row holding
// q0 - 1 (q0 at the first step); rows [.., i1) belong to the wave; fst =
// uint4 starts of the segment's nonempty rows (fst[nfr] = end), fr = their ids.
template <int U, int ABL, int EPV, bool COL = false>
__device__ __forceinline__ void flat_step(const uint4 (&v)[U], uint32_t q0, uint32_t qb, int& ic, int i1,
                                          const uint16_t* __restrict__ fst, const uint16_t* __restrict__ fr,
                                          int nfr, const double* __restrict__ bl, double* __restrict__ acc,
                                          int lane, ColArgs ca = ColArgs{}) {
    if constexpr (ABL == 3) {  // timing ablation (flat_step_c)
        uint32_t t = 0;
#pragma unroll
        for (int k = 0; k < U; ++k) t ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
        if (lane < nfr && t == 0x9E3779B9u) acc[lane] = (double)t;
        return;
    }
    const uint32_t s = q0 + (uint32_t)lane * U;
    const bool act = s < qb;
    // row of s: the largest i with start <= s; at most lane U + 1 rows
    // start in (q0 - 1, s] (rows are nonempty)
    int lo = ic, hi = min(i1 - 1, ic + lane * U + 1);
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((uint32_t)fst[mid] <= s) lo = mid; else hi = mid - 1;
    }
    const bool head = (uint32_t)fst[lo] < s;  // the run starts inside row lo
    uint32_t nb[U], rid[U];                 // starts of rows lo+1.., ids of rows lo..
#pragma unroll
    for (int k = 0; k < U; ++k) {
        nb[k] = fst[min(lo + 1 + k, nfr)];
        rid[k] = fr[min(lo + k, nfr - 1)];
    }
    u64 Bq[COL ? U : 1];  // the column side's B of rows lo..
    if (COL) {
#pragma unroll
        for (int k = 0; k < U; ++k) Bq[k] = ca.bblk[rid[k]];
    }
    double x = 0.0, h = 0.0, cv[U];
    uint32_t cr[U];
    bool inhead = head;
    int j = 0;  // row starts passed inside the run
#pragma unroll
    for (int k = 0; k < U; ++k) {
        cv[k] = 0.0;
        cr[k] = 0xFFFFFFFFu;
        if (k > 0) {
            uint32_t nxt = nb[0], crow = rid[0];
#pragma unroll
            for (int jj = 1; jj < k; ++jj)
                if (j == jj) {
                    nxt = nb[jj];
                    crow = rid[jj];
                }
            if (s + k == nxt && s + k < qb) {
                if (inhead) {
                    h = x;
                    inhead = false;
                } else if (U <= 4) {
                    cv[k] = x;
                    cr[k] = crow;
                } else {
                    acc[crow] += x;  // long runs: write at once (registers)
                }
                x = 0.0;
                ++j;
            }
        }
        x += ABL == 1 ? (double)(v[k].x + v[k].y + v[k].z + v[k].w) : flat_dot<EPV>(v[k], bl);
        if (COL) {
            u64 B = Bq[0];
#pragma unroll
            for (int jj = 1; jj <= k; ++jj)
                if (j == jj) B = Bq[jj];
            col_add<EPV>(v[k], B, ca.cacc);
        }
    }
    uint32_t orow = rid[0];
#pragma unroll
    for (int jj = 1; jj < U; ++jj)
        if (j == jj) orow = rid[jj];
    if (inhead) h = x;
    const bool tail = act && !inhead;
    // rows that start and end inside the run (independent read-modify-writes)
    if (U <= 4) {
        double old[U];
#pragma unroll
        for (int k = 1; k < U; ++k) old[k] = cr[k] != 0xFFFFFFFFu ? acc[cr[k]] : 0.0;
#pragma unroll
        for (int k = 1; k < U; ++k)
            if (cr[k] != 0xFFFFFFFFu) acc[cr[k]] = old[k] + cv[k];
    }
    // heads flow left: H_l = h_l + pass_l * H_{l+1}
    double H = act ? h : 0.0;
    int F = (!act || inhead) ? 1 : 0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double Hn = __shfl_down(H, o, 64);
        const int Fn = __shfl_down(F, o, 64);
        if (lane + o < 64 && F) {
            H += Hn;
            F = Fn;
        }
    }
    const double Hr = __shfl_down(H, 1, 64);
    if (tail) acc[orow] += x + (lane < 63 ? Hr : 0.0);
    if (lane == 0 && head) acc[rid[0]] += H;
    ic = __shfl(lo + j, 63, 64);
}

// flat_step with the accumulator indexed by compact row (the row's index in
// fst), not by row id: every nonempty row's first write is a plain store by
// the lane holding its start (a row that starts and ends in the run, or the
// tail + heads of one that continues), later steps add through lane 0 -- so
// no row ids, no stash and no read-modify-write inside the walk (registers
// for U = 8).  accc[i] is mapped to the row accumulator after the segment.
template <int U, int ABL, int EPV, bool COL = false>
__device__ __forceinline__ void flat_step_c(const uint4 (&v)[U], uint32_t q0, uint32_t qb, int& ic, int i1,
                                            const uint16_t* __restrict__ fst, int nfr,
                                            const double* __restrict__ bl, double* __restrict__ accc, int lane,
                                            ColArgs ca = ColArgs{}, const uint16_t* __restrict__ fid = nullptr) {
    if constexpr (ABL == 3) {  // timing ablation: the walk's skeleton only (no search, scan or gathers)
        uint32_t t = 0;
#pragma unroll
        for (int k = 0; k < U; ++k) t ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
        if (lane < nfr && t == 0x9E3779B9u) accc[lane] = (double)t;
        return;
    }
    const uint32_t s = q0 + (uint32_t)lane * U;
    const bool act = s < qb;
    int lo = ic, hi = min(i1 - 1, ic + lane * U + 1);
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((uint32_t)fst[mid] <= s) lo = mid; else hi = mid - 1;
    }
    const bool head = (uint32_t)fst[lo] < s;
    uint32_t nb[U];
#pragma unroll
    for (int k = 0; k < U - 1; ++k) nb[k] = fst[min(lo + 1 + k, nfr)];
    // the column side's B of compact rows lo .. lo + CB - 1 (fid: their row
    // ids, null = identity); a run reaching further rows (rare: ~3 uint4 per
    // row) loads those on the spot
    constexpr int CB = COL ? (U < 4 ? U : 4) : 1;
    u64 Bq[CB];
    if (COL) {
#pragma unroll
        for (int k = 0; k < CB; ++k) {
            const int i = min(lo + k, nfr - 1);
            Bq[k] = ca.bblk[fid ? (int)fid[i] : i];
        }
    }
    double x = 0.0, h = 0.0;
    bool inhead = head;
    int j = 0;
#pragma unroll
    for (int k = 0; k < U; ++k) {
        if (k > 0) {
            uint32_t nxt = nb[0];
#pragma unroll
            for (int jj = 1; jj < k; ++jj)
                if (j == jj) nxt = nb[jj];
            const bool starts = s + k == nxt && s + k < qb;
            if (starts) {
                if (inhead) {
                    h = x;
                    inhead = false;
                } else {
                    accc[lo + j] = x;  // started and ended in this run
                }
                x = 0.0;
                ++j;
            }
        }
        x += ABL == 1 ? (double)(v[k].x + v[k].y + v[k].z + v[k].w) : flat_dot<EPV>(v[k], bl);
        if (COL) {
            u64 B = Bq[0];
#pragma unroll
            for (int jj = 1; jj < CB && jj <= k; ++jj)
                if (j == jj) B = Bq[jj];
            if (k >= CB && j >= CB) {
                const int i = min(lo + j, nfr - 1);
                B = ca.bblk[fid ? (int)fid[i] : i];
            }
            col_add<EPV>(v[k], B, ca.cacc);
        }
    }
    if (inhead) h = x;
    const bool tail = act && !inhead;
    double H = act ? h : 0.0;
    int F = (!act || inhead) ? 1 : 0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double Hn = __shfl_down(H, o, 64);
        const int Fn = __shfl_down(F, o, 64);
        if (lane + o < 64 && F) {
            H += Hn;
            F = Fn;
        }
    }
    const double Hr = __shfl_down(H, 1, 64);
    if (tail) accc[lo + j] = x + (lane < 63 ? Hr : 0.0);  // the row's first write
    if (lane == 0 && head) accc[lo] += H;                 // continues a row of an earlier step
    ic = __shfl(lo + j, 63, 64);
}

template <int U, int ABL, int EPV, bool COL = false, bool ILV = false>
__device__ __forceinline__ void flat_seg_c(const uint4* __restrict__ pay4, uint4 (&v)[U], uint32_t qa, uint32_t qb,
                                           int i0, int i1, const uint16_t* __restrict__ fst, int nfr,
                                           const double* __restrict__ bl, double* __restrict__ accc, int lane,
                                           ColArgs ca = ColArgs{}, const uint16_t* __restrict__ fid = nullptr) {
    if (i0 >= i1) return;
    int ic = i0;
    for (uint32_t q0 = qa;;) {
        flat_step_c<U, ABL, EPV, COL>(v, q0, qb, ic, i1, fst, nfr, bl, accc, lane, ca, fid);
        q0 += 64u * U;
        if (q0 >= qb) break;
        flat_run<U, ILV>(pay4, q0, qa, qb, lane, v);
    }
}

// flat_seg_c / flat_seg with the next step's run loaded before the current
// step is walked (two runs in registers: the one-wave-per-tile kernel has
// the VGPRs for it); the same steps in the same order, bitwise the same sums
template <int U, int ABL, int EPV, bool COL = false, bool ILV = false>
__device__ __forceinline__ void flat_seg_c_pipe(const uint4* __restrict__ pay4, uint4 (&v)[U], uint32_t qa, uint32_t qb,
                                                int i0, int i1, const uint16_t* __restrict__ fst, int nfr,
                                                const double* __restrict__ bl, double* __restrict__ accc, int lane,
                                                ColArgs ca = ColArgs{}, const uint16_t* __restrict__ fid = nullptr) {
    if (i0 >= i1) return;
    int ic = i0;
    for (uint32_t q0 = qa;;) {
        const uint32_t qn = q0 + 64u * U;
        uint4 vn[U];
        if (qn < qb) flat_run<U, ILV>(pay4, qn, qa, qb, lane, vn);
        flat_step_c<U, ABL, EPV, COL>(v, q0, qb, ic, i1, fst, nfr, bl, accc, lane, ca, fid);
        if (qn >= qb) break;
#pragma unroll
        for (int k = 0; k < U; ++k) v[k] = vn[k];
        q0 = qn;
    }
}

template <int U, int ABL, int EPV, bool COL = false>
__device__ __forceinline__ void flat_seg_pipe(const uint4* __restrict__ pay4, uint4 (&v)[U], uint32_t qa, uint32_t qb,
                                              int i0, int i1, const uint16_t* __restrict__ fst,
                                              const uint16_t* __restrict__ fr, int nfr, const double* __restrict__ bl,
                                              double* __restrict__ acc, int lane, ColArgs ca = ColArgs{}) {
    if (i0 >= i1) return;
    int ic = i0;
    for (uint32_t q0 = qa;;) {
        const uint32_t qn = q0 + 64u * U;
        uint4 vn[U];
        if (qn < qb) flat_load<U>(pay4, qn + (uint32_t)lane * U, qa, qb, vn);
        flat_step<U, ABL, EPV, COL>(v, q0, qb, ic, i1, fst, fr, nfr, bl, acc, lane, ca);
        if (qn >= qb) break;
#pragma unroll
        for (int k = 0; k < U; ++k) v[k] = vn[k];
        q0 = qn;
    }
}

// A wave's rows [i0, i1) = uint4 [qa, qb) of one segment, the first step's
// run already loaded into v (its loads were issued before the tile's LDS
// staging, so they fly while the block stages).
template <int U, int ABL, int EPV, bool COL = false>
__device__ __forceinline__ void flat_seg(const uint4* __restrict__ pay4, uint4 (&v)[U], uint32_t qa, uint32_t qb,
                                         int i0, int i1, const uint16_t* __restrict__ fst,
                                         const uint16_t* __restrict__ fr, int nfr, const double* __restrict__ bl,
                                         double* __restrict__ acc, int lane, ColArgs ca = ColArgs{}) {
    if (i0 >= i1) return;
    int ic = i0;
    for (uint32_t q0 = qa;;) {
        flat_step<U, ABL, EPV, COL>(v, q0, qb, ic, i1, fst, fr, nfr, bl, acc, lane, ca);
        q0 += 64u * U;
        if (q0 >= qb) break;
        flat_load<U>(pay4, q0 + (uint32_t)lane * U, qa, qb, v);
    }
}

template <int NB, int ABL, int EPV, bool COL = false>
__device__ __forceinline__ void sweep_bands(const uint16_t* band, const uint4* pay4, const uint32_t* rp,
                                            const uint16_t* perm, const double* bl, double* acc, int wave,
                                            int lane, ColArgs ca = ColArgs{}) {
    if (band[1] > band[0]) band_rows<64, NB, ABL, EPV, COL>(pay4, rp, perm, band[0], band[1], bl, acc, wave, lane, ca);
    if (band[2] > band[1]) band_rows<32, NB, ABL, EPV, COL>(pay4, rp, perm, band[1], band[2], bl, acc, wave, lane, ca);
    if (band[3] > band[2]) band_rows<16, NB, ABL, EPV, COL>(pay4, rp, perm, band[2], band[3], bl, acc, wave, lane, ca);
    if (band[4] > band[3]) band_rows<8, NB, ABL, EPV, COL>(pay4, rp, perm, band[3], band[4], bl, acc, wave, lane, ca);
    if (band[5] > band[4]) band_rows<4, NB, ABL, EPV, COL>(pay4, rp, perm, band[4], band[5], bl, acc, wave, lane, ca);
}

template <int NB, int ABL, int EPV, bool COL = false>
__device__ __forceinline__ void sweep_rows(uint32_t mean, const uint4* pay4, const uint32_t* rp, const double* bl,
                                           double* acc, int ra, int rb, int wave, int lane, ColArgs ca = ColArgs{}) {
    if (mean >= 48) tile_rows<64, NB, ABL, EPV, COL>(pay4, rp, bl, acc, ra, rb, wave, lane, ca);
    else if (mean >= 24) tile_rows<32, NB, ABL, EPV, COL>(pay4, rp, bl, acc, ra, rb, wave, lane, ca);
    else if (mean >= 12) tile_rows<16, NB, ABL, EPV, COL>(pay4, rp, bl, acc, ra, rb, wave, lane, ca);
    else if (mean >= 6) tile_rows<8, NB, ABL, EPV, COL>(pay4, rp, bl, acc, ra, rb, wave, lane, ca);
    else tile_rows<4, NB, ABL, EPV, COL>(pay4, rp, bl, acc, ra, rb, wave, lane, ca);
}

// The tile's 8192 bias values -> LDS (rotated image), coalesced 16-B loads
// in R rounds (R > 1: fewer registers in flight).
template <int R = 1>
__device__ __forceinline__ void stage_bias(double* __restrict__ bl, const double* __restrict__ b, long long c0,
                                           long long n_bins) {
    if (c0 + kW <= n_bins) {
        constexpr int NV = kW / 2 / kSweepThreads / R;
        const double2* src = reinterpret_cast<const double2*>(b + c0);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            double2 v[NV];
#pragma unroll
            for (int k = 0; k < NV; ++k) v[k] = src[threadIdx.x + (r * NV + k) * kSweepThreads];
#pragma unroll
            for (int k = 0; k < NV; ++k) {
                const uint32_t e = 2u * (threadIdx.x + (r * NV + k) * kSweepThreads);
                bl[swz(e)] = v[k].x;
                bl[swz(e + 1)] = v[k].y;
            }
        }
    } else {
        for (int k = threadIdx.x; k < kW; k += kSweepThreads) bl[swz(k)] = c0 + k < n_bins ? b[c0 + k] : 0.0;
    }
}

// LDS of the three sweep bodies (one kernel each, or all three in one launch
// for small matrices: k_sweep_all, a union of the three)
template <bool UP>
struct TiledLds {
    double bl[kW];
    u64 cacc[UP ? kW : 1];  // column side of the current upper tile (rotated image)
    double acc2[2 * kR];  // narrow rows, then wide rows
    uint32_t rps[kR + 1], rpsn[kR + 1];
    uint16_t perm[2 * kR];
    uint16_t band[2 * kBandSlots];
};
template <bool UP>
struct FlatLds {
    double bl[kW];
    u64 cacc[UP ? kW : 1];
    double acc[kR];    // row sums (narrow + wide)
    double accc[kR];   // narrow sums by compact row
    uint16_t rec[kFrecU4 * 8];
};

// the block's column accumulator -> its slot (column order), zeroed for the
// next tile; every thread moves its own columns (no barrier between)
__device__ __forceinline__ void flush_cols(u64* __restrict__ cacc, u64* __restrict__ dst, int nthr) {
    for (int k = threadIdx.x; k < kW; k += nthr) {
        const uint32_t sk = swz((uint32_t)k);
        dst[k] = cacc[sk];
        cacc[sk] = 0;
    }
}

// One tiled-kernel work unit u.
template <int NB, int ABL, bool UP>
__device__ __forceinline__ void sweep_tiled_unit(const TileDev& T, const uint8_t* __restrict__ act, int u,
                                                 const double* __restrict__ b, long long n_bins,
                                                 double* __restrict__ part, TiledLds<UP>& L) {
    double* __restrict__ bl = L.bl;
    double* __restrict__ acc2 = L.acc2;
    uint32_t* __restrict__ rps = L.rps;
    uint32_t* __restrict__ rpsn = L.rpsn;
    uint16_t* __restrict__ perm = L.perm;
    uint16_t* __restrict__ band = L.band;
    {
        bool on = false;
        for (int g = T.u_glo[u]; g <= T.u_ghi[u]; ++g) on |= act[g] != 0;
        if (!on) return;
    }
    const int ra = T.u_rlo[u], rb = T.u_rhi[u];
    const bool whole = T.u_whole[u] != 0;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int k = threadIdx.x; k < 2 * (rb - ra); k += kSweepThreads) acc2[k] = 0.0;
    // upper-triangle tiles: the column side into L.cacc, one slot per tile
    const int urb = T.u_rb[u];
    const ColArgs ca{T.bfix + T.row_lo + (long long)urb * kR, L.cacc};
    const int upper = UP ? T.upper : 0;  // (UP: kernels with the column-side code)
    if (upper)
        for (int k = threadIdx.x; k < kW; k += kSweepThreads) L.cacc[k] = 0;
    int cslot = -1;  // the previous tile's column slot (its flush is pending)
    for (int t = T.u_tlo[u]; t < T.u_thi[u]; ++t) {
        const long long c0 = (long long)T.tile_J[t] * kW;
        __syncthreads();  // previous tile's LDS reads are done
        if (UP && cslot >= 0) flush_cols(L.cacc, T.colpart + (size_t)cslot * kW, kSweepThreads);
        const bool up = tile_is_upper(upper, T.row_lo, urb, T.tile_J[t]);
        cslot = up ? T.u_cslot[u] + (t - T.u_tlo[u]) : -1;
        if (ABL != 2) stage_bias(bl, b, c0, n_bins);  // ABL 2: timing ablation, no staging
        {
            const uint32_t* rpg = T.tile_rp + (size_t)t * (kR + 1);
            const uint32_t* rpgn = T.tile_rpn + (size_t)t * (kR + 1);
            for (int k = threadIdx.x; k <= kR; k += kSweepThreads) {
                rps[k] = rpg[k];
                rpsn[k] = rpgn[k];
            }
            if (whole) {
                const uint16_t* pg = T.tile_perm + (size_t)t * 2 * kR;
                for (int k = threadIdx.x; k < 2 * kR; k += kSweepThreads) perm[k] = pg[k];
                if (threadIdx.x < 2 * kBandSlots) band[threadIdx.x] = T.tile_band[(size_t)t * 2 * kBandSlots + threadIdx.x];
            }
        }
        __syncthreads();
        const uint32_t totn = rpsn[rb] - rpsn[ra], totw = rps[rb] - rps[ra];
        const uint4* payn4 = reinterpret_cast<const uint4*>(T.payn + T.tile_entn[t]);
        const uint4* payw4 = reinterpret_cast<const uint4*>(T.pay + T.tile_ent[t]);
        // narrow rows accumulate into acc2[0, nr), wide rows into acc2[nr, 2 nr):
        // disjoint, so the two passes need no barrier between them.  Lane-group
        // width from each segment's mean uint4 count per row.
        const int nr = rb - ra;
        if (whole) {  // ra == 0: acc2 index = row
            if (UP && cslot >= 0) {
                if (totn) sweep_bands<NB, ABL, 8, true>(band, payn4, rpsn, perm, bl, acc2, wave, lane, ca);
                if (totw)
                    sweep_bands<NB, ABL, 4, true>(band + kBandSlots, payw4, rps, perm + kR, bl, acc2 + nr, wave, lane,
                                                  ca);
            } else {
                if (totn) sweep_bands<NB, ABL, 8>(band, payn4, rpsn, perm, bl, acc2, wave, lane);
                if (totw) sweep_bands<NB, ABL, 4>(band + kBandSlots, payw4, rps, perm + kR, bl, acc2 + nr, wave, lane);
            }
        } else {
            if (UP && cslot >= 0) {
                if (totn)
                    sweep_rows<NB, ABL, 8, true>(totn / 8 / (uint32_t)nr, payn4, rpsn, bl, acc2, ra, rb, wave, lane, ca);
                if (totw)
                    sweep_rows<NB, ABL, 4, true>(totw / 4 / (uint32_t)nr, payw4, rps, bl, acc2 + nr, ra, rb, wave, lane,
                                                 ca);
            } else {
                if (totn) sweep_rows<NB, ABL, 8>(totn / 8 / (uint32_t)nr, payn4, rpsn, bl, acc2, ra, rb, wave, lane);
                if (totw) sweep_rows<NB, ABL, 4>(totw / 4 / (uint32_t)nr, payw4, rps, bl, acc2 + nr, ra, rb, wave, lane);
            }
        }
    }
    __syncthreads();
    if (UP && cslot >= 0) flush_cols(L.cacc, T.colpart + (size_t)cslot * kW, kSweepThreads);
    for (int k = threadIdx.x; k < rb - ra; k += kSweepThreads) part[T.u_slot[u] + k] = acc2[k] + acc2[(rb - ra) + k];
}

template <int NB, int ABL, bool UP>
__global__ __launch_bounds__(kSweepThreads, 4) void k_sweep_tiled(TileDev T, const uint8_t* __restrict__ act,
                                                                int n_list, const double* __restrict__ b,
                                                                long long n_bins, double* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) TiledLds<UP> L;
    if ((int)blockIdx.x >= n_list) return;
    sweep_tiled_unit<NB, ABL, UP>(T, act, T.u_order[blockIdx.x], b, n_bins, part, L);  // tiled units lead the list
}

// K1c: the flat tiles (whole row-blocks whose rows are all short).  Per
// tile the latency chain is kept to one hop: each wave's row / uint4 range
// (tile_fw, read one tile ahead) lets it issue the loads of its whole narrow
// run (U = 8 uint4 per lane: one step covers the typical tile) and its first
// wide run at once, while the block copies the bias slice and the tile's flat
// record (compacted row starts + row ids) into LDS in one pass; the narrow
// segment accumulates by compact row (flat_step_c), the few wide rows by row
// id, and after a barrier the compact sums are added to their rows.
template <int U, int ABL, bool UP>
__device__ __forceinline__ void sweep_flat_unit(const TileDev& T, const uint8_t* __restrict__ act, int u,
                                                const double* __restrict__ b, long long n_bins,
                                                double* __restrict__ part, FlatLds<UP>& L) {
    static_assert(kSweepWaves == kFlatWaves, "one plan split per wave");
    constexpr int UW = 2;  // wide runs: few wide entries in flat tiles
    double* __restrict__ bl = L.bl;
    double* __restrict__ acc = L.acc;
    double* __restrict__ accc = L.accc;
    uint16_t* __restrict__ rec = L.rec;
    {
        bool on = false;
        for (int g = T.u_glo[u]; g <= T.u_ghi[u]; ++g) on |= act[g] != 0;
        if (!on) return;
    }
    const int nr = T.u_rhi[u];  // whole row-block: rows [0, nr)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint16_t* fstn = rec;
    const uint16_t* fstw = rec + (kR + 1);
    const uint16_t* fidn = rec + 2 * (kR + 1);
    const uint16_t* fidw = fidn + kR;
    for (int k = threadIdx.x; k < nr; k += kSweepThreads) acc[k] = 0.0;
    const int urb = T.u_rb[u];
    const ColArgs ca{T.bfix + T.row_lo + (long long)urb * kR, L.cacc};
    const int upper = UP ? T.upper : 0;
    if (upper)
        for (int k = threadIdx.x; k < kW; k += kSweepThreads) L.cacc[k] = 0;
    int cslot = -1;
    const int t0 = T.u_tlo[u], t1 = T.u_thi[u];
    // a flat unit's tiles have consecutive flat records (plan order)
    const uint4* rg0 = T.frec + (size_t)T.tile_frec[t0] * kFrecU4;
    // the wave's split of tile t (wave-uniform scalars)
    struct Meta {
        uint32_t qan, qbn, qaw, qbw;
        int i0n, i1n, i0w, i1w, nfn, nfw, J;
        long long entn, ent;
    };
    auto meta = [&](int t) {
        const uint32_t* fw = T.tile_fw + (size_t)t * kFlatMeta;
        const uint32_t* fwn = fw + 2 * wave;
        const uint32_t* fww = fw + 2 * (kFlatWaves + 1) + 2 * wave;
        Meta m;
        m.qan = fwn[0], m.qbn = fwn[2], m.qaw = fww[0], m.qbw = fww[2];
        m.i0n = (int)fwn[1], m.i1n = (int)fwn[3], m.i0w = (int)fww[1], m.i1w = (int)fww[3];
        m.nfn = (int)fw[2 * kFlatWaves + 1], m.nfw = (int)fw[2 * (kFlatWaves + 1) + 2 * kFlatWaves + 1];
        m.J = T.tile_J[t];
        m.entn = T.tile_entn[t], m.ent = T.tile_ent[t];
        return m;
    };
    // The compact narrow sums of tile t are added to their rows after the
    // barrier that opens tile t + 1, beside its staging (row ids read from
    // tile t's record in global memory, an L2 hit: the LDS copy is being
    // replaced): two barriers per tile instead of three.
    const bool defer = T.flat_defer != 0;
    int nfn_prev = 0;
    const uint16_t* fidn_prev = nullptr;
    for (int t = t0; t < t1; ++t) {
        const Meta cm = meta(t);
        const uint32_t qan = cm.qan, qbn = cm.qbn, qaw = cm.qaw, qbw = cm.qbw;
        const int i0n = cm.i0n, i1n = cm.i1n, i0w = cm.i0w, i1w = cm.i1w, nfn = cm.nfn, nfw = cm.nfw;
        const uint4* payn4 = reinterpret_cast<const uint4*>(T.payn + cm.entn);
        const uint4* payw4 = reinterpret_cast<const uint4*>(T.pay + cm.ent);
        uint4 v[U], vw[UW];
        if (i0n < i1n) flat_load<U>(payn4, qan + (uint32_t)lane * U, qan, qbn, v);
        if (i0w < i1w) flat_load<UW>(payw4, qaw + (uint32_t)lane * UW, qaw, qbw, vw);
        const uint4* rg = rg0 + (size_t)(t - t0) * kFrecU4;
        __syncthreads();  // previous tile's walk (LDS reads, accc / acc writes) is done
        for (int k = threadIdx.x; k < nfn_prev; k += kSweepThreads) acc[fidn_prev[k]] += accc[k];
        if (UP && cslot >= 0) flush_cols(L.cacc, T.colpart + (size_t)cslot * kW, kSweepThreads);
        cslot = tile_is_upper(upper, T.row_lo, urb, cm.J) ? T.u_cslot[u] + (t - t0) : -1;
        if (ABL != 2) stage_bias(bl, b, (long long)cm.J * kW, n_bins);
        for (int k = threadIdx.x; k < kFrecU4; k += kSweepThreads) reinterpret_cast<uint4*>(rec)[k] = rg[k];
        __syncthreads();
        if (UP && cslot >= 0) {
            flat_seg_c<U, ABL, 8, true>(payn4, v, qan, qbn, i0n, i1n, fstn, nfn, bl, accc, lane, ca, fidn);
            flat_seg<UW, ABL, 4, true>(payw4, vw, qaw, qbw, i0w, i1w, fstw, fidw, nfw, bl, acc, lane, ca);
        } else {
            flat_seg_c<U, ABL, 8>(payn4, v, qan, qbn, i0n, i1n, fstn, nfn, bl, accc, lane);
            flat_seg<UW, ABL, 4>(payw4, vw, qaw, qbw, i0w, i1w, fstw, fidw, nfw, bl, acc, lane);
        }
        if (defer) {
            nfn_prev = nfn;
            fidn_prev = reinterpret_cast<const uint16_t*>(rg) + 2 * (kR + 1);
        } else {  // round-1 order: a third barrier, merge from the LDS record
            __syncthreads();
            for (int k = threadIdx.x; k < nfn; k += kSweepThreads) acc[fidn[k]] += accc[k];
        }
    }
    __syncthreads();  // the last tile's compact sums complete
    for (int k = threadIdx.x; k < nfn_prev; k += kSweepThreads) acc[fidn_prev[k]] += accc[k];
    if (UP && cslot >= 0) flush_cols(L.cacc, T.colpart + (size_t)cslot * kW, kSweepThreads);
    __syncthreads();
    for (int k = threadIdx.x; k < nr; k += kSweepThreads) part[T.u_slot[u] + k] = acc[k];
}

template <int U, int ABL, bool UP>
__global__ __launch_bounds__(kSweepThreads, 4) void k_sweep_flat(TileDev T, const uint8_t* __restrict__ act,
                                                               int n_list, int list_off,
                                                               const double* __restrict__ b, long long n_bins,
                                                               double* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) FlatLds<UP> L;
    if ((int)blockIdx.x >= n_list) return;
    sweep_flat_unit<U, ABL, UP>(T, act, T.u_order[list_off + blockIdx.x], b, n_bins, part, L);
}

// K1c' (round 3): the flat tiles swept by column tile.  A block takes a
// group of up to g_flat_group (auto: 11 .. 44) flat tiles sharing one column tile J (different
// row-blocks), stages b[J] once, and each of its 8 waves then walks whole
// tiles on its own -- the next tile of the group from an LDS counter, the
// tile's flat record in a per-wave LDS slot, its row sums in a per-wave LDS
// accumulator, written out as that tile's unit partials.  No block barrier
// per tile: the waves' load / walk / write chains drift apart and overlap
// (the round-2 kernel ran one tile at a time per block with two barriers per
// tile and re-staged 64 KB of b for every ~100 KB of sparse payload).  Per
// tile the walk is the round-2 one with the whole tile as the wave's range,
// so a row's sum is a fixed function of the tile: deterministic, and the
// same wherever the tile is swept.

template <int NW, bool UP>
struct FlatWLds {
    double bl[kW];
    u64 cacc[UP ? kW : 1];  // the group's column side (its strictly upper tiles), one slot per group
    uint16_t rec[NW][kFrecU4 * 8];
    double acc[NW][kR];
    int next;
};

__device__ __forceinline__ void wave_lds_sync() {
    // one wave's LDS writes before its later LDS reads (the LDS queue is in
    // order per wave; this orders the compiler and waits for the writes)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}


// NW waves per block share one staged b[J]: the LDS (64 KB of bias + 8 KB
// per wave) caps the block at 11 waves, and one block per CU is all that fits
template <int U, int ABL, int PIPE = 2, int NW = kFlatWaves, bool UP = false>
__global__ __launch_bounds__(NW * 64, NW > 8 ? 3 : 2) void k_sweep_flatw(TileDev T, const uint8_t* __restrict__ act,
                                                                       const double* __restrict__ b, long long n_bins,
                                                                       double* __restrict__ part) {
    constexpr int UW = 2;
    __shared__ __attribute__((aligned(16))) FlatWLds<NW, UP> L;
    const int k0 = T.fg_ptr[blockIdx.x], nk = T.fg_ptr[blockIdx.x + 1] - k0;
    {
        bool on = false;  // block-uniform: any active tile in the group
        for (int k = 0; k < nk && !on; ++k) {
            const int u = T.fg_unit[k0 + k];
            for (int g = T.u_glo[u]; g <= T.u_ghi[u]; ++g) on |= act[g] != 0;
        }
        if (!on) return;
    }
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int J = T.tile_J[T.u_tlo[T.fg_unit[k0]]];
    const FlatDesc* __restrict__ desc = T.fg_desc + k0;
    const int cslot = UP && T.upper ? T.fg_cslot[blockIdx.x] : -1;
    if (threadIdx.x == 0) L.next = 0;
    if (ABL != 2 && threadIdx.x < kSweepThreads) stage_bias(L.bl, b, (long long)J * kW, n_bins);
    if (cslot >= 0)
        for (int k = threadIdx.x; k < kW; k += NW * 64) L.cacc[k] = 0;
    __syncthreads();
    const double* __restrict__ bl = L.bl;
    uint16_t* __restrict__ rec = L.rec[wave];
    double* __restrict__ acc = L.acc[wave];
    const uint16_t* fstn = rec;
    const uint16_t* fstw = rec + (kR + 1);
    const uint16_t* fidn = rec + 2 * (kR + 1);
    const uint16_t* fidw = fidn + kR;
    struct Tw {
        int slot, frec, nr, nfn, nfw;
        uint32_t qbn, qbw;
        const uint4 *payn4, *payw4;
        int up;
        const u64* bblk;
    };
    // the group's next active tile (LDS counter), false when none is left:
    // one descriptor load (round 3; it was unit -> tile -> split / entries,
    // four dependent lookups per tile)
    auto grab = [&](Tw& x) -> bool {
        for (;;) {
            int k = 0;
            if (lane == 0) k = atomicAdd(&L.next, 1);
            k = __builtin_amdgcn_readfirstlane(__shfl(k, 0, 64));
            if (k >= nk) return false;
            const FlatDesc d = desc[k];
            // the tile's row groups' active flags, one per lane (one round
            // trip; a loop over the groups compiled to one load -> wait each)
            bool on = false;
            const int ngr = d.ghi - d.glo + 1;
            if (ngr <= 64) {
                const uint8_t a = act[d.glo + (lane < ngr ? lane : ngr - 1)];
                on = __ballot((a != 0) & (lane < ngr)) != 0;
            } else {
                for (int g = d.glo; g <= d.ghi; ++g) on |= act[g] != 0;
            }
            if (!on) continue;  // a converged group's rows: k_marg never reads them
            x = Tw{d.slot, d.frec, (int)d.nr, (int)d.nfn, (int)d.nfw, d.qbn, d.qbw,
                   reinterpret_cast<const uint4*>(T.payn + d.entn), reinterpret_cast<const uint4*>(T.pay + d.ent),
                   cslot >= 0 && d.upper ? 1 : 0, T.bfix + T.row_lo + (long long)d.rb * kR};
            return true;
        }
    };
    Tw cur;
    const bool any = grab(cur);
    uint4 v[U], vw[UW];
    if (any && cur.nfn) flat_load_ilv<U>(cur.payn4, 0u, cur.qbn, lane, v);
    if (any && cur.nfw) flat_load<UW>(cur.payw4, (uint32_t)lane * UW, 0u, cur.qbw, vw);
    for (; any;) {
        const uint4* rg = T.frec + (size_t)cur.frec * kFrecU4;
        // stage only the parts of the record the walk reads (the starts up
        // to each segment's end, the row ids of the nonempty rows), and no
        // narrow row ids when every row of the block is nonempty (they are
        // then 0, 1, 2, ...: the dense trans tiles): ~1.1 of 4.1 KB per tile
        const bool idn = cur.nfn == cur.nr;
        {
            // the four uint16 ranges [h0, h1) of the record the walk reads,
            // each at most 65 uint4 (kR = 512): two uint4 per lane.  All
            // eight loads are issued before the first LDS store (a load loop
            // per range compiled to load -> vmcnt(0) -> store, four to eight
            // round trips per tile); a lane past a range's end re-reads the
            // range's first uint4 (the same line: no extra bytes)
            // and stores its copy back to the same LDS slot (no branch around
            // the stores either, which would bring the waits back)
            static_assert((kR + 1 + 7) / 8 + 1 <= 2 * 64, "record range > 2 uint4 per lane");
            uint4* r4 = reinterpret_cast<uint4*>(rec);
            const int h0[4] = {0, kR + 1, 2 * (kR + 1), 2 * (kR + 1) + kR};
            const int h1[4] = {cur.nfn + 1, kR + 1 + cur.nfw + 1, idn ? 2 * (kR + 1) : 2 * (kR + 1) + cur.nfn,
                               2 * (kR + 1) + kR + cur.nfw};
            uint4 tq[4][2];
            int qs[4][2];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int q0 = h0[g] / 8, q1 = (h1[g] + 7) / 8;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int q = q0 + lane + 64 * h;
                    qs[g][h] = q < q1 ? q : q0;
                    tq[g][h] = rg[qs[g][h]];
                }
            }
#pragma unroll
            for (int g = 0; g < 4; ++g)
#pragma unroll
                for (int h = 0; h < 2; ++h) r4[qs[g][h]] = tq[g][h];
        }
        wave_lds_sync();
        const ColArgs ca{cur.bblk, L.cacc};
        if (UP && cur.up) {  // (not software-pipelined: the column side needs the registers)
            flat_seg_c<U, ABL, 8, true, true>(cur.payn4, v, 0u, cur.qbn, 0, cur.nfn, fstn, cur.nfn, bl, acc, lane,
                                              ca, idn ? nullptr : fidn);
        } else {
            if (PIPE)
                flat_seg_c_pipe<U, ABL, 8, false, true>(cur.payn4, v, 0u, cur.qbn, 0, cur.nfn, fstn, cur.nfn, bl, acc,
                                                        lane);
            else
                flat_seg_c<U, ABL, 8, false, true>(cur.payn4, v, 0u, cur.qbn, 0, cur.nfn, fstn, cur.nfn, bl, acc, lane);
        }
        wave_lds_sync();
        // compact narrow sums -> rows (zeros for rows without narrow entries)
        constexpr int PL = kR / 64;
        double cv[PL];
        int cid[PL];
#pragma unroll
        for (int q = 0; q < PL; ++q) {
            const int i = lane + 64 * q;
            cv[q] = i < cur.nfn ? acc[i] : 0.0;
            cid[q] = i < cur.nfn ? (idn ? i : (int)fidn[i]) : -1;
        }
        wave_lds_sync();
#pragma unroll
        for (int q = 0; q < PL; ++q) acc[lane + 64 * q] = 0.0;
        wave_lds_sync();
#pragma unroll
        for (int q = 0; q < PL; ++q)
            if (cid[q] >= 0) acc[cid[q]] = cv[q];
        wave_lds_sync();
        if (UP && cur.up) {
            if (PIPE)
                flat_seg_pipe<UW, ABL, 4, true>(cur.payw4, vw, 0u, cur.qbw, 0, cur.nfw, fstw, fidw, cur.nfw, bl, acc, lane,
                                                ca);
            else flat_seg<UW, ABL, 4, true>(cur.payw4, vw, 0u, cur.qbw, 0, cur.nfw, fstw, fidw, cur.nfw, bl, acc, lane, ca);
        } else {
            if (PIPE) flat_seg_pipe<UW, ABL, 4>(cur.payw4, vw, 0u, cur.qbw, 0, cur.nfw, fstw, fidw, cur.nfw, bl, acc, lane);
            else flat_seg<UW, ABL, 4>(cur.payw4, vw, 0u, cur.qbw, 0, cur.nfw, fstw, fidw, cur.nfw, bl, acc, lane);
        }
        wave_lds_sync();
        // PIPE 2: the next tile's first runs are in flight while this tile's
        // row sums go out
        Tw nxt;
        bool more = false;
        if (PIPE == 2) {
            more = grab(nxt);
            if (more) {
                if (nxt.nfn) flat_load_ilv<U>(nxt.payn4, 0u, nxt.qbn, lane, v);
                if (nxt.nfw) flat_load<UW>(nxt.payw4, (uint32_t)lane * UW, 0u, nxt.qbw, vw);
            }
        }
        double* __restrict__ out = part + cur.slot;
        for (int r = lane; r < cur.nr; r += 64) out[r] = acc[r];
        wave_lds_sync();  // this tile's LDS reads before the next tile's writes
        if (PIPE != 2) {
            more = grab(nxt);
            if (more) {
                if (nxt.nfn) flat_load_ilv<U>(nxt.payn4, 0u, nxt.qbn, lane, v);
                if (nxt.nfw) flat_load<UW>(nxt.payw4, (uint32_t)lane * UW, 0u, nxt.qbw, vw);
            }
        }
        if (!more) break;
        cur = nxt;
    }
    if (UP && cslot >= 0) {  // every wave's adds are in: the group's column partial out
        __syncthreads();
        flush_cols(L.cacc, T.colpart + (size_t)cslot * kW, NW * 64);
    }
}

// ---- diagnostics (hh_matrix_stream_probe): read rates of the layout's own
// buffers without any of the sweep's work, to separate what the buffers and
// access shapes allow from what the sweep kernels' structure costs.
// A linear grid-stride read, 8 uint4 per lane in flight.
// LM: lane-major runs (thread t reads U consecutive uint4, as the flat walk
// loads them) instead of coalesced instructions.
template <bool LM = false>
__global__ __launch_bounds__(256) void k_stream_probe(const uint4* __restrict__ p, long long n16,
                                                      unsigned* __restrict__ sink) {
    constexpr int U = 8;
    uint32_t x = 0;
    const long long step = (long long)gridDim.x * 256 * U;
    for (long long b0 = (long long)blockIdx.x * 256 * U; b0 < n16; b0 += step) {
        const long long i0 = LM ? b0 + (long long)threadIdx.x * U : b0 + threadIdx.x;
        uint4 v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const long long i = LM ? i0 + k : i0 + 256LL * k;
            v[k] = ld16(p + (i < n16 ? i : b0));
        }
#pragma unroll
        for (int k = 0; k < U; ++k) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    if (x == 0x9E3779B9u) sink[0] = x;
}

// The flat tiles' payload as k_sweep_flatw reaches it (column groups, a wave
// per tile from an LDS counter, one descriptor load per tile, two runs of U
// uint4 per lane in flight) but streamed only: no record, no walk, no bias.
// COAL: each run loaded as U coalesced instructions (lane l reads uint4 q0 +
// 64 j + l) instead of the walk's lane-major runs (lane l reads q0 + U l + j).
template <int U>
__device__ __forceinline__ void flat_load_coal(const uint4* __restrict__ pay4, uint32_t q0, uint32_t qb, int lane,
                                               uint4 (&v)[U]) {
    const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const uint32_t q = q0 + 64u * k + (uint32_t)lane;
        const bool on = q < qb;
        const uint4 x = ld16(pay4 + (on ? q : 0u));
        v[k] = on ? x : zero;
    }
}
template <int NW, int PADB, bool COAL = false>
__global__ __launch_bounds__(NW * 64) void k_flat_stream_probe(TileDev T, unsigned* __restrict__ sink) {
    constexpr int U = kFlatU, UW = 2;
    __shared__ int next;
    __shared__ uint4 pad[PADB / 16 > 0 ? PADB / 16 : 1];  // the sweep kernel's LDS footprint (occupancy)
    const int k0 = T.fg_ptr[blockIdx.x], nk = T.fg_ptr[blockIdx.x + 1] - k0;
    if (threadIdx.x == 0) next = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    uint32_t x = 0;
    for (;;) {
        int k = 0;
        if (lane == 0) k = atomicAdd(&next, 1);
        k = __builtin_amdgcn_readfirstlane(__shfl(k, 0, 64));
        if (k >= nk) break;
        const FlatDesc d = T.fg_desc[k0 + k];
        const uint4* pn = reinterpret_cast<const uint4*>(T.payn + d.entn);
        const uint4* pw = reinterpret_cast<const uint4*>(T.pay + d.ent);
        uint4 a[U], c[UW];
        if (d.qbn) {
            if (COAL) flat_load_coal<U>(pn, 0u, d.qbn, lane, a);
            else flat_load<U>(pn, (uint32_t)lane * U, 0u, d.qbn, a);
        }
        if (d.qbw) flat_load<UW>(pw, (uint32_t)lane * UW, 0u, d.qbw, c);
        for (uint32_t q0 = 0; q0 < d.qbn; q0 += 64u * U) {
            uint4 bn[U];
            const uint32_t qn = q0 + 64u * U;
            if (qn < d.qbn) {
                if (COAL) flat_load_coal<U>(pn, qn, d.qbn, lane, bn);
                else flat_load<U>(pn, qn + (uint32_t)lane * U, 0u, d.qbn, bn);
            }
#pragma unroll
            for (int j = 0; j < U; ++j) x ^= a[j].x ^ a[j].y ^ a[j].z ^ a[j].w;
            if (qn >= d.qbn) break;
#pragma unroll
            for (int j = 0; j < U; ++j) a[j] = bn[j];
        }
        for (uint32_t q0 = 0; q0 < d.qbw; q0 += 64u * UW) {
            uint4 bw[UW];
            const uint32_t qn = q0 + 64u * UW;
            if (qn < d.qbw) flat_load<UW>(pw, qn + (uint32_t)lane * UW, 0u, d.qbw, bw);
#pragma unroll
            for (int j = 0; j < UW; ++j) x ^= c[j].x ^ c[j].y ^ c[j].z ^ c[j].w;
            if (qn >= d.qbw) break;
#pragma unroll
            for (int j = 0; j < UW; ++j) c[j] = bw[j];
        }
    }
    if (x == 0x9E3779B9u) {
        pad[lane] = make_uint4(x, 0u, 0u, 0u);
        sink[0] = pad[(lane + 1) & 63].x;
    }
}

// ---------------------------------------------------------------- K2
// marg_r = b_r * (sum of the row's unit partials + wide entries + 2 diag b_r)
// K1b: the dense diagonal bands (uint8 counts near the diagonal, 4-bit
// counts beyond).  A band segment is a per-row run of slots s = 0, 1, ... for
// the diagonals d = dlo + s (zero padding at the end).  One block per
// (256-row block, 2048-byte chunk of the segment).  Row r is read in 16-byte
// groups (G = 128 / BITS slots) shifted back by m = r mod G, so the bias
// column of group l's slot k is (r - m) + dlo + s0 + G l + k: the window
// index (r & ~(G-1)) + G l + k is G-aligned per lane and the padded LDS
// address (one double of padding per G, conflict-free for the 64 lanes'
// stride-(G+1) reads) is p0 + k -- an immediate offset, no address
// arithmetic per count.  A lane's G shifted counts come from the previous
// and its own 16 bytes (two coalesced loads, the second an L1 hit; one
// alignbit per dword, the dword choice is wave-uniform).  Two rows in flight
// per wave, fixed per-lane order + xor-tree wave reduction: deterministic.
constexpr int kBandThreads = 512;
constexpr int kBandChunkB = kBandChunk;  // bytes of a segment per block
template <int BITS, int ROWS>
struct BandGeo {
    static constexpr int G = 128 / BITS;                 // slots per 16-byte group
    static constexpr int CS = kBandChunkB * 8 / BITS;    // slots per chunk
    static constexpr int WIN = ROWS + CS;                // window values
    static constexpr int LDS = WIN + WIN / G + 1;
};
template <int G>
__device__ __forceinline__ int bpadg(int k) { return k + k / G; }

// bits [128 - BITS m, 256 - BITS m) of prev ++ own (m < G, wave-uniform):
// output dword i = alignbit(d[q + i + 1], d[q + i], r) with B = 128 - BITS m,
// q = B / 32, r = B % 32.  Q is a template parameter so each case reads its
// source registers directly (a runtime dword choice costs a v_mov per dword).
template <int Q>
__device__ __forceinline__ uint4 band_shift_q(const uint4 prev, const uint4 own, int r) {
    const uint32_t d[9] = {prev.x, prev.y, prev.z, prev.w, own.x, own.y, own.z, own.w, 0u};
    if (r == 0) return make_uint4(d[Q], d[Q + 1], d[Q + 2], d[Q + 3]);
    return make_uint4(__builtin_amdgcn_alignbit(d[Q + 1], d[Q], r), __builtin_amdgcn_alignbit(d[Q + 2], d[Q + 1], r),
                      __builtin_amdgcn_alignbit(d[Q + 3], d[Q + 2], r), __builtin_amdgcn_alignbit(d[Q + 4], d[Q + 3], r));
}

// the row's counts shifted back by m slots (its 16-byte group aligned to the
// window)
template <int BITS>
__device__ __forceinline__ uint4 band_shifted(const uint4 prev, const uint4 own, int m) {
    const int B = 128 - BITS * m, r = B & 31;
    switch (B >> 5) {  // wave-uniform
        case 0: return band_shift_q<0>(prev, own, r);
        case 1: return band_shift_q<1>(prev, own, r);
        case 2: return band_shift_q<2>(prev, own, r);
        case 3: return band_shift_q<3>(prev, own, r);
        default: return band_shift_q<4>(prev, own, 0);  // m = 0
    }
}

// acc + the dot of half H of a shifted group (dwords 2H, 2H + 1: slots
// [H G/2, (H + 1) G/2)) with those slots' window values: the window is held
// in registers half at a time (G = 32 doubles for the 4-bit band was 64
// VGPRs), same summation order as one pass over the G slots
template <int BITS, int H>
__device__ __forceinline__ double band_dot_half(const uint4 v, const double* __restrict__ wh, double acc) {
    const unsigned x[2] = {H == 0 ? v.x : v.z, H == 0 ? v.y : v.w};
    constexpr int G2 = 64 / BITS, PER = 32 / BITS;
    constexpr unsigned MASK = (1u << BITS) - 1u;
#pragma unroll
    for (int k = 0; k < G2; ++k) acc = fma((double)((x[k / PER] >> (BITS * (k % PER))) & MASK), wh[k], acc);
    return acc;
}

// The band segments of one sweep (uint8 band; 4-bit band, negative and
// positive diagonals): slot s of a segment row <-> diagonal dlo + s; its nc
// chunks are grid rows [y0, y0 + nc) and write bpart chunks [ch, ch + nc).
struct BandSeg {
    const uint8_t* seg;
    long long stride, dlo;
    int bytes, nc, ch, bits;
};
constexpr int kMaxBandChunks = 64;
struct BandSegs {
    BandSeg s[3];
    int n;
    // grid row -> bpart chunk (heaviest chunks dispatched first: full 4-bit
    // chunks, full uint8 chunks, then the partial last chunks, so the light
    // blocks form the launch's tail; the chunk -> partial mapping is unchanged)
    uint8_t ord[kMaxBandChunks];
};

// One (ROWS-row block, 2048-byte chunk) of one segment.  ROWS = 256 on big
// matrices; 64 when the grid would not fill the chip (a wave walks ROWS / 8
// rows in sequence: on a single chromosome the 256-row chain, not the bytes,
// set the time).  A row's partial does not depend on ROWS (lane -> slot and
// the summation order are fixed by the row alone): bitwise the same sweep.
// lane l <- lane l - 1 (lane 0 <- 0): DPP wave_shr:1, no LDS
__device__ __forceinline__ uint4 dpp_shr1(const uint4 v) {
    return make_uint4(__builtin_amdgcn_update_dpp(0u, v.x, 0x138, 0xF, 0xF, false),
                      __builtin_amdgcn_update_dpp(0u, v.y, 0x138, 0xF, 0xF, false),
                      __builtin_amdgcn_update_dpp(0u, v.z, 0x138, 0xF, 0xF, false),
                      __builtin_amdgcn_update_dpp(0u, v.w, 0x138, 0xF, 0xF, false));
}

template <int BITS, int ABL, int ROWS, bool DPP = true>
__device__ __forceinline__ void band_block(const BandSeg& P, int rblk, int chunk, double* __restrict__ bl,
                                           uint8_t* __restrict__ ract, long long nloc, long long row_lo,
                                           long long n_bins, const uint8_t* __restrict__ act,
                                           const uint16_t* __restrict__ row_group, const double* __restrict__ b,
                                           double* __restrict__ bpart) {
    using Geo = BandGeo<BITS, ROWS>;
    constexpr int G = Geo::G;
    const uint8_t* __restrict__ seg = P.seg;
    const long long row_stride = P.stride;
    const long long r0 = (long long)rblk * ROWS;
    const int c0 = chunk * kBandChunkB, c1 = min(c0 + kBandChunkB, P.bytes);  // bytes
    const int s0 = c0 * 8 / BITS, s1 = c1 * 8 / BITS;                          // slots
    const int nr = (int)min((long long)ROWS, nloc - r0);
    const long long g0 = row_lo + r0 + P.dlo + s0;  // bias column of window index 0
    const int len = ((nr + G - 1) & ~(G - 1)) + (s1 - s0);
    for (int k = threadIdx.x; k < (ABL == 2 ? 0 : len); k += kBandThreads) {  // ABL 2: no staging (timing)
        // the band multiplies implicit zeros too: a NaN bias (an empty group
        // in cis-only mode, whose bins no stored pixel touches) must read 0
        const long long c = g0 + k;
        const double v = (c >= 0 && c < n_bins) ? b[c] : 0.0;
        bl[bpadg<G>(k)] = v == v ? v : 0.0;
    }
    for (int k = threadIdx.x; k < nr; k += kBandThreads) ract[k] = act[row_group[r0 + k]] != 0;
    __syncthreads();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    constexpr int NW = kBandThreads / 64;
    constexpr int RJ = 2;       // rows of a G-aligned row group handled together: they share the window
    constexpr int RPG = G / NW; // rows of a G-group per wave
    static_assert(G % NW == 0 && RPG % RJ == 0 && ROWS % G == 0, "whole rows per wave and group");
    const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
    double* __restrict__ out = bpart + (long long)(P.ch + chunk) * nloc;
    for (int gh = 0; gh < (nr + G - 1) / G * (RPG / RJ); ++gh) {
        // rows gb + wave + NW (j0 + j) (shift m = wave + NW (j0 + j), uniform):
        // the window values of a lane's slot group are read from LDS once for
        // the RJ rows
        const int gb = (gh / (RPG / RJ)) * G, j0 = (gh % (RPG / RJ)) * RJ;
        bool a[RJ];
#pragma unroll
        for (int j = 0; j < RJ; ++j) {
            const int r = gb + wave + NW * (j0 + j);
            a[j] = r < nr && ract[r] != 0;
        }
        double acc[RJ];
#pragma unroll
        for (int j = 0; j < RJ; ++j) acc[j] = 0.0;
        uint4 last[RJ];  // lane 63's bytes of the first half (the second half's lane 0 prev)
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            const int l = lane + 64 * g;
            const int cb = c0 + 16 * l;
            uint4 own[RJ], prev[RJ];
#pragma unroll
            for (int j = 0; j < RJ; ++j) {
                const uint8_t* row = seg + (r0 + gb + wave + NW * (j0 + j)) * row_stride;
                const bool on = a[j] && cb < c1, onp = on && cb >= 16;
                const uint4 x = ld16(reinterpret_cast<const uint4*>(on ? row + cb : seg));
                own[j] = on ? x : zero;
                if (DPP) {
                    // the previous 16 bytes are lane l - 1's: one DPP shift per
                    // dword instead of a second (L1-hit) load per lane; lane 0
                    // loads the chunk's preceding group (first half) or takes
                    // lane 63's of the first half
                    uint4 y = dpp_shr1(own[j]);
                    if (g == 0) {
                        if (lane == 0 && onp) y = ld16(reinterpret_cast<const uint4*>(row + cb - 16));
                    } else if (lane == 0) {
                        y = last[j];
                    }
                    prev[j] = onp ? y : zero;
                } else {
                    const uint4 y = ld16(reinterpret_cast<const uint4*>(onp ? row + cb - 16 : seg));
                    prev[j] = onp ? y : zero;
                }
            }
            if (DPP && g == 0) {
#pragma unroll
                for (int j = 0; j < RJ; ++j)
                    last[j] = make_uint4(__builtin_amdgcn_readlane(own[j].x, 63), __builtin_amdgcn_readlane(own[j].y, 63),
                                         __builtin_amdgcn_readlane(own[j].z, 63), __builtin_amdgcn_readlane(own[j].w, 63));
            }
            if (ABL == 1) {  // timing ablation: stream only
#pragma unroll
                for (int j = 0; j < RJ; ++j) acc[j] += (double)(own[j].x + own[j].y + own[j].z + own[j].w + prev[j].x);
            } else if (cb < c1) {
                uint4 sh[RJ];
#pragma unroll
                for (int j = 0; j < RJ; ++j) sh[j] = band_shifted<BITS>(prev[j], own[j], wave + NW * (j0 + j));
                const double* b0 = bl + bpadg<G>(gb + G * l);
                {
                    double w[G / 2];
#pragma unroll
                    for (int k = 0; k < G / 2; ++k) w[k] = b0[k];
#pragma unroll
                    for (int j = 0; j < RJ; ++j) acc[j] = band_dot_half<BITS, 0>(sh[j], w, acc[j]);
                }
                {
                    double w[G / 2];
#pragma unroll
                    for (int k = 0; k < G / 2; ++k) w[k] = b0[G / 2 + k];
#pragma unroll
                    for (int j = 0; j < RJ; ++j) acc[j] = band_dot_half<BITS, 1>(sh[j], w, acc[j]);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < RJ; ++j) {
            const double t = wave_sum(acc[j]);
            if (lane == 0 && a[j]) out[r0 + gb + wave + NW * (j0 + j)] = t;
        }
    }
}

// All band segments of a sweep in one launch (grid.y = their chunks, uint8
// first): the three used to run back to back, each with its own ramp and
// tail.  Registers / LDS are the larger (4-bit) body's.
template <int ROWS>
struct BandLds {
    static constexpr int L8 = BandGeo<8, ROWS>::LDS, L4 = BandGeo<4, ROWS>::LDS;
    double bl[L8 > L4 ? L8 : L4];
    uint8_t ract[ROWS];  // active flag per row (no dependent global loads in the row loop)
};

// grid row y of the band launch -> segment and its chunk
template <int ABL, int ROWS, bool DPP = true>
__device__ __forceinline__ void band_any(const BandSegs& S, int rblk, int y, BandLds<ROWS>& L, long long nloc,
                                         long long row_lo, long long n_bins, const uint8_t* __restrict__ act,
                                         const uint16_t* __restrict__ row_group, const double* __restrict__ b,
                                         double* __restrict__ bpart) {
    const int c = S.ord[y];
    int k = 0;
    while (k + 1 < S.n && c >= S.s[k + 1].ch) ++k;
    const BandSeg P = S.s[k];
    if (P.bits == 8)
        band_block<8, ABL, ROWS, DPP>(P, rblk, c - P.ch, L.bl, L.ract, nloc, row_lo, n_bins, act, row_group, b, bpart);
    else
        band_block<4, ABL, ROWS, DPP>(P, rblk, c - P.ch, L.bl, L.ract, nloc, row_lo, n_bins, act, row_group, b, bpart);
}

template <int ABL, int ROWS, bool DPP = true>
__global__ __launch_bounds__(kBandThreads, 4) void k_sweep_bands(BandSegs S, long long nloc, long long row_lo,
                                                              long long n_bins, const uint8_t* __restrict__ act,
                                                              const uint16_t* __restrict__ row_group,
                                                              const double* __restrict__ b,
                                                              double* __restrict__ bpart) {
    __shared__ BandLds<ROWS> L;
    band_any<ABL, ROWS, DPP>(S, blockIdx.x, blockIdx.y, L, nloc, row_lo, n_bins, act, row_group, b, bpart);
}

// ---------------------------------------------------------------- K1d
// Upper-band sweep (hh_tune "uband", default on).
// The band arrays hold both triangles (row r: diagonals -W..W); this sweep
// reads only the upper half of every row (diagonals d >= 0: half the bytes)
// and lets each count feed both marginals it belongs to: row r gets
// cnt * b[r + d] (row part) and column r + d gets cnt * b[r] (column part),
// from one load and one conversion.
//
// Work: one wave per (512-row block, chunk of 1008 slots); a workgroup is 4
// consecutive row blocks (2048 rows, globally aligned) of one chunk.  A wave
// walks its rows in groups of 16; row r = gb + m is read shifted back by m
// slots (funnel shift of the lane's previous and own bytes), so lane l's 16
// counts of every row of the group sit in the same 16 columns
// gb + base + 16 l + [0, 16) (base = diagonal of the chunk's slot 0), and
//   w[16]  (registers) the bias of those columns, shared by the 16 rows,
//   c[16]  (registers) the columns' partial column sums: c += cnt * b[row].
// Row part: a dot per row, reduced across the wave by a halving butterfly.
// After a group the lane windows move up 16 columns = one lane: w and c move
// down one lane (DPP wave_shl:1), the lowest lane's 16 sums are complete (the
// head, written to LDS), lane 63 takes the new window and starts from 0.  After
// the last group the lanes hold the partial sums of the next 1008 columns (the
// tail): added to the workgroup's LDS column buffer in two rounds (even
// waves, then odd: their tails are disjoint), giving H (the workgroup's 2048
// columns) and T (the next 1008, which belong to the next workgroup's heads).
// Every sum's order is fixed by global positions only: deterministic, and the
// same in a shard, which sweeps (from a halo copy of the rows above it) every
// workgroup whose columns reach its rows.
constexpr int kUbRows = 128;                       // rows per wave task (the length of its serial walk)
constexpr int kUbWaves = 4;                        // row blocks per workgroup
constexpr int kUbThreads = 64 * kUbWaves;
constexpr int kUbGroupRows = kUbRows * kUbWaves;   // rows per workgroup (global alignment)
constexpr int kUbChunk = 1008;                     // slots per chunk = 63 data lanes x 16
constexpr int kUbCols = kUbGroupRows + kUbChunk;   // LDS column buffer (doubles)
// a workgroup's rows are all local or all halo only because shards are cut
// at whole kR-row blocks: keep the workgroup a divisor of the row block
static_assert(kR % kUbGroupRows == 0, "upper-band workgroups must not straddle a shard's row-block boundary");
// a workgroup's tails reach kUbTails workgroups ahead: per chunk the partial
// arrays R (row parts), H (heads), T1 .. T_kUbTails (tails of the workgroups
// 1 .. kUbTails behind)
constexpr int kUbTails = (kUbChunk + kUbGroupRows - 1) / kUbGroupRows;
constexpr int kUbArrs = 2 + kUbTails;
constexpr int kMaxUbChunks = 40;

struct UbSeg {
    const uint8_t* loc;   // slot 0 of local row row_lo
    const uint8_t* halo;  // slot 0 of halo row halo_lo (shards)
    long long stride;     // bytes per row
    long long dlo;        // diagonal of slot 0
    int bytes;            // readable bytes of a row from slot 0 (zero padding included)
    int nc, ch, bits;     // chunks, first chunk index, bits per count
};
struct UbSegs {
    UbSeg s[2];
    int n;
    uint8_t ord[kMaxUbChunks];  // grid row -> chunk (heaviest first)
};
struct UbArgs {
    long long row_lo, row_hi, halo_lo, nloc, g_lo;
    const uint8_t* act;
    const uint16_t* row_group;
    const double* b;
    double* upart;  // per chunk c: R at kUbArrs c, H at + 1, T1.. at + 2.., nloc each
};

template <int BITS>
struct UbT;
template <>
struct UbT<8> {
    typedef uint4 V;
    static constexpr int LB = 16;  // bytes per lane per row
    static __device__ __forceinline__ V zero() { return make_uint4(0u, 0u, 0u, 0u); }
    static __device__ __forceinline__ V ld(const uint8_t* p) { return ld16(reinterpret_cast<const uint4*>(p)); }
    template <int M>
    static __device__ __forceinline__ V shift(const V prev, const V own) {
        if (M == 0) return own;
        constexpr int B = 128 - 8 * M;
        return band_shift_q<B / 32>(prev, own, B % 32);
    }
    static __device__ __forceinline__ uint32_t cnt(const V v, int k) {
        const uint32_t x = k < 4 ? v.x : k < 8 ? v.y : k < 12 ? v.z : v.w;
        return (x >> (8 * (k & 3))) & 0xFFu;
    }
};
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
template <>
struct UbT<4> {
    typedef uint2 V;
    static constexpr int LB = 8;
    static __device__ __forceinline__ V zero() { return make_uint2(0u, 0u); }
    static __device__ __forceinline__ V ld(const uint8_t* p) {
        const u32x2 v = *reinterpret_cast<const u32x2*>(p);
        return make_uint2(v.x, v.y);
    }
    // nibbles [16 - M, 32 - M) of prev ++ own
    template <int M>
    static __device__ __forceinline__ V shift(const V prev, const V own) {
        if (M == 0) return own;
        constexpr int B = 64 - 4 * M, Q = B / 32, R = B % 32;
        const uint32_t d[4] = {prev.x, prev.y, own.x, own.y};
        if (R == 0) return make_uint2(d[Q], d[Q + 1]);
        return make_uint2(__builtin_amdgcn_alignbit(d[Q + 1], d[Q], R), __builtin_amdgcn_alignbit(d[Q + 2], d[Q + 1], R));
    }
    static __device__ __forceinline__ uint32_t cnt(const V v, int k) {
        return ((k < 8 ? v.x : v.y) >> (4 * (k & 7))) & 0xFu;
    }
};

// lane l <- lane l + 1 (lane 63 <- 0): DPP wave_shl:1
__device__ __forceinline__ double dpp_shl1_d(double x) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), 0x130, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), 0x130, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

// count -> double in program order (volatile): left free, the scheduler
// converts a whole batch's counts up front and runs out of registers
__device__ __forceinline__ double ub_cvt(uint32_t x) {
    double r;
    asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

// b[c] for a band column: 0 outside the matrix or for a NaN bias (an empty
// cis-only group, which no stored count touches)
__device__ __forceinline__ double ub_bias(const double* __restrict__ b, long long c, long long n) {
    const bool in = c >= 0 && c < n;
    const double v = b[in ? c : 0];  // unconditional load (no branch per value)
    return (in && v == v) ? v : 0.0;
}

// Halving butterfly over the 8 values of every lane: afterwards lane l holds
// the wave-wide sum of value (l&1)*4 + (l&2) + (l&4)/4 (each pair's sum formed
// once, in one lane: fixed order).
template <int H, int MASK>
__device__ __forceinline__ void ub_halve(double (&v)[8], int lane) {
    const bool hi = (lane & MASK) != 0;
#pragma unroll
    for (int j = 0; j < H; ++j) {
        const double send = hi ? v[j] : v[j + H];
        const double keep = hi ? v[j + H] : v[j];
        v[j] = keep + __shfl_xor(send, MASK, 64);
    }
}
__device__ __forceinline__ double ub_reduce8(double (&v)[8], int lane) {
    ub_halve<4, 1>(v, lane);
    ub_halve<2, 2>(v, lane);
    ub_halve<1, 4>(v, lane);
    double x = v[0];
    x += __shfl_xor(x, 8, 64);
    x += __shfl_xor(x, 16, 64);
    x += __shfl_xor(x, 32, 64);
    return x;
}
__device__ __forceinline__ int ub_reduce8_row(int lane) { return (lane & 1) * 4 + (lane & 2) + ((lane >> 2) & 1); }

// One wave task: rows [r0, r0 + kUbRows) x chunk kc of segment P.  Lanes 1..63
// hold the chunk's 63 x 16 slots; lane 0 loads the 16 slots before them only
// to hand them to lane 1 (DPP wave_shr:1) as the bytes its shifted rows reach
// back into, and computes nothing (w = 0).  Heads go to heads[0, kUbRows);
// the tail is left in col[] of lanes 1..63 (columns r0 + kUbRows + base +
// 16 (lane - 1) + k).  The task's rows are all local or all halo (shards and
// the halo start are 512-row aligned); rows past the stored ones read 0.
// Every row is swept whatever its group's convergence flag: a converged
// cis-only group's partials are not read (k_marg skips its rows), and band
// counts never leave their chromosome.
// LDS image of the workgroup's column biases: one pad double per 16 (a lane's
// 16 window values are contiguous; lanes 136 B apart spread over the banks)
__device__ __forceinline__ int ub_pad(int j) { return j + (j >> 4); }
constexpr int kUbWin = kUbCols + kUbCols / 16 + 1;

template <int BITS>
__device__ __forceinline__ void ub_walk(const UbSeg& P, int kc, int chunk, long long r0, const UbArgs& a,
                                        long long n_bins, double* __restrict__ heads, double (&col)[16],
                                        const double* __restrict__ cwin, const double* __restrict__ rowb) {
    using T = UbT<BITS>;
    using V = typename T::V;
    const int lane = threadIdx.x & 63;
    int cb = (kc * kUbChunk + 16 * (lane - 1)) * BITS / 8;  // lane's bytes in a row (lane 0: the chunk's previous group)
    // lanes outside the segment read the row's last bytes: zero padding in the
    // nibble segment; in the uint8 band they hold diagonal W8's count, so
    // those lanes mask their words to 0
    const bool outside = cb < 0 || cb >= P.bytes;
    const uint32_t msk = (BITS == 8 && outside) ? 0u : ~0u;
    if (outside) cb = P.bytes - T::LB;
    const long long rhi = a.row_hi < r0 + kUbRows ? a.row_hi : r0 + kUbRows;
    const int nv = (int)(rhi - r0);  // stored rows of the task (uniform)
    const uint8_t* __restrict__ rows = (r0 >= a.row_lo ? P.loc + (r0 - a.row_lo) * P.stride
                                                       : P.halo + (r0 - a.halo_lo) * P.stride) + cb;
    const long long stride = P.stride;
    // rows past the stored ones read the last stored row: their counts only
    // reach columns past the shard (or carry a zero bias past the matrix), and
    // their row parts are not written
    auto load_row = [&](int i) -> V { return T::ld(rows + (long long)(i < nv ? i : nv - 1) * stride); };
    // the task's column biases and row biases come from the workgroup's LDS
    // images (staged once per workgroup: no per-group global loads)
    const int wo = (int)(r0 % kUbGroupRows);  // the task's offset in the workgroup
    double w[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) col[k] = 0.0;
    double* __restrict__ R = a.upart + (size_t)(kUbArrs * chunk) * a.nloc;
    V buf[2][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) buf[0][j] = load_row(j);
    const int ng = (nv + 15) / 16;
#pragma unroll 1
    for (int g = 0; g < kUbRows / 16; ++g) {
        const long long gb = r0 + 16 * g;
        if (g < ng) {
            {  // lane l's 16 columns gb + base + 16 (l - 1) + [0, 16); lane 0 computes nothing
                const double* src = cwin + ub_pad(wo + 16 * g + 16 * (lane > 0 ? lane - 1 : 0));
#pragma unroll
                for (int k = 0; k < 16; ++k) w[k] = lane ? src[k] : 0.0;
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                double racc[8];
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int bt = 2 * h + q;  // batch of 4 rows
#pragma unroll
                    for (int j = 0; j < 4; ++j) buf[(bt + 1) & 1][j] = load_row(16 * g + 4 * (bt + 1) + j);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int m = 4 * bt + j, mm = 4 * q + j;
                        V own = buf[bt & 1][j];
                        if (BITS == 8) {
                            uint4& o = *reinterpret_cast<uint4*>(&own);
                            o.x &= msk;
                            o.y &= msk;
                            o.z &= msk;
                            o.w &= msk;
                        }
                        V prev;
                        if (BITS == 8) {
                            const uint4 o = *reinterpret_cast<const uint4*>(&own);
                            const uint4 pv = dpp_shr1(o);
                            prev = *reinterpret_cast<const V*>(&pv);
                        } else {
                            const uint2 o = *reinterpret_cast<const uint2*>(&own);
                            const uint2 pv = make_uint2(__builtin_amdgcn_update_dpp(0u, o.x, 0x138, 0xF, 0xF, false),
                                                        __builtin_amdgcn_update_dpp(0u, o.y, 0x138, 0xF, 0xF, false));
                            prev = *reinterpret_cast<const V*>(&pv);
                        }
                        V sh;
                        switch (m) {  // compile-time after unrolling
                            case 0: sh = T::template shift<0>(prev, own); break;
                            case 1: sh = T::template shift<1>(prev, own); break;
                            case 2: sh = T::template shift<2>(prev, own); break;
                            case 3: sh = T::template shift<3>(prev, own); break;
                            case 4: sh = T::template shift<4>(prev, own); break;
                            case 5: sh = T::template shift<5>(prev, own); break;
                            case 6: sh = T::template shift<6>(prev, own); break;
                            case 7: sh = T::template shift<7>(prev, own); break;
                            case 8: sh = T::template shift<8>(prev, own); break;
                            case 9: sh = T::template shift<9>(prev, own); break;
                            case 10: sh = T::template shift<10>(prev, own); break;
                            case 11: sh = T::template shift<11>(prev, own); break;
                            case 12: sh = T::template shift<12>(prev, own); break;
                            case 13: sh = T::template shift<13>(prev, own); break;
                            case 14: sh = T::template shift<14>(prev, own); break;
                            default: sh = T::template shift<15>(prev, own); break;
                        }
                        const double br = rowb[wo + 16 * g + m];  // wave-uniform LDS broadcast
                        // two partial row sums (even / odd slots): shorter dependent chains
                        double a0 = 0.0, a1 = 0.0;
#pragma unroll
                        for (int k = 0; k < 16; k += 2) {
                            const double c0 = ub_cvt(T::cnt(sh, k)), c1 = ub_cvt(T::cnt(sh, k + 1));
                            a0 = fma(c0, w[k], a0);
                            a1 = fma(c1, w[k + 1], a1);
                            col[k] = fma(c0, br, col[k]);
                            col[k + 1] = fma(c1, br, col[k + 1]);
                            // each count's two uses together: left free, the
                            // compiler defers the column updates to the end of
                            // the batch and parks every converted count in AGPRs
                            asm volatile("" : "+v"(col[k]), "+v"(col[k + 1]), "+v"(a0), "+v"(a1));
                        }
                        racc[mm] = a0 + a1;
                    }
                    __builtin_amdgcn_sched_barrier(0);  // the next batch's loads stay after this one
                }
                const double s = ub_reduce8(racc, lane);
                const long long r = gb + 8 * h + ub_reduce8_row(lane);
                if (lane < 8 && r < rhi && r >= a.row_lo) R[r - a.row_lo] = s;
            }
        }
        if (lane == 1) {
#pragma unroll
            for (int k = 0; k < 16; ++k) heads[16 * g + k] = col[k];
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) col[k] = dpp_shl1_d(col[k]);
    }
}

// One workgroup: rows [g * kUbGroupRows, + kUbGroupRows) x one chunk.
__device__ __forceinline__ void ub_group(const UbSegs& S, long long grp, int chunk, const UbArgs& a, long long n_bins,
                                         double* __restrict__ cbuf, double* __restrict__ cwin,
                                         double* __restrict__ rowb) {
    int si = 0;
    while (si + 1 < S.n && chunk >= S.s[si + 1].ch) ++si;
    const UbSeg& P = S.s[si];
    const int kc = chunk - P.ch;
    const long long R0 = grp * kUbGroupRows;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const long long base = P.dlo + (long long)kc * kUbChunk;
    for (int j = threadIdx.x; j < kUbCols - kUbGroupRows; j += kUbThreads) cbuf[kUbGroupRows + j] = 0.0;
    for (int j = threadIdx.x; j < kUbCols; j += kUbThreads) cwin[ub_pad(j)] = ub_bias(a.b, R0 + base + j, n_bins);
    for (int j = threadIdx.x; j < kUbGroupRows; j += kUbThreads) rowb[j] = ub_bias(a.b, R0 + j, n_bins);
    __syncthreads();
    const long long r0 = R0 + (long long)kUbRows * wave;
    // rows this shard keeps, or columns it keeps, and rows it stores
    const bool rows_here = r0 < a.row_hi && r0 + kUbRows > a.row_lo;
    const bool cols_here = r0 + base < a.row_hi && r0 + kUbRows + base + kUbChunk > a.row_lo;
    const bool stored = r0 + kUbRows > a.halo_lo && r0 < a.row_hi;
    double col[16];
    double* heads = cbuf + (size_t)kUbRows * wave;
    if ((rows_here || cols_here) && stored) {
        if (P.bits == 8)
            ub_walk<8>(P, kc, chunk, r0, a, n_bins, heads, col, cwin, rowb);
        else
            ub_walk<4>(P, kc, chunk, r0, a, n_bins, heads, col, cwin, rowb);
    } else {
        for (int j = lane; j < kUbRows; j += 64) heads[j] = 0.0;
#pragma unroll
        for (int k = 0; k < 16; ++k) col[k] = 0.0;
    }
    // tails, one wave after the other (wave w's tail covers the heads of the
    // next kUbChunk / kUbRows waves): a fixed order per column
    for (int w = 0; w < kUbWaves; ++w) {
        __syncthreads();
        if (wave == w && lane > 0) {
            double* t = cbuf + (size_t)kUbRows * (wave + 1) + 16 * (lane - 1);
#pragma unroll
            for (int k = 0; k < 16; ++k) t[k] += col[k];
        }
    }
    __syncthreads();
    // H: the workgroup's own columns; T_e: those of the workgroup e ahead
    double* __restrict__ base_p = a.upart + (size_t)(kUbArrs * chunk + 1) * a.nloc;
    for (int j = threadIdx.x; j < kUbCols; j += kUbThreads) {
        const long long c = R0 + base + j;
        if (c >= a.row_lo && c < a.row_hi) base_p[(size_t)(j / kUbGroupRows) * a.nloc + (c - a.row_lo)] = cbuf[j];
    }
}

// grid: (workgroups, chunks).  xcd != 0: the blocks are re-dealt so that each
// XCD (blocks b, b + 8, ... share one) takes a contiguous range of (workgroup,
// chunk) pairs, chunks fastest: neighbouring chunks of the same rows, which
// share the cache lines at their boundaries (a chunk is 1008 B of uint8 /
// 504 B of nibbles per row, not a multiple of 128 B), run back to back on one L2
__global__ __launch_bounds__(kUbThreads, 3) void k_sweep_ubands(UbSegs S, UbArgs a, long long n_bins, int xcd) {
    __shared__ double cbuf[kUbCols];
    __shared__ double cwin[kUbWin];
    __shared__ double rowb[kUbGroupRows];
    long long grp = blockIdx.x;
    int y = blockIdx.y;
    if (xcd) {
        const long long nb = (long long)gridDim.x * gridDim.y, b = blockIdx.x + (long long)blockIdx.y * gridDim.x;
        const long long L = xcd_remap(b, nb);
        y = (int)(L % gridDim.y);
        grp = L / gridDim.y;
    }
    ub_group(S, a.g_lo + grp, S.ord[y], a, n_bins, cbuf, cwin, rowb);
}

// Halo of a shard (rows [halo_lo, row_lo), upper halves only): every count a
// halo row r' holds at diagonal d > 0 with r' + d in the shard is the shard
// row's count at diagonal -d.  One thread per (halo row, upper byte).
__global__ void k_ub_halo(const uint8_t* __restrict__ band, const uint8_t* __restrict__ band4, long long W8,
                          long long W4, long long row_lo, long long row_hi, long long halo_lo,
                          uint8_t* __restrict__ h8, uint8_t* __restrict__ h4) {
    const long long nh = row_lo - halo_lo;
    const long long st8 = band_stride(W8), st4 = band4_stride(W8, W4), sg = band4_seg(W8, W4);
    const long long per = W8 + (W4 > W8 ? sg : 0);  // bytes per halo row: uint8 diagonals 1..W8, nibble bytes
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nh * per) return;
    const long long hr = i / per, j = i % per, c = halo_lo + hr;
    if (j < W8) {
        const long long d = j + 1, r = c + d;
        if (r >= row_lo && r < row_hi) h8[hr * st8 + W8 + d] = band[(r - row_lo) * st8 + (W8 - d)];
    } else {
        const long long jb = j - W8;  // byte of the positive nibble segment: nibbles 2 jb, 2 jb + 1
        uint32_t v = 0;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const long long d = W8 + 1 + 2 * jb + q, r = c + d;
            if (d <= W4 && r >= row_lo && r < row_hi) {
                const long long nib = band4_nibble(-d, W8, W4);
                v |= ((band4[(r - row_lo) * st4 + (nib >> 1)] >> (4 * (nib & 1))) & 0xFu) << (4 * q);
            }
        }
        h4[hr * st4 + sg + jb] = (uint8_t)v;
    }
}

// Small matrices (one chromosome, a shard of a few hundred MB): the whole
// sweep -- tiled units, band blocks, flat units -- as ONE launch.  Each body
// is latency-bound there (few blocks, each a short dependent chain), and run
// as three kernels their ramps and tails add up; in one grid the blocks of
// all three share the CUs.  Same bodies, same partials: bitwise the same.
static_assert(kBandThreads == kSweepThreads, "one block shape");
template <int NB, int U, int ABL, bool UP>
__global__ __launch_bounds__(kSweepThreads, 4) void k_sweep_all(TileDev T, const uint8_t* __restrict__ act,
                                                              int n_tiled, int n_band, BandSegs S, int band_rb,
                                                              long long nloc, long long row_lo,
                                                              const uint16_t* __restrict__ row_group,
                                                              const double* __restrict__ b, long long n_bins,
                                                              double* __restrict__ part,
                                                              double* __restrict__ bpart,
                                                              unsigned long long* __restrict__ trace) {
    __shared__ __attribute__((aligned(16))) union Lds {
        TiledLds<UP> t;
        FlatLds<UP> f;
        BandLds<64> band;
    } L;
    // grid: [tiled units | band blocks (n_band = band_rb x chunks) | flat units]
    const int x = blockIdx.x;
    const unsigned long long t0 = trace ? wall_clock64() : 0ull;
    if (x < n_tiled) {
        sweep_tiled_unit<NB, ABL, UP>(T, act, T.u_order[x], b, n_bins, part, L.t);
    } else if (x < n_tiled + n_band) {
        const int y = x - n_tiled;
        band_any<ABL, 64>(S, y % band_rb, y / band_rb, L.band, nloc, row_lo, n_bins, act, row_group, b, bpart);
    } else {
        sweep_flat_unit<U, ABL, UP>(T, act, T.u_order[x - n_band], b, n_bins, part, L.f);  // flat units follow the tiled
    }
    if (trace) {  // diagnostic block timeline (hh_tune "sweep_trace"): start, end, CU of each block
        __syncthreads();
        if (threadIdx.x == 0) {
            trace[3 * (size_t)x] = t0;
            trace[3 * (size_t)x + 1] = wall_clock64();
            trace[3 * (size_t)x + 2] = (unsigned long long)__smid();
        }
    }
}

// One block per row-block (thread = row): the block's unit descriptors are
// staged in LDS in batches (every row used to re-read them from global
// memory, one dependent chain per unit), the partial loads are issued
// unconditionally from a clamped index and selected, so a batch's loads fly
// together.  Summation order per row is unchanged (units in order, then band
// chunks, wide entries, diagonal): bitwise the same marginals.
// the upper-band partials k_marg adds (K1d): chunk c's R / H / T1.. arrays at
// part + kUbArrs c nloc, and the column of chunk c's slot 0 at row 0
struct UbMarg {
    const double* part;
    int n;
    long long base[kMaxUbChunks];
};
constexpr int kMargThreads = kR;
constexpr int kMargU = 256;  // unit descriptors per LDS batch

// Stats tiles: the 512-row blocks cut at group boundaries, in row order
// (tile_lo sorted); blk_tile_ptr[B] = first tile of global row-block B.
struct TileArgs {
    const int32_t* tile_lo;
    const int32_t* tile_hi;
    const int32_t* tile_group;
    const int32_t* group_tile_ptr;
    const int32_t* blk_tile_ptr;
    double* tile_cnt;
    double* tile_sum;
    double* tile_sq;
    double* g_cnt;  // per group, from the stats tail
    double* g_sum;
    unsigned* counter;  // [2]: last-block-done counters (stats, update)
};

struct GroupState {
    double* var;
    double* mean;
    int32_t* iters;
    uint8_t* empty;
};

// One stats tile's nonzero count and sum; thread = row (block start +
// threadIdx.x), x = that row's marginal.  The same per-thread values and
// tree in k_marg (fused) and k_stats1 -> bitwise the same tile sums.
__device__ __forceinline__ void tile_stats(const TileArgs& ta, int t, long long row, double x, double* sh) {
    const bool in = row >= ta.tile_lo[t] && row < ta.tile_hi[t] && x != 0.0;
    const double c = block_sum(in ? 1.0 : 0.0, sh);
    const double s = block_sum(in ? x : 0.0, sh);
    if (threadIdx.x == 0) {
        ta.tile_cnt[t] = c;
        ta.tile_sum[t] = s;
    }
}

// Sum of v[t0..t1) by one wave in a fixed order (lane-strided, then the
// xor tree): the same bits wherever it is evaluated.
__device__ __forceinline__ double wave_range_sum(const double* v, int t0, int t1) {
    const int lane = threadIdx.x & 63;
    double a = 0.0;
#pragma unroll 4
    for (int t = t0 + lane; t < t1; t += 64) a += v[t];
    return wave_sum(a);
}

// Last-block-done: every block bumps counter[k] after a release fence (the
// values the tail reads were stored by thread 0); the block that sees
// gridDim.x - 1 returns true (after an acquire fence) and resets the counter
// for the next launch.  No block waits on another.
__device__ __forceinline__ bool last_block(unsigned* counter, int* flag) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        *flag = atomicAdd(counter, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!*flag) return false;
    __threadfence();
    if (threadIdx.x == 0) atomicExch(counter, 0u);
    return true;
}

// Stats tail (last block): per active group, one wave: count and sum over the
// group's tiles -> g_cnt / g_sum.
__device__ __forceinline__ void stats_tail(const TileArgs& ta, const uint8_t* act, int G) {
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int g = w; g < G; g += nw) {
        if (act[g] == 0) continue;
        const int t0 = ta.group_tile_ptr[g], t1 = ta.group_tile_ptr[g + 1];
        const double c = wave_range_sum(ta.tile_cnt, t0, t1);
        const double s = wave_range_sum(ta.tile_sum, t0, t1);
        if ((threadIdx.x & 63) == 0) {
            ta.g_cnt[g] = c;
            ta.g_sum[g] = s;
        }
    }
}

// One block per row-block (thread = row): the block's unit descriptors are
// staged in LDS in batches (every row used to re-read them from global
// memory, one dependent chain per unit), the partial loads are issued
// unconditionally from a clamped index and selected, so a batch's loads fly
// together.  Summation order per row is unchanged (units in order, then band
// chunks, wide entries, diagonal): bitwise the same marginals.  With
// `stats` (one GPU holds every row, out = the full marginal vector) the
// block also writes its stats tiles' count / sum, and the last block the
// per-group totals (k_stats1's work, without its launch).
__global__ __launch_bounds__(kMargThreads) void k_marg(TileDev T, const double* __restrict__ part,
                                                       const long long* __restrict__ wide_ptr,
                                                       const int32_t* __restrict__ wide_col,
                                                       const double* __restrict__ wide_cnt,
                                                       const double* __restrict__ diag,
                                                       const uint16_t* __restrict__ row_group,
                                                       const uint8_t* __restrict__ act, const double* __restrict__ b,
                                                       long long row_lo, int nloc, const double* __restrict__ bpart,
                                                       int nch, UbMarg ub, double* __restrict__ out, TileArgs ta,
                                                       int G, int stats, const u64* __restrict__ colacc) {
    __shared__ int su_lo[kMargU], su_n[kMargU], su_slot[kMargU];
    __shared__ double sh[16];
    __shared__ int flag;
    const int rbk = blockIdx.x, rl = threadIdx.x;
    const int i = rbk * kR + rl;
    const bool live = i < nloc && act[row_group[i < nloc ? i : 0]] != 0;
    const int u0 = T.blk_unit_ptr[rbk], u1 = T.blk_unit_ptr[rbk + 1];
    double s = 0.0;
    for (int ub = u0; ub < u1; ub += kMargU) {
        const int cnt = min(kMargU, u1 - ub);
        __syncthreads();
        if (rl < cnt) {
            su_lo[rl] = T.u_rlo[ub + rl];
            su_n[rl] = T.u_rhi[ub + rl] - T.u_rlo[ub + rl];
            su_slot[rl] = T.u_slot[ub + rl];
        }
        __syncthreads();
        if (live) {
            int k = 0;
            for (; k + 8 <= cnt; k += 8) {
                double x[8];
                bool in[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int o = rl - su_lo[k + q];
                    in[q] = (unsigned)o < (unsigned)su_n[k + q];
                    x[q] = part[su_slot[k + q] + (in[q] ? o : 0)];
                }
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    if (in[q]) s += x[q];
            }
            for (; k < cnt; ++k) {
                const int o = rl - su_lo[k];
                if ((unsigned)o < (unsigned)su_n[k]) s += part[su_slot[k] + o];
            }
        }
    }
    double v = 0.0;
    if (live) {
        // dense band chunks, fixed order; loads issued 8 at a time
        int c = 0;
        for (; c + 8 <= nch; c += 8) {
            double x[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) x[q] = bpart[(long long)(c + q) * nloc + i];
#pragma unroll
            for (int q = 0; q < 8; ++q) s += x[q];
        }
        for (; c < nch; ++c) s += bpart[(long long)c * nloc + i];
        // upper band (K1d): per chunk its row part, column head and, for the
        // first kUbChunk columns of a workgroup, the previous workgroup's tail
        // two chunks' loads in flight at a time (one chunk per iteration left a
        // dependent load chain per chunk: k_marg 109 us at C4)
        for (c = 0; c < ub.n; c += 2) {
            double x[2][kUbArrs];
            bool in[2][kUbArrs];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int cc = c + h < ub.n ? c + h : c;
                const double* __restrict__ p = ub.part + (size_t)(kUbArrs * cc) * nloc + i;
                const long long t = row_lo + i - ub.base[cc];  // column offset from the chunk's first workgroup
                const long long q = t >= 0 ? t / kUbGroupRows : -1, o = t - q * kUbGroupRows;
                in[h][0] = in[h][1] = c + h < ub.n;
#pragma unroll
                for (int e = 1; e <= kUbTails; ++e)
                    in[h][1 + e] = c + h < ub.n && q >= e && o + (long long)e * kUbGroupRows < kUbCols;
#pragma unroll
                for (int e = 0; e < kUbArrs; ++e) x[h][e] = p[in[h][e] ? (long long)e * nloc : 0];
            }
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int e = 0; e < kUbArrs; ++e)
                    if (in[h][e]) s += x[h][e];
        }
        // the column side of the upper-triangle tiles: sum_k count_k B[row_k]
        // over the stored entries of this column (exact int64), / 2^e
        if (colacc) s += (double)(long long)colacc[i] * T.fix[1];
        for (long long q = wide_ptr[i]; q < wide_ptr[i + 1]; ++q) s = fma(wide_cnt[q], b[wide_col[q]], s);
        const double br = b[row_lo + i];
        v = br * fma(2.0 * diag[i], br, s);
        out[i] = v;
    }
    if (!stats) return;
    const int B = (int)(row_lo / kR) + rbk;
    for (int t = ta.blk_tile_ptr[B]; t < ta.blk_tile_ptr[B + 1]; ++t)
        if (act[ta.tile_group[t]] != 0) tile_stats(ta, t, row_lo + i, v, sh);
    if (stats == 1 && last_block(ta.counter, &flag)) stats_tail(ta, act, G);  // 2: tile sums only (big mode)
}

// Column side of the upper-triangle tiles, per column c of [c0, c0 + n):
// the sum of the slots of its column tile (plan order; integers: exact).
__global__ __launch_bounds__(256) void k_colsum(const u64* __restrict__ colpart, const int32_t* __restrict__ jslot_ptr,
                                                const int32_t* __restrict__ jslot, long long c0, long long n,
                                                u64* __restrict__ out) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const long long c = c0 + i;
    const int J = (int)(c >> kWBits), k = (int)(c & (kW - 1));
    const int a = jslot_ptr[J], e = jslot_ptr[J + 1];
    u64 acc = 0;
    int q = a;
    for (; q + 8 <= e; q += 8) {  // eight loads in flight
        u64 x[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = colpart[(size_t)jslot[q + r] * kW + k];
#pragma unroll
        for (int r = 0; r < 8; ++r) acc += x[r];
    }
    for (; q < e; ++q) acc += colpart[(size_t)jslot[q] * kW + k];
    out[i] = acc;
}

// This sweep's fixed-point scale 2^e from the bias maximum the last update
// left (bmax[p], double bits) and the largest raw marginal rmax (a bound on
// any column's count total): every column sum count * round(b 2^e) stays
// below 2^62.  fix = {2^e, 2^-e}; the other bmax slot is cleared for the
// update that follows.
// Every thread derives the same e from the same two numbers, converts its
// bins' bias to B = round(b 2^e) (the walks then load B, no conversion in the
// hot loops; NaN / negative -> 0); thread 0 also clears the other slot.
__global__ __launch_bounds__(256) void k_fixscale(unsigned long long* __restrict__ bmax, int p, double rmax,
                                                  double* __restrict__ fix, const double* __restrict__ b, long long n,
                                                  u64* __restrict__ bfix) {
    double bm = __longlong_as_double((long long)bmax[p]);
    if (!(bm > 0.0) || !(bm < 1e300)) bm = 1.0;
    const double r = rmax > 1.0 ? rmax : 1.0;
    const int e = 61 - ilogb(r) - ilogb(bm);  // r < 2^(ilogb r + 1), bm < 2^(ilogb bm + 1)
    const double sc = ldexp(1.0, e);
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        const double x = b[i];
        bfix[i] = x > 0.0 ? (u64)__double2ll_rn(x * sc) : 0ull;  // (x < bm * 2: below 2^62)
    }
    if (i == 0) {
        fix[0] = sc;
        fix[1] = ldexp(1.0, -e);
        bmax[1 - p] = 0ull;
    }
}

// the all-bins column vector -> the per-rank padded blocks of the column
// exchange (rank k's rows at k * maxlen)
__global__ void k_colpad(const u64* __restrict__ col, int world, long long maxlen,
                         const long long* __restrict__ rank_rows, u64* __restrict__ out) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long long)world * maxlen) return;
    const int k = (int)(t / maxlen);
    const long long off = t - (long long)k * maxlen;
    const long long lo = rank_rows[k], hi = rank_rows[k + 1];
    out[t] = lo + off < hi ? col[lo + off] : 0ull;
}

// the all-gather fallback of the column exchange: rank `rank`'s block summed
// over the gathered vectors (world x (world x maxlen)), in rank order
__global__ void k_colgather(const u64* __restrict__ all, int world, long long maxlen, int rank, u64* __restrict__ out) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= maxlen) return;
    u64 acc = 0;
    for (int r = 0; r < world; ++r) acc += all[((size_t)r * world + rank) * maxlen + i];
    out[i] = acc;
}

__global__ void k_scatter(const double* __restrict__ g, int world, long long maxlen,
                          const long long* __restrict__ rank_rows, double* __restrict__ marg) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long long)world * maxlen) return;
    const int k = (int)(t / maxlen);
    const long long off = t - (long long)k * maxlen;
    const long long lo = rank_rows[k], hi = rank_rows[k + 1];
    if (lo + off < hi) marg[lo + off] = g[t];
}

__global__ void k_filter_lt(const double* __restrict__ marg, long long n, double thr,
                            double* __restrict__ bias) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && marg[i] < thr) bias[i] = 0.0;
}

// k_marg's stats part on the full (gathered) marginal vector: one block per
// stats tile, thread = row of the tile's 512-row block.
template <bool TAIL>
__global__ __launch_bounds__(kR) void k_stats1(TileArgs ta, const uint8_t* __restrict__ act,
                                               const double* __restrict__ marg, int G) {
    __shared__ double sh[16];
    __shared__ int flag;
    const int t = blockIdx.x;
    if (act[ta.tile_group[t]] != 0) {
        const long long row = (long long)(ta.tile_lo[t] / kR) * kR + threadIdx.x;
        const bool in = row >= ta.tile_lo[t] && row < ta.tile_hi[t];
        tile_stats(ta, t, row, in ? marg[row] : 0.0, sh);
    }
    if (TAIL && last_block(ta.counter, &flag)) stats_tail(ta, act, G);
}

// Large matrices (many stats tiles): no last-block tails -- their device-scope
// fences and one-wave reductions over ~1 200 tiles cost ~45 us per C4
// iteration -- but every block re-reduces its group's tile sums (block-wide,
// fixed order; the same function in k_stats2 and k_update_big -> the same
// mean), as in round 1: k_marg, k_stats1<false>, k_stats2, k_update_big.
__device__ __forceinline__ void group_totals_block(const TileArgs& ta, int g, double* sh, double& cnt, double& sum,
                                                   double* sq) {
    const int t0 = ta.group_tile_ptr[g], t1 = ta.group_tile_ptr[g + 1];
    double c = 0.0, s = 0.0, q = 0.0;
    for (int t = t0 + threadIdx.x; t < t1; t += blockDim.x) {
        c += ta.tile_cnt[t];
        s += ta.tile_sum[t];
        if (sq) q += ta.tile_sq[t];
    }
    cnt = block_sum(c, sh);
    sum = block_sum(s, sh);
    if (sq) *sq = block_sum(q, sh);
}

__global__ __launch_bounds__(kR) void k_stats2(TileArgs ta, const uint8_t* __restrict__ act,
                                               const double* __restrict__ marg) {
    __shared__ double sh[16];
    const int t = blockIdx.x;
    const int g = ta.tile_group[t];
    if (act[g] == 0) return;
    double cnt, sum;
    group_totals_block(ta, g, sh, cnt, sum, nullptr);
    const double mean = sum / cnt;
    const long long row = ta.tile_lo[t] + threadIdx.x;
    double q = 0.0;
    if (row < ta.tile_hi[t]) {
        const double x = marg[row];
        if (x != 0.0) {
            const double d = x - mean;
            q = d * d;
        }
    }
    q = block_sum(q, sh);
    if (threadIdx.x == 0) ta.tile_sq[t] = q;
}

// the largest finite positive bias of the wave's rows -> *bmax (double
// bits: for positive doubles the unsigned order is the numeric order); the
// next sweep's fixed-point scale (k_fixscale) comes from it
__device__ __forceinline__ void bias_max(double v, unsigned long long* bmax) {
    if (!bmax) return;
    double m = (v > 0.0 && v < 1e300) ? v : 0.0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0 && m > 0.0) atomicMax(bmax, (unsigned long long)__double_as_longlong(m));
}

__global__ __launch_bounds__(kR) void k_update_big(TileArgs ta, const uint8_t* __restrict__ act,
                                                   uint8_t* __restrict__ nxt, const double* __restrict__ marg,
                                                   double* __restrict__ bias, GroupState gs, double tol,
                                                   int max_iters, unsigned long long* __restrict__ bmax) {
    __shared__ double sh[16];
    const int t = blockIdx.x;
    const int g = ta.tile_group[t];
    const bool first = t == ta.group_tile_ptr[g];
    if (act[g] == 0) {
        if (first && threadIdx.x == 0) nxt[g] = 0;
        const long long row = ta.tile_lo[t] + threadIdx.x;
        bias_max(row < ta.tile_hi[t] ? bias[row] : 0.0, bmax);
        return;
    }
    double cnt, sum, sq;
    group_totals_block(ta, g, sh, cnt, sum, &sq);
    const long long row = ta.tile_lo[t] + threadIdx.x;
    const bool in = row < ta.tile_hi[t];
    if (cnt == 0.0) {  // no nonzero marginal: cooler sets the group's bias to NaN
        // (0 until the finalize turns it into NaN: a NaN here would leak
        // into the neighbouring chromosomes' rows through the dense bands'
        // zero slots across the boundary, 0 * NaN)
        if (in) bias[row] = 0.0;
        if (first && threadIdx.x == 0) {
            gs.empty[g] = 1;
            gs.var[g] = 0.0;
            gs.mean[g] = __builtin_nan("");
            gs.iters[g] += 1;
            nxt[g] = 0;
        }
        return;
    }
    const double mean = sum / cnt;
    double bnew = 0.0;
    if (in) {
        double m = marg[row] / mean;
        if (m == 0.0) m = 1.0;
        bnew = bias[row] / m;
        bias[row] = bnew;
    }
    bias_max(bnew, bmax);
    if (first && threadIdx.x == 0) {
        const double var = sq / cnt;
        gs.var[g] = var;
        gs.mean[g] = mean;
        const int it = gs.iters[g] + 1;
        gs.iters[g] = it;
        nxt[g] = (var < tol || it >= max_iters) ? 0 : 1;
    }
}

// One block per stats tile: b /= marg/mean with the group mean from the stats
// tail, and the tile's sum of squared deviations; the last block reduces those
// per group (one wave each) and records var / mean / iters / the next flag
// (cooler: bias updated, then `var < tol` tested).
__global__ __launch_bounds__(kR) void k_update(TileArgs ta, const uint8_t* __restrict__ act,
                                               uint8_t* __restrict__ nxt, const double* __restrict__ marg,
                                               double* __restrict__ bias, GroupState gs, double tol,
                                               int max_iters, int G, unsigned long long* __restrict__ bmax) {
    __shared__ double sh[16];
    __shared__ int flag;
    const int t = blockIdx.x;
    const int g = ta.tile_group[t];
    {
        const long long row = ta.tile_lo[t] + threadIdx.x;
        const bool in = row < ta.tile_hi[t];
        double bnew = 0.0;
        if (act[g] != 0) {
            const double cnt = ta.g_cnt[g], sum = ta.g_sum[g];
            double q = 0.0;
            if (cnt == 0.0) {  // no nonzero marginal: cooler's NaN, as 0 until the finalize (k_update_big)
                if (in) bias[row] = 0.0;
            } else if (in) {
                const double mean = sum / cnt;
                const double x = marg[row];
                double m = x / mean;
                if (m == 0.0) m = 1.0;
                bnew = bias[row] / m;
                bias[row] = bnew;
                if (x != 0.0) {
                    const double d = x - mean;
                    q = d * d;
                }
            }
            q = block_sum(q, sh);
            if (threadIdx.x == 0) ta.tile_sq[t] = q;
        } else if (in) {
            bnew = bias[row];
        }
        bias_max(bnew, bmax);
    }
    if (!last_block(ta.counter + 1, &flag)) return;
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6, lane = threadIdx.x & 63;
    for (int gg = w; gg < G; gg += nw) {
        if (act[gg] == 0) {
            if (lane == 0) nxt[gg] = 0;
            continue;
        }
        const double cnt = ta.g_cnt[gg];
        const double sq = wave_range_sum(ta.tile_sq, ta.group_tile_ptr[gg], ta.group_tile_ptr[gg + 1]);
        if (lane != 0) continue;
        const int it = gs.iters[gg] + 1;
        gs.iters[gg] = it;
        if (cnt == 0.0) {
            gs.empty[gg] = 1;
            gs.var[gg] = 0.0;
            gs.mean[gg] = __builtin_nan("");
            nxt[gg] = 0;
        } else {
            const double var = sq / cnt;
            gs.var[gg] = var;
            gs.mean[gg] = ta.g_sum[gg] / cnt;
            nxt[gg] = (var < tol || it >= max_iters) ? 0 : 1;
        }
    }
}

static double np_median(std::vector<double> v) {
    if (v.empty()) return std::numeric_limits<double>::quiet_NaN();
    const size_t k = v.size() / 2;
    std::nth_element(v.begin(), v.begin() + k, v.end());
    const double hi = v[k];
    if (v.size() & 1) return hi;
    const double lo = *std::max_element(v.begin(), v.begin() + k);
    return (lo + hi) / 2.0;
}

static inline unsigned nblocks(long long n, int t) { return (unsigned)((n + t - 1) / t); }

}  // namespace hh

using namespace hh;

namespace hh {
// the stats mode switch (hh_ice::small_stats): C2 (49 tiles) fused, C3 (149) / C4 (1 187) not
static int g_fuse_stats = -1;
constexpr int kFuseMaxTiles = 128;
}  // namespace hh

struct hh_ice {
    hh_matrix* m = nullptr;
    hh_ice_opts o{};
    int64_t n = 0, nloc = 0;
    int32_t G = 1;
    std::vector<int64_t> glo, ghi;
    int32_t n_tiles = 0;
    DBuf<int32_t> tile_lo, tile_hi, tile_group, group_tile_ptr, blk_tile_ptr;
    DBuf<double> bias, marg, part, tile_cnt, tile_sum, tile_sq, g_cnt, g_sum;
    DBuf<unsigned> counter;   // last-block-done counters of the stats / update tails
    bool stats_fresh = false; // tile + group stats of the current marginals already made (fused k_marg)
    DBuf<double> bpart;  // dense band partials: n_band_chunks x nloc
    int32_t nch = 0;
    // upper-band sweep (K1d): chunks, partials (R/H/T per chunk), a shard's
    // halo rows [halo_lo, row_lo) (upper halves), workgroups [ub_glo, ub_ghi)
    int32_t nchu = 0;
    DBuf<double> upart;
    DBuf<uint8_t> halo8, halo4;
    int64_t halo_lo = 0, ub_glo = 0, ub_ghi = 0;
    DBuf<uint8_t> active;  // 2 x G (parity double buffer)
    DBuf<double> g_var, g_mean;
    DBuf<int32_t> g_iters;
    DBuf<uint8_t> g_empty;
    DBuf<long long> rank_rows;
    std::vector<int64_t> h_rank_rows;
    // upper-triangle tiles: column slots, the all-bins column
    // vector (int64 fixed point), the fixed-point scale {2^e, 2^-e} and the
    // bias maximum (double bits, parity double buffer) it comes from; rmax =
    // the largest raw marginal (global once the filters have seen the
    // gathered marginals)
    DBuf<unsigned long long> colpart, colacc, bmax, bfix;
    DBuf<double> fix;
    double rmax = 1.0;
    bool rmax_global = false;
    // the column exchange of a shard: int64 reduce-scatter over the ranks'
    // padded row blocks (a caller's hh_reduce_fn, else through the all-gather)
    int32_t cx_world = 1, cx_rank = 0;
    int64_t cx_maxlen = 0;
    std::vector<int64_t> cx_rr;
    DBuf<long long> cx_rr_dev;
    hh_reduce_fn cx_fn = nullptr;
    void* cx_user = nullptr;
    hh_allgather_fn cx_ag = nullptr;
    void* cx_ag_user = nullptr;
    DBuf<unsigned long long> cx_send, cx_recv, cx_all;
    int32_t iters_done = 0;
    PinnedBuf<uint8_t> h_active;
    // timing of the last hh_ice_run
    std::vector<hipEvent_t> ev;
    double sweep_ms = 0.0, iter_ms = 0.0;
    int32_t sweep_launches = 0;
    // side stream for the dense-band sweep, run beside the tile sweep
    hipStream_t side = nullptr, side2 = nullptr;
    hipEvent_t fork = nullptr, join = nullptr, join2 = nullptr;
    ~hh_ice() {
        for (auto e : ev) (void)hipEventDestroy(e);
        if (join2) (void)hipEventDestroy(join2);
        if (side2) (void)hipStreamDestroy(side2);
        if (fork) (void)hipEventDestroy(fork);
        if (join) (void)hipEventDestroy(join);
        if (side) (void)hipStreamDestroy(side);
    }
    bool full() const { return m->row_lo == 0 && m->row_hi == m->n_bins; }
    TileArgs ta() {
        return TileArgs{tile_lo.p, tile_hi.p, tile_group.p, group_tile_ptr.p, blk_tile_ptr.p, tile_cnt.p,
                        tile_sum.p, tile_sq.p, g_cnt.p, g_sum.p, counter.p};
    }
    // stats mode: few tiles -> fused k_marg stats + last-block tails (2
    // launches after the sweep); many -> tile sums in k_marg, k_stats2,
    // k_update_big, no tails (hh_tune "fuse_stats": -1 auto, 0 never fused:
    // k_stats1 launched, 1 always the small mode, 2 always the big mode)
    bool small_stats() const { return hh::g_fuse_stats == 1 || (hh::g_fuse_stats < 0 && n_tiles <= hh::kFuseMaxTiles); }
    uint8_t* act() { return active.p + (iters_done & 1) * G; }
    uint8_t* nxt() { return active.p + (1 - (iters_done & 1)) * G; }
};

namespace hh {

// Tuning knobs (hh_tune; no effect on results except the ablations).
static int g_sweep_nb = 2;
static int g_band_dpp = 0;    // band sweep: a lane's previous 16 bytes by DPP shift (0: a second load;
                              // measured 4.34 vs 4.44 ms C4 sweep, profiles/r3_band_dpp_ab.log)
// waves per k_sweep_flatw block (8, 10 or 11; they share one staged b[J] and
// the block's LDS caps them at 11): the kernel waits on memory (SQ counters,
// profiles/r3b_c4_sq_counters.json: VALU active 21 % of wave cycles), and 11
// waves with 33-tile column groups (3 tiles per wave) took the C4 sweep from
// 3.52 to 3.33 ms (profiles/r3b_flatw_waves_*_ab.log); 44-tile groups 1 % more
static int g_flatw_waves = 11;
static int g_flatw_waves_up = 8;  // k_sweep_flatw with the column side: 8 (no spills) or 11
static int g_flatw_pipe = 2;  // k_sweep_flatw: 1 = the next run's loads before the current step's walk,
                              // 2 = and the next tile's first runs before the current tile's row sums go out
static int g_sweep_ablate = 0;
// Default: three streams per sweep -- band kernels (side), tiled kernel (side2),
// flat kernel (main) -- so each kernel's ramp and tail overlap the others'
// (C4: 4.80 -> 4.69 ms; the band beside tiled+flat on one stream alone was
// +2 %, profiles/r1v8_knobs_split.log).  All write disjoint partials.
static int g_band_concurrent = 1;  // dense-band sweep on a side stream, beside the tiles
static int g_split_tiles = 1;      // with band_concurrent: tiled kernel on a second side stream
static int g_conc_order = 1;       // three-stream sweep launch order: 0 band, tiled, flat; 1 flat, band, tiled; 2 flat, tiled, band
// below this payload the fork / join costs more than the overlap gains.
// Round 2, with the band kernel at 8 waves per SIMD: one stream is 4-5 %
// faster for C3 (3.0 GB) and the N = 8 C4 shards (1.6-1.9 GB), three streams
// 0.3 % faster for the whole C4 matrix (14.8 GB; profiles/r2_conc_probe.log)
static int64_t g_conc_min_bytes = 8LL << 30;
static int64_t g_conc_ub_min_bytes = 1LL << 30;  // the same with the upper-band sweep (round 4)
static int g_band_rows = 0;   // rows per band block: 0 = auto (64 or 256)
static int g_band_fused = 1;  // the band segments in one launch
static int g_band_lpt = 1;      // band chunks dispatched heaviest first (0: uint8 first, index order)
// upper-band sweep (K1d, round 3): read only the upper half of the bands, each
// count feeding its row and its column.  0: the round-2 symmetric band kernels;
// 1 (auto): the upper-band sweep when the WHOLE matrix's bands hold at least
// g_uband_min_bytes (a wave walks its rows in sequence: on one small
// chromosome that chain, not the bytes, sets the time -- C2's 0.06 GB of
// bands); 2: always.  From 128 MB (round 5, was 1 GB): C3 (0.22 GB of bands)
// 0.773 -> 0.717 ms per sweep, the 10 kb cis-only genome (0.78 GB) 0.69 ->
// 0.56 ms (profiles/r5f, r5g).  Decided at hh_ice_create from the whole
// matrix, so every shard of one matrix takes the same path.
static int g_uband = 1;
static int64_t g_uband_min_bytes = 128LL << 20;
static int g_ub_xcd = 1;  // upper-band blocks dealt in contiguous ranges per XCD (k_sweep_ubands)
static int g_sweep_single = -1;  // whole sweep in one launch: -1 auto (below g_single_max_bytes), 0 off, 1 on
static int g_iter_events = 1;    // hh_ice_run: HIP events around every sweep (0: first / last only)
static int64_t g_single_max_bytes = 1LL << 30;
// diagnostic: per-block timeline of the last single-launch sweep (hh_sweep_trace)
static unsigned long long* g_trace = nullptr;
static int64_t g_trace_cap = 0, g_trace_n = 0;

template <int NB, int ABL, bool UP>
static void launch_sweep_up(const hh_matrix* m, const TileDev& T, const uint8_t* act, const double* b, double* part,
                            hipStream_t s, hipStream_t s_tiled, int which) {
    const int n_tiled = (int)(m->n_units - m->n_units_flat), n_flat = (int)m->n_units_flat;
    auto tiled = [&] {
        if (!n_tiled) return;
        HH_KTIME("k_sweep_tiled", s_tiled);  // per-kernel registry timing (probes; off by default)
        hipLaunchKernelGGL((k_sweep_tiled<NB, ABL, UP>), dim3((unsigned)n_tiled), dim3(kSweepThreads), 0, s_tiled,
                           T, act, n_tiled, b, (long long)m->n_bins, part);
    };
    if (which & 1) tiled();
    if (!(which & 2)) return;
    HH_KTIME(n_flat ? "k_sweep_flat" : nullptr, s);
    if (n_flat && m->n_fgroups) {
        // (the column-grouped flat tiles' narrow segments are interleaved for
        // kFlatU uint4 per lane: finalize_flat_layout)
        HH_REQUIRE(m->flat_perm, "column-grouped flat tiles without the interleaved layout");
        auto kern = g_flatw_pipe == 2   ? k_sweep_flatw<kFlatU, ABL, 2>
                    : g_flatw_pipe == 1 ? k_sweep_flatw<kFlatU, ABL, 1>
                                        : k_sweep_flatw<kFlatU, ABL, 0>;
        int nw = 8;
        if constexpr (UP) {
            // the column side's registers: 8 waves (2 per SIMD, 256 VGPRs; at
            // 11 waves the walk spills), or 11 with hh_tune flatw_waves_up
            nw = g_flatw_waves_up == 11 ? 11 : 8;
            kern = nw == 11 ? k_sweep_flatw<kFlatU, ABL, 2, 11, true> : k_sweep_flatw<kFlatU, ABL, 2, 8, true>;
        } else {
            if (g_flatw_waves == 10) {
                kern = g_flatw_pipe == 2 ? k_sweep_flatw<kFlatU, ABL, 2, 10> : k_sweep_flatw<kFlatU, ABL, 0, 10>;
                nw = 10;
            } else if (g_flatw_waves == 11) {
                kern = g_flatw_pipe == 2 ? k_sweep_flatw<kFlatU, ABL, 2, 11> : k_sweep_flatw<kFlatU, ABL, 0, 11>;
                nw = 11;
            }
        }
        hipLaunchKernelGGL(kern, dim3((unsigned)m->n_fgroups), dim3(64 * nw), 0, s, T, act, b,
                           (long long)m->n_bins, part);
    } else if (n_flat) {
        hipLaunchKernelGGL((k_sweep_flat<kFlatU, ABL, UP>), dim3((unsigned)n_flat), dim3(kSweepThreads), 0, s, T,
                           act, n_flat, n_tiled, b, (long long)m->n_bins, part);
    }
}

template <int NB, int ABL>
static void launch_sweep(const hh_matrix* m, const TileDev& T, const uint8_t* act, const double* b, double* part,
                         hipStream_t s, hipStream_t s_tiled, int which) {
    if constexpr (kUpperBuild) {
        if (T.upper) return launch_sweep_up<NB, ABL, true>(m, T, act, b, part, s, s_tiled, which);
    }
    launch_sweep_up<NB, ABL, false>(m, T, act, b, part, s, s_tiled, which);
}

template <int ABL>
static void launch_sweep_nb(const hh_matrix* m, const TileDev& T, const uint8_t* act, const double* b, double* part,
                            hipStream_t s, hipStream_t st, int which) {
    switch (g_sweep_nb) {
        case 1: launch_sweep<1, ABL>(m, T, act, b, part, s, st, which); break;
        case 2: launch_sweep<2, ABL>(m, T, act, b, part, s, st, which); break;
        case 8: launch_sweep<8, ABL>(m, T, act, b, part, s, st, which); break;
        default: launch_sweep<4, ABL>(m, T, act, b, part, s, st, which); break;
    }
}

// s_tiled: stream of the tiled kernel (= s, or a side stream joined by the
// caller); which: 1 the tiled kernel, 2 the flat kernel, 3 both
static void sweep(const hh_matrix* m, const TileDev& T, const uint8_t* act, const double* b, double* part,
                  hipStream_t s, hipStream_t s_tiled = nullptr, int which = 3) {
    if (m->n_units == 0) return;
    if (!s_tiled) s_tiled = s;
    switch (g_sweep_ablate) {
        case 1: launch_sweep_nb<1>(m, T, act, b, part, s, s_tiled, which); break;
        case 2: launch_sweep_nb<2>(m, T, act, b, part, s, s_tiled, which); break;
        case 3: launch_sweep_nb<3>(m, T, act, b, part, s, s_tiled, which); break;
        default: launch_sweep_nb<0>(m, T, act, b, part, s, s_tiled, which); break;
    }
    HIP_CHECK(hipGetLastError());
}

// the tile view of a state's matrix (column slots and scale when the layout
// has upper-triangle tiles)
static TileDev tdev(const hh_ice* S) { return S->m->dev(S->colpart.p, S->fix.p, S->bfix.p); }

// The matrix's band segments; returns their total chunk count.
// Dispatch order of the band chunks: by work (counts in the chunk) descending,
// ties by index (g_band_lpt 0: index order, uint8 first).
static void band_order(BandSegs& segs, int ch) {
    std::vector<std::pair<long long, int>> w;
    for (int k = 0; k < segs.n; ++k)
        for (int c = 0; c < segs.s[k].nc; ++c) {
            const long long bytes = std::min<long long>(kBandChunkB, segs.s[k].bytes - (long long)c * kBandChunkB);
            w.push_back({g_band_lpt ? -bytes * (8 / segs.s[k].bits) : 0, segs.s[k].ch + c});
        }
    std::stable_sort(w.begin(), w.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    for (int y = 0; y < ch; ++y) segs.ord[y] = (uint8_t)w[y].second;
}

static int band_segs(const hh_matrix* m, BandSegs& segs) {
    const long long W8 = m->band_w, W4 = m->band_w4;
    segs = BandSegs{};
    int ch = 0;  // first bpart chunk of the segment
    auto add = [&](const uint8_t* seg, long long stride, long long bytes, long long dlo, int bits) {
        const int nc = (int)((bytes + kBandChunkB - 1) / kBandChunkB);
        segs.s[segs.n++] = BandSeg{seg, stride, dlo, (int)bytes, nc, ch, bits};
        ch += nc;
    };
    if (W8 > 0) add(m->band.p, band_stride(W8), band_stride(W8), -W8, 8);
    if (W4 > W8) {
        const long long st = band4_stride(W8, W4), sg = band4_seg(W8, W4);
        add(m->band4.p, st, sg, -W4, 4);
        add(m->band4.p + sg, st, sg, W8 + 1, 4);
    }
    HH_REQUIRE(ch <= kMaxBandChunks, "too many band chunks");
    band_order(segs, ch);
    return ch;
}

// The upper-band segments (K1d): uint8 diagonals 0..W8 from slot W8 of each
// row, nibble diagonals W8+1..W4 from the positive segment.  A chunk covers
// kUbChunk (1008) slots; row m of a 16-row group reaches back m slots into the previous
// chunk, so the last chunk must start within 15 slots of the segment end.
static int ub_segs(const hh_ice* S, UbSegs& u) {
    const hh_matrix* m = S->m;
    const long long W8 = m->band_w, W4 = m->band_w4;
    u = UbSegs{};
    int ch = 0;
    auto add = [&](const uint8_t* loc, const uint8_t* halo, long long stride, long long dlo, long long bytes,
                   long long slots, int bits) {
        const int nc = (int)((slots + 15 + kUbChunk - 1) / kUbChunk);
        u.s[u.n++] = UbSeg{loc, halo, stride, dlo, (int)bytes, nc, ch, bits};
        ch += nc;
    };
    if (W8 > 0)
        add(m->band.p + W8, S->halo8.p ? S->halo8.p + W8 : nullptr, band_stride(W8), 0, W8 + 16, W8 + 1, 8);
    if (W4 > W8) {
        const long long sg = band4_seg(W8, W4);
        add(m->band4.p + sg, S->halo4.p ? S->halo4.p + sg : nullptr, band4_stride(W8, W4), W8 + 1, sg, W4 - W8, 4);
    }
    HH_REQUIRE(ch <= kMaxUbChunks, "too many upper-band chunks");
    // dispatch: full chunks first (every full chunk is the same count work),
    // each segment's partial last chunk at the end
    std::vector<std::pair<long long, int>> w;
    for (int k = 0; k < u.n; ++k)
        for (int c = 0; c < u.s[k].nc; ++c) {
            const long long slots = u.s[k].bits == 8 ? W8 + 1 : W4 - W8;
            w.push_back({-std::min<long long>(kUbChunk, slots + 15 - (long long)c * kUbChunk), u.s[k].ch + c});
        }
    std::stable_sort(w.begin(), w.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    for (int y = 0; y < ch; ++y) u.ord[y] = (uint8_t)w[y].second;
    return ch;
}

static UbArgs ub_args(hh_ice* S) {
    const hh_matrix* m = S->m;
    return UbArgs{m->row_lo, m->row_hi, S->halo_lo, S->nloc, S->ub_glo, S->act(), m->row_group.p, S->bias.p,
                  S->upart.p};
}

static UbMarg ub_marg(const hh_ice* S) {
    UbMarg u{};
    u.part = S->upart.p;
    u.n = S->nchu;
    if (!S->nchu) return u;
    UbSegs segs;
    ub_segs(S, segs);
    for (int k = 0; k < segs.n; ++k)
        for (int c = 0; c < segs.s[k].nc; ++c) u.base[segs.s[k].ch + c] = segs.s[k].dlo + (long long)c * kUbChunk;
    return u;
}

static void sweep_uband(hh_ice* S, hipStream_t s) {
    UbSegs segs;
    const int ch = ub_segs(S, segs);
    const long long ng = S->ub_ghi - S->ub_glo;
    if (!ch || ng <= 0) return;
    HH_KTIME("k_sweep_ubands", s);
    hipLaunchKernelGGL(k_sweep_ubands, dim3((unsigned)ng, (unsigned)ch), dim3(kUbThreads), 0, s, segs, ub_args(S),
                       (long long)S->m->n_bins, g_ub_xcd);
    HIP_CHECK(hipGetLastError());
}

static void sweep_band(hh_ice* S, hipStream_t s) {
    if (S->nchu) {
        if (S->nloc) sweep_uband(S, s);
        return;
    }
    const hh_matrix* m = S->m;
    if (!S->nch || !S->nloc) return;
    BandSegs segs;
    const int ch = band_segs(m, segs);
    // 64-row blocks when 256-row blocks would give under ~4 per CU
    const int rows = g_band_rows ? g_band_rows : (((S->nloc + 255) / 256) * ch < 1024 ? 64 : 256);
    const bool abl = g_sweep_ablate == 1;  // timing ablation (stream only)
    auto launch = [&](const BandSegs& L, int nc) {
        const unsigned rb = (unsigned)((S->nloc + rows - 1) / rows);
        auto kern = rows == 64    ? (abl ? k_sweep_bands<1, 64> : k_sweep_bands<0, 64>)
                    : rows == 128 ? (abl ? k_sweep_bands<1, 128> : k_sweep_bands<0, 128>)
                                  : (abl ? k_sweep_bands<1, 256>
                                         : (g_band_dpp ? k_sweep_bands<0, 256, true> : k_sweep_bands<0, 256, false>));
        hipLaunchKernelGGL(kern, dim3(rb, (unsigned)nc), dim3(kBandThreads), 0, s, L, (long long)S->nloc,
                           (long long)m->row_lo, (long long)m->n_bins, S->act(), m->row_group.p, S->bias.p,
                           S->bpart.p);
        HIP_CHECK(hipGetLastError());
    };
    if (g_band_fused) {
        launch(segs, ch);
    } else {
        for (int k = 0; k < segs.n; ++k) {
            BandSegs one{};
            one.s[0] = segs.s[k];
            one.n = 1;
            for (int y = 0; y < segs.s[k].nc; ++y) one.ord[y] = (uint8_t)(segs.s[k].ch + y);
            launch(one, segs.s[k].nc);
        }
    }
}

// The whole sweep as one k_sweep_all launch (small matrices).
static void sweep_single(hh_ice* S, hipStream_t s) {
    const hh_matrix* m = S->m;
    BandSegs segs;
    const int ch = (S->nch && S->nloc && !S->nchu) ? band_segs(m, segs) : (segs = BandSegs{}, 0);
    const int band_rb = (int)((S->nloc + 63) / 64);
    const int n_tiled = (int)(m->n_units - m->n_units_flat), n_flat = (int)m->n_units_flat;
    const long long n_band = ch ? (long long)band_rb * ch : 0;
    const long long grid = n_tiled + n_band + n_flat;
    if (S->nchu && S->nloc) sweep_uband(S, s);  // its own launch (its registers would cap k_sweep_all's occupancy)
    if (!grid) return;
    HH_REQUIRE(grid < (1LL << 31), "sweep grid too large for one launch");
    unsigned long long* trace = grid <= g_trace_cap ? g_trace : nullptr;
    if (trace) g_trace_n = grid;
    auto kern = g_sweep_ablate == 1   ? k_sweep_all<2, kFlatU, 1, false>
                : g_sweep_ablate == 2 ? k_sweep_all<2, kFlatU, 2, false>
                                      : k_sweep_all<2, kFlatU, 0, false>;  // ablations: timing diagnostics only
    if constexpr (kUpperBuild) {
        if (m->upper && S->colpart.p)
            kern = g_sweep_ablate == 1   ? k_sweep_all<2, kFlatU, 1, true>
                   : g_sweep_ablate == 2 ? k_sweep_all<2, kFlatU, 2, true>
                                         : k_sweep_all<2, kFlatU, 0, true>;
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kSweepThreads), 0, s, tdev(S), S->act(), n_tiled,
                       (int)n_band, segs, band_rb, (long long)S->nloc, (long long)m->row_lo, m->row_group.p,
                       S->bias.p, (long long)m->n_bins, S->part.p, S->bpart.p, trace);
    HIP_CHECK(hipGetLastError());
}

// The three-stream sweep's side streams and events, created on first use
// (matrices below conc_min_bytes never need them; stream creation per
// hh_ice_create cost the small balances ~ms).
static void ensure_side_streams(hh_ice* S) {
    if (S->side) return;
    int cur = 0;
    HIP_CHECK(hipGetDevice(&cur));
    if (cur != S->m->device) HIP_CHECK(hipSetDevice(S->m->device));
    HIP_CHECK(hipStreamCreateWithFlags(&S->side, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreateWithFlags(&S->fork, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&S->join, hipEventDisableTiming));
    HIP_CHECK(hipStreamCreateWithFlags(&S->side2, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreateWithFlags(&S->join2, hipEventDisableTiming));
    if (cur != S->m->device) HIP_CHECK(hipSetDevice(cur));
}

static void marg_weighted(hh_ice* S, double* out, hipStream_t s, bool timed, int slot) {
    hh_matrix* m = S->m;
    const bool up = m->upper && S->colpart.p;
    const bool shard_x = up && S->cx_world > 1;  // the column side crosses ranks
    HH_REQUIRE(!shard_x || S->rmax_global,
               "upper-triangle tiles on a shard: run the filters on the gathered marginals first (global scale)");
    if (timed) HIP_CHECK(hipEventRecord(S->ev[2 * slot], s));
    if (up)
        hipLaunchKernelGGL(k_fixscale, dim3(nblocks(std::max<int64_t>(S->n, 1), 256)), dim3(256), 0, s, S->bmax.p,
                           S->iters_done & 1, S->rmax, S->fix.p, S->bias.p, (long long)S->n, S->bfix.p);
    const TileDev T = tdev(S);
    {
        HH_KTIME(timed ? nullptr : "ice_sweep", s);  // registry timing for the sharded driver (tiled + flat + band)
        // the two sweeps write disjoint partials (part / bpart): the band
        // kernel runs on a side stream so its blocks fill the CUs the tile
        // kernel leaves idle (both are HBM-bound; neither saturates alone)
        const int64_t bytes = 4 * m->n_slots + 2 * m->n_slots_narrow + (int64_t)m->band.n + (int64_t)m->band4.n;
        // (with the upper-band sweep -- C4 and its shards -- from 1 GB: the N = 8
        // C4 shards (1.85 GB) sweep in 0.567 vs 0.637 ms max, N = 4 0.976 vs
        // 1.018 ms; C3 (3.0 GB, no upper band) stays faster on one stream,
        // 1250 vs 1177 it/s; profiles/r4f_conc_ab.log)
        const bool conc = g_band_concurrent && (S->nch || S->nchu) && S->nloc && m->n_units &&
                          (bytes >= g_conc_min_bytes || (S->nchu && bytes >= g_conc_ub_min_bytes));
        // (not with upper tiles in column-grouped flat units: their column
        // side has one slot per group, which only k_sweep_flatw fills)
        // (k_sweep_all walks flat tiles per unit in the plain layout: never on
        // a layout with column-grouped, interleaved flat tiles)
        const bool single = g_sweep_nb == 2 && !(up && m->n_fgroups) && !m->flat_perm &&
                            (g_sweep_single == 1 || (g_sweep_single == -1 && bytes < g_single_max_bytes));
        if (single) {
            sweep_single(S, s);
        } else if (conc) {
            ensure_side_streams(S);
            HIP_CHECK(hipEventRecord(S->fork, s));
            HIP_CHECK(hipStreamWaitEvent(S->side, S->fork, 0));
            if (g_split_tiles) HIP_CHECK(hipStreamWaitEvent(S->side2, S->fork, 0));
            if (g_conc_order == 1) {
                // the flat blocks (most of a CU's LDS) dispatched first, then
                // the band blocks, then the tiled kernel (C4: sweep 2.98 ->
                // 2.89 ms, profiles/r6j/)
                sweep(m, T, S->act(), S->bias.p, S->part.p, s, s, 2);
                sweep_band(S, S->side);
                sweep(m, T, S->act(), S->bias.p, S->part.p, s, g_split_tiles ? S->side2 : s, 1);
            } else if (g_conc_order == 2) {  // flat, tiled, band
                sweep(m, T, S->act(), S->bias.p, S->part.p, s, s, 2);
                sweep(m, T, S->act(), S->bias.p, S->part.p, s, g_split_tiles ? S->side2 : s, 1);
                sweep_band(S, S->side);
            } else {
                sweep_band(S, S->side);
                sweep(m, T, S->act(), S->bias.p, S->part.p, s, g_split_tiles ? S->side2 : s);
            }
            HIP_CHECK(hipEventRecord(S->join, S->side));
            if (g_split_tiles) {
                HIP_CHECK(hipEventRecord(S->join2, S->side2));
                HIP_CHECK(hipStreamWaitEvent(s, S->join2, 0));
            }
            HIP_CHECK(hipStreamWaitEvent(s, S->join, 0));
        } else {
            sweep(m, T, S->act(), S->bias.p, S->part.p, s);
            sweep_band(S, s);
        }
        if (up && S->n > 0) {  // every column's upper-tile side: the slots of its column tile
            hipLaunchKernelGGL(k_colsum, dim3(nblocks(S->n, 256)), dim3(256), 0, s, S->colpart.p, m->jslot_ptr.p,
                               m->jslot.p, 0LL, (long long)S->n, S->colacc.p);
            HIP_CHECK(hipGetLastError());
        }
    }
    if (timed) HIP_CHECK(hipEventRecord(S->ev[2 * slot + 1], s));
    // the column side of this shard's rows: summed over the ranks
    const unsigned long long* col_own = up ? S->colacc.p + m->row_lo : nullptr;
    if (shard_x) {
        const long long tot = (long long)S->cx_world * S->cx_maxlen;
        hipLaunchKernelGGL(k_colpad, dim3(nblocks(tot, kThreads)), dim3(kThreads), 0, s, S->colacc.p, S->cx_world,
                           (long long)S->cx_maxlen, S->cx_rr_dev.p, S->cx_send.p);
        HIP_CHECK(hipGetLastError());
        int rc = 0;
        if (S->cx_fn) {
            rc = S->cx_fn(reinterpret_cast<const int64_t*>(S->cx_send.p), S->cx_maxlen,
                          reinterpret_cast<int64_t*>(S->cx_recv.p), S->cx_user, s);
        } else {  // through the all-gather: every rank's padded vector, summed here in rank order
            rc = S->cx_ag(reinterpret_cast<const double*>(S->cx_send.p), tot, reinterpret_cast<double*>(S->cx_all.p),
                          S->cx_ag_user, s);
            if (!rc)
                hipLaunchKernelGGL(k_colgather, dim3(nblocks(S->cx_maxlen, kThreads)), dim3(kThreads), 0, s,
                                   S->cx_all.p, S->cx_world, (long long)S->cx_maxlen, S->cx_rank, S->cx_recv.p);
        }
        if (rc) HH_THROW(rc < 0 ? rc : HH_ERR_HIP, std::string("column exchange failed: ") + hh_last_error());
        col_own = S->cx_recv.p;
    }
    S->stats_fresh = false;
    if (S->nloc == 0) return;
    // stats fused into k_marg when this GPU holds every row and `out` is the
    // marginal vector update() reads (k_stats1's tile sums, bitwise)
    // 1: tile sums + the last-block group tail (few tiles); 2: tile sums only
    // (k_stats1's work without its launch; k_stats2 / k_update_big reduce)
    const int stats = (g_fuse_stats != 0 && S->full() && out == S->marg.p && S->n_tiles > 0)
                          ? (S->small_stats() ? 1 : 2)
                          : 0;
    HH_KTIME(timed ? nullptr : "k_marg", s);
    hipLaunchKernelGGL(k_marg, dim3(nblocks(S->nloc, kR)), dim3(kMargThreads), 0, s, T, S->part.p,
                       m->wide_ptr.p, m->wide_col.p, m->wide_cnt.p, m->diag.p, m->row_group.p, S->act(),
                       S->bias.p, (long long)m->row_lo, (int)S->nloc, S->bpart.p, S->nchu ? 0 : (int)S->nch,
                       ub_marg(S), out, S->ta(),
                       (int)S->G, stats, col_own);
    HIP_CHECK(hipGetLastError());
    S->stats_fresh = stats != 0;
}

// the bias-maximum slot the update of this iteration fills (read by the next
// sweep's k_fixscale, which cleared it)
static unsigned long long* bmax_next(hh_ice* S) {
    return S->bmax.p ? S->bmax.p + (1 - (S->iters_done & 1)) : nullptr;
}

static void update(hh_ice* S, hipStream_t s) {
    TileArgs ta = S->ta();
    if (S->n_tiles) {
        GroupState gs{S->g_var.p, S->g_mean.p, S->g_iters.p, S->g_empty.p};
        if (S->small_stats()) {
            if (!S->stats_fresh)
                hipLaunchKernelGGL(k_stats1<true>, dim3(S->n_tiles), dim3(kR), 0, s, ta, S->act(), S->marg.p,
                                   (int)S->G);
            hipLaunchKernelGGL(k_update, dim3(S->n_tiles), dim3(kR), 0, s, ta, S->act(), S->nxt(), S->marg.p,
                               S->bias.p, gs, S->o.tol, S->o.max_iters, (int)S->G, bmax_next(S));
        } else {
            if (!S->stats_fresh)
                hipLaunchKernelGGL(k_stats1<false>, dim3(S->n_tiles), dim3(kR), 0, s, ta, S->act(), S->marg.p,
                                   (int)S->G);
            hipLaunchKernelGGL(k_stats2, dim3(S->n_tiles), dim3(kR), 0, s, ta, S->act(), S->marg.p);
            hipLaunchKernelGGL(k_update_big, dim3(S->n_tiles), dim3(kR), 0, s, ta, S->act(), S->nxt(), S->marg.p,
                               S->bias.p, gs, S->o.tol, S->o.max_iters, bmax_next(S));
        }
        HIP_CHECK(hipGetLastError());
    }
    S->stats_fresh = false;
    // groups without tiles never run; keep their flag cleared in the next buffer
    S->iters_done += 1;
}

static void check_opts(const hh_ice_opts* o) {
    HH_REQUIRE(o, "null options");
    HH_REQUIRE(o->max_iters >= 1, "max_iters must be >= 1");
    HH_REQUIRE(o->min_nnz >= 0 && o->mad_max >= 0, "negative filter threshold");
}

}  // namespace hh

// MIN-count and MAD-max filters (cooler balance_cooler): per-chromosome median
// normalisation of the raw marginal, then a log-MAD cutoff over the whole
// genome.  O(n) host work with numpy's median semantics; run once per balance.
// `gather` (may be null) turns this matrix's normalised marginals into the
// genome's (the cis-only-by-chromosome sharding: every rank holds whole
// chromosomes, so the per-chromosome medians are local and only the
// genome-wide median of the logs needs the other ranks' values).
static void filter_count_mad(hh_ice* S, hipStream_t s,
                             const std::function<std::vector<double>(const std::vector<double>&)>& gather) {
    if (S->o.min_count != 0.0)
        hipLaunchKernelGGL(k_filter_lt, dim3(nblocks(S->n, kThreads)), dim3(kThreads), 0, s, S->marg.p,
                           (long long)S->n, S->o.min_count, S->bias.p);
    HIP_CHECK(hipGetLastError());
    if (S->o.mad_max <= 0) return;
    std::vector<double> marg(S->n), bias(S->n);
    {
        PinnedDown dl;
        dl.add(S->marg.p, marg.data(), (size_t)S->n);
        dl.add(S->bias.p, bias.data(), (size_t)S->n);
        dl.run(s);
    }
    const auto& off = S->m->chrom_offsets;
    std::vector<double> pos;
    for (int c = 0; c < S->m->n_chroms; ++c) {
        pos.clear();
        for (int64_t i = off[c]; i < off[c + 1]; ++i)
            if (marg[i] > 0) pos.push_back(marg[i]);
        const double med = np_median(pos);
        for (int64_t i = off[c]; i < off[c + 1]; ++i) marg[i] = marg[i] / med;
    }
    const std::vector<double> all = gather ? gather(marg) : marg;
    std::vector<double> logm;
    for (double x : all)
        if (x > 0) logm.push_back(std::log(x));
    const double med = np_median(logm);
    std::vector<double> dev(logm.size());
    for (size_t k = 0; k < logm.size(); ++k) dev[k] = std::fabs(logm[k] - med);
    const double cutoff = std::exp(med - S->o.mad_max * np_median(dev));
    for (int64_t i = 0; i < S->n; ++i)
        if (marg[i] < cutoff) bias[i] = 0.0;
    upload_pinned_sync(S->bias.p, bias.data(), (size_t)S->n, s);
}

extern "C" {

int hh_tune(const char* key, int64_t value) {
    return guard([&] {
        HH_REQUIRE(key, "null key");
        const std::string k(key);
        if (k == "sweep_nb") {
            HH_REQUIRE(value == 1 || value == 2 || value == 4 || value == 8, "sweep_nb must be 1, 2, 4 or 8");
            g_sweep_nb = (int)value;
        } else if (k == "sweep_ablate") {
            HH_REQUIRE(value >= 0 && value <= 3, "sweep_ablate must be 0, 1, 2 or 3");
            g_sweep_ablate = (int)value;
        } else if (k == "band4_density_pct" || k == "band8_big_pct") {
            HH_REQUIRE(value >= 1 && value <= 100, "percent in [1, 100]");
            (k == "band4_density_pct" ? g_band4_density : g_band8_big) = (double)value / 100.0;
        } else if (k == "band4") {
            HH_REQUIRE(value == 0 || value == 1, "band4 in {0, 1}");
            g_band4 = value;
        } else if (k == "flat_cols") {
            HH_REQUIRE(value >= -1 && value <= 1, "flat_cols in {-1 (auto), 0, 1}");
            g_flat_cols = value;
        } else if (k == "flatw_pipe") {
            HH_REQUIRE(value >= 0 && value <= 2, "flatw_pipe in {0, 1, 2}");
            g_flatw_pipe = (int)value;
        } else if (k == "band_dpp") {
            HH_REQUIRE(value == 0 || value == 1, "band_dpp in {0, 1}");
            g_band_dpp = (int)value;
        } else if (k == "flatw_u") {  // (16 measured slower in round 4; the interleaved layout is for 8)
            HH_REQUIRE(value == 8, "flatw_u: 8 (the interleaved flat layout's run length)");
        } else if (k == "flatw_waves_up") {
            HH_REQUIRE(value == 8 || value == 11, "flatw_waves_up in {8, 11}");
            g_flatw_waves_up = (int)value;
        } else if (k == "upper_tiles") {
            HH_REQUIRE(value >= -1 && value <= 1, "upper_tiles in {-1 (auto), 0, 1}");
            HH_REQUIRE(kUpperBuild || value != 1,
                       "upper-triangle tiles need the 4096-column build (libhichap_hip_up.so, -DHH_KWBITS=12)");
            g_upper_tiles = value;
        } else if (k == "flat_max") {
            HH_REQUIRE(value >= 0 && value <= 255, "flat_max in [0, 255]");
            g_flat_max = value;
        } else if (k == "unit_entries") {
            HH_REQUIRE(value == 0 || (value >= 4096 && value <= (1 << 24)), "unit_entries must be 0 (auto) or in [4096, 2^24]");
            g_unit_entries = value;
        } else if (k == "flat_defer") {
            HH_REQUIRE(value == 0 || value == 1, "flat_defer in {0, 1}");
            g_flat_defer = (int)value;
        } else if (k == "unit_lpt") {
            HH_REQUIRE(value >= 0 && value <= 2, "unit_lpt in {0, 1, 2}");
            g_unit_lpt = value;
        } else if (k == "unit_lpt_lists") {
            HH_REQUIRE(value >= 0 && value <= 3, "unit_lpt_lists in [0, 3]");
            g_unit_lpt_lists = value;
        } else if (k == "tile_cost") {
            HH_REQUIRE(value >= 0 && value <= (1 << 20), "tile_cost in [0, 2^20] payload words");
            g_tile_cost = value;
        } else if (k == "parse_ablate") {
            HH_REQUIRE(value >= 0 && value <= 3, "parse_ablate in [0, 3]");
            g_parse_ablate = (int)value;
        } else if (k == "flatw_waves") {
            HH_REQUIRE(value == 8 || value == 10 || value == 11, "flatw_waves: 8, 10 or 11");
            g_flatw_waves = (int)value;
        } else if (k == "flat_group") {
            HH_REQUIRE(value >= 0 && value <= 256, "flat_group: 0 (auto) .. 256");
            g_flat_group = value;
        } else if (k == "uband") {
            HH_REQUIRE(value >= 0 && value <= 2, "uband: 0 (off), 1 (auto) or 2 (always)");
            g_uband = (int)value;
        } else if (k == "ub_xcd") {
            HH_REQUIRE(value == 0 || value == 1, "ub_xcd: 0 or 1");
            g_ub_xcd = (int)value;
        } else if (k == "uband_min_bytes") {
            HH_REQUIRE(value >= 0, "uband_min_bytes >= 0");
            g_uband_min_bytes = value;
        } else if (k == "band_w") {
            HH_REQUIRE(value >= -1 && value <= kBandMaxW && (value <= 0 || value % 16 == 0),
                       "band_w: -1 (auto), 0 (off) or a multiple of 16 <= 16384");
            g_band_w = value;
        } else if (k == "conc_min_bytes") {
            HH_REQUIRE(value >= 0, "conc_min_bytes >= 0");
            g_conc_min_bytes = value;
        } else if (k == "syrk_split") {
            HH_REQUIRE(value >= -1 && value <= 64, "syrk_split in [-1, 64]");
            g_syrk_split = (int)value;
        } else if (k == "band_lpt") {
            HH_REQUIRE(value == 0 || value == 1, "band_lpt in {0, 1}");
            g_band_lpt = (int)value;
        } else if (k == "fuse_stats") {
            HH_REQUIRE(value >= -1 && value <= 2, "fuse_stats in {-1, 0, 1, 2}");
            g_fuse_stats = (int)value;
        } else if (k == "conc_order") {
            HH_REQUIRE(value >= 0 && value <= 2, "conc_order in {0, 1, 2}");
            g_conc_order = (int)value;
        } else if (k == "split_tiles") {
            HH_REQUIRE(value == 0 || value == 1, "split_tiles in {0, 1}");
            g_split_tiles = (int)value;
        } else if (k == "pca_method") {
            HH_REQUIRE(value == 0 || value == 1, "pca_method in {0, 1}");
            g_pca_method = (int)value;
        } else if (k == "host_build") {
            HH_REQUIRE(value == 0 || value == 1, "host_build in {0, 1}");
            g_host_build = value;
        } else if (k == "build_debug") {
            g_build_debug = value;
        } else if (k == "pca_debug") {
            g_pca_debug = (int)value;
        } else if (k == "conc_ub_min_bytes") {
            HH_REQUIRE(value >= 0, "conc_ub_min_bytes >= 0");
            g_conc_ub_min_bytes = value;
        } else if (k == "ortho_lowsync") {
            g_ortho_lowsync = value ? 1 : 0;
        } else if (k == "ortho_grid_cap") {
            HH_REQUIRE(value >= 0 && value <= 64, "ortho_grid_cap in [0, 64]");
            g_ortho_grid_cap = (int)value;
        } else if (k == "symvc_rows") {
            HH_REQUIRE(value >= 16 && value <= 1024 && value % 16 == 0, "symvc_rows in [16, 1024], a multiple of 16");
            g_symvc_rows = (int)value;
        } else if (k == "symvc_out") {
            g_symvc_out = value ? 1 : 0;
        } else if (k == "twostep_budget_mb") {
            HH_REQUIRE(value >= 0, "twostep_budget_mb >= 0 (0: the free device memory)");
            g_twostep_budget = value << 20;
        } else if (k == "twostep_devglue") {
            g_twostep_devglue = value ? 1 : 0;
        } else if (k == "symvc_stream") {
            g_symvc_stream = value ? 1 : 0;
        } else if (k == "ortho_abort_test") {
            HH_REQUIRE(value >= 0 && value <= 2, "ortho_abort_test in {0, 1, 2}");
            g_ortho_abort_test = (int)value;
        } else if (k == "pca_coop") {
            HH_REQUIRE(value == 0 || value == 1, "pca_coop in {0, 1}");
            g_pca_coop = (int)value;
        } else if (k == "cor_sym") {
            HH_REQUIRE(value >= 0 && value <= 3, "cor_sym in {0, 1, 2, 3}");
            g_cor_sym = (int)value;
        } else if (k == "ortho_tpb") {
            HH_REQUIRE(value == 0 || value == 1 || value == 2 || value == 4 || value == 8,
                       "ortho_tpb in {0 (auto), 1, 2, 4, 8}");
            g_ortho_tpb = (int)value;
        } else if (k == "ortho_min_tpb") {
            HH_REQUIRE(value == 1 || value == 2, "ortho_min_tpb in {1, 2}");
            g_ortho_min_tpb = (int)value;
        } else if (k == "pca_p") {
            HH_REQUIRE(value >= 2 && value <= 8, "pca_p in [2, 8]");
            g_pca_p = (int)value;
        } else if (k == "band_rows") {
            HH_REQUIRE(value == 0 || value == 64 || value == 128 || value == 256,
                       "band_rows in {0 (auto), 64, 128, 256}");
            g_band_rows = (int)value;
        } else if (k == "sweep_trace") {
            HH_REQUIRE(value >= 0 && value < (1LL << 31), "sweep_trace: block capacity >= 0");
            if (g_trace) HIP_CHECK(hipFree(g_trace));
            g_trace = nullptr;
            g_trace_cap = g_trace_n = 0;
            if (value) HIP_CHECK(hipMalloc(&g_trace, (size_t)value * 3 * sizeof(unsigned long long)));
            g_trace_cap = value;
        } else if (k == "iter_events") {
            HH_REQUIRE(value == 0 || value == 1, "iter_events in {0, 1}");
            g_iter_events = (int)value;
        } else if (k == "sweep_single") {
            HH_REQUIRE(value >= -1 && value <= 1, "sweep_single in {-1 (auto), 0, 1}");
            g_sweep_single = (int)value;
        } else if (k == "single_max_bytes") {
            HH_REQUIRE(value >= 0, "single_max_bytes >= 0");
            g_single_max_bytes = value;
        } else if (k == "band_fused") {
            HH_REQUIRE(value == 0 || value == 1, "band_fused in {0, 1}");
            g_band_fused = (int)value;
        } else if (k == "band_concurrent") {
            HH_REQUIRE(value == 0 || value == 1, "band_concurrent in {0, 1}");
            g_band_concurrent = (int)value;
        } else {
            HH_THROW(HH_ERR_ARG, "unknown tuning key " + k);
        }
    });
}

int hh_ice_create(hh_matrix* m, const hh_ice_opts* o, hh_ice** out) {
    return guard([&] {
        HH_REQUIRE(m && out, "null");
        check_opts(o);
        HIP_CHECK(hipSetDevice(m->device));
        auto S = std::make_unique<hh_ice>();
        S->m = m;
        S->o = *o;
        if (S->o.check_every <= 0) S->o.check_every = 8;
        S->n = m->n_bins;
        S->nloc = m->nloc();
        if (m->cis_only) {
            S->G = m->n_chroms;
            for (int c = 0; c < m->n_chroms; ++c) {
                S->glo.push_back(m->chrom_offsets[c]);
                S->ghi.push_back(m->chrom_offsets[c + 1]);
            }
        } else {
            S->G = 1;
            S->glo = {0};
            S->ghi = {m->n_bins};
        }
        std::vector<int32_t> tlo, thi, tg, gtp(S->G + 1, 0);
        for (int g = 0; g < S->G; ++g) {
            gtp[g] = (int32_t)tlo.size();
            // stats tiles: the group's rows cut at 512-row block boundaries
            for (int64_t b = S->glo[g]; b < S->ghi[g];) {
                const int64_t e = std::min<int64_t>((b / kR + 1) * kR, S->ghi[g]);
                tlo.push_back((int32_t)b);
                thi.push_back((int32_t)e);
                tg.push_back(g);
                b = e;
            }
        }
        gtp[S->G] = (int32_t)tlo.size();
        S->n_tiles = (int32_t)tlo.size();
        const int64_t nblk = (S->n + kR - 1) / kR;
        std::vector<int32_t> btp(nblk + 1, 0);
        for (size_t t = 0, B = 0; B <= (size_t)nblk; ++B) {  // tiles are in row order
            while (t < tlo.size() && tlo[t] < (int64_t)B * kR) ++t;
            btp[B] = (int32_t)t;
        }
        hipStream_t s = 0;
        S->tile_lo = to_device(tlo, s);
        S->tile_hi = to_device(thi, s);
        S->tile_group = to_device(tg, s);
        S->group_tile_ptr = to_device(gtp, s);
        S->blk_tile_ptr = to_device(btp, s);
        S->g_cnt.alloc(S->G);
        S->g_sum.alloc(S->G);
        S->counter.alloc(2);
        S->counter.zero(s);
        S->bias.alloc(S->n);
        std::vector<double> ones(S->n, 1.0);
        upload_pinned_sync(S->bias.p, ones.data(), (size_t)S->n, s);
        S->marg.alloc(S->n);
        S->marg.zero(s);
        S->part.alloc(std::max<int64_t>(m->n_part, 1));
        S->nch = m->band_w > 0 ? (int32_t)((band_stride(m->band_w) + kBandChunk - 1) / kBandChunk) : 0;
        if (m->band_w4 > m->band_w)
            S->nch += 2 * (int32_t)((band4_seg(m->band_w, m->band_w4) + kBandChunk - 1) / kBandChunk);
        const int64_t band_all = m->n_bins * ((m->band_w > 0 ? band_stride(m->band_w) : 0) +
                                              (m->band_w4 > m->band_w ? band4_stride(m->band_w, m->band_w4) : 0));
        if (S->nch && (g_uband == 2 || (g_uband == 1 && band_all >= g_uband_min_bytes))) {
            // upper-band sweep: workgroups whose rows or columns reach the
            // shard, halo rows above it (upper halves from the shard's own
            // lower halves), zeroed partials (positions no workgroup writes
            // stay 0)
            const long long dmax = std::max<long long>(m->band_w, m->band_w4);
            S->ub_glo = std::max<long long>(0, m->row_lo - dmax - kUbCols) / kUbGroupRows;
            S->ub_ghi = (m->row_hi + kUbGroupRows - 1) / kUbGroupRows;
            S->halo_lo = std::min<long long>(m->row_lo, S->ub_glo * kUbGroupRows);
            const long long nh = m->row_lo - S->halo_lo;
            if (nh > 0 && S->nloc > 0) {  // (an empty shard sweeps nothing: no halo)
                const long long W8 = m->band_w, W4 = m->band_w4;
                const long long per = W8 + (W4 > W8 ? band4_seg(W8, W4) : 0);
                if (W8 > 0) {
                    S->halo8.alloc((size_t)(nh * band_stride(W8)));
                    S->halo8.zero(s);
                }
                if (W4 > W8) {
                    S->halo4.alloc((size_t)(nh * band4_stride(W8, W4)));
                    S->halo4.zero(s);
                }
                const long long nthr = nh * per;
                hipLaunchKernelGGL(k_ub_halo, dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, s, m->band.p,
                                   m->band4.p, W8, W4, (long long)m->row_lo, (long long)m->row_hi, S->halo_lo,
                                   S->halo8.p, S->halo4.p);
                HIP_CHECK(hipGetLastError());
            }
            UbSegs segs;
            S->nchu = ub_segs(S.get(), segs);
            S->upart.alloc(std::max<int64_t>((int64_t)kUbArrs * S->nchu * S->nloc, 1));
            S->upart.zero(s);
            S->nch = 0;
        }
        S->bpart.alloc(std::max<int64_t>((int64_t)S->nch * S->nloc, 1));
        // (the side streams of the three-stream sweep are made on first use)
        if (m->upper && m->n_cslots > 0) {
            S->colpart.alloc((size_t)m->n_cslots * kW);
            S->colpart.zero(s);
        }
        if (m->upper) {
            S->colacc.alloc((size_t)std::max<int64_t>(S->n, 1));
            S->colacc.zero(s);
            // the initial bias is 1 (filters only zero entries): bmax slot 0 = 1.0
            const unsigned long long one[2] = {0x3FF0000000000000ull, 0ull};
            S->bmax = to_device(std::vector<unsigned long long>(one, one + 2), s);
            S->fix.alloc(2);
            S->bfix.alloc((size_t)std::max<int64_t>(S->n, 1));
            // the largest raw marginal bounds every column's count total; a
            // shard's own rows are not enough (columns of other ranks): the
            // filters set the global one from the gathered marginals
            std::vector<double> rs((size_t)S->nloc);
            if (S->nloc) m->row_sum2.download(rs.data(), (size_t)S->nloc, s);
            HIP_CHECK(hipStreamSynchronize(s));
            for (double x : rs) S->rmax = std::max(S->rmax, x);
            S->rmax_global = S->full();
        }

        S->tile_cnt.alloc(std::max(S->n_tiles, 1));
        S->tile_sum.alloc(std::max(S->n_tiles, 1));
        S->tile_sq.alloc(std::max(S->n_tiles, 1));
        std::vector<uint8_t> act(2 * S->G, 0);
        std::vector<uint8_t> emp(S->G, 0);
        for (int g = 0; g < S->G; ++g) {
            act[g] = gtp[g + 1] > gtp[g] ? 1 : 0;
            emp[g] = act[g] ? 0 : 1;
        }
        S->active = to_device(act, s);
        S->g_empty = to_device(emp, s);
        S->g_var.alloc(S->G);
        S->g_var.zero(s);
        std::vector<double> nan(S->G, std::numeric_limits<double>::quiet_NaN());
        S->g_mean = to_device(nan, s);
        S->g_iters.alloc(S->G);
        S->g_iters.zero(s);
        S->h_active.alloc(2 * S->G);
        HIP_CHECK(hipStreamSynchronize(s));
        *out = S.release();
    });
}

int hh_ice_free(hh_ice* s) {
    return guard([&] {
        if (s) device_quiesce(s->m->device);
        delete s;
    });
}

int hh_ice_n_groups(const hh_ice* s, int32_t* n) {
    return guard([&] { HH_REQUIRE(s && n, "null"); *n = s->G; });
}

int hh_ice_marg_local(hh_ice* S, int32_t mode, double* marg_local, void* stream) {
    return guard([&] {
        HH_REQUIRE(S, "null");
        HH_REQUIRE(mode >= 0 && mode <= 2, "mode must be 0, 1 or 2");
        HH_REQUIRE(marg_local || S->full(), "marg_local required for a sharded matrix");
        hipStream_t s = as_stream(stream);
        double* out = marg_local ? marg_local : S->marg.p + S->m->row_lo;
        if (mode == 2) {
            marg_weighted(S, out, s, false, 0);
        } else {
            S->stats_fresh = false;
            const DBuf<double>& src = mode == 0 ? S->m->row_nnz2 : S->m->row_sum2;
            if (S->nloc)
                HIP_CHECK(hipMemcpyAsync(out, src.p, S->nloc * sizeof(double), hipMemcpyDeviceToDevice, s));
        }
    });
}

int hh_ice_set_marg(hh_ice* S, const double* gathered, int32_t world, int64_t maxlen,
                    const int64_t* rank_rows, void* stream) {
    return guard([&] {
        HH_REQUIRE(S && gathered && rank_rows && world >= 1 && maxlen >= 0, "bad arguments");
        hipStream_t s = as_stream(stream);
        std::vector<int64_t> rr(rank_rows, rank_rows + world + 1);
        HH_REQUIRE(rr[0] == 0 && rr[world] == S->n, "rank_rows must span [0, n_bins]");
        for (int k = 0; k < world; ++k) HH_REQUIRE(rr[k + 1] - rr[k] <= maxlen && rr[k] <= rr[k + 1], "bad rank_rows");
        if (rr != S->h_rank_rows) {
            HIP_CHECK(hipStreamSynchronize(s));
            S->h_rank_rows = rr;
            std::vector<long long> ll(rr.begin(), rr.end());
            S->rank_rows = to_device(ll, s);
        }
        S->stats_fresh = false;
        const long long tot = (long long)world * maxlen;
        if (tot)
            hipLaunchKernelGGL(k_scatter, dim3(nblocks(tot, kThreads)), dim3(kThreads), 0, s, gathered, world,
                               (long long)maxlen, S->rank_rows.p, S->marg.p);
        HIP_CHECK(hipGetLastError());
    });
}

int hh_ice_filter_nnz(hh_ice* S, void* stream) {
    return guard([&] {
        HH_REQUIRE(S, "null");
        if (S->o.min_nnz > 0)
            hipLaunchKernelGGL(k_filter_lt, dim3(nblocks(S->n, kThreads)), dim3(kThreads), 0, as_stream(stream),
                               S->marg.p, (long long)S->n, (double)S->o.min_nnz, S->bias.p);
        HIP_CHECK(hipGetLastError());
    });
}

int hh_ice_filter_count_mad(hh_ice* S, void* stream) {
    return guard([&] {
        HH_REQUIRE(S, "null");
        if (S->m->upper && !S->full()) {
            // S->marg holds every bin's raw marginal here (gathered, mode 1):
            // the global count bound of the column side's fixed-point scale
            std::vector<double> mg((size_t)S->n);
            S->marg.download(mg.data(), (size_t)S->n, as_stream(stream));
            HIP_CHECK(hipStreamSynchronize(as_stream(stream)));
            double r = 1.0;
            for (double x : mg) r = std::max(r, x);
            S->rmax = r;
            S->rmax_global = true;
        }
        filter_count_mad(S, as_stream(stream), nullptr);
    });
}

int hh_ice_update(hh_ice* S, void* stream) {
    return guard([&] {
        HH_REQUIRE(S, "null");
        update(S, as_stream(stream));
    });
}

int hh_ice_active_groups(hh_ice* S, int32_t* n_active, void* stream) {
    return guard([&] {
        HH_REQUIRE(S && n_active, "null");
        hipStream_t s = as_stream(stream);
        HIP_CHECK(hipMemcpyAsync(S->h_active.p, S->act(), S->G, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        int a = 0;
        for (int g = 0; g < S->G; ++g) a += S->h_active.p[g] ? 1 : 0;
        *n_active = a;
    });
}

int hh_ice_iterations_done(const hh_ice* S, int32_t* iters) {
    return guard([&] { HH_REQUIRE(S && iters, "null"); *iters = S->iters_done; });
}

int hh_ice_run(hh_ice* S, int32_t n, void* stream) {
    return guard([&] {
        HH_REQUIRE(S && n >= 0, "bad arguments");
        HH_REQUIRE(S->full(), "hh_ice_run needs a matrix holding every row (use the sharded API)");
        hipStream_t s = as_stream(stream);
        const size_t need = 2 * (size_t)n + 2;
        while (S->ev.size() < need) {
            hipEvent_t e;
            HIP_CHECK(hipEventCreate(&e));
            S->ev.push_back(e);
        }
        HIP_CHECK(hipEventRecord(S->ev[2 * n], s));
        const bool ev = g_iter_events != 0;  // (0: no per-sweep events; sweep_ms then 0)
        for (int k = 0; k < n; ++k) {
            marg_weighted(S, S->marg.p, s, ev, k);
            update(S, s);
        }
        HIP_CHECK(hipEventRecord(S->ev[2 * n + 1], s));
        HIP_CHECK(hipStreamSynchronize(s));
        double tot = 0.0;
        for (int k = 0; ev && k < n; ++k) {
            float ms = 0.f;
            HIP_CHECK(hipEventElapsedTime(&ms, S->ev[2 * k], S->ev[2 * k + 1]));
            tot += ms;
        }
        float all = 0.f;
        HIP_CHECK(hipEventElapsedTime(&all, S->ev[2 * n], S->ev[2 * n + 1]));
        S->sweep_ms = tot;
        S->iter_ms = all;
        S->sweep_launches = n;
    });
}

int hh_ice_last_sweep_timing(const hh_ice* S, double* sweep_ms_total, int32_t* sweep_launches,
                             double* iter_ms_total) {
    return guard([&] {
        HH_REQUIRE(S, "null");
        if (sweep_ms_total) *sweep_ms_total = S->sweep_ms;
        if (sweep_launches) *sweep_launches = S->sweep_launches;
        if (iter_ms_total) *iter_ms_total = S->iter_ms;
    });
}

int hh_ice_set_column_exchange(hh_ice* S, int32_t world, int32_t rank, const int64_t* rank_rows, hh_reduce_fn reduce,
                               void* reduce_user, hh_allgather_fn allgather, void* allgather_user) {
    return guard([&] {
        HH_REQUIRE(S && world >= 1 && rank_rows && rank >= -1 && rank < world, "bad arguments");
        HH_REQUIRE(world == 1 || reduce || allgather || (S->cx_fn && S->cx_world == world),
                   "a reduce or all-gather function is required for world > 1");
        std::vector<int64_t> rr(rank_rows, rank_rows + world + 1);
        HH_REQUIRE(rr[0] == 0 && rr[world] == S->n, "rank_rows must span [0, n_bins]");
        int64_t maxlen = 1;
        for (int k = 0; k < world; ++k) {
            HH_REQUIRE(rr[k] <= rr[k + 1], "rank_rows not monotone");
            maxlen = std::max<int64_t>(maxlen, rr[k + 1] - rr[k]);
        }
        if (rank < 0) {  // this shard's block (any of equal empty ranges: its rows are none)
            for (int k = 0; k < world && rank < 0; ++k)
                if (rr[k] == S->m->row_lo && rr[k + 1] == S->m->row_hi) rank = k;
            HH_REQUIRE(rank >= 0, "the matrix shard is none of rank_rows' ranges");
        }
        HH_REQUIRE(rr[rank] == S->m->row_lo && rr[rank + 1] == S->m->row_hi,
                   "the matrix shard does not hold rank_rows[rank] .. rank_rows[rank + 1]");
        if (!reduce && S->cx_fn && S->cx_world == world) {
            reduce = S->cx_fn;
            reduce_user = S->cx_user;
        }
        S->cx_world = world;
        S->cx_rank = rank;
        S->cx_maxlen = maxlen;
        S->cx_fn = reduce;
        S->cx_user = reduce_user;
        S->cx_ag = allgather;
        S->cx_ag_user = allgather_user;
        if (rr != S->cx_rr) {
            S->cx_rr = rr;
            std::vector<long long> ll(rr.begin(), rr.end());
            S->cx_rr_dev = to_device(ll, 0);
            HIP_CHECK(hipStreamSynchronize(0));
        }
        if (world > 1 && S->m->upper) {
            S->cx_send.alloc((size_t)world * maxlen);
            S->cx_recv.alloc((size_t)maxlen);
            if (!reduce) S->cx_all.alloc((size_t)world * world * maxlen);
        }
    });
}

int hh_ice_get_bias(const hh_ice* S, double* bias, void* stream) {
    return guard([&] {
        HH_REQUIRE(S && bias, "null");
        hipStream_t s = as_stream(stream);
        S->bias.download(bias, S->n, s);
        HIP_CHECK(hipStreamSynchronize(s));
    });
}

int hh_ice_swept_bytes(const hh_ice* S, int64_t* bytes) {
    return guard([&] {
        HH_REQUIRE(S && bytes, "null");
        const hh_matrix* m = S->m;
        int64_t b = 4 * m->n_slots + 2 * m->n_slots_narrow + (int64_t)8 * (kR + 1) * m->n_tiles;
        if (S->nchu) {
            const long long W8 = m->band_w, W4 = m->band_w4;
            const long long per = (W8 > 0 ? W8 + 16 : 0) + (W4 > W8 ? band4_seg(W8, W4) : 0);
            b += (int64_t)per * (S->nloc + (m->row_lo - S->halo_lo));
        } else {
            b += (int64_t)m->band.n + (int64_t)m->band4.n;
        }
        *bytes = b;
    });
}

// Diagnostic read rates: out[2 i] = ms per pass, out[2 i + 1] =
// bytes of probe i: 0 wide tile entries, 1 narrow tile entries, 2 uint8 band,
// 3 nibble band (linear reads); 4-6 the flat tiles' payload in
// k_sweep_flatw's order, streamed only: 11 waves at its LDS footprint (one
// block per CU), 11 waves and 16 waves without it; 7-8 the same with
// coalesced run loads (11 waves one block per CU, 8 waves); 9 the narrow
// entries linearly with lane-major runs.
int hh_matrix_stream_probe(const hh_matrix* m, int32_t reps, double* out, int32_t nout) {
    return guard([&] {
        HH_REQUIRE(m && out && nout >= 20 && reps > 0, "stream probe: 20 outputs");
        for (int i = 0; i < nout; ++i) out[i] = 0.0;
        HIP_CHECK(hipSetDevice(m->device));
        hipStream_t s;
        HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        hipEvent_t e0, e1;
        HIP_CHECK(hipEventCreate(&e0));
        HIP_CHECK(hipEventCreate(&e1));
        DBuf<unsigned> sink(1);
        auto timed = [&](int i, double bytes, auto launch) {
            launch();
            HIP_CHECK(hipEventRecord(e0, s));
            for (int r = 0; r < reps; ++r) launch();
            HIP_CHECK(hipEventRecord(e1, s));
            HIP_CHECK(hipEventSynchronize(e1));
            float ms = 0.f;
            HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
            out[2 * i] = ms / reps;
            out[2 * i + 1] = bytes;
        };
        auto lin = [&](int i, const void* p, size_t bytes, bool lm = false) {
            const long long n16 = (long long)(bytes / 16);
            if (!n16) return;
            timed(i, (double)n16 * 16, [&] {
                if (lm)
                    hipLaunchKernelGGL(k_stream_probe<true>, dim3(4096), dim3(256), 0, s,
                                       reinterpret_cast<const uint4*>(p), n16, sink.p);
                else
                    hipLaunchKernelGGL(k_stream_probe<false>, dim3(4096), dim3(256), 0, s,
                                       reinterpret_cast<const uint4*>(p), n16, sink.p);
            });
        };
        lin(0, m->pay.p, m->pay.bytes());
        lin(1, m->payn.p, m->payn.bytes());
        lin(2, m->band.p, m->band.bytes());
        lin(3, m->band4.p, m->band4.bytes());
        if (m->n_fgroups) {
            const TileDev T = m->dev();
            const unsigned g = (unsigned)m->n_fgroups;
            const double fb = (double)m->payload_bytes_flat;
            timed(4, fb, [&] { hipLaunchKernelGGL((k_flat_stream_probe<11, 152000>), dim3(g), dim3(704), 0, s, T, sink.p); });
            timed(5, fb, [&] { hipLaunchKernelGGL((k_flat_stream_probe<11, 0>), dim3(g), dim3(704), 0, s, T, sink.p); });
            timed(6, fb, [&] { hipLaunchKernelGGL((k_flat_stream_probe<16, 0>), dim3(g), dim3(1024), 0, s, T, sink.p); });
            timed(7, fb, [&] {
                hipLaunchKernelGGL((k_flat_stream_probe<11, 152000, true>), dim3(g), dim3(704), 0, s, T, sink.p);
            });
            timed(8, fb, [&] { hipLaunchKernelGGL((k_flat_stream_probe<8, 0, true>), dim3(g), dim3(512), 0, s, T, sink.p); });
        }
        lin(9, m->payn.p, m->payn.bytes(), true);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipStreamSynchronize(s));
        HIP_CHECK(hipEventDestroy(e0));
        HIP_CHECK(hipEventDestroy(e1));
        HIP_CHECK(hipStreamDestroy(s));
    });
}

int hh_sweep_trace(uint64_t* out, int64_t cap, int64_t* n) {
    return guard([&] {
        HH_REQUIRE(n, "null");
        *n = g_trace_n;
        if (out && g_trace && g_trace_n) {
            HH_REQUIRE(cap >= 3 * g_trace_n, "sweep_trace: out holds 3 x blocks words");
            HIP_CHECK(hipDeviceSynchronize());
            HIP_CHECK(hipMemcpy(out, g_trace, (size_t)g_trace_n * 3 * sizeof(uint64_t), hipMemcpyDeviceToHost));
        }
    });
}

int hh_ice_finalize(hh_ice* S, double* weights, double* scale, double* var, int32_t* iters,
                    int32_t* converged, void* stream) {
    return guard([&] {
        HH_REQUIRE(S && weights, "null");
        hipStream_t s = as_stream(stream);
        const int G = S->G;
        std::vector<double> b(S->n), gm(G), gv(G);
        std::vector<int32_t> gi(G);
        std::vector<uint8_t> ge(G);
        {
            PinnedDown dl;
            dl.add(S->bias.p, b.data(), (size_t)S->n);
            dl.add(S->g_mean.p, gm.data(), (size_t)G);
            dl.add(S->g_var.p, gv.data(), (size_t)G);
            dl.add(S->g_iters.p, gi.data(), (size_t)G);
            dl.add(S->g_empty.p, ge.data(), (size_t)G);
            dl.run(s);
        }
        for (int g = 0; g < G; ++g) {
            const double sc = gm[g];
            for (int64_t i = S->glo[g]; i < S->ghi[g]; ++i) {
                if (b[i] == 0.0) b[i] = std::numeric_limits<double>::quiet_NaN();
                if (S->o.rescale_marginals) b[i] /= std::sqrt(sc);
            }
            if (scale) scale[g] = sc;
            if (var) var[g] = gv[g];
            if (iters) iters[g] = gi[g];
            if (converged) converged[g] = gv[g] < S->o.tol ? 1 : 0;
        }
        std::copy(b.begin(), b.end(), weights);
    });
}

int hh_ice_balance(hh_matrix* m, const hh_ice_opts* o, double* weights, double* scale, double* var,
                   int32_t* iters, int32_t* converged, double* sweep_seconds, void* stream) {
    hh_ice* S = nullptr;
    const auto tc0 = std::chrono::steady_clock::now();
    auto ms_since = [](std::chrono::steady_clock::time_point a) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
    };
    int rc = hh_ice_create(m, o, &S);
    if (rc) return rc;
    if (g_build_debug) fprintf(stderr, "[ice] create %.3f ms\n", ms_since(tc0));
    rc = guard([&] {
        HH_REQUIRE(S->full(), "hh_ice_balance needs a matrix holding every row");
        auto ok = [](int r) { if (r) throw Error(r, hh_last_error()); };
        const auto tf0 = std::chrono::steady_clock::now();
        ok(hh_ice_marg_local(S, 0, nullptr, stream));
        ok(hh_ice_filter_nnz(S, stream));
        ok(hh_ice_marg_local(S, 1, nullptr, stream));
        ok(hh_ice_filter_count_mad(S, stream));
        HIP_CHECK(hipStreamSynchronize(as_stream(stream)));
        if (g_build_debug) fprintf(stderr, "[ice] filters %.3f ms\n", ms_since(tf0));
        const auto t0 = std::chrono::steady_clock::now();
        while (S->iters_done < S->o.max_iters) {
            const int k = std::min(S->o.check_every, S->o.max_iters - S->iters_done);
            hipStream_t s = as_stream(stream);
            for (int j = 0; j < k; ++j) {
                marg_weighted(S, S->marg.p, s, false, 0);
                update(S, s);
            }
            int32_t na = 0;
            ok(hh_ice_active_groups(S, &na, stream));
            if (na == 0) break;
        }
        const auto t1 = std::chrono::steady_clock::now();
        if (sweep_seconds) *sweep_seconds = std::chrono::duration<double>(t1 - t0).count();
        ok(hh_ice_finalize(S, weights, scale, var, iters, converged, stream));
        if (g_build_debug) fprintf(stderr, "[ice] finalize %.3f ms\n", ms_since(t1));
    });
    const auto tx0 = std::chrono::steady_clock::now();
    hh_ice_free(S);
    if (g_build_debug) fprintf(stderr, "[ice] free %.3f ms (balance total %.3f ms)\n", ms_since(tx0), ms_since(tc0));
    return rc;
}

// --cis-only ICE over world processes without a collective in the
// iterations: each rank holds whole chromosomes as a
// compact matrix (its chromosomes' bins renumbered consecutively), whose ICE
// groups (one per chromosome) converge independently; the one exchange is an
// all-gather of the per-chromosome-normalised raw marginals for the
// genome-wide MAD cutoff (padded with zeros to max_local_bins, which the
// cutoff ignores as cooler ignores zero marginals).
int hh_ice_balance_cis_local(hh_matrix* m, const hh_ice_opts* o, int32_t world, int64_t max_local_bins,
                             hh_allgather_fn allgather, void* user, double* weights, double* scale, double* var,
                             int32_t* iters, int32_t* converged, double* sweep_seconds, void* stream) {
    hh_ice* S = nullptr;
    int rc = guard([&] {
        HH_REQUIRE(o && world >= 1 && (world == 1 || allgather), "bad arguments");
    });
    if (rc) return rc;
    rc = guard([&] {
        hipStream_t s = as_stream(stream);
        auto ok = [](int r) { if (r) throw Error(r, hh_last_error()); };
        // this rank's setup; a failure is agreed on through the all-gather
        // before the MAD exchange, so the other ranks raise instead of
        // waiting in it
        int err_rc = 0;
        std::string err;
        try {
            HH_REQUIRE(m, "null matrix");
            HH_REQUIRE(m->cis_only, "hh_ice_balance_cis_local balances cis-only matrices");
            HH_REQUIRE(max_local_bins >= m->n_bins, "max_local_bins is below this rank's bins");
            ok(hh_ice_create(m, o, &S));
            HH_REQUIRE(S->full(), "the local matrix must hold every one of its rows");
            ok(hh_ice_marg_local(S, 0, nullptr, stream));
            ok(hh_ice_filter_nnz(S, stream));
            ok(hh_ice_marg_local(S, 1, nullptr, stream));
        } catch (const Error& e) {
            err_rc = e.code;
            err = e.what();
        } catch (const std::exception& e) {
            err_rc = HH_ERR_STATE;
            err = e.what();
        }
        if (world > 1) {
            DBuf<double> sb(1), gb((size_t)world);
            const double v = err_rc ? 0.0 : 1.0;
            std::vector<double> h(world, 0.0);
            HIP_CHECK(hipMemcpyAsync(sb.p, &v, sizeof(double), hipMemcpyHostToDevice, s));
            const int r = allgather(sb.p, 1, gb.p, user, stream);
            if (r) HH_THROW(r < 0 ? r : HH_ERR_HIP, std::string("all-gather callback failed: ") + hh_last_error());
            gb.download(h.data(), world, s);
            HIP_CHECK(hipStreamSynchronize(s));
            for (int q = 0; q < world; ++q)
                if (h[q] != 1.0 && !err_rc)
                    HH_THROW(HH_ERR_STATE, "rank " + std::to_string(q) + " of " + std::to_string(world) +
                                               " failed; the cis-only run stopped on every rank");
        }
        if (err_rc) throw Error(err_rc, err);
        auto gather = [&](const std::vector<double>& loc) {
            if (world == 1) return loc;
            DBuf<double> send, recv;
            send.alloc(std::max<int64_t>(max_local_bins, 1));
            send.zero(s);
            if (!loc.empty()) send.upload(loc.data(), (int64_t)loc.size(), s);
            recv.alloc((size_t)world * std::max<int64_t>(max_local_bins, 1));
            const int r = allgather(send.p, std::max<int64_t>(max_local_bins, 1), recv.p, user, stream);
            if (r) HH_THROW(r < 0 ? r : HH_ERR_HIP, std::string("all-gather callback failed: ") + hh_last_error());
            std::vector<double> all((size_t)world * std::max<int64_t>(max_local_bins, 1));
            recv.download(all.data(), (int64_t)all.size(), s);
            HIP_CHECK(hipStreamSynchronize(s));
            return all;
        };
        filter_count_mad(S, s, gather);
        const auto t0 = std::chrono::steady_clock::now();
        while (S->iters_done < S->o.max_iters) {
            const int k = std::min(S->o.check_every, S->o.max_iters - S->iters_done);
            for (int j = 0; j < k; ++j) {
                marg_weighted(S, S->marg.p, s, false, 0);
                update(S, s);
            }
            int32_t na = 0;
            ok(hh_ice_active_groups(S, &na, stream));
            if (na == 0) break;
        }
        if (sweep_seconds)
            *sweep_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        ok(hh_ice_finalize(S, weights, scale, var, iters, converged, stream));
    });
    if (S) hh_ice_free(S);
    return rc;
}

}  // extern "C"
