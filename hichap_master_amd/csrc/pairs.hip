// pairs.hip — pair binning on the GPU: HiCHap pair text (*_Valid.bed and the
// allelic M_M / P_P / M_P / P_M / Bi_Allelic beds) -> cooler pixel tables
// (upper triangle bin1 <= bin2, sorted by (bin1, bin2), integer counts).
//
// Replaces the per-line Python loops that fill dense N x N matrices:
//   TraditionalMatrixBuilding   HiCHap/matrixBuilding.py:566-596 (+ :457-525)
//   TraditionalMatrixInAllelic  matrixBuilding.py:817-854
//   HaplotypeMatrixBuilding     matrixBuilding.py:1126-1240 (unimputed passes)
// The dense `M[b1][b2] += 1; M[b2][b1] += 1` (once on the diagonal) followed
// by np.triu + np.nonzero is the same as counting the unordered pair
// (min(b1, b2), max(b1, b2)); that is what is built here, without the dense
// matrix: parse -> key per pair -> LSD radix sort -> run-length encode.
//
// Pipeline per text chunk (device resident):
//   k_nl_count / scan / k_nl_write   newline positions (4 KB tiles, uint4 loads)
//   k_parse_bin                      one thread per line: whitespace fields
//                                    (Python str.split semantics), 'chr'
//                                    lstrip, chromosome hash lookup, int parse,
//                                    pos // res + offset, per-target keys
//                                    appended with wave-ballot compaction
// Per target at finish:
//   k_rs_hist / scan / k_rs_scatter  stable LSD radix sort, 8-bit digits, LDS
//                                    staging so each digit run is written
//                                    contiguously
//   k_rle_*                          unique pixels + counts
#include <algorithm>
#include <cstring>

#include "hh_common.hpp"

namespace hh {

constexpr int kScanThreads = 256;
constexpr int kScanItems = 16;
constexpr int kScanTile = kScanThreads * kScanItems;  // 4096
constexpr int kMaxTargets = 16;

// ------------------------------------------------------------ block scans
__device__ __forceinline__ unsigned long long wave_incl_scan_u64(unsigned long long v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        unsigned long long t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// Exclusive scan over a 256-thread block; *total = block sum.  sh >= 4 entries.
__device__ __forceinline__ unsigned long long block_excl_scan_u64(unsigned long long v, unsigned long long* sh,
                                                                   unsigned long long* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long inc = wave_incl_scan_u64(v);
    __syncthreads();
    if (lane == 63) sh[w] = inc;
    __syncthreads();
    unsigned long long base = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kScanThreads / 64; ++k) {
        if (k < w) base += sh[k];
        tot += sh[k];
    }
    if (total) *total = tot;
    return base + inc - v;
}

template <class T>
__global__ __launch_bounds__(kScanThreads) void k_scan_tile_sum(const T* __restrict__ in, long long n,
                                                                unsigned long long* __restrict__ sums) {
    __shared__ unsigned long long sh[4];
    const long long base = (long long)blockIdx.x * kScanTile;
    unsigned long long s = 0;
#pragma unroll
    for (int r = 0; r < kScanItems; ++r) {
        const long long i = base + (long long)r * kScanThreads + threadIdx.x;
        if (i < n) s += (unsigned long long)in[i];
    }
    unsigned long long tot = 0;
    (void)block_excl_scan_u64(s, sh, &tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// out[i] = tile_off[tile] + exclusive prefix within the tile (blocked layout:
// thread t owns items [t*16, t*16+16) of its tile).
template <class T, class U>
__global__ __launch_bounds__(kScanThreads) void k_scan_tile_apply(const T* __restrict__ in, long long n,
                                                                  const unsigned long long* __restrict__ tile_off,
                                                                  U* __restrict__ out) {
    __shared__ unsigned long long sh[4];
    const long long base = (long long)blockIdx.x * kScanTile + (long long)threadIdx.x * kScanItems;
    unsigned long long v[kScanItems];
    unsigned long long s = 0;
#pragma unroll
    for (int r = 0; r < kScanItems; ++r) {
        const long long i = base + r;
        v[r] = i < n ? (unsigned long long)in[i] : 0ull;
        s += v[r];
    }
    unsigned long long run = tile_off[blockIdx.x] + block_excl_scan_u64(s, sh, nullptr);
#pragma unroll
    for (int r = 0; r < kScanItems; ++r) {
        const long long i = base + r;
        if (i < n) out[i] = (U)run;
        run += v[r];
    }
}

// Single-block exclusive scan of a short array in place (n <= a few 1e5).
__global__ __launch_bounds__(kScanThreads) void k_scan_single(unsigned long long* __restrict__ a, long long n,
                                                              unsigned long long* __restrict__ total) {
    __shared__ unsigned long long sh[4];
    unsigned long long carry = 0;
    for (long long base = 0; base < n; base += kScanThreads) {
        const long long i = base + threadIdx.x;
        const unsigned long long v = i < n ? a[i] : 0ull;
        unsigned long long tot = 0;
        const unsigned long long ex = block_excl_scan_u64(v, sh, &tot);
        if (i < n) a[i] = carry + ex;
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0 && total) *total = carry;
}

static inline unsigned grid_of(long long n, long long per) { return (unsigned)((n + per - 1) / per); }

// Exclusive scan of n values (any integer type) into out (U); *total_dev
// (device, may be null) = sum.  Scratch from the pool.
template <class T, class U>
static void exclusive_scan(const T* in, U* out, long long n, unsigned long long* total_dev, hipStream_t s) {
    if (n <= 0) {
        if (total_dev) HIP_CHECK(hipMemsetAsync(total_dev, 0, sizeof(unsigned long long), s));
        return;
    }
    const long long tiles = (n + kScanTile - 1) / kScanTile;
    DBuf<unsigned long long> sums(tiles);
    hipLaunchKernelGGL((k_scan_tile_sum<T>), dim3((unsigned)tiles), dim3(kScanThreads), 0, s, in, n, sums.p);
    if (tiles <= 65536) {
        hipLaunchKernelGGL(k_scan_single, dim3(1), dim3(kScanThreads), 0, s, sums.p, tiles, total_dev);
    } else {
        DBuf<unsigned long long> tmp(tiles);
        exclusive_scan<unsigned long long, unsigned long long>(sums.p, tmp.p, tiles, total_dev, s);
        HIP_CHECK(hipMemcpyAsync(sums.p, tmp.p, tiles * sizeof(unsigned long long), hipMemcpyDeviceToDevice, s));
    }
    hipLaunchKernelGGL((k_scan_tile_apply<T, U>), dim3((unsigned)tiles), dim3(kScanThreads), 0, s, in, n, sums.p,
                       out);
    HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------ newline scan
// Text is read as aligned 16-byte blocks: a 16 B-aligned block never crosses
// a page, so the bytes around [0, nbytes) that share a block with a valid
// byte are always mapped; they are masked out.
__device__ __forceinline__ uint4 load16(const char* base, long long blk) {
    return *reinterpret_cast<const uint4*>(base + blk * 16);
}

__device__ __forceinline__ unsigned byte_of(const uint4& v, int k) {
    const unsigned w = k < 4 ? v.x : k < 8 ? v.y : k < 12 ? v.z : v.w;
    return (w >> (8 * (k & 3))) & 0xffu;
}

// Newlines in the 16 bytes [pos0 + 16*j, ...) that are inside [0, nbytes),
// relative to an aligned text start (text % 16 == 0 handled by the caller
// passing the aligned base and the byte shift).
struct TextView {
    const char* abase;   // text rounded down to 16 B
    long long shift;     // text - abase
    long long nbytes;
};

__device__ __forceinline__ int nl_mask16(const TextView& tv, long long blk, unsigned* mask) {
    const uint4 v = load16(tv.abase, blk);
    unsigned m = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const long long p = blk * 16 + k - tv.shift;  // text-relative position
        if (p >= 0 && p < tv.nbytes && byte_of(v, k) == '\n') m |= 1u << k;
    }
    *mask = m;
    return __popc(m);
}

__global__ __launch_bounds__(kScanThreads) void k_nl_count(TextView tv, long long nblk, unsigned* __restrict__ cnt) {
    __shared__ unsigned long long sh[4];
    const long long blk = (long long)blockIdx.x * kScanThreads + threadIdx.x;
    unsigned m = 0;
    const int c = blk < nblk ? nl_mask16(tv, blk, &m) : 0;
    unsigned long long tot = 0;
    (void)block_excl_scan_u64((unsigned long long)c, sh, &tot);
    if (threadIdx.x == 0) cnt[blockIdx.x] = (unsigned)tot;
}

__global__ __launch_bounds__(kScanThreads) void k_nl_write(TextView tv, long long nblk,
                                                           const unsigned long long* __restrict__ off,
                                                           long long* __restrict__ nl) {
    __shared__ unsigned long long sh[4];
    const long long blk = (long long)blockIdx.x * kScanThreads + threadIdx.x;
    unsigned m = 0;
    const int c = blk < nblk ? nl_mask16(tv, blk, &m) : 0;
    unsigned long long o = off[blockIdx.x] + block_excl_scan_u64((unsigned long long)c, sh, nullptr);
    while (m) {
        const int k = __ffs(m) - 1;
        m &= m - 1;
        nl[o++] = blk * 16 + k - tv.shift;
    }
}

// ------------------------------------------------------------ line parsing
struct NameEntry {  // open-addressing table of accepted / erroneous names
    unsigned long long hash;  // 0 = empty slot
    int32_t off, len;         // into the name bytes
    int32_t id;               // >= 0 chromosome index; -2: reference raises (KeyError)
    int32_t pad;
};

struct TargetDev {
    const long long* start;  // [2 * n_chroms] first global bin of chrom c in haplotype h
    const int32_t* nbins;    // [n_chroms] l // res + 1
    unsigned long long* keys;
    unsigned long long* count;
    long long n_bins;
    long long res;
    int local;               // intra-chromosome matrix (localRes)
    int shift;               // key = min << shift | max
};

struct ParseArgs {
    TextView tv;
    const long long* nl;     // newline positions; line k = (nl[k-1]+1 .. nl[k])
    long long n_lines;
    long long line_base;     // global index of line 0 (error reports)
    const NameEntry* table;
    const char* names;
    int table_mask;
    int unknown_policy;      // names not in the table: 0 skip, 1 raise if all digits, 2 raise
    int f_c1, f_p1, f_c2, f_p2;
    int mark_len;            // > 0: skip lines whose last field != mark
    char mark[16];
    int hap1, hap2;          // 0 maternal/traditional, 1 paternal
    int n_chroms;
    int n_targets;
    int has_whole, has_local;
    unsigned long long* err;   // [0] min (line << 8 | code)
    unsigned long long* stats; // [0] lines, [1] kept, [2] skipped (chromosome check), [3] skipped (mark)
    TargetDev t[kMaxTargets];
};

enum : int { kErrFields = 1, kErrInt = 2, kErrName = 3, kErrBin = 4 };

struct Reader {  // 16-byte register cache over the text
    const TextView* tv;
    long long blk = -1;
    uint4 v;
    __device__ unsigned get(long long p) {  // p text-relative, in range
        const long long a = p + tv->shift;
        const long long b = a >> 4;
        if (b != blk) {
            v = load16(tv->abase, b);
            blk = b;
        }
        return byte_of(v, (int)(a & 15));
    }
};

__device__ __forceinline__ bool is_ws(unsigned c) {
    return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == 11 || c == 12;
}

__device__ __forceinline__ unsigned long long fnv1a_step(unsigned long long h, unsigned c) {
    return (h ^ c) * 0x100000001B3ull;
}

// Chromosome id of field [a, b) after lstrip('chr'); -1 = skip, -2 = raise.
__device__ int lookup_chrom(const ParseArgs& A, Reader& rd, long long a, long long b, unsigned long long* hout,
                            int* lout) {
    while (a < b) {
        const unsigned c = rd.get(a);
        if (c == 'c' || c == 'h' || c == 'r') ++a; else break;
    }
    unsigned long long h = 0xcbf29ce484222325ull;
    bool digits = a < b;
    for (long long p = a; p < b; ++p) {
        const unsigned c = rd.get(p);
        h = fnv1a_step(h, c);
        digits = digits && c >= '0' && c <= '9';
    }
    if (h == 0) h = 1;
    *hout = h;
    *lout = (int)(b - a);
    const int len = (int)(b - a);
    for (int k = 0, slot = (int)(h & A.table_mask);; ++k, slot = (slot + 1) & A.table_mask) {
        const NameEntry e = A.table[slot];
        if (e.hash == 0 || k > A.table_mask) break;
        if (e.hash != h || e.len != len) continue;
        bool eq = true;
        for (int q = 0; q < len && eq; ++q) eq = (unsigned char)A.names[e.off + q] == rd.get(a + q);
        if (eq) return e.id;
    }
    if (A.unknown_policy == 2 || (A.unknown_policy == 1 && digits)) return -2;
    return -1;
}

// Python int() of an ASCII field: optional sign, then digits only.
__device__ bool parse_int(Reader& rd, long long a, long long b, long long* out) {
    bool neg = false;
    if (a < b) {
        const unsigned c = rd.get(a);
        if (c == '+' || c == '-') { neg = c == '-'; ++a; }
    }
    if (a >= b || b - a > 18) return false;
    long long v = 0;
    for (long long p = a; p < b; ++p) {
        const unsigned c = rd.get(p);
        if (c < '0' || c > '9') return false;
        v = v * 10 + (c - '0');
    }
    *out = neg ? -v : v;
    return true;
}

__global__ __launch_bounds__(kScanThreads) void k_parse_bin(ParseArgs A) {
    __shared__ unsigned wcnt[4];
    __shared__ unsigned long long bbase;
    const long long li = (long long)blockIdx.x * kScanThreads + threadIdx.x;
    const bool live = li < A.n_lines;
    int status = 0;  // 0 none, 1 kept, 2 skip(check), 3 skip(mark), 4 error
    int ecode = 0;
    int id1 = -1, id2 = -1;
    long long p1 = 0, p2 = 0;
    bool same_name = false;
    if (live) {
        Reader rd{&A.tv};
        const long long ls = li == 0 ? 0 : A.nl[li - 1] + 1;
        const long long le = A.nl[li];
        long long fa[4] = {-1, -1, -1, -1}, fb[4] = {0, 0, 0, 0};
        const int want[4] = {A.f_c1, A.f_p1, A.f_c2, A.f_p2};
        int maxf = max(max(A.f_c1, A.f_p1), max(A.f_c2, A.f_p2));
        long long la = -1, lb = -1;  // last field
        int nf = 0;
        long long p = ls;
        while (p < le) {
            while (p < le && is_ws(rd.get(p))) ++p;
            if (p >= le) break;
            const long long a = p;
            while (p < le && !is_ws(rd.get(p))) ++p;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (want[k] == nf) { fa[k] = a; fb[k] = p; }
            la = a;
            lb = p;
            ++nf;
            if (A.mark_len == 0 && nf > maxf) break;
        }
        status = 1;
        if (A.mark_len > 0) {  // `if line[-1] != 'Both': continue` (:1133)
            if (nf == 0) {
                status = 4; ecode = kErrFields;
            } else {
                bool eq = (lb - la) == A.mark_len;
                for (int q = 0; q < A.mark_len && eq; ++q) eq = rd.get(la + q) == (unsigned char)A.mark[q];
                if (!eq) status = 3;
            }
        }
        if (status == 1 && (fa[0] < 0 || fa[2] < 0)) { status = 4; ecode = kErrFields; }
        unsigned long long h1 = 0, h2 = 0;
        int l1 = 0, l2 = 0;
        if (status == 1) {
            id1 = lookup_chrom(A, rd, fa[0], fb[0], &h1, &l1);
            id2 = lookup_chrom(A, rd, fa[2], fb[2], &h2, &l2);
            if (id1 == -1 || id2 == -1) status = 2;
        }
        if (status == 1) {
            same_name = h1 == h2 && l1 == l2;  // c1 == c2 (names; id compare below for known ids)
            if (id1 >= 0 && id2 >= 0) same_name = id1 == id2;
            const bool need_local = A.has_local && same_name && A.hap1 == A.hap2;
            const bool need = A.has_whole || need_local;
            if (need && (id1 == -2 || id2 == -2)) { status = 4; ecode = kErrName; }
            else if (id1 == -2 || id2 == -2) status = 2;  // never indexed by the reference: no effect
            else if (need) {
                if (fa[1] < 0 || fa[3] < 0) { status = 4; ecode = kErrFields; }
                else if (!parse_int(rd, fa[1], fb[1], &p1) || !parse_int(rd, fa[3], fb[3], &p2) || p1 < 0 || p2 < 0) {
                    status = 4; ecode = kErrInt;
                }
            }
        }
        if (status == 4) atomicMin(A.err, (unsigned long long)(A.line_base + li) << 8 | (unsigned)ecode);
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int t = 0; t < A.n_targets; ++t) {
        const TargetDev& T = A.t[t];
        bool ok = false;
        unsigned long long key = 0;
        if (status == 1) {
            long long b1, b2;
            bool in_range;
            if (T.local) {
                ok = same_name && A.hap1 == A.hap2;
                const long long s1 = p1 / T.res, s2 = p2 / T.res;
                in_range = ok ? (s1 < T.nbins[id1] && s2 < T.nbins[id2]) : true;
                b1 = ok ? T.start[A.hap1 * A.n_chroms + id1] + s1 : 0;
                b2 = ok ? T.start[A.hap2 * A.n_chroms + id2] + s2 : 0;
            } else {
                ok = true;
                b1 = T.start[A.hap1 * A.n_chroms + id1] + p1 / T.res;
                b2 = T.start[A.hap2 * A.n_chroms + id2] + p2 / T.res;
                in_range = b1 < T.n_bins && b2 < T.n_bins;
            }
            if (!in_range) {
                atomicMin(A.err, (unsigned long long)(A.line_base + li) << 8 | (unsigned)kErrBin);
                ok = false;
            }
            if (ok) {
                const unsigned long long lo = (unsigned long long)min(b1, b2), hi = (unsigned long long)max(b1, b2);
                key = lo << T.shift | hi;
            }
        }
        const unsigned long long m = __ballot(ok);
        const unsigned rk = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) wcnt[w] = (unsigned)__popcll(m);
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned tot = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
            bbase = tot ? atomicAdd(T.count, (unsigned long long)tot) : 0ull;
        }
        __syncthreads();
        unsigned before = 0;
        for (int k = 0; k < w; ++k) before += wcnt[k];
        if (ok) T.keys[bbase + before + rk] = key;
        __syncthreads();
    }
    // line statistics (one atomic per wave and kind)
    const unsigned long long m0 = __ballot(live), m1 = __ballot(status == 1), m2 = __ballot(status == 2),
                             m3 = __ballot(status == 3);
    if (lane == 0) {
        if (m0) atomicAdd(A.stats + 0, (unsigned long long)__popcll(m0));
        if (m1) atomicAdd(A.stats + 1, (unsigned long long)__popcll(m1));
        if (m2) atomicAdd(A.stats + 2, (unsigned long long)__popcll(m2));
        if (m3) atomicAdd(A.stats + 3, (unsigned long long)__popcll(m3));
    }
}

// ------------------------------------------------------------ radix sort
__global__ __launch_bounds__(kScanThreads) void k_rs_hist(const unsigned long long* __restrict__ keys, long long n,
                                                          int shift, long long n_tiles, unsigned* __restrict__ hist) {
    __shared__ unsigned h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const long long base = (long long)blockIdx.x * kScanTile;
#pragma unroll
    for (int r = 0; r < kScanItems; ++r) {
        const long long i = base + (long long)r * kScanThreads + threadIdx.x;
        if (i < n) atomicAdd(&h[(keys[i] >> shift) & 0xff], 1u);
    }
    __syncthreads();
    hist[(long long)threadIdx.x * n_tiles + blockIdx.x] = h[threadIdx.x];
}

// Stable scatter of one 4096-key tile: local ranks from wave ballots (the 8
// digit bits matched across the wave), staged in LDS in digit order, then
// written digit run by digit run.
__global__ __launch_bounds__(kScanThreads) void k_rs_scatter(const unsigned long long* __restrict__ in,
                                                             unsigned long long* __restrict__ out, long long n,
                                                             int shift, long long n_tiles,
                                                             const unsigned* __restrict__ hist_off) {
    __shared__ unsigned long long stage[kScanTile];
    __shared__ unsigned cnt[256], start[256], run[256], gofs_lo[256];
    __shared__ unsigned wc[4][256];
    __shared__ unsigned long long sh[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const long long base = (long long)blockIdx.x * kScanTile;
    const int nvalid = (int)min((long long)kScanTile, n - base);
    cnt[tid] = 0;
    run[tid] = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) wc[k][tid] = 0;
    __syncthreads();
    unsigned long long kv[kScanItems];
#pragma unroll
    for (int r = 0; r < kScanItems; ++r) {
        const int j = r * kScanThreads + tid;
        kv[r] = j < nvalid ? in[base + j] : 0ull;
        if (j < nvalid) atomicAdd(&cnt[(kv[r] >> shift) & 0xff], 1u);
    }
    __syncthreads();
    start[tid] = (unsigned)block_excl_scan_u64(cnt[tid], sh, nullptr);
    gofs_lo[tid] = hist_off[(long long)tid * n_tiles + blockIdx.x];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kScanItems; ++r) {
        const int j = r * kScanThreads + tid;
        const bool v = j < nvalid;
        const unsigned d = (unsigned)((kv[r] >> shift) & 0xff);
        unsigned long long m = __ballot(v);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const unsigned long long bb = __ballot((d >> b) & 1u);
            m &= ((d >> b) & 1u) ? bb : ~bb;
        }
        const unsigned wr = (unsigned)__popcll(m & ((1ull << lane) - 1ull));
        if (v && lane == 63 - __clzll(m)) wc[w][d] = (unsigned)__popcll(m);
        __syncthreads();
        if (v) {
            unsigned before = run[d];
            for (int k = 0; k < w; ++k) before += wc[k][d];
            stage[start[d] + before + wr] = kv[r];
        }
        __syncthreads();
        run[tid] += wc[0][tid] + wc[1][tid] + wc[2][tid] + wc[3][tid];
        wc[0][tid] = wc[1][tid] = wc[2][tid] = wc[3][tid] = 0;
        __syncthreads();
    }
    for (int j = tid; j < nvalid; j += kScanThreads) {
        const unsigned long long key = stage[j];
        const unsigned d = (unsigned)((key >> shift) & 0xff);
        out[(long long)gofs_lo[d] + (j - (long long)start[d])] = key;
    }
}

// ------------------------------------------------------------ run-length encode
__global__ void k_rle_heads(const unsigned long long* __restrict__ keys, long long n, unsigned* __restrict__ head) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) head[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u;
}

__global__ void k_rle_write(const unsigned long long* __restrict__ keys, long long n, const unsigned* __restrict__ head,
                            const unsigned* __restrict__ idx, int shift, int32_t* __restrict__ bin1,
                            int32_t* __restrict__ bin2, unsigned* __restrict__ first) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && head[i]) {
        const unsigned u = idx[i];
        const unsigned long long k = keys[i];
        bin1[u] = (int32_t)(k >> shift);
        bin2[u] = (int32_t)(k & ((1ull << shift) - 1ull));
        first[u] = (unsigned)i;
    }
}

__global__ void k_rle_count(const unsigned* __restrict__ first, long long nu, long long n, int32_t* __restrict__ count) {
    const long long u = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (u < nu) count[u] = (int32_t)((u + 1 < nu ? (long long)first[u + 1] : n) - (long long)first[u]);
}

// ------------------------------------------------------------ synthetic pair text
// Line i of a synthetic pair file, counter-based (same text for any chunking):
// chrom1 by length, uniform pos1; cis with probability cis_frac at a
// log-uniform distance (~1/d contact decay), else a length-weighted chrom2.
struct SynthPairsDev {
    const long long* cum;     // [n_chroms + 1] cumulative lengths
    const char* names;        // printed names (with the "chr" prefix)
    const int32_t* name_off;  // [n_chroms + 1]
    int n_chroms;
    int format;               // 0: 15-column *_Valid.bed; 1: allelic "c1 p1 c2 p2 mark"
    double cis_frac;
    double log_maxd;
    unsigned long long seed;
    long long line0;
};

__device__ int pick_chrom(const SynthPairsDev& P, unsigned long long u) {
    const long long tot = P.cum[P.n_chroms];
    const long long x = (long long)(u % (unsigned long long)tot);
    int lo = 0, hi = P.n_chroms - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (P.cum[mid + 1] > x) hi = mid; else lo = mid + 1;
    }
    return lo;
}

struct SynthLine {
    int c1, c2;
    long long p1, p2;
    int both;
};

__device__ SynthLine synth_line(const SynthPairsDev& P, long long i) {
    const unsigned long long h0 = mix64(P.seed ^ mix64((unsigned long long)(P.line0 + i)));
    const unsigned long long h1 = mix64(h0 + 1), h2 = mix64(h0 + 2), h3 = mix64(h0 + 3);
    SynthLine L;
    L.c1 = pick_chrom(P, h0);
    const long long len1 = P.cum[L.c1 + 1] - P.cum[L.c1];
    L.p1 = (long long)(h1 % (unsigned long long)len1);
    if (u01(h2) < P.cis_frac) {
        L.c2 = L.c1;
        const double d = exp((double)u01(h3) * P.log_maxd);
        long long q = (h3 & 1) ? L.p1 + (long long)d : L.p1 - (long long)d;
        L.p2 = q < 0 ? 0 : (q >= len1 ? len1 - 1 : q);
    } else {
        L.c2 = pick_chrom(P, h3);
        const long long len2 = P.cum[L.c2 + 1] - P.cum[L.c2];
        L.p2 = (long long)(mix64(h3 + 7) % (unsigned long long)len2);
    }
    L.both = (h2 >> 60) != 0;  // 15 of 16 allelic lines are "Both"
    return L;
}

__device__ __forceinline__ int ndig(long long v) {
    int d = 1;
    while (v >= 10) { v /= 10; ++d; }
    return d;
}

struct Emit {
    char* out;
    long long p;
    __device__ void ch(char c) { if (out) out[p] = c; ++p; }
    __device__ void num(long long v) {
        const int d = ndig(v);
        if (out) {
            for (int k = d - 1; k >= 0; --k) { out[p + k] = (char)('0' + v % 10); v /= 10; }
        }
        p += d;
    }
    __device__ void str(const char* s, int n) {
        if (out) for (int k = 0; k < n; ++k) out[p + k] = s[k];
        p += n;
    }
};

__device__ void emit_line(const SynthPairsDev& P, long long i, Emit& e) {
    const SynthLine L = synth_line(P, i);
    const char* n1 = P.names + P.name_off[L.c1];
    const int l1 = P.name_off[L.c1 + 1] - P.name_off[L.c1];
    const char* n2 = P.names + P.name_off[L.c2];
    const int l2 = P.name_off[L.c2 + 1] - P.name_off[L.c2];
    if (P.format == 0) {
        // read-id chrom strand pos frag frag-start mid snp | chrom strand pos frag frag-start mid snp
        const long long f1 = L.p1 / 4096, f2 = L.p2 / 4096;
        e.str("SRR", 3); e.num(P.line0 + i); e.ch('\t');
        e.str(n1, l1); e.ch('\t'); e.ch('+'); e.ch('\t'); e.num(L.p1); e.ch('\t'); e.num(f1); e.ch('\t');
        e.num(f1 * 4096); e.ch('\t'); e.num(L.p1); e.ch('\t'); e.ch('0'); e.ch('\t');
        e.str(n2, l2); e.ch('\t'); e.ch('-'); e.ch('\t'); e.num(L.p2); e.ch('\t'); e.num(f2); e.ch('\t');
        e.num(f2 * 4096); e.ch('\t'); e.num(L.p2); e.ch('\t'); e.ch('0'); e.ch('\n');
    } else {
        e.str(n1, l1); e.ch('\t'); e.num(L.p1); e.ch('\t'); e.str(n2, l2); e.ch('\t'); e.num(L.p2); e.ch('\t');
        if (L.both) e.str("Both", 4); else e.str("R1", 2);
        e.ch('\n');
    }
}

__global__ void k_synth_len(SynthPairsDev P, long long n, unsigned* __restrict__ len) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Emit e{nullptr, 0};
    emit_line(P, i, e);
    len[i] = (unsigned)e.p;
}

__global__ void k_synth_write(SynthPairsDev P, long long n, const unsigned long long* __restrict__ off,
                              char* __restrict__ out) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Emit e{out, (long long)off[i]};
    emit_line(P, i, e);
}

}  // namespace hh

using namespace hh;

// ------------------------------------------------------------ host object
struct hh_binner {
    struct Target {
        int32_t res = 0, local = 0, shift = 0;
        int64_t n_bins = 0;
        DBuf<long long> start;
        DBuf<int32_t> nbins;
        DBuf<unsigned long long> keys;
        DBuf<unsigned long long> count;  // device counter
        int64_t n_keys = 0;              // host mirror after sync
        // results of finish
        bool done = false;
        int64_t nnz = 0;
        DBuf<int32_t> bin1, bin2, cnt;
    };
    int device = 0;
    int32_t n_chroms = 0;
    int32_t unknown_policy = 0;
    int32_t table_mask = 0;
    DBuf<NameEntry> table;
    DBuf<char> names;
    std::vector<Target> t;
    DBuf<unsigned long long> err;    // [1]
    DBuf<unsigned long long> stats;  // [4]
    int64_t lines_seen = 0;
    // host staging for hh_binner_feed
    PinnedBuf<char> pin[2];
    DBuf<char> dtext[2];
    hipEvent_t ev[2] = {nullptr, nullptr};
    ~hh_binner() {
        for (auto e : ev)
            if (e) (void)hipEventDestroy(e);
    }
};

namespace hh {

static unsigned long long host_fnv(const char* s, int n) {
    unsigned long long h = 0xcbf29ce484222325ull;
    for (int k = 0; k < n; ++k) h = (h ^ (unsigned char)s[k]) * 0x100000001B3ull;
    return h == 0 ? 1 : h;
}

static void ensure_keys(hh_binner::Target& T, int64_t need, hipStream_t s) {
    if ((int64_t)T.keys.n >= need) return;
    const int64_t cap = std::max<int64_t>(need, (int64_t)(T.keys.n * 3 / 2) + (1 << 20));
    DBuf<unsigned long long> nk(cap);
    if (T.n_keys)
        HIP_CHECK(hipMemcpyAsync(nk.p, T.keys.p, T.n_keys * sizeof(unsigned long long), hipMemcpyDeviceToDevice, s));
    HIP_CHECK(hipStreamSynchronize(s));
    T.keys = std::move(nk);
}

static void raise_parse_error(hh_binner* B, hipStream_t s) {
    unsigned long long e = 0;
    HIP_CHECK(hipMemcpyAsync(&e, B->err.p, sizeof(e), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (e == ~0ull) return;
    const long long line = (long long)(e >> 8);
    const int code = (int)(e & 0xff);
    const char* what = code == kErrFields ? "missing field (IndexError in the reference)"
                       : code == kErrInt  ? "position is not a non-negative integer (ValueError in the reference)"
                       : code == kErrName ? "chromosome passes the chroms filter but is not in genomeSize (KeyError in the reference)"
                                          : "bin outside the matrix (IndexError in the reference)";
    // reset so the object stays usable for inspection; the caller discards it
    HIP_CHECK(hipMemsetAsync(B->err.p, 0xff, sizeof(unsigned long long), s));
    HH_THROW(HH_ERR_ARG, "pair line " + std::to_string(line + 1) + ": " + what);
}

// Parse one device-resident text chunk that starts at a line start.
static void feed_device(hh_binner* B, const char* text, int64_t nbytes, const hh_pairs_format* f, hipStream_t s) {
    if (nbytes <= 0) return;
    TextView tv;
    tv.abase = reinterpret_cast<const char*>(reinterpret_cast<uintptr_t>(text) & ~uintptr_t(15));
    tv.shift = text - tv.abase;
    tv.nbytes = nbytes;
    const long long nblk = (tv.shift + nbytes + 15) / 16;
    const long long ntile = (nblk + kScanThreads - 1) / kScanThreads;
    DBuf<unsigned> cnt(ntile);
    DBuf<unsigned long long> off(ntile), tot(1);
    hipLaunchKernelGGL(k_nl_count, dim3((unsigned)ntile), dim3(kScanThreads), 0, s, tv, nblk, cnt.p);
    exclusive_scan<unsigned, unsigned long long>(cnt.p, off.p, ntile, tot.p, s);
    unsigned long long n_nl = 0;
    char last = 0;
    HIP_CHECK(hipMemcpyAsync(&n_nl, tot.p, sizeof(n_nl), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(&last, text + nbytes - 1, 1, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    const long long n_lines = (long long)n_nl + (last != '\n' ? 1 : 0);
    DBuf<long long> nl(n_lines);
    hipLaunchKernelGGL(k_nl_write, dim3((unsigned)ntile), dim3(kScanThreads), 0, s, tv, nblk, off.p, nl.p);
    if (last != '\n') {  // final line without a newline: it ends at nbytes
        const long long endp = nbytes;
        HIP_CHECK(hipMemcpyAsync(nl.p + n_nl, &endp, sizeof(endp), hipMemcpyHostToDevice, s));
    }
    ParseArgs A{};
    A.tv = tv;
    A.nl = nl.p;
    A.n_lines = n_lines;
    A.line_base = B->lines_seen;
    A.table = B->table.p;
    A.names = B->names.p;
    A.table_mask = B->table_mask;
    A.unknown_policy = B->unknown_policy;
    A.f_c1 = f->col_chrom1;
    A.f_p1 = f->col_pos1;
    A.f_c2 = f->col_chrom2;
    A.f_p2 = f->col_pos2;
    A.mark_len = (int)strnlen(f->mark, sizeof(f->mark));
    std::memcpy(A.mark, f->mark, sizeof(A.mark));
    A.hap1 = f->hap1;
    A.hap2 = f->hap2;
    A.n_chroms = B->n_chroms;
    A.n_targets = (int)B->t.size();
    A.err = B->err.p;
    A.stats = B->stats.p;
    for (size_t k = 0; k < B->t.size(); ++k) {
        auto& T = B->t[k];
        HH_REQUIRE(!T.done, "hh_binner_feed after hh_binner_finish");
        ensure_keys(T, T.n_keys + n_lines, s);
        A.has_whole |= T.local == 0;
        A.has_local |= T.local != 0;
        A.t[k] = TargetDev{T.start.p, T.nbins.p, T.keys.p, T.count.p, (long long)T.n_bins, (long long)T.res,
                           T.local, T.shift};
    }
    if (n_lines)
        hipLaunchKernelGGL(k_parse_bin, dim3(grid_of(n_lines, kScanThreads)), dim3(kScanThreads), 0, s, A);
    HIP_CHECK(hipGetLastError());
    B->lines_seen += n_lines;
    // key counts back to the host (sizes the next chunk's capacity check)
    std::vector<unsigned long long> c(B->t.size());
    for (size_t k = 0; k < B->t.size(); ++k)
        HIP_CHECK(hipMemcpyAsync(&c[k], B->t[k].count.p, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    for (size_t k = 0; k < B->t.size(); ++k) B->t[k].n_keys = (int64_t)c[k];
    raise_parse_error(B, s);
}

static void sort_keys(DBuf<unsigned long long>& keys, int64_t n, int bits, hipStream_t s) {
    if (n <= 1) return;
    const long long tiles = (n + kScanTile - 1) / kScanTile;
    DBuf<unsigned long long> tmp(n);
    DBuf<unsigned> hist(256 * tiles), off(256 * tiles);
    unsigned long long* a = keys.p;
    unsigned long long* b = tmp.p;
    int passes = 0;
    for (int shift = 0; shift < bits; shift += 8, ++passes) {
        hipLaunchKernelGGL(k_rs_hist, dim3((unsigned)tiles), dim3(kScanThreads), 0, s, a, (long long)n, shift,
                           tiles, hist.p);
        exclusive_scan<unsigned, unsigned>(hist.p, off.p, 256 * tiles, nullptr, s);
        hipLaunchKernelGGL(k_rs_scatter, dim3((unsigned)tiles), dim3(kScanThreads), 0, s, a, b, (long long)n, shift,
                           tiles, off.p);
        HIP_CHECK(hipGetLastError());
        std::swap(a, b);
    }
    if (passes & 1) HIP_CHECK(hipMemcpyAsync(keys.p, a, n * sizeof(unsigned long long), hipMemcpyDeviceToDevice, s));
    HIP_CHECK(hipStreamSynchronize(s));  // tmp / hist are released to the pool
}

}  // namespace hh

extern "C" {

int hh_binner_create(int32_t n_chroms, const char* names, const int32_t* name_ids, int32_t n_names,
                     int32_t unknown_policy, hh_binner** out) {
    return guard([&] {
        HH_REQUIRE(out && n_chroms >= 0 && n_names >= 0 && (n_names == 0 || (names && name_ids)), "bad arguments");
        HH_REQUIRE(unknown_policy >= 0 && unknown_policy <= 2, "unknown_policy in {0,1,2}");
        auto B = std::make_unique<hh_binner>();
        HIP_CHECK(hipGetDevice(&B->device));
        B->n_chroms = n_chroms;
        B->unknown_policy = unknown_policy;
        // names: n_names NUL-terminated strings back to back (already lstrip('chr')-ed)
        std::vector<char> bytes;
        std::vector<std::pair<int, int>> span;
        const char* p = names;
        for (int k = 0; k < n_names; ++k) {
            const int len = (int)std::strlen(p);
            span.emplace_back((int)bytes.size(), len);
            bytes.insert(bytes.end(), p, p + len);
            p += len + 1;
            HH_REQUIRE(name_ids[k] >= -2 && name_ids[k] != -1 && name_ids[k] < n_chroms,
                       "name ids must be chromosome indices or -2");
        }
        int cap = 16;
        while (cap < 4 * std::max(n_names, 1)) cap <<= 1;
        std::vector<NameEntry> tab(cap);
        for (auto& e : tab) e = NameEntry{0, 0, 0, 0, 0};
        for (int k = 0; k < n_names; ++k) {
            const unsigned long long h = host_fnv(bytes.data() + span[k].first, span[k].second);
            int slot = (int)(h & (cap - 1));
            for (;;) {
                auto& e = tab[slot];
                if (e.hash == 0) {
                    e = NameEntry{h, span[k].first, span[k].second, name_ids[k], 0};
                    break;
                }
                HH_REQUIRE(!(e.hash == h && e.len == span[k].second &&
                             std::memcmp(bytes.data() + e.off, bytes.data() + span[k].first, e.len) == 0),
                           "duplicate chromosome name");
                slot = (slot + 1) & (cap - 1);
            }
        }
        hipStream_t s = 0;
        B->table_mask = cap - 1;
        B->table = to_device(tab, s);
        bytes.push_back(0);
        B->names = to_device(bytes, s);
        B->err.alloc(1);
        HIP_CHECK(hipMemsetAsync(B->err.p, 0xff, sizeof(unsigned long long), s));
        B->stats.alloc(4);
        B->stats.zero(s);
        HIP_CHECK(hipStreamSynchronize(s));
        *out = B.release();
    });
}

int hh_binner_free(hh_binner* b) {
    return guard([&] {
        if (b) device_quiesce(b->device);
        delete b;
    });
}

int hh_binner_add_target(hh_binner* B, int32_t res, int32_t local, const int64_t* chrom_start,
                         const int32_t* chrom_nbins, int64_t n_bins, int32_t* index_out) {
    return guard([&] {
        HH_REQUIRE(B && chrom_start && chrom_nbins && index_out, "null");
        HH_REQUIRE(res > 0 && n_bins > 0 && n_bins < (int64_t(1) << 31), "res > 0 and 0 < n_bins < 2^31");
        HH_REQUIRE((int)B->t.size() < kMaxTargets, "too many targets (max 16)");
        HH_REQUIRE(B->lines_seen == 0, "targets must be added before the first feed");
        for (int c = 0; c < 2 * B->n_chroms; ++c)
            HH_REQUIRE(chrom_start[c] >= 0 && chrom_start[c] < n_bins, "chrom_start out of range");
        hh_binner::Target T;
        T.res = res;
        T.local = local ? 1 : 0;
        T.n_bins = n_bins;
        int sh = 1;
        while ((int64_t(1) << sh) < n_bins) ++sh;
        T.shift = sh;
        hipStream_t s = 0;
        std::vector<long long> st(chrom_start, chrom_start + 2 * B->n_chroms);
        std::vector<int32_t> nb(chrom_nbins, chrom_nbins + B->n_chroms);
        if (st.empty()) st.push_back(0);
        if (nb.empty()) nb.push_back(0);
        T.start = to_device(st, s);
        T.nbins = to_device(nb, s);
        T.count.alloc(1);
        T.count.zero(s);
        HIP_CHECK(hipStreamSynchronize(s));
        *index_out = (int32_t)B->t.size();
        B->t.push_back(std::move(T));
    });
}

int hh_binner_feed_device(hh_binner* B, const char* text, int64_t nbytes, const hh_pairs_format* f, void* stream) {
    return guard([&] {
        HH_REQUIRE(B && f && (text || nbytes == 0) && nbytes >= 0, "bad arguments");
        HIP_CHECK(hipSetDevice(B->device));
        feed_device(B, text, nbytes, f, as_stream(stream));
    });
}

int hh_binner_feed(hh_binner* B, const char* text, int64_t nbytes, const hh_pairs_format* f, int64_t chunk_bytes,
                   void* stream) {
    return guard([&] {
        HH_REQUIRE(B && f && (text || nbytes == 0) && nbytes >= 0, "bad arguments");
        HIP_CHECK(hipSetDevice(B->device));
        hipStream_t s = as_stream(stream);
        if (chunk_bytes <= 0) chunk_bytes = int64_t(256) << 20;
        chunk_bytes = std::max<int64_t>(chunk_bytes, 4096);
        int64_t pos = 0;
        int k = 0;
        while (pos < nbytes) {
            int64_t len = std::min<int64_t>(chunk_bytes, nbytes - pos);
            if (pos + len < nbytes) {  // cut after the last newline of the window
                const char* q = static_cast<const char*>(memrchr(text + pos, '\n', (size_t)len));
                if (!q) {                // one line longer than the window: take it whole
                    const char* r = static_cast<const char*>(memchr(text + pos + len, '\n', (size_t)(nbytes - pos - len)));
                    len = r ? (r - (text + pos)) + 1 : nbytes - pos;
                } else {
                    len = (q - (text + pos)) + 1;
                }
            }
            const int slot = k & 1;
            if (B->ev[slot]) HIP_CHECK(hipEventSynchronize(B->ev[slot]));
            else HIP_CHECK(hipEventCreateWithFlags(&B->ev[slot], hipEventDisableTiming));
            if ((int64_t)B->pin[slot].n < len) B->pin[slot].alloc((size_t)std::max<int64_t>(len, chunk_bytes));
            if ((int64_t)B->dtext[slot].n < len) B->dtext[slot].alloc((size_t)std::max<int64_t>(len, chunk_bytes));
            std::memcpy(B->pin[slot].p, text + pos, (size_t)len);
            HIP_CHECK(hipMemcpyAsync(B->dtext[slot].p, B->pin[slot].p, (size_t)len, hipMemcpyHostToDevice, s));
            feed_device(B, B->dtext[slot].p, len, f, s);
            HIP_CHECK(hipEventRecord(B->ev[slot], s));
            pos += len;
            ++k;
        }
    });
}

int hh_binner_stats(const hh_binner* B, int64_t* stats4) {
    return guard([&] {
        HH_REQUIRE(B && stats4, "null");
        unsigned long long v[4];
        HIP_CHECK(hipMemcpy(v, B->stats.p, sizeof(v), hipMemcpyDeviceToHost));
        for (int k = 0; k < 4; ++k) stats4[k] = (int64_t)v[k];
    });
}

int hh_binner_finish(hh_binner* B, void* stream) {
    return guard([&] {
        HH_REQUIRE(B, "null");
        HIP_CHECK(hipSetDevice(B->device));
        hipStream_t s = as_stream(stream);
        for (auto& T : B->t) {
            if (T.done) continue;
            const int64_t n = T.n_keys;
            HH_REQUIRE(n < (int64_t(1) << 32) - 1, "more than 2^32 pairs in one matrix");
            {
                HH_KTIME("k_rs_sort", s);
                sort_keys(T.keys, n, 2 * T.shift, s);
            }
            DBuf<unsigned> head(std::max<int64_t>(n, 1)), idx(std::max<int64_t>(n, 1));
            DBuf<unsigned long long> tot(1);
            unsigned long long nu = 0;
            if (n) {
                hipLaunchKernelGGL(k_rle_heads, dim3(grid_of(n, 256)), dim3(256), 0, s, T.keys.p, (long long)n, head.p);
                exclusive_scan<unsigned, unsigned>(head.p, idx.p, n, tot.p, s);
                HIP_CHECK(hipMemcpyAsync(&nu, tot.p, sizeof(nu), hipMemcpyDeviceToHost, s));
                HIP_CHECK(hipStreamSynchronize(s));
            }
            T.nnz = (int64_t)nu;
            T.bin1.alloc(std::max<int64_t>(T.nnz, 1));
            T.bin2.alloc(std::max<int64_t>(T.nnz, 1));
            T.cnt.alloc(std::max<int64_t>(T.nnz, 1));
            if (n) {
                DBuf<unsigned> first(std::max<int64_t>(T.nnz, 1));
                hipLaunchKernelGGL(k_rle_write, dim3(grid_of(n, 256)), dim3(256), 0, s, T.keys.p, (long long)n, head.p,
                                   idx.p, T.shift, T.bin1.p, T.bin2.p, first.p);
                hipLaunchKernelGGL(k_rle_count, dim3(grid_of(T.nnz, 256)), dim3(256), 0, s, first.p,
                                   (long long)T.nnz, (long long)n, T.cnt.p);
                HIP_CHECK(hipGetLastError());
                HIP_CHECK(hipStreamSynchronize(s));
            }
            T.keys.release();
            T.done = true;
        }
    });
}

int hh_binner_target_nnz(const hh_binner* B, int32_t target, int64_t* nnz, int64_t* n_pairs) {
    return guard([&] {
        HH_REQUIRE(B && target >= 0 && target < (int)B->t.size(), "bad target");
        const auto& T = B->t[target];
        if (nnz) *nnz = T.done ? T.nnz : -1;
        if (n_pairs) *n_pairs = T.n_keys;
    });
}

int hh_binner_pixels_device(const hh_binner* B, int32_t target, const int32_t** bin1, const int32_t** bin2,
                            const int32_t** count) {
    return guard([&] {
        HH_REQUIRE(B && target >= 0 && target < (int)B->t.size(), "bad target");
        const auto& T = B->t[target];
        HH_REQUIRE(T.done, "call hh_binner_finish first");
        if (bin1) *bin1 = T.bin1.p;
        if (bin2) *bin2 = T.bin2.p;
        if (count) *count = T.cnt.p;
    });
}

int hh_binner_download(const hh_binner* B, int32_t target, int32_t* bin1, int32_t* bin2, int32_t* count) {
    return guard([&] {
        HH_REQUIRE(B && target >= 0 && target < (int)B->t.size(), "bad target");
        const auto& T = B->t[target];
        HH_REQUIRE(T.done, "call hh_binner_finish first");
        hipStream_t s = 0;
        if (bin1) T.bin1.download(bin1, T.nnz, s);
        if (bin2) T.bin2.download(bin2, T.nnz, s);
        if (count) T.cnt.download(count, T.nnz, s);
        HIP_CHECK(hipStreamSynchronize(s));
    });
}

int hh_synth_pairs_text(int32_t n_chroms, const char* names, const int64_t* lengths, int64_t n_lines,
                        double cis_frac, double max_dist, int32_t format, uint64_t seed, int64_t line0, char* out,
                        int64_t capacity, int64_t* nbytes, void* stream) {
    return guard([&] {
        HH_REQUIRE(n_chroms > 0 && names && lengths && nbytes && n_lines >= 0, "bad arguments");
        HH_REQUIRE(format == 0 || format == 1, "format 0 (Valid.bed) or 1 (allelic)");
        hipStream_t s = as_stream(stream);
        std::vector<long long> cum(n_chroms + 1, 0);
        std::vector<int32_t> noff(n_chroms + 1, 0);
        std::vector<char> nb;
        const char* p = names;
        for (int c = 0; c < n_chroms; ++c) {
            HH_REQUIRE(lengths[c] > 0, "chromosome lengths must be positive");
            cum[c + 1] = cum[c] + lengths[c];
            const int len = (int)std::strlen(p);
            nb.insert(nb.end(), p, p + len);
            noff[c + 1] = noff[c] + len;
            p += len + 1;
        }
        nb.push_back(0);
        DBuf<long long> dcum = to_device(cum, s);
        DBuf<char> dn = to_device(nb, s);
        DBuf<int32_t> doff = to_device(noff, s);
        SynthPairsDev P{dcum.p, dn.p, doff.p, n_chroms, format, cis_frac, std::log(std::max(max_dist, 1.0)), seed, line0};
        DBuf<unsigned> len(std::max<int64_t>(n_lines, 1));
        DBuf<unsigned long long> off(std::max<int64_t>(n_lines, 1)), tot(1);
        if (n_lines) {
            hipLaunchKernelGGL(k_synth_len, dim3(grid_of(n_lines, 256)), dim3(256), 0, s, P, (long long)n_lines, len.p);
            exclusive_scan<unsigned, unsigned long long>(len.p, off.p, n_lines, tot.p, s);
        }
        unsigned long long total = 0;
        if (n_lines) HIP_CHECK(hipMemcpyAsync(&total, tot.p, sizeof(total), hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        *nbytes = (int64_t)total;
        if (!out) return;  // size query
        HH_REQUIRE(capacity >= (int64_t)total, "output buffer too small");
        if (n_lines)
            hipLaunchKernelGGL(k_synth_write, dim3(grid_of(n_lines, 256)), dim3(256), 0, s, P, (long long)n_lines,
                               off.p, out);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipStreamSynchronize(s));
    });
}

}  // extern "C"
