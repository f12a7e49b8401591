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
//   k_parse_tile   one block per 8 KB of text: the tile (+4 KB lookahead)
//                  staged in LDS with coalesced 16 B loads, line starts found
//                  in LDS (block scan), then one thread per line: whitespace
//                  fields (Python str.split semantics), 'chr' lstrip,
//                  chromosome hash lookup, int parse, pos // res + offset,
//                  per-target keys appended with wave-ballot compaction
// Per target at finish:
//   k_rs_hist / scan / k_rs_scatter  stable LSD radix sort, 8-bit digits, LDS
//                                    staging so each digit run is written
//                                    contiguously
//   k_rle_*                          unique pixels + counts
#include <algorithm>
#include <cmath>
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
    // every load unconditional (an `if (i < n)` load compiled to one round
    // trip each): indices past n re-read in[n - 1], subtracted once at the end
    unsigned long long s = 0, over = 0;
    T xs[kScanItems];
#pragma unroll
    for (int r = 0; r < kScanItems; ++r) {
        const long long i = base + (long long)r * kScanThreads + threadIdx.x;
        xs[r] = in[i < n ? i : n - 1];
        over += i >= n;
    }
#pragma unroll
    for (int r = 0; r < kScanItems; ++r) s += (unsigned long long)xs[r];
    s -= over * (unsigned long long)in[n - 1];
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
    unsigned long long s = 0, over = 0;
    // unconditional loads as in k_scan_tile_sum; a thread's items past n
    // follow its valid ones, so only its total needs the correction
#pragma unroll
    for (int r = 0; r < kScanItems; ++r) {
        const long long i = base + r;
        v[r] = (unsigned long long)in[i < n ? i : n - 1];
        s += v[r];
        over += i >= n;
    }
    s -= over * (unsigned long long)in[n - 1];
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

// ------------------------------------------------------------ text access
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

struct TextView {
    const char* abase;   // text rounded down to 16 B
    long long shift;     // text - abase
    long long nbytes;
};

// ------------------------------------------------------------ line parsing
// Chromosome name table: open addressing on a 32-bit hash of the name's
// first 16 bytes (inline, zero padded) and its length.
struct NameEntry {
    uint32_t w[4];   // first 16 bytes of the name (little-endian words)
    int32_t len;
    int32_t id;      // >= 0 chromosome index; -2 reference raises (KeyError); -3 empty slot
    int32_t off;     // all name bytes in `names` (compared past byte 16)
    uint32_t hash;
};
constexpr int kEmptySlot = -3;

__host__ __device__ __forceinline__ uint32_t name_hash(const uint32_t w[4], int len) {
    uint32_t h = 0x9E3779B9u ^ (uint32_t)len;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        h ^= w[k] * 0x85EBCA6Bu;
        h = ((h << 13) | (h >> 19)) * 5u + 0xE6546B64u;
    }
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    return h;
}

struct TargetDev {
    const long long* start;  // [2 * n_chroms] first global bin of chrom c in haplotype h
    const int32_t* nbins;    // [n_chroms] l // res + 1
    unsigned long long* keys;
    unsigned long long* count;  // slots reserved (keys + sentinels)
    unsigned long long* gaps;   // sentinel slots
    long long n_bins;
    long long res;
    int local;               // intra-chromosome matrix (localRes)
    int shift;               // key = min << shift | max (ordered: row << shift | col)
    unsigned magic;          // division by res (div_res)
    int msh;
    // imputation targets (mode 1; HaplotypeMatrixBuilding :1251-1494)
    int ordered;             // keys keep (row, col) as incremented (asymmetric matrix)
    int imp_s;               // L = Imputation_region // res
    const long long* rowpref;  // unimputed whole matrix, per-row prefix sums, n_bins x (n_bins + 1)
    const int* disc_j0;      // disc row i of the (2L+1)^2 window covers columns [j0, j1]
    const int* disc_j1;
    long long imin;
    double ratio;
    long long pp_sum;        // the P pass's stale M_M_sub neighbourhood sum (:1445)
    int pp_ok;
};

struct ParseArgs {
    TextView tv;
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
    int mode;                  // 0 binning, 1 imputation (single-allele lines)
    int mark2_len;             // imputation: last field == mark2 ('R1') selects the R1 branch
    char mark2[16];
    unsigned long long byte_base;  // bytes fed before this chunk (line order across chunks)
    unsigned long long* lastq;     // max (global line-start byte + 1) << 8 | target of M-pass lines
                                   // that reached the neighbourhood step (the stale M_M_sub)
    int ablate;                // g_parse_ablate (timing only)
    unsigned long long* err;   // [0] min (line start byte << 8 | code)
    unsigned long long* stats; // [0] lines, [1] kept, [2] skipped (chromosome check), [3] skipped (mark)
    TargetDev t[kMaxTargets];
};

enum : int { kErrFields = 1, kErrInt = 2, kErrName = 3, kErrBin = 4, kErrStale = 5 };

// Tile geometry of k_parse_tile: a block owns the lines that START in its
// tile of aligned 16 B text blocks ([T0, T0 + TB), TB = 256..2560 blocks,
// picked per feed so a tile holds ~230 lines); it stages the tile, the block
// before it and 1 KB of lookahead (lines running further fall back to global
// loads) in LDS with coalesced 16 B loads, plus each staged block's
// whitespace / newline bitmasks.
constexpr int kPLookBlk = 64;   // 1 KB
constexpr int kPMaxSeg = 10;    // blocks per thread segment (TB <= 2560 = 40 KB)

// Exact per-byte classes of one little-endian word, as 4-bit masks.
__device__ __forceinline__ unsigned zero_bytes_hi(unsigned y) {  // 0x80 in each zero byte
    return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y | 0x7F7F7F7Fu);
}
__device__ __forceinline__ unsigned hi_to_nibble(unsigned h) { return (((h >> 7) * 0x204081u) >> 21) & 0xFu; }

__device__ __forceinline__ void word_classes(unsigned x, unsigned* ws, unsigned* nl) {
    const unsigned n = zero_bytes_hi(x ^ 0x0A0A0A0Au);
    const unsigned sp = zero_bytes_hi(x ^ 0x20202020u);
    // bytes 9..13 (\t \n \v \f \r): (c | 0x80) - 9 has no inter-byte borrow
    const unsigned r = (x | 0x80808080u) - 0x09090909u;
    const unsigned lt5 = ~((r & 0x7F7F7F7Fu) + 0x7B7B7B7Bu) & 0x80808080u;
    const unsigned rng = r & lt5 & ~x & 0x80808080u;
    *ws = hi_to_nibble(sp | rng);
    *nl = hi_to_nibble(n);
}

// Global 16-byte load for the rare out-of-window path.  Written as asm so the
// compiler cannot merge it with the LDS path into one flat load (a flat load
// waits on both the vector-memory and the LDS counters, serialising every LDS
// read of the parse behind outstanding global traffic).
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 load16_global_sync(const char* p) {
    u32x4_t v;
    asm volatile("global_load_dwordx4 %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return make_uint4(v.x, v.y, v.z, v.w);
}

struct TileText {
    const uint4* lds;      // text blocks [W0, W1)
    const unsigned* msk;   // their masks: ws | nl << 16
    long long W0, W1;
    const TextView* tv;
    long long nblk_all;    // aligned blocks holding text bytes
    __device__ uint4 blk(long long b) const {
        if (b >= W0 && b < W1) return lds[b - W0];
        if (b < 0 || b >= nblk_all) return make_uint4(0, 0, 0, 0);
        return load16_global_sync(tv->abase + b * 16);
    }
    __device__ unsigned get(long long p) const {  // text-relative byte; past the end reads '\n'
        if (p >= tv->nbytes) return '\n';
        const long long a = p + tv->shift;
        return byte_of(blk(a >> 4), (int)(a & 15));
    }
};

// ws | nl << 16 of aligned block b from its bytes; bytes past the end of the
// text count as newline (and whitespace).
__device__ __forceinline__ unsigned masks_of(const TextView& tv, uint4 v, long long b) {
    unsigned w0, w1, w2, w3, n0, n1, n2, n3;
    word_classes(v.x, &w0, &n0);
    word_classes(v.y, &w1, &n1);
    word_classes(v.z, &w2, &n2);
    word_classes(v.w, &w3, &n3);
    unsigned ws = w0 | w1 << 4 | w2 << 8 | w3 << 12;
    unsigned nl = n0 | n1 << 4 | n2 << 8 | n3 << 12;
    const long long lim = tv.shift + tv.nbytes - b * 16;  // valid bytes in this block
    if (lim < 16) {
        const unsigned past = lim <= 0 ? 0xffffu : (0xffffu << lim) & 0xffffu;
        ws |= past;
        nl |= past;
    }
    return ws | nl << 16;
}

__device__ __forceinline__ unsigned block_mask(const TileText& T, long long b) {
    if (b >= T.W0 && b < T.W1) return T.msk[b - T.W0];
    return masks_of(*T.tv, T.blk(b), b);
}

// 16 text bytes starting at p (little-endian words).
__device__ __forceinline__ void window16(const TileText& T, long long p, unsigned out[4]) {
    const long long a = p + T.tv->shift;
    const long long b = a >> 4;
    const int o = (int)(a & 15);
    const uint4 v0 = T.blk(b);
    const uint4 v1 = o ? T.blk(b + 1) : make_uint4(0, 0, 0, 0);
    const unsigned x[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    const int ow = o >> 2, ob = o & 3;
    unsigned y[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const unsigned a0 = x[k], a1 = x[k + 1], a2 = x[k + 2];
        const unsigned a3 = k + 3 < 8 ? x[k + 3] : 0u;
        y[k] = ow == 0 ? a0 : ow == 1 ? a1 : ow == 2 ? a2 : a3;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) out[k] = ob ? __builtin_amdgcn_alignbyte(y[k + 1], y[k], ob) : y[k];
}

__device__ __forceinline__ unsigned wbyte(const unsigned w[4], int k) { return (w[k >> 2] >> (8 * (k & 3))) & 0xffu; }

// Chromosome id of field [a, b) after lstrip('chr'); -1 = skip, -2 = raise.
__device__ int lookup_chrom(const ParseArgs& A, const TileText& T, long long a, long long b, int* key_len,
                            uint32_t* key_hash) {
    unsigned w[4];
    // lstrip('chr'): leading 'c' / 'h' / 'r' bytes, 16 at a time
    for (;;) {
        const long long L = b - a;
        if (L <= 0) break;
        window16(T, a, w);
        unsigned m = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const unsigned x = w[q];
            m |= hi_to_nibble(zero_bytes_hi(x ^ 0x63636363u) | zero_bytes_hi(x ^ 0x68686868u) |
                              zero_bytes_hi(x ^ 0x72727272u)) << (4 * q);
        }
        int k = __ffs(~m & 0x1ffffu) - 1;  // leading stripped bytes (<= 16)
        if (k > L) k = (int)L;
        a += k;
        if (k < 16) break;
    }
    const int len = (int)(b - a);
    window16(T, a, w);
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // zero the bytes past the name
        const int keep = len - 4 * q;
        w[q] = keep >= 4 ? w[q] : keep <= 0 ? 0u : (w[q] & ((1u << (8 * keep)) - 1u));
    }
    const uint32_t h = name_hash(w, len);
    *key_len = len;
    *key_hash = h;
    for (int k = 0, slot = (int)(h & A.table_mask); k <= A.table_mask; ++k, slot = (slot + 1) & A.table_mask) {
        const NameEntry& e = A.table[slot];
        const int id = e.id;
        if (id == kEmptySlot) break;
        if (e.hash != h || e.len != len || e.w[0] != w[0] || e.w[1] != w[1] || e.w[2] != w[2] || e.w[3] != w[3])
            continue;
        bool eq = true;
        for (int q = 16; q < len && eq; ++q) eq = (unsigned char)A.names[e.off + q] == T.get(a + q);
        if (eq) return id;
    }
    bool digits = len > 0;
    for (long long p = a; p < b && digits; ++p) {
        const unsigned c = T.get(p);
        digits = c >= '0' && c <= '9';
    }
    if (A.unknown_policy == 2 || (A.unknown_policy == 1 && digits)) return -2;
    return -1;
}

// Python int() of an ASCII field: optional sign, then 1..18 digits.
// Digits are validated with SWAR byte classes on a 16-byte window and
// accumulated by Horner steps in 32-bit (<= 9 digits; 64-bit beyond).
__device__ bool parse_int(const TileText& T, long long a, long long b, long long* out) {
    bool neg = false;
    if (a < b) {
        const unsigned c = T.get(a);
        if (c == '+' || c == '-') { neg = c == '-'; ++a; }
    }
    const long long L = b - a;
    if (L <= 0 || L > 18) return false;
    long long v = 0;
    if (L <= 16) {
        unsigned w[4];
        window16(T, a, w);
        const int n = (int)L;
        unsigned dm = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const unsigned x = w[q];
            const unsigned r = (x | 0x80808080u) - 0x30303030u;
            const unsigned lt10 = ~((r & 0x7F7F7F7Fu) + 0x76767676u) & 0x80808080u;
            dm |= hi_to_nibble(r & lt10 & ~x & 0x80808080u) << (4 * q);
        }
        const unsigned need = n >= 16 ? 0xFFFFu : ((1u << n) - 1u);
        if ((dm & need) != need) return false;
        unsigned lo = 0;
#pragma unroll
        for (int k = 0; k < 9; ++k)
            if (k < n) lo = (lo << 3) + (lo << 1) + (wbyte(w, k) - '0');
        v = lo;
        for (int k = 9; k < n; ++k) v = v * 10 + (long long)(wbyte(w, k) - '0');
    } else {
        for (long long p = a; p < b; ++p) {
            const unsigned c = T.get(p);
            if (c < '0' || c > '9') return false;
            v = v * 10 + (c - '0');
        }
    }
    *out = neg ? -v : v;
    return true;
}

// Position of the k-th (0-based) set bit of a 16-bit mask (branch-free).
__device__ __forceinline__ int kth_bit(unsigned m, int k) {
    int pos = 0;
    int c = __popc(m & 0xffu);
    bool g = k >= c;
    k -= g ? c : 0; m = g ? m >> 8 : m; pos += g ? 8 : 0;
    c = __popc(m & 0xfu);
    g = k >= c;
    k -= g ? c : 0; m = g ? m >> 4 : m; pos += g ? 4 : 0;
    c = __popc(m & 0x3u);
    g = k >= c;
    k -= g ? c : 0; m = g ? m >> 2 : m; pos += g ? 2 : 0;
    g = k >= (int)(m & 1u);
    return pos + (g ? 1 : 0);
}

struct LineOut {
    int status;  // 0 none, 1 kept, 2 skip(check), 3 skip(mark), 4 error
    int ecode;
    int id1, id2;
    long long p1, p2;
    bool same_name;
    bool r1;     // imputation: last field == mark2
};

// Field boundaries of the line starting at text position ls from the
// blocks' whitespace masks (Python `line.strip().split()`), then the
// reference's filters and int() parses.
__device__ LineOut parse_line(const ParseArgs& A, const TileText& T, long long ls) {
    LineOut o{1, 0, -1, -1, 0, 0, false, false};
    long long fa[4] = {-1, -1, -1, -1}, fb[4] = {0, 0, 0, 0};
    const int want[4] = {A.f_c1, A.f_p1, A.f_c2, A.f_p2};
    const int maxf = max(max(A.f_c1, A.f_p1), max(A.f_c2, A.f_p2));
    // One uniform pass over the line's blocks records, for each wanted field,
    // the block (its base position and start / end mask) holding its start
    // and its end; positions are resolved afterwards with kth_bit.  Lanes
    // stay converged (no per-field branches inside the block loop).
    long long sbase[4], ebase[4];
    unsigned smask[4], emask[4];
    int sk[4], ek[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) { sbase[q] = ebase[q] = 0; smask[q] = emask[q] = 0; sk[q] = ek[q] = -1; }
    long long lsb = 0, leb = 0;  // last start / end block (mark mode)
    unsigned lsm = 0, lem = 0;
    int nf = 0;  // fields started
    bool infield = false, done = false;
    const long long a0 = ls + T.tv->shift;
    long long b = a0 >> 4;
    unsigned pre = (1u << (a0 & 15)) - 1u;  // bytes of the first block before the line
    while (!done) {
        const unsigned mk = block_mask(T, b);
        const unsigned ws = (mk & 0xffffu) | pre;
        const unsigned nl = (mk >> 16) & ~pre;
        pre = 0;
        const int endk = nl ? __ffs(nl) - 1 : 16;                 // the line's '\n' (or 16)
        const unsigned live = endk == 16 ? 0xffffu : ((1u << endk) - 1u);
        const unsigned nonws = ~ws & live;
        const unsigned prev = ((nonws << 1) | (infield ? 1u : 0u)) & 0x1ffffu;
        const unsigned st = nonws & ~prev;
        const unsigned en = ~nonws & prev & (endk == 16 ? 0xffffu : ((2u << endk) - 1u));
        const long long pos0 = b * 16 - T.tv->shift;
        const int ns = __popc(st), ne = __popc(en);
        const int e0 = infield ? nf - 1 : nf;  // field index of this block's first end
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int js = want[q] - nf, je = want[q] - e0;
            const bool hs = js >= 0 && js < ns, he = je >= 0 && je < ne;
            sbase[q] = hs ? pos0 : sbase[q];
            smask[q] = hs ? st : smask[q];
            sk[q] = hs ? js : sk[q];
            ebase[q] = he ? pos0 : ebase[q];
            emask[q] = he ? en : emask[q];
            ek[q] = he ? je : ek[q];
        }
        lsb = st ? pos0 : lsb;
        lsm = st ? st : lsm;
        leb = en ? pos0 : leb;
        lem = en ? en : lem;
        nf += ns;
        infield = (nonws >> 15) & 1u;
        done = endk < 16 || (A.mark_len == 0 && nf - (infield ? 1 : 0) > maxf);
        ++b;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (sk[q] >= 0 && ek[q] >= 0) {
            fa[q] = sbase[q] + kth_bit(smask[q], sk[q]);
            fb[q] = ebase[q] + kth_bit(emask[q], ek[q]);
        }
    }
    long long la = -1, lb = -1;
    if (nf > 0) {
        la = lsb + 31 - __clz(lsm);
        lb = leb + 31 - __clz(lem);
    }
    if (A.mark_len > 0) {  // `if line[-1] != 'Both': continue` (:1133); imputation: `== 'Both'` (:1273)
        if (nf == 0) {
            o.status = 4; o.ecode = kErrFields;
            return o;
        }
        bool eq = (lb - la) == A.mark_len;
        for (int q = 0; q < A.mark_len && eq; ++q) eq = T.get(la + q) == (unsigned char)A.mark[q];
        if (eq == (A.mode == 1)) { o.status = 3; return o; }
        if (A.mode == 1) {
            bool e2 = (lb - la) == A.mark2_len;
            for (int q = 0; q < A.mark2_len && e2; ++q) e2 = T.get(la + q) == (unsigned char)A.mark2[q];
            o.r1 = e2;
        }
    }
    if (fa[0] < 0 || fa[2] < 0) { o.status = 4; o.ecode = kErrFields; return o; }
    int l1 = 0, l2 = 0;
    uint32_t h1 = 0, h2 = 0;
    o.id1 = lookup_chrom(A, T, fa[0], fb[0], &l1, &h1);
    o.id2 = lookup_chrom(A, T, fa[2], fb[2], &l2, &h2);
    if (o.id1 == -1 || o.id2 == -1) { o.status = 2; return o; }
    if (o.id1 >= 0 && o.id2 >= 0) {
        o.same_name = o.id1 == o.id2;
    } else {  // an unknown name: compare the stripped names byte by byte
        bool eq = l1 == l2 && h1 == h2;
        const long long s1 = fb[0] - l1, s2 = fb[2] - l2;
        for (int q = 0; q < l1 && eq; ++q) eq = T.get(s1 + q) == T.get(s2 + q);
        o.same_name = eq;
    }
    const bool need_local = A.has_local && o.same_name && A.hap1 == A.hap2;
    const bool need = A.has_whole || need_local;
    if (o.id1 == -2 || o.id2 == -2) {
        if (need) { o.status = 4; o.ecode = kErrName; }
        else o.status = 2;  // never indexed by the reference: no effect
        return o;
    }
    if (need) {
        if (fa[1] < 0 || fa[3] < 0) { o.status = 4; o.ecode = kErrFields; }
        else if (!parse_int(T, fa[1], fb[1], &o.p1) || !parse_int(T, fa[3], fb[3], &o.p2) || o.p1 < 0 || o.p2 < 0) {
            o.status = 4; o.ecode = kErrInt;
        }
    }
    return o;
}

// p // res with the target's round-up multiplier (Granlund-Montgomery:
// l = ceil(log2 res), magic = floor(2^32 (2^l - res) / res) + 1; exact for
// every 32-bit p; res == 1 -> msh = -1).
__device__ __forceinline__ long long div_res(long long p, const TargetDev& T) {
    if ((unsigned long long)p >= 0x100000000ull) return p / T.res;
    const unsigned n = (unsigned)p;
    if (T.msh < 0) return n;
    const unsigned t = __umulhi(T.magic, n);
    return (long long)((t + ((n - t) >> 1)) >> T.msh);
}

// Neighbourhood sum of the unimputed whole matrix over GetNeighborhoodIndex's
// disc (:721-738) in the window with top-left (r0, c0): per disc row, one
// difference of row prefix sums.
__device__ long long disc_sum(const TargetDev& T, long long r0, long long c0) {
    long long sum = 0;
    const long long w = T.n_bins + 1;
    for (int i = 0; i <= 2 * T.imp_s; ++i) {
        const int j0 = T.disc_j0[i], j1 = T.disc_j1[i];
        if (j1 < j0) continue;
        const long long* P = T.rowpref + (r0 + i) * w;
        sum += P[c0 + j1 + 1] - P[c0 + j0];
    }
    return sum;
}

// Imputation of one single-allele line into one target (:1270-1490): sets
// *ok / *key (ordered cell); *reached = the line got to the neighbourhood
// step (it rebinds M_M_sub in the M pass); returns an error code or 0.
__device__ int impute_key(const ParseArgs& A, const TargetDev& T, const LineOut& L, bool* ok,
                          unsigned long long* key, bool* reached) {
    *ok = false;
    *reached = false;
    const int n = A.n_chroms, hap = A.hap1;
    const long long q1 = div_res(L.p1, T), q2 = div_res(L.p2, T);
    long long row, col;
    if (L.same_name) {  // intra-chromosome: ordered count, R1 (bin1, bin2) else (bin2, bin1)
        if (T.local) {
            if (q1 >= T.nbins[L.id1] || q2 >= T.nbins[L.id2]) return kErrBin;
            const long long base = T.start[hap * n + L.id1];
            row = base + (L.r1 ? q1 : q2);
            col = base + (L.r1 ? q2 : q1);
        } else {
            const long long b1 = T.start[hap * n + L.id1] + q1, b2 = T.start[hap * n + L.id2] + q2;
            if (b1 >= T.n_bins || b2 >= T.n_bins) return kErrBin;
            row = L.r1 ? b1 : b2;
            col = L.r1 ? b2 : b1;
        }
    } else {
        if (T.local) return 0;  // inter-chromosome lines only impute the whole matrix
        const long long s = T.imp_s, N2 = T.n_bins;
        long long x, mb, pb;    // the allele's own bin, the partner's M / P copies
        if (L.r1) {
            x = q1 + T.start[hap * n + L.id1];
            mb = q2 + T.start[L.id2];
            pb = q2 + T.start[n + L.id2];
        } else {                // :1347-1349 (pos2 with chrom1's offset, pos1 with chrom2's)
            x = q2 + T.start[hap * n + L.id1];
            mb = q1 + T.start[L.id2];
            pb = q1 + T.start[n + L.id2];
        }
        if (x < s || mb < s || pb < s || x + s + 1 > N2 || mb + s + 1 > N2 || pb + s + 1 > N2) return 0;
        *reached = true;
        long long own, other, r_own, c_own, r_oth, c_oth;
        if (L.r1) {
            if (hap == 0) own = disc_sum(T, x - s, mb - s);
            else if (!T.pp_ok) return kErrStale;
            else own = T.pp_sum;                       // stale M_M_sub (:1445)
            other = disc_sum(T, x - s, pb - s);
            r_own = x; c_own = mb; r_oth = x; c_oth = pb;   // the P pass also adds to M_bin2 (:1451)
        } else if (hap == 0) {
            own = disc_sum(T, mb - s, x - s);
            other = disc_sum(T, pb - s, x - s);
            r_own = x; c_own = mb; r_oth = x; c_oth = pb;
        } else {
            own = disc_sum(T, pb - s, x - s);
            other = disc_sum(T, mb - s, x - s);
            r_own = pb; c_own = x; r_oth = mb; c_oth = x;
        }
        const double tot = (double)(own + other);
        if (own >= T.imin && (double)own / tot > T.ratio) { row = r_own; col = c_own; }
        else if (other >= T.imin && (double)other / tot > T.ratio) { row = r_oth; col = c_oth; }
        else return 0;
    }
    *ok = true;
    *key = (unsigned long long)row << T.shift | (unsigned long long)col;
    return 0;
}

// Fused line split + parse + bin.  Persistent grid: block i parses tiles
// i, i + G, ...; keys go to chunks of C slots of a target's key buffer that
// the block reserves with one atomic each (a single shared cursor bumped per
// round serialises ~1e6 same-address atomics); the unused tail of a block's
// last chunk is filled with the all-ones sentinel, which sorts after every
// key (keys use 2 * shift bits, bins < 2^shift - 1).
__global__ __launch_bounds__(kScanThreads) void k_parse_tile(ParseArgs A, int TB, long long n_tiles, int C) {
    extern __shared__ uint4 dyn[];
    __shared__ unsigned starts[kScanThreads];
    __shared__ unsigned long long sh[4];
    __shared__ unsigned wcnt4[4][4];
    __shared__ unsigned long long cbase[kMaxTargets];
    __shared__ unsigned cused[kMaxTargets];
    __shared__ unsigned long long nbase4[4];
    __shared__ unsigned long long blk_lastq;
    const TextView& tv = A.tv;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const long long nblk_all = (tv.shift + tv.nbytes + 15) >> 4;
    unsigned* msk = reinterpret_cast<unsigned*>(dyn + (TB + 1 + kPLookBlk));
    if (tid < kMaxTargets) {
        cbase[tid] = 0;
        cused[tid] = (unsigned)C;  // no chunk yet
    }
    if (tid == 0) blk_lastq = 0;
    unsigned n_kept = 0, n_chr = 0, n_mark = 0, n_lines = 0;
    for (long long tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const long long T0 = tile * TB;
        const long long T1 = min(T0 + TB, nblk_all);
        const long long W0 = max(0ll, T0 - 1);
        const long long W1 = min(nblk_all, T1 + kPLookBlk);
        const int nw = (int)(W1 - W0);
        __syncthreads();  // previous tile's readers are done with dyn / msk / starts
        for (int k = tid; k < nw; k += kScanThreads) {
            const uint4 v = load16(tv.abase, W0 + k);
            dyn[k] = v;
            msk[k] = masks_of(tv, v, W0 + k);
        }
        __syncthreads();
        const TileText T{dyn, msk, W0, W1, &tv, nblk_all};
        if (A.ablate == 1) continue;
        // line starts of this thread's segment as bitmasks: aligned coordinate a
        // starts a line when a == shift (text position 0) or byte a - 1 is '\n'
        const int SB = TB / kScanThreads;
        const long long s0 = T0 + (long long)tid * SB;
        unsigned m[kPMaxSeg];
        unsigned cnt = 0;
        unsigned carry = (s0 > 0 && s0 < T1) ? (msk[s0 - 1 - W0] >> 31) & 1u : 0u;
#pragma unroll
        for (int j = 0; j < kPMaxSeg; ++j) {
            m[j] = 0;
            if (j < SB && s0 + j < T1) {
                const long long b = s0 + j;
                const unsigned nl = msk[b - W0] >> 16;
                unsigned st = ((nl << 1) | carry) & 0xffffu;
                carry = (nl >> 15) & 1u;
                // only real text positions start lines: [shift, shift + nbytes)
                const long long lo = tv.shift - b * 16, hi = tv.shift + tv.nbytes - b * 16;
                if (lo > 0) st &= lo >= 16 ? 0u : (0xffffu << lo) & 0xffffu;
                if (lo >= 0 && lo < 16) st |= 1u << lo;  // text position 0
                if (hi < 16) st &= hi <= 0 ? 0u : ((1u << hi) - 1u);
                m[j] = st;
                cnt += __popc(st);
            }
        }
        unsigned long long total = 0;
        const unsigned mybase = (unsigned)block_excl_scan_u64(cnt, sh, &total);
        const int nlines = (int)total;
        n_lines += nlines;
        for (int base = 0; base < nlines; base += kScanThreads) {
            // this round's line starts (indices [base, base + 256)) into LDS
            if (mybase + cnt > (unsigned)base && mybase < (unsigned)base + kScanThreads) {
                unsigned idx = mybase;
#pragma unroll
                for (int j = 0; j < kPMaxSeg; ++j) {
                    unsigned x = m[j];
                    while (x) {
                        const int k = __ffs(x) - 1;
                        x &= x - 1;
                        if (idx >= (unsigned)base && idx < (unsigned)base + kScanThreads)
                            starts[idx - base] = (unsigned)((s0 + j - T0) * 16 + k);
                        ++idx;
                    }
                }
            }
            __syncthreads();
            if (A.ablate == 2) continue;
            const int li = base + tid;
            LineOut L{0, 0, -1, -1, 0, 0, false, false};
            long long ls = 0;
            if (li < nlines) {
                ls = T0 * 16 + starts[tid] - tv.shift;
                L = parse_line(A, T, ls);
                if (L.status == 4) atomicMin(A.err, (unsigned long long)ls << 8 | (unsigned)L.ecode);
                n_kept += L.status == 1;
                n_chr += L.status == 2;
                n_mark += L.status == 3;
            }
            // keys of up to 4 targets per compaction phase (3 barriers)
            for (int t0 = 0; t0 < (A.ablate == 3 ? 0 : A.n_targets); t0 += 4) {
                bool ok[4];
                unsigned long long key[4];
                unsigned rk[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int t = t0 + u;
                    ok[u] = false;
                    key[u] = 0;
                    if (t < A.n_targets && L.status == 1 && A.mode == 1) {
                        bool reached = false;
                        const int e = impute_key(A, A.t[t], L, &ok[u], &key[u], &reached);
                        if (e) atomicMin(A.err, (unsigned long long)ls << 8 | (unsigned)e);
                        if (reached && A.hap1 == 0)
                            atomicMax(&blk_lastq, (A.byte_base + (unsigned long long)ls + 1ull) << 8 | (unsigned)t);
                    } else if (t < A.n_targets && L.status == 1) {
                        const TargetDev& TG = A.t[t];
                        long long b1 = 0, b2 = 0;
                        bool in_range = true;
                        if (TG.local) {
                            ok[u] = L.same_name && A.hap1 == A.hap2;
                            if (ok[u]) {
                                const long long q1 = div_res(L.p1, TG), q2 = div_res(L.p2, TG);
                                in_range = q1 < TG.nbins[L.id1] && q2 < TG.nbins[L.id2];
                                b1 = TG.start[A.hap1 * A.n_chroms + L.id1] + q1;
                                b2 = TG.start[A.hap2 * A.n_chroms + L.id2] + q2;
                            }
                        } else {
                            ok[u] = true;
                            b1 = TG.start[A.hap1 * A.n_chroms + L.id1] + div_res(L.p1, TG);
                            b2 = TG.start[A.hap2 * A.n_chroms + L.id2] + div_res(L.p2, TG);
                            in_range = b1 < TG.n_bins && b2 < TG.n_bins;
                        }
                        if (!in_range) {
                            atomicMin(A.err, (unsigned long long)ls << 8 | (unsigned)kErrBin);
                            ok[u] = false;
                        }
                        if (ok[u]) {
                            const unsigned long long lo = (unsigned long long)min(b1, b2),
                                                     hi = (unsigned long long)max(b1, b2);
                            key[u] = lo << TG.shift | hi;
                        }
                    }
                    const unsigned long long mm = __ballot(ok[u]);
                    rk[u] = __popcll(mm & ((1ull << lane) - 1ull));
                    if (lane == 0) wcnt4[u][w] = (unsigned)__popcll(mm);
                }
                __syncthreads();
                if (tid < 4 && t0 + tid < A.n_targets) {  // one lane per target reserves a chunk if needed
                    const unsigned tot = wcnt4[tid][0] + wcnt4[tid][1] + wcnt4[tid][2] + wcnt4[tid][3];
                    const unsigned room = (unsigned)C - cused[t0 + tid];
                    if (tot > room) nbase4[tid] = atomicAdd(A.t[t0 + tid].count, (unsigned long long)C);
                }
                __syncthreads();
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int t = t0 + u;
                    if (t < A.n_targets && ok[u]) {
                        unsigned idx = rk[u];
                        for (int k = 0; k < w; ++k) idx += wcnt4[u][k];
                        const unsigned used = cused[t];
                        const unsigned room = (unsigned)C - used;
                        A.t[t].keys[idx < room ? cbase[t] + used + idx : nbase4[u] + (idx - room)] = key[u];
                    }
                }
                __syncthreads();  // everyone has read cused / cbase / nbase4
                if (tid < 4 && t0 + tid < A.n_targets) {
                    const int t = t0 + tid;
                    const unsigned tot = wcnt4[tid][0] + wcnt4[tid][1] + wcnt4[tid][2] + wcnt4[tid][3];
                    const unsigned used = cused[t];
                    const unsigned room = (unsigned)C - used;
                    if (tot > room) {
                        cbase[t] = nbase4[tid];
                        cused[t] = tot - room;
                    } else {
                        cused[t] = used + tot;
                    }
                }
            }
        }
    }
    __syncthreads();
    // sentinel-fill the unused tail of each target's last chunk
    for (int t = 0; t < A.n_targets; ++t) {
        const unsigned used = cused[t];
        const unsigned gap = (unsigned)C - used;
        for (unsigned k = tid; k < gap; k += kScanThreads) A.t[t].keys[cbase[t] + used + k] = ~0ull;
        if (tid == 0 && gap) atomicAdd(A.t[t].gaps, (unsigned long long)gap);
    }
    if (tid == 0 && blk_lastq) atomicMax(A.lastq, blk_lastq);
    // line statistics: one atomic per wave and kind
    const unsigned long long c1 = wave_sum_ll(n_kept), c2 = wave_sum_ll(n_chr), c3 = wave_sum_ll(n_mark);
    if (lane == 0) {
        if (w == 0 && n_lines) atomicAdd(A.stats + 0, (unsigned long long)n_lines);
        if (c1) atomicAdd(A.stats + 1, c1);
        if (c2) atomicAdd(A.stats + 2, c2);
        if (c3) atomicAdd(A.stats + 3, c3);
    }
}

// Lines before byte `upto` of a chunk (error reports only).
__global__ void k_count_nl(TextView tv, long long upto, unsigned long long* __restrict__ out) {
    unsigned long long c = 0;
    for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < upto; p += (long long)gridDim.x * blockDim.x) {
        const long long a = p + tv.shift;
        c += byte_of(load16(tv.abase, a >> 4), (int)(a & 15)) == '\n';
    }
    c = wave_sum_ll((long long)c);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}

// ------------------------------------------------------------ radix sort
// Key sources of a pass: entry i of the input -> (key, valid).  Loads are
// unconditional from clamped addresses (a conditional load compiles to one
// round trip each).
struct RsKeys {  // a key array
    static constexpr bool kTile = false;
    const unsigned long long* k;
    long long n;
    __device__ __forceinline__ void get(long long i, unsigned long long& key, bool& ok) const {
        key = k[i < n ? i : n - 1];
        ok = i < n;
    }
};
// H's off-diagonal cells keyed by column (the genome-wide correction's
// column lists, gw.hip): fmt 1 the packed cell col << 44 | row << 24 | count,
// fmt 0 col << ib | index.  Diagonal cells are not keys.
struct RsCells {
    static constexpr bool kTile = true;
    const int32_t* r;
    const int32_t* c;
    const uint32_t* v;
    long long n;
    int fmt, ib;
    // Whole-tile fast path (block-uniform): a full tile of 16-byte aligned
    // packed-format (fmt 1) cells is read as 16-byte loads, thread t taking
    // cells [16 t, 16 t + 16) of the tile -- 12 loads per thread instead of
    // 48 four-byte ones (the per-entry form's scatter was bound by issuing
    // them, SQ_WAIT_INST_ANY 0.53).  The key keeps validity: row == col is a
    // diagonal cell (not a key).
    __device__ __forceinline__ bool tile_vec(long long base) const {
        return fmt == 1 && base + kScanTile <= n &&
               ((reinterpret_cast<uintptr_t>(r) | reinterpret_cast<uintptr_t>(c) | reinterpret_cast<uintptr_t>(v)) &
                15) == 0;
    }
    __device__ __forceinline__ void load16(long long base, int t, unsigned long long* key, bool* ok) const {
        const int4* r4 = reinterpret_cast<const int4*>(r + base) + 4 * t;
        const int4* c4 = reinterpret_cast<const int4*>(c + base) + 4 * t;
        const uint4* v4 = reinterpret_cast<const uint4*>(v + base) + 4 * t;
        int4 ra[4], ca[4];
        uint4 va[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            ra[j] = r4[j];
            ca[j] = c4[j];
            va[j] = v4[j];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int32_t rr[4] = {ra[j].x, ra[j].y, ra[j].z, ra[j].w};
            const int32_t cc[4] = {ca[j].x, ca[j].y, ca[j].z, ca[j].w};
            const uint32_t vv[4] = {va[j].x, va[j].y, va[j].z, va[j].w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                key[4 * j + q] = ((unsigned long long)cc[q] << 44) | ((unsigned long long)rr[q] << 24) |
                                 (unsigned long long)vv[q];
                ok[4 * j + q] = rr[q] != cc[q];
            }
        }
    }
    __device__ __forceinline__ static bool ok_of(unsigned long long key) {  // fmt 1
        return ((key >> 24) & 0xFFFFFull) != (key >> 44);
    }
    __device__ __forceinline__ void get(long long i, unsigned long long& key, bool& ok) const {
        const long long q = i < n ? i : n - 1;
        const int32_t rr = r[q], cc = c[q];
        const uint32_t vv = v[q];
        ok = (i < n) & (rr != cc);
        // both forms, selected by mask: a `fmt ?` here became a branch per
        // entry, which kept each entry's loads from issuing with the others
        const unsigned long long k1 =
            ((unsigned long long)cc << 44) | ((unsigned long long)rr << 24) | (unsigned long long)vv;
        const unsigned long long k0 = ((unsigned long long)cc << (ib & 63)) | (unsigned long long)i;
        const unsigned long long m = 0ull - (unsigned long long)(fmt != 0);
        key = (k1 & m) | (k0 & ~m);
    }
};
// The same cells for a histogram: the digit bits of either form are the
// column's (col << ib), so the counts are not read
struct RsCellCols {
    static constexpr bool kTile = true;
    const int32_t* r;
    const int32_t* c;
    long long n;
    int ib;
    __device__ __forceinline__ bool tile_vec(long long base) const {
        return base + kScanTile <= n &&
               ((reinterpret_cast<uintptr_t>(r) | reinterpret_cast<uintptr_t>(c)) & 15) == 0;
    }
    __device__ __forceinline__ void load16(long long base, int t, unsigned long long* key, bool* ok) const {
        const int4* r4 = reinterpret_cast<const int4*>(r + base) + 4 * t;
        const int4* c4 = reinterpret_cast<const int4*>(c + base) + 4 * t;
        int4 ra[4], ca[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            ra[j] = r4[j];
            ca[j] = c4[j];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int32_t rr[4] = {ra[j].x, ra[j].y, ra[j].z, ra[j].w};
            const int32_t cc[4] = {ca[j].x, ca[j].y, ca[j].z, ca[j].w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                key[4 * j + q] = (unsigned long long)cc[q] << (ib & 63);
                ok[4 * j + q] = rr[q] != cc[q];
            }
        }
    }
    __device__ __forceinline__ void get(long long i, unsigned long long& key, bool& ok) const {
        const long long q = i < n ? i : n - 1;
        const int32_t rr = r[q], cc = c[q];
        ok = (i < n) & (rr != cc);
        key = (unsigned long long)cc << (ib & 63);
    }
};

// Digit histogram of one 4096-key tile: each wave counts its 1 024 keys by
// ballot matching into wave-private LDS counters (no LDS atomics: a skewed
// digit -- the high bits of a row index -- serialised them), then the four
// waves' counts are summed.
template <class Src>
__global__ __launch_bounds__(kScanThreads) void k_rs_hist(Src src, int shift, long long n_tiles,
                                                          unsigned* __restrict__ hist) {
    constexpr int NW = kScanThreads / 64;
    constexpr int PER = kScanTile / NW;
    __shared__ unsigned wcnt[NW][256];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#pragma unroll
    for (int k = 0; k < NW; ++k) wcnt[k][tid] = 0;
    const long long base = (long long)blockIdx.x * kScanTile;
    unsigned long long kv[kScanItems];
    bool okv[kScanItems];
    bool vec = false;
    if constexpr (Src::kTile) vec = src.tile_vec(base);
    if (vec) {  // counts are order-free: each thread's 16 consecutive entries
        if constexpr (Src::kTile) src.load16(base, tid, kv, okv);
    } else {
#pragma unroll
        for (int r = 0; r < kScanItems; ++r) src.get(base + w * PER + r * 64 + lane, kv[r], okv[r]);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kScanItems; ++r) {
        const bool v = okv[r];
        const unsigned d = (unsigned)((kv[r] >> shift) & 0xff);
        unsigned long long m = __ballot(v);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const unsigned long long bb = __ballot((d >> b) & 1u);
            m &= ((d >> b) & 1u) ? bb : ~bb;
        }
        if (v && lane == 63 - __clzll(m)) wcnt[w][d] += (unsigned)__popcll(m);
    }
    __syncthreads();
    unsigned tot = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) tot += wcnt[k][tid];
    hist[(long long)tid * n_tiles + blockIdx.x] = tot;
}

// Stable scatter of one 4096-key tile.  Each wave owns 1 024 consecutive keys
// (16 steps of 64) and ranks them with ballots (the 8 digit bits matched
// across the wave) against wave-private digit counters in LDS -- no block
// barrier inside the ranking loop (round 1: three per step, 48 per tile).
// Then one scan over (digit, wave) places the waves' runs in key order, the
// tile is staged in LDS in digit order and written digit run by digit run.
template <class Src>
__global__ __launch_bounds__(kScanThreads) void k_rs_scatter(Src src, unsigned long long* __restrict__ out,
                                                             int shift, long long n_tiles,
                                                             const unsigned* __restrict__ hist_off) {
    constexpr int NW = kScanThreads / 64;
    constexpr int PER = kScanTile / NW;  // keys per wave
    static_assert(PER == 64 * kScanItems, "a wave's run is kScanItems steps of 64 keys");
    // kScanTile / 16 entries of padding: the vector loader writes 16
    // consecutive entries per thread at 17-entry strides (fewer bank conflicts)
    __shared__ unsigned long long stage[kScanTile + kScanTile / 16];
    __shared__ unsigned wcnt[NW][256];
    __shared__ unsigned start[256], gofs_lo[256];
    __shared__ unsigned long long sh[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const long long base = (long long)blockIdx.x * kScanTile;
#pragma unroll
    for (int k = 0; k < NW; ++k) wcnt[k][tid] = 0;
    unsigned long long kv[kScanItems];
    bool okv[kScanItems];
    bool vec = false;
    if constexpr (Src::kTile) vec = src.tile_vec(base);
    if (vec) {
        if constexpr (Src::kTile) {
            // 16-byte loads (thread t: entries 16 t ..), then through LDS into
            // the ranking order (wave w's entries w * PER + r * 64 + lane)
            unsigned long long k16[kScanItems];
            bool o16[kScanItems];
            src.load16(base, tid, k16, o16);
#pragma unroll
            for (int k = 0; k < kScanItems; ++k) stage[tid * 17 + k] = k16[k];
            __syncthreads();
#pragma unroll
            for (int r = 0; r < kScanItems; ++r) {
                const int e = w * PER + r * 64 + lane;
                kv[r] = stage[e + (e >> 4)];
                okv[r] = Src::ok_of(kv[r]);
            }
            (void)o16;
        }
    } else {
#pragma unroll
        for (int r = 0; r < kScanItems; ++r) src.get(base + w * PER + r * 64 + lane, kv[r], okv[r]);
    }
    __syncthreads();
    const unsigned long long lt = (1ull << lane) - 1ull;
    unsigned rk[kScanItems];
#pragma unroll
    for (int r = 0; r < kScanItems; ++r) {
        const bool v = okv[r];
        const unsigned d = (unsigned)((kv[r] >> shift) & 0xff);
        unsigned long long m = __ballot(v);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const unsigned long long bb = __ballot((d >> b) & 1u);
            m &= ((d >> b) & 1u) ? bb : ~bb;
        }
        // wave-private counter: every lane reads it before the leader (the
        // highest matching lane) writes it; a wave's LDS ops are in order
        const unsigned prior = wcnt[w][d];
        rk[r] = prior + (unsigned)__popcll(m & lt);
        if (v && lane == 63 - __clzll(m)) wcnt[w][d] = prior + (unsigned)__popcll(m);
    }
    __syncthreads();
    unsigned tot = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) tot += wcnt[k][tid];
    unsigned long long nk = 0;  // the tile's keys
    const unsigned st = (unsigned)block_excl_scan_u64(tot, sh, &nk);
    start[tid] = st;
    gofs_lo[tid] = hist_off[(long long)tid * n_tiles + blockIdx.x];
    {
        unsigned acc = st;  // wave w's first slot for digit tid: start + the earlier waves' counts
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            const unsigned c = wcnt[k][tid];
            wcnt[k][tid] = acc;
            acc += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kScanItems; ++r) {
        const unsigned d = (unsigned)((kv[r] >> shift) & 0xff);
        if (okv[r]) stage[wcnt[w][d] + rk[r]] = kv[r];
    }
    __syncthreads();
    for (int j = tid; j < (int)nk; j += kScanThreads) {
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

// P[r][0] = 0, P[r][k] = sum_{c < k} M[r][c] (int64, one wave per row).
__global__ __launch_bounds__(256) void k_row_prefix_i64(const long long* __restrict__ M, long long n,
                                                        long long* __restrict__ P) {
    const long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= n) return;
    long long carry = 0;
    long long* out = P + r * (n + 1);
    if (lane == 0) out[0] = 0;
    for (long long c0 = 0; c0 < n; c0 += 64) {
        const long long c = c0 + lane;
        long long v = c < n ? M[r * n + c] : 0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const long long t = __shfl_up(v, o, 64);
            if (lane >= o) v += t;
        }
        v += carry;
        if (c < n) out[c + 1] = v;
        carry = __shfl(v, 63, 64);
    }
}

}  // namespace hh

using namespace hh;

// ------------------------------------------------------------ host object
struct hh_binner {
    struct Target {
        int32_t res = 0, local = 0, shift = 0;
        uint32_t magic = 0;  // division by res: see div_res
        int32_t msh = -1;
        int64_t n_bins = 0;
        DBuf<long long> start;
        DBuf<int32_t> nbins;
        DBuf<unsigned long long> keys;
        DBuf<unsigned long long> count;  // device: slots reserved (keys + sentinels)
        DBuf<unsigned long long> gaps;   // device: sentinel slots
        int64_t n_keys = 0;              // host mirror of count after each feed
        int64_t n_gaps = 0;              // host mirror of gaps
        // results of finish
        bool done = false;
        int64_t nnz = 0;
        DBuf<int32_t> bin1, bin2, cnt;
        // imputation
        int32_t ordered = 0, imp_s = 0, pp_ok = 0;
        int64_t imin = 0, pp_sum = 0;
        double ratio = 0.0;
        DBuf<long long> rowpref;
        DBuf<int32_t> disc_j0, disc_j1;
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
    int64_t bytes_seen = 0;
    DBuf<unsigned long long> lastq;  // see ParseArgs::lastq
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

static void ensure_keys(hh_binner::Target& T, int64_t need, hipStream_t s) {
    if ((int64_t)T.keys.n >= need) return;
    const int64_t cap = std::max<int64_t>(need, (int64_t)(T.keys.n * 3 / 2) + (1 << 20));
    DBuf<unsigned long long> nk(cap);
    if (T.n_keys)
        HIP_CHECK(hipMemcpyAsync(nk.p, T.keys.p, T.n_keys * sizeof(unsigned long long), hipMemcpyDeviceToDevice, s));
    HIP_CHECK(hipStreamSynchronize(s));
    T.keys = std::move(nk);
}

// First erroneous line of the chunk just parsed (byte offset from the error
// word) -> 1-based line number in the whole feed; raises.
static void raise_parse_error(hh_binner* B, const TextView& tv, int64_t lines_before, hipStream_t s) {
    unsigned long long e = 0;
    HIP_CHECK(hipMemcpyAsync(&e, B->err.p, sizeof(e), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (e == ~0ull) return;
    const long long at = (long long)(e >> 8);
    const int code = (int)(e & 0xff);
    DBuf<unsigned long long> nl(1);
    nl.zero(s);
    if (at > 0)
        hipLaunchKernelGGL(k_count_nl, dim3((unsigned)std::min<long long>(4096, (at + 255) / 256)), dim3(256), 0, s, tv,
                           at, nl.p);
    unsigned long long before = 0;
    HIP_CHECK(hipMemcpyAsync(&before, nl.p, sizeof(before), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemsetAsync(B->err.p, 0xff, sizeof(unsigned long long), s));
    HIP_CHECK(hipStreamSynchronize(s));
    const char* what = code == kErrFields ? "missing field (IndexError in the reference)"
                       : code == kErrInt  ? "position is not a non-negative integer (ValueError in the reference)"
                       : code == kErrName ? "chromosome passes the chroms filter but is not in genomeSize (KeyError in the reference)"
                       : code == kErrStale ? "no stale M_M_sub neighbourhood for the P pass (NameError / IndexError in the reference)"
                                          : "bin outside the matrix (IndexError in the reference)";
    HH_THROW(HH_ERR_ARG, "pair line " + std::to_string(lines_before + (long long)before + 1) + ": " + what);
}

// Parse one device-resident text chunk that starts at a line start.
static void feed_device(hh_binner* B, const char* text, int64_t nbytes, const hh_pairs_format* f, hipStream_t s) {
    if (nbytes <= 0) return;
    TextView tv;
    tv.abase = reinterpret_cast<const char*>(reinterpret_cast<uintptr_t>(text) & ~uintptr_t(15));
    tv.shift = text - tv.abase;
    tv.nbytes = nbytes;
    ParseArgs A{};
    A.tv = tv;
    A.table = B->table.p;
    A.names = B->names.p;
    A.table_mask = B->table_mask;
    A.unknown_policy = B->unknown_policy;
    A.f_c1 = f->col_chrom1;
    A.f_p1 = f->col_pos1;
    A.f_c2 = f->col_chrom2;
    A.f_p2 = f->col_pos2;
    HH_REQUIRE(std::min(std::min(A.f_c1, A.f_p1), std::min(A.f_c2, A.f_p2)) >= 0, "negative field index");
    A.mark_len = (int)strnlen(f->mark, sizeof(f->mark));
    HH_REQUIRE(A.mark_len < (int)sizeof(f->mark), "mark must be NUL-terminated (<= 15 bytes)");
    std::memcpy(A.mark, f->mark, sizeof(A.mark));
    A.hap1 = f->hap1;
    A.hap2 = f->hap2;
    A.mode = f->mode;
    HH_REQUIRE(A.mode == 0 || A.mode == 1, "mode in {0 (binning), 1 (imputation)}");
    A.mark2_len = (int)strnlen(f->mark2, sizeof(f->mark2));
    HH_REQUIRE(A.mark2_len < (int)sizeof(f->mark2), "mark2 must be NUL-terminated (<= 15 bytes)");
    std::memcpy(A.mark2, f->mark2, sizeof(A.mark2));
    HH_REQUIRE(A.mode == 0 || (A.mark_len > 0 && A.hap1 == A.hap2), "imputation needs mark ('Both') and hap1 == hap2");
    A.byte_base = (unsigned long long)B->bytes_seen;
    A.lastq = B->lastq.p;
    HH_REQUIRE((A.hap1 == 0 || A.hap1 == 1) && (A.hap2 == 0 || A.hap2 == 1), "hap1/hap2 in {0, 1}");
    A.n_chroms = B->n_chroms;
    A.n_targets = (int)B->t.size();
    A.err = B->err.p;
    A.stats = B->stats.p;
    A.ablate = g_parse_ablate;
    // tile size: ~230 lines per 256-thread block, from the mean line length
    // of the first 64 KB (multiples of 256 aligned blocks, 4..40 KB)
    const int64_t ns = std::min<int64_t>(nbytes, 65536);
    std::vector<char> sample(ns);
    HIP_CHECK(hipMemcpyAsync(sample.data(), text, ns, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    const int64_t nnl = std::count(sample.begin(), sample.end(), '\n');
    const double mean_len = nnl ? (double)ns / (double)nnl : (double)ns;
    int TB = (int)std::lround(230.0 * mean_len / 16.0 / kScanThreads) * kScanThreads;
    TB = std::min(std::max(TB, kScanThreads), kPMaxSeg * kScanThreads);
    const long long nblk_all = (tv.shift + nbytes + 15) >> 4;
    const long long n_tiles = (nblk_all + TB - 1) / TB;
    // persistent grid (4 blocks per CU) and key-chunk size: ~1/16 of a
    // block's expected lines, 256..4096 slots
    int dev = 0, n_cu = 256;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    const long long grid = std::max<long long>(1, std::min<long long>(n_tiles, 4ll * n_cu));
    const double lines_per_block = (double)nbytes / mean_len / (double)grid;
    int C = 256;
    while (C < 4096 && 2.0 * C * 16.0 <= lines_per_block) C <<= 1;
    // a line that yields a key has > max field index fields, each a byte plus
    // a separator: bounds the keys this chunk can append to any target
    const int maxf = std::max(std::max(A.f_c1, A.f_p1), std::max(A.f_c2, A.f_p2));
    const int64_t max_keys = (nbytes + 1) / (2 * (maxf + 1)) + 1;
    for (size_t k = 0; k < B->t.size(); ++k) {
        auto& T = B->t[k];
        HH_REQUIRE(!T.done, "hh_binner_feed after hh_binner_finish");
        // every chunk a block opens is filled except its last: keys + grid * C
        ensure_keys(T, T.n_keys + max_keys + grid * (int64_t)C, s);
        A.has_whole |= T.local == 0;
        A.has_local |= T.local != 0;
        HH_REQUIRE((A.mode == 1) == (T.ordered != 0), "imputation targets take imputation feeds only");
        A.t[k] = TargetDev{T.start.p, T.nbins.p, T.keys.p, T.count.p, T.gaps.p, (long long)T.n_bins,
                           (long long)T.res, T.local, T.shift, T.magic, T.msh, T.ordered, T.imp_s, T.rowpref.p,
                           T.disc_j0.p, T.disc_j1.p, (long long)T.imin, T.ratio, (long long)T.pp_sum, T.pp_ok};
    }
    const int64_t lines_before = B->lines_seen;
    const size_t lds = (size_t)(TB + 1 + kPLookBlk) * (sizeof(uint4) + sizeof(unsigned));
    {
        HH_KTIME("k_parse_tile", s);
        hipLaunchKernelGGL(k_parse_tile, dim3((unsigned)grid), dim3(kScanThreads), lds, s, A, TB, n_tiles, C);
    }
    HIP_CHECK(hipGetLastError());
    // slot / gap counts and lines back to the host (capacity of the next feed)
    std::vector<unsigned long long> c(2 * B->t.size() + 1);
    for (size_t k = 0; k < B->t.size(); ++k) {
        HIP_CHECK(hipMemcpyAsync(&c[2 * k], B->t[k].count.p, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipMemcpyAsync(&c[2 * k + 1], B->t[k].gaps.p, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    }
    HIP_CHECK(hipMemcpyAsync(&c.back(), B->stats.p, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    for (size_t k = 0; k < B->t.size(); ++k) {
        B->t[k].n_keys = (int64_t)c[2 * k];
        B->t[k].n_gaps = (int64_t)c[2 * k + 1];
    }
    B->lines_seen = (int64_t)c.back();
    B->bytes_seen += nbytes;
    raise_parse_error(B, tv, lines_before, s);
}

static void sort_keys(DBuf<unsigned long long>& keys, int64_t n, int bits, hipStream_t s, int lo_bit = 0) {
    if (n <= 1) return;
    const long long tiles = (n + kScanTile - 1) / kScanTile;
    // the ping-pong buffer has the keys buffer's capacity, so after an odd
    // number of passes the two are swapped instead of copied back (a 10 GB
    // device copy, 5 ms, in the genome-wide correction's column sort)
    DBuf<unsigned long long> tmp(std::max<size_t>(keys.n, (size_t)n));
    DBuf<unsigned> hist(256 * tiles), off(256 * tiles);
    unsigned long long* a = keys.p;
    unsigned long long* b = tmp.p;
    int passes = 0;
    for (int shift = lo_bit; shift < lo_bit + bits; shift += 8, ++passes) {
        {
            HH_KTIME("k_rs_hist", s);
            hipLaunchKernelGGL(k_rs_hist<RsKeys>, dim3((unsigned)tiles), dim3(kScanThreads), 0, s,
                               RsKeys{a, (long long)n}, shift, tiles, hist.p);
        }
        exclusive_scan<unsigned, unsigned>(hist.p, off.p, 256 * tiles, nullptr, s);
        {
            HH_KTIME("k_rs_scatter", s);
            hipLaunchKernelGGL(k_rs_scatter<RsKeys>, dim3((unsigned)tiles), dim3(kScanThreads), 0, s,
                               RsKeys{a, (long long)n}, b, shift, tiles, off.p);
        }
        HIP_CHECK(hipGetLastError());
        std::swap(a, b);
    }
    HIP_CHECK(hipStreamSynchronize(s));  // tmp (the old keys buffer after a swap) / hist are released to the pool
    if (passes & 1) std::swap(keys, tmp);
}

// Shared with the device matrix build (build.hip, ice_internal.hpp).
void dev_sort_u64(DBuf<unsigned long long>& keys, int64_t n, int bits, hipStream_t s, int lo_bit) {
    sort_keys(keys, n, bits, s, lo_bit);
}

// The genome-wide correction's column lists (gw.hip): H's off-diagonal cells
// keyed by column (RsCells) and sorted stably by the cbits column bits.  The
// first radix pass reads the cells themselves (its histogram and scatter
// form the keys; no key array is written and re-read first), the rest sort
// the keys.  Returns the key count; keys must hold nnz entries.
int64_t dev_sort_cells_by_col(const int32_t* r, const int32_t* c, const uint32_t* v, int64_t nnz, int fmt, int ib,
                              int cbits, DBuf<unsigned long long>& keys, hipStream_t s) {
    if (nnz <= 0) return 0;
    const long long tiles = (nnz + kScanTile - 1) / kScanTile;
    const RsCells src{r, c, v, (long long)nnz, fmt, ib};
    int64_t hn = 0;
    {
        DBuf<unsigned> hist(256 * tiles), off(256 * tiles);
        DBuf<unsigned long long> tot(1);
        {
            HH_KTIME("k_rs_hist", s);
            hipLaunchKernelGGL(k_rs_hist<RsCellCols>, dim3((unsigned)tiles), dim3(kScanThreads), 0, s,
                               RsCellCols{r, c, (long long)nnz, ib}, ib, tiles, hist.p);
        }
        exclusive_scan<unsigned, unsigned>(hist.p, off.p, 256 * tiles, tot.p, s);
        {
            HH_KTIME("k_rs_scatter", s);
            hipLaunchKernelGGL(k_rs_scatter<RsCells>, dim3((unsigned)tiles), dim3(kScanThreads), 0, s, src, keys.p,
                               ib, tiles, off.p);
        }
        HIP_CHECK(hipGetLastError());
        unsigned long long* pin = (unsigned long long*)pinned_stage().get(0, 8);
        tot.download(pin, 1, s);
        HIP_CHECK(hipStreamSynchronize(s));
        hn = (int64_t)*pin;
    }
    if (cbits > 8) sort_keys(keys, hn, cbits - 8, s, ib + 8);
    return hn;
}
void dev_excl_scan_i64(const long long* in, long long* out, long long n, unsigned long long* total_dev, hipStream_t s) {
    exclusive_scan<long long, long long>(in, out, n, total_dev, s);
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
        for (auto& e : tab) e = NameEntry{{0, 0, 0, 0}, 0, kEmptySlot, 0, 0};
        for (int k = 0; k < n_names; ++k) {
            NameEntry ne{{0, 0, 0, 0}, span[k].second, name_ids[k], span[k].first, 0};
            for (int q = 0; q < std::min(16, span[k].second); ++q)
                ne.w[q >> 2] |= (uint32_t)(unsigned char)bytes[span[k].first + q] << (8 * (q & 3));
            ne.hash = name_hash(ne.w, ne.len);
            int slot = (int)(ne.hash & (uint32_t)(cap - 1));
            for (;;) {
                auto& e = tab[slot];
                if (e.id == kEmptySlot) {
                    e = ne;
                    break;
                }
                HH_REQUIRE(!(e.len == ne.len &&
                             std::memcmp(bytes.data() + e.off, bytes.data() + ne.off, e.len) == 0),
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
        B->lastq.alloc(1);
        B->lastq.zero(s);
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
        while ((int64_t(1) << sh) <= n_bins) ++sh;  // bins < 2^sh - 1: the all-ones key is free
        T.shift = sh;
        if (res > 1) {
            int l = 0;
            while ((int64_t(1) << l) < res) ++l;
            T.magic = (uint32_t)(((unsigned __int128)1 << 32) * ((uint64_t(1) << l) - (uint64_t)res) / (uint64_t)res + 1);
            T.msh = l - 1;
        }
        hipStream_t s = 0;
        std::vector<long long> st(chrom_start, chrom_start + 2 * B->n_chroms);
        std::vector<int32_t> nb(chrom_nbins, chrom_nbins + B->n_chroms);
        if (st.empty()) st.push_back(0);
        if (nb.empty()) nb.push_back(0);
        T.start = to_device(st, s);
        T.nbins = to_device(nb, s);
        T.count.alloc(1);
        T.count.zero(s);
        T.gaps.alloc(1);
        T.gaps.zero(s);
        HIP_CHECK(hipStreamSynchronize(s));
        *index_out = (int32_t)B->t.size();
        B->t.push_back(std::move(T));
    });
}

int hh_binner_add_impute_target(hh_binner* B, int32_t res, int32_t local, const int64_t* chrom_start,
                                const int32_t* chrom_nbins, int64_t n_bins, const int64_t* unimputed, int32_t L,
                                int64_t imin, double ratio, int32_t* index_out) {
    int rc = hh_binner_add_target(B, res, local, chrom_start, chrom_nbins, n_bins, index_out);
    if (rc) return rc;
    return guard([&] {
        auto& T = B->t[*index_out];
        T.ordered = 1;
        if (local) return;
        HH_REQUIRE(unimputed && L >= 1 && 2 * (int64_t)L + 1 <= n_bins, "whole imputation target needs the unimputed matrix and 1 <= L");
        T.imp_s = L;
        T.imin = imin;
        T.ratio = ratio;
        // GetNeighborhoodIndex (:721-732): cells of the (2L+1)^2 window with
        // sqrt((i-(L+1))^2 + (j-(L+1))^2) < sqrt(L), as column intervals per row
        std::vector<int32_t> j0(2 * L + 1, 1), j1(2 * L + 1, 0);
        for (int i = 0; i <= 2 * L; ++i) {
            int lo = -1, hi = -2;
            for (int j = 0; j <= 2 * L; ++j) {
                const double d2 = (double)((i - (L + 1)) * (i - (L + 1)) + (j - (L + 1)) * (j - (L + 1)));
                if (std::sqrt(d2) < std::sqrt((double)L)) {
                    if (lo < 0) lo = j;
                    HH_REQUIRE(hi < 0 || hi == j - 1, "disc row not contiguous");
                    hi = j;
                }
            }
            if (lo >= 0) { j0[i] = lo; j1[i] = hi; }
        }
        hipStream_t s = 0;
        T.disc_j0 = to_device(j0, s);
        T.disc_j1 = to_device(j1, s);
        DBuf<long long> dm((size_t)n_bins * n_bins);
        dm.upload(reinterpret_cast<const long long*>(unimputed), (size_t)n_bins * n_bins, s);
        T.rowpref.alloc((size_t)n_bins * (n_bins + 1));
        hipLaunchKernelGGL(k_row_prefix_i64, dim3((unsigned)((n_bins + 3) / 4)), dim3(256), 0, s, dm.p, (long long)n_bins,
                           T.rowpref.p);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipStreamSynchronize(s));
    });
}

int hh_binner_set_stale(hh_binner* B, int32_t target, int64_t pp_sum, int32_t ok) {
    return guard([&] {
        HH_REQUIRE(B && target >= 0 && target < (int)B->t.size(), "bad target");
        B->t[target].pp_sum = pp_sum;
        B->t[target].pp_ok = ok ? 1 : 0;
    });
}

int hh_binner_last_reached(const hh_binner* B, int64_t* byte_offset, int32_t* target) {
    return guard([&] {
        HH_REQUIRE(B && byte_offset && target, "null");
        unsigned long long v = 0;
        HIP_CHECK(hipMemcpy(&v, B->lastq.p, sizeof(v), hipMemcpyDeviceToHost));
        *byte_offset = v ? (int64_t)(v >> 8) - 1 : -1;
        *target = v ? (int32_t)(v & 0xff) : -1;
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
            const int64_t n_all = T.n_keys;  // keys + sentinels (sorted last)
            HH_REQUIRE(n_all < (int64_t(1) << 32) - 1, "more than 2^32 pairs in one matrix");
            sort_keys(T.keys, n_all, 2 * T.shift, s);
            const int64_t n = T.n_keys - T.n_gaps;
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
        if (n_pairs) *n_pairs = T.n_keys - T.n_gaps;
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
