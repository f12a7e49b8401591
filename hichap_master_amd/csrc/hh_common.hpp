// Shared helpers for libhichap_hip.so: error plumbing across the C-ABI,
// device allocation RAII and small device utilities (wave64 reductions,
// XCD-aware block remap, counter-based hashing).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <sys/mman.h>
#include <map>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../include/hichap_hip.h"

namespace hh {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void set_error(const std::string& msg);

#define HH_THROW(code, msg)                                                   \
    do {                                                                      \
        throw ::hh::Error((code), std::string(__func__) + ": " + (msg));      \
    } while (0)

#define HH_REQUIRE(cond, msg)                                                 \
    do {                                                                      \
        if (!(cond)) HH_THROW(HH_ERR_ARG, msg);                               \
    } while (0)

#define HIP_CHECK(expr)                                                       \
    do {                                                                      \
        hipError_t e_ = (expr);                                               \
        if (e_ != hipSuccess) {                                               \
            throw ::hh::Error(e_ == hipErrorOutOfMemory ? HH_ERR_OOM : HH_ERR_HIP, \
                              std::string(#expr) + " -> " + hipGetErrorString(e_)); \
        }                                                                     \
    } while (0)

// Run a body and convert exceptions into C-ABI status codes.
template <class F>
int guard(F&& f) {
    try {
        f();
        return HH_OK;
    } catch (const Error& e) {
        set_error(e.what());
        return e.code;
    } catch (const std::bad_alloc&) {
        set_error("host allocation failed");
        return HH_ERR_OOM;
    } catch (const std::exception& e) {
        set_error(e.what());
        return HH_ERR_ARG;
    }
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Kernel timing registry (hh_ktime_*): when enabled, KTimeScope brackets a
// launch with HIP events on its stream; hh_ktime_query sums the elapsed
// times per kernel name.  Off by default (no events are created).
struct KTimeRec {
    const char* name;
    hipEvent_t a, b;
};
inline bool g_ktime_on = false;
inline std::mutex g_ktime_mu;
inline std::vector<KTimeRec> g_ktime;
struct KTimeScope {
    KTimeRec r{nullptr, nullptr, nullptr};
    hipStream_t s;
    bool on;
    KTimeScope(const char* name, hipStream_t s_) : s(s_), on(g_ktime_on && name) {
        if (!on) return;
        r.name = name;
        HIP_CHECK(hipEventCreate(&r.a));
        HIP_CHECK(hipEventCreate(&r.b));
        HIP_CHECK(hipEventRecord(r.a, s));
    }
    ~KTimeScope() {
        if (!on) return;
        (void)hipEventRecord(r.b, s);
        std::lock_guard<std::mutex> lk(g_ktime_mu);
        g_ktime.push_back(r);
    }
};
#define HH_KTIME(name, stream) ::hh::KTimeScope hh_kt_scope_(name, stream)

// Timing ablations of the pair parser (hh_tune "parse_ablate"; results are
// wrong while set): 1 stage text + masks only, 2 + line starts, 3 + parse
// without binning.
inline int g_parse_ablate = 0;

// Compartment PCA eigensolver (hh_tune "pca_method" 0 = block subspace
// iteration, 1 = block Krylov; "pca_p" = Cor products per Krylov cycle).
inline int g_pca_method = 1;
inline int g_syrk_split = -1;  // Cov K splits (hh_tune "syrk_split"): -1 auto, 0 never, n > 0 forced
inline int g_pca_p = 8;
inline int g_cor_sym = 3;  // hh_tune "cor_sym": Krylov Cor products read the upper triangle only (1 k_cor_sym, 2 k_cor_sym_pf, 3 the same with whole-line loads; 0 full)
inline int g_ortho_tpb = 0;  // hh_tune "ortho_tpb": k_ortho rows per block / 64 (0: auto)
inline int g_ortho_min_tpb = 2;  // hh_tune "ortho_min_tpb": the automatic choice's smallest rows per block / 64
inline int g_ortho_lowsync = 1;     // hh_tune "ortho_lowsync": k_ortho's Full mode as low-synch CGS2 (0: round 3's 8 reductions)
inline int g_ortho_grid_cap = 0;    // hh_tune "ortho_grid_cap": a lower cap on k_ortho's grid (0: occupancy-derived only)
inline int g_symvc_rows = 32;  // hh_tune "symvc_rows": rows per k_ts_gemv block (multiple of 16)
inline int g_symvc_out = 1;  // hh_tune "symvc_out": TwoStep pass 3 with one LDS tile (k_symvc_out; 0: k_symvc<T, 3>)
inline int g_twostep_devglue = 1;  // hh_tune "twostep_devglue": TwoStep gap / alpha glue on the device (0: host)
inline int64_t g_twostep_budget = 0;  // hh_tune "twostep_budget_mb": hh_twostep_batch workspace budget (0: free HBM)
inline int g_symvc_stream = 1;  // hh_tune "symvc_stream": TwoStep passes 1-2 as row-streaming GEMVs (0: the 64x64 tile-pair passes)
inline int g_ortho_abort_test = 0;  // hh_tune "ortho_abort_test": act as if k_ortho's barrier timed out (tests the fallback)
inline int g_pca_coop = 1;  // hh_tune "pca_coop": Krylov orthogonalisation in one launch per product (k_ortho)
inline int g_pca_debug = 0;  // hh_tune "pca_debug": per-cycle trace on stderr

// Device memory pool.  hipFree synchronises the device and costs ~0.2 ms per
// call, which dominated per-chromosome loops (a few large buffers per call),
// so released blocks are cached and reused (best fit within 2x).  Reuse is
// stream-safe because every C-ABI entry point either synchronises its stream
// before returning or keeps its buffers until a *_free that synchronises the
// device first (hh_device_quiesce).
struct PoolBlock {
    size_t bytes;
    int device;
};
inline std::mutex g_pool_mu;
inline std::multimap<size_t, std::pair<int, void*>> g_pool_free;  // bytes -> (device, ptr)
inline std::unordered_map<void*, PoolBlock> g_pool_live;
inline size_t g_pool_cached = 0;
constexpr size_t kPoolCacheCap = size_t(96) << 30;

inline void pool_trim_locked(size_t keep) {
    while (g_pool_cached > keep && !g_pool_free.empty()) {
        auto it = std::prev(g_pool_free.end());  // largest first
        int cur = 0;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(it->second.first);
        (void)hipFree(it->second.second);
        (void)hipSetDevice(cur);
        g_pool_cached -= it->first;
        g_pool_free.erase(it);
    }
}

inline void* pool_alloc(size_t bytes) {
    bytes = (bytes + 511) & ~size_t(511);
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (auto it = g_pool_free.lower_bound(bytes); it != g_pool_free.end() && it->first <= 2 * bytes; ++it) {
        if (it->second.first != dev) continue;
        void* p = it->second.second;
        g_pool_live[p] = PoolBlock{it->first, dev};
        g_pool_cached -= it->first;
        g_pool_free.erase(it);
        return p;
    }
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, bytes);
    if (e == hipErrorOutOfMemory) {
        (void)hipGetLastError();
        pool_trim_locked(0);
        e = hipMalloc(&p, bytes);
    }
    if (e != hipSuccess)
        throw Error(e == hipErrorOutOfMemory ? HH_ERR_OOM : HH_ERR_HIP,
                    std::string("hipMalloc(") + std::to_string(bytes) + ") -> " + hipGetErrorString(e));
    g_pool_live[p] = PoolBlock{bytes, dev};
    return p;
}

inline void pool_free(void* p) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    auto it = g_pool_live.find(p);
    if (it == g_pool_live.end()) return;
    g_pool_free.emplace(it->second.bytes, std::make_pair(it->second.device, p));
    g_pool_cached += it->second.bytes;
    g_pool_live.erase(it);
    if (g_pool_cached > kPoolCacheCap) pool_trim_locked(kPoolCacheCap / 2);
}

// Wait for all work on `device` (before releasing an object's buffers to the pool).
inline void device_quiesce(int device) {
    int cur = 0;
    HIP_CHECK(hipGetDevice(&cur));
    if (cur != device) HIP_CHECK(hipSetDevice(device));
    HIP_CHECK(hipDeviceSynchronize());
    if (cur != device) HIP_CHECK(hipSetDevice(cur));
}

// Owning device buffer (pooled).
template <class T>
struct DBuf {
    T* p = nullptr;
    size_t n = 0;
    DBuf() = default;
    explicit DBuf(size_t count) { alloc(count); }
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    DBuf(DBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
    DBuf& operator=(DBuf&& o) noexcept {
        if (this != &o) { release(); p = o.p; n = o.n; o.p = nullptr; o.n = 0; }
        return *this;
    }
    ~DBuf() { release(); }
    void alloc(size_t count) {
        release();
        n = count;
        if (count) p = static_cast<T*>(pool_alloc(count * sizeof(T)));
    }
    void release() {
        if (p) pool_free(p);
        p = nullptr;
        n = 0;
    }
    size_t bytes() const { return n * sizeof(T); }
    void upload(const T* h, size_t count, hipStream_t s, size_t offset = 0) {
        if (count) HIP_CHECK(hipMemcpyAsync(p + offset, h, count * sizeof(T), hipMemcpyHostToDevice, s));
    }
    void download(T* h, size_t count, hipStream_t s, size_t offset = 0) const {
        if (count) HIP_CHECK(hipMemcpyAsync(h, p + offset, count * sizeof(T), hipMemcpyDeviceToHost, s));
    }
    void zero(hipStream_t s) {
        if (n) HIP_CHECK(hipMemsetAsync(p, 0, bytes(), s));
    }
};

template <class T, class A>
DBuf<T> to_device(const std::vector<T, A>& v, hipStream_t s) {
    DBuf<T> d(v.size());
    d.upload(v.data(), v.size(), s);
    return d;
}

// Host allocator for the big tile-plan arrays (~6 KB per tile, 140 MB at
// 22 572 tiles): blocks of >= 2 MiB are anonymous mappings advised as
// transparent huge pages, so filling them takes a few hundred 2 MiB faults
// instead of ~35 000 4 KiB ones (the plan concatenation was first-touch bound).
template <class T>
struct HugeAlloc {
    using value_type = T;
    static constexpr size_t kHuge = size_t(2) << 20;
    HugeAlloc() = default;
    template <class U>
    HugeAlloc(const HugeAlloc<U>&) {}
    static size_t rounded(size_t b) { return (b + kHuge - 1) & ~(kHuge - 1); }
    T* allocate(size_t n) {
        const size_t b = n * sizeof(T);
        if (b >= kHuge) {
            void* p = mmap(nullptr, rounded(b), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
            if (p == MAP_FAILED) throw std::bad_alloc();
            (void)madvise(p, rounded(b), MADV_HUGEPAGE);
            return static_cast<T*>(p);
        }
        void* p = std::malloc(b ? b : 1);
        if (!p) throw std::bad_alloc();
        return static_cast<T*>(p);
    }
    void deallocate(T* p, size_t n) {
        const size_t b = n * sizeof(T);
        if (b >= kHuge) (void)munmap(p, rounded(b));
        else std::free(p);
    }
    // default-initialise (no zero fill): resize() does not touch the pages,
    // so threads can fault them in while they copy
    template <class U>
    void construct(U* p) noexcept { ::new ((void*)p) U; }
    template <class U, class... Args>
    void construct(U* p, Args&&... a) { ::new ((void*)p) U(std::forward<Args>(a)...); }
    template <class U>
    bool operator==(const HugeAlloc<U>&) const { return true; }
    template <class U>
    bool operator!=(const HugeAlloc<U>&) const { return false; }
};
template <class T>
using HVec = std::vector<T, HugeAlloc<T>>;

// Pinned host buffer.
template <class T>
struct PinnedBuf {
    T* p = nullptr;
    size_t n = 0;
    PinnedBuf() = default;
    explicit PinnedBuf(size_t count) { alloc(count); }
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(const PinnedBuf&) = delete;
    ~PinnedBuf() { if (p) (void)hipHostFree(p); }
    void alloc(size_t count) {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = count;
        if (count) HIP_CHECK(hipHostMalloc((void**)&p, count * sizeof(T), hipHostMallocDefault));
    }
};

// np.percentile(v, pct) with the default 'linear' method (NumPy 2.x:
// virtual index (n-1)*q, floor/next clipped to the ends, _lerp's two-sided
// form), so host-side gap and alpha decisions are bit-identical to the
// reference's NumPy calls.
// Only the two order statistics around the virtual index are needed: one
// nth_element and a min over the rest (O(n); a full sort of the ~6 000
// coverages / alphas of a chromosome was most of TwoStepCorrection's host
// time between its passes, profiles/r4m_twostep_trace.log).
inline double np_percentile(std::vector<double> v, double pct) {
    HH_REQUIRE(!v.empty(), "percentile of an empty array");
    const long long n = (long long)v.size();
    const double q = pct / 100.0;
    const double vi = (double)(n - 1) * q;
    long long prev = (long long)std::floor(vi), next = prev + 1;
    if (vi >= (double)(n - 1)) prev = next = n - 1;
    if (vi < 0) prev = next = 0;
    const double gamma = vi - (vi >= (double)(n - 1) ? -1.0 : (double)prev);
    std::nth_element(v.begin(), v.begin() + prev, v.end());
    const double a = v[prev];
    const double b = next == prev ? a : *std::min_element(v.begin() + prev + 1, v.end());
    const double d = b - a;
    return gamma >= 0.5 ? b - d * (1.0 - gamma) : a + d * gamma;
}

// Per-thread pinned host staging buffers (slot 0: downloads, 1: uploads),
// grown on demand and kept for the process (never freed: freeing pinned
// memory from a thread_local destructor at exit races the runtime's own
// teardown).  A call synchronises its stream before returning, so the next
// call on the thread may reuse them.
struct PinnedStage {
    void* p[2] = {nullptr, nullptr};
    size_t cap[2] = {0, 0};
    void* get(int slot, size_t bytes) {
        if (bytes > cap[slot]) {
            // the old buffer is idle (its copies completed before the last synchronisation)
            if (p[slot]) HIP_CHECK(hipHostFree(p[slot]));
            p[slot] = nullptr;
            cap[slot] = 0;
            const size_t want = std::max<size_t>(bytes, 1 << 20);
            HIP_CHECK(hipHostMalloc(&p[slot], want, hipHostMallocDefault));
            cap[slot] = want;
        }
        return p[slot];
    }
};
inline PinnedStage& pinned_stage() {
    static thread_local PinnedStage* st = new PinnedStage();
    return *st;
}

// Synchronous host transfers through the thread's pinned staging: pageable
// hipMemcpyAsync measured ~20 ms for a few MB (and 18 ms for 40 bytes) in
// processes holding tens of GB of device memory (the genome-wide correction,
// profiles/r4gw; the matrix build's count download), pinned DMA ~0.1 ms.
// PinnedDown batches downloads (slot 0) behind one synchronisation.
struct PinnedDown {
    struct Item {
        const void* d;
        void* h;
        size_t bytes, off;
    };
    std::vector<Item> items;
    size_t total = 0;
    template <class T>
    void add(const T* d, T* h, size_t count) {
        if (!count) return;
        items.push_back(Item{d, h, count * sizeof(T), total});
        total += (count * sizeof(T) + 15) & ~size_t(15);
    }
    void run(hipStream_t s) {
        if (items.empty()) return;
        char* base = (char*)pinned_stage().get(0, total);
        for (const Item& it : items)
            HIP_CHECK(hipMemcpyAsync(base + it.off, it.d, it.bytes, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        for (const Item& it : items) std::memcpy(it.h, base + it.off, it.bytes);
        items.clear();
        total = 0;
    }
};
// host -> device through pinned staging (slot 1), synchronised (the slot is
// free again on return)
template <class T>
inline void upload_pinned_sync(T* d, const T* h, size_t count, hipStream_t s) {
    if (!count) return;
    char* base = (char*)pinned_stage().get(1, count * sizeof(T));
    std::memcpy(base, h, count * sizeof(T));
    HIP_CHECK(hipMemcpyAsync(d, base, count * sizeof(T), hipMemcpyHostToDevice, s));
    HIP_CHECK(hipStreamSynchronize(s));
}

// ---------------------------------------------------------------- device
constexpr int kWave = 64;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

__device__ __forceinline__ long long wave_sum_ll(long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

// Block-wide sum of a double (blockDim.x multiple of 64, <= 1024); fixed
// reduction tree, so the result is deterministic. `sh` >= 16 doubles.
__device__ __forceinline__ double block_sum(double v, double* sh) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    v = wave_sum(v);
    __syncthreads();
    if (lane == 0) sh[wid] = v;
    __syncthreads();
    const int nw = blockDim.x >> 6;
    double t = 0.0;
    for (int k = 0; k < nw; ++k) t += sh[k];
    return t;
}

// XCD-aware remap of a linear block id: blocks dealt round-robin over the 8
// XCDs become contiguous logical ranges per XCD (bijective for any nb).
__device__ __forceinline__ long long xcd_remap(long long b, long long nb) {
    const long long x = b & 7, i = b >> 3;
    const long long per = nb >> 3, rem = nb & 7;
    return x < rem ? x * (per + 1) + i : rem * (per + 1) + (x - rem) * per + i;
}

// 64-bit counter-based mixing (splitmix64 finaliser).
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__host__ __device__ __forceinline__ float u01(uint64_t h) {
    return (float)(h >> 40) * (1.0f / 16777216.0f);  // [0,1)
}

}  // namespace hh
