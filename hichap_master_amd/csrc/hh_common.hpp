// Shared helpers for libhichap_hip.so: error plumbing across the C-ABI,
// device allocation RAII and small device utilities (wave64 reductions,
// XCD-aware block remap, counter-based hashing).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
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

// Owning device buffer.
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
        if (count) HIP_CHECK(hipMalloc(&p, count * sizeof(T)));
    }
    void release() {
        if (p) (void)hipFree(p);
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

template <class T>
DBuf<T> to_device(const std::vector<T>& v, hipStream_t s) {
    DBuf<T> d(v.size());
    d.upload(v.data(), v.size(), s);
    return d;
}

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
