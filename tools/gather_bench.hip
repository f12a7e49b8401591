// Microbenchmark: cost of 8-byte gathers vs. distinct cache lines per wave
// instruction, with the table resident in L1/L2/MALL.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstdint>

__global__ __launch_bounds__(256) void k_gather(const double* __restrict__ b, const uint32_t* __restrict__ idx,
                                                long long n_items, double* out) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long stride = (long long)gridDim.x * blockDim.x;
    double acc = 0;
    for (; i + 3 * stride < n_items; i += 4 * stride) {
        uint32_t a0 = idx[i], a1 = idx[i + stride], a2 = idx[i + 2 * stride], a3 = idx[i + 3 * stride];
        acc += b[a0] + b[a1] + b[a2] + b[a3];
    }
    if (acc == 12345.678) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_gatherf(const float* __restrict__ b, const uint32_t* __restrict__ idx,
                                                 long long n_items, double* out) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long stride = (long long)gridDim.x * blockDim.x;
    float acc = 0;
    for (; i + 3 * stride < n_items; i += 4 * stride) {
        uint32_t a0 = idx[i], a1 = idx[i + stride], a2 = idx[i + 2 * stride], a3 = idx[i + 3 * stride];
        acc += b[a0] + b[a1] + b[a2] + b[a3];
    }
    if (acc == 12345.678f) out[0] = acc;
}

int main() {
    const long long N = 1LL << 28;  // gathers
    std::vector<uint32_t> h(N);
    uint32_t* didx; double* db; float* dbf; double* dout;
    hipMalloc(&didx, N * 4); hipMalloc(&dout, 8);
    const long long tab = 1 << 23;  // max table 8M doubles = 64 MB
    hipMalloc(&db, tab * 8); hipMalloc(&dbf, tab * 4);
    hipMemset(db, 0, tab * 8); hipMemset(dbf, 0, tab * 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    struct Pat { const char* name; long long table; int stride; bool rnd; };
    Pat pats[] = {
        {"contig  tbl=256K", 32768, 1, false}, {"stride2 tbl=256K", 32768, 2, false},
        {"stride4 tbl=256K", 32768, 4, false}, {"stride16 tbl=256K", 32768, 16, false},
        {"random tbl=256K", 32768, 0, true}, {"random tbl=2.4M", 300000, 0, true},
        {"random tbl=4.8M", 600000, 0, true}, {"random tbl=64M", tab, 0, true},
        {"contig tbl=4.8M", 600000, 1, false}, {"stride4 tbl=4.8M", 600000, 4, false},
    };
    uint64_t x = 88172645463325252ull;
    for (auto& p : pats) {
        for (long long i = 0; i < N; ++i) {
            // lane-consecutive items are i, i+1 (stride pattern within wave)
            if (p.rnd) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = (uint32_t)(x % p.table); }
            else h[i] = (uint32_t)((i * p.stride) % p.table);
        }
        hipMemcpy(didx, h.data(), N * 4, hipMemcpyHostToDevice);
        for (int f = 0; f < 2; ++f) {
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(e0);
                if (f == 0) hipLaunchKernelGGL(k_gather, dim3(256 * 8), dim3(256), 0, 0, db, didx, N, dout);
                else hipLaunchKernelGGL(k_gatherf, dim3(256 * 8), dim3(256), 0, 0, dbf, didx, N, dout);
                hipEventRecord(e1); hipEventSynchronize(e1);
                float ms; hipEventElapsedTime(&ms, e0, e1);
                if (rep == 1)
                    printf("%-20s %s  %.3f ms  %.2f Ggather/s  idx-stream %.0f GB/s\n", p.name, f ? "f32" : "f64", ms,
                           N / ms / 1e6, N * 4.0 / ms / 1e6);
            }
        }
    }
    return 0;
}
