// Host <-> device copy latency on this stack: pageable vs pinned, by size,
// each copy after a short kernel (the pattern of the library's glue):
// hipcc --offload-arch=gfx950 -O2 -o copy_bench copy_bench.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s\n", hipGetErrorString(e)); std::exit(1); } } while (0)

__global__ void k_touch(double* p, size_t n) {
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] += 1.0;
}

int main() {
    const size_t sizes[] = {8, 100 << 10, 5 << 20};
    const size_t big = 64 << 20;
    double* dbig = nullptr;
    char* d = nullptr;
    CK(hipMalloc(&dbig, big * sizeof(double)));
    CK(hipMalloc(&d, 8 << 20));
    char* pin = nullptr;
    CK(hipHostMalloc((void**)&pin, 8 << 20, hipHostMallocDefault));
    std::vector<char> pg(8 << 20, 1);
    hipStream_t s;
    CK(hipStreamCreate(&s));
    for (double idle_us : {0.0, 2000.0, 20000.0})
    for (int pinned = 0; pinned < 2; ++pinned)
        for (int dir = 0; dir < 2; ++dir)
            for (size_t b : sizes) {
                double tot = 0;
                const int reps = 10;
                for (int r = 0; r < reps; ++r) {
                    hipLaunchKernelGGL(k_touch, dim3(1024), dim3(256), 0, s, dbig, big);
                    CK(hipStreamSynchronize(s));
                    if (idle_us) {  // host work while the GPU idles
                        auto w = std::chrono::steady_clock::now();
                        while (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - w).count() < idle_us) {}
                    }
                    char* h = pinned ? pin : pg.data();
                    auto t0 = std::chrono::steady_clock::now();
                    if (dir == 0) CK(hipMemcpyAsync(d, h, b, hipMemcpyHostToDevice, s));
                    else CK(hipMemcpyAsync(h, d, b, hipMemcpyDeviceToHost, s));
                    CK(hipStreamSynchronize(s));
                    tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
                }
                std::printf("idle %6.0f us %s %s %8zu B: %9.1f us\n", idle_us, pinned ? "pinned  " : "pageable",
                            dir ? "D2H" : "H2D", b, tot / reps);
            }
    return 0;
}
