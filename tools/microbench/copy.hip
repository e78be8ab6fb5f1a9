// Microbenchmark: the practical HBM ceiling for moving the headline's bytes (128 x 3 x 2160
// x 3840 bf16 read + the same written: 12.74 GB) with plain copies of several shapes, so the
// fused kernel's time can be read against what the memory system gives this access volume.
//   grid-stride float4 (walk.hip's copy), one-shot chunks of U float4 per thread (all loads
//   issued before the stores), the same with nontemporal loads / stores.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ __launch_bounds__(256) void copy_gs(const float4* __restrict__ x, float4* __restrict__ y, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        y[i] = x[i];
}

typedef float f4v __attribute__((ext_vector_type(4)));
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_chunk(const f4v* __restrict__ x, f4v* __restrict__ y, int64_t n) {
    const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
    f4v v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = base + (int64_t)u * 256;
        if (i < n) v[u] = NT ? __builtin_nontemporal_load(&x[i]) : x[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = base + (int64_t)u * 256;
        if (i < n) {
            if (NT) __builtin_nontemporal_store(v[u], &y[i]);
            else y[i] = v[u];
        }
    }
}

// one-shot copy of T elements: U per thread (lane-contiguous), all loads before the stores
template <typename T, int U>
__global__ __launch_bounds__(256) void copy_el(const T* __restrict__ x, T* __restrict__ y, int64_t n) {
    const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
    T v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = base + (int64_t)u * 256;
        if (i < n) v[u] = x[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = base + (int64_t)u * 256;
        if (i < n) y[i] = v[u];
    }
}

template <typename K>
float timeit(K k, int reps) {
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) k();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) k();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

// usage: copy [bytes per side]   (default: the headline's 6.37 GB; config 2's 1080p fp32 b32
// round trip moves 796262400 per side)
int main(int argc, char** argv) {
    const size_t bytes = argc > 1 ? (size_t)atoll(argv[1]) & ~(size_t)15 : (size_t)128 * 3 * 2160 * 3840 * 2;
    const int64_t n = (int64_t)(bytes / 16);
    float4 *x, *y;
    CK(hipMalloc(&x, bytes)); CK(hipMalloc(&y, bytes));
    CK(hipMemset(x, 0x3c, bytes)); CK(hipMemset(y, 0, bytes));
    const double gb = 2.0 * bytes / 1e9;
    auto rep = [&](const char* name, float ms) {
        printf("%-32s %.3f ms  %.0f GB/s  %.3f of 8 TB/s\n", name, ms, gb / ms * 1e3, gb / ms * 1e3 / 8000);
    };
    for (int g : {256 * 16, 256 * 64, 256 * 256})
        rep(g == 4096 ? "grid-stride float4, 4096 WGs" : g == 16384 ? "grid-stride float4, 16384 WGs" : "grid-stride float4, 65536 WGs",
            timeit([&] { hipLaunchKernelGGL(copy_gs, dim3(g), dim3(256), 0, 0, x, y, n); }, 10));
#define CH(U, NT) rep("chunk " #U " float4/thread" #NT, timeit([&] { \
        hipLaunchKernelGGL((copy_chunk<U, NT>), dim3((unsigned)((n + 256 * U - 1) / (256 * U))), dim3(256), 0, 0, (const f4v*)x, (f4v*)y, n); }, 10));
    CH(1, false) CH(4, false) CH(8, false) CH(4, true) CH(8, true)
    const int64_t nd = (int64_t)(bytes / 4), n2 = (int64_t)(bytes / 8);
#define EL(T, NN, U, NAME) rep(NAME, timeit([&] { \
        hipLaunchKernelGGL((copy_el<T, U>), dim3((unsigned)((NN + 256 * U - 1) / (256 * U))), dim3(256), 0, 0, (const T*)x, (T*)y, NN); }, 10));
    EL(uint32_t, nd, 1, "one-shot dword, 1 per thread") EL(uint32_t, nd, 4, "one-shot dword, 4 per thread")
    EL(uint32_t, nd, 16, "one-shot dword, 16 per thread") EL(uint2, n2, 1, "one-shot dwordx2, 1 per thread")
    EL(uint2, n2, 4, "one-shot dwordx2, 4 per thread")
    return 0;
}
