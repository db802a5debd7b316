// fetch_calib.hip — FETCH_SIZE calibration (rocprofv3 --pmc FETCH_SIZE):
// kernels that read a known number of bytes once, coalesced, at 4-, 8- and
// 16-byte lane widths, plus a gather of 8-byte words at random 64-byte
// lines (the access shape of scattered descriptor / index reads).  The
// buffer (1 GiB) is 4x the Infinity Cache, so the reads come from HBM.
// Prints the algorithmic bytes per kernel; pair it with the counter CSV.
// Build: hipcc -O3 --offload-arch=gfx950 tools/fetch_calib.hip -o gpurun_out/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

template <typename T>
__global__ void read_kernel(const T *__restrict__ p, size_t n, unsigned long long *out) {
    unsigned long long acc = 0;
    for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<size_t>(gridDim.x) * blockDim.x) {
        const T v = p[i];
        const uint32_t *w = reinterpret_cast<const uint32_t *>(&v);
        for (size_t k = 0; k < sizeof(T) / 4; ++k) acc += w[k];
    }
    if (acc == 0x123456789ull) out[0] = acc;  // keeps the loads
}

// one 8-byte word from each of n random 64-byte lines of the buffer
__global__ void gather_kernel(const uint64_t *__restrict__ p, size_t lines, size_t n, unsigned long long *out) {
    unsigned long long acc = 0;
    for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<size_t>(gridDim.x) * blockDim.x) {
        const uint64_t h = (i * 0x9e3779b97f4a7c15ull) >> 17;
        acc += p[(h % lines) * 8];
    }
    if (acc == 0x123456789ull) out[0] = acc;
}

int main() {
    const size_t bytes = size_t(1) << 30;
    void *buf;
    unsigned long long *out;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMalloc(&out, 8));
    CHECK(hipMemset(buf, 1, bytes));
    CHECK(hipDeviceSynchronize());
    const dim3 g(4096), b(256);
    hipLaunchKernelGGL((read_kernel<uint32_t>), g, b, 0, 0, static_cast<const uint32_t *>(buf), bytes / 4, out);
    hipLaunchKernelGGL((read_kernel<uint2>), g, b, 0, 0, static_cast<const uint2 *>(buf), bytes / 8, out);
    hipLaunchKernelGGL((read_kernel<uint4>), g, b, 0, 0, static_cast<const uint4 *>(buf), bytes / 16, out);
    const size_t n_gather = size_t(1) << 22;  // 4 M random lines
    hipLaunchKernelGGL(gather_kernel, g, b, 0, 0, static_cast<const uint64_t *>(buf), bytes / 64, n_gather, out);
    CHECK(hipDeviceSynchronize());
    printf("{\"read_kernel<uint32>\": %zu, \"read_kernel<uint2>\": %zu, \"read_kernel<uint4>\": %zu, "
           "\"gather_kernel_words\": %zu, \"gather_kernel_lines64\": %zu}\n",
           bytes, bytes, bytes, n_gather * 8, n_gather * 64);
    CHECK(hipFree(buf));
    CHECK(hipFree(out));
    return 0;
}
