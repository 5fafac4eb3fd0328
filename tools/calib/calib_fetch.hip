// FETCH_SIZE calibration for the access widths the ORB kernels use (MI355X_MICROARCH.md: only
// 16 B/lane streaming reads are calibrated, at 1/2). Streams a 1 GiB buffer once with 1, 4 and
// 16 bytes per lane; rocprofv3 --pmc FETCH_SIZE then gives KB per dispatch for a known byte count.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void rd_u8(const uint8_t* __restrict__ p, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc += p[i];
    if (acc == 0x12345678u) out[0] = acc;
}
__global__ void rd_u32(const uint32_t* __restrict__ p, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc += p[i];
    if (acc == 0x12345678u) out[0] = acc;
}
__global__ void rd_u128(const uint4* __restrict__ p, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}
int main() {
    const size_t bytes = 1ull << 30;
    uint8_t* buf = nullptr;
    uint32_t* out = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    hipMemset(buf, 1, bytes);
    // a 512 MiB scrub between dispatches evicts the Infinity Cache (256 MiB)
    uint8_t* scrub = nullptr;
    if (hipMalloc(&scrub, 512ull << 20) != hipSuccess) return 1;
    for (int rep = 0; rep < 2; rep++) {
        hipMemset(scrub, rep, 512ull << 20);
        hipLaunchKernelGGL(rd_u8, dim3(4096), dim3(256), 0, 0, buf, bytes, out);
        hipMemset(scrub, rep + 1, 512ull << 20);
        hipLaunchKernelGGL(rd_u32, dim3(4096), dim3(256), 0, 0, (const uint32_t*)buf, bytes / 4, out);
        hipMemset(scrub, rep + 2, 512ull << 20);
        hipLaunchKernelGGL(rd_u128, dim3(4096), dim3(256), 0, 0, (const uint4*)buf, bytes / 16, out);
    }
    hipDeviceSynchronize();
    printf("calibration: each rd_* kernel read %zu bytes\n", bytes);
    return 0;
}
