// FETCH_SIZE / WRITE_SIZE calibration on gfx950 (MI355X_MICROARCH.md § HBM: only
// 16-B/lane coalesced reads are calibrated — FETCH_SIZE = ½ of the bytes).
// Each kernel reads (or writes) a KNOWN number of distinct bytes from a buffer
// that is not resident in the Infinity Cache (a 1 GiB buffer, evicted by a
// 512 MiB sweep before every kernel), with the access widths the update
// kernels use: 16-B and 4-B and 2-B per lane coalesced, 16-B rows scattered,
// 4-B SoA rows (28-float component records split in 7 rows, as the map slabs).
// Run under rocprofv3 --pmc FETCH_SIZE (one pass) and --pmc WRITE_SIZE (one
// pass); scripts/calib/fetch_report.py divides by the known bytes.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                       \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                   \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__global__ void k_read16(const float4* __restrict__ a, long n, float* __restrict__ out) {
    float s = 0.f;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.f) out[blockIdx.x] = s;
}
__global__ void k_read4(const float* __restrict__ a, long n, float* __restrict__ out) {
    float s = 0.f;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) s += a[i];
    if (s == 12345.f) out[blockIdx.x] = s;
}
__global__ void k_read2(const unsigned short* __restrict__ a, long n, float* __restrict__ out) {
    unsigned s = 0;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) s += a[i];
    if (s == 12345u) out[blockIdx.x] = (float)s;
}
// every 16-B row exactly once, in a scattered order (odd multiplier mod 2^k)
__global__ void k_rows16(const float4* __restrict__ a, long n, float* __restrict__ out) {
    float s = 0.f;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const long r = (i * 2654435761L) & (n - 1);
        const float4 v = a[r];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.f) out[blockIdx.x] = s;
}
// map-slab pattern: one workgroup per slab of 7 SoA rows of `cap` floats, the
// first `g` entries of every row read at 4 B/lane (a particle's prior read)
__global__ void k_slab(const float* __restrict__ a, int cap, int g, float* __restrict__ out) {
    const float* s = a + (size_t)blockIdx.x * 7 * cap;
    float acc = 0.f;
    for (int k = threadIdx.x; k < g; k += blockDim.x)
        for (int f = 0; f < 7; f++) acc += s[(size_t)f * cap + k];
    if (acc == 12345.f) out[blockIdx.x] = acc;
}
__global__ void k_write16(float4* __restrict__ a, long n) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        a[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}
__global__ void k_write4(float* __restrict__ a, long n) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) a[i] = 1.f;
}
__global__ void k_sweep(float4* __restrict__ a, long n) {  // evicts the Infinity Cache
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        a[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}

int main() {
    const long NB = 1L << 30;  // bytes read per kernel
    const long SW = 512L << 20;
    char *a, *b;
    float* out;
    CHK(hipMalloc(&a, NB));
    CHK(hipMalloc(&b, SW));
    CHK(hipMalloc(&out, 1 << 20));
    CHK(hipMemset(a, 0, NB));
    const int grid = 256 * 8 * 4, blk = 256;
    auto sweep = [&]() { hipLaunchKernelGGL(k_sweep, dim3(grid), dim3(blk), 0, 0, (float4*)b, SW / 16); };
    // the map-slab pattern: cap 704, 512 of 704 entries read per row (config 3)
    const int cap = 704, g = 512;
    const long nslab = NB / (7L * cap * 4);
    printf("kernel,bytes\n");
    sweep();
    hipLaunchKernelGGL(k_read16, dim3(grid), dim3(blk), 0, 0, (const float4*)a, NB / 16, out);
    printf("k_read16,%ld\n", NB);
    sweep();
    hipLaunchKernelGGL(k_read4, dim3(grid), dim3(blk), 0, 0, (const float*)a, NB / 4, out);
    printf("k_read4,%ld\n", NB);
    sweep();
    hipLaunchKernelGGL(k_read2, dim3(grid), dim3(blk), 0, 0, (const unsigned short*)a, NB / 2, out);
    printf("k_read2,%ld\n", NB);
    sweep();
    hipLaunchKernelGGL(k_rows16, dim3(grid), dim3(blk), 0, 0, (const float4*)a, NB / 16, out);
    printf("k_rows16,%ld\n", NB);
    sweep();
    hipLaunchKernelGGL(k_slab, dim3((unsigned)nslab), dim3(256), 0, 0, (const float*)a, cap, g, out);
    printf("k_slab,%ld\n", nslab * 7L * g * 4);
    sweep();
    hipLaunchKernelGGL(k_write16, dim3(grid), dim3(blk), 0, 0, (float4*)a, NB / 16);
    printf("k_write16,%ld\n", NB);
    sweep();
    hipLaunchKernelGGL(k_write4, dim3(grid), dim3(blk), 0, 0, (float*)a, NB / 4);
    printf("k_write4,%ld\n", NB);
    CHK(hipDeviceSynchronize());
    CHK(hipFree(a));
    CHK(hipFree(b));
    CHK(hipFree(out));
    return 0;
}
