// Microbenchmark: dependent-load latency (pointer chase) by working-set size,
// LDS chase, and dependent VALU chain, single wave, gfx950.  Diagnostics only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstdlib>

__global__ void chase(const uint32_t* __restrict__ next, uint32_t steps, uint32_t* out, long long* cyc) {
    uint32_t p = next[threadIdx.x * 32u] * 0u + (threadIdx.x & 0u);   /* divergent-looking start: vector loads */
    p = __builtin_amdgcn_readfirstlane(p) + (threadIdx.x >> 10);
    long long t0 = clock64();
    for (uint32_t i = 0; i < steps; ++i) p = next[p];
    long long t1 = clock64();
    if (threadIdx.x == 0) { out[0] = p; cyc[0] = t1 - t0; }
}
__global__ void chaseLds(const uint32_t* __restrict__ next, uint32_t n, uint32_t steps, uint32_t* out, long long* cyc) {
    extern __shared__ uint32_t s[];
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) s[i] = next[i];
    __syncthreads();
    uint32_t p = threadIdx.x >> 10;
    long long t0 = clock64();
    for (uint32_t i = 0; i < steps; ++i) p = s[p];
    long long t1 = clock64();
    if (threadIdx.x == 0) { out[0] = p; cyc[0] = t1 - t0; }
}
__global__ void alu(float x, uint32_t steps, float* out, long long* cyc) {
    float a = x + threadIdx.x;
    long long t0 = clock64();
    for (uint32_t i = 0; i < steps; ++i) { a = a * 1.0001f + 0.5f; a = a * 0.9999f - 0.25f; a = a * 1.0001f + 0.5f; a = a * 0.9999f - 0.25f; }
    long long t1 = clock64();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    uint32_t* dout; long long* dcyc; float* fout;
    hipMalloc(&dout, 4); hipMalloc(&dcyc, 8); hipMalloc(&fout, 4 * 64);
    long long cyc;
    for (size_t bytes : {4096ul, 32768ul, 262144ul, 2097152ul, 16777216ul, 268435456ul}) {
        size_t n = bytes / 4;
        std::vector<uint32_t> h(n);
        // random cyclic permutation with stride of one cache line (32 words)
        size_t lines = n / 32;
        std::vector<uint32_t> perm(lines);
        for (size_t i = 0; i < lines; ++i) perm[i] = (uint32_t)i;
        srand(1);
        for (size_t i = lines - 1; i > 0; --i) { size_t j = rand() % (i + 1); std::swap(perm[i], perm[j]); }
        for (size_t i = 0; i < lines; ++i) h[perm[i] * 32] = perm[(i + 1) % lines] * 32;
        uint32_t* d; hipMalloc(&d, bytes); hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice);
        const uint32_t steps = 20000;
        hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
        hipLaunchKernelGGL(chase, 1, 64, 0, 0, d, steps, dout, dcyc);
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(chase, 1, 64, 0, 0, d, steps, dout, dcyc);
        hipEventRecord(e1, 0); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
        printf("global chase %9zu B: %.1f ticks/load, %.1f ns/load (events)\n", bytes, (double)cyc / steps, ms * 1e6 / steps);
        if (bytes <= 65536) {
            hipLaunchKernelGGL(chaseLds, 1, 64, bytes, 0, d, (uint32_t)n, steps, dout, dcyc);
            hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
            printf("LDS chase    %9zu B: %.1f cycles/load\n", bytes, (double)cyc / steps);
        }
        hipFree(d);
    }
    {
        hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
        hipLaunchKernelGGL(alu, 1, 64, 0, 0, 1.0f, 200000u, fout, dcyc);
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(alu, 1, 64, 0, 0, 1.0f, 200000u, fout, dcyc);
        hipEventRecord(e1, 0); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
        printf("dependent f32 op chain: %.2f ticks/op, %.3f ns/op (events)\n", (double)cyc / (200000.0 * 8), ms * 1e6 / (200000.0 * 8));
    }
    int clk = 0; hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
    printf("clock %d kHz, sharedMemPerBlock %zu, maxSharedMemoryPerMultiProcessor %zu, l2 %d\n", clk, p.sharedMemPerBlock, p.maxSharedMemoryPerMultiProcessor, p.l2CacheSize);
    return 0;
}
