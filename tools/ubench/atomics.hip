// Microbenchmark: device-scope atomicAdd throughput from many workgroups,
// one address vs K striped addresses (block b -> address b % K).  Diagnostics.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void blockAtomics(unsigned long long* ctr, uint32_t iters, uint32_t K, uint32_t strideWords, unsigned long long* sink) {
    __shared__ unsigned long long s;
    unsigned long long acc = 0;
    for (uint32_t it = 0; it < iters; ++it) {
        if (threadIdx.x == 0) s = atomicAdd(&ctr[(blockIdx.x % K) * strideWords], 37ull);
        __syncthreads();
        acc += s;
        __syncthreads();
    }
    if (threadIdx.x == 0) sink[blockIdx.x] = acc;
}
__global__ void waveAtomicsNoRet(uint32_t* ctr, uint32_t iters, uint32_t K, uint32_t strideWords) {
    for (uint32_t it = 0; it < iters; ++it)
        if ((threadIdx.x & 63) == 0) atomicAdd(&ctr[(blockIdx.x % K) * strideWords], 1u);
}

int main() {
    unsigned long long* ctr; unsigned long long* sink;
    hipMalloc(&ctr, 1 << 20); hipMalloc(&sink, 8 * 65536);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const uint32_t blocks = 2048, iters = 7;
    for (uint32_t K : {1u, 8u, 32u, 128u}) {
        for (uint32_t strideW : {1u, 16u}) {
            hipLaunchKernelGGL(blockAtomics, blocks, 256, 0, 0, ctr, iters, K, strideW, sink);
            hipEventRecord(e0, 0);
            hipLaunchKernelGGL(blockAtomics, blocks, 256, 0, 0, ctr, iters, K, strideW, sink);
            hipEventRecord(e1, 0); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            printf("returning block atomics: K=%3u stride=%2u words: %.3f ms for %u atomics -> %.1f ns/atomic\n", K, strideW, ms, blocks * iters,
                   ms * 1e6 / (blocks * iters));
        }
    }
    for (uint32_t K : {1u, 32u}) {
        hipLaunchKernelGGL(waveAtomicsNoRet, blocks, 256, 0, 0, (uint32_t*)ctr, iters, K, 32u);
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(waveAtomicsNoRet, blocks, 256, 0, 0, (uint32_t*)ctr, iters, K, 32u);
        hipEventRecord(e1, 0); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("non-returning wave atomics: K=%3u: %.3f ms for %u atomics -> %.2f ns/atomic\n", K, ms, blocks * 4 * iters, ms * 1e6 / (blocks * 4 * iters));
    }
    return 0;
}
