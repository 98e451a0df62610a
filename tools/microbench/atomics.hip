// Throughput of wave-aggregated global atomicAdd (one lane per wave) under contention:
// how many distinct counter addresses the atomics spread over, and their spacing.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(int *counters, int nAddr, int strideInts, int iters, int *sink) {
    int acc = 0;
    const int a = (blockIdx.x % nAddr) * strideInts;
    for (int i = 0; i < iters; ++i) {
        int b = 0;
        if (__lane_id() == 0) b = atomicAdd(&counters[a], 64);
        acc += __shfl(b, 0);
    }
    if (acc == 0x7fffffff) sink[0] = acc;
}

int main() {
    int *c, *sink;
    hipMalloc(&c, 64 << 20);
    hipMalloc(&sink, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 2048, iters = 16;
    struct Cfg { int nAddr, stride; } cfgs[] = {{1, 1}, {8, 1}, {8, 64}, {8, 1024}, {64, 64}, {64, 1024}, {2048, 64}};
    for (auto cf : cfgs) {
        hipMemset(c, 0, 64 << 20);
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, c, cf.nAddr, cf.stride, iters, sink);
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, c, cf.nAddr, cf.stride, iters, sink);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        double n = 5.0 * blocks * 4 * iters;  // wave atomics
        printf("addresses %5d stride %5d ints: %8.1f us/launch  %.2f ns/atomic  (%.0f M atomics/s)\n", cf.nAddr, cf.stride,
               ms * 1e3 / 5, ms * 1e6 / n, n / ms / 1e3);
    }
    return 0;
}
