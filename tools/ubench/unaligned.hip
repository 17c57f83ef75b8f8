// Microbenchmark: are unaligned 16-byte global loads correct on gfx950, and what do they cost?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <chrono>

__global__ void k_copy(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, size_t nblk, uint32_t shift) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i < nblk; i += (size_t)gridDim.x * blockDim.x) {
        uint4 v = *(const uint4*)(src + i * 16 + shift);
        *(uint4*)(dst + i * 16) = v;
    }
}

int main() {
    const size_t N = (size_t)2 << 30;  // 2 GiB
    uint8_t *src, *dst;
    hipMalloc(&src, N + 64);
    hipMalloc(&dst, N);
    std::vector<uint8_t> h(1 << 20);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (uint8_t)(i * 131 + 7);
    hipMemcpy(src, h.data(), h.size(), hipMemcpyHostToDevice);
    const size_t nblk = N / 16;
    std::vector<uint8_t> o(1 << 16);
    for (uint32_t sh : {0u, 1u, 5u, 8u, 13u}) {
        k_copy<<<4096, 256>>>(src, dst, 4096, sh);
        hipMemcpy(o.data(), dst, o.size(), hipMemcpyDeviceToHost);
        size_t bad = 0;
        for (size_t i = 0; i < o.size(); ++i) bad += o[i] != h[i + sh];
        hipEvent_t a, b;
        hipEventCreate(&a); hipEventCreate(&b);
        k_copy<<<8192, 256>>>(src, dst, nblk, sh);
        hipEventRecord(a);
        for (int r = 0; r < 5; ++r) k_copy<<<8192, 256>>>(src, dst, nblk, sh);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        ms /= 5;
        printf("shift=%2u mismatches=%zu  copy %.3f ms  %.2f TB/s (read+write)\n", sh, bad, ms, 2.0 * N / ms / 1e9);
    }
    return 0;
}
