// Copy ceiling of the fused tile's geometry (k_fx_tile): T workgroups of 512 threads, each copying
// one contiguous span of S bytes with 16-byte lane blocks (unaligned source, aligned destination),
// 2 workgroups per CU (LDS reservation like the fused tile's 74 KB), U blocks per lane per batch.
// Compared with a plain grid-stride copy of the same bytes. hipcc -O3 --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) v4u g16;

template <int U>
__global__ void __launch_bounds__(512) k_tiles(const uint8_t* in, uint8_t* out, uint64_t span, int lds_res) {
    extern __shared__ uint8_t lds[];
    if (lds_res && threadIdx.x == 0) lds[0] = 0;
    const uint64_t base = (uint64_t)blockIdx.x * span;
    const uint32_t nb = (uint32_t)(span / 16);
    const uint8_t* src = in + base + 1;  // unaligned source like the records
    uint8_t* dst = out + base;
    for (uint32_t b = threadIdx.x; b < nb; b += U * 512) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t bb = b + u * 512;
            v[u] = bb < nb ? *(g16*)(src + 16ull * bb) : v4u{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t bb = b + u * 512;
            if (bb < nb) __builtin_nontemporal_store(v[u], (v4u*)(dst + 16ull * bb));
        }
    }
}

__global__ void k_stride(const uint8_t* in, uint8_t* out, uint64_t n16) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const v4u v = *(g16*)(in + 16 * i + 1);
        __builtin_nontemporal_store(v, (v4u*)(out + 16 * i));
    }
}

__device__ __forceinline__ v4u shr1(v4u a, v4u b) {  // bytes 1..16 of a|b
    return v4u{__builtin_amdgcn_alignbyte(a.y, a.x, 1), __builtin_amdgcn_alignbyte(a.z, a.y, 1),
               __builtin_amdgcn_alignbyte(a.w, a.z, 1), __builtin_amdgcn_alignbyte(b.x, a.w, 1)};
}
// aligned loads + the next block from the neighbouring lane (last lane loads its own)
__global__ void k_stride_shfl(const uint8_t* in, uint8_t* out, uint64_t n16) {
    const int lane = threadIdx.x & 63;
    for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x; i0 < n16; i0 += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = i0 + threadIdx.x;
        const v4u a = *(g16*)(in + 16 * i);
        v4u b;
        b.x = __shfl_down(a.x, 1, 64);
        b.y = __shfl_down(a.y, 1, 64);
        b.z = __shfl_down(a.z, 1, 64);
        b.w = __shfl_down(a.w, 1, 64);
        if (lane == 63) b = *(g16*)(in + 16 * i + 16);
        if (i < n16) __builtin_nontemporal_store(shr1(a, b), (v4u*)(out + 16 * i));
    }
}
__global__ void k_stride_al(const uint8_t* in, uint8_t* out, uint64_t n16) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const v4u v = *(g16*)(in + 16 * i);
        __builtin_nontemporal_store(v, (v4u*)(out + 16 * i));
    }
}

int main() {
    const uint64_t bytes = 4294956928ull;  // config 2A input
    uint8_t *in, *out;
    hipMalloc(&in, bytes + 4096);
    hipMalloc(&out, bytes + 4096);
    hipMemset(in, 1, bytes + 4096);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto time = [&](auto launch) {
        launch();
        hipEventRecord(a);
        for (int i = 0; i < 5; ++i) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        return ms / 5;
    };
    hipFuncSetAttribute((const void*)k_tiles<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 75 * 1024);
    hipFuncSetAttribute((const void*)k_tiles<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 75 * 1024);
    for (uint64_t T : {4976ull, 2488ull, 9952ull, 512ull}) {
        const uint64_t span = (bytes / T) & ~15ull;
        for (int lds : {0, 1}) {
            float m2 = time([&] { k_tiles<2><<<T, 512, lds ? 75 * 1024 : 0>>>(in, out, span, lds); });
            float m4 = time([&] { k_tiles<4><<<T, 512, lds ? 75 * 1024 : 0>>>(in, out, span, lds); });
            printf("tiles T=%5llu span=%7.1f KB lds=%d: U2 %.3f ms %.2f TB/s | U4 %.3f ms %.2f TB/s (read+write)\n",
                   (unsigned long long)T, span / 1024.0, lds, m2, 2.0 * span * T / m2 / 1e9, m4,
                   2.0 * span * T / m4 / 1e9);
        }
    }
    const uint64_t n16 = bytes / 16;
    for (int g : {1024, 4096, 16384}) {
        float m = time([&] { k_stride<<<g, 256>>>(in, out, n16); });
        printf("grid-stride %5d x 256: %.3f ms %.2f TB/s\n", g, m, 2.0 * n16 * 16 / m / 1e9);
        float m2 = time([&] { k_stride_shfl<<<g, 256>>>(in, out, n16 - 64); });
        printf("grid-stride aligned+shfl %5d x 256: %.3f ms %.2f TB/s\n", g, m2, 2.0 * n16 * 16 / m2 / 1e9);
        float m3 = time([&] { k_stride_al<<<g, 256>>>(in, out, n16); });
        printf("grid-stride aligned %5d x 256: %.3f ms %.2f TB/s\n", g, m3, 2.0 * n16 * 16 / m3 / 1e9);
    }
    return 0;
}
