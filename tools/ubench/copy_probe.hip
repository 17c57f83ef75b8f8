// Copy-ceiling probe: which plain copy shape reaches the guide's ≈6.3 TB/s on this box?
// Variants: grid-stride with U independent 16-byte loads per lane before the stores, default or
// non-temporal loads/stores, aligned or +1-byte source, grid size; read-only and write-only legs.
// hipcc -O3 --offload-arch=gfx950 copy_probe.hip -o copy_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) k_copy(const uint8_t* in, uint8_t* out, uint64_t n16, uint32_t shift) {
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t i0 = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i0 < n16; i0 += stride) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = i0 + u * 256;
            const v4u* p = (const v4u*)(in + 16 * i + shift);
            if (i < n16) v[u] = NTL ? __builtin_nontemporal_load(p) : *p;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = i0 + u * 256;
            if (i < n16) {
                if (NTS) __builtin_nontemporal_store(v[u], (v4u*)(out + 16 * i));
                else *(v4u*)(out + 16 * i) = v[u];
            }
        }
    }
}

template <int U>
__global__ void __launch_bounds__(256) k_read(const uint8_t* in, uint64_t n16, uint32_t* sink) {
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    uint32_t acc = 0;
    for (uint64_t i0 = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i0 < n16; i0 += stride) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = i0 + u * 256;
            v[u] = i < n16 ? *(const v4u*)(in + 16 * i) : v4u{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void __launch_bounds__(256) k_write(uint8_t* out, uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride)
        __builtin_nontemporal_store(v4u{1, 2, 3, 4}, (v4u*)(out + 16 * i));
}

int main() {
    const uint64_t bytes = 4294956928ull & ~4095ull;
    uint8_t *in, *out;
    uint32_t* sink;
    hipMalloc(&in, bytes + 4096);
    hipMalloc(&out, bytes + 4096);
    hipMalloc(&sink, 64);
    hipMemset(in, 1, bytes + 4096);
    hipMemset(out, 0, bytes + 4096);
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
    const uint64_t n16 = bytes / 16;
    const double rw = 2.0 * bytes;
    for (int g : {2048, 4096, 8192, 32768}) {
        for (uint32_t sh : {0u, 1u}) {
            const uint64_t n = sh ? n16 - 1 : n16;
            float m1 = time([&] { k_copy<1, false, true><<<g, 256>>>(in, out, n, sh); });
            float m4 = time([&] { k_copy<4, false, true><<<g, 256>>>(in, out, n, sh); });
            float m4d = time([&] { k_copy<4, false, false><<<g, 256>>>(in, out, n, sh); });
            float m4n = time([&] { k_copy<4, true, true><<<g, 256>>>(in, out, n, sh); });
            float m8 = time([&] { k_copy<8, false, true><<<g, 256>>>(in, out, n, sh); });
            printf("grid %5d shift %u: U1 nt-st %.2f | U4 nt-st %.2f | U4 plain %.2f | U4 nt-ld+st %.2f | U8 nt-st %.2f TB/s\n",
                   g, sh, rw / m1 / 1e9, rw / m4 / 1e9, rw / m4d / 1e9, rw / m4n / 1e9, rw / m8 / 1e9);
        }
        float r = time([&] { k_read<4><<<g, 256>>>(in, n16, sink); });
        float w = time([&] { k_write<<<g, 256>>>(out, n16); });
        printf("grid %5d: read-only %.2f TB/s, write-only %.2f TB/s\n", g, bytes / r / 1e9, bytes / w / 1e9);
    }
    float mc = time([&] { hipMemcpyAsync(out, in, bytes, hipMemcpyDeviceToDevice, 0); });
    printf("hipMemcpy D2D: %.2f TB/s (read+write)\n", rw / mc / 1e9);
    return 0;
}
