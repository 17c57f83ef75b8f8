// Gather design study on the compaction's memory pattern (config 2A shape): 64 input streams of
// 281-byte records, output = records in merged (key) order with one version byte per 14,926
// records, so output records sit at arbitrary byte alignment. Variants:
//   copy    : aligned contiguous 16 B copy of the same byte count (the HBM copy ceiling)
//   rec1    : one thread per record, unaligned 16 B loads AND stores (tail by overlapping window)
//   rec4    : four lanes per record, each a quarter of the 16 B blocks
//   rec1_seq: rec1 with records in input order (no interleave)
// build: hipcc -O3 --offload-arch=gfx950 -o /tmp/gd tools/ubench/gather_designs.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e = (x);                                                \
        if (e != hipSuccess) {                                             \
            printf("%s failed: %s\n", #x, hipGetErrorString(e));           \
            return 1;                                                      \
        }                                                                  \
    } while (0)

__global__ void k_copy(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n16) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        uint4 a = in[i], b = in[i + stride], c = in[i + 2 * stride], d = in[i + 3 * stride];
        out[i] = a;
        out[i + stride] = b;
        out[i + 2 * stride] = c;
        out[i + 3 * stride] = d;
    }
    for (; i < n16; i += stride) out[i] = in[i];
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// NT: 0 plain, 1 non-temporal stores, 2 non-temporal loads+stores
template <int NT, int U>
__global__ void k_copy2(const u32x4* __restrict__ in, u32x4* __restrict__ out, uint64_t n16) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (; i + (U - 1) * stride < n16; i += U * stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NT == 2 ? __builtin_nontemporal_load(in + i + u * stride) : in[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NT) __builtin_nontemporal_store(v[u], out + i + u * stride);
            else out[i + u * stride] = v[u];
        }
    }
    for (; i < n16; i += stride) out[i] = in[i];
}

__device__ __forceinline__ uint4 ld16(const uint8_t* p) { return *(const uint4*)p; }
__device__ __forceinline__ void st16(uint8_t* p, uint4 v) { *(uint4*)p = v; }

// one thread per record: all loads of a 128 B chunk, then its stores
__global__ void k_rec1(const uint8_t* __restrict__ in, const uint64_t* __restrict__ src, const uint64_t* __restrict__ dst,
                       const uint32_t* __restrict__ len, uint8_t* __restrict__ out, uint64_t n) {
    uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint8_t* s = in + src[j];
    uint8_t* d = out + dst[j];
    const uint32_t L = len[j];
    uint32_t o = 0;
    for (; o + 128 <= L; o += 128) {
        uint4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = ld16(s + o + 16 * u);
#pragma unroll
        for (int u = 0; u < 8; ++u) st16(d + o + 16 * u, v[u]);
    }
    uint4 v[8];
    int m = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u)
        if (o + 16 * u + 16 <= L) { v[u] = ld16(s + o + 16 * u); m = u + 1; }
    uint4 t = L >= 16 ? ld16(s + L - 16) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < 8; ++u)
        if (u < m) st16(d + o + 16 * u, v[u]);
    if (L >= 16) st16(d + L - 16, t);
    else for (uint32_t b = 0; b < L; ++b) d[b] = s[b];
}

// four lanes per record: lane q of the group copies blocks q, q+4, ... (+ the tail window)
__global__ void k_rec4(const uint8_t* __restrict__ in, const uint64_t* __restrict__ src, const uint64_t* __restrict__ dst,
                       const uint32_t* __restrict__ len, uint8_t* __restrict__ out, uint64_t n) {
    uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t j = g >> 2;
    uint32_t q = g & 3;
    if (j >= n) return;
    const uint8_t* s = in + src[j];
    uint8_t* d = out + dst[j];
    const uint32_t L = len[j];
    const uint32_t nb = L / 16;
    uint4 v[5];
#pragma unroll
    for (int u = 0; u < 5; ++u) {
        uint32_t b = q + 4 * u;
        if (b < nb) v[u] = ld16(s + 16 * b);
    }
    uint4 t = (q == 3 && L >= 16) ? ld16(s + L - 16) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < 5; ++u) {
        uint32_t b = q + 4 * u;
        if (b < nb) st16(d + 16 * b, v[u]);
    }
    for (uint32_t b = q + 20; b < nb; b += 4) st16(d + 16 * b, ld16(s + 16 * b));
    if (q == 3 && L >= 16) st16(d + L - 16, t);
}

int main() {
    const uint32_t REC = 281, NS = 64;
    const uint64_t PER = 238821, N = NS * PER, RUN = 14926;
    const uint64_t IN = 1 + N * REC;  // treat as one buffer; streams are contiguous slices
    uint8_t *in, *out;
    uint64_t *so, *dof;
    uint32_t* ln;
    CK(hipMalloc(&in, IN + 4096));
    CK(hipMalloc(&out, N * REC + N / RUN + 4096));
    CK(hipMalloc(&so, N * 8));
    CK(hipMalloc(&dof, N * 8));
    CK(hipMalloc(&ln, N * 4));
    CK(hipMemset(in, 7, IN));
    std::vector<uint64_t> keys(N), idx(N), hs(N), hd(N);
    std::vector<uint32_t> hl(N, REC);
    std::mt19937_64 g(1);
    for (uint64_t i = 0; i < N; ++i) keys[i] = g();
    for (uint32_t s = 0; s < NS; ++s) std::sort(keys.begin() + s * PER, keys.begin() + (s + 1) * PER);
    for (uint64_t i = 0; i < N; ++i) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](uint64_t a, uint64_t b) { return keys[a] < keys[b]; });
    CK(hipMemcpy(ln, hl.data(), N * 4, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto timeit = [&](const char* name, auto launch, double bytes) {
        launch();
        hipDeviceSynchronize();
        hipEventRecord(a);
        for (int i = 0; i < 5; ++i) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        ms /= 5;
        printf("%-10s %.3f ms  %.2f TB/s (read+write %.2f GB)\n", name, ms, bytes / ms / 1e9, bytes / 1e9);
    };
    const uint64_t n16 = N * REC / 16;
    timeit("copy", [&] { k_copy<<<256 * 32, 256>>>((const uint4*)in, (uint4*)out, n16); }, 2.0 * n16 * 16);
    const u32x4* vi = (const u32x4*)in;
    u32x4* vo = (u32x4*)out;
    for (unsigned grid : {256u * 8, 256u * 32, 256u * 128, 256u * 512}) {
        char nm[64];
        snprintf(nm, sizeof nm, "c0u4g%u", grid / 256);
        timeit(nm, [&] { k_copy2<0, 4><<<grid, 256>>>(vi, vo, n16); }, 2.0 * n16 * 16);
        snprintf(nm, sizeof nm, "c1u4g%u", grid / 256);
        timeit(nm, [&] { k_copy2<1, 4><<<grid, 256>>>(vi, vo, n16); }, 2.0 * n16 * 16);
        snprintf(nm, sizeof nm, "c2u4g%u", grid / 256);
        timeit(nm, [&] { k_copy2<2, 4><<<grid, 256>>>(vi, vo, n16); }, 2.0 * n16 * 16);
        snprintf(nm, sizeof nm, "c1u8g%u", grid / 256);
        timeit(nm, [&] { k_copy2<1, 8><<<grid, 256>>>(vi, vo, n16); }, 2.0 * n16 * 16);
        snprintf(nm, sizeof nm, "c1u1g%u", grid / 256);
        timeit(nm, [&] { k_copy2<1, 1><<<grid, 256>>>(vi, vo, n16); }, 2.0 * n16 * 16);
    }
    timeit("c1u1full", [&] { k_copy2<1, 1><<<(unsigned)((n16 + 255) / 256), 256>>>(vi, vo, n16); }, 2.0 * n16 * 16);
    timeit("c0u1full", [&] { k_copy2<0, 1><<<(unsigned)((n16 + 255) / 256), 256>>>(vi, vo, n16); }, 2.0 * n16 * 16);
    for (int mode = 0; mode < 2; ++mode) {
        for (uint64_t j = 0; j < N; ++j) {
            uint64_t r = mode == 0 ? idx[j] : j;
            hs[j] = 1 + r * REC;
            hd[j] = 1 + j * REC + j / RUN;  // version byte per output run
        }
        CK(hipMemcpy(so, hs.data(), N * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(dof, hd.data(), N * 8, hipMemcpyHostToDevice));
        const double bytes = 2.0 * N * REC;
        timeit(mode == 0 ? "rec1" : "rec1_seq",
               [&] { k_rec1<<<(unsigned)((N + 255) / 256), 256>>>(in, so, dof, ln, out, N); }, bytes);
        timeit(mode == 0 ? "rec4" : "rec4_seq",
               [&] { k_rec4<<<(unsigned)((4 * N + 255) / 256), 256>>>(in, so, dof, ln, out, N); }, bytes);
    }
    return 0;
}
