// fetch_probe.hip — what one small read per record costs on MI355X (gfx950): the fused tile's
// key phase reads bytes 0..24 of every 281-byte record before its copy reads the whole record.
// Kernels (4 GiB buffer, 281-byte "records"):
//   full    every byte once, 16 B per lane, grid-stride (the streaming reference)
//   heads   one 16-byte load at the start of every record (+ one at +5, as fx_issue does)
//   heads64 the same, but only records whose head sits in the first 64 B of its 128-B line
// Each is timed with hipEvents (best of 5); run under rocprofv3 --pmc FETCH_SIZE (and separately
// TCC_EA0_RDREQ_sum / TCC_EA0_RDREQ_32B_sum) to see how many bytes a partial-line miss fetches.
// Build: hipcc -O3 --offload-arch=gfx950 -o fetch_probe tools/ubench/fetch_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                   \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

typedef unsigned int v4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) v4 g16;

__global__ void k_full(const uint8_t* __restrict__ p, uint64_t n16, unsigned* sink) {
    v4 acc = {0, 0, 0, 0};
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const v4 v = *(g16*)(p + 16 * i);
        acc ^= v;
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}

__global__ void k_heads(const uint8_t* __restrict__ p, uint64_t nrec, uint64_t S, int only64, unsigned* sink) {
    v4 acc = {0, 0, 0, 0};
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nrec; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t a = 1 + i * S;
        if (only64 && ((a & 127) + 25 > 64)) continue;
        const v4 h = *(g16*)(p + a);
        const v4 k = *(g16*)(p + a + 5);
        acc ^= h ^ k;
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}

int main(int argc, char** argv) {
    const uint64_t bytes = 4ull << 30, S = 281;
    const uint64_t nrec = (bytes - 64) / S;
    uint8_t* p;
    unsigned* sink;
    CK(hipMalloc(&p, bytes + 256));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(p, 1, bytes + 256));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* which = argc > 1 ? argv[1] : "all";
    auto run = [&](const char* name, auto launch) {
        if (strcmp(which, "all") && strcmp(which, name)) return;
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        printf("%-8s %.3f ms\n", name, best);
    };
    run("full", [&] { k_full<<<32768, 256>>>(p, bytes / 16, sink); });
    run("heads", [&] { k_heads<<<32768, 256>>>(p, nrec, S, 0, sink); });
    run("heads64", [&] { k_heads<<<32768, 256>>>(p, nrec, S, 1, sink); });
    CK(hipDeviceSynchronize());
    printf("records %llu, record size %llu, buffer %llu bytes\n", (unsigned long long)nrec, (unsigned long long)S,
           (unsigned long long)bytes);
    return 0;
}
