// Ceiling for the compaction gather's memory pattern: 64 input streams of 281-byte records,
// output in merged (interleaved) order. Variants:
//  A: thread per output 16-B block, source address from a per-record table (1 lookup/record),
//     unaligned 16-B loads, aligned stores (the "interior block" cost with no boundaries).
//  B: same but sources in input order (sequential) -> pure streaming reference.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>
#include <algorithm>

__global__ void k_gather(const uint8_t* __restrict__ in, const uint64_t* __restrict__ src_off,
                         const uint64_t* __restrict__ dst_off, uint8_t* __restrict__ out, uint64_t nrec, uint32_t rec) {
    // wave handles 4 records; lane covers one 16-B block of one record (18 blocks per 281 B)
    const uint32_t nb = (rec + 15) / 16;
    uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t r = gid / nb; uint32_t c = gid % nb;
    if (r >= nrec) return;
    uint64_t s = src_off[r] + 16ull * c, d = dst_off[r] + 16ull * c;
    uint32_t n = rec - 16 * c; if (n > 16) n = 16;
    if (n == 16 && (d & 15) == 0) { *(uint4*)(out + d) = *(const uint4*)(in + s); }
    else { for (uint32_t i = 0; i < n; ++i) out[d + i] = in[s + i]; }
}

int main() {
    const uint32_t REC = 281, NS = 64; const uint64_t PER = 238821, N = NS * PER;
    uint8_t *in, *out; uint64_t *so, *dof;
    hipMalloc(&in, N * REC + 64); hipMalloc(&out, N * REC + 64 + 16 * N);
    hipMalloc(&so, N * 8); hipMalloc(&dof, N * 8);
    std::vector<uint64_t> keys(N), idx(N);
    std::mt19937_64 g(1);
    for (uint64_t i = 0; i < N; ++i) keys[i] = g();
    for (uint32_t s = 0; s < NS; ++s) std::sort(keys.begin() + s * PER, keys.begin() + (s + 1) * PER);
    for (uint64_t i = 0; i < N; ++i) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](uint64_t a, uint64_t b) { return keys[a] < keys[b]; });
    std::vector<uint64_t> hs(N), hd(N);
    for (int mode = 0; mode < 2; ++mode) {
        for (uint64_t j = 0; j < N; ++j) { uint64_t r = mode == 0 ? idx[j] : j; hs[j] = 1 + r * REC; hd[j] = 1 + j * REC; }
        hipMemcpy(so, hs.data(), N * 8, hipMemcpyHostToDevice);
        hipMemcpy(dof, hd.data(), N * 8, hipMemcpyHostToDevice);
        for (int aligned = 0; aligned < 2; ++aligned) {
            if (aligned) { for (uint64_t j = 0; j < N; ++j) hd[j] = j * 288; hipMemcpy(dof, hd.data(), N * 8, hipMemcpyHostToDevice); }
            uint64_t threads = N * ((REC + 15) / 16);
            dim3 grid((threads + 255) / 256);
            k_gather<<<grid, 256>>>(in, so, dof, out, N, REC);
            hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
            hipEventRecord(a);
            for (int i = 0; i < 5; ++i) k_gather<<<grid, 256>>>(in, so, dof, out, N, REC);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b); ms /= 5;
            printf("%s order, %s dst: %.3f ms  %.2f TB/s algorithmic (2 x %.2f GB)\n", mode == 0 ? "merged" : "input ",
                   aligned ? "288B-aligned" : "packed(281)", ms, 2.0 * N * REC / ms / 1e9, N * REC / 1e9);
        }
    }
    return 0;
}
