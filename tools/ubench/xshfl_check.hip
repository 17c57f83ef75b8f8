#include <hip/hip_runtime.h>
#include <cstdint>
template <int M>
__device__ __forceinline__ uint32_t xshfl(uint32_t v) {
    const uint32_t lane = threadIdx.x & 63;
    if constexpr (M == 1) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
    } else if constexpr (M == 2) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
    } else if constexpr (M == 4) {
        const uint32_t a = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, false);
        const uint32_t b = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x12C, 0xF, 0xF, false);
        return (lane & 4) ? a : b;
    } else if constexpr (M == 8) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);
    } else if constexpr (M == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (lane & 16) ? r[0] : r[1];
    } else {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (lane & 32) ? r[0] : r[1];
    }
}
__global__ void k(unsigned* p) {
  unsigned v = p[threadIdx.x];
  unsigned o[6] = {xshfl<1>(v), xshfl<2>(v), xshfl<4>(v), xshfl<8>(v), xshfl<16>(v), xshfl<32>(v)};
  for (int i = 0; i < 6; ++i) p[64 + 64*i + threadIdx.x] = o[i];
}
int main() {
  unsigned* d; hipMalloc(&d, 7*64*4);
  unsigned h[7*64]; for (int i = 0; i < 64; ++i) h[i] = 1000 + i;
  hipMemcpy(d, h, 64*4, hipMemcpyHostToDevice);
  k<<<1, 64>>>(d); hipMemcpy(h, d, 7*64*4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int m = 0; m < 6; ++m) for (int l = 0; l < 64; ++l) if (h[64 + 64*m + l] != 1000 + (l ^ (1 << m))) { if (bad < 10) printf("m=%d lane %d got %u\n", 1<<m, l, h[64+64*m+l]); ++bad; }
  printf("xshfl check: %s (%d bad)\n", bad ? "FAIL" : "ok", bad);
  return bad != 0;
}
