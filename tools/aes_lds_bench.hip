// aes_lds_bench.hip -- AES-128 CBC encryption throughput per LDS T-table layout on gfx950.
// Each lane encrypts NBLK blocks in CBC with its own round keys (registers).  Variants:
//   V0: Te0 only, Te1..3 by rotate, one copy (random-address bank conflicts)
//   V1: Te0..Te3, one copy each
//   V2: Te0 replicated 16x (entry x of copy c at (x*16+c)*4; lane uses copy lane%16) + rotates
//   V3: Te0 replicated 32x (conflict-free for ds_read_b32) + rotates
//   V4: Te0..Te3 replicated 8x each
//   hipcc --offload-arch=gfx950 -O3 tools/aes_lds_bench.hip -o build/aes_lds_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define NBLK 256
__device__ __forceinline__ uint32_t ror(uint32_t x, int s) { return __builtin_rotateright32(x, s); }

template <int V>
__device__ __forceinline__ uint32_t T(const uint32_t *t, int k, uint32_t byte, uint32_t lane) {
    if (V == 0) return ror(t[byte], 8 * k);
    if (V == 1) return t[k * 256 + byte];
    if (V == 2) return ror(t[byte * 16 + (lane & 15)], 8 * k);
    if (V == 3) return ror(t[byte * 32 + (lane & 31)], 8 * k);
    return t[k * 2048 + byte * 8 + (lane & 7)];
}

template <int V>
__global__ void __launch_bounds__(256) k(const uint32_t *te, uint32_t *out, uint32_t seed) {
    extern __shared__ uint32_t L[];
    const int n = V == 0 ? 256 : V == 1 ? 1024 : V == 2 ? 4096 : V == 3 ? 8192 : 8192;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        int x, c, kk = 0;
        if (V == 0) x = i;
        else if (V == 1) { kk = i / 256; x = i % 256; }
        else if (V == 2) { x = i / 16; }
        else if (V == 3) { x = i / 32; }
        else { kk = i / 2048; x = (i % 2048) / 8; }
        (void)c;
        L[i] = ror(te[x], 8 * kk);
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    uint32_t rk[44];
#pragma unroll
    for (int i = 0; i < 44; i++) rk[i] = seed * (i + 1) ^ (threadIdx.x * 0x9E3779B9u) ^ blockIdx.x;
    uint32_t s0 = seed ^ threadIdx.x, s1 = s0 * 3, s2 = s0 * 5, s3 = s0 * 7;
    for (int b = 0; b < NBLK; b++) {
        s0 ^= rk[0] ^ b; s1 ^= rk[1]; s2 ^= rk[2]; s3 ^= rk[3];
#pragma unroll
        for (int r = 1; r < 10; r++) {
            uint32_t t0 = T<V>(L, 0, s0 >> 24, lane) ^ T<V>(L, 1, (s1 >> 16) & 255, lane) ^ T<V>(L, 2, (s2 >> 8) & 255, lane) ^ T<V>(L, 3, s3 & 255, lane) ^ rk[4 * r];
            uint32_t t1 = T<V>(L, 0, s1 >> 24, lane) ^ T<V>(L, 1, (s2 >> 16) & 255, lane) ^ T<V>(L, 2, (s3 >> 8) & 255, lane) ^ T<V>(L, 3, s0 & 255, lane) ^ rk[4 * r + 1];
            uint32_t t2 = T<V>(L, 0, s2 >> 24, lane) ^ T<V>(L, 1, (s3 >> 16) & 255, lane) ^ T<V>(L, 2, (s0 >> 8) & 255, lane) ^ T<V>(L, 3, s1 & 255, lane) ^ rk[4 * r + 2];
            uint32_t t3 = T<V>(L, 0, s3 >> 24, lane) ^ T<V>(L, 1, (s0 >> 16) & 255, lane) ^ T<V>(L, 2, (s1 >> 8) & 255, lane) ^ T<V>(L, 3, s2 & 255, lane) ^ rk[4 * r + 3];
            s0 = t0; s1 = t1; s2 = t2; s3 = t3;
        }
        s0 ^= rk[40]; s1 ^= rk[41]; s2 ^= rk[42]; s3 ^= rk[43];
    }
    if ((s0 ^ s1 ^ s2 ^ s3) == 0x1234567u) out[0] = s0;
}

template <int V>
void run(const char *name, uint32_t *te, uint32_t *out, size_t shm) {
    const int blocks = 256 * 16;
    hipFuncSetAttribute((const void *)k<V>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(256), shm, 0, te, out, 1u);
    (void)hipDeviceSynchronize();
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    for (int r = 0; r < 3; r++) hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(256), shm, 0, te, out, 2u + r);
    (void)hipEventRecord(b); (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b);
    double nb = 3.0 * blocks * 256.0 * NBLK;
    printf("%-34s LDS %6zu B/block  %.3f G AES-128 blocks/s (%.1f ns/ms)\n", name, shm, nb / (ms / 1e3) / 1e9, ms);
}

int main() {
    std::vector<uint32_t> h(256);
    for (int i = 0; i < 256; i++) h[i] = 0x01010101u * i ^ (i << 7);
    uint32_t *te, *out;
    (void)hipMalloc(&te, 1024); (void)hipMalloc(&out, 4);
    (void)hipMemcpy(te, h.data(), 1024, hipMemcpyHostToDevice);
    run<0>("V0 Te0+rot, 1 copy", te, out, 1024);
    run<1>("V1 Te0..3, 1 copy", te, out, 4096);
    run<2>("V2 Te0+rot, 16 copies", te, out, 16384);
    run<3>("V3 Te0+rot, 32 copies (no conflict)", te, out, 32768);
    run<4>("V4 Te0..3, 8 copies", te, out, 32768);
    return 0;
}
