/* Occupancy experiment for the PDF R3/R4 RC4 kernel: how many RC4 waves (16 KiB of S-boxes each) a CU holds,
 * and what the product KSA (rc4_dev.h) gains from the 10th one.
 *   A  one wave per workgroup, 16 KiB each (the LDS allocator gives 9 per CU)
 *   B  one 640-thread workgroup per CU declaring all 160 KiB: 10 RC4 waves, persistent over the batches
 *   A' A with the generated asm KSA (rc4_ksa_asm.h); same checksum required
 *   C  B + 4 key waves per workgroup doing dummy VALU work (MD5 x51) and a barrier pair per batch, as the
 *      product's key/RC4 split would
 * Each candidate: 20 x (KSA with a 16-byte key + the 2-byte early-reject PRGA); all variants must give the
 * same checksum.  Usage: rc4_wg [candidates_log2=22] [reps=3] */
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include "../dprf_amd/csrc/rc4_dev.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

DEVI uint32_t mix(uint32_t x) { x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16; return x; }

template <bool ASM = false>
DEVI uint32_t one_candidate(uint8_t *S, uint32_t lanebase, uint32_t g) {
    uint32_t h[4] = {mix(g), mix(g ^ 0x1111u), mix(g ^ 0x2222u), mix(g ^ 0x3333u)};
    uint32_t d[4] = {0x01234567u, 0, 0, 0};
    for (uint32_t x = 0; x < 20u; x++) {
        const uint32_t xx = x * 0x01010101u;
        uint32_t kx[4] = {h[0] ^ xx, h[1] ^ xx, h[2] ^ xx, h[3] ^ xx};
        if (ASM) {
            const uint32_t sb = (uint32_t)(size_t)(__attribute__((address_space(3))) uint8_t *)S;
            rc4_ksa_asm<16>(sb, sb + lanebase, kx);
        } else {
            rc4_ksa<16>(S, lanebase, kx);
        }
        rc4_prga<2>(S, lanebase, d);
    }
    return d[0] & 0xffffu;
}

template <bool ASM>
__global__ void __launch_bounds__(64) k_a(uint32_t nb, unsigned long long *sum) {
    __shared__ __attribute__((aligned(16))) uint8_t S[RC4_WAVE_BYTES];
    __builtin_amdgcn_s_setprio(3);
    const uint32_t lane = threadIdx.x;
    unsigned long long acc = 0;
    for (uint32_t b = 0; b < nb; b++) {
        const uint32_t g = (blockIdx.x * nb + b) * 64u + lane;
        acc += (unsigned long long)one_candidate<ASM>(S, lane << 2, g) * (g | 1u);
    }
    atomicAdd(sum, acc);
}

/* B / C: grid = CUs; wave w of workgroup k takes wave-batches k*10+w, +10*grid, ... */
template <int KEYW>
__global__ void __launch_bounds__(64 * (10 + KEYW)) k_b(uint32_t nwb, unsigned long long *sum, uint32_t *sink) {
    __shared__ __attribute__((aligned(16))) uint8_t S[10 * RC4_WAVE_BYTES];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t rounds = (nwb + 10u * gridDim.x - 1) / (10u * gridDim.x);
    if (w >= 10u) {
        /* key wave: MD5 x51 per candidate of two RC4 waves' batches (dummy values), between barriers */
        uint32_t h[4] = {lane, w, 0, 0};
        for (uint32_t r = 0; r < rounds; r++) {
            if (KEYW) {
                __syncthreads();
                __syncthreads();
                for (int c = 0; c < 10 / KEYW; c++)
                    for (int i = 0; i < 51; i++) {
                        uint32_t m[16] = {h[0], h[1], h[2], h[3], 0x80u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 128u, 0};
                        md5_iv(h);
                        md5_compress(h, m);
                    }
            }
        }
        if (h[0] == 0x12345678u) sink[threadIdx.x] = h[1];
        return;
    }
    __builtin_amdgcn_s_setprio(3);
    uint8_t *Sw = S + w * RC4_WAVE_BYTES;
    unsigned long long acc = 0;
    for (uint32_t r = 0; r < rounds; r++) {
        if (KEYW) { __syncthreads(); __syncthreads(); }
        const uint32_t wb = (r * gridDim.x + blockIdx.x) * 10u + w;
        if (wb >= nwb) continue;
        const uint32_t g = wb * 64u + lane;
        acc += (unsigned long long)one_candidate(Sw, lane << 2, g) * (g | 1u);
    }
    atomicAdd(sum, acc);
}

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 22;
    const int reps = argc > 2 ? atoi(argv[2]) : 3;
    const uint32_t n = 1u << lg, nwb = n / 64u;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    unsigned long long *sum;
    uint32_t *sink;
    CHECK(hipMalloc(&sum, 8));
    CHECK(hipMalloc(&sink, 4096));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int v = 0; v < 5; v++) {
        float best = 1e30f;
        unsigned long long h = 0;
        for (int r = 0; r < reps; r++) {
            CHECK(hipMemset(sum, 0, 8));
            CHECK(hipEventRecord(e0));
            if (v == 0) hipLaunchKernelGGL(k_a<false>, dim3(nwb / 8), dim3(64), 0, 0, 8u, sum);
            else if (v == 4) hipLaunchKernelGGL(k_a<true>, dim3(nwb / 8), dim3(64), 0, 0, 8u, sum);
            else if (v == 1) hipLaunchKernelGGL(k_b<0>, dim3(cus), dim3(640), 0, 0, nwb, sum, sink);
            else if (v == 2) hipLaunchKernelGGL(k_b<5>, dim3(cus), dim3(640 + 320), 0, 0, nwb, sum, sink);
            else hipLaunchKernelGGL(k_b<2>, dim3(cus), dim3(640 + 128), 0, 0, nwb, sum, sink);
            CHECK(hipGetLastError());
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
            CHECK(hipMemcpy(&h, sum, 8, hipMemcpyDeviceToHost));
        }
        static const char *name[] = {"A 1 wave/WG (9 per CU)", "B 10 RC4 waves, 160 KiB WG", "C B + 5 key waves, barriers",
                                     "C' B + 2 key waves, barriers", "A with the asm KSA (rc4_ksa_asm.h)"};
        printf("%-32s %9.3f ms  %7.1f M cand/s  checksum %016llx\n", name[v], best, n / (best * 1e3), h);
    }
    return 0;
}
