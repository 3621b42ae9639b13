// valu_peak.hip -- measures gfx950 integer VALU issue rate for the instructions the verification kernels
// are made of (v_add3_u32, v_bitop3_b32, v_alignbit_b32, v_xor_b32, v_lshl_add_u64).  Each lane runs
// 8 independent dependency chains so issue, not latency, is the limit.  Prints lane-instructions/s.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_peak.hip -o build/valu_peak && build/valu_peak
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 4096
#define CHAINS 8

template <int OP>
__global__ void __launch_bounds__(256) k(unsigned *out, unsigned seed) {
    unsigned x[CHAINS];
    unsigned y = seed ^ threadIdx.x, z = seed * 3u + blockIdx.x;
#pragma unroll
    for (int c = 0; c < CHAINS; c++) x[c] = seed + c * 77u + threadIdx.x;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) {
            if (OP == 0) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z));
            if (OP == 1) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[c]) : "v"(y), "v"(z));
            if (OP == 2) asm volatile("v_alignbit_b32 %0, %0, %0, 27" : "+v"(x[c]));
            if (OP == 3) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
            if (OP == 4) {
                unsigned long long v = ((unsigned long long)x[c] << 32) | y;
                asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(v) : "v"(((unsigned long long)z << 32) | z));
                x[c] = (unsigned)v ^ (unsigned)(v >> 32);
            }
        }
    }
    unsigned r = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; c++) r ^= x[c];
    if (r == 0x12345678u) out[0] = r;
}

template <int OP>
double run(const char *name, int blocks, int per_iter) {
    unsigned *d;
    (void)hipMalloc(&d, 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u + r);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    double lane_instr = (double)reps * blocks * 256.0 * ITERS * CHAINS * per_iter;
    double rate = lane_instr / (ms / 1e3);
    printf("%-16s blocks=%6d  %.2f T lane-instr/s  (%.1f%% of 256x4x32x2.4GHz = 78.64T)\n", name, blocks, rate / 1e12,
           100.0 * rate / 78.6432e12);
    (void)hipFree(d);
    return rate;
}

int main() {
    for (int blocks : {2048, 8192}) {
        run<0>("v_add3_u32", blocks, 1);
        run<1>("v_bitop3_b32", blocks, 1);
        run<2>("v_alignbit_b32", blocks, 1);
        run<3>("v_xor_b32", blocks, 1);
        run<4>("v_lshl_add_u64+", blocks, 1);
    }
    return 0;
}
