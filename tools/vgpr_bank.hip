// vgpr_bank.hip -- does the VGPR bank (register index mod 4) of a VALU op's source operands set its issue rate on
// gfx950?  Each lane runs 8 independent chains in fixed physical registers (the asm names them; the values are never
// checked, only the rate); the other sources come from the chain's bank or from different ones.  Prints
// lane-instructions/s against 256 CU x 4 SIMD x 32 lanes x 2.4 GHz = 78.64 T.
//   hipcc --offload-arch=gfx950 -O3 tools/vgpr_bank.hip -o build/vgpr_bank && build/vgpr_bank
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 2048
#define STR(x) #x
#define XSTR(x) STR(x)

#define I3(op, d, a, b) op " v" XSTR(d) ", v" XSTR(d) ", v" XSTR(a) ", v" XSTR(b) "\n\t"
#define I2(op, d, a) op " v" XSTR(d) ", v" XSTR(d) ", v" XSTR(a) "\n\t"
/* chains in bank 0 (v32, v36, ..., v60) */
#define B0_3(op, a, b) I3(op, 32, a, b) I3(op, 36, a, b) I3(op, 40, a, b) I3(op, 44, a, b) \
                       I3(op, 48, a, b) I3(op, 52, a, b) I3(op, 56, a, b) I3(op, 60, a, b)
#define B0_2(op, a) I2(op, 32, a) I2(op, 36, a) I2(op, 40, a) I2(op, 44, a) \
                    I2(op, 48, a) I2(op, 52, a) I2(op, 56, a) I2(op, 60, a)
#define CLOB "v32", "v36", "v40", "v44", "v48", "v52", "v56", "v60", "v64", "v65", "v66", "v67", "v68", "v72"

template <int OP>
__global__ void __launch_bounds__(256) k(unsigned seed) {
    asm volatile("v_mov_b32 v32, %0\n\tv_mov_b32 v36, %0\n\tv_mov_b32 v40, %0\n\tv_mov_b32 v44, %0\n\t"
                 "v_mov_b32 v48, %0\n\tv_mov_b32 v52, %0\n\tv_mov_b32 v56, %0\n\tv_mov_b32 v60, %0\n\t"
                 "v_mov_b32 v64, %0\n\tv_mov_b32 v65, %0\n\tv_mov_b32 v66, %0\n\tv_mov_b32 v67, %0\n\t"
                 "v_mov_b32 v68, %0\n\tv_mov_b32 v72, %0" : : "v"(seed ^ threadIdx.x) : CLOB);
    for (int i = 0; i < ITERS; i++) {
        /* sources v68 / v72 share bank 0 with the chains; v65 / v66 are banks 1 / 2 */
        if (OP == 0) asm volatile(B0_3("v_bitop3_b32", 68, 72) : : : CLOB);          /* b3 a=b0 b=b0 c=b0 */
        if (OP == 1) asm volatile(B0_3("v_bitop3_b32", 65, 66) : : : CLOB);          /* b0 b1 b2 */
        if (OP == 2) asm volatile(B0_3("v_bitop3_b32", 65, 72) : : : CLOB);          /* b0 b1 b0 */
        if (OP == 3) asm volatile(B0_3("v_add3_u32", 68, 72) : : : CLOB);
        if (OP == 4) asm volatile(B0_3("v_add3_u32", 65, 66) : : : CLOB);
        if (OP == 5) asm volatile(B0_3("v_alignbit_b32", 68, 72) : : : CLOB);
        if (OP == 6) asm volatile(B0_3("v_alignbit_b32", 65, 66) : : : CLOB);
        if (OP == 7) asm volatile(B0_2("v_xor_b32", 68) : : : CLOB);                 /* VOP2, both bank 0 */
        if (OP == 8) asm volatile(B0_2("v_xor_b32", 65) : : : CLOB);                 /* b0 b1 */
        if (OP == 9) asm volatile(B0_2("v_add_u32", 65) B0_3("v_add3_u32", 65, 66) : : : CLOB);
        if (OP == 10) asm volatile(B0_2("v_xor_b32", 65) B0_3("v_bitop3_b32", 65, 66) : : : CLOB);
    }
}

template <int OP>
void run(const char *name, int per_iter) {
    const int blocks = 32768;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, 1u);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, 1u + r);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    const double rate = (double)reps * blocks * 256.0 * ITERS * 8 * per_iter / (ms / 1e3);
    printf("%-34s %.2f T lane-instr/s (%.1f%%)\n", name, rate / 1e12, 100.0 * rate / 78.6432e12);
}

int main() {
    run<0>("bitop3 srcs bank 0,0,0", 1);
    run<1>("bitop3 srcs bank 0,1,2", 1);
    run<2>("bitop3 srcs bank 0,1,0", 1);
    run<3>("add3 srcs bank 0,0,0", 1);
    run<4>("add3 srcs bank 0,1,2", 1);
    run<5>("alignbit srcs bank 0,0,0", 1);
    run<6>("alignbit srcs bank 0,1,2", 1);
    run<7>("xor srcs bank 0,0", 1);
    run<8>("xor srcs bank 0,1", 1);
    run<9>("add (0,1) then add3 (0,1,2)", 2);
    run<10>("xor (0,1) then bitop3 (0,1,2)", 2);
    return 0;
}
