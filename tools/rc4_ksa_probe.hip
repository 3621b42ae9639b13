/* RC4 KSA S-box probe (round 5, VERDICT r4 "next" #1): runs the generated asm key schedule of rc4_dev.h
 * (rc4_ksa_asm_kb, the same call k_pdf_r24 makes) for every lane of many one-wave workgroups -- 9 per CU, as in
 * the product -- and copies each lane's S-box to HBM after pass 0 and after the last pass of an R3/R4-style pass
 * loop (key ^ x, x = 0..PASSES-1, pdf_password_verifier.c:164-176).  The host compares every box with a plain RC4
 * key schedule and prints, per variant header, how many lanes differ and WHERE: the positions that differ, the
 * rows (dword w = positions 4w..4w+3) they sit in, and lane 0's first difference.  Build one executable per header:
 *   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/rc4_ksa_probe.hip -o <exe>
 * (the shipped rc4_ksa_asm.h).  Usage: <exe> [blocks] [passes] */
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <map>
#include <cstring>
#include "../dprf_amd/csrc/rc4_dev.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(2); } } while (0)

template <int NK>
__global__ void __launch_bounds__(64) k_probe(const uint32_t *keys, uint8_t *out, int passes) {
    __shared__ __attribute__((aligned(16))) uint8_t S[RC4_WAVE_BYTES];
    const uint32_t sbase = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(__attribute__((address_space(3))) uint8_t *)S);
    const uint32_t lane = threadIdx.x;
    const size_t g = (size_t)blockIdx.x * 64u + lane;
    if (sbase & 0xffffu) {                       /* the asm's layout requirement; never true for one LDS object */
        out[g * 512] = 0xee;
        return;
    }
    uint32_t k[4] = {keys[4 * g], keys[4 * g + 1], keys[4 * g + 2], keys[4 * g + 3]};
    uint32_t kb[NK];
    rc4_kb_init<NK>(k, kb);
    for (int x = 0; x < passes; x++) {
        if (x) {
            const uint32_t dx = (uint32_t)x ^ (uint32_t)(x - 1);
#pragma unroll
            for (int q = 0; q < NK; q++) kb[q] ^= dx;
        }
        rc4_ksa_asm_kb<NK>(sbase, sbase + (lane << 2), kb);
        if (x == 0 || x == passes - 1) {
            uint8_t *o = out + g * 512 + (x ? 256 : 0);
            for (int i = 0; i < 256; i++) o[i] = S[((i >> 2) << 8) + (lane << 2) + (i & 3)];
        }
        __builtin_amdgcn_s_waitcnt(0);
    }
}

/* Timing mode (round 5, the R2-R4 latency bound): one R3/R4 pass = the asm KSA + the early-reject 2-byte PRGA, as
 * k_pdf_r24's RC4 wave runs it, repeated `passes` times by WPC one-wave workgroups per CU.  With one wave per CU
 * nothing queues in front of a wave's LDS reads: the pass time is the chain's own latency (issue + unloaded round
 * trips), and 9 chains per CU (the S-box capacity) at that latency is the most the KSA design can deliver. */
template <int NK, int R>
__global__ void __launch_bounds__(64) k_time(const uint32_t *keys, uint32_t *sink, int passes) {
    __shared__ __attribute__((aligned(16))) uint8_t S[RC4_WAVE_BYTES];
    const uint32_t sbase = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(__attribute__((address_space(3))) uint8_t *)S);
    const uint32_t lane = threadIdx.x;
    const size_t g = (size_t)blockIdx.x * 64u + lane;
    uint32_t k[4] = {keys[4 * (g & 4095)], keys[4 * (g & 4095) + 1], keys[4 * (g & 4095) + 2], keys[4 * (g & 4095) + 3]};
    uint32_t kb[NK];
    rc4_kb_init<NK>(k, kb);
    uint32_t d[4] = {0, 0, 0, 0};
    for (int x = 0; x < passes; x++) {
        const uint32_t dx = (uint32_t)x ^ (uint32_t)(x - 1);
#pragma unroll
        for (int q = 0; q < NK; q++) kb[q] ^= dx;
        rc4_ksa_asm_kb<NK>(sbase, sbase + (lane << 2), kb);
        if (R == 2) {                      /* R2: one KSA + the 4-byte early-reject PRGA per candidate */
            uint32_t jj = 0;
            rc4_prga_span<1, 4>(S, lane << 2, d, jj);
        } else {
            rc4_prga<2>(S, lane << 2, d);
        }
    }
    sink[g] = d[0];
}

/* Timing mode 2 (round 5): the same RC4 work in the product's workgroup shape -- 128 threads, wave 0 the RC4 chain, wave 1
 * resident but idle at the closing barrier (a waiting wave takes no issue slots) -- so the SIMDs and the LDS see the
 * product's placement of 9 chains per CU without its key derivation */
template <int NK, int R>
__global__ void __launch_bounds__(128) k_time2(const uint32_t *keys, uint32_t *sink, int passes) {
    __shared__ __attribute__((aligned(16))) uint8_t S[RC4_WAVE_BYTES];
    if (threadIdx.x >= 64) {
        __syncthreads();
        return;
    }
    const uint32_t sbase = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(__attribute__((address_space(3))) uint8_t *)S);
    const uint32_t lane = threadIdx.x;
    const size_t g = (size_t)blockIdx.x * 64u + lane;
    uint32_t k[4] = {keys[4 * (g & 4095)], keys[4 * (g & 4095) + 1], keys[4 * (g & 4095) + 2], keys[4 * (g & 4095) + 3]};
    uint32_t kb[NK];
    rc4_kb_init<NK>(k, kb);
    uint32_t d[4] = {0, 0, 0, 0};
    for (int x = 0; x < passes; x++) {
        const uint32_t dx = (uint32_t)x ^ (uint32_t)(x - 1);
#pragma unroll
        for (int q = 0; q < NK; q++) kb[q] ^= dx;
        rc4_ksa_asm_kb<NK>(sbase, sbase + (lane << 2), kb);
        if (R == 2) {
            uint32_t jj = 0;
            rc4_prga_span<1, 4>(S, lane << 2, d, jj);
        } else {
            rc4_prga<2>(S, lane << 2, d);
        }
    }
    sink[g] = d[0];
    __syncthreads();
}

/* Mode "tenth" (round 6, VERDICT r5 Next #6): would a 10th, quarter-width RC4 chain per CU add throughput?  Nine
 * product-shape workgroups (k_time2, 16 KiB of S-boxes each) leave ~6 KiB of a CU's ~152 KiB allocatable LDS; a wave
 * whose 16 active lanes own 256-byte S-boxes in 64-byte rows (4 KiB) fits there.  k_quarter is that wave: one 64-thread
 * workgroup per CU, lanes 16-63 retire at once (an idle lane is not skipped at issue, so the wave costs a full wave's
 * issue time per instruction), the KSA as a plain per-step loop on the 64-byte rows (the asm block assumes 256-byte
 * rows: its S[j] address is a byte insert).  Launched beside the nine on a second stream, it measures how much the
 * nine chains slow down with a tenth wave resident -- the cost side of the trade -- and what the quarter chain adds. */
template <int NK>
__global__ void __launch_bounds__(64) k_quarter(const uint32_t *keys, uint32_t *sink, int passes) {
    __shared__ __attribute__((aligned(16))) uint8_t S[16 * 256];
    const uint32_t lane = threadIdx.x;
    if (lane >= 16u) return;
    const size_t g = (size_t)blockIdx.x * 16u + lane;
    uint8_t *box = S + 4u * lane;                                     /* byte i at row i/4 (64 B), column 4 lane + i%4 */
    auto at = [&](uint32_t i) -> uint8_t & { return box[((i >> 2) << 6) + (i & 3u)]; };
    uint32_t k[4] = {keys[4 * (g & 4095)], keys[4 * (g & 4095) + 1], keys[4 * (g & 4095) + 2], keys[4 * (g & 4095) + 3]};
    uint32_t acc = 0;
    for (int x = 0; x < passes; x++) {
        for (uint32_t i = 0; i < 256u; i++) at(i) = (uint8_t)i;
        uint32_t j = 0;
#pragma unroll 8
        for (uint32_t i = 0; i < 256u; i++) {
            const uint32_t si = at(i);
            j = (j + si + (((k[(i % NK) >> 2] >> (8 * ((i % NK) & 3u))) ^ (uint32_t)x) & 0xffu)) & 0xffu;
            const uint32_t sj = at(j);
            at(i) = (uint8_t)sj;
            at(j) = (uint8_t)si;
        }
        acc += at(1) + at(2);                                         /* the PRGA-2 reads, roughly */
    }
    sink[g] = acc;
}

static void time_tenth(int passes, int qpasses) {
    int ncu = 0;
    CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<uint32_t> keys(4096 * 4);
    uint64_t st = 0x243F6A8885A308D3ull;
    for (auto &w : keys) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; w = (uint32_t)st; }
    uint32_t *dk, *ds, *dq;
    CHECK(hipMalloc(&dk, keys.size() * 4));
    CHECK(hipMalloc(&ds, (size_t)ncu * 9 * 64 * 4));
    CHECK(hipMalloc(&dq, (size_t)ncu * 16 * 4));
    CHECK(hipMemcpy(dk, keys.data(), keys.size() * 4, hipMemcpyHostToDevice));
    hipStream_t s1, s2;
    CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t a1, b1, a2, b2;
    CHECK(hipEventCreate(&a1)); CHECK(hipEventCreate(&b1)); CHECK(hipEventCreate(&a2)); CHECK(hipEventCreate(&b2));
    for (int r = 0; r < 8; r++) hipLaunchKernelGGL((k_time2<16, 3>), dim3(ncu * 9), dim3(128), 0, s1, dk, ds, passes);
    CHECK(hipDeviceSynchronize());
    for (int rep = 0; rep < 3; rep++) {
        for (int mode = 0; mode < 3; mode++) {                        /* 0: nine alone, 1: quarter alone, 2: both */
            float m1 = 0, m2 = 0;
            if (mode != 1) CHECK(hipEventRecord(a1, s1));
            if (mode != 0) CHECK(hipEventRecord(a2, s2));
            if (mode != 1) hipLaunchKernelGGL((k_time2<16, 3>), dim3(ncu * 9), dim3(128), 0, s1, dk, ds, passes);
            if (mode != 0) hipLaunchKernelGGL((k_quarter<16>), dim3(ncu), dim3(64), 0, s2, dk, dq, qpasses);
            if (mode != 1) CHECK(hipEventRecord(b1, s1));
            if (mode != 0) CHECK(hipEventRecord(b2, s2));
            CHECK(hipDeviceSynchronize());
            if (mode != 1) CHECK(hipEventElapsedTime(&m1, a1, b1));
            if (mode != 0) CHECK(hipEventElapsedTime(&m2, a2, b2));
            const double nine = mode != 1 ? (double)ncu * 9 * 64 * passes / 20.0 / (m1 * 1e-3) : 0;
            const double quarter = mode != 0 ? (double)ncu * 16 * qpasses / 20.0 / (m2 * 1e-3) : 0;
            printf("{\"mode\": \"%s\", \"rep\": %d, \"nine_ms\": %.3f, \"quarter_ms\": %.3f, "
                   "\"nine_cand_per_s\": %.4g, \"quarter_cand_per_s\": %.4g}\n",
                   mode == 0 ? "nine alone" : mode == 1 ? "quarter alone" : "nine + quarter", rep, m1, m2, nine, quarter);
        }
    }
    CHECK(hipFree(dk)); CHECK(hipFree(ds)); CHECK(hipFree(dq));
}

template <int NK, int R>
static void time_passes2(int passes) {
    int ncu = 0;
    CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<uint32_t> keys(4096 * 4);
    uint64_t st = 0x243F6A8885A308D3ull;
    for (auto &w : keys) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; w = (uint32_t)st; }
    uint32_t *dk, *ds;
    CHECK(hipMalloc(&dk, keys.size() * 4));
    CHECK(hipMalloc(&ds, (size_t)ncu * 10 * 64 * 4));
    CHECK(hipMemcpy(dk, keys.data(), keys.size() * 4, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    for (int r = 0; r < 8; r++) hipLaunchKernelGGL((k_time2<NK, R>), dim3(ncu * 9), dim3(128), 0, 0, dk, ds, passes);
    CHECK(hipDeviceSynchronize());
    for (int wpc : {4, 8, 9}) {
        const int blocks = ncu * wpc;
        float best = 1e30f;
        for (int rep = 0; rep < 3; rep++) {
            CHECK(hipEventRecord(a, 0));
            hipLaunchKernelGGL((k_time2<NK, R>), dim3(blocks), dim3(128), 0, 0, dk, ds, passes);
            CHECK(hipEventRecord(b, 0));
            CHECK(hipEventSynchronize(b));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, a, b));
            best = ms < best ? ms : best;
        }
        const double pass_ns = best * 1e6 / passes;
        const double rate = (double)blocks * 64 / ((R == 2 ? 1.0 : 20.0) * pass_ns * 1e-9);
        printf("{\"mode\": \"128-thread workgroups, idle second wave\", \"r\": %d, \"nk\": %d, \"chains_per_cu\": %d, "
               "\"passes\": %d, \"ms\": %.3f, \"pass_ns\": %.1f, \"cand_per_s\": %.4g}\n", R, NK, wpc, passes, best,
               pass_ns, rate);
    }
    /* many generations, as the product runs: 30 workgroups' worth per resident slot, each of passes / 20 passes, so
     * a SIMD that frees first takes the next workgroup (the single generation above waits for its busiest SIMD) */
    {
        const int gens = 30, wp = passes / 20 > 0 ? passes / 20 : 1;
        const int blocks = ncu * 9 * gens;
        uint32_t *dsb;
        CHECK(hipMalloc(&dsb, (size_t)blocks * 64 * 4));
        float best = 1e30f;
        for (int rep = 0; rep < 3; rep++) {
            CHECK(hipEventRecord(a, 0));
            hipLaunchKernelGGL((k_time2<NK, R>), dim3(blocks), dim3(128), 0, 0, dk, dsb, wp);
            CHECK(hipEventRecord(b, 0));
            CHECK(hipEventSynchronize(b));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, a, b));
            best = ms < best ? ms : best;
        }
        const double cand = (double)blocks * 64 * wp / (R == 2 ? 1.0 : 20.0);
        printf("{\"mode\": \"128-thread workgroups, idle second wave, %d generations of 9 per CU\", \"r\": %d, "
               "\"nk\": %d, \"passes_per_workgroup\": %d, \"ms\": %.3f, \"pass_ns_per_chain\": %.1f, "
               "\"cand_per_s\": %.4g}\n", gens, R, NK, wp, best, best * 1e6 * ncu * 9 / ((double)blocks * wp),
               cand / (best * 1e-3));
        CHECK(hipFree(dsb));
    }
    CHECK(hipFree(dk)); CHECK(hipFree(ds));
}

template <int NK, int R>
static void time_passes(int passes) {
    int ncu = 0;
    CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<uint32_t> keys(4096 * 4);
    uint64_t st = 0x243F6A8885A308D3ull;
    for (auto &w : keys) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; w = (uint32_t)st; }
    uint32_t *dk, *ds;
    CHECK(hipMalloc(&dk, keys.size() * 4));
    CHECK(hipMalloc(&ds, (size_t)ncu * 10 * 64 * 4));
    CHECK(hipMemcpy(dk, keys.data(), keys.size() * 4, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    /* warm-up: ~0.3 s of full-occupancy work, so the clock has ramped before the first timed launch */
    for (int r = 0; r < 8; r++) hipLaunchKernelGGL((k_time<NK, R>), dim3(ncu * 9), dim3(64), 0, 0, dk, ds, passes);
    CHECK(hipDeviceSynchronize());
    for (int wpc : {1, 2, 3, 4, 6, 8, 9, 10, 1}) {   /* 10: 160 KiB of S-boxes, every byte of the CU's LDS */
        const int blocks = ncu * wpc;
        float best = 1e30f;
        for (int rep = 0; rep < 3; rep++) {
            CHECK(hipEventRecord(a, 0));
            hipLaunchKernelGGL((k_time<NK, R>), dim3(blocks), dim3(64), 0, 0, dk, ds, passes);
            CHECK(hipEventRecord(b, 0));
            CHECK(hipEventSynchronize(b));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, a, b));
            best = ms < best ? ms : best;
        }
        const double pass_ns = best * 1e6 / passes;
        /* candidates/s if every CU ran 9 such chains at this pass time (R3/R4: 20 passes per candidate) */
        const double bound9 = (double)ncu * 9 * 64 / (20.0 * pass_ns * 1e-9);
        const double rate = (double)blocks * 64 / (20.0 * pass_ns * 1e-9);
        printf("{\"r\": %d, \"nk\": %d, \"waves_per_cu\": %d, \"cus\": %d, \"passes\": %d, \"ms\": %.3f, \"pass_ns\": %.1f, "
               "\"group_ns\": %.3f, \"r34_cand_per_s\": %.4g, \"r34_bound_9_chains_at_this_latency\": %.4g}\n",
               R, NK, wpc, ncu, passes, best, pass_ns, pass_ns / 128.0, rate, bound9);
    }
    CHECK(hipFree(dk)); CHECK(hipFree(ds));
}

static void ref_ksa(const uint8_t *key, int n, uint8_t S[256]) {
    for (int i = 0; i < 256; i++) S[i] = (uint8_t)i;
    uint32_t j = 0;
    for (int i = 0; i < 256; i++) {
        j = (j + S[i] + key[i % n]) & 0xffu;
        uint8_t t = S[i]; S[i] = S[j]; S[j] = t;
    }
}

template <int NK>
static int run(int blocks, int passes) {
    const size_t lanes = (size_t)blocks * 64;
    std::vector<uint32_t> keys(lanes * 4);
    uint64_t st = 0x9E3779B97F4A7C15ull ^ (uint64_t)NK;
    for (auto &w : keys) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; w = (uint32_t)st; }
    for (int q = 0; q < 4; q++) { keys[q] = 0; keys[4 + q] = 0x01010101u; }   /* lanes 0, 1: j == i collisions */
    uint32_t *dk; uint8_t *dout;
    CHECK(hipMalloc(&dk, keys.size() * 4));
    CHECK(hipMalloc(&dout, lanes * 512));
    CHECK(hipMemcpy(dk, keys.data(), keys.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemset(dout, 0, lanes * 512));
    hipLaunchKernelGGL(k_probe<NK>, dim3(blocks), dim3(64), 0, 0, dk, dout, passes);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    std::vector<uint8_t> out(lanes * 512);
    CHECK(hipMemcpy(out.data(), dout, out.size(), hipMemcpyDeviceToHost));
    CHECK(hipFree(dk)); CHECK(hipFree(dout));
    int bad_lanes[2] = {0, 0};
    std::map<int, long> pos_count[2], lane_count[2];
    long first_lane_report = 0;
    for (size_t g = 0; g < lanes; g++) {
        for (int which = 0; which < 2; which++) {
            const int x = which ? passes - 1 : 0;
            uint8_t key[16], S[256];
            for (int b = 0; b < 16; b++) key[b] = (uint8_t)(((keys[4 * g + b / 4] >> (8 * (b % 4))) & 0xffu) ^ (uint32_t)x);
            ref_ksa(key, NK, S);
            const uint8_t *o = &out[g * 512 + 256 * which];
            int nbad = 0, first = -1;
            for (int i = 0; i < 256; i++)
                if (o[i] != S[i]) { nbad++; pos_count[which][i]++; if (first < 0) first = i; }
            if (nbad) {
                bad_lanes[which]++;
                lane_count[which][(int)(g % 64)]++;
                if (first_lane_report < 4) {
                    first_lane_report++;
                    printf("  NK=%d lane %zu (wave lane %zu) pass %d: %d positions differ, first S[%d] = %d want %d\n",
                           NK, g, g % 64, x, nbad, first, o[first], S[first]);
                }
            }
        }
    }
    for (int which = 0; which < 2; which++) {
        printf("NK=%d pass %d: %d of %zu lanes wrong", NK, which ? passes - 1 : 0, bad_lanes[which], lanes);
        if (bad_lanes[which]) {
            printf("; positions (count):");
            int shown = 0;
            for (auto &kv : pos_count[which]) { if (shown++ < 40) printf(" %d(%ld)", kv.first, kv.second); }
            printf("%s; rows:", shown > 40 ? " ..." : "");
            std::map<int, long> rows;
            for (auto &kv : pos_count[which]) rows[kv.first >> 2] += kv.second;
            for (auto &kv : rows) printf(" %d", kv.first);
            printf("; wave lanes hit: %zu", lane_count[which].size());
        }
        printf("\n");
    }
    return bad_lanes[0] + bad_lanes[1];
}

int main(int argc, char **argv) {
    if (argc > 1 && !strcmp(argv[1], "tenth")) {         /* rc4_ksa_probe tenth [passes] [quarter passes] */
        const int passes = argc > 2 ? atoi(argv[2]) : 2000;
        const int qpasses = argc > 3 ? atoi(argv[3]) : 600;
        if (passes < 1 || passes > 100000 || qpasses < 1 || qpasses > 100000) { printf("bad args\n"); return 2; }
        time_tenth(passes, qpasses);
        return 0;
    }
    if (argc > 1 && !strcmp(argv[1], "time2")) {         /* rc4_ksa_probe time2 [passes] */
        const int passes = argc > 2 ? atoi(argv[2]) : 4000;
        if (passes < 1 || passes > 100000) { printf("bad args\n"); return 2; }
        time_passes2<16, 3>(passes);
        time_passes2<5, 2>(passes);
        return 0;
    }
    if (argc > 1 && !strcmp(argv[1], "time")) {          /* rc4_ksa_probe time [passes] */
        const int passes = argc > 2 ? atoi(argv[2]) : 4000;
        if (passes < 1 || passes > 100000) { printf("bad args\n"); return 2; }
        time_passes<16, 3>(passes);
        time_passes<5, 3>(passes);
        time_passes<5, 2>(passes);
        return 0;
    }
    const int blocks = argc > 1 ? atoi(argv[1]) : 4608;   /* 2 generations of 9 waves on 256 CUs */
    const int passes = argc > 2 ? atoi(argv[2]) : 20;
    if (blocks < 1 || blocks > 65536 || passes < 1 || passes > 256) { printf("bad args\n"); return 2; }
    const int bad = run<16>(blocks, passes) + run<5>(blocks, passes);
    printf("%s\n", bad ? "PROBE: WRONG S-BOXES" : "PROBE: all S-boxes == RC4");
    return bad ? 1 : 0;
}
