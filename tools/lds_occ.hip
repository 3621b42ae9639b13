/* How many one-wave workgroups with B bytes of LDS each are resident per CU at once (gfx950)?
 * Each wave spins ~200 us, records its CU id and realtime start/end; the host reports the max overlap. */
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
template <int B>
__global__ void __launch_bounds__(64) k_spin(unsigned long long *rec, int *sink) {
    __shared__ uint8_t S[B];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    S[threadIdx.x * 4] = (uint8_t)threadIdx.x;
    unsigned long long t = t0;
    while (t - t0 < 20000ull) t = __builtin_amdgcn_s_memrealtime();   /* 200 us at 100 MHz */
    if (S[(threadIdx.x * 7) % B] == 255) sink[0] = 1;
    if (threadIdx.x == 0) {
        rec[3 * blockIdx.x] = ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) | __builtin_amdgcn_s_getreg((31 << 11) | 4);
        rec[3 * blockIdx.x + 1] = t0;
        rec[3 * blockIdx.x + 2] = __builtin_amdgcn_s_memrealtime();
    }
}
template <int B>
int probe(int nblk, unsigned long long *drec, int *sink) {
    hipLaunchKernelGGL(k_spin<B>, dim3(nblk), dim3(64), 0, 0, drec, sink);
    CHECK(hipDeviceSynchronize());
    std::vector<unsigned long long> rec(3 * nblk);
    CHECK(hipMemcpy(rec.data(), drec, rec.size() * 8, hipMemcpyDeviceToHost));
    std::vector<std::vector<std::pair<unsigned long long, int>>> ev(8 * 8 * 2 * 16);
    for (int w = 0; w < nblk; w++) {
        unsigned long long id = rec[3 * w];
        unsigned hw = (unsigned)id, xcc = (unsigned)(id >> 32) & 7u;
        size_t key = ((xcc * 8 + ((hw >> 13) & 7u)) * 2 + ((hw >> 12) & 1u)) * 16 + ((hw >> 8) & 15u);
        ev[key].push_back({rec[3 * w + 1], 1});
        ev[key].push_back({rec[3 * w + 2], -1});
    }
    int mx = 0, mn = 1 << 30, ncu = 0;
    for (auto &e : ev) {
        if (e.empty()) continue;
        std::sort(e.begin(), e.end(), [](auto &a, auto &b) { return a.first < b.first || (a.first == b.first && a.second < b.second); });
        int c = 0, m = 0;
        for (auto &p : e) { c += p.second; m = std::max(m, c); }
        mx = std::max(mx, m); mn = std::min(mn, m); ncu++;
    }
    printf("LDS %6d B per one-wave workgroup: %d CUs, resident per CU min %d max %d\n", B, ncu, mn, mx);
    return 0;
}
int main() {
    const int nblk = 256 * 24;
    unsigned long long *drec; int *sink;
    CHECK(hipMalloc(&drec, 3 * 8 * nblk)); CHECK(hipMalloc(&sink, 4));
    probe<16384>(nblk, drec, sink); probe<16256>(nblk, drec, sink); probe<16208>(nblk, drec, sink); probe<16128>(nblk, drec, sink); probe<16000>(nblk, drec, sink); probe<15872>(nblk, drec, sink);
    probe<15360>(nblk, drec, sink); probe<14848>(nblk, drec, sink); probe<13312>(nblk, drec, sink);
    probe<8192>(nblk, drec, sink); probe<1024>(nblk, drec, sink);
    return 0;
}
