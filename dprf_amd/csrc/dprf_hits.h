/* dprf_hits.h -- the lowest-hit protocol of the verification kernels (device side).
 *
 * The reference stops every worker at its next candidate once one of them has found the password
 * (brute_force.py:111-114, :140-147: `found` is a shared Value every worker polls).  Here a hit lowers the
 * call's lowest-hit index on its device (dprf_results.first, atomicMin), and with stop_on_first a kernel block --
 * or, in the persistent R6 kernel, a candidate start -- is skipped when its lowest index lies above the lowest
 * hit known.  Every value either word ever holds is ~0 or the index of a candidate that verified, so a block
 * skipped above it can never hold the answer (the lowest verifying index), whatever order things happen in.
 *
 * Across devices (round 6): a multi-device call with stop_on_first hands every launch two host-mapped words
 * (fine-grained pinned host memory, dprf_host.cpp call_watch): `hit_mirror`, this device lane's own, which a hit
 * lowers with a plain system-scope store (a racing store of a higher hit can overwrite it: still a verified
 * index, see above), and `xfirst`, the lowest hit any device has reported, which a host thread keeps as the
 * minimum over every lane's mirror.  Kernels read xfirst beside their own device's `first`, so the launches
 * already running on the other GPUs skip their blocks above a hit within the host thread's poll interval instead
 * of at their next launch.  No atomics reach host memory (plain loads and stores only). */
#ifndef DPRF_HITS_H
#define DPRF_HITS_H
#include <hip/hip_runtime.h>
#include "dprf_params.h"

/* The lowest hit index this launch knows of: its device's, and with a cross-device word the call's. */
__device__ __forceinline__ unsigned long long lowest_known(const dprf_enum &e, dprf_results *R) {
    unsigned long long f = __hip_atomic_load(&R->first, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (e.xfirst) {
        const unsigned long long x = __hip_atomic_load(e.xfirst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        f = x < f ? x : f;
    }
    return f;
}

/* Record a verified candidate: the device hit list, the device's lowest hit and -- multi-device -- the lane's
 * host mirror. */
__device__ __forceinline__ void report_hit(const dprf_enum &e, dprf_results *R, unsigned long long idx, uint32_t cap,
                                           uint32_t stop_on_first) {
    const uint32_t slot = atomicAdd(&R->nhits, 1u);
    if (slot < cap) R->hits[slot] = idx;
    atomicMin(&R->first, idx);
    if (stop_on_first) atomicExch(&R->stop, 1u);
    if (e.hit_mirror && idx < __hip_atomic_load(e.hit_mirror, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))
        __hip_atomic_store(e.hit_mirror, idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
#endif
