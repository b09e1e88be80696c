// oneshot.h — one-shot all-reduce between the tensor-parallel ranks of one node over xGMI (SURVEY.md §5
// "Distributed communication backend", §8(e) upgrade): the decode step's two residual all-reduces per
// layer move B*D fp32 values (16 KiB at batch 1), which is latency-bound; a ring (RCCL) pays 2(N-1)
// dependent hops, the one-shot form one.
//
// Every rank owns a comm buffer in uncached device memory (hipDeviceMallocUncached), exported by IPC
// and mapped by every peer:
//   flags [2][kOsMaxRanks] u32        flag[par][r] = epoch: rank r's contribution for that epoch is in
//   data  [2][kOsMaxRanks][nmax] f32  data[par][r]: rank r's partial
// One call of epoch e (par = e & 1): each rank PUSHES its partial into data[par][rank] of every rank
// (itself included), drains, then sets flag[par][rank] = e on every rank with a system-scope release;
// then it waits (bounded) until its own flags[par][*] all read e (system-scope acquire) and reduces
// data[par][0 .. N-1] IN RANK ORDER (every rank computes bit-identical x). Double buffering by epoch
// parity makes the reuse of a slot safe: rank r writes a peer's slot of parity p again only at epoch
// e + 2, after it has seen that peer's flag for e + 1, which the peer raises only once its epoch-e
// reduction (the last read of the slot) has finished. The epoch is a device counter each rank advances
// identically (one thread of every call), so the captured graph replays it.
#pragma once
#include "common.h"
#include "step_state.h"

namespace sli {

constexpr int kOsMaxRanks = 8;
constexpr unsigned kOsSpinLimit = 1u << 24;  // bounded wait (~seconds): gives up with DevState::error bit 4
constexpr int kOsErrTimeout = 4;

struct OneShotArgs {
    char* peers[kOsMaxRanks];  // every rank's comm buffer, mapped in this process (own one included)
    int rank, nranks;
    int n;                     // elements of this call (floats; u64 keys count as 2)
    int nmax;                  // data slot capacity in floats
    const float* src;          // this rank's partial
    float* dst;                // the reduced result
    unsigned* epoch;           // this rank's call counter (plain device memory)
    DevState* st;              // error reporting
};

__device__ __forceinline__ unsigned* os_flag(char* buf, int par, int r) {
    return reinterpret_cast<unsigned*>(buf) + par * kOsMaxRanks + r;
}
__device__ __forceinline__ float* os_data(char* buf, int par, int r, int nmax) {
    return reinterpret_cast<float*>(buf + 256) + ((size_t)par * kOsMaxRanks + r) * nmax;
}

// OP 0: sum of fp32; OP 1: max of u64 (argmax keys, two floats per element)
template <int OP>
__global__ void __launch_bounds__(1024) oneshot_kernel(OneShotArgs a) {
    const unsigned e = *a.epoch + 1;  // (the previous call's write: stream-ordered)
    const int par = (int)(e & 1u);
    const int tid = threadIdx.x;
    const int n4 = a.n >> 2;  // fp32 sums: n is a multiple of 4 (B * D)
    // push my partial to every rank (fp32 sums as 16-byte stores; u64 keys one element each)
    for (int p = 0; p < a.nranks; ++p) {
        if constexpr (OP == 0) {
            const float4* s4 = reinterpret_cast<const float4*>(a.src);
            float4* d4 = reinterpret_cast<float4*>(os_data(a.peers[p], par, a.rank, a.nmax));
            for (int i = tid; i < n4; i += blockDim.x) d4[i] = s4[i];
        } else {
            const unsigned long long* s8 = reinterpret_cast<const unsigned long long*>(a.src);
            unsigned long long* d8 = reinterpret_cast<unsigned long long*>(os_data(a.peers[p], par, a.rank, a.nmax));
            for (int i = tid; i < (a.n >> 1); i += blockDim.x) d8[i] = s8[i];
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid < a.nranks)
        __hip_atomic_store(os_flag(a.peers[tid], par, a.rank), e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    // wait for every rank's contribution in my own buffer
    __shared__ int abort;
    if (tid == 0) abort = 0;
    __syncthreads();
    if (tid < a.nranks) {
        unsigned* f = os_flag(a.peers[a.rank], par, tid);
        for (unsigned spins = 0; __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != e; ++spins) {
            if (spins >= kOsSpinLimit) {
                __hip_atomic_fetch_or(&a.st->error, kOsErrTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                abort = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
    if (abort) {
        // stay in step with the peers that did not time out (they advance the epoch), and make the stale
        // result loud: NaN instead of the previous call's values (DevState::error already records it)
        if constexpr (OP == 0)
            for (int i = tid; i < a.n; i += blockDim.x) a.dst[i] = __builtin_nanf("");
        if (tid == 0) *a.epoch = e;
        return;
    }
    char* mine = a.peers[a.rank];
    if constexpr (OP == 0) {
        for (int i = tid; i < n4; i += blockDim.x) {
            float4 acc = reinterpret_cast<const float4*>(os_data(mine, par, 0, a.nmax))[i];
            for (int r = 1; r < a.nranks; ++r) {  // rank order: every rank adds identically
                const float4 v = reinterpret_cast<const float4*>(os_data(mine, par, r, a.nmax))[i];
                acc.x += v.x;
                acc.y += v.y;
                acc.z += v.z;
                acc.w += v.w;
            }
            reinterpret_cast<float4*>(a.dst)[i] = acc;
        }
    } else {
        const int nk = a.n >> 1;
        for (int i = tid; i < nk; i += blockDim.x) {
            unsigned long long b = 0;
            for (int r = 0; r < a.nranks; ++r) {
                const unsigned long long k = reinterpret_cast<const unsigned long long*>(os_data(mine, par, r, a.nmax))[i];
                b = k > b ? k : b;
            }
            reinterpret_cast<unsigned long long*>(a.dst)[i] = b;
        }
    }
    if (tid == 0) *a.epoch = e;
}

}  // namespace sli
