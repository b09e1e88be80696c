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
#include "bgemm.h"
#include "gemv.h"
#include "step_state.h"

namespace sli {

constexpr int kOsMaxRanks = 8;
constexpr unsigned kOsSpinLimit = 1u << 24;  // bounded wait (~seconds): gives up with DevState::error bit 4
constexpr int kOsErrTimeout = 4;
// A wait that has spun 4096 times looks at DevState::error: once one exchange of this process gave up (a peer that
// never arrives), every later one gives up at once instead of after its own kOsSpinLimit — a broken exchange then
// costs one timeout, not one per launch (bench.py's RCCL validation falls back within seconds).
__device__ __forceinline__ bool os_gave_up(DevState* st, unsigned spins) {
    return (spins & 4095u) == 4095u &&
           (__hip_atomic_load(&st->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) & kOsErrTimeout) != 0;
}
// Per-workgroup exchanges (EpiPush::wg_mode, oneshot_sliced_kernel): flags [region 3][par 2][kOsMaxWg][kOsMaxRanks]
// u32 after the 256-B header of the launch-level flags, then the data blocks of 8 slots x nmax floats: launch-level
// par 0 / 1, then region 0 (batch-1 wo) par 0 / 1, region 1 (batch-1 down), region 2 (the sliced launch), region 3
// (batched wo, BgEpiPush), region 4 (batched down). Per-workgroup epochs live in device memory,
// [kOsRegions][kOsMaxWg].
constexpr int kOsMaxWg = 512;
constexpr int kOsRegions = 5;
constexpr size_t kOsDataOff = 256 + sizeof(unsigned) * kOsRegions * 2 * kOsMaxWg * kOsMaxRanks;
// after the data blocks: the persistent layer stack's exchange granules (tp_layers.h), 8-byte {value, tag} per row,
// [region 2][kOsMaxRanks][nmax]
inline size_t os_gran_off(int nmax) { return kOsDataOff + sizeof(float) * (2 + 2 * kOsRegions) * (size_t)kOsMaxRanks * nmax; }
inline size_t os_buffer_bytes(int nmax) { return os_gran_off(nmax) + 8 * 2 * (size_t)kOsMaxRanks * nmax; }

struct OneShotArgs {
    char* peers[kOsMaxRanks];  // every rank's comm buffer, mapped in this process (own one included)
    int rank, nranks;
    int n;                     // elements of this call (floats; u64 keys count as 2)
    int nmax;                  // data slot capacity in floats
    const float* src;          // this rank's partial
    float* dst;                // the reduced result
    unsigned* epoch;           // this rank's call counter (plain device memory)
    DevState* st;              // error reporting
    int loopback = 0;          // debug (one process, SLI_DEBUG_OS_LOOPBACK): every peer is this rank's own buffer
                               // and the rank raises every rank's flag (timing of the exchange without peers)
};

__device__ __forceinline__ unsigned* os_flag(char* buf, int par, int r) {
    return reinterpret_cast<unsigned*>(buf) + par * kOsMaxRanks + r;
}
__device__ __forceinline__ float* os_data(char* buf, int par, int r, int nmax) {
    return reinterpret_cast<float*>(buf + kOsDataOff) + ((size_t)par * kOsMaxRanks + r) * nmax;
}
__device__ __forceinline__ unsigned* os_wg_flag(char* buf, int region, int par, int wg, int r) {
    return reinterpret_cast<unsigned*>(buf + 256) + ((size_t)(region * 2 + par) * kOsMaxWg + wg) * kOsMaxRanks + r;
}
__device__ __forceinline__ float* os_wg_data(char* buf, int region, int par, int r, int nmax) {
    return reinterpret_cast<float*>(buf + kOsDataOff) + ((size_t)(2 + region * 2 + par) * kOsMaxRanks + r) * nmax;
}

// Flags, bounded wait and the rank-order reduction of epoch e, by threads [0, nthr) of ONE workgroup
// whose pushes (and, in the fused form, every pushing workgroup's) have drained: raise flag[par][rank] on
// every rank (system-scope release), wait until this rank's flags[par][*] all read e (system-scope
// acquire, bounded), reduce data[par][0 .. N-1] in rank order into dst, advance the epoch.
// peers: the ranks' buffers, indexed by a runtime rank — the kernel-argument array, or a device-memory table
// (a runtime index into a struct held in a per-thread copy, as the GEMV epilogues are, would put the whole
// struct in scratch memory)
// SLI_OS_FENCE=0: relaxed flag store / poll here too (every comm-buffer access is uncached and drained first,
// as in EpiPush::finish_wg); 1 (default): system-scope release / acquire.
#ifndef SLI_OS_FENCE
#define SLI_OS_FENCE 1
#endif
template <int OP>
__device__ __forceinline__ void os_finish(const OneShotArgs& a, char* const* peers, unsigned e, int* abort_lds) {
    constexpr int kRel = SLI_OS_FENCE ? __ATOMIC_RELEASE : __ATOMIC_RELAXED;
    constexpr int kAcq = SLI_OS_FENCE ? __ATOMIC_ACQUIRE : __ATOMIC_RELAXED;
    const int par = (int)(e & 1u);
    const int tid = threadIdx.x, nthr = blockDim.x;
    if (tid < a.nranks)
        __hip_atomic_store(os_flag(peers[tid], par, a.loopback ? tid : a.rank), e, kRel, __HIP_MEMORY_SCOPE_SYSTEM);
    if (tid == 0) *abort_lds = 0;
    __syncthreads();
    if (tid < a.nranks) {
        unsigned* f = os_flag(peers[a.rank], par, tid);
        for (unsigned spins = 0; __hip_atomic_load(f, kAcq, __HIP_MEMORY_SCOPE_SYSTEM) != e; ++spins) {
            if (spins >= kOsSpinLimit || os_gave_up(a.st, spins)) {
                __hip_atomic_fetch_or(&a.st->error, kOsErrTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                *abort_lds = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
    if (*abort_lds) {
        // stay in step with the peers that did not time out (they advance the epoch), and make the stale
        // result loud: NaN instead of the previous call's values (DevState::error already records it)
        if constexpr (OP == 0)
            for (int i = tid; i < a.n; i += nthr) a.dst[i] = __builtin_nanf("");
        if (tid == 0) *a.epoch = e;
        return;
    }
    char* mine = peers[a.rank];
    if constexpr (OP == 0) {
        const int n4 = a.n >> 2;  // fp32 sums: n is a multiple of 4 (B * D)
        for (int i = tid; i < n4; i += nthr) {
            float4 v[kOsMaxRanks];  // every rank's slot in flight at once (one round trip), then summed
#pragma unroll
            for (int r = 0; r < kOsMaxRanks; ++r)
                v[r] = reinterpret_cast<const float4*>(os_data(mine, par, min(r, a.nranks - 1), a.nmax))[i];
            float4 acc = v[0];
#pragma unroll
            for (int r = 1; r < kOsMaxRanks; ++r) {  // rank order: every rank adds identically
                if (r < a.nranks) {
                    acc.x += v[r].x;
                    acc.y += v[r].y;
                    acc.z += v[r].z;
                    acc.w += v[r].w;
                }
            }
            reinterpret_cast<float4*>(a.dst)[i] = acc;
        }
    } else {
        const int nk = a.n >> 1;
        for (int i = tid; i < nk; i += nthr) {
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
    __shared__ int abort;
    os_finish<OP>(a, a.peers, e, &abort);
}

// The separate one-shot sum sliced over workgroups (region 2): workgroup w of every rank owns the same slice of the
// n floats; it pushes its slice of the partial into slot [rank] of every rank, raises flag[2][par][w][rank] on
// every rank (relaxed: every comm-buffer access is uncached and the pushes have drained), waits (bounded) for the
// N flags of w in its own buffer and sums its slice of the N slots in rank order into dst. A single summing
// workgroup moved N x B*D floats each way alone: 33 us per exchange at batch 8 (Llama-3-8B TP 8, loopback).
// Every workgroup waits for the same workgroup of the peers, so the grid is small (kOsSliceWgs, 256 threads
// each): ranks sharing one device (tests) still find room on the CUs for each other's workgroups.
constexpr int kOsSliceWgs = 64;
__global__ void __launch_bounds__(256) oneshot_sliced_kernel(OneShotArgs a, char* const* peer_tab, unsigned* wg_epoch) {
    const int w = blockIdx.x, nw = gridDim.x, tid = threadIdx.x;
    const unsigned e = wg_epoch[2 * kOsMaxWg + w] + 1;  // this workgroup index's previous sliced exchange
    const int par = (int)(e & 1u);
    const int n4 = a.n >> 2;  // fp32 sums: n is a multiple of 4 (B * D)
    const int i0 = (int)(((long long)w * n4) / nw), i1 = (int)(((long long)(w + 1) * n4) / nw);
    const float4* s4 = reinterpret_cast<const float4*>(a.src);
    for (int p = 0; p < a.nranks; ++p) {
        float4* d4 = reinterpret_cast<float4*>(os_wg_data(peer_tab[p], 2, par, a.rank, a.nmax));
        for (int i = i0 + tid; i < i1; i += blockDim.x) d4[i] = s4[i];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every pushing wave drains before the flags
    __syncthreads();
    __shared__ int abort;
    if (tid < a.nranks)
        __hip_atomic_store(os_wg_flag(peer_tab[tid], 2, par, w, a.loopback ? tid : a.rank), e, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    if (tid == 0) abort = 0;
    __syncthreads();
    if (tid < a.nranks) {
        const unsigned* f = os_wg_flag(peer_tab[a.rank], 2, par, w, tid);
        for (unsigned spins = 0; __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != e; ++spins) {
            if (spins >= kOsSpinLimit || os_gave_up(a.st, spins)) {
                __hip_atomic_fetch_or(&a.st->error, kOsErrTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                abort = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
    char* mine = peer_tab[a.rank];
    for (int i = i0 + tid; i < i1; i += blockDim.x) {
        float4 v[kOsMaxRanks];  // every rank's slot in flight at once, then summed in rank order
#pragma unroll
        for (int r = 0; r < kOsMaxRanks; ++r)
            v[r] = reinterpret_cast<const float4*>(os_wg_data(mine, 2, par, min(r, a.nranks - 1), a.nmax))[i];
        float4 acc = v[0];
#pragma unroll
        for (int r = 1; r < kOsMaxRanks; ++r) {
            if (r < a.nranks) {
                acc.x += v[r].x;
                acc.y += v[r].y;
                acc.z += v[r].z;
                acc.w += v[r].w;
            }
        }
        if (abort) acc = float4{__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf("")};
        reinterpret_cast<float4*>(a.dst)[i] = acc;
    }
    if (tid == 0) wg_epoch[2 * kOsMaxWg + w] = e;
}

// The batched (bgemm) wo / down with the exchange per group (SLI_ALLREDUCE_FUSED_WG, batch > 1): group g of every
// rank owns the same tiles, so its rows (x [B][D]: row r of every sequence b) are the same on every rank. The
// group's final stores go into slot [rank] of every rank (rank 0: plus the residual) instead of xpart; its
// finishing workgroup drains them, raises flag[region][par][g][rank] on every rank (relaxed: uncached, drained),
// waits (bounded) for the N flags of g and sums its rows' N slots in rank order into x. Regions 3 (wo) and 4
// (down); epochs per (region, group).
struct BgEpiPush {
    const float* resid;  // rank 0: the residual stream x [B][D]; other ranks nullptr
    OneShotArgs os;      // dst = x, n = B * D, nmax
    char* const* peer_tab;
    unsigned* wg_epoch;  // [kOsRegions][kOsMaxWg]
    int region;
    int nrows, ld, B, tpw, ntiles;
    __device__ int row(int t, int i) const { return min(t * 16 + i, nrows - 1); }
    __device__ void pre_a(int, int, int) {}
    __device__ void pre_b() {}
    __device__ unsigned epoch(int g) const { return wg_epoch[region * kOsMaxWg + g] + 1; }
    __device__ void one(int row, int b, float v, int par) const {
        if (row >= nrows) return;
        const size_t o = (size_t)b * ld + row;
        const float a = resid ? resid[o] + v : v;  // add_kernel.cpp:5-14, once (rank 0)
#pragma unroll
        for (int p = 0; p < kOsMaxRanks; ++p)
            if (p < os.nranks) os_wg_data(os.peers[p], region, par, os.rank, os.nmax)[o] = a;
    }
    // the group index is not passed to store(): the epoch parity comes from the tile's group (t / tpw)
    __device__ void store(int t, int i, int b, float v0, float v1, unsigned long long*) const {
        const int par = (int)(epoch(t / tpw) & 1u);
        one(t * 16 + i, b, v0, par);
        one(t * 16 + i + 8, b, v1, par);
    }
    __device__ void finish(unsigned long long* kl, int g, int) const {
        const int tid = threadIdx.x;
        const unsigned e = epoch(g);
        const int par = (int)(e & 1u);
        int* abort_lds = reinterpret_cast<int*>(kl + 10);  // bgemm scratch past the keys and the split flag
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every pushing wave drains before the flags
        __syncthreads();
        if (tid < os.nranks)
            __hip_atomic_store(os_wg_flag(peer_tab[tid], region, par, g, os.loopback ? tid : os.rank), e, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        if (tid == 0) *abort_lds = 0;
        __syncthreads();
        if (tid < os.nranks) {
            const unsigned* f = os_wg_flag(peer_tab[os.rank], region, par, g, tid);
            for (unsigned spins = 0; __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != e; ++spins) {
                if (spins >= kOsSpinLimit || os_gave_up(os.st, spins)) {
                    __hip_atomic_fetch_or(&os.st->error, kOsErrTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    *abort_lds = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
        const int t0 = g * tpw, ntg = min(tpw, ntiles - t0);
        const int nr = min(ntg * 16, nrows - t0 * 16);  // the group's rows (the last tile may be partial)
        char* mine = peer_tab[os.rank];
        for (int it = tid; it < nr * B; it += blockDim.x) {
            const int b = it / nr, row = t0 * 16 + (it - b * nr);
            const size_t o = (size_t)b * ld + row;
            float v[kOsMaxRanks];  // every rank's slot in flight at once, then summed in rank order
#pragma unroll
            for (int r = 0; r < kOsMaxRanks; ++r) v[r] = os_wg_data(mine, region, par, min(r, os.nranks - 1), os.nmax)[o];
            float acc = v[0];
#pragma unroll
            for (int r = 1; r < kOsMaxRanks; ++r)
                if (r < os.nranks) acc += v[r];
            os.dst[o] = *abort_lds ? __builtin_nanf("") : acc;
        }
        if (tid == 0) wg_epoch[region * kOsMaxWg + g] = e;
    }
};

// The residual all-reduce fused into the row-parallel GEMV that produces the partial (wo, down; batch 1):
// the epilogue pushes each finished row sum (rank 0: plus the residual) straight into slot [rank] of every
// rank's comm buffer instead of a local partial; every workgroup drains its pushes and counts its arrival,
// and the last workgroup to arrive runs os_finish (flags, bounded wait, rank-order sum into x, epoch). The
// separate oneshot launch and its kernel boundary disappear; the next launch reads x as usual. Only one
// workgroup per rank ever waits, so ranks that share a device cannot starve each other of CUs.
// Epilogue contract: gemv.h (units / rows / prefetch_a / prefetch_b / store / finish).
template <int R>
struct EpiPush {
    const float* resid;  // rank 0: the residual stream x; other ranks nullptr
    const float* rscale;
    float scale;
    int nrows;
    OneShotArgs os;      // dst = x, n = nrows (batch 1)
    unsigned* arrive;    // [9] arrival counters (8 shards + top), zero between launches (last arrivers reset)
    char* const* peer_tab;  // device copy of os.peers (the last arriver's runtime-indexed flags and slots)
    // Per-workgroup mode (SLI_ALLREDUCE_FUSED_WG): every rank runs the same grid over the same rows, so
    // workgroup w of every rank owns the same rows; w pushes its rows, raises flag[region][par][w][rank] on
    // every rank, waits for the N flags of w on its own buffer and sums its rows' N slots in rank order into
    // x. No launch-wide arrival and no single summing workgroup; each workgroup keeps its own epoch
    // (wg_epoch[region][w]). Every workgroup waits, so the ranks must not share a device (or their grids must
    // fit it together: SLI_DEBUG_GEMV_MAX_BLOCKS in the one-GPU tests).
    int wg_mode = 0;
    int region = 0;              // 0: wo, 1: down (their grids map rows to workgroups differently)
    unsigned* wg_epoch = nullptr;  // [kOsRegions][kOsMaxWg]
    unsigned e = 0;
    int pre_u = -1;
    float pre_r[R] = {}, pre_s[R] = {};
    int st_u0 = -1, st_n = 0;  // wg_mode: the units this thread stored (u0, u0 + 1024, ...)
    __device__ int units() const { return (nrows + R - 1) / R; }
    __device__ void rows(int u, int* r) const {
#pragma unroll
        for (int i = 0; i < R; ++i) r[i] = min(u * R + i, nrows - 1);
    }
    __device__ void prefetch_a(int u) {
        // written by the previous all-reduce's last arriver / this workgroup index's previous exchange (earlier launches)
        e = (wg_mode ? wg_epoch[region * kOsMaxWg + blockIdx.x] : *os.epoch) + 1;
        pre_u = u;
        const float* rp = resid ? resid : rscale ? rscale : os.dst;
        const float* sp = rscale ? rscale : os.dst;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int row = min(u * R + i, nrows - 1);
            pre_r[i] = rp[row];
            pre_s[i] = sp[row];
        }
    }
    __device__ void prefetch_b(int) {}
    __device__ void store(int u, const int*, const float* v) {
        const bool pre = u == pre_u;
        const int par = (int)(e & 1u);
        if (st_u0 < 0) st_u0 = u;
        ++st_n;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int row = u * R + i;
            if (row < nrows) {
                float a = rscale ? v[i] * (pre ? pre_s[i] : rscale[row]) : v[i];
                a = a * scale;
                if (resid) a = (pre ? pre_r[i] : resid[row]) + a;  // add_kernel.cpp:5-14, once (rank 0)
#pragma unroll
                for (int p = 0; p < kOsMaxRanks; ++p)
                    if (p < os.nranks)
                        (wg_mode ? os_wg_data(os.peers[p], region, par, os.rank, os.nmax)
                                 : os_data(os.peers[p], par, os.rank, os.nmax))[row] = a;
            }
        }
    }
    // wg_mode: flags, bounded wait and the rank-order sum of this workgroup's own rows. Every access to the comm
    // buffers bypasses the caches (uncached memory), and the pushes have drained (vmcnt 0, every wave, barrier)
    // before the flag store is issued, so the flag store / poll are relaxed: a system-scope release / acquire would
    // add an L2 write-back / invalidate per workgroup and order nothing the uncached accesses need (loopback TP-8
    // rank step 1.494 -> 1.339 ms, profiles/r4_tp_fused_wg_relaxed.txt). SLI_OS_WG_FENCE=1: the fenced form.
#ifndef SLI_OS_WG_FENCE
#define SLI_OS_WG_FENCE 0
#endif
    __device__ void finish_wg(int* sh) const {
        constexpr int kRel = SLI_OS_WG_FENCE ? __ATOMIC_RELEASE : __ATOMIC_RELAXED;
        constexpr int kAcq = SLI_OS_WG_FENCE ? __ATOMIC_ACQUIRE : __ATOMIC_RELAXED;
        const int tid = threadIdx.x, par = (int)(e & 1u);
        if (tid < os.nranks)
            __hip_atomic_store(os_wg_flag(peer_tab[tid], region, par, blockIdx.x, os.loopback ? tid : os.rank), e,
                               kRel, __HIP_MEMORY_SCOPE_SYSTEM);
        if (tid == 0) sh[1] = 0;
        __syncthreads();
        if (tid < os.nranks) {
            const unsigned* f = os_wg_flag(peer_tab[os.rank], region, par, blockIdx.x, tid);
            for (unsigned spins = 0; __hip_atomic_load(f, kAcq, __HIP_MEMORY_SCOPE_SYSTEM) != e; ++spins) {
                if (spins >= kOsSpinLimit || os_gave_up(os.st, spins)) {
                    __hip_atomic_fetch_or(&os.st->error, kOsErrTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    sh[1] = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
        char* mine = peer_tab[os.rank];
        for (int k = 0; k < st_n; ++k) {
            const int u = st_u0 + k * kGemvThreads;
#pragma unroll
            for (int i = 0; i < R; ++i) {
                const int row = u * R + i;
                if (row >= nrows) continue;
                float v[kOsMaxRanks];  // every rank's slot in flight at once, then summed in rank order
#pragma unroll
                for (int r = 0; r < kOsMaxRanks; ++r)
                    v[r] = os_wg_data(mine, region, par, min(r, os.nranks - 1), os.nmax)[row];
                float acc = v[0];
#pragma unroll
                for (int r = 1; r < kOsMaxRanks; ++r)
                    if (r < os.nranks) acc += v[r];
                os.dst[row] = sh[1] ? __builtin_nanf("") : acc;  // a timed-out wait: loud, not stale
            }
        }
        if (tid == 0) wg_epoch[region * kOsMaxWg + blockIdx.x] = e;
    }
    __device__ void finish(float* smem) const {
        int* sh = reinterpret_cast<int*>(smem) + 40;  // [0]: last arriver, [1]: abort (gemv LDS head)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every pushing wave drains before the arrival
        __syncthreads();
        if (wg_mode) {
            finish_wg(sh);
            return;
        }
        if (threadIdx.x == 0) {  // two-level arrival: a shard per blockIdx % 8 (an XCD under round-robin
                                 // placement: speed only), then the shards' last arrivers on arrive[8]
            const unsigned g = gridDim.x, sd = blockIdx.x & 7u;
            const unsigned nsh = g < 8u ? g : 8u, cnt = (g - sd + 7u) >> 3;
            int last = 0;
            if (__hip_atomic_fetch_add(arrive + sd, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == cnt - 1u) {
                __hip_atomic_store(arrive + sd, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (__hip_atomic_fetch_add(arrive + 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsh - 1u) {
                    __hip_atomic_store(arrive + 8, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    last = 1;
                }
            }
            sh[0] = last;
        }
        __syncthreads();
        if (!sh[0]) return;  // uniform
        os_finish<0>(os, peer_tab, e, sh + 1);
    }
};

}  // namespace sli
