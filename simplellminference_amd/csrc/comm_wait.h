// comm_wait.h — a host wait on the engine stream that cannot outlive a wedged communicator.
//
// The reference runs one process and never waits on a peer; its decode loop syncs once per token at the
// logits copy (source/model/model.cpp:175-179). Under tensor parallelism our step graph holds RCCL all-reduces
// where model.cpp has none (the two per layer that replace the reference's local wo / down outputs,
// model.cpp:86-90, 124-128) — a peer that dies or a communicator that faults would leave hipStreamSynchronize
// blocked forever, and the node's bench with it. So every host wait of a rank with RCCL collectives polls
// instead: the stream (or event) query, ncclCommGetAsyncError, and a deadline, and returns an error code when
// either the communicator reports one or the deadline expires. The caller then aborts the communicator
// (ncclCommAbort) so nothing of it is left waiting, and the process exits with that code.
//
// The policy is a template over its three probes so that it can be driven by mocks on a CPU
// (sli_debug_bounded_wait, tests/test_comm_wait.py) — a query that never completes must end in
// SLI_ERR_TIMEOUT, an async error in SLI_ERR_COMM, a failed query in SLI_ERR_HIP.
#pragma once
#include <chrono>
#include <cstdlib>
#include <string>
#include <thread>

#include "sli.h"

namespace sli {

// SLI_COMM_TIMEOUT_MS (default 120 s): the longest a rank waits on a stream that carries collectives. A C2 step
// is ~3 ms and the slowest legitimate wait (a 2048-token prefill under TP) well under a second, so 120 s only ever
// expires on a wedged peer, long before a driver's job limit.
inline double comm_timeout_ms() {
    const char* e = std::getenv("SLI_COMM_TIMEOUT_MS");
    const double v = e ? std::atof(e) : 0.0;
    return v > 0.0 ? v : 120000.0;
}

enum class WaitPoll { Done, Pending, Failed };

// query() -> WaitPoll; async_error() -> true (and a message) when the communicator reports an error;
// now_ms() -> a monotonic clock. Spins for the first millisecond (a step's tail should not pay a sleep), then
// polls every 50 us.
template <class Query, class AsyncError, class NowMs>
int bounded_wait(Query query, AsyncError async_error, NowMs now_ms, double deadline_ms, std::string& why,
                 bool sleep = true) {
    const double t0 = now_ms();
    for (long long it = 0;; ++it) {
        const WaitPoll p = query();
        if (p == WaitPoll::Done) return SLI_OK;
        if (p == WaitPoll::Failed) {
            why = "stream query failed";
            return SLI_ERR_HIP;
        }
        std::string msg;
        if (async_error(msg)) {
            why = "communicator error: " + msg;
            return SLI_ERR_COMM;
        }
        const double waited = now_ms() - t0;
        if (waited > deadline_ms) {
            why = "no progress for " + std::to_string((long long)waited) + " ms (SLI_COMM_TIMEOUT_MS " +
                  std::to_string((long long)deadline_ms) + "): a peer or the communicator is wedged";
            return SLI_ERR_TIMEOUT;
        }
        if (sleep && waited > 1.0) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

inline double steady_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace sli
