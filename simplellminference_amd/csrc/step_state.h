// step_state.h — the device-resident decode state that lets one captured hipGraph serve every step
// (the reference keeps token and position on the host: model.cpp:157-183, emb_kernel.cu:15).
#pragma once
#include "common.h"

namespace sli {

struct DevState {
    int32_t pos;          // position of the token being fed
    int32_t token;        // token fed at pos
    int32_t n_forced;     // prompt length (teacher forcing while pos < n_forced)
    int32_t last_argmax;  // greedy argmax of the last step's logits
    int32_t advance;      // 1: finalize advances pos/token; 0: idempotent step (bench)
    int32_t error;        // device-side error bits: kOsErrTimeout (oneshot.h), kAttnErrHand (attention.h);
                          // checked by every predict path
    unsigned long long key;  // argmax key of the last step (0 between steps)
};

// model.cpp:157-183: next position; teacher-forced prompt token while inside the prompt, else greedy.
__device__ __forceinline__ void finalize_state(DevState* st, const int32_t* prompt, int32_t* hist, int T) {
    const unsigned long long k = st->key;
    const int next = (int)argmax_key_index(k);
    st->last_argmax = next;
    st->key = 0;
    if (st->advance) {
        const int p = st->pos + 1;
        if (p < T) {
            st->pos = p;
            st->token = p < st->n_forced ? prompt[p] : next;
            hist[p] = st->token;
        }
    }
}

}  // namespace sli
