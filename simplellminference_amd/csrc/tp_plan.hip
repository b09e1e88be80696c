// tp_plan.hip — the tensor-parallel shard plan (include/sli.h sli_tp_plan / sli_tp_vocab), host only.
// The engine places weights with it and the CPU tests (tests/test_tp_gloo.py) slice the oracle's
// weights with it, so the sharding the GPU runs is the sharding the gloo tests check.
#include "../../include/sli_synth.h"
#include "common.h"

extern "C" {

int sli_tp_vocab(const sli_model_config* c, int32_t* vocab_lo, int32_t* vocab_n) {
    SLI_CHECK(c && vocab_lo && vocab_n, SLI_ERR_ARG, "sli_tp_vocab: null");
    SLI_CHECK(c->tp_size >= 1 && c->tp_rank >= 0 && c->tp_rank < c->tp_size, SLI_ERR_ARG, "bad tp rank/size");
    const int chunk = (c->vocab + c->tp_size - 1) / c->tp_size;
    const int lo = c->tp_rank * chunk;
    *vocab_lo = lo;
    *vocab_n = lo < c->vocab ? (c->vocab - lo < chunk ? c->vocab - lo : chunk) : 0;
    return SLI_OK;
}

int sli_tp_plan(const sli_model_config* c, int32_t kind, sli_shard_window* w) {
    SLI_CHECK(c && w, SLI_ERR_ARG, "sli_tp_plan: null");
    const int N = c->tp_size, r = c->tp_rank;
    SLI_CHECK(N >= 1 && r >= 0 && r < N, SLI_ERR_ARG, "bad tp rank/size");
    SLI_CHECK(c->n_heads % N == 0 && c->n_kv_heads % N == 0 && c->ffn % N == 0, SLI_ERR_SHAPE,
              "heads, kv heads and ffn must divide by tp_size");
    const int D = c->dim, hd = c->head_dim, I = c->ffn;
    const int qr = c->n_heads / N * hd, kr = c->n_kv_heads / N * hd, Il = I / N;
    auto set = [&](int row_lo, int n_rows, int col_lo, int n_cols, int full_cols, int dst) {
        w->row_lo = row_lo;
        w->n_rows = n_rows;
        w->col_lo = col_lo;
        w->n_cols = n_cols;
        w->full_cols = full_cols;
        w->dst_row_off = dst;
        return SLI_OK;
    };
    switch (kind) {
        case SLI_T_EMB: return set(0, c->vocab, 0, D, D, 0);
        case SLI_T_NORM: return set(0, 1, 0, D, D, 0);
        case SLI_T_WQ: return set(r * qr, qr, 0, D, D, 0);
        case SLI_T_WK: return set(r * kr, kr, 0, D, D, qr);
        case SLI_T_WV: return set(r * kr, kr, 0, D, D, qr + kr);
        case SLI_T_WO: return set(0, D, r * qr, qr, D, 0);
        case SLI_T_GATE: return set(r * Il, Il, 0, D, D, 0);
        case SLI_T_UP: return set(r * Il, Il, 0, D, D, Il);
        case SLI_T_DOWN: return set(0, D, r * Il, Il, I, 0);
        default: return sli::fail(SLI_ERR_ARG, "sli_tp_plan: unknown tensor kind");
    }
}

}  // extern "C"
