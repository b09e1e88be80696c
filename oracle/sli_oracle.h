/*
 * sli_oracle.h — TEST INFRASTRUCTURE ONLY. CPU restatement of Boundwhd/SimpleLLMInference's
 * transformer-decode path (reference CPU backend, /root/reference/source/kernel/cpu/ and
 * source/model/model.cpp). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / the timed CPU baseline — never as the product path.
 *
 * PARITY STATUS: "parity unpinned" — the reference cannot be built in this image without writing
 * stand-ins (every translation unit includes <cuda_runtime_api.h> via include/memory/alloc.h:8 and
 * must link libcudart for source/memory/alloc.cpp:15-33; add_kernel.cpp needs OpenBLAS <cblas.h>;
 * model.cpp needs sentencepiece via include/op/encode.h:5), and the reference holds no tests, golden
 * vectors or fixtures. This restatement is cross-checked against an
 * independent float64 numpy restatement (tests/refmath.py) and pinned by committed fixtures it
 * generated (tests/golden/), see DESIGN.md §2.
 *
 * Arithmetic contract: fp32 everywhere, sequential left-to-right sums, no FMA contraction
 * (built with -O2 -ffp-contract=off, no -march), libm expf/sqrtf/powf/sinf/cosf — the same
 * operations the reference's g++ -O2 CPU build performs.
 */
#ifndef SLI_ORACLE_H_
#define SLI_ORACLE_H_
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* ---- per-op restatements (reference file:line in sli_oracle.c) ---- */
void orc_matmul(const float* x, const float* w, float* y, int rows, int cols, float scale);
void orc_rmsnorm(const float* x, const float* w, float* y, int dim, float eps);
void orc_rope_cache(int head_dim, int max_seq_len, float* sin_cache, float* cos_cache, float theta);
void orc_rope(float* q, float* k, int pos, const float* sin_cache, const float* cos_cache, int q_dim, int k_dim,
              int head_dim);
void orc_softmax(float* x, int n);
/* kv caches in reference layout [L][T][KV] fp32; score scratch [H][T]. */
void orc_mha(const float* q, float* score, const float* kcache, const float* vcache, float* out, int layer, int pos,
             int max_seq_len, int head_dim, int n_heads, int n_kv_heads);
void orc_swiglu(const float* up, const float* gate, float* out, int n);
void orc_add(const float* a, const float* b, float* out, int n);
int orc_embedding(int token, const float* table, float* out, int vocab, int dim);
int orc_argmax(const float* logits, int n);

/* ---- numeric helpers shared with tests ---- */
uint16_t orc_f32_to_f16_bits(float f); /* round-to-nearest-even */
float orc_f16_bits_to_f32(uint16_t h);
float orc_round_f16(float f);
/* symmetric per-row int8: scale = max|row|/127, q = rint(w/scale); writes q and scale, returns 0 */
void orc_quant_row_i8(const float* row, int n, int8_t* q, float* scale);

/* ---- synthetic data (sli_synth.h) ---- */
void orc_synth_fill(float* dst, uint64_t n, uint32_t seed, uint32_t stream, float c, float offset);

/* ---- model (LlamaModel restatement, model.cpp:40-187) ---- */
typedef struct {
    int vocab, dim, n_heads, n_kv_heads, head_dim, ffn, n_layers, max_len;
    float eps, theta;
} orc_config;

enum { ORC_W_F32 = 0, ORC_W_F16 = 1, ORC_W_I8 = 2 };

typedef struct orc_model orc_model;
orc_model* orc_model_create(const orc_config* cfg);
/* full-size models: one layer of weights held, regenerated per layer inside orc_model_forward (same values) */
orc_model* orc_model_create_lazy(const orc_config* cfg);
void orc_model_free(orc_model* m);
/* weight mode: values are generated in fp32 and then rounded (F16) or per-row quantised+dequantised
 * (I8) so the oracle computes in fp32 on exactly the weights the device holds. */
int orc_model_init_synthetic(orc_model* m, uint32_t seed, int wmode);
/* reference-layout fp32 tensor of a kind/index (SLI_T_* from sli_synth.h). */
float* orc_model_weight(orc_model* m, int kind, int index);
void orc_model_set_kv_f16(orc_model* m, int on);
float* orc_model_kcache(orc_model* m);
float* orc_model_vcache(orc_model* m);
/* fill K/V rows [0, upto) of every layer with the bench's synthetic N(0,1) values (rounded if kv_f16). */
void orc_model_fill_kv_synthetic(orc_model* m, uint32_t seed, int upto);
/* one decode step: LlamaModel::forward with input_token = token, position = pos. */
int orc_model_forward(orc_model* m, int token, int pos, float* logits_out);
/* LlamaModel::predict restated on token ids: returns number of steps (= max_length). tokens_out[t] is the
 * token fed at position t; logits_out (optional) is [max_length][V]. */
int orc_model_predict(orc_model* m, const int* prompt, int n_prompt, int max_length, int* tokens_out,
                      float* logits_out);
/* GEMV rows of the forward split over n host threads (bit-identical results; the CPU baseline's secondary
 * all-cores line, BASELINE.md §4 — not the reference, which is single-threaded). Default 1. */
void orc_model_set_threads(orc_model* m, int n);
/* seconds spent in the last forward: embedding, transformer layers, final norm + LM head. */
void orc_model_last_timing(const orc_model* m, double* t_embed, double* t_layers, double* t_head);
/* write the reference's flat fp32 weight file (model.cpp:336-469 order). */
int orc_model_write_flat(const orc_model* m, const char* path);

#ifdef __cplusplus
}
#endif
#endif
