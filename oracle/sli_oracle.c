/*
 * sli_oracle.c — TEST INFRASTRUCTURE ONLY (see sli_oracle.h for the rules and parity status).
 * Every function cites the reference file:line it restates; paths are relative to /root/reference.
 */
#define _POSIX_C_SOURCE 200809L
#include "sli_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "../include/sli_synth.h"

/* source/kernel/cpu/matmul_kernel.cpp:5-28 — y zeroed (:16), per row a sequential fp32 sum (:19-27),
 * y[r] = sum * scale (:26). */
void orc_matmul(const float* x, const float* w, float* y, int rows, int cols, float scale) {
    memset(y, 0, sizeof(float) * (size_t)rows);
    for (int i = 0; i < rows; i++) {
        const float* wr = w + (size_t)i * cols;
        float sum = 0.0f;
        for (int j = 0; j < cols; j++) sum += x[j] * wr[j];
        y[i] = sum * scale;
    }
}

/* source/kernel/cpu/rms_kernel.cpp:5-23 */
void orc_rmsnorm(const float* x, const float* w, float* y, int dim, float eps) {
    float sum_sq = 0.0f;
    for (int i = 0; i < dim; ++i) sum_sq += x[i] * x[i];          /* :12-15 */
    float tep = sum_sq / (float)dim;                               /* :17 */
    float rms = sqrtf(tep + eps);                                  /* :18 */
    float inv_rms = 1.0f / rms;                                    /* :19 */
    for (int i = 0; i < dim; ++i) y[i] = (x[i] * inv_rms) * w[i]; /* :20-22 */
}

/* source/kernel/cpu/rope_kernel.cpp:4-19 — float powf/cosf/sinf table, [T][hd/2]. */
void orc_rope_cache(int head_dim, int max_seq_len, float* sin_cache, float* cos_cache, float theta) {
    for (int i = 0; i < max_seq_len; i++) {
        for (int d = 0; d < head_dim / 2; d++) {
            int tmp = 2 * d;
            float freq = 1.0f / powf(theta, (float)tmp / (float)head_dim);
            float val = freq * (float)i;
            sin_cache[i * (head_dim / 2) + d] = sinf(val);
            cos_cache[i * (head_dim / 2) + d] = cosf(val);
        }
    }
}

/* source/kernel/cpu/rope_kernel.cpp:22-41 — rotate-half pairing (d, d+hd/2) per head block.
 * The reference runs the k loop to dim = D even when k is only KV long (:27); under GQA that touches
 * cache rows past k (pos+1..pos+g-1, later overwritten) and past the cache end at pos >= T-g+1
 * (SURVEY.md §8(a) A3). The restatement rotates k over its own k_dim only: identical on every value
 * the reference later reads for pos < T-g+1. */
void orc_rope(float* q, float* k, int pos, const float* sin_cache, const float* cos_cache, int q_dim, int k_dim,
              int head_dim) {
    for (int v = 0; v < 2; v++) {
        float* vec = v == 0 ? q : k;
        int dim = v == 0 ? q_dim : k_dim;
        for (int i = 0; i < dim; i += head_dim) {
            for (int d = 0; d < head_dim / 2; d++) {
                float fci = sin_cache[pos * (head_dim / 2) + d];
                float fcr = cos_cache[pos * (head_dim / 2) + d];
                float v0 = vec[i + d];
                float v1 = vec[i + d + head_dim / 2];
                vec[i + d] = v0 * fcr - v1 * fci;
                vec[i + d + head_dim / 2] = v1 * fcr + v0 * fci;
            }
        }
    }
}

/* source/kernel/cpu/mha_kernel.cpp:7-20 */
void orc_softmax(float* x, int n) {
    float max_value = x[0];
    for (int i = 1; i < n; i++)
        if (x[i] > max_value) max_value = x[i]; /* std::max_element: first max */
    float sum = 0.0f;
    for (int i = 0; i < n; i++) {
        x[i] = expf(x[i] - max_value);
        sum += x[i];
    }
    for (int i = 0; i < n; i++) x[i] /= sum;
}

/* source/kernel/cpu/mha_kernel.cpp:36-77 (+ attention_output_kernel :22-34). */
void orc_mha(const float* q, float* score, const float* kcache, const float* vcache, float* out, int layer, int pos,
             int max_seq_len, int head_dim, int n_heads, int n_kv_heads) {
    int kv_dim = n_kv_heads * head_dim;
    int group = n_heads / n_kv_heads;
    size_t layer_offset = (size_t)layer * max_seq_len * kv_dim;
    float scale = 1.0f / sqrtf((float)head_dim);
    for (int h = 0; h < n_heads; h++) {
        float* sh = score + (size_t)h * max_seq_len;
        const float* qh = q + (size_t)h * head_dim;
        for (int t = 0; t <= pos; t++) { /* :51-60 — matmul_kernel_cpu(q, k_t, s_t, 1, hd, scale) */
            const float* kt = kcache + layer_offset + (size_t)t * kv_dim + (size_t)(h / group) * head_dim;
            orc_matmul(qh, kt, sh + t, 1, head_dim, scale);
        }
        orc_softmax(sh, pos + 1); /* :63 */
        float* oh = out + (size_t)h * head_dim;
        memset(oh, 0, sizeof(float) * head_dim); /* :66 */
        const float* vh = vcache + layer_offset + (size_t)(h / group) * head_dim;
        for (int p = 0; p <= pos; p++) { /* :28-33 */
            const float* vp = vh + (size_t)p * kv_dim;
            for (int j = 0; j < head_dim; j++) oh[j] += sh[p] * vp[j];
        }
    }
}

/* source/kernel/cpu/swiglu_kernel.cpp:5-15 — reference variant: sigmoid(gate) * up. */
void orc_swiglu(const float* up, const float* gate, float* out, int n) {
    for (int i = 0; i < n; i++) {
        float tmp = 1.0f / (1.0f + expf(-gate[i]));
        out[i] = tmp * up[i];
    }
}

/* source/kernel/cpu/add_kernel.cpp:5-14 — memcpy(in1 -> out) then cblas_saxpy(n, 1.0, in2, out):
 * out = in1 + 1.0*in2, which is exactly in1 + in2 in fp32. */
void orc_add(const float* a, const float* b, float* out, int n) {
    for (int i = 0; i < n; i++) out[i] = a[i] + b[i];
}

/* source/kernel/cpu/emb_kernel.cpp:4-21. The reference rejects token > vocab (:10, off by one); the
 * restatement rejects token >= vocab (the reference would read one row past the table). */
int orc_embedding(int token, const float* table, float* out, int vocab, int dim) {
    if (token < 0 || token >= vocab) return -1;
    memcpy(out, table + (size_t)token * dim, sizeof(float) * dim);
    return 0;
}

/* source/op/argmax.cpp:7-17 — std::max_element: first index of the maximum. */
int orc_argmax(const float* logits, int n) {
    int best = 0;
    for (int i = 1; i < n; i++)
        if (logits[best] < logits[i]) best = i;
    return best;
}

/* ------------------------------------------------------------------ numeric helpers */
uint16_t orc_f32_to_f16_bits(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t ex = (x >> 23) & 0xFFu;
    uint32_t mant = x & 0x7FFFFFu;
    if (ex == 0xFFu) return (uint16_t)(sign | 0x7C00u | (mant ? 0x200u : 0u));
    int e = (int)ex - 127 + 15;
    if (e >= 31) return (uint16_t)(sign | 0x7C00u);
    if (e <= 0) {
        if (e < -10) return (uint16_t)sign;
        mant |= 0x800000u;
        int shift = 14 - e;
        uint32_t hm = mant >> shift;
        uint32_t rem = mant & ((1u << shift) - 1u);
        uint32_t half = 1u << (shift - 1);
        if (rem > half || (rem == half && (hm & 1u))) hm++;
        return (uint16_t)(sign | hm);
    }
    uint32_t h = sign | ((uint32_t)e << 10) | (mant >> 13);
    uint32_t rem = mant & 0x1FFFu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
    return (uint16_t)h;
}

float orc_f16_bits_to_f32(uint16_t h) {
    uint32_t sign = ((uint32_t)h & 0x8000u) << 16;
    uint32_t ex = (h >> 10) & 0x1Fu;
    uint32_t mant = h & 0x3FFu;
    uint32_t x;
    if (ex == 0) {
        if (mant == 0) {
            x = sign;
        } else { /* subnormal: normalise */
            int e = -1;
            do {
                mant <<= 1;
                e++;
            } while (!(mant & 0x400u));
            mant &= 0x3FFu;
            x = sign | ((uint32_t)(127 - 15 - e) << 23) | (mant << 13);
        }
    } else if (ex == 0x1F) {
        x = sign | 0x7F800000u | (mant << 13);
    } else {
        x = sign | ((ex - 15 + 127) << 23) | (mant << 13);
    }
    float f;
    memcpy(&f, &x, 4);
    return f;
}

float orc_round_f16(float f) { return orc_f16_bits_to_f32(orc_f32_to_f16_bits(f)); }

void orc_quant_row_i8(const float* row, int n, int8_t* q, float* scale) {
    float mx = 0.0f;
    for (int i = 0; i < n; i++) {
        float a = fabsf(row[i]);
        if (a > mx) mx = a;
    }
    float s = mx / 127.0f;
    *scale = s;
    for (int i = 0; i < n; i++) {
        float r = s > 0.0f ? rintf(row[i] / s) : 0.0f;
        if (r > 127.0f) r = 127.0f;
        if (r < -127.0f) r = -127.0f;
        q[i] = (int8_t)r;
    }
}

void orc_synth_fill(float* dst, uint64_t n, uint32_t seed, uint32_t stream, float c, float offset) {
    for (uint64_t i = 0; i < n; i++) {
        float v = (float)sli_rng_ih4(seed, stream, i) * c;
        dst[i] = offset != 0.0f ? offset + v : v;
    }
}

/* ------------------------------------------------------------------ model */
struct orc_model {
    orc_config c;
    int kv_dim;
    int kv_f16;
    float* emb;   /* [V][D], tied LM head (model.cpp:343-358) */
    float** norm; /* 2L+1 x [D] (model.cpp:360-364) */
    float **wq, **wk, **wv, **wo, **up, **gate, **down;
    float *kcache, *vcache; /* [L][T][KV] (model.cpp:264-265) */
    float *x, *h, *q, *score, *attn, *o, *x1, *u, *g, *a, *f;
    float *sin_c, *cos_c;
    double t_embed, t_layers, t_head;
    int lazy;          /* orc_model_create_lazy: one layer of weights, regenerated per layer in forward */
    uint32_t seed;     /* lazy: the synthetic weights' seed and mode */
    int wmode;
    int cur_layer;     /* lazy: layer whose weights the [0] buffers hold (-1: none) */
    int threads;       /* orc_model_set_threads: GEMV rows over this many host threads (default 1) */
};

/* ---- synthetic weight generation over host threads (test-infrastructure speed only: every element is a
 * pure function of its index, so the values do not depend on the thread count; the forward pass itself
 * stays single-threaded, as the reference CPU path) */
typedef struct {
    float* dst;
    uint64_t lo, hi;
    uint32_t seed, stream;
    float c, offset;
    int wmode, rows_mode; /* rows_mode: lo/hi are rows of `cols` (apply_wmode), else elements (fill) */
    int cols;
} gen_job;

static int gen_threads(uint64_t work) {
    if (work < ((uint64_t)1 << 22)) return 1;
    const char* e = getenv("ORC_GEN_THREADS");
    long n = e ? atol(e) : sysconf(_SC_NPROCESSORS_ONLN);
    if (n < 1) n = 1;
    if (n > 32) n = 32;
    return (int)n;
}

static void apply_wmode_rows(float* w, int r0, int r1, int cols, int wmode);

static void* gen_worker(void* p) {
    gen_job* j = (gen_job*)p;
    if (j->rows_mode) {
        apply_wmode_rows(j->dst, (int)j->lo, (int)j->hi, j->cols, j->wmode);
    } else {
        for (uint64_t i = j->lo; i < j->hi; i++) {
            float v = (float)sli_rng_ih4(j->seed, j->stream, i) * j->c;
            j->dst[i] = j->offset != 0.0f ? j->offset + v : v;
        }
    }
    return NULL;
}

static void gen_run(gen_job proto, uint64_t n) {
    int nt = gen_threads(proto.rows_mode ? n * (uint64_t)proto.cols : n);
    pthread_t th[32];
    gen_job jobs[32];
    for (int t = 0; t < nt; t++) {
        jobs[t] = proto;
        jobs[t].lo = n * (uint64_t)t / (uint64_t)nt;
        jobs[t].hi = n * (uint64_t)(t + 1) / (uint64_t)nt;
        if (nt == 1 || pthread_create(&th[t], NULL, gen_worker, &jobs[t]) != 0) {
            gen_worker(&jobs[t]);
            th[t] = 0;
        }
    }
    for (int t = 0; t < nt; t++)
        if (th[t]) pthread_join(th[t], NULL);
}

static float** alloc_tab(int n, size_t each) {
    float** t = (float**)calloc((size_t)n, sizeof(float*));
    for (int i = 0; i < n; i++) t[i] = (float*)calloc(each, sizeof(float));
    return t;
}
static void free_tab(float** t, int n) {
    if (!t) return;
    for (int i = 0; i < n; i++) free(t[i]);
    free(t);
}

static orc_model* model_create(const orc_config* cfg, int lazy) {
    orc_model* m = (orc_model*)calloc(1, sizeof(orc_model));
    m->c = *cfg;
    const orc_config* c = &m->c;
    int L = c->n_layers, D = c->dim, I = c->ffn, V = c->vocab, T = c->max_len;
    m->kv_dim = c->n_kv_heads * c->head_dim;
    int KV = m->kv_dim;
    m->lazy = lazy;
    m->cur_layer = -1;
    m->threads = 1;
    int LW = lazy ? 1 : L; /* lazy: one buffer set, regenerated layer by layer */
    m->emb = (float*)calloc((size_t)V * D, sizeof(float));
    m->norm = alloc_tab(2 * L + 1, (size_t)D);
    m->wq = alloc_tab(LW, (size_t)D * D);
    m->wk = alloc_tab(LW, (size_t)KV * D);
    m->wv = alloc_tab(LW, (size_t)KV * D);
    m->wo = alloc_tab(LW, (size_t)D * D);
    m->up = alloc_tab(LW, (size_t)I * D);
    m->gate = alloc_tab(LW, (size_t)I * D);
    m->down = alloc_tab(LW, (size_t)D * I);
    m->kcache = (float*)calloc((size_t)L * T * KV, sizeof(float));
    m->vcache = (float*)calloc((size_t)L * T * KV, sizeof(float));
    m->x = (float*)calloc((size_t)D, 4);
    m->h = (float*)calloc((size_t)D, 4);
    m->q = (float*)calloc((size_t)D, 4);
    m->score = (float*)calloc((size_t)c->n_heads * T, 4);
    m->attn = (float*)calloc((size_t)D, 4);
    m->o = (float*)calloc((size_t)D, 4);
    m->x1 = (float*)calloc((size_t)D, 4);
    m->u = (float*)calloc((size_t)I, 4);
    m->g = (float*)calloc((size_t)I, 4);
    m->a = (float*)calloc((size_t)I, 4);
    m->f = (float*)calloc((size_t)D, 4);
    m->sin_c = (float*)calloc((size_t)T * (c->head_dim / 2), 4);
    m->cos_c = (float*)calloc((size_t)T * (c->head_dim / 2), 4);
    orc_rope_cache(c->head_dim, T, m->sin_c, m->cos_c, c->theta); /* model.cpp:309-316 */
    return m;
}

orc_model* orc_model_create(const orc_config* cfg) { return model_create(cfg, 0); }

/* Full-size models (e.g. the 32-layer 7B step, 27 GB of fp32 weights) without holding every layer: the
 * forward regenerates each layer's weights (bit-identical to orc_model_init_synthetic's) before using them.
 * orc_model_weight serves only the embedding and norms of such a model. */
orc_model* orc_model_create_lazy(const orc_config* cfg) { return model_create(cfg, 1); }

void orc_model_free(orc_model* m) {
    if (!m) return;
    int L = m->c.n_layers;
    free(m->emb);
    int LW = m->lazy ? 1 : L;
    free_tab(m->norm, 2 * L + 1);
    free_tab(m->wq, LW);
    free_tab(m->wk, LW);
    free_tab(m->wv, LW);
    free_tab(m->wo, LW);
    free_tab(m->up, LW);
    free_tab(m->gate, LW);
    free_tab(m->down, LW);
    free(m->kcache);
    free(m->vcache);
    free(m->x);
    free(m->h);
    free(m->q);
    free(m->score);
    free(m->attn);
    free(m->o);
    free(m->x1);
    free(m->u);
    free(m->g);
    free(m->a);
    free(m->f);
    free(m->sin_c);
    free(m->cos_c);
    free(m);
}

float* orc_model_weight(orc_model* m, int kind, int index) {
    if (m->lazy && kind != SLI_T_EMB && kind != SLI_T_NORM) return NULL;
    switch (kind) {
        case SLI_T_EMB: return m->emb;
        case SLI_T_NORM: return m->norm[index];
        case SLI_T_WQ: return m->wq[index];
        case SLI_T_WK: return m->wk[index];
        case SLI_T_WV: return m->wv[index];
        case SLI_T_WO: return m->wo[index];
        case SLI_T_UP: return m->up[index];
        case SLI_T_GATE: return m->gate[index];
        case SLI_T_DOWN: return m->down[index];
        default: return NULL;
    }
}

static void apply_wmode_rows(float* w, int r0, int r1, int cols, int wmode) {
    if (wmode == ORC_W_F16) {
        for (size_t i = (size_t)r0 * cols; i < (size_t)r1 * cols; i++) w[i] = orc_round_f16(w[i]);
    } else if (wmode == ORC_W_I8) {
        int8_t* q = (int8_t*)malloc((size_t)cols);
        for (int r = r0; r < r1; r++) {
            float s;
            float* row = w + (size_t)r * cols;
            orc_quant_row_i8(row, cols, q, &s);
            for (int j = 0; j < cols; j++) row[j] = (float)q[j] * s;
        }
        free(q);
    }
}

static void apply_wmode(float* w, int rows, int cols, int wmode) {
    if (wmode != ORC_W_F16 && wmode != ORC_W_I8) return;
    gen_job j = {w, 0, 0, 0, 0, 0.0f, 0.0f, wmode, 1, cols};
    gen_run(j, (uint64_t)rows);
}

/* orc_synth_fill over host threads (same values) */
static void synth_fill(float* dst, uint64_t n, uint32_t seed, uint32_t stream, float c, float offset) {
    gen_job j = {dst, 0, 0, seed, stream, c, offset, 0, 0, 0};
    gen_run(j, n);
}

/* layer l's seven matrices into the given buffers (model.cpp:366-398 shapes) */
static void gen_layer(orc_model* m, int l, float* wq, float* wk, float* wv, float* wo, float* up, float* gate,
                      float* down) {
    const orc_config* c = &m->c;
    int D = c->dim, I = c->ffn, KV = m->kv_dim;
    uint32_t seed = m->seed;
    float cD = SLI_SYNTH_C(1.0 / sqrt((double)D));
    float cI = SLI_SYNTH_C(1.0 / sqrt((double)I));
    synth_fill(wq, (uint64_t)D * D, seed, sli_stream_id(SLI_T_WQ, l), cD, 0.0f);
    synth_fill(wk, (uint64_t)KV * D, seed, sli_stream_id(SLI_T_WK, l), cD, 0.0f);
    synth_fill(wv, (uint64_t)KV * D, seed, sli_stream_id(SLI_T_WV, l), cD, 0.0f);
    synth_fill(wo, (uint64_t)D * D, seed, sli_stream_id(SLI_T_WO, l), cD, 0.0f);
    synth_fill(up, (uint64_t)I * D, seed, sli_stream_id(SLI_T_UP, l), cD, 0.0f);
    synth_fill(gate, (uint64_t)I * D, seed, sli_stream_id(SLI_T_GATE, l), cD, 0.0f);
    synth_fill(down, (uint64_t)D * I, seed, sli_stream_id(SLI_T_DOWN, l), cI, 0.0f);
    apply_wmode(wq, D, D, m->wmode);
    apply_wmode(wk, KV, D, m->wmode);
    apply_wmode(wv, KV, D, m->wmode);
    apply_wmode(wo, D, D, m->wmode);
    apply_wmode(up, I, D, m->wmode);
    apply_wmode(gate, I, D, m->wmode);
    apply_wmode(down, D, I, m->wmode);
}

int orc_model_init_synthetic(orc_model* m, uint32_t seed, int wmode) {
    const orc_config* c = &m->c;
    int L = c->n_layers, D = c->dim, V = c->vocab;
    m->seed = seed;
    m->wmode = wmode;
    m->cur_layer = -1;
    synth_fill(m->emb, (uint64_t)V * D, seed, sli_stream_id(SLI_T_EMB, 0), SLI_SYNTH_C(0.02), 0.0f);
    apply_wmode(m->emb, V, D, wmode);
    for (int i = 0; i < 2 * L + 1; i++)
        orc_synth_fill(m->norm[i], (uint64_t)D, seed, sli_stream_id(SLI_T_NORM, i), SLI_SYNTH_C(0.1), 1.0f);
    if (m->lazy) return 0; /* layers: regenerated in the forward */
    for (int l = 0; l < L; l++) gen_layer(m, l, m->wq[l], m->wk[l], m->wv[l], m->wo[l], m->up[l], m->gate[l], m->down[l]);
    return 0;
}

void orc_model_set_kv_f16(orc_model* m, int on) { m->kv_f16 = on; }
float* orc_model_kcache(orc_model* m) { return m->kcache; }
float* orc_model_vcache(orc_model* m) { return m->vcache; }

typedef struct {
    orc_model* m;
    uint32_t seed;
    int upto, l0, l1;
} kv_job;
static void fill_kv_layers(orc_model* m, uint32_t seed, int upto, int l0, int l1);
static void* kv_worker(void* p) {
    kv_job* j = (kv_job*)p;
    fill_kv_layers(j->m, j->seed, j->upto, j->l0, j->l1);
    return NULL;
}

/* one layer per host thread (test-infrastructure speed; the values do not depend on the split) */
void orc_model_fill_kv_synthetic(orc_model* m, uint32_t seed, int upto) {
    int L = m->c.n_layers;
    int nt = gen_threads((uint64_t)L * upto * m->kv_dim);
    if (nt > L) nt = L;
    pthread_t th[32];
    kv_job jobs[32];
    for (int t = 0; t < nt; t++) {
        jobs[t] = (kv_job){m, seed, upto, L * t / nt, L * (t + 1) / nt};
        if (nt == 1 || pthread_create(&th[t], NULL, kv_worker, &jobs[t]) != 0) {
            kv_worker(&jobs[t]);
            th[t] = 0;
        }
    }
    for (int t = 0; t < nt; t++)
        if (th[t]) pthread_join(th[t], NULL);
}

static void fill_kv_layers(orc_model* m, uint32_t seed, int upto, int l0, int l1) {
    int KV = m->kv_dim, T = m->c.max_len;
    float c1 = SLI_SYNTH_C(1.0);
    for (int l = l0; l < l1; l++) {
        for (int t = 0; t < upto; t++) {
            for (int j = 0; j < KV; j++) {
                uint64_t idx = (uint64_t)t * KV + j;
                float kv = (float)sli_rng_ih4(seed, sli_stream_id(SLI_T_KCACHE, l), idx) * c1;
                float vv = (float)sli_rng_ih4(seed, sli_stream_id(SLI_T_VCACHE, l), idx) * c1;
                if (m->kv_f16) {
                    kv = orc_round_f16(kv);
                    vv = orc_round_f16(vv);
                }
                size_t off = ((size_t)l * T + t) * KV + j;
                m->kcache[off] = kv;
                m->vcache[off] = vv;
            }
        }
    }
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* The CPU baseline's secondary "all host cores, not reference" line: a GEMV's rows split over
 * threads. Every row is still one sequential fp32 sum, so the results are bit-identical to orc_matmul. */
typedef struct {
    const float *x, *w;
    float* y;
    int r0, r1, cols;
} mm_job;
static void* mm_worker(void* p) {
    mm_job* j = (mm_job*)p;
    orc_matmul(j->x, j->w + (size_t)j->r0 * j->cols, j->y + j->r0, j->r1 - j->r0, j->cols, 1.0f);
    return NULL;
}
static void mm(const orc_model* m, const float* x, const float* w, float* y, int rows, int cols) {
    int nt = m->threads > 32 ? 32 : m->threads;
    if (nt <= 1 || rows < 2 * nt) {
        orc_matmul(x, w, y, rows, cols, 1.0f);
        return;
    }
    pthread_t th[32];
    mm_job jobs[32];
    for (int t = 0; t < nt; t++) {
        jobs[t] = (mm_job){x, w, y, (int)((int64_t)rows * t / nt), (int)((int64_t)rows * (t + 1) / nt), cols};
        if (pthread_create(&th[t], NULL, mm_worker, &jobs[t]) != 0) {
            mm_worker(&jobs[t]);
            th[t] = 0;
        }
    }
    for (int t = 0; t < nt; t++)
        if (th[t]) pthread_join(th[t], NULL);
}

void orc_model_set_threads(orc_model* m, int n) { m->threads = n < 1 ? 1 : n; }

/* source/model/model.cpp:40-140 */
int orc_model_forward(orc_model* m, int token, int pos, float* logits_out) {
    const orc_config* c = &m->c;
    int L = c->n_layers, D = c->dim, I = c->ffn, V = c->vocab, T = c->max_len, KV = m->kv_dim;
    if (pos < 0 || pos >= T) return -2;
    double t0 = now_s();
    if (orc_embedding(token, m->emb, m->x, V, D) != 0) return -1; /* :48 */
    double t1 = now_s();
    for (int l = 0; l < L; l++) {
        int lw = l; /* weight slot */
        if (m->lazy) {
            lw = 0;
            if (m->cur_layer != l) {
                gen_layer(m, l, m->wq[0], m->wk[0], m->wv[0], m->wo[0], m->up[0], m->gate[0], m->down[0]);
                m->cur_layer = l;
            }
        }
        orc_rmsnorm(m->x, m->norm[2 * l], m->h, D, c->eps);          /* :52 */
        float* krow = m->kcache + ((size_t)l * T + pos) * KV;        /* :54-55 slice_KV_cache */
        float* vrow = m->vcache + ((size_t)l * T + pos) * KV;
        mm(m, m->h, m->wq[lw], m->q, D, D);                /* :58 */
        mm(m, m->h, m->wk[lw], krow, KV, D);               /* :60 */
        mm(m, m->h, m->wv[lw], vrow, KV, D);               /* :62 */
        orc_rope(m->q, krow, pos, m->sin_c, m->cos_c, D, KV, c->head_dim); /* :66-67 */
        if (m->kv_f16) {
            for (int j = 0; j < KV; j++) {
                krow[j] = orc_round_f16(krow[j]);
                vrow[j] = orc_round_f16(vrow[j]);
            }
        }
        orc_mha(m->q, m->score, m->kcache, m->vcache, m->attn, l, pos, T, c->head_dim, c->n_heads,
                c->n_kv_heads);                                       /* :70-78 */
        mm(m, m->attn, m->wo[lw], m->o, D, D);             /* :80-83 */
        orc_add(m->x, m->o, m->x1, D);                               /* :86-90 */
        orc_rmsnorm(m->x1, m->norm[2 * l + 1], m->h, D, c->eps);     /* :93-96 */
        mm(m, m->h, m->up[lw], m->u, I, D);                /* :99-102 */
        mm(m, m->h, m->gate[lw], m->g, I, D);              /* :105-108 */
        orc_swiglu(m->u, m->g, m->a, I);                             /* :111-115 */
        mm(m, m->a, m->down[lw], m->f, D, I);              /* :118-121 */
        orc_add(m->f, m->x1, m->x, D);                               /* :124-128 */
    }
    double t2 = now_s();
    orc_rmsnorm(m->x, m->norm[2 * L], m->h, D, c->eps);              /* :131-134 */
    mm(m, m->h, m->emb, logits_out, V, D);               /* :136-139 tied head */
    double t3 = now_s();
    m->t_embed = t1 - t0;
    m->t_layers = t2 - t1;
    m->t_head = t3 - t2;
    return 0;
}

/* source/model/model.cpp:142-187 on token ids (the SPELayer tokenizer is out of scope). */
int orc_model_predict(orc_model* m, const int* prompt, int n_prompt, int max_length, int* tokens_out,
                      float* logits_out) {
    int V = m->c.vocab;
    float* logits = (float*)malloc(sizeof(float) * (size_t)V);
    int pos = 0;
    int token = prompt[0];
    while (pos < max_length) { /* :157 */
        tokens_out[pos] = token;
        int rc = orc_model_forward(m, token, pos, logits);
        if (rc != 0) {
            free(logits);
            return rc;
        }
        if (logits_out) memcpy(logits_out + (size_t)pos * V, logits, sizeof(float) * V);
        if (pos < n_prompt - 1) { /* :159-165 teacher forcing */
            pos++;
            token = prompt[pos];
        } else { /* :166-183 greedy */
            pos++;
            token = orc_argmax(logits, V);
        }
    }
    free(logits);
    return max_length;
}

void orc_model_last_timing(const orc_model* m, double* t_embed, double* t_layers, double* t_head) {
    if (t_embed) *t_embed = m->t_embed;
    if (t_layers) *t_layers = m->t_layers;
    if (t_head) *t_head = m->t_head;
}

static int wr(FILE* f, const float* p, size_t n) { return fwrite(p, sizeof(float), n, f) == n ? 0 : -1; }

/* model.cpp:336-469 order: embed, 2L+1 norms, wq[L], wk[L], wv[L], wo[L], up[L], gate[L], down[L]. */
int orc_model_write_flat(const orc_model* m, const char* path) {
    const orc_config* c = &m->c;
    if (m->lazy) return -2; /* its layers are not held */
    int L = c->n_layers, D = c->dim, I = c->ffn, V = c->vocab, KV = m->kv_dim;
    FILE* f = fopen(path, "wb");
    if (!f) return -1;
    int rc = wr(f, m->emb, (size_t)V * D);
    for (int i = 0; i < 2 * L + 1; i++) rc |= wr(f, m->norm[i], (size_t)D);
    for (int l = 0; l < L; l++) rc |= wr(f, m->wq[l], (size_t)D * D);
    for (int l = 0; l < L; l++) rc |= wr(f, m->wk[l], (size_t)KV * D);
    for (int l = 0; l < L; l++) rc |= wr(f, m->wv[l], (size_t)KV * D);
    for (int l = 0; l < L; l++) rc |= wr(f, m->wo[l], (size_t)D * D);
    for (int l = 0; l < L; l++) rc |= wr(f, m->up[l], (size_t)I * D);
    for (int l = 0; l < L; l++) rc |= wr(f, m->gate[l], (size_t)I * D);
    for (int l = 0; l < L; l++) rc |= wr(f, m->down[l], (size_t)D * I);
    fclose(f);
    return rc;
}
