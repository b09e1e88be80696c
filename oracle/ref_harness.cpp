// ref_harness.cpp — TEST INFRASTRUCTURE ONLY. A plain-pointer C ABI over the REFERENCE's own CPU kernels,
// compiled in place from /root/reference by oracle/Makefile (target `ref`, output oracle/_ref/libref.so).
// Nothing of the reference is copied: this file only wraps raw buffers in the reference's mem::Tensor
// (external, non-owning buffers, tensor.cpp:45-50) and calls the kernel::*_cpu functions, exactly as the
// reference's op layer does (source/op/*.cpp forward() on kDeviceCPU).
//
// It exists to pin oracle/sli_oracle.c (the restatement every test uses) against the reference itself:
// tests/golden/make_ref_golden.py writes tests/golden/ref_ops.npz from this library, and
// tests/test_oracle.py checks the restatement bit for bit against those committed vectors.
// Only tests/golden/make_ref_golden.py, tests/ and bench.py's cpu_baseline calibration may load it.
//
// Build notes: the reference headers include <cuda_runtime_api.h> / <driver_types.h>
// (include/memory/alloc.h:8, tensor.h:3); the genuine NVIDIA headers shipped in this image are used (no
// stand-ins). source/memory/alloc.cpp's CUDA allocator leaves cudaMalloc/cudaMemcpy/cudaMemset/cudaFree/
// cudaGetLastError unresolved; they are never reached on the CPU path, so the library is loaded with
// RTLD_LAZY. add_kernel.cpp (<cblas.h>, OpenBLAS absent) and model.cpp (sentencepiece via encode.h) are not
// built: `add` is done inline and the model composition is restated over the reference's op layers (below).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <ctime>
#include <map>
#include <memory>
#include <vector>

#include "argmax.h"
#include "config.h"
#include "embedding.h"
#include "matmul.h"
#include "mha.h"
#include "rmsnorm.h"
#include "rope.h"
#include "swiglu.h"
#include "weight_loader.h"

#include "emb_kernel.h"
#include "matmul_kernel.h"
#include "mha_kernel.h"
#include "rms_kernel.h"
#include "rope_kernel.h"
#include "swiglu_kernel.h"

namespace kernel {
// defined with external linkage in source/kernel/cpu/mha_kernel.cpp:7-20 (not declared in a header)
void softmax_kernel_cpu(const mem::Tensor& in, int32_t size);
}

namespace {
mem::Tensor view(const void* p, std::vector<int32_t> dims) {
    mem::Tensor t(std::move(dims), false, nullptr, const_cast<void*>(p));
    t.set_device_type(base::DeviceType::kDeviceCPU);
    return t;
}
}  // namespace

extern "C" {

// matmul_kernel.cpp:5-28 — y[rows] = scale * W[rows][cols] · x[cols]
void ref_matmul(const float* x, const float* w, float* y, int rows, int cols, float scale) {
    kernel::matmul_kernel_cpu(view(x, {cols}), view(w, {rows, cols}), view(y, {rows}), rows, cols, scale);
}

// rms_kernel.cpp:5-23
void ref_rmsnorm(const float* x, const float* w, float* y, int dim, float eps) {
    kernel::rmsnorm_kernel_cpu(view(x, {dim}), view(w, {dim}), view(y, {dim}), dim, eps);
}

// rope_kernel.cpp:4-19 — sin/cos tables [max_seq_len][head_dim/2]
void ref_rope_cache(int head_dim, int max_seq_len, float* sin_cache, float* cos_cache, float theta) {
    kernel::rope_cache_cal(head_dim, max_seq_len, view(sin_cache, {max_seq_len, head_dim / 2}),
                           view(cos_cache, {max_seq_len, head_dim / 2}), theta);
}

// rope_kernel.cpp:22-41 — rotates q AND k over `dim` floats (k must have room for dim)
void ref_rope(float* q, float* k, int pos, const float* sin_cache, const float* cos_cache, int dim, int head_dim,
              int max_seq_len) {
    int32_t p = pos;
    kernel::rope_kernel_cpu(view(q, {dim}), view(k, {dim}), view(&p, {1}), view(sin_cache, {max_seq_len, head_dim / 2}),
                            view(cos_cache, {max_seq_len, head_dim / 2}), dim, head_dim);
}

// mha_kernel.cpp:7-20
void ref_softmax(float* x, int n) { kernel::softmax_kernel_cpu(view(x, {n}), n); }

// mha_kernel.cpp:36-77 — caches [L][T][KV] fp32, score scratch [H][T]
void ref_mha(const float* q, float* score, const float* kcache, const float* vcache, float* out, int layer, int pos,
             int max_seq_len, int head_dim, int n_heads, int n_kv_heads, int n_layers) {
    const int dim = n_heads * head_dim, kv_dim = n_kv_heads * head_dim;
    kernel::mha_kernel_cpu(view(q, {dim}), view(score, {n_heads, max_seq_len}),
                           view(kcache, {n_layers, max_seq_len, kv_dim}), view(vcache, {n_layers, max_seq_len, kv_dim}),
                           view(out, {dim}), layer, pos, max_seq_len, head_dim, dim, kv_dim, n_heads / n_kv_heads,
                           n_heads, base::DeviceType::kDeviceCPU);
}

// swiglu_kernel.cpp:5-15 — out = sigmoid(gate) * up
void ref_swiglu(const float* up, const float* gate, float* out, int n) {
    kernel::swiglu_kernel_cpu(view(up, {n}), view(gate, {n}), view(out, {n}), n);
}

// emb_kernel.cpp:4-21 — the caller keeps token <= vocab (a larger token makes the reference exit(1))
void ref_embedding(int token, const float* table, float* out, int vocab, int dim) {
    int32_t t = token;
    kernel::emb_kernel_cpu(view(&t, {1}), view(table, {vocab, dim}), view(out, {dim}), vocab, dim);
}

// source/op/argmax.cpp:7-17 through the reference's own argmaxLayer (std::max_element, first max)
int ref_argmax(const float* logits, int n) {
    int32_t idx = -1;
    op::argmaxLayer a(base::DeviceType::kDeviceCPU, n);
    a.forward(view(logits, {n}), view(&idx, {1}));
    return idx;
}

}  // extern "C"


// ---- LlamaModel composition over the reference's own op layers -------------------------------------------
// model.cpp cannot be compiled here (model.h:10 includes encode.h -> sentencepiece), so the lines that wire
// the ops together (model.cpp:40-187 forward/predict, :203-245 read_model_file, :246-321 init_mem, :323-469
// create_*_layers) are restated below in the same order. Every op they call is the reference's own
// (source/op/*.cpp -> source/kernel/cpu/*.cpp), and the weights come from the reference's flat fp32 file
// through its own RawModelDataFp32 (weight_loader.cpp) at create_param_layers' offsets. The residual add is
// the one op done here: add_kernel.cpp needs <cblas.h>; its CPU semantics are memcpy + saxpy(alpha = 1), i.e.
// out = in1 + in2 in fp32 (add_kernel.cpp:5-14).

namespace {
// ModelBufferType (model.h:14-34)
enum Buf {
    input_token = 0, position, key_cache, value_cache, emb_output, rms_output, query, score, mha_output, att_output,
    ffn_input, up_output, gate_output, down_output, swi_output, ffn_output, model_pred, sin_cache, cos_cache
};
using LayerP = std::shared_ptr<op::Layer>;

struct RefModel {
    model::LlamaModelConfig c;
    std::shared_ptr<model::RawModelDataFp32> raw;
    LayerP emb, cls, mha, rope, swiglu;
    std::shared_ptr<op::argmaxLayer> argmax;
    std::vector<LayerP> norms, wq, wk, wv, wo, up, gate, down;
    std::map<int, mem::Tensor> buf;
    std::vector<float> kv_store[2];  // the K / V caches' memory (see ref_model_create)
    double t_emb = 0, t_layers = 0, t_head = 0;  // last forward, seconds (harness instrumentation)
    const mem::Tensor& get(Buf t) const { return buf.at(int(t)); }
};

double now_s() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

void add_fp32(const mem::Tensor& a, const mem::Tensor& b, const mem::Tensor& out, int n) {
    const float* x = a.ptr<float>();
    const float* y = b.ptr<float>();
    float* o = const_cast<float*>(out.ptr<float>());
    for (int i = 0; i < n; i++) o[i] = x[i] + y[i];
}

// model.cpp:40-140
void forward(RefModel& m) {
    const auto& c = m.c;
    int pos = const_cast<mem::Tensor&>(m.get(position)).index<int>(0);
    const double t0 = now_s();
    m.emb->forward(m.get(input_token), m.get(emb_output));
    const double t1 = now_s();
    for (int l = 0; l < c.num_hidden_layers; l++) {
        m.norms[2 * l]->forward(m.get(emb_output), m.get(rms_output));
        const auto& [key, value] =
            mem::slice_KV_cache(l, pos, c.max_length, c.kv_hidden_size, m.get(key_cache), m.get(value_cache));
        m.wq[l]->forward(m.get(rms_output), m.get(query));
        m.wk[l]->forward(m.get(rms_output), key);
        m.wv[l]->forward(m.get(rms_output), value);
        m.rope->forward(m.get(query), key, m.get(position), m.get(sin_cache), m.get(cos_cache));
        std::dynamic_pointer_cast<op::MultiHeadAttention>(m.mha)->set_pos(pos);
        std::dynamic_pointer_cast<op::MultiHeadAttention>(m.mha)->set_layer_index(l);
        m.mha->forward(m.get(query), m.get(score), m.get(key_cache), m.get(value_cache), m.get(mha_output));
        m.wo[l]->forward(m.get(mha_output), m.get(att_output));
        add_fp32(m.get(emb_output), m.get(att_output), m.get(ffn_input), c.hidden_size);
        m.norms[2 * l + 1]->forward(m.get(ffn_input), m.get(rms_output));
        m.up[l]->forward(m.get(rms_output), m.get(up_output));
        m.gate[l]->forward(m.get(rms_output), m.get(gate_output));
        m.swiglu->forward(m.get(up_output), m.get(gate_output), m.get(swi_output));
        m.down[l]->forward(m.get(swi_output), m.get(ffn_output));
        add_fp32(m.get(ffn_output), m.get(ffn_input), m.get(emb_output), c.hidden_size);
    }
    const double t2 = now_s();
    m.norms[2 * c.num_hidden_layers]->forward(m.get(emb_output), m.get(rms_output));
    m.cls->forward(m.get(rms_output), m.get(model_pred));
    m.t_emb = t1 - t0;
    m.t_layers = t2 - t1;
    m.t_head = now_s() - t2;
}

std::vector<LayerP> matmuls(RefModel& m, size_t& off, int rows, int cols) {
    std::vector<LayerP> v;
    for (int i = 0; i < m.c.num_hidden_layers; i++) {
        v.emplace_back(std::make_shared<op::MatmulLayer>(base::DeviceType::kDeviceCPU, rows, cols));
        v[i]->set_weight(0, {rows, cols}, m.raw->weight(off), base::DeviceType::kDeviceCPU);
        off += size_t(rows) * cols;
    }
    return v;
}
}  // namespace

extern "C" {

void ref_model_free(void* h);

// model.cpp:22-39 init(): read_model_file (:203-245), create_param_layers (:323-469),
// create_nonparam_layers (:312-321), init_mem (:246-310) — on the CPU device, config passed in (the
// reference hard-codes config.h). Returns nullptr if the file cannot be mapped.
static void* create(RefModel* m, int vocab, int dim, int n_heads, int n_kv_heads, int head_dim, int ffn,
                    int n_layers, int max_len, float eps, float theta, size_t file_bytes);

void* ref_model_create(int vocab, int dim, int n_heads, int n_kv_heads, int head_dim, int ffn, int n_layers,
                       int max_len, float eps, float theta, const char* path) {
    auto* m = new RefModel();
    m->raw = std::make_shared<model::RawModelDataFp32>();
    int fd = open(path, O_RDONLY);
    struct stat sb;
    if (fd == -1 || fstat(fd, &sb) == -1) { if (fd != -1) close(fd); delete m; return nullptr; }
    m->raw->fd = fd;
    m->raw->file_size = sb.st_size;
    m->raw->weight_data = mmap(nullptr, sb.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
    m->raw->data = m->raw->weight_data;  // so ~RawModelData unmaps it (the reference leaves `data` unset)
    if (m->raw->weight_data == MAP_FAILED) { m->raw->data = nullptr; delete m; return nullptr; }
    return create(m, vocab, dim, n_heads, n_kv_heads, head_dim, ffn, n_layers, max_len, eps, theta, sb.st_size);
}

// The same model over a flat fp32 image already in host memory (the caller keeps it alive): the CPU-baseline
// leg builds it from the synthetic weights instead of writing a multi-GB file.
void* ref_model_create_mem(int vocab, int dim, int n_heads, int n_kv_heads, int head_dim, int ffn, int n_layers,
                           int max_len, float eps, float theta, const float* flat, size_t n_floats) {
    auto* m = new RefModel();
    m->raw = std::make_shared<model::RawModelDataFp32>();
    m->raw->weight_data = const_cast<float*>(flat);
    return create(m, vocab, dim, n_heads, n_kv_heads, head_dim, ffn, n_layers, max_len, eps, theta,
                  n_floats * sizeof(float));
}

static void* create(RefModel* m, int vocab, int dim, int n_heads, int n_kv_heads, int head_dim, int ffn,
                    int n_layers, int max_len, float eps, float theta, size_t file_bytes) {
    auto& c = m->c;
    c.vocab_size = vocab; c.hidden_size = dim; c.num_attention_heads = n_heads; c.num_key_value_heads = n_kv_heads;
    c.head_dim = head_dim; c.kv_hidden_size = n_kv_heads * head_dim; c.intermediate_size = ffn;
    c.num_hidden_layers = n_layers; c.max_length = max_len; c.rms_norm_eps = eps; c.rope_theta = theta;
    const auto cpu = base::DeviceType::kDeviceCPU;

    size_t off = 0;
    m->emb = std::make_shared<op::EmbeddingLayer>(cpu, vocab, dim);
    m->emb->set_weight(0, {vocab, dim}, m->raw->weight(off), cpu);
    m->cls = std::make_shared<op::MatmulLayer>(cpu, vocab, dim);  // tied LM head, model.cpp:350-358
    m->cls->set_weight(0, {vocab, dim}, m->raw->weight(off), cpu);
    off += size_t(vocab) * dim;
    for (int i = 0; i < 2 * n_layers + 1; i++) {
        m->norms.emplace_back(std::make_shared<op::RmsNormLayer>(cpu, dim, eps));
        m->norms[i]->set_weight(0, {dim}, m->raw->weight(off), cpu);
        off += dim;
    }
    const int kv = c.kv_hidden_size;
    m->wq = matmuls(*m, off, dim, dim);
    m->wk = matmuls(*m, off, kv, dim);
    m->wv = matmuls(*m, off, kv, dim);
    m->wo = matmuls(*m, off, dim, dim);
    m->up = matmuls(*m, off, ffn, dim);
    m->gate = matmuls(*m, off, ffn, dim);
    m->down = matmuls(*m, off, dim, ffn);
    if (off * sizeof(float) > file_bytes) { ref_model_free(m); return nullptr; }

    m->argmax = std::make_shared<op::argmaxLayer>(cpu, vocab);
    m->mha = std::make_shared<op::MultiHeadAttention>(cpu, max_len, head_dim, n_heads, n_kv_heads);
    m->rope = std::make_shared<op::RoPELayer>(cpu, dim, head_dim);
    m->swiglu = std::make_shared<op::SwigluLayer>(cpu, ffn);

    auto alloc = mem::CPUDeviceAllocatorFactory::get_instance();
    auto put = [&](Buf t, std::vector<int32_t> dims) { m->buf.emplace(int(t), mem::Tensor(dims, true, alloc)); };
    put(input_token, {1}); put(position, {1});
    // The K / V caches: model.cpp:264-265 allocates exactly [L][T][KV]. Under GQA rope_kernel.cpp:27 rotates k
    // over D floats, so a step at position T - 1 of the last layer writes D - KV floats past the end of the cache
    // (a heap overflow in the reference itself). The harness gives the caches D floats of slack so
    // timing that step (the CPU baseline at pos ctx - 1) cannot corrupt the heap; every value read is the same.
    for (int i = 0; i < 2; i++) {
        m->kv_store[i].assign(size_t(n_layers) * max_len * kv + dim, 0.0f);
        m->buf.emplace(int(i == 0 ? key_cache : value_cache),
                       view(m->kv_store[i].data(), {n_layers, max_len, kv}));
    }
    put(emb_output, {dim}); put(rms_output, {dim}); put(query, {dim});
    // model.cpp:278 sizes the score scratch {head_dim, max_length} but mha uses it as [n_heads][max_length]
    put(score, {std::max(head_dim, n_heads), max_len});
    put(mha_output, {dim}); put(att_output, {dim}); put(ffn_input, {dim});
    put(up_output, {ffn}); put(gate_output, {ffn}); put(down_output, {dim}); put(swi_output, {ffn});
    put(ffn_output, {dim}); put(model_pred, {vocab});
    put(sin_cache, {max_len, head_dim / 2}); put(cos_cache, {max_len, head_dim / 2});
    kernel::rope_cache_cal(head_dim, max_len, m->get(sin_cache), m->get(cos_cache), theta);
    return m;
}

void ref_model_free(void* h) { delete static_cast<RefModel*>(h); }

// the model's K / V caches [L][T][KV] fp32 (model.cpp:264-265), e.g. to fill rows before timing a late position
void ref_model_kv(void* h, float** k, float** v) {
    auto& m = *static_cast<RefModel*>(h);
    *k = const_cast<float*>(m.get(key_cache).ptr<float>());
    *v = const_cast<float*>(m.get(value_cache).ptr<float>());
}

// seconds of the last forward: embedding, the transformer layers, final norm + LM head
void ref_model_last_timing(void* h, double* t_emb, double* t_layers, double* t_head) {
    auto& m = *static_cast<RefModel*>(h);
    *t_emb = m.t_emb;
    *t_layers = m.t_layers;
    *t_head = m.t_head;
}

// one LlamaModel::forward with input_token = token, position = pos; logits [vocab]
void ref_model_forward(void* h, int token, int pos, float* logits) {
    auto& m = *static_cast<RefModel*>(h);
    const_cast<mem::Tensor&>(m.get(input_token)).index<int32_t>(0) = token;
    const_cast<mem::Tensor&>(m.get(position)).index<int32_t>(0) = pos;
    forward(m);
    std::memcpy(logits, m.get(model_pred).ptr<float>(), sizeof(float) * m.c.vocab_size);
}

// model.cpp:142-187 predict() on token ids (no tokenizer): tokens_out[t] = the token fed at position t,
// logits_out [max_length][vocab] (optional). Returns the number of forwards (= max_length).
int ref_model_predict(void* h, const int* prompt, int n_prompt, int max_length, int* tokens_out, float* logits_out) {
    auto& m = *static_cast<RefModel*>(h);
    auto& tok = const_cast<mem::Tensor&>(m.get(input_token));
    auto& posT = const_cast<mem::Tensor&>(m.get(position));
    int32_t pos = 0;
    tok.index<int32_t>(0) = prompt[pos];
    posT.index<int32_t>(0) = pos;
    while (pos < max_length) {
        tokens_out[pos] = tok.index<int32_t>(0);
        forward(m);
        if (logits_out)
            std::memcpy(logits_out + size_t(pos) * m.c.vocab_size, m.get(model_pred).ptr<float>(),
                        sizeof(float) * m.c.vocab_size);
        if (pos < n_prompt - 1) {
            pos++;
            posT.index<int32_t>(0) = pos;
            tok.index<int32_t>(0) = prompt[pos];
        } else {
            pos++;
            posT.index<int32_t>(0) = pos;
            m.argmax->forward(m.get(model_pred), tok);
        }
    }
    return pos;
}

}  // extern "C"
