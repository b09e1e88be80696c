// dropin_llama.cpp — a reference-style client of the drop-in C++ API (include/op, include/memory,
// include/model). Part 1 rebuilds LlamaModel::forward/predict op by op exactly as the reference's
// source/model/model.cpp:40-187 and :336-469 do (mmap'd flat fp32 weights, set_weight + to_cuda,
// slice_KV_cache views, one op::Layer::forward per op), running on the HIP backend
// (DeviceType::kDeviceCUDA). Part 2 runs model::LlamaModel (the fused graph-captured engine) on the
// same file. Both write tokens and per-step logits; tests/test_gpu_dropin.py compares them with the
// oracle.
//
// usage: dropin_llama <weights.bin> <out_prefix> <max_length> V D H KV_HEADS HD I L T THETA [prompt ids...]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <memory>
#include <vector>

#include "kernels.h"
#include "model.h"
#include "ops.h"

using base::DeviceType;

static void dump(const std::string& path, const std::vector<int32_t>& toks, const std::vector<float>& logits) {
    std::ofstream f(path, std::ios::binary);
    const int32_t n = (int32_t)toks.size();
    f.write((const char*)&n, 4);
    f.write((const char*)toks.data(), 4 * toks.size());
    f.write((const char*)logits.data(), 4 * logits.size());
}

int main(int argc, char** argv) {
    if (argc < 14) {
        std::fprintf(stderr, "usage: %s weights out max_len V D H KVH HD I L T THETA [ids...]\n", argv[0]);
        return 2;
    }
    const std::string wpath = argv[1], out = argv[2];
    const int max_length = std::atoi(argv[3]);
    model::LlamaModelConfig cfg;
    cfg.vocab_size = std::atoi(argv[4]);
    cfg.hidden_size = std::atoi(argv[5]);
    cfg.num_attention_heads = std::atoi(argv[6]);
    cfg.num_key_value_heads = std::atoi(argv[7]);
    cfg.head_dim = std::atoi(argv[8]);
    cfg.intermediate_size = std::atoi(argv[9]);
    cfg.num_hidden_layers = std::atoi(argv[10]);
    cfg.max_length = std::atoi(argv[11]);
    cfg.rope_theta = (float)std::atof(argv[12]);
    cfg.kv_hidden_size = cfg.num_key_value_heads * cfg.head_dim;
    std::vector<int32_t> prompt;
    for (int i = 13; i < argc; ++i) prompt.push_back(std::atoi(argv[i]));
    const int V = cfg.vocab_size, D = cfg.hidden_size, KV = cfg.kv_hidden_size, I = cfg.intermediate_size;
    const int L = cfg.num_hidden_layers, T = cfg.max_length, hd = cfg.head_dim;
    const DeviceType dev = DeviceType::kDeviceCUDA;

    // ---------------- part 1: op by op (model.cpp:336-469 layer construction)
    model::RawModelDataFp32 raw;
    if (!raw.open_file(wpath)) LOG("Fail to open the weight file!\n");
    size_t pw = 0;
    auto emb = std::make_shared<op::EmbeddingLayer>(dev, V, D);
    emb->set_weight(0, {V, D}, raw.weight(pw), DeviceType::kDeviceCPU);
    emb->to_cuda();
    auto cls = std::make_shared<op::MatmulLayer>(dev, V, D);  // tied LM head: same offset as the embedding
    cls->set_weight(0, {V, D}, raw.weight(pw), DeviceType::kDeviceCPU);
    cls->to_cuda();
    pw += (size_t)V * D;
    std::vector<std::shared_ptr<op::RmsNormLayer>> norms;
    for (int i = 0; i < 2 * L + 1; ++i, pw += D) {
        norms.push_back(std::make_shared<op::RmsNormLayer>(dev, D, cfg.rms_norm_eps));
        norms.back()->set_weight(0, {D}, raw.weight(pw), DeviceType::kDeviceCPU);
        norms.back()->to_cuda();
    }
    auto linear = [&](int rows, int cols) {
        std::vector<std::shared_ptr<op::MatmulLayer>> v;
        for (int l = 0; l < L; ++l, pw += (size_t)rows * cols) {
            v.push_back(std::make_shared<op::MatmulLayer>(dev, rows, cols));
            v.back()->set_weight(0, {rows, cols}, raw.weight(pw), DeviceType::kDeviceCPU);
            v.back()->to_cuda();
        }
        return v;
    };
    auto wq = linear(D, D), wk = linear(KV, D), wv = linear(KV, D), wo = linear(D, D);
    auto up = linear(I, D), gate = linear(I, D), down = linear(D, I);
    auto rope = std::make_shared<op::RoPELayer>(dev, D, hd);
    auto mha = std::make_shared<op::MultiHeadAttention>(dev, T, hd, cfg.num_attention_heads, cfg.num_key_value_heads);
    auto add = std::make_shared<op::VecAddLayer>(dev, D);
    auto swiglu = std::make_shared<op::SwigluLayer>(dev, I);
    op::argmaxLayer argmax(DeviceType::kDeviceCPU, V);  // host argmax, as model.cpp create_nonparam_layers makes it

    auto da = mem::CUDADeviceAllocatorFactory::get_instance();
    auto ca = mem::CPUDeviceAllocatorFactory::get_instance();
    mem::Tensor input_token({1}, true, ca), position({1}, true, ca);  // host scalars (model.cpp:258-262)
    mem::Tensor kc({L, T, KV}, true, da), vc({L, T, KV}, true, da);
    da->memset_zero(kc.ptr<void>(), kc.byte_size());
    da->memset_zero(vc.ptr<void>(), vc.byte_size());
    mem::Tensor x({D}, true, da), h({D}, true, da), q({D}, true, da), score({hd, T}, true, da), attn({D}, true, da),
        o({D}, true, da), x1({D}, true, da), u({I}, true, da), g({I}, true, da), a({I}, true, da), f({D}, true, da),
        logits({V}, true, da), sin_c({T, hd / 2}, true, da), cos_c({T, hd / 2}, true, da);
    kernel::rope_cache_cal_cuda(hd, T, sin_c, cos_c, cfg.rope_theta);

    std::vector<int32_t> toks1;
    std::vector<float> log1;
    int32_t pos = 0;
    input_token.index<int32_t>(0) = prompt[0];
    position.index<int32_t>(0) = 0;
    while (pos < max_length) {  // model.cpp:157
        toks1.push_back(input_token.index<int32_t>(0));
        emb->forward(input_token, x);  // model.cpp:48
        for (int l = 0; l < L; ++l) {
            norms[2 * l]->forward(x, h);
            const auto& [k, v] = mem::slice_KV_cache(l, pos, T, KV, kc, vc);
            wq[l]->forward(h, q);
            wk[l]->forward(h, k);
            wv[l]->forward(h, v);
            rope->forward(q, k, position, sin_c, cos_c);
            mha->set_pos(pos);
            mha->set_layer_index(l);
            mha->forward(q, score, kc, vc, attn);
            wo[l]->forward(attn, o);
            add->forward(x, o, x1);
            norms[2 * l + 1]->forward(x1, h);
            up[l]->forward(h, u);
            gate[l]->forward(h, g);
            swiglu->forward(u, g, a);
            down[l]->forward(a, f);
            add->forward(f, x1, x);
        }
        norms[2 * L]->forward(x, h);
        cls->forward(h, logits);
        mem::Tensor pred_cpu({V}, true, ca);  // model.cpp:175-179: logits to the host, then the host argmax
        ca->memcpy(logits.ptr<float>(), pred_cpu.ptr<float>(), 4 * (size_t)V, base::MemcpyKind::kMemcpyCUDA2CPU);
        log1.insert(log1.end(), pred_cpu.ptr<float>(), pred_cpu.ptr<float>() + V);
        if (pos < (int)prompt.size() - 1) {
            input_token.index<int32_t>(0) = prompt[++pos];
        } else {
            ++pos;
            argmax.forward(pred_cpu, input_token);
        }
        position.index<int32_t>(0) = pos;
    }
    dump(out + ".ops.bin", toks1, log1);

    // ---------------- part 2: model::LlamaModel (fused engine) on the same file
    model::EngineOptions opt;  // fp32 weights and KV: the reference's numerics
    model::LlamaModel m("", wpath, dev, cfg, opt);
    m.init();
    std::vector<float> log2;
    const std::vector<int32_t> toks2 = m.predict_ids(prompt, max_length, &log2);
    dump(out + ".engine.bin", toks2, log2);
    double mx = 0.0;
    for (size_t i = 0; i < log1.size(); ++i) mx = std::max(mx, (double)std::abs(log1[i] - log2[i]));
    std::printf("dropin ok: steps %d, tokens %s, max |ops - engine| logit %.3g\n", max_length,
                toks1 == toks2 ? "equal" : "DIFFER", mx);
    return toks1 == toks2 ? 0 : 1;
}
