// model.h — drop-in for the reference's model::LlamaModel (include/model/model.h:59-89): init(),
// forward() (one decode step), predict(prompt, max_length) (teacher-forced prompt + greedy decode).
// The device work is libsli.so's fused, graph-captured step (sli_model_*). Prompts are whitespace-
// separated token ids (the sentencepiece tokenizer is out of scope); predict prints token ids.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "base.h"
#include "config.h"
#include "sli.h"
#include "weight_loader.h"

namespace model {

enum class ModelBufferType {  // model.h:14-34 (kept for source compatibility)
    input_token = 0, position = 1, key_cache = 2, value_cache = 3, emb_output = 4, rms_output = 5, query = 6,
    score = 7, mha_output = 8, att_output = 9, ffn_input = 10, up_output = 11, gate_output = 12, down_output = 13,
    swi_output = 14, ffn_output = 15, model_pred = 16, sin_cache = 17, cos_cache = 18,
};

struct EngineOptions {  // extension: storage types, activation variant and tensor parallelism
    base::DataType weight_type = base::DataType::kFp32;  // fp32 = the reference's numerics
    base::DataType kv_type = base::DataType::kFp32;
    int act_mode = 0;  // 0: sigmoid(gate)*up (swiglu_kernel.cpp:12-13); 1: SiLU
    int tp_rank = 0, tp_size = 1, device = 0;
    std::vector<char> comm_id;  // RCCL unique id (tp_size > 1)
    int synthetic_seed = -1;    // >= 0 and no model_path: seeded synthetic weights (include/sli_synth.h)
};

class LlamaModel {
public:
    explicit LlamaModel(std::string tokenizer_path, std::string model_path, base::DeviceType device_type);
    LlamaModel(std::string tokenizer_path, std::string model_path, base::DeviceType device_type,
               const LlamaModelConfig& config, EngineOptions options);
    ~LlamaModel();
    LlamaModel(const LlamaModel&) = delete;
    LlamaModel& operator=(const LlamaModel&) = delete;

    void init();
    void forward();
    void predict(const std::string prompt, const int max_length);

    // extensions over the reference API
    void set_input(int32_t token, int32_t pos);
    std::vector<int32_t> predict_ids(const std::vector<int32_t>& prompt, int max_length,
                                     std::vector<float>* logits = nullptr);
    std::vector<float> logits() const;  // this rank's vocab shard of the last step
    const LlamaModelConfig& config() const { return *config_; }
    sli_model* engine() const { return engine_; }

protected:
    void read_model_file();

    std::unique_ptr<LlamaModelConfig> config_;
    std::string tokenizer_path_;
    std::string model_path_;
    std::shared_ptr<RawModelData> raw_model_data_;
    base::DeviceType device_type_ = base::DeviceType::kDeviceUnknown;
    EngineOptions options_;
    sli_model* engine_ = nullptr;
};

}  // namespace model
