// model.cpp — drop-in model::LlamaModel over the fused engine (reference: source/model/model.cpp).
#include "model.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <iostream>
#include <sstream>

namespace model {

RawModelData::~RawModelData() {
    if (data && data != MAP_FAILED) munmap(data, file_size);
    if (fd != -1) close(fd);
}

bool RawModelData::open_file(const std::string& path) {
    fd = open(path.c_str(), O_RDONLY);
    if (fd == -1) return false;
    struct stat sb;
    if (fstat(fd, &sb) == -1) return false;
    file_size = (size_t)sb.st_size;
    data = mmap(nullptr, file_size, PROT_READ, MAP_PRIVATE, fd, 0);
    if (data == MAP_FAILED) {  // the reference checks !ptr (model.cpp:242); mmap reports MAP_FAILED
        data = nullptr;
        return false;
    }
    weight_data = data;
    return true;
}

const void* RawModelDataFp32::weight(size_t offset) const { return static_cast<const float*>(weight_data) + offset; }

namespace {
int to_sli(base::DataType t) {
    return t == base::DataType::kFp16 ? SLI_DT_F16 : t == base::DataType::kInt8 ? SLI_DT_I8 : SLI_DT_F32;
}
void check(int rc, const char* what) {
    if (rc != SLI_OK) LOG(std::string(what) + ": " + sli_status_str(rc) + " (" + sli_last_error() + ")");
}
}  // namespace

LlamaModel::LlamaModel(std::string tokenizer_path, std::string model_path, base::DeviceType device_type)
    : LlamaModel(std::move(tokenizer_path), std::move(model_path), device_type, LlamaModelConfig{}, EngineOptions{}) {}

LlamaModel::LlamaModel(std::string tokenizer_path, std::string model_path, base::DeviceType device_type,
                       const LlamaModelConfig& config, EngineOptions options)
    : config_(std::make_unique<LlamaModelConfig>(config)),
      tokenizer_path_(std::move(tokenizer_path)),
      model_path_(std::move(model_path)),
      device_type_(device_type),
      options_(std::move(options)) {}

LlamaModel::~LlamaModel() {
    if (engine_) sli_model_destroy(engine_);
}

void LlamaModel::read_model_file() {
    if (model_path_.empty()) LOG("No model weigth file!\n");
    auto raw = std::make_shared<RawModelDataFp32>();
    if (!raw->open_file(model_path_)) LOG("Fail to open the weight file!\n");
    raw_model_data_ = raw;
}

void LlamaModel::init() {
    if (device_type_ != base::DeviceType::kDeviceCUDA) LOG("Device Type ERROR!");  // HIP backend only
    const LlamaModelConfig& c = *config_;
    if (c.num_key_value_heads * c.head_dim != c.kv_hidden_size) LOG("kv_hidden_size != num_key_value_heads * head_dim");
    sli_model_config mc{};
    mc.vocab = c.vocab_size;
    mc.dim = c.hidden_size;
    mc.n_heads = c.num_attention_heads;
    mc.n_kv_heads = c.num_key_value_heads;
    mc.head_dim = c.head_dim;
    mc.ffn = c.intermediate_size;
    mc.n_layers = c.num_hidden_layers;
    mc.max_len = c.max_length;
    mc.eps = c.rms_norm_eps;
    mc.theta = c.rope_theta;
    mc.w_dtype = to_sli(options_.weight_type);
    mc.kv_dtype = to_sli(options_.kv_type);
    mc.act_mode = options_.act_mode;
    mc.tp_rank = options_.tp_rank;
    mc.tp_size = options_.tp_size;
    mc.device = options_.device;
    check(sli_model_create(&mc, options_.comm_id.empty() ? nullptr : options_.comm_id.data(), &engine_),
          "sli_model_create");
    if (!model_path_.empty()) {
        read_model_file();  // validates the path the way the reference does, then streams it to the device
        check(sli_model_load_flat(engine_, model_path_.c_str()), "sli_model_load_flat");
    } else if (options_.synthetic_seed >= 0) {
        check(sli_model_init_synthetic(engine_, (uint32_t)options_.synthetic_seed), "sli_model_init_synthetic");
    } else {
        LOG("No model weigth file!\n");
    }
}

void LlamaModel::set_input(int32_t token, int32_t pos) {
    check(sli_model_set_state(engine_, token, pos, 0), "sli_model_set_state");
}

void LlamaModel::forward() {
    check(sli_model_step(engine_), "sli_model_step");
    check(sli_model_sync(engine_), "sli_model_sync");
}

std::vector<float> LlamaModel::logits() const {
    const int32_t chunk = (config_->vocab_size + options_.tp_size - 1) / options_.tp_size;
    std::vector<float> out(chunk);
    int32_t lo = 0;
    check(sli_model_get_logits(engine_, out.data(), chunk, &lo), "sli_model_get_logits");
    out.resize(std::min(chunk, config_->vocab_size - lo));
    return out;
}

std::vector<int32_t> LlamaModel::predict_ids(const std::vector<int32_t>& prompt, int max_length,
                                             std::vector<float>* logits) {
    if (prompt.empty()) LOG("empty prompt");
    std::vector<int32_t> toks(max_length);
    // rows of the returned logits are this rank's actual vocab shard (the engine's row stride), which is
    // shorter than ceil(V / tp) on the last rank when tp_size does not divide the vocab
    int32_t lo = 0, vn = 0;
    const int32_t chunk = (config_->vocab_size + options_.tp_size - 1) / options_.tp_size;
    lo = std::min(config_->vocab_size, options_.tp_rank * chunk);
    vn = std::max(0, std::min(chunk, config_->vocab_size - lo));
    if (logits) logits->assign((size_t)max_length * vn, 0.0f);
    check(sli_model_predict(engine_, prompt.data(), (int32_t)prompt.size(), max_length, toks.data(),
                            logits ? logits->data() : nullptr),
          "sli_model_predict");
    return toks;
}

// model.cpp:142-187 on token ids: prints the fed token ids (prompt then greedy), space-separated.
void LlamaModel::predict(const std::string prompt, const int max_length) {
    std::istringstream in(prompt);
    std::vector<int32_t> ids;
    for (int32_t t; in >> t;) ids.push_back(t);
    const std::vector<int32_t> toks = predict_ids(ids, max_length);
    for (int32_t t : toks) std::cout << t << " ";
    std::cout << std::endl;
}

}  // namespace model
