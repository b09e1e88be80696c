// ops_internal.h — launchers shared between the kernel-level ABI (ops.hip) and the engine (engine.hip).
#pragma once
#include "attention.h"
#include "common.h"

namespace sli {

template <typename KT>
int mha_launch(const float* q, const KT* kc, const KT* vc, float* out, int layer, int pos, const int32_t* pos_dev,
               int T, int hd, int H, int Hkv, long long pos_stride, long long head_stride, long long layer_stride,
               float* part, unsigned* counters, hipStream_t s, int seq_heads = 0, int pos_seq_stride = 0,
               int cache_heads = 0, int defer_merge = 0);

size_t mha_part_bytes(int T, int H, int hd);       // split partials [H][splits][hd + pad], 256-B aligned
size_t mha_workspace_bytes(int T, int H, int hd);  // partials + per-kv-head arrival counters
int attn_wg_positions(int kv_dtype, int head_dim);  // context positions per attention workgroup

int embedding_launch(int token, const int32_t* token_dev, const void* table, int dtype, const float* row_scale,
                     float* out, int vocab, int dim, hipStream_t s);

}  // namespace sli
