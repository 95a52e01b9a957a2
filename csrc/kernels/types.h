// Types shared by device code and host code (runtime, pybind layer).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ddp_amd {

typedef unsigned short bf16_t;  // bf16 storage word

// Batch-index source for kernels that read the training batch straight out of
// the device-resident dataset.  offset = (*step_ctr) * batch_stride when
// step_ctr != nullptr (graph-replayable), else `offset` is used as is.
// Both lookups are clamped (n_idx = length of the index list, n_rows = dataset
// rows): a mis-sized replay must never become an out-of-bounds gather.
// idx == nullptr: the rows are already in epoch order (the fused engine permutes the
// dataset once per epoch), row = base + b - one dependent load fewer per step.
struct BatchIdx {
  const int* idx;       // epoch index list (int32), nullptr -> rows base + b
  const int* step_ctr;  // device step counter or nullptr
  int batch_stride;
  int offset;
  int n_idx = 0x7fffffff;
  int n_rows = 0x7fffffff;
  __device__ __forceinline__ int base() const {
    return step_ctr ? (*step_ctr) * batch_stride : offset;
  }
  __device__ __forceinline__ int row(int b, int base_) const {
    if (!idx) {
      const int r = base_ + b;
      return r < 0 ? 0 : (r >= n_rows ? n_rows - 1 : r);
    }
    int i = base_ + b;
    i = i < 0 ? 0 : (i >= n_idx ? n_idx - 1 : i);
    int r = idx[i];
    return r < 0 ? 0 : (r >= n_rows ? n_rows - 1 : r);
  }
};

// Source of SimpleCNN's first-layer activation when a kernel recomputes it on the fly
// (a1 = relu(conv1(x0[idx])) / bf16) instead of reading a stored a1 tensor.
struct C1Src {
  const unsigned char* x = nullptr;  // uint8 dataset [rows][H*W]
  BatchIdx bi{};
  const float* w = nullptr;          // conv1 weight [32][9]
  const float* b = nullptr;          // conv1 bias [32]
  // conv3x3_fwd only (optional): write the step's batch compactly - images xb[B][H*W]
  // (uint8) and labels yb[B] (from `labels` through bi) - so that the backward kernels
  // read it directly (identity BatchIdx) instead of repeating the step -> index -> row
  // lookup chain (two dependent memory round trips each).
  unsigned char* xb_out = nullptr;
  int* yb_out = nullptr;
  const int* labels = nullptr;
  // conv3x3_fwd only (optional): also store the recomputed a1 of the block's own pixels
  // (NHWC bf16, [B*H*W][Cin]) so the backward reads it instead of recomputing conv1
  bf16_t* a1_out = nullptr;
  // conv3x3_fwd only (optional): block b zeroes zero_i32[b * zero_per_block ...] - the
  // step's in-launch hand-off flags (fuse level 2), reset by the step's first kernel
  int* zero_i32 = nullptr;
  int zero_per_block = 0;
  int zero_total = 0x7fffffff;  // ints [0, zero_total) only (the words past it belong to others)
};

// torch.optim.SGD hyper-parameters of one step (first_step: momentum buffer init;
// update == 0: shadows only)
struct SgdArgs {
  float lr, momentum, dampening, weight_decay;
  int nesterov, maximize, first_step, update;
};

// diagnostic phase-stamp kernel ids / buffer geometry (common.h DDP_STAMP)
enum { STAMP_K_CONV_FWD = 0, STAMP_K_FC_BWD = 1, STAMP_K_DGRAD = 2, STAMP_K_WGRAD = 3,
       STAMP_K_GRAD_REDUCE = 4, STAMP_K_SGD = 5, STAMP_K_XENT = 6, STAMP_K_CONV1 = 7,
       STAMP_K_FWD_DZ = 8, STAMP_K_XGMI = 9, STAMP_K_HEAD = 10, STAMP_K_COUNT = 11 };
constexpr int STAMP_SLOTS = 8, STAMP_KSTRIDE = 4096 * STAMP_SLOTS;

}  // namespace ddp_amd
