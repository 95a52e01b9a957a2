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
struct BatchIdx {
  const int* idx;       // epoch index list (int32), nullptr -> identity (row b)
  const int* step_ctr;  // device step counter or nullptr
  int batch_stride;
  int offset;
  int n_idx = 0x7fffffff;
  int n_rows = 0x7fffffff;
  __device__ __forceinline__ int base() const {
    return step_ctr ? (*step_ctr) * batch_stride : offset;
  }
  __device__ __forceinline__ int row(int b, int base_) const {
    if (!idx) return b;
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
};

}  // namespace ddp_amd
