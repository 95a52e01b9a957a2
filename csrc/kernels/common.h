// Shared device helpers for the gfx950 (CDNA4) kernels of ddp_amd.
//
// Conventions used by every kernel in this directory:
//  * activations are NHWC bf16 (channels contiguous = the GEMM K dimension of an
//    implicit-GEMM convolution), stored as raw 16-bit words (bf16_t);
//  * master parameters are fp32; kernels that feed MFMA read bf16 "shadow"
//    copies that the fused SGD kernel rewrites after every update;
//  * MFMA tile = v_mfma_f32_16x16x32_bf16.  Lane maps (cdna_hip_programming.md §3):
//      A[row = l&15][k = 8*(l>>4) + j],  B[k = 8*(l>>4) + j][col = l&15],  j = 0..7
//      D[row = 4*(l>>4) + r][col = l&15], r = 0..3
//    The convolution kernels put output CHANNELS on the MFMA rows and PIXELS on
//    the columns, so each lane ends with 4 consecutive channels of one pixel
//    (one 8-byte NHWC store per 16x16 tile).
//  * wave = 64 lanes; all reductions are fixed-order (bitwise reproducible).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels/types.h"

namespace ddp_amd {

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) short bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
typedef __attribute__((address_space(3))) char lds_char;
// LDS pointer to bf16 element elem_off of an LDS byte base (32-bit address arithmetic)
__device__ __forceinline__ lds_bf16x4* lds_ptr4(lds_char* base, int elem_off) {
  return (lds_bf16x4*)(base + 2 * elem_off);
}
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2v;  // v_dot2c_f32_bf16 operand

constexpr int WAVE = 64;

// Block barrier that orders LDS only: each wave waits for its own LDS (and scalar-memory)
// operations, then s_barrier.  HIP's __syncthreads() also drains vmcnt, i.e. waits for the
// wave's outstanding GLOBAL loads and stores - a prefetch meant to land during the next
// phase, or write-through stores nobody in the block reads, would be waited for.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ---- diagnostic in-kernel phase stamps (scripts/stamps.py) ---------------------------
// Each kernel TU has its own device pointer (set by stamps_set(); null in normal runs,
// so a stamp costs one scalar load + branch).  DDP_STAMP(kid, slot) makes lane 0 of the
// block's first wave store the 100 MHz constant-rate clock (s_memrealtime, comparable
// across CUs) at buf[kid][block][slot]; kid = kernel id (STAMP_K_*), 8 slots per block.
// Blocks with blockIdx.y > 0 do not stamp: gridDim comes from the implicit kernel
// arguments through a vector load, and its wait (vmcnt in order) would also wait for
// every load the wave has in flight - a stamp must not change the schedule it measures.
namespace {
__constant__ unsigned long long* g_stamp_buf = nullptr;  // constant: a scalar load, no vmcnt wait
}
#define DDP_STAMP(kid, slot)                                                                 \
  do {                                                                                       \
    unsigned long long* _sb = g_stamp_buf;                                                   \
    if (_sb && threadIdx.x == 0 && blockIdx.y == 0 && blockIdx.x < 4096)                    \
      _sb[(kid) * STAMP_KSTRIDE + blockIdx.x * STAMP_SLOTS + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define DDP_STAMPS_SETTER(name)                                                              \
  void name(void* p) { (void)hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_buf), &p, sizeof(p)); }

__device__ __forceinline__ float bf2f(bf16_t b) {
  return __builtin_bit_cast(float, ((unsigned)b) << 16);
}
__device__ __forceinline__ bf16_t f2bf(float f) {  // RNE, NaN-preserving (v_cvt_pk_bf16_f32)
  return __builtin_bit_cast(bf16_t, (__bf16)f);
}
__device__ __forceinline__ float bf16_round(float f) { return bf2f(f2bf(f)); }

__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
  return z;
}
__device__ __forceinline__ bf16x8 ld8(const bf16_t* p) {  // 16-byte global load
  return *reinterpret_cast<const bf16x8*>(p);
}
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ---- 16-byte blobs (staging copies, any element type) --------------------------------
__device__ __forceinline__ bf16x8 ld16(const void* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ void st16(void* p, bf16x8 v) { *reinterpret_cast<bf16x8*>(p) = v; }

// ---- element-type traits of the MFMA convolution kernels ------------------------------
// The conv kernels are written once over an activation/weight element type T:
//  * bf16_t: one v_mfma_f32_16x16x32_bf16 per 32-wide K step; lane l's fragment is the 8
//    contiguous elements k = 8(l>>4) + j (common.h header);
//  * float (exact fp32, the reference's precision): eight v_mfma_f32_16x16x4_f32 per
//    32-wide K step; lane l's fragment is k = 4(l>>4) + j (lo) and 16 + 4(l>>4) + j (hi),
//    j = 0..3 - MFMA j pairs A[row][k] with B[k][col] from the SAME lane group, so the
//    eight products sum the whole K step.  Two ds_read_b128 per fragment, each with the
//    bf16 form's 4-dword-per-lane-group offsets, so the same "row stride = 8 mod 16
//    dwords" padding keeps both conflict-free.  Result = an exact k-ordered fp32 fma chain
//    (cdna_hip_programming.md §3 'FP32-input MFMA'); no xf32 on gfx950.
struct F32Frag {
  f32x4 lo, hi;
};
template <typename T>
struct Prec;
template <>
struct Prec<bf16_t> {
  using Frag = bf16x8;
  static constexpr int CE = 8;    // elements per 16-byte chunk
  static constexpr int PAD = 16;  // LDS row pad (elements): 8 dwords
  static __device__ __forceinline__ int kofs(int lane) { return 8 * (lane >> 4); }
  static __device__ __forceinline__ Frag frag(const bf16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }
  static __device__ __forceinline__ Frag zero() { return zero8(); }
  static __device__ __forceinline__ f32x4 mma(const Frag& a, const Frag& b, f32x4 c) { return mfma16(a, b, c); }
};
template <>
struct Prec<float> {
  using Frag = F32Frag;
  static constexpr int CE = 4;
  static constexpr int PAD = 8;
  static __device__ __forceinline__ int kofs(int lane) { return 4 * (lane >> 4); }
  static __device__ __forceinline__ Frag frag(const float* p) {
    return Frag{*reinterpret_cast<const f32x4*>(p), *reinterpret_cast<const f32x4*>(p + 16)};
  }
  static __device__ __forceinline__ Frag zero() { return Frag{{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}}; }
  static __device__ __forceinline__ f32x4 mma(const Frag& a, const Frag& b, f32x4 c) {
#pragma unroll
    for (int j = 0; j < 4; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.lo[j], b.lo[j], c, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.hi[j], b.hi[j], c, 0, 0, 0);
    return c;
  }
};
template <typename F>
__device__ __forceinline__ F fsel(bool ok, const F& v, const F& z) {
  return ok ? v : z;
}

// XCD-aware block order: workgroups are dispatched round-robin over the 8 XCDs (linear id
// % 8 = the XCD group), each with a private L2.  The remap gives XCD group k one
// contiguous range of the logical linear order, so blocks that share operand rows (e.g.
// every tile of one pixel chunk) hit one L2 instead of eight.  Bijective for any grid
// size: the first nb % 8 groups take one extra block.  Placement only changes speed.
__device__ __forceinline__ int xcd_remap(int b, int nb) {
  const int per = nb >> 3, rem = nb & 7, x = b & 7, i = b >> 3;
  return x < rem ? x * (per + 1) + i : rem * (per + 1) + (x - rem) * per + i;
}
// The logical (x, y, z) block of this workgroup after xcd_remap (x fastest).
__device__ __forceinline__ int3 xcd_block3() {
  const int gx = gridDim.x, gy = gridDim.y;
  const int b = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int l = xcd_remap(b, gx * gy * gridDim.z);
  return make_int3(l % gx, (l / gx) % gy, l / (gx * gy));
}

// 8 contiguous bytes = 4 bf16 packed from 4 floats
__device__ __forceinline__ uint2 pack4(float a, float b, float c, float d) {
  uint2 r;
  r.x = (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
  r.y = (unsigned)f2bf(c) | ((unsigned)f2bf(d) << 16);
  return r;
}
__device__ __forceinline__ void unpack4(uint2 v, float* o) {
  o[0] = __builtin_bit_cast(float, v.x << 16);
  o[1] = __builtin_bit_cast(float, v.x & 0xffff0000u);
  o[2] = __builtin_bit_cast(float, v.y << 16);
  o[3] = __builtin_bit_cast(float, v.y & 0xffff0000u);
}

// Element-wise ReLU mask of an 8-wide bf16 fragment by a second fragment (y > 0).
__device__ __forceinline__ bf16x8 mask8(bf16x8 g, bf16x8 y) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    // torch threshold_backward keeps grad unless (y <= 0): sign bit clear and not +0
    const unsigned short u = (unsigned short)y[j];
    const bool pos = (u & 0x8000u) == 0 && u != 0;
    r[j] = pos ? g[j] : (short)0;
  }
  return r;
}

// ReLU mask of a 16-byte blob of gradients by the matching blob of activations (y > 0)
template <typename T>
__device__ __forceinline__ bf16x8 mask16(bf16x8 g, bf16x8 y);
template <>
__device__ __forceinline__ bf16x8 mask16<bf16_t>(bf16x8 g, bf16x8 y) {
  return mask8(g, y);
}
template <>
__device__ __forceinline__ bf16x8 mask16<float>(bf16x8 g, bf16x8 y) {
  const f32x4 gf = __builtin_bit_cast(f32x4, g), yf = __builtin_bit_cast(f32x4, y);
  f32x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = yf[j] > 0.f ? gf[j] : 0.f;  // threshold_backward
  return __builtin_bit_cast(bf16x8, r);
}

// SimpleCNN conv1 (Cin = 1, 3x3): relu(b1[c] + sum_k w1[c*9+k] * v[k]) with exactly the
// FMA order of conv1_fwd_kernel, so kernels that recompute a1 instead of reading it
// from memory reproduce the stored bf16 values bit for bit.
__device__ __forceinline__ float conv1_eval(const float* w1, const float* b1, const float* v, int c) {
  float acc = b1[c];
#pragma unroll
  for (int k = 0; k < 9; ++k) acc = fmaf(w1[c * 9 + k], v[k], acc);
  return fmaxf(acc, 0.f);
}

// Recompute SimpleCNN's first layer a1 = relu(conv1(x)) (32 channels) into bf16 LDS
// rows, bit-identical to conv1_fwd_kernel (conv1_eval order).  Wave w of a 256-thread
// block owns channel group g = w (channels 8g..8g+7) for every position, so its conv1
// weights are wave-uniform: Conv1Group loads them ONCE per wave into registers (call
// conv1_group_load early - e.g. before the staging round - so the loads overlap it).
// With more than 4 waves, waves w and w + 4 share group w % 4 and split the positions
// (pos0 = 64 * (w / 4), pstride = 64 * waves / 4).
// The only LDS traffic is the 9 input taps and one 16-byte store per position.
//   valid(pos) -> position inside the image (else the row is zero-filled)
//   tap(pos, k) -> input value of tap k (0 outside the image)
//   dst(pos, g) -> bf16_t* of channels 8g..8g+7 of position pos
struct Conv1Group {
  float w[8][9];
  float b[8];
};
__device__ __forceinline__ Conv1Group conv1_group_load(const float* __restrict__ w1,
                                                       const float* __restrict__ b1, int g) {
  Conv1Group r;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
#pragma unroll
    for (int k = 0; k < 9; ++k) r.w[j][k] = w1[(8 * g + j) * 9 + k];
    r.b[j] = b1[8 * g + j];
  }
  return r;
}
__device__ __forceinline__ float conv1_eval_g(const Conv1Group& cg, const float* v, int j) {
  float acc = cg.b[j];
#pragma unroll
  for (int k = 0; k < 9; ++k) acc = fmaf(cg.w[j][k], v[k], acc);  // == conv1_eval
  return fmaxf(acc, 0.f);
}
template <typename T = bf16_t, typename ValidFn, typename TapFn, typename DstFn>
__device__ __forceinline__ void conv1_recompute_tile(int npos, const Conv1Group& cg, int g, int pos0,
                                                     int pstride, ValidFn valid, TapFn tap, DstFn dst) {
  for (int pos = pos0 + (threadIdx.x & 63); pos < npos; pos += pstride) {
    float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (valid(pos)) {
      float v[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) v[k] = tap(pos, k);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = conv1_eval_g(cg, v, j);
    }
    if constexpr (sizeof(T) == 4) {  // exact fp32 rows
      float* d = reinterpret_cast<float*>(dst(pos, g));
      *reinterpret_cast<float4*>(d) = make_float4(o[0], o[1], o[2], o[3]);
      *reinterpret_cast<float4*>(d + 4) = make_float4(o[4], o[5], o[6], o[7]);
    } else {
      uint4 pk;
      const uint2 lo = pack4(o[0], o[1], o[2], o[3]), hi = pack4(o[4], o[5], o[6], o[7]);
      pk.x = lo.x; pk.y = lo.y; pk.z = hi.x; pk.w = hi.y;
      *reinterpret_cast<uint4*>(dst(pos, g)) = pk;
    }
  }
}

// ---- system-scope (cross-GPU coherent) element access: sc0 sc1 global loads / stores
// (write-through; loads bypass the non-coherent caches).  Used for every byte another
// GPU reads over xGMI (kernels/allreduce.hip).
__device__ __forceinline__ float ld_sys(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- write-through stores for large once-read kernel outputs (split-K slabs, dZ2):
// agent-scope (sc1) stores leave L2 at store time instead of sitting dirty until the
// kernel-end write-back, which otherwise lengthens the next dependent launch boundary
// by ~bytes / 6 TB/s (MI355X_MICROARCH.md, price row 'boundary').
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(uint2* p, uint2 v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p),
                     ((unsigned long long)v.y << 32) | v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(bf16_t* p, bf16_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(float2* p, float2 v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p),
                     ((unsigned long long)__float_as_uint(v.y) << 32) | __float_as_uint(v.x),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(float4* p, float4 v) {  // two 8-byte write-through stores
  st_wt(reinterpret_cast<float2*>(p), make_float2(v.x, v.y));
  st_wt(reinterpret_cast<float2*>(p) + 1, make_float2(v.z, v.w));
}

// ---- optimizer element update (torch/optim/sgd.py _single_tensor_sgd semantics)
// destination index of element j (multiple of 4 for a quad) in the FCFRAG layout
__device__ __forceinline__ int fcfrag_index(int j, int HW, int C) {
  const int o = j / (HW * C);
  const int rem = j - o * HW * C;
  const int hw = rem / C, c = rem - (rem / C) * C;
  const int G = HW >> 4, T = C >> 4;
  return ((((o * G + (hw >> 4)) * T + (c >> 4)) * 4 + ((c >> 2) & 3)) * 16 + (hw & 15)) * 4 + (c & 3);
}

__device__ __forceinline__ float sgd_one(float v, float d, float* mb, const SgdArgs& a) {
  if (a.maximize) d = -d;
  if (a.weight_decay != 0.f) d = fmaf(a.weight_decay, v, d);
  if (a.momentum != 0.f) {
    const float buf = a.first_step ? d : fmaf(1.f - a.dampening, d, a.momentum * (*mb));
    *mb = buf;
    d = a.nesterov ? fmaf(a.momentum, buf, d) : buf;
  }
  return fmaf(-a.lr, d, v);
}

// ---- cross-lane reductions on DPP (VALU modifiers, no LDS round trips) --------------
// dpp<CTRL>(v): v of the lane selected by the DPP control (quad_perm 0x00-0xFF,
// row_half_mirror 0x141, row_mirror 0x140), all rows / banks enabled.
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                               0xF, 0xF, false));
}
// Sum / max over each 16-lane row (lanes sharing lane >> 4); every lane of the row
// gets the result.  Pairs, quads, halves, row: a fixed association order, identical
// on every lane (each step combines two equal-shaped partial sums commutatively).
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror
  v += dpp<0x140>(v);  // row_mirror
  return v;
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp<0xB1>(v));
  v = fmaxf(v, dpp<0x4E>(v));
  v = fmaxf(v, dpp<0x141>(v));
  v = fmaxf(v, dpp<0x140>(v));
  return v;
}
__device__ __forceinline__ float lane_bcast(float v, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}
// fixed-order sum over all 64 lanes (every lane gets the total): rows, then
// ((r0 + r1) + (r2 + r3)) from lane reads
__device__ __forceinline__ float wave_sum(float v) {
  v = row16_sum(v);
  return (lane_bcast(v, 0) + lane_bcast(v, 16)) + (lane_bcast(v, 32) + lane_bcast(v, 48));
}
// sum over the 16 lanes that share (lane >> 4)
__device__ __forceinline__ float sum16(float v) { return row16_sum(v); }
__device__ __forceinline__ float wave_max(float v) {
  v = row16_max(v);
  return fmaxf(fmaxf(lane_bcast(v, 0), lane_bcast(v, 16)), fmaxf(lane_bcast(v, 32), lane_bcast(v, 48)));
}

// Whole-batch softmax cross-entropy on one workgroup, fixed summation order.
// part: the fused conv2+fc epilogue's partial logits, one pair of [NO] rows per conv
// block of CH consecutive pixels of the flattened [B*HW] space: part[blk][slot][o],
// slot 0 = the image of the block's first pixel, slot 1 = the next image (CH <= HW).
// Image b's logits are the fixed-order sum over the blocks kb0..kb1 that touch it.
// Phase 0: thread b < B requests its row's label (a dependent step -> index -> label
// chain) before anything else.  Phase 1: one thread per logit (b, o) loads its <= 16
// block partials (clamped block index, masked) and adds the bias -> s_lg[b][o] (LDS
// scratch, B*NO floats; the prefetched labels go to s_lab, B ints).  Phase 2: one thread
// per logit again; each evaluates its row's max / sum-exp serially over the NO classes
// (same order in every thread of the row, so bit-identical) and then its own class.
// Writes dl[b*NO + o] = (softmax - onehot) * gscale and loss[b] = logsumexp - x[label].  Contains a __syncthreads(): every thread of the
// block must call it; dl / loss may be LDS or global, and the caller syncs before
// reading them.  Used by xent_rows (own kernel) and by the XENT prologue of fc_bwd, so
// both produce bit-identical values.
constexpr int XENT_MAX_BLK = 16;  // conv blocks per image: HW / CH + 2 <= 16
// The fc_bwd prologue's variant: the whole partial array (nblk * 2 * NO floats, 15.7 KB
// at B = 32) is copied to LDS with coalesced 16-byte loads issued FIRST in the kernel,
// then every logit sums its partials from LDS in the same fixed order.  (Per-logit
// global loads are 16 scattered 4-byte loads per thread: ~5k lane-addresses per block
// through the texture addresser, measured ~2 us.)
constexpr int XENT_PRE_Q = 4;  // float4 per thread held from the prefetch to the LDS write
// The two fixed-order pieces every producer of dL shares (xent_finish below, the fc_bwd
// prologue, and the level-3 conv forward that computes dZ2 itself): one inlined body each,
// so every caller evaluates the same float operations in the same order (bit-identical).
// Image b's raw logit o (before the bias): sum over the conv blocks kb0..kb1 touching it of
// part[kb][slot][o] (slot 1 only for a first block that started in the previous image).
template <typename Ld>
__device__ __forceinline__ float xent_logit_acc(int b, int o, int HW, int CH, int NO, Ld ld) {
  const int p0 = b * HW;
  const int kb0 = p0 / CH, kb1 = (p0 + HW - 1) / CH;
  const int slot0 = kb0 * CH == p0 ? 0 : 1;
  float a = 0.f;
#pragma unroll
  for (int j = 0; j < XENT_MAX_BLK; ++j) {
    const int kb = min(kb0 + j, kb1);
    const float v = ld((kb * 2 + (j == 0 ? slot0 : 0)) * NO + o);
    a += (kb0 + j <= kb1) ? v : 0.f;
  }
  return a;
}
// dL[o] of one row x[0..NO) (softmax - onehot, times gscale); *loss (if o == 0 and loss)
// = logsumexp - x[label].  label is clamped to [0, NO).
__device__ __forceinline__ float xent_row_dl(const float* x, int NO, int o, int label, float gscale,
                                             float* loss) {
  label = label < 0 ? 0 : (label >= NO ? NO - 1 : label);
  float mx = x[0];
  for (int k = 1; k < NO; ++k) mx = fmaxf(mx, x[k]);
  float se = 0.f;
  for (int k = 0; k < NO; ++k) se += __expf(x[k] - mx);
  const float inv = 1.f / se;
  if (o == 0 && loss) *loss = mx + __logf(se) - x[label];
  return (__expf(x[o] - mx) * inv - (o == label ? 1.f : 0.f)) * gscale;
}
struct XentPre {
  int lab0;
  float bias_o;  // bias[threadIdx.x % NO]
  float4 q[XENT_PRE_Q];
};
__device__ __forceinline__ void xent_prefetch(const float* __restrict__ part, int npart,
                                              const float* __restrict__ bias, int NO, int B,
                                              const int* __restrict__ labels32, const BatchIdx& bi,
                                              XentPre& pre) {
  const float4* p4 = reinterpret_cast<const float4*>(part);
  const int n4 = npart >> 2;
#pragma unroll
  for (int k = 0; k < XENT_PRE_Q; ++k) {
    const int i = threadIdx.x + k * blockDim.x;
    pre.q[k] = i < n4 ? p4[i] : make_float4(0.f, 0.f, 0.f, 0.f);  // fully defined: stays in VGPRs
  }
  pre.lab0 = (int)threadIdx.x < B ? labels32[bi.row(threadIdx.x, bi.base())] : 0;
  pre.bias_o = (int)threadIdx.x < B * NO ? bias[threadIdx.x % NO] : 0.f;
  DDP_STAMP(STAMP_K_XENT, 1);  // loads issued
}
// s_part: npart floats of LDS (may alias scratch the caller uses only afterwards).
__device__ __forceinline__ void xent_finish(const XentPre& pre, const float* __restrict__ part, int npart,
                                            int HW, int CH, const float* __restrict__ bias, int NO, int B,
                                            const int* __restrict__ labels32, const BatchIdx& bi,
                                            float gscale, float* dl, float* loss, float* s_lg, int* s_lab,
                                            float* s_part) {
  const int n4 = npart >> 2;
  float4* s4 = reinterpret_cast<float4*>(s_part);
#pragma unroll
  for (int k = 0; k < XENT_PRE_Q; ++k) {
    const int i = threadIdx.x + k * blockDim.x;
    if (i < n4) s4[i] = pre.q[k];
  }
  for (int i = threadIdx.x + XENT_PRE_Q * blockDim.x; i < n4; i += blockDim.x)
    s4[i] = reinterpret_cast<const float4*>(part)[i];
  if ((int)threadIdx.x < B) s_lab[threadIdx.x] = pre.lab0;
  __syncthreads();
  DDP_STAMP(STAMP_K_XENT, 2);  // partials in LDS
  // the thread's first logit uses only prefetched / LDS operands; later logits (B * NO >
  // blockDim) run in a separate guarded loop - a global load the compiler may hoist into
  // the first iteration would wait (vmcnt in order) for all of the caller's column loads
  auto logit_sum = [&](int t) {
    const int b = t / NO, o = t - (t / NO) * NO;
    return xent_logit_acc(b, o, HW, CH, NO, [&](int i) { return s_part[i]; });
  };
  if ((int)threadIdx.x < B * NO) s_lg[threadIdx.x] = pre.bias_o + logit_sum(threadIdx.x);
  if (B * NO > (int)blockDim.x)
    for (int t = threadIdx.x + blockDim.x; t < B * NO; t += blockDim.x) s_lg[t] = bias[t % NO] + logit_sum(t);
  DDP_STAMP(STAMP_K_FC_BWD, 5);
  __syncthreads();
  DDP_STAMP(STAMP_K_FC_BWD, 6);
  auto row_out = [&](int t, int label) {
    const int b = t / NO, o = t - (t / NO) * NO;
    dl[t] = xent_row_dl(s_lg + b * NO, NO, o, label, gscale, loss + b);
  };
  // first logit: b = threadIdx.x / NO < blockDim, so its label is in s_lab (no pointer
  // select: the compiler would merge LDS / global into one flat load counted in vmcnt)
  if ((int)threadIdx.x < B * NO) row_out(threadIdx.x, s_lab[threadIdx.x / NO]);
  if (B * NO > (int)blockDim.x)
    for (int t = threadIdx.x + blockDim.x; t < B * NO; t += blockDim.x) {
      const int b = t / NO;
      row_out(t, b < (int)blockDim.x ? s_lab[b] : labels32[bi.row(b, bi.base())]);
    }
  DDP_STAMP(STAMP_K_FC_BWD, 7);
}
__device__ __forceinline__ void xent_batch_block(const float* __restrict__ part, int HW, int CH,
                                                 const float* __restrict__ bias, int NO, int B,
                                                 const int* __restrict__ labels32, const BatchIdx& bi,
                                                 float gscale, float* dl, float* loss, float* s_lg,
                                                 int* s_lab) {
  const int base = bi.base();
  const int lab0 = (int)threadIdx.x < B ? labels32[bi.row(threadIdx.x, base)] : 0;
  for (int t = threadIdx.x; t < B * NO; t += blockDim.x) {
    // 32-bit index math only (B * HW < 2^31, checked on the host): 64-bit divisions
    // by runtime values are long software sequences.  Block kb0 is the only one that can
    // start in the previous image (slot 1); every later block starts inside image b.
    const int b = t / NO, o = t - (t / NO) * NO;
    s_lg[t] = bias[o] + xent_logit_acc(b, o, HW, CH, NO, [&](int i) { return part[i]; });
  }
  if ((int)threadIdx.x < B) s_lab[threadIdx.x] = lab0;
  __syncthreads();
  // Phase 2, one thread per logit again: every thread of row b evaluates the row's max
  // and sum-exp in the same serial order (bit-identical values), then its own class.
  for (int t = threadIdx.x; t < B * NO; t += blockDim.x) {
    const int b = t / NO, o = t - (t / NO) * NO;
    const int label = b < (int)blockDim.x ? s_lab[b] : labels32[bi.row(b, base)];
    dl[t] = xent_row_dl(s_lg + b * NO, NO, o, label, gscale, loss + b);
  }
}

}  // namespace ddp_amd
