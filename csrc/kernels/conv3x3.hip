// 3x3 / stride 1 / padding 1 convolution on NHWC activations with MFMA: forward, data
// gradient and weight gradient, in two precisions (element type T, common.h Prec<T>):
//  * bf16 operands on v_mfma_f32_16x16x32_bf16 (fp32 accumulate) - the default;
//  * exact fp32 operands on v_mfma_f32_16x16x4_f32 - the reference's precision
//    (--dtype fp32): same tiling, LDS staging and fusions, 8 MFMAs per 32-wide K step.
//
// Reference op: model.py:11-12 (nn.Conv2d(32,64,3,padding=1) -> nn.ReLU()), i.e.
// the layer that carries 95% of SimpleCNN's FLOPs.
//
// Implicit GEMM, output channels on the MFMA rows and pixels on the columns:
//   fwd   D[co][px] += W[co][tap][ci]   . X[px+tap][ci]        K = 9*Cin
//   dgrad D[ci][px] += WT[tap][ci][co]  . dY[px-tap][co]       K = 9*Cout
//   wgrad D[co][ci] += dY[px][co]       . X[px+tap][ci]        K = pixels (per tap)
// A K-step of 32 is one tap x 32 contiguous channels, so every A/B fragment is a
// single 16-byte load of 8 contiguous bf16 (fp32: two 16-byte loads).  Each lane
// finishes with 4 consecutive channels of one pixel -> one 8-byte (fp32: 16-byte) NHWC
// store per 16x16 tile.
//
// Fusions (templates):
//  * fwd:   bias + ReLU epilogue; FUSE_FC additionally dots the bf16 output tile
//           with the following Linear layer's weight (SimpleCNN's fc, given in
//           the MFMA-fragment order of SHADOW_BF16_FCFRAG so every lane's 8-byte
//           slice of a wave-instruction is contiguous) and writes per-16-pixel
//           partial logits, so the fc forward never re-reads the activation
//           (SURVEY.md §2.4 K5 note).
//  * dgrad: ReLU mask of the upstream gradient (MASK_DY, module path) and of the
//           layer input (MASK_X: d(relu1)); FUSE_W1 accumulates conv1's weight
//           and bias gradient from the just-computed dZ1 (Cin=1 conv, K11).
//  * wgrad: split-K over image-row chunks, one fp32 slab row per block, bias
//           gradient from an extra MFMA against a ones fragment; fixed-order
//           reduction in grad_reduce (bitwise reproducible, no float atomics).
#include <algorithm>
#include <stdexcept>

#include <cstdio>
#include <cstdlib>

#include "kernels/conv3x3_fwd.h"

namespace ddp_amd {

size_t conv3x3_fwd_lds(int W, int Cin, int pxt, bool a1x, int es) {
  return fwd_stage_lds(W, Cin, pxt, a1x, es) + fc_epi_lds(pxt, FC_MAX_NOF);
}

size_t conv3x3_dgrad_lds(int W, int Cout, int pxt, bool fuse_w1, int es) {
  const size_t XR = 64 * pxt + 2 * W + 2;
  const int pad = es == 2 ? 16 : 8;  // Prec<T>::PAD
  return (size_t)es * ((size_t)32 * (9 * Cout + pad) + XR * (Cout + pad)) +
         (fuse_w1 ? sizeof(float) * (XR + 4 * 320) + 4 * 64 * pxt : 0);
}

bool conv3x3_fwd_dz_fits(int B, int H, int W, int pxt, int es) {
  return es == 4 ? fwd_dz_fits<float>(B, H, W, pxt) : fwd_dz_fits<bf16_t>(B, H, W, pxt);
}

// ---------------------------------------------------------------- dist_mode 4 step head
// Step k's two bucket all-reduces (+ fused SGD, stored write-through) and step k + 1's bf16
// level-3 forward (256-thread blocks, pxt 1) in ONE launch: blocks [0, nblk1) all-reduce the
// conv bucket, the next nblk0 the fc bucket (xgmi_allreduce_pair's roles), the rest are
// forward blocks (fwd_body<MRG>), which stage their images while the all-reduce runs
// and wait for each bucket's blocks only where they first read its parameters.  The forward
// needs the conv bucket at its staging and the fc bucket only at its fc epilogue, so the
// fc bucket's 2 MB all-gather overlaps the staging, the conv1 recompute and the MFMA loop
// (profiles/r5_dist: the step's last kernel and the next step's first used to run back to
// back with a launch boundary between).  Deadlock freedom: the launcher requires the WHOLE
// grid to be resident at once (hipOccupancy of this kernel x CUs >= grid), so no block waits
// for an undispatched one; the all-reduce blocks wait only for their peers' same blocks.
// bf16, pxt 1 (256-thread blocks), level 3, three blocks per CU (next to the role blocks)
template <typename T>
__global__ __launch_bounds__(256, 3) void step_head_kernel(
    const T* __restrict__ Wt, const float* __restrict__ bias, T* __restrict__ Y, int B, const T* __restrict__ wfc,
    float* __restrict__ fc_part, C1Src c1, FwdDz dzo, FwdMerge mg) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nx = mg.nblk0 + mg.nblk1;
  if ((int)blockIdx.x < nx) {
    merge_allreduce_role(mg, smem);
    return;
  }
  fwd_body<T, 1, 4, true, 10, true, 28, 28, 32, 64, true, 2, true>(
      (int)blockIdx.x - nx, 0, static_cast<const T*>(nullptr), Wt, bias, Y, B, 28, 28, 32, 64, wfc, fc_part, c1,
      dzo, mg);
}

static int step_head_occupancy(size_t lds) {
  auto k = step_head_kernel<bf16_t>;
  lds_optin(k, lds);
  int dev = 0, cus = 0, occ = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, 256, lds) != hipSuccess) return 0;
  return occ * cus;
}

int conv3x3_step_head_slots() {
  return step_head_occupancy(std::max(conv3x3_fwd_lds(28, 32, 1, true, 2), (size_t)64 + sizeof(XgmiArgs)));
}

bool conv3x3_step_head_fits(int nx, int B) {
  if (B <= 0 || nx <= 0) return false;
  const long nf = ((long)B * 28 * 28 + 63) / 64;
  const bool ok = (long)conv3x3_step_head_slots() >= nx + nf;
  if (!ok && std::getenv("DDP_AMD_XAR_DEBUG"))
    fprintf(stderr, "[ddp_amd] step head does not fit: %d resident slots < %ld blocks\n", conv3x3_step_head_slots(),
            nx + nf);
  return ok;
}

bool conv3x3_step_head(const BwdXar& x, int* done_fc, int* done_conv, const bf16_t* Wt, const float* bias,
                       bf16_t* Y, int B, const bf16_t* wfc, float* fc_part, const C1Src& c1, const FwdDz& dz,
                       int* err, hipStream_t s, const ShadowSet* late) {
  const int nx = x.nblk0 + x.nblk1;
  const char* bad = !x.args ? "all-reduce arguments" : x.nblk0 < 0 || x.nblk1 <= 0 ? "the conv bucket's blocks"
                   : !done_fc || !done_conv ? "bucket-done counters" : !dz.dz2 || !dz.img_cnt || !dz.fc_bias
                   ? "the level-3 forward's dZ2 outputs" : !wfc ? "the fc weight shadow" : !c1.x ? "the images" : nullptr;
  if (bad) throw std::runtime_error(std::string("conv3x3_step_head: missing ") + bad);
  if (!conv3x3_step_head_fits(nx, B)) return false;
  const long nf = ((long)B * 28 * 28 + 63) / 64;
  const size_t lds = std::max(conv3x3_fwd_lds(28, 32, 1, true, 2), (size_t)64 + sizeof(XgmiArgs));
  FwdMerge mg;
  mg.args = x.args;
  mg.nblk0 = x.nblk0;
  mg.nblk1 = x.nblk1;
  mg.fc_done = done_fc;
  mg.conv_done = done_conv;
  mg.err = err;
  if (late) mg.late = *late;
  auto k = step_head_kernel<bf16_t>;
  lds_optin(k, lds);
  hipLaunchKernelGGL(k, dim3((unsigned)(nx + nf)), dim3(256), lds, s, Wt, bias, Y, B, wfc, fc_part, c1, dz, mg);
  return true;
}

template <typename T>
static void fwd_launch(const T* X, const T* Wt, const float* bias, T* Y, int B, int H, int W, int Cin,
                       int Cout, bool relu, const T* wfc, float* fc_part, int pxt, hipStream_t s,
                       const C1Src* c1, const FwdDz* dz) {
  const long P = (long)B * H * W;
  const int per_blk = 64 * pxt;
  const dim3 grid((unsigned)((P + per_blk - 1) / per_blk), Cout / 64);
  const bool a1x = c1 != nullptr;
  const size_t lds = conv3x3_fwd_lds(W, Cin, pxt, a1x, (int)sizeof(T));
  const bool fc = wfc != nullptr;  // host guarantees NO == 10 when fused
  const C1Src cs = a1x ? *c1 : C1Src();
  const bool g = simplecnn_geom(H, W, Cin, Cout);
  const FwdDz dzo = dz ? *dz : FwdDz();
  if (dz) {
    if (!g || !fc || !a1x || !(pxt == 1 || pxt == 2) || !(sizeof(T) == 2 ? (void*)dz->dz2 : (void*)dz->dz2_f32) ||
        !dz->img_cnt || !dz->fc_bias)
      throw std::runtime_error("conv3x3_fwd: the level-3 dZ2 epilogue is the SimpleCNN forward with the fc "
                               "epilogue and the conv1 recompute");
    if constexpr (sizeof(T) == 2) {
      if (pxt == 2 && fwd_dz_occ2(grid.x)) {
        auto k = fwd_dz_kernel<T, 2, 2>();
        lds_optin(k, lds);
        hipLaunchKernelGGL(k, grid, dim3(512), lds, s, X, Wt, bias, Y, B, H, W, Cin, Cout, wfc, fc_part, cs, dzo);
        return;
      }
    }
    auto k = pxt == 2 ? fwd_dz_kernel<T, 2>() : fwd_dz_kernel<T, 1>();
    lds_optin(k, lds);
    hipLaunchKernelGGL(k, grid, dim3(256 * pxt), lds, s, X, Wt, bias, Y, B, H, W, Cin, Cout, wfc, fc_part, cs, dzo);
    return;
  }
  // one 16-pixel tile per wave: pxt 2 -> 8 waves (2 per SIMD), pxt 1 -> 4 waves
#define LF(PX, RL, NF, AX)                                                                          \
  do {                                                                                              \
    if (g) {                                                                                        \
      auto k = conv3x3_fwd_kernel<T, 1, 4 * PX, RL, NF, AX, 28, 28, 32, 64>;                        \
      lds_optin(k, lds);                                                                            \
      hipLaunchKernelGGL(k, grid, dim3(256 * PX), lds, s, X, Wt, bias, Y, B, H, W, Cin, Cout, wfc,  \
                         fc_part, cs, dzo);                                                         \
    } else {                                                                                        \
      auto k = conv3x3_fwd_kernel<T, 1, 4 * PX, RL, NF, AX, 0, 0, 0, 0>;                            \
      lds_optin(k, lds);                                                                            \
      hipLaunchKernelGGL(k, grid, dim3(256 * PX), lds, s, X, Wt, bias, Y, B, H, W, Cin, Cout, wfc,  \
                         fc_part, cs, dzo);                                                         \
    }                                                                                               \
  } while (0)
  if (pxt == 2) {
    if (fc && a1x) LF(2, true, 10, true);
    else if (fc) LF(2, true, 10, false); else if (relu) LF(2, true, 0, false); else LF(2, false, 0, false);
  } else {
    if (fc && a1x) LF(1, true, 10, true);
    else if (fc) LF(1, true, 10, false); else if (relu) LF(1, true, 0, false); else LF(1, false, 0, false);
  }
#undef LF
}

void conv3x3_fwd(const bf16_t* X, const bf16_t* Wt, const float* bias, bf16_t* Y, int B, int H,
                 int W, int Cin, int Cout, bool relu, const bf16_t* wfc, float* fc_part, int NO,
                 int pxt, hipStream_t s, const C1Src* c1, const FwdDz* dz) {
  if (dz && NO != 10) throw std::runtime_error("conv3x3_fwd: the level-3 dZ2 epilogue is built for 10 classes");
  fwd_launch<bf16_t>(X, Wt, bias, Y, B, H, W, Cin, Cout, relu, wfc, fc_part, pxt, s, c1, dz);
}
void conv3x3_fwd(const float* X, const float* Wt, const float* bias, float* Y, int B, int H,
                 int W, int Cin, int Cout, bool relu, const float* wfc, float* fc_part, int NO,
                 int pxt, hipStream_t s, const C1Src* c1, const FwdDz* dz) {
  if (dz && NO != 10) throw std::runtime_error("conv3x3_fwd: the level-3 dZ2 epilogue is built for 10 classes");
  fwd_launch<float>(X, Wt, bias, Y, B, H, W, Cin, Cout, relu, wfc, fc_part, pxt, s, c1, dz);
}

template <typename T>
static void dgrad_launch(const T* dY, const T* Yact, const T* WT, const T* Xact, T* dX, int B, int H,
                         int W, int Cin, int Cout, const void* x0, bool x0_u8, BatchIdx bi,
                         float* w1slab, int pxt, hipStream_t s, const C1Src* c1) {
  const long P = (long)B * H * W;
  const int per_blk = 64 * pxt;
  const dim3 grid((unsigned)((P + per_blk - 1) / per_blk), Cin / 32);
  const bool mdy = Yact != nullptr, mx = Xact != nullptr || c1 != nullptr, w1 = w1slab != nullptr;
  const size_t lds = conv3x3_dgrad_lds(W, Cout, pxt, w1, (int)sizeof(T));
  const C1Src cs = c1 ? *c1 : C1Src();
  const bool g = simplecnn_geom(H, W, Cin, Cout);
#define LD(PX, A, Bm, C, AX)                                                                        \
  do {                                                                                              \
    if (g) {                                                                                        \
      auto k = conv3x3_dgrad_kernel<T, PX, A, Bm, C, AX, 28, 28, 32, 64>;                           \
      lds_optin(k, lds);                                                                            \
      hipLaunchKernelGGL(k, grid, dim3(256), lds, s, dY, Yact, WT, Xact, dX, B, H, W, Cin, Cout, x0,  \
                         (int)x0_u8, bi, w1slab, cs);                                               \
    } else {                                                                                        \
      auto k = conv3x3_dgrad_kernel<T, PX, A, Bm, C, AX, 0, 0, 0, 0>;                               \
      lds_optin(k, lds);                                                                            \
      hipLaunchKernelGGL(k, grid, dim3(256), lds, s, dY, Yact, WT, Xact, dX, B, H, W, Cin, Cout, x0,  \
                         (int)x0_u8, bi, w1slab, cs);                                               \
    }                                                                                               \
  } while (0)
  if (pxt == 2) {
    if (w1 && c1) LD(2, false, true, true, true);
    else if (w1) LD(2, false, true, true, false);
    else if (mdy && mx) LD(2, true, true, false, false);
    else if (mdy) LD(2, true, false, false, false);
    else if (mx) LD(2, false, true, false, false);
    else LD(2, false, false, false, false);
  } else {
    if (w1 && c1) LD(1, false, true, true, true);
    else if (w1) LD(1, false, true, true, false);
    else if (mdy && mx) LD(1, true, true, false, false);
    else if (mdy) LD(1, true, false, false, false);
    else if (mx) LD(1, false, true, false, false);
    else LD(1, false, false, false, false);
  }
#undef LD
}

void conv3x3_dgrad(const bf16_t* dY, const bf16_t* Yact, const bf16_t* WT, const bf16_t* Xact,
                   bf16_t* dX, int B, int H, int W, int Cin, int Cout, const void* x0, bool x0_u8,
                   BatchIdx bi, float* w1slab, int pxt, hipStream_t s, const C1Src* c1) {
  dgrad_launch<bf16_t>(dY, Yact, WT, Xact, dX, B, H, W, Cin, Cout, x0, x0_u8, bi, w1slab, pxt, s, c1);
}
void conv3x3_dgrad(const float* dY, const float* Yact, const float* WT, const float* Xact,
                   float* dX, int B, int H, int W, int Cin, int Cout, const void* x0, bool x0_u8,
                   BatchIdx bi, float* w1slab, int pxt, hipStream_t s, const C1Src* c1) {
  dgrad_launch<float>(dY, Yact, WT, Xact, dX, B, H, W, Cin, Cout, x0, x0_u8, bi, w1slab, pxt, s, c1);
}

int conv3x3_dgrad_blocks(int B, int H, int W, int pxt) {
  const long P = (long)B * H * W;
  const int per_blk = 64 * pxt;
  return (int)((P + per_blk - 1) / per_blk);
}

int conv3x3_wgrad_blocks(int B, int H, int R) { return B * ((H + R - 1) / R); }

size_t conv3x3_wgrad_lds(int W, int Cin, int Cout, int R, bool a1x, int es) {
  const int Wp = (W + 7) & ~7;
  const int nslot = ((R * Wp + 31) / 32) * 32;
  return (size_t)es * ((size_t)nslot * (Cout + 16) + (size_t)(R + 2) * (Wp + 2) * (Cin + 16)) +
         (a1x ? sizeof(float) * ((size_t)(R + 4) * (Wp + 4) + Cin * 10) : 0);
}

template <typename T>
static void wgrad_launch(const T* dY, const T* Yact, const T* X, float* slab, int B, int H, int W,
                         int Cin, int Cout, int R, hipStream_t s, const C1Src* c1) {
  const dim3 grid(conv3x3_wgrad_blocks(B, H, R), (Cout / 32) * (Cin / 16) / 4);
  const size_t lds = conv3x3_wgrad_lds(W, Cin, Cout, R, c1 != nullptr, (int)sizeof(T));
  const C1Src cs = c1 ? *c1 : C1Src();
  const bool g = simplecnn_geom(H, W, Cin, Cout);
#define LW(M, AX)                                                                                   \
  do {                                                                                              \
    if (g) {                                                                                        \
      auto k = conv3x3_wgrad_kernel<T, M, AX, 28, 28, 32, 64>;                                      \
      lds_optin(k, lds);                                                                            \
      hipLaunchKernelGGL(k, grid, dim3(256), lds, s, dY, Yact, X, slab, B, H, W, Cin, Cout, R, cs);  \
    } else {                                                                                        \
      auto k = conv3x3_wgrad_kernel<T, M, AX, 0, 0, 0, 0>;                                          \
      lds_optin(k, lds);                                                                            \
      hipLaunchKernelGGL(k, grid, dim3(256), lds, s, dY, Yact, X, slab, B, H, W, Cin, Cout, R, cs);  \
    }                                                                                               \
  } while (0)
  if (c1) { if (Yact) LW(true, true); else LW(false, true); }
  else { if (Yact) LW(true, false); else LW(false, false); }
#undef LW
}

void conv3x3_wgrad(const bf16_t* dY, const bf16_t* Yact, const bf16_t* X, float* slab, int B,
                   int H, int W, int Cin, int Cout, int R, hipStream_t s, const C1Src* c1) {
  wgrad_launch<bf16_t>(dY, Yact, X, slab, B, H, W, Cin, Cout, R, s, c1);
}
void conv3x3_wgrad(const float* dY, const float* Yact, const float* X, float* slab, int B,
                   int H, int W, int Cin, int Cout, int R, hipStream_t s, const C1Src* c1) {
  wgrad_launch<float>(dY, Yact, X, slab, B, H, W, Cin, Cout, R, s, c1);
}

DDP_STAMPS_SETTER(stamps_set_conv3x3)

}  // namespace ddp_amd
