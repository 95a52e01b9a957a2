// Launchers of the fused SimpleCNN conv backward (conv3x3_bwd_kernel, conv3x3_body.h): dgrad,
// wgrad, fc and in-launch all-reduce roles, the fused slab reduction; the residency sizing of
// the reducers and of the in-launch all-reduce.  (Own TU: its instantiations compile in
// parallel with conv3x3.hip's.)
#include <algorithm>
#include <stdexcept>

#include <cstdio>
#include <cstdlib>

#include "kernels/conv3x3_body.h"

namespace ddp_amd {

size_t conv3x3_bwd_lds(int W, int Cin, int Cout, int pxt, int R, int es, int cs) {
  if (es == 4 && cs == 2) {
    // exact fp32, both roles channel-split: dgrad (weights from global) = the dY tile + the
    // conv1 weight-gradient scratch; wgrad = dY slots + the half's compact X tile (+ the
    // conv1 recompute input); slab rows stored directly (no staging)
    const size_t XR = 64 * pxt + 2 * W + 2;
    const size_t a = 4 * (XR * (Cout + 8)) + sizeof(float) * (XR + 4 * 320) + 4 * 64 * pxt;
    const int Wp = (W + 7) & ~7;
    const size_t nslot = ((R * Wp + 31) / 32) * 32;
    const size_t b = 4 * (nslot * (Cout + 16) + (size_t)(R + 2) * (Wp + 2) * 16) +
                     sizeof(float) * ((size_t)(R + 4) * (Wp + 4) + Cin * 10);
    const size_t red = sizeof(float) * 3 * 16 * 64;  // the fused reducer's partials
    const size_t m = a > b ? a : b;
    return ((m > red ? m : red) + 15) & ~(size_t)15;
  }
  const size_t a = conv3x3_dgrad_lds(W, Cout, pxt, true, es), b = conv3x3_wgrad_lds(W, Cin, Cout, R, true, es);
  // the wgrad role's staged slab row (+ its bank skew, 4 floats per output channel)
  const size_t row = sizeof(float) * ((size_t)Cout * 9 * Cin + Cout + 4 * (size_t)Cout);
  const size_t m = a > b ? a : b;
  return m > row ? m : row;
}

// Resident-block budget of the fused reduction.  The reducers are the LAST conv blocks of
// the grid and wait only for blocks with lower indices, so with in-order dispatch every
// block a waiting reducer needs already holds a slot (or finished): no capacity makes it
// deadlock.  The budget - at most HALF of the launch's resident capacity as the occupancy
// API reports it for the exact instantiation - keeps room for what may share the GPU (a
// concurrent all-reduce kernel; ranks sharing a device never fuse, fused_step.py).  (A
// quarter was the rule while the wgrad blocks were dispatched FIRST: 128 waiting fp32
// reducers starved the rest of that grid.)  Returns the number of reducers (all the wgrad
// blocks), 0 when they do not fit (fewer reducers, two passes each, measured slower than
// the separate grad_reduce kernel: fp32 364k vs 383k img/s) or the capacity is unknown.
// exclusive (single process, no bucket all-reduce kernel on another stream): the budget is
// the whole resident capacity - all reducers can then be resident at once, and every other
// block of the grid runs to completion without waiting, so the argument above holds with
// nothing else on the GPU.  This lets the exact-fp32 step (one block per CU, 224 wgrad
// blocks at batch 32) fuse its reduction.
template <typename K>
static int fused_reducers(K kernel, size_t lds, int nblocks, bool exclusive) {
  int dev = 0, cus = 0, occ = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(kernel), 256, lds) != hipSuccess)
    return 0;
  const int budget = exclusive ? occ * cus : occ * cus / 2;
  return nblocks <= budget ? nblocks : 0;
}

template <typename T>
using BwdKFn = void (*)(const T*, const T*, T*, float*, float*, int, int, int, int, int, int, int, C1Src, const T*,
                        BwdReduce, BwdFc, BwdXar);

// The conv backward instantiation a launch runs (chosen BEFORE the fused reduction's residency
// query, so that query sees the exact kernel - its registers decide its residency).
// cs == 2 and FCR: the bf16 SimpleCNN variants only (FCR: pxt 2, channel split).
// xar: the in-launch all-reduce variant (FCR + FRED only: bf16 pxt 2 channel split, or the
// exact-fp32 double split) - callers check xar_ok first
template <typename T, int PX, bool DA, bool WA>
static BwdKFn<T> pick_bwd3(bool g, bool fred, int cs, bool fcr, int dg, bool xar = false) {
  if (!g) return conv3x3_bwd_kernel<T, PX, DA, WA, 0, 0, 0, 0, false>;
  if constexpr (sizeof(T) == 2) {
    if (cs == 2) {
      if constexpr (PX == 2) {
        if (xar && fcr && fred) return conv3x3_bwd_kernel<T, PX, DA, WA, 28, 28, 32, 64, true, 2, true, 1, true>;
        if (fcr)
          return fred ? conv3x3_bwd_kernel<T, PX, DA, WA, 28, 28, 32, 64, true, 2, true>
                      : conv3x3_bwd_kernel<T, PX, DA, WA, 28, 28, 32, 64, false, 2, true>;
      }
      return fred ? conv3x3_bwd_kernel<T, PX, DA, WA, 28, 28, 32, 64, true, 2>
                  : conv3x3_bwd_kernel<T, PX, DA, WA, 28, 28, 32, 64, false, 2>;
    }
  } else {
    // exact fp32, two blocks per CU (wgrad channel-split, dgrad weights from global, dgrad
    // channel-split too when dg == 2): pxt 2, conv1 recomputed
    if constexpr (PX == 2 && DA && WA) {
      if (cs == 2) {
        if (dg == 2) {
          if (xar && fcr && fred) return conv3x3_bwd_kernel<T, PX, DA, WA, 28, 28, 32, 64, true, 2, true, 2, true>;
          if (fcr)
            return fred ? conv3x3_bwd_kernel<T, PX, DA, WA, 28, 28, 32, 64, true, 2, true, 2>
                        : conv3x3_bwd_kernel<T, PX, DA, WA, 28, 28, 32, 64, false, 2, true, 2>;
          return fred ? conv3x3_bwd_kernel<T, PX, DA, WA, 28, 28, 32, 64, true, 2, false, 2>
                      : conv3x3_bwd_kernel<T, PX, DA, WA, 28, 28, 32, 64, false, 2, false, 2>;
        }
        if (fcr)
          return fred ? conv3x3_bwd_kernel<T, PX, DA, WA, 28, 28, 32, 64, true, 2, true>
                      : conv3x3_bwd_kernel<T, PX, DA, WA, 28, 28, 32, 64, false, 2, true>;
        return fred ? conv3x3_bwd_kernel<T, PX, DA, WA, 28, 28, 32, 64, true, 2>
                    : conv3x3_bwd_kernel<T, PX, DA, WA, 28, 28, 32, 64, false, 2>;
      }
    }
  }
  return fred ? conv3x3_bwd_kernel<T, PX, DA, WA, 28, 28, 32, 64, true>
              : conv3x3_bwd_kernel<T, PX, DA, WA, 28, 28, 32, 64, false>;
}
template <typename T>
static BwdKFn<T> pick_bwd(int pxt, bool da, bool wa, bool g, bool fred, int cs, bool fcr, int dg, bool xar = false) {
  if (pxt == 2) {
    if (da) return pick_bwd3<T, 2, true, true>(g, fred, cs, fcr, dg, xar);
    return wa ? pick_bwd3<T, 2, false, true>(g, fred, cs, fcr, dg, xar)
              : pick_bwd3<T, 2, false, false>(g, fred, cs, fcr, dg, xar);
  }
  if (da) return pick_bwd3<T, 1, true, true>(g, fred, cs, fcr, dg, xar);
  return wa ? pick_bwd3<T, 1, false, true>(g, fred, cs, fcr, dg, xar) : pick_bwd3<T, 1, false, false>(g, fred, cs, fcr, dg, xar);
}

bool conv3x3_bwd_fc_role_ok(int H, int W, int Cin, int Cout, int pxt, int wgrad_split) {
  return simplecnn_geom(H, W, Cin, Cout) && pxt == 2 && wgrad_split == 2;
}

template <typename T>
static bool bwd_launch(const T* dY, const T* WT, T* dX, float* w1slab, float* slab, int B, int H, int W,
                       int Cin, int Cout, int pxt, int R, const C1Src& c1, const T* Xact,
                       bool wgrad_load_a1, hipStream_t s, const SlabSet* fused, int* red_done, int* red_err,
                       int csplit, const BwdFc* fc, bool exclusive, const BwdXar* xar, bool* xar_used) {
  if (xar_used) *xar_used = false;
  const bool g = simplecnn_geom(H, W, Cin, Cout);
  // the channel split (SimpleCNN geometry): bf16 - two wgrad blocks per slab row; exact fp32
  // (pxt 2, conv1 recomputed) - two wgrad blocks per row AND two dgrad blocks per pixel
  // chunk, at two blocks per CU; otherwise one block each
  constexpr bool F32 = sizeof(T) == 4;
  const int cs = (csplit == 2 && g && (!F32 || (pxt == 2 && !Xact))) ? 2 : 1;
  // exact fp32: dgrad channel split (DDP_AMD_F32_DSPLIT=1 keeps one dgrad block per chunk)
  int dcs = 1;
  if (F32 && cs == 2) {
    const char* e = std::getenv("DDP_AMD_F32_DSPLIT");
    dcs = (e && e[0] == '1') ? 1 : 2;
  }
  const int nrows = conv3x3_wgrad_blocks(B, H, R);
  const int nd = conv3x3_dgrad_blocks(B, H, W, pxt) * dcs, nw = nrows * cs;
  size_t lds = conv3x3_bwd_lds(W, Cin, Cout, pxt, R, (int)sizeof(T), cs);
  if (((long)Cout * 9 * Cin + Cout) % 4 != 0 || (reinterpret_cast<uintptr_t>(slab) & 15) != 0)
    throw std::runtime_error("conv3x3_bwd: slab rows must be 16-byte multiples on a 16-byte aligned buffer");
  BwdFc fcr;
  int nfc = 0;
  const bool da = !Xact, wa = !Xact || !wgrad_load_a1;
  if (fc) {
    if (!conv3x3_bwd_fc_role_ok(H, W, Cin, Cout, pxt, cs) || !fc->dl || !fc->a2 || fc->K % 2 != 0 || B > BFC_MAXB ||
        fc->ex.last_ctr)
      throw std::runtime_error("conv3x3_bwd: the fc role is the SimpleCNN variant (pxt 2, channel split, dL "
                               "given, B <= 64, no last-block count)");
    fcr = *fc;
    fcr.nconv = nd + nw;
    // one 128-column chunk per wave (4 per block), blocks after every conv block: the first
    // take the resident slots the conv blocks leave free, the rest those the dgrad blocks
    // free first
    // (two chunks per wave - 49 blocks, all resident from the start at B = 32 - measured
    // slower: each fc wave's time doubles, 944k -> 935k in-call, B = 64 1.13M -> 1.05M;
    // profiles/r4_fc_cpw)
    nfc = (int)((fc->K + 127) / 128 + 3) / 4;
    fcr.nfc = nfc;
    // fc blocks after every conv block (default) or before them (A/B knob DDP_AMD_FC_FIRST=1:
    // B = 32 838k vs 954k img/s in-call, B = 64 within the spread - profiles/r4_b64); with
    // the in-launch all-reduce always first: the fc bucket's all-reduce waits for them
    const char* ff = std::getenv("DDP_AMD_FC_FIRST");
    const bool first = (ff && ff[0] == '1') || xar != nullptr;
    fcr.fc0 = first ? 0 : nd + nw;
    if ((size_t)B * (FCDW_LD + 10) * sizeof(float) > lds)
      throw std::runtime_error("conv3x3_bwd: LDS too small for the fc role");
  }
  BwdReduce red;
  red.nconv = nd + nw;
  {  // role order: interleaved for bf16 (+1.7-2.3 % in-call, profiles/r4_interleave), the
     // fp32 split keeps dgrad-then-wgrad (neutral there); A/B knob DDP_AMD_BWD_INTERLEAVE=0|1
    const char* e = std::getenv("DDP_AMD_BWD_INTERLEAVE");
    red.interleave = e && e[0] ? (e[0] == '1') : !F32;
  }
  if (fused) {
    // the reducer's 16-byte row loads need n >= 4; its summation order is grad_reduce's
    // 16-row-group one (deep slabs; shallow ones keep the separate kernel)
    if (grad_reduce_groups(*fused) != 16) fused = nullptr;
    for (int k = 0; fused && k < fused->count; ++k)
      if (fused->s[k].n < 4) fused = nullptr;
  }
  if (fused) {
    // reducers: the wgrad blocks (they finish last; extra early-finishing reducers measured
    // slower - their polling shares the CUs of the still-running wgrad blocks)
    // (channel split: the last nrows blocks - as many reducers as without the split).
    // Residency of the exact instantiation that will run.
    const BwdKFn<T> kf = pick_bwd<T>(pxt, da, wa, g, true, cs, fc != nullptr, dcs, xar != nullptr);
    lds_optin(kf, lds);
    const int nr = (g && red_done) ? fused_reducers(kf, lds, nrows, exclusive) : 0;
    if (nr <= 0) fused = nullptr;  // the caller reduces with grad_reduce
    else red.first_reducer = nd + nw - nr;
  }
  if (fused) {
    red.ss = *fused;
    red.nchunks = slab_chunks(*fused);
    {  // the largest segment's row count picks the reducer's load depth
      int kmax = 0;
      for (int k = 1; k < fused->count; ++k)
        if (fused->s[k].n > fused->s[kmax].n) kmax = k;
      const int rows = fused->s[kmax].rows;
      const char* e = std::getenv("DDP_AMD_RED_DEEP");  // A/B knob: 0 forces the 8-row reducer
      red.deep = (rows > 128 && rows <= 256 && !(e && e[0] == '0')) ? 1 : 0;
    }
    red.done = red_done;
    red.err = red_err;
    if (lds < sizeof(float) * 3 * 16 * 64) throw std::runtime_error("conv3x3_bwd: LDS too small for the reducer");
  }
  // the in-launch bucket all-reduce (BwdXar): needs the fc role and the fused reduction in
  // this launch (its waits count their blocks); otherwise the caller runs the bucket kernels
  BwdXar xv;
  int nx = 0;
  bool use_xar = xar && fc && fused && pick_bwd<T>(pxt, da, wa, g, true, cs, true, dcs, true) !=
                                          pick_bwd<T>(pxt, da, wa, g, true, cs, true, dcs, false);
  if (use_xar) {
    // residency of the exact instantiation that would run: the role blocks spin
    // at the head of the grid, so either everything fits at once or in-order dispatch is
    // opted into; otherwise the caller runs the bucket kernels
    const BwdKFn<T> kx = pick_bwd<T>(pxt, da, wa, g, true, cs, true, dcs, true);
    lds_optin(kx, lds);
    int dev = 0, cus = 0, occ = 0;
    const long total = (long)xar->nblk0 + xar->nblk1 + nd + nw + nfc;
    const bool fits = hipGetDevice(&dev) == hipSuccess &&
                      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
                      hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kx, 256, lds) == hipSuccess &&
                      (long)occ * cus >= total;
    if (!fits && !inorder_optin()) use_xar = false;
  }
  if (xar && !use_xar && std::getenv("DDP_AMD_XAR_DEBUG"))
    fprintf(stderr, "[ddp_amd] in-launch all-reduce not used: fc %d fused %d first_reducer %d nconv %d\n",
            fc != nullptr, fused != nullptr, red.first_reducer, nd + nw);
  if (use_xar) {
    xv = *xar;
    xv.fc_expect = nfc;
    xv.red_expect = nd + nw - red.first_reducer;  // the reducers
    nx = xv.nblk0 + xv.nblk1;
    if (xv.nblk1 <= 0 || !xv.args || !xv.fc_done || !xv.red_done || !xv.xar_done)
      throw std::runtime_error("conv3x3_bwd: in-launch all-reduce needs a conv bucket and its counters");
    if (lds < 64 + sizeof(XgmiArgs)) throw std::runtime_error("conv3x3_bwd: LDS too small for the all-reduce role");
    if (xar_used) *xar_used = true;
  }
  // the wgrad role needs a single (Cout/32)*(Cin/16)/4 == 1 y-block and the dgrad role Cin == 32
  const BwdKFn<T> k = pick_bwd<T>(pxt, da, wa, g, fused != nullptr, cs, fc != nullptr, dcs, use_xar);
  lds_optin(k, lds);
  hipLaunchKernelGGL(k, dim3(nx + nd + nw + nfc), dim3(256), lds, s, dY, WT, dX, w1slab, slab, B, H, W, Cin, Cout,
                     R, nd, c1, Xact, red, fcr, xv);
  return fused != nullptr;
}

bool conv3x3_bwd(const bf16_t* dY, const bf16_t* WT, bf16_t* dX, float* w1slab, float* slab, int B,
                 int H, int W, int Cin, int Cout, int pxt, int R, const C1Src& c1, const bf16_t* Xact,
                 bool wgrad_load_a1, hipStream_t s, const SlabSet* fused_reduce, int* red_done, int* red_err,
                 int wgrad_split, const BwdFc* fc, bool exclusive, const BwdXar* xar, bool* xar_used) {
  return bwd_launch<bf16_t>(dY, WT, dX, w1slab, slab, B, H, W, Cin, Cout, pxt, R, c1, Xact, wgrad_load_a1, s,
                     fused_reduce, red_done, red_err, wgrad_split, fc, exclusive, xar, xar_used);
}
bool conv3x3_bwd(const float* dY, const float* WT, float* dX, float* w1slab, float* slab, int B,
                 int H, int W, int Cin, int Cout, int pxt, int R, const C1Src& c1, const float* Xact,
                 bool wgrad_load_a1, hipStream_t s, const SlabSet* fused_reduce, int* red_done, int* red_err,
                 int wgrad_split, const BwdFc* fc, bool exclusive, const BwdXar* xar, bool* xar_used) {
  return bwd_launch<float>(dY, WT, dX, w1slab, slab, B, H, W, Cin, Cout, pxt, R, c1, Xact, wgrad_load_a1, s,
                    fused_reduce, red_done, red_err, wgrad_split, fc, exclusive, xar, xar_used);
}

DDP_STAMPS_SETTER(stamps_set_conv3x3_bwd)

}  // namespace ddp_amd
