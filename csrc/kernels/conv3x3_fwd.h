// The forward conv kernel template of the conv3x3 TU (conv3x3.hip only: the backward TU,
// conv3x3_bwd.hip, does not include it, so a forward-only change rebuilds ~2 min of device
// code instead of ~12): SimpleCNN's conv2 forward with the fused fc partials / level-3 dZ2
// epilogue, and its MRG instantiation, the dist_mode 4 step head.
#pragma once

#include "kernels/conv3x3_body.h"

namespace ddp_amd {

// ---------------------------------------------------------------- forward
// A1X: the input X is NOT read from memory but recomputed in the staging pass as
// relu(conv1(x)) from the uint8 dataset (x0 via the batch index list) - SimpleCNN's
// first layer folded into the second (Cin must equal conv1's 32 output channels).
// NW waves per block, PXT 16-pixel tiles per wave: a block covers CH = 16 * NW * PXT
// pixels (64 * pxt in launcher terms).  With NW = 8 two waves share each SIMD, which
// doubles the VALU issue rate of the conv1 recompute and the fc epilogue.
// DZ (fuse level 3, launchers.h FwdDz): after the fc partials, wait for every block of the
// block's image(s), evaluate dL and write dZ2 for the block's own pixels (see FwdDz).
constexpr unsigned long long FWD_DZ_WAIT_TICKS = 2000000;  // 20 ms of the 100 MHz clock
#ifndef DDP_AMD_F32_FC_PREFETCH
#define DDP_AMD_F32_FC_PREFETCH 0  // 1: measured neutral (block 22.6 vs 22.7 us, profiles/r4_fp32)
#endif
constexpr bool F32_FC_PREFETCH = DDP_AMD_F32_FC_PREFETCH;
#ifndef DDP_AMD_FWD_PF_SPLIT
#define DDP_AMD_FWD_PF_SPLIT 1
#endif  // see conv3x3_fwd_kernel (DZ, fp32)

// MRG (dist_mode 4, the step head): the forward runs in the SAME launch as the previous
// step's bucket all-reduces, whose fused SGD writes this step's parameters.  Its blocks stage
// the step's images first, wait for the conv bucket's all-reduce blocks (FwdMerge conv_done)
// before they read conv1's weights, conv2's bf16 weight shadow and bias, and for the fc
// bucket's (fc_done) before the fc epilogue reads the fc weight shadow and bias; every one of
// those reads is an sc1 (agent-coherent) load, the writers store write-through (xgmi_body.h
// WT) and drain before they count - the hand-off pattern of the fused slab reduction.  No fc
// weight prefetch (the weights are not final before the wait).
// The merged launch's grid: blocks [0, nblk1) all-reduce the conv (stage-1) bucket, the next
// nblk0 the fc (stage-0) bucket - exactly xgmi_allreduce_pair's roles, conv first because every
// forward block waits for it before its staging - then the forward blocks.  nblk0 = 0: one
// bucket holds every parameter (its count gates both waits).
struct FwdMerge {
  const XgmiArgs* args = nullptr;  // [0] fc / [1] conv bucket's arguments (device memory)
  int nblk0 = 0, nblk1 = 0;
  int* fc_done = nullptr;          // per-bucket block counts, zeroed by the previous fc role
  int* conv_done = nullptr;
  int* err = nullptr;
  ShadowSet late{};                // conv bucket shadows written after the count (see below)
};
constexpr int MRG_ERR = 5;  // sync_err code of a timed-out merged-forward wait

__device__ __forceinline__ bf16x8 ld16_sc1(__amdgpu_buffer_rsrc_t r, int byte_off) {
  typedef __attribute__((ext_vector_type(4))) int i32x4_t;
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16 /* sc1 */));
}
__device__ __forceinline__ Conv1Group conv1_group_load_sc1(const float* w1, const float* b1, int g) {
  Conv1Group r;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
#pragma unroll
    for (int k = 0; k < 9; ++k)
      r.w[j][k] = __hip_atomic_load(w1 + (8 * g + j) * 9 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    r.b[j] = __hip_atomic_load(b1 + 8 * g + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return r;
}
// the merged forward's waits: hundreds of blocks poll one counter while the all-reduce they
// wait for moves megabytes - poll ~10x less often than the conv backward's waits
constexpr int MRG_SLEEP = 16;

// one merged-launch all-reduce block (MRG kernels' blocks [0, nblk0 + nblk1))
__device__ __forceinline__ void merge_allreduce_role(FwdMerge mg, char* smem) {
  const int k = (int)blockIdx.x < mg.nblk1 ? 1 : 0;
  const int rb = k == 1 ? (int)blockIdx.x : (int)blockIdx.x - mg.nblk1;  // block within its channel
  __builtin_amdgcn_s_setprio(2);  // over the forward blocks beside it
  unsigned* s_sh = reinterpret_cast<unsigned*>(smem);
  XgmiArgs* s_xa = reinterpret_cast<XgmiArgs*>(smem + 64);
  {  // the bucket's arguments into LDS (from global memory every field was re-loaded per store)
    const int* src = reinterpret_cast<const int*>(mg.args + k);
    int* dst = reinterpret_cast<int*>(s_xa);
    for (int i = threadIdx.x; i < (int)(sizeof(XgmiArgs) / 4); i += (int)blockDim.x) dst[i] = src[i];
  }
  __syncthreads();
  DDP_STAMP(STAMP_K_HEAD, 0);
  xgmi_allreduce_body<true>(*s_xa, rb, k == 0 ? mg.nblk0 : mg.nblk1, s_sh, STAMP_K_HEAD);
  DDP_STAMP(STAMP_K_HEAD, 7);
  count_done(k == 0 ? mg.fc_done : mg.conv_done);  // drain (write-through) + one relaxed count
  DDP_STAMP(STAMP_K_HEAD, 6);
  if (k == 1 && mg.late.count) {
    // the shadows no forward block reads (conv2's [tap][ci][co] copy, 4 scattered 2-byte
    // stores per quad): refreshed after the count, from the parameters this block just
    // stored (system-scope loads: no stale cached line) - out of the drain the forward
    // waited for (stamps: conv bucket counted 9.2 -> 6.3 us, profiles/r6_dist).  Plain
    // stores: the next launch (the conv backward) reads them.
    const XgmiArgs& a = *s_xa;
    const ShadowSet late = mg.late;
    const long n = a.n, G = (long)mg.nblk1 * XGMI_THREADS;
    const float* pb = a.params + a.off;
    const __amdgpu_buffer_rsrc_t rp = sys_rsrc(pb);
    for (long q = (long)rb * XGMI_THREADS + threadIdx.x; 4 * q < n; q += G) {
      if (4 * q + 3 < n) {
        shadow_quad<false>(late, a.off + 4 * q, ld4_sys(rp, q));
      } else {
        for (long e = 4 * q; e < n; ++e) shadow_one<false>(late, a.off + e, ld_sys(pb + e));
      }
    }
  }
}

// The forward conv (+ fc partials, + level-3 dZ2): the plain kernel ...
template <typename T, int PXT, int NW, bool RELU, int NOF, bool A1X, int GH, int GW, int GCI, int GCO,
          bool DZ = false, int OCC = 1>
__global__ __launch_bounds__(NW * 64, OCC * NW / 4) void conv3x3_fwd_kernel(  // 2nd: waves per SIMD
    const T* __restrict__ X, const T* __restrict__ Wt, const float* __restrict__ bias,
    T* __restrict__ Y, int B, int H, int W, int Cin, int Cout,
    const T* __restrict__ wfc, float* __restrict__ fc_part, C1Src c1, FwdDz dzo) {
  constexpr bool MRG = false;
  const FwdMerge mg{};
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int bx = (int)blockIdx.x, by = (int)blockIdx.y;
#include "kernels/conv3x3_fwd_body.inc.h"
}

// ... and MRG, the dist_mode 4 step head's forward blocks (FwdMerge; conv3x3.hip
// step_head_kernel): block (bx, by) of the forward grid as a device function
template <typename T, int PXT, int NW, bool RELU, int NOF, bool A1X, int GH, int GW, int GCI, int GCO, bool DZ,
          int OCC, bool MRG>
__device__ __forceinline__ void fwd_body(
    const int bx, const int by, const T* __restrict__ X, const T* __restrict__ Wt, const float* __restrict__ bias,
    T* __restrict__ Y, int B, int H, int W, int Cin, int Cout, const T* __restrict__ wfc,
    float* __restrict__ fc_part, const C1Src& c1, const FwdDz& dzo, const FwdMerge& mg) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
#include "kernels/conv3x3_fwd_body.inc.h"
}

// the level-3 forward of SimpleCNN's conv2 (fc epilogue, conv1 recompute, pxt 1 / 2)
template <typename T, int PX, int OCC = 1>
static auto fwd_dz_kernel() {
  return conv3x3_fwd_kernel<T, 1, 4 * PX, true, 10, true, 28, 28, 32, 64, true, OCC>;
}

// bf16 level-3 forward at two blocks per CU (OCC 2, no fc weight prefetch) when the grid
// exceeds one block per CU (B > 32 at pxt 2); DDP_AMD_FWD_OCC2=0/1 forces it off/on
static bool fwd_dz_occ2(unsigned grid) {
  static const int env = [] { const char* e = getenv("DDP_AMD_FWD_OCC2"); return e ? atoi(e) : -1; }();
  if (env >= 0) return env == 1;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return false;
  return cus > 0 && grid > (unsigned)cus;
}

template <typename T>
static bool fwd_dz_fits(int B, int H, int W, int pxt) {
  if (H != 28 || W != 28 || (pxt != 1 && pxt != 2) || B <= 0) return false;
  const long P = (long)B * H * W;
  const int per_blk = 64 * pxt;
  if (per_blk > H * W || P >= (1L << 31)) return false;
  const long grid = (P + per_blk - 1) / per_blk;
  const size_t lds = conv3x3_fwd_lds(W, 32, pxt, true, (int)sizeof(T));
  // the kernel fwd_launch will pick for this grid (bf16 pxt 2 beyond one block per CU: OCC 2)
  bool occ2 = false;
  const void* k = pxt == 2 ? reinterpret_cast<const void*>(fwd_dz_kernel<T, 2>())
                           : reinterpret_cast<const void*>(fwd_dz_kernel<T, 1>());
  if constexpr (sizeof(T) == 2) {  // (no fp32 OCC 2 instantiation)
    occ2 = pxt == 2 && fwd_dz_occ2((unsigned)grid);
    if (occ2) {
      k = reinterpret_cast<const void*>(fwd_dz_kernel<T, 2, 2>());
      lds_optin(fwd_dz_kernel<T, 2, 2>(), lds);
    }
  }
  if (!occ2) lds_optin(pxt == 2 ? fwd_dz_kernel<T, 2>() : fwd_dz_kernel<T, 1>(), lds);
  int dev = 0, cus = 0, occ = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return false;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, occ2 ? 512 : 256 * pxt, lds) != hipSuccess) return false;
  // Every block spins on the other blocks of its image (a window of <= 8 consecutive block
  // indices: a block covers 64 * pxt <= H*W pixels).  Default: the whole grid must fit the
  // GPU at once (bf16 B = 64 does, with the OCC 2 forward: 392 blocks on 512 slots), so no
  // dispatch-order assumption is needed; otherwise the level-1 chain runs.
  if ((long)occ * cus >= grid) return true;
  // Opt-in (DDP_AMD_L3_INORDER=1): a grid larger than the GPU, relying on workgroups being
  // dispatched in index order round-robin over the XCDs - then on the XCD with the lowest
  // dispatch frontier F the oldest resident block b satisfies b + 8 < F whenever that XCD
  // holds >= 3 resident blocks (they sit 8 indices apart): every block of b's image is
  // dispatched, b's image completes and frees a slot.  The hardware does not promise this
  // order and a concurrent stream's kernels can hold the slots; the failure mode is the
  // bounded wait (FWD_DZ_WAIT_TICKS) setting the step's error word - the engine's
  // synchronize() raises and the start-up chain check downgrades to level 1.
  return inorder_optin() && (long)occ * cus >= 64;
}
}  // namespace ddp_amd
