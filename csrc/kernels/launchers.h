// Host-side launch API of the gfx950 kernel library (no torch types here: the
// runtime and the pybind layer both call these with raw pointers + a stream).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels/types.h"

namespace ddp_amd {

// ---- diagnostic phase stamps (common.h DDP_STAMP); buf = u64[STAMP_K_COUNT][4096][8] or null
void stamps_set(void* buf);

// ---- conv1 (Cin = 1) ---------------------------------------------------------------
void conv1_fwd(const void* x, bool x_is_u8, BatchIdx bi, const float* w, const float* b, bf16_t* y,
               int B, int H, int W, int Cout, hipStream_t s);
void conv1_fwd(const void* x, bool x_is_u8, BatchIdx bi, const float* w, const float* b, float* y,
               int B, int H, int W, int Cout, hipStream_t s);
int conv1_wgrad_blocks(int B, int H, int W, int chunk);
void conv1_wgrad(const void* x, bool x_is_u8, BatchIdx bi, const bf16_t* dy, const bf16_t* yact,
                 float* slab, int B, int H, int W, int Cout, int chunk, hipStream_t s);
void conv1_wgrad(const void* x, bool x_is_u8, BatchIdx bi, const float* dy, const float* yact,
                 float* slab, int B, int H, int W, int Cout, int chunk, hipStream_t s);

// ---- 3x3 / s1 / p1 NHWC conv (MFMA) --------------------------------------------------
// Fuse level 3 (bf16 SimpleCNN forward with the fc epilogue and the conv1 recompute): the
// forward also produces dZ2 = relu2'(a2) * (dL . W_fc) for its own pixels, so the fc
// backward leaves the critical path.  Every block publishes its partial logits
// (write-through) and adds 1 to the arrival counter of each image it touches, waits until
// every block of its image(s) has arrived, sums the image's logits in the fc_bwd prologue's
// fixed order, evaluates the softmax cross-entropy gradient dL of its image(s) and then dZ2
// from the bf16 fc weight fragments it already holds for the fc partials (fc_bwd's FMA
// order: bit-identical dZ2).  All blocks must be co-resident (conv3x3_fwd_dz_fits).
constexpr int FWD_DZ_CNT_STRIDE = 64;  // ints between two images' counters (256 B: no shared line)
struct FwdDz {
  bf16_t* dz2 = nullptr;          // [B*H*W][Cout] out (write-through)
  float* dz2_f32 = nullptr;       // the same, exact-fp32 step
  int* img_cnt = nullptr;         // [B][FWD_DZ_CNT_STRIDE] arrival counters (first int of each
                                  // row), zero on entry (re-zeroed by the step's fc backward:
                                  // FcBwdExtras::zero_i32)
  const float* fc_bias = nullptr;
  float gscale = 1.f;             // 1 / B (mean cross-entropy)
  int* err = nullptr;             // set to 3 when the wait times out (results invalid)
  // optional: dL [B][10] and the per-row losses [B] (the block holding an image's first
  // pixel writes its row) - the fc backward then needs no cross-entropy prologue
  float* dl_out = nullptr;
  float* loss_rows = nullptr;
};
// whether a level-3 forward of this shape keeps every block resident at once
bool conv3x3_fwd_dz_fits(int B, int H, int W, int pxt, int es = 2);
// bf16 operands (v_mfma_f32_16x16x32_bf16) or exact fp32 operands (v_mfma_f32_16x16x4_f32,
// the float overloads); `es` = element size of the LDS-size helpers (2 or 4).
void conv3x3_fwd(const bf16_t* X, const bf16_t* Wt, const float* bias, bf16_t* Y, int B, int H,
                 int W, int Cin, int Cout, bool relu, const bf16_t* wfc, float* fc_part, int NO,
                 int pxt, hipStream_t s, const C1Src* c1 = nullptr, const FwdDz* dz = nullptr);
// fp32: wfc (fused fc epilogue) is the fc weight in the FCFRAG order, fp32 (SHADOW_F32_FCFRAG)
void conv3x3_fwd(const float* X, const float* Wt, const float* bias, float* Y, int B, int H,
                 int W, int Cin, int Cout, bool relu, const float* wfc, float* fc_part, int NO,
                 int pxt, hipStream_t s, const C1Src* c1 = nullptr, const FwdDz* dz = nullptr);
void conv3x3_dgrad(const bf16_t* dY, const bf16_t* Yact, const bf16_t* WT, const bf16_t* Xact,
                   bf16_t* dX, int B, int H, int W, int Cin, int Cout, const void* x0, bool x0_u8,
                   BatchIdx bi, float* w1slab, int pxt, hipStream_t s, const C1Src* c1 = nullptr);
void conv3x3_dgrad(const float* dY, const float* Yact, const float* WT, const float* Xact,
                   float* dX, int B, int H, int W, int Cin, int Cout, const void* x0, bool x0_u8,
                   BatchIdx bi, float* w1slab, int pxt, hipStream_t s, const C1Src* c1 = nullptr);
int conv3x3_dgrad_blocks(int B, int H, int W, int pxt);
// fused level-1 conv backward (dgrad + conv1 wgrad slabs, and conv2 wgrad slabs) in one
// launch; Cin == 32 (conv1's channels), (Cout / 32) * (Cin / 16) == 4
// Xact != null: the dgrad role reads the forward's stored a1 (C1Src::a1_out) for its ReLU
// mask instead of recomputing conv1; the wgrad role too when wgrad_load_a1.
// fused_reduce != null: the same launch also does grad_reduce(*fused_reduce) (the wgrad
// blocks reduce the slabs after an in-launch arrival count, red_done: 8 counters 32 ints
// apart, zeroed beforehand - by the step's forward, C1Src::zero_i32); red_err[0] = 2 if
// that wait timed out.  SimpleCNN geometry only, and only while the wgrad blocks fit in
// half the launch's resident capacity (the whole capacity when `exclusive`: nothing else
// runs on the GPU meanwhile); returns whether the reduction was fused (false:
// the caller runs grad_reduce).  wgrad_split == 2 (bf16, SimpleCNN geometry): two wgrad
// blocks per slab row, one per half of the input channels (bit-identical slabs).
struct SlabSet;
struct BwdFc;
struct BwdXar;
constexpr int SYNC_RED_INTS = 256;  // ints of the 8 arrival counters (32 apart) of red_done
// fc != null (fuse level 3, single process): the same launch also runs the fc weight
// gradient + fused SGD as a third role (conv3x3_bwd_fc_role_ok shapes only; BwdFc below)
bool conv3x3_bwd(const bf16_t* dY, const bf16_t* WT, bf16_t* dX, float* w1slab, float* slab, int B,
                 int H, int W, int Cin, int Cout, int pxt, int R, const C1Src& c1, const bf16_t* Xact,
                 bool wgrad_load_a1, hipStream_t s, const SlabSet* fused_reduce = nullptr,
                 int* red_done = nullptr, int* red_err = nullptr, int wgrad_split = 1, const BwdFc* fc = nullptr,
                 bool exclusive = false, const BwdXar* xar = nullptr, bool* xar_used = nullptr);
bool conv3x3_bwd_fc_role_ok(int H, int W, int Cin, int Cout, int pxt, int wgrad_split);
// exact fp32: wgrad_split 2 (pxt 2, conv1 recomputed) splits both roles over input-channel
// halves at two blocks per CU (dgrad weights read from global); bit-identical to split 1
bool conv3x3_bwd(const float* dY, const float* WT, float* dX, float* w1slab, float* slab, int B,
                 int H, int W, int Cin, int Cout, int pxt, int R, const C1Src& c1, const float* Xact,
                 bool wgrad_load_a1, hipStream_t s, const SlabSet* fused_reduce = nullptr,
                 int* red_done = nullptr, int* red_err = nullptr, int wgrad_split = 1, const BwdFc* fc = nullptr,
                 bool exclusive = false, const BwdXar* xar = nullptr, bool* xar_used = nullptr);
size_t conv3x3_bwd_lds(int W, int Cin, int Cout, int pxt, int R, int es = 2, int cs = 1);
int conv3x3_wgrad_blocks(int B, int H, int R);
size_t conv3x3_wgrad_lds(int W, int Cin, int Cout, int R, bool a1x = false, int es = 2);
size_t conv3x3_fwd_lds(int W, int Cin, int pxt, bool a1x = false, int es = 2);
size_t conv3x3_dgrad_lds(int W, int Cout, int pxt, bool fuse_w1, int es = 2);
void conv3x3_wgrad(const bf16_t* dY, const bf16_t* Yact, const bf16_t* X, float* slab, int B,
                   int H, int W, int Cin, int Cout, int R, hipStream_t s, const C1Src* c1 = nullptr);
void conv3x3_wgrad(const float* dY, const float* Yact, const float* X, float* slab, int B,
                   int H, int W, int Cin, int Cout, int R, hipStream_t s, const C1Src* c1 = nullptr);

// ---- general NHWC implicit-GEMM convolution (conv_gemm.hip) ------------------------
struct ConvGeom {
  int N, H, W, Cin, OH, OW, Cout, KH, KW, stride, pad;
};
// A BatchNorm (+ ReLU) applied by the CONSUMER of a conv output while it loads it:
// value = bf16(relu(x * invstd * gamma + (beta - mean * invstd * gamma))), bitwise what
// bn_apply would have stored (resnet_ops.hip bn_affine8).  mean == nullptr: none.
struct BnAffine {
  const float* mean = nullptr;
  const float* invstd = nullptr;
  const float* gamma = nullptr;
  const float* beta = nullptr;
};
int* bn_ticket_slots(int n);  // zeroed, self-resetting ticket words (round-robin pool)
// launch plan: pixel tile bp (64/128), channel tile bc (64/128), K splits (grid.z)
struct ConvPlan {
  int bp, bc, splits, ks_per, grid_x, grid_y, grid_z;
  int parity;  // dgrad, stride 2: one dense GEMM per input-pixel parity class
  int halo;    // fwd, stride-1 3x3: LDS halo-tile kernel (conv_halo.hip)
};
// bp / bc / splits = 0, parity / halo = -1: chosen (tuned on ResNet-18, see conv_gemm.hip)
ConvPlan conv_gemm_plan(const ConvGeom& g, bool dgrad, int bp, int bc, int splits, int parity = -1,
                        int halo = -1);
bool conv_halo_fits(const ConvGeom& g, int bp);
int conv_halo_rows(const ConvGeom& g, int bp);
// tap-fused stride-1 3x3 weight gradient (conv_halo.hip): chunks of whole output rows
bool conv_halo_wgrad_ok(const ConvGeom& g);
int conv_halo_wgrad_row_quantum(const ConvGeom& g);  // rows per chunk must be a multiple
void conv_halo_wgrad(const ConvGeom& g, const bf16_t* dY, const bf16_t* X, float* out, int rows_per_chunk,
                     bool accum, hipStream_t s, int cit = 32,  // cit: input channels per block (16 | 32)
                     const BnAffine* aff = nullptr);           // aff: X is raw, BN + ReLU applied on load
// wgrad plan overrides for sweeps / A-B: halo 0 = never, 1 / 2 = every eligible stride-1
// 3x3 layer (default 1); target = blocks per launch
void conv_gemm_wgrad_set_halo(int halo, int target, int cit = 0);  // cit 0 = auto, 16, 32
// pixels per chunk the weight-gradient launcher accepts: multiples of 32 (per-tap GEMM), or
// whole-row chunks for the halo kernel
bool conv_gemm_wgrad_ppc_ok(const ConvGeom& g, int ppc);
void conv_halo_fwd(const ConvGeom& g, int bp, int bc, int splits, const bf16_t* X, const bf16_t* Wt,
                   bf16_t* Y, float* stats, float* part, hipStream_t s, const BnAffine* aff = nullptr);
void conv_halo_dgrad(const ConvGeom& g, int bp, int bc, int splits, const bf16_t* dY, const bf16_t* Wt,
                     const bf16_t* Xact, bf16_t* dX, float* part, hipStream_t s);
int conv_gemm_stat_rows(const ConvGeom& g, const ConvPlan& pl);  // BN stats slab rows (fwd)
// splits > 1: `part` = fp32 workspace [splits][P][C]; no bias / ReLU on the split path
void conv_gemm_fwd(const ConvGeom& g, const ConvPlan& pl, const bf16_t* X, const bf16_t* Wt,
                   const float* bias, bf16_t* Y, bool relu, float* stats, float* part, hipStream_t s,
                   const BnAffine* aff = nullptr);  // aff: halo plans only
// W: the OHWI forward weight itself (read transposed through LDS)
void conv_gemm_dgrad(const ConvGeom& g, const ConvPlan& pl, const bf16_t* dY, const bf16_t* W,
                     const bf16_t* Xact, bf16_t* dX, float* part, hipStream_t s);
int conv_gemm_wgrad_chunks(const ConvGeom& g, int px_per_chunk);
void conv_gemm_wgrad_force_tile(int bm, int bn);  // 0, 0 = auto
int conv_gemm_wgrad_tiles(const ConvGeom& g);  // blocks per pixel chunk
int conv_gemm_wgrad_ppc(const ConvGeom& g);    // tuned pixels per chunk
// one chunk: out = the gradient ([Cout][T][Cin], stem: [Cout][T][3]), `accum` adds to it;
// several: out = slab [chunks][...] for grad_reduce
void conv_gemm_wgrad(const ConvGeom& g, const bf16_t* dY, const bf16_t* X, float* out,
                     int px_per_chunk, bool accum, hipStream_t s, int ks = 0,
                     const BnAffine* aff = nullptr);  // aff: only where the halo kernel runs
// whether conv_gemm_wgrad runs the halo kernel for this layer at this chunking
bool conv_gemm_wgrad_uses_halo(const ConvGeom& g, int px_per_chunk);

// ---- ResNet ops (resnet_ops.hip) -----------------------------------------------------
int bn_finalize_groups(int rows);  // ws of bn_finalize: [groups][2][C]
void bn_finalize(const float* slab, int rows, int C, float count, float eps, float momentum,
                 float* running_mean, float* running_var, float* save_mean, float* save_invstd,
                 long long* nbt, float* ws, hipStream_t s);
void bn_apply(const bf16_t* x, long P, int C, const float* mean, const float* invstd,
              const float* gamma, const float* beta, const bf16_t* res, bool relu, bf16_t* y,
              hipStream_t s);
void bn_bwd_set_px_per_block(int px);
int bn_bwd_rows(long P, int C, int* rpb);  // ws of bn_bwd: [rows][2][C]
// dout2 (optional): a second upstream gradient of the same tensor, summed on load
// (bf16-rounded, == autograd's add) - the ResNet block input's two consumers
void bn_bwd(const bf16_t* dout, const bf16_t* out, const bf16_t* x, long P, int C, const float* mean,
            const float* invstd, const float* gamma, float count, float* ws, float* sums,
            float* dgamma, float* dbeta, bool accum, bf16_t* dx, bf16_t* dres, hipStream_t s,
            const bf16_t* dout2 = nullptr, const float* mask_beta = nullptr);
// out == nullptr && mask_beta != nullptr: the ReLU mask is recomputed from x (the BN input)
// as bf16(x * invstd * gamma + (beta - mean * invstd * gamma)) > 0 - bitwise the sign of
// the output bn_apply stored (no residual add); saves reading the output tensor
void maxpool_fwd(const bf16_t* x, int N, int H, int W, int C, int OH, int OW, bf16_t* y,
                 unsigned char* amax, hipStream_t s, const BnAffine* bn = nullptr);
void maxpool_bwd(const bf16_t* dy, const unsigned char* amax, int N, int H, int W, int C, int OH,
                 int OW, bf16_t* dx, hipStream_t s, const bf16_t* dy2 = nullptr);
void image_gather_nhwc4(const unsigned char* imgs, const long long* idx, int B, int HW, long N,
                        bf16_t* out, hipStream_t s);
void avgpool_fwd(const bf16_t* x, int N, int HW, int C, float* y, hipStream_t s);
void avgpool_bwd(const float* dy, int N, int HW, int C, bf16_t* dx, hipStream_t s);
// accum: C += alpha A.B (+ bias) instead of C =
void sgemm(int M, int N, int K, const void* A, bool a_bf16, long sam, long sak, const void* B,
           bool b_bf16, long sbk, long sbn, float* C, long ldc, const float* bias, float alpha,
           hipStream_t s, bool accum = false);
void transpose_w(const float* w, int Co, int T, int Ci, bf16_t* wt, hipStream_t s);

// ---- Linear over NHWC-flattened activations -----------------------------------------
void fc_partial(const bf16_t* X, const bf16_t* Wf, float* part, int B, int HW, int C, int NO,
                hipStream_t s);
void fc_partial(const float* X, const float* Wf, float* part, int B, int HW, int C, int NO,
                hipStream_t s);
void fc_reduce(const float* part, const float* bias, float* out, int B, int G, int NO,
               hipStream_t s);
// Optional extras of fc_bwd's first block: fc bias gradient and the batch-mean loss
// (from per-row losses), written at loss_out[*step_ctr] (or [0]).
struct FcBwdExtras {
  float* dbias = nullptr;
  float dbias_scale = 1.f;
  const float* loss_rows = nullptr;
  float* loss_out = nullptr;
  const int* step_ctr = nullptr;
  // XENT: compute dL (softmax cross-entropy backward) in the prologue of every block
  // from the fused conv+fc partials [B][G][NO] instead of reading dL; loss_rows unused.
  const float* part = nullptr;  // fused conv partials [blk][2][NO] (common.h xent_batch_block)
  int HW = 0, CH = 0;           // image pixels, pixels per conv block
  const float* fc_bias = nullptr;
  const int* labels32 = nullptr;
  BatchIdx bi{};
  float gscale = 1.f;
  // Fused optimizer for the fc WEIGHT (single-process steps, where dW is final when this
  // kernel writes it): sgd.update != 0 -> p_w -= SGD(dW) in the dW epilogue, plus the
  // bf16 shadows.  Each block updates only the columns it alone reads, so it is race
  // free; the fc bias (read by every block's prologue) is updated by grad_reduce.
  SgdArgs sgd{};
  float* p_w = nullptr;       // fp32 master [NO][K]
  float* m_w = nullptr;       // momentum buffer [NO][K] (momentum != 0)
  bf16_t* sh_plain = nullptr;  // bf16 shadow [NO][K]
  bf16_t* sh_frag = nullptr;   // FCFRAG shadow (conv3x3_fwd epilogue order)
  float* sh_frag32 = nullptr;  // fp32 FCFRAG copy (the exact-fp32 forward's fc operand)
  int frag_HW = 0, frag_C = 0;
  int sys_store = 0;  // dW / dbias with system-scope stores (read by peers over xGMI)
  // Last-block epilogue (fuse level 3: this kernel runs BESIDE the conv backward, so nothing
  // after it in the step can own the fc bias): instead of block 0 writing dbias / the loss,
  // every block adds 1 to *last_ctr (zero on entry) when it is done - after its prologue read
  // the fc bias - and the block that arrives last writes dbias and the loss, applies the
  // fused SGD to the fc bias (p_b / m_b, when sgd.update), advances *step_inc (after reading
  // the loss index from step_ctr) and zeroes zero_i32[0, n_zero) (the forward's per-image
  // arrival counters, FwdDz::img_cnt).
  int* last_ctr = nullptr;
  float* p_b = nullptr;
  float* m_b = nullptr;
  int* step_inc = nullptr;
  int* zero_i32 = nullptr;      // zero_i32[i * zero_stride] = 0 for i < n_zero
  int n_zero = 0, zero_stride = 1;
  int last_n = 0;               // arrivals of the last-block count (0: the grid size)
};
// The fc role of the level-3 conv backward launch (conv3x3_bwd, fc != null): the fc weight
// gradient + fused SGD without dX, dL given (the forward's FwdDz::dl_out), on blocks
// [fc0, fc0 + nfc) whose waves each own one 128-column chunk (fc_dw_wave_chunk,
// bit-identical to fc_bwd); they never wait and are not counted by the fused reduction.
// Block 0 of the role finishes the fc bias (gradient + SGD), the loss and the step counter -
// nothing else in the launch reads them (ex.last_ctr must be null).
struct BwdFc {
  const void* a2 = nullptr;    // ReLU2 output [B][K] (bf16, or fp32 for the exact-fp32 step)
  const float* dl = nullptr;   // dL [B][10]
  float* dW = nullptr;         // null: fused optimizer only
  float scale = 1.f;
  long K = 0;
  int nconv = 0, fc0 = 0, nfc = 0;  // (set by the launcher: nfc = one 128-column chunk per wave)
  FcBwdExtras ex{};
};
size_t fc_bwd_lds(int B, int NO, bool xent, long npart = 0);  // npart: see linear.hip
void noop(int blocks, int* sink, hipStream_t s);
// dX == nullptr: no data gradient (fuse level 3: the conv forward produced dZ2); the weight
// columns are then not read at all
void fc_bwd(const float* dL, const bf16_t* X, const bf16_t* Wf, bf16_t* dX, float* dW, float scale,
            int B, long K, int NO, bool mask, hipStream_t s, const FcBwdExtras& ex = FcBwdExtras());
void fc_bwd(const float* dL, const float* X, const float* Wf, float* dX, float* dW, float scale,
            int B, long K, int NO, bool mask, hipStream_t s, const FcBwdExtras& ex = FcBwdExtras());

// ---- cross-entropy --------------------------------------------------------------------
void xent(const float* part, int G, const float* bias, int C, int B, const long long* labels64,
          const int* labels32, BatchIdx bi, float* logits_out, float* dlogits, float* loss_out,
          float* dbias, float gscale, float dbias_scale, hipStream_t s);

// ResNet-width heads (C > 64, labels64, no bias fold): one wave per row; false if unsupported
bool xent_wave_rows(const float* logits, int C, int B, const long long* labels, float* dlogits,
                    float* loss_out, float gscale, hipStream_t s);

void xent_rows(const float* part, int HW, int CH, const float* bias, int NO, int B,
               const int* labels32, BatchIdx bi, float* dlogits, float* loss_rows, float gscale,
               hipStream_t s);

// ---- optimizer / reductions -----------------------------------------------------------
// SHADOW_BF16_FCFRAG: fc weight [o][hw][c] (a = HW, b = C) -> the MFMA-fragment order
// read by the conv3x3_fwd FC epilogue, [o][hw/16][c/16][(c/4)%4][hw%16][c%4], so each
// wave-instruction of that epilogue loads 512 contiguous bytes.
// SHADOW_BF16_PAD4: a [..][3] weight (the ResNet stem) -> [..][4] with the 4th channel left
// at its zero fill (the stem conv's 16-B weight loads read it); sgd_kernel and the xGMI
// fused-SGD all-gather (shadow_one).
// SHADOW_F32_TAPT: the exact-fp32 engine's [tap][ci][co] copy of the conv2 weight (the
// data-gradient operand), a transposed fp32 copy - not a reduced-precision shadow; dst32.
// SHADOW_F32_FCFRAG: the exact-fp32 engine's fc weight in the FCFRAG order (fp32, dst32):
// the forward's fused fc epilogue then loads 1 KB contiguous per wave-instruction instead
// of 16 strided 64-byte runs.
enum { SHADOW_BF16 = 1, SHADOW_BF16_TAPT = 2, SHADOW_BF16_FCFRAG = 3, SHADOW_BF16_PAD4 = 4,
       SHADOW_F32_TAPT = 5, SHADOW_F32_FCFRAG = 6 };
constexpr int MAX_SHADOWS = 4;
struct ShadowRegion {
  long off, n;
  bf16_t* dst;
  int kind, a, b, c;  // TAPT: a = Cout, b = taps, c = Cin
  float* dst32 = nullptr;  // SHADOW_F32_TAPT destination
};
struct ShadowSet {
  ShadowRegion r[MAX_SHADOWS];
  int count;
};
struct SlabSeg {
  const float* slab;
  long row_stride, src_off, n;
  int rows;
  float* dst;
  float scale;
  // fused optimizer (SlabSet::sgd.update): master / momentum at the gradient's index,
  // bf16 shadow (plain) and / or the [tap][ci][co] transposed shadow (t_co/t_taps/t_ci)
  float* p = nullptr;
  float* m = nullptr;
  bf16_t* sh = nullptr;
  bf16_t* sh_t = nullptr;
  float* sh_t32 = nullptr;  // exact-fp32 engine: fp32 [tap][ci][co] copy (same t_* geometry)
  int t_co = 0, t_taps = 0, t_ci = 0;
  int accum = 0;  // dst += reduced * scale (gradient accumulation) instead of dst =
};
constexpr int MAX_SLAB_SEGS = 6;
struct SlabSet {
  SlabSeg s[MAX_SLAB_SEGS];
  int count;
  SgdArgs sgd{};              // update != 0 -> apply SGD to segments with p set
  int* step_ctr = nullptr;    // += 1 at the end (the step's last kernel)
  int sys_store = 0;          // dst with system-scope stores (read by peers over xGMI)
};
void sgd_step(float* p, const float* g, float* mbuf, long n, const SgdArgs& a, const ShadowSet& sh,
              int* step_ctr, hipStream_t s);
void grad_reduce(const SlabSet& ss, hipStream_t s);
// row groups (16 or 4) of the fixed summation order grad_reduce uses for this SlabSet
int grad_reduce_groups(const SlabSet& ss);
void scale_copy(float* dst, const float* src, long n, float scale, hipStream_t s);

// ---- direct two-shot xGMI all-reduce (allreduce.hip) ----------------------------------
constexpr int XGMI_MAX_RANKS = 8, XGMI_THREADS = 256, XGMI_MAX_BLOCKS = 1024;
constexpr int XGMI_GRID_CAP = 256;  // blocks per all-reduce launch: one per CU (block-strided chunks beyond)
// signal words of one channel: [block][src rank] flags, [block] call counters, error word
constexpr int XGMI_FLAG_OFF = 0;
constexpr int XGMI_SEQ_OFF = XGMI_MAX_BLOCKS * XGMI_MAX_RANKS;
constexpr int XGMI_ERR_OFF = XGMI_SEQ_OFF + XGMI_MAX_BLOCKS;
constexpr int XGMI_SIG_WORDS = XGMI_ERR_OFF + 64;
// error word of a channel: 0 = ok, else the first barrier wait that timed out (sticky):
// bit 31 | block << 12 | peer rank << 4 | phase (0: entry barrier B0, 1: after the
// reduce-scatter B1, 2: the one-shot barrier)
enum { XGMI_PHASE_B0 = 0, XGMI_PHASE_B1 = 1, XGMI_PHASE_ONESHOT = 2 };
__host__ __device__ constexpr unsigned xgmi_error_code(int block, int peer, int phase) {
  return 0x80000000u | ((unsigned)block << 12) | ((unsigned)(peer & 0xff) << 4) | (unsigned)(phase & 0xf);
}
constexpr double XGMI_DEFAULT_TIMEOUT_S = 30.0;  // per barrier spin (a slow peer is not an error)
struct XgmiArgs {
  float* data[XGMI_MAX_RANKS];    // every rank's gradient buffer (peer-mapped; [rank] = own)
  float* stage[XGMI_MAX_RANKS];   // every rank's stage buffer, 2 x slice floats (one-shot: 2 x n)
  unsigned* sig[XGMI_MAX_RANKS];  // every rank's signal words (uncached)
  long off, n, slice;             // bucket offset / length in the gradient buffer; xgmi_slice(n, world)
  int oneshot;                    // 1: publish whole bucket, one barrier, every rank sums all (small buckets)
  int publish;                    // two-shot: re-store my bucket system-scope before B0 (producers used
                                  // plain stores, e.g. autograd kernels in the module path)
  float scale;                    // applied to the result (1: producers prescaled by 1/world)
  float prescale;                 // publish pass / one-shot publish: my values times this before the
                                  // rank-order sum (DDP's prescale-by-1/world, then SUM; 1 otherwise)
  int rank, world;
  unsigned long long timeout_ticks;  // per barrier spin, 100 MHz ticks
  // Optional optimizer fused into the all-gather (sgd.update != 0): every rank applies
  // the same SGD to the same reduced gradient, so parameters stay bitwise identical:
  // param / momentum at the element's flat index (params + off + k), bf16 shadows of
  // the regions in `sh` (indices relative to the flat parameter buffer).
  SgdArgs sgd;
  float* params;
  float* mbuf;
  ShadowSet sh;
  int* step_ctr;  // += 1 by block 0 at the end (the step's last kernel), may be null
};
long xgmi_slice(long n, int world);  // two-shot slice: n / world rounded up to whole quads
int xgmi_blocks(long n, int world, bool oneshot = false);
void xgmi_allreduce(const XgmiArgs& a, int blocks, hipStream_t s);

// In-launch bucket all-reduce of the multi-GPU level-3 step (engine dist_mode 2,
// conv3x3.hip XAR): role blocks at the HEAD of the conv backward grid run the direct xGMI
// all-reduce + fused SGD (xgmi_body.h) of each gradient bucket as soon as its gradients are
// final inside the same launch - bucket 0 (the fc bucket) once every fc-role block has
// counted itself into fc_done, bucket 1 (the conv bucket) once every fused slab reducer has
// counted itself into red_done (and the fc role too: a single bucket may hold both).  No
// kernel boundary and no cross-stream edge separates a gradient from its all-reduce.
struct BwdXar {
  // [0] / [1]: the stage-0 / stage-1 bucket's arguments (XgmiComm::make_args, step_ctr null)
  // in DEVICE memory - held in the kernel-argument struct, the compiler copied the whole
  // struct to scratch for the body's rank-indexed peer pointers
  const XgmiArgs* args = nullptr;
  int nblk0 = 0, nblk1 = 0;   // role blocks = the channel's grid (XgmiComm::blocks); 0 = none
  int* fc_done = nullptr;     // completion counters, zeroed by the step's forward
  int* red_done = nullptr;
  int* xar_done = nullptr;    // role blocks done: the last one advances step_ctr
  int fc_expect = 0, red_expect = 0;  // (set by the launcher)
  int* step_ctr = nullptr;
  int* err = nullptr;         // 4: a completion wait timed out
};
constexpr int XAR_ERR = 4;
// Both buckets' all-reduces in ONE launch (engine dist_mode 3, behind the conv backward on
// the compute stream): blocks [0, nblk0) run bucket 0, [nblk0, nblk0 + nblk1) bucket 1,
// concurrently; the waits / expected counts of BwdXar are unused, the last block advances
// step_ctr (xar_done).
void xgmi_allreduce_pair(const BwdXar& x, hipStream_t s);
// dist_mode 4: the pair's roles (fused SGD stored write-through, each block counted into
// done_fc / done_conv - zeroed beforehand) and the NEXT step's bf16 level-3 forward
// (pxt 1, B images; its blocks wait for the buckets' counts before reading their
// parameters) in ONE launch (conv3x3.hip step_head_kernel).  Returns false without
// launching when the whole grid does not fit the GPU at once (the caller then runs the pair
// and the forward as two launches - the same bits).  err: sync_err (code 5 on a wait timeout).
// late: shadows of the conv bucket the forward does not read (the conv2 weight's [tap][ci][co]
// copy for the next backward), written by the conv bucket's blocks AFTER their count - their
// scattered write-through stores no longer sit in the drain the forward waits for
bool conv3x3_step_head(const BwdXar& x, int* done_fc, int* done_conv, const bf16_t* Wt, const float* bias,
                       bf16_t* Y, int B, const bf16_t* wfc, float* fc_part, const C1Src& c1, const FwdDz& dz,
                       int* err, hipStream_t s, const ShadowSet* late = nullptr);
bool conv3x3_step_head_fits(int nx, int B);
int conv3x3_step_head_slots();  // resident blocks of the step-head kernel on this GPU

}  // namespace ddp_amd
