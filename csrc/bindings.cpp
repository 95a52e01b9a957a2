// pybind11 surface of ddp_amd._C: adapts at::Tensor to the raw-pointer kernel /
// runtime API.  Every op validates device, dtype, contiguity and shape before it
// launches (a wrong shape on a hand-written kernel is an out-of-bounds access on
// the GPU), and launches on torch's current HIP stream unless stated otherwise.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <optional>

#include "kernels/launchers.h"
#include "runtime/runtime.h"

namespace py = pybind11;
using at::Tensor;
using namespace ddp_amd;

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_cuda(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
void check(const Tensor& t, const char* name, at::ScalarType st) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == st, name, " has dtype ", t.scalar_type(), ", expected ", st);
}
bf16_t* bf(const Tensor& t) { return reinterpret_cast<bf16_t*>(t.data_ptr()); }
const bf16_t* cbf(const Tensor& t) { return reinterpret_cast<const bf16_t*>(t.data_ptr()); }
const bf16_t* obf(const std::optional<Tensor>& t, const char* name) {
  if (!t) return nullptr;
  check(*t, name, at::kBFloat16);
  return cbf(*t);
}

// Activation dtype of an op: bf16 (default path) or fp32 (--dtype fp32, exact-fp32 MFMA).
// Every activation / weight-operand tensor of one call must share it.
bool act_f32(const Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kFloat, name,
              " must be bfloat16 or float32, got ", t.scalar_type());
  return t.scalar_type() == at::kFloat;
}
void check_act(const Tensor& t, const char* name, bool f32) {
  check(t, name, f32 ? at::kFloat : at::kBFloat16);
}
template <typename T>
T* tp(const Tensor& t) { return reinterpret_cast<T*>(t.data_ptr()); }
template <typename T>
const T* otp(const std::optional<Tensor>& t, const char* name, bool f32) {
  if (!t) return nullptr;
  check_act(*t, name, f32);
  return tp<T>(*t);
}

BatchIdx make_bi(const std::optional<Tensor>& idx, const std::optional<Tensor>& ctr, int stride,
                 int offset, long n_rows = 0x7fffffff) {
  BatchIdx bi{nullptr, nullptr, stride, offset};
  bi.n_rows = (int)std::min<long>(n_rows, 0x7fffffff);
  if (idx) {
    check(*idx, "idx", at::kInt);
    bi.idx = idx->data_ptr<int>();
    bi.n_idx = (int)idx->numel();
    TORCH_CHECK(bi.n_idx > 0, "empty index list");
  }
  if (ctr) { check(*ctr, "step_ctr", at::kInt); bi.step_ctr = ctr->data_ptr<int>(); }
  return bi;
}

void kcheck() {
  hipError_t e = hipGetLastError();
  TORCH_CHECK(e == hipSuccess, "kernel launch failed: ", hipGetErrorString(e));
}

// ------------------------------------------------------------------ ops
void op_conv1_fwd(const Tensor& x, std::optional<Tensor> idx, std::optional<Tensor> ctr, int stride,
                  int offset, const Tensor& w, const Tensor& b, Tensor& y, int B, int H, int W) {
  check_cuda(x, "x");
  const bool u8 = x.scalar_type() == at::kByte;
  TORCH_CHECK(u8 || x.scalar_type() == at::kFloat, "x must be uint8 or float32");
  check(w, "w", at::kFloat); check(b, "b", at::kFloat);
  const bool f32 = act_f32(y, "y");
  const int Cout = (int)b.numel();
  TORCH_CHECK(Cout % 8 == 0 && 256 % (Cout / 8) == 0, "conv1: Cout must be 8..256, power of two");
  TORCH_CHECK(w.numel() == (long)Cout * 9, "conv1: weight must be [Cout,1,3,3]");
  TORCH_CHECK(y.numel() == (long)B * H * W * Cout, "conv1: bad output size");
  if (!u8) {
    TORCH_CHECK(x.numel() >= (long)B * H * W, "conv1: input too small");
  } else {
    TORCH_CHECK(x.numel() % ((long)H * W) == 0, "conv1: dataset must be [N,H,W]");
  }
  const BatchIdx bi = make_bi(idx, ctr, stride, offset, x.numel() / ((long)H * W));
  if (f32) conv1_fwd(x.data_ptr(), u8, bi, w.data_ptr<float>(), b.data_ptr<float>(), tp<float>(y), B, H, W, Cout, cur_stream());
  else conv1_fwd(x.data_ptr(), u8, bi, w.data_ptr<float>(), b.data_ptr<float>(), bf(y), B, H, W, Cout, cur_stream());
  kcheck();
}

void op_conv1_wgrad(const Tensor& x, std::optional<Tensor> idx, std::optional<Tensor> ctr,
                    int stride, int offset, const Tensor& dy, std::optional<Tensor> yact,
                    Tensor& slab, int B, int H, int W, int Cout, int chunk) {
  check_cuda(x, "x");
  const bool u8 = x.scalar_type() == at::kByte;
  const bool f32 = act_f32(dy, "dy");
  check(slab, "slab", at::kFloat);
  TORCH_CHECK(dy.numel() == (long)B * H * W * Cout, "conv1_wgrad: bad dy size");
  TORCH_CHECK(Cout * 10 <= 320 * 4, "conv1_wgrad: Cout too large");
  TORCH_CHECK(slab.numel() >= (long)conv1_wgrad_blocks(B, H, W, chunk) * Cout * 10, "slab too small");
  const BatchIdx bi = make_bi(idx, ctr, stride, offset, x.numel() / ((long)H * W));
  if (f32)
    conv1_wgrad(x.data_ptr(), u8, bi, tp<float>(dy), otp<float>(yact, "yact", true), slab.data_ptr<float>(), B, H,
                W, Cout, chunk, cur_stream());
  else
    conv1_wgrad(x.data_ptr(), u8, bi, cbf(dy), obf(yact, "yact"), slab.data_ptr<float>(), B, H, W, Cout, chunk,
                cur_stream());
  kcheck();
}

void op_conv3x3_fwd(const Tensor& X, const Tensor& Wt, const Tensor& bias, Tensor& Y, bool relu,
                    std::optional<Tensor> wfc, std::optional<Tensor> fc_part, int NO, int pxt) {
  const bool f32 = act_f32(X, "X");
  check_act(Wt, "Wt", f32); check(bias, "bias", at::kFloat); check_act(Y, "Y", f32);
  TORCH_CHECK(X.dim() == 4 && Y.dim() == 4, "conv3x3_fwd: X, Y must be NHWC 4-d");
  const int B = X.size(0), H = X.size(1), W = X.size(2), Cin = X.size(3), Cout = Y.size(3);
  TORCH_CHECK(Y.size(0) == B && Y.size(1) == H && Y.size(2) == W, "conv3x3_fwd: Y shape");
  TORCH_CHECK(Cin % 32 == 0 && Cout % 64 == 0, "conv3x3_fwd: Cin%32, Cout%64 required");
  TORCH_CHECK(Wt.numel() == (long)Cout * 9 * Cin && bias.numel() == Cout, "conv3x3_fwd: weight shape");
  TORCH_CHECK(pxt == 1 || pxt == 2, "pxt must be 1 or 2");
  TORCH_CHECK(conv3x3_fwd_lds(W, Cin, pxt, false, f32 ? 4 : 2) <= 160 * 1024, "conv3x3_fwd: LDS budget exceeded");
  const void* wf = nullptr;
  float* part = nullptr;
  if (wfc) {
    check_act(*wfc, "wfc", f32);
    TORCH_CHECK(fc_part.has_value(), "fc_part required with wfc");
    check(*fc_part, "fc_part", at::kFloat);
    TORCH_CHECK(Cout == 64 && (H * W) % 16 == 0 && NO == 10, "fused fc: Cout==64, HW%16==0, NO==10");
    TORCH_CHECK(wfc->numel() == (long)NO * H * W * Cout, "fused fc: wfc shape");
    TORCH_CHECK(fc_part->numel() >= 2L * conv3x3_dgrad_blocks(B, H, W, pxt) * NO,
                "fused fc: fc_part too small ([blocks][2][NO])");
    wf = wfc->data_ptr();
    part = fc_part->data_ptr<float>();
  }
  if (f32)
    conv3x3_fwd(tp<float>(X), tp<float>(Wt), bias.data_ptr<float>(), tp<float>(Y), B, H, W, Cin, Cout, relu,
                (const float*)wf, part, NO, pxt, cur_stream());
  else
    conv3x3_fwd(cbf(X), cbf(Wt), bias.data_ptr<float>(), bf(Y), B, H, W, Cin, Cout, relu, (const bf16_t*)wf,
                part, NO, pxt, cur_stream());
  kcheck();
}

void op_conv3x3_dgrad(const Tensor& dY, std::optional<Tensor> Yact, const Tensor& WT,
                      std::optional<Tensor> Xact, Tensor& dX, int pxt) {
  const bool f32 = act_f32(dY, "dY");
  check_act(WT, "WT", f32); check_act(dX, "dX", f32);
  TORCH_CHECK(dY.dim() == 4 && dX.dim() == 4, "conv3x3_dgrad: NHWC 4-d");
  const int B = dY.size(0), H = dY.size(1), W = dY.size(2), Cout = dY.size(3), Cin = dX.size(3);
  TORCH_CHECK(dX.size(0) == B && dX.size(1) == H && dX.size(2) == W, "conv3x3_dgrad: dX shape");
  TORCH_CHECK(Cin % 32 == 0 && Cout % 32 == 0, "conv3x3_dgrad: Cin%32, Cout%32 required");
  TORCH_CHECK(WT.numel() == (long)Cout * 9 * Cin, "conv3x3_dgrad: WT shape");
  if (Yact) TORCH_CHECK(Yact->sizes() == dY.sizes(), "Yact shape");
  if (Xact) TORCH_CHECK(Xact->sizes() == dX.sizes(), "Xact shape");
  TORCH_CHECK(pxt == 1 || pxt == 2, "pxt must be 1 or 2");
  TORCH_CHECK(conv3x3_dgrad_lds(W, Cout, pxt, false, f32 ? 4 : 2) <= 160 * 1024, "conv3x3_dgrad: LDS budget");
  BatchIdx bi{nullptr, nullptr, 0, 0};
  if (f32)
    conv3x3_dgrad(tp<float>(dY), otp<float>(Yact, "Yact", true), tp<float>(WT), otp<float>(Xact, "Xact", true),
                  tp<float>(dX), B, H, W, Cin, Cout, nullptr, false, bi, nullptr, pxt, cur_stream());
  else
    conv3x3_dgrad(cbf(dY), obf(Yact, "Yact"), cbf(WT), obf(Xact, "Xact"), bf(dX), B, H, W, Cin, Cout,
                  nullptr, false, bi, nullptr, pxt, cur_stream());
  kcheck();
}

void op_conv3x3_dgrad_fused_w1(const Tensor& dY, const Tensor& WT, const Tensor& Xact, Tensor& dX,
                               const Tensor& x0, std::optional<Tensor> idx,
                               std::optional<Tensor> ctr, int stride, int offset, Tensor& w1slab,
                               int pxt) {
  check(dY, "dY", at::kBFloat16); check(WT, "WT", at::kBFloat16); check(dX, "dX", at::kBFloat16);
  check(Xact, "Xact", at::kBFloat16); check(w1slab, "w1slab", at::kFloat); check_cuda(x0, "x0");
  const int B = dY.size(0), H = dY.size(1), W = dY.size(2), Cout = dY.size(3), Cin = dX.size(3);
  TORCH_CHECK(Cin == 32, "fused conv1 wgrad requires Cin == 32");
  TORCH_CHECK(WT.numel() == (long)Cout * 9 * Cin && Xact.sizes() == dX.sizes(), "shapes");
  TORCH_CHECK(w1slab.numel() >= (long)conv3x3_dgrad_blocks(B, H, W, pxt) * 320, "w1slab too small");
  const bool u8 = x0.scalar_type() == at::kByte;
  conv3x3_dgrad(cbf(dY), nullptr, cbf(WT), cbf(Xact), bf(dX), B, H, W, Cin, Cout, x0.data_ptr(), u8,
                make_bi(idx, ctr, stride, offset, x0.numel() / ((long)H * W)), w1slab.data_ptr<float>(), pxt, cur_stream());
  kcheck();
}

void op_conv3x3_wgrad(const Tensor& dY, std::optional<Tensor> Yact, const Tensor& X, Tensor& slab,
                      int R) {
  const bool f32 = act_f32(dY, "dY");
  check_act(X, "X", f32); check(slab, "slab", at::kFloat);
  const int B = dY.size(0), H = dY.size(1), W = dY.size(2), Cout = dY.size(3), Cin = X.size(3);
  TORCH_CHECK(X.size(0) == B && X.size(1) == H && X.size(2) == W, "conv3x3_wgrad: X shape");
  TORCH_CHECK(Cout % 32 == 0 && Cin % 16 == 0 && ((Cout / 32) * (Cin / 16)) % 4 == 0,
              "conv3x3_wgrad: unsupported channel counts");
  TORCH_CHECK(R >= 1 && R <= H, "conv3x3_wgrad: bad row chunk");
  TORCH_CHECK(conv3x3_wgrad_lds(W, Cin, Cout, R, false, f32 ? 4 : 2) <= 160 * 1024, "conv3x3_wgrad: LDS too large");
  TORCH_CHECK(slab.numel() >= (long)conv3x3_wgrad_blocks(B, H, R) * ((long)Cout * 9 * Cin + Cout),
              "conv3x3_wgrad: slab too small");
  if (Yact) TORCH_CHECK(Yact->sizes() == dY.sizes(), "Yact shape");
  if (f32)
    conv3x3_wgrad(tp<float>(dY), otp<float>(Yact, "Yact", true), tp<float>(X), slab.data_ptr<float>(), B, H, W,
                  Cin, Cout, R, cur_stream());
  else
    conv3x3_wgrad(cbf(dY), obf(Yact, "Yact"), cbf(X), slab.data_ptr<float>(), B, H, W, Cin, Cout, R,
                  cur_stream());
  kcheck();
}

void op_fc_partial(const Tensor& X, const Tensor& Wf, Tensor& part) {
  const bool f32 = act_f32(X, "X");
  check_act(Wf, "Wf", f32); check(part, "part", at::kFloat);
  TORCH_CHECK(X.dim() == 4, "fc_partial: X must be NHWC");
  const int B = X.size(0), HW = X.size(1) * X.size(2), C = X.size(3);
  TORCH_CHECK(HW % 16 == 0 && C % 8 == 0, "fc_partial: HW%16, C%8");
  const int NO = (int)(Wf.numel() / ((long)HW * C));
  TORCH_CHECK((long)NO * HW * C == Wf.numel() && NO <= 16, "fc_partial: weight shape");
  TORCH_CHECK(part.numel() >= (long)B * (HW / 16) * NO, "fc_partial: part too small");
  if (f32) fc_partial(tp<float>(X), tp<float>(Wf), part.data_ptr<float>(), B, HW, C, NO, cur_stream());
  else fc_partial(cbf(X), cbf(Wf), part.data_ptr<float>(), B, HW, C, NO, cur_stream());
  kcheck();
}

void op_fc_reduce(const Tensor& part, std::optional<Tensor> bias, Tensor& out, int B, int G, int NO) {
  check(part, "part", at::kFloat); check(out, "out", at::kFloat);
  TORCH_CHECK(part.numel() >= (long)B * G * NO && out.numel() >= (long)B * NO, "fc_reduce sizes");
  const float* bp = nullptr;
  if (bias) { check(*bias, "bias", at::kFloat); bp = bias->data_ptr<float>(); }
  fc_reduce(part.data_ptr<float>(), bp, out.data_ptr<float>(), B, G, NO, cur_stream());
  kcheck();
}

void op_fc_bwd(const Tensor& dL, const Tensor& X, const Tensor& Wf, Tensor& dX, Tensor& dW,
               double scale, bool mask, std::optional<Tensor> dbias, std::optional<Tensor> loss_rows,
               std::optional<Tensor> loss_out) {
  check(dL, "dL", at::kFloat);
  const bool f32 = act_f32(X, "X");
  check_act(Wf, "Wf", f32); check_act(dX, "dX", f32); check(dW, "dW", at::kFloat);
  const int B = dL.size(0), NO = dL.size(1);
  const long K = X.numel() / B;
  TORCH_CHECK(X.numel() == (long)B * K && dX.numel() == X.numel(), "fc_bwd: X/dX shape");
  TORCH_CHECK(Wf.numel() == (long)NO * K && dW.numel() == Wf.numel() && NO <= 16, "fc_bwd: W shape");
  TORCH_CHECK(fc_bwd_lds(B, NO, false) <= 160 * 1024, "fc_bwd: batch too large for LDS");
  TORCH_CHECK(K % 2 == 0, "fc_bwd: in_features must be even");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(dW.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(X.data_ptr()) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(dX.data_ptr()) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(Wf.data_ptr()) % 8 == 0,
              "fc_bwd: misaligned buffers");
  FcBwdExtras ex;
  if (dbias) {
    check(*dbias, "dbias", at::kFloat);
    TORCH_CHECK(dbias->numel() == NO, "dbias size");
    ex.dbias = dbias->data_ptr<float>();
    ex.dbias_scale = (float)scale;
  }
  if (loss_rows) {
    check(*loss_rows, "loss_rows", at::kFloat);
    TORCH_CHECK(loss_out.has_value() && loss_rows->numel() >= B, "loss_rows needs loss_out");
    check(*loss_out, "loss_out", at::kFloat);
    ex.loss_rows = loss_rows->data_ptr<float>();
    ex.loss_out = loss_out->data_ptr<float>();
  }
  if (f32)
    fc_bwd(dL.data_ptr<float>(), tp<float>(X), tp<float>(Wf), tp<float>(dX), dW.data_ptr<float>(), (float)scale,
           B, K, NO, mask, cur_stream(), ex);
  else
    fc_bwd(dL.data_ptr<float>(), cbf(X), cbf(Wf), bf(dX), dW.data_ptr<float>(), (float)scale, B, K,
           NO, mask, cur_stream(), ex);
  kcheck();
}

void op_xent(const Tensor& part, int G, std::optional<Tensor> bias, const Tensor& labels,
             std::optional<Tensor> logits_out, Tensor& dlogits, Tensor& loss_out,
             std::optional<Tensor> dbias, double gscale, double dbias_scale) {
  check(part, "part", at::kFloat); check(dlogits, "dlogits", at::kFloat);
  check(loss_out, "loss_out", at::kFloat);
  const int B = dlogits.size(0), C = dlogits.size(1);
  TORCH_CHECK(C <= 1024, "xent: at most 1024 classes");
  TORCH_CHECK(part.numel() >= (long)B * G * C, "xent: partials too small");
  check_cuda(labels, "labels");
  TORCH_CHECK(labels.numel() == B, "xent: labels size");
  const long long* l64 = nullptr;
  const int* l32 = nullptr;
  if (labels.scalar_type() == at::kLong) l64 = reinterpret_cast<const long long*>(labels.data_ptr());
  else { TORCH_CHECK(labels.scalar_type() == at::kInt, "labels int32/int64"); l32 = labels.data_ptr<int>(); }
  const float* bp = nullptr;
  if (bias) { check(*bias, "bias", at::kFloat); bp = bias->data_ptr<float>(); }
  float* lo = nullptr;
  if (logits_out) { check(*logits_out, "logits_out", at::kFloat); lo = logits_out->data_ptr<float>(); }
  float* db = nullptr;
  if (dbias) { check(*dbias, "dbias", at::kFloat); db = dbias->data_ptr<float>(); }
  BatchIdx bi{nullptr, nullptr, 0, 0};
  xent(part.data_ptr<float>(), G, bp, C, B, l64, l32, bi, lo, dlogits.data_ptr<float>(),
       loss_out.data_ptr<float>(), db, (float)gscale, (float)dbias_scale, cur_stream());
  kcheck();
}

void op_xent_rows(const Tensor& part, int HW, int CH, const Tensor& bias, const Tensor& labels32,
                  std::optional<Tensor> idx, Tensor& dlogits, Tensor& loss_rows, double gscale) {
  check(part, "part", at::kFloat); check(bias, "bias", at::kFloat); check(labels32, "labels", at::kInt);
  check(dlogits, "dlogits", at::kFloat); check(loss_rows, "loss_rows", at::kFloat);
  const int B = dlogits.size(0), NO = dlogits.size(1);
  TORCH_CHECK(bias.numel() == NO && NO <= 16, "xent_rows: at most 16 classes");
  TORCH_CHECK(CH > 0 && CH <= HW && HW / CH + 2 <= 16, "xent_rows: block geometry");
  TORCH_CHECK((long)B * HW < (1L << 31), "xent_rows: B * HW must fit in int32");
  const long nblk = ((long)B * HW + CH - 1) / CH;
  TORCH_CHECK(part.numel() >= nblk * 2 * NO && loss_rows.numel() >= B, "xent_rows: sizes");
  TORCH_CHECK((long)B * NO * 4 <= 64 * 1024, "xent_rows: batch too large");
  BatchIdx bi = make_bi(idx, std::nullopt, 0, 0, labels32.numel());
  if (!idx) TORCH_CHECK(labels32.numel() >= B, "xent_rows: labels");
  xent_rows(part.data_ptr<float>(), HW, CH, bias.data_ptr<float>(), NO, B, labels32.data_ptr<int>(),
            bi, dlogits.data_ptr<float>(), loss_rows.data_ptr<float>(), (float)gscale, cur_stream());
  kcheck();
}

// ------------------------------------------------------------------ ResNet ops
ConvGeom geom_of(const Tensor& X, const Tensor& Y, int KH, int KW, int stride, int pad) {
  TORCH_CHECK(X.dim() == 4 && Y.dim() == 4, "NHWC 4-d tensors expected");
  ConvGeom g{(int)X.size(0), (int)X.size(1), (int)X.size(2), (int)X.size(3), (int)Y.size(1),
             (int)Y.size(2), (int)Y.size(3), KH, KW, stride, pad};
  TORCH_CHECK(Y.size(0) == X.size(0), "batch mismatch");
  TORCH_CHECK(g.OH == (g.H + 2 * pad - KH) / stride + 1 && g.OW == (g.W + 2 * pad - KW) / stride + 1,
              "output spatial size does not match kernel/stride/pad");
  return g;
}

ConvPlan plan_of(const ConvGeom& g, bool dgrad, int bp, int bc, int splits, int parity = -1, int halo = -1) {
  TORCH_CHECK(bp == 0 || bp == 64 || bp == 128, "conv_gemm: pixel tile 64 or 128");
  TORCH_CHECK(bc == 0 || bc == 64 || bc == 128, "conv_gemm: channel tile 64 or 128");
  const int C = dgrad ? g.Cin : g.Cout;
  TORCH_CHECK(bc == 0 || C % bc == 0, "conv_gemm: channel tile must divide the channels");
  return conv_gemm_plan(g, dgrad, bp, bc, splits, parity, halo);
}

// bn (optional): (mean, invstd, gamma, beta) - x is the raw stem conv output and the window
// reads its BatchNorm + ReLU (no bn_apply pass)
static BnAffine bn_affine_of(const std::optional<std::vector<Tensor>>& bn, long C) {
  BnAffine a;
  if (!bn) return a;
  TORCH_CHECK(bn->size() == 4, "bn affine: (mean, invstd, gamma, beta)");
  for (const Tensor& t : *bn) { check(t, "bn affine", at::kFloat); TORCH_CHECK(t.numel() == C, "bn affine size"); }
  a.mean = (*bn)[0].data_ptr<float>();
  a.invstd = (*bn)[1].data_ptr<float>();
  a.gamma = (*bn)[2].data_ptr<float>();
  a.beta = (*bn)[3].data_ptr<float>();
  return a;
}

// (bp, bc, splits, stat_rows) of the plan; for dgrad X = dX-shaped layer input, Y = dY
py::tuple op_conv_gemm_plan(const Tensor& X, const Tensor& Y, int KH, int KW, int stride, int pad,
                            bool dgrad, int bp, int bc, int splits, int parity, int halo) {
  const ConvGeom g = geom_of(X, Y, KH, KW, stride, pad);
  const ConvPlan pl = plan_of(g, dgrad, bp, bc, splits, parity, halo);
  return py::make_tuple(pl.bp, pl.bc, pl.splits, dgrad ? 0 : conv_gemm_stat_rows(g, pl), pl.parity, pl.halo);
}

void op_conv_gemm_fwd(const Tensor& X, const Tensor& Wt, std::optional<Tensor> bias, Tensor& Y,
                      int KH, int KW, int stride, int pad, bool relu, std::optional<Tensor> stats,
                      std::optional<Tensor> part, int bp, int bc, int splits, int halo,
                      std::optional<std::vector<Tensor>> bn) {
  check(X, "X", at::kBFloat16); check(Wt, "Wt", at::kBFloat16); check(Y, "Y", at::kBFloat16);
  const ConvGeom g = geom_of(X, Y, KH, KW, stride, pad);
  TORCH_CHECK(g.Cin % 32 == 0 || (g.Cin == 4 && g.Cout % 64 == 0), "conv_gemm: Cin % 32 (or stem Cin=4)");
  TORCH_CHECK(g.Cout % 64 == 0, "conv_gemm: Cout % 64");
  TORCH_CHECK(Wt.numel() == (long)g.Cout * KH * KW * g.Cin, "conv_gemm: weight shape");
  const float* bp_ = nullptr;
  if (bias) { check(*bias, "bias", at::kFloat); TORCH_CHECK(bias->numel() == g.Cout, "bias"); bp_ = bias->data_ptr<float>(); }
  ConvPlan pl = plan_of(g, false, bp, bc, (bias || relu) ? 1 : splits, -1, (bias || relu) ? 0 : halo);
  float* st = nullptr;
  if (stats) {
    check(*stats, "stats", at::kFloat);
    TORCH_CHECK(stats->numel() >= (long)conv_gemm_stat_rows(g, pl) * 2 * g.Cout, "stats slab too small");
    st = stats->data_ptr<float>();
  }
  float* pt = nullptr;
  if (pl.splits > 1) {
    TORCH_CHECK(part.has_value(), "conv_gemm_fwd: split plan needs the fp32 `part` workspace");
    check(*part, "part", at::kFloat);
    TORCH_CHECK(part->numel() >= (long)pl.splits * g.N * g.OH * g.OW * g.Cout, "part workspace too small");
    pt = part->data_ptr<float>();
  }
  const BnAffine aff = bn_affine_of(bn, g.Cin);
  TORCH_CHECK(!aff.mean || (pl.halo && g.Cin <= 512), "conv_gemm_fwd: an input BatchNorm affine needs the halo plan");
  conv_gemm_fwd(g, pl, cbf(X), cbf(Wt), bp_, bf(Y), relu, st, pt, cur_stream(), &aff);
  kcheck();
}

void op_conv_gemm_dgrad(const Tensor& dY, const Tensor& W, std::optional<Tensor> Xact, Tensor& dX,
                        int KH, int KW, int stride, int pad, std::optional<Tensor> part, int bp, int bc,
                        int splits, int parity, int halo) {
  check(dY, "dY", at::kBFloat16); check(W, "W", at::kBFloat16); check(dX, "dX", at::kBFloat16);
  const ConvGeom g = geom_of(dX, dY, KH, KW, stride, pad);
  TORCH_CHECK(g.Cin % 64 == 0 && g.Cout % 32 == 0, "conv_gemm_dgrad: Cin % 64, Cout % 32");
  TORCH_CHECK(W.numel() == (long)g.Cout * KH * KW * g.Cin, "conv_gemm_dgrad: OHWI weight shape");
  if (Xact) TORCH_CHECK(Xact->sizes() == dX.sizes(), "Xact shape");
  const ConvPlan pl = plan_of(g, true, bp, bc, splits, parity, halo);
  float* pt = nullptr;
  if (pl.splits > 1) {
    TORCH_CHECK(part.has_value(), "conv_gemm_dgrad: split plan needs the fp32 `part` workspace");
    check(*part, "part", at::kFloat);
    TORCH_CHECK(part->numel() >= (long)pl.splits * g.N * g.H * g.W * g.Cin, "part workspace too small");
    pt = part->data_ptr<float>();
  }
  conv_gemm_dgrad(g, pl, cbf(dY), cbf(W), obf(Xact, "Xact"), bf(dX), pt, cur_stream());
  kcheck();
}

int op_conv_gemm_wgrad_chunks(const Tensor& X, const Tensor& dY, int KH, int KW, int stride, int pad,
                              int ppc) {
  return conv_gemm_wgrad_chunks(geom_of(X, dY, KH, KW, stride, pad), ppc);
}

void op_conv_gemm_wgrad(const Tensor& dY, const Tensor& X, Tensor& out, int KH, int KW, int stride,
                        int pad, int ppc, bool accum, int ks, std::optional<std::vector<Tensor>> bn) {
  check(dY, "dY", at::kBFloat16); check(X, "X", at::kBFloat16); check(out, "out", at::kFloat);
  const ConvGeom g = geom_of(X, dY, KH, KW, stride, pad);
  TORCH_CHECK((g.Cin % 64 == 0 || g.Cin == 4) && g.Cout % 64 == 0, "conv_gemm_wgrad: Cin % 64 (or 4), Cout % 64");
  TORCH_CHECK(conv_gemm_wgrad_ppc_ok(g, ppc), "pixels per chunk must be a multiple of 32 (or whole rows "
              "for the halo kernel)");
  const long row = (long)g.Cout * KH * KW * (g.Cin == 4 ? 3 : g.Cin);
  TORCH_CHECK(out.numel() >= (long)conv_gemm_wgrad_chunks(g, ppc) * row, "wgrad output too small");
  TORCH_CHECK(ks == 0 || ks == 32 || ks == 64, "conv_gemm_wgrad: ks 0 (auto), 32 or 64");
  const BnAffine aff = bn_affine_of(bn, g.Cin);
  TORCH_CHECK(!aff.mean || conv_gemm_wgrad_uses_halo(g, ppc),
              "conv_gemm_wgrad: an input BatchNorm affine needs the halo weight gradient");
  conv_gemm_wgrad(g, cbf(dY), cbf(X), out.data_ptr<float>(), ppc, accum, cur_stream(), ks, &aff);
  kcheck();
}

void op_bn_finalize(const Tensor& slab, int rows, int C, double count, double eps, double momentum,
                    std::optional<Tensor> rmean, std::optional<Tensor> rvar, Tensor& mean, Tensor& invstd,
                    std::optional<Tensor> nbt, Tensor& ws) {
  check(slab, "slab", at::kFloat); check(mean, "mean", at::kFloat); check(invstd, "invstd", at::kFloat);
  check(ws, "ws", at::kFloat);
  TORCH_CHECK(slab.numel() >= (long)rows * 2 * C && mean.numel() == C && invstd.numel() == C, "bn_finalize sizes");
  TORCH_CHECK(ws.numel() >= (long)bn_finalize_groups(rows) * 2 * C, "bn_finalize: ws too small");
  float *rm = nullptr, *rv = nullptr;
  if (rmean) { check(*rmean, "running_mean", at::kFloat); check(*rvar, "running_var", at::kFloat); rm = rmean->data_ptr<float>(); rv = rvar->data_ptr<float>(); }
  long long* nb = nullptr;
  if (nbt) { TORCH_CHECK(nbt->is_cuda() && nbt->scalar_type() == at::kLong && nbt->numel() == 1, "num_batches_tracked"); nb = reinterpret_cast<long long*>(nbt->data_ptr<int64_t>()); }
  bn_finalize(slab.data_ptr<float>(), rows, C, (float)count, (float)eps, (float)momentum, rm, rv,
              mean.data_ptr<float>(), invstd.data_ptr<float>(), nb, ws.data_ptr<float>(), cur_stream());
  kcheck();
}

void op_bn_apply(const Tensor& x, const Tensor& mean, const Tensor& invstd, const Tensor& gamma,
                 const Tensor& beta, std::optional<Tensor> res, bool relu, Tensor& y) {
  check(x, "x", at::kBFloat16); check(y, "y", at::kBFloat16);
  const int C = x.size(-1);
  TORCH_CHECK(C % 8 == 0 && 256 % (C / 8) == 0 && y.sizes() == x.sizes(),
              "bn_apply: C/8 must divide 256 (fixed channel group per thread), y shape");
  for (auto* t : {&mean, &invstd, &gamma, &beta}) { check(*t, "bn param", at::kFloat); TORCH_CHECK(t->numel() == C, "bn param size"); }
  if (res) TORCH_CHECK(res->sizes() == x.sizes(), "residual shape");
  bn_apply(cbf(x), x.numel() / C, C, mean.data_ptr<float>(), invstd.data_ptr<float>(),
           gamma.data_ptr<float>(), beta.data_ptr<float>(), obf(res, "res"), relu, bf(y), cur_stream());
  kcheck();
}

void op_bn_bwd(const Tensor& dout, std::optional<Tensor> out, const Tensor& x, const Tensor& mean,
               const Tensor& invstd, const Tensor& gamma, double count, Tensor& ws, Tensor& sums,
               std::optional<Tensor> dgamma, std::optional<Tensor> dbeta, bool accum, Tensor& dx,
               std::optional<Tensor> dres, std::optional<Tensor> dout2, std::optional<Tensor> mask_beta) {
  check(dout, "dout", at::kBFloat16); check(x, "x", at::kBFloat16); check(dx, "dx", at::kBFloat16);
  check(sums, "sums", at::kFloat); check(ws, "ws", at::kFloat);
  const int C = x.size(-1);
  const long P = x.numel() / C;
  TORCH_CHECK(C % 64 == 0 && 256 % (C / 8) == 0 && dout.sizes() == x.sizes() && dx.sizes() == x.sizes(),
              "bn_bwd: C % 64 with C/8 dividing 256, shapes");
  TORCH_CHECK(P < (1L << 31), "bn_bwd: too many pixels");
  TORCH_CHECK(sums.numel() == 2 * C, "bn_bwd: sums [2C]");
  TORCH_CHECK(ws.numel() >= (long)bn_bwd_rows(P, C, nullptr) * 2 * C, "bn_bwd: ws too small");
  for (auto* t : {&mean, &invstd, &gamma}) { check(*t, "bn param", at::kFloat); TORCH_CHECK(t->numel() == C, "bn param size"); }
  if (out) TORCH_CHECK(out->sizes() == x.sizes(), "out shape");
  float *dg = nullptr, *db = nullptr;
  if (dgamma) { check(*dgamma, "dgamma", at::kFloat); TORCH_CHECK(dgamma->numel() == C, "dgamma"); dg = dgamma->data_ptr<float>(); }
  if (dbeta) { check(*dbeta, "dbeta", at::kFloat); TORCH_CHECK(dbeta->numel() == C, "dbeta"); db = dbeta->data_ptr<float>(); }
  bf16_t* dr = nullptr;
  if (dres) { check(*dres, "dres", at::kBFloat16); TORCH_CHECK(dres->sizes() == x.sizes(), "dres"); dr = bf(*dres); }
  if (dout2) TORCH_CHECK(dout2->sizes() == x.sizes(), "dout2 shape");
  const float* mb = nullptr;
  if (mask_beta) {
    TORCH_CHECK(!out, "bn_bwd: give the saved output OR mask_beta (recomputed ReLU mask), not both");
    check(*mask_beta, "mask_beta", at::kFloat);
    TORCH_CHECK(mask_beta->numel() == C, "mask_beta size");
    mb = mask_beta->data_ptr<float>();
  }
  bn_bwd(cbf(dout), obf(out, "out"), cbf(x), P, C, mean.data_ptr<float>(), invstd.data_ptr<float>(),
         gamma.data_ptr<float>(), (float)count, ws.data_ptr<float>(), sums.data_ptr<float>(), dg, db,
         accum, bf(dx), dr, cur_stream(), obf(dout2, "dout2"), mb);
  kcheck();
}

void op_maxpool_fwd(const Tensor& x, Tensor& y, Tensor& amax, std::optional<std::vector<Tensor>> bn) {
  check(x, "x", at::kBFloat16); check(y, "y", at::kBFloat16); check(amax, "amax", at::kByte);
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3), OH = y.size(1), OW = y.size(2);
  TORCH_CHECK(OH == (H - 1) / 2 + 1 && OW == (W - 1) / 2 + 1 && y.size(3) == C, "maxpool 3x3/s2/p1 shape");
  TORCH_CHECK(amax.numel() == y.numel(), "amax size");
  TORCH_CHECK(C % 8 == 0 && x.numel() / 8 < (1L << 31), "maxpool: C % 8 (8 channels per thread)");
  const BnAffine aff = bn_affine_of(bn, C);
  maxpool_fwd(cbf(x), N, H, W, C, OH, OW, bf(y), amax.data_ptr<unsigned char>(), cur_stream(), &aff);
  kcheck();
}

void op_maxpool_bwd(const Tensor& dy, const Tensor& amax, Tensor& dx, std::optional<Tensor> dy2) {
  check(dy, "dy", at::kBFloat16); check(dx, "dx", at::kBFloat16); check(amax, "amax", at::kByte);
  const int N = dx.size(0), H = dx.size(1), W = dx.size(2), C = dx.size(3), OH = dy.size(1), OW = dy.size(2);
  TORCH_CHECK(OH == (H - 1) / 2 + 1 && OW == (W - 1) / 2 + 1 && amax.numel() == dy.numel(), "maxpool bwd shape");
  TORCH_CHECK(C % 8 == 0 && dy.size(3) == C && dx.numel() / 8 < (1L << 31), "maxpool bwd: C % 8");
  if (dy2) TORCH_CHECK(dy2->sizes() == dy.sizes(), "dy2 shape");
  maxpool_bwd(cbf(dy), amax.data_ptr<unsigned char>(), N, H, W, C, OH, OW, bf(dx), cur_stream(),
              obf(dy2, "dy2"));
  kcheck();
}

void op_image_gather_nhwc4(const Tensor& imgs, const Tensor& idx, Tensor& out) {
  TORCH_CHECK(imgs.is_cuda() && imgs.scalar_type() == at::kByte && imgs.is_contiguous() && imgs.dim() == 4 &&
              imgs.size(3) == 3, "images: contiguous uint8 [N,H,W,3] on the GPU");
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == at::kLong && idx.is_contiguous() && idx.dim() == 1, "idx: int64 [B]");
  check(out, "out", at::kBFloat16);
  TORCH_CHECK(out.dim() == 4 && out.size(0) == idx.size(0) && out.size(1) == imgs.size(1) &&
              out.size(2) == imgs.size(2) && out.size(3) == 4, "out: bf16 [B,H,W,4]");
  if (idx.numel() == 0) return;
  image_gather_nhwc4(imgs.data_ptr<unsigned char>(), reinterpret_cast<const long long*>(idx.data_ptr<int64_t>()),
                     (int)idx.size(0), (int)(imgs.size(1) * imgs.size(2)), imgs.size(0), bf(out), cur_stream());
  kcheck();
}

void op_avgpool_fwd(const Tensor& x, Tensor& y) {
  check(x, "x", at::kBFloat16); check(y, "y", at::kFloat);
  const int N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  TORCH_CHECK(y.numel() == (long)N * C, "avgpool out size");
  TORCH_CHECK(C % 64 == 0 && N < 65536, "avgpool: C % 64 (one block per 64 channels)");
  avgpool_fwd(cbf(x), N, HW, C, y.data_ptr<float>(), cur_stream());
  kcheck();
}

void op_avgpool_bwd(const Tensor& dy, Tensor& dx) {
  check(dy, "dy", at::kFloat); check(dx, "dx", at::kBFloat16);
  const int N = dx.size(0), HW = dx.size(1) * dx.size(2), C = dx.size(3);
  TORCH_CHECK(dy.numel() == (long)N * C, "avgpool dy size");
  avgpool_bwd(dy.data_ptr<float>(), N, HW, C, bf(dx), cur_stream());
  kcheck();
}

// C[M][N] = alpha * A(m,k) B(k,n) + bias; strides in elements (A/B: fp32 or bf16)
void op_sgemm(int M, int N, int K, const Tensor& A, long sam, long sak, const Tensor& B, long sbk,
              long sbn, Tensor& Cm, std::optional<Tensor> bias, double alpha, bool accum) {
  check_cuda(A, "A"); check_cuda(B, "B"); check(Cm, "C", at::kFloat);
  const bool abf = A.scalar_type() == at::kBFloat16, bbf = B.scalar_type() == at::kBFloat16;
  TORCH_CHECK(abf || A.scalar_type() == at::kFloat, "A dtype");
  TORCH_CHECK(bbf || B.scalar_type() == at::kFloat, "B dtype");
  TORCH_CHECK((long)(M - 1) * sam + (long)(K - 1) * sak < A.numel(), "A bounds");
  TORCH_CHECK((long)(K - 1) * sbk + (long)(N - 1) * sbn < B.numel(), "B bounds");
  TORCH_CHECK(Cm.numel() >= (long)M * N, "C size");
  const float* bp = nullptr;
  if (bias) { check(*bias, "bias", at::kFloat); TORCH_CHECK(bias->numel() == N, "bias"); bp = bias->data_ptr<float>(); }
  sgemm(M, N, K, A.data_ptr(), abf, sam, sak, B.data_ptr(), bbf, sbk, sbn, Cm.data_ptr<float>(), N,
        bp, (float)alpha, cur_stream(), accum);
  kcheck();
}

void op_transpose_w(const Tensor& w, Tensor& wt) {
  check(w, "w", at::kFloat); check(wt, "wt", at::kBFloat16);
  TORCH_CHECK(w.dim() == 4 && wt.numel() == w.numel(), "transpose_w: OHWI weight expected");
  transpose_w(w.data_ptr<float>(), w.size(0), w.size(1) * w.size(2), w.size(3), bf(wt), cur_stream());
  kcheck();
}

ShadowSet make_shadows(const py::list& shadows) {
  ShadowSet sh{};
  TORCH_CHECK((int)shadows.size() <= MAX_SHADOWS, "too many shadow regions");
  for (auto item : shadows) {
    auto t = item.cast<py::tuple>();  // (off, n, dst bf16 tensor, kind, a, b, c)
    Tensor dst = t[2].cast<Tensor>();
    check(dst, "shadow dst", at::kBFloat16);
    const long n = t[1].cast<long>();
    const int kind = t[3].cast<int>(), a = t[4].cast<int>(), b = t[5].cast<int>(), c = t[6].cast<int>();
    TORCH_CHECK(kind >= SHADOW_BF16 && kind <= SHADOW_BF16_PAD4, "unknown shadow kind");
    if (kind == SHADOW_BF16_PAD4) {
      TORCH_CHECK(n % 3 == 0 && dst.numel() == n / 3 * 4, "PAD4 shadow: dst must hold n/3 x 4");
    } else {
      TORCH_CHECK(dst.numel() == n, "shadow dst size mismatch");
    }
    if (kind == SHADOW_BF16_TAPT) TORCH_CHECK((long)a * b * c == n, "TAPT shadow: Co*T*Ci != n");
    if (kind == SHADOW_BF16_FCFRAG)
      TORCH_CHECK(a % 16 == 0 && b % 16 == 0 && n % ((long)a * b) == 0 && n < (1L << 31),
                  "FCFRAG shadow: HW and C must be multiples of 16, n a multiple of HW*C");
    sh.r[sh.count++] = ShadowRegion{t[0].cast<long>(), n, bf(dst), kind, a, b, c};
  }
  return sh;
}

void op_sgd(Tensor& p, const Tensor& g, std::optional<Tensor> mbuf, double lr, double momentum,
            double dampening, double wd, bool nesterov, bool maximize, bool first_step, bool update,
            const py::list& shadows) {
  check(p, "params", at::kFloat); check(g, "grads", at::kFloat);
  TORCH_CHECK(p.numel() == g.numel(), "sgd: param/grad size mismatch");
  TORCH_CHECK(((uintptr_t)p.data_ptr() & 15) == 0 && ((uintptr_t)g.data_ptr() & 15) == 0,
              "sgd: params/grads must be 16-byte aligned");
  float* mb = nullptr;
  if (momentum != 0.0) {
    TORCH_CHECK(mbuf.has_value(), "sgd: momentum buffer required");
    check(*mbuf, "momentum", at::kFloat);
    TORCH_CHECK(mbuf->numel() == p.numel(), "sgd: momentum size");
    mb = mbuf->data_ptr<float>();
    TORCH_CHECK(((uintptr_t)mb & 15) == 0, "sgd: momentum buffer must be 16-byte aligned");
  }
  SgdArgs a{(float)lr, (float)momentum, (float)dampening, (float)wd, nesterov, maximize,
            first_step, update};
  const ShadowSet sh = make_shadows(shadows);
  for (int r = 0; r < sh.count; ++r)
    TORCH_CHECK(sh.r[r].off >= 0 && sh.r[r].off + sh.r[r].n <= p.numel(), "shadow out of range");
  sgd_step(p.data_ptr<float>(), g.data_ptr<float>(), mb, p.numel(), a, sh, nullptr, cur_stream());
  kcheck();
}

void op_grad_reduce(const py::list& segs) {
  SlabSet ss{};
  TORCH_CHECK(segs.size() <= 4, "at most 4 slab segments");
  for (auto item : segs) {
    auto t = item.cast<py::tuple>();  // (slab, row_stride, src_off, n, rows, dst, scale[, accum])
    Tensor slab = t[0].cast<Tensor>(), dst = t[5].cast<Tensor>();
    check(slab, "slab", at::kFloat);
    TORCH_CHECK(dst.is_cuda() && dst.scalar_type() == at::kFloat && dst.is_contiguous(), "dst");
    const long rs = t[1].cast<long>(), so = t[2].cast<long>(), n = t[3].cast<long>();
    const int rows = t[4].cast<int>();
    TORCH_CHECK(dst.numel() == n, "grad_reduce: dst size");
    TORCH_CHECK(rows >= 1 && so + n <= rs && (long)(rows - 1) * rs + so + n <= slab.numel(),
                "grad_reduce: slab bounds");
    ss.s[ss.count] = SlabSeg{slab.data_ptr<float>(), rs, so, n, rows, dst.data_ptr<float>(),
                             (float)t[6].cast<double>()};
    if (t.size() > 7) ss.s[ss.count].accum = t[7].cast<bool>() ? 1 : 0;
    ++ss.count;
  }
  grad_reduce(ss, cur_stream());
  kcheck();
}

void op_scale_copy(Tensor& dst, const Tensor& src, double scale) {
  check(dst, "dst", at::kFloat); check(src, "src", at::kFloat);
  TORCH_CHECK(dst.numel() == src.numel(), "scale_copy: size");
  scale_copy(dst.data_ptr<float>(), src.data_ptr<float>(), dst.numel(), (float)scale, cur_stream());
  kcheck();
}

int dtype_code(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return 0;
    case at::kBFloat16: return 1;
    case at::kInt: return 2;
    case at::kLong: return 3;
    case at::kByte: return 4;
    default: TORCH_CHECK(false, "unsupported dtype for RCCL: ", t.scalar_type());
  }
  return -1;
}

hipStream_t stream_or_current(uint64_t s) {
  return s ? reinterpret_cast<hipStream_t>(s) : cur_stream();
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "ddp_amd native gfx950 kernels + RCCL runtime";
  m.def("conv1_fwd", &op_conv1_fwd);
  m.def("conv1_wgrad", &op_conv1_wgrad);
  m.def("conv1_wgrad_blocks", &conv1_wgrad_blocks);
  m.def("plan_buckets", &plan_buckets, "torch DDP bucket size rule over gradient-ready byte sizes",
        py::arg("nbytes"), py::arg("first_cap_bytes"), py::arg("cap_bytes"));
  py::class_<BucketState>(m, "BucketState")
      .def(py::init<std::vector<int>, int>())
      .def("mark_ready", &BucketState::mark_ready)
      .def("set_launched", &BucketState::set_launched)
      .def("unlaunched", &BucketState::unlaunched)
      .def("pending", &BucketState::pending)
      .def("reset", &BucketState::reset);
  m.def("noop", [](int blocks) { noop(blocks, nullptr, cur_stream()); kcheck(); });
  m.def("stamps_set", [](std::optional<Tensor> buf) {
    if (buf) TORCH_CHECK(buf->is_cuda() && buf->numel() * buf->element_size() >=
                             (int64_t)STAMP_K_COUNT * STAMP_KSTRIDE * 8, "stamp buffer too small");
    stamps_set(buf ? buf->data_ptr() : nullptr);
  });
  m.attr("STAMP_KSTRIDE") = STAMP_KSTRIDE;
  m.attr("STAMP_K_COUNT") = (int)STAMP_K_COUNT;
  m.def("conv3x3_fwd", &op_conv3x3_fwd);
  m.def("conv3x3_dgrad", &op_conv3x3_dgrad);
  m.def("conv3x3_dgrad_fused_w1", &op_conv3x3_dgrad_fused_w1);
  m.def("conv3x3_dgrad_blocks", &conv3x3_dgrad_blocks);
  m.def("conv3x3_wgrad", &op_conv3x3_wgrad);
  m.def("conv3x3_wgrad_blocks", &conv3x3_wgrad_blocks);
  m.def("fc_partial", &op_fc_partial);
  m.def("fc_reduce", &op_fc_reduce);
  m.def("fc_bwd", &op_fc_bwd, py::arg("dL"), py::arg("X"), py::arg("Wf"), py::arg("dX"), py::arg("dW"),
        py::arg("scale"), py::arg("mask"), py::arg("dbias") = py::none(),
        py::arg("loss_rows") = py::none(), py::arg("loss_out") = py::none());
  m.def("xent_rows", &op_xent_rows);
  m.def("xent", &op_xent);
  m.def("sgd", &op_sgd);
  m.def("grad_reduce", &op_grad_reduce);
  m.def("scale_copy", &op_scale_copy);
  m.def("_mark_exiting", &ddp_amd::mark_exiting);
  m.def("conv_gemm_fwd", &op_conv_gemm_fwd, py::arg("X"), py::arg("W"), py::arg("bias"), py::arg("Y"),
        py::arg("KH"), py::arg("KW"), py::arg("stride"), py::arg("pad"), py::arg("relu") = false,
        py::arg("stats") = py::none(), py::arg("part") = py::none(), py::arg("bp") = 0, py::arg("bc") = 0,
        py::arg("splits") = 0, py::arg("halo") = -1, py::arg("bn") = py::none());
  m.def("conv_gemm_dgrad", &op_conv_gemm_dgrad, py::arg("dY"), py::arg("W"), py::arg("Xact"), py::arg("dX"),
        py::arg("KH"), py::arg("KW"), py::arg("stride"), py::arg("pad"), py::arg("part") = py::none(),
        py::arg("bp") = 0, py::arg("bc") = 0, py::arg("splits") = 0, py::arg("parity") = -1,
        py::arg("halo") = -1);
  m.def("conv_gemm_wgrad_chunks", &op_conv_gemm_wgrad_chunks);
  m.def("conv_gemm_wgrad_set_halo", &conv_gemm_wgrad_set_halo, py::arg("halo"), py::arg("target") = 256,
        py::arg("cit") = 0,
        "weight-gradient plan override: halo 0 = the per-tap GEMM kernel only, 1 (default) / 2 = "
        "tap-fused halo kernel for every eligible stride-1 3x3 layer; target = blocks per launch; cit = "
        "input channels per halo block (0 auto, 16, 32)");
  m.def("conv_gemm_wgrad_force_tile", &conv_gemm_wgrad_force_tile);
  m.def("conv_gemm_wgrad_tiles", [](const Tensor& X, const Tensor& dY, int KH, int KW, int st, int pd) {
    return conv_gemm_wgrad_tiles(geom_of(X, dY, KH, KW, st, pd));
  });
  m.def("conv_gemm_wgrad_ppc", [](const Tensor& X, const Tensor& dY, int KH, int KW, int st, int pd) {
    return conv_gemm_wgrad_ppc(geom_of(X, dY, KH, KW, st, pd));
  });
  m.def("conv_gemm_wgrad", &op_conv_gemm_wgrad, py::arg("dY"), py::arg("X"), py::arg("out"), py::arg("KH"),
        py::arg("KW"), py::arg("stride"), py::arg("pad"), py::arg("ppc"), py::arg("accum") = false,
        py::arg("ks") = 0, py::arg("bn") = py::none());
  m.def("conv_gemm_wgrad_uses_halo", [](const Tensor& X, const Tensor& dY, int KH, int KW, int stride, int pad,
                                        int ppc) { return conv_gemm_wgrad_uses_halo(geom_of(X, dY, KH, KW, stride, pad), ppc); });
  m.def("conv_gemm_plan", &op_conv_gemm_plan, py::arg("X"), py::arg("Y"), py::arg("KH"), py::arg("KW"),
        py::arg("stride"), py::arg("pad"), py::arg("dgrad") = false, py::arg("bp") = 0, py::arg("bc") = 0,
        py::arg("splits") = 0, py::arg("parity") = -1, py::arg("halo") = -1);
  m.def("bn_finalize", &op_bn_finalize);
  // host-side wait policy of the device (before torch creates its context): 1 =
  // hipDeviceScheduleSpin - synchronize() polls the completion signal instead of sleeping
  m.def("hip_set_device_flags", [](int dev, unsigned flags) {
    hipError_t e = hipSetDevice(dev);
    if (e == hipSuccess) e = hipSetDeviceFlags(flags);
    return (int)e;
  });
  m.def("bn_apply", &op_bn_apply);
  m.def("bn_finalize_groups", &bn_finalize_groups);
  m.def("bn_bwd_rows", [](long P, int C) { return bn_bwd_rows(P, C, nullptr); });
  m.def("bn_bwd", &op_bn_bwd, py::arg("dout"), py::arg("out"), py::arg("x"), py::arg("mean"),
        py::arg("invstd"), py::arg("gamma"), py::arg("count"), py::arg("ws"), py::arg("sums"),
        py::arg("dgamma"), py::arg("dbeta"), py::arg("accum"), py::arg("dx"), py::arg("dres"),
        py::arg("dout2") = py::none(), py::arg("mask_beta") = py::none());
  m.def("bn_bwd_set_px_per_block", &bn_bwd_set_px_per_block);
  m.def("maxpool_fwd", &op_maxpool_fwd, py::arg("x"), py::arg("y"), py::arg("amax"), py::arg("bn") = py::none());
  m.def("maxpool_bwd", &op_maxpool_bwd, py::arg("dy"), py::arg("amax"), py::arg("dx"),
        py::arg("dy2") = py::none());
  m.def("avgpool_fwd", &op_avgpool_fwd);
  m.def("image_gather_nhwc4", &op_image_gather_nhwc4);
  m.def("avgpool_bwd", &op_avgpool_bwd);
  m.def("sgemm", &op_sgemm, py::arg("M"), py::arg("N"), py::arg("K"), py::arg("A"), py::arg("sam"),
        py::arg("sak"), py::arg("B"), py::arg("sbk"), py::arg("sbn"), py::arg("C"), py::arg("bias"),
        py::arg("alpha"), py::arg("accum") = false);
  m.def("transpose_w", &op_transpose_w);
  m.def("rccl_version", []() { int v = 0; ncclGetVersion(&v); return v; });
  // PCI bus id of a device: ranks compare these through the store to detect a shared GPU
  // (device counts cannot: HIP_VISIBLE_DEVICES-isolated ranks each see one device)
  m.def("pci_bus_id", [](int dev) {
    char buf[64] = {0};
    if (hipDeviceGetPCIBusId(buf, sizeof(buf) - 1, dev) != hipSuccess)
      throw std::runtime_error("hipDeviceGetPCIBusId failed");
    return std::string(buf);
  });

  py::class_<Comm, std::shared_ptr<Comm>>(m, "Comm")
      .def_static("new_unique_id", []() { return py::bytes(Comm::new_unique_id()); })
      .def(py::init([](py::bytes uid, int rank, int world, int device) {
             return std::make_shared<Comm>(std::string(uid), rank, world, device);
           }))
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("world", &Comm::world)
      .def("all_reduce", [](Comm& c, Tensor& t, int op, uint64_t stream) {
             check_cuda(t, "tensor");
             c.all_reduce(t.data_ptr(), t.numel(), dtype_code(t), op, stream_or_current(stream));
           }, py::arg("tensor"), py::arg("op") = 0, py::arg("stream") = 0)
      .def("all_reduce_premul", [](Comm& c, Tensor& t, double scale, uint64_t stream) {
             check_cuda(t, "tensor");
             TORCH_CHECK(t.scalar_type() == at::kFloat && t.is_contiguous(), "all_reduce_premul: contiguous fp32");
             c.all_reduce_premul(t.data_ptr<float>(), t.numel(), (float)scale, stream_or_current(stream));
           }, py::arg("tensor"), py::arg("scale"), py::arg("stream") = 0)
      .def("broadcast", [](Comm& c, Tensor& t, int root, uint64_t stream) {
             check_cuda(t, "tensor");
             c.broadcast(t.data_ptr(), t.numel(), dtype_code(t), root, stream_or_current(stream));
           }, py::arg("tensor"), py::arg("root") = 0, py::arg("stream") = 0)
      .def("all_gather", [](Comm& c, const Tensor& send, Tensor& recv, uint64_t stream) {
             check_cuda(send, "send"); check_cuda(recv, "recv");
             TORCH_CHECK(recv.numel() == send.numel() * c.world(), "all_gather: recv size");
             c.all_gather(send.data_ptr(), recv.data_ptr(), send.numel(), dtype_code(send),
                          stream_or_current(stream));
           }, py::arg("send"), py::arg("recv"), py::arg("stream") = 0)
      .def("reduce_scatter", [](Comm& c, const Tensor& send, Tensor& recv, int op, uint64_t stream) {
             check_cuda(send, "send"); check_cuda(recv, "recv");
             TORCH_CHECK(send.numel() == recv.numel() * c.world(), "reduce_scatter: send size");
             c.reduce_scatter(send.data_ptr(), recv.data_ptr(), recv.numel(), dtype_code(recv), op,
                              stream_or_current(stream));
           }, py::arg("send"), py::arg("recv"), py::arg("op") = 0, py::arg("stream") = 0);

  py::class_<XgmiComm, std::shared_ptr<XgmiComm>>(m, "XgmiComm")
      .def(py::init<int, int, int>(), py::arg("rank"), py::arg("world"), py::arg("device"))
      .def("add_channel", &XgmiComm::add_channel, py::arg("off"), py::arg("n"), py::arg("oneshot") = false,
           py::arg("grid_cap") = 0)
      .def("blocks", &XgmiComm::blocks)
      .def("bus_id", &XgmiComm::bus_id)
      .def("oneshot", &XgmiComm::oneshot)
      .def_property_readonly("channels", &XgmiComm::channels)
      .def("set_data", [](XgmiComm& x, Tensor& t) {
        check(t, "data", at::kFloat);
        x.set_data(t.data_ptr<float>(), t.numel());
      })
      .def("export_handles", [](const XgmiComm& x) { return py::bytes(x.export_handles()); })
      .def("import_handles", [](XgmiComm& x, const std::vector<py::bytes>& all) {
        std::vector<std::string> v;
        for (const auto& b : all) v.emplace_back(b);
        x.import_handles(v);
      })
      .def("all_reduce", [](XgmiComm& x, int ch, double scale, bool publish, double prescale) {
        x.all_reduce(ch, cur_stream(), (float)scale, publish, (float)prescale);
      }, py::arg("channel"), py::arg("scale") = 1.0, py::arg("publish") = false, py::arg("prescale") = 1.0)
      .def("error_flags", &XgmiComm::error_flags)
      .def("set_timeout", &XgmiComm::set_timeout)
      .def_property_readonly("rank", &XgmiComm::rank)
      .def_property_readonly("world", &XgmiComm::world);
  py::class_<Reducer, std::shared_ptr<Reducer>>(m, "Reducer")
      .def(py::init([](std::shared_ptr<Comm> comm, Tensor& flat, std::vector<long> poff,
                       std::vector<long> pnum, std::vector<int> pb, std::vector<long> boff,
                       std::vector<long> bnum, bool prescale) {
             check(flat, "flat_grad", at::kFloat);
             for (size_t i = 0; i < poff.size(); ++i)
               TORCH_CHECK(poff[i] >= 0 && poff[i] + pnum[i] <= flat.numel(), "param slot OOB");
             for (size_t i = 0; i < boff.size(); ++i)
               TORCH_CHECK(boff[i] >= 0 && boff[i] + bnum[i] <= flat.numel(), "bucket OOB");
             return std::make_shared<Reducer>(comm, flat.data_ptr<float>(), poff, pnum, pb, boff,
                                              bnum, prescale);
           }))
      .def("mark_ready", [](Reducer& r, int param, std::optional<Tensor> grad) {
             const float* src = nullptr;
             if (grad) { check(*grad, "grad", at::kFloat); src = grad->data_ptr<float>(); }
             r.mark_ready(param, src, cur_stream());
           })
      .def("finalize", [](Reducer& r) { r.finalize(cur_stream()); })
      .def("set_xgmi", &Reducer::set_xgmi, py::arg("xgmi"), py::arg("channels"))
      .def_property_readonly("world", &Reducer::world)
      .def("reset", &Reducer::reset)
      .def_property_readonly("num_buckets", &Reducer::num_buckets)
      .def_property_readonly("allreduce_calls", &Reducer::allreduce_calls);

  py::class_<SimpleCNNEngine, std::shared_ptr<SimpleCNNEngine>>(m, "SimpleCNNEngine")
      .def(py::init([](py::dict cfgd, py::dict t, py::dict offs, std::shared_ptr<Comm> comm) {
             EngineConfig c{};
             c.max_batch = cfgd["max_batch"].cast<int>();
             c.H = cfgd["H"].cast<int>(); c.W = cfgd["W"].cast<int>();
             c.C1 = cfgd["C1"].cast<int>(); c.C2 = cfgd["C2"].cast<int>(); c.NO = cfgd["NO"].cast<int>();
             c.pxt_fwd = cfgd["pxt_fwd"].cast<int>(); c.pxt_dgrad = cfgd["pxt_dgrad"].cast<int>();
             c.wgrad_rows = cfgd["wgrad_rows"].cast<int>();
             c.world = cfgd["world"].cast<int>(); c.rank = cfgd["rank"].cast<int>();
             c.lr = cfgd["lr"].cast<float>(); c.momentum = cfgd["momentum"].cast<float>();
             c.dampening = cfgd["dampening"].cast<float>();
             c.weight_decay = cfgd["weight_decay"].cast<float>();
             c.nesterov = cfgd["nesterov"].cast<bool>(); c.maximize = cfgd["maximize"].cast<bool>();
             c.force_allreduce = cfgd.contains("force_allreduce") ? cfgd["force_allreduce"].cast<bool>() : false;
             c.fuse_level = cfgd.contains("fuse_level") ? cfgd["fuse_level"].cast<int>() : 0;
             c.fuse_opt = cfgd.contains("fuse_opt") ? (int)cfgd["fuse_opt"].cast<bool>() : 1;
             c.store_a1 = cfgd.contains("store_a1") ? cfgd["store_a1"].cast<int>() : 0;
             c.f32 = cfgd.contains("f32") ? (int)cfgd["f32"].cast<bool>() : 0;
             c.fuse_reduce = cfgd.contains("fuse_reduce") ? cfgd["fuse_reduce"].cast<int>() : 1;
             c.wgrad_split = cfgd.contains("wgrad_split") ? cfgd["wgrad_split"].cast<int>() : 1;
             c.l3_fc_role = cfgd.contains("l3_fc_role") ? cfgd["l3_fc_role"].cast<int>() : 1;
             c.dist_mode = cfgd.contains("dist_mode") ? cfgd["dist_mode"].cast<int>() : 3;
             TORCH_CHECK(c.dist_mode >= 0 && c.dist_mode <= 3, "engine: dist_mode must be 0..3");
             TORCH_CHECK(c.l3_fc_role == 0 || c.l3_fc_role == 1, "engine: l3_fc_role must be 0 or 1");
             TORCH_CHECK(c.wgrad_split == 1 || c.wgrad_split == 2, "engine: wgrad_split must be 1 or 2");
             const int es = c.f32 ? 4 : 2;
             TORCH_CHECK(c.store_a1 >= 0 && c.store_a1 <= 2, "engine: store_a1 must be 0, 1 or 2");
             TORCH_CHECK(c.fuse_level == 0 || c.fuse_level == 1 || c.fuse_level == 3,
                         "engine: fuse_level must be 0, 1 or 3 (level 2 was removed in round 4)");
             TORCH_CHECK(conv3x3_fwd_lds(c.W, c.C1, c.pxt_fwd, c.fuse_level > 0, es) <= 160 * 1024 &&
                             conv3x3_wgrad_lds(c.W, c.C1, c.C2, c.wgrad_rows, c.fuse_level > 0, es) <= 160 * 1024 &&
                             conv3x3_dgrad_lds(c.W, c.C2, c.pxt_dgrad, true, es) <= 160 * 1024,
                         "engine: LDS budget exceeded for this tiling");
             auto T = [&](const char* k) { return t[k].cast<Tensor>(); };
             auto need = [&](const char* k, at::ScalarType st, long n) {
               Tensor x = T(k);
               check(x, k, st);
               TORCH_CHECK(x.numel() >= n, "engine buffer ", k, " too small: ", x.numel(), " < ", n);
               return x;
             };
             const long B = c.max_batch, HW = (long)c.H * c.W;
             EngineBuffers b{};
             Tensor params = need("params", at::kFloat, 1);
             b.params = params.data_ptr<float>();
             b.n_params = params.numel();
             b.grads = need("grads", at::kFloat, b.n_params).data_ptr<float>();
             b.momentum = (c.momentum != 0.f) ? need("momentum", at::kFloat, b.n_params).data_ptr<float>() : nullptr;
             auto O = [&](const char* k) { return offs[k].cast<long>(); };
             b.off_w1 = O("w1"); b.off_b1 = O("b1"); b.off_w2 = O("w2"); b.off_b2 = O("b2");
             b.off_wfc = O("wfc"); b.off_bfc = O("bfc");
             std::vector<EngineBucket> buckets;
             for (auto item : offs["buckets"].cast<py::list>()) {
               auto pr = item.cast<std::pair<long, long>>();
               buckets.push_back(EngineBucket{pr.first, pr.second});
             }
             TORCH_CHECK(b.off_wfc + (long)c.NO * HW * c.C2 <= b.n_params && b.off_w1 + 9L * c.C1 <= b.n_params &&
                         b.off_b2 + c.C2 <= b.n_params && b.off_w2 + 9L * c.C1 * c.C2 <= b.n_params,
                         "engine: parameter offsets out of range");
             TORCH_CHECK(fc_bwd_lds(c.max_batch, c.NO, true, ((long)c.max_batch * HW + 64L * c.pxt_fwd - 1) / (64L * c.pxt_fwd) * 2 * c.NO) <= 160 * 1024,
                         "engine: batch too large for fc_bwd LDS");
             if (c.f32) {  // exact fp32: fp32 activations + the conv2 weight's fp32 [tap][ci][co] copy
               TORCH_CHECK(c.fuse_level >= 1 && c.store_a1 == 0, "engine: fp32 needs fuse_level 1 or 3 and store_a1 0");
               b.a2_f32 = need("a2", at::kFloat, B * HW * c.C2).data_ptr<float>();
               b.dz2_f32 = need("dz2", at::kFloat, B * HW * c.C2).data_ptr<float>();
               b.w2t_f32 = need("w2t_f32", at::kFloat, 9L * c.C1 * c.C2).data_ptr<float>();
               b.wfc_frag32 = need("wfc_frag32", at::kFloat, (long)c.NO * HW * c.C2).data_ptr<float>();
             } else {
               b.w2_bf16 = bf(need("w2_bf16", at::kBFloat16, 9L * c.C1 * c.C2));
               b.w2t_bf16 = bf(need("w2t_bf16", at::kBFloat16, 9L * c.C1 * c.C2));
               b.wfc_bf16 = bf(need("wfc_bf16", at::kBFloat16, (long)c.NO * HW * c.C2));
               b.wfc_frag = bf(need("wfc_frag", at::kBFloat16, (long)c.NO * HW * c.C2));
               b.a1 = bf(need("a1", at::kBFloat16, B * HW * c.C1));
               b.a2 = bf(need("a2", at::kBFloat16, B * HW * c.C2));
               b.dz2 = bf(need("dz2", at::kBFloat16, B * HW * c.C2));
               b.dz1 = bf(need("dz1", at::kBFloat16, B * HW * c.C1));
             }
             b.fc_part = need("fc_part", at::kFloat, 2L * conv3x3_dgrad_blocks(B, c.H, c.W, c.pxt_fwd) * c.NO).data_ptr<float>();
             b.dlogits = need("dlogits", at::kFloat, B * c.NO).data_ptr<float>();
             b.loss_rows = need("loss_rows", at::kFloat, B).data_ptr<float>();
             b.loss_hist = need("loss_hist", at::kFloat, 1).data_ptr<float>();
             b.w2slab = need("w2slab", at::kFloat, (long)conv3x3_wgrad_blocks(B, c.H, c.wgrad_rows) * (9L * c.C1 * c.C2 + c.C2)).data_ptr<float>();
             b.w1slab = need("w1slab", at::kFloat, (long)conv3x3_dgrad_blocks(B, c.H, c.W, c.pxt_dgrad) * 320).data_ptr<float>();
             b.step_ctr = need("step_ctr", at::kInt, 1).data_ptr<int>();
             b.xb = need("xb", at::kByte, B * HW).data_ptr<unsigned char>();
             b.yb = need("yb", at::kInt, B).data_ptr<int>();
             if (t.contains("sync_flags")) {  // in-launch hand-offs (fused reduction, level 2)
               long nfl = SYNC_RED_INTS;
               // level 3: the forward's per-image arrival counters, FWD_DZ_CNT_STRIDE ints apart
               if (c.fuse_level >= 3) nfl = std::max(nfl, (long)L3_IMG_OFF + (long)FWD_DZ_CNT_STRIDE * B);
               b.sync_flags = need("sync_flags", at::kInt, nfl).data_ptr<int>();
               b.sync_err = need("sync_err", at::kInt, 1).data_ptr<int>();
             }
             Tensor images = need("images", at::kByte, HW);
             b.images = images.data_ptr<unsigned char>();
             Tensor labels = need("labels", at::kInt, 1);
             b.labels = labels.data_ptr<int>();
             Tensor idx = need("idx", at::kInt, 1);
             b.idx = idx.data_ptr<int>();
             b.n_idx = (int)idx.numel();
             b.n_rows = (int)std::min<long>(images.numel() / HW, labels.numel());
             // images / labels already permuted into the epoch's order: no index lookup
             if (cfgd.contains("epoch_order") && cfgd["epoch_order"].cast<bool>()) b.idx = nullptr;
             TORCH_CHECK(conv3x3_wgrad_lds(c.W, c.C1, c.C2, c.wgrad_rows, true, es) <= 160 * 1024, "wgrad rows too large");
             return std::make_shared<SimpleCNNEngine>(c, b, comm, buckets);
           }),
           py::arg("config"), py::arg("tensors"), py::arg("offsets"), py::arg("comm") = nullptr)
      .def("step", &SimpleCNNEngine::step, py::arg("batch"), py::arg("batch_stride"))
      .def("refresh_shadows", &SimpleCNNEngine::refresh_shadows)
      .def("set_lr", &SimpleCNNEngine::set_lr)
      .def("capture", &SimpleCNNEngine::capture)
      .def("replay", &SimpleCNNEngine::replay)
      .def("destroy_graph", &SimpleCNNEngine::destroy_graph)
      .def("synchronize", &SimpleCNNEngine::synchronize, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("last_fused_reduce", &SimpleCNNEngine::last_fused_reduce)
      .def_property_readonly("last_level3", &SimpleCNNEngine::last_level3)
      .def_property_readonly("last_fc_role", &SimpleCNNEngine::last_fc_role)
      .def_property_readonly("last_xar", &SimpleCNNEngine::last_xar)
      .def_property_readonly("last_pair", &SimpleCNNEngine::last_pair)
      .def("level3_active", &SimpleCNNEngine::level3_active, py::arg("batch"))
      .def_property_readonly("sync_error", &SimpleCNNEngine::sync_error)
      .def("set_momentum_started", &SimpleCNNEngine::set_momentum_started)
      .def("set_xgmi", &SimpleCNNEngine::set_xgmi, py::arg("xgmi"), py::arg("channels"))
      .def_property_readonly("num_buckets", &SimpleCNNEngine::num_buckets)
      .def("bucket_stage", &SimpleCNNEngine::bucket_stage)
      .def_property_readonly("graph_steps", &SimpleCNNEngine::graph_steps)
      .def_property_readonly("stream", [](SimpleCNNEngine& e) { return (uint64_t)e.stream(); });
}
