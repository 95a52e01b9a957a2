// Fused SimpleCNN DDP training step (the MI355X-native replacement of the
// reference's hot loop, train_ddp.py:195-200).
//
// Every kernel of a step is stream-ordered on the engine's compute stream (bucket
// all-reduces on a comm stream, joined by events), so a whole run of steps is captured
// in ONE hipGraph and replayed (no per-step host launches).  The default chain
// (EngineConfig::fuse_level 3, bf16, one GPU) is 2 kernels per step:
//
//   conv3x3_fwd   uint8 batch gather + /255 + conv1 (recomputed in the LDS staging pass)
//                 + conv2 (MFMA) + bias + ReLU -> a2, the fc partial logits; then a
//                 per-image in-launch wait for the image's other blocks, the softmax
//                 cross-entropy dL and dZ2 = relu2'(a2) * (dL . W_fc) for its own pixels
//   conv3x3_bwd   dgrad role (dZ1 + conv1 weight gradient), wgrad role (conv2 weight /
//                 bias gradient slabs, two blocks per slab row), the fc role (fc weight
//                 gradient + SGD of the fc weight and bias, the loss, the step counter)
//                 and the in-launch fixed-order slab reduction + SGD of the conv weights
//
// At world size > 1 the fc weight gradient is its own light kernel (fc_bwd without dX, dL
// given) on the comm stream, forked after the forward beside the conv backward, followed by
// the fc bucket's all-reduce - the direct xGMI kernels with SGD fused into their
// all-gather, or RCCL + one SGD pass; the conv bucket's all-reduce follows the conv
// backward (schedule_backward).
//
// Older chains stay selectable (tests pin them bit for bit against each other):
//   level 0: 8 kernels (conv1_fwd, conv3x3_fwd, xent, fc_bwd, dgrad, wgrad, grad_reduce,
//            sgd) with a1 materialised;
//   level 1: conv1 recomputed inside conv2 fwd / dgrad / wgrad, cross-entropy in the
//            fc_bwd prologue, optimizer in the epilogues, the slab reduction inside the
//            conv backward: 3 kernels (forward -> fc_bwd -> conv backward);
//   f32 = 1 (--dtype fp32): the same chains with exact fp32 operands (launch_step_f32): level 3
//            with both conv backward roles channel-split at two blocks per CU, or level 1.
//
// Buckets follow the reference DDP's rebuilt layout by default:
// bucket 0 = [fl.weight, fl.bias] (2.0 MB), bucket 1 = [net.2.*, net.0.*] (74 KB); any
// bucket plan works (stage 0 = fc-only buckets, stage 1 = the rest).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "runtime/runtime.h"

namespace ddp_amd {

SimpleCNNEngine::SimpleCNNEngine(const EngineConfig& cfg, const EngineBuffers& buf,
                                 std::shared_ptr<Comm> comm, std::vector<EngineBucket> buckets)
    : cfg_(cfg), b_(buf), comm_(std::move(comm)), buckets_(std::move(buckets)) {
  if (cfg_.C1 != 32) throw std::runtime_error("engine: fused conv1 wgrad needs C1 == 32");
  if (cfg_.C2 % 64 != 0) throw std::runtime_error("engine: C2 must be a multiple of 64");
  if ((cfg_.H * cfg_.W) % 16 != 0) throw std::runtime_error("engine: H*W must be a multiple of 16");
  if (cfg_.NO != 10) throw std::runtime_error("engine: the fused fc epilogue is built for 10 classes");
  if (cfg_.f32 && (cfg_.fuse_level < 1 || cfg_.store_a1 != 0))
    throw std::runtime_error("engine: fp32 mode needs fuse_level >= 1 (level 1 or 3) and store_a1 0");
  if (cfg_.f32 && !(b_.a2_f32 && b_.dz2_f32 && b_.w2t_f32 && b_.wfc_frag32))
    throw std::runtime_error("engine: fp32 mode needs the a2 / dz2 / w2t / wfc_frag32 fp32 buffers");
  // bucket plan: in-range, ordered, non-overlapping; stage by the first conv gradient
  const long conv0 = std::min(std::min(b_.off_w2, b_.off_b2), std::min(b_.off_w1, b_.off_b1));
  const long fc_hi = std::max(b_.off_wfc + (long)cfg_.NO * cfg_.H * cfg_.W * cfg_.C2, b_.off_bfc + cfg_.NO);
  if (fc_hi > conv0) throw std::runtime_error("engine: fc gradients must precede the conv gradients");
  long prev_end = 0;
  for (const EngineBucket& bk : buckets_) {
    if (bk.n <= 0 || bk.off < prev_end || bk.off + bk.n > b_.n_params)
      throw std::runtime_error("engine: bucket plan out of range / overlapping / unordered");
    prev_end = bk.off + bk.n;
    stage_.push_back(bk.off + bk.n <= conv0 ? 0 : 1);
  }
  last_bucket_ = (int)buckets_.size() - 1;
  for (int s : stage_) stage_used_[s] = true;
  xch_.assign(buckets_.size(), -1);
  DDP_HIP_CHECK(hipStreamCreateWithFlags(&cs_, hipStreamNonBlocking));
  DDP_HIP_CHECK(hipStreamCreateWithFlags(&ms_, hipStreamNonBlocking));
  for (hipEvent_t* e : {&e_b0_, &e_b1_, &e_d0_, &e_d1_, &e_fwd_, &e_fc_})
    DDP_HIP_CHECK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  l3_fits_.assign(cfg_.max_batch + 1, -1);
  // the in-launch wait-timeout word lives in coherent host memory: a kernel that times out
  // stores to it over the fabric and synchronize() reads it with a plain load - no
  // device-to-host copy (~10-20 us) after every synchronize
  if (b_.sync_err) {
    DDP_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&err_host_), sizeof(int),
                                hipHostMallocCoherent | hipHostMallocMapped));
    *err_host_ = 0;
    int* dev = nullptr;
    DDP_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dev), err_host_, 0));
    b_.sync_err = dev;
  }
}

SimpleCNNEngine::~SimpleCNNEngine() {
  // Streams are intentionally leaked (torch's caching allocators may still record
  // events on a stream that touched their blocks); nothing is released at exit.
  if (process_exiting()) return;
  if (cs_) hipStreamSynchronize(cs_);
  destroy_graph();
  for (hipEvent_t e : {e_b0_, e_b1_, e_d0_, e_d1_, e_fwd_, e_fc_}) hipEventDestroy(e);
  for (XarArgs& e : xar_cache_) hipFree(const_cast<XgmiArgs*>(e.dev));
  if (err_host_) hipHostFree(err_host_);
}

void SimpleCNNEngine::destroy_graph() {
  if (graph_exec_) hipGraphExecDestroy(graph_exec_);
  if (graph_) hipGraphDestroy(graph_);
  graph_exec_ = nullptr;
  graph_ = nullptr;
  graph_steps_ = 0;
}

void SimpleCNNEngine::synchronize() {
  DDP_HIP_CHECK(hipStreamSynchronize(cs_));
  if (const int e = sync_error()) {
    throw std::runtime_error(std::string("engine: an in-launch hand-off wait timed out (") +
                             (e == 2 ? "fused slab reduction" : e == XAR_ERR ? "in-launch all-reduce"
                                      : e == 5 ? "dist_mode 4 step head: forward waiting for the bucket all-reduce"
                                               : "level-3 forward dZ2") +
                             "); results invalid");
  }
}

bool SimpleCNNEngine::sync_ok_for_xar() const { return b_.sync_flags != nullptr && b_.sync_err != nullptr; }

bool SimpleCNNEngine::level3_active(int batch) {
  if (cfg_.fuse_level < 3 || !b_.sync_flags || !b_.sync_err) return false;
  if (batch <= 0 || batch > cfg_.max_batch) return false;
  signed char& f = l3_fits_[batch];
  if (f < 0)
    f = conv3x3_fwd_dz_fits(batch, cfg_.H, cfg_.W, cfg_.pxt_fwd, cfg_.f32 ? 4 : 2) && cfg_.C1 == 32 && cfg_.C2 == 64
            ? 1 : 0;
  return f == 1;
}

bool SimpleCNNEngine::overlap_active() {
  const bool use_x = xgmi_ && (xgmi_->world() > 1 || cfg_.force_allreduce);
  return cfg_.dist_mode == 4 && !cfg_.f32 && use_x && pair_plan_ok_ && cfg_.fuse_level >= 3 && cfg_.l3_fc_role &&
         cfg_.pxt_fwd == 1 && level3_active(cfg_.max_batch) &&
         conv3x3_bwd_fc_role_ok(cfg_.H, cfg_.W, cfg_.C1, cfg_.C2, cfg_.pxt_dgrad, cfg_.wgrad_split);
}

void SimpleCNNEngine::refresh_shadows() {
  SgdArgs a{0.f, 0.f, 0.f, 0.f, 0, 0, 0, /*update=*/0};
  ShadowSet sh{};
  const long n_w2 = (long)cfg_.C2 * 9 * cfg_.C1;
  if (cfg_.f32) {
    sh.r[0] = ShadowRegion{b_.off_w2, n_w2, nullptr, SHADOW_F32_TAPT, cfg_.C2, 9, cfg_.C1, b_.w2t_f32};
    sh.r[1] = ShadowRegion{b_.off_wfc, (long)cfg_.NO * cfg_.H * cfg_.W * cfg_.C2, nullptr, SHADOW_F32_FCFRAG,
                           cfg_.H * cfg_.W, cfg_.C2, 0, b_.wfc_frag32};
    sh.count = 2;
    sgd_step(b_.params, b_.grads, nullptr, b_.n_params, a, sh, nullptr, cs_);
    DDP_HIP_CHECK(hipGetLastError());
    return;
  }
  sh.r[0] = ShadowRegion{b_.off_w2, n_w2, b_.w2_bf16, SHADOW_BF16, 0, 0, 0};
  sh.r[1] = ShadowRegion{b_.off_w2, n_w2, b_.w2t_bf16, SHADOW_BF16_TAPT, cfg_.C2, 9, cfg_.C1};
  sh.r[2] = ShadowRegion{b_.off_wfc, (long)cfg_.NO * cfg_.H * cfg_.W * cfg_.C2, b_.wfc_bf16,
                         SHADOW_BF16, 0, 0, 0};
  sh.r[3] = ShadowRegion{b_.off_wfc, (long)cfg_.NO * cfg_.H * cfg_.W * cfg_.C2, b_.wfc_frag,
                         SHADOW_BF16_FCFRAG, cfg_.H * cfg_.W, cfg_.C2, 0};
  sh.count = 4;
  sgd_step(b_.params, b_.grads, nullptr, b_.n_params, a, sh, nullptr, cs_);
  DDP_HIP_CHECK(hipGetLastError());
}

void SimpleCNNEngine::launch_step(int B, int stride, bool first_momentum_step, unsigned parts) {
  if (cfg_.f32) {
    if (parts != PART_ALL) throw std::runtime_error("engine: the fp32 step runs whole (no step-head merge)");
    launch_step_f32(B, stride, first_momentum_step);
    return;
  }
  const int H = cfg_.H, W = cfg_.W, HW = H * W, C1 = cfg_.C1, C2 = cfg_.C2, NO = cfg_.NO;
  if (B <= 0 || B > cfg_.max_batch) throw std::runtime_error("engine: bad batch size");
  const bool use_x = xgmi_ && (xgmi_->world() > 1 || cfg_.force_allreduce);
  const bool dist = use_x || (comm_ && (comm_->world() > 1 || cfg_.force_allreduce));
  const float inv_ws = 1.f / (float)cfg_.world;
  BatchIdx bi{b_.idx, b_.step_ctr, stride, 0};
  bi.n_idx = b_.n_idx;
  bi.n_rows = b_.n_rows;
  float* P = b_.params;
  float* G = b_.grads;

  const bool f1 = cfg_.fuse_level >= 1;
  // level 1: the forward gathers the batch (step counter -> index list -> dataset row)
  // and writes it compactly (xb images, yb labels); every later kernel of the step reads
  // the compact copy with the identity index (no dependent lookup chain).
  C1Src c1;
  c1.x = b_.images;
  c1.bi = bi;
  c1.w = P + b_.off_w1;
  c1.b = P + b_.off_b1;
  c1.xb_out = b_.xb;
  c1.yb_out = b_.yb;
  c1.labels = b_.labels;
  if (cfg_.store_a1) c1.a1_out = b_.a1;
  const bool l3 = level3_active(B);
  const bool fred = f1 && cfg_.fuse_reduce && b_.sync_flags;  // grad_reduce inside the conv bwd
  const long n_fc = (long)NO * HW * C2;
  // dist_mode 3 on any chain (level 1 too: the same-GPU multi-rank rehearsals run level 1):
  // one stream, both buckets in one launch behind the conv backward
  const bool pair_mode = dist && use_x && f1 && cfg_.dist_mode >= 3 && sync_ok_for_xar();
  if (fred || l3 || pair_mode) {  // the forward resets the step's hand-off counters
    const int nfwd = conv3x3_dgrad_blocks(B, H, W, cfg_.pxt_fwd);
    const int nsync = SYNC_RED_INTS + ((l3 || pair_mode) ? L3_FC_INTS : 0);
    c1.zero_i32 = b_.sync_flags;
    c1.zero_per_block = (nsync + nfwd - 1) / nfwd;
    c1.zero_total = nsync;  // level 3: the per-image counters follow (L3_IMG_OFF)
  }
  if (!l3 && plain_stale_) {
    // the plain bf16 fc shadow (read by the level-1 fc backward) was not refreshed by the
    // level-3 steps before this one: re-derive every shadow from the fp32 master first
    refresh_shadows();
    plain_stale_ = false;
  }
  // level 3: the forward also writes dZ2 (per-image in-launch wait for the logits)
  FwdDz dzo;
  if (l3) {
    dzo.dz2 = b_.dz2;
    dzo.img_cnt = b_.sync_flags + L3_IMG_OFF;
    dzo.fc_bias = P + b_.off_bfc;
    dzo.gscale = 1.f / (float)B;
    dzo.err = b_.sync_err;
    dzo.dl_out = b_.dlogits;     // dL rows + per-row losses: the fc backward reads them
    dzo.loss_rows = b_.loss_rows;
  }
  // level 3, single process: the fc weight gradient runs as a third role of the conv
  // backward launch (2 kernels per step); at world size > 1 it runs as its own light kernel
  // before it (the fc bucket's all-reduce then overlaps the conv backward)
  // dist_mode 2 (xGMI): the same fc role inside the conv backward at world size > 1, its
  // gradient all-reduced in-launch (make_xar / BwdXar)
  const bool xar_mode = dist && use_x && l3 &&
                        ((cfg_.dist_mode == 2 && xar_plan_ok_) || cfg_.dist_mode >= 3);
  // the one-stream chains: fc weight gradient (role or kernel) -> conv backward -> the bucket
  // all-reduces on cs_ (in-launch: dist_mode 2; one pair launch: dist_mode 3 / 4)
  const bool one_stream = xar_mode || pair_mode;
  const bool fc_role = l3 && (!dist || xar_mode) && cfg_.l3_fc_role &&
                       conv3x3_bwd_fc_role_ok(H, W, C1, C2, cfg_.pxt_dgrad, cfg_.wgrad_split);
  // dist_mode 4 (the step head): mode 3's chain, but the step counter advances in the conv
  // backward's fc role (after it read the loss index) instead of the pair launch, so that the
  // pair launch can carry the NEXT step's forward (which reads the counter for its batch)
  const bool ov = dist && use_x && l3 && fc_role && cfg_.dist_mode == 4;
  if ((parts & (PART_HEAD | PART_AR)) && !ov && parts != PART_ALL)
    throw std::runtime_error("engine: a split step needs the dist_mode 4 chain");
  const C1Src* pc1 = f1 ? &c1 : nullptr;
  BatchIdx bid{nullptr, nullptr, 0, 0};
  bid.n_rows = B;
  C1Src c1b;
  c1b.x = b_.xb;
  c1b.bi = bid;
  c1b.w = c1.w;
  c1b.b = c1.b;

  // every bf16 shadow the chain reads; a bucket's fused SGD refreshes the ones inside its
  // range (level 3 never reads the plain fc shadow: plain_stale_ re-derives it on a switch)
  const long n_w2s = (long)C2 * 9 * C1;
  ShadowSet sh_all{};
  sh_all.r[0] = ShadowRegion{b_.off_w2, n_w2s, b_.w2_bf16, SHADOW_BF16, 0, 0, 0};
  sh_all.r[1] = ShadowRegion{b_.off_w2, n_w2s, b_.w2t_bf16, SHADOW_BF16_TAPT, C2, 9, C1};
  sh_all.r[2] = ShadowRegion{b_.off_wfc, n_fc, b_.wfc_frag, SHADOW_BF16_FCFRAG, HW, C2, 0};
  sh_all.r[3] = ShadowRegion{b_.off_wfc, n_fc, b_.wfc_bf16, SHADOW_BF16, 0, 0, 0};
  sh_all.count = l3 ? 3 : 4;
  // ---- forward (PART_HEAD: in one launch with the previous step's bucket all-reduces)
  const SgdArgs sa{cfg_.lr, cfg_.momentum, cfg_.dampening, cfg_.weight_decay, cfg_.nesterov,
                   cfg_.maximize, first_momentum_step ? 1 : 0, 1};
  float* M = b_.momentum;  // null when momentum == 0
  bool head_used = false;
  if (parts & PART_HEAD) {
    // the previous step's pair (its fused SGD writes this step's parameters write-through)
    // + this step's forward; two launches (same bits) when the merged grid does not fit
    if (first_momentum_step) throw std::runtime_error("engine: the step head runs the steady-state SGD only");
    // the head's fused SGD refreshes the shadows its forward reads (conv2 bf16, fc fragment
    // order); the conv2 [tap][ci][co] copy (the next backward's) is written after the conv
    // bucket's count (FwdMerge late).  The same bytes as sh_all, in two passes.
    // Only when the whole conv2 weight lies in the one-shot conv-stage bucket: its blocks
    // then rewrite exactly the quads they updated (no wait on another block); any other plan
    // refreshes every shadow in the SGD pass as before.
    ShadowSet sh_head = sh_all, late{};
    if (late_shadow_ok(b_.off_w2, n_w2s)) {
      sh_head.r[1] = sh_all.r[2];
      sh_head.count = 2;
      late.r[0] = sh_all.r[1];
      late.count = 1;
    }
    BwdXar hx;
    int* mc = b_.sync_flags + L3_IMG_OFF + (long)FWD_DZ_CNT_STRIDE * cfg_.max_batch;
    if (cfg_.pxt_fwd == 1 && B == cfg_.max_batch) {
      if (!make_xar(hx, sa, M, sh_head)) throw std::runtime_error("engine: the step head needs the pair plan");
      hx.step_ctr = nullptr;  // (advanced by the fc role)
      head_used = conv3x3_step_head(hx, mc, mc + FWD_DZ_CNT_STRIDE, b_.w2_bf16, P + b_.off_b2, b_.a2, B,
                                    b_.wfc_frag, b_.fc_part, c1, dzo, b_.sync_err, cs_, &late);
    }
    if (!head_used) {
      if (!make_xar(hx, sa, M, sh_all)) throw std::runtime_error("engine: the step head needs the pair plan");
      hx.step_ctr = nullptr;
      xgmi_allreduce_pair(hx, cs_);
    }
    DDP_HIP_CHECK(hipGetLastError());
  }
  if ((parts & PART_FWD) || ((parts & PART_HEAD) && !head_used)) {
    if (!f1) conv1_fwd(b_.images, true, bi, P + b_.off_w1, P + b_.off_b1, b_.a1, B, H, W, C1, cs_);
    conv3x3_fwd(f1 ? nullptr : b_.a1, b_.w2_bf16, P + b_.off_b2, b_.a2, B, H, W, C1, C2, true,
                b_.wfc_frag, b_.fc_part, NO, cfg_.pxt_fwd, cs_, pc1, l3 ? &dzo : nullptr);
  }
  if (parts & (PART_FWD | PART_HEAD)) last_head_ = head_used;
  if (head_used && capturing_) graph_heads_ += 1;
  if (!(parts & (PART_BWD | PART_AR))) return;
  // ---- loss + fc backward (bucket 0)
  if (!f1)
    xent_rows(b_.fc_part, HW, 64 * cfg_.pxt_fwd, P + b_.off_bfc, NO, B, b_.labels, bi, b_.dlogits,
              b_.loss_rows, 1.f / (float)B, cs_);
  FcBwdExtras ex;
  ex.dbias = G + b_.off_bfc;  // fc bias grad (bucket 0), prescaled
  ex.dbias_scale = inv_ws;
  ex.loss_rows = b_.loss_rows;
  ex.loss_out = b_.loss_hist;  // per-epoch history, indexed by the step counter
  ex.step_ctr = b_.step_ctr;
  if (f1) {
    ex.loss_rows = nullptr;
    ex.part = b_.fc_part;
    ex.HW = HW;
    ex.CH = 64 * cfg_.pxt_fwd;
    ex.fc_bias = P + b_.off_bfc;
    ex.labels32 = b_.yb;
    ex.bi = bid;
    ex.gscale = 1.f / (float)B;
  }
  // single-process steps: no all-reduce separates a gradient from its update, so the
  // optimizer runs in the epilogues of the kernels that finish each gradient (fc weight:
  // fc_bwd; convs + fc bias: grad_reduce) and the separate SGD pass disappears
  const bool fopt = !dist && cfg_.fuse_opt;
  const long n_w2 = (long)C2 * 9 * C1, w2row = n_w2 + C2;
  ex.sys_store = use_x ? 1 : 0;  // bucket 0 is read by the peers over xGMI
  if (fopt) {
    ex.sgd = sa;
    ex.p_w = P + b_.off_wfc;
    ex.m_w = M ? M + b_.off_wfc : nullptr;
    ex.sh_plain = b_.wfc_bf16;
    ex.sh_frag = b_.wfc_frag;
    ex.frag_HW = HW;
    ex.frag_C = C2;
  }
  // (fused optimizer: the fc weight gradient is consumed in registers and not stored)
  BwdFc fcr;  // the conv backward's fc role (fc_role)
  std::function<void(hipStream_t)> fc_launch;  // the fc weight-gradient kernel, when not a role
  if (l3) {
    // level 3: no dZ2 and no cross-entropy prologue here (the forward wrote dZ2, dL, losses)
    ex.part = nullptr;
    ex.loss_rows = b_.loss_rows;
    ex.zero_i32 = dzo.img_cnt;  // re-arm the forward's per-image counters for the next step
    // (dist_mode 4: and the step head's two bucket-done counters behind them)
    ex.n_zero = ov ? cfg_.max_batch + 2 : B;
    ex.zero_stride = FWD_DZ_CNT_STRIDE;
    if (fc_role) {
      // inside the conv backward launch: block 0 of the fc role owns the fc bias, the loss
      // and the step counter (nothing else in the launch reads them)
      if (fopt) {
        ex.p_b = P + b_.off_bfc;
        ex.m_b = M ? M + b_.off_bfc : nullptr;
        ex.step_inc = b_.step_ctr;
      }
      if (ov) ex.step_inc = b_.step_ctr;
      ex.sh_plain = nullptr;  // level 3 never reads the plain bf16 fc shadow (stale until refreshed)
      fcr.a2 = b_.a2;
      fcr.dl = b_.dlogits;
      fcr.dW = fopt ? nullptr : G + b_.off_wfc;
      fcr.scale = inv_ws;
      fcr.K = (long)HW * C2;
      fcr.ex = ex;
    } else {
      ex.sh_plain = nullptr;
      fc_launch = [&](hipStream_t s) {
        fc_bwd(b_.dlogits, b_.a2, nullptr, nullptr, fopt ? nullptr : G + b_.off_wfc, inv_ws, B, (long)HW * C2, NO,
               /*mask=*/true, s, ex);
      };
    }
    plain_stale_ = true;
  } else {
    fc_launch = [&](hipStream_t s) {
      fc_bwd(b_.dlogits, b_.a2, b_.wfc_bf16, b_.dz2, fopt ? nullptr : G + b_.off_wfc, inv_ws, B,
             (long)HW * C2, NO, /*mask=*/true, s, ex);
    };
  }
  // ---- conv backward (bucket 1) + the slab reduction (fused into it, or grad_reduce)
  SlabSet ss{};
  const int wblk = conv3x3_wgrad_blocks(B, H, cfg_.wgrad_rows);
  ss.s[0] = SlabSeg{b_.w2slab, w2row, 0, n_w2, wblk, G + b_.off_w2, inv_ws};
  ss.s[1] = SlabSeg{b_.w2slab, w2row, n_w2, (long)C2, wblk, G + b_.off_b2, inv_ws};
  const int dblk = conv3x3_dgrad_blocks(B, H, W, cfg_.pxt_dgrad);
  ss.s[2] = SlabSeg{b_.w1slab, 320, 0, (long)C1 * 9, dblk, G + b_.off_w1, inv_ws};
  ss.s[3] = SlabSeg{b_.w1slab, 320, (long)C1 * 9, (long)C1, dblk, G + b_.off_b1, inv_ws};
  ss.count = 4;
  if (fopt) {
    auto opt = [&](SlabSeg& sg, long off) {
      sg.p = P + off;
      sg.m = M ? M + off : nullptr;
    };
    opt(ss.s[0], b_.off_w2);
    ss.s[0].sh = b_.w2_bf16;
    ss.s[0].sh_t = b_.w2t_bf16;
    ss.s[0].t_co = C2; ss.s[0].t_taps = 9; ss.s[0].t_ci = C1;
    opt(ss.s[1], b_.off_b2);
    opt(ss.s[2], b_.off_w1);
    opt(ss.s[3], b_.off_b1);
    ss.count = 4;
    ss.sgd = sa;
    if (!fc_role) {
      // fc bias: its gradient (fc_bwd block 0) is already final; a 1-row "slab" in place
      // (level-3 fc role: its last block applies it - that role runs inside this launch)
      ss.s[4] = SlabSeg{G + b_.off_bfc, (long)NO, 0, (long)NO, 1, G + b_.off_bfc, 1.f};
      opt(ss.s[4], b_.off_bfc);
      ss.count = 5;
      ss.step_ctr = b_.step_ctr;  // the step's last kernel advances the batch window
    }
  }
  ss.sys_store = use_x ? 1 : 0;  // bucket 1 likewise
  bool reduced = false;  // the conv backward launch also did grad_reduce's work
  BwdXar xa;
  const bool want_xar = xar_mode && cfg_.dist_mode == 2 && fc_role && fred && make_xar(xa, sa, M, sh_all);
  if (dist && use_x && l3 && cfg_.dist_mode == 2 && !want_xar && std::getenv("DDP_AMD_XAR_DEBUG"))
    fprintf(stderr, "[ddp_amd] in-launch all-reduce off: plan_ok %d fc_role %d fred %d buckets %d\n",
            (int)xar_plan_ok_, (int)fc_role, (int)fred, (int)buckets_.size());
  bool xar_used = false, pair_used = false;
  auto conv_launch = [&]() {
    if (!(parts & PART_BWD)) {  // (dist_mode 4: the last step's pair alone)
    } else if (f1) {
      // dZ1 only feeds conv1's weight gradient, which the dgrad role computes in registers
      reduced = conv3x3_bwd(b_.dz2, b_.w2t_bf16, nullptr, b_.w1slab, b_.w2slab, B, H, W, C1, C2, cfg_.pxt_dgrad,
                            cfg_.wgrad_rows, c1b, cfg_.store_a1 ? b_.a1 : nullptr, cfg_.store_a1 == 2, cs_,
                            fred ? &ss : nullptr, b_.sync_flags, b_.sync_err, cfg_.wgrad_split,
                            fc_role ? &fcr : nullptr, !dist && cfg_.fuse_reduce == 2, want_xar ? &xa : nullptr,
                            &xar_used);
    } else {
      conv3x3_dgrad(b_.dz2, nullptr, b_.w2t_bf16, b_.a1, b_.dz1, B, H, W, C1, C2, b_.images, true, bi,
                    b_.w1slab, cfg_.pxt_dgrad, cs_, nullptr);
      conv3x3_wgrad(b_.dz2, nullptr, b_.a1, b_.w2slab, B, H, W, C1, C2, cfg_.wgrad_rows, cs_, nullptr);
    }
    if (!reduced && (parts & PART_BWD)) grad_reduce(ss, cs_);
    if (one_stream && !xar_used && (parts & PART_AR)) {
      // dist_mode 3 / 4 (or the in-launch all-reduce did not apply): the bucket all-reduces
      // behind the conv backward on the compute stream - both in one launch when the plan allows
      BwdXar pr;
      if (cfg_.dist_mode >= 3 && make_xar(pr, sa, M, sh_all)) {
        if (ov) pr.step_ctr = nullptr;  // (advanced by the fc role)
        xgmi_allreduce_pair(pr, cs_);
        pair_used = true;
        DDP_HIP_CHECK(hipGetLastError());
      } else {
        enqueue_buckets(0, use_x, cs_, sa, M, sh_all);
        enqueue_buckets(1, use_x, cs_, sa, M, sh_all);
      }
    }
  };
  // fc buckets overlap the conv backward: in-launch (dist_mode 2), or the fc weight gradient
  // forks off the compute stream after the forward (dist_mode 1); the one-stream chains run
  // the fc weight-gradient kernel (when it is not a role of the conv backward) first
  if (one_stream) {
    if (fc_launch && (parts & PART_BWD)) fc_launch(cs_);
    conv_launch();
  } else {
    schedule_backward(dist, dist && l3 && cfg_.dist_mode == 1, use_x, fc_launch, conv_launch, sa, M, sh_all);
  }
  if (!(parts & PART_BWD)) {  // (a lone pair: the step's other flags stay those of its backward)
    last_pair_ = pair_used;
    return;
  }
  last_fused_reduce_ = reduced;
  last_level3_ = l3;
  last_fc_role_ = fc_role;
  last_xar_ = xar_used;
  last_pair_ = pair_used || head_used;
  if (fopt) return;
  if (dist && use_x) return;  // the optimizer ran inside the all-reduces
  // ---- optimizer + bf16 shadows + next batch window
  sgd_step(P, G, M, b_.n_params, sa, sh_all, b_.step_ctr, cs_);
}

void SimpleCNNEngine::launch_buckets(int stage, bool use_x, const SgdArgs& sa, float* M, const ShadowSet& sh) {
  if (!stage_used_[stage]) return;
  hipEvent_t ready = stage == 0 ? e_b0_ : e_b1_;
  DDP_HIP_CHECK(hipEventRecord(ready, cs_));
  DDP_HIP_CHECK(hipStreamWaitEvent(ms_, ready, 0));
  enqueue_buckets(stage, use_x, ms_, sa, M, sh);
  DDP_HIP_CHECK(hipEventRecord(stage == 0 ? e_d0_ : e_d1_, ms_));
}

void SimpleCNNEngine::enqueue_buckets(int stage, bool use_x, hipStream_t s, const SgdArgs& sa, float* M,
                                      const ShadowSet& sh) {
  for (int b = 0; b < (int)buckets_.size(); ++b) {
    if (stage_[b] != stage) continue;
    if (use_x) {
      xgmi_->all_reduce_sgd(xch_[b], s, sa, b_.params, M, sh, b == last_bucket_ ? b_.step_ctr : nullptr);
    } else {
      comm_->all_reduce(b_.grads + buckets_[b].off, (size_t)buckets_[b].n, 0, 0, s);
    }
  }
}

bool SimpleCNNEngine::late_shadow_ok(long off, long n) const {
  if (!xgmi_) return false;
  bool inside = false;
  for (int b = 0; b < (int)buckets_.size(); ++b) {
    const long b0 = buckets_[b].off, b1 = b0 + (long)buckets_[b].n;
    const bool overlaps = b0 < off + n && off < b1;
    if (!overlaps) continue;
    if (stage_[b] != 1 || !xgmi_->oneshot(xch_[b]) || b0 > off || b1 < off + n) return false;
    inside = true;
  }
  return inside;
}

bool SimpleCNNEngine::make_xar(BwdXar& xa, const SgdArgs& sa, float* M, const ShadowSet& sh) {
  if (!xgmi_ || !(cfg_.dist_mode >= 3 ? pair_plan_ok_ : xar_plan_ok_)) return false;
  // the pair lives in device memory, one immutable copy per distinct content (a captured
  // graph keeps pointing at the copy it was captured with): the momentum-init step's and
  // the steady state's - both made on the first (eager) call, so a capture never needs a
  // new one - and a pair more if the learning rate changes
  auto build = [&](const SgdArgs& g, XgmiArgs* pair) {
    for (int b = 0; b < (int)buckets_.size(); ++b) {
      // the bucket's fused optimizer; the all-reduce roles advance the step counter themselves
      pair[stage_[b]] = xgmi_->make_args(xch_[b], g, b_.params, M, sh, nullptr);
      (stage_[b] == 0 ? xa.nblk0 : xa.nblk1) = xgmi_->blocks(xch_[b]);
    }
  };
  auto find = [&](const XgmiArgs* pair) -> const XgmiArgs* {
    for (const XarArgs& e : xar_cache_)
      if (std::memcmp(e.host, pair, sizeof(XgmiArgs) * 2) == 0) return e.dev;
    return nullptr;
  };
  XgmiArgs pair[2] = {};
  build(sa, pair);
  const XgmiArgs* dev = find(pair);
  if (!dev) {
    // (a first capture without an eager step before it lands here while capturing: the
    // capture is in relaxed mode, and the allocation and the copy run at once, outside the
    // graph, on a stream of their own)
    SgdArgs other = sa;
    other.first_step = sa.first_step ? 0 : 1;
    XgmiArgs pair2[2] = {};
    build(other, pair2);
    for (const XgmiArgs* p : {static_cast<const XgmiArgs*>(pair), static_cast<const XgmiArgs*>(pair2)}) {
      if (find(p)) continue;
      XarArgs e;
      std::memcpy(e.host, p, sizeof(e.host));
      XgmiArgs* d = nullptr;
      DDP_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&d), sizeof(e.host)));
      // (a private non-blocking stream: the legacy stream may not depend on a capture)
      if (!xs_) DDP_HIP_CHECK(hipStreamCreateWithFlags(&xs_, hipStreamNonBlocking));
      DDP_HIP_CHECK(hipMemcpyAsync(d, p, sizeof(e.host), hipMemcpyHostToDevice, xs_));
      DDP_HIP_CHECK(hipStreamSynchronize(xs_));
      e.dev = d;
      xar_cache_.push_back(e);
    }
    dev = find(pair);
  }
  xa.args = dev;
  // three counters of the step's zeroed hand-off words (the forward clears [0, L3_IMG_OFF))
  xa.fc_done = b_.sync_flags + SYNC_RED_INTS + 8;
  xa.red_done = b_.sync_flags + SYNC_RED_INTS + 16;
  xa.xar_done = b_.sync_flags + SYNC_RED_INTS + 24;
  xa.step_ctr = b_.step_ctr;
  xa.err = b_.sync_err;
  return true;
}

// World size > 1 (or forced), dist_mode 1, level 3 - the forward already wrote dL and dZ2, so
// the fc weight gradient depends on the forward alone:
//
//   cs_: forward -> conv backward (+ fused slab reduction) -> [xGMI] conv buckets -> join
//   ms_:         `-> fc_bwd -> fc buckets' all-reduce (+ fused SGD) -----------------'
//
// a two-branch graph: the conv backward starts right behind the forward instead of behind
// fc_bwd (DDP's bucket 0 fires while the conv backward
// still runs).  Over xGMI the conv buckets stay on the compute stream (no event hop after
// the conv backward; each bucket has its own channel, so the two branches' all-reduces
// never share flags); they wait for fc_bwd first, which reads the step counter that the
// last bucket advances.  RCCL keeps every collective on ms_ (one communicator: the ranks
// must issue its calls in one order).
void SimpleCNNEngine::schedule_backward(bool dist, bool fork, bool use_x, const std::function<void(hipStream_t)>& fc,
                                        const std::function<void()>& conv, const SgdArgs& sa, float* M,
                                        const ShadowSet& sh) {
  if (!dist) {
    if (fc) fc(cs_);
    conv();
    return;
  }
  if (!fork || !fc) {  // the round-4 order
    if (fc) fc(cs_);
    launch_buckets(0, use_x, sa, M, sh);
    conv();
    launch_buckets(1, use_x, sa, M, sh);
    join_buckets();
    return;
  }
  DDP_HIP_CHECK(hipEventRecord(e_fwd_, cs_));
  DDP_HIP_CHECK(hipStreamWaitEvent(ms_, e_fwd_, 0));
  fc(ms_);
  DDP_HIP_CHECK(hipEventRecord(e_fc_, ms_));
  if (stage_used_[0]) enqueue_buckets(0, use_x, ms_, sa, M, sh);
  DDP_HIP_CHECK(hipEventRecord(e_d0_, ms_));
  conv();
  if (use_x) {
    DDP_HIP_CHECK(hipStreamWaitEvent(cs_, e_fc_, 0));
    if (stage_used_[1]) enqueue_buckets(1, use_x, cs_, sa, M, sh);
    DDP_HIP_CHECK(hipStreamWaitEvent(cs_, e_d0_, 0));
  } else {
    if (stage_used_[1]) {
      DDP_HIP_CHECK(hipEventRecord(e_b1_, cs_));
      DDP_HIP_CHECK(hipStreamWaitEvent(ms_, e_b1_, 0));
      enqueue_buckets(1, use_x, ms_, sa, M, sh);
    }
    DDP_HIP_CHECK(hipEventRecord(e_d1_, ms_));
    DDP_HIP_CHECK(hipStreamWaitEvent(cs_, e_d1_, 0));
  }
}

void SimpleCNNEngine::join_buckets() {
  // the comm stream is in order: its last recorded event covers every earlier bucket
  DDP_HIP_CHECK(hipStreamWaitEvent(cs_, stage_used_[1] ? e_d1_ : e_d0_, 0));
}

// The exact-fp32 step: the bf16 chains on fp32 operands.  Level 3 (default): the forward
// also computes dL and dZ2 (per-image in-launch wait), and one conv backward launch runs the
// dgrad and wgrad roles (both split over input-channel halves at two blocks per CU:
// wgrad_split 2), the fc weight gradient + SGD as a third role (single process) and the
// fused slab reduction + SGD.  Level 1: forward -> fc backward (cross-entropy prologue) ->
// conv backward (+ the slab reduction).  Both chains give the same bits.
void SimpleCNNEngine::launch_step_f32(int B, int stride, bool first_momentum_step) {
  const int H = cfg_.H, W = cfg_.W, HW = H * W, C1 = cfg_.C1, C2 = cfg_.C2, NO = cfg_.NO;
  if (B <= 0 || B > cfg_.max_batch) throw std::runtime_error("engine: bad batch size");
  const bool use_x = xgmi_ && (xgmi_->world() > 1 || cfg_.force_allreduce);
  const bool dist = use_x || (comm_ && (comm_->world() > 1 || cfg_.force_allreduce));
  const float inv_ws = 1.f / (float)cfg_.world;
  BatchIdx bi{b_.idx, b_.step_ctr, stride, 0};
  bi.n_idx = b_.n_idx;
  bi.n_rows = b_.n_rows;
  float* P = b_.params;
  float* G = b_.grads;
  float* M = b_.momentum;
  C1Src c1;
  c1.x = b_.images;
  c1.bi = bi;
  c1.w = P + b_.off_w1;
  c1.b = P + b_.off_b1;
  c1.xb_out = b_.xb;
  c1.yb_out = b_.yb;
  c1.labels = b_.labels;
  BatchIdx bid{nullptr, nullptr, 0, 0};
  bid.n_rows = B;
  C1Src c1b;
  c1b.x = b_.xb;
  c1b.bi = bid;
  c1b.w = c1.w;
  c1b.b = c1.b;
  const bool l3 = level3_active(B);
  const bool fred = cfg_.fuse_reduce && b_.sync_flags;  // grad_reduce inside the conv bwd
  const bool pair_mode = dist && use_x && cfg_.dist_mode >= 3 && sync_ok_for_xar();  // (see launch_step)
  if (fred || l3 || pair_mode) {  // the forward resets the step's hand-off counters
    const int nfwd = conv3x3_dgrad_blocks(B, H, W, cfg_.pxt_fwd);
    const int nsync = SYNC_RED_INTS + ((l3 || pair_mode) ? L3_FC_INTS : 0);
    c1.zero_i32 = b_.sync_flags;
    c1.zero_per_block = (nsync + nfwd - 1) / nfwd;
    c1.zero_total = nsync;
  }
  const long n_w2 = (long)C2 * 9 * C1, w2row = n_w2 + C2, n_fc = (long)NO * HW * C2;
  const SgdArgs sa{cfg_.lr, cfg_.momentum, cfg_.dampening, cfg_.weight_decay, cfg_.nesterov,
                   cfg_.maximize, first_momentum_step ? 1 : 0, 1};
  const bool fopt = !dist && cfg_.fuse_opt;
  FwdDz dzo;
  if (l3) {
    dzo.dz2_f32 = b_.dz2_f32;
    dzo.img_cnt = b_.sync_flags + L3_IMG_OFF;
    dzo.fc_bias = P + b_.off_bfc;
    dzo.gscale = 1.f / (float)B;
    dzo.err = b_.sync_err;
    dzo.dl_out = b_.dlogits;
    dzo.loss_rows = b_.loss_rows;
  }
  const bool xar_mode = dist && use_x && l3 &&
                        ((cfg_.dist_mode == 2 && xar_plan_ok_) || cfg_.dist_mode >= 3);
  const bool one_stream = xar_mode || pair_mode;  // (fp32: dist_mode 4 runs mode 3's chain)
  const bool fc_role = l3 && (!dist || xar_mode) && cfg_.l3_fc_role &&
                       conv3x3_bwd_fc_role_ok(H, W, C1, C2, cfg_.pxt_dgrad, cfg_.wgrad_split);

  // ---- forward: conv1 (recomputed) + conv2 + bias + ReLU -> a2, fused fc partial logits
  //      (level 3: then dL and dZ2 after the per-image wait)
  conv3x3_fwd(static_cast<const float*>(nullptr), P + b_.off_w2, P + b_.off_b2, b_.a2_f32, B, H, W, C1, C2,
              true, b_.wfc_frag32, b_.fc_part, NO, cfg_.pxt_fwd, cs_, &c1, l3 ? &dzo : nullptr);
  // ---- loss + fc backward (bucket 0)
  FcBwdExtras ex;
  ex.dbias = G + b_.off_bfc;
  ex.dbias_scale = inv_ws;
  ex.loss_out = b_.loss_hist;
  ex.step_ctr = b_.step_ctr;
  ex.sys_store = use_x ? 1 : 0;
  if (l3) {
    ex.loss_rows = b_.loss_rows;  // dL and the row losses come from the forward
    ex.zero_i32 = dzo.img_cnt;    // re-arm the forward's per-image counters
    ex.n_zero = B;
    ex.zero_stride = FWD_DZ_CNT_STRIDE;
  } else {
    ex.part = b_.fc_part;
    ex.HW = HW;
    ex.CH = 64 * cfg_.pxt_fwd;
    ex.fc_bias = P + b_.off_bfc;
    ex.labels32 = b_.yb;
    ex.bi = bid;
    ex.gscale = 1.f / (float)B;
  }
  if (fopt) {  // each block / wave updates only the fc columns it alone reads: race free in place
    ex.sgd = sa;
    ex.p_w = P + b_.off_wfc;
    ex.m_w = M ? M + b_.off_wfc : nullptr;
    ex.sh_frag32 = b_.wfc_frag32;  // the forward's fc operand
    ex.frag_HW = HW;
    ex.frag_C = C2;
  }
  BwdFc fcr;
  std::function<void(hipStream_t)> fc_launch;  // the fc weight-gradient kernel, when not a role
  if (fc_role) {
    // inside the conv backward launch: block 0 of the fc role owns the fc bias, the loss and
    // the step counter (nothing else in the launch reads them)
    if (fopt) {
      ex.p_b = P + b_.off_bfc;
      ex.m_b = M ? M + b_.off_bfc : nullptr;
      ex.step_inc = b_.step_ctr;
    }
    fcr.a2 = b_.a2_f32;
    fcr.dl = b_.dlogits;
    fcr.dW = fopt ? nullptr : G + b_.off_wfc;
    fcr.scale = inv_ws;
    fcr.K = (long)HW * C2;
    fcr.ex = ex;
  } else if (l3) {
    fc_launch = [&](hipStream_t s) {
      fc_bwd(b_.dlogits, b_.a2_f32, nullptr, nullptr, fopt ? nullptr : G + b_.off_wfc, inv_ws, B, (long)HW * C2,
             NO, /*mask=*/true, s, ex);
    };
  } else {
    fc_launch = [&](hipStream_t s) {
      fc_bwd(b_.dlogits, b_.a2_f32, P + b_.off_wfc, b_.dz2_f32, fopt ? nullptr : G + b_.off_wfc, inv_ws, B,
             (long)HW * C2, NO, /*mask=*/true, s, ex);
    };
  }
  ShadowSet sh1{};
  sh1.r[0] = ShadowRegion{b_.off_w2, n_w2, nullptr, SHADOW_F32_TAPT, C2, 9, C1, b_.w2t_f32};
  sh1.r[1] = ShadowRegion{b_.off_wfc, n_fc, nullptr, SHADOW_F32_FCFRAG, HW, C2, 0, b_.wfc_frag32};
  sh1.count = 2;
  // ---- conv backward (bucket 1) + the slab reduction (fused into it, or grad_reduce)
  SlabSet ss{};
  const int wblk = conv3x3_wgrad_blocks(B, H, cfg_.wgrad_rows);
  ss.s[0] = SlabSeg{b_.w2slab, w2row, 0, n_w2, wblk, G + b_.off_w2, inv_ws};
  ss.s[1] = SlabSeg{b_.w2slab, w2row, n_w2, (long)C2, wblk, G + b_.off_b2, inv_ws};
  const int dblk = conv3x3_dgrad_blocks(B, H, W, cfg_.pxt_dgrad);
  ss.s[2] = SlabSeg{b_.w1slab, 320, 0, (long)C1 * 9, dblk, G + b_.off_w1, inv_ws};
  ss.s[3] = SlabSeg{b_.w1slab, 320, (long)C1 * 9, (long)C1, dblk, G + b_.off_b1, inv_ws};
  ss.count = 4;
  if (fopt) {
    auto opt = [&](SlabSeg& sg, long off) {
      sg.p = P + off;
      sg.m = M ? M + off : nullptr;
    };
    opt(ss.s[0], b_.off_w2);
    ss.s[0].sh_t32 = b_.w2t_f32;
    ss.s[0].t_co = C2; ss.s[0].t_taps = 9; ss.s[0].t_ci = C1;
    opt(ss.s[1], b_.off_b2);
    opt(ss.s[2], b_.off_w1);
    opt(ss.s[3], b_.off_b1);
    if (!fc_role) {
      // fc bias: its gradient (fc_bwd block 0) is already final; a 1-row "slab" in place
      ss.s[4] = SlabSeg{G + b_.off_bfc, (long)NO, 0, (long)NO, 1, G + b_.off_bfc, 1.f};
      opt(ss.s[4], b_.off_bfc);
      ss.count = 5;
      ss.step_ctr = b_.step_ctr;
    }
    ss.sgd = sa;
  }
  ss.sys_store = use_x ? 1 : 0;
  bool reduced = false;
  BwdXar xa;
  const bool want_xar = xar_mode && cfg_.dist_mode == 2 && fc_role && fred && make_xar(xa, sa, M, sh1);
  bool xar_used = false, pair_used = false;
  auto conv_launch = [&]() {
    reduced = conv3x3_bwd(b_.dz2_f32, b_.w2t_f32, nullptr, b_.w1slab, b_.w2slab, B, H, W, C1, C2, cfg_.pxt_dgrad,
                          cfg_.wgrad_rows, c1b, static_cast<const float*>(nullptr), false, cs_,
                          fred ? &ss : nullptr, b_.sync_flags, b_.sync_err, cfg_.wgrad_split,
                          fc_role ? &fcr : nullptr, !dist && cfg_.fuse_reduce == 2, want_xar ? &xa : nullptr,
                          &xar_used);
    if (!reduced) grad_reduce(ss, cs_);
    if (one_stream && !xar_used) {
      // dist_mode 3 (or the in-launch all-reduce did not apply): the bucket all-reduces behind
      // the conv backward on the compute stream - both in one launch when the plan allows
      BwdXar pr;
      if (cfg_.dist_mode >= 3 && make_xar(pr, sa, M, sh1)) {
        xgmi_allreduce_pair(pr, cs_);
        pair_used = true;
        DDP_HIP_CHECK(hipGetLastError());
      } else {
        enqueue_buckets(0, use_x, cs_, sa, M, sh1);
        enqueue_buckets(1, use_x, cs_, sa, M, sh1);
      }
    }
  };
  if (one_stream) {
    if (fc_launch) fc_launch(cs_);
    conv_launch();
  } else {
    schedule_backward(dist, dist && l3 && cfg_.dist_mode == 1, use_x, fc_launch, conv_launch, sa, M, sh1);
  }
  last_fused_reduce_ = reduced;
  last_level3_ = l3;
  last_fc_role_ = fc_role;
  last_xar_ = xar_used;
  last_pair_ = pair_used;
  if (fopt) return;
  if (dist && use_x) return;
  sgd_step(P, G, M, b_.n_params, sa, sh1, b_.step_ctr, cs_);
}

void SimpleCNNEngine::set_xgmi(std::shared_ptr<XgmiComm> x, std::vector<int> channels) {
  if (x) {
    if (channels.size() != buckets_.size())
      throw std::runtime_error("engine: one xgmi channel per bucket required");
    for (size_t i = 0; i < channels.size(); ++i) {
      if (channels[i] < 0 || channels[i] >= x->channels())
        throw std::runtime_error("engine: xgmi channel index out of range");
      for (size_t j = 0; j < i; ++j)
        if (channels[j] == channels[i]) throw std::runtime_error("engine: xgmi channels must be distinct");
    }
    if (x->world() != cfg_.world) throw std::runtime_error("engine: xgmi world size mismatch");
  }
  destroy_graph();
  xgmi_ = std::move(x);
  xch_ = xgmi_ ? channels : std::vector<int>(buckets_.size(), -1);
  // the in-launch all-reduce (dist_mode 2) takes at most one bucket per stage, a conv-stage
  // bucket, and a bounded number of role blocks (they wait at the head of the grid: <= 192
  // of its 512 resident slots, next to the fused reducers' <= 256)
  xar_plan_ok_ = false;
  pair_plan_ok_ = false;
  if (xgmi_ && sync_ok_for_xar()) {
    int per[2] = {0, 0}, nb = 0;
    for (int b = 0; b < (int)buckets_.size(); ++b) {
      ++per[stage_[b]];
      nb += xgmi_->blocks(xch_[b]);
    }
    xar_plan_ok_ = per[0] <= 1 && per[1] == 1 && nb <= 192;
    pair_plan_ok_ = per[0] <= 1 && per[1] == 1;
    if (std::getenv("DDP_AMD_XAR_DEBUG"))
      fprintf(stderr, "[ddp_amd] set_xgmi: stage buckets %d/%d, role blocks %d -> in-launch %d\n", per[0], per[1],
              nb, (int)xar_plan_ok_);
  }
}

void SimpleCNNEngine::step(int batch, int batch_stride) {
  const bool first = cfg_.momentum != 0.f && !momentum_started_;
  launch_step(batch, batch_stride, first);
  if (cfg_.momentum != 0.f) momentum_started_ = true;
  DDP_HIP_CHECK(hipGetLastError());
}

void SimpleCNNEngine::capture(int nsteps) {
  if (cfg_.momentum != 0.f && !momentum_started_)
    throw std::runtime_error("engine: run one eager step before capturing (momentum init)");
  destroy_graph();
  graph_heads_ = 0;
  capturing_ = true;
  DDP_HIP_CHECK(hipStreamBeginCapture(cs_, hipStreamCaptureModeRelaxed));
  try {
    if (overlap_active()) {
      // dist_mode 4: [fwd 0] [bwd 0] [pair 0 + fwd 1] [bwd 1] ... [bwd n-1] [pair n-1] - the
      // pair of every step but the last shares a launch with the next step's forward
      for (int i = 0; i < nsteps; ++i)
        launch_step(cfg_.max_batch, cfg_.max_batch, false, (i == 0 ? PART_FWD : PART_HEAD) | PART_BWD);
      launch_step(cfg_.max_batch, cfg_.max_batch, false, PART_AR);
    } else {
      for (int i = 0; i < nsteps; ++i) launch_step(cfg_.max_batch, cfg_.max_batch, false);
    }
  } catch (...) {
    capturing_ = false;
    hipGraph_t g = nullptr;
    hipStreamEndCapture(cs_, &g);
    if (g) hipGraphDestroy(g);
    throw;
  }
  capturing_ = false;
  DDP_HIP_CHECK(hipStreamEndCapture(cs_, &graph_));
  DDP_HIP_CHECK(hipGraphInstantiate(&graph_exec_, graph_, nullptr, nullptr, 0));
  // upload the exec's kernel-argument / node state now, on the engine stream, so its
  // first hipGraphLaunch (often inside a timed bracket) does not pay for it
  // (DDP_AMD_GRAPH_UPLOAD=0 skips it: A/B knob)
  const char* up = std::getenv("DDP_AMD_GRAPH_UPLOAD");
  if (!(up && up[0] == '0')) {
    DDP_HIP_CHECK(hipGraphUpload(graph_exec_, cs_));
    DDP_HIP_CHECK(hipStreamSynchronize(cs_));
  }
  graph_steps_ = nsteps;
}

void SimpleCNNEngine::replay() {
  if (!graph_exec_) throw std::runtime_error("engine: no captured graph");
  DDP_HIP_CHECK(hipGraphLaunch(graph_exec_, cs_));
}

}  // namespace ddp_amd
