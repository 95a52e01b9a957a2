// Native host runtime of ddp_amd: RCCL communicator, bucketed gradient reducer and
// the fused SimpleCNN training-step engine (with hipGraph capture).
// Plain HIP host API + RCCL; no torch types (the pybind layer adapts tensors).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "kernels/launchers.h"
#include "runtime/bucket_state.h"

#define DDP_HIP_CHECK(expr)                                                              \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__) + ": " #expr);  \
  } while (0)

#define DDP_NCCL_CHECK(expr)                                                             \
  do {                                                                                   \
    ncclResult_t _r = (expr);                                                            \
    if (_r != ncclSuccess)                                                               \
      throw std::runtime_error(std::string("RCCL error ") + ncclGetErrorString(_r) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__) + ": " #expr);  \
  } while (0)

namespace ddp_amd {

// Set from Python's atexit: once the interpreter is shutting down, destructors leak
// their HIP/RCCL handles instead of calling into a runtime that may be torn down.
void mark_exiting();
bool process_exiting();

// ---------------------------------------------------------------- RCCL communicator
// One communicator per process group, bootstrapped from an ncclUniqueId that rank 0
// creates and the Python layer distributes through the c10d TCPStore.
class Comm {
 public:
  static std::string new_unique_id();
  Comm(const std::string& uid, int rank, int world, int device);
  ~Comm();
  Comm(const Comm&) = delete;
  Comm& operator=(const Comm&) = delete;

  int rank() const { return rank_; }
  int world() const { return world_; }
  // dtype: 0 = f32, 1 = bf16, 2 = i32, 3 = i64, 4 = u8; op: 0 = sum, 1 = avg, 2 = max
  void all_reduce(void* buf, size_t count, int dtype, int op, hipStream_t s);
  void broadcast(void* buf, size_t count, int dtype, int root, hipStream_t s);
  void all_gather(const void* send, void* recv, size_t count, int dtype, hipStream_t s);
  void reduce_scatter(const void* send, void* recv, size_t count, int dtype, int op, hipStream_t s);
  // fp32 SUM of every rank's buffer times `scale` (RCCL's pre-multiplied sum: the multiply
  // happens inside the reduction - DDP's prescale-by-1/world without a separate pass)
  void all_reduce_premul(float* buf, size_t count, float scale, hipStream_t s);

 private:
  ncclComm_t comm_ = nullptr;
  int rank_ = 0, world_ = 1;
  std::vector<std::pair<float, ncclRedOp_t>> premul_;  // one op per scale, destroyed with the comm
};

// ---------------------------------------------------------------- direct xGMI all-reduce
// One channel per gradient bucket (a fixed [off, off + n) range of the gradient buffer);
// see xgmi.cpp / kernels/allreduce.hip.  Producers of a bucket must write it with
// system-scope stores (peers read it over xGMI right after the kernel boundary).
class XgmiComm {
 public:
  XgmiComm(int rank, int world, int device);
  ~XgmiComm();
  XgmiComm(const XgmiComm&) = delete;
  XgmiComm& operator=(const XgmiComm&) = delete;
  // grid_cap: most blocks for this channel's kernel (0: XGMI_GRID_CAP); a channel whose
  // all-reduce overlaps compute keeps its spinning grid small
  int add_channel(long off, long n, bool oneshot = false, int grid_cap = 0);
  int blocks(int channel) const { return ch_.at(channel).blocks; }
  std::string bus_id() const;  // PCI bus id of the device (ranks sharing a GPU compare these)
  bool oneshot(int channel) const { return ch_.at(channel).oneshot; }
  void set_data(float* data, long numel);
  std::string export_handles() const;
  void import_handles(const std::vector<std::string>& all);
  // publish: the bucket's producers used plain stores (module path): each block re-stores
  // its part system-scope before the entry barrier (no effect on one-shot channels, which
  // always copy the bucket to their stage buffer that way)
  // prescale (publish / one-shot only): my values times prescale before the rank-order sum
  void all_reduce(int channel, hipStream_t s, float scale = 1.f, bool publish = false, float prescale = 1.f);
  // the same, with SGD fused into the all-gather (see XgmiArgs)
  void all_reduce_sgd(int channel, hipStream_t s, const SgdArgs& sgd, float* params, float* mbuf,
                      const ShadowSet& sh, int* step_ctr, float scale = 1.f, bool publish = false,
                      float prescale = 1.f);
  // the kernel arguments all_reduce_sgd would launch with (the in-launch all-reduce role of
  // the conv backward runs the same body from them, with blocks(channel) blocks)
  XgmiArgs make_args(int channel, const SgdArgs& sgd, float* params, float* mbuf, const ShadowSet& sh,
                     int* step_ctr, float scale = 1.f, bool publish = false, float prescale = 1.f) const;
  // Two channels' all-reduces in ONE launch - the engine's dist_mode 3 kernel
  // (xgmi_allreduce_pair) as a standalone call: blocks [0, blocks(ch0)) run ch0, the rest
  // ch1, side by side, each with the fused SGD of all_reduce_sgd; the launch's last block
  // advances step_ctr.  (Multi-rank tests drive the production kernel through this.)
  void all_reduce_pair(int ch0, int ch1, hipStream_t s, const SgdArgs& sgd, float* params, float* mbuf,
                       const ShadowSet& sh, int* step_ctr);
  // != 0: a barrier timed out (result invalid) - the first failed channel's error word
  // (xgmi_error_code: block, peer, barrier)
  unsigned error_flags() const;
  void set_timeout(double seconds) { timeout_s_ = seconds; }
  int rank() const { return rank_; }
  int world() const { return world_; }
  int channels() const { return (int)ch_.size(); }
  long data_numel() const { return data_numel_; }

 private:
  struct Channel {
    long off = 0, n = 0, slice = 0;
    int blocks = 1;
    bool oneshot = false;
    float* stage_local = nullptr;
    unsigned* sig_local = nullptr;
    float* stage[XGMI_MAX_RANKS] = {};
    unsigned* sig[XGMI_MAX_RANKS] = {};
  };
  int rank_, world_, device_;
  float* data_ = nullptr;
  long data_numel_ = 0;
  char* data_base_ = nullptr;
  long data_off_ = 0;
  float* data_peer_[XGMI_MAX_RANKS] = {};
  std::vector<Channel> ch_;
  std::vector<void*> opened_;
  bool imported_ = false;
  double timeout_s_ = XGMI_DEFAULT_TIMEOUT_S;
  struct PairArgs {  // all_reduce_pair: device copies of the argument pairs, one per content
    XgmiArgs host[2];
    XgmiArgs* dev = nullptr;
  };
  std::vector<PairArgs> pair_cache_;
  int* pair_done_ = nullptr;  // the pair launch's last-block count (zeroed before each launch)
};

// ---------------------------------------------------------------- gradient reducer
// DDP gradient synchronisation for an arbitrary list of parameters (the module
// path).  Gradients live in one flat fp32 buffer cut into buckets; when the last
// gradient of a bucket is marked ready, an event is recorded on the compute
// stream, the comm stream waits for it and RCCL all-reduces the bucket, so
// communication of early buckets overlaps the rest of backward.  finalize()
// makes the compute stream wait for every bucket.  All of it is stream-ordered
// and therefore capturable into a hipGraph.
// comm == null with an XgmiComm (set_xgmi) reduces over the direct xGMI kernels only
// (e.g. ranks bootstrapped over gloo); world() comes from whichever data plane is set.
class Reducer {
 public:
  Reducer(std::shared_ptr<Comm> comm, float* flat_grad, std::vector<long> param_offsets,
          std::vector<long> param_numels, std::vector<int> param_bucket,
          std::vector<long> bucket_offsets, std::vector<long> bucket_numels, bool prescale);
  // bucket b all-reduced by xGMI channel channels[b] (its range must match the bucket)
  void set_xgmi(std::shared_ptr<XgmiComm> x, std::vector<int> channels);
  int world() const;
  ~Reducer();
  // grad_src == nullptr: gradient already written in place (bucket view)
  void mark_ready(int param, const float* grad_src, hipStream_t compute);
  void finalize(hipStream_t compute);
  void reset();
  int num_buckets() const { return (int)bucket_off_.size(); }
  long allreduce_calls() const { return calls_; }

 private:
  void launch_bucket(int b, hipStream_t compute);
  std::shared_ptr<Comm> comm_;
  std::shared_ptr<XgmiComm> xgmi_;
  std::vector<int> xch_;
  float* flat_;
  std::vector<long> poff_, pnum_;
  std::vector<int> pbucket_;
  std::vector<long> bucket_off_, bucket_num_;
  BucketState state_;
  std::vector<hipEvent_t> ready_, done_;
  hipStream_t comm_stream_ = nullptr;
  bool prescale_;
  long calls_ = 0;
};

// ---------------------------------------------------------------- fused SimpleCNN engine
struct EngineBuffers {
  // parameters / gradients: one flat fp32 buffer each (native layouts, see layers.py)
  float* params;
  float* grads;
  float* momentum;  // may be null (momentum == 0)
  long n_params;
  long off_w1, off_b1, off_w2, off_b2, off_wfc, off_bfc;
  // bf16 shadows
  bf16_t *w2_bf16, *w2t_bf16, *wfc_bf16, *wfc_frag;  // wfc_frag: FCFRAG order (conv2 fwd FC epilogue)
  // exact-fp32 engine (EngineConfig::f32): fp32 activations and the conv2 weight's
  // [tap][ci][co] fp32 copy (the data-gradient operand); the bf16 buffers are unused
  float *a2_f32 = nullptr, *dz2_f32 = nullptr, *w2t_f32 = nullptr;
  float* wfc_frag32 = nullptr;  // the fc weight in FCFRAG order, fp32 (the forward's fc operand)
  // activations / scratch (sized for max batch)
  bf16_t *a1, *a2, *dz2, *dz1;
  float *fc_part, *dlogits, *loss_rows, *loss_hist, *w2slab, *w1slab;
  int* step_ctr;
  unsigned char* xb;  // the step's batch, compact: u8 [max_batch][H*W] (fuse level 1)
  int* yb;            // its labels [max_batch]
  // in-launch hand-offs, zeroed by each step's forward (C1Src::zero_i32): [0, 256) the
  // fused conv backward's 8 arrival counters (32 ints apart), [256, 256 + fc blocks) the
  // level-2 dZ2 flags; level 3: [256] the fc backward's last-block counter (zeroed by the
  // forward too) and [L3_IMG_OFF, + max_batch) the forward's per-image arrival counters
  // (zeroed by the fc backward's last block); sync_err: wait-timeout word (0 = ok, 1 = dZ2
  // wait, 2 = reduction, 3 = level-3 forward wait)
  int* sync_flags = nullptr;
  int* sync_err = nullptr;
  // data
  const unsigned char* images;  // u8 [N][H*W]
  const int* labels;            // i32 [N]
  const int* idx;               // i32 epoch index list (nullptr: images / labels already in epoch order)
  int n_idx, n_rows;            // bounds for the clamped batch gather
};

constexpr int L3_FC_INTS = 32;                          // [SYNC_RED_INTS, + 32): fc last-block counter
constexpr int L3_IMG_OFF = SYNC_RED_INTS + L3_FC_INTS;  // per-image arrival counters

struct EngineConfig {
  int max_batch, H, W, C1, C2, NO;
  int pxt_fwd, pxt_dgrad, wgrad_rows;
  int world, rank;
  float lr, momentum, dampening, weight_decay;
  int nesterov, maximize;
  int force_allreduce;  // run the bucket all-reduces even at world size 1 (tests)
  // 0: 8 kernels (a1 materialised, separate cross-entropy kernel)
  // 1: 6 kernels - conv1 recomputed inside conv2 fwd/dgrad/wgrad from the uint8
  //    images (a1 never touches HBM) and cross-entropy folded into fc_bwd
  //    (4 per step with the fused optimizer: conv fwd, fc_bwd, conv bwd, grad_reduce)
  // (2: a level-1 variant with fc_bwd and the conv backward in one launch - measured
  //    slower than level 1 and removed in round 4)
  // 3: the fc backward leaves the critical path - the conv forward computes dZ2 itself
  //    (FwdDz: per-image in-launch wait, then dL and dZ2 from the fc weight fragments it
  //    holds) and the fc weight gradient + fused SGD (fc_bwd without dX, dL given) runs as
  //    a third role of the conv backward launch (single process, l3_fc_role: 2 kernels per
  //    step), or as a light kernel between the two (world size > 1: the fc bucket's
  //    all-reduce overlaps the conv backward).  bf16, where every forward block fits on the
  //    GPU at once (conv3x3_fwd_dz_fits); otherwise the level-1 chain
  int fuse_level = 0;
  // level 3, single process: 1 = the fc weight gradient as a role of the conv backward
  // launch, on blocks after every conv block (the resident slots they leave free); 0 = as
  // its own kernel (what world size > 1 runs).  (Placements 2 / 3 - right after the dgrad
  // blocks, on the dgrad blocks - measured slower and were removed in round 4.)
  int l3_fc_role = 1;
  // 1: single-process steps apply SGD in the epilogues of fc_bwd / grad_reduce (no
  //    separate optimizer kernel); 0: always the flat SGD kernel (equivalence tests)
  int fuse_opt = 1;
  // level 1: 0 = the conv backward recomputes conv1 from the compact batch; 1 = the
  // forward also stores a1 (own pixels) and the dgrad role reads its ReLU mask from it;
  // 2 = the wgrad role reads a1 tiles too
  int store_a1 = 0;
  // 1: exact fp32 operands everywhere (v_mfma_f32_16x16x4_f32 conv2, fp32 fc, fp32
  //    activations), the reference's precision; needs fuse_level 1 and store_a1 0
  int f32 = 0;
  // 1: the conv backward launch also reduces the split-K slabs + fused SGD (no separate
  //    grad_reduce kernel; level >= 1, needs sync_flags) while its reducers fit half the
  //    launch's resident capacity; 2: the whole capacity when the step has no bucket
  //    all-reduce on another stream (single process: the exact-fp32 step fuses too);
  //    0: grad_reduce kernel
  int fuse_reduce = 1;
  // 2: the fused conv backward's wgrad role runs two blocks per slab row, one per half of
  //    conv2's input channels (bf16; bit-identical slabs); 1: one block per row
  int wgrad_split = 1;
  // world size > 1, level 3 - how the backward meets the bucket all-reduces:
  //  2 = in-launch (xGMI, at most one bucket per stage): the fc weight gradient runs as the
  //      conv backward's fc role, and role blocks at the head of that same launch all-reduce
  //      each bucket (+ fused SGD) as soon as its gradients are final (BwdXar) - 2 kernels
  //      per step, no cross-stream edge; falls back to the bucket kernels on the compute
  //      stream when a condition fails (RCCL: mode 1)
  //  1 = fork: fc_bwd and the fc buckets' all-reduces on the comm stream, forked after the
  //      forward beside the conv backward (a graph branch), the conv buckets' all-reduces
  //      behind the conv backward
  //  3 = one stream (xGMI, the default): the fc role inside the conv backward as on one GPU,
  //      then ONE launch running both buckets' all-reduces (+ fused SGD) side by side on
  //      full grids (xgmi_allreduce_pair; the bucket kernels one by one when the plan has
  //      more buckets per stage) - 3 kernels per step, no cross-stream edge.  Fastest
  //      measured (forced world 1: 639k img/s vs 444k in-launch, 416k fork;
  //      profiles/r5_dist/README.md): the in-launch roles get too few blocks, a graph
  //      branch costs two cross-stream edges
  //  0 = the round-4 order (fc_bwd in front of the conv backward, all-reduces on ms_)
  //  4 = the step head (xGMI, bf16 level 3, pxt_fwd 1): mode 3's chain, but in a captured
  //      graph the pair launch of step k also carries step k + 1's forward (conv3x3.hip
  //      step_head_kernel: the forward blocks wait for each bucket's all-reduce blocks only
  //      where they first read its parameters) - 2 launches per step instead of 3; the step
  //      counter advances in the conv backward's fc role.  Same bits as mode 3.
  int dist_mode = 3;
};

// Gradient bucket of the engine's data plane: a [off, off + n) range of the flat gradient
// buffer.  Any plan works (DDP's bucket_cap_mb rule, sub-parameter chunks): a bucket is
// all-reduced as soon as every gradient in it is final - right after fc_bwd when it lies
// inside the fc parameters (overlapping the conv backward), after grad_reduce otherwise.
struct EngineBucket {
  long off, n;
};

class SimpleCNNEngine {
 public:
  SimpleCNNEngine(const EngineConfig& cfg, const EngineBuffers& buf, std::shared_ptr<Comm> comm,
                  std::vector<EngineBucket> buckets);
  ~SimpleCNNEngine();
  // eager launches of one full training step on the engine's compute stream
  void step(int batch, int batch_stride);
  void refresh_shadows();
  void set_lr(float lr) { cfg_.lr = lr; }
  // capture `nsteps` consecutive steps (batch = batch_stride = max_batch) into a graph
  void capture(int nsteps);
  void replay();
  bool has_graph() const { return graph_exec_ != nullptr; }
  int graph_steps() const { return graph_steps_; }
  void destroy_graph();
  hipStream_t stream() const { return cs_; }
  void synchronize();  // throws if a level-2 hand-off wait timed out
  // in-launch wait-timeout word (0 = ok, 1 = level-2 dZ2 wait, 2 = fused reduction,
  // 3 = level-3 forward's per-image wait); sticky
  int sync_error() const { return err_host_ ? __atomic_load_n(err_host_, __ATOMIC_ACQUIRE) : 0; }
  // whether a step of `batch` images runs the level-3 chain (fuse_level 3 and it applies)
  bool level3_active(int batch);
  // whether dist_mode 4's step head applies to a captured full-batch step
  bool overlap_active();
  // whether the last launched step reduced its weight-gradient slabs inside the conv
  // backward launch (false: separate grad_reduce kernel)
  bool last_fused_reduce() const { return last_fused_reduce_; }
  // whether the last launched step ran the level-3 chain (dZ2 in the forward, fc beside)
  bool last_level3() const { return last_level3_; }
  // ... and whether its fc weight gradient ran as a role of the conv backward launch
  bool last_fc_role() const { return last_fc_role_; }
  // ... and whether its bucket all-reduces ran inside the conv backward launch (dist_mode 2)
  bool last_xar() const { return last_xar_; }
  // ... or behind it in one launch for both buckets (dist_mode 3, xgmi_allreduce_pair)
  bool last_pair() const { return last_pair_; }
  // ... and whether its forward shared a launch with the previous step's pair (dist_mode 4)
  bool last_head() const { return last_head_; }
  // step-head launches (pair + next forward in one launch) in the captured graph
  int graph_heads() const { return graph_heads_; }
  void set_momentum_started(bool v) { momentum_started_ = v; }
  // bucket all-reduces over the direct xGMI kernel instead of RCCL: channels[b] serves
  // bucket b; set before capturing a graph
  void set_xgmi(std::shared_ptr<XgmiComm> x, std::vector<int> channels);
  int num_buckets() const { return (int)buckets_.size(); }
  int bucket_stage(int b) const { return stage_.at(b); }

 private:
  // parts of a step (dist_mode 4 splits steps inside a captured graph): the forward, the
  // backward, the bucket all-reduce pair; PART_HEAD = the forward merged with the PREVIOUS
  // step's pair (step_head_kernel)
  enum : unsigned { PART_FWD = 1, PART_BWD = 2, PART_AR = 4, PART_HEAD = 8, PART_ALL = 7 };
  void launch_step(int batch, int batch_stride, bool first_momentum_step, unsigned parts = PART_ALL);
  void launch_step_f32(int batch, int batch_stride, bool first_momentum_step);
  // enqueue the all-reduces of the buckets of `stage` (0: after fc_bwd, 1: after
  // grad_reduce) on the comm stream behind an event of the compute stream; with xGMI the
  // optimizer (+ the shadows in `sh`) runs inside each bucket's all-gather and the last
  // bucket of the step advances the step counter
  void launch_buckets(int stage, bool use_x, const SgdArgs& sa, float* M, const ShadowSet& sh);
  // compute stream waits for every launched stage
  void join_buckets();
  // the buckets of `stage` on stream s (no cross-stream ordering)
  void enqueue_buckets(int stage, bool use_x, hipStream_t s, const SgdArgs& sa, float* M, const ShadowSet& sh);
  // backward of a step whose forward is queued on cs_: the fc weight-gradient kernel `fc`
  // (may be empty: the fc role runs inside the conv backward), the conv backward `conv`
  // and, at world size > 1, the bucket all-reduces, ordered for the chain in use
  // (dist_mode 0 / 1); returns with every part of the step joined into cs_
  void schedule_backward(bool dist, bool fork, bool use_x, const std::function<void(hipStream_t)>& fc,
                         const std::function<void()>& conv, const SgdArgs& sa, float* M, const ShadowSet& sh);
  // dist_mode 2 with this bucket plan / data plane: the in-launch all-reduce's arguments for
  // this step (false: not applicable - the caller uses the bucket kernels)
  // the step head may defer a shadow of [off, off + n) to after the conv bucket's count
  bool late_shadow_ok(long off, long n) const;
  bool make_xar(BwdXar& xa, const SgdArgs& sa, float* M, const ShadowSet& sh);
  bool sync_ok_for_xar() const;
  EngineConfig cfg_;
  EngineBuffers b_;
  std::shared_ptr<Comm> comm_;
  std::shared_ptr<XgmiComm> xgmi_;
  std::vector<EngineBucket> buckets_;
  std::vector<int> stage_;  // 0: final after fc_bwd, 1: after grad_reduce
  std::vector<int> xch_;    // xGMI channel of each bucket
  int last_bucket_ = -1;    // the step's last collective (advances the step counter)
  bool stage_used_[2] = {false, false};
  hipStream_t cs_ = nullptr, ms_ = nullptr;
  hipEvent_t e_b0_, e_b1_, e_d0_, e_d1_, e_fwd_, e_fc_;
  std::vector<signed char> l3_fits_;  // per batch size: -1 unknown, 0 / 1
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t graph_exec_ = nullptr;
  int graph_steps_ = 0;
  bool momentum_started_ = false;
  bool last_fused_reduce_ = false;
  bool last_level3_ = false;
  bool last_fc_role_ = false;
  bool last_xar_ = false;
  bool last_pair_ = false;
  bool last_head_ = false;
  bool capturing_ = false;
  int graph_heads_ = 0;  // step-head launches in the captured graph (dist_mode 4)
  bool xar_plan_ok_ = false;  // set_xgmi: the bucket plan fits the in-launch all-reduce
  bool pair_plan_ok_ = false;  // ... and the one-launch pair of bucket kernels (dist_mode 3)
  struct XarArgs {
    XgmiArgs host[2];
    const XgmiArgs* dev = nullptr;
  };
  std::vector<XarArgs> xar_cache_;  // make_xar: device copies of the in-launch arguments
  hipStream_t xs_ = nullptr;        // ... and the stream their copies run on
  bool plain_stale_ = false;  // level-3 steps skipped the plain bf16 fc shadow
  int* err_host_ = nullptr;  // coherent host word behind b_.sync_err
};

}  // namespace ddp_amd
