// Bucketed DDP gradient reducer (MI355X equivalent of torch's C++ DDP Reducer,
// SURVEY.md §2.2 N3; reference trigger: DDP(model) at train_ddp.py:34 and
// loss.backward() at train_ddp.py:199).
//
// Semantics kept from the reference DDP: gradients are averaged as
// sum_r(g_r * 1/ws) (prescale, then SUM - per bucket at launch, or per parameter in
// mark_ready when constructed with prescale), buckets are launched as soon as their
// last gradient is ready (overlapping backward), and the optimizer only runs
// after every bucket finished.  What differs: buckets are views of one flat fp32
// gradient buffer owned by the model, the all-reduce runs on a dedicated HIP
// stream ordered by hipEvents (capturable), and the collective is RCCL directly - or,
// per bucket, the direct xGMI kernel (set_xgmi; two-shot with an in-kernel publish pass,
// since autograd produced the gradients with plain stores).
#include <cstdlib>

#include "runtime/runtime.h"

namespace ddp_amd {

Reducer::Reducer(std::shared_ptr<Comm> comm, float* flat_grad, std::vector<long> param_offsets,
                 std::vector<long> param_numels, std::vector<int> param_bucket,
                 std::vector<long> bucket_offsets, std::vector<long> bucket_numels, bool prescale)
    : comm_(std::move(comm)),
      flat_(flat_grad),
      poff_(std::move(param_offsets)),
      pnum_(std::move(param_numels)),
      pbucket_(std::move(param_bucket)),
      bucket_off_(std::move(bucket_offsets)),
      bucket_num_(std::move(bucket_numels)),
      prescale_(prescale) {
  const int nb = (int)bucket_off_.size();
  if (poff_.size() != pnum_.size() || poff_.size() != pbucket_.size() || bucket_num_.size() != (size_t)nb)
    throw std::runtime_error("reducer: inconsistent parameter / bucket tables");
  state_ = BucketState(pbucket_, nb);
  ready_.resize(nb);
  done_.resize(nb);
  for (int b = 0; b < nb; ++b) {
    DDP_HIP_CHECK(hipEventCreateWithFlags(&ready_[b], hipEventDisableTiming));
    DDP_HIP_CHECK(hipEventCreateWithFlags(&done_[b], hipEventDisableTiming));
  }
  DDP_HIP_CHECK(hipStreamCreateWithFlags(&comm_stream_, hipStreamNonBlocking));
}

Reducer::~Reducer() {
  // The comm stream is intentionally never destroyed (torch does the same with its
  // streams): torch's caching allocators may still record events on it later.
  if (process_exiting()) return;
  for (auto e : ready_) hipEventDestroy(e);
  for (auto e : done_) hipEventDestroy(e);
}

void Reducer::reset() { state_.reset(); }

void Reducer::set_xgmi(std::shared_ptr<XgmiComm> x, std::vector<int> channels) {
  if (x && channels.size() != bucket_off_.size())
    throw std::runtime_error("reducer: one xgmi channel per bucket required");
  if (x)
    for (int ch : channels)
      if (ch < 0 || ch >= x->channels()) throw std::runtime_error("reducer: xgmi channel out of range");
  xgmi_ = std::move(x);
  xch_ = std::move(channels);
}

int Reducer::world() const {
  if (xgmi_) return xgmi_->world();
  return comm_ ? comm_->world() : 1;
}

void Reducer::launch_bucket(int b, hipStream_t compute) {
  DDP_HIP_CHECK(hipEventRecord(ready_[b], compute));
  DDP_HIP_CHECK(hipStreamWaitEvent(comm_stream_, ready_[b], 0));
  const float inv = 1.f / (float)world();
  if (xgmi_ && xgmi_->world() > 1) {
    // torch DDP's averaging: every rank's gradient times 1/world (inside the kernel's publish
    // pass, no extra launch), then the fixed rank-order SUM
    xgmi_->all_reduce(xch_[b], comm_stream_, 1.f, true, prescale_ ? 1.f : inv);
    ++calls_;
  } else if (comm_ && comm_->world() > 1) {
    // DDP's prescale by 1/world: scale pass + SUM (torch DDP's own order).  RCCL's
    // pre-multiplied SUM folds the scale into the reduction (no extra pass) but is opt-in
    // (DDP_AMD_RCCL_PREMUL=1, and only for 16-byte-aligned buckets of whole quads): it was seen
    // leaving a non-multiple-of-4 tail unscaled at one rank, and no multi-rank run has pinned
    // its bits against scale + SUM; producers that prescaled already SUM
    static const bool premul = [] { const char* e = std::getenv("DDP_AMD_RCCL_PREMUL"); return e && e[0] == '1'; }();
    if (prescale_) {
      comm_->all_reduce(flat_ + bucket_off_[b], (size_t)bucket_num_[b], 0, 0, comm_stream_);
    } else if (premul && bucket_num_[b] % 4 == 0 && bucket_off_[b] % 4 == 0) {
      comm_->all_reduce_premul(flat_ + bucket_off_[b], (size_t)bucket_num_[b], inv, comm_stream_);
    } else {
      scale_copy(flat_ + bucket_off_[b], flat_ + bucket_off_[b], bucket_num_[b], inv, comm_stream_);
      comm_->all_reduce(flat_ + bucket_off_[b], (size_t)bucket_num_[b], 0, 0, comm_stream_);
    }
    ++calls_;
  }
  DDP_HIP_CHECK(hipEventRecord(done_[b], comm_stream_));
  state_.set_launched(b);
}

void Reducer::mark_ready(int param, const float* grad_src, hipStream_t compute) {
  if (param < 0 || param >= (int)poff_.size()) throw std::runtime_error("reducer: bad param index");
  float* dst = flat_ + poff_[param];
  const float scale = prescale_ ? 1.f / (float)world() : 1.f;
  if (grad_src != nullptr && grad_src != dst) scale_copy(dst, grad_src, pnum_[param], scale, compute);
  else if (scale != 1.f) scale_copy(dst, dst, pnum_[param], scale, compute);
  const int b = state_.mark_ready(param);
  if (b >= 0) launch_bucket(b, compute);
}

void Reducer::finalize(hipStream_t compute) {
  for (int b : state_.unlaunched()) launch_bucket(b, compute);  // unused params: reduce what is there
  for (int b = 0; b < (int)bucket_off_.size(); ++b) DDP_HIP_CHECK(hipStreamWaitEvent(compute, done_[b], 0));
  reset();
}

}  // namespace ddp_amd
