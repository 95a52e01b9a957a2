// Host-only DDP bucket bookkeeping (no HIP, no torch): the part of the reducer
// that decides WHEN a bucket is complete.  Kept free of device code so it can be
// built and exercised under -fsanitize=address,undefined on the host
// (tests/native/test_bucket_state.cpp).
//
// Mirrors the contract of torch's C++ Reducer that the reference relies on
// (reference trigger train_ddp.py:34,199): each parameter's
// gradient is marked ready exactly once per iteration; the bucket whose last
// pending gradient arrives is launched immediately; finalize launches whatever
// was not launched (unused parameters) and starts the next iteration.
#pragma once

#include <stdexcept>
#include <string>
#include <vector>

namespace ddp_amd {

class BucketState {
 public:
  BucketState() = default;
  BucketState(std::vector<int> param_bucket, int nbuckets)
      : pbucket_(std::move(param_bucket)), init_pending_(nbuckets, 0) {
    if (nbuckets <= 0) throw std::invalid_argument("bucket state: need at least one bucket");
    for (int b : pbucket_) {
      if (b < 0 || b >= nbuckets) throw std::invalid_argument("bucket state: parameter mapped to bad bucket");
      init_pending_[b]++;
    }
    reset();
  }

  int num_params() const { return (int)pbucket_.size(); }
  int num_buckets() const { return (int)init_pending_.size(); }

  // Marks one parameter's gradient ready; returns the bucket that became complete
  // (to be launched now) or -1.
  int mark_ready(int param) {
    if (param < 0 || param >= num_params())
      throw std::out_of_range("bucket state: bad parameter index " + std::to_string(param));
    if (seen_[param])
      throw std::logic_error("bucket state: parameter " + std::to_string(param) +
                             " marked ready twice in one iteration");
    seen_[param] = 1;
    const int b = pbucket_[param];
    if (--pending_[b] == 0) return b;
    return -1;
  }

  void set_launched(int b) {
    if (b < 0 || b >= num_buckets()) throw std::out_of_range("bucket state: bad bucket index");
    if (launched_[b]) throw std::logic_error("bucket state: bucket launched twice");
    launched_[b] = 1;
  }
  bool launched(int b) const { return launched_.at(b) != 0; }
  int pending(int b) const { return pending_.at(b); }

  // Buckets still to launch at the end of backward, in bucket order.
  std::vector<int> unlaunched() const {
    std::vector<int> out;
    for (int b = 0; b < num_buckets(); ++b)
      if (!launched_[b]) out.push_back(b);
    return out;
  }

  void reset() {
    pending_ = init_pending_;
    launched_.assign(init_pending_.size(), 0);
    seen_.assign(pbucket_.size(), 0);
  }

 private:
  std::vector<int> pbucket_;
  std::vector<int> init_pending_, pending_;
  std::vector<char> launched_, seen_;
};

// torch DDP's size rule (compute_bucket_assignment_by_size, as used for the rebuilt
// buckets): walk parameters in gradient-ready order, close the current bucket as soon
// as its byte size reaches the limit; the first bucket's limit is first_cap_bytes, the
// rest use cap_bytes.  Returns, per bucket, the indices into `nbytes`.
inline std::vector<std::vector<int>> plan_buckets(const std::vector<long>& nbytes,
                                                  long first_cap_bytes, long cap_bytes) {
  if (first_cap_bytes <= 0 || cap_bytes <= 0) throw std::invalid_argument("plan_buckets: caps must be > 0");
  std::vector<std::vector<int>> out;
  std::vector<int> cur;
  long size = 0, limit = first_cap_bytes;
  for (int i = 0; i < (int)nbytes.size(); ++i) {
    if (nbytes[i] < 0) throw std::invalid_argument("plan_buckets: negative size");
    cur.push_back(i);
    size += nbytes[i];
    if (size >= limit) {
      out.push_back(cur);
      cur.clear();
      size = 0;
      limit = cap_bytes;
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}

}  // namespace ddp_amd
