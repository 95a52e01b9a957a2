// Host-only unit test of the reducer's bucket bookkeeping, built with
// -fsanitize=address,undefined by tests/test_native_host.py.
#include <cstdio>
#include <cstdlib>
#include <stdexcept>

#include "runtime/bucket_state.h"

using ddp_amd::BucketState;
using ddp_amd::plan_buckets;

#define CHECK(c)                                                    \
  do {                                                              \
    if (!(c)) {                                                     \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                 \
    }                                                               \
  } while (0)

template <class E, class F>
static bool throws(F f) {
  try {
    f();
  } catch (const E&) {
    return true;
  }
  return false;
}

int main() {
  // SimpleCNN in gradient-ready order: fl.bias, fl.weight, net.2.bias, net.2.weight, net.0.bias, net.0.weight
  const std::vector<long> bytes = {40, 2007040, 256, 73728, 128, 1152};
  auto plan = plan_buckets(bytes, 1 << 20, 25 << 20);
  CHECK(plan.size() == 2);
  CHECK((plan[0] == std::vector<int>{0, 1}));
  CHECK((plan[1] == std::vector<int>{2, 3, 4, 5}));
  // tiny caps: one bucket per tensor; huge caps: a single bucket
  CHECK(plan_buckets(bytes, 1, 1).size() == bytes.size());
  CHECK(plan_buckets(bytes, 1L << 40, 1L << 40).size() == 1);
  CHECK(plan_buckets({}, 1, 1).empty());
  CHECK(throws<std::invalid_argument>([] { plan_buckets({1}, 0, 1); }));

  BucketState st({0, 0, 1, 1, 1, 1}, 2);
  for (int it = 0; it < 3; ++it) {
    CHECK(st.mark_ready(0) == -1);
    CHECK(st.mark_ready(1) == 0);
    st.set_launched(0);
    CHECK(st.pending(1) == 4);
    CHECK(st.mark_ready(5) == -1);
    CHECK(st.mark_ready(3) == -1);
    CHECK(st.mark_ready(2) == -1);
    CHECK(st.mark_ready(4) == 1);
    st.set_launched(1);
    CHECK(st.unlaunched().empty());
    st.reset();
  }
  // unused parameter: finalize must launch the incomplete bucket
  CHECK(st.mark_ready(0) == -1);
  CHECK(st.mark_ready(1) == 0);
  st.set_launched(0);
  CHECK((st.unlaunched() == std::vector<int>{1}));
  // misuse is an error, never silent corruption
  CHECK(throws<std::logic_error>([&] { st.mark_ready(0); }));
  CHECK(throws<std::logic_error>([&] { st.set_launched(0); }));
  CHECK(throws<std::out_of_range>([&] { st.mark_ready(6); }));
  CHECK(throws<std::out_of_range>([&] { st.mark_ready(-1); }));
  CHECK(throws<std::invalid_argument>([] { BucketState({0, 2}, 2); }));
  std::printf("bucket_state: all checks passed\n");
  return 0;
}
