// Host side of the direct xGMI all-reduce (kernels/allreduce.hip).
//
// Every rank registers its gradient buffer (any pointer into a hipMalloc allocation:
// the IPC handle names the allocation, the offset is exchanged next to it) and, per
// channel (= gradient bucket), allocates a stage buffer (2 x slice floats, call-parity
// double buffering) and uncached signal words.  The Python layer exchanges the opaque
// handle blobs through the c10d TCPStore; import_handles() maps every peer's buffers
// (hipIpcOpenMemHandle: xGMI peer mappings on a multi-GPU node, a second mapping of the
// same memory when several ranks share one GPU in tests).  all_reduce() is one kernel
// launch on the caller's stream, capturable in a hipGraph.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "runtime/runtime.h"

namespace ddp_amd {

namespace {
constexpr size_t kHandle = sizeof(hipIpcMemHandle_t);

void put_handle(std::string& out, void* base) {
  hipIpcMemHandle_t h;
  DDP_HIP_CHECK(hipIpcGetMemHandle(&h, base));
  out.append(reinterpret_cast<const char*>(&h), kHandle);
}
void put_i64(std::string& out, long long v) { out.append(reinterpret_cast<const char*>(&v), 8); }
}  // namespace

XgmiComm::XgmiComm(int rank, int world, int device) : rank_(rank), world_(world), device_(device) {
  if (world < 1 || world > XGMI_MAX_RANKS)
    throw std::runtime_error("xgmi: world size must be 1.." + std::to_string(XGMI_MAX_RANKS));
  if (rank < 0 || rank >= world) throw std::runtime_error("xgmi: bad rank");
  DDP_HIP_CHECK(hipSetDevice(device));
  // per-barrier spin bound (default XGMI_DEFAULT_TIMEOUT_S; set_timeout / this override)
  if (const char* e = std::getenv("DDP_AMD_XGMI_TIMEOUT_S")) timeout_s_ = std::atof(e);
}

XgmiComm::~XgmiComm() {
  if (process_exiting()) return;
  for (void* p : opened_) hipIpcCloseMemHandle(p);
  for (PairArgs& e : pair_cache_) hipFree(e.dev);
  if (pair_done_) hipFree(pair_done_);
  for (auto& c : ch_) {
    if (c.stage_local) hipFree(c.stage_local);
    if (c.sig_local) hipFree(c.sig_local);
  }
}

int XgmiComm::add_channel(long off, long n, bool oneshot, int grid_cap) {
  if (imported_) throw std::runtime_error("xgmi: add channels before import_handles");
  Channel c;
  c.off = off;
  c.n = n;
  c.oneshot = oneshot;
  c.slice = xgmi_slice(n, world_);
  c.blocks = xgmi_blocks(n, world_, oneshot);
  if (grid_cap > 0) c.blocks = std::min(c.blocks, grid_cap);
  // and a smaller grid, so the ranks' spinning blocks leave CUs to the others' kernels
  // (the kernel is block-strided; every rank must see the same value)
  if (const char* e = std::getenv("DDP_AMD_XGMI_GRID_CAP")) c.blocks = std::max(1, std::min(c.blocks, std::atoi(e)));
  if (c.blocks > XGMI_MAX_BLOCKS) throw std::runtime_error("xgmi: bucket too large for one channel");
  if (n * 4 >= (1L << 31)) throw std::runtime_error("xgmi: bucket over 2 GiB (32-bit buffer offsets)");
  const long stage = oneshot ? (n + 3) & ~3L : c.slice;  // per parity, whole quads
  DDP_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&c.stage_local), sizeof(float) * 2 * stage));
  DDP_HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&c.sig_local),
                                      sizeof(unsigned) * XGMI_SIG_WORDS, hipDeviceMallocUncached));
  DDP_HIP_CHECK(hipMemset(c.sig_local, 0, sizeof(unsigned) * XGMI_SIG_WORDS));
  DDP_HIP_CHECK(hipMemset(c.stage_local, 0, sizeof(float) * 2 * stage));
  DDP_HIP_CHECK(hipDeviceSynchronize());
  ch_.push_back(c);
  return (int)ch_.size() - 1;
}

void XgmiComm::set_data(float* data, long numel) {
  if (imported_) throw std::runtime_error("xgmi: set_data before import_handles");
  for (auto& c : ch_)
    if (c.off < 0 || c.off + c.n > numel) throw std::runtime_error("xgmi: channel outside the data buffer");
  data_ = data;
  data_numel_ = numel;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  DDP_HIP_CHECK(hipMemGetAddressRange(&base, &size, data));
  data_base_ = reinterpret_cast<char*>(base);
  data_off_ = reinterpret_cast<char*>(data) - data_base_;
}

std::string XgmiComm::bus_id() const {
  char buf[64] = {0};
  DDP_HIP_CHECK(hipDeviceGetPCIBusId(buf, sizeof(buf) - 1, device_));
  return std::string(buf);
}

std::string XgmiComm::export_handles() const {
  if (!data_) throw std::runtime_error("xgmi: set_data first");
  std::string out;
  put_i64(out, (long long)ch_.size());
  put_handle(out, data_base_);
  put_i64(out, data_off_);
  for (const auto& c : ch_) {
    put_handle(out, c.stage_local);
    put_handle(out, c.sig_local);
  }
  return out;
}

void XgmiComm::import_handles(const std::vector<std::string>& all) {
  if ((int)all.size() != world_) throw std::runtime_error("xgmi: need one handle blob per rank");
  const size_t want = 8 + kHandle + 8 + ch_.size() * 2 * kHandle;
  auto open = [&](const char* p) {
    hipIpcMemHandle_t h;
    std::memcpy(&h, p, kHandle);
    void* dev = nullptr;
    DDP_HIP_CHECK(hipIpcOpenMemHandle(&dev, h, hipIpcMemLazyEnablePeerAccess));
    opened_.push_back(dev);
    return reinterpret_cast<char*>(dev);
  };
  for (int r = 0; r < world_; ++r) {
    const std::string& b = all[r];
    if (b.size() != want) throw std::runtime_error("xgmi: handle blob size mismatch (channel layout differs)");
    long long nch = 0, off = 0;
    std::memcpy(&nch, b.data(), 8);
    if (nch != (long long)ch_.size()) throw std::runtime_error("xgmi: channel count differs across ranks");
    const char* p = b.data() + 8;
    std::memcpy(&off, p + kHandle, 8);
    if (r == rank_) {
      data_peer_[r] = data_;
    } else {
      data_peer_[r] = reinterpret_cast<float*>(open(p) + off);
    }
    p += kHandle + 8;
    for (auto& c : ch_) {
      if (r == rank_) {
        c.stage[r] = c.stage_local;
        c.sig[r] = c.sig_local;
      } else {
        c.stage[r] = reinterpret_cast<float*>(open(p));
        c.sig[r] = reinterpret_cast<unsigned*>(open(p + kHandle));
      }
      p += 2 * kHandle;
    }
  }
  imported_ = true;
}

void XgmiComm::all_reduce(int channel, hipStream_t s, float scale, bool publish, float prescale) {
  all_reduce_sgd(channel, s, SgdArgs{}, nullptr, nullptr, ShadowSet{}, nullptr, scale, publish, prescale);
}

XgmiArgs XgmiComm::make_args(int channel, const SgdArgs& sgd, float* params, float* mbuf, const ShadowSet& sh,
                              int* step_ctr, float scale, bool publish, float prescale) const {
  if (!imported_) throw std::runtime_error("xgmi: import_handles first");
  if (channel < 0 || channel >= (int)ch_.size()) throw std::runtime_error("xgmi: bad channel");
  const Channel& c = ch_[channel];
  if (prescale != 1.f && !publish && !c.oneshot)
    throw std::runtime_error("xgmi: prescale needs the publish pass (or a one-shot channel)");
  XgmiArgs a{};
  for (int r = 0; r < world_; ++r) {
    a.data[r] = data_peer_[r];
    a.stage[r] = c.stage[r];
    a.sig[r] = c.sig[r];
  }
  a.off = c.off;
  a.n = c.n;
  a.slice = c.slice;
  a.oneshot = c.oneshot ? 1 : 0;
  a.publish = publish ? 1 : 0;
  a.scale = scale;
  a.prescale = prescale;
  a.rank = rank_;
  a.world = world_;
  a.timeout_ticks = (unsigned long long)(timeout_s_ * 1e8);
  a.sgd = sgd;
  a.params = params;
  a.mbuf = mbuf;
  a.sh = sh;
  a.step_ctr = step_ctr;
  if (sgd.update && !params) throw std::runtime_error("xgmi: fused SGD needs the parameter buffer");
  return a;
}

void XgmiComm::all_reduce_sgd(int channel, hipStream_t s, const SgdArgs& sgd, float* params,
                              float* mbuf, const ShadowSet& sh, int* step_ctr, float scale, bool publish,
                              float prescale) {
  const XgmiArgs a = make_args(channel, sgd, params, mbuf, sh, step_ctr, scale, publish, prescale);
  xgmi_allreduce(a, ch_[channel].blocks, s);
  DDP_HIP_CHECK(hipGetLastError());
}

void XgmiComm::all_reduce_pair(int ch0, int ch1, hipStream_t s, const SgdArgs& sgd, float* params, float* mbuf,
                               const ShadowSet& sh, int* step_ctr) {
  if (ch0 == ch1) throw std::runtime_error("xgmi: all_reduce_pair needs two distinct channels");
  XgmiArgs pair[2];
  std::memset(static_cast<void*>(pair), 0, sizeof(pair));  // (compared bytewise below)
  pair[0] = make_args(ch0, sgd, params, mbuf, sh, nullptr);
  pair[1] = make_args(ch1, sgd, params, mbuf, sh, nullptr);
  const XgmiArgs* dev = nullptr;
  for (const PairArgs& e : pair_cache_)
    if (std::memcmp(e.host, pair, sizeof(pair)) == 0) dev = e.dev;
  if (!dev) {
    PairArgs e;
    std::memcpy(static_cast<void*>(e.host), pair, sizeof(pair));
    DDP_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&e.dev), sizeof(pair)));
    DDP_HIP_CHECK(hipMemcpy(e.dev, pair, sizeof(pair), hipMemcpyHostToDevice));
    pair_cache_.push_back(e);
    dev = e.dev;
  }
  if (!pair_done_) DDP_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&pair_done_), sizeof(int)));
  DDP_HIP_CHECK(hipMemsetAsync(pair_done_, 0, sizeof(int), s));
  BwdXar x;
  x.args = dev;
  x.nblk0 = ch_[ch0].blocks;
  x.nblk1 = ch_[ch1].blocks;
  x.xar_done = pair_done_;
  x.step_ctr = step_ctr;
  xgmi_allreduce_pair(x, s);
  DDP_HIP_CHECK(hipGetLastError());
}

unsigned XgmiComm::error_flags() const {
  for (const auto& c : ch_) {
    unsigned v = 0;
    DDP_HIP_CHECK(hipMemcpy(&v, c.sig_local + XGMI_ERR_OFF, sizeof(v), hipMemcpyDeviceToHost));
    if (v) return v;  // the first failed channel's code (codes must not be OR-ed together)
  }
  return 0;
}

}  // namespace ddp_amd
