// Direct (all-to-all) two-shot SUM all-reduce over xGMI for the DDP gradient buckets.
//
// Why not only RCCL: an 8x MI355X node is a full mesh of point-to-point xGMI links
// (7 per GPU).  A ring all-reduce moves 2(N-1)/N of the bucket over ONE link per step;
// the direct algorithm below moves each byte over its own link, all 7 links at once,
// in two hops, and runs as ONE kernel inside the step's hipGraph (no proxy thread, no
// protocol selection).  SimpleCNN's buckets are 2.0 MB and 75 KB (SURVEY.md §2.6
// I6/I7), i.e. latency-bound: two cross-GPU barriers + 2 x (bucket / N) per link.
//
//   B0  entry barrier: every rank's gradient bucket is final
//   RS  rank r pulls its slice r from all peers (system-scope loads over xGMI), sums in
//       FIXED rank order 0..N-1 (bitwise identical on every rank), writes the reduced
//       slice to its stage buffer (parity = call number & 1)
//   B1  every rank finished RS (so nobody reads any rank's gradient buffer any more)
//   AG  rank r pulls every peer's reduced slice from its stage buffer into its own
//       gradient buffer (local stores)
//
// Pull-only: no GPU ever writes another GPU's memory, so each GPU's own L2 stays
// coherent for its own buffers.  Everything a peer reads is produced with system-scope
// (write-through) stores and read with system-scope loads, and every storing wave
// drains its stores (s_waitcnt vmcnt(0)) before the block's flag store.  The stage
// buffer is double-buffered by call parity, which removes the exit barrier: call k+2
// reuses call k's stage only after every rank passed call k+1's B0.
//
// One-shot variant (XgmiArgs::oneshot, small buckets): every rank publishes its whole
// bucket to its stage buffer (parity-double-buffered), ONE barrier, then every rank pulls
// all N published buckets and sums them in fixed rank order - each rank computes the
// full result itself (bitwise identical everywhere), trading N x the bytes for one fewer
// cross-GPU barrier, which wins when the bucket is a few tens of KB (SimpleCNN's
// 75 KB conv bucket).  Stage reuse: call k+2 rewrites parity k's stage only after every
// rank passed call k+1's barrier, i.e. finished reading call k.
//
// Barriers are per block: block b of every rank handles the same element range of every
// slice, and only ever waits for block b of its peers.  Flags are monotonic per-block counters in
// uncached memory; every spin is bounded (XgmiArgs::timeout_ticks of the 100 MHz clock):
// on timeout the block sets the error word and stops waiting, so a broken peer makes
// the result wrong (detected by the host) instead of hanging the GPU.
#include "kernels/xgmi_body.h"

namespace ddp_amd {

__global__ __launch_bounds__(XGMI_THREADS) void xgmi_allreduce_kernel(XgmiArgs a) {
  __shared__ unsigned s_sh[2];
  // the arguments into LDS first: the body indexes the peer pointers by rank, which made the
  // compiler copy the by-value struct to scratch
  __shared__ __attribute__((aligned(16))) int s_raw[sizeof(XgmiArgs) / 4];
  {
    const int* src = reinterpret_cast<const int*>(&a);
    for (int i = threadIdx.x; i < (int)(sizeof(XgmiArgs) / 4); i += XGMI_THREADS) s_raw[i] = src[i];
  }
  __syncthreads();
  DDP_STAMP(STAMP_K_XGMI, 0);
  xgmi_allreduce_body(*reinterpret_cast<const XgmiArgs*>(s_raw), (int)blockIdx.x, (int)gridDim.x, s_sh);
  DDP_STAMP(STAMP_K_XGMI, 7);
}

// dist_mode 3: both buckets in one launch (BwdXar arguments in device memory, copied to LDS:
// from global memory inside the body every field was re-loaded after each store)
__global__ __launch_bounds__(XGMI_THREADS) void xgmi_allreduce_pair_kernel(BwdXar x) {
  __shared__ unsigned s_sh[2];
  __shared__ __attribute__((aligned(16))) int s_raw[sizeof(XgmiArgs) / 4];  // XgmiArgs has initializers
  const int nx = x.nblk0 + x.nblk1;
  const int k = (int)blockIdx.x < x.nblk0 ? 0 : 1;
  {
    const int* src = reinterpret_cast<const int*>(x.args + k);
    for (int i = threadIdx.x; i < (int)(sizeof(XgmiArgs) / 4); i += XGMI_THREADS) s_raw[i] = src[i];
  }
  __syncthreads();
  const XgmiArgs& s_xa = *reinterpret_cast<const XgmiArgs*>(s_raw);
  DDP_STAMP(STAMP_K_XGMI, 0);
  if (k == 0) xgmi_allreduce_body(s_xa, (int)blockIdx.x, x.nblk0, s_sh);
  else xgmi_allreduce_body(s_xa, (int)blockIdx.x - x.nblk0, x.nblk1, s_sh);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  DDP_STAMP(STAMP_K_XGMI, 7);
  if (threadIdx.x == 0) {
    // relaxed: the count only finds the last block (the step counter it advances is read by
    // later kernels).  An agent-scope acq_rel here compiled to buffer_wbl2 sc1 + buffer_inv
    // sc1 - an L2 write-back and invalidate of the XCD for each of the 275 blocks, ~3-5 us
    // at the end of every multi-GPU step.
    const int old = __hip_atomic_fetch_add(x.xar_done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == nx - 1 && x.step_ctr) x.step_ctr[0] += 1;
  }
}

void xgmi_allreduce_pair(const BwdXar& x, hipStream_t s) {
  hipLaunchKernelGGL(xgmi_allreduce_pair_kernel, dim3(x.nblk0 + x.nblk1), dim3(XGMI_THREADS), 0, s, x);
}

long xgmi_slice(long n, int world) { return (((n + world - 1) / world) + 3) & ~3L; }

int xgmi_blocks(long n, int world, bool oneshot) {
  const long quads = ((oneshot ? n : xgmi_slice(n, world)) + 3) / 4;
  long b = (quads + XGMI_THREADS - 1) / XGMI_THREADS;
  if (b > XGMI_GRID_CAP) b = XGMI_GRID_CAP;
  return (int)(b < 1 ? 1 : b);
}

void xgmi_allreduce(const XgmiArgs& a, int blocks, hipStream_t s) {
  hipLaunchKernelGGL(xgmi_allreduce_kernel, dim3(blocks), dim3(XGMI_THREADS), 0, s, a);
}

DDP_STAMPS_SETTER(stamps_set_allreduce)

}  // namespace ddp_amd
