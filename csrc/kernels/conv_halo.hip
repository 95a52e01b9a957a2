// Stride-1 3x3 forward convolution with an LDS halo tile (ResNet-18's 56/28/14-wide
// 3x3 layers; conv_gemm_plan picks it, conv_gemm_fwd launches it).
//
// The implicit GEMM of conv_gemm.hip gathers the B operand per K-step (one tap x 32
// input channels), so every input pixel is fetched from L2 once per tap - 9x.  Here a
// block owns R full output rows of one image (R*W <= 128 pixels) and, per 32-channel
// chunk, stages the (R+2) x (W+2) input halo into LDS once; the nine taps of the chunk
// then read their B fragments straight from the halo at a tap offset.  Weights are
// staged one kernel row (3 taps x [BC][32]) per barrier, so each barrier covers three
// MFMA K-steps.  The next chunk's halo is loaded into registers at the chunk's first
// barrier step and stored to the other halo buffer before the chunk switch.
//
// Same MFMA tiling as conv_gemm_fwd_kernel (4 waves = 2 co x 2 px, 16x16x32 bf16,
// 128-pixel column tile of which R*W are live), same epilogues: bf16 NHWC store with the
// per-block BatchNorm sum / sum-of-squares partials, or fp32 split-K partials for
// splitk_reduce.  K splits run over channel chunks (grid.z).
#include <stdexcept>

#include "kernels/bn_affine.h"
#include "kernels/common.h"
#include "kernels/launchers.h"

namespace ddp_amd {

constexpr int HL_KS = 32;   // channels per chunk (one MFMA K-step per tap)
constexpr int HL_RS = 48;   // LDS row stride (elements) per pixel / weight row: 24 dwords == 8 (mod 16)
constexpr int HL_BP = 128;  // pixel columns of the MFMA tile
constexpr int HL_MAXPX = 232;     // largest halo: (R+2) x (W+2) = 4 x 58 at W = 56 (R = 2)

// AFF: X is the producer conv's RAW output; the halo staging applies its BatchNorm + ReLU
// (BnAffine, bitwise bn_apply's value; the zero padding stays zero) - the producer's
// bn_apply pass disappears.  The per-channel sc / sh table sits in LDS (4 KB).
// GW: the image width as a template constant (56 / 28 / 14 for ResNet-18's layers; 0 =
// runtime) - the halo index divisions and the tap offsets then fold (the per-dispatch SQ
// counters showed ~10 VALU instructions per MFMA in this kernel, profiles/r4_resnet/pmc)
template <int BC, int BP, bool STATS, bool PART, bool AFF = false, int GW = 0>
__global__ __launch_bounds__(256) void conv3x3s1_halo_fwd_kernel(ConvGeom g, const bf16_t* __restrict__ X,
                                                                 const bf16_t* __restrict__ Wt,
                                                                 bf16_t* __restrict__ Y,
                                                                 float* __restrict__ stats,
                                                                 float* __restrict__ part, int R,
                                                                 int chunks_per_split, BnAffine bn) {
  constexpr int TCO = BC / 32, TPX = BP / 32;
  constexpr int HCH = (HL_MAXPX * 4 + 255) / 256;  // 16-B halo chunks per thread
  // weights of one kernel row (3 taps) per K-step: 3 MFMA K-steps between barriers
  __shared__ __attribute__((aligned(16))) bf16_t sA[2][3 * BC * HL_RS];
  __shared__ __attribute__((aligned(16))) bf16_t sH[2][HL_MAXPX * HL_RS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wco = wave >> 1, wpx = wave & 1;
  const int W = GW ? GW : g.W, H = g.H, Cin = g.Cin;
  const int RG = (H + R - 1) / R;
  const int3 bk = xcd_block3();  // XCD-contiguous block order
  const int n_ = bk.x / RG, rg = bk.x - n_ * RG;
  const int oh0 = rg * R;
  const int co0 = bk.y * BC;
  const int HW2 = W + 2, HR = R + 2, HPX = HR * HW2;
  const int NPX = R * W;
  const int nch = Cin / HL_KS;
  const int c_beg = bk.z * chunks_per_split;
  const int c_end = min(nch, c_beg + chunks_per_split);
  const int KWC = 9 * Cin;

  // halo chunk h of this thread: pixel hp = (tid + 256u) / 4, quarter (8 channels) = & 3
  // AFF: the loaded chunks that lie inside the image (hin) and the raw BatchNorm parameters
  // of this thread's 8 channels of the chunk travel with the halo registers
  unsigned hin = 0;
  BnRaw8 braw;
  auto load_halo = [&](int ch, bf16x8* rh) {
    if constexpr (AFF) hin = 0;
#pragma unroll
    for (int u = 0; u < HCH; ++u) {
      const int e = tid + 256 * u;
      const int hp = e >> 2, qq = e & 3;
      rh[u] = zero8();
      if (hp < HPX) {
        const int hr = hp / HW2, hc = hp - hr * HW2;
        const int ih = oh0 - 1 + hr, iw = hc - 1;
        if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) {
          rh[u] = ld8(X + (((long)n_ * H + ih) * W + iw) * Cin + ch * HL_KS + qq * 8);
          if constexpr (AFF) hin |= 1u << u;
        }
      }
    }
    if constexpr (AFF) braw = bn_raw8(bn.invstd, bn.gamma, bn.mean, bn.beta, ch * HL_KS + (tid & 3) * 8);
  };
  auto store_halo = [&](int buf, const bf16x8* rh, int ch) {
    (void)ch;
    float sc[8], sh[8];
    if constexpr (AFF) bn_affine8_of(braw, sc, sh);  // this thread's 8 channels (qq = tid & 3)
#pragma unroll
    for (int u = 0; u < HCH; ++u) {
      const int e = tid + 256 * u;
      const int hp = e >> 2, qq = e & 3;
      if (hp < HPX) {
        bf16x8 v = rh[u];
        if constexpr (AFF) {
          if ((hin >> u) & 1u) v = bn_relu8(v, sc, sh);
        }
        *reinterpret_cast<bf16x8*>(&sH[buf][hp * HL_RS + qq * 8]) = v;
      }
    }
  };
  // weight rows of kernel row kh: sA row = t * BC + co (t = kw), 32 channels each
  constexpr int WCH = 3 * BC * 4 / 256;  // 16-B weight chunks per thread
  auto load_w = [&](int ch, int kh, bf16x8* ra) {
#pragma unroll
    for (int u = 0; u < WCH; ++u) {
      const int c = tid + u * 256;
      const int row = c >> 2, off = (c & 3) * 8;
      const int t = row / BC, co = row - t * BC;
      ra[u] = ld8(Wt + (long)(co0 + co) * KWC + (kh * 3 + t) * Cin + ch * HL_KS + off);
    }
  };
  auto store_w = [&](int buf, const bf16x8* ra) {
#pragma unroll
    for (int u = 0; u < WCH; ++u) {
      const int c = tid + u * 256;
      *reinterpret_cast<bf16x8*>(&sA[buf][(c >> 2) * HL_RS + (c & 3) * 8]) = ra[u];
    }
  };

  // per-lane halo base of each pixel column tile (tap offset added per K-step)
  const int kofs = 8 * (lane >> 4), col = lane & 15;
  int hbase[TPX];
#pragma unroll
  for (int j = 0; j < TPX; ++j) {
    const int p = wpx * (BP / 2) + 16 * j + col;
    const int r = p / W, c = p - r * W;
    hbase[j] = p < NPX ? r * HW2 + c : 0;  // padding pixels read a valid row, masked later
  }
  f32x4 acc[TCO][TPX];
#pragma unroll
  for (int i = 0; i < TCO; ++i)
#pragma unroll
    for (int j = 0; j < TPX; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  bf16x8 ra[WCH], rh[HCH];
  if (c_beg < c_end) {
    load_halo(c_beg, rh);
    load_w(c_beg, 0, ra);
    store_halo(0, rh, c_beg);
    store_w(0, ra);
  }
  __syncthreads();
  int step = 0;
  for (int ch = c_beg; ch < c_end; ++ch) {
    const int hb = (ch - c_beg) & 1;
    const bool next_chunk = ch + 1 < c_end;
    for (int kh = 0; kh < 3; ++kh, ++step) {  // one kernel row (3 taps) per barrier
      const int cur = step & 1;
      const bool last = kh == 2;
      const bool more = !last || next_chunk;
      if (more) load_w(last ? ch + 1 : ch, last ? 0 : kh + 1, ra);
      if (kh == 0 && next_chunk) load_halo(ch + 1, rh);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int toff = kh * HW2 + kw;
        bf16x8 a[TCO], b[TPX];
#pragma unroll
        for (int i = 0; i < TCO; ++i)
          a[i] = *reinterpret_cast<const bf16x8*>(&sA[cur][(kw * BC + wco * (BC / 2) + 16 * i + col) * HL_RS + kofs]);
#pragma unroll
        for (int j = 0; j < TPX; ++j)
          b[j] = *reinterpret_cast<const bf16x8*>(&sH[hb][(hbase[j] + toff) * HL_RS + kofs]);
#pragma unroll
        for (int i = 0; i < TCO; ++i)
#pragma unroll
          for (int j = 0; j < TPX; ++j) acc[i][j] = mfma16(a[i], b[j], acc[i][j]);
      }
      if (last && next_chunk) store_halo(hb ^ 1, rh, ch + 1);  // buffer hb^1 was last read a chunk ago
      if (more) store_w(cur ^ 1, ra);
      __syncthreads();
    }
  }

  // ---- epilogue (block-local pixel p -> output row oh0 + p / W, column p % W)
  const int Ptot = g.N * g.OH * g.OW;
  float csum[TCO][4], csq[TCO][4];
#pragma unroll
  for (int i = 0; i < TCO; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) csum[i][r] = csq[i][r] = 0.f;
#pragma unroll
  for (int j = 0; j < TPX; ++j) {
    const int p = wpx * (BP / 2) + 16 * j + col;
    const int r = p / W;
    const int oh = oh0 + r;
    const bool ok = p < NPX && oh < g.OH;
    const long P = ((long)n_ * g.OH + oh) * g.OW + (p - r * W);
#pragma unroll
    for (int i = 0; i < TCO; ++i) {
      const int co = co0 + wco * (BC / 2) + 16 * i + 4 * (lane >> 4);
      if (PART) {
        if (ok)
          *reinterpret_cast<float4*>(part + ((long)bk.z * Ptot + P) * g.Cout + co) =
              make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
        continue;
      }
      const uint2 pk = pack4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      if (ok) *reinterpret_cast<uint2*>(Y + P * g.Cout + co) = pk;
      if (STATS) {
        float q[4];
        unpack4(pk, q);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const float x = ok ? q[rr] : 0.f;
          csum[i][rr] += x;
          csq[i][rr] = fmaf(x, x, csq[i][rr]);
        }
      }
    }
  }
  if (STATS && !PART) {
    // the weight tiles are dead after the K loop: their LDS holds the per-wave partials
    // (keeps two blocks per CU resident)
    float (*s_st)[2][BC] = reinterpret_cast<float (*)[2][BC]>(&sA[0][0]);
#pragma unroll
    for (int i = 0; i < TCO; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const float a = sum16(csum[i][rr]), b = sum16(csq[i][rr]);
        if (col == 0) {
          const int cl = wco * (BC / 2) + 16 * i + 4 * (lane >> 4) + rr;
          s_st[wpx][0][cl] = a;
          s_st[wpx][1][cl] = b;
        }
      }
    __syncthreads();
    for (int c = tid; c < BC; c += 256) {
      float* dst = stats + (long)bk.x * 2 * g.Cout;
      st_wt(dst + co0 + c, s_st[0][0][c] + s_st[1][0][c]);
      st_wt(dst + g.Cout + co0 + c, s_st[0][1][c] + s_st[1][1][c]);
    }
  }
}

// ---------------------------------------------------------------- data gradient
// Stride-1 3x3 data gradient = the forward convolution of dY with the weights transposed
// (ci <-> co) and the taps flipped: dX[ih][iw][ci] = sum W[co][kh][kw][ci] *
// dY[ih + 1 - kh][iw + 1 - kw][co].  Same halo tiling over dY rows; the weight tiles of
// one kernel row are staged as stored ([32 co][BC ci] per tap) and read with
// ds_read_b64_tr_b16, so the dY halo is stored in the transposed read's K order
// (dtrk_pos, as conv_gemm_dgrad_kernel does for its gathered tile).
__device__ __forceinline__ int dtrk_pos(int k4) { return k4 < 4 ? 8 * k4 : 8 * (k4 - 4) + 4; }

template <int BC, int BP, bool MASK_X, bool PART, int GW = 0>  // GW: see the forward kernel
__global__ __launch_bounds__(256) void conv3x3s1_halo_dgrad_kernel(ConvGeom g, const bf16_t* __restrict__ dY,
                                                                   const bf16_t* __restrict__ Wt,
                                                                   const bf16_t* __restrict__ Xact,
                                                                   bf16_t* __restrict__ dX,
                                                                   float* __restrict__ part, int R,
                                                                   int chunks_per_split) {
  constexpr int TCI = BC / 32, TPX = BP / 32;
  constexpr int HCH = (HL_MAXPX * 4 + 255) / 256;
  constexpr int AS = BC + 16;                  // [co][ci] weight row stride (odd multiple of 8 dwords)
  constexpr int WCH = 3 * HL_KS * BC / 8 / 256;  // 16-B weight chunks per thread (one kernel row)
  __shared__ __attribute__((aligned(16))) bf16_t sA[2][3 * HL_KS * AS];
  __shared__ __attribute__((aligned(16))) bf16_t sH[2][HL_MAXPX * HL_RS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wci = wave >> 1, wpx = wave & 1;
  const int W = GW ? GW : g.W, H = g.H, Cout = g.Cout;
  const int RG = (H + R - 1) / R;
  const int3 bk = xcd_block3();  // XCD-contiguous block order
  const int n_ = bk.x / RG, rg = bk.x - n_ * RG;
  const int ih0 = rg * R;
  const int ci0 = bk.y * BC;
  const int HW2 = W + 2, HPX = (R + 2) * HW2;
  const int NPX = R * W;
  const int nch = Cout / HL_KS;
  const int c_beg = bk.z * chunks_per_split;
  const int c_end = min(nch, c_beg + chunks_per_split);
  const int KWC = 9 * g.Cin;

  auto load_halo = [&](int ch, bf16x8* rh) {
#pragma unroll
    for (int u = 0; u < HCH; ++u) {
      const int e = tid + 256 * u;
      const int hp = e >> 2, qq = e & 3;
      rh[u] = zero8();
      if (hp < HPX) {
        const int hr = hp / HW2, hc = hp - hr * HW2;
        const int oh = ih0 - 1 + hr, ow = hc - 1;
        if ((unsigned)oh < (unsigned)H && (unsigned)ow < (unsigned)W)
          rh[u] = ld8(dY + (((long)n_ * H + oh) * W + ow) * Cout + ch * HL_KS + qq * 8);
      }
    }
  };
  auto store_halo = [&](int buf, const bf16x8* rh) {
#pragma unroll
    for (int u = 0; u < HCH; ++u) {
      const int e = tid + 256 * u;
      const int hp = e >> 2, qq = e & 3;
      if (hp < HPX) {
        const uint4 q = __builtin_bit_cast(uint4, rh[u]);
        *reinterpret_cast<uint2*>(&sH[buf][hp * HL_RS + dtrk_pos(2 * qq)]) = make_uint2(q.x, q.y);
        *reinterpret_cast<uint2*>(&sH[buf][hp * HL_RS + dtrk_pos(2 * qq + 1)]) = make_uint2(q.z, q.w);
      }
    }
  };
  // kernel row kh, co chunk ch: sA[(kw * 32 + co) * AS + ci] = W[co0 + co][kh][kw][ci0 + ci]
  auto load_w = [&](int ch, int kh, bf16x8* ra) {
#pragma unroll
    for (int u = 0; u < WCH; ++u) {
      const int c = tid + u * 256;
      const int row = c / (BC / 8), off = (c % (BC / 8)) * 8;
      const int kw = row / HL_KS, co = row - kw * HL_KS;
      ra[u] = ld8(Wt + (long)(ch * HL_KS + co) * KWC + (kh * 3 + kw) * g.Cin + ci0 + off);
    }
  };
  auto store_w = [&](int buf, const bf16x8* ra) {
#pragma unroll
    for (int u = 0; u < WCH; ++u) {
      const int c = tid + u * 256;
      const int row = c / (BC / 8), off = (c % (BC / 8)) * 8;
      *reinterpret_cast<bf16x8*>(&sA[buf][row * AS + off]) = ra[u];
    }
  };

  const int kofs = 8 * (lane >> 4), col = lane & 15;
  const int gq = lane >> 4, q = col >> 2, pq = col & 3;
  int hbase[TPX];
#pragma unroll
  for (int j = 0; j < TPX; ++j) {
    const int p = wpx * (BP / 2) + 16 * j + col;
    const int r = p / W, c = p - r * W;
    hbase[j] = p < NPX ? r * HW2 + c : 0;
  }
  f32x4 acc[TCI][TPX];
#pragma unroll
  for (int i = 0; i < TCI; ++i)
#pragma unroll
    for (int j = 0; j < TPX; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  bf16x8 ra[WCH], rh[HCH];
  if (c_beg < c_end) {
    load_halo(c_beg, rh);
    load_w(c_beg, 0, ra);
    store_halo(0, rh);
    store_w(0, ra);
  }
  __syncthreads();
  int step = 0;
  for (int ch = c_beg; ch < c_end; ++ch) {
    const int hb = (ch - c_beg) & 1;
    const bool next_chunk = ch + 1 < c_end;
    for (int kh = 0; kh < 3; ++kh, ++step) {
      const int cur = step & 1;
      const bool last = kh == 2;
      const bool more = !last || next_chunk;
      if (more) load_w(last ? ch + 1 : ch, last ? 0 : kh + 1, ra);
      if (kh == 0 && next_chunk) load_halo(ch + 1, rh);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int toff = (2 - kh) * HW2 + (2 - kw);  // flipped tap
        const bf16_t* wa = &sA[cur][kw * HL_KS * AS];
        bf16x8 a[TCI], b[TPX];
#pragma unroll
        for (int i = 0; i < TCI; ++i) {
          const int m = wci * (BC / 2) + 16 * i + 4 * pq;
          const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)&wa[(4 * gq + q) * AS + m]);
          const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)&wa[(16 + 4 * gq + q) * AS + m]);
          a[i] = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
#pragma unroll
        for (int j = 0; j < TPX; ++j)
          b[j] = *reinterpret_cast<const bf16x8*>(&sH[hb][(hbase[j] + toff) * HL_RS + kofs]);
#pragma unroll
        for (int i = 0; i < TCI; ++i)
#pragma unroll
          for (int j = 0; j < TPX; ++j) acc[i][j] = mfma16(a[i], b[j], acc[i][j]);
      }
      if (last && next_chunk) store_halo(hb ^ 1, rh);
      if (more) store_w(cur ^ 1, ra);
      __syncthreads();
    }
  }

  const long Ptot = (long)g.N * H * W;
#pragma unroll
  for (int j = 0; j < TPX; ++j) {
    const int p = wpx * (BP / 2) + 16 * j + col;
    const int r = p / W;
    const int ih = ih0 + r;
    if (p >= NPX || ih >= H) continue;
    const long P = ((long)n_ * H + ih) * W + (p - r * W);
#pragma unroll
    for (int i = 0; i < TCI; ++i) {
      const int ci = ci0 + wci * (BC / 2) + 16 * i + 4 * (lane >> 4);
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (PART) {
        *reinterpret_cast<float4*>(part + ((long)bk.z * Ptot + P) * g.Cin + ci) =
            make_float4(v[0], v[1], v[2], v[3]);
        continue;
      }
      if (MASK_X) {
        float xm[4];
        unpack4(*reinterpret_cast<const uint2*>(Xact + P * g.Cin + ci), xm);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) v[rr] = xm[rr] > 0.f ? v[rr] : 0.f;
      }
      *reinterpret_cast<uint2*>(dX + P * g.Cin + ci) = pack4(v[0], v[1], v[2], v[3]);
    }
  }
}

void conv_halo_dgrad(const ConvGeom& g, int bp, int bc, int splits, const bf16_t* dY, const bf16_t* Wt,
                     const bf16_t* Xact, bf16_t* dX, float* part, hipStream_t s) {
  const int R = bp / g.W;
  const int RG = (g.H + R - 1) / R;
  const int nch = g.Cout / HL_KS;
  const int cps = (nch + splits - 1) / splits;
  const dim3 grid(g.N * RG, g.Cin / bc, splits);
  const int gw = g.W == 56 ? 56 : g.W == 28 ? 28 : g.W == 14 ? 14 : 0;  // (see conv_halo_fwd)
#define HLD_W(BC, BP, MX, PT, GWV) \
  hipLaunchKernelGGL((conv3x3s1_halo_dgrad_kernel<BC, BP, MX, PT, GWV>), grid, dim3(256), 0, s, g, dY, Wt, Xact, dX, part, R, cps)
#define HLD(BC, BP, MX, PT)                                              \
  do {                                                                   \
    if (BC != 64 || gw == 0) HLD_W(BC, BP, MX, PT, 0);                   \
    else if (gw == 56) HLD_W(BC, BP, MX, PT, (BC == 64 ? 56 : 0));       \
    else if (gw == 28) HLD_W(BC, BP, MX, PT, (BC == 64 ? 28 : 0));       \
    else HLD_W(BC, BP, MX, PT, (BC == 64 ? 14 : 0));                     \
  } while (0)
#define HLD_BP(BC, BP)                                  \
  if (splits > 1) HLD(BC, BP, false, true);             \
  else if (Xact) HLD(BC, BP, true, false);              \
  else HLD(BC, BP, false, false);
  if (bp == 128) { if (bc == 128) { HLD_BP(128, 128) } else { HLD_BP(64, 128) } }
  else { if (bc == 128) { HLD_BP(128, 64) } else { HLD_BP(64, 64) } }
#undef HLD_BP
#undef HLD
#undef HLD_W
}

// bp: pixel columns of the block's MFMA tile (128 or 64); R = bp / W full rows per block
bool conv_halo_fits(const ConvGeom& g, int bp) {
  if (g.KH != 3 || g.KW != 3 || g.stride != 1 || g.pad != 1 || g.Cin % HL_KS != 0) return false;
  if (g.OH != g.H || g.OW != g.W || (bp != 64 && bp != 128)) return false;
  const int R = bp / g.W;
  return R >= 1 && (R + 2) * (g.W + 2) <= HL_MAXPX;
}

int conv_halo_rows(const ConvGeom& g, int bp) { return bp / g.W; }

void conv_halo_fwd(const ConvGeom& g, int bp, int bc, int splits, const bf16_t* X, const bf16_t* Wt,
                   bf16_t* Y, float* stats, float* part, hipStream_t s, const BnAffine* aff) {
  const bool af = aff && aff->mean;
  if (af && g.Cin > 512) throw std::runtime_error("conv_halo_fwd: input BatchNorm affine needs Cin <= 512");
  const BnAffine a = af ? *aff : BnAffine{};
  const int R = conv_halo_rows(g, bp);
  const int RG = (g.H + R - 1) / R;
  const int nch = g.Cin / HL_KS;
  const int cps = (nch + splits - 1) / splits;
  const dim3 grid(g.N * RG, g.Cout / bc, splits);
  // the 64-channel tiles ResNet-18's planner picks get a width-specialised build
  const int gw = g.W == 56 ? 56 : g.W == 28 ? 28 : g.W == 14 ? 14 : 0;
#define HLF_W(BC, BP, ST, PT, GWV)                                                                              \
  do {                                                                                                          \
    if (af) hipLaunchKernelGGL((conv3x3s1_halo_fwd_kernel<BC, BP, ST, PT, true, GWV>), grid, dim3(256), 0, s, g, X, Wt, Y, stats, part, R, cps, a); \
    else hipLaunchKernelGGL((conv3x3s1_halo_fwd_kernel<BC, BP, ST, PT, false, GWV>), grid, dim3(256), 0, s, g, X, Wt, Y, stats, part, R, cps, a); \
  } while (0)
#define HLF(BC, BP, ST, PT)                                              \
  do {                                                                   \
    if (BC != 64 || gw == 0) HLF_W(BC, BP, ST, PT, 0);                   \
    else if (gw == 56) HLF_W(BC, BP, ST, PT, (BC == 64 ? 56 : 0));       \
    else if (gw == 28) HLF_W(BC, BP, ST, PT, (BC == 64 ? 28 : 0));       \
    else HLF_W(BC, BP, ST, PT, (BC == 64 ? 14 : 0));                     \
  } while (0)
#define HLF_BP(BC, BP)                                  \
  if (splits > 1) HLF(BC, BP, false, true);             \
  else if (stats) HLF(BC, BP, true, false);             \
  else HLF(BC, BP, false, false);
  if (bp == 128) { if (bc == 128) { HLF_BP(128, 128) } else { HLF_BP(64, 128) } }
  else { if (bc == 128) { HLF_BP(128, 64) } else { HLF_BP(64, 64) } }
#undef HLF_BP
#undef HLF
#undef HLF_W
}


// ---------------------------------------------------------------- weight gradient
// Tap-fused stride-1 3x3 weight gradient (ResNet-18's 56/28/14/7-wide 3x3 layers).
//   D[co][tap][ci] = sum_p dY[p][co] * X[p @ tap][ci]
// conv_gemm_wgrad_kernel makes one block per (co tile, tap, ci tile) and re-gathers X per
// tap - dY and X are fetched from L2 nine times.  Here a block owns (64 co) x (32 ci) x
// all 9 taps: it walks its chunk of output rows in groups of R rows of one image
// (R * Wp = 224 K slots, Wp = W rounded up to 8), stages the group's dY rows and the
// (R+2) x (Wp+2) input halo into LDS once, and every wave runs its 2 co tiles x 9 taps
// (18 MFMAs per 32-slot K-step, operands via ds_read_b64_tr_b16 at 32-bit LDS offsets,
// the tap offsets folded into the instruction).  The next group's tiles are loaded into
// registers while the current one computes.  One fp32 slab row per chunk (grid.z) in the
// weight's OHWI layout, reduced by grad_reduce in fixed order - the same output contract
// as conv_gemm_wgrad (a single chunk writes / accumulates the gradient directly).
// Padding slots (rows past the group, columns >= W) carry dY == 0.  Images shorter than
// a group (the 7x7 layers: R = 28) are stacked: a group is R / H whole images, each with
// its own 2 halo rows (chunks then hold whole images).
constexpr int HWG_SLOTS = 224;              // K slots per row group
constexpr int HWG_DS = 64 + 16;             // sdY row stride: 40 dwords (odd multiple of 8)
constexpr int HWG_XS = 32 + 16;             // sX row stride: 24 dwords (odd multiple of 8)
constexpr int HWG_MAXPOS = 360;             // largest halo: 4 x (7 + 2) x (8 + 2) (W = 56: 6 x 58)
constexpr int HWG_DYC = HWG_SLOTS * 8 / 256;         // 16-byte dY chunks per thread (7)
// 16-byte X chunks per thread: CIT / 8 chunks per halo position (32 ci: 6, 16 ci: 3)
template <int CIT>
constexpr int hwg_xc() { return (HWG_MAXPOS * (CIT / 8) + 255) / 256; }

__host__ __device__ inline int hwg_wp(int W) { return (W + 7) & ~7; }
size_t conv_halo_wgrad_lds() {
  return sizeof(bf16_t) * ((size_t)HWG_SLOTS * HWG_DS + (size_t)HWG_MAXPOS * HWG_XS);
}

// CIT: input channels per block (32: 4 waves = 2 co pairs x 2 ci halves; 16: 4 waves x one
// 16-wide co tile - twice the blocks per chunk, so half the chunks and slab bytes for the
// same launch size, at twice the dY re-reads)
// AFF: X is the producer conv's RAW output; the staging applies its BatchNorm + ReLU
// (BnAffine) to the in-image halo positions - each thread's 8 input channels are fixed
// (chunk c % (CIT / 8) == tid % (CIT / 8)), so its sc / sh are computed once.
// WP: W rounded up to 8 (8 / 16 / 32 / 56 - ResNet-18's 7 / 14 / 28 / 56-wide layers), a
// template constant so the slot -> (row, column) divisions and the tap offsets fold away
// (one block per CU: the planner launches ~256 blocks, one per CU, so the register budget
// is a whole SIMD's 512 - the pipelined K-steps below need ~270)
template <int CIT, bool AFF, int WP>
__global__ __launch_bounds__(256, 1) void conv3x3s1_halo_wgrad_kernel(ConvGeom g, const bf16_t* __restrict__ dY,
                                                                      const bf16_t* __restrict__ X,
                                                                      float* __restrict__ out, int rows_per_chunk,
                                                                      int accum, BnAffine bn) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = g.H, W = g.W, Cin = g.Cin, Cout = g.Cout;
  constexpr int Wp = WP, R = HWG_SLOTS / Wp, XW = Wp + 2;
  // segment = rows sharing one halo: a group of R rows of one image, or nimg stacked images
  const int Hs = H < R ? H : R, nimg = R / Hs, live = nimg * Hs;
  constexpr int XCP = CIT / 8, HWG_XC = hwg_xc<CIT>();        // 16-byte chunks per position / thread
  const int nxc = nimg * (Hs + 2) * XW * XCP;  // 16-byte X chunks of the halo(s)
  bf16_t* sdY = reinterpret_cast<bf16_t*>(smem);
  bf16_t* sX = sdY + HWG_SLOTS * HWG_DS;
  const int co0 = blockIdx.x * 64, ci0 = blockIdx.y * CIT;
  const int rows = g.N * H;
  const int rbeg = blockIdx.z * rows_per_chunk;
  const int rend = min(rows, rbeg + rows_per_chunk);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // rows of the group starting at flattened row r: at most R, never past the image (or,
  // stacked, the last whole image) or the chunk
  auto group_rows = [&](int r) { return min(H < R ? live : min(R, H - r % H), rend - r); };
  bf16x8 vd[HWG_DYC], vx[HWG_XC];
  // per-thread staging geometry, the same for every row group (the divisions by the
  // runtime Wp / XW / Hs + 2 were ~1.5k VALU instructions per group when done in load()):
  // dY chunk u -> packed (slot row rr | column col << 8); X chunk u -> packed (segment k |
  // halo row loc << 8 | halo column cc << 16 | channel chunk << 24), 0xff in k = past the halo
  // (the dY chunk geometry is recomputed in load(): Wp is a constant, the divisions are
  // multiplies - 7 VGPRs fewer across the MFMA loop)
  unsigned xgeo[HWG_XC];
#pragma unroll
  for (int u = 0; u < HWG_XC; ++u) {
    const int c = tid + 256 * u;
    const int pos = c / XCP, chk = c - pos * XCP;
    const int hr = pos / XW, cc = pos - hr * XW;
    const int k = hr / (Hs + 2), loc = hr - k * (Hs + 2);
    xgeo[u] = c < nxc ? ((unsigned)k | (unsigned)loc << 8 | (unsigned)cc << 16 | (unsigned)chk << 24) : 0xffu;
  }
  float asc[8], ash[8];
  unsigned xin = 0;  // AFF: bit u = X chunk u of the loaded group lies inside an image
  auto load = [&](int r, int cnt) {
    // group start: image n0, row h0 (stacked groups start on an image: h0 = 0, segment k
    // is image n0 + k; a single-image group has k = 0 only)
    const int n0 = r / H, h0 = r - n0 * H;
    if constexpr (AFF) xin = 0;
#pragma unroll
    for (int u = 0; u < HWG_DYC; ++u) {
      const int slot = (tid + 256 * u) >> 3;
      const int rr = slot / Wp, col = slot - (slot / Wp) * Wp, ch = ((tid + 256 * u) & 7) * 8;
      vd[u] = (rr < cnt && col < W) ? ld8(dY + ((long)(r + rr) * W + col) * Cout + co0 + ch) : zero8();
    }
#pragma unroll
    for (int u = 0; u < HWG_XC; ++u) {
      const unsigned gq8 = xgeo[u];
      const int k = gq8 & 0xff, loc = (gq8 >> 8) & 0xff, cc = (gq8 >> 16) & 0xff, ch = (int)(gq8 >> 24) * 8;
      const int n = n0 + k, hh = h0 - 1 + loc, ww = cc - 1;
      // segments past the group's rows (a partial stacked group at the end of a chunk:
      // their images may not exist) stay zero, like the halo outside the image
      const bool in = k != 0xff && k * Hs < cnt && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
      vx[u] = in ? ld8(X + ((long)(n * H + hh) * W + ww) * Cin + ci0 + ch) : zero8();
      if constexpr (AFF) xin |= (in ? 1u : 0u) << u;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < HWG_DYC; ++u) {
      const int c = tid + 256 * u;
      *reinterpret_cast<bf16x8*>(sdY + (c >> 3) * HWG_DS + (c & 7) * 8) = vd[u];
    }
#pragma unroll
    for (int u = 0; u < HWG_XC; ++u) {
      const int c = tid + 256 * u;
      bf16x8 v = vx[u];
      if constexpr (AFF) {
        if ((xin >> u) & 1u) v = bn_relu8(v, asc, ash);
      }
      if (c < nxc) *reinterpret_cast<bf16x8*>(sX + (c / XCP) * HWG_XS + (c % XCP) * 8) = v;
    }
  };
  // wave tile: co pair (wave >> 1: 2 x 16 co) x ci half (wave & 1: 16 ci), all 9 taps
  constexpr int NCT = CIT == 32 ? 2 : 1;  // 16-wide co tiles per wave
  const int coT = CIT == 32 ? (wave >> 1) * 32 : wave * 16, ciT = CIT == 32 ? (wave & 1) * 16 : 0;
  const int gq = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
  f32x4 acc[NCT][9];
#pragma unroll
  for (int c = 0; c < NCT; ++c)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[c][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  lds_char* lsm = (lds_char*)smem;
  const int ldsX = HWG_SLOTS * HWG_DS;  // element offset of sX
  // LDS operand offsets of the group's 7 K-steps - the same for every group, so computed
  // once (the runtime divisions by Wp / Hs per K-step were a VALU chain in front of every
  // step's LDS reads; at one wave per SIMD nothing hid it: ~576 cycles per 288-cycle step).
  // The K-step loop is then fully unrolled so the next step's reads issue under this step's
  // MFMAs.  Each accumulator still sees its K slots in the same order (bitwise unchanged).
  constexpr int NKS = HWG_SLOTS / 32;
  const int aA = (4 * gq + q) * HWG_DS + coT + 4 * p;  // + 32 * ks * HWG_DS (+ 16 rows: sB)
  // halo position of K slot sl (Wp a constant: the divisions are multiplies): slot row r
  // -> halo row r + 2 per preceding segment; rows past the live ones (dY 0) are clamped
  // onto staged halo rows
  auto xo = [&](int sl) {
    const int r0 = min(sl / Wp, live - 1), c0 = sl - (sl / Wp) * Wp;
    return ldsX + ((r0 + 2 * (r0 / Hs)) * XW + c0) * HWG_XS + ciT + 4 * p;
  };
  const int sL = 4 * gq + q;  // this lane's first K row of a step
  int r0 = rbeg, cnt = r0 < rend ? group_rows(r0) : 0;
  if (cnt > 0) load(r0, cnt);
  // (after the first group's loads are in flight: the parameters land behind them)
  if constexpr (AFF) bn_affine8(bn.invstd, bn.gamma, bn.mean, bn.beta, ci0 + (tid % XCP) * 8, asc, ash);
  while (cnt > 0) {
    store();
    __syncthreads();
    const int r1 = r0 + cnt;
    const int cnt1 = r1 < rend ? group_rows(r1) : 0;
    if (cnt1 > 0) load(r1, cnt1);  // lands while this group's MFMAs run
    // step ks + 1's operand reads are issued under step ks's MFMAs: the a fragments double
    // buffered, each tap's b fragment re-read for the next step right after its two MFMAs
    bf16x8 a[2][NCT], b[9];
    auto rd_a = [&](int ks, int u) {
#pragma unroll
      for (int c = 0; c < NCT; ++c) {
        const int ao = aA + 32 * ks * HWG_DS + 16 * c;
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(lds_ptr4(lsm, ao));
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(lds_ptr4(lsm, ao + 16 * HWG_DS));
        a[u][c] = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
    };
    int xa = 0, xb = 0;  // the step's two halo offsets (recomputed per step: a few VALU under the MFMAs)
    auto rd_b = [&](int tap) {
      const int to = ((tap / 3) * XW + tap % 3) * HWG_XS;
      const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(lds_ptr4(lsm, xa + to));
      const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(lds_ptr4(lsm, xb + to));
      b[tap] = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    };
    auto set_x = [&](int ks) {
      xa = xo(32 * ks + sL);
      xb = xo(32 * ks + sL + 16);
    };
    rd_a(0, 0);
    set_x(0);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) rd_b(tap);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int u = ks & 1;
      if (ks + 1 < NKS) {
        rd_a(ks + 1, u ^ 1);
        set_x(ks + 1);
      }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
#pragma unroll
        for (int c = 0; c < NCT; ++c) acc[c][tap] = mfma16(a[u][c], b[tap], acc[c][tap]);
        if (ks + 1 < NKS) rd_b(tap);
      }
      if (ks + 1 < NKS) {
        // issue order: the next a reads, then per tap its MFMAs and the next b reads (left
        // alone the scheduler hoisted all reads and kept two b sets live: spills)
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * NCT, 0);
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          __builtin_amdgcn_sched_group_barrier(0x008, NCT, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // no further hoisting of reads (registers)
    }
    __syncthreads();  // every wave is done with this group's tiles
    r0 = r1;
    cnt = cnt1;
  }
  // slab row of this chunk: [co][tap][ci] (OHWI); 16 lanes hold 16 consecutive ci
  float* o = out + (long)blockIdx.z * Cout * 9 * Cin;
#pragma unroll
  for (int c = 0; c < NCT; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = co0 + coT + 16 * c + 4 * gq + r;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const long idx = ((long)co * 9 + tap) * Cin + ci0 + ciT + i16;
        o[idx] = accum ? o[idx] + acc[c][tap][r] : acc[c][tap][r];
      }
    }
}

bool conv_halo_wgrad_ok(const ConvGeom& g) {
  if (g.KH != 3 || g.KW != 3 || g.stride != 1 || g.pad != 1) return false;
  if (g.OH != g.H || g.OW != g.W || g.Cin % 32 != 0 || g.Cout % 64 != 0) return false;
  const int Wp = hwg_wp(g.W), R = HWG_SLOTS / Wp;
  if (HWG_SLOTS % Wp != 0) return false;
  const int Hs = g.H < R ? g.H : R;
  return (R / Hs) * (Hs + 2) * (Wp + 2) <= HWG_MAXPOS;
}

// rows per chunk must keep stacked groups on image starts: a multiple of H when H < R
int conv_halo_wgrad_row_quantum(const ConvGeom& g) {
  const int R = HWG_SLOTS / hwg_wp(g.W);
  return g.H < R ? g.H : 1;
}

void conv_halo_wgrad(const ConvGeom& g, const bf16_t* dY, const bf16_t* X, float* out, int rows_per_chunk,
                     bool accum, hipStream_t s, int cit, const BnAffine* aff) {
  const bool af = aff && aff->mean;
  const BnAffine a = af ? *aff : BnAffine{};
  const int chunks = (g.N * g.H + rows_per_chunk - 1) / rows_per_chunk;
  const dim3 grid(g.Cout / 64, g.Cin / cit, chunks);
  const size_t lds = conv_halo_wgrad_lds();
  const int wp = hwg_wp(g.W);
  if (wp != 8 && wp != 16 && wp != 32 && wp != 56) throw std::runtime_error("conv_halo_wgrad: W outside 7..56");
  const int acc = accum && chunks == 1 ? 1 : 0;
#define HWG_L(CIT, AF, WPV)                                                                                       \
  do {                                                                                                           \
    auto k = conv3x3s1_halo_wgrad_kernel<CIT, AF, WPV>;                                                          \
    static bool opted = false;                                                                                   \
    if (!opted) {                                                                                                \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
      opted = true;                                                                                              \
    }                                                                                                            \
    hipLaunchKernelGGL(k, grid, dim3(256), lds, s, g, dY, X, out, rows_per_chunk, acc, a);                      \
  } while (0)
#define HWG_W(CIT, AF)                       \
  do {                                       \
    if (wp == 8) HWG_L(CIT, AF, 8);          \
    else if (wp == 16) HWG_L(CIT, AF, 16);   \
    else if (wp == 32) HWG_L(CIT, AF, 32);   \
    else HWG_L(CIT, AF, 56);                 \
  } while (0)
  if (cit == 16) { if (af) HWG_W(16, true); else HWG_W(16, false); }
  else { if (af) HWG_W(32, true); else HWG_W(32, false); }
#undef HWG_W
#undef HWG_L
}

}  // namespace ddp_amd
