// The forward conv kernel's body - NOT a self-contained header: included inside
// conv3x3_fwd.h's conv3x3_fwd_kernel (the plain forward) and fwd_body (the step head's
// forward, a device function), which both define X, Wt, bias, Y, B, H, W, Cin, Cout, wfc,
// fc_part, c1, dzo, mg, bx, by, MRG and smem before including it.  One body, two codegens:
// as a device function called by a wrapper kernel the OCC 2 plain forward spilled 22 VGPRs
// (116 -> 128 + 92 B scratch), and as the kernel itself the step head measured 3 us slower
// (677k vs 720k img/s forced dist_mode 4, same call, profiles/r6_dist/ab_head_codegen.txt).
  using P = Prec<T>;
  constexpr bool F32 = sizeof(T) == 4;
  static_assert(!DZ || (NOF == 10 && A1X), "level-3 dZ2 needs the fc epilogue and the conv1 recompute");
  static_assert(!MRG || (DZ && !F32), "the merged forward is the bf16 level-3 forward");
  constexpr int CE = P::CE;
  DDP_STAMP(STAMP_K_CONV_FWD, 0);
  DDP_GEOM_OVERRIDE();
  constexpr int CH = 16 * NW * PXT, NT = NW * 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int HW = H * W;
  const long Ptot = (long)B * HW;
  const int co0 = by * 64;
  // row strides = 8 mod 16 dwords: conflict-free b128 fragment reads
  const int KW = 9 * Cin, WS = KW + P::PAD, XS = Cin + P::PAD;
  const int XR = CH + 2 * W + 2;
  T* sW = reinterpret_cast<T*>(smem);
  T* sX = sW + 64 * WS;
  const long P0 = (long)bx * CH;
  const long Pbase = P0 - W - 1;

  const int wc = KW / CE;
  const int xc = Cin / CE;
  if (A1X && c1.zero_i32)  // the step's level-2 hand-off flags (see C1Src)
    for (int i = threadIdx.x; i < c1.zero_per_block; i += NT) {
      const long z = (long)bx * c1.zero_per_block + i;
      if (z < c1.zero_total) c1.zero_i32[z] = 0;
    }
  Conv1Group cg;
  if constexpr (!MRG) {
  if (A1X) cg = conv1_group_load(c1.w, c1.b, wave & 3);  // lands during the staging round
  // weights and (unless recomputed) the input rows in ONE round of loads
  stage2<(64 / NW) * (F32 ? 2 : 1), NT>(64 * wc,
             [&](int i) { const int r = i / wc, c = (i - r * wc) * CE; return ld16(Wt + (long)(co0 + r) * KW + c); },
             [&](int i, bf16x8 v) { const int r = i / wc, c = (i - r * wc) * CE; st16(sW + r * WS + c, v); },
             A1X ? 0 : XR * xc,
             [&](int i) {
               const int r = i / xc, c = (i - r * xc) * CE;
               const long Pq = Pbase + r;
               return (Pq >= 0 && Pq < Ptot) ? ld16(X + Pq * Cin + c) : zero8();
             },
             [&](int i, bf16x8 v) { const int r = i / xc, c = (i - r * xc) * CE; st16(sX + r * XS + c, v); });
  }
  if (A1X) {
    // x for the linear range [Pbase - W - 1, Pbase + XR + W + 1), then a1 (conv1 recompute).
    // The block also writes its own pixels (and the labels of images starting in them)
    // to the step's compact batch buffers, if given.
    float* sxx = reinterpret_cast<float*>(sX + XR * XS);
    const int NXX = XR + 2 * W + 2;
    const int base = c1.bi.base();
    for (int r = threadIdx.x; r < NXX; r += NT) {
      const long Pq = Pbase - W - 1 + r;
      float v = 0.f;
      if (Pq >= 0 && Pq < Ptot) {
        const int n = (int)(Pq / HW), rm = (int)(Pq - (long)n * HW);
        const int row = c1.bi.row(n, base);
        const unsigned char u = c1.x[(long)row * HW + rm];
        v = (float)u / 255.0f;
        if (c1.xb_out && Pq >= P0 && Pq < P0 + CH) {
          c1.xb_out[Pq] = u;
          if (rm == 0) c1.yb_out[n] = c1.labels[row];
        }
      }
      sxx[r] = v;
    }
    if constexpr (MRG) {
      // the step's images are staged; now this step's conv parameters must be final
      DDP_STAMP(STAMP_K_HEAD, 4);
      wait_count<MRG_SLEEP>(mg.conv_done, mg.nblk1, mg.err, MRG_ERR);
      DDP_STAMP(STAMP_K_HEAD, 5);
      cg = conv1_group_load_sc1(c1.w, c1.b, wave & 3);
      const __amdgpu_buffer_rsrc_t rw =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(Wt), (short)0, 0x7fffffff, 0x00020000);
      stage2<64 / NW, NT>(64 * wc,
          [&](int i) { const int r = i / wc, c = (i - r * wc) * CE; return ld16_sc1(rw, (int)(((co0 + r) * KW + c) * sizeof(T))); },
          [&](int i, bf16x8 v) { const int r = i / wc, c = (i - r * wc) * CE; st16(sW + r * WS + c, v); },
          0, [&](int) { return zero8(); }, [&](int, bf16x8) {});
    }
    __syncthreads();
    DDP_STAMP(STAMP_K_CONV_FWD, 1);
    conv1_recompute_tile<T>(
        XR, cg, wave & 3, 64 * (wave >> 2), 64 * (NW / 4),
        [&](int r) { const long Pq = Pbase + r; return Pq >= 0 && Pq < Ptot; },
        [&](int r, int k) {
          const long Pq = Pbase + r;
          const int rm = (int)(Pq % HW);
          const int hh = rm / W, ww = rm - (rm / W) * W;
          const int dh = k / 3 - 1, dw = k % 3 - 1;
          const bool ok = (unsigned)(hh + dh) < (unsigned)H && (unsigned)(ww + dw) < (unsigned)W;
          return ok ? sxx[r + W + 1 + dh * W + dw] : 0.f;
        },
        [&](int r, int g) { return sX + r * XS + 8 * g; });
    DDP_STAMP(STAMP_K_CONV_FWD, 5);
  }

  const int kofs = P::kofs(lane);
  const int col = lane & 15;
  int h[PXT], w[PXT], rowc[PXT], rem[PXT];
  bool valid[PXT];
  long Pp[PXT];
#pragma unroll
  for (int pt = 0; pt < PXT; ++pt) {
    const int lp = (wave * PXT + pt) * 16 + col;  // pixel within the block
    Pp[pt] = P0 + lp;
    valid[pt] = Pp[pt] < Ptot;
    const long Pc = valid[pt] ? Pp[pt] : 0;
    const int n = (int)(Pc / HW);
    rem[pt] = (int)(Pc - (long)n * HW);
    h[pt] = rem[pt] / W;
    w[pt] = rem[pt] - h[pt] * W;
    rowc[pt] = lp + W + 1;  // sX row of the pixel itself
  }
  // fc weight prefetch (lands while the MFMAs run; issued before the staging it delayed
  // it - in-order vmcnt - by more than it saved); fp32 reads its FCFRAG-order fp32 weight in
  // the epilogue instead (160 more VGPRs would not fit next to the fp32 fragments)
  // OCC 2 (level 3 at B > 32, two blocks per CU): no prefetch - the 80 VGPRs of bf16 weight
  // pairs would hold the kernel at one block per CU; they are read where used (L2 hits),
  // the other block of the CU hides that latency
  constexpr bool PFW = NOF > 0 && !F32 && OCC == 1 && !MRG;
  if constexpr (DZ) DDP_STAMP(STAMP_K_FWD_DZ, 6);  // (pixel index math done)
  // buffer loads: one per-lane VGPR offset per pixel tile and a uniform (o, t) SGPR offset
  // (flat loads: two 64-bit adds per load; without the prefetch (!PFW) the compiler kept 40
  // 64-bit addresses live between the fc partials and dZ2 and spilled)
  const __amdgpu_buffer_rsrc_t rwfc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(wfc), (short)0, 0x7fffffff, 0x00020000);
  auto fcw = [&](int pt, int t, int o) {
    const int vo = (((rem[pt] >> 4) * (Cout >> 4) + (co0 >> 4)) * 64 + lane) * 4 * (int)sizeof(T);
    const int so = ((o * (HW >> 4) * (Cout >> 4) + t) * 64) * 4 * (int)sizeof(T);
    return __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rwfc, vo, so, MRG ? 16 : 0));
  };
  uint2 wv[PFW ? PXT : 1][4][PFW ? NOF : 1];
  // PF_SPLIT: the prefetch is issued in slices between the MFMA loop's taps instead of all
  // ahead of it (80 b64 loads per wave, 327 KB per block: the CU's vector-memory path needs
  // ~1.2 us to take them - stamps, profiles/r4_diag - time the MFMAs can cover)
  constexpr bool PF_SPLIT = PFW && DDP_AMD_FWD_PF_SPLIT;
  constexpr int NPF = PXT * 4 * (NOF > 0 ? NOF : 1);
  auto wv_slice = [&](int tap) {
#pragma unroll
    for (int i = 0; i < NPF; ++i)
      if (i * 9 / NPF == tap) {
        const int pt = i / (4 * NOF), t = (i / NOF) % 4, o = i % NOF;
        wv[pt][t][o] = fcw(pt, t, o);
      }
  };
  if constexpr (PFW && !PF_SPLIT) {
#pragma unroll
    for (int pt = 0; pt < PXT; ++pt)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int o = 0; o < (NOF > 0 ? NOF : 1); ++o)
          wv[pt][t][o] = fcw(pt, t, o);
  }
  // DZ, exact fp32: the fc weight quads are needed twice (fc partials, then dZ2) and held in
  // registers anyway - request them here too, so they land during the MFMA loop (the fp32
  // MFMA loop reads only LDS: no vmcnt wait inside it); F32_FC_PREFETCH = 0 loads them in
  // the epilogue instead
  float4 wq[DZ && F32 ? PXT : 1][DZ && F32 ? 4 : 1][DZ && F32 ? NOF : 1];
  if constexpr (DZ && F32 && F32_FC_PREFETCH) {
#pragma unroll
    for (int pt = 0; pt < PXT; ++pt)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int o = 0; o < NOF; ++o)
          wq[pt][t][o] = *reinterpret_cast<const float4*>(
              wfc + ((((long)o * (HW >> 4) + (rem[pt] >> 4)) * (Cout >> 4) + (co0 >> 4) + t) * 64 + lane) * 4);
  }
  if constexpr (DZ) DDP_STAMP(STAMP_K_FWD_DZ, 7);  // (fc weight prefetch issued)
  // LDS-only barrier: the fc weight prefetch stays in flight through the MFMA loop
  // (__syncthreads drained it here: ~2 us per block, stamps s5 -> s2)
  lds_barrier();
  DDP_STAMP(STAMP_K_CONV_FWD, 2);
  if (A1X && !F32 && c1.a1_out) {
    // the block's own a1 rows (LDS rows W+1 .. W+CH) -> a1_out, 16 bytes per thread-step,
    // write-through (sc1): no dirty L2 lines for the kernel-end release to write back
    const int xc8 = Cin / 8;
    typedef __attribute__((ext_vector_type(4))) int i32x4_t;
    const long a1_bytes = Ptot * Cin * (long)sizeof(T);
    const __amdgpu_buffer_rsrc_t ra1 = __builtin_amdgcn_make_buffer_rsrc(
        c1.a1_out, (short)0, (int)(a1_bytes < 0x7fffffffL ? a1_bytes : 0x7fffffffL), 0x00020000);
    for (int i = threadIdx.x; i < CH * xc8; i += NT) {
      const int lp = i / xc8, c = (i - lp * xc8) * 8;
      const long P = P0 + lp;
      if (P < Ptot)
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(i32x4_t, *reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16_t*>(sX) +
                                                                        (lp + W + 1) * XS + c)),
            ra1, (int)((P * Cin + c) * (long)sizeof(T)), 0, 16 /* sc1: write-through */);
    }
  }

  f32x4 acc[PXT][4];
#pragma unroll
  for (int pt = 0; pt < PXT; ++pt)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[pt][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // the epilogue's bias quads, requested before the MFMA loop (a dependent global load at
  // the start of the epilogue cost ~1-2 us per block)
  float4 bq[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
    bq[t] = MRG ? slab_ld4_sc1(bias, co0 + 16 * t + 4 * (lane >> 4))
                : *reinterpret_cast<const float4*>(bias + co0 + 16 * t + 4 * (lane >> 4));

  const T* wrow = sW + col * WS + kofs;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int dh = tap / 3 - 1, dw = tap % 3 - 1;
    for (int ci0 = 0; ci0 < Cin; ci0 += 32) {
      typename P::Frag a[4], b[PXT];
#pragma unroll
      for (int t = 0; t < 4; ++t) a[t] = P::frag(wrow + 16 * t * WS + tap * Cin + ci0);
#pragma unroll
      for (int pt = 0; pt < PXT; ++pt) {
        const int hh = h[pt] + dh, ww = w[pt] + dw;
        const bool ok = valid[pt] && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
        // unconditional read (the row is always inside the staged range), then a select:
        // no exec-masked LDS read, so the reads of a tap pipeline ahead of the MFMAs
        const typename P::Frag v = P::frag(sX + (rowc[pt] + dh * W + dw) * XS + ci0 + kofs);
        b[pt] = fsel(ok, v, P::zero());
      }
#pragma unroll
      for (int pt = 0; pt < PXT; ++pt)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[pt][t] = P::mma(a[t], b[pt], acc[pt][t]);
    }
    if constexpr (PF_SPLIT) {
      __builtin_amdgcn_sched_barrier(0);
      wv_slice(tap);
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  DDP_STAMP(STAMP_K_CONV_FWD, 3);
  if constexpr (MRG) {  // the fc weight shadow is final
    wait_count<MRG_SLEEP>(mg.fc_done, mg.nblk0, mg.err, MRG_ERR);
    DDP_STAMP(STAMP_K_HEAD, 6);
  }
  // epilogue: bias + ReLU + bf16 store (+ fc partial logits: per block and image,
  // layout [block][2][NOF], see FC_BLOCK_PARTIALS in launchers.h)
  float* s_fc = reinterpret_cast<float*>(smem + fwd_stage_lds(W, Cin, CH / 64, A1X, (int)sizeof(T)));
  uint2 a2pk[DZ && !F32 ? PXT : 1][4];  // DZ: the stored bf16 a2 quads (dZ2's ReLU mask)
  // DZ, exact fp32: the stored a2 quads (and wq, the fc weight quads), kept for dZ2
  float4 a2q[DZ && F32 ? PXT : 1][4];
#pragma unroll
  for (int pt = 0; pt < PXT; ++pt) {
    float fcs[NOF > 0 ? NOF : 1];
#pragma unroll
    for (int o = 0; o < (NOF > 0 ? NOF : 1); ++o) fcs[o] = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if constexpr (NOF > 0 && !PFW && !F32) __builtin_amdgcn_sched_barrier(0);  // 20 VGPRs of weights at a time
      const int co = co0 + 16 * t + 4 * (lane >> 4);
      const float4 bv = bq[t];
      float v0 = acc[pt][t][0] + bv.x, v1 = acc[pt][t][1] + bv.y;
      float v2 = acc[pt][t][2] + bv.z, v3 = acc[pt][t][3] + bv.w;
      if (RELU) { v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f); }
      float q[4] = {v0, v1, v2, v3};  // the values actually stored (what backward re-reads)
      if constexpr (F32) {
        // (DZ: stored after the partial logits are published - see the dZ2 section)
        if constexpr (!DZ) {
          if (valid[pt]) st_wt(reinterpret_cast<float4*>(Y + Pp[pt] * Cout + co), make_float4(v0, v1, v2, v3));
        }
        if constexpr (DZ) a2q[pt][t] = make_float4(v0, v1, v2, v3);
      } else {
        const uint2 pk = pack4(v0, v1, v2, v3);
        if constexpr (!DZ) {
          if (valid[pt]) st_wt(reinterpret_cast<uint2*>(Y + Pp[pt] * Cout + co), pk);  // a2: write-through
        }
        unpack4(pk, q);
        if constexpr (DZ) a2pk[pt][t] = pk;
      }
      if (NOF > 0) {
#pragma unroll
        for (int o = 0; o < (NOF > 0 ? NOF : 1); ++o) {
          float s = fcs[o];
          if constexpr (F32) {  // fp32 FCFRAG weight: 4 consecutive channels, 1 KB per wave load
            float4 w4;
            if constexpr (DZ && F32_FC_PREFETCH) {
              w4 = wq[pt][t][o];
            } else {
              w4 = *reinterpret_cast<const float4*>(
                  wfc + ((((long)o * (HW >> 4) + (rem[pt] >> 4)) * (Cout >> 4) + (co0 >> 4) + t) * 64 + lane) * 4);
              if constexpr (DZ) wq[pt][t][o] = w4;
            }
            s = fmaf(q[0], w4.x, s); s = fmaf(q[1], w4.y, s);
            s = fmaf(q[2], w4.z, s); s = fmaf(q[3], w4.w, s);
          } else {
            // the stored bf16 pairs against the bf16 weight pairs: v_dot2c_f32_bf16 (exact
            // bf16 products, fp32 accumulate) - no unpacking of either operand
            const uint2 pk = pack4(v0, v1, v2, v3);
            uint2 wo;
            if constexpr (PFW) wo = wv[pt][t][o]; else wo = fcw(pt, t, o);
            s = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2v, pk.x),
                                                __builtin_bit_cast(bf16x2v, wo.x), s, false);
            s = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2v, pk.y),
                                                __builtin_bit_cast(bf16x2v, wo.y), s, false);
          }
          fcs[o] = valid[pt] ? s : 0.f;
        }
      }
    }
    if (NOF > 0) {
      // sum over the tile's 16 pixels (the 16 lanes of a row share a channel group)
#pragma unroll
      for (int o = 0; o < (NOF > 0 ? NOF : 1); ++o) {
        const float s = sum16(fcs[o]);
        if ((lane & 15) == 0) s_fc[(((wave * PXT + pt) * 4) + (lane >> 4)) * NOF + o] = s;
      }
    }
  }
  DDP_STAMP(STAMP_K_CONV_FWD, 6);
  if (NOF > 0) {
    lds_barrier();  // (the a2 write-through stores need not land before the tile sums)
    // per (image slot, class): fixed-order sum over the block's tiles of that image and
    // the 4 channel groups.  Slot 0 = the image of the block's first pixel, slot 1 = the
    // next one (a block of 64*PXT <= HW pixels spans at most two images).
    if ((int)threadIdx.x < 2 * NOF) {
      const int slot = threadIdx.x / NOF, o = threadIdx.x - (threadIdx.x / NOF) * NOF;
      const long img = P0 / HW + slot;
      // every read unconditional and unrolled (the reads go out together; a branch per tile
      // kept them one LDS round trip apart), the other image's tiles added as +0.0f - an
      // exact no-op for a sum that starts at +0.0f, so the same bits as skipping them
      float acc_o = 0.f;
#pragma unroll
      for (int tile = 0; tile < NW * PXT; ++tile) {
        const long tp = P0 + tile * 16;
        const bool in = tp < Ptot && tp / HW == img;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float v = s_fc[(tile * 4 + g) * NOF + o];
          acc_o += in ? v : 0.f;
        }
      }
      float* dst = fc_part + ((long)bx * 2 + slot) * NOF + o;
      if constexpr (DZ) st_wt(dst, acc_o);  // read by the other blocks of the image in-launch
      else *dst = acc_o;
    }
  }
  DDP_STAMP(STAMP_K_CONV_FWD, 4);
  if constexpr (DZ) {
    // ---- level 3: dL of the block's image(s), then dZ2 of its own pixels.
    // Hand-off (MI355X_MICROARCH.md, hand-off table row 1): the partials were stored sc1 by
    // wave 0 (threads < 2 * NOF), which drains them and then adds 1 to each touched image's
    // counter (one lane per counter); the same wave polls the counters with sc1 loads and
    // reads the partials with sc1 loads; the other waves only read LDS after a barrier.
    const int HWi = H * W;
    const int img0 = (int)(P0 / HWi);
    const long plast = (P0 + CH < Ptot ? P0 + CH : Ptot) - 1;
    const int nimg = (int)(plast / HWi) - img0 + 1;  // 1 or 2 (CH <= HW)
    float* s_lg = s_fc + NW * PXT * 4 * NOF;          // [2][NOF] logits
    float* s_dl = s_lg + 2 * NOF;                     // [2][NOF] dL
    // the stored a2 (write-through; the conv backward reads it): deferred out of the epilogue
    // so that wave 0's drain before its arrival add waits for the partial logits only
    auto store_a2 = [&]() {
#pragma unroll
      for (int pt = 0; pt < PXT; ++pt)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int co = co0 + 16 * t + 4 * (lane >> 4);
          if (!valid[pt]) continue;
          if constexpr (F32) st_wt(reinterpret_cast<float4*>(Y + Pp[pt] * Cout + co), a2q[pt][t]);
          else st_wt(reinterpret_cast<uint2*>(Y + Pp[pt] * Cout + co), a2pk[pt][t]);
        }
    };
    DDP_STAMP(STAMP_K_FWD_DZ, 0);
    if (wave != 0) store_a2();
    if (wave == 0) {
      int label = 0;
      if (lane < 2 * NOF) {  // the label of this thread's row, requested before the wait (its
        // dependent-load chain overlaps the store drain below; loading it in the prologue
        // instead measured -0.6 %: it delayed the x staging loads, profiles/r4_label)
        const int im = img0 + (lane >= NOF ? 1 : 0);
        if (im < B) label = c1.labels[c1.bi.row(im, c1.bi.base())];
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the partial-logit stores are out
      DDP_STAMP(STAMP_K_FWD_DZ, 1);
      if (lane < nimg)
        __hip_atomic_fetch_add(dzo.img_cnt + (img0 + lane) * FWD_DZ_CNT_STRIDE, 1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      store_a2();  // wave 0's a2 stores: after the drain above (it waited only for the partials)
      {
        const int im = img0 + (lane < nimg ? lane : 0);
        const int kb0 = im * HWi / CH, kb1 = (im * HWi + HWi - 1) / CH;
        const int want = kb1 - kb0 + 1;  // blocks touching image im
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (true) {
          const int v = lane < nimg ? __hip_atomic_load(dzo.img_cnt + im * FWD_DZ_CNT_STRIDE, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT)
                                    : want;
          if (__all(v >= want)) break;
          if (__builtin_amdgcn_s_memrealtime() - t0 > FWD_DZ_WAIT_TICKS) {
            if (lane == 0 && dzo.err) __hip_atomic_store(dzo.err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      DDP_STAMP(STAMP_K_FWD_DZ, 2);
      if (lane < 2 * NOF) {
        const int slot = lane >= NOF ? 1 : 0, o = lane - slot * NOF;
        if (slot < nimg) {
          const float a = xent_logit_acc(img0 + slot, o, HWi, CH, NOF, [&](int i) {
            return __hip_atomic_load(fc_part + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          });
          s_lg[lane] = (MRG ? __hip_atomic_load(dzo.fc_bias + o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                            : dzo.fc_bias[o]) + a;
        }
      }
      DDP_STAMP(STAMP_K_FWD_DZ, 4);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the row's logits (other lanes) are in LDS
      if (lane < 2 * NOF) {
        const int slot = lane >= NOF ? 1 : 0, o = lane - slot * NOF;
        if (slot < nimg) {
          float lossv = 0.f;
          const float d = xent_row_dl(s_lg + slot * NOF, NOF, o, label, dzo.gscale, &lossv);
          s_dl[lane] = d;
          // the block holding the image's first pixel publishes its dL row and loss
          if (dzo.dl_out && (slot == 1 || P0 == (long)img0 * HWi)) {
            const int im = img0 + slot;
            dzo.dl_out[im * NOF + o] = d;
            if (o == 0) dzo.loss_rows[im] = lossv;
          }
        }
      }
    }
    lds_barrier();
    DDP_STAMP(STAMP_K_FWD_DZ, 3);
    // dZ2 = relu2'(a2) * sum_o dL[o] W[o][p][c], in fc_bwd's order (o = 0..9, fma from 0)
#pragma unroll
    for (int pt = 0; pt < PXT; ++pt) {
      const long tp = P0 + (wave * PXT + pt) * 16;  // a 16-pixel tile never straddles images (HW % 16 == 0)
      const float* dl = s_dl + (tp / HWi != img0 ? NOF : 0);
      float d[NOF];
#pragma unroll
      for (int o = 0; o < NOF; ++o) d[o] = dl[o];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if constexpr (!PFW && !F32) __builtin_amdgcn_sched_barrier(0);
        float dz[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int o = 0; o < NOF; ++o) {
          float w4[4];
          if constexpr (F32) {
            const float4 wf = wq[pt][t][o];
            w4[0] = wf.x; w4[1] = wf.y; w4[2] = wf.z; w4[3] = wf.w;
          } else if constexpr (PFW) {
            unpack4(wv[pt][t][o], w4);
          } else {
            unpack4(fcw(pt, t, o), w4);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) dz[j] = fmaf(d[o], w4[j], dz[j]);
        }
        float q[4];
        if constexpr (F32) {
          q[0] = a2q[pt][t].x; q[1] = a2q[pt][t].y; q[2] = a2q[pt][t].z; q[3] = a2q[pt][t].w;
        } else {
          unpack4(a2pk[pt][t], q);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) dz[j] = q[j] > 0.f ? dz[j] : 0.f;
        const int co = co0 + 16 * t + 4 * (lane >> 4);
        if constexpr (F32) {
          if (valid[pt]) st_wt(reinterpret_cast<float4*>(dzo.dz2_f32 + Pp[pt] * Cout + co), make_float4(dz[0], dz[1], dz[2], dz[3]));
        } else {
          if (valid[pt]) st_wt(reinterpret_cast<uint2*>(dzo.dz2 + Pp[pt] * Cout + co), pack4(dz[0], dz[1], dz[2], dz[3]));
        }
      }
    }
    DDP_STAMP(STAMP_K_CONV_FWD, 7);
    DDP_STAMP(STAMP_K_FWD_DZ, 5);
  }
