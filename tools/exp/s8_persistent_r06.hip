// Round-6 experiment (NOT built into the product; DESIGN.md §4.2b 'Round 6'): the FWD / DX kinds as a
// persistent launch with a register epilogue and the next tile's first K step staged during the
// epilogue, plus a start-delay stagger of co-resident blocks. Measured slower in the update's
// minibatch than the hardware-dispatched per-tile launch (static tile lists lose the dispatcher's
// dynamic balance; the stagger bought nothing under the power-limited clock). Excerpt of
// legged_gym_custom_amd/csrc/lgx_s8.hip at that commit (device code, then the host launcher).

// ---------------------------------------------------------------- persistent FWD / DX (round 6)
// The forward and input-gradient kinds as a persistent launch: each block (2 per CU) walks a list
// of output tiles, and its epilogue runs from the accumulator registers — no fp32 LDS image, no
// barrier — so the LDS stages stay owned by the K loop and the NEXT tile's first K step is staged
// (LDS-DMA) while this tile's epilogue runs. The block's K steps are numbered across its tiles
// (stage = step & 1), so the pipeline of lgxs::s8_gemm_kernel continues over tile boundaries.
//
// The MFMA operands are swapped (weights as the MFMA's A operand, activations as its B operand):
// the same three products per K step in the same accumulation order (lo*hi, hi*lo, hi*hi), but
// each lane then holds 4 CONSECUTIVE output columns of one row (C/D map: column = 4 (lane >> 4) + r,
// row = lane & 15). Lanes l and l + 16 hold the two halves of one 8-column S8 group: after the
// bf16 hi / lo split one v_permlane16_swap per dword gives lane l the group's 8 hi values and lane
// l + 16 its 8 lo values — one 16-B store each, the 32-B group written whole. The DX epilogue's
// ELU' operand y (S8) is loaded the mirror way (lane l the group's hi, lane l + 16 its lo, then
// swapped). Column sums (the next weight gradient's bias gradient) per 64-row half tile: the
// wave's 4 row tiles summed in registers, then the 16 lanes of a row by DPP (fixed order).
struct PGroup {
  int n, per_xcd;
  int stagger, delay;    // blocks that start `delay` cycles late (0: none; 1: odd slots; 2: the upper half of the slots)
  int start[GMAX + 1];   // first tile of each problem in the launch's tile list
  int xstart[9];         // XCD slot x: tiles [xstart[x], xstart[x + 1]), its block s every per_xcd-th from s
  Prob p[GMAX];
};
static_assert(sizeof(PGroup) <= 4096, "kernel argument segment");

__device__ __forceinline__ float dpp_row_sum(float v) {
  // sum over the 16 lanes of each DPP row (every lane of the row gets it): quad swaps, then
  // rotations by 4 and 8 within the row — a fixed order, so the result is deterministic
  int x = __float_as_int(v);
  v += __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0xB1, 0xf, 0xf, false));  // quad_perm [1,0,3,2]
  x = __float_as_int(v);
  v += __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x4E, 0xf, 0xf, false));  // quad_perm [2,3,0,1]
  x = __float_as_int(v);
  v += __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x124, 0xf, 0xf, false));  // row_ror:4
  x = __float_as_int(v);
  v += __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x128, 0xf, 0xf, false));  // row_ror:8
  return v;
}

template <int KIND>
__global__ __launch_bounds__(Cfg::NT, 2) __attribute__((amdgpu_waves_per_eu(1, 2))) void s8p_kernel(PGroup g) {
  static_assert(KIND == LGX_S8_FWD || KIND == LGX_S8_DX, "FWD / DX");
  constexpr bool BTR = KIND == LGX_S8_DX;
  constexpr int BM = Cfg::BM, NW = Cfg::NW;
  using OA = Op<false, BM, NW>;
  using OB = Op<BTR, BN, NW>;
  constexpr int STAGE = OA::IMG + OB::IMG;
  static_assert(2 * STAGE <= Cfg::LDS_STAGES, "two stages");
  extern __shared__ __align__(16) char lds[];

  const int x = blockIdx.x & 7, slot = blockIdx.x >> 3;
  int t = g.xstart[x] + slot;
  const int tend = g.xstart[x + 1];
  if (t >= tend) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave % Cfg::WR) * 64, wn = (wave / Cfg::WR) * 64;
  const uint32_t lds0 = (uint32_t)(uintptr_t)((LDS_AS char*)lds);
  const int wv = __builtin_amdgcn_readfirstlane(wave);

  auto find = [&](int tt) {
    int pi = 0;
    while (pi + 1 < g.n && tt >= g.start[pi + 1]) ++pi;
    return pi;
  };
  // tile tt -> problem, tile origin, K steps; per-lane DMA offsets of its step 0
  struct Geo { int pi, m0, n0, nk; };
  auto geo = [&](int tt, uint32_t (&oa)[OA::PW], uint32_t (&ob)[OB::PW]) {
    Geo r;
    r.pi = find(tt);
    const Prob& P = g.p[r.pi];
    const int l = tt - g.start[r.pi];
    r.n0 = (l % P.tiles_n) * BN;
    r.m0 = (l / P.tiles_n) * BM;
    r.nk = (P.K + BK - 1) / BK;
    OA::offsets(oa, wave, lane, r.m0, P.M, P.lda, 0);
    OB::offsets(ob, wave, lane, r.n0, P.N, P.ldb, 0);
    return r;
  };
  auto issue = [&](int stage, const Geo& q, const uint32_t (&oa)[OA::PW], const uint32_t (&ob)[OB::PW], int step) {
    const Prob& P = g.p[q.pi];
    const uint32_t st = lds0 + (uint32_t)(stage * STAGE);
    OA::issue(P.A + step * OA::step_bytes(P.lda), oa, st, wv);
    OB::issue(P.B + step * OB::step_bytes(P.ldb), ob, st + OA::IMG, wv);
  };

  uint32_t offA[OA::PW], offB[OB::PW], nxA[OA::PW], nxB[OB::PW];
  Geo cur = geo(t, offA, offB), nxt = cur;
  issue(0, cur, offA, offB, 0);
  if (g.stagger && (g.stagger == 1 ? (slot & 1) : slot >= (g.per_xcd + 1) / 2)) {
    // a co-resident pair of blocks started together runs its epilogues (VALU) at the same time;
    // one of them starting late puts each epilogue beside the partner's K loop (MFMA)
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t0 < (uint64_t)g.delay) __builtin_amdgcn_s_sleep(2);
  }
  int gs = 0;  // the block's K step number across its tiles (stage = gs & 1)
  const int lr = lane & 15, q4 = lane >> 4, odd = q4 & 1;
#ifdef LGX_S8_CLOCK
  uint64_t ck0 = clock64(), ckl = ck0;
  uint32_t ckw = 0, ckb = 0, ckc = 0, cke = 0, ntl = 0, nks = 0;
#endif

  for (;;) {
    const Prob& P = g.p[cur.pi];
    const bool more = t + g.per_xcd < tend;
    // the tile's scalars (uniform: SGPRs, loaded once instead of per use)
    const int M = P.M, N = P.N, epi = P.epi;
    char* const Cp = P.C;
    float* const C32p = P.C32;
    const int64_t ldc = P.ldc, ldc32 = P.ldc32;
    const bool delu = KIND == LGX_S8_DX && (epi & LGX_S8_EPI_DELU);
    const bool has_add = KIND == LGX_S8_DX && P.addend != nullptr && P.add_cols > 0;
    const bool has_bias = KIND == LGX_S8_FWD && (epi & LGX_S8_EPI_BIAS);
    const bool full = cur.m0 + BM <= M && cur.n0 + BN <= N;  // no row / column checks
    f32x4 acc[NJ][4];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto compute = [&](int stage) {
      const char* st = lds + stage * STAGE;
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        bf16x8 ah[4], al[4], bh[NJ], bl[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) OB::frag(st + OA::IMG, wn + 16 * j, kk, lane, bh[j], bl[j]);
#pragma unroll
        for (int i = 0; i < 4; ++i) OA::frag(st, wm + 16 * i, kk, lane, ah[i], al[i]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[j], al[i], acc[j][i], 0, 0, 0);
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl[j], ah[i], acc[j][i], 0, 0, 0);
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[j], ah[i], acc[j][i], 0, 0, 0);
          }
      }
    };
    for (int k = 0; k + 1 < cur.nk; ++k) {
      S8CK(ckc);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      S8CK(ckw);
      asm volatile("s_barrier" ::: "memory");
      S8CK(ckb);
      issue((gs + 1) & 1, cur, offA, offB, k + 1);
      compute(gs & 1);
      ++gs;
    }
    // the last K step: the next tile's first step is staged, and the FWD bias requested before this
    // step's MFMAs, so their latency runs beside them
    S8CK(ckc);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    S8CK(ckw);
    asm volatile("s_barrier" ::: "memory");
    S8CK(ckb);
    if (more) {
      nxt = geo(t + g.per_xcd, nxA, nxB);
      issue((gs + 1) & 1, nxt, nxA, nxB, 0);
    }
    float bv[NJ][4];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int nq = cur.n0 + wn + 16 * j + 4 * q4;
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[j][r] = 0.f;
      if (has_bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[j][r] = P.bias[min(nq + r, N - 1)];
      }
    }
    compute(gs & 1);
    ++gs;
    S8CK(ckc);
#ifdef LGX_S8_CLOCK
    nks += cur.nk;
    ++ntl;
#endif
    // the DX epilogue operand per (j, i), all requested before the first use (clamped: no load under
    // a condition; after the MFMAs — beside them they would not fit the 256 registers): the ELU'
    // operand's half group (DELU) or the addend's 4 values (their bits) in one register set (a
    // problem has one or the other: launch_persistent)
    u32x4 yv[NJ][4];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int nq = cur.n0 + wn + 16 * j + 4 * q4;
      if (delu) {
        const int grp = min((cur.n0 + wn + 16 * j) / 8 + (q4 >> 1), (N - 1) / 8);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = min(cur.m0 + wm + 16 * i + lr, M - 1);
          yv[j][i] = *reinterpret_cast<const u32x4*>(P.act + (int64_t)m * P.ld_act + grp * 32 + odd * 16);
        }
      }
      if (has_add) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = min(cur.m0 + wm + 16 * i + lr, M - 1);
#pragma unroll
          for (int r = 0; r < 4; ++r)
            yv[j][i][r] = __float_as_uint(P.addend[(int64_t)m * P.ld_add + min(nq + r, P.add_cols - 1)]);
        }
      }
    }

    // ---- epilogue from the accumulators: lane (lr, q4) holds rows m0 + wm + 16 i + lr, columns
    // n0 + wn + 16 j + 4 q4 + r of acc[j][i][r]
    float cs[NJ][4];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[j][r] = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int nq = cur.n0 + wn + 16 * j + 4 * q4;  // this lane's first column
      const int grp = (cur.n0 + wn + 16 * j) / 8 + (q4 >> 1);
      bool colok[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) colok[r] = full || nq + r < N;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = cur.m0 + wm + 16 * i + lr;
        const bool rowok = full || m < M;
        float v[4] = {acc[j][i][0], acc[j][i][1], acc[j][i][2], acc[j][i][3]};
        if constexpr (KIND == LGX_S8_FWD) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += bv[j][r];
          if (epi & LGX_S8_EPI_ELU) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = elu(v[r]);
          }
        } else {
          if (delu) {
            u32x4 Y = yv[j][i];
            // lane l (even row) loaded the group's hi, lane l + 16 its lo: swap the halves so each
            // holds hi and lo of its own 4 columns (hi = {Y0, Y1}, lo = {Y2, Y3})
            const auto s0 = __builtin_amdgcn_permlane16_swap(Y[0], Y[2], false, false);
            const auto s1 = __builtin_amdgcn_permlane16_swap(Y[1], Y[3], false, false);
            const unsigned h0 = s0[0], l0 = s0[1], h1 = s1[0], l1 = s1[1];
            float y[4];
            y[0] = __uint_as_float(h0 << 16) + __uint_as_float(l0 << 16);
            y[1] = __uint_as_float(h0 & 0xffff0000u) + __uint_as_float(l0 & 0xffff0000u);
            y[2] = __uint_as_float(h1 << 16) + __uint_as_float(l1 << 16);
            y[3] = __uint_as_float(h1 & 0xffff0000u) + __uint_as_float(l1 & 0xffff0000u);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] *= y[r] > 0.f ? 1.f : y[r] + 1.f;
          }
          if (has_add) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += nq + r < P.add_cols ? __uint_as_float(yv[j][i][r]) : 0.f;
          }
        }
        if (!full) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = colok[r] ? v[r] : 0.f;  // zero pad columns
        }
        if (Cp != nullptr) {
          __bf16 h[4], lo[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            h[r] = (__bf16)v[r];
            lo[r] = (__bf16)(v[r] - (float)h[r]);
          }
          const auto s0 = __builtin_amdgcn_permlane16_swap(pack2(h[0], h[1]), pack2(lo[0], lo[1]), false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(pack2(h[2], h[3]), pack2(lo[2], lo[3]), false, false);
          // even-row lanes: {own hi, partner hi} = the group's 8 hi; odd-row: its 8 lo
          const u32x4 out = {s0[0], s1[0], s0[1], s1[1]};
          if (rowok && (full || grp * 8 < N))
            *reinterpret_cast<u32x4*>(Cp + (int64_t)m * ldc + grp * 32 + odd * 16) = out;
        }
        if (C32p != nullptr && rowok) {
          float* d = C32p + (int64_t)m * ldc32 + nq;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (colok[r]) d[r] = v[r];
        }
        if (rowok) {
#pragma unroll
          for (int r = 0; r < 4; ++r) cs[j][r] += v[r];
        }
      }
    }
    if (P.colsum_ws != nullptr) {
      // per 64-row half tile: partial index (m0 + wm) / 64, columns n of this wave
      const int part = (cur.m0 + wm) / LGX_S8_TILE_M;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int nq = cur.n0 + wn + 16 * j + 4 * q4;
        float sv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) sv[r] = dpp_row_sum(cs[j][r]);
        if (lr == 0 && cur.m0 + wm < M) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (nq + r < N) P.colsum_ws[(int64_t)part * N + nq + r] = sv[r];
        }
      }
    }
    S8CK(cke);
    if (!more) break;
    t += g.per_xcd;
    cur = nxt;
#pragma unroll
    for (int u = 0; u < OA::PW; ++u) offA[u] = nxA[u];
#pragma unroll
    for (int u = 0; u < OB::PW; ++u) offB[u] = nxB[u];
  }
#ifdef LGX_S8_CLOCK
  if (lane == 0 && (wave == 0 || wave == NW - 1) && g_s8clk != nullptr) {
    const uint64_t tn = clock64();
    uint32_t* o = g_s8clk + ((size_t)blockIdx.x * 2 + (wave != 0)) * 12;
    o[0] = ckw; o[1] = ckb; o[2] = ckc; o[3] = cke; o[4] = (uint32_t)(tn - ck0);
    o[5] = nks; o[6] = __builtin_amdgcn_s_getreg(20 | (31 << 11)) & 15; o[7] = ntl;
  }
#endif
}


// ---- host launcher
static bool persistent_on() {
  static int on = -1;
  if (on < 0) {
    const char* e = LGX_DEV_KNOB("LGX_S8_PERSIST");  // dev knob: 0 = the per-tile kernel for FWD / DX
#ifndef LGX_S8_PERSIST_DEFAULT
#define LGX_S8_PERSIST_DEFAULT 1  // (dev builds: -DLGX_S8_PERSIST_DEFAULT=0 for the A/B variant)
#endif
    on = e ? atoi(e) != 0 : LGX_S8_PERSIST_DEFAULT;
  }
  return on != 0;
}

// The persistent FWD / DX launch: problems ordered by per-tile cost (K steps + an epilogue
// allowance), so each block's last tiles are the cheapest; the tile list cut into 8 contiguous
// XCD ranges of equal cost (an XCD's blocks share its L2: a row tile's column tiles stay together);
// up to 2 blocks per CU (64 per XCD), block s of XCD slot x taking every per_xcd-th tile from s.
template <int KIND>
static void launch_persistent(const lgxs::Group& g0, hipStream_t s) {
  lgxs::PGroup g;
  memset(&g, 0, sizeof g);
  int order[lgxs::GMAX];
  for (int i = 0; i < g0.n; ++i) order[i] = i;
  constexpr int EPI = 4;  // epilogue allowance in K steps
  auto nk = [&](int i) { return (g0.p[i].K + lgxs::BK - 1) / lgxs::BK; };
  std::stable_sort(order, order + g0.n, [&](int a, int b) { return nk(a) > nk(b); });
  int64_t total = 0;
  int ntiles = 0;
  for (int k = 0; k < g0.n; ++k) {
    g.p[k] = g0.p[order[k]];
    g.start[k] = ntiles;
    ntiles += g.p[k].tiles;
    total += (int64_t)g.p[k].tiles * (nk(order[k]) + EPI);
  }
  g.n = g0.n;
  g.start[g.n] = ntiles;
  // contiguous XCD ranges of (about) equal cost
  g.xstart[0] = 0;
  int x = 1, pi = 0;
  int64_t acc = 0;
  for (int tt = 0; tt < ntiles && x < 8; ++tt) {
    while (tt >= g.start[pi + 1]) ++pi;
    acc += nk(order[pi]) + EPI;
    if (acc * 8 >= total * x) g.xstart[x++] = tt + 1;
  }
  while (x <= 8) g.xstart[x++] = ntiles;
  int mx = 0;
  for (int k = 0; k < 8; ++k) mx = std::max(mx, g.xstart[k + 1] - g.xstart[k]);
  static int st = -1, dl = 0, cap = 64;
  if (st < 0) {
    const char* e = LGX_DEV_KNOB("LGX_S8_STAGGER");
    const char* d = LGX_DEV_KNOB("LGX_S8_STAGGER_DELAY");
    const char* c = LGX_DEV_KNOB("LGX_S8_PERSIST_CAP");  // blocks per XCD slot (large: one tile per block)
    st = e ? atoi(e) : 0;
    dl = d ? atoi(d) : 10000;
    cap = c ? std::max(1, atoi(c)) : 64;
  }
  g.per_xcd = std::min(mx, cap);
  {
    g.stagger = st;
    g.delay = dl;
  }
  constexpr int lds = lgxs::Cfg::LDS_STAGES;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)lgxs::s8p_kernel<KIND>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  if (g.per_xcd > 0)
    hipLaunchKernelGGL((lgxs::s8p_kernel<KIND>), dim3(8 * g.per_xcd), dim3(lgxs::Cfg::NT), lds, s, g);
}

