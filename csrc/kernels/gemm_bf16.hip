// bf16 GEMM on the gfx950 bf16 matrix cores (v_mfma_f32_16x16x32_bf16), f32
// accumulate, with fused epilogues.  This is the workhorse of the north-star
// models (BERT-base linear layers, ResNet-50 convolutions as implicit GEMM,
// BASELINE.json configs 4-5); the reference itself only runs f32 dense layers
// (worker.py:50-53), which use gemm_f32.hip.
//
//   C[M,N] = epi( alpha * op(A)[M,K] . op(B)[K,N] )
//   op(A) = A stored [M][lda] (k contiguous)      or A^T, A stored [K][lda]
//   op(B) = B stored [K][ldb] (n contiguous)      or B^T, B stored [N][ldb]
//
// so the three products of a linear layer need no transpose pass:
//   forward  Y  = X . W^T       (TA=0, TB=1)
//   dgrad    dX = dY . W        (TA=0, TB=0)
//   wgrad    dW = dY^T . X      (TA=1, TB=0)
//
// Epilogue (all optional, in this order, f32):
//   v = alpha*acc  (+ bias[n])  -> aux_out[m][n] = v (pre-activation, bf16)
//   v = act(v)                   (gelu(tanh) / relu; act 3: gelu, and aux_out receives
//                                 gelu'(v) instead of v)
//   v *= act'(aux_in[m][n])      (backward through an activation; act_grad 3: v *= aux_in,
//                                 the derivative an act-3 forward stored)
//   v += residual[m][n]          (bf16; convolutions: added BEFORE act', so a conv dgrad
//                                 can emit dL/d(BN output) = (dgrad + shortcut) * relu'(y))
//   v += beta * C_old            (f32 output only: gradient accumulation)
//   C = v as bf16 or f32
//
// Tiling: 128x128 output tile per 256-thread workgroup (4 waves, 2x2, each a
// 64x64 sub-tile = 4x4 MFMA tiles), BK = 64, two LDS buffers of 32 KB.
// Operand tiles are staged HBM->LDS with global_load_lds_dwordx4 (no VGPR
// round trip; lane-linear LDS destination, so the bank swizzle is applied to
// the per-lane SOURCE address).  LDS images keep the global layout of each
// operand:
//   k-contiguous operand  -> [128 rows][64 k]  128-B rows, fragments by
//                            ds_read_b128, 16-B chunk c of row r stored at
//                            chunk c ^ ((r >> 1) & 7)
//   k-strided operand     -> [64 k][128 cols]  256-B rows, fragments by
//                            two ds_read_b64_tr_b16 (hardware transpose),
//                            chunk c of k-row r stored at c ^ swz_tr(r)
// The next K tile is in flight while the current one feeds the MFMAs (one
// barrier per K tile).  Block ids are XCD-remapped (bijective) so the tiles
// that share an A row-panel run on one XCD's L2.
//
// Shape contract (checked on the host): K % 64 == 0, lda/ldb % 8 == 0 and
// 16-byte aligned bases; M, N arbitrary (edge rows are clamped on load and
// masked on store).
#include "gemm_bf16_common.h"

#include <cstdlib>
#include <stdexcept>
#include <string>

namespace dtfx {

// Tile BM_ x BN_ (128x128: 4 waves of 64x64, 2 blocks/CU; 256x128: 8 waves of 64x64;
// 256x256: 8 waves of 128x64; 256x64 (conv fwd with 64 output channels): 4 waves of 64x64
// stacked along M, 2 blocks/CU -- no MFMA work on a 128-wide tile's dead half).  NBUF = LDS stages (2: next tile in flight during
// compute; 3: two tiles in flight, counted vmcnt + raw barrier).
// a value the compiler cannot see through (no code): keeps per-tile address math in the tile loop
__device__ __forceinline__ int opaque_v(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

template <int MODE, bool TA, bool TB, bool OUT_F32, int BM_, int NBUF, int BN_, bool F1 = false,
          bool PERS = false>
__global__ __launch_bounds__(NBUF == 8 ? 512 : (BM_ / (BN_ == 256 ? 128 : 64)) * (BN_ / 64) * 64,
                             (BM_ == 128 || BN_ == 64) && NBUF == 2 ? 2 : 1) void gemm_bf16_kernel(
    int M, int N, int K, const unsigned short* __restrict__ A, int lda,
    const unsigned short* __restrict__ B, int ldb, void* __restrict__ Cv, int ldc, GemmEpi e,
    long long sA, long long sB, long long sC, ConvDesc cd) {
  using namespace gb;
  static_assert(!PERS || (NBUF == 8 && MODE == 0), "the persistent tile loop: 8-phase plain GEMM");
  constexpr int BM = BM_, BN = BN_;
  // wave tile WM x 64 (8-phase: 4 pieces of 32 x SW, one per block quadrant, 8 waves)
  constexpr int WM = (BN_ == 256 || NBUF == 8) ? 128 : 64;
  constexpr int NWN = NBUF == 8 ? 4 : BN / 64, NW = NBUF == 8 ? 8 : (BM / WM) * NWN;
  constexpr int TM = WM / 16;                      // 16-row MFMA tiles per wave
  constexpr int NQN = BN / 2, SW = NQN / 2;        // 8-phase: B half width, wave slab width
  static_assert(BN_ == 128 || MODE == 0 || MODE == 1 || (MODE == 2 && BN_ == 64) || NBUF == 8,
                "gathered B operands need BN = 128 (dgrad: or 64) or the 8-phase tile");
  constexpr int TILE_A = BM * BK * 2, TILE_B = BN * BK * 2, BUF_BYTES = TILE_A + TILE_B;
  constexpr int LPT = (BM / 8) / NW + (BN / 8) / NW;  // glds per thread per K tile
  // strided batch over blockIdx.z (attention's per-(batch, head) products)
  A += sA * blockIdx.z;
  B += sB * blockIdx.z;
  Cv = (char*)Cv + sC * blockIdx.z * (OUT_F32 ? 4 : 2);
  if constexpr (MODE == 2) {  // phase class blockIdx.z: its pixels, its taps
    M = dgrad_class(cd, blockIdx.z);
    K = cd.ktot;
  }
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  // Split-K (gridDim.y > 1): one XCD-contiguous range of (split, tile) pairs per XCD, so the
  // tiles of one K chunk -- which read the same operand rows (conv wgrad: the same dy chunk
  // and the same x neighbourhood for every tap) -- share that XCD's L2 instead of fetching
  // them once per XCD.  Otherwise the tiles sharing an A row-panel are XCD-contiguous.
  int bid, split;
  if (gridDim.y > 1) {
    const int T = tiles_n * tiles_m;
    const int lam = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y);
    bid = lam % T;
    split = lam / T;
  } else {
    // (MODE 2: the grid is sized for the largest phase class)
    bid = xcd_remap(blockIdx.x, MODE == 2 ? (int)gridDim.x : tiles_n * tiles_m);
    split = 0;
    if (MODE == 2 && bid >= tiles_n * tiles_m) return;
  }
  // tile id -> (first row, first column); grouped raster on the 8-phase tile: an XCD's
  // consecutive tile ids walk GM tile-rows column by column, so its ~32 resident blocks share 4
  // A and ~8 B panels in its L2 instead of 1 A and 32 B
  auto tile_origin = [&](int tid, int& mo, int& no) {
    int tm = tid / tiles_n, tn = tid % tiles_n;
    if (NBUF == 8 && gridDim.y == 1) {
      const int GM = 4, group = GM * tiles_n, fm = (tid / group) * GM;
      const int gm = min(tiles_m - fm, GM), r = tid % group;
      tm = fm + r % gm;
      tn = r / gm;
    }
    mo = tm * BM;
    no = tn * BN;
  };
  int m0, n0;
  tile_origin(bid, m0, n0);
  // PERS (persistent tile loop, one resident block per CU): this block runs virtual blocks
  // blockIdx.x, + gridDim.x, ... -- tile xcd_remap(vb) of each, the tile the one-shot grid's
  // block vb would run (gridDim.x % 8 == 0 keeps vb on this block's XCD), so every round of
  // 256 tiles shares its panels in the XCDs' L2 exactly as before.  The next tile's first K
  // tile is staged into LDS buffer 0 before this tile's epilogue (which then uses buffer 1 and
  // the LDS past the 8 half images), so its HBM round trip overlaps the epilogue instead of
  // following a fresh block's dispatch.
  int vb = blockIdx.x;
  bool pre = false;  // PERS: buffer 0 already holds this tile's first K tile
  // Clamp limits for edge tiles: k-contiguous rows clamp to the last row; k-strided
  // column chunks clamp to the last full 8-column chunk (ld % 8 == 0 makes it in-bounds).
  const int a_max = TA ? ((M - 1) & ~7) : M - 1;
  const int b_max = TB ? N - 1 : ((N - 1) & ~7);

  for (;;) {  // PERS: one iteration per tile of this block (otherwise exactly one)
  // (PERS: the lane / wave ids pass an opaque copy per tile, so the lane-dependent address math
  // of the staging, the fragment reads and the epilogue is formed again per tile instead of
  // being hoisted out of the tile loop and held live through it -- which spilled)
  const int lane = PERS ? opaque_v(threadIdx.x & 63) : threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(PERS ? opaque_v(threadIdx.x >> 6) : threadIdx.x >> 6);
  const int wm = wave / NWN, wn = wave % NWN;
  f32x4 acc[TM][4];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // split-K: split owns K tiles [kt0, kt0 + nk)
  const int nk_all = (K + BK - 1) / BK, per = (nk_all + gridDim.y - 1) / gridDim.y;
  const int kt0 = split * per;
  const int nk = max(0, min(per, nk_all - kt0));
  RowState rs;
  if (NBUF != 8 && (MODE == 1 || MODE == 2)) conv_rows<NW, BM / 8 / NW>(cd, MODE, M, m0, wave, lane, rs);
  Im2colCols ics;  // MODE 3: the lane's gathered columns, decoded once
  if constexpr (MODE == 3) im2col_cols<NW>(cd, n0, wave, lane, ics);
  auto stage_all = [&](int buf, int kt) {
    char* base = smem + buf * BUF_BYTES;
    const int k0 = (kt0 + kt) * BK;
    if (MODE == 1 || MODE == 2) stage_a_conv<NW, BM / 8 / NW>(cd, MODE, rs, A, k0, base, wave, lane);
    else stage<!TA, BM, NW>(A, lda, m0, a_max, k0, base, wave, lane, K - 1);
    if (MODE == 2) stage_b_wtap<NW, BN>(cd, B, n0, k0, base + TILE_A, wave, lane);
    else if (MODE == 3) stage_b_im2col_h<NW>(cd, B, K, k0, ics, base + TILE_A, wave, lane);
    else stage<TB, BN, NW>(B, ldb, n0, b_max, k0, base + TILE_A, wave, lane, K - 1);
  };
  auto compute = [&](int buf) {
    const char* At = smem + buf * BUF_BYTES;
    const char* Bt = At + TILE_A;
    if constexpr (NBUF == 2 && ((BM_ == 128 && BN_ == 128) || (BM_ == 256 && BN_ == 64))) {
      // 128x128 / 256x64 (two blocks per CU, 64x64 per wave): both k-halves' fragments are requested before the
      // first MFMA (half 1's LDS latency hides under half 0's MFMAs) and the MFMAs issue at
      // raised priority, so the partner wave on the SIMD does its reads in the gaps
      bf16x8 af2[2][TM], bf2[2][4];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int i = 0; i < TM; ++i) af2[kk][i] = frag<!TA, BM>(At, wm * WM + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) bf2[kk][j] = frag<TB, BN>(Bt, wn * 64 + j * 16, kk, lane);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af2[kk][i], bf2[kk][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      return;
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[TM], bfr[4];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = frag<!TA, BM>(At, wm * WM + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag<TB, BN>(Bt, wn * 64 + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  if constexpr (NBUF == 8) {
    // 8-phase schedule (256x256 tile, BK = 64, 8 waves, 128 KB of LDS as 8 half-tile
    // images of 16 KB: [buffer 0/1][A rows 0-127, A rows 128-255, B cols 0-127, B cols
    // 128-255]).  A K tile is four phases, one per block quadrant (MQ, NQ) in the order
    // (0,0) (1,0) (1,1) (0,1); in each quadrant wave (wm8, wn8) = (wave / 2, wave % 2) owns
    // a 32 x 64 piece (2 x 4 MFMA tiles, K = 64: 16 MFMAs).  Fragments are kept across
    // phases (A0 + B0 read in phase 1, A1 in 2, B1 in 3, A0 again in 4), so the half images
    // retire one per phase and every phase restages ONE half image (2 LDS-DMA loads per
    // thread); the schedule is listed at the loop.  Counted vmcnt (never 0 inside the loop
    // while a next tile exists) and raw s_barrier everywhere: __syncthreads' fence would
    // drain every DMA in flight.  One K tile per iteration with the buffer parity computed at
    // run time: a two-tile body with literal buffers let hipcc hoist a per-lane LDS address
    // for every buffer x half x fragment and spill ~100 VGPRs.
    // (cdna_hip_programming.md §5 "The 256^2 8-phase template" and its glds rules.)
    constexpr int HB = 16384;
    const int wm8 = wave >> 1, wn8 = wave & 1;
    auto hbuf = [&](int buf, int which) -> char* { return smem + (buf * 4 + which) * HB; };
    // Staging through buffer loads with LDS destination: each lane's byte offset at k = 0 is
    // computed ONCE (8 VGPRs for the 4 half images x 2 instructions); the K advance is the
    // wave-uniform soffset.  (64-bit per-lane pointers for 8 staging sites spilled.)
    // Convolutions (MODE 1 / 2): the A rows are gathered pixels.  NHWC makes a tap's offset
    // from the pixel the same for every lane, so each lane keeps its row's pixel base and
    // (y0, x0) and per K tile forms base + tap delta, or an offset past the buffer's extent
    // (the hardware then returns zeros) for padding taps and rows past M; the channel offset
    // inside the tap is the uniform soffset.  (Host: source < 2 GB, channels % 64 == 0.)
    constexpr bool CONV8 = MODE == 1 || MODE == 2;
    const int csh = MODE == 1 ? cd.H : cd.OH, csw = MODE == 1 ? cd.W : cd.OW;  // source image
    const int cch = MODE == 1 ? cd.C : cd.K;                                   // source channels
    const int a_bytes = CONV8 ? (int)min((long long)cd.N * csh * csw * cch * 2, 0x7fffffffLL) : 0x7fffffff;
    const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, a_bytes, 0x00020000);
    int cpb[4] = {0, 0, 0, 0}, cyx[4] = {0, 0, 0, 0};  // per A row (half * 2 + i): pixel base, y0 << 16 | x0
    // F1 (its own instantiation, cfg 7): a 1x1 / stride-1 / pad-0 convolution (forward, or the
    // data gradient's single phase class).  Every row reads its own pixel for every K tile, so
    // the row's byte offset is final at setup (cpb holds it) and a K tile is the uniform
    // soffset alone: no per-tile tap decode (scalar divisions + per-load address math left
    // these products 34-46 % behind the plain GEMM on the same tile; a runtime branch for it
    // slowed the 3x3 instantiation: profiles/r4/resnet_fast1_negative/)
    if constexpr (CONV8) {
      const int PW = MODE == 1 ? cd.OW : cd.Wc, PHW = MODE == 1 ? cd.OH * cd.OW : cd.Hc * cd.Wc;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + (r >> 1) * 128 + ((r & 1) * NW + wave) * 8 + (lane >> 3);
        int n, rem, py, px;
        fdivmod(min(m, M - 1), PHW, 1.f / PHW, n, rem);
        fdivmod(rem, PW, 1.f / PW, py, px);
        const int y0 = m < M ? (MODE == 1 ? py * cd.stride - cd.pad : py + cd.oy) : -30000;
        const int x0 = MODE == 1 ? px * cd.stride - cd.pad : px + cd.ox;
        cpb[r] = (n * csh + y0) * csw + x0;
        cyx[r] = (y0 << 16) | (x0 & 0xffff);
        if constexpr (F1) {
          const int row = ((r & 1) * NW + wave) * 8 + (lane >> 3);
          cpb[r] = m < M ? cpb[r] * cch * 2 + (((lane & 7) ^ swz_kc(row)) << 4) : (int)0x80000000;
        }
      }
    }
    auto conv_stage_a = [&](int buf, int which, int kt) {
      if constexpr (F1) {
        const int k0f = (kt0 + kt) * BK;
        char* df = smem + (buf * 4 + which) * 16384;
#pragma unroll
        for (int i = 0; i < 2; ++i)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void*)(df + (i * NW + wave) * 1024), 16,
                                                   cpb[which * 2 + i], k0f * 2, 0, 0);
        return;
      }
      const int k0 = (kt0 + kt) * BK, tap = k0 / cch, ch0 = k0 - tap * cch;
      const int tw_ = MODE == 1 ? cd.KW : max(cd.nkw, 1);
      const int th = tap / tw_, tw = tap - th * tw_;
      const int dy = MODE == 1 ? th : -th, dx = MODE == 1 ? tw : -tw;  // source pixel delta
      char* d_ = smem + (buf * 4 + which) * 16384;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = which * 2 + i, row = (i * NW + wave) * 8 + (lane >> 3);
        const int y = (cyx[r] >> 16) + dy, x = (int)(short)(cyx[r] & 0xffff) + dx;
        const bool ok = (unsigned)y < (unsigned)csh && (unsigned)x < (unsigned)csw;
        const int vo = ok ? (cpb[r] + dy * csw + dx) * cch * 2 + (((lane & 7) ^ swz_kc(row)) << 4)
                          : (int)0x80000000;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void*)(d_ + (i * NW + wave) * 1024), 16, vo,
                                                 ch0 * 2, 0, 0);
      }
    };
    // MODE 2 B (weights, k-strided [64 co][ci] image): row co0 + kr of the tap's column block
    auto wtap_soff = [&](int kt) {
      if constexpr (F1) return (kt0 + kt) * BK * ldb * 2;  // tap 0: weight row k0
      const int k0 = (kt0 + kt) * BK, ctap = k0 / cd.K, co0 = k0 - ctap * cd.K;
      const int th = ctap / max(cd.nkw, 1), tw = ctap - th * cd.nkw;
      const int tap = (cd.kh0 + cd.stride * th) * cd.KW + cd.kw0 + cd.stride * tw;
      return (co0 * ldb + tap * cd.C) * 2;
    };
    const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, 0x7fffffff, 0x00020000);
    // MODE 3 (weight gradient) B = im2col(x) [64 pixels][256 columns j = (kh, kw, ci)]: a lane's
    // two loads per half image keep their k-rows and swizzled chunks, so their columns decode
    // ONCE here (wdh / wdw / wci, per half and load); each K tile decodes only its pixels.
    // Padding taps and pixels past K point past the buffer (the hardware returns zeros).
    int wdh[4] = {0, 0, 0, 0}, wdw[4] = {0, 0, 0, 0}, wci[4] = {0, 0, 0, 0}, wjok = 0;
    if constexpr (MODE == 3) {
      const int jtot = cd.KH * cd.KW * cd.C;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int kr = ((q & 1) * NW + wave) * 4 + (lane >> 4);
        const int j = n0 + (q >> 1) * NQN + (((lane & 15) ^ swz_tr(kr)) << 3);
        int tap, ci, kh, kw;
        fdivmod(min(j, jtot - 8), cd.C, 1.f / cd.C, tap, ci);
        fdivmod(tap, cd.KW, 1.f / cd.KW, kh, kw);
        wdh[q] = kh - cd.pad;
        wdw[q] = kw - cd.pad;
        wci[q] = ci;
        wjok |= (j < jtot ? 1 : 0) << q;
      }
    }
    auto wg_stage_b = [&](int buf, int which, int kt) {
      const int k0 = (kt0 + kt) * BK, ohw = cd.OH * cd.OW;
      char* d_ = smem + (buf * 4 + which) * 16384;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int q = (which - 2) * 2 + i;
        const int kr = (i * NW + wave) * 4 + (lane >> 4), p = k0 + kr;
        int n, rem, oh, ow;
        fdivmod(min(p, K - 1), ohw, 1.f / ohw, n, rem);
        fdivmod(rem, cd.OW, 1.f / cd.OW, oh, ow);
        const int yy = oh * cd.stride + wdh[q], xx = ow * cd.stride + wdw[q];
        const bool ok = p < K && ((wjok >> q) & 1) && (unsigned)yy < (unsigned)cd.H &&
                        (unsigned)xx < (unsigned)cd.W;
        const int vo = ok ? (((n * cd.H + yy) * cd.W + xx) * cd.C + wci[q]) * 2 : (int)0x80000000;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void*)(d_ + (i * NW + wave) * 1024), 16, vo,
                                                 0, 0, 0);
      }
    };
    auto voffx = [&](bool isA, int which, int i, int mo, int no) -> int {
      const bool kc = isA ? !TA : TB;
      const int ld = isA ? lda : ldb, omax = isA ? a_max : b_max;
      // B halves start NQN apart (BN = 192: 96-column halves staged as 128-column images,
      // the last 32 columns loaded but never read)
      const int outer0 = isA ? mo + which * 128 : no + (which - 2) * NQN;
      const int blk = i * NW + wave;
      if (kc) {
        const int row = blk * 8 + (lane >> 3), c = (lane & 7) ^ swz_kc(row);
        return (min(outer0 + row, omax) * ld + c * 8) * 2;
      }
      const int kr = blk * 4 + (lane >> 4), c = (lane & 15) ^ swz_tr(kr);
      return (kr * ld + min(outer0 + c * 8, omax)) * 2;
    };
    auto voff = [&](bool isA, int which, int i) { return voffx(isA, which, i, m0, n0); };
    // (PERS: reassigned to the next tile's offsets for its buffer-0 prefetch after the K loop)
    int vo0_0 = voff(true, 0, 0), vo0_1 = voff(true, 0, 1);
    int vo1_0 = voff(true, 1, 0), vo1_1 = voff(true, 1, 1);
    int vo2_0 = voff(false, 2, 0), vo2_1 = voff(false, 2, 1);
    int vo3_0 = voff(false, 3, 0), vo3_1 = voff(false, 3, 1);
#define DTFX_PH8_STAGE(BUF, WHICH, KT)                                                          \
  do {                                                                                          \
    if constexpr (CONV8 && (WHICH) < 2) {                                                       \
      conv_stage_a((BUF), (WHICH), (KT));                                                       \
      break;                                                                                    \
    }                                                                                           \
    if constexpr (MODE == 3 && (WHICH) >= 2) {                                                  \
      wg_stage_b((BUF), (WHICH), (KT));                                                         \
      break;                                                                                    \
    }                                                                                           \
    const int k0_ = (kt0 + (KT)) * BK;                                                          \
    const int so_ = (WHICH) < 2 ? (TA ? k0_ * lda * 2 : k0_ * 2)                                \
                                : (MODE == 2 ? wtap_soff(KT) : TB ? k0_ * 2 : k0_ * ldb * 2);   \
    char* d_ = hbuf((BUF), (WHICH));                                                            \
    __builtin_amdgcn_raw_ptr_buffer_load_lds((WHICH) < 2 ? rA : rB, (lds_void*)(d_ + wave * 1024), \
                                             16, vo##WHICH##_0, so_, 0, 0);                     \
    __builtin_amdgcn_raw_ptr_buffer_load_lds((WHICH) < 2 ? rA : rB,                             \
                                             (lds_void*)(d_ + (NW + wave) * 1024), 16,          \
                                             vo##WHICH##_1, so_, 0, 0);                         \
  } while (0)
    bf16x8 af[2][2], bq[4][2];
    auto loadA = [&](int buf, int mq) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) af[mi][kk] = frag<!TA, 128>(hbuf(buf, mq), wm8 * 32 + mi * 16, kk, lane);
    };
    auto loadB = [&](int buf, int nq) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int j = 0; j < SW / 16; ++j) bq[j][kk] = frag<TB, 128>(hbuf(buf, 2 + nq), wn8 * SW + j * 16, kk, lane);
    };
#define DTFX_PH8_MMA(Q)                                                                         \
  __builtin_amdgcn_s_barrier();                                                                 \
  __builtin_amdgcn_sched_barrier(0);                                                            \
  __builtin_amdgcn_s_setprio(1);                                                                \
  _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                              \
  _Pragma("unroll") for (int mi = 0; mi < 2; ++mi)                                              \
  _Pragma("unroll") for (int j = 0; j < SW / 16; ++j)                                           \
    acc[(Q) * 2 + mi][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi][kk], bq[j][kk],       \
                                                                   acc[(Q) * 2 + mi][j], 0, 0, 0); \
  __builtin_amdgcn_s_setprio(0);                                                                \
  __builtin_amdgcn_sched_barrier(0);                                                            \
  __builtin_amdgcn_s_barrier();                                                                 \
  __builtin_amdgcn_sched_barrier(0);
    // Waves 4-7 (the second wave of every SIMD) run one barrier behind waves 0-3, so on each
    // SIMD one wave issues its 16 MFMAs while the other reads fragments / issues its staging
    // (cdna_hip_programming.md: the template's `if (wr == 1) s_barrier`).  With the groups a
    // barrier apart a half image is restaged TWO phases after its last read (WAR), and read
    // at least one phase after the vmcnt that retires it (RAW).
    //   iteration kt (buffer b = kt & 1):
    //     phase 1 (0,0): read A0 B0   stage B1 of tile kt+1 -> b^1 (B1 of b^1 last read kt-1 ph3)
    //     phase 2 (1,0): read A1      stage A0 of tile kt+1 -> b^1 (read kt-1 ph4)
    //     phase 3 (1,1): read B1      stage B0 of tile kt+2 -> b   (read ph1)
    //     phase 4 (0,1): read A0      stage A1 of tile kt+2 -> b   (read ph2)
    //   vmcnt(4) in phase 4 retires tile kt+1 (its last half, A0, went out in phase 2).
    const bool late = wave >= NW / 2;
    // prologue: tile 0 -> buffer 0 (PERS: staged before the previous tile's epilogue); tile
    // 1's B0 and A1 halves -> buffer 1
    if (nk > 0 && !pre) {
      DTFX_PH8_STAGE(0, 2, 0); DTFX_PH8_STAGE(0, 1, 0); DTFX_PH8_STAGE(0, 3, 0); DTFX_PH8_STAGE(0, 0, 0);
    }
    if (nk > 1) {
      DTFX_PH8_STAGE(1, 2, 1); DTFX_PH8_STAGE(1, 1, 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (late) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    for (int kt = 0; kt < nk; ++kt) {
      const int b = kt & 1;
      const bool has1 = kt + 1 < nk, has2 = kt + 2 < nk;
      loadA(b, 0); loadB(b, 0);                       // phase 1: quadrant (0,0)
      if (has1) DTFX_PH8_STAGE(b ^ 1, 3, kt + 1);
      DTFX_PH8_MMA(0)
      loadA(b, 1);                                    // phase 2: (1,0), B0 kept
      if (has1) DTFX_PH8_STAGE(b ^ 1, 0, kt + 1);
      DTFX_PH8_MMA(2)
      loadB(b, 1);                                    // phase 3: (1,1), A1 kept
      if (has2) DTFX_PH8_STAGE(b, 2, kt + 2);
      DTFX_PH8_MMA(3)
      loadA(b, 0);                                    // phase 4: (0,1), B1 kept
      if (has2) DTFX_PH8_STAGE(b, 1, kt + 2);
      if (has2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      DTFX_PH8_MMA(1)
    }
    if (!late) __builtin_amdgcn_s_barrier();  // the early group's share of the offset
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (PERS) {
      // every wave has read its last fragments: buffer 0 is free.  The next tile's first K tile
      // (4 half images, soffset 0: MODE 0) goes out now, ahead of this tile's epilogue stores.
      __syncthreads();
      pre = false;
      if (vb + (int)gridDim.x < tiles_n * tiles_m && nk > 0) {
        int mn, nn;
        tile_origin(xcd_remap(vb + (int)gridDim.x, tiles_n * tiles_m), mn, nn);
        // (the prologue's order B0, A1, B1, A0: the DTFX_PH8_STAGE sites with the next
        // tile's lane offsets and soffset 0)
        vo2_0 = voffx(false, 2, 0, mn, nn); vo2_1 = voffx(false, 2, 1, mn, nn);
        vo1_0 = voffx(true, 1, 0, mn, nn); vo1_1 = voffx(true, 1, 1, mn, nn);
        vo3_0 = voffx(false, 3, 0, mn, nn); vo3_1 = voffx(false, 3, 1, mn, nn);
        vo0_0 = voffx(true, 0, 0, mn, nn); vo0_1 = voffx(true, 0, 1, mn, nn);
        DTFX_PH8_STAGE(0, 2, -kt0); DTFX_PH8_STAGE(0, 1, -kt0);
        DTFX_PH8_STAGE(0, 3, -kt0); DTFX_PH8_STAGE(0, 0, -kt0);
        pre = true;
      }
    }
#undef DTFX_PH8_MMA
#undef DTFX_PH8_STAGE
  } else if (NBUF == 2) {
    if (nk > 0) stage_all(0, 0);
    __syncthreads();  // emits vmcnt(0): tile 0 landed for every wave
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) stage_all(cur ^ 1, kt + 1);
      compute(cur);
      __syncthreads();
    }
  } else {
    // 3 stages: tiles kt+1 and kt+2 in flight while tile kt computes.  Before computing
    // tile t every wave has retired its own loads of t (counted vmcnt: the younger tiles
    // stay in flight) and passed a barrier, so all waves' DMA into that buffer is visible.
    if (nk > 0) stage_all(0, 0);
    if (nk > 1) stage_all(1, 1);
    if (nk > 1) vm_barrier<LPT>();
    else vm_barrier<0>();
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      const bool issue = kt + 2 < nk;
      if (issue) stage_all(cur == 0 ? 2 : cur - 1, kt + 2);  // buffer of tile kt-1: retired
      compute(cur);
      // retire tile kt+1 (one younger tile may stay in flight)
      if (issue) vm_barrier<LPT>();
      else vm_barrier<0>();
      cur = cur == 2 ? 0 : cur + 1;
    }
  }
  if constexpr (!PERS) __syncthreads();

  // Epilogue.  The accumulators (C/D map: col = lane & 15, row = (lane >> 4) * 4 + r)
  // go through a per-wave LDS transpose, 32 rows at a time, so every lane then owns 8
  // consecutive columns of a row: bias / aux / residual / C_old are read and the
  // outputs written as 16-32 B vectors instead of 2-byte scattered accesses.
  // Each wave uses its own 32 x 68 f32 region (row pad 4 floats: the 4 row groups of a
  // ds_write land on distinct banks); the K loop's final barrier freed the buffers.
  constexpr int EP_LD = 68;
  // Side inputs of a slab are prefetched before its LDS transpose, except where the registers
  // are not there: f32 outputs, and the 8-phase dgrad with the fused BatchNorm backward
  // (3 side inputs beside 128 accumulators) -- those load at use.
  constexpr bool PREF = !OUT_F32 && !(NBUF == 8 && MODE == 2);
  // The 8-phase dgrad loads its side inputs per slab right after the slab's accumulators went
  // to LDS (their registers are free then): one memory round trip per 32-row slab.  Loaded at
  // use, each of the slab's 4 row groups waited on two dependent round trips (aux / residual,
  // then bn_x and the BN mean / rstd) -- ~25 us of exposed latency per block on the ResNet-50
  // layer3 / layer4 data gradients (3x3: 100 us against the forward's 75).
  constexpr bool LATE = NBUF == 8 && MODE == 2 && !OUT_F32;
  // (PERS: past LDS buffer 0, which holds the next tile's first K tile by now)
  constexpr int EP_BASE = PERS ? 65536 : 0, RED_BASE = PERS ? 65536 + 8 * 32 * EP_LD * 4 : 98304;
  float* ep = (float*)(smem + EP_BASE) + wave * (32 * EP_LD);
  const int col_l = lane & 15, row_l = (lane >> 4) * 4;
  float cs[8], cq[8];  // fused column sums / sums of squares of this lane's 8 columns
#pragma unroll
  for (int u = 0; u < 8; ++u) cs[u] = cq[u] = 0.f;
  float bmu[8], brs[8];  // BN mean / rstd of this lane's 8 columns (bn_x epilogue only)
  auto load_bn = [&](int c0) {
    const int n = n0 + c0 + (lane & 7) * 8;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      bmu[u] = n + u < N ? e.bn_mean[n + u] : 0.f;
      brs[u] = n + u < N ? e.bn_rstd[n + u] : 0.f;
    }
  };
  if (MODE == 2 && PREF && e.bn_x) load_bn(wn * 64);
  // Rows / columns of the wave's h-th 32 x 64 output slab: 8-phase layout (one slab per block
  // quadrant) or a contiguous WM x 64 wave tile.
  auto slab_r0 = [&](int h) { return NBUF == 8 ? (h >> 1) * 128 + (wave >> 1) * 32 : wm * WM + h * 32; };
  auto slab_c0 = [&](int h) { return NBUF == 8 ? (h & 1) * NQN + (wave & 1) * SW : wn * 64; };
  constexpr int SLW = NBUF == 8 ? SW : 64;  // slab width (columns)
  auto flush_cols = [&](int c0) {
    // lanes l, l^8, ..., l^56 hold the same 8 columns for different rows
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      cs[u] += __shfl_xor(cs[u], 8);
      cs[u] += __shfl_xor(cs[u], 16);
      cs[u] += __shfl_xor(cs[u], 32);
      cq[u] += __shfl_xor(cq[u], 8);
      cq[u] += __shfl_xor(cq[u], 16);
      cq[u] += __shfl_xor(cq[u], 32);
    }
    const int n = n0 + c0 + (lane & 7) * 8;
    if (e.col_partial) {
      // one partial row per 64-row wave slab (launchers use WM == 64 for partial stats)
      const size_t prow = (size_t)((MODE == 2 ? blockIdx.z * cd.prc : 0) + m0 / 64 + wm) * N;
      if (lane < 8 && m0 + wm * 64 < M)
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (n + u < N) {
            if (e.colsum) e.colsum[prow + n + u] = cs[u];
            if (e.colsq) e.colsq[prow + n + u] = cq[u];
          }
    } else if (lane < 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (n + u < N) {
          if (e.colsum) unsafeAtomicAdd(e.colsum + n + u, cs[u]);
          if (e.colsq) unsafeAtomicAdd(e.colsq + n + u, cq[u]);
        }
    }
  };
  // (unrolled for the late prefetch: a slab's accumulators are then known dead once they are in
  // LDS, and its side inputs take their registers)
#pragma unroll LATE ? 4 : 1
  for (int h = 0; h < WM / 32; ++h) {
    const int r0 = slab_r0(h), c0 = slab_c0(h);
    // (8-phase: consecutive slabs alternate between the two column halves)
    // (issued before the slab's LDS transpose, so their latency overlaps it)
    // Side inputs (aux_in / residual) of the slab's 4 row groups are all
    // loaded before any is used: one memory round trip per 32-row slab instead of one per
    // 8-row group (the loads used to sit between dependent compute and stores).
    bool full[4], live[4];
    int mm[4], nn[4], pm[4];  // pm: memory row of GEMM row mm (MODE 2: class pixel -> pixel)
    bf16x8 a8[4], r8[4], x8[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int rr = it * 8 + (lane >> 3), cg = (lane & 7) * 8;
      mm[it] = m0 + r0 + rr;
      nn[it] = n0 + c0 + cg;
      live[it] = mm[it] < M && nn[it] < N && cg < SLW;
      full[it] = live[it] && nn[it] + 8 <= N;  // N % 8 != 0 only with a ragged last group
      const int ms = live[it] ? mm[it] : 0, ns = full[it] ? nn[it] : 0;
      pm[it] = ms;
      if (MODE == 2 && cd.stride > 1) {
        int nimg, rem, i, j;
        fdivmod(ms, cd.Hc * cd.Wc, 1.f / (cd.Hc * cd.Wc), nimg, rem);
        fdivmod(rem, cd.Wc, 1.f / cd.Wc, i, j);
        pm[it] = (nimg * cd.H + i * cd.stride + cd.ph) * cd.W + j * cd.stride + cd.pw;
      }
      if (PREF) {
        if (e.act_grad) a8[it] = __builtin_nontemporal_load((const bf16x8*)&e.aux_in[(size_t)pm[it] * e.ld_aux + ns]);
        if (e.residual) r8[it] = __builtin_nontemporal_load((const bf16x8*)&e.residual[(size_t)pm[it] * e.ld_res + ns]);
        if (MODE == 2 && e.bn_x) x8[it] = *(const bf16x8*)&e.bn_x[(size_t)pm[it] * ldc + ns];
      }
    }
    // static accumulator indices only (a runtime acc[2h+ii] index would put acc in scratch)
#pragma unroll
    for (int t = 0; t < TM; ++t)
      if ((t >> 1) == h)
#pragma unroll
        for (int j = 0; j < SLW / 16; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            ep[((t & 1) * 16 + row_l + r) * EP_LD + j * 16 + col_l] = acc[t][j][r];
    if constexpr (LATE) {
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int ns = full[it] ? nn[it] : 0;
        if (e.act_grad) a8[it] = __builtin_nontemporal_load((const bf16x8*)&e.aux_in[(size_t)pm[it] * e.ld_aux + ns]);
        if (e.residual) r8[it] = __builtin_nontemporal_load((const bf16x8*)&e.residual[(size_t)pm[it] * e.ld_res + ns]);
        if (e.bn_x) x8[it] = *(const bf16x8*)&e.bn_x[(size_t)pm[it] * ldc + ns];
      }
      if (e.bn_x) {  // the lane's 8 columns are the same for the slab's 4 row groups
        const int nb = n0 + c0 + (lane & 7) * 8;
        if ((lane & 7) * 8 < SLW && nb + 8 <= N) {
          *(f32x4*)&bmu[0] = *(const f32x4*)&e.bn_mean[nb];
          *(f32x4*)&bmu[4] = *(const f32x4*)&e.bn_mean[nb + 4];
          *(f32x4*)&brs[0] = *(const f32x4*)&e.bn_rstd[nb];
          *(f32x4*)&brs[4] = *(const f32x4*)&e.bn_rstd[nb + 4];
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    if (OUT_F32 && gridDim.y > 1) {
      // split-K partial: alpha only; hardware f32 atomics, one 256-B row segment per
      // wave instruction (lane = column) so each instruction is 4 full 64-B requests
      const int n = n0 + c0 + lane;
      for (int rr = 0; rr < 32; ++rr) {
        const int m = m0 + r0 + rr;
        if (m < M && n < N && lane < SLW)
          if (e.ws) __builtin_nontemporal_store(e.alpha * ep[rr * EP_LD + lane], &e.ws[((size_t)split * M + m) * N + n]);
          else unsafeAtomicAdd((float*)Cv + (size_t)m * ldc + n, e.alpha * ep[rr * EP_LD + lane]);
      }
      __builtin_amdgcn_wave_barrier();
      continue;
    }
    // the bias of this lane's 8 columns: the same for the slab's 4 row groups, loaded once
    float bn[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) bn[u] = 0.f;
    if (e.bias) {
      const int nb = n0 + c0 + (lane & 7) * 8;
      if ((lane & 7) * 8 < SLW && nb + 8 <= N) {
        *(f32x4*)&bn[0] = *(const f32x4*)&e.bias[nb];
        *(f32x4*)&bn[4] = *(const f32x4*)&e.bias[nb + 4];
      } else if ((lane & 7) * 8 < SLW) {
        for (int u = 0; u < 8 && nb + u < N; ++u) bn[u] = e.bias[nb + u];
      }
    }
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int rr = it * 8 + (lane >> 3), cg = (lane & 7) * 8;
      const int n = nn[it];
      const size_t mp = pm[it];
      float v[8];
      *(f32x4*)&v[0] = *(const f32x4*)&ep[rr * EP_LD + cg];
      *(f32x4*)&v[4] = *(const f32x4*)&ep[rr * EP_LD + cg + 4];
      if (!live[it]) continue;
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = __builtin_fmaf(e.alpha, v[u], bn[u]);
      if (full[it]) {
        if (e.act == 3) {
          bf16x8 o;
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            float gp;
            v[u] = gelu_fg(v[u], gp);
            o[u] = (short)f2bf(gp);
          }
          __builtin_nontemporal_store(o, (bf16x8*)&e.aux_out[(size_t)mp * e.ld_aux + n]);
        } else if (e.aux_out) {
          bf16x8 o;
#pragma unroll
          for (int u = 0; u < 8; ++u) o[u] = (short)f2bf(v[u]);
          __builtin_nontemporal_store(o, (bf16x8*)&e.aux_out[(size_t)mp * e.ld_aux + n]);
        }
        if (e.act == 1) {
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = gelu_f(v[u]);
        } else if (e.act == 2) {
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = fmaxf(v[u], 0.f);
        }
        if (MODE != 0 && e.residual) {  // convolutions: shortcut gradient before the mask
          if (!PREF && !LATE) r8[it] = __builtin_nontemporal_load((const bf16x8*)&e.residual[(size_t)mp * e.ld_res + n]);
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] += bf2f((unsigned short)r8[it][u]);
        }
        if (e.act_grad) {
          if (!PREF && !LATE) a8[it] = __builtin_nontemporal_load((const bf16x8*)&e.aux_in[(size_t)mp * e.ld_aux + n]);
          if (e.act_grad == 3) {
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] *= bf2f((unsigned short)a8[it][u]);
          } else {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              const float uu = bf2f((unsigned short)a8[it][u]);
              v[u] *= (e.act_grad == 1) ? gelu_grad_f(uu) : (uu > 0.f ? 1.f : 0.f);
            }
          }
        }
        if (MODE == 0 && e.residual) {
          if (!PREF) r8[it] = __builtin_nontemporal_load((const bf16x8*)&e.residual[(size_t)mp * e.ld_res + n]);
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] += bf2f((unsigned short)r8[it][u]);
        }
        if (e.colsum || e.colsq) {
          if (MODE == 2 && !OUT_F32 && e.bn_x) {
            // statistics of the VALUES STORED (bf16-rounded), as a separate reduction over
            // the output tensor would see them
            if (!PREF && !LATE) {  // load at use: x, and the BN mean / rstd of the 8 columns
              x8[it] = *(const bf16x8*)&e.bn_x[mp * ldc + n];
              *(f32x4*)&bmu[0] = *(const f32x4*)&e.bn_mean[n];
              *(f32x4*)&bmu[4] = *(const f32x4*)&e.bn_mean[n + 4];
              *(f32x4*)&brs[0] = *(const f32x4*)&e.bn_rstd[n];
              *(f32x4*)&brs[4] = *(const f32x4*)&e.bn_rstd[n + 4];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              const float vr = bf2f(f2bf(v[u]));
              cs[u] += vr;
              cq[u] += vr * (bf2f((unsigned short)x8[it][u]) - bmu[u]) * brs[u];
            }
          } else {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              cs[u] += v[u];
              cq[u] += v[u] * v[u];
            }
          }
        }
        if (OUT_F32) {
          float* C = (float*)Cv + (size_t)mp * ldc + n;
          if (e.beta != 0.f) {  // (f32 outputs: C_old read here, no 32-VGPR slab batch)
            const f32x4 c0 = *(const f32x4*)C, c1 = *(const f32x4*)(C + 4);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              v[u] += e.beta * c0[u];
              v[u + 4] += e.beta * c1[u];
            }
          }
          __builtin_nontemporal_store(*(f32x4*)&v[0], (f32x4*)C);
          __builtin_nontemporal_store(*(f32x4*)&v[4], (f32x4*)(C + 4));
        } else {
          bf16x8 o;
#pragma unroll
          for (int u = 0; u < 8; ++u) o[u] = (short)f2bf(v[u]);
          // non-temporal (streaming) stores for the bf16 outputs and aux: +2-3 % on every GEMM
          // shape of tools/probes/gemm_k_sweep.py, BERT-base +0.8 %, ResNet-50 neutral
          // (profiles/r5/gemm_nt/)
          __builtin_nontemporal_store(o, (bf16x8*)((unsigned short*)Cv + (size_t)mp * ldc + n));
        }
      } else {
        if (MODE == 2 && !PREF && e.bn_x)
          for (int u = 0; u < 8 && n + u < N; ++u) {
            bmu[u] = e.bn_mean[n + u];
            brs[u] = e.bn_rstd[n + u];
          }
        for (int u = 0; u < 8 && n + u < N; ++u) {
          float w = v[u];
          if (e.act == 3) {
            float gp;
            w = gelu_fg(w, gp);
            e.aux_out[(size_t)mp * e.ld_aux + n + u] = f2bf(gp);
          } else if (e.aux_out) {
            e.aux_out[(size_t)mp * e.ld_aux + n + u] = f2bf(w);
          }
          if (e.act == 1) w = gelu_f(w);
          else if (e.act == 2) w = fmaxf(w, 0.f);
          if (MODE != 0 && e.residual) w += bf2f(e.residual[(size_t)mp * e.ld_res + n + u]);
          if (e.act_grad) {
            const float uu = bf2f(e.aux_in[(size_t)mp * e.ld_aux + n + u]);
            w *= (e.act_grad == 3) ? uu : (e.act_grad == 1) ? gelu_grad_f(uu) : (uu > 0.f ? 1.f : 0.f);
          }
          if (MODE == 0 && e.residual) w += bf2f(e.residual[(size_t)mp * e.ld_res + n + u]);
          if (MODE == 2 && !OUT_F32 && e.bn_x) {
            const float wr = bf2f(f2bf(w));
            cs[u] += wr;
            cq[u] += wr * (bf2f(e.bn_x[(size_t)mp * ldc + n + u]) - bmu[u]) * brs[u];
          } else {
            cs[u] += w;
            cq[u] += w * w;
          }
          if (OUT_F32) {
            float* C = (float*)Cv + (size_t)mp * ldc + n + u;
            *C = (e.beta != 0.f) ? w + e.beta * *C : w;
          } else {
            ((unsigned short*)Cv)[(size_t)mp * ldc + n + u] = f2bf(w);
          }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    if (NBUF == 8 && (e.colsum || e.colsq)) {
      // the next slab covers other columns: park this slab's column sums in LDS (beyond the
      // per-wave transpose regions), reduced across the block below -- one atomic per column
      // per block instead of one per slab and wave (8x fewer same-address atomics; the BERT
      // FFN dgrad with its fused bias gradient ran 225 us with per-slab atomics)
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        cs[u] += __shfl_xor(cs[u], 8);
        cs[u] += __shfl_xor(cs[u], 16);
        cs[u] += __shfl_xor(cs[u], 32);
        cq[u] += __shfl_xor(cq[u], 8);
        cq[u] += __shfl_xor(cq[u], 16);
        cq[u] += __shfl_xor(cq[u], 32);
      }
      float* red = (float*)(smem + RED_BASE);  // [colsum|colsq][Nq][wn8][wm8 * 2 + Mq][64]
      const int slot = (((h & 1) * 2 + (wave & 1)) * 8 + (wave >> 1) * 2 + (h >> 1)) * 64;
      if (lane < SLW / 8)
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          red[slot + lane * 8 + u] = cs[u];
          red[2048 + slot + lane * 8 + u] = cq[u];
        }
#pragma unroll
      for (int u = 0; u < 8; ++u) cs[u] = cq[u] = 0.f;
    }
  }
  if constexpr (NBUF == 8) {
    if (e.colsum || e.colsq) {
      __syncthreads();
      const float* red = (const float*)(smem + RED_BASE);
      if (e.col_partial && threadIdx.x < BN) {
        // partial rows, one per 64-row output slab (the conv launchers' layout, reduced by
        // colpart_reduce): slab g of the block is entries wm8 * 2 + Mq with Mq = g >> 1,
        // wm8 >> 1 = g & 1 (slab_r0: rows Mq * 128 + wm8 * 32)
        const int c = threadIdx.x, nq = c / NQN, w = (c % NQN) / SW, col = c % SW;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int i0 = (g & 1) * 4 + (g >> 1), i1 = i0 + 2;
          const int e0 = ((nq * 2 + w) * 8 + i0) * 64 + col, e1 = ((nq * 2 + w) * 8 + i1) * 64 + col;
          if (m0 + g * 64 < M && n0 + c < N) {
            const size_t prow = (size_t)((MODE == 2 ? blockIdx.z * cd.prc : 0) + m0 / 64 + g) * N + n0 + c;
            if (e.colsum) e.colsum[prow] = red[e0] + red[e1];
            if (e.colsq) e.colsq[prow] = red[2048 + e0] + red[2048 + e1];
          }
        }
      } else if (threadIdx.x < BN) {
        const int c = threadIdx.x, nq = c / NQN, w = (c % NQN) / SW, col = c % SW;
        float a = 0.f, q = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          a += red[((nq * 2 + w) * 8 + i) * 64 + col];
          q += red[2048 + ((nq * 2 + w) * 8 + i) * 64 + col];
        }
        if (n0 + c < N) {
          if (e.colsum) unsafeAtomicAdd(e.colsum + n0 + c, a);
          if (e.colsq) unsafeAtomicAdd(e.colsq + n0 + c, q);
        }
      }
    }
  } else if (e.colsum || e.colsq) {
    flush_cols(wn * 64);
  }
  if constexpr (!PERS) break;
  vb += gridDim.x;
  if (vb >= tiles_n * tiles_m) break;
  tile_origin(xcd_remap(vb, tiles_n * tiles_m), m0, n0);
  __syncthreads();  // the epilogue's LDS (buffer 1's image, the colsum rows) is free again
  }  // tile loop
}

// ---------------------------------------------------------------------------
// Launch-configuration choice.  cfg 0: 128x128 tile, 4 waves, 2 LDS stages (64 KB, 2 blocks
// per CU); cfg 1: 256x128, 8 waves, 3 stages (144 KB, counted-vmcnt pipeline); cfg 2:
// 256x128, 2 stages (96 KB); cfg 3 (plain GEMM only): 256x256, 8 waves of 128x64, 2 stages
// (128 KB); cfg 4 (convolutions): 256x64; cfg 5 (plain GEMM only): 256x256, 8-phase
// schedule (128 KB) -- the default large tile.  Auto: by wave quantisation (choose_cfg).
// DTFX_GEMM_CFG=0..5 or gemm_bf16_set_cfg() forces one (tests, benchmarks).
// ---------------------------------------------------------------------------
static int g_gemm_cfg = -2;  // -2: not read yet; -1: auto; 0..5 forced
static int gemm_cfg_env() {
  if (g_gemm_cfg == -2) {
    const char* e = getenv("DTFX_GEMM_CFG");
    g_gemm_cfg = e ? atoi(e) : -1;
  }
  return g_gemm_cfg;
}
// Force a tile configuration (-1 = auto) for tests and A/B benchmarks in one process.
void gemm_bf16_set_cfg(int cfg) { g_gemm_cfg = cfg; }

static int choose_cfg(int M, int N, int zdim, int mode, bool ta = false) {
  const int f = gemm_cfg_env();
  if (f >= 0 && f <= 6) return (f >= 5 && mode != 0) ? 0 : f;
  if (mode == 0) {
    // The 8-phase schedules (cfg 5: 256x256, cfg 6: 256x192) replaced the 2-stage 256x256
    // (cfg 3) on every BERT forward / dgrad shape and on squares (tools/gemm_cfg_ab.py,
    // interleaved rounds: ffn1 dgrad 16384x768x3072 987 (cfg 6) / 915 (cfg 5) vs 745 (cfg 3)
    // TFLOP/s, 4096^3 1303 vs 1209).  Choice by a time model calibrated on those shapes:
    // waves x tile work / relative per-block efficiency, one block per CU for the 8-phase
    // tiles, two for 128x128 (cfg 6: 0.75 of a 256x256 block's work at 0.81 of its efficiency
    // -- the N = 768 GEMMs fill all 256 CUs instead of 192; cfg 0: 0.25 at 0.47).
    // A^T operands (weight gradients) stay on 128x128 + split-K (760 vs 705 TFLOP/s).
    // DTFX_GEMM_TA8=1: weight gradients on the 8-phase tile too; =2: only the large ones
    // (>= 2 M outputs: BERT-base's FFN weight gradients, 808 vs 731 TFLOP/s standalone, while
    // the QKV one is slower there, 632 vs 730: profiles/r6/gemm/wgrad_cfg/)
    static const int ta8 = [] {
      const char* e = getenv("DTFX_GEMM_TA8");
      return e ? atoi(e) : 0;
    }();
    if (ta && (ta8 <= 0 || (ta8 == 2 && (long long)M * N < 2000000))) return 0;
    static const int big = [] {  // DTFX_GEMM_BIG=3: the previous 2-stage large tile (A/B runs)
      const char* e = getenv("DTFX_GEMM_BIG");
      return e && atoi(e) == 3 ? 3 : 5;
    }();
    const long long t3 = (long long)((M + 255) / 256) * ((N + 255) / 256) * zdim;
    const long long t6 = (long long)((M + 255) / 256) * ((N + 191) / 192) * zdim;
    const long long t0 = (long long)((M + 127) / 128) * ((N + 127) / 128) * zdim;
    if (big == 3) {
      if (t3 < 256) return 0;
      const double e3 = (double)t3 / (double)(((t3 + 255) / 256) * 256);
      const double e0 = (double)t0 / (double)(((t0 + 511) / 512) * 512);
      return e3 * 1.15 >= e0 ? 3 : 0;
    }
    const double est5 = (double)((t3 + 255) / 256);
    const double est6 = (double)((t6 + 255) / 256) * 0.75 / 0.81;
    const double est0 = (double)((t0 + 511) / 512) * 0.25 / 0.47;
    // cfg 6 is opt-in (DTFX_GEMM_TILE192=1): alone it is 6-8 % faster on the N = 768
    // GEMMs, but in the BERT step those run beside the weight-gradient kernels on a second
    // stream, which use the 64 CUs a 192-block 256x256 grid leaves free (BERT-base, same box,
    // two rounds: 7928 / 7890 seq/s with cfg 5 vs 7697 / 7639 with cfg 6; without the second
    // stream both ~7840 -- scripts/gpu_bert_ab.sh)
    static const bool use6 = [] {
      const char* e = getenv("DTFX_GEMM_TILE192");
      return e && atoi(e) == 1;
    }();
    if (use6 && est6 < est5 && est6 < est0 && N > 128) return 6;
    // vocabulary-wide outputs (BERT's MLM logits, 2432 x 30528 x 768): the model rates the
    // 128x128 tile 4 % ahead, the 8-phase tile measures 11 % ahead (735 vs 662 TFLOP/s,
    // profiles/r6/gemm/decoder/) -- within 10 % of the model, wide outputs take the big tile
    static const bool wide5 = [] {  // DTFX_GEMM_WIDE=0: the model's choice (A/B runs)
      const char* e = getenv("DTFX_GEMM_WIDE");
      return !(e && atoi(e) == 0);
    }();
    if (wide5 && zdim == 1 && !ta && N >= 16384 && t3 >= 256 && est5 <= est0 * 1.1) return 5;
    // the 8-phase tile with its sparse last round's rows on the 128x128 tile (gemm_tail_rows):
    // the whole rounds plus the tail's 128x128 rounds (BERT-base QKV: 2 + 0.53 against the
    // 128x128 tile's 2.66 -- 746 vs 737 TFLOP/s, profiles/r6/probe2/)
    if (zdim == 1 && !ta) {
      const long long F = t3 / 256, R = t3 % 256;
      const int tn = (N + 255) / 256;
      if (F >= 1 && R > 0 && R <= 128) {
        const int rows5 = (int)(F * 256 / tn) * 256;
        if (rows5 > 0 && rows5 < M) {
          const long long p5 = (long long)(rows5 / 256) * tn;
          const long long tt = (long long)((M - rows5 + 127) / 128) * ((N + 127) / 128);
          const double est5t = (double)((p5 + 255) / 256) + (double)((tt + 511) / 512) * 0.25 / 0.47;
          if (est5t < est5 && est5t < est0) return 5;
        }
      }
    }
    // (a 4-wave 256x256 tile with one 128 x 128 wave per SIMD -- hipBLASLt's pick for these
    // shapes -- measured slower in both its per-K-tile rate and its epilogue:
    // profiles/r3/bert_gemm/w4_tile.md, tools/probes/w4_bench.hip)
    return est5 <= est0 ? 5 : 0;
  }
  // convolutions (ResNet-50 end to end: 6881 img/s on 128x128 vs 6411-6416 on 256x128);
  // a forward conv with <= 64 output channels, or a dgrad with <= 64 input channels, takes
  // the 256x64 tile (no dead half)
  if ((mode == 1 || mode == 2) && N <= 64) return 4;
  return 0;
}

// Persistent 8-phase tile loop (PERS) for a plain GEMM whose 256x256 tiles
// fill more than one round of the CUs.  Opt-in (DTFX_GEMM_PERS=1): exact and bit-identical to
// one block per tile (tests/test_bf16_gpu.py), but per call 1-2.4 % SLOWER on every bf16-output
// shape (FFN1 forward 109.2 vs 106.5 us, QKV 72.6 vs 71.9, 8192^3 1415 vs 1432 TFLOP/s) and
// +2.4 % only with an f32 output; BERT-base 8,377-8,394 vs 8,387-8,389 seq/s
// (profiles/r6/gemm_pers/).  What the ~11 us per tile round is NOT, then: the block dispatch
// and the prologue's first K tile (both overlapped here).  It is the epilogue itself -- the LDS
// transpose and 128 KB of stores per block that the next tile's counted vmcnt waits out
// (gfx9 counts stores and loads in one vmcnt), so a store-overlapping epilogue would need
// separate store waves and LDS the 8-phase tile does not have free.
static int g_gemm_pers = -1;  // -1: read DTFX_GEMM_PERS on first use
static bool gemm_pers_on() {
  if (g_gemm_pers < 0) {
    const char* e = getenv("DTFX_GEMM_PERS");
    g_gemm_pers = e && atoi(e) == 1 ? 1 : 0;
  }
  return g_gemm_pers == 1;
}
int gemm_bf16_set_pers(int on) {  // tests / A/B in one process; returns the previous setting
  const int old = gemm_pers_on() ? 1 : 0;
  g_gemm_pers = on ? 1 : 0;
  return old;
}
static int gemm_num_cus() {
  static const int n = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return cus > 0 ? cus : 256;
  }();
  return n;
}

template <int MODE, bool TA, bool TB, bool F, int BM_, int NBUF, int BN_ = 128, bool F1 = false,
          bool PERS = false>
static void launch_one(dim3 grid_yz, int M, int N, int K, const unsigned short* A, int lda,
                       const unsigned short* B, int ldb, void* C, int ldc, const GemmEpi& e,
                       long long sA, long long sB, long long sC, const ConvDesc& d,
                       hipStream_t stream) {
  // 8-phase: 8 half-tile images of 16 KB; PERS: + the epilogue's transpose rows and column-sum
  // rows past buffer 0 (65536 + 8 x 8704 + 16384)
  constexpr size_t lds = PERS ? (size_t)151552
                       : NBUF == 8 ? (size_t)131072
                                   : (size_t)NBUF * (BM_ * gb::BK * 2 + BN_ * gb::BK * 2);
  constexpr int threads = NBUF == 8 ? 512 : (BM_ / (BN_ == 256 ? 128 : 64)) * (BN_ / 64) * 64;
  static bool attr = false;
  if (!attr) {
    DTFX_HIP_CHECK(hipFuncSetAttribute(
        (const void*)gemm_bf16_kernel<MODE, TA, TB, F, BM_, NBUF, BN_, F1, PERS>,
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  const int tiles = ((M + BM_ - 1) / BM_) * ((N + BN_ - 1) / BN_);
  // One K tile (and no split): only LDS stage 0 is ever staged, so the block needs just that
  // stage or the epilogue's per-wave transpose rows, whichever is larger -- three resident
  // 128x128 blocks per CU instead of two (ResNet-50 layer1 conv3 forward, K = 64: 236 -> 194
  // us; DTFX_GEMM_1STAGE=0: full stages)
  static const bool one_stage_ok = [] {
    const char* v = getenv("DTFX_GEMM_1STAGE");
    return v ? atoi(v) != 0 : true;
  }();
  size_t lds_launch = lds;
  if (NBUF == 2 && one_stage_ok && K <= gb::BK && grid_yz.y == 1) {
    const size_t stage = (size_t)(BM_ * gb::BK * 2 + BN_ * gb::BK * 2);
    const size_t ep = (size_t)(threads / 64) * 32 * 68 * 4;
    lds_launch = stage > ep ? stage : ep;
  }
  // PERS: one block per CU (a multiple of 8: a block's virtual ids stay on its XCD)
  const int gx = PERS ? (tiles < gemm_num_cus() ? tiles : gemm_num_cus() & ~7) : tiles;
  hipLaunchKernelGGL((gemm_bf16_kernel<MODE, TA, TB, F, BM_, NBUF, BN_, F1, PERS>),
                     dim3(gx, grid_yz.y, grid_yz.z), dim3(threads), lds_launch, stream, M, N, K, A, lda,
                     B, ldb, C, ldc, e, sA, sB, sC, d);
  DTFX_HIP_CHECK(hipGetLastError());
}

template <int MODE, bool TA, bool TB, bool F>
static void launch_cfg(int cfg, dim3 grid_yz, int M, int N, int K, const unsigned short* A, int lda,
                       const unsigned short* B, int ldb, void* C, int ldc, const GemmEpi& e,
                       long long sA, long long sB, long long sC, const ConvDesc& d,
                       hipStream_t stream) {
  if constexpr (MODE == 0) {
    if (cfg == 5) {
      // PERS instantiations: A k-contiguous, and B k-contiguous or an f32 output (the bf16
      // dY.W form with its prefetched epilogue side inputs spilled 15 VGPRs in the tile loop)
      if constexpr (!TA && (TB || F)) {
        const long long t5 = (long long)((M + 255) / 256) * ((N + 255) / 256);
        if (gemm_pers_on() && grid_yz.y == 1 && grid_yz.z == 1 && t5 > gemm_num_cus() &&
            gemm_num_cus() >= 8) {
          launch_one<MODE, TA, TB, F, 256, 8, 256, false, true>(grid_yz, M, N, K, A, lda, B, ldb,
                                                                C, ldc, e, sA, sB, sC, d, stream);
          return;
        }
      }
      launch_one<MODE, TA, TB, F, 256, 8, 256>(grid_yz, M, N, K, A, lda, B, ldb, C, ldc, e, sA,
                                               sB, sC, d, stream);
      return;
    }
    if (cfg == 6) {
      launch_one<MODE, TA, TB, F, 256, 8, 192>(grid_yz, M, N, K, A, lda, B, ldb, C, ldc, e, sA, sB, sC,
                                               d, stream);
      return;
    }
    if (cfg == 3) {
      launch_one<MODE, TA, TB, F, 256, 2, 256>(grid_yz, M, N, K, A, lda, B, ldb, C, ldc, e, sA, sB, sC,
                                               d, stream);
      return;
    }
  }
  if constexpr (MODE == 1 || MODE == 2) {
    if (cfg == 7) {  // the 8-phase tile with the 1x1 / stride-1 staging (F1)
      launch_one<MODE, TA, TB, F, 256, 8, 256, true>(grid_yz, M, N, K, A, lda, B, ldb, C, ldc, e, sA,
                                                     sB, sC, d, stream);
      return;
    }
  }
  if constexpr (MODE == 1 || MODE == 2 || MODE == 3) {
    if (cfg == 5) {
      launch_one<MODE, TA, TB, F, 256, 8, 256>(grid_yz, M, N, K, A, lda, B, ldb, C, ldc, e, sA, sB, sC,
                                               d, stream);
      return;
    }
    if constexpr (MODE != 3) {
      if (cfg == 4) {
        launch_one<MODE, TA, TB, F, 256, 2, 64>(grid_yz, M, N, K, A, lda, B, ldb, C, ldc, e, sA, sB,
                                                sC, d, stream);
        return;
      }
    }
  }
  if (cfg == 1)
    launch_one<MODE, TA, TB, F, 256, 3>(grid_yz, M, N, K, A, lda, B, ldb, C, ldc, e, sA, sB, sC, d, stream);
  else if (cfg == 2)
    launch_one<MODE, TA, TB, F, 256, 2>(grid_yz, M, N, K, A, lda, B, ldb, C, ldc, e, sA, sB, sC, d, stream);
  else
    launch_one<MODE, TA, TB, F, 128, 2>(grid_yz, M, N, K, A, lda, B, ldb, C, ldc, e, sA, sB, sC, d, stream);
}

// C[m][n] = beta * C[m][n] + sum_s ws[s][m][n] (N % 4 == 0, C rows 16-byte aligned).  A block
// covers 256 / L float4 columns with L split lanes each (L = 1..16, a power of two): lane l sums
// splits l, l + L, ... (each wave reads contiguous 1 KB runs of one plane), then the L partial
// sums meet in LDS.  (A plain loop over S per thread ran the ResNet-50 layer1 weight gradients,
// S = 102-256 splits of a 64 x 576 output, 3x slower than the atomics it replaced.)
__global__ __launch_bounds__(256) void splitk_reduce_kernel(int M, int N, int S, int L,
                                                            const float* __restrict__ ws,
                                                            float* __restrict__ C, int ldc,
                                                            float beta) {
  __shared__ f32x4 red[256];
  const int nq = N >> 2, cpb = 256 / L;
  const int col = threadIdx.x % cpb, sl = threadIdx.x / cpb;
  const long long i = (long long)blockIdx.x * cpb + col, total = (long long)M * nq;
  const bool live = i < total;
  const int m = live ? (int)(i / nq) : 0, n = live ? (int)(i - (long long)m * nq) * 4 : 0;
  const size_t plane = (size_t)M * N;
  const float* w = ws + (size_t)m * N + n;
  f32x4 a = {0.f, 0.f, 0.f, 0.f};
  if (live) {
#pragma unroll 4
    for (int s = sl; s < S; s += L) a += *(const f32x4*)(w + s * plane);
  }
  red[threadIdx.x] = a;
  __syncthreads();
  if (sl == 0 && live) {
    for (int j = 1; j < L; ++j) a += red[j * cpb + col];
    float* c = C + (size_t)m * ldc + n;
    if (beta != 0.f) a += beta * *(const f32x4*)c;
    *(f32x4*)c = a;
  }
}

// Few splits (S <= 8: the BERT weight gradients, S = 3 / 4 / 14 -> 14 takes the lane-split
// kernel above): one thread per float4 output, all S plane loads issued before the first add,
// two outputs per thread (grid-stride, 8..16 loads in flight) -- the one-load-per-lane shape
// above left 3 of 4 lanes' latency exposed at S = 3 (1.2 TB/s, 31 us for the 28 MB of the
// FFN weight gradients).  Sum order s = 0, 1, .. (the same as the lane-split kernel for S <= L).
template <int SMAX>
__global__ __launch_bounds__(256) void splitk_reduce_few_kernel(int M, int N, int S,
                                                                const float* __restrict__ ws,
                                                                float* __restrict__ C, int ldc,
                                                                float beta) {
  const int nq = N >> 2;
  const long long total = (long long)M * nq;
  const size_t plane = (size_t)M * N;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += 2 * stride) {
    f32x4 v[2][SMAX];
    int m[2], n[2];
    bool live[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const long long j = i + u * stride;
      live[u] = j < total;
      m[u] = live[u] ? (int)(j / nq) : 0;
      n[u] = live[u] ? (int)(j - (long long)m[u] * nq) * 4 : 0;
      const float* w = ws + (size_t)m[u] * N + n[u];
#pragma unroll
      for (int s = 0; s < SMAX; ++s)
        if (s < S && live[u]) v[u][s] = __builtin_nontemporal_load((const f32x4*)(w + s * plane));
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (!live[u]) continue;
      f32x4 a = v[u][0];
#pragma unroll
      for (int s = 1; s < SMAX; ++s)
        if (s < S) a += v[u][s];
      float* c = C + (size_t)m[u] * ldc + n[u];
      if (beta != 0.f) a += beta * *(const f32x4*)c;
      *(f32x4*)c = a;
    }
  }
}

// Split-K through the partial workspace when it fits (else f32 atomics into a pre-zeroed /
// accumulating C).  Returns true when the caller must NOT pre-zero C.
static bool splitk_ws_ok(float* ws, long long ws_floats, int splitk, int M, int N, void* C, int ldc) {
  return ws && splitk > 1 && N % 4 == 0 && ldc % 4 == 0 && ((uintptr_t)C & 15) == 0 &&
         ((uintptr_t)ws & 15) == 0 && (long long)splitk * M * N <= ws_floats;
}
static void splitk_reduce(int M, int N, int S, const float* ws, float* C, int ldc, float beta,
                          hipStream_t stream) {
  if (S <= 8) {
    const long long n4 = (long long)M * (N / 4);
    const long long blocks = std::min<long long>((n4 + 511) / 512, 2048);
    hipLaunchKernelGGL(splitk_reduce_few_kernel<8>, dim3((unsigned)blocks), dim3(256), 0, stream,
                       M, N, S, ws, C, ldc, beta);
    DTFX_HIP_CHECK(hipGetLastError());
    return;
  }
  int L = 1;
  while (L < S && L < 16) L <<= 1;
  const long long n = (long long)M * (N / 4), cpb = 256 / L;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((n + cpb - 1) / cpb)), dim3(256), 0,
                     stream, M, N, S, L, ws, C, ldc, beta);
  DTFX_HIP_CHECK(hipGetLastError());
}

// Epilogue of a split-K convolution (fwd / stride-1 dgrad with few output tiles, see
// conv_splitk): y = sum_s ws[s] (split order) (+ residual) (* (relu_y > 0)) -> bf16, and the
// BatchNorm statistics of one partial row per 64-row slab, exactly as the GEMM epilogue
// writes them (fwd: sum / sum of squares of the f32 values; dgrad with bn_x: sum of the
// stored bf16 values and of value * xhat).  Block: 64 rows x 256 columns, thread = 8 columns
// x 8 rows (row lane rl = rows rl, rl + 8, ...); the 8 row lanes meet in LDS.
__global__ __launch_bounds__(256) void conv_splitk_epi_kernel(
    int M, int N, int S, const float* __restrict__ ws, unsigned short* __restrict__ y, int ldc,
    const unsigned short* __restrict__ res, const unsigned short* __restrict__ relu_y,
    const unsigned short* __restrict__ bn_x, const float* __restrict__ bn_mean,
    const float* __restrict__ bn_rstd, float* __restrict__ psum, float* __restrict__ psq) {
  __shared__ float red[2][8][257];
  const int cg = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int n = blockIdx.x * 256 + cg * 8, m0 = blockIdx.y * 64;
  const bool live_n = n < N;  // (N % 8 == 0)
  const size_t plane = (size_t)M * N;
  float cs[8], cq[8], mu[8], rs[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) cs[u] = cq[u] = 0.f;
  if (bn_x && live_n) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      mu[u] = bn_mean[n + u];
      rs[u] = bn_rstd[n + u];
    }
  }
  if (live_n) {
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + rl + 8 * i;
      if (m >= M) break;
      const float* w = ws + (size_t)m * N + n;
      float v[8];
      *(f32x4*)&v[0] = *(const f32x4*)w;
      *(f32x4*)&v[4] = *(const f32x4*)(w + 4);
      for (int sp = 1; sp < S; ++sp) {
        const f32x4 a = *(const f32x4*)(w + sp * plane), b = *(const f32x4*)(w + sp * plane + 4);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          v[u] += a[u];
          v[u + 4] += b[u];
        }
      }
      const size_t o = (size_t)m * ldc + n;
      if (res) {
        const bf16x8 r = *(const bf16x8*)&res[o];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] += bf2f((unsigned short)r[u]);
      }
      if (relu_y) {
        const bf16x8 a = *(const bf16x8*)&relu_y[o];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] *= bf2f((unsigned short)a[u]) > 0.f ? 1.f : 0.f;
      }
      bf16x8 out;
#pragma unroll
      for (int u = 0; u < 8; ++u) out[u] = (short)f2bf(v[u]);
      if (psum) {
        if (bn_x) {
          const bf16x8 xq = *(const bf16x8*)&bn_x[o];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const float vr = bf2f((unsigned short)out[u]);
            cs[u] += vr;
            cq[u] += vr * (bf2f((unsigned short)xq[u]) - mu[u]) * rs[u];
          }
        } else {
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            cs[u] += v[u];
            cq[u] += v[u] * v[u];
          }
        }
      }
      *(bf16x8*)&y[o] = out;
    }
  }
  if (!psum) return;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    red[0][rl][cg * 8 + u] = cs[u];
    red[1][rl][cg * 8 + u] = cq[u];
  }
  __syncthreads();
  const int c = threadIdx.x, nc = blockIdx.x * 256 + c;
  if (nc < N) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      a += red[0][r][c];
      b += red[1][r][c];
    }
    psum[(size_t)blockIdx.y * N + nc] = a;
    psq[(size_t)blockIdx.y * N + nc] = b;
  }
}

// Split-K factor of a GEMM (splitk <= 0: auto) and its tile configuration.
static int gemm_splitk(bool ta, bool out_f32, int M, int N, int K, int splitk, int batch, float beta,
                       bool plain_epilogue, int* cfg_out) {
  const int nkt = K / gb::BK;
  const bool auto_split = splitk <= 0;
  const int cfg = choose_cfg(M, N, batch * (auto_split ? 1 : splitk), 0, ta);
  *cfg_out = cfg;
  if (!auto_split) return splitk;
  const int bm = cfg == 0 ? 128 : 256, bn = (cfg == 3 || cfg == 5) ? 256 : cfg == 6 ? 192 : 128;
  const int tiles = ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  // Fill the 256 CUs when the output has few tiles and K is deep: the largest split with
  // tiles * splitk <= resident block slots (cfg 0: 2 blocks/CU x 256 CUs; else 1/CU), ONE
  // wave.  Measured on the BERT-base weight gradients (tools/gemm_sweep.py): 144 tiles x 3 =
  // 432 blocks 110 us vs x 2 (288, unbalanced) 146 us and x 4 (576, a second partial wave)
  // 154 us; 108 x 4 and 36 x 12 likewise the fastest of 1..16.
  if (batch == 1 && out_f32 && plain_epilogue && (beta == 0.f || beta == 1.f)) {
    // DTFX_GEMM_TA8_SLOTS: block slots a weight gradient on the 8-phase tile splits for
    // (DTFX_GEMM_TA8=1 A/B runs; fewer splits = fewer partial planes for the optimizer to read
    // while the data gradients hold the rest of the chip)
    static const int ta8_slots = [] {
      const char* e = getenv("DTFX_GEMM_TA8_SLOTS");
      return e ? std::max(1, atoi(e)) : 256;
    }();
    const int slots = cfg == 0 ? 512 : ta ? ta8_slots : 256;
    if (tiles < slots / 2) return std::max(1, std::min(slots / tiles, nkt / 8));
  }
  return 1;
}

// f32 elements of the split-K partial workspace gemm_bf16_launch can use for this GEMM (0: no
// split-K), for callers that provide one.
long long gemm_bf16_ws_floats(bool ta, bool out_f32, int M, int N, int K, int splitk, float beta) {
  int cfg;
  const int s = gemm_splitk(ta, out_f32, M, N, (K + gb::BK - 1) / gb::BK * gb::BK, splitk, 1, beta,
                            true, &cfg);
  return s > 1 ? (long long)s * M * N : 0;
}

static void gemm_bf16_launch_cfg(bool ta, bool tb, bool out_f32, int M, int N, int K, const void* A,
                                 int lda, const void* B, int ldb, void* C, int ldc, float alpha,
                                 float beta, const float* bias, int act, const void* aux_in,
                                 void* aux_out, int ld_aux, const void* residual, int ld_res,
                                 int act_grad, int splitk, int batch, long long sA, long long sB,
                                 long long sC, float* colsum, hipStream_t stream, float* ws,
                                 long long ws_floats, bool defer_reduce, int force_cfg);

// Tail split of an 8-phase GEMM whose 256x256 tiles fill F >= 1 whole rounds of the 256 CUs
// plus a sparse last one (<= half the CUs busy for a whole tile's time): the rows of the whole
// rounds stay on the 8-phase tile, the remaining rows go to the 128x128 tile (two resident
// blocks per CU, a quarter of the work per block), so the tail costs ~half a round instead of
// a full one.  BERT-base's QKV projection (16384 x 2304, K = 768): 576 tiles = 2.25 rounds ->
// 56 tile rows (504 tiles, 2 rounds) + 2048 rows x 2304 on 288 128x128 blocks.  Row-local
// epilogues only (bias / act / aux / residual; column sums accumulate from both parts);
// DTFX_GEMM_TAILSPLIT=0 turns it off.  Returns the rows left for the 8-phase part (M: none).
static int gemm_tail_rows(int M, int N, int cfg, bool ta, int splitk, int batch) {
  static const bool on = [] {
    const char* e = getenv("DTFX_GEMM_TAILSPLIT");
    return !(e && atoi(e) == 0);
  }();
  if (!on || cfg != 5 || ta || splitk > 1 || batch != 1) return M;
  const int tm = (M + 255) / 256, tn = (N + 255) / 256;
  const long long T = (long long)tm * tn;
  const long long F = T / 256, R = T % 256;
  if (F < 1 || R == 0 || R > 128) return M;
  const int rows5 = (int)(F * 256 / tn) * 256;
  return rows5 > 0 && rows5 < M ? rows5 : M;
}

void gemm_bf16_launch(bool ta, bool tb, bool out_f32, int M, int N, int K, const void* A, int lda,
                      const void* B, int ldb, void* C, int ldc, float alpha, float beta,
                      const float* bias, int act, const void* aux_in, void* aux_out, int ld_aux,
                      const void* residual, int ld_res, int act_grad, int splitk, int batch,
                      long long sA, long long sB, long long sC, float* colsum,
                      hipStream_t stream, float* ws, long long ws_floats, bool defer_reduce) {
  gemm_bf16_launch_cfg(ta, tb, out_f32, M, N, K, A, lda, B, ldb, C, ldc, alpha, beta, bias, act,
                       aux_in, aux_out, ld_aux, residual, ld_res, act_grad, splitk, batch, sA, sB,
                       sC, colsum, stream, ws, ws_floats, defer_reduce, -1);
}

static void gemm_bf16_launch_cfg(bool ta, bool tb, bool out_f32, int M, int N, int K, const void* A,
                                 int lda, const void* B, int ldb, void* C, int ldc, float alpha,
                                 float beta, const float* bias, int act, const void* aux_in,
                                 void* aux_out, int ld_aux, const void* residual, int ld_res,
                                 int act_grad, int splitk, int batch, long long sA, long long sB,
                                 long long sC, float* colsum, hipStream_t stream, float* ws,
                                 long long ws_floats, bool defer_reduce, int force_cfg) {
  if (M <= 0 || N <= 0 || batch <= 0) return;
  if (batch > 1 && (bias || aux_in || aux_out || residual || colsum))
    throw std::runtime_error("gemm_bf16: batched GEMM supports alpha/beta/act epilogues only");
  if (batch > 1 && ((sA | sB | sC) % 8))
    throw std::runtime_error("gemm_bf16: batch strides must be multiples of 8 elements");
  if (K % gb::BK) throw std::runtime_error("gemm_bf16: K must be a multiple of 64, got " + std::to_string(K));
  if ((lda | ldb) % 8) throw std::runtime_error("gemm_bf16: lda/ldb must be multiples of 8");
  if (((uintptr_t)A | (uintptr_t)B) & 15) throw std::runtime_error("gemm_bf16: A/B must be 16-byte aligned");
  if (ta && M % 8) throw std::runtime_error("gemm_bf16: transposed A needs M % 8 == 0");
  if (!tb && N % 8) throw std::runtime_error("gemm_bf16: non-transposed B needs N % 8 == 0");
  if ((ldc % 8) || ((uintptr_t)C & 15))
    throw std::runtime_error("gemm_bf16: C must be 16-byte aligned with ldc % 8 == 0");
  if ((aux_in || aux_out) && (ld_aux % 8 || (((uintptr_t)aux_in | (uintptr_t)aux_out) & 15)))
    throw std::runtime_error("gemm_bf16: aux must be 16-byte aligned with ld_aux % 8 == 0");
  if (residual && (ld_res % 8 || ((uintptr_t)residual & 15)))
    throw std::runtime_error("gemm_bf16: residual must be 16-byte aligned with ld_res % 8 == 0");
  if (bias && ((uintptr_t)bias & 15)) throw std::runtime_error("gemm_bf16: bias must be 16-byte aligned");
  if (act_grad && !aux_in) throw std::runtime_error("gemm_bf16: act_grad needs aux_in");
  if (act < 0 || act > 3 || act_grad < 0 || act_grad > 3)
    throw std::runtime_error("gemm_bf16: act / act_grad must be 0..3");
  if (act == 3 && !aux_out) throw std::runtime_error("gemm_bf16: act 3 stores gelu' in aux_out");
  const bool plain = !colsum && !bias && !act && !act_grad && !residual && !aux_out;
  int cfg;
  splitk = gemm_splitk(ta, out_f32, M, N, K, splitk, batch, beta, plain, &cfg);
  if (force_cfg >= 0) {
    cfg = force_cfg;
  } else {
    const int rows5 = gemm_tail_rows(M, N, cfg, ta, splitk, batch);
    if (rows5 < M) {
      const size_t eb = out_f32 ? 4 : 2;
      auto adv = [](const void* p, size_t bytes) -> const void* {
        return p ? (const void*)((const char*)p + bytes) : nullptr;
      };
      gemm_bf16_launch_cfg(ta, tb, out_f32, rows5, N, K, A, lda, B, ldb, C, ldc, alpha, beta,
                           bias, act, aux_in, aux_out, ld_aux, residual, ld_res, act_grad, 1, 1,
                           0, 0, 0, colsum, stream, ws, ws_floats, defer_reduce, 5);
      gemm_bf16_launch_cfg(ta, tb, out_f32, M - rows5, N, K, adv(A, (size_t)rows5 * lda * 2), lda,
                           B, ldb, (void*)adv(C, (size_t)rows5 * ldc * eb), ldc, alpha, beta,
                           bias, act, adv(aux_in, (size_t)rows5 * ld_aux * 2),
                           (void*)adv(aux_out, (size_t)rows5 * ld_aux * 2), ld_aux,
                           adv(residual, (size_t)rows5 * ld_res * 2), ld_res, act_grad, 1, 1, 0,
                           0, 0, colsum, stream, ws, ws_floats, defer_reduce, 0);
      return;
    }
  }
  if (splitk > 1) {
    if (batch > 1) throw std::runtime_error("gemm_bf16: split-K with batch > 1 is not supported");
    if (!out_f32 || bias || act || act_grad || residual || aux_out || colsum ||
        (beta != 0.f && beta != 1.f))
      throw std::runtime_error("gemm_bf16: split-K supports f32 output with alpha and beta in {0,1} only");
    if (splitk_ws_ok(ws, ws_floats, splitk, M, N, C, ldc)) {
      // (C is only read by the reduce: nothing to zero)
    } else if (beta == 0.f) {
      if (ldc == N) DTFX_HIP_CHECK(hipMemsetAsync(C, 0, sizeof(float) * (size_t)M * N, stream));
      else DTFX_HIP_CHECK(hipMemset2DAsync(C, sizeof(float) * ldc, 0, sizeof(float) * N, M, stream));
    }
  }
  GemmEpi e{alpha, beta, bias, act, (const unsigned short*)aux_in, (unsigned short*)aux_out,
            ld_aux, (const unsigned short*)residual, ld_res, act_grad, colsum, nullptr, 0};
  const bool use_ws = splitk > 1 && splitk_ws_ok(ws, ws_floats, splitk, M, N, C, ldc);
  if (use_ws) e.ws = ws;
  // defer_reduce: the caller consumes the split planes itself (the BERT optimizer sums them,
  // adam_mixed_launch with segments) -- C is not written when the GEMM splits
  if (defer_reduce && splitk > 1 && !use_ws)
    throw std::runtime_error("gemm_bf16: defer_reduce needs a workspace of splitk * M * N floats");
  const bool reduce = use_ws && !defer_reduce;
  const dim3 gyz(1, splitk, batch);
  auto* Au = (const unsigned short*)A;
  auto* Bu = (const unsigned short*)B;
#define DTFX_GB(TA_, TB_, F_)                                                                  \
  if (ta == TA_ && tb == TB_ && out_f32 == F_) {                                               \
    launch_cfg<0, TA_, TB_, F_>(cfg, gyz, M, N, K, Au, lda, Bu, ldb, C, ldc, e, sA, sB, sC,    \
                                ConvDesc{}, stream);                                           \
    if (reduce) splitk_reduce(M, N, splitk, ws, (float*)C, ldc, beta, stream);                 \
    return;                                                                                    \
  }
  DTFX_GB(false, true, false)
  DTFX_GB(false, true, true)
  DTFX_GB(false, false, false)
  DTFX_GB(false, false, true)
  DTFX_GB(true, false, false)
  DTFX_GB(true, false, true)
  DTFX_GB(true, true, false)
  DTFX_GB(true, true, true)
#undef DTFX_GB
}

// Convolutions on the 8-phase 256x256 schedule (gathered A rows, gemm_bf16_kernel): when the
// plain-GEMM tile model picks it for the GEMM shape, the source channels are a multiple of 64
// (a K tile stays inside one tap), the source tensor is < 2 GB (32-bit buffer offsets) and the
// reduction has >= 4 K tiles: with 1-2 tiles nothing overlaps the one resident block's loads
// and epilogue (ResNet-50 layer1 1x1 dgrads with the fused BN backward, K = 64 / 128: 377 ->
// 525 us and 426 -> 548 us on the 8-phase tile; layer3 3x3 forward, K = 2304: 120 -> 74 us).
// DTFX_CONV_PH8=0 keeps every convolution on the 128x128 / 256x64 tiles (A/B runs).
static bool conv_ph8(int M, int N, int K, int zdim, int src_ch, long long src_elems) {
  static const bool on = [] {
    const char* v = getenv("DTFX_CONV_PH8");
    return v ? atoi(v) != 0 : true;
  }();
  return on && K >= 4 * gb::BK && src_ch % 64 == 0 && src_elems * 2 < 0x7fffffffLL &&
         choose_cfg(M, N, zdim, 0) == 5;
}

// cfg 5 -> 7 for a 1x1 / stride-1 / pad-0 convolution (the F1 staging; DTFX_CONV_F1=0: off)
static int conv_f1(int cfg, int KH, int KW, int stride, int pad) {
  static const bool on = [] {
    const char* v = getenv("DTFX_CONV_F1");
    return v ? atoi(v) != 0 : true;
  }();
  return on && cfg == 5 && KH == 1 && KW == 1 && stride == 1 && pad == 0 ? 7 : cfg;
}

// Split-K of a forward / stride-1 data-gradient convolution on the 8-phase tile: the layer4
// shapes (M = 12544 pixels x 512 channels, K = 2048 .. 4608) have 98 256x256 tiles for 256 CUs,
// so the 128x128 tile (392 blocks) was chosen and ran them at 450-510 TFLOP/s.  Two K splits on
// the 8-phase tile (196 blocks, >= 8 K tiles each) + conv_splitk_epi_kernel instead.  1: none.
// DTFX_CONV_SPLITK=0 disables (A/B runs).
int conv_splitk(int mode, int N, int H, int W, int C, int Cout, int KH, int KW, int stride,
                int pad) {
  static const bool on = [] {
    const char* v = getenv("DTFX_CONV_SPLITK");
    return v ? atoi(v) != 0 : true;
  }();
  if (!on || gemm_cfg_env() >= 0 || (mode != 1 && !(mode == 2 && stride == 1))) return 1;
  const int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  const int M = mode == 1 ? N * OH * OW : N * H * W, Nn = mode == 1 ? Cout : C;
  const int K = KH * KW * (mode == 1 ? C : Cout), src_ch = mode == 1 ? C : Cout;
  const long long src_elems = (long long)N * (mode == 1 ? H * W * C : OH * OW * Cout);
  if (src_ch % 64 || Nn % 8 || src_elems * 2 >= 0x7fffffffLL) return 1;
  const int tiles = ((M + 255) / 256) * ((Nn + 255) / 256), nkt = K / gb::BK;
  if (tiles > 128) return 1;
  return std::max(1, std::min(256 / tiles, nkt / 8));
}
long long conv_splitk_ws_floats(int mode, int N, int H, int W, int C, int Cout, int KH, int KW,
                                int stride, int pad) {
  const int s = conv_splitk(mode, N, H, W, C, Cout, KH, KW, stride, pad);
  if (s <= 1) return 0;
  const int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  return (long long)s * (mode == 1 ? (long long)N * OH * OW * Cout : (long long)N * H * W * C);
}

// A gathered (3x3 / strided) weight gradient on the 8-phase 256x256 tile: >= 256 output
// channels (a 128-channel output would leave half the tile idle), whole 64-pixel K tiles (the
// dy^T operand is not range-checked) and a source < 2 GB (32-bit buffer offsets).  On the
// 128x128 tile these ran at 470-530 TFLOP/s (LDS-bound: 2 x 8 KB of fragments per 128x128x64
// step).  DTFX_CONV_WGRAD_PH8=0 keeps them there (A/B runs).
static bool conv_wgrad_ph8(int M, int Nn, int K, long long src_elems) {
  static const bool on = [] {
    const char* v = getenv("DTFX_CONV_WGRAD_PH8");
    return v ? atoi(v) != 0 : true;
  }();
  return on && gemm_cfg_env() < 0 && M >= 256 && K % gb::BK == 0 && Nn >= 256 &&
         src_elems * 2 < 0x7fffffffLL;
}
// Split-K of a conv weight gradient (M = Cout, N = KH*KW*C, K = pixels): one wave of the 512
// resident 128x128 slots (see gemm_splitk), or of the 256 8-phase blocks (>= 8 K tiles each)
static int conv_wgrad_splitk(int M, int Nn, int K, bool ph8 = false) {
  const int nkt = (K + 63) / 64;
  if (ph8) {
    const int tiles = ((M + 255) / 256) * ((Nn + 255) / 256);
    return tiles < 256 ? std::max(1, std::min(256 / tiles, nkt / 8)) : 1;
  }
  const int tiles = ((M + 127) / 128) * ((Nn + 127) / 128);
  return tiles < 256 ? std::max(1, std::min(512 / tiles, nkt / 4)) : 1;
}
static bool conv_wgrad_ph8_for(int N, int H, int W, int C, int Cout, int KH, int KW, int stride,
                               int pad) {
  const int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  const bool gathered = !(KH == 1 && KW == 1 && stride == 1 && pad == 0);
  return gathered && conv_wgrad_ph8(Cout, KH * KW * C, N * OH * OW, (long long)N * H * W * C);
}
long long conv_wgrad_ws_floats(int N, int H, int W, int C, int Cout, int KH, int KW, int stride,
                               int pad) {
  const int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  const bool ph8 = conv_wgrad_ph8_for(N, H, W, C, Cout, KH, KW, stride, pad);
  const int Nn = KH * KW * C, s = conv_wgrad_splitk(Cout, Nn, N * OH * OW, ph8);
  return s > 1 ? (long long)s * Cout * Nn : 0;
}

// Convolution launcher (modes in the ConvDesc comment above).
//  fwd  : x [N*H*W][C], w [Cout][ldw >= ceil64(KH*KW*C)] (zero-padded), y [N*OH*OW][Cout]
//         optional fused BatchNorm statistics: colsum / colsq = per-wave-slab partial rows
//         [ceil(N*OH*OW / 64)][Cout] (f32, fully overwritten)
//  dgrad: dy [N*OH*OW][Cout], w [Cout][ldw], dx [N*H*W][C]
//         (+ residual); optional fused BatchNorm backward of the BN that produced x
//         (y = relu(bn(bn_x) [+ res])): relu_y masks the output, dx = (dgrad + residual) *
//         (relu_y > 0) = dL/d(BN output), and colsum / colsq (partial rows [ceil(M/64)][C])
//         receive sum(dx) and sum(dx * xhat) -- BatchNorm backward's two reductions
//  wgrad: dy, x -> dw [Cout][ldw] f32 (first KH*KW*C columns; += when beta == 1)
void conv_bf16_launch(int mode, int N, int H, int W, int C, int Cout, int KH, int KW, int stride,
                      int pad, const void* a, const void* b, int ldw, void* out, float beta,
                      const void* residual, float* colsum, float* colsq, int splitk,
                      hipStream_t stream, const void* relu_y, const void* bn_x,
                      const float* bn_mean, const float* bn_rstd, float* ws, long long ws_floats,
                      int defer_reduce) {
  const int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  if (C % 8 || Cout % 8) throw std::runtime_error("conv_bf16: channel counts must be multiples of 8");
  if (((uintptr_t)a | (uintptr_t)b | (uintptr_t)out) & 15)
    throw std::runtime_error("conv_bf16: tensors must be 16-byte aligned");
  ConvDesc d{N, H, W, C, OH, OW, Cout, KH, KW, stride, pad, 0, ldw > 0 ? ldw : KH * KW * C};
  // fwd statistics go to partial rows [ceil(M / 64)][Cout] (reduced by
  // colpart_reduce in cnn.hip): thousands of blocks would otherwise serialise on the same
  // Cout addresses (f32 atomics execute at the memory side)
  GemmEpi e{1.f, beta, nullptr, 0, nullptr, nullptr, 0, (const unsigned short*)residual, 0, 0,
            colsum, colsq, mode == 1 ? 1 : 0};
  int M, Nn, K;
  if (mode == 1) {
    d.ktot = KH * KW * C;
    M = N * OH * OW; Nn = Cout; K = d.ktot;
    if (ldw < (K + 63) / 64 * 64) throw std::runtime_error("conv_bf16: fwd weights need ld >= ceil64(KH*KW*C)");
    e.ld_res = Cout;
    static const int plain1x1 = [] {  // DTFX_CONV1X1_GEMM=0: keep 1x1 convs on the gather path
      const char* v = getenv("DTFX_CONV1X1_GEMM");
      return v ? atoi(v) : 1;
    }();
    if (plain1x1 && KH == 1 && KW == 1 && stride == 1 && pad == 0 && C % 64 == 0 && C >= 256) {
      // a 1x1 stride-1 convolution is the plain GEMM y[M][Cout] = x[M][C] W[Cout][C]^T:
      // the 8-phase 256x256 tile when the time model picks it (partial statistic rows per
      // 64-row slab, as above) and K >= 4 tiles (layer1 conv3, K = 64: 224 us on the 8-phase
      // tile vs 194 on the 128x128 gather path; layer3 conv1, K = 1024: 40 vs 45 us)
      const int cfg = choose_cfg(M, Nn, 1, 0);
      if (cfg == 5) {
        launch_cfg<0, false, true, false>(cfg, dim3(1, 1, 1), M, Nn, K, (const unsigned short*)a, C,
                                          (const unsigned short*)b, ldw, out, Cout, e, 0LL, 0LL,
                                          0LL, d, stream);
        return;
      }
    }
    const int sk = conv_splitk(1, N, H, W, C, Cout, KH, KW, stride, pad);
    if (sk > 1 && ws && ws_floats >= (long long)sk * M * Nn && ((uintptr_t)ws & 15) == 0 &&
        (colsum != nullptr) == (colsq != nullptr)) {
      GemmEpi ep{};
      ep.alpha = 1.f;
      ep.ws = ws;
      launch_cfg<1, false, true, true>(conv_f1(5, KH, KW, stride, pad), dim3(1, sk, 1), M, Nn, K, (const unsigned short*)a, 0,
                                       (const unsigned short*)b, ldw, ws, Nn, ep, 0LL, 0LL, 0LL, d,
                                       stream);
      hipLaunchKernelGGL(conv_splitk_epi_kernel, dim3((Nn + 255) / 256, (M + 63) / 64), dim3(256), 0,
                         stream, M, Nn, sk, ws, (unsigned short*)out, Cout,
                         (const unsigned short*)residual, nullptr, nullptr, nullptr, nullptr, colsum,
                         colsq);
      DTFX_HIP_CHECK(hipGetLastError());
      return;
    }
    const int cfg1 = conv_ph8(M, Nn, K, 1, C, (long long)N * H * W * C) ? 5 : choose_cfg(M, Nn, 1, 1);
    launch_cfg<1, false, true, false>(conv_f1(cfg1, KH, KW, stride, pad), dim3(1, 1, 1), M, Nn, K,
                                      (const unsigned short*)a, 0, (const unsigned short*)b, ldw,
                                      out, Cout, e, 0LL, 0LL, 0LL, d, stream);
  } else if (mode == 2) {
    if (Cout % 64) throw std::runtime_error("conv_bf16: dgrad needs Cout % 64 == 0");
    d.ktot = KH * KW * Cout;
    M = N * H * W; Nn = C; K = d.ktot;
    e.ld_res = C;
    if (relu_y) {
      if ((uintptr_t)relu_y & 15) throw std::runtime_error("conv_bf16: relu_y must be 16-byte aligned");
      e.aux_in = (const unsigned short*)relu_y;
      e.ld_aux = C;
      e.act_grad = 2;
    }
    if (bn_x) {
      if (!colsum || !colsq || !bn_mean || !bn_rstd ||
          (((uintptr_t)bn_x | (uintptr_t)bn_mean | (uintptr_t)bn_rstd) & 15))
        throw std::runtime_error("conv_bf16: fused BN statistics need colsum, colsq, mean, rstd");
      e.bn_x = (const unsigned short*)bn_x;
      e.bn_mean = bn_mean;
      e.bn_rstd = bn_rstd;
    }
    e.col_partial = (colsum || colsq) ? 1 : 0;
    // stride x stride phase classes over blockIdx.z (ConvDesc comment); the grid and the
    // partial statistic rows are sized for the largest class, ceil(H / s) x ceil(W / s)
    const int s = stride, Hc = (H + s - 1) / s, Wc = (W + s - 1) / s;
    M = N * Hc * Wc;
    d.prc = (M + 63) / 64;
    if (e.col_partial && (H % s || W % s)) {
      // smaller classes leave some of their partial rows unwritten: zero them all first
      const size_t bytes = sizeof(float) * (size_t)s * s * d.prc * C;
      if (colsum) DTFX_HIP_CHECK(hipMemsetAsync(colsum, 0, bytes, stream));
      if (colsq) DTFX_HIP_CHECK(hipMemsetAsync(colsq, 0, bytes, stream));
    }
    const int sk = conv_splitk(2, N, H, W, C, Cout, KH, KW, stride, pad);
    if (sk > 1 && ws && ws_floats >= (long long)sk * M * Nn && ((uintptr_t)ws & 15) == 0 &&
        (!e.col_partial || (colsum && colsq))) {
      GemmEpi ep{};
      ep.alpha = 1.f;
      ep.ws = ws;
      launch_cfg<2, false, false, true>(conv_f1(5, KH, KW, stride, pad), dim3(1, sk, 1), M, Nn, K, (const unsigned short*)a, 0,
                                        (const unsigned short*)b, d.wld, ws, Nn, ep, 0LL, 0LL, 0LL,
                                        d, stream);
      hipLaunchKernelGGL(conv_splitk_epi_kernel, dim3((Nn + 255) / 256, (M + 63) / 64), dim3(256), 0,
                         stream, M, Nn, sk, ws, (unsigned short*)out, C,
                         (const unsigned short*)residual, (const unsigned short*)relu_y,
                         (const unsigned short*)bn_x, bn_mean, bn_rstd,
                         e.col_partial ? colsum : nullptr, e.col_partial ? colsq : nullptr);
      DTFX_HIP_CHECK(hipGetLastError());
      return;
    }
    const int cfg2 = conv_ph8(M, Nn, ((KH + s - 1) / s) * ((KW + s - 1) / s) * Cout, s * s, Cout, (long long)N * OH * OW * Cout)
                         ? 5 : choose_cfg(M, Nn, s * s, 2);
    launch_cfg<2, false, false, false>(conv_f1(cfg2, KH, KW, stride, pad), dim3(1, 1, s * s), M, Nn, K,
                                       (const unsigned short*)a, 0, (const unsigned short*)b, d.wld,
                                       out, C, e, 0LL, 0LL, 0LL, d, stream);
  } else if (mode == 3) {
    if (residual || colsum || colsq || relu_y || bn_x)
      throw std::runtime_error("conv_bf16: wgrad has no epilogue options");
    M = Cout; Nn = KH * KW * C; K = N * OH * OW;
    const bool ph8 = conv_wgrad_ph8_for(N, H, W, C, Cout, KH, KW, stride, pad);
    if (splitk <= 0) splitk = conv_wgrad_splitk(M, Nn, K, ph8);
    const int ldo = ldw > 0 ? ldw : Nn;  // dW row stride (the padded fwd weight layout)
    if (ldo < Nn || ldo % 8) throw std::runtime_error("conv_bf16: wgrad ld must be >= KH*KW*C, % 8");
    if (splitk > 1) {
      if (beta != 0.f && beta != 1.f) throw std::runtime_error("conv_bf16: split-K wgrad needs beta 0/1");
      if (beta == 0.f && !splitk_ws_ok(ws, ws_floats, splitk, M, Nn, out, ldo))
        DTFX_HIP_CHECK(hipMemset2DAsync(out, sizeof(float) * ldo, 0, sizeof(float) * Nn, M, stream));
    }
    const bool use_ws = splitk > 1 && splitk_ws_ok(ws, ws_floats, splitk, M, Nn, out, ldo);
    if (defer_reduce && (!use_ws || ws_floats != (long long)splitk * M * Nn))
      throw std::runtime_error("conv_bf16: defer_reduce needs the exact split-K workspace "
                               "(conv_wgrad_ws_floats)");
    if (use_ws) e.ws = ws;
    static const bool plain1x1w = [] {  // DTFX_CONV1X1_WGRAD_GEMM=0: 1x1 wgrads on the gather path
      const char* v = getenv("DTFX_CONV1X1_WGRAD_GEMM");
      return v ? atoi(v) != 0 : true;
    }();
    if (plain1x1w && KH == 1 && KW == 1 && stride == 1 && pad == 0 && K % gb::BK == 0) {
      // a 1x1 stride-1 weight gradient is the plain product dW[co][ci] = sum_p dy[p][co] x[p][ci]
      // (A^T B, both operands k-strided): staged by the plain glds loader instead of the
      // im2col gather, whose per-lane pixel / tap address math (4 float divmods per 16-B
      // chunk) ran these at 370-430 TFLOP/s (profiles/r3/evidence/resnet_layers.jsonl)
      launch_cfg<0, true, false, true>(choose_cfg(M, Nn, splitk, 0, true), dim3(1, splitk, 1), M, Nn,
                                       K, (const unsigned short*)a, Cout, (const unsigned short*)b, C,
                                       out, ldo, e, 0LL, 0LL, 0LL, d, stream);
    } else {
      launch_cfg<3, true, false, true>(ph8 ? 5 : choose_cfg(M, Nn, splitk, 3), dim3(1, splitk, 1), M, Nn, K,
                                       (const unsigned short*)a, Cout, (const unsigned short*)b, 0,
                                       out, ldo, e, 0LL, 0LL, 0LL, d, stream);
    }
    // defer_reduce: the S partial planes [S][Cout][KH*KW*C] stay in ws for the optimizer to
    // sum (sgd_momentum_mixed with segments: one GPU, nothing between the gradient and SGD)
    if (use_ws && !defer_reduce) splitk_reduce(M, Nn, splitk, ws, (float*)out, ldo, beta, stream);
  } else {
    throw std::runtime_error("conv_bf16: mode must be 1 (fwd), 2 (dgrad) or 3 (wgrad)");
  }
}

// Column sums of a bf16 matrix (bias gradients): out[n] (+)= sum_m G[m][n], f32.
// Vector form (ldg % 8 == 0, 16-B aligned G): each thread owns 8 columns and streams rows
// with 16-B loads, 4 rows in flight; blockIdx.y splits the rows (partials combined with one
// atomic per column and row group).
template <int U>  // rows in flight per thread (4, or 8: DTFX_COLSUM_U)
__global__ __launch_bounds__(256) void colsum8_bf16_kernel(const unsigned short* __restrict__ G,
                                                           int M, int N, int ldg,
                                                           float* __restrict__ out, float beta) {
  const int ch = blockIdx.x * 256 + threadIdx.x, n0 = ch * 8;
  if (n0 >= N) return;
  float s[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) s[u] = 0.f;
  const int per = (M + gridDim.y - 1) / gridDim.y;
  const int m0 = blockIdx.y * per, m1 = min(M, m0 + per);
  int m = m0;
  for (; m + U <= m1; m += U) {
    bf16x8 v[U];
#pragma unroll
    for (int i = 0; i < U; ++i) v[i] = *(const bf16x8*)(G + (size_t)(m + i) * ldg + n0);
#pragma unroll
    for (int i = 0; i < U; ++i)
#pragma unroll
      for (int u = 0; u < 8; ++u) s[u] += bf2f((unsigned short)v[i][u]);
  }
  for (; m < m1; ++m) {
    const bf16x8 v = *(const bf16x8*)(G + (size_t)m * ldg + n0);
#pragma unroll
    for (int u = 0; u < 8; ++u) s[u] += bf2f((unsigned short)v[u]);
  }
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int n = n0 + u;
    if (n < N) {
      if (gridDim.y == 1) out[n] = s[u] + (beta != 0.f ? beta * out[n] : 0.f);
      else unsafeAtomicAdd(out + n, s[u]);
    }
  }
}

// Scalar form for unaligned / odd-stride inputs.
__global__ __launch_bounds__(256) void colsum_bf16_kernel(const unsigned short* __restrict__ G, int M,
                                                          int N, int ldg, float* __restrict__ out,
                                                          float beta) {
  // block: 64 columns x 4 row-groups; each thread sums a strided set of rows
  __shared__ float part[4][64];
  const int n = blockIdx.x * 64 + (threadIdx.x & 63), rg = threadIdx.x >> 6;
  float s = 0.f;
  if (n < N)
    for (int m = blockIdx.y * 4 + rg; m < M; m += 4 * gridDim.y) s += bf2f(G[(size_t)m * ldg + n]);
  part[rg][threadIdx.x & 63] = s;
  __syncthreads();
  if (rg == 0 && n < N) {
    s = part[0][threadIdx.x] + part[1][threadIdx.x] + part[2][threadIdx.x] + part[3][threadIdx.x];
    if (gridDim.y == 1) out[n] = s + (beta != 0.f ? beta * out[n] : 0.f);
    else atomicAdd(out + n, s);
  }
}

static int g_colsum_u = 0;  // 0: DTFX_COLSUM_U; 4 / 8 forced (tests, probes)
void colsum_set_rows_in_flight(int u) { g_colsum_u = (u == 4 || u == 8) ? u : 0; }

void colsum_bf16_launch(const void* G, int M, int N, int ldg, float* out, float beta,
                        hipStream_t stream) {
  if (N <= 0) return;
  const bool vec = ldg % 8 == 0 && ((uintptr_t)G & 15) == 0 && ldg >= ((N + 7) / 8) * 8;
  const int gx = vec ? (N + 2047) / 2048 : (N + 63) / 64;
  // Split rows over blocks when the matrix is tall (>= ~1024 blocks in flight); the
  // caller's out is pre-scaled then.
  int gy = 1;
  if (M >= 512 && (beta == 0.f || beta == 1.f)) gy = std::min(std::max(1, M / (vec ? 64 : 32)), std::max(1, 1024 / gx));
  if (gy > 1) {
    if (beta == 0.f) DTFX_HIP_CHECK(hipMemsetAsync(out, 0, sizeof(float) * N, stream));
    else if (beta != 1.f) throw std::runtime_error("colsum_bf16: beta must be 0 or 1 for tall inputs");
  }
  static const int u_env = [] {
    const char* e = getenv("DTFX_COLSUM_U");
    return e && atoi(e) == 8 ? 8 : 4;
  }();
  const int u = g_colsum_u > 0 ? g_colsum_u : u_env;
  if (vec && u == 8)
    hipLaunchKernelGGL(colsum8_bf16_kernel<8>, dim3(gx, gy), dim3(256), 0, stream,
                       (const unsigned short*)G, M, N, ldg, out, beta);
  else if (vec)
    hipLaunchKernelGGL(colsum8_bf16_kernel<4>, dim3(gx, gy), dim3(256), 0, stream,
                       (const unsigned short*)G, M, N, ldg, out, beta);
  else
    hipLaunchKernelGGL(colsum_bf16_kernel, dim3(gx, gy), dim3(256), 0, stream,
                       (const unsigned short*)G, M, N, ldg, out, beta);
  DTFX_HIP_CHECK(hipGetLastError());
}

}  // namespace dtfx
