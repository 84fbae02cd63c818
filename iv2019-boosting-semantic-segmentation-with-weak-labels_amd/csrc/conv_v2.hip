// bf16 implicit-GEMM convolution, forward + data-gradient ("NT"), v2 structure for gfx950:
//
//  * 512 threads = 8 waves, block tile BM=256 pixels x BN output channels, K-step 64 bf16;
//  * operands staged HBM -> LDS with LDS-DMA (global_load_lds_dwordx4, no VGPR staging),
//    STAGES-deep ring, loads of the next K-steps in flight across the barrier (counted
//    s_waitcnt vmcnt + raw s_barrier: __syncthreads would drain the DMA);
//  * the implicit-GEMM gather is per-lane SOURCE addressing (TF SAME / explicit padding,
//    dilation, forward stride, transposed-conv stride for dgrad); out-of-bounds taps read
//    from a 16-byte zero buffer, so the LDS image is always written whole;
//  * XOR-swizzled 128-byte LDS rows (chunk ^ ((row>>1)&7)) applied on the source address,
//    conflict-free ds_read_b128 fragment reads, v_mfma_f32_16x16x32_bf16;
//  * XCD-aware block -> tile map (blocks sharing an A panel land on one XCD's L2);
//  * epilogue staged through LDS in fp32 column chunks: optional residual adds, one 16-byte
//    store per 8 outputs, and the per-column BN partial statistics (sum, M2 about the tile
//    mean) for the fused batch-norm.
#include "conv.h"
#include <algorithm>
#include <cstdlib>

// s_setprio(1) around the MFMA clusters: +1-2 % measured

// 16-byte zero source for out-of-bounds (padding) taps of the LDS-DMA gather
__device__ __attribute__((aligned(64))) bf16_t g_zero16[64];

namespace {

constexpr int V2_THREADS = 512;
constexpr int BK = 64;     // bf16 elements per K-step (128 B per row)

__device__ __forceinline__ int swz(int row, int ch) { return ch ^ ((row >> 1) & 7); }

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else static_assert(N < 0, "unsupported vmcnt");
}

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

template <int TO_F32>
struct OutT;
template <> struct OutT<0> { typedef bf16_t T; };
template <> struct OutT<1> { typedef float T; };

// BM = 256; waves laid out WMW (M) x WNW (N); STAGES-deep ring of 64-deep K-steps.
// (Measured and rejected: splitting each stage into two 32-deep units refilled one phase
// after their last read -- 1.5 K-steps of prefetch instead of 1 -- ran 5-8 % slower: the
// extra barrier per K-step costs more than the deeper prefetch gains.)
template <int MF> struct AccOf;
template <> struct AccOf<16> { typedef f32x4_t T; static constexpr int N = 4; };

// MF: MFMA shape (16: v_mfma_f32_16x16x32_bf16). A v_mfma_f32_32x32x16_bf16 main loop with
// fragments double-buffered across k16-steps was measured 5-9 % slower on the C2 layer shapes
// and removed; the epilogue keeps the shape-generic (row_of / col_of) accumulator walk.
// DU: dense 1x1 rows plus a K-concatenated second GEMM (x2, w2), the ping-pong kernel's ST = 4
// for output tiles of <= 128 channels (csrc/lbf.h: the folded conv3 data gradient of block1-2)
template <typename E, int BN, int WMW, int WNW, int STAGES, int ST, int T8 = 0, int MF = 16, int BM_ = 256,
          int DU = 0>
__global__ __launch_bounds__(V2_THREADS, BM_ == 256 ? 1 : 2) void conv_nt_v2_kernel(ConvArgs a) {
  typedef typename Half<E>::V V;
  const E* zero = (const E*)g_zero16;
  constexpr int BM = BM_;
  constexpr int WM = BM / WMW, WN = BN / WNW;
  constexpr int FM = WM / MF, FN = WN / MF;
  constexpr int NA = AccOf<MF>::N;   // accumulator elements per lane per fragment
  typedef typename AccOf<MF>::T acc_t;
  constexpr int AI = BM * 8 / V2_THREADS;       // A glds per lane per K-step (4)
  constexpr int BI = BN * 8 / V2_THREADS;       // B glds per lane per K-step
  constexpr int LPK = AI + BI;
  constexpr int STAGE_BYTES = (BM + BN) * 128;
  constexpr int EPI_COLS = 64;                  // epilogue chunk width (fp32 staging)
  constexpr int EPI_LD = EPI_COLS + 4;          // padded fp32 row
  constexpr int LDS_BYTES = STAGES * STAGE_BYTES > BM * EPI_LD * 4 ? STAGES * STAGE_BYTES : BM * EPI_LD * 4;
  static_assert(WMW * WNW == 8, "8 waves");
  static_assert(BI >= 1, "BN >= 64");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  (void)LDS_BYTES;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WNW, wn = wave % WNW;
  const int lr = lane & 15, lq = lane >> 4;
  const long M = (long)a.N * a.Ho * a.Wo;
  const int mtiles = (int)((M + BM - 1) / BM);
  const int ntiles = (a.Co + BN - 1) / BN;
  // XCD-aware bijective remap: blocks dealt round-robin over 8 XCDs; give each XCD a
  // contiguous run of tiles (n fastest) so blocks sharing an A panel share an L2
  const int nwg = mtiles * ntiles;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int mt = wg / ntiles, nt = wg - mt * ntiles;
  const long m0 = (long)mt * BM;
  const int n0 = nt * BN;
  const int K = a.KH * a.KW * a.C;
  const int nk1 = T8 ? (K + BK - 1) / BK : K / BK;   // tap mode: taps beyond KH*KW read zeros
  const int nk = nk1 + (DU ? a.C2 / BK : 0);
  const E* X = (const E*)a.x;
  const E* Wt = (const E*)a.w;

  // ---- per-lane A rows (fixed over K): image base and the tap-independent coordinates ----
  constexpr int AR = AI;          // A rows per lane per K-step
  constexpr int RPW = 8;          // rows per wave-instruction (128-B rows)
  const int pc = lane & 7;        // physical 16-B chunk this lane fills
  long a_nb[AR];                  // n * H
  int a_h0[AR], a_w0[AR], a_row[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int row = (i * 8 + wave) * RPW + (lane >> 3);
    a_row[i] = row;
    const long m = m0 + row;
    const bool ok = m < M;
    // 32-bit decode (M < 2^31: conv_nt_v2_ok); the 64-bit div/rem it replaces was a library
    // call per row and per tile
    const unsigned mm = ok ? (unsigned)m : 0u;
    const unsigned t = mm / (unsigned)a.Wo;
    const int wo = (int)(mm - t * (unsigned)a.Wo);
    const unsigned nimg = t / (unsigned)a.Ho;
    const int ho = (int)(t - nimg * (unsigned)a.Ho);
    a_nb[i] = (long)nimg * a.H;
    a_h0[i] = ok ? ho * a.sf - a.pad_h : -(1 << 28);  // invalid rows never pass the bounds test
    a_w0[i] = wo * a.sf - a.pad_w;
  }

  // K-step order (not tap8): channel chunk outer, tap inner -- the KH*KW shifted reads of one
  // chunk's source rows follow each other while they are still in L2
  const int ntaps = a.KH * a.KW;
  auto kcol = [&](int kb) { return T8 ? kb * BK : (kb % ntaps) * a.C + (kb / ntaps) * BK; };
  auto issue_a = [&](int kb, int stage) {
    if constexpr (DU) {   // the second GEMM's K-steps: the same pixels of x2 (dense 1x1)
      if (kb >= nk1) {
        char* sA = smem + stage * STAGE_BYTES;
#pragma unroll
        for (int i = 0; i < AR; ++i) {
          const int lc = swz(a_row[i], pc);
          const bool ok = a_h0[i] >= 0;
          const size_t off = ((size_t)(a_nb[i] + a_h0[i]) * a.W + a_w0[i]) * a.ldx2 + (kb - nk1) * BK + lc * 8;
          glds16(ok ? (const void*)((const E*)a.x2 + off) : (const void*)zero, sA + (i * 8 + wave) * 1024);
        }
        return;
      }
    }
    const int tap = T8 ? 0 : kb % ntaps;
    const int c0 = T8 ? 0 : (kb / ntaps) * BK;
    const int kh = tap / a.KW, kw = tap - kh * a.KW;
    const int dh = kh * a.dil, dw = kw * a.dil;
    char* sA = smem + stage * STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int lc = swz(a_row[i], pc);
      int hi = a_h0[i] + dh, wi = a_w0[i] + dw;
      int coff = 0;
      if constexpr (T8) {   // tap mode: a tap is T8 16-B chunks (8 channels each); this lane's
                            // chunk is kb*8 + lc, its tap (kb*8 + lc) / T8
        const int ch = kb * 8 + lc;
        const int t8 = ch / T8;
        coff = (ch - t8 * T8) * 8;
        const int kh8 = t8 / a.KW, kw8 = t8 - kh8 * a.KW;
        hi = t8 < a.KH * a.KW ? a_h0[i] + kh8 * a.dil : -1;
        wi = a_w0[i] + kw8 * a.dil;
      }
      bool ok;
      if constexpr (ST == 1) {
        ok = ((unsigned)hi < (unsigned)a.H) & ((unsigned)wi < (unsigned)a.W);
      } else {  // transposed-conv gather (strided dgrad): source index must divide by ST
        ok = (hi >= 0) & (wi >= 0) & ((hi % ST) == 0) & ((wi % ST) == 0);
        hi /= ST;
        wi /= ST;
        ok &= (hi < a.H) & (wi < a.W);
      }
      const size_t off = ((size_t)(a_nb[i] + hi) * a.W + wi) * a.ldx + c0 + (T8 ? coff : lc * 8);
      glds16(ok ? (const void*)(X + off) : (const void*)zero, sA + (i * 8 + wave) * 1024);
    }
  };
  auto issue_b = [&](int kb, int stage) {
    const bool sec = DU && kb >= nk1;
    const int k0 = sec ? (kb - nk1) * BK : kcol(kb);
    const E* Wb = sec ? (const E*)a.w2 : Wt;
    const int ldw = sec ? a.ldw2 : a.ldw;
    char* sB = smem + stage * STAGE_BYTES + BM * 128;
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int row = (i * 8 + wave) * 8 + (lane >> 3);
      const int co = n0 + row;
      const int lc = swz(row, pc);
      const E* src = co < a.Co ? Wb + (size_t)co * ldw + k0 + lc * 8 : zero;
      glds16(src, sB + (i * 8 + wave) * 1024);
    }
  };

  acc_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int k = 0; k < NA; ++k) acc[i][j][k] = 0.f;
  // accumulator element (i, j, k) -> tile row / column
  auto row_of = [&](int i, int k) {
    if constexpr (MF == 16) return wm * WM + i * 16 + lq * 4 + k;
    else return wm * WM + i * 32 + (k >> 2) * 8 + (lane >> 5) * 4 + (k & 3);
  };
  auto col_of = [&](int j) {
    if constexpr (MF == 16) return wn * WN + j * 16 + lr;
    else return wn * WN + j * 32 + (lane & 31);
  };
  const bool col_writer = MF == 16 ? lq == 0 : lane < 32;   // one lane per column after merges

  // one K-step of MFMAs; the next stage's LDS-DMA is issued in two parts, one ahead of each
  // 32-deep k-substep, so its issue cost spreads over the MFMA stream
  auto compute = [&](int stage, int nkb, int nstage) {
    const char* A = smem + stage * STAGE_BYTES;
    const char* B = A + BM * 128;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (nkb >= 0) {
        if (s == 0) issue_a(nkb, nstage);
        else issue_b(nkb, nstage);
      }
      V af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = wm * WM + i * 16 + lr;
        af[i] = *(const V*)(A + row * 128 + swz(row, lq + 4 * s) * 16);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = wn * WN + j * 16 + lr;
        bfr[j] = *(const V*)(B + row * 128 + swz(row, lq + 4 * s) * 16);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = Half<E>::mma(af[i], bfr[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
  };

  // ---- main loop: STAGES-deep LDS ring filled by LDS-DMA ----
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) { issue_a(s, s); issue_b(s, s); }
  for (int kb = 0; kb < nk; ++kb) {
    // K-step kb has landed for this lane once at most (issued later) steps remain in flight
    if constexpr (STAGES == 3) {
      if (kb + 1 < nk) wait_vmcnt<LPK>();
      else wait_vmcnt<0>();
    } else {
      wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();   // every lane's DMA for kb landed; stage (kb-1) is free
    const int nkb = kb + STAGES - 1 < nk ? kb + STAGES - 1 : -1;
    compute(kb % STAGES, nkb, (kb + STAGES - 1) % STAGES);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  // ---- epilogue ----
  const int rows_valid = (int)((M - m0) < BM ? (M - m0) : BM);
  float* red = (float*)smem;          // [WMW][BN] column partials
  if (a.stats && rows_valid == BM) {
    // full tile, one pass over the accumulators: per lane and column, (sum, M2) of its 4*FM
    // rows from (sum, sum of squares); then Chan merges of equal-count groups over the lane
    // groups (shfl 16, 32) and the WMW waves (LDS), fixed order
    float2* red2 = (float2*)smem;     // [WMW][BN] (sum, M2)
    constexpr float NL = (float)(NA * FM);   // rows per lane
    float sj[FN], mj[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float sm = 0.f, sq = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int k = 0; k < NA; ++k) {
          const float x = acc[i][j][k];
          sm += x;
          sq = __builtin_fmaf(x, x, sq);
        }
      sj[j] = sm;
      mj[j] = fmaxf(sq - sm * sm * (1.f / NL), 0.f);
    }
    float n = NL;
#pragma unroll
    for (int o = MF; o <= 32; o <<= 1) {   // lanes holding other rows of the same column
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const float s2 = __shfl_xor(sj[j], o, 64), m2 = __shfl_xor(mj[j], o, 64);
        const float d = (s2 - sj[j]) / n;
        mj[j] = mj[j] + m2 + d * d * (0.5f * n);
        sj[j] += s2;
      }
      n *= 2.f;
    }
    if (col_writer)
#pragma unroll
      for (int j = 0; j < FN; ++j) red2[wm * BN + col_of(j)] = make_float2(sj[j], mj[j]);
    __syncthreads();
    if (wm == 0 && col_writer) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int c = col_of(j);
        float2 t = red2[c];
        float nt = (float)WM;
#pragma unroll
        for (int w = 1; w < WMW; ++w) {
          const float2 u = red2[w * BN + c];
          const float d = u.x / (float)WM - t.x / nt;
          t.y = t.y + u.y + d * d * (nt * (float)WM / (nt + (float)WM));
          t.x += u.x;
          nt += (float)WM;
        }
        if (n0 + c < a.Co)   // one (sum, M2) per BM-row tile (conv_nt_stat_rows)
          *(float2*)(a.stats + 2 * ((size_t)mt * a.Co + n0 + c)) = t;
      }
    }
    __syncthreads();
  } else if (a.stats) {
    // partial tile: two passes with row masks, from the fp32 accumulators:
    // column sums over the wave's rows -> lane groups (shfl) -> the WMW waves (LDS)
    float cs[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float v = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int k = 0; k < NA; ++k) v += row_of(i, k) < rows_valid ? acc[i][j][k] : 0.f;
#pragma unroll
      for (int o = MF; o <= 32; o <<= 1) v += __shfl_xor(v, o, 64);
      cs[j] = v;
    }
    if (col_writer)
#pragma unroll
      for (int j = 0; j < FN; ++j) red[wm * BN + col_of(j)] = cs[j];
    __syncthreads();
    float mean[FN], tot[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = col_of(j);
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < WMW; ++w) t += red[w * BN + c];
      tot[j] = t;
      mean[j] = t / (float)rows_valid;
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float v = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int k = 0; k < NA; ++k) {
          const float d = acc[i][j][k] - mean[j];
          v += row_of(i, k) < rows_valid ? d * d : 0.f;
        }
#pragma unroll
      for (int o = MF; o <= 32; o <<= 1) v += __shfl_xor(v, o, 64);
      cs[j] = v;
    }
    __syncthreads();
    if (col_writer)
#pragma unroll
      for (int j = 0; j < FN; ++j) red[wm * BN + col_of(j)] = cs[j];
    __syncthreads();
    if (wm == 0 && col_writer) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int c = col_of(j);
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < WMW; ++w) t += red[w * BN + c];
        if (n0 + c < a.Co)   // one (sum, M2) per BM-row tile (conv_nt_stat_rows)
          *(float2*)(a.stats + 2 * ((size_t)mt * a.Co + n0 + c)) = make_float2(tot[j], t);
      }
    }
    __syncthreads();
  }
  // coalesced stores: fp32 tile staged through LDS 64 columns at a time, 16 B per lane
  float* stage = (float*)smem;
  E* Y = (E*)a.y;
  const E* R1 = (const E*)a.r;
  const E* R2 = (const E*)a.r2;
  const int s_rl = tid >> 3, s_cc = tid & 7;   // store phase: row lane (0..63), 8-col chunk
#pragma unroll
  for (int pass = 0; pass < BN / EPI_COLS; ++pass) {
    const int cbase = pass * EPI_COLS;
    if (wn * WN + WN > cbase && wn * WN < cbase + EPI_COLS) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = col_of(j);
        if (col >= cbase && col < cbase + EPI_COLS) {
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int k = 0; k < NA; ++k) stage[row_of(i, k) * EPI_LD + (col - cbase)] = acc[i][j][k];
        }
      }
    }
    __syncthreads();
    const int n = n0 + cbase + s_cc * 8;
    if (n < a.Co) {   // Co % 8 == 0 on this path
#pragma unroll
      for (int rr = 0; rr < BM / 64; ++rr) {
        const int row = s_rl + 64 * rr;
        const long m = m0 + row;
        if (m < M) {
          const float* sp = stage + row * EPI_LD + s_cc * 8;
          const float4 v0 = *(const float4*)sp, v1 = *(const float4*)(sp + 4);
          float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
          if (R1) {
            float u[8];
            Vec8<E>::load(R1 + (size_t)m * a.ldr + n, u);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += u[e];
          }
          if (R2) {
            float u[8];
            Vec8<E>::load(R2 + (size_t)m * a.ldr2 + n, u);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += u[e];
          }
          store8_nt(Y + (size_t)m * a.ldy + n, v);
        }
      }
    }
    __syncthreads();
  }
}

template <typename E, int BN, int WMW, int WNW, int STAGES, int ST, int T8 = 0, int MF = 16, int BM = 256,
          int DU = 0>
hipError_t v2_launch(const ConvArgs& a, hipStream_t s) {
  constexpr int STAGE_BYTES = (BM + BN) * 128;
  constexpr int EPI = BM * (64 + 4) * 4;
  constexpr int LDS = STAGES * STAGE_BYTES > EPI ? STAGES * STAGE_BYTES : EPI;
  static_assert(LDS <= 160 * 1024, "LDS budget");
  auto kern = conv_nt_v2_kernel<E, BN, WMW, WNW, STAGES, ST, T8, MF, BM, DU>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  long M = (long)a.N * a.Ho * a.Wo;
  int nwg = ceil_div(M, BM) * ceil_div(a.Co, BN);
  hipLaunchKernelGGL(kern, dim3(nwg), dim3(V2_THREADS), LDS, s, a);
  return hipGetLastError();
}

// ======================================================================================
// Small-channel 3x3 convolutions (stride 1, dilation 1, C in {64, 128}, Co in {64, 128}): the
// v2 gather re-reads every input pixel once per tap (9 L2 -> LDS passes over the same rows),
// which bounds those layers at 0.15-0.25 of their attainable time (profiles/r02_step_report).
// Here a tile is 8 output rows x 32 pixels of one image; its input patch (10 x 34 pixels x 64
// channels = 43.5 KB per channel chunk, XOR-swizzled 128-B rows) is staged in LDS once per
// chunk by LDS-DMA, and the nine taps read their A fragments from the patch at shifted rows
// (16 consecutive output pixels -> 16 consecutive patch rows: the conflict-free ds_read_b128
// pattern of the v2 kernel). Weights stream through a 3-stage ring per K-step (tap-minor);
// chunk 1's patch goes into the second patch buffer one 64-row piece per K-step during chunk
// 0, issued before that K-step's weights so every counted vmcnt stays exact. Epilogue as v2
// (BN partial statistics per 256-row tile, fp32 staging, 16-B stores) with the tile's rows
// mapped back to pixels.
// ======================================================================================
constexpr int PT_H = 8, PT_W = 32;            // output tile
constexpr int PP_H = PT_H + 2, PP_W = PT_W + 2;  // input patch (3x3, dilation 1)
constexpr int PP_ROWS = 384;                  // 340 patch pixels padded to 6 x 64 DMA rows
constexpr int PP_BYTES = PP_ROWS * 128;

// NPB patch buffers (2: chunk 1 streamed during chunk 0; 1: reloaded between chunks), NST weight
// stages, OCC workgroups per CU (2 when the LDS fits 80 KB: the other workgroup hides this one's
// barrier and fragment-read latency)
// epilogue of the patch kernels (every tile is full: Ho % 8 == 0, Wo % 32 == 0): BN partial
// statistics of the 256-row tile (index pt), fp32 staging through LDS, 16-B stores of the
// tile's pixels (+ residuals)
template <typename E, int BN, int WMW, int WNW>
__device__ __forceinline__ void patch_epilogue(const ConvArgs& a, f32x4_t (&acc)[(PT_H * PT_W / WMW) / 16][(BN / WNW) / 16],
                                               char* smem, int pt, int n0, int nimg, int ty0, int tx0) {
  constexpr int BM = PT_H * PT_W;
  constexpr int WM = BM / WMW, WN = BN / WNW;
  constexpr int FM = WM / 16, FN = WN / 16;
  constexpr int EPI_COLS = 64, EPI_LD = EPI_COLS + 4;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WNW, wn = wave % WNW;
  const int lr = lane & 15, lq = lane >> 4;
  auto row_of = [&](int i, int k) { return wm * WM + i * 16 + lq * 4 + k; };
  auto col_of = [&](int j) { return wn * WN + j * 16 + lr; };
  if (a.stats) {
    // as conv_nt_v2_kernel's full-tile path: per lane (sum, M2) of its 4 * FM rows, Chan
    // merges over the lane groups (shfl 16, 32) and the WMW waves (LDS), fixed order
    float2* red2 = (float2*)smem;
    constexpr float NL = (float)(4 * FM);
    float sj[FN], mj[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float sm = 0.f, sq = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float x = acc[i][j][k];
          sm += x;
          sq = __builtin_fmaf(x, x, sq);
        }
      sj[j] = sm;
      mj[j] = fmaxf(sq - sm * sm * (1.f / NL), 0.f);
    }
    float n = NL;
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const float s2 = __shfl_xor(sj[j], o, 64), m2 = __shfl_xor(mj[j], o, 64);
        const float d = (s2 - sj[j]) / n;
        mj[j] = mj[j] + m2 + d * d * (0.5f * n);
        sj[j] += s2;
      }
      n *= 2.f;
    }
    if (lq == 0)
#pragma unroll
      for (int j = 0; j < FN; ++j) red2[wm * BN + col_of(j)] = make_float2(sj[j], mj[j]);
    __syncthreads();
    if (wm == 0 && lq == 0) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int c = col_of(j);
        float2 t = red2[c];
        float nt = (float)WM;
#pragma unroll
        for (int w = 1; w < WMW; ++w) {
          const float2 u = red2[w * BN + c];
          const float d = u.x / (float)WM - t.x / nt;
          t.y = t.y + u.y + d * d * (nt * (float)WM / (nt + (float)WM));
          t.x += u.x;
          nt += (float)WM;
        }
        *(float2*)(a.stats + 2 * ((size_t)pt * a.Co + n0 + c)) = t;
      }
    }
    __syncthreads();
  }
  float* stage = (float*)smem;
  E* Y = (E*)a.y;
  const E* R1 = (const E*)a.r;
  const E* R2 = (const E*)a.r2;
  const int s_rl = tid >> 3, s_cc = tid & 7;
#pragma unroll
  for (int pass = 0; pass < BN / EPI_COLS; ++pass) {
    const int cbase = pass * EPI_COLS;
    if (wn * WN + WN > cbase && wn * WN < cbase + EPI_COLS) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = col_of(j);
        if (col >= cbase && col < cbase + EPI_COLS) {
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int k = 0; k < 4; ++k) stage[row_of(i, k) * EPI_LD + (col - cbase)] = acc[i][j][k];
        }
      }
    }
    __syncthreads();
    const int n = n0 + cbase + s_cc * 8;
    {
#pragma unroll
      for (int rr = 0; rr < BM / 64; ++rr) {
        const int row = s_rl + 64 * rr;
        const int ty = row / PT_W, tx = row - ty * PT_W;
        const long m = ((long)nimg * a.Ho + ty0 + ty) * a.Wo + tx0 + tx;
        const float* sp = stage + row * EPI_LD + s_cc * 8;
        const float4 v0 = *(const float4*)sp, v1 = *(const float4*)(sp + 4);
        float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        if (R1) {
          float u[8];
          Vec8<E>::load(R1 + (size_t)m * a.ldr + n, u);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += u[e];
        }
        if (R2) {
          float u[8];
          Vec8<E>::load(R2 + (size_t)m * a.ldr2 + n, u);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += u[e];
        }
        store8_nt(Y + (size_t)m * a.ldy + n, v);
      }
    }
    __syncthreads();
  }
}

template <typename E, int BN, int WMW, int WNW, int NPB, int NST, int OCC>
__global__ __launch_bounds__(V2_THREADS, 2 * OCC) void conv_nt_patch_kernel(ConvArgs a) {   // (waves per SIMD)
  typedef typename Half<E>::V V;
  const E* zero = (const E*)g_zero16;
  constexpr int BM = PT_H * PT_W;
  constexpr int WM = BM / WMW, WN = BN / WNW;
  constexpr int FM = WM / 16, FN = WN / 16;
  constexpr int BI = BN * 8 / V2_THREADS;     // weight glds per lane per K-step
  constexpr int BSTAGE = BN * 128;
  static_assert(WMW * WNW == 8 && (WM % PT_W == 0 || PT_W % WM == 0), "wave rows");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const patch = smem;                     // NPB chunk buffers
  char* const bring = smem + NPB * PP_BYTES;    // NST weight stages

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WNW, wn = wave % WNW;
  const int lr = lane & 15, lq = lane >> 4;
  const int tiles_x = a.Wo / PT_W, tiles_y = a.Ho / PT_H;
  const int ntiles = a.Co / BN;   // output-channel tiles (n fastest: they share the patch in L2)
  const int nwg = a.N * tiles_y * tiles_x * ntiles;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int n0 = (wg % ntiles) * BN;
  const int pt = wg / ntiles;     // pixel tile = BN-statistics partial index
  const int tx0 = (pt % tiles_x) * PT_W;
  const int ty0 = ((pt / tiles_x) % tiles_y) * PT_H;
  const int nimg = pt / (tiles_x * tiles_y);
  const int nch = a.C / BK;
  const int nk = 9 * nch;
  const E* X = (const E*)a.x;
  const E* Wt = (const E*)a.w;
  const int pc = lane & 7;

  // patch piece i (64 rows) of channel chunk c into buffer c & 1
  auto issue_piece = [&](int c, int i) {
    const int row = (i * 8 + wave) * 8 + (lane >> 3);
    const int py = row / PP_W, px = row - py * PP_W;
    const int hi = ty0 - a.pad_h + py, wi = tx0 - a.pad_w + px;
    const bool ok = row < PP_H * PP_W && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
    const size_t off = ((size_t)((long)nimg * a.H + hi) * a.W + wi) * a.ldx + c * BK + swz(row, pc) * 8;
    glds16(ok ? (const void*)(X + off) : (const void*)zero, patch + (c % NPB) * PP_BYTES + (i * 8 + wave) * 1024);
  };
  auto issue_b = [&](int kb) {
    const int tap = kb % 9, c = kb / 9;
    const int k0 = tap * a.C + c * BK;
    char* sB = bring + (kb % NST) * BSTAGE;
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int row = (i * 8 + wave) * 8 + (lane >> 3);
      glds16(Wt + (size_t)(n0 + row) * a.ldw + k0 + swz(row, pc) * 8, sB + (i * 8 + wave) * 1024);
    }
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  // A fragment row i of this wave -> (output row, column) inside the tile
  auto frag_pix = [&](int i, int& ty, int& tx) {
    const int r = wm * WM + i * 16;
    ty = r / PT_W;
    tx = r - ty * PT_W;
  };

  // prologue: patch chunk 0 (6 pieces), weights of K-steps 0 and 1
#pragma unroll
  for (int i = 0; i < 6; ++i) issue_piece(0, i);
  issue_b(0);
  if (NST == 3 && nk > 1) issue_b(1);
  for (int kb = 0; kb < nk; ++kb) {
    // wait for B(kb) (and everything before it: the current chunk's patch); after it were
    // issued: iteration kb-1's patch piece (if any) and B(kb+1) (3 stages)
    const bool piece_prev = NPB == 2 && kb >= 1 && nch == 2 && kb - 1 < 6;
    const bool b_next = NST == 3 && kb + 1 < nk;
    if (b_next && piece_prev) wait_vmcnt<BI + 1>();
    else if (b_next) wait_vmcnt<BI>();
    else if (piece_prev) wait_vmcnt<1>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();   // every lane's DMA for kb landed; stage (kb - 1) % NST is free
    if (NPB == 1 && kb > 0 && kb % 9 == 0) {   // one patch buffer: reload it for the next chunk
      if (NST == 2 && kb + 1 < nk) issue_b(kb + 1);
#pragma unroll
      for (int i = 0; i < 6; ++i) issue_piece(kb / 9, i);
      wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
    } else if (NST == 2 && kb + 1 < nk) {
      issue_b(kb + 1);
    }
    if (NPB == 2 && nch == 2 && kb < 6) issue_piece(1, kb);
    if (NST == 3 && kb + 2 < nk) issue_b(kb + 2);
    const int tap = kb % 9, c = kb / 9;
    const int kh = tap / 3, kw = tap - kh * 3;
    const char* P = patch + (c % NPB) * PP_BYTES;
    const char* B = bring + (kb % NST) * BSTAGE;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      V af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        int ty, tx;
        frag_pix(i, ty, tx);
        const int prow = (ty + kh) * PP_W + tx + kw + lr;
        af[i] = *(const V*)(P + prow * 128 + swz(prow, lq + 4 * s2) * 16);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = wn * WN + j * 16 + lr;
        bfr[j] = *(const V*)(B + row * 128 + swz(row, lq + 4 * s2) * 16);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = Half<E>::mma(af[i], bfr[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  patch_epilogue<E, BN, WMW, WNW>(a, acc, smem, pt, n0, nimg, ty0, tx0);
}

// The space-to-depth stem (tap mode: a 4 x 4 VALID conv over 16-channel s2d pixels, K = 256)
// on the same tiles: the tile's 11 x 35-pixel s2d patch (32-B pixels, 12.3 KB; the 16-B halves
// swapped on every other group of 8 pixels so 16 consecutive pixels hit distinct banks) and all
// 256 K-columns of the 64 output channels' weights (32 KB) are staged once; a K-step is 4 taps x 2
// chunks, each lane's chunk addressed at its tap's shifted patch pixel. (The v2 tap-mode gather
// re-read every s2d pixel once per tap: 16 L2 -> LDS passes.)
constexpr int PS_H = PT_H + 3, PS_W = PT_W + 3;   // 4 x 4 taps
constexpr int PS_PIX = 512;                       // 385 patch pixels padded to 2 DMA rounds

template <typename E>
__global__ __launch_bounds__(V2_THREADS, 4) void conv_nt_patch_s2d_kernel(ConvArgs a) {
  typedef typename Half<E>::V V;
  constexpr int BN = 64, WMW = 8, WNW = 1;
  constexpr int WM = PT_H * PT_W / WMW, WN = BN / WNW;
  constexpr int FM = WM / 16, FN = WN / 16;
  const E* zero = (const E*)g_zero16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const patch = smem;                      // PS_PIX x 32 B
  char* const wb = smem + PS_PIX * 32;           // 4 K-steps x 64 rows x 128 B
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave;
  const int lr = lane & 15, lq = lane >> 4;
  const int tiles_x = a.Wo / PT_W, tiles_y = a.Ho / PT_H;
  const int nwg = a.N * tiles_y * tiles_x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int pt = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tx0 = (pt % tiles_x) * PT_W;
  const int ty0 = ((pt / tiles_x) % tiles_y) * PT_H;
  const int nimg = pt / (tiles_x * tiles_y);
  const E* X = (const E*)a.x;
  const E* Wt = (const E*)a.w;
  auto sw = [](int p) { return (p >> 3) & 1; };   // 16-B half swap per 8-pixel group
  // patch: 2 rounds of 512 x 16 B (pixel p = 256 i + tid / 2, physical half tid & 1)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int p = (i * 8 + wave) * 32 + (lane >> 1);
    const int py = p / PS_W, px = p - py * PS_W;
    const bool ok = p < PS_H * PS_W;   // VALID: inside the (Ho + 3) x (Wo + 3) s2d image
    const size_t off = ((size_t)((long)nimg * a.H + ty0 + py) * a.W + tx0 + px) * 16 + ((lane & 1) ^ sw(p)) * 8;
    glds16(ok ? (const void*)(X + off) : (const void*)zero, patch + (i * 8 + wave) * 1024);
  }
  // weights: 4 K-steps x 64 rows of 128 B (rows swizzled as the v2 B operand)
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    const int row = wave * 8 + (lane >> 3);
    glds16(Wt + (size_t)row * a.ldw + kb * BK + swz(row, lane & 7) * 8, wb + kb * 8192 + wave * 1024);
  }
  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    const char* B = wb + kb * 8192;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int cc = lq + 4 * s2;                 // this lane's 16-B chunk of the K-step
      const int tap = kb * 4 + (cc >> 1), hf = cc & 1;
      const int kh = tap >> 2, kw = tap & 3;
      V af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = wm * WM + i * 16;
        const int ty = r / PT_W, tx = r - ty * PT_W;
        const int p = (ty + kh) * PS_W + tx + kw + lr;
        af[i] = *(const V*)(patch + p * 32 + ((hf ^ sw(p)) << 4));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = j * 16 + lr;
        bfr[j] = *(const V*)(B + row * 128 + swz(row, cc) * 16);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = Half<E>::mma(af[i], bfr[j], acc[i][j]);
    }
  }
  __builtin_amdgcn_s_barrier();   // every wave's patch / weight reads done: LDS -> epilogue
  patch_epilogue<E, BN, WMW, WNW>(a, acc, smem, pt, 0, nimg, ty0, tx0);
}

template <typename E, int BN, int WMW, int WNW, int NPB, int NST, int OCC>
hipError_t patch_launch(const ConvArgs& a, hipStream_t s) {
  constexpr int LDS = NPB * PP_BYTES + NST * BN * 128;
  static_assert(LDS * OCC <= 160 * 1024 && LDS >= 256 * (64 + 4) * 4, "LDS budget / epilogue staging");
  auto kern = conv_nt_patch_kernel<E, BN, WMW, WNW, NPB, NST, OCC>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int nwg = a.N * (a.Ho / PT_H) * (a.Wo / PT_W) * (a.Co / BN);
  hipLaunchKernelGGL(kern, dim3(nwg), dim3(V2_THREADS), LDS, s, a);
  return hipGetLastError();
}

// the stem's patch kernel: the s2d tap mode with 64 output channels on whole 8 x 32 tiles
bool conv_nt_patch_s2d_ok(const ConvArgs& a) {
  return a.tap8 == 2 && a.C == 16 && a.ldx == 16 && a.Co == 64 && a.KH == 4 && a.KW == 4 &&
         a.sf == 1 && a.pad_h == 0 && a.pad_w == 0 && a.dil == 1 && a.ldw >= 256 && a.ldw % 8 == 0 &&
         a.H == a.Ho + 3 && a.W == a.Wo + 3 && a.Ho % PT_H == 0 && a.Wo % PT_W == 0 && a.ldy % 8 == 0 &&
         !a.r && !a.r2;
}

template <typename E>
hipError_t patch_s2d_launch(const ConvArgs& a, hipStream_t s) {
  constexpr int LDS = 256 * (64 + 4) * 4;   // the epilogue staging (> 16 KB patch + 32 KB weights)
  static_assert(PS_PIX * 32 + 4 * 8192 <= LDS, "LDS");
  auto kern = conv_nt_patch_s2d_kernel<E>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(kern, dim3(a.N * (a.Ho / PT_H) * (a.Wo / PT_W)), dim3(V2_THREADS), LDS, s, a);
  return hipGetLastError();
}

// the patch kernel's shapes (see above; measured against the v2 gather in
// profiles/r02_ab_v19_patch_stem.txt)
bool conv_nt_patch_ok(const ConvArgs& a) {
  return !a.tap8 && a.st == 1 && a.sf == 1 && a.dil == 1 && a.KH == 3 && a.KW == 3 &&
         (a.C == 64 || a.C == 128) && (a.Co == 64 || a.Co == 128) && a.ldw == 9 * a.C &&
         a.H == a.Ho && a.W == a.Wo && a.Ho % PT_H == 0 && a.Wo % PT_W == 0 &&
         a.pad_h >= 0 && a.pad_h <= 2 && a.pad_w >= 0 && a.pad_w <= 2 &&
         a.ldx % 8 == 0 && a.ldy % 8 == 0;
}

}  // namespace

// bf16 fast path: C % 64 == 0, ld/co multiples of 8; stats tiles are 256 rows
bool conv_nt_v2_ok(const ConvArgs& a) {
  if (a.tap8)   // tap mode (the space-to-depth stem): taps of C = 8 * tap8 channels (tap8 = 2),
                // weights [Co][ldw >= ceil(KH*KW*C/64)*64]
    return a.tap8 == 2 && a.st == 1 && a.C == 16 && a.ldx == 16 && a.Co <= 64 && (a.Co % 8) == 0 &&
           (a.ldy % 8) == 0 && a.ldw >= (a.KH * a.KW * a.C + BK - 1) / BK * BK && (a.ldw % 8) == 0 &&
           !a.r && !a.r2 && (long)a.N * a.Ho * a.Wo < (1L << 31);
  return (a.st == 1 || a.st == 2) && (a.C % BK) == 0 && (a.ldx % 8) == 0 && (a.ldw % 8) == 0 && (a.Co % 8) == 0 &&
         (a.ldy % 8) == 0 && (!a.r || a.ldr % 8 == 0) && (!a.r2 || a.ldr2 % 8 == 0) &&
         (long)a.N * a.Ho * a.Wo < (1L << 31);   // 32-bit pixel decode
}

// rows per tile of the v2 config launch_conv_nt_v2 picks (= BN-statistics partial rows).
// (Measured and rejected: 128 x 128 tiles with a 64 KB ring, two workgroups per CU, for short
// reductions K <= 512 -- 10-20 % slower than 256-row tiles on the C2 1x1 layers.)
// 128-row tiles, two workgroups per CU, for the narrow (Co <= 64) layers -- the stem and block1:
// short reductions whose one-tile-per-CU 256-row launches were latency-bound (stem forward
// 287 -> 241 us, block1 1x1 / 3x3 layers 4-18 % faster)
static bool v2_small_tile(const ConvArgs& a) { return a.Co <= 64; }

int conv_nt_v2_rows(const ConvArgs& a) {
  // the ping-pong kernel writes one partial per wave row (128 rows), the v2 kernels one per tile
  if (a.Co > 128 && !a.r && !a.r2 && conv_nt_pp_ok(a)) return 128;
  if (conv_nt_patch_ok(a) || conv_nt_patch_s2d_ok(a)) return 256;
  return v2_small_tile(a) ? 128 : 256;
}

// K-concatenated second GEMM on output tiles of <= 128 channels (dense 1x1 rows only)
bool conv_nt_v2_dual_ok(const ConvArgs& a) {
  return a.x2 && a.st == 1 && a.sf == 1 && a.KH == 1 && a.KW == 1 && a.pad_h == 0 && a.pad_w == 0 &&
         a.H == a.Ho && a.W == a.Wo && a.Co <= 128 && a.C2 % BK == 0 && a.ldx2 % 8 == 0 &&
         a.ldw2 % 8 == 0 && !a.r && !a.r2 && !a.stats && !a.tap8;
}

template <typename E, int ST>
hipError_t v2_dispatch(int dtype, const ConvArgs& a, hipStream_t s) {
  if constexpr (ST == 1) {
    if (a.x2) {
      if (!conv_nt_v2_dual_ok(a) || !conv_nt_v2_ok(a)) return hipErrorInvalidValue;
      if (a.Co > 64) return v2_launch<E, 128, 4, 2, 3, 1, 0, 16, 256, 1>(a, s);
      return v2_launch<E, 64, 8, 1, 3, 1, 0, 16, 128, 1>(a, s);
    }
  }
  if (ST == 1 && conv_nt_patch_ok(a)) {
    // 64-channel output tiles with one patch buffer fit 72 KB and 110 VGPRs: two workgroups
    // per CU hide each other's barrier and fragment-read latency (a 128-channel tile at two
    // per CU needs <= 128 VGPRs and spilled); Co = 128 runs as two such tiles per patch, the
    // 128-channel input as two chunks with the patch reloaded between them
    return patch_launch<E, 64, 8, 1, 1, 3, 2>(a, s);
  }
  if (a.Co > 128) {
    if (conv_nt_pp_ok(a)) return launch_conv_nt_pp(dtype, a, s);
    return v2_launch<E, 256, 4, 2, 2, ST>(a, s);
  }
  if (a.Co > 64) return v2_launch<E, 128, 4, 2, 3, ST>(a, s);
  if (v2_small_tile(a)) return v2_launch<E, 64, 8, 1, 3, ST, 0, 16, 128>(a, s);
  return v2_launch<E, 64, 8, 1, 3, ST>(a, s);
}

template <typename E>
hipError_t nt_v2_e(int dtype, const ConvArgs& a, hipStream_t s) {
  if (a.tap8) {
    if (conv_nt_patch_s2d_ok(a)) return patch_s2d_launch<E>(a, s);
    if (v2_small_tile(a)) return v2_launch<E, 64, 8, 1, 3, 1, 2, 16, 128>(a, s);
    return v2_launch<E, 64, 8, 1, 3, 1, 2>(a, s);
  }
  if (a.st == 1) return v2_dispatch<E, 1>(dtype, a, s);
  if (a.st == 2) return v2_dispatch<E, 2>(dtype, a, s);
  return hipErrorInvalidValue;
}

hipError_t launch_conv_nt_v2(int dtype, const ConvArgs& a, hipStream_t s) {
  if (dtype == SEG_F16) return nt_v2_e<f16_t>(dtype, a, s);
  return nt_v2_e<bf16_t>(dtype, a, s);
}

// ======================================================================================
// bf16 weight gradient ("TN"), v2: C[co][tap*Ci+ci] = sum_p dy[p][co] * x[src(p,tap)][ci]
//  * 512 threads = 8 waves (2 x 4), block tile BM co x BN (tap,ci) columns, K-step 64
//    pixels, 3-stage LDS ring filled by LDS-DMA (counted vmcnt across raw barriers);
//  * both operands are pixel-major: LDS rows are pixels; a lane's column chunk (and so its
//    (tap, ci) decode) is fixed for the whole launch, only the pixel advances; padding taps
//    and pixels past the split read the zero buffer;
//  * rows are XOR-swizzled on 16-B chunks (chunk ^ (2*(r&3) + 8*((r>>3)&1))) so the
//    ds_read_b64_tr_b16 transposed fragment reads (8 pixels of one column per lane) are
//    bank-conflict free;
//  * split-K over pixels into fp32 slabs (reduced in fixed order by splitk_reduce).
// ======================================================================================
namespace {

constexpr int WG_THREADS = 512;

template <int COLS>
__device__ __forceinline__ int wswz(int row, int ch) {
  if constexpr (COLS >= 128) return ch ^ (2 * (row & 3) + 8 * ((row >> 3) & 1));
  else return ch ^ (2 * (row & 3));
}

template <typename E, int BM, int BN, int WMW, int WNW, int STAGES, int WBK>
__global__ __launch_bounds__(WG_THREADS, 1) void conv_wgrad_v2_kernel(WgradArgs a) {
  constexpr int ROWB_A = BM * 2, ROWB_B = BN * 2;            // bytes per pixel row
  constexpr int CPR_A = BM / 8, CPR_B = BN / 8;              // 16-B chunks per row
  constexpr int RPI_A = 64 / CPR_A, RPI_B = 64 / CPR_B;      // rows per wave-instruction
  constexpr int AI = WBK * CPR_A / WG_THREADS;               // glds per lane per K-step
  constexpr int BI = WBK * CPR_B / WG_THREADS;
  constexpr int LPK = AI + BI;
  constexpr int A_BYTES = WBK * ROWB_A, B_BYTES = WBK * ROWB_B;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int WM = BM / WMW, WN = BN / WNW;
  constexpr int FM = WM / 16, FN = WN / 16;
  static_assert(WMW * WNW == 8, "8 waves");
  static_assert(AI >= 1 && BI >= 1, "tile too small");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WNW, wn = wave % WNW;
  const int Ncol = a.KH * a.KW * a.C;
  const int P = a.N * a.Ho * a.Wo;
  // XCD-aware bijective remap of the 1-D grid: workgroups are dealt round-robin over the 8
  // XCDs; give each XCD a contiguous run of (split-major, co fastest) tiles so all tiles of a
  // pixel split share one L2 (dy rows reused across column tiles, x rows across co tiles)
  const int mtn = (a.Co + BM - 1) / BM, ntn = (Ncol + BN - 1) / BN;
  const int nwg = mtn * ntn * a.splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int split = wg / (mtn * ntn);
  const int rem = wg - split * mtn * ntn;
  const int nt_ = rem / mtn, mt_ = rem - nt_ * mtn;
  const int m0 = mt_ * BM;   // co
  const int n0 = nt_ * BN;   // (tap, ci)
  const int chunk = ((P + a.splits - 1) / a.splits + WBK - 1) / WBK * WBK;
  const int p_begin = split * chunk;
  const int p_end = (p_begin + chunk < P) ? p_begin + chunk : P;
  const int nk = p_end > p_begin ? (p_end - p_begin + WBK - 1) / WBK : 0;
  typedef typename Half<E>::V V;
  const E* DY = (const E*)a.dy;
  const E* X = (const E*)a.x;
  const E* zero = (const E*)g_zero16;

  // ---- launch-invariant per-lane decode ----
  // a lane's 8 output rows come from dy, or from dy2 at rows >= Co1 (WgradArgs::dy2; Co1 % 8
  // == 0, so a 16-B chunk never straddles the two)
  int a_row[AI], a_co[AI], a_col[AI], a_ld[AI];
  const E* a_src[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    a_row[i] = (i * 8 + wave) * RPI_A + lane / CPR_A;
    a_co[i] = m0 + wswz<BM>(a_row[i], lane % CPR_A) * 8;
    const bool sec = a.dy2 && a_co[i] >= a.Co1;
    a_src[i] = sec ? (const E*)a.dy2 : DY;
    a_col[i] = sec ? a_co[i] - a.Co1 : a_co[i];
    a_ld[i] = sec ? a.lddy2 : a.lddy;
  }
  int b_row[BI], b_dh[BI], b_dw[BI], b_ci[BI];
  bool b_ok[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    b_row[i] = (i * 8 + wave) * RPI_B + lane / CPR_B;
    const int col = n0 + wswz<BN>(b_row[i], lane % CPR_B) * 8;
    b_ok[i] = col < Ncol;
    const int cc = b_ok[i] ? col : 0;
    const int tap = cc / a.C;
    b_ci[i] = cc - tap * a.C;
    const int kh = tap / a.KW, kw = tap - kh * a.KW;
    b_dh[i] = kh * a.dil - a.pad_h;
    b_dw[i] = kw * a.dil - a.pad_w;
  }

  auto issue = [&](int kb, int stg) {
    const int p0 = p_begin + kb * WBK;
    char* sA = smem + stg * STAGE;
    char* sB = sA + A_BYTES;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int p = p0 + a_row[i];
      const bool ok = (p < p_end) & (a_co[i] < a.Co);
      glds16(ok ? (const void*)(a_src[i] + (size_t)p * a_ld[i] + a_col[i]) : (const void*)zero,
             sA + (i * 8 + wave) * 1024);
    }
    // pixel decode of the K-step's first pixel (wave-uniform), then per-row carries
    const int wo0 = p0 % a.Wo, t0 = p0 / a.Wo;
    const int ho0 = t0 % a.Ho, nn0 = t0 / a.Ho;
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int r = b_row[i];
      const int p = p0 + r;
      int wo = wo0 + r, ho = ho0, nn = nn0;
      if (a.Wo >= WBK) {                 // at most one row carry
        if (wo >= a.Wo) { wo -= a.Wo; if (++ho == a.Ho) { ho = 0; ++nn; } }
      } else {
        const int q = p;
        wo = q % a.Wo;
        const int t = q / a.Wo;
        ho = t % a.Ho;
        nn = t / a.Ho;
      }
      const int hi = ho * a.sf + b_dh[i], wi = wo * a.sf + b_dw[i];
      const bool ok = (p < p_end) & b_ok[i] & ((unsigned)hi < (unsigned)a.H) &
                      ((unsigned)wi < (unsigned)a.W);
      const size_t off = ((size_t)((long)nn * a.H + hi) * a.W + wi) * a.ldx + b_ci[i];
      glds16(ok ? (const void*)(X + off) : (const void*)zero, sB + (i * 8 + wave) * 1024);
    }
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const int lq = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  auto tr_read = [&](const char* base, int rowb, int row, int col) -> s16x4_t {
    const int lc = col >> 3, within = (col & 7) * 2;
    const int ph = rowb >= 256 ? lc ^ (2 * (row & 3) + 8 * ((row >> 3) & 1)) : lc ^ (2 * (row & 3));
    // inline asm: the builtin makes hipcc wait vmcnt(0) (every LDS-DMA in flight) before the
    // read, which defeats the STAGES-deep ring; ordering is by the counted vmcnt + barrier, and
    // compute() waits lgkmcnt(0) before the MFMAs
    const uint32_t addr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)(
        base + row * rowb + ph * 16 + within);
    s16x4_t r;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr));
    return r;
  };

  auto compute = [&](int stg) {
    const char* A = smem + stg * STAGE;
    const char* B = A + A_BYTES;
#pragma unroll
    for (int s = 0; s < WBK / 32; ++s) {     // 32-pixel MFMA k-steps per stage
      const int kr = 32 * s + 8 * lq + q4;
      V af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int col = wm * WM + i * 16 + 4 * p4;
        s16x4_t lo = tr_read(A, ROWB_A, kr, col), hi = tr_read(A, ROWB_A, kr + 4, col);
        short t8[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        __builtin_memcpy(&af[i], t8, 16);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = wn * WN + j * 16 + 4 * p4;
        s16x4_t lo = tr_read(B, ROWB_B, kr, col), hi = tr_read(B, ROWB_B, kr + 4, col);
        short t8[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        __builtin_memcpy(&bfr[j], t8, 16);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = Half<E>::mma(af[i], bfr[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
  };

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue(s, s);
  for (int kb = 0; kb < nk; ++kb) {
    // K-step kb has landed once only the (already issued) later steps remain in flight
    const int later = min(STAGES - 2, nk - 1 - kb);
    if constexpr (STAGES >= 4) {
      if (later >= 2) wait_vmcnt<2 * LPK>();
      else if (later == 1) wait_vmcnt<LPK>();
      else wait_vmcnt<0>();
    } else if constexpr (STAGES == 3) {
      if (later >= 1) wait_vmcnt<LPK>();
      else wait_vmcnt<0>();
    } else {
      wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    if (kb + STAGES - 1 < nk) issue(kb + STAGES - 1, (kb + STAGES - 1) % STAGES);
    compute(kb % STAGES);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  float* O = a.out + (size_t)split * a.Co * Ncol;
  const int lr = lane & 15;
  if (m0 + BM <= a.Co && n0 + BN <= Ncol && (long)a.Co * Ncol * 4 < (1L << 31)) {
    // whole tile: buffer stores, row offset in an SGPR, column in the immediate (as
    // conv_wgrad_pp_body)
    const auto rs_o = __builtin_amdgcn_make_buffer_rsrc((void*)O, (short)0, (int)((long)a.Co * Ncol * 4), 0x00020000);
    const uint32_t vb = (uint32_t)(((m0 + wm * WM + lq * 4) * Ncol + n0 + wn * WN + lr) * 4);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int so = __builtin_amdgcn_readfirstlane((i * 16 + r) * Ncol * 4);
#pragma unroll
        for (int j = 0; j < FN; ++j)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[i][j][r]), rs_o, vb + j * 16 * 4, so, 0);
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * WN + j * 16 + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * WM + i * 16 + lq * 4 + r;
        if (m < a.Co && n < Ncol) O[(size_t)m * Ncol + n] = acc[i][j][r];
      }
    }
}

template <typename E, int BM, int BN, int WMW, int WNW, int STAGES, int WBK = 64>
hipError_t wg2_launch(const WgradArgs& a, hipStream_t s) {
  constexpr int LDS = STAGES * WBK * (BM + BN) * 2;
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static_assert(STAGES <= 4 && (STAGES < 4 || 2 * (WBK * (BM + BN) / 8 / WG_THREADS) <= 16), "vmcnt");
  auto kern = conv_wgrad_v2_kernel<E, BM, BN, WMW, WNW, STAGES, WBK>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int Ncol = a.KH * a.KW * a.C;
  const int nwg = ceil_div(a.Co, BM) * ceil_div(Ncol, BN) * a.splits;
  hipLaunchKernelGGL(kern, dim3(nwg), dim3(WG_THREADS), LDS, s, a);
  return hipGetLastError();
}

}  // namespace

bool conv_wgrad_v2_ok(const WgradArgs& a) {
  return (a.C % 8) == 0 && (a.ldx % 8) == 0 && (a.Co % 8) == 0 && (a.lddy % 8) == 0 &&
         (long)a.N * a.Ho * a.Wo < (1L << 31) &&
         (!a.dy2 || (a.Co1 % 8 == 0 && a.Co1 < a.Co && a.lddy2 % 8 == 0));
}

// tile (BM co x BN cols): the largest the extents fill -- 256 x 256 (wave tiles 128 x 64)
// keeps LDS fragment traffic below the MFMA time and halves L2 re-reads vs 128 x 256 -- then
// halved (larger side first) while tiles x pixel splits would leave fewer than 128 workgroups
// (small outputs such as 256 x 256 1x1 convs: 1 tile x 64 splits = 64 workgroups otherwise).
// 128, the side stream's workgroup target (wgrad_splits): halving down to 256 workgroups
// (round 5) gave block2 / head 1 x 1 layers 128 x 128 tiles where 128 x 256 / 256 x 128 now
// run at the same workgroup count with half the operand re-reads: step +0.53 % (three
// interleaved pairs, profiles/r06_s30_wgrad_tile_target.txt; 64: +0.27 %)
void conv_wgrad_v2_tile(int Co, int Ncol, long P, int* bm, int* bn) {
  int m = Co <= 64 ? 64 : (Co <= 128 ? 128 : 256);
  int n = Ncol <= 64 ? 64 : (Ncol <= 128 ? 128 : 256);
  const long maxs = std::min<long>(256, std::max<long>(1, P / 2048));
  auto blocks = [&]() { return (long)((Co + m - 1) / m) * ((Ncol + n - 1) / n) * maxs; };
#ifndef WG_TILE_TARGET
#define WG_TILE_TARGET 128
#endif
  while (blocks() < WG_TILE_TARGET) {
    if (m >= n && m > 64) m /= 2;
    else if (n > 64) n /= 2;
    else break;
  }
  *bm = m;
  *bn = n;
}

hipError_t launch_conv_wgrad_v2(int dtype, const WgradArgs& a, hipStream_t s) {
  int bm, bn;
  conv_wgrad_v2_tile(a.Co, a.KH * a.KW * a.C, (long)a.N * a.Ho * a.Wo, &bm, &bn);
  return launch_conv_wgrad_v2_tile(dtype, a, bm, bn, s);
}

// explicit tile (bm, bn in {64, 128, 256}); 256 x 256 runs the ping-pong kernel
template <typename E>
hipError_t wgrad_v2_tile_e(int dtype, const WgradArgs& a, int bm, int bn, hipStream_t s) {
  if (bm == 64) {
    if (bn == 64) return wg2_launch<E, 64, 64, 4, 2, 3>(a, s);
    if (bn == 128) return wg2_launch<E, 64, 128, 2, 4, 3>(a, s);
    return wg2_launch<E, 64, 256, 2, 4, 3>(a, s);
  }
  if (bm == 128) {
    if (bn == 64) return wg2_launch<E, 128, 64, 4, 2, 3>(a, s);
    if (bn == 128) return wg2_launch<E, 128, 128, 4, 2, 3>(a, s);
    return wg2_launch<E, 128, 256, 2, 4, 3>(a, s);
  }
  if (bn == 64) return wg2_launch<E, 256, 64, 8, 1, 3>(a, s);
  if (bn == 128) return wg2_launch<E, 256, 128, 4, 2, 3>(a, s);
  if (conv_wgrad_pp_ok(a)) return launch_conv_wgrad_pp(dtype, a, s);
  return wg2_launch<E, 256, 256, 2, 4, 2>(a, s);
}

hipError_t launch_conv_wgrad_v2_tile(int dtype, const WgradArgs& a, int bm, int bn, hipStream_t s) {
  if (dtype == SEG_F16) return wgrad_v2_tile_e<f16_t>(dtype, a, bm, bn, s);
  return wgrad_v2_tile_e<bf16_t>(dtype, a, bm, bn, s);
}
