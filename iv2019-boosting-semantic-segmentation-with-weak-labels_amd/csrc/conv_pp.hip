// 16-bit (bf16 / fp16) implicit-GEMM convolution, forward + data-gradient, "ping-pong"
// schedule for gfx950.
//
// Same operands, gather and epilogue as conv_nt_v2_kernel (conv_v2.hip), different main loop:
//
//  * 256 x 256 tile, 8 waves as 2 (M) x 4 (N), each wave owns 128 rows x 64 columns split in
//    four 64 x 32 quadrants;
//  * every 64-deep K-tile is two PHASES of two quadrants each, (qm,qn) = (0,0), (0,1) then
//    (1,1), (1,0); a phase is a LOAD segment (the ds_read_b128 fragments the quadrants need
//    that are not already in registers, plus LDS-DMA of the next K-tile's halves: A0, B0, B1
//    in phase 0, A1 in phase 1) and an MFMA segment (32 x v_mfma_f32_16x16x32_bf16),
//    separated by s_barrier (round 2: four one-quadrant phases had twice the barriers; two
//    phases run the block4 3x3 forward / data gradient 3-7 % faster, the step +1 %);
//  * the two wave rows are staggered by one barrier (wave row 1 starts with an extra
//    s_barrier), so on every SIMD one wave is in its MFMA segment while the other issues its
//    LDS reads and DMA: the matrix pipe does not idle across barriers;
//  * LDS holds two K-tile buffers, each four 16 KB half-tiles (A rows 0-127 / 128-255, B rows
//    0-127 / 128-255). K-tile k+1 goes into the other buffer, whose halves were last read in
//    K-tile k-1 (by the lagging wave row one segment before the refill: WAR), and each half is
//    waited for with a counted vmcnt before the barrier that precedes its first read (RAW):
//    vmcnt(6) before phase 1 (A0, B0, B1 of k+1 in flight), vmcnt(2) before the next phase 0
//    (A1 of k+1 in flight);
//  * operands are fetched with buffer_load ... lds through buffer resources: a 32-bit byte
//    offset per lane, padding taps and rows past the tensor given an out-of-range offset so
//    the buffer unit writes zeros (4 VALU per A DMA, 1 per B DMA: the load segment is short);
//  * K-tiles run channel-chunk-major, tap-minor, so the KH*KW shifted reads of one chunk's
//    source rows hit L2 (dilated 3x3: +6 %);
//  * persistent over tiles (the next tile's K-tile 0 in flight during the epilogue); the data
//    gradients with one residual (dense 1 x 1 rows) take the residual tile by LDS-DMA and add it
//    in place (RQP, PERSIST = 3); two residuals or other shapes run one tile per workgroup.
#include "conv.h"
#include <cstdlib>

#ifdef PP_DBG_TIMING
// A/B only: per-block, per-tile timestamps (s_memtime) of the NT persistent loop
// (stamps 0-3: tile start, main loop done, prologue issued, epilogue done; 4-11: per column half
// qn the staging writes, statistics, staging barrier and stores, at 4 + 4 qn + 0..3; RQP: per
// half the residual wait, in-place sums + barrier and stores at 4 + 3 qn + 0..2)
__device__ unsigned long long g_pp_dbg[256 * 16 * 16];
#define PP_TS(it, k) \
  if (threadIdx.x == 0 && blockIdx.x < 256 && (it) < 16) g_pp_dbg[(blockIdx.x * 16 + (it)) * 16 + (k)] = __builtin_amdgcn_s_memtime()
#else
#define PP_TS(it, k)
#endif

#ifdef NT_DBG_TIMING
// A/B only: per-wave segment timestamps (s_memtime) of the NT ping-pong loop, blocks 0-7, the
// first tile, 8 K-tiles from K-tile 16 (or 0 when the tile has fewer than 24), 8 stamps per
// K-tile (loop top, before / after barrier A, after the first MFMA segment, after barrier B,
// before / after barrier C, after the second MFMA segment)
__device__ unsigned long long g_nt_dbg[8 * 8 * 8 * 8];
#ifndef NT_DBG_IT
#define NT_DBG_IT 0   // which tile of the persistent loop is stamped
#endif
#define NT_TS(kb, k)                                                                             \
  if ((threadIdx.x & 63) == 0 && blockIdx.x < 8 && dbg_it == NT_DBG_IT && (kb) >= nt_kb0 && (kb) < nt_kb0 + 8) \
    g_nt_dbg[((blockIdx.x * 8 + (threadIdx.x >> 6)) * 8 + ((kb) - nt_kb0)) * 8 + (k)] =            \
        __builtin_amdgcn_s_memtime()
#else
#define NT_TS(kb, k)
#endif

#ifdef WG_DBG_TIMING
// A/B only: per-wave segment timestamps (s_memtime) of the wgrad ping-pong loop, blocks 0-7,
// K-tiles 16-23, 8 stamps per K-tile (loop top, before / after barrier A, after the first MFMA
// segment, after barrier B, before / after barrier C, after the second MFMA segment)
__device__ unsigned long long g_wg_dbg[8 * 8 * 8 * 8];
#define WG_TS(kb, k)                                                                           \
  if ((threadIdx.x & 63) == 0 && blockIdx.x < 8 && (kb) >= 16 && (kb) < 24)                     \
    g_wg_dbg[((blockIdx.x * 8 + (threadIdx.x >> 6)) * 8 + ((kb) - 16)) * 8 + (k)] =             \
        __builtin_amdgcn_s_memtime()
#else
#define WG_TS(kb, k)
#endif

namespace {

constexpr int PP_THREADS = 512;
constexpr int PBK = 64;                    // 16-bit K-elements per K-tile (128-B LDS rows)
constexpr int HALF = 128 * 128;            // one half-tile: 128 rows x 128 B
constexpr int BUF = 4 * HALF;              // A0 A1 B0 B1
constexpr int PP_LDS = 2 * BUF;            // 128 KB

__device__ __forceinline__ int swz(int row, int ch) { return ch ^ ((row >> 1) & 7); }

template <typename E> __device__ __forceinline__ E lo16(uint32_t w) {
  const uint16_t b = (uint16_t)(w & 0xffffu);
  E e;
  __builtin_memcpy(&e, &b, 2);
  return e;
}
template <typename E> __device__ __forceinline__ E hi16(uint32_t w) {
  const uint16_t b = (uint16_t)(w >> 16);
  E e;
  __builtin_memcpy(&e, &b, 2);
  return e;
}

// compiler fences around the raw barrier: nothing moves across it (IR or machine schedule)
__device__ __forceinline__ void pp_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}

// v[r] += v[r] of the DPP partner lane, as one v_add_f32_dpp per value (the builtin form was a
// v_mov_b32_dpp + v_add pair), 4 butterfly steps over 8 values in one block: a value's next
// step is 8 instructions after its previous one, so only the block's entry and exit need the
// s_nop for the VALU-write -> DPP-read hazard (inline asm is opaque to the hazard recognizer;
// the 4-value form needed one per step)
#define PP_ROW_SUM8(CTRL)                                                           \
  "v_add_f32_dpp %0, %0, %0 " CTRL " row_mask:0xf bank_mask:0xf\n"                   \
  "v_add_f32_dpp %1, %1, %1 " CTRL " row_mask:0xf bank_mask:0xf\n"                   \
  "v_add_f32_dpp %2, %2, %2 " CTRL " row_mask:0xf bank_mask:0xf\n"                   \
  "v_add_f32_dpp %3, %3, %3 " CTRL " row_mask:0xf bank_mask:0xf\n"                   \
  "v_add_f32_dpp %4, %4, %4 " CTRL " row_mask:0xf bank_mask:0xf\n"                   \
  "v_add_f32_dpp %5, %5, %5 " CTRL " row_mask:0xf bank_mask:0xf\n"                   \
  "v_add_f32_dpp %6, %6, %6 " CTRL " row_mask:0xf bank_mask:0xf\n"                   \
  "v_add_f32_dpp %7, %7, %7 " CTRL " row_mask:0xf bank_mask:0xf\n"
__device__ __forceinline__ void row_total8(float (&v)[8]) {
  asm volatile("s_nop 1\n" PP_ROW_SUM8("quad_perm:[1,0,3,2]") PP_ROW_SUM8("quad_perm:[2,3,0,1]")
               PP_ROW_SUM8("row_half_mirror") PP_ROW_SUM8("row_mirror") "s_nop 1"
               : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
                 "+v"(v[7]));
}

// PERSIST: 1 = loop over tiles (grid = CU count) with the next tile's first DMA overlapping the
// epilogue; 0 = one tile per workgroup (the residual-epilogue launches: their register
// budget goes to the residual prefetch instead of the next tile's address state); 3 =
// persistent, dense 1 x 1 rows with one residual fetched by LDS-DMA (RQP below)
template <typename E, int ST, int PERSIST>
__device__ __forceinline__ void conv_nt_pp_body(const ConvArgs& a) {
  typedef typename Half<E>::V V;
  constexpr int BM = 256, BN = 256;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;   // wm = wave row = ping-pong group
  const int lr = lane & 15, lq = lane >> 4;
  const long M = (long)a.N * a.Ho * a.Wo;
  const int mtiles = (int)((M + BM - 1) / BM);
  const int ntiles = (a.Co + BN - 1) / BN;
  const int nwg = mtiles * ntiles;
  // persistent: block b runs tiles t = b, b + G, ... (G = gridDim.x, a multiple of 8); the
  // XCD-aware bijective remap of t (XCD = t % 8 = b % 8) gives each XCD a contiguous run of
  // tiles, n fastest, so blocks sharing an A panel share an L2
  auto tile_of = [&](int t, int& mt_, int& nt_) {
    const int xcd = t & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (t >> 3);
    mt_ = wg / ntiles;
    nt_ = wg - mt_ * ntiles;
  };
  int tile = blockIdx.x;
  int mt, nt;
  tile_of(tile, mt, nt);
  long m0 = (long)mt * BM;
  int n0 = nt * BN;
  // ST == 4: the dense 1x1 path of ST == 0 plus a K-concatenated second GEMM (x2, w2) whose
  // K-tiles follow the first's (a separate instantiation: the extra addressing state cost the
  // plain 1x1 launches 4 % when it was a runtime branch of ST == 0)
  constexpr bool dual = ST == 4;
  const int nk = (a.KH * a.KW * a.C) / PBK + (dual ? a.C2 / PBK : 0);
  const int ntaps = a.KH * a.KW;
  // K-tile kb of the current tile is in buffer (kb + par) % 2; RQP starts a tile in whichever
  // buffer its predecessor's epilogue freed first (always 0 otherwise)
  int par = 0;
  const E* X = (const E*)a.x;
  const E* Wt = (const E*)a.w;

  // ---- operand addressing: buffer resources, 32-bit byte offsets per lane ----
  // Out-of-range taps and rows get the offset OOB (>= num_records): the buffer unit returns
  // zeros, so the LDS image is written whole with no zero-source select. The host guarantees
  // both operands are < 2^31 bytes.
  constexpr uint32_t OOB = 0x80000000u;
  const auto rs_x = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0,
                                                      (int)((long)a.N * a.H * a.W * a.ldx * 2), 0x00020000);
  const auto rs_w = __builtin_amdgcn_make_buffer_rsrc((void*)Wt, (short)0, (int)((long)a.Co * a.ldw * 2), 0x00020000);
  const auto rs_x2 = dual ? __builtin_amdgcn_make_buffer_rsrc((void*)a.x2, (short)0,
                                                              (int)((long)a.N * a.H * a.W * a.ldx2 * 2), 0x00020000)
                          : rs_x;
  const auto rs_w2 = dual ? __builtin_amdgcn_make_buffer_rsrc((void*)a.w2, (short)0, (int)((long)a.Co * a.ldw2 * 2), 0x00020000)
                          : rs_w;
  // A rows: half h, DMA instruction i -> tile row h*128 + (i*8+wave)*8 + lane/8 (j = h*2 + i).
  // ST == 1: byte offset of the tap-(0,0) source and a validity mask, bit kh (0-3) for the row
  // and bit 4+kw for the column of every tap; ST == 2 (transposed gather) decodes per tap.
  const int pc = lane & 7;
  int a_voff[4], a_bits[4], a_h0[4], a_w0[4], a_lc[4];
  long a_nb[4];
  uint32_t b_voff[4];
  int a_voff2[4];        // dual: the same rows of x2
  uint32_t b_voff2[4];   // dual: the same output channels of w2
  auto setup_lanes = [&](long m0_, int n0_) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int rr = ((j & 1) * 8 + wave) * 8 + (lane >> 3);
      // LDS half h = j >> 1, position rr -> tile row: wave row rr / 64 owns the contiguous
      // tile rows [128 * (rr / 64), +128) (quadrant qm = h: rows qm * 64 + 0..63)
      const int row = (rr >> 6) * 128 + (j >> 1) * 64 + (rr & 63);
      a_lc[j] = swz(rr, pc);
      // 32-bit index math (M, N*H*W < 2^31: host check): 64-bit div/rem per row was ~1/3 of
      // the per-tile setup on short-K layers
      const int m = (int)m0_ + row;
      const bool ok = m < (int)M;
      if constexpr (ST == 0 || ST == 4) {
        // 1x1, stride 1, no padding (H x W = Ho x Wo): the source row IS pixel m, every tap
        // valid; no pixel decode (the divisions were ~2.5k cycles of the per-tile setup)
        a_voff[j] = (ok ? m : 0) * a.ldx * 2 + a_lc[j] * 16;
        a_voff2[j] = dual ? (ok ? m : 0) * a.ldx2 * 2 + a_lc[j] * 16 : 0;
        a_bits[j] = ok ? 0x11 : 0;
        continue;
      }
      const unsigned mm = ok ? (unsigned)m : 0u;
      const unsigned t = mm / (unsigned)a.Wo;
      const int wo = (int)(mm - t * (unsigned)a.Wo);
      const unsigned nimg = t / (unsigned)a.Ho;
      const int ho = (int)(t - nimg * (unsigned)a.Ho);
      a_nb[j] = (long)(nimg * (unsigned)a.H);
      a_h0[j] = ok ? ho * a.sf - a.pad_h : -(1 << 28);
      a_w0[j] = wo * a.sf - a.pad_w;
      a_voff[j] = (((int)a_nb[j] + a_h0[j]) * a.W + a_w0[j]) * a.ldx * 2 + a_lc[j] * 16;
      int bits = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (q < a.KH) bits |= ((unsigned)(a_h0[j] + q * a.dil) < (unsigned)a.H) << q;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (q < a.KW) bits |= ((unsigned)(a_w0[j] + q * a.dil) < (unsigned)a.W) << (4 + q);
      a_bits[j] = bits;
    }
    // B rows: half g, instruction i -> output channel n0 + g*128 + (i*8+wave)*8 + lane/8
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int rr = ((j & 1) * 8 + wave) * 8 + (lane >> 3);
      const int co = n0_ + (j >> 1) * 128 + rr;
      b_voff[j] = co < a.Co ? (uint32_t)((co * a.ldw + swz(rr, pc) * 8) * 2) : OOB;
      b_voff2[j] = dual && co < a.Co ? (uint32_t)((co * a.ldw2 + swz(rr, pc) * 8) * 2) : OOB;
    }
  };
  setup_lanes(m0, n0);

  // per-K-tile wave-uniform decode. K-tile order: channel chunk outer, tap inner, so the
  // KH*KW shifted reads of one chunk's source rows follow each other while they are in L2
  struct KT { int need, s_tap2, k02, dh, dw, c0, sec; };
  int nx_tap = 0, nx_c0 = 0, nx_sec = 0;   // (tap, chunk, GEMM) of the next K-tile to decode
  auto ktile_next = [&]() {
    KT t;
    const int tap = nx_tap;
    t.c0 = nx_c0;
    t.sec = nx_sec;
    if (++nx_tap == ntaps) { nx_tap = 0; nx_c0 += PBK; }
    if (dual && nx_sec == 0 && nx_c0 == a.C) { nx_sec = 1; nx_c0 = 0; }
    const int kh = tap / a.KW, kw = tap - kh * a.KW;
    t.dh = kh * a.dil;
    t.dw = kw * a.dil;
    t.need = (1 << kh) | (16 << kw);
    t.s_tap2 = ((t.dh * a.W + t.dw) * a.ldx + t.c0) * 2;
    t.k02 = (tap * a.C + t.c0) * 2;   // weight column, bytes
    return t;
  };

  // half ids: 0 = A0, 1 = A1, 2 = B0, 3 = B1 (LDS offset hid * HALF inside a K-tile buffer)
  auto issue_half = [&](int kb, const KT& t, int hid, int i0 = 0, int i1 = 2) {
    char* dst = smem + ((kb + par) & 1) * BUF + hid * HALF;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i < i0 || i >= i1) continue;
      auto* ldst = (__attribute__((address_space(3))) void*)(dst + (i * 8 + wave) * 1024);
      if (hid < 2) {
        const int j = hid * 2 + i;
        uint32_t off;
        if (dual && t.sec) {   // wave-uniform: the second GEMM's A rows (dense 1x1)
          off = a_bits[j] ? (uint32_t)(a_voff2[j] + t.s_tap2) : OOB;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_x2, ldst, 16, off, 0, 0, 0);
          continue;
        }
        if constexpr (ST <= 1 || ST == 4) {
          off = (a_bits[j] & t.need) == t.need ? (uint32_t)(a_voff[j] + t.s_tap2) : OOB;
        } else {
          int hi = a_h0[j] + t.dh, wi = a_w0[j] + t.dw;
          bool ok = (hi >= 0) & (wi >= 0) & ((hi % ST) == 0) & ((wi % ST) == 0);
          hi /= ST;
          wi /= ST;
          ok &= (hi < a.H) & (wi < a.W);
          off = ok ? (uint32_t)(((int)((a_nb[j] + hi) * a.W + wi) * a.ldx + t.c0 + a_lc[j] * 8) * 2) : OOB;
        }
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_x, ldst, 16, off, 0, 0, 0);
      } else {
        const int j = (hid - 2) * 2 + i;
        if (dual && t.sec) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_w2, ldst, 16, b_voff2[j] + t.k02, 0, 0, 0);
        else __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_w, ldst, 16, b_voff[j] + t.k02, 0, 0, 0);
      }
    }
  };

  f32x4_t acc[2][2][4][2];   // [qm][qn][fi][fj]

  V af[4][2], bfq[2][2][2];   // [frag][k-half]; B per quadrant qn: B0 kept for phase 3
  auto read_a = [&](const char* buf, int qm) {
    const char* A = buf + qm * HALF;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + i * 16 + lr;
#pragma unroll
      for (int s = 0; s < 2; ++s) af[i][s] = *(const V*)(A + row * 128 + swz(row, lq + 4 * s) * 16);
    }
  };
  auto read_b = [&](const char* buf, int qn) {
    const char* B = buf + (2 + qn) * HALF;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = wn * 32 + j * 16 + lr;
#pragma unroll
      for (int s = 0; s < 2; ++s) bfq[qn][j][s] = *(const V*)(B + row * 128 + swz(row, lq + 4 * s) * 16);
    }
  };
  auto mfma_q = [&](int qm, int qn) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          // transposed accumulators (lane = 4 channels of one pixel) for the register-side
          // statistics and 8-byte staging writes
          acc[qm][qn][i][j] = Half<E>::mma(bfq[qn][j][s], af[i][s], acc[qm][qn][i][j]);
  };

  // ---- prologue of a tile: K-tile 0, halves in issue order A0, B0, B1, A1 ----
  auto prologue = [&]() {
    nx_tap = 0;
    nx_c0 = 0;
    nx_sec = 0;
    const KT t0 = ktile_next();
    issue_half(0, t0, 0);
    issue_half(0, t0, 2);
    issue_half(0, t0, 3);
    issue_half(0, t0, 1);
  };
  // RQP (round 6): the residual data gradients (dense 1 x 1 rows, one residual: the identity
  // units' conv1, DESIGN.md staged residuals) run persistent, the residual tile fetched by
  // LDS-DMA instead of global loads in the epilogue, whose latency the per-tile stamps showed
  // exposed (one-tile launches: epilogue 21k cycles against 6k without a residual,
  // profiles/r06_s18_rqp.txt): the tile's column half 0 (128 columns, 64 KB) streams into the
  // K-tile buffer the last K-tile does not read, during that K-tile; half 1 into the other
  // buffer as soon as the main loop ends. Each wave adds its accumulators to the residual in
  // place, in the accumulator layout, then every wave streams rows out of the sums; once half
  // 0's rows are out, the next tile's mask bytes and K-tile 0 go into its buffer, in flight
  // during half 1. dx = round(dgrad + r) (one rounding), then the consumer's ReLU bits
  constexpr bool RQP = PERSIST == 3;
  static_assert(!RQP || ST == 0, "RQP: dense 1 x 1 rows only");
  // pp_launch_st: a.r set, a.r2 not, M * ldr * 2 < 2^31
  const auto rs_r = __builtin_amdgcn_make_buffer_rsrc((void*)a.r, (short)0,
                                                      (int)(RQP ? (long)M * a.ldr * 2 : 0), 0x00020000);
  // Each wave fetches exactly the residual it adds in place -- rows wm * 128 .. + 127, columns wn * 32 .. + 31 of a 128-column half: 8
  // pieces of 16 rows x 64 B. LDS: half = 4 column groups (wn) of 256 rows x 64 B; 16-B chunk
  // s of row r at slot s ^ ((r / 4) % 4): conflict-free 8-B accesses for the 16 rows of a
  // fragment and 16-B reads of 4 rows x 4 groups per instruction
  // offsets: a lane part (tile-independent, one register) plus a wave-uniform part; rows past
  // M fall past the buffer's end (zeros), columns past Co are read but never stored
  const uint32_t rw_lane = RQP ? (uint32_t)(((lane >> 2) * a.ldr + (((lane & 3) ^ ((lane >> 4) & 3)) << 3)) * 2) : 0u;
  auto issue_resw = [&](int hh, char* dst) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      // (unsigned: rows past M may wrap; they are read, never stored)
      const uint32_t sb = ((uint32_t)m0 + (uint32_t)(wm * 128 + i * 16)) * (uint32_t)a.ldr * 2u +
                          (uint32_t)(n0 + hh * 128 + wn * 32) * 2u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs_r, (__attribute__((address_space(3))) void*)(dst + wn * 16384 + (wm * 128 + i * 16) * 64), 16, rw_lane + sb, 0, 0, 0);
    }
  };
  // RQP: the consumer's ReLU bytes of the chunks a thread stores (row k * 32 + wave * 4 +
  // (lane / 4) % 4, chunk 4 * (lane / 16) + lane % 4 of half qn), by byte buffer loads (rows
  // past M read 0)
  const auto rs_m = __builtin_amdgcn_make_buffer_rsrc((void*)a.omask, (short)0,
                                                      (int)(RQP && a.omask ? M * a.ldm : 0), 0x00020000);
  const uint32_t mk_lane = RQP ? (uint32_t)(((lane >> 2) & 3) * a.ldm + (lane >> 4) * 4 + (lane & 3)) : 0u;
  auto load_mask = [&](long m0_, int n0_, uint32_t (&mbx)[16]) {
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t sb = (uint32_t)(((int)m0_ + k * 32 + wave * 4) * a.ldm + ((n0_ + qn * 128) >> 3));
        mbx[qn * 8 + k] = __builtin_amdgcn_raw_buffer_load_b8(rs_m, mk_lane + sb, 0, 0);
      }
  };
  // consumer ReLU bits (ConvArgs::omask, one-tile and RQP launches): one byte per 16-B chunk
  // the epilogue stores, one to a register (packing them would wait for the loads here), loaded
  // before the K-tile 0 DMA so their latency hides behind it and the main loop (loaded in the
  // epilogue, their latency cost ~4 us per tile: block4 conv1 dgrad +20 %): half qn, pass k
  // in mb[qn * 8 + k] (one-tile: rows k * 32 + tid / 16, chunk tid % 16 of the half; RQP:
  // load_mask), all ones in RQP launches without a mask
  uint32_t mb[16];
  const bool omask = PERSIST != 1 && a.omask;   // wave-uniform
  if constexpr (RQP) {
    if (omask) load_mask(m0, n0, mb);
    else
#pragma unroll
      for (int k = 0; k < 16; ++k) mb[k] = ~0u;
    __builtin_amdgcn_sched_barrier(0);
  } else if (omask) {
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const long m = m0 + k * 32 + (tid >> 4);
        const int n = n0 + qn * 128 + (tid & 15) * 8;
        mb[qn * 8 + k] = m < M && n < a.Co ? a.omask[(size_t)m * a.ldm + (n >> 3)] : 0u;
      }
    __builtin_amdgcn_sched_barrier(0);   // keep the loads here, ahead of the prologue's DMA
  }
  prologue();
  int dbg_it = 0; (void)dbg_it;
  for (;;) {   // ---- persistent tile loop ----
  PP_TS(dbg_it, 0);
#pragma unroll
  for (int qm = 0; qm < 2; ++qm)
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[qm][qn][i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  // A0, B0 of K-tile 0 landed (B1, A1 in flight; a previous tile's epilogue stores, issued
  // after them, count too and are waited for here)
  asm volatile("s_waitcnt vmcnt(2)" ::: "memory");   // A0, B0, B1 landed (A1 in flight)
  // RQP: the tile's mask bytes (issued before its K-tile 0) landed too: four to a register
  // through the main loop
  uint32_t mp[4];
  if constexpr (RQP) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      mp[q] = (mb[4 * q] & 0xffu) | (mb[4 * q + 1] & 0xffu) << 8 | (mb[4 * q + 2] & 0xffu) << 16 | mb[4 * q + 3] << 24;
  }
  pp_barrier();
  if (wm == 1) pp_barrier();   // stagger: wave row 1 runs one segment behind
  // the lagging row loses every issue arbitration at equal priority: one static raise for the
  // main loop instead of per-segment flips (MI355X_MICROARCH.md, two waves per SIMD, item 4)
  if (wm == 1) __builtin_amdgcn_s_setprio(1);

  {
    // two phases per K-tile (half the barriers): phase 0 = quadrants (0,0), (0,1) from A0, B0,
    // B1; phase 1 = (1,1), (1,0) from A1 (B kept in registers).
    // balanced DMA (as the weight-gradient kernel): K-tile k's halves are issued A0 + B1 in
    // L1(k-2) and B0 + A1 in L0(k-1) (K-tile 1's A0 + B1 in L0(0): buffer 1 holds the previous
    // tile's epilogue staging until the tile-start barrier); every load segment ends with its
    // LDS reads complete, so a DMA issued after the next barrier cannot overwrite a half that
    // another wave is still reading
    KT tn1{};
#ifdef NT_DBG_TIMING
    const int nt_kb0 = nk >= 24 ? 16 : 0;
#endif
    for (int kb = 0; kb < nk; ++kb) {
      const char* buf = smem + ((kb + par) & 1) * BUF;
      const bool m1 = kb + 1 < nk, m2 = kb + 2 < nk;
      NT_TS(kb, 0);
      read_a(buf, 0);
      read_b(buf, 0);
      read_b(buf, 1);
      if (kb == 0 && m1) {
        tn1 = ktile_next();
        issue_half(1, tn1, 0);
        issue_half(1, tn1, 3);
      }
      if (m1) {
        issue_half(kb + 1, tn1, 2);
        issue_half(kb + 1, tn1, 1);
      }
      if constexpr (RQP) {   // the last K-tile: residual half 0 into the buffer it does not read
        if (!m1) issue_resw(0, smem + ((nk + par) & 1) * BUF);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (wm == 1) {
        if (m1 || RQP) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // (RQP: its 8 residual pieces)
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      NT_TS(kb, 1);
      pp_barrier();
      NT_TS(kb, 2);
      mfma_q(0, 0);
      mfma_q(0, 1);
      if (wm == 0) {
        if (m1 || RQP) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      NT_TS(kb, 3);
      pp_barrier();
      NT_TS(kb, 4);
      read_a(buf, 1);
      if (m2) {
        tn1 = ktile_next();
        issue_half(kb + 2, tn1, 0);
        issue_half(kb + 2, tn1, 3);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (m1 && wm == 1) {
        if (m2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      }
      NT_TS(kb, 5);
      pp_barrier();
      NT_TS(kb, 6);
      mfma_q(1, 1);
      mfma_q(1, 0);
      NT_TS(kb, 7);
      if (m1 && wm == 0) {
        if (m2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      }
      pp_barrier();
    }
  }
  if (wm == 0) pp_barrier();   // realign the two wave rows: every LDS read of the tile is done
  __builtin_amdgcn_s_setprio(0);
  PP_TS(dbg_it, 1);
  // next tile: its K-tile 0 goes into buffer 0 now, in flight during this tile's epilogue
  const int tile_n = tile + (int)gridDim.x;
  const bool has_next = (PERSIST == 1 || RQP) && tile_n < nwg;
  int mt_n = 0, nt_n = 0;
  if (PERSIST == 1 && has_next) {
    tile_of(tile_n, mt_n, nt_n);
    setup_lanes((long)mt_n * BM, nt_n * BN);
    prologue();
  }
  {
      // ---- epilogue: transposed accumulators (mfma(B, A)): lane (lq, lr) of
      // fragment acc[qm][qn][i][j] holds output pixel m = m0 + wm*128 + qm*64 + i*16 + lr and
      // the four channels n = n0 + qn*128 + wn*32 + j*16 + lq*4 + 0..3
    const long mw = m0 + wm * 128;                      // this wave row's 128 contiguous rows
    const long mrows = M - mw;
    const int nvalid = (int)(mrows < 0 ? 0 : (mrows < 128 ? mrows : 128));
    const int nbase = n0 + wn * 32 + lq * 4;
    // per channel (sum, M2) over the wave row's rows: 8 values in the lane, then a butterfly
    // over the 16 lanes (lr) holding the same channels; one partial per 128 rows
    // (conv_nt_stat_rows); the ragged last tile merges with per-lane counts. Run per column
    // half between that half's staging writes and the barrier, so the VALU work overlaps the
    // LDS traffic and the other waves' arrival
    const bool full = nvalid == 128;
    auto store_stats = [&](const int qn, const int j, const float* sm, const float* m2) {
      const int n = nbase + qn * 128 + j * 16;
      if (lr == 0 && n < a.Co) {
        float* dst = a.stats + 2 * ((size_t)(mt * 2 + wm) * a.Co + n);
        *(float4*)dst = make_float4(sm[0], m2[0], sm[1], m2[1]);
        *(float4*)(dst + 4) = make_float4(sm[2], m2[2], sm[3], m2[3]);
      }
    };
    auto stats_half = [&](const int qn) {
      if (full) {
        // exact two-pass moments over the wave row's 128 rows, both column fragments j at once:
        // the 8 rows of the lane are summed, the sums are completed over the 16 lanes of the
        // row group by a DPP-add butterfly (quad_perm xor 1, xor 2, row_half_mirror,
        // row_mirror: every lane ends with the totals), then the squared deviations from those
        // means the same way
        float sm[8], m2[8];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x4_t s4 = acc[0][qn][0][j];
#pragma unroll
          for (int f = 1; f < 8; ++f) s4 += acc[f >> 2][qn][f & 3][j];
#pragma unroll
          for (int r = 0; r < 4; ++r) sm[j * 4 + r] = s4[r];
        }
        row_total8(sm);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x4_t mu;
#pragma unroll
          for (int r = 0; r < 4; ++r) mu[r] = sm[j * 4 + r] * (1.f / 128.f);
          f32x4_t q4 = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int f = 0; f < 8; ++f) {
            const f32x4_t d = acc[f >> 2][qn][f & 3][j] - mu;
            q4 += d * d;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) m2[j * 4 + r] = q4[r];
        }
        row_total8(m2);
        store_stats(qn, 0, sm, m2);
        store_stats(qn, 1, sm + 4, m2 + 4);
        return;
      }
  #pragma unroll
        for (int j = 0; j < 2; ++j) {
          float sm[4], m2[4];
          {
            // ragged last tile: per-lane counts, general merges
            int c = 0;
  #pragma unroll
            for (int qm = 0; qm < 2; ++qm)
  #pragma unroll
              for (int i = 0; i < 4; ++i) c += (qm * 64 + i * 16 + lr) < nvalid;
            const float cnt = (float)c;
  #pragma unroll
            for (int r = 0; r < 4; ++r) {
              float s_ = 0.f;
  #pragma unroll
              for (int qm = 0; qm < 2; ++qm)
  #pragma unroll
                for (int i = 0; i < 4; ++i)
                  s_ += (qm * 64 + i * 16 + lr) < nvalid ? acc[qm][qn][i][j][r] : 0.f;
              const float mu = cnt > 0.f ? s_ / cnt : 0.f;
              float q_ = 0.f;
  #pragma unroll
              for (int qm = 0; qm < 2; ++qm)
  #pragma unroll
                for (int i = 0; i < 4; ++i) {
                  const float d = acc[qm][qn][i][j][r] - mu;
                  q_ += (qm * 64 + i * 16 + lr) < nvalid ? d * d : 0.f;
                }
              sm[r] = s_;
              m2[r] = q_;
            }
            float nn = cnt;
  #pragma unroll
            for (int o = 1; o <= 8; o <<= 1) {
              const float n2 = __shfl_xor(nn, o, 64);
  #pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float s2 = __shfl_xor(sm[r], o, 64), q2 = __shfl_xor(m2[r], o, 64);
                const float tot = nn + n2;
                const float d = (n2 > 0.f && nn > 0.f) ? s2 / n2 - sm[r] / nn : 0.f;
                m2[r] = m2[r] + q2 + (tot > 0.f ? d * d * (nn * n2 / tot) : 0.f);
                sm[r] += s2;
              }
              nn = nn + n2;
            }
          }
          store_stats(qn, j, sm, m2);
        }
    };
    PP_TS(dbg_it, 2);
    // output: packed to 16-bit in registers, staged one 128-column half at a time through the
    // buffer-1 region (row-major, 16-B chunks XOR-swizzled by row: conflict-free 8-B writes
    // and 16-B reads), then 16 B per lane, 256 contiguous bytes per row, streaming stores
    typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
    typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
    auto pack4 = [](const f32x4_t& v) {
      u32x2_t w;
#pragma unroll
      for (int h = 0; h < 2; ++h) w[h] = pack2<E>(v[2 * h], v[2 * h + 1]);
      return w;
    };
    char* const stg = smem + BUF;
    E* Y = (E*)a.y;
    const int s_row = tid >> 4, s_ch = tid & 15;

    // residuals (dgrad: dx = dgrad + r1 [+ r2]; one-tile launches only, pp_launch_st) are read
    // in the staged layout -- 16 B per lane, 256 contiguous bytes per row, issued before the
    // half's staging writes -- and added after the LDS round trip, in fp32, rounded once more
    // (round 3: they were read in the accumulator layout, 8 B per lane from 16 rows per load,
    // a quadrant at a time, and added before the single rounding: the short-K residual data
    // gradients 6-8 % slower, the step -0.6 %; profiles/r03_res_staged.txt)
    if constexpr (RQP) {
      char* const hres[2] = {smem + ((nk + par) & 1) * BUF,       // half 0: the last K-tile's DMA
                             smem + ((nk - 1 + par) & 1) * BUF};  // half 1: free from here on
      issue_resw(1, hres[1]);
      // every store of half 0 issues (8 per thread): the wait for half 1 may count them
      const bool fullt = m0 + BM <= M && n0 + BN <= a.Co;
      typedef float f32x2_t __attribute__((ext_vector_type(2)));
      // lane-derived addresses from an opaque zero: hoisted out of the tile loop they were live
      // through the main loop (spilled)
      int ez;
      asm volatile("s_mov_b32 %0, 0" : "=s"(ez));
      const int lre = lr + ez, lanee = lane + ez;
#pragma unroll
      for (int qn = 0; qn < 2; ++qn) {
        char* const hw = hres[qn] + wn * 16384;
        // this wave's residual of half qn landed (each wave adds only what it fetched); half 1:
        // half 0's 8 stores, the next tile's 16 mask loads and 8 K-tile-0 pieces are younger
        if (qn == 0) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if (!fullt) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if (has_next) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        PP_TS(dbg_it, 4 + 3 * qn);
        // in place, accumulator layout: dx = round(dgrad + r), one rounding
        u32x2_t rr[2][4][2];
#pragma unroll
        for (int qm = 0; qm < 2; ++qm)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const int row = wm * 128 + qm * 64 + i * 16 + lre;
              const int sl = j * 2 + (lq >> 1);
              rr[qm][i][j] = *(const u32x2_t*)(hw + row * 64 + ((sl ^ ((row >> 2) & 3)) << 4) + (lq & 1) * 8);
            }
#pragma unroll
        for (int qm = 0; qm < 2; ++qm)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const int row = wm * 128 + qm * 64 + i * 16 + lre;
              const int sl = j * 2 + (lq >> 1);
              const f32x4_t& x = acc[qm][qn][i][j];
              u32x2_t o;
#pragma unroll
              for (int w = 0; w < 2; ++w) {
                const uint32_t r = rr[qm][i][j][w];
                const f32x2_t xs = {x[2 * w], x[2 * w + 1]};
                const f32x2_t rs = {TypeOps<E>::to_f(lo16<E>(r)), TypeOps<E>::to_f(hi16<E>(r))};
                const f32x2_t sum = xs + rs;
                o[w] = pack2<E>(sum[0], sum[1]);
              }
              *(u32x2_t*)(hw + row * 64 + ((sl ^ ((row >> 2) & 3)) << 4) + (lq & 1) * 8) = o;
            }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        pp_barrier();
        PP_TS(dbg_it, 5 + 3 * qn);
        // rows out: per instruction 4 rows x 256 B (lane: group lane / 16, row (lane / 4) % 4,
        // chunk lane % 4 of the group), masked by the consumer's ReLU bits
        const int g = lanee >> 4, sl = lanee & 3;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int row = k * 32 + wave * 4 + ((lanee >> 2) & 3);
          u32x4_t v = *(const u32x4_t*)(hres[qn] + g * 16384 + row * 64 + ((sl ^ ((row >> 2) & 3)) << 4));
          const uint32_t b = mp[qn * 2 + (k >> 2)] >> (8 * (k & 3));
#pragma unroll
          for (int w = 0; w < 4; ++w)
            v[w] &= ((b >> (2 * w)) & 1u ? 0x0000ffffu : 0u) | ((b >> (2 * w)) & 2u ? 0xffff0000u : 0u);
          const long m = m0 + row;
          const int n = n0 + qn * 128 + g * 32 + sl * 8;
          if (m < M && n < a.Co) __builtin_nontemporal_store(v, (u32x4_t*)(Y + (size_t)m * a.ldy + n));
        }
        PP_TS(dbg_it, 6 + 3 * qn);
        if (qn == 0 && has_next) {
          // half 0's buffer is free once every wave's reads of it are done: the next tile's
          // mask bytes and K-tile 0 go there, in flight during half 1
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          pp_barrier();
          tile_of(tile_n, mt_n, nt_n);
          const long m0n = (long)mt_n * BM;
          const int n0n = nt_n * BN;
          if (omask) load_mask(m0n, n0n, mb);   // (the current tile's bits are in mp)
          setup_lanes(m0n, n0n);
          par = (nk + par) & 1;
          prologue();
        }
      }
      goto rq_done;
    }
    const E* R1 = (const E*)a.r;
    const E* R2 = (const E*)a.r2;
    const int nres = PERSIST == 1 ? 0 : (R1 ? 1 : 0) + (R2 ? 1 : 0);   // wave-uniform
#pragma unroll
    for (int qn = 0; qn < 2; ++qn) {
      u32x4_t rs1[8], rs2[8];
      if (nres) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const long m = m0 + k * 32 + s_row;
          const long mc = m < M ? m : M - 1;
          const int n = n0 + qn * 128 + s_ch * 8;
          const int nc = n < a.Co ? n : 0;
          rs1[k] = *(const u32x4_t*)(R1 + (size_t)mc * a.ldr + nc);
          if (nres == 2) rs2[k] = *(const u32x4_t*)(R2 + (size_t)mc * a.ldr2 + nc);
        }
      }
#pragma unroll
      for (int qm = 0; qm < 2; ++qm) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int row = wm * 128 + qm * 64 + i * 16 + lr;
            const int ch = wn * 4 + j * 2 + (lq >> 1);
            *(u32x2_t*)(stg + row * 256 + ((ch ^ (row & 15)) << 4) + (lq & 1) * 8) = pack4(acc[qm][qn][i][j]);
          }
      }
      PP_TS(dbg_it, 4 + 4 * qn);
      if (a.stats && nvalid > 0) stats_half(qn);
      PP_TS(dbg_it, 5 + 4 * qn);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      pp_barrier();
      PP_TS(dbg_it, 6 + 4 * qn);
      u32x4_t v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int row = k * 32 + s_row;
        v[k] = *(const u32x4_t*)(stg + row * 256 + ((s_ch ^ (row & 15)) << 4));
      }
      const int n = n0 + qn * 128 + s_ch * 8;
      if (nres) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const uint32_t x = v[k][w], r = rs1[k][w], r2 = nres == 2 ? rs2[k][w] : 0u;
            float lo = TypeOps<E>::to_f(lo16<E>(x)) + TypeOps<E>::to_f(lo16<E>(r));
            float hi = TypeOps<E>::to_f(hi16<E>(x)) + TypeOps<E>::to_f(hi16<E>(r));
            if (nres == 2) { lo += TypeOps<E>::to_f(lo16<E>(r2)); hi += TypeOps<E>::to_f(hi16<E>(r2)); }
            v[k][w] = pack2<E>(lo, hi);
          }
      }
      if (omask) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const uint32_t b = mb[qn * 8 + k] >> (2 * w);
            v[k][w] &= ((b & 1u) ? 0x0000ffffu : 0u) | ((b & 2u) ? 0xffff0000u : 0u);
          }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const long m = m0 + k * 32 + s_row;
        if (m < M && n < a.Co) __builtin_nontemporal_store(v[k], (u32x4_t*)(Y + (size_t)m * a.ldy + n));
      }
      PP_TS(dbg_it, 7 + 4 * qn);
      if (qn == 0) {   // the second half overwrites the staging area
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        pp_barrier();
      }
    }
  }
rq_done:
  PP_TS(dbg_it, 3);
  ++dbg_it;
  if (!has_next) break;
  tile = tile_n;
  mt = mt_n;
  nt = nt_n;
  m0 = (long)mt * BM;
  n0 = nt * BN;
  }   // persistent tile loop
}

// (the body is a device function: the host pass does not parse buffer-resource values)
template <typename E, int ST, int PERSIST>
__global__ __launch_bounds__(PP_THREADS, 1) void conv_nt_pp_kernel(ConvArgs a) {
  conv_nt_pp_body<E, ST, PERSIST>(a);
}

int pp_grid(int nwg) {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
    ncu = (ncu + 7) / 8 * 8;   // a multiple of the XCD count keeps tile t on XCD t % 8
  }
  return nwg < ncu ? nwg : ncu;
}

template <typename E, int ST, int PERSIST>
hipError_t pp_launch(const ConvArgs& a, hipStream_t s) {
  // two K-tile buffers (the epilogue stages through buffer 1; RQP: the residual tile)
  constexpr int LDS = PP_LDS;
  auto kern = conv_nt_pp_kernel<E, ST, PERSIST>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const long M = (long)a.N * a.Ho * a.Wo;
  const int nwg = ceil_div(M, 256) * ceil_div(a.Co, 256);
  hipLaunchKernelGGL(kern, dim3(PERSIST == 1 || PERSIST == 3 ? pp_grid(nwg) : nwg), dim3(PP_THREADS), LDS, s, a);
  return hipGetLastError();
}

template <typename E, int ST>
hipError_t pp_launch_st(const ConvArgs& a, hipStream_t s) {
  if constexpr (ST == 0) {   // dense 1 x 1 rows, one residual: the residual tile by LDS-DMA
    if (a.r && !a.r2 && (long)a.N * a.Ho * a.Wo * a.ldr * 2 < (1L << 31))
      return pp_launch<E, 0, 3>(a, s);
  }
  if (a.r || a.r2 || a.omask) return pp_launch<E, ST, 0>(a, s);
  return pp_launch<E, ST, 1>(a, s);
}

}  // namespace

// ping-pong config: the v2 fast-path preconditions (conv_nt_v2_ok, no tap8), Co > 128 and an
// operands of < 2^31 bytes (32-bit buffer offsets), kernels up to 4 x 4 (tap validity bits)
bool conv_nt_pp_ok(const ConvArgs& a) {
  // 16-byte epilogue stores: channel counts and row strides multiples of 8
  return !a.tap8 && a.Co > 128 && a.Co % 8 == 0 && a.ldy % 8 == 0 &&
         a.KH <= 4 && a.KW <= 4 && conv_nt_v2_ok(a) &&
         (long)a.N * a.H * a.W * a.ldx * 2 < (1L << 31) && (long)a.Co * a.ldw * 2 < (1L << 31) &&
         (long)a.N * a.Ho * a.Wo < (1L << 31) &&   // 32-bit pixel indices
         (!a.x2 || (a.KH == 1 && a.KW == 1 && a.st == 1 && a.sf == 1 && a.pad_h == 0 && a.pad_w == 0 &&
                    a.H == a.Ho && a.W == a.Wo && a.C % 64 == 0 && a.C2 % 64 == 0 && a.ldx2 % 8 == 0 &&
                    a.ldw2 % 8 == 0 && (long)a.N * a.H * a.W * a.ldx2 * 2 < (1L << 31) &&
                    (long)a.Co * a.ldw2 * 2 < (1L << 31) && !a.r && !a.r2));
}

bool conv_nt_omask_ok(int dtype, const ConvArgs& a) {
  return seg_half(dtype) && !a.tap8 && a.st == 1 && a.KH == 1 && a.KW == 1 && a.sf == 1 &&
         a.pad_h == 0 && a.pad_w == 0 && a.H == a.Ho && a.W == a.Wo && a.Co > 128 &&
         conv_nt_pp_ok(a) && a.ldm >= a.Co / 8;
}

template <typename E>
hipError_t nt_pp_e(const ConvArgs& a, hipStream_t s) {
  if (a.st == 1 && a.KH == 1 && a.KW == 1 && a.sf == 1 && a.pad_h == 0 && a.pad_w == 0 &&
      a.H == a.Ho && a.W == a.Wo)
    return a.x2 ? pp_launch_st<E, 4>(a, s)    // dense 1x1 rows + the second GEMM
                : pp_launch_st<E, 0>(a, s);   // dense 1x1 rows
  if (a.st == 1) return pp_launch_st<E, 1>(a, s);
  if (a.st == 2) return pp_launch_st<E, 2>(a, s);
  return hipErrorInvalidValue;
}

hipError_t launch_conv_nt_pp(int dtype, const ConvArgs& a, hipStream_t s) {
  if (dtype == SEG_F16) return nt_pp_e<f16_t>(a, s);
  return nt_pp_e<bf16_t>(a, s);
}

// ======================================================================================
// 16-bit weight gradient, ping-pong schedule: C[co][tap*Ci+ci] = sum_p dy[p][co] * x[src(p,tap)][ci]
//
// The NT kernel's main loop (two phases of two quadrants per K-tile) transposed to the TN
// problem of conv_wgrad_v2_kernel: 256 (co) x 256 (tap,ci) tile, 8 waves as 2 x 4 with 128 x 64
// wave tiles in four 64 x 32 quadrants; a K-tile is 64 pixels; each half-tile is 64 pixel rows x 256 B (128 co of dy, or 128 columns
// of the gathered x) read by ds_read_b64_tr_b16 through the XOR swizzle of the v2 kernel.
// Operands come through buffer resources: dy rows are one add per DMA, x rows are decoded once
// per K-tile and lane (pixel -> n, ho, wo by row carries) and shared by both x halves.
// Split-K over pixels into fp32 slabs as in v2 (reduced by splitk_reduce).
// Round 3: the 8 DMA pieces of a K-tile are spread so that the load segments (fragment reads)
// and the MFMA segments of the partner wave row take about the same time: per-segment s_memtime
// stamps (tools/wg_timing.py) had the load segments at 1.5-2x the MFMA segments. 6/2 -> 4/4 over
// the two load segments (block4 3x3 622 -> 599 us), then the four dy pieces (one VALU of address
// math each) moved into the MFMA segments, one per quadrant (599 -> 572 us; the 1x1 layers 2-6 %
// each step; profiles/r03_wgrad_bal.txt, r03_wgrad_mseg.txt). Moving the x pieces too, or the
// x-row decode, made the MFMA segments the longer ones (rejected).
// ======================================================================================
namespace {

constexpr int WHALF = 64 * 256;
constexpr int WBUF = 4 * WHALF;
constexpr int WPP_LDS = 2 * WBUF;

__device__ __forceinline__ int wpp_swz(int row, int ch) { return ch ^ (2 * (row & 3) + 8 * ((row >> 3) & 1)); }

// FAST: 1 = Wo >= 64 (a K-tile's rows need at most one row carry); 2 = strip order (Wo a
// multiple of 64): a K-tile is 64 pixels of one output row, and consecutive K-tiles walk DOWN a
// 64-pixel-wide column strip (n, strip, ho; ho fastest) instead of along the rows. A dilated 3x3
// layer reads input rows ho - d, ho, ho + d for output row ho, so one input row is re-read d
// K-tiles later in strip order against d * Wo / 64 K-tiles in raster order: with the 32
// workgroups of an XCD walking the same split, the reuse window is ~1 MB of L2 instead of ~4 MB
// (block4, rate 4, Wo 256), which is the XCD's whole L2.
template <typename E, int FAST>
__device__ __forceinline__ void conv_wgrad_pp_body(const WgradArgs& a) {
  typedef typename Half<E>::V V;
  constexpr int BM = 256, BN = 256, PK = 64;
  constexpr uint32_t OOB = 0x80000000u;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int Ncol = a.KH * a.KW * a.C;
  const int P = a.N * a.Ho * a.Wo;
  const int mtn = (a.Co + BM - 1) / BM, ntn = (Ncol + BN - 1) / BN;
  const int nwg = mtn * ntn * a.splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int split = wg / (mtn * ntn);
  const int rem = wg - split * mtn * ntn;
  const int nt_ = rem / mtn, mt_ = rem - nt_ * mtn;
  const int m0 = mt_ * BM, n0 = nt_ * BN;
  // splits cut the K-tile sequence (strip order: whole K-tiles of 64 pixels; raster: pixels)
  const int chunk = ((P + a.splits - 1) / a.splits + PK - 1) / PK * PK;
  const int p_begin = split * chunk;
  const int p_end = (p_begin + chunk < P) ? p_begin + chunk : P;
  const int nk = p_end > p_begin ? (p_end - p_begin + PK - 1) / PK : 0;
  const int nstrips = a.Wo / PK;

  // dy source of this tile's rows (WgradArgs::dy2: rows >= Co1 from the second source)
  const bool sec = a.dy2 && m0 >= a.Co1;   // wave-uniform
  const int lddy = sec ? a.lddy2 : a.lddy;
  const int co_b = sec ? a.Co1 : 0;
  const int co_e = a.dy2 && !sec ? a.Co1 : a.Co;
  const auto rs_dy = __builtin_amdgcn_make_buffer_rsrc((void*)(sec ? a.dy2 : a.dy), (short)0,
                                                       (int)((long)P * lddy * 2), 0x00020000);
  const auto rs_x = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0,
                                                      (int)((long)a.N * a.H * a.W * a.ldx * 2), 0x00020000);

  // DMA rows: instruction i -> pixel row r_i = (i*8 + wave)*4 + lane/16, physical chunk lane&15
  const int pc = lane & 15;
  int r_[2];
  uint32_t a_voff[4];          // j = half*2 + i: dy byte offset of (row r_i, co) (OOB: co >= Co)
  int b_dh[4], b_dw[4], b_toff[4];
#pragma unroll
  for (int i = 0; i < 2; ++i) r_[i] = (i * 8 + wave) * 4 + (lane >> 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = j & 1, h = j >> 1;
    const int lc = wpp_swz(r_[i], pc);
    const int co = m0 + h * 128 + lc * 8;
    a_voff[j] = co < co_e ? (uint32_t)((r_[i] * lddy + co - co_b) * 2) : OOB;
    const int col = n0 + h * 128 + lc * 8;
    const bool okc = col < Ncol;
    const int cc = okc ? col : 0;
    const int tap = cc / a.C, ci = cc - tap * a.C;
    const int kh = tap / a.KW, kw = tap - kh * a.KW;
    b_dh[j] = okc ? kh * a.dil - a.pad_h : -(1 << 28);
    b_dw[j] = kw * a.dil - a.pad_w;
    b_toff[j] = (b_dh[j] * a.W + b_dw[j]) * a.ldx + ci;
  }

  // next K-tile to issue: first pixel p0 decoded to (n, ho, wo), stepped by PK pixels (raster)
  // or by one row down the strip (strip order: K-tile index t = (n * nstrips + strip) * Ho + ho)
  int nx_p0 = p_begin, nx_n, nx_ho, nx_wo;
  if constexpr (FAST == 2) {
    const int t = p_begin / PK;
    nx_ho = t % a.Ho;
    const int u = t / a.Ho;
    nx_wo = (u % nstrips) * PK;
    nx_n = u / nstrips;
    nx_p0 = (nx_n * a.Ho + nx_ho) * a.Wo + nx_wo;
  } else {
    nx_wo = p_begin % a.Wo;
    const int t = p_begin / a.Wo;
    nx_ho = t % a.Ho;
    nx_n = t / a.Ho;
  }
  // per-lane x-row decode of the K-tile being issued (shared by both x halves)
  int hb[2], wb[2], pixb[2];
  bool pv[2];
  int cur_p0 = 0, cur_prem = 0;
  int kt_left = nk;   // strip order: K-tiles left in this split (all full)
  auto decode_next = [&]() {
    cur_p0 = nx_p0;
    if constexpr (FAST == 2) {
      cur_prem = kt_left-- > 0 ? PK : 0;
    } else {
      cur_prem = p_end - nx_p0;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int n, ho, wo;
      if constexpr (FAST == 2) {
        wo = nx_wo + r_[i];
        ho = nx_ho;
        n = nx_n;
      } else if constexpr (FAST) {
        wo = nx_wo + r_[i];
        const bool c = wo >= a.Wo;
        wo = c ? wo - a.Wo : wo;
        ho = nx_ho + (c ? 1 : 0);
        const bool c2 = ho == a.Ho;
        ho = c2 ? 0 : ho;
        n = nx_n + (c2 ? 1 : 0);
      } else {
        const int p = nx_p0 + r_[i];
        wo = p % a.Wo;
        const int t = p / a.Wo;
        ho = t % a.Ho;
        n = t / a.Ho;
      }
      hb[i] = ho * a.sf;
      wb[i] = wo * a.sf;
      pixb[i] = ((n * a.H + hb[i]) * a.W + wb[i]) * a.ldx;
      pv[i] = r_[i] < cur_prem;
    }
    if constexpr (FAST == 2) {
      if (++nx_ho == a.Ho) {
        nx_ho = 0;
        nx_wo += PK;
        if (nx_wo == a.Wo) { nx_wo = 0; ++nx_n; }
      }
      nx_p0 = (nx_n * a.Ho + nx_ho) * a.Wo + nx_wo;
    } else {
      nx_p0 += PK;
      nx_wo += PK;
      while (nx_wo >= a.Wo) {
        nx_wo -= a.Wo;
        if (++nx_ho == a.Ho) { nx_ho = 0; ++nx_n; }
      }
    }
  };

  // half ids: 0 = dy co 0-127, 1 = dy co 128-255, 2 = x cols 0-127, 3 = x cols 128-255
  // (pieces i0 .. i1-1 of the half: 2 DMA instructions per wave and half)
  auto issue_half = [&](int kb, int hid, int i0 = 0, int i1 = 2) {
    char* dst = smem + (kb & 1) * WBUF + hid * WHALF;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i < i0 || i >= i1) continue;
      auto* ldst = (__attribute__((address_space(3))) void*)(dst + (i * 8 + wave) * 1024);
      if (hid < 2) {
        const int j = hid * 2 + i;
        const uint32_t off = r_[i] < cur_prem ? a_voff[j] + (uint32_t)(cur_p0 * lddy * 2) : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_dy, ldst, 16, off, 0, 0, 0);
      } else {
        const int j = (hid - 2) * 2 + i;
        const int hi = hb[i] + b_dh[j], wi = wb[i] + b_dw[j];
        const bool ok = pv[i] & ((unsigned)hi < (unsigned)a.H) & ((unsigned)wi < (unsigned)a.W);
        const uint32_t off = ok ? (uint32_t)((pixb[i] + b_toff[j]) * 2) : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_x, ldst, 16, off, 0, 0, 0);
      }
    }
  };

  f32x4_t acc[2][2][4][2];
#pragma unroll
  for (int qm = 0; qm < 2; ++qm)
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[qm][qn][i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  // transposed fragment reads (ds_read_b64_tr_b16) as inline asm: with the compiler's own
  // intrinsic hipcc waits vmcnt(0) before every read (it cannot prove that the LDS-DMA in
  // flight does not alias it), which drains the prefetch each phase. The reads are ordered
  // by the barrier protocol above; the MFMA segment waits lgkmcnt(0) before using them.
  // Fragment f of a quadrant: LDS byte address base + k-substep s * 32 rows (+8192) and the
  // second 4-row group (+1024); the per-lane base (row kr = 8*lq + q4, swizzled column
  // chunk) is loop-invariant.
  const int lq = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  const uint32_t smem_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  auto tr_base = [&](int col) -> uint32_t {
    const int kr = 8 * lq + q4;
    return (uint32_t)(kr * 256 + wpp_swz(kr, col >> 3) * 16 + (col & 7) * 2);
  };
  uint32_t a_rb[4], b_rb[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) a_rb[i] = tr_base(wm * 64 + i * 16 + 4 * p4);
#pragma unroll
  for (int j = 0; j < 2; ++j) b_rb[j] = tr_base(wn * 32 + j * 16 + 4 * p4);
  typedef short s16x8_t __attribute__((ext_vector_type(8)));
  auto frag2 = [&](uint32_t addr, V& f0, V& f1) {   // k-substeps 0 and 1
    s16x4_t l0, h0, l1, h1;
    asm volatile("ds_read_b64_tr_b16 %0, %4\n\t"
                 "ds_read_b64_tr_b16 %1, %4 offset:1024\n\t"
                 "ds_read_b64_tr_b16 %2, %4 offset:8192\n\t"
                 "ds_read_b64_tr_b16 %3, %4 offset:9216"
                 : "=&v"(l0), "=&v"(h0), "=&v"(l1), "=&v"(h1) : "v"(addr));
    const s16x8_t v0 = __builtin_shufflevector(l0, h0, 0, 1, 2, 3, 4, 5, 6, 7);
    const s16x8_t v1 = __builtin_shufflevector(l1, h1, 0, 1, 2, 3, 4, 5, 6, 7);
    __builtin_memcpy(&f0, &v0, 16);
    __builtin_memcpy(&f1, &v1, 16);
  };
  // both B quadrants stay in registers for the K-tile (phase 3 reuses B0 from phase 0: one
  // LDS read burst in three fewer per K-tile)
  V af[4][2], bfq[2][2][2];   // bfq[qn][frag][k-substep]
  auto read_a = [&](int kb, int qm) {
    const uint32_t off = smem_lds + (kb & 1) * WBUF + qm * WHALF;
#pragma unroll
    for (int i = 0; i < 4; ++i) frag2(off + a_rb[i], af[i][0], af[i][1]);
  };
  auto read_b = [&](int kb, int qn) {
    const uint32_t off = smem_lds + (kb & 1) * WBUF + (2 + qn) * WHALF;
#pragma unroll
    for (int j = 0; j < 2; ++j) frag2(off + b_rb[j], bfq[qn][j][0], bfq[qn][j][1]);
  };
  // one quadrant's 16 MFMAs with one DMA piece of (kbi, hid) issued after the first 8
  auto mfma_q_dma = [&](int qm, int qn, bool dma, int kbi, int hid, int piece) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the asm fragment reads
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (s == 1 && dma) {
        __builtin_amdgcn_sched_barrier(0);
        issue_half(kbi, hid, piece, piece + 1);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[qm][qn][i][j] = Half<E>::mma(af[i][s], bfq[qn][j][s], acc[qm][qn][i][j]);
    }
  };
  if (nk > 0) {
    // DMA in the MFMA segments: per K-tile, B0(kb+1) in L0(kb), A1(kb+1) in M0(kb) (one piece
    // per quadrant), B1(kb+2) in L1(kb), A0(kb+2) in M1(kb). The dy pieces (one VALU of
    // address math each) move out of the load segments, which were ~1.5x the MFMA segments.
    decode_next();
    issue_half(0, 0);
    issue_half(0, 3);
    issue_half(0, 2);
    issue_half(0, 1);
    if (nk > 1) {
      decode_next();
      issue_half(1, 3);
      issue_half(1, 0);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // A0, B1, B0 of K-tile 0 landed
    } else {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    }
    pp_barrier();
    if (wm == 1) pp_barrier();
    if (wm == 1) __builtin_amdgcn_s_setprio(1);
    for (int kb = 0; kb < nk; ++kb) {
      const bool m1 = kb + 1 < nk, m2 = kb + 2 < nk;
      WG_TS(kb, 0);
      read_a(kb, 0);
      read_b(kb, 0);
      read_b(kb, 1);
      if (m1) issue_half(kb + 1, 2);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      // A1(kb) (issued in M0(kb-1)) landed: younger are B1(kb+1), A0(kb+1), B0(kb+1) (+A1(kb+1))
      if (wm == 1) {
        if (m1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      WG_TS(kb, 1);
      pp_barrier();
      WG_TS(kb, 2);
      mfma_q_dma(0, 0, m1, kb + 1, 1, 0);
      mfma_q_dma(0, 1, m1, kb + 1, 1, 1);
      WG_TS(kb, 3);
      if (wm == 0) {
        if (m1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      pp_barrier();
      WG_TS(kb, 4);
      read_a(kb, 1);
      if (m2) {
        decode_next();
        issue_half(kb + 2, 3);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      // A0, B0, B1 of kb+1 landed: younger than B0(kb+1) are A1(kb+1), B1(kb+2) (+A0(kb+2))
      if (wm == 1 && m1) {
        if (m2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      }
      WG_TS(kb, 5);
      pp_barrier();
      WG_TS(kb, 6);
      mfma_q_dma(1, 1, m2, kb + 2, 0, 0);
      mfma_q_dma(1, 0, m2, kb + 2, 0, 1);
      WG_TS(kb, 7);
      if (wm == 0 && m1) {
        if (m2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      }
      pp_barrier();
    }
    if (wm == 0) pp_barrier();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }

  float* O = a.out + (size_t)split * a.Co * Ncol;
  const int lr = lane & 15;
  if (m0 + BM <= a.Co && n0 + BN <= Ncol && (long)a.Co * Ncol * 4 < (1L << 31)) {
    // whole tile: buffer stores with the row offset in an SGPR (one per (qm, i, r), shared by
    // the qn / j stores) and the column in the immediate; the checked form below spent ~9
    // instructions per value (bounds compare, exec mask, 64-bit multiply-add) on 128 values
    // per lane, 10 % of a 32-K-tile 1x1 launch
    const auto rs_o = __builtin_amdgcn_make_buffer_rsrc((void*)O, (short)0, (int)((long)a.Co * Ncol * 4), 0x00020000);
    const uint32_t vb = (uint32_t)(((m0 + wm * 64 + lq * 4) * Ncol + n0 + wn * 32 + lr) * 4);
#pragma unroll
    for (int qm = 0; qm < 2; ++qm)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int so = __builtin_amdgcn_readfirstlane((qm * 128 + i * 16 + r) * Ncol * 4);
#pragma unroll
          for (int qn = 0; qn < 2; ++qn)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[qm][qn][i][j][r]), rs_o,
                                                    vb + (qn * 128 + j * 16) * 4, so, 0);
        }
    return;
  }
#pragma unroll
  for (int qm = 0; qm < 2; ++qm)
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int n = n0 + qn * 128 + wn * 32 + j * 16 + lr;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = m0 + qm * 128 + wm * 64 + i * 16 + lq * 4 + r;
            if (m < a.Co && n < Ncol) O[(size_t)m * Ncol + n] = acc[qm][qn][i][j][r];
          }
        }
}

template <typename E, int FAST>
__global__ __launch_bounds__(PP_THREADS, 1) void conv_wgrad_pp_kernel(WgradArgs a) {
  conv_wgrad_pp_body<E, FAST>(a);
}

}  // namespace

// 256 x 256 wgrad tiles with operands < 2^31 bytes (32-bit buffer offsets)
bool conv_wgrad_pp_ok(const WgradArgs& a) {
  const long P = (long)a.N * a.Ho * a.Wo;
  return (a.C % 8) == 0 && (a.ldx % 8) == 0 && (a.Co % 8) == 0 && (a.lddy % 8) == 0 &&
         P * a.lddy * 2 < (1L << 31) && (long)a.N * a.H * a.W * a.ldx * 2 < (1L << 31) &&
         (!a.dy2 || (a.Co1 % 256 == 0 && a.Co1 < a.Co && a.lddy2 % 8 == 0 && P * a.lddy2 * 2 < (1L << 31)));
}

hipError_t launch_conv_wgrad_pp(int dtype, const WgradArgs& a, hipStream_t s) {
  const int Ncol = a.KH * a.KW * a.C;
  const int nwg = ceil_div(a.Co, 256) * ceil_div(Ncol, 256) * a.splits;
  auto launch = [&](auto kern) -> hipError_t {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, WPP_LDS);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(PP_THREADS), WPP_LDS, s, a);
    return hipGetLastError();
  };
  // strip order where the rows split into whole 64-pixel K-tiles and the pixel rows repeat
  // across taps (KH > 1); 1x1 layers read every x row once, raster order is as good there
  const bool strip = (a.Wo % 64) == 0 && a.KH > 1;
  if (dtype == SEG_F16) {
    if (strip) return launch(conv_wgrad_pp_kernel<f16_t, 2>);
    if (a.Wo >= 64) return launch(conv_wgrad_pp_kernel<f16_t, 1>);
    return launch(conv_wgrad_pp_kernel<f16_t, 0>);
  }
  if (strip) return launch(conv_wgrad_pp_kernel<bf16_t, 2>);
  if (a.Wo >= 64) return launch(conv_wgrad_pp_kernel<bf16_t, 1>);
  return launch(conv_wgrad_pp_kernel<bf16_t, 0>);
}

#ifdef NT_DBG_TIMING
extern "C" int seg_dbg_nt_timing(void* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_nt_dbg), sizeof(g_nt_dbg)) == hipSuccess ? 0 : -1;
}
#endif

#ifdef WG_DBG_TIMING
extern "C" int seg_dbg_wg_timing(void* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wg_dbg), sizeof(g_wg_dbg)) == hipSuccess ? 0 : -1;
}
#endif

#ifdef PP_DBG_TIMING
extern "C" int seg_dbg_pp_timing(void* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pp_dbg), sizeof(g_pp_dbg)) == hipSuccess ? 0 : -1;
}
#endif
