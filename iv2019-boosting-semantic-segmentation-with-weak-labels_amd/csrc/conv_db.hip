// 16-bit dense 1x1 implicit GEMM (forward / data gradient) for SHORT reductions, with
// double-buffered accumulators: the epilogue of one tile runs inside the next tile's main loop.
//
// Why: on the short-K 1x1 layers (K = 64..512: every unit's conv3 forward, the conv1 data
// gradients) the 256 x 256 ping-pong kernel (conv_pp.hip) spends a third of each tile in its
// epilogue (BN statistics, LDS staging, a synchronised 128 KB store burst per CU) with the matrix
// cores idle, and its 256 x 256 tile uses every register of both waves on a SIMD, so nothing
// can overlap that epilogue (DESIGN.md §5b', §5b'''').
//
// Design (one 512-thread workgroup per CU, persistent over tiles):
//  * 256 (M) x 128 (N) tiles; 8 waves as 4 (M) x 2 (N), 64 x 64 per wave = 4 x 4 fragments of
//    v_mfma_f32_16x16x32 (64 accumulator registers); TWO accumulator sets: tile t accumulates in
//    set t & 1 while set (t - 1) & 1 still holds the previous tile;
//  * the K-tiles of all of a workgroup's tiles form one stream (item g = tile g / nk, K-tile
//    g % nk); three 48 KB LDS buffers (A 256 x 64 + B 128 x 64 16-bit, 128-B rows, 16-B chunks
//    XOR-swizzled by row); item g + 2 is fetched by LDS-DMA (buffer resources, 6 x 1 KB per wave)
//    while item g is computed, across tile boundaries;
//  * every item is a LOAD segment (16 ds_read_b128 fragments, the DMA of item g + 2, the
//    previous tile's epilogue work) and an MFMA segment (32 MFMAs), separated by barriers; the
//    two wave groups (waves 0-3 / 4-7: one of each on every SIMD) are staggered by one barrier
//    so one wave per SIMD is always in its MFMA segment;
//  * epilogue of tile t - 1 during tile t: BN statistics (exact two-pass over the wave's 64 rows,
//    DPP butterflies, one 8-byte (sum, M2) store per lane) and the outputs stored straight from
//    the accumulators: the B rows are permuted at DMA time so a lane holds 8 consecutive output
//    channels per store (4 lanes = 64 contiguous bytes of a pixel, the two stores of a pixel
//    fill its 128-B line), no LDS staging; the 8 stores per lane are spread over the tile's
//    K-tiles;
//  * vmcnt: loads and stores retire in issue order on one counter, so each wait for an item's
//    DMA counts the stores issued after it (wave-uniform count, vm_wait below) instead of
//    draining them: the stores stay in flight for about one K-tile.
// Preconditions (conv_nt_db_ok): dense 1x1 stride-1 geometry, M % 256 == 0, Co % 128 == 0,
// C % 64 == 0 with 64 <= C <= DB_MAX_K, no residual / second GEMM / consumer mask.
#include "conv.h"
#include <cstdlib>

#ifdef DB_DBG_TIMING
// A/B only: per-wave segment stamps (s_memtime) of stream items 16-23, blocks 0-7, 10 stamps
// per item: load-segment start, after the epilogue work, after the DMA issue, after the fragment
// reads (lgkmcnt 0), after group 1's vmcnt wait, after barrier A, after the MFMAs, after group
// 0's vmcnt wait, after barrier B
__device__ unsigned long long g_db_dbg[8 * 8 * 8 * 10];
#define DB_TS(it, k)                                                                             \
  if ((threadIdx.x & 63) == 0 && blockIdx.x < 8 && (it) >= 16 && (it) < 24)                     \
    g_db_dbg[((blockIdx.x * 8 + (threadIdx.x >> 6)) * 8 + ((it) - 16)) * 10 + (k)] =             \
        __builtin_amdgcn_s_memtime()
#else
#define DB_TS(it, k)
#endif

namespace {

constexpr int DB_THREADS = 512;
constexpr int DB_BM = 256, DB_BN = 128, DB_BK = 64;
constexpr int DB_ABYTES = DB_BM * 128;           // 32 KB: 256 rows x 64 16-bit K-elements
constexpr int DB_BBYTES = DB_BN * 128;           // 16 KB
constexpr int DB_BUF = DB_ABYTES + DB_BBYTES;    // 48 KB per K-tile
constexpr int DB_NBUF = 3;
constexpr int DB_LDS = DB_NBUF * DB_BUF;         // 144 KB
constexpr int DB_MAX_K = 1024;

__device__ __forceinline__ int swz(int row, int ch) { return ch ^ ((row >> 1) & 7); }

__device__ __forceinline__ void db_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform n (a larger n would be a weaker wait: callers pass the
// exact count of VMEM operations issued after the ones they need, capped at 30 = stronger)
__device__ __forceinline__ void vm_wait(int n) {
#define DB_VMW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
  switch (n < 30 ? n : 30) {
    DB_VMW(0) DB_VMW(1) DB_VMW(2) DB_VMW(3) DB_VMW(4) DB_VMW(5) DB_VMW(6) DB_VMW(7) DB_VMW(8)
    DB_VMW(9) DB_VMW(10) DB_VMW(11) DB_VMW(12) DB_VMW(13) DB_VMW(14) DB_VMW(15) DB_VMW(16)
    DB_VMW(17) DB_VMW(18) DB_VMW(19) DB_VMW(20) DB_VMW(21) DB_VMW(22) DB_VMW(23) DB_VMW(24)
    DB_VMW(25) DB_VMW(26) DB_VMW(27) DB_VMW(28) DB_VMW(29)
    default: asm volatile("s_waitcnt vmcnt(30)" ::: "memory"); break;
  }
#undef DB_VMW
}

// v[r] summed over the 16 lanes of a DPP row (quad_perm xor 1, xor 2, half-row mirror, row
// mirror): every lane of the row ends with the totals
#define DB_ROW_SUM8(CTRL)                                                           \
  "v_add_f32_dpp %0, %0, %0 " CTRL " row_mask:0xf bank_mask:0xf\n"                   \
  "v_add_f32_dpp %1, %1, %1 " CTRL " row_mask:0xf bank_mask:0xf\n"                   \
  "v_add_f32_dpp %2, %2, %2 " CTRL " row_mask:0xf bank_mask:0xf\n"                   \
  "v_add_f32_dpp %3, %3, %3 " CTRL " row_mask:0xf bank_mask:0xf\n"                   \
  "v_add_f32_dpp %4, %4, %4 " CTRL " row_mask:0xf bank_mask:0xf\n"                   \
  "v_add_f32_dpp %5, %5, %5 " CTRL " row_mask:0xf bank_mask:0xf\n"                   \
  "v_add_f32_dpp %6, %6, %6 " CTRL " row_mask:0xf bank_mask:0xf\n"                   \
  "v_add_f32_dpp %7, %7, %7 " CTRL " row_mask:0xf bank_mask:0xf\n"
__device__ __forceinline__ void row_total8(float* v) {
  asm volatile("s_nop 1\n" DB_ROW_SUM8("quad_perm:[1,0,3,2]") DB_ROW_SUM8("quad_perm:[2,3,0,1]")
               DB_ROW_SUM8("row_half_mirror") DB_ROW_SUM8("row_mirror") "s_nop 1"
               : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
                 "+v"(v[7]));
}

// v[idx] for a lane-varying idx in 0..15 without indexed register access: a 4-level select tree
// on bit masks (a ?: tree on floats is turned into a private-memory array index by LLVM)
__device__ __forceinline__ uint32_t sel16(const float* v, int idx) {
  uint32_t l[8];
  const uint32_t m0 = 0u - (uint32_t)(idx & 1), m1 = 0u - (uint32_t)((idx >> 1) & 1),
                 m2 = 0u - (uint32_t)((idx >> 2) & 1), m3 = 0u - (uint32_t)((idx >> 3) & 1);
#pragma unroll
  for (int k = 0; k < 8; ++k)
    l[k] = (__float_as_uint(v[2 * k]) & ~m0) | (__float_as_uint(v[2 * k + 1]) & m0);
#pragma unroll
  for (int k = 0; k < 4; ++k) l[k] = (l[2 * k] & ~m1) | (l[2 * k + 1] & m1);
#pragma unroll
  for (int k = 0; k < 2; ++k) l[k] = (l[2 * k] & ~m2) | (l[2 * k + 1] & m2);
  return (l[0] & ~m3) | (l[1] & m3);
}

template <typename E>
__global__ __launch_bounds__(DB_THREADS, 1) void conv_nt_db_kernel(ConvArgs a) {
  typedef typename Half<E>::V V;
  typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;    // 4 x 2 waves, 64 x 64 each
  const int grp = wave >> 2;                  // stagger group: one wave of each on every SIMD
  const int lr = lane & 15, lq = lane >> 4;
  const int pc = lane & 7;
  const int M = a.N * a.Ho * a.Wo;            // < 2^31 (host check), a multiple of 256
  const int mtiles = M / DB_BM;
  const int ntiles = a.Co / DB_BN;
  const int nwg = mtiles * ntiles;
  const int nk = a.C / DB_BK;
  // XCD-aware bijective remap (as conv_pp.hip): tile t runs on XCD t % 8; each XCD takes a
  // contiguous run of tiles, n fastest, so workgroups sharing an A panel share an L2
  auto tile_of = [&](int t, int& mt_, int& nt_) {
    const int xcd = t & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (t >> 3);
    mt_ = wg / ntiles;
    nt_ = wg - mt_ * ntiles;
  };
  const int G = gridDim.x;

  const auto rs_x = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, (int)((long)M * a.ldx * 2), 0x00020000);
  const auto rs_w = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, (int)((long)a.Co * a.ldw * 2), 0x00020000);

  // ---- issue cursor: the item whose DMA goes out next (two items ahead of the compute) ----
  int is_tile = blockIdx.x, is_kb = 0;
  // one VGPR per operand: piece i of a wave is 64 rows (A) / 64 channels (B) further on, a
  // wave-uniform step passed as the buffer instruction's scalar offset (the row swizzle and the
  // B-row permutation do not change with i)
  uint32_t a_off, b_off;
  const int a_step = 64 * a.ldx * 2, b_step = 64 * a.ldw * 2;
  auto issue_setup = [&](int t) {
    int mt_, nt_;
    tile_of(t, mt_, nt_);
    const int row = wave * 8 + (lane >> 3);                      // A LDS row of piece 0
    a_off = (uint32_t)(((mt_ * DB_BM + row) * a.ldx + swz(row, pc) * 8) * 2);
    const int qr = wave * 8 + (lane >> 3);                       // B LDS row of piece 0 (< 64)
    const int j = (qr >> 4) & 3, q = qr & 15;
    // fragment j, position q -> channel (j/2)*32 + (q/4)*8 + (j%2)*4 + q%4: a lane's four
    // fragments then hold 2 runs of 8 consecutive channels (see the store below)
    const int co = nt_ * DB_BN + (j >> 1) * 32 + (q >> 2) * 8 + (j & 1) * 4 + (q & 3);
    b_off = (uint32_t)((co * a.ldw + swz(qr, pc) * 8) * 2);
  };
  int issued = 0;   // stream items issued so far (item g -> LDS buffer g % 3)
  // DMA of the next stream item (6 pieces per wave); returns the pieces issued (0 at the end)
  auto issue_next = [&]() -> int {
    if (is_tile >= nwg) return 0;
    char* buf = smem + (issued % DB_NBUF) * DB_BUF;
    const int k2 = is_kb * DB_BK * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs_x, (__attribute__((address_space(3))) void*)(buf + (wave + 8 * i) * 1024), 16,
          a_off, k2 + i * a_step, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs_w, (__attribute__((address_space(3))) void*)(buf + DB_ABYTES + (wave + 8 * i) * 1024), 16,
          b_off, k2 + i * b_step, 0, 0);
    ++issued;
    if (++is_kb == nk) {
      is_kb = 0;
      is_tile += G;
      if (is_tile < nwg) issue_setup(is_tile);
    }
    return 6;
  };

  f32x4_t acc[2][4][4];
  V af[4][2], bf[4][2];
  float sm[16], m2[16];   // BN statistics of the previous tile: [j * 4 + r]

  // ---- epilogue pieces of a finished tile held in acc[P] ----
  E* const Y = (E*)a.y;
  auto store_out = [&](auto PC, auto IC, auto HC, int m0_, int n0_) {
    constexpr int P = decltype(PC)::value;
    constexpr int i = decltype(IC)::value, h = decltype(HC)::value;
    const int m = m0_ + wm * 64 + i * 16 + lr;
    const int n = n0_ + wn * 64 + h * 32 + lq * 8;
    u32x4_t v;
    v[0] = pack2<E>(acc[P][i][2 * h][0], acc[P][i][2 * h][1]);
    v[1] = pack2<E>(acc[P][i][2 * h][2], acc[P][i][2 * h][3]);
    v[2] = pack2<E>(acc[P][i][2 * h + 1][0], acc[P][i][2 * h + 1][1]);
    v[3] = pack2<E>(acc[P][i][2 * h + 1][2], acc[P][i][2 * h + 1][3]);
    __builtin_nontemporal_store(v, (u32x4_t*)(Y + (size_t)m * a.ldy + n));
  };
  auto store_all = [&](auto PC, int m0_, int n0_) {
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    store_out(PC, I0(), I0(), m0_, n0_); store_out(PC, I0(), I1(), m0_, n0_);
    store_out(PC, I1(), I0(), m0_, n0_); store_out(PC, I1(), I1(), m0_, n0_);
    store_out(PC, I2(), I0(), m0_, n0_); store_out(PC, I2(), I1(), m0_, n0_);
    store_out(PC, I3(), I0(), m0_, n0_); store_out(PC, I3(), I1(), m0_, n0_);
  };
  // BN partial statistics over the wave's 64 rows, exact two-pass: sums (pass 1), then squared
  // deviations from those means (pass 2) + the (sum, M2) store: lane lr writes channel lr of its
  // row group's 16 (one 8-byte store per lane, all lanes active)
  auto stats1 = [&](auto PC) {
    constexpr int P = decltype(PC)::value;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        sm[j * 4 + r] = (acc[P][0][j][r] + acc[P][1][j][r]) + (acc[P][2][j][r] + acc[P][3][j][r]);
    row_total8(sm);
    row_total8(sm + 8);
  };
  auto stats2 = [&](auto PC, int mt_, int n0_) {
    constexpr int P = decltype(PC)::value;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float mu = sm[j * 4 + r] * (1.f / 64.f);
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float d = acc[P][i][j][r] - mu;
          q += d * d;
        }
        m2[j * 4 + r] = q;
      }
    row_total8(m2);
    row_total8(m2 + 8);
    // lane lr: index lr = j*4 + r -> channel (lr/8)*32 + lq*8 + lr%8
    const int n = n0_ + wn * 64 + (lr >> 3) * 32 + lq * 8 + (lr & 7);
    float* dst = a.stats + 2 * ((size_t)(mt_ * 4 + wm) * a.Co + n);
    u32x2_t v;
    v[0] = sel16(sm, lr);
    v[1] = sel16(m2, lr);
    *(u32x2_t*)dst = v;
  };
  const bool stats = a.stats != nullptr;   // wave-uniform

  auto read_frags = [&](const char* buf) {
    const char* A = buf;
    const char* B = buf + DB_ABYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + i * 16 + lr;
#pragma unroll
      for (int s = 0; s < 2; ++s) af[i][s] = *(const V*)(A + row * 128 + swz(row, lq + 4 * s) * 16);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = wn * 64 + j * 16 + lr;
#pragma unroll
      for (int s = 0; s < 2; ++s) bf[j][s] = *(const V*)(B + row * 128 + swz(row, lq + 4 * s) * 16);
    }
  };
  auto mfma_all = [&](auto PC) {
    constexpr int P = decltype(PC)::value;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          // transposed accumulators: lane (lq, lr) = pixel lr, 4 channels of fragment row lq*4
          acc[P][i][j] = Half<E>::mma(bf[j][s], af[i][s], acc[P][i][j]);
  };

  // ---- prologue: items 0 and 1 ----
  issue_setup(is_tile);
  int p0 = issue_next();
  int p1 = issue_next();
  (void)p0;
  vm_wait(p1);               // item 0 landed (item 1 in flight)
  db_barrier();
  if (grp == 1) db_barrier();   // stagger: group 1 runs one segment behind
  if (grp == 1) __builtin_amdgcn_s_setprio(1);

  int g = 0;                 // compute cursor: stream item
  int tile = blockIdx.x;
  int mt, nt;
  tile_of(tile, mt, nt);
  int pmt = 0, pnt = 0;      // the previous tile (its epilogue runs during this one)
  bool has_prev = false;

  // one tile: accumulate into acc[P]; the previous tile's epilogue (acc[1 - P]) in the load
  // segments: statistics at K-tiles 0 / 1 (0 when nk == 1), the 8 stores (i, h) spread as
  // store q at K-tile q * nk / 8
  auto run_tile = [&](auto PC) {
    constexpr int P = decltype(PC)::value;
    constexpr int Q = 1 - P;
    std::integral_constant<int, Q> QC;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[P][i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    const int pm0 = pmt * DB_BM, pn0 = pnt * DB_BN;
    for (int kb = 0; kb < nk; ++kb, ++g) {
      const char* buf = smem + (g % DB_NBUF) * DB_BUF;
      // ---- load segment: the previous tile's epilogue work first (its temporaries are dead
      // before the fragments go live), then the DMA of item g + 2, then this item's fragments
      DB_TS(g, 0);
      int s = 0;
#ifndef DB_NOSTORE
      if (has_prev) {
        if (stats && kb == 0) {
          stats1(QC);
          stats2(QC, pmt, pn0);
          ++s;
        }
        // store q = (i, h) = (q / 2, q % 2) at K-tile q * nk / 8 (explicit constants: a
        // runtime fragment index would put the accumulators in scratch)
#define DB_STQ(q)                                                                          \
        if ((((q) * nk) >> 3) == kb) {                                                     \
          store_out(QC, std::integral_constant<int, (q) / 2>(), std::integral_constant<int, (q) % 2>(), pm0, pn0); \
          ++s;                                                                             \
        }
        DB_STQ(0) DB_STQ(1) DB_STQ(2) DB_STQ(3) DB_STQ(4) DB_STQ(5) DB_STQ(6) DB_STQ(7)
#undef DB_STQ
      }
#endif
      DB_TS(g, 1);
      const int p = issue_next();   // item g + 2
      DB_TS(g, 2);
      read_frags(buf);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      DB_TS(g, 3);
      const bool more = g + 1 < issued;   // item g + 1 exists (its DMA is out)
      // item g + 1's DMA went out at the end of the previous load segment's VMEM work: after it
      // come this segment's stores and DMA
      const int nwait = s + p;
      if (grp == 1 && more) vm_wait(nwait);
      DB_TS(g, 4);
      db_barrier();
      DB_TS(g, 5);
      // ---- MFMA segment ----
      mfma_all(PC);
      DB_TS(g, 6);
      if (grp == 0 && more) vm_wait(nwait);
      DB_TS(g, 7);
      db_barrier();
      DB_TS(g, 8);
    }
  };

  for (;;) {
    run_tile(std::integral_constant<int, 0>());
    has_prev = true; pmt = mt; pnt = nt;
    tile += G;
    if (tile >= nwg) {
      // last tile's epilogue (acc[0]), not overlapped
      if (stats) { stats1(std::integral_constant<int, 0>()); stats2(std::integral_constant<int, 0>(), pmt, pnt * DB_BN); }
      store_all(std::integral_constant<int, 0>(), pmt * DB_BM, pnt * DB_BN);
      break;
    }
    tile_of(tile, mt, nt);
    run_tile(std::integral_constant<int, 1>());
    pmt = mt; pnt = nt;
    tile += G;
    if (tile >= nwg) {
      if (stats) { stats1(std::integral_constant<int, 1>()); stats2(std::integral_constant<int, 1>(), pmt, pnt * DB_BN); }
      store_all(std::integral_constant<int, 1>(), pmt * DB_BM, pnt * DB_BN);
      break;
    }
    tile_of(tile, mt, nt);
  }
  __builtin_amdgcn_s_setprio(0);
}

int db_grid(int nwg) {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
    ncu = (ncu + 7) / 8 * 8;
  }
  return nwg < ncu ? nwg : ncu;
}

template <typename E>
hipError_t db_launch(const ConvArgs& a, hipStream_t s) {
  auto kern = conv_nt_db_kernel<E>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, DB_LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const long M = (long)a.N * a.Ho * a.Wo;
  const int nwg = (int)(M / DB_BM) * (a.Co / DB_BN);
  hipLaunchKernelGGL(kern, dim3(db_grid(nwg)), dim3(DB_THREADS), DB_LDS, s, a);
  return hipGetLastError();
}

}  // namespace

// Off by default (measured slower than the 256 x 256 ping-pong kernel on every short-K layer,
// DESIGN.md §5d); SEG_NT_DB=1 turns it on for A/B, SEG_NT_DB_MAXK sets the longest reduction
// it takes (default 512)
static int db_max_k() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("SEG_NT_DB");
    const char* k = getenv("SEG_NT_DB_MAXK");
    v = !(e && e[0] == '1') ? 0 : (k ? atoi(k) : 512);
    if (v > DB_MAX_K) v = DB_MAX_K;
  }
  return v;
}

bool conv_nt_db_ok(const ConvArgs& a) {
  const long M = (long)a.N * a.Ho * a.Wo;
  return !a.tap8 && a.KH == 1 && a.KW == 1 && a.st == 1 && a.sf == 1 && a.pad_h == 0 &&
         a.pad_w == 0 && a.H == a.Ho && a.W == a.Wo && !a.x2 && !a.r && !a.r2 && !a.omask &&
         M % DB_BM == 0 && a.Co % DB_BN == 0 && a.C % DB_BK == 0 && a.C >= DB_BK &&
         a.C <= db_max_k() && a.ldx % 8 == 0 && a.ldw % 8 == 0 && a.ldy % 8 == 0 &&
         M * a.ldx * 2 < (1L << 31) && (long)a.Co * a.ldw * 2 < (1L << 31) && M < (1L << 31);
}

hipError_t launch_conv_nt_db(int dtype, const ConvArgs& a, hipStream_t s) {
  if (!conv_nt_db_ok(a)) return hipErrorInvalidValue;
  if (dtype == SEG_F16) return db_launch<f16_t>(a, s);
  return db_launch<bf16_t>(a, s);
}

#ifdef DB_DBG_TIMING
extern "C" int seg_dbg_db_timing(void* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_db_dbg), sizeof(g_db_dbg)) == hipSuccess ? 0 : -1;
}
#endif
