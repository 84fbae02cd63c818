// 16-bit weight gradient of the small-channel 3 x 3 stride-1 convolutions (block1 / block2
// conv2 at C2: 64 and 128 channels, 256 x 512 and 128 x 256 pixels) on input patches.
//
//   dw[co][kh][kw][ci] = sum_p dy[p][co] * x[p + ((kh - 1) d, (kw - 1) d)][ci]
//
// The implicit-GEMM weight gradient (conv_wgrad_v2_kernel) gathers the shifted input once per
// tap column block: for these layers (K = 9 x 64 columns in 256-wide tiles) every input pixel
// is fetched 12 times and every dy pixel 3 times, and the kernel runs at ~0.15 of its attainable
// rate. Here a workgroup owns a 64 (co) x 9 x 64 (ci) output block, so one K-step (a strip of 64
// output pixels of one row) needs the dy strip (64 px x 64 co) and ONE input patch (3 rows x
// (64 + 2d) px x 64 ci): the nine taps are the patch read at nine row offsets.
//
//  * LDS image: 128-B rows (one pixel's 64 channels), the 16-B chunk c of row r stored at chunk
//    c ^ s(r), s(r) = 2 * (bit1(r) | bit3(r) << 1): a ds_read_b64_tr_b16 half-wave reads rows
//    {b..b+3, b+8..b+11} for ANY base b (the taps shift the base by kh (64+2d) + kw d), and those
//    eight rows' 32-B segments land on 16 distinct 16-B bank slots (conflict-free).
//  * operands by LDS-DMA (buffer_load ... lds, 16 B per lane, source chunk pre-swizzled; padding
//    pixels get an out-of-range offset -> zeros), a 3-stage ring of 40 KB stages (25 patch
//    pieces + 8 dy pieces + 7 pad pieces: five per wave), one barrier per K-step, counted vmcnt.
//  * 8 waves = 2 (32 co) x 4 (16 ci); per 32-pixel sub-step a wave reads 2 A fragments (dy^T)
//    and 9 B fragments (one per tap) by transposed reads and issues 18 16x16x32 MFMAs; the next
//    sub-step's fragments are read while the current MFMAs run.
//  * split-K over pixel strips into fp32 slabs [split][Co][9 C] (reduced by splitk_reduce, the
//    layout of the other weight-gradient kernels).
#include "conv.h"

namespace {

constexpr int WP_THREADS = 512;
constexpr int WP_PIECES = 40;                 // DMA pieces per stage (1 KB each)
constexpr int WP_STAGE = WP_PIECES * 1024;    // bytes per stage
constexpr int WP_STAGES = 3;
constexpr int WP_LDS = WP_STAGES * WP_STAGE;  // 120 KB
constexpr int WP_MAXPW = 64 + 2 * 4;          // patch width bound (dilation <= 4)
constexpr int WP_PATCH_PIECES = (3 * WP_MAXPW + 7) / 8;   // 27 at d = 4; 25 at d = 1
constexpr int WP_DY_PIECE0 = 32;              // dy strip pieces 32..39 (rows 256..319)

__device__ __forceinline__ int wp_swz(int r) { return 2 * (((r >> 1) & 1) | ((r >> 2) & 2)); }

template <typename E>
__global__ __launch_bounds__(WP_THREADS, 1) void conv_wgrad_patch_kernel(WgradArgs a) {
  typedef typename Half<E>::V V;
  constexpr uint32_t OOB = 0x80000000u;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wco = wave & 1, wci = wave >> 1;
  const int d = a.dil, PW = 64 + 2 * d;
  const int cob = a.Co / 64, cib = a.C / 64;
  const int blocks = cob * cib;
  const int split = blockIdx.x / blocks, blk = blockIdx.x - split * blocks;
  const int co0 = (blk % cob) * 64, ci0 = (blk / cob) * 64;
  const int nstrip_row = a.Wo / 64;
  const long T = (long)a.N * a.Ho * nstrip_row;
  const long t_begin = T * split / a.splits, t_end = T * (split + 1) / a.splits;

  const auto rs_x = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0,
                                                      (int)((long)a.N * a.H * a.W * a.ldx * 2), 0x00020000);
  const auto rs_dy = __builtin_amdgcn_make_buffer_rsrc((void*)a.dy, (short)0,
                                                       (int)((long)a.N * a.Ho * a.Wo * a.lddy * 2), 0x00020000);

  // this lane's DMA rows: piece j = wave + 8 i (i = 0..4), LDS row 8 j + lane / 8, chunk lane % 8
  // (stage-relative); patch rows decode to (kh, u) once, dy rows to the strip pixel p
  int pk_kh[5], pk_u[5], pk_off[5];
  bool pk_live[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int j = wave + 8 * i;
    const int row = 8 * j + (lane >> 3);
    const int chunk = (lane & 7) ^ wp_swz(row);
    pk_live[i] = false;
    pk_kh[i] = 0;
    pk_u[i] = 0;
    pk_off[i] = 0;
    if (j < WP_PATCH_PIECES) {
      pk_live[i] = row < 3 * PW;
      pk_kh[i] = row / PW;
      pk_u[i] = row - pk_kh[i] * PW;
      pk_off[i] = (ci0 + chunk * 8) * 2;
    } else if (j >= WP_DY_PIECE0) {
      pk_live[i] = true;
      pk_u[i] = row - 8 * WP_DY_PIECE0;   // strip pixel
      pk_off[i] = (co0 + chunk * 8) * 2;
    }
  }
  auto issue = [&](long t, int stg) {
    const int wb = (int)(t % nstrip_row);
    const long t2 = t / nstrip_row;
    const int ho = (int)(t2 % a.Ho), n = (int)(t2 / a.Ho);
    const int wo0 = wb * 64;
    char* sbase = smem + stg * WP_STAGE;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int j = wave + 8 * i;
      auto* ldst = (__attribute__((address_space(3))) void*)(sbase + j * 1024);
      if (j < WP_PATCH_PIECES || j >= WP_DY_PIECE0) {
        if (j >= WP_DY_PIECE0) {
          const uint32_t off = (uint32_t)(((long)(n * a.Ho + ho) * a.Wo + wo0 + pk_u[i]) * a.lddy * 2) + pk_off[i];
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_dy, ldst, 16, off, 0, 0, 0);
        } else {
          const int hi = ho + (pk_kh[i] - 1) * d, wi = wo0 - d + pk_u[i];
          const bool ok = pk_live[i] & ((unsigned)hi < (unsigned)a.H) & ((unsigned)wi < (unsigned)a.W);
          const uint32_t off = ok ? (uint32_t)(((long)(n * a.H + hi) * a.W + wi) * a.ldx * 2) + pk_off[i] : OOB;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_x, ldst, 16, off, 0, 0, 0);
        }
      } else {   // pad piece: keeps five pieces per wave per stage (one vmcnt for every wave)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_dy, ldst, 16, OOB, 0, 0, 0);
      }
    }
  };

  // transposed-read byte offsets (stage-relative, sub-step 0; sub-step 1 = +32 rows = +4096 B,
  // which keeps the swizzle since 32 = 0 mod 16): A = dy rows, B = patch rows of each tap
  const int lq = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  auto tr_off = [&](int row, int col) -> uint32_t {
    return (uint32_t)(row * 128 + ((((col >> 3)) ^ wp_swz(row)) << 4) + (col & 7) * 2);
  };
  uint32_t a_off[2][2], b_off[9][2];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int h = 0; h < 2; ++h)
      a_off[f][h] = tr_off(8 * WP_DY_PIECE0 + 8 * lq + q4 + 4 * h, wco * 32 + f * 16 + 4 * p4);
#pragma unroll
  for (int tp = 0; tp < 9; ++tp)
#pragma unroll
    for (int h = 0; h < 2; ++h)
      b_off[tp][h] = tr_off((tp / 3) * PW + (tp % 3) * d + 8 * lq + q4 + 4 * h, wci * 16 + 4 * p4);

  f32x4_t acc[2][9];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) acc[f][tp] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  // inline-asm transposed reads (the builtin makes hipcc wait for every LDS-DMA in flight)
  V fa[2][2], fb[2][9];   // [sub-step parity][fragment]
  auto read_sub = [&](uint32_t sb, int par) {
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      s16x4_t lo, hi;
      asm volatile("ds_read_b64_tr_b16 %0, %2\n\t"
                   "ds_read_b64_tr_b16 %1, %3"
                   : "=&v"(lo), "=&v"(hi) : "v"(sb + a_off[f][0]), "v"(sb + a_off[f][1]));
      const auto v8 = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      __builtin_memcpy(&fa[par][f], &v8, 16);
    }
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) {
      s16x4_t lo, hi;
      asm volatile("ds_read_b64_tr_b16 %0, %2\n\t"
                   "ds_read_b64_tr_b16 %1, %3"
                   : "=&v"(lo), "=&v"(hi) : "v"(sb + b_off[tp][0]), "v"(sb + b_off[tp][1]));
      const auto v8 = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      __builtin_memcpy(&fb[par][tp], &v8, 16);
    }
  };
  auto mfma_sub = [&](int par) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int tp = 0; tp < 9; ++tp)
#pragma unroll
      for (int f = 0; f < 2; ++f) acc[f][tp] = Half<E>::mma(fa[par][f], fb[par][tp], acc[f][tp]);
    __builtin_amdgcn_s_setprio(0);
  };

  const long nk = t_end - t_begin;
  if (nk > 0) {
    issue(t_begin, 0);
    if (nk > 1) issue(t_begin + 1, 1);
    for (long k = 0; k < nk; ++k) {
      // stage k landed: only stage k+1's five pieces (if issued) may stay in flight
      if (k + 1 < nk) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();   // every wave's pieces of stage k landed; stage k-1 read
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("" ::: "memory");
      if (k + 2 < nk) issue(t_begin + k + 2, (int)((k + 2) % WP_STAGES));
      const uint32_t sb = lds0 + (uint32_t)((k % WP_STAGES) * WP_STAGE);
      read_sub(sb, 0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      read_sub(sb + 4096, 1);   // sub-step 1's fragments in flight under sub-step 0's MFMAs
      __builtin_amdgcn_sched_barrier(0);
      mfma_sub(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      mfma_sub(1);
    }
  }

  // slab [split][Co][9 C]: lane (lq, lr) of acc[f][tp] holds co = co0 + 32 wco + 16 f + 4 lq + r,
  // ci = ci0 + 16 wci + lr of tap tp
  const int Ncol = 9 * a.C;
  float* O = a.out + (size_t)split * a.Co * Ncol;
  const int lr = lane & 15;
  // buffer stores: per-lane base (co row group, ci), (f, tap, r) as an SGPR offset (the 64-bit
  // index math per value was ~5 instructions of 72 stores per lane)
  const auto rs_o = __builtin_amdgcn_make_buffer_rsrc((void*)O, (short)0, (int)((long)a.Co * Ncol * 4), 0x00020000);
  const uint32_t vb = (uint32_t)(((co0 + wco * 32 + lq * 4) * Ncol + ci0 + wci * 16 + lr) * 4);
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int tp = 0; tp < 9; ++tp)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int so = __builtin_amdgcn_readfirstlane(((f * 16 + r) * Ncol + tp * a.C) * 4);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[f][tp][r]), rs_o, vb, so, 0);
      }
}

}  // namespace

// 3 x 3, stride 1, SAME (pad = dilation <= 4), output rows in 64-pixel strips, 64-channel blocks
// of both Co and C (at most 128 each: the wider layers keep the ping-pong 256 x 256 tiles),
// operands < 2^31 bytes (32-bit buffer offsets)
bool conv_wgrad_patch_ok(const WgradArgs& a) {
  return a.KH == 3 && a.KW == 3 && a.sf == 1 && a.dil >= 1 && a.dil <= 4 && a.pad_h == a.dil &&
         a.pad_w == a.dil && a.H == a.Ho && a.W == a.Wo && a.Wo % 64 == 0 && a.C % 64 == 0 &&
         a.Co % 64 == 0 && a.C <= 128 && a.Co <= 128 && a.ldx % 8 == 0 && a.lddy % 8 == 0 &&
         (long)a.N * a.H * a.W * a.ldx * 2 < (1L << 31) && (long)a.N * a.Ho * a.Wo * a.lddy * 2 < (1L << 31);
}

int conv_wgrad_patch_blocks(const WgradArgs& a) { return (a.Co / 64) * (a.C / 64); }

hipError_t launch_conv_wgrad_patch(int dtype, const WgradArgs& a, hipStream_t s) {
  if (!conv_wgrad_patch_ok(a) || a.splits < 1) return hipErrorInvalidValue;
  const int grid = conv_wgrad_patch_blocks(a) * a.splits;
  auto launch = [&](auto kern) -> hipError_t {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, WP_LDS);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(WP_THREADS), WP_LDS, s, a);
    return hipGetLastError();
  };
  if (dtype == SEG_F16) return launch(conv_wgrad_patch_kernel<f16_t>);
  return launch(conv_wgrad_patch_kernel<bf16_t>);
}
