// Implicit-GEMM convolution kernels for gfx950 (see conv.h for the math).
//
// NT kernel (forward + data-gradient): C[M=pixels][N=out ch] = A[M][K] * B[N][K]^T, both
// operands K-contiguous (NHWC channels / [Co][KH][KW][Ci] weights). 256 threads = 4 waves
// in a 2x2 grid, block tile BM x BN, K-step = 128 bytes of K per row (64 bf16 / 32 f32),
// register-staged double-buffered LDS with an XOR swizzle (chunk ^= (row>>1)&7) that makes
// the 16-lane ds_read_b128 groups conflict-free. MFMA: v_mfma_f32_16x16x32_bf16 for bf16,
// v_mfma_f32_16x16x4_f32 (exact fp32) for the fp32 parity mode; for fp32 each lane group q
// feeds k = 8q..8q+7 over eight MFMAs so the LDS fragment read is still two 16-B reads.
// Epilogue: optional residual add, store, and per-column BN partial statistics (sum and
// M2 about the tile mean — merged with Chan's formula in bn.hip; deterministic).
//
// TN kernel (weight gradient): C[M=Co][N=KH*KW*Ci] = sum over pixels; both operands are
// pixel-major, staged row-major [BK pixels][cols] and read with ds_read_b64_tr_b16
// (bf16) so each lane receives 8 consecutive pixels of one column. Split-K over pixels
// into fp32 slabs, reduced in a fixed order by splitk_reduce (bitwise reproducible).
#include "conv.h"

namespace {

constexpr int NT_THREADS = 256;

template <typename T> struct MmaT;
template <> struct MmaT<bf16_t> { static constexpr int BK = 64; };
template <> struct MmaT<f16_t> { static constexpr int BK = 64; };
template <> struct MmaT<float> { static constexpr int BK = 32; };

__device__ __forceinline__ int swz(int row, int ch) { return ch ^ ((row >> 1) & 7); }

template <typename TO> __device__ __forceinline__ void store_out(TO* p, float v);
template <> __device__ __forceinline__ void store_out<float>(float* p, float v) { *p = v; }
template <> __device__ __forceinline__ void store_out<bf16_t>(bf16_t* p, float v) { *p = f2bf(v); }
template <> __device__ __forceinline__ void store_out<f16_t>(f16_t* p, float v) { *p = (f16_t)v; }
template <typename TO> __device__ __forceinline__ float round_as(float v);
template <> __device__ __forceinline__ float round_as<float>(float v) { return v; }
template <> __device__ __forceinline__ float round_as<bf16_t>(float v) { return bf2f(f2bf(v)); }
template <> __device__ __forceinline__ float round_as<f16_t>(float v) { return (float)(f16_t)v; }

// ======================================================================================
// NT kernel
// ======================================================================================
template <typename T, typename TO, int BM, int BN, bool GENERIC>
__global__ __launch_bounds__(NT_THREADS, 2) void conv_nt_kernel(ConvArgs a) {
  constexpr int BK = MmaT<T>::BK;
  constexpr int EPC = 16 / sizeof(T);        // elements per 16-B chunk
  constexpr int AR = BM / 32;                // A chunks per thread
  constexpr int BR = BN / 32;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int FM = WM / 16, FN = WN / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * (BM + BN) * 128];
  auto As = [&](int b) { return smem + b * (BM * 128); };
  auto Bs = [&](int b) { return smem + 2 * BM * 128 + b * (BN * 128); };

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int lr = lane & 15, lq = lane >> 4;
  const long M = (long)a.N * a.Ho * a.Wo;
  const long m0 = (long)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int K = a.KH * a.KW * a.C;
  const int nk = (K + BK - 1) / BK;
  const T* X = (const T*)a.x;
  const T* Wt = (const T*)a.w;

  // per-thread A rows: pixel coordinates
  int a_n[AR], a_ho[AR], a_wo[AR];
  bool a_ok[AR];
  const int ch = tid & 7;
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    long m = m0 + (tid >> 3) + 32 * i;
    a_ok[i] = m < M;
    long mm = a_ok[i] ? m : 0;
    a_wo[i] = (int)(mm % a.Wo);
    long t = mm / a.Wo;
    a_ho[i] = (int)(t % a.Ho);
    a_n[i] = (int)(t / a.Ho);
  }

  uint4 ra[AR], rb[BR];

  auto src_coord = [&](int o, int k, int pad, int lim, int& s) -> bool {
    int num = o * a.sf - pad + k * a.dil;
    if (a.st > 1) {
      if (num < 0 || (num % a.st) != 0) return false;
      num /= a.st;
    }
    s = num;
    return num >= 0 && num < lim;
  };

  auto load_tiles = [&](int kb) {
    const int k0 = kb * BK;
    if constexpr (!GENERIC) {
      const int tap = k0 / a.C;
      const int c0 = k0 - tap * a.C;
      const int kh = tap / a.KW, kw = tap - (tap / a.KW) * a.KW;
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        int hi, wi;
        bool ok = a_ok[i] && src_coord(a_ho[i], kh, a.pad_h, a.H, hi) &&
                  src_coord(a_wo[i], kw, a.pad_w, a.W, wi);
        if (ok) {
          const T* p = X + ((size_t)((long)a_n[i] * a.H + hi) * a.W + wi) * a.ldx + c0 + ch * EPC;
          ra[i] = *(const uint4*)p;
        } else {
          ra[i] = make_uint4(0, 0, 0, 0);
        }
      }
#pragma unroll
      for (int i = 0; i < BR; ++i) {
        int co = n0 + (tid >> 3) + 32 * i;
        if (co < a.Co) rb[i] = *(const uint4*)(Wt + (size_t)co * a.ldw + k0 + ch * EPC);
        else rb[i] = make_uint4(0, 0, 0, 0);
      }
    } else {
      // element-wise gather (small-C stem): k -> (tap, c)
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        T vals[EPC];
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          int k = k0 + ch * EPC + e;
          float v = 0.f;
          if (a_ok[i] && k < K) {
            int tap = k / a.C, c = k - (k / a.C) * a.C;
            int kh = tap / a.KW, kw = tap - (tap / a.KW) * a.KW;
            int hi, wi;
            if (src_coord(a_ho[i], kh, a.pad_h, a.H, hi) && src_coord(a_wo[i], kw, a.pad_w, a.W, wi))
              v = ldf(X + ((size_t)((long)a_n[i] * a.H + hi) * a.W + wi) * a.ldx + c);
          }
          vals[e] = TypeOps<T>::from_f(v);
        }
        __builtin_memcpy(&ra[i], vals, 16);
      }
#pragma unroll
      for (int i = 0; i < BR; ++i) {
        int co = n0 + (tid >> 3) + 32 * i;
        T vals[EPC];
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          int k = k0 + ch * EPC + e;
          vals[e] = (co < a.Co && k < K) ? Wt[(size_t)co * a.ldw + k] : TypeOps<T>::from_f(0.f);
        }
        __builtin_memcpy(&rb[i], vals, 16);
      }
    }
  };

  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      int row = (tid >> 3) + 32 * i;
      *(uint4*)(As(buf) + row * 128 + swz(row, ch) * 16) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      int row = (tid >> 3) + 32 * i;
      *(uint4*)(Bs(buf) + row * 128 + swz(row, ch) * 16) = rb[i];
    }
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const char* A = As(buf);
    const char* B = Bs(buf);
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        typename Half<T>::V af[FM], bfr[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          int row = wm * WM + i * 16 + lr;
          af[i] = *(const typename Half<T>::V*)(A + row * 128 + swz(row, lq + 4 * s) * 16);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          int row = wn * WN + j * 16 + lr;
          bfr[j] = *(const typename Half<T>::V*)(B + row * 128 + swz(row, lq + 4 * s) * 16);
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = Half<T>::mma(af[i], bfr[j], acc[i][j]);
      }
    } else {
      float af[FM][8], bfr[FN][8];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        int row = wm * WM + i * 16 + lr;
        float4 u = *(const float4*)(A + row * 128 + swz(row, 2 * lq) * 16);
        float4 v = *(const float4*)(A + row * 128 + swz(row, 2 * lq + 1) * 16);
        af[i][0] = u.x; af[i][1] = u.y; af[i][2] = u.z; af[i][3] = u.w;
        af[i][4] = v.x; af[i][5] = v.y; af[i][6] = v.z; af[i][7] = v.w;
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        int row = wn * WN + j * 16 + lr;
        float4 u = *(const float4*)(B + row * 128 + swz(row, 2 * lq) * 16);
        float4 v = *(const float4*)(B + row * 128 + swz(row, 2 * lq + 1) * 16);
        bfr[j][0] = u.x; bfr[j][1] = u.y; bfr[j][2] = u.z; bfr[j][3] = u.w;
        bfr[j][4] = v.x; bfr[j][5] = v.y; bfr[j][6] = v.z; bfr[j][7] = v.w;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][e], bfr[j][e], acc[i][j], 0, 0, 0);
    }
  };

  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  for (int kb = 0; kb < nk; ++kb) {
    const int cur = kb & 1;
    if (kb + 1 < nk) load_tiles(kb + 1);
    compute(cur);
    if (kb + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
  }

  // ---------------- epilogue ----------------
  TO* Y = (TO*)a.y;
  const TO* R = (const TO*)a.r;
  const TO* R2 = (const TO*)a.r2;
  float colsum[FN], colm2[FN];
  const int rows_valid = (int)((M - m0) < BM ? (M - m0) : BM);
#pragma unroll
  for (int j = 0; j < FN; ++j) { colsum[j] = 0.f; colm2[j] = 0.f; }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * WN + j * 16 + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = wm * WM + i * 16 + lq * 4 + r;
        const long m = m0 + rl;
        float v = acc[i][j][r];
        if (m < M && n < a.Co) {
          if (R) v += TypeOps<TO>::to_f(R[(size_t)m * a.ldr + n]);
          if (R2) v += TypeOps<TO>::to_f(R2[(size_t)m * a.ldr2 + n]);
          store_out<TO>(Y + (size_t)m * a.ldy + n, v);
          v = round_as<TO>(v);
          colsum[j] += v;
        } else {
          v = 0.f;
        }
        acc[i][j][r] = v;  // keep rounded value for the M2 pass
      }
    }
  }
  if (a.stats) {
    // reduce column sums over the 4 lane groups, then over the two wm waves via LDS
    float* red = (float*)smem;  // [2][BN] sums, then [2][BN] m2
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float s = colsum[j];
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      colsum[j] = s;
    }
    if (lq == 0) {
#pragma unroll
      for (int j = 0; j < FN; ++j) red[wm * BN + wn * WN + j * 16 + lr] = colsum[j];
    }
    __syncthreads();
    float mean[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      int c = wn * WN + j * 16 + lr;
      mean[j] = (red[c] + red[BN + c]) / (float)rows_valid;
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long m = m0 + wm * WM + i * 16 + lq * 4 + r;
          if (m < M) {
            float d = acc[i][j][r] - mean[j];
            colm2[j] += d * d;
          }
        }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float s = colm2[j];
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      colm2[j] = s;
    }
    __syncthreads();
    if (lq == 0) {
#pragma unroll
      for (int j = 0; j < FN; ++j) red[2 * BN + wm * BN + wn * WN + j * 16 + lr] = colm2[j];
    }
    __syncthreads();
    if (wm == 0 && lq == 0) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        int c = wn * WN + j * 16 + lr;
        int n = n0 + c;
        if (n < a.Co) {
          float2 o = make_float2(red[c] + red[BN + c], red[2 * BN + c] + red[3 * BN + c]);
          *(float2*)(a.stats + 2 * ((size_t)blockIdx.x * a.Co + n)) = o;
        }
      }
    }
  }
}

// ======================================================================================
// TN (weight-gradient) kernel
// ======================================================================================
constexpr int TN_BK = 32;  // pixels per K-step

template <typename T, int BM, int BN, bool GENERIC>
__global__ __launch_bounds__(NT_THREADS, 2) void conv_wgrad_kernel(WgradArgs a) {
  constexpr int EPC = 16 / sizeof(T);
  constexpr int ROWB_A = BM * sizeof(T) + 16;  // padded LDS row bytes
  constexpr int ROWB_B = BN * sizeof(T) + 16;
  constexpr int CPR_A = BM / EPC, CPR_B = BN / EPC;  // chunks per row
  constexpr int ACH = TN_BK * CPR_A / NT_THREADS;    // chunks per thread
  constexpr int BCH = TN_BK * CPR_B / NT_THREADS;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int FM = WM / 16, FN = WN / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * TN_BK * (ROWB_A + ROWB_B)];
  auto As = [&](int b) { return smem + b * (TN_BK * ROWB_A); };
  auto Bs = [&](int b) { return smem + 2 * TN_BK * ROWB_A + b * (TN_BK * ROWB_B); };

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int lr = lane & 15, lq = lane >> 4;
  const int m0 = blockIdx.x * BM;   // co
  const int n0 = blockIdx.y * BN;   // (tap, ci)
  const int Ncol = a.KH * a.KW * a.C;
  const long P = (long)a.N * a.Ho * a.Wo;
  const long chunk = ((P + a.splits - 1) / a.splits + TN_BK - 1) / TN_BK * TN_BK;
  const long p_begin = (long)blockIdx.z * chunk;
  const long p_end = (p_begin + chunk < P) ? p_begin + chunk : P;
  const T* DY = (const T*)a.dy;
  const T* X = (const T*)a.x;

  // B-column decode per thread chunk (fixed across K-steps)
  int b_dh[BCH], b_dw[BCH], b_c[BCH], b_row[BCH], b_cc[BCH];
  bool b_ok[BCH];
#pragma unroll
  for (int i = 0; i < BCH; ++i) {
    int c = tid + NT_THREADS * i;
    b_row[i] = c / CPR_B;
    b_cc[i] = c % CPR_B;
    int col = n0 + b_cc[i] * EPC;
    b_ok[i] = col < Ncol;
    int cc = b_ok[i] ? col : 0;
    int tap = cc / a.C;
    b_c[i] = cc - tap * a.C;
    int kh = tap / a.KW, kw = tap - kh * a.KW;
    b_dh[i] = kh * a.dil - a.pad_h;
    b_dw[i] = kw * a.dil - a.pad_w;
  }
  uint4 ra[ACH], rb[BCH];

  auto load_tiles = [&](long p0) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      int c = tid + NT_THREADS * i;
      int row = c / CPR_A, cc = c % CPR_A;
      long p = p0 + row;
      int co = m0 + cc * EPC;
      if (p < p_end && co < a.Co) ra[i] = *(const uint4*)(DY + (size_t)p * a.lddy + co);
      else ra[i] = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      long p = p0 + b_row[i];
      bool pv = p < p_end;
      long pp = pv ? p : 0;
      int wo = (int)(pp % a.Wo);
      long t = pp / a.Wo;
      int ho = (int)(t % a.Ho);
      int n = (int)(t / a.Ho);
      if constexpr (!GENERIC) {
        int hi = ho * a.sf + b_dh[i], wi = wo * a.sf + b_dw[i];
        if (pv && b_ok[i] && hi >= 0 && hi < a.H && wi >= 0 && wi < a.W)
          rb[i] = *(const uint4*)(X + ((size_t)((long)n * a.H + hi) * a.W + wi) * a.ldx + b_c[i]);
        else
          rb[i] = make_uint4(0, 0, 0, 0);
      } else {
        T vals[EPC];
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          int col = n0 + b_cc[i] * EPC + e;
          float v = 0.f;
          if (pv && col < Ncol) {
            int tap = col / a.C, ci = col - (col / a.C) * a.C;
            int kh = tap / a.KW, kw = tap - (tap / a.KW) * a.KW;
            int hi = ho * a.sf + kh * a.dil - a.pad_h, wi = wo * a.sf + kw * a.dil - a.pad_w;
            if (hi >= 0 && hi < a.H && wi >= 0 && wi < a.W)
              v = ldf(X + ((size_t)((long)n * a.H + hi) * a.W + wi) * a.ldx + ci);
          }
          vals[e] = TypeOps<T>::from_f(v);
        }
        __builtin_memcpy(&rb[i], vals, 16);
      }
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      int c = tid + NT_THREADS * i;
      int row = c / CPR_A, cc = c % CPR_A;
      *(uint4*)(As(buf) + row * ROWB_A + cc * 16) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i)
      *(uint4*)(Bs(buf) + b_row[i] * ROWB_B + b_cc[i] * 16) = rb[i];
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const char* A = As(buf);
    const char* B = Bs(buf);
    if constexpr (sizeof(T) == 2) {
      const int q = (lane & 15) >> 2, pq = lane & 3;
      typename Half<T>::V af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        int col = wm * WM + i * 16 + 4 * pq;
        s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (s16x4_t __attribute__((address_space(3)))*)(A + (8 * lq + q) * ROWB_A + col * 2));
        s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (s16x4_t __attribute__((address_space(3)))*)(A + (8 * lq + 4 + q) * ROWB_A + col * 2));
        short tmp[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        __builtin_memcpy(&af[i], tmp, 16);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        int col = wn * WN + j * 16 + 4 * pq;
        s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (s16x4_t __attribute__((address_space(3)))*)(B + (8 * lq + q) * ROWB_B + col * 2));
        s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (s16x4_t __attribute__((address_space(3)))*)(B + (8 * lq + 4 + q) * ROWB_B + col * 2));
        short tmp[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        __builtin_memcpy(&bfr[j], tmp, 16);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = Half<T>::mma(af[i], bfr[j], acc[i][j]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float af[FM], bfr[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
          af[i] = *(const float*)(A + (8 * lq + e) * ROWB_A + (wm * WM + i * 16 + lr) * 4);
#pragma unroll
        for (int j = 0; j < FN; ++j)
          bfr[j] = *(const float*)(B + (8 * lq + e) * ROWB_B + (wn * WN + j * 16 + lr) * 4);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  };

  const int nk = (int)((p_end - p_begin + TN_BK - 1) / TN_BK);
  if (nk > 0) {
    load_tiles(p_begin);
    store_tiles(0);
    __syncthreads();
    for (int kb = 0; kb < nk; ++kb) {
      const int cur = kb & 1;
      if (kb + 1 < nk) load_tiles(p_begin + (long)(kb + 1) * TN_BK);
      compute(cur);
      if (kb + 1 < nk) store_tiles(cur ^ 1);
      __syncthreads();
    }
  }
  float* O = a.out + (size_t)blockIdx.z * a.Co * Ncol;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      int n = n0 + wn * WN + j * 16 + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int m = m0 + wm * WM + i * 16 + lq * 4 + r;
        if (m < a.Co && n < Ncol) O[(size_t)m * Ncol + n] = acc[i][j][r];
      }
    }
}

__global__ void splitk_reduce_kernel(const float* __restrict__ part, int splits, long stride,
                                     long n, float* __restrict__ out, int accumulate) {
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t * 4 < n; t += (long)gridDim.x * blockDim.x) {
  const long i4 = t * 4;
  if (i4 + 3 < n && (stride & 3) == 0) {
    float4 s = accumulate ? *(const float4*)(out + i4) : make_float4(0.f, 0.f, 0.f, 0.f);
    // loads of 8 slabs in flight, summed in slab order (same result as the serial loop)
    int z = 0;
    for (; z + 8 <= splits; z += 8) {
      float4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = *(const float4*)(part + (size_t)(z + k) * stride + i4);
#pragma unroll
      for (int k = 0; k < 8; ++k) { s.x += v[k].x; s.y += v[k].y; s.z += v[k].z; s.w += v[k].w; }
    }
    for (; z < splits; ++z) {
      float4 v = *(const float4*)(part + (size_t)z * stride + i4);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    *(float4*)(out + i4) = s;
  } else {
    for (long i = i4; i < n && i < i4 + 4; ++i) {
      float s = accumulate ? out[i] : 0.f;
      for (int z = 0; z < splits; ++z) s += part[(size_t)z * stride + i];
      out[i] = s;
    }
  }
  }
}

template <typename T>
__global__ void weight_flip_transpose_kernel(const T* __restrict__ w, T* __restrict__ wt, int co,
                                             int kh, int kw, int ci) {
  long total = (long)co * kh * kw * ci;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  // output index i over [ci][kh][kw][co]
  int o = (int)(i % co);
  long t = i / co;
  int x = (int)(t % kw);
  t /= kw;
  int y = (int)(t % kh);
  int c = (int)(t / kh);
  wt[i] = w[(((size_t)o * kh + (kh - 1 - y)) * kw + (kw - 1 - x)) * ci + c];
}

// every layer's dgrad weight flip [co][k][k][ci] -> [ci][k][k][co] (taps reversed) in one
// launch: one block per 64 x 64 (co x ci) tile of one tap of one layer, transposed through
// LDS so both the reads (ci) and the writes (co) are contiguous; FlipJob.prefix = the layer's
// first tile (the per-element version with a per-element job search and 64-bit div/mod took
// 205 us per step)
template <typename T>
__global__ __launch_bounds__(256) void weight_flip_tiled_kernel(const FlipJob* __restrict__ jobs, int njobs) {
  __shared__ T tile[64][65];
  const long b = blockIdx.x;
  int lo = 0, hi = njobs - 1;   // last job with prefix <= b
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].prefix <= b) lo = mid; else hi = mid - 1;
  }
  const FlipJob J = jobs[lo];
  const int tl = (int)(b - J.prefix);
  const int tco = (J.co + 63) / 64, tci = (J.ci + 63) / 64;
  const int tap = tl / (tco * tci), rem = tl - tap * (tco * tci);
  const int o0 = (rem / tci) * 64, c0 = (rem % tci) * 64;
  const int y = tap / J.k, x = tap - y * J.k;
  const int sy = J.k - 1 - y, sx = J.k - 1 - x;
  const T* W = (const T*)J.w;
  T* WT = (T*)J.wt;
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int r = e >> 6, cc = e & 63;   // r: output channel, cc: input channel
    const int o = o0 + r, ci = c0 + cc;
    if (o < J.co && ci < J.ci) tile[r][cc] = W[(((size_t)o * J.k + sy) * J.k + sx) * J.ci + ci];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int r = e >> 6, cc = e & 63;   // r: input channel, cc: output channel
    const int ci = c0 + r, o = o0 + cc;
    if (o < J.co && ci < J.ci) WT[(((size_t)ci * J.k + y) * J.k + x) * J.co + o] = tile[cc][r];
  }
}

template <typename T, typename TO, int BM, int BN, bool G>
hipError_t nt_launch(const ConvArgs& a, hipStream_t s) {
  long M = (long)a.N * a.Ho * a.Wo;
  dim3 grid(ceil_div(M, BM), ceil_div(a.Co, BN));
  hipLaunchKernelGGL((conv_nt_kernel<T, TO, BM, BN, G>), grid, dim3(NT_THREADS), 0, s, a);
  return hipGetLastError();
}

template <typename T, typename TO>
hipError_t nt_dispatch(const ConvArgs& a, hipStream_t s) {
  const bool generic = (a.C % MmaT<T>::BK) != 0 || (a.ldx % (16 / (int)sizeof(T))) != 0 ||
                       (a.ldw % (16 / (int)sizeof(T))) != 0;
  if (generic) return nt_launch<T, TO, 128, 64, true>(a, s);
  if (a.Co <= 64) return nt_launch<T, TO, 128, 64, false>(a, s);
  return nt_launch<T, TO, 128, 128, false>(a, s);
}

template <typename T, int BM, int BN, bool G>
hipError_t wg_launch(const WgradArgs& a, hipStream_t s) {
  int Ncol = a.KH * a.KW * a.C;
  dim3 grid(ceil_div(a.Co, BM), ceil_div(Ncol, BN), a.splits);
  hipLaunchKernelGGL((conv_wgrad_kernel<T, BM, BN, G>), grid, dim3(NT_THREADS), 0, s, a);
  return hipGetLastError();
}

template <typename T>
hipError_t wg_dispatch(const WgradArgs& a, hipStream_t s) {
  const int epc = 16 / (int)sizeof(T);
  const bool generic = (a.C % epc) != 0 || (a.ldx % epc) != 0;
  if (a.Co % epc != 0 || a.lddy % epc != 0) return hipErrorInvalidValue;
  const int BM = a.Co <= 64 ? 64 : 128;
  if (generic) {
    if (BM == 64) return wg_launch<T, 64, 64, true>(a, s);
    return wg_launch<T, 128, 64, true>(a, s);
  }
  if (BM == 64) return wg_launch<T, 64, 128, false>(a, s);
  return wg_launch<T, 128, 128, false>(a, s);
}

}  // namespace

int conv_nt_mtiles(long M) { return ceil_div(M, 128); }

int conv_nt_stat_rows(int dtype, int out_f32, const ConvArgs& a) {
  return (seg_half(dtype) && !out_f32 && conv_nt_v2_ok(a)) ? conv_nt_v2_rows(a) : 128;
}

namespace {
template <typename E>
__device__ __forceinline__ uint32_t bits16(float v) {
  const E h = TypeOps<E>::from_f(v);
  uint16_t b;
  __builtin_memcpy(&b, &h, 2);
  return b;
}
// space-to-depth stem image: one thread per s2d pixel (i, j) of image n: the 2 x 2 source
// block (rows 2i + dh - pad_h, columns 2j + dw - pad_w), 3 channels each, as 12 16-bit values
// plus 4 zeros, two 16-B stores
template <typename E>
__global__ void cast_s2d_kernel(const float* __restrict__ src, E* __restrict__ dst, int N, int H,
                                int W, int Hs, int Ws, int ph, int pw) {
  const long total = (long)N * Hs * Ws;
  for (long q = (long)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int j = (int)(q % Ws);
    const long t = q / Ws;
    const int i = (int)(t % Hs), n = (int)(t / Hs);
    uint32_t w[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
#pragma unroll
    for (int dh = 0; dh < 2; ++dh)
#pragma unroll
      for (int dw = 0; dw < 2; ++dw) {
        const int h = 2 * i + dh - ph, x = 2 * j + dw - pw;
        const bool ok = (unsigned)h < (unsigned)H && (unsigned)x < (unsigned)W;
        const float* p = src + (((size_t)n * H + (ok ? h : 0)) * W + (ok ? x : 0)) * 3;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const int ch = (dh * 2 + dw) * 3 + c;
          w[ch >> 1] |= (ok ? bits16<E>(p[c]) : 0u) << ((ch & 1) * 16);
        }
      }
    E* o = dst + (size_t)q * 16;
    *(uint4*)o = make_uint4(w[0], w[1], w[2], w[3]);
    *(uint4*)(o + 8) = make_uint4(w[4], w[5], w[6], w[7]);
  }
}
// inverse view for the parity tests: [N][H][W][8], channels 0..2 = the 16-bit image
__global__ void unshuffle_s2d_kernel(const uint16_t* __restrict__ src, uint16_t* __restrict__ dst,
                                     int N, int H, int W, int Hs, int Ws, int ph, int pw) {
  const long total = (long)N * H * W;
  for (long q = (long)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int x = (int)(q % W);
    const long t = q / W;
    const int h = (int)(t % H), n = (int)(t / H);
    const int hh = h + ph, xx = x + pw;
    const uint16_t* p = src + (((size_t)n * Hs + (hh >> 1)) * Ws + (xx >> 1)) * 16 + ((hh & 1) * 2 + (xx & 1)) * 3;
    uint16_t* o = dst + (size_t)q * 8;
    o[0] = p[0]; o[1] = p[1]; o[2] = p[2];
#pragma unroll
    for (int c = 3; c < 8; ++c) o[c] = 0;
  }
}
// w'[co][a][b][(dh*2 + dw)*3 + c] = w[co][2a + dh][2b + dw][c] inside the 7 x 7 kernel, else 0
__global__ void stem_s2d_weights_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ wp, int co) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= co * 256) return;
  const int o = i >> 8, k = i & 255;
  const int tap = k >> 4, ch = k & 15;
  const int a = tap >> 2, b = tap & 3;
  bf16_t v = 0;
  if (ch < 12) {
    const int q = ch / 3, c = ch - q * 3;
    const int kh = 2 * a + (q >> 1), kw = 2 * b + (q & 1);
    if (kh < 7 && kw < 7) v = w[((o * 7 + kh) * 7 + kw) * 3 + c];
  }
  wp[i] = v;
}
// stem weight gradient: few outputs (co * 147) over many splits, so 8 lanes per output each sum
// every 8th split, then a fixed-order sum over the lanes; output (o, kh, kw, c) reads the s2d
// column ((kh/2)*4 + kw/2)*16 + ((kh%2)*2 + kw%2)*3 + c
constexpr int RS_OUT = 32, RS_LANES = 8;
__global__ __launch_bounds__(RS_OUT * RS_LANES) void splitk_reduce_s2d_kernel(
    const float* __restrict__ part, int splits, long stride, int co, float* __restrict__ out) {
  __shared__ float sh[RS_LANES][RS_OUT];
  const int ol = threadIdx.x % RS_OUT, zl = threadIdx.x / RS_OUT;
  const int i = blockIdx.x * RS_OUT + ol;
  const int n = co * 147;
  float acc = 0.f;
  if (i < n) {
    const int o = i / 147, r = i - o * 147;
    const int kh = r / 21, kw = (r - kh * 21) / 3, c = r - kh * 21 - kw * 3;
    const long src = (long)o * 256 + ((kh >> 1) * 4 + (kw >> 1)) * 16 + ((kh & 1) * 2 + (kw & 1)) * 3 + c;
#pragma unroll 4
    for (int z = zl; z < splits; z += RS_LANES) acc += part[(size_t)z * stride + src];
  }
  sh[zl][ol] = acc;
  __syncthreads();
  if (zl == 0 && i < n) {
    float v = sh[0][ol];
#pragma unroll
    for (int k = 1; k < RS_LANES; ++k) v += sh[k][ol];
    out[i] = v;
  }
}
}  // namespace

static dim3 grid_of(long items) {
  long g = (items + 255) / 256;
  if (g > 8192) g = 8192;
  return dim3((unsigned)(g < 1 ? 1 : g));
}

hipError_t launch_cast_s2d(int dtype, const float* src, void* dst, int N, int H, int W, int Hs, int Ws,
                           int pad_h, int pad_w, hipStream_t s) {
  const dim3 g = grid_of((long)N * Hs * Ws);
  if (dtype == SEG_F16)
    hipLaunchKernelGGL(cast_s2d_kernel<f16_t>, g, dim3(256), 0, s, src, (f16_t*)dst, N, H, W, Hs, Ws,
                       pad_h, pad_w);
  else
    hipLaunchKernelGGL(cast_s2d_kernel<bf16_t>, g, dim3(256), 0, s, src, (bf16_t*)dst, N, H, W, Hs, Ws,
                       pad_h, pad_w);
  return hipGetLastError();
}
hipError_t launch_unshuffle_s2d(const void* src, void* dst, int N, int H, int W, int Hs, int Ws,
                                int pad_h, int pad_w, hipStream_t s) {
  hipLaunchKernelGGL(unshuffle_s2d_kernel, grid_of((long)N * H * W), dim3(256), 0, s,
                     (const uint16_t*)src, (uint16_t*)dst, N, H, W, Hs, Ws, pad_h, pad_w);
  return hipGetLastError();
}
hipError_t launch_stem_s2d_weights(const bf16_t* w, bf16_t* wp, int co, hipStream_t s) {
  hipLaunchKernelGGL(stem_s2d_weights_kernel, dim3(ceil_div((long)co * 256, 256)), dim3(256), 0, s, w,
                     wp, co);
  return hipGetLastError();
}
hipError_t launch_splitk_reduce_s2d(const float* part, int splits, long split_stride, int co,
                                    float* out, hipStream_t s) {
  hipLaunchKernelGGL(splitk_reduce_s2d_kernel, dim3(ceil_div((long)co * 147, RS_OUT)),
                     dim3(RS_OUT * RS_LANES), 0, s, part, splits, split_stride, co, out);
  return hipGetLastError();
}

bool conv_nt_uses_v2(int dtype, int out_f32, const ConvArgs& a) {
  return seg_half(dtype) && !out_f32 && conv_nt_v2_ok(a);
}

hipError_t launch_conv_nt(int dtype, int out_f32, const ConvArgs& a, hipStream_t s) {
  if (a.omask && (out_f32 || !conv_nt_omask_ok(dtype, a))) return hipErrorInvalidValue;
  if (conv_nt_uses_v2(dtype, out_f32, a)) return launch_conv_nt_v2(dtype, a, s);
  if (conv_skinny_ok(dtype, out_f32, a)) return launch_conv_skinny(dtype, a, s);
  if (dtype == SEG_BF16) {
    if (out_f32) return nt_dispatch<bf16_t, float>(a, s);
    return nt_dispatch<bf16_t, bf16_t>(a, s);
  }
  if (dtype == SEG_F16) {
    if (out_f32) return nt_dispatch<f16_t, float>(a, s);
    return nt_dispatch<f16_t, f16_t>(a, s);
  }
  return nt_dispatch<float, float>(a, s);
}

hipError_t launch_conv_wgrad(int dtype, const WgradArgs& a, hipStream_t s) {
  if (a.dy2 && !(seg_half(dtype) && a.KH == 1 && a.KW == 1 && conv_wgrad_v2_ok(a))) return hipErrorInvalidValue;
  if (seg_half(dtype) && conv_wgrad_patch_ok(a)) return launch_conv_wgrad_patch(dtype, a, s);
  if (seg_half(dtype) && conv_wgrad_v2_ok(a)) return launch_conv_wgrad_v2(dtype, a, s);
  if (dtype == SEG_BF16) return wg_dispatch<bf16_t>(a, s);
  if (dtype == SEG_F16) return wg_dispatch<f16_t>(a, s);
  return wg_dispatch<float>(a, s);
}

hipError_t launch_splitk_reduce(const float* part, int splits, long split_stride, long n,
                                float* out, int accumulate, hipStream_t s) {
  long threads = (n + 3) / 4;
  // at most 512 grid-stride workgroups: the reduces run on the weight-gradient stream beside the
  // data-gradient chain, and a full-size grid (one float4 per thread, up to ~2300 workgroups)
  // takes CUs from it in one burst; 256 / 512 / 1024 measured +0.2-0.3 % per step against the
  // full grid, 128 -0.1 % (profiles/r04_splitk_grid.txt); per-element sums unchanged
  long blocks = ceil_div(threads, 256);
  if (blocks > 512) blocks = 512;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, s, part,
                     splits, split_stride, n, out, accumulate);
  return hipGetLastError();
}


hipError_t launch_weight_flip_batched(int dtype, const FlipJob* jobs, int njobs, long total,
                                      hipStream_t s) {
  // total = number of 64 x 64 tiles over all jobs (flip_tiles)
  if (seg_half(dtype))   // a bit copy: one 16-bit instantiation serves bf16 and fp16
    hipLaunchKernelGGL(weight_flip_tiled_kernel<bf16_t>, dim3((int)total), dim3(256), 0, s, jobs, njobs);
  else
    hipLaunchKernelGGL(weight_flip_tiled_kernel<float>, dim3((int)total), dim3(256), 0, s, jobs, njobs);
  return hipGetLastError();
}

hipError_t launch_weight_flip_transpose(int dtype, const void* w, void* wt, int co, int kh, int kw,
                                        int ci, hipStream_t s) {
  long total = (long)co * kh * kw * ci;
  dim3 g(ceil_div(total, 256));
  if (seg_half(dtype))
    hipLaunchKernelGGL(weight_flip_transpose_kernel<bf16_t>, g, dim3(256), 0, s,
                       (const bf16_t*)w, (bf16_t*)wt, co, kh, kw, ci);
  else
    hipLaunchKernelGGL(weight_flip_transpose_kernel<float>, g, dim3(256), 0, s, (const float*)w,
                       (float*)wt, co, kh, kw, ci);
  return hipGetLastError();
}

long flip_tiles(int co, int k, int ci) {
  return (long)k * k * ((co + 63) / 64) * ((ci + 63) / 64);
}
