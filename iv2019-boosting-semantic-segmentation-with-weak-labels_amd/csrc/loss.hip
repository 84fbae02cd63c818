// Fused loss head (see loss.h).
//
// Work decomposition (deterministic, no atomics): a workgroup OWNS a block of LA x LB
// low-resolution pixels of one image and gathers every full-resolution pixel whose bilinear
// footprint touches them (a halo of one low-res cell each side). The gradient w.r.t. the
// low-res logits is the transpose of the separable resize: per full-res row the pixel
// gradients are reduced along x into the owned columns (weights 1-xl / xl), then folded
// into the owned rows (weights 1-yl / yl) held in registers -- or, when the block's columns fit
// one chunk (C2: 249 of 256), each thread first sums its column over the rows into the owned
// rows and the x-reduction runs once per owned row (YF; 409 -> 326 us per call at C2). Loss
// sums and decisions are produced only by the owner of a pixel (the block containing its
// top-left source corner).
#include "loss.h"

namespace {

#ifndef LOSS_LA
#define LOSS_LA 3   // 3 x 30: 1548 blocks at C2 = 2 full waves of 3 blocks per CU (4: 1.5 waves, +12 %)
#endif
#ifndef LOSS_LB
#define LOSS_LB 30
#endif
#ifndef LOSS_YF
#define LOSS_YF 1   // A/B builds: 0 = the per-row x-reduction for every geometry
#endif
constexpr int LA = LOSS_LA;   // owned low-res rows per block
constexpr int LB = LOSS_LB;   // owned low-res cols per block
constexpr int THREADS = 256;
constexpr int GLD = THREADS + 1;   // gbuf row stride

__device__ __forceinline__ void lerp_of(int o, int n_in, int n_out, int& lo, int& hi, float& l) {
  // TF ResizeBilinear legacy scaler, align_corners=True
  const float scale = n_out > 1 ? (float)(n_in - 1) / (float)(n_out - 1) : 0.f;
  const float fin = (float)o * scale;
  lo = (int)fin;
  hi = lo + 1 < n_in - 1 ? lo + 1 : n_in - 1;
  l = fin - (float)lo;
}

__device__ __forceinline__ int lo_of(int o, int n_in, int n_out) {
  const float scale = n_out > 1 ? (float)(n_in - 1) / (float)(n_out - 1) : 0.f;
  return (int)((float)o * scale);
}

// first o in [0, n_out) with lo_of(o) >= target (n_out if none)
__device__ int first_with_lo_ge(int target, int n_in, int n_out) {
  if (target <= 0) return 0;
  const float scale = n_out > 1 ? (float)(n_in - 1) / (float)(n_out - 1) : 0.f;
  int o = scale > 0.f ? (int)((float)target / scale) : n_out;
  if (o > n_out) o = n_out;
  if (o < 0) o = 0;
  while (o < n_out && lo_of(o, n_in, n_out) < target) ++o;
  while (o > 0 && lo_of(o - 1, n_in, n_out) >= target) --o;
  return o;
}

// YF (y first, the block's full-resolution columns fit one THREADS chunk): a thread keeps its
// column's gradient summed over the rows into the LA owned low-res rows (weights 1-yl / yl) in
// registers, and the x-transpose reduction into the owned columns runs once per owned row at the
// end instead of once per full-resolution row (~32 LDS passes and barrier pairs per block). The
// same products, summed h-then-w instead of w-then-h.
template <int C1, int C2, int C3, int YF = 0>
__global__ __launch_bounds__(THREADS) void loss_head_kernel(LossArgs a, LossTables t) {
  constexpr int CT = C1 + C2 + C3;
  constexpr int WIN_R = LA + 2, WIN_C = LB + 2;
  constexpr int PAIRS = LB * CT;
  constexpr int PPT = (PAIRS + THREADS - 1) / THREADS;  // owned (col, ch) pairs per thread
  __shared__ float win[WIN_R * WIN_C * CT];
  __shared__ float gbuf[CT * GLD];   // [channel][pixel], padded: (c, w) -> bank (c + w) % 64
  __shared__ int wstart[LB + 3];
  __shared__ int rng[4];
  constexpr int XT = 512;          // per-block x-lerp table (full-res columns of the footprint)
  __shared__ float xlt[XT];        // xl(w)
  __shared__ short xlo_t[XT], xhi_t[XT];
  __shared__ float wa_t[XT], wb_t[XT];   // x-transpose weights: to column lo / to column hi
  __shared__ float red[6][THREADS / 64];

  const int tid = threadIdx.x;
  const int nbx = (a.Wl + LB - 1) / LB, nby = (a.Hl + LA - 1) / LA;
  const int bx = blockIdx.x % nbx;
  const int by = (blockIdx.x / nbx) % nby;
  const int n = blockIdx.x / (nbx * nby);
  const int i0 = by * LA, j0 = bx * LB;
  const int i_own_end = min(i0 + LA, a.Hl), j_own_end = min(j0 + LB, a.Wl);

  if (tid == 0) {
    rng[0] = first_with_lo_ge(i0 - 1, a.Hl, a.H);               // h_begin
    rng[1] = first_with_lo_ge(i_own_end, a.Hl, a.H);            // h_end (exclusive)
    rng[2] = first_with_lo_ge(j0 - 1, a.Wl, a.W);               // w_begin
    rng[3] = first_with_lo_ge(j_own_end, a.Wl, a.W);            // w_end (exclusive)
  }
  // wstart[q] = first w with lo_x(w) >= j0 - 1 + q, q = 0..LB+2
  for (int q = tid; q < LB + 3; q += THREADS) wstart[q] = first_with_lo_ge(j0 - 1 + q, a.Wl, a.W);
  // low-res logits window rows i0-1..i0+LA, cols j0-1..j0+LB
  for (int e = tid; e < WIN_R * WIN_C * CT; e += THREADS) {
    int c = e % CT, q = (e / CT) % WIN_C, r = e / (CT * WIN_C);
    int i = i0 - 1 + r, j = j0 - 1 + q;
    float v = 0.f;
    if (i >= 0 && i < a.Hl && j >= 0 && j < a.Wl)
      v = a.logits[((size_t)((long)n * a.Hl + i) * a.Wl + j) * a.ldl + c];
    win[e] = v;
  }
  __syncthreads();
  const int h_begin = rng[0], h_end = rng[1], w_begin = rng[2], w_end = rng[3];
  const bool use_xt = w_end - w_begin <= XT;
  if (use_xt) {
    for (int w = w_begin + tid; w < w_end; w += THREADS) {
      int lo, hi;
      float xl;
      lerp_of(w, a.Wl, a.W, lo, hi, xl);
      xlt[w - w_begin] = xl;
      xlo_t[w - w_begin] = (short)lo;
      xhi_t[w - w_begin] = (short)hi;
      wa_t[w - w_begin] = hi == lo ? 1.f : 1.f - xl;   // clamped last column takes both shares
      wb_t[w - w_begin] = xl;
    }
    __syncthreads();
  }

  float acc[PPT][LA];
#pragma unroll
  for (int u = 0; u < PPT; ++u)
#pragma unroll
    for (int r = 0; r < LA; ++r) acc[u][r] = 0.f;

  float colacc[YF ? LA : 1][YF ? CT : 1];
#pragma unroll
  for (int r = 0; r < (YF ? LA : 1); ++r)
#pragma unroll
    for (int c = 0; c < (YF ? CT : 1); ++c) colacc[r][c] = 0.f;

  float s1 = 0.f, s2v = 0.f, s2h = 0.f, c1n = 0.f, c2vn = 0.f, c2hn = 0.f;
  const bool strong = n < a.npp;
  const float* soft = nullptr;
  if (!strong) {
    soft = (n < a.npp + a.npb) ? a.bbox_soft + (size_t)(n - a.npp) * a.H * a.W * t.n_pb
                               : a.tag_soft + (size_t)(n - a.npp - a.npb) * a.H * a.W * t.n_pb;
  }

  // x-reduction into the owned columns of one THREADS-wide chunk of gbuf (columns from wc):
  // ra(j, c) += sum_w wx(w, j) gbuf(c, w)
  auto xred = [&](int wc, float (&ra)[PPT]) {
#pragma unroll
    for (int u = 0; u < PPT; ++u) {
      const int pr = tid + THREADS * u;
      if (pr < PAIRS) {
        const int jj = pr / CT, c = pr % CT;
        const int j = j0 + jj;
        if (j < j_own_end) {
          const int cend = min(w_end, wc + THREADS);
          float sacc = 0.f;
          // w with lo == j  -> weight (1 - xl) [+ xl if j is the clamped last column]
          int wa = max(wstart[jj + 1], wc), wb = min(wstart[jj + 2], cend);
          if (use_xt) {
            // precomputed weights: one gbuf read + one broadcast table read per w
            for (int w = wa; w < wb; ++w) sacc += gbuf[c * GLD + (w - wc)] * wa_t[w - w_begin];
            wa = max(wstart[jj], wc);
            wb = min(wstart[jj + 1], cend);
            for (int w = wa; w < wb; ++w) sacc += gbuf[c * GLD + (w - wc)] * wb_t[w - w_begin];
            ra[u] += sacc;
            continue;
          }
          for (int w = wa; w < wb; ++w) {
            int lo, hi;
            float xl;
            if (use_xt) { xl = xlt[w - w_begin]; lo = xlo_t[w - w_begin]; hi = xhi_t[w - w_begin]; }
            else lerp_of(w, a.Wl, a.W, lo, hi, xl);
            float gv = gbuf[c * GLD + (w - wc)];
            sacc += gv * (1.f - xl);
            if (hi == lo) sacc += gv * xl;
          }
          // w with lo == j-1 (hi == j) -> weight xl
          wa = max(wstart[jj], wc);
          wb = min(wstart[jj + 1], cend);
          for (int w = wa; w < wb; ++w) {
            int lo, hi;
            float xl;
            if (use_xt) { xl = xlt[w - w_begin]; lo = xlo_t[w - w_begin]; hi = xhi_t[w - w_begin]; }
            else lerp_of(w, a.Wl, a.W, lo, hi, xl);
            if (hi == j) sacc += gbuf[c * GLD + (w - wc)] * xl;
          }
          ra[u] += sacc;
        }
      }
    }
  };

  for (int h = h_begin; h < h_end; ++h) {
    int ylo, yhi;
    float yl;
    lerp_of(h, a.Hl, a.H, ylo, yhi, yl);
    const bool row_owned = ylo >= i0 && ylo < i_own_end;
    float rowacc[PPT];
#pragma unroll
    for (int u = 0; u < PPT; ++u) rowacc[u] = 0.f;

    for (int wc = w_begin; wc < w_end; wc += THREADS) {
      const int w = wc + tid;
      if (w < w_end) {
        int xlo, xhi;
        float xl;
        if (use_xt) { xl = xlt[w - w_begin]; xlo = xlo_t[w - w_begin]; xhi = xhi_t[w - w_begin]; }
        else lerp_of(w, a.Wl, a.W, xlo, xhi, xl);
        const float* tl = win + (((ylo - (i0 - 1)) * WIN_C) + (xlo - (j0 - 1))) * CT;
        const float* tr = win + (((ylo - (i0 - 1)) * WIN_C) + (xhi - (j0 - 1))) * CT;
        const float* bl = win + (((yhi - (i0 - 1)) * WIN_C) + (xlo - (j0 - 1))) * CT;
        const float* br = win + (((yhi - (i0 - 1)) * WIN_C) + (xhi - (j0 - 1))) * CT;
        float x[CT];
#pragma unroll
        for (int c = 0; c < CT; ++c) {
          float top = tl[c] + (tr[c] - tl[c]) * xl;
          float bot = bl[c] + (br[c] - bl[c]) * xl;
          x[c] = top + (bot - top) * yl;
        }
        // ---- softmaxes ----
        float p[CT];
        float lse1, lse2, lse3, m1, m2, m3;
        {
          m1 = x[0];
#pragma unroll
          for (int c = 1; c < C1; ++c) m1 = fmaxf(m1, x[c]);
          float s = 0.f;
#pragma unroll
          for (int c = 0; c < C1; ++c) { p[c] = __expf(x[c] - m1); s += p[c]; }
          const float rs = 1.f / s;
#pragma unroll
          for (int c = 0; c < C1; ++c) p[c] = p[c] * rs;
          lse1 = logf(s);
        }
        {
          m2 = x[C1];
#pragma unroll
          for (int c = 1; c < C2; ++c) m2 = fmaxf(m2, x[C1 + c]);
          float s = 0.f;
#pragma unroll
          for (int c = 0; c < C2; ++c) { p[C1 + c] = __expf(x[C1 + c] - m2); s += p[C1 + c]; }
          const float rs = 1.f / s;
#pragma unroll
          for (int c = 0; c < C2; ++c) p[C1 + c] = p[C1 + c] * rs;
          lse2 = logf(s);
        }
        {
          m3 = x[C1 + C2];
#pragma unroll
          for (int c = 1; c < C3; ++c) m3 = fmaxf(m3, x[C1 + C2 + c]);
          float s = 0.f;
#pragma unroll
          for (int c = 0; c < C3; ++c) { p[C1 + C2 + c] = __expf(x[C1 + C2 + c] - m3); s += p[C1 + C2 + c]; }
          const float rs = 1.f / s;
#pragma unroll
          for (int c = 0; c < C3; ++c) p[C1 + C2 + c] = p[C1 + C2 + c] * rs;
          lse3 = logf(s);
        }
        // l1 argmax over probabilities (first max)
        int d1 = 0;
        {
          float best = p[0];
#pragma unroll
          for (int c = 1; c < C1; ++c)
            if (p[c] > best) { best = p[c]; d1 = c; }
        }
        // ---- labels ----
        float y2[C2], y3[C3];
        float w1 = 0.f, w2 = 0.f, w3 = 0.f;
        int l1lab = -1;
        const size_t pix = ((size_t)((long)(strong ? n : 0) * a.H + h)) * a.W + w;
        if (strong) {
          const int lab = a.px_labels[pix];
          l1lab = t.pp2l1[lab];
          w1 = l1lab <= t.l1_wmax ? 1.f : 0.f;
          const int v = t.pp2veh[lab], hm = t.pp2hum[lab];
#pragma unroll
          for (int c = 0; c < C2; ++c) y2[c] = c == v ? 1.f : 0.f;
#pragma unroll
          for (int c = 0; c < C3; ++c) y3[c] = c == hm ? 1.f : 0.f;
          w2 = 1.f - y2[C2 - 1];
          w3 = 1.f - y3[C3 - 1];
        } else {
          const float* sp = soft + ((size_t)h * a.W + w) * t.n_pb;
#pragma unroll
          for (int c = 0; c < C2; ++c) y2[c] = 0.f;
#pragma unroll
          for (int c = 0; c < C3; ++c) y3[c] = 0.f;
          for (int c = 0; c < t.n_pb; ++c) {  // unsorted_segment_sum, index order
            const float v = sp[c];
            const int sv = t.pb2veh[c], sh = t.pb2hum[c];
#pragma unroll
            for (int k = 0; k < C2; ++k) if (k == sv) y2[k] += v;
#pragma unroll
            for (int k = 0; k < C3; ++k) if (k == sh) y3[k] += v;
          }
          float mx2 = y2[0], mx3 = y3[0];
#pragma unroll
          for (int k = 1; k < C2 - 1; ++k) mx2 = fmaxf(mx2, y2[k]);
#pragma unroll
          for (int k = 1; k < C3 - 1; ++k) mx3 = fmaxf(mx3, y3[k]);
          w2 = ((1.f - y2[C2 - 1]) > 0.01f && d1 == t.cid_l1_vehicle && mx2 >= 0.01f) ? 1.f : 0.f;
          w3 = ((1.f - y3[C3 - 1]) > 0.01f && d1 == t.cid_l1_human && mx3 >= 0.01f) ? 1.f : 0.f;
        }
        // ---- losses (owner only) ----
        const bool owned = row_owned && xlo >= j0 && xlo < j_own_end;
        if (owned) {
          if (strong) {
            float xl1 = 0.f;
#pragma unroll
            for (int c = 0; c < C1; ++c) if (c == l1lab) xl1 = x[c];
            s1 += w1 * (lse1 - (xl1 - m1));
            c1n += w1 != 0.f ? 1.f : 0.f;
          }
          float l2 = 0.f, l3 = 0.f;
#pragma unroll
          for (int c = 0; c < C2; ++c) l2 += y2[c] * (lse2 - (x[C1 + c] - m2));
#pragma unroll
          for (int c = 0; c < C3; ++c) l3 += y3[c] * (lse3 - (x[C1 + C2 + c] - m3));
          s2v += w2 * l2;
          s2h += w3 * l3;
          c2vn += w2 != 0.f ? 1.f : 0.f;
          c2hn += w3 != 0.f ? 1.f : 0.f;
          if (a.decisions || a.l1_decisions) {
            const size_t op = ((size_t)((long)n * a.H + h)) * a.W + w;
            if (a.l1_decisions) a.l1_decisions[op] = d1;
            if (a.decisions) {
              int d;
              if (d1 == t.cid_l1_vehicle) {
                int b = 0;
                float bv = p[C1];
#pragma unroll
                for (int c = 1; c < C2; ++c) if (p[C1 + c] > bv) { bv = p[C1 + c]; b = c; }
                d = t.veh_to_common[b];
              } else if (d1 == t.cid_l1_human) {
                int b = 0;
                float bv = p[C1 + C2];
#pragma unroll
                for (int c = 1; c < C3; ++c) if (p[C1 + C2 + c] > bv) { bv = p[C1 + C2 + c]; b = c; }
                d = t.hum_to_common[b];
              } else {
                d = t.l1_to_common[d1];
              }
              a.decisions[op] = d;
            }
          }
        }
        // ---- gradients: TF xent backprop = p - y, times the weight ----
        if constexpr (YF) {
          float gv[CT];
#pragma unroll
          for (int c = 0; c < C1; ++c) gv[c] = strong ? w1 * (p[c] - (c == l1lab ? 1.f : 0.f)) : 0.f;
#pragma unroll
          for (int c = 0; c < C2; ++c) gv[C1 + c] = w2 * (p[C1 + c] - y2[c]);
#pragma unroll
          for (int c = 0; c < C3; ++c) gv[C1 + C2 + c] = w3 * (p[C1 + C2 + c] - y3[c]);
#pragma unroll
          for (int r = 0; r < (YF ? LA : 1); ++r) {
            const int i = i0 + r;
            if (i == ylo)
#pragma unroll
              for (int c = 0; c < CT; ++c) colacc[r][c] += gv[c] * (1.f - yl);
            if (i == yhi)
#pragma unroll
              for (int c = 0; c < CT; ++c) colacc[r][c] += gv[c] * yl;
          }
        } else {
#pragma unroll
          for (int c = 0; c < C1; ++c)
            gbuf[c * GLD + tid] = strong ? w1 * (p[c] - (c == l1lab ? 1.f : 0.f)) : 0.f;
#pragma unroll
          for (int c = 0; c < C2; ++c) gbuf[(C1 + c) * GLD + tid] = w2 * (p[C1 + c] - y2[c]);
#pragma unroll
          for (int c = 0; c < C3; ++c) gbuf[(C1 + C2 + c) * GLD + tid] = w3 * (p[C1 + C2 + c] - y3[c]);
        }
      }
      if constexpr (YF) continue;   // (one chunk: wc == w_begin)
      __syncthreads();
      xred(wc, rowacc);
      __syncthreads();
    }
    // ---- fold the row into owned low-res rows ----
    if constexpr (!YF) {
#pragma unroll
      for (int u = 0; u < PPT; ++u) {
#pragma unroll
        for (int r = 0; r < LA; ++r) {
          const int i = i0 + r;
          if (i == ylo) acc[u][r] += rowacc[u] * (1.f - yl);
          if (i == yhi) acc[u][r] += rowacc[u] * yl;
        }
      }
    }
  }
  if constexpr (YF) {   // the column sums of each owned row through the x-reduction, once
#pragma unroll
    for (int r = 0; r < (YF ? LA : 1); ++r) {
      if (w_begin + tid < w_end)
#pragma unroll
        for (int c = 0; c < CT; ++c) gbuf[c * GLD + tid] = colacc[r][c];
      __syncthreads();
      float ra[PPT];
#pragma unroll
      for (int u = 0; u < PPT; ++u) ra[u] = 0.f;
      xred(w_begin, ra);
#pragma unroll
      for (int u = 0; u < PPT; ++u) acc[u][r] = ra[u];
      __syncthreads();
    }
  }
  // ---- write owned gradient ----
#pragma unroll
  for (int u = 0; u < PPT; ++u) {
    const int pr = tid + THREADS * u;
    if (pr < PAIRS) {
      const int jj = pr / CT, c = pr % CT;
      const int j = j0 + jj;
      if (j < j_own_end) {
#pragma unroll
        for (int r = 0; r < LA; ++r) {
          const int i = i0 + r;
          if (i < i_own_end)
            a.grad_un[((size_t)((long)n * a.Hl + i) * a.Wl + j) * a.ldl + c] = acc[u][r];
        }
      }
    }
  }
  // ---- loss partials ----
  float vals[6] = {s1, s2v, s2h, c1n, c2vn, c2hn};
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    float v = wave_sum(vals[k]);
    if ((tid & 63) == 0) red[k][tid >> 6] = v;
  }
  __syncthreads();
  if (tid < 6) {
    float v = 0.f;
    for (int q = 0; q < THREADS / 64; ++q) v += red[tid][q];
    a.part[(size_t)blockIdx.x * 8 + tid] = v;
  }
}

__global__ void loss_finalize_kernel(const float* __restrict__ part, int nblocks, int c1, int c2,
                                     int c3, int ldl, float* out, float* dzscale, float loss_scale) {
  __shared__ double sh[6][256];
  double v[6] = {0, 0, 0, 0, 0, 0};
  for (int b = threadIdx.x; b < nblocks; b += 256)
    for (int k = 0; k < 6; ++k) v[k] += part[(size_t)b * 8 + k];
  for (int k = 0; k < 6; ++k) sh[k][threadIdx.x] = v[k];
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st)
      for (int k = 0; k < 6; ++k) sh[k][threadIdx.x] += sh[k][threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    double S1 = sh[0][0], S2 = sh[1][0], S3 = sh[2][0], n1 = sh[3][0], n2 = sh[4][0], n3 = sh[5][0];
    float l1 = n1 > 0 ? (float)(S1 / n1) : 0.f;   // SUM_BY_NONZERO_WEIGHTS, safe division
    float l2 = n2 > 0 ? (float)(S2 / n2) : 0.f;
    float l3 = n3 > 0 ? (float)(S3 / n3) : 0.f;
    out[0] = l1 + 0.1f * (l2 + l3);
    out[1] = l1; out[2] = l2; out[3] = l3;
    out[4] = (float)n1; out[5] = (float)n2; out[6] = (float)n3;
    out[7] = n1 > 0 ? (float)(1.0 / n1) : 0.f;
    out[8] = n2 > 0 ? (float)(0.1 / n2) : 0.f;
    out[9] = n3 > 0 ? (float)(0.1 / n3) : 0.f;
  }
  __syncthreads();
  if (threadIdx.x < ldl) {
    int c = threadIdx.x;
    double S = 0;
    if (c < c1) S = sh[3][0] > 0 ? 1.0 / sh[3][0] : 0.0;
    else if (c < c1 + c2) S = sh[4][0] > 0 ? 0.1 / sh[4][0] : 0.0;
    else if (c < c1 + c2 + c3) S = sh[5][0] > 0 ? 0.1 / sh[5][0] : 0.0;
    dzscale[c] = (float)(S * loss_scale);   // the gradient seed carries the loss scale (fp16)
  }
}

__global__ void confusion_kernel(const int* __restrict__ lab, const int* __restrict__ dec, long n,
                                 int nc, int* cm) {
  __shared__ int h[64 * 64];
  for (int i = threadIdx.x; i < nc * nc; i += blockDim.x) h[i] = 0;
  __syncthreads();
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    int l = lab[i], d = dec[i];
    if (l >= 0 && l < nc && d >= 0 && d < nc) atomicAdd(&h[l * nc + d], 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nc * nc; i += blockDim.x)
    if (h[i]) atomicAdd(&cm[i], h[i]);
}


// TF 1.12 ResizeNearestNeighbor(align_corners=True) source index (legacy scaler, roundf)
__device__ __forceinline__ int nn_src(int o, int n_in, int n_out) {
  const float scale = n_out > 1 ? (float)(n_in - 1) / (float)(n_out - 1) : (float)n_in / (float)n_out;
  const int i = (int)roundf((float)o * scale);
  return i < n_in - 1 ? i : n_in - 1;
}

// one thread per output pixel; the 4 source cells of the bilinear footprint are read from
// HBM/L2 directly (eval is one forward per batch: this kernel is ~0.1 % of it)
template <int C1, int C2, int C3>
__global__ __launch_bounds__(256) void eval_decisions_kernel(EvalArgs a, LossTables t) {
  constexpr int CT = C1 + C2 + C3;
  const long total = (long)a.N * a.Ho * a.Wo;
  for (long id = (long)blockIdx.x * blockDim.x + threadIdx.x; id < total;
       id += (long)gridDim.x * blockDim.x) {
    const int xo = (int)(id % a.Wo);
    const int yo = (int)((id / a.Wo) % a.Ho);
    const int n = (int)(id / ((long)a.Wo * a.Ho));
    const int h = nn_src(yo, a.H, a.Ho), w = nn_src(xo, a.W, a.Wo);
    int ylo, yhi, xlo, xhi;
    float yl, xl;
    lerp_of(h, a.Hl, a.H, ylo, yhi, yl);
    lerp_of(w, a.Wl, a.W, xlo, xhi, xl);
    const float* base = a.logits + (size_t)n * a.Hl * a.Wl * a.ldl;
    const float* tl = base + ((size_t)ylo * a.Wl + xlo) * a.ldl;
    const float* tr = base + ((size_t)ylo * a.Wl + xhi) * a.ldl;
    const float* bl = base + ((size_t)yhi * a.Wl + xlo) * a.ldl;
    const float* br = base + ((size_t)yhi * a.Wl + xhi) * a.ldl;
    float p[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      float top = tl[c] + (tr[c] - tl[c]) * xl;
      float bot = bl[c] + (br[c] - bl[c]) * xl;
      p[c] = top + (bot - top) * yl;
    }
    // softmax per head (the same arithmetic as the loss head), argmax first max
    auto softmax = [&](int c0, int nc) {
      float m = p[c0];
#pragma unroll
      for (int c = 1; c < nc; ++c) m = fmaxf(m, p[c0 + c]);
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < nc; ++c) { p[c0 + c] = __expf(p[c0 + c] - m); s += p[c0 + c]; }
      const float rs = 1.f / s;
#pragma unroll
      for (int c = 0; c < nc; ++c) p[c0 + c] = p[c0 + c] * rs;
    };
    softmax(0, C1);
    softmax(C1, C2);
    softmax(C1 + C2, C3);
    int d1 = 0;
    float b1 = p[0];
#pragma unroll
    for (int c = 1; c < C1; ++c) if (p[c] > b1) { b1 = p[c]; d1 = c; }
    int d;
    if (d1 == t.cid_l1_vehicle) {
      int b = 0;
      float bv = p[C1];
#pragma unroll
      for (int c = 1; c < C2; ++c) if (p[C1 + c] > bv) { bv = p[C1 + c]; b = c; }
      d = t.veh_to_common[b];
    } else if (d1 == t.cid_l1_human) {
      int b = 0;
      float bv = p[C1 + C2];
#pragma unroll
      for (int c = 1; c < C3; ++c) if (p[C1 + C2 + c] > bv) { bv = p[C1 + C2 + c]; b = c; }
      d = t.hum_to_common[b];
    } else {
      d = t.l1_to_common[d1];
    }
    d = a.map[d];   // tf.gather(ocids2ncids, decs)
    if (a.replace_voids == 2) {
      // PREDICT order (define_estimator_hierarchical.py:227-231): _resize_predictions first --
      // decisions NEAREST (above), l1_probabilities ResizeBilinear(align_corners) from the
      // network to the output size -- then _replace_voids on the RESIZED probabilities
      // (top_k(k=2), stable; void = decision C1 - 1). The 4 network-resolution pixels of the
      // output pixel's footprint get their l1 softmax from the low-res logits as above.
      int y0, y1, x0, x1;
      float ylp, xlp;
      lerp_of(yo, a.H, a.Ho, y0, y1, ylp);
      lerp_of(xo, a.W, a.Wo, x0, x1, xlp);
      float q[4][C1];
      const int ys[2] = {y0, y1}, xs[2] = {x0, x1};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        int ya, yb, xa, xb;
        float ly, lx;
        lerp_of(ys[k >> 1], a.Hl, a.H, ya, yb, ly);
        lerp_of(xs[k & 1], a.Wl, a.W, xa, xb, lx);
        const float* ta = base + ((size_t)ya * a.Wl + xa) * a.ldl;
        const float* tb = base + ((size_t)ya * a.Wl + xb) * a.ldl;
        const float* ba = base + ((size_t)yb * a.Wl + xa) * a.ldl;
        const float* bb = base + ((size_t)yb * a.Wl + xb) * a.ldl;
        float m = -INFINITY;
#pragma unroll
        for (int c = 0; c < C1; ++c) {
          float top = ta[c] + (tb[c] - ta[c]) * lx;
          float bot = ba[c] + (bb[c] - ba[c]) * lx;
          q[k][c] = top + (bot - top) * ly;
          m = fmaxf(m, q[k][c]);
        }
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < C1; ++c) { q[k][c] = __expf(q[k][c] - m); s += q[k][c]; }
        const float rs = 1.f / s;
#pragma unroll
        for (int c = 0; c < C1; ++c) q[k][c] = q[k][c] * rs;
      }
      int i1 = -1, i2 = -1;
      float v1 = 0.f, v2 = 0.f;
#pragma unroll
      for (int c = 0; c < C1; ++c) {
        const float top = q[0][c] + (q[1][c] - q[0][c]) * xlp;
        const float bot = q[2][c] + (q[3][c] - q[2][c]) * xlp;
        const float v = top + (bot - top) * ylp;
        if (i1 < 0 || v > v1) { i2 = i1; v2 = v1; i1 = c; v1 = v; }
        else if (i2 < 0 || v > v2) { i2 = c; v2 = v; }
      }
      d = d == C1 - 1 ? i2 : i1;
    } else if (a.replace_voids) {
      // top_k(l1_probabilities, 2) (stable: equal values keep the lower index first);
      // l1_probabilities keep C1 channels (the segment-sum remap does not apply to them)
      int d2 = -1;
      float b2 = 0.f;
#pragma unroll
      for (int c = 0; c < C1; ++c)
        if (c != d1 && (d2 < 0 || p[c] > b2)) { b2 = p[c]; d2 = c; }
      d = d == C1 - 1 ? d2 : d1;
    }
    a.out[id] = d;
  }
}
// The model's full-resolution `predictions` (hierarchical.py:84-130), materialised on demand:
// per network-resolution pixel the align-corners bilinear logits of the three heads, their
// softmax, per-head argmax and the fused common-cid decision. Same arithmetic as the loss
// head / eval kernel (one thread per pixel, the 4 low-res source cells read through L2); every
// output is optional. Stores are per pixel runs of CT floats (float4 where CT % 4 == 0).
template <int C1, int C2, int C3>
__global__ __launch_bounds__(256) void full_predictions_kernel(FullPredArgs a, LossTables t) {
  constexpr int CT = C1 + C2 + C3;
  const long total = (long)a.N * a.H * a.W;
  for (long id = (long)blockIdx.x * blockDim.x + threadIdx.x; id < total;
       id += (long)gridDim.x * blockDim.x) {
    const int w = (int)(id % a.W);
    const int h = (int)((id / a.W) % a.H);
    const int n = (int)(id / ((long)a.W * a.H));
    int ylo, yhi, xlo, xhi;
    float yl, xl;
    lerp_of(h, a.Hl, a.H, ylo, yhi, yl);
    lerp_of(w, a.Wl, a.W, xlo, xhi, xl);
    const float* base = a.logits + (size_t)n * a.Hl * a.Wl * a.ldl;
    const float* tl = base + ((size_t)ylo * a.Wl + xlo) * a.ldl;
    const float* tr = base + ((size_t)ylo * a.Wl + xhi) * a.ldl;
    const float* bl = base + ((size_t)yhi * a.Wl + xlo) * a.ldl;
    const float* br = base + ((size_t)yhi * a.Wl + xhi) * a.ldl;
    float p[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      float top = tl[c] + (tr[c] - tl[c]) * xl;
      float bot = bl[c] + (br[c] - bl[c]) * xl;
      p[c] = top + (bot - top) * yl;
    }
    auto store = [&](float* dst) {
      float* o = dst + (size_t)id * CT;
      if constexpr (CT % 4 == 0) {
#pragma unroll
        for (int c = 0; c < CT; c += 4)
          *reinterpret_cast<float4*>(o + c) = make_float4(p[c], p[c + 1], p[c + 2], p[c + 3]);
      } else {
#pragma unroll
        for (int c = 0; c < CT; ++c) o[c] = p[c];
      }
    };
    if (a.logits_out) store(a.logits_out);
    auto softmax = [&](int c0, int nc) {
      float m = p[c0];
#pragma unroll
      for (int c = 1; c < nc; ++c) m = fmaxf(m, p[c0 + c]);
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < nc; ++c) { p[c0 + c] = __expf(p[c0 + c] - m); s += p[c0 + c]; }
      const float rs = 1.f / s;
#pragma unroll
      for (int c = 0; c < nc; ++c) p[c0 + c] = p[c0 + c] * rs;
    };
    softmax(0, C1);
    softmax(C1, C2);
    softmax(C1 + C2, C3);
    if (a.probs_out) store(a.probs_out);
    auto argmax = [&](int c0, int nc) {   // tf.argmax: first maximum
      int b = 0;
      float bv = p[c0];
#pragma unroll
      for (int c = 1; c < nc; ++c) if (p[c0 + c] > bv) { bv = p[c0 + c]; b = c; }
      return b;
    };
    const int d1 = argmax(0, C1), dv = argmax(C1, C2), dh = argmax(C1 + C2, C3);
    if (a.head_decs_out) {
      int* o = a.head_decs_out + (size_t)id * 3;
      o[0] = d1; o[1] = dv; o[2] = dh;
    }
    if (a.decs_out)
      a.decs_out[id] = d1 == t.cid_l1_vehicle ? t.veh_to_common[dv]
                     : d1 == t.cid_l1_human ? t.hum_to_common[dh] : t.l1_to_common[d1];
  }
}

__global__ void confusion_global_kernel(const int* __restrict__ lab, const int* __restrict__ dec,
                                        long n, int nc, int* cm) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    int l = lab[i], d = dec[i];
    if (l >= 0 && l < nc && d >= 0 && d < nc) atomicAdd(&cm[l * nc + d], 1);
  }
}

}  // namespace

int loss_head_blocks(int N, int Hl, int Wl) {
  return N * ((Hl + LA - 1) / LA) * ((Wl + LB - 1) / LB);
}

bool loss_head_yf(int W, int Wl) {
  // y-first accumulation when every block's full-resolution columns fit one chunk: (LB + 1)
  // low-res cells of (W - 1) / (Wl - 1) columns each, plus the two boundary columns
  const double span = Wl > 1 ? (LB + 1) * (double)(W - 1) / (double)(Wl - 1) + 3.0 : 1e9;
  return LOSS_YF && span <= THREADS;
}

hipError_t launch_loss_head(const LossArgs& a, const LossTables& t, hipStream_t s) {
  dim3 g(loss_head_blocks(a.N, a.Hl, a.Wl));
  const bool yf = loss_head_yf(a.W, a.Wl);
  if (t.c1 == 14 && t.c2 == 7 && t.c3 == 3 && yf)
    hipLaunchKernelGGL((loss_head_kernel<14, 7, 3, 1>), g, dim3(THREADS), 0, s, a, t);
  else if (t.c1 == 14 && t.c2 == 7 && t.c3 == 3)
    hipLaunchKernelGGL((loss_head_kernel<14, 7, 3>), g, dim3(THREADS), 0, s, a, t);
  else if (t.c1 == 53 && t.c2 == 12 && t.c3 == 5)
    hipLaunchKernelGGL((loss_head_kernel<53, 12, 5>), g, dim3(THREADS), 0, s, a, t);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_loss_finalize(const float* part, int nblocks, const LossTables& t, int ldl,
                                float loss_scale,
                                float* out, float* dzscale, hipStream_t s) {
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(256), 0, s, part, nblocks, t.c1, t.c2,
                     t.c3, ldl, out, dzscale, loss_scale);
  return hipGetLastError();
}

hipError_t launch_confusion(const int* labels, const int* decisions, long n, int num_classes,
                            int* cm, hipStream_t s) {
  if (num_classes <= 0 || num_classes > 256) return hipErrorInvalidValue;
  long g = (n + 255) / 256;
  if (num_classes > 64) {   // Vistas (66 classes): the histogram does not fit the LDS tile
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(confusion_global_kernel, dim3((int)g), dim3(256), 0, s, labels, decisions,
                       n, num_classes, cm);
    return hipGetLastError();
  }
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(confusion_kernel, dim3((int)g), dim3(256), 0, s, labels, decisions, n,
                     num_classes, cm);
  return hipGetLastError();
}

hipError_t launch_eval_decisions(const EvalArgs& a, const LossTables& t, hipStream_t s) {
  const long total = (long)a.N * a.Ho * a.Wo;
  if (total <= 0) return hipSuccess;
  long g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  if (t.c1 == 14 && t.c2 == 7 && t.c3 == 3)
    hipLaunchKernelGGL((eval_decisions_kernel<14, 7, 3>), dim3((int)g), dim3(256), 0, s, a, t);
  else if (t.c1 == 53 && t.c2 == 12 && t.c3 == 5)
    hipLaunchKernelGGL((eval_decisions_kernel<53, 12, 5>), dim3((int)g), dim3(256), 0, s, a, t);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_full_predictions(const FullPredArgs& a, const LossTables& t, hipStream_t s) {
  const long total = (long)a.N * a.H * a.W;
  if (total <= 0) return hipSuccess;
  long g = (total + 255) / 256;
  if (g > 16384) g = 16384;
  if (t.c1 == 14 && t.c2 == 7 && t.c3 == 3)
    hipLaunchKernelGGL((full_predictions_kernel<14, 7, 3>), dim3((int)g), dim3(256), 0, s, a, t);
  else if (t.c1 == 53 && t.c2 == 12 && t.c3 == 5)
    hipLaunchKernelGGL((full_predictions_kernel<53, 12, 5>), dim3((int)g), dim3(256), 0, s, a, t);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}
