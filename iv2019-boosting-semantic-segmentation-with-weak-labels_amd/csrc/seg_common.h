// Common device/host helpers for the MI355X (gfx950) segmentation training path.
// Layout convention everywhere: NHWC activations with a pixel stride `ld` (>= C) so that
// channel slices of a concat buffer are first-class tensors; weights [Co][KH][KW][Ci].
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <stddef.h>
#include <type_traits>

typedef uint16_t bf16_t;  // storage type of bf16 activations/weights

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

typedef _Float16 f16_t;   // storage type of fp16 activations/weights (BASELINE config C5)
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));

enum SegDType { SEG_F32 = 0, SEG_BF16 = 1, SEG_F16 = 2 };
// 16-bit storage (bf16 or fp16): the same kernels, data movement and fp32 accumulation; only
// the MFMA opcode and the element conversions differ
static inline bool seg_half(int dt) { return dt == SEG_BF16 || dt == SEG_F16; }

// ---- scalar conversions ------------------------------------------------------------
__device__ __host__ __forceinline__ float bf2f(bf16_t v) {
  uint32_t u = ((uint32_t)v) << 16;
  float f;
  __builtin_memcpy(&f, &u, 4);
  return f;
}
__device__ __forceinline__ bf16_t f2bf(float f) {
  // plain cast: hipcc emits v_cvt_pk_bf16_f32 (round-to-nearest-even, NaN preserved)
  __bf16 b = (__bf16)f;
  bf16_t r;
  __builtin_memcpy(&r, &b, 2);
  return r;
}

template <typename T> struct TypeOps;
template <> struct TypeOps<float> {
  static __device__ __forceinline__ float to_f(float v) { return v; }
  static __device__ __forceinline__ float from_f(float v) { return v; }
};
template <> struct TypeOps<bf16_t> {
  static __device__ __forceinline__ float to_f(bf16_t v) { return bf2f(v); }
  static __device__ __forceinline__ bf16_t from_f(float v) { return f2bf(v); }
};
template <> struct TypeOps<f16_t> {
  static __device__ __forceinline__ float to_f(f16_t v) { return (float)v; }
  static __device__ __forceinline__ f16_t from_f(float v) { return (f16_t)v; }   // RNE
};
// two values -> one packed 16-bit pair (lo in bits 0-15) by ONE v_cvt_pk_bf16_f32 /
// v_cvt_pk_f16_f32 (RNE, as the scalar casts): converting the halves separately costs two
// conversions plus a shift and an SDWA or per pair (the conv epilogues pack 128 values per lane)
typedef float pk_f32x2_t __attribute__((ext_vector_type(2)));
template <typename E> __device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  typedef __attribute__((ext_vector_type(2))) typename std::conditional<std::is_same<E, f16_t>::value, _Float16, __bf16>::type h2_t;
  const h2_t r = __builtin_convertvector((pk_f32x2_t){lo, hi}, h2_t);
  uint32_t u;
  __builtin_memcpy(&u, &r, 4);
  return u;
}

template <typename T> __device__ __forceinline__ float ldf(const T* p) { return TypeOps<T>::to_f(*p); }
template <typename T> __device__ __forceinline__ void stf(T* p, float v) { *p = TypeOps<T>::from_f(v); }

// ---- 8-element vector load/store to/from float[8] -----------------------------------
template <typename T> struct Vec8;
template <> struct Vec8<float> {
  static __device__ __forceinline__ void load(const float* p, float* o) {
    float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* p, const float* v) {
    *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
    *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
};
template <> struct Vec8<bf16_t> {
  static __device__ __forceinline__ void load(const bf16_t* p, float* o) {
    uint4 u = *(const uint4*)p;
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[2 * i] = bf2f((bf16_t)(w[i] & 0xffff));
      o[2 * i + 1] = bf2f((bf16_t)(w[i] >> 16));
    }
  }
  static __device__ __forceinline__ void store(bf16_t* p, const float* v) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = pack2<bf16_t>(v[2 * i], v[2 * i + 1]);
    *(uint4*)p = make_uint4(w[0], w[1], w[2], w[3]);
  }
};

template <> struct Vec8<f16_t> {
  static __device__ __forceinline__ void load(const f16_t* p, float* o) {
    const f16x8_t v = *(const f16x8_t*)p;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (float)v[i];
  }
  static __device__ __forceinline__ void store(f16_t* p, const float* v) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = pack2<f16_t>(v[2 * i], v[2 * i + 1]);
    *(uint4*)p = make_uint4(w[0], w[1], w[2], w[3]);
  }
};

// 8 values -> one 16-byte non-temporal store (conv outputs: written once, read by the next
// kernel from HBM anyway; the streaming hint lets the epilogue's stores drain sooner)
template <typename E>
__device__ __forceinline__ void store8_nt(E* p, const float* v) {
  typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
  if constexpr (sizeof(E) == 4) {
    typedef float f32x4v_t __attribute__((ext_vector_type(4)));
    const f32x4v_t a = {v[0], v[1], v[2], v[3]}, b = {v[4], v[5], v[6], v[7]};
    __builtin_nontemporal_store(a, (f32x4v_t*)p);
    __builtin_nontemporal_store(b, (f32x4v_t*)(p + 4));
  } else {
    u32x4_t w;
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = pack2<E>(v[2 * i], v[2 * i + 1]);
    __builtin_nontemporal_store(w, (u32x4_t*)p);
  }
}


// 16-bit element traits of the MFMA kernels: fragment vector type, the 16x16x32 MFMA, and
// the unpack of a raw 16-byte chunk
template <typename E> struct Half;
template <> struct Half<bf16_t> {
  typedef bf16x8_t V;
  static __device__ __forceinline__ f32x4_t mma(V a, V b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ void unpack(const uint4 u, float* o) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) { o[2 * i] = bf2f((bf16_t)(w[i] & 0xffff)); o[2 * i + 1] = bf2f((bf16_t)(w[i] >> 16)); }
  }
};
template <> struct Half<f16_t> {
  typedef f16x8_t V;
  static __device__ __forceinline__ f32x4_t mma(V a, V b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ void unpack(const uint4 u, float* o) {
    f16x8_t h;
    __builtin_memcpy(&h, &u, 16);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (float)h[i];
  }
};

// ---- wave reductions (wave64) -------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

#define SEG_CHECK_HIP(expr)                                                      \
  do {                                                                           \
    hipError_t _e = (expr);                                                      \
    if (_e != hipSuccess) return seg_fail(__FILE__, __LINE__, hipGetErrorString(_e)); \
  } while (0)

static inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }
