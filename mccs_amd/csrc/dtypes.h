// dtypes.h — element types and reduction functors for the gfx950 kernels.
//
// Semantics follow the reference functors (src/collectives/src/reduce_kernel.h):
//   FuncSum/FuncProd  x+y, x*y in T, integers wrap (:16-30, :72-103 for int8/uint8)
//   FuncMax/FuncMin   (x<y)?y:x / (x<y)?x:y for integers, float, double (:32-46)
//   half / bfloat16   computed in binary32 and rounded once to nearest even; this
//                     is bit-identical to __hadd2/__hmul2 (:237-259, :287-309)
//                     because binary32 has >= 2p+2 bits for p = 11 and p = 8;
//                     Max/Min use fmaxf/fminf then round (:338-404).
// Everything operates on 16-byte packs (one global_load_dwordx4 per lane).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mccs_devcomm.h"

namespace mccs {

enum RedOp : int { OpSum = mccsDevSum, OpProd = mccsDevProd, OpMax = mccsDevMax, OpMin = mccsDevMin };

using u32x4 = uint32_t __attribute__((ext_vector_type(4)));
using f32x4 = float __attribute__((ext_vector_type(4)));
using f64x2 = double __attribute__((ext_vector_type(2)));
using h16x8 = _Float16 __attribute__((ext_vector_type(8)));
using i8x16 = int8_t __attribute__((ext_vector_type(16)));
using u8x16 = uint8_t __attribute__((ext_vector_type(16)));
using i32x4 = int32_t __attribute__((ext_vector_type(4)));
using i64x2 = int64_t __attribute__((ext_vector_type(2)));
using u64x2 = uint64_t __attribute__((ext_vector_type(2)));
using bf16x2 = __bf16 __attribute__((ext_vector_type(2)));
using f32x2 = float __attribute__((ext_vector_type(2)));

// Storage type for each mccsDevDataType_t.
template <int DT> struct Elem;
template <> struct Elem<mccsInt8> { using T = int8_t; };
template <> struct Elem<mccsUint8> { using T = uint8_t; };
template <> struct Elem<mccsInt32> { using T = int32_t; };
template <> struct Elem<mccsUint32> { using T = uint32_t; };
template <> struct Elem<mccsInt64> { using T = int64_t; };
template <> struct Elem<mccsUint64> { using T = uint64_t; };
template <> struct Elem<mccsFloat16> { using T = _Float16; };
template <> struct Elem<mccsFloat32> { using T = float; };
template <> struct Elem<mccsFloat64> { using T = double; };
template <> struct Elem<mccsBfloat16> { using T = uint16_t; };  // raw bits

template <int DT> constexpr int kElemBytes = (int)sizeof(typename Elem<DT>::T);
template <int DT> constexpr int kPackElems = 16 / kElemBytes<DT>;

__host__ __device__ constexpr int elem_bytes(int dt) {
  return (dt == mccsInt8 || dt == mccsUint8) ? 1
         : (dt == mccsFloat16 || dt == mccsBfloat16) ? 2
         : (dt == mccsInt32 || dt == mccsUint32 || dt == mccsFloat32) ? 4
         : 8;
}

// ---- scalar functor: fn(x, y) in T ------------------------------------------
template <typename T, int OP>
__device__ __forceinline__ T int_op(T x, T y) {
  using U = typename std::make_unsigned<T>::type;
  if constexpr (OP == OpSum) return (T)((U)x + (U)y);
  else if constexpr (OP == OpProd) return (T)((U)x * (U)y);
  else if constexpr (OP == OpMax) return (x < y) ? y : x;
  else return (x < y) ? x : y;
}

template <int OP>
__device__ __forceinline__ float f32_op_fmax(float x, float y) {
  if constexpr (OP == OpSum) return x + y;
  else if constexpr (OP == OpProd) return x * y;
  else if constexpr (OP == OpMax) return fmaxf(x, y);
  else return fminf(x, y);
}

__device__ __forceinline__ float bf16_lo(uint32_t w) { return __builtin_bit_cast(float, w << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t w) { return __builtin_bit_cast(float, w & 0xffff0000u); }
// two binary32 -> packed bfloat16x2, round to nearest even (v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  f32x2 f = {lo, hi};
  bf16x2 b = __builtin_convertvector(f, bf16x2);
  return __builtin_bit_cast(uint32_t, b);
}

template <int DT, int OP>
__device__ __forceinline__ typename Elem<DT>::T scalar_op(typename Elem<DT>::T x,
                                                          typename Elem<DT>::T y) {
  using T = typename Elem<DT>::T;
  if constexpr (DT == mccsFloat16) {
    float r = f32_op_fmax<OP>((float)x, (float)y);
    return (_Float16)r;
  } else if constexpr (DT == mccsBfloat16) {
    float r = f32_op_fmax<OP>(bf16_lo(x), bf16_lo(y));
    return (T)(pack_bf16x2(r, 0.f) & 0xffffu);
  } else if constexpr (DT == mccsFloat32 || DT == mccsFloat64) {
    if constexpr (OP == OpSum) return x + y;
    else if constexpr (OP == OpProd) return x * y;
    else if constexpr (OP == OpMax) return (x < y) ? y : x;
    else return (x < y) ? x : y;
  } else {
    return int_op<T, OP>(x, y);
  }
}

// ---- 16-byte pack functor: lane-wise fn(a, b) -------------------------------
template <int DT, int OP>
__device__ __forceinline__ u32x4 pack_op(u32x4 a, u32x4 b) {
  if constexpr (DT == mccsFloat32) {
    f32x4 x = __builtin_bit_cast(f32x4, a), y = __builtin_bit_cast(f32x4, b), r;
    if constexpr (OP == OpSum) r = x + y;
    else if constexpr (OP == OpProd) r = x * y;
    else {
#pragma unroll
      for (int i = 0; i < 4; ++i) r[i] = scalar_op<DT, OP>(x[i], y[i]);
    }
    return __builtin_bit_cast(u32x4, r);
  } else if constexpr (DT == mccsFloat16) {
    h16x8 x = __builtin_bit_cast(h16x8, a), y = __builtin_bit_cast(h16x8, b), r;
    if constexpr (OP == OpSum) r = x + y;        // v_pk_add_f16, RNE == __hadd2
    else if constexpr (OP == OpProd) r = x * y;  // v_pk_mul_f16, RNE == __hmul2
    else {
#pragma unroll
      for (int i = 0; i < 8; ++i) r[i] = scalar_op<DT, OP>(x[i], y[i]);
    }
    return __builtin_bit_cast(u32x4, r);
  } else if constexpr (DT == mccsBfloat16) {
    u32x4 r;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      r[i] = pack_bf16x2(f32_op_fmax<OP>(bf16_lo(a[i]), bf16_lo(b[i])),
                         f32_op_fmax<OP>(bf16_hi(a[i]), bf16_hi(b[i])));
    return r;
  } else if constexpr (DT == mccsFloat64) {
    f64x2 x = __builtin_bit_cast(f64x2, a), y = __builtin_bit_cast(f64x2, b), r;
#pragma unroll
    for (int i = 0; i < 2; ++i) r[i] = scalar_op<DT, OP>(x[i], y[i]);
    return __builtin_bit_cast(u32x4, r);
  } else if constexpr (DT == mccsInt8 || DT == mccsUint8) {
    using V = std::conditional_t<DT == mccsInt8, i8x16, u8x16>;
    V x = __builtin_bit_cast(V, a), y = __builtin_bit_cast(V, b), r;
    if constexpr (OP == OpSum) {
      u8x16 s = __builtin_bit_cast(u8x16, x) + __builtin_bit_cast(u8x16, y);
      return __builtin_bit_cast(u32x4, s);
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) r[i] = scalar_op<DT, OP>(x[i], y[i]);
      return __builtin_bit_cast(u32x4, r);
    }
  } else if constexpr (DT == mccsInt32 || DT == mccsUint32) {
    if constexpr (OP == OpSum) return a + b;
    else if constexpr (OP == OpProd) return a * b;
    else {
      using V = std::conditional_t<DT == mccsInt32, i32x4, u32x4>;
      V x = __builtin_bit_cast(V, a), y = __builtin_bit_cast(V, b), r;
#pragma unroll
      for (int i = 0; i < 4; ++i) r[i] = scalar_op<DT, OP>(x[i], y[i]);
      return __builtin_bit_cast(u32x4, r);
    }
  } else {  // int64 / uint64
    using V = std::conditional_t<DT == mccsInt64, i64x2, u64x2>;
    V x = __builtin_bit_cast(V, a), y = __builtin_bit_cast(V, b), r;
#pragma unroll
    for (int i = 0; i < 2; ++i) r[i] = scalar_op<DT, OP>(x[i], y[i]);
    return __builtin_bit_cast(u32x4, r);
  }
}

// ---- dispatch helpers (host + device) ----------------------------------------
#define MCCS_FOR_EACH_DTYPE(X) \
  X(mccsInt8) X(mccsUint8) X(mccsInt32) X(mccsUint32) X(mccsInt64) X(mccsUint64) \
  X(mccsFloat16) X(mccsFloat32) X(mccsFloat64) X(mccsBfloat16)

}  // namespace mccs
