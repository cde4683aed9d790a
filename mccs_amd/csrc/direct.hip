// direct.hip — the direct (two-shot) AllReduce kernels (direct_kernel.h), one
// per (dtype, op), and the host's lookup.
#include "direct_kernel.h"

namespace mccs {

template <int OP>
static const void* direct_for_op(int dtype) {
  switch (dtype) {
    case mccsInt8: return (const void*)&direct_kernel<mccsInt8, OP>;
    case mccsUint8: return (const void*)&direct_kernel<mccsUint8, OP>;
    case mccsInt32: return (const void*)&direct_kernel<mccsInt32, OP>;
    case mccsUint32: return (const void*)&direct_kernel<mccsUint32, OP>;
    case mccsInt64: return (const void*)&direct_kernel<mccsInt64, OP>;
    case mccsUint64: return (const void*)&direct_kernel<mccsUint64, OP>;
    case mccsFloat16: return (const void*)&direct_kernel<mccsFloat16, OP>;
    case mccsFloat32: return (const void*)&direct_kernel<mccsFloat32, OP>;
    case mccsFloat64: return (const void*)&direct_kernel<mccsFloat64, OP>;
    case mccsBfloat16: return (const void*)&direct_kernel<mccsBfloat16, OP>;
    default: return nullptr;
  }
}

const void* direct_kernel_ptr(int dtype, int op) {
  switch (op) {
    case OpSum: return direct_for_op<OpSum>(dtype);
    case OpProd: return direct_for_op<OpProd>(dtype);
    case OpMax: return direct_for_op<OpMax>(dtype);
    case OpMin: return direct_for_op<OpMin>(dtype);
    default: return nullptr;
  }
}

}  // namespace mccs

// Phase timeline of the latest direct launch (-DMCCS_DIRECT_TRACE builds,
// tools/direct_trace.py): out[slot * kDtEvents + event] = s_memrealtime of workgroup
// 0 of rank slot `slot` (direct_kernel.h kDt*); cleared after reading.
// Returns the words written, or -1 when this build has no trace.
extern "C" int mccs_direct_trace(unsigned long long* out, int max_words) {
#ifdef MCCS_DIRECT_TRACE
  constexpr int kWords = MCCS_MULTI_MAX_RANKS * mccs::kDtEvents;
  if (max_words < kWords) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mccs::g_dtrace), sizeof(unsigned long long) * kWords, 0,
                          hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  static unsigned long long zero[kWords];
  (void)hipMemcpyToSymbol(HIP_SYMBOL(mccs::g_dtrace), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
  return kWords;
#else
  (void)out;
  (void)max_words;
  return -1;
#endif
}
