// reduce.hip — device-resident chunk reduce / reduce-copy over a whole MI355X.
//
// C-ABI: mccs_hip_reduce / mccs_hip_reduce_copy (include/mccs_hip.h).  This is
// the standalone form of the reference's per-chunk ReduceOrCopyMulti
// (src/collectives/src/common_kernel.h:485-685): y = src0 (op) src1 (op) ...
// stored to every dst, in the element type (reduce_kernel.h functors).  The
// reference runs that loop inside 1-2 ring blocks; here it is a full-chip,
// HBM-bound streaming kernel (bytes per element = (nsrcs + ndsts) * sizeof(T),
// 0.083 flop/B for fp32 2->1: no MFMA).
//
// Two main-loop designs, selected at run time (mccs_hip_reduce_tune):
//   REG  register streaming: each lane keeps U 16-byte packs per source in
//        flight (global_load_dwordx4), packed VALU op, global_store_dwordx4.
//   LDS  LDS-DMA staging: each wave streams its sources with
//        global_load_lds_dwordx4 into an S-stage ring in LDS (S-1 tiles in
//        flight per wave, counted s_waitcnt vmcnt), reads its own lanes back
//        with ds_read_b128, applies the op and stores.  Bytes in flight are
//        bounded by LDS (160 KiB/CU) instead of VGPRs.
// Grid: persistent, blocks_per_cu * 256 CUs, grid-stride over tiles.
// Default: LDS with nt DMA reads (the fastest from HBM).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <cstring>

#include "dtypes.h"
#include "mccs_hip.h"
#include "lds_dma.h"
#include "reduce_copy.h"

namespace mccs {

constexpr int kMaxSrcs = MCCS_REDUCE_MAX_SRCS;
constexpr int kMaxDsts = MCCS_REDUCE_MAX_DSTS;

struct ReduceArgs {
  const void* srcs[kMaxSrcs];
  void* dsts[kMaxDsts];
  int nsrcs;
  int ndsts;
  int64_t count;
};

// ---------------------------------------------------------------------------
// REG: NS/ND > 0 are compile-time source/destination counts; 0 = runtime.
// MAP bit 0 clear: tiles grid-strided over blocks (the chip sweeps one
// contiguous window); set: each block owns a contiguous run of tiles.
// MAP bit 1: wave-contiguous rows (wave w reads U consecutive 1 KiB rows of
// the tile) instead of block-strided packs (pack u of thread t at u*256+t).
template <int DT, int OP, int NS, int ND, int U, int LDP, int STP, int MAP = 0>
__global__ void __launch_bounds__(256) reduce_reg_kernel(ReduceArgs a) {
  using T = typename Elem<DT>::T;
  constexpr int PACK = kPackElems<DT>;
  constexpr int B = 256;
  const int nsrcs = NS > 0 ? NS : a.nsrcs;
  const int ndsts = ND > 0 ? ND : a.ndsts;
  constexpr int MS = NS > 0 ? NS : kMaxSrcs;
  constexpr int MD = ND > 0 ? ND : kMaxDsts;
  const int64_t npack = a.count / PACK;
  const int64_t tile = (int64_t)B * U;
  const int tid = threadIdx.x;

  constexpr bool BLOCKED = MAP & 1, ROWS = MAP & 2;
  constexpr int S = ROWS ? 64 : B;  // pack stride between a thread's U packs
  const int lt = ROWS ? (tid >> 6) * 64 * U + (tid & 63) : tid;
  const int64_t ntiles = (npack + tile - 1) / tile;
  const int64_t per = BLOCKED ? (ntiles + gridDim.x - 1) / gridDim.x : 0;
  const int64_t t0 = BLOCKED ? (int64_t)blockIdx.x * per : blockIdx.x;
  const int64_t t1 = BLOCKED ? (t0 + per < ntiles ? t0 + per : ntiles) : ntiles;
  const int64_t tstep = BLOCKED ? 1 : gridDim.x;
  for (int64_t t = t0; t < t1; t += tstep) {
    const int64_t base = t * tile + lt;
    if ((t + 1) * tile <= npack) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = ld16<LDP>((const u32x4*)a.srcs[0] + base + u * S);
#pragma unroll
      for (int s = 1; s < MS; ++s) {
        if (s < nsrcs) {
          u32x4 w[U];
#pragma unroll
          for (int u = 0; u < U; ++u) w[u] = ld16<LDP>((const u32x4*)a.srcs[s] + base + u * S);
#pragma unroll
          for (int u = 0; u < U; ++u) v[u] = pack_op<DT, OP>(v[u], w[u]);
        }
      }
#pragma unroll
      for (int d = 0; d < MD; ++d) {
        if (d < ndsts) {
#pragma unroll
          for (int u = 0; u < U; ++u) st16<STP>((u32x4*)a.dsts[d] + base + u * S, v[u]);
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t p = base + u * S;
        if (p < npack) {
          u32x4 v = ld16<LDP>((const u32x4*)a.srcs[0] + p);
#pragma unroll
          for (int s = 1; s < MS; ++s)
            if (s < nsrcs) v = pack_op<DT, OP>(v, ld16<LDP>((const u32x4*)a.srcs[s] + p));
#pragma unroll
          for (int d = 0; d < MD; ++d)
            if (d < ndsts) st16<STP>((u32x4*)a.dsts[d] + p, v);
        }
      }
    }
  }
  // < 16-byte tail: last block, typed scalar
  if (blockIdx.x == gridDim.x - 1) {
    for (int64_t e = npack * PACK + tid; e < a.count; e += B) {
      T v = ((const T*)a.srcs[0])[e];
      for (int s = 1; s < nsrcs; ++s) v = scalar_op<DT, OP>(v, ((const T*)a.srcs[s])[e]);
      for (int d = 0; d < ndsts; ++d) ((T*)a.dsts[d])[e] = v;
    }
  }
}

// Unaligned pointers: typed grid-stride loop (reference ReduceCopyMulti path).
template <int DT, int OP>
__global__ void __launch_bounds__(256) reduce_scalar_kernel(ReduceArgs a) {
  using T = typename Elem<DT>::T;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < a.count; e += stride) {
    T v = ((const T*)a.srcs[0])[e];
    for (int s = 1; s < a.nsrcs; ++s) v = scalar_op<DT, OP>(v, ((const T*)a.srcs[s])[e]);
    for (int d = 0; d < a.ndsts; ++d) ((T*)a.dsts[d])[e] = v;
  }
}

// ---------------------------------------------------------------------------
// LDS: 2 sources -> 1 destination, per-wave LDS-DMA ring of S stages.
// A wave tile = 64 lanes x U packs per source = U KiB per source.
// wait until at most nd*G + ns*U vector-memory ops are outstanding
// (nd, ns < S <= 4; vmcnt immediates must be compile-time constants)
template <int G, int U, int S>
__device__ __forceinline__ void wait_younger(int nd, int ns) {
  static_assert(S >= 2 && S <= 4, "stages");
  static_assert((S - 1) * (G + U) < 64, "vmcnt range");
#define MCCS_WY(ND, NS) \
  case (ND) * 4 + (NS): wait_vmcnt<((ND) < S && (NS) < S) ? (ND) * G + (NS) * U : 0>(); break;
  switch (nd * 4 + ns) {
    MCCS_WY(0, 0) MCCS_WY(0, 1) MCCS_WY(0, 2) MCCS_WY(0, 3)
    MCCS_WY(1, 0) MCCS_WY(1, 1) MCCS_WY(1, 2) MCCS_WY(1, 3)
    MCCS_WY(2, 0) MCCS_WY(2, 1) MCCS_WY(2, 2) MCCS_WY(2, 3)
    MCCS_WY(3, 0) MCCS_WY(3, 1) MCCS_WY(3, 2)
    default: wait_vmcnt<0>(); break;
  }
#undef MCCS_WY
}

#ifdef MCCS_REDUCE_TRACE
// A/B builds only (tools/reduce_skew.py): per wave of the latest launch,
// {entry, exit} s_memrealtime and the XCC the wave ran on.
constexpr int kRTraceWaves = 8192;
__device__ unsigned long long g_rtrace[kRTraceWaves * 3];
__device__ __forceinline__ void rtrace(int gw, int k) {
  if ((threadIdx.x & 63) != 0 || gw >= kRTraceWaves) return;
  g_rtrace[gw * 3 + k] = __builtin_amdgcn_s_memrealtime();
  if (k == 1) g_rtrace[gw * 3 + 2] = __builtin_amdgcn_s_getreg((20 /* HW_REG_XCC_ID */) | (0 << 6) | (15 << 11)) & 15;
}
#define MCCS_RTRACE(gw, k) rtrace((int)(gw), k)
#else
#define MCCS_RTRACE(gw, k) ((void)0)
#endif

template <int DT, int OP, int U, int S, int W, int LDP, int STP>
__global__ void __launch_bounds__(W * 64) reduce_lds_kernel(ReduceArgs a) {
  constexpr int PACK = kPackElems<DT>;
  constexpr int G = 2 * U;        // LDS-DMA instructions per wave tile (2 sources)
  constexpr int STAGE_BYTES = G * 1024;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t wave_lds =
      (uint32_t)(uintptr_t)smem + (uint32_t)(wave * S * STAGE_BYTES);
  const int64_t npack = a.count / PACK;
  const int64_t wtile = 64 * U;
  const int64_t ntiles = (npack + wtile - 1) / wtile;
  const int64_t gw = (int64_t)blockIdx.x * W + wave;  // global wave id
  const int64_t nw = (int64_t)gridDim.x * W;
  const u32x4* s0 = (const u32x4*)a.srcs[0];
  const u32x4* s1 = (const u32x4*)a.srcs[1];
  u32x4* d0 = (u32x4*)a.dsts[0];
  MCCS_RTRACE(gw, 0);

  auto issue = [&](int64_t tile, int stage) {
    const uint32_t base = wave_lds + (uint32_t)(stage * STAGE_BYTES);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int64_t p = tile * wtile + u * 64 + lane;
      p = p < npack ? p : npack - 1;  // clamp: partial last tile re-reads a valid pack
      glds16<LDP>(s0 + p, base + u * 1024);
      glds16<LDP>(s1 + p, base + (U + u) * 1024);
    }
  };

  // k-th tile of this wave is gw + k*nw
  int64_t nmine = gw < ntiles ? (ntiles - gw + nw - 1) / nw : 0;
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nmine) issue(gw + s * nw, s);

  for (int64_t k = 0; k < nmine; ++k) {
    const int stage = (int)(k % S);
    const int64_t ahead = k + S - 1;
    if (ahead < nmine) issue(gw + ahead * nw, (int)(ahead % S));
    // vmcnt retires in issue order (loads, stores and LDS-DMA together), so
    // "tile k landed" = at most (younger DMA groups)*G + (younger store
    // groups)*U operations outstanding.  Younger DMA: tiles k+1..k+S-1 that
    // exist; younger stores: tiles max(0,k-S+1)..k-1 (stored after tile k's
    // DMA was issued).  Every tile issues exactly U stores (clamped below).
    const int nd = (int)((nmine - 1 - k) < (S - 1) ? (nmine - 1 - k) : (S - 1));
    const int ns = (int)(k < (S - 1) ? k : (S - 1));
    wait_younger<G, U, S>(nd, ns);
    const char* st = smem + (size_t)(wave * S + stage) * STAGE_BYTES;
    const int64_t tbase = (gw + k * nw) * wtile;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      u32x4 x = *(const u32x4*)(st + u * 1024 + lane * 16);
      u32x4 y = *(const u32x4*)(st + (U + u) * 1024 + lane * 16);
      int64_t p = tbase + u * 64 + lane;
      // lanes past the end recompute and rewrite the last pack (same value,
      // from the same clamped loads) so the store count stays U per tile
      p = p < npack ? p : npack - 1;
      st16<STP>(d0 + p, pack_op<DT, OP>(x, y));
    }
  }
  MCCS_RTRACE(gw, 1);
  if (blockIdx.x == gridDim.x - 1) {
    using T = typename Elem<DT>::T;
    for (int64_t e = npack * PACK + threadIdx.x; e < a.count; e += W * 64) {
      T v = scalar_op<DT, OP>(((const T*)a.srcs[0])[e], ((const T*)a.srcs[1])[e]);
      ((T*)a.dsts[0])[e] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// Run-time configuration (process-wide; set before launches).  Defaults are
// the fastest measured on MI355X in the regime bench.py times (50+
// back-to-back launches, inputs streamed from HBM; bench.py --sweep-cfgs
// --sweep-launches 60 on three boxes): the LDS-DMA loop, strict double
// buffering (2 stages), 4 KiB per source per wave tile, 4 waves, one block
// per CU, non-temporal DMA reads, write-through (sc1) stores.  It ties the
// 3-stage nt-store ring and beats the best REG loop by ~1.2 %; the 3-stage
// ring with sc1 stores, best in 12-launch bursts, is 1.3 % slower sustained.
// Without nt on the DMA reads the loop streams 5.9 TB/s.  See DESIGN.md §3.1.
struct ReduceTune {
  int variant = MCCS_REDUCE_VARIANT_LDS;
  int unroll = 4;  // LDS: 4 KiB per source per wave tile
  int policy = 4;  // nt LDS-DMA reads + write-through (sc1) stores; 1 = nt stores
  int blocks_per_cu = 1;  // LDS: one 4-wave block per CU (64 KiB of LDS ring)
  int stages = 2;  // double buffer: one tile landing while the other is consumed
  int waves = 4;
};
static ReduceTune g_tune;
static int g_grid_cap = 0;  // mccs_hip_reduce_tune_grid
static int g_num_cus = 0;

static int num_cus() {
  if (g_num_cus > 0) return g_num_cus;
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
    n = 256;
  g_num_cus = n;
  return n;
}

// A launch's own status.  hipGetLastError() after a launch would also return
// any earlier failure left on the calling thread by another call (the
// caller's, another library's), reporting it as this launch's.
template <typename K>
static hipError_t launch_k(K k, int grid, int block, size_t lds, hipStream_t st, const ReduceArgs& a) {
  void* args[] = {(void*)&a};
  return hipLaunchKernel((const void*)k, dim3(grid), dim3(block), args, lds, st);
}

template <int DT, int OP>
constexpr bool tuned_grid() { return OP == OpSum && (DT == mccsFloat32 || DT == mccsFloat16 || DT == mccsBfloat16); }

// pol: 0 plain, 1 nt loads + nt stores, 2 nt loads + plain stores,
// 3 plain loads + nt stores (2/3 and map 1 only in the tuning grid).
template <int DT, int OP, int NS, int ND, int U, int MAP>
static hipError_t launch_reg(const ReduceArgs& a, int pol, int grid, hipStream_t st) {
#define MCCS_REG(LP, SP) launch_k((reduce_reg_kernel<DT, OP, NS, ND, U, LP, SP, MAP>), grid, 256, 0, st, a)
  if constexpr (tuned_grid<DT, OP>()) {
    if (pol == 2) return MCCS_REG(kNonTemporal, kPlain);
    if (pol == 3) return MCCS_REG(kPlain, kNonTemporal);
  }
  if (pol) return MCCS_REG(kNonTemporal, kNonTemporal);
  return MCCS_REG(kPlain, kPlain);
#undef MCCS_REG
}

template <int DT, int OP, int NS, int ND>
static hipError_t launch_reg_u(const ReduceArgs& a, int u, int pol, int map, int grid, hipStream_t st) {
  if constexpr (tuned_grid<DT, OP>()) {
    if (map == 1) {
      if (u == 2) return launch_reg<DT, OP, NS, ND, 2, 1>(a, pol, grid, st);
      if (u == 8) return launch_reg<DT, OP, NS, ND, 8, 1>(a, pol, grid, st);
      return launch_reg<DT, OP, NS, ND, 4, 1>(a, pol, grid, st);
    }
    if (map == 2) {
      if (u == 2) return launch_reg<DT, OP, NS, ND, 2, 2>(a, pol, grid, st);
      if (u == 8) return launch_reg<DT, OP, NS, ND, 8, 2>(a, pol, grid, st);
      return launch_reg<DT, OP, NS, ND, 4, 2>(a, pol, grid, st);
    }
    if (u == 2) return launch_reg<DT, OP, NS, ND, 2, 0>(a, pol, grid, st);
    if (u == 8) return launch_reg<DT, OP, NS, ND, 8, 0>(a, pol, grid, st);
  }
  return launch_reg<DT, OP, NS, ND, 4, 0>(a, pol, grid, st);
}

template <int U, int S, int W>
constexpr bool lds_fits() { return W * S * 2 * U <= 160; }  // KiB of LDS per block

template <int DT, int OP, int U, int S, int W>
static hipError_t launch_lds(const ReduceArgs& a, int pol, int bpc, hipStream_t st) {
  static_assert(lds_fits<U, S, W>(), "LDS budget");
  const size_t lds = (size_t)W * S * 2 * U * 1024;
  // pol: 0 plain DMA + plain stores, 1 nt DMA + nt stores, 2 plain DMA + nt
  // stores; nt DMA with write-through stores (tuning grid only): 3 nt+sc1,
  // 4 sc1, 5 sc0+sc1+nt; sc1 stores with 6 "sc1 nt" / 7 "sc0 sc1 nt" DMA reads
  auto kn = reduce_lds_kernel<DT, OP, U, S, W, kNonTemporal, kNonTemporal>;
  auto kp = reduce_lds_kernel<DT, OP, U, S, W, kPlain, kPlain>;
  auto ks = reduce_lds_kernel<DT, OP, U, S, W, kPlain, kNonTemporal>;
  static std::atomic<bool> attr_set{false};
  if (!attr_set.load(std::memory_order_relaxed)) {
    (void)hipFuncSetAttribute((const void*)kn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)kp, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)ks, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set.store(true, std::memory_order_relaxed);
  }
  if constexpr (tuned_grid<DT, OP>() && U == 4 && (S == 2 || S == 3) && W == 4) {
    if (pol >= 3) {
      auto kw = pol == 3   ? reduce_lds_kernel<DT, OP, U, S, W, kNonTemporal, kNtWriteThrough>
                : pol == 4 ? reduce_lds_kernel<DT, OP, U, S, W, kNonTemporal, kWriteThrough>
                : pol == 5 ? reduce_lds_kernel<DT, OP, U, S, W, kNonTemporal, kSystemNt>
                : pol == 6 ? reduce_lds_kernel<DT, OP, U, S, W, kNtWriteThrough, kWriteThrough>
                           : reduce_lds_kernel<DT, OP, U, S, W, kSystemNt, kWriteThrough>;
      static std::atomic<unsigned> wt_attr_set{0};  // bit per policy 3..7
      const unsigned bit = 1u << (pol - 3);
      if (!(wt_attr_set.load(std::memory_order_relaxed) & bit)) {
        (void)hipFuncSetAttribute((const void*)kw, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        wt_attr_set.fetch_or(bit, std::memory_order_relaxed);
      }
      constexpr int PACK = kPackElems<DT>;
      const int64_t npack = a.count / PACK;
      const int64_t wtiles = (npack + 64 * U - 1) / (64 * U);
      int64_t blocks = (wtiles + W - 1) / W;
      const int64_t gmax = g_grid_cap > 0 ? g_grid_cap : (int64_t)num_cus() * bpc;
      const int grid = (int)(blocks < gmax ? (blocks > 0 ? blocks : 1) : gmax);
      return launch_k(kw, grid, W * 64, lds, st, a);
    }
  }
  constexpr int PACK = kPackElems<DT>;
  const int64_t npack = a.count / PACK;
  const int64_t wtiles = (npack + 64 * U - 1) / (64 * U);
  int64_t blocks = (wtiles + W - 1) / W;
  const int64_t gmax = g_grid_cap > 0 ? g_grid_cap : (int64_t)num_cus() * bpc;
  const int grid = (int)(blocks < gmax ? (blocks > 0 ? blocks : 1) : gmax);
  if (pol == 1 || pol >= 3) return launch_k(kn, grid, W * 64, lds, st, a);
  if (pol == 2) return launch_k(ks, grid, W * 64, lds, st, a);
  return launch_k(kp, grid, W * 64, lds, st, a);
}

// (U, S, W) run-time -> template.  The default (2, 3, 4) exists for every
// dtype/op; the tuning grid only for Sum over fp32/fp16/bf16.
template <int DT, int OP>
static hipError_t launch_lds_cfg(const ReduceArgs& a, const ReduceTune& t, bool* ok, hipStream_t st) {
  *ok = true;
#define MCCS_LDS(U, S, W) \
  if (t.unroll == U && t.stages == S && t.waves == W) return launch_lds<DT, OP, U, S, W>(a, t.policy, t.blocks_per_cu, st);
  MCCS_LDS(4, 2, 4)
  if constexpr (OP == OpSum && (DT == mccsFloat32 || DT == mccsFloat16 || DT == mccsBfloat16)) {
    MCCS_LDS(1, 3, 4) MCCS_LDS(2, 2, 4) MCCS_LDS(2, 3, 4) MCCS_LDS(4, 3, 4) MCCS_LDS(4, 4, 4) MCCS_LDS(8, 2, 4)
    MCCS_LDS(4, 3, 5) MCCS_LDS(2, 3, 6) MCCS_LDS(4, 2, 6) MCCS_LDS(4, 3, 6)
    MCCS_LDS(1, 2, 8) MCCS_LDS(2, 2, 8) MCCS_LDS(4, 2, 8)
  }
#undef MCCS_LDS
  *ok = false;
  return hipSuccess;
}

template <int DT, int OP>
static hipError_t dispatch(const ReduceArgs& a, hipStream_t st) {
  constexpr int PACK = kPackElems<DT>;
  const ReduceTune t = g_tune;
  const int cus = num_cus();
  uintptr_t mis = 0;
  for (int s = 0; s < a.nsrcs; ++s) mis |= (uintptr_t)a.srcs[s];
  for (int d = 0; d < a.ndsts; ++d) mis |= (uintptr_t)a.dsts[d];
  if (mis & 15) {
    int64_t blocks = (a.count + 255) / 256;
    int grid = (int)(blocks < (int64_t)cus * 8 ? (blocks > 0 ? blocks : 1) : (int64_t)cus * 8);
    return launch_k((reduce_scalar_kernel<DT, OP>), grid, 256, 0, st, a);
  }
  if (t.variant == MCCS_REDUCE_VARIANT_LDS && a.nsrcs == 2 && a.ndsts == 1) {
    bool ok = false;
    hipError_t e = launch_lds_cfg<DT, OP>(a, t, &ok, st);
    if (ok) return e;
    // untuned (U,S,W) for this dtype/op: fall through to the REG loop
  }
  const bool reg = t.variant != MCCS_REDUCE_VARIANT_LDS;
  const int map = t.variant == MCCS_REDUCE_VARIANT_REG_BLOCKED ? 1 : t.variant == MCCS_REDUCE_VARIANT_REG_ROWS ? 2 : 0;
  const int unroll = reg ? t.unroll : 4;
  const int bpc = reg ? t.blocks_per_cu : 32;
  const int64_t npack = a.count / PACK;
  const int64_t tile = 256LL * unroll;
  int64_t tiles = (npack + tile - 1) / tile;
  if (tiles < 1) tiles = 1;
  const int64_t gmax = (int64_t)cus * (bpc > 0 ? bpc : 8);
  const int grid = (int)(tiles < gmax ? tiles : gmax);
  if (a.nsrcs == 2 && a.ndsts == 1) return launch_reg_u<DT, OP, 2, 1>(a, unroll, t.policy, map, grid, st);
  if (a.nsrcs == 1 && a.ndsts == 1) return launch_reg_u<DT, OP, 1, 1>(a, unroll, t.policy, 0, grid, st);
  return launch_reg<DT, OP, 0, 0, 4, 0>(a, t.policy ? 1 : 0, grid, st);
}

template <int DT>
static hipError_t dispatch_op(int op, const ReduceArgs& a, hipStream_t st) {
  switch (op) {
    case OpSum: return dispatch<DT, OpSum>(a, st);
    case OpProd: return dispatch<DT, OpProd>(a, st);
    case OpMax: return dispatch<DT, OpMax>(a, st);
    case OpMin: return dispatch<DT, OpMin>(a, st);
  }
  return hipErrorInvalidValue;
}

static hipError_t dispatch_all(int dtype, int op, const ReduceArgs& a, hipStream_t st) {
  switch (dtype) {
#define X(D) \
  case D: return dispatch_op<D>(op, a, st);
    MCCS_FOR_EACH_DTYPE(X)
#undef X
  }
  return hipErrorInvalidValue;
}

}  // namespace mccs

using namespace mccs;

extern "C" mccsResult_t mccs_hip_reduce_copy(void* const* dsts, int ndsts, const void* const* srcs,
                                             int nsrcs, size_t count, int dtype, int op,
                                             hipStream_t stream) {
  if (nsrcs < 1 || nsrcs > kMaxSrcs || ndsts < 1 || ndsts > kMaxDsts || !srcs || !dsts)
    return mccsInvalidArgument;
  if (dtype < 0 || dtype >= mccsNumTypes || op < 0 || op > mccsDevMin) return mccsInvalidArgument;
  ReduceArgs a{};
  for (int s = 0; s < nsrcs; ++s) {
    if (!srcs[s]) return mccsInvalidArgument;
    a.srcs[s] = srcs[s];
  }
  for (int d = 0; d < ndsts; ++d) {
    if (!dsts[d]) return mccsInvalidArgument;
    a.dsts[d] = dsts[d];
  }
  a.nsrcs = nsrcs;
  a.ndsts = ndsts;
  a.count = (int64_t)count;
  if (count == 0) return mccsSuccess;
  hipError_t e = dispatch_all(dtype, op, a, stream);
  return e == hipSuccess ? mccsSuccess : mccsUnhandledCudaError;
}

extern "C" mccsResult_t mccs_hip_reduce(void* dst, const void* const* srcs, int nsrcs, size_t count,
                                        int dtype, int op, hipStream_t stream) {
  void* d[1] = {dst};
  return mccs_hip_reduce_copy(d, 1, srcs, nsrcs, count, dtype, op, stream);
}

extern "C" mccsResult_t mccs_hip_reduce_tune(int variant, int unroll, int policy, int blocks_per_cu,
                                             int stages, int waves) {
  if (variant < 0 || variant > MCCS_REDUCE_VARIANT_REG_ROWS) return mccsInvalidArgument;
  if (policy > 7) return mccsInvalidArgument;
  if (unroll < 0 || unroll > 8 || (unroll & (unroll - 1))) return mccsInvalidArgument;
  if (stages < 0 || stages == 1 || stages > 4 || waves < 0 || (waves != 0 && (waves < 4 || waves > 8 || waves == 7)))
    return mccsInvalidArgument;
  ReduceTune d;
  ReduceTune t;
  t.variant = variant ? variant : d.variant;
  const bool reg = t.variant != MCCS_REDUCE_VARIANT_LDS;
  t.unroll = unroll ? unroll : 4;
  t.policy = policy < 0 ? (reg ? 1 : d.policy) : (reg ? (policy > 3 ? 1 : policy) : policy);
  t.blocks_per_cu = blocks_per_cu > 0 ? blocks_per_cu : (reg ? 32 : 1);
  t.stages = stages ? stages : d.stages;
  t.waves = waves ? waves : d.waves;
  if (!reg && t.waves * t.stages * 2 * t.unroll > 160) return mccsInvalidArgument;
  g_tune = t;
  return mccsSuccess;
}

extern "C" void mccs_hip_reduce_get_tune(int* variant, int* unroll, int* policy, int* blocks_per_cu,
                                         int* stages, int* waves) {
  if (variant) *variant = g_tune.variant;
  if (unroll) *unroll = g_tune.unroll;
  if (policy) *policy = g_tune.policy;
  if (blocks_per_cu) *blocks_per_cu = g_tune.blocks_per_cu;
  if (stages) *stages = g_tune.stages;
  if (waves) *waves = g_tune.waves;
}

#ifdef MCCS_REDUCE_TRACE
extern "C" int mccs_reduce_trace(unsigned long long* out, int max_words) {
  if (max_words < kRTraceWaves * 3) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rtrace), sizeof(g_rtrace), 0, hipMemcpyDeviceToHost)) return -1;
  return kRTraceWaves * 3;
}
#endif

extern "C" mccsResult_t mccs_hip_reduce_tune_grid(int blocks) {
  if (blocks < 0) return mccsInvalidArgument;
  g_grid_cap = blocks;
  return mccsSuccess;
}
