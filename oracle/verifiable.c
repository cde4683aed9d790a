/*
 * verifiable.c — TEST INFRASTRUCTURE ONLY (part of libmccs_oracle.so).
 *
 * Restatement of the nccl-tests "verifiable" float-sum vectors that the
 * reference vendors for its own benchmark checks
 * (nccl-tests-mccs/verifiable/verifiable.cu).  For every element index the
 * generator yields one input per rank and the expected output such that
 * the inputs sum EXACTLY to the output in ANY order (all partial sums are
 * integers of at most mantissa_bits+1 bits times one power of two), so a
 * ring AllReduce of the inputs must equal the output bit for bit whatever
 * its summation order.  Also restated: the reference's tolerance formula
 * for inexact float sums.
 *
 *   mixBits / hashOf ............. verifiable.cu:58-77
 *   FloatLayout / makeFloat ...... verifiable.cu:300-333
 *   umul32hi / umul64hi / clz .... verifiable.cu:340-370
 *   shuffleRank .................. verifiable.cu:380-411
 *   genSumXY ..................... verifiable.cu:418-463
 *   genInOutFloatSum ............. verifiable.cu:466-512
 *   genInput/genOutput(ReduceSum)  verifiable.cu:664-676 (same_sign = false)
 *   genInput/genOutput(ReduceAvg)  verifiable.cu:737-749 (same_sign = true)
 *   calcSumFloatTolerance ........ verifiable.cu:981-1004
 *
 * dtype codes follow mccsDevDataType_t: 6 = half, 7 = float, 9 = bfloat16
 * (raw 16-bit patterns), 8 = double.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

/* 64-bit mixer: high word bumped, folded into the low word, golden-ratio
 * multiply, then the new high word's halves swapped into the low word. */
static uint64_t vf_mix(uint64_t x) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  hi += 1u;
  lo ^= hi;
  x = ((uint64_t)hi << 32 | lo) * 0x9e3779b97f4a7c13ull;
  lo = (uint32_t)x;
  hi = (uint32_t)(x >> 32);
  lo ^= (hi << 16) ^ (hi >> 16);
  return (uint64_t)hi << 32 | lo;
}

static uint64_t vf_hash(uint64_t a, uint64_t b) {
  a += 1ull << 32;
  a += b;
  a ^= a >> 32;
  a *= 0x9e3779b97f4a7c13ull;
  a += (b >> 16) ^ (b << 48);
  a ^= a >> 32;
  a *= 0xc4ceb9fe1a85ec53ull;
  return a;
}

static uint64_t vf_mulhi32(uint32_t a, uint32_t b) { return ((uint64_t)a * b) >> 32; }
static uint64_t vf_mulhi64(uint64_t a, uint64_t b) { return (uint64_t)(((unsigned __int128)a * b) >> 64); }
static int vf_clz32(uint32_t x) { return x ? __builtin_clz(x) : 32; }
static int vf_clz64(uint64_t x) { return x ? __builtin_clzll(x) : 64; }

/* A bijective scramble of [0, rank_n): two rounds of (x*odd + c) and the
 * triangular map on the largest power-of-two block, rotating the remainder. */
static int vf_shuffle_rank(int rank_n, int rank_me, uint64_t *rng) {
  const uint32_t a = (uint32_t)*rng, b = (uint32_t)(*rng >> 32);
  *rng = vf_mix(*rng);
  const uint32_t n2 = (0xffffffffu >> 1) >> vf_clz32((uint32_t)rank_n);
  uint32_t r = (uint32_t)rank_me;
  if (r <= n2) {
    r = (r * (a | 1u) + b) & n2;
    r = ((r * r + r) / 2) & n2;
    r += (uint32_t)rank_n - (n2 + 1);
  } else {
    r -= n2 + 1;
  }
  if (r <= n2) {
    r = (r * (b | 1u) + a) & n2;
    r = ((r * r + r) / 2) & n2;
  }
  return (int)r;
}

/* Picks y in [y_max/2, y_max] (or, with avoid_y, a value != the incoming y)
 * and this rank's integer share x of it: the first s*pn ranks submit their
 * partition index + 1, the last rank the remainder.  W = mantissa width
 * class: 32 or 64 bits (the reference templates on the unsigned type). */
static void vf_sum_xy(int W, int rank_n, int rank_me, uint64_t *rng, uint64_t y_max, uint64_t *x, uint64_t *y,
                      int avoid_y) {
  const uint64_t mask = W == 32 ? 0xffffffffull : ~0ull;
  {
    const uint64_t y_min = ((y_max + 1) / 2) & mask;
    const uint64_t span = (y_max / 2 + (avoid_y ? 0 : 1)) & mask;
    const uint64_t d = W > 32 ? vf_mulhi64(*rng, span) : vf_mulhi32((uint32_t)*rng, (uint32_t)span);
    const uint64_t y1 = ((avoid_y ? *y + 1 : y_min) + d) & mask;
    *y = (y1 - ((avoid_y && (y1 < y_min || y_max < y1)) ? y_max / 2 : 0)) & mask;
  }
  *rng = vf_mix(*rng);
  const uint64_t r = (uint32_t)rank_me, rn = (uint32_t)rank_n;
  uint64_t pn = rn == 1 ? 1 : ((2 * (*y / rn) - 1) & mask);  /* wraps when y < rn, clamped below */
  if (pn == 0) pn = 1;
  if (rn < pn) pn = rn;
  uint64_t p_sum;
  if (y_max <= 0x7fffffffull) p_sum = (uint32_t)((uint32_t)pn * (uint32_t)(pn + 1) / 2);
  else p_sum = pn * (pn + 1) / 2;
  p_sum &= mask;
  const uint32_t s = (uint32_t)(*y / p_sum < rn / pn ? *y / p_sum : rn / pn);
  uint64_t xv = (r / s < pn) ? 1 + r / s : 0;
  if (r == rn - 1) xv += *y - (uint64_t)s * p_sum;
  *x = xv & mask;
}

struct vf_layout {
  int exp_bits, mant_bits, width_bits, W;
};

static int vf_layout_of(int dtype, struct vf_layout *L) {
  switch (dtype) {
    case 6: *L = (struct vf_layout){5, 10, 16, 32}; return 0;
    case 7: *L = (struct vf_layout){8, 23, 32, 32}; return 0;
    case 8: *L = (struct vf_layout){11, 52, 64, 64}; return 0;
    case 9: *L = (struct vf_layout){8, 7, 16, 32}; return 0;
  }
  return -1;
}

/* One value of genInOutFloatSum: the raw bit pattern (low width_bits). */
static uint64_t vf_float_sum_bits(const struct vf_layout *L, int input_not_output, int rank_n, int rank_me,
                                  uint64_t seed, int64_t index, int same_sign) {
  const int exp_lo = 1 + L->mant_bits;
  const int exp_hi = (1 << L->exp_bits) - 1;
  const uint64_t mant_mask = (1ull << L->mant_bits) - 1;
  const uint64_t max_mant = 2 * mant_mask + 1; /* implicit leading one */
  uint64_t rng = vf_hash(seed, (uint64_t)index);
  int y_sign = (int)(rng & 1);
  int x_sign = y_sign;
  const int xy_exp = exp_lo + (int)vf_mulhi32((uint32_t)(rng >> 32), (uint32_t)(exp_hi - exp_lo));
  rng = vf_mix(rng);
  rank_me = vf_shuffle_rank(rank_n, rank_me, &rng);
  const int sub_n = same_sign ? rank_n : (rank_n + 1) / 2;
  const int sub_me = same_sign ? rank_me : rank_me / 2;
  uint64_t x0 = 0, y0 = 0;
  vf_sum_xy(L->W, sub_n, sub_me, &rng, max_mant, &x0, &y0, 0);
  if (!same_sign && rank_n / 2 != 0) {
    /* odd shuffled ranks carry a negative partial sum y1 != y0 */
    uint64_t x1 = 0, y1 = y0;
    vf_sum_xy(L->W, rank_n / 2, rank_me / 2, &rng, max_mant, &x1, &y1, 1);
    y_sign ^= y0 < y1 ? 1 : 0;
    y0 = y0 < y1 ? y1 - y0 : y0 - y1;
    x_sign ^= rank_me % 2;
    x0 = rank_me % 2 == 0 ? x0 : x1;
  }
  uint64_t m = input_not_output ? x0 : y0;
  if (m == 0) return 0; /* +0 */
  const int shift = vf_clz64(m) - (64 - L->mant_bits - 1);
  const int sign = input_not_output ? x_sign : y_sign;
  const int ex = xy_exp - shift;
  m <<= shift;
  uint64_t bits = (uint64_t)sign;
  bits = (bits << L->exp_bits) | (uint64_t)ex;
  bits = (bits << L->mant_bits) | (m & mant_mask);
  return bits;
}

/* Fills out[0..count) with the values for element indices index0+i: rank
 * rank_me's input when input_not_output, else the expected sum.  Returns
 * -1 for an unsupported dtype. */
int oracle_verifiable_float_sum(int dtype, int input_not_output, int rank_n, int rank_me, uint64_t seed,
                                int64_t index0, size_t count, int same_sign, void *out) {
  struct vf_layout L;
  if (vf_layout_of(dtype, &L) || rank_n < 1 || rank_me < 0 || rank_me >= rank_n) return -1;
  for (size_t i = 0; i < count; ++i) {
    const uint64_t b = vf_float_sum_bits(&L, input_not_output, rank_n, input_not_output ? rank_me : 0, seed,
                                         index0 + (int64_t)i, same_sign);
    switch (L.width_bits) {
      case 16: ((uint16_t *)out)[i] = (uint16_t)b; break;
      case 32: ((uint32_t *)out)[i] = (uint32_t)b; break;
      default: ((uint64_t *)out)[i] = b; break;
    }
  }
  return 0;
}

/* Bit-distance tolerance of an inexact n-term float sum (empirical fit in
 * the reference: 1 + coef * n^power). */
unsigned oracle_sum_float_tolerance(int rank_n, int dtype) {
  float power = 0.f, coef = 0.f;
  switch (dtype) {
    case 7: case 8: power = .51f; coef = 1.25f; break;
    case 6: power = .91f; coef = .75f; break;
    case 9: power = .91f; coef = .66f; break;
    default: return 0;
  }
  return 1u + (unsigned)(coef * powf((float)rank_n, power));
}
