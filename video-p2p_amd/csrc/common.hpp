// Shared gfx950 device helpers for the controlled-attention kernels.
//
// All three attention kernels use the same "swapped" MFMA formulation on 32x32 tiles:
//   S^T[key][query] = K[key][:] . Q[query][:]       (A = K rows, B = Q^T, v_mfma_f32_32x32x16_bf16
//                                                     or v_mfma_f32_32x32x2_f32)
// so a lane (r = lane & 31, h = lane >> 5) ends up holding query r's scores for the 16 keys
//   key(i) = (i & 3) + 8 * (i >> 2) + 4 * h,  i = 0..15          (accumulator register i)
// The row softmax is therefore lane-local plus one exchange with lane r ^ 32, and the probability
// tile is already the B operand of the second product
//   O^T[dcol][query] += V^T[dcol][key] . P^T[key][query]
// when V^T's keys are supplied in the same permuted order (CDNA4 guide §3, "an accumulator tile as
// the next MFMA's operand").  O^T keeps the query on the lane, so per-query rescales and the final
// 1/l are lane-local too.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vp2p {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kNegInf = -__builtin_huge_valf();

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// key index held in accumulator register i by lane half h (see header comment)
__device__ __forceinline__ constexpr int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// value of x held by lane l ^ 32 (the other half of the same 32x32 column)
__device__ __forceinline__ float xhalf(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(lane_id() < 32 ? r[1] : r[0]);
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// ------------------------------------------------------------------------------------------------
// Per-dtype MFMA traits.
//   KD : head-dim elements per QK^T k-step;   the A/B fragment of a lane covers
//        [KD*s + 8h, +8) (bf16) or element KD*s + h (f32).
//   KK : keys per PV k-step (16 for bf16: two k-steps per 32-key block; 2 for f32: sixteen).
// ------------------------------------------------------------------------------------------------
template <typename T> struct Mfma;

template <> struct Mfma<bf16> {
  static constexpr int KD = 16;
  static constexpr int PV_STEPS = 2;     // per 32-key block
  typedef bf16x8 frag;
  static __device__ __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ frag zero() {
    frag z;
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = (bf16)0.f;
    return z;
  }
  // Row fragment of k-step s from a row of `d` valid elements (16-byte aligned for 16s+8h < d).
  static __device__ __forceinline__ frag row_frag(const bf16* row, int s, int h, int d) {
    const int c = KD * s + 8 * h;
    if (c < d) return *reinterpret_cast<const frag*>(row + c);
    return zero();
  }
  // B fragment of P^T for PV k-step sp (0..1) of a 32-key score block.
  static __device__ __forceinline__ frag p_frag(const f32x16& p, int sp) {
    frag r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (bf16)p[8 * sp + j];
    return r;
  }
  static __device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }
  static __device__ __forceinline__ bf16 from_f32(float x) { return (bf16)x; }
};

template <> struct Mfma<float> {
  static constexpr int KD = 2;
  static constexpr int PV_STEPS = 16;
  typedef float frag;
  static __device__ __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ frag zero() { return 0.f; }
  static __device__ __forceinline__ frag row_frag(const float* row, int s, int h, int d) {
    const int c = KD * s + h;
    return c < d ? row[c] : 0.f;
  }
  static __device__ __forceinline__ frag p_frag(const f32x16& p, int sp) { return p[sp]; }
  static __device__ __forceinline__ float to_f32(float x) { return x; }
  static __device__ __forceinline__ float from_f32(float x) { return x; }
};

// Keys covered by PV k-step sp for lane half h within a 32-key block (f32 form: one key).
__device__ __forceinline__ int f32_pv_key(int sp, int h) { return (sp & 3) + 8 * (sp >> 2) + 4 * h; }

// ------------------------------------------------------------------------------------------------
// ds_read_b64_tr_b16 (gfx950): transposed read of a 4-row x 16-column block of a row-major bf16
// LDS image.  Lane 4q+p of each 16-lane group passes the address of row q, columns 4p..4p+3 and
// receives column (lane & 15) of the four rows.  EXEC must be all ones.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ bf16x4 lds_read_tr(const bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4*)(p));
}

// A fragment of V^T for PV k-step sp, output tile t, from a row-major [key][VROW] bf16 LDS image
// whose first key is key0: element j of lane (r, h) = V[key0 + 16sp + 8(j>>2) + 4h + (j&3)][32t + r].
template <int VROW>
__device__ __forceinline__ bf16x8 vt_frag_lds(const bf16* vlds, int key0, int sp, int t) {
  const int l = lane_id();
  const int h = l >> 5, g = (l >> 4) & 1, q = (l >> 2) & 3, p = l & 3;
  const bf16* base = vlds + (key0 + 16 * sp + 4 * h + q) * VROW + 32 * t + 16 * g + 4 * p;
  bf16x4 lo = lds_read_tr(base);
  bf16x4 hi = lds_read_tr(base + 8 * VROW);
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// Bijective XCD-grouping remap of a 1-D grid (CDNA4 guide §5 "XCD swizzle must be bijective"):
// consecutive logical ids land on the same XCD (same L2) under round-robin dispatch.  Speed only.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

template <typename T> struct DtypeOf;
template <> struct DtypeOf<float> { static constexpr int value = 0; };
template <> struct DtypeOf<bf16> { static constexpr int value = 1; };

constexpr __host__ __device__ int round_up(int x, int m) { return (x + m - 1) / m * m; }

}  // namespace vp2p
