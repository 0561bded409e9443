// K3b — backward of the plain hooked temporal attention (attn_temp under the DummyController:
// attention.py:262-268 -> ptp_utils.py:206-220, 225-234), for the null-text optimisation's
// loss.backward() (run_videop2p.py:601).
//
// Every (batch, token, head) is an independent f x f attention (f <= 32), so the kernel is a plain
// VALU kernel: a group of FP = next_pow2(f) lanes owns one (b, token, head), lane i = frame i.
//   phase 1 (lane = query i): s_j = q_i.k_j, dp_j = dO_i.v_j, p = softmax(scale s),
//            ds_j = p_j (dp_j - sum_j p_j dp_j), dq_i = scale sum_j ds_j k_j;  P, dS rows -> LDS
//   phase 2 (lane = key j):   dk_j = scale sum_i dS_ij q_i,  dv_j = sum_i P_ij dO_i
// Rows are read in 8-channel (16-byte bf16 / 2x16-byte f32) vectors; the other lanes' rows of the
// same (b, token, head) are L1 hits.  The rearrange '(b f) d c -> (b d) f c' is never materialised:
// every tensor is addressed through (b, frame, token) strides.
#include "common.hpp"
#include "vp2p.h"

namespace vp2p {

template <typename T> struct Vec8;
template <> struct Vec8<bf16> {
  static __device__ __forceinline__ void load(const bf16* p, float (&v)[8]) {
    const bf16x8 r = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)r[j];
  }
  static __device__ __forceinline__ void store(bf16* p, const float (&v)[8]) {
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (bf16)v[j];
    *reinterpret_cast<bf16x8*>(p) = r;
  }
};
template <> struct Vec8<float> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[8]) {
    const f32x4 a = reinterpret_cast<const f32x4*>(p)[0], b = reinterpret_cast<const f32x4*>(p)[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = b[j]; }
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[8]) {
    f32x4 a, b;
#pragma unroll
    for (int j = 0; j < 4; ++j) { a[j] = v[j]; b[j] = v[4 + j]; }
    reinterpret_cast<f32x4*>(p)[0] = a;
    reinterpret_cast<f32x4*>(p)[1] = b;
  }
};

template <typename T, int FP>
__global__ __launch_bounds__(256) void temporal_bwd_kernel(const vp2p_temporal_attn_bwd_args a) {
  constexpr int GPB = 256 / FP;                  // groups per block
  extern __shared__ __attribute__((aligned(16))) float tsm[];
  const int tid = threadIdx.x, grp = tid / FP, i = tid % FP;
  float* Pl = tsm + grp * 2 * FP * FP;           // [FP][FP]
  float* Sl = Pl + FP * FP;
  const int F = a.frames, N = a.tokens, D = a.head_dim;
  const int64_t gg = (int64_t)blockIdx.x * GPB + grp;
  const int64_t ngroups = (int64_t)a.batch * N * a.heads;
  const bool gv = gg < ngroups;
  const int head = gv ? (int)(gg % a.heads) : 0;
  const int64_t bn = gv ? gg / a.heads : 0;
  const int n = (int)(bn % N), b = (int)(bn / N);
  const bool lv = gv && i < F;
  auto at = [&](const void* base, int64_t sb, int64_t sf, int64_t sn, int fr) {
    return static_cast<const T*>(base) + b * sb + (int64_t)fr * sf + (int64_t)n * sn + head * D;
  };
  auto atw = [&](void* base, int64_t sb, int64_t sf, int64_t sn, int fr) {
    return static_cast<T*>(base) + b * sb + (int64_t)fr * sf + (int64_t)n * sn + head * D;
  };

  if (lv) {
    float s[FP], dp[FP];
#pragma unroll
    for (int j = 0; j < FP; ++j) { s[j] = 0.f; dp[j] = 0.f; }
    const T* qi = at(a.q, a.q_sb, a.q_sf, a.q_sn, i);
    const T* di = at(a.dout, a.do_sb, a.do_sf, a.do_sn, i);
    for (int c = 0; c < D; c += 8) {
      float qv[8], dv[8];
      Vec8<T>::load(qi + c, qv);
      Vec8<T>::load(di + c, dv);
#pragma unroll
      for (int j = 0; j < FP; ++j) {
        if (j < F) {
          float kv[8], vv[8];
          Vec8<T>::load(at(a.k, a.k_sb, a.k_sf, a.k_sn, j) + c, kv);
          Vec8<T>::load(at(a.v, a.v_sb, a.v_sf, a.v_sn, j) + c, vv);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            s[j] = fmaf(qv[e], kv[e], s[j]);
            dp[j] = fmaf(dv[e], vv[e], dp[j]);
          }
        }
      }
    }
    float m = -__builtin_huge_valf();
#pragma unroll
    for (int j = 0; j < FP; ++j)
      if (j < F) m = fmaxf(m, s[j] * a.scale);
    float l = 0.f;
#pragma unroll
    for (int j = 0; j < FP; ++j) {
      s[j] = j < F ? __expf(s[j] * a.scale - m) : 0.f;
      l += s[j];
    }
    const float inv = 1.f / l;
    float delta = 0.f;
#pragma unroll
    for (int j = 0; j < FP; ++j) {
      s[j] *= inv;
      delta = fmaf(s[j], dp[j], delta);
    }
#pragma unroll
    for (int j = 0; j < FP; ++j) {
      dp[j] = s[j] * (dp[j] - delta);
      Pl[i * FP + j] = s[j];
      Sl[i * FP + j] = dp[j];
    }
    T* dqi = atw(a.dq, a.dq_sb, a.dq_sf, a.dq_sn, i);
    for (int c = 0; c < D; c += 8) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < FP; ++j) {
        if (j < F) {
          float kv[8];
          Vec8<T>::load(at(a.k, a.k_sb, a.k_sf, a.k_sn, j) + c, kv);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] = fmaf(dp[j], kv[e], acc[e]);
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] *= a.scale;
      Vec8<T>::store(dqi + c, acc);
    }
  }
  __syncthreads();
  if (!lv) return;
  const int jk = i;   // this lane now owns key frame jk
  T* dkj = atw(a.dk, a.dk_sb, a.dk_sf, a.dk_sn, jk);
  T* dvj = atw(a.dv, a.dv_sb, a.dv_sf, a.dv_sn, jk);
  for (int c = 0; c < D; c += 8) {
    float ak[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float av[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int iq = 0; iq < FP; ++iq) {
      if (iq < F) {
        float qv[8], dv[8];
        Vec8<T>::load(at(a.q, a.q_sb, a.q_sf, a.q_sn, iq) + c, qv);
        Vec8<T>::load(at(a.dout, a.do_sb, a.do_sf, a.do_sn, iq) + c, dv);
        const float ds = Sl[iq * FP + jk], p = Pl[iq * FP + jk];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          ak[e] = fmaf(ds, qv[e], ak[e]);
          av[e] = fmaf(p, dv[e], av[e]);
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) ak[e] *= a.scale;
    Vec8<T>::store(dkj + c, ak);
    Vec8<T>::store(dvj + c, av);
  }
}

template <typename T, int FP>
static void launch_tbwd(const vp2p_temporal_attn_bwd_args* a, hipStream_t s) {
  const int64_t groups = (int64_t)a->batch * a->tokens * a->heads;
  const int64_t blocks = (groups + 256 / FP - 1) / (256 / FP);
  const size_t lds = (size_t)(256 / FP) * 2 * FP * FP * sizeof(float);
  hipLaunchKernelGGL((temporal_bwd_kernel<T, FP>), dim3((unsigned)blocks), dim3(256), lds, s, *a);
}

}  // namespace vp2p

using namespace vp2p;

extern "C" int vp2p_temporal_attn_bwd(const vp2p_temporal_attn_bwd_args* a, void* stream) {
  if (!a || !a->q || !a->k || !a->v || !a->dout || !a->dq || !a->dk || !a->dv) return VP2P_E_ARG;
  if (a->batch <= 0 || a->frames <= 0 || a->tokens <= 0 || a->heads <= 0 || a->head_dim <= 0) return VP2P_E_ARG;
  if (a->dtype != VP2P_BF16 && a->dtype != VP2P_F32) return VP2P_E_DTYPE;
  if (a->frames > 32) return VP2P_E_SHAPE;
  if (a->head_dim % 8) return VP2P_E_HEAD_DIM;
  const int epc = a->dtype == VP2P_BF16 ? 8 : 4;
  const int64_t st[] = {a->q_sb, a->q_sf, a->q_sn, a->k_sb, a->k_sf, a->k_sn, a->v_sb, a->v_sf, a->v_sn,
                        a->do_sb, a->do_sf, a->do_sn, a->dq_sb, a->dq_sf, a->dq_sn, a->dk_sb, a->dk_sf,
                        a->dk_sn, a->dv_sb, a->dv_sf, a->dv_sn};
  for (int64_t s : st)
    if (s % epc) return VP2P_E_ARG;
  const void* ptrs[] = {a->q, a->k, a->v, a->dout, a->dq, a->dk, a->dv};
  for (const void* p : ptrs)
    if (reinterpret_cast<uintptr_t>(p) & 15) return VP2P_E_ARG;
  if ((int64_t)a->batch * a->tokens * a->heads > (int64_t)0x7fffffff * 8) return VP2P_E_SHAPE;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int fp = a->frames <= 8 ? 8 : a->frames <= 16 ? 16 : 32;
  if (a->dtype == VP2P_BF16) {
    if (fp == 8) launch_tbwd<bf16, 8>(a, s);
    else if (fp == 16) launch_tbwd<bf16, 16>(a, s);
    else launch_tbwd<bf16, 32>(a, s);
  } else {
    if (fp == 8) launch_tbwd<float, 8>(a, s);
    else if (fp == 16) launch_tbwd<float, 16>(a, s);
    else launch_tbwd<float, 32>(a, s);
  }
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}
