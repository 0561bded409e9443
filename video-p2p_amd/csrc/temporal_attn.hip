// K3 — hooked temporal attention (attn_temp) + replace_self_attention.
//
// Reference path: BasicTransformerBlock rearranges '(b f) d c -> (b d) f c' (attention.py:262-268),
// the hooked forward (ptp_utils.py:196-221) computes an f x f softmax per (b, token, head) and the
// controller, for steps in [0, int(50 * self_replace_steps)), overwrites the edited prompts'
// conditional maps with the source prompt's (run_videop2p.py:293-298, 306, 315) before attn @ v.
//
// Here no rearrange is materialised: Q/K/V/O are addressed in place through (b, frame, token)
// strides.  One 32-lane MFMA tile packs G = 32 / fpad tokens x fpad frames (fpad = next power of
// two >= f); cross-token scores are masked to -inf, so one 32x32x16 product serves G tokens.
// The source prompt's probability fragments stay in registers and are fed straight to the edited
// prompts' P.V products: the self-replace is free.
#include <stdlib.h>

#include "common.hpp"
#include "vp2p.h"

namespace vp2p {

template <typename T, int D>
struct TempCfg {
  static constexpr bool BF = sizeof(T) == 2;
  static constexpr int KD = Mfma<T>::KD;
  static constexpr int DP = round_up(D, KD);
  static constexpr int KS = DP / KD;
  static constexpr int DV = round_up(D, 32);
  static constexpr int NT = DV / 32;
  static constexpr int EPC = 16 / (int)sizeof(T);
  static constexpr int CPR = D / EPC;
  static constexpr int vrow_bf16() {
    int v = DV;
    while (!((v / 2) % 64 == 16 || (v / 2) % 64 == 48)) v += 8;
    return v;
  }
  static constexpr int VROW = BF ? vrow_bf16() : DV;
  static constexpr int WAVE_LDS = 32 * VROW * (int)sizeof(T);
};

// One wave owns one (CFG half, G-token block, head) and walks the half's prompts; heads are spread
// over blockIdx.y.  For d <= 80 the next prompt's Q, K and V rows are fetched while the current
// prompt computes (and the first prompt's V with its Q and K), so each wave exposes one HBM
// latency instead of two per prompt.
// WPB waves per workgroup = WPB heads of the same token block.  (Eight heads per workgroup -- whole
// q / k / v / O rows per workgroup -- measured bit-equal but 6 % slower at res-64 and 45-52 % slower
// at res-16: profiles/r03_k3_wpb8_rejected.jsonl.)
template <typename T, int D, int WPB = 4>
__global__ __launch_bounds__(64 * WPB, sizeof(T) == 2 ? 8 / WPB : 1) void temporal_attn_p2p_kernel(const vp2p_temporal_attn_args a, int lf) {
  using M = Mfma<T>;
  using C = TempCfg<T, D>;
  constexpr bool PF = C::KS <= 5;
  constexpr int VN = (C::CPR + 1) / 2;          // V vectors per lane (c = h, h + 2, ...)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, r = l & 31, h = l >> 5;
  const int head = blockIdx.y * WPB + w;
  if (head >= a.heads) return;
  T* Vs = reinterpret_cast<T*>(smem + w * C::WAVE_LDS);
  for (int i = l; i < C::WAVE_LDS / 16; i += 64) reinterpret_cast<u32x4*>(Vs)[i] = u32x4{0, 0, 0, 0};

  const int fpad = 1 << lf, G = 32 >> lf;
  const int F = a.frames, N = a.tokens;
  const int pblocks = (N + G - 1) / G;
  const bool p2p = a.prompts > 0 && a.batch == (a.cond_only ? 1 : 2) * a.prompts;
  const int RP = p2p ? a.prompts : 1;
  const int g = blockIdx.x / pblocks;
  const int pb = blockIdx.x - g * pblocks;
  const bool replace = p2p && (a.cond_only || g == 1) && a.self_replace;

  // this lane's (token slot, frame) as a query row, and as the key row of the same index
  const int slot = r >> lf, fr = r & (fpad - 1);
  const int pos = pb * G + slot;
  const bool rv = fr < F && pos < N;
  const float cs = a.scale * kLog2e;

  // operand rows of prompt p (Q, K only when its scores are computed, V always)
  typename M::frag qn[C::KS], kn[C::KS];
  u32x4 vn[VN];
  auto load = [&](int p, typename M::frag* qd, typename M::frag* kd, u32x4* vd) {
    const int b = g * RP + p;
    if (!(replace && p > 0)) {
      const T* qrow = static_cast<const T*>(a.q) + (rv ? b * a.q_sb + fr * a.q_sf + pos * a.q_sn + head * D : 0);
      const T* krow = static_cast<const T*>(a.k) + (rv ? b * a.k_sb + fr * a.k_sf + pos * a.k_sn + head * D : 0);
#pragma unroll
      for (int s = 0; s < C::KS; ++s) {
        qd[s] = rv ? M::row_frag(qrow, s, h, D) : M::zero();
        kd[s] = rv ? M::row_frag(krow, s, h, D) : M::zero();
      }
    }
    const T* vrow = static_cast<const T*>(a.v) + (rv ? b * a.v_sb + fr * a.v_sf + pos * a.v_sn + head * D : 0);
#pragma unroll
    for (int i = 0; i < VN; ++i) {
      const int c = h + 2 * i;
      vd[i] = (rv && c < C::CPR) ? *reinterpret_cast<const u32x4*>(vrow + c * C::EPC) : u32x4{0, 0, 0, 0};
    }
  };
  if constexpr (PF) load(0, qn, kn, vn);

  typename M::frag psrc[M::PV_STEPS];
  f32x16 prob_src;
  for (int p = 0; p < RP; ++p) {
    const int b = g * RP + p;
    typename M::frag qf[C::KS], kf[C::KS];
    u32x4 vv[VN];
    if constexpr (PF) {
#pragma unroll
      for (int s = 0; s < C::KS; ++s) { qf[s] = qn[s]; kf[s] = kn[s]; }
#pragma unroll
      for (int i = 0; i < VN; ++i) vv[i] = vn[i];
      if (p + 1 < RP) load(p + 1, qn, kn, vn);
    } else {
      load(p, qf, kf, vv);
    }
    f32x16 sc;
    typename M::frag pf[M::PV_STEPS];
    if (replace && p > 0) {
#pragma unroll
      for (int sp = 0; sp < M::PV_STEPS; ++sp) pf[sp] = psrc[sp];
      sc = prob_src;
    } else {
      sc = zero16();
#pragma unroll
      for (int s = 0; s < C::KS; ++s) sc = M::mma(kf[s], qf[s], sc);
      float mx = kNegInf;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int kk = acc_row(i, h);
        const bool ok = (kk >> lf) == slot && (kk & (fpad - 1)) < F;
        const float v = ok ? sc[i] * cs : kNegInf;
        sc[i] = v;
        mx = fmaxf(mx, v);
      }
      mx = fmaxf(mx, xhalf(mx));
      float sum = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float e = fast_exp2(sc[i] - mx);
        sc[i] = e;
        sum += e;
      }
      sum += xhalf(sum);
      const float inv = 1.f / sum;
#pragma unroll
      for (int i = 0; i < 16; ++i) sc[i] *= inv;
#pragma unroll
      for (int sp = 0; sp < M::PV_STEPS; ++sp) pf[sp] = M::p_frag(sc, sp);
      if (replace) {
#pragma unroll
        for (int sp = 0; sp < M::PV_STEPS; ++sp) psrc[sp] = pf[sp];
        prob_src = sc;
      }
    }
    if (a.probs_out && rv) {
      float* prow = a.probs_out + ((((int64_t)b * N + pos) * a.heads + head) * F + fr) * F;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int kk = acc_row(i, h);
        if ((kk >> lf) == slot && (kk & (fpad - 1)) < F) prow[kk & (fpad - 1)] = sc[i];
      }
    }

    // stage this tile's 32 V rows (row index = lane row r) in the wave's LDS image
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < VN; ++i) {
      const int c = h + 2 * i;
      if (c < C::CPR) *reinterpret_cast<u32x4*>(Vs + r * C::VROW + c * C::EPC) = vv[i];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    f32x16 o[C::NT];
#pragma unroll
    for (int t = 0; t < C::NT; ++t) o[t] = zero16();
#pragma unroll
    for (int sp = 0; sp < M::PV_STEPS; ++sp)
#pragma unroll
      for (int t = 0; t < C::NT; ++t) {
        typename M::frag vf;
        if constexpr (C::BF) vf = vt_frag_lds<C::VROW>(Vs, 0, sp, t);
        else vf = Vs[f32_pv_key(sp, h) * C::VROW + 32 * t + r];
        o[t] = M::mma(vf, pf[sp], o[t]);
      }
    if (rv) {
      T* orow = static_cast<T*>(a.o) + b * a.o_sb + fr * a.o_sf + pos * a.o_sn + head * D;
#pragma unroll
      for (int t = 0; t < C::NT; ++t)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const int dc = 32 * t + 8 * gq + 4 * h;
          if (dc < D) {
            if constexpr (C::BF) {
              bf16x4 v;
#pragma unroll
              for (int j = 0; j < 4; ++j) v[j] = (bf16)o[t][4 * gq + j];
              *reinterpret_cast<bf16x4*>(orow + dc) = v;
            } else {
              f32x4 v;
#pragma unroll
              for (int j = 0; j < 4; ++j) v[j] = o[t][4 * gq + j];
              *reinterpret_cast<f32x4*>(orow + dc) = v;
            }
          }
        }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Long clips (32 < frames <= 128, e.g. configs[4]'s 128-frame clip): the f x f map of one (b, token,
// head) no longer fits one tile, so one wave owns 32 query frames of one (CFG half, token, head) and
// holds the scores against all KB*32 key frames in registers (KB <= 4 blocks, exact two-pass row
// softmax as in the hooked forward, ptp_utils.py:217), walking the half's prompts.  K rows are MFMA A
// fragments read straight from global memory (16 bytes per lane); the V rows of each 32-frame key
// block are staged in the wave's LDS image and read transposed (ds_read_b64_tr_b16) for O^T = V^T P^T.
// Self-replace keeps the source prompt's P fragments (KB x 2 bf16x8) and feeds them to the edited
// prompts' PV products, so it is free here too.
// ------------------------------------------------------------------------------------------------
template <typename T, int D, int KB>
__global__ __launch_bounds__(256) void temporal_attn_long_kernel(const vp2p_temporal_attn_args a) {
  using M = Mfma<T>;
  using C = TempCfg<T, D>;
  constexpr int VN = (C::CPR + 1) / 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, r = l & 31, h = l >> 5;
  const int head = blockIdx.y * 4 + w;
  if (head >= a.heads) return;
  T* Vs = reinterpret_cast<T*>(smem + w * C::WAVE_LDS);
  for (int i = l; i < C::WAVE_LDS / 16; i += 64) reinterpret_cast<u32x4*>(Vs)[i] = u32x4{0, 0, 0, 0};

  const int F = a.frames, N = a.tokens;
  const int qblocks = (F + 31) >> 5;
  const bool p2p = a.prompts > 0 && a.batch == (a.cond_only ? 1 : 2) * a.prompts;
  const int RP = p2p ? a.prompts : 1;
  const int per_g = N * qblocks;
  const int g = blockIdx.x / per_g;
  const int rem = blockIdx.x - g * per_g;
  const int pos = rem / qblocks, qb = rem - (rem / qblocks) * qblocks;
  const bool replace = p2p && (a.cond_only || g == 1) && a.self_replace;
  const int qf_idx = qb * 32 + r;             // this lane's query frame
  const bool qvalid = qf_idx < F;
  const float cs = a.scale * kLog2e;

  typename M::frag psrc[KB][M::PV_STEPS];
  for (int p = 0; p < RP; ++p) {
    const int b = g * RP + p;
    typename M::frag pf[KB][M::PV_STEPS];
    if (replace && p > 0) {
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int sp = 0; sp < M::PV_STEPS; ++sp) pf[kb][sp] = psrc[kb][sp];
    } else {
      typename M::frag qf[C::KS];
      const T* qrow = static_cast<const T*>(a.q) + (qvalid ? b * a.q_sb + qf_idx * a.q_sf + pos * a.q_sn + head * D : 0);
#pragma unroll
      for (int s = 0; s < C::KS; ++s) qf[s] = qvalid ? M::row_frag(qrow, s, h, D) : M::zero();
      f32x16 sc[KB];
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const int kf = kb * 32 + r;           // this lane's key frame (A-fragment row)
        const bool kvalid = kf < F;
        const T* krow = static_cast<const T*>(a.k) + (kvalid ? b * a.k_sb + kf * a.k_sf + pos * a.k_sn + head * D : 0);
        sc[kb] = zero16();
#pragma unroll
        for (int s = 0; s < C::KS; ++s) sc[kb] = M::mma(kvalid ? M::row_frag(krow, s, h, D) : M::zero(), qf[s], sc[kb]);
      }
      float mx = kNegInf;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float v = (kb * 32 + acc_row(i, h) < F) ? sc[kb][i] * cs : kNegInf;
          sc[kb][i] = v;
          mx = fmaxf(mx, v);
        }
      mx = fmaxf(mx, xhalf(mx));
      float sum = 0.f;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float e = fast_exp2(sc[kb][i] - mx);
          sc[kb][i] = e;
          sum += e;
        }
      sum += xhalf(sum);
      const float inv = 1.f / sum;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
#pragma unroll
        for (int i = 0; i < 16; ++i) sc[kb][i] *= inv;
#pragma unroll
        for (int sp = 0; sp < M::PV_STEPS; ++sp) pf[kb][sp] = M::p_frag(sc[kb], sp);
      }
      if (replace) {
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
          for (int sp = 0; sp < M::PV_STEPS; ++sp) psrc[kb][sp] = pf[kb][sp];
      }
      if (a.probs_out && qvalid) {
        // with the self-replace on, the edited prompts' maps ARE the source's: write them here too
        for (int pp = p; pp < (replace ? RP : p + 1); ++pp) {
          float* prow = a.probs_out + ((((int64_t)(g * RP + pp) * N + pos) * a.heads + head) * F + qf_idx) * F;
#pragma unroll
          for (int kb = 0; kb < KB; ++kb)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int kk = kb * 32 + acc_row(i, h);
              if (kk < F) prow[kk] = sc[kb][i];
            }
        }
      }
    }

    // O^T = V^T P^T, one 32-frame key block at a time through the wave's LDS image
    f32x16 o[C::NT];
#pragma unroll
    for (int t = 0; t < C::NT; ++t) o[t] = zero16();
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const int kf = kb * 32 + r;
      const bool kvalid = kf < F;
      const T* vrow = static_cast<const T*>(a.v) + (kvalid ? b * a.v_sb + kf * a.v_sf + pos * a.v_sn + head * D : 0);
      u32x4 vv[VN];
#pragma unroll
      for (int i = 0; i < VN; ++i) {
        const int c = h + 2 * i;
        vv[i] = (kvalid && c < C::CPR) ? *reinterpret_cast<const u32x4*>(vrow + c * C::EPC) : u32x4{0, 0, 0, 0};
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int i = 0; i < VN; ++i) {
        const int c = h + 2 * i;
        if (c < C::CPR) *reinterpret_cast<u32x4*>(Vs + r * C::VROW + c * C::EPC) = vv[i];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int sp = 0; sp < M::PV_STEPS; ++sp)
#pragma unroll
        for (int t = 0; t < C::NT; ++t) {
          typename M::frag vf;
          if constexpr (C::BF) vf = vt_frag_lds<C::VROW>(Vs, 0, sp, t);
          else vf = Vs[f32_pv_key(sp, h) * C::VROW + 32 * t + r];
          o[t] = M::mma(vf, pf[kb][sp], o[t]);
        }
    }
    if (qvalid) {
      T* orow = static_cast<T*>(a.o) + b * a.o_sb + qf_idx * a.o_sf + pos * a.o_sn + head * D;
#pragma unroll
      for (int t = 0; t < C::NT; ++t)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const int dc = 32 * t + 8 * gq + 4 * h;
          if (dc < D) {
            if constexpr (C::BF) {
              bf16x4 v;
#pragma unroll
              for (int j = 0; j < 4; ++j) v[j] = (bf16)o[t][4 * gq + j];
              *reinterpret_cast<bf16x4*>(orow + dc) = v;
            } else {
              f32x4 v;
#pragma unroll
              for (int j = 0; j < 4; ++j) v[j] = o[t][4 * gq + j];
              *reinterpret_cast<f32x4*>(orow + dc) = v;
            }
          }
        }
    }
  }
}

template <typename T, int D, int KB>
static int launch_temporal_long(const vp2p_temporal_attn_args* a, hipStream_t s) {
  using C = TempCfg<T, D>;
  const bool p2p = a->prompts > 0 && a->batch == (a->cond_only ? 1 : 2) * a->prompts;
  const int groups = p2p ? (a->cond_only ? 1 : 2) : a->batch;
  const int64_t nwg = (int64_t)groups * a->tokens * ((a->frames + 31) / 32);
  if (nwg <= 0 || nwg > 0x7fffffff) return VP2P_E_SHAPE;
  hipLaunchKernelGGL((temporal_attn_long_kernel<T, D, KB>), dim3((unsigned)nwg, (unsigned)((a->heads + 3) / 4)),
                     dim3(256), 4 * C::WAVE_LDS, s, *a);
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

template <typename T, int D>
static int launch_temporal(const vp2p_temporal_attn_args* a, hipStream_t s) {
  if (a->frames > 64) return launch_temporal_long<T, D, 4>(a, s);
  if (a->frames > 32) return launch_temporal_long<T, D, 2>(a, s);
  using C = TempCfg<T, D>;
  int lf = 0;
  while ((1 << lf) < a->frames) ++lf;
  const int G = 32 >> lf;
  const bool p2p = a->prompts > 0 && a->batch == (a->cond_only ? 1 : 2) * a->prompts;
  const int groups = p2p ? (a->cond_only ? 1 : 2) : a->batch;
  const int64_t nwg = (int64_t)groups * ((a->tokens + G - 1) / G);
  if (nwg <= 0 || nwg > 0x7fffffff) return VP2P_E_SHAPE;
  hipLaunchKernelGGL((temporal_attn_p2p_kernel<T, D, 4>), dim3((unsigned)nwg, (unsigned)((a->heads + 3) / 4)), dim3(256),
                     4 * C::WAVE_LDS, s, *a, lf);
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

}  // namespace vp2p

using namespace vp2p;

extern "C" int vp2p_temporal_attn_p2p_fwd(const vp2p_temporal_attn_args* a, void* stream) {
  if (!a || !a->q || !a->k || !a->v || !a->o) return VP2P_E_ARG;
  if (a->batch <= 0 || a->frames <= 0 || a->tokens <= 0 || a->heads <= 0 || a->head_dim <= 0)
    return VP2P_E_ARG;
  if (a->frames > 128) return VP2P_E_SHAPE;
  const int esz = a->dtype == VP2P_BF16 ? 2 : (a->dtype == VP2P_F32 ? 4 : 0);
  if (!esz) return VP2P_E_DTYPE;
  const int epc = 16 / esz;
  const int64_t strides[] = {a->q_sb, a->q_sf, a->q_sn, a->k_sb, a->k_sf, a->k_sn,
                             a->v_sb, a->v_sf, a->v_sn, a->o_sb, a->o_sf, a->o_sn};
  for (int64_t st : strides)
    if (st % epc) return VP2P_E_ARG;
  const void* ptrs[] = {a->q, a->k, a->v, a->o};
  for (const void* p : ptrs)
    if (reinterpret_cast<uintptr_t>(p) & 15) return VP2P_E_ARG;
  if (a->head_dim % epc) return VP2P_E_ARG;
  if (a->cond_only && !(a->prompts > 0 && a->batch == a->prompts)) return VP2P_E_ARG;
  if (a->self_replace && !(a->prompts > 0 && a->batch == (a->cond_only ? 1 : 2) * a->prompts)) return VP2P_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
#define VP2P_TEMP(DIM) \
  case DIM: return a->dtype == VP2P_BF16 ? launch_temporal<bf16, DIM>(a, s) : launch_temporal<float, DIM>(a, s);
  switch (a->head_dim) {
    VP2P_TEMP(32) VP2P_TEMP(40) VP2P_TEMP(64) VP2P_TEMP(80) VP2P_TEMP(128) VP2P_TEMP(160)
    default: return VP2P_E_HEAD_DIM;
  }
#undef VP2P_TEMP
}
