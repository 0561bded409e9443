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

// ------------------------------------------------------------------------------------------------
// K3s -- the res-64 form as a persistent stream (bf16, head_dim 40, 8 frames, q|k|v the three slices of
// one projection row, batch rows in pairs: the P2P source / edited prompt pair of a CFG half, or two
// plain rows).  Persistent workgroups (two per CU with the default 2-slot ring) walk items = (row pair,
// token); an item is the 2 x 8 frame rows of q|k|v (1920 B each, 30 KB), brought by LDS-DMA into a
// ring of NS slots, so NS - 1 items are in flight while one is computed.  The per-tile arithmetic is the short kernel's (same MFMAs, masks,
// roundings and self-replace): the outputs are bit-equal to it.
//  * every DMA instruction moves 1 KB of CONTIGUOUS global memory: a prompt's 8 rows, taken as one
//    15 KB run (row f at byte 1920 f), are its 15 lane-linear instructions, so each instruction covers
//    8 whole 128-byte lines and each line is requested once (a head-sliced fetch touched 16 half
//    lines per instruction, each line again by two or three later instructions: 2.7 TB/s read-only);
//  * the fragments are read from that natural image at per-lane offsets fixed for the whole stream
//    (a 16-byte chunk of q / k per k-step, 8-byte V pieces for the transposed reads);
//  * the outputs go through a per-wave LDS staging tile and leave as whole 320-byte row runs (16 bytes
//    a lane: 5 stores per item, not 10 scattered 8-byte stores over 32 rows each);
//  * wave w DMAs prompt w's rows and computes tile w (heads 4w .. 4w+3) of both prompts; the replaced
//    prompt's q / k lanes re-read a v chunk of their own instruction instead (no new lines), so its
//    q / k never leave HBM and every wave's vector-memory count per item stays fixed (counted vmcnt).
// ------------------------------------------------------------------------------------------------
// lab-only timing diagnostics (wrong results): bit 0 no output stores, 1 no compute, 2 no DMA
#ifndef VP2P_K3S_DIAG
#define VP2P_K3S_DIAG 0
#endif
// item order: 0 = strided over the grid (all workgroups sweep the tokens together), 1 = a contiguous
// run of items per workgroup (lab)
#ifndef VP2P_K3S_ORDER
#define VP2P_K3S_ORDER 0
#endif
namespace k3s {
constexpr int kD = 40, kF = 8, kW = 2, kDiag = VP2P_K3S_DIAG;
constexpr int kRow = 1920;                                     // one q|k|v row (3 x 320 bf16)
constexpr int kPrompt = kF * kRow;                             // 15 KB: a prompt's 8 frame rows
constexpr int kSlot = 2 * kPrompt;                             // 30 KB per item
constexpr int kDmaW = kPrompt / 1024;                          // 15 lane-linear 1 KB instructions a wave
constexpr int kStage = 2 * kF * 320;                           // per-wave output staging: [p][f][4 heads x 80 B]
constexpr int kStW = kStage / 1024;                            // 5 output stores a wave per item
// ring of NS slots: LDS, and the in-order vmcnt that retires a wave's DMA of item k (issued after it:
// the stores of items k-NS+1 .. k-1 and the DMA of items k+1 .. k+NS-2)
template <int NS> struct Ring {
  static constexpr int kStg = NS * kSlot;                      // staging tiles of the two waves
  static constexpr int kZero = kStg + kW * kStage + 128;       // 16 zero bytes on bank 32
  static constexpr int kLds = kZero + 128;
  static constexpr int kYoung = (NS - 1) * kStW + (NS - 2) * kDmaW;
  static_assert(kYoung <= 63, "counted vmcnt");
  static_assert((kZero / 4) % 64 == 32, "zero run on bank 32");
};
static_assert(kPrompt % 1024 == 0 && kStage % 1024 == 0, "whole 1 KB instructions");
typedef __attribute__((address_space(3))) char lchar;
__device__ __forceinline__ bf16x8 ld128(const lchar* p) { return *reinterpret_cast<const __attribute__((address_space(3))) bf16x8*>(p); }
__device__ __forceinline__ bf16x4 ldtr(const lchar* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4*)(p));
}
}  // namespace k3s

template <int kNS>
__global__ __launch_bounds__(64 * k3s::kW, 1) void temporal_attn_stream_kernel(const vp2p_temporal_attn_args a) {
  using namespace k3s;
  using M = Mfma<bf16>;
  constexpr int kZero = Ring<kNS>::kZero, kYoung = Ring<kNS>::kYoung;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  lchar* const L = (lchar*)smem;
  const int tid = threadIdx.x, l = tid & 63, r = l & 31, h = l >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int N = a.tokens;
  const int items = (a.batch / 2) * N;
  const int G = gridDim.x, g0 = blockIdx.x;
#if VP2P_K3S_ORDER
  const int per = (items + G - 1) / G, first = g0 * per;
  const int nmine = first < items ? min(per, items - first) : 0;
  auto item_of = [&](int k) { return first + k; };
#else
  const int nmine = g0 < items ? (items - g0 + G - 1) / G : 0;
  auto item_of = [&](int k) { return g0 + k * G; };
#endif
  const bool p2p = a.prompts > 0;                 // launcher: p2p => prompts == 2 (a row pair)
  const float cs = a.scale * kLog2e;

  // one buffer resource over the fused q|k|v rows (32-bit offsets: checked by the launcher)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(a.q), 0, (uint32_t)((int64_t)a.batch * a.q_sb * 2), 0x00020000);
  // lane l of instruction m moves bytes [1024 m + 16 l, +16) of prompt w's 15 KB run; the replaced
  // prompt's q / k lanes re-read the first v chunk of a row of the same instruction
  uint32_t voff[kDmaW], vrep[kDmaW];
#pragma unroll
  for (int m = 0; m < kDmaW; ++m) {
    const int v = 1024 * m + 16 * l, f = v / kRow, o = v - f * kRow;
    voff[m] = (uint32_t)((w * a.q_sb + f * a.q_sf) * 2 + o);
    const int f1 = (1024 * m) / kRow, o1 = 1024 * m - f1 * kRow;   // the instruction's first row
    const int fv = o1 < 1280 ? f1 : (f1 + 1 < kF ? f1 + 1 : f1);   // a row whose v chunk it covers
    vrep[m] = o >= 1280 ? voff[m] : (uint32_t)((w * a.q_sb + fv * a.q_sf) * 2 + (fv == f1 && o1 > 1280 ? o1 : 1280));
  }
  const uint32_t lds_base = (uint32_t)(uintptr_t)L;
  auto dma = [&](int k) {
    if constexpr ((kDiag & 4) != 0) return;
    const int it = item_of(k);
    const int pg = it / N, n = it - pg * N;
    const bool skip_qk = p2p && a.self_replace && (a.cond_only || pg == 1) && w == 1;
    const uint32_t so = (uint32_t)((2 * pg * a.q_sb + n * a.q_sn) * 2);
    const uint32_t dst = lds_base + (uint32_t)((k % kNS) * kSlot + w * kPrompt);
#pragma unroll
    for (int m = 0; m < kDmaW; ++m) {
      const uint32_t m0 = __builtin_amdgcn_readfirstlane(dst + m * 1024);
      asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
                   :: "v"(skip_qk ? vrep[m] : voff[m]), "s"(rs), "{m0}"(m0), "s"(so) : "memory");
    }
  };
  for (int i = tid; i < 8; i += 64 * kW) reinterpret_cast<__attribute__((address_space(3))) u32x4*>(L + kZero)[i] = u32x4{0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < kNS - 1; ++k)
    if (k < nmine) dma(k);

  // per-lane fragment offsets within a prompt's image (tile w: query / key row r = 8 (head - 4w) + f)
  const int slot_q = r >> 3, head = 4 * w + slot_q, fr = r & 7;
  const int q_s0 = fr * kRow + head * 80 + 16 * (0 + h);
  const int q_s1 = fr * kRow + head * 80 + 16 * (2 + h);
  const int q_s2 = fr * kRow + head * 80 + 64;                  // lanes h == 0 (dims 32..39)
  const int vg = (l >> 4) & 1, q4 = (l >> 2) & 3, p4 = l & 3;
  const bool vt1 = vg == 0 && p4 < 2;            // V^T tile 1 provider lanes (dims 32..39)
  int v_off[2][2][2];                            // [sp][t][lo / hi]; -1: the zero run
#pragma unroll
  for (int sp = 0; sp < 2; ++sp)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int hi = 0; hi < 2; ++hi) {
        const int R = 16 * sp + 4 * h + q4 + 8 * hi, hd = 4 * w + (R >> 3), f = R & 7;
        const int col = t == 0 ? 16 * vg + 4 * p4 : 32 + 4 * p4;
        v_off[sp][t][hi] = (t == 0 || vt1) ? f * kRow + 1280 + hd * 80 + 2 * col : -1;
      }
  lchar* const stg = L + Ring<kNS>::kStg + w * kStage;

  for (int k = 0; k < nmine; ++k) {
    if (k >= kNS - 1 && k + kNS - 2 < nmine) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kYoung) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();            // item k landed (every wave's DMA); item k-1's slot free
    if (k + kNS - 1 < nmine) dma(k + kNS - 1);
    const int it = item_of(k);
    const int pg = it / N, n = it - pg * N;
    const bool rep = p2p && a.self_replace && (a.cond_only || pg == 1);
    const lchar* slot = L + (k % kNS) * kSlot;
    M::frag psrc[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const lchar* I = slot + p * kPrompt;
      M::frag pf[2];
      if constexpr ((kDiag & 2) != 0) {
        pf[0] = pf[1] = M::zero();
      } else if (rep && p > 0) {
        pf[0] = psrc[0];
        pf[1] = psrc[1];
      } else {
        const bf16x8 q0 = ld128(I + q_s0), q1 = ld128(I + q_s1), q2 = ld128(h ? L + kZero : I + q_s2);
        const bf16x8 k0 = ld128(I + 640 + q_s0), k1 = ld128(I + 640 + q_s1), k2 = ld128(h ? L + kZero : I + 640 + q_s2);
        f32x16 sc = M::mma(k0, q0, zero16());
        sc = M::mma(k1, q1, sc);
        sc = M::mma(k2, q2, sc);
        float mx = kNegInf;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const bool ok = (acc_row(i, h) >> 3) == slot_q;
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
        pf[0] = M::p_frag(sc, 0);
        pf[1] = M::p_frag(sc, 1);
        if (rep) {
          psrc[0] = pf[0];
          psrc[1] = pf[1];
        }
      }
      f32x16 o[2] = {zero16(), zero16()};
      if constexpr ((kDiag & 2) == 0) {
#pragma unroll
        for (int sp = 0; sp < 2; ++sp)
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const int ol = v_off[sp][t][0], oh = v_off[sp][t][1];
            const bf16x4 lo = ldtr(ol >= 0 ? I + ol : L + kZero), hi = ldtr(oh >= 0 ? I + oh : L + kZero);
            bf16x8 vf;
#pragma unroll
            for (int j = 0; j < 4; ++j) { vf[j] = lo[j]; vf[4 + j] = hi[j]; }
            o[t] = M::mma(vf, pf[sp], o[t]);
          }
      }
      // O^T (query on the lane) -> the staging tile [p][frame][4 heads x 80 B]
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq)
          if (32 * t + 8 * gq < kD) {
            bf16x4 v;
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = (bf16)o[t][4 * gq + j];
            *reinterpret_cast<__attribute__((address_space(3))) bf16x4*>(
                stg + p * (kF * 320) + fr * 320 + slot_q * 80 + 2 * (32 * t + 8 * gq + 4 * h)) = v;
          }
    }
    if constexpr ((kDiag & 1) != 0) continue;
    // whole 320-byte row runs (heads 4w .. 4w+3 of a (prompt, frame) row), 16 bytes a lane
#pragma unroll
    for (int i = 0; i < kStW; ++i) {
      const int c = 64 * i + l, p = c / (kF * 20), cc = c - p * (kF * 20), f = cc / 20, e = cc - f * 20;
      const u32x4 v = *reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(stg + 16 * c);
      char* orow = static_cast<char*>(a.o) + 2 * ((2 * pg + p) * a.o_sb + f * a.o_sf + (int64_t)n * a.o_sn + 4 * w * kD);
      *reinterpret_cast<u32x4*>(orow + 16 * e) = v;
    }
  }
}

// the stream applies to: bf16, d 40, 8 frames, rows in pairs, no probability output, enough items to
// keep every CU streaming, 32-bit byte offsets within each operand
static int stream_cus() {
  static int n_cu_of[64] = {};
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
  if (dev < 64) n = n_cu_of[dev];
  if (!n) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    if (dev < 64) n_cu_of[dev] = n;
  }
  return n;
}

// lab A/B switch VP2P_K3_STREAM: 0 = the short kernel everywhere, 2 / 3 / 4 = the ring depth.
// Default 2: two workgroups per CU with one item in flight each measured fastest with q|k|v just
// written by their projection (as in the edit): res-64 B4 self-replace 52.2 us (ring 3: 57.0, ring 4:
// 57.9; the short kernel 83.6), profiles/r06_k3s_ab.jsonl
static int stream_ring() {
  const char* e = getenv("VP2P_K3_STREAM");
  if (e && e[0] >= '0' && e[0] <= '4' && e[0] != '1') return e[0] - '0';
  return 2;
}

static bool stream_applies(const vp2p_temporal_attn_args* a, int n_cu) {
  if (a->dtype != VP2P_BF16 || a->head_dim != 40 || a->frames != 8 || a->probs_out || a->heads != 8) return false;
  const bool p2p = a->prompts > 0 && a->batch == (a->cond_only ? 1 : 2) * a->prompts;
  if (p2p ? a->prompts != 2 : (a->prompts > 0 || a->batch % 2)) return false;
  if ((int64_t)(a->batch / 2) * a->tokens < 8 * (int64_t)n_cu) return false;
  // q, k, v: the three 320-wide slices of one 960-wide projection row, same strides
  const char* q = static_cast<const char*>(a->q);
  if (static_cast<const char*>(a->k) != q + 640 || static_cast<const char*>(a->v) != q + 1280) return false;
  if (a->k_sb != a->q_sb || a->v_sb != a->q_sb || a->k_sf != a->q_sf || a->v_sf != a->q_sf ||
      a->k_sn != a->q_sn || a->v_sn != a->q_sn || a->q_sn < 960)
    return false;
  // every row of an item inside the batch stride, all offsets within 32 bits
  if (a->q_sb < 8 * a->q_sf || a->q_sf < (int64_t)a->tokens * a->q_sn) return false;
  if (a->batch * a->q_sb * 2 >= ((int64_t)1 << 32)) return false;
  return true;
}

template <int NS>
static int launch_temporal_stream(const vp2p_temporal_attn_args* a, hipStream_t s, int n_cu) {
  constexpr int lds = k3s::Ring<NS>::kLds;
  static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&temporal_attn_stream_kernel<NS>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
  if (!attr) return VP2P_E_LAUNCH;
  const int64_t items = (int64_t)(a->batch / 2) * a->tokens;
  const int64_t per_cu = (160 * 1024) / lds;                       // co-resident workgroups per CU
  const int64_t want = per_cu * n_cu;
  const int grid = (int)(items < want ? items : want);
  vp2p_temporal_attn_args b = *a;
  if (!(a->prompts > 0 && a->batch == (a->cond_only ? 1 : 2) * a->prompts)) b.prompts = 0;   // plain rows
  hipLaunchKernelGGL((temporal_attn_stream_kernel<NS>), dim3((unsigned)grid), dim3(64 * k3s::kW), lds, s, b);
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
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
  if constexpr (sizeof(T) == 2 && D == 40) {
    const int n_cu = stream_cus(), ring = stream_ring();
    if (ring && stream_applies(a, n_cu)) {
      if (ring == 2) return launch_temporal_stream<2>(a, s, n_cu);
      if (ring == 3) return launch_temporal_stream<3>(a, s, n_cu);
      return launch_temporal_stream<4>(a, s, n_cu);
    }
  }
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
