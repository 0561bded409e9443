// K1 — FrameAttention with first-frame K/V (tuneavideo/models/attention.py:282-322).
//
// Reference semantics: every frame's queries attend to the keys/values of frame 0 of the same
// batch element ('key[:, [0] * video_length]', attention.py:296-302), plain row softmax with scale
// head_dim**-0.5 (diffusers _attention / xformers, :314-322).  The reference materialises the gather
// (f copies of frame-0 K/V) and, without xformers, the (B*f*h, HW, HW) score tensor.
//
// MI355X design:
//  * K/V are only ever the B*h distinct frame-0 tensors; the f*HW queries of one (b, head) form one
//    long query axis, so a workgroup = 128 query rows (4 waves x 32) of one (b, head) streams
//    frame-0 K/V tiles through LDS, and the grid is XCD-remapped so the workgroups of one (b, head)
//    share an L2.
//  * swapped 32x32 MFMA tiles (common.hpp): softmax is lane-local, P never leaves registers,
//    V is read transposed from its row-major LDS image with ds_read_b64_tr_b16.
//  * the kernel is VALU-bound at d = 40 (7 MFMAs per 32x32 block against 16 scores per lane), so the
//    per-score VALU work is cut to max3 + fma + exp2 + cvt:
//      - scores stay unscaled; p = exp2(s * c - m) is one v_fma + one v_exp,
//      - the row sum rides in the MFMA: a spare row of the padded V^T (d = 40 -> 64 rows) is all
//        ones, so O^T's row `D` accumulates sum_k P (rescaled together with O),
//      - lazy rescale: m only moves when the block max exceeds it by > kRescaleThr (log2 units),
//        so O is rarely touched; P <= 2^kRescaleThr in between (bf16-safe, fp32 accumulators),
//      - masking only on the ragged last tile.
//  * next K/V tile prefetched into registers while the current one is consumed
//    (issue early / write late); two barriers per 128-key tile.
//  * bf16, d <= 64 (the res-64 layers, 88% of the FLOPs): frame_attn_kernel_x2 gives every wave
//    64 query rows as two independent 32-row sets sharing each K/V fragment read (half the LDS
//    traffic per query, two independent MFMA/VALU chains per wave): +5% over one set per wave in
//    an interleaved A/B (profiles/r01_k1_ab.txt).
#include <stdlib.h>

#include <type_traits>

#include "common.hpp"
#include "vp2p.h"

namespace vp2p {

constexpr float kRescaleThr = 8.0f;

template <typename T, int D>
struct FrameCfg {
  static constexpr bool BF = sizeof(T) == 2;
  static constexpr int KD = Mfma<T>::KD;
  static constexpr int DP = round_up(D, KD);
  static constexpr int KS = DP / KD;
  static constexpr int DV = round_up(D, 32);
  static constexpr int NT = DV / 32;
  static constexpr bool ONES = D < DV;                           // spare V^T row carries the row sum
  static constexpr int KT = (BF && D <= 80) ? 128 : 64;          // keys per LDS tile
  static constexpr int NB = D <= 80 ? 2 : 1;                     // 32-key score blocks in flight
  static constexpr int SUBK = 32 * NB;
  static constexpr int EPC = 16 / (int)sizeof(T);                // elements per 16-byte chunk
  static constexpr int CPR = D / EPC;                            // chunks per K/V row
  static constexpr int NCH = (KT * CPR + 255) / 256;             // chunks per thread per tile
  // bf16: K rows read with ds_read_b128 by 16-lane groups -> stride = 4 (mod 8) dwords;
  //       V rows read with ds_read_b64_tr_b16 -> stride = 16 or 48 (mod 64) dwords.
  // f32 : K read one dword per lane down a column -> odd stride; V read along rows.
  static constexpr int vrow_bf16() {
    int v = DV;
    while (!((v / 2) % 64 == 16 || (v / 2) % 64 == 48)) v += 8;
    return v;
  }
  static constexpr int KROW = BF ? DP + 8 : DP + 1;
  static constexpr int VROW = BF ? vrow_bf16() : DV;
  static constexpr int LDS_BYTES = (KT * KROW + KT * VROW) * (int)sizeof(T);
  // accumulator slot of O^T row D (the ones row): tile, register, lane half
  static constexpr int ONE_T = D / 32, ONE_L = D % 32;
  static constexpr int ONE_H = (ONE_L >> 2) & 1, ONE_I = (ONE_L & 3) + 4 * (ONE_L >> 3);
};

template <typename T, int D>
__global__ __launch_bounds__(256, sizeof(T) == 2 ? 2 : 1) void frame_attn_kernel(const vp2p_frame_attn_args a) {
  using M = Mfma<T>;
  using C = FrameCfg<T, D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* Ks = reinterpret_cast<T*>(smem);
  T* Vs = Ks + C::KT * C::KROW;

  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, r = l & 31, h = l >> 5;
  const int FQ = a.frames * a.tokens_q;
  const int qblocks = (FQ + 127) >> 7;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = bid / qblocks, qb = bid - bh * qblocks;
  const int b = bh / a.heads, head = bh - b * a.heads;
  const int Nk = a.tokens_kv;

  const int qi = qb * 128 + w * 32 + r;
  const bool qv = qi < FQ;
  const int fr = qv ? qi / a.tokens_q : 0;
  const int pos = qv ? qi - fr * a.tokens_q : 0;
  const T* qrow = static_cast<const T*>(a.q) + b * a.q_sb + fr * a.q_sf + pos * a.q_sn + head * D;
  typename M::frag qf[C::KS];
#pragma unroll
  for (int s = 0; s < C::KS; ++s) qf[s] = qv ? M::row_frag(qrow, s, h, D) : M::zero();

  // LDS image: zero once (padding columns are never rewritten); the ones column of V
  for (int i = tid; i < C::LDS_BYTES / 16; i += 256) reinterpret_cast<u32x4*>(smem)[i] = u32x4{0, 0, 0, 0};
  if constexpr (C::ONES) {
    __syncthreads();
    for (int k = tid; k < C::KT; k += 256) Vs[k * C::VROW + D] = (T)1.0f;
  }

  const T* kbase = static_cast<const T*>(a.k) + b * a.k_sb + head * D;
  const T* vbase = static_cast<const T*>(a.v) + b * a.v_sb + head * D;
  u32x4 kreg[C::NCH], vreg[C::NCH];

  auto load_tile = [&](int kt) {
#pragma unroll
    for (int i = 0; i < C::NCH; ++i) {
      const int c = tid + i * 256;
      const int row = c / C::CPR, col = (c - row * C::CPR) * C::EPC;
      const int key = kt + row;
      if (c < C::KT * C::CPR && key < Nk) {
        kreg[i] = *reinterpret_cast<const u32x4*>(kbase + (int64_t)key * a.k_sn + col);
        vreg[i] = *reinterpret_cast<const u32x4*>(vbase + (int64_t)key * a.v_sn + col);
      } else {
        kreg[i] = u32x4{0, 0, 0, 0};
        vreg[i] = u32x4{0, 0, 0, 0};
      }
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < C::NCH; ++i) {
      const int c = tid + i * 256;
      if (c < C::KT * C::CPR) {
        const int row = c / C::CPR, col = (c - row * C::CPR) * C::EPC;
        if constexpr (C::BF) {
          *reinterpret_cast<u32x4*>(Ks + row * C::KROW + col) = kreg[i];
        } else {
          float* kd = reinterpret_cast<float*>(Ks) + row * C::KROW + col;
#pragma unroll
          for (int j = 0; j < 4; ++j) kd[j] = __uint_as_float(kreg[i][j]);
        }
        *reinterpret_cast<u32x4*>(Vs + row * C::VROW + col) = vreg[i];
      }
    }
  };

  const float cs = a.scale * kLog2e;
  float m = kNegInf;            // running max of s*cs (log2 units), shared by lanes r and r+32
  float lsum = 0.f;             // only without the ones row
  f32x16 o[C::NT];
#pragma unroll
  for (int t = 0; t < C::NT; ++t) o[t] = zero16();

  // one K/V tile: QK^T, online softmax, PV.  MASKED only for the ragged last tile, so the hot loop
  // carries no per-score key-bound compare/select.
  auto compute_tile = [&](int kt, auto masked_tag) {
    constexpr bool MASKED = decltype(masked_tag)::value;
  #pragma unroll
      for (int sub = 0; sub < C::KT / C::SUBK; ++sub) {
        const int key0 = sub * C::SUBK;
        if (MASKED && kt + key0 >= Nk) break;
        f32x16 sc[C::NB];
  #pragma unroll
        for (int nb = 0; nb < C::NB; ++nb) sc[nb] = zero16();
  #pragma unroll
        for (int si = 0; si < C::KS; ++si) {
  #pragma unroll
          for (int nb = 0; nb < C::NB; ++nb) {
            const T* krow = Ks + (key0 + 32 * nb + r) * C::KROW;
            typename M::frag af;
            if constexpr (C::BF) af = *reinterpret_cast<const bf16x8*>(krow + 16 * si + 8 * h);
            else af = krow[2 * si + h];
            sc[nb] = M::mma(af, qf[si], sc[nb]);
          }
        }
        if constexpr (MASKED) {
  #pragma unroll
          for (int nb = 0; nb < C::NB; ++nb)
  #pragma unroll
            for (int i = 0; i < 16; ++i)
              if (kt + key0 + 32 * nb + acc_row(i, h) >= Nk) sc[nb][i] = kNegInf;
        }
        float mx = sc[0][0];
  #pragma unroll
        for (int nb = 0; nb < C::NB; ++nb)
  #pragma unroll
          for (int i = 0; i < 16; ++i) mx = fmaxf(mx, sc[nb][i]);
        mx = fmaxf(mx, xhalf(mx)) * cs;
        if (__any(mx > m + kRescaleThr)) {
          const float mn = fmaxf(m, mx);
          const float alpha = fast_exp2(m - mn);
          m = mn;
  #pragma unroll
          for (int t = 0; t < C::NT; ++t)
  #pragma unroll
            for (int i = 0; i < 16; ++i) o[t][i] *= alpha;
          if constexpr (!C::ONES) lsum *= alpha;
        }
        const float nm = -m;
  #pragma unroll
        for (int nb = 0; nb < C::NB; ++nb)
  #pragma unroll
          for (int i = 0; i < 16; ++i) sc[nb][i] = fast_exp2(__builtin_fmaf(sc[nb][i], cs, nm));
        if constexpr (!C::ONES) {
  #pragma unroll
          for (int nb = 0; nb < C::NB; ++nb)
  #pragma unroll
            for (int i = 0; i < 16; ++i) lsum += sc[nb][i];
        }
  #pragma unroll
        for (int nb = 0; nb < C::NB; ++nb) {
  #pragma unroll
          for (int sp = 0; sp < M::PV_STEPS; ++sp) {
            const typename M::frag pf = M::p_frag(sc[nb], sp);
  #pragma unroll
            for (int t = 0; t < C::NT; ++t) {
              typename M::frag vf;
              if constexpr (C::BF) vf = vt_frag_lds<C::VROW>(Vs, key0 + 32 * nb, sp, t);
              else vf = Vs[(key0 + 32 * nb + f32_pv_key(sp, h)) * C::VROW + 32 * t + r];
              o[t] = M::mma(vf, pf, o[t]);
            }
          }
        }
      }

  };

  load_tile(0);
  int kt = 0;
  for (; kt + C::KT <= Nk; kt += C::KT) {
    __syncthreads();
    store_tile();
    __syncthreads();
    if (kt + C::KT < Nk) load_tile(kt + C::KT);
    compute_tile(kt, std::false_type{});
  }
  if (kt < Nk) {
    __syncthreads();
    store_tile();
    __syncthreads();
    compute_tile(kt, std::true_type{});
  }

  float lrow;
  if constexpr (C::ONES) {
    const float mine = o[C::ONE_T][C::ONE_I];
    const float other = xhalf(mine);
    lrow = (h == C::ONE_H) ? mine : other;
  } else {
    lrow = lsum + xhalf(lsum);
  }
  if (a.lse && qv) a.lse[(int64_t)(b * a.heads + head) * FQ + qi] = m + log2f(lrow);
  if (qv) {
    const float inv = 1.f / lrow;
    T* orow = static_cast<T*>(a.o) + b * a.o_sb + fr * a.o_sf + pos * a.o_sn + head * D;
#pragma unroll
    for (int t = 0; t < C::NT; ++t) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int dc = 32 * t + 8 * g + 4 * h;
        if (dc < D) {
          if constexpr (C::BF) {
            bf16x4 v;
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = (bf16)(o[t][4 * g + j] * inv);
            *reinterpret_cast<bf16x4*>(orow + dc) = v;
          } else {
            f32x4 v;
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = o[t][4 * g + j] * inv;
            *reinterpret_cast<f32x4*>(orow + dc) = v;
          }
        }
      }
    }
  }
}

// Variant with 64 query rows per wave: two independent 32-row sets share every K/V fragment read
// (half the LDS traffic per query) and give the scheduler two independent MFMA/VALU chains.
// bf16, head dims with a spare ones row (d = 32 excluded), d <= 64.
template <int D>
__global__ __launch_bounds__(256, 2) void frame_attn_kernel_x2(const vp2p_frame_attn_args a) {
  using T = bf16;
  using M = Mfma<T>;
  using C = FrameCfg<T, D>;
  static_assert(C::ONES && D <= 64, "x2 variant: bf16, spare ones row");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* Ks = reinterpret_cast<T*>(smem);
  T* Vs = Ks + C::KT * C::KROW;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, r = l & 31, h = l >> 5;
  const int FQ = a.frames * a.tokens_q;
  const int qblocks = (FQ + 255) >> 8;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = bid / qblocks, qb = bid - bh * qblocks;
  const int b = bh / a.heads, head = bh - b * a.heads;
  const int Nk = a.tokens_kv;

  int qi[2], fr[2], pos[2];
  bool qv[2];
  bf16x8 qf[2][C::KS];
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    qi[st] = qb * 256 + w * 64 + st * 32 + r;
    qv[st] = qi[st] < FQ;
    fr[st] = qv[st] ? qi[st] / a.tokens_q : 0;
    pos[st] = qv[st] ? qi[st] - fr[st] * a.tokens_q : 0;
    const T* qrow = static_cast<const T*>(a.q) + b * a.q_sb + fr[st] * a.q_sf + pos[st] * a.q_sn + head * D;
#pragma unroll
    for (int s = 0; s < C::KS; ++s) qf[st][s] = qv[st] ? M::row_frag(qrow, s, h, D) : M::zero();
  }
  for (int i = tid; i < C::LDS_BYTES / 16; i += 256) reinterpret_cast<u32x4*>(smem)[i] = u32x4{0, 0, 0, 0};
  __syncthreads();
  for (int k = tid; k < C::KT; k += 256) Vs[k * C::VROW + D] = (T)1.0f;

  const T* kbase = static_cast<const T*>(a.k) + b * a.k_sb + head * D;
  const T* vbase = static_cast<const T*>(a.v) + b * a.v_sb + head * D;
  u32x4 kreg[C::NCH], vreg[C::NCH];
  auto load_tile = [&](int kt) {
#pragma unroll
    for (int i = 0; i < C::NCH; ++i) {
      const int c = tid + i * 256;
      const int row = c / C::CPR, col = (c - row * C::CPR) * C::EPC;
      const int key = kt + row;
      if (c < C::KT * C::CPR && key < Nk) {
        kreg[i] = *reinterpret_cast<const u32x4*>(kbase + (int64_t)key * a.k_sn + col);
        vreg[i] = *reinterpret_cast<const u32x4*>(vbase + (int64_t)key * a.v_sn + col);
      } else {
        kreg[i] = u32x4{0, 0, 0, 0};
        vreg[i] = u32x4{0, 0, 0, 0};
      }
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < C::NCH; ++i) {
      const int c = tid + i * 256;
      if (c < C::KT * C::CPR) {
        const int row = c / C::CPR, col = (c - row * C::CPR) * C::EPC;
        *reinterpret_cast<u32x4*>(Ks + row * C::KROW + col) = kreg[i];
        *reinterpret_cast<u32x4*>(Vs + row * C::VROW + col) = vreg[i];
      }
    }
  };

  const float cs = a.scale * kLog2e;
  float m[2] = {kNegInf, kNegInf};
  f32x16 o[2][C::NT];
#pragma unroll
  for (int st = 0; st < 2; ++st)
#pragma unroll
    for (int t = 0; t < C::NT; ++t) o[st][t] = zero16();

  auto compute_tile = [&](int kt, auto masked_tag) {
    constexpr bool MASKED = decltype(masked_tag)::value;
#pragma unroll
    for (int key0 = 0; key0 < C::KT; key0 += 32) {
      if (MASKED && kt + key0 >= Nk) break;
      f32x16 s[2] = {zero16(), zero16()};
#pragma unroll
      for (int si = 0; si < C::KS; ++si) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(Ks + (key0 + r) * C::KROW + 16 * si + 8 * h);
        s[0] = M::mma(af, qf[0][si], s[0]);
        s[1] = M::mma(af, qf[1][si], s[1]);
      }
      float mx[2];
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        if constexpr (MASKED) {
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (kt + key0 + acc_row(i, h) >= Nk) s[st][i] = kNegInf;
        }
        float v = s[st][0];
#pragma unroll
        for (int i = 1; i < 16; ++i) v = fmaxf(v, s[st][i]);
        mx[st] = fmaxf(v, xhalf(v)) * cs;
      }
      if (__any(mx[0] > m[0] + kRescaleThr || mx[1] > m[1] + kRescaleThr)) {
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const float mn = fmaxf(m[st], mx[st]);
          const float alpha = fast_exp2(m[st] - mn);
          m[st] = mn;
#pragma unroll
          for (int t = 0; t < C::NT; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) o[st][t][i] *= alpha;
        }
      }
      bf16x8 pf[2][2];
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const float nm = -m[st];
#pragma unroll
        for (int i = 0; i < 16; ++i) s[st][i] = fast_exp2(__builtin_fmaf(s[st][i], cs, nm));
        pf[st][0] = M::p_frag(s[st], 0);
        pf[st][1] = M::p_frag(s[st], 1);
      }
#pragma unroll
      for (int sp = 0; sp < 2; ++sp)
#pragma unroll
        for (int t = 0; t < C::NT; ++t) {
          const bf16x8 vf = vt_frag_lds<C::VROW>(Vs, key0, sp, t);
          o[0][t] = M::mma(vf, pf[0][sp], o[0][t]);
          o[1][t] = M::mma(vf, pf[1][sp], o[1][t]);
        }
    }
  };

  load_tile(0);
  int kt = 0;
  for (; kt + C::KT <= Nk; kt += C::KT) {
    __syncthreads();
    store_tile();
    __syncthreads();
    if (kt + C::KT < Nk) load_tile(kt + C::KT);
    compute_tile(kt, std::false_type{});
  }
  if (kt < Nk) {
    __syncthreads();
    store_tile();
    __syncthreads();
    compute_tile(kt, std::true_type{});
  }
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    const float mine = o[st][C::ONE_T][C::ONE_I];
    const float other = xhalf(mine);
    const float lrow = (h == C::ONE_H) ? mine : other;
    if (a.lse && qv[st]) a.lse[(int64_t)(b * a.heads + head) * FQ + qi[st]] = m[st] + log2f(lrow);
    if (qv[st]) {
      const float inv = 1.f / lrow;
      T* orow = static_cast<T*>(a.o) + b * a.o_sb + fr[st] * a.o_sf + pos[st] * a.o_sn + head * D;
#pragma unroll
      for (int t = 0; t < C::NT; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int dc = 32 * t + 8 * g + 4 * h;
          if (dc < D) {
            bf16x4 v;
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = (bf16)(o[st][t][4 * g + j] * inv);
            *reinterpret_cast<bf16x4*>(orow + dc) = v;
          }
        }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// v3: bf16, d = 40 (the res-64 layers, 88% of the FLOPs).  Two changes over frame_attn_kernel_x2:
//  * the running max is folded into the QK^T MFMA.  d = 40 pads to a 48-wide K-dim, so K carries a
//    constant 1 in column 40 and Q (pre-scaled by scale*log2 e) carries -m in that column: the MFMA
//    returns s*scale*log2e - m directly and p = exp2(acc) is ONE VALU op per score (no fma).  m is
//    kept as a bf16 value (exact in the MFMA); softmax is invariant to it, so its rounding does not
//    matter, only the lazy-rescale bound does.  The per-block max is only needed to detect the rare
//    case "some score exceeds m + kRescaleThr" (one v_max3 chain + one wave vote, no cross-lane
//    exchange); then m moves, O (and its ones-row sum) is rescaled and Q's column 40 is rewritten.
//  * K/V tiles stream global -> LDS with global_load_lds_dwordx4 (no VGPR staging, no compiler
//    vmcnt(0) before the first MFMA of a tile), double buffered, one barrier per 128-key tile.  The
//    LDS image is plane-major: plane c holds 16-byte piece c (8 channels) of every key, planes
//    2112 B apart (16 banks), so K row reads (ds_read_b128) and V^T transposed reads
//    (ds_read_b64_tr_b16) are both conflict-free.  Constant planes supply K's column 40 (= 1), V's
//    ones row (d = 40, the row sum rides in the PV MFMA) and V's zero rows 41..63.
// ------------------------------------------------------------------------------------------------
namespace k1v3 {
constexpr int D = 40;
constexpr int KT = 128;                    // keys per tile
constexpr int CSTRIDE = KT * 16 + 64;      // bytes per plane (+64 B: consecutive planes 16 banks apart)
constexpr int KPL = 6;                     // K planes: d 0..39 + [1, 0 x 7]
constexpr int VPL = 8;                     // V planes: d 0..39 + [1, 0 x 7] + 2 zero planes (d 48..63)
constexpr int KBYTES = KPL * CSTRIDE, VBYTES = VPL * CSTRIDE;
constexpr int BUF = KBYTES + VBYTES;
constexpr int LDS_BYTES = 2 * BUF;
constexpr int DATA_PL = D / 8;             // 5 planes loaded per tile
}  // namespace k1v3

__device__ __forceinline__ bf16x8 vt_frag_planes(const char* vbuf, int key0, int sp, int t) {
  const int l = lane_id();
  const int h = l >> 5, g = (l >> 4) & 1, q = (l >> 2) & 3, p = l & 3;
  const int c0 = 32 * t + 16 * g + 4 * p;
  const char* base = vbuf + (c0 >> 3) * k1v3::CSTRIDE + (c0 & 7) * 2 + (key0 + 16 * sp + 4 * h + q) * 16;
  const bf16x4 lo = lds_read_tr(reinterpret_cast<const bf16*>(base));
  const bf16x4 hi = lds_read_tr(reinterpret_cast<const bf16*>(base + 8 * 16));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

template <int UNR>
__global__ __launch_bounds__(256, 2) void frame_attn_kernel_v3(const vp2p_frame_attn_args a) {
  using namespace k1v3;
  using M = Mfma<bf16>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, r = l & 31, h = l >> 5;
  const int FQ = a.frames * a.tokens_q;
  const int qblocks = (FQ + 255) >> 8;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = bid / qblocks, qb = bid - bh * qblocks;
  const int b = bh / a.heads, head = bh - b * a.heads;
  const int Nk = a.tokens_kv;
  const float cs = a.scale * kLog2e;

  // constant planes of both stages: K plane 5 / V plane 5 = [1, 0 x 7] per key, V planes 6, 7 = 0
  for (int i = tid; i < 2 * KT; i += 256) {
    char* st = smem + (i >= KT ? BUF : 0);
    const int k = i & (KT - 1);
    const u32x4 one = {0x3F80u, 0u, 0u, 0u};
    *reinterpret_cast<u32x4*>(st + 5 * CSTRIDE + k * 16) = one;
    *reinterpret_cast<u32x4*>(st + KBYTES + 5 * CSTRIDE + k * 16) = one;
    *reinterpret_cast<u32x4*>(st + KBYTES + 6 * CSTRIDE + k * 16) = u32x4{0, 0, 0, 0};
    *reinterpret_cast<u32x4*>(st + KBYTES + 7 * CSTRIDE + k * 16) = u32x4{0, 0, 0, 0};
  }

  const bf16* kbase = static_cast<const bf16*>(a.k) + (int64_t)b * a.k_sb + head * D;
  const bf16* vbase = static_cast<const bf16*>(a.v) + (int64_t)b * a.v_sb + head * D;
  // one tile = 2 tensors x 5 planes x 2 halves of 64 keys = 20 wave-wide DMA pieces, 5 per wave
  auto issue_tile = [&](int kt, int stage) {
    char* st = smem + stage * BUF;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int id = w + 4 * j;
      const int x = id >= 10 ? 1 : 0, rem = id - 10 * x, c = rem >> 1, hf = rem & 1;
      int key = kt + hf * 64 + l;
      key = key < Nk ? key : Nk - 1;                      // clamp: those keys are masked
      const bf16* src = (x ? vbase + (int64_t)key * a.v_sn : kbase + (int64_t)key * a.k_sn) + c * 8;
      char* dst = st + (x ? KBYTES : 0) + c * CSTRIDE + hf * 1024;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
  };
  issue_tile(0, 0);

  int qi[2], fr[2], pos[2];
  bool qv[2];
  bf16x8 qf[2][3];
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    qi[st] = qb * 256 + w * 64 + st * 32 + r;
    qv[st] = qi[st] < FQ;
    fr[st] = qv[st] ? qi[st] / a.tokens_q : 0;
    pos[st] = qv[st] ? qi[st] - fr[st] * a.tokens_q : 0;
    const bf16* qrow = static_cast<const bf16*>(a.q) + (int64_t)b * a.q_sb + (int64_t)fr[st] * a.q_sf +
                       (int64_t)pos[st] * a.q_sn + head * D;
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      bf16x8 f = qv[st] ? M::row_frag(qrow, s, h, D) : M::zero();
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = (bf16)((float)f[j] * cs);
      qf[st][s] = f;                                       // s = 2, h = 1: column 40 = -m = 0 for now
    }
  }
  float m[2] = {0.f, 0.f};                                 // the (bf16-exact) max in Q's column 40
  f32x16 o[2][2];
#pragma unroll
  for (int st = 0; st < 2; ++st) o[st][0] = o[st][1] = zero16();

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  auto compute_tile = [&](const char* kb, const char* vb, int kt, auto masked_tag) {
    constexpr bool MASKED = decltype(masked_tag)::value;
#pragma unroll UNR
    for (int key0 = 0; key0 < KT; key0 += 32) {
      if (MASKED && kt + key0 >= Nk) break;
      f32x16 s[2] = {zero16(), zero16()};
#pragma unroll
      for (int si = 0; si < 3; ++si) {
        const bf16x8 ka = *reinterpret_cast<const bf16x8*>(kb + (2 * si + h) * CSTRIDE + (key0 + r) * 16);
        s[0] = M::mma(ka, qf[0][si], s[0]);
        s[1] = M::mma(ka, qf[1][si], s[1]);
      }
      float mx[2];
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        if constexpr (MASKED) {
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (kt + key0 + acc_row(i, h) >= Nk) s[st][i] = kNegInf;
        }
        float v = fmaxf(s[st][0], s[st][1]);
#pragma unroll
        for (int i = 2; i < 16; i += 2) v = fmaxf(v, fmaxf(s[st][i], s[st][i + 1]));
        mx[st] = v;
      }
      const bool first = kt == 0 && key0 == 0;
      if (first || __any(mx[0] > kRescaleThr || mx[1] > kRescaleThr)) {
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const float rm = fmaxf(mx[st], xhalf(mx[st]));  // row max relative to the current m
          if (first || rm > kRescaleThr) {
            const bf16 mb = (bf16)(m[st] + rm);
            const float delta = (float)mb - m[st];
            const float alpha = fast_exp2(-delta);
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
              for (int i = 0; i < 16; ++i) o[st][t][i] *= alpha;
#pragma unroll
            for (int i = 0; i < 16; ++i) s[st][i] -= delta;
            m[st] = (float)mb;
            if (h) qf[st][2][0] = -mb;
          }
        }
      }
      bf16x8 pf[2][2];
#pragma unroll
      for (int st = 0; st < 2; ++st) {
#pragma unroll
        for (int i = 0; i < 16; ++i) s[st][i] = fast_exp2(s[st][i]);
        pf[st][0] = M::p_frag(s[st], 0);
        pf[st][1] = M::p_frag(s[st], 1);
      }
#pragma unroll
      for (int sp = 0; sp < 2; ++sp)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const bf16x8 vf = vt_frag_planes(vb, key0, sp, t);
          o[0][t] = M::mma(vf, pf[0][sp], o[0][t]);
          o[1][t] = M::mma(vf, pf[1][sp], o[1][t]);
        }
    }
  };

  int stage = 0;
  for (int kt = 0; kt < Nk; kt += KT) {
    if (kt + KT < Nk) issue_tile(kt + KT, stage ^ 1);
    const char* kb = smem + stage * BUF;
    if (kt + KT <= Nk) compute_tile(kb, kb + KBYTES, kt, std::false_type{});
    else compute_tile(kb, kb + KBYTES, kt, std::true_type{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    stage ^= 1;
  }

#pragma unroll
  for (int st = 0; st < 2; ++st) {
    const float mine = o[st][1][4];                        // O^T row 40 = the ones row: lanes h = 0, reg 4
    const float other = xhalf(mine);                       // all 64 lanes take part in the swap
    const float lrow = h == 0 ? mine : other;
    if (a.lse && qv[st]) a.lse[(int64_t)(b * a.heads + head) * FQ + qi[st]] = m[st] + log2f(lrow);
    if (qv[st]) {
      const float inv = 1.f / lrow;
      bf16* orow = static_cast<bf16*>(a.o) + (int64_t)b * a.o_sb + (int64_t)fr[st] * a.o_sf +
                   (int64_t)pos[st] * a.o_sn + head * D;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int dc = 32 * t + 8 * g + 4 * h;
          if (dc < D) {
            bf16x4 v;
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = (bf16)(o[st][t][4 * g + j] * inv);
            *reinterpret_cast<bf16x4*>(orow + dc) = v;
          }
        }
    }
  }
}

static int k1_variant() {  // VP2P_K1_VARIANT=0 / 2 force the one-set / x2 kernels (A/B experiments)
  const char* e = getenv("VP2P_K1_VARIANT");
  return e ? atoi(e) : 2;
}

template <typename T, int D>
static int launch_frame(const vp2p_frame_attn_args* a, hipStream_t stream) {
  using C = FrameCfg<T, D>;
  const int FQ = a->frames * a->tokens_q;
  if constexpr (C::BF && D == k1v3::D) {
    const int var = k1_variant();
    if (var == 3 || var == 4) {
      const int64_t nwg = (int64_t)a->batch * a->heads * ((FQ + 255) / 256);
      if (nwg <= 0 || nwg > 0x7fffffff) return VP2P_E_SHAPE;
      if (var == 3)
        hipLaunchKernelGGL(frame_attn_kernel_v3<4>, dim3((unsigned)nwg), dim3(256), k1v3::LDS_BYTES, stream, *a);
      else
        hipLaunchKernelGGL(frame_attn_kernel_v3<1>, dim3((unsigned)nwg), dim3(256), k1v3::LDS_BYTES, stream, *a);
      return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
    }
  }
  if constexpr (C::BF && C::ONES && D <= 64) {
    if (k1_variant() >= 2) {
      const int64_t nwg = (int64_t)a->batch * a->heads * ((FQ + 255) / 256);
      if (nwg <= 0 || nwg > 0x7fffffff) return VP2P_E_SHAPE;
      hipLaunchKernelGGL((frame_attn_kernel_x2<D>), dim3((unsigned)nwg), dim3(256), C::LDS_BYTES, stream, *a);
      return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
    }
  }
  const int64_t nwg = (int64_t)a->batch * a->heads * ((FQ + 127) / 128);
  if (nwg <= 0 || nwg > 0x7fffffff) return VP2P_E_SHAPE;
  hipLaunchKernelGGL((frame_attn_kernel<T, D>), dim3((unsigned)nwg), dim3(256), C::LDS_BYTES, stream, *a);
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace vp2p

using namespace vp2p;

extern "C" int vp2p_frame_attn_fwd(const vp2p_frame_attn_args* a, void* stream) {
  if (!a || !a->q || !a->k || !a->v || !a->o) return VP2P_E_ARG;
  if (a->batch <= 0 || a->frames <= 0 || a->tokens_q <= 0 || a->tokens_kv <= 0 || a->heads <= 0 ||
      a->head_dim <= 0)
    return VP2P_E_ARG;
  const int esz = a->dtype == VP2P_BF16 ? 2 : (a->dtype == VP2P_F32 ? 4 : 0);
  if (!esz) return VP2P_E_DTYPE;
  const int epc = 16 / esz;
  // 16-byte row segments: base pointers, strides and the head slice must stay 16-byte aligned
  const int64_t strides[] = {a->q_sb, a->q_sf, a->q_sn, a->k_sb, a->k_sn, a->v_sb, a->v_sn,
                             a->o_sb, a->o_sf, a->o_sn};
  for (int64_t s : strides)
    if (s % epc) return VP2P_E_ARG;
  if (a->head_dim % epc || !aligned16(a->q) || !aligned16(a->k) || !aligned16(a->v) || !aligned16(a->o))
    return VP2P_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
#define VP2P_FRAME_CASE(DIM)                                                   \
  case DIM:                                                                    \
    return a->dtype == VP2P_BF16 ? launch_frame<bf16, DIM>(a, s) : launch_frame<float, DIM>(a, s);
  switch (a->head_dim) {
    VP2P_FRAME_CASE(32)
    VP2P_FRAME_CASE(40)
    VP2P_FRAME_CASE(64)
    VP2P_FRAME_CASE(80)
    VP2P_FRAME_CASE(128)
    VP2P_FRAME_CASE(160)
    default:
      return VP2P_E_HEAD_DIM;
  }
#undef VP2P_FRAME_CASE
}
