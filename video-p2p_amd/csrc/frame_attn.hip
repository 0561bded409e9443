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
//    (issue early / write late); two barriers per 128-key tile (the folded d = 40 form: two LDS
//    tiles and one barrier per tile).
//  * bf16, d <= 80 (the res-64 and res-32 layers, 98% of the FLOPs): frame_attn_kernel_x2f gives
//    every wave 64 query rows as two independent 32-row sets sharing each K/V fragment read (half
//    the LDS traffic per query, two independent MFMA/VALU chains per wave) -- see its header.
#include <stdlib.h>

#include <type_traits>

#include "frame_attn.hpp"

namespace vp2p {

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

  const float cs = a.q_prescaled ? 1.f : a.scale * kLog2e;
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

// ------------------------------------------------------------------------------------------------
// x2f: bf16, d <= 80 with a spare V^T row (d = 40: the res-64 layers, 88% of the FLOPs, 256-key
// tiles; d = 80: the res-32 layers, 64-key tiles to stay within the register budget).
// frame_attn_kernel_x2 with the inner 128-key tile made one straight-line, software-pipelined block:
//  * no per-score max: m starts at the exact row max of the first 32-key block; afterwards growth
//    is read off the ones-row sum (O^T row D) once per tile: if the tile's sum dl = l - l_prev
//    exceeds kSumThr, m moves up by log2(dl) (so the tile's largest p is <= 1 again) and O and l
//    are rescaled.  P is bf16 and O/l fp32, so between checks p up to 2^127 is still exact to
//    rounding; only a score more than 127 log2 units (88 nats) above the running max overflows,
//    and a row whose final sum is not finite is recomputed exactly by a per-lane two-pass path
//    at the end (never taken on real data; forced by a test);
//  * with no branch inside a tile, QK^T of block j+1 is issued before the exp2/cvt of block j, so
//    the VALU softmax of one block runs under the MFMAs of the next (T15 "att[2]").
// ------------------------------------------------------------------------------------------------
// Two forms of the inner loop:
//   FOLD = false: p = exp2(s * c - m) (c = scale * log2 e): one v_fma + one v_exp + half a v_cvt per
//                 score; set 0's QK^T then set 1's, then the two softmax + PV halves;
//   FOLD = true (the caller passed q already multiplied by c -- its projection GEMM's alpha -- and the
//                 head dim has a padding column in the QK^T k-steps, d = 40: 48): -m rides in the MFMA
//                 through that column (Q'[D] = -m held exactly in bf16, K[D] = 1 in the LDS image), so
//                 the accumulator already holds s * c - m and the softmax is one v_exp + half a v_cvt
//                 per score.  m is kept bf16-representable and O is rescaled by the exact
//                 exp2(m_old - m_new) when it moves.  The blocks are set-staggered: set 1's QK^T of
//                 block j and set 0's QK^T of block j + 1 are issued ahead of the other set's softmax,
//                 so each set's exp/cvt run under MFMAs (128-key tiles keep the extra score registers
//                 within the 2-waves/SIMD budget).
// LDS tiles of x2f: two for the folded d = 40 form (tile t+1 is stored from registers while tile t
// is consumed: one barrier per key tile instead of two; 77.8 KB, two workgroups per CU: 0.813 ->
// 0.800 ms at res-64, profiles/r02_k1_lab_q.jsonl), one elsewhere (d = 80 spills with two).
constexpr int x2f_bufs(int D, int KT, bool FOLD) { return FOLD && D <= 64 && KT <= 128 ? 2 : 1; }

template <int D, int KT, bool FOLD>
__global__ __launch_bounds__(256, 2) void frame_attn_kernel_x2f(const vp2p_frame_attn_args a) {
  constexpr int kK1Bufs = x2f_bufs(D, KT, FOLD);
  using T = bf16;
  using M = Mfma<T>;
  using C = FrameCfg<T, D>;
  static_assert(C::ONES && D <= 80 && D % 8 == 0, "x2f: bf16, spare ones row");
  static_assert(!FOLD || C::DP > D, "folded max needs a padding column in the QK^T k-steps");
  constexpr int PAD_S = D / 16, PAD_H = (D % 16) / 8, PAD_J = D % 8;   // qf slot of column D
  constexpr int NBLK = KT / 32;
  constexpr int NCH = (KT * C::CPR + 255) / 256;          // 16-byte chunks per thread per tile
  constexpr int TILE_BYTES = KT * (C::KROW + C::VROW) * 2;
  constexpr int LDS_BYTES = kK1Bufs * TILE_BYTES;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* Ks = reinterpret_cast<T*>(smem);
  T* Vs = Ks + KT * C::KROW;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, r = l & 31, h = l >> 5;
  const int FQ = a.frames * a.tokens_q;
  const int qblocks = (FQ + 255) >> 8;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  // (b, head)-major: all query blocks of one (b, head) on one XCD, its frame-0 K/V fetched into one L2
  // (FETCH x2 + WRITE 427 MB at the res-64 launch vs 778 MB head-fastest, same time:
  // profiles/r03_k1_grid_ab.txt)
  const int bh = bid / qblocks, qb = bid - bh * qblocks;
  const int b = bh / a.heads, head = bh - b * a.heads;
  const int Nk = a.tokens_kv;
  const float cs = a.q_prescaled ? 1.f : a.scale * kLog2e;

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
  for (int i = tid; i < LDS_BYTES / 16; i += 256) reinterpret_cast<u32x4*>(smem)[i] = u32x4{0, 0, 0, 0};
  __syncthreads();
  for (int k = tid; k < kK1Bufs * KT; k += 256) {
    const int bi = k / KT, kk = k - bi * KT;
    T* kb_ = reinterpret_cast<T*>(smem + bi * TILE_BYTES);
    kb_[KT * C::KROW + kk * C::VROW + D] = (T)1.0f;     // O^T row D = sum_k p
    if constexpr (FOLD) kb_[kk * C::KROW + D] = (T)1.0f; // S^T += 1 * Q'[D] = -m
  }

  const T* kbase = static_cast<const T*>(a.k) + b * a.k_sb + head * D;
  const T* vbase = static_cast<const T*>(a.v) + b * a.v_sb + head * D;
  u32x4 kreg[NCH], vreg[NCH];
  auto load_tile = [&](int kt) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = tid + i * 256;
      const int row = c / C::CPR, col = (c - row * C::CPR) * C::EPC;
      const int key = kt + row;
      if (c < KT * C::CPR && key < Nk) {
        kreg[i] = *reinterpret_cast<const u32x4*>(kbase + (int64_t)key * a.k_sn + col);
        vreg[i] = *reinterpret_cast<const u32x4*>(vbase + (int64_t)key * a.v_sn + col);
      } else {
        kreg[i] = u32x4{0, 0, 0, 0};
        vreg[i] = u32x4{0, 0, 0, 0};
      }
    }
  };
  auto store_tile = [&](int buf) {
    T* kd = reinterpret_cast<T*>(smem + buf * TILE_BYTES);
    T* vd = kd + KT * C::KROW;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = tid + i * 256;
      if (c < KT * C::CPR) {
        const int row = c / C::CPR, col = (c - row * C::CPR) * C::EPC;
        *reinterpret_cast<u32x4*>(kd + row * C::KROW + col) = kreg[i];
        *reinterpret_cast<u32x4*>(vd + row * C::VROW + col) = vreg[i];
      }
    }
  };

  float m[2] = {0.f, 0.f}, lp[2] = {0.f, 0.f};
  f32x16 o[2][C::NT];
#pragma unroll
  for (int st = 0; st < 2; ++st)
#pragma unroll
    for (int t = 0; t < C::NT; ++t) o[st][t] = zero16();

  // folded max: the Q' slot of column D holds -m (lanes of half PAD_H own that column)
  auto set_negm = [&](int st) {
    if constexpr (FOLD) {
      const bf16 nm = (bf16)(-m[st]);
      if (h == PAD_H) qf[st][PAD_S][PAD_J] = nm;   // the other half holds column D - 8 (real data)
    }
  };

  // m starts at the exact row max of keys 0..31 (tile 0 in LDS; ragged Nk < 32 masked)
  auto init_max = [&]() {
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      f32x16 s = zero16();
#pragma unroll
      for (int si = 0; si < C::KS; ++si)
        s = M::mma(*reinterpret_cast<const bf16x8*>(Ks + r * C::KROW + 16 * si + 8 * h), qf[st][si], s);
      float v = kNegInf;
#pragma unroll
      for (int i = 0; i < 16; ++i) v = fmaxf(v, acc_row(i, h) < Nk ? s[i] : kNegInf);
      if constexpr (FOLD) {
        m[st] = (float)(bf16)fmaxf(v, xhalf(v));   // already in log2 units; bf16-exact offset
        set_negm(st);
      } else {
        m[st] = fmaxf(v, xhalf(v)) * cs;
      }
    }
  };

  auto compute_tile = [&](int kt, auto masked_tag) {
    constexpr bool MASKED = decltype(masked_tag)::value;
    auto qk = [&](int key0, int st) {
      f32x16 acc = zero16();
#pragma unroll
      for (int si = 0; si < C::KS; ++si)
        acc = M::mma(*reinterpret_cast<const bf16x8*>(Ks + (key0 + r) * C::KROW + 16 * si + 8 * h), qf[st][si], acc);
      if constexpr (MASKED) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (kt + key0 + acc_row(i, h) >= Nk) acc[i] = kNegInf;
      }
      return acc;
    };
    auto softmax_pv = [&](f32x16& sc, int key0, int st) {
      if constexpr (FOLD) {
#pragma unroll
        for (int i = 0; i < 16; ++i) sc[i] = fast_exp2(sc[i]);
      } else {
        const float nm = -m[st];
#pragma unroll
        for (int i = 0; i < 16; ++i) sc[i] = fast_exp2(__builtin_fmaf(sc[i], cs, nm));
      }
      const bf16x8 p0 = M::p_frag(sc, 0), p1 = M::p_frag(sc, 1);
#pragma unroll
      for (int t = 0; t < C::NT; ++t) o[st][t] = M::mma(vt_frag_lds<C::VROW>(Vs, key0, 0, t), p0, o[st][t]);
#pragma unroll
      for (int t = 0; t < C::NT; ++t) o[st][t] = M::mma(vt_frag_lds<C::VROW>(Vs, key0, 1, t), p1, o[st][t]);
    };
    if constexpr (FOLD) {
      // set-staggered: s0 of block j was issued during block j - 1
      const int nblk = MASKED ? min(NBLK, (Nk - kt + 31) >> 5) : NBLK;
      f32x16 s0 = qk(0, 0);
#pragma unroll
      for (int j = 0; j < NBLK; ++j) {
        if (MASKED && j >= nblk) break;
        const int key0 = 32 * j;
        f32x16 s1 = qk(key0, 1);
        softmax_pv(s0, key0, 0);
        if (j + 1 < NBLK && (!MASKED || j + 1 < nblk)) s0 = qk(key0 + 32, 0);
        softmax_pv(s1, key0, 1);
      }
    } else {
      // set 0's QK^T, then set 1's, so set 0's softmax runs while set 1's MFMAs execute and set 1's
      // softmax while set 0's PV MFMAs execute (the other wave of the SIMD fills the rest)
#pragma unroll
      for (int j = 0; j < NBLK; ++j) {
        const int key0 = 32 * j;
        if (MASKED && kt + key0 >= Nk) break;
        f32x16 s0 = qk(key0, 0);
        f32x16 s1 = qk(key0, 1);
        softmax_pv(s0, key0, 0);
        softmax_pv(s1, key0, 1);
      }
    }
    // once per tile: the tile's row sum (valid on lanes h == ONE_H; the other half reads a zero row)
    float lc[2];
#pragma unroll
    for (int st = 0; st < 2; ++st) lc[st] = o[st][C::ONE_T][C::ONE_I];
    if (__any(lc[0] - lp[0] > kSumThr || lc[1] - lp[1] > kSumThr)) {
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const float mine = lc[st] - lp[st];
        const float other = xhalf(mine);
        const float dl = h == C::ONE_H ? mine : other;
        const float delta = dl > kSumThr ? __log2f(dl) : 0.f;   // rows that did not grow: alpha = 1
        float alpha;
        if constexpr (FOLD) {
          const float mn = dl > kSumThr ? (float)(bf16)(m[st] + delta) : m[st];
          alpha = fast_exp2(m[st] - mn);
          m[st] = mn;
          set_negm(st);
        } else {
          alpha = fast_exp2(-delta);
          m[st] += delta;
        }
#pragma unroll
        for (int t = 0; t < C::NT; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i) o[st][t][i] *= alpha;
        lc[st] *= alpha;
      }
    }
    lp[0] = lc[0];
    lp[1] = lc[1];
  };

  load_tile(0);
  if constexpr (kK1Bufs == 2) {
    // two LDS tiles: tile t+1 is stored (from registers loaded during tile t-1) while tile t is
    // consumed, and one barrier per tile both publishes it and retires the reads of tile t-1
    __syncthreads();
    store_tile(0);
    __syncthreads();
    if (KT < Nk) load_tile(KT);
    init_max();
    int it = 0, kt = 0;
    for (; kt + KT <= Nk; kt += KT, ++it) {
      const int cur = it & 1;
      Ks = reinterpret_cast<T*>(smem + cur * TILE_BYTES);
      Vs = Ks + KT * C::KROW;
      compute_tile(kt, std::false_type{});
      if (kt + KT < Nk) {
        store_tile(cur ^ 1);
        if (kt + 2 * KT < Nk) load_tile(kt + 2 * KT);
        __syncthreads();
      }
    }
    if (kt < Nk) {
      Ks = reinterpret_cast<T*>(smem + (it & 1) * TILE_BYTES);
      Vs = Ks + KT * C::KROW;
      compute_tile(kt, std::true_type{});
    }
  } else {
    int kt = 0;
    for (; kt + KT <= Nk; kt += KT) {
      __syncthreads();
      store_tile(0);
      __syncthreads();
      if (kt + KT < Nk) load_tile(kt + KT);
      if (kt == 0) init_max();
      compute_tile(kt, std::false_type{});
    }
    if (kt < Nk) {
      __syncthreads();
      store_tile(0);
      __syncthreads();
      if (kt == 0) init_max();
      compute_tile(kt, std::true_type{});
    }
  }
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    const float mine = o[st][C::ONE_T][C::ONE_I];
    const float other = xhalf(mine);
    const float lrow = (h == C::ONE_H) ? mine : other;
    // inf / NaN by exponent bits (the file builds with -fno-honor-nans), in the row sum or in any of
    // this lane's O values (p <= 2^127 between growth checks times |v| > 2 can overflow O while l
    // stays finite)
    bool bad = qv[st] && (__float_as_uint(lrow) & 0x7f800000u) == 0x7f800000u;
#pragma unroll
    for (int t = 0; t < C::NT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) bad |= qv[st] && (__float_as_uint(o[st][t][i]) & 0x7f800000u) == 0x7f800000u;
    if (qv[st] && !bad) {
      if (a.lse) a.lse[(int64_t)(b * a.heads + head) * FQ + qi[st]] = m[st] + log2f(lrow);
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
    if (bad) frame_attn_exact_row<D>(a, b, head, fr[st], pos[st], qi[st], h, cs);
  }
}

template <int D, int KT, bool FOLD>
static int launch_x2f(const vp2p_frame_attn_args* a, int64_t nwg, hipStream_t stream) {
  constexpr int lds = x2f_bufs(D, KT, FOLD) * KT * (FrameCfg<bf16, D>::KROW + FrameCfg<bf16, D>::VROW) * 2;
  static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&frame_attn_kernel_x2f<D, KT, FOLD>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
  if (!attr) return VP2P_E_LAUNCH;
  hipLaunchKernelGGL((frame_attn_kernel_x2f<D, KT, FOLD>), dim3((unsigned)nwg), dim3(256), lds, stream, *a);
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

template <typename T, int D>
static int launch_frame(const vp2p_frame_attn_args* a, hipStream_t stream) {
  using C = FrameCfg<T, D>;
  const int FQ = a->frames * a->tokens_q;
  if constexpr (C::BF && C::ONES && D <= 80) {
    constexpr int KT = D <= 64 ? 256 : 64;   // d 80: 64-key tiles (32: 0.106, 128: 0.137 vs 0.103 ms, r04_k1_d80_kt_ab.jsonl)
    const int64_t nwg = (int64_t)a->batch * a->heads * ((FQ + 255) / 256);
    if (nwg <= 0 || nwg > 0x7fffffff) return VP2P_E_SHAPE;
#ifndef VP2P_K1_LAB_X2F   // (lab builds only: x2f for every d = 40 launch, the A/B baseline)
    if constexpr (D == 40) {
      // the software-pipelined res-64 kernel (frame_attn_pp.hip) wherever its layout applies
      // (VP2P_E_SHAPE: it does not, x2f below takes the call)
      const int rc = launch_frame_attn_pp(a, stream);
      if (rc != VP2P_E_SHAPE) return rc;
    }
#endif
    if constexpr (C::DP > D)
      if (a->q_prescaled) return launch_x2f<D, 128, true>(a, nwg, stream);
    return launch_x2f<D, KT, false>(a, nwg, stream);
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
