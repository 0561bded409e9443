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
//    frame-0 K/V tiles of 64 keys through LDS, and the grid is XCD-remapped so the workgroups of one
//    (b, head) share an L2.
//  * swapped 32x32 MFMA tiles (common.hpp): softmax is lane-local, P never leaves registers,
//    V is read transposed from its row-major LDS image with ds_read_b64_tr_b16.
//  * online softmax in the log2 domain (one v_fma + v_exp per score), next K/V tile prefetched into
//    registers while the current one is consumed (issue early / write late).
#include "common.hpp"
#include "vp2p.h"

namespace vp2p {

template <typename T, int D>
struct FrameCfg {
  static constexpr bool BF = sizeof(T) == 2;
  static constexpr int KD = Mfma<T>::KD;
  static constexpr int DP = round_up(D, KD);
  static constexpr int KS = DP / KD;
  static constexpr int DV = round_up(D, 32);
  static constexpr int NT = DV / 32;
  static constexpr int KT = 64;                                  // keys per LDS tile
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

  // zero the LDS image once: the padding columns (D..DP, D..DV) are never written again
  for (int i = tid; i < C::LDS_BYTES / 16; i += 256) reinterpret_cast<u32x4*>(smem)[i] = u32x4{0, 0, 0, 0};

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
  float m = kNegInf, lsum = 0.f;
  f32x16 o[C::NT];
#pragma unroll
  for (int t = 0; t < C::NT; ++t) o[t] = zero16();

  load_tile(0);
  for (int kt = 0; kt < Nk; kt += C::KT) {
    __syncthreads();
    store_tile();
    __syncthreads();
    if (kt + C::KT < Nk) load_tile(kt + C::KT);

#pragma unroll
    for (int blk = 0; blk < 2; ++blk) {
      const int key0 = blk * 32;
      if (kt + key0 >= Nk) break;
      f32x16 s = zero16();
      const T* krow = Ks + (key0 + r) * C::KROW;
#pragma unroll
      for (int si = 0; si < C::KS; ++si) {
        typename M::frag af;
        if constexpr (C::BF) af = *reinterpret_cast<const bf16x8*>(krow + 16 * si + 8 * h);
        else af = krow[2 * si + h];
        s = M::mma(af, qf[si], s);
      }
      float mx = kNegInf;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float v = (kt + key0 + acc_row(i, h) < Nk) ? s[i] * cs : kNegInf;
        s[i] = v;
        mx = fmaxf(mx, v);
      }
      mx = fmaxf(mx, xhalf(mx));
      const float mn = fmaxf(m, mx);
      const float alpha = fast_exp2(m - mn);
      float rs = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = fast_exp2(s[i] - mn);
        s[i] = p;
        rs += p;
      }
      rs += xhalf(rs);
      lsum = lsum * alpha + rs;
      m = mn;
#pragma unroll
      for (int t = 0; t < C::NT; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[t][i] *= alpha;
#pragma unroll
      for (int sp = 0; sp < M::PV_STEPS; ++sp) {
        const typename M::frag pf = M::p_frag(s, sp);
#pragma unroll
        for (int t = 0; t < C::NT; ++t) {
          typename M::frag vf;
          if constexpr (C::BF) vf = vt_frag_lds<C::VROW>(Vs, key0, sp, t);
          else vf = Vs[(key0 + f32_pv_key(sp, h)) * C::VROW + 32 * t + r];
          o[t] = M::mma(vf, pf, o[t]);
        }
      }
    }
  }

  if (qv) {
    const float inv = 1.f / lsum;
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

template <typename T, int D>
static int launch_frame(const vp2p_frame_attn_args* a, hipStream_t stream) {
  using C = FrameCfg<T, D>;
  const int FQ = a->frames * a->tokens_q;
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
