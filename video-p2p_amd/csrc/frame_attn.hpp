// K1 pieces shared by frame_attn.hip (one-set / x2f kernels) and frame_attn_pp.hip (the pipelined
// res-64 kernel): LDS image geometry, softmax constants, the exact overflow fallback row.
#pragma once
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

constexpr float kSumThr = 4096.f;


// Exact two-pass softmax row of one query in plain fp32 VALU (the overflow fallback of x2f):
// writes this lane's epilogue slots of the output row and the row's log-sum-exp.
// Small register footprint (the query row is re-read from memory, one 4-column output slot
// accumulated at a time) so this rare path does not add to the kernel's register budget.
template <int D>
__device__ __forceinline__ void frame_attn_exact_row(const vp2p_frame_attn_args& a, int b, int head, int fr,
                                                     int pos, int64_t qi, int h, float cs) {
  const bf16* qrow = static_cast<const bf16*>(a.q) + b * a.q_sb + (int64_t)fr * a.q_sf + (int64_t)pos * a.q_sn + head * D;
  const bf16* kb = static_cast<const bf16*>(a.k) + b * a.k_sb + head * D;
  const bf16* vb = static_cast<const bf16*>(a.v) + b * a.v_sb + head * D;
  auto score = [&](int key) {
    const bf16* kr = kb + (int64_t)key * a.k_sn;
    float s = 0.f;
    for (int c = 0; c < D; ++c) s = __builtin_fmaf((float)qrow[c], (float)kr[c], s);
    return s;
  };
  float mx = kNegInf;
  for (int key = 0; key < a.tokens_kv; ++key) mx = fmaxf(mx, score(key) * cs);
  float l = 0.f;
  for (int key = 0; key < a.tokens_kv; ++key) l += exp2f(__builtin_fmaf(score(key), cs, -mx));
  const int FQ = a.frames * a.tokens_q;
  if (a.lse) a.lse[(int64_t)(b * a.heads + head) * FQ + qi] = mx + log2f(l);
  const float inv = 1.f / l;
  bf16* orow = static_cast<bf16*>(a.o) + b * a.o_sb + (int64_t)fr * a.o_sf + (int64_t)pos * a.o_sn + head * D;
  for (int dc = 4 * h; dc < D; dc += 8) {        // this lane's 4-column slots of each 8-column group
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int key = 0; key < a.tokens_kv; ++key) {
      const float p = exp2f(__builtin_fmaf(score(key), cs, -mx));
      const bf16* vr = vb + (int64_t)key * a.v_sn + dc;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_fmaf(p, (float)vr[j], acc[j]);
    }
    bf16x4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = (bf16)(acc[j] * inv);
    *reinterpret_cast<bf16x4*>(orow + dc) = v;
  }
}

// the pipelined d = 40 kernel (frame_attn_pp.hip): pre-scaled q, tokens_kv % 128 == 0
int launch_frame_attn_pp(const vp2p_frame_attn_args* a, hipStream_t stream);

}  // namespace vp2p
